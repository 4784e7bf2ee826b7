// hostio.cpp — gVAMPomi file formats (see hostio.h for the reference lines).
#include "hostio.h"

#include <fcntl.h>
#include <unistd.h>

#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <fstream>
#include <thread>

#include <sys/stat.h>

namespace vio {

static bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n' || c == '\v' || c == '\f'; }

int64_t read_phen(const std::string& path, std::vector<double>& y) {
    std::ifstream in(path);
    if (!in.is_open()) return -1;
    y.clear();
    std::string line;
    while (std::getline(in, line)) {
        // third token of the "\\s+" split with submatch -1: a leading run of
        // whitespace produces an empty first token.
        std::vector<std::string> tok;
        size_t i = 0;
        const size_t n = line.size();
        for (;;) {
            size_t j = i;
            while (j < n && !is_ws(line[j])) ++j;
            if (j == n) {  // suffix after the last separator: only if non-empty
                if (j > i || tok.empty()) tok.push_back(line.substr(i, j - i));
                break;
            }
            tok.push_back(line.substr(i, j - i));  // text before a separator (may be empty)
            while (j < n && is_ws(line[j])) ++j;
            i = j;
            if (i == n) break;
        }
        if (tok.size() < 3) continue;
        if (tok[2] == "NA") return -2;
        y.push_back(std::atof(tok[2].c_str()));
    }
    return (int64_t)y.size();
}

double standardize_phen(std::vector<double>& y) {
    double sum = 0.0;
    for (double v : y) sum += v;
    const int64_t nonas = (int64_t)y.size();
    const double avg = sum / double(nonas);
    double sqn = 0.0;
    for (size_t i = 0; i < y.size(); ++i)
        if (y[i] != DBL_MAX) sqn += (y[i] - avg) * (y[i] - avg);
    sqn = std::sqrt(double(nonas - 1) / sqn);
    for (size_t i = 0; i < y.size(); ++i) y[i] *= sqn;
    return sqn;
}

bool store_vec(const std::string& path, const double* v, int64_t S, int64_t M) {
    int fd = ::open(path.c_str(), O_CREAT | O_WRONLY, 0666);
    if (fd < 0) return false;
    const size_t want = (size_t)M * sizeof(double);
    size_t done = 0;
    while (done < want) {
        ssize_t w = ::pwrite(fd, (const char*)v + done, want - done, (off_t)S * 8 + (off_t)done);
        if (w <= 0) break;
        done += (size_t)w;
    }
    ::close(fd);
    return done == want;
}

bool read_vec(const std::string& path, double* v, int64_t S, int64_t M) {
    int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) return false;
    std::memset(v, 0, (size_t)M * sizeof(double));
    const size_t want = (size_t)M * sizeof(double);
    size_t done = 0;
    while (done < want) {
        ssize_t r = ::pread(fd, (char*)v + done, want - done, (off_t)S * 8 + (off_t)done);
        if (r <= 0) break;
        done += (size_t)r;
    }
    ::close(fd);
    return true;
}

bool csv_create_with_header(const std::string& path, const std::vector<std::string>& fields) {
    ::unlink(path.c_str());
    int fd = ::open(path.c_str(), O_CREAT | O_WRONLY | O_EXCL, 0666);
    if (fd < 0) return false;
    std::string s = fields.empty() ? std::string() : fields[0];
    for (size_t i = 1; i < fields.size(); ++i) s += ", " + fields[i];
    s += "\n";
    ssize_t w = ::pwrite(fd, s.data(), s.size(), 0);
    ::close(fd);
    return w == (ssize_t)s.size();
}

bool read_text_vec(const std::string& path, double* v, int64_t S, int64_t M) {
    std::ifstream f(path);
    if (!f) return false;
    double value;
    int64_t it = 0;
    while (f >> value) {
        if (it >= S + M) break;
        if (it >= S) v[it - S] = value;
        ++it;
    }
    return true;
}

bool csv_create(const std::string& path) {
    ::unlink(path.c_str());
    int fd = ::open(path.c_str(), O_CREAT | O_WRONLY | O_EXCL, 0666);
    if (fd < 0) return false;
    ::close(fd);
    return true;
}

std::string csv_format_row(int it, const double* vals, int n) {
    char buf[50000];
    int cx = std::snprintf(buf, sizeof buf, "%5d", it);
    for (int i = 0; i < n; ++i) cx += std::snprintf(buf + cx, sizeof buf - (size_t)cx, ", %20.15f", vals[i]);
    cx += std::snprintf(buf + cx, sizeof buf - (size_t)cx, "\n");
    return std::string(buf, (size_t)cx);
}

bool csv_write_row(const std::string& path, int it, const double* vals, int n) {
    const std::string row = csv_format_row(it, vals, n);
    int fd = ::open(path.c_str(), O_WRONLY);
    if (fd < 0) return false;
    ssize_t w = ::pwrite(fd, row.data(), row.size(), (off_t)it * (off_t)row.size());
    ::close(fd);
    return w == (ssize_t)row.size();
}

static const char kRdzvMagic[] = "VAMPOMI-RDZV1";

std::string rdzv_nonce() {
    // a job id every rank of the job sees: ours, torchrun's, the MPI / PMIx
    // namespace (mpirun), slurm's job and step
    for (const char* v : {"VAMPOMI_RUN_ID", "TORCHELASTIC_RUN_ID", "PMIX_NAMESPACE", "OMPI_MCA_ess_base_jobid",
                          "PMI_KVSNAME"}) {
        const char* e = std::getenv(v);
        if (e && *e) return std::string(v) + "=" + e;
    }
    const char* sj = std::getenv("SLURM_JOB_ID");
    const char* ss = std::getenv("SLURM_STEP_ID");
    if (sj && *sj) return std::string("slurm=") + sj + "." + (ss ? ss : "");
    const char* a = std::getenv("MASTER_ADDR");
    const char* p = std::getenv("MASTER_PORT");
    if (a && p && *a && *p) return std::string("master=") + a + ":" + p;
    return std::string();
}

// magic '\n' nonce '\n' id bytes, written to path.tmp and renamed into place
// (readers never see a partial file); any file already at path is removed first
bool rdzv_publish(const std::string& path, const std::string& nonce, const void* id, int nbytes) {
    ::unlink(path.c_str());
    const std::string tmp = path + ".tmp";
    {
        std::ofstream f(tmp, std::ios::binary | std::ios::trunc);
        if (!f) return false;
        f << kRdzvMagic << '\n' << nonce << '\n';
        f.write((const char*)id, nbytes);
        if (!f.good()) return false;
    }
    return std::rename(tmp.c_str(), path.c_str()) == 0;
}

static bool rdzv_try(const std::string& path, const std::string& nonce, double not_before, void* id, int nbytes) {
    struct stat st;
    if (::stat(path.c_str(), &st) != 0) return false;
    if (nonce.empty() && (double)st.st_mtime < not_before) return false;  // an earlier job's file
    std::ifstream f(path, std::ios::binary);
    std::string magic, n;
    if (!std::getline(f, magic) || magic != kRdzvMagic || !std::getline(f, n) || n != nonce) return false;
    f.read((char*)id, nbytes);
    return f.gcount() == nbytes;
}

bool rdzv_fetch(const std::string& path, const std::string& nonce, double not_before, void* id, int nbytes,
                int timeout_ms) {
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<unsigned char> first((size_t)nbytes), again((size_t)nbytes);
    for (;;) {
        // checked on every path round the loop: a file rewritten or flapping
        // within the recheck below must not keep this rank here past the limit
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms)) return false;
        if (rdzv_try(path, nonce, not_before, first.data(), nbytes)) {
            if (!nonce.empty()) {
                std::memcpy(id, first.data(), (size_t)nbytes);
                return true;
            }
            // No job id: a file left by an earlier job whose rank 0 died before
            // removing it could pass the time window.  Rank 0 of THIS job
            // replaces any such file as it starts; accept only an id that is
            // still there, unchanged, 3 s later.
            std::this_thread::sleep_for(std::chrono::seconds(3));
            if (rdzv_try(path, nonce, not_before, again.data(), nbytes) &&
                std::memcmp(first.data(), again.data(), (size_t)nbytes) == 0) {
                std::memcpy(id, again.data(), (size_t)nbytes);
                return true;
            }
            continue;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(50));
    }
}

void rdzv_remove(const std::string& path) { ::unlink(path.c_str()); }

}  // namespace vio
