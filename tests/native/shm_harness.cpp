// tests/native/shm_harness.cpp — CPU harness of the test-only cross-process
// communicator (vampomi_amd/csrc/shmcomm.cpp), no GPU: P forked ranks join
// one segment and run all-reduces of assorted sizes (larger than the slot:
// chunked), checking rank-ordered sums bit for bit; modes:
//   ok <P> <ncoll>        every rank agrees; exit 0
//   mismatch <P>          rank 1 calls from another site: every rank fails
//   kill <P>              rank P-1 exits during the run: the others fail fast
//   late <P> <ms>         rank P-1 joins <ms> late: the join waits for it
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

struct ShmComm;
std::shared_ptr<ShmComm> shm_join(const void* id, int P, int rank, double limit_s, std::string* err);
std::string shm_allreduce(ShmComm& s, int rank, double* buf, size_t n, uint64_t seq, const char* site, int line,
                          double limit_s);

static int rank_main(const unsigned char* id, const std::string& mode, int P, int r, int ncoll, int late_ms) {
    if (mode == "late" && r == P - 1) std::this_thread::sleep_for(std::chrono::milliseconds(late_ms));
    std::string err;
    auto s = shm_join(id, P, r, 20.0, &err);
    if (!s) {
        std::printf("rank %d join: %s\n", r, err.c_str());
        return 2;
    }
    for (int k = 0; k < ncoll; ++k) {
        if (mode == "kill" && r == P - 1 && k == 3) {
            std::fflush(stdout);
            _exit(9);  // gone mid-run
        }
        const size_t n = 1 + (size_t)(k % 5) * 300001;         // > the 524288-double slot: chunked
        std::vector<double> b(n);
        for (size_t i = 0; i < n; ++i) b[i] = (r + 1) * 0.1 + k * 1e-3 + (double)(i % 97) * 1e-7;
        const char* site = mode == "mismatch" && r == 1 && k == 2 ? "other_site" : "site";
        const std::string e = shm_allreduce(*s, r, b.data(), n, k + 1, site, 10, 20.0);
        if (!e.empty()) {
            std::printf("rank %d collective %d: %s\n", r, k, e.c_str());
            return 3;
        }
        for (size_t i = 0; i < n; ++i) {
            double want = 0.0;  // the rank-ordered sum, as the last rank to arrive forms it
            for (int q = 0; q < P; ++q) want += (q + 1) * 0.1 + k * 1e-3 + (double)(i % 97) * 1e-7;
            if (b[i] != want) {
                std::printf("rank %d collective %d element %zu: %.17g != %.17g\n", r, k, i, b[i], want);
                return 4;
            }
        }
    }
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 3) return 64;
    const std::string mode = argv[1];
    const int P = std::atoi(argv[2]);
    const int ncoll = mode == "ok" && argc > 3 ? std::atoi(argv[3]) : 8;
    const int late_ms = mode == "late" && argc > 3 ? std::atoi(argv[3]) : 0;
    unsigned char id[128];
    const unsigned long long salt = (unsigned long long)getpid() * 6364136223846793005ull ^
                                    (unsigned long long)std::chrono::steady_clock::now().time_since_epoch().count();
    for (int i = 0; i < 128; ++i) id[i] = (unsigned char)(salt >> ((i % 8) * 8)) ^ (unsigned char)(i * 131);
    std::vector<pid_t> kids;
    for (int r = 0; r < P; ++r) {
        const pid_t p = fork();
        if (p == 0) {
            const int rc = rank_main(id, mode, P, r, ncoll, late_ms);
            std::fflush(stdout);  // (_exit does not flush: the messages would be lost in a pipe)
            _exit(rc);
        }
        kids.push_back(p);
    }
    const auto t0 = std::chrono::steady_clock::now();
    std::string codes;
    for (pid_t p : kids) {
        int st = 0;
        waitpid(p, &st, 0);
        codes += std::to_string(WIFEXITED(st) ? WEXITSTATUS(st) : 128 + WTERMSIG(st)) + " ";
    }
    std::printf("exit codes: %s\nseconds: %.2f\n", codes.c_str(),
                std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    return 0;
}
