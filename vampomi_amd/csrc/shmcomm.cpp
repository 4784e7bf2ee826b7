// shmcomm.cpp — test-only cross-process communicator (VAMPOMI_COMM=shm).
//
// The ranks of a job are PROCESSES on one host (e.g. main_meth.exe started P
// times with VAMPOMI_RANK / VAMPOMI_NRANKS, possibly all on one GPU, where
// RCCL refuses two ranks per device), and an all-reduce is a rendezvous in a
// POSIX shared-memory segment that sums the ranks' buffers in rank order: the
// loopback communicator's contract (engine.cpp), across processes.  It runs
// every multi-process path of the drop-in CLI that a multi-GPU node would run
// through RCCL (the id rendezvous file, per-rank shards, each all-reduce site,
// per-rank pwrite of the .bin files at S*8, the all-ok exit agreement) where
// one GPU is available.
//
// Segment: /vampomi_shm_<hex of the communicator id>, created by whichever
// rank comes first (ftruncate zero-fills it: every counter starts at 0),
// unlinked as soon as all P ranks have mapped it (so a crashed job leaves no
// name behind).  Per collective: each rank writes its buffer and descriptor
// (sequence number, size, call site), then arrives; the last to arrive checks
// the descriptors, sums in rank order, and starts the next generation.  A
// waiting rank fails (and poisons the segment, failing every rank at once)
// when a peer process is gone, on a descriptor mismatch, or after the
// collective's time limit.
#include <fcntl.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>

#include "ctx.h"

namespace {
constexpr int kShmMaxRanks = 64;
struct ShmDesc {
    uint64_t seq, n, site;
    int64_t line;
};
struct ShmHdr {
    std::atomic<uint64_t> gen;   // completed collectives
    std::atomic<int> arrived;    // ranks in the current one
    std::atomic<int> poisoned;   // non-zero: the job failed; why[] says why
    std::atomic<int> joined;     // ranks that hold a mapping of the segment
    std::atomic<int> opened;     // ranks that ever mapped it (monotone: the join barrier)
    std::atomic<int> why_lock;
    int P;
    uint64_t cap;  // doubles per rank slot
    char why[512];
    ShmDesc desc[kShmMaxRanks];
    int pid[kShmMaxRanks];
};
static_assert(std::atomic<uint64_t>::is_always_lock_free && std::atomic<int>::is_always_lock_free,
              "lock-free atomics are address-free: they work between processes");

uint64_t fnv1a(const char* s) {
    uint64_t h = 1469598103934665603ull;
    for (; s && *s; ++s) h = (h ^ (unsigned char)*s) * 1099511628211ull;
    return h;
}

size_t shm_cap() {
    const char* e = std::getenv("VAMPOMI_SHM_CAP");
    const long long v = e ? std::atoll(e) : 0;
    return v > 0 ? (size_t)v : (size_t)1 << 19;  // 4 MiB per rank; larger all-reduces go in chunks
}

// the process is gone (or a zombie nobody has reaped yet)
bool pid_gone(int pid) {
    if (pid <= 0) return false;
    if (::kill(pid, 0) != 0 && errno == ESRCH) return true;
    char path[64], buf[256];
    std::snprintf(path, sizeof path, "/proc/%d/stat", pid);
    FILE* f = std::fopen(path, "r");
    if (!f) return true;
    const size_t n = std::fread(buf, 1, sizeof buf - 1, f);
    std::fclose(f);
    buf[n] = 0;
    const char* p = std::strrchr(buf, ')');  // "pid (comm) S ..."
    return p && p[1] == ' ' && (p[2] == 'Z' || p[2] == 'X');
}
}  // namespace

struct ShmComm {
    std::string name;
    void* base = nullptr;
    size_t bytes = 0;
    int P = 0;
    ShmHdr* h = nullptr;
    double* in(int r) const { return reinterpret_cast<double*>(h + 1) + (size_t)r * h->cap; }
    double* out() const { return in(P); }
    ~ShmComm() {
        if (h) h->joined.fetch_sub(1);
        if (base) ::munmap(base, bytes);
    }
};

void shm_poison(ShmComm& s, const std::string& why) {
    ShmHdr* h = s.h;
    int expect = 0;
    if (h->why_lock.compare_exchange_strong(expect, 1)) {
        std::snprintf(h->why, sizeof h->why, "%s", why.c_str());
        h->poisoned.store(1, std::memory_order_release);
    }
}

std::string shm_why(const ShmComm& s) {
    if (!s.h->poisoned.load(std::memory_order_acquire)) return std::string();
    return std::string(s.h->why, strnlen(s.h->why, sizeof s.h->why));
}

std::shared_ptr<ShmComm> shm_join(const void* id, int P, int rank, double limit_s, std::string* err) {
    if (P < 1 || P > kShmMaxRanks || rank < 0 || rank >= P) {
        *err = "shm communicator: 1..64 ranks";
        return nullptr;
    }
    auto s = std::make_shared<ShmComm>();
    char hex[33];
    for (int i = 0; i < 16; ++i) std::snprintf(hex + 2 * i, 3, "%02x", ((const unsigned char*)id)[i]);
    s->name = std::string("/vampomi_shm_") + hex;
    const size_t cap = shm_cap();
    s->P = P;
    s->bytes = sizeof(ShmHdr) + (size_t)(P + 1) * cap * sizeof(double);
    const int fd = ::shm_open(s->name.c_str(), O_RDWR | O_CREAT, 0600);
    if (fd < 0) {
        *err = "shm_open " + s->name + ": " + std::strerror(errno);
        return nullptr;
    }
    struct stat st {};
    // every rank sizes it the same; a second ftruncate to the same size keeps the contents
    if (::fstat(fd, &st) != 0 || ((size_t)st.st_size < s->bytes && ::ftruncate(fd, (off_t)s->bytes) != 0)) {
        *err = "sizing " + s->name + ": " + std::strerror(errno);
        ::close(fd);
        return nullptr;
    }
    s->base = ::mmap(nullptr, s->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    ::close(fd);
    if (s->base == MAP_FAILED) {
        s->base = nullptr;
        *err = "mmap " + s->name + ": " + std::strerror(errno);
        return nullptr;
    }
    s->h = static_cast<ShmHdr*>(s->base);
    ShmHdr* h = s->h;
    if ((h->P != 0 && h->P != P) || (h->cap != 0 && h->cap != cap)) {
        *err = "shm communicator: the ranks disagree on the rank count or VAMPOMI_SHM_CAP";
        shm_poison(*s, *err);
        return nullptr;
    }
    h->P = P;
    h->cap = cap;
    h->pid[rank] = (int)::getpid();
    h->joined.fetch_add(1);
    // the last rank to map the segment removes its name (every rank holds a mapping)
    if (h->opened.fetch_add(1) + 1 == P) ::shm_unlink(s->name.c_str());
    // Joining is collective, like RCCL's communicator init: every rank returns
    // once all P have joined (main_meth.exe's rank 0 removes the id's
    // rendezvous file after its open returns, so every rank must have read it
    // by then), or fails after limit_s / when a joined peer process is gone.
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t spin = 1; h->opened.load(std::memory_order_acquire) < P; ++spin) {
        if (h->poisoned.load(std::memory_order_acquire)) {
            *err = "shm communicator: " + std::string(h->why, strnlen(h->why, sizeof h->why));
            return nullptr;
        }
        for (int r = 0; r < P; ++r)
            if (r != rank && pid_gone(h->pid[r])) {
                *err = "shm communicator: rank " + std::to_string(r) + " exited before every rank joined";
                shm_poison(*s, *err);
                return nullptr;
            }
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit_s) {
            *err = "shm communicator: not every rank joined within " + std::to_string((int)limit_s) +
                   " s (VAMPOMI_COMM_INIT_TIMEOUT_S)";
            shm_poison(*s, *err);
            ::shm_unlink(s->name.c_str());
            return nullptr;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(spin < 1000 ? 50 : 2000));
    }
    return s;
}

// SUM of n doubles (host buffer, in place) over the ranks, in rank order;
// "" on success, else why the job failed (the segment is then poisoned)
std::string shm_allreduce(ShmComm& s, int rank, double* buf, size_t n, uint64_t seq, const char* site, int line,
                          double limit_s) {
    ShmHdr* h = s.h;
    const int P = s.P;
    for (size_t off = 0, part = 0; off < n; off += h->cap, ++part) {
        const size_t m = std::min<size_t>(h->cap, n - off);
        if (!shm_why(s).empty()) return "shm communicator failed earlier: " + shm_why(s);
        const uint64_t my_gen = h->gen.load(std::memory_order_acquire);
        std::memcpy(s.in(rank), buf + off, m * sizeof(double));
        h->desc[rank] = ShmDesc{seq * 4096 + part, n, fnv1a(site), line};
        if (h->arrived.fetch_add(1, std::memory_order_acq_rel) + 1 == P) {
            for (int r = 1; r < P; ++r) {
                const ShmDesc& a = h->desc[0];
                const ShmDesc& b = h->desc[r];
                if (a.seq != b.seq || a.n != b.n || a.site != b.site || a.line != b.line) {
                    char why[200];
                    std::snprintf(why, sizeof why,
                                  "ranks disagree on the collective: rank 0 #%llu of %llu doubles (line %lld), rank %d "
                                  "#%llu of %llu doubles (line %lld)",
                                  (unsigned long long)(a.seq / 4096), (unsigned long long)a.n, (long long)a.line, r,
                                  (unsigned long long)(b.seq / 4096), (unsigned long long)b.n, (long long)b.line);
                    shm_poison(s, why);
                    break;
                }
            }
            double* o = s.out();
            for (size_t i = 0; i < m; ++i) o[i] = 0.0;
            for (int r = 0; r < P; ++r) {
                const double* x = s.in(r);
                for (size_t i = 0; i < m; ++i) o[i] += x[i];
            }
            h->arrived.store(0, std::memory_order_relaxed);
            h->gen.store(my_gen + 1, std::memory_order_release);
        } else {
            const auto t0 = std::chrono::steady_clock::now();
            for (uint64_t spin = 1;; ++spin) {
                if (h->gen.load(std::memory_order_acquire) != my_gen) break;
                if (h->poisoned.load(std::memory_order_acquire)) break;
                if ((spin & 1023) == 0) {
                    for (int r = 0; r < P; ++r)
                        if (r != rank && pid_gone(h->pid[r]) && h->gen.load(std::memory_order_acquire) == my_gen) {
                            shm_poison(s, "rank " + std::to_string(r) + " (pid " + std::to_string(h->pid[r]) +
                                              ") exited during collective #" + std::to_string(seq) + " at " + site);
                            break;
                        }
                    const double el =
                        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                    if (el > limit_s && h->gen.load(std::memory_order_acquire) == my_gen)
                        shm_poison(s, "not every rank arrived within " + std::to_string((int)limit_s) +
                                          " s at collective #" + std::to_string(seq) + " (" + site + ")");
                    std::this_thread::sleep_for(std::chrono::microseconds(spin < 65536 ? 2 : 200));
                }
            }
        }
        const std::string why = shm_why(s);
        if (!why.empty()) return "shm all-reduce: " + why;
        std::memcpy(buf + off, s.out(), m * sizeof(double));
    }
    return std::string();
}
