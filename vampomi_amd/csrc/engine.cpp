// engine.cpp — libvampomi: the C ABI of include/vampomi.h over HIP + RCCL.
//
// One context = one process = one gfx950 device = one contiguous marker shard
// (the reference's MPI rank).  The design matrix shard, the marker statistics
// and every M- and N-vector of the VAMP state stay resident in HBM; the host
// holds only the handful of scalars the algorithm branches on (gam1, gam2,
// gamw, the mixture, CG stopping tests), which it reads back after fixed-order
// device reductions.  Cross-rank sums are RCCL all-reduces on the context's
// stream (the reference's MPI_Allreduce call sites).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <chrono>
#include <condition_variable>
#include <map>
#include <mutex>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include <fcntl.h>
#include <unistd.h>

#include "ctx.h"
#include "hostio.h"
#include "writer.h"

// ---------------------------------------------------------------------------
// errors and device memory
// ---------------------------------------------------------------------------
static thread_local std::string g_err;
static thread_local vampomi_ctx* g_coll_ctx = nullptr;  // innermost CollScope of this thread

CollScope::CollScope(vampomi_ctx* c) : prev(g_coll_ctx) { g_coll_ctx = c; }
CollScope::~CollScope() { g_coll_ctx = prev; }

vampomi_status fail(vampomi_status s, const std::string& msg) {
    g_err = msg;
    if (g_coll_ctx && g_coll_ctx->use_comm && !g_coll_ctx->aborted) comm_abort(g_coll_ctx, msg);
    return s;
}

vampomi_status dev_alloc(double** p, size_t n) {
    if (n == 0) n = 1;
    hipError_t e = hipMalloc((void**)p, n * sizeof(double));
    if (e != hipSuccess)
        return fail(VAMPOMI_ERR_OOM, "hipMalloc(" + std::to_string(n * sizeof(double)) + " B): " + hipGetErrorString(e));
    return VAMPOMI_OK;
}

void dev_free(double*& p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}

// ---------------------------------------------------------------------------
// timing of the A / A^T kernels (HIP events on the context's stream)
// ---------------------------------------------------------------------------
static hipEvent_t ev_get(vampomi_ctx* c) {
    if (!c->ev_pool.empty()) {
        hipEvent_t e = c->ev_pool.back();
        c->ev_pool.pop_back();
        return e;
    }
    // timestamps only: no system-scope fence (neutral at C2,
    // profiles/r03t_event_fence_ab.txt; timed launches cost 1-2.6 % of a C2
    // iteration either way, hence the sampled timing, bench.py --timing-period)
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return nullptr;
    return e;
}

// algorithmic bytes / flops of one pass with K right-hand sides:
// X once, the K N-vectors, mave/msig and the K M-vectors; (x - mu) once per
// element and one fma per right-hand side.
static double pass_bytes(const vampomi_ctx* c, int K) {
    return 8.0 * (double)c->N * (double)c->M + 8.0 * K * (double)c->N + 8.0 * (2.0 + K) * (double)c->M;
}
static double pass_flops(const vampomi_ctx* c, int K) { return (double)c->N * (double)c->M * (1.0 + 2.0 * K); }

static vampomi_kernel_stat* stat_of(vampomi_ctx* c, int cls) {
    return cls == 0 ? &c->stats.ax : cls == 1 ? &c->stats.atx : cls == 3 ? &c->stats.op : cls == 4 ? &c->stats.coll
                                                                                                : &c->stats.loo;
}
static vampomi_kernel_stat* stat_k_of(vampomi_ctx* c, int cls, int K) {
    return cls == 0 ? &c->stats.ax_k[K - 1] : cls == 1 ? &c->stats.atx_k[K - 1] : cls == 3 ? &c->stats.op_k[K - 1]
                                                                                           : nullptr;
}

// Every launch is counted exactly (launches, algorithmic bytes and flops);
// with timing on, one in tperiod launches of each (class, K) (hashed
// positions) also gets HIP events in its dispatch packet.  The per-class time is the sampled average
// times the exact launch count (vampomi_get_stats), so skipped or dropped
// samples never inflate it.
TimedLaunch launch_stat(vampomi_ctx* c, int cls, int K, double bytes, double flops) {
    for (vampomi_kernel_stat* x : {stat_of(c, cls), stat_k_of(c, cls, K)}) {
        if (!x) continue;
        x->launches += 1;
        x->bytes_total += bytes;
        x->flops_total += flops;
    }
    TimedLaunch t{};
    // which launches carry events: a hash of the launch's index in its class,
    // so the sampled launches fall at every position of a CG solve alike (a
    // fixed stride of 4 met the same steps of every 8-launch iteration)
    if (!c->timing) return t;
    uint64_t h = (uint64_t)c->tcount[cls][K - 1]++ * 0x9E3779B97F4A7C15ULL + (uint64_t)(cls * 8 + K);
    h ^= h >> 31;
    h *= 0xBF58476D1CE4E5B9ULL;
    h ^= h >> 29;
    // collectives (class 4) are bracketed by hipEventRecord markers of their
    // own (no dispatch packet to carry them), each a few us of idle queue:
    // sampled 8x more sparsely (the 1-rank RCCL line lost 1 % to them, r05c)
    const uint64_t period = (uint64_t)std::max(c->tperiod, 1) * (cls == 4 ? 8 : 1);
    // the first launch of each (class, K) since the stats were reset is always
    // sampled: a (class, K) with launches and no sample would count its bytes
    // and no time (c4's one K = 4 A.x pass per iteration, r05j)
    const vampomi_kernel_stat* xk = stat_k_of(c, cls, K);
    const bool first = (xk ? xk : stat_of(c, cls))->launches == 1;
    if (period > 1 && h % period != 0 && !first) return t;
    t.a = ev_get(c);
    t.b = ev_get(c);
    t.cls = cls;
    t.K = K;
    t.bytes = bytes;
    t.flops = flops;
    c->pending.push_back(t);
    return t;
}

void resolve_timing(vampomi_ctx* c) {
    for (auto& t : c->pending) {
        float ms = 0.f;
        if (hipEventSynchronize(t.b) == hipSuccess && hipEventElapsedTime(&ms, t.a, t.b) == hipSuccess) {
            for (vampomi_kernel_stat* x : {stat_of(c, t.cls), stat_k_of(c, t.cls, t.K)}) {
                if (!x) continue;
                x->timed += 1;
                x->ms_timed += (double)ms;
            }
        }
        c->ev_pool.push_back(t.a);
        c->ev_pool.push_back(t.b);
    }
    c->pending.clear();
}

// the launches of a CG step queued after its solve had stopped did nothing
// (gated): forget their counts and samples (pcg.cpp)
void drop_launches(vampomi_ctx* c, size_t pending_mark, const vampomi_stats& before) {
    for (size_t q = pending_mark; q < c->pending.size(); ++q) {
        c->ev_pool.push_back(c->pending[q].a);
        c->ev_pool.push_back(c->pending[q].b);
    }
    c->pending.resize(pending_mark);
    // counts back to `before`; samples (timed, ms_timed) are only resolved
    // outside a solve, and the dropped ones were removed above
    auto undo = [](vampomi_kernel_stat& x, const vampomi_kernel_stat& b) {
        x.launches = b.launches;
        x.bytes_total = b.bytes_total;
        x.flops_total = b.flops_total;
    };
    undo(c->stats.ax, before.ax);
    undo(c->stats.atx, before.atx);
    undo(c->stats.op, before.op);
    undo(c->stats.loo, before.loo);
    undo(c->stats.coll, before.coll);
    for (int k = 0; k < 4; ++k) {
        undo(c->stats.ax_k[k], before.ax_k[k]);
        undo(c->stats.atx_k[k], before.atx_k[k]);
        undo(c->stats.op_k[k], before.op_k[k]);
    }
    c->stats.a_passes_exec = before.a_passes_exec;
}

// ---------------------------------------------------------------------------
// reductions
// ---------------------------------------------------------------------------
// Host waits without hipStreamSynchronize's completion path: the stream
// stores increasing sequence numbers into a mapped host word (system-scope
// release) and the host spins on it — a few microseconds sooner, once per
// dependency level of the iteration.  host_sync waits for everything queued
// (a 1-thread kernel stores the flag); a one-rank DotBatch waits for its last
// reduction kernel, whose last block stores the flag itself.  Faults are
// still reported: the spin polls hipStreamQuery, and gives up after 10 min.
//
// With an RCCL communicator the waits also watch the job: a peer that died or
// a communicator RCCL reports broken (ncclCommGetAsyncError) or a wait longer
// than VAMPOMI_COLL_TIMEOUT_S (default 120 s; the queued all-reduce waits for
// a peer that never comes) aborts this rank's communicator (ncclCommAbort)
// and fails, instead of blocking forever in a collective.  A healthy job's
// ranks reach each collective within milliseconds of each other; the one
// legitimate long wait is the first collective after the data load, when the
// ranks' shards come off a slow shared filesystem at different rates: that
// one is vampomi_barrier_timeout's, with its own limit (main_meth.exe: after
// the shard load, VAMPOMI_LOAD_TIMEOUT_S, default one hour).
static double coll_timeout_s() {
    static const double t = [] {
        const char* e = std::getenv("VAMPOMI_COLL_TIMEOUT_S");
        const double v = e ? std::atof(e) : 0.0;
        return v > 0 ? v : 120.0;
    }();
    return t;
}

// this context's limit for the collective in progress
static double coll_limit_s(const vampomi_ctx* c) { return c->coll_limit_s > 0 ? c->coll_limit_s : coll_timeout_s(); }

// nullptr while the job is healthy, else why it is not
static const char* job_broken(vampomi_ctx* c, std::chrono::steady_clock::time_point t0) {
    if (c->comm && !c->loopback) {
        ncclResult_t r = ncclSuccess;
        if (ncclCommGetAsyncError(c->comm, &r) == ncclSuccess && r != ncclSuccess && r != ncclInProgress)
            return "RCCL communicator error";
    }
    const double lim = c->use_comm ? coll_limit_s(c) : 600.0;
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > lim)
        return c->use_comm ? "no completion within VAMPOMI_COLL_TIMEOUT_S (a peer rank stopped?)"
                           : "device did not signal completion within 10 minutes";
    return nullptr;
}

static vampomi_status job_failed(vampomi_ctx* c, const char* why) {
    const std::string msg = std::string(why) + " (rank " + std::to_string(c->rank) + ")";
    comm_abort(c, msg);  // ncclCommAbort: this rank's queued collectives are released
    return fail(c->use_comm ? VAMPOMI_ERR_RCCL : VAMPOMI_ERR_HIP, msg);
}

// The communicator is NON-BLOCKING (ncclConfig_t.blocking = 0, vampomi_open):
// any RCCL call may return ncclInProgress, and the next call on the
// communicator must wait until ncclCommGetAsyncError leaves that state.  Every
// call goes through here: it returns at once on ncclSuccess (the steady
// state), otherwise polls the communicator until it settles, at most
// limit_s seconds, and aborts it after that (a peer that never joins the
// bootstrap, a transport that never connects) instead of blocking forever.
static vampomi_status nccl_settle(vampomi_ctx* c, ncclResult_t r, const char* what, double limit_s) {
    if (r == ncclSuccess) return VAMPOMI_OK;
    if (r != ncclInProgress || !c->comm)
        return fail(VAMPOMI_ERR_RCCL, std::string(what) + ": " + ncclGetErrorString(r));
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t spin = 1;; ++spin) {
        ncclResult_t s = ncclSuccess;
        const ncclResult_t q = ncclCommGetAsyncError(c->comm, &s);
        if (q != ncclSuccess) return fail(VAMPOMI_ERR_RCCL, std::string(what) + ": " + ncclGetErrorString(q));
        if (s == ncclSuccess) return VAMPOMI_OK;
        if (s != ncclInProgress) {
            const std::string msg = std::string(what) + ": " + ncclGetErrorString(s) + " (rank " + std::to_string(c->rank) + ")";
            comm_abort(c, msg);
            return fail(VAMPOMI_ERR_RCCL, msg);
        }
        if ((spin & 1023) == 0 &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit_s) {
            const std::string msg = std::string(what) + ": not finished within " + std::to_string((int)limit_s) +
                                    " s (a peer rank never joined?) (rank " + std::to_string(c->rank) + ")";
            comm_abort(c, msg);
            return fail(VAMPOMI_ERR_RCCL, msg);
        }
        std::this_thread::sleep_for(std::chrono::microseconds(spin < 4096 ? 1 : 200));
    }
}

// seconds the communicator's creation may take (VAMPOMI_COMM_INIT_TIMEOUT_S,
// default 120): the bootstrap waits for every rank, so a rank that died or
// never started shows up here
static double comm_init_timeout_s() {
    const char* e = std::getenv("VAMPOMI_COMM_INIT_TIMEOUT_S");
    const double v = e ? std::atof(e) : 0.0;
    return v > 0 ? v : 120.0;
}

// hipStreamQuery is NOT free for the stream: it can put a marker packet behind
// the work queued so far, i.e. between the last queued kernel and the next one
// the host queues after this wait (a CG step's cg_update and the next operator
// launch: 6-7 us of idle GPU at every C2 step, profiles/r04c_gaps.txt).  So the
// spin asks the runtime only after kQueryAfterS of waiting (far longer than
// any step), and every kQueryEveryS after that: a fault or a stream that
// finished without the flag is still seen, within a second.
static constexpr double kQueryAfterS = 0.5, kQueryEveryS = 0.25;

vampomi_status wait_flag(vampomi_ctx* c, unsigned long long seq, int word) {
    const auto t0 = std::chrono::steady_clock::now();
    double next_query = kQueryAfterS;
    hipStream_t st = c->st;
    for (uint64_t spin = 1;; ++spin) {
        if (__atomic_load_n(c->h_flag + word, __ATOMIC_ACQUIRE) >= seq) return VAMPOMI_OK;
        if ((spin & 4095) == 0) {
            const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (el >= next_query) {
                next_query = el + kQueryEveryS;
                const hipError_t e = hipStreamQuery(st);
                if (e != hipSuccess && e != hipErrorNotReady)
                    return fail(VAMPOMI_ERR_HIP, std::string("stream failed: ") + hipGetErrorString(e));
                if (e == hipSuccess) {  // finished, flag not seen yet: complete through the runtime
                    if (__atomic_load_n(c->h_flag + word, __ATOMIC_ACQUIRE) >= seq) return VAMPOMI_OK;
                    HIPCHK(hipStreamSynchronize(st));
                    return VAMPOMI_OK;
                }
            }
            if (const char* why = job_broken(c, t0)) return job_failed(c, why);
        }
        __builtin_ia32_pause();
    }
}

vampomi_status sync_stream(vampomi_ctx* c, hipStream_t st) {
    if (!c->comm || c->loopback) {
        HIPCHK(hipStreamSynchronize(st));
        return VAMPOMI_OK;
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t spin = 1;; ++spin) {
        const hipError_t e = hipStreamQuery(st);
        if (e == hipSuccess) return VAMPOMI_OK;
        if (e != hipErrorNotReady) return fail(VAMPOMI_ERR_HIP, std::string("stream failed: ") + hipGetErrorString(e));
        if ((spin & 255) == 0)
            if (const char* why = job_broken(c, t0)) return job_failed(c, why);
        __builtin_ia32_pause();
    }
}

vampomi_status host_sync(vampomi_ctx* c) {
    c->stats.host_syncs++;
    if (!c->h_flag) {
        STCHK(sync_stream(c, c->st));
        return VAMPOMI_OK;
    }
    const unsigned long long seq = ++c->sync_seq;
    HIPCHK(vk::signal_host(c->d_flag, seq, c->st));
    return wait_flag(c, seq);
}

// ---------------------------------------------------------------------------
// test-only loopback communicator (VAMPOMI_COMM=loopback): the ranks of a job
// are contexts driven by threads of ONE process, possibly on one GPU, and an
// all-reduce is a host rendezvous that sums the ranks' buffers in rank order.
// It exercises every multi-rank code path of the engine (divide_work shards,
// per-rank partials, each all-reduce site, the post-reduce division) where
// only one GPU is available; jobs across GPUs use RCCL.
// ---------------------------------------------------------------------------
struct LoopbackComm {
    std::mutex mu;
    std::condition_variable cv;
    int P = 0, arrived = 0;
    uint64_t gen = 0;
    std::string poison;  // non-empty: the job failed (mismatch, abort); every later call fails with it
    struct Desc {
        uint64_t seq;      // the rank's collective sequence number
        size_t n;
        const char* site;  // the calling function (static string) and line
        int line;
    };
    std::vector<Desc> desc;
    std::vector<std::vector<double>> in;
    std::vector<double> out;
};

static std::mutex g_loopback_mu;
static std::map<std::string, std::weak_ptr<LoopbackComm>> g_loopback;

static std::shared_ptr<LoopbackComm> loopback_join(const void* id, int P) {
    const std::string key((const char*)id, VAMPOMI_UNIQUE_ID_BYTES);
    std::lock_guard<std::mutex> g(g_loopback_mu);
    std::shared_ptr<LoopbackComm> lb = g_loopback[key].lock();
    if (!lb) {
        lb = std::make_shared<LoopbackComm>();
        lb->P = P;
        lb->in.resize((size_t)P);
        lb->desc.resize((size_t)P);
        g_loopback[key] = lb;
    }
    return lb;
}

static std::string coll_desc(int r, const LoopbackComm::Desc& d) {
    return "rank " + std::to_string(r) + ": collective #" + std::to_string(d.seq) + " of " + std::to_string(d.n) +
           " doubles at " + d.site + ":" + std::to_string(d.line);
}

// Every rank deposits its buffer with a descriptor (sequence number, size,
// call site).  The last to arrive checks that all descriptors agree before it
// sums; a disagreement (ranks that took different branches) poisons the
// communicator, and every rank fails at once with every rank's descriptor.
static vampomi_status loopback_allreduce(vampomi_ctx* c, double* buf, size_t n, const char* site, int line) {
    LoopbackComm& lb = *c->loopback;
    const LoopbackComm::Desc me{++c->coll_seq, n, site, line};
    std::vector<double> mine(n);
    HIPCHK(hipMemcpyAsync(mine.data(), buf, n * 8, hipMemcpyDeviceToHost, c->st));
    STCHK(sync_stream(c, c->st));
    std::string err;  // reported after the lock is released (fail() may abort the communicator)
    {
        std::unique_lock<std::mutex> g(lb.mu);
        if (!lb.poison.empty()) {
            err = "loopback communicator failed earlier: " + lb.poison;
        } else {
            const uint64_t my_gen = lb.gen;
            lb.in[(size_t)c->rank] = std::move(mine);
            lb.desc[(size_t)c->rank] = me;
            if (++lb.arrived == lb.P) {
                bool agree = true;
                for (int r = 1; r < lb.P; ++r) {
                    const auto& a = lb.desc[0];
                    const auto& b = lb.desc[(size_t)r];
                    agree = agree && a.seq == b.seq && a.n == b.n && a.line == b.line && std::strcmp(a.site, b.site) == 0;
                }
                if (!agree) {
                    std::string why = "ranks disagree on the collective:";
                    for (int r = 0; r < lb.P; ++r) why += " [" + coll_desc(r, lb.desc[(size_t)r]) + "]";
                    lb.poison = why;
                } else {
                    lb.out.assign(n, 0.0);
                    for (int r = 0; r < lb.P; ++r)
                        for (size_t i = 0; i < n; ++i) lb.out[i] += lb.in[(size_t)r][i];
                }
                lb.arrived = 0;
                ++lb.gen;
                lb.cv.notify_all();
            } else if (!lb.cv.wait_for(g, std::chrono::duration<double>(c->coll_limit_s > 0 ? c->coll_limit_s : 60.0),
                                       [&] { return lb.gen != my_gen || !lb.poison.empty(); })) {
                // a rank that failed without aborting never arrives: end this
                // rank with an error instead of waiting forever
                --lb.arrived;
                lb.poison = "not every rank arrived in time at " + coll_desc(c->rank, me);
                lb.cv.notify_all();
            }
            if (!lb.poison.empty())
                err = "loopback all-reduce: " + lb.poison;
            else
                mine = lb.out;  // lb.out is only rewritten once every rank has arrived again
        }
    }
    if (!err.empty()) {
        c->aborted = true;  // the communicator is poisoned already
        return fail(VAMPOMI_ERR_STATE, err);
    }
    HIPCHK(hipMemcpyAsync(buf, mine.data(), n * 8, hipMemcpyHostToDevice, c->st));
    STCHK(sync_stream(c, c->st));
    return VAMPOMI_OK;
}

// VAMPOMI_COLL_CHECK=1 (RCCL): before every all-reduce, the ranks all-reduce
// their descriptor (sequence number, size, call-site line) as max and -min and
// compare on the host: a divergence fails on every rank instead of hanging.
// Costs a host round trip per collective; a debugging aid.
static vampomi_status rccl_check(vampomi_ctx* c, size_t n, const char* site, int line) {
    double* d = c->scal + SL_CHECK;
    const double v[3] = {(double)c->coll_seq, (double)n, (double)line};
    double h[6] = {v[0], v[1], v[2], -v[0], -v[1], -v[2]};
    HIPCHK(hipMemcpyAsync(d, h, sizeof h, hipMemcpyHostToDevice, c->st));
    STCHK(nccl_settle(c, ncclAllReduce(d, d, 6, ncclDouble, ncclMax, c->comm, c->st), "ncclAllReduce (check)",
                      coll_limit_s(c)));
    HIPCHK(hipMemcpyAsync(h, d, sizeof h, hipMemcpyDeviceToHost, c->st));
    STCHK(sync_stream(c, c->st));
    for (int q = 0; q < 3; ++q)
        if (h[q] != v[q] || -h[3 + q] != v[q])
            return fail(VAMPOMI_ERR_STATE, "ranks disagree on collective #" + std::to_string(c->coll_seq) + " (this rank: " +
                                               std::to_string(n) + " doubles at " + site + ":" + std::to_string(line) + ")");
    return VAMPOMI_OK;
}

// the shm communicator (shmcomm.cpp): the buffer through the host, summed in
// rank order in the shared segment, like the loopback one
static vampomi_status shm_allreduce_dev(vampomi_ctx* c, double* buf, size_t n, const char* site, int line) {
    std::vector<double> h(n);
    HIPCHK(hipMemcpyAsync(h.data(), buf, n * 8, hipMemcpyDeviceToHost, c->st));
    STCHK(sync_stream(c, c->st));
    const std::string err = shm_allreduce(*c->shm, c->rank, h.data(), n, ++c->coll_seq, site, line, coll_limit_s(c));
    if (!err.empty()) {
        c->aborted = true;  // the segment is poisoned already: every rank fails at its next collective
        return fail(VAMPOMI_ERR_STATE, err + " (rank " + std::to_string(c->rank) + ")");
    }
    HIPCHK(hipMemcpyAsync(buf, h.data(), n * 8, hipMemcpyHostToDevice, c->st));
    STCHK(sync_stream(c, c->st));
    return VAMPOMI_OK;
}

vampomi_status allreduce_dev(vampomi_ctx* c, double* buf, size_t n, const char* site, int line) {
    if (!c->use_comm || n == 0) return VAMPOMI_OK;
    if (c->loopback) return loopback_allreduce(c, buf, n, site, line);
    if (c->shm) return shm_allreduce_dev(c, buf, n, site, line);
    ++c->coll_seq;
    static const bool check = std::getenv("VAMPOMI_COLL_CHECK") && std::atoi(std::getenv("VAMPOMI_COLL_CHECK"));
    if (check) STCHK(rccl_check(c, n, site, line));
    const TimedLaunch t = launch_stat(c, 4, 1, 8.0 * (double)n, 0.0);
    if (t.a) HIPCHK(hipEventRecord(t.a, c->st));
    STCHK(nccl_settle(c, ncclAllReduce(buf, buf, n, ncclDouble, ncclSum, c->comm, c->st), "ncclAllReduce",
                      coll_limit_s(c)));
    if (t.b) HIPCHK(hipEventRecord(t.b, c->st));
    return VAMPOMI_OK;
}

vampomi_status sum_over_ranks(vampomi_ctx* c, double local, double* total, const char* site, int line) {
    if (!c->use_comm) {
        *total = local;
        return VAMPOMI_OK;
    }
    double* d = c->scal + SL_AGREE;
    HIPCHK(vk::set_scalar(d, local, c->st));
    STCHK(allreduce_dev(c, d, 1, site, line));
    HIPCHK(hipMemcpyAsync(c->h_scal + SL_AGREE, d, 8, hipMemcpyDeviceToHost, c->st));
    STCHK(sync_stream(c, c->st));
    *total = c->h_scal[SL_AGREE];
    return VAMPOMI_OK;
}

// Ends the job's communicator after a rank-local failure, so that no other
// rank waits for this one: the loopback communicator is poisoned (every rank's
// next or pending collective fails at once), RCCL's is aborted.
void comm_abort(vampomi_ctx* c, const std::string& why) {
    if (!c || !c->use_comm) return;
    if (c->loopback) {
        std::lock_guard<std::mutex> g(c->loopback->mu);
        if (c->loopback->poison.empty()) c->loopback->poison = "rank " + std::to_string(c->rank) + " aborted: " + why;
        c->loopback->cv.notify_all();
    } else if (c->shm) {
        shm_poison(*c->shm, "rank " + std::to_string(c->rank) + " aborted: " + why);
    } else if (c->comm) {
        (void)ncclCommAbort(c->comm);
        c->comm = nullptr;
    }
    c->aborted = true;
}

extern "C" vampomi_status vampomi_all_ok(vampomi_ctx* c, int local_ok, int* all_ok) {
    CollScope cs_(c);
    if (!c || !all_ok) return fail(VAMPOMI_ERR_ARG, "null argument");
    HIPCHK(hipSetDevice(c->device));
    double bad = 0.0;
    STCHK(sum_over_ranks(c, local_ok ? 0.0 : 1.0, &bad));
    *all_ok = bad == 0.0 ? 1 : 0;
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_comm_abort(vampomi_ctx* c) {
    if (!c) return fail(VAMPOMI_ERR_ARG, "null context");
    comm_abort(c, "vampomi_comm_abort");
    return VAMPOMI_OK;
}

vampomi_status DotBatch::sink(int nq, bool sync, double* out, vk::RedOut* ro) {
    int& used = sync ? nsync_ : nlocal_;
    const int base = sync ? SL_SYNC : SL_LOCAL, cap = sync ? SL_NSYNC : SL_NLOCAL;
    if (used + nq > cap) return fail(VAMPOMI_ERR_STATE, "DotBatch overflow");
    ro->part = c_->red_part;
    ro->out = (c_->use_comm ? c_->scal : c_->d_hscal) + base + used;
    ro->ticket = c_->ticket;
    ro->flag = nullptr;
    ro->seq = 0;
    // results land in host memory: the kernel flags their arrival (a sequence
    // number along the stream, monotone)
    if (!c_->use_comm && c_->h_flag) {
        ro->flag = c_->d_flag;
        ro->seq = last_seq_ = ++c_->sync_seq;
    }
    sinks_.push_back(Sink{base + used, nq, out});
    used += nq;
    return VAMPOMI_OK;
}

vampomi_status DotBatch::add(std::initializer_list<vk::DotTerm> terms, int64_t n, bool sync, double* out) {
    vk::DotArgs a{};
    a.nt = (int)terms.size();
    if (a.nt < 1 || a.nt > vk::kMaxTerms) return fail(VAMPOMI_ERR_ARG, "DotBatch: 1.." + std::to_string(vk::kMaxTerms) + " terms");
    int q = 0;
    for (const auto& t : terms) {
        a.t[q] = t;
        if (t.op == vk::SUM) a.t[q].b = t.a;  // the kernel loads both operands of every term
        ++q;
    }
    vk::RedOut ro{};
    STCHK(sink(a.nt, sync, out, &ro));
    HIPCHK(vk::dots(a, n, ro, stream()));
    return VAMPOMI_OK;
}

vampomi_status DotBatch::add_many(int64_t n, const std::vector<Group>& groups, const vk::G1Chain* chain,
                                  const double* chain_of,
                                  const std::vector<std::pair<const double*, double*>>& copies) {
    vk::DotArgs a{};
    vk::RedOut ro{};
    STCHK(build(groups, chain, chain_of, copies, a, ro));
    HIPCHK(vk::dots(a, n, ro, stream()));
    return VAMPOMI_OK;
}

vampomi_status DotBatch::add_pair(int64_t na, const std::vector<Group>& ga, const vk::G1Chain* chain,
                                  const double* chain_of, const std::vector<std::pair<const double*, double*>>& ca,
                                  int64_t nb, const std::vector<Group>& gb,
                                  const std::vector<std::pair<const double*, double*>>& cb) {
    vk::DotArgs a{}, b{};
    vk::RedOut roa{}, rob{};
    STCHK(build(ga, chain, chain_of, ca, a, roa));
    STCHK(build(gb, nullptr, nullptr, cb, b, rob));
    const size_t need = (size_t)vk::red_blocks(na) * a.nt + (size_t)vk::red_blocks(nb) * b.nt;
    if (a.nt == 10 && b.nt == 11 && need <= c_->red_cap) {  // (the pairing vk::dots2 instantiates)
        roa.flag = nullptr;  // b's flag (the later sequence number) covers both
        rob.part = roa.part + (int64_t)vk::red_blocks(na) * a.nt;
        rob.ticket = roa.ticket;
        HIPCHK(vk::dots2(a, na, roa, b, nb, rob, stream()));
    } else {
        HIPCHK(vk::dots(a, na, roa, stream()));
        HIPCHK(vk::dots(b, nb, rob, stream()));
    }
    return VAMPOMI_OK;
}

vampomi_status DotBatch::build(const std::vector<Group>& groups, const vk::G1Chain* chain, const double* chain_of,
                               const std::vector<std::pair<const double*, double*>>& copies, vk::DotArgs& a,
                               vk::RedOut& ro) {
    if (copies.size() > 2) return fail(VAMPOMI_ERR_ARG, "DotBatch: at most 2 device copies per launch");
    // terms in the order [local groups..., synced groups...]: each kind's
    // results land in one contiguous slot range (out, then out2 from split)
    a = vk::DotArgs{};
    int nloc = 0, nsyn = 0;
    for (const Group& g : groups) (g.sync ? nsyn : nloc) += (int)g.terms.size();
    a.nt = nloc + nsyn;
    if (a.nt < 1 || a.nt > vk::kMaxTerms) return fail(VAMPOMI_ERR_ARG, "DotBatch: 1.." + std::to_string(vk::kMaxTerms) + " terms");
    if (nloc + nlocal_ > SL_NLOCAL || nsyn + nsync_ > SL_NSYNC) return fail(VAMPOMI_ERR_STATE, "DotBatch overflow");
    double* base = c_->use_comm ? c_->scal : c_->d_hscal;
    int ql = 0, qs = nloc;
    for (bool want_sync : {false, true}) {
        for (const Group& g : groups) {
            if (g.sync != want_sync) continue;
            int& q = g.sync ? qs : ql;
            sinks_.push_back(Sink{g.sync ? SL_SYNC + nsync_ + (q - nloc) : SL_LOCAL + nlocal_ + q,
                                  (int)g.terms.size(), g.out});
            if (chain && g.out == chain_of) {
                a.g1 = *chain;
                a.g1.term = q;
            }
            for (const auto& cp : copies)
                if (g.out == cp.first) {
                    a.copy.term[a.copy.n] = q;
                    a.copy.dst[a.copy.n++] = cp.second;
                }
            for (const auto& t : g.terms) {
                a.t[q] = t;
                if (t.op == vk::SUM) a.t[q].b = t.a;  // the kernel loads both operands of every term
                ++q;
            }
        }
    }
    if (chain && !a.g1.out) return fail(VAMPOMI_ERR_ARG, "DotBatch: the chained group is not in the launch");
    if (a.copy.n != (int)copies.size()) return fail(VAMPOMI_ERR_ARG, "DotBatch: a copied group is not in the launch");
    ro = vk::RedOut{};
    ro.part = c_->red_part;
    ro.ticket = c_->ticket;
    ro.out = base + SL_LOCAL + nlocal_;
    ro.out2 = base + SL_SYNC + nsync_;
    ro.split = nloc;
    if (!c_->use_comm && c_->h_flag) {  // one flag for the launch (see sink)
        ro.flag = c_->d_flag;
        ro.seq = last_seq_ = ++c_->sync_seq;
    }
    nlocal_ += nloc;
    nsync_ += nsyn;
    return VAMPOMI_OK;
}

const double* DotBatch::dev_result(const double* out) const {
    if (c_->use_comm || !c_->d_hscal) return nullptr;
    for (const Sink& k : sinks_)
        if (k.out == out) return c_->d_hscal + k.slot;
    return nullptr;
}

double* DotBatch::dev_slot(const double* out) const {
    if (!c_->use_comm) return nullptr;
    for (const Sink& k : sinks_)
        if (k.out == out) return c_->scal + k.slot;
    return nullptr;
}

vampomi_status DotBatch::reduce_now() {
    if (!c_->use_comm || nsync_ == nred_) return VAMPOMI_OK;
    STCHK(allreduce_dev(c_, c_->scal + SL_SYNC + nred_, (size_t)(nsync_ - nred_)));
    nred_ = nsync_;
    return VAMPOMI_OK;
}

hipStream_t DotBatch::stream() const { return c_->st; }

vampomi_status DotBatch::flush() {
    if (sinks_.empty()) return VAMPOMI_OK;
    if (c_->use_comm) {  // slots in device memory: all-reduce the synced ones, then publish both ranges
        if (nsync_ > nred_) STCHK(allreduce_dev(c_, c_->scal + SL_SYNC + nred_, (size_t)(nsync_ - nred_)));
        if (c_->h_flag) {
            const unsigned long long seq = ++c_->sync_seq;
            HIPCHK(vk::publish_host(c_->scal + SL_SYNC, nsync_, c_->d_hscal + SL_SYNC, c_->scal + SL_LOCAL, nlocal_,
                                    c_->d_hscal + SL_LOCAL, c_->d_flag, seq, c_->st));
            c_->stats.host_syncs++;
            STCHK(wait_flag(c_, seq));
        } else {
            if (nsync_ > 0)
                HIPCHK(hipMemcpyAsync(c_->h_scal + SL_SYNC, c_->scal + SL_SYNC, sizeof(double) * nsync_,
                                      hipMemcpyDeviceToHost, c_->st));
            if (nlocal_ > 0)
                HIPCHK(hipMemcpyAsync(c_->h_scal + SL_LOCAL, c_->scal + SL_LOCAL, sizeof(double) * nlocal_,
                                      hipMemcpyDeviceToHost, c_->st));
            STCHK(host_sync(c_));
        }
    } else if (last_seq_) {
        c_->stats.host_syncs++;
        STCHK(wait_flag(c_, last_seq_));
    } else {
        STCHK(host_sync(c_));
    }
    for (const Sink& k : sinks_)
        for (int i = 0; i < k.count; ++i) k.out[i] = c_->h_scal[k.slot + i];
    sinks_.clear();
    nsync_ = nlocal_ = nred_ = 0;
    last_seq_ = 0;
    return VAMPOMI_OK;
}

// ---------------------------------------------------------------------------
// operators on device buffers
// ---------------------------------------------------------------------------
// out_k = Ax(x_k) for K <= 4; outputs at outbase + k*ld (contiguous so that one
// all-reduce carries them all).  COLLECTIVE.
vampomi_status ax_dev(vampomi_ctx* c, int K, const double* const* x, double* outbase, const vk::AxFuse* fu,
                      const vk::DotArgs* tail) {
    if (!c->have_X) return fail(VAMPOMI_ERR_STATE, "Ax before the methylation data was loaded");
    vk::CPtrs xs{};
    vk::Ptrs os{};
    for (int k = 0; k < K; ++k) {
        xs.p[k] = x[k];
        os.p[k] = outbase + (int64_t)k * c->ld;
    }
    TimedLaunch t = launch_stat(c, 0, K, pass_bytes(c, K), pass_flops(c, K));
    const vk::AxFuse none{};
    const vk::AxFuse& f = fu ? *fu : none;
    HIPCHK(vk::ax_partial(c->shard(), c->axp, K, xs, c->ax_part, c->st, vk::Timing{t.a, t.b}, f));
    c->stats.a_passes_exec++;
    if (!c->use_comm) {
        HIPCHK(vk::ax_reduce(c->axp, K, c->N, c->ld, c->ax_part, os, c->sqrtN, c->st, f.gate));
    } else {
        HIPCHK(vk::ax_reduce(c->axp, K, c->N, c->ld, c->ax_part, os, 0.0, c->st, f.gate));
        size_t n = (size_t)K * c->ld;
        if (tail) {
            HIPCHK(vk::dots(*tail, c->M, vk::RedOut{c->red_part, outbase + n, c->ticket, nullptr, 0, f.gate}, c->st));
            n += (size_t)tail->nt;
        }
        STCHK(allreduce_dev(c, outbase, n));  // src/data.cpp:367
        HIPCHK(vk::vec_div(K, c->N, c->ld, os, c->sqrtN, c->st));
    }
    return VAMPOMI_OK;
}

// out_k = ATx(u_k) (mode 0) or tau*ATx(u_k) + gam2*p_k with <out_k,p_k> summed
// over ranks into ctx->scal[SL_DP + k] (mode 1).  u_k are ld-padded N-vectors.
vampomi_status atx_dev(vampomi_ctx* c, int K, const double* const* u, double* const* out, int mode,
                              double tau, double gam2, const double* const* p, const int* gate,
                              const double* const* zf, const double* beta, bool dp, double* const* sraw) {
    if (!c->have_X) return fail(VAMPOMI_ERR_STATE, "ATx before the methylation data was loaded");
    if (c->M <= 0) return VAMPOMI_OK;
    vk::CPtrs us{}, ps{}, zs{};
    vk::Ptrs os{}, ss{};
    for (int k = 0; k < K; ++k) {
        us.p[k] = u[k];
        os.p[k] = out[k];
        ss.p[k] = sraw ? sraw[k] : nullptr;
        ps.p[k] = p ? p[k] : nullptr;
        zs.p[k] = zf ? zf[k] : nullptr;
    }
    TimedLaunch t = launch_stat(c, 1, K, pass_bytes(c, K), pass_flops(c, K));
    HIPCHK(vk::atx(c->shard(), K, us, os, 1.0 / c->sqrtN, mode, tau, gam2, ps, c->st, c->atx_variant, vk::Timing{t.a, t.b}, gate, zs,
                   zf ? beta : nullptr, ss));
    c->stats.a_passes_exec++;
    if (mode == 1 && dp) {
        // <d_k, p_k> with the fixed-geometry reduction (depends on M only, not on
        // the A^T kernel variant chosen for this K), so a system's CG iterates are
        // bitwise the same whether it runs alone or batched with another
        vk::DotArgs a{};
        a.nt = K;
        for (int k = 0; k < K; ++k)
            a.t[k] = zf ? vk::DotTerm{out[k], p[k], vk::PUPD, zf[k], beta + k} : vk::DotTerm{out[k], p[k], vk::DOT};
        HIPCHK(vk::dots(a, c->M, vk::RedOut{c->red_part, c->scal + SL_DP, c->ticket, nullptr, 0, gate}, c->st));
        STCHK(allreduce_dev(c, c->scal + SL_DP, K));
    }
    return VAMPOMI_OK;
}

// ---------------------------------------------------------------------------
// one-pass CG operator (batch_rhs 4)
// ---------------------------------------------------------------------------
// doubles of the per-block reduction partials (every reduction kernel's grid)
static size_t red_capacity(int64_t Mx) {
    return std::max<size_t>({(size_t)vk::kRedBlocks * 3 * vk::kMaxRhs, (size_t)vk::kRedBlocks * vk::kMaxTerms,
                             (size_t)((Mx + 255) / 256) * (1 + 2 * (vk::kMaxL - 1)),
                             (size_t)(Mx / 8 + 1) * vk::kMaxRhs, (size_t)4096});  // ATx partials at G >= 2
}

// 8-byte words of the team hand-off granules: M columns x K x T granule pairs,
// then a dummy pair per workgroup and K, then one XCD word per workgroup
static size_t op_xg_words_for(int64_t Mx, const vk::OpPlan& p) {
    return (size_t)(Mx + p.grid) * vk::kOpMaxK * (size_t)p.T * 2 + (size_t)p.grid * (2 * vk::kOpMaxK + 1);
}

static vampomi_status op_plan_local(vampomi_ctx* c) {
    if (c->cus <= 0) HIPCHK(hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, c->device));
    const int64_t M = std::max<int64_t>(c->M, 1);
    bool op_ok = vk::op_plan(c->N, M, c->cus, c->op_variant, &c->opp);
    if (op_ok && c->opp.T >= 1) {
        // a team launch waits for members that must all be resident at once:
        // the device must hold the whole grid (one workgroup per CU) for every
        // K; a device that cannot (or an occupancy query that failed) runs the
        // CG on the two-pass schedule instead
        for (int K = 1; K <= vk::kOpMaxK && op_ok; ++K) {
            const int occ = vk::team_occupancy(c->opp, K);
            if ((int64_t)occ * c->cus < c->opp.grid) {
                std::fprintf(stderr, "libvampomi: one-pass operator off: %s fits %d workgroup(s) per CU; the plan "
                                     "needs %lld resident on %d CUs (two passes per CG step)\n",
                             vk::team_kernel_name(K, c->opp).c_str(), occ, (long long)c->opp.grid, c->cus);
                op_ok = false;
            }
        }
    }
    // the head-start plan: optional (no plan, or a grid the device cannot
    // hold, only means the solves start without it)
    bool hs_ok = op_ok && vk::team_plain_plan(c->N, M, c->cus, c->opp, &c->opp_hs);
    if (hs_ok && (int64_t)vk::team_occupancy(c->opp_hs, 1 + vk::kOpPlain) * c->cus < c->opp_hs.grid) hs_ok = false;
    c->op_ok_mine = op_ok;
    c->hs_ok_mine = hs_ok;
    if (!c->op_ts && std::getenv("VAMPOMI_OP_TS") && std::atoi(std::getenv("VAMPOMI_OP_TS"))) {
        HIPCHK(hipMalloc((void**)&c->op_ts, (size_t)4 * 8 * std::max(c->cus, 1) * 2));
        HIPCHK(hipMemsetAsync(c->op_ts, 0, (size_t)4 * 8 * std::max(c->cus, 1) * 2, c->st));
    }
    if (!c->op_nvec) {
        STCHK(dev_alloc(&c->op_nvec, (size_t)3 * vk::kMaxRhs * c->ld + 16));
        HIPCHK(hipMemsetAsync(c->op_nvec, 0, ((size_t)3 * vk::kMaxRhs * c->ld + 16) * 8, c->st));
    }
    if (op_ok) {
        const int64_t slots = std::max<int64_t>(c->opp.nslots, hs_ok ? c->opp_hs.nslots : 0);
        if (slots > c->op_part_slots) {
            dev_free(c->op_part);
            STCHK(dev_alloc(&c->op_part, (size_t)slots * vk::kMaxRhs * c->ld));
            c->op_part_slots = slots;
        }
        if (c->opp.T > 1 || (hs_ok && c->opp_hs.T > 1)) {
            size_t words = c->opp.T > 1 ? op_xg_words_for(M, c->opp) : 0;
            if (hs_ok && c->opp_hs.T > 1) words = std::max(words, op_xg_words_for(M, c->opp_hs));
            if (words > c->op_xg_words) {
                if (c->op_xg) (void)hipFree(c->op_xg);
                c->op_xg = nullptr;
                c->op_xg_words = 0;
                HIPCHK(hipMalloc((void**)&c->op_xg, words * 8));
                HIPCHK(hipMemsetAsync(c->op_xg, 0, words * 8, c->st));  // tags start below every launch's
                c->op_xg_words = words;
            }
        }
    }
    c->op_ready = true;
    return VAMPOMI_OK;
}

vampomi_status op_prepare(vampomi_ctx* c) {
    if (!c->op_ready) STCHK(op_plan_local(c));
    if (!c->use_comm) {
        c->op_ok = c->op_ok_mine;
        c->hs_ok = c->hs_ok_mine && c->hs_on;
    } else if (!c->op_agreed) {  // no agreement yet: the two-pass schedule, the same on every rank
        c->op_ok = c->hs_ok = false;
    }
    return VAMPOMI_OK;
}

vampomi_status op_agree(vampomi_ctx* c) {
    if (!c->use_comm) return VAMPOMI_OK;
    if (c->op_variant_req != c->op_variant || c->hs_on_req != c->hs_on) {
        c->op_variant = c->op_variant_req;
        c->hs_on = c->hs_on_req;
        c->op_ready = false;
    }
    bool op = false, hs = false;
    if (c->have_X) {
        if (!c->op_ready) STCHK(op_plan_local(c));
        op = c->op_ok_mine;
        hs = c->hs_ok_mine;
    }
    // one all-reduce of the four refusals, each in its own base-2^10 digit (a
    // digit counts the ranks that refuse: up to 1023 ranks); VAMPOMI_MR_TAIL
    // changes the tail's collective sequence too (vamp.cpp), so it is agreed
    // here with the others: the host-free tail only if every rank has it on
    const double mine = (op ? 0.0 : 1.0) + (hs ? 0.0 : 1024.0) + (c->hs_on ? 0.0 : 1048576.0) +
                        (c->mr_tail_req ? 0.0 : 1073741824.0);
    double all = 0.0;
    STCHK(sum_over_ranks(c, mine, &all));
    const int64_t a = (int64_t)all;
    c->op_ok = a % 1024 == 0;
    c->hs_ok = c->op_ok && (a / 1024) % 1024 == 0 && (a / 1048576) % 1024 == 0;
    c->mr_tail = a / 1073741824 == 0;
    c->op_agreed = true;
    return VAMPOMI_OK;
}

vampomi_status headstart_available(vampomi_ctx* c, bool* yes) {
    *yes = false;
    if (!c->have_X) return VAMPOMI_OK;
    STCHK(op_prepare(c));  // hs_ok: agreed over the ranks at vamp_begin, VAMPOMI_HEADSTART / set_variant(5) included
    *yes = c->op_ok && c->hs_ok;
    return VAMPOMI_OK;
}

// word 4 of the mapped flag block (zeroed at open)
unsigned* op_err_dev(vampomi_ctx* c) { return reinterpret_cast<unsigned*>(c->d_flag + 4); }

// A team launch needs every workgroup of its grid resident at once (one per
// CU).  Two of them running together on one device (contexts of one process
// on the same GPU, e.g. ranks as threads) could each hold part of the CUs and
// wait for members that never start, until the hand-off times out.  So while
// a process has several contexts on a device, their team launches are ordered
// by an event chain: each waits (on the device, no host sync) for the
// previous one.  With one context (the usual case) its stream orders them and
// no event is recorded: the chain's packets left the GPU idle after every
// operator launch (C2 kernel trace, operator -> cg_update: 6.7 -> 1.2 us).  When a
// second context appears, the next team launch first waits for everything
// already queued on the other contexts' streams (an event recorded on each).
struct TeamGate {
    std::mutex mu;
    hipEvent_t last = nullptr;          // the previous team launch (several contexts)
    std::vector<vampomi_ctx*> ctxs;     // live contexts on the device
    bool fence = false;                 // a context joined since the last team launch
};
static TeamGate g_team_gate[64];

static void team_gate_join(vampomi_ctx* c) {
    if (c->device < 0 || c->device >= 64) return;
    TeamGate& g = g_team_gate[c->device];
    std::lock_guard<std::mutex> lk(g.mu);
    if (hipEventCreateWithFlags(&c->team_ev, hipEventDisableTiming) != hipSuccess) c->team_ev = nullptr;
    g.ctxs.push_back(c);
    if (g.ctxs.size() > 1) g.fence = true;
    c->team_reg = true;
}

static void team_gate_leave(vampomi_ctx* c) {  // after the context's stream has drained
    if (!c->team_reg) return;
    TeamGate& g = g_team_gate[c->device];
    std::lock_guard<std::mutex> lk(g.mu);
    g.ctxs.erase(std::remove(g.ctxs.begin(), g.ctxs.end(), c), g.ctxs.end());
    if (c->team_ev) (void)hipEventDestroy(c->team_ev);
    c->team_ev = nullptr;
    c->team_reg = false;
}

// T: the launch's team size (its plan's)
template <class Launch>
static vampomi_status team_launch(vampomi_ctx* c, int T, Launch&& launch) {
    if (T <= 1 || !c->team_reg) {
        HIPCHK(launch());
        return VAMPOMI_OK;
    }
    TeamGate& g = g_team_gate[c->device];
    std::lock_guard<std::mutex> lk(g.mu);
    if (g.ctxs.size() <= 1) {  // one context: its stream orders its launches
        HIPCHK(launch());
        return VAMPOMI_OK;
    }
    if (g.fence) {  // behind everything the other contexts queued before (unchained launches included)
        for (vampomi_ctx* o : g.ctxs) {
            if (o == c) continue;
            if (!o->team_ev) return fail(VAMPOMI_ERR_HIP, "team gate: no event for a context");
            HIPCHK(hipEventRecord(o->team_ev, o->st));
            HIPCHK(hipStreamWaitEvent(c->st, o->team_ev, 0));
        }
        g.fence = false;
    } else if (g.last) {
        HIPCHK(hipStreamWaitEvent(c->st, g.last, 0));
    }
    HIPCHK(launch());
    if (!g.last) HIPCHK(hipEventCreateWithFlags(&g.last, hipEventDisableTiming));
    HIPCHK(hipEventRecord(g.last, c->st));
    return VAMPOMI_OK;
}

// reads and clears the word: each check reports the launches since the last
// one, so one timed-out launch does not fail every later solve of the context
vampomi_status op_check_err(vampomi_ctx* c) {
    const unsigned e = c->h_flag ? __atomic_exchange_n(reinterpret_cast<unsigned*>(c->h_flag + 4), 0u, __ATOMIC_ACQ_REL) : 0u;
    if (e > 1)  // TM_SAFE diagnostic builds: address-check codes above the flag bit
        return fail(VAMPOMI_ERR_HIP, "one-pass operator: address checks failed (codes " + std::to_string(e >> 1) + ")");
    if (e)
        return fail(VAMPOMI_ERR_HIP, "one-pass operator: a team hand-off timed out (a workgroup of the team never "
                                     "ran: fewer compute units than planned?)");
    return VAMPOMI_OK;
}

// One operator launch is charged SURVEY §8(d)'s bytes of ONE pass
// (pass_bytes: X once, K N-vectors, mave/msig, K M-vectors), the work it
// replaces being two such passes; its other traffic (p, z, d, A r, q_old and
// the per-slot A d partials, < 1% at C2) is not counted as algorithmic.
vampomi_status op_dev(vampomi_ctx* c, int K, const vk::OpArgs& a, const int* gate, bool reduce, bool divide) {
    if (!c->have_X) return fail(VAMPOMI_ERR_STATE, "A before the methylation data was loaded");
    STCHK(op_prepare(c));
    if (!c->op_ok || K < 1 || K > vk::kOpMaxK)
        return fail(VAMPOMI_ERR_ARG, "one-pass operator: K <= 2 and a plan for N = " + std::to_string(c->N));
    double* ad = c->op_nvec + (int64_t)2 * vk::kMaxRhs * c->ld;
    vk::OpArgs x = a;
    x.part = c->op_part;
    x.scale = 1.0 / c->sqrtN;
    if (c->opp.T > 1) {
        x.xg = c->op_xg;
        if (++c->op_tag == 0) ++c->op_tag;
        x.tag = c->op_tag;
        x.err = op_err_dev(c);
    }
    static const int dbg = std::getenv("VAMPOMI_OP_DBG") ? std::atoi(std::getenv("VAMPOMI_OP_DBG")) : 0;
    x.dbg = dbg;
    x.ts = c->op_ts;
    // <d,p>: one rank into scal[SL_DP+k]; several: behind the A d block, all-reduced with it
    x.ro = vk::RedOut{c->red_part, c->use_comm ? ad + (int64_t)K * c->ld : c->scal + SL_DP, c->ticket, nullptr, 0,
                      gate};
    TimedLaunch t = launch_stat(c, 3, K, pass_bytes(c, K), 2.0 * pass_flops(c, K));
    STCHK(team_launch(c, c->opp.T,
                      [&] { return vk::atax(c->shard(), c->opp, K, x, c->st, vk::Timing{t.a, t.b}, gate); }));
    c->stats.a_passes_exec++;
    vk::Ptrs os{};
    for (int k = 0; k < K; ++k) os.p[k] = ad + (int64_t)k * c->ld;
    if (!c->use_comm) {
        if (reduce) HIPCHK(vk::op_reduce(c->opp, K, c->N, c->ld, c->op_part, os, c->sqrtN, c->st, gate));
    } else {
        HIPCHK(vk::op_reduce(c->opp, K, c->N, c->ld, c->op_part, os, 0.0, c->st, gate));
        STCHK(allreduce_dev(c, ad, (size_t)K * c->ld + K));  // src/data.cpp:367
        if (divide) HIPCHK(vk::vec_div(K, c->N, c->ld, os, c->sqrtN, c->st));
    }
    return VAMPOMI_OK;
}

vampomi_status op_dev_plain(vampomi_ctx* c, const vk::OpArgs& a, const double* const* px, double* const* out,
                            const int* gate) {
    if (!c->have_X) return fail(VAMPOMI_ERR_STATE, "A before the methylation data was loaded");
    STCHK(op_prepare(c));
    if (!c->hs_ok) return fail(VAMPOMI_ERR_ARG, "head-start launch: no plan for N = " + std::to_string(c->N));
    constexpr int KT = 1 + vk::kOpPlain;  // partial slots: the system's A d, then the plain products
    double* ad = c->op_nvec + (int64_t)2 * vk::kMaxRhs * c->ld;
    vk::OpArgs x = a;
    x.part = c->op_part;
    x.scale = 1.0 / c->sqrtN;
    for (int k = 0; k < vk::kOpPlain; ++k) x.px.p[k] = px[k];
    if (c->opp_hs.T > 1) {
        x.xg = c->op_xg;
        if (++c->op_tag == 0) ++c->op_tag;
        x.tag = c->op_tag;
        x.err = op_err_dev(c);
    }
    x.dbg = 0;
    x.ro = vk::RedOut{c->red_part, c->use_comm ? ad + (int64_t)KT * c->ld : c->scal + SL_DP, c->ticket, nullptr, 0,
                      gate};
    TimedLaunch t = launch_stat(c, 3, KT, pass_bytes(c, KT), pass_flops(c, 1) + pass_flops(c, KT));
    STCHK(team_launch(c, c->opp_hs.T, [&] {
        return vk::atax_team_plain(c->shard(), c->opp_hs, x, c->st, vk::Timing{t.a, t.b}, gate);
    }));
    c->stats.a_passes_exec++;
    if (!c->use_comm) {
        vk::Ptrs os{};
        for (int k = 0; k < vk::kOpPlain; ++k) os.p[k] = out[k];
        HIPCHK(vk::op_reduce(c->opp_hs, vk::kOpPlain, c->N, c->ld, c->op_part, os, c->sqrtN, c->st, gate, 1));
    } else {
        vk::Ptrs os{};
        for (int k = 0; k < KT; ++k) os.p[k] = ad + (int64_t)k * c->ld;
        HIPCHK(vk::op_reduce(c->opp_hs, KT, c->N, c->ld, c->op_part, os, 0.0, c->st, gate));
        STCHK(allreduce_dev(c, ad, (size_t)KT * c->ld + 1));  // src/data.cpp:367
        // the system's A d divided in place, the plain products divided into their destinations (one launch)
        vk::Ptrs dst = os;
        for (int k = 0; k < vk::kOpPlain; ++k) dst.p[1 + k] = out[k];
        HIPCHK(vk::vec_div(KT, c->N, c->ld, os, c->sqrtN, c->st, &dst));
    }
    return VAMPOMI_OK;
}

// d_k = tau*A^T A v_k + gam2*v_k (lmmse_mult, src/vamp.cpp:645-662) for K
// vectors that are not all-zero; <d_k, v_k> lands in scal[SL_DP+k]. COLLECTIVE
vampomi_status lmmse_dev(vampomi_ctx* c, int K, const double* const* v, double* const* d, double tau,
                                double gam2, double* nscratch) {
    STCHK(ax_dev(c, K, v, nscratch));
    const double* u[vk::kMaxRhs];
    for (int k = 0; k < K; ++k) u[k] = nscratch + (int64_t)k * c->ld;
    return atx_dev(c, K, u, d, 1, tau, gam2, v);
}

// ---------------------------------------------------------------------------
// context lifecycle
// ---------------------------------------------------------------------------
extern "C" int vampomi_abi_version(void) { return VAMPOMI_ABI_VERSION; }
extern "C" const char* vampomi_last_error(void) { return g_err.c_str(); }

extern "C" void vampomi_divide_work(int64_t Mt, int nranks, int rank, int64_t* M, int64_t* S, int64_t* Mm) {
    // src/utilities.cpp:207-239
    const int64_t modu = Mt % nranks, size = Mt / nranks;
    int64_t cum = 0;
    for (int r = 0; r < nranks; ++r) {
        const int64_t len = r < modu ? size + 1 : size;
        if (r == rank) {
            if (M) *M = len;
            if (S) *S = cum;
        }
        cum += len;
    }
    if (Mm) *Mm = modu != 0 ? size + 1 : size;
}

extern "C" vampomi_status vampomi_comm_unique_id(void* out) {
    if (!out) return fail(VAMPOMI_ERR_ARG, "null argument");
    ncclUniqueId id;
    NCCLCHK(ncclGetUniqueId(&id));
    static_assert(sizeof(ncclUniqueId) == VAMPOMI_UNIQUE_ID_BYTES, "unique id size");
    std::memcpy(out, &id, sizeof id);
    return VAMPOMI_OK;
}

// releases everything the context owns (also on a failed vampomi_open);
// called by ~vampomi_ctx after the VAMP run state is gone
void release_ctx_resources(vampomi_ctx* c) {
    (void)hipSetDevice(c->device);
    if (c->st) (void)hipStreamSynchronize(c->st);
    team_gate_leave(c);
    resolve_timing(c);
    for (auto e : c->ev_pool) (void)hipEventDestroy(e);
    c->ev_pool.clear();
    for (double** p : {&c->X, &c->mave, &c->msig, &c->y, &c->ax_part, &c->red_part, &c->scal, &c->nbuf, &c->mbuf,
                       &c->op_part, &c->op_nvec})
        dev_free(*p);
    if (c->op_xg) (void)hipFree(c->op_xg);
    c->op_xg = nullptr;
    if (c->op_ts) (void)hipFree(c->op_ts);
    c->op_ts = nullptr;
    c->op_xg_words = 0;
    c->op_part_slots = 0;
    c->op_ready = false;
    c->op_agreed = false;
    if (c->h_scal) (void)hipHostFree(c->h_scal);
    c->h_scal = nullptr;
    if (c->ticket) (void)hipFree(c->ticket);
    c->ticket = nullptr;
    if (c->h_flag) (void)hipHostFree(c->h_flag);
    c->h_flag = nullptr;
    if (c->h_cgm) (void)hipHostFree(c->h_cgm);
    c->h_cgm = nullptr;
    if (c->cgs) (void)hipFree(c->cgs);
    c->cgs = nullptr;
    if (c->comm) {
        // a non-blocking communicator: finalize (flushes its pending work,
        // may return ncclInProgress), then destroy; abort if it never settles
        if (nccl_settle(c, ncclCommFinalize(c->comm), "ncclCommFinalize", 30.0) == VAMPOMI_OK && c->comm)
            (void)ncclCommDestroy(c->comm);
        else if (c->comm)
            (void)ncclCommAbort(c->comm);
    }
    c->comm = nullptr;

    if (c->st) (void)hipStreamDestroy(c->st);
    c->st = nullptr;
}

extern "C" void vampomi_close(vampomi_ctx* c) { delete c; }

extern "C" vampomi_status vampomi_open(const vampomi_shard_desc* d, vampomi_ctx** out) {
    if (!d || !out) return fail(VAMPOMI_ERR_ARG, "null argument");
    *out = nullptr;
    if (d->N < 2 || d->Mt < 1 || d->nranks < 1 || d->rank < 0 || d->rank >= d->nranks)
        return fail(VAMPOMI_ERR_ARG, "invalid shard description (N >= 2, Mt >= 1, 0 <= rank < nranks)");
    if (d->nranks > 1 && !d->comm_id) return fail(VAMPOMI_ERR_ARG, "nranks > 1 needs a communicator id");
    if (d->Mt < d->nranks) return fail(VAMPOMI_ERR_ARG, "every rank needs at least one marker (Mt >= nranks)");
    std::unique_ptr<vampomi_ctx> c(new vampomi_ctx());
    c->rank = d->rank;
    c->nranks = d->nranks;
    c->N = d->N;
    c->Mt = d->Mt;
    c->alpha_scale = d->alpha_scale == 0.0 ? 1.0 : d->alpha_scale;
    vampomi_divide_work(c->Mt, c->nranks, c->rank, &c->M, &c->S, &c->Mm);
    c->ld = (c->N + 15) / 16 * 16;  // 128-byte aligned columns
    c->sqrtN = std::sqrt((double)c->N);
    int ndev = 0;
    HIPCHK(hipGetDeviceCount(&ndev));
    if (ndev < 1) return fail(VAMPOMI_ERR_HIP, "no HIP device visible");
    c->device = d->device >= 0 ? d->device : c->rank % ndev;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking));
    team_gate_join(c.get());
    const int64_t Mx = std::max<int64_t>(c->M, 1);
    c->axp = vk::ax_plan(c->N, Mx);
    STCHK(dev_alloc(&c->mave, Mx));
    STCHK(dev_alloc(&c->msig, Mx));
    STCHK(dev_alloc(&c->y, c->ld));
    HIPCHK(hipMemsetAsync(c->y, 0, c->ld * 8, c->st));
    STCHK(dev_alloc(&c->ax_part, (size_t)c->axp.nslots * vk::kMaxRhs * c->ld));
    c->red_cap = red_capacity(Mx);
    STCHK(dev_alloc(&c->red_part, c->red_cap));
    c->writer.reset(new IterWriter());  // the per-iteration output (writer.h): staging and thread now
    STCHK(c->writer->open(c.get()));
    STCHK(dev_alloc(&c->scal, SL_TOTAL));
    HIPCHK(hipHostMalloc((void**)&c->h_scal, SL_TOTAL * sizeof(double), hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(hipHostGetDevicePointer((void**)&c->d_hscal, c->h_scal, 0));
    HIPCHK(hipHostMalloc((void**)&c->h_flag, 64, hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(c->h_flag, 0, 64);  // word 0: stream sync sequence; word 4: operator hand-off error
    HIPCHK(hipHostGetDevicePointer((void**)&c->d_flag, c->h_flag, 0));
    HIPCHK(hipMalloc((void**)&c->ticket, 64 * sizeof(unsigned)));
    HIPCHK(hipMemsetAsync(c->ticket, 0, 64 * sizeof(unsigned), c->st));
    STCHK(dev_alloc(&c->nbuf, (size_t)vk::kMaxRhs * c->ld));
    HIPCHK(hipMemsetAsync(c->nbuf, 0, (size_t)vk::kMaxRhs * c->ld * 8, c->st));
    STCHK(dev_alloc(&c->mbuf, (size_t)2 * vk::kMaxRhs * Mx));
    HIPCHK(hipMalloc((void**)&c->cgs, 2 * sizeof(vk::CgState)));  // [1]: the folded decisions' second state (pcg.cpp)
    HIPCHK(hipMemsetAsync(c->cgs, 0, 2 * sizeof(vk::CgState), c->st));
    HIPCHK(hipHostMalloc((void**)&c->h_cgm, vk::kCgMirrorSlots * sizeof(vk::CgMirror),
                         hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(c->h_cgm, 0, vk::kCgMirrorSlots * sizeof(vk::CgMirror));
    HIPCHK(hipHostGetDevicePointer((void**)&c->d_cgm, c->h_cgm, 0));
    // VAMPOMI_FORCE_RCCL=1 runs a 1-rank job through the multi-rank code path
    // (RCCL communicator, all-reduces, post-reduce division) so that path can
    // be exercised on a single GPU
    const char* force = std::getenv("VAMPOMI_FORCE_RCCL");
    c->use_comm = c->nranks > 1 || (force && std::atoi(force) != 0);
    if (const char* mv = std::getenv("VAMPOMI_MR_TAIL")) c->mr_tail = c->mr_tail_req = std::atoi(mv) != 0;
    if (const char* fv = std::getenv("VAMPOMI_CG_FOLD")) c->cg_fold = std::atoi(fv) != 0;
    if (const char* hv = std::getenv("VAMPOMI_HEADSTART")) c->hs_on = c->hs_on_req = std::atoi(hv) != 0;
    const char* mode = std::getenv("VAMPOMI_COMM");
    if (c->use_comm && mode && std::strcmp(mode, "loopback") == 0) {
        if (!d->comm_id) return fail(VAMPOMI_ERR_ARG, "the loopback communicator needs a communicator id");
        c->loopback = loopback_join(d->comm_id, c->nranks);
    } else if (c->use_comm && mode && std::strcmp(mode, "shm") == 0) {
        if (!d->comm_id) return fail(VAMPOMI_ERR_ARG, "the shm communicator needs a communicator id");
        std::string err;
        c->shm = shm_join(d->comm_id, c->nranks, c->rank, comm_init_timeout_s(), &err);
        if (!c->shm) return fail(VAMPOMI_ERR_STATE, err);
    } else if (c->use_comm) {
        ncclUniqueId id;
        if (d->comm_id)
            std::memcpy(&id, d->comm_id, sizeof id);
        else
            NCCLCHK(ncclGetUniqueId(&id));
        // non-blocking creation, bounded: the bootstrap waits for every rank,
        // so a rank that never arrives fails this one after
        // VAMPOMI_COMM_INIT_TIMEOUT_S instead of hanging the job
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        cfg.blocking = 0;
        STCHK(nccl_settle(c.get(), ncclCommInitRankConfig(&c->comm, c->nranks, id, c->rank, &cfg),
                          "ncclCommInitRankConfig", comm_init_timeout_s()));
    }
    STCHK(sync_stream(c.get(), c->st));
    *out = c.release();
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_shard_info(const vampomi_ctx* c, int64_t* M, int64_t* S, int64_t* ld) {
    if (!c) return fail(VAMPOMI_ERR_ARG, "null context");
    if (M) *M = c->M;
    if (S) *S = c->S;
    if (ld) *ld = c->ld;
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_sync(vampomi_ctx* c) {
    if (!c) return fail(VAMPOMI_ERR_ARG, "null context");
    HIPCHK(hipSetDevice(c->device));
    STCHK(sync_stream(c, c->st));
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_barrier(vampomi_ctx* c) {
    CollScope cs_(c);
    if (!c) return fail(VAMPOMI_ERR_ARG, "null context");
    if (c->use_comm) STCHK(allreduce_dev(c, c->scal + SL_BARRIER, 1));
    STCHK(sync_stream(c, c->st));
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_barrier_timeout(vampomi_ctx* c, double seconds) {
    if (!c || !(seconds > 0)) return fail(VAMPOMI_ERR_ARG, "null context or no limit");
    c->coll_limit_s = seconds;
    const vampomi_status st = vampomi_barrier(c);
    c->coll_limit_s = 0.0;
    return st;
}

// ---------------------------------------------------------------------------
// data ingest
// ---------------------------------------------------------------------------
static vampomi_status ensure_X(vampomi_ctx* c) {
    if (c->X) return VAMPOMI_OK;
    return dev_alloc(&c->X, (size_t)std::max<int64_t>(c->M, 1) * (size_t)c->ld);
}

static vampomi_status finish_X(vampomi_ctx* c) {
    if (c->ld > c->N && c->M > 0)
        HIPCHK(hipMemset2DAsync(c->X + c->N, (size_t)c->ld * 8, 0, (size_t)(c->ld - c->N) * 8, (size_t)c->M, c->st));
    // compute_markers_statistics with nonas = N (read_phen asserts N rows, src/data.cpp:85)
    HIPCHK(vk::marker_stats(c->X, c->ld, c->N, c->M, (double)c->N, c->alpha_scale, c->mave, c->msig, c->st));
    STCHK(sync_stream(c, c->st));
    c->have_X = true;
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_load_meth_host(vampomi_ctx* c, const double* X, int64_t ld_in) {
    if (!c || (!X && c->M > 0) || ld_in < c->N) return fail(VAMPOMI_ERR_ARG, "invalid host shard");
    HIPCHK(hipSetDevice(c->device));
    STCHK(ensure_X(c));
    if (c->M > 0)
        HIPCHK(hipMemcpy2DAsync(c->X, (size_t)c->ld * 8, X, (size_t)ld_in * 8, (size_t)c->N * 8, (size_t)c->M,
                                hipMemcpyHostToDevice, c->st));
    return finish_X(c);
}

// [off, off + want) of fd into dst, split over nt reader threads (page cache
// and NVMe both need several requests in flight to stream at full rate)
static bool pread_parallel(int fd, char* dst, size_t want, off_t off, int nt) {
    if (nt <= 1 || want < ((size_t)8 << 20)) nt = 1;
    const size_t per = ((want + nt - 1) / nt + 4095) & ~(size_t)4095;
    std::atomic<bool> ok{true};
    auto work = [&](size_t lo, size_t hi) {
        size_t got = 0;
        while (lo + got < hi) {
            const ssize_t r = ::pread(fd, dst + lo + got, hi - lo - got, off + (off_t)(lo + got));
            if (r <= 0) {
                ok = false;
                return;
            }
            got += (size_t)r;
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) {
        const size_t lo = (size_t)t * per;
        if (lo < want) th.emplace_back(work, lo, std::min(want, lo + per));
    }
    work(0, std::min(want, per));
    for (auto& x : th) x.join();
    return ok;
}

// read_methylation_data (src/data.cpp:116-153): this rank's M*N doubles at byte
// offset S*N*8 (64-bit offsets: the reference's int i*N overflows past 2^31
// elements), streamed through three pinned 256 MB staging buffers: the
// parallel read of chunk k+1 overlaps the host-to-device copy of chunk k,
// which lands directly in the ld-padded column layout.  Marker statistics
// follow on the device (finish_X).
extern "C" vampomi_status vampomi_load_meth_file(vampomi_ctx* c, const char* path) {
    if (!c || !path) return fail(VAMPOMI_ERR_ARG, "null argument");
    HIPCHK(hipSetDevice(c->device));
    int fd = ::open(path, O_RDONLY);
    if (fd < 0) return fail(VAMPOMI_ERR_IO, std::string("cannot open methylation file ") + path);
    STCHK(ensure_X(c));
    const size_t colb = (size_t)c->N * 8;
    const size_t chunk_cols = std::max<size_t>(1, ((size_t)256 << 20) / colb);
    const char* env = std::getenv("VAMPOMI_IO_THREADS");
    const int nt = env ? std::max(1, std::atoi(env)) : (int)std::min(8u, std::max(1u, std::thread::hardware_concurrency()));
    constexpr int NB = 3;
    double* pin[NB] = {};
    hipEvent_t done[NB];
    bool used[NB] = {};
    for (int b = 0; b < NB; ++b) {
        if (hipHostMalloc((void**)&pin[b], chunk_cols * colb, hipHostMallocDefault) != hipSuccess) {
            for (int k = 0; k < b; ++k) (void)hipHostFree(pin[k]);
            ::close(fd);
            return fail(VAMPOMI_ERR_OOM, "pinned staging buffer");
        }
        (void)hipEventCreate(&done[b]);
    }
    vampomi_status st = VAMPOMI_OK;
    int64_t i0 = 0;
    int b = 0;
    while (i0 < c->M && st == VAMPOMI_OK) {
        const int64_t nc = std::min<int64_t>((int64_t)chunk_cols, c->M - i0);
        if (used[b]) (void)hipEventSynchronize(done[b]);
        const size_t want = (size_t)nc * colb;
        const off_t off = (off_t)(c->S + i0) * (off_t)colb;
        if (!pread_parallel(fd, (char*)pin[b], want, off, nt)) {
            st = fail(VAMPOMI_ERR_IO, std::string("short read from methylation file ") + path);
            break;
        }
        if (hipMemcpy2DAsync(c->X + i0 * c->ld, (size_t)c->ld * 8, pin[b], colb, colb, (size_t)nc, hipMemcpyHostToDevice,
                             c->st) != hipSuccess ||
            hipEventRecord(done[b], c->st) != hipSuccess) {
            st = fail(VAMPOMI_ERR_HIP, "host-to-device copy of the methylation shard");
            break;
        }
        used[b] = true;
        i0 += nc;
        b = (b + 1) % NB;
    }
    (void)hipStreamSynchronize(c->st);
    for (int k = 0; k < NB; ++k) {
        (void)hipHostFree(pin[k]);
        (void)hipEventDestroy(done[k]);
    }
    ::close(fd);
    if (st != VAMPOMI_OK) return st;
    return finish_X(c);
}

extern "C" vampomi_status vampomi_generate_meth(vampomi_ctx* c, uint64_t seed, int kind) {
    if (!c || (kind != VAMPOMI_GEN_GAUSS && kind != VAMPOMI_GEN_METH)) return fail(VAMPOMI_ERR_ARG, "bad argument");
    HIPCHK(hipSetDevice(c->device));
    STCHK(ensure_X(c));
    HIPCHK(vk::gen_markers(seed, kind, c->N, c->ld, c->S, c->M, c->X, c->st));
    return finish_X(c);
}

static vampomi_status upload_phen(vampomi_ctx* c) {
    HIPCHK(hipMemcpyAsync(c->y, c->y_host.data(), (size_t)c->N * 8, hipMemcpyHostToDevice, c->st));
    STCHK(sync_stream(c, c->st));
    c->have_y = true;
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_read_phen(vampomi_ctx* c, const char* path, int standardize) {
    if (!c || !path) return fail(VAMPOMI_ERR_ARG, "null argument");
    HIPCHK(hipSetDevice(c->device));
    std::vector<double> y;
    const int64_t n = vio::read_phen(path, y);
    if (n == -1) return fail(VAMPOMI_ERR_IO, std::string("FATAL: could not open phenotype file: ") + path);
    if (n == -2) return fail(VAMPOMI_ERR_NAN_PHEN, "NAN in data!");
    if (n != c->N)
        return fail(VAMPOMI_ERR_ARG, "phenotype rows (" + std::to_string(n) + ") != N (" + std::to_string(c->N) + ")");
    if (standardize) vio::standardize_phen(y);
    c->y_host = y;
    return upload_phen(c);
}

extern "C" vampomi_status vampomi_set_phen(vampomi_ctx* c, const double* y, int standardize) {
    if (!c || !y) return fail(VAMPOMI_ERR_ARG, "null argument");
    HIPCHK(hipSetDevice(c->device));
    c->y_host.assign(y, y + c->N);
    if (standardize) vio::standardize_phen(c->y_host);
    return upload_phen(c);
}

extern "C" vampomi_status vampomi_get_phen(vampomi_ctx* c, double* y) {
    if (!c || !y) return fail(VAMPOMI_ERR_ARG, "null argument");
    if (!c->have_y) return fail(VAMPOMI_ERR_STATE, "no phenotype loaded");
    std::memcpy(y, c->y_host.data(), (size_t)c->N * 8);
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_get_marker_stats(vampomi_ctx* c, double* mave, double* msig) {
    if (!c) return fail(VAMPOMI_ERR_ARG, "null context");
    if (!c->have_X) return fail(VAMPOMI_ERR_STATE, "no methylation data loaded");
    HIPCHK(hipSetDevice(c->device));
    if (mave && c->M > 0) HIPCHK(hipMemcpyAsync(mave, c->mave, (size_t)c->M * 8, hipMemcpyDeviceToHost, c->st));
    if (msig && c->M > 0) HIPCHK(hipMemcpyAsync(msig, c->msig, (size_t)c->M * 8, hipMemcpyDeviceToHost, c->st));
    STCHK(sync_stream(c, c->st));
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_read_markers(vampomi_ctx* c, int64_t i0, int64_t count, double* out) {
    if (!c || !out || i0 < 0 || count < 0 || i0 + count > c->M) return fail(VAMPOMI_ERR_ARG, "bad marker range");
    if (!c->have_X) return fail(VAMPOMI_ERR_STATE, "no methylation data loaded");
    HIPCHK(hipSetDevice(c->device));
    if (count > 0)
        HIPCHK(hipMemcpy2DAsync(out, (size_t)c->N * 8, c->X + i0 * c->ld, (size_t)c->ld * 8, (size_t)c->N * 8,
                                (size_t)count, hipMemcpyDeviceToHost, c->st));
    STCHK(sync_stream(c, c->st));
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_simulate_phen(vampomi_ctx* c, uint64_t seed, double lam, double h2, double* beta_out) {
    CollScope cs_(c);
    if (!c || !c->have_X) return fail(VAMPOMI_ERR_STATE, "load methylation data first");
    HIPCHK(hipSetDevice(c->device));
    double* beta = c->mbuf;
    const int64_t M = c->M;
    double cm = 0.0;
    DotBatch db(c);
    vk::RedOut ro{};
    STCHK(db.sink(1, true, &cm, &ro));  // CM summed over ranks
    HIPCHK(vk::gen_beta(seed, lam, c->S, M, beta, ro, c->st));
    STCHK(db.flush());
    if (cm > 0) HIPCHK(vk::scale_vec(M, beta, std::sqrt(h2 / cm), c->st));  // sigma2 = h2 / CM (data_sim.py:39)
    if (beta_out && M > 0) {
        HIPCHK(hipMemcpyAsync(beta_out, beta, (size_t)M * 8, hipMemcpyDeviceToHost, c->st));
    }
    double* bs = c->mbuf + std::max<int64_t>(M, 1);
    HIPCHK(vk::axpby(M, c->sqrtN, beta, 0.0, beta, bs, c->st));  // Ax divides by sqrt(N)
    const double* xs[1] = {bs};
    STCHK(ax_dev(c, 1, xs, c->nbuf));
    HIPCHK(vk::add_noise(seed, c->N, std::sqrt(1.0 - h2), c->nbuf, c->st));  // data_sim.py:47
    std::vector<double> y((size_t)c->N);
    HIPCHK(hipMemcpyAsync(y.data(), c->nbuf, (size_t)c->N * 8, hipMemcpyDeviceToHost, c->st));
    STCHK(host_sync(c));
    vio::standardize_phen(y);
    c->y_host = y;
    return upload_phen(c);
}

extern "C" vampomi_status vampomi_simulate_phen_binary(vampomi_ctx* c, uint64_t seed, double lam, double h2,
                                                       double* beta_out) {
    STCHK(vampomi_simulate_phen(c, seed, lam, h2, beta_out));
    for (double& v : c->y_host) v = v > 0 ? 1.0 : 0.0;  // the scaling is positive: same sign as the liability
    return upload_phen(c);
}

// ---------------------------------------------------------------------------
// operator entry points
// ---------------------------------------------------------------------------
static vampomi_status stage_in(vampomi_ctx* c, const double* src, int64_t n, int mem, double* dst) {
    if (n <= 0) return VAMPOMI_OK;
    HIPCHK(hipMemcpyAsync(dst, src, (size_t)n * 8, mem == VAMPOMI_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                          c->st));
    return VAMPOMI_OK;
}

static vampomi_status stage_out(vampomi_ctx* c, const double* src, int64_t n, int mem, double* dst) {
    if (n > 0)
        HIPCHK(hipMemcpyAsync(dst, src, (size_t)n * 8, mem == VAMPOMI_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost,
                              c->st));
    STCHK(sync_stream(c, c->st));
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_ax(vampomi_ctx* c, const double* x, double* out, int mem) {
    CollScope cs_(c);
    if (!c || (!x && c->M > 0) || !out) return fail(VAMPOMI_ERR_ARG, "null argument");
    HIPCHK(hipSetDevice(c->device));
    STCHK(stage_in(c, x, c->M, mem, c->mbuf));
    const double* xs[1] = {c->mbuf};
    STCHK(ax_dev(c, 1, xs, c->nbuf));
    STCHK(stage_out(c, c->nbuf, c->N, mem, out));
    if (c->timing) resolve_timing(c);
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_atx(vampomi_ctx* c, const double* u, double* out, int mem) {
    if (!c || !u || (!out && c->M > 0)) return fail(VAMPOMI_ERR_ARG, "null argument");
    HIPCHK(hipSetDevice(c->device));
    STCHK(stage_in(c, u, c->N, mem, c->nbuf));  // pad rows of nbuf stay zero
    const double* us[1] = {c->nbuf};
    double* os[1] = {c->mbuf};
    STCHK(atx_dev(c, 1, us, os, 0, 0.0, 0.0, nullptr));
    STCHK(stage_out(c, c->mbuf, c->M, mem, out));
    if (c->timing) resolve_timing(c);
    return VAMPOMI_OK;
}

static bool host_all_zero(const double* v, int64_t n) {
    for (int64_t i = 0; i < n; ++i)
        if (v[i] != 0.0) return false;
    return true;
}

// Is v zero on EVERY rank?  The reference tests its local slice only
// (src/vamp.cpp:647-648) and then skips Ax and its MPI_Allreduce: a rank whose
// slice is zero while another's is not leaves the other ranks waiting.  Here the
// ranks count their non-zero slices together (COLLECTIVE), so they all take the
// same branch; on one rank this is the reference's test.
static vampomi_status is_zero_vec(vampomi_ctx* c, const double* v, int64_t n, int mem, bool* z) {
    bool local = true;
    if (mem == VAMPOMI_MEM_HOST) {
        local = host_all_zero(v, n);
    } else {
        std::vector<double> h((size_t)std::max<int64_t>(n, 1));
        if (n > 0) HIPCHK(hipMemcpyAsync(h.data(), v, (size_t)n * 8, hipMemcpyDeviceToHost, c->st));
        STCHK(sync_stream(c, c->st));
        local = host_all_zero(h.data(), n);
    }
    double nonzero = 0.0;
    STCHK(sum_over_ranks(c, local ? 0.0 : 1.0, &nonzero));
    *z = nonzero == 0.0;
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_lmmse_mult(vampomi_ctx* c, const double* v, double tau, double gam2, double* out,
                                             int mem) {
    CollScope cs_(c);
    if (!c || (c->M > 0 && (!v || !out))) return fail(VAMPOMI_ERR_ARG, "null argument");
    HIPCHK(hipSetDevice(c->device));
    bool zero = false;
    STCHK(is_zero_vec(c, v, c->M, mem, &zero));  // src/vamp.cpp:647-648 (local check)
    double* vin = c->mbuf;
    double* d = c->mbuf + std::max<int64_t>(c->M, 1);
    if (zero) {
        HIPCHK(hipMemsetAsync(d, 0, (size_t)std::max<int64_t>(c->M, 1) * 8, c->st));
    } else {
        STCHK(stage_in(c, v, c->M, mem, vin));
        const double* vs[1] = {vin};
        double* ds[1] = {d};
        STCHK(lmmse_dev(c, 1, vs, ds, tau, gam2, c->nbuf));
    }
    STCHK(stage_out(c, d, c->M, mem, out));
    if (c->timing) resolve_timing(c);
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_pcg(vampomi_ctx* c, const double* v, const double* mu0, double tau, double gam2,
                                      int onsager, int max_iter, double tol, double* mu, int* iters, int mem) {
    CollScope cs_(c);
    if (!c || (c->M > 0 && (!v || !mu))) return fail(VAMPOMI_ERR_ARG, "null argument");
    HIPCHK(hipSetDevice(c->device));
    const int64_t Mx = std::max<int64_t>(c->M, 1);
    double* w = c->mbuf;  // 8*Mx: v, mu, r, z, p, d
    CgSystem s{};
    s.v = w;
    s.mu = w + Mx;
    s.r = w + 2 * Mx;
    s.z = w + 3 * Mx;
    s.p = w + 4 * Mx;
    s.d = w + 5 * Mx;
    s.onsager = onsager != 0;
    STCHK(stage_in(c, v, c->M, mem, w));
    bool zero = true;  // no mu0 on this rank: zeros (still counted with the others)
    if (mu0 || c->use_comm) STCHK(is_zero_vec(c, mu0, mu0 ? c->M : 0, mem, &zero));
    // zero is collective (every rank runs the same lmmse pass), but only a rank
    // that holds mu0 stages it in: the others start from a zero local slice
    s.mu0_nonzero = !zero;
    if (zero || !mu0)
        HIPCHK(hipMemsetAsync(s.mu, 0, (size_t)Mx * 8, c->st));
    else
        STCHK(stage_in(c, mu0, c->M, mem, s.mu));
    STCHK(pcg_run(c, {&s}, tau, gam2, max_iter, tol, c->nbuf, nullptr, nullptr));
    STCHK(stage_out(c, s.mu, c->M, mem, mu));
    if (iters) *iters = s.iters;
    if (c->timing) resolve_timing(c);
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_denoise(vampomi_ctx* c, const double* r1, double gam1, const double* probs,
                                          const double* vars, int L, double* x1, double* x1d, double* sum_d, int mem) {
    CollScope cs_(c);
    if (!c || !probs || !vars || L < 1 || L > VAMPOMI_MAX_L) return fail(VAMPOMI_ERR_ARG, "bad argument");
    HIPCHK(hipSetDevice(c->device));
    const int64_t Mx = std::max<int64_t>(c->M, 1);
    double* rin = c->mbuf;
    double* xo = c->mbuf + Mx;
    double* xd = c->mbuf + 2 * Mx;
    STCHK(stage_in(c, r1, c->M, mem, rin));
    vk::Mix mix{};
    mix.L = L;
    for (int j = 0; j < L; ++j) {
        mix.probs[j] = probs[j];
        mix.vars[j] = vars[j];
    }
    double sd = 0.0;
    DotBatch db(c);
    vk::RedOut ro{};
    STCHK(db.sink(1, true, &sd, &ro));
    HIPCHK(vk::denoise(c->M, rin, gam1, mix, xo, rin, 0, 1.0, xd, ro, c->st));
    STCHK(db.flush());
    if (x1) STCHK(stage_out(c, xo, c->M, mem, x1));
    if (x1d) STCHK(stage_out(c, xd, c->M, mem, x1d));
    if (sum_d) *sum_d = sd;
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_denoise_bin(vampomi_ctx* c, const double* p1, double tau1, double* z1,
                                              double* sum_d, int mem) {
    if (!c || !p1) return fail(VAMPOMI_ERR_ARG, "null argument");
    if (!c->have_y) return fail(VAMPOMI_ERR_STATE, "set the phenotype first");
    HIPCHK(hipSetDevice(c->device));
    double* pin = c->nbuf;
    double* zo = c->nbuf + c->ld;
    STCHK(stage_in(c, p1, c->N, mem, pin));
    double sd = 0.0;
    DotBatch db(c);
    vk::RedOut ro{};
    STCHK(db.sink(1, false, &sd, &ro));
    HIPCHK(vk::probit_denoise(c->N, pin, c->y, tau1, zo, ro, c->st));
    STCHK(db.flush());
    if (z1) STCHK(stage_out(c, zo, c->N, mem, z1));
    if (sum_d) *sum_d = sd;
    return VAMPOMI_OK;
}

// --run-mode association_test --pval-method loo (src/main_meth.cpp:245-264,
// data::pvals_loo src/data.cpp:385-417).  COLLECTIVE (one A.x).
extern "C" vampomi_status vampomi_assoc_loo(vampomi_ctx* c, const double* est, double* pvals, double* stats,
                                            int mem) {
    CollScope cs_(c);
    if (!c || (!est && c->M > 0)) return fail(VAMPOMI_ERR_ARG, "null argument");
    if (!c->have_X || !c->have_y) return fail(VAMPOMI_ERR_STATE, "load methylation data and phenotype first");
    HIPCHK(hipSetDevice(c->device));
    const int64_t M = c->M, N = c->N, Mx = std::max<int64_t>(M, 1), ld = c->ld;
    double* e = c->mbuf;            // estimate-file values
    double* x1 = c->mbuf + Mx;      // x1_hat * sqrt(N)
    double* pv = c->mbuf + 2 * Mx;  // p-values
    double* st = c->mbuf + 3 * Mx;  // 5 sums per marker (slots 3..7)
    double* z1 = c->nbuf;
    double* ymod = c->nbuf + ld;
    STCHK(stage_in(c, est, M, mem, e));
    HIPCHK(vk::mul_scalar(M, e, std::sqrt((double)N), x1, c->st));  // :254-255
    const double* xs[1] = {x1};
    STCHK(ax_dev(c, 1, xs, z1));                                     // :257
    HIPCHK(vk::axpby(N, 1.0, c->y, -1.0, z1, ymod, c->st));          // y_mod = y - z1 (data.cpp:390-391)
    if (ld > N) HIPCHK(hipMemsetAsync(ymod + N, 0, (size_t)(ld - N) * 8, c->st));
    // raw X once, ymod, x1, the five sums; per element 1 div, 2 mul + 1 add
    // for ym, 5 accumulations (3 of them products)
    TimedLaunch t = launch_stat(c, 2, 1, 8.0 * (double)N * (double)M + 8.0 * (double)N + 8.0 * 6.0 * (double)M,
                                11.0 * (double)N * (double)M);
    HIPCHK(vk::loo_sums(c->shard(), ymod, x1, std::sqrt((double)N), st, c->st, c->loo_variant, vk::Timing{t.a, t.b}));  // :393-416
    c->stats.a_passes_exec++;
    HIPCHK(vk::loo_pvals(M, st, (int)N, pv, c->st));
    if (stats) STCHK(stage_out(c, st, 5 * M, mem, stats));
    if (pvals) STCHK(stage_out(c, pv, M, mem, pvals));
    STCHK(sync_stream(c, c->st));
    if (c->timing) resolve_timing(c);
    return VAMPOMI_OK;
}

// --run-mode test (src/main_meth.cpp:165-199): one estimate's R2 test and
// squared correlation on the context's (test) data set.  COLLECTIVE (one A.x).
extern "C" vampomi_status vampomi_test_metrics(vampomi_ctx* c, const double* est, double* r2, double* corr2,
                                               int mem) {
    CollScope cs_(c);
    if (!c || (!est && c->M > 0)) return fail(VAMPOMI_ERR_ARG, "null argument");
    if (!c->have_X || !c->have_y) return fail(VAMPOMI_ERR_STATE, "load methylation data and phenotype first");
    HIPCHK(hipSetDevice(c->device));
    const int64_t M = c->M, N = c->N, Mx = std::max<int64_t>(M, 1);
    STCHK(stage_in(c, est, M, mem, c->mbuf));
    HIPCHK(vk::mul_scalar(M, c->mbuf, std::sqrt((double)N), c->mbuf + Mx, c->st));  // :172-174
    const double* xs[1] = {c->mbuf + Mx};
    double* z = c->nbuf;
    STCHK(ax_dev(c, 1, xs, z));  // :177
    double s[5] = {};
    DotBatch b(c);  // the N-side is replicated: local sums (inner_prod(., 1)'s rank factor cancels)
    STCHK(b.add({T(c->y, z, vk::DIFF2), T(c->y, nullptr, vk::SUM), T(c->y, c->y), T(z, c->y), T(z, z)}, N, false, s));
    STCHK(b.flush());
    const double mean = s[1] / (double)N;                                                  // calc_stdev
    const double stdev = std::sqrt((s[2] - (double)N * mean * mean) / (double)(N - 1));  // utilities.cpp:202
    if (r2) *r2 = 1 - s[0] / (stdev * stdev * (double)N);                                  // :187
    const double corr = s[3] / std::sqrt(s[4] * s[2]);                                     // :190
    if (corr2) *corr2 = corr * corr;
    if (c->timing) resolve_timing(c);
    return VAMPOMI_OK;
}

// --pval-method se (src/main_meth.cpp:218-242): rank-local
extern "C" vampomi_status vampomi_assoc_se(vampomi_ctx* c, const double* r1, double gam1, double* pvals, int mem) {
    if (!c || (!r1 && c->M > 0) || (!pvals && c->M > 0)) return fail(VAMPOMI_ERR_ARG, "null argument");
    HIPCHK(hipSetDevice(c->device));
    const int64_t Mx = std::max<int64_t>(c->M, 1);
    STCHK(stage_in(c, r1, c->M, mem, c->mbuf));
    HIPCHK(vk::se_pvals(c->M, c->mbuf, gam1, c->N, c->mbuf + Mx, c->st));
    STCHK(stage_out(c, c->mbuf + Mx, c->M, mem, pvals));
    return VAMPOMI_OK;
}

// ---------------------------------------------------------------------------
// parameters / measurement
// ---------------------------------------------------------------------------
extern "C" vampomi_status vampomi_set_timing(vampomi_ctx* c, int on) {
    if (!c) return fail(VAMPOMI_ERR_ARG, "null context");
    c->timing = on != 0;
    c->tperiod = on > 1 ? on : 1;
    for (auto& row : c->tcount)
        for (auto& n : row) n = 0;
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_get_stats(vampomi_ctx* c, vampomi_stats* out) {
    if (!c || !out) return fail(VAMPOMI_ERR_ARG, "null argument");
    STCHK(sync_stream(c, c->st));
    resolve_timing(c);
    *out = c->stats;
    // estimated device time of every launch: the sampled average x the exact count
    auto fill = [](vampomi_kernel_stat& x) {
        x.ms_total = x.timed > 0 ? x.ms_timed / (double)x.timed * (double)x.launches : 0.0;
    };
    for (vampomi_kernel_stat* x : {&out->loo, &out->coll}) fill(*x);
    // a class's time is the sum of its per-K estimates (launches of different K
    // take different times: one average over the mix would weigh them by where
    // the samples fell)
    for (int k = 0; k < 4; ++k)
        for (vampomi_kernel_stat* x : {&out->ax_k[k], &out->atx_k[k], &out->op_k[k]}) fill(*x);
    for (auto pr : {std::make_pair(&out->ax, out->ax_k), std::make_pair(&out->atx, out->atx_k),
                    std::make_pair(&out->op, out->op_k)}) {
        int64_t n = 0;
        double ms = 0.0;
        for (int k = 0; k < 4; ++k) {
            n += pr.second[k].launches;
            ms += pr.second[k].ms_total;
        }
        if (n == pr.first->launches) pr.first->ms_total = ms;
        else fill(*pr.first);
    }
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_reset_stats(vampomi_ctx* c) {
    if (!c) return fail(VAMPOMI_ERR_ARG, "null context");
    STCHK(sync_stream(c, c->st));
    resolve_timing(c);
    c->stats = vampomi_stats{};
    return VAMPOMI_OK;
}

// ---------------------------------------------------------------------------
// development hooks (tools/kbench.py): kernel variant selection and timing
// ---------------------------------------------------------------------------
extern "C" vampomi_status vampomi_dev_set_variant(vampomi_ctx* c, int which, int variant) {
    if (!c) return fail(VAMPOMI_ERR_ARG, "null context");
    HIPCHK(hipSetDevice(c->device));
    STCHK(sync_stream(c, c->st));
    if (which == 0) {
        if (!vk::ax_variant_ok(variant)) return fail(VAMPOMI_ERR_ARG, "no such A.x variant");
        const vk::AxPlan np = vk::ax_plan(c->N, std::max<int64_t>(c->M, 1), variant);
        if (np.nslots > c->axp.nslots) {
            dev_free(c->ax_part);
            STCHK(dev_alloc(&c->ax_part, (size_t)np.nslots * vk::kMaxRhs * c->ld));
        }
        c->axp = np;
    } else if (which == 1) {
        if (!vk::atx_variant_ok(variant)) return fail(VAMPOMI_ERR_ARG, "no such A^T.u variant");
        c->atx_variant = variant;
    } else if (which == 3) {
        vk::OpPlan p{};
        if (!vk::op_plan(c->N, std::max<int64_t>(c->M, 1), c->cus > 0 ? c->cus : 256, variant, &p))
            return fail(VAMPOMI_ERR_ARG, "no such one-pass operator plan for this N");
        c->op_variant_req = variant;  // several ranks: applied and agreed at the next vampomi_vamp_begin
        if (!c->use_comm) {
            c->op_variant = variant;
            c->op_ready = false;
        }
    } else if (which == 4) {  // (the side stream of rounds 2-5: removed in round 6)
        return fail(VAMPOMI_ERR_ARG, "no side stream: every launch runs on the context's stream (DESIGN.md §6)");
    } else if (which == 5) {  // the CG head start (pcg.cpp): 0 off, 1 on
        if (variant != 0 && variant != 1) return fail(VAMPOMI_ERR_ARG, "head start: 0 or 1");
        c->hs_on_req = variant == 1;  // several ranks: applied and agreed at the next vampomi_vamp_begin
        if (!c->use_comm) c->hs_on = c->hs_on_req;
    } else if (which == 6) {  // several ranks: the host-free iteration tail (vamp.cpp, VAMPOMI_MR_TAIL): 0 off, 1 on
        if (variant != 0 && variant != 1) return fail(VAMPOMI_ERR_ARG, "multi-rank tail: 0 or 1");
        c->mr_tail_req = variant == 1;  // agreed at the next vampomi_vamp_begin (it changes the collectives)
        if (!c->use_comm) c->mr_tail = c->mr_tail_req;
    } else {
        if (!vk::loo_variant_ok(variant)) return fail(VAMPOMI_ERR_ARG, "no such association-pass variant");
        c->loo_variant = variant;
    }
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_dev_time_pass(vampomi_ctx* c, int which, int K, int reps, double* avg_ms) {
    if (!c || !avg_ms || K < 1 || K > (which == 0 ? 4 : which == 1 ? 3 : which == 3 ? 2 : 1) || reps < 1)
        return fail(VAMPOMI_ERR_ARG, "bad argument");
    if (!c->have_X) return fail(VAMPOMI_ERR_STATE, "no methylation data loaded");
    HIPCHK(hipSetDevice(c->device));
    if (which == 3) {
        STCHK(op_prepare(c));  // a timing hook: this rank's plan, no agreement
        if (!c->op_ok_mine) return fail(VAMPOMI_ERR_ARG, "no one-pass operator plan for this N");
    }
    const int64_t Mx = std::max<int64_t>(c->M, 1);
    vk::CPtrs in{};
    vk::Ptrs out{};
    for (int k = 0; k < K; ++k) {
        in.p[k] = which == 0 ? c->mbuf + k * Mx : c->nbuf + k * c->ld;
        out.p[k] = which == 0 ? c->nbuf + k * c->ld : c->mbuf + k * Mx;
    }
    hipEvent_t a, b;
    HIPCHK(hipEventCreate(&a));
    HIPCHK(hipEventCreate(&b));
    HIPCHK(hipEventRecord(a, c->st));
    for (int r = 0; r < reps; ++r) {
        if (which == 0)
            HIPCHK(vk::ax_partial(c->shard(), c->axp, K, in, c->ax_part, c->st));
        else if (which == 1)
            HIPCHK(vk::atx(c->shard(), K, in, out, 1.0 / c->sqrtN, 0, 0.0, 0.0, vk::CPtrs{}, c->st, c->atx_variant));
        else if (which == 3) {  // the operator on q = nbuf/1, p = mbuf slots 0..1, d into slots 2..3
            vk::OpArgs x{};
            for (int k = 0; k < K; ++k) {
                x.ar.p[k] = c->nbuf + k * c->ld;
                x.p.p[k] = c->mbuf + k * Mx;
                x.d.p[k] = c->mbuf + (2 + k) * Mx;
            }
            x.diag = 1.0;
            x.scale = 1.0 / c->sqrtN;
            x.tau = 1.0;
            x.part = c->op_part;
            x.ro = vk::RedOut{c->red_part, c->scal + SL_DP, c->ticket, nullptr, 0, nullptr};
            if (c->opp.T > 1) {
                x.xg = c->op_xg;
                if (++c->op_tag == 0) ++c->op_tag;
                x.tag = c->op_tag;
                x.err = op_err_dev(c);
            }
            x.dbg = std::getenv("VAMPOMI_OP_DBG") ? std::atoi(std::getenv("VAMPOMI_OP_DBG")) : 0;
            if (c->opp.T > 1) x.err = op_err_dev(c);
            x.ts = c->op_ts;
            STCHK(team_launch(c, c->opp.T, [&] { return vk::atax(c->shard(), c->opp, K, x, c->st); }));
        }
        else  // association pass: ymod = nbuf slot 0, x1 = mbuf slot 0, sums in mbuf slots 3..7
            HIPCHK(vk::loo_sums(c->shard(), c->nbuf, c->mbuf, c->sqrtN, c->mbuf + 3 * Mx, c->st, c->loo_variant));
    }
    HIPCHK(hipEventRecord(b, c->st));
    HIPCHK(hipEventSynchronize(b));
    if (which == 3 && std::getenv("VAMPOMI_OP_DBG") && (std::atoi(std::getenv("VAMPOMI_OP_DBG")) & 64)) {
        unsigned* w = reinterpret_cast<unsigned*>(c->h_flag + 4);
        std::fprintf(stderr, "op dbg: slow polls %u, spins %u, columns polled %u (over %d launches)\n", w[1], w[2], w[3],
                     reps);
        w[1] = w[2] = w[3] = 0;
    }
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    *avg_ms = (double)ms / reps;
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_dev_op_apply(vampomi_ctx* c, int K, const double* ar, const double* qo,
                                               const double* p, const double* z, const double* beta, double diag,
                                               double tau, double gam2, double* d, double* ad, double* dp) {
    if (!c || K < 1 || K > vk::kOpMaxK || !ar || !p || !d || !ad || !dp || (z && (!qo || !beta)))
        return fail(VAMPOMI_ERR_ARG, "bad argument");
    if (c->use_comm) return fail(VAMPOMI_ERR_ARG, "vampomi_dev_op_apply: one rank only");
    HIPCHK(hipSetDevice(c->device));
    STCHK(op_prepare(c));
    if (!c->op_ok) return fail(VAMPOMI_ERR_ARG, "no one-pass operator plan for this N");
    const int64_t Mx = std::max<int64_t>(c->M, 1);
    double* AR = c->op_nvec;
    double* Q = c->op_nvec + (int64_t)vk::kMaxRhs * c->ld;
    vk::OpArgs a{};
    for (int k = 0; k < K; ++k) {
        STCHK(stage_in(c, ar + k * c->N, c->N, VAMPOMI_MEM_HOST, AR + k * c->ld));
        STCHK(stage_in(c, p + k * c->M, c->M, VAMPOMI_MEM_HOST, c->mbuf + k * Mx));
        a.ar.p[k] = AR + k * c->ld;
        a.p.p[k] = c->mbuf + k * Mx;
        a.d.p[k] = c->mbuf + (2 + k) * Mx;
        if (z) {
            STCHK(stage_in(c, qo + k * c->N, c->N, VAMPOMI_MEM_HOST, Q + k * c->ld));
            STCHK(stage_in(c, z + k * c->M, c->M, VAMPOMI_MEM_HOST, c->mbuf + (4 + k) * Mx));
            a.qo.p[k] = Q + k * c->ld;
            a.z.p[k] = c->mbuf + (4 + k) * Mx;
        }
    }
    double* dbeta = c->mbuf + 6 * Mx;  // K <= 2 <= M... at least K doubles: mbuf slot 6 (Mx >= 1)
    if (z) {
        if (Mx < K) return fail(VAMPOMI_ERR_ARG, "vampomi_dev_op_apply: fused form needs M >= K");
        STCHK(stage_in(c, beta, K, VAMPOMI_MEM_HOST, dbeta));
        a.beta = dbeta;
        a.fuse = (1 << K) - 1;
    }
    a.diag = diag;
    a.tau = tau;
    a.gam2 = gam2;
    STCHK(op_dev(c, K, a, nullptr));
    const double* AD = c->op_nvec + (int64_t)2 * vk::kMaxRhs * c->ld;
    for (int k = 0; k < K; ++k) {
        STCHK(stage_out(c, c->mbuf + (2 + k) * Mx, c->M, VAMPOMI_MEM_HOST, d + k * c->M));
        STCHK(stage_out(c, AD + k * c->ld, c->N, VAMPOMI_MEM_HOST, ad + k * c->N));
    }
    HIPCHK(hipMemcpyAsync(dp, c->scal + SL_DP, (size_t)K * 8, hipMemcpyDeviceToHost, c->st));
    STCHK(sync_stream(c, c->st));
    return op_check_err(c);
}

// experiment builds (TM_TS=1, VAMPOMI_OP_TS=1): the last operator launch's
// per-workgroup {start, end, XCC id, HW id}, 4 x grid words
extern "C" vampomi_status vampomi_dev_op_timestamps(vampomi_ctx* c, unsigned long long* out, int cap, int* n) {
    if (!c || !out || !n) return fail(VAMPOMI_ERR_ARG, "null argument");
    if (!c->op_ts) return fail(VAMPOMI_ERR_STATE, "no timestamps (VAMPOMI_OP_TS=1 at the first operator use)");
    STCHK(sync_stream(c, c->st));
    *n = std::min(cap, 4 * c->opp.grid);
    HIPCHK(hipMemcpy(out, c->op_ts, (size_t)*n * 8, hipMemcpyDeviceToHost));
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_dev_ax_plan(int64_t N, int64_t M, int cus, int variant, int K, int* T, int* TR,
                                              int* S, int* grid, int* nslots, char* name, int cap) {
    if (N < 1 || M < 1 || cus < 1 || K < 1 || K > vk::kMaxRhs || !vk::ax_variant_ok(variant))
        return fail(VAMPOMI_ERR_ARG, "bad argument");
    const vk::AxPlan p = vk::ax_plan_for(N, M, cus, variant);
    if (T) *T = p.T;
    if (TR) *TR = p.TR;
    if (S) *S = p.S;
    if (grid) *grid = p.groups;
    if (nslots) *nslots = p.nslots;
    if (name && cap > 0) std::snprintf(name, (size_t)cap, "%s", vk::ax_kernel_name(K, false, p).c_str());
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_dev_op_plan(int64_t N, int64_t M, int cus, int variant, int K, int* T, int* S,
                                              int* TR, int* grid, int64_t* nslots, char* name, int cap) {
    vk::OpPlan p{};
    if (K < 1 || K > vk::kOpMaxK || !vk::op_plan(N, std::max<int64_t>(M, 1), cus, variant, &p))
        return fail(VAMPOMI_ERR_ARG, "no one-pass operator plan");
    if (T) *T = p.T;
    if (S) *S = p.S;
    if (TR) *TR = p.TR;
    if (grid) *grid = p.grid;
    if (nslots) *nslots = p.nslots;
    if (name && cap > 0) std::snprintf(name, (size_t)cap, "%s", vk::op_kernel_name(K, p).c_str());
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_dev_op_lds(int64_t N, int64_t M, int cus, int variant, int K, int64_t* out) {
    vk::OpPlan p{};
    if (!out || !vk::op_plan(N, std::max<int64_t>(M, 1), cus, variant, &p) || !vk::team_lds_layout(p, N, K, out))
        return fail(VAMPOMI_ERR_ARG, "no team plan with that system count");
    return VAMPOMI_OK;
}

// Device bytes one rank's context allocates for a VAMP run: the same sizes
// vampomi_open, the data load, op_prepare (the one-pass operator's buffers,
// batch_rhs 4), vamp_alloc / probit_begin and the iteration writer allocate,
// summed (each hipMalloc rounded up to 2 MiB, the allocator's granularity for
// large blocks).  RCCL's own buffers and the HIP runtime are not included.
extern "C" vampomi_status vampomi_dev_mem_plan(int64_t N, int64_t Mt, int nranks, int rank, int cus, int probit,
                                               int writer, int64_t* bytes) {
    if (!bytes || N < 2 || Mt < nranks || nranks < 1 || rank < 0 || rank >= nranks || cus < 1)
        return fail(VAMPOMI_ERR_ARG, "bad argument");
    int64_t M = 0, S = 0, Mm = 0;
    vampomi_divide_work(Mt, nranks, rank, &M, &S, &Mm);
    const int64_t Mx = std::max<int64_t>(M, 1), ld = (N + 15) / 16 * 16;
    int64_t total = 0;
    auto add = [&](int64_t n, int64_t elem) {
        const int64_t b = std::max<int64_t>(n, 1) * elem, g = 2 << 20;
        total += (b + g - 1) / g * g;
    };
    const vk::AxPlan axp = vk::ax_plan(N, Mx);
    add(Mx * ld, 8);                                   // X
    add(Mx, 8), add(Mx, 8), add(ld, 8);                // mave, msig, y
    add((int64_t)axp.nslots * vk::kMaxRhs * ld, 8);    // ax_part
    add((int64_t)red_capacity(Mx), 8), add((int64_t)red_capacity(Mx), 8);
    add(SL_TOTAL, 8), add(64, 4), add(64, 4);          // scal, tickets
    add((int64_t)vk::kMaxRhs * ld, 8);                 // nbuf
    add((int64_t)2 * vk::kMaxRhs * Mx, 8);             // mbuf
    add((int64_t)sizeof(vk::CgState), 1);
    vk::OpPlan op{}, hs{};
    if (vk::op_plan(N, Mx, cus, vk::kOpDefault, &op)) {
        const bool h = vk::team_plain_plan(N, Mx, cus, op, &hs);
        add((int64_t)3 * vk::kMaxRhs * ld + 16, 8);    // op_nvec
        add(std::max<int64_t>(op.nslots, h ? hs.nslots : 0) * vk::kMaxRhs * ld, 8);  // op_part
        size_t w = op.T > 1 ? op_xg_words_for(Mx, op) : 0;
        if (h && hs.T > 1) w = std::max(w, op_xg_words_for(Mx, hs));
        if (w) add((int64_t)w, 8);
    }
    for (int q = 0; q < 25; ++q) add(Mx, 8);           // VampRun M-vectors (15 + cgw[10])
    add(ld, 8), add((int64_t)vk::kMaxRhs * ld, 8), add((int64_t)vk::kMaxRhs * ld, 8), add(ld, 8);
    add(2 * ld, 8);                                    // abern (the head start, two slots)
    if (probit) {
        for (int q = 0; q < 3; ++q) add(ld, 8);
        for (int q = 0; q < 3; ++q) add(Mx, 8);
    }
    (void)writer;  // the writer's staging is pinned host memory (writer.h), allocated with every context
    *bytes = total;
    return VAMPOMI_OK;
}

// the operator's kernel as rocprofv3 prints it, for the context's plan
static std::string op_name(const vampomi_ctx* c, int K) {
    vk::OpPlan p{};
    int cus = c->cus;
    if (cus <= 0 && hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess) cus = 256;
    if (!vk::op_plan(c->N, std::max<int64_t>(c->M, 1), cus, c->op_variant, &p)) return "(no one-pass plan)";
    if (K == 1 + vk::kOpPlain) {  // the head-start launch
        vk::OpPlan h{};
        if (!vk::team_plain_plan(c->N, std::max<int64_t>(c->M, 1), cus, p, &h)) return "(no head-start plan)";
        return vk::team_kernel_name(K, h);
    }
    return vk::op_kernel_name(K, p);
}

extern "C" vampomi_status vampomi_dev_read_ceiling(vampomi_ctx* c, int reps, double* us_med, double* bytes,
                                                   int* variant) {
    if (!c || reps < 1 || !us_med) return fail(VAMPOMI_ERR_ARG, "bad argument");
    if (!c->have_X) return fail(VAMPOMI_ERR_STATE, "no methylation data loaded");
    HIPCHK(hipSetDevice(c->device));
    if (c->cus <= 0) HIPCHK(hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, c->device));
    STCHK(sync_stream(c, c->st));
    const int64_t n = std::max<int64_t>(c->M, 1) * c->ld;
    hipEvent_t a, b;
    HIPCHK(hipEventCreate(&a));
    HIPCHK(hipEventCreate(&b));
    double best = -1.0, best_bytes = 0.0;
    int best_kind = -1;
    for (int kind = 0; kind < 2; ++kind) {
        double nb = 0.0;
        if (vk::stream_read(c->X, n, kind, c->cus, c->st, vk::Timing{}, c->red_part, &nb) != hipSuccess) {
            (void)hipGetLastError();
            continue;  // the buffer is too small for this shape
        }
        std::vector<float> ms((size_t)reps);
        for (int r = 0; r < reps; ++r) {
            HIPCHK(vk::stream_read(c->X, n, kind, c->cus, c->st, vk::Timing{a, b}, c->red_part, &nb));
            HIPCHK(hipEventSynchronize(b));
            HIPCHK(hipEventElapsedTime(&ms[(size_t)r], a, b));
        }
        std::sort(ms.begin(), ms.end());
        const double med = 1e3 * (double)ms[(size_t)reps / 2];
        if (best < 0.0 || nb / med > best_bytes / best) {
            best = med;
            best_bytes = nb;
            best_kind = kind;
        }
    }
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    if (best_kind < 0) return fail(VAMPOMI_ERR_ARG, "the matrix is too small for a read-ceiling stream");
    *us_med = best;
    if (bytes) *bytes = best_bytes;
    if (variant) *variant = best_kind;
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_dev_kernel_name(const vampomi_ctx* c, int which, int K, int mode, char* out,
                                                  int cap) {
    if (!c || !out || cap < 1) return fail(VAMPOMI_ERR_ARG, "bad argument");
    // which = 3: mode carries N (the operator's instantiation depends on it)
    const std::string n = which == 2   ? vk::loo_kernel_name(c->loo_variant)
                          : which == 3 ? op_name(c, K)
                          : which == 0 ? vk::ax_kernel_name(K, mode == 1, c->axp)
                                       : vk::kernel_name(1, K, mode, c->atx_variant);
    std::snprintf(out, (size_t)cap, "%s", n.c_str());
    return VAMPOMI_OK;
}
