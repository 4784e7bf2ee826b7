// ctx.h — libvampomi internals shared by engine.cpp, pcg.cpp and vamp.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <initializer_list>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "../../include/vampomi.h"
#include "kernels.h"

// ---- errors ---------------------------------------------------------------
vampomi_status fail(vampomi_status s, const std::string& msg);

#define HIPCHK(expr)                                                                                  \
    do {                                                                                              \
        hipError_t _e = (expr);                                                                       \
        if (_e != hipSuccess)                                                                         \
            return fail(VAMPOMI_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));          \
    } while (0)

#define NCCLCHK(expr)                                                                                 \
    do {                                                                                              \
        ncclResult_t _r = (expr);                                                                     \
        if (_r != ncclSuccess)                                                                        \
            return fail(VAMPOMI_ERR_RCCL, std::string(#expr) + ": " + ncclGetErrorString(_r));        \
    } while (0)

#define STCHK(expr)                                   \
    do {                                              \
        vampomi_status _s = (expr);                   \
        if (_s != VAMPOMI_OK) return _s;              \
    } while (0)

// ---- the context ------------------------------------------------------------
struct vampomi_ctx;
// Marks a COLLECTIVE entry point on this thread: an error raised inside it
// (fail()) aborts the context's communicator first (comm_abort), so that the
// other ranks fail at their next collective instead of waiting for this one.
struct CollScope {
    explicit CollScope(vampomi_ctx* c);
    ~CollScope();
    vampomi_ctx* prev;
};
struct VampRun;
class IterWriter;
struct LoopbackComm;  // engine.cpp: test-only in-process communicator
struct ShmComm;       // shmcomm.cpp: test-only cross-process communicator (VAMPOMI_COMM=shm)
std::shared_ptr<ShmComm> shm_join(const void* id, int P, int rank, double limit_s, std::string* err);
std::string shm_allreduce(ShmComm& s, int rank, double* buf, size_t n, uint64_t seq, const char* site, int line,
                          double limit_s);
void shm_poison(ShmComm& s, const std::string& why);

struct TimedLaunch {
    hipEvent_t a, b;
    int cls;  // 0 ax, 1 atx, 2 loo, 3 one-pass operator, 4 all-reduce
    int K;
    double bytes, flops;
};

// scalar slots in ctx->scal: <d,p> of the fused lmmse epilogue, then the
// synced (summed over ranks) and local halves of a DotBatch
// (SL_CG: the 3K sums of a CG step, decided on the device; SL_CGI: the 2K sums
// of cg_init, read by cg_start_from)
// (SL_CHAIN, device, one rank: [0, 3) gam1, eta2, alpha2 of G1Chain; [3, 8)
// the next prelude's scalars (vk::PreOut); [8] tn, [9] tc (DotCopy))
enum : int { SL_DP = 0, SL_CG = 4, SL_SYNC = 16, SL_NSYNC = 256, SL_LOCAL = SL_SYNC + SL_NSYNC, SL_NLOCAL = 128,
             SL_CGI = SL_LOCAL + SL_NLOCAL, SL_CHECK = SL_CGI + 16, SL_AGREE = SL_CHECK + 8, SL_CHAIN = SL_AGREE + 8, SL_TOTAL = 512, SL_BARRIER = SL_TOTAL - 1 };

struct vampomi_ctx {
    int rank = 0, nranks = 1, device = 0;
    int64_t N = 0, Mt = 0, M = 0, S = 0, Mm = 0, ld = 0;
    double alpha_scale = 1.0;
    double sqrtN = 1.0;
    hipStream_t st = nullptr;  // every launch and collective of the context (one stream: DESIGN.md §6)
    bool mr_tail = true;   // several ranks: the linear iteration's tail without host waits (vamp.cpp), as agreed
    double coll_limit_s = 0.0;  // > 0: the limit of the collective in progress (vampomi_barrier_timeout)
    bool mr_tail_req = true;  // this rank's VAMPOMI_MR_TAIL (0: off), agreed over the ranks by op_agree
    bool cg_fold = true;   // several ranks: each CG decision formed by the next operator launch (pcg.cpp); VAMPOMI_CG_FOLD=0
    bool team_reg = false;           // registered with its device's team gate (engine.cpp)
    hipEvent_t team_ev = nullptr;    // recorded on st when another context must order behind it
    ncclComm_t comm = nullptr;
    bool use_comm = false;  // nranks > 1 (or VAMPOMI_FORCE_RCCL): all-reduces through RCCL
    std::shared_ptr<LoopbackComm> loopback;  // VAMPOMI_COMM=loopback: ranks are threads of one process
    std::shared_ptr<ShmComm> shm;            // VAMPOMI_COMM=shm: ranks are processes of one host
    uint64_t coll_seq = 0;  // collectives issued so far (divergence checks)
    bool aborted = false;   // comm_abort ran: no further collective

    double* X = nullptr;     // M columns x ld, marker-major, pad rows zero
    double* mave = nullptr;
    double* msig = nullptr;
    double* y = nullptr;     // ld, zero pad
    std::vector<double> y_host;
    bool have_X = false, have_y = false;

    vk::AxPlan axp{};
    int atx_variant = vk::kAtxDefault, loo_variant = vk::kLooDefault;  // per context (dev hooks)
    double* ax_part = nullptr;  // nslots x kMaxRhs x ld partial sums of A.x
    double* red_part = nullptr;  // per-block partials of every reduction
    size_t red_cap = 0;
    double* scal = nullptr;     // device scalars (SL_*)
    double* h_scal = nullptr;   // pinned host mirror, mapped and coherent: one-rank reductions land here directly
    double* d_hscal = nullptr;  // its device-side address
    unsigned* ticket = nullptr; // arrival counter of the fused reductions (zero between launches)
    unsigned long long* h_flag = nullptr;  // mapped host word the stream stores sync sequence numbers into
    unsigned long long* d_flag = nullptr;
    unsigned long long sync_seq = 0;
    vk::CgState* cgs = nullptr;     // device-side CG control (pcg.cpp), two states (the folded decisions alternate)
    vk::CgMirror* h_cgm = nullptr;  // its mapped host mirror, and the mirror's device address
    vk::CgMirror* d_cgm = nullptr;
    // one-pass CG operator (batch_rhs 4; allocated on first use, pcg.cpp)
    vk::OpPlan opp{};
    int op_variant = vk::kOpDefault;  // plan choice (dev hook: vampomi_dev_set_variant(c, 3, v))
    bool op_ready = false;            // opp planned (locally) and its buffers allocated
    bool op_ok_mine = false;          // this rank's plan exists and its grid fits the device
    bool op_ok = false;               // the operator runs: op_ok_mine on one rank; the agreed value on several
    // several ranks: the one-pass / head-start choice is agreed at one fixed
    // collective point every rank reaches (op_agree, at vampomi_vamp_begin);
    // set_variant(3 / 5) requests wait for it (applied at once on one rank)
    bool op_agreed = false;
    int op_variant_req = vk::kOpDefault;
    int cus = 0;                // compute units of the device (the operator's grid)
    double* op_part = nullptr;  // opp.nslots x kMaxRhs x ld partial A d
    int64_t op_part_slots = 0;
    double* op_nvec = nullptr;  // 3 x kMaxRhs x ld + 16: A r, q = A p, A d (+ <d,p> tail)
    unsigned long long* op_xg = nullptr;  // team hand-off granules (M x kOpMaxK x T x 2), zeroed once
    size_t op_xg_words = 0;
    unsigned op_tag = 0;        // the last team launch's tag
    // the head-start launch (pcg.cpp): its plan and whether it runs (default
    // on; VAMPOMI_HEADSTART=0 or vampomi_dev_set_variant(c, 5, 0) turns it off)
    vk::OpPlan opp_hs{};
    bool hs_ok_mine = false;  // this rank's head-start plan exists and fits
    bool hs_ok = false;       // the head start runs (hs_on included; agreed on several ranks)
    bool hs_on = true;
    bool hs_on_req = true;
    unsigned long long* op_ts = nullptr;  // VAMPOMI_OP_TS=1 (TM_TS builds): the last launch's workgroup times
    double* nbuf = nullptr;     // kMaxRhs * ld scratch N-vectors (API calls)
    double* mbuf = nullptr;     // (2*kMaxRhs) * M scratch M-vectors (API calls)

    bool timing = false;
    int tperiod = 1;            // time 1 in tperiod launches of each (class, K)
    int64_t tcount[5][vk::kMaxRhs] = {};
    std::vector<TimedLaunch> pending;
    std::vector<hipEvent_t> ev_pool;
    vampomi_stats stats{};

    std::unique_ptr<VampRun> run;
    std::unique_ptr<IterWriter> writer;  // per-iteration output (writer.h), created with the context

    vk::Shard shard() const { return vk::Shard{X, ld, N, M, mave, msig}; }
    vampomi_ctx();   // defined in vamp.cpp, where VampRun is complete
    ~vampomi_ctx();
};

vampomi_status dev_alloc(double** p, size_t n);
void dev_free(double*& p);
vampomi_status host_sync(vampomi_ctx* c);
// spins until word `word` of the context's host flag block reaches seq (stores
// from the stream; word 0 the stream's sync sequence, kCgPackWord.. the CG's
// packed decisions)
vampomi_status wait_flag(vampomi_ctx* c, unsigned long long seq, int word = 0);
// hipStreamSynchronize, except with an RCCL communicator: polls the stream and
// the communicator, and aborts / fails on a broken job or after
// VAMPOMI_COLL_TIMEOUT_S (engine.cpp) instead of blocking forever
vampomi_status sync_stream(vampomi_ctx* c, hipStream_t st);
// SUM all-reduce of n doubles over the ranks (nothing on one rank). COLLECTIVE:
// every rank must make the same calls in the same order; site/line identify
// the call for the divergence checks (loopback always, RCCL with
// VAMPOMI_COLL_CHECK=1)
vampomi_status allreduce_dev(vampomi_ctx* c, double* buf, size_t n, const char* site = __builtin_FUNCTION(),
                             int line = __builtin_LINE());
// *total = local summed over the ranks (one all-reduce; *total = local on one
// rank).  COLLECTIVE: how ranks agree on a decision that started rank-local
vampomi_status sum_over_ranks(vampomi_ctx* c, double local, double* total, const char* site = __builtin_FUNCTION(),
                              int line = __builtin_LINE());
// poisons (loopback) or aborts (RCCL) the communicator after a rank-local error
void comm_abort(vampomi_ctx* c, const std::string& why);
void resolve_timing(vampomi_ctx* c);
// counts a launch of class cls with K right-hand sides (bytes, flops: its
// algorithmic work); returns HIP events for it if it is sampled (else nulls)
TimedLaunch launch_stat(vampomi_ctx* c, int cls, int K, double bytes, double flops);
// forgets the counts since `before` and the samples queued since pending_mark
// (the gated launches of a CG step queued after the solve had stopped)
void drop_launches(vampomi_ctx* c, size_t pending_mark, const vampomi_stats& before);
void release_ctx_resources(vampomi_ctx* c);

// ---- operators on device buffers ---------------------------------------------
// out_k = A x_k (K <= 4), outputs at outbase + k*ld (one all-reduce). COLLECTIVE
// fu (may be null): fused direction update and gate (vk::AxFuse).  tail (may
// be null; several ranks only): local M-sums all-reduced in the same call,
// landing at outbase[K*ld + q] (outbase must hold K*ld + tail->nt doubles)
vampomi_status ax_dev(vampomi_ctx* c, int K, const double* const* x, double* outbase,
                      const vk::AxFuse* fu = nullptr, const vk::DotArgs* tail = nullptr);
// out_k = A^T u_k (mode 0) or tau*A^T u_k + gam2*p_k with <out_k,p_k> summed over
// ranks into scal[SL_DP + k] (mode 1).  u_k: ld-padded N-vectors.  gate: as in
// vk::AxFuse; zf/beta (may be null): p_k stands for zf_k + beta[k]*p_k
// dp = false (mode 1): <out_k,p_k> is not formed (the caller has it otherwise)
vampomi_status atx_dev(vampomi_ctx* c, int K, const double* const* u, double* const* out, int mode, double tau,
                       double gam2, const double* const* p, const int* gate = nullptr,
                       const double* const* zf = nullptr, const double* beta = nullptr, bool dp = true,
                       double* const* sraw = nullptr);
// d_k = tau*A^T A v_k + gam2*v_k (lmmse_mult), <d_k,v_k> in scal[SL_DP+k]. COLLECTIVE
vampomi_status lmmse_dev(vampomi_ctx* c, int K, const double* const* v, double* const* d, double tau, double gam2,
                         double* nscratch);

// ---- batched scalar reductions ---------------------------------------------------
// Every inner_prod / l2_norm2 of the reference (src/utilities.cpp:138-162) is a
// fixed-order device reduction into a scalar slot.  A DotBatch queues several
// of them (each with its own sync flag: sync = summed over ranks, the
// reference's inner_prod(..., 1)) and resolves them with ONE all-reduce, ONE
// device-to-host copy and ONE host synchronisation.
class DotBatch {
   public:
    explicit DotBatch(vampomi_ctx* c) : c_(c) {}
    vampomi_status add(std::initializer_list<vk::DotTerm> terms, int64_t n, bool sync, double* out);
    // several groups of terms over the same length n in ONE kernel (<= 8 terms
    // in all): each group's results reach its out at flush(), exactly as its
    // own add() would give them (per-term sums do not depend on the other terms)
    struct Group {
        std::vector<vk::DotTerm> terms;
        bool sync;
        double* out;
    };
    // chain (may be null): its arithmetic rides in the launch, on the sum of
    // the group whose out is chain_of (a one-term group); copies: the result
    // of each one-term group whose out is .first is also stored at .second
    // (device memory) by the launch (at most 2)
    vampomi_status add_many(int64_t n, const std::vector<Group>& groups, const vk::G1Chain* chain = nullptr,
                            const double* chain_of = nullptr,
                            const std::vector<std::pair<const double*, double*>>& copies = {});
    // add_many over [0, na) with ga and over [0, nb) with gb in one launch
    // where vk::dots2 has the pairing (else two launches): the same results
    vampomi_status add_pair(int64_t na, const std::vector<Group>& ga, const vk::G1Chain* chain,
                            const double* chain_of, const std::vector<std::pair<const double*, double*>>& ca,
                            int64_t nb, const std::vector<Group>& gb,
                            const std::vector<std::pair<const double*, double*>>& cb);
    // reserves nq result slots for a fused reduction kernel: *ro says where the
    // kernel writes; the values reach out[0..nq) at flush()
    vampomi_status sink(int nq, bool sync, double* out, vk::RedOut* ro);
    vampomi_status flush();
    bool empty() const { return sinks_.empty(); }
    // one rank: the device address where the result that flush() will copy to
    // out is written (mapped host memory), for a kernel queued before the
    // flush; null if out is not a sink of this batch or with a communicator
    const double* dev_result(const double* out) const;
    // several ranks: all-reduces the synced slots filled since the last call,
    // on the main stream, with no host copy or wait (flush() then publishes
    // them without reducing them again), so that a kernel queued next can read
    // the final sums at dev_slot(); nothing on one rank.  COLLECTIVE
    vampomi_status reduce_now();
    // several ranks: the device address of the slot whose value flush() will
    // copy to out (final after reduce_now() for a synced result); else null
    double* dev_slot(const double* out) const;
    // the stream the batch's launches go to (the context's)
    hipStream_t stream() const;

   private:
    // a launch's DotArgs and RedOut from its groups (sinks registered, flag sequence taken)
    vampomi_status build(const std::vector<Group>& groups, const vk::G1Chain* chain, const double* chain_of,
                         const std::vector<std::pair<const double*, double*>>& copies, vk::DotArgs& a,
                         vk::RedOut& ro);
    struct Sink {
        int slot, count;
        double* out;
    };
    vampomi_ctx* c_;
    int nsync_ = 0, nlocal_ = 0;
    int nred_ = 0;  // synced slots [0, nred_) already all-reduced (reduce_now)
    unsigned long long last_seq_ = 0;  // one rank: flag value the last reduction kernel stores
    std::vector<Sink> sinks_;
};

inline vk::DotTerm T(const double* a, const double* b, int op = vk::DOT) { return vk::DotTerm{a, b, op}; }

// ---- PCG (vamp::precondCG_solver) ----------------------------------------------
struct CgSystem {
    const double* v = nullptr;     // right-hand side (device, M)
    double* mu = nullptr;          // in: start (if mu0_nonzero), out: solution
    bool mu0_nonzero = false;      // false: start from zeros (lmmse_mult short-circuit)
    const double* atx0 = nullptr;  // optional: A^T(A mu0) computed earlier (saves the start's passes)
    // optional recurrence (batch_rhs 2): W (device, M) holds A^T A mu0 on entry
    // (zeros when mu0 = 0) and A^T A mu on return, updated with each step's raw
    // A^T(A p) kept in S (device, M scratch); W may alias atx0
    double* W = nullptr;
    double* S = nullptr;
    // optional (batch_rhs 3): AW (device, ld) holds A mu0 on entry (zeros when
    // mu0 = 0) and A mu on return, updated with each step's A p
    double* AW = nullptr;
    bool onsager = false;          // denoiser == 0 in the reference: extra Onsager stop
    int iters = 0;
    double *r = nullptr, *z = nullptr, *p = nullptr, *d = nullptr;  // work vectors (device, M)
};
// Solves the systems together: every CG step streams X twice for all still
// active systems; each keeps its own scalars and stopping rule.  `init` (may
// be null) is flushed together with the initial residual reductions.
// extra_x (may be null, device M): ex_out (device, ld) = A extra_x, carried as
// one more right-hand side of the first step's A.x pass (its own pass if no
// step runs).  nscratch holds kMaxRhs*ld + kMaxRhs doubles.
// onepass (K <= 2): every CG step reads X once (vk::atax; A r0 by one A.x pass
// per solve, which also carries extra_x); otherwise two passes per step.
// ar0 (may be null; onepass only): ar0[k] (device, ld, may be null) already
// holds A r0 of system k (its start is zero, so r0 = v), and the first A.x
// pass covers only the systems without it (no pass if none).
//
// hs (may be null; onepass, K = 2, extra_x): the HEAD START.  System 0 must
// start from zero (r0 = v, e.g. the Onsager solve, whose v is a probe known an
// iteration early).  hs->abern (device ld) holds A v of system 0: then system
// 0's first CG step runs in the pass that would only compute A r0 of system 1
// and A extra_x (one operator launch with plain right-hand sides,
// op_dev_plain), and the two systems step together from there, system 0 one
// step ahead, so the solve takes 1 + max(k1 - 1, k2) passes instead of
// 1 + max(k1, k2).  Every step is the reference's (src/vamp.cpp:697-757).
// hs->xnext (may be null, device M): one more right-hand side of that pass,
// hs->axnext = A xnext (the next solve's abern).  Without hs->abern the first
// A.x pass carries xnext instead.
struct HeadStart {
    double* abern = nullptr;  // (the Onsager solve's A r: updated in place)
    const double* xnext = nullptr;
    double* axnext = nullptr;
    bool used = false;  // out: the head start ran
};
// pre (may be null; init must be null): the caller's prelude launch, fused
// with the solve's start (vk::prelude_cg_init).  pm (one rank, with pre):
// ahead: queue only that launch, its scalars from the device (pre->dev; tau
// and gam2 unused), and return; queued: that launch was queued ahead (the same
// sys, hs and pre): the solve goes on after it
enum class PreMode { normal, ahead, queued };
vampomi_status pcg_run(vampomi_ctx* c, const std::vector<CgSystem*>& sys, double tau, double gam2, int max_iter,
                       double tol, double* nscratch, int64_t* ref_passes, DotBatch* init,
                       const double* extra_x = nullptr, double* ex_out = nullptr, bool onepass = false,
                       const double* const* ar0 = nullptr, HeadStart* hs = nullptr,
                       const vk::Prelude* pre = nullptr, PreMode pm = PreMode::normal);
// plans the one-pass operator on this rank (c->opp, op_ok_mine, hs_ok_mine)
// and allocates its buffers (idempotent until the plan or the head-start
// switch changes); never a collective.  Sets op_ok / hs_ok: this rank's plan
// on one rank; on several the values op_agree agreed (both false before it)
vampomi_status op_prepare(vampomi_ctx* c);
// COLLECTIVE (several ranks; nothing on one): applies pending set_variant(3 /
// 5) requests, plans, and agrees op_ok and hs_ok over the ranks (both change
// the job's collective sequence; each rank planned from its own shard size,
// CU count and VAMPOMI_HEADSTART).  Called unconditionally by
// vampomi_vamp_begin, the one point every rank of a run reaches
vampomi_status op_agree(vampomi_ctx* c);
// whether pcg_run's head start can run on this context (plans the operator;
// the same answer on every rank)
vampomi_status headstart_available(vampomi_ctx* c, bool* yes);
// the device word a team launch sets when a hand-off timed out, and its host view
unsigned* op_err_dev(vampomi_ctx* c);
vampomi_status op_check_err(vampomi_ctx* c);
// d_k = tau*A^T q_k + gam2*p_k and A d_k (into op_nvec's A d block, /sqrt(N),
// summed over ranks with <d_k,p_k> at its tail; one rank: <d_k,p_k> in
// scal[SL_DP+k]) from one pass over X.  COLLECTIVE.  reduce = false (one
// rank only): the per-slot A d partials stay in op_part for cg_update to sum
// divide = false (several ranks): A d stays all-reduced but undivided, for a
// consumer that divides as it reads (cg_update's addiv)
vampomi_status op_dev(vampomi_ctx* c, int K, const vk::OpArgs& a, const int* gate, bool reduce = true,
                      bool divide = true);
// the head-start launch (c->opp_hs): op_dev's work for ONE system (a, K = 1),
// and out[kp] = A px[kp] (device ld, /sqrt(N), summed over ranks) for the
// kOpPlain plain right-hand sides, from the same pass over X.  One rank: the
// system's A d partials stay in op_part (opp_hs.nslots slots) for cg_update;
// several: its A d is op_nvec's A d block row 0, <d,p> at A d + (1 + kOpPlain)*ld.
// COLLECTIVE
vampomi_status op_dev_plain(vampomi_ctx* c, const vk::OpArgs& a, const double* const* px, double* const* out,
                            const int* gate);
