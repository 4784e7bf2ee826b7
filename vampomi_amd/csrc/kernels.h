// kernels.h — launch wrappers for the gfx950 kernels of the VAMP hot path
// (internal to libvampomi; the public boundary is include/vampomi.h).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <string>

namespace vk {

constexpr int kMaxRhs = 4;     // right-hand sides sharing one pass over X
constexpr int kMaxL = 64;      // mixture components (VAMPOMI_MAX_L)
constexpr int kMaxTerms = 12;  // dot-product terms per reduction launch
constexpr int kRedBlocks = 1024;  // max partial blocks of a reduction

struct CPtrs { const double* p[kMaxRhs]; };
// optional HIP events recorded by a launch's own dispatch (hipExtLaunchKernelGGL)
struct Timing { hipEvent_t start = nullptr, stop = nullptr; };
// Destination of a fused two-stage reduction (see red_finish in kernels.hip):
// per-block partials in part, the final sums in out[0..nq) (device memory or
// mapped host memory), ticket a zeroed device counter the kernel re-arms;
// flag (may be null): the last block stores seq there (system scope, after out);
// gate (may be null): the launch does nothing while *gate == 0;
// out2 (may be null): results q >= split go to out2[q - split] instead (one
// launch serving two slot ranges, DotBatch::add_many)
struct RedOut {
    double* part;
    double* out;
    unsigned* ticket;
    unsigned long long* flag = nullptr;
    unsigned long long seq = 0;
    const int* gate = nullptr;
    double* out2 = nullptr;
    int split = 0;
};
struct Ptrs { double* p[kMaxRhs]; };

// The device-resident marker shard: M columns (markers) of N samples, column
// stride ld >= N doubles (ld % 16 == 0, pad rows zero), plus marker stats.
struct Shard {
    const double* X;
    int64_t ld, N, M;
    const double* mave;
    const double* msig;
};

// ---- A.x : two-stage, deterministic --------------------------------------
// Stage 1 (ax_partial): the (row tile, marker) segments are split into equal
// shares, one per workgroup (two per CU): a fixed fraction of one or two
// tiles in every marker band (band plan), or a contiguous tile-major stripe;
// each tile a workgroup touches gets its own partial slot, written to
// part[slot][k][ld].  Stage 2 (ax_reduce): sums every tile's slots in order.
struct AxPlan {
    int variant;      // row/unroll variant (tuning table in kernels.hip)
    int64_t rows;     // rows per tile
    int64_t tiles;    // ceil(N / rows)
    int64_t total;    // tiles * M segments
    int64_t span;     // stripe plan: segments per workgroup
    int64_t nband;    // band plan: marker bands (0: stripe plan)
    int64_t sa, sb;   // tile t's first slot-owning workgroup is t*sa/sb
    int groups;       // workgroups (grid)
    int nslots;       // partial slots of the busiest tile (part holds nslots x kMaxRhs x ld)
    // team plan (variant kAxTeam, ax_team_kernel): T workgroups per team split
    // the rows (TR each, S loads per lane per column), every team a full
    // N-vector slot over its interleaved columns; one tile of N rows (sa =
    // nslots teams, sb = 1).  T = 0: the tile plans above
    int T = 0, TR = 0, S = 0;
};
// partial slots tile t uses: the workgroups whose share meets it
inline int64_t ax_slots(const AxPlan& p, int64_t t) { return ((t + 1) * p.sa - 1) / p.sb - (t * p.sa) / p.sb + 1; }
// Kernel variants (tuning tables in kernels.hip) are per-context launch
// settings: the defaults are the measured winners, other values are
// development hooks (tools/kbench.py, vampomi_dev_set_variant).
// kAxDefault: the team plan where it has teams of >= kAxTeamMinT (N above
// ~16k rows: C3/C4/C5; 3.7-3.8 % faster than the best tile plan there,
// profiles/r05s_lockstep_ab.txt), else variant 0 (C2 keeps its bits)
constexpr int kAxDefault = -1, kAxTeam = 7, kAxTeamMinT = 8, kAtxDefault = -1 /* per-K choice */, kLooDefault = 16;
AxPlan ax_plan(int64_t N, int64_t M, int variant = kAxDefault);
AxPlan ax_plan_for(int64_t N, int64_t M, int cus, int variant);  // (ax_plan on `cus` compute units)
int ax_variant_count();
bool ax_variant_ok(int v);
int atx_variant_count();
bool atx_variant_ok(int v);
// Optional fusion into the A.x pass (the CG direction update of the previous
// step): with z set, the pass multiplies x_k = z_k + beta[k]*p_k, where
// p_k is the `x` argument (every consumer of the new direction forms it the
// same way; cg_update stores it).  gate (may be null): no work while *gate == 0.
struct AxFuse {
    CPtrs z{};
    const double* beta = nullptr;  // device
    const int* gate = nullptr;
};
hipError_t ax_partial(const Shard& s, const AxPlan& pl, int K, CPtrs x, double* part, hipStream_t st,
                      const Timing& tm = Timing{}, const AxFuse& fu = AxFuse{});
// A pure read stream of x[0, n) (the read ceiling, vampomi_dev_read_ceiling):
// kind 0 lockstep 8-wave workgroups (cus of them), kind 1 a 1 MiB chunk per
// wave; returns the bytes read in *bytes (whole 8 KiB / 1 MiB units)
hipError_t stream_read(const double* x, int64_t n, int kind, int cus, hipStream_t st, const Timing& tm,
                       double* sink, double* bytes);
// the team plan (atax_team.hip): false if N has none (rows per member past 4
// loads per lane of 1024-row steps at every team size)
bool ax_team_plan(int64_t N, int64_t M, int cus, AxPlan* out);
hipError_t ax_team(const Shard& s, const AxPlan& pl, int K, CPtrs x, double* part, hipStream_t st, const Timing& tm,
                   const AxFuse& fu);
std::string ax_kernel_name(int K, bool fused, const AxPlan& pl);  // as rocprofv3 prints it
// out_k[j] = sum_c part[c][k][j]; if div > 0 then out_k[j] /= div
hipError_t ax_reduce(const AxPlan& pl, int K, int64_t N, int64_t ld, const double* part, Ptrs out,
                     double div, hipStream_t st, const int* gate = nullptr);
// out_k[j] /= div (after the cross-rank all-reduce)
// v_k / div into dst_k (dst null: in place)
hipError_t vec_div(int K, int64_t n, int64_t ld, Ptrs v, double div, hipStream_t st, const Ptrs* dst = nullptr);

// ---- A^T.u : one wave per group of markers --------------------------------
// mode 0: out_k[i] = (msig_i * dot_k(i)) * scale
// mode 1 (lmmse_mult): out_k[i] = ((msig_i*dot)*scale)*tau + gam2*p_k[i]
// (<out_k, p_k> is a separate fixed-geometry reduction); gate as in AxFuse
int atx_blocks(int64_t M, int K, int variant);
std::string kernel_name(int which, int K, int mode, int variant);  // as rocprofv3 prints it
// zf/beta (mode 1, may be null): the epilogue's p_k is zf_k + beta[k]*p_k;
// sraw (mode 1, may be null): also stores the raw product (msig_i*dot)*scale
hipError_t atx(const Shard& s, int K, CPtrs u, Ptrs out, double scale, int mode, double tau,
               double gam2, CPtrs p, hipStream_t st, int variant = kAtxDefault, const Timing& tm = Timing{},
               const int* gate = nullptr, CPtrs zf = CPtrs{}, const double* beta = nullptr, Ptrs sraw = Ptrs{});

// ---- one-pass CG operator: A^T q and A d from ONE read of X ----------------
// A CG step needs d = tau*A^T(A p) + gam2*p.  With q = A p carried as an
// N-vector recurrence (q = A r/diag + beta*q_old, A r -= alpha*A d), the pass
// over X computes, per marker i, t_i = (msig_i*sum_j (X_ij - mave_i) q_j)/sqrt(N)
// and d_i = tau*t_i + gam2*p_i, and while the column is still in registers
// accumulates (A d)_j += (X_ij - mave_i)*(msig_i*d_i): A^T and A in one read.
// Two kernels:
//  * T = 0 (atax_kernel, kernels.hip): one workgroup per CU owns whole
//    columns, q in LDS, so K*N <= 20,000;
//  * T >= 1 (atax_team_kernel, atax_team.hip): teams of T workgroups split
//    the rows of each column and hand the column dots over inside the launch
//    (T = 1: no hand-off), for N up to 32 x 8 x 896 rows.
constexpr int kOpMaxK = 2;
// the head-start launch (pcg.cpp): one operator system plus kOpPlain plain
// right-hand sides A x_kp from the same read of X (stats: K = 1 + kOpPlain)
constexpr int kOpPlain = 3;
struct OpPlan {
    int grid;       // workgroups (at most one per CU)
    int S;          // 16-byte loads per lane per column
    int64_t nslots; // partial A d slots (nslots x kMaxRhs x ld): workgroups (T = 0) or teams
    int T = 0;      // team size (0: the whole-column kernel)
    int TR = 0;     // rows per team member (T >= 1)
    int cfg = 0;    // team kernel configuration (prefetch, lag, polls in flight)
};
// variant: -1 the default choice for N; 0 the whole-column kernel; T*10 + cfg (cfg < 10) or 1000 + T*100 + cfg
// a team plan (development hook, tools/kbench.py)
constexpr int kOpDefault = -1;
bool op_plan(int64_t N, int64_t M, int cus, int variant, OpPlan* out);
bool op_supported(int64_t N, int K);
bool team_plan(int64_t N, int64_t M, int cus, int T, int cfg, OpPlan* out);
// the team kernel's dynamic LDS for plan pl with K operator systems (the one
// layout its launches and team_plan use, atax_team.hip tm_lds), in doubles:
// out[0] head words, [1] q offset, [2] q stride, [3] partials offset,
// [4] totals offset, [5] total words; false: pl is not a team plan
bool team_lds_layout(const OpPlan& pl, int64_t N, int K, int64_t out[6]);
// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device):
// bit d of done is device d; a failure is returned, never left pending
hipError_t lds_allow(const void* kern, std::atomic<unsigned long long>& done, int bytes);
struct CgState;
struct CgMirror;
// Several ranks (pcg.cpp): the previous CG step's decision (cg_decide on its
// all-reduced sums red) formed by the operator launch that needs its beta,
// instead of by a launch of its own between the all-reduce and this one: every
// workgroup decides from src (the same arithmetic, the same bits), workgroup 0
// stores the new state to dst (a second state: src is still being read) and
// publishes it (mirror / flag, as cg_decide); the launch then runs on the new
// beta, gated on its "any".  on = 0: a.beta and the gate as given
struct OpFold {
    const CgState* src = nullptr;
    CgState* dst = nullptr;
    const double* red = nullptr;
    int on = 0, it = 0, mask = 0xf, pack = 0;
    CgMirror* mirror = nullptr;
    unsigned long long* flag = nullptr;
    unsigned long long seq = 0;
};
struct OpArgs {
    CPtrs ar, qo;       // q_k = ar_k/diag [+ beta_k*qo_k when fuse] (N-space, replicated)
    CPtrs p, z;         // p_k [= z_k + beta_k*p_k when fuse] (M-space)
    const double* beta; // device (CgState.beta)
    int fuse;           // bit k: system k's direction update p = z + beta p is fused into this launch
    double diag, scale, tau, gam2;
    Ptrs d, sraw;       // d_k (M); sraw_k = t_k (may be null)
    CPtrs px;           // head-start launch only: the kOpPlain plain right-hand sides (M), A x_kp into
                        // partial slots 1 .. kOpPlain
    double* part;       // nslots x kMaxRhs x ld partial A d (before the sum over slots)
    RedOut ro;          // <d_k, p_k> summed over the shard (K values)
    // team kernel with T > 1: hand-off granules ((M + grid) x kOpMaxK x T x 2
    // words, then 2 x kOpMaxK dummy words per workgroup, then one XCD word per
    // workgroup; zeroed once), this launch's
    // tag (never 0, new every launch) and a mapped host word set when a
    // hand-off timed out
    unsigned long long* xg;
    unsigned tag;
    unsigned* err;
    unsigned long long* ts;  // experiment builds (TM_TS=1) only: per workgroup {start, end, XCC id, HW id}
    int dbg;  // timing experiments only (VAMPOMI_OP_DBG; results are wrong when set, except bit 5):
              // bit 0 no poll waits, 1 no publishes, 2 no butterfly, 3 no A d accumulation,
              // 5 write-through hand-off even when the team shares an XCD, 11 no LDS q reads,
              // 12 no hand-off work (the hand-off wave only keeps the step barriers)
    OpFold fold;  // team kernels only (atax_team.hip)
};
std::string op_kernel_name(int K, const OpPlan& pl);
std::string team_kernel_name(int K, const OpPlan& pl);
// workgroups of the team kernel of plan pl (T >= 1) with K right-hand sides one
// CU holds at once (0: it cannot run); a plan needs grid <= this x CUs, since
// a team launch needs all its workgroups resident together
int team_occupancy(const OpPlan& pl, int K);
hipError_t atax(const Shard& s, const OpPlan& pl, int K, const OpArgs& a, hipStream_t st, const Timing& tm = Timing{},
                const int* gate = nullptr);
hipError_t atax_team(const Shard& s, const OpPlan& pl, int K, const OpArgs& a, hipStream_t st, const Timing& tm,
                     const int* gate);
// the head-start launch: the team kernel with K = 1 and the kOpPlain plain
// right-hand sides a.px (plan from team_plain_plan)
hipError_t atax_team_plain(const Shard& s, const OpPlan& pl, const OpArgs& a, hipStream_t st, const Timing& tm,
                           const int* gate);
// a team plan for the head-start kernel (the main plan's team size if its rows
// fit, else larger teams); false: none (the solve starts without a head start)
bool team_plain_plan(int64_t N, int64_t M, int cus, const OpPlan& main, OpPlan* out);
// out_k[j] = sum_b part[b][k0 + k][j] (slots in order); if div > 0 then /= div
hipError_t op_reduce(const OpPlan& pl, int K, int64_t N, int64_t ld, const double* part, Ptrs out, double div,
                     hipStream_t st, const int* gate = nullptr, int k0 = 0);

// ---- marker statistics (data::compute_markers_statistics) ----------------
hipError_t marker_stats(const double* X, int64_t ld, int64_t N, int64_t M, double nonas,
                        double alpha_scale, double* mave, double* msig, hipStream_t st);

// ---- synthetic data --------------------------------------------------------
hipError_t gen_markers(uint64_t seed, int kind, int64_t N, int64_t ld, int64_t S, int64_t M, double* X,
                       hipStream_t st);
// beta_i = gauss(seed) for causal markers (uniform < lam), else 0; the count
// of causal markers in ro.out[0]
hipError_t gen_beta(uint64_t seed, double lam, int64_t S, int64_t M, double* beta, const RedOut& ro, hipStream_t st);
hipError_t scale_vec(int64_t n, double* v, double a, hipStream_t st);
// y_j = y_j + sqrt1mh2 * gauss(seed, noise stream, j)
hipError_t add_noise(uint64_t seed, int64_t N, double sd, double* y, hipStream_t st);

// ---- reductions --------------------------------------------------------------
// PUPD: a . (c + *beta * b) (a CG step's <d, p> with p = z + beta p fused);
// SQPUPD: (c + *beta * b)^2 (a is not used; pass b)
enum DotOp { DOT = 0, DIFF2 = 1, SUM = 2, PUPD = 3, SQPUPD = 4 };
struct DotTerm {
    const double* a;
    const double* b;
    int op;
    const double* c = nullptr;
    const double* beta = nullptr;
};
// gam1 chain (rides in a reduction launch, after the sum a2 = <bern, invQ>): from
// the sum of term `term`, a2: alpha2 = gam2*a2, eta2 = gam2/alpha2, gam1 =
// rho*min(max(eta2 - gam2, 1e-11), 1e11) + (1 - rho)*gam1_prev into out[0] =
// gam1, out[1] = eta2, out[2] = alpha2 (out null: none)
struct G1Chain {
    int term = 0;
    double gam2 = 0.0, rho = 0.0, gam1_prev = 0.0;
    double* out = nullptr;
};
// device copies of chosen results (the results themselves may land in mapped
// host memory, which a later kernel reads at a PCIe round trip's cost)
struct DotCopy {
    int n = 0;
    int term[2] = {0, 0};
    double* dst[2] = {nullptr, nullptr};
};
struct DotArgs {
    DotTerm t[kMaxTerms];
    int nt;
    G1Chain g1;    // formed by the launch's last block from its final sums
    DotCopy copy;  // ... and these copies stored by it
};
int red_blocks(int64_t n);
// ro.out[q] = term q summed over [0, n): per-block partials, then the blocks'
// sums in block order (fixed geometry: depends on n only)
hipError_t dots(const DotArgs& a, int64_t n, const RedOut& ro, hipStream_t st);
// a over [0, na) and b over [0, nb) in ONE launch, each bitwise as its own
// dots launch (its partials at its RedOut's part; one shared ticket; roa
// without a flag, rob's flag after both).  No PUPD / SQPUPD terms; the term
// counts of the pairs instantiated (10, 11) only, else hipErrorInvalidValue
hipError_t dots2(const DotArgs& a, int64_t na, const RedOut& roa, const DotArgs& b, int64_t nb, const RedOut& rob,
                 hipStream_t st);

// ---- denoiser (vamp::g1 / g1d) ---------------------------------------------
struct Mix {
    double probs[kMaxL];
    double vars[kMaxL];
    int L;
};
// The mixture words of the device EM update, kMixWords doubles: [0] L,
// [1, 1 + kMaxL) probs, [1 + kMaxL, 1 + 2 kMaxL) vars, [1 + 2 kMaxL] eta_max
constexpr int kMixWords = 2 + 2 * kMaxL;
// x1 = g1(r1) (then rho*x1 + (1-rho)*x1_prev if damp), x1d = g1d(r1),
// sum of x1d in ro.out[0].  mixw / gam1dev (may be null): the mixture's words
// (kMixWords, device: an EM round's update, em_sums' upd) and gam1 (G1Chain)
// from the device instead of mix and gam1.
// po (may be null, with mixw): the launch's last block also forms the next
// prelude's scalars (PreOut) from the sum of x1d
struct PreOut;
hipError_t denoise(int64_t M, const double* r1, double gam1, const Mix& mix, double* x1,
                   const double* x1_prev, int damp, double rho, double* x1d, const RedOut& ro, hipStream_t st,
                   const double* mixw = nullptr, const double* gam1dev = nullptr, const PreOut* po = nullptr);

// ---- EM prior update (vamp::updatePrior) per-marker sums --------------------
// the round's update of the mixture, formed on the device by the launch that
// finishes the round's sums (em_sums): out non-null
struct EmUpd {
    int64_t Mt = 0;
    int learn_vars = 0;
    double merge_vars_thr = 0.0;
    double* out = nullptr;     // the updated mixture's words (kMixWords, device: denoise's mixw)
    double* mirror = nullptr;  // the same words in mapped host memory, for the host's check
};
struct EmArgs {
    double omegas[kMaxL];
    double vars[kMaxL];
    double v[kMaxL];
    double lambda, noise_var, gam1, max_sigma;
    int L;
    // r1out (may be null): the round also forms r1 = (la*lx - lb*ly)/lc (the
    // lincomb_div of src/vamp.cpp:348-350, bit for bit) and stores it, instead
    // of reading r1: one launch where there were two
    const double* lx;
    const double* ly;
    double la, lb, lc;
    double* r1out;
    // dsc (may be null): gam1 = dsc[0] and la = eta2 = dsc[1] come from the
    // device (G1Chain), and noise_var = 1/gam1, v[j-1] = 1/(1/vars[j] + gam1)
    // are formed here, with the host's expressions (the host fields are unused)
    const double* dsc;
    // upd.out (may be null): the launch's last block also forms this round's
    // update of the mixture (vars and L here; vamp.cpp em_finish with one
    // round and the merging of close variances, src/vamp.cpp:598-642: the
    // host's expressions, bit for bit) into upd.out and upd.mirror
    EmUpd upd;
};
// ro.out[q], Q = 1 + 2(L-1): q=0 sum pin; q=j (1..L-1) sum beta_j pin;
// q=L-1+j sum beta_j (g_j^2 + v_j) pin
hipError_t em_sums(int64_t M, const double* r1, const EmArgs& a, const RedOut& ro, hipStream_t st);

// ---- elementwise VAMP updates -----------------------------------------------
// out = (a*x - b*y) / c        (r2 and r1 updates, src/vamp.cpp:259-261, 348-350)
hipError_t lincomb_div(int64_t n, double a, const double* x, double b, const double* y, double c,
                       double* out, hipStream_t st);
// out = a*x + b*y              (v = gamw*ATx(y) + gam2*r2, src/vamp.cpp:305-306)
hipError_t axpby(int64_t n, double a, const double* x, double b, const double* y, double* out,
                 hipStream_t st);
// bern[i] = (2*bit(seed,it,S+i) - 1) / sqrtMt
hipError_t bernoulli(uint64_t seed, int it, int64_t S, int64_t M, double sqrtMt, double* out,
                     hipStream_t st);
// The linear iteration's elementwise work before its CG solves, one launch
// (the same arithmetic as the separate kernels above, element for element):
//   r2 = (eta1*x1 - gam1*r1) / gam2      (src/vamp.cpp:259-261)
//   v = gamw*atxy + gam2*r2              (:303-306)
//   bern = the probe of iteration it     (:295-296, P2); bern_next: of it + 1 (may be null)
//   zero[z][i] = 0 for the non-null zero[z] (the CG solves' zero starts)
// The next iteration's prelude scalars, formed on the device by the launch
// that finishes its last sum (denoise, one rank), so that the prelude can be
// queued before the host has them: alpha1 = sum_d/Mt, eta1 = gam1/alpha1,
// gam2 = min(max(eta1 - gam1, 1e-11), 1e11), gamw = N/(tn + tc*Mt) (src/vamp.
// cpp:223, 230, 255-256, 521-528) and the CG's diag = gamw*(N-1)/N + gam2
// (:676-677): the host's expressions, bit for bit.  out (device) = {eta1, gam2, gamw, diag,
// gam1}, mirror (mapped host) = its first four, for the host's check.  tn,
// tc: device copies (DotCopy) of earlier launches' results
struct PreOut {
    const double* tn = nullptr;
    const double* tc = nullptr;
    double Mt = 0.0, N = 0.0;
    double* out = nullptr;
    double* mirror = nullptr;
};
// Several ranks: what the one-rank launches' last blocks form from their final
// sums (G1Chain, EmArgs.upd, PreOut), formed by one thread after the sums'
// all-reduce (vamp.cpp's host-free tail; the same expressions, bit for bit).
// mode 0: gam1_chain from src[0] = a2 into g1.out, and the device copies
// cp_dst[i] = *cp_src[i]; 1: one EM round's update of the mixture (L, vars)
// from src (1 + 2(L-1) sums) into upd.out / upd.mirror; 2: the next prelude's
// scalars from src[0] = the sum of x1d and gam1 = gam1dev[0] into po
struct TailPost {
    int mode = 0;
    const double* src = nullptr;
    G1Chain g1;
    const double* cp_src[2] = {nullptr, nullptr};
    double* cp_dst[2] = {nullptr, nullptr};
    int L = 0;
    double vars[kMaxL] = {};
    EmUpd upd;
    PreOut po;
    const double* gam1dev = nullptr;
};
hipError_t tail_post(const TailPost& t, hipStream_t st);
// scal (device, may be null): the prelude's scalars {eta1, gam2, gamw, diag,
// gam1} from PreOut.out instead of the Prelude's own (prelude_cg_init only)
struct PreDev {
    const double* scal = nullptr;
};
struct Prelude {
    double eta1, gam1, gam2, gamw;
    PreDev dev;  // prelude_cg_init only
    const double* x1;
    const double* r1;
    const double* atxy;
    double* r2;
    double* v;
    uint64_t seed;
    int it;
    int64_t S;
    double sqrtMt;
    double* bern;
    double* bern_next;
    double* zero[2];
};
hipError_t prelude(int64_t M, const Prelude& p, hipStream_t st);
// out = x / d
hipError_t div_scalar(int64_t n, const double* x, double d, double* out, hipStream_t st);
// out[0, n) = x / d and out[n, 2n) = r / d in one launch (the iteration writer)
hipError_t div2_scalar(int64_t n, const double* x, const double* r, double d, double* out, hipStream_t st);

// ---- probit model (src/vamp_probit.cpp) -------------------------------------
// z1[i] = g1_bin_class(p1[i], tau1, y[i]); the sum of g1d_bin_class in ro.out[0]
// (src/vamp_probit.cpp:213-233, 469-488; probit_var = 1, m_cov = 0)
hipError_t probit_denoise(int64_t N, const double* p1, const double* y, double tau1, double* z1, const RedOut& ro,
                          hipStream_t st);
// predict_probit(z_k, 0.5) + confusion_matrix against y (src/vamp_probit.cpp:619-651),
// nz <= 2 vectors at z + k*ld; ro.out[4k + {TP, TN, FP, FN}]
hipError_t probit_confusion(int64_t N, int nz, const double* z, int64_t ld, const double* y, const RedOut& ro,
                            hipStream_t st);
// P2 start: p1[i] = gauss(seed ^ salt, 0, i) (replaces simulate(N, {1}, {1}), :53)
hipError_t probit_p1(uint64_t seed, int64_t N, double* p1, hipStream_t st);

// ---- association tests (src/main_meth.cpp:206-264, src/data.cpp:385-417) -------
// stats[5j + {0..4}] = sum X, sum X^2, sum X*ym, sum ym, sum ym^2 over the
// samples of marker j (RAW X), ym = ymod + X / sqrtN * x1[j]  (data::pvals_loo)
hipError_t loo_sums(const Shard& s, const double* ymod, const double* x1, double sqrtN, double* stats,
                    hipStream_t st, int variant = kLooDefault, const Timing& tm = Timing{});
std::string loo_kernel_name(int variant);
int loo_variant_count();
bool loo_variant_ok(int v);
// pvals[j] = linear_reg1d_pvals(stats[5j..5j+4], n)  (src/utilities.cpp:269-282)
hipError_t loo_pvals(int64_t M, const double* stats, int n, double* pvals, hipStream_t st);
// pvals[j] = P(N(r1_j, 1/(gam1 N)) <= 0), flipped for r1_j <= 0 (src/main_meth.cpp:231-236)
hipError_t se_pvals(int64_t M, const double* r1, double gam1, int64_t N, double* pvals, hipStream_t st);
// *p = v (one thread; a host value placed in stream order)
hipError_t set_scalar(double* p, double v, hipStream_t st);
// out = x * a
hipError_t mul_scalar(int64_t n, const double* x, double a, double* out, hipStream_t st);

// ---- host completion flag (system-scope store into mapped host memory) -------
hipError_t signal_host(unsigned long long* flag, unsigned long long seq, hipStream_t st);
// the same with a relaxed store (what it announces was written by earlier kernels)
hipError_t post_flag(unsigned long long* flag, unsigned long long seq, hipStream_t st);
// copies a[0..na) -> ha and b[0..nb) -> hb (mapped host memory), then stores seq into flag
hipError_t publish_host(const double* a, int na, double* ha, const double* b, int nb, double* hb,
                        unsigned long long* flag, unsigned long long seq, hipStream_t st);

// ---- PCG (vamp::precondCG_solver), K right-hand sides --------------------------
struct CgVecs {
    double* mu[kMaxRhs];
    double* r[kMaxRhs];
    double* z[kMaxRhs];
    double* p[kMaxRhs];
    const double* d[kMaxRhs];   // lmmse_mult(mu0) for init (nullptr: mu0 == 0), A p in the loop
    const double* v[kMaxRhs];
    const double* atx0[kMaxRhs];  // init only: A^T(A mu0) computed earlier (then d is ignored)
    double tau, gam2;             // init only, with atx0
    // cg_update only (may be null): W += alpha * S alongside mu += alpha * p,
    // S = the step's raw A^T(A p) (atx sraw), so W tracks A^T A mu
    double* W[kMaxRhs];
    const double* S[kMaxRhs];
    // cg_update only (may be null): AW += alpha * AS over nA samples, AS = the
    // step's A p (the replicated N-vector of the A.x pass), so AW tracks A mu
    double* AW[kMaxRhs];
    const double* AS[kMaxRhs];
    int64_t nA;
    // cg_update only, one-pass operator (may be null): over nA samples,
    // q = AR/diag [+ beta*Q when fuse] is stored in Q (the step's A p, as the
    // pass formed it), AW += alpha*q, AR -= AD*alpha (A r tracks r -= d*alpha)
    double* Q[kMaxRhs];
    double* AR[kMaxRhs];
    const double* AD[kMaxRhs];
    // one rank, one-pass operator (may be null): AD is not read; A d of
    // sample i is summed here from the operator's per-slot partials
    // adpart[(t*kMaxRhs + k)*adld + i], t < adslots, in op_reduce's order, and
    // divided by addiv (the separate op_reduce launch folded into this one).
    // Without adpart, addiv > 0: AD holds the all-reduced sums not yet divided,
    // and each is divided here as it is read (the vec_div launch folded in)
    const double* adpart;
    int64_t adld;
    int adslots;
    double addiv;
};
// r = v - d (or v, or v - (atx0*tau + gam2*mu)), z = r/diag, p = z;
// <r,z>, <v,v> per system in ro.out (2K values)
hipError_t cg_init(int K, int64_t M, const CgVecs& c, double diag, const RedOut& ro, hipStream_t st);
// Device-side CG control.  The scalar recurrences of a CG step (alpha, the
// Onsager and residual stops, beta) run on the device from a CgState, so the
// host can queue the next step before this one's sums are known: every launch
// of a step is gated on `any` (a step queued after the last system stopped
// does nothing).  `mirror` (mapped host memory, two slots) receives
// seq/any/iters of step `it` in slot it & 1, then the step's flag.  Two slots:
// when the host reads step i-1's decision, step i is already queued and may
// have decided too (a gated step decides in microseconds); one shared slot let
// ranks read different steps' decisions and issue different collectives.
// off[k]: steps system k took before step 0 (the head start, pcg.cpp), so its
// count after step `it` is it + 1 + off[k]; a system stops after maxit steps.
struct CgState {
    double rz[kMaxRhs], vv[kMaxRhs], prev_ons[kMaxRhs], beta[kMaxRhs];
    double gam2, tol;
    int active[kMaxRhs], iters[kMaxRhs], onsager[kMaxRhs], off[kMaxRhs];
    int K, any, maxit;
};
// A step's decision in ONE 64-bit word (the one-pass CG: K <= 2 systems,
// iteration counts below 2^15): the step's sequence number in the high half
// (so the word grows with it), any in bit 30, iters[1] in bits 15-29 and
// iters[0] in bits 0-14.  One system-scope store publishes it whole: no
// mirror, no ordering wait.
constexpr int kCgPackMaxIter = (1 << 15) - 2;
__host__ __device__ inline unsigned long long cg_pack(unsigned long long seq, int any, int it0, int it1) {
    return (seq << 32) | ((unsigned long long)(any ? 1 : 0) << 30) | ((unsigned long long)(it1 & 0x7fff) << 15) |
           (unsigned long long)(it0 & 0x7fff);
}
struct CgMirror {
    unsigned long long seq;  // the step's flag value: the slot holds that step's decision
    int any;
    int iters[kMaxRhs];
};
constexpr int kCgMirrorSlots = 2;
// *dst = init (one thread)
hipError_t cg_start(const CgState& init, CgState* dst, hipStream_t st);
// *dst = init with rz[k], vv[k] = sums[2k], sums[2k+1] (cg_init's sums, in device memory)
// gam2dev (may be null): init.gam2 from the device (a start queued ahead: the
// next prelude's scalars, PreOut.out + 1)
hipError_t cg_start_from(const CgState& init, const double* sums, CgState* dst, hipStream_t st,
                         const double* gam2dev = nullptr);
// prelude() and cg_init() in one launch (cg_init's grid and sums: bitwise the
// two launches), where cg_init's v_k may be the prelude's v or bern (taken from
// registers).  start (may be null): the last block also writes *dst = *start
// with rz[k], vv[k] from the sums (cg_start_from; one rank, the sums final)
hipError_t prelude_cg_init(int K, int64_t M, const Prelude& p, const CgVecs& c, double diag, const RedOut& ro,
                           const CgState* start, CgState* dst, hipStream_t st);
// for active k: [fuse: p = z + beta_k p, stored] alpha_k = rz[k] / dp_dev[k];
// mu += alpha p; r -= d alpha; z = r/diag; <r,z>, <r,r>, <v,mu> in ro.out (3K
// values, k-major; zeros for stopped systems); gated on cs->any.  dc.on (one
// rank: the sums are final): the last block also takes cg_decide's decisions.
struct CgDecide {
    int on = 0, it = 0;
    // pack: *flag receives the decision as ONE word (cg_pack) instead of the
    // mirror slot + sequence number
    int pack = 0;
    int mask = 0xf;  // the systems this step is for (the others keep their state; see cg_update)
    CgMirror* mirror = nullptr;
    unsigned long long* flag = nullptr;
    unsigned long long seq = 0;
};
// pp_dev (may be null): dp_dev holds |A p_k|^2 and pp_dev |p_k|^2, and
// <d,p> = tau*|A p|^2 + gam2*|p|^2 (c.tau, c.gam2).  fuse: bit k set when
// system k's direction update is fused into this step; dc.mask: the systems
// this step updates (the others are left as they are: the head start's step
// of one system, pcg.cpp)
hipError_t cg_update(int K, int64_t M, const CgVecs& c, double diag, CgState* cs, const double* dp_dev,
                     const double* pp_dev, int fuse, const RedOut& ro, const CgDecide& dc, hipStream_t st);
// step `it`'s decisions from red (the 3K sums of cg_update, summed over ranks),
// src/vamp.cpp:700-750, for the systems in mask; then mirror and flag (each
// stored when non-null, even when gated off)
hipError_t cg_decide(CgState* cs, const double* red, int it, CgMirror* mirror, unsigned long long* flag,
                     unsigned long long seq, hipStream_t st, int mask = 0xf, int pack = 0);

}  // namespace vk
