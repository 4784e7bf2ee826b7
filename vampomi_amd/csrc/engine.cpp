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
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include <fcntl.h>
#include <unistd.h>

#include "../../include/vampomi.h"
#include "hostio.h"
#include "kernels.h"

// ---------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------
static thread_local std::string g_err;

static vampomi_status fail(vampomi_status s, const std::string& msg) {
    g_err = msg;
    return s;
}

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

// ---------------------------------------------------------------------------
// the context
// ---------------------------------------------------------------------------
struct VampRun;

struct TimedLaunch {
    hipEvent_t a, b;
    int cls;  // 0 ax, 1 atx
    int K;
    double bytes, flops;
};

struct vampomi_ctx {
    int rank = 0, nranks = 1, device = 0;
    int64_t N = 0, Mt = 0, M = 0, S = 0, Mm = 0, ld = 0;
    double alpha_scale = 1.0;
    double sqrtN = 1.0;
    hipStream_t st = nullptr;
    ncclComm_t comm = nullptr;

    double* X = nullptr;
    double* mave = nullptr;
    double* msig = nullptr;
    double* y = nullptr;  // ld, zero pad
    std::vector<double> y_host;
    bool have_X = false, have_y = false;

    vk::AxPlan axp{};
    double* ax_part = nullptr;
    double* red_part = nullptr;
    size_t red_cap = 0;
    double* scal = nullptr;     // device scalars
    double* h_scal = nullptr;   // pinned mirror
    double* nbuf = nullptr;     // kMaxRhs * ld scratch N-vectors (API calls)
    double* mbuf = nullptr;     // (2*kMaxRhs) * M scratch M-vectors (API calls)

    bool timing = false;
    std::vector<TimedLaunch> pending;
    std::vector<hipEvent_t> ev_pool;
    vampomi_stats stats{};

    std::unique_ptr<VampRun> run;

    vk::Shard shard() const { return vk::Shard{X, ld, N, M, mave, msig}; }
};

// scalar slots in ctx->scal
enum : int { SL_DOTS = 0, SL_DP = 16, SL_CG = 32, SL_EM = 64, SL_TOTAL = 256 };

static vampomi_status dev_alloc(double** p, size_t n) {
    if (n == 0) n = 1;
    hipError_t e = hipMalloc((void**)p, n * sizeof(double));
    if (e != hipSuccess)
        return fail(VAMPOMI_ERR_OOM, "hipMalloc(" + std::to_string(n * sizeof(double)) + " B): " + hipGetErrorString(e));
    return VAMPOMI_OK;
}

static void dev_free(double*& p) {
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
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

static void resolve_timing(vampomi_ctx* c) {
    for (auto& t : c->pending) {
        float ms = 0.f;
        if (hipEventSynchronize(t.b) == hipSuccess && hipEventElapsedTime(&ms, t.a, t.b) == hipSuccess) {
            vampomi_kernel_stat* s = t.cls == 0 ? &c->stats.ax : &c->stats.atx;
            vampomi_kernel_stat* sk = t.cls == 0 ? &c->stats.ax_k[t.K - 1] : &c->stats.atx_k[t.K - 1];
            for (vampomi_kernel_stat* x : {s, sk}) {
                x->launches += 1;
                x->ms_total += ms;
                x->bytes_total += t.bytes;
                x->flops_total += t.flops;
            }
        }
        c->ev_pool.push_back(t.a);
        c->ev_pool.push_back(t.b);
    }
    c->pending.clear();
}

// algorithmic bytes / flops of one pass with K right-hand sides:
// X once, the K N-vectors, mave/msig and the K M-vectors; (x - mu) once per
// element and one fma per right-hand side.
static double pass_bytes(const vampomi_ctx* c, int K) {
    return 8.0 * (double)c->N * (double)c->M + 8.0 * K * (double)c->N + 8.0 * (2.0 + K) * (double)c->M;
}
static double pass_flops(const vampomi_ctx* c, int K) { return (double)c->N * (double)c->M * (1.0 + 2.0 * K); }

// ---------------------------------------------------------------------------
// reductions
// ---------------------------------------------------------------------------
static vampomi_status host_sync(vampomi_ctx* c) {
    HIPCHK(hipStreamSynchronize(c->st));
    c->stats.host_syncs++;
    return VAMPOMI_OK;
}

static vampomi_status allreduce_dev(vampomi_ctx* c, double* buf, size_t n) {
    if (c->nranks > 1 && n > 0) NCCLCHK(ncclAllReduce(buf, buf, n, ncclDouble, ncclSum, c->comm, c->st));
    return VAMPOMI_OK;
}

// Q (<= 8) dot terms over length n; sync => summed over ranks (the
// reference's inner_prod(..., sync=1)).  Results land in out[0..Q).
static vampomi_status dots(vampomi_ctx* c, const std::vector<vk::DotTerm>& terms, int64_t n, bool sync, double* out) {
    vk::DotArgs a{};
    a.nt = (int)terms.size();
    for (int q = 0; q < a.nt; ++q) a.t[q] = terms[q];
    const int nb = vk::red_blocks(n);
    HIPCHK(vk::dots_partial(a, n, c->red_part, c->st));
    HIPCHK(vk::sum_partials(c->red_part, nb, a.nt, c->scal + SL_DOTS, c->st));
    if (sync) STCHK(allreduce_dev(c, c->scal + SL_DOTS, a.nt));
    HIPCHK(hipMemcpyAsync(c->h_scal + SL_DOTS, c->scal + SL_DOTS, sizeof(double) * a.nt, hipMemcpyDeviceToHost, c->st));
    STCHK(host_sync(c));
    for (int q = 0; q < a.nt; ++q) out[q] = c->h_scal[SL_DOTS + q];
    return VAMPOMI_OK;
}

static vk::DotTerm T(const double* a, const double* b, int op = vk::DOT) { return vk::DotTerm{a, b, op}; }

// ---------------------------------------------------------------------------
// operators on device buffers
// ---------------------------------------------------------------------------
// out_k = Ax(x_k) for K <= 4; outputs at outbase + k*ld (contiguous so that one
// all-reduce carries them all).  COLLECTIVE.
static vampomi_status ax_dev(vampomi_ctx* c, int K, const double* const* x, double* outbase) {
    if (!c->have_X) return fail(VAMPOMI_ERR_STATE, "Ax before the methylation data was loaded");
    vk::CPtrs xs{};
    vk::Ptrs os{};
    for (int k = 0; k < K; ++k) {
        xs.p[k] = x[k];
        os.p[k] = outbase + (int64_t)k * c->ld;
    }
    TimedLaunch t{};
    if (c->timing) {
        t.a = ev_get(c);
        t.b = ev_get(c);
        HIPCHK(hipEventRecord(t.a, c->st));
    }
    HIPCHK(vk::ax_partial(c->shard(), c->axp, K, xs, c->ax_part, c->st));
    if (c->timing) {
        HIPCHK(hipEventRecord(t.b, c->st));
        t.cls = 0;
        t.K = K;
        t.bytes = pass_bytes(c, K);
        t.flops = pass_flops(c, K);
        c->pending.push_back(t);
    }
    c->stats.a_passes_exec++;
    if (c->nranks == 1) {
        HIPCHK(vk::ax_reduce(c->axp, K, c->N, c->ld, c->ax_part, os, c->sqrtN, c->st));
    } else {
        HIPCHK(vk::ax_reduce(c->axp, K, c->N, c->ld, c->ax_part, os, 0.0, c->st));
        STCHK(allreduce_dev(c, outbase, (size_t)K * c->ld));  // src/data.cpp:367
        HIPCHK(vk::vec_div(K, c->N, c->ld, os, c->sqrtN, c->st));
    }
    return VAMPOMI_OK;
}

// out_k = ATx(u_k) (mode 0) or tau*ATx(u_k) + gam2*p_k with <out_k,p_k> summed
// over ranks into ctx->scal[SL_DP + k] (mode 1).  u_k are ld-padded N-vectors.
static vampomi_status atx_dev(vampomi_ctx* c, int K, const double* const* u, double* const* out, int mode,
                              double tau, double gam2, const double* const* p) {
    if (!c->have_X) return fail(VAMPOMI_ERR_STATE, "ATx before the methylation data was loaded");
    if (c->M <= 0) return VAMPOMI_OK;
    vk::CPtrs us{}, ps{};
    vk::Ptrs os{};
    for (int k = 0; k < K; ++k) {
        us.p[k] = u[k];
        os.p[k] = out[k];
        ps.p[k] = p ? p[k] : nullptr;
    }
    TimedLaunch t{};
    if (c->timing) {
        t.a = ev_get(c);
        t.b = ev_get(c);
        HIPCHK(hipEventRecord(t.a, c->st));
    }
    HIPCHK(vk::atx(c->shard(), K, us, os, 1.0 / c->sqrtN, mode, tau, gam2, ps, c->red_part, c->st));
    if (c->timing) {
        HIPCHK(hipEventRecord(t.b, c->st));
        t.cls = 1;
        t.K = K;
        t.bytes = pass_bytes(c, K);
        t.flops = pass_flops(c, K);
        c->pending.push_back(t);
    }
    c->stats.a_passes_exec++;
    if (mode == 1) {
        HIPCHK(vk::sum_partials(c->red_part, vk::atx_blocks(c->M), K, c->scal + SL_DP, c->st));
        STCHK(allreduce_dev(c, c->scal + SL_DP, K));
    }
    return VAMPOMI_OK;
}

// d_k = tau*A^T A v_k + gam2*v_k (lmmse_mult, src/vamp.cpp:645-662) for K
// vectors that are not all-zero; <d_k, v_k> lands in scal[SL_DP+k]. COLLECTIVE
static vampomi_status lmmse_dev(vampomi_ctx* c, int K, const double* const* v, double* const* d, double tau,
                                double gam2, double* nscratch) {
    STCHK(ax_dev(c, K, v, nscratch));
    const double* u[vk::kMaxRhs];
    for (int k = 0; k < K; ++k) u[k] = nscratch + (int64_t)k * c->ld;
    return atx_dev(c, K, u, d, 1, tau, gam2, v);
}

// ---------------------------------------------------------------------------
// PCG (vamp::precondCG_solver, src/vamp.cpp:664-757) for up to kMaxRhs
// independent right-hand sides that share the operator tau*A^T A + gam2*I.
// With batch=true every CG step streams X twice for all still-active systems
// together; each system keeps its own scalars and stopping rule, so its
// iterates are exactly those of a solo solve.
// ---------------------------------------------------------------------------
struct CgSystem {
    const double* v;      // right-hand side (device, M)
    double* mu;           // in: start (if mu0_nonzero), out: solution
    bool mu0_nonzero;     // false: start from zeros (lmmse_mult short-circuit)
    bool onsager;         // denoiser == 0 in the reference: extra Onsager stop
    int iters = 0;
    // work vectors (device, M)
    double *r, *z, *p, *d;
};

static vampomi_status pcg_run(vampomi_ctx* c, std::vector<CgSystem*> sys, double tau, double gam2, int max_iter,
                              double tol, double* nscratch, int64_t* ref_passes) {
    const int64_t M = c->M, N = c->N;
    const double diag = tau * (double)(N - 1) / (double)N + gam2;  // :676-677
    const int K = (int)sys.size();
    // initial residual r = v - lmmse_mult(mu0)
    {
        std::vector<CgSystem*> nz;
        for (auto* s : sys)
            if (s->mu0_nonzero) nz.push_back(s);
        if (!nz.empty()) {
            const double* vv[vk::kMaxRhs];
            double* dd[vk::kMaxRhs];
            for (size_t k = 0; k < nz.size(); ++k) {
                vv[k] = nz[k]->mu;
                dd[k] = nz[k]->d;
            }
            STCHK(lmmse_dev(c, (int)nz.size(), vv, dd, tau, gam2, nscratch));
            if (ref_passes) *ref_passes += 2 * (int64_t)nz.size();
        }
        vk::CgVecs cv{};
        for (int k = 0; k < K; ++k) {
            cv.mu[k] = sys[k]->mu;
            cv.r[k] = sys[k]->r;
            cv.z[k] = sys[k]->z;
            cv.p[k] = sys[k]->p;
            cv.d[k] = sys[k]->mu0_nonzero ? sys[k]->d : nullptr;
            cv.v[k] = sys[k]->v;
        }
        int nb = 0;
        HIPCHK(vk::cg_init(K, M, cv, diag, c->red_part, &nb, c->st));
        HIPCHK(vk::sum_partials(c->red_part, nb, 2 * K, c->scal + SL_CG, c->st));
        STCHK(allreduce_dev(c, c->scal + SL_CG, 2 * K));
        HIPCHK(hipMemcpyAsync(c->h_scal + SL_CG, c->scal + SL_CG, sizeof(double) * 2 * K, hipMemcpyDeviceToHost, c->st));
        STCHK(host_sync(c));
    }
    std::vector<double> rz(K), vv(K), prev_ons(K, 0.0);
    std::vector<int> active;
    for (int k = 0; k < K; ++k) {
        rz[k] = c->h_scal[SL_CG + 2 * k];
        vv[k] = c->h_scal[SL_CG + 2 * k + 1];
        sys[k]->iters = 0;
        active.push_back(k);
    }
    for (int i = 0; i < max_iter && !active.empty(); ++i) {
        const int Ka = (int)active.size();
        vk::CgVecs cv{};
        vk::CgScalars rzs{};
        const double* pp[vk::kMaxRhs];
        double* dd[vk::kMaxRhs];
        for (int a = 0; a < Ka; ++a) {
            CgSystem* s = sys[active[a]];
            cv.mu[a] = s->mu;
            cv.r[a] = s->r;
            cv.z[a] = s->z;
            cv.p[a] = s->p;
            cv.d[a] = s->d;
            cv.v[a] = s->v;
            rzs.rz[a] = rz[active[a]];
            pp[a] = s->p;
            dd[a] = s->d;
        }
        // d = lmmse_mult(p)   (:700)
        STCHK(lmmse_dev(c, Ka, pp, dd, tau, gam2, nscratch));
        if (ref_passes) *ref_passes += 2 * (int64_t)Ka;
        // alpha = <r,z>/<d,p>; mu += alpha p; r -= alpha d; z = r/diag
        int nb = 0;
        HIPCHK(vk::cg_update(Ka, M, cv, diag, rzs, c->scal + SL_DP, c->red_part, &nb, c->st));
        HIPCHK(vk::sum_partials(c->red_part, nb, 3 * Ka, c->scal + SL_CG, c->st));
        STCHK(allreduce_dev(c, c->scal + SL_CG, 3 * Ka));
        HIPCHK(hipMemcpyAsync(c->h_scal + SL_CG, c->scal + SL_CG, sizeof(double) * 3 * Ka, hipMemcpyDeviceToHost,
                              c->st));
        STCHK(host_sync(c));
        std::vector<int> still;
        vk::CgVecs pv{};
        vk::CgBeta beta{};
        int np = 0;
        for (int a = 0; a < Ka; ++a) {
            const int k = active[a];
            CgSystem* s = sys[k];
            s->iters = i + 1;
            const double rz_new = c->h_scal[SL_CG + 3 * a];
            const double rr = c->h_scal[SL_CG + 3 * a + 1];
            const double vmu = c->h_scal[SL_CG + 3 * a + 2];
            if (s->onsager) {  // :708-726
                const double ons = gam2 * vmu;
                const double rel = ons != 0 ? std::fabs((ons - prev_ons[k]) / ons) : 1;
                if (rel < 1e-8) continue;
                prev_ons[k] = ons;
            }
            double b = std::pow(rz[k], -1);  // :731
            b *= rz_new;                       // :736
            rz[k] = rz_new;
            const double rel_err = std::sqrt(rr) / std::sqrt(vv[k]);  // :742-744
            if (rel_err < tol) continue;                               // :750
            still.push_back(k);
            pv.z[np] = s->z;
            pv.p[np] = s->p;
            beta.beta[np] = b;
            ++np;
        }
        if (np > 0) HIPCHK(vk::cg_pupdate(np, M, pv, beta, c->st));  // p = z + beta p
        active.swap(still);
    }
    return VAMPOMI_OK;
}

// ---------------------------------------------------------------------------
// VAMP linear model state (vamp::vamp + vamp::infere_linear)
// ---------------------------------------------------------------------------
struct VampRun {
    vampomi_params prm{};
    vampomi_result* res = nullptr;
    bool write = false;
    std::string out_dir, out_name, p_params, p_metrics, p_prior;
    int it = 0;
    bool stopped = false;
    int L = 0;
    double probs[VAMPOMI_MAX_L] = {}, vars[VAMPOMI_MAX_L] = {};
    double gam1 = 0, gam2 = 0, gamw = 0;
    double alpha1 = 0, alpha2 = 0, eta1 = 0, eta2 = 0;
    double metrics[6] = {0, 0, 0, 0, 0, 0}, params[5] = {0, 0, 0, 0, 0};
    // device M-vectors
    double *r1 = nullptr, *x1 = nullptr, *x1p = nullptr, *x1d = nullptr, *r2 = nullptr, *x2 = nullptr;
    double *bern = nullptr, *invQ = nullptr, *v = nullptr, *atxy = nullptr, *ts = nullptr, *tmpM = nullptr;
    double* cgw[8] = {};  // r,z,p,d for 2 systems
    // device N-vectors (ld each)
    double *z1 = nullptr, *nb2 = nullptr /* 2*ld: Ax(x2), Ax(invQ) */, *nsc = nullptr /* kMaxRhs*ld */;
    std::vector<double> hM;
    int64_t passes_ref = 0;

    ~VampRun() {
        for (double** p : {&r1, &x1, &x1p, &x1d, &r2, &x2, &bern, &invQ, &v, &atxy, &ts, &tmpM, &z1, &nb2, &nsc})
            dev_free(*p);
        for (auto& p : cgw) dev_free(p);
    }
};

static double smax(double a, double b) { return (a < b) ? b : a; }  // std::max
static double smin(double a, double b) { return (b < a) ? b : a; }  // std::min

// updatePrior (src/vamp.cpp:531-643)
static vampomi_status update_prior(vampomi_ctx* c, VampRun& R) {
    const double noise_var = 1 / R.gam1;
    double lambda = 1 - R.probs[0];
    double omegas[VAMPOMI_MAX_L];
    for (int j = 0; j < R.L; ++j) omegas[j] = R.probs[j];
    for (int j = 1; j < R.L; ++j) omegas[j] /= lambda;
    for (int emit = 0; emit < R.prm.EM_max_iter; ++emit) {
        const int L = R.L;
        double max_sigma = R.vars[0];
        for (int j = 1; j < L; ++j) max_sigma = smax(max_sigma, R.vars[j]);  // std::max_element
        double probs_prev[VAMPOMI_MAX_L], vars_prev[VAMPOMI_MAX_L];
        std::memcpy(probs_prev, R.probs, sizeof probs_prev);
        std::memcpy(vars_prev, R.vars, sizeof vars_prev);
        vk::EmArgs a{};
        for (int j = 0; j < L; ++j) {
            a.omegas[j] = omegas[j];
            a.vars[j] = R.vars[j];
        }
        for (int j = 1; j < L; ++j) a.v[j - 1] = 1.0 / (1.0 / R.vars[j] + R.gam1);
        a.lambda = lambda;
        a.noise_var = noise_var;
        a.gam1 = R.gam1;
        a.max_sigma = max_sigma;
        a.L = L;
        const int Q = 1 + 2 * (L - 1);
        int nb = 0;
        HIPCHK(vk::em_sums(c->M, R.r1, a, c->red_part, &nb, c->st));
        HIPCHK(vk::sum_partials(c->red_part, nb, Q, c->scal + SL_EM, c->st));
        STCHK(allreduce_dev(c, c->scal + SL_EM, Q));
        HIPCHK(hipMemcpyAsync(c->h_scal + SL_EM, c->scal + SL_EM, sizeof(double) * Q, hipMemcpyDeviceToHost, c->st));
        STCHK(host_sync(c));
        const double lambda_total = c->h_scal[SL_EM];
        lambda = lambda_total / (double)c->Mt;
        const double sum_of_pin = lambda_total;
        for (int j = 0; j < L - 1; ++j) {
            const double res_total = c->h_scal[SL_EM + 1 + j];
            const double res_gammas_total = c->h_scal[SL_EM + L + j];
            if (R.prm.learn_vars == 1) R.vars[j + 1] = res_gammas_total / res_total;
            omegas[j + 1] = res_total / sum_of_pin;
            R.probs[j + 1] = lambda * omegas[j + 1];
        }
        R.probs[0] = 1 - lambda;
        double dprob = 0, nprob = 0, dvar = 0, nvar = 0;
        for (int j = 0; j < L; ++j) {
            dprob += (R.probs[j] - probs_prev[j]) * (R.probs[j] - probs_prev[j]);
            nprob += R.probs[j] * R.probs[j];
            dvar += (R.vars[j] - vars_prev[j]) * (R.vars[j] - vars_prev[j]);
            nvar += R.vars[j] * R.vars[j];
        }
        const double dist_probs = std::sqrt(dprob / nprob), dist_vars = std::sqrt(dvar / nvar);
        if (R.prm.verbosity == 1 && c->rank == 0)
            std::printf("it = %d: dist_probs = %g & dist_vars = %g\n", emit, dist_probs, dist_vars);
        if (dist_probs < R.prm.EM_err_thr && dist_vars < R.prm.EM_err_thr) break;
    }
    // merging close variances (:626-642)
    for (int j = 0; j < R.L; ++j) {
        for (int k = j + 1; k < R.L; ++k) {
            const double denom = R.vars[j] != 0 ? smin(R.vars[j], R.vars[k]) : 1e-7;
            if (std::fabs(R.vars[j] - R.vars[k]) / denom < R.prm.merge_vars_thr) {
                const double sum2probs = R.probs[j] + R.probs[k];
                for (int q = k; q + 1 < R.L; ++q) {
                    R.vars[q] = R.vars[q + 1];
                    R.probs[q] = R.probs[q + 1];
                }
                R.L--;
                R.probs[j] = sum2probs;
                k--;
            }
        }
    }
    return VAMPOMI_OK;
}

// err_measures (src/vamp.cpp:760-852), scalars only; Axest = A xhat already
// computed (z1 for ind 1, Ax(x2_hat) for ind 2: the reference recomputes the
// latter at :826 with the same operator on the same input).
static vampomi_status err_measures(vampomi_ctx* c, VampRun& R, const double* xhat, const double* Axest, int ind) {
    double m3[3], nu[2], ns[3];
    STCHK(dots(c, {T(xhat, R.ts), T(xhat, xhat), T(R.ts, R.ts)}, c->M, true, m3));
    const double corr = m3[0] / std::sqrt(m3[1] * m3[2]);
    STCHK(dots(c, {T(c->y, Axest, vk::DIFF2), T(c->y, c->y)}, c->N, false, nu));
    STCHK(dots(c, {T(Axest, c->y), T(Axest, Axest), T(c->y, c->y)}, c->N, true, ns));
    const double l2_pred_err = std::sqrt(nu[0] / nu[1]);
    const double R2 = 1 - l2_pred_err * l2_pred_err;
    const double corr_y = ns[0] / std::sqrt(ns[1] * ns[2]);
    const double corr_y_2 = corr_y * corr_y;
    if (ind == 1) {
        R.metrics[1] = corr;
        R.metrics[0] = R2;
        R.metrics[4] = corr_y_2;
    } else {
        R.metrics[3] = corr;
        R.metrics[2] = R2;
        R.metrics[5] = corr_y_2;
    }
    return VAMPOMI_OK;
}

static vampomi_status vamp_alloc(vampomi_ctx* c, VampRun& R) {
    const size_t M = (size_t)std::max<int64_t>(c->M, 1), ld = (size_t)c->ld;
    for (double** p : {&R.r1, &R.x1, &R.x1p, &R.x1d, &R.r2, &R.x2, &R.bern, &R.invQ, &R.v, &R.atxy, &R.ts, &R.tmpM})
        STCHK(dev_alloc(p, M));
    for (auto& p : R.cgw) STCHK(dev_alloc(&p, M));
    STCHK(dev_alloc(&R.z1, ld));
    STCHK(dev_alloc(&R.nb2, 2 * ld));
    STCHK(dev_alloc(&R.nsc, vk::kMaxRhs * ld));
    HIPCHK(hipMemsetAsync(R.z1, 0, ld * 8, c->st));
    HIPCHK(hipMemsetAsync(R.nb2, 0, 2 * ld * 8, c->st));
    HIPCHK(hipMemsetAsync(R.nsc, 0, vk::kMaxRhs * ld * 8, c->st));
    return VAMPOMI_OK;
}

static vampomi_status upload_or_zero(vampomi_ctx* c, double* dst, const double* host, int64_t n) {
    if (n <= 0) return VAMPOMI_OK;
    if (host)
        HIPCHK(hipMemcpyAsync(dst, host, (size_t)n * 8, hipMemcpyHostToDevice, c->st));
    else
        HIPCHK(hipMemsetAsync(dst, 0, (size_t)n * 8, c->st));
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_vamp_begin(vampomi_ctx* c, const vampomi_params* p, vampomi_result* r) {
    if (!c || !p) return fail(VAMPOMI_ERR_ARG, "null argument");
    if (!c->have_X || !c->have_y) return fail(VAMPOMI_ERR_STATE, "load methylation data and phenotype first");
    if (p->model && std::strcmp(p->model, "linear") != 0)
        return fail(VAMPOMI_ERR_MODEL, std::string("model '") + p->model + "' is not supported (linear only)");
    if (p->L < 1 || p->L > VAMPOMI_MAX_L) return fail(VAMPOMI_ERR_ARG, "number of mixture components out of range");
    c->run.reset(new VampRun());
    VampRun& R = *c->run;
    R.prm = *p;
    R.res = r;
    R.out_dir = p->out_dir ? p->out_dir : "";
    R.out_name = p->out_name ? p->out_name : "";
    R.write = !R.out_dir.empty();
    R.L = p->L;
    for (int j = 0; j < R.L; ++j) {
        R.probs[j] = p->probs[j];
        R.vars[j] = p->vars[j] * (double)c->N;  // src/vamp.cpp:87-88
    }
    R.gam1 = p->gam1;
    R.gamw = 1.0 / (1.0 - p->h2);  // src/main_meth.cpp:52
    R.gam2 = 0;
    STCHK(vamp_alloc(c, R));
    STCHK(upload_or_zero(c, R.ts, p->true_signal, c->M));
    // P1 (src/vamp.cpp:70-79): x1_hat = r1 = x1hat_init / sqrt(N)
    R.hM.assign((size_t)std::max<int64_t>(c->M, 1), 0.0);
    for (int64_t i = 0; i < c->M; ++i) R.hM[i] = (p->x1hat_init ? p->x1hat_init[i] : 0.0) / std::sqrt((double)c->N);
    STCHK(upload_or_zero(c, R.x1, R.hM.data(), c->M));
    STCHK(upload_or_zero(c, R.r1, R.hM.data(), c->M));
    STCHK(upload_or_zero(c, R.x2, nullptr, c->M));
    // A^T y is the same every iteration (y is fixed, src/vamp.cpp:303): one pass
    {
        const double* u[1] = {c->y};
        double* o[1] = {R.atxy};
        STCHK(atx_dev(c, 1, u, o, 0, 0.0, 0.0, nullptr));
    }
    if (R.write) {
        R.p_metrics = R.out_dir + "/" + R.out_name + "_metrics.csv";
        R.p_params = R.out_dir + "/" + R.out_name + "_params.csv";
        R.p_prior = R.out_dir + "/" + R.out_name + "_prior.csv";
        if (c->rank == 0) {
            std::vector<std::string> prior_h{"iteration", "number of components"};
            for (int i = 0; i < R.L; ++i) prior_h.push_back("prob" + std::to_string(i));
            for (int i = 0; i < R.L; ++i) prior_h.push_back("var" + std::to_string(i));
            bool ok = vio::csv_create_with_header(
                          R.p_metrics, {"iteration", "R2 denoising", "x1 correlation denoising", "R2 LMMSE",
                                        "x2 correlation LMMSE", "z1 correlation denoising", "z2 correlation LMMSE"}) &&
                      vio::csv_create_with_header(R.p_params, {"iteration", "alpha1", "gam1", "alpha2", "gam2", "gamw"}) &&
                      vio::csv_create_with_header(R.p_prior, prior_h);
            if (!ok) return fail(VAMPOMI_ERR_IO, "cannot create output CSV files in " + R.out_dir);
        }
    }
    if (r) {
        r->iterations_run = 0;
        r->a_passes_ref = 0;
        r->a_passes_exec = 0;
    }
    R.passes_ref = 0;
    HIPCHK(hipStreamSynchronize(c->st));
    return VAMPOMI_OK;
}

static vampomi_status write_bins(vampomi_ctx* c, VampRun& R) {
    const bool hist = R.res && (R.res->x1_hist || R.res->r1_hist);
    if (!R.write && !hist) return VAMPOMI_OK;
    const int64_t M = c->M;
    std::vector<double> hx((size_t)std::max<int64_t>(M, 1)), hr((size_t)std::max<int64_t>(M, 1));
    HIPCHK(hipMemcpyAsync(hx.data(), R.x1, (size_t)M * 8, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipMemcpyAsync(hr.data(), R.r1, (size_t)M * 8, hipMemcpyDeviceToHost, c->st));
    STCHK(host_sync(c));
    const double sqrtN = std::sqrt((double)c->N);
    for (int64_t i = 0; i < M; ++i) {
        hx[i] = hx[i] / sqrtN;  // x1_hat_scaled (src/vamp.cpp:237-238)
        hr[i] = hr[i] / sqrtN;  // r1_scaled (:246-248)
    }
    if (R.res && R.res->x1_hist) std::memcpy(R.res->x1_hist + (int64_t)(R.it - 1) * M, hx.data(), (size_t)M * 8);
    if (R.res && R.res->r1_hist) std::memcpy(R.res->r1_hist + (int64_t)(R.it - 1) * M, hr.data(), (size_t)M * 8);
    if (R.write) {
        const std::string base = R.out_dir + "/" + R.out_name;
        if (!vio::store_vec(base + "_it_" + std::to_string(R.it) + ".bin", hx.data(), c->S, M) ||
            !vio::store_vec(base + "_r1_it_" + std::to_string(R.it) + ".bin", hr.data(), c->S, M))
            return fail(VAMPOMI_ERR_IO, "cannot write iteration vectors to " + R.out_dir);
    }
    return VAMPOMI_OK;
}

// one VAMP iteration (src/vamp.cpp:148-428)
extern "C" vampomi_status vampomi_vamp_step(vampomi_ctx* c, int* stopped) {
    if (!c || !c->run) return fail(VAMPOMI_ERR_STATE, "vampomi_vamp_begin not called");
    VampRun& R = *c->run;
    if (R.stopped || R.it >= R.prm.max_iter) {
        R.stopped = true;
        if (stopped) *stopped = 1;
        return VAMPOMI_OK;
    }
    const int64_t M = c->M, N = c->N, Mt = c->Mt;
    const int it = ++R.it;
    vampomi_result* res = R.res;

    // ---------------- denoising ----------------
    if (it > R.prm.learn_prior_delay) STCHK(update_prior(c, R));  // :186-187
    if (res && res->L_hist) res->L_hist[it - 1] = R.L;
    std::swap(R.x1, R.x1p);  // x1_hat_prev = x1_hat (:203)
    {
        vk::Mix mix{};
        mix.L = R.L;
        for (int j = 0; j < R.L; ++j) {
            mix.probs[j] = R.probs[j];
            mix.vars[j] = R.vars[j];
        }
        int nb = 0;
        HIPCHK(vk::denoise(M, R.r1, R.gam1, mix, R.x1, R.x1p, it > 1 ? 1 : 0, R.prm.rho, R.x1d, c->red_part, &nb, c->st));
        HIPCHK(vk::sum_partials(c->red_part, nb, 1, c->scal + SL_DOTS, c->st));
        STCHK(allreduce_dev(c, c->scal + SL_DOTS, 1));  // :222
        HIPCHK(hipMemcpyAsync(c->h_scal + SL_DOTS, c->scal + SL_DOTS, 8, hipMemcpyDeviceToHost, c->st));
        STCHK(host_sync(c));
        R.alpha1 = c->h_scal[SL_DOTS] / (double)Mt;  // :223
    }
    R.eta1 = R.gam1 / R.alpha1;  // :230
    {
        const double* xs[1] = {R.x1};
        STCHK(ax_dev(c, 1, xs, R.z1));  // z1 = Ax(x1_hat) (:232)
        R.passes_ref += 1;
    }
    STCHK(write_bins(c, R));  // :235-249
    R.gam2 = smin(smax(R.eta1 - R.gam1, 1e-11), 1e11);  // :255-256
    HIPCHK(vk::lincomb_div(M, R.eta1, R.x1, R.gam1, R.r1, R.gam2, R.r2, c->st));  // r2 (:259-261)
    STCHK(err_measures(c, R, R.x1, R.z1, 1));  // :272
    R.params[0] = R.alpha1;
    R.params[1] = R.gam1;

    // ---------------- LMMSE ----------------
    HIPCHK(vk::bernoulli(R.prm.seed, it, c->S, M, std::sqrt((double)Mt), R.bern, c->st));  // :295-296 (P2)
    HIPCHK(vk::axpby(M, R.gamw, R.atxy, R.gam2, R.r2, R.v, c->st));  // v = gamw ATx(y) + gam2 r2 (:303-306)
    R.passes_ref += 1;
    CgSystem sx{}, so{};
    sx.v = R.v;
    sx.mu = R.x2;  // mu_CG_last: warm start, updated in place (:308-311, :753-754)
    sx.mu0_nonzero = it > 1;
    sx.onsager = false;
    sx.r = R.cgw[0];
    sx.z = R.cgw[1];
    sx.p = R.cgw[2];
    sx.d = R.cgw[3];
    so.v = R.bern;
    so.mu = R.invQ;
    so.mu0_nonzero = false;  // g2d_onsager starts from zeros (:496, :664-669)
    so.onsager = true;
    so.r = R.cgw[4];
    so.z = R.cgw[5];
    so.p = R.cgw[6];
    so.d = R.cgw[7];
    if (it == 1) HIPCHK(hipMemsetAsync(R.x2, 0, (size_t)std::max<int64_t>(M, 1) * 8, c->st));
    HIPCHK(hipMemsetAsync(R.invQ, 0, (size_t)std::max<int64_t>(M, 1) * 8, c->st));
    const bool batch = R.prm.batch_rhs != 0;
    if (batch) {
        STCHK(pcg_run(c, {&sx, &so}, R.gamw, R.gam2, R.prm.CG_max_iter, R.prm.CG_err_tol, R.nsc, &R.passes_ref));
    } else {
        STCHK(pcg_run(c, {&sx}, R.gamw, R.gam2, R.prm.CG_max_iter, R.prm.CG_err_tol, R.nsc, &R.passes_ref));
        STCHK(pcg_run(c, {&so}, R.gamw, R.gam2, R.prm.CG_max_iter, R.prm.CG_err_tol, R.nsc, &R.passes_ref));
    }
    if (res && res->cg_iters) res->cg_iters[it - 1] = sx.iters;
    if (res && res->ons_iters) res->ons_iters[it - 1] = so.iters;
    {
        double a[1];
        STCHK(dots(c, {T(R.bern, R.invQ)}, M, true, a));
        R.alpha2 = R.gam2 * a[0];  // :498
    }
    R.eta2 = R.gam2 / R.alpha2;  // :341
    const double gam1_prev = R.gam1;
    R.gam1 = smin(smax(R.eta2 - R.gam2, 1e-11), 1e11);
    R.gam1 = R.prm.rho * R.gam1 + (1 - R.prm.rho) * gam1_prev;  // :346
    HIPCHK(vk::lincomb_div(M, R.eta2, R.x2, R.gam2, R.r2, R.gam1, R.r1, c->st));  // r1 (:348-350)

    // updateNoisePrec (:504-529): Ax(x2_hat) and Ax(invQ_bern_vec) share one pass
    {
        const double* xs[2] = {R.x2, R.invQ};
        STCHK(ax_dev(c, 2, xs, R.nb2));
        R.passes_ref += 2;
        double tn[1];
        STCHK(dots(c, {T(R.nb2, c->y, vk::DIFF2)}, N, false, tn));  // l2_norm2(temp, 0)
        const double* u[1] = {R.nb2 + c->ld};
        double* o[1] = {R.tmpM};
        STCHK(atx_dev(c, 1, u, o, 0, 0.0, 0.0, nullptr));
        R.passes_ref += 1;
        double tc[1];
        STCHK(dots(c, {T(R.bern, R.tmpM)}, M, true, tc));
        const double trace_corr = tc[0] * (double)Mt;
        if (R.prm.verbosity >= 1 && c->rank == 0)
            std::printf("l2_norm2(temp) / N = %g\ntrace_correction / N = %g\n", tn[0] / (double)N, trace_corr / (double)N);
        R.gamw = (double)N / (tn[0] + trace_corr);
    }
    STCHK(err_measures(c, R, R.x2, R.nb2, 2));  // :365 (Ax(x2_hat) of :826 == nb2)
    R.passes_ref += 1;
    R.params[2] = R.alpha2;
    R.params[3] = R.gam2;
    R.params[4] = R.gamw;
    if (res && res->params) std::memcpy(res->params + (int64_t)(it - 1) * 5, R.params, sizeof R.params);
    if (res && res->metrics) std::memcpy(res->metrics + (int64_t)(it - 1) * 6, R.metrics, sizeof R.metrics);
    if (R.write && c->rank == 0) {
        if (!vio::csv_write_row(R.p_params, it, R.params, 5) || !vio::csv_write_row(R.p_metrics, it, R.metrics, 6))
            return fail(VAMPOMI_ERR_IO, "cannot write CSV rows");
    }
    if (R.prm.verbosity >= 1 && c->rank == 0)
        std::printf("it %d: alpha1 %.6g gam1 %.6g alpha2 %.6g gam2 %.6g gamw %.6g L %d cg %d/%d\n", it, R.alpha1,
                    R.gam1, R.alpha2, R.gam2, R.gamw, R.L, sx.iters, so.iters);

    // stopping criteria (:409-423)
    double nm[2];
    STCHK(dots(c, {T(R.x1p, R.x1, vk::DIFF2), T(R.x1p, R.x1p)}, M, true, nm));
    const double NMSE = std::sqrt(nm[0] / nm[1]);
    if (res) {
        res->iterations_run = it;
        res->a_passes_ref = R.passes_ref;
        res->a_passes_exec = c->stats.a_passes_exec;
    }
    if ((it > 1 && NMSE < R.prm.stop_criteria_thr) || it >= R.prm.max_iter) R.stopped = true;
    if (c->timing) resolve_timing(c);
    if (stopped) *stopped = R.stopped ? 1 : 0;
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_vamp_end(vampomi_ctx* c) {
    if (!c || !c->run) return fail(VAMPOMI_ERR_STATE, "vampomi_vamp_begin not called");
    VampRun& R = *c->run;
    vampomi_result* res = R.res;
    if (res) {
        if (res->x1_final && c->M > 0) {
            HIPCHK(hipMemcpyAsync(res->x1_final, R.x1, (size_t)c->M * 8, hipMemcpyDeviceToHost, c->st));
            STCHK(host_sync(c));
            const double sqrtN = std::sqrt((double)c->N);
            for (int64_t i = 0; i < c->M; ++i) res->x1_final[i] = res->x1_final[i] / sqrtN;
        }
        res->L_final = R.L;
        for (int j = 0; j < R.L; ++j) {
            res->probs_final[j] = R.probs[j];
            res->vars_final[j] = R.vars[j] / (double)c->N;
        }
        res->a_passes_ref = R.passes_ref;
        res->a_passes_exec = c->stats.a_passes_exec;
    }
    if (c->timing) resolve_timing(c);
    c->run.reset();
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_infere(vampomi_ctx* c, const vampomi_params* p, vampomi_result* r) {
    STCHK(vampomi_vamp_begin(c, p, r));
    int stopped = 0;
    while (!stopped) {
        vampomi_status s = vampomi_vamp_step(c, &stopped);
        if (s != VAMPOMI_OK) {
            c->run.reset();
            return s;
        }
    }
    return vampomi_vamp_end(c);
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

extern "C" void vampomi_close(vampomi_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->st) (void)hipStreamSynchronize(c->st);
    c->run.reset();
    resolve_timing(c);
    for (auto e : c->ev_pool) (void)hipEventDestroy(e);
    for (double** p : {&c->X, &c->mave, &c->msig, &c->y, &c->ax_part, &c->red_part, &c->scal, &c->nbuf, &c->mbuf})
        dev_free(*p);
    if (c->h_scal) (void)hipHostFree(c->h_scal);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    if (c->st) (void)hipStreamDestroy(c->st);
    delete c;
}

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
    const int64_t Mx = std::max<int64_t>(c->M, 1);
    c->axp = vk::ax_plan(c->N, Mx);
    STCHK(dev_alloc(&c->mave, Mx));
    STCHK(dev_alloc(&c->msig, Mx));
    STCHK(dev_alloc(&c->y, c->ld));
    HIPCHK(hipMemsetAsync(c->y, 0, c->ld * 8, c->st));
    STCHK(dev_alloc(&c->ax_part, (size_t)c->axp.nchunks * vk::kMaxRhs * c->ld));
    c->red_cap = std::max<size_t>({(size_t)vk::kRedBlocks * 3 * vk::kMaxRhs,
                                   (size_t)((Mx + 255) / 256) * (1 + 2 * (vk::kMaxL - 1)),
                                   (size_t)(Mx / 8 + 1) * vk::kMaxRhs, (size_t)4096});  // ATx partials at G >= 2
    STCHK(dev_alloc(&c->red_part, c->red_cap));
    STCHK(dev_alloc(&c->scal, SL_TOTAL));
    HIPCHK(hipHostMalloc((void**)&c->h_scal, SL_TOTAL * sizeof(double), hipHostMallocDefault));
    STCHK(dev_alloc(&c->nbuf, (size_t)vk::kMaxRhs * c->ld));
    HIPCHK(hipMemsetAsync(c->nbuf, 0, (size_t)vk::kMaxRhs * c->ld * 8, c->st));
    STCHK(dev_alloc(&c->mbuf, (size_t)2 * vk::kMaxRhs * Mx));
    if (c->nranks > 1) {
        ncclUniqueId id;
        std::memcpy(&id, d->comm_id, sizeof id);
        NCCLCHK(ncclCommInitRank(&c->comm, c->nranks, id, c->rank));
    }
    HIPCHK(hipStreamSynchronize(c->st));
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
    HIPCHK(hipStreamSynchronize(c->st));
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_barrier(vampomi_ctx* c) {
    if (!c) return fail(VAMPOMI_ERR_ARG, "null context");
    if (c->nranks > 1) STCHK(allreduce_dev(c, c->scal + SL_TOTAL - 1, 1));
    HIPCHK(hipStreamSynchronize(c->st));
    return VAMPOMI_OK;
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
    HIPCHK(hipStreamSynchronize(c->st));
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

// read_methylation_data (src/data.cpp:116-153): this rank's M*N doubles at byte
// offset S*N*8, streamed through a pinned staging buffer (64-bit offsets).
extern "C" vampomi_status vampomi_load_meth_file(vampomi_ctx* c, const char* path) {
    if (!c || !path) return fail(VAMPOMI_ERR_ARG, "null argument");
    HIPCHK(hipSetDevice(c->device));
    int fd = ::open(path, O_RDONLY);
    if (fd < 0) return fail(VAMPOMI_ERR_IO, std::string("cannot open methylation file ") + path);
    STCHK(ensure_X(c));
    const size_t colb = (size_t)c->N * 8;
    const size_t chunk_cols = std::max<size_t>(1, ((size_t)64 << 20) / colb);
    double* pin[2] = {nullptr, nullptr};
    hipEvent_t done[2];
    for (int b = 0; b < 2; ++b) {
        if (hipHostMalloc((void**)&pin[b], chunk_cols * colb, hipHostMallocDefault) != hipSuccess) {
            ::close(fd);
            return fail(VAMPOMI_ERR_OOM, "pinned staging buffer");
        }
        (void)hipEventCreate(&done[b]);
    }
    vampomi_status st = VAMPOMI_OK;
    int64_t i0 = 0;
    int b = 0;
    bool used[2] = {false, false};
    while (i0 < c->M && st == VAMPOMI_OK) {
        const int64_t nc = std::min<int64_t>((int64_t)chunk_cols, c->M - i0);
        if (used[b]) (void)hipEventSynchronize(done[b]);
        const size_t want = (size_t)nc * colb;
        const off_t off = (off_t)(c->S + i0) * (off_t)colb;
        size_t got = 0;
        while (got < want) {
            ssize_t r = ::pread(fd, (char*)pin[b] + got, want - got, off + (off_t)got);
            if (r <= 0) break;
            got += (size_t)r;
        }
        if (got != want) {
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
        b ^= 1;
    }
    (void)hipStreamSynchronize(c->st);
    for (int k = 0; k < 2; ++k) {
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
    HIPCHK(hipStreamSynchronize(c->st));
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
    HIPCHK(hipStreamSynchronize(c->st));
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_read_markers(vampomi_ctx* c, int64_t i0, int64_t count, double* out) {
    if (!c || !out || i0 < 0 || count < 0 || i0 + count > c->M) return fail(VAMPOMI_ERR_ARG, "bad marker range");
    if (!c->have_X) return fail(VAMPOMI_ERR_STATE, "no methylation data loaded");
    HIPCHK(hipSetDevice(c->device));
    if (count > 0)
        HIPCHK(hipMemcpy2DAsync(out, (size_t)c->N * 8, c->X + i0 * c->ld, (size_t)c->ld * 8, (size_t)c->N * 8,
                                (size_t)count, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_simulate_phen(vampomi_ctx* c, uint64_t seed, double lam, double h2, double* beta_out) {
    if (!c || !c->have_X) return fail(VAMPOMI_ERR_STATE, "load methylation data first");
    HIPCHK(hipSetDevice(c->device));
    double* beta = c->mbuf;
    int nb = 0;
    const int64_t M = c->M;
    double cm = 0.0;
    if (M > 0) {
        HIPCHK(vk::gen_beta(seed, lam, c->S, M, beta, c->red_part, &nb, c->st));
        HIPCHK(vk::sum_partials(c->red_part, nb, 1, c->scal + SL_DOTS, c->st));
    } else {
        HIPCHK(hipMemsetAsync(c->scal + SL_DOTS, 0, 8, c->st));
    }
    STCHK(allreduce_dev(c, c->scal + SL_DOTS, 1));
    HIPCHK(hipMemcpyAsync(c->h_scal + SL_DOTS, c->scal + SL_DOTS, 8, hipMemcpyDeviceToHost, c->st));
    STCHK(host_sync(c));
    cm = c->h_scal[SL_DOTS];
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
    HIPCHK(hipStreamSynchronize(c->st));
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_ax(vampomi_ctx* c, const double* x, double* out, int mem) {
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

static vampomi_status is_zero_vec(vampomi_ctx* c, const double* v, int64_t n, int mem, bool* z) {
    if (mem == VAMPOMI_MEM_HOST) {
        *z = host_all_zero(v, n);
        return VAMPOMI_OK;
    }
    std::vector<double> h((size_t)std::max<int64_t>(n, 1));
    if (n > 0) HIPCHK(hipMemcpyAsync(h.data(), v, (size_t)n * 8, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    *z = host_all_zero(h.data(), n);
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_lmmse_mult(vampomi_ctx* c, const double* v, double tau, double gam2, double* out,
                                             int mem) {
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
    bool zero = true;
    if (mu0) STCHK(is_zero_vec(c, mu0, c->M, mem, &zero));
    s.mu0_nonzero = !zero;
    if (zero)
        HIPCHK(hipMemsetAsync(s.mu, 0, (size_t)Mx * 8, c->st));
    else
        STCHK(stage_in(c, mu0, c->M, mem, s.mu));
    STCHK(pcg_run(c, {&s}, tau, gam2, max_iter, tol, c->nbuf, nullptr));
    STCHK(stage_out(c, s.mu, c->M, mem, mu));
    if (iters) *iters = s.iters;
    if (c->timing) resolve_timing(c);
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_denoise(vampomi_ctx* c, const double* r1, double gam1, const double* probs,
                                          const double* vars, int L, double* x1, double* x1d, double* sum_d, int mem) {
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
    int nb = 0;
    HIPCHK(vk::denoise(c->M, rin, gam1, mix, xo, rin, 0, 1.0, xd, c->red_part, &nb, c->st));
    HIPCHK(vk::sum_partials(c->red_part, nb, 1, c->scal + SL_DOTS, c->st));
    STCHK(allreduce_dev(c, c->scal + SL_DOTS, 1));
    HIPCHK(hipMemcpyAsync(c->h_scal + SL_DOTS, c->scal + SL_DOTS, 8, hipMemcpyDeviceToHost, c->st));
    if (x1) STCHK(stage_out(c, xo, c->M, mem, x1));
    if (x1d) STCHK(stage_out(c, xd, c->M, mem, x1d));
    STCHK(host_sync(c));
    if (sum_d) *sum_d = c->h_scal[SL_DOTS];
    return VAMPOMI_OK;
}

// ---------------------------------------------------------------------------
// parameters / measurement
// ---------------------------------------------------------------------------
extern "C" void vampomi_params_default(vampomi_params* p) {
    // src/options.hpp:62-104 (code defaults, not the README table)
    std::memset(p, 0, sizeof *p);
    p->gam1 = 1e-6;
    p->h2 = 0.5;
    p->max_iter = 50;
    p->CG_max_iter = 500;
    p->CG_err_tol = 1e-5;
    p->EM_max_iter = 1;
    p->EM_err_thr = 1e-2;
    p->rho = 0.5;
    p->learn_vars = 1;
    p->learn_prior_delay = 1;
    p->stop_criteria_thr = 0.01;
    p->merge_vars_thr = 5e-1;
    static const double v[10] = {0, 1e-06, 6e-06, 3e-05, 2e-04, 1e-03, 6e-03, 3e-02, 2e-01, 1e+00};
    static const double q[10] = {9.90000e-01, 5.00000e-03, 2.50000e-03, 1.25000e-03, 6.25000e-04,
                                 3.12500e-04, 1.56250e-04, 7.81250e-05, 3.90625e-05, 3.90625e-05};
    p->L = 10;
    for (int j = 0; j < 10; ++j) {
        p->vars[j] = v[j];
        p->probs[j] = q[j];
    }
    p->seed = 0x5EED5EEDULL;
    p->batch_rhs = 1;
    p->model = "linear";
}

extern "C" vampomi_status vampomi_set_timing(vampomi_ctx* c, int on) {
    if (!c) return fail(VAMPOMI_ERR_ARG, "null context");
    c->timing = on != 0;
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_get_stats(vampomi_ctx* c, vampomi_stats* out) {
    if (!c || !out) return fail(VAMPOMI_ERR_ARG, "null argument");
    HIPCHK(hipStreamSynchronize(c->st));
    resolve_timing(c);
    *out = c->stats;
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_reset_stats(vampomi_ctx* c) {
    if (!c) return fail(VAMPOMI_ERR_ARG, "null context");
    HIPCHK(hipStreamSynchronize(c->st));
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
    HIPCHK(hipStreamSynchronize(c->st));
    if (which == 0) {
        if (!vk::set_ax_variant(variant)) return fail(VAMPOMI_ERR_ARG, "no such A.x variant");
        const vk::AxPlan np = vk::ax_plan(c->N, std::max<int64_t>(c->M, 1));
        if (np.nchunks > c->axp.nchunks) {
            dev_free(c->ax_part);
            STCHK(dev_alloc(&c->ax_part, (size_t)np.nchunks * vk::kMaxRhs * c->ld));
        }
        c->axp = np;
    } else {
        if (!vk::set_atx_variant(variant)) return fail(VAMPOMI_ERR_ARG, "no such A^T.u variant");
    }
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_dev_time_pass(vampomi_ctx* c, int which, int K, int reps, double* avg_ms) {
    if (!c || !avg_ms || K < 1 || K > (which == 0 ? 4 : 3) || reps < 1) return fail(VAMPOMI_ERR_ARG, "bad argument");
    if (!c->have_X) return fail(VAMPOMI_ERR_STATE, "no methylation data loaded");
    HIPCHK(hipSetDevice(c->device));
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
        else
            HIPCHK(vk::atx(c->shard(), K, in, out, 1.0 / c->sqrtN, 0, 0.0, 0.0, vk::CPtrs{}, c->red_part, c->st));
    }
    HIPCHK(hipEventRecord(b, c->st));
    HIPCHK(hipEventSynchronize(b));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    *avg_ms = (double)ms / reps;
    return VAMPOMI_OK;
}
