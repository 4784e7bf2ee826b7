/*
 * vampomi.h — C ABI of the MI355X-native gVAMPomi VAMP engine.
 *
 * Plain C, plain pointers and sizes.  One context per process, driving one
 * gfx950 device and one contiguous marker shard [S, S+M) of the Mt markers
 * (the reference's MPI rank, src/utilities.cpp:207-239).  Contexts of a job
 * are joined by an RCCL communicator over xGMI; every entry point marked
 * COLLECTIVE must be called by all ranks in the same order, exactly like the
 * reference's MPI_Allreduce-bearing calls.
 *
 * Reference seams replaced (paths relative to the reference repository):
 *   data::data / read_methylation_data / compute_markers_statistics
 *        src/data.cpp:24-53, 116-153, 233-283 -> vampomi_open + vampomi_load_meth_*
 *   data::read_phen            src/data.cpp:58-110      -> vampomi_read_phen / vampomi_set_phen
 *   data::Ax                   src/data.cpp:340-373     -> vampomi_ax      (COLLECTIVE)
 *   data::ATx / dot_product    src/data.cpp:294-333     -> vampomi_atx
 *   data::get_mave/get_msig    src/data.hpp:56-57       -> vampomi_get_marker_stats
 *   data::get_phen             src/data.hpp:48          -> vampomi_get_phen
 *   vamp::lmmse_mult           src/vamp.cpp:645-662     -> vampomi_lmmse_mult (COLLECTIVE)
 *   vamp::precondCG_solver     src/vamp.cpp:664-757     -> vampomi_pcg      (COLLECTIVE)
 *   vamp::g1 / vamp::g1d       src/vamp.cpp:440-492     -> vampomi_denoise  (COLLECTIVE: alpha1 sum)
 *   vamp::updatePrior          src/vamp.cpp:531-643     -> vampomi_update_prior (COLLECTIVE)
 *   vamp::g1_bin_class / g1d_bin_class
 *        src/vamp_probit.cpp:469-488                    -> vampomi_denoise_bin
 *   vamp::vamp + vamp::infere / infere_linear / infere_bin_class
 *        src/vamp.cpp:18-91, 94-107, 110-438,
 *        src/vamp_probit.cpp:19-488                     -> vampomi_infere   (COLLECTIVE)
 *        (or vampomi_vamp_begin / _step / _end, one VAMP iteration per step)
 *   divide_work                src/utilities.cpp:207-239 -> vampomi_divide_work
 *   run mode test              src/main_meth.cpp:112-205 -> vampomi_test_metrics (COLLECTIVE)
 *   association_test loo / se  src/main_meth.cpp:206-264, src/data.cpp:385-417,
 *                              src/utilities.cpp:269-282 -> vampomi_assoc_loo / _se
 *
 * Testing aid: with VAMPOMI_COMM=loopback in the environment, the contexts
 * of a multi-rank job are driven by threads of ONE process (any device, the
 * same one allowed) and all-reduces become an in-process rendezvous that sums
 * in rank order; comm_id is then any 128 bytes shared by the ranks.
 *
 * Errors: every call returns a vampomi_status; nothing aborts the process
 * (the reference calls MPI_Abort / exit / throw).  vampomi_last_error() gives
 * a message for the calling thread.
 */
#ifndef VAMPOMI_H
#define VAMPOMI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VAMPOMI_ABI_VERSION 3
#define VAMPOMI_MAX_L 64          /* mixture components */
#define VAMPOMI_UNIQUE_ID_BYTES 128

typedef enum {
    VAMPOMI_OK = 0,
    VAMPOMI_ERR_ARG = 1,          /* bad argument / shape */
    VAMPOMI_ERR_HIP = 2,          /* HIP runtime failure */
    VAMPOMI_ERR_RCCL = 3,         /* RCCL failure */
    VAMPOMI_ERR_IO = 4,           /* file could not be opened / read / written */
    VAMPOMI_ERR_NAN_PHEN = 5,     /* "NA" in phenotype file (src/data.cpp:73-74) */
    VAMPOMI_ERR_STATE = 6,        /* call out of order (e.g. Ax before data load) */
    VAMPOMI_ERR_OOM = 7,          /* device or host allocation failed */
    VAMPOMI_ERR_MODEL = 8         /* unsupported --model (src/vamp.cpp:103-104) */
} vampomi_status;

/* where a caller buffer lives */
#define VAMPOMI_MEM_HOST 0
#define VAMPOMI_MEM_DEVICE 1

/* synthetic design kinds for vampomi_generate_meth */
#define VAMPOMI_GEN_GAUSS 0       /* i.i.d. N(0,1)-like (simulation/data_sim.py:35) */
#define VAMPOMI_GEN_METH 1        /* methylation-like beta values in [0,1] */

typedef struct vampomi_ctx vampomi_ctx;

typedef struct {
    int64_t N;                    /* individuals (--N) */
    int64_t Mt;                   /* total markers (--Mt) */
    int rank, nranks;             /* this process's shard */
    int device;                   /* HIP device ordinal; -1: rank % visible devices */
    const void* comm_id;          /* VAMPOMI_UNIQUE_ID_BYTES from vampomi_comm_unique_id
                                     on rank 0, broadcast by the caller; NULL if nranks==1 */
    double alpha_scale;           /* --alpha-scale (src/data.cpp:261-264) */
} vampomi_shard_desc;

/* ---- job / context ---- */
int vampomi_abi_version(void);
const char* vampomi_last_error(void);
/* src/utilities.cpp:207-239 */
void vampomi_divide_work(int64_t Mt, int nranks, int rank, int64_t* M, int64_t* S, int64_t* Mm);
vampomi_status vampomi_comm_unique_id(void* out /* VAMPOMI_UNIQUE_ID_BYTES */);
vampomi_status vampomi_open(const vampomi_shard_desc* desc, vampomi_ctx** out);
void vampomi_close(vampomi_ctx* ctx);
/* M (local markers), S (first global marker), ld (device leading dimension) */
vampomi_status vampomi_shard_info(const vampomi_ctx* ctx, int64_t* M, int64_t* S, int64_t* ld);
vampomi_status vampomi_sync(vampomi_ctx* ctx);          /* drain the context's stream */
vampomi_status vampomi_barrier(vampomi_ctx* ctx);       /* COLLECTIVE: RCCL barrier + drain */
/* COLLECTIVE: vampomi_barrier with its own wait limit instead of
 * VAMPOMI_COLL_TIMEOUT_S: the barrier after a rank-local phase of uneven
 * length, e.g. the shard load, where the ranks' files come off storage at
 * different rates (there is no MPI_Barrier in the reference's data::data,
 * src/data.cpp:23-46; its first collective simply waits). */
vampomi_status vampomi_barrier_timeout(vampomi_ctx* ctx, double seconds);
/* COLLECTIVE: *all_ok = 1 iff local_ok != 0 on every rank.  How ranks agree on
   a rank-local outcome (a file read) before the next collective; the
   reference's rank-local exits (exit(1), throw) leave the other MPI ranks
   blocked in MPI_Allreduce instead. */
vampomi_status vampomi_all_ok(vampomi_ctx* ctx, int local_ok, int* all_ok);
/* After a rank-local failure: poisons the test-only loopback communicator
   (every rank's pending and later collectives fail at once) or aborts the RCCL
   communicator, so no rank waits for this one.  Every COLLECTIVE entry point
   does this itself when it fails. */
vampomi_status vampomi_comm_abort(vampomi_ctx* ctx);

/* ---- data ingest (data::data) ---- */
/* marker-major fp64 file (README.md:15): this shard's bytes [S*N*8, (S+M)*N*8) */
vampomi_status vampomi_load_meth_file(vampomi_ctx* ctx, const char* path);
/* host shard: M columns of N samples, column stride ld_in >= N doubles */
vampomi_status vampomi_load_meth_host(vampomi_ctx* ctx, const double* X, int64_t ld_in);
/* synthetic shard generated on the device (bit-identical to the oracle's) */
vampomi_status vampomi_generate_meth(vampomi_ctx* ctx, uint64_t seed, int kind);
/* PLINK phenotype, standardize = scale to unit variance, NOT centred */
vampomi_status vampomi_read_phen(vampomi_ctx* ctx, const char* path, int standardize);
vampomi_status vampomi_set_phen(vampomi_ctx* ctx, const double* y /* N, host */, int standardize);
vampomi_status vampomi_get_phen(vampomi_ctx* ctx, double* y /* N, host */);
/* synthetic phenotype y = sqrt(N)*A*beta + N(0,1-h2) noise, beta spike-and-slab
 * (lam causal fraction, h2 heritability), then read_phen scaling.  beta_out
 * (M local, host, may be NULL) receives beta = the true signal. COLLECTIVE */
vampomi_status vampomi_simulate_phen(vampomi_ctx* ctx, uint64_t seed, double lam, double h2,
                                     double* beta_out);
/* binary phenotype for the probit model: the liability of vampomi_simulate_phen
 * thresholded at 0 (y = 1 if > 0 else 0), stored raw (read_phen(false),
 * src/data.cpp:40-41). COLLECTIVE */
vampomi_status vampomi_simulate_phen_binary(vampomi_ctx* ctx, uint64_t seed, double lam, double h2,
                                            double* beta_out);
vampomi_status vampomi_get_marker_stats(vampomi_ctx* ctx, double* mave, double* msig);
/* copy local markers [i0, i0+count) back to the host, count x N doubles
 * (data::get_meth_data, src/data.hpp:53) */
vampomi_status vampomi_read_markers(vampomi_ctx* ctx, int64_t i0, int64_t count, double* out);

/* ---- operators ---- */
/* out (N) = (sum over all ranks of (X_i - mave_i) * msig_i * x_i) / sqrt(N). COLLECTIVE */
vampomi_status vampomi_ax(vampomi_ctx* ctx, const double* x /* M */, double* out /* N */, int mem);
/* out (M) = msig_i * sum_j (X_ij - mave_i) * u_j * (1/sqrt(N)) */
vampomi_status vampomi_atx(vampomi_ctx* ctx, const double* u /* N */, double* out /* M */, int mem);
/* out = tau * ATx(Ax(v)) + gam2 * v, zero v short-circuits. COLLECTIVE */
vampomi_status vampomi_lmmse_mult(vampomi_ctx* ctx, const double* v, double tau, double gam2,
                                  double* out, int mem);
/* preconditioned CG on (tau*A^T A + gam2*I) mu = v from mu0 (NULL = zeros);
 * onsager != 0 adds the Onsager stop of src/vamp.cpp:708-726. COLLECTIVE */
vampomi_status vampomi_pcg(vampomi_ctx* ctx, const double* v, const double* mu0, double tau,
                           double gam2, int onsager, int max_iter, double tol, double* mu,
                           int* iters, int mem);
/* x1 = g1(r1), x1d = g1d(r1) for the mixture (probs, vars) with vars ALREADY
 * multiplied by N (src/vamp.cpp:87-88); *sum_d = sum over all ranks of x1d.
 * COLLECTIVE */
vampomi_status vampomi_denoise(vampomi_ctx* ctx, const double* r1, double gam1, const double* probs,
                               const double* vars, int L, double* x1, double* x1d, double* sum_d,
                               int mem);

/* vamp::updatePrior (src/vamp.cpp:531-643): EM_max_iter EM passes over r1 (this
 * shard's M values) at noise precision gam1 for the mixture (*L, probs, vars;
 * vars ALREADY multiplied by N), then the merging of variances closer than
 * merge_vars_thr; the mixture is updated in place (*L may shrink). COLLECTIVE */
vampomi_status vampomi_update_prior(vampomi_ctx* ctx, const double* r1, double gam1, int* L, double* probs,
                                    double* vars, int EM_max_iter, double EM_err_thr, int learn_vars,
                                    double merge_vars_thr, int mem);

/* probit z-denoiser: z1[i] = g1_bin_class(p1[i], tau1, y[i]) with the context's
 * phenotype y (raw 0/1), *sum_d = sum_i g1d_bin_class(p1[i], tau1, y[i]) (local:
 * the N-side is replicated on every rank).  probit_var = 1, no covariates.
 * src/vamp_probit.cpp:213-233, 469-488; erfcx src/utilities.cpp:293-363 */
vampomi_status vampomi_denoise_bin(vampomi_ctx* ctx, const double* p1, double tau1, double* z1,
                                   double* sum_d, int mem);

/* ---- the VAMP linear and probit models (vamp::infere) ---- */
typedef struct {
    double gam1, h2;              /* --gam1, --h2 (gamw = 1/(1-h2), src/main_meth.cpp:52) */
    int max_iter, CG_max_iter;    /* --iterations, --CG-max-iter */
    double CG_err_tol;            /* --CG-err-tol */
    int EM_max_iter;              /* --EM-max-iter */
    double EM_err_thr, rho;       /* --EM-err-thr, --rho */
    int learn_vars, learn_prior_delay;
    double stop_criteria_thr, merge_vars_thr;
    int L;                        /* number of mixture components */
    double vars[VAMPOMI_MAX_L];   /* as on the command line (NOT multiplied by N) */
    double probs[VAMPOMI_MAX_L];
    uint64_t seed;                /* index-keyed Bernoulli probe seed */
    const char* out_dir;          /* NULL or "" => write no files */
    const char* out_name;
    int verbosity;
    const double* true_signal;    /* local slice (M) or NULL => zeros (host) */
    const double* x1hat_init;     /* local slice (M) or NULL => zeros (host) */
    int batch_rhs;                /* 4 (default): 3, and each CG step reads X ONCE: A^T q
                                     and A d from the same pass, with q = A p and A r
                                     carried as N-vector recurrences (one A.x pass per
                                     solve for A r0; equal up to rounding);
                                     3: 2, plus A x2 carried through the CG steps
                                     and z1 = A x1 in the first CG pass (no pass over X
                                     outside the CG; equal up to rounding); 2: 1, plus the
                                     linear model's updateNoisePrec products A^T A x2 /
                                     A^T A invQ carried through the CG steps (one pass over
                                     X fewer per iteration; equal up to rounding);
                                     1: share each A/A^T pass between the x2
                                     and Onsager CG solves (every value bitwise that of 0);
                                     0: run them back to back */
    const char* model;            /* "linear" (NULL == "linear") or "bin_class" (probit,
                                     src/vamp_probit.cpp; phenotype must be raw 0/1, i.e. read
                                     with standardize = 0; h2/gamw unused; seed also keys the
                                     Gaussian start p1) */
} vampomi_params;

typedef struct {
    int iterations_run;
    /* per-iteration arrays, caller allocated (max_iter entries; may be NULL) */
    int* cg_iters;                /* k1 */
    int* ons_iters;               /* k2 */
    int* L_hist;                  /* mixture components after updatePrior */
    double* params;               /* per iteration, 5 (linear): alpha1 gam1 alpha2 gam2 gamw;
                                     8 (bin_class): alpha1 beta1 gam1 tau1 alpha2 beta2 gam2 tau2 */
    double* metrics;              /* per iteration, 6 (linear); 12 (bin_class): TP TN FP FN
                                     acc1 x1_corr TP TN FP FN acc2 x2_corr */
    double* x1_hist;              /* M per iteration: x1_hat/sqrt(N) (== _it_K.bin slice) */
    double* r1_hist;              /* M per iteration: r1/sqrt(N)     (== _r1_it_K.bin slice) */
    double* x1_final;             /* M: what vamp::infere returns: x1_hat_scaled for linear
                                     (src/vamp.cpp:437), x1_hat for bin_class (vamp_probit.cpp:465) */
    double probs_final[VAMPOMI_MAX_L];
    double vars_final[VAMPOMI_MAX_L];   /* divided by N, as printed/written */
    int L_final;
    int64_t a_passes_ref;         /* A/A^T passes the reference would have run */
    int64_t a_passes_exec;        /* passes actually executed (X streamed from HBM) */
    double* prior_hist;           /* bin_class: (1 + 2*VAMPOMI_MAX_L) per iteration: the
                                     _prior.csv row L, probs[L], vars[L] (vars x N), zero padded */
} vampomi_result;

void vampomi_params_default(vampomi_params* p);   /* src/options.hpp:62-104 defaults */
vampomi_status vampomi_infere(vampomi_ctx* ctx, const vampomi_params* p, vampomi_result* r);
/* step-wise form of vampomi_infere: begin, then one VAMP iteration per step
 * (*stopped = 1 once the stopping rule fired or max_iter was reached), end. */
vampomi_status vampomi_vamp_begin(vampomi_ctx* ctx, const vampomi_params* p, vampomi_result* r);
vampomi_status vampomi_vamp_step(vampomi_ctx* ctx, int* stopped);
vampomi_status vampomi_vamp_end(vampomi_ctx* ctx);
/* the last step's phase times as the host sees them (rank-local wall clock),
 * replacing the reference's per-iteration stopwatches "CG took" / "onsager
 * took" (src/vamp.cpp:313-316, :326-333; one interval here: both solves share
 * every pass) and "Total iteration time" (:396-401): *solve_s from the start
 * of the step's CG solves to their stop (the linear model queues their start
 * at the end of the previous step, so the device begins a little earlier),
 * *step_s the whole vampomi_vamp_step.  Either pointer may be NULL. */
vampomi_status vampomi_step_phases(vampomi_ctx* ctx, double* solve_s, double* step_s);

/* ---- association tests (--run-mode association_test) ----
 * loo: src/main_meth.cpp:245-264 + data::pvals_loo src/data.cpp:385-417.
 * est = this shard's slice of the estimate file as stored (x1_hat/sqrt(N));
 * the engine multiplies by sqrt(N), forms y_mod = y - Ax(x1_hat) (COLLECTIVE),
 * then per marker the five sums over y_mark = y_mod + X_j/sqrt(N)*x1_hat_j with
 * the RAW marker values, and linear_reg1d_pvals (src/utilities.cpp:269-282;
 * Student-t tail restated, Boost absent).  stats (5*M: sumx sumsqx sumxy sumy
 * sumsqy per marker) may be NULL.
 * se: src/main_meth.cpp:218-242, p_j = P(N(r1_j, 1/(gam1 N)) <= 0), 1 - p_j when
 * r1_j <= 0; rank-local. */
vampomi_status vampomi_assoc_loo(vampomi_ctx* ctx, const double* est, double* pvals, double* stats,
                                 int mem);
vampomi_status vampomi_assoc_se(vampomi_ctx* ctx, const double* r1, double gam1, double* pvals, int mem);

/* ---- --run-mode test (src/main_meth.cpp:112-205) ----
 * On a context holding the TEST data set (N = N_test, its own marker
 * statistics, phenotype read like the training one): x = est*sqrt(N_test),
 * z = A x (COLLECTIVE); *r2 = 1 - |y - z|^2 / (calc_stdev(y)^2 * N_test),
 * *corr2 = (<z,y> / sqrt(|z|^2 |y|^2))^2 — one row of _test.csv. */
vampomi_status vampomi_test_metrics(vampomi_ctx* ctx, const double* est, double* r2, double* corr2, int mem);

/* ---- measurement ---- */
typedef struct {
    int64_t launches;             /* kernel launches of this class that did work (exact) */
    double ms_total;              /* their device time: ms_timed / timed x launches (per K; a
                                     class's is the sum over its K) */
    double bytes_total;           /* algorithmic HBM bytes of those launches */
    double flops_total;
    int64_t timed;                /* launches timed with HIP events (vampomi_set_timing) */
    double ms_timed;              /* device time of the timed launches */
} vampomi_kernel_stat;

typedef struct {
    vampomi_kernel_stat ax;       /* A.x partial-sum kernels (all batch widths) */
    vampomi_kernel_stat atx;      /* A^T.u kernels */
    vampomi_kernel_stat ax_k[4];  /* per batch width K = 1..4 (index K-1) */
    vampomi_kernel_stat atx_k[4];
    int64_t a_passes_exec;
    int64_t host_syncs;
    vampomi_kernel_stat loo;      /* association-test pass (vampomi_assoc_loo) */
    vampomi_kernel_stat op;       /* one-pass CG operator (A^T q and A d, batch_rhs 4) */
    vampomi_kernel_stat op_k[4];  /* index K-1 for K = 1, 2 systems; index 3: the head-start launch
                                     (one system + 3 plain A.x right-hand sides, pcg.cpp) */
    vampomi_kernel_stat coll;     /* RCCL all-reduces (several ranks): launches, bytes; with timing
                                     on, HIP events on the stream around each (its time on the
                                     stream, waits for the slowest rank included) */
} vampomi_stats;

/* HIP-event timing of the A/A^T kernels: on = 0 off, 1 every launch, n > 1 one
 * launch in n of each (kernel class, K) (each timed launch carries an event
 * pair in its dispatch, a few microseconds; the first launch of each (class, K)
 * after a reset is always timed).  Launch counts and bytes in the stats are
 * always exact; ms_total extrapolates the timed average to them. */
vampomi_status vampomi_set_timing(vampomi_ctx* ctx, int on);
vampomi_status vampomi_get_stats(vampomi_ctx* ctx, vampomi_stats* out);
vampomi_status vampomi_reset_stats(vampomi_ctx* ctx);

/* ---- development hooks (kernel tuning; not part of the reference interface) ----
 * which: 0 = A.x partial-sum kernel, 1 = A^T.u kernel, 2 = association-test pass
 * (K = 1), 3 = one-pass CG operator (K = 1, 2).  Variants index the
 * tuning tables in vampomi_amd/csrc/kernels.hip and are settings of this
 * context only; the defaults are 0 (A.x), -1 (A^T.u: the per-K choice), 16
 * (association pass: loo_wg_kernel<4,2,8>; variants 8-19 are the kernels whose
 * workgroups share their markers, and they add the sums in another order than
 * the wave-per-marker variants 0-7, so results differ at rounding level) and
 * -1 (operator: whole columns per workgroup while
 * K*N fits the LDS, else teams of workgroups; 0 forces the whole-column
 * kernel, T*10 + c (c < 10) or 1000 + T*100 + c the team kernel with team size T and configuration c,
 * vampomi_amd/csrc/atax_team.hip).  which = 4 (the side stream of rounds
 * 2-5) was removed: VAMPOMI_ERR_ARG.
 * which = 5: the CG head start of the linear model (the Onsager solve's first
 * step in the pass that starts the x2 solve, pcg.cpp), 0 off, 1 on (default
 * on; VAMPOMI_HEADSTART=0 turns it off at vampomi_open).  which = 6: the
 * linear iteration's tail without host waits on several ranks, 0 off, 1 on
 * (default on; VAMPOMI_MR_TAIL=0 turns it off at vampomi_open).  On a context
 * with several ranks, which = 3, 5 and 6 take effect at the next
 * vampomi_vamp_begin (or vampomi_infere), where the ranks agree on them: the
 * one-pass operator runs only if every rank has a plan for it, the head start
 * and the host-free tail only if every rank has them on (each changes the
 * job's collective sequence). */
vampomi_status vampomi_dev_set_variant(vampomi_ctx* ctx, int which, int variant);
/* average device time (HIP events) of `reps` back-to-back launches, K RHS */
vampomi_status vampomi_dev_time_pass(vampomi_ctx* ctx, int which, int K, int reps, double* avg_ms);
/* The HBM read ceiling of this device for this shard: a pure read stream of
 * the resident matrix (every byte once, 16-byte nontemporal loads; variant 0
 * lockstep 8-wave workgroups, one per CU, variant 1 a 1 MiB contiguous chunk
 * per wave), `reps` timed launches of each; the faster variant's median launch
 * time in *us_med, the bytes it read in *bytes, the variant in *variant.  No
 * effect on the run's state or statistics. */
vampomi_status vampomi_dev_read_ceiling(vampomi_ctx* ctx, int reps, double* us_med, double* bytes, int* variant);
/* the kernel (as rocprofv3 names it) that pass `which` with K RHS launches now
 * (mode 1: the CG form, i.e. A^T.u with the lmmse_mult epilogue, A.x with the
 * fused direction update; which = 2: the association-test pass of
 * vampomi_assoc_loo) */
vampomi_status vampomi_dev_kernel_name(const vampomi_ctx* ctx, int which, int K, int mode, char* out, int cap);
/* The A.x plan for N samples, M markers and `cus` compute units under
 * `variant` (-1 the default, 0-6 the tile plans, 7 the team plan), no device
 * needed: team size T (0: a tile plan), rows per member TR, loads per lane S,
 * workgroups grid, partial slots nslots, and the kernel name for K
 * right-hand sides. */
vampomi_status vampomi_dev_ax_plan(int64_t N, int64_t M, int cus, int variant, int K, int* T, int* TR, int* S,
                                   int* grid, int* nslots, char* name, int cap);
/* The one-pass operator's plan for N samples, M markers and `cus` compute
 * units under `variant` (as vampomi_dev_set_variant(ctx, 3, variant)), no
 * device needed: team size T (0: the whole-column kernel), loads per lane per
 * column S, rows per team member TR, workgroups grid, partial-sum slots
 * nslots, and the kernel name for K right-hand sides.  VAMPOMI_ERR_ARG if
 * no such plan exists. */
vampomi_status vampomi_dev_op_plan(int64_t N, int64_t M, int cus, int variant, int K, int* T, int* S, int* TR,
                                   int* grid, int64_t* nslots, char* name, int cap);
/* The dynamic LDS layout (in doubles) a team-plan operator launch with K
 * systems uses for that plan, no device needed: out[0] head words (the folded
 * CG decision), [1] q offset, [2] q stride, [3] wave partials offset, [4]
 * hand-off totals offset, [5] total words.  The kernel's pointers, the plan's
 * feasibility check and the launch size all come from this one layout.
 * VAMPOMI_ERR_ARG if there is no such team plan (or it is the whole-column
 * kernel's). */
vampomi_status vampomi_dev_op_lds(int64_t N, int64_t M, int cus, int variant, int K, int64_t* out);
/* Experiment builds only (atax_team.hip compiled with TM_TS=1, and
 * VAMPOMI_OP_TS=1 set before the context's first operator use): the last
 * operator launch's per-workgroup {start, end, XCC id, HW_ID} (s_memrealtime
 * ticks, 100 MHz), *n = min(cap, 4 x grid) words. VAMPOMI_ERR_STATE otherwise. */
vampomi_status vampomi_dev_op_timestamps(vampomi_ctx* ctx, unsigned long long* out, int cap, int* n);
/* Device bytes the context of `rank` (of nranks, markers split by
 * vampomi_divide_work) allocates for a VAMP run on N samples and Mt markers
 * with `cus` compute units: the shard, marker statistics, scratch, the
 * one-pass operator's buffers and the run state (probit != 0: the probit
 * model's too); the per-iteration output writer stages in pinned host memory
 * (`writer` is kept for the ABI and ignored).  No device needed; RCCL's
 * buffers and the HIP runtime are not included. */
vampomi_status vampomi_dev_mem_plan(int64_t N, int64_t Mt, int nranks, int rank, int cus, int probit, int writer,
                                    int64_t* bytes);
/* One application of the one-pass CG operator (K <= 2 systems, one rank),
 * host buffers: q_k = ar_k/diag [+ beta_k*qo_k], p_k [= z_k + beta_k*p_k]
 * when z is not null (then qo and beta are required), and
 *   d_k = tau * A^T q_k + gam2 * p_k   (M doubles each, k-major),
 *   ad_k = A d_k                      (N doubles each),
 *   dp_k = <d_k, p_k>.
 * ar, qo: K x N; p, z: K x M. */
vampomi_status vampomi_dev_op_apply(vampomi_ctx* ctx, int K, const double* ar, const double* qo, const double* p,
                                    const double* z, const double* beta, double diag, double tau, double gam2,
                                    double* d, double* ad, double* dp);

#ifdef __cplusplus
}
#endif
#endif
