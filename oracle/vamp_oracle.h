/*
 * vamp_oracle.h — CPU restatement of the gVAMPomi linear VAMP hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker
 * (or the timed CPU baseline), never as the product path.
 *
 * Pinning, by part:
 *  - OPERATORS pinned to the reference: its src/data.cpp (no Boost) builds here
 *    where it lies (oracle/Makefile target ref -> oracle/_ref/ref_data), and
 *    this file's A.x, A^T.u, marker statistics and read_phen reproduce its
 *    outputs (tests/test_ref_pin.py: A.x bit-exact, the rest <= 4e-15);
 *  - ITERATION PARITY UNPINNED: the reference's src/vamp.cpp / vamp_probit.cpp
 *    (medical-genomics-group/VAMPomi @ 2025-07-11) cannot be built in this
 *    image (Boost.Math / Boost.uBLAS / Boost.StringAlgo are absent, and the
 *    published linear path indexes two never-sized vectors at
 *    src/vamp.cpp:70,77,204-205), and it ships no tests, fixtures or golden
 *    vectors.  This restatement follows the reference
 * source line by line (citations on every function) with two documented
 * deviations that the reference itself needs to be runnable at all:
 *   P1  x1_hat and r1 are sized M (the commented-out lines src/vamp.cpp:70,77);
 *   P2  the Bernoulli probe vector (src/vamp.cpp:295-296, std::random_device)
 *       is drawn from an index-keyed generator, so results are reproducible
 *       and independent of the rank count.
 * See DESIGN.md §"Oracle".
 */
#ifndef VAMP_ORACLE_H
#define VAMP_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_MAX_L 64

/* In-place SUM all-reduce of n doubles across ranks (stands for the
 * MPI_Allreduce(MPI_SUM, MPI_COMM_WORLD) calls of the reference).  NULL means
 * one rank. */
typedef void (*orc_allreduce_fn)(double* buf, int64_t n, void* user);

/* ---- index-keyed generators (shared specification with the HIP engine) ---- */
uint64_t orc_splitmix64(uint64_t x);
/* Bernoulli bit for marker `gidx` (global index) in VAMP iteration `it`. */
int orc_bern_bit(uint64_t seed, int it, int64_t gidx);
/* Synthetic design value: dyadic Irwin-Hall(12) N(0,1)-like draw for element
 * (global marker i, sample j); exactly representable, bit-identical anywhere. */
double orc_gauss_dyadic(uint64_t seed, int64_t i, int64_t j);
/* Methylation-like value in [0,1]: per-marker dyadic mean/sd + gauss_dyadic. */
double orc_meth_dyadic(uint64_t seed, int64_t i, int64_t j);
/* Fill `M` marker columns [S, S+M) of N samples (leading dim ld, pad zeroed). */
void orc_generate_markers(uint64_t seed, int kind, int64_t N, int64_t ld, int64_t S, int64_t M,
                          double* X);

/* ---- data:: operators (src/data.cpp) ---- */
/* src/utilities.cpp:207-239 divide_work */
void orc_divide_work(int64_t Mt, int nranks, int rank, int64_t* M, int64_t* S, int64_t* Mm);
/* src/data.cpp:58-110 read_phen.  Returns number of rows read (nonas) or
 * -1 (cannot open) / -2 ("NA" in data).  y must hold at least cap doubles. */
int64_t orc_read_phen(const char* path, int standardize, double* y, int64_t cap,
                      double* intercept, double* scale);
/* standardisation step of read_phen (src/data.cpp:97-107) on an in-memory vector */
void orc_standardize_phen(double* y, int64_t n);
/* src/data.cpp:233-283 compute_markers_statistics */
void orc_marker_stats(const double* X, int64_t N, int64_t ld, int64_t M, int64_t nonas,
                      double alpha_scale, double* mave, double* msig);
/* src/data.cpp:340-373 Ax, LOCAL part (before the all-reduce and the /sqrt(N)) */
void orc_ax_local(const double* X, int64_t N, int64_t ld, int64_t M, const double* mave,
                  const double* msig, const double* x, double* out);
/* full Ax: local + allreduce + division by sqrt(N) (src/data.cpp:367-371) */
void orc_ax(const double* X, int64_t N, int64_t ld, int64_t M, const double* mave,
            const double* msig, const double* x, double* out, orc_allreduce_fn ar, void* user);
/* src/data.cpp:294-333 ATx (dot_product per marker, then * 1/sqrt(N)) */
void orc_atx(const double* X, int64_t N, int64_t ld, int64_t M, const double* mave,
             const double* msig, const double* u, double* out);

/* sensitivity mode: orc_atx sums samples in blocks of B rows (0 = sequential,
 * the reference's order); process-wide, test infrastructure only */
void orc_set_atx_block(int B);
/* Association modes (sensitivity measurement, vamp_oracle.c): the default
 * restatement; the MI355X engine's grouping of every scalar reduction at a
 * team plan (a = team size T, b = workgroups); one reference rank's OpenMP
 * inner_prod with a = threads and a seeded arrival order of their sums. */
#define ORC_ASSOC_DEFAULT 0
#define ORC_ASSOC_DEVICE 1
#define ORC_ASSOC_REFRUN 2
void orc_set_assoc(int mode, int a, int b, uint64_t seed);
double orc_assoc_dot(const double* a, const double* b, int64_t n, int kind);
double orc_dev_dp(const double* d, const double* p, int64_t M, int T, int grid);

/* ---- denoiser (src/vamp.cpp:440-492) ---- */
double orc_g1(double y, double gam1, const double* probs, const double* vars, int L);
double orc_g1d(double y, double gam1, const double* probs, const double* vars, int L);

/* deterministic blocked dot product (src/utilities.cpp:138-162 restated) */
double orc_dot(const double* a, const double* b, int64_t n);

/* ---- the whole linear VAMP run (src/vamp.cpp:18-91,110-438) ---- */
typedef struct {
    int64_t N, Mt, M, S, ld;
    int rank, nranks;
    const double* X;            /* local shard, M columns x ld, marker-major */
    const double* mave;         /* M, from orc_marker_stats */
    const double* msig;         /* M */
    const double* y;            /* N, phenotype after read_phen */
    const double* true_signal;  /* M (local slice) or NULL => zeros */
    const double* x1hat_init;   /* M (local slice) or NULL => zeros */
    orc_allreduce_fn allreduce;
    void* user;
} orc_problem;

typedef struct {
    double gam1, h2;            /* gamw = 1/(1-h2) (src/main_meth.cpp:52) */
    int max_iter, CG_max_iter;
    double CG_err_tol;
    int EM_max_iter;
    double EM_err_thr, rho;
    int learn_vars, learn_prior_delay;
    double stop_criteria_thr, merge_vars_thr;
    int L;
    double vars[ORC_MAX_L];     /* as given on the command line (NOT yet * N) */
    double probs[ORC_MAX_L];
    uint64_t seed;              /* Bernoulli generator seed (P2) */
    const char* out_dir;        /* NULL or "" => no files */
    const char* out_name;
    int verbosity;
} orc_params;

typedef struct {
    int iterations_run;
    /* per iteration (caller-allocated, max_iter entries each, may be NULL) */
    int* cg_iters;              /* k1: CG iterations of the x2 solve */
    int* ons_iters;             /* k2: CG iterations of the Onsager solve */
    int* L_hist;                /* mixture components after updatePrior */
    double* params;             /* 5 per iteration: alpha1 gam1 alpha2 gam2 gamw */
    double* metrics;            /* 6 per iteration */
    double* x1_hist;            /* M per iteration: x1_hat/sqrt(N) (== _it_K.bin) */
    double* r1_hist;            /* M per iteration: r1/sqrt(N)     (== _r1_it_K.bin) */
    double* x1_final;           /* M: returned x1_hat_scaled */
    double* probs_final;        /* ORC_MAX_L */
    double* vars_final;         /* ORC_MAX_L (divided by N, as printed) */
    int L_final;
    int64_t a_passes;           /* reference-equivalent A/A^T passes executed */
    double* prior_hist;         /* probit: 1 + 2*ORC_MAX_L per iteration: L, probs, vars (x N) */
    double* it_wall;            /* omp_get_wtime() at the end of each iteration (timing only; may be NULL) */
    double wall_start;          /* omp_get_wtime() before iteration 1 */
} orc_result;

/* returns 0 on success */
int orc_vamp_infere_linear(const orc_problem* pb, const orc_params* prm, orc_result* res);

/* ---- the probit model (src/vamp_probit.cpp:19-467) ----
 * Same problem/params as the linear run, y = raw 0/1 phenotype
 * (read_phen(false), src/data.cpp:40-43).  h2 is unused.  Result widths:
 * params 8 per iteration (alpha1 beta1 gam1 tau1 alpha2 beta2 gam2 tau2),
 * metrics 12 (TP TN FP FN acc1 x1_corr | TP TN FP FN acc2 x2_corr),
 * x1_final = x1_hat NOT divided by sqrt(N) (src/vamp_probit.cpp:465).
 * P2 also covers the Gaussian start p1 (src/vamp_probit.cpp:53, simulate()
 * with std::random_device): p1[i] = orc_probit_p1(seed, i). */
int orc_vamp_infere_probit(const orc_problem* pb, const orc_params* prm, orc_result* res);
double orc_probit_p1(uint64_t seed, int64_t i);
/* src/utilities.cpp:293-363 (published erfcx, with the reference's clamps) */
double orc_erfcx(double x);
/* src/vamp_probit.cpp:469-488, probit_var = 1 (src/vamp.hpp:35), m_cov = 0 */
double orc_g1_bin(double p, double tau1, double y);
double orc_g1d_bin(double p, double tau1, double y);

/* ---- association tests (--run-mode association_test) ---- */
/* linear_reg1d_pvals, src/utilities.cpp:269-282 */
double orc_reg1d_pval(double sumx, double sumsqx, double sumxy, double sumy, double sumsqy, int n);
/* Student t upper tail P(T > t) (stands for Boost's complemented cdf) */
double orc_t_sf(double t, double df);
double orc_lnbeta_half(double a);
/* --pval-method loo (src/main_meth.cpp:245-264, src/data.cpp:385-417): est is
 * the estimate-file slice (x1_hat/sqrt(N)); uses pb->X/mave/msig/y and
 * pb->allreduce for the Ax.  stats (5 per marker: sumx sumsqx sumxy sumy
 * sumsqy) may be NULL. */
void orc_assoc_loo(const orc_problem* pb, const double* est, double* pvals, double* stats);
/* --pval-method se (src/main_meth.cpp:218-242) */
void orc_assoc_se(const double* r1, int64_t M, double gam1, int64_t N, double* pvals);

/* ---- --run-mode test (src/main_meth.cpp:112-205) ----
 * pb = the TEST data set; est = estimate-file slice (x1_hat/sqrt(N));
 * out[0] = R2 test, out[1] = z correlation test (squared) */
void orc_test_metrics(const orc_problem* pb, const double* est, double* out);

/* updatePrior alone (src/vamp.cpp:531-643): uses prm's EM_max_iter,
 * EM_err_thr, learn_vars, merge_vars_thr; vars multiplied by N */
int orc_update_prior(const orc_problem* pb, const double* r1, double gam1, const orc_params* prm, int* L,
                     double* probs, double* vars);

/* ---- output writers (src/utilities.cpp:241-249, 366-401) ---- */
int orc_store_vec(const char* path, const double* v, int64_t S, int64_t M);
int orc_csv_header(const char* path, const char* const* fields, int n);
int orc_csv_row(const char* path, int it, const double* vals, int n);
/* setup_io without a header (the probit path writes none) */
int orc_csv_create(const char* path);

#ifdef __cplusplus
}
#endif
#endif
