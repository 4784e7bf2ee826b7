// run.h — state of one VAMP run (linear or probit) on the device, shared by
// vamp.cpp (vamp::infere_linear, begin/step/end) and probit.cpp
// (vamp::infere_bin_class).  Internal to libvampomi.
#pragma once
#include <string>
#include <vector>

#include "ctx.h"
#include "writer.h"

struct Mixture {
    int L = 0;
    double probs[VAMPOMI_MAX_L] = {};
    double vars[VAMPOMI_MAX_L] = {};  // multiplied by N (src/vamp.cpp:87-88)
};

inline double smax(double a, double b) { return (a < b) ? b : a; }  // std::max
inline double smin(double a, double b) { return (b < a) ? b : a; }  // std::min

struct VampRun {
    vampomi_params prm{};
    vampomi_result* res = nullptr;
    bool probit = false;  // model "bin_class"
    bool write = false;
    bool fuse = true;  // batch_rhs >= 1: share passes + prefetch the next denoising step
    bool recur = false;  // batch_rhs >= 2: A^T A x2 and A^T A invQ by CG recurrences (no pass)
    bool arec = false;   // batch_rhs >= 3: also A x2 by a CG recurrence, z1 in the first CG pass
    bool onepass = false;  // batch_rhs >= 4: each CG step reads X once (vk::atax)
    int z1n_slot = 2;    // nb3 slot of the prefetched z1
    int bern_it = 0;     // probit: the iteration whose probe bern holds (drawn one iteration early)
    int abern_it = 0;    // probit: the iteration whose A.bern is in nb3 slot 3
    // probit: iteration it+1's head, resolved at iteration it's last flush
    // (probit.cpp): its updatePrior applied (em_head == it+1), and its z-side
    // denoising sums and accuracy counts (z_head == it+1)
    int em_head = 0, z_head = 0;
    double zh_bsum = 0, zh_cnt[4] = {}, zh_xc[3] = {};
    int hs_it = 0;       // linear: the iteration whose A.bern is in abern (the CG head start)
    std::string out_dir, out_name, p_params, p_metrics, p_prior;
    int it = 0;
    bool stopped = false;
    // a file write failed on this rank: reported on every rank by agree_io, so
    // the ranks leave the collective sequence together (src/vamp.cpp writes
    // rank-locally; a rank that stopped there would leave the others waiting)
    bool io_err = false;
    std::string io_msg;
    // per-iteration vectors and CSV rows, written off the critical path: the
    // context's writer (writer.h) while this run writes files or keeps history
    IterWriter* writer = nullptr;
    Mixture mix, mix_next;
    bool have_next = false;  // x1n, alpha1_next, mix_next, z1 (nb3 slot 2), atx0 valid
    double gam1 = 0, gam2 = 0, gamw = 0;
    double alpha1 = 0, alpha2 = 0, eta1 = 0, eta2 = 0, alpha1_next = 0;
    double metrics[12] = {}, params[8] = {};
    // reduction sinks
    double e1m[3] = {}, e1n[2] = {}, e1s[3] = {}, e2m[3] = {}, e2n[2] = {}, e2s[3] = {};
    double tn = 0, tc = 0, nm[2] = {}, sum_d = 0, a2 = 0;
    // device M-vectors
    double *r1 = nullptr, *x1 = nullptr, *x1p = nullptr, *x1n = nullptr, *x1d = nullptr, *r2 = nullptr;
    double *x2 = nullptr, *bern = nullptr, *invQ = nullptr, *v = nullptr, *atxy = nullptr, *ts = nullptr;
    double *tmpM = nullptr, *atx0 = nullptr;
    double* cgw[10] = {};  // r, z, p, d of the two CG systems; raw A^T A p of each (recur)
    // device N-vectors (ld each)
    double *z1buf = nullptr, *nb3 = nullptr /* A.x2, A.invQ, A.x1_next */, *nsc = nullptr;
    double* ax2 = nullptr;  // arec: A x2, carried from iteration to iteration
    double* abern = nullptr;      // the head start: A.bern of iteration hs_it in slot hs_it & 1 (2 x ld)
    double* bern_next = nullptr;  // ... and the next iteration's probe (M)
    // the device EM update (vk::EmArgs.upd): the mixture it formed (device
    // words, read by the next denoising) and its mapped host mirror, checked
    // against the host's update (mix_expect) once a later launch has flagged
    // (check_device_mix)
    double* mixw = nullptr;
    double* mixh = nullptr;
    double* mixh_dev = nullptr;
    bool mix_pending = false;
    Mixture mix_expect;
    // the iteration whose prelude and solves' start the previous iteration
    // queued ahead (0: none), its scalars formed on the device (vk::PreOut);
    // mixh + kMixWords holds them (eta1, gam2, gamw, diag), checked against
    // the host's (check_device_values).  VAMPOMI_PRE_AHEAD=0: off
    int pre_ahead = 0;
    bool pre_ahead_on = true;
    const double* z1 = nullptr;
    int64_t passes_ref = 0;
    // probit (src/vamp_probit.cpp) state
    double tau1 = 0, tau2 = 0, beta1 = 0, beta2 = 0;
    double* p1 = nullptr;   // N
    double* p2 = nullptr;   // N
    double* z1h = nullptr;  // N: z1_hat
    double* x1s = nullptr;  // M: x1_hat / sqrt(N)
    double* x1sn = nullptr; // M: next iteration's x1_hat / sqrt(N)
    double* x2s = nullptr;  // M: x2_hat / sqrt(N)
    double* prior_row = nullptr;  // host staging, unused by the linear model
    // the last step's phases as the host sees them (vampomi_step_phases): the
    // solves (entering pcg_run to its return: the device's CG and Onsager
    // steps, with the linear model's start queued ahead running a little
    // earlier) and the whole step
    double ph_solve_s = 0, ph_step_s = 0;

    ~VampRun();
};

struct EmParams {
    int EM_max_iter;
    double EM_err_thr;
    int learn_vars;
    double merge_vars_thr;
    int verbosity;
};
EmParams em_params(const VampRun& R);
vampomi_status update_prior(vampomi_ctx* c, const EmParams& P, Mixture& m, double gam1, const double* r1);
vampomi_status update_prior(vampomi_ctx* c, const VampRun& R, Mixture& m, double gam1, const double* r1);
// updatePrior in two halves (vamp.cpp): em_begin queues the first EM round's
// sums into b; after b.flush(), em_finish completes the update
struct EmState {
    int emit = 0;
    double lambda = 0;
    double omegas[VAMPOMI_MAX_L] = {};
    double sums[2 * VAMPOMI_MAX_L] = {};
};
// r1from (may be null): round 0 also forms r1 itself (vk::EmArgs.r1out) from
// these lincomb_div inputs, in the same launch (em_begin queues round 0 only
// if EM_max_iter >= 1: the caller forms r1 otherwise)
struct R1From {
    const double* x2;
    const double* r2;
    double eta2, gam2, gam1;
    const double* dsc = nullptr;  // device: gam1, eta2 (vk::G1Chain); then eta2 and gam1 above are unused
};
// upd (may be null, one round): the round's launch also forms the update of
// the mixture on the device (vk::EmArgs.upd)
vampomi_status em_begin(vampomi_ctx* c, const EmParams& P, const Mixture& m, double gam1, const double* r1,
                        DotBatch& b, EmState& s, const R1From* r1from = nullptr, const vk::EmUpd* upd = nullptr);
vampomi_status em_queue(vampomi_ctx* c, const Mixture& m, double gam1, const double* r1, DotBatch& b, EmState& s,
                        const R1From* r1from = nullptr, const vk::EmUpd* upd = nullptr);
vampomi_status em_finish(vampomi_ctx* c, const EmParams& P, Mixture& m, double gam1, const double* r1, EmState& s);
// mixw / gam1dev (may be null): the mixture's words and gam1 from the device
// (vk::denoise)
vampomi_status denoise_into(vampomi_ctx* c, const Mixture& m, double gam1, const double* r1, double* x1,
                            const double* x1_prev, bool damp, double rho, double* x1d, DotBatch& b, double* sum_out,
                            const double* mixw = nullptr, const double* gam1dev = nullptr,
                            const vk::PreOut* po = nullptr);
vampomi_status upload_or_zero(vampomi_ctx* c, double* dst, const double* host, int64_t n);
// queues this iteration's x1/sqrt(N), r1/sqrt(N) for the _it_K.bin /
// _r1_it_K.bin files and the x1/r1 history (R.writer)
vampomi_status write_bins(vampomi_ctx* c, VampRun& R);
// queues a CSV row (rank 0 writes them) behind the iteration's vectors
void write_row(VampRun& R, const std::string& path, int it, const double* vals, int n);
// a rank-local I/O failure (R.io_err, or a finished writer job) becomes every
// rank's ERR_IO; wait_all: first wait for every queued write (the last
// iteration).  COLLECTIVE
vampomi_status agree_io(vampomi_ctx* c, VampRun& R, bool wait_all = false);
// the end of an iteration's output (after R.stopped is decided): the history
// row is in place, and write failures so far (all writes after the last
// iteration) are agreed over the ranks.  COLLECTIVE when writing files
vampomi_status end_iteration_io(vampomi_ctx* c, VampRun& R);
// probit.cpp
vampomi_status probit_begin(vampomi_ctx* c, VampRun& R);
vampomi_status probit_step(vampomi_ctx* c, VampRun& R);
