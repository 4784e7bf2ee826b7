// vamp.cpp — the gVAMPomi linear VAMP model on the device
// (vamp::vamp + vamp::infere_linear, src/vamp.cpp:18-91, 110-438).
//
// Every vector of the VAMP state lives in HBM; the host keeps the scalars
// the algorithm branches on.  Per iteration the work is the reference's, in
// the reference's arithmetic, with three bandwidth reformulations that leave
// every value bitwise unchanged (batch_rhs=1; tests/test_gpu_parity.py checks
// it against batch_rhs=0 bit for bit):
//   1. the x2 CG solve and the Onsager CG solve share each pass over X
//      (pcg.cpp);
//   2. updateNoisePrec's A.x2 and A.invQ_bern_vec (:508, :518) share one
//      pass, which also carries the NEXT iteration's z1 = A.x1_hat (:232):
//      denoising of iteration it+1 (updatePrior, g1, g1d) needs only r1 and
//      gam1 of iteration it, so it runs before updateNoisePrec of it;
//   3. updateNoisePrec's A^T pass (:519) also computes A^T(A x2_hat), which
//      is the next x2 solve's warm-start product lmmse_mult(mu_CG_last)
//      (:681) up to the tau / gam2 epilogue applied when those are known.
// err_measures' A.x2_hat (:826) is the product of (2); A^T y (:303) is
// computed once.  Scalar reductions are batched per dependency level.
// batch_rhs=2 replaces the A^T pass of (3) by recurrences: the CG
// keeps W += alpha*A^T(A p) beside mu += alpha*p for both systems, so the
// pass count per iteration is 1 + 2*max(k1, k2) instead of 2 + 2*max(k1, k2);
// the vectors are the same up to rounding (parity within 1e-10, counts exact).
// batch_rhs=3 also carries A x2 as A x2 += alpha * A p through the CG steps
// (from the previous iteration's A x2) and computes z1 = A x1_hat as one more
// right-hand side of the first CG pass, so no pass over X is left outside the
// CG: 2*max(k1, k2) passes per iteration.
// batch_rhs=4 (the default) reads X once per CG step: A p is carried as an
// N-vector recurrence and the one-pass operator (atax_team.hip) forms A^T q
// and A d from the same column read: 1 + max(k1, k2) passes per iteration.
// On one rank the iteration's tail after the solves runs without the host
// (DESIGN.md §4.4 item 5): its reductions in one launch (vk::dots2) whose
// last block also forms gam1 (vk::G1Chain); the EM round, whose last block
// forms the mixture update; the next denoising, whose last block forms the
// next prelude's scalars (vk::PreOut); and the next prelude + CG start
// (pcg_run's PreMode::ahead).  The host waits once, at the end, forms the
// same scalars and mixture from the same sums, and checks the device's bit
// for bit after the next solves (check_device_values).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>

#include "ctx.h"
#include "hostio.h"
#include "run.h"

VampRun::~VampRun() {
    if (writer) writer->drain(nullptr);  // its kernels read x1 / r1, its thread writes the caller's history arrays
    for (double** p : {&r1, &x1, &x1p, &x1n, &x1d, &r2, &x2, &bern, &invQ, &v, &atxy, &ts, &tmpM, &atx0, &z1buf,
                       &nb3, &nsc, &ax2, &p1, &p2, &z1h, &x1s, &x1sn, &x2s, &abern, &bern_next})
        dev_free(*p);
    for (auto& p : cgw) dev_free(p);
    dev_free(mixw);
    if (mixh) (void)hipHostFree(mixh);
}

vampomi_ctx::vampomi_ctx() = default;

vampomi_ctx::~vampomi_ctx() {
    run.reset();
    writer.reset();  // drained, its thread joined, before the staging buffers go
    release_ctx_resources(this);
}

// updatePrior (src/vamp.cpp:531-643) on mixture m, from r1 and gam1, split in
// two so that a caller can queue the first EM round's sums early, with other
// reductions, and resolve them together: em_begin queues round 0
// into b; after b.flush(), em_finish does its host part, the further rounds
// (each with its own batch) and the merge.  update_prior runs both.
vampomi_status em_begin(vampomi_ctx* c, const EmParams& P, const Mixture& m, double gam1, const double* r1,
                        DotBatch& b, EmState& s, const R1From* r1from, const vk::EmUpd* upd) {
    s.emit = 0;
    s.lambda = 1 - m.probs[0];
    for (int j = 0; j < m.L; ++j) s.omegas[j] = m.probs[j];
    for (int j = 1; j < m.L; ++j) s.omegas[j] /= s.lambda;
    if (P.EM_max_iter < 1) return VAMPOMI_OK;
    return em_queue(c, m, gam1, r1, b, s, r1from, upd);
}

// one EM round's per-slab sums (:555-597) into b, on b's current stream
vampomi_status em_queue(vampomi_ctx* c, const Mixture& m, double gam1, const double* r1, DotBatch& b,
                        EmState& s, const R1From* r1from, const vk::EmUpd* upd) {
    const int L = m.L;
    double max_sigma = m.vars[0];
    for (int j = 1; j < L; ++j) max_sigma = smax(max_sigma, m.vars[j]);  // std::max_element
    vk::EmArgs a{};
    for (int j = 0; j < L; ++j) {
        a.omegas[j] = s.omegas[j];
        a.vars[j] = m.vars[j];
    }
    for (int j = 1; j < L; ++j) a.v[j - 1] = 1.0 / (1.0 / m.vars[j] + gam1);
    a.lambda = s.lambda;
    a.noise_var = 1 / gam1;
    a.gam1 = gam1;
    a.max_sigma = max_sigma;
    a.L = L;
    if (r1from) {
        a.lx = r1from->x2;
        a.ly = r1from->r2;
        a.la = r1from->eta2;
        a.lb = r1from->gam2;
        a.lc = r1from->gam1;
        a.r1out = const_cast<double*>(r1);
        a.dsc = r1from->dsc;
    }
    if (upd) a.upd = *upd;
    vk::RedOut ro{};
    STCHK(b.sink(1 + 2 * (L - 1), true, s.sums, &ro));  // :578, :596-597
    HIPCHK(vk::em_sums(c->M, r1, a, ro, b.stream()));
    return VAMPOMI_OK;
}

vampomi_status em_finish(vampomi_ctx* c, const EmParams& P, Mixture& m, double gam1, const double* r1,
                         EmState& s) {
    for (; s.emit < P.EM_max_iter; ++s.emit) {
        if (s.emit > 0) {  // round 0 was queued by em_begin and resolved by its batch
            DotBatch b(c);
            STCHK(em_queue(c, m, gam1, r1, b, s));
            STCHK(b.flush());
        }
        const int L = m.L;
        double probs_prev[VAMPOMI_MAX_L], vars_prev[VAMPOMI_MAX_L];
        std::memcpy(probs_prev, m.probs, sizeof probs_prev);
        std::memcpy(vars_prev, m.vars, sizeof vars_prev);
        const double lambda_total = s.sums[0];
        s.lambda = lambda_total / (double)c->Mt;
        const double sum_of_pin = lambda_total;
        for (int j = 0; j < L - 1; ++j) {
            const double res_total = s.sums[1 + j];
            const double res_gammas_total = s.sums[L + j];
            if (P.learn_vars == 1) m.vars[j + 1] = res_gammas_total / res_total;
            s.omegas[j + 1] = res_total / sum_of_pin;
            m.probs[j + 1] = s.lambda * s.omegas[j + 1];
        }
        m.probs[0] = 1 - s.lambda;
        double dprob = 0, nprob = 0, dvar = 0, nvar = 0;
        for (int j = 0; j < L; ++j) {
            dprob += (m.probs[j] - probs_prev[j]) * (m.probs[j] - probs_prev[j]);
            nprob += m.probs[j] * m.probs[j];
            dvar += (m.vars[j] - vars_prev[j]) * (m.vars[j] - vars_prev[j]);
            nvar += m.vars[j] * m.vars[j];
        }
        const double dist_probs = std::sqrt(dprob / nprob), dist_vars = std::sqrt(dvar / nvar);
        if (P.verbosity == 1 && c->rank == 0)
            std::printf("it = %d: dist_probs = %g & dist_vars = %g\n", s.emit, dist_probs, dist_vars);
        if (dist_probs < P.EM_err_thr && dist_vars < P.EM_err_thr) break;
    }
    // merging close variances (:626-642)
    for (int j = 0; j < m.L; ++j) {
        for (int k = j + 1; k < m.L; ++k) {
            const double denom = m.vars[j] != 0 ? smin(m.vars[j], m.vars[k]) : 1e-7;
            if (std::fabs(m.vars[j] - m.vars[k]) / denom < P.merge_vars_thr) {
                const double sum2probs = m.probs[j] + m.probs[k];
                for (int q = k; q + 1 < m.L; ++q) {
                    m.vars[q] = m.vars[q + 1];
                    m.probs[q] = m.probs[q + 1];
                }
                m.L--;
                m.probs[j] = sum2probs;
                k--;
            }
        }
    }
    return VAMPOMI_OK;
}

vampomi_status update_prior(vampomi_ctx* c, const EmParams& P, Mixture& m, double gam1, const double* r1) {
    EmState s;
    DotBatch b(c);
    STCHK(em_begin(c, P, m, gam1, r1, b, s));
    STCHK(b.flush());
    return em_finish(c, P, m, gam1, r1, s);
}

EmParams em_params(const VampRun& R) {
    return EmParams{R.prm.EM_max_iter, R.prm.EM_err_thr, R.prm.learn_vars, R.prm.merge_vars_thr, R.prm.verbosity};
}

vampomi_status update_prior(vampomi_ctx* c, const VampRun& R, Mixture& m, double gam1, const double* r1) {
    return update_prior(c, em_params(R), m, gam1, r1);
}

// x1 = g1(r1) [damped], x1d = g1d(r1); sum of x1d over ranks queued in b
vampomi_status denoise_into(vampomi_ctx* c, const Mixture& m, double gam1, const double* r1, double* x1,
                                   const double* x1_prev, bool damp, double rho, double* x1d, DotBatch& b,
                                   double* sum_out, const double* mixw, const double* gam1dev,
                                   const vk::PreOut* po) {
    vk::Mix mix{};
    mix.L = m.L;
    for (int j = 0; j < m.L; ++j) {
        mix.probs[j] = m.probs[j];
        mix.vars[j] = m.vars[j];
    }
    vk::RedOut ro{};
    STCHK(b.sink(1, true, sum_out, &ro));  // :214-222
    HIPCHK(vk::denoise(c->M, r1, gam1, mix, x1, x1_prev, damp ? 1 : 0, rho, x1d, ro, b.stream(), mixw, gam1dev, po));
    return VAMPOMI_OK;
}

// err_measures (src/vamp.cpp:760-852): the reductions (queued) ...  xm / xn:
// another group of reductions over M / over N that shares the launch (one
// kernel per vector length instead of one per group)
static void err_groups(vampomi_ctx* c, VampRun& R, const double* xhat, const double* Axest, double* m3, double* n2,
                       double* s3, std::vector<DotBatch::Group>& gm, std::vector<DotBatch::Group>& gn) {
    gm.push_back({{T(xhat, R.ts), T(xhat, xhat), T(R.ts, R.ts)}, true, m3});
    gn.push_back({{T(c->y, Axest, vk::DIFF2), T(c->y, c->y)}, false, n2});  // l2_norm2(., 0)
    gn.push_back({{T(Axest, c->y), T(Axest, Axest), T(c->y, c->y)}, true, s3});
}

static vampomi_status err_queue(vampomi_ctx* c, VampRun& R, const double* xhat, const double* Axest, DotBatch& b,
                                double* m3, double* n2, double* s3, std::vector<DotBatch::Group> gm = {},
                                std::vector<DotBatch::Group> gn = {}) {
    err_groups(c, R, xhat, Axest, m3, n2, s3, gm, gn);
    STCHK(b.add_many(c->M, gm));
    return b.add_many(c->N, gn);
}

// ... and the scalar formulas once they are back
static void err_finish(VampRun& R, const double* m3, const double* n2, const double* s3, int ind) {
    const double corr = m3[0] / std::sqrt(m3[1] * m3[2]);
    const double l2_pred_err = std::sqrt(n2[0] / n2[1]);
    const double R2 = 1 - l2_pred_err * l2_pred_err;
    const double corr_y = s3[0] / std::sqrt(s3[1] * s3[2]);
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
}

vampomi_status upload_or_zero(vampomi_ctx* c, double* dst, const double* host, int64_t n) {
    if (n <= 0) return VAMPOMI_OK;
    if (host)
        HIPCHK(hipMemcpyAsync(dst, host, (size_t)n * 8, hipMemcpyHostToDevice, c->st));
    else
        HIPCHK(hipMemsetAsync(dst, 0, (size_t)n * 8, c->st));
    return VAMPOMI_OK;
}

static bool keeps_hist(const VampRun& R) { return R.res && (R.res->x1_hist || R.res->r1_hist); }
vampomi_status ensure_writer(vampomi_ctx* c, VampRun& R);

static vampomi_status vamp_alloc(vampomi_ctx* c, VampRun& R) {
    const size_t M = (size_t)std::max<int64_t>(c->M, 1), ld = (size_t)c->ld;
    for (double** p : {&R.r1, &R.x1, &R.x1p, &R.x1n, &R.x1d, &R.r2, &R.x2, &R.bern, &R.invQ, &R.v, &R.atxy, &R.ts,
                       &R.tmpM, &R.atx0, &R.bern_next})
        STCHK(dev_alloc(p, M));
    for (auto& p : R.cgw) STCHK(dev_alloc(&p, M));
    STCHK(dev_alloc(&R.z1buf, ld));
    STCHK(dev_alloc(&R.nb3, vk::kMaxRhs * ld));  // probit: slot 3 carries the next A.bern_vec
    STCHK(dev_alloc(&R.nsc, vk::kMaxRhs * ld));
    STCHK(dev_alloc(&R.ax2, ld));
    STCHK(dev_alloc(&R.abern, 2 * ld));  // two slots: A.bern of it (consumed in place) and of it + 1
    STCHK(dev_alloc(&R.mixw, vk::kMixWords));
    HIPCHK(hipHostMalloc((void**)&R.mixh, (vk::kMixWords + 4) * sizeof(double),
                         hipHostMallocMapped | hipHostMallocCoherent));
    {
        const char* e = std::getenv("VAMPOMI_PRE_AHEAD");
        R.pre_ahead_on = !e || std::atoi(e) != 0;
    }
    HIPCHK(hipHostGetDevicePointer((void**)&R.mixh_dev, R.mixh, 0));
    HIPCHK(hipMemsetAsync(R.ax2, 0, ld * 8, c->st));
    HIPCHK(hipMemsetAsync(R.abern, 0, 2 * ld * 8, c->st));
    HIPCHK(hipMemsetAsync(R.z1buf, 0, ld * 8, c->st));
    HIPCHK(hipMemsetAsync(R.nb3, 0, vk::kMaxRhs * ld * 8, c->st));
    HIPCHK(hipMemsetAsync(R.nsc, 0, vk::kMaxRhs * ld * 8, c->st));
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_vamp_begin(vampomi_ctx* c, const vampomi_params* p, vampomi_result* r) {
    CollScope cs_(c);
    if (!c || !p) return fail(VAMPOMI_ERR_ARG, "null argument");
    if (!c->have_X || !c->have_y) return fail(VAMPOMI_ERR_STATE, "load methylation data and phenotype first");
    const bool probit = p->model && std::strcmp(p->model, "bin_class") == 0;
    if (p->model && !probit && std::strcmp(p->model, "linear") != 0)  // src/vamp.cpp:98-104
        return fail(VAMPOMI_ERR_MODEL, std::string("Invalid model specification! ('") + p->model + "')");
    if (p->L < 1 || p->L > VAMPOMI_MAX_L) return fail(VAMPOMI_ERR_ARG, "number of mixture components out of range");
    HIPCHK(hipSetDevice(c->device));
    STCHK(op_agree(c));  // several ranks: the one-pass / head-start choice, agreed here, where every rank is
    c->run.reset(new VampRun());
    VampRun& R = *c->run;
    R.prm = *p;
    R.res = r;
    R.probit = probit;
    R.fuse = p->batch_rhs != 0;
    R.recur = p->batch_rhs >= 2;
    R.arec = p->batch_rhs >= 3;
    R.onepass = p->batch_rhs >= 4;
    R.out_dir = p->out_dir ? p->out_dir : "";
    R.out_name = p->out_name ? p->out_name : "";
    R.write = !R.out_dir.empty();
    R.mix.L = p->L;
    for (int j = 0; j < p->L; ++j) {
        R.mix.probs[j] = p->probs[j];
        R.mix.vars[j] = p->vars[j] * (double)c->N;  // src/vamp.cpp:87-88
    }
    R.gam1 = p->gam1;
    R.gamw = 1.0 / (1.0 - p->h2);  // src/main_meth.cpp:52
    R.gam2 = 0;
    STCHK(vamp_alloc(c, R));
    if (R.write || keeps_hist(R)) STCHK(ensure_writer(c, R));  // its pinned buffers before iteration 1
    STCHK(upload_or_zero(c, R.ts, p->true_signal, c->M));
    // P1 (src/vamp.cpp:70-79): x1_hat = r1 = x1hat_init / sqrt(N)
    std::vector<double> h((size_t)std::max<int64_t>(c->M, 1), 0.0);
    for (int64_t i = 0; i < c->M; ++i) h[i] = (p->x1hat_init ? p->x1hat_init[i] : 0.0) / std::sqrt((double)c->N);
    STCHK(upload_or_zero(c, R.x1, h.data(), c->M));
    STCHK(upload_or_zero(c, R.r1, h.data(), c->M));
    STCHK(upload_or_zero(c, R.x2, nullptr, c->M));
    if (R.probit) {
        if (r) {
            r->iterations_run = 0;
            r->a_passes_ref = 0;
            r->a_passes_exec = 0;
        }
        STCHK(probit_begin(c, R));
        STCHK(sync_stream(c, c->st));
        return VAMPOMI_OK;
    }
    {  // A^T y is the same every iteration (y fixed, src/vamp.cpp:303): one pass
        const double* u[1] = {c->y};
        double* o[1] = {R.atxy};
        STCHK(atx_dev(c, 1, u, o, 0, 0.0, 0.0, nullptr));
    }
    if (R.write) {
        R.p_metrics = R.out_dir + "/" + R.out_name + "_metrics.csv";
        R.p_params = R.out_dir + "/" + R.out_name + "_params.csv";
        R.p_prior = R.out_dir + "/" + R.out_name + "_prior.csv";
        if (c->rank == 0) {  // setup_io + headers (src/vamp.cpp:115-123, 854-882)
            std::vector<std::string> prior_h{"iteration", "number of components"};
            for (int i = 0; i < R.mix.L; ++i) prior_h.push_back("prob" + std::to_string(i));
            for (int i = 0; i < R.mix.L; ++i) prior_h.push_back("var" + std::to_string(i));
            const bool ok =
                vio::csv_create_with_header(R.p_metrics, {"iteration", "R2 denoising", "x1 correlation denoising",
                                                          "R2 LMMSE", "x2 correlation LMMSE", "z1 correlation denoising",
                                                          "z2 correlation LMMSE"}) &&
                vio::csv_create_with_header(R.p_params, {"iteration", "alpha1", "gam1", "alpha2", "gam2", "gamw"}) &&
                vio::csv_create_with_header(R.p_prior, prior_h);
            if (!ok) {
                R.io_err = true;
                R.io_msg = "cannot create output CSV files in " + R.out_dir;
            }
        }
        STCHK(agree_io(c, R));
    }
    if (r) {
        r->iterations_run = 0;
        r->a_passes_ref = 0;
        r->a_passes_exec = 0;
    }
    STCHK(sync_stream(c, c->st));
    return VAMPOMI_OK;
}

vampomi_status ensure_writer(vampomi_ctx* c, VampRun& R) {
    if (R.writer) return VAMPOMI_OK;
    if (!c->writer) return fail(VAMPOMI_ERR_STATE, "context without an iteration writer");
    c->writer->drain(nullptr);  // (an earlier run that ended with an error)
    c->writer->clear_error();
    R.writer = c->writer.get();
    return VAMPOMI_OK;
}

// x1_hat_scaled (src/vamp.cpp:237-238) and r1_scaled (:246-248), written by
// R.writer while the iteration goes on (writer.h)
vampomi_status write_bins(vampomi_ctx* c, VampRun& R) {
    const bool hist = keeps_hist(R);
    if (!R.write && !hist) return VAMPOMI_OK;
    STCHK(ensure_writer(c, R));
    const int64_t off = (int64_t)(R.it - 1) * c->M;
    std::string px, pr;
    if (R.write) {
        const std::string base = R.out_dir + "/" + R.out_name;
        px = base + "_it_" + std::to_string(R.it) + ".bin";
        pr = base + "_r1_it_" + std::to_string(R.it) + ".bin";
    }
    return R.writer->submit_vectors(c, R.x1, R.r1, px, pr, hist && R.res->x1_hist ? R.res->x1_hist + off : nullptr,
                                    hist && R.res->r1_hist ? R.res->r1_hist + off : nullptr);
}

void write_row(VampRun& R, const std::string& path, int it, const double* vals, int n) {
    std::vector<double> v(vals, vals + n);
    auto job = [path, it, v](std::string* msg) {
        if (vio::csv_write_row(path, it, v.data(), (int)v.size())) return true;
        *msg = "cannot write CSV rows to " + path;
        return false;
    };
    if (R.writer) {
        R.writer->submit_host(job);
    } else {
        std::string msg;
        if (!job(&msg)) {
            R.io_err = true;
            R.io_msg = msg;
        }
    }
}

vampomi_status agree_io(vampomi_ctx* c, VampRun& R, bool wait_all) {
    if (R.writer && !R.io_err) {
        std::string msg;
        if (wait_all ? R.writer->drain(&msg) : R.writer->failed(&msg)) {
            R.io_err = true;
            R.io_msg = msg;
        }
    }
    double bad = 0.0;
    STCHK(sum_over_ranks(c, R.io_err ? 1.0 : 0.0, &bad));
    if (bad > 0)
        return fail(VAMPOMI_ERR_IO, R.io_err ? R.io_msg
                                             : "output file write failed on " + std::to_string((int)bad) + " other rank(s)");
    return VAMPOMI_OK;
}

vampomi_status end_iteration_io(vampomi_ctx* c, VampRun& R) {
    if (keeps_hist(R) && R.writer) R.writer->drain(nullptr);  // the history row of this iteration is in place
    if (R.write) return agree_io(c, R, R.stopped);  // files written so far; all of them after the last iteration
    std::string msg;
    if (R.writer && R.writer->failed(&msg)) return fail(VAMPOMI_ERR_HIP, msg);
    return VAMPOMI_OK;
}

// The mixture the device denoised with (devem) is the host's, bit for bit.
// Called once a launch queued after that denoising has flagged the host (its
// stores are then visible) and before the next denoising overwrites them.
static vampomi_status check_device_mix(VampRun& R) {
    if (!R.mix_pending) return VAMPOMI_OK;
    R.mix_pending = false;
    const Mixture& m = R.mix_expect;
    bool same = (double)m.L == R.mixh[0];
    for (int j = 0; same && j < m.L; ++j)
        same = std::memcmp(&m.probs[j], &R.mixh[1 + j], 8) == 0 &&
               std::memcmp(&m.vars[j], &R.mixh[1 + vk::kMaxL + j], 8) == 0;
    if (!same) return fail(VAMPOMI_ERR_STATE, "vamp: the device's EM update differs from the host's");
    return VAMPOMI_OK;
}

// The LMMSE half's solves of iteration it (src/vamp.cpp:289-350): their
// vectors, schedule flags and the prelude (r2, the probe bern, v and the zero
// starts, :259-261, :295-306, :496), from R's scalars and x1 (iteration it's
// x1_hat).  No launches: vamp_step queues them, and the previous iteration
// may queue the prelude and the solves' start ahead (R.pre_ahead).
struct LmmseSetup {
    CgSystem sx{}, so{};
    bool rec = false, arec = false, hs_av = false, pre_in_cg = false;
    HeadStart hs;
    vk::Prelude pr{};
};

static vampomi_status lmmse_setup(vampomi_ctx* c, VampRun& R, int it, const double* x1, LmmseSetup& L) {
    const int64_t ld = c->ld;
    CgSystem& sx = L.sx;
    CgSystem& so = L.so;
    sx.v = R.v;
    sx.mu = R.x2;  // mu_CG_last: warm start, updated in place (:308-311, :753-754)
    sx.mu0_nonzero = it > 1;
    sx.atx0 = (it > 1 && R.have_next) ? R.atx0 : nullptr;
    sx.r = R.cgw[0];
    sx.z = R.cgw[1];
    sx.p = R.cgw[2];
    sx.d = R.cgw[3];
    so.v = R.bern;
    so.mu = R.invQ;  // g2d_onsager starts from zeros (:496, :664-669)
    so.onsager = true;
    so.r = R.cgw[4];
    so.z = R.cgw[5];
    so.p = R.cgw[6];
    so.d = R.cgw[7];
    // batch_rhs 2: updateNoisePrec's A^T(A x2) (the next warm start, :681) and
    // A^T(A invQ) (the trace, :519) are carried through the CG steps as
    // W += alpha * A^T(A p) beside mu += alpha * p, instead of one more pass
    // over X per iteration (mathematically the same vectors; rounding differs)
    L.rec = R.recur && R.fuse && (it == 1 || sx.atx0);
    if (L.rec) {
        sx.W = R.atx0;  // holds A^T A mu0 on entry (the warm start's product), in place
        sx.S = R.cgw[8];
        so.W = R.tmpM;  // invQ starts from zeros
        so.S = R.cgw[9];
    }
    // batch_rhs 3: A x2 (updateNoisePrec :508, err_measures :826, and the next
    // warm start) is carried as AW += alpha * A p beside mu += alpha * p, from
    // the previous iteration's A x2; z1 = A x1_hat (:232) is one more
    // right-hand side of the first CG pass
    L.arec = R.arec && L.rec;
    if (L.arec) sx.AW = R.ax2;
    // the head start (pcg.cpp, ctx.h HeadStart): the Onsager solve (system 0)
    // takes its first CG step in the pass that starts the x2 solve, from
    // A.bern computed one iteration early (bern depends on (seed, it, marker)
    // only, P2); that pass also forms A.bern of the next iteration
    if (R.fuse && L.arec && R.onepass) STCHK(headstart_available(c, &L.hs_av));
    if (L.hs_av) {
        // slot it & 1 holds A.bern(it): the Onsager solve's A r, updated in
        // place by its CG steps; A.bern(it + 1) goes to the other slot
        L.hs.abern = R.hs_it == it ? R.abern + (it & 1) * ld : nullptr;
        if (it < R.prm.max_iter) {
            L.hs.xnext = R.bern_next;  // the probe of it + 1, formed by the prelude below
            L.hs.axnext = R.abern + ((it + 1) & 1) * ld;
        }
    }
    // the iteration's elementwise work before the CG solves, in one launch
    // (it replaces five: r2, bern, v, and the zeroed invQ (:496) and its W)
    vk::Prelude& pr = L.pr;
    pr.eta1 = R.eta1;
    pr.gam1 = R.gam1;
    pr.gam2 = R.gam2;
    pr.gamw = R.gamw;
    pr.x1 = x1;
    pr.r1 = R.r1;
    pr.atxy = R.atxy;
    pr.r2 = R.r2;
    pr.v = R.v;
    pr.seed = R.prm.seed;
    pr.it = it;
    pr.S = c->S;
    pr.sqrtMt = std::sqrt((double)c->Mt);
    pr.bern = R.bern;
    pr.bern_next = L.hs.xnext ? R.bern_next : nullptr;
    pr.zero[0] = R.invQ;
    pr.zero[1] = L.rec ? R.tmpM : nullptr;
    // where the solve starts on the device (no caller batch), the prelude rides
    // in its first launch (pcg_run's pre); else it is a launch of its own
    L.pre_in_cg = R.fuse && (L.hs_av || L.arec);
    return VAMPOMI_OK;
}

// ... and the scalars of a prelude queued ahead are the host's, bit for bit
static vampomi_status check_device_values(vampomi_ctx* c, VampRun& R, int it) {
    STCHK(check_device_mix(R));
    if (R.pre_ahead != it) return VAMPOMI_OK;
    R.pre_ahead = 0;
    const double diag = R.gamw * (double)(c->N - 1) / (double)c->N + R.gam2;  // pcg_run (:676-677)
    const double want[4] = {R.eta1, R.gam2, R.gamw, diag};
    if (std::memcmp(want, R.mixh + vk::kMixWords, sizeof want) != 0)
        return fail(VAMPOMI_ERR_STATE, "vamp: the prelude queued ahead formed other scalars than the host");
    return VAMPOMI_OK;
}

// one VAMP iteration (src/vamp.cpp:148-428)
extern "C" vampomi_status vampomi_vamp_step(vampomi_ctx* c, int* stopped) {
    CollScope cs_(c);
    if (!c || !c->run) return fail(VAMPOMI_ERR_STATE, "vampomi_vamp_begin not called");
    VampRun& R = *c->run;
    if (R.stopped || R.it >= R.prm.max_iter) {
        R.stopped = true;
        if (stopped) *stopped = 1;
        return VAMPOMI_OK;
    }
    HIPCHK(hipSetDevice(c->device));
    const auto t_step = std::chrono::steady_clock::now();
    if (R.probit) {
        STCHK(probit_step(c, R));
        R.ph_step_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_step).count();
        if (c->timing) resolve_timing(c);
        if (stopped) *stopped = R.stopped ? 1 : 0;
        return VAMPOMI_OK;
    }
    const int64_t M = c->M, N = c->N, Mt = c->Mt, ld = c->ld;
    const int it = ++R.it;
    vampomi_result* res = R.res;

    // ---------------- denoising (:177-232) ----------------
    if (!R.have_next) {
        if (it > R.prm.learn_prior_delay) STCHK(update_prior(c, R, R.mix, R.gam1, R.r1));  // :186-187
        std::swap(R.x1, R.x1p);  // x1_hat_prev = x1_hat (:203)
        DotBatch b(c);
        STCHK(denoise_into(c, R.mix, R.gam1, R.r1, R.x1, R.x1p, it > 1, R.prm.rho, R.x1d, b, &R.sum_d));
        STCHK(b.flush());
        R.alpha1 = R.sum_d / (double)Mt;  // :223
        if (!R.arec) {  // (arec: z1 rides in the first CG pass below)
            const double* xs[1] = {R.x1};
            STCHK(ax_dev(c, 1, xs, R.z1buf));  // z1 = Ax(x1_hat) (:232)
        }
        R.z1 = R.z1buf;
    } else {  // prefetched by iteration it-1 (see file comment, item 2)
        double* old = R.x1p;
        R.x1p = R.x1;
        R.x1 = R.x1n;
        R.x1n = old;
        R.mix = R.mix_next;
        R.alpha1 = R.alpha1_next;
        R.z1 = R.arec ? R.z1buf : R.nb3 + R.z1n_slot * ld;
    }
    R.passes_ref += 1;
    if (res && res->L_hist) res->L_hist[it - 1] = R.mix.L;
    R.eta1 = R.gam1 / R.alpha1;  // :230
    STCHK(write_bins(c, R));     // :235-249
    R.gam2 = smin(smax(R.eta1 - R.gam1, 1e-11), 1e11);  // :255-256
    DotBatch e1(c);
    if (!R.arec) STCHK(err_queue(c, R, R.x1, R.z1, e1, R.e1m, R.e1n, R.e1s));  // :272, flushed with the CG start
    R.params[0] = R.alpha1;
    R.params[1] = R.gam1;

    // ---------------- LMMSE (:289-350) ----------------
    // (r2 (:259-261), the probe bern (:295-296, P2) and v = gamw ATx(y) + gam2 r2
    // (:303-306) are formed by the prelude launch below, with the zero starts)
    R.passes_ref += 1;
    LmmseSetup L;
    STCHK(lmmse_setup(c, R, it, R.x1, L));
    CgSystem& sx = L.sx;
    CgSystem& so = L.so;
    const bool rec = L.rec, arec = L.arec, hs_av = L.hs_av;
    HeadStart& hs = L.hs;
    vk::Prelude& pr = L.pr;
    if (it == 1) {  // the zero starts of the first iteration
        HIPCHK(hipMemsetAsync(R.x2, 0, (size_t)std::max<int64_t>(M, 1) * 8, c->st));
        if (rec) HIPCHK(hipMemsetAsync(R.atx0, 0, (size_t)std::max<int64_t>(M, 1) * 8, c->st));
        if (arec) HIPCHK(hipMemsetAsync(R.ax2, 0, (size_t)ld * 8, c->st));
    }
    // the prelude and the solves' start of this iteration queued by the
    // previous one (its scalars from the device, R.pre_ahead)
    const PreMode pm = R.pre_ahead == it ? PreMode::queued : PreMode::normal;
    if (pm == PreMode::queued && !(L.pre_in_cg && R.fuse && hs_av))
        return fail(VAMPOMI_ERR_STATE, "vamp: the start queued ahead does not match this iteration's schedule");
    if (!L.pre_in_cg) HIPCHK(vk::prelude(M, pr, c->st));
    const auto t_solve = std::chrono::steady_clock::now();
    if (R.fuse && hs_av) {
        STCHK(pcg_run(c, {&so, &sx}, R.gamw, R.gam2, R.prm.CG_max_iter, R.prm.CG_err_tol, R.nsc, &R.passes_ref,
                      nullptr, R.x1, R.z1buf, true, nullptr, &hs, &pr, pm));
        R.hs_it = hs.xnext ? it + 1 : 0;
    } else if (R.fuse) {
        STCHK(pcg_run(c, {&sx, &so}, R.gamw, R.gam2, R.prm.CG_max_iter, R.prm.CG_err_tol, R.nsc, &R.passes_ref,
                      arec ? nullptr : &e1, arec ? R.x1 : nullptr, arec ? R.z1buf : nullptr, R.onepass, nullptr,
                      nullptr, arec ? &pr : nullptr));
        R.hs_it = 0;
    } else {
        STCHK(pcg_run(c, {&sx}, R.gamw, R.gam2, R.prm.CG_max_iter, R.prm.CG_err_tol, R.nsc, &R.passes_ref, &e1));
        STCHK(pcg_run(c, {&so}, R.gamw, R.gam2, R.prm.CG_max_iter, R.prm.CG_err_tol, R.nsc, &R.passes_ref, nullptr));
    }
    R.ph_solve_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_solve).count();
    STCHK(check_device_values(c, R, it));  // (the solves' flags came after the previous iteration's launches)
    if (res && res->cg_iters) res->cg_iters[it - 1] = sx.iters;
    if (res && res->ons_iters) res->ons_iters[it - 1] = so.iters;
    // r1 (:348-350): its own launch, or (the EM round below) formed by the
    // first EM round's kernel
    const bool next = R.fuse && it < R.prm.max_iter;
    const bool em_next = next && it + 1 > R.prm.learn_prior_delay;
    const bool r1_in_em = next && arec && em_next && R.prm.EM_max_iter >= 1;
    // chain: alpha2 -> eta2 -> gam1 (:341-346) are formed on the device from
    // the reduction's result (vk::G1Chain), so the EM round and the reductions
    // after it are queued without the host waiting for alpha2; the host forms
    // the same values from the same sum at the next flush.  Several ranks
    // (mr): the sums are final only after their all-reduce, so each value the
    // one-rank launches' last blocks form is formed by a one-thread launch
    // after it (vk::tail_post), all on the main stream (DotBatch::reduce_now);
    // VAMPOMI_MR_TAIL=0: the host waits at each level instead (round 4)
    const bool chain = r1_in_em && (!c->use_comm || c->mr_tail);
    const bool mr = chain && c->use_comm;
    const DotBatch::Group ga2{{T(R.bern, R.invQ)}, true, &R.a2};  // :498
    const double gam1_prev = R.gam1;
    auto host_gam1 = [&] {
        R.alpha2 = R.gam2 * R.a2;  // :498
        err_finish(R, R.e1m, R.e1n, R.e1s, 1);
        R.eta2 = R.gam2 / R.alpha2;  // :341
        R.gam1 = smin(smax(R.eta2 - R.gam2, 1e-11), 1e11);
        R.gam1 = R.prm.rho * R.gam1 + (1 - R.prm.rho) * gam1_prev;  // :346
    };
    // ---- prefetch: denoising of iteration it+1 (discarded if the stop fires) ----
    DotBatch fin(c);
    double* dsc = c->scal + SL_CHAIN;
    // updateNoisePrec's two sums (:508-521) and the NMSE sums (:409-413); with
    // arec they ride in err_measures' launches (one per vector length)
    const DotBatch::Group gtc{{T(R.bern, R.tmpM)}, true, &R.tc};  // <u, A^T A invQ>
    const DotBatch::Group gtn{{T(R.ax2, c->y, vk::DIFF2)}, false, &R.tn};  // l2_norm2(temp, 0), temp = A x2 - y
    const DotBatch::Group gnm{{T(R.x1p, R.x1, vk::DIFF2), T(R.x1p, R.x1p)}, true, R.nm};
    if (chain) {
        // every reduction of the iteration's tail reads vectors the solves have
        // just finished: err_measures of x1 (:272) and of x2 (:365, A x2 from
        // the CG) with the sums above: 10 terms over M and 11 over N, in ONE
        // launch (vk::dots2); each term's sum is the same fixed-order reduction
        // as in its own launch (the geometry depends on the length only)
        std::vector<DotBatch::Group> gm{ga2}, gn;
        err_groups(c, R, R.x1, R.z1, R.e1m, R.e1n, R.e1s, gm, gn);
        gm.push_back(gtc);
        gm.push_back(gnm);
        gn.push_back(gtn);
        err_groups(c, R, R.x2, R.ax2, R.e2m, R.e2n, R.e2s, gm, gn);
        // alpha2 -> eta2 -> gam1 in the M launch's last block (vk::G1Chain)
        vk::G1Chain g1;
        g1.gam2 = R.gam2;
        g1.rho = R.prm.rho;
        g1.gam1_prev = gam1_prev;
        g1.out = dsc;
        // (tc and tn also into device memory, for the next prelude's scalars: vk::PreOut)
        if (!mr) {
            STCHK(fin.add_pair(M, gm, &g1, &R.a2, {{&R.tc, dsc + 9}}, N, gn, {{&R.tn, dsc + 8}}));  // one launch
        } else {
            STCHK(fin.add_pair(M, gm, nullptr, nullptr, {}, N, gn, {}));
            STCHK(fin.reduce_now());
            vk::TailPost t;
            t.mode = 0;
            t.src = fin.dev_slot(&R.a2);
            t.g1 = g1;
            t.cp_src[0] = fin.dev_slot(&R.tc);
            t.cp_dst[0] = dsc + 9;
            t.cp_src[1] = fin.dev_slot(&R.tn);
            t.cp_dst[1] = dsc + 8;
            HIPCHK(vk::tail_post(t, c->st));
        }
    } else {
        DotBatch b(c);
        if (arec)
            STCHK(err_queue(c, R, R.x1, R.z1, b, R.e1m, R.e1n, R.e1s, {ga2}));  // :272
        else
            STCHK(b.add_many(M, {ga2}));
        STCHK(b.flush());
        host_gam1();
        if (!r1_in_em) HIPCHK(vk::lincomb_div(M, R.eta2, R.x2, R.gam2, R.r2, R.gam1, R.r1, c->st));
    }
    R1From r1from{R.x2, R.r2, R.eta2, R.gam2, R.gam1};
    if (chain) r1from.dsc = dsc;
    // devem (the chain, one EM round): the EM round's launch also forms the
    // update of the mixture (vk::EmArgs.upd), and the next denoising follows
    // with no host wait between them; the host forms the same mixture from the same
    // sums at the iteration's one flush, and checks it against the device's,
    // bit for bit
    const bool devem = chain && R.prm.EM_max_iter == 1;
    // ahead (devem): iteration it+1's prelude and solves' start are queued at
    // the end of this iteration, its scalars formed by the next denoising's
    // launch (vk::PreOut): the GPU runs it while the host waits for this
    // iteration's flush, instead of idling from the end of this iteration's
    // last launch to the host's first launch of the next.  If the stop fires,
    // it has only written vectors that no later read depends on (r2, v, bern,
    // the CG start, the zero starts)
    LmmseSetup A;
    vk::PreOut po;
    bool ahead = false;
    if (devem && R.pre_ahead_on && next) {
        const bool had = R.have_next;
        R.have_next = true;  // (it + 1's view: its x1_hat is x1n)
        const vampomi_status st = lmmse_setup(c, R, it + 1, R.x1n, A);
        R.have_next = had;
        STCHK(st);
        po.tn = dsc + 8;  // (device copies, above)
        po.tc = dsc + 9;
        po.Mt = (double)Mt;
        po.N = (double)N;
        po.out = dsc + 3;
        po.mirror = R.mixh_dev + vk::kMixWords;
        ahead = A.pre_in_cg && R.fuse && A.hs_av && A.sx.atx0 && po.tn && po.tc;
        A.pr.dev.scal = po.out;
    }
    EmState em;
    if (next) R.mix_next = R.mix;
    if (next && arec) {  // iteration it+1's EM sums, queued before these reductions
        if (em_next) {
            vk::EmUpd eu;
            eu.Mt = Mt;
            eu.learn_vars = R.prm.learn_vars;
            eu.merge_vars_thr = R.prm.merge_vars_thr;
            eu.out = R.mixw;
            eu.mirror = R.mixh_dev;
            STCHK(em_begin(c, em_params(R), R.mix_next, R.gam1, R.r1, fin, em, r1_in_em ? &r1from : nullptr,
                           devem && !mr ? &eu : nullptr));
            if (devem && mr) {  // the round's update of the mixture, from its all-reduced sums
                STCHK(fin.reduce_now());
                vk::TailPost t;
                t.mode = 1;
                t.src = fin.dev_slot(em.sums);
                t.L = R.mix_next.L;
                for (int j = 0; j < R.mix_next.L; ++j) t.vars[j] = R.mix_next.vars[j];
                t.upd = eu;
                HIPCHK(vk::tail_post(t, c->st));
            }
            if (devem) {
                STCHK(denoise_into(c, R.mix_next, R.gam1, R.r1, R.x1n, R.x1, true, R.prm.rho, R.x1d, fin, &R.sum_d,
                                   R.mixw, dsc, ahead && !mr ? &po : nullptr));
                if (ahead && mr) {  // the next prelude's scalars, from the all-reduced sum of x1d
                    STCHK(fin.reduce_now());
                    vk::TailPost t;
                    t.mode = 2;
                    t.src = fin.dev_slot(&R.sum_d);
                    t.po = po;
                    t.gam1dev = dsc;
                    HIPCHK(vk::tail_post(t, c->st));
                }
            }
        }
    }
    if (next && !arec) {  // the pass below carries the next z1 = A x1_hat: denoise first
        if (em_next) STCHK(update_prior(c, R, R.mix_next, R.gam1, R.r1));
        STCHK(denoise_into(c, R.mix_next, R.gam1, R.r1, R.x1n, R.x1, true, R.prm.rho, R.x1d, fin, &R.sum_d));
    }

    // ---- updateNoisePrec (:504-529) + the next z1 in the same pass ----
    const double* ax2 = R.nb3;  // A.x2_hat
    bool shared = false;
    if (arec) {  // no pass: A x2 came with the CG, the next z1 comes with the next CG
        ax2 = R.ax2;
        R.passes_ref += 3;  // :508, :518, :519
        shared = true;
    } else if (rec) {  // A.x2 and the next z1 in one pass; the A^T products came with the CG
        const double* xs[2] = {R.x2, R.x1n};
        STCHK(ax_dev(c, next ? 2 : 1, xs, R.nb3));
        R.z1n_slot = 1;
        R.passes_ref += 2;
        STCHK(fin.add({T(R.nb3, c->y, vk::DIFF2)}, N, false, &R.tn));  // l2_norm2(temp, 0)
        R.passes_ref += 1;
        STCHK(fin.add({T(R.bern, R.tmpM)}, M, true, &R.tc));  // <u, A^T A invQ>
    } else {
        const double* xs[3] = {R.x2, R.invQ, R.x1n};
        STCHK(ax_dev(c, next ? 3 : 2, xs, R.nb3));
        R.z1n_slot = 2;
        R.passes_ref += 2;
        STCHK(fin.add({T(R.nb3, c->y, vk::DIFF2)}, N, false, &R.tn));  // l2_norm2(temp, 0)
        const double* u[2] = {R.nb3 + ld, R.nb3};  // A.invQ (trace), A.x2 (next warm start)
        double* o[2] = {R.tmpM, R.atx0};
        STCHK(atx_dev(c, next ? 2 : 1, u, o, 0, 0.0, 0.0, nullptr));
        R.passes_ref += 1;
        STCHK(fin.add({T(R.bern, R.tmpM)}, M, true, &R.tc));
    }
    // (shared: the NMSE sums (:409-413) too; they read x1 and x1_prev, which
    // the prefetched denoising below does not write; chain: queued above)
    if (shared && !chain)
        STCHK(err_queue(c, R, R.x2, ax2, fin, R.e2m, R.e2n, R.e2s, {gtc, gnm}, {gtn}));  // :365 (A.x2_hat of :826)
    else if (!shared)
        STCHK(err_queue(c, R, R.x2, ax2, fin, R.e2m, R.e2n, R.e2s));
    R.passes_ref += 1;
    // Iteration it+1's EM sums share these reductions' all-reduce and host
    // wait; then its denoiser (g1, g1d, sum of g1d) shares the NMSE sums'
    // (several EM rounds, or VAMPOMI_MR_TAIL=0 on several ranks: the host's
    // mixture update between them)
    if (next && arec && em_next && !devem) {
        STCHK(fin.flush());
        if (chain) host_gam1();  // (the device formed the same values for the EM round)
        STCHK(em_finish(c, em_params(R), R.mix_next, R.gam1, R.r1, em));
    }
    if (next && arec && !devem)
        STCHK(denoise_into(c, R.mix_next, R.gam1, R.r1, R.x1n, R.x1, true, R.prm.rho, R.x1d, fin, &R.sum_d));
    if (!shared) STCHK(fin.add_many(M, {gnm}));  // NMSE (:409-413)
    // iteration it+1's prelude and solves' start, queued now (set up above)
    if (ahead) {
        STCHK(pcg_run(c, {&A.so, &A.sx}, 0.0, 0.0, R.prm.CG_max_iter, R.prm.CG_err_tol, R.nsc, nullptr, nullptr,
                      R.x1n, R.z1buf, true, nullptr, &A.hs, &A.pr, PreMode::ahead));
        R.pre_ahead = it + 1;
    }
    STCHK(fin.flush());
    if (devem) {
        host_gam1();  // (the device formed the same values)
        STCHK(em_finish(c, em_params(R), R.mix_next, R.gam1, R.r1, em));
        R.mix_expect = R.mix_next;  // checked after the next solves (or at the end)
        R.mix_pending = true;
    }
    const double trace_corr = R.tc * (double)Mt;  // :521
    if (R.prm.verbosity >= 1 && c->rank == 0)
        std::printf("l2_norm2(temp) / N = %g\ntrace_correction / N = %g\n", R.tn / (double)N, trace_corr / (double)N);
    R.gamw = (double)N / (R.tn + trace_corr);  // :528
    err_finish(R, R.e2m, R.e2n, R.e2s, 2);
    R.params[2] = R.alpha2;
    R.params[3] = R.gam2;
    R.params[4] = R.gamw;
    if (res && res->params) std::memcpy(res->params + (int64_t)(it - 1) * 5, R.params, 5 * sizeof(double));
    if (res && res->metrics) std::memcpy(res->metrics + (int64_t)(it - 1) * 6, R.metrics, 6 * sizeof(double));
    if (R.write && c->rank == 0) {  // :388-393
        write_row(R, R.p_params, it, R.params, 5);
        write_row(R, R.p_metrics, it, R.metrics, 6);
    }
    if (R.prm.verbosity >= 1 && c->rank == 0)
        std::printf("it %d: alpha1 %.6g gam1 %.6g alpha2 %.6g gam2 %.6g gamw %.6g L %d cg %d/%d\n", it, R.alpha1,
                    R.gam1, R.alpha2, R.gam2, R.gamw, R.mix.L, sx.iters, so.iters);

    // stopping criteria (:409-423)
    const double NMSE = std::sqrt(R.nm[0] / R.nm[1]);
    if ((it > 1 && NMSE < R.prm.stop_criteria_thr) || it >= R.prm.max_iter) R.stopped = true;
    STCHK(end_iteration_io(c, R));
    R.have_next = next && !R.stopped;
    if (R.have_next) R.alpha1_next = R.sum_d / (double)Mt;
    if (res) {
        res->iterations_run = it;
        res->a_passes_ref = R.passes_ref;
        res->a_passes_exec = c->stats.a_passes_exec;
    }
    if (c->timing) resolve_timing(c);
    if (stopped) *stopped = R.stopped ? 1 : 0;
    R.ph_step_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_step).count();
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_step_phases(vampomi_ctx* c, double* solve_s, double* step_s) {
    if (!c || !c->run) return fail(VAMPOMI_ERR_STATE, "vampomi_vamp_begin not called");
    if (solve_s) *solve_s = c->run->ph_solve_s;
    if (step_s) *step_s = c->run->ph_step_s;
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_vamp_end(vampomi_ctx* c) {
    if (!c || !c->run) return fail(VAMPOMI_ERR_STATE, "vampomi_vamp_begin not called");
    VampRun& R = *c->run;
    vampomi_result* res = R.res;
    if (R.writer) {  // (a run ended before its last iteration: the writes queued so far)
        std::string msg;
        if (R.writer->drain(&msg)) {
            c->run.reset();
            return fail(VAMPOMI_ERR_IO, msg);
        }
    }
    if (R.mix_pending) {  // the last device EM update (one rank: a stream sync)
        STCHK(host_sync(c));
        const vampomi_status s = check_device_mix(R);
        if (s != VAMPOMI_OK) {
            c->run.reset();
            return s;
        }
    }
    if (res) {
        if (res->x1_final && c->M > 0) {
            HIPCHK(hipMemcpyAsync(res->x1_final, R.x1, (size_t)c->M * 8, hipMemcpyDeviceToHost, c->st));
            STCHK(host_sync(c));
            const double sqrtN = std::sqrt((double)c->N);
            if (!R.probit)  // linear returns x1_hat_scaled (:437), probit x1_hat (src/vamp_probit.cpp:465)
                for (int64_t i = 0; i < c->M; ++i) res->x1_final[i] = res->x1_final[i] / sqrtN;
        }
        res->L_final = R.mix.L;
        for (int j = 0; j < R.mix.L; ++j) {
            res->probs_final[j] = R.mix.probs[j];
            res->vars_final[j] = R.mix.vars[j] / (double)c->N;
        }
        res->a_passes_ref = R.passes_ref;
        res->a_passes_exec = c->stats.a_passes_exec;
    }
    if (c->timing) resolve_timing(c);
    c->run.reset();
    return VAMPOMI_OK;
}

extern "C" vampomi_status vampomi_infere(vampomi_ctx* c, const vampomi_params* p, vampomi_result* r) {
    CollScope cs_(c);
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
    p->batch_rhs = 4;
    p->model = "linear";
}

// vamp::updatePrior (src/vamp.cpp:531-643) on its own: EM for the
// spike-and-slab prior from r1 (this shard's slice) at noise precision gam1,
// then the merging of close variances.  vars are multiplied by N, as the
// reference keeps them (src/vamp.cpp:87-88).  COLLECTIVE.
extern "C" vampomi_status vampomi_update_prior(vampomi_ctx* c, const double* r1, double gam1, int* L, double* probs,
                                               double* vars, int EM_max_iter, double EM_err_thr, int learn_vars,
                                               double merge_vars_thr, int mem) {
    CollScope cs_(c);
    if (!c || !L || !probs || !vars || (!r1 && c->M > 0)) return fail(VAMPOMI_ERR_ARG, "null argument");
    if (*L < 1 || *L > VAMPOMI_MAX_L) return fail(VAMPOMI_ERR_ARG, "number of mixture components out of range");
    HIPCHK(hipSetDevice(c->device));
    double* rin = c->mbuf;
    if (c->M > 0)
        HIPCHK(hipMemcpyAsync(rin, r1, (size_t)c->M * 8,
                              mem == VAMPOMI_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, c->st));
    Mixture m;
    m.L = *L;
    for (int j = 0; j < m.L; ++j) {
        m.probs[j] = probs[j];
        m.vars[j] = vars[j];
    }
    const EmParams ep{EM_max_iter, EM_err_thr, learn_vars, merge_vars_thr, 0};
    STCHK(update_prior(c, ep, m, gam1, rin));
    *L = m.L;
    for (int j = 0; j < m.L; ++j) {
        probs[j] = m.probs[j];
        vars[j] = m.vars[j];
    }
    return VAMPOMI_OK;
}
