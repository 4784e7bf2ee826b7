// probit.cpp — the gVAMPomi probit model on the device
// (vamp::infere_bin_class, src/vamp_probit.cpp:19-467).
//
// The x side (g1/g1d, updatePrior, the two CG solves) reuses the linear
// model's kernels; the z side is one N-vector kernel (g1_bin_class with the
// reference's erfcx and the sum of g1d_bin_class) plus elementwise updates.
// The reference runs, per iteration, A.(x1/sqrtN) (:271), A^T p2 (:300),
// 2(k1+k2) CG passes (:307, :311), A.x2 (:352) and A.(x2/sqrtN) (:403).
// Here, with every value bitwise unchanged (tests check batch_rhs=0 vs 1):
//   1. the x2 solve and the Onsager solve share each pass (pcg.cpp);
//   2. A.x2, A.(x2/sqrtN) and the NEXT iteration's A.(x1/sqrtN) are one K=3
//      pass: x1 of iteration it+1 is g1(r1, gam1) damped with x1 of it, and
//      r1, gam1 and the mixture are final once r1 is updated (:337-346);
//      the mixture update of it+1 (:139) runs after g1 there, so it is done
//      at the start of step it+1 exactly as in the reference.
// true_g = A.(true_signal*sqrtN) (:46) is never read; it is counted in
// a_passes_ref and not computed.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>

#include "ctx.h"
#include "hostio.h"
#include "run.h"

namespace {
constexpr double kGamMin = 1e-11, kGamMax = 1e11;  // src/vamp.hpp:33-34
double clip(double v) { return smin(smax(v, kGamMin), kGamMax); }
}  // namespace

vampomi_status probit_begin(vampomi_ctx* c, VampRun& R) {
    const size_t M = (size_t)std::max<int64_t>(c->M, 1), ld = (size_t)c->ld;
    for (double** p : {&R.p1, &R.p2, &R.z1h}) {
        STCHK(dev_alloc(p, ld));
        HIPCHK(hipMemsetAsync(*p, 0, ld * 8, c->st));
    }
    for (double** p : {&R.x1s, &R.x1sn, &R.x2s}) STCHK(dev_alloc(p, M));
    HIPCHK(vk::scale_vec(c->M, R.ts, c->sqrtN, c->st));  // true_signal_scaled (:41-44)
    R.passes_ref += 1;                                    // true_g (:46)
    HIPCHK(vk::probit_p1(R.prm.seed, c->N, R.p1, c->st));  // p1 (:53, P2)
    HIPCHK(hipMemsetAsync(R.r1, 0, M * 8, c->st));         // r1 = r2 = 0 (:56-57)
    R.tau1 = R.gam1;                                       // :35
    R.alpha1 = 0;                                          // :58
    if (R.write) {
        R.p_metrics = R.out_dir + "/" + R.out_name + "_metrics.csv";
        R.p_params = R.out_dir + "/" + R.out_name + "_params.csv";
        R.p_prior = R.out_dir + "/" + R.out_name + "_prior.csv";
        // setup_io (src/vamp.cpp:854-882); infere_bin_class writes no header
        if (c->rank == 0 &&
            !(vio::csv_create(R.p_metrics) && vio::csv_create(R.p_params) && vio::csv_create(R.p_prior))) {
            R.io_err = true;
            R.io_msg = "cannot create output CSV files in " + R.out_dir;
        }
        STCHK(agree_io(c, R));
    }
    return VAMPOMI_OK;
}

static void confusion_finish(const double* cnt, double* out) {  // :273-282, :653-663
    const double TP = cnt[0], TN = cnt[1], FP = cnt[2], FN = cnt[3];
    out[0] = TP;
    out[1] = TN;
    out[2] = FP;
    out[3] = FN;
    out[4] = (double)((int64_t)TP + (int64_t)TN) / (double)((int64_t)TP + (int64_t)TN + (int64_t)FP + (int64_t)FN);
}

vampomi_status probit_step(vampomi_ctx* c, VampRun& R) {
    const int64_t M = c->M, N = c->N, Mt = c->Mt, ld = c->ld;
    const int it = ++R.it;
    vampomi_result* res = R.res;
    const double rho = R.prm.rho, sqrtN = std::sqrt((double)N);

    // ---------------- denoising x (:104-198) ----------------
    const double alpha1_prev = R.alpha1;  // :105
    double alpha1_raw;
    const double* zx1;  // A.(x1_hat/sqrtN) (:271)
    if (!R.have_next) {
        std::swap(R.x1, R.x1p);  // x1_hat_prev = x1_hat (:104)
        DotBatch b(c);
        STCHK(denoise_into(c, R.mix, R.gam1, R.r1, R.x1, R.x1p, it > 1, rho, R.x1d, b, &R.sum_d));
        STCHK(b.flush());
        alpha1_raw = R.sum_d / (double)Mt;  // :127-129
        HIPCHK(vk::div_scalar(M, R.x1, sqrtN, R.x1s, c->st));
        const double* xs[1] = {R.x1s};
        STCHK(ax_dev(c, 1, xs, R.z1buf));
        zx1 = R.z1buf;
    } else {  // prefetched by iteration it-1 (file comment, item 2)
        double* old = R.x1p;
        R.x1p = R.x1;
        R.x1 = R.x1n;
        R.x1n = old;
        std::swap(R.x1s, R.x1sn);
        alpha1_raw = R.alpha1_next;
        zx1 = R.nb3 + 2 * ld;
    }
    R.passes_ref += 1;
    R.eta1 = R.gam1 / alpha1_raw;                                        // :130
    if (it > 1 && R.em_head != it) STCHK(update_prior(c, R, R.mix, R.gam1, R.r1));  // :139, after g1/g1d
    if (res && res->L_hist) res->L_hist[it - 1] = R.mix.L;
    R.alpha1 = it > 1 ? rho * alpha1_raw + (1 - rho) * alpha1_prev : alpha1_raw;  // :160-165
    STCHK(write_bins(c, R));                                             // :168-186
    R.gam2 = clip(R.eta1 - R.gam1);                                      // :194
    HIPCHK(vk::lincomb_div(M, R.eta1, R.x1, R.gam1, R.r1, R.gam2, R.r2, c->st));  // :197-198

    // ---------------- denoising z (:202-253) + accuracy of x1 (:189, :271-282) ----------------
    double bsum = 0, cnt1[4] = {}, xc1[3] = {};
    // (queued by iteration it-1 with its last batch, z_head: the same launches on the same inputs)
    auto queue_z = [&](DotBatch& b, const double* x1v, const double* zx, double* bs, double* cnt, double* xc) {
        vk::RedOut ro{};
        STCHK(b.sink(1, false, bs, &ro));  // y, p1 replicated: local sum
        HIPCHK(vk::probit_denoise(N, R.p1, c->y, R.tau1, R.z1h, ro, c->st));
        STCHK(b.sink(4, false, cnt, &ro));
        HIPCHK(vk::probit_confusion(N, 1, zx, ld, c->y, ro, c->st));
        STCHK(b.add({T(x1v, R.ts), T(x1v, x1v), T(R.ts, R.ts)}, M, true, xc));
        return VAMPOMI_OK;
    };
    if (R.z_head == it) {
        bsum = R.zh_bsum;
        std::memcpy(cnt1, R.zh_cnt, sizeof cnt1);
        std::memcpy(xc1, R.zh_xc, sizeof xc1);
    } else {
        DotBatch b(c);
        STCHK(queue_z(b, R.x1, zx1, &bsum, cnt1, xc1));
        STCHK(b.flush());
    }
    R.beta1 = bsum;
    if (R.beta1 >= N) R.beta1 = N - 1.0;  // :234-236
    R.beta1 /= N;
    HIPCHK(vk::lincomb_div(N, 1.0, R.z1h, R.beta1, R.p1, 1 - R.beta1, R.p2, c->st));  // :250-251
    R.tau2 = R.tau1 * (1 - R.beta1) / R.beta1;                                           // :253
    R.params[0] = R.alpha1;
    R.params[1] = R.beta1;
    R.params[2] = R.gam1;
    R.params[3] = R.tau1;
    confusion_finish(cnt1, R.metrics);
    R.metrics[5] = xc1[0] / std::sqrt(xc1[1] * xc1[2]);

    // ---------------- LMMSE (:297-385) ----------------
    if (R.bern_it != it)  // (drawn at the end of iteration it-1 when its A.x pass carried A.bern)
        HIPCHK(vk::bernoulli(R.prm.seed, it, c->S, M, std::sqrt((double)Mt), R.bern, c->st));  // :297-298 (P2)
    R.bern_it = it;
    // v = tau2*A^T p2 + gam2*r2 (:300-303).  Both CG solves start from zero, so
    // r0 = v and the x2 solve's first A.x pass needs A v: with the one-pass
    // operator ONE launch forms v (as d = tau*A^T q + gam2*p with q = p2/1,
    // p = r2) and A v from one read of X; the Onsager solve's A r0 = A.bern
    // came with the previous iteration's last A.x pass.  2 + max(k1, k2) reads
    // of X per iteration instead of 3 + max(k1, k2)
    const double* ar0[2] = {nullptr, nullptr};
    bool merged = R.onepass && R.fuse && c->have_X;
    if (merged) {
        STCHK(op_prepare(c));
        merged = c->op_ok;
    }
    if (merged) {
        vk::OpArgs a{};
        a.ar.p[0] = R.p2;  // ld-padded, zero pads
        a.p.p[0] = R.r2;
        a.d.p[0] = R.v;
        a.diag = 1.0;
        a.tau = R.tau2;
        a.gam2 = R.gam2;
        STCHK(op_dev(c, 1, a, nullptr));  // COLLECTIVE (the A v all-reduce)
        R.passes_ref += 1;
        ar0[0] = c->op_nvec + (int64_t)2 * vk::kMaxRhs * ld;  // A v, read by pcg_run before any other launch
        if (R.abern_it == it) ar0[1] = R.nb3 + 3 * ld;
    } else {
        const double* u[1] = {R.p2};
        double* o[1] = {R.tmpM};
        STCHK(atx_dev(c, 1, u, o, 0, 0.0, 0.0, nullptr));  // :300
        R.passes_ref += 1;
        HIPCHK(vk::axpby(M, R.tau2, R.tmpM, R.gam2, R.r2, R.v, c->st));  // :302-303
    }
    CgSystem sx{}, so{};
    sx.v = R.v;
    sx.mu = R.x2;  // zero start (:307)
    sx.r = R.cgw[0];
    sx.z = R.cgw[1];
    sx.p = R.cgw[2];
    sx.d = R.cgw[3];
    so.v = R.bern;
    so.mu = R.invQ;  // g2d_onsager(gam2, tau2) (:311)
    so.onsager = true;
    so.r = R.cgw[4];
    so.z = R.cgw[5];
    so.p = R.cgw[6];
    so.d = R.cgw[7];
    const size_t Mb = (size_t)std::max<int64_t>(M, 1) * 8;
    HIPCHK(hipMemsetAsync(R.x2, 0, Mb, c->st));
    HIPCHK(hipMemsetAsync(R.invQ, 0, Mb, c->st));
    const auto t_solve = std::chrono::steady_clock::now();
    if (R.fuse) {
        STCHK(pcg_run(c, {&sx, &so}, R.tau2, R.gam2, R.prm.CG_max_iter, R.prm.CG_err_tol, R.nsc, &R.passes_ref,
                      nullptr, nullptr, nullptr, R.onepass, merged ? ar0 : nullptr));
    } else {
        STCHK(pcg_run(c, {&sx}, R.tau2, R.gam2, R.prm.CG_max_iter, R.prm.CG_err_tol, R.nsc, &R.passes_ref, nullptr));
        STCHK(pcg_run(c, {&so}, R.tau2, R.gam2, R.prm.CG_max_iter, R.prm.CG_err_tol, R.nsc, &R.passes_ref, nullptr));
    }
    R.ph_solve_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_solve).count();
    if (res && res->cg_iters) res->cg_iters[it - 1] = sx.iters;
    if (res && res->ons_iters) res->ons_iters[it - 1] = so.iters;
    double xc2[3] = {};
    {
        DotBatch b(c);
        STCHK(b.add({T(R.bern, R.invQ)}, M, true, &R.a2));
        STCHK(b.add({T(R.x2, R.ts), T(R.x2, R.x2), T(R.ts, R.ts)}, M, true, xc2));  // :324
        STCHK(b.flush());
    }
    R.alpha2 = R.gam2 * R.a2;
    HIPCHK(vk::div_scalar(M, R.x2, sqrtN, R.x2s, c->st));  // x2_hat_s (:318-320)
    R.eta2 = R.gam2 / R.alpha2;                             // :326
    HIPCHK(vk::lincomb_div(M, 1.0, R.x2, R.alpha2, R.r2, 1 - R.alpha2, R.r1, c->st));  // :337-338
    R.gam1 = clip(R.gam2 * (1 - R.alpha2) / R.alpha2);                                  // :345-346

    // ---- prefetch: x1 of iteration it+1 (discarded if the stop fires) ----
    const bool next = R.fuse && it < R.prm.max_iter;
    DotBatch fin(c);
    if (next) {
        STCHK(denoise_into(c, R.mix, R.gam1, R.r1, R.x1n, R.x1, true, rho, R.x1d, fin, &R.sum_d));
        HIPCHK(vk::div_scalar(M, R.x1n, sqrtN, R.x1sn, c->st));
    }
    // ---- A.x2 (:352), A.x2_hat_s (:403) [+ the next A.(x1/sqrtN) and, with the
    // merged launch, the next iteration's probe and its A.bern]: one pass ----
    {
        const bool carry = next && merged;
        if (carry) {  // bern (of this iteration) was last read by the a2 batch above
            HIPCHK(vk::bernoulli(R.prm.seed, it + 1, c->S, M, std::sqrt((double)Mt), R.bern, c->st));
            R.bern_it = it + 1;
            R.abern_it = it + 1;
        }
        const double* xs[4] = {R.x2, R.x2s, R.x1sn, R.bern};
        STCHK(ax_dev(c, carry ? 4 : next ? 3 : 2, xs, R.nb3));
        R.passes_ref += 2;
    }
    R.beta2 = (double)Mt / N * (1 - R.alpha2);                                            // :354
    HIPCHK(vk::lincomb_div(N, 1.0, R.nb3, R.beta2, R.p2, 1 - R.beta2, R.p1, c->st));      // :366-368
    R.tau1 = clip(R.tau2 * (1 - R.beta2) / R.beta2);                                      // :374-376
    double cnt2[4] = {};
    {
        vk::RedOut ro{};
        STCHK(fin.sink(4, false, cnt2, &ro));
        HIPCHK(vk::probit_confusion(N, 1, R.nb3 + ld, ld, c->y, ro, c->st));  // :403-408
    }
    STCHK(fin.add({T(R.x1p, R.x1, vk::DIFF2), T(R.x1p, R.x1p)}, M, true, R.nm));  // NMSE (:444-448)
    // iteration it+1's head, queued with this iteration's last reductions so
    // that it needs no host waits of its own (discarded if the stop fires):
    // its updatePrior (:139) reads r1 and gam1 of this iteration and runs
    // after its g1 / g1d (the prefetched denoising above used this mixture);
    // its z-side denoising (:202-253) reads p1 and tau1 formed just above, and
    // its accuracy counts A.(x1n/sqrtN), which the pass above carried
    EmState em_h;
    const bool em_h_on = next && R.prm.EM_max_iter >= 1;
    if (em_h_on) STCHK(em_begin(c, em_params(R), R.mix, R.gam1, R.r1, fin, em_h));
    if (next) STCHK(queue_z(fin, R.x1n, R.nb3 + 2 * ld, &R.zh_bsum, R.zh_cnt, R.zh_xc));
    STCHK(fin.flush());
    R.params[4] = R.alpha2;
    R.params[5] = R.beta2;
    R.params[6] = R.gam2;
    R.params[7] = R.tau2;
    confusion_finish(cnt2, R.metrics + 6);
    R.metrics[11] = xc2[0] / std::sqrt(xc2[1] * xc2[2]);
    // prior row (:423-428): L, probs, vars (multiplied by N)
    double prior[1 + 2 * VAMPOMI_MAX_L] = {};
    int np = 0;
    prior[np++] = (double)R.mix.L;
    for (int j = 0; j < R.mix.L; ++j) prior[np++] = R.mix.probs[j];
    for (int j = 0; j < R.mix.L; ++j) prior[np++] = R.mix.vars[j];
    if (res && res->params) std::memcpy(res->params + (int64_t)(it - 1) * 8, R.params, 8 * sizeof(double));
    if (res && res->metrics) std::memcpy(res->metrics + (int64_t)(it - 1) * 12, R.metrics, 12 * sizeof(double));
    if (res && res->prior_hist) std::memcpy(res->prior_hist + (int64_t)(it - 1) * (1 + 2 * VAMPOMI_MAX_L), prior,
                                            sizeof prior);
    if (R.write && c->rank == 0) {  // :430-435
        write_row(R, R.p_params, it, R.params, 8);
        write_row(R, R.p_metrics, it, R.metrics, 12);
        write_row(R, R.p_prior, it, prior, np);
    }
    if (R.prm.verbosity >= 1 && c->rank == 0)
        std::printf("it %d: alpha1 %.6g beta1 %.6g gam1 %.6g tau1 %.6g alpha2 %.6g beta2 %.6g L %d cg %d/%d\n", it,
                    R.alpha1, R.beta1, R.gam1, R.tau1, R.alpha2, R.beta2, R.mix.L, sx.iters, so.iters);

    // stopping criteria (:444-458)
    const double NMSE = std::sqrt(R.nm[0] / R.nm[1]);
    if ((it > 1 && NMSE < R.prm.stop_criteria_thr) || it >= R.prm.max_iter) R.stopped = true;
    STCHK(end_iteration_io(c, R));  // write_bins' and the rows' failures, on every rank at once
    R.have_next = next && !R.stopped;
    if (R.have_next) {  // (after this iteration's prior row: the update is iteration it+1's)
        if (em_h_on) {
            STCHK(em_finish(c, em_params(R), R.mix, R.gam1, R.r1, em_h));
            R.em_head = it + 1;
        }
        R.z_head = it + 1;
    }
    if (R.have_next) R.alpha1_next = R.sum_d / (double)Mt;
    if (res) {
        res->iterations_run = it;
        res->a_passes_ref = R.passes_ref;
        res->a_passes_exec = c->stats.a_passes_exec;
    }
    return VAMPOMI_OK;
}
