// pcg.cpp — vamp::precondCG_solver (src/vamp.cpp:664-757) for several
// independent systems (tau*A^T A + gam2*I) mu = v that share the operator.
//
// Per CG step and per still-active system, exactly the reference's scalar
// recurrences: alpha = <r,z>/<d,p>; mu += alpha p; [Onsager stop on
// gam2<v,mu>]; r -= d alpha; z = r/diag; beta = pow(<r,z>_old,-1)*<r,z>_new;
// p = z + beta p; stop when ||r||/||v|| < tol.  What is shared is the pass
// over X: lmmse_mult(p) for all active systems is one A.x and one A^T.u
// launch with K right-hand sides, so two systems cost 2*max(k1, k2) passes
// instead of 2*(k1 + k2), with every iterate bitwise equal to a solo solve.
#include <cmath>

#include "ctx.h"

vampomi_status pcg_run(vampomi_ctx* c, const std::vector<CgSystem*>& sys, double tau, double gam2, int max_iter,
                       double tol, double* nscratch, int64_t* ref_passes, DotBatch* init) {
    const int64_t M = c->M, N = c->N;
    const double diag = tau * (double)(N - 1) / (double)N + gam2;  // :676-677
    const int K = (int)sys.size();
    if (K < 1 || K > vk::kMaxRhs) return fail(VAMPOMI_ERR_ARG, "pcg: 1..4 systems");
    // initial residual r = v - lmmse_mult(mu0)  (:681-684)
    {
        std::vector<CgSystem*> nz;
        for (auto* s : sys) {
            if (s->mu0_nonzero && !s->atx0) nz.push_back(s);
            if (s->mu0_nonzero && ref_passes) *ref_passes += 2;
        }
        if (!nz.empty()) {
            const double* vv[vk::kMaxRhs];
            double* dd[vk::kMaxRhs];
            for (size_t k = 0; k < nz.size(); ++k) {
                vv[k] = nz[k]->mu;
                dd[k] = nz[k]->d;
            }
            STCHK(lmmse_dev(c, (int)nz.size(), vv, dd, tau, gam2, nscratch));
        }
    }
    vk::CgVecs cv{};
    cv.tau = tau;
    cv.gam2 = gam2;
    for (int k = 0; k < K; ++k) {
        CgSystem* s = sys[k];
        cv.mu[k] = s->mu;
        cv.r[k] = s->r;
        cv.z[k] = s->z;
        cv.p[k] = s->p;
        cv.v[k] = s->v;
        cv.atx0[k] = s->mu0_nonzero ? s->atx0 : nullptr;
        cv.d[k] = (s->mu0_nonzero && !s->atx0) ? s->d : nullptr;
    }
    std::vector<double> rzvv(2 * K);
    DotBatch local(c);
    DotBatch& b0 = init ? *init : local;
    vk::RedOut ro{};
    STCHK(b0.sink(2 * K, true, rzvv.data(), &ro));
    HIPCHK(vk::cg_init(K, M, cv, diag, ro, c->st));
    STCHK(b0.flush());
    std::vector<double> rz(K), vv(K), prev_ons(K, 0.0);
    std::vector<int> active;
    for (int k = 0; k < K; ++k) {
        rz[k] = rzvv[2 * k];
        vv[k] = rzvv[2 * k + 1];
        sys[k]->iters = 0;
        active.push_back(k);
    }
    std::vector<double> red(3 * vk::kMaxRhs);
    for (int i = 0; i < max_iter && !active.empty(); ++i) {
        const int Ka = (int)active.size();
        vk::CgVecs cu{};
        vk::CgScalars rzs{};
        const double* pp[vk::kMaxRhs];
        double* dd[vk::kMaxRhs];
        for (int a = 0; a < Ka; ++a) {
            CgSystem* s = sys[active[a]];
            cu.mu[a] = s->mu;
            cu.r[a] = s->r;
            cu.z[a] = s->z;
            cu.p[a] = s->p;
            cu.d[a] = s->d;
            cu.v[a] = s->v;
            rzs.rz[a] = rz[active[a]];
            pp[a] = s->p;
            dd[a] = s->d;
        }
        // d = lmmse_mult(p)   (:700); <d,p> lands in scal[SL_DP + a]
        STCHK(lmmse_dev(c, Ka, pp, dd, tau, gam2, nscratch));
        if (ref_passes) *ref_passes += 2 * (int64_t)Ka;
        DotBatch b(c);
        vk::RedOut rou{};
        STCHK(b.sink(3 * Ka, true, red.data(), &rou));
        HIPCHK(vk::cg_update(Ka, M, cu, diag, rzs, c->scal + SL_DP, rou, c->st));
        STCHK(b.flush());
        std::vector<int> still;
        vk::CgVecs pv{};
        vk::CgBeta beta{};
        int np = 0;
        for (int a = 0; a < Ka; ++a) {
            const int k = active[a];
            CgSystem* s = sys[k];
            s->iters = i + 1;
            const double rz_new = red[3 * a], rr = red[3 * a + 1], vmu = red[3 * a + 2];
            if (s->onsager) {  // :708-726
                const double ons = gam2 * vmu;
                const double rel = ons != 0 ? std::fabs((ons - prev_ons[k]) / ons) : 1;
                if (rel < 1e-8) continue;
                prev_ons[k] = ons;
            }
            double bt = std::pow(rz[k], -1);  // :731
            bt *= rz_new;                      // :736
            rz[k] = rz_new;
            const double rel_err = std::sqrt(rr) / std::sqrt(vv[k]);  // :742-744
            if (rel_err < tol) continue;                               // :750
            still.push_back(k);
            pv.z[np] = s->z;
            pv.p[np] = s->p;
            beta.beta[np] = bt;
            ++np;
        }
        if (np > 0) HIPCHK(vk::cg_pupdate(np, M, pv, beta, c->st));  // p = z + beta p (:738-739)
        active.swap(still);
    }
    return VAMPOMI_OK;
}
