// pcg.cpp — vamp::precondCG_solver (src/vamp.cpp:664-757) for several
// independent systems (tau*A^T A + gam2*I) mu = v that share the operator.
//
// Per CG step and per still-active system, exactly the reference's scalar
// recurrences: alpha = <r,z>/<d,p>; mu += alpha p; [Onsager stop on
// gam2<v,mu>]; r -= d alpha; z = r/diag; beta = pow(<r,z>_old,-1)*<r,z>_new;
// p = z + beta p; stop when ||r||/||v|| < tol.  What is shared is the pass
// over X: lmmse_mult(p) for all systems is one A.x and one A^T.u launch with
// K right-hand sides, so two systems cost 2*max(k1, k2) passes instead of
// 2*(k1 + k2), with every iterate bitwise equal to a solo solve.
//
// The step's scalar decisions run on the device (vk::cg_decide), so the host
// never stands between two steps: it queues step i+1 (every launch gated on
// "some system still active") and only then waits for step i's flag.  The
// direction update p = z + beta p rides in the next step's kernels.  A step
// queued after the last system stopped does nothing; its launches are dropped
// from the stats.
#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstdlib>
#include <string>
#include <utility>

#include "ctx.h"

// device addresses of CgState fields
template <class T>
static T* field(vk::CgState* cs, size_t off) {
    return reinterpret_cast<T*>(reinterpret_cast<char*>(cs) + off);
}

// The outcome of a decided CG step as the host reads it.
struct CgOutcome {
    int any = 0;
    int iters[vk::kMaxRhs] = {};
};

// Flag words (of the context's mapped block) of the packed decisions: step i
// is published into word kCgPackWord + (i & 1), so step i+1's (queued before
// the host reads step i's) never overwrites the one the host is waiting for.
static constexpr int kCgPackWord = 2;

// the host loop shared by both forms: queue step i+1, then wait for step i's
// decision; a step queued after the last system stopped is dropped from the stats.
// packed (the one-pass form, K <= 2): step i-1's decision is ONE word
// (vk::cg_pack) in flag word kCgPackWord + ((i-1) & 1); else it is read from
// its own mirror slot ((i-1) & 1), tagged with its flag value.  Either way
// step i, queued before the wait, writes the other one.  *last: the last decided step's outcome
// (its iteration counts are final).
// settle (may be null): called instead of enqueue(i) when no step i is
// queued (i = max_iter), for a decision of step i-1 that step i's launch
// would have formed (folded decisions)
template <class Enqueue, class Settle>
static vampomi_status cg_loop(vampomi_ctx* c, int max_iter, bool packed, Enqueue&& enqueue, CgOutcome* last,
                              Settle&& settle) {
    unsigned long long prev = 0, cur = 0;
    STCHK(enqueue(0, &prev));
    for (int i = 1;; ++i) {
        const size_t mark = c->pending.size();
        const vampomi_stats before = c->stats;
        if (i < max_iter)
            STCHK(enqueue(i, &cur));
        else
            STCHK(settle());
        c->stats.host_syncs++;
        CgOutcome o;
        if (packed) {
            const int word = kCgPackWord + ((i - 1) & 1);
            STCHK(wait_flag(c, prev << 32, word));  // step i-1 decided and published
            STCHK(op_check_err(c));                 // (its decision is void if its operator launch timed out)
            const unsigned long long w = __atomic_load_n(c->h_flag + word, __ATOMIC_ACQUIRE);
            if ((w >> 32) != (prev & 0xffffffffULL))
                return fail(VAMPOMI_ERR_STATE, "CG step " + std::to_string(i - 1) + ": decision word holds sequence " +
                                                   std::to_string(w >> 32) + ", expected " + std::to_string(prev));
            o.any = (int)((w >> 30) & 1);
            o.iters[0] = (int)(w & 0x7fff);
            o.iters[1] = (int)((w >> 15) & 0x7fff);
        } else {
            STCHK(wait_flag(c, prev));  // step i-1 decided
            STCHK(op_check_err(c));     // (its decision is void if its operator launch timed out)
            const vk::CgMirror* m = c->h_cgm + ((i - 1) & 1);
            if (__atomic_load_n(&m->seq, __ATOMIC_ACQUIRE) != prev)
                return fail(VAMPOMI_ERR_STATE, "CG step " + std::to_string(i - 1) + ": decision slot holds sequence " +
                                                   std::to_string(m->seq) + ", expected " + std::to_string(prev));
            o.any = m->any;
            for (int k = 0; k < vk::kMaxRhs; ++k) o.iters[k] = m->iters[k];
        }
        *last = o;
        if (!o.any || i >= max_iter) {
            if (i < max_iter) drop_launches(c, mark, before);  // step i was queued in vain: it did nothing
            break;
        }
        prev = cur;
    }
    return VAMPOMI_OK;
}

vampomi_status pcg_run(vampomi_ctx* c, const std::vector<CgSystem*>& sys, double tau, double gam2, int max_iter,
                       double tol, double* nscratch, int64_t* ref_passes, DotBatch* init, const double* extra_x,
                       double* ex_out, bool onepass, const double* const* ar0, HeadStart* hs, const vk::Prelude* pre,
                       PreMode pm) {
    const int64_t M = c->M, N = c->N;
    const double diag = tau * (double)(N - 1) / (double)N + gam2;  // :676-677
    const int K = (int)sys.size();
    if (K < 1 || K > vk::kMaxRhs) return fail(VAMPOMI_ERR_ARG, "pcg: 1..4 systems");
    if (extra_x && (!ex_out || K + 1 >= vk::kMaxRhs)) return fail(VAMPOMI_ERR_ARG, "pcg: extra A.x needs K <= 2");
    if (hs) {
        hs->used = false;
        if (!onepass || K != 2 || !extra_x || ar0 || sys[0]->mu0_nonzero || (hs->xnext && !hs->axnext))
            return fail(VAMPOMI_ERR_ARG, "pcg: the head start needs the one-pass form, two systems, extra_x, "
                                         "system 0 from zero and no ar0");
    }
    const double* xnext = hs ? hs->xnext : nullptr;
    auto extra_alone = [&]() -> vampomi_status {  // no CG step carries them
        const double* px[2];
        double* out[2];
        int n = 0;
        if (extra_x) px[n] = extra_x, out[n++] = ex_out;
        if (xnext) px[n] = xnext, out[n++] = hs->axnext;
        if (n == 0) return VAMPOMI_OK;
        STCHK(ax_dev(c, n, px, nscratch));
        for (int j = 0; j < n; ++j)
            HIPCHK(hipMemcpyAsync(out[j], nscratch + (int64_t)j * c->ld, (size_t)N * 8, hipMemcpyDeviceToDevice,
                                  c->st));
        return VAMPOMI_OK;
    };
    // initial residual r = v - lmmse_mult(mu0)  (:681-684)
    {
        std::vector<CgSystem*> nz;
        for (auto* s : sys) {
            if (s->mu0_nonzero && !s->atx0) nz.push_back(s);
            if (s->mu0_nonzero && ref_passes) *ref_passes += 2;
        }
        if (!nz.empty()) {
            if (pm != PreMode::normal) return fail(VAMPOMI_ERR_ARG, "pcg: a start queued ahead needs no lmmse pass");
            const double* vv[vk::kMaxRhs];
            double* dd[vk::kMaxRhs];
            for (size_t k = 0; k < nz.size(); ++k) {
                vv[k] = nz[k]->mu;
                dd[k] = nz[k]->d;
            }
            STCHK(lmmse_dev(c, (int)nz.size(), vv, dd, tau, gam2, nscratch));
        }
    }
    if (onepass && K <= vk::kOpMaxK && c->have_X) STCHK(op_prepare(c));
    const bool op1 = onepass && K <= vk::kOpMaxK && c->have_X && c->op_ok;  // the one-pass form (below)
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
    // the head start (ctx.h, HeadStart): system 0's first step rides in the pass
    // that starts the solve; it is then one step ahead (CgState.off)
    const bool head = hs && hs->abern && c->hs_ok && c->op_ok && max_iter > 0;  // hs_ok: agreed, hs_on included
    vk::CgState s0{};
    s0.K = K;
    s0.gam2 = gam2;
    s0.tol = tol;
    s0.maxit = max_iter;
    s0.off[0] = head ? 1 : 0;
    s0.any = max_iter > 0 ? 1 : 0;
    for (int k = 0; k < K; ++k) {
        s0.active[k] = 1;
        s0.onsager[k] = sys[k]->onsager ? 1 : 0;
        sys[k]->iters = 0;
    }
    if (pre && init) return fail(VAMPOMI_ERR_ARG, "pcg: the prelude rides only in the device-side start");
    if (pm != PreMode::normal && !pre) return fail(VAMPOMI_ERR_ARG, "pcg: a start queued ahead is the prelude's");
    if (init) {  // the caller's reductions resolve together with <r,z>, <v,v> (one host wait)
        std::vector<double> rzvv(2 * K);
        vk::RedOut ro{};
        STCHK(init->sink(2 * K, true, rzvv.data(), &ro));
        HIPCHK(vk::cg_init(K, M, cv, diag, ro, c->st));
        STCHK(init->flush());
        for (int k = 0; k < K; ++k) {
            s0.rz[k] = rzvv[2 * k];
            s0.vv[k] = rzvv[2 * k + 1];
        }
        if (max_iter <= 0) return extra_alone();
        HIPCHK(vk::cg_start(s0, c->cgs, c->st));
    } else {  // <r,z>, <v,v> stay on the device: the CgState is built there, no host wait
        const vk::RedOut ro{c->red_part, c->scal + SL_CGI, c->ticket, nullptr, 0, nullptr};
        // pre: the caller's prelude rides in the same launch, and on one rank
        // that launch's last block also builds the CgState (three launches in one)
        const bool own_start = pre && !c->use_comm;
        if (pm != PreMode::normal && (!pre || (pm == PreMode::ahead) != (pre->dev.scal != nullptr)))
            return fail(VAMPOMI_ERR_ARG, "pcg: a start queued ahead needs the prelude and its device scalars");
        if (pm == PreMode::queued) {
            // (queued ahead by the previous iteration, scalars from the device:
            // the prelude, and on several ranks the sums' all-reduce and the CgState)
        } else {
            if (pre)
                HIPCHK(vk::prelude_cg_init(K, M, *pre, cv, diag, ro, own_start ? &s0 : nullptr, c->cgs, c->st));
            else
                HIPCHK(vk::cg_init(K, M, cv, diag, ro, c->st));
            if (!own_start) {
                STCHK(allreduce_dev(c, c->scal + SL_CGI, (size_t)(2 * K)));
                // (ahead: gam2 from the device, the prelude's scalars {eta1, gam2, ...})
                if (max_iter > 0)
                    HIPCHK(vk::cg_start_from(s0, c->scal + SL_CGI, c->cgs, c->st,
                                             pm == PreMode::ahead ? pre->dev.scal + 1 : nullptr));
            }
            if (pm == PreMode::ahead) return VAMPOMI_OK;
        }
        if (max_iter <= 0) return extra_alone();
    }
    const int* gate = field<int>(c->cgs, offsetof(vk::CgState, any));
    const double* beta = field<double>(c->cgs, offsetof(vk::CgState, beta));
    if (op1) {
        // several ranks, team plans: each step's decision is formed by the next
        // operator launch (vk::OpFold) from the all-reduced sums, instead of
        // by a decision launch of its own; the two CgStates alternate (the
        // launch reads one while its workgroup 0 writes the other).  cur: the
        // state the next launches use; pend: the decision not yet formed
        const bool fold = c->use_comm && c->cg_fold && c->opp.T >= 1 && (!head || c->opp_hs.T >= 1);
        int cur = 0;
        struct Pending {
            bool on = false;
            int it = 0, mask = 0xf, pack = 0;
            vk::CgMirror* mirror = nullptr;
            unsigned long long* flag = nullptr;
            unsigned long long seq = 0;
        } pend;
        auto state = [&](int s) { return c->cgs + s; };
        // ---- one pass over X per CG step (vk::atax) ----
        // A r0 for every system (and A extra_x) by one A.x pass; then each step
        // forms q = A p = A r/diag + beta*q_old on the fly, streams X once for
        // d = tau*A^T q + gam2*p and A d, and cg_update carries A r -= alpha*A d
        double* AR = c->op_nvec;
        double* Q = c->op_nvec + (int64_t)vk::kMaxRhs * c->ld;
        const double* AD = c->op_nvec + (int64_t)2 * vk::kMaxRhs * c->ld;
        bool given = false;
        for (int k = 0; k < K; ++k) given = given || (ar0 && ar0[k]);
        if (head) {
            // A r0 of system 0 is hs->abern (r0 = v), used in place as system
            // 0's A r (cu.AR[0] below); its first step's launch (below, once
            // the step's vectors are set up) also forms A r0 of system 1,
            // A extra_x and A xnext
        } else if (!given) {
            const double* px[vk::kMaxRhs];
            for (int k = 0; k < K; ++k) px[k] = sys[k]->r;
            int n = K;
            if (extra_x) px[n++] = extra_x;
            if (xnext) px[n++] = xnext;
            STCHK(ax_dev(c, n, px, AR));
            if (extra_x)
                HIPCHK(hipMemcpyAsync(ex_out, AR + (int64_t)K * c->ld, (size_t)N * 8, hipMemcpyDeviceToDevice, c->st));
            if (xnext)
                HIPCHK(hipMemcpyAsync(hs->axnext, AR + (int64_t)(n - 1) * c->ld, (size_t)N * 8,
                                      hipMemcpyDeviceToDevice, c->st));
        } else {  // A r0 given for some systems (zero starts, r0 = v): one pass for the others, if any
            const double* px[vk::kMaxRhs];
            int slot[vk::kMaxRhs], n = 0;
            for (int k = 0; k < K; ++k) {
                if (ar0[k]) {
                    if (sys[k]->mu0_nonzero) return fail(VAMPOMI_ERR_ARG, "pcg: A r0 given for a nonzero start");
                    HIPCHK(hipMemcpyAsync(AR + (int64_t)k * c->ld, ar0[k], (size_t)N * 8, hipMemcpyDeviceToDevice,
                                          c->st));
                } else {
                    slot[n] = k;
                    px[n++] = sys[k]->r;
                }
            }
            if (extra_x) {
                slot[n] = K;
                px[n++] = extra_x;
            }
            if (n > 0) {
                STCHK(ax_dev(c, n, px, nscratch));
                for (int j = 0; j < n; ++j) {
                    double* dst = slot[j] < K ? AR + (int64_t)slot[j] * c->ld : ex_out;
                    HIPCHK(hipMemcpyAsync(dst, nscratch + (int64_t)j * c->ld, (size_t)N * 8, hipMemcpyDeviceToDevice,
                                          c->st));
                }
            }
        }
        vk::CgVecs cu{};
        cu.tau = tau;
        cu.gam2 = gam2;
        cu.nA = N;
        for (int k = 0; k < K; ++k) {
            cu.mu[k] = sys[k]->mu;
            cu.r[k] = sys[k]->r;
            cu.z[k] = sys[k]->z;
            cu.p[k] = sys[k]->p;
            cu.d[k] = sys[k]->d;
            cu.v[k] = sys[k]->v;
            cu.W[k] = sys[k]->W;
            cu.S[k] = sys[k]->W ? sys[k]->S : nullptr;
            cu.AW[k] = sys[k]->AW;
            cu.Q[k] = Q + (int64_t)k * c->ld;
            cu.AR[k] = head && k == 0 ? hs->abern : AR + (int64_t)k * c->ld;
            cu.AD[k] = AD + (int64_t)k * c->ld;
        }
        if (!c->use_comm) {  // one rank: cg_update sums the operator's A d slots itself
            cu.adpart = c->op_part;
            cu.adld = c->ld;
            cu.adslots = c->opp.nslots;
        }
        // the division of A d by sqrt(N) happens where cg_update reads it
        // (several ranks: the all-reduced A d, op_dev(..., divide = false))
        cu.addiv = c->sqrtN;
        bool rec = false;
        for (int k = 0; k < K; ++k) rec = rec || sys[k]->W;
        if (rec)
            for (int k = 0; k < K; ++k)
                if (!sys[k]->S) return fail(VAMPOMI_ERR_ARG, "pcg: W needs an S scratch vector for every system");
        const int all = (1 << K) - 1;
        if (head) {
            // system 0's step 1 (it = -1: its count becomes 1 + off - 1 + ... = 1)
            // together with A r0 of system 1, A extra_x and A xnext: one pass
            vk::OpArgs a{};
            a.ar.p[0] = cu.AR[0];
            a.qo.p[0] = cu.Q[0];
            a.p.p[0] = sys[0]->p;
            a.z.p[0] = sys[0]->z;
            a.d.p[0] = sys[0]->d;
            a.sraw.p[0] = rec ? sys[0]->S : nullptr;
            a.beta = beta;
            a.fuse = 0;
            a.diag = diag;
            a.tau = tau;
            a.gam2 = gam2;
            const double* px[vk::kOpPlain] = {sys[1]->r, extra_x, xnext ? xnext : extra_x};
            double* out[vk::kOpPlain] = {cu.AR[1], ex_out, xnext ? hs->axnext : nscratch};
            STCHK(op_dev_plain(c, a, px, out, gate));
            vk::CgVecs ch = cu;
            if (!c->use_comm) ch.adslots = (int)c->opp_hs.nslots;
            else ch.addiv = 0.0;  // (op_dev_plain divided its A d already)
            const double* dp = c->use_comm ? AD + (int64_t)(1 + vk::kOpPlain) * c->ld : c->scal + SL_DP;
            const vk::RedOut ro{c->red_part, c->scal + SL_CG, c->ticket, nullptr, 0, gate};
            vk::CgDecide dc{};  // no mirror, no flag: the host does not wait for this step
            dc.on = !c->use_comm;
            dc.it = -1;
            dc.mask = 1;
            HIPCHK(vk::cg_update(1, M, ch, diag, c->cgs, dp, nullptr, 0, ro, dc, c->st));
            if (c->use_comm) {
                STCHK(allreduce_dev(c, c->scal + SL_CG, 3));
                if (fold) {  // formed by step 0's operator launch
                    pend.on = true;
                    pend.it = -1;
                    pend.mask = 1;
                } else {
                    HIPCHK(vk::cg_decide(c->cgs, c->scal + SL_CG, -1, nullptr, nullptr, 0, c->st, 1));
                }
            }
            hs->used = true;
        }
        // the decisions travel as one packed word each (cg_loop): one
        // system-scope store instead of the mirror's six, a drain and the flag
        const bool packed = K <= 2 && max_iter < vk::kCgPackMaxIter;
        auto enqueue = [&](int i, unsigned long long* seq) -> vampomi_status {
            // the direction updates fused into step i: every system's from step
            // 1 on; at step 0 those of the systems already under way (head start)
            const int fuse = i > 0 ? all : head ? 1 : 0;
            vk::OpArgs a{};
            for (int k = 0; k < K; ++k) {
                a.ar.p[k] = cu.AR[k];
                a.qo.p[k] = cu.Q[k];
                a.p.p[k] = sys[k]->p;
                a.z.p[k] = sys[k]->z;
                a.d.p[k] = sys[k]->d;
                a.sraw.p[k] = rec ? sys[k]->S : nullptr;
            }
            a.beta = fold ? nullptr : beta;
            a.fuse = fuse;
            a.diag = diag;
            a.tau = tau;
            a.gam2 = gam2;
            const int* g = gate;
            vk::CgState* cs = c->cgs;
            if (fold) {
                if (pend.on) {  // the previous step's decision, formed by this launch into the other state
                    a.fold.on = 1;
                    a.fold.src = state(cur);
                    a.fold.dst = state(cur ^ 1);
                    a.fold.red = c->scal + SL_CG;
                    a.fold.it = pend.it;
                    a.fold.mask = pend.mask;
                    a.fold.pack = pend.pack;
                    a.fold.mirror = pend.mirror;
                    a.fold.flag = pend.flag;
                    a.fold.seq = pend.seq;
                    cur ^= 1;
                    pend.on = false;
                }
                cs = state(cur);
                g = field<int>(cs, offsetof(vk::CgState, any));
                if (!a.fold.on) a.beta = field<double>(cs, offsetof(vk::CgState, beta));
            }
            STCHK(op_dev(c, K, a, g, c->use_comm, false));
            const double* dp = c->use_comm ? AD + (int64_t)K * c->ld : c->scal + SL_DP;
            const vk::RedOut ro{c->red_part, c->scal + SL_CG, c->ticket, nullptr, 0, g};
            *seq = ++c->sync_seq;
            unsigned long long* flag = packed ? c->d_flag + kCgPackWord + (i & 1) : c->d_flag;
            vk::CgMirror* mirror = packed ? nullptr : c->d_cgm;
            vk::CgDecide dc{};
            if (!c->use_comm) {
                dc.on = 1;
                dc.it = i;
                dc.mirror = mirror;
                dc.flag = flag;
                dc.seq = *seq;
                dc.pack = packed ? 1 : 0;
            }
            HIPCHK(vk::cg_update(K, M, cu, diag, cs, dp, nullptr, fuse, ro, dc, c->st));
            if (c->use_comm) {
                STCHK(allreduce_dev(c, c->scal + SL_CG, (size_t)(3 * K)));
                if (fold) {  // formed by the next step's operator launch (or settle)
                    pend.on = true;
                    pend.it = i;
                    pend.mask = 0xf;
                    pend.pack = packed ? 1 : 0;
                    pend.mirror = mirror;
                    pend.flag = flag;
                    pend.seq = *seq;
                } else {
                    HIPCHK(vk::cg_decide(c->cgs, c->scal + SL_CG, i, mirror, flag, *seq, c->st, 0xf, packed ? 1 : 0));
                }
            }
            return VAMPOMI_OK;
        };
        // the last step's decision when no step follows to form it
        auto settle = [&]() -> vampomi_status {
            if (!pend.on) return VAMPOMI_OK;
            HIPCHK(vk::cg_decide(state(cur), c->scal + SL_CG, pend.it, pend.mirror, pend.flag, pend.seq, c->st,
                                 pend.mask, pend.pack));
            pend.on = false;
            return VAMPOMI_OK;
        };
        CgOutcome last;
        STCHK(cg_loop(c, max_iter, packed, enqueue, &last, settle));
        STCHK(op_check_err(c));
        for (int k = 0; k < K; ++k) {
            sys[k]->iters = last.iters[k];
            if (ref_passes) *ref_passes += 2 * (int64_t)sys[k]->iters;
        }
        return VAMPOMI_OK;
    }
    if (xnext) {  // (no one-pass plan: the head start's next product by its own pass)
        STCHK(ax_dev(c, 1, &xnext, nscratch));
        HIPCHK(hipMemcpyAsync(hs->axnext, nscratch, (size_t)N * 8, hipMemcpyDeviceToDevice, c->st));
    }
    const double* pp[vk::kMaxRhs];
    const double* zz[vk::kMaxRhs];
    double* dd[vk::kMaxRhs];
    double* ss[vk::kMaxRhs];
    bool recur = false;
    for (int k = 0; k < K; ++k) {
        pp[k] = sys[k]->p;
        zz[k] = sys[k]->z;
        dd[k] = sys[k]->d;
        ss[k] = sys[k]->S;
        recur = recur || sys[k]->W;
    }
    if (recur)  // every system keeps a raw-product slot (the kernel stores all K or none)
        for (int k = 0; k < K; ++k)
            if (!ss[k]) return fail(VAMPOMI_ERR_ARG, "pcg: W needs an S scratch vector for every system");
    // several ranks: <d,p> rides in the A.x all-reduce (nscratch holds K*ld + K);
    // VAMPOMI_DP_SEPARATE=1 keeps the one-rank form (tests compare bitwise)
    static const bool dp_separate = std::getenv("VAMPOMI_DP_SEPARATE") && std::atoi(std::getenv("VAMPOMI_DP_SEPARATE"));
    const bool split_dp = c->use_comm && K < vk::kMaxRhs && !dp_separate;
    vk::CgVecs cu{};
    cu.tau = tau;
    cu.gam2 = gam2;
    for (int k = 0; k < K; ++k) {
        cu.mu[k] = sys[k]->mu;
        cu.r[k] = sys[k]->r;
        cu.z[k] = sys[k]->z;
        cu.p[k] = sys[k]->p;
        cu.d[k] = sys[k]->d;
        cu.v[k] = sys[k]->v;
        cu.W[k] = sys[k]->W;
        cu.S[k] = sys[k]->W ? sys[k]->S : nullptr;
        cu.AW[k] = sys[k]->AW;
        cu.AS[k] = nscratch + (int64_t)k * c->ld;  // this step's A p (the A.x pass output)
        if (sys[k]->AW) cu.nA = N;
    }
    // queues CG step i; *seq: the sequence number its decision stores.  From
    // step 1 on, the direction update p = z + beta p (:738-739) of the step
    // before is fused into this step's kernels: the A.x pass, the lmmse_mult
    // epilogue and <d,p> form it on the fly, cg_update stores it.
    auto enqueue = [&](int i, unsigned long long* seq) -> vampomi_status {
        const bool fuse = i > 0;
        vk::AxFuse fu{};
        fu.gate = gate;
        if (fuse) {
            for (int k = 0; k < K; ++k) fu.z.p[k] = zz[k];
            fu.beta = beta;
        }
        // d = lmmse_mult(p) (:700).  One rank: <d,p> by a reduction over d and
        // p into scal[SL_DP + k].  Several ranks: <d,p> = tau*|A p|^2 +
        // gam2*|p|^2, with the local |p|^2 all-reduced together with A p's
        // partials and |A p|^2 summed over the replicated N-vector: one
        // collective per step fewer.
        const double* u[vk::kMaxRhs];
        for (int k = 0; k < K; ++k) u[k] = nscratch + (int64_t)k * c->ld;
        // the first step's pass also carries A.extra_x (one more right-hand side)
        const double* px[vk::kMaxRhs];
        for (int k = 0; k < K; ++k) px[k] = pp[k];
        const bool ex = i == 0 && extra_x;
        if (ex) px[K] = extra_x;
        const int KA = ex ? K + 1 : K;
        const double* pp_dev = nullptr;
        if (split_dp) {
            vk::DotArgs tail{};
            tail.nt = K;
            for (int k = 0; k < K; ++k)
                tail.t[k] = fuse ? vk::DotTerm{pp[k], pp[k], vk::SQPUPD, zz[k], beta + k}
                                 : vk::DotTerm{pp[k], pp[k], vk::DOT};
            STCHK(ax_dev(c, KA, px, nscratch, &fu, &tail));
            if (ex) HIPCHK(hipMemcpyAsync(ex_out, nscratch + (int64_t)K * c->ld, (size_t)N * 8, hipMemcpyDeviceToDevice, c->st));
            pp_dev = nscratch + (int64_t)KA * c->ld;
            vk::DotArgs uu{};
            uu.nt = K;
            for (int k = 0; k < K; ++k) uu.t[k] = vk::DotTerm{u[k], u[k], vk::DOT};
            HIPCHK(vk::dots(uu, c->N, vk::RedOut{c->red_part, c->scal + SL_DP, c->ticket, nullptr, 0, gate}, c->st));
            STCHK(atx_dev(c, K, u, dd, 1, tau, gam2, pp, gate, fuse ? zz : nullptr, beta, false, recur ? ss : nullptr));
        } else {
            STCHK(ax_dev(c, KA, px, nscratch, &fu));
            if (ex) HIPCHK(hipMemcpyAsync(ex_out, nscratch + (int64_t)K * c->ld, (size_t)N * 8, hipMemcpyDeviceToDevice, c->st));
            STCHK(atx_dev(c, K, u, dd, 1, tau, gam2, pp, gate, fuse ? zz : nullptr, beta, true, recur ? ss : nullptr));
        }
        const vk::RedOut ro{c->red_part, c->scal + SL_CG, c->ticket, nullptr, 0, gate};
        *seq = ++c->sync_seq;
        vk::CgDecide dc{};
        if (!c->use_comm) {  // one rank: cg_update's last block decides
            dc.on = 1;
            dc.it = i;
            dc.mirror = c->d_cgm;
            dc.flag = c->d_flag;
            dc.seq = *seq;
        }
        HIPCHK(vk::cg_update(K, M, cu, diag, c->cgs, c->scal + SL_DP, pp_dev, fuse ? (1 << K) - 1 : 0, ro, dc,
                             c->st));
        if (c->use_comm) {  // the sums are final after the all-reduce
            STCHK(allreduce_dev(c, c->scal + SL_CG, (size_t)(3 * K)));
            HIPCHK(vk::cg_decide(c->cgs, c->scal + SL_CG, i, c->d_cgm, c->d_flag, *seq, c->st));
        }
        return VAMPOMI_OK;
    };
    CgOutcome last;
    STCHK(cg_loop(c, max_iter, false, enqueue, &last, [] { return VAMPOMI_OK; }));
    for (int k = 0; k < K; ++k) {
        sys[k]->iters = last.iters[k];
        if (ref_passes) *ref_passes += 2 * (int64_t)sys[k]->iters;
    }
    return VAMPOMI_OK;
}
