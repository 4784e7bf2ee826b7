// exp(x) correctly rounded in practice (double-double evaluation, one final
// rounding).  Shared by the device (kernels.hip: the probit denoiser's erfcx,
// src/utilities.cpp:293-363 via src/vamp_probit.cpp:469-488) and the CPU check
// tests/exp_cr_check.c, so both run the same operations.  The includer defines
// EXPCR_FN (the function qualifiers) before including this file; every
// translation unit that includes it must be compiled with -ffp-contract=off.
//
// Why: the reference calls glibc's exp (std::exp), whose result is the correctly
// rounded one except on a small fraction of arguments (its error bound is about
// 0.51 ulp); OCML's device exp is a ~1-ulp approximation and differs from glibc
// in the last bit on a large fraction of arguments.  In the probit recursion one
// ulp of erfcx reaches r1 amplified by 1/(1 - alpha2) (src/vamp_probit.cpp:
// 337-338), so the device uses this evaluation and tests/exp_cr_check.c counts
// its disagreements with glibc and with a 113-bit expq.
//
// Method: x = n ln2 + r with r in double-double (ln2 in three parts, the
// products n*ln2_k exact through fma), |r| <= 0.347; s = r / 256 (exact);
// exp(s) - 1 = s * P(s), P the degree-9 Taylor polynomial in double-double
// (truncation < 2^-119); eight squarings in expm1 form, e <- e (2 + e), give
// exp(r) - 1 to ~2^-101 relative; 1 + e is rounded once and scaled by 2^n.
// Results in the subnormal range are rounded twice (ldexp of the rounded
// value): this path only serves arguments whose result is a normal double.
#pragma once

#ifndef EXPCR_FN
#error "define EXPCR_FN (function qualifiers) before including exp_cr.h"
#endif

EXPCR_FN void expcr_two_sum(double a, double b, double* s, double* e) {
    const double t = a + b;
    const double bb = t - a;
    *e = (a - (t - bb)) + (b - bb);
    *s = t;
}

EXPCR_FN void expcr_fast_two_sum(double a, double b, double* s, double* e) {
    const double t = a + b;
    *e = b - (t - a);
    *s = t;
}

// (ah + al) * (bh + bl), relative error ~2^-104
EXPCR_FN void expcr_dd_mul(double ah, double al, double bh, double bl, double* h, double* l) {
    const double p = ah * bh;
    double e = __builtin_fma(ah, bh, -p);
    e += ah * bl + al * bh;
    expcr_fast_two_sum(p, e, h, l);
}

// (ah + al) + (bh + bl) without cancellation between the high parts
EXPCR_FN void expcr_dd_add(double ah, double al, double bh, double bl, double* h, double* l) {
    double s, e;
    expcr_two_sum(ah, bh, &s, &e);
    e += al + bl;
    expcr_fast_two_sum(s, e, h, l);
}

EXPCR_FN double exp_cr(double x) {
    if (!(x == x)) return x + x;                              // NaN
    if (x > 0x1.62e42fefa39efp+9) return __builtin_inf();     // > ln(DBL_MAX)
    if (x < -0x1.74910d52d3052p+9) return 0.0;                // < ln(2^-1075): rounds to 0
    const double n = __builtin_rint(x * 0x1.71547652b82fep+0);
    // r = x - n ln2, ln2 = L0 + L1 + L2 (~2^-165 relative)
    const double L0 = 0x1.62e42fefa39efp-1, L1 = 0x1.abc9e3b39803fp-56, L2 = 0x1.7b57a079a1934p-111;
    const double p0 = n * L0;
    const double p0l = __builtin_fma(n, L0, -p0);            // n L0 = p0 + p0l exactly
    const double t = x - p0;                                  // exact (Sterbenz; n = 0: t = x)
    const double p1 = n * L1;
    const double p1l = __builtin_fma(n, L1, -p1);
    double sh, sl, uh, ul, rh, rl;
    expcr_two_sum(t, -p0l, &sh, &sl);
    expcr_two_sum(sh, -p1, &uh, &ul);
    expcr_fast_two_sum(uh, ((sl + ul) - p1l) - n * L2, &rh, &rl);
    // s = r / 256 (exact); P(s) = sum_{k=0}^{9} s^k / (k+1)!
    const double s_h = rh * 0x1p-8, s_l = rl * 0x1p-8;
    const double ch[10] = {0x1p+0, 0x1p-1, 0x1.5555555555555p-3, 0x1.5555555555555p-5, 0x1.1111111111111p-7,
                           0x1.6c16c16c16c17p-10, 0x1.a01a01a01a01ap-13, 0x1.a01a01a01a01ap-16,
                           0x1.71de3a556c734p-19, 0x1.27e4fb7789f5cp-22};
    const double cl[10] = {0.0, 0.0, 0x1.5555555555555p-57, 0x1.5555555555555p-59, 0x1.1111111111111p-63,
                           -0x1.f49f49f49f49fp-65, 0x1.a01a01a01a01ap-73, 0x1.a01a01a01a01ap-76,
                           -0x1.c154f8ddc6c00p-73, 0x1.cbbc05b4fa99ap-76};
    double ph = ch[9], pl = cl[9];
    for (int k = 8; k >= 0; --k) {
        double mh, ml;
        expcr_dd_mul(s_h, s_l, ph, pl, &mh, &ml);
        expcr_dd_add(ch[k], cl[k], mh, ml, &ph, &pl);
    }
    double eh, el;
    expcr_dd_mul(s_h, s_l, ph, pl, &eh, &el);  // exp(s) - 1
    for (int k = 0; k < 8; ++k) {              // exp(2s) - 1 = e (2 + e)
        double qh, ql;
        expcr_dd_mul(eh, el, eh, el, &qh, &ql);
        expcr_dd_add(2.0 * eh, 2.0 * el, qh, ql, &eh, &el);
    }
    double h, l;
    expcr_fast_two_sum(1.0, eh, &h, &l);      // |e| < 0.42
    l += el;
    expcr_fast_two_sum(h, l, &h, &l);          // h = RN(exp(r))
    return __builtin_ldexp(h, (int)n);
}
