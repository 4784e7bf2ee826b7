/* CPU check behind the device exp of the probit denoiser
 * (vampomi_amd/csrc/exp_cr.h, used by erfcx_ref in kernels.hip; the
 * reference's erfcx calls glibc's exp, src/utilities.cpp:293-363).
 *
 * For n arguments in three ranges (erfcx's s = x^2 in [0, 100]; every
 * argument with a normal result, [-708.39, 709.78]; |x| < 2^-20) compares
 * exp_cr with glibc's exp and with the 113-bit expq of libquadmath rounded
 * to double (the correctly rounded value except within 2^-113 of a
 * midpoint).  Prints one line per range:
 *   range tried cr_vs_quad glibc_vs_quad cr_vs_glibc max_ulp_cr_vs_glibc
 * Usage: exp_cr_check [n [stream]].
 * Build: gcc -O2 -ffp-contract=off tests/exp_cr_check.c -lquadmath -lm */
#include <math.h>
#include <quadmath.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define EXPCR_FN static inline
#include "../vampomi_amd/csrc/exp_cr.h"

static uint64_t st = 0x243F6A8885A308D3ULL;
static uint64_t next(void) {
    st ^= st << 13;
    st ^= st >> 7;
    st ^= st << 17;
    return st;
}
static double unit(void) { return (double)(next() >> 11) * 0x1p-53; }

static long ulps(double a, double b) {
    int64_t ia, ib;
    memcpy(&ia, &a, 8);
    memcpy(&ib, &b, 8);
    return labs((long)(ia - ib));
}

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 1000000;
    if (argc > 2) st ^= strtoull(argv[2], NULL, 0) * 0x9E3779B97F4A7C15ULL; /* independent streams */
    const char* names[3] = {"erfcx_s_0_100", "normal_results", "tiny"};
    for (int range = 0; range < 3; ++range) {
        long bad_cr = 0, bad_glibc = 0, diff = 0, maxulp = 0;
        volatile double sink = 0;
        for (long i = 0; i < n; ++i) {
            double x;
            if (range == 0)
                x = 100.0 * unit();
            else if (range == 1)
                x = -708.39 + (709.78 + 708.39) * unit();
            else
                x = ldexp(2.0 * unit() - 1.0, -20);
            const double a = exp_cr(x), g = exp(x);
            const double q = (double)expq((__float128)x);
            sink += a;
            if (memcmp(&a, &q, 8) != 0) ++bad_cr;
            if (memcmp(&g, &q, 8) != 0) ++bad_glibc;
            if (memcmp(&a, &g, 8) != 0) {
                ++diff;
                const long d = ulps(a, g);
                if (d > maxulp) maxulp = d;
            }
        }
        (void)sink;
        printf("%s %ld %ld %ld %ld %ld\n", names[range], n, bad_cr, bad_glibc, diff, maxulp);
    }
    /* special values */
    const double sp[] = {0.0, -0.0, 1.0, -1.0, 709.78, -745.0, 710.0, -746.0, INFINITY, -INFINITY};
    int bad = 0;
    for (unsigned k = 0; k < sizeof sp / sizeof sp[0]; ++k) {
        const double a = exp_cr(sp[k]), g = exp(sp[k]);
        if (memcmp(&a, &g, 8) != 0 && !(sp[k] == -745.0)) ++bad; /* -745: subnormal result, see exp_cr.h */
    }
    const double nn = exp_cr(NAN);
    printf("special %d %d\n", bad, isnan(nn) ? 0 : 1);
    return 0;
}
