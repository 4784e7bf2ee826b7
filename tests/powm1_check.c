/* CPU check behind the device CG step (vampomi_amd/csrc/kernels.hip
 * cg_decide_kernel): the reference forms beta with pow(rz, -1)
 * (src/vamp.cpp:731); the device uses the correctly rounded 1.0 / rz.
 * glibc's pow is not correctly rounded: prints the number of mismatches, the
 * number of values tried and the largest distance in ulps. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t st = 0x9E3779B97F4A7C15ULL;
static uint64_t next(void) {
    st ^= st << 13;
    st ^= st >> 7;
    st ^= st << 17;
    return st;
}

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 1000000;
    volatile double m1 = -1.0;  /* keep pow() a library call */
    long bad = 0, tot = 0, maxulp = 0;
    for (long i = 0; i < n; ++i) {
        const uint64_t u = next();
        double x;
        if (i & 1) {  /* CG's <r,z> range: positive, 1e-300 .. 1e300 */
            x = (1.0 + (double)(u >> 11) * 0x1p-53) * ldexp(1.0, (int)(next() % 1990) - 995);
        } else {      /* any finite, nonzero bit pattern */
            memcpy(&x, &u, 8);
            if (!isfinite(x) || x == 0.0) continue;
        }
        const double a = pow(x, m1), b = 1.0 / x;
        if (memcmp(&a, &b, 8) != 0) {
            int64_t ia, ib;
            memcpy(&ia, &a, 8);
            memcpy(&ib, &b, 8);
            const long d = labs((long)(ia - ib));
            if (d > maxulp) maxulp = d;
            ++bad;
        }
        ++tot;
    }
    printf("%ld %ld %ld\n", bad, tot, maxulp);
    return 0;
}
