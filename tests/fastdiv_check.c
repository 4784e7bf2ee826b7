/* CPU check of the association pass's division (vampomi_amd/csrc/kernels.hip
 * loo_kernel, FASTDIV): q = fma(fma(-x*r, d, x), r, x*r) with r = RN(1/d)
 * equals the IEEE quotient x / d.  Prints the number of mismatches. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t st = 88172645463325252ULL;
static uint64_t next(void) {
    st ^= st << 13;
    st ^= st >> 7;
    st ^= st << 17;
    return st;
}

int main(int argc, char** argv) {
    const long per = argc > 1 ? atol(argv[1]) : 1000000;
    const long Ns[] = {2, 3, 5, 7, 10, 100, 257, 1000, 4099, 10000, 50000, 100000, 123457, 1048576, 999999};
    long bad = 0, tot = 0;
    for (int k = 0; k < (int)(sizeof Ns / sizeof Ns[0]); ++k) {
        const double d = sqrt((double)Ns[k]), r = 1.0 / d;
        for (long i = 0; i < per; ++i) {
            const uint64_t u = next();
            double x;
            if (i & 1) {
                x = ((double)(u >> 11) * 0x1p-53 * 2 - 1) * ldexp(1.0, (int)(next() % 80) - 40);
            } else {
                memcpy(&x, &u, 8);
                if (!isfinite(x) || fabs(x) > 1e300 || fabs(x) < 1e-290) continue;
            }
            const double q0 = x * r;
            const double q = fma(fma(-q0, d, x), r, q0);
            ++tot;
            if (q != x / d) ++bad;
        }
    }
    printf("%ld %ld\n", bad, tot);
    return 0;
}
