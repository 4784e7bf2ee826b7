// cgu_bench — one CG step's cg_update (the one-rank, one-pass form: the A d
// slot sums folded in) launched back to back, alone, on zero-filled buffers
// of a workload's shape; prints the mean launch-to-launch time.  Linked
// against libvampomi.so, so LD_LIBRARY_PATH picks the library under test
// (the production build or a CGU_ABL experiment build):
//
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 -I vampomi_amd/csrc tools/cgu_bench.hip \
//         -L vampomi_amd/lib -lvampomi -o build_cgu/cgu_bench
//   LD_LIBRARY_PATH=<lib dir> build_cgu/cgu_bench <N> <M> <slots> [launches]
//
// The state never converges (tol 0) and publishes nothing (no flag): every
// launch does a whole step's work.  Tool only (tools/cgu_ablation.sh).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "kernels.h"

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

static double* zeros(size_t n) {
    double* p = nullptr;
    CK(hipMalloc(&p, n * sizeof(double)));
    CK(hipMemset(p, 0, n * sizeof(double)));
    return p;
}

int main(int argc, char** argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: cgu_bench N M slots [launches]\n");
        return 2;
    }
    const int64_t N = std::atoll(argv[1]), M = std::atoll(argv[2]);
    const int slots = std::atoi(argv[3]), n = argc > 4 ? std::atoi(argv[4]) : 400;
    constexpr int K = 2;
    const int64_t ld = (N + 15) / 16 * 16;
    vk::CgVecs c{};
    for (int k = 0; k < K; ++k) {
        c.mu[k] = zeros(M);
        c.r[k] = zeros(M);
        c.z[k] = zeros(M);
        c.p[k] = zeros(M);
        c.d[k] = zeros(M);
        c.v[k] = zeros(M);
        c.Q[k] = zeros(ld);
        c.AR[k] = zeros(ld);
    }
    c.nA = N;
    c.adpart = zeros((size_t)slots * vk::kMaxRhs * ld);
    c.adld = ld;
    c.adslots = slots;
    c.addiv = 100.0;
    vk::CgState s{};
    s.K = K;
    s.any = 1;
    s.maxit = 1 << 30;
    s.tol = 0.0;
    s.gam2 = 1.0;
    for (int k = 0; k < K; ++k) {
        s.active[k] = 1;
        s.rz[k] = s.vv[k] = 1.0;
        s.beta[k] = 0.5;
    }
    vk::CgState* cs = nullptr;
    CK(hipMalloc(&cs, sizeof s));
    CK(hipMemcpy(cs, &s, sizeof s, hipMemcpyHostToDevice));
    double* dp = zeros(K);
    std::vector<double> one(K, 1.0);
    CK(hipMemcpy(dp, one.data(), K * sizeof(double), hipMemcpyHostToDevice));
    vk::RedOut ro{};
    ro.part = zeros((size_t)vk::kRedBlocks * 3 * vk::kMaxRhs);
    ro.out = zeros(3 * vk::kMaxRhs);
    CK(hipMalloc(&ro.ticket, 64 * sizeof(unsigned)));
    CK(hipMemset(ro.ticket, 0, 64 * sizeof(unsigned)));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    vk::CgDecide dc{};
    dc.on = 1;
    dc.pack = 1;
    auto step = [&](int it) {
        dc.it = it;
        CK(vk::cg_update(K, M, c, 1.0, cs, dp, nullptr, (1 << K) - 1, ro, dc, st));
    };
    for (int i = 0; i < 20; ++i) step(i);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, st));
    for (int i = 0; i < n; ++i) step(20 + i);
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    vk::CgState e{};
    CK(hipMemcpy(&e, cs, sizeof e, hipMemcpyDeviceToHost));
    std::printf("N %lld M %lld slots %d: %.2f us per cg_update launch (%d launches; state any %d, iters %d)\n",
                (long long)N, (long long)M, slots, 1e3 * ms / n, n, e.any, e.iters[0]);
    return 0;
}
