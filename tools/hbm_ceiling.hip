// hbm_ceiling.hip — what read bandwidth can one MI355X sustain for the access
// shapes the A passes use?  Standalone (no engine); prints one JSON line per
// variant.  Build: hipcc --offload-arch=gfx950 -O3 -o hbm_ceiling hbm_ceiling.hip
//
// Variants (all read a B-byte fp64 buffer once with 16-byte loads per lane and
// reduce it, so nothing is dead code):
//   chunk<U,NT>   a wave reads one contiguous chunk of `chunk` bytes, U loads in
//                 flight per lane; one chunk per wave, in-order dispatch
//   persist<U,NT> grid = CUs * wgs_per_cu, every wave an equal contiguous share
//   lock<U,NT,SYNC> 8-wave workgroups, one contiguous stream each (barrier per round)
//   cols<G,U,NT>  like atx_kernel: a wave walks G columns of `col` bytes at once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double v2d __attribute__((ext_vector_type(2)));

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(2);                                                              \
        }                                                                              \
    } while (0)

template <bool NT>
__device__ __forceinline__ v2d ldv(const double* p) {
    if (NT) return __builtin_nontemporal_load(reinterpret_cast<const v2d*>(p));
    return *reinterpret_cast<const v2d*>(p);
}

__device__ __forceinline__ double wsum(double v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// one wave = one chunk of cw doubles (cw multiple of 128*U)
template <int U, bool NT>
__global__ __launch_bounds__(256) void chunk_kernel(const double* __restrict__ x, int64_t n, int64_t cw,
                                                    double* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t b = w * cw;
    if (b >= n) return;
    const int64_t e = b + cw < n ? b + cw : n;
    double a0 = 0, a1 = 0;
    for (int64_t j = b + 2 * lane; j + 128 * (U - 1) < e; j += 128 * U) {
        v2d v[U];
#pragma unroll
        for (int t = 0; t < U; ++t) v[t] = ldv<NT>(x + j + 128 * t);
#pragma unroll
        for (int t = 0; t < U; ++t) {
            a0 += v[t].x;
            a1 += v[t].y;
        }
    }
    const double s = wsum(a0 + a1);
    if (lane == 0) out[w] = s;
}

// equal contiguous share per wave over a fixed grid
template <int U, bool NT>
__global__ __launch_bounds__(256) void persist_kernel(const double* __restrict__ x, int64_t n, double* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    const int64_t w = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t units = n / 128;  // 1 KiB units
    const int64_t b = units * w / nw * 128, e = units * (w + 1) / nw * 128;
    double a0 = 0, a1 = 0;
    int64_t j = b + 2 * lane;
    for (; j + 128 * (U - 1) < e; j += 128 * U) {
        v2d v[U];
#pragma unroll
        for (int t = 0; t < U; ++t) v[t] = ldv<NT>(x + j + 128 * t);
#pragma unroll
        for (int t = 0; t < U; ++t) {
            a0 += v[t].x;
            a1 += v[t].y;
        }
    }
    for (; j < e; j += 128) {
        v2d v = ldv<NT>(x + j);
        a0 += v.x;
        a1 += v.y;
    }
    const double s = wsum(a0 + a1);
    if (lane == 0) out[w] = s;
}

// lockstep: 8-wave workgroups (one or two per CU), each a contiguous share;
// per round the 8 waves read 8U consecutive KiB, then (SYNC) meet at a barrier,
// so a workgroup reads one stream as the team kernels do (a barrier per column)
template <int U, bool NT, bool SYNC>
__global__ __launch_bounds__(512) void lock_kernel(const double* __restrict__ x, int64_t n, double* __restrict__ out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t units = n / 1024;  // 8 KiB units
    const int64_t b = units * blockIdx.x / gridDim.x * 1024, e = units * (blockIdx.x + 1) / gridDim.x * 1024;
    double a0 = 0, a1 = 0;
    int64_t j = b + 128 * wave + 2 * lane;
    for (; j + 1024 * (U - 1) < e; j += 1024 * U) {
        v2d v[U];
#pragma unroll
        for (int t = 0; t < U; ++t) v[t] = ldv<NT>(x + j + 1024 * t);
#pragma unroll
        for (int t = 0; t < U; ++t) {
            a0 += v[t].x;
            a1 += v[t].y;
        }
        if (SYNC) __syncthreads();
    }
    for (; j < e; j += 1024) {
        v2d v = ldv<NT>(x + j);
        a0 += v.x;
        a1 += v.y;
    }
    const double s = wsum(a0 + a1);
    if (lane == 0) out[(int64_t)blockIdx.x * 8 + wave] = s;
}

// atx shape: a wave owns G columns of ld doubles, walks them together
template <int G, int U, bool NT>
__global__ __launch_bounds__(256) void cols_kernel(const double* __restrict__ x, int64_t ld, int64_t ncol,
                                                   double* __restrict__ out, int wpb) {
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6);
    const int64_t m0 = w * G;
    if (m0 >= ncol) return;
    double acc[G];
    const double* c[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        c[g] = x + std::min(m0 + g, ncol - 1) * ld;
        acc[g] = 0;
    }
    int64_t j = 2 * lane;
    for (; j + 128 * (U - 1) < ld; j += 128 * U) {
        v2d v[U][G];
#pragma unroll
        for (int t = 0; t < U; ++t)
#pragma unroll
            for (int g = 0; g < G; ++g) v[t][g] = ldv<NT>(c[g] + j + 128 * t);
#pragma unroll
        for (int t = 0; t < U; ++t)
#pragma unroll
            for (int g = 0; g < G; ++g) acc[g] += v[t][g].x + v[t][g].y;
    }
    for (; j < ld; j += 128) {  // tail (ld is even: the pair never straddles a column)
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const v2d v = ldv<NT>(c[g] + j);
            acc[g] += v.x + v.y;
        }
    }
    double s = 0;
#pragma unroll
    for (int g = 0; g < G; ++g) s += acc[g];
    s = wsum(s);
    if (lane == 0) out[w] = s;
}

__global__ void fill_kernel(double* x, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        x[i] = (double)(i & 1023) * 0.5;
}

template <class F>
static void timeit(const char* name, double bytes, int reps, F&& launch) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    launch();
    CK(hipDeviceSynchronize());
    std::vector<float> ms(reps);
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(a, 0));
        launch();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms[r], a, b));
    }
    std::sort(ms.begin(), ms.end());
    const double med = ms[reps / 2], best = ms[0];
    std::printf("{\"variant\": \"%s\", \"bytes\": %.0f, \"us_med\": %.1f, \"us_best\": %.1f, \"GBs_med\": %.1f, "
                "\"GBs_best\": %.1f}\n",
                name, bytes, med * 1e3, best * 1e3, bytes / (med * 1e-3) / 1e9, bytes / (best * 1e-3) / 1e9);
    std::fflush(stdout);
}

int main(int argc, char** argv) {
    const double gb = argc > 1 ? std::atof(argv[1]) : 4.0;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 15;
    const int64_t n = (int64_t)(gb * 1e9 / 8) / 1024 * 1024;
    const double bytes = 8.0 * n;
    double *x, *out;
    CK(hipMalloc(&x, n * 8));
    CK(hipMalloc(&out, (int64_t)1 << 26));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, x, n);
    CK(hipDeviceSynchronize());
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    char nm[128];
    // contiguous chunk per wave
    for (int64_t ckb : {64, 256, 1024}) {
        const int64_t cw = ckb * 1024 / 8;
        const unsigned blocks = (unsigned)((n / cw + 3) / 4);
        std::snprintf(nm, sizeof nm, "chunk%lldK_U4_nt", (long long)ckb);
        timeit(nm, bytes, reps, [&] { hipLaunchKernelGGL((chunk_kernel<4, true>), dim3(blocks), dim3(256), 0, 0, x, n, cw, out); });
        std::snprintf(nm, sizeof nm, "chunk%lldK_U8_nt", (long long)ckb);
        timeit(nm, bytes, reps, [&] { hipLaunchKernelGGL((chunk_kernel<8, true>), dim3(blocks), dim3(256), 0, 0, x, n, cw, out); });
        std::snprintf(nm, sizeof nm, "chunk%lldK_U4", (long long)ckb);
        timeit(nm, bytes, reps, [&] { hipLaunchKernelGGL((chunk_kernel<4, false>), dim3(blocks), dim3(256), 0, 0, x, n, cw, out); });
    }
    // persistent equal shares
    for (int wpc : {1, 2, 4, 8}) {
        const unsigned blocks = (unsigned)(cus * wpc);
        std::snprintf(nm, sizeof nm, "persist_wg%d_U4_nt", wpc);
        timeit(nm, bytes, reps, [&] { hipLaunchKernelGGL((persist_kernel<4, true>), dim3(blocks), dim3(256), 0, 0, x, n, out); });
        std::snprintf(nm, sizeof nm, "persist_wg%d_U8_nt", wpc);
        timeit(nm, bytes, reps, [&] { hipLaunchKernelGGL((persist_kernel<8, true>), dim3(blocks), dim3(256), 0, 0, x, n, out); });
        std::snprintf(nm, sizeof nm, "persist_wg%d_U4", wpc);
        timeit(nm, bytes, reps, [&] { hipLaunchKernelGGL((persist_kernel<4, false>), dim3(blocks), dim3(256), 0, 0, x, n, out); });
    }
    // lockstep workgroups (the team kernels' access)
    for (int wpc : {1, 2}) {
        const unsigned blocks = (unsigned)(cus * wpc);
        std::snprintf(nm, sizeof nm, "lock_wg%d_U4_nt_sync", wpc);
        timeit(nm, bytes, reps, [&] { hipLaunchKernelGGL((lock_kernel<4, true, true>), dim3(blocks), dim3(512), 0, 0, x, n, out); });
        std::snprintf(nm, sizeof nm, "lock_wg%d_U8_nt_sync", wpc);
        timeit(nm, bytes, reps, [&] { hipLaunchKernelGGL((lock_kernel<8, true, true>), dim3(blocks), dim3(512), 0, 0, x, n, out); });
        std::snprintf(nm, sizeof nm, "lock_wg%d_U4_sync", wpc);
        timeit(nm, bytes, reps, [&] { hipLaunchKernelGGL((lock_kernel<4, false, true>), dim3(blocks), dim3(512), 0, 0, x, n, out); });
        std::snprintf(nm, sizeof nm, "lock_wg%d_U4_nt_nosync", wpc);
        timeit(nm, bytes, reps, [&] { hipLaunchKernelGGL((lock_kernel<4, true, false>), dim3(blocks), dim3(512), 0, 0, x, n, out); });
    }
    if (argc > 3 && std::atoi(argv[3]) == 1) {  // lockstep and persistent only
        CK(hipFree(x));
        CK(hipFree(out));
        return 0;
    }
    // atx shape: N=10,000 (ld 10,000) and 100,000 columns
    for (int64_t ld : {(int64_t)10000, (int64_t)100000}) {
        const int64_t ncol = n / ld;
        const double cb = 8.0 * ncol * ld;
        for (int wpb : {2, 4}) {
            const unsigned b4 = (unsigned)((ncol + 4 * wpb - 1) / (4 * wpb));
            std::snprintf(nm, sizeof nm, "cols_ld%lld_G4_U4_nt_wpb%d", (long long)ld, wpb);
            timeit(nm, cb, reps, [&] { hipLaunchKernelGGL((cols_kernel<4, 4, true>), dim3(b4), dim3(64 * wpb), 0, 0, x, ld, ncol, out, wpb); });
            std::snprintf(nm, sizeof nm, "cols_ld%lld_G4_U2_nt_wpb%d", (long long)ld, wpb);
            timeit(nm, cb, reps, [&] { hipLaunchKernelGGL((cols_kernel<4, 2, true>), dim3(b4), dim3(64 * wpb), 0, 0, x, ld, ncol, out, wpb); });
            const unsigned b2 = (unsigned)((ncol + 2 * wpb - 1) / (2 * wpb));
            std::snprintf(nm, sizeof nm, "cols_ld%lld_G2_U4_nt_wpb%d", (long long)ld, wpb);
            timeit(nm, cb, reps, [&] { hipLaunchKernelGGL((cols_kernel<2, 4, true>), dim3(b2), dim3(64 * wpb), 0, 0, x, ld, ncol, out, wpb); });
            const unsigned b1 = (unsigned)((ncol + wpb - 1) / wpb);
            std::snprintf(nm, sizeof nm, "cols_ld%lld_G1_U8_nt_wpb%d", (long long)ld, wpb);
            timeit(nm, cb, reps, [&] { hipLaunchKernelGGL((cols_kernel<1, 8, true>), dim3(b1), dim3(64 * wpb), 0, 0, x, ld, ncol, out, wpb); });
        }
    }
    CK(hipFree(x));
    CK(hipFree(out));
    return 0;
}
