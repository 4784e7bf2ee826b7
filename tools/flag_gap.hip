// flag_gap.hip — what does a kernel's store into mapped host memory cost the
// NEXT kernel on the stream?  (cg_update's last block publishes the CG decision
// to the host; rocprofv3 showed 5.6 us of idle after every such kernel.)
//
// Pairs (W, B) back to back on one stream, W = a 256-block kernel that updates
// `mb` MB of device vectors (like cg_update), B = a small kernel.  Modes of W's
// last block:
//   0  nothing
//   1  release store of a sequence number at system scope (as now)
//   2  relaxed system-scope stores + s_waitcnt (no L2 writeback)
//   3  release store at agent scope into device memory (control)
//   4  a relaxed system-scope LOAD from mapped host memory, its value stored
//      into device memory (what a kernel's read of a host-side result costs)
// Prints us per pair.   hipcc --offload-arch=gfx950 -O3 -o flag_gap flag_gap.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(2);                                                                  \
        }                                                                                  \
    } while (0)

__global__ void w_kernel(double* v, int64_t n, int mode, unsigned long long* hflag, double* hdata,
                         unsigned long long* dflag, unsigned long long seq, unsigned* ticket) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        v[i] = v[i] * 0.5 + 1.0;
    __syncthreads();
    __shared__ int last;
    if (threadIdx.x == 0)
        last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    __syncthreads();
    if (!last || threadIdx.x != 0) return;
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (mode == 1) {
        hdata[0] = (double)seq;
        __hip_atomic_store(hflag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    } else if (mode == 2) {
        __hip_atomic_store(hdata, (double)seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_s_waitcnt(0);
        __hip_atomic_store(hflag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else if (mode == 3) {
        __hip_atomic_store(dflag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else if (mode == 4) {
        const double h = __hip_atomic_load(hdata, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(dflag, (unsigned long long)h + seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ void b_kernel(const double* v, double* out) {
    if (threadIdx.x == 0) out[blockIdx.x] = v[blockIdx.x];
}

int main(int argc, char** argv) {
    const double mb = argc > 1 ? std::atof(argv[1]) : 3.2;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 400;
    const int64_t n = (int64_t)(mb * 1e6 / 8);
    double *v, *out, *hdata;
    unsigned long long *hflag, *dflag, *hflag_d;
    double* hdata_d;
    unsigned* ticket;
    CK(hipMalloc(&v, n * 8));
    CK(hipMemset(v, 0, n * 8));
    CK(hipMalloc(&out, 4096 * 8));
    CK(hipMalloc(&dflag, 64));
    CK(hipMalloc(&ticket, 64));
    CK(hipMemset(ticket, 0, 64));
    CK(hipHostMalloc((void**)&hflag, 64, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostMalloc((void**)&hdata, 64, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer((void**)&hflag_d, hflag, 0));
    CK(hipHostGetDevicePointer((void**)&hdata_d, hdata, 0));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int mode : {0, 1, 2, 3, 4, 0, 1, 2, 3, 4}) {
        for (int withb : {0, 1}) {
            unsigned long long seq = 1;
            auto pair = [&] {
                hipLaunchKernelGGL(w_kernel, dim3(256), dim3(256), 0, st, v, n, mode, hflag_d, hdata_d, dflag, seq++, ticket);
                if (withb) hipLaunchKernelGGL(b_kernel, dim3(64), dim3(64), 0, st, v, out);
            };
            for (int r = 0; r < 20; ++r) pair();
            CK(hipStreamSynchronize(st));
            CK(hipEventRecord(a, st));
            for (int r = 0; r < reps; ++r) pair();
            CK(hipEventRecord(b, st));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            std::printf("{\"mode\": %d, \"with_b\": %d, \"mb\": %.1f, \"us_per_iter\": %.2f}\n", mode, withb, mb,
                        ms * 1e3 / reps);
            std::fflush(stdout);
        }
    }
    return 0;
}
