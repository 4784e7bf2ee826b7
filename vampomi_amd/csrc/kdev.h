// kdev.h — device helpers shared by the gfx950 kernel files (kernels.hip,
// atax_team.hip).  Internal to libvampomi.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.h"

namespace vk {

typedef double v2d __attribute__((ext_vector_type(2)));

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;  // butterfly: every lane holds the same value
}

// Fused finish of a two-stage reduction.  Thread 0 of every block publishes
// its per-block partials with red_put (agent-coherent, write-through stores);
// red_finish drains them (s_waitcnt) and takes a ticket; the LAST block to
// arrive sums the partials in block order, exactly as a separate one-block
// sum kernel would (so results are bitwise those of the two-launch form),
// writes out[0..nq) (device memory or mapped host memory) and re-arms the
// ticket.  No __threadfence: an agent-scope fence writes back the XCD's whole
// L2 (every dirty line of the vectors the kernel just updated), which made
// the fused kernels slower than the two launches (MI355X_MICROARCH.md,
// handoff-flag: drained sc1 payload, then the flag).
__device__ __forceinline__ void red_put(const RedOut& ro, int64_t idx, double v) {
    __hip_atomic_store(ro.part + idx, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wave 0 of every block: after thread 0 has red_put this block's K values at
// part[block*K + k], take the ticket; the last block sums the blocks' values
// in block order per k (lanes stride the blocks, then a butterfly) into
// ro.out[0..K) and re-arms the ticket.  Call from wave 0 only.
template <int K>
__device__ __forceinline__ void ticket_sum_blocks(const RedOut& ro) {
    const int lane = threadIdx.x & 63;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned old = 0;
    if (lane == 0) old = __hip_atomic_fetch_add(ro.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = __shfl(old, 0, 64);
    if (old != gridDim.x - 1) return;
    const int nblk = (int)gridDim.x;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        double t = 0.0;
        for (int b = lane; b < nblk; b += 64)
            t += __hip_atomic_load(ro.part + (int64_t)b * K + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        t = wave_sum(t);
        if (lane == 0) ro.out[k] = t;
    }
    if (lane == 0) __hip_atomic_store(ro.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace vk
