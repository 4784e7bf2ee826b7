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

// one thread: the host loop of vamp::precondCG_solver after each step's sums
// red[3k..3k+2] = <r,z>, <r,r>, <v,mu> of system k, applied to the state s
// (in place; nothing if the solve had stopped: s.any == 0).  Returns whether
// the step ran (s.any on entry).
__device__ inline bool cg_decide_into(CgState& s, const double* red, int it, int mask) {
    const bool ran = s.any != 0;  // a step queued after the solve stopped decides (and publishes) nothing
    if (ran) {
        int any = 0;
#pragma unroll
        for (int k = 0; k < kMaxRhs; ++k) {
            if (k >= s.K || !s.active[k]) continue;
            if (!((mask >> k) & 1)) {  // not this step's: unchanged, still running
                any = 1;
                continue;
            }
            s.iters[k] = it + 1 + s.off[k];
            const double rz_new = red[3 * k], rr = red[3 * k + 1], vmu = red[3 * k + 2];
            if (s.onsager[k]) {  // :708-726
                const double ons = s.gam2 * vmu;
                const double rel = ons != 0 ? fabs((ons - s.prev_ons[k]) / ons) : 1;
                if (rel < 1e-8) {
                    s.active[k] = 0;
                    continue;
                }
                s.prev_ons[k] = ons;
            }
            // :731 pow(rz, -1): the correctly rounded reciprocal; glibc's pow
            // differs from it by one ulp on ~0.1% of inputs (tests/powm1_check.c)
            double bt = 1.0 / s.rz[k];
            bt *= rz_new;                 // :736
            s.rz[k] = rz_new;
            const double rel_err = sqrt(rr) / sqrt(s.vv[k]);  // :742-744
            if (rel_err < s.tol) {                            // :750
                s.active[k] = 0;
                continue;
            }
            s.beta[k] = bt;
            if (s.iters[k] >= s.maxit) {  // the solver's loop bound (:697)
                s.active[k] = 0;
                continue;
            }
            any = 1;
        }
        s.any = any;
    }
    return ran;
}

// the decided state s to the host: pack: *flag receives the decision as one
// word (cg_pack), no mirror; else the mirror slot (it & 1) then the flag
__device__ inline void cg_publish(const CgState& s, bool ran, int it, CgMirror* mirror, unsigned long long* flag,
                                  unsigned long long seq, int pack) {
    if (pack) {  // one word, one system-scope store: nothing to order
        if (flag && ran)
            __hip_atomic_store(flag, cg_pack(seq, s.any, s.iters[0], s.iters[1]), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    // the mirror (mapped host memory) written through and drained, then the
    // flag: the host reads the mirror after the flag (no release fence, which
    // would write back this XCD's whole L2 first)
    if (mirror) {
        CgMirror* m = mirror + (it & 1);  // (it >= 0 whenever a mirror is given)
        __hip_atomic_store(&m->seq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&m->any, s.any, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#pragma unroll
        for (int k = 0; k < kMaxRhs; ++k)
            __hip_atomic_store(&m->iters[k], s.iters[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (flag) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// s: the state as *cs holds it (read by the caller in one burst); it is
// written back once (a chain of dependent device loads and stores otherwise:
// this runs at the end of every CG step), then published
__device__ inline void cg_decide_from(CgState s, CgState* cs, const double* red, int it, CgMirror* mirror,
                                      unsigned long long* flag, unsigned long long seq, int mask, int pack = 0) {
    const bool ran = cg_decide_into(s, red, it, mask);
    if (ran) *cs = s;
    cg_publish(s, ran, it, mirror, flag, seq, pack);
}

__device__ inline void cg_decide_body(CgState* cs, const double* red, int it, CgMirror* mirror, unsigned long long* flag,
                                      unsigned long long seq, int mask, int pack = 0) {
    const CgState s = *cs;
    double r[3 * kMaxRhs];
#pragma unroll
    for (int q = 0; q < 3 * kMaxRhs; ++q) r[q] = q < 3 * s.K ? red[q] : 0.0;
    cg_decide_from(s, cs, r, it, mirror, flag, seq, mask, pack);
}

}  // namespace vk
