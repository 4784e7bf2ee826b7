// kernels.hip — gfx950 (CDNA4) kernels for the gVAMPomi VAMP hot path.
//
// The design matrix X is fp64, marker-major (each marker = one column of N
// samples, contiguous, README.md:15 / src/data.cpp:127-142), resident in HBM
// with a 128-byte aligned column stride ld.  A.x and A^T.u are HBM-bound
// GEMVs (0.375 flop/B); they stream X with 16-byte-per-lane nontemporal loads
// and never use MFMA.  All reductions are two-stage with fixed block counts
// and fixed summation order, so every result is bitwise reproducible run to
// run and independent of the rank count's effect on scheduling.
#include "kernels.h"
#include "kdev.h"

#include <algorithm>
#include <cstdlib>

#include <hip/hip_ext.h>

#include <hip/hip_runtime.h>

#include <cstdio>
#include <mutex>
#include <string>

namespace vk {

static constexpr int kBlock = 256;   // 4 waves of 64

// ---------------------------------------------------------------------------
// small helpers
// ---------------------------------------------------------------------------
// sum over a 256-thread block; every thread gets the result
__device__ __forceinline__ double block_sum(double v, double* lds4) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) lds4[w] = v;
    __syncthreads();
    return ((lds4[0] + lds4[1]) + lds4[2]) + lds4[3];
}

// red_put (kdev.h) publishes a block's partials; red_finish (below) takes the
// ticket and sums them in block order (the protocol is described in kdev.h).

// Block sums of nq <= NQ values at once, published with red_put at
// part[base + q]: every wave reduces all values in registers, ONE barrier,
// then thread q adds the four wave sums in wave order — the additions of nq
// separate block_sum calls, with one barrier instead of 2*nq.
template <int NQ>
__device__ __forceinline__ void block_put_sums(double (&v)[NQ], int nq, const RedOut& ro, int64_t base) {
    __shared__ double lds[4 * NQ];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < NQ; ++q)
        if (q < nq) v[q] = wave_sum(v[q]);
    if (lane == 0) {
#pragma unroll
        for (int q = 0; q < NQ; ++q)
            if (q < nq) lds[w * NQ + q] = v[q];
    }
    __syncthreads();
    if ((int)threadIdx.x < nq) {
        const int q = threadIdx.x;
        red_put(ro, base + q, ((lds[q] + lds[NQ + q]) + lds[2 * NQ + q]) + lds[3 * NQ + q]);
    }
}

// The last block sums up to 8 results per round: each thread adds its
// blocks' partials of every result (blocks in order), then each result is
// wave-reduced and the four wave sums added in wave order — per result, the
// operations of block_sum, so the sums are bitwise those of one block_sum per
// result, with one barrier round per 8 results instead of one per result.
// Returns true in the last block (after out[] is written; thread 0 wrote it).
// keep (LDS, may be null): thread 0 also leaves the results there (a caller
// that goes on with them in thread 0 then reads no global memory).
// (red_finish's halves, for a launch that finishes two reductions: dots2)
// every partial store of this block is acknowledged before the ticket moves;
// true in the block that brings it to nblocks (block-uniform)
__device__ bool red_ticket(const RedOut& ro, int nblocks) {
    __shared__ int is_last;
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __syncthreads();
    if (threadIdx.x == 0)
        is_last = __hip_atomic_fetch_add(ro.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                  (unsigned)nblocks - 1;
    __syncthreads();
    return is_last;
}

// red_ticket for a block that published nothing: no wait for its own stores
// (block-uniform; the barrier: every wave of the block is past its start)
__device__ bool red_ticket_nowait(const RedOut& ro, int nblocks) {
    __shared__ int is_last;
    __syncthreads();
    if (threadIdx.x == 0)
        is_last = __hip_atomic_fetch_add(ro.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                  (unsigned)nblocks - 1;
    __syncthreads();
    return is_last;
}

// the last block's sums of the nblk blocks' partials at ro.part, into ro.out
// (and keep); finish: then re-arm the ticket and store the host flag
__device__ void red_final(const RedOut& ro, int nq, int nblk, double* keep, bool finish) {
    __shared__ double lds[4 * 8];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int q0 = 0; q0 < nq; q0 += 8) {
        const int nc = nq - q0 < 8 ? nq - q0 : 8;
        double s[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) s[c] = 0.0;
        for (int b = threadIdx.x; b < nblk; b += kBlock) {
#pragma unroll
            for (int c = 0; c < 8; ++c)
                if (c < nc)
                    s[c] += __hip_atomic_load(ro.part + (int64_t)b * nq + q0 + c, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int c = 0; c < 8; ++c)
            if (c < nc) s[c] = wave_sum(s[c]);
        __syncthreads();  // lds of the previous round consumed
        if (lane == 0) {
#pragma unroll
            for (int c = 0; c < 8; ++c)
                if (c < nc) lds[w * 8 + c] = s[c];
        }
        __syncthreads();
        if (threadIdx.x == 0)
            for (int c = 0; c < nc; ++c) {
                const double v = ((lds[c] + lds[8 + c]) + lds[16 + c]) + lds[24 + c];
                const int q = q0 + c;
                double* dst = ro.out2 && q >= ro.split ? ro.out2 + (q - ro.split) : ro.out + q;
                if (ro.flag || !finish)  // mapped host memory: written through, drained before the flag below
                    __hip_atomic_store(dst, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                else
                    *dst = v;
                if (keep) keep[q0 + c] = v;
            }
    }
    if (finish && threadIdx.x == 0) {
        __hip_atomic_store(ro.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // host completion flag, after the results above have landed (drained
        // write-through stores: no release fence, which would first write back
        // this XCD's whole L2, MI355X_MICROARCH.md)
        if (ro.flag) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(ro.flag, ro.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// The last block sums up to 8 results per round: each thread adds its
// blocks' partials of every result (blocks in order), then each result is
// wave-reduced and the four wave sums added in wave order — per result, the
// operations of block_sum, so the sums are bitwise those of one block_sum per
// result, with one barrier round per 8 results instead of one per result.
// Returns true in the last block (after out[] is written; thread 0 wrote it).
// keep (LDS, may be null): thread 0 also leaves the results there (a caller
// that goes on with them in thread 0 then reads no global memory).
__device__ bool red_finish(const RedOut& ro, int nq, double* /*lds4*/, double* keep = nullptr) {
    if (!red_ticket(ro, (int)gridDim.x)) return false;
    red_final(ro, nq, (int)gridDim.x, keep, true);
    return true;
}

__device__ __forceinline__ v2d ld_stream(const double* p) {
    return __builtin_nontemporal_load(reinterpret_cast<const v2d*>(p));
}

__device__ __forceinline__ v2d ld2(const double* p) { return *reinterpret_cast<const v2d*>(p); }

// x^1.5, correctly rounded except in hard midpoint cases (glibc's pow is within
// 0.52 ulp, i.e. the same double in practice).  sqrt is correctly rounded;
// e = x - s^2 and the product's low part are exact through fma, so
// t + (t_lo + x*e/(2s)) is x*sqrt(x) to ~2^-105 before the final rounding.
// g1d's pkdd term needs this: at gam1 = 1e-6 (sigma = 1e6) it feeds a
// cancellation 1 + sigma*(...) ~ 5e-8 that amplifies one ulp ~1e7-fold.
__device__ __forceinline__ double pow_1p5(double x) {
    if (!(x > 0.0) || x == __builtin_huge_val()) return pow(x, 1.5);
    const double s = sqrt(x);
    const double e = __builtin_fma(-s, s, x);
    const double t = x * s;
    const double t_lo = __builtin_fma(x, s, -t);
    return t + (t_lo + x * (e / (2.0 * s)));
}

// exp correctly rounded in practice (the probit denoiser's erfcx; exp_cr.h)
#define EXPCR_FN __device__ __forceinline__
#include "exp_cr.h"

__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

// Irwin-Hall(12) dyadic normal draw; same specification as the oracle's
// orc_gauss_dyadic (oracle/vamp_oracle.c), exactly representable.
__device__ __forceinline__ double gauss_dyadic(uint64_t seed, int64_t i, int64_t j) {
    const uint64_t k = splitmix64(splitmix64(seed ^ 0x4741555353ULL) + (uint64_t)i);
    uint64_t acc = 0;
#pragma unroll
    for (uint64_t t = 0; t < 3; ++t) {
        const uint64_t h = splitmix64(k ^ (((uint64_t)j << 2) | t));
        acc += (h & 0xFFFFULL) + ((h >> 16) & 0xFFFFULL) + ((h >> 32) & 0xFFFFULL) + (h >> 48);
    }
    return (double)(2 * acc + 12) * (1.0 / 131072.0) - 6.0;
}

__device__ __forceinline__ double meth_dyadic(uint64_t seed, int64_t i, int64_t j) {
    const uint64_t hm = splitmix64(splitmix64(seed ^ 0x6D657468ULL) + (uint64_t)i);
    const double mu = (double)(51 + (hm & 1023ULL) % 922ULL) * (1.0 / 1024.0);
    const double sd = (double)(10 + ((hm >> 10) & 127ULL)) * (1.0 / 1024.0);
    const double v = mu + sd * gauss_dyadic(seed ^ 0x5A5A5A5AULL, i, j);
    return v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v);
}

__device__ __forceinline__ int bern_bit(uint64_t seed, int it, int64_t gidx) {
    const uint64_t k = splitmix64(seed ^ 0xB5AD4ECEDA1CE2A9ULL);
    const uint64_t h = splitmix64(k ^ (((uint64_t)(uint32_t)it << 40) ^ (uint64_t)gidx));
    return (int)(h >> 63);
}

static inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ---------------------------------------------------------------------------
// A.x   (data::Ax, src/data.cpp:340-373)
// ---------------------------------------------------------------------------
// Work split.  The rows are cut into tiles of 256*R, and the (tile, marker)
// segments, tiles*M of them, into G equal shares, one per workgroup, with
// G = two workgroups per CU: one resident round in which every CU carries the
// same load (a tile x chunk grid leaves some CUs a third workgroup whenever
// tiles*chunks is not a multiple of the CU count, and those set the kernel's
// time).  Two layouts of the shares:
//  * band plan (tiles <= G): the markers are cut into bands of about 64 MiB
//    of columns, and workgroup g owns the same fraction [g*tiles, (g+1)*tiles)
//    / G of the tile-major (tile, marker-in-band) space of every band: one or
//    two tiles, a run of each band's columns per tile.  All workgroups walk
//    the bands together, so the reads in flight stay inside one band (page
//    translation and DRAM locality: equal contiguous stripes spread over a
//    50 GB matrix ran 4% slower).  A band's column boundaries are dithered
//    per band so floor rounding does not favour the same workgroups.
//  * stripe plan (tiles > G): workgroup g owns the contiguous stripe
//    [g*span, (g+1)*span) of the tile-major space (whole tiles, in order).
// Either way the piece of tile t that workgroup g streams lands in partial
// slot g - lo(t) of that tile, lo(t) = t*sa/sb ((sa, sb) = (G, tiles) for
// bands, (M, span) for stripes).  The plan does not depend on the batch width
// K, so batched and solo passes sum identically.
//
// Within a piece, wave w owns the contiguous slab of 64*R rows
// [tile0 + 64*R*w, ...); lane l owns rows 2l + 128q (q < R/2), i.e. each
// 16-byte load instruction reads 1 KiB contiguous, and the workgroup streams
// 2*R KiB of every marker column.  U markers are loaded before any
// arithmetic (U*R/2 16-byte loads in flight per lane).  Per-sample summation
// order within a slot is the reference's: markers in index order,
// acc += (x - mave_i) * (msig_i * x_i).
// x_k[i] of the pass: p_k[i], or with fusion (FU) z_k[i] + beta_k*p_k[i]
// (the CG direction update, src/vamp.cpp:738-739, as every consumer of the new
// direction forms it).  The kernel stores nothing but its partials, so the
// compiler keeps the per-marker loads scalar.
template <int K, int R, int U, bool NT, bool FU>
__device__ __forceinline__ void ax_piece(const double* __restrict__ X, int64_t ld, int64_t N,
                                         const double* __restrict__ mave, const double* __restrict__ msig,
                                         const CPtrs& xs, const AxFuse& fu, const double (&bk)[K], int64_t j0,
                                         int64_t i0, int64_t i1, double (&acc)[K][R]) {
    constexpr int P = R / 2;  // 16-byte pieces per lane per marker
    int64_t off[P];  // invalid pieces read row 0 of the column (in bounds) and are discarded at the store
#pragma unroll
    for (int q = 0; q < P; ++q) off[q] = (j0 + 128 * q < N) ? 128 * q : -j0;
    const double* col = X + i0 * ld + j0;
    int64_t i = i0;
    for (; i + (U - 1) < i1; i += U) {
        v2d xv[U][P];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int q = 0; q < P; ++q)
                xv[u][q] = NT ? ld_stream(col + (int64_t)u * ld + off[q]) : ld2(col + (int64_t)u * ld + off[q]);
        double xk[U][K];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int k = 0; k < K; ++k)
                xk[u][k] = FU ? fu.z.p[k][i + u] + bk[k] * xs.p[k][i + u] : xs.p[k][i + u];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const double ave = mave[i + u];
            const double sg = msig[i + u];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const double w = sg * xk[u][k];
#pragma unroll
                for (int q = 0; q < P; ++q) {
                    acc[k][2 * q] += (xv[u][q].x - ave) * w;
                    acc[k][2 * q + 1] += (xv[u][q].y - ave) * w;
                }
            }
        }
        col += (int64_t)U * ld;
    }
    for (; i < i1; ++i) {
        v2d xv[P];
#pragma unroll
        for (int q = 0; q < P; ++q) xv[q] = NT ? ld_stream(col + off[q]) : ld2(col + off[q]);
        double xk[K];
#pragma unroll
        for (int k = 0; k < K; ++k) xk[k] = FU ? fu.z.p[k][i] + bk[k] * xs.p[k][i] : xs.p[k][i];
        const double ave = mave[i];
        const double sg = msig[i];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const double w = sg * xk[k];
#pragma unroll
            for (int q = 0; q < P; ++q) {
                acc[k][2 * q] += (xv[q].x - ave) * w;
                acc[k][2 * q + 1] += (xv[q].y - ave) * w;
            }
        }
        col += ld;
    }
}

template <int K, int R>
__device__ __forceinline__ void ax_store(double* __restrict__ part, int64_t slot, int64_t ld, int64_t N, int64_t j0,
                                         const double (&acc)[K][R]) {
    double* dst = part + slot * K * ld + j0;
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
        for (int q = 0; q < R / 2; ++q) {
            if (j0 + 128 * q < N) {
                dst[(int64_t)k * ld + 128 * q] = acc[k][2 * q];
                if (j0 + 128 * q + 1 < N) dst[(int64_t)k * ld + 128 * q + 1] = acc[k][2 * q + 1];
            }
        }
}

template <int K, int R>
__device__ __forceinline__ void ax_zero(double (&acc)[K][R]) {
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
        for (int r = 0; r < R; ++r) acc[k][r] = 0.0;
}

template <int K, int R, int U, bool NT, bool FU>
__global__ __launch_bounds__(kBlock) void ax_partial_kernel(const double* __restrict__ X, int64_t ld,
                                                            int64_t N, int64_t M,
                                                            const double* __restrict__ mave,
                                                            const double* __restrict__ msig, CPtrs xs,
                                                            int64_t tiles, int64_t span, int64_t nband,
                                                            double* __restrict__ part, AxFuse fu) {
    if (fu.gate && !*fu.gate) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t g = blockIdx.x, G = gridDim.x;
    double bk[K];
#pragma unroll
    for (int k = 0; k < K; ++k) bk[k] = FU ? fu.beta[k] : 0.0;
    const int64_t slab = (int64_t)wave * (64 * R) + 2 * lane;  // row offset inside a tile
    double acc[K][R];
    if (nband > 0) {
        // band plan: u-space [g*tiles, (g+1)*tiles) over tiles of G units each
        const int64_t ulo = g * tiles, uhi = ulo + tiles;
        const int64_t tA = ulo / G;
        const int64_t xa0 = ulo - tA * G, xa1 = ((uhi < (tA + 1) * G) ? uhi : (tA + 1) * G) - tA * G;
        const bool hasB = uhi > (tA + 1) * G;
        const int64_t xb1 = uhi - (tA + 1) * G;
        const int64_t jA = tA * (kBlock * R) + slab, jB = jA + kBlock * R;
        double accB[K][R];
        ax_zero<K, R>(acc);
        ax_zero<K, R>(accB);
        // boundaries in whole groups of U markers (full-width load trips); the
        // last group boundary stands for M (the M % U leftover markers)
        const int64_t Mu = M / U;
        for (int64_t p = 0; p < nband; ++p) {
            const int64_t c = p * Mu / nband, w = (p + 1) * Mu / nband - c;
            const int64_t phi = (int64_t)(((uint64_t)p * 0x9E3779B97F4A7C15ULL) >> 40) % G;  // dither in [0, G)
            if (jA < N) {
                const int64_t u0 = c + (xa0 * w + phi) / G, u1 = c + (xa1 * w + phi) / G;
                ax_piece<K, R, U, NT, FU>(X, ld, N, mave, msig, xs, fu, bk, jA, u0 == Mu ? M : u0 * U,
                                      u1 == Mu ? M : u1 * U, acc);
            }
            if (hasB && jB < N) {
                const int64_t u1 = c + (xb1 * w + phi) / G;
                ax_piece<K, R, U, NT, FU>(X, ld, N, mave, msig, xs, fu, bk, jB, c * U, u1 == Mu ? M : u1 * U,
                                      accB);
            }
        }
        if (jA < N) ax_store<K, R>(part, g - (tA * G) / tiles, ld, N, jA, acc);
        if (hasB && jB < N) ax_store<K, R>(part, g - ((tA + 1) * G) / tiles, ld, N, jB, accB);
        return;
    }
    // stripe plan
    const int64_t total = tiles * M;
    int64_t pos = g * span;
    const int64_t end = (pos + span < total) ? pos + span : total;
    while (pos < end) {
        const int64_t t = pos / M;
        const int64_t i0 = pos - t * M;
        const int64_t i1 = (i0 + (end - pos) < M) ? i0 + (end - pos) : M;
        pos += i1 - i0;
        const int64_t j0 = t * (kBlock * R) + slab;
        if (j0 >= N) continue;
        ax_zero<K, R>(acc);
        ax_piece<K, R, U, NT, FU>(X, ld, N, mave, msig, xs, fu, bk, j0, i0, i1, acc);
        ax_store<K, R>(part, g - (t * M) / span, ld, N, j0, acc);
    }
}

// tuning table (rows per lane R, markers in flight U, nontemporal loads)
struct AxVariant { int R, U; bool NT; };
static constexpr AxVariant kAxVariants[] = {
    {2, 8, true}, {2, 8, false}, {4, 4, true}, {4, 8, true}, {8, 4, true}, {2, 4, true}, {2, 12, true},
};
static constexpr int kNumAxVariants = sizeof(kAxVariants) / sizeof(kAxVariants[0]);
// default 0: R=2, U=8, nontemporal (tools/kbench.py)

int ax_variant_count() { return kNumAxVariants + 1; }  // + kAxTeam
bool ax_variant_ok(int v) { return v == kAxDefault || (v >= 0 && v < kNumAxVariants) || v == kAxTeam; }
static_assert(kAxTeam == kNumAxVariants, "the team plan numbers after the tile variants");

static int device_cus() {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        return 256;
    return cus;
}

AxPlan ax_plan(int64_t N, int64_t M, int variant) { return ax_plan_for(N, M, device_cus(), variant); }

AxPlan ax_plan_for(int64_t N, int64_t M, int cus, int variant) {
    AxPlan p;
    if (variant == kAxDefault || variant == kAxTeam) {
        if (ax_team_plan(N, M, cus, &p) && (variant == kAxTeam || p.T >= kAxTeamMinT)) return p;
        p = AxPlan{};
    }
    p.variant = variant >= 0 && variant < kNumAxVariants ? variant : 0;
    p.rows = (int64_t)kBlock * kAxVariants[p.variant].R;
    p.tiles = cdiv(N, p.rows);
    p.total = p.tiles * M;
    // tuning experiments: VAMPOMI_AX_WPC workgroups per CU, VAMPOMI_AX_BANDSEG
    // segments per workgroup per band (0: stripe plan)
    int64_t wpc = 2, bandseg = 32;
    if (const char* f = std::getenv("VAMPOMI_AX_WPC")) wpc = std::max(1, std::atoi(f));
    if (const char* f = std::getenv("VAMPOMI_AX_BANDSEG")) bandseg = std::max(0, std::atoi(f));
    int64_t G = std::min<int64_t>(wpc * cus, cdiv(p.total, 64));  // >= 64 segments per workgroup
    if (G < 1) G = 1;
    p.span = cdiv(p.total, G);
    if (p.tiles <= G && bandseg > 0 && M >= (int64_t)kAxVariants[p.variant].U) {
        p.groups = (int)G;
        p.nband = std::max<int64_t>(1, std::min<int64_t>(M / kAxVariants[p.variant].U, p.total / (bandseg * G)));
        p.sa = G;
        p.sb = p.tiles;
    } else {
        p.groups = (int)cdiv(p.total, p.span);
        p.nband = 0;
        p.sa = M;
        p.sb = p.span;
    }
    int64_t ns = 1;
    for (int64_t t = 0; t < p.tiles; ++t) ns = std::max(ns, ax_slots(p, t));
    p.nslots = (int)ns;
    return p;
}

// launches go through hipExtLaunchKernelGGL: the optional start / stop events
// are written by the kernel's own dispatch (no extra marker packets around it)
template <int K, int R, int U, bool NT>
static void launch_ax(const Shard& s, const AxPlan& pl, CPtrs x, double* part, hipStream_t st, const Timing& tm,
                      const AxFuse& fu) {
    if (fu.z.p[0])
        hipExtLaunchKernelGGL((ax_partial_kernel<K, R, U, NT, true>), dim3(pl.groups), dim3(kBlock), 0, st, tm.start,
                              tm.stop, 0, s.X, s.ld, s.N, s.M, s.mave, s.msig, x, pl.tiles, pl.span, pl.nband, part,
                              fu);
    else
        hipExtLaunchKernelGGL((ax_partial_kernel<K, R, U, NT, false>), dim3(pl.groups), dim3(kBlock), 0, st,
                              tm.start, tm.stop, 0, s.X, s.ld, s.N, s.M, s.mave, s.msig, x, pl.tiles, pl.span,
                              pl.nband, part, fu);
}

template <int K>
static bool launch_ax_v(int v, const Shard& s, const AxPlan& pl, CPtrs x, double* part, hipStream_t st,
                        const Timing& tm, const AxFuse& fu) {
    switch (v) {
        case 0: launch_ax<K, 2, 8, true>(s, pl, x, part, st, tm, fu); return true;
        case 1: launch_ax<K, 2, 8, false>(s, pl, x, part, st, tm, fu); return true;
        case 2: launch_ax<K, 4, 4, true>(s, pl, x, part, st, tm, fu); return true;
        case 3: launch_ax<K, 4, 8, true>(s, pl, x, part, st, tm, fu); return true;
        case 4: launch_ax<K, 8, 4, true>(s, pl, x, part, st, tm, fu); return true;
        case 5: launch_ax<K, 2, 4, true>(s, pl, x, part, st, tm, fu); return true;
        case 6: launch_ax<K, 2, 12, true>(s, pl, x, part, st, tm, fu); return true;
        default: return false;
    }
}

hipError_t ax_partial(const Shard& s, const AxPlan& pl, int K, CPtrs x, double* part, hipStream_t st,
                      const Timing& tm, const AxFuse& fu) {
    if (pl.T > 0) return ax_team(s, pl, K, x, part, st, tm, fu);
    if (pl.rows != (int64_t)kBlock * kAxVariants[pl.variant].R || pl.total != pl.tiles * s.M ||
        pl.tiles * pl.rows < s.N)
        return hipErrorInvalidValue;  // plan made for another shape
    bool ok = false;
    switch (K) {
        case 1: ok = launch_ax_v<1>(pl.variant, s, pl, x, part, st, tm, fu); break;
        case 2: ok = launch_ax_v<2>(pl.variant, s, pl, x, part, st, tm, fu); break;
        case 3: ok = launch_ax_v<3>(pl.variant, s, pl, x, part, st, tm, fu); break;
        case 4: ok = launch_ax_v<4>(pl.variant, s, pl, x, part, st, tm, fu); break;
        default: break;
    }
    if (!ok) return hipErrorInvalidValue;
    return hipGetLastError();
}

// Stage 2: out_k[j] = sum over tile(j)'s slots of part[s][k][j].  A 512-thread
// block covers 64 consecutive samples (one wave per slot group, coalesced
// across lanes); group q sums its contiguous slot range in index order, then
// the 8 group sums are added in group order: a fixed tree, short dependent
// chains.
constexpr int kRedGroups = 8;
__global__ __launch_bounds__(64 * kRedGroups) void ax_reduce_kernel(int K, int64_t N, int64_t ld, int64_t sa,
                                                                    int64_t rows, int64_t sb,
                                                                    const double* __restrict__ part, Ptrs out,
                                                                    double div, const int* gate) {
    if (gate && !*gate) return;
    __shared__ double lds[kRedGroups][64];
    const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int64_t e = (int64_t)blockIdx.x * 64 + lane;
    const bool valid = e < (int64_t)K * N;
    const int k = valid ? (int)(e / N) : 0;
    const int64_t j = valid ? e - (int64_t)k * N : 0;
    const int64_t t = j / rows;
    const int nslots = (int)(((t + 1) * sa - 1) / sb - (t * sa) / sb + 1);
    const int per = (nslots + kRedGroups - 1) / kRedGroups;
    const int c0 = g * per, c1 = (c0 + per < nslots) ? c0 + per : nslots;
    const int64_t stride = (int64_t)K * ld;
    const double* p = part + (int64_t)k * ld + j;
    double s = 0.0;
    if (valid) {
        int c = c0;
        for (; c + 4 <= c1; c += 4) {
            const double q0 = p[(int64_t)(c + 0) * stride], q1 = p[(int64_t)(c + 1) * stride];
            const double q2 = p[(int64_t)(c + 2) * stride], q3 = p[(int64_t)(c + 3) * stride];
            s += q0;
            s += q1;
            s += q2;
            s += q3;
        }
        for (; c < c1; ++c) s += p[(int64_t)c * stride];
    }
    lds[g][lane] = s;
    __syncthreads();
    if (g == 0 && valid) {
        double t2 = lds[0][lane];
#pragma unroll
        for (int q = 1; q < kRedGroups; ++q) t2 += lds[q][lane];
        if (div > 0.0) t2 /= div;  // src/data.cpp:369-370: Ax_total[i] /= sqrt(N)
        out.p[k][j] = t2;
    }
}

hipError_t ax_reduce(const AxPlan& pl, int K, int64_t N, int64_t ld, const double* part, Ptrs out, double div,
                     hipStream_t st, const int* gate) {
    const int64_t n = (int64_t)K * N;
    hipLaunchKernelGGL(ax_reduce_kernel, dim3((unsigned)cdiv(n, 64)), dim3(64 * kRedGroups), 0, st, K, N, ld,
                       pl.sa, pl.rows, pl.sb, part, out, div, gate);
    return hipGetLastError();
}

// A pure read stream (the read ceiling of vampomi_dev_read_ceiling; the same
// shapes as tools/hbm_ceiling's lock and chunk variants).  The sums feed a
// store that never happens (the comparison with the NaN `never`), so no load
// is dead.
__global__ __launch_bounds__(512) void stream_lock_kernel(const double* __restrict__ x, int64_t units,
                                                          double never, double* __restrict__ sink) {
    constexpr int U = 8;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t b = units * blockIdx.x / gridDim.x * 1024, e = units * (blockIdx.x + 1) / gridDim.x * 1024;
    double a0 = 0.0, a1 = 0.0;
    int64_t j = b + 128 * wave + 2 * lane;
    for (; j + 1024 * (U - 1) < e; j += 1024 * U) {
        v2d v[U];
#pragma unroll
        for (int t = 0; t < U; ++t) v[t] = __builtin_nontemporal_load(reinterpret_cast<const v2d*>(x + j + 1024 * t));
#pragma unroll
        for (int t = 0; t < U; ++t) {
            a0 += v[t].x;
            a1 += v[t].y;
        }
        __syncthreads();
    }
    for (; j < e; j += 1024) {
        const v2d v = __builtin_nontemporal_load(reinterpret_cast<const v2d*>(x + j));
        a0 += v.x;
        a1 += v.y;
    }
    if (a0 + a1 == never) sink[0] = a0;
}

__global__ __launch_bounds__(256) void stream_chunk_kernel(const double* __restrict__ x, int64_t nchunks,
                                                           double never, double* __restrict__ sink) {
    constexpr int U = 8;
    constexpr int64_t CW = 1 << 17;  // 1 MiB of doubles per wave
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= nchunks) return;
    double a0 = 0.0, a1 = 0.0;
    for (int64_t j = w * CW + 2 * lane; j < (w + 1) * CW; j += 128 * U) {
        v2d v[U];
#pragma unroll
        for (int t = 0; t < U; ++t) v[t] = __builtin_nontemporal_load(reinterpret_cast<const v2d*>(x + j + 128 * t));
#pragma unroll
        for (int t = 0; t < U; ++t) {
            a0 += v[t].x;
            a1 += v[t].y;
        }
    }
    if (a0 + a1 == never) sink[0] = a0;
}

hipError_t stream_read(const double* x, int64_t n, int kind, int cus, hipStream_t st, const Timing& tm,
                       double* sink, double* bytes) {
    const double never = __builtin_nan("");
    if (kind == 0) {
        const int64_t units = n / 1024;
        if (units < cus) return hipErrorInvalidValue;
        *bytes = 8.0 * (double)(units * 1024);
        hipExtLaunchKernelGGL(stream_lock_kernel, dim3(cus), dim3(512), 0, st, tm.start, tm.stop, 0, x, units, never,
                              sink);
    } else {
        const int64_t nch = n / (1 << 17);
        if (nch < 1) return hipErrorInvalidValue;
        *bytes = 8.0 * (double)(nch << 17);
        hipExtLaunchKernelGGL(stream_chunk_kernel, dim3((unsigned)((nch + 3) / 4)), dim3(256), 0, st, tm.start,
                              tm.stop, 0, x, nch, never, sink);
    }
    return hipGetLastError();
}

__global__ void vec_div_kernel(int K, int64_t n, Ptrs v, double div, Ptrs dst) {
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= (int64_t)K * n) return;
    const int k = (int)(e / n);
    const int64_t j = e - (int64_t)k * n;
    dst.p[k][j] = v.p[k][j] / div;
}

hipError_t vec_div(int K, int64_t n, int64_t /*ld*/, Ptrs v, double div, hipStream_t st, const Ptrs* dst) {
    hipLaunchKernelGGL(vec_div_kernel, dim3((unsigned)cdiv((int64_t)K * n, kBlock)), dim3(kBlock), 0, st, K, n, v,
                       div, dst ? *dst : v);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// A^T.u  (data::ATx + data::dot_product, src/data.cpp:294-333)
// ---------------------------------------------------------------------------
// A wave owns G consecutive markers (workgroups of two waves, dispatched in
// order: the dispatcher balances the CUs); lanes stride the samples two at a time,
// so each load instruction reads 1 KiB of one column, UJ such 128-row steps
// per loop trip.  Every u value loaded serves G markers.  The wave's partial
// dots are reduced with an xor butterfly; mode 1 fuses the lmmse_mult
// epilogue (src/vamp.cpp:656-659).
template <int G, int K, int MODE, int UJ, bool NT>
__global__ __launch_bounds__(kBlock) void atx_kernel(const double* __restrict__ X, int64_t ld, int64_t N, int64_t M,
                                                     const double* __restrict__ mave,
                                                     const double* __restrict__ msig, CPtrs u, Ptrs out,
                                                     double scale, double tau, double gam2, CPtrs pv,
                                                     const int* __restrict__ gate, CPtrs zf,
                                                     const double* __restrict__ beta, Ptrs sraw) {
    if (gate && !*gate) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t m0 = ((int64_t)blockIdx.x * (blockDim.x >> 6) + wave) * G;
    double acc[G][K];
    double mu[G];
    const double* col[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int64_t m = (m0 + g < M) ? m0 + g : M - 1;  // clamp: in-bounds, discarded
        mu[g] = mave[m];
        col[g] = X + m * ld;
#pragma unroll
        for (int k = 0; k < K; ++k) acc[g][k] = 0.0;
    }
    int64_t j = 2 * lane;
    for (; j + 128 * (UJ - 1) < N; j += 128 * UJ) {
        v2d uu[UJ][K], xx[UJ][G];
#pragma unroll
        for (int t = 0; t < UJ; ++t)
#pragma unroll
            for (int g = 0; g < G; ++g) xx[t][g] = NT ? ld_stream(col[g] + j + 128 * t) : ld2(col[g] + j + 128 * t);
#pragma unroll
        for (int t = 0; t < UJ; ++t)
#pragma unroll
            for (int k = 0; k < K; ++k) uu[t][k] = ld2(u.p[k] + j + 128 * t);
#pragma unroll
        for (int g = 0; g < G; ++g) {
#pragma unroll
            for (int t = 0; t < UJ; ++t) {
                const double d0 = xx[t][g].x - mu[g], d1 = xx[t][g].y - mu[g];
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    acc[g][k] += d0 * uu[t][k].x;
                    acc[g][k] += d1 * uu[t][k].y;
                }
            }
        }
    }
    for (; j < N; j += 128) {  // tail; j+1 may be the zero pad row (u pad is zero too)
        v2d uu[K], xx[G];
#pragma unroll
        for (int g = 0; g < G; ++g) xx[g] = NT ? ld_stream(col[g] + j) : ld2(col[g] + j);
#pragma unroll
        for (int k = 0; k < K; ++k) uu[k] = ld2(u.p[k] + j);
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const double d0 = xx[g].x - mu[g], d1 = xx[g].y - mu[g];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                acc[g][k] += d0 * uu[k].x;
                acc[g][k] += d1 * uu[k].y;
            }
        }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const double dot = wave_sum(acc[g][k]);
            const int64_t m = m0 + g;
            if (m < M && lane == 0) {
                double val = msig[m] * dot;  // sigma_inv * dpa
                val *= scale;                // ATx[mloc] *= 1/sqrt(N)
                if (MODE == 1 && sraw.p[0]) sraw.p[k][m] = val;  // A^T(A p) itself (CG recurrences)
                if (MODE == 1) {
                    const double pk = zf.p[0] ? zf.p[k][m] + beta[k] * pv.p[k][m] : pv.p[k][m];
                    val *= tau;        // res[i] *= tau
                    val += gam2 * pk;  // res[i] += gam2 * v[i]
                }
                out.p[k][m] = val;
            }
        }
    }
}

// tuning table (markers per wave G, 128-row steps per trip UJ, nontemporal)
struct AtxVariant { int G, UJ; bool NT; };
static constexpr AtxVariant kAtxVariants[] = {
    {4, 2, true}, {4, 2, false}, {2, 2, true}, {8, 2, true}, {4, 4, true}, {4, 1, true}, {8, 1, true}, {2, 4, true},
};
static constexpr int kNumAtxVariants = sizeof(kAtxVariants) / sizeof(kAtxVariants[0]);
// -1 (the default): per-K choice measured on MI355X at C2 (tools/kbench.py,
// profiles/r01_kbench.json): K=1 -> G=2,UJ=2 (6.86 TB/s); K>=2 -> G=4,UJ=4 (6.70 TB/s at K=2)
static int atx_variant_for(int variant, int K) { return variant >= 0 ? variant : (K == 1 ? 2 : 4); }

int atx_variant_count() { return kNumAtxVariants; }
bool atx_variant_ok(int v) { return v >= -1 && v < kNumAtxVariants; }

// rocprofv3 kernel name of the launch that ax_partial / atx would make now
std::string kernel_name(int which, int K, int mode, int variant) {
    char b[160];
    if (which == 0) {
        const AxVariant& v = kAxVariants[variant >= 0 && variant < kNumAxVariants ? variant : 0];
        std::snprintf(b, sizeof b, "ax_partial_kernel<%d, %d, %d, %s, %s>", K, v.R, v.U, v.NT ? "true" : "false",
                      mode == 1 ? "true" : "false");
    } else {
        const AtxVariant& v = kAtxVariants[atx_variant_for(variant, K)];
        std::snprintf(b, sizeof b, "atx_kernel<%d, %d, %d, %d, %s>", v.G, K, mode, v.UJ, v.NT ? "true" : "false");
    }
    return b;
}

int atx_blocks(int64_t M, int K, int variant) { return (int)cdiv(M, 4 * kAtxVariants[atx_variant_for(variant, K)].G); }

template <int G, int K, int MODE, int UJ, bool NT>
static void launch_atx(const Shard& s, CPtrs u, Ptrs out, double scale, double tau, double gam2, CPtrs p,
                       const int* gate, CPtrs zf, const double* beta, Ptrs sraw, hipStream_t st, const Timing& tm) {
    // two waves per workgroup: a finer dispatch grain than four (C2: -2..4%,
    // profiles/r01_kbench_ax_swap.txt); VAMPOMI_ATX_WPB: tuning experiments
    static const int wpb = std::getenv("VAMPOMI_ATX_WPB") ? std::max(1, std::min(4, std::atoi(std::getenv("VAMPOMI_ATX_WPB")))) : 2;
    hipExtLaunchKernelGGL((atx_kernel<G, K, MODE, UJ, NT>), dim3((unsigned)cdiv(s.M, wpb * G)), dim3(64 * wpb), 0, st,
                          tm.start, tm.stop, 0, s.X, s.ld, s.N, s.M, s.mave, s.msig, u, out, scale, tau, gam2, p,
                          gate, zf, beta, sraw);
}

template <int K, int MODE>
static bool launch_atx_v(int v, const Shard& s, CPtrs u, Ptrs out, double scale, double tau, double gam2, CPtrs p,
                         const int* gate, CPtrs zf, const double* beta, Ptrs sraw, hipStream_t st, const Timing& tm) {
    switch (v) {
        case 0: launch_atx<4, K, MODE, 2, true>(s, u, out, scale, tau, gam2, p, gate, zf, beta, sraw, st, tm); return true;
        case 1: launch_atx<4, K, MODE, 2, false>(s, u, out, scale, tau, gam2, p, gate, zf, beta, sraw, st, tm); return true;
        case 2: launch_atx<2, K, MODE, 2, true>(s, u, out, scale, tau, gam2, p, gate, zf, beta, sraw, st, tm); return true;
        case 3: launch_atx<8, K, MODE, 2, true>(s, u, out, scale, tau, gam2, p, gate, zf, beta, sraw, st, tm); return true;
        case 4: launch_atx<4, K, MODE, 4, true>(s, u, out, scale, tau, gam2, p, gate, zf, beta, sraw, st, tm); return true;
        case 5: launch_atx<4, K, MODE, 1, true>(s, u, out, scale, tau, gam2, p, gate, zf, beta, sraw, st, tm); return true;
        case 6: launch_atx<8, K, MODE, 1, true>(s, u, out, scale, tau, gam2, p, gate, zf, beta, sraw, st, tm); return true;
        case 7: launch_atx<2, K, MODE, 4, true>(s, u, out, scale, tau, gam2, p, gate, zf, beta, sraw, st, tm); return true;
        default: return false;
    }
}

hipError_t atx(const Shard& s, int K, CPtrs u, Ptrs out, double scale, int mode, double tau, double gam2, CPtrs p,
               hipStream_t st, int variant, const Timing& tm, const int* gate, CPtrs zf, const double* beta,
               Ptrs sraw) {
    if (!atx_variant_ok(variant)) return hipErrorInvalidValue;
    const int v = atx_variant_for(variant, K);
    bool ok = false;
    if (mode == 0) {
        switch (K) {
            case 1: ok = launch_atx_v<1, 0>(v, s, u, out, scale, tau, gam2, p, gate, zf, beta, sraw, st, tm); break;
            case 2: ok = launch_atx_v<2, 0>(v, s, u, out, scale, tau, gam2, p, gate, zf, beta, sraw, st, tm); break;
            case 3: ok = launch_atx_v<3, 0>(v, s, u, out, scale, tau, gam2, p, gate, zf, beta, sraw, st, tm); break;
            default: break;
        }
    } else {
        switch (K) {
            case 1: ok = launch_atx_v<1, 1>(v, s, u, out, scale, tau, gam2, p, gate, zf, beta, sraw, st, tm); break;
            case 2: ok = launch_atx_v<2, 1>(v, s, u, out, scale, tau, gam2, p, gate, zf, beta, sraw, st, tm); break;
            case 3: ok = launch_atx_v<3, 1>(v, s, u, out, scale, tau, gam2, p, gate, zf, beta, sraw, st, tm); break;
            default: break;
        }
    }
    if (!ok) return hipErrorInvalidValue;
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// One-pass CG operator (kernels.h: atax).  A^T q (data::ATx,
// src/data.cpp:294-333, with the lmmse_mult epilogue src/vamp.cpp:656-659)
// and A d (data::Ax, src/data.cpp:340-373) from one read of X.
// ---------------------------------------------------------------------------
// One workgroup per CU (kOpWaves waves) owns whole columns: markers
// [b*M/grid, (b+1)*M/grid).  Wave w, lane l owns rows 1024*s + 128*w + 2l
// (+1), s < S = ceil(N/1024): every load instruction reads 1 KiB contiguous
// of one column.  Per marker i (a column of X in registers, the next one
// loading):
//   t_i = msig_i * sum_j (X_ij - mave_i) q_j * scale   (the wave partials
//         meet in LDS, one barrier; every wave sums them in wave order)
//   d_i = t_i*tau + gam2*p_i,  c_i = msig_i*d_i
//   acc_j += (X_ij - mave_i) * c_i                      (registers)
// q = A r/diag [+ beta*q_old] is formed once per launch into LDS (K*N
// doubles, each thread only ever reads its own rows: no barrier), so
// K*N <= kOpLdsDoubles.  The column is read from HBM once for both products;
// the workgroup's A d partial (K*N) goes to its slot, op_reduce sums the
// slots in order.  Summation orders are fixed, results bitwise reproducible.
static constexpr int kOpWaves = 8;               // 2 per SIMD: <= 256 VGPRs
static constexpr int kOpThreads = 64 * kOpWaves;
static constexpr int kOpRows = 128 * kOpWaves;   // rows per load step of the workgroup
static constexpr int kOpMaxS = 10;               // rows per workgroup <= kOpRows*kOpMaxS = 10,240
static constexpr int64_t kOpLdsDoubles = 20480 - 2 - 2 * kOpWaves * 2;  // the CU's 160 KiB of LDS

static bool whole_column_ok(int64_t N) {
    return N >= 1 && kOpMaxK * (N + 2) <= kOpLdsDoubles && (N + kOpRows - 1) / kOpRows <= kOpMaxS;
}

// The default: whole columns per workgroup (team size 1, the team kernel
// without a hand-off: 585 us against 646 us for atax_kernel at C2, K = 2,
// profiles/r02c_op_sweep.txt) while the rows fit one workgroup, else the
// smallest team whose members' rows fit the registers (configuration 7:
// 4 columns prefetched, a lag of 5 steps, polls 2 steps ahead, measured best
// at N = 50,000 and 100,000, profiles/r02c_op_sweep.txt; with the teams'
// columns interleaved, team t taking columns t, t + nteams, ..., so that all
// teams stream neighbouring columns instead of 8-16 ranges gigabytes apart:
// 10-13 % faster at the C3 shard, config 4 whole and 240 GB,
// profiles/r02i_op_interleave.txt).
bool op_plan(int64_t N, int64_t M, int cus, int variant, OpPlan* out) {
    if (N < 1 || cus < 1) return false;
    if (variant == kOpDefault) {
        // one workgroup per column range (team size 1): two columns prefetched
        // where they fit the registers (S <= 8), else one, up to S = 9; at
        // S = 10 (252-256 VGPRs) a team of 4 is faster (C2, N = 10,000, K = 2:
        // 585-588 against 597 us; N = 9,216, S = 9: 543 against 560 us for the
        // team; profiles/r02g_op_plans_by_N.txt)
        OpPlan p{};
        if ((team_plan(N, M, cus, 1, 1, &p) || team_plan(N, M, cus, 1, 0, &p)) && p.S <= 9) {
            *out = p;
            return true;
        }
    }
    if (variant == kOpDefault) {
        // just past one workgroup's rows (9,216 < N <= 10,752, C2 among them): a
        // team of 2 with six loads per lane (configuration 5, round 3's 12: F = 2, L = 3,
        // 253 VGPRs) beats the team of 4 (C2: 589.7-590.2 against 594.5-595.8 us
        // per launch in VAMP, 192.0-192.3 against 191.0-191.3 it/s, three rounds
        // on one box, profiles/r03pl_c2_plans.txt)
        OpPlan p{};
        if (team_plan(N, M, cus, 2, 5, &p)) {
            *out = p;
            return true;
        }
    }
    if (variant == 0) {
        if (!whole_column_ok(N)) return false;
        OpPlan p{};
        p.S = (int)std::max<int64_t>(1, (N + kOpRows - 1) / kOpRows);
        p.grid = (int)std::max<int64_t>(1, std::min<int64_t>(cus, M));
        p.nslots = p.grid;
        p.T = 0;
        *out = p;
        return true;
    }
    if (variant >= 1000) return team_plan(N, M, cus, (variant - 1000) / 100, variant % 100, out);  // 1000 + T*100 + cfg
    if (variant > 0) return team_plan(N, M, cus, variant / 10, variant % 10, out);
    for (int cfg : {2, 4}) {  // then fewer columns in flight for one more load per lane (S <= 5)
        for (int T = 2; T <= 32; T *= 2) {
            OpPlan p{};
            if (!team_plan(N, M, cus, T, cfg, &p)) continue;
            *out = p;
            return true;
        }
    }
    return false;  // N beyond 32 x 5 x 896 rows: the CG step keeps two passes (pcg.cpp)
}

bool op_supported(int64_t N, int K) {
    OpPlan p{};
    return K >= 1 && K <= kOpMaxK && op_plan(N, 1 << 20, 256, kOpDefault, &p);
}

// one column in registers: its X rows and the marker's mean
template <int K, int S>
struct OpCol {
    v2d x[S];
    double mu;
};

template <int K, int S>
__global__ __launch_bounds__(kOpThreads) void atax_kernel(const double* __restrict__ X, int64_t ld, int64_t N,
                                                          int64_t M, const double* __restrict__ mave,
                                                          const double* __restrict__ msig, OpArgs a,
                                                          const int* __restrict__ gate) {
    if (gate && !*gate) return;
    // LDS: q (K x NL; each thread only ever touches its own rows), a zero
    // pair, then 2 x kOpWaves x K dot partials
    extern __shared__ double q_lds[];
    const int NL = (int)N + 1 + ((int)N & 1);  // even stride; q[N] = 0 (the odd-N pad row)
    const int zslot = K * NL;
    double* s_part = q_lds + zslot + 2;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t mb = (int64_t)blockIdx.x * M / gridDim.x, me = (int64_t)(blockIdx.x + 1) * M / gridDim.x;
    // row of this thread in step s: jb + kOpRows*s (recomputed, not kept in registers)
    const int jb = 128 * wave + 2 * lane;
    const int n32 = (int)N;
#define OP_J(s) (jb + kOpRows * (s))
#define OP_OK(s) (OP_J(s) < n32)
    if (threadIdx.x == 0) {  // rows past N meet q = 0: the zero pair, and q[N] for odd N
        q_lds[zslot] = 0.0;
        q_lds[zslot + 1] = 0.0;
#pragma unroll
        for (int k = 0; k < K; ++k) q_lds[k * NL + n32] = 0.0;
    }
    v2d acc[K][S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            acc[k][s] = v2d{0.0, 0.0};
            if (!OP_OK(s)) continue;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int jj = OP_J(s) + h;
                if (jj < N) {
                    double q = a.ar.p[k][jj] / a.diag;              // A z = A r / diag
                    if ((a.fuse >> k) & 1) q = q + a.beta[k] * a.qo.p[k][jj];  // A p = A z + beta A p
                    q_lds[k * NL + jj] = q;
                }
            }
        }
    }
    __syncthreads();  // the zero pair and q[N] (thread 0) are read by other threads
    double bk[K];
#pragma unroll
    for (int k = 0; k < K; ++k) bk[k] = ((a.fuse >> k) & 1) ? a.beta[k] : 0.0;
    double dpacc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) dpacc[k] = 0.0;
    // columns in registers: three where they fit beside acc, else two
    constexpr int NB = K * S <= 16 ? 3 : 2;
    OpCol<K, S> cb[NB];
    auto load = [&](OpCol<K, S>& c, int64_t m) {
        const char* col = reinterpret_cast<const char*>(X + m * ld);
#pragma unroll
        for (int s = 0; s < S; ++s)
            if (OP_OK(s)) c.x[s] = __builtin_nontemporal_load(reinterpret_cast<const v2d*>(col + (unsigned)(OP_J(s) * 8)));
        c.mu = mave[m];
    };
    // dot partials of column c -> s_part[par][wave][k]
    auto dots = [&](const OpCol<K, S>& c, int par) {
        double v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = 0.0;
#pragma unroll
        for (int s = 0; s < S; ++s) {
            if (!OP_OK(s)) continue;
            const double dx = c.x[s].x - c.mu, dy = c.x[s].y - c.mu;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const v2d q = *reinterpret_cast<const v2d*>(q_lds + k * NL + OP_J(s));  // q[N] = 0 for odd N
                v[k] += dx * q.x;
                v[k] += dy * q.y;
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {  // the K butterflies interleaved: their exchanges fly together
            double t[K];
#pragma unroll
            for (int k = 0; k < K; ++k) t[k] = __shfl_xor(v[k], o, 64);
#pragma unroll
            for (int k = 0; k < K; ++k) v[k] += t[k];
        }
        if (lane == 0) {
#pragma unroll
            for (int k = 0; k < K; ++k) s_part[(par * kOpWaves + wave) * K + k] = v[k];
        }
    };
    // the column's d (all waves, identically) and acc += (x - mave)*msig*d
    auto finish = [&](const OpCol<K, S>& c, int64_t m, int par) {
        const double sg = msig[m];
        double cc[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            double dot = 0.0;
#pragma unroll
            for (int w = 0; w < kOpWaves; ++w) dot += s_part[(par * kOpWaves + w) * K + k];
            double t = sg * dot;  // sigma_inv * dpa
            t *= a.scale;         // ATx[mloc] *= 1/sqrt(N)
            double pk = a.p.p[k][m];
            if ((a.fuse >> k) & 1) pk = a.z.p[k][m] + bk[k] * pk;  // p = z + beta p
            double val = t * a.tau;  // res[i] *= tau
            val += a.gam2 * pk;      // res[i] += gam2 * v[i]
            if (threadIdx.x == 0) {
                if (a.sraw.p[0]) a.sraw.p[k][m] = t;
                a.d.p[k][m] = val;
            }
            dpacc[k] += val * pk;
            cc[k] = sg * val;  // Ax: (x - mave) * (msig * x_i)
        }
#pragma unroll
        for (int s = 0; s < S; ++s) {
            if (!OP_OK(s)) continue;
            const double dx = c.x[s].x - c.mu, dy = c.x[s].y - c.mu;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                acc[k][s].x += dx * cc[k];
                acc[k][s].y += dy * cc[k];
            }
        }
    };
    // NB columns in registers: m is finished while m+1 .. m+NB-1 load; the
    // buffer m frees takes m+NB.  Dot partials alternate between two LDS slots.
    auto step = [&](OpCol<K, S>& cur, OpCol<K, S>& nxt, int64_t m, int par) {
        finish(cur, m, par);
        if (m + NB < me) load(cur, m + NB);
        if (m + 1 < me) {
            dots(nxt, par ^ 1);
            __syncthreads();
        }
    };
    if (mb < me) {
#pragma unroll
        for (int b = 0; b < NB; ++b)
            if (mb + b < me) load(cb[b], mb + b);
        dots(cb[0], 0);
        __syncthreads();
        int par = 0;
        for (int64_t m = mb; m < me; m += NB) {
            step(cb[0], cb[1], m, par);
            par ^= 1;
            if constexpr (NB == 2) {
                if (m + 1 < me) {
                    step(cb[1], cb[0], m + 1, par);
                    par ^= 1;
                }
            } else {
                if (m + 1 < me) {
                    step(cb[1], cb[2 % NB], m + 1, par);
                    par ^= 1;
                }
                if (m + 2 < me) {
                    step(cb[2 % NB], cb[0], m + 2, par);
                    par ^= 1;
                }
            }
        }
    }
    // this workgroup's partial A d
    double* dst = a.part + (int64_t)blockIdx.x * kMaxRhs * ld;
#pragma unroll
    for (int s = 0; s < S; ++s) {
        if (!OP_OK(s)) continue;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            dst[(int64_t)k * ld + OP_J(s)] = acc[k][s].x;
            if (OP_J(s) + 1 < n32) dst[(int64_t)k * ld + OP_J(s) + 1] = acc[k][s].y;
        }
    }
#undef OP_J
#undef OP_OK
    // <d_k, p_k>: this workgroup's sums over its markers in order (every
    // thread holds them), then the last workgroup adds them in block order
    const RedOut& ro = a.ro;
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) red_put(ro, (int64_t)blockIdx.x * K + k, dpacc[k]);
    }
    if (wave == 0) ticket_sum_blocks<K>(ro);
}

std::string op_kernel_name(int K, const OpPlan& pl) {
    if (pl.T > 0) return team_kernel_name(K, pl);
    char b[96];
    std::snprintf(b, sizeof b, "atax_kernel<%d, %d>", K, pl.S);
    return b;
}

// hipFuncSetAttribute(MaxDynamicSharedMemorySize, bytes) for `kern` on the
// current device, once per (kernel, device): bit d of `done` is device d.  A
// failure is returned (and not left behind as the thread's last error, which
// the next launch's hipGetLastError would report as its own).
hipError_t lds_allow(const void* kern, std::atomic<unsigned long long>& done, int bytes) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const unsigned long long bit = dev >= 0 && dev < 64 ? 1ull << dev : 0ull;
    if (bit && (done.load(std::memory_order_acquire) & bit)) return hipSuccess;
    e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return e;
    }
    done.fetch_or(bit, std::memory_order_acq_rel);
    return hipSuccess;
}

template <int K, int S>
static hipError_t launch_op(const Shard& s, const OpPlan& pl, const OpArgs& a, hipStream_t st, const Timing& tm,
                            const int* gate) {
    const size_t lds = ((size_t)K * (s.N + 1 + (s.N & 1)) + 2 + 2 * kOpWaves * K) * sizeof(double);
    static std::atomic<unsigned long long> allowed{0};  // more than 64 KiB of dynamic LDS must be allowed explicitly
    if (const hipError_t e = lds_allow(reinterpret_cast<const void*>(&atax_kernel<K, S>), allowed, 160 * 1024))
        return e;
    hipExtLaunchKernelGGL((atax_kernel<K, S>), dim3(pl.grid), dim3(kOpThreads), lds, st, tm.start, tm.stop, 0, s.X,
                          s.ld, s.N, s.M, s.mave, s.msig, a, gate);
    return hipSuccess;
}

template <int K>
static hipError_t launch_op_s(int S, const Shard& s, const OpPlan& pl, const OpArgs& a, hipStream_t st,
                              const Timing& tm, const int* gate) {
    switch (S) {
        case 1: return launch_op<K, 1>(s, pl, a, st, tm, gate);
        case 2: return launch_op<K, 2>(s, pl, a, st, tm, gate);
        case 3: return launch_op<K, 3>(s, pl, a, st, tm, gate);
        case 4: return launch_op<K, 4>(s, pl, a, st, tm, gate);
        case 5: return launch_op<K, 5>(s, pl, a, st, tm, gate);
        case 6: return launch_op<K, 6>(s, pl, a, st, tm, gate);
        case 7: return launch_op<K, 7>(s, pl, a, st, tm, gate);
        case 8: return launch_op<K, 8>(s, pl, a, st, tm, gate);
        case 9: return launch_op<K, 9>(s, pl, a, st, tm, gate);
        case 10: return launch_op<K, 10>(s, pl, a, st, tm, gate);
        default: return hipErrorInvalidValue;
    }
}

hipError_t atax(const Shard& s, const OpPlan& pl, int K, const OpArgs& a, hipStream_t st, const Timing& tm,
                const int* gate) {
    if (pl.T > 0) return atax_team(s, pl, K, a, st, tm, gate);
    if (K < 1 || K > kOpMaxK || !whole_column_ok(s.N) ||
        pl.S != (int)std::max<int64_t>(1, (s.N + kOpRows - 1) / kOpRows))
        return hipErrorInvalidValue;
    if (s.M <= 0) return hipSuccess;
    hipError_t e = hipErrorInvalidValue;
    switch (K) {
        case 1: e = launch_op_s<1>(pl.S, s, pl, a, st, tm, gate); break;
        case 2: e = launch_op_s<2>(pl.S, s, pl, a, st, tm, gate); break;
        default: break;
    }
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

// The per-slot A d partials summed over the slots: a workgroup takes 128
// samples of one system (two per lane, 16-byte loads); wave w sums the slots
// [w*ns/4, (w+1)*ns/4) in order with up to 32 loads in flight, wave 0 adds
// the four wave sums in order.  cg_update's one-rank form (cg_update_kernel,
// c.adpart) sums in exactly this order, so the two paths agree bit for bit.
// (Every load of a round is issued before the first add: the adds stay in
// slot order, so the round size changes the latency, not the bits.)
// W: the largest round (32: 128 VGPRs of loads in flight; 8 for the few slots
// of the large-N plans, so that cg_update's workgroups are not held to one per
// CU by a round they never run)
template <int W = 32>
__device__ __forceinline__ v2d slot_sum(const double* src, int64_t ss, int t0, int t1) {
    v2d acc = {0.0, 0.0};
    int t = t0;
    for (; W >= 32 && t + 32 <= t1; t += 32) {  // (C2, team of 2: 128 slots, 32 per wave, one round trip)
        v2d x[32];
#pragma unroll
        for (int u = 0; u < 32; ++u) x[u] = *reinterpret_cast<const v2d*>(src + (t + u) * ss);
#pragma unroll
        for (int u = 0; u < 32; ++u) acc += x[u];
    }
    for (; W >= 16 && t + 16 <= t1; t += 16) {
        v2d x[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) x[u] = *reinterpret_cast<const v2d*>(src + (t + u) * ss);
#pragma unroll
        for (int u = 0; u < 16; ++u) acc += x[u];
    }
    for (; t + 8 <= t1; t += 8) {
        v2d x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = *reinterpret_cast<const v2d*>(src + (t + u) * ss);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += x[u];
    }
    for (; t < t1; ++t) acc += *reinterpret_cast<const v2d*>(src + t * ss);
    return acc;
}

__global__ __launch_bounds__(256) void op_reduce_kernel(int64_t N, int64_t ld, int nslots,
                                                        const double* __restrict__ part, Ptrs out, double div,
                                                        const int* __restrict__ gate) {
    if (gate && !*gate) return;
    __shared__ v2d wsum[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t tpk = (N + 127) / 128;
    const int k = (int)(blockIdx.x / tpk);
    const int64_t i = (blockIdx.x - k * tpk) * 128 + 2 * lane;  // < ld (a multiple of 16)
    const bool ok = i < N;
    wsum[w][lane] = ok ? slot_sum(part + (int64_t)k * ld + i, (int64_t)kMaxRhs * ld, w * nslots / 4,
                                  (w + 1) * nslots / 4)
                       : v2d{0.0, 0.0};
    __syncthreads();
    if (w != 0 || !ok) return;
    v2d r = ((wsum[0][lane] + wsum[1][lane]) + wsum[2][lane]) + wsum[3][lane];
    if (div > 0) r /= div;
    out.p[k][i] = r.x;
    if (i + 1 < N) out.p[k][i + 1] = r.y;
}

hipError_t op_reduce(const OpPlan& pl, int K, int64_t N, int64_t ld, const double* part, Ptrs out, double div,
                     hipStream_t st, const int* gate, int k0) {
    const int64_t n = (int64_t)K * N;
    if (n <= 0) return hipSuccess;
    if (k0 < 0 || k0 + K > kMaxRhs) return hipErrorInvalidValue;
    hipLaunchKernelGGL(op_reduce_kernel, dim3((unsigned)(K * cdiv(N, 128))), dim3(256), 0, st, N, ld, (int)pl.nslots,
                       part + (int64_t)k0 * ld, out, div, gate);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// marker statistics (src/data.cpp:233-283): one wave per marker, two passes
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void stats_kernel(const double* __restrict__ X, int64_t ld, int64_t N, int64_t M,
                                                       double nonas, double alpha_scale, double* __restrict__ mave,
                                                       double* __restrict__ msig) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t m = (int64_t)blockIdx.x * 4 + wave;
    if (m >= M) return;
    const double* col = X + m * ld;
    double s = 0.0;
    for (int64_t j = 2 * lane; j < N; j += 128) {
        const v2d x = ld2(col + j);
        s += x.x;
        if (j + 1 < N) s += x.y;
    }
    s = wave_sum(s);
    const double mean = s / nonas;
    double q = 0.0;
    for (int64_t j = 2 * lane; j < N; j += 128) {
        const v2d x = ld2(col + j);
        const double a = x.x - mean;
        q += a * a;
        if (j + 1 < N) {
            const double b = x.y - mean;
            q += b * b;
        }
    }
    q = wave_sum(q);
    if (lane == 0) {
        mave[m] = mean;
        double sg;
        if (q != 0.0) {
            if (alpha_scale == 1.0)
                sg = 1.0 / sqrt(q / (nonas - 1.0));
            else
                sg = 1.0 / pow(sqrt(q / (nonas - 1.0)), alpha_scale);
        } else {
            sg = 1.0;
        }
        msig[m] = sg;
    }
}

hipError_t marker_stats(const double* X, int64_t ld, int64_t N, int64_t M, double nonas, double alpha_scale,
                        double* mave, double* msig, hipStream_t st) {
    if (M <= 0) return hipSuccess;
    hipLaunchKernelGGL(stats_kernel, dim3((unsigned)cdiv(M, 4)), dim3(kBlock), 0, st, X, ld, N, M, nonas, alpha_scale,
                       mave, msig);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// synthetic data
// ---------------------------------------------------------------------------
__global__ void gen_kernel(uint64_t seed, int kind, int64_t N, int64_t ld, int64_t S, int64_t M, double* X) {
    const int64_t total = M * ld;
    for (int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x; e < total; e += (int64_t)gridDim.x * kBlock) {
        const int64_t i = e / ld, j = e - i * ld;
        double v = 0.0;
        if (j < N) v = kind == 1 ? meth_dyadic(seed, S + i, j) : gauss_dyadic(seed, S + i, j);
        X[e] = v;
    }
}

hipError_t gen_markers(uint64_t seed, int kind, int64_t N, int64_t ld, int64_t S, int64_t M, double* X,
                       hipStream_t st) {
    int64_t blocks = cdiv(M * ld, kBlock);
    if (blocks > 65536) blocks = 65536;
    if (blocks < 1) return hipSuccess;
    hipLaunchKernelGGL(gen_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, st, seed, kind, N, ld, S, M, X);
    return hipGetLastError();
}

__global__ __launch_bounds__(kBlock) void gen_beta_kernel(uint64_t seed, double lam, int64_t S, int64_t M,
                                                          double* beta, RedOut ro) {
    __shared__ double lds[4];
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    double c = 0.0;
    if (i < M) {
        const uint64_t h = splitmix64(splitmix64(seed ^ 0x63617573ULL) + (uint64_t)(S + i));
        const double uni = (double)(h >> 11) * (1.0 / 9007199254740992.0);
        const bool causal = uni < lam;
        beta[i] = causal ? gauss_dyadic(seed ^ 0x62657461ULL, S + i, 0) : 0.0;
        c = causal ? 1.0 : 0.0;
    }
    c = block_sum(c, lds);
    if (threadIdx.x == 0) red_put(ro, blockIdx.x, c);
    red_finish(ro, 1, lds);
}

hipError_t gen_beta(uint64_t seed, double lam, int64_t S, int64_t M, double* beta, const RedOut& ro, hipStream_t st) {
    const int nblk = (int)std::max<int64_t>(1, cdiv(M, kBlock));
    hipLaunchKernelGGL(gen_beta_kernel, dim3(nblk), dim3(kBlock), 0, st, seed, lam, S, M, beta, ro);
    return hipGetLastError();
}

__global__ void scale_kernel(int64_t n, double* v, double a) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) v[i] *= a;
}

hipError_t scale_vec(int64_t n, double* v, double a, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(scale_kernel, dim3((unsigned)cdiv(n, kBlock)), dim3(kBlock), 0, st, n, v, a);
    return hipGetLastError();
}

__global__ void noise_kernel(uint64_t seed, int64_t N, double sd, double* y) {
    const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j < N) y[j] = y[j] + sd * gauss_dyadic(seed ^ 0x6E6F697365ULL, -1, j);
}

hipError_t add_noise(uint64_t seed, int64_t N, double sd, double* y, hipStream_t st) {
    hipLaunchKernelGGL(noise_kernel, dim3((unsigned)cdiv(N, kBlock)), dim3(kBlock), 0, st, seed, N, sd, y);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// reductions (inner_prod / l2_norm2, src/utilities.cpp:138-162)
// ---------------------------------------------------------------------------
int red_blocks(int64_t n) {
    int64_t b = cdiv(n, 512);  // >= 2 elements per thread; enough blocks to fill 256 CUs at M ~ 1e5
    if (b < 1) b = 1;
    if (b > kRedBlocks) b = kRedBlocks;
    return (int)b;
}

// src/vamp.cpp:341-346, 498 (G1Chain): the host's expressions
__device__ __forceinline__ void gam1_chain(double a2, double gam2, double rho, double gam1_prev, double* out) {
    const double alpha2 = gam2 * a2;    // :498
    const double eta2 = gam2 / alpha2;  // :341
    const double d = eta2 - gam2;
    double g = d < 1e-11 ? 1e-11 : d;  // std::max(d, 1e-11)
    g = 1e11 < g ? 1e11 : g;           // std::min(., 1e11)
    out[0] = rho * g + (1 - rho) * gam1_prev;  // :346
    out[1] = eta2;
    out[2] = alpha2;
}

// every term loads both operands unconditionally (a SUM term's b is its a,
// set on the host) so a thread's loads for all terms are in flight together;
// the op is a per-launch uniform selected per element.  UPD: some term is a
// PUPD / SQPUPD (its c and beta are loaded); a launch without one does not
// keep those pointers (up to 12 terms without scalar-register spills)
// one reduction's blocks [bid of nblk]: the per-block partials of its NT terms
template <int NT, bool UPD>
__device__ __forceinline__ void dots_part(const DotArgs& a, int64_t n, const RedOut& ro, int bid, int nblk) {
    double bt[NT];
#pragma unroll
    for (int q = 0; q < NT; ++q) bt[q] = UPD && (a.t[q].op == PUPD || a.t[q].op == SQPUPD) ? *a.t[q].beta : 0.0;
    double acc[NT];
#pragma unroll
    for (int q = 0; q < NT; ++q) acc[q] = 0.0;
    for (int64_t e = (int64_t)bid * kBlock + threadIdx.x; e < n; e += (int64_t)nblk * kBlock) {
        double va[NT], vb[NT];
#pragma unroll
        for (int q = 0; q < NT; ++q) {
            va[q] = a.t[q].a[e];
            vb[q] = UPD && (a.t[q].op == PUPD || a.t[q].op == SQPUPD) ? a.t[q].c[e] + bt[q] * a.t[q].b[e]
                                                                     : a.t[q].b[e];
        }
#pragma unroll
        for (int q = 0; q < NT; ++q) {
            const double d = va[q] - vb[q];
            const int op = a.t[q].op;
            const double v = (op == DOT || op == PUPD) ? va[q] * vb[q]
                             : op == SQPUPD            ? vb[q] * vb[q]
                             : op == DIFF2             ? d * d
                                                       : va[q];
            acc[q] += v;
        }
    }
    block_put_sums<NT>(acc, NT, ro, (int64_t)bid * NT);
}

// the launch's hooks on its final sums (thread 0 of the last block)
__device__ __forceinline__ void dots_post(const DotArgs& a, const double* fin) {
    if (a.g1.out) gam1_chain(fin[a.g1.term], a.g1.gam2, a.g1.rho, a.g1.gam1_prev, a.g1.out);
    for (int j = 0; j < a.copy.n && j < 2; ++j) a.copy.dst[j][0] = fin[a.copy.term[j]];
}

template <int NT, bool UPD>
__global__ __launch_bounds__(kBlock) void dots_kernel(DotArgs a, int64_t n, RedOut ro) {
    if (ro.gate && !*ro.gate) return;
    __shared__ double lds[4];
    dots_part<NT, UPD>(a, n, ro, (int)blockIdx.x, (int)gridDim.x);
    __shared__ double fin[NT];
    const bool post = a.g1.out || a.copy.n;
    if (red_finish(ro, NT, lds, post ? fin : nullptr) && post && threadIdx.x == 0) dots_post(a, fin);
}

// Two reductions in one launch (dots2): blocks [0, ba) are reduction A's
// (red_blocks(na) of them), the rest B's; each part's partials, final sums and
// hooks are those of its own dots launch, bit for bit.  One ticket counts every
// block; the last one finishes A, then B (B's RedOut carries the flag).
template <int NA, int NB>
__global__ __launch_bounds__(kBlock) void dots2_kernel(DotArgs a, int64_t na, RedOut roa, int ba, DotArgs b,
                                                       int64_t nb, RedOut rob) {
    if ((int)blockIdx.x < ba)
        dots_part<NA, false>(a, na, roa, (int)blockIdx.x, ba);
    else
        dots_part<NB, false>(b, nb, rob, (int)blockIdx.x - ba, (int)gridDim.x - ba);
    if (!red_ticket(roa, (int)gridDim.x)) return;
    __shared__ double fa[NA], fb[NB];
    red_final(roa, NA, ba, fa, false);
    red_final(rob, NB, (int)gridDim.x - ba, fb, true);
    if (threadIdx.x == 0) {
        dots_post(a, fa);
        dots_post(b, fb);
    }
}

hipError_t dots2(const DotArgs& a, int64_t na, const RedOut& roa, const DotArgs& b, int64_t nb, const RedOut& rob,
                 hipStream_t st) {
    const int ba = red_blocks(na), bb = red_blocks(nb);
    if (roa.flag || roa.gate || rob.gate || rob.ticket != roa.ticket) return hipErrorInvalidValue;
    for (const DotArgs* x : {&a, &b})
        for (int q = 0; q < x->nt; ++q)
            if (x->t[q].op == PUPD || x->t[q].op == SQPUPD) return hipErrorInvalidValue;
    const dim3 g(ba + bb), blk(kBlock);
    if (a.nt == 10 && b.nt == 11)
        hipLaunchKernelGGL((dots2_kernel<10, 11>), g, blk, 0, st, a, na, roa, ba, b, nb, rob);
    else
        return hipErrorInvalidValue;  // (the one pairing in use: vamp.cpp's iteration tail)
    return hipGetLastError();
}

template <bool UPD>
static hipError_t dots_launch(const DotArgs& a, int64_t n, const RedOut& ro, hipStream_t st) {
    const dim3 g(red_blocks(n)), b(kBlock);
    switch (a.nt) {
        case 1: hipLaunchKernelGGL((dots_kernel<1, UPD>), g, b, 0, st, a, n, ro); break;
        case 2: hipLaunchKernelGGL((dots_kernel<2, UPD>), g, b, 0, st, a, n, ro); break;
        case 3: hipLaunchKernelGGL((dots_kernel<3, UPD>), g, b, 0, st, a, n, ro); break;
        case 4: hipLaunchKernelGGL((dots_kernel<4, UPD>), g, b, 0, st, a, n, ro); break;
        case 5: hipLaunchKernelGGL((dots_kernel<5, UPD>), g, b, 0, st, a, n, ro); break;
        case 6: hipLaunchKernelGGL((dots_kernel<6, UPD>), g, b, 0, st, a, n, ro); break;
        case 7: hipLaunchKernelGGL((dots_kernel<7, UPD>), g, b, 0, st, a, n, ro); break;
        case 8: hipLaunchKernelGGL((dots_kernel<8, UPD>), g, b, 0, st, a, n, ro); break;
        case 9: if (!UPD) { hipLaunchKernelGGL((dots_kernel<9, false>), g, b, 0, st, a, n, ro); break; } return hipErrorInvalidValue;
        case 10: if (!UPD) { hipLaunchKernelGGL((dots_kernel<10, false>), g, b, 0, st, a, n, ro); break; } return hipErrorInvalidValue;
        case 11: if (!UPD) { hipLaunchKernelGGL((dots_kernel<11, false>), g, b, 0, st, a, n, ro); break; } return hipErrorInvalidValue;
        case 12: if (!UPD) { hipLaunchKernelGGL((dots_kernel<12, false>), g, b, 0, st, a, n, ro); break; } return hipErrorInvalidValue;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// (at most 8 terms when one of them is a PUPD / SQPUPD)
hipError_t dots(const DotArgs& a, int64_t n, const RedOut& ro, hipStream_t st) {
    bool upd = false;
    for (int q = 0; q < a.nt && q < kMaxTerms; ++q) upd = upd || a.t[q].op == PUPD || a.t[q].op == SQPUPD;
    return upd ? dots_launch<true>(a, n, ro, st) : dots_launch<false>(a, n, ro, st);
}

constexpr int Q_MAX_EM = 1 + 2 * (kMaxL - 1);  // an EM round's sums

// ---------------------------------------------------------------------------
// denoiser: vamp::g1 / vamp::g1d (src/vamp.cpp:440-492)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void g1_g1d(double y, double gam1, const double* probs, const double* vars, int L,
                                       double eta_max, double* g, double* gd) {
    const double sigma = 1 / gam1;
    if (sigma < 1e-10 && sigma > -1e-10) {
        *g = y;
        *gd = 1;
        return;
    }
    double pk = 0, pkd = 0, pkdd = 0;
    for (int i = 0; i < L; ++i) {
        const double vs = vars[i] + sigma;
        const double expe_sum = -0.5 * (y * y) * (eta_max - vars[i]) / vs / (eta_max + sigma);
        const double ex = exp(expe_sum);
        double z = probs[i] / sqrt(vs) * ex;
        pk = pk + z;
        z = z / vs * y;
        pkd = pkd - z;
        const double z2 = z / vs * y;
        pkdd = pkdd - probs[i] / pow_1p5(vs) * ex + z2;
    }
    *g = y + sigma * pkd / pk;
    const double q = pkd / pk;
    *gd = 1 + sigma * (pkdd / pk - q * q);
}

// One EM round's update of the mixture (L components, variances vars) from
// the round's sums q (1 + 2(L-1)) and the merging of close variances
// (vamp.cpp em_finish with one round, the host's expressions in the host's
// order: src/vamp.cpp:598-642; every prob is rewritten), by ONE thread, into
// the mixture words w (kMixWords, LDS: [0] L, probs, vars, eta_max)
__device__ void em_update_mix(const double* q, int L, const double* vars, const EmUpd& u, double* w) {
    double* pr = w + 1;
    double* va = w + 1 + kMaxL;
    for (int j = 0; j < L; ++j) va[j] = vars[j];
    const double lambda_total = q[0];
    const double lambda = lambda_total / (double)u.Mt;
    const double sum_of_pin = lambda_total;
    for (int j = 0; j < L - 1; ++j) {
        const double res_total = q[1 + j];
        const double res_gammas_total = q[L + j];
        if (u.learn_vars == 1) va[j + 1] = res_gammas_total / res_total;
        const double omega = res_total / sum_of_pin;
        pr[j + 1] = lambda * omega;
    }
    pr[0] = 1 - lambda;
    for (int j = 0; j < L; ++j) {  // merging close variances (src/vamp.cpp:626-642)
        for (int k = j + 1; k < L; ++k) {
            const double denom = va[j] != 0 ? (va[k] < va[j] ? va[k] : va[j]) : 1e-7;  // std::min
            if (fabs(va[j] - va[k]) / denom < u.merge_vars_thr) {
                const double sum2probs = pr[j] + pr[k];
                for (int r = k; r + 1 < L; ++r) {
                    va[r] = va[r + 1];
                    pr[r] = pr[r + 1];
                }
                L--;
                pr[j] = sum2probs;
                k--;
            }
        }
    }
    double eta_max = va[0];  // (denoise: the host's loop)
    for (int i = 1; i < L; ++i)
        if (va[i] > eta_max) eta_max = va[i];
    w[0] = (double)L;
    w[1 + 2 * kMaxL] = eta_max;
}

// the next prelude's scalars (kernels.h PreOut) from the sum of x1d, gam1 and
// the two updateNoisePrec sums: the host's expressions
__device__ void pre_scalars(double sum_d, double gam1, double tn, double tc, const PreOut& po) {
    const double alpha1 = sum_d / po.Mt;  // :223
    const double eta1 = gam1 / alpha1;    // :230
    const double dg = eta1 - gam1;
    double gam2 = dg < 1e-11 ? 1e-11 : dg;  // std::max(., 1e-11) (:255-256)
    gam2 = 1e11 < gam2 ? 1e11 : gam2;       // std::min(., 1e11)
    const double trace_corr = tc * po.Mt;    // :521
    const double gamw = po.N / (tn + trace_corr);  // :528
    const double diag = gamw * (po.N - 1) / po.N + gam2;  // :676-677 (pcg_run)
    const double v[5] = {eta1, gam2, gamw, diag, gam1};
    for (int q = 0; q < 5; ++q) po.out[q] = v[q];
    for (int q = 0; q < 4; ++q) po.mirror[q] = v[q];
}

// the mixture words w (em_update_mix) into upd.out and upd.mirror
__device__ void em_write(const double* w, const EmUpd& u) {
    const int Ln = (int)w[0];
    for (double* o : {u.out, u.mirror}) {
        o[0] = w[0];
        for (int j = 0; j < Ln; ++j) {
            o[1 + j] = w[1 + j];
            o[1 + kMaxL + j] = w[1 + kMaxL + j];
        }
        o[1 + 2 * kMaxL] = w[1 + 2 * kMaxL];
    }
}

// Dev: the mixture's words (an EM round's update, em_kernel) and gam1
// (G1Chain) from the device, the words staged in LDS; else mix and gam1
template <bool Dev>
__global__ __launch_bounds__(kBlock) void denoise_kernel(int64_t M, const double* __restrict__ r1, double gam1,
                                                         Mix mix, double eta_max, double* __restrict__ x1,
                                                         const double* __restrict__ x1_prev, int damp, double rho,
                                                         double* __restrict__ x1d, RedOut ro,
                                                         const double* __restrict__ mixw,
                                                         const double* __restrict__ gam1dev, PreOut po) {
    __shared__ double lds[4];
    __shared__ double sm[Dev ? kMixWords : 1];
    // po: tn and tc (device copies) are loaded at the start, their latency
    // behind the launch's work; the last block uses them
    double tn = 0.0, tc = 0.0;
    if (Dev && po.out && threadIdx.x == 0) {
        tn = po.tn[0];
        tc = po.tc[0];
    }
    const double* probs = mix.probs;
    const double* vars = mix.vars;
    int L = mix.L;
    if (Dev) {
        for (int q = threadIdx.x; q < kMixWords; q += kBlock) sm[q] = mixw[q];
        gam1 = gam1dev[0];
        __syncthreads();
        L = (int)sm[0];
        probs = sm + 1;
        vars = sm + 1 + kMaxL;
        eta_max = sm[1 + 2 * kMaxL];
    }
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < M; i += (int64_t)gridDim.x * kBlock) {
        double g, gd;
        g1_g1d(r1[i], gam1, probs, vars, L, eta_max, &g, &gd);
        if (damp) g = rho * g + (1 - rho) * x1_prev[i];  // src/vamp.cpp:208-211
        x1[i] = g;
        x1d[i] = gd;
        acc += gd;
    }
    acc = block_sum(acc, lds);
    if (threadIdx.x == 0) red_put(ro, blockIdx.x, acc);
    __shared__ double fin[1];
    const bool last = red_finish(ro, 1, lds, Dev && po.out ? fin : nullptr);
    if (Dev && po.out && last && threadIdx.x == 0) pre_scalars(fin[0], gam1, tn, tc, po);
}

hipError_t denoise(int64_t M, const double* r1, double gam1, const Mix& mix, double* x1, const double* x1_prev,
                   int damp, double rho, double* x1d, const RedOut& ro, hipStream_t st, const double* mixw,
                   const double* gam1dev, const PreOut* po) {
    double eta_max = mix.vars[0];
    for (int i = 1; i < mix.L; ++i)
        if (mix.vars[i] > eta_max) eta_max = mix.vars[i];
    if (mixw) {
        if (!gam1dev || (po && (!po->out || !po->mirror || !po->tn || !po->tc))) return hipErrorInvalidValue;
        hipLaunchKernelGGL(denoise_kernel<true>, dim3(red_blocks(M)), dim3(kBlock), 0, st, M, r1, gam1, mix, eta_max,
                           x1, x1_prev, damp, rho, x1d, ro, mixw, gam1dev, po ? *po : PreOut{});
    } else {
        if (po) return hipErrorInvalidValue;
        hipLaunchKernelGGL(denoise_kernel<false>, dim3(red_blocks(M)), dim3(kBlock), 0, st, M, r1, gam1, mix,
                           eta_max, x1, x1_prev, damp, rho, x1d, ro, nullptr, nullptr, PreOut{});
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// EM prior update sums (src/vamp.cpp:554-597), one marker per thread
// ---------------------------------------------------------------------------
__device__ __forceinline__ double em_num(const EmArgs& a, double noise_var, double r, int j) {
    return a.lambda * a.omegas[j] *
           exp(-(r * r) / 2 * (a.max_sigma - a.vars[j]) / (a.vars[j] + noise_var) / (a.max_sigma + noise_var)) /
           sqrt(a.vars[j] + noise_var) / sqrt(2 * M_PI);
}

// The Q = 1 + 2(L-1) block sums: each wave reduces every value in registers
// and leaves it in LDS, ONE barrier, then thread q adds the four wave sums in
// wave order: per value the arithmetic of block_sum (bitwise), with one
// barrier instead of 2Q.  a.r1out: r1 is formed here (lincomb_div's
// expression) and stored, not read.
__global__ __launch_bounds__(kBlock) void em_kernel(int64_t M, const double* __restrict__ r1, EmArgs a, RedOut ro) {
    __shared__ double lds[4];
    __shared__ double wl[4][1 + 2 * (kMaxL - 1)];
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const bool valid = i < M;
    // gam1 and eta2 from the device (a.dsc) or the host; the derived scalars
    // with the host's expressions (vamp.cpp em_queue)
    const double gam1 = a.dsc ? a.dsc[0] : a.gam1;
    const double noise_var = a.dsc ? 1 / gam1 : a.noise_var;
    double r = 0.0;
    if (valid) {
        if (a.r1out) {
            const double la = a.dsc ? a.dsc[1] : a.la, lc = a.dsc ? gam1 : a.lc;
            r = (la * a.lx[i] - a.lb * a.ly[i]) / lc;  // lincomb_div_kernel's expression
            a.r1out[i] = r;
        } else {
            r = r1[i];
        }
    }
    const int L = a.L, Q = 1 + 2 * (L - 1);
    // em_num of the first kEmC - 1 slabs is formed once and kept in registers
    // (fixed-bound unrolled loops: no run-time register indexing); the same
    // values, summed in the same order, as forming it twice
    constexpr int kEmC = 12;
    double en[kEmC];
    double sum_of_elems = 0.0;
#pragma unroll
    for (int j = 1; j < kEmC; ++j)
        if (j < L) {
            en[j] = em_num(a, noise_var, r, j);
            sum_of_elems += en[j];
        }
    for (int j = kEmC; j < L; ++j) sum_of_elems += em_num(a, noise_var, r, j);
    const double pin = 1 / (1 + (1 - a.lambda) / sqrt(2 * M_PI * noise_var) *
                                    exp(-(r * r) / 2 * a.max_sigma / noise_var / (noise_var + a.max_sigma)) /
                                    sum_of_elems);
    double s = wave_sum(valid ? pin : 0.0);
    if (lane == 0) wl[w][0] = s;
    auto slab = [&](int j, double num) {
        const double beta = num / sum_of_elems;
        const double g = gam1 * r / (1 / a.vars[j] + gam1);
        const double vj = a.dsc ? 1.0 / (1.0 / a.vars[j] + gam1) : a.v[j - 1];
        const double gam = beta * (g * g + vj);
        const double sb = wave_sum(valid ? beta * pin : 0.0);
        const double sg = wave_sum(valid ? gam * pin : 0.0);
        if (lane == 0) {
            wl[w][j] = sb;
            wl[w][(L - 1) + j] = sg;
        }
    };
#pragma unroll
    for (int j = 1; j < kEmC; ++j)
        if (j < L) slab(j, en[j]);
    for (int j = kEmC; j < L; ++j) slab(j, em_num(a, noise_var, r, j));
    __syncthreads();
    for (int q = threadIdx.x; q < Q; q += kBlock)
        red_put(ro, (int64_t)blockIdx.x * Q + q, ((wl[0][q] + wl[1][q]) + wl[2][q]) + wl[3][q]);
    __shared__ double fin[Q_MAX_EM];
    const bool last = red_finish(ro, Q, lds, a.upd.out ? fin : nullptr);
    if (last && a.upd.out && threadIdx.x == 0) {  // the round's update of the mixture (EmArgs.upd)
        __shared__ double w[kMixWords];
        em_update_mix(fin, L, a.vars, a.upd, w);
        em_write(w, a.upd);
    }
}

// kernels.h TailPost: the one-rank last blocks' work, after the all-reduce
__global__ void tail_post_kernel(TailPost t) {
    if (threadIdx.x != 0) return;
    if (t.mode == 0) {
        gam1_chain(t.src[0], t.g1.gam2, t.g1.rho, t.g1.gam1_prev, t.g1.out);
        for (int i = 0; i < 2; ++i)
            if (t.cp_dst[i]) *t.cp_dst[i] = *t.cp_src[i];
    } else if (t.mode == 1) {
        __shared__ double w[kMixWords];
        em_update_mix(t.src, t.L, t.vars, t.upd, w);
        em_write(w, t.upd);
    } else {
        pre_scalars(t.src[0], t.gam1dev[0], t.po.tn[0], t.po.tc[0], t.po);
    }
}

hipError_t tail_post(const TailPost& t, hipStream_t st) {
    if (!t.src || t.mode < 0 || t.mode > 2 || (t.mode == 0 && !t.g1.out) || (t.mode == 1 && (!t.upd.out || !t.upd.mirror)) ||
        (t.mode == 2 && (!t.gam1dev || !t.po.out || !t.po.mirror || !t.po.tn || !t.po.tc)))
        return hipErrorInvalidValue;
    for (int i = 0; i < 2; ++i)
        if (t.cp_dst[i] && !t.cp_src[i]) return hipErrorInvalidValue;
    hipLaunchKernelGGL(tail_post_kernel, dim3(1), dim3(64), 0, st, t);
    return hipGetLastError();
}

hipError_t em_sums(int64_t M, const double* r1, const EmArgs& a, const RedOut& ro, hipStream_t st) {
    const int nblk = (int)std::max<int64_t>(1, cdiv(M, kBlock));
    hipLaunchKernelGGL(em_kernel, dim3(nblk), dim3(kBlock), 0, st, M, r1, a, ro);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// elementwise
// ---------------------------------------------------------------------------
__global__ void lincomb_div_kernel(int64_t n, double a, const double* __restrict__ x, double b,
                                   const double* __restrict__ y, double c, double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) out[i] = (a * x[i] - b * y[i]) / c;
}

hipError_t lincomb_div(int64_t n, double a, const double* x, double b, const double* y, double c, double* out,
                       hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(lincomb_div_kernel, dim3((unsigned)cdiv(n, kBlock)), dim3(kBlock), 0, st, n, a, x, b, y, c,
                       out);
    return hipGetLastError();
}

__global__ void axpby_kernel(int64_t n, double a, const double* __restrict__ x, double b,
                             const double* __restrict__ y, double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) out[i] = a * x[i] + b * y[i];
}

hipError_t axpby(int64_t n, double a, const double* x, double b, const double* y, double* out, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(axpby_kernel, dim3((unsigned)cdiv(n, kBlock)), dim3(kBlock), 0, st, n, a, x, b, y, out);
    return hipGetLastError();
}

__global__ void bern_kernel(uint64_t seed, int it, int64_t S, int64_t M, double sqrtMt, double* out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < M) out[i] = (double)(2 * bern_bit(seed, it, S + i) - 1) / sqrtMt;
}

hipError_t bernoulli(uint64_t seed, int it, int64_t S, int64_t M, double sqrtMt, double* out, hipStream_t st) {
    if (M <= 0) return hipSuccess;
    hipLaunchKernelGGL(bern_kernel, dim3((unsigned)cdiv(M, kBlock)), dim3(kBlock), 0, st, seed, it, S, M, sqrtMt,
                       out);
    return hipGetLastError();
}

__global__ void prelude_kernel(int64_t M, Prelude p) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= M) return;
    const double r2 = (p.eta1 * p.x1[i] - p.gam1 * p.r1[i]) / p.gam2;  // lincomb_div's expression
    p.r2[i] = r2;
    p.v[i] = p.gamw * p.atxy[i] + p.gam2 * r2;                         // axpby's
    p.bern[i] = (double)(2 * bern_bit(p.seed, p.it, p.S + i) - 1) / p.sqrtMt;
    if (p.bern_next) p.bern_next[i] = (double)(2 * bern_bit(p.seed, p.it + 1, p.S + i) - 1) / p.sqrtMt;
    if (p.zero[0]) p.zero[0][i] = 0.0;
    if (p.zero[1]) p.zero[1][i] = 0.0;
}

hipError_t prelude(int64_t M, const Prelude& p, hipStream_t st) {
    if (M <= 0) return hipSuccess;
    hipLaunchKernelGGL(prelude_kernel, dim3((unsigned)cdiv(M, kBlock)), dim3(kBlock), 0, st, M, p);
    return hipGetLastError();
}

__global__ void set_scalar_kernel(double* p, double v) {
    if (threadIdx.x == 0) *p = v;
}

hipError_t set_scalar(double* p, double v, hipStream_t st) {
    hipLaunchKernelGGL(set_scalar_kernel, dim3(1), dim3(64), 0, st, p, v);
    return hipGetLastError();
}

__global__ void div_scalar_kernel(int64_t n, const double* __restrict__ x, double d, double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) out[i] = x[i] / d;
}

hipError_t div_scalar(int64_t n, const double* x, double d, double* out, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(div_scalar_kernel, dim3((unsigned)cdiv(n, kBlock)), dim3(kBlock), 0, st, n, x, d, out);
    return hipGetLastError();
}

// out[0, n) = x / d, out[n, 2n) = r / d (IEEE division, as the host's x / sqrt(N))
__global__ void div2_scalar_kernel(int64_t n, const double* __restrict__ x, const double* __restrict__ r, double d,
                                   double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) {
        out[i] = x[i] / d;
        out[n + i] = r[i] / d;
    }
}

hipError_t div2_scalar(int64_t n, const double* x, const double* r, double d, double* out, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(div2_scalar_kernel, dim3((unsigned)cdiv(n, kBlock)), dim3(kBlock), 0, st, n, x, r, d, out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// PCG vector steps (src/vamp.cpp:671-757), K right-hand sides per launch
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void cg_init_kernel(int K, int64_t M, CgVecs c, double diag, RedOut ro) {
    __shared__ double lds[4];
    double acc[2 * kMaxRhs];
#pragma unroll
    for (int q = 0; q < 2 * kMaxRhs; ++q) acc[q] = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < M; i += (int64_t)gridDim.x * kBlock) {
#pragma unroll
        for (int k = 0; k < kMaxRhs; ++k) {
            if (k < K) {
                const double vi = c.v[k][i];
                double r;
                if (c.atx0[k]) {  // lmmse_mult(mu0) from a precomputed A^T(A mu0): res*=tau; res+=gam2*v
                    double dv = c.atx0[k][i];
                    dv *= c.tau;
                    dv += c.gam2 * c.mu[k][i];
                    r = vi - dv;
                } else {
                    r = c.d[k] ? vi - c.d[k][i] : vi - 0.0;  // r = v - lmmse_mult(mu0)
                }
                const double z = r / diag;
                c.r[k][i] = r;
                c.z[k][i] = z;
                c.p[k][i] = z;
                acc[2 * k] += r * z;
                acc[2 * k + 1] += vi * vi;
            }
        }
    }
    block_put_sums<2 * kMaxRhs>(acc, 2 * K, ro, (int64_t)blockIdx.x * 2 * K);
    red_finish(ro, 2 * K, lds);
}

// prelude_kernel's and cg_init_kernel's work in one launch, on cg_init's grid
// (the same sums, in the same order); v_k that the prelude forms (v, bern) is
// used from registers.  Two elements per round (i, i + stride), all of both
// elements' loads issued before either is used; the sums still run over i,
// i + stride, ... in order.  start: the last block builds the CgState
// (cg_start_from)
__global__ __launch_bounds__(kBlock) void prelude_cg_init_kernel(int K, int64_t M, Prelude p, CgVecs c, double diag,
                                                                 RedOut ro, CgState start, CgState* dst) {
    __shared__ double lds[4];
    __shared__ double fin[2 * kMaxRhs];
    double eta1 = p.eta1, gam1 = p.gam1, gam2 = p.gam2, gamw = p.gamw, tau = c.tau, cgam2 = c.gam2;
    if (p.dev.scal) {  // the scalars from the device (kernels.h PreDev, formed by the denoiser's launch)
        const double* q = p.dev.scal;
        eta1 = q[0];
        gam2 = cgam2 = q[1];
        gamw = tau = q[2];
        diag = q[3];
        gam1 = q[4];
    }
    double acc[2 * kMaxRhs];
#pragma unroll
    for (int q = 0; q < 2 * kMaxRhs; ++q) acc[q] = 0.0;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i0 = (int64_t)blockIdx.x * kBlock + threadIdx.x; i0 < M; i0 += 2 * stride) {
        const bool two = i0 + stride < M;
        double x1v[2], r1v[2], ayv[2], vo[2][kMaxRhs], a0[2][kMaxRhs], muv[2][kMaxRhs], dd[2][kMaxRhs];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int64_t i = i0 + h * stride;
            if (h == 1 && !two) break;
            x1v[h] = p.x1[i];
            r1v[h] = p.r1[i];
            ayv[h] = p.atxy[i];
#pragma unroll
            for (int k = 0; k < kMaxRhs; ++k) {
                if (k >= K) continue;
                vo[h][k] = c.v[k] == p.v || c.v[k] == p.bern ? 0.0 : c.v[k][i];
                a0[h][k] = c.atx0[k] ? c.atx0[k][i] : 0.0;
                muv[h][k] = c.atx0[k] ? c.mu[k][i] : 0.0;
                dd[h][k] = !c.atx0[k] && c.d[k] ? c.d[k][i] : 0.0;
            }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int64_t i = i0 + h * stride;
            if (h == 1 && !two) break;
            // prelude_kernel's expressions
            const double r2 = (eta1 * x1v[h] - gam1 * r1v[h]) / gam2;  // lincomb_div's expression
            p.r2[i] = r2;
            const double vv = gamw * ayv[h] + gam2 * r2;                  // axpby's
            p.v[i] = vv;
            const double bn = (double)(2 * bern_bit(p.seed, p.it, p.S + i) - 1) / p.sqrtMt;
            p.bern[i] = bn;
            if (p.bern_next) p.bern_next[i] = (double)(2 * bern_bit(p.seed, p.it + 1, p.S + i) - 1) / p.sqrtMt;
            if (p.zero[0]) p.zero[0][i] = 0.0;
            if (p.zero[1]) p.zero[1][i] = 0.0;
            // cg_init_kernel's
#pragma unroll
            for (int k = 0; k < kMaxRhs; ++k) {
                if (k >= K) continue;
                const double vi = c.v[k] == p.v ? vv : c.v[k] == p.bern ? bn : vo[h][k];
                double r;
                if (c.atx0[k]) {  // lmmse_mult(mu0) from a precomputed A^T(A mu0): res*=tau; res+=gam2*v
                    double dv = a0[h][k];
                    dv *= tau;
                    dv += cgam2 * muv[h][k];
                    r = vi - dv;
                } else {
                    r = c.d[k] ? vi - dd[h][k] : vi - 0.0;  // r = v - lmmse_mult(mu0)
                }
                const double z = r / diag;
                c.r[k][i] = r;
                c.z[k][i] = z;
                c.p[k][i] = z;
                acc[2 * k] += r * z;
                acc[2 * k + 1] += vi * vi;
            }
        }
    }
    block_put_sums<2 * kMaxRhs>(acc, 2 * K, ro, (int64_t)blockIdx.x * 2 * K);
    if (red_finish(ro, 2 * K, lds, fin) && dst && threadIdx.x == 0) {
        *dst = start;  // then its sums (indexed in place: no stack copy of the state)
        dst->gam2 = cgam2;
        for (int k = 0; k < K; ++k) {
            dst->rz[k] = fin[2 * k];
            dst->vv[k] = fin[2 * k + 1];
        }
    }
}

hipError_t prelude_cg_init(int K, int64_t M, const Prelude& p, const CgVecs& c, double diag, const RedOut& ro,
                           const CgState* start, CgState* dst, hipStream_t st) {
    hipLaunchKernelGGL(prelude_cg_init_kernel, dim3(red_blocks(M)), dim3(kBlock), 0, st, K, M, p, c, diag, ro,
                       start ? *start : CgState{}, start ? dst : nullptr);
    return hipGetLastError();
}

hipError_t cg_init(int K, int64_t M, const CgVecs& c, double diag, const RedOut& ro, hipStream_t st) {
    hipLaunchKernelGGL(cg_init_kernel, dim3(red_blocks(M)), dim3(kBlock), 0, st, K, M, c, diag, ro);
    return hipGetLastError();
}

__global__ void cg_start_kernel(CgState init, CgState* dst) {
    if (threadIdx.x == 0) *dst = init;
}

hipError_t cg_start(const CgState& init, CgState* dst, hipStream_t st) {
    hipLaunchKernelGGL(cg_start_kernel, dim3(1), dim3(64), 0, st, init, dst);
    return hipGetLastError();
}

__global__ void cg_start_from_kernel(CgState init, const double* __restrict__ sums, CgState* dst,
                                     const double* __restrict__ gam2dev) {
    if (threadIdx.x != 0) return;
    for (int k = 0; k < init.K; ++k) {
        init.rz[k] = sums[2 * k];
        init.vv[k] = sums[2 * k + 1];
    }
    if (gam2dev) init.gam2 = gam2dev[0];
    *dst = init;
}

hipError_t cg_start_from(const CgState& init, const double* sums, CgState* dst, hipStream_t st,
                         const double* gam2dev) {
    hipLaunchKernelGGL(cg_start_from_kernel, dim3(1), dim3(64), 0, st, init, sums, dst, gam2dev);
    return hipGetLastError();
}

__global__ void cg_decide_kernel(CgState* cs, const double* __restrict__ red, int it, CgMirror* mirror,
                                 unsigned long long* flag, unsigned long long seq, int mask, int pack) {
    if (threadIdx.x == 0) cg_decide_body(cs, red, it, mirror, flag, seq, mask, pack);
}

// Latency, not bytes, sets this kernel's time at C2 (~25 MB in ~16 us): a
// chain of dependent memory round trips.  So every scalar comes in one burst
// (the whole CgState: the deciding block needs no further state load), both
// M-elements of a thread and a tile's N-vectors are loaded before the
// dependent work, and the decision takes its sums from LDS.  One
// instantiation per system count K: the unrolled per-system loops then carry
// K systems, not kMaxRhs (at K = 2: a quarter of the live registers, no
// spills, and only the K systems' vector pointers loaded from the arguments);
// every per-element operation and every sum is the same, in the same order.
// CGU_ABL (experiment builds only, results wrong; tools/cgu_ablation.sh):
// 1 = no slot sums / N-side updates, 2 = no M-side loads / stores, 4 = no
// decision, 8 = no last-block sums (nor decision), 16 = no partials and no
// ticket, 32 = a constant state instead of *cs and <d,p>
#ifndef CGU_ABL
#define CGU_ABL 0
#endif
template <int K, int W>
__global__ __launch_bounds__(kBlock) void cg_update_kernel(int64_t M, CgVecs c, double diag,
                                                           CgState* cs, const double* __restrict__ dp_dev,
                                                           const double* __restrict__ pp_dev, int fuse, RedOut ro,
                                                           CgDecide dc, int mblocks) {
#if CGU_ABL & 32
    CgState st{};
    st.K = K;
    st.any = 1;
    for (int k = 0; k < K; ++k) {
        st.active[k] = 1;
        st.rz[k] = st.vv[k] = 1.0;
    }
    double dpv[K], ppv[K];
    for (int k = 0; k < K; ++k) dpv[k] = 1.0, ppv[k] = 0.0;
#else
    const CgState st = *cs;
    double dpv[K], ppv[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        dpv[k] = dp_dev[k];
        ppv[k] = pp_dev ? pp_dev[k] : 0.0;
    }
#endif
    if (!st.any) return;
    __shared__ double fin[3 * kMaxRhs];  // the step's final sums, for the deciding thread
    // blocks [0, mblocks) stream the M-vectors; with c.adpart the blocks past
    // them sum the operator's A d partials and update the N-vectors
    const bool mpart = (int)blockIdx.x < mblocks;
    double alpha[K];
    bool on[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        on[k] = st.active[k] && ((dc.mask >> k) & 1);
        const double dp = pp_dev ? c.tau * dpv[k] + c.gam2 * ppv[k] : dpv[k];  // <d,p>
        alpha[k] = on[k] ? st.rz[k] / dp : 0.0;  // :702
    }
    double acc[3 * K];
#pragma unroll
    for (int q = 0; q < 3 * K; ++q) acc[q] = 0.0;
    double beta[K];
    bool fk[K];  // system k's direction update p = z + beta p rides in this step
#pragma unroll
    for (int k = 0; k < K; ++k) {
        fk[k] = on[k] && ((fuse >> k) & 1);
        beta[k] = fk[k] ? st.beta[k] : 0.0;
    }
    // two elements per round (i, i + stride), both loaded before either is
    // stored (the vectors may alias as far as the compiler knows: loads after
    // a store would wait for it); the sums still run over i, i + stride, ...
    // in order, as one element per round would
    const int64_t mstride = (int64_t)mblocks * kBlock;
    // (W < 32, the large-N plans: one element per round, fewer registers and
    // more workgroups per CU; the same sums in the same order)
    constexpr int H = W >= 32 || K >= 3 ? 2 : 1;  // (K >= 3 keeps two: one would spill to scratch)
    for (int64_t i0 = (int64_t)blockIdx.x * kBlock + threadIdx.x; mpart && !(CGU_ABL & 2) && i0 < M;
         i0 += H * mstride) {
        double pv[H][K], zv[H][K], muv[H][K], rv[H][K], dv[H][K], vv[H][K], wv[H][K], sv[H][K];
        const bool two = H == 2 && i0 + mstride < M;
#pragma unroll
        for (int h = 0; h < H; ++h) {
            const int64_t i = i0 + h * mstride;
            if (h == 1 && !two) break;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                if (on[k]) {
                    pv[h][k] = c.p[k][i];
                    zv[h][k] = fk[k] ? c.z[k][i] : 0.0;
                    muv[h][k] = c.mu[k][i];
                    rv[h][k] = c.r[k][i];
                    dv[h][k] = c.d[k][i];
                    vv[h][k] = c.v[k][i];
                    wv[h][k] = c.W[k] ? c.W[k][i] : 0.0;
                    sv[h][k] = c.W[k] ? c.S[k][i] : 0.0;
                }
            }
        }
#pragma unroll
        for (int h = 0; h < H; ++h) {
            const int64_t i = i0 + h * mstride;
            if (h == 1 && !two) break;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                if (on[k]) {
                    double pi = pv[h][k];
                    if (fk[k]) {  // p = z + beta p (:738-739)
                        pi = zv[h][k] + beta[k] * pi;
                        c.p[k][i] = pi;
                    }
                    const double mu = muv[h][k] + alpha[k] * pi;  // mu += alpha * p
                    const double r = rv[h][k] - dv[h][k] * alpha[k];  // r -= d * alpha
                    const double z = r / diag;
                    c.mu[k][i] = mu;
                    c.r[k][i] = r;
                    c.z[k][i] = z;
                    if (c.W[k]) c.W[k][i] = wv[h][k] + alpha[k] * sv[h][k];  // A^T A mu, as mu += alpha p
                    acc[3 * k] += r * z;
                    acc[3 * k + 1] += r * r;
                    acc[3 * k + 2] += vv[h][k] * mu;
                }
            }
        }
    }
    // A mu alongside mu (replicated N-vectors, the same on every rank)
    if (c.adpart) {
        // one rank, one-pass operator: A d from the operator's slots, in
        // op_reduce's order (tiles of 128 samples of one system)
        __shared__ v2d wsum[4][64];
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, ns = c.adslots;
        const int nb = (int)gridDim.x - mblocks;
        const int64_t tpk = (c.nA + 127) / 128;  // tiles per system
        for (int64_t tile = (int)blockIdx.x - mblocks; !(CGU_ABL & 1) && !mpart && tile < K * tpk; tile += nb) {
            const int k = (int)(tile / tpk);
            const int64_t i = (tile - k * tpk) * 128 + 2 * lane;  // < adld (a multiple of 16)
            const bool ok = i < c.nA;
            bool onk = false, fuk = false;  // on[k], fk[k], alpha[k], beta[k] without indexing registers at run time
            double alk = 0.0, bek = 0.0;
#pragma unroll
            for (int kk = 0; kk < (K < kOpMaxK ? K : kOpMaxK); ++kk)
                if (kk == k) {
                    onk = on[kk];
                    fuk = fk[kk];
                    alk = alpha[kk];
                    bek = beta[kk];
                }
            // wave 0's N-vectors of the tile, loaded before the slot sums (pairs
            // of samples: i + 1 < adld, the pads lie inside the vectors)
            const bool upd = w == 0 && ok && onk;
            v2d arv{0.0, 0.0}, qov{0.0, 0.0}, awv{0.0, 0.0};
            if (upd) {
                arv = *reinterpret_cast<const v2d*>(c.AR[k] + i);
                if (fuk) qov = *reinterpret_cast<const v2d*>(c.Q[k] + i);
                if (c.AW[k]) awv = *reinterpret_cast<const v2d*>(c.AW[k] + i);
            }
            wsum[w][lane] = ok ? slot_sum<W>(c.adpart + (int64_t)k * c.adld + i, (int64_t)kMaxRhs * c.adld,
                                             w * ns / 4, (w + 1) * ns / 4)
                               : v2d{0.0, 0.0};
            __syncthreads();
            if (upd) {
                const v2d ad = (((wsum[0][lane] + wsum[1][lane]) + wsum[2][lane]) + wsum[3][lane]) / c.addiv;
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const int64_t j = i + e;
                    if (j >= c.nA) break;
                    double q = arv[e] / diag;
                    if (fuk) q = q + bek * qov[e];
                    c.Q[k][j] = q;
                    if (c.AW[k]) c.AW[k][j] = awv[e] + alk * q;
                    c.AR[k][j] = arv[e] - ad[e] * alk;
                }
            }
            __syncthreads();
        }
    } else if (c.Q[0]) {  // one-pass operator: q (the step's A p) from A r, then A r -= A d * alpha
        for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < c.nA; i += (int64_t)gridDim.x * kBlock) {
            double ar[K], qo[K], ad[K], aw[K];
#pragma unroll
            for (int k = 0; k < K; ++k)
                if (on[k]) {
                    ar[k] = c.AR[k][i];
                    qo[k] = fk[k] ? c.Q[k][i] : 0.0;
                    ad[k] = c.addiv > 0 ? c.AD[k][i] / c.addiv : c.AD[k][i];  // (vec_div's division)
                    aw[k] = c.AW[k] ? c.AW[k][i] : 0.0;
                }
#pragma unroll
            for (int k = 0; k < K; ++k)
                if (on[k]) {
                    double q = ar[k] / diag;  // A z = A r / diag
                    if (fk[k]) q = q + beta[k] * qo[k];  // A p = A z + beta A p
                    c.Q[k][i] = q;
                    if (c.AW[k]) c.AW[k][i] = aw[k] + alpha[k] * q;
                    c.AR[k][i] = ar[k] - ad[k] * alpha[k];
                }
        }
    } else
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < c.nA; i += (int64_t)gridDim.x * kBlock) {
        double aw[K], as[K];
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (on[k] && c.AW[k]) {
                aw[k] = c.AW[k][i];
                as[k] = c.AS[k][i];
            }
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (on[k] && c.AW[k]) c.AW[k][i] = aw[k] + alpha[k] * as[k];
    }
    // The M-side blocks publish their sums.  The slot-sum blocks' sums are
    // zero: they publish none, and the last block adds the first mblocks
    // blocks' partials (the same partials in the same order, without the
    // zeros: the same bits).  Every block still takes the ticket, so that the
    // decision below, which rewrites *cs, follows every block's read of the
    // state; a slot-sum block takes it without waiting for its vector stores
    // (the decision reads none of them; the next launch sees them after the
    // kernel boundary).
    bool last = false;
    if (CGU_ABL & 16) {
    } else if (mpart) {
        block_put_sums<3 * K>(acc, 3 * K, ro, (int64_t)blockIdx.x * 3 * K);
        last = red_ticket(ro, (int)gridDim.x);
    } else {
        last = red_ticket_nowait(ro, (int)gridDim.x);
    }
    if (last && !(CGU_ABL & 8)) red_final(ro, 3 * K, mblocks, fin, true);
    // one rank: the last block decides the step itself (its sums are final),
    // from the state read at the start (only this decision writes it)
    if (last && dc.on && threadIdx.x == 0 && !(CGU_ABL & 12)) {
        double r[3 * kMaxRhs];
#pragma unroll
        for (int q = 0; q < 3 * kMaxRhs; ++q) r[q] = q < 3 * K ? fin[q] : 0.0;
        cg_decide_from(st, cs, r, dc.it, dc.mirror, dc.flag, dc.seq, dc.mask, dc.pack);
    }
}

constexpr int kCguBlocks = 512;
hipError_t cg_update(int K, int64_t M, const CgVecs& c, double diag, CgState* cs, const double* dp_dev,
                     const double* pp_dev, int fuse, const RedOut& ro, const CgDecide& dc, hipStream_t st) {
    // VAMPOMI_CG_EPT: M elements per thread (tuning experiments; default 2, red_blocks)
    static const int ept = std::getenv("VAMPOMI_CG_EPT") ? std::max(1, std::atoi(std::getenv("VAMPOMI_CG_EPT"))) : 2;
    const int mb = (int)std::min<int64_t>(std::max<int64_t>(cdiv(M, (int64_t)kBlock * ept), 1), kRedBlocks / 2);
    int nb = 0;
    if (c.adpart) {
        if (K > kOpMaxK || c.adslots < 1 || !c.Q[0]) return hipErrorInvalidValue;
        // at most kCguBlocks workgroups in all (two per CU): every one takes the
        // step's ticket, and beyond that their arrivals cost more than the tiles
        // they share (C4 shard, 782 slot-sum workgroups: 164.8 -> 127.4 us of
        // cg_update per iteration at 400, 142.0 at 158; C2's 158 is best at C2,
        // profiles/r06n_cgu_blocks.txt).  Each workgroup takes tiles nb apart,
        // the same tiles summed the same way: bitwise the same for any nb.
        // VAMPOMI_CGU_NB: the count itself (tuning experiments)
        static const int nbset = std::getenv("VAMPOMI_CGU_NB") ? std::atoi(std::getenv("VAMPOMI_CGU_NB")) : 0;
        nb = (int)std::min<int64_t>(K * cdiv(c.nA, 128), nbset > 0 ? nbset : std::max(kCguBlocks - mb, 1));
        nb = std::max(std::min(nb, kRedBlocks - mb), 1);
    }
    // the 32-load slot rounds only where a wave sums >= 32 slots (C2's team of
    // 2); else rounds of <= 8 loads and the registers of more workgroups per CU
    const bool wide = c.adpart && c.adslots >= 4 * 32;
#define VAMPOMI_CGU(KK)                                                                                          \
    case KK:                                                                                                     \
        if (wide)                                                                                                \
            hipLaunchKernelGGL((cg_update_kernel<KK, 32>), dim3(mb + nb), dim3(kBlock), 0, st, M, c, diag, cs,   \
                               dp_dev, pp_dev, fuse, ro, dc, mb);                                                \
        else                                                                                                     \
            hipLaunchKernelGGL((cg_update_kernel<KK, 8>), dim3(mb + nb), dim3(kBlock), 0, st, M, c, diag, cs,    \
                               dp_dev, pp_dev, fuse, ro, dc, mb);                                                \
        break;
    switch (K) {
        VAMPOMI_CGU(1)
        VAMPOMI_CGU(2)
        VAMPOMI_CGU(3)
        VAMPOMI_CGU(4)
        default: return hipErrorInvalidValue;
    }
#undef VAMPOMI_CGU
    return hipGetLastError();
}

hipError_t cg_decide(CgState* cs, const double* red, int it, CgMirror* mirror, unsigned long long* flag,
                     unsigned long long seq, hipStream_t st, int mask, int pack) {
    hipLaunchKernelGGL(cg_decide_kernel, dim3(1), dim3(64), 0, st, cs, red, it, mirror, flag, seq, mask, pack);
    return hipGetLastError();
}


// ---------------------------------------------------------------------------
// probit model: N-side denoiser and accuracy counts (src/vamp_probit.cpp)
// ---------------------------------------------------------------------------
// erfcx as the reference evaluates it (src/utilities.cpp:293-363: N. Juffa's
// published fma approximation, with +inf below -10 and lowest() above 10).
// Same operations in the same order as the oracle's orc_erfcx.  exp() is the
// correctly rounded exp_cr (exp_cr.h), not OCML's ~1-ulp exp: it equals glibc's
// (the oracle's, the reference's) except where glibc misrounds, 0.08 % of the
// arguments (tests/exp_cr_check.c).
__constant__ double kErfcxPoly[24] = {
    0x1.edcad78fc8044p-31,  0x1.b1548f14735d1p-30,  -0x1.a1ad2e6c4a7a8p-27, -0x1.1985b48f08574p-26,
    0x1.c6a8093ac4f83p-24,  0x1.31c2b2b44b731p-24,  -0x1.b87373facb29fp-21, 0x1.3fef1358803b7p-22,
    0x1.7eec072bb0be3p-18,  -0x1.78a680a741c4ap-17, -0x1.9951f39295cf4p-16, 0x1.3be1255ce180bp-13,
    -0x1.a1df71176b791p-13, -0x1.8d4aaa0099bc8p-11, 0x1.49c673066c831p-8,   -0x1.0962386ea02b7p-6,
    0x1.3079edf465cc3p-5,   -0x1.0fb06dfedc4ccp-4,  0x1.7fee004e266dfp-4,   -0x1.9ddb23c3e14d2p-4,
    0x1.16ecefcfa4865p-4,   0x1.f7f5df66fc349p-7,   -0x1.1df1ad154a27fp-3,  0x1.dd2c8b74febf6p-3};

__device__ __forceinline__ double erfcx_ref(double x) {
    if (x < -10.0) return __builtin_inf();
    if (x > 10.0) return -1.7976931348623157e308;
    const double a = fmax(x, 0.0 - x);
    const double inv = 1.0 / (a + 4.0);
    double q = (a - 4.0) * inv;
    const double t0 = __builtin_fma(q + 1.0, -4.0, a);
    q = __builtin_fma(inv, __builtin_fma(q, -a, t0), q);
    double p = kErfcxPoly[0];
#pragma unroll
    for (int k = 1; k < 24; ++k) p = __builtin_fma(p, q, kErfcxPoly[k]);
    const double h = (1.0 / (a + 0.5)) * 0.5;
    const double q1 = __builtin_fma(p, h, h);
    const double res = (p - q1) + __builtin_fma(q1 + q1, -a, 1.0);
    double r = __builtin_fma(res, h, q1);
    if (a > 1.7976931348623157e308) r = 0.0;
    if (x < 0.0) {
        const double s = x * x;
        const double lo = __builtin_fma(x, x, -s);
        const double e = exp_cr(s);
        r = __builtin_fma(e, lo + lo, e - r) + e;
        if (e > 1.7976931348623157e308) r = e;
    }
    return r;
}

__global__ __launch_bounds__(kBlock) void probit_denoise_kernel(int64_t N, const double* __restrict__ p1,
                                                                const double* __restrict__ y, double tau1,
                                                                double* __restrict__ z1, RedOut ro) {
    __shared__ double lds[4];
    const double sq = sqrt(1.0 + 1.0 / tau1);           // sqrt(probit_var + 1/tau1)
    const double k0 = 2.0 / sqrt(2 * M_PI), rt2 = sqrt(2.0);
    const double den = 1 + tau1 * 1.0;                  // 1 + tau1*probit_var
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < N; i += (int64_t)gridDim.x * kBlock) {
        const double p = p1[i], s = 2 * y[i] - 1;
        const double c = (p + 0.0) / sq;
        const double ratio = k0 / erfcx_ref(-s * c / rt2);
        z1[i] = p + s * ratio / tau1 / sq;
        acc += 1 - ratio / den * (s * c + ratio);
    }
    acc = block_sum(acc, lds);
    if (threadIdx.x == 0) red_put(ro, blockIdx.x, acc);
    red_finish(ro, 1, lds);
}

hipError_t probit_denoise(int64_t N, const double* p1, const double* y, double tau1, double* z1, const RedOut& ro,
                          hipStream_t st) {
    hipLaunchKernelGGL(probit_denoise_kernel, dim3(red_blocks(N)), dim3(kBlock), 0, st, N, p1, y, tau1, z1, ro);
    return hipGetLastError();
}

__global__ __launch_bounds__(kBlock) void confusion_kernel(int64_t N, int nz, const double* __restrict__ z,
                                                           int64_t ld, const double* __restrict__ y,
                                                           RedOut ro) {
    __shared__ double lds[4];
    double cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < N; i += (int64_t)gridDim.x * kBlock) {
        const double yi = y[i];
        for (int k = 0; k < nz; ++k) {
            const double yh = (0.5 * erfc(-z[k * ld + i] * M_SQRT1_2) >= 0.5) ? 1.0 : 0.0;  // normal_cdf >= th
            if (yi == 1 && yh == 1)
                cnt[4 * k + 0] += 1;
            else if (yi == 0 && yh == 0)
                cnt[4 * k + 1] += 1;
            else if (yi == 0 && yh == 1)
                cnt[4 * k + 2] += 1;
            else if (yi == 1 && yh == 0)
                cnt[4 * k + 3] += 1;
        }
    }
    block_put_sums<8>(cnt, 4 * nz, ro, (int64_t)blockIdx.x * 4 * nz);
    red_finish(ro, 4 * nz, lds);
}

hipError_t probit_confusion(int64_t N, int nz, const double* z, int64_t ld, const double* y, const RedOut& ro,
                            hipStream_t st) {
    if (nz < 1 || nz > 2) return hipErrorInvalidValue;
    hipLaunchKernelGGL(confusion_kernel, dim3(red_blocks(N)), dim3(kBlock), 0, st, N, nz, z, ld, y, ro);
    return hipGetLastError();
}

__global__ void probit_p1_kernel(uint64_t seed, int64_t N, double* p1) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < N) p1[i] = gauss_dyadic(seed ^ 0x50524F4249545031ULL, 0, i);
}

hipError_t probit_p1(uint64_t seed, int64_t N, double* p1, hipStream_t st) {
    if (N <= 0) return hipSuccess;
    hipLaunchKernelGGL(probit_p1_kernel, dim3((unsigned)cdiv(N, kBlock)), dim3(kBlock), 0, st, seed, N, p1);
    return hipGetLastError();
}


// ---------------------------------------------------------------------------
// association tests: data::pvals_loo (src/data.cpp:385-417) and the SE
// p-values (src/main_meth.cpp:218-242)
// ---------------------------------------------------------------------------
// One pass over the RAW shard: a wave owns G markers, lanes stride the
// samples (16-B nontemporal loads, 1 KiB per wave per load), every ymod
// value serves G markers.  Per element exactly the reference's
// ym = ymod + (X / sqrt(N)) * x1_j, then the five sums of linear_reg1d_pvals.
// Pad rows are zero in X and ymod and add exact zeros.
//
// X / sqrt(N) is the correctly rounded quotient either way: FASTDIV computes
// q0 = X*r (r = RN(1/sqrt(N))), the exact residual e = fma(-q0, sqrt(N), X)
// and q = fma(e, r, q0), which is RN(X/sqrt(N)) whenever r is the rounded
// reciprocal and q0 is within one ulp (Markstein's theorem; checked
// bit for bit against IEEE division in tests/test_hostio.py and on the
// device in tests/test_gpu_assoc.py) — 3 instructions instead of the ~10 of
// the IEEE division sequence, which made the pass ALU-bound.  Only the sign
// of a zero quotient can differ, which no sum can see.  Every lane adds its
// samples in increasing order whatever G / UJ are, so all variants give
// bitwise identical sums.
template <int G, int UJ, bool FASTDIV>
__global__ __launch_bounds__(kBlock) void loo_kernel(const double* __restrict__ X, int64_t ld, int64_t N, int64_t M,
                                                     const double* __restrict__ ymod, const double* __restrict__ x1,
                                                     double sqrtN, double* __restrict__ stats) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t m0 = ((int64_t)blockIdx.x * (blockDim.x >> 6) + wave) * G;
    const double rinv = 1.0 / sqrtN;
    double acc[G][5];
    double xj[G];
    const double* col[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int64_t m = (m0 + g < M) ? m0 + g : M - 1;  // clamp: in-bounds, discarded
        xj[g] = x1[m];
        col[g] = X + m * ld;
#pragma unroll
        for (int q = 0; q < 5; ++q) acc[g][q] = 0.0;
    }
    auto add = [&](int g, double m, double y) {
        double q;
        if (FASTDIV) {
            const double q0 = m * rinv;
            q = __builtin_fma(__builtin_fma(-q0, sqrtN, m), rinv, q0);
        } else {
            q = m / sqrtN;
        }
        const double ym = y + q * xj[g];
        acc[g][0] += m;
        acc[g][1] += m * m;
        acc[g][2] += m * ym;
        acc[g][3] += ym;
        acc[g][4] += ym * ym;
    };
    int64_t j = 2 * lane;
    for (; j + 128 * (UJ - 1) < N; j += 128 * UJ) {
        v2d yy[UJ], xx[UJ][G];
#pragma unroll
        for (int t = 0; t < UJ; ++t)
#pragma unroll
            for (int g = 0; g < G; ++g) xx[t][g] = ld_stream(col[g] + j + 128 * t);
#pragma unroll
        for (int t = 0; t < UJ; ++t) yy[t] = ld2(ymod + j + 128 * t);
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int t = 0; t < UJ; ++t) {
                add(g, xx[t][g].x, yy[t].x);
                add(g, xx[t][g].y, yy[t].y);
            }
    }
    for (; j < N; j += 128) {
        v2d xx[G];
#pragma unroll
        for (int g = 0; g < G; ++g) xx[g] = ld_stream(col[g] + j);
        const v2d yy = ld2(ymod + j);
#pragma unroll
        for (int g = 0; g < G; ++g) {
            add(g, xx[g].x, yy.x);
            add(g, xx[g].y, yy.y);
        }
    }
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            const double s = wave_sum(acc[g][q]);
            if (lane == 0 && m0 + g < M) stats[5 * (m0 + g) + q] = s;
        }
}

// The same sums with W waves of a workgroup sharing its G markers: wave w,
// lane l takes rows 2l + 128 (w + W t), so one load round of the workgroup
// reads W KiB contiguous of each column (the wave-per-marker form above reads
// 1 KiB per wave from columns all over the shard); the W wave sums meet in
// LDS and are added in wave order.
template <int G, int UJ, int W>
__global__ __launch_bounds__(64 * W) void loo_wg_kernel(const double* __restrict__ X, int64_t ld, int64_t N, int64_t M,
                                                        const double* __restrict__ ymod, const double* __restrict__ x1,
                                                        double sqrtN, double* __restrict__ stats) {
    __shared__ double part[W][5 * G];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t m0 = (int64_t)blockIdx.x * G;
    const double rinv = 1.0 / sqrtN;
    double acc[G][5];
    double xj[G];
    const double* col[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int64_t m = (m0 + g < M) ? m0 + g : M - 1;  // clamp: in-bounds, discarded
        xj[g] = x1[m];
        col[g] = X + m * ld;
#pragma unroll
        for (int q = 0; q < 5; ++q) acc[g][q] = 0.0;
    }
    auto add = [&](int g, double m, double y) {  // loo_kernel's, fma-corrected division
        const double q0 = m * rinv;
        const double q = __builtin_fma(__builtin_fma(-q0, sqrtN, m), rinv, q0);
        const double ym = y + q * xj[g];
        acc[g][0] += m;
        acc[g][1] += m * m;
        acc[g][2] += m * ym;
        acc[g][3] += ym;
        acc[g][4] += ym * ym;
    };
    constexpr int64_t RS = 128 * W;  // rows per load round of the workgroup
    int64_t j = 2 * lane + 128 * wave;
    for (; j + RS * (UJ - 1) < N; j += RS * UJ) {
        v2d yy[UJ], xx[UJ][G];
#pragma unroll
        for (int t = 0; t < UJ; ++t)
#pragma unroll
            for (int g = 0; g < G; ++g) xx[t][g] = ld_stream(col[g] + j + RS * t);
#pragma unroll
        for (int t = 0; t < UJ; ++t) yy[t] = ld2(ymod + j + RS * t);
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int t = 0; t < UJ; ++t) {
                add(g, xx[t][g].x, yy[t].x);
                add(g, xx[t][g].y, yy[t].y);
            }
    }
    for (; j < N; j += RS) {  // (N even or the pad row: ld-padded columns, zero pads)
        v2d xx[G];
#pragma unroll
        for (int g = 0; g < G; ++g) xx[g] = ld_stream(col[g] + j);
        const v2d yy = ld2(ymod + j);
#pragma unroll
        for (int g = 0; g < G; ++g) {
            add(g, xx[g].x, yy.x);
            add(g, xx[g].y, yy.y);
        }
    }
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            const double s = wave_sum(acc[g][q]);
            if (lane == 0) part[wave][5 * g + q] = s;
        }
    __syncthreads();
    if ((int)threadIdx.x < 5 * G && m0 + threadIdx.x / 5 < M) {
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < W; ++w) s += part[w][threadIdx.x];
        stats[5 * m0 + threadIdx.x] = s;
    }
}

struct LooVariant { int G, UJ; bool FD; int W = 0; };  // W > 0: loo_wg_kernel
static constexpr LooVariant kLooVariants[] = {
    {4, 2, true}, {4, 2, false}, {2, 2, true}, {8, 1, true}, {4, 1, true}, {4, 4, true}, {2, 4, true}, {8, 2, true},
    {1, 2, true, 8}, {2, 2, true, 8}, {1, 4, true, 8}, {2, 4, true, 8}, {2, 2, true, 4}, {4, 2, true, 4},
    {4, 1, true, 4}, {8, 1, true, 4}, {4, 2, true, 8}, {4, 2, true, 2}, {8, 2, true, 2}, {4, 4, true, 2},
};
static constexpr int kNumLooVariants = sizeof(kLooVariants) / sizeof(kLooVariants[0]);
// default (round 3): 16, loo_wg_kernel<4, 2, 8>: 7.00 TB/s at the c5 shard (N=100,000 x 62,500) on
// MI355X against 6.81 TB/s for the round-1 default 2 (loo_kernel<2, 2, true>, fma-corrected division,
// itself 6.80 against 5.63 TB/s with the IEEE division sequence); tools/kbench.py,
// profiles/r03l_kbench_loo.txt, profiles/r01_kbench_loo.json
int loo_variant_count() { return kNumLooVariants; }
bool loo_variant_ok(int v) { return v >= 0 && v < kNumLooVariants; }

std::string loo_kernel_name(int variant) {
    const LooVariant& v = kLooVariants[loo_variant_ok(variant) ? variant : kLooDefault];
    char b[64];
    if (v.W > 0)
        std::snprintf(b, sizeof b, "loo_wg_kernel<%d, %d, %d>", v.G, v.UJ, v.W);
    else
        std::snprintf(b, sizeof b, "loo_kernel<%d, %d, %s>", v.G, v.UJ, v.FD ? "true" : "false");
    return b;
}

template <int G, int UJ, bool FD>
static void launch_loo(const Shard& s, const double* ymod, const double* x1, double sqrtN, double* stats,
                       hipStream_t st, const Timing& tm) {
    // two waves per workgroup, as A^T.u (C5 shape: 7339 vs 7477 us with four);
    // VAMPOMI_LOO_WPB: tuning experiments
    static const int wpb = std::getenv("VAMPOMI_LOO_WPB") ? std::max(1, std::min(4, std::atoi(std::getenv("VAMPOMI_LOO_WPB")))) : 2;
    hipExtLaunchKernelGGL((loo_kernel<G, UJ, FD>), dim3((unsigned)cdiv(s.M, wpb * G)), dim3(64 * wpb), 0, st, tm.start,
                          tm.stop, 0, s.X, s.ld, s.N, s.M, ymod, x1, sqrtN, stats);
}

template <int G, int UJ, int W>
static void launch_loo_wg(const Shard& s, const double* ymod, const double* x1, double sqrtN, double* stats,
                          hipStream_t st, const Timing& tm) {
    hipExtLaunchKernelGGL((loo_wg_kernel<G, UJ, W>), dim3((unsigned)cdiv(s.M, G)), dim3(64 * W), 0, st, tm.start,
                          tm.stop, 0, s.X, s.ld, s.N, s.M, ymod, x1, sqrtN, stats);
}

hipError_t loo_sums(const Shard& s, const double* ymod, const double* x1, double sqrtN, double* stats,
                    hipStream_t st, int variant, const Timing& tm) {
    if (s.M <= 0) return hipSuccess;
    switch (variant) {
        case 8: launch_loo_wg<1, 2, 8>(s, ymod, x1, sqrtN, stats, st, tm); break;
        case 9: launch_loo_wg<2, 2, 8>(s, ymod, x1, sqrtN, stats, st, tm); break;
        case 10: launch_loo_wg<1, 4, 8>(s, ymod, x1, sqrtN, stats, st, tm); break;
        case 11: launch_loo_wg<2, 4, 8>(s, ymod, x1, sqrtN, stats, st, tm); break;
        case 12: launch_loo_wg<2, 2, 4>(s, ymod, x1, sqrtN, stats, st, tm); break;
        case 13: launch_loo_wg<4, 2, 4>(s, ymod, x1, sqrtN, stats, st, tm); break;
        case 14: launch_loo_wg<4, 1, 4>(s, ymod, x1, sqrtN, stats, st, tm); break;
        case 15: launch_loo_wg<8, 1, 4>(s, ymod, x1, sqrtN, stats, st, tm); break;
        case 16: launch_loo_wg<4, 2, 8>(s, ymod, x1, sqrtN, stats, st, tm); break;
        case 17: launch_loo_wg<4, 2, 2>(s, ymod, x1, sqrtN, stats, st, tm); break;
        case 18: launch_loo_wg<8, 2, 2>(s, ymod, x1, sqrtN, stats, st, tm); break;
        case 19: launch_loo_wg<4, 4, 2>(s, ymod, x1, sqrtN, stats, st, tm); break;
        case 0: launch_loo<4, 2, true>(s, ymod, x1, sqrtN, stats, st, tm); break;
        case 1: launch_loo<4, 2, false>(s, ymod, x1, sqrtN, stats, st, tm); break;
        case 2: launch_loo<2, 2, true>(s, ymod, x1, sqrtN, stats, st, tm); break;
        case 3: launch_loo<8, 1, true>(s, ymod, x1, sqrtN, stats, st, tm); break;
        case 4: launch_loo<4, 1, true>(s, ymod, x1, sqrtN, stats, st, tm); break;
        case 5: launch_loo<4, 4, true>(s, ymod, x1, sqrtN, stats, st, tm); break;
        case 6: launch_loo<2, 4, true>(s, ymod, x1, sqrtN, stats, st, tm); break;
        case 7: launch_loo<8, 2, true>(s, ymod, x1, sqrtN, stats, st, tm); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ln B(a, 1/2) and the Student-t upper tail: the same operations as the
// oracle's orc_lnbeta_half / ibeta_cf / orc_t_sf (oracle/vamp_oracle.c),
// standing for Boost's complemented students_t cdf (src/utilities.cpp:278-279)
__device__ double lnbeta_half(double a) {
    if (a >= 30.0) {
        const double i1 = 1.0 / a, i2 = i1 * i1;
        const double d = 0.5 * log(a) - i1 * (1.0 / 8.0) + i1 * i2 * (1.0 / 192.0) - i1 * i2 * i2 * (1.0 / 640.0) +
                         i1 * i2 * i2 * i2 * (17.0 / 14336.0);
        return 0.57236494292470008707 - d;
    }
    return lgamma(a) + lgamma(0.5) - lgamma(a + 0.5);
}

__device__ double ibeta_cf(double a, double b, double x) {
    const double tiny = 1e-300, eps = 4e-16;
    const double qab = a + b, qap = a + 1.0, qam = a - 1.0;
    double c = 1.0, d = 1.0 - qab * x / qap;
    if (fabs(d) < tiny) d = tiny;
    d = 1.0 / d;
    double h = d;
    for (int m = 1; m <= 20000; ++m) {
        const double m2 = 2.0 * m;
        double aa = m * (b - m) * x / ((qam + m2) * (a + m2));
        d = 1.0 + aa * d;
        if (fabs(d) < tiny) d = tiny;
        c = 1.0 + aa / c;
        if (fabs(c) < tiny) c = tiny;
        d = 1.0 / d;
        h *= d * c;
        aa = -(a + m) * (qab + m) * x / ((a + m2) * (qap + m2));
        d = 1.0 + aa * d;
        if (fabs(d) < tiny) d = tiny;
        c = 1.0 + aa / c;
        if (fabs(c) < tiny) c = tiny;
        d = 1.0 / d;
        const double del = d * c;
        h *= del;
        if (fabs(del - 1.0) < eps) break;
    }
    return h;
}

__device__ double t_sf_pos(double t, double df) {  // t > 0
    const double a = 0.5 * df, b = 0.5, tt = t * t;
    const double lx = -log1p(tt / df);
    const double l1x = log(tt / (df + tt));
    const double x = df / (df + tt);
    const double front = exp(a * lx + b * l1x - lnbeta_half(a));
    if (t >= 3.0 && x < (a + 1.0) / (a + b + 2.0)) return 0.5 * (front * ibeta_cf(a, b, x) / a);
    return 0.5 * (1.0 - front * ibeta_cf(b, a, tt / (df + tt)) / b);
}

__device__ double t_sf(double t, double df) {
    if (isnan(t) || isnan(df)) return __builtin_nan("");
    if (t == 0.0) return 0.5;
    return t > 0.0 ? t_sf_pos(t, df) : 1.0 - t_sf_pos(-t, df);
}

__global__ void loo_pval_kernel(int64_t M, const double* __restrict__ stats, int n, double* __restrict__ pvals) {
    const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= M) return;
    const double* s = stats + 5 * j;
    const double sumx = s[0], sumsqx = s[1], sumxy = s[2], sumy = s[3], sumsqy = s[4];
    const double s2y = (sumsqy - sumy * sumy / n) / (n - 1);
    const double s2x = (sumsqx - sumx * sumx / n) / (n - 1);
    const double sxy = (sumxy - sumx * sumy / n) / (n - 1);
    const double rxy = sxy / sqrt(s2x * s2y);
    const double t = rxy * sqrt((n - 2) / (1 - rxy * rxy));
    pvals[j] = 2.0 * t_sf(t > 0 ? t : (0 - t), (double)(n - 2));
}

hipError_t loo_pvals(int64_t M, const double* stats, int n, double* pvals, hipStream_t st) {
    if (M <= 0) return hipSuccess;
    hipLaunchKernelGGL(loo_pval_kernel, dim3((unsigned)cdiv(M, kBlock)), dim3(kBlock), 0, st, M, stats, n, pvals);
    return hipGetLastError();
}

__global__ void se_pval_kernel(int64_t M, const double* __restrict__ r1, double sd, double* __restrict__ pvals) {
    const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= M) return;
    const double diff = (0.0 - r1[j]) / sd;  // boost normal cdf at 0: erfc(-diff / sqrt(2)) / 2
    double p = erfc(-diff / M_SQRT2) / 2;
    if (r1[j] <= 0.0) p = 1 - p;
    pvals[j] = p;
}

hipError_t se_pvals(int64_t M, const double* r1, double gam1, int64_t N, double* pvals, hipStream_t st) {
    if (M <= 0) return hipSuccess;
    const double sd = sqrt(1.0 / (gam1 * (double)N));
    hipLaunchKernelGGL(se_pval_kernel, dim3((unsigned)cdiv(M, kBlock)), dim3(kBlock), 0, st, M, r1, sd, pvals);
    return hipGetLastError();
}

__global__ void mul_scalar_kernel(int64_t n, const double* __restrict__ x, double a, double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) out[i] = x[i] * a;
}

hipError_t mul_scalar(int64_t n, const double* x, double a, double* out, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(mul_scalar_kernel, dim3((unsigned)cdiv(n, kBlock)), dim3(kBlock), 0, st, n, x, a, out);
    return hipGetLastError();
}

// completion flag for the host: a system-scope release store of seq into
// mapped host memory, after everything earlier on the stream
__global__ void signal_kernel(unsigned long long* flag, unsigned long long seq) {
    __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// a sequence number into mapped host memory after everything earlier on the
// stream; the iteration writer's "slot landed" word.  The staging data it
// announces was written by an earlier kernel with plain stores, so the store
// is a system-scope RELEASE: it writes back the L2 (the whole device's, not
// only this kernel's writes) before the word can be seen by the host, which
// does not rely on the packet fence scope or on the staging memory's mapping
// type.  One thread, once per iteration: the writeback costs nothing
__global__ void post_flag_kernel(unsigned long long* flag, unsigned long long seq) {
    __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t post_flag(unsigned long long* flag, unsigned long long seq, hipStream_t st) {
    hipLaunchKernelGGL(post_flag_kernel, dim3(1), dim3(1), 0, st, flag, seq);
    return hipGetLastError();
}

hipError_t signal_host(unsigned long long* flag, unsigned long long seq, hipStream_t st) {
    hipLaunchKernelGGL(signal_kernel, dim3(1), dim3(1), 0, st, flag, seq);
    return hipGetLastError();
}

// multi-rank DotBatch results: after the all-reduce, copy the synced and the
// local slot ranges into mapped host memory, then raise the host flag
__global__ void publish_kernel(const double* __restrict__ a, int na, double* __restrict__ ha, const double* __restrict__ b,
                               int nb, double* __restrict__ hb, unsigned long long* flag, unsigned long long seq) {
    for (int i = threadIdx.x; i < na; i += blockDim.x) ha[i] = a[i];
    for (int i = threadIdx.x; i < nb; i += blockDim.x) hb[i] = b[i];
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t publish_host(const double* a, int na, double* ha, const double* b, int nb, double* hb,
                        unsigned long long* flag, unsigned long long seq, hipStream_t st) {
    hipLaunchKernelGGL(publish_kernel, dim3(1), dim3(256), 0, st, a, na, ha, b, nb, hb, flag, seq);
    return hipGetLastError();
}

}  // namespace vk
