// atax_team.hip — the one-pass CG operator (kernels.h: atax) for every N:
// workgroup TEAMS that split each column's rows, with a lagged hand-off of
// the column dot products.
//
// A CG step needs, per marker i of the shard (src/vamp.cpp:645-662, 700;
// data::ATx src/data.cpp:294-333, data::Ax :340-373):
//   t_i = msig_i * sum_j (X_ij - mave_i) q_j / sqrt(N)       (A^T q)
//   d_i = tau*t_i + gam2*p_i                                  (lmmse_mult epilogue)
//   (A d)_j += (X_ij - mave_i) * msig_i * d_i                 (A d)
// and the axpy of column i needs column i's complete dot first.  A team of T
// workgroups (one per CU) shares a marker range; member r holds rows
// [r*TR, (r+1)*TR) of every column of it in registers.  Per column, each
// member sums its rows' partial dot (7 streaming waves, one LDS barrier) and
// publishes it as data-tagged 8-byte granules (MI355X_MICROARCH.md, hand-off
// R2: {tag, 32 bits}, write-through sc1 stores, no flag, no fence); an 8th,
// non-streaming wave polls the granules of the column L steps back, sums the
// T members in a fixed order and hands the total to the streaming waves
// through LDS, which finish that column from the copy still in registers.
// So X is read from HBM once per CG step for both products, at any N, and the
// hand-off latency hides behind L columns of streaming.  T = 1 (small N) is
// the same kernel without a hand-off: the 8 waves stream, L = 0.
//
// Memory ordering: every wave issues the same VMEM instructions per column
// (the X loads through a buffer descriptor whose range check drops the rows
// past the tile; the last column is re-issued instead of skipping), so the
// compiler's in-order vmcnt waits never drain the prefetched columns.  The
// polling wave streams nothing, so its waits on granule loads wait for
// nothing else.
//
// Results: every member forms the same totals (the T partials are summed by
// a fixed butterfly over lanes), the member owning a column (column % T)
// stores d and adds <d,p>; partial A d per team -> op_reduce (teams in
// order).  Bitwise reproducible run to run.
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdio>
#include <mutex>
#include <string>

#include "kdev.h"

namespace vk {

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned int v2u __attribute__((ext_vector_type(2)));

#ifndef TM_FMA
#define TM_FMA 1  // fused multiply-adds in the dot and the A d accumulation
#endif
static constexpr int kTmThreads = 512;        // 8 waves, 2 per SIMD: <= 256 VGPRs per lane
static constexpr int kTmMaxT = 32;            // members per team (one XCD under round-robin dealing)
static constexpr unsigned kTmMaxSpins = 1u << 21;  // ~2 s of polling, then the launch gives up (err)

// configurations: F columns prefetched, L steps of lag, P polls in flight,
// hand-off (T > 1), and the most 16-byte loads per lane per column that fit
// 256 VGPRs at K = 2 without spilling (gfx950, ROCm 7.2 compiler)
struct TmCfg {
    int F, L, P;
    bool comm;
    int maxS;
};
static constexpr TmCfg kTmCfg[] = {
    {1, 0, 0, false, 10},  // 0: T = 1, one column prefetched
    {2, 0, 0, false, 8},   // 1: T = 1, two
    {3, 5, 2, true, 4},    // 2
    {2, 4, 2, true, 5},    // 3
    {3, 6, 3, true, 4},    // 4
    {3, 6, 2, true, 4},    // 5
    {4, 5, 2, true, 4},    // 6
    {4, 6, 2, true, 4},    // 7
    {3, 4, 2, true, 4},    // 8
};
static constexpr int kTmNCfg = sizeof(kTmCfg) / sizeof(kTmCfg[0]);

__host__ __device__ constexpr int tm_rows_per_step(bool comm) { return 128 * (comm ? 7 : 8); }
// q in LDS: every lane row of the S steps (zeros past the tile, so those
// rows need no mask) when that fits beside the partials, else the tile only
// (rows past it masked)
__host__ __device__ constexpr bool tm_qfull(int K, int S, bool comm) {
    return (K * S * tm_rows_per_step(comm) + 4 * 8 * K) * 8 <= 160 * 1024;
}
__host__ __device__ constexpr int64_t tm_qstride(int K, int S, bool comm, int64_t tile_rows) {
    return tm_qfull(K, S, comm) ? (int64_t)S * tm_rows_per_step(comm) : (tile_rows + 1) & ~(int64_t)1;
}

__device__ __forceinline__ double readlane_d(double v, int l) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// Untracked 16-byte granule traffic of the hand-off wave (see there).
__device__ __forceinline__ void tm_poll(v4u& dst, const unsigned long long* p) {
    asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(dst) : "v"(p) : "memory");
}
template <int N>
__device__ __forceinline__ void tm_wait(v4u& r) {
    asm volatile("s_waitcnt vmcnt(%1)" : "+v"(r) : "n"(N) : "memory");
}
__device__ __forceinline__ void tm_load8(v2u& dst, const double* p) {
    asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(dst) : "v"(p) : "memory");
}
template <int N>
__device__ __forceinline__ void tm_wait2(v4u& r, v2u& q) {
    asm volatile("s_waitcnt vmcnt(%2)" : "+v"(r), "+v"(q) : "n"(N) : "memory");
}
__device__ __forceinline__ void tm_publish(unsigned long long* p, const v4u& v) {
    asm volatile("s_nop 4\n\tglobal_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
// the same store without write-through: the line stays in this XCD's L2
__device__ __forceinline__ void tm_publish_l2(unsigned long long* p, const v4u& v) {
    asm volatile("s_nop 4\n\tglobal_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

template <int K, int S, int F, int L, int P, bool COMM>
__global__ __launch_bounds__(kTmThreads) void atax_team_kernel(const double* __restrict__ X, int64_t ld, int64_t N,
                                                               int64_t M, const double* __restrict__ mave,
                                                               const double* __restrict__ msig, OpArgs a, int T,
                                                               int TR, const int* __restrict__ gate) {
    if (gate && !*gate) return;
    constexpr int CW = COMM ? 7 : 8;  // streaming waves
    constexpr int RS = tm_rows_per_step(COMM);
    constexpr int RING = F + L + 1;
    static_assert(COMM || L == 0, "without a hand-off the column is finished in its own step");
    static_assert(!COMM || (P >= 1 && P <= L), "polls in flight");
    static_assert(!COMM || P < RING, "a poll's slot is consumed before it is reissued");
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int g = blockIdx.x >> 3;
    const int member = g % T;
    const int team = (blockIdx.x & 7) + 8 * (g / T);  // members share blockIdx % 8: one XCD (speed only)
    const int nteams = gridDim.x / T;
    const int64_t mb = (int64_t)team * M / nteams, me = (int64_t)(team + 1) * M / nteams;
    const int n = (int)(me - mb);  // the team's columns
    const int64_t r0 = (int64_t)member * TR;
    const int nrows = (int)(N - r0 < TR ? N - r0 : TR);  // >= 1 (op_plan)
    constexpr bool QFULL = tm_qfull(K, S, COMM);
    const int QS = (int)tm_qstride(K, S, COMM, TR < N ? TR : N);  // q stride
    double* q_lds = lds;                                  // K x QS
    double* s_part = lds + K * QS;                        // [2][CW][K] wave partials of a column's dot
    double* s_tot = s_part + 2 * CW * K;                  // [2][K] team totals (hand-off)
    const int jb = 128 * wave + 2 * lane;                 // row of this lane in step s: RS*s + jb
    const int nbytes = ((nrows + 1) & ~1) * 8;            // the tile of a column (+ the zero pad row for odd N)

    if (COMM && wave == CW) {
        // ---------------- the hand-off wave ----------------
        // Per step: polls the granules of the column finished P steps later
        // together with that column's scalars (msig, p_k, z_k), sums the T
        // member partials of the column finished now, forms its d (the
        // lmmse_mult epilogue, stored by the member that owns the column,
        // which also adds <d,p>) and hands c_k = msig*d_k to the streaming
        // waves through LDS; after the barrier it publishes this member's
        // dot of the step's column.  Its polls and publishes are inline asm
        // the compiler does not track: exactly three per step (the scalars,
        // the 16-byte poll, the 16-byte publish, to a dummy slot when there
        // is nothing to publish), so the poll of step m - P is waited for
        // with vmcnt(3P) while the younger ones stay in flight (the d stores
        // and the compiler's own loads only add younger operations: the wait
        // stays sufficient).  Every poll register passes through such a wait
        // before it is read or reused (the compiler sees the wait as its writer).
        const int nq = K * T;
        unsigned long long* xg = a.xg + mb * nq * 2;  // the team's first column
        unsigned long long* dummy = a.xg + M * kOpMaxK * T * 2 + (int64_t)blockIdx.x * 2 * K;
        const int ql = lane < nq ? lane : 0;  // lanes past nq re-read lane 0's granules (no divergence)
        const unsigned tag = a.tag;
        // per-lane source of a column's scalars: lane 0 msig, 1.. p_k, 1+K.. z_k
        const double* scp = msig;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (lane == 1 + k) scp = a.p.p[k];
            if (lane == 1 + K + k && a.fuse) scp = a.z.p[k];
        }
        scp += mb;
        double bk[K], dpacc[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            bk[k] = a.fuse ? a.beta[k] : 0.0;
            dpacc[k] = 0.0;
        }
        v4u pl[RING];
        v2u ps[RING];
        bool dead = false;
        unsigned nslow = 0, nspin = 0;
        if (n > 0) {
            // Are all members on this CU's XCD?  Then the granules go to the
            // shared L2 (plain stores; the polls read L2), a round trip that
            // does not queue behind the HBM stream; otherwise write-through
            // (sc1).  Each member posts {XCC id, tag} write-through, then reads all T.
            bool l2 = false;
            {
                unsigned long long* hdr = a.xg + M * kOpMaxK * T * 2 + (int64_t)gridDim.x * 2 * K + (int64_t)team * T;
                unsigned xcc;
                asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
                xcc &= 0xf;
                if (lane == 0)
                    __hip_atomic_store(hdr + member, ((unsigned long long)tag << 32) | xcc, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                unsigned long long h = 0;
                for (unsigned spins = 0;; ++spins) {
                    h = lane < T ? __hip_atomic_load(hdr + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                 : ((unsigned long long)tag << 32) | xcc;
                    if (__all((unsigned)(h >> 32) == tag)) break;
                    if (spins >= kTmMaxSpins) {
                        dead = true;
                        if (lane == 0) __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
                l2 = !dead && __all((unsigned)h == xcc);
                if (a.dbg & 32) l2 = false;
            }
            // the streaming waves' step numbering (m from -F, column c in slot
            // (c + F) % RING, whole rounds of RING steps, a barrier in every step)
            for (int base = -F; base < n + L; base += RING) {
#pragma unroll
                for (int i = 0; i < RING; ++i) {
                    const int m = base + i;  // columns relative to mb (32-bit: scalar compares)
                    // the column polled now (finished P steps later), the column finished now
                    const int ci = m - L + P, cf = m - L;
                    const int cic = ci < 0 ? 0 : ci < n ? ci : n - 1;
                    tm_load8(ps[(i + RING - L + P) % RING], scp + cic);
                    tm_poll(pl[(i + RING - L + P) % RING], xg + ((int64_t)cic * nq + ql) * 2);
                    v4u& g = pl[(i + RING - L) % RING];
                    v2u& sc = ps[(i + RING - L) % RING];
                    if (!(a.dbg & 1)) tm_wait2<3 * P>(g, sc);  // step m - P's poll; 3P younger operations in flight
                    if (cf >= 0 && cf < n) {
                        for (unsigned spins = 0;; ++spins) {
                            const bool ok = g.y == tag && g.w == tag;  // {lo, tag} {hi, tag}
                            if (__all(ok) || dead || (a.dbg & 1)) break;
                            if (a.dbg & 64) {
                                nslow += spins == 0;
                                nspin++;
                            }
                            if (spins >= kTmMaxSpins) {  // a member never published: give up this launch (err)
                                dead = true;
                                if (lane == 0) __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                                break;
                            }
                            __builtin_amdgcn_s_sleep(2);
                            tm_poll(g, xg + ((int64_t)cf * nq + ql) * 2);
                            tm_wait<0>(g);
                        }
                        double v = lane < nq ? __builtin_bit_cast(double, ((unsigned long long)g.z << 32) | g.x) : 0.0;
                        for (int o = T >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);  // fixed order per k group
                        // d of column cf (src/vamp.cpp:656-659, data::ATx's scaling src/data.cpp:327-330)
                        const double scv = __builtin_bit_cast(double, ((unsigned long long)sc.y << 32) | sc.x);
                        const double sg = readlane_d(scv, 0);
                        const bool own = (cf % T) == member;
                        const int64_t mg = mb + cf;  // the shard's column index
#pragma unroll
                        for (int k = 0; k < K; ++k) {
                            double t = sg * readlane_d(v, k * T);  // sigma_inv * dpa
                            t *= a.scale;                          // ATx[mloc] *= 1/sqrt(N)
                            double p = readlane_d(scv, 1 + k);
                            if (a.fuse) p = readlane_d(scv, 1 + K + k) + bk[k] * p;  // p = z + beta p
                            double val = t * a.tau;  // res[i] *= tau
                            val += a.gam2 * p;       // res[i] += gam2 * v[i]
                            if (own) {
                                if (lane == 0) {
                                    if (a.sraw.p[0]) a.sraw.p[k][mg] = t;
                                    a.d.p[k][mg] = val;
                                }
                                dpacc[k] += val * p;
                            }
                            if (lane == 0) s_tot[(cf & 1) * K + k] = sg * val;  // c_k: Ax's (x - mave)*(msig*d)
                        }
                    }
                    __syncthreads();
                    if (lane < K && !(a.dbg & 2)) {  // this member's dot of column m: the streaming waves' partials in order
                        const bool real = m >= 0 && m < n;
                        double v = 0.0;
                        if (real) {
#pragma unroll
                            for (int w = 0; w < CW; ++w) v += s_part[((m & 1) * CW + w) * K + lane];
                        }
                        const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
                        const v4u gr = {(unsigned)u, tag, (unsigned)(u >> 32), tag};
                        unsigned long long* dst = real ? xg + ((int64_t)m * nq + lane * T + member) * 2 : dummy + 2 * lane;
                        if (l2)
                            tm_publish_l2(dst, gr);
                        else
                            tm_publish(dst, gr);
                    }
                }
            }
#pragma unroll
            for (int s = 0; s < RING; ++s) tm_wait2<0>(pl[s], ps[s]);  // nothing of ours lands after the loop
            if ((a.dbg & 64) && lane == 0) {  // timing experiments: slow-path counts into the flag block
                __hip_atomic_fetch_add(a.err + 1, nslow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_fetch_add(a.err + 2, nspin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_fetch_add(a.err + 3, (unsigned)n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        // <d_k, p_k> over the columns this member owns, in order; drained
        // before the barrier after which wave 0 takes the ticket
        if (lane == 0) {
#pragma unroll
            for (int k = 0; k < K; ++k) red_put(a.ro, (int64_t)blockIdx.x * K + k, dpacc[k]);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        return;
    }

    // ---------------- the streaming waves ----------------
    // q = A r/diag [+ beta*q_old] over the tile (each lane only reads its own rows)
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int jl = RS * s + jb;
        if (jl >= QS) continue;  // (never with QFULL)
#pragma unroll
        for (int k = 0; k < K; ++k) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                double q = 0.0;
                if (jl + h < nrows) {
                    const int64_t j = r0 + jl + h;
                    q = a.ar.p[k][j] / a.diag;
                    if (a.fuse) q = q + a.beta[k] * a.qo.p[k][j];
                }
                q_lds[k * QS + jl + h] = q;
            }
        }
    }
    double bk[K];
#pragma unroll
    for (int k = 0; k < K; ++k) bk[k] = a.fuse ? a.beta[k] : 0.0;
    // per-lane source of the column's scalars: lane 0 mave, 1 msig, 2.. p_k, 2+K.. z_k
    const double* pkp = mave;
    if (lane == 1) pkp = msig;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        if (lane == 2 + k) pkp = a.p.p[k];
        if (lane == 2 + K + k && a.fuse) pkp = a.z.p[k];
    }
    pkp += mb;  // column m (relative) is pkp[m]
    bool valid[S];
#pragma unroll
    for (int s = 0; s < S; ++s) valid[s] = RS * s + jb < nrows;
    v2d acc[K][S];
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
        for (int s = 0; s < S; ++s) acc[k][s] = v2d{0.0, 0.0};
    double dpacc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) dpacc[k] = 0.0;

    v2d xr[RING][S];
    double pk[RING];
    const char* xtile = reinterpret_cast<const char*>(X + mb * ld + r0);
    auto load = [&](int slot, int m) {
        pk[slot] = pkp[m];  // older than the column's X loads: it lands first
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void*)(xtile + (int64_t)m * ld * 8), (short)0, nbytes, 0x00020000);
#pragma unroll
        for (int s = 0; s < S; ++s)
            xr[slot][s] = __builtin_bit_cast(v2d, __builtin_amdgcn_raw_buffer_load_b128(rs, (RS * s + jb) * 8, 0, 2));
    };
    // this wave's partial dots of the column in `slot` -> s_part[par]
    // this wave's partial dots of the column in `slot` -> s_part[par]; the
    // slot is centred in place (x - mave), the form finish() uses
    auto dot = [&](int slot, int par) {
        const double mu = readlane_d(pk[slot], 0);
        double v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = 0.0;
#pragma unroll
        for (int s = 0; s < S; ++s) {
            // rows past the tile load 0; with QFULL their q is 0, else mave is masked
            const double me_ = QFULL || valid[s] ? mu : 0.0;
            const double dx = xr[slot][s].x - me_, dy = xr[slot][s].y - me_;
            xr[slot][s] = v2d{dx, dy};
            const int jq = QFULL || RS * s + jb < QS ? RS * s + jb : QS - 2;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const v2d q = *reinterpret_cast<const v2d*>(q_lds + k * QS + jq);
#if TM_FMA
                v[k] = __builtin_fma(dx, q.x, v[k]);
                v[k] = __builtin_fma(dy, q.y, v[k]);
#else
                v[k] += dx * q.x;
                v[k] += dy * q.y;
#endif
            }
        }
        if (K == 2) {
            // reduce-scatter: the xor-32 exchange leaves k = 0 in lanes 0-31 and
            // k = 1 in lanes 32-63 (one exchange instead of two), then 5 steps
            const bool hi = lane >= 32;
            const double send = hi ? v[0] : v[K - 1];
            double keep = hi ? v[K - 1] : v[0];
            keep += __shfl_xor(send, 32, 64);
#pragma unroll
            for (int o = 16; o > 0; o >>= 1) {
                if (a.dbg & 4) break;
                keep += __shfl_xor(keep, o, 64);
            }
            if ((lane & 31) == 0) s_part[(par * CW + wave) * K + (lane >> 5)] = keep;
        } else {
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                if (a.dbg & 4) break;
                v[0] += __shfl_xor(v[0], o, 64);
            }
            if (lane == 0) s_part[(par * CW + wave) * K] = v[0];
        }
    };
    // d of column m from its total dot, and acc += (x - mave) * msig * d
    // tot: the column's total dots, or (COMM) the c_k the hand-off wave formed
    auto finish = [&](int slot, int m, const double (&tot)[K]) {
        double cc[K];
        if constexpr (COMM) {
#pragma unroll
            for (int k = 0; k < K; ++k) cc[k] = tot[k];
        } else {
        const double sg = readlane_d(pk[slot], 1);
        const bool own = (m % T) == member;
        const int64_t mg = mb + m;  // the shard's column index
#pragma unroll
        for (int k = 0; k < K; ++k) {
            double t = sg * tot[k];  // sigma_inv * dpa
            t *= a.scale;            // ATx[mloc] *= 1/sqrt(N)
            double p = readlane_d(pk[slot], 2 + k);
            if (a.fuse) p = readlane_d(pk[slot], 2 + K + k) + bk[k] * p;  // p = z + beta p
            double val = t * a.tau;  // res[i] *= tau
            val += a.gam2 * p;       // res[i] += gam2 * v[i]
            if (own) {
                if (threadIdx.x == 0) {
                    if (a.sraw.p[0]) a.sraw.p[k][mg] = t;
                    a.d.p[k][mg] = val;
                }
                dpacc[k] += val * p;
            }
            cc[k] = sg * val;  // Ax: (x - mave) * (msig * x_i)
        }
        }
#pragma unroll
        for (int s = 0; s < S; ++s) {
            if (a.dbg & 8) break;
            const double dx = xr[slot][s].x, dy = xr[slot][s].y;  // centred by dot()
#pragma unroll
            for (int k = 0; k < K; ++k) {
#if TM_FMA
                acc[k][s].x = __builtin_fma(dx, cc[k], acc[k][s].x);
                acc[k][s].y = __builtin_fma(dy, cc[k], acc[k][s].y);
#else
                acc[k][s].x += dx * cc[k];
                acc[k][s].y += dy * cc[k];
#endif
            }
        }
    };
    if (n > 0) {
        // Steps m = -F .. in whole rounds of RING; the first F only issue
        // loads.  Starting the loop there (instead of a prologue) leaves no
        // load pending on entry, and straight-line rounds (guards, no
        // break/continue) keep the compiler's waits at the loop head those of
        // the steady state.  Column c lives in ring slot (c + F) % RING.
        for (int base = -F; base < n + L; base += RING) {
#pragma unroll
            for (int i = 0; i < RING; ++i) {
                const int m = base + i;  // columns relative to mb (32-bit: scalar compares)
                // every step issues one column (clamped to [0, n): fixed vmcnt counts)
                load((i + F) % RING, m + F < n ? m + F : n - 1);
                if (m >= 0 && m < n) dot(i, m & 1);
                __syncthreads();
                const int cf = m - L;
                if (cf >= 0 && cf < n) {
                    double tot[K];
                    if (COMM) {
#pragma unroll
                        for (int k = 0; k < K; ++k) tot[k] = s_tot[(cf & 1) * K + k];
                    } else {
#pragma unroll
                        for (int k = 0; k < K; ++k) {
                            double t = 0.0;
#pragma unroll
                            for (int w = 0; w < CW; ++w) t += s_part[((m & 1) * CW + w) * K + k];
                            tot[k] = t;
                        }
                    }
                    finish((i + RING - L) % RING, cf, tot);
                }
            }
        }
    }
    // this member's rows of its team's partial A d
    double* dst = a.part + (int64_t)team * kMaxRhs * ld + r0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int jl = RS * s + jb;
        if (jl >= nrows) continue;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            dst[(int64_t)k * ld + jl] = acc[k][s].x;
            if (jl + 1 < nrows) dst[(int64_t)k * ld + jl + 1] = acc[k][s].y;
        }
    }
    // <d_k, p_k>: each workgroup's sums over the columns it owns, in order
    // (COMM: the hand-off wave's, put before the barrier below); the last
    // workgroup adds them in block order
    if constexpr (COMM) {
        __syncthreads();
    } else if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) red_put(a.ro, (int64_t)blockIdx.x * K + k, dpacc[k]);
    }
    if (wave == 0) ticket_sum_blocks<K>(a.ro);
}

// ---------------------------------------------------------------------------
// host side: plans, instantiations, launch
// ---------------------------------------------------------------------------
static int tm_S(int64_t rows, bool comm) {
    const int rs = tm_rows_per_step(comm);
    return (int)((rows + rs - 1) / rs);
}

// the team plan for team size T and configuration cfg (false: not possible)
bool team_plan(int64_t N, int64_t M, int cus, int T, int cfg, OpPlan* out) {
    if (cfg < 0 || cfg >= kTmNCfg || N < 1) return false;
    const TmCfg& c = kTmCfg[cfg];
    if ((T == 1) == c.comm) return false;
    if (T < 1 || T > kTmMaxT || (T & (T - 1))) return false;
    const int grid = (cus / (8 * T)) * 8 * T;
    if (grid < T) return false;
    int64_t TR = N;
    if (T > 1) {
        TR = ((N + T - 1) / T + 127) / 128 * 128;
        if ((int64_t)(T - 1) * TR >= N) return false;  // every member holds rows
    }
    const int S = tm_S(TR, c.comm);
    if (S > c.maxS) return false;
    const int64_t QS = tm_qfull(kOpMaxK, S, c.comm) ? (int64_t)S * tm_rows_per_step(c.comm) : (std::min<int64_t>(TR, N) + 1) & ~1;
    const int64_t lds = (QS * kOpMaxK + 2 * 8 * kOpMaxK + 2 * kOpMaxK) * 8;
    if (lds > 160 * 1024) return false;
    OpPlan p{};
    p.grid = grid;
    p.S = S;
    p.T = T;
    p.TR = (int)TR;
    p.cfg = cfg;
    p.nslots = grid / T;
    (void)M;
    *out = p;
    return true;
}

template <int K, int S, int C>
static void launch_tm(const Shard& s, const OpPlan& pl, const OpArgs& a, hipStream_t st, const Timing& tm,
                      const int* gate) {
    constexpr TmCfg c = kTmCfg[C];
    constexpr int CW = c.comm ? 7 : 8;
    auto kern = atax_team_kernel<K, S, c.F, c.L, c.P, c.comm>;
    const int64_t QS = tm_qstride(K, S, c.comm, std::min<int64_t>(pl.TR, s.N));
    const size_t lds = (size_t)(K * QS + 2 * CW * K + 2 * K) * sizeof(double);
    static std::once_flag once;  // more than 64 KiB of dynamic LDS must be allowed explicitly
    std::call_once(once, [&] {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
    });
    hipExtLaunchKernelGGL(kern, dim3(pl.grid), dim3(kTmThreads), lds, st, tm.start, tm.stop, 0, s.X, s.ld, s.N, s.M,
                          s.mave, s.msig, a, pl.T, pl.TR, gate);
}

template <int K, int C, int S>
static bool launch_tm_if(const Shard& s, const OpPlan& pl, const OpArgs& a, hipStream_t st, const Timing& tm,
                         const int* gate) {
    if constexpr (S <= kTmCfg[C].maxS) {
        launch_tm<K, S, C>(s, pl, a, st, tm, gate);
        return true;
    }
    return false;
}

template <int K, int C>
static bool launch_tm_s(int S, const Shard& s, const OpPlan& pl, const OpArgs& a, hipStream_t st,
                        const Timing& tm, const int* gate) {
    switch (S) {
        case 1: return launch_tm_if<K, C, 1>(s, pl, a, st, tm, gate);
        case 2: return launch_tm_if<K, C, 2>(s, pl, a, st, tm, gate);
        case 3: return launch_tm_if<K, C, 3>(s, pl, a, st, tm, gate);
        case 4: return launch_tm_if<K, C, 4>(s, pl, a, st, tm, gate);
        case 5: return launch_tm_if<K, C, 5>(s, pl, a, st, tm, gate);
        case 6: return launch_tm_if<K, C, 6>(s, pl, a, st, tm, gate);
        case 7: return launch_tm_if<K, C, 7>(s, pl, a, st, tm, gate);
        case 8: return launch_tm_if<K, C, 8>(s, pl, a, st, tm, gate);
        case 9: return launch_tm_if<K, C, 9>(s, pl, a, st, tm, gate);
        case 10: return launch_tm_if<K, C, 10>(s, pl, a, st, tm, gate);
        default: return false;
    }
}

template <int K>
static bool launch_tm_c(const Shard& s, const OpPlan& pl, const OpArgs& a, hipStream_t st, const Timing& tm,
                        const int* gate) {
    switch (pl.cfg) {
        case 0: return launch_tm_s<K, 0>(pl.S, s, pl, a, st, tm, gate);
        case 1: return launch_tm_s<K, 1>(pl.S, s, pl, a, st, tm, gate);
        case 2: return launch_tm_s<K, 2>(pl.S, s, pl, a, st, tm, gate);
        case 3: return launch_tm_s<K, 3>(pl.S, s, pl, a, st, tm, gate);
        case 4: return launch_tm_s<K, 4>(pl.S, s, pl, a, st, tm, gate);
        case 5: return launch_tm_s<K, 5>(pl.S, s, pl, a, st, tm, gate);
        case 6: return launch_tm_s<K, 6>(pl.S, s, pl, a, st, tm, gate);
        case 7: return launch_tm_s<K, 7>(pl.S, s, pl, a, st, tm, gate);
        case 8: return launch_tm_s<K, 8>(pl.S, s, pl, a, st, tm, gate);
        default: return false;
    }
}

hipError_t atax_team(const Shard& s, const OpPlan& pl, int K, const OpArgs& a, hipStream_t st, const Timing& tm,
                     const int* gate) {
    if (pl.T < 1 || pl.grid < pl.T || pl.grid % pl.T) return hipErrorInvalidValue;
    if (pl.T > 1 && (!a.xg || !a.err || a.tag == 0)) return hipErrorInvalidValue;
    if (s.M <= 0) return hipSuccess;
    bool ok = false;
    switch (K) {
        case 1: ok = launch_tm_c<1>(s, pl, a, st, tm, gate); break;
        case 2: ok = launch_tm_c<2>(s, pl, a, st, tm, gate); break;
        default: break;
    }
    if (!ok) return hipErrorInvalidValue;
    return hipGetLastError();
}

std::string team_kernel_name(int K, const OpPlan& pl) {
    const TmCfg& c = kTmCfg[pl.cfg];
    char b[128];
    std::snprintf(b, sizeof b, "atax_team_kernel<%d, %d, %d, %d, %d, %s>", K, pl.S, c.F, c.L, c.P,
                  c.comm ? "true" : "false");
    return b;
}

}  // namespace vk
