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
#define TM_FMA 1  // fused multiply-adds in the dot and the A d accumulation (DESIGN.md §3;
                  // A/B in one gpurun call: C3 shard K=2 7207 vs 7332 us, C2 587 vs 600 us)
#endif
#ifndef TM_SAFE
#define TM_SAFE 0
#endif
#ifndef TM_TS
#define TM_TS 0  // 1: record each workgroup's start/end time (s_memrealtime, 100 MHz) into OpArgs.ts
#endif
#ifndef TM_TEAMS_BY_XCD
#define TM_TEAMS_BY_XCD 1
#endif
#ifndef TM_DBG
#define TM_DBG 0  // 1: honour OpArgs.dbg (timing experiments); 0: its branches compile out
#endif
#ifndef TM_ABL
#define TM_ABL 0  // ablation builds (tools/op_ablation.py): these VAMPOMI_OP_DBG bits baked in as constants, so the
                  // rest of the schedule is the production kernel's (a TM_DBG build's run-time branches are not)
#endif
static constexpr int kTmThreads = 512;        // 8 waves, 2 per SIMD: <= 256 VGPRs per lane
static constexpr int kTmLdsHead = 4;          // dynamic LDS words before q: the folded decision (team_plan's +4)
static constexpr int kTmMaxT = 32;            // members per team (one XCD under round-robin dealing)
static constexpr unsigned kTmMaxSpins = 1u << 21;  // ~2 s of polling, then the launch gives up (err)

// configurations: F columns prefetched, L steps of lag, P polls in flight,
// hand-off (T > 1), the most loads per lane per column that fit 256 VGPRs at
// K = 2 without spilling (gfx950, ROCm 7.2 compiler), E doubles per lane per
// load (2: 16-byte loads, rows in steps of 128 per wave), and whether team t
// takes columns t, t + nteams, ... (interleaved) or a contiguous range.  Only
// the configurations op_plan / team_plain_plan select are kept, plus 6 (the
// interleaving ablation).  (Round 3 numbered them differently: 7 -> 2, 8 -> 3,
// 9 -> 4, 12 -> 5; the dynamic-chunk configurations 17/18 and the other
// swept entries were removed in round 4, profiles/r03_op_experiments.txt.)
struct TmCfg {
    int F, L, P;
    bool comm;
    int maxS;
    int E;
    bool ilv;  // team t takes columns t, t + nteams, ... (else a contiguous range)
};
static constexpr TmCfg kTmCfg[] = {
    {1, 0, 0, false, 10, 2, false},  // 0: T = 1, one column prefetched
    {2, 0, 0, false, 8, 2, false},   // 1: T = 1, two
    {4, 5, 2, true, 4, 2, true},     // 2: teams, four loads per lane (large N)
    {3, 5, 2, true, 4, 2, true},     // 3: the head-start kernel's short ring
    {2, 4, 2, true, 5, 2, true},     // 4: one more load per lane, fewer columns in flight
    {2, 3, 2, true, 6, 2, true},     // 5: six loads per lane (T = 2 at N = 10,000: C2)
    {4, 5, 2, true, 4, 2, false},    // 6: 2 with contiguous column ranges (interleaving ablation)
};
static constexpr int kTmNCfg = sizeof(kTmCfg) / sizeof(kTmCfg[0]);

__host__ __device__ constexpr int tm_rows_per_step(bool comm, int E) { return 64 * E * (comm ? 7 : 8); }

// q in LDS: every lane row of the S steps (zeros past the tile, so those
// rows need no mask) when that fits beside the partials, else the tile only
// (rows past it masked)
__host__ __device__ constexpr bool tm_qfull(int K, int S, bool comm, int E) {
    return (K * S * tm_rows_per_step(comm, E) + 4 * 8 * K) * 8 <= 160 * 1024;
}
__host__ __device__ constexpr int64_t tm_qstride(int K, int S, bool comm, int E, int64_t tile_rows) {
    return tm_qfull(K, S, comm, E) ? (int64_t)S * tm_rows_per_step(comm, E) : (tile_rows + 1) & ~(int64_t)1;
}

// The dynamic LDS of a team-kernel launch, in doubles from its start: the
// head (the folded CG decision: beta_k, then go), q (K x qs), the streaming
// waves' partials of a column's dot ([2][CW][K]) and the hand-off totals
// ([2][K]).  The ONE description of it: the kernel's pointers, team_plan's
// feasibility check and launch_tm's launch size all come from here.
struct TmLds {
    int64_t qs;    // q stride (doubles per system)
    int64_t q;     // offsets
    int64_t part;
    int64_t tot;
    int64_t words;  // total
};
static_assert(kOpMaxK + 1 <= kTmLdsHead, "the head holds beta_k (k < kOpMaxK) and the go word after them");
__host__ __device__ constexpr TmLds tm_lds(int K, int S, bool comm, int E, int64_t tile_rows) {
    const int64_t qs = tm_qstride(K, S, comm, E, tile_rows);
    const int cw = comm ? 7 : 8;  // streaming waves
    const int64_t q = kTmLdsHead, part = q + (int64_t)K * qs, tot = part + 2 * (int64_t)cw * K;
    return TmLds{qs, q, part, tot, tot + 2 * (int64_t)K};
}
static constexpr int64_t kTmLdsMaxBytes = 160 * 1024;  // gfx950: LDS per workgroup

__device__ __forceinline__ double readlane_d(double v, int l) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// Cross-lane sums without the LDS (DPP moves and the gfx950 permlane swaps are
// VALU; ds_bpermute shuffles queue behind the streaming waves' LDS reads).
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)u, CTRL, 0xf, 0xf, false);
    const unsigned hi = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)(u >> 32), CTRL, 0xf, 0xf, false);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ double pack_d(unsigned lo, unsigned hi) {
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
// v_permlane16_swap(x, x): the first result holds rows {0,0,2,2}, the second
// {1,1,3,3} of x (16-lane rows), so their sum is row 0+1 / 2+3 in every lane
__device__ __forceinline__ double swap16_sum(double v) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const auto l = __builtin_amdgcn_permlane16_swap((unsigned)u, (unsigned)u, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap((unsigned)(u >> 32), (unsigned)(u >> 32), false, false);
    return pack_d(l[0], h[0]) + pack_d(l[1], h[1]);
}
// v_permlane32_swap(a, b): the first result is {a lanes 0-31, b lanes 0-31},
// the second {a lanes 32-63, b lanes 32-63}
__device__ __forceinline__ void swap32(double a, double b, double& r0, double& r1) {
    const unsigned long long ua = __builtin_bit_cast(unsigned long long, a), ub = __builtin_bit_cast(unsigned long long, b);
    const auto l = __builtin_amdgcn_permlane32_swap((unsigned)ua, (unsigned)ub, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap((unsigned)(ua >> 32), (unsigned)(ub >> 32), false, false);
    r0 = pack_d(l[0], h[0]);
    r1 = pack_d(l[1], h[1]);
}
// the sum over each aligned group of G lanes, in every lane of the group; the
// pairs are added in the same order in every lane (a + b = b + a), so every
// lane of a group holds the same bits
template <int G>
__device__ __forceinline__ double group_sum(double v) {
    if constexpr (G >= 2) v = v + dpp_d<0xb1>(v);   // quad_perm [1,0,3,2]: lane ^ 1
    if constexpr (G >= 4) v = v + dpp_d<0x4e>(v);   // quad_perm [2,3,0,1]: lane ^ 2
    if constexpr (G >= 8) v = v + dpp_d<0x141>(v);  // row_half_mirror: the other quad of 8
    if constexpr (G >= 16) v = v + dpp_d<0x140>(v); // row_mirror: the other half of the row
    if constexpr (G >= 32) v = swap16_sum(v);       // the other row of 32
    if constexpr (G >= 64) {
        double a, b;
        swap32(v, v, a, b);
        v = a + b;
    }
    return v;
}

// x[0] + x[s] + ... + x[(N-1)s] as a fixed pairwise tree (halves, the odd
// one last): log2 N dependent adds instead of N - 1
template <int N>
__device__ __forceinline__ double tree_sum(const double* x, int s) {
    if constexpr (N == 1) {
        return x[0];
    } else {
        constexpr int H = N / 2;
        return tree_sum<H>(x, s) + tree_sum<N - H>(x + H * s, s);
    }
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

// KP > 0 (the head-start launch, pcg.cpp): KP plain right-hand sides ride
// along, z_kp = A x_kp = sum_i (X_i - mave_i) * (msig_i * x_kp[i]) (data::Ax,
// src/data.cpp:340-373): their coefficients are known when the column is
// loaded, so the streaming waves accumulate them in the column's own step
// (no hand-off), into partial slots K .. K+KP-1 of the team.
// TM_SAFE diagnostic builds: an address outside [lo, hi) is reported in
// a.err (bit `code`, shifted past the timeout flag) and replaced by lo
template <class Tp>
__device__ __forceinline__ Tp* tm_chk(Tp* p, const void* lo, const void* hi, unsigned code, unsigned* err) {
#if TM_SAFE
    if ((const char*)p < (const char*)lo || (const char*)p >= (const char*)hi) {
        __hip_atomic_fetch_or(err, 1u | (code << 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return (Tp*)lo;
    }
#endif
    return p;
}

template <int K, int S, int F, int L, int P, bool COMM, int E, bool FMA, int KP>
__device__ __forceinline__ void atax_team_body(const double* __restrict__ X, int64_t ld, int64_t N, int64_t M,
                                               const double* __restrict__ mave, const double* __restrict__ msig,
                                               const OpArgs& a, int T, int TR, int ilv,
                                               const int* __restrict__ gate) {
    // the dynamic LDS: kTmLdsHead words for the folded decision (beta_k, go),
    // then q and the partials.  (No static __shared__ in this kernel: its
    // launches set the dynamic limit to the whole 160 KiB.)
    extern __shared__ __attribute__((aligned(16))) double lds[];
    // beta_k of the fused direction updates: from the previous step's decision
    // when this launch forms it (OpArgs.fold), else a.beta
    double* s_beta = lds;
    if (a.fold.on) {
        double& s_go = lds[kOpMaxK];
        if (threadIdx.x == 0) {
            CgState cs = *a.fold.src;
            double r[3 * kMaxRhs];
#pragma unroll
            for (int q = 0; q < 3 * kMaxRhs; ++q) r[q] = q < 3 * cs.K ? a.fold.red[q] : 0.0;
            const bool ran = cg_decide_into(cs, r, a.fold.it, a.fold.mask);
            if (blockIdx.x == 0) {
                *a.fold.dst = cs;
                cg_publish(cs, ran, a.fold.it, a.fold.mirror, a.fold.flag, a.fold.seq, a.fold.pack);
            }
            s_go = cs.any ? 1.0 : 0.0;
#pragma unroll
            for (int k = 0; k < kOpMaxK; ++k) s_beta[k] = cs.beta[k];
        }
        __syncthreads();
        if (s_go == 0.0) return;
    } else if (gate && !*gate) {
        return;
    }
    const double* beta = a.fold.on ? s_beta : a.beta;
    static_assert(K + KP <= kMaxRhs, "partial slots per team");
#if TM_TS
    const unsigned long long ts0 = __builtin_amdgcn_s_memrealtime();
#endif
    // timing experiments (VAMPOMI_OP_DBG): with a hand-off only in a TM_DBG
    // build (the branches cost the hand-off wave's chain 2 % at the C3 shard);
    // T = 1 keeps them: at 252-256 VGPRs its schedule without them waits more
    // (C2 K = 2: 613 against 591 us, profiles/r02f_op_experiments.txt)
    const int dbg = TM_ABL ? TM_ABL : (TM_DBG || !COMM) ? a.dbg : 0;
    constexpr int CW = COMM ? 7 : 8;  // streaming waves
    constexpr int RS = tm_rows_per_step(COMM, E);
    static_assert(E == 1 || E == 2, "doubles per lane per load");
    constexpr int RING = F + L + 1;
    static_assert(COMM || L == 0, "without a hand-off the column is finished in its own step");
    static_assert(!COMM || (P >= 1 && P <= L), "polls in flight");
    static_assert(!COMM || P < RING, "a poll's slot is consumed before it is reissued");
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int g = blockIdx.x >> 3;
    const int member = g % T;
    const int nteams = gridDim.x / T;  // a multiple of 8 (team_plan)
    // members share blockIdx % 8: one XCD (speed only).  Teams t of one XCD are
    // numbered consecutively (t = local + nteams/8 * xcd), so under interleaved
    // columns the markers of one 64-byte line of d (8 neighbours) belong to teams
    // of one XCD and their 8-byte owner stores merge in that XCD's L2
    // (TM_TEAMS_BY_XCD 0: xcd + 8 * local, the round-2 numbering)
#if TM_TEAMS_BY_XCD
    const int team = g / T + (nteams >> 3) * (int)(blockIdx.x & 7);
#else
    const int team = (blockIdx.x & 7) + 8 * (g / T);
#endif
    // the team's columns: mb + cs*m, m < n (a contiguous range, or every nteams-th)
    const int64_t cs = ilv ? nteams : 1;
    const int64_t mb = ilv ? team : (int64_t)team * M / nteams;
    const int n = (int)(ilv ? (M - team + nteams - 1) / nteams : (int64_t)(team + 1) * M / nteams - mb);
    const int64_t nmax = (M + nteams - 1) / nteams;  // granule rows per team
    const int64_t gwords = (M + gridDim.x) * kOpMaxK * T * 2;  // the granule block (OpArgs.xg)
    const int64_t r0 = (int64_t)member * TR;
    const int nrows = (int)(N - r0 < TR ? N - r0 : TR);  // >= 1 (op_plan)
    constexpr bool QFULL = tm_qfull(K, S, COMM, E);
    const TmLds lay = tm_lds(K, S, COMM, E, TR < N ? TR : N);  // (launch_tm sized the launch from the same)
    const int QS = (int)lay.qs;                           // q stride
    double* q_lds = lds + lay.q;                          // K x QS
    double* s_part = lds + lay.part;                      // [2][CW][K] wave partials of a column's dot
    double* s_tot = lds + lay.tot;                        // [2][K] team totals (hand-off)
    const int jb = 64 * E * wave + E * lane;              // row of this lane in step s: RS*s + jb
    // the tile of a column (E = 2: + the zero pad row for odd N)
    const int nbytes = (E == 2 ? (nrows + 1) & ~1 : nrows) * 8;

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
        // granules of step m at xg + m * nq2: the team's m-th column
        unsigned long long* xg = a.xg + (int64_t)team * nmax * nq * 2;
        unsigned long long* dummy = a.xg + gwords + (int64_t)blockIdx.x * 2 * K;
        // lane 32k + j reads member j's granule of system k (j < T), so one
        // fixed 32-lane butterfly sums every team size (the zeros of lanes
        // j >= T leave the sums' bits unchanged); other lanes re-read granule 0
        const bool qv = (lane >> 5) < K && (lane & 31) < T;
        const int ql2 = qv ? 2 * ((lane >> 5) * T + (lane & 31)) : 0;
        const int nq2 = 2 * nq;          // words per column of the granule block
        const int csi = (int)cs;         // column stride (1 or nteams)
        const unsigned tag = a.tag;
        // per-lane source of a column's scalars: lane 0 msig, 1.. p_k, 1+K.. z_k
        const double* scp = msig;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (lane == 1 + k) scp = a.p.p[k];
            if (lane == 1 + K + k && ((a.fuse >> k) & 1)) scp = a.z.p[k];
        }
        scp += mb;  // column m (relative) is scp[m * cs]
        double bk[K], dpacc[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            bk[k] = ((a.fuse >> k) & 1) ? beta[k] : 0.0;
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
                unsigned long long* hdr = a.xg + gwords + (int64_t)gridDim.x * 2 * kOpMaxK + (int64_t)team * T;
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
                if (dbg & 32) l2 = false;
            }
            // the streaming waves' step numbering (m from -F, column c in slot
            // (c + F) % RING, whole rounds of RING steps, a barrier in every step)
            for (int base = -F; base - L < n; base += RING) {
#pragma unroll
                for (int i = 0; i < RING; ++i) {
                    const int m = base + i;  // columns relative to mb (32-bit: scalar compares)
                    if (dbg & 4096) {  // timing experiment: no hand-off work at all, only the step's barrier
                        __syncthreads();
                        continue;
                    }
                    // the column polled now (finished P steps later), the column finished now
                    const int ci = m - L + P, cf = m - L;
                    const int cic = ci < 0 ? 0 : ci < n ? ci : n - 1;
                    tm_load8(ps[(i + RING - L + P) % RING], scp + cic * csi);  // offsets < 2^31: 32-bit math
                    tm_poll(pl[(i + RING - L + P) % RING], xg + (cic * nq2 + ql2));
                    v4u& g = pl[(i + RING - L) % RING];
                    v2u& sc = ps[(i + RING - L) % RING];
                    if (!(dbg & 1)) tm_wait2<3 * P>(g, sc);  // step m - P's poll; 3P younger operations in flight
                    if (cf >= 0 && cf < n) {
                        // every granule of column cf carries this launch's tag {lo, tag} {hi, tag}
                        if (!(__all(g.y == tag && g.w == tag) || dead || (dbg & 1))) {
#pragma unroll 1
                            for (unsigned spins = 0;; ++spins) {  // slow path: poll again until it does
                                if (dbg & 64) {
                                    nslow += spins == 0;
                                    nspin++;
                                }
                                if (spins >= kTmMaxSpins) {  // a member never published: give up this launch (err)
                                    dead = true;
                                    if (lane == 0) __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                                    break;
                                }
                                __builtin_amdgcn_s_sleep(2);
                                tm_poll(g, tm_chk(xg + ((int64_t)cf * nq2 + ql2), a.xg, a.xg + gwords, 64, a.err));
                                tm_wait<0>(g);
                                if (__all(g.y == tag && g.w == tag)) break;
                            }
                        }
                        double v = qv ? __builtin_bit_cast(double, ((unsigned long long)g.z << 32) | g.x) : 0.0;
                        if (dbg & 512) {  // timing experiment: the ds_bpermute butterfly
                            for (int o = T >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
                        } else if (!(dbg & 256)) {
                            v = group_sum<32>(v);  // the T members of system k in lanes 32k.., fixed order
                        }
                        // d of column cf (src/vamp.cpp:656-659, data::ATx's scaling src/data.cpp:327-330)
                        const double scv = __builtin_bit_cast(double, ((unsigned long long)sc.y << 32) | sc.x);
                        const double sg = readlane_d(scv, 0);
                        const bool own = (cf & (T - 1)) == member;  // T: a power of two
                        const int64_t mg = mb + cf * csi;  // the shard's column index
                        // both systems' chains first (independent: interleaved), then the
                        // LDS hand-over, then the owner's stores and <d,p>
                        double tsc[K], dval[K], pdir[K];
#pragma unroll
                        for (int k = 0; k < K; ++k) {
                            double t = sg * readlane_d(v, 32 * k);  // sigma_inv * dpa
                            t *= a.scale;                           // ATx[mloc] *= 1/sqrt(N)
                            double p = readlane_d(scv, 1 + k);
                            if ((a.fuse >> k) & 1) p = readlane_d(scv, 1 + K + k) + bk[k] * p;  // p = z + beta p
                            double val = t * a.tau;  // res[i] *= tau
                            val += a.gam2 * p;       // res[i] += gam2 * v[i]
                            tsc[k] = t;
                            dval[k] = val;
                            pdir[k] = p;
                        }
#pragma unroll
                        for (int k = 0; k < K; ++k)  // c_k: Ax's (x - mave)*(msig*d)
                            if (lane == 0) s_tot[(cf & 1) * K + k] = (dbg & 128) ? 0.0 : sg * dval[k];
                        if (own) {
#pragma unroll
                            for (int k = 0; k < K; ++k) {
                                if (lane == 0 && !(dbg & 1024)) {  // (timing experiment 1024: no d stores)
                                    if (a.sraw.p[0]) a.sraw.p[k][mg] = tsc[k];
                                    *tm_chk(a.d.p[k] + mg, a.d.p[k], a.d.p[k] + M, 128, a.err) = dval[k];
                                }
                                dpacc[k] += dval[k] * pdir[k];
                            }
                        }
                    }
                    __syncthreads();
                    if (lane < K && !(dbg & 2)) {  // this member's dot of column m: the streaming waves' partials in order
                        const bool real = m >= 0 && m < n;
                        double v = 0.0;
                        if (real) v = tree_sum<CW>(s_part + (m & 1) * CW * K + lane, K);  // fixed pairwise order
                        const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
                        const v4u gr = {(unsigned)u, tag, (unsigned)(u >> 32), tag};
                        unsigned long long* dst =
                            tm_chk(real ? xg + ((int64_t)m * nq2 + (lane * T + member) * 2) : dummy + 2 * lane, a.xg,
                                   a.xg + gwords + (int64_t)gridDim.x * 2 * kOpMaxK, 512, a.err);
                        if (l2)
                            tm_publish_l2(dst, gr);
                        else
                            tm_publish(dst, gr);
                    }
                }
            }
#pragma unroll
            for (int s = 0; s < RING; ++s) tm_wait2<0>(pl[s], ps[s]);  // nothing of ours lands after the loop
            if ((dbg & 64) && lane == 0) {  // timing experiments: slow-path counts into the flag block
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
            for (int h = 0; h < E; ++h) {
                double q = 0.0;
                if (jl + h < nrows) {
                    const int64_t j = r0 + jl + h;
                    q = a.ar.p[k][j] / a.diag;
                    if ((a.fuse >> k) & 1) q = q + beta[k] * a.qo.p[k][j];
                }
                q_lds[k * QS + jl + h] = q;
            }
        }
    }
    double bk[K];
#pragma unroll
    for (int k = 0; k < K; ++k) bk[k] = ((a.fuse >> k) & 1) ? beta[k] : 0.0;
    // per-lane source of the column's scalars: lane 0 mave, 1 msig, 2.. p_k,
    // 2+K.. z_k, 2+2K.. the plain right-hand sides x_kp
    const double* pkp = mave;
    if (lane == 1) pkp = msig;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        if (lane == 2 + k) pkp = a.p.p[k];
        if (lane == 2 + K + k && ((a.fuse >> k) & 1)) pkp = a.z.p[k];
    }
#pragma unroll
    for (int k = 0; k < KP; ++k)
        if (lane == 2 + 2 * K + k) pkp = a.px.p[k];
    pkp += mb;  // column m (relative) is pkp[m * cs]
    bool valid[S];
#pragma unroll
    for (int s = 0; s < S; ++s) valid[s] = RS * s + jb < nrows;
    double acc[K][S][E];
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
        for (int s = 0; s < S; ++s)
#pragma unroll
            for (int e = 0; e < E; ++e) acc[k][s][e] = 0.0;
    double dpacc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) dpacc[k] = 0.0;
    constexpr int KPA = KP > 0 ? KP : 1;
    double accp[KPA][S][E];  // the plain right-hand sides' rows of A x
#pragma unroll
    for (int k = 0; k < KPA; ++k)
#pragma unroll
        for (int s = 0; s < S; ++s)
#pragma unroll
            for (int e = 0; e < E; ++e) accp[k][s][e] = 0.0;

    double xr[RING][S][E];
    double pk[RING];
    const char* xtile = reinterpret_cast<const char*>(X + mb * ld + r0);
    auto load = [&](int slot, int m) {
        const int64_t c = m * cs;  // offset from mb
        pk[slot] = *tm_chk(pkp + c, pkp - mb, pkp - mb + M, 1024, a.err);  // older than the column's X loads: it lands first
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void*)(xtile + c * ld * 8), (short)0, nbytes, 0x00020000);
#pragma unroll
        for (int s = 0; s < S; ++s) {
            if constexpr (E == 2) {
                const v2d x = __builtin_bit_cast(v2d, __builtin_amdgcn_raw_buffer_load_b128(rs, (RS * s + jb) * 8, 0, 2));
                xr[slot][s][0] = x.x;
                xr[slot][s][E - 1] = x.y;
            } else {
                xr[slot][s][0] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, (RS * s + jb) * 8, 0, 2));
            }
        }
    };
    // this wave's partial dots of the column in `slot` -> s_part[par]; the
    // slot is centred in place (x - mave), the form finish() uses
    auto dot = [&](int slot, int par) {
        const double mu = readlane_d(pk[slot], 0);
        double cp[KPA];  // msig_i * x_kp[i]: Ax's (x - mave) * (msig * x_i)
        if constexpr (KP > 0) {
            const double sgp = readlane_d(pk[slot], 1);
#pragma unroll
            for (int k = 0; k < KP; ++k) cp[k] = sgp * readlane_d(pk[slot], 2 + 2 * K + k);
        }
        double v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = 0.0;
#pragma unroll
        for (int s = 0; s < S; ++s) {
            // rows past the tile load 0; with QFULL their q is 0, else mave is masked
            const double me_ = QFULL || valid[s] ? mu : 0.0;
            const int jq = QFULL || RS * s + jb < QS ? RS * s + jb : QS - E;
            double dx[E], q[K][E];
#pragma unroll
            for (int e = 0; e < E; ++e) {
                dx[e] = xr[slot][s][e] - me_;
                xr[slot][s][e] = dx[e];
            }
            if constexpr (KP > 0) {
#pragma unroll
                for (int k = 0; k < KP; ++k)
#pragma unroll
                    for (int e = 0; e < E; ++e) {
                        if constexpr (FMA)
                            accp[k][s][e] = __builtin_fma(dx[e], cp[k], accp[k][s][e]);
                        else
                            accp[k][s][e] += dx[e] * cp[k];
                    }
            }
#pragma unroll
            for (int k = 0; k < K; ++k) {
                if ((TM_DBG || TM_ABL) && (dbg & 2048)) {  // timing experiment: no LDS q reads
                    q[k][0] = 0.5;
                    q[k][E - 1] = 0.25;
                } else if constexpr (E == 2) {
                    const v2d qq = *reinterpret_cast<const v2d*>(q_lds + k * QS + jq);
                    q[k][0] = qq.x;
                    q[k][E - 1] = qq.y;
                } else {
                    q[k][0] = q_lds[k * QS + jq];
                }
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    if constexpr (FMA)
                        v[k] = __builtin_fma(dx[e], q[k][e], v[k]);
                    else
                        v[k] += dx[e] * q[k][e];
                }
            }
        }
        if (K == 2) {
            // reduce-scatter: one permlane32 swap leaves k = 0 in lanes 0-31
            // and k = 1 in lanes 32-63, then sums within each half
            double r0, r1;
            swap32(v[0], v[K - 1], r0, r1);
            double keep = r0 + r1;
            if (dbg & 512) {  // timing experiment: the ds_bpermute butterfly
                for (int o = 16; o > 0; o >>= 1) keep += __shfl_xor(keep, o, 64);
            } else if (!(dbg & 4)) {
                keep = group_sum<32>(keep);
            }
            if ((lane & 31) == 0) s_part[(par * CW + wave) * K + (lane >> 5)] = keep;
        } else {
            if (!(dbg & 4)) v[0] = group_sum<64>(v[0]);
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
            const int64_t mg = mb + m * cs;  // the shard's column index
#pragma unroll
            for (int k = 0; k < K; ++k) {
                double t = sg * tot[k];  // sigma_inv * dpa
                t *= a.scale;            // ATx[mloc] *= 1/sqrt(N)
                double p = readlane_d(pk[slot], 2 + k);
                if ((a.fuse >> k) & 1) p = readlane_d(pk[slot], 2 + K + k) + bk[k] * p;  // p = z + beta p
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
            if (dbg & 8) break;
#pragma unroll
            for (int k = 0; k < K; ++k)
#pragma unroll
                for (int e = 0; e < E; ++e) {  // xr is centred by dot()
                    if constexpr (FMA)
                        acc[k][s][e] = __builtin_fma(xr[slot][s][e], cc[k], acc[k][s][e]);
                    else
                        acc[k][s][e] += xr[slot][s][e] * cc[k];
                }
        }
    };
    if (n > 0) {
        // Steps m = -F .. in whole rounds of RING; the first F only issue
        // loads.  Starting the loop there (instead of a prologue) leaves no
        // load pending on entry, and straight-line rounds (guards, no
        // break/continue) keep the compiler's waits at the loop head those of
        // the steady state.  Column c lives in ring slot (c + F) % RING.
        for (int base = -F;; base += RING) {
            if (base - L >= n) break;
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
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int e = 0; e < E; ++e)
                if (jl + e < nrows) dst[(int64_t)k * ld + jl + e] = acc[k][s][e];
        if constexpr (KP > 0) {
#pragma unroll
            for (int k = 0; k < KP; ++k)
#pragma unroll
                for (int e = 0; e < E; ++e)
                    if (jl + e < nrows) dst[(int64_t)(K + k) * ld + jl + e] = accp[k][s][e];
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
#if TM_TS
    if (a.ts && threadIdx.x == 0) {
        unsigned xcc, hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        unsigned long long* t = a.ts + 4 * (int64_t)blockIdx.x;
        t[0] = ts0;
        t[1] = __builtin_amdgcn_s_memrealtime();
        t[2] = xcc;
        t[3] = hw;
    }
#endif
}

template <int K, int S, int F, int L, int P, bool COMM, int E, bool FMA>
__global__ __launch_bounds__(kTmThreads) void atax_team_kernel(const double* __restrict__ X, int64_t ld, int64_t N,
                                                               int64_t M, const double* __restrict__ mave,
                                                               const double* __restrict__ msig, OpArgs a, int T,
                                                               int TR, int ilv, const int* __restrict__ gate) {
    atax_team_body<K, S, F, L, P, COMM, E, FMA, 0>(X, ld, N, M, mave, msig, a, T, TR, ilv, gate);
}

// the head-start launch: one operator system (the Onsager solve's first CG
// step) and kTmPlain plain right-hand sides (pcg.cpp)
static constexpr int kTmPlain = kOpPlain;
template <int S, int F, int L, int P, bool COMM, int E, bool FMA>
__global__ __launch_bounds__(kTmThreads) void atax_team_plain_kernel(const double* __restrict__ X, int64_t ld,
                                                                     int64_t N, int64_t M,
                                                                     const double* __restrict__ mave,
                                                                     const double* __restrict__ msig, OpArgs a, int T,
                                                                     int TR, int ilv, const int* __restrict__ gate) {
    atax_team_body<1, S, F, L, P, COMM, E, FMA, kTmPlain>(X, ld, N, M, mave, msig, a, T, TR, ilv, gate);
}

// ---------------------------------------------------------------------------
// A.x alone (data::Ax, src/data.cpp:340-373) at large N: the team layout
// without the operator system.  A plain product needs no column dot, so the T
// members of a team need no hand-off: each holds rows [r*TR, (r+1)*TR) of the
// team's interleaved columns (team t: t, t + nteams, ...) and accumulates
//   acc_k[j] += (X_ij - mave_i) * (msig_i * x_k[i])
// in registers over all of them (8 streaming waves, 16-byte buffer loads,
// F columns prefetched), then writes its rows of the team's slot
// part[team][k][ld]; ax_reduce sums the nteams slots in order.  The tile
// plans (ax_partial_kernel) cut each column into 4 KB pieces over 512-row
// tiles; here a member reads TR rows (25 KB at N = 100,000) of every column
// it takes.  FU: x_k = z_k + beta_k * p_k (AxFuse), as ax_partial_kernel forms it.
#ifndef AX_TEAM_SYNC
#define AX_TEAM_SYNC 1  // 0: experiment builds without the per-column barrier (3.7 % slower, r05s)
#endif
#ifndef AX_TEAM_F
#define AX_TEAM_F 4
#endif
static constexpr int kAxTmF = AX_TEAM_F;  // columns prefetched (AX_TEAM_F: experiment builds)
static constexpr int kAxTmMaxS = 4;    // loads per lane per column (1024-row steps)
template <int S, int KP, bool FU>
__global__ __launch_bounds__(kTmThreads) void ax_team_kernel(const double* __restrict__ X, int64_t ld, int64_t N,
                                                             int64_t M, const double* __restrict__ mave,
                                                             const double* __restrict__ msig, CPtrs xs,
                                                             double* __restrict__ part, AxFuse fu, int T, int TR) {
    if (fu.gate && !*fu.gate) return;
    constexpr int E = 2, F = kAxTmF, RING = F + 1;
    constexpr int RS = tm_rows_per_step(false, E);  // 1024
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int g = blockIdx.x >> 3;
    const int member = g % T;
    const int nteams = gridDim.x / T;  // a multiple of 8 (ax_team_plan)
    const int team = g / T + (nteams >> 3) * (int)(blockIdx.x & 7);  // teams of one XCD numbered together
    const int n = team < M ? (int)((M - team + nteams - 1) / nteams) : 0;
    const int64_t r0 = (int64_t)member * TR;
    const int nrows = (int)(N - r0 < TR ? N - r0 : TR);  // >= 1 (ax_team_plan)
    const int nbytes = ((nrows + 1) & ~1) * 8;            // the tile (+ the zero pad row for odd N)
    const int jb = 64 * E * wave + E * lane;              // row of this lane in step s: RS*s + jb
    double bk[KP];
#pragma unroll
    for (int k = 0; k < KP; ++k) bk[k] = FU ? fu.beta[k] : 0.0;
    // per-lane source of a column's scalars: lane 0 mave, 1 msig, 2.. x_k, 2+KP.. z_k
    const double* pkp = mave;
    if (lane == 1) pkp = msig;
#pragma unroll
    for (int k = 0; k < KP; ++k) {
        if (lane == 2 + k) pkp = xs.p[k];
        if (FU && lane == 2 + KP + k) pkp = fu.z.p[k];
    }
    pkp += team;  // column m of the team is pkp[m * nteams]
    double acc[KP][S][E];
#pragma unroll
    for (int k = 0; k < KP; ++k)
#pragma unroll
        for (int s = 0; s < S; ++s)
#pragma unroll
            for (int e = 0; e < E; ++e) acc[k][s][e] = 0.0;
    double xr[RING][S][E];
    double pk[RING];
    const char* xtile = reinterpret_cast<const char*>(X + (int64_t)team * ld + r0);
    auto load = [&](int slot, int m) {
        const int64_t c = (int64_t)m * nteams;
        pk[slot] = pkp[c];  // older than the column's X loads: it lands first
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void*)(xtile + c * ld * 8), (short)0, nbytes, 0x00020000);
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const v2d x = __builtin_bit_cast(v2d, __builtin_amdgcn_raw_buffer_load_b128(rs, (RS * s + jb) * 8, 0, 2));
            xr[slot][s][0] = x.x;
            xr[slot][s][1] = x.y;
        }
    };
    if (n > 0) {
        // steps m = -F .. in whole rounds of RING (the first F only load);
        // column c lives in ring slot (c + F) % RING, every step issues one
        // load (clamped to the last column: fixed vmcnt counts)
        for (int base = -F; base < n; base += RING) {
#pragma unroll
            for (int i = 0; i < RING; ++i) {
                const int m = base + i;
                load((i + F) % RING, m + F < n ? m + F : n - 1);
                if (m >= 0 && m < n) {
                    const double mu = readlane_d(pk[i], 0);
                    const double sg = readlane_d(pk[i], 1);
                    double cp[KP];  // msig_i * x_k[i]
#pragma unroll
                    for (int k = 0; k < KP; ++k) {
                        double xk = readlane_d(pk[i], 2 + k);
                        if (FU) xk = readlane_d(pk[i], 2 + KP + k) + bk[k] * xk;
                        cp[k] = sg * xk;
                    }
#pragma unroll
                    for (int s = 0; s < S; ++s)
#pragma unroll
                        for (int e = 0; e < E; ++e) {
                            const double dx = xr[i][s][e] - mu;  // rows past the tile: never stored
#pragma unroll
                            for (int k = 0; k < KP; ++k) {
                                if constexpr (TM_FMA)
                                    acc[k][s][e] = __builtin_fma(dx, cp[k], acc[k][s][e]);
                                else
                                    acc[k][s][e] += dx * cp[k];
                            }
                        }
                }
                // the waves stay on one column together (as the operator's
                // per-column barrier keeps them): one column's rows are read
                // as one stream, not 8 drifting ones
                if (AX_TEAM_SYNC) __syncthreads();
            }
        }
    }
    // this member's rows of the team's slot (zeros for a team without columns)
    double* dst = part + (int64_t)team * KP * ld + r0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int jl = RS * s + jb;
        if (jl >= nrows) continue;
#pragma unroll
        for (int k = 0; k < KP; ++k)
#pragma unroll
            for (int e = 0; e < E; ++e)
                if (jl + e < nrows) dst[(int64_t)k * ld + jl + e] = acc[k][s][e];
    }
}

// ---------------------------------------------------------------------------
// host side: plans, instantiations, launch
// ---------------------------------------------------------------------------
static int tm_S(int64_t rows, bool comm, int E) {
    const int rs = tm_rows_per_step(comm, E);
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
        // E = 2: tiles on 128-row (1 KiB) boundaries; E = 1: tiles of ceil(N/T) rows
        TR = c.E == 2 ? ((N + T - 1) / T + 127) / 128 * 128 : (N + T - 1) / T;
        if ((int64_t)(T - 1) * TR >= N) return false;  // every member holds rows
    }
    const int S = tm_S(TR, c.comm, c.E);
    if (S > c.maxS) return false;
    // every system count the plan may launch with (the head-start kernel is K = 1)
    for (int K = 1; K <= kOpMaxK; ++K)
        if (tm_lds(K, S, c.comm, c.E, std::min<int64_t>(TR, N)).words * 8 > kTmLdsMaxBytes) return false;
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

bool team_lds_layout(const OpPlan& pl, int64_t N, int K, int64_t out[6]) {
    if (pl.T < 1 || pl.cfg < 0 || pl.cfg >= kTmNCfg || K < 1 || K > kOpMaxK || N < 1) return false;
    const TmCfg& c = kTmCfg[pl.cfg];
    const TmLds l = tm_lds(K, pl.S, c.comm, c.E, std::min<int64_t>(pl.TR, N));
    out[0] = kTmLdsHead;
    out[1] = l.q;
    out[2] = l.qs;
    out[3] = l.part;
    out[4] = l.tot;
    out[5] = l.words;
    return true;
}

// occ != null: no launch, *occ = the workgroups of this instantiation one CU
// holds at once (hipOccupancyMaxActiveBlocksPerMultiprocessor).  PL: the
// head-start kernel (K = 1 operator system + kTmPlain plain right-hand sides)
template <int K, int S, int C, bool PL>
static hipError_t launch_tm(const Shard& s, const OpPlan& pl, const OpArgs& a, hipStream_t st, const Timing& tm,
                            const int* gate, int* occ) {
    constexpr TmCfg c = kTmCfg[C];
    static_assert(!PL || K == 1, "the head-start kernel has one operator system");
    void (*kern)(const double*, int64_t, int64_t, int64_t, const double*, const double*, OpArgs, int, int, int,
                 const int*);
    if constexpr (PL)
        kern = atax_team_plain_kernel<S, c.F, c.L, c.P, c.comm, c.E, (bool)TM_FMA>;
    else
        kern = atax_team_kernel<K, S, c.F, c.L, c.P, c.comm, c.E, (bool)TM_FMA>;
    const size_t lds = (size_t)tm_lds(K, S, c.comm, c.E, std::min<int64_t>(pl.TR, s.N)).words * sizeof(double);
    if (lds > (size_t)kTmLdsMaxBytes) return hipErrorInvalidValue;  // (team_plan refuses such plans)
    // more than 64 KiB of dynamic LDS must be allowed explicitly, once per
    // instantiation and device
    static std::atomic<unsigned long long> allowed{0};  // bit d: done on device d
    if (const hipError_t e = lds_allow(reinterpret_cast<const void*>(kern), allowed, (int)kTmLdsMaxBytes))
        return e;
    if (occ) {
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, kern, kTmThreads, lds) != hipSuccess) *occ = 0;
        return hipSuccess;
    }
    hipExtLaunchKernelGGL(kern, dim3(pl.grid), dim3(kTmThreads), lds, st, tm.start, tm.stop, 0, s.X, s.ld, s.N, s.M,
                          s.mave, s.msig, a, pl.T, pl.TR, c.ilv ? 1 : 0, gate);
    return hipSuccess;
}

// the most loads per lane per column the head-start kernel is instantiated
// for, per configuration (0: none): its 3 plain accumulators cost 12*S
// registers beside the ring (register counts and spills checked with
// tools/regcheck.py)
static constexpr int tm_plain_maxS(int cfg) {
    return cfg == 0 ? 8 : cfg == 2 ? 3 : cfg == 3 ? 4 : cfg == 4 ? 5 : 0;
}

// hipErrorInvalidValue: no such instantiation (or an LDS size over the limit)
template <int K, int C, int S, bool PL>
static hipError_t launch_tm_if(const Shard& s, const OpPlan& pl, const OpArgs& a, hipStream_t st, const Timing& tm,
                               const int* gate, int* occ) {
    if constexpr (S <= (PL ? tm_plain_maxS(C) : kTmCfg[C].maxS))
        return launch_tm<K, S, C, PL>(s, pl, a, st, tm, gate, occ);
    return hipErrorInvalidValue;
}

template <int K, int C, bool PL>
static hipError_t launch_tm_s(int S, const Shard& s, const OpPlan& pl, const OpArgs& a, hipStream_t st,
                        const Timing& tm, const int* gate, int* occ) {
    switch (S) {
        case 1: return launch_tm_if<K, C, 1, PL>(s, pl, a, st, tm, gate, occ);
        case 2: return launch_tm_if<K, C, 2, PL>(s, pl, a, st, tm, gate, occ);
        case 3: return launch_tm_if<K, C, 3, PL>(s, pl, a, st, tm, gate, occ);
        case 4: return launch_tm_if<K, C, 4, PL>(s, pl, a, st, tm, gate, occ);
        case 5: return launch_tm_if<K, C, 5, PL>(s, pl, a, st, tm, gate, occ);
        case 6: return launch_tm_if<K, C, 6, PL>(s, pl, a, st, tm, gate, occ);
        case 7: return launch_tm_if<K, C, 7, PL>(s, pl, a, st, tm, gate, occ);
        case 8: return launch_tm_if<K, C, 8, PL>(s, pl, a, st, tm, gate, occ);
        case 9: return launch_tm_if<K, C, 9, PL>(s, pl, a, st, tm, gate, occ);
        case 10: return launch_tm_if<K, C, 10, PL>(s, pl, a, st, tm, gate, occ);
        default: return hipErrorInvalidValue;
    }
}

template <int K, bool PL = false>
static hipError_t launch_tm_c(const Shard& s, const OpPlan& pl, const OpArgs& a, hipStream_t st, const Timing& tm,
                        const int* gate, int* occ = nullptr) {
    if constexpr (PL) {
        switch (pl.cfg) {
            case 0: return launch_tm_s<1, 0, true>(pl.S, s, pl, a, st, tm, gate, occ);
            case 2: return launch_tm_s<1, 2, true>(pl.S, s, pl, a, st, tm, gate, occ);
            case 3: return launch_tm_s<1, 3, true>(pl.S, s, pl, a, st, tm, gate, occ);
            case 4: return launch_tm_s<1, 4, true>(pl.S, s, pl, a, st, tm, gate, occ);
            default: return hipErrorInvalidValue;
        }
    }
    switch (pl.cfg) {
        case 0: return launch_tm_s<K, 0, false>(pl.S, s, pl, a, st, tm, gate, occ);
        case 1: return launch_tm_s<K, 1, false>(pl.S, s, pl, a, st, tm, gate, occ);
        case 2: return launch_tm_s<K, 2, false>(pl.S, s, pl, a, st, tm, gate, occ);
        case 3: return launch_tm_s<K, 3, false>(pl.S, s, pl, a, st, tm, gate, occ);
        case 4: return launch_tm_s<K, 4, false>(pl.S, s, pl, a, st, tm, gate, occ);
        case 5: return launch_tm_s<K, 5, false>(pl.S, s, pl, a, st, tm, gate, occ);
        case 6: return launch_tm_s<K, 6, false>(pl.S, s, pl, a, st, tm, gate, occ);
        default: return hipErrorInvalidValue;
    }
}

hipError_t atax_team(const Shard& s, const OpPlan& pl, int K, const OpArgs& a, hipStream_t st, const Timing& tm,
                     const int* gate) {
    if (pl.T < 1 || pl.grid < pl.T || pl.grid % pl.T) return hipErrorInvalidValue;
    if (pl.T > 1 && (!a.xg || !a.err || a.tag == 0)) return hipErrorInvalidValue;
    if (s.M <= 0) return hipSuccess;
    hipError_t e = hipErrorInvalidValue;
    switch (K) {
        case 1: e = launch_tm_c<1>(s, pl, a, st, tm, gate); break;
        case 2: e = launch_tm_c<2>(s, pl, a, st, tm, gate); break;
        default: break;
    }
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

hipError_t atax_team_plain(const Shard& s, const OpPlan& pl, const OpArgs& a, hipStream_t st, const Timing& tm,
                           const int* gate) {
    if (pl.T < 1 || pl.grid < pl.T || pl.grid % pl.T) return hipErrorInvalidValue;
    if (pl.T > 1 && (!a.xg || !a.err || a.tag == 0)) return hipErrorInvalidValue;
    for (int k = 0; k < kTmPlain; ++k)
        if (!a.px.p[k]) return hipErrorInvalidValue;
    if (s.M <= 0) return hipSuccess;
    if (const hipError_t e = launch_tm_c<1, true>(s, pl, a, st, tm, gate)) return e;
    return hipGetLastError();
}

bool ax_team_plan(int64_t N, int64_t M, int cus, AxPlan* out) {
    if (N < 1 || cus < 8) return false;
    constexpr int RS = tm_rows_per_step(false, 2);
    for (int T = 1; T <= kTmMaxT; T *= 2) {
        if (cus / (8 * T) < 1) break;
        const int grid = (cus / (8 * T)) * 8 * T;
        const int64_t TR = T == 1 ? N : ((N + T - 1) / T + 127) / 128 * 128;
        if ((int64_t)(T - 1) * TR >= N) continue;  // every member holds rows
        const int S = (int)((TR + RS - 1) / RS);
        if (S > kAxTmMaxS) continue;
        AxPlan p{};
        p.variant = kAxTeam;
        p.T = T;
        p.TR = (int)TR;
        p.S = S;
        p.groups = grid;
        p.nslots = grid / T;
        p.rows = N;  // one tile: every row sums the nslots team slots
        p.tiles = 1;
        p.total = M;
        p.sa = p.nslots;
        p.sb = 1;
        *out = p;
        return true;
    }
    return false;
}

template <int S, int K, bool FU>
static void launch_axt(const Shard& s, const AxPlan& pl, CPtrs x, double* part, hipStream_t st, const Timing& tm,
                       const AxFuse& fu) {
    hipExtLaunchKernelGGL((ax_team_kernel<S, K, FU>), dim3(pl.groups), dim3(kTmThreads), 0, st, tm.start, tm.stop, 0,
                          s.X, s.ld, s.N, s.M, s.mave, s.msig, x, part, fu, pl.T, pl.TR);
}

template <int S>
static bool launch_axt_k(int K, bool fused, const Shard& s, const AxPlan& pl, CPtrs x, double* part,
                         hipStream_t st, const Timing& tm, const AxFuse& fu) {
    switch (K * 2 + (fused ? 1 : 0)) {
        case 2: launch_axt<S, 1, false>(s, pl, x, part, st, tm, fu); return true;
        case 3: launch_axt<S, 1, true>(s, pl, x, part, st, tm, fu); return true;
        case 4: launch_axt<S, 2, false>(s, pl, x, part, st, tm, fu); return true;
        case 5: launch_axt<S, 2, true>(s, pl, x, part, st, tm, fu); return true;
        case 6: launch_axt<S, 3, false>(s, pl, x, part, st, tm, fu); return true;
        case 7: launch_axt<S, 3, true>(s, pl, x, part, st, tm, fu); return true;
        case 8: launch_axt<S, 4, false>(s, pl, x, part, st, tm, fu); return true;
        case 9: launch_axt<S, 4, true>(s, pl, x, part, st, tm, fu); return true;
        default: return false;
    }
}

hipError_t ax_team(const Shard& s, const AxPlan& pl, int K, CPtrs x, double* part, hipStream_t st, const Timing& tm,
                   const AxFuse& fu) {
    // the plan must be this shard's: every member holds rows, S loads cover them
    if (pl.T < 1 || pl.groups % (8 * pl.T) || pl.nslots != pl.groups / pl.T || pl.S < 1 || pl.S > kAxTmMaxS ||
        (int64_t)(pl.T - 1) * pl.TR >= s.N || (int64_t)pl.T * pl.TR < s.N ||
        (int64_t)pl.S * tm_rows_per_step(false, 2) < std::min<int64_t>(pl.TR, s.N) || pl.rows < s.N)
        return hipErrorInvalidValue;
    if (s.M <= 0) return hipSuccess;
    const bool fused = fu.z.p[0] != nullptr;
    if (fused && !fu.beta) return hipErrorInvalidValue;
    bool ok = false;
    switch (pl.S) {
        case 1: ok = launch_axt_k<1>(K, fused, s, pl, x, part, st, tm, fu); break;
        case 2: ok = launch_axt_k<2>(K, fused, s, pl, x, part, st, tm, fu); break;
        case 3: ok = launch_axt_k<3>(K, fused, s, pl, x, part, st, tm, fu); break;
        case 4: ok = launch_axt_k<4>(K, fused, s, pl, x, part, st, tm, fu); break;
        default: break;
    }
    if (!ok) return hipErrorInvalidValue;
    return hipGetLastError();
}

std::string ax_kernel_name(int K, bool fused, const AxPlan& pl) {
    if (pl.T <= 0) return kernel_name(0, K, fused ? 1 : 0, pl.variant);
    char b[96];
    std::snprintf(b, sizeof b, "ax_team_kernel<%d, %d, %s>", pl.S, K, fused ? "true" : "false");
    return b;
}

bool team_plain_plan(int64_t N, int64_t M, int cus, const OpPlan& main, OpPlan* out) {
    // the main plan's team size when the head-start kernel fits its rows, else
    // larger teams (fewer rows per member); configurations with short rings
    const int cfgs1[] = {0};
    const int cfgsT[] = {2, 3, 4};
    for (int T = std::max(main.T, 1); T <= kTmMaxT; T *= 2) {
        const int* cf = T == 1 ? cfgs1 : cfgsT;
        const int ncf = T == 1 ? 1 : 3;
        for (int i = 0; i < ncf; ++i) {
            OpPlan p{};
            if (!team_plan(N, M, cus, T, cf[i], &p) || p.S > tm_plain_maxS(cf[i])) continue;
            *out = p;
            return true;
        }
    }
    return false;
}

int team_occupancy(const OpPlan& pl, int K) {
    int occ = 0;
    const Shard s{nullptr, 0, (int64_t)pl.TR * pl.T, 1, nullptr, nullptr};  // the LDS size needs TR and N only
    const OpArgs a{};
    hipError_t e = hipErrorInvalidValue;
    switch (K) {
        case 1: e = launch_tm_c<1>(s, pl, a, nullptr, Timing{}, nullptr, &occ); break;
        case 2: e = launch_tm_c<2>(s, pl, a, nullptr, Timing{}, nullptr, &occ); break;
        case 1 + kTmPlain: e = launch_tm_c<1, true>(s, pl, a, nullptr, Timing{}, nullptr, &occ); break;
        default: break;
    }
    return e == hipSuccess ? occ : 0;
}

std::string team_kernel_name(int K, const OpPlan& pl) {
    const TmCfg& c = kTmCfg[pl.cfg];
    char b[128];
    if (K == 1 + kTmPlain)  // the head-start kernel
        std::snprintf(b, sizeof b, "atax_team_plain_kernel<%d, %d, %d, %d, %s, %d>", pl.S, c.F, c.L, c.P,
                      c.comm ? "true" : "false", c.E);
    else
        std::snprintf(b, sizeof b, "atax_team_kernel<%d, %d, %d, %d, %d, %s, %d>", K, pl.S, c.F, c.L, c.P,
                      c.comm ? "true" : "false", c.E);
    return b;
}

}  // namespace vk
