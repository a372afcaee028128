// kernels.hip -- gfx950 (CDNA4) kernels of the SBPMF Gibbs sweep.
//
// Hot path = the per-row univariate conditional of the reference
// (users: src/libfm/gibbs_sbpmf_final.cpp:453-491, items :495-535): for every
// row, K coordinates drawn sequentially in k, each from
//     P = sum_n v_nk^2,  Q = sum_n v_nk (E_n + v_nk u_k),
//     var = 1/(sigma_k + tau P),  mean = var (tau Q + sigma_k mu_k),
//     u_k <- mean + s z  (s = var under the reference quirk, sqrt(var) else),
//     E_n += v_nk (old - new).
// Rows are independent given the partner table, so a half-sweep is one
// launch per degree bin:
//   * k_gblock<T, V, NW, RPW>  rows of <= 8 ratings f64 / 16 f32 (<= 256 / 512 with tune bits
//     8-11): 1 wave per row (RPW rows per block) or NW waves per row; per
//     16-wide k-block the row's partner slices sit in VGPRs, G_B = S^T S by MFMA,
//     the 16 draws as the exact recurrence over G_B, e -= S_B D_B
//     by DPP;
//   * k_gres<T, NW, SIDE>  longer rows and the chunks of split rows: one
//     persistent launch, the same per-block steps with a task's slices held in
//     the VGPRs of NW waves and split rows' (G_B, c_B) partials summed across
//     workgroups in chunk order;
//   * k_grow<T, NW, SIDE>  rows of 9..256 ratings f64 / 17..512 f32: k_gres' code on whole
//     rows, one workgroup of one (<= 128 f64 / 256 f32 ratings) or two waves per row.
// Layout: factor tables row-major [rows][Kp] (Kp = K padded to 16), so a
// partner row is one contiguous 4K/8K-byte record; ratings in CSR (users)
// and CSC (items) order; residuals kept per orientation and gathered through
// a fixed permutation (no atomics, deterministic).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "kernels.h"
#include "rng.h"

// Diagnostic hooks: defined away here.  The diagnostic builds (Makefile CHECK=1 /
// KPROF=1) pre-include kernels_instr.h, which defines them first; the product
// build never includes it.
//   CHK(i, extent)           a global index (CHECK=1: validated, printed, redirected)
//   SBMF_GBLOCK_PHASES(on)   declares stamp(phase) in k_gblock (KPROF=1: wave 0's
//   SBMF_GRES_PHASES(nch)    cycles per phase) / in k_gres' task loop
#ifndef SBMF_KERNELS_INSTR_H_
#define CHK(i, lim) (i)
#define SBMF_GBLOCK_PHASES(on) auto stamp = [](int) {}
#define SBMF_GRES_PHASES(nch) auto stamp = [](int) {}
#endif

namespace sbmf {
namespace {

// ------------------------------------------------------------------ wave64 helpers
template <int CTRL, int ROWM>
__device__ __forceinline__ int dpp_i(int v) {
    // quad_perm (0x00-0xff), row_ror (0x121-0x12f) and the row mirrors over all rows write
    // every lane: no "old" value to materialise (saves a v_mov per DPP)
    if constexpr (ROWM == 0xf && (CTRL <= 0xff || (CTRL >= 0x121 && CTRL <= 0x12f) || CTRL == 0x140 || CTRL == 0x141))
        return __builtin_amdgcn_mov_dpp(v, CTRL, ROWM, 0xf, false);
    else
        return __builtin_amdgcn_update_dpp(0, v, CTRL, ROWM, 0xf, false);
}
template <int CTRL, int ROWM>
__device__ __forceinline__ float dpp(float v) {
    return __int_as_float(dpp_i<CTRL, ROWM>(__float_as_int(v)));
}
template <int CTRL, int ROWM>
__device__ __forceinline__ double dpp(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = dpp_i<CTRL, ROWM>((int)(b & 0xffffffffLL));
    const int hi = dpp_i<CTRL, ROWM>((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ float readlane(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ double readlane(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// Sum over the 64 lanes; result uniform.  quad_perm x2, row_shr:4, row_shr:8,
// row_bcast:15 (rows 1,3), row_bcast:31 (rows 2,3) -> total in lane 63.
template <typename T>
__device__ __forceinline__ T wave_sum(T x) {
    x += dpp<0xb1, 0xf>(x);
    x += dpp<0x4e, 0xf>(x);
    x += dpp<0x114, 0xf>(x);
    x += dpp<0x118, 0xf>(x);
    x += dpp<0x142, 0xa>(x);
    x += dpp<0x143, 0xc>(x);
    return readlane(x, 63);
}

template <typename T, int B>
struct Slice {
    T v[B];
};
// 32-byte partner slice load (two 16-byte vector loads).
__device__ __forceinline__ void load_slice(const double* p, double (&o)[4]) {
    const double2 a = reinterpret_cast<const double2*>(p)[0];
    const double2 b = reinterpret_cast<const double2*>(p)[1];
    o[0] = a.x; o[1] = a.y; o[2] = b.x; o[3] = b.y;
}
__device__ __forceinline__ void load_slice(const float* p, float (&o)[8]) {
    const float4 a = reinterpret_cast<const float4*>(p)[0];
    const float4 b = reinterpret_cast<const float4*>(p)[1];
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
    o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}

template <typename T>
__device__ __forceinline__ T tsqrt(T x);
template <typename T>
__device__ __forceinline__ T tsqrt_if(T x, int want);
template <>
__device__ __forceinline__ float tsqrt<float>(float x) { return sqrtf(x); }
template <>
__device__ __forceinline__ double tsqrt<double>(double x) { return sqrt(x); }
// sqrt(x) if `want` (a kernel argument: wave-uniform), else x -- as a real branch: the
// compiler if-converts the plain select and runs the whole f64 square-root sequence
// (about 20 dependent instructions) on the solving wave's critical path even under the
// variance-as-stdev quirk, where it is never used
template <typename T>
__device__ __forceinline__ T tsqrt_if(T x, int want) {
    if (__builtin_amdgcn_readfirstlane(want)) {
        asm volatile("" ::: "memory");
        x = tsqrt(x);
    }
    return x;
}

// One coordinate draw, shared by all row paths.
template <typename T>
__device__ __forceinline__ T draw_coord(T P, T Q, T sg, T mu, T tau, T z, int sd_is_var) {
    const T var = T(1) / (sg + tau * P);
    const T mean = var * (tau * Q + sg * mu);
    const T sd = sd_is_var ? var : tsqrt(var);
    return mean + sd * z;
}


// ------------------------------------------------------------ Gram-block rows (MFMA)
// Layout: 16 lanes per rating, 4 ratings per 64-lane vector; lane (r = l>>4,
// i = l&15) holds s = partner[j_r][16b + i] of k-block b -- one 128-byte line
// per rating per block (f64), fully coalesced.  Per block:
//   G_B = S_B^T S_B   one MFMA 16x16x4 per vector (A = B = the same register:
//                     lane l supplies S[l>>4][l&15], verified by
//                     tests/hip/mfma_layout.hip),
//   c_B = S_B^T e     one FMA per vector (e replicated over the rating's
//                     16 lanes) + a cross-row reduction,
//   16 draws          lane c holds row c of G_B (LDS transpose); for step j:
//                     new = A + Bq q, D = new - old, q_c -= G[c][j] D_j
//                     (Q_k = c_k + G_kk u_k - sum_{l<k} G_kl D_l, exact),
//   e -= S_B D_B      16-lane DPP rotate-reduce per vector.
// A row is handled by one wave (RPW rows per block) or by NW waves (one row
// per block, per-wave partials summed in LDS in wave order).
template <typename T>
struct MfmaT;
template <>
struct MfmaT<double> {
    typedef double acc_t __attribute__((ext_vector_type(4)));
    static __device__ __forceinline__ acc_t mfma(double a, acc_t c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, c, 0, 0, 0);
    }
    static __device__ __forceinline__ acc_t mfma2(double a, double b, acc_t c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    // C/D map: col = l&15, row = (l>>4) + 4j
    static __device__ __forceinline__ int row(int l, int j) { return (l >> 4) + 4 * j; }
};
template <>
struct MfmaT<float> {
    typedef float acc_t __attribute__((ext_vector_type(4)));
    static __device__ __forceinline__ acc_t mfma(float a, acc_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, c, 0, 0, 0);
    }
    static __device__ __forceinline__ acc_t mfma2(float a, float b, acc_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    // C/D map: col = l&15, row = 4*(l>>4) + j
    static __device__ __forceinline__ int row(int l, int j) { return 4 * (l >> 4) + j; }
};

// sum over the 16 lanes of each DPP row, result in every lane of the row
template <typename T>
__device__ __forceinline__ T row16_sum(T x) {
    x += dpp<0x121, 0xf>(x);  // row_ror:1
    x += dpp<0x122, 0xf>(x);  // row_ror:2
    x += dpp<0x124, 0xf>(x);  // row_ror:4
    x += dpp<0x128, 0xf>(x);  // row_ror:8
    return x;
}
// Same sum, bit-identical in all 16 lanes of the row: xor-1 and xor-2 pairs
// (quad_perm), then rotations by 8 and 4 -- every lane adds the same two
// operands at every step (in one order or the other), so no lane rounds
// differently.
template <typename T>
__device__ __forceinline__ T row16_sum_sym(T x) {
    x += dpp<0xb1, 0xf>(x);   // quad_perm [1,0,3,2]
    x += dpp<0x4e, 0xf>(x);   // quad_perm [2,3,0,1]
    x += dpp<0x128, 0xf>(x);  // row_ror:8
    x += dpp<0x124, 0xf>(x);  // row_ror:4
    return x;
}
// One level of a butterfly reduce-scatter over the 16 lanes of each DPP row:
// values s[0..M) (M/2 pairs); the lane pairs given by CTRL (an involution)
// split each pair by `key` (the lane's bit for this level): the lane keeps one
// member summed with its partner's copy of that member, so s[0..M/2) then hold
// sums over twice the lanes for this lane's half of the vectors.
template <int CTRL, int M, typename T, int N>
__device__ __forceinline__ void bfly_level(T (&s)[N], bool key) {
#pragma unroll
    for (int j = 0; j < M / 2; ++j) {
        // members past the array (N not a power of two: M rounds it up) are zero vectors
        const T lo = s[j], hi = j + M / 2 < N ? s[j + M / 2] : T(0);
        const T keep = key ? hi : lo, send = key ? lo : hi;
        s[j] = keep + dpp<CTRL, 0xf>(send);
    }
}
// Row sums of V vectors at once: s[v] (lane ci of each 16-lane row = one
// term) -> the complete sums of vectors vb .. vb + max(1, V/16) - 1 in s[0..),
// vb returned.  Four butterfly levels (row_ror:8, row_half_mirror, quad_perm
// xor 2, xor 1); a level past log2(V) adds both lanes' value (every lane that
// holds a vector ends with the same bits: the two operands of each add are
// the same in either lane, only swapped).
template <int V, typename T>
__device__ __forceinline__ int row16_scatter(T (&s)[V], int ci) {
    if constexpr (V >= 2) bfly_level<0x128, V>(s, ci & 8); else s[0] = s[0] + dpp<0x128, 0xf>(s[0]);
    if constexpr (V >= 4) bfly_level<0x141, V / 2>(s, ci & 4); else s[0] = s[0] + dpp<0x141, 0xf>(s[0]);
    if constexpr (V >= 8) bfly_level<0x4e, V / 4>(s, ci & 2); else s[0] = s[0] + dpp<0x4e, 0xf>(s[0]);
    if constexpr (V >= 16) bfly_level<0xb1, V / 8>(s, ci & 1); else s[0] = s[0] + dpp<0xb1, 0xf>(s[0]);
    return ((V >= 2 && (ci & 8)) ? V / 2 : 0) + ((V >= 4 && (ci & 4)) ? V / 4 : 0) +
           ((V >= 8 && (ci & 2)) ? V / 8 : 0) + ((V >= 16 && (ci & 1)) ? V / 16 : 0);
}
__device__ __forceinline__ float shfl_xor_t(float v, int m) { return __shfl_xor(v, m); }
__device__ __forceinline__ double shfl_xor_t(double v, int m) { return __shfl_xor(v, m); }
__device__ __forceinline__ float shfl_t(float v, int src) { return __shfl(v, src); }
__device__ __forceinline__ double shfl_t(double v, int src) { return __shfl(v, src); }

// Workgroup barrier for LDS hand-offs that keeps global loads in flight:
// __syncthreads() emits s_waitcnt vmcnt(0), which would drain the next
// block's prefetched slices (CDNA guide §5 "Pipelining across barriers").
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// s_waitcnt vmcnt(N): all but this wave's N youngest vector-memory operations are done
// (the counter holds at most 63: a larger N waits for the oldest N - 63 of them too)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0, "vmcnt range");
    if constexpr (N >= 63) asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
    else if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (N == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if constexpr (N == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if constexpr (N == 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    else if constexpr (N == 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
    else if constexpr (N == 48) asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
    else static_assert(N == 0, "add the count");
}

constexpr int GB = 16;      // k per block
constexpr int GLD = GB + 1; // padded LDS row (conflict-free row reads)

// The 16 draws of a block in "gamma form": with H[c][l] = Bq_c G[c][l] for
// l < c (0 otherwise) and gamma_c = A_c - old_c + Bq_c (c_c + P_c old_c),
// step j reads d_j = gamma_j (final: it only receives corrections from
// l < j) and applies gamma_c -= H[c][j] d_j.  After 16 steps lane c holds
// d_c = new_c - old_c.  Same arithmetic as q_c -= G[c][j] d_j followed by
// new = A + Bq q, with a 2-instruction dependency chain per step.
template <typename T>
__device__ __forceinline__ T gblock_solve(const T (&H)[GB], T gam) {
#pragma unroll
    for (int j = 0; j < GB; ++j) {
        const T dj = readlane(gam, j);
        gam -= H[j] * dj;
    }
    return gam;
}

// Same recurrence with the H row read from LDS (row `hrow`, scaled by Bq)
// step by step, for kernels without the registers to hold it.
// Lane j of each 16-lane DPP row, broadcast to the row (row_newbcast: one 64-bit DPP move
// on gfx950 where a readlane pair put the value through an SGPR pair and a wait state).
// Every row of the solving wave holds the same 16-lane system, so each row broadcasting
// its own lane j gives every lane what readlane(x, j) gave.
template <int J>
__device__ __forceinline__ double row_bcast(double v) {
    return __longlong_as_double(__builtin_amdgcn_mov_dpp(__double_as_longlong(v), 0x150 + J, 0xf, 0xf, false));
}
template <int J>
__device__ __forceinline__ float row_bcast(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x150 + J, 0xf, 0xf, false));
}
template <int J, typename T>
__device__ __forceinline__ void solve_steps(const T* __restrict__ hrow, T Bq, T& gam) {
    const T dj = row_bcast<J>(gam);
    gam -= (Bq * hrow[J]) * dj;
    if constexpr (J + 1 < GB) solve_steps<J + 1>(hrow, Bq, gam);
}

template <typename T>
__device__ __forceinline__ T gblock_solve_lds(const T* __restrict__ hrow, T Bq, T gam) {
    solve_steps<0>(hrow, Bq, gam);
    return gam;
}

// Occupancy hints (waves/SIMD): 5 for 8 f64 vectors per wave (<= 102 VGPRs),
// 3 for the 16-vector f32 kind, 4 for the 16-vector f64 kind (<= 128).  They
// hold because the per-rating values (partner-row offsets, residuals, scatter
// targets) and the row's normals sit in LDS, and the block solve reads its H
// row from LDS.
#define GBLOCK_OCC(T, V) ((V) * sizeof(T) > 64 ? 4 : (sizeof(T) == 8 ? 5 : 3))
template <typename T, int V, int NW, int RPW>
__global__ __launch_bounds__(64 * (NW > 1 ? NW : RPW), GBLOCK_OCC(T, V)) void k_gblock(const uint32_t* __restrict__ rows,
                                                                     uint32_t nrows, HalfArgs<T> a) {
    typedef typename MfmaT<T>::acc_t acc_t;
    constexpr int NWAVE = NW > 1 ? NW : RPW;
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int wr = NW > 1 ? wv : 0;           // wave within the row
    const uint32_t ri = NW > 1 ? blockIdx.x : blockIdx.x * RPW + wv;
    if (ri >= nrows) return;                  // NW>1: whole block; RPW: this wave only (no block barriers)
    SBMF_GBLOCK_PHASES(NW > 1);  // stamp(phase): the diagnostic phase profile (multi-wave rows)
    const uint32_t row = rows[ri];
    const uint32_t beg = a.ptr[row];
    const uint32_t n = a.ptr[row + 1] - beg;
    const uint32_t K = a.K, Kp = a.Kp;
    const int ci = lane & 15;                 // k within block / solve row
    const int rr = lane >> 4;                 // rating within vector

    __shared__ T Ls[NWAVE][GB][GLD];          // strictly lower part of G_B (row layout)
    __shared__ T Ps[NWAVE][GB];               // diagonal of G_B
    __shared__ T Cs[NWAVE][GB];               // c_B
    __shared__ T newS[NW > 1 ? 256 : 1];
    __shared__ T Dsh[GB];                     // multi-wave rows: the block's D from the solving wave
    const int ws = NW > 1 ? 0 : wv;           // LDS slot holding this row's reduced G / c

    // Per-rating and per-row values live in LDS, not VGPRs (occupancy): the row's
    // normals zS (read by the solving wave), this wave's partner-row offsets pjS
    // (row * Kp; the host checks (P+2) Kp < 2^32), residuals eS and scatter
    // targets pmS -- vector v, rating rr at [4 v + rr], read by all 16 lanes of the
    // rating; a residual is updated by the lane whose row sum covers it.
    __shared__ T zS[NW > 1 ? 1 : RPW][256];
    __shared__ uint32_t pjS[NWAVE][V * 4];
    __shared__ uint32_t pmS[NWAVE][V * 4];
    __shared__ T eS[NWAVE][V * 4];
    {  // per-half normals (host reference stream or launch_philox_fill)
        const uint32_t k0 = NW > 1 ? threadIdx.x : lane, kst = NW > 1 ? 64 * NW : 64;
        for (uint32_t k = k0; k < Kp; k += kst) zS[ws][k] = k < K ? a.zbuf[(size_t)CHK(row, a.lim_rows) * K + k] : T(0);
    }
    // ratings of this wave: vector v covers ratings q = (wr*V + v)*4 + rr;
    // slots past the row's end gather the partner table's zero row
    T e[V];  // the starting residuals (then kept in LDS)
    T* const eR = &eS[wv][rr];
    const uint32_t* const pjR = &pjS[wv][rr];
    // the row's ids, scatter targets and residuals by unconditional loads, issued a group
    // of (at most) 8 vectors at a time before their first use (a slot past the row's end
    // reads case 0 and then takes the zero row and a zero residual): per-slot conditional
    // loads were one dependent round trip each
    constexpr int SG = V < 8 ? V : V >= 16 ? 4 : 8;
#pragma unroll
    for (int g0 = 0; g0 < V; g0 += SG) {
        uint32_t pjv[SG], pmv[SG];
        T ev[SG];
#pragma unroll
        for (int u = 0; u < SG; ++u) {
            const uint32_t q = (uint32_t)((wr * V + g0 + u) * 4 + rr);
            const uint32_t qi = (uint32_t)CHK(q < n ? beg + q : 0u, a.lim_this);
            pjv[u] = a.part[qi];
            pmv[u] = a.perm[qi];
            ev[u] = a.e_from_dot ? T(0) : a.E_this[qi];
        }
#pragma unroll
        for (int u = 0; u < SG; ++u) {
            const int v = g0 + u;
            const uint32_t q = (uint32_t)((wr * V + v) * 4 + rr);
            const uint32_t pj = q < n ? pjv[u] : a.zrow;
            if (ci == 0) {
                pjS[wv][4 * v + rr] = pj * Kp;
                pmS[wv][4 * v + rr] = q < n ? pmv[u] : 0u;
                eR[4 * v] = q < n ? ev[u] : T(0);
            }
        }
    }
    asm volatile("" ::: "memory");  // read back by the other lanes of the wave (LDS keeps its order)
    const T* __restrict__ pbase = a.partner + ci;
#define PROW(v) (pbase + pjR[4 * (v)])
    // vector v's slice at column k0
    auto gat = [&](int v, uint32_t k0) -> T { return pbase[CHK(pjR[4 * v] + k0 + ci, a.lim_partner) - ci]; };
    if (a.e_from_dot) {  // validation mode (tune bit 1): e0 = r - own.partner
        T dot[V];
#pragma unroll
        for (int v = 0; v < V; ++v) dot[v] = T(0);
        for (uint32_t k0 = 0; k0 < K; k0 += GB) {
            const T o = a.own[(size_t)row * Kp + k0 + ci];  // padding columns are zero
#pragma unroll
            for (int v = 0; v < V; ++v) dot[v] += PROW(v)[k0] * o;
        }
#pragma unroll
        for (int v = 0; v < V; ++v) {
            const T d = row16_sum(dot[v]);
            const uint32_t q = (uint32_t)((wr * V + v) * 4 + rr);
            const T e0 = q < n ? a.r_this[beg + q] - d : T(0);
            if (ci == 0) eR[4 * v] = e0;
        }
    }
    asm volatile("" ::: "memory");  // read back by the other lanes of the wave (LDS keeps its order)
    const T tau = a.tau;
    const T* __restrict__ orow = a.own + (size_t)CHK(row, a.lim_rows) * Kp + ci;
    stamp(0);  // row setup (ids, residuals, normals)
    // software pipeline: block b+1's slices and own/sigma/mu values are in
    // flight while block b is reduced, solved and applied.  The prefetch past
    // the last block stays inside the tables (slack row / padding).
    // ratings for the train error, parked in LDS (read back by the same lanes
    // in the epilogue) so the epilogue waits on no global load
    __shared__ T Rs[NWAVE * V * 4];
    const bool want_r = a.row_tr != nullptr;
    if (want_r) {
#pragma unroll
        for (int g0 = 0; g0 < V; g0 += SG) {
            T rv[SG];
#pragma unroll
            for (int u = 0; u < SG; ++u) {
                const uint32_t q = (uint32_t)((wr * V + g0 + u) * 4 + rr);
                rv[u] = a.r_this[q < n ? beg + q : 0u];
            }
            if (ci == 0) {
#pragma unroll
                for (int u = 0; u < SG; ++u) {
                    const uint32_t q = (uint32_t)((wr * V + g0 + u) * 4 + rr);
                    Rs[(wv * V + g0 + u) * 4 + rr] = q < n ? rv[u] : T(0);
                }
            }
        }
    }
    T s[V], sn[V];
#pragma unroll
    for (int v = 0; v < V; ++v) s[v] = gat(v, 0);
    T oldc = orow[0], sgc = a.sig[ci], muc = a.mu[ci];
    for (uint32_t b0 = 0; b0 < K; b0 += GB) {
        const uint32_t kk = b0 + ci;
        const bool kin = kk < K;
        const uint32_t kn = b0 + GB;
        const T oldn = orow[kn];
        const T sgn = a.sig[kn + ci];
        const T mun = a.mu[kn + ci];
#pragma unroll
        for (int v = 0; v < V; ++v) sn[v] = gat(v, kn);
        acc_t g = {T(0), T(0), T(0), T(0)};
        T cc = T(0);
#pragma unroll
        for (int v = 0; v < V; ++v) {
            g = MfmaT<T>::mfma(s[v], g);
            cc += s[v] * eR[4 * v];
        }
        cc += shfl_xor_t(cc, 16);
        cc += shfl_xor_t(cc, 32);
        stamp(1);  // slice loads + G / c
        // ---- 2. G (strictly lower + diagonal), c -> LDS; multi-wave rows sum in wave order
        if constexpr (NW > 1) lds_barrier();  // previous block's readers of Ls are done
        stamp(2);  // barrier: other waves
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int r = MfmaT<T>::row(lane, j);
            Ls[NW > 1 ? wr : ws][r][ci] = ci < r ? g[j] : T(0);
            if (r == ci) Ps[NW > 1 ? wr : ws][ci] = g[j];
        }
        if (lane < GB) Cs[NW > 1 ? wr : ws][lane] = cc;
        if constexpr (NW > 1) {
            lds_barrier();
            for (int x = threadIdx.x; x < GB * GB; x += 64 * NW) {
                const int r0 = x >> 4, c0 = x & 15;
                if (c0 < r0) {
                    T sum = Ls[0][r0][c0];
#pragma unroll
                    for (int w = 1; w < NW; ++w) sum += Ls[w][r0][c0];
                    Ls[0][r0][c0] = sum;  // each entry owned by one thread: read-then-write is safe
                }
                if (x < GB) {
                    T cs = Cs[0][x], ps = Ps[0][x];
#pragma unroll
                    for (int w = 1; w < NW; ++w) {
                        cs += Cs[w][x];
                        ps += Ps[w][x];
                    }
                    Cs[0][x] = cs;
                    Ps[0][x] = ps;
                }
            }
            lds_barrier();
            stamp(3);  // cross-wave reduction
        } else {
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): own LDS writes visible to own reads
            __builtin_amdgcn_wave_barrier();
        }
        // ---- 3. the 16 sequential draws: the row's one wave, or -- multi-wave
        // rows -- wave 0 alone, handing D to the others through LDS (their issue
        // slots go to other rows)
        T dlt = T(0);
        if (NW == 1 || wr == 0) {
            const T P = Ps[ws][ci];
            const T old = oldc, sg = sgc, mu = muc;
            const T z = zS[ws][kk];
            const T var = kin ? T(1) / (sg + tau * P) : T(0);  // k >= K: var = 0 -> d = -old = 0
            const T sd = tsqrt_if(var, !a.sd_is_var);
            const T A = var * sg * mu + sd * z;
            const T Bq = var * tau;
            dlt = gblock_solve_lds(&Ls[ws][ci][0], Bq, A - old + Bq * (Cs[ws][ci] + P * old));
            const T nwv = old + dlt;
            if constexpr (NW > 1) {
                // staged in LDS, written after the last barrier: no wave of this
                // row can still have a load of the same own value in flight
                if (wr == 0 && lane < GB && kin) newS[kk] = nwv;
                if (lane < GB) Dsh[lane] = dlt;
            } else {
                if (lane < GB && kin) a.own[(size_t)row * Kp + kk] = nwv;  // one wave: program order
            }
        }
        if constexpr (NW > 1) {
            lds_barrier();
            dlt = Dsh[ci];
        }
        stamp(4);  // solve + D hand-off
        // ---- 4. e -= S_B D_B (lane (r,i) holds D_i): one butterfly reduce-scatter of the
        // V row sums (row16_scatter), each lane updating the residuals its sums cover
        {
#pragma unroll
            for (int v = 0; v < V; ++v) s[v] = s[v] * dlt;
            const int vb = row16_scatter(s, ci);
            constexpr int RV = V >= 16 ? V / 16 : 1;
#pragma unroll
            for (int j = 0; j < RV; ++j) eR[4 * (vb + j)] = eR[4 * (vb + j)] - s[j];
            asm volatile("" ::: "memory");
        }
        stamp(5);  // residual update
#pragma unroll
        for (int v = 0; v < V; ++v) s[v] = sn[v];
        oldc = oldn;
        sgc = sgn;
        muc = mun;
    }

    if constexpr (NW > 1) {
        lds_barrier();
        for (uint32_t k = threadIdx.x; k < K; k += 64 * NW) a.own[(size_t)row * Kp + k] = newS[k];
    }
    // ---- epilogue: residuals out, per-row partial sums
    T sq = T(0), trs = T(0);
#pragma unroll
    for (int v = 0; v < V; ++v) e[v] = eR[4 * v];
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const uint32_t q = (uint32_t)((wr * V + v) * 4 + rr);
        if (q < n && ci == 0) {
            a.E_other[CHK(pmS[wv][4 * v + rr], a.lim_other)] = e[v];
            sq += e[v] * e[v];
            if (want_r) {
                const T r = Rs[(wv * V + v) * 4 + rr];
                T pr = r - e[v];
                pr = (pr < a.hi) ? pr : a.hi;
                pr = (a.lo < pr) ? pr : a.lo;
                trs += (pr - r) * (pr - r);
            }
        }
    }
    if (a.row_sq || a.row_tr) {
        double dsq = wave_sum((double)sq);
        double dtr = wave_sum((double)trs);
        if constexpr (NW > 1) {
            __shared__ double red2[NW][2];
            if (lane == 0) {
                red2[wr][0] = dsq;
                red2[wr][1] = dtr;
            }
            lds_barrier();  // LDS only: the residual scatter stores stay in flight
            dsq = 0.0;
            dtr = 0.0;
            for (int w = 0; w < NW; ++w) {
                dsq += red2[w][0];
                dtr += red2[w][1];
            }
        }
        if (wr == 0 && lane == 0) {
            if (a.row_sq) a.row_sq[row] = dsq;
            if (a.row_tr) a.row_tr[row] = dtr;
        }
    }
    stamp(6);  // epilogue
#undef PROW
}


// ------------------------------------------------- register-resident streaming rows
// The default kernel for rows above the Gram-block bins: one NW-wave workgroup
// (4, 8 or 16 waves) per task of at most CAP = 4*NW*VW ratings (a whole row, or
// one equal chunk of a longer row), in one ordinary persistent launch per stream
// set, tasks claimed in list order from a queue head by whichever workgroup is
// free; a split row's chunks are consecutive, so a chunk waits only for peers
// the next free workgroups claim (no co-residency requirement).  Wave w owns
// vectors w, w+NW, ... (4 ratings x 16 k each).
// The partner slice of the current k-block stays in VGPRs from the accumulate
// (G_B = S^T S by MFMA, c_B = S^T e) until the apply (e -= S_B D_B) after the
// block's draws, so each slice is gathered once per half-sweep (k_gstream
// gathers it twice: to accumulate, and again one traversal later to apply).
// Per block t, per vector: apply D_{t-1} with the held slice, then issue the
// gather of slice t into the same registers; then accumulate block t.  The
// task's partner ids, residuals, scatter targets and ratings sit in LDS.
// Split rows hand their (G_B, c_B) partials over without fences: each chunk
// writes its packed partial (152 doubles: the lower triangle of G_B with its
// diagonal, then c_B) with write-through (sc1) stores, drains them and adds
// once to the block's agent-scope counter; every chunk polls the counter (sc1
// loads) for nch and then reads all partials -- MI355X_MICROARCH.md hand-off
// table, first row.  The chunk sum of an entry is split over the workgroup's
// spare threads (3 per entry for 8 waves), each summing a fixed range of
// chunks in order, the pieces added in piece order, so it never depends on
// which chunk arrives last and every chunk gets the same bits.
__device__ __forceinline__ void st_sc1(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
struct GresSums {
    double sq, tr;
};
// Residual slot of rating q (of a task) in LDS: slot q.  The butterfly residual
// update has lane ci of a rating write the residuals of vectors vb(ci) + j, whose
// slots are 4*NW apart, so all 16 lanes of a rating hit one bank pair (16-way
// conflicts on two writes per lane per block); an XOR swizzle that removed them
// measured 5 % slower on the item stage (VGPR spills, r03b), a pad slot per 32
// 1 % slower.
// The order in which k_gres' residual update issues the next block's gathers:
// the butterfly frees vectors [VP/2, VC) first, then [VP/4, VP/2), ..., and the
// vectors whose residuals the lane updates ([0, RV)) last.
// (measured: item streaming 3.56 -> 3.49 ms, user 1.515 -> 1.49 against index order, r03s3)
template <int VC>
struct GresOrder {
    static constexpr int VP = VC <= 8 ? 8 : VC <= 16 ? 16 : VC <= 32 ? 32 : VC <= 64 ? 64 : 128;
    static constexpr int RV = VP >= 16 ? VP / 16 : 1;
    struct Arr {
        int a[VC];
    };
    static constexpr Arr make() {
        Arr o{};
        int n = 0;
        const int lo[4] = {VP / 2, VP / 4, VP / 8, VP / 16};
        const int hi[4] = {VC, VP / 2, VP / 4, VP / 8};
        for (int l = 0; l < 4; ++l) {
            if (l == 3 && VP < 16) break;
            for (int j = lo[l]; j < hi[l] && j < VC; ++j) o.a[n++] = j;
        }
        for (int j = 0; j < RV && j < VC; ++j) o.a[n++] = j;
        return o;
    }
    static constexpr Arr arr = make();
    static constexpr const int* v = arr.a;
};
template <typename T>
struct GresW {  // vectors (of 4 ratings) per wave held in VGPRs: 64 VGPRs of slices
    static constexpr int VW = sizeof(T) == 8 ? 32 : 64;
};
// LIST: whole rows of a Gram-block bin, one workgroup per row of the list (k_grow; NW 1 or 2,
// no split rows), instead of tasks claimed from a queue (k_gres).  One wave (NW = 1) takes
// its G_B straight from the MFMA registers into the solve's image and its D from its own
// solve, with no cross-wave sum and no hand-off: the per-row LDS is small enough for four
// one-wave workgroups per SIMD.
template <typename T, int NW, int SIDE, bool LIST, int KL = 256>
__device__ __forceinline__ void gres_run(const SplitTask* __restrict__ tasks, const uint32_t* __restrict__ lrows,
                                         uint32_t ntask, const HalfArgs<T>& a, const SplitSync& sy) {
    typedef typename MfmaT<T>::acc_t acc_t;
    constexpr bool ONE = NW == 1;
    // whole rows of a list: the solving waves write the new own row themselves; KL (>= Kp) sizes
    // the row's LDS copies of its normals, old values, sigma and mu.  At KL = 256 a list kernel
    // reads sigma and mu from memory (four one-wave workgroups per SIMD fit the LDS only
    // without those copies), which puts an L2 round trip in front of every block's draws
    constexpr bool DIRECT = LIST;
    constexpr bool SMG = LIST && KL > 128;
    constexpr int VW = GresW<T>::VW;
    constexpr uint32_t CAP = 4 * NW * VW;
    constexpr int SL = GB * GB + GB;  // slab doubles per (chunk, block): 16x16 image (lower + diagonal) | c
    const int lane = threadIdx.x & 63;
    const int wr = threadIdx.x >> 6;
    const int ci = lane & 15;
    const int rr = lane >> 4;
    const uint32_t K = a.K, Kp = a.Kp;
    const uint32_t nblk = (K + GB - 1) / GB;
    const T tau = a.tau;
    __shared__ uint32_t pjL[CAP];      // partner row offset (row * Kp) per rating slot (zero row past the end)
    __shared__ uint32_t pmL[CAP];      // residual scatter target per rating
    __shared__ T eL[CAP];              // residuals (bit-identical in the 16 lanes of a rating)
    // per-wave block partials: the 16x17 image of G_B (row r, column c at r*GLD + c, all 256
    // entries as the MFMA leaves them) followed by c_B; Rr: the reduced entries in the same
    // layout, except that the diagonal goes to Rr[PW + r]: the image's diagonal and upper part
    // stay zero (cleared once), so the solve reads whole H rows unmasked
    constexpr int PW = GB * GLD + GB;
    __shared__ T Pw[NW][ONE ? 1 : PW];
    __shared__ T Rr[PW + GB + (ONE ? 64 : 0)];  // (one wave: + a slot per lane for the upper part)
    __shared__ T newS[DIRECT ? 1 : 256];
    __shared__ double red2[NW][2];
    // packed exchange entries: SLP = 136 (lower triangle incl. diagonal) + 16 (c);
    // thread x < SLP owns entry x; XP threads per entry share a split row's chunk sum
    // (NW >= 3; one- and two-wave workgroups take whole rows only and loop over the entries)
    constexpr int SLP = GB * (GB + 1) / 2 + GB;
    constexpr bool XCH = NW >= 3;
    constexpr int XP = XCH ? (64 * NW) / SLP : 1;
    static_assert(XP >= 1 && SLP <= SL, "exchange geometry");
    __shared__ double xsum[XP][XCH ? SLP : 1];
    // packed entry x -> its offset in a partial image, and in Rr (computed once: no per-block geometry)
    __shared__ uint16_t xoff[ONE ? 1 : SLP], xdst[ONE ? 1 : SLP];
    // the row's normals and old values, sigma and mu: read by the solving wave from LDS
    // (kept out of the VGPRs the held slices need)
    __shared__ T zL[KL], oL[KL], sgL[SMG ? 1 : KL], muL[SMG ? 1 : KL];
    if constexpr (!ONE)
    for (int x = threadIdx.x; x < SLP; x += 64 * NW) {
        int r = 0;
        while ((r + 1) * (r + 2) / 2 <= x && r < GB) ++r;  // row of the packed triangle
        const int c = x - r * (r + 1) / 2;  // column (packed triangle entries)
        xoff[x] = (uint16_t)(x < GB * (GB + 1) / 2 ? r * GLD + c : GB * GLD + (x - GB * (GB + 1) / 2));
        xdst[x] = (uint16_t)(x < GB * (GB + 1) / 2 && c == r ? PW + r : xoff[x]);
    }
    for (int x = threadIdx.x; x < PW + GB; x += 64 * NW) Rr[x] = T(0);
    // this wave's index as a scalar, and the lane: the thread id is rebuilt from them in the
    // block loop (no VGPR held across it, no spill slot to reload)
    const int wr_s = __builtin_amdgcn_readfirstlane(wr);
    if constexpr (!SMG)
    for (uint32_t k = threadIdx.x; k < Kp; k += 64 * NW) {
        sgL[k] = a.sig[k];
        muL[k] = a.mu[k];
    }
    // this lane's slots: vector j of wave wr is rating 4*(wr + j*NW) + rr, i.e.
    // a fixed per-lane base plus j*4*NW (an immediate LDS offset)
    const uint32_t* const pjW = pjL + 4 * wr + rr;
    const uint32_t lb = 4 * wr + rr;  // this lane's slot in every vector
    constexpr int JS = 4 * NW;
    // residual slot of this lane's rating in vector j of its wave (j = vector index / NW):
    // a fixed per-lane base plus an immediate offset per j
    auto eS = [&](uint32_t j) -> T& { return eL[j * JS + lb]; };

    // task order: a queue claimed in list order, one returning atomic per task,
    // so a split row's chunks start as soon as enough workgroups are free
    __shared__ uint32_t qti;
    // (the task loop in this form, also for the one-task LIST case: written as a task lambda
    // called once or in the loop, k_grow compiles to 50-70 spilled VGPRs instead of 1-2)
    for (uint32_t it = 0;; ++it) {
        uint32_t ti;
        if constexpr (LIST) {
            ti = blockIdx.x;
            if (it > 0 || ti >= ntask) break;
        } else {
            if (threadIdx.x == 0)
                qti = __hip_atomic_fetch_add(sy.counters + sy.ncounters, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __syncthreads();
            ti = qti;
            __syncthreads();  // every thread has its ticket before thread 0 claims the next
            if (ti >= ntask) break;
        }
        SplitTask tk;
        if constexpr (LIST) {
            const uint32_t r = lrows[ti];
            tk = SplitTask{r, a.ptr[r], a.ptr[r + 1] - a.ptr[r], 1u, 0u, 0u, 0u, 0u};
        } else {
            tk = tasks[ti];
        }
        const uint32_t n = tk.len;
        if (n == 0) continue;  // empty round slot (uniform)
        const uint32_t row = tk.row, beg = tk.beg, nch = tk.nch;
        const uint32_t vpw = ((n + 3) / 4 + NW - 1) / NW;  // vectors per wave
        SBMF_GRES_PHASES(nch);  // stamp(phase): the diagnostic phase profile
        // size class: the task's vectors per wave, rounded up to VW/4, VW/2, 3VW/4 or VW
        auto body = [&](auto vc) {
            constexpr int VC = decltype(vc)::value;
            const uint32_t npad = 4 * NW * VC;
            for (uint32_t x = threadIdx.x; x < npad; x += 64 * NW) {
                const bool in = x < n;
                const uint32_t qx = in ? (uint32_t)CHK(beg + x, a.lim_this) : 0u;
                pjL[x] = (in ? a.part[qx] : a.zrow) * Kp;  // host checks (P+2)*Kp < 2^32
                pmL[x] = in ? a.perm[qx] : 0u;
                if (!a.e_from_dot) eL[x] = in ? a.E_this[qx] : T(0);
            }
            for (uint32_t k = threadIdx.x; k < Kp; k += 64 * NW) {  // per-half normals and old values of the row
                zL[k] = k < K ? a.zbuf[(size_t)CHK(row, a.lim_rows) * K + k] : T(0);
                oL[k] = a.own[(size_t)CHK(row, a.lim_rows) * Kp + k];  // padding columns are zero
            }
            __syncthreads();
            if (a.e_from_dot) {  // validation mode (tune bit 1): e0 = r - own.partner
                for (uint32_t v = wr; v < (npad >> 2); v += NW) {
                    const uint32_t q = 4 * v + rr;
                    const uint32_t pj = pjL[q];
                    T d = T(0);
                    for (uint32_t k0 = 0; k0 < K; k0 += GB)
                        d += a.partner[(size_t)pj + k0 + ci] * a.own[(size_t)row * Kp + k0 + ci];
                    d = row16_sum(d);
                    if (ci == 0) eL[q] = q < n ? a.r_this[beg + q] - d : T(0);
                }
                __syncthreads();
            }
            stamp(0);  // staging
            const T* __restrict__ pbase = a.partner + ci;
            // the gather of vector j's slice of block t
            auto gat = [&](int j, uint32_t t) -> T {
                return pbase[CHK((size_t)pjW[j * JS] + t * GB + ci, a.lim_partner) - ci];
            };
            // Residual update e_v -= S_v D (vector v: 4 ratings x 16 columns, lane ci
            // holding column ci): s_v *= D in place, then a butterfly reduce-scatter
            // over the 16 lanes of each rating (row_ror:8, row_half_mirror, quad_perm
            // xor 2, xor 1), after which lane ci holds the complete sums of
            // max(1, VC/16) vectors and updates their residuals in LDS -- 2 (VC - 1)
            // DPP moves instead of 4 VC row-sum steps.  The registers each level
            // frees take their next slices at once (next(j) = the gather of vector j).
            auto apply = [&](auto& s, T D, auto&& next) {
                // VC rounded up to a power of two (VP); vectors VC..VP-1 are zero
                constexpr int VP = VC <= 8 ? 8 : VC <= 16 ? 16 : VC <= 32 ? 32 : VC <= 64 ? 64 : 128;
#pragma unroll
                for (int j = 0; j < VC; ++j) s[j] = s[j] * D;
                bfly_level<0x128, VP>(s, ci & 8);
#pragma unroll
                for (int j = VP / 2; j < VC; ++j) next(j);
                bfly_level<0x141, VP / 2>(s, ci & 4);
#pragma unroll
                for (int j = VP / 4; j < VP / 2; ++j) next(j);
                bfly_level<0x4e, VP / 4>(s, ci & 2);
#pragma unroll
                for (int j = VP / 8; j < VP / 4; ++j) next(j);
                if constexpr (VP >= 16) {
                    bfly_level<0xb1, VP / 8>(s, ci & 1);
#pragma unroll
                    for (int j = VP / 16; j < VP / 8; ++j) next(j);
                } else {
                    s[0] = s[0] + dpp<0xb1, 0xf>(s[0]);  // both lanes of the pair: the same sum
                }
                constexpr int RV = VP >= 16 ? VP / 16 : 1;
                const int vb = ((ci & 8) ? VP / 2 : 0) + ((ci & 4) ? VP / 4 : 0) + ((ci & 2) ? VP / 8 : 0) +
                               ((VP >= 16 && (ci & 1)) ? VP / 16 : 0);
#pragma unroll
                for (int j = 0; j < RV; ++j) {
                    if (VP == VC || vb + j < VC) {  // a zero vector's sum updates nothing
                        T& pe = eS(vb + j);
                        pe = pe - s[j];
                    }
                }
                // other lanes of this wave read these residuals next (LDS keeps a wave's
                // accesses in order); keep the compiler from moving reads above the writes
                asm volatile("" ::: "memory");
#pragma unroll
                for (int j = 0; j < RV; ++j) next(j);
            };
            T Dl = T(0);
            // G_t = S_t^T S_t by MFMA, c_t = S_t^T e (this lane's column, summed over
            // the 4 ratings of each vector)
            auto accumulate = [&](auto& s, acc_t& g, T& cc) {
#pragma unroll
                for (int i = 0; i < VC; ++i) {
                    // vectors in the order their gathers were issued (GresOrder): the first
                    // MFMAs wait only for the oldest loads, not for all of them
                    const int j = GresOrder<VC>::v[i];
                    g = MfmaT<T>::mfma(s[j], g);
                    cc += s[j] * eS(j);
                }
                cc += shfl_xor_t(cc, 16);
                cc += shfl_xor_t(cc, 32);
            };
            // the block's partials into LDS, the cross-wave sum, the split-row
            // exchange and the 16 draws: returns D_t (every lane: its column's)
            // pf: a prefetch of the next block's slices (NPF vector-memory loads per wave),
            // issued here so that it stays in flight through the block's exchange and draws.
            // Every barrier below is an LDS-only barrier (lds_barrier: __syncthreads() would
            // wait vmcnt(0) and drain the prefetch); a split row's partial stores are issued
            // before the prefetch and waited for with vmcnt(NPF).
            auto finish_block = [&](const acc_t& g, T cc, uint32_t t, auto&& pf, auto npf) -> T {
                constexpr int NPF = decltype(npf)::value;
                T Dl;
                if (nch == 1) pf();
                if constexpr (ONE) {
                    // one wave: the image straight from the MFMA registers (strict lower part,
                    // the diagonal apart, c after it); its upper part stays zero: those entries
                    // go to a slot of their lane past the image (no exec-mask branches)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int r = MfmaT<T>::row(lane, j);
                        Rr[ci < r ? r * GLD + ci : ci == r ? PW + r : PW + GB + lane] = g[j];
                    }
                    if (lane < GB) Rr[GB * GLD + lane] = cc;
                    lds_barrier();
                } else {
                    T* const pw = &Pw[wr_s][0];
#pragma unroll
                    for (int j = 0; j < 4; ++j) pw[MfmaT<T>::row(lane, j) * GLD + ci] = g[j];
                    if (lane < GB) pw[GB * GLD + lane] = cc;
                    lds_barrier();
                }
                stamp(3);  // wait for the other waves
                if constexpr (NW == 2) {  // two waves: each thread sums its entries in wave order
                    const int tid = wr_s * 64 + (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
                    for (int x = tid; x < SLP; x += 64 * NW) {
                        const int xo = xoff[x];
                        T val = T(0);
#pragma unroll
                        for (int w = 0; w < NW; ++w) val += Pw[w][xo];
                        Rr[xdst[x]] = val;
                    }
                    lds_barrier();
                }
                if constexpr (XCH) {
                // cross-wave sum in wave order: thread x < SLP holds packed entry x
                // (lower triangle incl. the diagonal, then c); the entry's geometry is
                // recomputed here from an opaque thread id so it holds no VGPRs across
                // the block loop
                const int tid = wr_s * 64 + (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
                const int xe = tid % SLP, xpart = tid / SLP;
                const bool xin = tid < SLP;
                const int xo = xin ? (int)xoff[xe] : 0;  // the entry's offset in every partial image
                const int xd = xin ? (int)xdst[xe] : 0;  // and in Rr
                T val = T(0);
                if (xin) {
#pragma unroll
                    for (int w = 0; w < NW; ++w)
                        val += Pw[w][xo];
                }
                const bool xchg = nch > 1;
                if (xchg) {
                    // cross-chunk sum over the row's chunks (see the header comment):
                    // every chunk stores its packed partial, adds once to the block's
                    // counter and, once all nch have added, sums the partials in chunk
                    // order -- XP threads per entry, each over a fixed third (or so) of
                    // the chunks, the XP pieces added in piece order in LDS
                    const size_t cstride = (size_t)nblk * SL;  // between one chunk's slabs and the next's
                    const double* pb = sy.slabs + ((size_t)tk.slab0 * nblk + t) * SL;
                    (void)CHK(((size_t)(tk.slab0 + nch - 1) * nblk + t) * SL + SL - 1, sy.lim_slab);  // the row's last slab
                    if (xin) st_sc1(const_cast<double*>(pb) + tk.chunk * cstride + xe, (double)val);
                    asm volatile("" ::: "memory");
                    pf();
                    asm volatile("" ::: "memory");
                    // this wave's partial stores (older than the prefetch) are done; the last block
                    // prefetches nothing, so it waits for everything
                    if (NPF > 0 && t + 1 < nblk)
                        wait_vmcnt<NPF>();
                    else
                        wait_vmcnt<0>();
                    lds_barrier();
                    uint32_t* cnt = sy.counters + CHK((size_t)tk.cnt0 + t, sy.ncounters);
                    if (threadIdx.x == 0) {
                        // no return value to wait for: the poll follows at once
                        __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        uint32_t spins = 0;
                        while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < nch) {
                            __builtin_amdgcn_s_sleep(1);
                            if (++spins > (1u << 26)) {  // give up: flag, never hang the device
                                __hip_atomic_store(sy.timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                break;
                            }
                        }
                    }
                    lds_barrier();
                    if (xpart < XP) {
                        const uint32_t c0 = xpart * nch / XP, c1 = (xpart + 1) * nch / XP;
                        const double* p0 = pb + xe;
                        double sum = 0.0;
                        uint32_t c = c0;
                        for (; c + 8 <= c1; c += 8) {  // 8 sc1 loads in flight
                            double v[8];
#pragma unroll
                            for (int u = 0; u < 8; ++u) v[u] = ld_sc1(p0 + (c + u) * cstride);
#pragma unroll
                            for (int u = 0; u < 8; ++u) sum += v[u];
                        }
                        for (; c < c1; ++c) sum += ld_sc1(p0 + c * cstride);
                        xsum[xpart][xe] = sum;
                    }
                    lds_barrier();
                    if (xin) {
                        double sum = xsum[0][xe];
#pragma unroll
                        for (int q = 1; q < XP; ++q) sum += xsum[q][xe];
                        val = (T)sum;
                    }
                }
                if (xin) Rr[xd] = val;
                lds_barrier();
                }  // XCH
                stamp(4);  // cross-wave sum + split-row exchange
                // the 16 draws: every wave draws the same 16 from the same LDS image (the same
                // bits), so D needs no hand-off -- one barrier per block fewer than wave 0 drawing
                // and handing D over in LDS (item stage 3.49-3.54 -> 3.44 ms, r05s13)
                T dlt;
                {
                    const uint32_t kk = t * GB + ci;
                    const bool kin = kk < K;
                    // the block's old values, hyperparameters and normals (zero padded)
                    T sg, mu;
                    if constexpr (SMG) {
                        sg = a.sig[kk];
                        mu = a.mu[kk];
                    } else {
                        sg = sgL[kk];
                        mu = muL[kk];
                    }
                    const T old = oL[kk], z = zL[kk];
                    const T P = Rr[PW + ci];
                    const T Cc = Rr[GB * GLD + ci];
                    const T var = kin ? T(1) / (sg + tau * P) : T(0);
                    const T sd = tsqrt_if(var, !a.sd_is_var);  // no square root under the quirk
                    const T A = var * sg * mu + sd * z;
                    const T Bq = var * tau;
                    dlt = gblock_solve_lds(&Rr[ci * GLD], Bq, A - old + Bq * (Cc + P * old));
                    if (lane < GB && wr == 0) {
                        if constexpr (DIRECT) {
                            if (kin) a.own[(size_t)CHK(row, a.lim_rows) * Kp + kk] = old + dlt;
                        } else {
                            if (kin) newS[kk] = old + dlt;
                        }
                    }
                }
                Dl = dlt;  // every 16-lane row of every wave solved the same system
                stamp(5);  // solve
                return Dl;
            };
            {
                T s[VC];
#pragma unroll
                for (int j = 0; j < VC; ++j) s[j] = gat(j, 0);
                for (uint32_t t = 0; t < nblk; ++t) {
                    // keep the per-vector partner offsets in LDS: hoisting them out of
                    // the block loop would hold VC 64-bit addresses in VGPRs
                    asm volatile("" ::: "memory");
                    if (t > 0) {
                        // apply block t-1 with the held slice, then gather slice t into it
                        apply(s, Dl, [&](int j) { s[j] = gat(j, t); });
                    }
                    stamp(1);  // apply + gather issue
                    acc_t g = {T(0), T(0), T(0), T(0)};
                    T cc = T(0);
                    accumulate(s, g, cc);
                    stamp(2);  // gather wait + accumulate
                    Dl = finish_block(g, cc, t, [] {}, std::integral_constant<int, 0>{});
                }
                // apply the last block
                apply(s, Dl, [](int) {});
            }
            // residuals out and the per-row sums, one rating per thread in rating
            // order (no per-vector branches)
            __syncthreads();
            double sq = 0.0, trs = 0.0;
            for (uint32_t x = threadIdx.x; x < n; x += 64 * NW) {
                const T e = eL[x];
                a.E_other[CHK(pmL[x], a.lim_other)] = e;
                sq += (double)(e * e);
                if (a.row_tr) {
                    const T r = a.r_this[beg + x];
                    T pr = r - e;
                    pr = (pr < a.hi) ? pr : a.hi;
                    pr = (a.lo < pr) ? pr : a.lo;
                    trs += (double)((pr - r) * (pr - r));
                }
            }
            return GresSums{sq, trs};
        };
        GresSums sums;
        if (vpw <= (uint32_t)VW / 4)
            sums = body(std::integral_constant<int, VW / 4>{});
        else if (vpw <= (uint32_t)VW / 2)
            sums = body(std::integral_constant<int, VW / 2>{});
        else if (vpw <= (uint32_t)(3 * VW / 4))  // (user rows: 3 % faster, r03; item rows since round 5:
            sums = body(std::integral_constant<int, 3 * VW / 4>{});  // stage 3.51-3.55 -> 3.47-3.48 ms, r05s33)
        else
            sums = body(std::integral_constant<int, VW>{});
        // ---- new own row: whole rows write it, split rows stage it (k_split_finish publishes)
        if (!DIRECT && tk.chunk == 0)
            for (uint32_t k = threadIdx.x; k < K; k += 64 * NW) {
                if (nch > 1)
                    static_cast<T*>(sy.newown)[(size_t)CHK(tk.slab0, sy.lim_chunk) * Kp + k] = newS[k];
                else
                    a.own[(size_t)CHK(row, a.lim_rows) * Kp + k] = newS[k];
            }
        double dsq = wave_sum(sums.sq);
        double dtr = wave_sum(sums.tr);
        if (lane == 0) {
            red2[wr][0] = dsq;
            red2[wr][1] = dtr;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            dsq = 0.0;
            dtr = 0.0;
            for (int w = 0; w < NW; ++w) {
                dsq += red2[w][0];
                dtr += red2[w][1];
            }
            if (nch > 1) {
                sy.chunk_sq[CHK(tk.slab0 + tk.chunk, sy.lim_chunk)] = dsq;
                sy.chunk_tr[CHK(tk.slab0 + tk.chunk, sy.lim_chunk)] = dtr;
            } else {
                if (a.row_sq) a.row_sq[row] = dsq;
                if (a.row_tr) a.row_tr[row] = dtr;
            }
        }
        __syncthreads();  // LDS (ids, residuals, newS, red2) is reused by the next task
        stamp(6);  // epilogue
    }
}
template <typename T, int NW, int SIDE>
__global__ __launch_bounds__(64 * NW, 4) void k_gres(
    const SplitTask* __restrict__ tasks, uint32_t ntask, HalfArgs<T> a, SplitSync sy) {
    gres_run<T, NW, SIDE, false>(tasks, nullptr, ntask, a, sy);
}
template <typename T, int NW, int SIDE, int KL>
__global__ __launch_bounds__(64 * NW, 4) void k_grow(
    const uint32_t* __restrict__ rows, uint32_t nrows, HalfArgs<T> a) {
    const SplitSync sy{};
    gres_run<T, NW, SIDE, true, KL>(nullptr, rows, nrows, a, sy);
}

// Split rows: publish the new own rows and fold the chunk partial sums; and (every launch, with
// at least one block) put the set's split-row counters and queue head back to zero for the next
// streaming launch on this area, in stream order after k_gres.  (That clear was a fill launch per
// streaming stage on the compute stream: a kernel and a packet gap, r06s10 trace.  Done by
// k_gres's last workgroup instead, the exit count kept sy alive across the task loop: spilled
// SGPRs 80 -> 93 and VGPRs 14 -> 20 in the 16-wave item kernel, item half 3.57 -> 3.83-3.92 ms,
// r06s11 / r06s12.)
template <typename T>
__global__ __launch_bounds__(64) void k_split_finish(const SplitRow* __restrict__ srows, uint32_t nrows, HalfArgs<T> a,
                                                     SplitSync sy) {
    for (uint32_t i = blockIdx.x * 64 + threadIdx.x; i <= sy.ncounters; i += gridDim.x * 64) sy.counters[i] = 0u;
    if (blockIdx.x >= nrows) return;
    const SplitRow sr = srows[blockIdx.x];
    const uint32_t K = a.K, Kp = a.Kp;
    for (uint32_t k = threadIdx.x; k < K; k += 64) a.own[(size_t)sr.row * Kp + k] = static_cast<const T*>(sy.newown)[(size_t)sr.slab0 * Kp + k];
    if (threadIdx.x == 0) {
        double s = 0.0, t = 0.0;
        for (uint32_t c = 0; c < sr.nch; ++c) {
            s += sy.chunk_sq[sr.slab0 + c];
            t += sy.chunk_tr[sr.slab0 + c];
        }
        if (a.row_sq) a.row_sq[sr.row] = s;
        if (a.row_tr) a.row_tr[sr.row] = t;
    }
}


// ------------------------------------------------------------------ residual recompute
// One wave per row; 16 lanes per rating (lane (r = l>>4, i = l&15) covers
// k = 16b + i), so each partner row is read as whole 128-byte lines.
template <typename T>
__global__ __launch_bounds__(256) void k_resid(const ResidTask* __restrict__ tasks, uint32_t ntask,
                                                const uint32_t* __restrict__ part, const uint32_t* __restrict__ perm,
                                                const T* __restrict__ r, const T* __restrict__ own,
                                                const T* __restrict__ partner, uint32_t K, uint32_t Kp,
                                                T* __restrict__ E_other, double* __restrict__ task_sq,
                                                const double* __restrict__ b_own, const double* __restrict__ b_part,
                                                double b0) {
    const uint32_t ti = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (ti >= ntask) return;
    const ResidTask tk = tasks[ti];
    const int ci = lane & 15, rr = lane >> 4;
    const T* o = own + (size_t)tk.row * Kp;
    T ov[16];  // own row, this lane's k values (k = 16b + ci); padding columns are zero
#pragma unroll
    for (int b = 0; b < 16; ++b) ov[b] = 16 * b < (int)Kp ? o[16 * b + ci] : T(0);
    double sq = 0.0;
    const uint32_t end = tk.beg + tk.len;
    for (uint32_t i0 = tk.beg; i0 < end; i0 += 4) {
        const uint32_t idx = i0 + rr;
        const bool ok = idx < end;
        const T* src = partner + (size_t)part[ok ? idx : tk.beg] * Kp;
        T d = T(0);
#pragma unroll
        for (int b = 0; b < 16; ++b)
            if (16 * b < (int)Kp) d += ov[b] * src[16 * b + ci];
        d = row16_sum(d);
        if (ok && ci == 0) {
            // biased sampler: E = r - (((b0 + b_user) + b_item) + u.v) (gibbs_sbpmf2.cpp:342-359)
            const T e = b_own ? r[idx] - ((T)((b0 + b_part[part[idx]]) + b_own[tk.row]) + d) : r[idx] - d;
            E_other[perm[idx]] = e;
            sq += (double)(e * e);
        }
    }
    sq = wave_sum(sq);
    if (lane == 0) task_sq[ti] = sq;
}

// row_sq[row] = the row's task partials in task order (deterministic)
__global__ __launch_bounds__(256) void k_resid_rows(const uint32_t* __restrict__ tptr, uint32_t r0, uint32_t r1,
                                                     const double* __restrict__ task_sq, double* __restrict__ row_sq) {
    const uint32_t row = r0 + blockIdx.x * 256 + threadIdx.x;
    if (row >= r1) return;
    double s = 0.0;
    for (uint32_t t = tptr[row - r0]; t < tptr[row - r0 + 1]; ++t) s += task_sq[t];
    row_sq[row] = s;
}

// ------------------------------------------------------------------ column statistics
// Both tables in one launch: blocks [0, nA) take table A's 256-row chunks, the rest
// table B's.  Wave w sums rows 64w .. 64w+63 of its chunk in row order, loading RB
// rows at a time before their adds (one coalesced row segment per load, lane l on
// columns l, l + 64, ...); the four waves' partials are added in wave order (fixed:
// bitwise repeatable, and the same for any 256-aligned rank split).  Round 4 had
// four rows in flight per wave: the two tables ran at 1.3 / 0.35 TB/s (98 / 71 us at
// ML-20M K=100).
template <typename T, int CPL>
__global__ __launch_bounds__(256) void k_colstats(const T* __restrict__ tabA, uint32_t rA, const T* __restrict__ muA,
                                                   double* __restrict__ outA, uint32_t nA, const T* __restrict__ tabB,
                                                   uint32_t rB, const T* __restrict__ muB, double* __restrict__ outB,
                                                   uint32_t K, uint32_t Kp) {
    constexpr int RW = 64;                   // rows per wave
    constexpr int RB = CPL <= 2 ? 16 : 8;    // rows loaded at once (<= 32 doubles in flight per lane)
    const bool first = blockIdx.x < nA;
    const T* __restrict__ tab = first ? tabA : tabB;
    const T* __restrict__ mu = first ? muA : muB;
    double* __restrict__ out = first ? outA : outB;
    const uint32_t R = first ? rA : rB;
    const uint32_t c = first ? blockIdx.x : blockIdx.x - nA;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double m[CPL], s1[CPL], s2[CPL];
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
        const uint32_t k = lane + 64 * j;
        m[j] = k < K ? (double)mu[k] : 0.0;
        s1[j] = 0.0;
        s2[j] = 0.0;
    }
    const uint32_t rb = c * 256 + w * RW;
    for (int b0 = 0; b0 < RW; b0 += RB) {
        double x[RB][CPL];
#pragma unroll
        for (int i = 0; i < RB; ++i) {
            const uint32_t r = rb + b0 + i;
            const T* row = tab + (size_t)(r < R ? r : 0) * Kp + lane;
#pragma unroll
            for (int j = 0; j < CPL; ++j) x[i][j] = lane + 64 * j < Kp ? (double)row[64 * j] : 0.0;
        }
#pragma unroll
        for (int i = 0; i < RB; ++i) {
            if (rb + b0 + i < R) {
#pragma unroll
                for (int j = 0; j < CPL; ++j) {
                    s2[j] += (x[i][j] - m[j]) * (x[i][j] - m[j]);
                    s1[j] += x[i][j];
                }
            }
        }
    }
    __shared__ double red[4][2][64 * CPL];
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
        red[w][0][lane + 64 * j] = s2[j];
        red[w][1][lane + 64 * j] = s1[j];
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < K; k += 256) {
        out[(size_t)c * 2 * K + k] = ((red[0][0][k] + red[1][0][k]) + red[2][0][k]) + red[3][0][k];
        out[(size_t)c * 2 * K + K + k] = ((red[0][1][k] + red[1][1][k]) + red[2][1][k]) + red[3][1][k];
    }
}

// ------------------------------------------------------------------ test evaluation
// 256 test ratings per block: each 16-lane group of a wave takes 16 consecutive
// ratings (user order), two at a time, 16 lanes per rating (coalesced 128-byte
// reads of both factor rows).  Lane i of a group first loads everything rating i
// of its 16 needs besides the rows -- ids, target, running sum -- in one round
// trip; the ids reach the group's lanes by shuffles, and lane i updates rating
// i's running sum itself.  (Round 4 loaded the ids of each pair, then the rows,
// then the sum and target: three dependent round trips per pair.)
template <typename T, int PR, int CB, bool REUSE>
__global__ __launch_bounds__(256) void k_test(const uint32_t* __restrict__ tu, const uint32_t* __restrict__ ti,
                                               const double* __restrict__ tr, uint64_t t0, uint64_t t1,
                                               const T* __restrict__ U, const T* __restrict__ V, uint32_t K,
                                               uint32_t Kp, T lo, T hi, int collect, double div,
                                               double* __restrict__ sum, double* __restrict__ part,
                                               const double* __restrict__ bu, const double* __restrict__ bv,
                                               double b0) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int ci = lane & 15, rr = lane >> 4;
    // group rr of wave w: ratings gbase + 0..15
    const uint64_t gbase = t0 + (uint64_t)blockIdx.x * 256 + (uint64_t)w * 64 + (uint64_t)rr * 16;
    const uint32_t nb = Kp / 16;  // k-blocks; the padding columns are zero in both tables
    const uint64_t mt = gbase + ci;  // this lane's own rating
    const bool mok = mt < t1;
    const uint64_t mtc = mok ? mt : t0;
    const uint32_t myu = tu[mtc], myi = ti[mtc];
    const double myr = tr[mtc], mys = sum[mtc];
    double myb = 0.0;
    if (bu) myb = (b0 + bu[myu]) + bv[myi];
    double a2 = 0.0, t2 = 0.0;
    // products summed in k order, the zero padding columns adding +0 (the clamped
    // prediction is the same as over K columns); PR ratings per group at a time, CB
    // k-blocks of each loaded before the first product
    // REUSE (a row of at most CB k-blocks): the ratings are in user order, so a rating whose
    // user is the previous rating's keeps that user's row slices instead of loading them again
    T uc[REUSE ? CB : 1];
    uint32_t ucur = 0xffffffffu;
    for (int it = 0; it < 16; it += PR) {
        uint32_t uu[PR], ii[PR];
#pragma unroll
        for (int j = 0; j < PR; ++j) {
            const int src = (lane & 48) + it + j;  // lane it+j of this group
            uu[j] = (uint32_t)__shfl((int)myu, src);
            ii[j] = (uint32_t)__shfl((int)myi, src);
        }
        T p[PR];
#pragma unroll
        for (int j = 0; j < PR; ++j) p[j] = T(0);
        if constexpr (REUSE) {
            T ub[PR][CB], vb[PR][CB];
#pragma unroll
            for (int j = 0; j < PR; ++j) {
#pragma unroll
                for (int b = 0; b < CB; ++b)
                    if (b < (int)nb) vb[j][b] = V[(size_t)ii[j] * Kp + b * 16 + ci];
                if (uu[j] != ucur) {
#pragma unroll
                    for (int b = 0; b < CB; ++b)
                        if (b < (int)nb) uc[b] = U[(size_t)uu[j] * Kp + b * 16 + ci];
                    ucur = uu[j];
                }
#pragma unroll
                for (int b = 0; b < CB; ++b) ub[j][b] = uc[b];
            }
#pragma unroll
            for (int j = 0; j < PR; ++j)
#pragma unroll
                for (int b = 0; b < CB; ++b)
                    if (b < (int)nb) p[j] += ub[j][b] * vb[j][b];
        } else
        for (uint32_t c0 = 0; c0 < nb; c0 += CB) {
            T ub[PR][CB], vb[PR][CB];
#pragma unroll
            for (int j = 0; j < PR; ++j)
#pragma unroll
                for (int b = 0; b < CB; ++b)
                    if (c0 + b < nb) {
                        ub[j][b] = U[(size_t)uu[j] * Kp + (c0 + b) * 16 + ci];
                        vb[j][b] = V[(size_t)ii[j] * Kp + (c0 + b) * 16 + ci];
                    }
#pragma unroll
            for (int j = 0; j < PR; ++j)
#pragma unroll
                for (int b = 0; b < CB; ++b)
                    if (c0 + b < nb) p[j] += ub[j][b] * vb[j][b];
        }
#pragma unroll
        for (int j = 0; j < PR; ++j) {
            T pj = row16_sum(p[j]);  // the same value in the group's 16 lanes
            if (ci == it + j && mok) {
                if (bu) pj = (T)myb + pj;  // biased sampler (gibbs_sbpmf2.cpp:614-618)
                pj = (pj < hi) ? pj : hi;
                pj = (lo < pj) ? pj : lo;
                double s = mys;
                if (collect) {
                    s += (double)pj;
                    sum[mt] = s;
                }
                const double d = myr - s / div;
                a2 += d * d;
                const double dt = myr - (double)pj;
                t2 += dt * dt;
            }
        }
    }
    __shared__ double red[4][2];
    a2 = wave_sum(a2);
    t2 = wave_sum(t2);
    if (lane == 0) {
        red[w][0] = a2;
        red[w][1] = t2;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint64_t b = t0 / 256 + blockIdx.x;  // global block index
        part[2 * b] = red[0][0] + red[1][0] + red[2][0] + red[3][0];
        part[2 * b + 1] = red[0][1] + red[1][1] + red[2][1] + red[3][1];
    }
}

// ------------------------------------------------------------------ deterministic sums
__global__ __launch_bounds__(256) void k_sum_blocks(const double* __restrict__ in, uint64_t n, double* __restrict__ out) {
    const uint64_t b0 = (uint64_t)blockIdx.x * 1024;
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint64_t i = b0 + threadIdx.x * 4 + q;
        if (i < n) s += in[i];
    }
    s = wave_sum(s);
    __shared__ double red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
}

// out[w] = sum over chunks of in[c][w]: one block per column, thread t sums
// chunks t, t+256, ... in order, then a fixed tree -> deterministic.  Blocks
// [width, 2 width) do the same for a second array (in2, nchunk2 -> out2).
__global__ __launch_bounds__(256) void k_sum_cols(const double* __restrict__ in, uint32_t nchunk, uint32_t width,
                                                   double* __restrict__ out, const double* __restrict__ in2,
                                                   uint32_t nchunk2, double* __restrict__ out2) {
    uint32_t w = blockIdx.x;
    if (w >= width) {
        w -= width;
        in = in2;
        nchunk = nchunk2;
        out = out2;
    }
    double s = 0.0;
    for (uint32_t c = threadIdx.x; c < nchunk; c += 256) s += in[(size_t)c * width + w];
    s = wave_sum(s);
    __shared__ double red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) out[w] = ((red[0] + red[1]) + red[2]) + red[3];
}

// Per-half normals in throughput mode: z[row][2p + j] = pair p of the Philox
// stream (seed, row, sweep, tag) -- one thread per pair.
template <typename T>
__global__ __launch_bounds__(256) void k_philox_fill(T* __restrict__ z, uint32_t K, uint32_t r0, uint32_t r1,
                                                     uint64_t seed, uint32_t sweep, uint32_t tag) {
    const uint32_t npair = (K + 1) / 2;
    const uint64_t x = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint32_t row = r0 + (uint32_t)(x / npair), p = (uint32_t)(x % npair);
    if (row >= r1) return;
    double z0, z1;
    philox_normal_pair(seed, row, sweep, tag, p, z0, z1);
    z[(size_t)row * K + 2 * p] = (T)z0;
    if (2 * p + 1 < K) z[(size_t)row * K + 2 * p + 1] = (T)z1;
}

// Both tables' normals of one sweep in one launch: blocks [0, nbu) fill the user rows, the rest
// the item rows (each thread the pair k_philox_fill's thread would draw)
template <typename T>
__global__ __launch_bounds__(256) void k_philox_fill2(T* __restrict__ zu, uint32_t u0, uint32_t u1, T* __restrict__ zv,
                                                      uint32_t v0, uint32_t v1, uint32_t K, uint32_t nbu,
                                                      uint64_t seed, uint32_t sweep, uint32_t tagu, uint32_t tagv) {
    const uint32_t npair = (K + 1) / 2;
    const bool users = blockIdx.x < nbu;
    const uint64_t x = (uint64_t)(users ? blockIdx.x : blockIdx.x - nbu) * 256 + threadIdx.x;
    T* const z = users ? zu : zv;
    const uint32_t r0 = users ? u0 : v0, r1 = users ? u1 : v1;
    const uint32_t row = r0 + (uint32_t)(x / npair), p = (uint32_t)(x % npair);
    if (row >= r1) return;
    double z0, z1;
    philox_normal_pair(seed, row, sweep, users ? tagu : tagv, p, z0, z1);
    z[(size_t)row * K + 2 * p] = (T)z0;
    if (2 * p + 1 < K) z[(size_t)row * K + 2 * p + 1] = (T)z1;
}

template <typename T>
__global__ __launch_bounds__(256) void k_init_philox(T* __restrict__ tab, uint32_t K, uint32_t Kp, uint32_t r0,
                                                      uint32_t r1, double sd, uint64_t seed, uint32_t tag) {
    const uint32_t row = r0 + blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= r1) return;
    for (uint32_t zs = 0; 128 * zs < K; ++zs) {
        double z0, z1;
        philox_normal_pair(seed, row, 0xffffffffu, tag, 64 * zs + lane, z0, z1);
        const uint32_t i0 = 128 * zs + 2 * lane;
        if (i0 < K) tab[(size_t)row * Kp + i0] = (T)(sd * z0);
        if (i0 + 1 < K) tab[(size_t)row * Kp + i0 + 1] = (T)(sd * z1);
    }
}

// ------------------------------------------------------------------ biased sampler
// Per-row bias step of the biased sampler (top-level gibbs_sbpmf2.cpp
// users :470-489 + :515-530, items :492-511 + :563-578; same algorithm in
// src/libfm/gibbs_sbpmf22.cpp).  One wave per row, run before the row's
// factor draws:
//   sigma_b ~ G(ag + 1, bg + 0.5 (b - mu_b)^2),  s = 1/(sg + sigma_b),
//   mu_b ~ N(s (sg mg + b sigma_b), s'),
//   e += d0 (the global-bias delta, folded into the user half),
//   sb = 1/(sigma_b + alpha n),  b' ~ N(sb (sigma_b mu_b + alpha sum(e + b)), sb'),
//   e += b - b'          (s' = s under the reference quirk, sqrt(s) otherwise).
// Variates: var3[row] = {gamma, normal, normal} from the host reference
// stream, or a per-row Philox stream (TAG_BIAS_*) when var3 is null.  Every
// lane evaluates the same draws (wave-uniform control flow); the row sum is
// a fixed-order lane fold + DPP tree, so results are deterministic.
template <typename T>
__global__ __launch_bounds__(256) void k_bias_rows(const uint32_t* __restrict__ ptr, uint32_t r0, uint32_t r1,
                                                    T* __restrict__ E, double* __restrict__ b,
                                                    double* __restrict__ mu_b, double* __restrict__ sig_b,
                                                    const double* __restrict__ var3, BiasArgs p) {
    // no FMA contraction: rows without ratings replay the host's shadow walk
    // (sbmf.cpp fill_bias_variates) operation for operation
#pragma clang fp contract(off)
    const uint32_t row = r0 + blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= r1) return;
    double g, zm, zb;
    if (var3) {
        g = var3[3 * (size_t)row];
        zm = var3[3 * (size_t)row + 1];
        zb = var3[3 * (size_t)row + 2];
    } else {
        PhiloxRowStream rs(p.seed, row, p.sweep, p.tag);
        g = mt_gamma(rs, p.ag + 1.0);
        zm = leva_normal(rs);
        zb = leva_normal(rs);
    }
    const double bo = b[row], mo = mu_b[row];
    const double sig = g / (p.bg + (0.5 * (bo - mo) * (bo - mo)));
    const double s4 = 1.0 / (p.sg + sig);
    const double mu = s4 * ((p.sg * p.mg) + bo * sig) + (p.sd_is_var ? s4 : sqrt(s4)) * zm;  // zm = 0: draw skipped
    const uint32_t beg = ptr[row], end = ptr[row + 1];
    const T d0 = (T)p.d0;
    // each lane's cases in order, eight loads in flight (a long item row is one wave's
    // serial walk: one load round trip per 64 ratings without them)
    double acc = 0.0;
    uint32_t q = beg + lane;
    for (; q + 7 * 64 < end; q += 8 * 64) {
        T ev[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) ev[u] = E[q + u * 64];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += (double)(ev[u] + d0) + bo;
    }
    for (; q < end; q += 64) acc += (double)(E[q] + d0) + bo;
    acc = wave_sum(acc);
    const double sb = 1.0 / (sig + (p.alpha * (double)(end - beg)));
    const double mb = sb * ((sig * mu) + p.alpha * acc);
    const double bn = mb + (p.sd_is_var ? sb : sqrt(sb)) * zb;
    const T db = (T)(bo - bn);
    q = beg + lane;
    for (; q + 7 * 64 < end; q += 8 * 64) {
        T ev[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) ev[u] = E[q + u * 64];
#pragma unroll
        for (int u = 0; u < 8; ++u) E[q + u * 64] = (ev[u] + d0) + db;
    }
    for (; q < end; q += 64) E[q] = (E[q] + d0) + db;
    if (lane == 0) {
        b[row] = bn;
        mu_b[row] = mu;
        sig_b[row] = sig;
    }
}

// Per-1024 block partials of sum(e) and sum(e^2) over E[0..n): part[2b], part[2b+1].
template <typename T>
__global__ __launch_bounds__(256) void k_esum2(const T* __restrict__ E, uint64_t n, double* __restrict__ part) {
    const uint64_t b0 = (uint64_t)blockIdx.x * 1024;
    double s = 0.0, s2 = 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint64_t i = b0 + threadIdx.x * 4 + q;
        if (i < n) {
            const double e = (double)E[i];
            s += e;
            s2 += e * e;
        }
    }
    s = wave_sum(s);
    s2 = wave_sum(s2);
    __shared__ double red[4][2];
    if ((threadIdx.x & 63) == 0) {
        red[threadIdx.x >> 6][0] = s;
        red[threadIdx.x >> 6][1] = s2;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = ((red[0][0] + red[1][0]) + red[2][0]) + red[3][0];
        part[2 * blockIdx.x + 1] = ((red[0][1] + red[1][1]) + red[2][1]) + red[3][1];
    }
}

// Per-row sum(e) and sum(e^2) over the rows [r0, r1) of one orientation
// (E in its order): out[2r], out[2r+1].  One wave per row, fixed lane order;
// summed over rows afterwards, the totals do not depend on the rank split.
template <typename T>
__global__ __launch_bounds__(256) void k_rowsum2(const uint32_t* __restrict__ ptr, uint32_t r0, uint32_t r1,
                                                 const T* __restrict__ E, double* __restrict__ out) {
    const uint32_t r = r0 + blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= r1) return;
    const int lane = threadIdx.x & 63;
    double s = 0.0, s2 = 0.0;
    const uint32_t end = ptr[r + 1];
    uint32_t q = ptr[r] + lane;
    for (; q + 7 * 64 < end; q += 8 * 64) {  // eight loads in flight, each lane's cases in order
        T ev[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) ev[u] = E[q + u * 64];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const double e = (double)ev[u];
            s += e;
            s2 += e * e;
        }
    }
    for (; q < end; q += 64) {
        const double e = (double)E[q];
        s += e;
        s2 += e * e;
    }
    s = wave_sum(s);
    s2 = wave_sum(s2);
    if (lane == 0) {
        out[2 * (size_t)r] = s;
        out[2 * (size_t)r + 1] = s2;
    }
}

// Multi-GPU residual exchange: residuals other ranks computed for this
// rank's rows arrive packed; put each at its position in this orientation.
template <typename T>
__global__ __launch_bounds__(256) void k_unpack(const T* __restrict__ recv, const uint32_t* __restrict__ idx,
                                                 uint64_t n, T* __restrict__ E) {
    const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (j < n) E[idx[j]] = recv[j];
}

}  // namespace

// ===================================================================== launchers
template <typename T>
hipError_t launch_gblock(int kind, const uint32_t* rows, uint32_t nrows, const HalfArgs<T>& a, hipStream_t st) {
    if (nrows == 0) return hipSuccess;
    if (a.K > 256) return hipErrorInvalidValue;
    // f64: 8 vectors (32 ratings) per wave; f32: 16 vectors (64 ratings) per wave
    constexpr int V = sizeof(T) == 8 ? 8 : 16;
    switch (kind) {
        case GK_W4:  // 1 wave / row, V/4 vectors, 4 rows / block
            k_gblock<T, V / 4, 1, 4><<<(nrows + 3) / 4, 256, 0, st>>>(rows, nrows, a);
            break;
        case GK_W16:  // 1 wave / row
            if (sizeof(T) == 8 && !(a.tune & 8u))  // wide (default): 16 vectors (64 ratings), 2 waves/SIMD
                k_gblock<T, 16, 1, 2><<<(nrows + 1) / 2, 128, 0, st>>>(rows, nrows, a);
            else
                k_gblock<T, V, 1, 4><<<(nrows + 3) / 4, 256, 0, st>>>(rows, nrows, a);
            break;
        case GK_B2:  // 2 waves / row
            k_gblock<T, V, 2, 1><<<nrows, 128, 0, st>>>(rows, nrows, a);
            break;
        case GK_B4:  // 4 waves / row
            k_gblock<T, V, 4, 1><<<nrows, 256, 0, st>>>(rows, nrows, a);
            break;
        case GK_B8:  // 8 waves / row
            k_gblock<T, V, 8, 1><<<nrows, 512, 0, st>>>(rows, nrows, a);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// Streaming rows: k_gres.  Tune bit 7 = 4-wave workgroups (4 per CU, 512-rating
// f64 tasks), bit 17 = 16-wave workgroups (one per CU, 2048-rating tasks),
// default 8-wave (two per CU); sbmf.cpp picks the shape per side and row length.
static int gres_nw(uint32_t tune) { return (tune & 128u) ? 4 : (tune & 0x20000u) ? 16 : 8; }
int gstream_wg_target(uint32_t tune) { return 16 / gres_nw(tune); }

// Multi-wave Gram-block rows of nw 8-vector waves (f64) / 16-vector waves (f32);
// f64 rows of 5-8 waves run as 3-4 waves of 16 vectors (measured faster: fewer
// waves meet at each block's barriers).
template <typename T>
hipError_t launch_gblock_nw(int nw, const uint32_t* rows, uint32_t nrows, const HalfArgs<T>& a, hipStream_t st) {
    if (nrows == 0) return hipSuccess;
    constexpr int V = sizeof(T) == 8 ? 8 : 16;
    const bool wide = sizeof(T) == 8 && nw >= 5;
#define SBMF_GB_NW(V_, NW_)                                                                      \
    case NW_:                                                                                    \
        k_gblock<T, V_, NW_, 1><<<nrows, 64 * NW_, 0, st>>>(rows, nrows, a);                     \
        break;
    if (wide) {
        switch ((nw + 1) / 2) {
            SBMF_GB_NW(16, 3)
            SBMF_GB_NW(16, 4)
            default:
                return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    switch (nw) {
        SBMF_GB_NW(V, 2)
        SBMF_GB_NW(V, 3)
        SBMF_GB_NW(V, 4)
        SBMF_GB_NW(V, 5)
        SBMF_GB_NW(V, 6)
        SBMF_GB_NW(V, 7)
        SBMF_GB_NW(V, 8)
        default:
            return hipErrorInvalidValue;
    }
#undef SBMF_GB_NW
    return hipGetLastError();
}

// Whole rows of a Gram-block bin on the streaming kernel's code, one workgroup per row:
// one wave per row (nw = 1: rows of <= 128 f64 / 256 f32 ratings) or two (nw = 2: twice that)
template <typename T>
hipError_t launch_grow(int nw, const uint32_t* rows, uint32_t nrows, const HalfArgs<T>& a, hipStream_t st) {
    if (nrows == 0) return hipSuccess;
    if (a.K > 256) return hipErrorInvalidValue;
    const bool side = a.tag == TAG_ITEMS;
    // Kp <= 128: the row's sigma and mu in LDS too (KL = 128); larger K: from memory (KL = 256)
    auto go = [&](auto kl) {
        constexpr int KL = decltype(kl)::value;
        if (nw == 1) {
            if (side)
                k_grow<T, 1, 1, KL><<<nrows, 64, 0, st>>>(rows, nrows, a);
            else
                k_grow<T, 1, 0, KL><<<nrows, 64, 0, st>>>(rows, nrows, a);
        } else if (nw == 2) {
            if (side)
                k_grow<T, 2, 1, KL><<<nrows, 128, 0, st>>>(rows, nrows, a);
            else
                k_grow<T, 2, 0, KL><<<nrows, 128, 0, st>>>(rows, nrows, a);
        } else {
            return hipErrorInvalidValue;
        }
        return hipGetLastError();
    };
    return a.Kp <= 128 && !(a.tune & 0x1000u) ? go(std::integral_constant<int, 128>{})
                                               : go(std::integral_constant<int, 256>{});
}
uint32_t grow_maxdeg(int nw, bool f64) { return 4u * (uint32_t)nw * (f64 ? GresW<double>::VW : GresW<float>::VW); }

template <typename T>
static const void* gstream_fn(uint32_t tune, uint32_t side = 0) {
    if (gres_nw(tune) == 4) return side ? (const void*)k_gres<T, 4, 1> : (const void*)k_gres<T, 4, 0>;
    if (gres_nw(tune) == 16) return side ? (const void*)k_gres<T, 16, 1> : (const void*)k_gres<T, 16, 0>;
    return side ? (const void*)k_gres<T, 8, 1> : (const void*)k_gres<T, 8, 0>;
}

template <typename T>
uint32_t gstream_cmax(uint32_t tune) {
    return 4 * gres_nw(tune) * GresW<T>::VW;  // the VGPR-resident task
}

template <typename T>
int gstream_blocks_per_cu(uint32_t cmax, uint32_t tune) {
    (void)cmax;
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, gstream_fn<T>(tune), 64 * gres_nw(tune), 0) != hipSuccess)
        return 1;
    return n;
}

template <typename T>
hipError_t launch_gstream(const SplitTask* tasks, uint32_t ntask, uint32_t grid, const SplitRow* srows, uint32_t nsrow,
                          const HalfArgs<T>& a, const SplitSync& sy, hipStream_t st) {
    if (ntask == 0) return hipSuccess;
    if (a.K > 256 || sy.cmax == 0 || grid == 0) return hipErrorInvalidValue;
    hipError_t err;
    // Tasks are claimed from a queue in list order by running workgroups, so only
    // the most recently claimed split row can have chunks still unclaimed, and its
    // waiting chunks (fewer than its chunk count, far below the resident
    // workgroups) never block the claims that complete it: an ordinary launch in
    // every schedule.  Tune bit 24 (experiments only) launches it cooperatively,
    // which checks that the whole grid fits (the host sizes it to residency); a
    // process that did so faulted in exit() under rocprofv3 (r04s16).
    const SplitTask* tp = tasks;
    HalfArgs<T> ap = a;
    SplitSync syp = sy;
    void* args[] = {(void*)&tp, (void*)&ntask, (void*)&ap, (void*)&syp};
    const void* fn = gstream_fn<T>(a.tune, a.tag == TAG_ITEMS ? 1u : 0u);
    const dim3 g(std::min(grid, ntask)), b(64 * gres_nw(a.tune));
    if (a.tune & 0x1000000u)
        err = hipLaunchCooperativeKernel(fn, g, b, args, 0, st);
    else
        err = hipLaunchKernel(fn, g, b, args, 0, st);
    if (err != hipSuccess) return err;
    {  // (no split rows: one block, the counter clear only)
        k_split_finish<T><<<std::max(nsrow, 1u), 64, 0, st>>>(srows, nsrow, a, sy);
        return hipGetLastError();
    }
    return hipSuccess;
}

template <typename T>
hipError_t launch_resid(const ResidTask* tasks, uint32_t ntask, const uint32_t* tptr, uint32_t r0, uint32_t r1,
                        const uint32_t* part, const uint32_t* perm, const T* r, const T* own, const T* partner,
                        uint32_t K, uint32_t Kp, T* E_other, double* task_sq, double* row_sq, const double* b_own,
                        const double* b_part, double b0, hipStream_t st) {
    if (r1 <= r0) return hipSuccess;
    if (Kp > 256) return hipErrorInvalidValue;
    if (ntask) k_resid<T><<<(ntask + 3) / 4, 256, 0, st>>>(tasks, ntask, part, perm, r, own, partner, K, Kp, E_other,
                                                          task_sq, b_own, b_part, b0);
    k_resid_rows<<<(r1 - r0 + 255) / 256, 256, 0, st>>>(tptr, r0, r1, task_sq, row_sq);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_colstats(const T* tabA, uint32_t rA, const T* muA, double* outA, const T* tabB, uint32_t rB,
                           const T* muB, double* outB, uint32_t K, uint32_t Kp, hipStream_t st) {
    const uint32_t nA = (rA + 255) / 256, nB = (rB + 255) / 256;
    if (nA + nB == 0) return hipSuccess;
    if (K > 256 || Kp > 256) return hipErrorInvalidValue;
    if (Kp <= 64)
        k_colstats<T, 1><<<nA + nB, 256, 0, st>>>(tabA, rA, muA, outA, nA, tabB, rB, muB, outB, K, Kp);
    else if (Kp <= 128)
        k_colstats<T, 2><<<nA + nB, 256, 0, st>>>(tabA, rA, muA, outA, nA, tabB, rB, muB, outB, K, Kp);
    else
        k_colstats<T, 4><<<nA + nB, 256, 0, st>>>(tabA, rA, muA, outA, nA, tabB, rB, muB, outB, K, Kp);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_test(const uint32_t* tu, const uint32_t* ti, const double* tr, uint64_t t0, uint64_t t1, const T* U,
                       const T* V, uint32_t K, uint32_t Kp, T lo, T hi, int collect, double div, double* sum,
                       double* part, const double* bu, const double* bv, double b0, hipStream_t st) {
    if (t1 <= t0) return hipSuccess;
    const uint64_t nb = (t1 - t0 + 255) / 256;
    // (4 ratings x 4 k-blocks per load round instead of 2 x 8: neutral, r05s7; the user-row
    // reuse: evaluation 0.30 -> 0.26 ms, sweep 7.36 -> 7.32 ms at ML-20M K=100, r05s9)
    if (Kp <= 128)
        k_test<T, 2, 8, true><<<(uint32_t)nb, 256, 0, st>>>(tu, ti, tr, t0, t1, U, V, K, Kp, lo, hi, collect, div, sum,
                                                            part, bu, bv, b0);
    else
        k_test<T, 2, 8, false><<<(uint32_t)nb, 256, 0, st>>>(tu, ti, tr, t0, t1, U, V, K, Kp, lo, hi, collect, div, sum,
                                                             part, bu, bv, b0);
    return hipGetLastError();
}

hipError_t launch_sum(const double* in, uint64_t n, double* out, double* scratch, hipStream_t st) {
    if (n == 0) return hipMemsetAsync(out, 0, sizeof(double), st);
    const double* cur = in;
    double* buf[2] = {scratch, scratch + (n + 1023) / 1024 + 1};
    int which = 0;
    while (n > 1) {
        const uint64_t nb = (n + 1023) / 1024;
        double* dst = (nb == 1) ? out : buf[which];
        k_sum_blocks<<<(uint32_t)nb, 256, 0, st>>>(cur, n, dst);
        hipError_t err = hipGetLastError();
        if (err != hipSuccess) return err;
        cur = dst;
        n = nb;
        which ^= 1;
        if (nb == 1) return hipSuccess;
    }
    return hipMemcpyAsync(out, cur, sizeof(double), hipMemcpyDeviceToDevice, st);
}

hipError_t launch_sum_cols(const double* in, uint32_t nchunk, uint32_t width, double* out, hipStream_t st) {
    k_sum_cols<<<width, 256, 0, st>>>(in, nchunk, width, out, nullptr, 0, nullptr);
    return hipGetLastError();
}
hipError_t launch_sum_cols2(const double* in, uint32_t nchunk, double* out, const double* in2, uint32_t nchunk2,
                            double* out2, uint32_t width, hipStream_t st) {
    k_sum_cols<<<2 * width, 256, 0, st>>>(in, nchunk, width, out, in2, nchunk2, out2);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_philox_fill(T* z, uint32_t K, uint32_t r0, uint32_t r1, uint64_t seed, uint32_t sweep, uint32_t tag,
                              hipStream_t st) {
    if (r1 <= r0 || K == 0) return hipSuccess;
    const uint64_t n = (uint64_t)(r1 - r0) * ((K + 1) / 2);
    k_philox_fill<T><<<(unsigned)((n + 255) / 256), 256, 0, st>>>(z, K, r0, r1, seed, sweep, tag);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_philox_fill2(T* zu, uint32_t u0, uint32_t u1, uint32_t tagu, T* zv, uint32_t v0, uint32_t v1,
                               uint32_t tagv, uint32_t K, uint64_t seed, uint32_t sweep, hipStream_t st) {
    const uint64_t npair = (K + 1) / 2;
    const uint64_t nbu = ((uint64_t)(u1 > u0 ? u1 - u0 : 0) * npair + 255) / 256;
    const uint64_t nbv = ((uint64_t)(v1 > v0 ? v1 - v0 : 0) * npair + 255) / 256;
    if (nbu + nbv == 0) return hipSuccess;
    k_philox_fill2<T><<<(unsigned)(nbu + nbv), 256, 0, st>>>(zu, u0, u1, zv, v0, v1, K, (uint32_t)nbu, seed, sweep, tagu,
                                                             tagv);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_init_philox(T* tab, uint32_t K, uint32_t Kp, uint32_t r0, uint32_t r1, double sd, uint64_t seed,
                              uint32_t tag, hipStream_t st) {
    if (r1 <= r0) return hipSuccess;
    k_init_philox<T><<<(r1 - r0 + 3) / 4, 256, 0, st>>>(tab, K, Kp, r0, r1, sd, seed, tag);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_bias_rows(const uint32_t* ptr, uint32_t r0, uint32_t r1, T* E, double* b, double* mu_b,
                            double* sig_b, const double* var3, const BiasArgs& p, hipStream_t st) {
    if (r1 <= r0) return hipSuccess;
    k_bias_rows<T><<<(r1 - r0 + 3) / 4, 256, 0, st>>>(ptr, r0, r1, E, b, mu_b, sig_b, var3, p);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_esum2(const T* E, uint64_t n, double* part, double* out2, hipStream_t st) {
    if (n == 0) return hipMemsetAsync(out2, 0, 2 * sizeof(double), st);
    const uint64_t nb = (n + 1023) / 1024;
    k_esum2<T><<<(uint32_t)nb, 256, 0, st>>>(E, n, part);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) return err;
    return launch_sum_cols(part, (uint32_t)nb, 2, out2, st);
}

template <typename T>
hipError_t launch_rowsum2(const uint32_t* ptr, uint32_t r0, uint32_t r1, const T* E, double* out, hipStream_t st) {
    if (r1 <= r0) return hipSuccess;
    k_rowsum2<T><<<(r1 - r0 + 3) / 4, 256, 0, st>>>(ptr, r0, r1, E, out);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_unpack(const T* recv, const uint32_t* idx, uint64_t n, T* E, hipStream_t st) {
    if (n == 0) return hipSuccess;
    k_unpack<T><<<(unsigned)((n + 255) / 256), 256, 0, st>>>(recv, idx, n, E);
    return hipGetLastError();
}

#define SBMF_INST(T)                                                                                                 \
    template hipError_t launch_gblock<T>(int, const uint32_t*, uint32_t, const HalfArgs<T>&, hipStream_t);          \
    template hipError_t launch_gblock_nw<T>(int, const uint32_t*, uint32_t, const HalfArgs<T>&, hipStream_t);       \
    template hipError_t launch_gstream<T>(const SplitTask*, uint32_t, uint32_t, const SplitRow*, uint32_t,           \
                                          const HalfArgs<T>&, const SplitSync&, hipStream_t);                        \
    template int gstream_blocks_per_cu<T>(uint32_t, uint32_t);                                                      \
    template hipError_t launch_grow<T>(int, const uint32_t*, uint32_t, const HalfArgs<T>&, hipStream_t);            \
    template uint32_t gstream_cmax<T>(uint32_t);                                                                    \
    template hipError_t launch_resid<T>(const ResidTask*, uint32_t, const uint32_t*, uint32_t, uint32_t,              \
                                        const uint32_t*, const uint32_t*, const T*, const T*, const T*, uint32_t,     \
                                        uint32_t, T*, double*, double*, const double*, const double*, double,         \
                                        hipStream_t);                                                                \
    template hipError_t launch_philox_fill<T>(T*, uint32_t, uint32_t, uint32_t, uint64_t, uint32_t, uint32_t,        \
                                              hipStream_t);                                                          \
    template hipError_t launch_philox_fill2<T>(T*, uint32_t, uint32_t, uint32_t, T*, uint32_t, uint32_t, uint32_t,   \
                                               uint32_t, uint64_t, uint32_t, hipStream_t);                           \
    template hipError_t launch_colstats<T>(const T*, uint32_t, const T*, double*, const T*, uint32_t, const T*,    \
                                           double*, uint32_t, uint32_t, hipStream_t);                                \
    template hipError_t launch_test<T>(const uint32_t*, const uint32_t*, const double*, uint64_t, uint64_t,         \
                                       const T*, const T*, uint32_t, uint32_t, T, T, int, double, double*, double*, \
                                       const double*, const double*, double, hipStream_t);                          \
    template hipError_t launch_init_philox<T>(T*, uint32_t, uint32_t, uint32_t, uint32_t, double, uint64_t,          \
                                              uint32_t, hipStream_t);                                                \
    template hipError_t launch_bias_rows<T>(const uint32_t*, uint32_t, uint32_t, T*, double*, double*, double*,      \
                                            const double*, const BiasArgs&, hipStream_t);                            \
    template hipError_t launch_esum2<T>(const T*, uint64_t, double*, double*, hipStream_t);                        \
    template hipError_t launch_unpack<T>(const T*, const uint32_t*, uint64_t, T*, hipStream_t);                    \
    template hipError_t launch_rowsum2<T>(const uint32_t*, uint32_t, uint32_t, const T*, double*, hipStream_t);
SBMF_INST(float)
SBMF_INST(double)

}  // namespace sbmf
