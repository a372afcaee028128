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
//   * k_rows<..., NW=1>  one 64-lane wave per row (deg <= 512): lanes own
//     ratings, the row's residuals live in VGPRs, partner slices of 32 B are
//     gathered per k-block, the two k-reductions per coordinate are DPP
//     wave sums (row_shr / row_bcast, no LDS);
//   * k_rows<..., NW>1>  NW waves cooperate on one row (deg <= 4096); wave
//     sums meet in LDS once per coordinate (double-buffered, one barrier);
//   * Gram route (deg > gram threshold): G = S^T S and b = S^T e0 per chunk
//     (k_gram_partial), fixed-order chunk reduction + the exact K-step
//     recurrence Q_k = b_k - sum_{l<k} G_kl D_l + G_kk u_k (k_gram_solve),
//     and e = r - S u_new (k_gram_update).  Algebraically identical to the
//     sequential coordinate loop.
// Layout: factor tables row-major [rows][Kp] (Kp = K padded to 32 B), so a
// partner row is one contiguous 4K/8K-byte record; ratings in CSR (users)
// and CSC (items) order; residuals kept per orientation and gathered through
// a fixed permutation (no atomics, deterministic).
#include <hip/hip_runtime.h>

#include "kernels.h"
#include "rng.h"

namespace sbmf {
namespace {

// ------------------------------------------------------------------ wave64 helpers
template <int CTRL, int ROWM>
__device__ __forceinline__ int dpp_i(int v) {
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
template <>
__device__ __forceinline__ float tsqrt<float>(float x) { return sqrtf(x); }
template <>
__device__ __forceinline__ double tsqrt<double>(double x) { return sqrt(x); }

// One coordinate draw, shared by all row paths.
template <typename T>
__device__ __forceinline__ T draw_coord(T P, T Q, T sg, T mu, T tau, T z, int sd_is_var) {
    const T var = T(1) / (sg + tau * P);
    const T mean = var * (tau * Q + sg * mu);
    const T sd = sd_is_var ? var : tsqrt(var);
    return mean + sd * z;
}

// ------------------------------------------------------------ light / medium rows
// NW waves per row, RPB rows per block (NW==1) ; KS = ceil(K/64) <= 4.
template <typename T, int MMAX, int NW, int RPB, int KS>
__global__ __launch_bounds__(64 * NW * RPB) void k_rows(const uint32_t* __restrict__ rows, uint32_t nrows,
                                                          HalfArgs<T> a) {
    constexpr int B = 32 / sizeof(T);  // slice width (k values per 32-byte gather)
    constexpr int ZS = (KS + 1) / 2;
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int wr = wv % NW;
    const int rib = wv / NW;
    const uint32_t ri = blockIdx.x * RPB + rib;
    if (ri >= nrows) return;  // uniform per row group (NW>1 => RPB==1: whole block)
    const uint32_t row = rows[ri];
    const uint32_t beg = a.ptr[row];
    const uint32_t n = a.ptr[row + 1] - beg;
    constexpr uint32_t G = 64 * NW;
    const uint32_t g = wr * 64 + lane;
    const int m = (int)((n + G - 1) / G);
    const uint32_t K = a.K, Kp = a.Kp;

    T own_r[KS], sig_r[KS], mu_r[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
        const uint32_t k = 64 * s + lane;
        own_r[s] = k < K ? a.own[(size_t)row * Kp + k] : T(0);
        sig_r[s] = k < K ? a.sig[k] : T(0);
        mu_r[s] = k < K ? a.mu[k] : T(0);
    }
    T z_r[ZS][2];
#pragma unroll
    for (int zs = 0; zs < ZS; ++zs) {
        const uint32_t i0 = 128 * zs + 2 * lane;
        if (a.zbuf) {
            z_r[zs][0] = i0 < K ? a.zbuf[(size_t)row * K + i0] : T(0);
            z_r[zs][1] = i0 + 1 < K ? a.zbuf[(size_t)row * K + i0 + 1] : T(0);
        } else {
            double z0, z1;
            philox_normal_pair(a.seed, row, a.sweep, a.tag, 64 * zs + lane, z0, z1);
            z_r[zs][0] = (T)z0;
            z_r[zs][1] = (T)z1;
        }
    }

    T e[MMAX];
    uint32_t pj[MMAX];
    bool ok[MMAX];
#pragma unroll
    for (int t = 0; t < MMAX; ++t) {
        const uint32_t nl = g + t * G;
        ok[t] = (t < m) && (nl < n);
        pj[t] = ok[t] ? a.part[beg + nl] : 0u;
        e[t] = T(0);
    }
    if (a.e_from_dot) {
        // e0 = r - own . partner  (pre-pass over the partner rows)
        T dot[MMAX];
#pragma unroll
        for (int t = 0; t < MMAX; ++t) dot[t] = T(0);
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            if (64 * s >= (int)K) break;
            for (int kb = 0; kb < 64; kb += B) {
                const int k0 = 64 * s + kb;
                if (k0 >= (int)K) break;
#pragma unroll
                for (int t = 0; t < MMAX; ++t) {
                    if (t < m) {
                        T sl[B];
                        if (ok[t]) load_slice(a.partner + (size_t)pj[t] * Kp + k0, sl);
                        else
#pragma unroll
                            for (int b = 0; b < B; ++b) sl[b] = T(0);
#pragma unroll
                        for (int b = 0; b < B; ++b) dot[t] += sl[b] * readlane(own_r[s], kb + b);
                    }
                }
            }
        }
#pragma unroll
        for (int t = 0; t < MMAX; ++t)
            if (ok[t]) e[t] = a.r_this[beg + g + t * G] - dot[t];
    } else {
#pragma unroll
        for (int t = 0; t < MMAX; ++t)
            if (ok[t]) e[t] = a.E_in[a.perm[beg + g + t * G]];
    }

    __shared__ T red[NW > 1 ? 2 : 1][NW][2];
    int par = 0;
    const T tau = a.tau;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
        if (64 * s >= (int)K) break;
        for (int kb = 0; kb < 64; kb += B) {
            const int k0 = 64 * s + kb;
            if (k0 >= (int)K) break;
            T sl[MMAX][B];
#pragma unroll
            for (int t = 0; t < MMAX; ++t) {
                if (t < m) {
                    if (ok[t]) load_slice(a.partner + (size_t)pj[t] * Kp + k0, sl[t]);
                    else
#pragma unroll
                        for (int b = 0; b < B; ++b) sl[t][b] = T(0);
                }
            }
#pragma unroll
            for (int b = 0; b < B; ++b) {
                const int kl = kb + b;
                if (k0 + b >= (int)K) break;
                T p = T(0), q = T(0);
#pragma unroll
                for (int t = 0; t < MMAX; ++t) {
                    if (t < m) {
                        p += sl[t][b] * sl[t][b];
                        q += sl[t][b] * e[t];
                    }
                }
                T P = wave_sum(p);
                T Qe = wave_sum(q);
                if constexpr (NW > 1) {
                    if (lane == 0) {
                        red[par][wr][0] = P;
                        red[par][wr][1] = Qe;
                    }
                    __syncthreads();
                    P = T(0);
                    Qe = T(0);
#pragma unroll
                    for (int w = 0; w < NW; ++w) {
                        P += red[par][w][0];
                        Qe += red[par][w][1];
                    }
                    par ^= 1;
                }
                const T old = readlane(own_r[s], kl);
                const T sg = readlane(sig_r[s], kl);
                const T mu = readlane(mu_r[s], kl);
                const T z = readlane(z_r[s >> 1][b & 1], ((s & 1) << 5) + (kl >> 1));
                const T nw = draw_coord(P, Qe + P * old, sg, mu, tau, z, a.sd_is_var);
                const T d = old - nw;
#pragma unroll
                for (int t = 0; t < MMAX; ++t)
                    if (t < m) e[t] += sl[t][b] * d;
                own_r[s] = (lane == kl) ? nw : own_r[s];
            }
        }
    }

    // epilogue: own row, residuals, per-row partial sums
    if (wr == 0) {
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const uint32_t k = 64 * s + lane;
            if (k < K) a.own[(size_t)row * Kp + k] = own_r[s];
        }
    }
    T sq = T(0), tr = T(0);
#pragma unroll
    for (int t = 0; t < MMAX; ++t) {
        if (ok[t]) {
            const uint32_t idx = beg + g + t * G;
            a.E_out[idx] = e[t];
            sq += e[t] * e[t];
            if (a.row_tr) {
                const T r = a.r_this[idx];
                T pr = r - e[t];
                pr = (pr < a.hi) ? pr : a.hi;
                pr = (a.lo < pr) ? pr : a.lo;
                tr += (pr - r) * (pr - r);
            }
        }
    }
    if (a.row_sq || a.row_tr) {
        double dsq = wave_sum((double)sq);
        double dtr = wave_sum((double)tr);
        if constexpr (NW > 1) {
            __shared__ double red2[NW][2];
            if (lane == 0) {
                red2[wr][0] = dsq;
                red2[wr][1] = dtr;
            }
            __syncthreads();
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
}

// ------------------------------------------------------------------ Gram route
constexpr int GT = 128;  // Gram tile edge (K padded to 16 inside)
constexpr int GSUB = 32; // ratings staged per LDS sub-chunk

// One block per (chunk, tile_i, tile_j) with tile_i >= tile_j.  256 threads as
// 16x16, each owning an 8x8 sub-grid of the 128x128 tile.  slab layout per
// chunk: [Kt*Kt G (row-major) | Kt b].
template <typename T>
__global__ __launch_bounds__(256) void k_gram_partial(const GramItem* __restrict__ items, HalfArgs<T> a,
                                                       double* __restrict__ slabs, uint32_t Kt, uint32_t ntile) {
    const uint32_t npair = ntile * (ntile + 1) / 2;
    const uint32_t it = blockIdx.x / npair;
    uint32_t pr = blockIdx.x % npair, ti = 0;
    while (pr > ti) { pr -= ti + 1; ++ti; }
    const uint32_t tj = pr;
    const GramItem w = items[it];
    const uint32_t K = a.K, Kp = a.Kp;
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    __shared__ T As[GSUB][GT];
    __shared__ T Bs[GSUB][GT];
    __shared__ T es[GSUB];
    __shared__ T ownS[256];
    for (uint32_t k = threadIdx.x; k < 256; k += 256) ownS[k] = (k < K) ? a.own[(size_t)w.row * Kp + k] : T(0);
    double acc[8][8];
    double bacc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        bacc[i] = 0.0;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = 0.0;
    }
    const uint32_t ci = ti * GT, cj = tj * GT;
    for (uint32_t s0 = 0; s0 < w.len; s0 += GSUB) {
        __syncthreads();
        const uint32_t ns = min((uint32_t)GSUB, w.len - s0);
        // stage: thread -> (rating r = tid / 8, 16-col segment c = tid % 8) for both tiles
        for (uint32_t x = threadIdx.x; x < GSUB * (GT / 16); x += 256) {
            const uint32_t r = x / (GT / 16), c = (x % (GT / 16)) * 16;
            const bool v = r < ns;
            const uint32_t pj = v ? a.part[w.beg + s0 + r] : 0u;
            const T* src = a.partner + (size_t)pj * Kp;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const uint32_t ka = ci + c + q, kb = cj + c + q;
                As[r][c + q] = (v && ka < K) ? src[ka] : T(0);
                Bs[r][c + q] = (v && kb < K) ? src[kb] : T(0);
            }
        }
        if (threadIdx.x < GSUB) {
            const uint32_t r = threadIdx.x;
            T ev = T(0);
            if (r < ns) {
                const uint32_t idx = w.beg + s0 + r;
                if (a.e_from_dot) {
                    const T* src = a.partner + (size_t)a.part[idx] * Kp;
                    T d = T(0);
                    for (uint32_t k = 0; k < K; ++k) d += src[k] * ownS[k];
                    ev = a.r_this[idx] - d;
                } else {
                    ev = a.E_in[a.perm[idx]];
                }
            }
            es[r] = ev;
        }
        __syncthreads();
        for (uint32_t r = 0; r < ns; ++r) {
            T av[8], bv[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) av[i] = As[r][ty + 16 * i];
#pragma unroll
            for (int j = 0; j < 8; ++j) bv[j] = Bs[r][tx + 16 * j];
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 8; ++j) acc[i][j] += (double)(av[i] * bv[j]);
            if (tj == 0 && tx == 0) {
                const T ev = es[r];
#pragma unroll
                for (int i = 0; i < 8; ++i) bacc[i] += (double)(av[i] * ev);
            }
        }
    }
    double* slab = slabs + (size_t)w.slab * ((size_t)Kt * Kt + Kt);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t gi = ci + ty + 16 * i;
        if (gi >= Kt) continue;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t gj = cj + tx + 16 * j;
            if (gj < Kt) slab[(size_t)gi * Kt + gj] = acc[i][j];
        }
        if (tj == 0 && tx == 0) slab[(size_t)Kt * Kt + gi] = bacc[i];
    }
}

// One block (256 threads) per heavy row: fixed-order slab reduction into
// gsum (global, [Kt*Kt + Kt] per row), then one wave runs the recurrence.
template <typename T, int KS>
__global__ __launch_bounds__(256) void k_gram_solve(const GramRow* __restrict__ grows, const double* __restrict__ slabs,
                                                     double* __restrict__ gsum, T* __restrict__ delta, HalfArgs<T> a,
                                                     uint32_t Kt) {
    const GramRow gr = grows[blockIdx.x];
    const size_t SL = (size_t)Kt * Kt + Kt;
    double* Gs = gsum + (size_t)blockIdx.x * SL;
    const uint32_t K = a.K, Kp = a.Kp;
    // lower triangle + diagonal + b only
    for (size_t x = threadIdx.x; x < SL; x += 256) {
        const uint32_t gi = (uint32_t)(x / Kt), gj = (uint32_t)(x % Kt);
        if (x < (size_t)Kt * Kt && (gj > gi || gi >= K)) continue;
        double s = 0.0;
        for (uint32_t c = 0; c < gr.nslab; ++c) s += slabs[(size_t)(gr.slab0 + c) * SL + x];
        Gs[x] = s;
    }
    __syncthreads();
    __threadfence_block();
    if (threadIdx.x >= 64) return;
    const int lane = threadIdx.x;
    const uint32_t row = gr.row;
    constexpr int ZS = (KS + 1) / 2;
    T own_r[KS], sig_r[KS], mu_r[KS], dl[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
        const uint32_t k = 64 * s + lane;
        own_r[s] = k < K ? a.own[(size_t)row * Kp + k] : T(0);
        sig_r[s] = k < K ? a.sig[k] : T(0);
        mu_r[s] = k < K ? a.mu[k] : T(0);
        dl[s] = T(0);
    }
    T z_r[ZS][2];
#pragma unroll
    for (int zs = 0; zs < ZS; ++zs) {
        const uint32_t i0 = 128 * zs + 2 * lane;
        if (a.zbuf) {
            z_r[zs][0] = i0 < K ? a.zbuf[(size_t)row * K + i0] : T(0);
            z_r[zs][1] = i0 + 1 < K ? a.zbuf[(size_t)row * K + i0 + 1] : T(0);
        } else {
            double z0, z1;
            philox_normal_pair(a.seed, row, a.sweep, a.tag, 64 * zs + lane, z0, z1);
            z_r[zs][0] = (T)z0;
            z_r[zs][1] = (T)z1;
        }
    }
    const double* bvec = Gs + (size_t)Kt * Kt;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
        for (int kl = 0; kl < 64; ++kl) {
            const uint32_t k = 64 * s + kl;
            if (k >= K) break;
            // dot = sum_{l<k} G_kl D_l
            double part = 0.0;
#pragma unroll
            for (int s2 = 0; s2 < KS; ++s2) {
                const uint32_t l = 64 * s2 + lane;
                if (l < k) part += Gs[(size_t)k * Kt + l] * (double)dl[s2];
            }
            const double dot = wave_sum(part);
            const T P = (T)Gs[(size_t)k * Kt + k];
            const T old = readlane(own_r[s], kl);
            const T Q = (T)(bvec[k] - dot) + P * old;
            const T sg = readlane(sig_r[s], kl), mu = readlane(mu_r[s], kl);
            const T z = readlane(z_r[s >> 1][kl & 1], ((s & 1) << 5) + (kl >> 1));
            const T nw = draw_coord(P, Q, sg, mu, a.tau, z, a.sd_is_var);
            own_r[s] = (lane == kl) ? nw : own_r[s];
            dl[s] = (lane == kl) ? (nw - old) : dl[s];
        }
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) {
        const uint32_t k = 64 * s + lane;
        if (k < K) {
            a.own[(size_t)row * Kp + k] = own_r[s];
            delta[(size_t)blockIdx.x * Kp + k] = dl[s];
        }
    }
    if (lane == 0) {
        if (a.row_sq) a.row_sq[row] = 0.0;  // heavy rows report through chunk_sq
        if (a.row_tr) a.row_tr[row] = 0.0;
    }
}

// e = r - S u_new  (or e0 - S delta when no ratings array), one thread per rating.
template <typename T>
__global__ __launch_bounds__(256) void k_gram_update(const GramItem* __restrict__ items, HalfArgs<T> a,
                                                      double* __restrict__ chunk_sq, double* __restrict__ chunk_tr) {
    const GramItem w = items[blockIdx.x];
    const uint32_t K = a.K, Kp = a.Kp;
    __shared__ T ownS[256];
    for (uint32_t k = threadIdx.x; k < 256; k += 256) ownS[k] = (k < K) ? a.own[(size_t)w.row * Kp + k] : T(0);
    __syncthreads();
    double sq = 0.0, trs = 0.0;
    for (uint32_t x = threadIdx.x; x < w.len; x += 256) {
        const uint32_t idx = w.beg + x;
        const T* src = a.partner + (size_t)a.part[idx] * Kp;
        T d = T(0);
        for (uint32_t k = 0; k < K; ++k) d += src[k] * ownS[k];
        const T r = a.r_this[idx];
        const T e = r - d;
        a.E_out[idx] = e;
        sq += (double)(e * e);
        if (chunk_tr) {
            T pr = d;
            pr = (pr < a.hi) ? pr : a.hi;
            pr = (a.lo < pr) ? pr : a.lo;
            trs += (double)((pr - r) * (pr - r));
        }
    }
    __shared__ double red[4][2];
    sq = wave_sum(sq);
    trs = wave_sum(trs);
    if ((threadIdx.x & 63) == 0) {
        red[threadIdx.x >> 6][0] = sq;
        red[threadIdx.x >> 6][1] = trs;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        chunk_sq[w.slab] = red[0][0] + red[1][0] + red[2][0] + red[3][0];
        if (chunk_tr) chunk_tr[w.slab] = red[0][1] + red[1][1] + red[2][1] + red[3][1];
    }
}

// Heavy rows: fold chunk partial sums into the per-row arrays (chunk order).
__global__ __launch_bounds__(64) void k_gram_rowsum(const GramRow* __restrict__ grows, uint32_t ngrows,
                                                     const double* __restrict__ chunk_sq,
                                                     const double* __restrict__ chunk_tr, double* __restrict__ row_sq,
                                                     double* __restrict__ row_tr) {
    const uint32_t h = blockIdx.x * 64 + threadIdx.x;
    if (h >= ngrows) return;
    const GramRow gr = grows[h];
    double s = 0.0, t = 0.0;
    for (uint32_t c = 0; c < gr.nslab; ++c) {
        s += chunk_sq[gr.slab0 + c];
        if (chunk_tr) t += chunk_tr[gr.slab0 + c];
    }
    if (row_sq) row_sq[gr.row] = s;
    if (row_tr) row_tr[gr.row] = t;
}

// ------------------------------------------------------------------ residual recompute
template <typename T>
__global__ __launch_bounds__(256) void k_resid(const uint32_t* __restrict__ ptr, const uint32_t* __restrict__ part,
                                                const T* __restrict__ r, const T* __restrict__ own,
                                                const T* __restrict__ partner, uint32_t K, uint32_t Kp, uint32_t r0,
                                                uint32_t r1, T* __restrict__ E, double* __restrict__ row_sq) {
    const uint32_t row = r0 + blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= r1) return;
    const uint32_t beg = ptr[row], end = ptr[row + 1];
    const T* o = own + (size_t)row * Kp;
    double sq = 0.0;
    for (uint32_t idx = beg + lane; idx < end; idx += 64) {
        const T* src = partner + (size_t)part[idx] * Kp;
        T d = T(0);
        for (uint32_t k = 0; k < K; ++k) d += o[k] * src[k];
        const T e = r[idx] - d;
        E[idx] = e;
        sq += (double)(e * e);
    }
    sq = wave_sum(sq);
    if (lane == 0) row_sq[row] = sq;
}

// ------------------------------------------------------------------ column statistics
template <typename T>
__global__ __launch_bounds__(256) void k_colstats(const T* __restrict__ tab, uint32_t K, uint32_t Kp, uint32_t r0,
                                                   uint32_t r1, const T* __restrict__ mu, double* __restrict__ out) {
    const uint32_t c = r0 / 256 + blockIdx.x;  // global chunk index (r0 is chunk aligned)
    const uint32_t rb = c * 256, re = min(rb + 256, r1);
    for (uint32_t k = threadIdx.x; k < K; k += 256) {
        const double m = (double)mu[k];
        double s2 = 0.0, s1 = 0.0;
        for (uint32_t r = max(rb, r0); r < re; ++r) {
            const double x = (double)tab[(size_t)r * Kp + k];
            s2 += (x - m) * (x - m);
            s1 += x;
        }
        out[(size_t)c * 2 * K + k] = s2;
        out[(size_t)c * 2 * K + K + k] = s1;
    }
}

// ------------------------------------------------------------------ test evaluation
template <typename T>
__global__ __launch_bounds__(256) void k_test(const uint32_t* __restrict__ tu, const uint32_t* __restrict__ ti,
                                               const double* __restrict__ tr, uint64_t t0, uint64_t t1,
                                               const T* __restrict__ U, const T* __restrict__ V, uint32_t K,
                                               uint32_t Kp, T lo, T hi, int collect, double div,
                                               double* __restrict__ sum, double* __restrict__ part) {
    const uint64_t t = t0 + (uint64_t)blockIdx.x * 256 + threadIdx.x;
    double a2 = 0.0, t2 = 0.0;
    if (t < t1) {
        const T* u = U + (size_t)tu[t] * Kp;
        const T* v = V + (size_t)ti[t] * Kp;
        T p = T(0);
        for (uint32_t k = 0; k < K; ++k) p += u[k] * v[k];
        p = (p < hi) ? p : hi;
        p = (lo < p) ? p : lo;
        double s = sum[t];
        if (collect) {
            s += (double)p;
            sum[t] = s;
        }
        const double d = tr[t] - s / div;
        a2 = d * d;
        const double dt = tr[t] - (double)p;
        t2 = dt * dt;
    }
    __shared__ double red[4][2];
    a2 = wave_sum(a2);
    t2 = wave_sum(t2);
    if ((threadIdx.x & 63) == 0) {
        red[threadIdx.x >> 6][0] = a2;
        red[threadIdx.x >> 6][1] = t2;
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

__global__ __launch_bounds__(256) void k_sum_cols(const double* __restrict__ in, uint32_t nchunk, uint32_t width,
                                                   double* __restrict__ out) {
    const uint32_t w = blockIdx.x * 256 + threadIdx.x;
    if (w >= width) return;
    double s = 0.0;
    for (uint32_t c = 0; c < nchunk; ++c) s += in[(size_t)c * width + w];
    out[w] = s;
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

}  // namespace

// ===================================================================== launchers
template <typename T, int KS>
static hipError_t launch_rows_ks(int kind, const uint32_t* rows, uint32_t nrows, const HalfArgs<T>& a,
                                 hipStream_t st) {
    if (nrows == 0) return hipSuccess;
    switch (kind) {
        case RK_W2:
            k_rows<T, 2, 1, 4, KS><<<(nrows + 3) / 4, 256, 0, st>>>(rows, nrows, a);
            break;
        case RK_W8:
            k_rows<T, 8, 1, 4, KS><<<(nrows + 3) / 4, 256, 0, st>>>(rows, nrows, a);
            break;
        case RK_B4:
            k_rows<T, 8, 4, 1, KS><<<nrows, 256, 0, st>>>(rows, nrows, a);
            break;
        case RK_B8:
            k_rows<T, 8, 8, 1, KS><<<nrows, 512, 0, st>>>(rows, nrows, a);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <typename T>
hipError_t launch_rows(int kind, const uint32_t* rows, uint32_t nrows, const HalfArgs<T>& a, hipStream_t st) {
    if (a.K <= 64) return launch_rows_ks<T, 1>(kind, rows, nrows, a, st);
    if (a.K <= 128) return launch_rows_ks<T, 2>(kind, rows, nrows, a, st);
    if (a.K <= 256) return launch_rows_ks<T, 4>(kind, rows, nrows, a, st);
    return hipErrorInvalidValue;
}

template <typename T>
hipError_t launch_gram(const GramItem* items, uint32_t nitems, const GramRow* grows, uint32_t ngrows, double* slabs,
                       T* delta, double* chunk_sq, double* chunk_tr, const HalfArgs<T>& a, hipStream_t st) {
    if (nitems == 0) return hipSuccess;
    const uint32_t Kt = (a.K + 15) / 16 * 16;
    const uint32_t ntile = (Kt + GT - 1) / GT;
    const uint32_t npair = ntile * (ntile + 1) / 2;
    k_gram_partial<T><<<nitems * npair, 256, 0, st>>>(items, a, slabs, Kt, ntile);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) return err;
    double* gsum = slabs + (size_t)nitems * ((size_t)Kt * Kt + Kt);
    if (a.K <= 64)
        k_gram_solve<T, 1><<<ngrows, 256, 0, st>>>(grows, slabs, gsum, delta, a, Kt);
    else if (a.K <= 128)
        k_gram_solve<T, 2><<<ngrows, 256, 0, st>>>(grows, slabs, gsum, delta, a, Kt);
    else
        k_gram_solve<T, 4><<<ngrows, 256, 0, st>>>(grows, slabs, gsum, delta, a, Kt);
    err = hipGetLastError();
    if (err != hipSuccess) return err;
    k_gram_update<T><<<nitems, 256, 0, st>>>(items, a, chunk_sq, chunk_tr);
    err = hipGetLastError();
    if (err != hipSuccess) return err;
    if (a.row_sq || a.row_tr)
        k_gram_rowsum<<<(ngrows + 63) / 64, 64, 0, st>>>(grows, ngrows, chunk_sq, a.row_tr ? chunk_tr : nullptr,
                                                           a.row_sq, a.row_tr);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_resid(const uint32_t* ptr, const uint32_t* part, const T* r, const T* own, const T* partner,
                        uint32_t K, uint32_t Kp, uint32_t r0, uint32_t r1, T* E, double* row_sq, hipStream_t st) {
    if (r1 <= r0) return hipSuccess;
    k_resid<T><<<(r1 - r0 + 3) / 4, 256, 0, st>>>(ptr, part, r, own, partner, K, Kp, r0, r1, E, row_sq);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_colstats(const T* tab, uint32_t K, uint32_t Kp, uint32_t r0, uint32_t r1, const T* mu, double* out,
                           hipStream_t st) {
    if (r1 <= r0) return hipSuccess;
    const uint32_t c0 = r0 / 256, c1 = (r1 + 255) / 256;
    k_colstats<T><<<c1 - c0, 256, 0, st>>>(tab, K, Kp, r0, r1, mu, out);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_test(const uint32_t* tu, const uint32_t* ti, const double* tr, uint64_t t0, uint64_t t1, const T* U,
                       const T* V, uint32_t K, uint32_t Kp, T lo, T hi, int collect, double div, double* sum,
                       double* part, hipStream_t st) {
    if (t1 <= t0) return hipSuccess;
    const uint64_t nb = (t1 - t0 + 255) / 256;
    k_test<T><<<(uint32_t)nb, 256, 0, st>>>(tu, ti, tr, t0, t1, U, V, K, Kp, lo, hi, collect, div, sum, part);
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
    k_sum_cols<<<(width + 255) / 256, 256, 0, st>>>(in, nchunk, width, out);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_init_philox(T* tab, uint32_t K, uint32_t Kp, uint32_t r0, uint32_t r1, double sd, uint64_t seed,
                              uint32_t tag, hipStream_t st) {
    if (r1 <= r0) return hipSuccess;
    k_init_philox<T><<<(r1 - r0 + 3) / 4, 256, 0, st>>>(tab, K, Kp, r0, r1, sd, seed, tag);
    return hipGetLastError();
}

#define SBMF_INST(T)                                                                                                 \
    template hipError_t launch_rows<T>(int, const uint32_t*, uint32_t, const HalfArgs<T>&, hipStream_t);            \
    template hipError_t launch_gram<T>(const GramItem*, uint32_t, const GramRow*, uint32_t, double*, T*, double*,   \
                                       double*, const HalfArgs<T>&, hipStream_t);                                    \
    template hipError_t launch_resid<T>(const uint32_t*, const uint32_t*, const T*, const T*, const T*, uint32_t,     \
                                        uint32_t, uint32_t, uint32_t, T*, double*, hipStream_t);                     \
    template hipError_t launch_colstats<T>(const T*, uint32_t, uint32_t, uint32_t, uint32_t, const T*, double*,     \
                                           hipStream_t);                                                             \
    template hipError_t launch_test<T>(const uint32_t*, const uint32_t*, const double*, uint64_t, uint64_t,         \
                                       const T*, const T*, uint32_t, uint32_t, T, T, int, double, double*, double*, \
                                       hipStream_t);                                                                 \
    template hipError_t launch_init_philox<T>(T*, uint32_t, uint32_t, uint32_t, uint32_t, double, uint64_t,          \
                                              uint32_t, hipStream_t);
SBMF_INST(float)
SBMF_INST(double)

}  // namespace sbmf
