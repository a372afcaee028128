// vbo.hip -- gfx950 kernels of the online variational-Bayes learner
// (`sbmf -method vb`; the reference's fm_learn_vb_online on rating data).
//
// The work unit is an attribute row of one batch: a user (or an item) and the
// batch's cases that carry it.  A group of G lanes owns a row, G the power of
// two (1..256) that covers the row's cases VB_CASES_PER_LANE per lane, so a
// 256-thread block holds up to 256 short user rows or one popular item; longer
// rows loop.  Each block reads a task {first row, rows, log2 G} built on the
// host.  The row's natural-parameter sums are fixed-order group reductions.
// A case's residual e and variance term t travel as one 16-byte {e, t}
// record, kept in ONE copy in the batch's user-grouped order.  A user pass
// reads its rows' records (consecutive lanes, consecutive records), keeps
// them in registers between the row's two traversals (sums, then updates) and
// writes them back in place.  An item pass gathers e through the case's
// user-grouped position (iu[q].x) and the partner user's fresh {mean, variance}
// (VS, one 16-byte record), and writes nothing per case: its e / t updates
// depend on the case only through the user's values, so they are left per
// item (D) and applied by the next user pass -- the same operations in the
// same order as applying them at once.  No pass scatters 16-byte records
// over a batch-sized array (the r03 PMC passes: that scatter and the split
// {mean}/{variance} gathers cost 3-5x the algorithmic bytes in HBM traffic).
// Item factors of column f for the user pass stay in L2.  Every reduction
// has a fixed order, so results are bitwise repeatable run to run.
//
// With x = 1 for every feature the reference's cached sums collapse:
// q - x mu = partner mean, t.q - x^2 sigma = partner variance, t.z - ... =
// partner mean^2 (fm_learn_vb_online.h:729-733,781-784), and the prediction
// 1/2 sum_f (v_u + v_i)^2 - 1/2 sum_f (v_u^2 + v_i^2) = sum_f v_u v_i.  The
// GPU uses the collapsed forms (same values up to rounding).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "vbo.h"

namespace sbmf {
namespace {

constexpr int KBMAX = 16;  // Kp / 16 <= 16 (K <= 256)

// sum over the 16 lanes of a row group, lane 0's value broadcast to the group
__device__ __forceinline__ double sum16(double x) {
    x += __shfl_xor(x, 8, 16);
    x += __shfl_xor(x, 4, 16);
    x += __shfl_xor(x, 2, 16);
    x += __shfl_xor(x, 1, 16);
    return __shfl(x, 0, 16);
}

// fixed-order block sum of 256 threads (every thread gets the total)
__device__ __forceinline__ double block_sum256(double x, double* red);

__device__ __forceinline__ double block_sum256(double x, double* red) {
    red[threadIdx.x] = x;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    const double t = red[0];
    __syncthreads();
    return t;
}

__global__ __launch_bounds__(256) void k_transpose(const double* __restrict__ src, double* __restrict__ dst, uint32_t K,
                                                    uint32_t Kp, uint32_t p) {
    __shared__ double tile[32][33];
    const uint32_t a0 = blockIdx.x * 32, f0 = blockIdx.y * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    for (int j = ty; j < 32; j += 8) {
        const uint32_t f = f0 + j, a = a0 + tx;
        tile[j][tx] = (f < K && a < p) ? src[(size_t)f * p + a] : 0.0;
    }
    __syncthreads();
    for (int j = ty; j < 32; j += 8) {
        const uint32_t a = a0 + j, f = f0 + tx;
        if (a < p && f < K) dst[(size_t)a * Kp + f] = tile[tx][j];
    }
}

// predict_data_and_write_to_eterms + predict_t_and_write_to_qterms
// (fm_learn_vb_online.h:80-310) for the cases of the batch's user rows:
//   e = r - (sum_f v_u v_i + w_u + w_i + mu_0'),
//   t = sum_f (s_u s_i + s_u v_i^2 + s_i v_u^2) + s^w_u + s^w_i + sigma_0'.
__global__ __launch_bounds__(256) void k_predict(const VRow* __restrict__ rows, uint32_t nrows,
                                                  const uint32_t* __restrict__ part,
                                                  const float* __restrict__ r, const double* __restrict__ muT,
                                                  const double* __restrict__ sgT, VBTables tb, uint32_t Kp,
                                                  VBCases ET) {
    const uint32_t ri = blockIdx.x * 16 + (threadIdx.x >> 4);
    const int ci = threadIdx.x & 15;
    if (ri >= nrows) return;  // whole 16-lane groups
    const VRow rw = rows[ri];
    const uint32_t nb = Kp / 16;
    double vu[KBMAX], su[KBMAX];
#pragma unroll
    for (int b = 0; b < KBMAX; ++b) {
        vu[b] = b < (int)nb ? muT[(size_t)rw.attr * Kp + 16 * b + ci] : 0.0;
        su[b] = b < (int)nb ? sgT[(size_t)rw.attr * Kp + 16 * b + ci] : 0.0;
    }
    const double wu = tb.mu_w[rw.attr], swu = tb.sg_w[rw.attr];
    const double mu0 = tb.scal->mu0, sg0 = tb.scal->sg0;
    for (uint32_t x = 0; x < rw.len; ++x) {
        const uint32_t q = rw.start + x;
        const uint32_t pa = part[q];
        double d = 0.0, tv = 0.0;
#pragma unroll
        for (int b = 0; b < KBMAX; ++b) {
            if (b < (int)nb) {
                const double vi = muT[(size_t)pa * Kp + 16 * b + ci], si = sgT[(size_t)pa * Kp + 16 * b + ci];
                d += vu[b] * vi;
                tv += su[b] * si + su[b] * (vi * vi) + si * (vu[b] * vu[b]);
            }
        }
        d = sum16(d);
        tv = sum16(tv);
        if (ci == 0) {
            double2 o;
            o.x = (double)r[q] - (((d + wu) + tb.mu_w[pa]) + mu0);
            o.y = ((tv + swu) + tb.sg_w[pa]) + sg0;
            ET.E[q] = o.x;
            ET.T[q] = o.y;
        }
    }
}

// update_w0 (:586-633): partial sums of the per-case natural mean
// (1 - rho0) nm0 + rho0 N alpha (e + mu0'), 1024 cases per block
__global__ __launch_bounds__(256) void k_w0_partial(VBCases ET, uint32_t B, VBTables tb,
                                                     double* __restrict__ part) {
    __shared__ double red[256];
    const VBScal s = *tb.scal;
    const double cmu = (1 - s.rho0) * s.nm0, kmu = s.rho0 * tb.N * s.alpha;
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const uint32_t c = blockIdx.x * 1024 + threadIdx.x * 4 + u;
        if (c < B) acc += cmu + kmu * (ET.E[c] + s.mu0);
    }
    acc = block_sum256(acc, red);
    if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

__global__ __launch_bounds__(256) void k_w0_final(const double* __restrict__ part, uint32_t nblk, uint32_t B,
                                                   VBTables tb) {
    __shared__ double red[256];
    double acc = 0.0;
    for (uint32_t i = threadIdx.x; i < nblk; i += 256) acc += part[i];
    acc = block_sum256(acc, red);
    if (threadIdx.x == 0) {
        VBScal& s = *tb.scal;
        // every case contributes the same natural precision; their mean is that value
        const double ns = ((1 - s.rho0) * s.ns0) + s.rho0 * (s.sigma_0 + tb.N * s.alpha);
        const double nm = acc / B;
        const double mu = nm / ns, sg = 1.0 / ns;
        s.d_mu0 = s.mu0 - mu;
        s.d_sg0 = sg - s.sg0;
        s.nm0 = nm;
        s.ns0 = ns;
        s.mu0 = mu;
        s.sg0 = sg;
    }
}

// Reduction over a group of G lanes (G = 4..256, block-uniform): butterfly
// shuffles inside a wave, an LDS tree for 128 / 256; lane 0's value is
// returned to every lane, so the result is one fixed-order sum.
__device__ __forceinline__ double gsum(double x, int G, double* red) {
    if (G <= 64) {
        for (int m = G >> 1; m > 0; m >>= 1) x += __shfl_xor(x, m, G);
        return __shfl(x, 0, G);
    }
    // 128 / 256 lanes: each wave's butterfly sum, then the waves' sums in wave order
    // (one barrier pair instead of one per tree level)
    for (int m = 32; m > 0; m >>= 1) x += __shfl_xor(x, m, 64);
    const int w = threadIdx.x >> 6, w0 = (threadIdx.x & ~(G - 1)) >> 6;
    if ((threadIdx.x & 63) == 0) red[w] = x;
    __syncthreads();
    double t = red[w0];
    for (int k = 1; k < G / 64; ++k) t += red[w0 + k];
    __syncthreads();
    return t;
}

constexpr int MC = VB_CASES_PER_LANE;        // user rows: cases a lane keeps in registers between the two passes
constexpr int MI = VB_ITEM_CASES_PER_LANE;   // item rows: cases a lane has in flight
#ifndef SBMF_VB_OCC
#define SBMF_VB_OCC 5  // waves per SIMD the update kernels are compiled for (r03: 6 or 8 slower)
#endif


enum { VB_FUSED = 0, VB_PART = 1 };  // item passes: update here | local sums (several ranks)

// The record an item pass leaves per item for the next user pass (VBItemRec,
// three 16-byte loads): the item's mean and variance of the factor that user
// pass updates (v, s), and the item pass's own e / t updates (dmu, dsg, dm2,
// ok), which the user pass applies to its cases before its sums.  Bias pass
// (update_w :700-708): e += dmu, t += dsg; factor pass fp (update_v :790-798):
// e += h dmu, t += (h1 + h^2) dsg, t += h1 dm2, h and h1 the user's mean and
// variance of factor fp (final since that factor's user pass).  The same
// operations in the same order as applying them in the item pass.
struct IRec {
    double v, s, dmu, dsg, dm2, ok;
};
__device__ __forceinline__ IRec get_rec(const VBItemRec* __restrict__ D, uint32_t i) {
    const double2* p = reinterpret_cast<const double2*>(D + i);
    const double2 a = p[0], b = p[1], c = p[2];
    return IRec{a.x, a.y, b.x, b.y, c.x, c.y};
}
__device__ __forceinline__ void put_rec(VBItemRec* __restrict__ D, uint32_t i, double v, double s, bool ok, double dmu,
                                        double dsg, double dm2) {
    double2* p = reinterpret_cast<double2*>(D + i);
    p[0] = make_double2(v, s);
    p[1] = ok ? make_double2(dmu, dsg) : make_double2(0.0, 0.0);
    p[2] = ok ? make_double2(dm2, 1.0) : make_double2(0.0, 0.0);
}
// the item's mean and variance of factor f (0, 0 past the last factor)
__device__ __forceinline__ double2 item_vs(const VBTables& tb, uint32_t f, uint32_t a) {
    return f < tb.K ? make_double2(tb.mu_v[(size_t)f * tb.p + a], tb.sg_v[(size_t)f * tb.p + a]) : make_double2(0.0, 0.0);
}
template <int PEND>
__device__ __forceinline__ void vb_pending(double2& o, const IRec& d, double hp, double sp) {
    if (d.ok == 0.0) return;
    if (PEND == VB_PEND_W) {
        o.x += d.dmu;
        o.y += d.dsg;
    } else {
        o.x += hp * d.dmu;
        o.y += (sp + hp * hp) * d.dsg;
        o.y += sp * d.dm2;
    }
}

// the block's task: rows [row0, row0 + nrows), 2^lg lanes per row
struct VLane {
    VRow rw;
    uint32_t n, rid;  // rid: the row's index in the row list
    int G, ci;
    bool live;
};
__device__ __forceinline__ VLane vb_lane(const VTask* __restrict__ tasks, const VRow* __restrict__ rows) {
    const VTask tk = tasks[blockIdx.x];
    VLane L;
    L.G = 1 << tk.lg;
    const uint32_t g = threadIdx.x >> tk.lg;
    L.ci = threadIdx.x & (L.G - 1);
    L.live = g < tk.nrows;  // G >= 128 blocks hold one row: always live
    L.rid = tk.row0 + (L.live ? g : 0);
    L.rw = rows[L.rid];
    L.n = L.live ? L.rw.len : 0;
    return L;
}

// update_w (:635-710) of the batch's users, update_w0's deltas applied first
// (the user pass touches every case once); e / t updated in place.
__global__ __launch_bounds__(256, SBMF_VB_OCC) void k_user_w(const VTask* __restrict__ tasks,
                                                             const VRow* __restrict__ rows, VBTables tb,
                                                             VBCases ET) {
    __shared__ double red[256];
    const VLane L = vb_lane(tasks, rows);
    const int G = L.G, ci = L.ci;
    const uint32_t a = L.rw.attr, n = L.n, q0 = L.rw.start;
    const double alpha = tb.scal->alpha, sigma_w = tb.scal->sigma_w;
    const double dm = tb.scal->d_mu0, ds = tb.scal->d_sg0;
    const double md = tb.mu_w[a], sd = tb.sg_w[a], mo = tb.nm_w[a], so = tb.ns_w[a], rho = tb.rho_w[a];
    const double cc = (double)tb.cc[a];
    const double cs = ((1 - rho) * so) + rho * (sigma_w + alpha * cc * 1.0);
    double2 et[MC];
    double e1 = 0.0, e2 = 0.0;
#pragma unroll
    for (int j = 0; j < MC; ++j) {
        const uint32_t x = ci + j * G;
        if (x < n) {
            et[j] = make_double2(ET.E[q0 + x], ET.T[q0 + x]);
            et[j].x = et[j].x + dm;
            et[j].y = et[j].y + ds;
            e1 += ((1 - rho) * mo) + rho * cc * alpha * (et[j].x + md);
            e2 += cs;
        }
    }
    for (uint32_t x = ci + MC * G; x < n; x += G) {  // rows longer than MC * G
        const double e = ET.E[q0 + x] + dm;
        e1 += ((1 - rho) * mo) + rho * cc * alpha * (e + md);
        e2 += cs;
    }
    e1 = gsum(e1, G, red);
    e2 = gsum(e2, G, red);
    if (!L.live) return;  // after the last block-wide reduction
    const uint32_t tw = tb.t_w[a] + n;
    const double nm = e1 / n, ns = e2 / n;
    const double mu = nm / ns;
    double sigma = 1 / ns;
    if (std::isnan(sigma) || std::isinf(sigma)) sigma = sd;
    const bool ok = !(std::isnan(mu) || std::isinf(mu));
    if (ci == 0) {
        tb.t_w[a] = tw;
        tb.rho_w[a] = pow((double)(1 + tw), -0.5);
        tb.nm_w[a] = nm;
        tb.ns_w[a] = ns;
        tb.sg_w[a] = sigma;
        tb.mu_w[a] = ok ? mu : md;
    }
    // the reference reverts a non-finite mean and leaves e, t alone (the w0 deltas stay)
    const double dmu = ok ? md - mu : 0.0, dsg = ok ? sigma - sd : 0.0;
#pragma unroll
    for (int j = 0; j < MC; ++j) {
        const uint32_t x = ci + j * G;
        if (x < n) {
            double2 o = et[j];
            if (ok) {
                o.x += dmu;
                o.y += dsg;
            }
            ET.E[q0 + x] = o.x;
            ET.T[q0 + x] = o.y;
        }
    }
    for (uint32_t x = ci + MC * G; x < n; x += G) {
        double2 o = make_double2(ET.E[q0 + x], ET.T[q0 + x]);
        o.x = o.x + dm;
        o.y = o.y + ds;
        if (ok) {
            o.x += dmu;
            o.y += dsg;
        }
        ET.E[q0 + x] = o.x;
        ET.T[q0 + x] = o.y;
    }
}

// update_v (:712-800) of factor f for the batch's users: per case the item's
// record (its column-f mean and variance, and the previous item pass's
// updates, applied first), then the sums, the update and the user's own
// e / t updates, in place.  VS[row] = the user's new {mean, variance} of f
// (by the user's row in the batch), the record the item pass gathers.
template <int PEND>
__global__ __launch_bounds__(256, SBMF_VB_OCC) void k_user_v(const VTask* __restrict__ tasks,
                                                             const VRow* __restrict__ rows,
                                                             const uint32_t* __restrict__ part, uint32_t f,
                                                             uint32_t fp, VBTables tb,
                                                             const VBItemRec* __restrict__ D, VBCases ET,
                                                             double2* __restrict__ VS) {
    __shared__ double red[256];
    const VLane L = vb_lane(tasks, rows);
    const int G = L.G, ci = L.ci;
    const uint32_t a = L.rw.attr, n = L.n, q0 = L.rw.start, I = tb.I;
    const size_t off = (size_t)f * tb.p;
    double* __restrict__ v = tb.mu_v + off;
    double* __restrict__ s = tb.sg_v + off;
    const double alpha = tb.scal->alpha, svg = tb.sigma_v[f];
    const double md = v[a], sd = s[a], mo = tb.nm_v[off + a], so = tb.ns_v[off + a], rho = tb.rho_v[a];
    const double cc = (double)tb.cc[a];
    double hp = 0.0, sp = 0.0;  // the pending factor's user values
    if (PEND == VB_PEND_V) {
        hp = tb.mu_v[(size_t)fp * tb.p + a];
        sp = tb.sg_v[(size_t)fp * tb.p + a];
    }
    double hh[MC], hs[MC];  // the partners' column-f values, kept for the updates
    double2 et[MC];
    double e1 = 0.0, e2 = 0.0;
    // a lane's cases by unconditional loads, all issued before the sums (a slot past the
    // row reads case 0 and is not summed): per-slot conditional loads were two dependent
    // round trips each
    uint32_t pr[MC];
#pragma unroll
    for (int j = 0; j < MC; ++j) {
        const uint32_t x = ci + j * G;
        const uint32_t xi = x < n ? q0 + x : 0u;
        pr[j] = part[xi];
        et[j] = make_double2(ET.E[xi], ET.T[xi]);
    }
#pragma unroll
    for (int j = 0; j < MC; ++j) {
        const uint32_t x = ci + j * G;
        const IRec r = get_rec(D, pr[j] - I);
        if (x < n) {
            hh[j] = r.v;
            hs[j] = r.s;
            vb_pending<PEND>(et[j], r, hp, sp);
            const double h = r.v;
            e2 += (1 - rho) * so + rho * (svg + alpha * cc * (h * h + r.s));
            e1 += ((1 - rho) * mo) + rho * cc * alpha * (h * (et[j].x + md * h));
        }
    }
    for (uint32_t x = ci + MC * G; x < n; x += G) {  // rows longer than MC * G
        const uint32_t q = q0 + x;
        const IRec r = get_rec(D, part[q] - I);
        const double h = r.v;
        double2 o = make_double2(ET.E[q], ET.T[q]);
        vb_pending<PEND>(o, r, hp, sp);
        e2 += (1 - rho) * so + rho * (svg + alpha * cc * (h * h + r.s));
        e1 += ((1 - rho) * mo) + rho * cc * alpha * (h * (o.x + md * h));
    }
    e1 = gsum(e1, G, red);
    e2 = gsum(e2, G, red);
    if (!L.live) return;
    const double nm = e1 / n, ns = e2 / n;
    const double mu = nm / ns;
    double sigma = 1 / ns;
    if (std::isnan(sigma) || std::isinf(sigma)) sigma = sd;
    const bool ok = !(std::isnan(mu) || std::isinf(mu));
    if (ci == 0) {
        tb.nm_v[off + a] = nm;
        tb.ns_v[off + a] = ns;
        s[a] = sigma;
        v[a] = ok ? mu : md;
        VS[L.rid] = make_double2(ok ? mu : md, sigma);
        if (f == 0) tb.t_v[a] += n;  // the caller's count (:447-450)
    }
    // a non-finite mean: the reference returns before touching e, t
    const double dmu = ok ? md - mu : 0.0, dsg = ok ? sigma - sd : 0.0, dm2 = ok ? mu * mu - md * md : 0.0;
#pragma unroll
    for (int j = 0; j < MC; ++j) {
        const uint32_t x = ci + j * G;
        if (x < n) {
            double2 o = et[j];
            if (ok) {
                const double h = hh[j], h1 = hs[j];
                o.x += h * dmu;
                o.y += (h1 + h * h) * dsg;
                o.y += h1 * dm2;
            }
            ET.E[q0 + x] = o.x;
            ET.T[q0 + x] = o.y;
        }
    }
    for (uint32_t x = ci + MC * G; x < n; x += G) {
        const uint32_t q = q0 + x;
        const IRec r = get_rec(D, part[q] - I);
        double2 o = make_double2(ET.E[q], ET.T[q]);
        vb_pending<PEND>(o, r, hp, sp);
        if (ok) {
            const double h = r.v, h1 = r.s;
            o.x += h * dmu;
            o.y += (h1 + h * h) * dsg;
            o.y += h1 * dm2;
        }
        ET.E[q] = o.x;
        ET.T[q] = o.y;
    }
}

// the last item pass's updates of a batch, applied before the hyperparameter sums
template <int PEND>
__global__ __launch_bounds__(256) void k_user_flush(const VTask* __restrict__ tasks, const VRow* __restrict__ rows,
                                                    const uint32_t* __restrict__ part, uint32_t fp, VBTables tb,
                                                    const VBItemRec* __restrict__ D, VBCases ET) {
    const VLane L = vb_lane(tasks, rows);
    const uint32_t a = L.rw.attr;
    double hp = 0.0, sp = 0.0;
    if (PEND == VB_PEND_V && L.live) {
        hp = tb.mu_v[(size_t)fp * tb.p + a];
        sp = tb.sg_v[(size_t)fp * tb.p + a];
    }
    for (uint32_t x = L.ci; x < L.n; x += L.G) {
        const uint32_t q = L.rw.start + x;
        double2 o = make_double2(ET.E[q], ET.T[q]);
        vb_pending<PEND>(o, get_rec(D, part[q] - tb.I), hp, sp);
        ET.E[q] = o.x;
        ET.T[q] = o.y;
    }
}

// update_w (:635-710) of the batch's items: e gathered from the user-grouped
// records (iu[q].x: a case's position there), read only.  MODE VB_FUSED: the
// update, its deltas to D[item]; VB_PART (several ranks): the row's local
// sums {e1, e2} to sums[VRow.pad].
template <int MODE>
__global__ __launch_bounds__(256, SBMF_VB_OCC) void k_item_wp(const VTask* __restrict__ tasks,
                                                              const VRow* __restrict__ rows,
                                                              const uint2* __restrict__ iu, VBTables tb,
                                                              VBCases ET,
                                                              VBItemRec* __restrict__ D, double2* __restrict__ sums) {
    __shared__ double red[256];
    const VLane L = vb_lane(tasks, rows);
    const int G = L.G, ci = L.ci;
    const uint32_t a = L.rw.attr, n = L.n, q0 = L.rw.start;
    const double alpha = tb.scal->alpha, sigma_w = tb.scal->sigma_w;
    const double md = tb.mu_w[a], sd = tb.sg_w[a], mo = tb.nm_w[a], so = tb.ns_w[a], rho = tb.rho_w[a];
    const double cc = (double)tb.cc[a];
    const double cs = ((1 - rho) * so) + rho * (sigma_w + alpha * cc * 1.0);
    double ev[MI];
#pragma unroll
    for (int j = 0; j < MI; ++j) {
        const uint32_t x = ci + j * G;
        if (x < n) ev[j] = ET.E[iu[q0 + x].x];
    }
    double e1 = 0.0, e2 = 0.0;
#pragma unroll
    for (int j = 0; j < MI; ++j) {
        const uint32_t x = ci + j * G;
        if (x < n) {
            e1 += ((1 - rho) * mo) + rho * cc * alpha * (ev[j] + md);
            e2 += cs;
        }
    }
    for (uint32_t x = ci + MI * G; x < n; x += G) {
        const double e = ET.E[iu[q0 + x].x];
        e1 += ((1 - rho) * mo) + rho * cc * alpha * (e + md);
        e2 += cs;
    }
    e1 = gsum(e1, G, red);
    e2 = gsum(e2, G, red);
    if (!L.live || ci != 0) return;
    if (MODE == VB_PART) {
        sums[L.rw.pad] = make_double2(e1, e2);
        return;
    }
    const uint32_t tw = tb.t_w[a] + n;
    const double nm = e1 / n, ns = e2 / n;
    const double mu = nm / ns;
    double sigma = 1 / ns;
    if (std::isnan(sigma) || std::isinf(sigma)) sigma = sd;
    const bool ok = !(std::isnan(mu) || std::isinf(mu));
    tb.t_w[a] = tw;
    tb.rho_w[a] = pow((double)(1 + tw), -0.5);
    tb.nm_w[a] = nm;
    tb.ns_w[a] = ns;
    tb.sg_w[a] = sigma;
    tb.mu_w[a] = ok ? mu : md;
    const double2 nv = item_vs(tb, 0, a);  // factor 0: the next user pass's
    put_rec(D, a - tb.I, nv.x, nv.y, ok, md - mu, sigma - sd, 0.0);
}

// update_v (:712-800) of factor f for the batch's items: per case e (gathered
// through iu[q].x) and the user's fresh {mean, variance} of f (VS by the user's
// batch row iu[q].y; one 16-byte gather); nothing per case is written.  MODE as
// k_item_wp.
template <int MODE>
__global__ __launch_bounds__(256, SBMF_VB_OCC) void k_item_vp(const VTask* __restrict__ tasks,
                                                              const VRow* __restrict__ rows,
                                                              const uint2* __restrict__ iu, uint32_t f,
                                                              VBTables tb, VBCases ET,
                                                              const double2* __restrict__ VS,
                                                              VBItemRec* __restrict__ D, double2* __restrict__ sums) {
    __shared__ double red[256];
    const VLane L = vb_lane(tasks, rows);
    const int G = L.G, ci = L.ci;
    const uint32_t a = L.rw.attr, n = L.n, q0 = L.rw.start;
    const size_t off = (size_t)f * tb.p;
    double* __restrict__ v = tb.mu_v + off;
    double* __restrict__ s = tb.sg_v + off;
    const double alpha = tb.scal->alpha, svg = tb.sigma_v[f];
    const double md = v[a], sd = s[a], mo = tb.nm_v[off + a], so = tb.ns_v[off + a], rho = tb.rho_v[a];
    const double cc = (double)tb.cc[a];
    double ev[MI];
    double2 hv[MI];
    // unconditional loads, all issued before the sums (a slot past the row reads case 0)
    uint2 cv[MI];
#pragma unroll
    for (int j = 0; j < MI; ++j) {
        const uint32_t x = ci + j * G;
        cv[j] = iu[x < n ? q0 + x : 0u];
    }
#pragma unroll
    for (int j = 0; j < MI; ++j) {
        ev[j] = ET.E[cv[j].x];
        hv[j] = VS[cv[j].y];
    }
    double e1 = 0.0, e2 = 0.0;
#pragma unroll
    for (int j = 0; j < MI; ++j) {
        const uint32_t x = ci + j * G;
        if (x < n) {
            const double h = hv[j].x;
            e2 += (1 - rho) * so + rho * (svg + alpha * cc * (h * h + hv[j].y));
            e1 += ((1 - rho) * mo) + rho * cc * alpha * (h * (ev[j] + md * h));
        }
    }
    for (uint32_t x = ci + MI * G; x < n; x += G) {
        const uint2 c = iu[q0 + x];
        const double e = ET.E[c.x];
        const double2 hw = VS[c.y];
        const double h = hw.x;
        e2 += (1 - rho) * so + rho * (svg + alpha * cc * (h * h + hw.y));
        e1 += ((1 - rho) * mo) + rho * cc * alpha * (h * (e + md * h));
    }
    e1 = gsum(e1, G, red);
    e2 = gsum(e2, G, red);
    if (!L.live || ci != 0) return;
    if (MODE == VB_PART) {
        sums[L.rw.pad] = make_double2(e1, e2);
        return;
    }
    const double nm = e1 / n, ns = e2 / n;
    const double mu = nm / ns;
    double sigma = 1 / ns;
    if (std::isnan(sigma) || std::isinf(sigma)) sigma = sd;
    const bool ok = !(std::isnan(mu) || std::isinf(mu));
    tb.nm_v[off + a] = nm;
    tb.ns_v[off + a] = ns;
    s[a] = sigma;
    v[a] = ok ? mu : md;
    if (f == 0) tb.t_v[a] += n;
    const double2 nv = item_vs(tb, f + 1, a);
    put_rec(D, a - tb.I, nv.x, nv.y, ok, md - mu, sigma - sd, mu * mu - md * md);
}

// Several ranks (or one rank's XCD slices): one thread per item g of the
// batch's item list; its partial sums (recv[r][g], r = rank or slice, in order,
// the parts present in VGItem.mask), its case count,
// then exactly k_item_vp / k_item_wp's update; the deltas go to D[item] for
// the next user pass.  Identical inputs on every rank, so identical results.
__global__ __launch_bounds__(256) void k_item_v(const VGItem* __restrict__ gi, uint32_t nG,
                                                 const double2* __restrict__ recv, int R, uint32_t f, VBTables tb,
                                                 VBItemRec* __restrict__ D) {
    const uint32_t g = blockIdx.x * 256 + threadIdx.x;
    if (g >= nG) return;
    const uint32_t a = gi[g].attr, n = gi[g].n;
    double e1 = 0.0, e2 = 0.0;
    for (int r = 0; r < R; ++r)
        if (gi[g].mask >> r & 1u) {  // r < 32: vbo.cpp refuses more ranks
            e1 += recv[(size_t)r * nG + g].x;
            e2 += recv[(size_t)r * nG + g].y;
        }
    const size_t off = (size_t)f * tb.p;
    double* __restrict__ v = tb.mu_v + off;
    double* __restrict__ s = tb.sg_v + off;
    const double md = v[a], sd = s[a];
    const double nm = e1 / n, ns = e2 / n;
    const double mu = nm / ns;
    double sigma = 1 / ns;
    if (std::isnan(sigma) || std::isinf(sigma)) sigma = sd;
    const bool ok = !(std::isnan(mu) || std::isinf(mu));
    tb.nm_v[off + a] = nm;
    tb.ns_v[off + a] = ns;
    s[a] = sigma;
    v[a] = ok ? mu : md;
    if (f == 0) tb.t_v[a] += n;
    const double2 nv = item_vs(tb, f + 1, a);
    put_rec(D, a - tb.I, nv.x, nv.y, ok, md - mu, sigma - sd, mu * mu - md * md);
}
__global__ __launch_bounds__(256) void k_item_w(const VGItem* __restrict__ gi, uint32_t nG,
                                                 const double2* __restrict__ recv, int R, VBTables tb,
                                                 VBItemRec* __restrict__ D) {
    const uint32_t g = blockIdx.x * 256 + threadIdx.x;
    if (g >= nG) return;
    const uint32_t a = gi[g].attr, n = gi[g].n;
    double e1 = 0.0, e2 = 0.0;
    for (int r = 0; r < R; ++r)
        if (gi[g].mask >> r & 1u) {  // r < 32: vbo.cpp refuses more ranks
            e1 += recv[(size_t)r * nG + g].x;
            e2 += recv[(size_t)r * nG + g].y;
        }
    const double md = tb.mu_w[a], sd = tb.sg_w[a];
    const uint32_t tw = tb.t_w[a] + n;
    const double nm = e1 / n, ns = e2 / n;
    const double mu = nm / ns;
    double sigma = 1 / ns;
    if (std::isnan(sigma) || std::isinf(sigma)) sigma = sd;
    const bool ok = !(std::isnan(mu) || std::isinf(mu));
    tb.t_w[a] = tw;
    tb.rho_w[a] = pow((double)(1 + tw), -0.5);
    tb.nm_w[a] = nm;
    tb.ns_w[a] = ns;
    tb.sg_w[a] = sigma;
    tb.mu_w[a] = ok ? mu : md;
    const double2 nv = item_vs(tb, 0, a);
    put_rec(D, a - tb.I, nv.x, nv.y, ok, md - mu, sigma - sd, 0.0);
}

// fixed-order sum of n doubles into out[0] (one block)
__global__ __launch_bounds__(256) void k_sum_fixed(const double* __restrict__ in, uint32_t n, double* __restrict__ out) {
    __shared__ double red[256];
    double acc = 0.0;
    for (uint32_t i = threadIdx.x; i < n; i += 256) acc += in[i];
    acc = block_sum256(acc, red);
    if (threadIdx.x == 0) out[0] = acc;
}
// out[r] = sum over c of part[r * nchunk + c], in chunk order (rows r <= K)
__global__ __launch_bounds__(256) void k_fold_rows(const double* __restrict__ part, uint32_t nrow, uint32_t nchunk,
                                                    double* __restrict__ out) {
    const uint32_t r = blockIdx.x * 256 + threadIdx.x;
    if (r >= nrow) return;
    double t = 0.0;
    for (uint32_t c = 0; c < nchunk; ++c) t += part[(size_t)r * nchunk + c];
    out[r] = t;
}
// every rank's [alpha sum | K + 1 user-range sig sums] (recv, rank order) plus the
// item range's sig sums (replicated) -> out = [alpha sum | K + 1 sig sums]
__global__ __launch_bounds__(256) void k_vb_combine(const double* __restrict__ recv, int R, uint32_t K,
                                                     const double* __restrict__ items, double* __restrict__ out) {
    const uint32_t x = blockIdx.x * 256 + threadIdx.x;
    const uint32_t W = K + 2;
    if (x >= W) return;
    double t = 0.0;
    for (int r = 0; r < R; ++r) t += recv[(size_t)r * W + x];
    out[x] = x == 0 ? t : t + items[x - 1];
}

__global__ __launch_bounds__(256) void k_rho_v(VBTables tb) {
    const uint32_t a = blockIdx.x * 256 + threadIdx.x;
    if (a < tb.p) tb.rho_v[a] = pow((double)(1 + tb.t_v[a]), -0.5);
}

// alpha's sum of e^2 + t over the batch, 1024 cases per block
__global__ __launch_bounds__(256) void k_alpha_partial(VBCases ET, uint32_t B,
                                                        double* __restrict__ part) {
    __shared__ double red[256];
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const uint32_t c = blockIdx.x * 1024 + threadIdx.x * 4 + u;
        if (c < B) acc += ET.E[c] * ET.E[c] + ET.T[c];
    }
    acc = block_sum256(acc, red);
    if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

// sum over the attributes [a0, a1) of mean^2 + variance: row r < K = factor r, r == K = bias
__global__ __launch_bounds__(256) void k_sig_partial(VBTables tb, uint32_t a0, uint32_t a1, double* __restrict__ part,
                                                      uint32_t nchunk) {
    __shared__ double red[256];
    const uint32_t r = blockIdx.y, c = blockIdx.x;
    const double* m = r < tb.K ? tb.mu_v + (size_t)r * tb.p : tb.mu_w;
    const double* v = r < tb.K ? tb.sg_v + (size_t)r * tb.p : tb.sg_w;
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        const uint32_t a = a0 + c * 2048 + u * 256 + threadIdx.x;
        if (a < a1) acc += m[a] * m[a] + v[a];
    }
    acc = block_sum256(acc, red);
    if (threadIdx.x == 0) part[(size_t)r * nchunk + c] = acc;
}

// the blends of :523-580; a NaN / inf alpha reverts and skips the rest, as the reference returns
__global__ __launch_bounds__(256) void k_hyper_final(const double* __restrict__ apart, uint32_t nab,
                                                      const double* __restrict__ spart, uint32_t nchunk, uint32_t B,
                                                      VBTables tb) {
    __shared__ double red[256];
    __shared__ int skip;
    double acc = 0.0;
    for (uint32_t i = threadIdx.x; i < nab; i += 256) acc += apart[i];
    acc = block_sum256(acc, red);
    VBScal& s = *tb.scal;
    const double rho0 = s.rho0;
    if (threadIdx.x == 0) {
        const double alpha = (1 - rho0) * s.alpha + rho0 * ((double)B / acc);
        skip = std::isnan(alpha) || std::isinf(alpha);
        if (skip)
            s.n_skip += 1;
        else
            s.alpha = alpha;
    }
    __syncthreads();
    if (skip) return;
    const double pd = (double)tb.p;
    for (uint32_t r = threadIdx.x; r <= tb.K; r += 256) {
        double t = 0.0;
        for (uint32_t c = 0; c < nchunk; ++c) t += spart[(size_t)r * nchunk + c];
        if (r < tb.K)
            tb.sigma_v[r] = (1 - rho0) * tb.sigma_v[r] + rho0 * (pd / t);
        else
            red[0] = t;  // bias sum, read by thread 0 below
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        s.sigma_0 = (1 - rho0) * s.sigma_0 + rho0 * (1.0 / (s.mu0 * s.mu0 + s.sg0));
        s.sigma_w = (1 - rho0) * s.sigma_w + rho0 * (pd / red[0]);
        s.t_w0 += 1;
        s.rho0 = pow((double)(1 + s.t_w0), -0.5);
    }
}

// test predictions: 16 lanes per case, 256 cases per block
__global__ __launch_bounds__(256) void k_test(const uint32_t* __restrict__ tu, const uint32_t* __restrict__ ti,
                                               const double* __restrict__ tr, uint64_t n, uint32_t I,
                                               const double* __restrict__ muT, VBTables tb, uint32_t Kp, double lo,
                                               double hi, double* __restrict__ pred, double* __restrict__ part) {
    __shared__ double red[256];
    const int g = threadIdx.x >> 4, ci = threadIdx.x & 15;
    const uint32_t nb = Kp / 16;
    const double mu0 = tb.scal->mu0;
    double se = 0.0;
    for (int m = 0; m < 16; ++m) {
        const uint64_t c = (uint64_t)blockIdx.x * 256 + g + 16 * m;
        if (c >= n) break;  // uniform per group
        const uint32_t u = tu[c], it = I + ti[c];
        double d = 0.0;
        for (uint32_t b = 0; b < nb; ++b) d += muT[(size_t)u * Kp + 16 * b + ci] * muT[(size_t)it * Kp + 16 * b + ci];
        d = sum16(d);
        double p = ((d + tb.mu_w[u]) + tb.mu_w[it]) + mu0;
        p = (p < hi) ? p : hi;  // std::min(max_target, p), std::max(min_target, p)
        p = (lo < p) ? p : lo;
        if (ci == 0) {
            pred[c] = p;
            const double err = p - (double)(float)tr[c];
            se += err * err;
        }
    }
    se = block_sum256(se, red);
    if (threadIdx.x == 0) part[blockIdx.x] = se;
}

}  // namespace

hipError_t vbo_transpose(const double* src, double* dst, uint32_t K, uint32_t Kp, uint32_t p, hipStream_t st) {
    if (p == 0 || K == 0) return hipSuccess;
    k_transpose<<<dim3((p + 31) / 32, (K + 31) / 32), 256, 0, st>>>(src, dst, K, Kp, p);
    return hipGetLastError();
}

hipError_t vbo_predict(const VRow* rows, uint32_t nrows, const uint32_t* part, const float* r, const double* muT,
                       const double* sgT, const VBTables& tb, uint32_t Kp, VBCases ET, hipStream_t st) {
    if (nrows == 0) return hipSuccess;
    if (Kp > 16 * KBMAX) return hipErrorInvalidValue;
    k_predict<<<(nrows + 15) / 16, 256, 0, st>>>(rows, nrows, part, r, muT, sgT, tb, Kp, ET);
    return hipGetLastError();
}

hipError_t vbo_update_w0(VBCases ET, uint32_t B, const VBTables& tb, double* part, hipStream_t st) {
    if (B == 0) return hipErrorInvalidValue;
    const uint32_t nblk = (B + 1023) / 1024;
    k_w0_partial<<<nblk, 256, 0, st>>>(ET, B, tb, part);
    k_w0_final<<<1, 256, 0, st>>>(part, nblk, B, tb);
    return hipGetLastError();
}

hipError_t vbo_user_w(const VTask* tasks, uint32_t ntask, const VRow* rows, const VBTables& tb, VBCases ET,
                      hipStream_t st) {
    if (ntask == 0) return hipSuccess;
    k_user_w<<<ntask, 256, 0, st>>>(tasks, rows, tb, ET);
    return hipGetLastError();
}

hipError_t vbo_user_v(const VTask* tasks, uint32_t ntask, const VRow* rows, const uint32_t* part, uint32_t f, int pend,
                      uint32_t fp, const VBTables& tb, const VBItemRec* D, VBCases ET, double2* VS, hipStream_t st) {
    if (ntask == 0) return hipSuccess;
    // every user pass follows an item pass, whose records carry the column-f values
    if (pend == VB_PEND_V)
        k_user_v<VB_PEND_V><<<ntask, 256, 0, st>>>(tasks, rows, part, f, fp, tb, D, ET, VS);
    else if (pend == VB_PEND_W)
        k_user_v<VB_PEND_W><<<ntask, 256, 0, st>>>(tasks, rows, part, f, fp, tb, D, ET, VS);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t vbo_user_flush(const VTask* tasks, uint32_t ntask, const VRow* rows, const uint32_t* part, int pend,
                          uint32_t fp, const VBTables& tb, const VBItemRec* D, VBCases ET, hipStream_t st) {
    if (ntask == 0 || pend == VB_PEND_NONE) return hipSuccess;
    if (pend == VB_PEND_V)
        k_user_flush<VB_PEND_V><<<ntask, 256, 0, st>>>(tasks, rows, part, fp, tb, D, ET);
    else
        k_user_flush<VB_PEND_W><<<ntask, 256, 0, st>>>(tasks, rows, part, fp, tb, D, ET);
    return hipGetLastError();
}

hipError_t vbo_item_w(const VTask* tasks, uint32_t ntask, const VRow* rows, const uint2* iu, const VBTables& tb,
                      VBCases ET, VBItemRec* D, double2* sums, hipStream_t st) {
    if (ntask == 0) return hipSuccess;
    if (sums)
        k_item_wp<VB_PART><<<ntask, 256, 0, st>>>(tasks, rows, iu, tb, ET, D, sums);
    else
        k_item_wp<VB_FUSED><<<ntask, 256, 0, st>>>(tasks, rows, iu, tb, ET, D, sums);
    return hipGetLastError();
}

hipError_t vbo_item_v(const VTask* tasks, uint32_t ntask, const VRow* rows, const uint2* iu, uint32_t f, const VBTables& tb, VBCases ET, const double2* VS, VBItemRec* D, double2* sums,
                      hipStream_t st) {
    if (ntask == 0) return hipSuccess;
    if (sums)
        k_item_vp<VB_PART><<<ntask, 256, 0, st>>>(tasks, rows, iu, f, tb, ET, VS, D, sums);
    else
        k_item_vp<VB_FUSED><<<ntask, 256, 0, st>>>(tasks, rows, iu, f, tb, ET, VS, D, sums);
    return hipGetLastError();
}

hipError_t vbo_item_update(const VGItem* gi, uint32_t nG, const double2* recv, int R, int factor, uint32_t f,
                           const VBTables& tb, VBItemRec* D, hipStream_t st) {
    if (nG == 0) return hipSuccess;
    if (factor)
        k_item_v<<<(nG + 255) / 256, 256, 0, st>>>(gi, nG, recv, R, f, tb, D);
    else
        k_item_w<<<(nG + 255) / 256, 256, 0, st>>>(gi, nG, recv, R, tb, D);
    return hipGetLastError();
}

hipError_t vbo_hyper(VBCases ET, uint32_t B, const VBTables& tb, double* part, hipStream_t st) {
    k_rho_v<<<(tb.p + 255) / 256, 256, 0, st>>>(tb);
    const uint32_t nab = (B + 1023) / 1024, nchunk = (tb.p + 2047) / 2048;
    double* spart = part + nab + 8;
    k_alpha_partial<<<nab, 256, 0, st>>>(ET, B, part);
    k_sig_partial<<<dim3(nchunk, tb.K + 1), 256, 0, st>>>(tb, 0, tb.p, spart, nchunk);
    k_hyper_final<<<1, 256, 0, st>>>(part, nab, spart, nchunk, B, tb);
    return hipGetLastError();
}

// ---- several ranks: local partial sums, then the final steps from every rank's sums
hipError_t vbo_w0_local(VBCases ET, uint32_t B, const VBTables& tb, double* part, double* out, hipStream_t st) {
    if (B == 0) return hipMemsetAsync(out, 0, sizeof(double), st);
    const uint32_t nblk = (B + 1023) / 1024;
    k_w0_partial<<<nblk, 256, 0, st>>>(ET, B, tb, part);
    k_sum_fixed<<<1, 256, 0, st>>>(part, nblk, out);
    return hipGetLastError();
}
hipError_t vbo_w0_final(const double* recv, int R, uint32_t B, const VBTables& tb, hipStream_t st) {
    k_w0_final<<<1, 256, 0, st>>>(recv, (uint32_t)R, B, tb);
    return hipGetLastError();
}
hipError_t vbo_hyper_local(VBCases ET, uint32_t B, const VBTables& tb, uint32_t u0, uint32_t u1, double* part,
                           size_t part_cap, double* out, hipStream_t st) {
    const uint32_t nab = (B + 1023) / 1024;
    if ((size_t)nab + 8 + (size_t)(tb.K + 1) * std::max(1u, (u1 - u0 + 2047) / 2048) > part_cap)
        return hipErrorInvalidValue;  // scratch too small for this layout
    k_rho_v<<<(tb.p + 255) / 256, 256, 0, st>>>(tb);
    if (B) {
        k_alpha_partial<<<nab, 256, 0, st>>>(ET, B, part);
        k_sum_fixed<<<1, 256, 0, st>>>(part, nab, out);
    } else {
        hipError_t e = hipMemsetAsync(out, 0, sizeof(double), st);
        if (e != hipSuccess) return e;
    }
    const uint32_t nchunk = std::max(1u, (u1 - u0 + 2047) / 2048);
    double* spart = part + nab + 8;
    k_sig_partial<<<dim3(nchunk, tb.K + 1), 256, 0, st>>>(tb, u0, u1, spart, nchunk);
    k_fold_rows<<<(tb.K + 1 + 255) / 256, 256, 0, st>>>(spart, tb.K + 1, nchunk, out + 1);
    return hipGetLastError();
}
hipError_t vbo_hyper_final(const double* recv, int R, uint32_t B, const VBTables& tb, uint32_t I, double* part,
                           size_t part_cap, hipStream_t st) {
    // the item range's sums (replicated on every rank), then the combined totals
    const uint32_t nchunk = std::max(1u, (tb.p - I + 2047) / 2048);
    if (vbo_hyper_final_doubles(tb.K, nchunk) > part_cap) return hipErrorInvalidValue;  // layout below
    double* items = part;
    double* spart = part + tb.K + 8;
    double* comb = spart + (size_t)(tb.K + 1) * nchunk + 8;
    k_sig_partial<<<dim3(nchunk, tb.K + 1), 256, 0, st>>>(tb, I, tb.p, spart, nchunk);
    k_fold_rows<<<(tb.K + 1 + 255) / 256, 256, 0, st>>>(spart, tb.K + 1, nchunk, items);
    k_vb_combine<<<(tb.K + 2 + 255) / 256, 256, 0, st>>>(recv, R, tb.K, items, comb);
    k_hyper_final<<<1, 256, 0, st>>>(comb, 1, comb + 1, 1, B, tb);
    return hipGetLastError();
}

hipError_t vbo_test(const uint32_t* tu, const uint32_t* ti, const double* tr, uint64_t n, uint32_t I,
                    const double* muT, const VBTables& tb, uint32_t Kp, double lo, double hi, double* pred,
                    double* part, hipStream_t st) {
    if (n == 0) return hipSuccess;
    k_test<<<(uint32_t)((n + 255) / 256), 256, 0, st>>>(tu, ti, tr, n, I, muT, tb, Kp, lo, hi, pred, part);
    return hipGetLastError();
}

}  // namespace sbmf
