// fmm.hip -- gfx950 kernels of the libFM-order MCMC / ALS learner (fmm.h).
//
// A factor pass is one launch over the attribute rows of one side: a row
// gathers its cases' residuals (its own order, sequential) and the partner
// attribute's value of factor f (column f of the f-major table, L2-resident),
// reduces sum h e and sum h^2 in a fixed order, draws its value, and writes
// every case's updated residual into the other side's order (e_out[perm[q]]),
// which is exactly the order the next pass reads.  The libFM cache q (sum of
// the case's two factor values) is not stored: the user pass rebuilds it as
// v_u + v_i, the item pass as (v_u_old + v_i) - (v_u_old - v_u_new), the
// same operations fm_learn_mcmc.h:385-409 and :826-834 apply to it.
#include <hip/hip_runtime.h>

#include "fmm.h"

namespace sbmf {
namespace {

__device__ __forceinline__ double wsum(double x) {  // xor butterfly: bit-identical in every lane
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) x += __shfl_xor(x, m);
    return x;
}

// The row's draw from its sums m = sum h e, s2 = sum h^2 (fm_learn_mcmc.h:700-719,
// :815-835); keep: a non-finite draw restores the old value (the reference returns).
template <int MODE>
__device__ __forceinline__ double fmm_draw(const FMPassArgs& a, uint32_t at, double old, double m, double s2,
                                           bool& keep) {
    if constexpr (MODE == 1) m -= old * s2;
    s2 = 1.0 / (a.lambda + a.alpha * s2);
    m = -s2 * (a.alpha * m - a.mu * a.lambda);
    double nv;
    if (isnan(s2) || isinf(s2)) {
        nv = 0.0;
    } else if (a.do_sample) {  // ran_gaussian(mean, stdev), random.h:166-172
        const double sd = sqrt(s2);
        nv = (sd == 0.0 || isnan(sd)) ? m : m + sd * a.z[(size_t)at * a.zs + a.zoff];
    } else {
        nv = m;
    }
    keep = isnan(nv) || isinf(nv);
    return keep ? old : nv;
}

// MODE 0: draw_w (fm_learn_mcmc.h:670-719); MODE 1: draw_v (:780-835).
// NT threads per row; a 256-thread block holds 256 / NT rows (NT <= 256) or
// one row (NT = 1024).
template <int MODE, int NT, bool IP>
__global__ __launch_bounds__(NT > 256 ? NT : 256) void k_fmm_pass(FMPassArgs a) {
    constexpr int RPB = NT >= 256 ? 1 : 256 / NT;
    constexpr int NWR = NT >= 64 ? NT / 64 : 1;  // waves per row
    const int sub = threadIdx.x / NT, lt = threadIdx.x % NT;
    const uint32_t ri = blockIdx.x * RPB + sub;
    if (NT == 64 && ri >= a.nrows) return;  // a whole wave: no block barriers on this path
    uint32_t row, beg, n, di;  // di: the row's slot in sums / delta
    if (a.chunks) {            // a chunk of a long row (one rank)
        const uint4 ck = a.chunks[ri];
        row = ck.x;
        beg = ck.y;
        n = ck.z;
        di = ck.w;
    } else {
        row = a.rows[ri];
        beg = a.ptr[row];
        n = a.ptr[row + 1] - beg;
        di = row;
    }
    const uint32_t at = a.a0 + row;
    const int xm = a.xmode;
    const double4 dl = xm == 2 ? a.delta[di] : make_double4(0.0, 0.0, 0.0, 0.0);
    const double old = xm == 2 ? dl.x : a.own[at];
    const float x = 1.0f;  // one-hot value (DATA_FLOAT)
    // IP: this user's values of the factor of the item pass to be applied on read
    double qo = 0.0, qn = 0.0;
    if constexpr (IP) {
        if (a.pend == 2 && !a.item_side) {
            if (xm == 2) {  // chunks: the draw has replaced the record, its old one kept in qq
                const double2 r = a.qq[di];
                qo = r.x;
                qn = r.y;
            } else {
                const double2 r = a.rec[at];
                qo = r.x;
                qn = r.y;
            }
        }
    }
    // IP: the other side's last pass applied to case q's residual e (its record: old,
    // value kept -- a kept draw records old twice, so its update is e - h * 0 = e), with
    // the h that pass used -- the scatter form's update
    auto pend = [&](uint32_t q, double e) -> double {
        if constexpr (!IP) {
            return e;
        } else {
            if (a.pend == 0) return e;
            const double2 r = a.rec[a.pa0 + a.part[q]];
            double h;
            if (a.pend == 1) {
                h = (double)x;  // a w pass
            } else if (a.item_side) {  // the user pass of this factor: h of its hval
                const double qc = (0.0 + r.x * x) + old * x;
                h = x * (qc - x * r.x);
            } else {  // the item pass of the previous factor: h of its hval
                const double qc = ((0.0 + qo * x) + r.x * x) - x * (qo - qn);
                h = x * (qc - x * r.x);
            }
            // a draw that was not kept recorded {old, old}: leave e alone, as libFM does
            // (e - h * 0 would turn a non-finite h into NaN and can flip a -0.0)
            return r.x == r.y ? e : e - h * (r.x - r.y);
        }
    };
    // h of the case at position q (factor pass): x * (q_c - x * v) with the
    // case's q rebuilt from the factor column (see the file header)
    auto hval = [&](uint32_t q) {
        const uint32_t pr = a.part[q];
        double qc;
        if (a.item_side) {
            double vo, vn;
            if constexpr (IP) {  // the user's record of this factor's user pass
                const double2 r = a.rec[pr];
                vo = r.x;
                vn = r.y;
            } else {
                vo = a.vold_u[pr];
                vn = a.partner_col[pr];
            }
            qc = ((0.0 + vo * x) + old * x) - x * (vo - vn);
        } else {
            qc = (0.0 + old * x) + a.partner_col[a.pa0 + pr] * x;
        }
        return x * (qc - x * old);
    };
    const double* __restrict__ ein = IP ? a.e_io : a.e_in;
    // a lane's first MCF cases stay in registers (residual, h, scatter target) from
    // the sums to the residual update; the rest are reloaded (same values: the pass
    // changes neither h nor e before the update)
    constexpr int MCF = 4;
    double ce[MCF], ch[MCF];
    uint32_t cp[MCF];
    double m = 0.0, s2 = 0.0;
    const uint32_t nsum = xm == 2 ? 0u : n;
#pragma unroll
    for (int j = 0; j < MCF; ++j) {
        const uint32_t k = lt + j * NT;
        ce[j] = 0.0;
        ch[j] = x;
        cp[j] = 0;
        if (k < nsum) {
            const uint32_t q = beg + k;
            const double e = pend(q, ein[q]);
            ce[j] = e;
            cp[j] = IP ? 0u : a.perm[q];
            if constexpr (MODE == 0) {
                m += x * (e - old * x);
                s2 += x * x;
            } else {
                const double h = hval(q);
                ch[j] = h;
                m += h * e;
                s2 += h * h;
            }
        }
    }
    for (uint32_t k = lt + MCF * NT; k < nsum; k += NT) {
        const double e = pend(beg + k, ein[beg + k]);
        if constexpr (MODE == 0) {
            m += x * (e - old * x);
            s2 += x * x;
        } else {
            const double h = hval(beg + k);
            m += h * e;
            s2 += h * h;
        }
    }
    m = wsum(m);
    s2 = wsum(s2);
    if constexpr (NWR > 1) {  // waves of the row meet in LDS, summed in wave order
        __shared__ double red[2][NWR];
        const int w = lt >> 6;
        if ((lt & 63) == 0) {
            red[0][w] = m;
            red[1][w] = s2;
        }
        __syncthreads();
        m = 0.0;
        s2 = 0.0;
#pragma unroll
        for (int k = 0; k < NWR; ++k) {
            m += red[0][k];
            s2 += red[1][k];
        }
    }
    if (xm == 1) {  // several ranks: this rank's share of the row's sums (chunks: the chunk's)
        if (lt == 0) a.sums[a.chunks ? ri : row] = make_double2(m, s2);
        return;
    }
    double nv;
    bool keep;
    if (xm == 2) {
        nv = dl.y;
        keep = dl.z != 0.0;
    } else {
        nv = fmm_draw<MODE>(a, at, old, m, s2, keep);
        if (lt == 0) {
            a.own[at] = nv;
            if constexpr (IP) a.rec[at] = make_double2(old, nv);  // nv == old when kept
        }
    }
#pragma unroll
    for (int j = 0; j < MCF; ++j) {
        const uint32_t k = lt + j * NT;
        if (k < n) {
            const uint32_t q = beg + k;
            const bool cached = xm != 2;  // the forwarding pass (several ranks, chunks) summed nothing
            const double e = cached ? ce[j] : (IP ? pend(q, ein[q]) : a.e_in[q]);
            double eo = e;
            if (!keep) {
                const double h = MODE == 0 ? (double)x : (cached ? ch[j] : hval(q));
                eo = e - h * (old - nv);
            }
            if constexpr (IP)
                a.e_io[q] = eo;
            else
                a.e_out[cached ? cp[j] : a.perm[q]] = eo;
        }
    }
    for (uint32_t k = lt + MCF * NT; k < n; k += NT) {
        const uint32_t q = beg + k;
        const double e = IP ? pend(q, ein[q]) : a.e_in[q];
        double eo = e;
        if (!keep) {
            if constexpr (MODE == 0) {
                const double h = x;
                eo = e - h * (old - nv);
            } else {
                eo = e - hval(q) * (old - nv);
            }
        }
        if constexpr (IP)
            a.e_io[q] = eo;
        else
            a.e_out[a.perm[q]] = eo;
    }
}

__global__ __launch_bounds__(256) void k_fmm_esums(const double* __restrict__ e, uint64_t n, double w0,
                                                   double* __restrict__ part) {
    const uint64_t b0 = (uint64_t)blockIdx.x * 1024;
    double s = 0.0, d = 0.0;
    for (int k = 0; k < 4; ++k) {
        const uint64_t q = b0 + k * 256 + threadIdx.x;
        if (q < n) {
            const double v = e[q];
            s += v * v;
            d += v - w0;
        }
    }
    s = wsum(s);
    d = wsum(d);
    __shared__ double red[2][4];
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = s;
        red[1][threadIdx.x >> 6] = d;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
        part[2 * blockIdx.x + 1] = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
    }
}

// The sums the hyperparameter draws of fm_learn_mcmc.h:951-1089 take over one column of the
// model (v column f for blockIdx f < K, w for blockIdx K), in the host loop's order: one
// sequential chain each, gm from its initial value (beta_0 (mu - mu_0)^2 + gamma_0, host)
// adding (x_i - mu)^2 for i = 0..p-1, and m from 0 adding x_i -- so the result is the host
// loop's, bit for bit (no contraction).  The whole workgroup stages 2048-value chunks of the
// column and their squared deviations in LDS (double-buffered); lane 0 runs the gm chain and
// lane 1 the m chain, side by side in one instruction stream.
__global__ __launch_bounds__(256) void k_fmm_hsums(const double* __restrict__ v, const double* __restrict__ w,
                                                   uint32_t p, uint32_t K, const double2* __restrict__ mg,
                                                   double2* __restrict__ out) {
#pragma clang fp contract(off)
    constexpr uint32_t CH = 2048;
    __shared__ __align__(16) double xs[2][CH];
    __shared__ __align__(16) double ds[2][CH];
    const uint32_t c = blockIdx.x;
    const double* __restrict__ x = c < K ? v + (size_t)c * p : w;
    const double mu = mg[c].x;
    double acc = threadIdx.x == 0 ? mg[c].y : 0.0;  // lane 0: gm, lane 1: m
    const uint32_t nch = (p + CH - 1) / CH;
    auto stage = [&](uint32_t ch, int b) {
        for (uint32_t i = threadIdx.x; i < CH; i += 256) {
            const uint64_t q = (uint64_t)ch * CH + i;
            const double t = q < p ? x[q] : 0.0;
            const double d = t - mu;
            xs[b][i] = t;
            ds[b][i] = d * d;
        }
    };
    stage(0, 0);
    __syncthreads();
    for (uint32_t ch = 0; ch < nch; ++ch) {
        const int b = ch & 1;
        if (ch + 1 < nch) stage(ch + 1, b ^ 1);
        if (threadIdx.x < 2) {
            const double* __restrict__ src = threadIdx.x == 0 ? ds[b] : xs[b];
            const uint32_t n = min(CH, p - ch * CH);
            uint32_t j = 0;
            for (; j + 32 <= n; j += 32) {
                double2 t[16];  // 16-byte LDS reads, all issued before the first add
#pragma unroll
                for (int u = 0; u < 16; ++u) t[u] = reinterpret_cast<const double2*>(src + j)[u];
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    acc = acc + t[u].x;
                    acc = acc + t[u].y;
                }
            }
            for (; j < n; ++j) acc = acc + src[j];
        }
        __syncthreads();
    }
    __shared__ double res[2];
    if (threadIdx.x < 2) res[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0) out[c] = make_double2(res[0], res[1]);
}

__global__ __launch_bounds__(256) void k_fmm_shift(double* __restrict__ e, uint64_t n, double d) {
    const uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (q < n) e[q] -= d;
}

__global__ __launch_bounds__(256) void k_fmm_transpose(const double* __restrict__ v, double* __restrict__ vT,
                                                       uint32_t K, uint32_t Kp, uint32_t p) {
    __shared__ double tile[32][33];
    const uint32_t a0 = blockIdx.x * 32, f0 = blockIdx.y * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
    for (int r = ty; r < 32; r += 8) {
        const uint32_t f = f0 + r, a = a0 + tx;
        tile[r][tx] = (f < K && a < p) ? v[(size_t)f * p + a] : 0.0;
    }
    __syncthreads();
    for (int r = ty; r < 32; r += 8) {
        const uint32_t a = a0 + r, f = f0 + tx;
        if (a < p && f < Kp) vT[(size_t)a * Kp + f] = tile[tx][r];
    }
}

// prediction of the case with attributes (p0 < p1), in the order of
// predict_data_and_write_to_eterms: e = sum_f 1/2 q_f^2, q2 = sum_f (-1/2 v0^2 x^2 - 1/2 v1^2 x^2)
// (+ w0 x + w1 x), e + q2 (+ w0)
__device__ __forceinline__ double fm_pred(const FMPredictArgs& a, uint32_t p0, uint32_t p1) {
    const float x = 1.0f;
    const double* v0 = a.vT + (size_t)p0 * a.Kp;
    const double* v1 = a.vT + (size_t)p1 * a.Kp;
    double e = 0.0, q2 = 0.0;
    auto term = [&](double x0, double x1) {
        const double q = (0.0 + x0 * x) + x1 * x;
        e += 0.5 * q * q;
        q2 -= 0.5 * x0 * x0 * x * x;
        q2 -= 0.5 * x1 * x1 * x * x;
    };
    // the rows are read 4 factors at a time (two 16-byte loads per row: a quarter of the
    // load instructions of one double per factor, whose lanes each touched a different
    // row); the terms are added one factor at a time in factor order, as before
    uint32_t f = 0;
    for (; f + 4 <= a.K; f += 4) {
        const double2 a0 = *reinterpret_cast<const double2*>(v0 + f), a1 = *reinterpret_cast<const double2*>(v0 + f + 2);
        const double2 b0 = *reinterpret_cast<const double2*>(v1 + f), b1 = *reinterpret_cast<const double2*>(v1 + f + 2);
        term(a0.x, b0.x);
        term(a0.y, b0.y);
        term(a1.x, b1.x);
        term(a1.y, b1.y);
    }
    for (; f < a.K; ++f) term(v0[f], v1[f]);
    if (a.k1) {
        q2 += a.w[p0] * x;
        q2 += a.w[p1] * x;
    }
    e = e + q2;
    if (a.k0) e += a.w0;
    return e;
}

__device__ __forceinline__ double clampd(double p, double lo, double hi) {
    p = p < hi ? p : hi;  // std::min(max_target, p)
    return p > lo ? p : lo;  // std::max(min_target, p)
}

__device__ __forceinline__ double block_sum(double s, double* red) {  // 256 threads, fixed order
    s = wsum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    return ((red[0] + red[1]) + red[2]) + red[3];
}

__global__ __launch_bounds__(256) void k_fmm_predict_train(FMPredictArgs a, const uint32_t* __restrict__ own_u,
                                                           const uint32_t* __restrict__ part_u,
                                                           const float* __restrict__ y, uint64_t n,
                                                           double* __restrict__ e, double* __restrict__ part) {
    const uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    double se = 0.0;
    if (q < n) {
        const double pr = fm_pred(a, own_u[q], a.I + part_u[q]);
        const double err = clampd(pr, a.lo, a.hi) - y[q];
        se = err * err;
        e[q] = pr - y[q];
    }
    __shared__ double red[4];
    se = block_sum(se, red);
    if (threadIdx.x == 0) part[blockIdx.x] = se;
}

__global__ __launch_bounds__(256) void k_fmm_predict_test(FMPredictArgs a, const uint32_t* __restrict__ su,
                                                          const uint32_t* __restrict__ si,
                                                          const float* __restrict__ y, uint64_t n, double it1,
                                                          double* __restrict__ pthis, double* __restrict__ sum_all,
                                                          double* __restrict__ part) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    double sa = 0.0, st = 0.0;
    if (t < n) {
        const double pr = fm_pred(a, su[t], a.I + si[t]);
        pthis[t] = pr;
        const double s = sum_all[t] + clampd(pr, a.lo, a.hi);
        sum_all[t] = s;
        const double ea = clampd(s * (1.0 / it1), a.lo, a.hi) - y[t];  // _evaluate: pred * normalizer
        const double et = clampd(pr * 1.0, a.lo, a.hi) - y[t];
        sa = ea * ea;
        st = et * et;
    }
    __shared__ double red[2][4];
    sa = block_sum(sa, red[0]);
    st = block_sum(st, red[1]);
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = sa;
        part[2 * blockIdx.x + 1] = st;
    }
}

// several ranks: one thread per item row, sums added in rank order, then the draw
template <int MODE>
__global__ __launch_bounds__(256) void k_fmm_item(FMPassArgs a, const double2* __restrict__ recv, int R,
                                                  uint32_t nrows, double4* __restrict__ delta) {
    const uint32_t row = blockIdx.x * 256 + threadIdx.x;
    if (row >= nrows) return;
    double m = 0.0, s2 = 0.0;
    for (int r = 0; r < R; ++r) {
        m += recv[(size_t)r * nrows + row].x;
        s2 += recv[(size_t)r * nrows + row].y;
    }
    const uint32_t at = a.a0 + row;
    const double old = a.own[at];
    bool keep;
    const double nv = fmm_draw<MODE>(a, at, old, m, s2, keep);
    a.own[at] = nv;
    delta[row] = make_double4(old, nv, keep ? 1.0 : 0.0, 0.0);
}

// one rank, long rows in chunks: one thread per long row, chunk sums in chunk order
template <int MODE>
__global__ __launch_bounds__(256) void k_fmm_chunk_draw(FMPassArgs a, const uint32_t* __restrict__ rows,
                                                        const uint32_t* __restrict__ cfirst, uint32_t nlong,
                                                        const double2* __restrict__ csums, double4* __restrict__ delta,
                                                        double2* __restrict__ qq) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= nlong) return;
    double m = 0.0, s2 = 0.0;
    for (uint32_t c = cfirst[i]; c < cfirst[i + 1]; ++c) {
        m += csums[c].x;
        s2 += csums[c].y;
    }
    const uint32_t at = a.a0 + rows[i];
    const double old = a.own[at];
    bool keep;
    const double nv = fmm_draw<MODE>(a, at, old, m, s2, keep);
    a.own[at] = nv;
    if (a.rec) {
        qq[i] = a.rec[at];
        a.rec[at] = make_double2(old, nv);  // nv == old when kept
    }
    delta[i] = make_double4(old, nv, keep ? 1.0 : 0.0, 0.0);
}

template <int MODE, bool IP>
hipError_t launch_pass_ip(const FMPassArgs& a, int tpr, hipStream_t st) {
    switch (tpr) {
        case 64:
            k_fmm_pass<MODE, 64, IP><<<(a.nrows + 3) / 4, 256, 0, st>>>(a);
            break;
        case 256:
            k_fmm_pass<MODE, 256, IP><<<a.nrows, 256, 0, st>>>(a);
            break;
        case 1024:
            k_fmm_pass<MODE, 1024, IP><<<a.nrows, 1024, 0, st>>>(a);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
template <int MODE>
hipError_t launch_pass(const FMPassArgs& a, int tpr, hipStream_t st) {
    if (a.nrows == 0) return hipSuccess;
    if (a.e_io) {
        if ((a.xmode != 0 && !a.chunks) || !a.rec) return hipErrorInvalidValue;  // in place: one rank only
        return launch_pass_ip<MODE, true>(a, tpr, st);
    }
    return launch_pass_ip<MODE, false>(a, tpr, st);
}

}  // namespace

hipError_t fmm_item_update(const FMPassArgs& a, const double2* recv, int R, uint32_t nrows, int vpass, double4* delta,
                           hipStream_t st) {
    if (nrows == 0) return hipSuccess;
    if (vpass)
        k_fmm_item<1><<<(nrows + 255) / 256, 256, 0, st>>>(a, recv, R, nrows, delta);
    else
        k_fmm_item<0><<<(nrows + 255) / 256, 256, 0, st>>>(a, recv, R, nrows, delta);
    return hipGetLastError();
}

hipError_t fmm_chunk_draw(const FMPassArgs& a, const uint32_t* rows, const uint32_t* cfirst, uint32_t nlong,
                          const double2* csums, int vpass, double4* delta, double2* qq, hipStream_t st) {
    if (nlong == 0) return hipSuccess;
    if (vpass)
        k_fmm_chunk_draw<1><<<(nlong + 255) / 256, 256, 0, st>>>(a, rows, cfirst, nlong, csums, delta, qq);
    else
        k_fmm_chunk_draw<0><<<(nlong + 255) / 256, 256, 0, st>>>(a, rows, cfirst, nlong, csums, delta, qq);
    return hipGetLastError();
}

hipError_t fmm_wpass(const FMPassArgs& a, int tpr, hipStream_t st) { return launch_pass<0>(a, tpr, st); }
hipError_t fmm_vpass(const FMPassArgs& a, int tpr, hipStream_t st) { return launch_pass<1>(a, tpr, st); }

hipError_t fmm_esums(const double* e, uint64_t n, double w0, double* part, hipStream_t st) {
    if (n == 0) return hipSuccess;
    k_fmm_esums<<<(unsigned)((n + 1023) / 1024), 256, 0, st>>>(e, n, w0, part);
    return hipGetLastError();
}

hipError_t fmm_hsums(const double* v, const double* w, uint32_t p, uint32_t K, const double2* mg, double2* out,
                     hipStream_t st) {
    if (p == 0) return hipSuccess;
    k_fmm_hsums<<<K + 1, 256, 0, st>>>(v, w, p, K, mg, out);
    return hipGetLastError();
}

hipError_t fmm_shift(double* e, uint64_t n, double d, hipStream_t st) {
    if (n == 0) return hipSuccess;
    k_fmm_shift<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(e, n, d);
    return hipGetLastError();
}

hipError_t fmm_transpose(const double* v, double* vT, uint32_t K, uint32_t Kp, uint32_t p, hipStream_t st) {
    dim3 grid((p + 31) / 32, (Kp + 31) / 32);
    k_fmm_transpose<<<grid, 256, 0, st>>>(v, vT, K, Kp, p);
    return hipGetLastError();
}

hipError_t fmm_predict_train(const FMPredictArgs& a, const uint32_t* own_u, const uint32_t* part_u, const float* y,
                             uint64_t n, double* e, double* part, hipStream_t st) {
    if (n == 0) return hipSuccess;
    k_fmm_predict_train<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(a, own_u, part_u, y, n, e, part);
    return hipGetLastError();
}

hipError_t fmm_predict_test(const FMPredictArgs& a, const uint32_t* su, const uint32_t* si, const float* y,
                            uint64_t n, double it1, double* pthis, double* sum_all, double* part, hipStream_t st) {
    if (n == 0) return hipSuccess;
    k_fmm_predict_test<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(a, su, si, y, n, it1, pthis, sum_all, part);
    return hipGetLastError();
}

}  // namespace sbmf
