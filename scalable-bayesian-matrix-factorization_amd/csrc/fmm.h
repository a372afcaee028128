// fmm.h -- libFM-order MCMC and ALS (`-method mcmc --order libfm`, `-method
// als`): the reference's fm_learn_mcmc / fm_learn_mcmc_simultaneous learner
// (src/libfm/src/fm_learn_mcmc.h:411-623 draw_all, :627-835 draw_w0/w/v,
// :901-1089 hyperparameters; fm_learn_mcmc_simultaneous.h:50-303) on rating
// data, on the GPU.
//
// Model: a factorization machine over libFM's users-first one-hot layout
// (attribute u for user u, I + i for item i, p = the libFM attribute count):
// global bias w0, per-attribute bias w[p] and factors v[K][p] (f-major, as
// fm_model::v), one attribute group with Normal-Gamma hyperpriors, noise
// precision alpha.  A sweep draws alpha, w0, the w group hyperparameters and
// every w (users, then items), the v hyperparameters, then per factor f
// every v[f][.] (users, then items: the "f-outer" order), re-predicts train
// and test, and evaluates the running-mean test RMSE.  Per-row conditionals
// are independent within one (factor, side) pass, so a pass is one launch.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/sbmf.h"

namespace sbmf {

// One attribute row of an orientation: its cases are [ptr[row], ptr[row+1]).
// Rows are binned by length; a bin is launched with 64, 256 or 1024 threads
// per row.
struct FMPassArgs {
    const uint32_t* rows;   // [nrows] rows of this bin
    uint32_t nrows;
    const uint32_t* ptr;    // [R+1] case offsets of the orientation (rows past the data: empty)
    const uint32_t* part;   // [N] partner row of each case (users: item id, items: user id)
    const uint32_t* perm;   // [N] position of the case in the other orientation's order
    const double* e_in;     // [N] residuals e = prediction - target, this orientation's order
    double* e_out;          // [N] residuals, the other orientation's order (e_out[perm[q]])
    double* own;            // w (bias pass) or column f of v (factor pass), indexed by attribute
    const double* partner_col;  // factor pass: column f of v (partner values, by attribute)
    const double* vold_u;   // factor pass, item side: the users' column f before the user pass
    const double* z;        // normals, z[a * zs + zoff] (do_sample)
    uint32_t zs, zoff;
    uint32_t a0;            // attribute of row 0 (0: users, I: items)
    uint32_t pa0;           // attribute of partner row 0 (I for users, 0 for items)
    double alpha, mu, lambda;
    int do_sample;
    int item_side;          // factor pass: 1 = items (q carries the user pass's updates)
    // several ranks, item rows (xmode 1): write the row's local {sum m, sum s2} to
    // sums[row]; (xmode 2): take {old, new, keep} from delta[row] (fmm_item_update)
    // and update the local cases' residuals; 0: one rank, sums and draw in one pass
    int xmode;
    double2* sums;
    const double4* delta;
    // one rank (e_io non-null): the residuals are kept in BOTH orders, each read and
    // written in place by its own side's passes (sequential, no scatter); the other
    // side's last pass is applied to a case on read, from that side's per-attribute
    // records -- the same operations the scatter form applied, in the same order
    double* e_io;
    double2* rec;   // [p] by attribute: {old, value kept} of the attribute's last draw (a kept
                    // draw, non-finite in the reference's sense, records old twice)
    int pend;       // the other side's last pass: 0 none, 1 a w pass, 2 a v pass
    // one rank, long rows cut into chunks (non-null: the pass runs over chunks {row, first
    // case, cases, long-row index}): xmode 1 writes chunk ri's sums to sums[ri], xmode 2
    // takes {old, new, keep} from delta[long-row index] and the user rows' {qo, qn} (the
    // record the draw replaced) from qq[long-row index]
    const uint4* chunks;
    const double2* qq;
};
// several ranks: every item row's draw from every rank's local sums (recv
// [R][nrows], rank order), the same on every rank; a.own / a.z / a.mu ... as for
// the pass; writes own[a0 + row] and delta[row] = {old, new, keep}
hipError_t fmm_item_update(const FMPassArgs& a, const double2* recv, int R, uint32_t nrows, int vpass, double4* delta,
                           hipStream_t st);
// one rank, long rows in chunks: row i of `rows` (nlong rows) owns chunks [cfirst[i],
// cfirst[i+1]); its chunk sums added in chunk order, the draw, own / rec written, and
// delta[i] = {old, new, keep}, qq[i] = the record the draw replaced ({qo, qn})
hipError_t fmm_chunk_draw(const FMPassArgs& a, const uint32_t* rows, const uint32_t* cfirst, uint32_t nlong,
                          const double2* csums, int vpass, double4* delta, double2* qq, hipStream_t st);
// draw_w (:670-719) over the rows of a bin
hipError_t fmm_wpass(const FMPassArgs& a, int threads_per_row, hipStream_t st);
// draw_v (:780-835) of one factor over the rows of a bin
hipError_t fmm_vpass(const FMPassArgs& a, int threads_per_row, hipStream_t st);
// part[b] = {sum e^2, sum (e - w0)} over 1024-case blocks
hipError_t fmm_esums(const double* e, uint64_t n, double w0, double* part, hipStream_t st);
// the hyperparameter sums {gm, m} of each v column (out[f]) and of w (out[K]) in the host's
// order; mg[c] = {mu, gm's initial value} (fm_learn_mcmc.h:951-1089)
hipError_t fmm_hsums(const double* v, const double* w, uint32_t p, uint32_t K, const double2* mg, double2* out,
                     hipStream_t st);
// e[q] -= d (the w0 update, :663-666)
hipError_t fmm_shift(double* e, uint64_t n, double d, hipStream_t st);
// [K][p] -> [p][Kp] (attribute-major rows for the predictions)
hipError_t fmm_transpose(const double* v, double* vT, uint32_t K, uint32_t Kp, uint32_t p, hipStream_t st);
// predict_data_and_write_to_eterms (:117-348) per case, in the reference's
// accumulation order.  Train (cases in user order, a0 = own_u[q], a1 = I +
// part_u[q]): e[q] = pred - y[q]; part[b] = sum over the block of
// (clamp(pred) - y)^2.  Test: pthis[t] = pred, sum_all[t] += clamp(pred);
// part[2b] = (clamp(sum_all / it1) - y)^2, part[2b+1] = (clamp(pthis) - y)^2.
struct FMPredictArgs {
    const double* vT;       // [p][Kp]
    const double* w;        // [p]
    double w0;
    uint32_t K, Kp, I;
    int k0, k1;
    double lo, hi;          // train target range (the reference's min/max_target)
};
hipError_t fmm_predict_train(const FMPredictArgs& a, const uint32_t* own_u, const uint32_t* part_u, const float* y,
                             uint64_t n, double* e, double* part, hipStream_t st);
hipError_t fmm_predict_test(const FMPredictArgs& a, const uint32_t* su, const uint32_t* si, const float* y,
                            uint64_t n, double it1, double* pthis, double* sum_all, double* part, hipStream_t st);

// ---- host learner (fmm.cpp), driven by the C ABI in sbmf.cpp
struct FMLearner;
class Comm;
// comm: null, or R > 1 ranks (one process per GPU): users split by
// sbmf_partition_rows, every case local to its user's rank, item rows summed
// over the ranks (as the online VB learner, vbo.cpp)
FMLearner* fmm_create(const sbmf_config& c, uint64_t n, const uint32_t* u, const uint32_t* i, const double* r,
                      uint64_t nt, const uint32_t* tu, const uint32_t* ti, const double* tr, uint32_t I, uint32_t J,
                      hipStream_t st, Comm* comm = nullptr);
void fmm_destroy(FMLearner* L);
void fmm_run(FMLearner* L, uint32_t iters, sbmf_sweep_cb cb, void* user);
void fmm_predict_out(FMLearner* L, double* out);       // the -out predictions (fm_learn_mcmc::predict)
void fmm_factors(FMLearner* L, double* U, double* V);  // v of the users [I][K] and items [J][K]
void fmm_biases(FMLearner* L, double* bu, double* bv, double* b0);  // w of users, items; w0
void fmm_hyper_out(FMLearner* L, double* h4k, double* alpha);       // [v_lambda | v_mu | w_lambda,w_mu,0.. | 0]
uint32_t fmm_launches(const FMLearner* L);
uint32_t fmm_num_attribute(const FMLearner* L);

}  // namespace sbmf
