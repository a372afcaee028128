// vbo.h -- online variational Bayes (`-method vb`): the reference's
// fm_learn_vb_online learner (src/libfm/src/fm_learn_vb_online.h,
// fm_learn_vb_online_simultaneous.h) on rating data, on the GPU.
//
// Model: attributes 0..I-1 are users, I..I+J-1 items (libFM's users-first
// one-hot layout); per attribute a bias mean / variance (mu_w, sigma_w') and
// K factor means / variances (mu_v, sigma_v'), each with its natural
// parameters; the global bias (mu_0', sigma_0'); the noise precision alpha
// and the prior precisions sigma_0, sigma_w, sigma_v[f].  One epoch = a
// shuffle into 30 batches, and per batch: predictions and their variances,
// update_w0, update_w (users, then items), update_v (factor-outer: users,
// then items, per factor), hyperparameter blends.  Step sizes (t0 + t)^-0.5.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "../../include/sbmf.h"

namespace sbmf {

// One attribute's cases inside one batch: entries [start, start + len) of
// the orientation's case arrays (partner attribute, position of the case in
// the other orientation's order), which hold the epoch's cases batch-major.
struct VRow {
    uint32_t attr, start, len, pad;
};

// Scalar state kept on the device so a batch needs no host round trip.
struct VBScal {
    double alpha, sigma_0, mu0, sg0, nm0, ns0, sigma_w, rho0;
    double d_mu0, d_sg0;  // this batch's update_w0 deltas, applied by the user bias pass
    uint32_t t_w0, n_skip;  // n_skip: batches whose alpha was NaN/inf (the reference then skips the blends)
};

// Parameter tables, f-major [K][p] like the reference's DMatrix (the column
// of factor f is contiguous and small enough to stay in L2 during a pass).
struct VBTables {
    double *mu_v, *sg_v, *nm_v, *ns_v;  // [K][p]
    double *mu_w, *sg_w, *nm_w, *ns_w;  // [p]
    double *rho_w, *rho_v;              // [p] step sizes (t0 + t)^-0.5
    uint32_t *t_w, *t_v, *cc;           // [p] step counts, train column counts
    double* sigma_v;                    // [K] prior precisions of the factors
    VBScal* scal;
    uint32_t K, p, N;                   // N: train ratings (the reference's _size)
    uint32_t I;                         // users (attributes [0, I)); items are [I, p)
};

// A batch's per-case terms in its user-grouped order: E = e (the residual),
// T = t (its variance term), two arrays so an item pass's gathers of e touch
// half the bytes.
struct VBCases {
    double *E, *T;
    VBCases at(size_t o) const { return VBCases{E + o, T + o}; }
};
// [K][p] -> [p][Kp] (attribute-major rows for the prediction gathers)
hipError_t vbo_transpose(const double* src, double* dst, uint32_t K, uint32_t Kp, uint32_t p, hipStream_t st);
// e = r - prediction and t = its variance for every case of a batch, driven
// by the batch's user rows (fm_learn_vb_online.h:80-310)
hipError_t vbo_predict(const VRow* rows, uint32_t nrows, const uint32_t* part, const float* r, const double* muT,
                       const double* sgT, const VBTables& tb, uint32_t Kp, VBCases ET, hipStream_t st);
// update_w0 (:586-633): the global bias blend; its deltas are applied to e / t
// by vbo_user_w
hipError_t vbo_update_w0(VBCases ET, uint32_t B, const VBTables& tb, double* part, hipStream_t st);
// Several ranks: an item present in a batch (any rank's cases) and its global
// case count there; a rank's item rows carry their index in this list in VRow.pad.
struct VGItem {
    uint32_t attr, n, mask;  // mask: the parts (ranks or XCD slices) holding its cases
};
// One 256-thread block of an update pass: rows [row0, row0 + nrows) of the
// orientation's row list, each owned by 2^lg lanes (256 >> lg rows at most);
// a lane keeps up to VB_CASES_PER_LANE of its row's cases in registers.
constexpr uint32_t VB_CASES_PER_LANE = 4;
// item rows (long, read-only passes: only e and the partner record per case in flight)
#ifndef SBMF_VB_ITEM_CPL
#define SBMF_VB_ITEM_CPL 8
#endif
constexpr uint32_t VB_ITEM_CASES_PER_LANE = SBMF_VB_ITEM_CPL;
struct VTask {
    uint32_t row0, nrows, lg, pad;
};
// The passes of a batch keep one {e, t} record per case, in the batch's
// user-grouped order (ET).  A user pass reads and writes its rows' records in
// place; an item pass gathers e through its user-grouped position
// (iu[q] = {that position, the user's batch row}) and writes nothing per case: its e / t updates are left per item in D
// (VBItemRec, indexed by item - I) and applied by the next user pass (pend)
// or by vbo_user_flush before the hyperparameter sums.
enum { VB_PEND_NONE = 0, VB_PEND_W = 1, VB_PEND_V = 2 };
// per item, from the item pass for the user pass after it: the item's mean and
// variance of that user pass's factor, and the item pass's e / t updates
struct VBItemRec {
    double v, s, dmu, dsg, dm2, ok;
};  // pending: none | bias pass | factor pass
// update_w (:635-710) of the users (update_w0's deltas applied first)
hipError_t vbo_user_w(const VTask* tasks, uint32_t ntask, const VRow* rows, const VBTables& tb, VBCases ET,
                      hipStream_t st);
// update_v (:712-800) of factor f for the users, after the pending item updates
// (pend; factor fp for VB_PEND_V); VS[row] = the user's new {mean, variance}
// of f, by its row in the batch (rows: the batch's user rows, tasks index them)
hipError_t vbo_user_v(const VTask* tasks, uint32_t ntask, const VRow* rows, const uint32_t* part, uint32_t f, int pend,
                      uint32_t fp, const VBTables& tb, const VBItemRec* D, VBCases ET, double2* VS, hipStream_t st);
hipError_t vbo_user_flush(const VTask* tasks, uint32_t ntask, const VRow* rows, const uint32_t* part, int pend,
                          uint32_t fp, const VBTables& tb, const VBItemRec* D, VBCases ET, hipStream_t st);
// update_w / update_v of factor f for the items (D[item] = the deltas); several
// ranks: sums != null -> each row's local sums to sums[VRow.pad] only
hipError_t vbo_item_w(const VTask* tasks, uint32_t ntask, const VRow* rows, const uint2* iu, const VBTables& tb,
                      VBCases ET, VBItemRec* D, double2* sums, hipStream_t st);
hipError_t vbo_item_v(const VTask* tasks, uint32_t ntask, const VRow* rows, const uint2* iu, uint32_t f, const VBTables& tb, VBCases ET, const double2* VS, VBItemRec* D, double2* sums,
                      hipStream_t st);
// several ranks: the items of a batch updated from every rank's local sums
// (recv [R][nG], rank order; factor f, or the biases when factor == 0)
hipError_t vbo_item_update(const VGItem* gi, uint32_t nG, const double2* recv, int R, int factor, uint32_t f,
                           const VBTables& tb, VBItemRec* D, hipStream_t st);
// several ranks: update_w0's local sum (out[0]) and the update from every rank's (recv[R])
hipError_t vbo_w0_local(VBCases ET, uint32_t B, const VBTables& tb, double* part, double* out, hipStream_t st);
hipError_t vbo_w0_final(const double* recv, int R, uint32_t B, const VBTables& tb, hipStream_t st);
// several ranks: out = [alpha's local sum | K + 1 sig sums over the users [u0, u1)],
// then the blends from every rank's (recv [R][K + 2]) plus the item range [I, p)
hipError_t vbo_hyper_local(VBCases ET, uint32_t B, const VBTables& tb, uint32_t u0, uint32_t u1, double* part,
                           size_t part_cap, double* out, hipStream_t st);
hipError_t vbo_hyper_final(const double* recv, int R, uint32_t B, const VBTables& tb, uint32_t I, double* part,
                           size_t part_cap, hipStream_t st);
// step sizes of update_v (:447-453) and the hyperparameter blends (:523-580)
hipError_t vbo_hyper(VBCases ET, uint32_t B, const VBTables& tb, double* part, hipStream_t st);
// test predictions clamped to [lo, hi] and their squared errors per 256-case block
hipError_t vbo_test(const uint32_t* tu, const uint32_t* ti, const double* tr, uint64_t n, uint32_t I,
                    const double* muT, const VBTables& tb, uint32_t Kp, double lo, double hi, double* pred,
                    double* part, hipStream_t st);
// ---- host learner (vbo.cpp), driven by the C ABI in sbmf.cpp
struct VBLearner;
class Comm;
// comm: null, or a communicator of R > 1 ranks (one process per GPU): each
// rank then owns a contiguous, rating-balanced user range and every case of
// those users; item rows are summed over the ranks (see vbo.cpp)
VBLearner* vbo_create(const sbmf_config& c, uint64_t n, const uint32_t* u, const uint32_t* i, const double* r,
                      uint64_t nt, const uint32_t* tu, const uint32_t* ti, const double* tr, uint32_t I, uint32_t J,
                      hipStream_t st, Comm* comm = nullptr);
void vbo_destroy(VBLearner* L);
void vbo_run(VBLearner* L, uint32_t epochs, sbmf_sweep_cb cb, void* user);
void vbo_predict_out(VBLearner* L, double* out);  // clamped test predictions of the means
void vbo_factors(VBLearner* L, double* U, double* V);  // factor means, users [I][K], items [J][K]
void vbo_biases(VBLearner* L, double* bu, double* bv, double* b0);
void vbo_hyper_out(VBLearner* L, double* h4k, double* alpha);  // [sigma_v | 0 | 0 | 0], alpha
double vbo_layout_ms(const VBLearner* L);  // host time of the last epoch's shuffle + batch layout
uint32_t vbo_launches(const VBLearner* L);
// device time of an epoch's factor passes (every mini-batch's 2K vbo_user_v / vbo_item_v launches,
// HIP events around each batch's factor loop), averaged over the last vbo_run's epochs
double vbo_factor_ms(const VBLearner* L);

// scratch doubles vbo_update_w0 / vbo_hyper (one rank) and vbo_hyper_local /
// vbo_hyper_final (several ranks) need for B cases:
//   vbo_hyper:       [alpha partials nab | 8 | sig partials (K+1) x nchunk(p)]
//   vbo_hyper_final: [item sums K+1 | 7 | sig partials (K+1) x nchunk(p-I) | 8 | combined K+2]
inline size_t vbo_hyper_final_doubles(uint32_t K, uint32_t nchunk) {
    return (size_t)K + 8 + (size_t)(K + 1) * nchunk + 8 + (K + 2);
}
inline size_t vbo_scratch_doubles(uint32_t B, uint32_t K, uint32_t p) {
    const uint32_t nc = std::max(1u, (p + 2047) / 2048);
    const size_t one = (size_t)(B + 1023) / 1024 + 16 + (size_t)(K + 1) * (nc + 1);
    return std::max(one, vbo_hyper_final_doubles(K, nc));
}

}  // namespace sbmf
