// fmm.cpp -- host side of the libFM-order MCMC / ALS learner (fmm.h):
// the reference's `bin/libFM -method mcmc` / `-method als` chain
// (src/libfm/src/fm_learn_mcmc.h, fm_learn_mcmc_simultaneous.h, set up by
// libfm.cpp:124-136,386-513) on rating data in libFM's users-first layout.
//
// Per iteration (fm_learn_mcmc_simultaneous.h:96-245 around draw_all,
// fm_learn_mcmc.h:411-623):
//   1. alpha ~ Gamma((alpha_0 + N)/2, (gamma_0 + sum e^2)/2)      (device sums, host draw)
//   2. w0 ~ N(...), e -= w0_old - w0                                 (device sum, host draw)
//   3. w group hyperparameters (host, from the device copy of w), then every
//      w: users pass, items pass                                     (device)
//   4. v group hyperparameters per factor (host), then per factor f: users
//      pass, items pass                                              (device, 2K launches)
//   5. re-predict train and test, running-mean test RMSE              (device)
// Reference RNG mode replays the reference's glibc rand() stream draw for
// draw (rng.h): the host draws the scalars in consumption order and fills
// the per-attribute normals of the w and v passes ahead of the launches
// (libFM consumes exactly one normal per drawn attribute).  Philox mode
// fills those normals on the device.  ALS (do_sample = do_multilevel = 0)
// draws nothing: alpha = 1, the w / v draws take their posterior means.
//
// Several ranks (one process per GPU), as the online VB learner: rank k owns
// the users sbmf_partition_rows gives it and every case of those users.  User
// rows are drawn locally; an item pass writes each item row's local sums, one
// all-gather delivers every rank's, and every rank draws every item the same
// way (sums added in rank order) and forwards the change to its own cases.
// The scalar sums (alpha, w0, the train RMSE) are all-gathered per rank; the
// owned users' w and v are broadcast after each sweep's passes, so the host
// hyperparameter draws, the test predictions and the factors see every
// attribute.  The host draws every variate on every rank (the same stream).
#include "fmm.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>
#include <vector>

#include "comm.h"
#include "common.h"
#include "kernels.h"
#include "rng.h"

namespace sbmf {

enum : uint32_t { TAG_FMM_W = 8, TAG_FMM_V = 9, TAG_FMM_INIT = 10 };

struct FMBin {
    std::vector<uint32_t> rows;
    DBuf d_rows;
    int tpr;
    // one rank, the long-row bin: each row cut into chunks of at most fmm_chunk cases
    // {row, first case, cases, row index in this bin}; row i owns [cfirst[i], cfirst[i+1])
    std::vector<uint4> chunks;
    std::vector<uint32_t> cfirst;
    DBuf d_chunks, d_cfirst, d_csums, d_cdelta, d_cqq;
};

struct FMLearner {
    sbmf_config cfg{};
    uint32_t K = 0, Kp = 0, I = 0, J = 0, p = 0, p_train = 0, p_test = 0, RI = 0;  // RI: item-side rows (p - I)
    uint64_t N = 0, T = 0, NL = 0;  // N: train cases (all ranks), NL: this rank's
    int k0 = 1, k1 = 1, do_sample = 1, do_multilevel = 1;
    double lo = 1.0, hi = 5.0;  // the train target range (min/max_target)
    double alpha = 1.0, w0 = 0.0, w_mu = 0.0, w_lambda = 0.0;
    std::vector<double> v_mu, v_lambda;
    uint32_t it = 0, n_launch = 0;
    GlibcRand grand{1};
    hipStream_t st = nullptr;
    hipEvent_t ev[3] = {};
    FMBin ubins[3], ibins[3];
    // device
    DBuf d_uptr, d_upart, d_uperm, d_uown, d_uy, d_iptr, d_ipart, d_iperm;
    DBuf d_eu, d_ei, d_w, d_v, d_vT, d_vold, d_zw, d_zv, d_su, d_si, d_sy, d_pthis, d_sum, d_part, d_tpart, d_res,
        d_scratch;
    std::vector<double> h_w, h_v;  // the initial model (released after the upload)
    // the hyperparameter draws' sums (k_fmm_hsums): per v column f and for w (index K),
    // {mu, gm's initial value} in, {gm, m} out
    DBuf d_hmg, d_hsum;
    std::vector<double> h_mg, h_hs;
    // several ranks
    Comm* comm = nullptr;
    int R = 1;
    // one rank: residuals in both orders updated in place (FMPassArgs::e_io), the
    // attributes' last draws in d_rec; the pass each side must apply on read
    DBuf d_rec;
    int pend_u = 0, pend_i = 0;
    std::vector<uint64_t> ubounds;
    DBuf d_sums, d_recvg, d_delta, d_recv;

    // R ranks: every rank's `n` doubles at d (device) -> host, summed in rank order
    void gather_sums(const double* d, int n, double* out) {
        comm->allgather(d, n * sizeof(double), d_recv.p, st);
        std::vector<double> h((size_t)R * n);
        HIPCHK(hipMemcpyAsync(h.data(), d_recv.p, h.size() * sizeof(double), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        for (int k = 0; k < n; ++k) {
            double t = 0.0;
            for (int r = 0; r < R; ++r) t += h[(size_t)r * n + k];
            out[k] = t;
        }
    }
    // R ranks: the owned users' w and v to every rank
    void sync_users() {
        if (R <= 1) return;
        comm->group_begin();
        comm->bcast_ranges(d_w.p, sizeof(double), ubounds, st);
        for (uint32_t f = 0; f < K; ++f) comm->bcast_ranges(d_v.as<double>() + (size_t)f * p, sizeof(double), ubounds, st);
        comm->group_end();
    }

    ~FMLearner() {
        for (auto& e : ev) event_destroy(e);
    }

    template <class G>
    double gaussian(G& g, double mean, double stdev) {  // random.h:166-172
        if (stdev == 0.0 || std::isnan(stdev)) return mean;
        return mean + stdev * leva_normal(g);
    }
    template <class G>
    void init_model(G& g) {  // fm_model::init (fm_model.h:87-96), libfm.cpp:412
        const double sd = cfg.init_stdev >= 0 ? cfg.init_stdev : 0.1;
        h_v.resize((size_t)K * p);
        h_w.resize(p);
        for (uint32_t f = 0; f < K; ++f)
            for (uint32_t a = 0; a < p; ++a) h_v[(size_t)f * p + a] = gaussian(g, 0.0, sd);
        for (uint32_t a = 0; a < p; ++a) h_w[a] = gaussian(g, 0.0, sd);
    }
    // fm_learn_mcmc.h:951-1009 (one group: every attribute)
    template <class G>
    void draw_hyper_w(G& g) {
        const double alpha_0 = 1.0, beta_0 = 1.0, mu_0 = 0.0;
        if (do_multilevel) {
            // gm = beta_0 (w_mu - mu_0)^2 + gamma_0 + sum_i (w_i - w_mu)^2 and m = sum_i w_i,
            // summed on the device in this order (sweep_draws)
            double gm = h_hs[2 * K];
            const double a = alpha_0 + p + 1;
            const double old = w_lambda;
            w_lambda = do_sample ? mt_gamma(g, a / 2.0) / (gm / 2.0) : a / gm;
            if (std::isnan(w_lambda) || std::isinf(w_lambda)) w_lambda = old;
            double m = h_hs[2 * K + 1];
            m = (m + beta_0 * mu_0) / (p + beta_0);
            const double s2 = 1.0 / ((p + beta_0) * w_lambda);
            const double om = w_mu;
            w_mu = do_sample ? gaussian(g, m, std::sqrt(s2)) : m;
            if (std::isnan(w_mu) || std::isinf(w_mu)) w_mu = om;
        } else {
            w_mu = mu_0;
        }
    }
    // fm_learn_mcmc.h:1011-1089 (a NaN / inf ends that draw's factor loop)
    template <class G>
    void draw_hyper_v(G& g) {
        const double alpha_0 = 1.0, beta_0 = 1.0, mu_0 = 0.0;
        if (!do_multilevel) {
            std::fill(v_mu.begin(), v_mu.end(), mu_0);
            return;
        }
        // the sums over each column (device, the loops' order): gm from beta_0 (mu_f - mu_0)^2 +
        // gamma_0 adding (v_fi - mu_f)^2, m = sum_i v_fi
        for (uint32_t f = 0; f < K; ++f) {
            const double gm = h_hs[2 * f];
            const double a = alpha_0 + p + 1;
            const double old = v_lambda[f];
            v_lambda[f] = do_sample ? mt_gamma(g, a / 2.0) / (gm / 2.0) : a / gm;
            if (std::isnan(v_lambda[f]) || std::isinf(v_lambda[f])) {
                v_lambda[f] = old;
                break;
            }
        }
        for (uint32_t f = 0; f < K; ++f) {
            double m = h_hs[2 * f + 1];
            m = (m + beta_0 * mu_0) / (p + beta_0);
            const double s2 = 1.0 / ((p + beta_0) * v_lambda[f]);
            const double old = v_mu[f];
            v_mu[f] = do_sample ? gaussian(g, m, std::sqrt(s2)) : m;
            if (std::isnan(v_mu[f]) || std::isinf(v_mu[f])) {
                v_mu[f] = old;
                break;
            }
        }
    }

    FMPassArgs pass_args(bool items) {
        FMPassArgs a{};
        a.ptr = (items ? d_iptr : d_uptr).as<uint32_t>();
        a.part = (items ? d_ipart : d_upart).as<uint32_t>();
        a.perm = (items ? d_iperm : d_uperm).as<uint32_t>();
        a.e_in = (items ? d_ei : d_eu).as<double>();
        a.e_out = (items ? d_eu : d_ei).as<double>();
        a.a0 = items ? I : 0;
        a.pa0 = items ? 0 : I;
        a.alpha = alpha;
        a.do_sample = do_sample;
        a.item_side = items ? 1 : 0;
        if (R == 1) {
            a.e_io = (items ? d_ei : d_eu).as<double>();
            a.rec = d_rec.as<double2>();
            a.pend = items ? pend_i : pend_u;
        }
        return a;
    }
    // one rank: the item-order copy of the residuals from the user-order one (after the
    // train re-prediction and the w0 shift); nothing is pending on either side
    void start_passes() {
        if (R != 1) return;
        if (NL) HIPCHK(launch_unpack<double>(d_eu.as<double>(), d_uperm.as<uint32_t>(), NL, d_ei.as<double>(), st));
        ++n_launch;
        pend_u = pend_i = 0;
    }
    void run_bins(FMPassArgs a, bool items, bool vpass) {
        auto launch = [&](int xmode) {
            a.xmode = xmode;
            for (FMBin& b : items ? ibins : ubins) {
                if (b.rows.empty()) continue;
                a.rows = b.d_rows.as<uint32_t>();
                a.nrows = (uint32_t)b.rows.size();
                if (xmode == 0 && !b.chunks.empty()) {
                    // one rank, long rows in chunks: the chunks' sums, the draw per row (chunk
                    // sums in chunk order), then every chunk's residual update -- the row's
                    // cases spread over many workgroups instead of one
                    FMPassArgs c = a;
                    c.chunks = b.d_chunks.as<uint4>();
                    c.nrows = (uint32_t)b.chunks.size();
                    c.xmode = 1;
                    c.sums = b.d_csums.as<double2>();
                    HIPCHK(vpass ? fmm_vpass(c, b.tpr, st) : fmm_wpass(c, b.tpr, st));
                    HIPCHK(fmm_chunk_draw(a, b.d_rows.as<uint32_t>(), b.d_cfirst.as<uint32_t>(), a.nrows,
                                          b.d_csums.as<double2>(), vpass ? 1 : 0, b.d_cdelta.as<double4>(),
                                          b.d_cqq.as<double2>(), st));
                    c.xmode = 2;
                    c.delta = b.d_cdelta.as<double4>();
                    c.qq = b.d_cqq.as<double2>();
                    HIPCHK(vpass ? fmm_vpass(c, b.tpr, st) : fmm_wpass(c, b.tpr, st));
                    n_launch += 3;
                    continue;
                }
                HIPCHK(vpass ? fmm_vpass(a, b.tpr, st) : fmm_wpass(a, b.tpr, st));
                ++n_launch;
            }
        };
        if (!(items && R > 1)) {
            launch(0);
            // one rank: the other side applies this pass on read
            if (items)
                pend_u = vpass ? 2 : 1;
            else
                pend_i = vpass ? 2 : 1;
            return;
        }
        // several ranks: local sums of every item row -> all-gather -> the same draw everywhere
        a.sums = d_sums.as<double2>();
        launch(1);
        comm->allgather(d_sums.p, (size_t)RI * sizeof(double2), d_recvg.p, st);
        HIPCHK(fmm_item_update(a, d_recvg.as<double2>(), R, RI, vpass ? 1 : 0, d_delta.as<double4>(), st));
        a.delta = d_delta.as<double4>();
        launch(2);
        ++n_launch;
    }
    FMPredictArgs predict_args() {
        FMPredictArgs a{};
        a.vT = d_vT.as<double>();
        a.w = d_w.as<double>();
        a.w0 = w0;
        a.K = K;
        a.Kp = Kp;
        a.I = I;
        a.k0 = k0;
        a.k1 = k1;
        a.lo = lo;
        a.hi = hi;
        return a;
    }
    // predict_data_and_write_to_eterms for the train set (+ e = pred - y);
    // returns nothing on the host (sums land in d_res)
    void predict_train() {
        HIPCHK(fmm_transpose(d_v.as<double>(), d_vT.as<double>(), K, Kp, p, st));
        HIPCHK(fmm_predict_train(predict_args(), d_uown.as<uint32_t>(), d_upart.as<uint32_t>(), d_uy.as<float>(), NL,
                                 d_eu.as<double>(), d_part.as<double>(), st));
        n_launch += 2;
    }

    template <class G>
    void sweep_draws(G& g) {
        double* res = d_res.as<double>();
        const bool ref = cfg.rng_mode == SBMF_RNG_REFERENCE;
        // ---- alpha and w0 (fm_learn_mcmc.h:901-929, :627-668)
        const uint64_t nb = (NL + 1023) / 1024;
        double s[2];
        if (NL) {
            HIPCHK(fmm_esums(d_eu.as<double>(), NL, w0, d_part.as<double>(), st));
            HIPCHK(launch_sum_cols(d_part.as<double>(), (uint32_t)nb, 2, res, st));
        } else {
            HIPCHK(hipMemsetAsync(res, 0, 2 * sizeof(double), st));
        }
        if (R > 1)
            gather_sums(res, 2, s);  // every rank's {sum e^2, sum (e - w0)}, rank order
        else
            HIPCHK(hipMemcpyAsync(s, res, sizeof s, hipMemcpyDeviceToHost, st));
        if (do_multilevel) {
            // the hyperparameter draws' column sums (fm_learn_mcmc.h:951-1089) on the device, in
            // the host loops' order: w and v do not change before the draws that read them
            const double beta_0 = 1.0, gamma_0 = 1.0, mu_0 = 0.0;
            for (uint32_t c = 0; c <= K; ++c) {
                const double mu = c < K ? v_mu[c] : w_mu;
                h_mg[2 * c] = mu;
                h_mg[2 * c + 1] = beta_0 * (mu - mu_0) * (mu - mu_0) + gamma_0;
            }
            HIPCHK(hipMemcpyAsync(d_hmg.p, h_mg.data(), h_mg.size() * sizeof(double), hipMemcpyHostToDevice, st));
            HIPCHK(fmm_hsums(d_v.as<double>(), d_w.as<double>(), p, K, d_hmg.as<double2>(), d_hsum.as<double2>(), st));
            HIPCHK(hipMemcpyAsync(h_hs.data(), d_hsum.p, h_hs.size() * sizeof(double), hipMemcpyDeviceToHost, st));
            ++n_launch;
        }
        HIPCHK(hipStreamSynchronize(st));
        n_launch += 2;
        if (!do_multilevel) {
            alpha = 1.0;  // alpha_0
        } else {
            const double an = 1.0 + (double)N, gn = 1.0 + s[0];
            const double old = alpha;
            alpha = mt_gamma(g, an / 2.0) / (gn / 2.0);
            if (std::isnan(alpha) || std::isinf(alpha)) alpha = old;
        }
        if (k0) {
            const double reg0 = cfg.reg0;
            const double s2 = 1.0 / (reg0 + alpha * (double)N);
            const double m = -s2 * (alpha * s[1] - 0.0 * reg0);
            const double old = w0;
            w0 = do_sample ? gaussian(g, m, std::sqrt(s2)) : m;
            if (std::isnan(w0) || std::isinf(w0)) {
                w0 = old;
            } else {
                HIPCHK(fmm_shift(d_eu.as<double>(), NL, old - w0, st));
                ++n_launch;
            }
        }
        start_passes();
        // ---- w (:422-455): group hyperparameters, then users and items
        if (k1) {
            draw_hyper_w(g);
            if (do_sample) {
                if (ref) {
                    std::vector<double> z(p);
                    for (uint32_t a = 0; a < p; ++a) z[a] = leva_normal(g);
                    HIPCHK(hipMemcpyAsync(d_zw.p, z.data(), p * sizeof(double), hipMemcpyHostToDevice, st));
                    HIPCHK(hipStreamSynchronize(st));  // z is a local
                } else {
                    HIPCHK(launch_philox_fill<double>(d_zw.as<double>(), 1, 0, p, cfg.seed, it, TAG_FMM_W, st));
                }
            }
            for (int side = 0; side < 2; ++side) {
                FMPassArgs a = pass_args(side == 1);
                a.own = d_w.as<double>();
                a.z = d_zw.as<double>();
                a.zs = 1;
                a.zoff = 0;
                a.mu = w_mu;
                a.lambda = w_lambda;
                run_bins(a, side == 1, false);
            }
        }
        // ---- v (:526-621): per factor, users then items
        if (K) {
            draw_hyper_v(g);
            if (do_sample) {
                if (ref) {
                    std::vector<double> z((size_t)p * K);  // [a][K], drawn f-major (the reference's order)
                    for (uint32_t f = 0; f < K; ++f)
                        for (uint32_t a = 0; a < p; ++a) z[(size_t)a * K + f] = leva_normal(g);
                    HIPCHK(hipMemcpyAsync(d_zv.p, z.data(), z.size() * sizeof(double), hipMemcpyHostToDevice, st));
                    HIPCHK(hipStreamSynchronize(st));
                } else {
                    HIPCHK(launch_philox_fill<double>(d_zv.as<double>(), K, 0, p, cfg.seed, it, TAG_FMM_V, st));
                }
            }
            for (uint32_t f = 0; f < K; ++f) {
                double* col = d_v.as<double>() + (size_t)f * p;
                if (R > 1)  // one rank: the item pass reads the users' old values from d_rec
                    HIPCHK(hipMemcpyAsync(d_vold.p, col, (size_t)I * sizeof(double), hipMemcpyDeviceToDevice, st));
                for (int side = 0; side < 2; ++side) {
                    FMPassArgs a = pass_args(side == 1);
                    a.own = col;
                    a.partner_col = col;
                    a.vold_u = d_vold.as<double>();
                    a.z = d_zv.as<double>();
                    a.zs = K;
                    a.zoff = f;
                    a.mu = v_mu[f];
                    a.lambda = v_lambda[f];
                    run_bins(a, side == 1, true);
                }
            }
        }
        sync_users();  // several ranks: the owned users' fresh w and v to every rank
    }

    void run(uint32_t iters, sbmf_sweep_cb cb, void* user) {
        double* res = d_res.as<double>();
        for (uint32_t k = 0; k < iters; ++k) {
            n_launch = 0;
            HIPCHK(hipEventRecord(ev[0], st));
            if (cfg.rng_mode == SBMF_RNG_REFERENCE) {
                sweep_draws(grand);
            } else {
                PhiloxStream ps(cfg.seed, it, 3);
                sweep_draws(ps);
            }
            HIPCHK(hipEventRecord(ev[1], st));
            // ---- predict train and test, evaluate (fm_learn_mcmc_simultaneous.h:134-245)
            predict_train();
            if (NL)
                HIPCHK(launch_sum(d_part.as<double>(), (NL + 255) / 256, res + 2, d_scratch.as<double>(), st));
            else
                HIPCHK(hipMemsetAsync(res + 2, 0, sizeof(double), st));
            const uint64_t tb = (T + 255) / 256;
            if (T) {
                HIPCHK(fmm_predict_test(predict_args(), d_su.as<uint32_t>(), d_si.as<uint32_t>(), d_sy.as<float>(), T,
                                        (double)(it + 1), d_pthis.as<double>(), d_sum.as<double>(),
                                        d_tpart.as<double>(), st));
                HIPCHK(launch_sum_cols(d_tpart.as<double>(), (uint32_t)tb, 2, res + 3, st));
                n_launch += 2;
            }
            HIPCHK(hipEventRecord(ev[2], st));
            double h[3] = {0, 0, 0};
            HIPCHK(hipMemcpyAsync(h, res + 2, sizeof h, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            if (R > 1) gather_sums(res + 2, 1, h);  // the train sum of every rank (test: every rank has all)
            float ms0 = 0.f, ms1 = 0.f;
            HIPCHK(hipEventElapsedTime(&ms0, ev[0], ev[1]));
            HIPCHK(hipEventElapsedTime(&ms1, ev[1], ev[2]));
            sbmf_sweep_info info{};
            info.sweep = it;
            info.collected = 1;
            info.rmse_train = std::sqrt(h[0] / (double)N);
            info.rmse_avg = T ? std::sqrt(h[1] / (double)T) : NAN;
            info.rmse_this = T ? std::sqrt(h[2] / (double)T) : NAN;
            info.tau = alpha;
            info.ms_sweep = ms0;
            info.ms_eval = ms1;
            ++it;
            if (cb && cb(&info, user)) break;
        }
    }
};

FMLearner* fmm_create(const sbmf_config& c, uint64_t n, const uint32_t* u, const uint32_t* i, const double* r,
                      uint64_t nt, const uint32_t* tu, const uint32_t* ti, const double* tr, uint32_t I, uint32_t J,
                      hipStream_t st, Comm* comm) {
    std::unique_ptr<FMLearner> L(new FMLearner());
    L->cfg = c;
    L->st = st;
    if (comm && comm->nranks() > 1) {
        L->comm = comm;
        L->R = comm->nranks();
    }
    L->K = c.num_factor;
    L->Kp = (L->K + 15) / 16 * 16;
    L->I = I;
    L->J = J;
    L->N = n;
    L->T = nt;
    L->k0 = (c.libfm_dim & 1u) ? 1 : 0;
    L->k1 = (c.libfm_dim & 2u) ? 1 : 0;
    const bool als = c.method == SBMF_METHOD_ALS;
    L->do_sample = als ? 0 : 1;  // libfm.cpp:132-136
    L->do_multilevel = als ? 0 : 1;
    if (n >= 0xffffffffull) fail(SBMF_E_ARG, "more than 2^32-1 ratings are not supported");
    // libFM attribute layout: user u -> u, item i -> I + i; num_feature = largest id + 1 (Data.h:221),
    // num_all_attribute = max(train, test) + 1 (libfm.cpp:330)
    uint32_t imax_tr = 0, imax_te = 0;
    for (uint64_t x = 0; x < n; ++x) imax_tr = std::max(imax_tr, i[x]);
    for (uint64_t x = 0; x < nt; ++x) imax_te = std::max(imax_te, ti[x]);
    L->p_train = I + imax_tr + 1;
    L->p_test = nt ? I + imax_te + 1 : 0;
    L->p = std::max(L->p_train, L->p_test) + 1;
    L->RI = L->p - I;
    const uint32_t p = L->p, K = L->K;
    // DATA_FLOAT targets (fm_data.h:25) and the train range (Data.h:200-203)
    std::vector<float> y(n), ys(nt);
    float mn = 3.4028234663852886e38f, mx = -3.4028234663852886e38f;
    for (uint64_t x = 0; x < n; ++x) {
        y[x] = (float)r[x];
        mn = std::min(y[x], mn);
        mx = std::max(y[x], mx);
    }
    for (uint64_t x = 0; x < nt; ++x) ys[x] = (float)tr[x];
    L->lo = mn;
    L->hi = mx;
    // several ranks: the user ranges (sbmf_partition_rows over the users' rating counts);
    // a rank keeps the cases of its users only
    L->ubounds.assign(L->R + 1, 0);
    L->ubounds[L->R] = I;
    uint32_t u0 = 0, u1 = I;
    std::vector<uint8_t> mine(n, 1);
    L->NL = n;
    if (L->R > 1) {
        std::vector<uint32_t> cnt(I + 1, 0);
        for (uint64_t x = 0; x < n; ++x) cnt[u[x] + 1]++;
        for (uint32_t k = 0; k < I; ++k) cnt[k + 1] += cnt[k];
        if (sbmf_partition_rows(cnt.data(), I, L->R, L->ubounds.data()) != SBMF_OK)
            fail(SBMF_E_ARG, "libFM learner: user partition failed");
        u0 = (uint32_t)L->ubounds[comm->rank()];
        u1 = (uint32_t)L->ubounds[comm->rank() + 1];
        L->NL = 0;
        for (uint64_t x = 0; x < n; ++x) {
            mine[x] = u[x] >= u0 && u[x] < u1;
            L->NL += mine[x];
        }
    }
    const uint64_t nl = L->NL;
    // user order (CSR over users, cases in file order) and item order (CSC over item rows [0, RI)),
    // over this rank's cases
    std::vector<uint32_t> uptr(I + 1, 0), iptr(L->RI + 1, 0);
    for (uint64_t x = 0; x < n; ++x) {
        if (!mine[x]) continue;
        uptr[u[x] + 1]++;
        iptr[i[x] + 1]++;
    }
    for (uint32_t k = 0; k < I; ++k) uptr[k + 1] += uptr[k];
    for (uint32_t k = 0; k < L->RI; ++k) iptr[k + 1] += iptr[k];
    std::vector<uint32_t> upos(n), ipos(n), uown(nl), upart(nl), ipart(nl), uperm(nl), iperm(nl);
    std::vector<float> uy(nl);
    {
        std::vector<uint32_t> fu(uptr.begin(), uptr.end() - 1), fi(iptr.begin(), iptr.end() - 1);
        for (uint64_t x = 0; x < n; ++x) {
            if (!mine[x]) continue;
            upos[x] = fu[u[x]]++;
            ipos[x] = fi[i[x]]++;
        }
    }
    for (uint64_t x = 0; x < n; ++x) {
        if (!mine[x]) continue;
        uown[upos[x]] = u[x];
        upart[upos[x]] = i[x];
        uy[upos[x]] = y[x];
        uperm[upos[x]] = ipos[x];
        ipart[ipos[x]] = u[x];
        iperm[ipos[x]] = upos[x];
    }
    // rows binned by length: <= 256 cases 64 threads, <= 4096 256, longer 1024
    // (users: this rank's range; items: every item row, each rank over its own cases;
    // SBMF_FMM_LONG moves the long-row bound, for tests of the chunked long rows)
    uint32_t longb = 4096;
    if (const char* e = std::getenv("SBMF_FMM_LONG")) longb = (uint32_t)std::max(256, std::atoi(e));
    auto bin = [longb](const std::vector<uint32_t>& ptr, uint32_t r0, uint32_t r1, FMBin* b) {
        b[0].tpr = 64;
        b[1].tpr = 256;
        b[2].tpr = 1024;
        for (uint32_t k = r0; k < r1; ++k) {
            const uint32_t len = ptr[k + 1] - ptr[k];
            b[len <= 256 ? 0 : len <= longb ? 1 : 2].rows.push_back(k);
        }
        // longest rows first: blocks start roughly in index order, so a long row dispatched
        // late would set the launch's tail (one block per row; rows are independent, so the
        // order changes no result)
        for (int j = 0; j < 3; ++j)
            std::stable_sort(b[j].rows.begin(), b[j].rows.end(),
                             [&](uint32_t x, uint32_t y) { return ptr[x + 1] - ptr[x] > ptr[y + 1] - ptr[y]; });
    };
    bin(uptr, u0, u1, L->ubins);
    bin(iptr, 0, L->RI, L->ibins);
    for (FMBin* bs : {L->ubins, L->ibins})
        for (int k = 0; k < 3; ++k) upload(bs[k].d_rows, bs[k].rows, st);
    // one rank: the long-row bin's rows cut into chunks of at most `chunk` cases (the
    // 1024-thread workgroup's four cases per thread), the chunks of one row consecutive
    // (SBMF_FMM_CHUNK overrides the size, 0 turns the chunks off)
    uint32_t chunk = 4096;
    if (const char* e = std::getenv("SBMF_FMM_CHUNK")) chunk = (uint32_t)std::max(0, std::atoi(e));
    if (L->R == 1 && chunk)
        for (FMBin* bs : {L->ubins, L->ibins}) {
            FMBin& b = bs[2];
            const std::vector<uint32_t>& pt = bs == L->ubins ? uptr : iptr;
            b.chunks.clear();
            b.cfirst.assign(1, 0);
            for (uint32_t i = 0; i < (uint32_t)b.rows.size(); ++i) {
                const uint32_t r = b.rows[i], c0 = pt[r], len = pt[r + 1] - c0;
                const uint32_t nch = (len + chunk - 1) / chunk;
                for (uint32_t c = 0; c < nch; ++c) {
                    const uint32_t cb = c0 + (uint32_t)((uint64_t)len * c / nch);
                    const uint32_t ce = c0 + (uint32_t)((uint64_t)len * (c + 1) / nch);
                    b.chunks.push_back(make_uint4(r, cb, ce - cb, i));
                }
                b.cfirst.push_back((uint32_t)b.chunks.size());
            }
            if (b.chunks.empty()) continue;
            upload(b.d_chunks, b.chunks, st);
            upload(b.d_cfirst, b.cfirst, st);
            b.d_csums.alloc(b.chunks.size() * sizeof(double2));
            b.d_cdelta.alloc(b.rows.size() * sizeof(double4));
            b.d_cqq.alloc(b.rows.size() * sizeof(double2));
        }
    upload(L->d_uptr, uptr, st);
    upload(L->d_iptr, iptr, st);
    upload(L->d_upart, upart, st);
    upload(L->d_ipart, ipart, st);
    upload(L->d_uperm, uperm, st);
    upload(L->d_iperm, iperm, st);
    upload(L->d_uown, uown, st);
    upload(L->d_uy, uy, st);
    std::vector<uint32_t> su(tu, tu + nt), si(ti, ti + nt);
    upload(L->d_su, su, st);
    upload(L->d_si, si, st);
    upload(L->d_sy, ys, st);
    L->d_eu.alloc(std::max<uint64_t>(nl, 1) * sizeof(double));
    L->d_ei.alloc(std::max<uint64_t>(nl, 1) * sizeof(double));
    if (L->R > 1) {
        L->d_sums.alloc((size_t)std::max(L->RI, 1u) * sizeof(double2));
        L->d_recvg.alloc((size_t)L->R * std::max(L->RI, 1u) * sizeof(double2));
        L->d_delta.alloc((size_t)std::max(L->RI, 1u) * sizeof(double4));
        L->d_recv.alloc((size_t)L->R * 4 * sizeof(double));
    }
    L->d_w.alloc((size_t)p * sizeof(double));
    L->d_v.alloc(std::max<size_t>((size_t)K * p, 1) * sizeof(double));
    L->d_vT.alloc(std::max<size_t>((size_t)p * L->Kp, 1) * sizeof(double));
    HIPCHK(hipMemsetAsync(L->d_vT.p, 0, L->d_vT.bytes, st));
    L->d_vold.alloc((size_t)std::max(I, 1u) * sizeof(double));
    L->d_rec.alloc((size_t)p * sizeof(double2));
    L->d_zw.alloc((size_t)p * sizeof(double));
    L->d_zv.alloc(std::max<size_t>((size_t)K * p, 1) * sizeof(double));
    L->d_pthis.alloc(std::max<uint64_t>(nt, 1) * sizeof(double));
    L->d_sum.alloc(std::max<uint64_t>(nt, 1) * sizeof(double));
    HIPCHK(hipMemsetAsync(L->d_sum.p, 0, L->d_sum.bytes, st));
    L->d_part.alloc((std::max<uint64_t>((nl + 255) / 256, 2 * ((nl + 1023) / 1024)) + 2) * sizeof(double));
    L->d_tpart.alloc((2 * ((nt + 255) / 256) + 2) * sizeof(double));
    L->d_res.alloc(8 * sizeof(double));
    L->d_hmg.alloc(2 * ((size_t)K + 1) * sizeof(double));
    L->d_hsum.alloc(2 * ((size_t)K + 1) * sizeof(double));
    L->h_mg.assign(2 * ((size_t)K + 1), 0.0);
    L->h_hs.assign(2 * ((size_t)K + 1), 0.0);
    L->d_scratch.alloc(((nl + 255) / 256 / 1024 + 16) * 2 * sizeof(double));
    L->v_mu.assign(K, 0.0);
    // fm_learn_mcmc::init (:1099-1116) and the -regular values (libfm.cpp:484-513)
    L->w_lambda = c.regw;
    L->v_lambda.assign(K, c.regv);
    // model init and the starting predictions (fm_learn_mcmc_simultaneous.h:75-93)
    if (c.rng_mode == SBMF_RNG_REFERENCE) {
        L->grand.seed_((unsigned)c.seed);  // libfm.cpp:124 srand(time) -- here the pinned seed
        L->init_model(L->grand);
    } else {
        PhiloxStream ps(c.seed, 0xffffffffu, TAG_FMM_INIT);
        L->init_model(ps);
    }
    HIPCHK(hipMemcpyAsync(L->d_w.p, L->h_w.data(), (size_t)p * sizeof(double), hipMemcpyHostToDevice, st));
    if (K) HIPCHK(hipMemcpyAsync(L->d_v.p, L->h_v.data(), (size_t)K * p * sizeof(double), hipMemcpyHostToDevice, st));
    L->predict_train();
    HIPCHK(hipStreamSynchronize(st));
    std::vector<double>().swap(L->h_v);  // the host copies served the upload only
    std::vector<double>().swap(L->h_w);
    for (auto& e : L->ev) event_create(&e);
    return L.release();
}

void fmm_destroy(FMLearner* L) { delete L; }
void fmm_run(FMLearner* L, uint32_t iters, sbmf_sweep_cb cb, void* user) { L->run(iters, cb, user); }

// fm_learn_mcmc::predict (:357-380): the running sum over the iterations run
// (MCMC) or the last prediction (ALS), clamped to the train range
void fmm_predict_out(FMLearner* L, double* out) {
    HIPCHK(hipStreamSynchronize(L->st));
    if (!L->T) return;
    HIPCHK(hipMemcpy(out, (L->do_sample ? L->d_sum : L->d_pthis).p, L->T * sizeof(double), hipMemcpyDeviceToHost));
    for (uint64_t t = 0; t < L->T; ++t) {
        double o = L->do_sample ? out[t] / std::max(1u, L->it) : out[t];
        o = std::min(L->hi, o);
        o = std::max(L->lo, o);
        out[t] = o;
    }
}
void fmm_factors(FMLearner* L, double* U, double* V) {
    HIPCHK(hipStreamSynchronize(L->st));
    std::vector<double> h((size_t)L->K * L->p);
    if (L->K) HIPCHK(hipMemcpy(h.data(), L->d_v.p, h.size() * sizeof(double), hipMemcpyDeviceToHost));
    for (uint32_t f = 0; f < L->K; ++f) {
        if (U)
            for (uint32_t a = 0; a < L->I; ++a) U[(size_t)a * L->K + f] = h[(size_t)f * L->p + a];
        if (V)  // items past libFM's attribute count (sbmf_set_dims with trailing unrated ids) have no factors: 0
            for (uint32_t a = 0; a < L->J; ++a) V[(size_t)a * L->K + f] = a < L->RI ? h[(size_t)f * L->p + L->I + a] : 0.0;
    }
}
void fmm_biases(FMLearner* L, double* bu, double* bv, double* b0) {
    HIPCHK(hipStreamSynchronize(L->st));
    std::vector<double> h(L->p);
    HIPCHK(hipMemcpy(h.data(), L->d_w.p, h.size() * sizeof(double), hipMemcpyDeviceToHost));
    if (bu) std::copy(h.begin(), h.begin() + L->I, bu);
    if (bv) {  // as fmm_factors: items past the attribute count read 0
        const uint32_t nj = std::min(L->J, L->RI);
        std::copy(h.begin() + L->I, h.begin() + L->I + nj, bv);
        std::fill(bv + nj, bv + L->J, 0.0);
    }
    if (b0) *b0 = L->w0;
}
// [v_lambda (K) | v_mu (K) | w_lambda, w_mu, 0... (K) | 0 (K)] and alpha
void fmm_hyper_out(FMLearner* L, double* h4k, double* alpha) {
    const uint32_t K = L->K;
    if (h4k) {
        std::fill(h4k, h4k + 4 * (size_t)K, 0.0);
        std::copy(L->v_lambda.begin(), L->v_lambda.end(), h4k);
        std::copy(L->v_mu.begin(), L->v_mu.end(), h4k + K);
        h4k[2 * K] = L->w_lambda;
        if (K > 1) h4k[2 * K + 1] = L->w_mu;
    }
    if (alpha) *alpha = L->alpha;
}
uint32_t fmm_launches(const FMLearner* L) { return L->n_launch; }
uint32_t fmm_num_attribute(const FMLearner* L) { return L->p; }

}  // namespace sbmf
