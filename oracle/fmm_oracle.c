/* fmm_oracle.c -- TEST INFRASTRUCTURE ONLY (checker and CPU baseline; never
 * linked into the product).
 *
 * Serial C restatement of libFM's MCMC / ALS learner as the reference's
 * `bin/libFM -method mcmc|als` runs it on rating data
 * (/root/reference/src/libfm/src/fm_learn_mcmc.h, fm_learn_mcmc_simultaneous.h,
 * driven by libfm.cpp), for cases with exactly two one-hot attributes a0 < a1
 * (libFM text "r a0:1 a1:1"; users-first rating data puts the user at a0 = u
 * and the item at a1 = I + i).  No relations, no -meta file: one attribute
 * group.  Every block cites the reference lines it follows; the arithmetic
 * keeps the reference's operation order so the results can be pinned
 * bit-for-bit to libFM compiled from its own sources (oracle/Makefile ref,
 * oracle/make_golden.py).
 *
 * RNG: glibc rand() through the same Leva normal / Marsaglia-Tsang gamma as
 * sbpmf_oracle.c (src/util/random.h:118-176), seeded like libfm.cpp:124
 * (srand of the pinned time value).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "sbpmf_oracle.h"

/* random.h:166-172: the mean without a draw when stdev is 0 or NaN */
static double g_gaussian(double mean, double stdev) {
    if (stdev == 0.0 || isnan(stdev)) return mean;
    return mean + stdev * oracle_ran_gaussian();
}
static double g_gamma(double alpha, double beta) { return oracle_ran_gamma(alpha) / beta; } /* random.h:146-148 */

void oracle_fmm_config_default(oracle_fmm_config *c) {
    memset(c, 0, sizeof(*c));
    c->K = 8;
    c->iters = 100;
    c->seed = 1;
    c->k0 = 1;
    c->k1 = 1;
    c->do_sample = 1;
    c->do_multilevel = 1;
    c->init_stdev = 0.1; /* libfm.cpp:127 */
}

/* libFM's transpose (Data::create_data_t, Data.h:472-...): per attribute, its
 * cases in ascending case order. */
typedef struct {
    uint32_t *ptr, *cs;
} tcols;
static void build_t(uint64_t n, const uint32_t *a0, const uint32_t *a1, uint32_t rows, tcols *T) {
    T->ptr = (uint32_t *)calloc((size_t)rows + 1, sizeof(uint32_t));
    T->cs = (uint32_t *)malloc((2 * n + 1) * sizeof(uint32_t));
    for (uint64_t c = 0; c < n; ++c) {
        T->ptr[a0[c] + 1]++;
        T->ptr[a1[c] + 1]++;
    }
    for (uint32_t r = 0; r < rows; ++r) T->ptr[r + 1] += T->ptr[r];
    uint32_t *fill = (uint32_t *)malloc((size_t)rows * sizeof(uint32_t));
    memcpy(fill, T->ptr, (size_t)rows * sizeof(uint32_t));
    for (uint64_t c = 0; c < n; ++c) {
        T->cs[fill[a0[c]]++] = (uint32_t)c;
        T->cs[fill[a1[c]]++] = (uint32_t)c;
    }
    free(fill);
}

/* predict_data_and_write_to_eterms (fm_learn_mcmc.h:117-348) for one data
 * set without relations: e = w0 + sum w x + 1/2 sum_f [(sum_i v x)^2 - sum_i
 * v^2 x^2], accumulated stage by stage in the reference's order (attribute
 * rows ascending, their cases ascending).  x = 1.0f. */
static void predict_eterms(uint32_t K, uint32_t p, int k0, int k1, double w0, const double *w, const double *v,
                           uint64_t n, const tcols *T, uint32_t trows, double *e, double *q) {
    const float x = 1.0f;
    for (uint64_t c = 0; c < n; ++c) e[c] = 0.0, q[c] = 0.0;
    for (uint32_t f = 0; f < K; ++f) { /* (1) */
        const double *vf = v + (size_t)f * p;
        for (uint32_t a = 0; a < trows; ++a)
            for (uint32_t k = T->ptr[a]; k < T->ptr[a + 1]; ++k) q[T->cs[k]] += vf[a] * x;
        for (uint64_t c = 0; c < n; ++c) {
            e[c] += 0.5 * q[c] * q[c];
            q[c] = 0.0;
        }
    }
    for (uint32_t f = 0; f < K; ++f) { /* (2) */
        const double *vf = v + (size_t)f * p;
        for (uint32_t a = 0; a < trows; ++a)
            for (uint32_t k = T->ptr[a]; k < T->ptr[a + 1]; ++k) q[T->cs[k]] -= 0.5 * vf[a] * vf[a] * x * x;
    }
    if (k1) /* (3) */
        for (uint32_t a = 0; a < trows; ++a)
            for (uint32_t k = T->ptr[a]; k < T->ptr[a + 1]; ++k) q[T->cs[k]] += w[a] * x;
    for (uint64_t c = 0; c < n; ++c) { /* merge */
        e[c] = e[c] + q[c];
        if (k0) e[c] += w0;
        q[c] = 0.0;
    }
}

/* One group of attributes (no -meta): the group hyperparameter draws,
 * fm_learn_mcmc.h:951-1089. */
static void draw_hyper_w(const oracle_fmm_config *cf, uint32_t p, const double *w, double *w_mu, double *w_lambda) {
    const double alpha_0 = 1.0, gamma_0 = 1.0, beta_0 = 1.0, mu_0 = 0.0;
    if (cf->do_multilevel) { /* draw_w_lambda :979-1009 */
        double g = beta_0 * (*w_mu - mu_0) * (*w_mu - mu_0) + gamma_0;
        for (uint32_t i = 0; i < p; ++i) g += (w[i] - *w_mu) * (w[i] - *w_mu);
        const double a = alpha_0 + p + 1;
        const double old = *w_lambda;
        *w_lambda = cf->do_sample ? g_gamma(a / 2.0, g / 2.0) : a / g;
        if (isnan(*w_lambda) || isinf(*w_lambda)) *w_lambda = old;
    }
    if (!cf->do_multilevel) { /* draw_w_mu :951-977 */
        *w_mu = mu_0;
    } else {
        double m = 0.0;
        for (uint32_t i = 0; i < p; ++i) m += w[i];
        m = (m + beta_0 * mu_0) / (p + beta_0);
        const double s2 = 1.0 / ((p + beta_0) * *w_lambda);
        const double old = *w_mu;
        *w_mu = cf->do_sample ? g_gaussian(m, sqrt(s2)) : m;
        if (isnan(*w_mu) || isinf(*w_mu)) *w_mu = old;
    }
}
static void draw_hyper_v(const oracle_fmm_config *cf, uint32_t p, const double *v, double *v_mu, double *v_lambda) {
    const double alpha_0 = 1.0, gamma_0 = 1.0, beta_0 = 1.0, mu_0 = 0.0;
    const uint32_t K = cf->K;
    if (cf->do_multilevel) { /* draw_v_lambda :1043-1089 (per f; a NaN/inf returns from the whole draw) */
        for (uint32_t f = 0; f < K; ++f) {
            double g = beta_0 * (v_mu[f] - mu_0) * (v_mu[f] - mu_0) + gamma_0;
            for (uint32_t i = 0; i < p; ++i) g += (v[(size_t)f * p + i] - v_mu[f]) * (v[(size_t)f * p + i] - v_mu[f]);
            const double a = alpha_0 + p + 1;
            const double old = v_lambda[f];
            v_lambda[f] = cf->do_sample ? g_gamma(a / 2.0, g / 2.0) : a / g;
            if (isnan(v_lambda[f]) || isinf(v_lambda[f])) {
                v_lambda[f] = old;
                break;
            }
        }
    }
    if (!cf->do_multilevel) { /* draw_v_mu :1011-1041 */
        for (uint32_t f = 0; f < K; ++f) v_mu[f] = mu_0;
    } else {
        for (uint32_t f = 0; f < K; ++f) {
            double m = 0.0;
            for (uint32_t i = 0; i < p; ++i) m += v[(size_t)f * p + i];
            m = (m + beta_0 * mu_0) / (p + beta_0);
            const double s2 = 1.0 / ((p + beta_0) * v_lambda[f]);
            const double old = v_mu[f];
            v_mu[f] = cf->do_sample ? g_gaussian(m, sqrt(s2)) : m;
            if (isnan(v_mu[f]) || isinf(v_mu[f])) {
                v_mu[f] = old;
                break;
            }
        }
    }
}

int oracle_fmm_run(const oracle_fmm_config *cf, uint64_t n, const uint32_t *ta0, const uint32_t *ta1,
                   const double *ty, uint64_t nt, const uint32_t *sa0, const uint32_t *sa1, const double *sy,
                   uint32_t p_train, uint32_t p_test, oracle_fmm_result *res) {
    const uint32_t K = cf->K;
    /* libfm.cpp:330 (num_feature = max id + 1, Data.h:221) */
    const uint32_t p = (p_train > p_test ? p_train : p_test) + 1;
    if (n == 0) return -1;
    for (uint64_t c = 0; c < n; ++c)
        if (ta0[c] >= ta1[c] || ta1[c] >= p_train) return -2;
    for (uint64_t c = 0; c < nt; ++c)
        if (sa0[c] >= sa1[c] || sa1[c] >= p_test) return -2;
    /* DATA_FLOAT targets (fm_data.h:25); min/max over the train file (Data.h:200-203) */
    float *y = (float *)malloc(n * sizeof(float)), *yt = (float *)malloc((nt ? nt : 1) * sizeof(float));
    float mn = 3.4028234663852886e38f, mx = -3.4028234663852886e38f;
    for (uint64_t c = 0; c < n; ++c) {
        y[c] = (float)ty[c];
        if (y[c] < mn) mn = y[c];
        if (y[c] > mx) mx = y[c];
    }
    for (uint64_t c = 0; c < nt; ++c) yt[c] = (float)sy[c];
    const double min_target = mn, max_target = mx;
    tcols T, Tt;
    build_t(n, ta0, ta1, p_train, &T);
    build_t(nt, sa0, sa1, p_test, &Tt);

    /* model init: fm_model::init (fm_model.h:87-96: v ~ N(mean, init_stdev),
     * f-major [K][p]) then, for mcmc, w.init_normal (libfm.cpp:412;
     * DVectorDouble::init_normal, matrix.h:334-338: N(mean, stdev)); w0 = 0 */
    srand(cf->seed);
    double *v = (double *)malloc((size_t)K * p * sizeof(double) + 8);
    double *w = (double *)malloc((size_t)p * sizeof(double));
    for (uint32_t f = 0; f < K; ++f)
        for (uint32_t a = 0; a < p; ++a) v[(size_t)f * p + a] = g_gaussian(0.0, cf->init_stdev);
    for (uint32_t a = 0; a < p; ++a) w[a] = g_gaussian(0.0, cf->init_stdev);
    double w0 = 0.0;
    /* fm_learn_mcmc::init (:1099-1116) then libfm.cpp:484-513 (-regular) */
    const double alpha_0 = 1.0, gamma_0 = 1.0, w0_mean_0 = 0.0;
    double alpha = 1.0, w_mu = 0.0, w_lambda = cf->regw;
    const double reg0 = cf->reg0;
    double *v_mu = (double *)calloc(K ? K : 1, sizeof(double)), *v_lambda = (double *)malloc((K ? K : 1) * sizeof(double));
    for (uint32_t f = 0; f < K; ++f) v_lambda[f] = cf->regv;

    double *e = (double *)malloc(n * sizeof(double)), *q = (double *)malloc(n * sizeof(double));
    double *et = (double *)malloc((nt ? nt : 1) * sizeof(double)), *qt = (double *)malloc((nt ? nt : 1) * sizeof(double));
    double *sum_all = (double *)calloc(nt ? nt : 1, sizeof(double)), *pthis = (double *)calloc(nt ? nt : 1, sizeof(double));
    const float x = 1.0f;

    /* fm_learn_mcmc_simultaneous::_learn :75-93 */
    predict_eterms(K, p, cf->k0, cf->k1, w0, w, v, n, &T, p_train, e, q);
    predict_eterms(K, p, cf->k0, cf->k1, w0, w, v, nt, &Tt, p_test, et, qt);
    for (uint64_t c = 0; c < n; ++c) e[c] = e[c] - y[c];

    uint32_t it;
    for (it = 0; it < cf->iters; ++it) {
        /* ---- draw_all (fm_learn_mcmc.h:411-623) ---- */
        /* draw_alpha :901-929 */
        if (!cf->do_multilevel) {
            alpha = alpha_0;
        } else {
            const double an = alpha_0 + (double)n;
            double gn = gamma_0;
            for (uint64_t c = 0; c < n; ++c) gn += e[c] * e[c];
            const double old = alpha;
            alpha = g_gamma(an / 2.0, gn / 2.0);
            if (isnan(alpha) || isinf(alpha)) alpha = old;
        }
        if (cf->k0) { /* draw_w0 :627-668 */
            double m = 0.0;
            for (uint64_t c = 0; c < n; ++c) m += e[c] - w0;
            const double s2 = 1.0 / (reg0 + alpha * (double)n);
            m = -s2 * (alpha * m - w0_mean_0 * reg0);
            const double old = w0;
            w0 = cf->do_sample ? g_gaussian(m, sqrt(s2)) : m;
            if (isnan(w0) || isinf(w0)) {
                w0 = old;
            } else {
                for (uint64_t c = 0; c < n; ++c) e[c] -= (old - w0);
            }
        }
        if (cf->k1) { /* :422-455 */
            draw_hyper_w(cf, p, w, &w_mu, &w_lambda);
            for (uint32_t a = 0; a < p; ++a) { /* draw_w :670-719 (attributes past the train rows: empty) */
                const uint32_t b = a < p_train ? T.ptr[a] : 0, en = a < p_train ? T.ptr[a + 1] : 0;
                double s2 = 0.0, m = 0.0;
                for (uint32_t k = b; k < en; ++k) {
                    const uint32_t c = T.cs[k];
                    m += x * (e[c] - w[a] * x);
                    s2 += x * x;
                }
                s2 = 1.0 / (w_lambda + alpha * s2);
                m = -s2 * (alpha * m - w_mu * w_lambda);
                const double old = w[a];
                if (isnan(s2) || isinf(s2))
                    w[a] = 0.0;
                else
                    w[a] = cf->do_sample ? g_gaussian(m, sqrt(s2)) : m;
                if (isnan(w[a]) || isinf(w[a])) {
                    w[a] = old;
                    continue;
                }
                for (uint32_t k = b; k < en; ++k) e[T.cs[k]] -= (double)x * (old - w[a]);
            }
        }
        if (K > 0) draw_hyper_v(cf, p, v, v_mu, v_lambda); /* :526-536 */
        for (uint32_t f = 0; f < K; ++f) { /* :538-621 */
            double *vf = v + (size_t)f * p;
            for (uint64_t c = 0; c < n; ++c) q[c] = 0.0;
            for (uint32_t a = 0; a < p_train; ++a) /* add_main_q :385-409 */
                for (uint32_t k = T.ptr[a]; k < T.ptr[a + 1]; ++k) q[T.cs[k]] += vf[a] * x;
            for (uint32_t a = 0; a < p; ++a) { /* draw_v :780-835 */
                const uint32_t b = a < p_train ? T.ptr[a] : 0, en = a < p_train ? T.ptr[a + 1] : 0;
                double s2 = 0.0, m = 0.0;
                for (uint32_t k = b; k < en; ++k) {
                    const uint32_t c = T.cs[k];
                    const double h = x * (q[c] - x * vf[a]);
                    m += h * e[c];
                    s2 += h * h;
                }
                m -= vf[a] * s2;
                s2 = 1.0 / (v_lambda[f] + alpha * s2);
                m = -s2 * (alpha * m - v_mu[f] * v_lambda[f]);
                const double old = vf[a];
                if (isnan(s2) || isinf(s2))
                    vf[a] = 0.0;
                else
                    vf[a] = cf->do_sample ? g_gaussian(m, sqrt(s2)) : m;
                if (isnan(vf[a]) || isinf(vf[a])) {
                    vf[a] = old;
                    continue;
                }
                for (uint32_t k = b; k < en; ++k) {
                    const uint32_t c = T.cs[k];
                    const double h = x * (q[c] - x * old);
                    q[c] -= x * (old - vf[a]);
                    e[c] -= h * (old - vf[a]);
                }
            }
        }
        /* ---- predict train and test, evaluate (fm_learn_mcmc_simultaneous.h:134-245) ---- */
        predict_eterms(K, p, cf->k0, cf->k1, w0, w, v, n, &T, p_train, e, q);
        predict_eterms(K, p, cf->k0, cf->k1, w0, w, v, nt, &Tt, p_test, et, qt);
        for (uint64_t c = 0; c < nt; ++c) {
            double pr = et[c];
            pthis[c] = pr;
            pr = pr < max_target ? pr : max_target;
            pr = pr > min_target ? pr : min_target;
            sum_all[c] += pr;
        }
        double rmse_train = 0.0;
        for (uint64_t c = 0; c < n; ++c) {
            double pr = e[c];
            pr = pr < max_target ? pr : max_target;
            pr = pr > min_target ? pr : min_target;
            const double err = pr - y[c];
            rmse_train += err * err;
            e[c] = e[c] - y[c];
        }
        rmse_train = sqrt(rmse_train / n);
        /* _evaluate :307-325 */
        double se_all = 0.0, se_this = 0.0;
        const double norm = 1.0 / (it + 1);
        for (uint64_t c = 0; c < nt; ++c) {
            double pa = sum_all[c] * norm, pt = pthis[c] * 1.0;
            pa = pa < max_target ? pa : max_target;
            pa = pa > min_target ? pa : min_target;
            pt = pt < max_target ? pt : max_target;
            pt = pt > min_target ? pt : min_target;
            se_all += (pa - yt[c]) * (pa - yt[c]);
            se_this += (pt - yt[c]) * (pt - yt[c]);
        }
        if (res->rmse_test && it < res->cap) res->rmse_test[it] = sqrt(se_all / nt);
        if (res->rmse_this && it < res->cap) res->rmse_this[it] = sqrt(se_this / nt);
        if (res->rmse_train && it < res->cap) res->rmse_train[it] = rmse_train;
        if (res->alpha && it < res->cap) res->alpha[it] = alpha;
    }
    res->iters_done = it;
    res->num_attribute = p;
    res->w0 = w0;
    res->min_target = min_target;
    res->max_target = max_target;
    if (res->w) memcpy(res->w, w, (size_t)p * sizeof(double));
    if (res->v) memcpy(res->v, v, (size_t)K * p * sizeof(double));
    if (res->pred) /* fm_learn_mcmc::predict :357-380 (the -out file) */
        for (uint64_t c = 0; c < nt; ++c) {
            double o = cf->do_sample ? sum_all[c] / cf->iters : pthis[c];
            o = o < max_target ? o : max_target;
            o = o > min_target ? o : min_target;
            res->pred[c] = o;
        }
    free(y), free(yt), free(v), free(w), free(v_mu), free(v_lambda), free(e), free(q), free(et), free(qt);
    free(sum_all), free(pthis);
    free(T.ptr), free(T.cs), free(Tt.ptr), free(Tt.cs);
    return 0;
}
