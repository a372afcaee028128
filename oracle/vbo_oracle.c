/*
 * vbo_oracle.c -- CPU restatement of the reference's online variational-Bayes
 * learner (`bin/libFM -method vb_online`) for rating data: every case has
 * exactly one user feature and one item feature, both with value 1.
 *
 * TEST INFRASTRUCTURE ONLY (like sbpmf_oracle.c): used by tests/ and by
 * bench.py's cpu_baseline leg; the product path never links or calls it.
 *
 * Pinning: per-epoch test RMSE checked bit-for-bit ("%.17g") against the
 * reference learner itself, compiled from the unmodified headers under
 * /root/reference and driven by oracle/ref_vbo_harness.cpp (fixtures
 * tests/golden/ref_vbo_*.txt, generator oracle/make_golden.py).
 *
 * What it restates (file:line under /root/reference/src):
 *   start state        libfm/libfm.cpp:387,433 (fm_model v and w draws, which
 *                      only advance the stream here), libfm/src/
 *                      fm_learn_vb_online.h:841-946 (alpha, sigma_0, mu/sigma
 *                      dash, natural parameters, step sizes (t0 + t)^-0.5),
 *                      util/matrix.h:358-380 (0.1 * N(0,1) means)
 *   epoch / batches    fm_learn_vb_online_simultaneous.h:58-72 (30 batches of
 *                      ceil(N/30)), :148-178 (random_shuffle of the 1-based
 *                      case ids, kept across epochs; a case goes to batch
 *                      ceil(id/size), batches keep file order)
 *   e and t terms      fm_learn_vb_online.h:80-216 (prediction as
 *                      1/2 sum_f (sum_i v x)^2 - 1/2 sum_f sum_i v^2 x^2 + w + w0),
 *                      :220-310 (its variance), :_learn target - e
 *   update_w0          fm_learn_vb_online.h:586-633
 *   update_w           :635-710   (users' columns, then items', in id order)
 *   update_v           :712-800   (f outer; per f: add_main_q :352-380, then
 *                      every column in id order)
 *   hyperparameters    :523-580   (alpha, sigma_0, sigma_w, sigma_v blends)
 *   test RMSE          fm_learn_vb_online_simultaneous.h:348-360,441-447,506-525
 * Every floating-point expression keeps the reference's evaluation order with
 * x = 1 substituted only where the product by 1 is exact, so a gcc -O3 build
 * (SSE2, no FMA) reproduces the reference bit for bit.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "sbpmf_oracle.h"

double oracle_ran_gaussian(void);

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

void oracle_vbo_config_default(oracle_vbo_config *c) {
    memset(c, 0, sizeof *c);
    c->K = 8;
    c->epochs = 10;
    c->seed = 1;
    c->num_batch = 30;
}

/* batch-local column lists: for every attribute a, the batch's cases that
 * carry it, in increasing batch-local index (create_data_t order) */
typedef struct {
    uint32_t *ptr; /* [p+1] */
    uint32_t *cas; /* [2B] */
} cols;

static void build_cols(uint32_t B, const uint32_t *au, const uint32_t *ai, uint32_t p, cols *C, uint32_t *fill) {
    memset(C->ptr, 0, ((size_t)p + 1) * sizeof(uint32_t));
    for (uint32_t c = 0; c < B; c++) {
        C->ptr[au[c] + 1]++;
        C->ptr[ai[c] + 1]++;
    }
    for (uint32_t a = 0; a < p; a++) C->ptr[a + 1] += C->ptr[a];
    memcpy(fill, C->ptr, (size_t)p * sizeof(uint32_t));
    for (uint32_t c = 0; c < B; c++) { /* a user and an item attribute never coincide */
        C->cas[fill[au[c]]++] = c;
        C->cas[fill[ai[c]]++] = c;
    }
}

/* the e-term of predict_data_and_write_to_eterms (fm_learn_vb_online.h:80-216)
 * for one case with attributes (a0 < a1): returns the prediction */
static double predict_case(uint32_t K, uint32_t p, const double *mu_v, const double *mu_w, double mu0, uint32_t a0,
                           uint32_t a1) {
    double e = 0.0;
    for (uint32_t f = 0; f < K; f++) { /* (1) */
        const double *v = mu_v + (size_t)f * p;
        double q = 0.0;
        q += v[a0];
        q += v[a1];
        e += 0.5 * q * q;
    }
    double q = 0.0;
    for (uint32_t f = 0; f < K; f++) { /* (2) */
        const double *v = mu_v + (size_t)f * p;
        q -= 0.5 * v[a0] * v[a0];
        q -= 0.5 * v[a1] * v[a1];
    }
    q += mu_w[a0]; /* (3) k1 */
    q += mu_w[a1];
    e = e + q;
    e += mu0; /* k0 */
    return e;
}

/* the t-term of predict_t_and_write_to_qterms (:220-310) */
static double variance_case(uint32_t K, uint32_t p, const double *mu_v, const double *sg_v, const double *sg_w,
                            double sg0, uint32_t a0, uint32_t a1) {
    double t = 0.0;
    for (uint32_t f = 0; f < K; f++) {
        const double *v = mu_v + (size_t)f * p, *s = sg_v + (size_t)f * p;
        double q = 0.0, z = 0.0;
        q += v[a0] * v[a0];
        z += s[a0];
        q += v[a1] * v[a1];
        z += s[a1];
        t += (0.5 * z * z + z * q);
    }
    double q = 0.0;
    for (uint32_t f = 0; f < K; f++) {
        const double *v = mu_v + (size_t)f * p, *s = sg_v + (size_t)f * p;
        q -= (v[a0] * v[a0] * s[a0] + 0.5 * s[a0] * s[a0]);
        q -= (v[a1] * v[a1] * s[a1] + 0.5 * s[a1] * s[a1]);
    }
    q += sg_w[a0];
    q += sg_w[a1];
    t = t + q;
    t += sg0;
    return t;
}

int oracle_vbo_run(const oracle_vbo_config *cfg, uint64_t n_train, const uint32_t *tu, const uint32_t *ti,
                   const double *tr, uint64_t n_test, const uint32_t *su, const uint32_t *si, const double *sr,
                   uint32_t num_users, uint32_t num_items, oracle_vbo_result *res) {
    const uint32_t K = cfg->K, NB = cfg->num_batch ? cfg->num_batch : 30;
    const uint32_t N = (uint32_t)n_train;
    uint32_t I = num_users, J = num_items;
    if (I == 0 || J == 0) {
        uint32_t um = 0, im = 0;
        for (uint64_t c = 0; c < n_train; c++) {
            if (tu[c] > um) um = tu[c];
            if (ti[c] > im) im = ti[c];
        }
        for (uint64_t c = 0; c < n_test; c++) {
            if (su[c] > um) um = su[c];
            if (si[c] > im) im = si[c];
        }
        I = um + 1;
        J = im + 1;
    }
    /* attributes: user u -> u, item i -> I + i (users-first libFM layout);
     * num_attribute = largest id + 1 over train and test (libfm.cpp:328) */
    const uint32_t p = I + J;
    const uint32_t S = (uint32_t)ceil((double)N / NB);
    if (N == 0 || (uint64_t)S * (NB - 1) >= N) return -1; /* an empty batch: the reference divides by 0 */
    res->num_attribute = p;

    float min_t = 3.402823466e+38f, max_t = -3.402823466e+38f; /* train targets as DATA_FLOAT (libfm.cpp:199-214) */
    for (uint32_t c = 0; c < N; c++) {
        const float r = (float)tr[c];
        min_t = r < min_t ? r : min_t;
        max_t = r > max_t ? r : max_t;
    }
    const double lo = min_t, hi = max_t;

    double *mu_v = malloc((size_t)K * p * sizeof(double)), *sg_v = malloc((size_t)K * p * sizeof(double));
    double *nm_v = malloc((size_t)K * p * sizeof(double)), *ns_v = malloc((size_t)K * p * sizeof(double));
    double *mu_w = malloc((size_t)p * sizeof(double)), *sg_w = malloc((size_t)p * sizeof(double));
    double *nm_w = malloc((size_t)p * sizeof(double)), *ns_w = malloc((size_t)p * sizeof(double));
    double *rho_w = malloc((size_t)p * sizeof(double)), *rho_v = malloc((size_t)p * sizeof(double));
    uint32_t *t_w = calloc(p, sizeof(uint32_t)), *t_v = calloc(p, sizeof(uint32_t)), *cc = calloc(p, sizeof(uint32_t));
    double *sigma_v = malloc((size_t)K * sizeof(double));

    srand(cfg->seed);
    for (size_t x = 0; x < (size_t)K * p + p; x++) (void)oracle_ran_gaussian(); /* fm.v, fm.w (libfm.cpp:387,433) */
    for (uint32_t a = 0; a < p; a++) mu_w[a] = 0.1 * oracle_ran_gaussian(); /* matrix.h:362 */
    for (size_t x = 0; x < (size_t)K * p; x++) mu_v[x] = 0.1 * oracle_ran_gaussian(); /* matrix.h:377, f-major */
    for (uint32_t a = 0; a < p; a++) {
        sg_w[a] = .02;
        nm_w[a] = mu_w[a] / 0.02;
        ns_w[a] = 1 / sg_w[a];
    }
    for (size_t x = 0; x < (size_t)K * p; x++) {
        sg_v[x] = .02;
        nm_v[x] = mu_v[x] / 0.02;
        ns_v[x] = 1 / sg_v[x];
    }
    const double lamda = 0.5;
    const uint32_t t0 = 1;
    double alpha = 1.0, sigma_0 = 1.0, mu0 = 0.0, sg0 = 0.02, nm0 = 0.0, ns0 = 1 / sg0, sigma_w = 1;
    for (uint32_t f = 0; f < K; f++) sigma_v[f] = 1;
    uint32_t t_w0 = 0;
    double rho0 = pow((double)(t0 + t_w0), -lamda);
    for (uint32_t a = 0; a < p; a++) rho_w[a] = rho_v[a] = pow((double)(t0 + 0), -lamda);
    for (uint32_t c = 0; c < N; c++) { /* column counts of the whole train set (fm_learn_vb_online.h:877-900) */
        cc[tu[c]]++;
        cc[I + ti[c]]++;
    }

    uint32_t *shuffle = malloc((size_t)N * sizeof(uint32_t));
    for (uint32_t c = 0; c < N; c++) shuffle[c] = c + 1;
    uint32_t *bau = malloc((size_t)N * sizeof(uint32_t)), *bai = malloc((size_t)N * sizeof(uint32_t));
    float *btg = malloc((size_t)N * sizeof(float));
    uint32_t *bstart = calloc(NB + 1, sizeof(uint32_t)), *bfill = malloc((NB + 1) * sizeof(uint32_t));
    cols C;
    C.ptr = malloc(((size_t)p + 1) * sizeof(uint32_t));
    C.cas = malloc(2 * (size_t)S * sizeof(uint32_t));
    uint32_t *cfill = malloc(((size_t)p + 1) * sizeof(uint32_t));
    double *e = malloc((size_t)S * sizeof(double)), *t = malloc((size_t)S * sizeof(double));
    double *q = malloc((size_t)S * sizeof(double)), *tq = malloc((size_t)S * sizeof(double));
    double *tz = malloc((size_t)S * sizeof(double));

    const double t_start = now_s();
    res->epochs_done = 0;
    for (uint32_t k = 0; k < cfg->epochs; k++) {
        /* random_shuffle (libstdc++): for i = 1..N-1, swap(i, rand() % (i + 1)) */
        for (uint32_t i = 1; i < N; i++) {
            const uint32_t j = (uint32_t)(rand() % (long)(i + 1));
            if (i != j) {
                const uint32_t tmp = shuffle[i];
                shuffle[i] = shuffle[j];
                shuffle[j] = tmp;
            }
        }
        /* batches in file order */
        memset(bstart, 0, (NB + 1) * sizeof(uint32_t));
        for (uint32_t l = 0; l < N; l++) bstart[(uint32_t)ceil((double)shuffle[l] / S)]++;
        for (uint32_t j = 0; j < NB; j++) bstart[j + 1] += bstart[j];
        memcpy(bfill, bstart, (NB + 1) * sizeof(uint32_t));
        for (uint32_t l = 0; l < N; l++) {
            const uint32_t g = (uint32_t)ceil((double)shuffle[l] / S); /* 1-based */
            const uint32_t pos = bfill[g - 1]++;
            bau[pos] = tu[l];
            bai[pos] = I + ti[l];
            btg[pos] = (float)tr[l];
        }
        for (uint32_t j = 0; j < NB; j++) {
            const uint32_t b0 = bstart[j], B = bstart[j + 1] - bstart[j];
            const uint32_t *au = bau + b0, *ai = bai + b0;
            build_cols(B, au, ai, p, &C, cfill);
            for (uint32_t c = 0; c < B; c++) {
                e[c] = predict_case(K, p, mu_v, mu_w, mu0, au[c], ai[c]);
                t[c] = variance_case(K, p, mu_v, sg_v, sg_w, sg0, au[c], ai[c]);
                e[c] = btg[b0 + c] - e[c];
            }
            /* ---- update_w0 (:586-633) */
            {
                const double sigma_dash = sg0, mu_dash = mu0, mu_old = nm0, sigma_old = ns0;
                double eta1 = 0.0, eta2 = 0.0;
                for (uint32_t c = 0; c < B; c++) {
                    const double w0_temp = e[c] + mu0;
                    ns0 = ((1 - rho0) * sigma_old) + rho0 * (sigma_0 + N * alpha);
                    nm0 = ((1 - rho0) * mu_old) + rho0 * N * alpha * w0_temp;
                    eta1 += nm0;
                    eta2 += ns0;
                }
                nm0 = eta1 / B;
                ns0 = eta2 / B;
                mu0 = nm0 / ns0;
                sg0 = 1.0 / ns0;
                for (uint32_t c = 0; c < B; c++) {
                    e[c] = e[c] + (mu_dash - mu0);
                    t[c] = t[c] + (sg0 - sigma_dash);
                }
            }
            /* ---- update_w (:635-710), columns in id order */
            for (uint32_t a = 0; a < p; a++) {
                const uint32_t n = C.ptr[a + 1] - C.ptr[a];
                if (n == 0) continue;
                const uint32_t *cs = C.cas + C.ptr[a];
                const double mu_dash = mu_w[a], sigma_dash = sg_w[a], mu_old = nm_w[a], sigma_old = ns_w[a];
                double eta1 = 0.0, eta2 = 0.0;
                for (uint32_t x = 0; x < n; x++) {
                    const double w_mean = 1.0 * (e[cs[x]] + 1.0 * mu_w[a]);
                    const double w_sigma_sqr = 1.0;
                    ns_w[a] = ((1 - rho_w[a]) * sigma_old) + rho_w[a] * (sigma_w + alpha * cc[a] * w_sigma_sqr);
                    nm_w[a] = ((1 - rho_w[a]) * mu_old) + rho_w[a] * cc[a] * alpha * w_mean;
                    eta1 += nm_w[a];
                    eta2 += ns_w[a];
                }
                t_w[a] += n;
                rho_w[a] = pow((double)(t0 + t_w[a]), -lamda);
                nm_w[a] = eta1 / n;
                ns_w[a] = eta2 / n;
                double mu = nm_w[a] / ns_w[a], sigma = 1 / ns_w[a];
                if (isnan(sigma) || isinf(sigma)) sigma = sigma_dash;
                sg_w[a] = sigma;
                if (isnan(mu) || isinf(mu)) {
                    mu_w[a] = mu_dash;
                    continue;
                }
                mu_w[a] = mu;
                for (uint32_t x = 0; x < n; x++) {
                    const uint32_t c = cs[x];
                    e[c] += 1.0 * (mu_dash - mu);
                    t[c] += 1.0 * 1.0 * (sigma - sigma_dash);
                }
            }
            /* ---- update_v (:712-800), factor-outer */
            for (uint32_t f = 0; f < K; f++) {
                double *v = mu_v + (size_t)f * p, *s = sg_v + (size_t)f * p;
                double *nmv = nm_v + (size_t)f * p, *nsv = ns_v + (size_t)f * p;
                for (uint32_t c = 0; c < B; c++) { /* add_main_q (:352-380), rows in id order */
                    q[c] = 0.0;
                    tq[c] = 0.0;
                    tz[c] = 0.0;
                    q[c] += v[au[c]];
                    tq[c] += s[au[c]];
                    tz[c] += v[au[c]] * v[au[c]];
                    q[c] += v[ai[c]];
                    tq[c] += s[ai[c]];
                    tz[c] += v[ai[c]] * v[ai[c]];
                }
                for (uint32_t a = 0; a < p; a++) {
                    const uint32_t n = C.ptr[a + 1] - C.ptr[a];
                    if (n == 0) continue;
                    const uint32_t *cs = C.cas + C.ptr[a];
                    const double mu_dash = v[a], sigma_dash = s[a], mu_old = nmv[a], sigma_old = nsv[a];
                    double eta1 = 0.0, eta2 = 0.0;
                    for (uint32_t x = 0; x < n; x++) {
                        const uint32_t c = cs[x];
                        const double h = q[c] - 1.0 * v[a];
                        const double h1 = tq[c] - 1.0 * 1.0 * s[a];
                        const double v_mean = 1.0 * h * (e[c] + 1.0 * v[a] * h);
                        const double v_sigma_sqr = 1.0 * 1.0 * h * h + 1.0 * 1.0 * h1;
                        nsv[a] = (1 - rho_v[a]) * sigma_old + rho_v[a] * (sigma_v[f] + alpha * cc[a] * v_sigma_sqr);
                        nmv[a] = ((1 - rho_v[a]) * mu_old) + rho_v[a] * cc[a] * alpha * v_mean;
                        eta1 += nmv[a];
                        eta2 += nsv[a];
                    }
                    nmv[a] = eta1 / n;
                    nsv[a] = eta2 / n;
                    double mu = nmv[a] / nsv[a], sigma = 1 / nsv[a];
                    if (isnan(sigma) || isinf(sigma)) sigma = sigma_dash;
                    s[a] = sigma;
                    if (f == 0) t_v[a] += n; /* the caller's count, after update_v (:447-450) */
                    if (isnan(mu) || isinf(mu)) {
                        v[a] = mu_dash;
                        continue;
                    }
                    v[a] = mu;
                    for (uint32_t x = 0; x < n; x++) {
                        const uint32_t c = cs[x];
                        const double h = 1.0 * (q[c] - 1.0 * mu_dash);
                        const double h1 = 1.0 * 1.0 * (tq[c] - 1.0 * 1.0 * sigma_dash);
                        const double h2 = 1.0 * 1.0 * (tz[c] - 1.0 * 1.0 * mu_dash * mu_dash);
                        q[c] += 1.0 * (mu - mu_dash);
                        tq[c] += 1.0 * 1.0 * (sigma - sigma_dash);
                        tz[c] += 1.0 * 1.0 * (mu * mu - mu_dash * mu_dash);
                        e[c] += h * (mu_dash - mu);
                        t[c] += (h1 + h2) * (sigma - sigma_dash);
                        t[c] += h1 * (mu * mu - mu_dash * mu_dash);
                    }
                }
            }
            for (uint32_t a = 0; a < p; a++) rho_v[a] = pow((double)(t0 + t_v[a]), -lamda);
            /* ---- hyperparameters (:523-580) */
            {
                double alpha_temp = 0.0;
                for (uint32_t c = 0; c < B; c++) alpha_temp += e[c] * e[c] + t[c];
                const double alpha_old = alpha;
                alpha = (1 - rho0) * alpha_old + rho0 * ((double)B / alpha_temp);
                if (isnan(alpha) || isinf(alpha)) {
                    alpha = alpha_old;
                    continue; /* the reference returns before the remaining blends and the step count */
                }
            }
            sigma_0 = (1 - rho0) * sigma_0 + rho0 * (1.0 / (mu0 * mu0 + sg0));
            {
                double tmp = 0.0;
                for (uint32_t a = 0; a < p; a++) tmp += mu_w[a] * mu_w[a] + sg_w[a];
                sigma_w = (1 - rho0) * sigma_w + rho0 * ((double)p / tmp);
            }
            for (uint32_t f = 0; f < K; f++) {
                const double *v = mu_v + (size_t)f * p, *s = sg_v + (size_t)f * p;
                double tmp = 0.0;
                for (uint32_t a = 0; a < p; a++) tmp += v[a] * v[a] + s[a];
                sigma_v[f] = (1 - rho0) * sigma_v[f] + rho0 * ((double)p / tmp);
            }
            t_w0 += 1;
            rho0 = pow((double)(t0 + t_w0), -lamda);
        }
        /* ---- test RMSE of the clamped mean prediction */
        double se = 0.0;
        for (uint64_t c = 0; c < n_test; c++) {
            double pr = predict_case(K, p, mu_v, mu_w, mu0, su[c], I + si[c]);
            pr = (pr < hi) ? pr : hi; /* std::min(max_target, p), std::max(min_target, p) */
            pr = (lo < pr) ? pr : lo;
            if (res->pred && k + 1 == cfg->epochs) res->pred[c] = pr;
            double pe = pr * 1.0;
            pe = (pe < hi) ? pe : hi;
            pe = (lo < pe) ? pe : lo;
            const double err = pe - (double)(float)sr[c];
            se += err * err;
        }
        if (res->rmse && k < res->rmse_cap) res->rmse[k] = sqrt(se / n_test);
        res->epochs_done = k + 1;
        if (cfg->seconds_limit > 0 && now_s() - t_start > cfg->seconds_limit) break;
    }
    res->seconds = now_s() - t_start;
    res->alpha = alpha;
    res->mu0 = mu0;
    if (res->mu_w) memcpy(res->mu_w, mu_w, (size_t)p * sizeof(double));
    if (res->mu_v) /* attribute-major [p][K] */
        for (uint32_t a = 0; a < p; a++)
            for (uint32_t f = 0; f < K; f++) res->mu_v[(size_t)a * K + f] = mu_v[(size_t)f * p + a];
    free(mu_v); free(sg_v); free(nm_v); free(ns_v); free(mu_w); free(sg_w); free(nm_w); free(ns_w);
    free(rho_w); free(rho_v); free(t_w); free(t_v); free(cc); free(sigma_v); free(shuffle); free(bau); free(bai);
    free(btg); free(bstart); free(bfill); free(C.ptr); free(C.cas); free(cfill); free(e); free(t); free(q); free(tq);
    free(tz);
    return 0;
}
