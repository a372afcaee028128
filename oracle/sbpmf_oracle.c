/*
 * sbpmf_oracle.c -- CPU restatement of the reference SBPMF Gibbs sampler.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity oracle: it is imported
 * (as liboracle.so / the `sbpmf_oracle` binary) only by tests/, by
 * __graft_entry__.smoke() as the checker, and by bench.py's `cpu_baseline`
 * leg.  The product path (libsbmf.so, HIP kernels) never links or calls it.
 *
 * Pinning: its per-sweep test RMSE trajectory is checked bit-for-bit (%.17g)
 * against the reference itself, compiled unmodified from
 * /root/reference/src/libfm/gibbs_sbpmf_final.cpp and gibbs_sbpmf2.cpp by
 * oracle/Makefile into oracle/_ref/ (fixtures: tests/golden/, generator:
 * oracle/make_golden.py).  See DESIGN.md "Oracle".
 *
 * What it restates (file:line under /root/reference):
 *   RNG               src/util/random.h:118-148 (ran_gamma, Marsaglia-Tsang),
 *                     :150-164 (ran_gaussian, Leva), :166-172 (mean/stdev
 *                     form, returns mean on stdev==0 or NaN), :174-176
 *                     (ran_uniform = rand()/(RAND_MAX+1)).  Uses glibc rand()
 *                     itself, exactly like the reference.
 *   loader            src/libfm/gibbs_sbpmf_final.cpp:26-215 (sscanf
 *                     "%u%c%u%c%lf", max id over train+test, R/R_t in file
 *                     order)
 *   init              :236-250 (U i-major, V k-major, N(0,init_sd))
 *   E recompute       :317-334
 *   tau               :339-342
 *   hyperparameters   :375-414 (sbpmf2 quirks: gibbs_sbpmf2.cpp:386,406,412)
 *   user half-sweep   :453-491
 *   item half-sweep   :495-535
 *   test RMSE         :539-563 (running mean of clamped predictions)
 * and the biased sampler (quirks BIAS2 / BIAS22, run_bias below):
 * /root/reference/gibbs_sbpmf2.cpp (top level) = src/libfm/gibbs_sbpmf22.cpp
 * up to init scale, test clamp and D.
 * The floating-point operation order of every expression follows the
 * reference so that a gcc -O3 build (SSE2, no FMA contraction) reproduces
 * it bit for bit.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "sbpmf_oracle.h"

/* ---------------------------------------------------------------- RNG --- */
/* random.h:174-176 */
static double o_uniform(void) { return rand() / ((double)RAND_MAX + 1); }

/* random.h:150-164 (Joseph L. Leva) */
double oracle_ran_gaussian(void) {
    double u, v, x, y, Q;
    do {
        do {
            u = o_uniform();
        } while (u == 0.0);
        v = 1.7156 * (o_uniform() - 0.5);
        x = u - 0.449871;
        y = fabs(v) + 0.386595;
        Q = x * x + y * (0.19600 * y - 0.25472 * x);
        if (Q < 0.27597) { break; }
    } while ((Q > 0.27846) || ((v * v) > (-4.0 * u * u * log(u))));
    return v / u;
}

/* random.h:166-172 */
static double o_gaussian(double mean, double stdev) {
    if ((stdev == 0.0) || isnan(stdev)) return mean;
    return mean + stdev * oracle_ran_gaussian();
}

/* random.h:118-142 (Marsaglia & Tsang; shape<1 boost) */
double oracle_ran_gamma(double alpha) {
    if (alpha < 1.0) {
        double u;
        do {
            u = o_uniform();
        } while (u == 0.0);
        return oracle_ran_gamma(alpha + 1.0) * pow(u, 1.0 / alpha);
    } else {
        double d, c, x, v, u;
        d = alpha - 1.0 / 3.0;
        c = 1.0 / sqrt(9.0 * d);
        do {
            do {
                x = oracle_ran_gaussian();
                v = 1.0 + c * x;
            } while (v <= 0.0);
            v = v * v * v;
            u = o_uniform();
        } while ((u >= (1.0 - 0.0331 * (x * x) * (x * x))) &&
                 (log(u) >= (0.5 * x * x + d * (1.0 - v + log(v)))));
        return d * v;
    }
}

/* random.h:146-148 */
static double o_gamma(double alpha, double beta) { return oracle_ran_gamma(alpha) / beta; }

/* ------------------------------------------------- Philox stream mode --- */
/* The GPU build's throughput RNG (scalable-bayesian-matrix-factorization_amd/
 * csrc/rng.h), restated so the oracle can run the same chain the benchmark
 * runs (oracle_config.rng = 1): Philox4x32-10 keyed by the seed; per-coordinate
 * normals are Box-Muller pairs of (row, sweep, tag | pair << 8, salt); the
 * host hyperparameter draws use a sequential uniform stream (index, sweep,
 * TAG_HOST, salt) through the same Leva / Marsaglia-Tsang algorithms as
 * random.h:118-164.  Not a reference algorithm: it pins the GPU's own mode. */
enum { PX_TAG_USERS = 0, PX_TAG_ITEMS = 1, PX_TAG_HOST = 2, PX_TAG_INIT_U = 3, PX_TAG_INIT_V = 4 };
#define PX_SALT 0x53424d46u

static uint32_t px_mulhi(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }

static void px_block(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; ++r) {
        uint32_t h0 = px_mulhi(0xD2511F53u, c[0]), l0 = 0xD2511F53u * c[0];
        uint32_t h1 = px_mulhi(0xCD9E8D57u, c[2]), l1 = 0xCD9E8D57u * c[2];
        uint32_t n0 = h1 ^ c[1] ^ k0, n2 = h0 ^ c[3] ^ k1;
        c[0] = n0;
        c[1] = l1;
        c[2] = n2;
        c[3] = l0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

/* normal k of (row, sweep, tag): pair k/2, component k&1 */
static double px_normal(uint64_t seed, uint32_t row, uint32_t sweep, uint32_t tag, uint32_t k) {
    uint32_t c[4] = {row, sweep, tag | ((k >> 1) << 8), PX_SALT};
    px_block(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    uint64_t a = ((((uint64_t)c[0] << 32) | c[1]) >> 11), b = ((((uint64_t)c[2] << 32) | c[3]) >> 11);
    double u1 = (double)(a + 1) * (1.0 / 9007199254740992.0);
    double u2 = (double)b * (1.0 / 9007199254740992.0);
    double rr = sqrt(-2.0 * log(u1));
    double th = 6.283185307179586476925286766559 * u2;
    return (k & 1) ? rr * sin(th) : rr * cos(th);
}

typedef struct {
    uint64_t seed;
    uint32_t sweep, idx;
    double buf[2];
    int have;
} px_stream;

static double px_uniform(px_stream *s) {
    if (s->have == 0) {
        uint32_t c[4] = {s->idx++, s->sweep, PX_TAG_HOST, PX_SALT};
        px_block(c, (uint32_t)s->seed, (uint32_t)(s->seed >> 32));
        s->buf[0] = ((((uint64_t)c[0] << 32) | c[1]) >> 11) * (1.0 / 9007199254740992.0);
        s->buf[1] = ((((uint64_t)c[2] << 32) | c[3]) >> 11) * (1.0 / 9007199254740992.0);
        s->have = 2;
    }
    return s->buf[--s->have];
}

/* random.h:150-164 over the Philox uniform stream */
static double px_leva(px_stream *g) {
    double u, v, x, y, Q;
    do {
        do {
            u = px_uniform(g);
        } while (u == 0.0);
        v = 1.7156 * (px_uniform(g) - 0.5);
        x = u - 0.449871;
        y = fabs(v) + 0.386595;
        Q = x * x + y * (0.19600 * y - 0.25472 * x);
        if (Q < 0.27597) break;
    } while ((Q > 0.27846) || ((v * v) > (-4.0 * u * u * log(u))));
    return v / u;
}

/* random.h:118-148 over the Philox uniform stream (shapes here are > 1) */
static double px_gamma(px_stream *g, double alpha) {
    double boost = 1.0;
    int small = alpha < 1.0;
    if (small) {
        double u;
        do {
            u = px_uniform(g);
        } while (u == 0.0);
        boost = pow(u, 1.0 / alpha);
        alpha = alpha + 1.0;
    }
    double d = alpha - 1.0 / 3.0, c = 1.0 / sqrt(9.0 * d), x, v, u;
    do {
        do {
            x = px_leva(g);
            v = 1.0 + c * x;
        } while (v <= 0.0);
        v = v * v * v;
        u = px_uniform(g);
    } while ((u >= (1.0 - 0.0331 * (x * x) * (x * x))) && (log(u) >= (0.5 * x * x + d * (1.0 - v + log(v)))));
    return small ? (d * v) * boost : d * v;
}

void oracle_srand(unsigned seed) { srand(seed); }
int oracle_rand(void) { return rand(); }
double oracle_ran_uniform(void) { return o_uniform(); }

/* ------------------------------------------------------------- loader --- */
/* gibbs_sbpmf_final.cpp:35-71: a line counts iff sscanf("%u%c%u%c%lf")>=5 */
static int read_triples(const char *path, uint32_t **u, uint32_t **i, double **r, uint64_t *n) {
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    size_t cap = 1024, cnt = 0;
    uint32_t *uu = malloc(cap * sizeof *uu), *ii = malloc(cap * sizeof *ii);
    double *rr = malloc(cap * sizeof *rr);
    char *line = NULL;
    size_t lcap = 0;
    while (getline(&line, &lcap, f) >= 0) {
        unsigned a, b;
        char c1, c2;
        double v;
        if (sscanf(line, "%u%c%u%c%lf", &a, &c1, &b, &c2, &v) >= 5) {
            if (cnt == cap) {
                cap *= 2;
                uu = realloc(uu, cap * sizeof *uu);
                ii = realloc(ii, cap * sizeof *ii);
                rr = realloc(rr, cap * sizeof *rr);
            }
            uu[cnt] = a;
            ii[cnt] = b;
            rr[cnt] = v;
            cnt++;
        }
    }
    free(line);
    fclose(f);
    *u = uu;
    *i = ii;
    *r = rr;
    *n = cnt;
    return 0;
}

/* ------------------------------------------------------------ sampler --- */
void oracle_config_default(oracle_config *c) {
    memset(c, 0, sizeof *c);
    c->K = 20;
    c->iters = 100;
    c->burnin = 0;
    c->seed = 1;
    c->quirks = ORACLE_QUIRKS_FINAL;
    c->init_stdev = -1.0; /* -1: quirk-set default (final 1.0, sbpmf2 0.1) */
    c->clamp_lo = -1.0;   /* <0: quirk-set default (final 1.0, sbpmf2 0.5) */
    c->clamp_hi = 5.0;
    c->sweep_seconds_limit = 0.0;
    c->rng = 0;
}

typedef struct {
    uint32_t *ptr; /* [rows+1] */
    uint32_t *cas; /* case id per entry, file order */
    uint32_t *oth; /* partner id per entry */
} lists;

static void build_lists(uint64_t n, const uint32_t *key, const uint32_t *other, uint32_t rows, lists *L) {
    L->ptr = calloc((size_t)rows + 1, sizeof(uint32_t));
    L->cas = malloc((n ? n : 1) * sizeof(uint32_t));
    L->oth = malloc((n ? n : 1) * sizeof(uint32_t));
    for (uint64_t c = 0; c < n; c++) L->ptr[key[c] + 1]++;
    for (uint32_t r = 0; r < rows; r++) L->ptr[r + 1] += L->ptr[r];
    uint32_t *fill = malloc(((size_t)rows + 1) * sizeof(uint32_t));
    memcpy(fill, L->ptr, ((size_t)rows + 1) * sizeof(uint32_t));
    for (uint64_t c = 0; c < n; c++) {
        uint32_t p = fill[key[c]]++;
        L->cas[p] = (uint32_t)c;
        L->oth[p] = other[c];
    }
    free(fill);
}

static void free_lists(lists *L) {
    free(L->ptr);
    free(L->cas);
    free(L->oth);
}

#include <time.h>
static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

/* ------------------------------------------------------- biased sampler --- */
/* /root/reference/gibbs_sbpmf2.cpp (top level; BIAS2) and the same algorithm
 * in src/libfm/gibbs_sbpmf22.cpp (BIAS22).  Line numbers: top-level file
 * first, then gibbs_sbpmf22.cpp.  Global bias b_0 with a Normal-Gamma prior,
 * per-user / per-item biases b_i, b_j each with its own (sigma, mu) pair drawn
 * every sweep, tau named alpha with shape a0' + N and rate b0' + sum E^2, and
 * factor hyperparameters with shape alpha + I (not (I+1)/2).  All six prior
 * groups use alpha = beta = sigma = 1, mu = 0 (:284-318 / :290-325). */
static int run_bias(const oracle_config *cfg, uint64_t n_train, const uint32_t *tu, const uint32_t *ti,
                    const double *tr, uint64_t n_test, const uint32_t *su, const uint32_t *si, const double *sr,
                    uint32_t I, uint32_t J, oracle_result *res) {
    const uint32_t D = cfg->K;
    const int top = cfg->quirks == ORACLE_QUIRKS_BIAS2;
    const double init_scale = cfg->init_stdev >= 0 ? cfg->init_stdev : (top ? 0.1 : 1.0); /* :242 / :186 */
    const double lo = cfg->clamp_lo >= 0 ? cfg->clamp_lo : (top ? 0.5 : 1.0);            /* :628 / :578 */
    const double hi = cfg->clamp_hi;
    lists R, Rt;
    build_lists(n_train, tu, ti, I, &R);
    build_lists(n_train, ti, tu, J, &Rt);

    srand(cfg->seed);
    double *U = malloc((size_t)I * D * sizeof(double));
    double *V = malloc((size_t)D * J * sizeof(double));
    for (uint32_t i = 0; i < I; i++) /* :240-244 */
        for (uint32_t k = 0; k < D; k++) U[(size_t)i * D + k] = init_scale * o_gaussian(0.0, 1.0);
    for (uint32_t k = 0; k < D; k++) /* :246-250 */
        for (uint32_t j = 0; j < J; j++) V[(size_t)k * J + j] = init_scale * o_gaussian(0.0, 1.0);
    double *sigma_u = calloc(D, sizeof(double)), *mu_u = calloc(D, sizeof(double));
    double *sigma_v = calloc(D, sizeof(double)), *mu_v = calloc(D, sizeof(double));
    double *b_i = calloc(I ? I : 1, sizeof(double)), *mu_b_i = calloc(I ? I : 1, sizeof(double));
    double *sigma_b_i = calloc(I ? I : 1, sizeof(double));
    double *b_j = calloc(J ? J : 1, sizeof(double)), *mu_b_j = calloc(J ? J : 1, sizeof(double));
    double *sigma_b_j = calloc(J ? J : 1, sizeof(double));
    const double ag = 1.0, bg = 1.0, sg = 1.0, mg = 0.0; /* alpha_k, beta_k, sigma_k, mu_k of every group */
    double mu_b_0 = 0.0, sigma_b_0 = 0.0, b_0 = 0.0, alpha = 0.0; /* :315-318 */

    double *E = calloc(n_train ? n_train : 1, sizeof(double));
    double *sum = calloc(n_test ? n_test : 1, sizeof(double));
    const uint32_t iters = cfg->iters; /* burn_iter = 0 (:323) */
    double t_start = now_s();
    res->sweeps_done = 0;
    for (uint32_t iter = 0; iter < iters; iter++) {
        /* E recompute, sum E, sum E^2 :342-359 */
        double es = 0.0, esq = 0.0;
        for (uint64_t c = 0; c < n_train; c++) {
            uint32_t user = tu[c], item = ti[c];
            double temp = 0.0;
            for (uint32_t k = 0; k < D; k++) temp += U[(size_t)user * D + k] * V[(size_t)k * J + item];
            E[c] = tr[c] - (b_0 + b_i[user] + b_j[item] + temp);
            es += E[c];
            esq += (E[c] * E[c]);
        }
        /* alpha :366-372 */
        alpha = o_gamma(1.0 + n_train, 1.0 + esq);
        /* sigma_b_0, mu_b_0, b_0 :376-410 */
        sigma_b_0 = o_gamma(ag + 1, bg + (0.5 * (b_0 - mu_b_0) * (b_0 - mu_b_0)));
        double s0 = 1.0 / (sg + sigma_b_0);
        mu_b_0 = o_gaussian(s0 * ((sg * mg) + b_0 * sigma_b_0), s0);
        double sb0 = 1 / (sigma_b_0 + alpha * n_train);
        double mb0 = sb0 * (sigma_b_0 * mu_b_0 + alpha * (es + n_train * b_0));
        double old_b0 = b_0;
        b_0 = o_gaussian(mb0, sb0);
        for (uint64_t c = 0; c < n_train; c++) E[c] += (old_b0 - b_0);
        /* factor hyperparameters :415-467 */
        for (uint32_t k = 0; k < D; k++) {
            double temp = 0.0, temp2 = 0.0;
            for (uint32_t i = 0; i < I; i++) {
                double x = U[(size_t)i * D + k];
                temp += (x - mu_u[k]) * (x - mu_u[k]);
                temp2 += x;
            }
            sigma_u[k] = o_gamma(ag + I, bg + (0.5) * temp);
            double s2 = 1 / (sg + sigma_u[k] * I);
            mu_u[k] = o_gaussian(s2 * (sg * mg + sigma_u[k] * temp2), s2);
            temp = 0.0;
            temp2 = 0.0;
            for (uint32_t j = 0; j < J; j++) {
                double x = V[(size_t)k * J + j];
                temp += (x - mu_v[k]) * (x - mu_v[k]);
                temp2 += x;
            }
            sigma_v[k] = o_gamma(ag + J, bg + (0.5) * temp);
            double s1 = 1 / (sg + sigma_v[k] * J);
            mu_v[k] = o_gaussian(s1 * (sg * mg + sigma_v[k] * temp2), s1);
        }
        /* per-row bias hyperparameters: users :470-489, items :492-511 */
        for (uint32_t i = 0; i < I; i++) {
            sigma_b_i[i] = o_gamma(ag + 1, bg + (0.5 * (b_i[i] - mu_b_i[i]) * (b_i[i] - mu_b_i[i])));
            double s4 = 1.0 / (sg + sigma_b_i[i]);
            mu_b_i[i] = o_gaussian(s4 * ((sg * mg) + b_i[i] * sigma_b_i[i]), s4);
        }
        for (uint32_t j = 0; j < J; j++) {
            sigma_b_j[j] = o_gamma(ag + 1, bg + (0.5 * (b_j[j] - mu_b_j[j]) * (b_j[j] - mu_b_j[j])));
            double s5 = 1.0 / (sg + sigma_b_j[j]);
            mu_b_j[j] = o_gaussian(s5 * ((sg * mg) + b_j[j] * sigma_b_j[j]), s5);
        }
        /* users: b_i then the k-loop :515-558 */
        for (uint32_t i = 0; i < I; i++) {
            uint32_t b = R.ptr[i], e = R.ptr[i + 1];
            double sbi = 1 / (sigma_b_i[i] + (alpha * (e - b)));
            double temp = 0.0;
            for (uint32_t p = b; p < e; p++) temp += (E[R.cas[p]] + b_i[i]);
            double mbi = sbi * ((sigma_b_i[i] * mu_b_i[i]) + alpha * temp);
            double old = b_i[i];
            b_i[i] = o_gaussian(mbi, sbi);
            for (uint32_t p = b; p < e; p++) E[R.cas[p]] += (old - b_i[i]);
            for (uint32_t k = 0; k < D; k++) {
                const double *Vk = V + (size_t)k * J;
                double t1 = 0.0, t2 = 0.0;
                double *Uik = &U[(size_t)i * D + k];
                for (uint32_t p = b; p < e; p++) {
                    double v = Vk[R.oth[p]];
                    t1 += (v * v);
                    t2 += (v * (E[R.cas[p]] + v * *Uik));
                }
                double s_star = 1 / (sigma_u[k] + (alpha * t1));
                double m_star = s_star * (alpha * t2 + sigma_u[k] * mu_u[k]);
                double ou = *Uik;
                *Uik = o_gaussian(m_star, s_star);
                for (uint32_t p = b; p < e; p++) E[R.cas[p]] += Vk[R.oth[p]] * (ou - *Uik);
            }
        }
        /* items: b_j then the k-loop :563-606 */
        for (uint32_t j = 0; j < J; j++) {
            uint32_t b = Rt.ptr[j], e = Rt.ptr[j + 1];
            double sbj = 1 / (sigma_b_j[j] + (alpha * (e - b)));
            double temp = 0.0;
            for (uint32_t p = b; p < e; p++) temp += (E[Rt.cas[p]] + b_j[j]);
            double mbj = sbj * ((sigma_b_j[j] * mu_b_j[j]) + alpha * temp);
            double old = b_j[j];
            b_j[j] = o_gaussian(mbj, sbj);
            for (uint32_t p = b; p < e; p++) E[Rt.cas[p]] += (old - b_j[j]);
            for (uint32_t k = 0; k < D; k++) {
                double t1 = 0.0, t2 = 0.0;
                double *Vjk = &V[(size_t)k * J + j];
                for (uint32_t p = b; p < e; p++) {
                    double u = U[(size_t)Rt.oth[p] * D + k];
                    t1 += (u * u);
                    t2 += (u * (E[Rt.cas[p]] + *Vjk * u));
                }
                double s_star = 1 / (sigma_v[k] + (alpha * t1));
                double m_star = s_star * (alpha * t2 + sigma_v[k] * mu_v[k]);
                double ov = *Vjk;
                *Vjk = o_gaussian(m_star, s_star);
                for (uint32_t p = b; p < e; p++) E[Rt.cas[p]] += U[(size_t)Rt.oth[p] * D + k] * (ov - *Vjk);
            }
        }
        /* test RMSE of the running mean :610-636 (every sweep, divides by iter+1) */
        double diff = 0.0, diff_this = 0.0;
        for (uint64_t t = 0; t < n_test; t++) {
            uint32_t user = su[t], item = si[t];
            double temp = b_0 + b_i[user] + b_j[item];
            for (uint32_t k = 0; k < D; k++) temp += U[(size_t)user * D + k] * V[(size_t)k * J + item];
            temp = (temp < hi) ? temp : hi;
            temp = (lo < temp) ? temp : lo;
            sum[t] += temp;
            diff += (sr[t] - ((double)sum[t] / (iter + 1))) * (sr[t] - ((double)sum[t] / (iter + 1)));
            diff_this += (sr[t] - temp) * (sr[t] - temp);
        }
        if (res->rmse && iter < res->rmse_cap) res->rmse[iter] = sqrt(diff / n_test);
        if (res->rmse_this && iter < res->rmse_cap) res->rmse_this[iter] = sqrt(diff_this / n_test);
        if (res->tau && iter < res->rmse_cap) res->tau[iter] = alpha;
        res->sweeps_done = iter + 1;
        if (cfg->sweep_seconds_limit > 0 && now_s() - t_start > cfg->sweep_seconds_limit) break;
    }
    res->seconds = now_s() - t_start;
    if (res->U) memcpy(res->U, U, (size_t)I * D * sizeof(double));
    if (res->V)
        for (uint32_t j = 0; j < J; j++)
            for (uint32_t k = 0; k < D; k++) res->V[(size_t)j * D + k] = V[(size_t)k * J + j];
    if (res->hyper) {
        memcpy(res->hyper, sigma_u, D * sizeof(double));
        memcpy(res->hyper + D, mu_u, D * sizeof(double));
        memcpy(res->hyper + 2 * D, sigma_v, D * sizeof(double));
        memcpy(res->hyper + 3 * D, mu_v, D * sizeof(double));
    }
    if (res->pred_sum && n_test) memcpy(res->pred_sum, sum, n_test * sizeof(double));
    if (res->bu) memcpy(res->bu, b_i, (size_t)I * sizeof(double));
    if (res->bv) memcpy(res->bv, b_j, (size_t)J * sizeof(double));
    res->b0 = b_0;
    free(U); free(V); free(sigma_u); free(mu_u); free(sigma_v); free(mu_v);
    free(b_i); free(mu_b_i); free(sigma_b_i); free(b_j); free(mu_b_j); free(sigma_b_j);
    free(E); free(sum);
    free_lists(&R); free_lists(&Rt);
    return 0;
}

int oracle_run_arrays(const oracle_config *cfg, uint64_t n_train, const uint32_t *tu, const uint32_t *ti,
                      const double *tr, uint64_t n_test, const uint32_t *su, const uint32_t *si,
                      const double *sr, uint32_t num_users, uint32_t num_items, oracle_result *res) {
    const uint32_t D = cfg->K;
    const int q2 = cfg->quirks == ORACLE_QUIRKS_SBPMF2;
    const int qnone = cfg->quirks == ORACLE_QUIRKS_NONE;
    double init_sd = cfg->init_stdev >= 0 ? cfg->init_stdev : (q2 ? 0.1 : 1.0);
    double lo = cfg->clamp_lo >= 0 ? cfg->clamp_lo : (q2 ? 0.5 : 1.0);
    double hi = cfg->clamp_hi;
    uint32_t I = num_users, J = num_items;
    if (I == 0 || J == 0) {
        uint32_t umax = 0, imax = 0;
        for (uint64_t c = 0; c < n_train; c++) {
            if (tu[c] > umax) umax = tu[c];
            if (ti[c] > imax) imax = ti[c];
        }
        for (uint64_t c = 0; c < n_test; c++) {
            if (su[c] > umax) umax = su[c];
            if (si[c] > imax) imax = si[c];
        }
        I = umax + 1; /* gibbs_sbpmf_final.cpp:147-148 */
        J = imax + 1;
    }
    res->num_users = I;
    res->num_items = J;
    if (cfg->quirks == ORACLE_QUIRKS_BIAS2 || cfg->quirks == ORACLE_QUIRKS_BIAS22)
        return run_bias(cfg, n_train, tu, ti, tr, n_test, su, si, sr, I, J, res);

    lists R, Rt;
    build_lists(n_train, tu, ti, I, &R);  /* R[u] = {case, item}  :204-205 */
    build_lists(n_train, ti, tu, J, &Rt); /* R_t[j] = {case, user} :206-207 */

    const int px = cfg->rng == 1; /* Philox stream mode (the GPU's throughput RNG) */
    const uint64_t pseed = cfg->seed;
    srand(cfg->seed);
    double *U = malloc((size_t)I * D * sizeof(double));  /* U[i][k] */
    double *V = malloc((size_t)D * J * sizeof(double));  /* V[k][j]  (k-major, :229-233) */
    if (px) { /* U[i][k] = sd * z(seed, sweep 0xffffffff, TAG_INIT_U, i, k), V likewise */
        for (uint32_t i = 0; i < I; i++)
            for (uint32_t k = 0; k < D; k++)
                U[(size_t)i * D + k] = init_sd * px_normal(pseed, i, 0xffffffffu, PX_TAG_INIT_U, k);
        for (uint32_t k = 0; k < D; k++)
            for (uint32_t j = 0; j < J; j++)
                V[(size_t)k * J + j] = init_sd * px_normal(pseed, j, 0xffffffffu, PX_TAG_INIT_V, k);
    } else {
    for (uint32_t i = 0; i < I; i++)
        for (uint32_t k = 0; k < D; k++) U[(size_t)i * D + k] = o_gaussian(0.0, init_sd); /* :236-242 */
    for (uint32_t k = 0; k < D; k++)
        for (uint32_t j = 0; j < J; j++) V[(size_t)k * J + j] = o_gaussian(0.0, init_sd); /* :244-250 */
    }

    double *sigma_u = calloc(D, sizeof(double)), *mu_u = calloc(D, sizeof(double));
    double *sigma_v = calloc(D, sizeof(double)), *mu_v = calloc(D, sizeof(double));
    const double a_0 = 1, b_0 = 1, alpha_0 = 1, beta_0 = 1, nu_0 = 1, mu_0 = 0.0; /* :256-269 */
    const double mu = 0, alpha_i = 0, beta_j = 0; /* biases compiled out (:276-295) */
    double tau = 1;

    double *E = calloc(n_train ? n_train : 1, sizeof(double));
    double *sum = calloc(n_test ? n_test : 1, sizeof(double));
    const uint32_t iters = cfg->iters + cfg->burnin;
    double t_start = now_s();
    res->sweeps_done = 0;

    /* Philox mode only (the glibc stream is sequential): rows of a half-sweep are
     * independent given the partner table and touch disjoint E entries */
    const int nth = (px && cfg->threads > 1) ? cfg->threads : 1;
    (void)nth;
    for (uint32_t iter = 0; iter < iters; iter++) {
        /* E recompute :317-334 */
        double esq = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : esq) num_threads(nth) if (nth > 1)
        for (uint64_t c = 0; c < n_train; c++) {
            uint32_t user = tu[c], item = ti[c];
            double temp = 0.0;
            for (uint32_t k = 0; k < D; k++) temp += U[(size_t)user * D + k] * V[(size_t)k * J + item];
            E[c] = tr[c] - (mu + alpha_i + beta_j + temp);
            esq += (E[c] * E[c]);
        }
        /* tau :339-342 */
        px_stream ps = {pseed, iter, 0, {0, 0}, 0};
        tau = px ? px_gamma(&ps, a_0 + 0.5 * (double)n_train) / (b_0 + 0.5 * esq)
                 : o_gamma(a_0 + 0.5 * (double)n_train, b_0 + 0.5 * esq);
        /* hyperparameters :375-414 */
        for (uint32_t k = 0; k < D; k++) {
            double temp = 0.0, temp2 = 0.0;
            for (uint32_t i = 0; i < I; i++) {
                double x = U[(size_t)i * D + k];
                temp += (x - mu_u[k]) * (x - mu_u[k]);
                temp2 += x;
            }
            double a_star = alpha_0 + 0.5 * (I + 1);
            double b_star = q2 ? beta_0 + nu_0 * (mu_u[k] - mu_0) * (mu_u[k] - mu_0) + (0.5) * temp
                               : beta_0 + 0.5 * nu_0 * (mu_u[k] - mu_0) * (mu_u[k] - mu_0) + (0.5) * temp;
            sigma_u[k] = px ? px_gamma(&ps, a_star) / b_star : o_gamma(a_star, b_star);
            double su_star = (double)1.0 / (nu_0 * sigma_u[k] + sigma_u[k] * I);
            double mu_star = su_star * (nu_0 * mu_0 * sigma_u[k] + sigma_u[k] * temp2);
            if (px)
                mu_u[k] = mu_star + (qnone ? sqrt(su_star) : su_star) * px_leva(&ps);
            else
                mu_u[k] = o_gaussian(mu_star, qnone ? sqrt(su_star) : su_star);

            temp = 0.0;
            temp2 = 0.0;
            for (uint32_t j = 0; j < J; j++) {
                double x = V[(size_t)k * J + j];
                temp += (x - mu_v[k]) * (x - mu_v[k]);
                temp2 += x;
            }
            a_star = alpha_0 + 0.5 * (J + 1);
            b_star = q2 ? beta_0 + nu_0 * (mu_v[k] - mu_0) * (mu_v[k] - mu_0) + (0.5) * temp
                        : beta_0 + 0.5 * nu_0 * (mu_v[k] - mu_0) * (mu_v[k] - mu_0) + (0.5) * temp;
            sigma_v[k] = px ? px_gamma(&ps, a_star) / b_star : o_gamma(a_star, b_star);
            double sv_star = (double)1.0 / (nu_0 * sigma_v[k] + sigma_v[k] * J);
            double mv_star = (q2 ? su_star : sv_star) * (nu_0 * mu_0 * sigma_v[k] + sigma_v[k] * temp2);
            if (px)
                mu_v[k] = mv_star + (qnone ? sqrt(sv_star) : sv_star) * px_leva(&ps);
            else
                mu_v[k] = o_gaussian(mv_star, qnone ? sqrt(sv_star) : sv_star);
        }
        /* users :453-491 */
#pragma omp parallel for schedule(dynamic, 64) num_threads(nth) if (nth > 1)
        for (uint32_t i = 0; i < I; i++) {
            uint32_t b = R.ptr[i], e = R.ptr[i + 1];
            for (uint32_t k = 0; k < D; k++) {
                const double *Vk = V + (size_t)k * J;
                double temp = 0.0, temp2 = 0.0;
                double *Uik = &U[(size_t)i * D + k];
                for (uint32_t p = b; p < e; p++) {
                    double v = Vk[R.oth[p]];
                    temp += (v * v);
                    temp2 += (v * (E[R.cas[p]] + v * *Uik));
                }
                double s_star = (double)1.0 / (sigma_u[k] + (tau * temp));
                double m_star = s_star * (tau * temp2 + sigma_u[k] * mu_u[k]);
                double old = *Uik;
                if (px)
                    *Uik = m_star + (qnone ? sqrt(s_star) : s_star) * px_normal(pseed, i, iter, PX_TAG_USERS, k);
                else
                    *Uik = o_gaussian(m_star, qnone ? sqrt(s_star) : s_star); /* serial: nth == 1 */
                for (uint32_t p = b; p < e; p++) E[R.cas[p]] += Vk[R.oth[p]] * (old - *Uik);
            }
        }
        /* items :495-535 */
#pragma omp parallel for schedule(dynamic, 16) num_threads(nth) if (nth > 1)
        for (uint32_t j = 0; j < J; j++) {
            uint32_t b = Rt.ptr[j], e = Rt.ptr[j + 1];
            for (uint32_t k = 0; k < D; k++) {
                double temp = 0.0, temp2 = 0.0;
                double *Vjk = &V[(size_t)k * J + j];
                for (uint32_t p = b; p < e; p++) {
                    double u = U[(size_t)Rt.oth[p] * D + k];
                    temp += (u * u);
                    temp2 += (u * (E[Rt.cas[p]] + *Vjk * u));
                }
                double s_star = (double)1.0 / (sigma_v[k] + (tau * temp));
                double m_star = s_star * (tau * temp2 + sigma_v[k] * mu_v[k]);
                double old = *Vjk;
                if (px)
                    *Vjk = m_star + (qnone ? sqrt(s_star) : s_star) * px_normal(pseed, j, iter, PX_TAG_ITEMS, k);
                else
                    *Vjk = o_gaussian(m_star, qnone ? sqrt(s_star) : s_star);
                for (uint32_t p = b; p < e; p++) E[Rt.cas[p]] += U[(size_t)Rt.oth[p] * D + k] * (old - *Vjk);
            }
        }
        /* test RMSE :539-563 (sbpmf2 gates on iter>=0, i.e. always) */
        double rmse = NAN, rmse_this = NAN;
        if (iter >= cfg->burnin || q2) {
            double diff = 0.0, diff_this = 0.0;
            for (uint64_t t = 0; t < n_test; t++) {
                uint32_t user = su[t], item = si[t];
                double temp = mu + alpha_i + beta_j;
                for (uint32_t k = 0; k < D; k++) temp += U[(size_t)user * D + k] * V[(size_t)k * J + item];
                temp = (temp < hi) ? temp : hi; /* std::min(5.0, temp) */
                temp = (lo < temp) ? temp : lo; /* std::max(1.0, temp) */
                sum[t] += temp;
                diff += (sr[t] - ((double)sum[t] / (iter + 1))) * (sr[t] - ((double)sum[t] / (iter + 1)));
                diff_this += (sr[t] - temp) * (sr[t] - temp);
            }
            rmse = sqrt(diff / n_test);
            rmse_this = sqrt(diff_this / n_test);
        }
        if (res->rmse && iter < res->rmse_cap) res->rmse[iter] = rmse;
        if (res->rmse_this && iter < res->rmse_cap) res->rmse_this[iter] = rmse_this;
        if (res->tau && iter < res->rmse_cap) res->tau[iter] = tau;
        res->sweeps_done = iter + 1;
        if (cfg->sweep_seconds_limit > 0 && now_s() - t_start > cfg->sweep_seconds_limit) break;
    }
    res->seconds = now_s() - t_start;

    /* export factors row-major: U[i][k], V[j][k] */
    if (res->U)
        memcpy(res->U, U, (size_t)I * D * sizeof(double));
    if (res->V)
        for (uint32_t j = 0; j < J; j++)
            for (uint32_t k = 0; k < D; k++) res->V[(size_t)j * D + k] = V[(size_t)k * J + j];
    if (res->hyper) { /* [sigma_u | mu_u | sigma_v | mu_v], K each */
        memcpy(res->hyper, sigma_u, D * sizeof(double));
        memcpy(res->hyper + D, mu_u, D * sizeof(double));
        memcpy(res->hyper + 2 * D, sigma_v, D * sizeof(double));
        memcpy(res->hyper + 3 * D, mu_v, D * sizeof(double));
    }
    if (res->pred_sum && n_test) memcpy(res->pred_sum, sum, n_test * sizeof(double));

    free(U); free(V); free(sigma_u); free(mu_u); free(sigma_v); free(mu_v);
    free(E); free(sum);
    free_lists(&R); free_lists(&Rt);
    return 0;
}

int oracle_load_triples(const char *path, uint64_t *n, uint32_t **u, uint32_t **i, double **r) {
    return read_triples(path, u, i, r, n);
}

void oracle_free(void *p) { free(p); }

#ifdef ORACLE_MAIN
/* CLI: sbpmf_oracle TRAIN TEST K ITERS SEED [final|sbpmf2|none|bias2|bias22]
 * prints "rmse is %.17g" per collection sweep, like gibbs_sbpmf_final.cpp:562 */
int main(int argc, char **argv) {
    if (argc < 6) {
        fprintf(stderr, "usage: %s TRAIN TEST K ITERS SEED [final|sbpmf2|none|bias2|bias22]\n", argv[0]);
        return 2;
    }
    oracle_config cfg;
    oracle_config_default(&cfg);
    cfg.K = atoi(argv[3]);
    cfg.iters = atoi(argv[4]);
    cfg.seed = (unsigned)strtoul(argv[5], NULL, 10);
    if (argc > 6) {
        if (!strcmp(argv[6], "sbpmf2")) cfg.quirks = ORACLE_QUIRKS_SBPMF2;
        else if (!strcmp(argv[6], "none")) cfg.quirks = ORACLE_QUIRKS_NONE;
        else if (!strcmp(argv[6], "bias2")) cfg.quirks = ORACLE_QUIRKS_BIAS2;
        else if (!strcmp(argv[6], "bias22")) cfg.quirks = ORACLE_QUIRKS_BIAS22;
    }
    uint64_t n, nt;
    uint32_t *u, *i, *su, *si;
    double *r, *sr;
    if (read_triples(argv[1], &u, &i, &r, &n) || read_triples(argv[2], &su, &si, &sr, &nt)) {
        fprintf(stderr, "cannot read input\n");
        return 1;
    }
    double *rm = calloc(cfg.iters, sizeof(double));
    oracle_result res;
    memset(&res, 0, sizeof res);
    res.rmse = rm;
    res.rmse_cap = cfg.iters;
    oracle_run_arrays(&cfg, n, u, i, r, nt, su, si, sr, 0, 0, &res);
    for (uint32_t s = 0; s < res.sweeps_done; s++) printf("rmse is %.17g\n", rm[s]);
    return 0;
}
#endif
