/* sbpmf_oracle.h -- TEST INFRASTRUCTURE ONLY (see sbpmf_oracle.c header). */
#ifndef SBPMF_ORACLE_H_
#define SBPMF_ORACLE_H_
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* BIAS2: the biased sampler /root/reference/gibbs_sbpmf2.cpp (top level: init
 * 0.1*N(0,1), test clamp [0.5,5]); BIAS22: src/libfm/gibbs_sbpmf22.cpp (same
 * algorithm, init N(0,1), clamp [1,5]). */
enum { ORACLE_QUIRKS_FINAL = 0, ORACLE_QUIRKS_SBPMF2 = 1, ORACLE_QUIRKS_NONE = 2, ORACLE_QUIRKS_BIAS2 = 3,
       ORACLE_QUIRKS_BIAS22 = 4 };

typedef struct {
    uint32_t K, iters, burnin;
    unsigned seed;
    int quirks;
    double init_stdev, clamp_lo, clamp_hi;
    double sweep_seconds_limit; /* >0: stop after this many seconds (bounded CPU baseline) */
    int rng;                    /* 0: glibc rand() stream (the reference's); 1: the GPU build's Philox
                                   stream mode (unbiased samplers only) */
    int threads;                /* Philox mode: >1 = rows of each half-sweep in parallel over this many
                                   OpenMP threads (SURVEY.md §8(d)(ii) all-core CPU baseline) */
} oracle_config;

typedef struct {
    double *rmse, *rmse_this, *tau; /* [rmse_cap] or NULL */
    uint32_t rmse_cap;
    double *U, *V;     /* row-major [I][K], [J][K] or NULL */
    double *hyper;     /* [4K] or NULL */
    double *pred_sum;  /* [n_test] or NULL */
    uint32_t num_users, num_items, sweeps_done;
    double seconds;
    double *bu, *bv;   /* biased samplers: b_i [I], b_j [J] or NULL */
    double b0;         /* biased samplers: global bias b_0 */
} oracle_result;

void oracle_config_default(oracle_config *c);
int oracle_run_arrays(const oracle_config *cfg, uint64_t n_train, const uint32_t *tu, const uint32_t *ti,
                      const double *tr, uint64_t n_test, const uint32_t *su, const uint32_t *si,
                      const double *sr, uint32_t num_users, uint32_t num_items, oracle_result *res);
int oracle_load_triples(const char *path, uint64_t *n, uint32_t **u, uint32_t **i, double **r);
void oracle_free(void *p);
void oracle_srand(unsigned seed);
int oracle_rand(void);
double oracle_ran_uniform(void);
double oracle_ran_gaussian(void);
double oracle_ran_gamma(double alpha);

/* Online VB (vbo_oracle.c): the reference's `-method vb_online` learner on
 * rating data (user attribute u, item attribute num_users + i). */
typedef struct {
    uint32_t K, epochs;
    unsigned seed;
    uint32_t num_batch;     /* 0: the reference's 30 */
    double seconds_limit;   /* >0: stop after the epoch that crosses it (bounded CPU baseline) */
} oracle_vbo_config;

typedef struct {
    double *rmse;           /* [rmse_cap] per-epoch test RMSE, or NULL */
    uint32_t rmse_cap;
    double *pred;           /* [n_test] clamped predictions after the last epoch, or NULL */
    double *mu_w;           /* [num_attribute] or NULL */
    double *mu_v;           /* [num_attribute][K] or NULL */
    double alpha, mu0, seconds;
    uint32_t num_attribute, epochs_done;
} oracle_vbo_result;

void oracle_vbo_config_default(oracle_vbo_config *c);
int oracle_vbo_run(const oracle_vbo_config *cfg, uint64_t n_train, const uint32_t *tu, const uint32_t *ti,
                   const double *tr, uint64_t n_test, const uint32_t *su, const uint32_t *si, const double *sr,
                   uint32_t num_users, uint32_t num_items, oracle_vbo_result *res);

/* libFM MCMC / ALS (fmm_oracle.c): the reference's `bin/libFM -method mcmc|als`
 * learner (fm_learn_mcmc.h, fm_learn_mcmc_simultaneous.h) on cases with two
 * one-hot attributes a0 < a1, one attribute group, no relations. */
typedef struct {
    uint32_t K, iters;
    unsigned seed;        /* srand() value (libfm.cpp:124 seeds with time(NULL)) */
    int k0, k1;           /* -dim 'k0,k1,K' */
    int do_sample;        /* 0: ALS (libfm.cpp:132-136) */
    int do_multilevel;    /* 0: ALS */
    double init_stdev;    /* -init_stdev (default 0.1) */
    double reg0, regw, regv; /* -regular (initial / fixed lambdas; libfm.cpp:484-513) */
} oracle_fmm_config;

typedef struct {
    double *rmse_test, *rmse_this, *rmse_train, *alpha; /* [cap] per iteration, or NULL */
    uint32_t cap;
    double *pred;         /* [n_test] the -out predictions, or NULL */
    double *w;            /* [num_attribute] or NULL */
    double *v;            /* [K][num_attribute] (f-major, as fm_model::v) or NULL */
    double w0, min_target, max_target;
    uint32_t num_attribute, iters_done;
} oracle_fmm_result;

void oracle_fmm_config_default(oracle_fmm_config *c);
/* p_train / p_test: the data sets' num_feature (largest attribute id + 1). */
int oracle_fmm_run(const oracle_fmm_config *cfg, uint64_t n_train, const uint32_t *ta0, const uint32_t *ta1,
                   const double *ty, uint64_t n_test, const uint32_t *sa0, const uint32_t *sa1, const double *sy,
                   uint32_t p_train, uint32_t p_test, oracle_fmm_result *res);

#ifdef __cplusplus
}
#endif
#endif
