/*
 * sbmf.h -- C ABI of the MI355X-native Scalable-BPMF (SBPMF) Gibbs sampler.
 *
 * This is the drop-in boundary for the reference's hot path.  The reference
 * has no library interface: its sampler is the body of main() in
 * src/libfm/gibbs_sbpmf_final.cpp:23-595 (and the libFM learner behind
 * `bin/libFM -method mcmc`, src/libfm/libfm.cpp:72-644 ->
 * fm_learn_mcmc::learn, fm_learn_mcmc.h:1154).  Each entry point below names
 * the reference code it replaces.  Plain C types only: no torch, no HIP types.
 * The CLI (`sbmf`, libFM flag grammar) and the Python mirror (package
 * sbmf/) are built on exactly these calls; INTEGRATION.md shows the ctypes
 * binding a maintainer would add.
 *
 * Ownership: the caller owns every host array it passes (they are copied in);
 * the library owns all device memory, streams and RCCL communicators.
 * Errors: every call returns SBMF_OK (0) or a negative SBMF_E_* code and
 * records a message readable with sbmf_last_error(ctx) (or
 * sbmf_last_global_error() when no context exists).  The reference instead
 * throws std::string / const char* and still exits 0 (libfm.cpp:636-640).
 * Threading: a context is used by one host thread at a time.
 * Device: every compute entry point requires a gfx950 GPU; there is no CPU
 * fallback (sbmf_create fails with SBMF_E_DEVICE without one).
 */
#ifndef SBMF_H_
#define SBMF_H_
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SBMF_ABI_VERSION 2
#define SBMF_NKIND 11 /* kernel kinds reported by sbmf_get_timing */

enum sbmf_status {
    SBMF_OK = 0,
    SBMF_E_ARG = -1,      /* invalid argument / configuration                    */
    SBMF_E_STATE = -2,    /* call out of order (e.g. run before set_train)       */
    SBMF_E_DEVICE = -3,   /* HIP runtime error or no usable GPU                  */
    SBMF_E_IO = -4,       /* file open / parse error                             */
    SBMF_E_COMM = -5,     /* RCCL error                                          */
    SBMF_E_NOMEM = -6     /* host or device allocation failed                    */
};

/* RNG mode. REFERENCE replays the reference's exact variate stream (glibc
 * rand(), Leva normals, Marsaglia-Tsang gammas; src/util/random.h:118-176),
 * generated on the host and consumed by the GPU; PHILOX draws counter-based
 * normals inside the kernels (throughput mode, rank-count independent). */
enum sbmf_rng_mode { SBMF_RNG_REFERENCE = 0, SBMF_RNG_PHILOX = 1 };

/* Quirk set. FINAL = gibbs_sbpmf_final.cpp semantics (posterior VARIANCE
 * passed as the stdev of ran_gaussian, :393,413,485,529; init N(0,1); clamp
 * [1,5]).  SBPMF2 = src/libfm/gibbs_sbpmf2.cpp (:240,248,386,406,412,557:
 * init N(0,0.1), nu0 without 1/2, mu_v uses sigma_u*, clamp [0.5,5]).
 * NONE = the statistically correct sampler (stdev = sqrt(variance)).
 * BIAS2 = the biased sampler at the top level of the reference,
 * gibbs_sbpmf2.cpp:335-637 (the paper's Algorithm 1, libFM -dim '1,1,K'):
 * global bias b0 and per-user / per-item biases with Normal-Gamma priors,
 * alpha ~ G(a0 + N, b0 + sum E^2), factor precisions with shape alpha0 + I,
 * posterior variance as stdev, init N(0,0.1), clamp [0.5,5].  BIAS22 = the
 * same sampler as src/libfm/gibbs_sbpmf22.cpp (init N(0,1), clamp [1,5]). */
enum sbmf_quirks { SBMF_QUIRKS_FINAL = 0, SBMF_QUIRKS_SBPMF2 = 1, SBMF_QUIRKS_NONE = 2, SBMF_QUIRKS_BIAS2 = 3,
                   SBMF_QUIRKS_BIAS22 = 4 };

/* Learner (libFM -method, libfm.cpp:394-445).  MCMC = the SBPMF Gibbs sampler.
 * VB = online variational Bayes, the reference's fm_learn_vb_online
 * (src/libfm/src/fm_learn_vb_online.h, -method vb_online; its batch -method vb
 * is a no-op as shipped): per epoch a shuffle into
 * mini-batches and natural-gradient steps (t0 + t)^-0.5 on the per-attribute
 * Gaussian posteriors of w0, w and V.  With VB a "sweep" of sbmf_run is an
 * epoch, rmse_avg is the test RMSE of the posterior-mean prediction, tau is
 * alpha, factors / biases are the posterior means, and only F64 is offered. */
/* LIBFM_MCMC = libFM's own MCMC chain (bin/libFM -method mcmc,
 * src/libfm/src/fm_learn_mcmc.h:411-623 draw_all, fm_learn_mcmc_simultaneous.h):
 * a factorization machine over the users-first one-hot attributes (user u,
 * item I + i) with global bias w0, attribute biases w and factors v, one
 * attribute group with Normal-Gamma hyperpriors, noise precision alpha, the
 * factors drawn f-outer (per factor: every user, then every item) with the
 * posterior standard deviation; a sweep re-predicts train and test.  ALS =
 * the same learner without sampling or hyperparameter inference (bin/libFM
 * -method als, libfm.cpp:132-136): deterministic.  Both use libfm_dim and
 * reg0 / regw / regv, f64 only; rmse_train / rmse_avg are libFM's "Train=" /
 * "Test=", tau is alpha.  On several GPUs (sbmf_comm_init) each rank owns a
 * sbmf_partition_rows user range and every case of those users; the item sums
 * are all-gathered and added in rank order, so every rank draws the same items
 * and the chain equals one rank's up to the rounding of that sum. */
enum sbmf_method { SBMF_METHOD_MCMC = 0, SBMF_METHOD_VB = 1, SBMF_METHOD_LIBFM_MCMC = 2, SBMF_METHOD_ALS = 3 };

/* Arithmetic type of factors, residuals and reductions on the GPU.  F64 is
 * the reference's (all-double) arithmetic. */
enum sbmf_precision { SBMF_F64 = 0, SBMF_F32 = 1 };

typedef struct sbmf_config {
    uint32_t num_factor;   /* K: -dim 'k0,k1,K' (libfm.cpp:93); reference D=20 (:218)          */
    uint32_t num_iter;     /* collection sweeps: -iter (libfm.cpp:97); reference 100 (:299)     */
    uint32_t burnin;       /* burn-in sweeps before collection; reference 0 (:300)              */
    uint64_t seed;         /* -seed (honoured; the reference ignores it, libfm.cpp:124)         */
    int32_t rng_mode;      /* enum sbmf_rng_mode                                               */
    int32_t quirks;        /* enum sbmf_quirks                                                 */
    int32_t precision;     /* enum sbmf_precision                                              */
    int32_t device;        /* HIP device ordinal for this context                              */
    double init_stdev;     /* <0: quirk-set default (1.0 final / 0.1 sbpmf2); -init_stdev      */
    double clamp_lo;       /* prediction clamp; <0: quirk-set default (1.0 / 0.5)              */
    double clamp_hi;       /* default 5.0 (gibbs_sbpmf_final.cpp:556)                          */
    /* hyperpriors (gibbs_sbpmf_final.cpp:256-269) */
    double a0, b0, alpha0, beta0, nu0, mu0;
    uint32_t recompute_every; /* recompute E=r-UV from scratch every n sweeps (reference: every
                                 sweep, :317-334); 0 = only at start                            */
    uint32_t eval_train;      /* 1: compute train RMSE of the current sample each sweep          */
    uint32_t eval_test;       /* 1: test prediction + running-mean RMSE each sweep (:539-563)    */
    uint32_t gram_threshold;  /* reserved, must be 0 (the full-Gram row route was removed)       */
    uint32_t row_kernel;      /* reserved, must be 0 (the per-coordinate row kernels were removed:
                                 the MFMA Gram-block kernels are the only row kernels)          */
    uint32_t stream_threshold;/* rows with more ratings use the streaming Gram-block kernel
                                 k_gres (0 = default: 256 f64 / 512 f32)                        */
    uint32_t split_chunk;     /* streaming-kernel task size: rows longer than this are split
                                 into chunks on co-resident workgroups (0 = the register
                                 capacity of the workgroup shape; larger values are capped to it) */
    uint32_t tune;            /* kernel-variant bits for experiments (0 = tuned defaults):
                                 bit 1 = residuals from r - own.partner as on several GPUs,
                                 bit 2 = power-of-two waves per Gram-block row (2/4/8) instead
                                         of ceil(ratings / ratings-per-wave),
                                 bit 3 = f64 rows of 33..64 ratings on two 8-vector waves instead
                                         of one 16-vector wave,
                                 bit 7 = k_gres on 4-wave workgroups (both sides),
                                 bit 8 = f64 rows of 65..128 ratings as 3-4-wave Gram-block rows
                                         (default: one-wave k_grow workgroups),
                                 bit 9 = f64 rows of 129..256 ratings as 3-4-wave Gram-block rows
                                         (default: two-wave k_grow workgroups),
                                 bit 10 = f64 rows of 9..64 ratings on the one-wave Gram-block
                                          kind (default: one-wave k_grow workgroups),
                                 bit 11 = f32 rows of 17..512 ratings on the Gram-block kinds
                                          (default: one- / two-wave k_grow workgroups),
                                 bit 12 = k_grow reads sigma and mu from memory at every K
                                          (default: from LDS when Kp <= 128),
                                 bit 13 = f64 user streaming rows all on one 4-wave k_gres set
                                          (default: rows above 512 ratings on a second, 8-wave set),
                                 bit 14 = (experiment) that second user set on 16-wave workgroups,
                                 bit 17 = k_gres on 16-wave workgroups (both sides),
                                 bit 23 = f64 user streaming rows all on 8-wave k_gres workgroups
                                          (default: up to 512 ratings on 4-wave ones, 512-rating
                                          tasks, longer rows on a second, 8-wave set),
                                 bit 24 = k_gres as a cooperative launch (experiments only; the
                                          default is an ordinary launch in every schedule: tasks are
                                          claimed in queue order, no co-residency needed),
                                 bit 25 = a half's Gram-block kinds all on one side stream
                                          (default since round 5: alternating between two side
                                          streams, beside each other and the streaming launch),
                                 bit 26 = no overlap of the next sweep's prologue (sums, column
                                          statistics, host draws) with the test evaluation
                                          (Philox mode; the chain is the same either way),
                                 bit 27 = f64 item rows on 8-wave k_gres workgroups (default:
                                          rows > 1024 ratings on 16-wave ones, the rest 8-wave),
                                 bit 29 = a half's Gram-block launches after its streaming launch
                                          on one stream (default: on a second stream beside it),
                                 bit 30 = a half's two streaming sets (items: rows > 1024 and the
                                          rest) one after the other (default: side by side),
                                 bit 28 = (one rank) the test evaluation after the next sweep's
                                          prologue kernels on the compute stream (default: on the
                                          second stream beside them; the results are the same).
                                 Every other bit is refused (SBMF_E_ARG): bits 0, 4-6, 15, 16,
                                 18-22 and 31 selected variants removed in rounds 1-6 (measured
                                 slower or neutral, kept in git history).  Bits whose meaning
                                 changed between rounds: 24 (round 4: ordinary
                                 launch; since round 5 the cooperative one), 25 (round-4 LDS-DMA
                                 prefetch; since round 5 one side stream).  */
    uint32_t method;          /* enum sbmf_method: -method mcmc (default) | vb                   */
    uint32_t vb_batches;      /* online VB: mini-batches per epoch (0 = the reference's 30,
                                 fm_learn_vb_online_simultaneous.h:62)                           */
    uint32_t average;         /* running mean of the test prediction: 0 = quirk-set default
                                 (sum / (sweep + 1), gibbs_sbpmf_final.cpp:559, which counts
                                 burn-in sweeps; quirks none: collected sweeps), 1 = sum over
                                 the collected sweeps / their number, 2 = sum / (sweep + 1)       */
    uint32_t libfm_dim;       /* LIBFM_MCMC / ALS: the k0,k1 of -dim 'k0,k1,K' as bits: bit 0 =
                                 global bias w0, bit 1 = attribute biases w (default 3)          */
    double reg0, regw, regv;  /* LIBFM_MCMC / ALS: -regular 'r0,r1,r2' (libfm.cpp:484-513): ALS's
                                 fixed precisions, MCMC's starting w / v precisions (default 0) */
    uint32_t pipeline;        /* SBPMF sampler, throughput mode (Philox, prologue overlap on): 1 =
                                 sweep s+1's start (its hyperparameter upload and user half) is
                                 queued before sweep s is reported to the run callback, so the
                                 device does not idle through the host's per-sweep work.  The
                                 chain and the reports are the same; the callback must not read
                                 device state (factors, predictions), and a stop it asks for takes
                                 effect after sweep s+1.  0 (default): each sweep is reported with
                                 the device idle after it                                         */
} sbmf_config;

/* Per-sweep report passed to the run callback. */
typedef struct sbmf_sweep_info {
    uint32_t sweep;            /* 0-based sweep index (burn-in included)                     */
    uint32_t collected;        /* 1 if this sweep entered the running mean                   */
    double rmse_avg;           /* test RMSE of the running-mean prediction (the reference's
                                  "rmse is", gibbs_sbpmf_final.cpp:562); NaN if no test set  */
    double rmse_this;          /* test RMSE of this sweep's sample alone                      */
    double rmse_train;         /* train RMSE of this sample (clamped), NaN if not evaluated   */
    double tau;                /* noise precision drawn this sweep                           */
    double ms_sweep;           /* device time of the sweep from its start to the end of the item
                                  half, ms.  Throughput mode (overlapped start): the sweep's start
                                  work -- residual sum, column statistics, both normal fills and
                                  the hyperparameter upload -- was queued at the end of the
                                  previous sweep, beside its test evaluation, and is not in here
                                  (sbmf_timing.ms_hyper of the previous sweep holds it)        */
    double ms_eval;            /* device time of the test evaluation, ms                      */
} sbmf_sweep_info;

/* Return non-zero to stop the run early. */
typedef int (*sbmf_sweep_cb)(const sbmf_sweep_info* info, void* user);

typedef struct sbmf_ctx sbmf_ctx;

/* --- configuration / lifetime -------------------------------------------------------------- */
/* Fill reference defaults (gibbs_sbpmf_final.cpp:218,256-269,299-300). */
int sbmf_config_default(sbmf_config* cfg);
/* Create a context on cfg->device.  Replaces the reference's setup in main()
 * (gibbs_sbpmf_final.cpp:252-306).  Fails with SBMF_E_DEVICE without a GPU. */
int sbmf_create(const sbmf_config* cfg, sbmf_ctx** out);
void sbmf_destroy(sbmf_ctx* ctx);
const char* sbmf_last_error(const sbmf_ctx* ctx);
const char* sbmf_last_global_error(void);
int sbmf_abi_version(void);

/* --- data ---------------------------------------------------------------------------------- */
/* Training triples (0-based ids, any order; file order is preserved as the
 * reference's R / R_t entry order, gibbs_sbpmf_final.cpp:192-215). */
int sbmf_set_train(sbmf_ctx* ctx, uint64_t n, const uint32_t* user, const uint32_t* item, const double* rating);
int sbmf_set_test(sbmf_ctx* ctx, uint64_t n, const uint32_t* user, const uint32_t* item, const double* rating);
/* Optional: row counts.  Default (0,0) = max id + 1 over train and test
 * (gibbs_sbpmf_final.cpp:146-148); empty ids are kept and sampled. */
int sbmf_set_dims(sbmf_ctx* ctx, uint32_t num_users, uint32_t num_items);

/* Build the device layout (CSR / CSC, degree bins), upload, and initialise
 * U, V (draws the init variates, :236-250).  Implicitly called by sbmf_run. */
int sbmf_prepare(sbmf_ctx* ctx);

/* Run `sweeps` Gibbs sweeps (continuing the chain across calls).  One sweep =
 * the reference loop body gibbs_sbpmf_final.cpp:309-564: tau, per-factor
 * hyperparameters, user half-sweep, item half-sweep, test evaluation. */
int sbmf_run(sbmf_ctx* ctx, uint32_t sweeps, sbmf_sweep_cb cb, void* user);

/* --- results ------------------------------------------------------------------------------- */
/* Averaged clamped test prediction (sum / collected sweeps; libfm -out,
 * libfm.cpp:629-634).  out: [n_test]. */
int sbmf_predict(sbmf_ctx* ctx, double* out);
/* Factors as row-major doubles: U [num_users][K], V [num_items][K]. Either may be NULL. */
int sbmf_get_factors(sbmf_ctx* ctx, double* U, double* V);
/* Overwrite the factors (row-major doubles).  For checkpoints and tests. */
int sbmf_set_factors(sbmf_ctx* ctx, const double* U, const double* V);
/* Hyperparameters [sigma_u | mu_u | sigma_v | mu_v] (4K doubles) and tau. */
int sbmf_get_hyper(sbmf_ctx* ctx, double* hyper4k, double* tau);
int sbmf_get_dims(sbmf_ctx* ctx, uint32_t* num_users, uint32_t* num_items, uint64_t* n_train, uint64_t* n_test);
/* Biased sampler only: b_i [num_users], b_j [num_items] and the global b_0
 * (gibbs_sbpmf2.cpp:276-318 state).  Any pointer may be NULL. */
int sbmf_get_biases(sbmf_ctx* ctx, double* bu, double* bv, double* b0);

/* --- measurement --------------------------------------------------------------------------- */
/* Device times of the last sweep (HIP events on the context's stream).
 * kern_*[side][kind]: side 0 = user half, 1 = item half; kind =
 *   0..4  MFMA Gram-block row kernels: 1 wave/row (two sizes), then 2..8
 *         waves/row (ceil(ratings/32) f64, /64 f32) timed in three groups; up to
 *         8/64/64/128/256 ratings (f64), 16/64/128/256/512 (f32),
 *   5     streaming MFMA Gram-block kernel k_gres: one persistent launch per
 *         stream set over tasks of <= 512 / 1024 / 2048 (f64, 4- / 8- / 16-wave
 *         workgroups) ratings held in VGPRs -- whole rows, or chunks of longer
 *         rows on co-resident workgroups -- plus the publish of split rows,
 *   6..10 reserved (the removed per-coordinate and full-Gram row kernels: 0).
 * kern_ms of the streaming kind is the last sweep's; those of kinds 0..4 are timed on
 * the first sweep of each sbmf_run call and kept (an event between two launches on a
 * stream leaves the device idle for microseconds).  kern_bytes is the
 * algorithmic traffic of that launch per SURVEY.md §8(d): per rating
 * s*K (partner row) + 4 (partner id) + s (residual), per row 2*s*K (own row
 * read + write), s = 4 (f32) or 8 (f64). */
typedef struct sbmf_timing {
    double ms_user_half, ms_item_half, ms_hyper, ms_eval, ms_comm;
    double kern_ms[2][SBMF_NKIND];
    uint64_t kern_bytes[2][SBMF_NKIND];
    uint32_t kern_rows[2][SBMF_NKIND];
    uint64_t bytes_algorithmic;  /* whole sweep, both halves                                    */
    uint32_t n_launch;           /* kernel launches in the last sweep                           */
    double ms_vb_factor;         /* online VB: device time of an epoch's factor passes (the 2K
                                    vbo_user_v / vbo_item_v launches of every mini-batch, HIP
                                    events around each batch's factor loop), mean over the last
                                    run's epochs (round 6); 0 for the other learners              */
} sbmf_timing;
int sbmf_get_timing(sbmf_ctx* ctx, sbmf_timing* t);

/* --- multi-GPU (one process per GPU, RCCL over xGMI) ---------------------------------------- */
/* 128-byte RCCL unique id, produced by rank 0 and shared by the launcher. */
int sbmf_comm_unique_id(uint8_t id[128]);
/* Join an nranks-wide communicator; users and items are then block-partitioned
 * (nnz-balanced) and U / V blocks are all-gathered between half-sweeps. */
int sbmf_comm_init(sbmf_ctx* ctx, int nranks, int rank, const uint8_t id[128]);
/* One communicator for the whole process, shared by several contexts in turn (a
 * driver running many learners on the same ranks, e.g. bench.py's legs): RCCL's
 * set-up (ncclCommInitRank) runs once.  sbmf_comm_attach joins a context to it
 * in place of sbmf_comm_init (before sbmf_prepare); the communicator must
 * outlive every context attached to it.  Contexts attached to one communicator
 * must not run at the same time.  `device` is this rank's HIP device (the contexts'
 * sbmf_config.device); RCCL binds the communicator to it. */
typedef struct sbmf_comm sbmf_comm;
int sbmf_comm_create(int device, int nranks, int rank, const uint8_t id[128], sbmf_comm** out);
int sbmf_comm_attach(sbmf_ctx* ctx, sbmf_comm* comm);
void sbmf_comm_destroy(sbmf_comm* comm);

/* --- loaders (the reference's input formats) ------------------------------------------------ */
typedef struct sbmf_ratings {
    uint64_t n;
    uint32_t* user;
    uint32_t* item;
    double* rating;
} sbmf_ratings;
/* SBPMF triple format "u<sep>i<sep>r" per line, lines accepted iff
 * sscanf("%u%c%u%c%lf") >= 5 (gibbs_sbpmf_final.cpp:43).  Replaces the three
 * serial text passes of gibbs_sbpmf_final.cpp:26-215: one read, line-aligned
 * chunks parsed on threads (SBMF_LOAD_THREADS, default min(cores,
 * OMP_NUM_THREADS)), concatenated in file order. */
int sbmf_load_triples(const char* path, sbmf_ratings* out);
/* libFM text "r f1:v f2:v" (Data.h:192-217) with exactly one user and one
 * item feature per line: the first feature is the user id, the second the
 * item id minus item_offset (users-first layout, e.g. data/m1m/m100k). */
int sbmf_load_libfm(const char* path, uint32_t item_offset, sbmf_ratings* out);
/* libFM binary input <stem>.x + <stem>.y (or .data + .target, preferred as in
 * Data::load, Data.h:113-160): the files tools/convert.cpp:55-205 writes,
 * layouts fmatrix.h:36-52 (sparse rows) and matrix.h:280-328 (targets).  Same
 * one-user-one-item rule and item_offset meaning as sbmf_load_libfm.  Replaces
 * the binary branch of Data::load (Data.h:115-160). */
int sbmf_load_libfm_binary(const char* stem, uint32_t item_offset, sbmf_ratings* out);
/* The transpose <stem>.xt + <stem>.y (or .datat + .target, preferred): the
 * file tools/transpose.cpp:54-172 writes from a .x, one sparse row per
 * feature listing its cases.  This is what bin/libFM -method mcmc|als reads:
 * its data sets are built with has_x = false (libfm.cpp:132-149), so Data::load
 * (Data.h:113-117,143-151) opens only the transpose.  Each case must hold two
 * features; the lower id is the user, the higher the item (item_offset as
 * above).  Replaces the has_xt branch of Data::load. */
int sbmf_load_libfm_binary_t(const char* stem, uint32_t item_offset, sbmf_ratings* out);
/* Data::load's choice of input (Data.h:112-117) for a data set that needs the
 * row-major cases (has_x) and / or the transpose (has_xt): 1 = <stem>.data
 * [+ .datat] + .target, 2 = <stem>.x [+ .xt] + .y, 0 = neither (Data::load
 * then parses <stem> as libFM text); SBMF_E_ARG if both flags are 0. */
int sbmf_libfm_binary_kind(const char* stem, int has_x, int has_xt);
/* Data::load (Data.h:106-283) for rating data: the binary input
 * sbmf_libfm_binary_kind picks for (has_x, has_xt) -- the cases read from the
 * row-major file when has_x, from the transpose otherwise -- else <stem> as libFM text
 * (sbmf_load_libfm).  bin/libFM's sets: has_x = 0, has_xt = 1 for -method
 * mcmc and als, both 1 for the other methods (libfm.cpp:132-149). */
int sbmf_load_libfm_data(const char* stem, int has_x, int has_xt, uint32_t item_offset, sbmf_ratings* out);
/* Writes <stem>.xt / <stem>.y: what tools/convert.cpp then tools/transpose.cpp
 * write for the same cases, byte for byte (rows per feature 0..num_cols-1,
 * ascending case ids, value 1). */
int sbmf_save_libfm_binary_t(const char* stem, const sbmf_ratings* in, uint32_t item_offset, uint32_t num_cols);
/* Writes <stem>.x / <stem>.y in that format (the convert tool's output for
 * rating data): row q = {user[q]:1, item_offset + item[q]:1}, f32 targets;
 * num_cols = max(num_cols, largest feature id + 1). */
int sbmf_save_libfm_binary(const char* stem, const sbmf_ratings* in, uint32_t item_offset, uint32_t num_cols);
/* Writes the SBPMF triple format "u\tv\tr\n" (0-based ids) that the reference's
 * data scripts produce (data/m100k/create_file_scalable_bpmf.py:6-12) and
 * sbmf_load_triples reads back bit for bit: integer ratings as integers, others
 * with %.17g. */
int sbmf_save_triples(const char* path, const sbmf_ratings* in);
void sbmf_free_ratings(sbmf_ratings* r);

/* --- multi-GPU layout (host only) ---------------------------------------------------------- */
/* The row partition every rank uses: contiguous row blocks balanced by
 * ratings (ptr = CSR/CSC offsets [R+1]), boundaries rounded to 256 rows.
 * bounds: [nranks+1]; rank k owns rows [bounds[k], bounds[k+1]). */
int sbmf_partition_rows(const uint32_t* ptr, uint32_t R, int nranks, uint64_t* bounds);

/* --- process exit (host only; not a reference interface) -------------------------------- */
/* First call: registers an exit handler that ends the process with _Exit(rc) once
 * the exit handlers registered after it (a profiler's, e.g. rocprofv3's output
 * writer) have run, skipping the shared-library finalizers -- under rocprofv3
 * (ROCm 7.2) the HIP runtime's finalizer faults after the profiler has finished
 * (profiles/r03_rocprof_teardown.txt).  Call it before the first HIP call; later
 * calls only set rc.  The handler belongs to libsbmf: do not dlclose it after.
 * Opt-in since round 4 (SBMF_EXIT=guard in bench.py and the CLI): the fault came
 * with RCCL linked at load time, and libsbmf now loads RCCL (dlopen) only for a
 * multi-GPU communicator, so a single-GPU process of the default schedule exits
 * normally under rocprofv3; a process that launched k_gres cooperatively (tune
 * bit 24, experiments only since round 5) faulted there. */
int sbmf_exit_guard(int rc);

/* --- test hooks ---------------------------------------------------------------------------- */
/* The host glibc-compatible stream (reference mode): n values of rand(),
 * ran_gaussian() and ran_gamma(shape) for seed. */
int sbmf_ref_stream(uint32_t seed, int kind, double shape, uint64_t n, double* out);
/* Philox normals as the kernels draw them: z for (seed, sweep, tag, row, k<K). out [K]. */
int sbmf_philox_normals(uint64_t seed, uint32_t sweep, uint32_t tag, uint32_t row, uint32_t K, double* out);

/* Timing only: make this context rank `rank` of an `nranks`-rank sampler run on
 * its one GPU, with every exchange skipped (no communicator: other ranks' rows
 * keep their initial values, residuals from other ranks read as 0).  The rank
 * runs exactly its own row blocks, stages, bins and streaming tasks, so its
 * device time is the per-rank compute of the multi-GPU schedule; its numbers are
 * not a chain.  Before sbmf_prepare; the SBPMF sampler only. */
int sbmf_test_virtual_rank(sbmf_ctx* ctx, int nranks, int rank);
/* A virtual rank's device time per stage of the last sweep's halves
 * (HIP events on the compute stream): ms[side * nstages + stage]. */
int sbmf_test_stage_ms(sbmf_ctx* ctx, double* ms, uint32_t cap, uint32_t* nstages);
/* RCCL self-test on one GPU (a prepared one-rank sampler context after at least
 * one sweep): a one-rank RCCL communicator through the library's own dlopen /
 * dlsym table issues, per repetition and on the multi-GPU comm stream, the
 * exchange's calls -- one group of three in-place ncclBroadcast over adjacent
 * blocks of an nbytes buffer, the grouped ncclSend / ncclRecv of the residual
 * exchange (to the rank itself), an ncclAllGather of nbytes/4 -- while the item
 * half's persistent k_gres grids run on the compute streams.  Every byte is
 * checked; the comm stream must finish within deadline_s (else SBMF_E_COMM). */
typedef struct sbmf_rccl_selftest {
    double ms_half;        /* the repetitions' item halves on the compute stream          */
    double ms_rccl;        /* the RCCL calls on the comm stream, first to last            */
    double ms_rccl_end;    /* from the first half's start to the last RCCL call's end     */
    uint64_t bad_bcast;    /* bytes the in-place broadcasts changed (must be 0)           */
    uint64_t bad_p2p;      /* received bytes that differ from the sent ones               */
    uint64_t bad_allgather;
    uint32_t n_calls;      /* RCCL collective / point-to-point calls issued               */
    uint32_t overlapped;   /* 1: the RCCL calls finished while the halves were running    */
} sbmf_rccl_selftest;
int sbmf_test_rccl_selftest(sbmf_ctx* ctx, uint64_t nbytes, uint32_t reps, double deadline_s,
                            sbmf_rccl_selftest* out);
/* The self-test runs `reps` extra item halves on the context's live chain, so the
 * context is spent afterwards: sbmf_run returns SBMF_E_STATE on it (create a new
 * one).  On a timeout the communicator is aborted (ncclCommAbort), the buffers
 * are left allocated, and sbmf_destroy leaks the context instead of waiting on
 * its queued work. */

/* Resource audit: hipMemGetInfo of `device` and what the library holds in this
 * process right now, counted where it is created and released (every device
 * buffer, pinned host buffer, stream, event, context and RCCL communicator of
 * every learner kind).  A process that has destroyed all of its contexts holds
 * nothing: the counts return to zero. */
typedef struct sbmf_device_usage {
    uint64_t device_free, device_total; /* hipMemGetInfo                                  */
    int64_t dev_bytes, dev_allocs;      /* device buffers the library holds              */
    int64_t pinned_bytes, pinned_allocs;/* pinned host buffers                           */
    int64_t streams, events, contexts, comms;
} sbmf_device_usage;
int sbmf_test_device_usage(int device, sbmf_device_usage* out);

#ifdef __cplusplus
}
#endif
#endif /* SBMF_H_ */
