// kernels.h -- host-callable launchers for the gfx950 kernels in kernels.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace sbmf {

// Arguments of one half-sweep over the rows of one orientation (users: own =
// U, partner = V, CSR; items: own = V, partner = U, CSC).  T = float|double.
template <typename T>
struct HalfArgs {
    const uint32_t* ptr;   // [R+1] rating offsets of this orientation
    const uint32_t* part;  // [N] partner row id per rating
    const uint32_t* perm;  // [N] position of the rating in the other orientation's order
    const T* E_this;       // [N] residuals in this orientation's order (read sequentially)
    T* E_other;            // [N] residuals in the other orientation's order: E_other[perm[q]] (scatter)
    const T* r_this;       // [N] ratings in this order (e_from_dot, train RMSE)
    T* own;                // [R][Kp]
    const T* partner;      // [P+2][Kp]: row P is all zeros (sentinel), row P+1 slack
    const T* sig;          // [Kp] precision hyperparameter of this side (zero padded)
    const T* mu;           // [Kp] mean hyperparameter of this side (zero padded)
    uint32_t zrow;         // P: the partner table's zero row (ratings past a row's end point here)
    const T* zbuf;         // [R][K] N(0,1) variates of this half (host reference stream or launch_philox_fill)
    T tau;
    uint32_t K, Kp;
    int sd_is_var;         // quirk FINAL/SBPMF2: posterior variance used as stdev
    uint64_t seed;
    uint32_t sweep, tag;
    double* row_sq;        // [R] per-row sum of squared residuals after the half (or null)
    double* row_tr;        // [R] per-row train squared error of the clamped sample (or null)
    T lo, hi;
    int e_from_dot;        // 1: e0 = r - own.partner (no gather; multi-GPU)
    uint32_t tune;         // kernel variant bits (sbmf_config.tune)
    unsigned long long* prof;  // [8] phase cycles of wave 0 (SBMF_KPROF diagnostics) or null
    // extents of the arrays above, checked on every index by CHECK=1 builds (SBMF_CHECK_BUILD)
    uint64_t lim_partner;  // elements of `partner` ((P+2) Kp)
    uint64_t lim_other;    // elements of E_other (N + multi-GPU send area)
    uint64_t lim_this;     // N (part, perm, E_this, r_this)
    uint32_t lim_rows;     // R (own rows; zbuf rows)
};

// Gram-block (MFMA) row kernels.  Max ratings per row for each kind: f64
// holds 8 vectors (32 ratings) per wave, f32 16 (64 ratings).
enum GblockKind { GK_W4 = 0, GK_W16 = 1, GK_B2 = 2, GK_B4 = 3, GK_B8 = 4, GK_NUM = 5 };
inline uint32_t gk_maxdeg(int kind, bool f64, bool wide = false) {
    static const uint32_t waves4[GK_NUM] = {1, 4, 8, 16, 32};  // (waves x vectors) / V*4 ratings
    const uint32_t per_wave = f64 ? 32 : 64;
    // wide (f64 default; tune bit 3 turns it off): the 1-wave kind holds 16 vectors (64 ratings)
    if (wide && f64 && (kind == GK_W16 || kind == GK_B2)) return 64;
    return kind == GK_W4 ? per_wave / 4 : per_wave * waves4[kind] / 4;
}

// Multi-wave Gram-block rows with exactly `nw` (2..8) waves per row.
template <typename T>
hipError_t launch_gblock_nw(int nw, const uint32_t* rows, uint32_t nrows, const HalfArgs<T>& a, hipStream_t st);
template <typename T>
hipError_t launch_gblock(int kind, const uint32_t* rows, uint32_t nrows, const HalfArgs<T>& a, hipStream_t st);

// Whole rows of a Gram-block bin on the streaming kernel's code (k_grow), one workgroup of
// nw (1 or 2) waves per row: rows of at most grow_maxdeg(nw, f64) ratings.
template <typename T>
hipError_t launch_grow(int nw, const uint32_t* rows, uint32_t nrows, const HalfArgs<T>& a, hipStream_t st);
uint32_t grow_maxdeg(int nw, bool f64);

// Streaming-kernel task: at most `cmax` ratings of one row (the whole row,
// or one chunk of a row split over `nch` co-resident workgroups).  A task
// with len == 0 is an empty slot (round padding).
struct SplitTask {
    uint32_t row;    // global row id
    uint32_t beg;    // first rating of the chunk (absolute index)
    uint32_t len;    // ratings in the chunk
    uint32_t nch;    // chunks of the row (1 = whole row, no exchange)
    uint32_t chunk;  // chunk index within the row
    uint32_t slab0;  // split rows: first chunk slab of the row (also its new-own slot)
    uint32_t cnt0;   // split rows: first block counter of the row
    uint32_t pad;
};
struct SplitRow {
    uint32_t row, slab0, nch, pad;
};
struct SplitSync {
    double* slabs;       // [nchunk_total][nblk][16*16+16]
    uint32_t* counters;  // [nsplit_rows * nblk], then the task-queue head: zero at launch (k_split_finish clears them)
    uint32_t ncounters;
    uint32_t nblk;       // ceil(K/16)
    double* chunk_sq;    // [nchunk_total]
    double* chunk_tr;    // [nchunk_total]
    void* newown;        // [nchunk_total][Kp] (T), slot slab0 of each split row
    uint32_t* timeout;   // set to 1 if a spin gave up
    uint32_t cmax;       // ratings per task
    unsigned long long* prof;  // [8] phase cycles of wave 0 (SBMF_KPROF diagnostics) or null
    uint64_t lim_slab;   // doubles of `slabs` (CHECK=1 builds)
    uint32_t lim_chunk;  // entries of chunk_sq / chunk_tr (and rows of newown)
};
// Task capacity (ratings) of the streaming kernel k_gres for the variant `tune`:
// 4 * waves * vectors-per-wave, the partner slices held in VGPRs.
template <typename T>
uint32_t gstream_cmax(uint32_t tune);
// Workgroups per CU the streaming kernel variant `tune` is sized for.
int gstream_wg_target(uint32_t tune);
// Co-resident k_gres workgroups per CU (occupancy API).
template <typename T>
int gstream_blocks_per_cu(uint32_t cmax, uint32_t tune);
// All streaming tasks of a half-sweep in one persistent launch of `grid`
// (<= residency) workgroups.  Tasks are one list, claimed in order from a queue
// head by whichever workgroup is free; a split row's chunks are consecutive, so
// a chunk only waits for peers that the next free workgroups claim.  Split rows
// are then published by k_split_finish.  sy.counters[0..ncounters] must be zero
// when the launch starts: sbmf.cpp clears every set's counters with one memset
// per half, ahead of the half's launches.
template <typename T>
hipError_t launch_gstream(const SplitTask* tasks, uint32_t ntask, uint32_t grid, const SplitRow* srows, uint32_t nsrow,
                          const HalfArgs<T>& a, const SplitSync& sy, hipStream_t st);

// Full residual recompute over rows [r0, r1) of one orientation, split into
// tasks of <= RESID_CHUNK ratings (one wave each): e = r - own.partner is
// scattered into the other orientation's order (E_other[perm[q]]), each task
// writes its sum of squares, and row_sq[row] folds the row's tasks in order.
constexpr uint32_t RESID_CHUNK = 1024;
struct ResidTask {
    uint32_t row, beg, len, pad;
};
template <typename T>
hipError_t launch_resid(const ResidTask* tasks, uint32_t ntask, const uint32_t* tptr, uint32_t r0, uint32_t r1,
                        const uint32_t* part, const uint32_t* perm, const T* r, const T* own, const T* partner,
                        uint32_t K, uint32_t Kp, T* E_other, double* task_sq, double* row_sq, const double* b_own,
                        const double* b_part, double b0, hipStream_t st);

// Column partials of two tables in one launch, over rows [0, rA) of A and [0, rB)
// of B: out[c][0..K) = sum (x-mu)^2, out[c][K..2K) = sum x, c = chunk of 256 rows
// (outA: (rA+255)/256 chunks, outB: (rB+255)/256).
template <typename T>
hipError_t launch_colstats(const T* tabA, uint32_t rA, const T* muA, double* outA, const T* tabB, uint32_t rB,
                           const T* muB, double* outB, uint32_t K, uint32_t Kp, hipStream_t st);

// Test predictions: pred = clamp(dot(U[u],V[i])) (+ b0 + bu[u] + bv[i] when bu
// is non-null: the biased sampler); sum[t] += pred if collect;
// part[b][0] += (r - sum/div)^2, part[b][1] += (r-pred)^2 per 256-rating block.
template <typename T>
hipError_t launch_test(const uint32_t* tu, const uint32_t* ti, const double* tr, uint64_t t0, uint64_t t1,
                       const T* U, const T* V, uint32_t K, uint32_t Kp, T lo, T hi, int collect, double div,
                       double* sum, double* part, const double* bu, const double* bv, double b0, hipStream_t st);

// Biased sampler (top-level gibbs_sbpmf2.cpp, src/libfm/gibbs_sbpmf22.cpp):
// per-row bias hyperparameters + bias draw + residual shift, one wave per row
// over rows [r0, r1) of one orientation, E in that orientation's order.
struct BiasArgs {
    double alpha;          // noise precision of this sweep
    double d0;             // global-bias delta added to every residual first (user half), else 0
    double ag, bg, sg, mg; // prior of every bias group (reference: 1, 1, 1, 0)
    uint64_t seed;
    uint32_t sweep, tag;   // Philox row stream (TAG_BIAS_U / TAG_BIAS_V) when var3 is null
    int sd_is_var;
};
template <typename T>
hipError_t launch_bias_rows(const uint32_t* ptr, uint32_t r0, uint32_t r1, T* E, double* b, double* mu_b,
                            double* sig_b, const double* var3, const BiasArgs& p, hipStream_t st);
// out2[0] = sum(E), out2[1] = sum(E^2) over E[0..n), fixed order (part: 2*ceil(n/1024) doubles).
template <typename T>
hipError_t launch_esum2(const T* E, uint64_t n, double* part, double* out2, hipStream_t st);

// out[2r] = sum(e), out[2r+1] = sum(e^2) over the ratings of rows [r0, r1) (E in their order)
template <typename T>
hipError_t launch_rowsum2(const uint32_t* ptr, uint32_t r0, uint32_t r1, const T* E, double* out, hipStream_t st);

// E[idx[j]] = recv[j] for j < n (multi-GPU residual exchange, receiving side)
template <typename T>
hipError_t launch_unpack(const T* recv, const uint32_t* idx, uint64_t n, T* E, hipStream_t st);

// Deterministic fixed-order sum of in[n] (contiguous) into one double at out.
// scratch: >= ceil(n/1024) + ceil(n/1024^2) + 2 doubles.
hipError_t launch_sum(const double* in, uint64_t n, double* out, double* scratch, hipStream_t st);
// out[w] = sum_c in[c*width + w], c ascending (width columns, nchunk rows)
hipError_t launch_sum_cols(const double* in, uint32_t nchunk, uint32_t width, double* out, hipStream_t st);
// The same for two arrays of the same width in one launch.
hipError_t launch_sum_cols2(const double* in, uint32_t nchunk, double* out, const double* in2, uint32_t nchunk2,
                            double* out2, uint32_t width, hipStream_t st);

// Philox init: tab[r][k] = sd * z(seed, sweep=0xffffffff, tag, r, k), rows [r0,r1).
// z[row][k] = N(0,1) Philox normal (seed, sweep, tag, row, pair k/2) for rows [r0, r1):
// the per-half variates of throughput mode, the same stream the kernels drew inline.
template <typename T>
hipError_t launch_philox_fill(T* z, uint32_t K, uint32_t r0, uint32_t r1, uint64_t seed, uint32_t sweep, uint32_t tag,
                              hipStream_t st);
// Both tables' normals of one sweep in one launch: launch_philox_fill over users [u0, u1) with
// tagu and over items [v0, v1) with tagv.
template <typename T>
hipError_t launch_philox_fill2(T* zu, uint32_t u0, uint32_t u1, uint32_t tagu, T* zv, uint32_t v0, uint32_t v1,
                               uint32_t tagv, uint32_t K, uint64_t seed, uint32_t sweep, hipStream_t st);
template <typename T>
hipError_t launch_init_philox(T* tab, uint32_t K, uint32_t Kp, uint32_t r0, uint32_t r1, double sd, uint64_t seed,
                              uint32_t tag, hipStream_t st);

}  // namespace sbmf
