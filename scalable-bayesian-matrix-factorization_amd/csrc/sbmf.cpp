// sbmf.cpp -- host side of the MI355X SBPMF sampler: the C ABI of include/sbmf.h.
//
// Per sweep (reference loop body gibbs_sbpmf_final.cpp:309-564):
//   1. residual sum of squares + column statistics of U and V (device,
//      fixed-order reductions)            -> one small D2H
//   2. tau, sigma_u/mu_u, sigma_v/mu_v drawn on the host in fp64 with the
//      reference's expressions (:339-342, :375-414)  -> H2D hyper buffer
//   3. user half-sweep (kernels.hip), [RCCL: broadcast U row blocks]
//   4. item half-sweep,               [RCCL: broadcast V row blocks]
//   5. test prediction + running mean RMSE (:539-563)
// Reference RNG mode pre-generates the sweep's whole variate stream on the
// host (it is data independent, see rng.h) and uploads it; Philox mode draws
// in-kernel.  No CPU compute fallback exists: without a GPU, sbmf_create fails.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "../../include/sbmf.h"
#include "comm.h"
#include "common.h"
#include <rccl/rccl.h>
#include "kernels.h"
#include "rng.h"
#include "fmm.h"
#include "vbo.h"

namespace {
thread_local std::string g_err;
}

struct sbmf_ctx;

namespace sbmf {

[[noreturn]] void comm_fail(const char* what, ncclResult_t r) {
    fail(SBMF_E_COMM, "%s failed: %s", what, rccl_error_string((int)r));
}

// ------------------------------------------------------------------ host layout
// One orientation: users (CSR by user, partner = item) or items (CSC).
static const int NBIN = GK_NUM + 1;  // row bins: Gram-block kinds GK_* (0..4), streaming rows (5)

struct Side {
    uint32_t R = 0;                     // rows
    std::vector<uint32_t> ptr;          // [R+1]
    std::vector<uint32_t> part;         // [N] partner id
    std::vector<uint32_t> perm;         // [N] position in the other orientation
    std::vector<double> r;              // [N] ratings
    uint32_t r0 = 0, r1 = 0;            // owned row range (multi-GPU)
    std::vector<uint64_t> bounds;       // [nranks+1] row ranges of every rank
    // streaming rows (k_gres): set 0 and set 1 (f64 items: rows above 1024 ratings,
    // on 16-wave workgroups) -- see prepare_T
    struct StreamSet {
        std::vector<SplitTask> stasks;  // tasks, in rounds of `sgrid` slots
        std::vector<SplitRow> xrows;    // rows split over several tasks
        uint32_t nxchunk = 0;           // tasks belonging to split rows (slab / staging slots)
        uint32_t sgrid = 0;             // persistent grid of the launch
        uint32_t cmax = 0;              // task capacity (ratings)
        uint32_t tune = 0;              // kernel variant bits of the launch
    };
    // A stage: the rows [r0, r1) of this rank's block, binned for their own launches.
    // One stage per half unless the multi-GPU exchange is pipelined: then the block is
    // cut into nnz-balanced stages and stage s's fresh rows and residuals travel while
    // stage s+1 computes (run_sweeps_T).  Results do not depend on the cut: every row's
    // draws are the same in any launch.
    struct Stage {
        uint32_t r0 = 0, r1 = 0;
        std::vector<uint32_t> bin_rows[NBIN];  // kinds: GK_* (0..4), KIND_STREAM (5)
        StreamSet ss[2];
        std::vector<std::array<uint32_t, 3>> gsub[GK_NUM];  // multi-wave bins: (waves, offset, count) sub-ranges
        DBuf d_bins[NBIN], d_stasks[2], d_xrows[2];
        // multi-GPU residual exchange of this stage: [peer] segments of the send / receive areas
        std::vector<size_t> soff, scnt, roff, rcnt;
        size_t rbeg = 0, rend = 0;  // this stage's receive elements [rbeg, rend)
    };
    std::vector<std::unique_ptr<Stage>> stg;
    std::vector<std::vector<uint64_t>> sbounds;  // [rank][stage + 1]: every rank's stage cuts
    std::vector<ResidTask> rtasks;   // residual recompute: own rows in chunks of <= RESID_CHUNK
    std::vector<uint32_t> rtptr;     // [r1-r0+1] first task of each own row
    // multi-GPU residual exchange (see build_exchange): where this rank's rows
    // scatter their residuals (the other orientation's position, or a send slot
    // past its end), and where the residuals other ranks send land
    std::vector<uint32_t> perm2, unpack;
    size_t nsend = 0, nrecv = 0;
};

// Multi-GPU residuals.  A half-sweep on rank p updates the residuals of its
// own rows' ratings and scatters them into the other orientation's order
// (E_other[perm[idx]]); the next half on rank q reads the residuals of q's
// rows, which every rank contributed to.  So each half ends with a
// point-to-point exchange: rank p's kernels write the residuals bound for
// rank q into a send area past the end of E_other (perm2 = N + slot), in
// rating order, and rank q unpacks what arrives from p into its positions
// (unpack, the same order).  Both lists follow from the rating structure,
// which every rank holds, so no index travels.  About N / P residuals per
// rank per half cross xGMI -- instead of recomputing every residual from
// r - own.partner, which re-reads every partner row.
static void build_exchange(Side& s, const Side& other, int nranks, int rank) {
    const uint64_t N = s.perm.size();
    const size_t P = s.stg.size();
    std::vector<uint64_t> obase(nranks + 1);
    for (int k = 0; k <= nranks; ++k) obase[k] = other.ptr[other.bounds[k]];
    auto owner = [&](uint32_t pos) {
        return (int)(std::upper_bound(obase.begin(), obase.end(), (uint64_t)pos) - obase.begin()) - 1;
    };
    // send area: [stage][peer] segments, each in rating order
    size_t off = 0;
    for (size_t p = 0; p < P; ++p) {
        Side::Stage& g = *s.stg[p];
        g.scnt.assign(nranks, 0);
        for (uint64_t idx = s.ptr[g.r0]; idx < s.ptr[g.r1]; ++idx) {
            const int q = owner(s.perm[idx]);
            if (q != rank) g.scnt[q]++;
        }
        g.soff.assign(nranks, 0);
        for (int k = 0; k < nranks; ++k) {
            g.soff[k] = off;
            off += g.scnt[k];
        }
    }
    s.nsend = off;
    s.perm2.assign(s.perm.begin(), s.perm.end());
    for (size_t p = 0; p < P; ++p) {
        Side::Stage& g = *s.stg[p];
        std::vector<size_t> fill(g.soff);
        for (uint64_t idx = s.ptr[g.r0]; idx < s.ptr[g.r1]; ++idx) {
            const int q = owner(s.perm[idx]);
            if (q != rank) s.perm2[idx] = (uint32_t)(N + fill[q]++);
        }
    }
    // receive area: what rank k's stage p sends here, in k's rating order, [stage][peer]
    s.unpack.clear();
    for (size_t p = 0; p < P; ++p) {
        Side::Stage& g = *s.stg[p];
        g.roff.assign(nranks, 0);
        g.rcnt.assign(nranks, 0);
        g.rbeg = s.unpack.size();
        for (int k = 0; k < nranks; ++k) {
            g.roff[k] = s.unpack.size();
            if (k == rank) continue;
            for (uint64_t idx = s.ptr[s.sbounds[k][p]]; idx < s.ptr[s.sbounds[k][p + 1]]; ++idx)
                if (owner(s.perm[idx]) == rank) s.unpack.push_back(s.perm[idx]);
            g.rcnt[k] = s.unpack.size() - g.roff[k];
        }
        g.rend = s.unpack.size();
    }
    s.nrecv = s.unpack.size();
    if (N + s.nsend >= 0xffffffffull) fail(SBMF_E_ARG, "too many ratings for the 32-bit residual exchange");
}

static void build_side(uint64_t N, const uint32_t* key, const uint32_t* other, const double* rat, uint32_t R,
                       Side& s, std::vector<uint32_t>& pos_of_case) {
    s.R = R;
    s.ptr.assign((size_t)R + 1, 0);
    for (uint64_t c = 0; c < N; ++c) s.ptr[key[c] + 1]++;
    for (uint32_t i = 0; i < R; ++i) s.ptr[i + 1] += s.ptr[i];
    std::vector<uint32_t> fill(s.ptr.begin(), s.ptr.end() - 1);
    s.part.resize(N);
    s.r.resize(N);
    pos_of_case.resize(N);
    for (uint64_t c = 0; c < N; ++c) {  // file order within a row (gibbs_sbpmf_final.cpp:204-209)
        const uint32_t p = fill[key[c]]++;
        s.part[p] = other[c];
        s.r[p] = rat[c];
        pos_of_case[c] = p;
    }
}

// nnz-balanced contiguous partition, boundaries aligned to 256 rows.
static void partition_bounds(const uint32_t* ptr, uint32_t R, int nranks, uint64_t* bounds) {
    bounds[0] = 0;
    for (int k = 1; k <= nranks; ++k) {
        uint32_t row = R;
        if (k < nranks) {
            const double target = (double)ptr[R] * k / nranks;
            row = (uint32_t)(std::lower_bound(ptr, ptr + R + 1, (uint32_t)std::llround(target)) - ptr);
            row = std::min((row + 128) / 256 * 256, R);
        }
        bounds[k] = std::max<uint64_t>(bounds[k - 1], row);
    }
}
static void partition(Side& s, int nranks, int rank, uint32_t nstages) {
    s.bounds.assign(nranks + 1, 0);
    partition_bounds(s.ptr.data(), (uint32_t)s.ptr.size() - 1, nranks, s.bounds.data());
    s.r0 = (uint32_t)s.bounds[rank];
    s.r1 = (uint32_t)s.bounds[rank + 1];
    // every rank's block cut into nstages nnz-balanced stages (known to every rank:
    // the exchange of stage p involves every rank's stage p)
    s.sbounds.assign(nranks, std::vector<uint64_t>(nstages + 1, 0));
    for (int k = 0; k < nranks; ++k) {
        const uint64_t b0 = s.bounds[k], b1 = s.bounds[k + 1];
        std::vector<uint64_t>& sb = s.sbounds[k];
        sb[0] = b0;
        for (uint32_t p = 1; p <= nstages; ++p) {
            uint64_t row = b1;
            if (p < nstages) {
                const double target = s.ptr[b0] + (double)(s.ptr[b1] - s.ptr[b0]) * p / nstages;
                row = (uint64_t)(std::lower_bound(s.ptr.begin() + b0, s.ptr.begin() + b1 + 1,
                                                  (uint32_t)std::llround(target)) - s.ptr.begin());
                row = std::min<uint64_t>(std::max<uint64_t>(row, b0), b1);
            }
            sb[p] = std::max<uint64_t>(sb[p - 1], row);
        }
    }
    s.stg.clear();
    for (uint32_t p = 0; p < nstages; ++p) {
        s.stg.emplace_back(new Side::Stage);
        s.stg.back()->r0 = (uint32_t)s.sbounds[rank][p];
        s.stg.back()->r1 = (uint32_t)s.sbounds[rank][p + 1];
    }
}

static const int KIND_STREAM = GK_NUM;  // 5: streaming kernel (row bin: every streaming row)

static void build_bins(const Side& s, Side::Stage& g, uint32_t stream_thr, bool f64, bool wide) {
    for (auto& b : g.bin_rows) b.clear();
    std::vector<uint32_t> order(g.r1 - g.r0);
    std::iota(order.begin(), order.end(), g.r0);
    auto deg = [&](uint32_t r) { return s.ptr[r + 1] - s.ptr[r]; };
    // heaviest first: blocks are dispatched roughly in index order, so the
    // longest rows start earliest (LPT)
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return deg(a) > deg(b); });
    for (uint32_t r : order) {
        const uint32_t d = deg(r);
        if (d > stream_thr) {
            g.bin_rows[KIND_STREAM].push_back(r);
            continue;
        }
        int kind = GK_W4;
        while (d > gk_maxdeg(kind, f64, wide)) ++kind;
        g.bin_rows[kind].push_back(r);
    }
}

Audit& audit() {
    static Audit a;
    return a;
}

}  // namespace sbmf

using namespace sbmf;

struct sbmf_ctx {
    sbmf_ctx() { sbmf::audit().contexts++; }
    sbmf_config cfg{};
    std::string err;
    // sbmf_test_rccl_selftest ran extra item halves on this chain (it is no longer
    // the sampler's): sweeps are refused.  dead: the self-test timed out with RCCL
    // work still queued; sbmf_destroy then leaks the context instead of waiting.
    bool spent = false, dead = false;
    // host data
    std::vector<uint32_t> tu, ti, su, si;
    std::vector<double> tr, sr;
    uint32_t I = 0, J = 0, I_req = 0, J_req = 0;
    bool prepared = false;
    // derived settings
    double init_sd = 1.0, lo = 1.0, hi = 5.0;
    int sd_is_var = 1;
    uint32_t K = 0, Kp = 0;
    // layout
    Side users, items;
    uint64_t t0 = 0, t1 = 0;  // owned test range
    std::vector<uint64_t> tbounds, tbblocks;  // every rank's test range (ratings, 256-blocks)
    std::vector<uint64_t> tperm;  // device test order (user order) -> file order
    // hyper state (fp64 host copy)
    std::vector<double> sig_u, mu_u, sig_v, mu_v;
    double tau = 1.0;
    // biased sampler (quirks BIAS2 / BIAS22): global bias + Normal-Gamma state
    bool bias = false;
    double b0 = 0.0, mu_b0 = 0.0, sig_b0 = 0.0;
    // reference mode: host shadow (b, mu_b, sigma_b) of the rows without train
    // ratings, whose bias walk depends only on its own variates (see fill_bias_variates)
    std::vector<uint32_t> empty_u, empty_v;
    std::vector<std::array<double, 3>> shadow_u, shadow_v;
    uint32_t sweep = 0, collected = 0;
    // rng
    GlibcRand grand{1};
    // multi-GPU
    int nranks = 1, rank = 0;
    Comm own_comm;            // this context's communicator (sbmf_comm_init) ...
    Comm* comm = &own_comm;   // ... or a process-wide one it borrows (sbmf_comm_attach)
    // device
    hipStream_t st = nullptr;
    hipEvent_t ev[10] = {};
    std::vector<hipEvent_t> kevs;  // [stage][side][kind][begin, end] launch timing
    hipEvent_t& kev(uint32_t stage, int side, int kind, int e) {
        return kevs[(((size_t)stage * 2 + side) * SBMF_NKIND + kind) * 2 + e];
    }
    // [stage][side][kind]: the kind launched just before this one on the same stream, whose
    // end event is this kind's start (no begin event recorded), or -1.  Two timing events
    // back to back on a stream cost ~12 us of idle device between the launches (r04f trace).
    std::vector<int8_t> kprev;
    int8_t& kpv(uint32_t stage, int side, int kind) { return kprev[((size_t)stage * 2 + side) * SBMF_NKIND + kind]; }
    // [stage][side][kind]: the begin event a kind's time is read from when kprev is -1 -- its own
    // kev(.., 0), or an event its half's caller had just recorded on the compute stream (the
    // sweep start, the user half's end), which then also forks the side streams
    std::vector<hipEvent_t> kbegin;
    hipEvent_t& kbg(uint32_t stage, int side, int kind) { return kbegin[((size_t)stage * 2 + side) * SBMF_NKIND + kind]; }
    uint32_t nstages = 1;          // stages per half (see Side::Stage); > 1 only with several ranks
    hipStream_t stc = nullptr;     // multi-GPU: the exchange of stage p runs here while stage p+1 computes
    std::vector<hipEvent_t> sev;   // [side][stage]: stage computed (compute stream)
    // sbmf_test_virtual_rank (timing only): one rank of an nranks-rank run on this GPU,
    // every exchange skipped; tsev [side][stage + 1] times its stages on the compute stream
    bool virt = false;
    std::vector<hipEvent_t> tsev;
    hipEvent_t cev[2] = {};        // [side]: the half's exchange done (comm stream)
    hipStream_t sto = nullptr;     // a half's Gram-block launches, beside its streaming launch
    hipStream_t sto2 = nullptr;    // tune bit 25: half of them on a second side stream
    hipEvent_t oev[4] = {};        // [fork, join] of those launches, [2]: stream set 0 done, [3]: sto2 join
    DBuf d_uptr, d_upart, d_uperm, d_ur, d_vptr, d_vpart, d_vperm, d_vr;
    DBuf d_U, d_V, d_Eu, d_Ev, d_zU, d_zV, d_hyper;
    DBuf d_rowsq_u, d_rowtr_u, d_rowsq_v, d_rowtr_v;
    DBuf d_colpart, d_res, d_scratch;
    size_t scratch_half = 0;  // doubles: d_scratch + scratch_half is the evaluation's

    bool kprof = false; // SBMF_KPROF=1: streaming-kernel phase cycles printed per sweep
    int kprof_set = 0;  // SBMF_KPROF_SET: which streaming launch of a half is stamped (0: the 8-wave one)
    DBuf d_kprof;
    DBuf d_rtasks, d_rtptr, d_rtsq;  // residual recompute (item side)
    DBuf d_xslabs, d_xcnt, d_xchunk_sq, d_xchunk_tr, d_xnewown;
    bool time_kinds = true;   // this sweep records every launch kind's events (else the streaming kind's only)
    size_t xset_nx = 1, xset_nr = 1;  // set 0's split chunks / rows: set 1's areas follow them
    DBuf d_tu, d_ti, d_tr, d_tsum, d_tpart;
    DBuf d_uperm2, d_vperm2, d_uunpack, d_vunpack, d_xrecv;  // multi-GPU residual exchange
    DBuf d_bu, d_bv, d_mbu, d_mbv, d_sbu, d_sbv;  // biases b_i / b_j and their per-row (mu, sigma)
    DBuf d_var3u, d_var3v, d_epart;              // reference-mode per-row bias variates; sum(E) partials
    std::vector<double> h_res;
    double* h_pre = nullptr;     // pinned: the prologue's sums (residual, column statistics)
    // pinned: the sweep's results (8 doubles), the split-row timeout flag, and the staged
    // hyperparameter upload [sig_u | mu_u | sig_v | mu_v] (4 Kp of T)
    void* h_io = nullptr;
    double* h_out() { return static_cast<double*>(h_io); }
    void* h_hyper() { return static_cast<char*>(h_io) + 128; }
    hipEvent_t hev = nullptr;  // the last upload from h_hyper done (the area is rewritten after it)
    // throughput mode: the next sweep's hyperparameters, drawn at the end of the
    // previous sweep while its test evaluation runs (run_sweeps_T)
    struct PreDraw {
        bool valid = false;
        bool staged = false;  // uploaded to d_hyper, and the sweep's normals filled, ahead
        uint32_t sweep = 0;
        double tau = 0, b0 = 0, mu_b0 = 0, sig_b0 = 0, d0 = 0;
        std::vector<double> sig_u, mu_u, sig_v, mu_v;
    } pre;
    // d_hyper holds the drawn-ahead values (pre), not the current ones: a sweep that does not
    // use them (pre dropped by sbmf_set_factors) restores the current ones before its
    // prologue, whose column statistics read the current mu from d_hyper
    bool hyper_ahead = false;
    double* h_pinned = nullptr;  // pinned staging for z streams
    size_t h_pinned_bytes = 0, h_pre_bytes = 0, h_io_bytes = 0;
    sbmf_timing timing{};
    VBLearner* vb = nullptr;  // -method vb (vbo.cpp)
    FMLearner* fm = nullptr;  // -method mcmc --order libfm / als (fmm.cpp)
    ~sbmf_ctx();
};

namespace sbmf {

// result slots in d_res
// d_res slots; RES_TIMEOUT holds k_gres's split-row timeout flag (a uint32, sticky), so the
// sweep's one result copy carries it
enum { RES_ESQ = 0, RES_TRSQ = 1, RES_TEST_AVG = 2, RES_TEST_THIS = 3, RES_ES = 4, RES_ESQ2 = 5, RES_TIMEOUT = 7, RES_COL = 8 };

static size_t tsize(const sbmf_ctx* c) { return c->cfg.precision == SBMF_F32 ? 4 : 8; }

// running-mean divisor: collected sweeps (average 1, or quirks none by default) or sweep + 1
static bool avg_collected(const sbmf_config& cf) {
    return cf.average == 1 || (cf.average == 0 && cf.quirks == SBMF_QUIRKS_NONE);
}

template <typename T>
static std::vector<T> to_T(const std::vector<double>& v) {
    return std::vector<T>(v.begin(), v.end());
}

// table [R][Kp] (T) from row-major doubles [R][K]
template <typename T>
static void upload_table(sbmf_ctx* c, DBuf& d, const double* src, uint32_t R) {
    std::vector<T> h((size_t)R * c->Kp, T(0));
    for (uint32_t r = 0; r < R; ++r)
        for (uint32_t k = 0; k < c->K; ++k) h[(size_t)r * c->Kp + k] = (T)src[(size_t)r * c->K + k];
    HIPCHK(hipMemcpy(d.p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
}
template <typename T>
static void download_table(sbmf_ctx* c, const DBuf& d, double* dst, uint32_t R) {
    std::vector<T> h((size_t)R * c->Kp);
    HIPCHK(hipMemcpy(h.data(), d.p, h.size() * sizeof(T), hipMemcpyDeviceToHost));
    for (uint32_t r = 0; r < R; ++r)
        for (uint32_t k = 0; k < c->K; ++k) dst[(size_t)r * c->K + k] = (double)h[(size_t)r * c->Kp + k];
}

static void ensure_pinned(sbmf_ctx* c, size_t bytes) {
    if (c->h_pinned_bytes >= bytes) return;
    pinned_free(c->h_pinned, c->h_pinned_bytes);
    c->h_pinned_bytes = 0;
    pinned_alloc((void**)&c->h_pinned, bytes);
    c->h_pinned_bytes = bytes;
}

static void fill_kernel_bytes(sbmf_ctx* c);
static void build_stream_tasks(const Side& s, Side::StreamSet& S, const std::vector<uint32_t>& rows, uint32_t gres,
                               uint32_t nblk);

// ------------------------------------------------------------------ prepare
template <typename T>
static void prepare_T(sbmf_ctx* c) {
    const sbmf_config& cf = c->cfg;
    const uint64_t N = c->tu.size();
    // dims: max id + 1 over train and test (gibbs_sbpmf_final.cpp:146-148)
    uint32_t umax = 0, imax = 0;
    for (uint64_t x = 0; x < N; ++x) {
        umax = std::max(umax, c->tu[x]);
        imax = std::max(imax, c->ti[x]);
    }
    for (size_t x = 0; x < c->su.size(); ++x) {
        umax = std::max(umax, c->su[x]);
        imax = std::max(imax, c->si[x]);
    }
    c->I = std::max(c->I_req, (N || !c->su.empty()) ? umax + 1 : 0);
    c->J = std::max(c->J_req, (N || !c->si.empty()) ? imax + 1 : 0);
    if (c->I == 0 || c->J == 0) fail(SBMF_E_STATE, "no ratings: call sbmf_set_train first");
    if (N >= 0xffffffffull) fail(SBMF_E_ARG, "more than 2^32-1 ratings are not supported");
    c->K = cf.num_factor;
    c->Kp = (c->K + 15) / 16 * 16;  // k-blocks of 16 start on 128-byte (f64) / 64-byte (f32) boundaries
    // the streaming kernel keeps partner-row element offsets (row * Kp) in 32 bits
    if ((uint64_t)(std::max(c->I, c->J) + 2) * c->Kp >= 0xffffffffull)
        fail(SBMF_E_ARG, "factor tables of %u x %u rows at K=%u exceed 2^32 elements", c->I, c->J, c->K);

    std::vector<uint32_t> pos_u, pos_v;
    build_side(N, c->tu.data(), c->ti.data(), c->tr.data(), c->I, c->users, pos_u);
    build_side(N, c->ti.data(), c->tu.data(), c->tr.data(), c->J, c->items, pos_v);
    c->users.perm.resize(N);
    c->items.perm.resize(N);
    for (uint64_t x = 0; x < N; ++x) {
        c->users.perm[pos_u[x]] = pos_v[x];
        c->items.perm[pos_v[x]] = pos_u[x];
    }
    // stages per half: the multi-GPU exchange of a stage overlaps the next stage's
    // compute; one rank needs no exchange (SBMF_STAGES overrides, for tests).  Two: each
    // extra stage costs its launches' fixed latency -- per-rank compute of the 8-way split
    // at 1 / 2 / 4 stages is 1.25 / 1.50 / 1.99 ms at K=100 and 2.01 / 2.31 / 2.90 ms at
    // K=200 (virtual ranks, r05s6) -- against about half the exchange hidden per doubling
    // (0.6 / 0.9 ms per sweep at an assumed 330 GB/s all-gather): two stages are the best
    // or tied over 150-600 GB/s at both K
    c->nstages = c->nranks > 1 ? 2u : 1u;
    if (const char* e = std::getenv("SBMF_STAGES")) c->nstages = std::max(1, std::min(16, std::atoi(e)));
    partition(c->users, c->nranks, c->rank, c->nstages);
    partition(c->items, c->nranks, c->rank, c->nstages);
    if (c->nranks > 1) {
        build_exchange(c->users, c->items, c->nranks, c->rank);  // user half -> item order
        build_exchange(c->items, c->users, c->nranks, c->rank);  // item half -> user order
    }
    // Gram-block kernels for rows <= the stream threshold, the streaming kernel above it
    const bool f64 = sizeof(T) == 8;
    const bool wide = !(cf.tune & 8u);  // f64 rows <= 64 ratings on one wave (default)
    const uint32_t gkmax = gk_maxdeg(GK_NUM - 1, f64, wide);
    const uint32_t sthr = std::min<uint32_t>(cf.stream_threshold ? cf.stream_threshold : gkmax, gkmax);
    for (Side* sd : {&c->users, &c->items})
        for (auto& g : sd->stg) build_bins(*sd, *g, sthr, f64, wide);
    // multi-wave Gram-block bins: ceil(deg / ratings-per-wave) waves per row,
    // contiguous sub-ranges since each bin is degree-descending
    for (Side* sd : {&c->users, &c->items})
        for (auto& gp : sd->stg)
        for (int k = GK_B2; k < GK_NUM; ++k) {
            Side::Stage& g = *gp;
            g.gsub[k].clear();
            const std::vector<uint32_t>& rows = g.bin_rows[k];
            const uint32_t per_wave = f64 ? 32 : 64;
            for (uint32_t i = 0; i < rows.size();) {
                const uint32_t d = sd->ptr[rows[i] + 1] - sd->ptr[rows[i]];
                const uint32_t nw = std::max(2u, (d + per_wave - 1) / per_wave);
                uint32_t j = i;
                while (j < rows.size() &&
                       std::max(2u, (sd->ptr[rows[j] + 1] - sd->ptr[rows[j]] + per_wave - 1) / per_wave) == nw)
                    ++j;
                // f64 rows of 5-8 eight-vector waves run as (nw + 1) / 2 sixteen-vector waves
                // (launch_gblock_nw): groups that launch the same kernel shape are one launch
                // (nw 5+6 and 7+8; the merged group carries its larger nw)
                auto shape = [&](uint32_t w) { return f64 && w >= 5 ? 100 + (w + 1) / 2 : w; };
                if (!g.gsub[k].empty() && shape(g.gsub[k].back()[0]) == shape(nw)) {
                    auto& last = g.gsub[k].back();  // degree-descending: the earlier group has the larger nw
                    last[2] += j - i;
                } else {
                    g.gsub[k].push_back({nw, i, j - i});
                }
                i = j;
            }
        }
    const uint32_t nblk = (c->K + 15) / 16;
    {
        int dev_cus = 0;
        HIPCHK(hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, cf.device));
        for (Side* sd : {&c->users, &c->items}) {
            // f64 item rows above 1024 ratings (75 % of the item ratings sit in rows
            // split over several tasks) on 16-wave k_gres workgroups, 2048-rating
            // tasks: half the chunks per split row, a quarter of the all-read
            // exchange; shorter item rows and every user row on 8-wave workgroups
            // (two independent tasks per CU).  Measured item launch 4.04 ms (all
            // 8-wave) / 3.88 (all 16-wave) / 3.70 (this split); the user side is
            // slower with any 16-wave share (1.59 / 2.23 / 1.66 ms).  Tune bit 27,
            // or an explicit workgroup-shape or hybrid bit, keeps 8-wave items.
            const bool item16 = sd == &c->items && sizeof(T) == 8 && !(cf.tune & (128u | 0x20000u | 0x8000000u));
            // f64 user rows on 4-wave k_gres workgroups (512-rating tasks, four workgroups per
            // CU): measured user streaming 1.49 -> 1.40 ms against 8-wave (r03s10); tune bit 23,
            // or an explicit workgroup-shape bit, keeps them on 8-wave workgroups
            const bool user4 = sd == &c->users && sizeof(T) == 8 && !(cf.tune & (128u | 0x20000u | 0x800000u));
            // f64 user rows above 512 ratings as a second set on 8-wave workgroups (1024-rating tasks:
            // rows up to 1024 whole, longer ones in half as many chunks) beside the 4-wave set of the
            // rest: the r05s26 phase profile had the 4-wave set's split-row chunks 63 % in the hand-off
            // phase; user half 2.85-2.89 -> 2.80-2.81 ms (r05s27, 3 rounds).  Tune bit 13 keeps one
            // 4-wave set; bit 14 (experiment) puts the long rows on 16-wave workgroups instead (slower)
            const bool user2 = user4 && (!(cf.tune & 0x2000u) || (cf.tune & 0x4000u));
            const uint32_t stunes[2] = {user4 ? cf.tune | 128u : cf.tune,
                                        user2 && !(cf.tune & 0x4000u) ? cf.tune : cf.tune | 0x20000u};
            // (round 4 measured a second user set neutral to slower -- rows above 1024 / 2048 ratings
            // on 16-wave workgroups, above 512 / 1024 on 8-wave ones: r04s9, r04s15 -- with the user
            // rows of 9..256 ratings still on the Gram-block kinds)
            for (auto& gp : sd->stg) {
            std::vector<uint32_t> rows[2];
            for (uint32_t r : gp->bin_rows[KIND_STREAM]) {  // degree-descending
                const uint32_t d = sd->ptr[r + 1] - sd->ptr[r];
                rows[(item16 && d > 1024u) || (user2 && d > 512u) ? 1 : 0].push_back(r);
            }
            for (int k = 0; k < 2; ++k) {
                Side::StreamSet& S = gp->ss[k];
                S.tune = stunes[k];
                // task capacity: the kernel's on-chip maximum, or smaller if split_chunk asks
                S.cmax = gstream_cmax<T>(S.tune);
                if (cf.split_chunk) S.cmax = std::min(S.cmax, std::max(cf.split_chunk, 1u));
                // (fewer persistent workgroups per CU, leaving CU slots to the Gram-block launches
                // beside the streaming one from its start: user 3 / 2 per CU +0.03 / +0.13 ms, item
                // 8-wave set 1 per CU +0.2 ms per sweep, r05s8)
                const int per_cu =
                    std::max(1, std::min(gstream_wg_target(S.tune), gstream_blocks_per_cu<T>(S.cmax, S.tune)));
                // (per-XCD task queues, each split row on one XCD: item stage 3.59 -> 3.77 ms standalone,
                // r06s3; removed, profiles/r06/ab/r06s3_xcd_queues.patch)
                build_stream_tasks(*sd, S, rows[k], (uint32_t)(dev_cus * per_cu), nblk);
            }
            }
        }
    }
    {  // test split in 256-aligned blocks
        const uint64_t T_ = c->su.size(), nb = (T_ + 255) / 256;
        c->tbounds.assign(c->nranks + 1, 0);
        c->tbblocks.assign(c->nranks + 1, 0);
        for (int k = 0; k <= c->nranks; ++k) {
            c->tbblocks[k] = nb * k / c->nranks;
            c->tbounds[k] = std::min<uint64_t>(T_, c->tbblocks[k] * 256);
        }
        c->t0 = c->tbounds[c->rank];
        c->t1 = c->tbounds[c->rank + 1];
    }

    hipStream_t st = c->st;
    upload(c->d_uptr, c->users.ptr, st);
    upload(c->d_upart, c->users.part, st);
    upload(c->d_uperm, c->users.perm, st);
    upload(c->d_ur, to_T<T>(c->users.r), st);
    upload(c->d_vptr, c->items.ptr, st);
    upload(c->d_vpart, c->items.part, st);
    upload(c->d_vperm, c->items.perm, st);
    upload(c->d_vr, to_T<T>(c->items.r), st);
    for (Side* sd : {&c->users, &c->items})
        for (auto& g : sd->stg)
            for (int k = 0; k < NBIN; ++k) upload(g->d_bins[k], g->bin_rows[k], st);
    {  // residual recompute tasks over the own item rows
        Side& s = c->items;
        s.rtasks.clear();
        s.rtptr.assign(1, 0);
        for (uint32_t r = s.r0; r < s.r1; ++r) {
            for (uint32_t b = s.ptr[r]; b < s.ptr[r + 1]; b += RESID_CHUNK)
                s.rtasks.push_back(ResidTask{r, b, std::min<uint32_t>(RESID_CHUNK, s.ptr[r + 1] - b), 0});
            s.rtptr.push_back((uint32_t)s.rtasks.size());
        }
        upload(c->d_rtasks, s.rtasks, st);
        upload(c->d_rtptr, s.rtptr, st);
        c->d_rtsq.alloc(std::max<size_t>(s.rtasks.size(), 1) * sizeof(double));
    }
    // split-row slots of stream set k: the largest over the stages and sides (set 0 and
    // set 1 of a half may run at the same time, so each set has an area of its own)
    size_t nxk[2] = {0, 0}, nrk[2] = {0, 0};
    for (Side* sd : {&c->users, &c->items})
        for (auto& g : sd->stg)
            for (int k = 0; k < 2; ++k) {
                const Side::StreamSet& S = g->ss[k];
                upload(g->d_stasks[k], S.stasks, st);
                upload(g->d_xrows[k], S.xrows, st);
                nxk[k] = std::max<size_t>(nxk[k], S.nxchunk);
                nrk[k] = std::max<size_t>(nrk[k], S.xrows.size());
            }
    c->xset_nx = std::max<size_t>(nxk[0], 1);
    c->xset_nr = std::max<size_t>(nrk[0], 1);
    {
        const size_t nx = c->xset_nx + std::max<size_t>(nxk[1], 1), nr = c->xset_nr + std::max<size_t>(nrk[1], 1);
        c->d_xslabs.alloc(nx * nblk * (16 * 16 + 16) * sizeof(double));
        // + each set's task-queue head.  Zeroed once here: every streaming launch leaves its set's
        // area zero again (k_split_finish clears it after k_gres)
        c->d_xcnt.alloc((nr * nblk + 2 + 3) / 4 * 4 * sizeof(uint32_t));
        HIPCHK(hipMemsetAsync(c->d_xcnt.p, 0, c->d_xcnt.bytes, st));
        c->d_xchunk_sq.alloc(nx * sizeof(double));
        c->d_xchunk_tr.alloc(nx * sizeof(double));
        HIPCHK(hipMemsetAsync(c->d_xchunk_tr.p, 0, c->d_xchunk_tr.bytes, st));
        c->d_xnewown.alloc(nx * c->Kp * sizeof(T));
    }
    // factor tables [rows + 2][Kp]: row `rows` stays zero (the sentinel partner of
    // padded rating slots), row `rows + 1` is slack for the next-block prefetch
    // past the last column block; padding columns K..Kp-1 stay zero.
    c->d_U.alloc((size_t)(c->I + 2) * c->Kp * sizeof(T));
    c->d_V.alloc((size_t)(c->J + 2) * c->Kp * sizeof(T));
    HIPCHK(hipMemsetAsync(c->d_U.p, 0, c->d_U.bytes, st));
    HIPCHK(hipMemsetAsync(c->d_V.p, 0, c->d_V.bytes, st));
    // E_v: the user half's scatter target (+ its send area), E_u: the item half's
    c->d_Eu.alloc(std::max<uint64_t>(N + c->items.nsend, 1) * sizeof(T));
    c->d_Ev.alloc(std::max<uint64_t>(N + c->users.nsend, 1) * sizeof(T));
    if (c->nranks > 1) {
        upload(c->d_uperm2, c->users.perm2, st);
        upload(c->d_vperm2, c->items.perm2, st);
        upload(c->d_uunpack, c->users.unpack, st);
        upload(c->d_vunpack, c->items.unpack, st);
        c->d_xrecv.alloc(std::max<size_t>(std::max(c->users.nrecv, c->items.nrecv), 1) * sizeof(T));
        HIPCHK(hipMemsetAsync(c->d_xrecv.p, 0, c->d_xrecv.bytes, st));  // read as 0 by a virtual rank
    }
    HIPCHK(hipMemsetAsync(c->d_Eu.p, 0, c->d_Eu.bytes, st));
    HIPCHK(hipMemsetAsync(c->d_Ev.p, 0, c->d_Ev.bytes, st));
    c->d_rowsq_u.alloc((size_t)c->I * sizeof(double));
    c->d_rowtr_u.alloc((size_t)c->I * sizeof(double));
    c->d_rowsq_v.alloc((size_t)c->J * sizeof(double));
    c->d_rowtr_v.alloc((size_t)c->J * sizeof(double));
    HIPCHK(hipMemsetAsync(c->d_rowsq_v.p, 0, c->d_rowsq_v.bytes, st));
    HIPCHK(hipMemsetAsync(c->d_rowtr_v.p, 0, c->d_rowtr_v.bytes, st));
    // [sig_u | mu_u | sig_v | mu_v], each Kp long and zero padded, + 16 slack for prefetch
    c->d_hyper.alloc((4 * (size_t)c->Kp + 16) * sizeof(T));
    HIPCHK(hipMemsetAsync(c->d_hyper.p, 0, c->d_hyper.bytes, st));
    const uint32_t nchunk = (c->I + 255) / 256 + (c->J + 255) / 256;  // both tables' 256-row chunks
    c->d_colpart.alloc((size_t)nchunk * 2 * c->K * sizeof(double));
    c->h_res.assign(RES_COL + 4 * (size_t)c->K, 0.0);
    c->d_res.alloc(c->h_res.size() * sizeof(double));
    HIPCHK(hipMemsetAsync(c->d_res.p, 0, c->d_res.bytes, st));
    pinned_free(c->h_pre, c->h_pre_bytes);
    c->h_pre_bytes = c->h_res.size() * sizeof(double);
    pinned_alloc((void**)&c->h_pre, c->h_pre_bytes);
    pinned_free(c->h_io, c->h_io_bytes);
    c->h_io_bytes = 128 + 4 * (size_t)c->Kp * sizeof(T);
    pinned_alloc(&c->h_io, c->h_io_bytes);
    c->pre.valid = false;
    c->hyper_ahead = false;
    const uint64_t big = std::max<uint64_t>({(uint64_t)c->I, (uint64_t)c->J, c->su.size() / 128 + 2});
    // two halves: the prologue's sums and the evaluation's, which run side by side (one rank)
    c->d_scratch.alloc((big / 1024 + 16) * 4 * sizeof(double));
    c->scratch_half = (big / 1024 + 16) * 2;
    // test set, on the device in user order (a counting sort, stable: file order within a
    // user), so the evaluation's consecutive ratings share their user's row in cache; the
    // file order comes back through tperm in sbmf_predict.  The RMSE partial sums run in
    // this order.
    const uint64_t T_ = c->su.size();
    {
        std::vector<uint64_t> start((size_t)c->I + 1, 0);
        for (uint64_t x = 0; x < T_; ++x) ++start[c->su[x] + 1];
        for (uint32_t u = 0; u < c->I; ++u) start[u + 1] += start[u];
        c->tperm.resize(T_);
        std::vector<uint32_t> su2(T_), si2(T_);
        std::vector<double> sr2(T_);
        for (uint64_t x = 0; x < T_; ++x) {
            const uint64_t j = start[c->su[x]]++;
            c->tperm[j] = x;
            su2[j] = c->su[x];
            si2[j] = c->si[x];
            sr2[j] = c->sr[x];
        }
        upload(c->d_tu, su2, st);
        upload(c->d_ti, si2, st);
        upload(c->d_tr, sr2, st);
        HIPCHK(hipStreamSynchronize(st));  // the sorted copies are locals
    }
    c->d_tsum.alloc(std::max<uint64_t>(T_, 1) * sizeof(double));
    HIPCHK(hipMemsetAsync(c->d_tsum.p, 0, c->d_tsum.bytes, st));
    c->d_tpart.alloc(((T_ + 255) / 256 + 1) * 2 * sizeof(double));
    HIPCHK(hipMemsetAsync(c->d_tpart.p, 0, c->d_tpart.bytes, st));
    {  // per-half normals: host reference stream, or launch_philox_fill in throughput mode
        c->d_zU.alloc((size_t)c->I * c->K * sizeof(T));
        c->d_zV.alloc((size_t)c->J * c->K * sizeof(T));
    }
    {  // biased sampler state: b_i, b_j, their (mu, sigma) start at 0 (gibbs_sbpmf2.cpp:276-318)
        const size_t nb = c->bias ? 1 : 0;
        for (DBuf* d : {&c->d_bu, &c->d_mbu, &c->d_sbu}) {
            d->alloc(nb * c->I * sizeof(double));
            HIPCHK(hipMemsetAsync(d->p, 0, d->bytes, st));
        }
        for (DBuf* d : {&c->d_bv, &c->d_mbv, &c->d_sbv}) {
            d->alloc(nb * c->J * sizeof(double));
            HIPCHK(hipMemsetAsync(d->p, 0, d->bytes, st));
        }
        const bool refm = cf.rng_mode == SBMF_RNG_REFERENCE;
        c->d_var3u.alloc((refm ? nb : 0) * 3 * c->I * sizeof(double));
        c->d_var3v.alloc((refm ? nb : 0) * 3 * c->J * sizeof(double));
        c->d_epart.alloc(nb * 2 * ((size_t)c->I + 1) * sizeof(double));  // per user row {sum e, sum e^2}
        c->b0 = c->mu_b0 = c->sig_b0 = 0.0;
        c->empty_u.clear();
        c->empty_v.clear();
        for (uint32_t i = 0; c->bias && i < c->I; ++i)
            if (c->users.ptr[i + 1] == c->users.ptr[i]) c->empty_u.push_back(i);
        for (uint32_t j = 0; c->bias && j < c->J; ++j)
            if (c->items.ptr[j + 1] == c->items.ptr[j]) c->empty_v.push_back(j);
        c->shadow_u.assign(c->empty_u.size(), {0.0, 0.0, 0.0});
        c->shadow_v.assign(c->empty_v.size(), {0.0, 0.0, 0.0});
    }
    c->sig_u.assign(c->K, 0.0);
    c->mu_u.assign(c->K, 0.0);
    c->sig_v.assign(c->K, 0.0);
    c->mu_v.assign(c->K, 0.0);
    c->tau = 1.0;

    // initial factors (gibbs_sbpmf_final.cpp:236-250)
    if (cf.rng_mode == SBMF_RNG_REFERENCE) {
        c->grand.seed_((unsigned)cf.seed);
        std::vector<double> U((size_t)c->I * c->K), V((size_t)c->J * c->K);
        for (uint32_t i = 0; i < c->I; ++i)
            for (uint32_t k = 0; k < c->K; ++k) U[(size_t)i * c->K + k] = 0.0 + c->init_sd * leva_normal(c->grand);
        for (uint32_t k = 0; k < c->K; ++k)  // V is k-major in the reference
            for (uint32_t j = 0; j < c->J; ++j) V[(size_t)j * c->K + k] = 0.0 + c->init_sd * leva_normal(c->grand);
        HIPCHK(hipStreamSynchronize(st));
        upload_table<T>(c, c->d_U, U.data(), c->I);
        upload_table<T>(c, c->d_V, V.data(), c->J);
    } else {
        HIPCHK(launch_init_philox<T>(c->d_U.as<T>(), c->K, c->Kp, 0, c->I, c->init_sd, cf.seed, TAG_INIT_U, st));
        HIPCHK(launch_init_philox<T>(c->d_V.as<T>(), c->K, c->Kp, 0, c->J, c->init_sd, cf.seed, TAG_INIT_V, st));
    }
    HIPCHK(hipStreamSynchronize(st));
    c->kprof = std::getenv("SBMF_KPROF") && std::atoi(std::getenv("SBMF_KPROF")) > 0;
    if (c->kprof) {
        if (const char* e = std::getenv("SBMF_KPROF_SET")) c->kprof_set = std::atoi(e) ? 1 : 0;
        c->d_kprof.alloc(96 * sizeof(unsigned long long));
        HIPCHK(hipMemset(c->d_kprof.p, 0, 96 * sizeof(unsigned long long)));
    }
    for (hipEvent_t& e : c->kevs) event_destroy(e);
    for (hipEvent_t& e : c->sev) event_destroy(e);
    c->kevs.assign((size_t)c->nstages * 2 * SBMF_NKIND * 2, nullptr);
    c->kprev.assign((size_t)c->nstages * 2 * SBMF_NKIND, (int8_t)-1);
    c->kbegin.assign((size_t)c->nstages * 2 * SBMF_NKIND, nullptr);
    c->sev.assign((size_t)2 * c->nstages, nullptr);
    for (hipEvent_t& e : c->kevs) event_create(&e);
    for (hipEvent_t& e : c->sev) event_create(&e, hipEventDisableTiming);
    for (hipEvent_t& e : c->tsev) event_destroy(e);
    c->tsev.assign(c->virt ? (size_t)2 * (c->nstages + 1) : 0, nullptr);
    for (hipEvent_t& e : c->tsev) event_create(&e);
    c->sweep = 0;
    c->collected = 0;
    fill_kernel_bytes(c);
    c->prepared = true;
}

// Streaming-kernel tasks (at most `cmax` ratings each: a whole row, or the
// equal chunks of a longer row) in one list, largest rows first, claimed in
// order by the running workgroups of a launch of `gres` workgroups (k_gres'
// queue); a split row's chunks are consecutive.
static void build_stream_tasks(const Side& s, Side::StreamSet& S, const std::vector<uint32_t>& rows, uint32_t gres,
                               uint32_t nblk) {
    const uint32_t cmax = S.cmax;
    S.stasks.clear();
    S.xrows.clear();
    S.nxchunk = 0;
    S.sgrid = 0;
    for (uint32_t r : rows) {  // rows: degree-descending
        const uint32_t n = s.ptr[r + 1] - s.ptr[r];
        const uint32_t nch = (n + cmax - 1) / cmax;
        if (nch > gres)
            fail(SBMF_E_ARG, "row %u has %u ratings: more than %u co-resident chunks of %u", r, n, gres, cmax);
        if (nch == 1) {
            S.stasks.push_back(SplitTask{r, s.ptr[r], n, 1, 0, 0, 0, 0});
        } else {
            const uint32_t slab0 = S.nxchunk;
            const uint32_t cnt0 = (uint32_t)S.xrows.size() * nblk;
            const uint32_t per = (n + nch - 1) / nch;
            for (uint32_t c = 0; c < nch; ++c) {
                const uint32_t b = c * per, e = std::min(n, b + per);
                S.stasks.push_back(SplitTask{r, s.ptr[r] + b, e - b, nch, c, slab0, cnt0, 0});
            }
            S.xrows.push_back(SplitRow{r, slab0, nch, 0});
            S.nxchunk += nch;
        }
    }
    S.sgrid = std::min<uint32_t>(gres, (uint32_t)S.stasks.size());
}

// ------------------------------------------------------------------ one sweep
struct HostStream {  // variates of one sweep, in the reference's consumption order
    double g_tau;
    double g_sb0 = 0, z_mb0 = 0, z_b0 = 0;  // biased sampler: sigma_b0, mu_b0, b0
    std::vector<double> g_su, z_mu, g_sv, z_mv;
};

// Unbiased samplers: tau (:339-342), then per k {sigma_u, mu_u, sigma_v, mu_v}
// (:375-414).  Biased sampler (top-level gibbs_sbpmf2.cpp:366-467): alpha with
// shape a0 + N, sigma_b0 / mu_b0 / b0, then per k with shapes alpha0 + I / + J.
template <class G>
static void draw_hyper_variates(G& g, sbmf_ctx* c, HostStream& hs) {
    const sbmf_config& cf = c->cfg;
    const uint64_t N = c->tu.size();
    if (c->bias) {
        hs.g_tau = mt_gamma(g, cf.a0 + (double)N);
        hs.g_sb0 = mt_gamma(g, cf.alpha0 + 1);
        hs.z_mb0 = leva_normal(g);
        hs.z_b0 = leva_normal(g);
    } else {
        hs.g_tau = mt_gamma(g, cf.a0 + 0.5 * (double)N);
    }
    hs.g_su.resize(c->K);
    hs.z_mu.resize(c->K);
    hs.g_sv.resize(c->K);
    hs.z_mv.resize(c->K);
    const double shu = c->bias ? cf.alpha0 + c->I : cf.alpha0 + 0.5 * (c->I + 1);
    const double shv = c->bias ? cf.alpha0 + c->J : cf.alpha0 + 0.5 * (c->J + 1);
    for (uint32_t k = 0; k < c->K; ++k) {
        hs.g_su[k] = mt_gamma(g, shu);
        hs.z_mu[k] = leva_normal(g);
        hs.g_sv[k] = mt_gamma(g, shv);
        hs.z_mv[k] = leva_normal(g);
    }
}

// Reference mode, biased sampler: the per-row bias hyperparameter variates of
// every user then every item (:470-489, :492-511), then per user {b_i, K
// factor normals} (:515-558) and per item {b_j, K normals} (:563-606).
//
// ran_gaussian(mean, stdev) consumes no variate when stdev is 0 or NaN
// (random.h:166-172).  That happens for rows without train ratings: their
// bias draw has variance 1/sigma_b (no data term), so under the reference's
// variance-as-stdev quirk the walk b -> N(mu, 1/sigma_b), sigma_b ~ 1/b^2
// grows like b^2 per sweep, overflows, and turns NaN within a few dozen
// sweeps.  From then on the reference skips those draws.  The walk of such a
// row depends only on its own variates, so the host replays it here in the
// reference's exact expressions to know which draws the stream skips (a
// skipped slot carries 0: the device then yields the mean, as the reference
// does); k_bias_rows evaluates the same expressions without contraction and
// reaches the same values.
template <typename T>
static void fill_bias_variates(sbmf_ctx* c) {
    const uint32_t K = c->K;
    const sbmf_config& cf = c->cfg;
    auto sdv = [&](double var) { return c->sd_is_var ? var : std::sqrt(var); };
    auto consumes = [](double sd) { return !(sd == 0.0 || std::isnan(sd)); };
    auto hyper_rows = [&](uint32_t R, const std::vector<uint32_t>& empty, std::vector<std::array<double, 3>>& sh,
                          std::vector<double>& v) {
        size_t e = 0;
        for (uint32_t r = 0; r < R; ++r) {
            const double g = mt_gamma(c->grand, cf.alpha0 + 1);
            v[3 * (size_t)r] = g;
            if (e < empty.size() && empty[e] == r) {  // shadow: (b, mu, sigma)
                std::array<double, 3>& x = sh[e++];
                x[2] = g / (cf.beta0 + (0.5 * (x[0] - x[1]) * (x[0] - x[1])));
                const double s4 = 1.0 / (cf.nu0 + x[2]);
                const double mean = s4 * ((cf.nu0 * cf.mu0) + x[0] * x[2]);
                const double z = consumes(sdv(s4)) ? leva_normal(c->grand) : 0.0;
                v[3 * (size_t)r + 1] = z;
                x[1] = consumes(sdv(s4)) ? mean + sdv(s4) * z : mean;
            } else {
                v[3 * (size_t)r + 1] = leva_normal(c->grand);
            }
        }
    };
    auto bias_draw = [&](const std::vector<uint32_t>& empty, std::vector<std::array<double, 3>>& sh, uint32_t r,
                         size_t& e) -> double {
        if (e < empty.size() && empty[e] == r) {
            std::array<double, 3>& x = sh[e++];
            const double sb = 1 / (x[2] + (c->tau * 0.0));
            const double mb = sb * ((x[2] * x[1]) + c->tau * 0.0);
            if (!consumes(sdv(sb))) {
                x[0] = mb;
                return 0.0;
            }
            const double z = leva_normal(c->grand);
            x[0] = mb + sdv(sb) * z;
            return z;
        }
        return leva_normal(c->grand);
    };
    std::vector<double> vu((size_t)3 * c->I), vv((size_t)3 * c->J);
    hyper_rows(c->I, c->empty_u, c->shadow_u, vu);
    hyper_rows(c->J, c->empty_v, c->shadow_v, vv);
    const size_t nz = ((size_t)c->I + c->J) * K;
    ensure_pinned(c, nz * sizeof(T));
    T* h = reinterpret_cast<T*>(c->h_pinned);
    size_t e = 0;
    for (uint32_t i = 0; i < c->I; ++i) {
        vu[3 * (size_t)i + 2] = bias_draw(c->empty_u, c->shadow_u, i, e);
        for (uint32_t k = 0; k < K; ++k) h[(size_t)i * K + k] = (T)leva_normal(c->grand);
    }
    T* hv = h + (size_t)c->I * K;
    e = 0;
    for (uint32_t j = 0; j < c->J; ++j) {
        vv[3 * (size_t)j + 2] = bias_draw(c->empty_v, c->shadow_v, j, e);
        for (uint32_t k = 0; k < K; ++k) hv[(size_t)j * K + k] = (T)leva_normal(c->grand);
    }
    HIPCHK(hipMemcpy(c->d_zU.p, h, (size_t)c->I * K * sizeof(T), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->d_zV.p, hv, (size_t)c->J * K * sizeof(T), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->d_var3u.p, vu.data(), vu.size() * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->d_var3v.p, vv.data(), vv.size() * sizeof(double), hipMemcpyHostToDevice));
}

static BiasArgs bias_args(const sbmf_ctx* c, bool users, double d0) {
    BiasArgs p{};
    p.alpha = c->tau;
    p.d0 = d0;
    p.ag = c->cfg.alpha0;
    p.bg = c->cfg.beta0;
    p.sg = c->cfg.nu0;
    p.mg = c->cfg.mu0;
    p.seed = c->cfg.seed;
    p.sweep = c->sweep;
    p.tag = users ? TAG_BIAS_U : TAG_BIAS_V;
    p.sd_is_var = c->sd_is_var;
    return p;
}

template <typename T>
static void fill_z(sbmf_ctx* c, uint32_t R, DBuf& d) {
    const size_t n = (size_t)R * c->K;
    ensure_pinned(c, n * sizeof(T));
    T* h = reinterpret_cast<T*>(c->h_pinned);
    for (size_t x = 0; x < n; ++x) h[x] = (T)leva_normal(c->grand);
    HIPCHK(hipMemcpy(d.p, h, n * sizeof(T), hipMemcpyHostToDevice));
}

template <typename T>
static HalfArgs<T> half_args(sbmf_ctx* c, bool users) {
    HalfArgs<T> a{};
    const bool md = c->nranks > 1;
    if (users) {
        a.ptr = c->d_uptr.as<uint32_t>();
        a.part = c->d_upart.as<uint32_t>();
        a.perm = (md ? c->d_uperm2 : c->d_uperm).as<uint32_t>();
        a.E_this = c->d_Eu.as<T>();   // user order
        a.E_other = c->d_Ev.as<T>();  // item order
        a.r_this = c->d_ur.as<T>();
        a.own = c->d_U.as<T>();
        a.partner = c->d_V.as<T>();
        a.sig = c->d_hyper.as<T>();
        a.mu = c->d_hyper.as<T>() + c->Kp;
        a.zrow = c->J;
        a.zbuf = c->d_zU.as<T>();
        a.tag = TAG_USERS;
        a.row_sq = nullptr;
        a.row_tr = nullptr;
    } else {
        a.ptr = c->d_vptr.as<uint32_t>();
        a.part = c->d_vpart.as<uint32_t>();
        a.perm = (md ? c->d_vperm2 : c->d_vperm).as<uint32_t>();
        a.E_this = c->d_Ev.as<T>();   // item order
        a.E_other = c->d_Eu.as<T>();  // user order
        a.r_this = c->d_vr.as<T>();
        a.own = c->d_V.as<T>();
        a.partner = c->d_U.as<T>();
        a.sig = c->d_hyper.as<T>() + 2 * c->Kp;
        a.mu = c->d_hyper.as<T>() + 3 * c->Kp;
        a.zrow = c->I;
        a.zbuf = c->d_zV.as<T>();
        a.tag = TAG_ITEMS;
        a.row_sq = c->d_rowsq_v.as<double>();
        a.row_tr = c->cfg.eval_train ? c->d_rowtr_v.as<double>() : nullptr;
    }
    a.tune = c->cfg.tune;
    a.prof = c->kprof ? c->d_kprof.as<unsigned long long>() + 16 + 8 * (users ? 0 : 1) : nullptr;
    a.tau = (T)c->tau;
    a.K = c->K;
    a.Kp = c->Kp;
    a.sd_is_var = c->sd_is_var;
    a.seed = c->cfg.seed;
    a.sweep = c->sweep;
    a.lo = (T)c->lo;
    a.hi = (T)c->hi;
    a.lim_partner = (uint64_t)((users ? c->J : c->I) + 2) * c->Kp;
    a.lim_other = (uint64_t)c->tu.size() + (users ? c->users.nsend : c->items.nsend);
    a.lim_this = c->tu.size();
    a.lim_rows = users ? c->I : c->J;
    // tune bit 1: residuals from r - own.partner (the former multi-GPU form, kept for validation);
    // otherwise every rank reads the residuals the exchange delivered
    a.e_from_dot = (c->cfg.tune & 2u) ? 1 : 0;
    return a;
}

// `start` (optional): a timing event the caller has just recorded on the compute stream with
// nothing queued there since.  The half then forks its side streams from it and, when nothing
// precedes its first kind on the compute stream, times that kind from it: two event records
// back to back on a stream leave the device idle ~6 us each (r04f trace; ML-1M K=50 r05s42:
// 37 us between the user half's end and the item half's streaming launch).
template <typename T>
static void run_half(sbmf_ctx* c, bool users, uint32_t stage, hipEvent_t start = nullptr) {
    Side& s = users ? c->users : c->items;
    Side::Stage& g = *s.stg[stage];
    HalfArgs<T> a = half_args<T>(c, users);
    hipStream_t st = c->st;
    const int sd = users ? 0 : 1;
    // Overlap (default; tune bit 29 off): the streaming launch (persistent, queue
    // order) on `st`, every other bin on `sto` beside it, so the short Gram-block
    // launches fill the CU time the streaming launch's serial phases (solve,
    // split-row hand-offs) and its tail leave idle.  Rows of different bins are
    // disjoint and no launch reads another's outputs, so the results do not
    // depend on the interleaving.  The streaming launch is an ordinary one in every
    // schedule (its claiming workgroups are resident by construction; tune bit 24's
    // cooperative launch, experiments only, would wait for the whole device).
    int others = 0;
    for (int k = 0; k < NBIN; ++k) others += k != KIND_STREAM && !g.bin_rows[k].empty();
    const bool serial = (c->cfg.tune & 0x20000000u) != 0;
    const bool ovl = !serial && others && !g.bin_rows[KIND_STREAM].empty();
    // The Gram-block kinds alternate between two side streams (sto, sto2), so they also run
    // beside each other: a small stage's kinds are each bound by one row's latency through
    // its k-blocks, which a chain of launches adds up (r05s2 per-rank trace).  Per-rank
    // compute of the 8-way split, 4 stages: K=100 2.06 -> 1.96 ms, K=200 3.09 -> 2.76 ms;
    // the single-GPU sweep is unchanged (7.33 both ways, r05s5).  Tune bit 25: one side stream.
    // With two stream sets (items: rows > 1024 on 16-wave workgroups, set 1, and the
    // rest on 8-wave ones, set 0), set 1 runs on `st` and set 0 on `sto` beside it
    // (tune bit 30: one after the other), each with split-row areas of its own.
    // Side by side pays nothing at ML-20M (r05s32, neutral) and costs on small stages (ML-1M K=50:
    // 0.424-0.453 ms side by side, 0.416-0.423 in turn, r05s43): below kSetsSideMin ratings in the
    // stage (ML-1M, a rank's stage of an 8-way ML-20M split) the sets run one after the other
    // (SBMF_SETS_SIDE_MIN overrides the threshold: measurements only)
    static const uint64_t kSetsSideMin = [] {
        const char* e = std::getenv("SBMF_SETS_SIDE_MIN");
        return e ? (uint64_t)std::strtoull(e, nullptr, 10) : (uint64_t)4000000;
    }();
    const bool big = (uint64_t)(s.ptr[g.r1] - s.ptr[g.r0]) >= kSetsSideMin;
    const bool sov = ovl && big && !(c->cfg.tune & 0x40000000u) && !g.ss[0].stasks.empty() && !g.ss[1].stasks.empty();
    // Beside two streaming sets every Gram-block kind goes to sto2: on sto it would queue behind
    // set 0 (r05s14 trace: two item kinds, 0.18 ms, ran after the stage; measured neutral, 6.91
    // ms both ways, r05s15: the persistent sets hold every CU, so the kinds' work only moves)
    const bool two = !serial && (others >= 2 || sov) && !(c->cfg.tune & 0x2000000u);
    const bool side = ovl || two;
    // (the long-row set alone first, every other launch of the half after it, so its split rows'
    // chunks share no CU with other launches' workgroups: user half 2.77-2.81 -> 2.86-3.04 ms,
    // item half neutral, r06s6; not kept)
    // (the split-row counters and queue heads of both stream sets are zero: each streaming
    // launch's k_split_finish clears its own)
    bool st_busy = false;  // something queued on the compute stream since `start`
    auto fork = [&] {
        hipEvent_t f = start && !st_busy ? start : c->oev[0];
        if (f == c->oev[0]) HIPCHK(hipEventRecord(c->oev[0], c->st));
        HIPCHK(hipStreamWaitEvent(c->sto, f, 0));
        if (two) HIPCHK(hipStreamWaitEvent(c->sto2, f, 0));
    };
    if (side) fork();
    // (the Gram-block launches on `sto` ahead of set 0 instead of behind it: neutral, r04s22)
    int last[3] = {-1, -1, -1};  // the last kind launched on st / sto / sto2 (its end event recorded there)
    int nside = 0;  // Gram-block kinds launched so far (two: even ones on sto, odd ones on sto2)
    for (int k = NBIN - 1; k >= 0; --k) {
        if (g.bin_rows[k].empty()) continue;
        st = side && k != KIND_STREAM ? (two && (sov || (nside++ & 1)) ? c->sto2 : c->sto) : c->st;
        // launch-kind events: the streaming kind's every sweep (the bench's roofline), the
        // others' on the first sweep of a run only (each event between two launches on a
        // stream leaves the device idle ~6 us)
        const bool timed = c->time_kinds || k == KIND_STREAM;
        int& lk = last[st == c->st ? 0 : st == c->sto ? 1 : 2];
        if (timed) {
            c->kpv(stage, sd, k) = (int8_t)lk;
            if (lk < 0) {
                if (st == c->st && start && !st_busy) {
                    c->kbg(stage, sd, k) = start;  // the caller's event is this kind's start
                } else {
                    HIPCHK(hipEventRecord(c->kev(stage, sd, k, 0), st));
                    c->kbg(stage, sd, k) = c->kev(stage, sd, k, 0);
                }
            }
            lk = k;
        } else {
            lk = -1;  // no end event behind this launch
        }
        // f64 rows of 65..128 ratings on one-wave k_grow workgroups, 129..256 on two-wave ones
        // (the streaming kernel's code on whole rows: 32 vectors per wave, one wave with no
        // cross-wave sum or D hand-off) instead of 3-4-wave Gram-block rows: user half
        // 3.20-3.24 -> 2.93-3.04 ms, sweep 7.22-7.25 -> 7.02-7.06 (r05s11, 2 interleaved
        // rounds); the 9..64-rating bin too, on one-wave k_grow workgroups (sweep 6.99-7.03 ->
        // 6.90-6.95, r05s12).  Tune bits 8 / 9 / 10 keep the Gram-block kinds of these bins.
        const uint32_t tn = c->cfg.tune;
        // f32 rows of 17..256 ratings on one-wave k_grow workgroups, 257..512 on two-wave ones (64
        // vectors per f32 wave): f32 sweep 5.46 -> 4.63 ms (r05s18); tune bit 11 keeps the
        // Gram-block kinds
        const bool g32 = sizeof(T) == 4 && !(tn & 0x800u);
        const int gw = g32 ? (k == GK_W16 || k == GK_B2 || k == GK_B4 ? 1 : k == GK_B8 ? 2 : 0)
                       : sizeof(T) != 8                               ? 0
                       : k == GK_B4 && !(tn & 0x100u)                 ? 1
                       : k == GK_B8 && !(tn & 0x200u)                 ? 2
                       : k == GK_W16 && !(tn & 0x400u) && !(tn & 8u)  ? 1
                                                                      : 0;
        if (gw) {
            HIPCHK(launch_grow<T>(gw, g.d_bins[k].as<uint32_t>(), (uint32_t)g.bin_rows[k].size(), a, st));
        } else if (k < GK_NUM && k >= GK_B2 && !(c->cfg.tune & 4u)) {
            for (const auto& gs : g.gsub[k])
                HIPCHK(launch_gblock_nw<T>((int)gs[0], g.d_bins[k].as<uint32_t>() + gs[1], gs[2], a, st));
        } else if (k < GK_NUM)
            HIPCHK(launch_gblock<T>(k, g.d_bins[k].as<uint32_t>(), (uint32_t)g.bin_rows[k].size(), a, st));
        else {
            for (int q = 0; q < 2; ++q) {
                const int set = sov ? 1 - q : q;  // set 1 (the long rows) first
                const Side::StreamSet& S = g.ss[set];
                if (S.stasks.empty()) continue;
                const hipStream_t ss = sov && set == 0 ? c->sto : st;
                const size_t ox = set ? c->xset_nx : 0, orow = set ? c->xset_nr : 0;
                SplitSync sy{};
                sy.nblk = (c->K + 15) / 16;
                sy.slabs = c->d_xslabs.as<double>() + ox * sy.nblk * (16 * 16 + 16);
                sy.counters = c->d_xcnt.as<uint32_t>() + (set ? orow * sy.nblk + 1 : 0);
                sy.ncounters = (uint32_t)S.xrows.size() * sy.nblk;
                sy.chunk_sq = c->d_xchunk_sq.as<double>() + ox;
                sy.chunk_tr = c->d_xchunk_tr.as<double>() + ox;
                sy.newown = c->d_xnewown.as<T>() + ox * c->Kp;
                sy.timeout = reinterpret_cast<uint32_t*>(c->d_res.as<double>() + RES_TIMEOUT);
                sy.cmax = S.cmax;
                sy.lim_slab = (uint64_t)(c->d_xslabs.bytes / sizeof(double)) - ox * sy.nblk * (16 * 16 + 16);
                sy.lim_chunk = (uint32_t)(c->d_xchunk_sq.bytes / sizeof(double) - ox);
                sy.prof = c->kprof && set == c->kprof_set ? c->d_kprof.as<unsigned long long>() + 8 * (users ? 0 : 1) : nullptr;
                HalfArgs<T> as = a;
                as.tune = S.tune;
                HIPCHK(launch_gstream<T>(g.d_stasks[set].as<SplitTask>(), (uint32_t)S.stasks.size(), S.sgrid,
                                         g.d_xrows[set].as<SplitRow>(), (uint32_t)S.xrows.size(), as, sy, ss));
                if (ss == c->st) st_busy = true;
            }
            if (sov) {  // the streaming stage ends with both sets
                HIPCHK(hipEventRecord(c->oev[2], c->sto));
                HIPCHK(hipStreamWaitEvent(st, c->oev[2], 0));
            }
        }
        if (st == c->st) st_busy = true;
        // (a kind launched next on this stream starts its time at this event)
        if (timed) HIPCHK(hipEventRecord(c->kev(stage, sd, k, 1), st));
        c->timing.n_launch++;
    }
    if (side) {
        HIPCHK(hipEventRecord(c->oev[1], c->sto));
        HIPCHK(hipStreamWaitEvent(c->st, c->oev[1], 0));
        if (two) {
            HIPCHK(hipEventRecord(c->oev[3], c->sto2));
            HIPCHK(hipStreamWaitEvent(c->st, c->oev[3], 0));
        }
    }
}

// SURVEY.md §8(d) algorithmic bytes of one launch over `rows`.
static uint64_t alg_bytes(const Side& s, const std::vector<uint32_t>& rows, uint32_t K, uint64_t tsz) {
    uint64_t b = 0;
    for (uint32_t r : rows) b += (uint64_t)(s.ptr[r + 1] - s.ptr[r]) * (tsz * K + 4 + tsz) + 2 * tsz * K;
    return b;
}
static void fill_kernel_bytes(sbmf_ctx* c) {
    const uint64_t tsz = tsize(c);
    for (int sd = 0; sd < 2; ++sd) {
        const Side& s = sd == 0 ? c->users : c->items;
        for (int k = 0; k < SBMF_NKIND; ++k) {
            c->timing.kern_bytes[sd][k] = 0;
            c->timing.kern_rows[sd][k] = 0;
        }
        for (const auto& g : s.stg) {  // a kind's launches summed over the stages
            for (int k = 0; k < NBIN; ++k) {
                c->timing.kern_bytes[sd][k] += alg_bytes(s, g->bin_rows[k], c->K, tsz);
                c->timing.kern_rows[sd][k] += (uint32_t)g->bin_rows[k].size();
            }
        }
    }
}

static double ev_ms(hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return NAN;
    return ms;
}

// After a stage of a half (users: scatter into item order, E_v; items: into
// E_u): send the stage's residuals bound for other ranks' rows, unpack what
// every rank's same stage sends here.  `with(p)` (optional) issues the stage's
// block broadcasts first, all in one RCCL group (collectives only: they run
// concurrently); the residual send/receive keeps a group of its own; the
// unpack follows it.  Offsets are taken relative to the stage's segments, so a
// transfer touches only this stage's part of the send and receive areas.
template <typename T, class F>
static void exchange_stage(sbmf_ctx* c, bool users, uint32_t p, hipStream_t st, F&& with) {
    if (c->nranks <= 1) return;
    const Side& s = users ? c->users : c->items;
    const Side::Stage& g = *s.stg[p];
    DBuf& E = users ? c->d_Ev : c->d_Eu;
    auto rel = [](const std::vector<size_t>& v, size_t base) {
        std::vector<size_t> b(v);
        for (size_t& x : b) x = (x - base) * sizeof(T);
        return b;
    };
    auto bytes = [](const std::vector<size_t>& v) {
        std::vector<size_t> b(v);
        for (size_t& x : b) x *= sizeof(T);
        return b;
    };
    c->comm->group_begin();
    with(p);
    c->comm->group_end();
    const size_t s0 = g.soff.empty() ? 0 : g.soff[0];
    c->comm->alltoallv(E.as<T>() + c->tu.size() + s0, rel(g.soff, s0), bytes(g.scnt), c->d_xrecv.as<T>() + g.rbeg,
                      rel(g.roff, g.rbeg), bytes(g.rcnt), st);
    HIPCHK(launch_unpack<T>(c->d_xrecv.as<T>() + g.rbeg, (users ? c->d_uunpack : c->d_vunpack).as<uint32_t>() + g.rbeg,
                            g.rend - g.rbeg, E.as<T>(), st));
}
// Every stage's residual exchange, on `st` (no broadcasts: the prologue's recompute)
template <typename T>
static void exchange_residuals(sbmf_ctx* c, bool users, hipStream_t st) {
    for (uint32_t p = 0; p < c->nstages; ++p) exchange_stage<T>(c, users, p, st, [](uint32_t) {});
}
// Every rank's units of stage p of `s` (its rows [sbounds[k][p], sbounds[k][p+1]))
static void bcast_stage(sbmf_ctx* c, const Side& s, uint32_t p, void* base, size_t unit_bytes) {
    std::vector<uint64_t> lo(c->nranks), hi(c->nranks);
    for (int k = 0; k < c->nranks; ++k) {
        lo[k] = s.sbounds[k][p];
        hi[k] = s.sbounds[k][p + 1];
    }
    c->comm->bcast_blocks(base, unit_bytes, lo, hi, c->stc);
}
// A half's stages, each followed -- on the comm stream, while the next stage
// computes -- by its exchange; the compute stream then waits for the last one.
template <typename T, class F>
static void run_half_pipelined(sbmf_ctx* c, bool users, F&& bcasts, hipEvent_t start = nullptr) {
    const int sd = users ? 0 : 1;
    const size_t tb = (size_t)sd * (c->nstages + 1);
    if (c->virt) HIPCHK(hipEventRecord(c->tsev[tb], c->st));
    for (uint32_t p = 0; p < c->nstages; ++p) {
        run_half<T>(c, users, p, p == 0 && !c->virt ? start : nullptr);
        if (c->nranks > 1) HIPCHK(hipEventRecord(c->sev[(size_t)sd * c->nstages + p], c->st));
        if (c->virt) HIPCHK(hipEventRecord(c->tsev[tb + p + 1], c->st));
    }
    HIPCHK(hipEventRecord(c->ev[users ? 2 : 4], c->st));
    if (c->nranks <= 1) return;  // no exchange: ev[3] / ev[5] are not recorded (the sweep uses ev[2] / ev[4])
    for (uint32_t p = 0; p < c->nstages; ++p) {
        HIPCHK(hipStreamWaitEvent(c->stc, c->sev[(size_t)sd * c->nstages + p], 0));
        exchange_stage<T>(c, users, p, c->stc, bcasts);
    }
    HIPCHK(hipEventRecord(c->cev[sd], c->stc));
    HIPCHK(hipStreamWaitEvent(c->st, c->cev[sd], 0));
}

template <typename T>
static void run_sweeps_T(sbmf_ctx* c, uint32_t nsweeps, sbmf_sweep_cb cb, void* user) {
    const sbmf_config& cf = c->cfg;
    hipStream_t st = c->st;
    const uint32_t K = c->K;
    const uint64_t N = c->tu.size();
    const bool ref = cf.rng_mode == SBMF_RNG_REFERENCE;
    const bool q2 = cf.quirks == SBMF_QUIRKS_SBPMF2;
    double* d_res = c->d_res.as<double>();
    double* scratch = c->d_scratch.as<double>();
    // Throughput mode (Philox: the draws of sweep s depend only on (seed, s)): the
    // next sweep's prologue -- residual sum of squares, column statistics and the
    // host hyperparameter draws -- is issued at the end of this sweep, its kernels
    // beside the test evaluation (one rank; before it otherwise) and its host draws
    // while the evaluation runs, so
    // the GPU does not wait for the host round trip at the start of the next
    // sweep.  The inputs are the same (U, V and the residuals do not change in
    // between), so the chain is bitwise the same.  Tune bit 26 turns it off.
    const bool overlap = !ref && !(cf.tune & 0x4000000u);
    // ---- 1. the prologue's kernels for sweep sw; its sums land in c->h_pre (copy: here; the
    // overlapped prologue's sums travel with the sweep's results in one copy)
    auto prologue_gpu = [&](uint32_t sw, bool copy = true) {
        // ---- 1. residual sum of squares (E recompute at sweep start, :317-334)
        const bool recompute = sw == 0 || (cf.recompute_every && sw % cf.recompute_every == 0);
        if (recompute) {
            // residuals of every rating, scattered into user order for the user half
            HIPCHK(launch_resid<T>(c->d_rtasks.as<ResidTask>(), (uint32_t)c->items.rtasks.size(),
                                   c->d_rtptr.as<uint32_t>(), c->items.r0, c->items.r1, c->d_vpart.as<uint32_t>(),
                                   (c->nranks > 1 ? c->d_vperm2 : c->d_vperm).as<uint32_t>(), c->d_vr.as<T>(),
                                   c->d_V.as<T>(), c->d_U.as<T>(), K,
                                   c->Kp, c->d_Eu.as<T>(), c->d_rtsq.as<double>(), c->d_rowsq_v.as<double>(),
                                   c->bias ? c->d_bv.as<double>() : nullptr, c->d_bu.as<double>(), c->b0, st));
            c->timing.n_launch++;
            if (c->nranks > 1) c->comm->bcast_ranges(c->d_rowsq_v.p, sizeof(double), c->items.bounds, st);
            exchange_residuals<T>(c, false, st);
        }
        HIPCHK(launch_sum(c->d_rowsq_v.as<double>(), c->J, d_res + RES_ESQ, scratch, st));
        // biased sampler: sum(E) and sum(E^2) of the sweep-start residuals (:342-359), per
        // own user row, rows exchanged, summed in row order (the same for any rank split)
        if (c->bias) {
            double* rs2 = c->d_epart.as<double>();
            HIPCHK(launch_rowsum2<T>(c->d_uptr.as<uint32_t>(), c->users.r0, c->users.r1, c->d_Eu.as<T>(), rs2, st));
            if (c->nranks > 1) c->comm->bcast_ranges(rs2, 2 * sizeof(double), c->users.bounds, st);
            HIPCHK(launch_sum_cols(rs2, c->I, 2, d_res + RES_ES, st));
        }
        // ---- column statistics with the current mu (:378-381, :397-401)
        const T* hyp = c->d_hyper.as<T>();
        double* colpart = c->d_colpart.as<double>();
        double* colpart_v = colpart + (size_t)((c->I + 255) / 256) * 2 * K;
        HIPCHK(launch_colstats<T>(c->d_U.as<T>(), c->I, hyp + c->Kp, colpart, c->d_V.as<T>(), c->J, hyp + 3 * c->Kp,
                                  colpart_v, K, c->Kp, st));
        HIPCHK(launch_sum_cols2(colpart, (c->I + 255) / 256, d_res + RES_COL, colpart_v, (c->J + 255) / 256,
                                d_res + RES_COL + 2 * K, 2 * K, st));
        c->timing.n_launch += 3;
        if (copy) HIPCHK(hipMemcpyAsync(c->h_pre, d_res, c->h_res.size() * sizeof(double), hipMemcpyDeviceToHost, st));
    };
    // ---- 2. host draws (:339-342, :375-414) from the prologue's sums: updates
    // c->tau, sigma / mu (and the biased sampler's globals); returns d0
    auto host_draw = [&](const HostStream& hs) -> double {
        const double* res = c->h_pre;
        const double* Su2 = &res[RES_COL];
        const double* Su1 = Su2 + K;
        const double* Sv2 = Su2 + 2 * K;
        const double* Sv1 = Su2 + 3 * K;
        auto sd = [&](double var) { return c->sd_is_var ? var : std::sqrt(var); };
        double d0 = 0.0;  // biased sampler: global-bias delta, folded into the user half's residual pass
        if (c->bias) {
            // top-level gibbs_sbpmf2.cpp:366-467 (= src/libfm/gibbs_sbpmf22.cpp:345-446)
            const double es = res[RES_ES], esq = res[RES_ESQ2];
            c->tau = hs.g_tau / (cf.b0 + esq);
            c->sig_b0 = hs.g_sb0 / (cf.beta0 + (0.5 * (c->b0 - c->mu_b0) * (c->b0 - c->mu_b0)));
            const double s0 = 1.0 / (cf.nu0 + c->sig_b0);
            c->mu_b0 = s0 * ((cf.nu0 * cf.mu0) + c->b0 * c->sig_b0) + sd(s0) * hs.z_mb0;
            const double sb0 = 1 / (c->sig_b0 + c->tau * (double)N);
            const double mb0 = sb0 * (c->sig_b0 * c->mu_b0 + c->tau * (es + (double)N * c->b0));
            const double old = c->b0;
            c->b0 = mb0 + sd(sb0) * hs.z_b0;
            d0 = old - c->b0;
            for (uint32_t k = 0; k < K; ++k) {
                c->sig_u[k] = hs.g_su[k] / (cf.beta0 + (0.5) * Su2[k]);
                const double s2 = 1 / (cf.nu0 + c->sig_u[k] * c->I);
                c->mu_u[k] = s2 * (cf.nu0 * cf.mu0 + c->sig_u[k] * Su1[k]) + sd(s2) * hs.z_mu[k];
                c->sig_v[k] = hs.g_sv[k] / (cf.beta0 + (0.5) * Sv2[k]);
                const double s1 = 1 / (cf.nu0 + c->sig_v[k] * c->J);
                c->mu_v[k] = s1 * (cf.nu0 * cf.mu0 + c->sig_v[k] * Sv1[k]) + sd(s1) * hs.z_mv[k];
            }
        } else {
        const double esq = res[RES_ESQ];
        c->tau = hs.g_tau / (cf.b0 + 0.5 * esq);
        for (uint32_t k = 0; k < K; ++k) {
            const double du = c->mu_u[k] - cf.mu0;
            const double bu = q2 ? cf.beta0 + cf.nu0 * du * du + (0.5) * Su2[k]
                                 : cf.beta0 + 0.5 * cf.nu0 * du * du + (0.5) * Su2[k];
            c->sig_u[k] = hs.g_su[k] / bu;
            const double su_star = (double)1.0 / (cf.nu0 * c->sig_u[k] + c->sig_u[k] * c->I);
            const double mu_star = su_star * (cf.nu0 * cf.mu0 * c->sig_u[k] + c->sig_u[k] * Su1[k]);
            c->mu_u[k] = mu_star + sd(su_star) * hs.z_mu[k];
            const double dv = c->mu_v[k] - cf.mu0;
            const double bv = q2 ? cf.beta0 + cf.nu0 * dv * dv + (0.5) * Sv2[k]
                                 : cf.beta0 + 0.5 * cf.nu0 * dv * dv + (0.5) * Sv2[k];
            c->sig_v[k] = hs.g_sv[k] / bv;
            const double sv_star = (double)1.0 / (cf.nu0 * c->sig_v[k] + c->sig_v[k] * c->J);
            const double mv_star = (q2 ? su_star : sv_star) * (cf.nu0 * cf.mu0 * c->sig_v[k] + c->sig_v[k] * Sv1[k]);
            c->mu_v[k] = mv_star + sd(sv_star) * hs.z_mv[k];
        }
        }
        return d0;
    };
    // one rank: nothing between the halves and after the item half, so their events are the
    // halves' end events (two timing events back to back leave the device idle ~12 us)
    hipEvent_t& ev3 = c->nranks > 1 ? c->ev[3] : c->ev[2];
    hipEvent_t& ev5 = c->nranks > 1 ? c->ev[5] : c->ev[4];
    // the sweep's hyperparameters [sig_u | mu_u | sig_v | mu_v] into the pinned staging area
    // and on to d_hyper (stream order: after every launch already queued that reads it)
    auto stage_hyper = [&](const std::vector<double>& su, const std::vector<double>& mu, const std::vector<double>& sv,
                           const std::vector<double>& mv) {
        const size_t Kp = c->Kp;
        T* h = static_cast<T*>(c->h_hyper());
        HIPCHK(hipEventSynchronize(c->hev));
        std::fill(h, h + 4 * Kp, T(0));
        for (uint32_t k = 0; k < K; ++k) {
            h[k] = (T)su[k];
            h[Kp + k] = (T)mu[k];
            h[2 * Kp + k] = (T)sv[k];
            h[3 * Kp + k] = (T)mv[k];
        }
        HIPCHK(hipMemcpyAsync(c->d_hyper.p, h, 4 * Kp * sizeof(T), hipMemcpyHostToDevice, st));
        HIPCHK(hipEventRecord(c->hev, st));
    };
    // A sweep's start: its hyperparameters (drawn here, or staged at the end of the previous sweep in
    // throughput mode) and its user half.  Returns whether the start work was staged ahead.
    auto start_sweep = [&](bool first) -> bool {
        c->time_kinds = first;  // every launch kind timed on the first sweep of the run
        c->timing.n_launch = 0;
        HIPCHK(hipEventRecord(c->ev[0], st));
        double d0;
        // throughput mode: this sweep's hyperparameters already on the device and its normals
        // filled (both queued at the end of the previous sweep)
        const bool staged = c->pre.valid && c->pre.sweep == c->sweep && c->pre.staged;
        if (!staged && c->hyper_ahead) stage_hyper(c->sig_u, c->mu_u, c->sig_v, c->mu_v);
        c->hyper_ahead = false;
        if (c->pre.valid && c->pre.sweep == c->sweep) {  // drawn at the end of the previous sweep
            c->tau = c->pre.tau;
            c->b0 = c->pre.b0;
            c->mu_b0 = c->pre.mu_b0;
            c->sig_b0 = c->pre.sig_b0;
            c->sig_u = c->pre.sig_u;
            c->mu_u = c->pre.mu_u;
            c->sig_v = c->pre.sig_v;
            c->mu_v = c->pre.mu_v;
            d0 = c->pre.d0;
        } else {
            HostStream hs;
            if (ref) {
                draw_hyper_variates(c->grand, c, hs);
            } else {
                PhiloxStream ps(cf.seed, c->sweep, 0);
                draw_hyper_variates(ps, c, hs);
            }
            prologue_gpu(c->sweep, true);
            HIPCHK(hipStreamSynchronize(st));
            d0 = host_draw(hs);
        }
        c->pre.valid = false;
        c->pre.staged = false;
        if (!staged) {
            stage_hyper(c->sig_u, c->mu_u, c->sig_v, c->mu_v);
            if (ref && c->bias) {
                fill_bias_variates<T>(c);
            } else if (ref) {  // user variates then item variates (:485 then :529)
                fill_z<T>(c, c->I, c->d_zU);
                fill_z<T>(c, c->J, c->d_zV);
            }
            HIPCHK(hipStreamSynchronize(st));
            HIPCHK(hipEventRecord(c->ev[1], st));
        }
        hipEvent_t& ev1 = staged ? c->ev[0] : c->ev[1];
        // ---- 3. user half-sweep (throughput mode: this half's normals first)
        if (!ref && !staged)
            HIPCHK(launch_philox_fill<T>(c->d_zU.as<T>(), K, c->users.r0, c->users.r1, cf.seed, c->sweep, TAG_USERS, st));
        if (c->bias)  // per-user bias hyperparameters + b_i draw + residual shift (:470-489, :515-530)
            HIPCHK(launch_bias_rows<T>(c->d_uptr.as<uint32_t>(), c->users.r0, c->users.r1, c->d_Eu.as<T>(),
                                       c->d_bu.as<double>(), c->d_mbu.as<double>(), c->d_sbu.as<double>(),
                                       ref ? c->d_var3u.as<double>() : nullptr, bias_args(c, true, d0), st));
        // several ranks: each stage's fresh U (and b_i) blocks (one RCCL group), then its
        // residuals, while the next stage computes.  One rank: the half starts from the sweep's
        // start event when nothing was queued after it (staged start work, no bias pass)
        run_half_pipelined<T>(c, true, [&](uint32_t p) {
            bcast_stage(c, c->users, p, c->d_U.p, c->Kp * sizeof(T));
            if (c->bias) bcast_stage(c, c->users, p, c->d_bu.p, sizeof(double));
        }, c->nranks == 1 && staged && !c->bias ? ev1 : nullptr);
        if (c->nranks > 1) HIPCHK(hipEventRecord(c->ev[3], st));
        return staged;
    };
    // cfg.pipeline (throughput mode): sweep s+1's start is queued before sweep s is reported, so
    // the device does not idle through the host's per-sweep work (the report, the callback, the
    // next sweep's enqueue).  A stop the callback asks for then takes effect after sweep s+1.
    bool queued = false, q_staged = false, stop_after = false;
    for (uint32_t it = 0; it < nsweeps; ++it) {
        const bool staged = queued ? q_staged : start_sweep(it == 0);
        queued = false;
        hipEvent_t& ev1 = staged ? c->ev[0] : c->ev[1];
        const bool collect = q2 ? true : (c->sweep >= cf.burnin);
        if (collect) c->collected++;
        const double div = avg_collected(cf) ? (double)std::max(1u, c->collected) : (double)(c->sweep + 1);
        const uint64_t T_ = c->su.size();
        const bool par_eval = overlap && c->nranks == 1 && !(cf.tune & 0x10000000u);
        // The sweep's device work, from the item half to the results' copy (with the overlap the
        // next sweep's prologue kernels and normals are part of it).  (Captured once as a hipGraph
        // and replayed, one rank: ML-1M K=50 0.45 -> 0.77-0.90 ms, ML-20M 7.11 -> 7.57-7.82 ms
        // per sweep, r06s3 -- the halves unchanged, the replay slower than the eager launches;
        // removed, profiles/r06/ab/r06s3_sweep_graph.patch)
        {
        // ---- 4. item half-sweep
        if (!ref && !staged)
            HIPCHK(launch_philox_fill<T>(c->d_zV.as<T>(), K, c->items.r0, c->items.r1, cf.seed, c->sweep, TAG_ITEMS, st));
        if (c->bias)  // per-item (:492-511, :563-578)
            HIPCHK(launch_bias_rows<T>(c->d_vptr.as<uint32_t>(), c->items.r0, c->items.r1, c->d_Ev.as<T>(),
                                       c->d_bv.as<double>(), c->d_mbv.as<double>(), c->d_sbv.as<double>(),
                                       ref ? c->d_var3v.as<double>() : nullptr, bias_args(c, false, 0.0), st));
        // fresh V (and b_j) blocks and the per-row sums (one RCCL group), then the residuals.  One
        // rank: the half starts from the user half's end event (ev[2], just recorded)
        run_half_pipelined<T>(c, false, [&](uint32_t p) {
            bcast_stage(c, c->items, p, c->d_V.p, c->Kp * sizeof(T));
            if (c->bias) bcast_stage(c, c->items, p, c->d_bv.p, sizeof(double));
            bcast_stage(c, c->items, p, c->d_rowsq_v.p, sizeof(double));
            if (cf.eval_train) bcast_stage(c, c->items, p, c->d_rowtr_v.p, sizeof(double));
        }, c->nranks == 1 && staged && !c->bias ? c->ev[2] : nullptr);
        if (c->nranks > 1) HIPCHK(hipEventRecord(c->ev[5], st));
        // ---- 5. evaluation, and (overlap) the next sweep's prologue kernels.  One rank: the
        // evaluation runs on the second stream beside the prologue kernels -- both only read
        // U and V and they write different result slots, so nothing changes -- where it used
        // to follow them (tune bit 28 restores that order; measured 7.64-7.73 -> 7.61 ms, r04s22)
        auto evaluate = [&](hipStream_t se) {
            if (cf.eval_test && T_) {
                HIPCHK(launch_test<T>(c->d_tu.as<uint32_t>(), c->d_ti.as<uint32_t>(), c->d_tr.as<double>(), c->t0,
                                      c->t1, c->d_U.as<T>(), c->d_V.as<T>(), K, c->Kp, (T)c->lo, (T)c->hi,
                                      collect ? 1 : 0, div, c->d_tsum.as<double>(), c->d_tpart.as<double>(),
                                      c->bias ? c->d_bu.as<double>() : nullptr, c->d_bv.as<double>(), c->b0, se));
                if (c->nranks > 1) c->comm->bcast_ranges(c->d_tpart.p, 2 * sizeof(double), c->tbblocks, se);
                const uint32_t nb = (uint32_t)((T_ + 255) / 256);
                HIPCHK(launch_sum_cols(c->d_tpart.as<double>(), nb, 2, d_res + RES_TEST_AVG, se));
            }
            if (cf.eval_train)
                HIPCHK(launch_sum(c->d_rowtr_v.as<double>(), c->J, d_res + RES_TRSQ, scratch + c->scratch_half, se));
            HIPCHK(hipEventRecord(c->ev[6], se));
        };
        if (par_eval) {
            HIPCHK(hipStreamWaitEvent(c->sto, ev5, 0));
            evaluate(c->sto);
        }
        if (overlap) {  // the next sweep's prologue kernels, ahead of the evaluation
            prologue_gpu(c->sweep + 1, true);
            HIPCHK(hipEventRecord(c->ev[7], st));  // the host draws from here on
            // and the next sweep's normals, both tables in one launch (Philox: a function of (seed,
            // sweep) only; this sweep's halves, which read them, are queued before)
            HIPCHK(launch_philox_fill2<T>(c->d_zU.as<T>(), c->users.r0, c->users.r1, TAG_USERS, c->d_zV.as<T>(),
                                          c->items.r0, c->items.r1, TAG_ITEMS, K, cf.seed, c->sweep + 1, st));
            HIPCHK(hipEventRecord(c->ev[8], st));  // the next sweep's start work ends here
        }
        if (par_eval)
            HIPCHK(hipStreamWaitEvent(st, c->ev[6], 0));
        else
            evaluate(st);
        // the results, with the split-row timeout flag in the same copy (one copy less per sweep;
        // the prologue's sums go to the host ahead of them, so the host draws while the
        // evaluation and the normals run: one copy of everything after them put the host round
        // trip on the path, ML-1M 0.40 -> 0.43 ms, r06s11)
        HIPCHK(hipMemcpyAsync(c->h_out(), d_res, 8 * sizeof(double), hipMemcpyDeviceToHost, st));
        HIPCHK(hipEventRecord(c->ev[9], st));  // this sweep's device work ends here
        }
        if (overlap) {  // the next sweep's draws from the copied sums; this sweep's values kept
            HIPCHK(hipEventSynchronize(c->ev[7]));
            HostStream hs;
            PhiloxStream ps(cf.seed, c->sweep + 1, 0);
            draw_hyper_variates(ps, c, hs);
            const double tau0 = c->tau, b00 = c->b0, mb00 = c->mu_b0, sb00 = c->sig_b0;
            std::vector<double> su0 = c->sig_u, mu0 = c->mu_u, sv0 = c->sig_v, mv0 = c->mu_v;
            c->pre.d0 = host_draw(hs);
            c->pre.tau = c->tau;
            c->pre.b0 = c->b0;
            c->pre.mu_b0 = c->mu_b0;
            c->pre.sig_b0 = c->sig_b0;
            c->pre.sig_u.swap(c->sig_u);
            c->pre.mu_u.swap(c->mu_u);
            c->pre.sig_v.swap(c->sig_v);
            c->pre.mu_v.swap(c->mu_v);
            c->tau = tau0;
            c->b0 = b00;
            c->mu_b0 = mb00;
            c->sig_b0 = sb00;
            c->sig_u.swap(su0);
            c->mu_u.swap(mu0);
            c->sig_v.swap(sv0);
            c->mu_v.swap(mv0);
            c->pre.sweep = c->sweep + 1;
            c->pre.valid = true;
            // the next sweep's hyperparameters to the device now (every launch of this sweep that
            // reads d_hyper -- the halves and the prologue's column statistics -- is queued before)
            stage_hyper(c->pre.sig_u, c->pre.mu_u, c->pre.sig_v, c->pre.mu_v);
            c->pre.staged = true;
            c->hyper_ahead = true;
        }
        // ---- 6. the report.  With the overlap the host is past ev[7]: every event up to the item
        // half's end is done, so the half and launch-kind times are read first; cfg.pipeline then
        // queues the next sweep's start (which records those events again) before the host waits
        // for this sweep's results (ev[9]) and runs the callback
        const uint32_t s_cur = c->sweep;
        if (!overlap) HIPCHK(hipEventSynchronize(c->ev[9]));
        sbmf_sweep_info info{};
        info.sweep = s_cur;
        info.collected = collect ? 1u : 0u;
        info.tau = c->tau;
        const double ms_start = staged ? 0.0 : ev_ms(c->ev[0], ev1);
        c->timing.ms_user_half = ev_ms(ev1, c->ev[2]);
        c->timing.ms_item_half = ev_ms(ev3, c->ev[4]);
        c->timing.ms_comm = c->nranks > 1 ? ev_ms(c->ev[2], c->ev[3]) + ev_ms(c->ev[4], c->ev[5]) : 0.0;
        for (int sd = 0; sd < 2; ++sd) {
            const Side& sdd = sd == 0 ? c->users : c->items;
            for (int k = 0; k < SBMF_NKIND; ++k) {
                if (!c->time_kinds && k != KIND_STREAM) continue;  // kept from the run's first sweep
                double ms = 0.0;
                for (uint32_t p = 0; p < c->nstages; ++p) {
                    const Side::Stage& g = *sdd.stg[p];
                    const bool ran = k < NBIN && !g.bin_rows[k].empty();
                    const int kp = ran ? c->kpv(p, sd, k) : -1;
                    if (ran) ms += ev_ms(kp >= 0 ? c->kev(p, sd, kp, 1) : c->kbg(p, sd, k), c->kev(p, sd, k, 1));
                }
                c->timing.kern_ms[sd][k] = ms;
            }
        }
        info.ms_sweep = ev_ms(c->ev[0], ev5);
        c->sweep++;
        if (overlap && cf.pipeline && it + 1 < nsweeps && !c->kprof && !stop_after) {
            const uint32_t nl = c->timing.n_launch;
            q_staged = start_sweep(false);
            queued = true;
            c->timing.n_launch = nl;  // (this sweep's count in its report; the next start's is redone)
        }
        if (overlap) HIPCHK(hipEventSynchronize(c->ev[9]));  // this sweep's results (not the upload after them)
        const double* res8 = c->h_out();
        std::copy(res8, res8 + 8, c->h_res.begin());
        uint32_t split_timeout;
        std::memcpy(&split_timeout, res8 + RES_TIMEOUT, sizeof(split_timeout));
        if (c->kprof) {
            unsigned long long h[96];
            HIPCHK(hipMemcpy(h, c->d_kprof.p, sizeof(h), hipMemcpyDeviceToHost));
            HIPCHK(hipMemset(c->d_kprof.p, 0, sizeof(h)));
            static const char* gn[7] = {"setup", "load+mfma", "barrier", "reduce", "solve+handoff", "e-update",
                                        "epilogue"};
            for (int sd = 0; sd < 2; ++sd) {
                double tot = 0;
                for (int k = 0; k < 7; ++k) tot += (double)h[16 + 8 * sd + k];
                if (tot == 0) continue;
                std::fprintf(stderr, "[kprof] sweep %u %s gblock multi-wave rows (wave-0 Gcycles total):", s_cur,
                             sd ? "items" : "users");
                for (int k = 0; k < 7; ++k)
                    std::fprintf(stderr, " %s %.3f (%.0f%%)", gn[k], (double)h[16 + 8 * sd + k] / 1e9,
                                 100.0 * (double)h[16 + 8 * sd + k] / tot);
                std::fprintf(stderr, "\n");
            }
            static const char* nm[7] = {"stage", "apply+issue", "gather+acc", "wg-wait", "xwave+xchg", "solve", "epilogue"};
            for (int sd = 0; sd < 2; ++sd) {
                const Side& S = sd ? c->items : c->users;
                double tot = 0;
                for (int k = 0; k < 7; ++k) tot += (double)h[8 * sd + k];
                if (tot == 0) continue;
                std::fprintf(stderr, "[kprof] sweep %u gres %s (grid %u, %zu tasks, wave-0 Mcycles per WG):", s_cur,
                             sd ? "items" : "users", S.stg[0]->ss[c->kprof_set].sgrid,
                             S.stg[0]->ss[c->kprof_set].stasks.size());
                for (int k = 0; k < 7; ++k)
                    std::fprintf(stderr, " %s %.3f (%.0f%%)", nm[k], (double)h[8 * sd + k] / S.stg[0]->ss[c->kprof_set].sgrid / 1e6,
                                 100.0 * (double)h[8 * sd + k] / tot);
                std::fprintf(stderr, "\n");
                static const char* cn[3] = {"whole rows", "2-16 chunks", ">16 chunks"};
                for (int cl = 0; cl < 3; ++cl) {
                    const unsigned long long* hc = h + 32 + 24 * sd + 8 * cl;
                    if (!hc[7]) continue;
                    std::fprintf(stderr, "[kprof]   %s: %llu tasks, kcycles per task:", cn[cl], hc[7]);
                    for (int k = 0; k < 7; ++k) std::fprintf(stderr, " %s %.1f", nm[k], (double)hc[k] / hc[7] / 1e3);
                    std::fprintf(stderr, "\n");
                }
            }
        }
        if (split_timeout)  // a bounded spin in k_gres gave up: the sweep's results are not valid
            fail(SBMF_E_STATE, "sweep %u: split-row hand-off timed out (workgroups not co-resident)", s_cur);
        info.rmse_avg = (cf.eval_test && T_) ? std::sqrt(c->h_res[RES_TEST_AVG] / T_) : NAN;
        info.rmse_this = (cf.eval_test && T_) ? std::sqrt(c->h_res[RES_TEST_THIS] / T_) : NAN;
        info.rmse_train = cf.eval_train && N ? std::sqrt(c->h_res[RES_TRSQ] / N) : NAN;
        // with the overlap the next sweep's start work -- the prologue's kernels and both
        // tables' normals -- runs between ev[5] and ev[8], counted here
        c->timing.ms_hyper = ms_start + (overlap ? ev_ms(ev5, c->ev[8]) : 0.0);
        c->timing.ms_eval = overlap && !par_eval ? ev_ms(c->ev[8], c->ev[6]) : ev_ms(ev5, c->ev[6]);
        info.ms_eval = c->timing.ms_eval;
        if (cb && cb(&info, user)) {
            if (!queued) break;
            stop_after = true;  // the next sweep's start is queued: it completes, then the run stops
        } else if (stop_after) {
            break;
        }
    }
}

}  // namespace sbmf

// ===================================================================== C ABI
sbmf_ctx::~sbmf_ctx() {
    vbo_destroy(vb);
    fmm_destroy(fm);
    using namespace sbmf;
    pinned_free(h_pinned, h_pinned_bytes);
    pinned_free(h_pre, h_pre_bytes);
    pinned_free(h_io, h_io_bytes);
    for (hipEvent_t& e : ev) event_destroy(e);
    for (hipEvent_t& e : kevs) event_destroy(e);
    for (hipEvent_t& e : sev) event_destroy(e);
    for (hipEvent_t& e : tsev) event_destroy(e);
    for (hipEvent_t& e : cev) event_destroy(e);
    for (hipEvent_t& e : oev) event_destroy(e);
    event_destroy(hev);
    stream_destroy(sto);
    stream_destroy(sto2);
    stream_destroy(stc);
    stream_destroy(st);
    audit().contexts--;
}

namespace sbmf {
// sbmf_test_rccl_selftest: the exchange's RCCL calls through Comm's dlsym table on
// a one-rank communicator, issued on the comm stream while the item half's
// persistent k_gres grids (and its Gram-block launches) run on the compute
// streams -- the situation of the pipelined multi-GPU half (stage p's exchange
// beside stage p+1's compute), minus the peers.  Per repetition, one RCCL group of
// three in-place ncclBroadcast calls over adjacent blocks of a patterned buffer
// (as bcast_stage issues for U, the biases and the row sums), then the grouped
// ncclSend / ncclRecv of alltoallv (here to the rank itself), then an
// ncclAllGather.  Every byte is checked afterwards; the comm stream must finish
// within the deadline.
template <typename T>
void rccl_selftest(sbmf_ctx* c, uint64_t nbytes, uint32_t reps, double deadline_s, sbmf_rccl_selftest* out) {
    *out = sbmf_rccl_selftest{};
    Comm loop;
    loop.init_loopback();
    const size_t n = (size_t)nbytes, nag = n / 4;
    std::vector<uint8_t> pa(n), pb(n), pc(nag);
    for (size_t x = 0; x < n; ++x) {
        pa[x] = (uint8_t)(x * 2654435761u >> 13);
        pb[x] = (uint8_t)(x * 40503u + 17u);
    }
    for (size_t x = 0; x < nag; ++x) pc[x] = (uint8_t)(x * 97u + 5u);
    DBuf blk, snd, rcv, ags, agr;
    blk.alloc(n);
    snd.alloc(n);
    rcv.alloc(n);
    ags.alloc(nag);
    agr.alloc(nag);
    HIPCHK(hipMemcpy(blk.p, pa.data(), n, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(snd.p, pb.data(), n, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(ags.p, pc.data(), nag, hipMemcpyHostToDevice));
    HIPCHK(hipDeviceSynchronize());
    struct Events {  // destroyed on every path but a timeout (below)
        hipEvent_t e[4] = {};
        bool keep = false;
        ~Events() {
            if (!keep)
                for (hipEvent_t& x : e) event_destroy(x);
        }
    } evs;
    hipEvent_t* e = evs.e;
    for (int x = 0; x < 4; ++x) event_create(&e[x]);
    // three adjacent blocks of blk; the p2p segments [0, n/2) -> [n/2, n) and [n/2, n) -> [0, n/2)
    const std::vector<uint64_t> b0{0}, b1{n / 3}, b2{2 * (n / 3)}, b3{n};
    const std::vector<size_t> soff{0}, scnt{n / 2}, roff{n / 2}, rcnt{n / 2};
    const std::vector<size_t> soff2{n / 2}, scnt2{n / 2}, roff2{0}, rcnt2{n / 2};
    HIPCHK(hipEventRecord(e[0], c->st));
    for (uint32_t r = 0; r < reps; ++r) {
        run_half<T>(c, false, 0);  // the item half: persistent k_gres grids on st (+ sto)
        if (r == 0) HIPCHK(hipEventRecord(e[2], c->stc));
        loop.group_begin();
        loop.bcast_blocks(blk.p, 1, b0, b1, c->stc);
        loop.bcast_blocks(blk.p, 1, b1, b2, c->stc);
        loop.bcast_blocks(blk.p, 1, b2, b3, c->stc);
        loop.group_end();
        loop.alltoallv(snd.p, r & 1 ? soff2 : soff, r & 1 ? scnt2 : scnt, rcv.p, r & 1 ? roff2 : roff,
                       r & 1 ? rcnt2 : rcnt, c->stc);
        loop.allgather(ags.p, nag, agr.p, c->stc);
        out->n_calls += 3 + 2 + 1;
    }
    HIPCHK(hipEventRecord(e[1], c->st));
    HIPCHK(hipEventRecord(e[3], c->stc));
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t q = hipEventQuery(e[3]);
        if (q == hipSuccess) break;
        if (q != hipErrorNotReady) fail(SBMF_E_COMM, "RCCL self-test: %s", hipGetErrorString(q));
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > deadline_s) {
            // RCCL work is still queued on stc: abort the communicator instead of
            // destroying it, and leave the buffers and events in place (freeing them
            // would wait on the stuck stream); the context is dead from here on
            loop.abort();
            evs.keep = true;
            for (DBuf* b : {&blk, &snd, &rcv, &ags, &agr}) b->leak();
            c->dead = true;
            fail(SBMF_E_COMM, "RCCL self-test: the comm stream did not finish within %.1f s (communicator aborted, "
                              "context unusable)", deadline_s);
        }
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    HIPCHK(hipEventSynchronize(e[1]));
    float f = 0.f;
    HIPCHK(hipEventElapsedTime(&f, e[0], e[1]));
    out->ms_half = f;
    HIPCHK(hipEventElapsedTime(&f, e[2], e[3]));
    out->ms_rccl = f;
    HIPCHK(hipEventElapsedTime(&f, e[0], e[3]));
    out->ms_rccl_end = f;
    std::vector<uint8_t> h(n);
    HIPCHK(hipMemcpy(h.data(), blk.p, n, hipMemcpyDeviceToHost));
    for (size_t x = 0; x < n; ++x) out->bad_bcast += h[x] != pa[x];
    HIPCHK(hipMemcpy(h.data(), rcv.p, n, hipMemcpyDeviceToHost));
    // even repetitions send snd[0, n/2) to rcv[n/2, n), odd ones snd[n/2, n) to rcv[0, n/2)
    for (size_t x = 0; x < n; ++x) {
        if (x < n / 2 && reps == 1) continue;  // never written
        out->bad_p2p += h[x] != pb[x < n / 2 ? x + n / 2 : x - n / 2];
    }
    h.resize(nag);
    HIPCHK(hipMemcpy(h.data(), agr.p, nag, hipMemcpyDeviceToHost));
    for (size_t x = 0; x < nag; ++x) out->bad_allgather += h[x] != pc[x];
    out->overlapped = out->ms_rccl_end < out->ms_half ? 1u : 0u;
}
}  // namespace sbmf

#define API_BEGIN try {
#define API_END(ctx)                                  \
    }                                                 \
    catch (const sbmf::Error& e) {                    \
        g_err = e.msg;                                \
        if (ctx) (ctx)->err = e.msg;                  \
        return e.code;                                \
    }                                                 \
    catch (const std::bad_alloc&) {                   \
        g_err = "host allocation failed";             \
        if (ctx) (ctx)->err = g_err;                  \
        return SBMF_E_NOMEM;                          \
    }                                                 \
    catch (const std::exception& e) {                 \
        g_err = e.what();                             \
        if (ctx) (ctx)->err = g_err;                  \
        return SBMF_E_ARG;                            \
    }                                                 \
    return SBMF_OK;

extern "C" {

int sbmf_abi_version(void) { return SBMF_ABI_VERSION; }

namespace {
int g_exit_rc = 1;
bool g_exit_guarded = false;
void exit_guard_handler() {
    std::fflush(nullptr);
    std::_Exit(g_exit_rc);
}
}  // namespace
int sbmf_exit_guard(int rc) {
    g_exit_rc = rc;
    if (g_exit_guarded) return SBMF_OK;
    if (std::atexit(exit_guard_handler) != 0) {
        g_err = "sbmf_exit_guard: atexit failed";
        return SBMF_E_STATE;
    }
    g_exit_guarded = true;
    return SBMF_OK;
}

int sbmf_config_default(sbmf_config* c) {
    if (!c) return SBMF_E_ARG;
    std::memset(c, 0, sizeof *c);
    c->num_factor = 20;  // gibbs_sbpmf_final.cpp:218
    c->num_iter = 100;   // :299
    c->burnin = 0;       // :300
    c->seed = 1;         // glibc default seed (the sampler never calls srand)
    c->rng_mode = SBMF_RNG_REFERENCE;
    c->quirks = SBMF_QUIRKS_FINAL;
    c->precision = SBMF_F64;
    c->device = 0;
    c->init_stdev = -1.0;
    c->clamp_lo = -1.0;
    c->clamp_hi = 5.0;
    c->a0 = 1;
    c->b0 = 1;
    c->alpha0 = 1;
    c->beta0 = 1;
    c->nu0 = 1;
    c->mu0 = 0.0;
    c->recompute_every = 1;
    c->eval_train = 0;
    c->eval_test = 1;
    c->libfm_dim = 3;  // libfm.cpp:130 default -dim 1,1,8
    return SBMF_OK;
}

const char* sbmf_last_error(const sbmf_ctx* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }
const char* sbmf_last_global_error(void) { return g_err.c_str(); }

int sbmf_create(const sbmf_config* cfg, sbmf_ctx** out) {
    sbmf_ctx* ctx = nullptr;
    API_BEGIN
    if (!cfg || !out) sbmf::fail(SBMF_E_ARG, "null argument");
    *out = nullptr;
    if (cfg->num_factor == 0 || cfg->num_factor > 256) sbmf::fail(SBMF_E_ARG, "num_factor must be in [1,256]");
    if (cfg->rng_mode != SBMF_RNG_REFERENCE && cfg->rng_mode != SBMF_RNG_PHILOX) sbmf::fail(SBMF_E_ARG, "bad rng_mode");
    if (cfg->quirks < 0 || cfg->quirks > 4) sbmf::fail(SBMF_E_ARG, "bad quirks");
    if (cfg->average > 2) sbmf::fail(SBMF_E_ARG, "bad average (0 default, 1 collected sweeps, 2 sweep + 1)");
    if (cfg->precision != SBMF_F64 && cfg->precision != SBMF_F32) sbmf::fail(SBMF_E_ARG, "bad precision");
    if (cfg->method > SBMF_METHOD_ALS) sbmf::fail(SBMF_E_ARG, "bad method");
    if (cfg->method == SBMF_METHOD_VB && cfg->precision != SBMF_F64)
        sbmf::fail(SBMF_E_ARG, "the online VB learner computes in f64 (the reference's double) only");
    if ((cfg->method == SBMF_METHOD_LIBFM_MCMC || cfg->method == SBMF_METHOD_ALS) && cfg->precision != SBMF_F64)
        sbmf::fail(SBMF_E_ARG, "the libFM MCMC / ALS learner computes in f64 (the reference's double) only");
    if (cfg->libfm_dim > 3) sbmf::fail(SBMF_E_ARG, "bad libfm_dim (bit 0 = w0, bit 1 = w)");
    {
        // the tune bits with a meaning in this build (include/sbmf.h); a bit of a removed variant
        // is refused, so a value saved for an older build does not silently pick something else
        // (INTEGRATION.md lists what changed between rounds)
        constexpr uint32_t known = (1u << 1) | (1u << 2) | (1u << 3) | (1u << 7) | (1u << 8) | (1u << 9) | (1u << 10) |
                                   (1u << 11) | (1u << 12) | (1u << 13) | (1u << 14) | (1u << 17) |
                                   (1u << 23) | (1u << 24) | (1u << 25) | (1u << 26) | (1u << 27) | (1u << 28) |
                                   (1u << 29) | (1u << 30);
        if (cfg->tune & ~known)
            sbmf::fail(SBMF_E_ARG, "tune bits 0x%x have no meaning in this build (variants removed earlier; see "
                                   "include/sbmf.h and INTEGRATION.md)", cfg->tune & ~known);
    }
    if (cfg->gram_threshold || cfg->row_kernel)
        sbmf::fail(SBMF_E_ARG, "gram_threshold / row_kernel are reserved (must be 0): the per-coordinate and "
                               "full-Gram row kernels were removed (measured slower than the Gram-block kernels)");
    int ndev = 0;
    const hipError_t derr = hipGetDeviceCount(&ndev);
    if (derr != hipSuccess || ndev <= 0)
        sbmf::fail(SBMF_E_DEVICE, "no HIP device available (%s; this library has no CPU fallback)",
                   derr != hipSuccess ? hipGetErrorString(derr) : "0 devices");
    if (cfg->device < 0 || cfg->device >= ndev) sbmf::fail(SBMF_E_DEVICE, "device %d out of range (%d)", cfg->device, ndev);
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, cfg->device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        sbmf::fail(SBMF_E_DEVICE, "device %d is %s; this build targets gfx950 (MI355X)", cfg->device, prop.gcnArchName);
    HIPCHK(hipSetDevice(cfg->device));
    std::unique_ptr<sbmf_ctx> c(new sbmf_ctx());
    c->cfg = *cfg;
    // init 0.1 / clamp 0.5: src/libfm/gibbs_sbpmf2.cpp:240,557 and the top-level gibbs_sbpmf2.cpp:242,628
    const bool q2 = cfg->quirks == SBMF_QUIRKS_SBPMF2 || cfg->quirks == SBMF_QUIRKS_BIAS2;
    c->bias = cfg->quirks == SBMF_QUIRKS_BIAS2 || cfg->quirks == SBMF_QUIRKS_BIAS22;
    if (c->bias && (cfg->tune & 2u))
        sbmf::fail(SBMF_E_ARG, "tune bit 1 (residuals from r - own.partner) does not carry biases");
    c->init_sd = cfg->init_stdev >= 0 ? cfg->init_stdev : (q2 ? 0.1 : 1.0);
    c->lo = cfg->clamp_lo >= 0 ? cfg->clamp_lo : (q2 ? 0.5 : 1.0);
    c->hi = cfg->clamp_hi;
    c->sd_is_var = cfg->quirks == SBMF_QUIRKS_NONE ? 0 : 1;
    sbmf::stream_create(&c->st);
    sbmf::stream_create(&c->stc);
    for (auto& e : c->ev) sbmf::event_create(&e);
    for (auto& e : c->cev) sbmf::event_create(&e, hipEventDisableTiming);
    sbmf::stream_create(&c->sto);
    sbmf::stream_create(&c->sto2);
    for (auto& e : c->oev) sbmf::event_create(&e, hipEventDisableTiming);
    sbmf::event_create(&c->hev, hipEventDisableTiming);
    *out = c.release();
    API_END(ctx)
}

void sbmf_destroy(sbmf_ctx* ctx) {
    if (!ctx || ctx->dead) return;  // dead: work may still be queued (see sbmf_ctx::dead); leaked
    (void)hipSetDevice(ctx->cfg.device);
    (void)hipStreamSynchronize(ctx->st);
    delete ctx;
}

// -method vb: dims as for the sampler (max id + 1 over train and test)
static void prepare_vb(sbmf_ctx* c) {
    uint32_t umax = 0, imax = 0;
    for (size_t x = 0; x < c->tu.size(); ++x) {
        umax = std::max(umax, c->tu[x]);
        imax = std::max(imax, c->ti[x]);
    }
    for (size_t x = 0; x < c->su.size(); ++x) {
        umax = std::max(umax, c->su[x]);
        imax = std::max(imax, c->si[x]);
    }
    c->I = std::max(c->I_req, umax + 1);
    c->J = std::max(c->J_req, imax + 1);
    c->K = c->cfg.num_factor;
    c->vb = vbo_create(c->cfg, c->tu.size(), c->tu.data(), c->ti.data(), c->tr.data(), c->su.size(), c->su.data(),
                       c->si.data(), c->sr.data(), c->I, c->J, c->st, c->nranks > 1 ? c->comm : nullptr);
    c->prepared = true;
}

static bool is_fmm(const sbmf_ctx* c) {
    return c->cfg.method == SBMF_METHOD_LIBFM_MCMC || c->cfg.method == SBMF_METHOD_ALS;
}

// -method mcmc --order libfm / als: I (the item attribute offset of the
// users-first layout) and J as for the sampler (max id + 1 over train and
// test, or sbmf_set_dims)
static void prepare_fmm(sbmf_ctx* c) {
    uint32_t umax = 0, imax = 0;
    for (size_t x = 0; x < c->tu.size(); ++x) {
        umax = std::max(umax, c->tu[x]);
        imax = std::max(imax, c->ti[x]);
    }
    for (size_t x = 0; x < c->su.size(); ++x) {
        umax = std::max(umax, c->su[x]);
        imax = std::max(imax, c->si[x]);
    }
    c->I = std::max(c->I_req, umax + 1);
    c->J = std::max(c->J_req, imax + 1);
    c->K = c->cfg.num_factor;
    c->fm = fmm_create(c->cfg, c->tu.size(), c->tu.data(), c->ti.data(), c->tr.data(), c->su.size(), c->su.data(),
                       c->si.data(), c->sr.data(), c->I, c->J, c->st, c->nranks > 1 ? c->comm : nullptr);
    c->prepared = true;
}

static void set_triples(uint64_t n, const uint32_t* u, const uint32_t* i, const double* r, std::vector<uint32_t>& U,
                        std::vector<uint32_t>& I, std::vector<double>& R) {
    if (n && (!u || !i || !r)) sbmf::fail(SBMF_E_ARG, "null array with n > 0");
    U.assign(u, u + n);
    I.assign(i, i + n);
    R.assign(r, r + n);
}

int sbmf_set_train(sbmf_ctx* ctx, uint64_t n, const uint32_t* user, const uint32_t* item, const double* rating) {
    API_BEGIN
    if (!ctx) sbmf::fail(SBMF_E_ARG, "null context");
    if (ctx->prepared) sbmf::fail(SBMF_E_STATE, "data already prepared");
    set_triples(n, user, item, rating, ctx->tu, ctx->ti, ctx->tr);
    API_END(ctx)
}

int sbmf_set_test(sbmf_ctx* ctx, uint64_t n, const uint32_t* user, const uint32_t* item, const double* rating) {
    API_BEGIN
    if (!ctx) sbmf::fail(SBMF_E_ARG, "null context");
    if (ctx->prepared) sbmf::fail(SBMF_E_STATE, "data already prepared");
    set_triples(n, user, item, rating, ctx->su, ctx->si, ctx->sr);
    API_END(ctx)
}

int sbmf_set_dims(sbmf_ctx* ctx, uint32_t num_users, uint32_t num_items) {
    API_BEGIN
    if (!ctx) sbmf::fail(SBMF_E_ARG, "null context");
    if (ctx->prepared) sbmf::fail(SBMF_E_STATE, "data already prepared");
    ctx->I_req = num_users;
    ctx->J_req = num_items;
    API_END(ctx)
}

int sbmf_prepare(sbmf_ctx* ctx) {
    API_BEGIN
    if (!ctx) sbmf::fail(SBMF_E_ARG, "null context");
    HIPCHK(hipSetDevice(ctx->cfg.device));
    if (ctx->prepared) return SBMF_OK;
    if (ctx->tu.empty()) sbmf::fail(SBMF_E_STATE, "no training data (sbmf_set_train)");
    for (size_t x = 0; x < ctx->tu.size(); ++x)
        if ((ctx->I_req && ctx->tu[x] >= ctx->I_req) || (ctx->J_req && ctx->ti[x] >= ctx->J_req))
            sbmf::fail(SBMF_E_ARG, "rating %zu has an id beyond sbmf_set_dims", x);
    if (ctx->cfg.method == SBMF_METHOD_VB)
        prepare_vb(ctx);
    else if (is_fmm(ctx))
        prepare_fmm(ctx);
    else if (ctx->cfg.precision == SBMF_F32)
        prepare_T<float>(ctx);
    else
        prepare_T<double>(ctx);
    API_END(ctx)
}

int sbmf_run(sbmf_ctx* ctx, uint32_t sweeps, sbmf_sweep_cb cb, void* user) {
    API_BEGIN
    if (!ctx) sbmf::fail(SBMF_E_ARG, "null context");
    if (ctx->spent || ctx->dead)
        sbmf::fail(SBMF_E_STATE, "sbmf_test_rccl_selftest ran extra item halves on this context: its chain is no "
                                 "longer the sampler's; create a new context");
    HIPCHK(hipSetDevice(ctx->cfg.device));
    if (!ctx->prepared && ctx->cfg.method == SBMF_METHOD_VB) {
        if (ctx->tu.empty()) sbmf::fail(SBMF_E_STATE, "no training data (sbmf_set_train)");
        prepare_vb(ctx);
    }
    if (!ctx->prepared && is_fmm(ctx)) {
        if (ctx->tu.empty()) sbmf::fail(SBMF_E_STATE, "no training data (sbmf_set_train)");
        prepare_fmm(ctx);
    }
    if (ctx->vb) {
        vbo_run(ctx->vb, sweeps, cb, user);
        ctx->timing = sbmf_timing{};
        ctx->timing.n_launch = vbo_launches(ctx->vb);
        ctx->timing.ms_vb_factor = vbo_factor_ms(ctx->vb);
        return SBMF_OK;
    }
    if (ctx->fm) {
        fmm_run(ctx->fm, sweeps, cb, user);
        ctx->timing = sbmf_timing{};
        ctx->timing.n_launch = fmm_launches(ctx->fm);
        return SBMF_OK;
    }
    if (!ctx->prepared) {
        if (ctx->tu.empty()) sbmf::fail(SBMF_E_STATE, "no training data (sbmf_set_train)");
        if (ctx->cfg.precision == SBMF_F32)
            prepare_T<float>(ctx);
        else
            prepare_T<double>(ctx);
    }
    if (ctx->cfg.precision == SBMF_F32)
        run_sweeps_T<float>(ctx, sweeps, cb, user);
    else
        run_sweeps_T<double>(ctx, sweeps, cb, user);
    API_END(ctx)
}

int sbmf_predict(sbmf_ctx* ctx, double* out) {
    API_BEGIN
    if (!ctx || !out) sbmf::fail(SBMF_E_ARG, "null argument");
    if (!ctx->prepared) sbmf::fail(SBMF_E_STATE, "not prepared");
    HIPCHK(hipSetDevice(ctx->cfg.device));
    if (ctx->vb) {
        vbo_predict_out(ctx->vb, out);
        return SBMF_OK;
    }
    if (ctx->fm) {
        fmm_predict_out(ctx->fm, out);
        return SBMF_OK;
    }
    const uint64_t T_ = ctx->su.size();
    if (ctx->nranks > 1) ctx->comm->bcast_ranges(ctx->d_tsum.p, sizeof(double), ctx->tbounds, ctx->st);
    HIPCHK(hipStreamSynchronize(ctx->st));
    std::vector<double> h(T_);
    HIPCHK(hipMemcpy(h.data(), ctx->d_tsum.p, T_ * sizeof(double), hipMemcpyDeviceToHost));
    const double div = sbmf::avg_collected(ctx->cfg) ? (double)std::max(1u, ctx->collected) : (double)std::max(1u, ctx->sweep);
    for (uint64_t j = 0; j < T_; ++j) out[ctx->tperm[j]] = h[j] / div;  // device (user) order -> file order
    API_END(ctx)
}

int sbmf_get_factors(sbmf_ctx* ctx, double* U, double* V) {
    API_BEGIN
    if (!ctx) sbmf::fail(SBMF_E_ARG, "null context");
    if (!ctx->prepared) sbmf::fail(SBMF_E_STATE, "not prepared");
    HIPCHK(hipSetDevice(ctx->cfg.device));
    HIPCHK(hipStreamSynchronize(ctx->st));
    if (ctx->vb) {
        vbo_factors(ctx->vb, U, V);
        return SBMF_OK;
    }
    if (ctx->fm) {
        fmm_factors(ctx->fm, U, V);
        return SBMF_OK;
    }
    if (ctx->cfg.precision == SBMF_F32) {
        if (U) sbmf::download_table<float>(ctx, ctx->d_U, U, ctx->I);
        if (V) sbmf::download_table<float>(ctx, ctx->d_V, V, ctx->J);
    } else {
        if (U) sbmf::download_table<double>(ctx, ctx->d_U, U, ctx->I);
        if (V) sbmf::download_table<double>(ctx, ctx->d_V, V, ctx->J);
    }
    API_END(ctx)
}

int sbmf_set_factors(sbmf_ctx* ctx, const double* U, const double* V) {
    API_BEGIN
    if (!ctx) sbmf::fail(SBMF_E_ARG, "null context");
    if (!ctx->prepared) sbmf::fail(SBMF_E_STATE, "not prepared");
    if (ctx->vb || ctx->fm) sbmf::fail(SBMF_E_STATE, "sbmf_set_factors is not supported by the VB / libFM learners");
    HIPCHK(hipSetDevice(ctx->cfg.device));
    HIPCHK(hipStreamSynchronize(ctx->st));
    ctx->pre.valid = false;  // hyperparameters drawn ahead from the old tables
    if (ctx->cfg.precision == SBMF_F32) {
        if (U) sbmf::upload_table<float>(ctx, ctx->d_U, U, ctx->I);
        if (V) sbmf::upload_table<float>(ctx, ctx->d_V, V, ctx->J);
    } else {
        if (U) sbmf::upload_table<double>(ctx, ctx->d_U, U, ctx->I);
        if (V) sbmf::upload_table<double>(ctx, ctx->d_V, V, ctx->J);
    }
    API_END(ctx)
}

int sbmf_get_hyper(sbmf_ctx* ctx, double* h, double* tau) {
    API_BEGIN
    if (!ctx) sbmf::fail(SBMF_E_ARG, "null context");
    if (!ctx->prepared) sbmf::fail(SBMF_E_STATE, "not prepared");
    if (ctx->vb) {
        HIPCHK(hipSetDevice(ctx->cfg.device));
        vbo_hyper_out(ctx->vb, h, tau);
        return SBMF_OK;
    }
    if (ctx->fm) {
        fmm_hyper_out(ctx->fm, h, tau);
        return SBMF_OK;
    }
    const uint32_t K = ctx->K;
    if (h) {
        std::copy(ctx->sig_u.begin(), ctx->sig_u.end(), h);
        std::copy(ctx->mu_u.begin(), ctx->mu_u.end(), h + K);
        std::copy(ctx->sig_v.begin(), ctx->sig_v.end(), h + 2 * K);
        std::copy(ctx->mu_v.begin(), ctx->mu_v.end(), h + 3 * K);
    }
    if (tau) *tau = ctx->tau;
    API_END(ctx)
}

int sbmf_get_biases(sbmf_ctx* ctx, double* bu, double* bv, double* b0) {
    API_BEGIN
    if (!ctx) sbmf::fail(SBMF_E_ARG, "null context");
    if (!ctx->prepared) sbmf::fail(SBMF_E_STATE, "not prepared");
    HIPCHK(hipSetDevice(ctx->cfg.device));
    if (ctx->vb) {  // posterior means of w (users, items) and w0
        vbo_biases(ctx->vb, bu, bv, b0);
        return SBMF_OK;
    }
    if (ctx->fm) {  // libFM's w (users, items) and w0
        fmm_biases(ctx->fm, bu, bv, b0);
        return SBMF_OK;
    }
    if (!ctx->bias) sbmf::fail(SBMF_E_STATE, "not a biased sampler (quirks bias2 / bias22) or the VB learner");
    HIPCHK(hipStreamSynchronize(ctx->st));
    if (bu) HIPCHK(hipMemcpy(bu, ctx->d_bu.p, (size_t)ctx->I * sizeof(double), hipMemcpyDeviceToHost));
    if (bv) HIPCHK(hipMemcpy(bv, ctx->d_bv.p, (size_t)ctx->J * sizeof(double), hipMemcpyDeviceToHost));
    if (b0) *b0 = ctx->b0;
    API_END(ctx)
}

int sbmf_get_dims(sbmf_ctx* ctx, uint32_t* nu, uint32_t* ni, uint64_t* ntr, uint64_t* nte) {
    API_BEGIN
    if (!ctx) sbmf::fail(SBMF_E_ARG, "null context");
    if (nu) *nu = ctx->I;
    if (ni) *ni = ctx->J;
    if (ntr) *ntr = ctx->tu.size();
    if (nte) *nte = ctx->su.size();
    API_END(ctx)
}

int sbmf_get_timing(sbmf_ctx* ctx, sbmf_timing* t) {
    API_BEGIN
    if (!ctx || !t) sbmf::fail(SBMF_E_ARG, "null argument");
    *t = ctx->timing;
    // per sweep, both halves: N*(sK + 4 + 4) + rows*2*sK
    const uint64_t s = sbmf::tsize(ctx);
    const uint64_t N = ctx->tu.size();
    t->bytes_algorithmic = 2 * N * (s * ctx->K + 4 + s) + ((uint64_t)ctx->I + ctx->J) * 2 * s * ctx->K;
    API_END(ctx)
}

int sbmf_comm_unique_id(uint8_t id[128]) {
    sbmf_ctx* ctx = nullptr;
    API_BEGIN
    if (!id) sbmf::fail(SBMF_E_ARG, "null id");
    sbmf::Comm::unique_id(id);
    API_END(ctx)
}

int sbmf_comm_init(sbmf_ctx* ctx, int nranks, int rank, const uint8_t id[128]) {
    API_BEGIN
    if (!ctx || !id) sbmf::fail(SBMF_E_ARG, "null argument");
    if (ctx->prepared) sbmf::fail(SBMF_E_STATE, "sbmf_comm_init must precede sbmf_prepare");
    if (nranks < 1 || rank < 0 || rank >= nranks) sbmf::fail(SBMF_E_ARG, "bad rank %d / %d", rank, nranks);
    HIPCHK(hipSetDevice(ctx->cfg.device));
    ctx->nranks = nranks;
    ctx->rank = rank;
    if (ctx->comm != &ctx->own_comm) sbmf::fail(SBMF_E_STATE, "context already attached to a communicator");
    if (nranks > 1) ctx->comm->init(nranks, rank, id);
    API_END(ctx)
}

// one communicator per process, shared by every context of the process (bench.py's
// legs): RCCL's set-up runs once, not once per learner
struct sbmf_comm {
    sbmf::Comm c;
    int device = 0, nranks = 1, rank = 0;
};

int sbmf_comm_create(int device, int nranks, int rank, const uint8_t id[128], sbmf_comm** out) {
    sbmf_ctx* ctx = nullptr;
    API_BEGIN
    if (!id || !out) sbmf::fail(SBMF_E_ARG, "null argument");
    *out = nullptr;
    if (nranks < 1 || rank < 0 || rank >= nranks) sbmf::fail(SBMF_E_ARG, "bad rank %d / %d", rank, nranks);
    if (device < 0) sbmf::fail(SBMF_E_ARG, "bad device %d", device);
    std::unique_ptr<sbmf_comm> cm(new sbmf_comm());
    cm->device = device;
    cm->nranks = nranks;
    cm->rank = rank;
    if (nranks > 1) {
        // RCCL binds the communicator to the current device: this rank's, set first
        HIPCHK(hipSetDevice(device));
        cm->c.init(nranks, rank, id);
    }
    *out = cm.release();
    API_END(ctx)
}

int sbmf_comm_attach(sbmf_ctx* ctx, sbmf_comm* comm) {
    API_BEGIN
    if (!ctx || !comm) sbmf::fail(SBMF_E_ARG, "null argument");
    if (ctx->prepared) sbmf::fail(SBMF_E_STATE, "sbmf_comm_attach must precede sbmf_prepare");
    if (ctx->own_comm.active() || ctx->virt) sbmf::fail(SBMF_E_STATE, "context already joined a communicator");
    if (comm->nranks > 1 && comm->device != ctx->cfg.device)
        sbmf::fail(SBMF_E_ARG, "communicator on device %d, context on device %d", comm->device, ctx->cfg.device);
    ctx->nranks = comm->nranks;
    ctx->rank = comm->rank;
    ctx->comm = &comm->c;
    API_END(ctx)
}

void sbmf_comm_destroy(sbmf_comm* comm) { delete comm; }

int sbmf_test_virtual_rank(sbmf_ctx* ctx, int nranks, int rank) {
    API_BEGIN
    if (!ctx) sbmf::fail(SBMF_E_ARG, "null context");
    if (ctx->prepared) sbmf::fail(SBMF_E_STATE, "sbmf_test_virtual_rank must precede sbmf_prepare");
    if (nranks < 2 || rank < 0 || rank >= nranks) sbmf::fail(SBMF_E_ARG, "bad rank %d / %d", rank, nranks);
    if (ctx->cfg.method != SBMF_METHOD_MCMC) sbmf::fail(SBMF_E_ARG, "virtual ranks: the SBPMF sampler only");
    if (ctx->comm->active() || ctx->comm != &ctx->own_comm)
        sbmf::fail(SBMF_E_STATE, "context already joined a communicator");
    ctx->nranks = nranks;
    ctx->rank = rank;
    ctx->virt = true;
    API_END(ctx)
}

int sbmf_test_stage_ms(sbmf_ctx* ctx, double* ms, uint32_t cap, uint32_t* nstages) {
    API_BEGIN
    if (!ctx || !nstages) sbmf::fail(SBMF_E_ARG, "null argument");
    if (!ctx->virt || !ctx->prepared) sbmf::fail(SBMF_E_STATE, "stage times need a prepared virtual rank");
    *nstages = ctx->nstages;
    if (ms && cap < 2 * ctx->nstages) sbmf::fail(SBMF_E_ARG, "need %u slots", 2 * ctx->nstages);
    HIPCHK(hipStreamSynchronize(ctx->st));
    for (uint32_t sd = 0; ms && sd < 2; ++sd)
        for (uint32_t p = 0; p < ctx->nstages; ++p) {
            float f = 0.f;
            const size_t tb = (size_t)sd * (ctx->nstages + 1);
            HIPCHK(hipEventElapsedTime(&f, ctx->tsev[tb + p], ctx->tsev[tb + p + 1]));
            ms[sd * ctx->nstages + p] = f;
        }
    API_END(ctx)
}

int sbmf_test_rccl_selftest(sbmf_ctx* ctx, uint64_t nbytes, uint32_t reps, double deadline_s,
                            sbmf_rccl_selftest* out) {
    API_BEGIN
    if (!ctx || !out) sbmf::fail(SBMF_E_ARG, "null argument");
    HIPCHK(hipSetDevice(ctx->cfg.device));
    if (!ctx->prepared || ctx->nranks != 1 || ctx->cfg.method != SBMF_METHOD_MCMC)
        sbmf::fail(SBMF_E_STATE, "the RCCL self-test needs a prepared one-rank sampler context");
    if (nbytes < 64 || nbytes % 64 || reps == 0) sbmf::fail(SBMF_E_ARG, "nbytes a positive multiple of 64, reps >= 1");
    if (ctx->spent || ctx->dead) sbmf::fail(SBMF_E_STATE, "the RCCL self-test already ran on this context");
    ctx->spent = true;  // from the first extra half on, the chain is not the sampler's
    if (ctx->cfg.precision == SBMF_F32)
        sbmf::rccl_selftest<float>(ctx, nbytes, reps, deadline_s, out);
    else
        sbmf::rccl_selftest<double>(ctx, nbytes, reps, deadline_s, out);
    API_END(ctx)
}

int sbmf_test_device_usage(int device, sbmf_device_usage* out) {
    sbmf_ctx* ctx = nullptr;
    API_BEGIN
    if (!out) sbmf::fail(SBMF_E_ARG, "null argument");
    *out = sbmf_device_usage{};
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        sbmf::fail(SBMF_E_DEVICE, "no HIP device %d", device);
    HIPCHK(hipSetDevice(device));
    size_t fr = 0, tot = 0;
    HIPCHK(hipMemGetInfo(&fr, &tot));
    out->device_free = fr;
    out->device_total = tot;
    const sbmf::Audit& a = sbmf::audit();
    out->dev_bytes = a.dev_bytes.load();
    out->dev_allocs = a.dev_allocs.load();
    out->pinned_bytes = a.pinned_bytes.load();
    out->pinned_allocs = a.pinned_allocs.load();
    out->streams = a.streams.load();
    out->events = a.events.load();
    out->contexts = a.contexts.load();
    out->comms = a.comms.load();
    API_END(ctx)
}

int sbmf_partition_rows(const uint32_t* ptr, uint32_t R, int nranks, uint64_t* bounds) {
    sbmf_ctx* ctx = nullptr;
    API_BEGIN
    if (!ptr || !bounds || nranks < 1) sbmf::fail(SBMF_E_ARG, "bad arguments");
    sbmf::partition_bounds(ptr, R, nranks, bounds);
    API_END(ctx)
}

int sbmf_ref_stream(uint32_t seed, int kind, double shape, uint64_t n, double* out) {
    sbmf_ctx* ctx = nullptr;
    API_BEGIN
    if (!out && n) sbmf::fail(SBMF_E_ARG, "null out");
    sbmf::GlibcRand g(seed);
    for (uint64_t x = 0; x < n; ++x) {
        if (kind == 0)
            out[x] = g.next();
        else if (kind == 1)
            out[x] = sbmf::leva_normal(g);
        else
            out[x] = sbmf::mt_gamma(g, shape);
    }
    API_END(ctx)
}

int sbmf_philox_normals(uint64_t seed, uint32_t sweep, uint32_t tag, uint32_t row, uint32_t K, double* out) {
    sbmf_ctx* ctx = nullptr;
    API_BEGIN
    if (!out && K) sbmf::fail(SBMF_E_ARG, "null out");
    for (uint32_t k = 0; k < K; k += 2) {
        double z0, z1;
        sbmf::philox_normal_pair(seed, row, sweep, tag, k / 2, z0, z1);
        out[k] = z0;
        if (k + 1 < K) out[k + 1] = z1;
    }
    API_END(ctx)
}

}  // extern "C"
