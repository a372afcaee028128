// vbo.cpp -- host side of the online variational-Bayes learner (`-method vb`):
// the reference's fm_learn_vb_online (src/libfm/src/fm_learn_vb_online.h,
// fm_learn_vb_online_simultaneous.h) on rating data.
//
// Per epoch (fm_learn_vb_online_simultaneous.h:58-447):
//   1. shuffle the 1-based case ids (libstdc++ random_shuffle over rand() in
//      reference RNG mode, the array kept across epochs; Fisher-Yates over
//      Philox otherwise); case l goes to batch ceil(id_l / ceil(N/30));
//   2. group every batch's cases by user and by item (host, O(N)) and upload;
//   3. per batch, on the device: e / t terms, update_w0, update_w (users,
//      items), update_v (per factor: users, items), hyperparameter blends;
//   4. test predictions of the means, clamped to the train target range.
// The reference writes each epoch's 30 batches to text files and parses them
// back (:148-203); here a batch is an index range in device memory.
//
// Several ranks (one process per GPU): rank k owns the users [u_k, u_k+1)
// (sbmf_partition_rows over the users' rating counts) and every case of those users, so
// user rows are local.  Every rank replays the same shuffle and keeps the
// item tables replicated: an item row of a batch is summed over the ranks --
// each rank writes its cases' {e1, e2} for the batch's items, an all-gather
// delivers every rank's sums, and every rank applies the same update (rank
// order) and forwards the deltas to its own cases.  update_w0's and the
// blends' sums are all-gathered per rank the same way.  One all-gather per
// item pass (2K + 4 per batch) and the owned user means broadcast once per
// epoch (test RMSE, factors).  Results agree with one rank to rounding (the
// item sums are added rank by rank), and are identical on every rank.
#include "vbo.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <memory>
#include <exception>
#include <thread>
#include <utility>
#include <vector>

#include "comm.h"
#include "common.h"
#include "rng.h"

namespace sbmf {

// One epoch's batch layout (host side), built by a worker thread while the
// GPU runs the previous epoch, and its device copy.
struct VBLayout {
    // per batch and orientation: rows stably sorted by lane-group size (records in row
    // order) and the 256-thread tasks over them (row0 relative to the batch's first row);
    // on the device every batch's rows and tasks at urow0[b] / utask0[b] (batch-major)
    struct Part {
        std::vector<VRow> rows;
        std::vector<VTask> tasks;
    };
    std::vector<Part> pu, pi;
    std::vector<uint32_t> urow0, irow0, utask0, itask0, bsize, bbase;
    std::vector<uint32_t> upart;  // [N] user order: the case's item attribute
    std::vector<uint2> iu;        // [N] item order: {user-grouped position, the user's batch row}
    std::vector<float> ur;                          // [N] target per user-order entry
    // several ranks: bsize / bbase count this rank's cases; gbsize the whole batch;
    // gitems the batch's items over all ranks (entries [gitem0[b], gitem0[b+1]))
    std::vector<uint32_t> gbsize, gitem0;
    std::vector<VGItem> gitems;
    DBuf d_urows, d_irows, d_utasks, d_itasks, d_upart, d_iu, d_ur, d_gitems;
};

struct VBLearner {
    sbmf_config cfg{};
    uint32_t K = 0, Kp = 0, I = 0, J = 0, p = 0, N = 0, NB = 30, S = 0;
    double lo = 1.0, hi = 5.0;
    uint32_t epoch = 0;
    GlibcRand grand{1};
    hipStream_t st = nullptr;
    hipEvent_t ev[4] = {};
    // host data
    std::vector<uint32_t> tu, ti, su, si;
    std::vector<double> tr, sr;
    std::vector<uint32_t> shuffle, bid;
    std::vector<uint32_t> btu, bti, bupos;  // the (own) cases batch-major, file order inside a batch
    std::vector<float> btr;
    VBLayout lay[2];                 // epoch e uses lay[e & 1]
    std::thread worker;              // builds and uploads lay[(e + 1) & 1] during epoch e
    std::exception_ptr worker_err;   // its failure, rethrown by run()
    int dev = 0;
    hipStream_t ust = nullptr;       // layout uploads (the worker's)
    hipEvent_t uev[2] = {}, done[2] = {};  // layout e & 1: uploaded / free again
    uint32_t built = 0;              // epochs whose layout exists (ready or being built)
    // device
    DBuf d_mu_v, d_sg_v, d_nm_v, d_ns_v, d_mu_w, d_sg_w, d_nm_w, d_ns_w, d_rho_w, d_rho_v, d_t_w, d_t_v, d_cc;
    DBuf d_sigma_v, d_scal, d_muT, d_sgT, d_E, d_T, d_part;
    DBuf d_D, d_VS;  // per item: the last item pass's pending deltas; per user: fresh {mean, variance} of f
    size_t part_cap = 0;  // doubles in d_part
    DBuf d_tu, d_ti, d_tr, d_pred, d_tpart;
    VBTables tb{};
    // several ranks
    Comm* comm = nullptr;
    int R = 1, rank = 0;
    uint32_t u0 = 0, u1 = 0, NL = 0;  // owned users [u0, u1), their cases (NL)
    std::vector<uint64_t> ubounds;     // [R + 1] user ranges of every rank
    std::vector<uint8_t> mine;         // [N] case belongs to an owned user
    uint32_t gmax = 0;                 // largest per-batch item count
    // one rank: item rows cut into XS slices by the partner case's user-grouped position
    // (equal case counts); slice x's tasks take blocks x, x + XS, ...,
    // i.e. XCD x under the round-robin block dispatch, so its gathers (e and the users'
    // {mean, variance}) stay inside 1/XS of the batch -- resident in that XCD's L2.
    // SBMF_VB_SLICES (default 8): 838 ms per Netflix-shaped K=200 epoch vs 1061 unsliced (r03r)
    uint32_t XS = 1;
    DBuf d_send, d_recv, d_sums, d_recvg;
    double last_rmse = NAN, last_alpha = NAN;
    double ms_layout = 0.0;
    uint32_t n_launch = 0;
    // [batch][begin, end]: each mini-batch's 2K factor passes (vbo_user_v / vbo_item_v), timed
    // with HIP events on the compute stream -- the epoch's dominant kernels (bench.py's roofline)
    std::vector<hipEvent_t> fev;
    double ms_factor_sum = 0.0;  // the last run's epochs: factor-pass time summed ...
    uint32_t n_factor_epochs = 0;  // ... over this many epochs

    ~VBLearner() {
        if (worker.joinable()) worker.join();
        for (auto& e : ev) event_destroy(e);
        for (auto& e : fev) event_destroy(e);
        for (hipEvent_t* e : {&uev[0], &uev[1], &done[0], &done[1]}) event_destroy(*e);
        stream_destroy(ust);
    }

    void init(const sbmf_config& c, uint64_t n, const uint32_t* u, const uint32_t* i, const double* r, uint64_t nt,
              const uint32_t* tu_, const uint32_t* ti_, const double* tr_, uint32_t I_, uint32_t J_, hipStream_t s,
              Comm* cm);
    void build_layout(VBLayout& L, uint32_t ep);
    void stage_layout(VBLayout& L, uint32_t e);
    void run(uint32_t epochs, sbmf_sweep_cb cb, void* user);
    void item_pass(const VBLayout& L, uint32_t b, const VTask* it_, uint32_t nit, const VRow* ir_, const uint2* iu_,
                   int factor, uint32_t f, VBCases ETu);
    void sync_users();
};

void VBLearner::init(const sbmf_config& c, uint64_t n, const uint32_t* u, const uint32_t* i, const double* r,
                     uint64_t nt, const uint32_t* tu_, const uint32_t* ti_, const double* tr_, uint32_t I_, uint32_t J_,
                     hipStream_t s, Comm* cm) {
    cfg = c;
    st = s;
    if (cm && cm->nranks() > 1) {
        comm = cm;
        R = cm->nranks();
        rank = cm->rank();
        // VGItem.mask holds one bit per rank's part (the combine kernels test bit r)
        if (R > 32) fail(SBMF_E_ARG, "online VB: at most 32 ranks (%d given)", R);
    }
    K = c.num_factor;
    Kp = (K + 15) / 16 * 16;
    I = I_;
    J = J_;
    p = I + J;  // user u -> u, item i -> I + i; num_attribute = largest id + 1 (libfm.cpp:328)
    N = (uint32_t)n;
    NB = c.vb_batches ? c.vb_batches : 30;  // fm_learn_vb_online_simultaneous.h:62
    S = (uint32_t)std::ceil((double)N / NB);
    if (N == 0 || (uint64_t)S * (NB - 1) >= N)
        fail(SBMF_E_ARG, "online VB: %u ratings leave a batch of %u empty (the reference divides by zero)", N, NB);
    tu.assign(u, u + n);
    ti.assign(i, i + n);
    tr.assign(r, r + n);
    su.assign(tu_, tu_ + nt);
    si.assign(ti_, ti_ + nt);
    sr.assign(tr_, tr_ + nt);
    // train target range as DATA_FLOAT (libfm.cpp:199-214, fm_learn min/max_target)
    float mn = 3.402823466e+38f, mx = -3.402823466e+38f;
    for (double x : tr) {
        mn = std::min(mn, (float)x);
        mx = std::max(mx, (float)x);
    }
    lo = mn;
    hi = mx;

    // ---- start state (libfm.cpp:387,433; fm_learn_vb_online.h:841-946; matrix.h:358-380)
    std::vector<double> mu_v((size_t)K * p), mu_w(p);
    if (c.rng_mode == SBMF_RNG_REFERENCE) {
        grand.seed_((unsigned)c.seed);
        for (size_t x = 0; x < (size_t)K * p + p; ++x) (void)leva_normal(grand);  // fm_model v, w
        for (uint32_t a = 0; a < p; ++a) mu_w[a] = 0.1 * leva_normal(grand);
        for (size_t x = 0; x < (size_t)K * p; ++x) mu_v[x] = 0.1 * leva_normal(grand);
    } else {
        PhiloxStream ps(c.seed, 0xfffffff0u, 5);
        for (uint32_t a = 0; a < p; ++a) mu_w[a] = 0.1 * leva_normal(ps);
        for (size_t x = 0; x < (size_t)K * p; ++x) mu_v[x] = 0.1 * leva_normal(ps);
    }
    std::vector<double> sg_v((size_t)K * p, .02), nm_v((size_t)K * p), ns_v((size_t)K * p, 1 / .02);
    std::vector<double> sg_w(p, .02), nm_w(p), ns_w(p, 1 / .02), ones(p, 1.0);
    for (size_t x = 0; x < (size_t)K * p; ++x) nm_v[x] = mu_v[x] / 0.02;
    for (uint32_t a = 0; a < p; ++a) nm_w[a] = mu_w[a] / 0.02;
    std::vector<uint32_t> cc(p, 0), zeros(p, 0);
    for (uint32_t x = 0; x < N; ++x) {  // column counts of the whole train set (:877-900)
        cc[tu[x]]++;
        cc[I + ti[x]]++;
    }
    // user ranges: the sampler's row partition (sbmf_partition_rows: contiguous,
    // rating-balanced, 256-aligned) over the users' rating counts
    ubounds.assign(R + 1, 0);
    {
        std::vector<uint32_t> uptr(I + 1, 0);
        for (uint32_t a = 0; a < I; ++a) uptr[a + 1] = uptr[a] + cc[a];
        if (sbmf_partition_rows(uptr.data(), I, R, ubounds.data()) != SBMF_OK)
            fail(SBMF_E_ARG, "online VB: user partition failed");
    }
    if (R == 1) {
        const char* xs = std::getenv("SBMF_VB_SLICES");
        XS = xs ? (uint32_t)std::min(32, std::max(1, std::atoi(xs))) : 8u;
    }
    u0 = (uint32_t)ubounds[rank];
    u1 = (uint32_t)ubounds[rank + 1];
    mine.assign(N, 1);
    NL = N;
    if (R > 1) {
        NL = 0;
        for (uint32_t x = 0; x < N; ++x) {
            mine[x] = tu[x] >= u0 && tu[x] < u1;
            NL += mine[x];
        }
    }
    upload(d_mu_v, mu_v, st);
    upload(d_sg_v, sg_v, st);
    upload(d_nm_v, nm_v, st);
    upload(d_ns_v, ns_v, st);
    upload(d_mu_w, mu_w, st);
    upload(d_sg_w, sg_w, st);
    upload(d_nm_w, nm_w, st);
    upload(d_ns_w, ns_w, st);
    upload(d_rho_w, ones, st);  // (t0 + 0)^-0.5 = 1
    upload(d_rho_v, ones, st);
    upload(d_t_w, zeros, st);
    upload(d_t_v, zeros, st);
    upload(d_cc, cc, st);
    upload(d_sigma_v, std::vector<double>(K, 1.0), st);
    VBScal sc{};
    sc.alpha = 1.0;
    sc.sigma_0 = 1.0;
    sc.mu0 = 0.0;
    sc.sg0 = 0.02;
    sc.nm0 = 0.0;
    sc.ns0 = 1 / sc.sg0;
    sc.sigma_w = 1.0;
    sc.rho0 = 1.0;
    d_scal.alloc(sizeof(VBScal));
    HIPCHK(hipMemcpyAsync(d_scal.p, &sc, sizeof sc, hipMemcpyHostToDevice, st));
    d_muT.alloc((size_t)p * Kp * sizeof(double));
    d_sgT.alloc((size_t)p * Kp * sizeof(double));
    HIPCHK(hipMemsetAsync(d_muT.p, 0, d_muT.bytes, st));
    HIPCHK(hipMemsetAsync(d_sgT.p, 0, d_sgT.bytes, st));
    d_E.alloc((size_t)std::max(NL, 1u) * sizeof(double));  // e, t per (own) case, user-grouped epoch order
    d_T.alloc((size_t)std::max(NL, 1u) * sizeof(double));
    d_D.alloc((size_t)std::max(J, 1u) * sizeof(VBItemRec));
    d_VS.alloc((size_t)std::max(I, 1u) * sizeof(double2));  // a batch has at most I user rows
    HIPCHK(hipMemsetAsync(d_D.p, 0, d_D.bytes, st));
    if (R > 1) {
        d_send.alloc((size_t)(K + 2) * sizeof(double));
        d_recv.alloc((size_t)R * (K + 2) * sizeof(double));
    }
    part_cap = vbo_scratch_doubles(S, K, p);
    d_part.alloc(part_cap * sizeof(double));
    upload(d_tu, su, st);
    upload(d_ti, si, st);
    upload(d_tr, sr, st);
    d_pred.alloc(std::max<size_t>(su.size(), 1) * sizeof(double));
    d_tpart.alloc(((su.size() + 255) / 256 + 1) * sizeof(double));
    tb.mu_v = d_mu_v.as<double>();
    tb.sg_v = d_sg_v.as<double>();
    tb.nm_v = d_nm_v.as<double>();
    tb.ns_v = d_ns_v.as<double>();
    tb.mu_w = d_mu_w.as<double>();
    tb.sg_w = d_sg_w.as<double>();
    tb.nm_w = d_nm_w.as<double>();
    tb.ns_w = d_ns_w.as<double>();
    tb.rho_w = d_rho_w.as<double>();
    tb.rho_v = d_rho_v.as<double>();
    tb.t_w = d_t_w.as<uint32_t>();
    tb.t_v = d_t_v.as<uint32_t>();
    tb.cc = d_cc.as<uint32_t>();
    tb.sigma_v = d_sigma_v.as<double>();
    tb.scal = d_scal.as<VBScal>();
    tb.K = K;
    tb.p = p;
    tb.N = N;
    tb.I = I;
    shuffle.resize(N);
    for (uint32_t x = 0; x < N; ++x) shuffle[x] = x + 1;
    for (auto& e : ev) event_create(&e);
    fev.assign(2 * (size_t)NB, nullptr);
    for (auto& e : fev) event_create(&e);
    HIPCHK(hipGetDevice(&dev));
    stream_create(&ust);
    for (int k = 0; k < 2; ++k) {
        event_create(&uev[k], hipEventDisableTiming);
        event_create(&done[k], hipEventDisableTiming);
        HIPCHK(hipEventRecord(done[k], st));
    }
    HIPCHK(hipStreamSynchronize(st));
}

namespace {
unsigned host_threads() { return std::max(1u, std::min(16u, std::thread::hardware_concurrency())); }
// f(t, lo, hi) over [0, n) split into host_threads() contiguous chunks
template <class F>
void parallel_chunks(uint32_t n, F&& f) {
    const unsigned nth = host_threads();
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nth; ++t) {
        const uint32_t lo = (uint32_t)((uint64_t)n * t / nth), hi = (uint32_t)((uint64_t)n * (t + 1) / nth);
        th.emplace_back([&f, t, lo, hi] { f(t, lo, hi); });
    }
    for (auto& x : th) x.join();
}
// Keyed pseudorandom permutation of [0, n) (throughput mode's shuffle): a
// 4-round unbalanced Feistel network on bits = ceil(log2 n) (halves of a and
// c = bits - a bits, swapping sizes every round), cycle-walking back into
// [0, n) (< 2 steps on average).  Round function: a murmur3 finaliser of the
// half keyed per (seed, epoch, round) with Philox.  O(1) per case, no shared
// state, so every case's batch is computed in parallel.
struct FeistelPerm {
    uint32_t n, a, c, key[4];
    FeistelPerm(uint64_t seed, uint32_t ep, uint32_t n_) : n(n_) {
        uint32_t bits = 2;
        while ((1ull << bits) < n) ++bits;
        a = bits / 2;
        c = bits - a;
        const P4 o = philox4x32_10(ep, 0, 0x56424f00u, PHILOX_SALT, (uint32_t)seed, (uint32_t)(seed >> 32));
        for (int r = 0; r < 4; ++r) key[r] = o.x[r];
    }
    static uint32_t mix(uint32_t h) {
        h ^= h >> 16;
        h *= 0x85ebca6bu;
        h ^= h >> 13;
        h *= 0xc2b2ae35u;
        h ^= h >> 16;
        return h;
    }
    uint32_t operator()(uint32_t x) const {
        do {
            uint32_t hl = a, hr = c;  // bits of L and R
            uint32_t L = x >> hr, R = x & ((1u << hr) - 1);
            for (int r = 0; r < 4; ++r) {
                const uint32_t nl = R, nr = (L ^ mix(R ^ key[r])) & ((1u << hl) - 1);
                L = nl;
                R = nr;
                std::swap(hl, hr);
            }
            x = (L << hr) | R;
        } while (x >= n);
        return x;
    }
};
}  // namespace

// One epoch's batches: shuffle, batch membership in file order, and each
// batch's cases grouped by user and by item.  The reference-mode shuffle is
// sequential (the reference's rand() stream); everything else runs on
// host_threads() threads (one batch per thread for the grouping).
void VBLearner::build_layout(VBLayout& L, uint32_t ep) {
    bid.resize(N);
    if (cfg.rng_mode == SBMF_RNG_REFERENCE) {
        // libstdc++ random_shuffle: for i = 1..N-1, j = rand() % (i + 1), swap
        for (uint32_t x = 1; x < N; ++x) {
            const uint32_t j = (uint32_t)((long)grand.next() % (long)(x + 1));
            if (x != j) std::swap(shuffle[x], shuffle[j]);
        }
        parallel_chunks(N, [&](unsigned, uint32_t lo, uint32_t hi) {
            for (uint32_t l = lo; l < hi; ++l) bid[l] = (uint32_t)std::ceil((double)shuffle[l] / S) - 1;  // :175
        });
    } else {
        const FeistelPerm perm(cfg.seed, ep, N);
        parallel_chunks(N, [&](unsigned, uint32_t lo, uint32_t hi) {
            for (uint32_t l = lo; l < hi; ++l) bid[l] = perm(l) / S;  // = ceil((perm + 1) / S) - 1
        });
    }
    const bool trace = std::getenv("SBMF_VB_TRACE") != nullptr;
    auto t0 = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!trace) return;
        const auto t1 = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[vbo] layout %u: %s %.1f ms\n", ep, what,
                     std::chrono::duration<double, std::milli>(t1 - t0).count());
        t0 = t1;
    };
    lap("shuffle");
    // per-thread counts of each batch (all cases / own cases), then the fill positions:
    // thread t's own cases of batch b go after threads < t's, each chunk in file order
    const unsigned nth = host_threads();
    std::vector<uint32_t> tcnt((size_t)nth * NB * 2, 0);
    parallel_chunks(N, [&](unsigned t, uint32_t lo, uint32_t hi) {
        uint32_t* c = &tcnt[(size_t)t * NB * 2];
        for (uint32_t l = lo; l < hi; ++l) {
            c[2 * bid[l]]++;
            c[2 * bid[l] + 1] += mine[l];
        }
    });
    L.bsize.assign(NB, 0);
    L.gbsize.assign(NB, 0);
    for (unsigned t = 0; t < nth; ++t)
        for (uint32_t b = 0; b < NB; ++b) {
            L.gbsize[b] += tcnt[((size_t)t * NB + b) * 2];
            L.bsize[b] += tcnt[((size_t)t * NB + b) * 2 + 1];
        }
    L.bbase.assign(NB + 1, 0);  // a batch's (own) cases are entries [bbase[b], bbase[b+1]) of either order
    for (uint32_t b = 0; b < NB; ++b) L.bbase[b + 1] = L.bbase[b] + L.bsize[b];
    btu.resize(NL);  // the (own) cases of each batch, in file order: user, item, rating
    bti.resize(NL);
    btr.resize(NL);
    {
        std::vector<uint32_t> fill((size_t)nth * NB);
        for (uint32_t b = 0; b < NB; ++b) {
            uint32_t at = L.bbase[b];
            for (unsigned t = 0; t < nth; ++t) {
                fill[(size_t)t * NB + b] = at;
                at += tcnt[((size_t)t * NB + b) * 2 + 1];
            }
        }
        parallel_chunks(N, [&](unsigned t, uint32_t lo, uint32_t hi) {
            uint32_t* f = &fill[(size_t)t * NB];
            for (uint32_t l = lo; l < hi; ++l)
                if (mine[l]) {
                    const uint32_t x = f[bid[l]]++;
                    btu[x] = tu[l];
                    bti[x] = ti[l];
                    btr[x] = (float)tr[l];
                }
        });
    }
    lap("batches");
    // several ranks (every batch's items over all ranks) or XCD slices: each batch's item
    // list, and each item's index there
    std::vector<uint32_t> gidx;
    if (R > 1 || XS > 1) {
        std::vector<uint32_t> cnt((size_t)NB * J, 0);
        {
            std::vector<std::vector<uint32_t>> tc(nth);
            parallel_chunks(N, [&](unsigned t, uint32_t lo, uint32_t hi) {
                tc[t].assign((size_t)NB * J, 0);
                for (uint32_t l = lo; l < hi; ++l) tc[t][(size_t)bid[l] * J + ti[l]]++;
            });
            parallel_chunks(NB * J, [&](unsigned, uint32_t lo, uint32_t hi) {
                for (auto& c : tc)
                    if (!c.empty())
                        for (uint32_t x = lo; x < hi; ++x) cnt[x] += c[x];
            });
        }
        L.gitems.clear();
        L.gitem0.assign(NB + 1, 0);
        gidx.assign((size_t)NB * J, 0);
        for (uint32_t b = 0; b < NB; ++b) {
            L.gitem0[b] = (uint32_t)L.gitems.size();
            for (uint32_t a = 0; a < J; ++a)
                if (cnt[(size_t)b * J + a]) {
                    gidx[(size_t)b * J + a] = (uint32_t)L.gitems.size() - L.gitem0[b];
                    L.gitems.push_back(VGItem{I + a, cnt[(size_t)b * J + a], XS > 1 ? 0u : R == 32 ? ~0u : (1u << R) - 1});
                }
            gmax = std::max(gmax, (uint32_t)L.gitems.size() - L.gitem0[b]);
        }
        L.gitem0[NB] = (uint32_t)L.gitems.size();
    }
    lap("item lists");
    bupos.resize(NL);  // a batch case's user-grouped position
    L.iu.resize(NL);
    L.upart.resize(NL);
    L.ur.resize(NL);
    using Part = VBLayout::Part;
    L.pu.resize(NB);
    L.pi.resize(NB);
    std::vector<Part>& pu = L.pu;
    std::vector<Part>& pi = L.pi;
    // lane-group size of a row: the fewest lanes (a power of two, 1..256) that hold its
    // cases at VB_CASES_PER_LANE per lane in registers -- a user row of a batch (a few
    // cases) takes one lane, so a task covers up to 256 rows and every lane has several
    // independent loads in flight
    auto lg_of = [](uint32_t n, uint32_t cpl) {
        uint32_t lg = 0;
        while (lg < 8 && (cpl << lg) < n) ++lg;
        return lg;
    };
    // rows of one orientation (and slice) in attribute order -> stably sorted by lane-group
    // size, records in that order from position run (a task's rows are one contiguous run
    // of records: coalesced reads, whole-line writes from one block), and its tasks
    auto place = [&](std::vector<VRow>& rows, uint32_t& run, std::vector<VRow>& out, std::vector<VTask>& tasks,
                     uint32_t cpl) {
        std::vector<uint32_t> cls(10, 0);
        for (const VRow& r : rows) cls[lg_of(r.len, cpl)]++;
        uint32_t at = 0;
        std::vector<uint32_t> first(10, 0);
        for (int lg = 8; lg >= 0; --lg) {
            first[lg] = at;
            at += cls[lg];
        }
        const uint32_t r0 = (uint32_t)out.size();
        out.resize(r0 + rows.size());
        for (const VRow& r : rows) out[r0 + first[lg_of(r.len, cpl)]++] = r;
        for (uint32_t r = r0; r < out.size(); ++r) {
            out[r].start = run;
            run += out[r].len;
        }
        for (uint32_t r = r0; r < out.size();) {
            const uint32_t lg = lg_of(out[r].len, cpl);
            uint32_t m = 0;
            while (r + m < out.size() && m < (256u >> lg) && lg_of(out[r + m].len, cpl) == lg) ++m;
            tasks.push_back(VTask{r, m, lg, 0});
            r += m;
        }
    };
    // users of batch b: urow[user] = its row in the batch (the item side's partner index)
    auto group_users = [&](uint32_t b, std::vector<uint32_t>& off, std::vector<uint32_t>& urow, Part& P) {
        const uint32_t c0 = L.bbase[b], c1 = L.bbase[b + 1];
        std::fill(off.begin(), off.end(), 0u);
        for (uint32_t x = c0; x < c1; ++x) off[btu[x]]++;
        std::vector<VRow> rows;
        for (uint32_t a = 0; a < I; ++a)
            if (off[a]) rows.push_back(VRow{a, 0u, off[a], 0u});
        P.rows.clear();
        P.tasks.clear();
        uint32_t run = c0;
        place(rows, run, P.rows, P.tasks, VB_CASES_PER_LANE);
        for (uint32_t r = 0; r < P.rows.size(); ++r) {
            off[P.rows[r].attr] = P.rows[r].start;  // becomes the fill position
            urow[P.rows[r].attr] = r;
        }
        for (uint32_t x = c0; x < c1; ++x) {
            const uint32_t q = off[btu[x]]++;
            bupos[x] = q;
            L.upart[q] = I + bti[x];
            L.ur[q] = btr[x];
        }
    };
    // items of batch b, cut into XS slices by the partner's user row (XS = 1: whole rows);
    // a (sub-)row's pad: several ranks -> the item's index in the batch's global list,
    // slices -> x * nG + that index (its slot among the partial sums)
    auto group_items = [&](uint32_t b, std::vector<uint32_t>& off, const std::vector<uint32_t>& urow, uint32_t nu,
                           Part& P) {
        const uint32_t c0 = L.bbase[b], c1 = L.bbase[b + 1];
        const uint32_t nG = (R > 1 || XS > 1) ? L.gitem0[b + 1] - L.gitem0[b] : 0;
        // slice x: the cases at user-grouped positions [c0 + x B / XS, c0 + (x+1) B / XS) --
        // equal case counts, and whole users' rows but the boundary ones (positions follow rows)
        const uint64_t B = c1 - c0;
        auto slice = [&](uint32_t x) { return XS > 1 ? (uint32_t)((uint64_t)(bupos[x] - c0) * XS / B) : 0u; };
        (void)nu;
        std::fill(off.begin(), off.end(), 0u);  // [XS][J]
        for (uint32_t x = c0; x < c1; ++x) off[(size_t)slice(x) * J + bti[x]]++;
        P.rows.clear();
        P.tasks.clear();
        std::vector<std::vector<VTask>> st(XS);
        uint32_t run = c0;
        for (uint32_t xs = 0; xs < XS; ++xs) {
            std::vector<VRow> rows;
            for (uint32_t a = 0; a < J; ++a) {
                const uint32_t n = off[(size_t)xs * J + a];
                if (!n) continue;
                const uint32_t g = (R > 1 || XS > 1) ? gidx[(size_t)b * J + a] : 0u;
                rows.push_back(VRow{I + a, 0u, n, XS > 1 ? xs * nG + g : g});
                if (XS > 1) L.gitems[L.gitem0[b] + g].mask |= 1u << xs;
            }
            const uint32_t r0 = (uint32_t)P.rows.size();
            place(rows, run, P.rows, st[xs], VB_ITEM_CASES_PER_LANE);
            for (uint32_t r = r0; r < P.rows.size(); ++r)
                off[(size_t)xs * J + (P.rows[r].attr - I)] = P.rows[r].start;
        }
        // slice x's tasks at x, x + XS, x + 2 XS, ...; empty tasks fill the gaps
        size_t most = 0;
        for (auto& t : st) most = std::max(most, t.size());
        for (size_t t = 0; t < most; ++t)
            for (uint32_t xs = 0; xs < XS; ++xs)
                P.tasks.push_back(t < st[xs].size() ? st[xs][t] : VTask{0u, 0u, 0u, 0u});
        for (uint32_t x = c0; x < c1; ++x) {
            const uint32_t q = off[(size_t)slice(x) * J + bti[x]]++;
            L.iu[q] = make_uint2(bupos[x], urow[btu[x]]);
        }
    };
    {
        std::vector<std::thread> th;
        for (unsigned t = 0; t < nth; ++t)
            th.emplace_back([&, t] {
                std::vector<uint32_t> offu(I), urow(I), offi((size_t)XS * J);
                for (uint32_t b = t; b < NB; b += nth) {
                    group_users(b, offu, urow, pu[b]);
                    group_items(b, offi, urow, (uint32_t)pu[b].rows.size(), pi[b]);
                }
            });
        for (auto& x : th) x.join();
    }
    lap("grouping");
    // every batch's rows and tasks, batch-major on the device (stage_layout copies them)
    auto offsets = [&](const std::vector<Part>& P, std::vector<uint32_t>& row0, std::vector<uint32_t>& task0) {
        row0.assign(NB + 1, 0);
        task0.assign(NB + 1, 0);
        for (uint32_t b = 0; b < NB; ++b) {
            row0[b + 1] = row0[b] + (uint32_t)P[b].rows.size();
            task0[b + 1] = task0[b] + (uint32_t)P[b].tasks.size();
        }
    };
    offsets(pu, L.urow0, L.utask0);
    offsets(pi, L.irow0, L.itask0);
    lap("offsets");
}

// Several ranks: one item pass of a batch (the update_w biases, factor == 0,
// or update_v of factor f): local sums -> all-gather -> the same update on
// every rank, its deltas to D for the next user pass.
void VBLearner::item_pass(const VBLayout& L, uint32_t b, const VTask* it_, uint32_t nit, const VRow* ir_,
                          const uint2* iu_, int factor, uint32_t f, VBCases ETu) {
    const uint32_t nG = L.gitem0[b + 1] - L.gitem0[b];
    if (nG == 0) return;  // every rank sees the same global list
    double2* sums = d_sums.as<double2>();
    HIPCHK(hipMemsetAsync(sums, 0, (size_t)nG * sizeof(double2), st));
    if (factor)
        HIPCHK(vbo_item_v(it_, nit, ir_, iu_, f, tb, ETu, d_VS.as<double2>(),
                          d_D.as<VBItemRec>(), sums, st));
    else
        HIPCHK(vbo_item_w(it_, nit, ir_, iu_, tb, ETu, d_D.as<VBItemRec>(), sums, st));
    comm->allgather(sums, (size_t)nG * sizeof(double2), d_recvg.p, st);
    HIPCHK(vbo_item_update(L.d_gitems.as<VGItem>() + L.gitem0[b], nG, d_recvg.as<double2>(), R, factor, f, tb,
                           d_D.as<VBItemRec>(), st));
    n_launch += 1;  // vbo_item_update (the item pass itself is counted by run)
}

// Several ranks: every rank's owned user means (factors and biases) to every rank
void VBLearner::sync_users() {
    if (R <= 1) return;
    for (uint32_t f = 0; f < K; ++f) comm->bcast_ranges(tb.mu_v + (size_t)f * p, sizeof(double), ubounds, st);
    comm->bcast_ranges(tb.mu_w, sizeof(double), ubounds, st);
}

// Epoch e's layout to the device on the upload stream once the kernels of epoch
// e - 2 (the last users of these buffers, which may be reallocated here) are
// done; uev[e & 1] marks completion.  Pageable copies: the calling (worker)
// thread blocks, the compute stream does not.
void VBLearner::stage_layout(VBLayout& L, uint32_t e) {
    const auto h0 = std::chrono::steady_clock::now();
    HIPCHK(hipEventSynchronize(done[e & 1]));
    auto parts = [&](const std::vector<VBLayout::Part>& P, const std::vector<uint32_t>& row0,
                     const std::vector<uint32_t>& task0, DBuf& drows, DBuf& dtasks) {
        drows.ensure(std::max<size_t>(row0[NB], 1) * sizeof(VRow));
        dtasks.ensure(std::max<size_t>(task0[NB], 1) * sizeof(VTask));
        for (uint32_t b = 0; b < NB; ++b) {
            if (!P[b].rows.empty())
                HIPCHK(hipMemcpyAsync(drows.as<VRow>() + row0[b], P[b].rows.data(), P[b].rows.size() * sizeof(VRow),
                                      hipMemcpyHostToDevice, ust));
            if (!P[b].tasks.empty())
                HIPCHK(hipMemcpyAsync(dtasks.as<VTask>() + task0[b], P[b].tasks.data(),
                                      P[b].tasks.size() * sizeof(VTask), hipMemcpyHostToDevice, ust));
        }
    };
    parts(L.pu, L.urow0, L.utask0, L.d_urows, L.d_utasks);
    parts(L.pi, L.irow0, L.itask0, L.d_irows, L.d_itasks);
    upload_grow(L.d_upart, L.upart, ust);
    upload_grow(L.d_ur, L.ur, ust);
    upload_grow(L.d_iu, L.iu, ust);
    if (R > 1 || XS > 1) upload_grow(L.d_gitems, L.gitems, ust);
    HIPCHK(hipEventRecord(uev[e & 1], ust));
    if (std::getenv("SBMF_VB_TRACE")) {
        HIPCHK(hipEventSynchronize(uev[e & 1]));
        std::fprintf(stderr, "[vbo] layout %u: upload %.1f ms (to completion)\n", e,
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h0).count());
    }
}

void VBLearner::run(uint32_t epochs, sbmf_sweep_cb cb, void* user) {
    for (uint32_t it = 0; it < epochs; ++it) {
        const auto h0 = std::chrono::steady_clock::now();
        // this epoch's layout: built and uploaded by the worker during the previous epoch
        // (or now); the compute stream waits for its upload
        if (built == epoch) {
            build_layout(lay[epoch & 1], epoch);
            stage_layout(lay[epoch & 1], epoch);
            built = epoch + 1;
        } else if (worker.joinable()) {
            worker.join();
            if (worker_err) std::rethrow_exception(std::exchange(worker_err, nullptr));
        }
        VBLayout& L = lay[epoch & 1];
        HIPCHK(hipStreamWaitEvent(st, uev[epoch & 1], 0));
        if (R > 1 || XS > 1) d_sums.ensure((size_t)XS * std::max(gmax, 1u) * sizeof(double2));
        if (R > 1) d_recvg.ensure((size_t)R * std::max(gmax, 1u) * sizeof(double2));
        if (std::getenv("SBMF_VB_TRACE"))
            std::fprintf(stderr, "[vbo] epoch %u: waited %.1f ms for its layout\n", epoch,
                         std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h0).count());
        ms_layout = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h0).count();
        n_launch = 0;
        HIPCHK(hipEventRecord(ev[0], st));
        const VBCases ETu{d_E.as<double>(), d_T.as<double>()};
        VBItemRec* D = d_D.as<VBItemRec>();
        double2* VS = d_VS.as<double2>();
        double* part = d_part.as<double>();

        for (uint32_t b = 0; b < NB; ++b) {
            const uint32_t B = L.bsize[b];
            const uint32_t nu = L.urow0[b + 1] - L.urow0[b];
            HIPCHK(vbo_transpose(tb.mu_v, d_muT.as<double>(), K, Kp, p, st));
            HIPCHK(vbo_transpose(tb.sg_v, d_sgT.as<double>(), K, Kp, p, st));
            const VRow* ur_ = L.d_urows.as<VRow>() + L.urow0[b];  // tasks index the batch's rows
            const VRow* ir_ = L.d_irows.as<VRow>() + L.irow0[b];
            HIPCHK(vbo_predict(ur_, nu, L.d_upart.as<uint32_t>(), L.d_ur.as<float>(), d_muT.as<double>(),
                               d_sgT.as<double>(), tb, Kp, ETu, st));
            if (R > 1) {  // update_w0 from every rank's local sum
                HIPCHK(vbo_w0_local(ETu.at(L.bbase[b]), B, tb, part, d_send.as<double>(), st));
                comm->allgather(d_send.p, sizeof(double), d_recv.p, st);
                HIPCHK(vbo_w0_final(d_recv.as<double>(), R, L.gbsize[b], tb, st));
            } else {
                HIPCHK(vbo_update_w0(ETu.at(L.bbase[b]), B, tb, part, st));
            }
            const VTask* ut = L.d_utasks.as<VTask>() + L.utask0[b];
            const VTask* it_ = L.d_itasks.as<VTask>() + L.itask0[b];
            const uint32_t nut = L.utask0[b + 1] - L.utask0[b], nit = L.itask0[b + 1] - L.itask0[b];
            const uint32_t* upart_ = L.d_upart.as<uint32_t>();
            const uint2* iu_ = L.d_iu.as<uint2>();
            // users update their records in place; items read them (through i2u) and leave
            // their updates in D, which the next user pass (or the flush) applies
            // one rank, XS > 1: the slices' partial sums, then the items' updates
            const VGItem* gi_ = XS > 1 ? L.d_gitems.as<VGItem>() + L.gitem0[b] : nullptr;
            const uint32_t nG = XS > 1 ? L.gitem0[b + 1] - L.gitem0[b] : 0;
            double2* sums = XS > 1 ? d_sums.as<double2>() : nullptr;
            HIPCHK(vbo_user_w(ut, nut, ur_, tb, ETu, st));
            if (R > 1) {
                item_pass(L, b, it_, nit, ir_, iu_, 0, 0, ETu);
            } else {
                HIPCHK(vbo_item_w(it_, nit, ir_, iu_, tb, ETu, D, sums, st));
                if (XS > 1) HIPCHK(vbo_item_update(gi_, nG, sums, (int)XS, 0, 0, tb, D, st));
            }
            int pend = VB_PEND_W;
            HIPCHK(hipEventRecord(fev[2 * (size_t)b], st));
            for (uint32_t f = 0; f < K; ++f) {
                HIPCHK(vbo_user_v(ut, nut, ur_, upart_, f, pend, f - 1, tb, D, ETu, VS, st));
                if (R > 1) {
                    item_pass(L, b, it_, nit, ir_, iu_, 1, f, ETu);
                } else {
                    HIPCHK(vbo_item_v(it_, nit, ir_, iu_, f, tb, ETu, VS, D, sums, st));
                    if (XS > 1) HIPCHK(vbo_item_update(gi_, nG, sums, (int)XS, 1, f, tb, D, st));
                }
                pend = VB_PEND_V;
            }
            HIPCHK(hipEventRecord(fev[2 * (size_t)b + 1], st));
            HIPCHK(vbo_user_flush(ut, nut, ur_, upart_, pend, K - 1, tb, D, ETu, st));
            if (R > 1) {  // the blends from every rank's alpha sum and user-range sig sums
                HIPCHK(vbo_hyper_local(ETu.at(L.bbase[b]), B, tb, u0, u1, part, part_cap, d_send.as<double>(), st));
                comm->allgather(d_send.p, (K + 2) * sizeof(double), d_recv.p, st);
                HIPCHK(vbo_hyper_final(d_recv.as<double>(), R, L.gbsize[b], tb, I, part, part_cap, st));
            } else {
                HIPCHK(vbo_hyper(ETu.at(L.bbase[b]), B, tb, part, st));
            }
            n_launch += 2 * K + 12 + (XS > 1 ? K + 1 : 0);  // transposes 2, predict, w0 2, bias passes 2, factor passes 2K, flush, hyper 4
        }
        // the next epoch's shuffle and layout, on the host while this epoch runs
        // (the reference stream after this epoch's shuffle is exactly the next one's)
        HIPCHK(hipEventRecord(done[epoch & 1], st));  // this layout's device buffers are free after this
        if (built == epoch + 1) {
            built = epoch + 2;
            const uint32_t nx = epoch + 1;
            worker = std::thread([this, nx] {
                try {
                    HIPCHK(hipSetDevice(dev));
                    build_layout(lay[nx & 1], nx);
                    stage_layout(lay[nx & 1], nx);
                } catch (...) {
                    worker_err = std::current_exception();
                }
            });
        }
        sync_users();  // several ranks: owned user means to every rank (test RMSE, factors)
        HIPCHK(hipEventRecord(ev[1], st));
        // ---- test RMSE of the clamped means (fm_learn_vb_online_simultaneous.h:348-360,441-447)
        const uint64_t nt = su.size();
        double rmse = NAN;
        if (nt) {
            HIPCHK(vbo_transpose(tb.mu_v, d_muT.as<double>(), K, Kp, p, st));
            HIPCHK(vbo_test(d_tu.as<uint32_t>(), d_ti.as<uint32_t>(), d_tr.as<double>(), nt, I, d_muT.as<double>(), tb,
                            Kp, lo, hi, d_pred.as<double>(), d_tpart.as<double>(), st));
            std::vector<double> h((nt + 255) / 256);
            HIPCHK(hipMemcpyAsync(h.data(), d_tpart.p, h.size() * sizeof(double), hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            double se = 0.0;
            for (double x : h) se += x;
            rmse = std::sqrt(se / nt);
        }
        HIPCHK(hipEventRecord(ev[2], st));
        VBScal sc;
        HIPCHK(hipMemcpyAsync(&sc, d_scal.p, sizeof sc, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        last_rmse = rmse;
        last_alpha = sc.alpha;
        float ms_epoch = 0.f, ms_eval = 0.f;
        (void)hipEventElapsedTime(&ms_epoch, ev[0], ev[1]);
        (void)hipEventElapsedTime(&ms_eval, ev[1], ev[2]);
        for (uint32_t b = 0; b < NB; ++b) {
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, fev[2 * (size_t)b], fev[2 * (size_t)b + 1]);
            ms_factor_sum += ms;
        }
        ++n_factor_epochs;
        sbmf_sweep_info info{};
        info.sweep = epoch;
        info.collected = 1;
        info.rmse_avg = rmse;
        info.rmse_this = rmse;
        info.rmse_train = NAN;
        info.tau = sc.alpha;
        info.ms_sweep = ms_epoch;
        info.ms_eval = ms_eval;
        ++epoch;
        if (cb && cb(&info, user)) break;
    }
}

// ---------------------------------------------------------------- entry points used by sbmf.cpp
VBLearner* vbo_create(const sbmf_config& c, uint64_t n, const uint32_t* u, const uint32_t* i, const double* r,
                      uint64_t nt, const uint32_t* tu, const uint32_t* ti, const double* tr, uint32_t I, uint32_t J,
                      hipStream_t st, Comm* comm) {
    std::unique_ptr<VBLearner> L(new VBLearner());
    L->init(c, n, u, i, r, nt, tu, ti, tr, I, J, st, comm);
    return L.release();
}
void vbo_destroy(VBLearner* L) { delete L; }
void vbo_run(VBLearner* L, uint32_t epochs, sbmf_sweep_cb cb, void* user) {
    L->ms_factor_sum = 0.0;
    L->n_factor_epochs = 0;
    L->run(epochs, cb, user);
}
void vbo_predict_out(VBLearner* L, double* out) {
    HIPCHK(hipStreamSynchronize(L->st));
    if (!L->su.empty()) HIPCHK(hipMemcpy(out, L->d_pred.p, L->su.size() * sizeof(double), hipMemcpyDeviceToHost));
}
// means of the factors: users [I][K], items [J][K]
void vbo_factors(VBLearner* L, double* U, double* V) {
    HIPCHK(hipStreamSynchronize(L->st));
    std::vector<double> h((size_t)L->K * L->p);
    HIPCHK(hipMemcpy(h.data(), L->d_mu_v.p, h.size() * sizeof(double), hipMemcpyDeviceToHost));
    for (uint32_t f = 0; f < L->K; ++f) {
        if (U)
            for (uint32_t a = 0; a < L->I; ++a) U[(size_t)a * L->K + f] = h[(size_t)f * L->p + a];
        if (V)
            for (uint32_t a = 0; a < L->J; ++a) V[(size_t)a * L->K + f] = h[(size_t)f * L->p + L->I + a];
    }
}
void vbo_biases(VBLearner* L, double* bu, double* bv, double* b0) {
    HIPCHK(hipStreamSynchronize(L->st));
    std::vector<double> h(L->p);
    HIPCHK(hipMemcpy(h.data(), L->d_mu_w.p, h.size() * sizeof(double), hipMemcpyDeviceToHost));
    if (bu) std::copy(h.begin(), h.begin() + L->I, bu);
    if (bv) std::copy(h.begin() + L->I, h.end(), bv);
    if (b0) {
        VBScal sc;
        HIPCHK(hipMemcpy(&sc, L->d_scal.p, sizeof sc, hipMemcpyDeviceToHost));
        *b0 = sc.mu0;
    }
}
// [sigma_v (K) | 0 ...] and alpha
void vbo_hyper_out(VBLearner* L, double* h4k, double* alpha) {
    HIPCHK(hipStreamSynchronize(L->st));
    if (h4k) {
        std::fill(h4k, h4k + 4 * (size_t)L->K, 0.0);
        HIPCHK(hipMemcpy(h4k, L->d_sigma_v.p, L->K * sizeof(double), hipMemcpyDeviceToHost));
    }
    if (alpha) {
        VBScal sc;
        HIPCHK(hipMemcpy(&sc, L->d_scal.p, sizeof sc, hipMemcpyDeviceToHost));
        *alpha = sc.alpha;
    }
}
double vbo_layout_ms(const VBLearner* L) { return L->ms_layout; }
uint32_t vbo_launches(const VBLearner* L) { return L->n_launch; }
double vbo_factor_ms(const VBLearner* L) { return L->n_factor_epochs ? L->ms_factor_sum / L->n_factor_epochs : 0.0; }

}  // namespace sbmf
