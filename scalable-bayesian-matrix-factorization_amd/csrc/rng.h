// rng.h -- random streams for the SBPMF sampler (host side + Philox device helpers).
//
// Two modes (sbmf_config::rng_mode):
//   SBMF_RNG_REFERENCE  the reference's own variate stream: glibc rand()
//                       (src/util/random.h:174-176), Leva normals (:150-164),
//                       Marsaglia-Tsang gammas (:118-148).  Restated here as a
//                       self-contained per-context generator (glibc random_r
//                       TYPE_3 additive feedback, r[i] = r[i-31] + r[i-3]) so
//                       several contexts / threads never share libc state.
//                       The number of rand() calls per variate depends only on
//                       the uniform stream and the (data-independent) gamma
//                       shapes, so a whole sweep's variates can be generated
//                       ahead of the GPU and consumed in parallel.
//   SBMF_RNG_PHILOX     counter-based Philox4x32-10: a normal for (sweep,
//                       half, row, k) is a pure function of the key, so the
//                       GPU draws it in-kernel and any number of ranks agree.
#pragma once
#include <cmath>
#include <cstdint>

namespace sbmf {

// glibc random_r.c TYPE_3 (degree 31, separation 3), as used by rand().
class GlibcRand {
  public:
    explicit GlibcRand(unsigned seed = 1) { seed_(seed); }
    void seed_(unsigned seed) {
        int32_t word = seed == 0 ? 1 : (int32_t)seed;
        s_[0] = word;
        for (int i = 1; i < 31; ++i) {
            // Schrage: word = 16807 * word % 2147483647 without overflow
            const int32_t hi = word / 127773, lo = word % 127773;
            word = 16807 * lo - 2836 * hi;
            if (word < 0) word += 2147483647;
            s_[i] = word;
        }
        f_ = 3;
        r_ = 0;
        for (int i = 0; i < 310; ++i) next();
    }
    int32_t next() {  // == rand()
        s_[f_] = (int32_t)((uint32_t)s_[f_] + (uint32_t)s_[r_]);
        const int32_t out = (int32_t)(((uint32_t)s_[f_] >> 1) & 0x7fffffff);
        if (++f_ == 31) f_ = 0;
        if (++r_ == 31) r_ = 0;
        return out;
    }
    double uniform() { return next() / ((double)2147483647 + 1); }  // random.h:174-176

  private:
    int32_t s_[31];
    int f_, r_;
};

// Leva normal + Marsaglia-Tsang gamma over any uniform source `U`
// (U::uniform() in [0,1)).  Expression order follows random.h so that the
// GlibcRand instantiation reproduces the reference bit for bit.
#if defined(__HIPCC__)
#define SBMF_HDT __host__ __device__
#else
#define SBMF_HDT
#endif

template <class U>
SBMF_HDT double leva_normal(U& g) {
    double u, v, x, y, Q;
    do {
        do {
            u = g.uniform();
        } while (u == 0.0);
        v = 1.7156 * (g.uniform() - 0.5);
        x = u - 0.449871;
        y = std::fabs(v) + 0.386595;
        Q = x * x + y * (0.19600 * y - 0.25472 * x);
        if (Q < 0.27597) break;
    } while ((Q > 0.27846) || ((v * v) > (-4.0 * u * u * std::log(u))));
    return v / u;
}

// The shape < 1 boost draws its uniform first and multiplies the boosted
// draw by u^(1/alpha), as random.h:121-126 does through recursion.
template <class U>
SBMF_HDT double mt_gamma(U& g, double alpha) {
    double boost = 1.0;
    const bool small = alpha < 1.0;
    if (small) {
        double u;
        do {
            u = g.uniform();
        } while (u == 0.0);
        boost = std::pow(u, 1.0 / alpha);
        alpha = alpha + 1.0;
    }
    const double d = alpha - 1.0 / 3.0;
    const double c = 1.0 / std::sqrt(9.0 * d);
    double x, v, u;
    do {
        do {
            x = leva_normal(g);
            v = 1.0 + c * x;
        } while (v <= 0.0);
        v = v * v * v;
        u = g.uniform();
    } while ((u >= (1.0 - 0.0331 * (x * x) * (x * x))) && (std::log(u) >= (0.5 * x * x + d * (1.0 - v + std::log(v)))));
    return small ? (d * v) * boost : d * v;
}

// ----------------------------------------------------------- Philox4x32-10
struct P4 {
    uint32_t x[4];
};

#if defined(__HIPCC__)
#define SBMF_HD __host__ __device__ __forceinline__
#else
#define SBMF_HD inline
#endif

SBMF_HD uint32_t mulhi32(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }

SBMF_HD P4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t h0 = mulhi32(0xD2511F53u, c0), l0 = 0xD2511F53u * c0;
        const uint32_t h1 = mulhi32(0xCD9E8D57u, c2), l1 = 0xCD9E8D57u * c2;
        const uint32_t n0 = h1 ^ c1 ^ k0, n2 = h0 ^ c3 ^ k1;
        c0 = n0;
        c1 = l1;
        c2 = n2;
        c3 = l0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    P4 o;
    o.x[0] = c0;
    o.x[1] = c1;
    o.x[2] = c2;
    o.x[3] = c3;
    return o;
}

// Stream tags (counter word 2, low byte).
enum : uint32_t { TAG_USERS = 0, TAG_ITEMS = 1, TAG_HOST = 2, TAG_INIT_U = 3, TAG_INIT_V = 4, TAG_BIAS_U = 5,
                  TAG_BIAS_V = 6 };
static const uint32_t PHILOX_SALT = 0x53424d46u;  // "SBMF"

// Two N(0,1) variates (Box-Muller, 53-bit uniforms): normal indices 2*pair
// and 2*pair+1 of the given (row, sweep, tag).  A row's K <= 256 normals use
// pairs 0..127; lane l of a wave draws pairs l and 64+l.
SBMF_HD void philox_normal_pair(uint64_t seed, uint32_t row, uint32_t sweep, uint32_t tag, uint32_t pair,
                                double& z0, double& z1) {
    const P4 o = philox4x32_10(row, sweep, tag | (pair << 8), PHILOX_SALT, (uint32_t)seed, (uint32_t)(seed >> 32));
    const uint64_t a = (((uint64_t)o.x[0] << 32) | o.x[1]) >> 11;
    const uint64_t b = (((uint64_t)o.x[2] << 32) | o.x[3]) >> 11;
    const double u1 = (double)(a + 1) * (1.0 / 9007199254740992.0);  // (0,1]
    const double u2 = (double)b * (1.0 / 9007199254740992.0);        // [0,1)
    const double rr = sqrt(-2.0 * log(u1));
    const double th = 6.283185307179586476925286766559 * u2;
    double sn, cs;
    sincos(th, &sn, &cs);  // one argument reduction for both (the values of sin / cos)
    z0 = rr * cs;
    z1 = rr * sn;
}

// Host-side sequential uniform stream over Philox (hyperparameter draws in
// Philox mode): counter = (index, sweep, TAG_HOST | sub<<8, salt).
class PhiloxStream {
  public:
    PhiloxStream(uint64_t seed, uint32_t sweep, uint32_t sub) : seed_(seed), sweep_(sweep), sub_(sub) {}
    double uniform() {
        if (have_ == 0) {
            const P4 o = philox4x32_10(idx_++, sweep_, TAG_HOST | (sub_ << 8), PHILOX_SALT, (uint32_t)seed_,
                                       (uint32_t)(seed_ >> 32));
            buf_[0] = ((((uint64_t)o.x[0] << 32) | o.x[1]) >> 11) * (1.0 / 9007199254740992.0);
            buf_[1] = ((((uint64_t)o.x[2] << 32) | o.x[3]) >> 11) * (1.0 / 9007199254740992.0);
            have_ = 2;
        }
        return buf_[--have_];
    }

  private:
    uint64_t seed_;
    uint32_t sweep_, sub_, idx_ = 0;
    double buf_[2];
    int have_ = 0;
};

// Per-row sequential uniform stream on the device (biased sampler, Philox
// mode): counter = (row, sweep, tag | index<<8, salt), two 53-bit uniforms
// per Philox block.  Feeds leva_normal / mt_gamma for the per-row bias
// hyperparameter and bias draws, whose rejection loops need a stream.
class PhiloxRowStream {
  public:
    SBMF_HD PhiloxRowStream(uint64_t seed, uint32_t row, uint32_t sweep, uint32_t tag)
        : seed_(seed), row_(row), sweep_(sweep), tag_(tag) {}
    SBMF_HD double uniform() {
        if (have_ == 0) {
            const P4 o = philox4x32_10(row_, sweep_, tag_ | (idx_++ << 8), PHILOX_SALT, (uint32_t)seed_,
                                       (uint32_t)(seed_ >> 32));
            buf_[0] = ((((uint64_t)o.x[0] << 32) | o.x[1]) >> 11) * (1.0 / 9007199254740992.0);
            buf_[1] = ((((uint64_t)o.x[2] << 32) | o.x[3]) >> 11) * (1.0 / 9007199254740992.0);
            have_ = 2;
        }
        return buf_[--have_];
    }

  private:
    uint64_t seed_;
    uint32_t row_, sweep_, tag_, idx_ = 0;
    double buf_[2];
    int have_ = 0;
};

}  // namespace sbmf
