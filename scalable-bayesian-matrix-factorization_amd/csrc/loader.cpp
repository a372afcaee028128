// loader.cpp -- the reference's two input formats (host side of the boundary).
//
// * SBPMF triples: a line is a rating iff sscanf(line, "%u%c%u%c%lf") >= 5
//   (gibbs_sbpmf_final.cpp:43,86,107,136,202); other lines are skipped.  The
//   common "digits SEP digits SEP number" shape is parsed directly and any
//   other line goes through sscanf itself, so acceptance is identical.
// * libFM text: "target id:value id:value ..." (Data.h:192-217): leading
//   blanks skipped, empty and '#' lines skipped, target read as DATA_FLOAT
//   (float, fm_data.h:25), anything unparsable is an error.  The SBPMF path
//   needs exactly two features per line: user id, then item id.
//
// The reference parses in three serial passes (gibbs_sbpmf_final.cpp:26-215);
// here the file is read once and cut at line boundaries into one chunk per
// thread, each chunk parsed into its own arrays, and the chunks concatenated
// in file order -- the same ratings in the same order as a serial parse.
// Numbers: "digits[.digits]" with a mantissa below 2^53 (2^24 for float) and at
// most 22 (10) fraction digits is m / 10^k, one correctly rounded division of
// two exactly representable values -- the value strtod (strtof) returns
// (Clinger's fast path); anything else goes through strtod / strtof itself.
#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <thread>
#include <vector>

#include "../../include/sbmf.h"

namespace {

thread_local std::string g_lerr;

inline bool parse_uint(const char*& p, unsigned& out) {
    if (*p < '0' || *p > '9') return false;
    unsigned long long v = 0;
    while (*p >= '0' && *p <= '9') {
        v = v * 10 + (unsigned)(*p - '0');
        if (v > 0xffffffffull) return false;
        ++p;
    }
    out = (unsigned)v;
    return true;
}

// "digits[.digits]" ending where strtod would stop (not at e/E/x/X/p/P/.):
// m / 10^k when exact operands make it strtod's correctly rounded result.
// Returns false (caller uses strtod / strtof) for every other form.
template <typename F>
inline bool parse_fast(const char* q, F& out, const char*& end) {
    constexpr unsigned long long MMAX = sizeof(F) == 8 ? (1ull << 53) : (1ull << 24);
    constexpr int KMAX = sizeof(F) == 8 ? 22 : 10;
    static const double p10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                   1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
    const char* p = q;
    unsigned long long m = 0;
    int nd = 0, k = 0;
    while (*p >= '0' && *p <= '9') {
        m = m * 10 + (unsigned)(*p - '0');
        if (++nd > 18) return false;
        ++p;
    }
    if (nd == 0) return false;
    if (*p == '.') {
        ++p;
        while (*p >= '0' && *p <= '9') {
            m = m * 10 + (unsigned)(*p - '0');
            ++k;
            if (++nd > 18) return false;
            ++p;
        }
    }
    const char c = *p;
    if (c == 'e' || c == 'E' || c == 'x' || c == 'X' || c == 'p' || c == 'P' || c == '.') return false;
    if (m > MMAX || k > KMAX) return false;
    if (sizeof(F) == 8)
        out = (F)((double)m / p10[k]);
    else
        out = (F)((float)m / (float)p10[k]);
    end = p;
    return true;
}

// Line-aligned chunks of buf[0, n): one per thread, each at least `min_bytes`.
int nthreads();
std::vector<size_t> line_chunks(const char* buf, size_t n, size_t min_bytes) {
    const int th = nthreads();
    const size_t want = std::max<size_t>(1, std::min<size_t>((size_t)th, n / std::max<size_t>(min_bytes, 1)));
    std::vector<size_t> cut{0};
    for (size_t c = 1; c < want; ++c) {
        size_t at = std::max(cut.back(), n * c / want);
        const void* nl = at < n ? std::memchr(buf + at, '\n', n - at) : nullptr;
        at = nl ? (size_t)(static_cast<const char*>(nl) - buf) + 1 : n;
        if (at > cut.back() && at < n) cut.push_back(at);
    }
    cut.push_back(n);
    return cut;
}

// A chunk's output: the ratings it parsed, written straight into the result
// arrays from slot `base` (its first line's index: a chunk never yields more
// ratings than lines), compacted afterwards.
struct Part {
    uint32_t* u = nullptr;
    uint32_t* i = nullptr;
    double* r = nullptr;
    size_t n = 0;               // ratings parsed
    size_t lines = 0;           // lines seen
    long err_line = -1;         // first bad line in the chunk (0-based within it), libFM text
    std::string err;
    void push(uint32_t a, uint32_t b, double v) {
        u[n] = a;
        i[n] = b;
        r[n] = v;
        ++n;
    }
};

// Large buffers on transparent huge pages where the kernel offers them (madvise
// mode): the first touch of a few hundred MB then takes hundreds of faults
// instead of ~10^5 (measured 1.05 -> see DESIGN §6 on a VM host).  free()able.
void* big_alloc(size_t bytes) {
    constexpr size_t HP = 2u << 20;
    if (bytes < HP) return std::malloc(bytes);
    void* p = std::aligned_alloc(HP, (bytes + HP - 1) / HP * HP);
    if (p) (void)madvise(p, (bytes + HP - 1) / HP * HP, MADV_HUGEPAGE);
    return p;
}

int nthreads() {
    int th = (int)std::thread::hardware_concurrency();
    if (const char* e = std::getenv("SBMF_LOAD_THREADS")) th = std::atoi(e);
    else if (const char* o = std::getenv("OMP_NUM_THREADS")) th = std::min(th, std::atoi(o));
    return std::max(1, std::min(th, 64));
}

template <class F>
void parallel_for(size_t n, F&& f) {
    std::vector<std::thread> ths;
    for (size_t c = 1; c < n; ++c) ths.emplace_back(f, c);
    if (n) f(0);
    for (auto& t : ths) t.join();
}

// The whole file into an uninitialised buffer (+ a terminating 0), read by
// several threads (pread of disjoint ranges).
struct FreeDel {
    void operator()(char* p) const { std::free(p); }
};
using CBuf = std::unique_ptr<char, FreeDel>;
bool read_par(const char* path, CBuf& buf, size_t& n) {
    FILE* f = std::fopen(path, "rb");
    if (!f) return false;
    std::fseek(f, 0, SEEK_END);
    const long sz = std::ftell(f);
    n = sz > 0 ? (size_t)sz : 0;
    buf.reset(static_cast<char*>(big_alloc(n + 1)));
    if (!buf) {
        std::fclose(f);
        return false;
    }
    const int fd = fileno(f);
    const size_t nt = std::max<size_t>(1, std::min<size_t>((size_t)nthreads(), n >> 24));
    std::vector<char> ok(nt, 1);
    parallel_for(nt, [&](size_t t) {
        size_t at = n * t / nt;
        const size_t e = n * (t + 1) / nt;
        while (at < e) {
            const ssize_t got = pread(fd, buf.get() + at, e - at, (off_t)at);
            if (got <= 0) {
                ok[t] = 0;
                return;
            }
            at += (size_t)got;
        }
    });
    std::fclose(f);
    buf.get()[n] = 0;
    return std::all_of(ok.begin(), ok.end(), [](char x) { return x != 0; });
}

// Runs parse(part, begin, end) over line-aligned chunks on threads, each writing
// from its first line's slot, then closes the gaps in chunk order.  Returns the
// first error (chunk order) with its file line number.
template <class F>
int run_chunks(const char* buf, size_t n, const char* path, F&& parse, sbmf_ratings* out) {
    size_t min_bytes = 4u << 20;  // SBMF_LOAD_CHUNK: smaller chunks (tests)
    if (const char* e = std::getenv("SBMF_LOAD_CHUNK")) min_bytes = (size_t)std::max(1L, std::atol(e));
    const std::vector<size_t> cut = line_chunks(buf, n, min_bytes);
    const size_t nc = cut.size() - 1;
    // lines per chunk (a chunk ends after a newline, except possibly the last)
    std::vector<size_t> base(nc + 1, 0);
    parallel_for(nc, [&](size_t c) {
        size_t k = 0;
        const char* p = buf + cut[c];
        const char* const e = buf + cut[c + 1];
        while (p < e) {
            const void* nl = std::memchr(p, '\n', (size_t)(e - p));
            ++k;
            p = nl ? static_cast<const char*>(nl) + 1 : e;
        }
        base[c + 1] = k;
    });
    for (size_t c = 0; c < nc; ++c) base[c + 1] += base[c];
    const size_t cap = base[nc] ? base[nc] : 1;
    out->user = static_cast<uint32_t*>(big_alloc(cap * sizeof(uint32_t)));
    out->item = static_cast<uint32_t*>(big_alloc(cap * sizeof(uint32_t)));
    out->rating = static_cast<double*>(big_alloc(cap * sizeof(double)));
    if (!out->user || !out->item || !out->rating) {
        sbmf_free_ratings(out);
        return SBMF_E_NOMEM;
    }
    std::vector<Part> parts(nc);
    parallel_for(nc, [&](size_t c) {
        parts[c].u = out->user + base[c];
        parts[c].i = out->item + base[c];
        parts[c].r = out->rating + base[c];
        parse(parts[c], buf + cut[c], buf + cut[c + 1]);
    });
    size_t before = 0, total = 0;
    for (size_t c = 0; c < nc; ++c) {
        const Part& p = parts[c];
        if (p.err_line >= 0) {
            g_lerr = p.err + " line " + std::to_string(before + (size_t)p.err_line + 1) + " of " + path;
            sbmf_free_ratings(out);
            return SBMF_E_IO;
        }
        before += p.lines;
        if (total != base[c] && p.n) {  // close the gap left by skipped lines
            std::memmove(out->user + total, p.u, p.n * sizeof(uint32_t));
            std::memmove(out->item + total, p.i, p.n * sizeof(uint32_t));
            std::memmove(out->rating + total, p.r, p.n * sizeof(double));
        }
        total += p.n;
    }
    out->n = total;
    return SBMF_OK;
}

// Line parsers over read-only bytes (a mapped file).  A line is [p, le) with
// le at its '\n' or at the end of the data; the fast paths read at most up to
// that '\n' (a byte no number or id continues through), and the final line,
// which may have no '\n', is always parsed from a terminated copy.  Anything
// the fast path does not take is parsed from a terminated copy of the line by
// the reference's own rule (sscanf / strtod / strtof / strtol), so acceptance
// and values are those of the serial parser.

// SBPMF triples: sscanf(line, "%u%c%u%c%lf") >= 5 (gibbs_sbpmf_final.cpp:43)
void triple_line(Part& P, const char* p, const char* le, bool copy_only, std::string& tmp) {
    if (!copy_only) {  // fast path: digits SEP digits SEP <short decimal>
        const char* q = p;
        unsigned a, b;
        double v;
        const char* e2;
        if (parse_uint(q, a) && q < le) {
            ++q;
            if (parse_uint(q, b) && q < le) {
                ++q;
                if (q < le && *q != ' ' && *q != '\t' && parse_fast(q, v, e2)) {
                    P.push(a, b, v);
                    return;
                }
            }
        }
    }
    tmp.assign(p, le);
    const char* t = tmp.c_str();
    const char* q = t;
    unsigned a, b;
    if (parse_uint(q, a) && *q) {  // the direct form with strtod
        ++q;
        if (parse_uint(q, b) && *q) {
            ++q;
            if (*q && *q != ' ' && *q != '\t') {
                char* e2;
                errno = 0;
                const double v = std::strtod(q, &e2);
                if (e2 != q) {
                    P.push(a, b, v);
                    return;
                }
            }
        }
    }
    unsigned uu, ii;
    char c1, c2;
    double v;
    if (std::sscanf(t, "%u%c%u%c%lf", &uu, &c1, &ii, &c2, &v) >= 5) P.push(uu, ii, v);  // the exact rule
}

void parse_triples(Part& P, const char* p, const char* const end) {
    std::string tmp;
    while (p < end) {
        const char* nl = static_cast<const char*>(std::memchr(p, '\n', (size_t)(end - p)));
        const char* le = nl ? nl : end;
        ++P.lines;
        triple_line(P, p, le, nl == nullptr, tmp);
        p = le + 1;
    }
}

// libFM text (Data.h:192-217).  Returns false with P.err set on a bad line.
bool libfm_line_slow(Part& P, const char* t, uint32_t item_offset) {
    const char* q = t;
    while (*q == ' ' || *q == '\t') ++q;
    if (*q == 0 || *q == '#' || *q == '\r') return true;
    char* e;
    const float target = std::strtof(q, &e);
    if (e == q) return P.err = "cannot parse libFM", false;
    q = e;
    long feats[3];
    int nf = 0;
    while (true) {
        while (*q == ' ' || *q == '\t') ++q;
        if (*q == 0 || *q == '#' || *q == '\r') break;
        char* e1;
        const long id = std::strtol(q, &e1, 10);
        if (e1 == q || *e1 != ':') return P.err = "cannot parse libFM", false;
        q = e1 + 1;
        char* e3;
        (void)std::strtof(q, &e3);
        if (e3 == q) return P.err = "cannot parse libFM", false;
        q = e3;
        if (nf < 3) feats[nf] = id;
        ++nf;
    }
    if (nf != 2 || feats[0] < 0 || feats[1] < (long)item_offset || (item_offset > 0 && feats[0] >= (long)item_offset)) {
        P.err = item_offset > 0 ? "the SBPMF sampler needs exactly one user and one item feature per line "
                                  "(user id < item_offset <= item id): libFM"
                                : "the SBPMF sampler needs exactly one user and one item feature per line: libFM";
        return false;
    }
    P.push((uint32_t)feats[0], (uint32_t)(feats[1] - (long)item_offset), (double)target);
    return true;
}

// fast path: "target u:v i:v" with short decimals and ids, blanks between, then
// the end of the line (or '#' / '\r')
bool libfm_line_fast(Part& P, const char* p, const char* le, uint32_t item_offset) {
    const char* q = p;
    while (q < le && (*q == ' ' || *q == '\t')) ++q;
    if (q == le || *q == '#' || *q == '\r') return true;  // blank / comment line
    float target;
    const char* e;
    if (!parse_fast(q, target, e)) return false;
    q = e;
    unsigned id[2];
    for (int f = 0; f < 2; ++f) {
        if (q >= le || (*q != ' ' && *q != '\t')) return false;
        while (q < le && (*q == ' ' || *q == '\t')) ++q;
        if (q >= le || !parse_uint(q, id[f]) || id[f] > 0x7fffffffu || q >= le || *q != ':') return false;
        ++q;
        float fv;
        if (!parse_fast(q, fv, e)) return false;
        q = e;
    }
    while (q < le && (*q == ' ' || *q == '\t')) ++q;
    if (q < le && *q != '#' && *q != '\r') return false;  // more features, or anything else
    if (id[1] < item_offset || (item_offset > 0 && id[0] >= item_offset)) return false;  // the slow path reports it
    P.push(id[0], id[1] - item_offset, (double)target);
    return true;
}

void parse_libfm(Part& P, const char* p, const char* const end, uint32_t item_offset) {
    std::string tmp;
    while (p < end) {
        const char* nl = static_cast<const char*>(std::memchr(p, '\n', (size_t)(end - p)));
        const char* le = nl ? nl : end;
        const size_t lineno = P.lines++;
        if (!nl || !libfm_line_fast(P, p, le, item_offset)) {
            tmp.assign(p, le);
            if (!libfm_line_slow(P, tmp.c_str(), item_offset)) {
                P.err_line = (long)lineno;
                return;
            }
        }
        p = le + 1;
    }
}

// A whole input file, read-only: mapped (MAP_POPULATE: the page-cache pages are
// mapped in one pass, no copy) or, where mapping fails, read into a buffer.
struct InFile {
    const char* p = "";
    size_t n = 0;
    void* map = nullptr;
    CBuf buf;
    ~InFile() {
        if (map) munmap(map, n);
    }
};
bool open_in(const char* path, InFile& f) {
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return false;
    struct stat st;
    if (fstat(fd, &st) == 0 && S_ISREG(st.st_mode) && st.st_size > 0) {
        void* m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
        if (m != MAP_FAILED) {
            close(fd);
            f.map = m;
            f.n = (size_t)st.st_size;
            f.p = static_cast<const char*>(m);
            return true;
        }
    }
    close(fd);
    if (!read_par(path, f.buf, f.n)) return false;
    f.p = f.buf.get();
    return true;
}

}  // namespace

extern "C" {

int sbmf_load_triples(const char* path, sbmf_ratings* out) {
    if (!path || !out) return SBMF_E_ARG;
    std::memset(out, 0, sizeof *out);
    InFile f;
    if (!open_in(path, f)) {
        g_lerr = std::string("unable to open ") + path;
        return SBMF_E_IO;
    }
    return run_chunks(f.p, f.n, path, parse_triples, out);
}

int sbmf_load_libfm(const char* path, uint32_t item_offset, sbmf_ratings* out) {
    if (!path || !out) return SBMF_E_ARG;
    std::memset(out, 0, sizeof *out);
    InFile f;
    if (!open_in(path, f)) {
        g_lerr = std::string("unable to open ") + path;
        return SBMF_E_IO;
    }
    return run_chunks(f.p, f.n, path,
                      [item_offset](Part& P, const char* p, const char* e) { parse_libfm(P, p, e, item_offset); }, out);
}

// The SBPMF triple format the reference's data scripts write
// (data/*/create_file_scalable_bpmf.py: "u\ti\tr" per line, 0-based ids),
// ratings printed with %.17g unless they are integers (as "4", "3.5" in
// MovieLens), so sbmf_load_triples reads back the same doubles.
int sbmf_save_triples(const char* path, const sbmf_ratings* in) {
    if (!path || !in || (in->n && (!in->user || !in->item || !in->rating))) return SBMF_E_ARG;
    FILE* f = std::fopen(path, "wb");
    if (!f) {
        g_lerr = std::string("unable to write ") + path;
        return SBMF_E_IO;
    }
    auto put_u = [](char* o, unsigned long long v) {  // decimal digits of v at o, returns the end
        char t[24];
        int k = 0;
        do {
            t[k++] = (char)('0' + v % 10);
            v /= 10;
        } while (v);
        while (k) *o++ = t[--k];
        return o;
    };
    std::vector<char> buf(1 << 22);
    size_t at = 0;
    bool ok = true;
    for (uint64_t q = 0; ok && q < in->n; ++q) {
        if (at + 96 > buf.size()) {
            ok = std::fwrite(buf.data(), 1, at, f) == at;
            at = 0;
        }
        char* o = buf.data() + at;
        o = put_u(o, in->user[q]);
        *o++ = '\t';
        o = put_u(o, in->item[q]);
        *o++ = '\t';
        const double r = in->rating[q];
        if (r >= 0 && r < 1e15 && r == (double)(long long)r && !std::signbit(r))
            o = put_u(o, (unsigned long long)r);
        else
            o += std::snprintf(o, 40, "%.17g", r);
        *o++ = '\n';
        at = (size_t)(o - buf.data());
    }
    if (ok && at) ok = std::fwrite(buf.data(), 1, at, f) == at;
    ok = (std::fclose(f) == 0) & ok;
    if (!ok) {
        g_lerr = std::string("write error on ") + path;
        return SBMF_E_IO;
    }
    return SBMF_OK;
}

}  // extern "C"


extern "C" {

// ---- libFM binary input: <stem>.x (or .data) + <stem>.y (or .target), the
// files tools/convert.cpp writes.  Layouts (fmatrix.h:36-52, matrix.h:280-328):
//   .x  file_header {u32 id = 2; u32 float_size = 4; u64 num_values; u32 num_rows;
//       u32 num_cols} (24 bytes, natural alignment), then per row u32 size and
//       size x sparse_entry {u32 id; f32 value}
//   .y  u32 version = 1; u32 float_size = 4; u32 num_rows; num_rows x f32
// Data::load (Data.h:113-160) prefers .data/.target over .x/.y and asserts
// target.dim == rows; the same order and checks apply here, as errors.
namespace {
struct FmHeader {
    uint32_t id, float_size;
    uint64_t num_values;
    uint32_t num_rows, num_cols;
};
static_assert(sizeof(FmHeader) == 24, "fmatrix.h file_header layout");

bool file_exists(const std::string& f) {
    FILE* h = std::fopen(f.c_str(), "rb");
    if (h) std::fclose(h);
    return h != nullptr;
}
}  // namespace

namespace {
int load_x(const std::string& xf, const std::string& yf, uint32_t item_offset, sbmf_ratings* out);
int load_xt(const std::string& xf, const std::string& yf, uint32_t item_offset, sbmf_ratings* out);
}  // namespace

int sbmf_load_libfm_binary(const char* stem, uint32_t item_offset, sbmf_ratings* out) {
    if (!stem || !out) return SBMF_E_ARG;
    std::memset(out, 0, sizeof *out);
    const std::string s(stem);
    if (file_exists(s + ".data") && file_exists(s + ".target")) return load_x(s + ".data", s + ".target", item_offset, out);
    if (file_exists(s + ".x") && file_exists(s + ".y")) return load_x(s + ".x", s + ".y", item_offset, out);
    g_lerr = "unable to open " + s + ".x/.y (or .data/.target)";
    return SBMF_E_IO;
}

int sbmf_load_libfm_binary_t(const char* stem, uint32_t item_offset, sbmf_ratings* out) {
    if (!stem || !out) return SBMF_E_ARG;
    std::memset(out, 0, sizeof *out);
    const std::string s(stem);
    if (file_exists(s + ".datat") && file_exists(s + ".target"))
        return load_xt(s + ".datat", s + ".target", item_offset, out);
    if (file_exists(s + ".xt") && file_exists(s + ".y")) return load_xt(s + ".xt", s + ".y", item_offset, out);
    g_lerr = "unable to open " + s + ".xt/.y (or .datat/.target)";
    return SBMF_E_IO;
}

// Data::load (Data.h:106-283) for rating data: the binary files of
// sbmf_libfm_binary_kind when present (the row-major file when the set has one;
// the transpose for a set without, which is what bin/libFM's MCMC / ALS sets
// read), else <stem> as libFM text.
int sbmf_load_libfm_data(const char* stem, int has_x, int has_xt, uint32_t item_offset, sbmf_ratings* out) {
    if (!stem || !out || (!has_x && !has_xt)) return SBMF_E_ARG;
    std::memset(out, 0, sizeof *out);
    const std::string s(stem);
    const int kind = sbmf_libfm_binary_kind(stem, has_x, has_xt);
    if (kind == 1)
        return has_x ? load_x(s + ".data", s + ".target", item_offset, out)
                     : load_xt(s + ".datat", s + ".target", item_offset, out);
    if (kind == 2)
        return has_x ? load_x(s + ".x", s + ".y", item_offset, out) : load_xt(s + ".xt", s + ".y", item_offset, out);
    return sbmf_load_libfm(stem, item_offset, out);
}

namespace {
int load_x(const std::string& xf, const std::string& yf, uint32_t item_offset, sbmf_ratings* out) {
    std::memset(out, 0, sizeof *out);
    InFile xin, yin;
    if (!open_in(xf.c_str(), xin) || !open_in(yf.c_str(), yin)) {
        g_lerr = "unable to open " + xf + " / " + yf;
        return SBMF_E_IO;
    }
    const char* const xb = xin.p;
    const char* const yb = yin.p;
    const size_t xn = xin.n, yn = yin.n;
    if (yn < 12) {
        g_lerr = yf + ": truncated header";
        return SBMF_E_IO;
    }
    uint32_t yh[3];
    std::memcpy(yh, yb, 12);
    if (yh[0] != 1 || yh[1] != sizeof(float) || yn < 12 + (size_t)yh[2] * sizeof(float)) {
        g_lerr = yf + ": not a libFM DVector<float> file (version 1, 4-byte values)";
        return SBMF_E_IO;
    }
    FmHeader h;
    if (xn < sizeof h) {
        g_lerr = xf + ": truncated header";
        return SBMF_E_IO;
    }
    std::memcpy(&h, xb, sizeof h);
    if (h.id != 2 || h.float_size != sizeof(float)) {
        g_lerr = xf + ": not a libFM sparse matrix file (id 2, 4-byte values)";
        return SBMF_E_IO;
    }
    if (h.num_rows != yh[2]) {
        g_lerr = xf + ": " + std::to_string(h.num_rows) + " rows but " + std::to_string(yh[2]) + " targets";
        return SBMF_E_IO;
    }
    const size_t R = h.num_rows, m = R ? R : 1;
    out->user = static_cast<uint32_t*>(big_alloc(m * sizeof(uint32_t)));
    out->item = static_cast<uint32_t*>(big_alloc(m * sizeof(uint32_t)));
    out->rating = static_cast<double*>(big_alloc(m * sizeof(double)));
    if (!out->user || !out->item || !out->rating) {
        sbmf_free_ratings(out);
        return SBMF_E_NOMEM;
    }
    auto bad_row = [&](uint64_t row) {
        g_lerr = xf + " row " + std::to_string(row) +
                 ": the SBPMF sampler needs exactly one user and one item feature per row" +
                 (item_offset > 0 ? " (user id < item_offset <= item id)" : "");
        sbmf_free_ratings(out);
        return SBMF_E_IO;
    };
    auto take = [&](size_t row, const char* rec) -> bool {  // rec: {u32 size; 2 x {u32 id; f32 value}}
        uint32_t sz, f0, f1;
        std::memcpy(&sz, rec, 4);
        std::memcpy(&f0, rec + 4, 4);
        std::memcpy(&f1, rec + 12, 4);
        if (sz != 2 || f1 < item_offset || (item_offset > 0 && f0 >= item_offset)) return false;
        float t;
        std::memcpy(&t, yb + 12 + row * 4, 4);
        out->user[row] = f0;
        out->item[row] = f1 - item_offset;
        out->rating[row] = (double)t;
        return true;
    };
    // what the rating converter writes: every row {user, item}, 20 bytes, so row q
    // sits at 24 + 20 q -- rows taken in parallel; any other file is scanned row by row
    constexpr size_t REC = 4 + 2 * 8;
    if (xn == sizeof h + R * REC && h.num_values == 2 * (uint64_t)R) {
        const size_t nt = std::max<size_t>(1, std::min<size_t>((size_t)nthreads(), R >> 18));
        std::vector<uint64_t> first_bad(nt, UINT64_MAX);
        parallel_for(nt, [&](size_t t) {
            for (size_t q = R * t / nt, e = R * (t + 1) / nt; q < e; ++q)
                if (!take(q, xb + sizeof h + q * REC)) {
                    first_bad[t] = q;
                    return;
                }
        });
        for (uint64_t q : first_bad)
            if (q != UINT64_MAX) return bad_row(q);
        out->n = R;
        return SBMF_OK;
    }
    size_t at = sizeof h;
    uint64_t nv = 0;
    for (uint32_t row = 0; row < h.num_rows; ++row) {
        uint32_t sz;
        if (at + 4 > xn) {
            g_lerr = xf + ": truncated at row " + std::to_string(row);
            sbmf_free_ratings(out);
            return SBMF_E_IO;
        }
        std::memcpy(&sz, xb + at, 4);
        if (at + 4 + (size_t)sz * 8 > xn) {
            g_lerr = xf + ": truncated at row " + std::to_string(row);
            sbmf_free_ratings(out);
            return SBMF_E_IO;
        }
        if (sz != 2 || !take(row, xb + at)) return bad_row(row);
        at += 4 + (size_t)sz * 8;
        nv += sz;
    }
    if (nv != h.num_values) {
        g_lerr = xf + ": header says " + std::to_string(h.num_values) + " values, rows hold " + std::to_string(nv);
        sbmf_free_ratings(out);
        return SBMF_E_IO;
    }
    out->n = R;
    return SBMF_OK;
}
}  // namespace

// Data::load's file choice (Data.h:112-117): 1 = <stem>.data/.datat/.target,
// 2 = <stem>.x/.xt/.y, each file of the pair required only when the data set
// needs that orientation (has_x: row-major cases; has_xt: the transpose, rows
// per feature), 0 = neither, Data::load reads <stem> as text.  bin/libFM builds
// its train / test sets with has_x = (method != "mcmc") after rewriting als to
// mcmc, and has_xt = true except for sgd / sgda (libfm.cpp:132-149): the MCMC
// and ALS chains read only the transpose.
int sbmf_libfm_binary_kind(const char* stem, int has_x, int has_xt) {
    if (!stem || (!has_x && !has_xt)) return SBMF_E_ARG;
    const std::string s(stem);
    if ((!has_x || file_exists(s + ".data")) && (!has_xt || file_exists(s + ".datat")) && file_exists(s + ".target"))
        return 1;
    if ((!has_x || file_exists(s + ".x")) && (!has_xt || file_exists(s + ".xt")) && file_exists(s + ".y")) return 2;
    return 0;
}

// libFM's transpose <stem>.xt + <stem>.y (or .datat + .target, preferred as
// Data::load does, Data.h:113-117,143-151): the file tools/transpose.cpp:54-172
// writes from a .x, with the .x header's roles swapped (num_rows = features,
// num_cols = cases) and one sparse row per feature {u32 size; size x {u32 case
// id; f32 value}}, case ids ascending.  This is the only file bin/libFM -method
// mcmc|als reads (has_x = false, libfm.cpp:140-149).  For rating data a
// feature's row is its user's or item's rating list, so the per-case pair is
// rebuilt: each case must hold exactly two features, the lower id is the user,
// the higher the item (users-first ids), and item_offset has the meaning of
// sbmf_load_libfm_binary.
namespace {
int load_xt(const std::string& xf, const std::string& yf, uint32_t item_offset, sbmf_ratings* out) {
    std::memset(out, 0, sizeof *out);
    InFile xin, yin;
    if (!open_in(xf.c_str(), xin) || !open_in(yf.c_str(), yin)) {
        g_lerr = "unable to open " + xf + " / " + yf;
        return SBMF_E_IO;
    }
    const char* const xb = xin.p;
    const char* const yb = yin.p;
    const size_t xn = xin.n, yn = yin.n;
    if (yn < 12) {
        g_lerr = yf + ": truncated header";
        return SBMF_E_IO;
    }
    uint32_t yh[3];
    std::memcpy(yh, yb, 12);
    if (yh[0] != 1 || yh[1] != sizeof(float) || yn < 12 + (size_t)yh[2] * sizeof(float)) {
        g_lerr = yf + ": not a libFM DVector<float> file (version 1, 4-byte values)";
        return SBMF_E_IO;
    }
    FmHeader h;
    if (xn < sizeof h) {
        g_lerr = xf + ": truncated header";
        return SBMF_E_IO;
    }
    std::memcpy(&h, xb, sizeof h);
    if (h.id != 2 || h.float_size != sizeof(float)) {
        g_lerr = xf + ": not a libFM sparse matrix file (id 2, 4-byte values)";
        return SBMF_E_IO;
    }
    // the transpose's columns are the cases; Data::load takes num_cases from the
    // targets (Data.h:167), so the two must agree
    if (h.num_cols != yh[2]) {
        g_lerr = xf + ": " + std::to_string(h.num_cols) + " cases but " + std::to_string(yh[2]) + " targets";
        return SBMF_E_IO;
    }
    const uint32_t F = h.num_rows;
    const size_t C = h.num_cols, m = C ? C : 1;
    // pass 1 (serial, one u32 per feature row): row offsets and the value count
    std::vector<size_t> off((size_t)F + 1);
    size_t at = sizeof h;
    for (uint32_t f = 0; f < F; ++f) {
        uint32_t sz;
        if (at + 4 > xn) {
            g_lerr = xf + ": truncated at feature row " + std::to_string(f);
            return SBMF_E_IO;
        }
        std::memcpy(&sz, xb + at, 4);
        if (at + 4 + (size_t)sz * 8 > xn) {
            g_lerr = xf + ": truncated at feature row " + std::to_string(f);
            return SBMF_E_IO;
        }
        off[f] = at;
        at += 4 + (size_t)sz * 8;
    }
    off[F] = at;
    const uint64_t nv = (at - sizeof h - 4ull * F) / 8;
    if (nv != h.num_values) {
        g_lerr = xf + ": header says " + std::to_string(h.num_values) + " values, rows hold " + std::to_string(nv);
        return SBMF_E_IO;
    }
    out->user = static_cast<uint32_t*>(big_alloc(m * sizeof(uint32_t)));
    out->item = static_cast<uint32_t*>(big_alloc(m * sizeof(uint32_t)));
    out->rating = static_cast<double*>(big_alloc(m * sizeof(double)));
    std::unique_ptr<std::atomic<uint32_t>[]> cnt(new (std::nothrow) std::atomic<uint32_t>[m]);
    if (!out->user || !out->item || !out->rating || !cnt) {
        sbmf_free_ratings(out);
        return SBMF_E_NOMEM;
    }
    const size_t nc = std::max<size_t>(1, std::min<size_t>((size_t)nthreads(), C >> 16));
    parallel_for(nc, [&](size_t t) {
        for (size_t c = C * t / nc, e = C * (t + 1) / nc; c < e; ++c) cnt[c].store(0, std::memory_order_relaxed);
    });
    // pass 2: feature rows cut into nt ranges of about equal value counts; a
    // case's first two features land in user[] / item[] in any order (sorted
    // below), a third one or a case id past the targets is an error
    const size_t nt = std::max<size_t>(1, std::min<size_t>((size_t)nthreads(), (size_t)(nv >> 17)));
    std::vector<uint32_t> fcut(nt + 1, F);
    fcut[0] = 0;
    for (size_t t = 1, f = 0; t < nt; ++t) {
        const size_t want = sizeof h + (off[F] - sizeof h) * t / nt;
        while (f < F && off[f] < want) ++f;
        fcut[t] = (uint32_t)f;
    }
    std::vector<uint64_t> bad(nt, UINT64_MAX);  // (kind << 56) | case / feature
    parallel_for(nt, [&](size_t t) {
        for (uint32_t f = fcut[t]; f < fcut[t + 1]; ++f) {
            uint32_t sz;
            std::memcpy(&sz, xb + off[f], 4);
            const char* rec = xb + off[f] + 4;
            for (uint32_t k = 0; k < sz; ++k, rec += 8) {
                uint32_t c;
                std::memcpy(&c, rec, 4);
                if (c >= C) {
                    bad[t] = (1ull << 56) | f;
                    return;
                }
                const uint32_t slot = cnt[c].fetch_add(1, std::memory_order_relaxed);
                if (slot == 0) out->user[c] = f;
                else if (slot == 1) out->item[c] = f;
            }
        }
    });
    for (uint64_t b : bad)
        if (b != UINT64_MAX) {
            g_lerr = xf + " feature row " + std::to_string(b & 0xffffffffull) + ": case id past the " +
                     std::to_string(C) + " targets";
            sbmf_free_ratings(out);
            return SBMF_E_IO;
        }
    std::vector<uint64_t> first_bad(nc, UINT64_MAX);
    parallel_for(nc, [&](size_t t) {
        for (size_t c = C * t / nc, e = C * (t + 1) / nc; c < e; ++c) {
            const uint32_t a = out->user[c], b = out->item[c];
            const uint32_t lo = std::min(a, b), hi = std::max(a, b);
            if (cnt[c].load(std::memory_order_relaxed) != 2 || hi < item_offset ||
                (item_offset > 0 && lo >= item_offset)) {
                first_bad[t] = c;
                return;
            }
            float y;
            std::memcpy(&y, yb + 12 + c * 4, 4);
            out->user[c] = lo;
            out->item[c] = hi - item_offset;
            out->rating[c] = (double)y;
        }
    });
    for (uint64_t c : first_bad)
        if (c != UINT64_MAX) {
            g_lerr = xf + " case " + std::to_string(c) + ": the learners need exactly one user and one item feature "
                     "per case (" + std::to_string(cnt[c].load()) + " features" +
                     (item_offset > 0 ? "; user id < item_offset <= item id)" : ")");
            sbmf_free_ratings(out);
            return SBMF_E_IO;
        }
    out->n = C;
    return SBMF_OK;
}
}  // namespace

// tools/transpose.cpp:54-172 for rating data: <stem>.xt holds one row per
// feature 0..num_cols-1 (num_cols = max(num_cols, largest feature id + 1), as
// the .x writer), each the ascending case ids of that feature with value 1, and
// <stem>.y the f32 targets -- byte for byte what convert + transpose write for
// the same cases (a .x row {user, item} with value 1 each).
int sbmf_save_libfm_binary_t(const char* stem, const sbmf_ratings* in, uint32_t item_offset, uint32_t num_cols) {
    if (!stem || !in || (in->n && (!in->user || !in->item || !in->rating))) return SBMF_E_ARG;
    if (in->n > 0xffffffffull) return SBMF_E_ARG;
    uint64_t cols = num_cols;
    for (uint64_t q = 0; q < in->n; ++q) {
        cols = std::max<uint64_t>(cols, (uint64_t)in->user[q] + 1);
        cols = std::max<uint64_t>(cols, (uint64_t)item_offset + in->item[q] + 1);
    }
    if (cols > 0xffffffffull) {
        g_lerr = "feature id past UINT32_MAX - 1 (item_offset + item id): not representable in the .xt format";
        return SBMF_E_ARG;
    }
    for (uint64_t q = 0; q < in->n; ++q)
        if (in->user[q] == (uint64_t)item_offset + in->item[q]) {
            g_lerr = "case " + std::to_string(q) + ": user and item feature ids coincide";
            return SBMF_E_ARG;
        }
    // counting sort of the 2n (feature, case) entries by feature, cases ascending
    std::vector<uint64_t> start(cols + 1, 0);
    for (uint64_t q = 0; q < in->n; ++q) {
        ++start[in->user[q] + 1];
        ++start[(uint64_t)item_offset + in->item[q] + 1];
    }
    for (uint64_t f = 0; f < cols; ++f) start[f + 1] += start[f];
    std::vector<uint32_t> cs(2 * in->n);
    {
        std::vector<uint64_t> fill(start.begin(), start.end() - 1);
        for (uint64_t q = 0; q < in->n; ++q) {
            cs[fill[in->user[q]]++] = (uint32_t)q;
            cs[fill[(uint64_t)item_offset + in->item[q]]++] = (uint32_t)q;
        }
    }
    const std::string s(stem);
    FILE* fx = std::fopen((s + ".xt").c_str(), "wb");
    FILE* fy = fx ? std::fopen((s + ".y").c_str(), "wb") : nullptr;
    if (!fx || !fy) {
        if (fx) std::fclose(fx);
        g_lerr = "unable to write " + s + ".xt/.y";
        return SBMF_E_IO;
    }
    const FmHeader h{2, (uint32_t)sizeof(float), 2 * in->n, (uint32_t)cols, (uint32_t)in->n};
    bool ok = std::fwrite(&h, sizeof h, 1, fx) == 1;
    std::vector<char> buf;
    const float one = 1.0f;
    for (uint64_t f = 0; ok && f < cols; ++f) {
        const uint32_t sz = (uint32_t)(start[f + 1] - start[f]);
        buf.resize(4 + (size_t)sz * 8);
        std::memcpy(buf.data(), &sz, 4);
        for (uint32_t k = 0; k < sz; ++k) {
            std::memcpy(buf.data() + 4 + 8 * (size_t)k, &cs[start[f] + k], 4);
            std::memcpy(buf.data() + 8 + 8 * (size_t)k, &one, 4);
        }
        ok = std::fwrite(buf.data(), 1, buf.size(), fx) == buf.size();
    }
    const uint32_t yh[3] = {1, (uint32_t)sizeof(float), (uint32_t)in->n};
    ok = ok && std::fwrite(yh, sizeof yh, 1, fy) == 1;
    constexpr size_t CH = 1 << 16;
    std::vector<float> yb(CH);
    for (uint64_t q0 = 0; ok && q0 < in->n; q0 += CH) {
        const size_t m = (size_t)std::min<uint64_t>(CH, in->n - q0);
        for (size_t k = 0; k < m; ++k) yb[k] = (float)in->rating[q0 + k];
        ok = std::fwrite(yb.data(), 4, m, fy) == m;
    }
    ok = (std::fclose(fx) == 0) & ok;
    ok = (std::fclose(fy) == 0) & ok;
    if (!ok) {
        g_lerr = "write error on " + s + ".xt/.y";
        return SBMF_E_IO;
    }
    return SBMF_OK;
}

// the convert tool's output for rating data (tools/convert.cpp:55-205): row q
// holds {user[q]:1, item_offset + item[q]:1}, target rating[q] as f32
int sbmf_save_libfm_binary(const char* stem, const sbmf_ratings* in, uint32_t item_offset, uint32_t num_cols) {
    if (!stem || !in || (in->n && (!in->user || !in->item || !in->rating))) return SBMF_E_ARG;
    if (in->n > 0xffffffffull) return SBMF_E_ARG;
    // feature ids are written as uint32 and num_cols = max id + 1 must fit too:
    // computed in 64 bits, anything past UINT32_MAX - 1 is refused (no wrap)
    uint64_t cols = num_cols;
    for (uint64_t q = 0; q < in->n; ++q) {
        cols = std::max<uint64_t>(cols, (uint64_t)in->user[q] + 1);
        cols = std::max<uint64_t>(cols, (uint64_t)item_offset + in->item[q] + 1);
    }
    if (cols > 0xffffffffull) {
        g_lerr = "feature id past UINT32_MAX - 1 (item_offset + item id): not representable in the .x format";
        return SBMF_E_ARG;
    }
    const std::string s(stem);
    FILE* fx = std::fopen((s + ".x").c_str(), "wb");
    FILE* fy = fx ? std::fopen((s + ".y").c_str(), "wb") : nullptr;
    if (!fx || !fy) {
        if (fx) std::fclose(fx);
        g_lerr = "unable to write " + s + ".x/.y";
        return SBMF_E_IO;
    }
    const FmHeader h{2, (uint32_t)sizeof(float), 2 * in->n, (uint32_t)in->n, (uint32_t)cols};
    bool ok = std::fwrite(&h, sizeof h, 1, fx) == 1;
    constexpr size_t CH = 1 << 16;  // rows per buffered write
    std::vector<char> xb(CH * 20), yb(CH * 4);
    for (uint64_t q0 = 0; ok && q0 < in->n; q0 += CH) {
        const size_t m = (size_t)std::min<uint64_t>(CH, in->n - q0);
        for (size_t k = 0; k < m; ++k) {
            const uint64_t q = q0 + k;
            const uint32_t sz = 2, a = in->user[q], b = item_offset + in->item[q];
            const float one = 1.0f;
            char* row = xb.data() + k * 20;
            std::memcpy(row, &sz, 4);
            std::memcpy(row + 4, &a, 4);
            std::memcpy(row + 8, &one, 4);
            std::memcpy(row + 12, &b, 4);
            std::memcpy(row + 16, &one, 4);
        }
        ok = std::fwrite(xb.data(), 20, m, fx) == m;
    }
    const uint32_t yh[3] = {1, (uint32_t)sizeof(float), (uint32_t)in->n};
    ok = ok && std::fwrite(yh, sizeof yh, 1, fy) == 1;
    for (uint64_t q0 = 0; ok && q0 < in->n; q0 += CH) {
        const size_t m = (size_t)std::min<uint64_t>(CH, in->n - q0);
        for (size_t k = 0; k < m; ++k) {
            const float t = (float)in->rating[q0 + k];
            std::memcpy(yb.data() + k * 4, &t, 4);
        }
        ok = std::fwrite(yb.data(), 4, m, fy) == m;
    }
    ok = (std::fclose(fx) == 0) & ok;
    ok = (std::fclose(fy) == 0) & ok;
    if (!ok) {
        g_lerr = "write error on " + s + ".x/.y";
        return SBMF_E_IO;
    }
    return SBMF_OK;
}

void sbmf_free_ratings(sbmf_ratings* r) {
    if (!r) return;
    std::free(r->user);
    std::free(r->item);
    std::free(r->rating);
    r->user = r->item = nullptr;
    r->rating = nullptr;
    r->n = 0;
}

const char* sbmf_loader_error(void) { return g_lerr.c_str(); }

}  // extern "C"
