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
#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/sbmf.h"

namespace {

thread_local std::string g_lerr;

bool read_file(const char* path, std::vector<char>& buf) {
    FILE* f = std::fopen(path, "rb");
    if (!f) return false;
    std::fseek(f, 0, SEEK_END);
    const long sz = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    buf.resize((size_t)(sz > 0 ? sz : 0) + 1);
    const size_t got = sz > 0 ? std::fread(buf.data(), 1, (size_t)sz, f) : 0;
    std::fclose(f);
    buf[got] = 0;
    buf.resize(got + 1);
    return true;
}

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

int fill(sbmf_ratings* out, std::vector<uint32_t>& u, std::vector<uint32_t>& i, std::vector<double>& r) {
    out->n = u.size();
    const size_t n = u.size() ? u.size() : 1;
    out->user = static_cast<uint32_t*>(std::malloc(n * sizeof(uint32_t)));
    out->item = static_cast<uint32_t*>(std::malloc(n * sizeof(uint32_t)));
    out->rating = static_cast<double*>(std::malloc(n * sizeof(double)));
    if (!out->user || !out->item || !out->rating) {
        sbmf_free_ratings(out);
        return SBMF_E_NOMEM;
    }
    if (!u.empty()) {
        std::memcpy(out->user, u.data(), u.size() * sizeof(uint32_t));
        std::memcpy(out->item, i.data(), i.size() * sizeof(uint32_t));
        std::memcpy(out->rating, r.data(), r.size() * sizeof(double));
    }
    return SBMF_OK;
}

}  // namespace

extern "C" {

int sbmf_load_triples(const char* path, sbmf_ratings* out) {
    if (!path || !out) return SBMF_E_ARG;
    std::memset(out, 0, sizeof *out);
    std::vector<char> buf;
    if (!read_file(path, buf)) {
        g_lerr = std::string("unable to open ") + path;
        return SBMF_E_IO;
    }
    std::vector<uint32_t> u, i;
    std::vector<double> r;
    u.reserve(buf.size() / 12);
    i.reserve(buf.size() / 12);
    r.reserve(buf.size() / 12);
    char* p = buf.data();
    char* const end = buf.data() + buf.size() - 1;
    std::string line;
    while (p < end) {
        char* nl = static_cast<char*>(std::memchr(p, '\n', (size_t)(end - p)));
        char* le = nl ? nl : end;
        const char saved = *le;
        *le = 0;
        // fast path: digits SEP digits SEP <strtod number>
        const char* q = p;
        unsigned a, b;
        bool ok = false;
        if (parse_uint(q, a) && *q && *q != '\n') {
            ++q;
            if (parse_uint(q, b) && *q) {
                ++q;
                if (*q && *q != ' ' && *q != '\t') {
                    char* e2;
                    errno = 0;
                    const double v = std::strtod(q, &e2);
                    if (e2 != q) {
                        u.push_back(a);
                        i.push_back(b);
                        r.push_back(v);
                        ok = true;
                    }
                }
            }
        }
        if (!ok) {  // exact reference acceptance rule
            unsigned uu, ii;
            char c1, c2;
            double v;
            if (std::sscanf(p, "%u%c%u%c%lf", &uu, &c1, &ii, &c2, &v) >= 5) {
                u.push_back(uu);
                i.push_back(ii);
                r.push_back(v);
            }
        }
        *le = saved;
        p = le + 1;
    }
    return fill(out, u, i, r);
}

int sbmf_load_libfm(const char* path, uint32_t item_offset, sbmf_ratings* out) {
    if (!path || !out) return SBMF_E_ARG;
    std::memset(out, 0, sizeof *out);
    std::vector<char> buf;
    if (!read_file(path, buf)) {
        g_lerr = std::string("unable to open ") + path;
        return SBMF_E_IO;
    }
    std::vector<uint32_t> u, i;
    std::vector<double> r;
    char* p = buf.data();
    char* const end = buf.data() + buf.size() - 1;
    size_t lineno = 0;
    while (p < end) {
        ++lineno;
        char* nl = static_cast<char*>(std::memchr(p, '\n', (size_t)(end - p)));
        char* le = nl ? nl : end;
        *le = 0;
        const char* q = p;
        while (*q == ' ' || *q == '\t') ++q;
        if (*q == 0 || *q == '#' || *q == '\r') {
            p = le + 1;
            continue;
        }
        char* e;
        const float target = std::strtof(q, &e);
        if (e == q) {
            g_lerr = "cannot parse libFM line " + std::to_string(lineno) + " of " + path;
            return SBMF_E_IO;
        }
        q = e;
        long feats[3];
        int nf = 0;
        while (true) {
            while (*q == ' ' || *q == '\t') ++q;
            if (*q == 0 || *q == '#' || *q == '\r') break;
            char* e1;
            const long id = std::strtol(q, &e1, 10);
            if (e1 == q || *e1 != ':') {
                g_lerr = "cannot parse libFM line " + std::to_string(lineno) + " of " + path;
                return SBMF_E_IO;
            }
            q = e1 + 1;
            char* e3;
            (void)std::strtof(q, &e3);
            if (e3 == q) {
                g_lerr = "cannot parse libFM line " + std::to_string(lineno) + " of " + path;
                return SBMF_E_IO;
            }
            q = e3;
            if (nf < 3) feats[nf] = id;
            ++nf;
        }
        if (nf != 2 || feats[0] < 0 || feats[1] < (long)item_offset || (item_offset > 0 && feats[0] >= (long)item_offset)) {
            g_lerr = "libFM line " + std::to_string(lineno) + " of " + path +
                     ": the SBPMF sampler needs exactly one user and one item feature per line" +
                     (item_offset > 0 ? " (user id < item_offset <= item id)" : "");
            return SBMF_E_IO;
        }
        u.push_back((uint32_t)feats[0]);
        i.push_back((uint32_t)(feats[1] - (long)item_offset));
        r.push_back((double)target);
        p = le + 1;
    }
    return fill(out, u, i, r);
}

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

int sbmf_load_libfm_binary(const char* stem, uint32_t item_offset, sbmf_ratings* out) {
    if (!stem || !out) return SBMF_E_ARG;
    std::memset(out, 0, sizeof *out);
    const std::string s(stem);
    std::string xf, yf;
    if (file_exists(s + ".data") && file_exists(s + ".target")) {
        xf = s + ".data";
        yf = s + ".target";
    } else if (file_exists(s + ".x") && file_exists(s + ".y")) {
        xf = s + ".x";
        yf = s + ".y";
    } else {
        g_lerr = "unable to open " + s + ".x/.y (or .data/.target)";
        return SBMF_E_IO;
    }
    std::vector<char> xb, yb;
    if (!read_file(xf.c_str(), xb) || !read_file(yf.c_str(), yb)) {
        g_lerr = "unable to open " + xf + " / " + yf;
        return SBMF_E_IO;
    }
    // read_file appends one terminating byte
    const size_t xn = xb.size() - 1, yn = yb.size() - 1;
    if (yn < 12) {
        g_lerr = yf + ": truncated header";
        return SBMF_E_IO;
    }
    uint32_t yh[3];
    std::memcpy(yh, yb.data(), 12);
    if (yh[0] != 1 || yh[1] != sizeof(float) || yn < 12 + (size_t)yh[2] * sizeof(float)) {
        g_lerr = yf + ": not a libFM DVector<float> file (version 1, 4-byte values)";
        return SBMF_E_IO;
    }
    FmHeader h;
    if (xn < sizeof h) {
        g_lerr = xf + ": truncated header";
        return SBMF_E_IO;
    }
    std::memcpy(&h, xb.data(), sizeof h);
    if (h.id != 2 || h.float_size != sizeof(float)) {
        g_lerr = xf + ": not a libFM sparse matrix file (id 2, 4-byte values)";
        return SBMF_E_IO;
    }
    if (h.num_rows != yh[2]) {
        g_lerr = xf + ": " + std::to_string(h.num_rows) + " rows but " + std::to_string(yh[2]) + " targets";
        return SBMF_E_IO;
    }
    std::vector<uint32_t> u, i;
    std::vector<double> r;
    u.reserve(h.num_rows);
    i.reserve(h.num_rows);
    r.reserve(h.num_rows);
    size_t at = sizeof h;
    uint64_t nv = 0;
    for (uint32_t row = 0; row < h.num_rows; ++row) {
        uint32_t sz;
        if (at + 4 > xn) {
            g_lerr = xf + ": truncated at row " + std::to_string(row);
            return SBMF_E_IO;
        }
        std::memcpy(&sz, xb.data() + at, 4);
        at += 4;
        if (at + (size_t)sz * 8 > xn) {
            g_lerr = xf + ": truncated at row " + std::to_string(row);
            return SBMF_E_IO;
        }
        uint32_t f0 = 0, f1 = 0;
        if (sz == 2) {
            std::memcpy(&f0, xb.data() + at, 4);
            std::memcpy(&f1, xb.data() + at + 8, 4);
        }
        if (sz != 2 || f1 < item_offset || (item_offset > 0 && f0 >= item_offset)) {
            g_lerr = xf + " row " + std::to_string(row) +
                     ": the SBPMF sampler needs exactly one user and one item feature per row" +
                     (item_offset > 0 ? " (user id < item_offset <= item id)" : "");
            return SBMF_E_IO;
        }
        at += (size_t)sz * 8;
        nv += sz;
        float t;
        std::memcpy(&t, yb.data() + 12 + (size_t)row * 4, 4);
        u.push_back(f0);
        i.push_back(f1 - item_offset);
        r.push_back((double)t);
    }
    if (nv != h.num_values) {
        g_lerr = xf + ": header says " + std::to_string(h.num_values) + " values, rows hold " + std::to_string(nv);
        return SBMF_E_IO;
    }
    return fill(out, u, i, r);
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
    std::vector<char> row(4 + 16);
    for (uint64_t q = 0; ok && q < in->n; ++q) {
        const uint32_t sz = 2, a = in->user[q], b = item_offset + in->item[q];
        const float one = 1.0f;
        std::memcpy(row.data(), &sz, 4);
        std::memcpy(row.data() + 4, &a, 4);
        std::memcpy(row.data() + 8, &one, 4);
        std::memcpy(row.data() + 12, &b, 4);
        std::memcpy(row.data() + 16, &one, 4);
        ok = std::fwrite(row.data(), row.size(), 1, fx) == 1;
    }
    const uint32_t yh[3] = {1, (uint32_t)sizeof(float), (uint32_t)in->n};
    ok = ok && std::fwrite(yh, sizeof yh, 1, fy) == 1;
    for (uint64_t q = 0; ok && q < in->n; ++q) {
        const float t = (float)in->rating[q];
        ok = std::fwrite(&t, 4, 1, fy) == 1;
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
