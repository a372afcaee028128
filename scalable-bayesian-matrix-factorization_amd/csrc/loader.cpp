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
        if (nf != 2 || feats[0] < 0 || feats[1] < (long)item_offset) {
            g_lerr = "libFM line " + std::to_string(lineno) + " of " + path +
                     ": the SBPMF sampler needs exactly one user and one item feature per line";
            return SBMF_E_IO;
        }
        u.push_back((uint32_t)feats[0]);
        i.push_back((uint32_t)(feats[1] - (long)item_offset));
        r.push_back((double)target);
        p = le + 1;
    }
    return fill(out, u, i, r);
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
