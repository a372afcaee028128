// sbmf_cli.cpp -- `sbmf`, a drop-in for `bin/libFM -task r -method mcmc`
// on the SBPMF path, driving the C ABI of include/sbmf.h.
//
// Flag grammar follows src/util/cmdline.h:33-70,113-119: "-name value" or
// "--name value"; a flag directly followed by another flag gets the empty
// value; a repeated flag or an unregistered flag is an error.  Registered
// flags are libFM's (libfm.cpp:86-111) plus the sampler's own settings.
// Output follows fm_learn_mcmc_simultaneous.h: per sweep
//   "#Iter=%3d\tTrain=<rmse>\tTest=<rmse>"                      (:244)
// and the file test_rmse_<k0><k1><K>_<method> (truncated at start, one
// running-mean test RMSE per line, :57-62,146); -out writes one averaged
// prediction per test line (libfm.cpp:629-634).
// Differences, by design: -seed is honoured (libfm.cpp:124 ignores it); on
// error the exit code is 1 (the reference prints "ERROR" and returns 0).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <limits>
#include <map>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/sbmf.h"

extern "C" const char* sbmf_loader_error(void);

namespace {

struct CmdLine {
    std::map<std::string, std::string> help, value;
    static bool parse_name(std::string& s) {
        if (!s.empty() && s[0] == '-') {
            s = (s.size() > 1 && s[1] == '-') ? s.substr(2) : s.substr(1);
            return true;
        }
        return false;
    }
    CmdLine(int argc, char** argv) {
        for (int i = 1; i < argc; ++i) {
            std::string s(argv[i]);
            if (!parse_name(s)) throw std::runtime_error("cannot parse " + s);
            if (value.count(s)) throw std::runtime_error("the parameter " + s + " is already specified");
            if (i + 1 < argc) {
                std::string nx(argv[i + 1]);
                if (!parse_name(nx)) {
                    value[s] = argv[i + 1];
                    ++i;
                } else {
                    value[s] = "";
                }
            } else {
                value[s] = "";
            }
        }
    }
    void reg(const std::string& n, const std::string& h) { help[n] = h; }
    void check() const {
        for (auto& kv : value)
            if (!help.count(kv.first)) throw std::runtime_error("the parameter " + kv.first + " does not exist");
    }
    bool has(const std::string& n) const { return value.count(n) != 0; }
    std::string get(const std::string& n, const std::string& d) const { return has(n) ? value.at(n) : d; }
    double getd(const std::string& n, double d) const { return has(n) ? std::atof(value.at(n).c_str()) : d; }
    long getl(const std::string& n, long d) const { return has(n) ? std::atol(value.at(n).c_str()) : d; }
    void print_help() const {
        for (auto& kv : help) {
            std::cout << "-" << kv.first;
            for (size_t i = kv.first.size() + 1; i < 16; ++i) std::cout << " ";
            std::cout << kv.second << "\n";
        }
    }
};

// cmdline.h getStrValues: comma / semicolon separated tokens
std::vector<std::string> split_strs(const std::string& s) {
    std::vector<std::string> out;
    std::string cur;
    for (char ch : s) {
        if (ch == ',' || ch == ';') {
            out.push_back(cur);
            cur.clear();
        } else {
            cur += ch;
        }
    }
    if (!cur.empty()) out.push_back(cur);
    return out;
}

std::vector<int> split_ints(const std::string& s) {
    std::vector<int> out;
    std::string cur;
    for (char ch : s) {
        if (ch == ',' || ch == ';') {
            out.push_back(std::atoi(cur.c_str()));
            cur.clear();
        } else {
            cur += ch;
        }
    }
    if (!cur.empty()) out.push_back(std::atoi(cur.c_str()));
    return out;
}

bool looks_libfm(const std::string& path) {
    std::ifstream f(path);
    std::string line;
    while (std::getline(f, line)) {
        size_t p = line.find_first_not_of(" \t\r");
        if (p == std::string::npos || line[p] == '#') continue;
        return line.find(':') != std::string::npos;
    }
    return false;
}

bool exists(const std::string& f) { return std::ifstream(f).good(); }

// Data::load (Data.h:112-117) takes <stem>.data/.datat/.target or <stem>.x/.xt/.y,
// each orientation only when the data set needs it, before the text file itself.
// bin/libFM's sets (libfm.cpp:132-149): -method mcmc and als (rewritten to mcmc
// first) have no row-major data, has_x = 0, so they read only the transpose
// (.xt / .datat, tools/transpose.cpp); the other methods need both files.
bool has_binary(const std::string& stem, bool has_x) { return sbmf_libfm_binary_kind(stem.c_str(), has_x, 1) > 0; }

// The row-major pair alone (.x/.y, .data/.target: tools/convert.cpp's output), with
// no transpose beside it and no text file of that name: libFM would fail to open
// <stem>; sbmf reads the pair (an extension, noted on stderr).
bool rowmajor_only(const std::string& stem) {
    return !exists(stem) && ((exists(stem + ".x") && exists(stem + ".y")) ||
                             (exists(stem + ".data") && exists(stem + ".target")));
}

void load(const std::string& path, const std::string& fmt, uint32_t item_offset, bool has_x, sbmf_ratings& r) {
    int rc;
    if (fmt == "binary" || (fmt == "auto" && has_binary(path, has_x))) {
        if (has_binary(path, has_x)) {
            rc = sbmf_load_libfm_data(path.c_str(), has_x, 1, item_offset, &r);
        } else if (rowmajor_only(path) || fmt == "binary") {
            rc = sbmf_load_libfm_binary(path.c_str(), item_offset, &r);
        } else {
            rc = sbmf_load_libfm(path.c_str(), item_offset, &r);
        }
    } else if (fmt == "auto" && rowmajor_only(path)) {
        std::cerr << "note: " << path << ": no " << (has_x ? "" : "transpose (.xt/.datat) or ")
                  << "text file of that name (bin/libFM would stop here); reading the row-major binary pair"
                  << std::endl;
        rc = sbmf_load_libfm_binary(path.c_str(), item_offset, &r);
    } else {
        const bool libfm = fmt == "libfm" || (fmt == "auto" && looks_libfm(path));
        rc = libfm ? sbmf_load_libfm(path.c_str(), item_offset, &r) : sbmf_load_triples(path.c_str(), &r);
    }
    if (rc != SBMF_OK) throw std::runtime_error(sbmf_loader_error());
}

// The users-first item offset of a libFM file loaded with offset 0 (user =
// first feature, item = raw second feature): libFM's num_user, max user id + 1
// over train and test (libfm.cpp:375).  The items are rebased onto it in place;
// a file whose item ids do not all lie above every user id has no users-first
// reading and is refused.
uint32_t users_first_offset(sbmf_ratings& tr, sbmf_ratings& te) {
    uint64_t umax = 0;
    bool any = false;
    for (const sbmf_ratings* r : {&tr, &te})
        for (uint64_t q = 0; q < r->n; ++q) {
            umax = std::max<uint64_t>(umax, r->user[q]);
            any = true;
        }
    if (!any) return 0;
    const uint32_t I = (uint32_t)(umax + 1);
    for (sbmf_ratings* r : {&tr, &te})
        for (uint64_t q = 0; q < r->n; ++q)
            if (r->item[q] < I)
                throw std::runtime_error(std::string("libFM input: ") + (r == &tr ? "train" : "test") + " case " +
                                         std::to_string(q + 1) + " has item feature id " +
                                         std::to_string(r->item[q]) + " <= the largest user feature id " +
                                         std::to_string(umax) +
                                         "; the learners read one user feature then one item feature per line, "
                                         "users first (pass -item_offset to set the split)");
    for (sbmf_ratings* r : {&tr, &te})
        for (uint64_t q = 0; q < r->n; ++q) r->item[q] -= I;
    return I;
}

struct RunState {
    std::string rmse_file;
    bool vb = false;  // online VB prints "#Iter=..\tTest=.." (fm_learn_vb_online_simultaneous.h:447)
    bool lfm = false;  // libFM's fm_learn_mcmc chain: one attribute group with w (fm_learn_mcmc.h:1140-1149)
    bool k1 = false;   // -dim k1: libFM logs wmu / wlambda (fm_learn_mcmc.h:422-431)
    bool avg_collected = false;  // the running mean divides by the collected sweeps
    uint32_t K = 0, ncol = 0;
    sbmf_ctx* ctx = nullptr;
    const sbmf_ratings* test = nullptr;
    double lo = 1.0, hi = 5.0;  // clamp of the running-mean prediction (min/max train target)
    std::vector<double> pred, sum4;  // this sweep's running mean; the prediction sums after sweep 4
    std::ofstream* rlog = nullptr;
    int verbosity = 0;
};

// -rlog: libFM's RLog columns (rlog.h:47-90) in its field order -- fm_learn::init
// (fm_learn.h:82-127), then fm_learn_mcmc::init (fm_learn_mcmc.h:1120-1149) or
// fm_learn_vb_online::init (fm_learn_vb_online.h:944-970) -- written with the
// default stream precision; fields a learner never logs print libFM's default
// (nan).  The SBPMF sampler has two hyperprior groups (users g=0, items g=1),
// which libFM would log as vmu[g,f] / vlambda[g,f] of two attribute groups.
// Our own columns follow at full precision, named sbmf_*.
void rlog_header(std::ostream& o, const RunState& rs) {
    o << "rmse\tmae\ttime_pred\ttime_learn\ttime_learn2\ttime_learn4\talpha\trmse_mcmc_this\trmse_mcmc_all";
    if (!rs.vb) o << "\trmse_mcmc_all_but5";
    const int ng = (rs.lfm || rs.vb) ? 1 : 2;
    for (int g = 0; g < ng; ++g) {
        o << "\twmu[" << g << "]\twlambda[" << g << "]";
        for (uint32_t f = 0; f < rs.K; ++f) o << "\tvmu[" << g << "," << f << "]\tvlambda[" << g << "," << f << "]";
    }
    o << "\tsbmf_iter\tsbmf_rmse_all\tsbmf_rmse_this\tsbmf_rmse_train\tsbmf_tau\tsbmf_ms_sweep\tsbmf_ms_eval\n";
}

// rmse / mae of clamp(sum * norm) against the test targets (fm_learn_mcmc_simultaneous.h:307-324)
void eval_sums(const RunState& rs, const std::vector<double>& sum, double norm, double& rmse, double& mae) {
    double se = 0.0, ae = 0.0;
    const uint64_t n = rs.test->n;
    for (uint64_t t = 0; t < n; ++t) {
        double p = sum[t] * norm;
        p = std::min(rs.hi, p);
        p = std::max(rs.lo, p);
        const double err = p - rs.test->rating[t];
        se += err * err;
        ae += std::abs(err);
    }
    rmse = std::sqrt(se / (double)n);
    mae = ae / (double)n;
}

void rlog_line(const sbmf_sweep_info* in, RunState& rs) {
    std::ostream& o = *rs.rlog;
    const double nan = std::numeric_limits<double>::quiet_NaN();
    const uint64_t n = rs.test ? rs.test->n : 0;
    double mae = nan, rmse_but5 = nan;
    if (n && !rs.vb) {
        // the running mean this sweep (clamped sums / divisor); its divisor gives the sums back
        rs.pred.resize(n);
        if (sbmf_predict(rs.ctx, rs.pred.data()) != SBMF_OK) throw std::runtime_error(sbmf_last_error(rs.ctx));
        const double div = rs.avg_collected ? (double)std::max(1u, rs.ncol) : (double)in->sweep + 1;
        std::vector<double> sum(n);
        for (uint64_t t = 0; t < n; ++t) sum[t] = rs.pred[t] * div;
        double r;
        eval_sums(rs, sum, 1.0 / div, r, mae);
        // all_but5 sums the sweeps from 5 on; libFM's normalizer 1.0/(i-5+1) is an unsigned
        // expression, so sweeps 0-3 divide by ~2^32 and sweep 4 by 0 (clamping 0 / NaN to the bounds)
        const uint32_t i = in->sweep;
        if (i == 4) rs.sum4 = sum;
        std::vector<double> but5(n, 0.0);
        if (i >= 5)
            for (uint64_t t = 0; t < n; ++t) but5[t] = sum[t] - rs.sum4[t];
        const double norm = 1.0 / (double)(uint32_t)(i - 5 + 1);
        if (i == 4) {
            std::fill(but5.begin(), but5.end(), std::numeric_limits<double>::quiet_NaN());
            eval_sums(rs, but5, 1.0, rmse_but5, r);
        } else {
            eval_sums(rs, but5, norm, rmse_but5, r);
        }
    }
    const double tl = in->ms_sweep / 1000.0;
    // online VB logs time_learn* and rmse_mcmc_this only (fm_learn_vb_online_simultaneous.h:436-450)
    o << (rs.vb ? nan : in->rmse_avg) << "\t" << mae << "\t" << nan << "\t" << tl << "\t" << tl << "\t" << tl << "\t";
    std::vector<double> h(4 * (size_t)rs.K, nan);
    double alpha = nan;
    if (!rs.vb && sbmf_get_hyper(rs.ctx, h.data(), &alpha) != SBMF_OK) throw std::runtime_error(sbmf_last_error(rs.ctx));
    o << (rs.vb ? nan : alpha) << "\t" << in->rmse_this << "\t" << (rs.vb ? nan : in->rmse_avg);
    if (!rs.vb) o << "\t" << rmse_but5;
    const uint32_t K = rs.K;
    if (rs.vb) {
        o << "\t" << nan << "\t" << nan;
        for (uint32_t f = 0; f < K; ++f) o << "\t" << nan << "\t" << nan;
    } else if (rs.lfm) {  // sbmf_get_hyper: [v_lambda | v_mu | w_lambda, w_mu | 0]
        o << "\t" << (rs.k1 ? h[2 * K + (K > 1 ? 1 : 0)] : nan) << "\t" << (rs.k1 ? h[2 * K] : nan);
        for (uint32_t f = 0; f < K; ++f) o << "\t" << h[K + f] << "\t" << h[f];
    } else {  // [sigma_u | mu_u | sigma_v | mu_v]: users g=0, items g=1
        for (int g = 0; g < 2; ++g) {
            o << "\t" << nan << "\t" << nan;
            for (uint32_t f = 0; f < K; ++f) o << "\t" << h[(2 * g + 1) * K + f] << "\t" << h[2 * g * K + f];
        }
    }
    const std::streamsize pr = o.precision(17);
    o << "\t" << in->sweep << "\t" << in->rmse_avg << "\t" << in->rmse_this << "\t" << in->rmse_train << "\t" << in->tau
      << "\t" << in->ms_sweep << "\t" << in->ms_eval << "\n";
    o.precision(pr);
    o.flush();
}

int on_sweep(const sbmf_sweep_info* in, void* user) {
    RunState* rs = static_cast<RunState*>(user);
    if (in->collected) rs->ncol++;
    if (rs->vb)
        std::cout << "#Iter=" << std::setw(3) << in->sweep << "\tTest=" << in->rmse_avg << std::endl;
    else
        std::cout << "#Iter=" << std::setw(3) << in->sweep << "\tTrain=" << in->rmse_train << "\tTest=" << in->rmse_avg
                  << std::endl;
    std::ofstream f(rs->rmse_file, std::ios_base::app);
    f << in->rmse_avg << "\n";
    if (rs->rlog) rlog_line(in, *rs);
    if (rs->verbosity > 0)
        std::cout << "  tau=" << in->tau << " sweep_ms=" << in->ms_sweep << " eval_ms=" << in->ms_eval << std::endl;
    return 0;
}

// SBMF_EXIT=guard (opt-in; round 3's default): leave through sbmf_exit_guard's
// handler (registered at main's start, before the first HIP call), so a profiler's
// exit handlers still run and the shared-library finalizers do not.  The finalizer
// fault it skipped under rocprofv3 came with RCCL linked at load time; libsbmf
// dlopens RCCL only for a multi-GPU communicator now, and the CLI exits normally
// under rocprofv3 (profiles/r04/r04s2_cli_rocprof_kernel_stats.csv).
bool g_guarded = false;
int leave(int rc) {
    std::cout.flush();
    std::cerr.flush();
    if (g_guarded) (void)sbmf_exit_guard(rc);
    return rc;
}

}  // namespace

int main(int argc, char** argv) {
    const char* em = std::getenv("SBMF_EXIT");
    g_guarded = em && std::strcmp(em, "guard") == 0 && sbmf_exit_guard(1) == SBMF_OK;
    try {
        CmdLine cl(argc, argv);
        std::cout << "----------------------------------------------------------------------------\n"
                  << "sbmf -- Scalable-BPMF Gibbs sampler for AMD Instinct MI355X (libFM command line)\n"
                  << "----------------------------------------------------------------------------" << std::endl;
        // libFM's flags (libfm.cpp:86-111)
        cl.reg("task", "r=regression [MANDATORY]");
        cl.reg("meta", "filename for meta information about data set (ignored: one user and one item group)");
        cl.reg("train", "filename for training data [MANDATORY] (SBPMF triples or libFM text)");
        cl.reg("test", "filename for test data [MANDATORY]");
        cl.reg("validation", "unused (SGDA only in libFM)");
        cl.reg("out", "filename for output: averaged test predictions");
        cl.reg("dim", "'k0,k1,k2': k0=use bias, k1=use 1-way interactions, k2=dim of 2-way interactions; default=1,1,8");
        cl.reg("regular", "'r0,r1,r2' (or one value for all) for -method als and -method mcmc -order libfm: "
                          "fixed / starting precisions of w0, w, v (libfm.cpp:484-513); default=0");
        cl.reg("init_stdev", "stdev for initialization of the factors; default: 1.0 (quirks final) / 0.1 (sbpmf2)");
        cl.reg("stdev", "unused");
        cl.reg("iter", "number of collection sweeps; default=100");
        cl.reg("learn_rate", "unused (SGD only)");
        cl.reg("method", "learning method: mcmc (SBPMF Gibbs; with -order libfm libFM's own MCMC chain) | "
                         "als (libFM's ALS) | vb (online variational Bayes, libFM's vb_online; alias vb_online); "
                         "default=mcmc");
        cl.reg("order", "-method mcmc: libfm (libFM's fm_learn_mcmc chain: f-outer, one hyperprior group, w0 / w "
                        "per -dim k0,k1, sqrt(variance) stdev; default on libFM text / binary input, as bin/libFM) | "
                        "sbpmf (the SBPMF sampler of gibbs_sbpmf_final.cpp; default on SBPMF triple input)");
        cl.reg("verbosity", "how much infos to print; default=0");
        cl.reg("rlog", "write per-sweep measurements to a TSV file; default=''");
        cl.reg("seed", "integer seed; default=1 (glibc default seed of the reference samplers)");
        cl.reg("help", "this screen");
        cl.reg("relation", "unused (block structure relations)");
        cl.reg("cache_size", "unused (binary data format)");
        // sampler settings
        cl.reg("rng", "ref (reference glibc/Leva/Marsaglia-Tsang stream; default) | philox (in-kernel, throughput)");
        cl.reg("quirks", "final (gibbs_sbpmf_final.cpp; default) | sbpmf2 | none (stdev = sqrt(variance)) | bias2 | bias22 "
                         "(biased sampler, top-level gibbs_sbpmf2.cpp / gibbs_sbpmf22.cpp; needs -dim '1,1,K')");
        cl.reg("precision", "f64 (default) | f32");
        cl.reg("burnin", "burn-in sweeps before collection; default=0");
        cl.reg("average", "running-mean divisor: default (quirk set) | collected (collected sweeps only) | "
                          "reference (sweep + 1, counts burn-in as gibbs_sbpmf_final.cpp:559 does)");
        cl.reg("format", "auto (default: libFM's binary files if present -- <name>.xt/.y or .datat/.target for "
                          "-method mcmc|als, <name>.x/.xt/.y or .data/.datat/.target for vb (Data.h:112-117) --, else "
                          "triple or libfm text) | triple | libfm | binary");
        cl.reg("item_offset", "libFM input: item feature id offset; default: libFM's num_user (max user feature "
                              "id + 1, libfm.cpp:375) for -method mcmc (libFM order) / als / vb, 0 for -order sbpmf");
        cl.reg("device", "HIP device ordinal; default=0");
        cl.reg("recompute_every", "recompute residuals from scratch every n sweeps; default=1");
        cl.reg("stream_threshold", "rows with more ratings take the streaming kernel; default=256 (f64) / 512 (f32)");
        cl.reg("split_chunk", "streaming task size; longer rows are split into chunks on several workgroups; default: "
                              "the register capacity of the workgroup shape (512 / 1024 / 2048 f64 ratings for 4 / 8 / "
                              "16 waves), larger values are capped to it");
        if (cl.has("help") || argc == 1) {
            cl.print_help();
            return leave(0);
        }
        cl.check();
        const std::string task = cl.get("task", "");
        if (task != "r") throw std::runtime_error("only -task r (regression) is supported by the SBPMF sampler");
        const std::string method = cl.get("method", "mcmc");
        const bool vb = method == "vb" || method == "vb_online";
        const std::string fmt = cl.get("format", "auto");
        if (fmt != "auto" && fmt != "triple" && fmt != "libfm" && fmt != "binary")
            throw std::runtime_error("unknown -format " + fmt);
        // bin/libFM -method mcmc runs fm_learn_mcmc on libFM data (libfm.cpp:411-419); the SBPMF
        // sampler reads the triple files of gibbs_sbpmf_final.cpp:43
        const std::string trainf = cl.get("train", "");
        // the MCMC and ALS sets carry no row-major data (libfm.cpp:140-149): they read the transpose
        const bool has_x = vb;
        const bool libfm_input = fmt == "libfm" || fmt == "binary" ||
                                 (fmt == "auto" && (has_binary(trainf, has_x) || rowmajor_only(trainf) ||
                                                    looks_libfm(trainf)));
        const std::string order = cl.get("order", libfm_input ? "libfm" : "sbpmf");
        if (order != "sbpmf" && order != "libfm") throw std::runtime_error("unknown -order " + order);
        const bool als = method == "als";
        const std::string q = cl.get("quirks", "final");
        const bool biased = q == "bias2" || q == "bias22";
        // libFM's fm_learn_mcmc learner; -quirks (the SBPMF samplers' variants) selects the SBPMF sampler
        const bool lfm = als || (method == "mcmc" && order == "libfm" && !(cl.has("quirks") && !cl.has("order")));
        if (method != "mcmc" && !vb && !als)
            throw std::runtime_error("-method " + method + " is not supported (use mcmc, als or vb)");
        if (!cl.has("train") || !cl.has("test")) throw std::runtime_error("-train and -test are mandatory");
        std::vector<int> dim = split_ints(cl.get("dim", "1,1,8"));
        if (dim.size() != 3) throw std::runtime_error("dim must have 3 numbers");
        if (dim[2] <= 0 || dim[2] > 256) throw std::runtime_error("dim k2 must be in [1,256]");
        if (vb && !(dim[0] == 1 && dim[1] == 1))
            throw std::runtime_error("the online VB learner updates w0 and the user/item w: use -dim '1,1,K'");
        if (lfm && biased) throw std::runtime_error("-quirks bias2|bias22 selects the SBPMF biased sampler, not libFM's");
        if (!vb && !lfm && !biased && (dim[0] || dim[1]))  // stdout stays libFM's
            std::cerr << "note: -order sbpmf: bias terms (k0,k1) are not sampled; the reference SBPMF sampler has "
                         "them compiled out (gibbs_sbpmf_final.cpp:276-295); -quirks bias2|bias22 selects the biased "
                         "sampler, -order libfm libFM's own chain"
                      << std::endl;
        if (biased && !(dim[0] == 1 && dim[1] == 1))
            throw std::runtime_error("the biased sampler (gibbs_sbpmf2.cpp) samples b0 and the user/item biases: "
                                     "use -dim '1,1,K'");

        sbmf_config cfg;
        sbmf_config_default(&cfg);
        cfg.num_factor = (uint32_t)dim[2];
        cfg.num_iter = (uint32_t)cl.getl("iter", 100);
        cfg.burnin = (uint32_t)cl.getl("burnin", 0);
        {
            const std::string av = cl.get("average", "default");
            if (av == "default") cfg.average = 0;
            else if (av == "collected") cfg.average = 1;
            else if (av == "reference") cfg.average = 2;
            else throw std::runtime_error("unknown -average " + av);
        }
        cfg.seed = (uint64_t)cl.getl("seed", 1);
        const std::string rng = cl.get("rng", "ref");
        cfg.rng_mode = rng == "philox" ? SBMF_RNG_PHILOX : SBMF_RNG_REFERENCE;
        // on_sweep prints and appends to files, never stops the run and reads no device state: in
        // Philox mode the next sweep's start is queued before it runs (sbmf_config.pipeline)
        cfg.pipeline = 1;
        if (q == "sbpmf2")
            cfg.quirks = SBMF_QUIRKS_SBPMF2;
        else if (q == "none")
            cfg.quirks = SBMF_QUIRKS_NONE;
        else if (q == "bias2")
            cfg.quirks = SBMF_QUIRKS_BIAS2;
        else if (q == "bias22")
            cfg.quirks = SBMF_QUIRKS_BIAS22;
        else if (q == "final")
            cfg.quirks = SBMF_QUIRKS_FINAL;
        else
            throw std::runtime_error("unknown -quirks " + q);
        cfg.precision = cl.get("precision", "f64") == "f32" ? SBMF_F32 : SBMF_F64;
        cfg.device = (int32_t)cl.getl("device", 0);
        if (cl.has("init_stdev")) cfg.init_stdev = cl.getd("init_stdev", 1.0);
        cfg.recompute_every = (uint32_t)cl.getl("recompute_every", 1);
        cfg.stream_threshold = (uint32_t)cl.getl("stream_threshold", 0);
        cfg.split_chunk = (uint32_t)cl.getl("split_chunk", 0);
        cfg.eval_train = vb ? 0 : 1;
        cfg.method = vb ? SBMF_METHOD_VB : als ? SBMF_METHOD_ALS : lfm ? SBMF_METHOD_LIBFM_MCMC : SBMF_METHOD_MCMC;
        if (lfm) {
            cfg.libfm_dim = (dim[0] ? 1u : 0u) | (dim[1] ? 2u : 0u);
            if (!cl.has("init_stdev")) cfg.init_stdev = 0.1;  // libfm.cpp:127
            std::vector<double> reg;
            for (const std::string& x : split_strs(cl.get("regular", ""))) reg.push_back(std::stod(x));
            if (reg.size() == 1) reg = {reg[0], reg[0], reg[0]};
            if (!reg.empty() && reg.size() != 3)
                throw std::runtime_error("-regular takes 'r' or 'r0,r1,r2' (no -meta groups in this build)");
            if (reg.size() == 3) {
                cfg.reg0 = reg[0];
                cfg.regw = reg[1];
                cfg.regv = reg[2];
            }
        }
        cfg.eval_test = 1;

        uint32_t off = (uint32_t)cl.getl("item_offset", 0);
        std::cout << "Loading train...\t" << std::endl;
        sbmf_ratings tr{}, te{};
        load(cl.get("train", ""), fmt, off, has_x, tr);
        std::cout << "Loading test... \t" << std::endl;
        load(cl.get("test", ""), fmt, off, has_x, te);
        // libFM's learners (fm_learn_mcmc, fm_learn_vb_online) take the file's feature ids as
        // their attribute ids: num_user = max first feature id + 1 over train and test
        // (libfm.cpp:219-221,263-265,375) and num_all_attribute = max feature id + 1 (:328).
        // With one user and one item feature per line that is the users-first layout with
        // item offset num_user, so no flag is needed (-item_offset overrides it).
        if ((lfm || vb) && libfm_input && !cl.has("item_offset")) off = users_first_offset(tr, te);

        sbmf_ctx* ctx = nullptr;
        if (sbmf_create(&cfg, &ctx) != SBMF_OK) throw std::runtime_error(sbmf_last_global_error());
        auto chk = [&](int rc) {
            if (rc != SBMF_OK) throw std::runtime_error(sbmf_last_error(ctx));
        };
        chk(sbmf_set_train(ctx, tr.n, tr.user, tr.item, tr.rating));
        chk(sbmf_set_test(ctx, te.n, te.user, te.item, te.rating));
        // libFM's attributes are the file's feature ids: users first, items from the
        // (inferred or given) item offset on
        if ((lfm || vb) && off) chk(sbmf_set_dims(ctx, off, 0));
        chk(sbmf_prepare(ctx));
        uint32_t nu, ni;
        uint64_t ntr, nte;
        chk(sbmf_get_dims(ctx, &nu, &ni, &ntr, &nte));
        std::cout << "#users=" << nu << "\t#items=" << ni << "\t#train=" << ntr << "\t#test=" << nte << "\tK=" << cfg.num_factor
                  << std::endl;

        RunState rs;
        std::ostringstream nm;
        nm << dim[0] << dim[1] << dim[2];
        // libFM names the file after "mcmc" for als too (the als switch rewrites -method, libfm.cpp:133)
        rs.rmse_file = "test_rmse_" + nm.str() + "_" + (vb ? std::string("vb_online") : std::string("mcmc"));
        rs.vb = vb;
        rs.lfm = lfm;
        rs.k1 = dim[1] != 0;
        rs.K = cfg.num_factor;
        rs.ctx = ctx;
        rs.test = &te;
        rs.avg_collected = !lfm && (cfg.average == 1 || (cfg.average == 0 && cfg.quirks == SBMF_QUIRKS_NONE));  // sbmf.cpp avg_collected
        if (lfm) {  // libFM clamps to the train target range (libfm.cpp:459-460)
            rs.lo = *std::min_element(tr.rating, tr.rating + tr.n);
            rs.hi = *std::max_element(tr.rating, tr.rating + tr.n);
        } else {
            rs.lo = cfg.clamp_lo >= 0 ? cfg.clamp_lo
                                      : (cfg.quirks == SBMF_QUIRKS_SBPMF2 || cfg.quirks == SBMF_QUIRKS_BIAS2 ? 0.5 : 1.0);
            rs.hi = cfg.clamp_hi;
        }
        { std::ofstream trunc(rs.rmse_file); }
        std::ofstream rlog;
        if (cl.has("rlog") && !cl.get("rlog", "").empty()) {
            rlog.open(cl.get("rlog", ""));
            if (!rlog.is_open()) throw std::runtime_error("Unable to open file " + cl.get("rlog", ""));
            std::cout << "logging to " << cl.get("rlog", "") << std::endl;
            rlog_header(rlog, rs);
            rs.rlog = &rlog;
        }
        rs.verbosity = (int)cl.getl("verbosity", 0);
        chk(sbmf_run(ctx, cfg.num_iter + cfg.burnin, on_sweep, &rs));
        if (cl.has("out") && !cl.get("out", "").empty()) {
            std::vector<double> pred(nte);
            chk(sbmf_predict(ctx, pred.data()));
            std::ofstream out(cl.get("out", ""));
            for (double p : pred) out << p << "\n";
        }
        sbmf_destroy(ctx);
        sbmf_free_ratings(&tr);
        sbmf_free_ratings(&te);
    } catch (const std::exception& e) {
        std::cerr << "ERROR: " << e.what() << std::endl;
        return leave(1);
    }
    return leave(0);
}
