// comm.cpp -- RCCL exchange (see comm.h).
#include "comm.h"
#include "common.h"

#include <rccl/rccl.h>

#include <dlfcn.h>
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <random>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

namespace sbmf {

[[noreturn]] void comm_fail(const char* what, ncclResult_t r);

// RCCL is loaded on first use (dlopen), not linked: a single-GPU process never
// maps librccl.so or runs its initialisers, and a library user without RCCL can
// still run one GPU.  The entry points are RCCL's own (rccl/rccl.h prototypes).
//
// It is opened BY PATH, from the directory of the HIP runtime this library is bound
// to: a process that imported torch has torch's bundled librccl.so (soname
// librccl.so.1) mapped already, bound to torch's own copy of libamdhip64 / the HSA
// runtime, and dlopen("librccl.so.1") returns that copy -- whose first HIP call fails
// ("ncclCommInitRank failed: unhandled cuda error", the round-5 in-suite failure:
// pytest had imported torch.distributed while collecting test_multirank_cpu.py, and
// bench.py imports it for its gloo bootstrap).  Opened by path, the system RCCL is a
// separate object whose HIP symbols bind to this library's runtime (LD_DEBUG=bindings).
// SBMF_RCCL overrides the path.
namespace {
std::string hip_runtime_dir() {
    Dl_info info{};
    if (dladdr(reinterpret_cast<void*>(&hipGetDevice), &info) && info.dli_fname) {
        std::string f(info.dli_fname);
        const size_t sl = f.rfind('/');
        if (sl != std::string::npos) return f.substr(0, sl);
    }
    return std::string();
}
void* open_rccl(std::string& where) {
    std::vector<std::string> tries;
    if (const char* e = std::getenv("SBMF_RCCL")) tries.push_back(e);
    const std::string dir = hip_runtime_dir();
    if (!dir.empty()) tries.push_back(dir + "/librccl.so.1");
    tries.push_back("librccl.so.1");  // the loader's search (no HIP runtime path found)
    std::string errs;
    for (const std::string& t : tries) {
        if (void* h = dlopen(t.c_str(), RTLD_NOW | RTLD_LOCAL)) {
            where = t;
            return h;
        }
        errs += std::string(" [") + t + ": " + dlerror() + "]";
    }
    where = errs;
    return nullptr;
}
struct Rccl {
    decltype(&::ncclGetUniqueId) GetUniqueId;
    decltype(&::ncclCommInitRank) CommInitRank;
    decltype(&::ncclCommDestroy) CommDestroy;
    decltype(&::ncclCommAbort) CommAbort;
    decltype(&::ncclGetErrorString) GetErrorString;
    decltype(&::ncclBroadcast) Broadcast;
    decltype(&::ncclSend) Send;
    decltype(&::ncclRecv) Recv;
    decltype(&::ncclAllGather) AllGather;
    decltype(&::ncclGroupStart) GroupStart;
    decltype(&::ncclGroupEnd) GroupEnd;
};
const Rccl& rccl() {
    static const Rccl r = [] {
        std::string where;
        void* h = open_rccl(where);
        if (!h) throw std::runtime_error("multi-GPU needs RCCL: dlopen failed:" + where);
        Rccl t{};
        auto sym = [&](auto& f, const char* name) {
            f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(h, name));
            if (!f) throw std::runtime_error(std::string("RCCL symbol missing: ") + name);
        };
        sym(t.GetUniqueId, "ncclGetUniqueId");
        sym(t.CommInitRank, "ncclCommInitRank");
        sym(t.CommDestroy, "ncclCommDestroy");
        sym(t.CommAbort, "ncclCommAbort");
        sym(t.GetErrorString, "ncclGetErrorString");
        sym(t.Broadcast, "ncclBroadcast");
        sym(t.Send, "ncclSend");
        sym(t.Recv, "ncclRecv");
        sym(t.AllGather, "ncclAllGather");
        sym(t.GroupStart, "ncclGroupStart");
        sym(t.GroupEnd, "ncclGroupEnd");
        return t;
    }();
    return r;
}
}  // namespace

const char* rccl_error_string(int r) { return rccl().GetErrorString((ncclResult_t)r); }

namespace {
const char kHostMagic[8] = {'S', 'B', 'M', 'F', 'H', 'O', 'S', 'T'};
constexpr size_t kHostHeader = 128;         // barrier counters
constexpr size_t kHostWindow = 64ull << 20;  // bytes exchanged per round
struct HostBarrier {
    std::atomic<int> count;
    std::atomic<int> sense;
};
std::string host_name(const uint8_t id[128]) {
    uint64_t tok;
    std::memcpy(&tok, id + 8, 8);
    return "/sbmf_" + std::to_string(tok);
}
}  // namespace

Comm::~Comm() {
    if (comm_) {
        (void)rccl().CommDestroy((ncclComm_t)comm_);
        audit().comms--;
    }
    if (shm_) munmap(shm_, shm_bytes_);
}

void Comm::abort() {
    if (!comm_) return;
    (void)rccl().CommAbort((ncclComm_t)comm_);
    audit().comms--;
    comm_ = nullptr;
}

namespace {
// ncclCommInitRank's failure, with what this process holds at that moment: free
// device memory and the library's live resources (the audit of common.h)
[[noreturn]] void init_fail(ncclResult_t r) {
    size_t fr = 0, tot = 0;
    (void)hipMemGetInfo(&fr, &tot);
    const Audit& a = audit();
    fail(SBMF_E_COMM,
         "ncclCommInitRank failed: %s [device free %.1f of %.1f GiB; library holds %lld contexts, %lld streams, "
         "%lld events, %lld device buffers (%.1f MiB), %lld pinned buffers (%.1f MiB), %lld RCCL communicators]",
         rccl_error_string((int)r), fr / 1073741824.0, tot / 1073741824.0, a.contexts.load(), a.streams.load(),
         a.events.load(), a.dev_allocs.load(), a.dev_bytes.load() / 1048576.0, a.pinned_allocs.load(),
         a.pinned_bytes.load() / 1048576.0, a.comms.load());
}
}  // namespace

void Comm::unique_id(uint8_t id[128]) {
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    const char* mode = std::getenv("SBMF_COMM");
    if (mode && std::string(mode) == "host") {
        std::memset(id, 0, 128);
        std::memcpy(id, kHostMagic, 8);
        std::random_device rd;
        const uint64_t tok = ((uint64_t)rd() << 32) ^ rd() ^ (uint64_t)getpid() ^
                             (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count();
        std::memcpy(id + 8, &tok, 8);
        return;
    }
    ncclUniqueId u;
    ncclResult_t r = rccl().GetUniqueId(&u);
    if (r != ncclSuccess) comm_fail("ncclGetUniqueId", r);
    std::memcpy(id, &u, 128);
}

void Comm::host_barrier() {
    HostBarrier* b = reinterpret_cast<HostBarrier*>(shm_);
    sense_ ^= 1;
    if (b->count.fetch_add(1) == nranks_ - 1) {
        b->count.store(0);
        b->sense.store(sense_);
    } else {
        const auto t0 = std::chrono::steady_clock::now();
        while (b->sense.load() != sense_) {
            sched_yield();
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120))
                throw std::runtime_error("host comm barrier timed out (a rank is gone)");
        }
    }
}

void Comm::init(int nranks, int rank, const uint8_t id[128]) {
    nranks_ = nranks;
    rank_ = rank;
    if (std::memcmp(id, kHostMagic, 8) == 0) {
        const std::string name = host_name(id);
        shm_bytes_ = kHostHeader + kHostWindow;
        const int fd = shm_open(name.c_str(), O_CREAT | O_RDWR, 0600);
        if (fd < 0) throw std::runtime_error("shm_open " + name + " failed");
        if (ftruncate(fd, (off_t)shm_bytes_) != 0) {
            close(fd);
            throw std::runtime_error("ftruncate of the host comm segment failed");
        }
        void* p = mmap(nullptr, shm_bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (p == MAP_FAILED) throw std::runtime_error("mmap of the host comm segment failed");
        shm_ = static_cast<unsigned char*>(p);
        host_barrier();  // every rank has mapped the segment: the name can go
        if (rank_ == 0) shm_unlink(name.c_str());
        return;
    }
    ncclUniqueId u;
    std::memcpy(&u, id, 128);
    ncclComm_t c;
    ncclResult_t r = rccl().CommInitRank(&c, nranks, u, rank);
    if (r != ncclSuccess) init_fail(r);
    comm_ = c;
    audit().comms++;
}

void Comm::init_loopback() {
    ncclUniqueId u;
    ncclResult_t r = rccl().GetUniqueId(&u);
    if (r != ncclSuccess) comm_fail("ncclGetUniqueId", r);
    ncclComm_t c;
    r = rccl().CommInitRank(&c, 1, u, 0);
    if (r != ncclSuccess) init_fail(r);
    comm_ = c;
    audit().comms++;
    nranks_ = 1;
    rank_ = 0;
    loopback_ = true;
}

void Comm::bcast_ranges(void* base, size_t unit_bytes, const std::vector<uint64_t>& bounds, hipStream_t st) {
    if (!live()) return;
    if (shm_) {  // host backend: windows of the whole range through the segment
        if (hipStreamSynchronize(st) != hipSuccess) throw std::runtime_error("hipStreamSynchronize failed");
        unsigned char* win = shm_ + kHostHeader;
        const size_t lo = (size_t)bounds[0] * unit_bytes, hi = (size_t)bounds[nranks_] * unit_bytes;
        const size_t mlo = (size_t)bounds[rank_] * unit_bytes, mhi = (size_t)bounds[rank_ + 1] * unit_bytes;
        char* dev = static_cast<char*>(base);
        for (size_t w0 = lo; w0 < hi; w0 += kHostWindow) {
            const size_t w1 = std::min(hi, w0 + kHostWindow);
            const size_t a = std::max(w0, mlo), b = std::min(w1, mhi);
            if (a < b && hipMemcpy(win + (a - w0), dev + a, b - a, hipMemcpyDeviceToHost) != hipSuccess)
                throw std::runtime_error("host comm: D2H failed");
            host_barrier();
            if (a < b) {
                if (w0 < a && hipMemcpy(dev + w0, win, a - w0, hipMemcpyHostToDevice) != hipSuccess)
                    throw std::runtime_error("host comm: H2D failed");
                if (b < w1 && hipMemcpy(dev + b, win + (b - w0), w1 - b, hipMemcpyHostToDevice) != hipSuccess)
                    throw std::runtime_error("host comm: H2D failed");
            } else if (hipMemcpy(dev + w0, win, w1 - w0, hipMemcpyHostToDevice) != hipSuccess) {
                throw std::runtime_error("host comm: H2D failed");
            }
            host_barrier();
        }
        return;
    }
    if (!comm_) return;
    ncclResult_t r = rccl().GroupStart();
    if (r != ncclSuccess) comm_fail("ncclGroupStart", r);
    for (int k = 0; k < nranks_; ++k) {
        const size_t bytes = (size_t)(bounds[k + 1] - bounds[k]) * unit_bytes;
        if (bytes == 0) continue;
        char* p = static_cast<char*>(base) + (size_t)bounds[k] * unit_bytes;
        r = rccl().Broadcast(p, p, bytes, ncclUint8, k, (ncclComm_t)comm_, st);
        if (r != ncclSuccess) comm_fail("ncclBroadcast", r);
    }
    r = rccl().GroupEnd();
    if (r != ncclSuccess) comm_fail("ncclGroupEnd", r);
}

void Comm::bcast_blocks(void* base, size_t unit_bytes, const std::vector<uint64_t>& starts,
                        const std::vector<uint64_t>& ends, hipStream_t st) {
    if (!live()) return;
    char* dev = static_cast<char*>(base);
    if (shm_) {  // host backend: each owner's block through the window, window by window
        if (hipStreamSynchronize(st) != hipSuccess) throw std::runtime_error("hipStreamSynchronize failed");
        unsigned char* win = shm_ + kHostHeader;
        for (int k = 0; k < nranks_; ++k) {
            const size_t lo = (size_t)starts[k] * unit_bytes, hi = (size_t)ends[k] * unit_bytes;
            for (size_t w0 = lo; w0 < hi; w0 += kHostWindow) {
                const size_t w1 = std::min(hi, w0 + kHostWindow);
                if (k == rank_ && hipMemcpy(win, dev + w0, w1 - w0, hipMemcpyDeviceToHost) != hipSuccess)
                    throw std::runtime_error("host comm: D2H failed");
                host_barrier();
                if (k != rank_ && hipMemcpy(dev + w0, win, w1 - w0, hipMemcpyHostToDevice) != hipSuccess)
                    throw std::runtime_error("host comm: H2D failed");
                host_barrier();
            }
        }
        return;
    }
    if (!comm_) return;
    ncclResult_t r = rccl().GroupStart();
    if (r != ncclSuccess) comm_fail("ncclGroupStart", r);
    for (int k = 0; k < nranks_; ++k) {
        const size_t bytes = (size_t)(ends[k] - starts[k]) * unit_bytes;
        if (bytes == 0) continue;
        char* p = dev + (size_t)starts[k] * unit_bytes;
        r = rccl().Broadcast(p, p, bytes, ncclUint8, k, (ncclComm_t)comm_, st);
        if (r != ncclSuccess) comm_fail("ncclBroadcast", r);
    }
    r = rccl().GroupEnd();
    if (r != ncclSuccess) comm_fail("ncclGroupEnd", r);
}

void Comm::alltoallv(const void* sendbuf, const std::vector<size_t>& soff, const std::vector<size_t>& scnt,
                     void* recvbuf, const std::vector<size_t>& roff, const std::vector<size_t>& rcnt, hipStream_t st) {
    if (!live()) return;
    if (shm_) {  // host backend: rank s publishes [offsets | its send buffer], every other rank takes its part
        if (hipStreamSynchronize(st) != hipSuccess) throw std::runtime_error("hipStreamSynchronize failed");
        unsigned char* win = shm_ + kHostHeader;
        const size_t hdr = 16 * (size_t)nranks_;
        for (int s = 0; s < nranks_; ++s) {
            if (rank_ == s) {
                size_t* h = reinterpret_cast<size_t*>(win);
                for (int k = 0; k < nranks_; ++k) {
                    h[2 * k] = soff[k];
                    h[2 * k + 1] = scnt[k];
                }
                size_t end = 0;
                for (int k = 0; k < nranks_; ++k)
                    if (k != rank_ && scnt[k]) end = std::max(end, soff[k] + scnt[k]);
                if (hdr + end > kHostWindow) throw std::runtime_error("host comm: exchange larger than the window");
                if (end && hipMemcpy(win + hdr, sendbuf, end, hipMemcpyDeviceToHost) != hipSuccess)
                    throw std::runtime_error("host comm: D2H failed");
            }
            host_barrier();
            if (rank_ != s && rcnt[s]) {
                const size_t* h = reinterpret_cast<const size_t*>(win);
                if (h[2 * rank_ + 1] != rcnt[s]) throw std::runtime_error("host comm: exchange size mismatch");
                if (hipMemcpy(static_cast<char*>(recvbuf) + roff[s], win + hdr + h[2 * rank_], rcnt[s],
                              hipMemcpyHostToDevice) != hipSuccess)
                    throw std::runtime_error("host comm: H2D failed");
            }
            host_barrier();
        }
        return;
    }
    if (!comm_) return;
    ncclResult_t r = rccl().GroupStart();
    if (r != ncclSuccess) comm_fail("ncclGroupStart", r);
    for (int k = 0; k < nranks_; ++k) {
        if (k == rank_ && !loopback_) continue;
        if (scnt[k]) {
            r = rccl().Send(static_cast<const char*>(sendbuf) + soff[k], scnt[k], ncclUint8, k, (ncclComm_t)comm_, st);
            if (r != ncclSuccess) comm_fail("ncclSend", r);
        }
        if (rcnt[k]) {
            r = rccl().Recv(static_cast<char*>(recvbuf) + roff[k], rcnt[k], ncclUint8, k, (ncclComm_t)comm_, st);
            if (r != ncclSuccess) comm_fail("ncclRecv", r);
        }
    }
    r = rccl().GroupEnd();
    if (r != ncclSuccess) comm_fail("ncclGroupEnd", r);
}

void Comm::group_begin() {
    if (!comm_) return;
    const ncclResult_t r = rccl().GroupStart();
    if (r != ncclSuccess) comm_fail("ncclGroupStart", r);
}
void Comm::group_end() {
    if (!comm_) return;
    const ncclResult_t r = rccl().GroupEnd();
    if (r != ncclSuccess) comm_fail("ncclGroupEnd", r);
}

void Comm::allgather(const void* sendbuf, size_t bytes, void* recvbuf, hipStream_t st) {
    if (!live()) {
        if (bytes && hipMemcpyAsync(recvbuf, sendbuf, bytes, hipMemcpyDeviceToDevice, st) != hipSuccess)
            throw std::runtime_error("allgather: copy failed");
        return;
    }
    if (shm_) {  // host backend: every rank writes its block into the window, then every rank reads all of it
        if ((size_t)nranks_ * bytes > kHostWindow) throw std::runtime_error("host comm: all-gather larger than the window");
        if (hipStreamSynchronize(st) != hipSuccess) throw std::runtime_error("hipStreamSynchronize failed");
        unsigned char* win = shm_ + kHostHeader;
        if (bytes && hipMemcpy(win + (size_t)rank_ * bytes, sendbuf, bytes, hipMemcpyDeviceToHost) != hipSuccess)
            throw std::runtime_error("host comm: D2H failed");
        host_barrier();
        if (bytes && hipMemcpy(recvbuf, win, (size_t)nranks_ * bytes, hipMemcpyHostToDevice) != hipSuccess)
            throw std::runtime_error("host comm: H2D failed");
        host_barrier();
        return;
    }
    if (!comm_ || !bytes) return;
    ncclResult_t r = rccl().AllGather(sendbuf, recvbuf, bytes, ncclUint8, (ncclComm_t)comm_, st);
    if (r != ncclSuccess) comm_fail("ncclAllGather", r);
}

}  // namespace sbmf
