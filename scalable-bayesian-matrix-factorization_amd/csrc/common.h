// common.h -- host-side helpers shared by the learner runtimes (sbmf.cpp,
// vbo.cpp): error type, HIP status checks, owning device buffers.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/sbmf.h"

namespace sbmf {

struct Error {
    int code;
    std::string msg;
};
[[noreturn]] inline void fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    throw Error{code, buf};
}
#define HIPCHK(x)                                                                                     \
    do {                                                                                              \
        hipError_t e_ = (x);                                                                          \
        if (e_ != hipSuccess) sbmf::fail(SBMF_E_DEVICE, "%s: %s (%s:%d)", #x, hipGetErrorString(e_), \
                                         __FILE__, __LINE__);                                         \
    } while (0)

// Resource audit (sbmf_test_device_usage): what the library holds right now,
// counted where it is created and released -- device and pinned host bytes,
// streams, events, contexts and RCCL communicators.  Every stream, event and
// pinned buffer goes through the helpers below, every device buffer through DBuf.
struct Audit {
    std::atomic<long long> dev_bytes{0}, dev_allocs{0}, pinned_bytes{0}, pinned_allocs{0};
    std::atomic<long long> streams{0}, events{0}, contexts{0}, comms{0};
};
Audit& audit();
inline void stream_create(hipStream_t* s) {
    HIPCHK(hipStreamCreateWithFlags(s, hipStreamNonBlocking));
    audit().streams++;
}
inline void stream_destroy(hipStream_t& s) {
    if (!s) return;
    (void)hipStreamDestroy(s);
    audit().streams--;
    s = nullptr;
}
inline void event_create(hipEvent_t* e, unsigned flags = hipEventDefault) {
    HIPCHK(hipEventCreateWithFlags(e, flags));
    audit().events++;
}
inline void event_destroy(hipEvent_t& e) {
    if (!e) return;
    (void)hipEventDestroy(e);
    audit().events--;
    e = nullptr;
}
// pinned host memory: the byte count is kept by the caller (freed with the same size)
inline void pinned_alloc(void** p, size_t bytes) {
    HIPCHK(hipHostMalloc(p, bytes, hipHostMallocDefault));
    audit().pinned_bytes += (long long)bytes;
    audit().pinned_allocs++;
}
template <typename P>
inline void pinned_free(P*& p, size_t bytes) {
    if (!p) return;
    (void)hipHostFree((void*)p);
    audit().pinned_bytes -= (long long)bytes;
    audit().pinned_allocs--;
    p = nullptr;
}

// Owning device allocation.
struct DBuf {
    void* p = nullptr;
    size_t bytes = 0;
    DBuf() = default;
    DBuf(const DBuf&) = delete;
    DBuf& operator=(const DBuf&) = delete;
    ~DBuf() { release(); }
    void release() {
        if (p) {
            (void)hipFree(p);
            audit().dev_bytes -= (long long)bytes;
            audit().dev_allocs--;
        }
        p = nullptr;
        bytes = 0;
    }
    void alloc(size_t b) {
        release();
        if (b == 0) b = 16;
        hipError_t e = hipMalloc(&p, b);
        if (e != hipSuccess) {
            p = nullptr;
            fail(SBMF_E_NOMEM, "hipMalloc(%zu) failed: %s", b, hipGetErrorString(e));
        }
        bytes = b;
        audit().dev_bytes += (long long)b;
        audit().dev_allocs++;
    }
    void leak() {  // give the allocation up without freeing it (it stays counted as held)
        p = nullptr;
        bytes = 0;
    }
    void ensure(size_t b) {  // grow-only (per-epoch staging)
        if (b > bytes) alloc(b);
    }
    template <typename U>
    U* as() const {
        return static_cast<U*>(p);
    }
};
template <typename U>
inline void upload(DBuf& d, const std::vector<U>& h, hipStream_t st) {
    d.alloc(h.size() * sizeof(U));
    if (!h.empty()) HIPCHK(hipMemcpyAsync(d.p, h.data(), h.size() * sizeof(U), hipMemcpyHostToDevice, st));
}

// per-epoch staging: keeps the allocation when it is large enough
template <typename U>
inline void upload_grow(DBuf& d, const std::vector<U>& h, hipStream_t st) {
    d.ensure(std::max<size_t>(h.size(), 1) * sizeof(U));
    if (!h.empty()) HIPCHK(hipMemcpyAsync(d.p, h.data(), h.size() * sizeof(U), hipMemcpyHostToDevice, st));
}

}  // namespace sbmf
