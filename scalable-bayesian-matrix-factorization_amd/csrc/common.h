// common.h -- host-side helpers shared by the learner runtimes (sbmf.cpp,
// vbo.cpp): error type, HIP status checks, owning device buffers.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
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

// Owning device allocation.
struct DBuf {
    void* p = nullptr;
    size_t bytes = 0;
    DBuf() = default;
    DBuf(const DBuf&) = delete;
    DBuf& operator=(const DBuf&) = delete;
    ~DBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    void alloc(size_t b) {
        release();
        if (b == 0) b = 16;
        hipError_t e = hipMalloc(&p, b);
        if (e != hipSuccess) fail(SBMF_E_NOMEM, "hipMalloc(%zu) failed: %s", b, hipGetErrorString(e));
        bytes = b;
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
