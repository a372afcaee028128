// kernels_instr.h -- diagnostic instrumentation of the row kernels (kernels.hip).
// Never part of the product build: the Makefile pre-includes it (-include) only
// for CHECK=1 / KPROF=1 builds, which go to their own output directory
// (OUT=../build_check, ../build_kprof).  kernels.hip defines these hooks away
// when this header is absent.
#pragma once
#define SBMF_KERNELS_INSTR_H_ 1

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#ifdef SBMF_CHECK_BUILD
// CHECK=1: CHK(i, extent) validates a global index; a violation is printed (the
// first 32 over the process) and the access goes to element 0 instead, so a bad
// index is reported without faulting the device.
__device__ unsigned int g_chk_count = 0;
__device__ __noinline__ uint64_t chk_fail(uint64_t i, uint64_t lim, int line) {
    if (atomicAdd(&g_chk_count, 1u) < 32u)
        printf("[sbmf check] kernels.hip:%d index %llu >= extent %llu (block %u thread %u)\n", line,
               (unsigned long long)i, (unsigned long long)lim, blockIdx.x, threadIdx.x);
    return 0;
}
#define CHK(i, lim) ((uint64_t)(i) < (uint64_t)(lim) ? (uint64_t)(i) : chk_fail((uint64_t)(i), (uint64_t)(lim), __LINE__))
#else
#define CHK(i, lim) (i)
#endif

#ifdef SBMF_KPROF_BUILD
// KPROF=1 (run with SBMF_KPROF=1): wave 0's clock cycles per phase, added into
// a.prof / sy.prof (sbmf.cpp prints them).  k_gblock: multi-wave rows only.
// k_gres: also per chunk-count class (whole rows / 2..16 chunks / more) at
// [32 + 24*SIDE + 8*cls], slot 7 of a class counting its tasks.
#define SBMF_GBLOCK_PHASES(on)                                                   \
    unsigned long long tp_ = (a.prof && threadIdx.x == 0) ? clock64() : 0ull;   \
    auto stamp = [&](int ph) {                                                   \
        if ((on) && a.prof && threadIdx.x == 0) {                                \
            const unsigned long long now = clock64();                            \
            atomicAdd(&a.prof[ph], now - tp_);                                   \
            tp_ = now;                                                           \
        }                                                                        \
    }
#define SBMF_GRES_PHASES(nch)                                                                          \
    unsigned long long tp_ = (sy.prof && threadIdx.x == 0) ? clock64() : 0ull;                         \
    unsigned long long* const pcls_ =                                                                  \
        sy.prof ? sy.prof - 8 * SIDE + 32 + 24 * SIDE + 8 * ((nch) == 1 ? 0 : (nch) <= 16 ? 1 : 2) : nullptr; \
    if (sy.prof && threadIdx.x == 0) atomicAdd(&pcls_[7], 1ull);                                       \
    auto stamp = [&](int ph) {                                                                         \
        if (sy.prof && threadIdx.x == 0) {                                                             \
            const unsigned long long now = clock64();                                                  \
            atomicAdd(&sy.prof[ph], now - tp_);                                                        \
            atomicAdd(&pcls_[ph], now - tp_);                                                          \
            tp_ = now;                                                                                 \
        }                                                                                              \
    }
#else
#define SBMF_GBLOCK_PHASES(on) auto stamp = [](int) {}
#define SBMF_GRES_PHASES(nch) auto stamp = [](int) {}
#endif
