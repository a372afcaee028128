// mfma_f64_peak.hip -- chip-wide f64 MFMA throughput on gfx950, timed by HIP
// events over the whole grid (no per-wave clock interpretation): the number
// the Gram-route design of the streaming stage hinges on (K^2 MFMA work per
// rating vs the block-diagonal k_gres).  Variants: waves per SIMD 1/2/4/8
// (256-thread workgroups, k per CU), accumulator chains per wave 1/4/8,
// operands from registers or re-read from LDS before every MFMA.
// Build: hipcc -O3 --offload-arch=gfx950 tests/hip/mfma_f64_peak.hip -o tests/hip/mfma_f64_peak
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);                    \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int IT = 4096;

template <int NC, bool LDS>
__global__ __launch_bounds__(256) void k_peak(double* out, double seed) {
    __shared__ double sh[4][64 * 16];
    d4 c[NC];
#pragma unroll
    for (int i = 0; i < NC; ++i) c[i] = d4{0, 0, 0, 0};
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    double a = seed + threadIdx.x * 1e-3, b = seed - threadIdx.x * 1e-3;
    if (LDS) {
        for (int i = l; i < 64 * 16; i += 64) sh[w][i] = seed + i * 1e-4;
        __syncthreads();
    }
    for (int it = 0; it < IT; ++it) {
#pragma unroll
        for (int i = 0; i < NC; ++i) {
            if (LDS) {  // A and B re-read from LDS for every MFMA (as an LDS-staged Gram would)
                a = sh[w][((it + i) & 15) * 64 + l];
                b = sh[w][((it + 2 * i + 1) & 15) * 64 + l];
            }
            c[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[i], 0, 0, 0);
        }
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < NC; ++i) s += c[i][0] + c[i][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NC, bool LDS>
static void run(int cus, double* out, int wps) {
    const int nb = cus * wps;  // 256-thread workgroups: wps waves on each of a CU's 4 SIMDs
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_peak<NC, LDS>), dim3(nb), dim3(256), 0, 0, out, 1.0);  // warm
    CK(hipEventRecord(e0));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((k_peak<NC, LDS>), dim3(nb), dim3(256), 0, 0, out, 1.0);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double mfma = 5.0 * nb * 4.0 * IT * NC;  // per wave: IT * NC
    const double flop = mfma * 16 * 16 * 4 * 2;
    printf("f64 16x16x4 %s chains/wave=%d waves/SIMD=%d: %.1f TFLOP/s, %.1f cycles per MFMA per SIMD @2.4GHz\n",
           LDS ? "LDS-fed " : "register", NC, wps, flop / (ms * 1e-3) / 1e12,
           (ms * 1e-3) * 2.4e9 / (mfma / (cus * 4.0)));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    double* out;
    CK(hipMalloc(&out, (size_t)cus * 8 * 256 * sizeof(double)));
    for (int wps : {1, 2, 4, 8}) {
        run<1, false>(cus, out, wps);
        run<4, false>(cus, out, wps);
        run<8, false>(cus, out, wps);
        run<4, true>(cus, out, wps);
    }
    CK(hipFree(out));
    return 0;
}
