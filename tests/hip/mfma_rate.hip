// mfma_rate.hip -- cycles per instruction on gfx950 for the ops of the
// Gram-block kernels (measurement tool, not product code):
//   v_mfma_f64_16x16x4_f64 / v_mfma_f32_16x16x4_f32 (4 independent chains),
//   f64 FMA (8 independent chains), the 16-lane DPP row sum of an f64.
// One wave per SIMD (grid = 4 x CUs x 64 threads) and 4 waves per SIMD.
// Build: hipcc -O3 --offload-arch=gfx950 -o mfma_rate mfma_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int IT = 2048;

__global__ void k_mfma64(double* out, long long* cyc, double seed) {
    d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    double a = seed + threadIdx.x * 1e-3;
    const long long t0 = clock64();
    for (int i = 0; i < IT; ++i) {
        c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, c3, 0, 0, 0);
    }
    const long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void k_mfma32(double* out, long long* cyc, double seed) {
    f4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    float a = (float)seed + threadIdx.x * 1e-3f;
    const long long t0 = clock64();
    for (int i = 0; i < IT; ++i) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, c3, 0, 0, 0);
    }
    const long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void k_fma64(double* out, long long* cyc, double seed) {
    double x[8];
    for (int j = 0; j < 8; ++j) x[j] = seed + j + threadIdx.x;
    const double m = 1.0000001, b = 1e-9;
    const long long t0 = clock64();
    for (int i = 0; i < IT; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = __builtin_fma(x[j], m, b);
    }
    const long long t1 = clock64();
    double s = 0;
    for (int j = 0; j < 8; ++j) s += x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;  // per IT: 8 FMAs
}

template <int CTRL>
__device__ __forceinline__ double dpp64(double x) {
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffLL), CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xf, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__global__ void k_row16(double* out, long long* cyc, double seed) {
    double x[8];
    for (int j = 0; j < 8; ++j) x[j] = seed + j + threadIdx.x;
    const long long t0 = clock64();
    for (int i = 0; i < IT / 8; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {  // 8 independent row16 sums
            double y = x[j];
            y += dpp64<0x121>(y);
            y += dpp64<0x122>(y);
            y += dpp64<0x124>(y);
            y += dpp64<0x128>(y);
            x[j] = y * 1e-3;
        }
    }
    const long long t1 = clock64();
    double s = 0;
    for (int j = 0; j < 8; ++j) s += x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;  // per IT/8: 8 row sums
}

int main() {
    int cus = 0, lds_blk = 0, lds_cu = 0, lds_optin = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    CK(hipDeviceGetAttribute(&lds_blk, hipDeviceAttributeMaxSharedMemoryPerBlock, 0));
    CK(hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, 0));
    (void)hipDeviceGetAttribute(&lds_optin, hipDeviceAttributeSharedMemPerBlockOptin, 0);
    printf("CUs %d, LDS per block %d B, per CU %d B, opt-in per block %d B\n", cus, lds_blk, lds_cu, lds_optin);
    const int maxb = cus * 4 * 8;
    double* out;
    long long* cyc;
    CK(hipMalloc(&out, (size_t)maxb * 64 * sizeof(double)));
    CK(hipMalloc(&cyc, (size_t)maxb * sizeof(long long)));
    long long* h = (long long*)malloc(maxb * sizeof(long long));
    struct K { const char* name; void (*fn)(double*, long long*, double); double per; };
    // per: instructions of the measured kind per loop iteration (per wave)
    K ks[] = {{"mfma_f64_16x16x4", k_mfma64, 4.0 * IT}, {"mfma_f32_16x16x4", k_mfma32, 4.0 * IT},
              {"fma_f64", k_fma64, 8.0 * IT}, {"row16_sum_f64", k_row16, 8.0 * (IT / 8)}};
    for (const K& k : ks) {
        for (int wps : {1, 4}) {
            const int nb = cus * 4 * wps;  // 64-thread blocks: wps waves per SIMD
            hipLaunchKernelGGL(k.fn, dim3(nb), dim3(64), 0, 0, out, cyc, 1.0);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h, cyc, nb * sizeof(long long), hipMemcpyDeviceToHost));
            double avg = 0;
            for (int i = 0; i < nb; ++i) avg += (double)h[i];
            avg /= nb;
            printf("%-18s waves/SIMD=%d  %8.2f cycles per op per wave  (%.2f per op per SIMD)\n", k.name, wps,
                   avg / k.per, avg / k.per / wps);
        }
    }
    free(h);
    return 0;
}
