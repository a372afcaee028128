// mfma_layout.hip -- exact-integer check of the MFMA operand / accumulator
// layouts the Gram-block kernel relies on (CDNA guide §3: "check the map with
// exact integer data").  Each lane supplies the SAME value as A and B:
//   f64 16x16x4 : lane l -> S[r = l>>4][c = l&15]          (4 ratings x 16 k)
//   f32 32x32x2 : lane l -> S[r = l>>5][c = l&31]          (2 ratings x 32 k)
// so D = S^T S.  Host prints max |D - S^T S| under the assumed C/D maps.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
__global__ void k64(const double* S, double* D) {
    int l = threadIdx.x;
    double a = S[(l >> 4) * 16 + (l & 15)];
    d4 acc = {0, 0, 0, 0};
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, acc, 0, 0, 0);
    for (int j = 0; j < 4; ++j) {  // assumed: col = l&15, row = (l>>4) + 4j
        int row = (l >> 4) + 4 * j, col = l & 15;
        D[row * 16 + col] = acc[j];
    }
}
__global__ void k32(const float* S, float* D) {
    int l = threadIdx.x;
    float a = S[(l >> 5) * 32 + (l & 31)];
    f16v acc = {};
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, a, acc, 0, 0, 0);
    for (int j = 0; j < 16; ++j) {  // assumed: col = l&31, row = (j&3) + 8*(j>>2) + 4*(l>>5)
        int row = (j & 3) + 8 * (j >> 2) + 4 * (l >> 5), col = l & 31;
        D[row * 32 + col] = acc[j];
    }
}
int main() {
    double hS[64], hD[256], *dS, *dD;
    for (int i = 0; i < 64; ++i) hS[i] = (double)((i * 7 + 3) % 11) - 5.0;
    hipMalloc(&dS, sizeof hS); hipMalloc(&dD, sizeof hD);
    hipMemcpy(dS, hS, sizeof hS, hipMemcpyHostToDevice);
    k64<<<1, 64>>>(dS, dD);
    hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
    double e64 = 0;
    for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) {
        double ref = 0; for (int r = 0; r < 4; ++r) ref += hS[r * 16 + i] * hS[r * 16 + j];
        e64 = fmax(e64, fabs(ref - hD[i * 16 + j]));
    }
    float fS[64], fD[1024], *fdS, *fdD;
    for (int i = 0; i < 64; ++i) fS[i] = (float)((i * 5 + 1) % 13) - 6.f;
    hipMalloc(&fdS, sizeof fS); hipMalloc(&fdD, sizeof fD);
    hipMemcpy(fdS, fS, sizeof fS, hipMemcpyHostToDevice);
    k32<<<1, 64>>>(fdS, fdD);
    hipMemcpy(fD, fdD, sizeof fD, hipMemcpyDeviceToHost);
    double e32 = 0;
    for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) {
        double ref = 0; for (int r = 0; r < 2; ++r) ref += fS[r * 32 + i] * fS[r * 32 + j];
        e32 = fmax(e32, fabs(ref - fD[i * 32 + j]));
    }
    printf("mfma f64 16x16x4 max err %g ; f32 32x32x2 max err %g\n", e64, e32);
    return (e64 == 0 && e32 == 0) ? 0 : 1;
}
