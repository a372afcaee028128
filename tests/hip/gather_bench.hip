// gather_bench.hip -- ceiling of the half-sweep's partner-row gather on gfx950.
// Not part of the product: a measurement tool for DESIGN.md's roofline notes.
//
// Table: R rows x Kp doubles (row-major, like the factor tables).  N random
// row ids (uniform).  Each variant reads every rating's K values once and
// folds them into a per-lane sum (written out so nothing is elided):
//   blk8   16 lanes x 8 B per rating per 16-wide k-block, 4 ratings per
//          vector, V vectors in flight, block-outer loop (the Gram-block
//          kernels' access shape)
//   blk16  8 lanes x 16 B per rating per k-block, 8 ratings per vector
//   row16  whole rows: lanes stride over the row with 16 B loads
//          (rating-outer, all blocks of one rating back to back)
//   seq16  streaming read of the table itself (no gather): HBM/MALL reference
// Build: hipcc -O3 --offload-arch=gfx950 -o gather_bench gather_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <random>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int V>
__global__ __launch_bounds__(256) void blk8(const double* __restrict__ tab, const uint32_t* __restrict__ idx, uint64_t n,
                                            int Kp, double* __restrict__ out) {
    const int lane = threadIdx.x & 63, ci = lane & 15, rr = lane >> 4;
    const uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6;
    const uint64_t nw = (gridDim.x * (uint64_t)blockDim.x) >> 6;
    double acc = 0;
    for (uint64_t base = wave * 4 * V; base < n; base += nw * 4 * V) {
        uint32_t pj[V];
#pragma unroll
        for (int v = 0; v < V; ++v) {
            const uint64_t q = base + v * 4 + rr;
            pj[v] = q < n ? idx[q] : 0;
        }
        for (int b = 0; b < Kp; b += 16) {
            double s[V];
#pragma unroll
            for (int v = 0; v < V; ++v) s[v] = tab[(size_t)pj[v] * Kp + b + ci];
#pragma unroll
            for (int v = 0; v < V; ++v) acc += s[v];
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int V>
__global__ __launch_bounds__(256) void blk16(const double* __restrict__ tab, const uint32_t* __restrict__ idx, uint64_t n,
                                             int Kp, double* __restrict__ out) {
    const int lane = threadIdx.x & 63, ci = lane & 7, rr = lane >> 3;
    const uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6;
    const uint64_t nw = (gridDim.x * (uint64_t)blockDim.x) >> 6;
    double acc = 0;
    for (uint64_t base = wave * 8 * V; base < n; base += nw * 8 * V) {
        uint32_t pj[V];
#pragma unroll
        for (int v = 0; v < V; ++v) {
            const uint64_t q = base + v * 8 + rr;
            pj[v] = q < n ? idx[q] : 0;
        }
        for (int b = 0; b < Kp; b += 16) {
            double2 s[V];
#pragma unroll
            for (int v = 0; v < V; ++v) s[v] = *(const double2*)&tab[(size_t)pj[v] * Kp + b + 2 * ci];
#pragma unroll
            for (int v = 0; v < V; ++v) acc += s[v].x + s[v].y;
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// 8 lanes per rating cover one 16-wide block at a time (like blk16) but the
// block loop is innermost: all of a rating's blocks are issued back to back.
template <int V>
__global__ __launch_bounds__(256) void row16(const double* __restrict__ tab, const uint32_t* __restrict__ idx, uint64_t n,
                                             int Kp, double* __restrict__ out) {
    const int lane = threadIdx.x & 63, ci = lane & 7, rr = lane >> 3;
    const uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6;
    const uint64_t nw = (gridDim.x * (uint64_t)blockDim.x) >> 6;
    double acc = 0;
    const int nb = Kp / 16;
    for (uint64_t base = wave * 8 * V; base < n; base += nw * 8 * V) {
#pragma unroll
        for (int v = 0; v < V; ++v) {
            const uint64_t q = base + v * 8 + rr;
            const uint32_t pj = q < n ? idx[q] : 0;
            double2 s[8];
#pragma unroll
            for (int b = 0; b < 8; ++b)
                if (b < nb) s[b] = *(const double2*)&tab[(size_t)pj * Kp + 16 * b + 2 * ci];
#pragma unroll
            for (int b = 0; b < 8; ++b)
                if (b < nb) acc += s[b].x + s[b].y;
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ __launch_bounds__(256) void seq16(const double2* __restrict__ tab, uint64_t n2, double* __restrict__ out) {
    double acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n2; i += (uint64_t)gridDim.x * blockDim.x) {
        const double2 s = tab[i];
        acc += s.x + s.y;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main(int argc, char** argv) {
    const int R = argc > 1 ? atoi(argv[1]) : 138493;
    const int K = argc > 2 ? atoi(argv[2]) : 100;
    const uint64_t N = argc > 3 ? strtoull(argv[3], nullptr, 10) : 18000237ull;
    const int Kp = (K + 15) / 16 * 16;
    std::vector<uint32_t> h(N);
    std::mt19937_64 g(1);
    for (auto& x : h) x = (uint32_t)(g() % R);
    double *tab, *out;
    uint32_t* idx;
    const int grid = 256 * 8 * 4;
    const int max_grid = grid * 4;  // largest grid launched below: out holds one double per thread
    CK(hipMalloc(&tab, (size_t)R * Kp * 8));
    CK(hipMalloc(&idx, N * 4));
    CK(hipMalloc(&out, (size_t)max_grid * 256 * 8));
    CK(hipMemset(tab, 0, (size_t)R * Kp * 8));
    CK(hipMemcpy(idx, h.data(), N * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double gbytes = (double)N * K * 8 / 1e9;  // algorithmic partner bytes
    printf("table %d x %d f64 (%.1f MB), %llu gathers, %.2f GB algorithmic\n", R, Kp, R * (double)Kp * 8 / 1e6,
           (unsigned long long)N, gbytes);
    auto run = [&](const char* name, auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int it = 0; it < 5; ++it) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= 5;
        printf("%-10s %8.3f ms  %7.0f GB/s\n", name, ms, gbytes / (ms * 1e-3));
    };
    for (int g2 : {grid / 4, grid, grid * 4}) {
        printf("-- grid %d x 256\n", g2);
        run("blk8 V4", [&] { blk8<4><<<g2, 256>>>(tab, idx, N, Kp, out); });
        run("blk8 V8", [&] { blk8<8><<<g2, 256>>>(tab, idx, N, Kp, out); });
        run("blk16 V4", [&] { blk16<4><<<g2, 256>>>(tab, idx, N, Kp, out); });
        run("blk16 V8", [&] { blk16<8><<<g2, 256>>>(tab, idx, N, Kp, out); });
        run("row16 V2", [&] { row16<2><<<g2, 256>>>(tab, idx, N, Kp, out); });
        run("row16 V4", [&] { row16<4><<<g2, 256>>>(tab, idx, N, Kp, out); });
    }
    {
        const uint64_t n2 = (uint64_t)R * Kp / 2;
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        seq16<<<grid, 256>>>((const double2*)tab, n2, out);
        CK(hipEventRecord(a));
        for (int it = 0; it < 5; ++it) seq16<<<grid, 256>>>((const double2*)tab, n2, out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= 5;
        printf("seq16 table read %.3f ms %.0f GB/s\n", ms, n2 * 16 / (ms * 1e-3) / 1e9);
    }
    return 0;
}
