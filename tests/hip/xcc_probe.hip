// xcc_probe.hip -- which XCD each workgroup of a persistent-shaped grid lands on.
// Reads HW_REG_XCC_ID (hwreg 20, bits [3:0]) with s_getreg_b32 and prints, per
// launch shape, the workgroups per XCD and whether blockIdx % 8 predicts the XCD
// (the dispatcher's observed round-robin: MI355X_MICROARCH.md, Workgroup dispatch).
// Used to check the per-XCD task queues of k_gres (kernels.hip) read the id right.
//   hipcc --offload-arch=gfx950 -O2 -o xcc_probe xcc_probe.hip && ./xcc_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ void probe(unsigned* out) {
    if (threadIdx.x == 0) out[blockIdx.x] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11)) & 15u;
}

int main() {
    for (int threads : {1024, 512, 256}) {
        const int grid = 256 * (1024 / threads);
        unsigned* d;
        if (hipMalloc(&d, grid * sizeof(unsigned)) != hipSuccess) return 1;
        hipLaunchKernelGGL(probe, dim3(grid), dim3(threads), 0, 0, d);
        std::vector<unsigned> h(grid);
        if (hipMemcpy(h.data(), d, grid * sizeof(unsigned), hipMemcpyDeviceToHost) != hipSuccess) return 1;
        int per[16] = {0};
        int consistent = 1;
        for (int b = 0; b < grid; ++b) {
            per[h[b] & 15]++;
            if (b >= 8 && h[b] != h[b - 8]) consistent = 0;
        }
        std::printf("threads %4d grid %4d: per XCD", threads, grid);
        for (int x = 0; x < 8; ++x) std::printf(" %d", per[x]);
        std::printf(" | other ids %d | block b and b+8 share an XCD: %s | block0 on %u\n",
                    grid - per[0] - per[1] - per[2] - per[3] - per[4] - per[5] - per[6] - per[7],
                    consistent ? "yes" : "no", h[0]);
        (void)hipFree(d);
    }
    return 0;
}
