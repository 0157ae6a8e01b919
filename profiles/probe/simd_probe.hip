// Which SIMD does each wave of a workgroup land on?  One workgroup of NW waves
// per CU (LDS sized to force it), HW_ID read per wave (s_getreg, read only).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void probe(unsigned* out, int nw) {
    __shared__ float pad[36000];   // ~144 KB: one workgroup per CU
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        pad[w] = 1.0f;
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
        out[blockIdx.x * nw + w] = hw;
    }
    __syncthreads();
    if (pad[0] == 2.0f) out[0] = 0;
}
int main() {
    for (int nw : {8, 10, 12, 16}) {
        const int nb = 512;
        unsigned* d;
        hipMalloc(&d, nb * nw * 4);
        hipLaunchKernelGGL(probe, dim3(nb), dim3(64 * nw), 0, 0, d, nw);
        std::vector<unsigned> h(nb * nw);
        hipMemcpy(h.data(), d, nb * nw * 4, hipMemcpyDeviceToHost);
        // histogram of the SIMD of wave w over the blocks
        printf("waves %d: SIMD of wave w (counts over %d blocks for SIMD 0..3)\n", nw, nb);
        for (int w = 0; w < nw; w++) {
            int c[4] = {0, 0, 0, 0};
            for (int b = 0; b < nb; b++) c[(h[b * nw + w] >> 4) & 3]++;
            printf("  wave %2d: %4d %4d %4d %4d\n", w, c[0], c[1], c[2], c[3]);
        }
        // per block pattern of the first 3 blocks
        for (int b = 0; b < 3; b++) {
            printf("  block %d:", b);
            for (int w = 0; w < nw; w++) printf(" %u", (h[b * nw + w] >> 4) & 3);
            printf("\n");
        }
        hipFree(d);
    }
    return 0;
}
