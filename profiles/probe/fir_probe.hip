// FIR issue-rate probe: the front's fir_dec / fir_head alone, NW waves per CU
// (one workgroup per CU), every wave filtering its own LDS block REPS times.
// Prints cycles per call per wave (s_memtime = shader clock) for 1..4 waves
// per SIMD.  Built by profiles/probe/build.sh against the product source.
#include "../../singlecarrier_amd/csrc/qpsk_rx.hip"
#include <cstdio>
#include <vector>

namespace {
constexpr int kMb = 1024;
template <int KIND>
__global__ void __launch_bounds__(1024) fir_bench(float* out, unsigned long long* cyc, int reps) {
    __shared__ __attribute__((aligned(16))) float2 Mb[16][kMb];
    __shared__ __attribute__((aligned(16))) float2 Db[8][300];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (int i = lane; i < kMb; i += 64)
        Mb[w][i] = make_float2(0.001f * (float)((i * 37 + w) % 101), -0.002f * (float)((i * 11) % 53));
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; r++) {
        if (KIND == 0) fir_dec(lane, (r * 3) & 31, Mb[w], Db[w & 7]);
        else if (KIND == 1) fir_head_at(lane, Mb[w] + 2 * (r & 7), Db[w & 7] + 188);
        else { fir_dec(lane, (r * 3) & 31, Mb[w], Db[w & 7]); fir_head_at(lane, Mb[w] + 2 * (r & 7), Db[w & 7] + 188); }
        wave_lds_sync();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[blockIdx.x * (blockDim.x >> 6) + w] = t1 - t0;
    out[blockIdx.x * blockDim.x + threadIdx.x] = Db[w & 7][lane].x + Db[w & 7][lane + 200].y;
}
}  // namespace

int main() {
    const int nb = 256, reps = 400;
    float* out;
    unsigned long long* cyc;
    hipMalloc(&out, nb * 1024 * 4);
    hipMalloc(&cyc, nb * 16 * 8);
    const char* names[3] = {"fir_dec (D, 294 pk/lane-stream)", "fir_head (196 pk)", "both (490 pk)"};
    for (int kind = 0; kind < 3; kind++) {
        for (int nw : {4, 8, 12, 16}) {
            for (int it = 0; it < 2; it++) {
                if (kind == 0) hipLaunchKernelGGL(fir_bench<0>, dim3(nb), dim3(64 * nw), 0, 0, out, cyc, reps);
                if (kind == 1) hipLaunchKernelGGL(fir_bench<1>, dim3(nb), dim3(64 * nw), 0, 0, out, cyc, reps);
                if (kind == 2) hipLaunchKernelGGL(fir_bench<2>, dim3(nb), dim3(64 * nw), 0, 0, out, cyc, reps);
            }
            std::vector<unsigned long long> h(nb * nw);
            hipMemcpy(h.data(), cyc, nb * nw * 8, hipMemcpyDeviceToHost);
            double s = 0;
            for (auto v : h) s += (double)v;
            const double per = s / h.size() / reps;
            printf("%-34s waves/SIMD %d: %8.1f cycles per call per wave, %7.1f per call per SIMD\n", names[kind],
                   nw / 4, per, per / (nw / 4));
        }
    }
    return 0;
}
