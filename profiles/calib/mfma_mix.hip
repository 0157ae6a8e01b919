// mfma_mix.hip -- does an f32 MFMA chain on one wave slow the packed-fp32
// VALU of another wave on the same SIMD?  (The front wave's hunt runs 36
// dependent v_mfma_f32_16x16x4_f32 per channel beside the back wave's and the
// other front wave's v_pk_* stream.)
// One workgroup per CU, 4 or 8 waves: waves 0..3 (one per SIMD) run C
// independent chains of v_pk_add_f32 (or v_add_f32); waves 4..7, when
// present, run a partner stream: a dependent MFMA chain, 4 independent MFMA
// chains, or another pk_add stream.  Cycles per VALU instruction of waves 0..3
// are printed.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16 __attribute__((ext_vector_type(16)));

template <int OP, int PARTNER>
__global__ void k(float* out, unsigned long long* cyc, int n) {
    const int wave = threadIdx.x >> 6;
    float s = 0.0f;
    if (wave < 4) {
        constexpr int C = 8;
        f2 v[C];
        for (int c = 0; c < C; c++) v[c] = f2{(float)threadIdx.x * 1e-3f + c, 1.0f};
        const f2 d = f2{1e-7f, 2e-7f};
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < n; i += 16) {
#pragma unroll
            for (int u = 0; u < 16; u++) {
#pragma unroll
                for (int c = 0; c < C; c++) {
                    if (OP == 0) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(v[c]) : "v"(d));
                    if (OP == 1) asm volatile("v_add_f32 %0, %0, %1" : "+v"(v[c].x) : "v"(d.x));
                }
            }
        }
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        for (int c = 0; c < C; c++) s += v[c].x + v[c].y;
        if ((threadIdx.x & 63) == 0) atomicAdd(cyc, t1 - t0);
    } else {
        // partner: as many iterations as keep it busy for the VALU waves' whole run
        const float a = (float)threadIdx.x * 1e-3f, b = 1.0f;
        f4 acc0 = {0, 0, 0, 0}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
        f16 acc16 = {};
        f2 w = f2{a, 1.0f};
        const f2 d = f2{1e-7f, 2e-7f};
        const int m = n;
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < m; i++) {
            if (PARTNER == 1) {   // dependent chain (the hunt)
                acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc0, 0, 0, 0);
                acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc0, 0, 0, 0);
            }
            if (PARTNER == 2) {   // four independent chains
                acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc1, 0, 0, 0);
                acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc2, 0, 0, 0);
                acc3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc3, 0, 0, 0);
            }
            if (PARTNER == 4) {   // dependent 32x32x2 chain (2048 FMAs per MFMA)
                acc16 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc16, 0, 0, 0);
            }
            if (PARTNER == 5) {   // dependent 4x4x1 (16 blocks) chain
                acc0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc0, 0, 0, 0);
                acc0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc0, 0, 0, 0);
            }
            if (PARTNER == 3) {   // a packed-VALU partner of the same length
#pragma unroll
                for (int u = 0; u < 16; u++) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(w) : "v"(d));
            }
        }
        s = acc0[0] + acc1[1] + acc2[2] + acc3[3] + w.x + acc16[5];
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        if ((threadIdx.x & 63) == 0) atomicAdd(cyc + 1, t1 - t0);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP, int PARTNER>
void run(const char* name, const char* partner, float* out, unsigned long long* cyc) {
    const int n = 8192;
    (void)hipMemset(cyc, 0, 16);
    const int waves = PARTNER ? 8 : 4;
    hipLaunchKernelGGL((k<OP, PARTNER>), dim3(256), dim3(64 * waves), 0, 0, out, cyc, n);
    (void)hipDeviceSynchronize();
    unsigned long long c[2];
    (void)hipMemcpy(c, cyc, 16, hipMemcpyDeviceToHost);
    const double per_wave = (double)c[0] / (256.0 * 4);
    const double pw = (double)c[1] / (256.0 * 4);
    const double nm = PARTNER == 1 || PARTNER == 5 ? 2.0 * n : PARTNER == 2 ? 4.0 * n : PARTNER == 4 ? 1.0 * n : 16.0 * n;
    printf("%-13s 8 chains, partner %-22s cycles/instr = %.2f   partner: %.0f cycles, %.1f per instr\n", name,
           partner, per_wave / (n * 8.0), pw, PARTNER ? pw / nm : 0.0);
}

int main() {
    float* out;
    unsigned long long* cyc;
    (void)hipMalloc(&out, 256 * 512 * sizeof(float));
    (void)hipMalloc(&cyc, 16);
    for (int rep = 0; rep < 2; rep++) {
        run<0, 0>("v_pk_add_f32", "none", out, cyc);
        run<0, 1>("v_pk_add_f32", "dependent mfma chain", out, cyc);
        run<0, 2>("v_pk_add_f32", "4 mfma chains", out, cyc);
        run<0, 3>("v_pk_add_f32", "pk_add stream", out, cyc);
        run<0, 4>("v_pk_add_f32", "dep. 32x32x2 chain", out, cyc);
        run<0, 5>("v_pk_add_f32", "dep. 4x4x1 chain", out, cyc);
        run<1, 0>("v_add_f32", "none", out, cyc);
        run<1, 1>("v_add_f32", "dependent mfma chain", out, cyc);
        run<1, 2>("v_add_f32", "4 mfma chains", out, cyc);
        run<1, 3>("v_add_f32", "pk_add stream", out, cyc);
    }
    return 0;
}
