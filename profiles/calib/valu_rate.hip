// valu_rate.hip -- cycles per instruction of v_add_f32 / v_pk_add_f32 /
// v_pk_mul_f32 on gfx950 vs waves per SIMD and independent chains (ILP).
// One workgroup per CU (256 CUs), W waves per SIMD (blockDim = 256*W... 64*4*W).
// Each wave runs C independent chains of N dependent ops; s_memtime around it.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int OP, int C>
__global__ void k(float* out, unsigned long long* cyc, int n) {
    f2 v[C];
    for (int c = 0; c < C; c++) v[c] = f2{(float)threadIdx.x * 1e-3f + c, 1.0f};
    const f2 d = f2{1e-7f, 2e-7f};
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i += 16) {
#pragma unroll
        for (int u = 0; u < 16; u++) {
#pragma unroll
            for (int c = 0; c < C; c++) {
                if (OP == 0) asm volatile("v_add_f32 %0, %0, %1" : "+v"(v[c].x) : "v"(d.x));
                if (OP == 1) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(v[c]) : "v"(d));
                if (OP == 2) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(v[c]) : "v"(d));
                if (OP == 3) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(v[c].x) : "v"(d.x));
            }
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int c = 0; c < C; c++) s += v[c].x + v[c].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) atomicAdd(cyc, t1 - t0);
}

template <int OP, int C>
void run(const char* name, int W, float* out, unsigned long long* cyc) {
    const int n = 4096;
    (void)hipMemset(cyc, 0, 8);
    hipLaunchKernelGGL((k<OP, C>), dim3(256), dim3(256 * W), 0, 0, out, cyc, n);
    (void)hipDeviceSynchronize();
    unsigned long long c;
    (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    const double waves = 256.0 * 4 * W;
    const double per_wave = (double)c / waves;
    const double instr = (double)n * C;
    printf("%-14s chains=%2d waves/SIMD=%d  cycles/instr/wave=%.2f  SIMD cycles/instr=%.2f\n", name, C, W,
           per_wave / instr, per_wave / instr / W);
}

int main() {
    float* out;
    unsigned long long* cyc;
    (void)hipMalloc(&out, 256 * 1024 * 4 * sizeof(float));
    (void)hipMalloc(&cyc, 8);
    for (int W = 1; W <= 4; W *= 2) {
        run<0, 1>("v_add_f32", W, out, cyc);
        run<0, 8>("v_add_f32", W, out, cyc);
        run<3, 8>("v_mul_f32", W, out, cyc);
        run<3, 1>("v_mul_f32", W, out, cyc);
        run<0, 2>("v_add_f32", W, out, cyc);
        run<0, 4>("v_add_f32", W, out, cyc);
        run<1, 1>("v_pk_add_f32", W, out, cyc);
        run<1, 2>("v_pk_add_f32", W, out, cyc);
        run<1, 4>("v_pk_add_f32", W, out, cyc);
        run<1, 8>("v_pk_add_f32", W, out, cyc);
        run<2, 8>("v_pk_mul_f32", W, out, cyc);
    }
    return 0;
}
