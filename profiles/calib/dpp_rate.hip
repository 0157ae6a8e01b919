// dpp_rate.hip -- issue cost and dependent latency of the instruction kinds
// the quad Kalman step (qpsk_rx.hip qstep) is made of, one wave per SIMD and
// more: quad-perm DPP moves, DPP adds, VOP3 cndmask with an SGPR mask,
// v_rcp_f32, packed multiplies with op_sel, and a VALU write read by DPP
// right after.  Same method as valu_rate.hip: C independent chains of n
// operations, s_memtime around the loop, cycles per instruction per wave.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, true));
}

// OP: 0 v_mov_b32_dpp, 1 v_add_f32_dpp, 2 v_cndmask_b32_e64 (SGPR mask),
// 3 v_rcp_f32, 4 v_pk_mul_f32 op_sel_hi:[0,1], 5 v_add_f32 then a DPP move of
// its result (2 instructions per op), 6 v_pk_add_f32 neg_lo, 7 v_sub_f32
template <int OP, int C>
__global__ void k(float* out, unsigned long long* cyc, int n, int sel) {
    float v[C];
    f2 w[C];
    for (int c = 0; c < C; c++) {
        v[c] = (float)threadIdx.x * 1e-3f + c + 1.0f;
        w[c] = f2{v[c], 1.0f};
    }
    const float d = 1e-7f;
    const f2 d2 = f2{1e-7f, 2e-7f};
    const bool m = ((threadIdx.x >> sel) & 1) != 0;   // lane mask, SGPR pair
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i += 16) {
#pragma unroll
        for (int u = 0; u < 16; u++) {
#pragma unroll
            for (int c = 0; c < C; c++) {
                if (OP == 0) v[c] = dpp<0x93>(v[c]);
                if (OP == 1) v[c] = v[c] + dpp<0x39>(v[c]);
                if (OP == 2) { v[c] = m ? v[c] : -v[c]; asm volatile("" : "+v"(v[c])); }
                if (OP == 3) v[c] = __builtin_amdgcn_rcpf(v[c]);
                if (OP == 4) asm volatile("v_pk_mul_f32 %0, %0, %1 op_sel_hi:[0,1]" : "+v"(w[c]) : "v"(d2));
                if (OP == 5) { v[c] = v[c] + d; v[c] = dpp<0x93>(v[c]); }
                if (OP == 6) asm volatile("v_pk_add_f32 %0, %0, %1 neg_lo:[0,1]" : "+v"(w[c]) : "v"(d2));
                if (OP == 7) asm volatile("v_sub_f32 %0, %0, %1" : "+v"(v[c]) : "v"(d));
            }
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int c = 0; c < C; c++) s += v[c] + w[c].x + w[c].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) atomicAdd(cyc, t1 - t0);
}

template <int OP, int C>
void run(const char* name, int W, float* out, unsigned long long* cyc) {
    const int n = 2048;
    (void)hipMemset(cyc, 0, 8);
    hipLaunchKernelGGL((k<OP, C>), dim3(256), dim3(256 * W), 0, 0, out, cyc, n, 2);
    (void)hipDeviceSynchronize();
    unsigned long long c;
    (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    const double waves = 256.0 * 4 * W;
    const double per_wave = (double)c / waves;
    const double instr = (double)n * C;
    printf("%-26s chains=%2d waves/SIMD=%d  cycles/op/wave=%.2f  SIMD cycles/op=%.2f\n", name, C, W,
           per_wave / instr, per_wave / instr / W);
}

int main() {
    float* out;
    unsigned long long* cyc;
    (void)hipMalloc(&out, 256 * 1024 * 4 * sizeof(float));
    (void)hipMalloc(&cyc, 8);
    for (int W = 1; W <= 3; W++) {
        run<0, 1>("v_mov_b32_dpp", W, out, cyc);
        run<0, 8>("v_mov_b32_dpp", W, out, cyc);
        run<1, 1>("v_add_f32_dpp", W, out, cyc);
        run<1, 8>("v_add_f32_dpp", W, out, cyc);
        run<2, 1>("v_cndmask_b32 (sgpr mask)", W, out, cyc);
        run<2, 8>("v_cndmask_b32 (sgpr mask)", W, out, cyc);
        run<3, 1>("v_rcp_f32", W, out, cyc);
        run<3, 8>("v_rcp_f32", W, out, cyc);
        run<4, 1>("v_pk_mul_f32 op_sel", W, out, cyc);
        run<4, 8>("v_pk_mul_f32 op_sel", W, out, cyc);
        run<5, 1>("v_add_f32 + dpp mov (pair)", W, out, cyc);
        run<5, 8>("v_add_f32 + dpp mov (pair)", W, out, cyc);
        run<6, 8>("v_pk_add_f32 neg_lo", W, out, cyc);
        run<7, 8>("v_sub_f32", W, out, cyc);
    }
    return 0;
}
