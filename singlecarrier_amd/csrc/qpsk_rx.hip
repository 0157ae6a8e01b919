// qpsk_rx.hip -- MI355X receive path for the single-carrier QPSK modem.
//
// Replaces the reference's per-frame receiver qpsk_rx_frame()
// (/root/reference/src/qpsk.c:133-239) and everything it calls (fir
// src/fir.c:22-44, correlate src/qpsk.c:88-96, kalman_calculate
// src/kalman.c:85-141, train_eq/data_eq src/equalizer.c:25-90, qpsk_demod
// src/qpsk.c:268-271, scramble src/scramble.c:57-84), batched over many
// independent 8 kHz channels.  Output is bit-identical to the reference
// (gcc -O2 build): every fp32 operation is issued in the
// reference's order with no contraction (-ffp-contract=off + the pragma below),
// divisions are correctly rounded, denormals are kept.
//
// One persistent workgroup of two waves owns a group of 64 channels for every
// frame of a call (DESIGN.md "Kernels"):
//   front wave (channel after channel, LDS-staged): mixer -> RRC FIR (only the
//        290 observable outputs) -> decimation -> 128-lag preamble correlation
//        -> argmax -> equalizer window dec[mi .. mi+162] -> HBM (L2)
//   back wave (lane per channel): 128 train_eq + 31 data_eq steps of the
//        square-root Kalman equalizer, slicer, descrambler.
// The front of frame n+1 needs only rx_timing of frame n, so in iteration n the
// front wave works on frame n+1 while the back wave finishes frame n; one
// __syncthreads() per frame hands rx_timing (LDS) and the window (global) over.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <utility>
#include <vector>

#include "qpsk_batch.h"
#include "qpsk_fft.h"
#include "qpsk_consts.h"
#include "qpsk_fft_dev.h"
#include "qpsk_fft_tables.h"
#include "qpsk_hunt.h"
#include "qpsk_rcp.h"
#include "qpsk_rx_internal.h"
#include "qpsk_split.h"

#pragma clang fp contract(off)

namespace {

// A workgroup owns G groups of 64 channels: waves 0..G-1 are their back waves,
// waves G.. are front waves, FP per group (rx_kernel<G, FP>).  Every shape has
// 8 front waves, so the LDS footprint is the same; large batches use G = 4
// (256 channels per CU), smaller ones spread over more CUs with G = 2 or 1.
constexpr int kMaxGroups = 4;
constexpr int kWinStride = 168;        // window row: slot k+1 = dec[mi+k], 84 float4
constexpr int kDec = 296;
// Receiver semantics (qpsk_batch.h QPSK_MODE_*): 0 = the reference as built
// (gcc -O2 "model A" decimated_frame overflow); 1 = dec752, the
// array with the 752 entries its loop writes (NOT
// reference parity).  Only the front wave's inputs and FIR differ.
//
// front LDS (float2 units), MODE 0:
//   M = m_{n-2}[1832..1879] ++ m_{n-1}[0..1191]   (1240)  -> D_n[0..187]
//    ++ m_{n-1}[1832..1879] ++ m_n[0..103]        (152)   -> F_{n+1}[0..101]
// MODE 1:
//   M = m_{n-2}[1832..1879] ++ m_{n-1}[0..1701]   (1750)  -> D_n[0..289]
// TU (255 correlator terms, permuted) reuses M once the FIR is done.  MODE 1
// keeps one dec buffer per front wave (LDS budget); the previous channel's
// window is read from it before the FIR overwrites it (same wave, in order).
#ifndef QPSK_FB
#define QPSK_FB 15   // FIR samples per LDS batch (A/B knob)
#endif
#ifndef QPSK_RX_ATTR
#define QPSK_RX_ATTR   // A/B: e.g. __attribute__((amdgpu_num_vgpr(128))) to price a 4-wave budget
#endif
#ifndef QPSK_FRESH
#define QPSK_FRESH 0   // 1: recompute the prefetch/mixer per-lane constants at each use (register A/B knob)
#endif
#ifndef QPSK_HUNT_MFMA
#define QPSK_HUNT_MFMA 1   // 1: hunt on the matrix cores; 0: packed VALU chains (A/B knob)
#endif
#ifndef QPSK_HUNT_FILTER
#define QPSK_HUNT_FILTER 1   // 1: bf16 first pass, exact chain only when the argmax is in doubt (qpsk_hunt.h)
#endif
#ifndef QPSK_FIR_WAIT
#define QPSK_FIR_WAIT 1   // the FIRs: one lgkmcnt(0) per sample batch, not one per sample (0: A/B knob)
#endif
#ifndef QPSK_LATE_YIELD
// 4x2 fronts: the frame's last K channels at the back wave's issue priority.
// Since the anchored FIR the back is the frame's last wave (4.4% of a frame
// alone, profiles/r06_c19_stamps_c3_both.json); K = 2: C3 -0.7% over 12
// interleaved rounds (10 faster), K = 1 / 4 +-0, K = 8 +2.4%
// (profiles/r06_ly_ab.txt, r06_ly2_ab.txt); 0: off
#define QPSK_LATE_YIELD 2
#endif
#ifndef QPSK_FIR_ANCHOR
// the batched FIRs' accumulators pinned per LDS batch (anchor_f2).  Without it
// LLVM sinks every multiply-add below the batch's last wait (the FIR ran as
// rounds of loads, all the arithmetic after them, 59 samples live).  1: the
// split FIR (the 4x2 kernel: 0 VGPR spills instead of 5, C3 -1.2% over 5
// interleaved rounds, profiles/r06_anc_ab.txt); 2: every FIR (the dual shapes:
// +-0 at 8,192-32,768 channels, +1% at 4,096: not kept); 0: round 5's code
#define QPSK_FIR_ANCHOR 1
#endif
#ifndef QPSK_FRESH_SPLIT
#define QPSK_FRESH_SPLIT 1   // QPSK_FRESH of the 4x2 kernel's fronts with the split FIR (A/B knob)
#endif
#ifndef QPSK_FIR_SPLIT
// the 4x2 kernel in reference mode (MODE 0, not the head pre-pass, not the
// FFT hunt): before the hunt only dec[0..254], the entries it correlates, in
// two passes on all 64 lanes (392 packed operations instead of 490);
// dec[255..289] after it, only when the window's observable part reaches them
// (fir_split below).  The dual-chain shapes keep fir_dec + fir_head_at: their
// fronts are latency-bound and the split's extra LDS reads cost them ~1%
// (profiles/r05_split_ab.txt); 0: A/B knob; 2: every MODE-0 shape (A/B knob)
#define QPSK_FIR_SPLIT 1
#endif
#ifndef QPSK_QDMUL
#define QPSK_QDMUL 1   // quad step: rotated h times its column mask as v_mul_f32_dpp (qd_mul); 0: A/B knob
#endif
#ifndef QPSK_TRAIN_PRETAB
// 1: the lane back's preamble signs as one scalar load per step from kPreTab
// instead of ~6 scalar instructions of bit extraction (967 -> 943 instructions
// per 4 steps; C3 -0.3%, profiles/r05_pretab_data_ab.txt); 0: A/B knob
#define QPSK_TRAIN_PRETAB 1
#endif
#ifndef QPSK_DYNPRIO
// dynamic issue priority of the dual-chain back waves (rx_kernel): they train
// at the highest priority unless another back wave waits for its fronts.
// 1: quad-back shapes (-1.5% at 8,192 channels, -4% at 4,096; lane backs +1..4%:
// profiles/r03_dynprio_ab.txt); 0: off; 2: every dual-chain shape (A/B knob)
#define QPSK_DYNPRIO 1
#endif

constexpr int kM1 = 1240;
template <int MODE> struct Cfg;
template <> struct Cfg<0> { static constexpr int kM = 1392, kDecBuf = 2; };
template <> struct Cfg<1> { static constexpr int kM = 1750, kDecBuf = 1; };

// (re, im) pairs as 2-wide vectors: a complex add / complex*real product is one
// packed fp32 instruction (v_pk_add_f32 / v_pk_mul_f32: IEEE per lane, no
// fusion), and the halves never need repacking.
typedef float f2 __attribute__((ext_vector_type(2)));

constexpr unsigned long long kPreLo = qhunt::pre_mask(0), kPreHi = qhunt::pre_mask(1);

// the preamble as +-1.0f, read by the training loops as wave-uniform scalar
// loads (s_load): one per 4 steps instead of bit extraction per step
struct alignas(16) PreTab {
    float v[QK_NPRE];
};
constexpr PreTab make_pretab() {
    PreTab t{};
    for (int i = 0; i < QK_NPRE; i++) t.v[i] = ((i < 64 ? kPreLo >> i : kPreHi >> (i - 64)) & 1ull) ? 1.0f : -1.0f;
    return t;
}
__constant__ PreTab kPreTab = make_pretab();

struct RxArgs {
    const int16_t* in;       // [nch][F][1880]
    int16_t* hist;           // [nch][2][1880]: frames -2, -1 of this call
    const float2* ptab;      // [1880] mixer table P[t] * 2^-14
    const unsigned long long* ks;  // [1057] keystream bits of frame g (mod 1057)
    float2* win0;            // [nslot][168] equalizer windows, even global frames
    float2* win1;            //                                odd global frames
    int* mi0;                // [nslot] preamble position (even / odd frames)
    int* mi1;
    int* rt0;                // [nslot] rx_timing (even / odd frames)
    int* rt1;
    uint8_t* bits;           // [nch][F][62]
    uint8_t* valid;          // [nch][F]
    int32_t* trace;          // [nch][F][4] or null
    float2* soft;            // [nch][F][31] or null
    float4* jobs;            // data-symbol jobs of valid frames (rx_data_kernel)
    unsigned* njobs;         // their count (this call's counter)
    int nch, F;
    unsigned g0;             // global index of the call's first frame
    size_t jcap;             // job queue capacity (plane stride of the jobs)
    int roles;               // bit 0: back, bit 1: front (3 in production); bits 4-5:
                             // issue priority boost (0 none, 1 front, 2 back);
                             // bits 8-15: front stagger; bits 16-19: front split
    int* err;                // device error word (kErrStall)
    const float2* heads;     // [nch][F][102] head pre-pass outputs (HP), or null
};

// Diagnostic build only (-DQPSK_STAMPS): per-phase cycle sums of the front
// wave, read back with qpsk_debug_stamps().  In the product build every stamp
// is compiled out.
#ifdef QPSK_STAMPS
__device__ unsigned long long g_stamps[16];
#define STAMP_DECL unsigned long long st_acc[16] = {}; unsigned long long st_t0 = stamp_now();
#define STAMP(i) do { const unsigned long long t_ = stamp_now(); st_acc[i] += t_ - st_t0; st_t0 = t_; } while (0)
#define STAMP_FLUSH() do { if (lane == 0) for (int i_ = 0; i_ < 16; i_++) atomicAdd(&g_stamps[i_], st_acc[i_]); } while (0)
__device__ __forceinline__ unsigned long long stamp_now() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#else
#define STAMP_DECL
#define STAMP(i) do { } while (0)
#define STAMP_FLUSH() do { } while (0)
#endif

__device__ __forceinline__ float2* win_of(const RxArgs& a, unsigned g) { return (g & 1u) ? a.win1 : a.win0; }
__device__ __forceinline__ int* mi_of(const RxArgs& a, unsigned g) { return (g & 1u) ? a.mi1 : a.mi0; }
__device__ __forceinline__ int* rt_of(const RxArgs& a, unsigned g) { return (g & 1u) ? a.rt1 : a.rt0; }

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Dual-chain kernel (rx_kernel<.., DUAL = true>): per-frame progress counters
// in LDS instead of a workgroup barrier.  Every wave of the (single) workgroup
// is resident, and every counter is advanced by every frame of its producer,
// so each wait ends.  The bound keeps a logic error from hanging the GPU: a
// wait that runs out sets kErrStall in the call's device error word, which
// the host returns as QPSK_ESTALL (qpsk_rx_sync / qpsk_rx_batch /
// qpsk_stream_retrieve), so stale windows or rx_timing never pass as a result.
// The timeout is sticky per workgroup: it also sets the LDS word `dead`, and
// every later wait of the workgroup returns at once, so a broken counter costs
// one bound per workgroup, not one per frame.
constexpr unsigned kSpinBound = 1u << 22;   // ~0.1 s; a frame is ~2.5k spins
constexpr int kErrStall = 1;                // device error word bits

__device__ __forceinline__ void spin_wait(int* p, int v, int* err, int* dead,
                                          unsigned bound = kSpinBound) {
    unsigned it = 0;
    for (; it < bound; it++) {
        const int c = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        const int d = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(dead, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        if (c >= v || d != 0) break;
        __builtin_amdgcn_s_sleep(1);
    }
    if (it == bound && __lane_id() == 0) {
        __hip_atomic_store(dead, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        atomicOr(err, kErrStall);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// publish: every earlier store of this wave (LDS and global) is visible to the
// workgroup before the counter moves
__device__ __forceinline__ void signal_add(int* p, int v, int lane) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ const int16_t* frame_ptr(const RxArgs& a, int ch, int k) {
    return k >= 0 ? a.in + ((size_t)ch * a.F + k) * QK_FRAME
                  : a.hist + ((size_t)ch * 2 + (k + 2)) * QK_FRAME;
}

// ---------------------------------------------------------------- front wave
// Input of one channel for frame n: kM/2 two-sample items d, item d -> M[2d..2d+1]:
// MODE 0 (696 items):
//   d <  24 : x_{n-2}[1832 + 2d]          d < 620 : x_{n-1}[2(d-24)]
//   d < 644 : x_{n-1}[1832 + 2(d-620)]    d < 696 : x_n[2(d-644)]
// MODE 1 (875 items):
//   d <  24 : x_{n-2}[1832 + 2d]          d < 875 : x_{n-1}[2(d-24)]
// Lane l owns items l + 64i, i < kPf; i is a compile-time constant below.
template <int MODE> constexpr int kItems = Cfg<MODE>::kM / 2;
template <int MODE> constexpr int kPf = (kItems<MODE> + 63) / 64;   // 11 / 14 dwords per lane

struct Src {
    const int16_t* xm2;
    const int16_t* xm1;
    const int16_t* x0;
};

__device__ __forceinline__ Src srcs(const RxArgs& a, int ch, int n) {
    return {frame_ptr(a, ch, n - 2), frame_ptr(a, ch, n - 1), frame_ptr(a, ch, n)};
}

// which frame (0: x_{n-2}, 1: x_{n-1}, 2: x_n; -1: none) and sample index of item l + 64i
template <int MODE, int i>
__device__ __forceinline__ int item(int lane, int& t) {
    const int d = lane + 64 * i;
    if (i == 0) {
        if (lane < 24) { t = 1832 + 2 * lane; return 0; }
        t = 2 * (lane - 24);
        return 1;
    }
    if (MODE == 1) {
        if (d < kItems<1>) { t = 2 * (d - 24); return 1; }
        t = 0;
        return -1;
    }
    if (i < 9) { t = 2 * (d - 24); return 1; }
    if (i == 9) { t = d < 620 ? 2 * (d - 24) : 1832 + 2 * (d - 620); return 1; }
    if (d < 644) { t = 1832 + 2 * (d - 620); return 1; }
    if (d < kItems<0>) { t = 2 * (d - 644); return 2; }
    t = 0;
    return -1;
}

// CG: the three frames are consecutive rows of `in` (frame n >= 2): items 0
// and 10 (MODE 0), which take each lane's sample from one of two frames, are
// then addressed from one wave-uniform base with a 32-bit lane offset instead
// of a per-lane 64-bit pointer, which the quad-back kernels kept live across
// the channel loop and spilled; its reload waited for every load in flight,
// this prefetch included (profiles/r03_prefetch_ab.txt)
template <int MODE, int i, bool CG>
__device__ __forceinline__ void load_item(const Src& s, int lane, int& r) {
    int t;
    const int f = item<MODE, i>(lane, t);
    if constexpr (CG) {
        if (f >= 0) r = *reinterpret_cast<const int*>(s.xm2 + (unsigned)(f * QK_FRAME + t));
    } else {
        if (f >= 0) r = *reinterpret_cast<const int*>((f == 0 ? s.xm2 : f == 1 ? s.xm1 : s.x0) + t);
    }
}

template <int MODE, bool CG, int... I>
__device__ __forceinline__ void prefetch_seq(const Src& s, int lane, int (&r)[kPf<MODE>],
                                             std::integer_sequence<int, I...>) {
    (load_item<MODE, I, CG>(s, lane, r[I]), ...);
}

// the lane index, laundered: per-lane item offsets and signs derived from it are
// recomputed at each use (a few VALU) instead of being hoisted out of the
// channel loop as live registers
__device__ __forceinline__ int fresh_lane(int lane) {
    asm volatile("" : "+v"(lane));
    return lane;
}

template <int MODE, bool CG = false, int FR = QPSK_FRESH>
__device__ __forceinline__ void prefetch(const Src& s, int lane, int (&r)[kPf<MODE>]) {
    prefetch_seq<MODE, CG>(s, (FR & 1) ? fresh_lane(lane) : lane, r, std::make_integer_sequence<int, kPf<MODE>>{});
}

// src/qpsk.c:139-144 as (-1)^G * P[t] * (x * 2^-14), two samples per item.
// NO: frame g-1 (f == 1) is the negated one (then g-2 and g are not).  Items
// 1..9 (MODE 0) / 1..13 (MODE 1) hold frame g-1 in every lane, so their sign is
// a compile-time negation (a free source modifier); items 0 and 10 (MODE 0)
// straddle two frames per lane.
template <int MODE, int i, bool NO>
__device__ __forceinline__ void mix_item(int lane, int r, const float2* P, float2* M) {
    int t;
    const int f = item<MODE, i>(lane, t);
    if (f < 0) return;
    const float4 p = *reinterpret_cast<const float4*>(P + t);
    const float v0 = (float)(int16_t)(r & 0xffff);
    const float v1 = (float)(int16_t)(r >> 16);
    float4 o;
    constexpr bool kAllPrev = MODE == 1 ? i >= 1 : (i >= 1 && i <= 9);
    if (kAllPrev) {
        o = NO ? make_float4((-p.x) * v0, (-p.y) * v0, (-p.z) * v1, (-p.w) * v1)
               : make_float4(p.x * v0, p.y * v0, p.z * v1, p.w * v1);
    } else {
        const float sg = ((f == 1) == NO) ? -1.0f : 1.0f;   // exact sign flip
        o = make_float4((sg * p.x) * v0, (sg * p.y) * v0, (sg * p.z) * v1, (sg * p.w) * v1);
    }
    *reinterpret_cast<float4*>(M + 2 * (lane + 64 * i)) = o;
}

template <int MODE, bool NO, int... I>
__device__ __forceinline__ void mix_seq(int lane, const int (&r)[kPf<MODE>], const float2* P,
                                        float2* M, std::integer_sequence<int, I...>) {
    (mix_item<MODE, I, NO>(lane, r[I], P, M), ...);
}

template <int MODE, int FR = QPSK_FRESH>
__device__ __forceinline__ void mix(int lane, const int (&r)[kPf<MODE>], unsigned g,
                                    const float2* P, float2* M) {
    constexpr auto kSeq = std::make_integer_sequence<int, kPf<MODE>>{};
    if (FR & 2) lane = fresh_lane(lane);
    if (((g - 1u) & 1u) != 0) mix_seq<MODE, true>(lane, r, P, M, kSeq);   // frame g-1 odd
    else mix_seq<MODE, false>(lane, r, P, M, kSeq);
}

using qhunt::wave_max_u32;

// same, but volatile so the load/store optimizer does not pair it into a
// ds_read2_b64 (8 LDS cycles per pair vs 2 per ds_read_b64: MI355X_MICROARCH.md)
typedef __attribute__((address_space(3))) const volatile f2 lds_vf2;
__device__ __forceinline__ f2 ld2nt(const float2* p) {
    return *(lds_vf2*)p;   // p points into LDS
}
// an accumulator pinned in a VGPR at this point of the instruction stream
// (QPSK_FIR_ANCHOR: keeps a batch's arithmetic inside it)
__device__ __forceinline__ void anchor_f2(f2& y) { asm volatile("" : "+v"(y)); }

#ifdef QPSK_STAMPS
#define FSTAMP(i) do { const unsigned long long t_ = stamp_now(); facc[8 + (i)] += t_ - ft0; ft0 = t_; } while (0)
#define FACC_PARAM , unsigned long long (&facc)[16]
#define FACC_ARG , st_acc
#define FACC_FWD , facc
#else
#define FSTAMP(i) do { } while (0)
#define FACC_PARAM
#define FACC_ARG
#define FACC_FWD
#endif
// MODE 1 (dec752): dec_{n+1} = D_n[0..289] only; lane l makes D[5l .. 5l+4]
// from the 69 samples M[25l + rt + s] (58 lanes: 290 outputs, 490 packed
// instructions per channel like MODE 0's 188 + 102).  Lane stride 25 float2
// = 50 dwords (odd multiple of 2): the b64 reads of 32 lanes cover the 64
// banks once.
__device__ __forceinline__ void fir_dec752(int lane, int rt, const float2* M, float2* dec) {
    if (lane < QK_NDECOBS / 5) {
        const float2* b = M + 25 * lane + rt;
        f2 y[5] = {{0.0f, 0.0f}, {0.0f, 0.0f}, {0.0f, 0.0f}, {0.0f, 0.0f}, {0.0f, 0.0f}};
#pragma unroll
        for (int s0 = 0; s0 < 69; s0 += QPSK_FB) {
            f2 v[QPSK_FB];
#pragma unroll
            for (int j = 0; j < QPSK_FB; j++)
                if (s0 + j < 69) v[j] = ld2nt(b + s0 + j);
            if (QPSK_FIR_WAIT) {
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int j = 0; j < QPSK_FB; j++) {
                const int s = s0 + j;
#pragma unroll
                for (int m = 0; m < 5; m++) {
                    const int k = s - 5 * m;
                    if (s < 69 && k >= 0 && k < QK_NTAPS) y[m] = y[m] + v[j] * QK_RRC[k];
                }
            }
            if (QPSK_FIR_ANCHOR == 2) {
#pragma unroll
                for (int m = 0; m < 5; m++) anchor_f2(y[m]);
            }
        }
#pragma unroll
        for (int m = 0; m < 5; m++) {
            const f2 o = y[m] * QK_GAIN;
            dec[5 * lane + m] = make_float2(o.x, o.y);
        }
    }
}

// The FFT-correlation hunt of the QPSK_MODE_FFT_HUNT variant (cpu_ref.h
// qc_fft_hunt): S = ifft(fft(dec[0..255]) * Q) with the reference's kiss_fft
// (qpsk_fft_dev.h, bit-identical to src/fft.c), then the hunt loop of
// src/qpsk.c:172-183 over cnormf(S[l]), l < 128.  The two 256-point buffers
// reuse M (free after the FIR).  HT (LDS): twiddles forward [0, 256) and
// inverse [256, 512), Q [512, 768) as (re, im) pairs, then kf_work's input
// permutation as 256 ints.
constexpr int kFftHT = 768 * 2 + 256;   // floats
// hunt tables (floats): the bf16 pass's B table + the exact chain's p line, or
// the exact chain's B table
constexpr int kHuntTab = QPSK_HUNT_FILTER ? qhunt::kBH + qhunt::kPL : qhunt::kBT;
__device__ __forceinline__ int fft_hunt(int lane, float2* M, const float2* dec, const float* HT) {
    const qfft::cf* tw = reinterpret_cast<const qfft::cf*>(HT);
    const int* perm = reinterpret_cast<const int*>(HT + 768 * 2);
    qfft::cf* X = reinterpret_cast<qfft::cf*>(M);
    qfft::cf* Y = X + 256;
    const qfft::cf* d = reinterpret_cast<const qfft::cf*>(dec);
    for (int pos = lane; pos < 256; pos += 64) X[pos] = d[perm[pos]];   // kf_work leaves
    qfft::lds_sync();
    qfft::stages(lane, 256, X, tw, false);
    for (int pos = lane; pos < 256; pos += 64) {   // Y = X * Q, in the inverse's leaf order
        const int k = perm[pos];
        Y[pos] = qfft::mul(X[k], tw[512 + k]);
    }
    qfft::lds_sync();
    qfft::stages(lane, 256, Y, tw + 256, true);
    const qfft::cf s0 = Y[lane], s1 = Y[lane + 64];   // lags lane and 64 + lane
    const float c0 = s0.r * s0.r + s0.i * s0.i;       // cnormf, src/qpsk.c:75-80
    const float c1 = s1.r * s1.r + s1.i * s1.i;
    const unsigned k0 = c0 > 0.0f ? __float_as_uint(c0) : 0u;   // as the direct hunt below
    const unsigned k1 = c1 > 0.0f ? __float_as_uint(c1) : 0u;
    const unsigned km = wave_max_u32(max(k0, k1));
    qfft::lds_sync();   // X / Y (M) are rewritten by the next channel's mixer
    if (km == 0u) return 0;
    const unsigned long long m0 = __ballot(k0 == km), m1 = __ballot(k1 == km);
    return m0 ? __ffsll((long long)m0) - 1 : 64 + __ffsll((long long)m1) - 1;
}

// RRC (src/fir.c:36-42), outputs accumulated in tap order.  Decimated outputs
// D[o] = fir_out[5o + rt] (model A): lane l makes o = 3l..3l+2
// from the 59 samples M[15l + rt + s], read in batches of FB samples.
template <int FB = QPSK_FB>
__device__ __forceinline__ void fir_dec(int lane, int rt, const float2* M, float2* dec) {
    if (lane < 63) {
        const float2* b = M + 15 * lane + rt;
        f2 y[3] = {{0.0f, 0.0f}, {0.0f, 0.0f}, {0.0f, 0.0f}};
#pragma unroll
        for (int s0 = 0; s0 < 59; s0 += FB) {
            f2 v[FB];
#pragma unroll
            for (int j = 0; j < FB; j++)
                if (s0 + j < 59) v[j] = ld2nt(b + s0 + j);
            if (QPSK_FIR_WAIT) {   // one wait per batch instead of one per sample
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int j = 0; j < FB; j++) {
                const int s = s0 + j;
#pragma unroll
                for (int m = 0; m < 3; m++) {
                    const int k = s - 5 * m;
                    if (s < 59 && k >= 0 && k < QK_NTAPS) y[m] = y[m] + v[j] * QK_RRC[k];
                }
            }
            if (QPSK_FIR_ANCHOR == 2) {
#pragma unroll
                for (int m = 0; m < 3; m++) anchor_f2(y[m]);
            }
        }
#pragma unroll
        for (int m = 0; m < 3; m++)
            if (3 * lane + m < QK_NDEC) {
                const f2 o = y[m] * QK_GAIN;
                dec[3 * lane + m] = make_float2(o.x, o.y);
            }
    }
}

// One FIR output per lane: out = GAIN * sum_k b[k] * RRC[k], k ascending
// (the same operations in the same order as fir_dec / fir_head_at).
#ifndef QPSK_FB1
#define QPSK_FB1 8   // fir_one's samples per LDS batch (A/B knob)
#endif
__device__ __forceinline__ f2 fir_one(const float2* b) {
    f2 y = {0.0f, 0.0f};
#pragma unroll
    for (int s0 = 0; s0 < QK_NTAPS; s0 += QPSK_FB1) {
        f2 v[QPSK_FB1];
#pragma unroll
        for (int j = 0; j < QPSK_FB1; j++)
            if (s0 + j < QK_NTAPS) v[j] = ld2nt(b + s0 + j);
        if (QPSK_FIR_WAIT) {
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int j = 0; j < QPSK_FB1; j++)
            if (s0 + j < QK_NTAPS) y = y + v[j] * QK_RRC[s0 + j];
        if (QPSK_FIR_ANCHOR >= 1) anchor_f2(y);
    }
    return y * QK_GAIN;
}

// The split FIR of reference mode (QPSK_FIR_SPLIT).  dec = [D_n[0..187],
// F_{n+1}[0..101]]; the hunt correlates dec[0..254] (lags < 128 over 128
// symbols) and the window's observable entries are dec[mi .. mi+162]
// (slots past the data symbols never reach an output), so
// F_{n+1}[67..101] = dec[255..289] matter only when mi >= 93.  Every output is
// one 49-tap dot product over consecutive samples, so a lane's outputs may come
// from D or from F as long as its code is the same:
//   pass 1 (fir_dec's code: 3 outputs 5 samples apart): lanes 0..62 D[3l ..
//     3l+2] (D[188] of lane 62 discarded), lane 63 F[56], F[61], F[66];
//   pass 2 (one output per lane): F[l + (l >= 56) + (l >= 60)], 0..66 less
//     56, 61, 66;
//   after the hunt, mi >= 93: F[67 + l], l < 35 (fir_split_tail).
// 392 packed operations before the hunt (294 + 98) instead of 490, and 98 more
// for the ~27% of channels whose window reaches past dec[254].
constexpr int kSplitMi = 255 - (QK_NPRE + QK_NDSYM + 3);   // 93: mi + 162 >= 255
// LDS banks (ds_read_b64: lanes 0-31 and 32-63 are serviced apart, float2 f in
// bank pair f mod 32; MI355X_MICROARCH.md "LDS").  Pass 1's lanes 32..62 read
// M[15l + rt + s]: 31 distinct pairs, so lane 63's base must be the 32nd,
// (15*63 + rt) mod 32; its outputs F[j1], F[j1+5], F[j1+10] follow from that
// residue r: j1 = r + 32 (r <= 24) or r (both <= 56).  Pass 2 reads M[kM1 + j
// + s] for the 64 other j of [0, 66]: lanes 32..63 take j = 35..66 with each of
// pass 1's j in that range replaced by j - 32 (one j per bank pair), lanes 0..31
// the rest.  [0, 66] holds the pairs of j = 0, 1, 2 three times and pass 1's
// triple is 5 apart, so one lane group always keeps a 2-way conflict: 49 extra
// LDS cycles per channel in pass 2, none in pass 1 (before this mapping: pass 1
// lane 63 at F[56] collided for 31 of 32 rt mod 32, and pass 2's j = 64, 65
// with j = 32, 33 -- profiles/probe/fir_split_banks.py).
// The map is qpsk_split.h (split_r, split_j1, make_split_tab), checked on the
// host for every rt by tests/test_split_tab.py.
// QPSK_SPLIT_BANKS 0: the round-5 mapping (A/B knob).
#ifndef QPSK_SPLIT_BANKS
#define QPSK_SPLIT_BANKS 1
#endif
static_assert(kSplitM1 == kM1, "qpsk_split.h: F_{n+1}'s offset in M");
__constant__ SplitTab kSplitTab = make_split_tab();
constexpr int kSplitTabWords = QPSK_SPLIT_BANKS ? (int)sizeof(SplitTab) / 4 : 1;

__device__ __forceinline__ void fir_split(int lane, int rt, const float2* M, float2* dec,
                                          const uint8_t* p2tab) {
    lane = fresh_lane(lane);   // the per-lane bases below are recomputed, not kept live across the loop
#if QPSK_SPLIT_BANKS
    const int r = split_r(__builtin_amdgcn_readfirstlane(rt));
    const int j1 = split_j1(r);
    const int j2 = p2tab[r * 64 + lane];
#else
    (void)p2tab;
    constexpr int j1 = 56;
    const int j2 = lane + (lane >= 56 ? 1 : 0) + (lane >= 60 ? 1 : 0);
#endif
    {   // pass 1
        const float2* b = lane < 63 ? M + 15 * lane + rt : M + kM1 + j1;
        f2 y[3] = {{0.0f, 0.0f}, {0.0f, 0.0f}, {0.0f, 0.0f}};
#pragma unroll
        for (int s0 = 0; s0 < 59; s0 += QPSK_FB) {
            f2 v[QPSK_FB];
#pragma unroll
            for (int j = 0; j < QPSK_FB; j++)
                if (s0 + j < 59) v[j] = ld2nt(b + s0 + j);
            if (QPSK_FIR_WAIT) {
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int j = 0; j < QPSK_FB; j++) {
                const int s = s0 + j;
#pragma unroll
                for (int m = 0; m < 3; m++) {
                    const int k = s - 5 * m;
                    if (s < 59 && k >= 0 && k < QK_NTAPS) y[m] = y[m] + v[j] * QK_RRC[k];
                }
            }
            if (QPSK_FIR_ANCHOR >= 1) {
#pragma unroll
                for (int m = 0; m < 3; m++) anchor_f2(y[m]);
            }
        }
#pragma unroll
        for (int m = 0; m < 3; m++) {
            const f2 o = y[m] * QK_GAIN;
            const int d = lane < 63 ? 3 * lane + m : QK_NDEC + j1 + 5 * m;
            if (d < QK_NDEC || lane == 63) dec[d] = make_float2(o.x, o.y);
        }
    }
    {   // pass 2
        const f2 o = fir_one(M + kM1 + j2);
        dec[QK_NDEC + j2] = make_float2(o.x, o.y);
    }
}

__device__ __forceinline__ void fir_split_tail(int lane, const float2* M, float2* dec) {
    lane = fresh_lane(lane);
    if (lane < QK_NHEAD - 67) {
        const f2 o = fir_one(M + kM1 + 67 + lane);
        dec[QK_NDEC + 67 + lane] = make_float2(o.x, o.y);
    }
}

// Undecimated head F_{n+1}[j] = fir_out'[j], j < 102: lane l makes j = 2l, 2l+1
// from M[kM1 + 2l + s], s < 50, read as 16-B sample pairs (lane stride 16 B:
// ds_read_b128's lane groups cover the 64 banks once; a b64 read at that
// stride is 2-way conflicted).  It does not depend on rx_timing.
__device__ __forceinline__ void fir_head_at(int lane, const float2* H, float2* out) {
    if (lane < 51) {
        const float2* b = H + 2 * lane;
        f2 y[2] = {{0.0f, 0.0f}, {0.0f, 0.0f}};
#pragma unroll
        for (int s0 = 0; s0 < 50; s0 += 10) {
            f2 v[10];
#pragma unroll
            for (int j = 0; j < 10; j += 2) {
                const float4 q = *reinterpret_cast<const float4*>(b + s0 + j);
                v[j] = f2{q.x, q.y};
                v[j + 1] = f2{q.z, q.w};
            }
            if (QPSK_FIR_WAIT) {
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int j = 0; j < 10; j++) {
                const int s = s0 + j;
#pragma unroll
                for (int m = 0; m < 2; m++) {
                    const int k = s - m;
                    if (k >= 0 && k < QK_NTAPS) y[m] = y[m] + v[j] * QK_RRC[k];
                }
            }
            if (QPSK_FIR_ANCHOR == 2) {
#pragma unroll
                for (int m = 0; m < 2; m++) anchor_f2(y[m]);
            }
        }
        const f2 o0 = y[0] * QK_GAIN, o1 = y[1] * QK_GAIN;   // one 16-B store
        *reinterpret_cast<float4*>(out + 2 * lane) = make_float4(o0.x, o0.y, o1.x, o1.y);
    }
}

// ---------------------------------------------------------------- head pre-pass
// SURVEY.md 8f rank 4, as an execution strategy (QPSK_HEADPASS=1; not the
// default, measured slower: profiles/r03_headpass_ab.txt).  F_{n+1}[0..101],
// the undecimated FIR head that dec_{n+1} ends with, does not depend on
// rx_timing, so it is computed for every frame of the call at once, ahead of
// the serial frame loop: one wave per channel-frame mixes the 152 samples the
// head reads -- x_{n-1}[1832..1879] ++ x_n[0..103], each (-1)^k P[t] x 2^-14
// for its global frame k, as mix_item -- and runs the front's fir_head on
// them.  The fronts of the frame loop then copy the 102 outputs into dec
// instead of filtering (front_channel<.., HP>).
constexpr int kHeadM = 152;
constexpr int kHeadOut = QK_NHEAD;   // 102 outputs per channel-frame
__global__ void __launch_bounds__(256) head_kernel(const int16_t* in, const int16_t* hist,
                                                  const float2* ptab, float2* heads, int nch,
                                                  int F, unsigned g0) {
    __shared__ __attribute__((aligned(16))) float2 Mh[4][kHeadM];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const size_t cf = (size_t)blockIdx.x * 4 + w;   // channel-frame ch * F + n
    if (cf >= (size_t)nch * F) return;              // wave-uniform
    const int ch = (int)(cf / (size_t)F), n = (int)(cf % (size_t)F);
    const unsigned g = g0 + (unsigned)n;            // global index of frame n
    const int16_t* xm1 = n >= 1 ? in + ((size_t)ch * F + (n - 1)) * QK_FRAME
                                : hist + ((size_t)ch * 2 + 1) * QK_FRAME;
    const int16_t* x0 = in + ((size_t)ch * F + n) * QK_FRAME;
    float2* H = Mh[w];
    for (int e = lane; e < kHeadM / 2; e += 64) {   // item e: two samples
        const bool prev = e < 24;                   // x_{n-1} tail, else x_n head
        const int t = prev ? 1832 + 2 * e : 2 * (e - 24);
        const int r = *reinterpret_cast<const int*>((prev ? xm1 : x0) + t);
        const float4 p = *reinterpret_cast<const float4*>(ptab + t);
        const float v0 = (float)(int16_t)(r & 0xffff);
        const float v1 = (float)(int16_t)(r >> 16);
        const unsigned k = prev ? g - 1u : g;       // (-1)^k
        const float sg = (k & 1u) ? -1.0f : 1.0f;   // exact sign flip
        *reinterpret_cast<float4*>(H + 2 * e) =
            make_float4((sg * p.x) * v0, (sg * p.y) * v0, (sg * p.z) * v1, (sg * p.w) * v1);
    }
    wave_lds_sync();
    fir_head_at(lane, H, heads + cf * kHeadOut);
}

// correlate (src/qpsk.c:88-96) for all 128 lags of dec and the hunt's argmax
// (src/qpsk.c:172-183).  The T images reuse M (the FIR is done with it).
template <int MODE>
__device__ __forceinline__ int hunt(int lane, float2* M, const float2* dec, const float* BT FACC_PARAM) {
#ifdef QPSK_STAMPS
    unsigned long long ft0 = stamp_now();
#endif
    if constexpr ((MODE & 2) != 0) return fft_hunt(lane, M, dec, BT);
#if QPSK_HUNT_MFMA && QPSK_HUNT_FILTER
    // bf16 pass, exact chain when in doubt (qpsk_hunt.h hunt_index)
    bool fb;
    const int mi = qhunt::hunt_index(lane, dec, reinterpret_cast<float*>(M), BT, wave_max_u32, fb);
#ifdef QPSK_STAMPS
    facc[2] += 1;          // hunts
    facc[3] += fb ? 1 : 0; // of which the exact chain decided
#endif
    FSTAMP(2);
    return mi;
#else
#if QPSK_HUNT_MFMA
    // exact chain only (qpsk_hunt.h: bit-identical k-ordered chain)
    float* TK = reinterpret_cast<float*>(M);
    qhunt::store_t(lane, dec, TK);
    wave_lds_sync();
    FSTAMP(2);
    const qhunt::f4 acc = qhunt::correlate_bt(lane, TK, BT);
    FSTAMP(3);
    return qhunt::argmax_exact(acc, wave_max_u32, qhunt::lag_lo, qhunt::lag_hi);
#else
    // as packed VALU chains (qpsk_hunt.h correlate_valu: the same k-ordered sums)
    float2* TV = M;
    qhunt::store_tv(lane, dec, TV);
    wave_lds_sync();
    FSTAMP(2);
    const qhunt::f4 acc = qhunt::correlate_valu(lane, TV);
    FSTAMP(3);
    return qhunt::argmax_exact(acc, wave_max_u32, qhunt::lag_lo_valu, qhunt::lag_hi_valu);
#endif
#endif
}

// One channel of frame n's front: D_n (decimated with rx_timing rt), F_{n+1},
// correlation of dec_{n+1} = [D_n, F_{n+1}] and its argmax mi.
// HP (QPSK_HEADPASS): F_{n+1} comes from the head pre-pass (head_kernel), at
// `head` (global, 51 x 16 B), instead of the head FIR.
template <int MODE, bool HP = false, bool SPLIT = false>
__device__ __forceinline__ int front_channel(int lane, int rt, float2* M, float2* dec,
                                             const float* BT, const uint8_t* p2tab,
                                             const float2* head FACC_PARAM) {
#ifdef QPSK_STAMPS
    unsigned long long ft0 = stamp_now();
#endif
    if constexpr ((MODE & 1) != 0) {
        fir_dec752(lane, rt, M, dec);
        FSTAMP(0);
    } else if constexpr (HP) {
        float4 h = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (lane < kHeadOut / 2) h = reinterpret_cast<const float4*>(head)[lane];   // under the FIR
        fir_dec(lane, rt, M, dec);
        FSTAMP(0);
        if (lane < kHeadOut / 2) *reinterpret_cast<float4*>(dec + QK_NDEC + 2 * lane) = h;
    } else if constexpr (MODE == 0 && SPLIT) {
        fir_split(lane, rt, M, dec, p2tab);   // dec[0..254]
        FSTAMP(0);
        wave_lds_sync();
        FSTAMP(1);
        const int mi = hunt<MODE>(lane, M, dec, BT FACC_FWD);
        if (mi >= kSplitMi) {          // wave-uniform
            fir_split_tail(lane, M, dec);   // dec[255..289]
            wave_lds_sync();
        }
        return mi;
    } else {
        fir_dec(lane, rt, M, dec);
        FSTAMP(0);
        fir_head_at(lane, M + kM1, dec + QK_NDEC);   // F_{n+1}: M[kM1 ..] (head input)
    }
    wave_lds_sync();
    FSTAMP(1);
    return hunt<MODE>(lane, M, dec, BT FACC_FWD);
}

// window slots (2q, 2q+1) = dec[mi+2q-1], dec[mi+2q] (slot 0 unused); 84
// float4 = 1344 B per channel, full 128-B lines
__device__ __forceinline__ void store_window(int lane, int mi, const float2* dec, float2* out) {
    float4* o = reinterpret_cast<float4*>(out);
    {
        const float2 lo = dec[max(mi + 2 * lane - 1, 0)], hi = dec[mi + 2 * lane];
        o[lane] = make_float4(lo.x, lo.y, hi.x, hi.y);
    }
    if (lane < kWinStride / 2 - 64) {
        const int q = lane + 64;
        const float2 lo = dec[mi + 2 * q - 1], hi = dec[mi + 2 * q];
        o[q] = make_float4(lo.x, lo.y, hi.x, hi.y);
    }
}

// carry the samples the next call needs: x_{F-1}[0..hi), x_{F-1}[1832..1879],
// x_{F-2}[1832..1879]; hi = 1192 (MODE 0) or 1704 (MODE 1), in 8-sample units
template <int MODE>
__device__ __forceinline__ void carry_history(const int16_t* in, int16_t* hist, int F, int ch0, int nlive, int lane) {
    constexpr int kHead8 = MODE == 1 ? 213 : 149;
    for (int c = 0; c < nlive; c++) {
        const int ch = ch0 + c;
        int16_t* h0 = hist + (size_t)ch * 2 * QK_FRAME;
        int16_t* h1 = h0 + QK_FRAME;
        const int16_t* last = F >= 1 ? in + ((size_t)ch * F + (F - 1)) * QK_FRAME : h1;
        const int16_t* prev = F >= 2 ? in + ((size_t)ch * F + (F - 2)) * QK_FRAME : h1;
        if (lane < 6) {   // F == 1: prev is h1; its load completes before the h1 stores
            const int t = 1832 + 8 * lane;
            *reinterpret_cast<int4*>(h0 + t) = *reinterpret_cast<const int4*>(prev + t);
        }
        for (int u = lane; u < kHead8 + 6; u += 64) {
            const int t = u < kHead8 ? 8 * u : 1832 + 8 * (u - kHead8);
            *reinterpret_cast<int4*>(h1 + t) = *reinterpret_cast<const int4*>(last + t);
        }
    }
}

// ---------------------------------------------------------------- back role
// Complex values are f2 = (re, im).  cmul(A, C) = (ac - bd, ad + bc) with every
// product and the final sum/difference rounded once, exactly as gcc expands
// the reference's complex products for finite operands: two packed multiplies
// and one packed add (neg on the low half), no fusion.
// (a.x - b.x, a.y + b.y) as ONE v_pk_add_f32 with the low half of b negated
// (LLVM builds it from two packed adds plus moves otherwise); a + (-b) == a - b.
__device__ __forceinline__ f2 addsub(f2 a, f2 b) {
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// The two products, each ONE v_pk_mul_f32 with the broadcast/swap done by
// op_sel (written out: LLVM otherwise copies the high half to a new register
// before broadcasting it).
__device__ __forceinline__ f2 mul_xx(f2 A, f2 C) {   // (A.x * C.x, A.x * C.y)
    f2 r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(r) : "v"(A), "v"(C));
    return r;
}
__device__ __forceinline__ f2 mul_yy_swap(f2 A, f2 C) {   // (A.y * C.y, A.y * C.x)
    f2 r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0]" : "=v"(r) : "v"(A), "v"(C));
    return r;
}
__device__ __forceinline__ f2 cmul(f2 A, f2 C) {
    const f2 t1 = mul_xx(A, C);        // (ac, ad)
    const f2 t2 = mul_yy_swap(A, C);   // (bd, bc)
    return addsub(t1, t2);             // (ac - bd, ad + bc)
}
// A * conj(C) as the reference rounds it: (a*c - b*(-d), a*(-d) + b*c).  Since
// b*(-d) == -(b*d) and a*(-d) == -(a*d) exactly, that is (ac + bd, -(ad) + bc):
// the same two packed products and ONE packed add with the high half of t1 negated.
__device__ __forceinline__ f2 cmulc(f2 A, f2 C) {
    const f2 t1 = mul_xx(A, C);        // (ac, ad)
    const f2 t2 = mul_yy_swap(A, C);   // (bd, bc)
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 neg_hi:[1,0]" : "=v"(r) : "v"(t1), "v"(t2));
    return r;
}
// a + conj(b) = (a.x + b.x, a.y + (-b.y)), one packed add
__device__ __forceinline__ f2 addc(f2 a, f2 b) {
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ f2 conj2(f2 A) { return f2{A.x, -A.y}; }

struct Kal {
    f2 eq[5];                // eq_coeff     src/kalman.c:19
    f2 g[5];                 // kalman_gain  src/kalman.c:20
    f2 u[10];                // u[i][j], i < j (src/kalman.c:25), index uix(i, j)
    f2 d[5];                 // src/kalman.c:29, kept as (d, d) for packed g = f*d
};

__host__ __device__ constexpr int uix(int i, int j) { return j * (j - 1) / 2 + i; }

// kalman_calculate (src/kalman.c:85-141) then update_eq (src/equalizer.c:25-40)
// EXACT = false: the five divisions use the fast correctly-rounded reciprocal
// (qpsk_rcp.h), valid inside [2^-125, 2^125]; `bad` collects lanes whose
// operands left that range (never seen: they are >= 0.1), and the caller then
// recomputes the whole frame with EXACT = true (IEEE division).  No branch in
// the step, so the step is one basic block.
// the gain half of update_eq: kalman_calculate (src/kalman.c:85-141); returns
// kalman_y (the last 6.22 y).  It never reads eq or the error: the gain
// recursion of a frame depends only on its window.
// EXACT = false: `bmax` collects the bit pattern of the step's largest
// reciprocal operand xs[4] (the callers test bmax <= bits(2^125) once per
// frame or job: qk_rcp_in_range() for every step, a NaN or -x has larger bits).
template <bool EXACT>
__device__ __forceinline__ float kal_gain(Kal& k, const f2 (&x)[5], unsigned& bmax) {
    const float E = QK_KAL_E, q = QK_KAL_Q;
    f2 f[5];
    float a[5];
    f[0] = conj2(x[0]);                                   // 6.2  f0 = conj(x0)
#pragma unroll
    for (int j = 1; j < 5; j++) {
        // u0j*conj(x0) + conj(xj) (the double conj() sum rounds to the fp32 sum)
        f[j] = addc(cmulc(k.u[uix(0, j)], x[0]), x[j]);
#pragma unroll
        for (int i = 1; i < j; i++) f[j] = f[j] + cmulc(k.u[uix(i, j)], x[i]);
    }
#pragma unroll
    for (int j = 0; j < 5; j++) k.g[j] = f[j] * k.d[j];   // 6.4  g = f*d (both halves d)
#pragma unroll
    for (int j = 0; j < 5; j++) {                         // 6.5/6.6 Re(g * conj(f))
        // gr*fr - gi*(-fi) == gr*fr + gi*fi (gi*(-fi) == -(gi*fi) exactly)
        const f2 t = k.g[j] * f[j];
        a[j] = (j == 0 ? E : a[j - 1]) + (t.x + t.y);
    }
    const float hq = 1.0f + q;                            // 6.7
    const float ht = a[4] * q;
    // the five divisor operands of 6.19 / 6.22.  They are nondecreasing in j:
    // a_j = a_{j-1} + (gr*fr + gi*fi) and every g*conj(f) term is >= 0 (g = f*d,
    // d > 0), so xs[0] >= E = 0.1 and xs[4] is the largest; one check of xs[4]
    // (false for +inf/NaN, which propagate into a_4) covers all five
    // (qk_rcp_fast == 1.0f / x inside [2^-125, 2^125], see qpsk_rcp.h).
    float xs[5], ys[5];
#pragma unroll
    for (int j = 0; j < 5; j++) xs[j] = a[j] + ht;
    if (EXACT) {
#pragma unroll
        for (int j = 0; j < 5; j++) ys[j] = qk_div_ieee(xs[j]);
    } else {
        // the one check: xs[0] >= E unless NaN, and a NaN reaches xs[4] too
        bmax = max(bmax, __float_as_uint(xs[4]));
        // (the Newton steps as packed pairs: 15 fewer instructions per 4
        // steps but 4 more spilled VGPRs in the 4x2 kernel, C3 +0.8%,
        // profiles/r05_knobs_ab.txt, code in commit 868e9f0)
#pragma unroll
        for (int j = 0; j < 5; j++) ys[j] = qk_rcp_fast(xs[j]);
    }
    float y = ys[0];                                      // 6.19
    k.d[0] = k.d[0] * ((hq * (E + ht)) * y);              // 6.20 (both halves)
#pragma unroll
    for (int j = 1; j < 5; j++) {
        const float B = a[j - 1] + ht;                    // 6.21
        const f2 h = (-f[j]) * y;                         // 6.11
        y = ys[j];                                        // 6.22
        k.d[j] = k.d[j] * ((hq * B) * y);                 // 6.13
#pragma unroll
        for (int i = 0; i < j; i++) {
            const f2 B1 = k.u[uix(i, j)];
            k.u[uix(i, j)] = B1 + cmulc(h, k.g[i]);          // 6.15
            k.g[i] = k.g[i] + cmulc(k.g[j], B1);             // 6.16
        }
    }
    return y;
}

// update_eq (src/equalizer.c:25-40): the gain, then error *= kalman_y and
// eq_i += error * conj(g_i)
template <bool EXACT>
__device__ __forceinline__ void update_eq(Kal& k, const f2 (&x)[5], f2 e, unsigned& bmax) {
    const float y = kal_gain<EXACT>(k, x, bmax);
    e = e * y;                                            // error *= kalman_y
#pragma unroll
    for (int i = 0; i < 5; i++) k.eq[i] = k.eq[i] + cmulc(e, k.g[i]);
}

// A valid frame handed from the back wave to rx_data_kernel: the window
// samples of its data symbols, the equalizer state after the 128 training
// steps, and where its outputs go.  112 floats (28 x 16 B), plane-major: 16-B
// word q of job slot s is at jobs[q * cap + s] (cap = the queue's capacity), so
// the lanes of a wave, which hold consecutive slots, read and write adjacent
// 16-B words (one uncoalesced 448-B job per lane touched 64 cache lines per
// load instruction):
//   [0, 70)  x = dec[mi+128+t], t < 35, as (re, im)
//   [70, 80) eq[5]   [80, 100) u[10]   [100, 105) d[5] (one copy of each)
//   [105, 107) cf (channel-frame index, 64-bit)   [107] keystream frame index
constexpr int kJobF4 = 28;
struct DataJob {
    Kal k;
    size_t cf;
    unsigned ks;
};

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// one job float (compile-time index i < 112) from its source
__device__ __forceinline__ float job_word(int i, const DataJob& j, const float* xf) {
    if (i < 70) return xf[i];
    if (i < 80) return (i & 1) ? j.k.eq[(i - 70) >> 1].y : j.k.eq[(i - 70) >> 1].x;
    if (i < 100) return (i & 1) ? j.k.u[(i - 80) >> 1].y : j.k.u[(i - 80) >> 1].x;
    if (i < 105) return j.k.d[i - 100].x;
    if (i == 105) return __uint_as_float((unsigned)(j.cf & 0xffffffffu));
    if (i == 106) return __uint_as_float((unsigned)(j.cf >> 32));
    if (i == 107) return __uint_as_float(j.ks);
    return 0.0f;
}

// Streamed: each 16-B store right after the window loads it needs (the job
// queue may alias the window as far as the compiler knows, so staging the
// whole job first would hold all 112 floats in registers).
// Addresses: plane base (wave-uniform, SGPRs) + 32-bit lane byte offset slot * 16
// (global_load/store saddr form; the queue holds < 2^28 jobs, qpsk_rx_batch_device).
__device__ __forceinline__ const char* job_plane(const float4* jobs, size_t cap, int q) {
    return reinterpret_cast<const char*>(jobs) + (size_t)q * cap * sizeof(float4);
}

__device__ __forceinline__ void put_job(float4* jobs, size_t cap, unsigned slot, const DataJob& j,
                                        const f2* x35) {
    const float* xf = reinterpret_cast<const float*>(x35);
    const unsigned off = slot * (unsigned)sizeof(float4);
#pragma unroll
    for (int q = 0; q < kJobF4; q++)
        *reinterpret_cast<float4*>(const_cast<char*>(job_plane(jobs, cap, q)) + off) = make_float4(job_word(4 * q, j, xf), job_word(4 * q + 1, j, xf),
                             job_word(4 * q + 2, j, xf), job_word(4 * q + 3, j, xf));
}

__device__ __forceinline__ void get_job(const float4* jobs, size_t cap, unsigned off, DataJob& j) {
    float v[112];
#pragma unroll
    for (int q = 17; q < kJobF4; q++) {   // floats 68..111 (state and indices)
        const float4 w = *reinterpret_cast<const float4*>(job_plane(jobs, cap, q) + off);
        v[4 * q] = w.x; v[4 * q + 1] = w.y; v[4 * q + 2] = w.z; v[4 * q + 3] = w.w;
    }
#pragma unroll
    for (int t = 0; t < 5; t++) j.k.eq[t] = f2{v[70 + 2 * t], v[71 + 2 * t]};
#pragma unroll
    for (int t = 0; t < 10; t++) j.k.u[t] = f2{v[80 + 2 * t], v[81 + 2 * t]};
#pragma unroll
    for (int t = 0; t < 5; t++) { j.k.d[t] = f2{v[100 + t], v[100 + t]}; j.k.g[t] = f2{0.0f, 0.0f}; }
    j.cf = (size_t)__float_as_uint(v[105]) | ((size_t)__float_as_uint(v[106]) << 32);
    j.ks = __float_as_uint(v[107]);
}

// Window reads are plain loads: the window was stored by the front wave of this
// workgroup before the frame's __syncthreads(), which makes it visible to the
// whole workgroup (same CU).  (Non-temporal loads re-fetch each line from L2/HBM
// per step: 2x the traffic in profiles/calib.)
__device__ __forceinline__ float4 ldw(const float4* p) { return *p; }

// kalman_reset, src/kalman.c:42-55
__device__ __forceinline__ Kal kal_reset() {
    Kal k;
#pragma unroll
    for (int i = 0; i < 5; i++) {
        k.eq[i] = k.g[i] = f2{0.0f, 0.0f};
        k.d[i] = f2{1.0f, 1.0f};
    }
#pragma unroll
    for (int i = 0; i < 10; i++) k.u[i] = f2{0.0f, 0.0f};
    return k;
}

// window slots 1..5 = dec[mi .. mi+4]
__device__ __forceinline__ void load_x0(const float4* wp, f2 (&x)[5]) {
    const float4 w0 = ldw(wp + 0), w1 = ldw(wp + 1), w2 = ldw(wp + 2);
    x[0] = f2{w0.z, w0.w};
    x[1] = f2{w1.x, w1.y};
    x[2] = f2{w1.z, w1.w};
    x[3] = f2{w2.x, w2.y};
    x[4] = f2{w2.z, w2.w};
}

constexpr int kForceExact = 64;   // roles bit: take the exact-division path (tests)
constexpr int kDebugStall = 128;  // roles bit: force one progress wait past its bound (tests)
constexpr int kFrontIdle = 1 << 20;  // roles bit (QPSK_ABLATE=frontidle, profiling; output invalid):
                                     // dual-chain fronts skip their channels from frame 2 on, so
                                     // the back waves train (stale windows) with the SIMDs to themselves

// 128 x train_eq (src/equalizer.c:45-58) from the window; returns matches.
// (The window load one step ahead stays: a 4-step ring loaded an iteration
// ahead, as qtrain's, changes this loop's schedule to one with ~50 s_nop per
// step in the 4x2 kernel.)
template <bool EXACT, typename PollFn>
__device__ __forceinline__ int train(Kal& k, f2 (&x)[5], const f2* wp2, bool& bad, PollFn poll) {
    int matches = 0;
    unsigned bmax = 0u;
#pragma unroll 4
    for (int i = 0; i < QK_NPRE; i++) {
        if ((i & 3) == 0) poll();                  // every 4 steps (dynamic priority)
        const f2 nx = wp2[i + 6];                  // slot i+6 (next step)
#if QPSK_TRAIN_PRETAB
        const float ref = kPreTab.v[i];            // wave-uniform scalar load (kPreTab)
#else
        const unsigned long long m = i < 64 ? kPreLo : kPreHi;
        const float ref = ((m >> (i & 63)) & 1ull) ? 1.0f : -1.0f;
#endif
        f2 v = {0.0f, 0.0f};
#pragma unroll
        for (int t = 0; t < 5; t++) v = v + cmul(x[t], k.eq[t]);
        const float er = ref - v.x;                // conjf(ref - val) = (ref - vr, vi)
        update_eq<EXACT>(k, x, f2{er, v.y}, bmax);
        if (er * ref > 0.0f) matches++;
#pragma unroll
        for (int t = 0; t < 4; t++) x[t] = x[t + 1];
        x[4] = nx;
    }
    if (!EXACT) bad |= bmax > __float_as_uint(0x1p125f);
    return matches;
}

// One frame of the back wave: lane = channel.  Window slots 1..163 hold
// dec[mi .. mi+162]; read two slots (16 B) every two steps.
// get_rt() yields rx_timing of frame n; it is called only after the training,
// so the dual-chain kernel can wait for the previous frame's decision there.
template <typename RtFn, typename PollFn>
__device__ __forceinline__ void back_frame(const RxArgs& a, int ch, bool live, int n, int mi,
                                           RtFn get_rt, const float2* win, int* rt_next,
                                           PollFn poll) {
    const float4* wp = reinterpret_cast<const float4*>(win);
    Kal k = kal_reset();
    f2 x[5];
    load_x0(wp, x);
    // equalize(): 128 x train_eq (src/qpsk.c:111-123, src/equalizer.c:45-58)
    const f2* wp2 = reinterpret_cast<const f2*>(win);
    bool bad = (a.roles & kForceExact) != 0;
    int matches = train<false>(k, x, wp2, bad, poll);
    if (__builtin_expect(__ballot(bad) != 0ull, 0)) {   // recompute the frame exactly
        k = kal_reset();
        load_x0(wp, x);
        matches = train<true>(k, x, wp2, bad, poll);
    }
    const bool valid = live && matches > QK_MATCH_MIN;   // src/qpsk.c:196
    const size_t cf = (size_t)ch * a.F + n;
    // Valid frames continue in rx_data_kernel (data_eq needs nothing the next
    // frame depends on): enqueue the equalizer state and the 35 window samples
    // of the data symbols.  One slot reservation per wave.
    const unsigned long long vm = __ballot(valid);
    if (vm) {
        unsigned base = 0;
        if (lane_id() == 0) base = atomicAdd(a.njobs, (unsigned)__popcll(vm));
        base = __builtin_amdgcn_readfirstlane(base);
        if (valid) {
            const unsigned slot = base + (unsigned)__popcll(vm & ((1ull << lane_id()) - 1ull));
            DataJob j;
            j.k = k;
            j.cf = cf;
            j.ks = (a.g0 + (unsigned)n) % QK_KS_FRAMES;
            put_job(a.jobs, a.jcap, slot, j, wp2 + 129);
        }
    }
    if (live && !valid) {   // invalid frame: bits (and soft symbols) are zero
        uint16_t* bo = reinterpret_cast<uint16_t*>(a.bits + cf * QK_NBITS);
        for (int ss = 0; ss < QK_NDSYM; ss++) bo[ss] = 0;
        if (a.soft) {
            float2* so = a.soft + cf * QK_NDSYM;
            for (int ss = 0; ss < QK_NDSYM; ss++) so[ss] = make_float2(0.0f, 0.0f);
        }
    }
    const int rt = get_rt();
    const int rtn = valid ? mi + QK_NPRE : rt;    // src/qpsk.c:219
    if (rt_next) *rt_next = rtn;   // null: a lane past its block (no channel)
    if (live) {
        a.valid[cf] = valid ? 1 : 0;
        if (a.trace)
            *reinterpret_cast<int4*>(a.trace + cf * 4) = make_int4(mi, matches, valid ? 1 : 0, rtn);
    }
}

// ---------------------------------------------------------------- quad back
// Small batches (the dual-chain kernel at <= 32 channels per workgroup) are
// bound by the latency of one channel's 128 serial train_eq steps, and a lane
// per channel issues every one of the step's ~234 instructions: one wave
// cannot issue faster than one VALU instruction per ~4.7 cycles
// (profiles/calib/valu_rate_r01.txt), so a step costs ~1,100 cycles however
// idle the SIMD is.  Here a QUAD of lanes owns a channel and splits the step:
// lane c (0..3) of the quad holds
//   row c of u          R[d-1] = u[c][c+d]        (0 past column 4)
//   column c+1 of u     C[d-1] = u[c+1-d][c+1]    (0 above row 0; C[0] is R[0])
//   d[c+1], eq[c] and (lane 3) eq[4]; d[0] is kept by all four lanes,
// computes column c+1's f/g/s/y/d/h, row c's chain of 6.15/6.16 updates and the
// 5-term sums by quad DPP (v_*_dpp quad_perm), ~135 instructions per step.
// Every fp32 operation is the one update_eq() issues, on the same operands and
// in the same order: the prefix sums (a[j], val) run sequentially over the
// quad's lanes, zero padding enters only as (+-0) addends / factors of a
// finite value, which leave every nonzero sum unchanged (the row chains are
// independent across rows: row i uses only its own running g[i] and the
// ORIGINAL g[j], h[j] of the columns right of it, src/kalman.c:131-139).
namespace qd {
constexpr int kB0 = 0x00, kB1 = 0x55, kB2 = 0xAA, kB3 = 0xFF;   // broadcast lane k of the quad
constexpr int kRot1 = 0x93;   // [3,0,1,2]: lane c <- lane c-1 (lane 0 <- lane 3)
constexpr int kRot2 = 0x4E;   // [2,3,0,1]: lane c <- lane c-2
constexpr int kRot3 = 0x39;   // [1,2,3,0]: lane c <- lane c+1
}

template <int CTRL>
__device__ __forceinline__ float qdf(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, true));
}
template <int CTRL>
__device__ __forceinline__ f2 qd2(f2 v) { return f2{qdf<CTRL>(v.x), qdf<CTRL>(v.y)}; }
// qd2<CTRL>(v) * m as two v_mul_f32_dpp (the moves fold into the products);
// the empty asm keeps the products scalar, else they pack into a v_pk_mul_f32
// that takes no DPP source and the two moves stay
template <int CTRL>
__device__ __forceinline__ f2 qd_mul(f2 v, float m) {
    float x = qdf<CTRL>(v.x) * m, y = qdf<CTRL>(v.y) * m;
    if (QPSK_QDMUL) asm("" : "+v"(x), "+v"(y));
    return f2{x, y};
}

struct QKal {
    f2 R[4];      // R[d-1] = u[c][c+d]
    f2 C[3];      // C[d-2] = u[c+1-d][c+1], d = 2..4
    f2 eqr;       // eq_coeff[c]
    f2 eq4;       // eq_coeff[4] (lane 3)
    f2 dd;        // (d[0], d[c+1]): one packed multiply updates both
};

__device__ __forceinline__ QKal qkal_reset() {   // kalman_reset, src/kalman.c:42-55
    QKal k;
#pragma unroll
    for (int i = 0; i < 4; i++) k.R[i] = f2{0.0f, 0.0f};
#pragma unroll
    for (int i = 0; i < 3; i++) k.C[i] = f2{0.0f, 0.0f};
    k.eqr = k.eq4 = f2{0.0f, 0.0f};
    k.dd = f2{1.0f, 1.0f};
    return k;
}

// Packed products with the conj() of the reference folded into a negate
// modifier (conj never materialised; (-a)*b == -(a*b) exactly):
// (x.x * d0, (-x.y) * d0) with d0 = dd.x broadcast: conj(x) * d[0]
__device__ __forceinline__ f2 mul_conj_d0(f2 x, f2 dd) {
    f2 r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0] neg_hi:[1,0]" : "=v"(r) : "v"(x), "v"(dd));
    return r;
}
// (a.x * b.x, a.y * (-b.y)): a * conj(b) componentwise
__device__ __forceinline__ f2 mul_conjb(f2 a, f2 b) {
    f2 r;
    asm("v_pk_mul_f32 %0, %1, %2 neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// (f.x * dc, f.y * dc) with dc = dd.y broadcast
__device__ __forceinline__ f2 mul_dc(f2 f, f2 dd) {
    f2 r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1]" : "=v"(r) : "v"(f), "v"(dd));
    return r;
}


// one train_eq step (src/equalizer.c:45-58 with update_eq/kalman_calculate,
// exactly update_eq<EXACT>'s operations) on the quad layout.  X0..X4 = x[c+1-d]
// (x[index+t] of the reference), zero before x[0].  Returns er = Re(error).
// EXACT = false: `bmax` collects the bit patterns of the step's largest
// reciprocal operand (xso, lane c: xs[c+1], nondecreasing in j, and >= xs[0]
// >= E unless NaN); the caller tests bmax <= bits(2^125) once per frame, which
// is qk_rcp_in_range() for every step (a NaN or -x has larger bits).
template <bool EXACT>
__device__ __forceinline__ float qstep(QKal& k, const f2& X0, const f2& X1, const f2& X2, const f2& X3,
                                       const f2& X4, float ref, int c, unsigned& bmax) {
    const float E = QK_KAL_E, q = QK_KAL_Q;
    // 1 where row c has column c+d (d = 2, 3, 4), else 0: h of a missing
    // column is multiplied by 0, so the padding entries of R stay +0
    const float m2 = c < 3 ? 1.0f : 0.0f, m3 = c < 2 ? 1.0f : 0.0f, m4 = c < 1 ? 1.0f : 0.0f;
    // val = sum_t x[t] * eq[t], t = 0..4 in order (src/equalizer.c:49-51); the
    // reference's 0 + x[0]*eq[0] only differs from x[0]*eq[0] in the sign of a
    // zero, which no output observes, so the chain starts with
    // the broadcast itself
    const f2 p = cmul(X1, k.eqr);         // lane c: x[c] * eq[c]
    const f2 p4 = cmul(X0, k.eq4);        // lane 3: x[4] * eq[4]
    // (the empty asm keeps the two components scalar adds, so each folds its
    // DPP source into one v_add_f32_dpp instead of two moves and a packed add)
    float vr = qdf<qd::kB0>(p.x), vi = qdf<qd::kB0>(p.y);
#define QV(CT, P)                                                   \
    vr = vr + qdf<CT>(P.x); vi = vi + qdf<CT>(P.y);                 \
    asm("" : "+v"(vr), "+v"(vi))
    QV(qd::kB1, p); QV(qd::kB2, p); QV(qd::kB3, p); QV(qd::kB3, p4);
#undef QV
    const float er = ref - vr;            // conjf(ref - val) = (ref - vr, vi)
    // column 0 (every lane): f0 = conj(x0), 6.2; g0 = f0 * d0, 6.4; t0 = g0 * f0
    const f2 x0 = qd2<qd::kB0>(X1);
    const f2 g0 = mul_conj_d0(x0, k.dd);
    const f2 t0 = mul_conjb(g0, x0);
    const float a0 = E + (t0.x + t0.y);                   // 6.5
    // column c+1: f = u[0][j]*conj(x0) + conj(xj) + sum_{0<i<j} u[i][j]*conj(xi)
    f2 f = addc(cmulc(k.C[2], X4), X0);
    f = f + cmulc(k.C[1], X3);
    f = f + cmulc(k.C[0], X2);
    f = f + cmulc(k.R[0], X1);
    const f2 g = mul_dc(f, k.dd);                         // 6.4
    const f2 t = g * f;
    const float s = t.x + t.y;
    // 6.6 a[j] = a[j-1] + Re(g conj f), the quad's s in column order
    const float a1 = a0 + qdf<qd::kB0>(s);
    const float a2 = a1 + qdf<qd::kB1>(s);
    const float a3 = a2 + qdf<qd::kB2>(s);
    const float a4 = a3 + qdf<qd::kB3>(s);
    const float hq = 1.0f + q;                            // 6.7
    const float ht = a4 * q;
    const float ap = c == 0 ? a0 : c == 1 ? a1 : c == 2 ? a2 : a3;   // a[c]
    const float ao = ap + s;                              // a[c+1], the chain's own add
    const f2 xs = f2{a0, ao} + f2{ht, ht};               // (xs[0], xs[c+1]), 6.19 / 6.22 operands
    f2 y;
    if (EXACT) {
        y = f2{qk_div_ieee(xs.x), qk_div_ieee(xs.y)};
    } else {
        bmax = max(bmax, __float_as_uint(xs.y));
        y = f2{qk_rcp_fast(xs.x), qk_rcp_fast(xs.y)};
    }
    // 6.20 / 6.21+6.13: d[0] *= (hq * (E + ht)) * y0, d[c+1] *= (hq * (a[c] + ht)) * y[c+1]
    k.dd = k.dd * ((f2{hq, hq} * (f2{E, ap} + f2{ht, ht})) * y);
    const float y0 = y.x, yo = y.y;
    // (every DPP move is made unconditionally, then selected: a move inside
    // a conditional would become a branch, the intrinsic being convergent)
    const float yr = qdf<qd::kRot1>(yo);
    const float yp = c == 0 ? y0 : yr;                    // y[c]
    const f2 h = (-f) * yp;                               // 6.11 h[c+1]
    // row c (6.15/6.16) from g[c]: column c's gain (lane c-1; column 0: g0)
    const f2 gr = qd2<qd::kRot1>(g);
    f2 G = c == 0 ? g0 : gr;
    {   // column c+1: this lane
        const f2 B1 = k.R[0];
        k.R[0] = B1 + cmulc(h, G);
        G = G + cmulc(g, B1);
    }
    {   // column c+2 (lane c+1); none for row 3
        const f2 hd = qd_mul<qd::kRot3>(h, m2);
        const f2 gd = qd2<qd::kRot3>(g);
        const f2 B1 = k.R[1];
        k.R[1] = B1 + cmulc(hd, G);
        G = G + cmulc(gd, B1);
    }
    {   // column c+3 (lane c+2); none for rows 2, 3
        const f2 hd = qd_mul<qd::kRot2>(h, m3);
        const f2 gd = qd2<qd::kRot2>(g);
        const f2 B1 = k.R[2];
        k.R[2] = B1 + cmulc(hd, G);
        G = G + cmulc(gd, B1);
    }
    {   // column c+4 (lane c+3); row 0 only
        const f2 hd = qd_mul<qd::kRot1>(h, m4);
        const f2 B1 = k.R[3];
        k.R[3] = B1 + cmulc(hd, G);
        G = G + cmulc(gr, B1);
    }
    // next step's columns: C[d-2](c) = R[d-1](c+1-d); the lanes with no such
    // row read a padding entry of R (zero) through the rotation
    k.C[0] = qd2<qd::kRot1>(k.R[1]);
    k.C[1] = qd2<qd::kRot2>(k.R[2]);
    k.C[2] = qd2<qd::kRot3>(k.R[3]);
    // update_eq: error *= kalman_y (y[4], lane 3); eq[i] += error * conj(g[i])
    const float y4 = qdf<qd::kB3>(yo);
    const f2 e = f2{er, vi} * y4;
    k.eqr = k.eqr + cmulc(e, G);     // row c's final gain
    k.eq4 = k.eq4 + cmulc(e, g);     // lane 3: g[4] (row 4 has no updates)
    return er;
}

// x[index+t] at step 0: X[d] = x[c+1-d] = window slot c+2-d (slot k+1 = dec[mi+k])
__device__ __forceinline__ void qload_x0(const f2* wp2, int c, f2 (&X)[5]) {
#pragma unroll
    for (int d = 0; d < 5; d++) X[d] = d <= c + 1 ? wp2[c + 2 - d] : f2{0.0f, 0.0f};
}

// The window as a ring of 8 samples per lane, w[s mod 8] = x[c+1] of step s
// (wl[s]; w of a negative step: X of step 0, zero-padded); step s reads
// X[d] = w[(s - d) mod 8].  Eight steps per loop iteration, so the ring's
// roles repeat every iteration and no register moves at the back edge; the
// sample of step s+4 is loaded right after step s, into the slot step s read
// last (reads run to step 131, inside the 168-slot window row).
template <bool EXACT, typename PollFn>
__device__ __forceinline__ int qtrain(QKal& k, const f2 (&X)[5], const f2* wl, int c, bool& bad, PollFn poll) {
    int matches = 0;
    unsigned bmax = 0u;
    f2 w[8];
    w[0] = X[0];
    w[7] = X[1];
    w[6] = X[2];
    w[5] = X[3];
    w[4] = X[4];
#pragma unroll
    for (int t = 1; t < 4; t++) w[t] = wl[t];
    for (int i = 0; i < QK_NPRE; i += 8) {
        const float4 r0 = *reinterpret_cast<const float4*>(&kPreTab.v[i]);
        const float4 r1 = *reinterpret_cast<const float4*>(&kPreTab.v[i + 4]);
        const float ref8[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
#pragma unroll
        for (int t = 0; t < 8; t++) {
            if ((t & 3) == 0) poll();   // every 4 steps (dynamic priority, rx_kernel kDyn)
            const float ref = ref8[t];
            const float er = qstep<EXACT>(k, w[t & 7], w[(t + 7) & 7], w[(t + 6) & 7], w[(t + 5) & 7],
                                          w[(t + 4) & 7], ref, c, bmax);
            matches += (er * ref > 0.0f) ? 1 : 0;
            w[(t + 4) & 7] = wl[i + t + 4];   // sample of step i+t+4
        }
    }
    if (!EXACT) bad |= bmax > __float_as_uint(0x1p125f);
    return matches;
}

// back_frame() for a quad per channel: every lane of the quad has the same
// matches / valid / rt; the quad's lane 0 writes the per-channel outputs.
template <typename RtFn, typename PollFn>
__device__ __forceinline__ void back_frame_quad(const RxArgs& a, int ch, bool live, int n, int mi,
                                                RtFn get_rt, const float2* win, int* rt_next,
                                                PollFn poll) {
    const int c = lane_id() & 3;
    const bool lead = c == 0;
    const f2* wp2 = reinterpret_cast<const f2*>(win);
    QKal k = qkal_reset();
    f2 X[5];
    qload_x0(wp2, c, X);
    bool bad = (a.roles & kForceExact) != 0;
    int matches = qtrain<false>(k, X, wp2 + c + 2, c, bad, poll);
    if (__builtin_expect(__ballot(bad) != 0ull, 0)) {   // recompute the frame exactly
        k = qkal_reset();
        qload_x0(wp2, c, X);
        matches = qtrain<true>(k, X, wp2 + c + 2, c, bad, poll);
    }
    const bool valid = live && matches > QK_MATCH_MIN;   // src/qpsk.c:196
    const size_t cf = (size_t)ch * a.F + n;
    const unsigned long long vm = __ballot(valid && lead);
    if (vm) {   // gather the quad's state (all lanes take part in the DPP moves)
        DataJob j;
        j.k.eq[0] = qd2<qd::kB0>(k.eqr);
        j.k.eq[1] = qd2<qd::kB1>(k.eqr);
        j.k.eq[2] = qd2<qd::kB2>(k.eqr);
        j.k.eq[3] = qd2<qd::kB3>(k.eqr);
        j.k.eq[4] = qd2<qd::kB3>(k.eq4);
#define QU(i, jj, CT) j.k.u[uix(i, jj)] = qd2<CT>(k.R[(jj) - (i) - 1])
        QU(0, 1, qd::kB0); QU(0, 2, qd::kB0); QU(0, 3, qd::kB0); QU(0, 4, qd::kB0);
        QU(1, 2, qd::kB1); QU(1, 3, qd::kB1); QU(1, 4, qd::kB1);
        QU(2, 3, qd::kB2); QU(2, 4, qd::kB2);
        QU(3, 4, qd::kB3);
#undef QU
        j.k.d[0] = f2{k.dd.x, k.dd.x};
        const float d1 = qdf<qd::kB0>(k.dd.y), d2 = qdf<qd::kB1>(k.dd.y);
        const float d3 = qdf<qd::kB2>(k.dd.y), d4 = qdf<qd::kB3>(k.dd.y);
        j.k.d[1] = f2{d1, d1};
        j.k.d[2] = f2{d2, d2};
        j.k.d[3] = f2{d3, d3};
        j.k.d[4] = f2{d4, d4};
        unsigned base = 0;
        if (lane_id() == 0) base = atomicAdd(a.njobs, (unsigned)__popcll(vm));
        base = __builtin_amdgcn_readfirstlane(base);
        if (valid && lead) {
            const unsigned slot = base + (unsigned)__popcll(vm & ((1ull << lane_id()) - 1ull));
            j.cf = cf;
            j.ks = (a.g0 + (unsigned)n) % QK_KS_FRAMES;
            put_job(a.jobs, a.jcap, slot, j, wp2 + 129);
        }
    }
    if (live && !valid) {   // invalid frame: bits (and soft symbols) are zero
        uint16_t* bo = reinterpret_cast<uint16_t*>(a.bits + cf * QK_NBITS);
        for (int ss = c; ss < QK_NDSYM; ss += 4) bo[ss] = 0;
        if (a.soft) {
            float2* so = a.soft + cf * QK_NDSYM;
            for (int ss = c; ss < QK_NDSYM; ss += 4) so[ss] = make_float2(0.0f, 0.0f);
        }
    }
    const int rt = get_rt();
    const int rtn = valid ? mi + QK_NPRE : rt;    // src/qpsk.c:219
    if (lead) *rt_next = rtn;
    if (live && lead) {
        a.valid[cf] = valid ? 1 : 0;
        if (a.trace)
            *reinterpret_cast<int4*>(a.trace + cf * 4) = make_int4(mi, matches, valid ? 1 : 0, rtn);
    }
}

// 31 x data_eq + qpsk_demod (src/equalizer.c:64-90, src/qpsk.c:268-271) from
// the job's window samples xs; returns the raw dibits (bit 2s = Q, 2s+1 = I).
// Decisions collect in a register; the caller stores the 62 bytes after the
// loop, so no wait on a store sits inside it.
// the job's window samples: x[t] is float2 (t & 1) of 16-B word t >> 1
struct JobX {
    const float4* jobs;
    size_t cap;
    unsigned off;   // slot * 16
    __device__ __forceinline__ f2 operator[](int t) const {
        return *reinterpret_cast<const f2*>(job_plane(jobs, cap, t >> 1) + off + 8u * (t & 1));
    }
};

#ifndef QPSK_DATA_RING
#define QPSK_DATA_RING 4   // job samples loaded this many steps ahead (1: one step; profiles/r02_data_ring_ab.txt)
#endif
template <bool EXACT>
__device__ __forceinline__ void data_step(Kal& k, f2 (&x)[5], f2 nx, int s, unsigned long long& dib,
                                          float2* so, unsigned& bmax) {
    f2 sy = {0.0f, 0.0f};
#pragma unroll
    for (int t = 0; t < 5; t++) sy = sy + cmulc(x[t], k.eq[t]);
    const int dI = sy.x < 0.0f, dQ = sy.y < 0.0f;
    const f2 cst = {dI ? -1.0f : 1.0f, dQ ? -1.0f : 1.0f};
    update_eq<EXACT>(k, x, (cst - sy) * 0.1f, bmax);
    dib |= (unsigned long long)(dQ | (dI << 1)) << (2 * s);
    if (so) so[s] = make_float2(sy.x, sy.y);
#pragma unroll
    for (int t = 0; t < 4; t++) x[t] = x[t + 1];
    x[4] = nx;
}

template <bool EXACT>
__device__ __forceinline__ unsigned long long data_steps(Kal& k, f2 (&x)[5], const JobX xs,
                                                         float2* so, bool& bad) {
    unsigned long long dib = 0;
    unsigned bmax = 0u;
#if QPSK_DATA_RING > 1
    // the job's samples arrive from HBM (written ~ms earlier by rx_kernel):
    // each is loaded R steps before it enters x
    constexpr int R = QPSK_DATA_RING;
    f2 cur[R];
#pragma unroll
    for (int t = 0; t < R; t++) cur[t] = xs[min(5 + t, 34)];
    for (int s0 = 0; s0 < QK_NDSYM; s0 += R) {
        f2 nxt[R];
#pragma unroll
        for (int t = 0; t < R; t++) nxt[t] = xs[min(s0 + R + 5 + t, 34)];
#pragma unroll
        for (int t = 0; t < R; t++)
            if (s0 + t < QK_NDSYM) data_step<EXACT>(k, x, cur[t], s0 + t, dib, so, bmax);
#pragma unroll
        for (int t = 0; t < R; t++) cur[t] = nxt[t];
    }
#else
    for (int s = 0; s < QK_NDSYM; s++) data_step<EXACT>(k, x, xs[min(s + 5, 34)], s, dib, so, bmax);
#endif
    if (!EXACT) bad |= bmax > __float_as_uint(0x1p125f);
    return dib;
}

// ---------------------------------------------------------------- data kernel
// The 31 data symbols of every valid frame (src/qpsk.c:204-215: data_eq
// src/equalizer.c:64-90, qpsk_demod src/qpsk.c:268-271, scramble
// src/scramble.c:57-84), one job per lane, packed: only ~1 frame in 5 is
// valid, so running them inside the lane-per-channel back wave would idle most
// lanes for 31 of its 159 steps.  Jobs come from the call's rx_kernel in any
// order; every output location is fixed by the job, so results do not depend
// on it.
__global__ void __launch_bounds__(256) rx_data_kernel(const float4* jobs, unsigned long long jcap,
                                                      unsigned* njobs,
                                                      const unsigned long long* ks_tab,
                                                      uint8_t* bits, float2* soft, int parity,
                                                      int force_exact, int* err, int* err_to) {
    // err_to (host calls, qpsk_rx_batch): the context's error word, taken in one
    // atomic exchange after rx_kernel (stream order), stored with the outputs:
    // no separate launch for it
    if (err_to && blockIdx.x == 0 && threadIdx.x == 0) *err_to = atomicExch(err, 0);
    const size_t cap = (size_t)jcap;
    const unsigned n = njobs[parity];
    const unsigned stride = gridDim.x * blockDim.x;
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const unsigned off = i * (unsigned)sizeof(float4);
        DataJob j;
        get_job(jobs, cap, off, j);
        const JobX xs{jobs, cap, off};   // x = dec[mi+128+t], t < 35
        f2 x[5];
#pragma unroll
        for (int t = 0; t < 5; t++) x[t] = xs[t];
        const unsigned long long ks = ks_tab[j.ks];
        float2* so = soft ? soft + j.cf * QK_NDSYM : nullptr;
        bool bad = force_exact != 0;
        unsigned long long dib = data_steps<false>(j.k, x, xs, so, bad);
        if (__builtin_expect(bad, 0)) {   // recompute the job with IEEE division
            get_job(jobs, cap, off, j);
#pragma unroll
            for (int t = 0; t < 5; t++) x[t] = xs[t];
            dib = data_steps<true>(j.k, x, xs, so, bad);
        }
        dib ^= ks;   // descramble (src/scramble.c:57-84): keystream bits 62g .. 62g+61
        uint16_t* bo = reinterpret_cast<uint16_t*>(bits + j.cf * QK_NBITS);
#pragma unroll
        for (int q = 0; q < QK_NDSYM; q++)
            bo[q] = (uint16_t)(((dib >> (2 * q)) & 1ull) | (((dib >> (2 * q + 1)) & 1ull) << 8));
    }
    // the next call's counter (calls on one context are stream-ordered)
    if (blockIdx.x == 0 && threadIdx.x == 0) njobs[parity ^ 1] = 0u;
}

// Plain pointer parameters (not a by-value struct): the compiler then knows every
// pointer is a global-memory pointer (global_load/store, no flat) and nothing of
// the argument block is indexed dynamically (no scratch copy).
// 12 waves per workgroup, 3 per SIMD (<= 168 VGPRs), one workgroup per CU (LDS).
//
// DUAL (G <= 2): two back waves per group, one for the even and one for the odd
// frames of the call.  Frame n's training needs only frame n-1's front, and
// frame n-1's front needs frame n-2's decision, so consecutive frames' training
// is independent: the back of frame n+1 starts as soon as the front of frame n
// is done, while the back of frame n is still running.  The per-frame time
// drops from max(back, front) to (back + front) / 2 where one serial back wave
// per CU bounds the kernel (<= 16,384 channels per GPU).  Progress is handed
// over through LDS counters (bseq: frames decided per back wave; fcnt: front
// frames finished, by frame parity) instead of __syncthreads().
//
// W (DUAL only): channels per group, 64, 32 or 16.  A narrower group leaves
// back lanes idle but spreads a small batch over more CUs and gives each front
// wave fewer channels per frame, which shortens the front half of the chain.
//
// QUAD (DUAL, G == 1 only): the back waves hold a quad of lanes per channel
// (back_frame_quad), 16 channels per wave, W / 16 waves per frame chain.
template <int G, int FP, int MODE, bool DUAL, int W, bool QUAD>
constexpr int kBackWavesOf = DUAL ? 2 * G * (QUAD ? W / 16 : 1) : G;

// waves per SIMD = ceil(waves / 4): 3 (<= 168 VGPRs) for the 12-wave shapes
template <int G, int FP, int MODE, bool DUAL, int W, bool QUAD>
constexpr int kWavesOf = kBackWavesOf<G, FP, MODE, DUAL, W, QUAD> + G * FP;

//
// HP: the fronts take F_{n+1} from the head pre-pass (head_kernel, QPSK_HEADPASS).
template <int G, int FP, int MODE, bool DUAL, int W = QK_GROUP, bool QUAD = false, bool HP = false>
__global__ void __launch_bounds__((64 * kWavesOf<G, FP, MODE, DUAL, W, QUAD>),
                                  ((kWavesOf<G, FP, MODE, DUAL, W, QUAD> + 3) / 4)) QPSK_RX_ATTR rx_kernel(
    const int16_t* in, int16_t* hist, const float2* ptab, const unsigned long long* ks,
    float2* win0, float2* win1, int* mi0, int* mi1, int* rt0, int* rt1, uint8_t* bits,
    uint8_t* valid, int32_t* trace, float2* soft, float4* jobs, unsigned* njobs, int nch, int F,
    unsigned g0, int roles, const float* fft_tab, unsigned long long jcap, int* err) {
    static_assert(W == QK_GROUP || (DUAL && G == 1 && W % FP == 0 && W <= QK_GROUP), "group width");
    static_assert(!QUAD || (DUAL && G == 1 && W % 16 == 0), "quad backs: dual chain, one group");
    constexpr int kGroups = G, kFrontPer = FP;
    constexpr int kBackWaves = kBackWavesOf<G, FP, MODE, DUAL, W, QUAD>;
    constexpr int kChainWaves = QUAD ? W / 16 : 1;     // back waves per frame chain and group
    constexpr bool kDyn = DUAL && (QPSK_DYNPRIO == 2 || (QPSK_DYNPRIO == 1 && QUAD));
    constexpr int kFrontCh = W / kFrontPer;            // channels per front wave
    constexpr int kFrontWaves = kGroups * kFrontPer;
    constexpr int kBlock = 64 * (kBackWaves + kFrontWaves);
    const RxArgs a{in, hist, ptab, ks, win0, win1, mi0, mi1, rt0, rt1, bits, valid, trace, soft,
                   jobs, njobs, nch, F, g0, (size_t)jcap, roles, err,
                   // HP (reference mode only): fft_tab carries the head pre-pass outputs
                   HP ? reinterpret_cast<const float2*>(fft_tab) : nullptr};
    __shared__ __attribute__((aligned(16))) float2 P[QK_FRAME];
    constexpr int DM = MODE & 1;   // decimation semantics; MODE & 2: FFT hunt
    constexpr int kM = Cfg<DM>::kM, kDecBuf = Cfg<DM>::kDecBuf;
    __shared__ __attribute__((aligned(16))) float2 Ms[kFrontWaves][kM];
    __shared__ __attribute__((aligned(16))) float2 decs[kFrontWaves][kDecBuf][kDec];
    __shared__ int mi_s[kGroups][2][QK_GROUP], rt_s[kGroups][2][QK_GROUP];
    // hunt tables: the MFMA correlator's B, or the FFT hunt's twiddles / Q / permutation
    __shared__ __attribute__((aligned(16))) float BT[(MODE & 2) ? kFftHT : kHuntTab];
    // the split FIR's pass-2 lane map (kSplitTab; 2 KB, reference mode only)
    constexpr bool kSplitK = MODE == 0 && !HP && QPSK_FIR_SPLIT && (!DUAL || QPSK_FIR_SPLIT == 2);
    __shared__ uint32_t p2w[kSplitK ? kSplitTabWords : 1];
    const uint8_t* p2tab = reinterpret_cast<const uint8_t*>(p2w);
    // DUAL progress counters, per group, frame parity and channel block (one
    // block per back wave of a chain)
    __shared__ int bseq[kGroups][2][kChainWaves], fcnt[kGroups][2][kChainWaves];
    __shared__ int dead_s;                               // DUAL: a wait of this workgroup timed out
    __shared__ int nwait_s;                              // kDyn: back waves waiting for their fronts
#ifdef QPSK_STAMPS
    // diagnostic (4x2): each wave's arrival at the frame barrier and its SIMD;
    // a back wave sums the cycles it trains after the last front of its SIMD
    // arrived (stamp 15) and counts the frames it arrived last (stamp 5)
    __shared__ unsigned long long tarr_s[16];
    __shared__ int tsimd_s[16];
#define TAIL_INIT() do { if (lane == 0 && wave < 16) tsimd_s[wave] = (int)((__builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4) >> 4) & 3); } while (0)
#define TAIL_ARRIVE() do { if (lane == 0 && wave < 16) tarr_s[wave] = stamp_now(); } while (0)
#define TAIL_BACK()                                                                           \
    do {                                                                                      \
        unsigned long long tf = 0;                                                            \
        for (int w2 = kBackWaves; w2 < kBackWaves + kFrontWaves && w2 < 16; w2++)             \
            if (tsimd_s[w2] == tsimd_s[wave] && tarr_s[w2] > tf) tf = tarr_s[w2];            \
        if (tf > 0 && tarr_s[wave] > tf) { st_acc[15] += tarr_s[wave] - tf; st_acc[5] += 1; } \
        st_t0 = stamp_now();                                                                  \
    } while (0)
#else
#define TAIL_INIT() do { } while (0)
#define TAIL_ARRIVE() do { } while (0)
#define TAIL_BACK() do { } while (0)
#endif
    // a launch whose block is not this instantiation's waves would leave roles
    // unserved and every progress wait to its bound: report it and do nothing
    if (blockDim.x != (unsigned)kBlock) {
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(err, kErrStall);
        return;
    }
    const int lane = threadIdx.x & 63;
    // wave-uniform by construction; readfirstlane tells the compiler, so every
    // per-wave index and pointer below lives in SGPRs
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int grp0 = blockIdx.x * kGroups;
    TAIL_INIT();
    for (int i = threadIdx.x; i < QK_FRAME / 2; i += kBlock)
        reinterpret_cast<float4*>(P)[i] = reinterpret_cast<const float4*>(a.ptab)[i];
    if constexpr (kSplitK && QPSK_SPLIT_BANKS)
        for (int i = threadIdx.x; i < kSplitTabWords; i += kBlock)
            p2w[i] = reinterpret_cast<const uint32_t*>(&kSplitTab)[i];
    if constexpr ((MODE & 2) != 0) {
        for (int i = threadIdx.x; i < kFftHT; i += kBlock) BT[i] = fft_tab[i];
    } else {
#if QPSK_HUNT_FILTER
        qhunt::bconst_h_lds(threadIdx.x, kBlock, BT);
#else
        qhunt::bconst_lds(threadIdx.x, kBlock, BT);
#endif
    }
    if (wave < kGroups) {   // per-channel state of the groups at the call's first frame
        const int ch = (grp0 + wave) * W + lane;
        if (lane < W && ch < a.nch) {
            mi_s[wave][0][lane] = mi_of(a, a.g0)[ch];
            rt_s[wave][0][lane] = rt_of(a, a.g0)[ch];
        }
    }
    if (threadIdx.x < 2 * kGroups * kChainWaves) (&bseq[0][0][0])[threadIdx.x] = (&fcnt[0][0][0])[threadIdx.x] = 0;
    if (threadIdx.x == 0) dead_s = nwait_s = 0;
    __syncthreads();
    if constexpr (DUAL) {
        // Channel blocks: a group's channels split into one block per back wave
        // of a chain (QUAD: 16 channels; lane backs: the whole group).  A back
        // wave waits only for the fronts of its own block, and the front waves
        // serve the blocks one at a time (every front wave takes its share of
        // block 0, signals, then block 1): a block's windows are ready after
        // its share of the front work, not the group's, and the chain waves
        // settle into a stagger of one block's front time
        // (profiles/r03_blocks_ab.txt; lane backs split into 32-channel blocks
        // were measured too: slower, two back waves issue every step).
        // bseq[gi][p][b]: frames of parity p decided by block b's back wave;
        // fcnt[gi][p][b]: front waves done with block b of parity-p frames.
        constexpr int kBlkCh = W / kChainWaves;            // channels per block
        constexpr int kFrontChB = kBlkCh / kFrontPer;      // per front wave and block
        static_assert(kBlkCh % kFrontPer == 0, "block split");
        if (wave < kBackWaves) {
            // ---------------------------------------------------- back of group
            // gi = (wave >> 1) / kChainWaves, block b, frames n = wave mod 2
            const int gi = (wave >> 1) / kChainWaves;
            const int b = (wave >> 1) % kChainWaves;
            // channel of this lane within the block: the lane, or its quad.
            // Lanes past the block (lane backs with W < 64) own no channel:
            // they read their block's first channel's slots and write none.
            const int sub = QUAD ? lane >> 2 : lane;
            const bool own = sub < kBlkCh;
            const int idx = kBlkCh * b + (own ? sub : 0);
            const int ch = (grp0 + gi) * W + idx;
            const bool live = own && ch < a.nch;
            if (kDyn || ((a.roles >> 4) & 3) == 2) __builtin_amdgcn_s_setprio(2);
            // kDyn (QPSK_DYNPRIO): every 4 training steps, drop to the lowest
            // issue priority while another back wave waits for its fronts, else the highest
            auto poll = [&] {
                if constexpr (kDyn) {
                    const int w = __builtin_amdgcn_readfirstlane(
                        __hip_atomic_load(&nwait_s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
                    if (w > 0) __builtin_amdgcn_s_setprio(0);
                    else __builtin_amdgcn_s_setprio(2);
                }
            };
            // tests (roles bit kDebugStall): one wait that cannot end, on the
            // first back wave of workgroup 0, with a short bound
            if ((a.roles & kDebugStall) && blockIdx.x == 0 && wave == 0)
                spin_wait(&fcnt[gi][0][0], 1 << 30, a.err, &dead_s, 1u << 12);
            // diagnostic stamps (QPSK_STAMPS): 13 frame work, 14 wait for the
            // fronts, 15 wait for the other chain's decision
            STAMP_DECL
            for (int n = wave & 1; n < a.F; n += 2) {
                const int p = n & 1;
                // front(n-1) done by every front wave for this block: window n and mi_n
                if (n > 0) {
                    int* const fc = &fcnt[gi][p ^ 1][b];
                    const int need = kFrontPer * ((n - 1) / 2 + 1);
                    if constexpr (kDyn) {
                        const bool waits = __builtin_amdgcn_readfirstlane(__hip_atomic_load(
                                               fc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < need;
                        if (waits) {   // wait at the lowest priority; poll() resets it
                            __builtin_amdgcn_s_setprio(0);
                            if (lane == 0)
                                __hip_atomic_fetch_add(&nwait_s, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        }
                        spin_wait(fc, need, a.err, &dead_s);
                        if (waits && lane == 0)
                            __hip_atomic_fetch_add(&nwait_s, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    } else {
                        spin_wait(fc, need, a.err, &dead_s);
                    }
                }
                STAMP(14);
                const int mi = mi_s[gi][p][idx];
                auto get_rt = [&] {   // rx_timing of frame n = the decision of frame n-1
                    STAMP(13);
                    if (n > 0) spin_wait(&bseq[gi][p ^ 1][b], (n - 1) / 2 + 1, a.err, &dead_s);
                    STAMP(15);
                    return rt_s[gi][p][idx];
                };
                const float2* wn = win_of(a, a.g0 + (unsigned)n) + (size_t)(live ? ch : 0) * kWinStride;
                int* rtn = own ? &rt_s[gi][p ^ 1][idx] : nullptr;
                if constexpr (QUAD)
                    back_frame_quad(a, live ? ch : 0, live, n, mi, get_rt, wn, rtn, poll);
                else
                    back_frame(a, live ? ch : 0, live, n, mi, get_rt, wn, rtn, poll);
                signal_add(&bseq[gi][p][b], 1, lane);
                STAMP(13);
            }
            STAMP_FLUSH();
        } else {
            // ---------------------------------------------------- front
            const int f = wave - kBackWaves;
            const int gi = f / kFrontPer;
            const int fl = f % kFrontPer;
            // roles bits 16-19 (split s, one group and one block per workgroup
            // only; pick_shape sets 2 at W = 64): the front waves that share a
            // SIMD with a back wave (waves 4, 5, 8, 9 when waves map to SIMDs by
            // wave % 4) take s channels fewer, the others s more
            const int split = (kGroups == 1 && kChainWaves == 1) ? (a.roles >> 16) & 15 : 0;
            auto share = [&](int x) { return ((x + kBackWaves) & 3) < kBackWaves; };
            int cbeg = 0;
            for (int x = 0; x < fl; x++) cbeg += kFrontChB + (share(x) ? -split : split);
            const int mych = kFrontChB + (share(fl) ? -split : split);
            // this wave's channels of block bb: group index kBlkCh * bb + cbeg + c
            auto bch0 = [&](int bb) { return (grp0 + gi) * W + kBlkCh * bb + cbeg; };
            auto blive = [&](int bb) { return max(0, min(mych, a.nch - bch0(bb))); };
            float2* M = Ms[f];
            int pf[kPf<DM>];
            // QPSK_FIR_SPLIT == 2 (A/B knob): the split FIR here too
            constexpr bool kSplitD = MODE == 0 && !HP && QPSK_FIR_SPLIT == 2;
            constexpr int kFrD = kSplitD ? QPSK_FRESH_SPLIT : QPSK_FRESH;
            if (kDyn) __builtin_amdgcn_s_setprio(1);
            else if (((a.roles >> 4) & 3) == 1) __builtin_amdgcn_s_setprio(2);
            if (blive(0) > 0) prefetch<DM, false, kFrD>(srcs(a, bch0(0), 0), lane, pf);
            // diagnostic stamps (QPSK_STAMPS): 7 wait for the backs, 0 mix,
            // 4 window store, 1 prefetch, 8-12 front_channel phases, 6 its tail,
            // 5 signal
            STAMP_DECL
            int k = 0;   // channels done, for the dec buffer ring
// One frame n of a dual-chain front wave's channels.  CG: frame n >= 2, so
// every prefetch reads consecutive rows of `in` (prefetch<.., true>, see
// load_item); the quad-back kernels peel frames 0 and 1 off for it (in the
// lane-back kernels the single loop keeps their code unchanged).
#define QPSK_DUAL_FRONT_FRAME(CG)                                                                              \
    do {                                                                                                       \
        const int p = n & 1;                                                                                   \
        const unsigned g = a.g0 + (unsigned)n;                                                                 \
        float2* wout = win_of(a, g + 1u);                                                                      \
        for (int bb = 0; bb < kChainWaves; bb++) {                                                             \
            /* back(n-1) of this block done: rx_timing of frame n, and */                                      \
            /* window n+1's buffer (window n-1) and mi_{n-1} are free */                                       \
            if (n > 0) spin_wait(&bseq[gi][p ^ 1][bb], (n - 1) / 2 + 1, a.err, &dead_s);                       \
            STAMP(7);                                                                                          \
            const int c0 = bch0(bb), nl = ((a.roles & kFrontIdle) && n >= 2) ? 0 : blive(bb);                  \
            const int i0 = kBlkCh * bb + cbeg;                                                                 \
            int pmi = 0;                                                                                       \
            for (int c = 0; c < nl; c++, k++) {                                                                \
                const int ch = c0 + c;                                                                         \
                float2* dcur = decs[f][k % kDecBuf];                                                           \
                mix<DM, kFrD>(lane, pf, g, P, M);                                                              \
                STAMP(0);                                                                                      \
                if (c > 0)                                                                                     \
                    store_window(lane, pmi, decs[f][(k - 1) % kDecBuf], wout + (size_t)(ch - 1) * kWinStride); \
                STAMP(4);                                                                                      \
                {   /* the next channel: of this block, the next live block, or frame n+1 */                   \
                    int nb = bb, nc = c + 1, nn = n;                                                           \
                    if (nc >= nl) {                                                                            \
                        nc = 0;                                                                                \
                        nb = bb + 1;                                                                           \
                        while (nb < kChainWaves && blive(nb) == 0) nb++;                                       \
                        if (nb == kChainWaves) { nb = 0; nn = n + 1; }                                         \
                    }                                                                                          \
                    if (nn < a.F) prefetch<DM, CG, kFrD>(srcs(a, bch0(nb) + nc, nn), lane, pf);                \
                }                                                                                              \
                wave_lds_sync();                                                                               \
                STAMP(1);                                                                                      \
                pmi = front_channel<MODE, HP, kSplitD>(lane, rt_s[gi][p][i0 + c], M, dcur, BT, p2tab,         \
                                              a.heads + ((size_t)ch * a.F + n) * kHeadOut FACC_ARG);           \
                if (lane == 0) mi_s[gi][p ^ 1][i0 + c] = pmi;                                                  \
                if (c + 1 == nl) store_window(lane, pmi, dcur, wout + (size_t)ch * kWinStride);                \
                wave_lds_sync();                                                                               \
                STAMP(6);                                                                                      \
            }                                                                                                  \
            signal_add(&fcnt[gi][p][bb], 1, lane);                                                             \
            STAMP(5);                                                                                          \
        }                                                                                                      \
    } while (0)
            if constexpr (QUAD) {
                auto frame_iter = [&](auto cg, int n) {
                    constexpr bool CG = decltype(cg)::value;
                    QPSK_DUAL_FRONT_FRAME(CG);
                };
                for (int n = 0; n < a.F && n < 2; n++) frame_iter(std::false_type{}, n);
                for (int n = 2; n < a.F; n++) frame_iter(std::true_type{}, n);
            } else {
                for (int n = 0; n < a.F; n++) QPSK_DUAL_FRONT_FRAME(false);
            }
#undef QPSK_DUAL_FRONT_FRAME
            STAMP_FLUSH();
            for (int bb = 0; bb < kChainWaves; bb++)
                carry_history<DM>(a.in, a.hist, a.F, bch0(bb), blive(bb), lane);
        }
        __syncthreads();
        if (wave < kBackWaves && (wave & 1) == 0) {   // state after the call's last frame
            const int gi = (wave >> 1) / kChainWaves;
            const int sub = QUAD ? lane >> 2 : lane;
            const int idx = kBlkCh * ((wave >> 1) % kChainWaves) + sub;
            const int ch = (grp0 + gi) * W + idx;
            if (sub < kBlkCh && ch < a.nch && (!QUAD || (lane & 3) == 0)) {
                const unsigned ge = a.g0 + (unsigned)a.F;
                mi_of(a, ge)[ch] = mi_s[gi][a.F & 1][idx];
                rt_of(a, ge)[ch] = rt_s[gi][a.F & 1][idx];
            }
        }
        return;
    }
    if (wave < kBackWaves) {
        // ------------------------------------------------------------ back
        const int gi = wave;
        const int ch = (grp0 + gi) * QK_GROUP + lane;
        const bool live = ch < a.nch;
        const bool any = (grp0 + gi) * QK_GROUP < a.nch;
        if (((a.roles >> 4) & 3) == 2) __builtin_amdgcn_s_setprio(2);
        STAMP_DECL
        for (int n = 0; n < a.F; n++) {
            const int p = n & 1;
            if (any && (a.roles & 1)) {
                const int rt = rt_s[gi][p][lane];
                back_frame(a, live ? ch : 0, live, n, mi_s[gi][p][lane], [=] { return rt; },
                           win_of(a, a.g0 + (unsigned)n) + (size_t)(live ? ch : 0) * kWinStride,
                           &rt_s[gi][p ^ 1][lane], [] {});
            }
            else
                rt_s[gi][p ^ 1][lane] = rt_s[gi][p][lane];
            STAMP(13);
            TAIL_ARRIVE();
            __syncthreads();
            STAMP(14);
            TAIL_BACK();
        }
        STAMP_FLUSH();
        if (live) {   // per-channel state after the call's last frame
            const unsigned ge = a.g0 + (unsigned)a.F;
            mi_of(a, ge)[ch] = mi_s[gi][a.F & 1][lane];
            rt_of(a, ge)[ch] = rt_s[gi][a.F & 1][lane];
        }
    } else {
        // ------------------------------------------------------------ front
        // channel by channel: mix (prefetched samples) -> store the previous
        // channel's window -> prefetch the next channel -> FIR/correlate/argmax
        // the split FIR (fir_split) and, to keep the channel loop's per-lane
        // constants out of scratch beside it, recomputed prefetch offsets
        constexpr bool kSplit = MODE == 0 && !HP && QPSK_FIR_SPLIT;
        constexpr int kFr = kSplit ? QPSK_FRESH_SPLIT : QPSK_FRESH;
        const int f = wave - kBackWaves;
        const int gi = f / kFrontPer;
        const int cbeg = (f % kFrontPer) * kFrontCh;
        const int ch0 = (grp0 + gi) * QK_GROUP + cbeg;
        const int nlive = max(0, min(kFrontCh, a.nch - ch0));
        float2* M = Ms[f];
        const bool on = (a.roles & 2) != 0 && nlive > 0;
        if (((a.roles >> 4) & 3) == 1) __builtin_amdgcn_s_setprio(2);
        int pf[kPf<DM>];
        if (on) prefetch<DM, false, kFr>(srcs(a, ch0, 0), lane, pf);
        STAMP_DECL
        for (int n = 0; n < a.F; n++) {
            const int p = n & 1;
            const unsigned g = a.g0 + (unsigned)n;
            float2* wout = win_of(a, g + 1u);
            int pmi = 0;
            // roles bits 8-15 (stagger, kStagger): the second half of the front waves
            // (the younger partner on each SIMD) starts each frame that many x
            // 512 cycles late, so partners' FIR and MFMA/LDS phases interleave
            // (MI355X_MICROARCH.md "two waves per SIMD", item 9)
            for (int z = (f >= kFrontWaves / 2) ? (a.roles >> 8) & 255 : 0; z > 0; z--)
                __builtin_amdgcn_s_sleep(8);
            for (int c = 0; on && c < nlive; c++) {
                const int ch = ch0 + c;
                float2* dcur = decs[f][c % kDecBuf];
                // QPSK_LATE_YIELD (A/B knob): the last K channels of a frame at
                // the back wave's issue priority, so the back (the frame's last
                // wave) gets its share before the fronts reach the barrier
                if (QPSK_LATE_YIELD > 0 && c == nlive - QPSK_LATE_YIELD && ((a.roles >> 4) & 3) == 1)
                    __builtin_amdgcn_s_setprio(0);
                mix<DM, kFr>(lane, pf, g, P, M);
                STAMP(0);
                if (c > 0) store_window(lane, pmi, decs[f][(c - 1) % kDecBuf], wout + (size_t)(ch - 1) * kWinStride);
                {   // next channel of this frame, else the first of the next frame
                    const bool same = c + 1 < nlive;
                    if (same || n + 1 < a.F)
                        prefetch<DM, false, kFr>(srcs(a, same ? ch + 1 : ch0, same ? n : n + 1), lane, pf);
                }
                wave_lds_sync();
                STAMP(1);
                pmi = front_channel<MODE, HP, kSplit>(lane, rt_s[gi][p][cbeg + c], M, dcur, BT, p2tab,
                                              a.heads + ((size_t)ch * a.F + n) * kHeadOut FACC_ARG);
                if (lane == 0) mi_s[gi][p ^ 1][cbeg + c] = pmi;
                if (c + 1 == nlive) store_window(lane, pmi, dcur, wout + (size_t)ch * kWinStride);
                wave_lds_sync();
                STAMP(6);
            }
            TAIL_ARRIVE();
            __syncthreads();
            if (QPSK_LATE_YIELD > 0 && ((a.roles >> 4) & 3) == 1) __builtin_amdgcn_s_setprio(2);
            STAMP(7);
        }
        STAMP_FLUSH();
        carry_history<DM>(a.in, a.hist, a.F, ch0, nlive, lane);
    }
}

// ---------------------------------------------------------------- host side

float bits2f(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}

}  // namespace

// rx_kernel instantiations (pick_shape below)
struct Shape {
    enum Kind { k4x2, k2x4d, k1x8d64, k1x8q16, k1x8q32 };
    int kind;
    int roles;
};

// front stagger, 512-cycle units (roles bits 8-15): round 1 measured 12 as
// -0.7%; on round 5's kernels 0 is -0.4% (profiles/r05_stagger_ab.txt)
constexpr int kStagger = 0;
// rx_data_kernel grid: persistent, 4 workgroups of 256 per CU (other geometries
// measured within 2%, profiles/r01_data_ab.txt)
constexpr int kDataGrid = 1024, kDataBlock = 256;

struct qpsk_ctx {
    int device = 0, nch = 0, ngroup = 0;
    int mode = QPSK_MODE_REFERENCE;   // receiver semantics, fixed at creation
    float* d_fft = nullptr;           // FFT-hunt tables (kFftHT floats), QPSK_MODE_FFT_HUNT
    uint64_t frames = 0;
    hipStream_t stream = nullptr;
    float2* d_ptab = nullptr;
    unsigned long long* d_ks = nullptr;
    int16_t* d_hist = nullptr;
    float2* d_win[2] = {nullptr, nullptr};
    int* d_mi[2] = {nullptr, nullptr};
    int* d_rt[2] = {nullptr, nullptr};
    // data-symbol jobs of valid frames (rx_kernel -> rx_data_kernel)
    float4* d_jobs = nullptr;
    size_t jobs_cap = 0;           // jobs (one per channel-frame of the largest call)
    unsigned* d_njobs = nullptr;   // [2] counters, alternating by call
    uint64_t calls = 0;
    // staging for the host-memory entry point (qpsk_rx_batch): one device block
    // [in | bits | valid | trace | soft] (stage_grow) and, for small calls, a
    // pinned host image of it, so a call is one H2D and one D2H of pinned
    // memory (the per-frame drop-in qpsk_rx_frame is such a call)
    char* s_dev = nullptr;
    char* s_pin = nullptr;          // pinned, same layout; only while small
    size_t s_frames = 0;
    // kernel-span accounting: events before rx_kernel, between the kernels, after
    // rx_data_kernel
    static constexpr int kEv = 64;
    hipEvent_t ev[kEv][3] = {};
    int ev_frames[kEv] = {};
    int ev_n = 0;
    bool timing = false;
    // roles + front issue priority + front stagger (0 since round 5; 12 x 512
    // cycles was -0.7% in round 1,
    // profiles/r01_stagger_ab.txt); QPSK_ABLATE (profiling), QPSK_FORCE_EXACT /
    // QPSK_DEBUG_STALL (tests)
    int roles = 3 | (1 << 4) | (kStagger << 8);
    int ncu = 256;              // compute units of the device
    int shape = -1;             // Shape::Kind forced by QPSK_SHAPE (A/B runs); -1: by batch size
    int width = 0;              // dual-chain group width forced by QPSK_WIDTH; 0: by batch size
    int prio = -1;              // issue priority forced by QPSK_PRIO (0 none, 1 front, 2 back)
    bool headpass = false;      // QPSK_HEADPASS: the FIR-head pre-pass (reference mode only)
    float2* d_heads = nullptr;  // its outputs, [nch][F][102] for the largest call
    size_t heads_cap = 0;       // channel-frames d_heads holds
    int* d_err = nullptr;       // [0] device error word (kErrStall), taken by qpsk_rx_sync;
                                // [1] the value it took
    hipEvent_t done = nullptr;  // recorded after the latest call's kernels, on its stream
    bool called = false;        // `done` has been recorded
    float pend_ms[2] = {0.0f, 0.0f};
    int pend_frames = 0;
    uint64_t epoch = 0;         // qpsk_rx_reset() count (qpsk_rx_epoch)
    int stall_calls = -1;       // QPSK_DEBUG_STALL=first: the stall only in the first launch; -1: every call
    int short_block = 0;        // QPSK_DEBUG_BLOCK (tests): rx_kernel launched one wave short
    uint64_t launches = 0;      // calls launched over the context's life (qpsk_rx_reset keeps it)
    const qpsk_stream* owner = nullptr;   // the stream this context belongs to, if any
    // a call reported QPSK_ESTALL since the last reset: the per-channel state
    // is undefined, and qpsk_rx_state_save refuses to export it
    bool stalled = false;
    // qpsk_rx_state_load of a channel range into a fresh context (frame 0) from
    // a snapshot at frame G != 0: the context takes frame index G, so every
    // channel must be loaded before it may receive (asm_left channels to go;
    // asm_cover marks the loaded ones)
    std::vector<uint8_t> asm_cover;
    int asm_left = 0;
};

extern "C" int qpsk_rx_timing_split(qpsk_ctx* c, float* ms_rx, float* ms_data, int* frames);

static int herr(hipError_t e) { return e == hipSuccess ? QPSK_OK : QPSK_EHIP - (int)e; }
#define HCHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return herr(e_); } while (0)

// The receiver's constant tables, built once per process on first use (a C++11
// function-local static: its initialisation is thread-safe, and contexts
// created from several host threads at once share the one read-only copy).
struct RxTables {
    float2 ptab[QK_FRAME];                 // P[t] * 2^-14
    unsigned long long ksf[QK_KS_FRAMES];  // keystream bits of frame f, 62 per word
};

static RxTables* make_rx_tables() {
    RxTables* t = new RxTables();
    // P[t] = R^(t+1): fbb_rx_phase *= fbb_rx_rect (src/qpsk.c:139), fp32, host
    const float rr = bits2f(QK_RX_RECT_RE_BITS), ri = bits2f(QK_RX_RECT_IM_BITS);
    volatile float pr = 1.0f, pi = 0.0f;  // volatile: keep every op a rounded fp32 op
    for (int k = 0; k < QK_FRAME; k++) {
        const float a = pr * rr - pi * ri;
        const float b = pr * ri + pi * rr;
        pr = a;
        pi = b;
        t->ptab[k] = make_float2(a * 0x1p-14f, b * 0x1p-14f);  // exact power-of-two scale
    }
    // keystream of the RX descrambler (src/scramble.c:57-69), 62 bits per frame
    std::vector<uint8_t> ks(QK_KS_PERIOD);
    uint16_t m = QK_SEED;
    for (int k = 0; k < QK_KS_PERIOD; k++) {
        const uint16_t o = (uint16_t)(((m & 2) >> 1) ^ (m & 1));
        ks[k] = (uint8_t)o;
        m = (uint16_t)((m >> 1) | (o << 14));
    }
    for (int f = 0; f < QK_KS_FRAMES; f++) {
        unsigned long long w = 0;
        for (int b = 0; b < QK_NBITS; b++)
            w |= (unsigned long long)ks[(62 * f + b) % QK_KS_PERIOD] << b;
        t->ksf[f] = w;
    }
    return t;
}

static const RxTables& rx_tables() {
    static const RxTables* const t = make_rx_tables();   // never freed: process lifetime
    return *t;
}

// state arrays cover whole workgroups of the largest shape (kMaxGroups groups)
static size_t nslot(const qpsk_ctx* c) {
    return (size_t)((c->ngroup + kMaxGroups - 1) / kMaxGroups) * kMaxGroups * QK_GROUP;
}

static int ctx_alloc(qpsk_ctx* c) {
    HCHECK(hipMalloc(&c->d_ptab, sizeof(float2) * QK_FRAME));
    HCHECK(hipMalloc(&c->d_ks, sizeof(unsigned long long) * QK_KS_FRAMES));
    HCHECK(hipMalloc(&c->d_hist, sizeof(int16_t) * nslot(c) * 2 * QK_FRAME));
    HCHECK(hipMalloc(&c->d_njobs, sizeof(unsigned) * 2));
    HCHECK(hipMalloc(&c->d_err, 2 * sizeof(int)));
    HCHECK(hipEventCreateWithFlags(&c->done, hipEventDisableTiming));
    for (int p = 0; p < 2; p++) {
        HCHECK(hipMalloc(&c->d_win[p], sizeof(float2) * nslot(c) * kWinStride));
        HCHECK(hipMalloc(&c->d_mi[p], sizeof(int) * nslot(c)));
        HCHECK(hipMalloc(&c->d_rt[p], sizeof(int) * nslot(c)));
    }
    return QPSK_OK;
}

extern "C" int qpsk_rx_reset(qpsk_ctx* c) {
    if (!c) return QPSK_EINVAL;
    // a stream's chunks in flight run on the state cleared here (and one that
    // stalled must keep its epoch): refuse until the stream is drained
    if (c->owner && qpsk_stream_pending(c->owner) > 0) return QPSK_EBUSY;
    HCHECK(hipSetDevice(c->device));
    // calls in flight on other streams read and write the state cleared here
    if (c->called) HCHECK(hipEventSynchronize(c->done));
    const size_t ns = nslot(c);
    HCHECK(hipMemsetAsync(c->d_hist, 0, sizeof(int16_t) * ns * 2 * QK_FRAME, c->stream));
    HCHECK(hipMemsetAsync(c->d_njobs, 0, sizeof(unsigned) * 2, c->stream));
    HCHECK(hipMemsetAsync(c->d_err, 0, 2 * sizeof(int), c->stream));
    for (int p = 0; p < 2; p++) {
        HCHECK(hipMemsetAsync(c->d_win[p], 0, sizeof(float2) * ns * kWinStride, c->stream));
        HCHECK(hipMemsetAsync(c->d_mi[p], 0, sizeof(int) * ns, c->stream));
    }
    int* rt0 = (int*)malloc(sizeof(int) * ns);
    if (!rt0) return QPSK_ENOMEM;
    for (size_t i = 0; i < ns; i++) rt0[i] = QK_RT0;
    hipError_t e = hipMemcpy(c->d_rt[0], rt0, sizeof(int) * ns, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(c->d_rt[1], rt0, sizeof(int) * ns, hipMemcpyHostToDevice);
    free(rt0);
    HCHECK(e);
    HCHECK(hipStreamSynchronize(c->stream));
    c->frames = 0;
    c->calls = 0;
    c->epoch++;
    c->stalled = false;
    c->asm_cover.clear();
    c->asm_left = 0;
    return QPSK_OK;
}

int* qpsk_rx_err_word(qpsk_ctx* c) { return c ? c->d_err : nullptr; }
void qpsk_rx_set_owner(qpsk_ctx* c, const qpsk_stream* s) { if (c) c->owner = s; }
uint64_t qpsk_rx_epoch(const qpsk_ctx* c) { return c ? c->epoch : 0; }
void qpsk_rx_mark_stalled(qpsk_ctx* c, uint64_t epoch) {
    if (c && epoch == c->epoch) c->stalled = true;
}

static void ctx_free(qpsk_ctx* c) {
    for (int i = 0; i < qpsk_ctx::kEv; i++)
        for (int j = 0; j < 3; j++)
            if (c->ev[i][j]) (void)hipEventDestroy(c->ev[i][j]);
    (void)hipFree(c->d_ptab);
    (void)hipFree(c->d_err);
    if (c->done) (void)hipEventDestroy(c->done);
    (void)hipFree(c->d_jobs);
    (void)hipFree(c->d_njobs);
    (void)hipFree(c->d_ks);
    (void)hipFree(c->d_hist);
    (void)hipFree(c->d_fft);
    (void)hipFree(c->d_heads);
    for (int p = 0; p < 2; p++) {
        (void)hipFree(c->d_win[p]);
        (void)hipFree(c->d_mi[p]);
        (void)hipFree(c->d_rt[p]);
    }
    (void)hipFree(c->s_dev);
    (void)hipHostFree(c->s_pin);
    if (c->stream) (void)hipStreamDestroy(c->stream);
}

// The FFT hunt's LDS image (fft_hunt()): twiddles of fft_alloc(256, 0/1)
// (src/fft.c:67-74, host C: qpsk_fft_host.c), Q = conj(fft(c)) with
// c[i] = conj(preambletable[i]) for i < 128 (computed by the GPU FFT itself),
// and kf_work's input permutation.
static int fft_hunt_tables(qpsk_ctx* c) {
    float tab[kFftHT];
    qpsk_fft_twiddle_table(256, 0, tab);
    qpsk_fft_twiddle_table(256, 1, tab + 512);
    qpsk_fft_perm_table(256, reinterpret_cast<int*>(tab + 1536));
    float cq[512] = {};
    for (int i = 0; i < QK_NPRE; i++) {
        cq[2 * i] = (float)QK_PRE[i];
        cq[2 * i + 1] = -(float)QK_PRE[i];
    }
    int r = QPSK_OK;
    qpsk_fft_plan* plan = qpsk_fft_alloc(c->device, 256, 0, &r);
    if (!plan) return r;
    r = qpsk_fft(plan, cq, cq, 1);
    qpsk_fft_free(plan);
    if (r != QPSK_OK) return r;
    for (int k = 0; k < 256; k++) {
        tab[1024 + 2 * k] = cq[2 * k];
        tab[1024 + 2 * k + 1] = -cq[2 * k + 1];
    }
    HCHECK(hipMalloc(&c->d_fft, sizeof tab));
    HCHECK(hipMemcpy(c->d_fft, tab, sizeof tab, hipMemcpyHostToDevice));
    return QPSK_OK;
}

extern "C" qpsk_ctx* qpsk_rx_create(int device, int nch, int* err) {
    return qpsk_rx_create_mode(device, nch, QPSK_MODE_REFERENCE, err);
}

extern "C" qpsk_ctx* qpsk_rx_create_mode(int device, int nch, int mode, int* err) {
    int dummy;
    if (!err) err = &dummy;
    if (nch < 1 || mode < 0 || mode > (QPSK_MODE_DEC752 | QPSK_MODE_FFT_HUNT)) {
        *err = QPSK_EINVAL;
        return nullptr;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
        *err = QPSK_ENODEV;
        return nullptr;
    }
    qpsk_ctx* c = new (std::nothrow) qpsk_ctx();
    if (!c) { *err = QPSK_ENOMEM; return nullptr; }
    c->device = device;
    c->nch = nch;
    c->mode = mode;
    c->ngroup = (nch + QK_GROUP - 1) / QK_GROUP;
    if (const char* ab = getenv("QPSK_ABLATE")) {   // timing experiments; output invalid
        if (!strcmp(ab, "front")) c->roles = (c->roles & ~3) | 2;
        else if (!strcmp(ab, "back")) c->roles = (c->roles & ~3) | 1;
        else if (!strcmp(ab, "frontidle")) c->roles |= kFrontIdle;
    }
    if (getenv("QPSK_FORCE_EXACT")) c->roles |= kForceExact;   // tests: exact-division path
    if (const char* ds = getenv("QPSK_DEBUG_STALL")) {          // tests: the QPSK_ESTALL path
        c->roles |= kDebugStall;
        if (!strcmp(ds, "first")) c->stall_calls = 1;           // only the context's first call
    }
    if (getenv("QPSK_DEBUG_BLOCK")) c->short_block = 64;          // tests: rx_kernel's launch-shape guard
    if (const char* w = getenv("QPSK_WIDTH")) {
        const int v = atoi(w);
        c->width = (v == 16 || v == 32 || v == 64) ? v : 0;
    }
    if (const char* hv = getenv("QPSK_HEADPASS")) c->headpass = atoi(hv) != 0 && mode == QPSK_MODE_REFERENCE;
    if (const char* sv = getenv("QPSK_STAGGER")) {   // A/B: the 4x2 fronts' stagger, 512-cycle units
        const int v = atoi(sv);
        if (v >= 0 && v < 256) c->roles = (c->roles & ~(255 << 8)) | (v << 8);
    }
    if (const char* pv = getenv("QPSK_PRIO"))
        c->prio = !strcmp(pv, "none") ? 0 : !strcmp(pv, "front") ? 1 : !strcmp(pv, "back") ? 2 : -1;
    if (const char* sh = getenv("QPSK_SHAPE")) {
        c->shape = !strcmp(sh, "4x2") ? Shape::k4x2
                 : !strcmp(sh, "2x4d") ? Shape::k2x4d
                 : !strcmp(sh, "1x8") ? Shape::k1x8d64 : -1;
    }
    int r = herr(hipSetDevice(device));
    if (r == QPSK_OK) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess &&
            n > 0)
            c->ncu = n;
    }
    if (r == QPSK_OK) r = herr(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    if (r == QPSK_OK) r = ctx_alloc(c);
    if (r == QPSK_OK) {
        const RxTables& t = rx_tables();
        r = herr(hipMemcpy(c->d_ptab, t.ptab, sizeof t.ptab, hipMemcpyHostToDevice));
        if (r == QPSK_OK) r = herr(hipMemcpy(c->d_ks, t.ksf, sizeof t.ksf, hipMemcpyHostToDevice));
    }
    if (r == QPSK_OK && (mode & QPSK_MODE_FFT_HUNT)) r = fft_hunt_tables(c);
    if (r == QPSK_OK) r = qpsk_rx_reset(c);
    if (r != QPSK_OK) {
        ctx_free(c);
        delete c;
        *err = r;
        return nullptr;
    }
    *err = QPSK_OK;
    return c;
}

// ---------------------------------------------------------------- state snapshots
// qpsk_batch.h qpsk_rx_state_*: the per-channel state the kernels carry from
// one call to the next, for the context's frame index G (the next frame):
// the history int16 [2][1880] (frames G-2, G-1: carry_history), window G's
// row float2 [168] with mi_G, and rt_G, the last three in the arrays of
// parity G & 1 (rx_kernel reads mi_of / rt_of / win_of (g0) at a call's start
// and writes parity g0 + F at its end).  Layout: a 64-byte header, then the
// four fields channel-major, each as one contiguous block.
namespace {
constexpr char kStateMagic[8] = {'Q', 'P', 'S', 'K', 'S', 'T', 'A', '1'};
struct StateHdr {
    char magic[8];
    uint32_t version, hdr_bytes;
    int32_t mode, n;
    uint64_t frame;
    uint32_t hist_bytes, win_bytes;   // per channel
    uint8_t pad[24];
};
static_assert(sizeof(StateHdr) == 64, "state header");
constexpr size_t kHistB = sizeof(int16_t) * 2 * QK_FRAME, kWinB = sizeof(float2) * kWinStride;
constexpr size_t kChanB = kHistB + kWinB + 2 * sizeof(int);
constexpr int kWinObs = QK_NPRE + QK_NDSYM + 5;   // slots 0..163 = dec[mi-1 .. mi+162]
static_assert(kWinObs == 164 && kWinObs <= kWinStride, "window slots");
}  // namespace

extern "C" size_t qpsk_rx_state_size(int n) { return n < 1 ? 0 : sizeof(StateHdr) + (size_t)n * kChanB; }

// the checks both directions share; waits for the context's calls in flight
static int state_begin(qpsk_ctx* c, int c0, int n, const void* buf, size_t size) {
    if (!c || !buf || n < 1 || c0 < 0 || c0 > c->nch - n || size < qpsk_rx_state_size(n)) return QPSK_EINVAL;
    if (c->owner && qpsk_stream_pending(c->owner) > 0) return QPSK_EBUSY;
    HCHECK(hipSetDevice(c->device));
    if (c->called) HCHECK(hipEventSynchronize(c->done));
    return QPSK_OK;
}

extern "C" int qpsk_rx_state_save(qpsk_ctx* c, int c0, int n, void* buf, size_t size) {
    int r = state_begin(c, c0, n, buf, size);
    if (r != QPSK_OK) return r;
    // channels still to be loaded (qpsk_rx_state_load) hold no state of frame G
    if (c->asm_left > 0) return QPSK_EINVAL;
    // a stall (reported, or still in the error word: peeked, not taken, so
    // qpsk_rx_sync still reports it) leaves the state undefined
    if (!c->stalled) {
        int e = 0;
        HCHECK(hipMemcpyAsync(&e, c->d_err, sizeof e, hipMemcpyDeviceToHost, c->stream));
        HCHECK(hipStreamSynchronize(c->stream));
        if (e != 0) return QPSK_ESTALL;
    }
    if (c->stalled) return QPSK_ESTALL;
    StateHdr h{};
    memcpy(h.magic, kStateMagic, sizeof h.magic);
    h.version = 1;
    h.hdr_bytes = sizeof h;
    h.mode = c->mode;
    h.n = n;
    h.frame = c->frames;
    h.hist_bytes = (uint32_t)kHistB;
    h.win_bytes = (uint32_t)kWinB;
    char* o = static_cast<char*>(buf);
    memcpy(o, &h, sizeof h);
    o += sizeof h;
    const int p = (int)(c->frames & 1u);
    const size_t nn = (size_t)n;
    HCHECK(hipMemcpyAsync(o, c->d_hist + (size_t)c0 * 2 * QK_FRAME, nn * kHistB, hipMemcpyDeviceToHost, c->stream));
    o += nn * kHistB;
    char* w = o;
    HCHECK(hipMemcpyAsync(o, c->d_win[p] + (size_t)c0 * kWinStride, nn * kWinB, hipMemcpyDeviceToHost, c->stream));
    o += nn * kWinB;
    HCHECK(hipMemcpyAsync(o, c->d_mi[p] + c0, nn * sizeof(int), hipMemcpyDeviceToHost, c->stream));
    o += nn * sizeof(int);
    HCHECK(hipMemcpyAsync(o, c->d_rt[p] + c0, nn * sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HCHECK(hipStreamSynchronize(c->stream));
    // window slots past dec[mi+162] (the last data symbol's taps, SURVEY.md
    // A.6) are never read; the fronts leave whatever their dec buffer held
    // there (the split FIR skips dec[255..289] when mi < 93).  Zeroed, so a
    // snapshot is a function of the channel's state alone.
    for (size_t i = 0; i < nn; i++)
        memset(w + i * kWinB + kWinObs * sizeof(float2), 0, (kWinStride - kWinObs) * sizeof(float2));
    return QPSK_OK;
}

extern "C" int qpsk_rx_state_load(qpsk_ctx* c, int c0, int n, const void* buf, size_t size) {
    int r = state_begin(c, c0, n, buf, size);
    if (r != QPSK_OK) return r;
    StateHdr h;
    memcpy(&h, buf, sizeof h);
    if (memcmp(h.magic, kStateMagic, sizeof h.magic) != 0 || h.version != 1 || h.hdr_bytes != sizeof h ||
        h.n != n || h.mode != c->mode || h.hist_bytes != kHistB || h.win_bytes != kWinB)
        return QPSK_EINVAL;
    if (c->frames != h.frame && c->frames != 0) return QPSK_EINVAL;   // one frame index per context
    // a channel range at frame G != 0 into a fresh context moves the context's
    // frame index to G for every channel: the others must be loaded too
    // (from this or other snapshots at G) before the context may receive
    const bool assemble = c->asm_left > 0 || (c->frames == 0 && h.frame != 0 && n < c->nch);
    const char* o = static_cast<const char*>(buf) + sizeof h;
    const int p = (int)(h.frame & 1u);
    const size_t nn = (size_t)n;
    HCHECK(hipMemcpyAsync(c->d_hist + (size_t)c0 * 2 * QK_FRAME, o, nn * kHistB, hipMemcpyHostToDevice, c->stream));
    o += nn * kHistB;
    HCHECK(hipMemcpyAsync(c->d_win[p] + (size_t)c0 * kWinStride, o, nn * kWinB, hipMemcpyHostToDevice, c->stream));
    o += nn * kWinB;
    HCHECK(hipMemcpyAsync(c->d_mi[p] + c0, o, nn * sizeof(int), hipMemcpyHostToDevice, c->stream));
    o += nn * sizeof(int);
    HCHECK(hipMemcpyAsync(c->d_rt[p] + c0, o, nn * sizeof(int), hipMemcpyHostToDevice, c->stream));
    HCHECK(hipStreamSynchronize(c->stream));
    if (assemble) {
        if (c->asm_cover.empty()) {
            c->asm_cover.assign((size_t)c->nch, 0);
            c->asm_left = c->nch;
        }
        for (int i = c0; i < c0 + n; i++)
            if (!c->asm_cover[(size_t)i]) {
                c->asm_cover[(size_t)i] = 1;
                c->asm_left--;
            }
        if (c->asm_left == 0) c->asm_cover.clear();
    }
    c->frames = h.frame;
    return QPSK_OK;
}

extern "C" void qpsk_rx_destroy(qpsk_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    ctx_free(c);
    delete c;
}

extern "C" int qpsk_rx_channels(const qpsk_ctx* c) { return c ? c->nch : 0; }
extern "C" int qpsk_rx_mode(const qpsk_ctx* c) { return c ? c->mode : QPSK_EINVAL; }
extern "C" uint64_t qpsk_rx_frames(const qpsk_ctx* c) { return c ? c->frames : 0; }

// The rx_kernel instantiation for a call (DESIGN.md "Kernels"):
//   > 2 groups per CU (C3's 65,536 channels): 4x2, one back wave per group;
//   2 groups per CU: 2x4 with dual-chain backs (11% faster at 32,768 channels,
//     profiles/r01_dual_ab.txt);
//   1 group per CU: 1x8 dual-chain, at the narrowest group width (16/32/64
//     channels) that still fits the batch in one wave of workgroups: quad
//     backs at W = 16 / 32, lane backs at W = 64 (quad backs there need 16
//     waves, whose 128-VGPR budget spills the front: profiles/r02_quad_ab.txt)
//     with back priority and 2 channels moved off each front wave that
//     shares a SIMD with a back wave (-3%, profiles/r01_split_ab.txt).
// QPSK_SHAPE (4x2 | 2x4d | 1x8) and QPSK_WIDTH force a shape for tests and A/B
// runs.  Measured and dropped (records in profiles/, DESIGN.md "Measured and
// not kept"): 4x1d, 2x4 and 1x8 with single back waves, the early-terminated
// flow kernel (r01_flow_ab.txt), lane backs at W = 16 / 32, one front per SIMD
// (1x4) and the 4x3 C3 shape (round 5 removed the last three from the build).
static Shape pick_shape(const qpsk_ctx* c) {
    Shape sh{c->shape, c->roles};
    if (sh.kind < 0)
        sh.kind = c->ngroup <= c->ncu ? Shape::k1x8d64 : c->ngroup <= 2 * c->ncu ? Shape::k2x4d
                                                                                  : Shape::k4x2;
    if (sh.kind == Shape::k1x8d64) {
        const int W = c->width > 0 ? c->width
                    : (size_t)c->nch <= (size_t)16 * c->ncu ? 16
                    : (size_t)c->nch <= (size_t)32 * c->ncu ? 32 : 64;
        if (W == 16) sh.kind = Shape::k1x8q16;
        else if (W == 32) sh.kind = Shape::k1x8q32;
        else sh.roles = (sh.roles & ~((3 << 4) | (15 << 16))) | (2 << 4) | (2 << 16);
    }
    if (c->prio >= 0) sh.roles = (sh.roles & ~(3 << 4)) | (c->prio << 4);
    return sh;
}

// The two launches of a call (qpsk_rx_batch_device), with the device error word
// the call's progress waits report to: the context's (qpsk_rx_sync takes it),
// or a caller's own (qpsk_stream.hip: one per stream slot, so a stall is
// reported with the chunk it belongs to).
int qpsk_rx_launch(qpsk_ctx* c, const int16_t* d_in, int F, uint8_t* d_bits, uint8_t* d_valid,
                   int32_t* d_trace, float* d_soft, hipStream_t s, int* d_err, int* err_to) {
    if (!c || F < 0 || (F > 0 && (!d_in || !d_bits || !d_valid))) return QPSK_EINVAL;
    if (c->asm_left > 0) return QPSK_EINVAL;   // channels not yet loaded (qpsk_rx_state_load)
    if (F == 0) return QPSK_OK;
    if ((reinterpret_cast<uintptr_t>(d_in) & 15u) != 0) return QPSK_EINVAL;  // int4 loads
    HCHECK(hipSetDevice(c->device));
    if (!d_err) d_err = c->d_err;
    const size_t need = (size_t)c->nch * (size_t)F;   // every frame valid, at most
    // job slots are addressed with 32-bit byte offsets (slot * 16); 2^28 channel-
    // frames would be 1 TB of input, beyond any device's memory
    if (need >= ((size_t)1 << 28)) return QPSK_EINVAL;
    if (need > c->jobs_cap) {
        HCHECK(hipDeviceSynchronize());   // an earlier call may still use the queue
        (void)hipFree(c->d_jobs);
        c->d_jobs = nullptr;
        c->jobs_cap = 0;
        HCHECK(hipMalloc(&c->d_jobs, sizeof(float4) * kJobF4 * need));
        c->jobs_cap = need;
    }
    const bool hp = c->headpass;
    if (hp && need > c->heads_cap) {
        HCHECK(hipDeviceSynchronize());   // an earlier call may still read the heads
        (void)hipFree(c->d_heads);
        c->d_heads = nullptr;
        c->heads_cap = 0;
        HCHECK(hipMalloc(&c->d_heads, sizeof(float2) * kHeadOut * need));
        c->heads_cap = need;
    }
    int slot = -1;
    if (c->timing) {
        if (c->ev_n == qpsk_ctx::kEv) {   // pool full: fold pending spans into the totals
            float ms[2];
            int l;
            int r = qpsk_rx_timing_split(c, &ms[0], &ms[1], &l);
            if (r != QPSK_OK) return r;
            c->pend_ms[0] += ms[0];
            c->pend_ms[1] += ms[1];
            c->pend_frames += l;
        }
        slot = c->ev_n++;
        for (int j = 0; j < 3; j++)
            if (!c->ev[slot][j]) HCHECK(hipEventCreate(&c->ev[slot][j]));
        HCHECK(hipEventRecord(c->ev[slot][0], s));
        c->ev_frames[slot] = F;
    }
    const int parity = (int)(c->calls & 1u);
    Shape sh = pick_shape(c);
    if (c->stall_calls >= 0 && c->launches >= (uint64_t)c->stall_calls) sh.roles &= ~kDebugStall;
#define QPSK_LAUNCH(GG, FF, MM, DD, WW, QQ, HH)                                                \
    hipLaunchKernelGGL((rx_kernel<GG, FF, MM, DD, WW, QQ, HH>),                                \
                       dim3((unsigned)((c->nch + (size_t)GG * WW - 1) / ((size_t)GG * WW))),   \
                       dim3(64 * (kBackWavesOf<GG, FF, MM, DD, WW, QQ> + (GG) * (FF)) - c->short_block), 0, s, \
                       d_in, c->d_hist, c->d_ptab,                                             \
                       c->d_ks, c->d_win[0], c->d_win[1], c->d_mi[0], c->d_mi[1], c->d_rt[0],  \
                       c->d_rt[1], d_bits, d_valid, d_trace, reinterpret_cast<float2*>(d_soft), \
                       c->d_jobs, c->d_njobs + parity, c->nch, F,                               \
                       (unsigned)(c->frames & 0xffffffffu), sh.roles,                          \
                       HH ? reinterpret_cast<const float*>(c->d_heads) : c->d_fft,             \
                       (unsigned long long)c->jobs_cap, d_err)
#define QPSK_LAUNCH_SHAPES(MM, HH)                                                             \
    do {                                                                                       \
        switch (sh.kind) {                                                                     \
            case Shape::k2x4d: QPSK_LAUNCH(2, 4, MM, true, 64, false, HH); break;              \
            case Shape::k1x8d64: QPSK_LAUNCH(1, 8, MM, true, 64, false, HH); break;            \
            case Shape::k1x8q16: QPSK_LAUNCH(1, 8, MM, true, 16, true, HH); break;             \
            case Shape::k1x8q32: QPSK_LAUNCH(1, 8, MM, true, 32, true, HH); break;             \
            default: QPSK_LAUNCH(4, 2, MM, false, 64, false, HH); break;                       \
        }                                                                                      \
    } while (0)
#define QPSK_LAUNCH_MODE(MM) QPSK_LAUNCH_SHAPES(MM, false)
    if (hp) {   // head pre-pass: every channel-frame's F_{n+1}, then the frame loop
        const size_t ncf = (size_t)c->nch * (size_t)F;
        hipLaunchKernelGGL(head_kernel, dim3((unsigned)((ncf + 3) / 4)), dim3(256), 0, s, d_in,
                           c->d_hist, c->d_ptab, c->d_heads, c->nch, F,
                           (unsigned)(c->frames & 0xffffffffu));
        HCHECK(hipGetLastError());
        QPSK_LAUNCH_SHAPES(0, true);
    } else
    switch (c->mode) {
        case 0: QPSK_LAUNCH_MODE(0); break;
        case 1: QPSK_LAUNCH_MODE(1); break;
        case 2: QPSK_LAUNCH_MODE(2); break;
        default: QPSK_LAUNCH_MODE(3); break;
    }
#undef QPSK_LAUNCH_MODE
#undef QPSK_LAUNCH_SHAPES
#undef QPSK_LAUNCH
    HCHECK(hipGetLastError());
    if (slot >= 0) HCHECK(hipEventRecord(c->ev[slot][1], s));
    // at most one job per channel-frame: a small call (the per-frame drop-in
    // qpsk_rx_frame is one job at most) launches only the workgroups it can use
    const unsigned dgrid = (unsigned)std::min<size_t>(kDataGrid, (need + kDataBlock - 1) / kDataBlock);
    hipLaunchKernelGGL(rx_data_kernel, dim3(dgrid), dim3(kDataBlock), 0, s, c->d_jobs,
                       (unsigned long long)c->jobs_cap, c->d_njobs, c->d_ks, d_bits,
                       reinterpret_cast<float2*>(d_soft), parity, c->roles & kForceExact, c->d_err,
                       err_to);
    HCHECK(hipGetLastError());
    if (slot >= 0) HCHECK(hipEventRecord(c->ev[slot][2], s));
    HCHECK(hipEventRecord(c->done, s));
    c->called = true;
    c->frames += (uint64_t)F;
    c->calls++;
    c->launches++;
    return QPSK_OK;
}

extern "C" int qpsk_rx_batch_device(qpsk_ctx* c, const int16_t* d_in, int F, uint8_t* d_bits,
                                    uint8_t* d_valid, int32_t* d_trace, float* d_soft,
                                    void* stream) {
    return qpsk_rx_launch(c, d_in, F, d_bits, d_valid, d_trace, d_soft, (hipStream_t)stream,
                          nullptr, nullptr);
}

namespace {
// read and clear the error word in one atomic exchange: a stall reported by a
// kernel between a read and a separate clear cannot be lost
__global__ void err_take_kernel(int* err) {
    if (threadIdx.x == 0) err[1] = atomicExch(&err[0], 0);
}
}  // namespace

// Waits for the context's latest call (an event recorded on its stream, so the
// stream may since have been destroyed) and reports a device-side failure of
// any call since the previous check.  Calls on one context depend on each
// other through the per-channel state, so they are ordered (one stream, or
// streams the caller chains); the latest call's completion covers them all.
extern "C" int qpsk_rx_sync(qpsk_ctx* c) {
    if (!c) return QPSK_EINVAL;
    HCHECK(hipSetDevice(c->device));
    if (c->called) HCHECK(hipEventSynchronize(c->done));
    hipLaunchKernelGGL(err_take_kernel, dim3(1), dim3(64), 0, c->stream, c->d_err);
    HCHECK(hipGetLastError());
    int e = 0;
    HCHECK(hipMemcpyAsync(&e, c->d_err + 1, sizeof e, hipMemcpyDeviceToHost, c->stream));
    HCHECK(hipStreamSynchronize(c->stream));
    if (e != 0) c->stalled = true;
    return e == 0 ? QPSK_OK : QPSK_ESTALL;
}

extern "C" int qpsk_rx_timing_enable(qpsk_ctx* c, int on) {
    if (!c) return QPSK_EINVAL;
    c->timing = on != 0;
    return QPSK_OK;
}

extern "C" int qpsk_rx_timing_split(qpsk_ctx* c, float* ms_rx, float* ms_data, int* frames) {
    if (!c || !ms_rx || !ms_data || !frames) return QPSK_EINVAL;
    HCHECK(hipSetDevice(c->device));
    float tot[2] = {c->pend_ms[0], c->pend_ms[1]};
    int nf = c->pend_frames;
    for (int i = 0; i < c->ev_n; i++) {
        HCHECK(hipEventSynchronize(c->ev[i][2]));
        for (int k = 0; k < 2; k++) {
            float t = 0.0f;
            HCHECK(hipEventElapsedTime(&t, c->ev[i][k], c->ev[i][k + 1]));
            tot[k] += t;
        }
        nf += c->ev_frames[i];
    }
    c->ev_n = 0;
    c->pend_ms[0] = c->pend_ms[1] = 0.0f;
    c->pend_frames = 0;
    *ms_rx = tot[0];
    *ms_data = tot[1];
    *frames = nf;
    return QPSK_OK;
}

extern "C" int qpsk_rx_timing_collect(qpsk_ctx* c, float* ms, int* frames) {
    if (!ms) return QPSK_EINVAL;
    float a = 0.0f, b = 0.0f;
    const int r = qpsk_rx_timing_split(c, &a, &b, frames);
    if (r == QPSK_OK) *ms = a + b;
    return r;
}

// byte offsets of the staging block for cf channel-frames
struct Stage {
    size_t in, bits, valid, err, trace, soft, end;
};
static Stage stage_of(size_t cf) {
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    Stage g;
    g.in = 0;
    g.bits = up(sizeof(int16_t) * cf * QK_FRAME);
    g.valid = g.bits + cf * QK_NBITS;   // bits, valid and the taken error word
    g.err = (g.valid + cf + 3) & ~(size_t)3;   // adjacent: one D2H
    g.trace = up(g.err + sizeof(int));
    g.soft = up(g.trace + sizeof(int32_t) * cf * 4);
    g.end = up(g.soft + sizeof(float) * cf * QK_NDSYM * 2);
    return g;
}
// calls up to this many input bytes stage through pinned memory
constexpr size_t kPinnedStage = (size_t)8 << 20;
// calls up to this many channel-frames (the drop-in qpsk_rx_frame: one) run
// their kernels on the pinned block itself, no copies (QPSK_ZERO_COPY A/B knob)
#ifndef QPSK_ZERO_COPY
#define QPSK_ZERO_COPY 64
#endif
constexpr size_t kZeroCopyCF = QPSK_ZERO_COPY;

static int stage_grow(qpsk_ctx* c, size_t F) {
    if (F <= c->s_frames) return QPSK_OK;
    (void)hipFree(c->s_dev);
    (void)hipHostFree(c->s_pin);
    c->s_dev = nullptr;
    c->s_pin = nullptr;
    c->s_frames = 0;
    const size_t cf = (size_t)c->nch * F;
    const Stage g = stage_of(cf);
    HCHECK(hipMalloc(&c->s_dev, g.end));
    if (g.bits <= kPinnedStage) HCHECK(hipHostMalloc((void**)&c->s_pin, g.end, hipHostMallocDefault));
    c->s_frames = F;
    return QPSK_OK;
}

extern "C" int qpsk_rx_batch(qpsk_ctx* c, const int16_t* in, int F, uint8_t* bits, uint8_t* valid,
                             int32_t* trace, float* soft) {
    if (!c || F < 0 || (F > 0 && (!in || !bits || !valid))) return QPSK_EINVAL;
    if (c->asm_left > 0) return QPSK_EINVAL;   // channels not yet loaded (qpsk_rx_state_load)
    if (F == 0) return QPSK_OK;
    HCHECK(hipSetDevice(c->device));
    int r = stage_grow(c, (size_t)F);
    if (r != QPSK_OK) return r;
    const size_t cf = (size_t)c->nch * F;
    const Stage g = stage_of(cf);
    char* d = c->s_dev;
    const bool pin = c->s_pin && g.bits <= kPinnedStage;
    // pinned: the caller's input is copied into the pinned image (a host memcpy)
    // and moves in one DMA, outputs come back in one; pageable otherwise
    char* h = pin ? c->s_pin : nullptr;
    const size_t nin = sizeof(int16_t) * cf * QK_FRAME;
    const size_t ntr = sizeof(int32_t) * cf * 4, nso = sizeof(float) * cf * QK_NDSYM * 2;
    if (pin && cf <= kZeroCopyCF) {
        // tiny calls: the kernels read the input from and write the outputs to
        // the pinned block directly (device-accessible host memory); the
        // per-frame latency is then two launches and one synchronisation, not
        // two copies besides (the kernels touch these few KB once)
        memcpy(h + g.in, in, nin);
        // the error word comes back with the outputs (rx_data_kernel's err_to)
        r = qpsk_rx_launch(c, reinterpret_cast<int16_t*>(h + g.in), F,
                           reinterpret_cast<uint8_t*>(h + g.bits), reinterpret_cast<uint8_t*>(h + g.valid),
                           trace ? reinterpret_cast<int32_t*>(h + g.trace) : nullptr,
                           soft ? reinterpret_cast<float*>(h + g.soft) : nullptr, c->stream, nullptr,
                           reinterpret_cast<int*>(h + g.err));
        if (r != QPSK_OK) return r;
        HCHECK(hipStreamSynchronize(c->stream));
        memcpy(bits, h + g.bits, cf * QK_NBITS);
        memcpy(valid, h + g.valid, cf);
        if (trace) memcpy(trace, h + g.trace, ntr);
        if (soft) memcpy(soft, h + g.soft, nso);
        int e;
        memcpy(&e, h + g.err, sizeof e);
        if (e != 0) c->stalled = true;
        return e != 0 ? QPSK_ESTALL : QPSK_OK;
    }
    if (pin) memcpy(h + g.in, in, nin);
    HCHECK(hipMemcpyAsync(d + g.in, pin ? (const void*)(h + g.in) : (const void*)in, nin,
                          hipMemcpyHostToDevice, c->stream));
    // pinned: the error word is taken by rx_data_kernel (err_to) into the
    // staging block right after the valid flags, so bits, flags and error word
    // come back in one copy; pageable: qpsk_rx_sync() takes it
    r = qpsk_rx_launch(c, reinterpret_cast<int16_t*>(d + g.in), F,
                       reinterpret_cast<uint8_t*>(d + g.bits), reinterpret_cast<uint8_t*>(d + g.valid),
                       trace ? reinterpret_cast<int32_t*>(d + g.trace) : nullptr,
                       soft ? reinterpret_cast<float*>(d + g.soft) : nullptr, c->stream, nullptr,
                       pin ? reinterpret_cast<int*>(d + g.err) : nullptr);
    if (r != QPSK_OK) return r;
    if (!pin) {
        HCHECK(hipMemcpyAsync(bits, d + g.bits, cf * QK_NBITS, hipMemcpyDeviceToHost, c->stream));
        HCHECK(hipMemcpyAsync(valid, d + g.valid, cf, hipMemcpyDeviceToHost, c->stream));
        if (trace) HCHECK(hipMemcpyAsync(trace, d + g.trace, ntr, hipMemcpyDeviceToHost, c->stream));
        if (soft) HCHECK(hipMemcpyAsync(soft, d + g.soft, nso, hipMemcpyDeviceToHost, c->stream));
        return qpsk_rx_sync(c);
    }
    // (the error word was taken in one atomic exchange behind rx_kernel, as
    // qpsk_rx_sync does: a stream on this context, qpsk_stream_ctx, ORs its
    // slots' stalls into the same word from another HIP stream, and a read
    // followed by a separate clear could lose one merged in between)
    HCHECK(hipMemcpyAsync(h + g.bits, d + g.bits, g.err + sizeof(int) - g.bits, hipMemcpyDeviceToHost, c->stream));
    if (trace) HCHECK(hipMemcpyAsync(h + g.trace, d + g.trace, ntr, hipMemcpyDeviceToHost, c->stream));
    if (soft) HCHECK(hipMemcpyAsync(h + g.soft, d + g.soft, nso, hipMemcpyDeviceToHost, c->stream));
    HCHECK(hipStreamSynchronize(c->stream));
    memcpy(bits, h + g.bits, cf * QK_NBITS);
    memcpy(valid, h + g.valid, cf);
    if (trace) memcpy(trace, h + g.trace, ntr);
    if (soft) memcpy(soft, h + g.soft, nso);
    int e;
    memcpy(&e, h + g.err, sizeof e);
    if (e != 0) c->stalled = true;
    return e != 0 ? QPSK_ESTALL : QPSK_OK;
}

#ifdef QPSK_STAMPS
extern "C" int qpsk_debug_stamps(unsigned long long* out16, int reset) {
    if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 16) != hipSuccess)
        return -1;
    if (reset) {
        unsigned long long z[16] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
}
#endif

#ifndef QPSK_KERNEL_HASH
#define QPSK_KERNEL_HASH "unknown"
#endif
// the Makefile's hash of the receive kernels' sources and build rules
extern "C" const char* qpsk_kernel_hash(void) { return QPSK_KERNEL_HASH; }

extern "C" const char* qpsk_strerror(int err) {
    switch (err) {
        case QPSK_OK: return "success";
        case QPSK_EINVAL: return "invalid argument";
        case QPSK_ENOMEM: return "out of memory";
        case QPSK_ENODEV: return "no such HIP device";
        case -4: return "every stream slot is in flight (retrieve first)";
        case QPSK_ESTALL: return "a device-side progress wait exceeded its bound; the call's outputs are undefined";
        default: break;
    }
    if (err <= QPSK_EHIP) return hipGetErrorString((hipError_t)(QPSK_EHIP - err));
    return "unknown error";
}
