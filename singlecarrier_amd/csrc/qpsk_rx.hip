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
// Per frame the work splits at the preamble decision (DESIGN.md "Kernels"):
//   front  (wave per channel, LDS-staged):  mixer -> RRC FIR (only the ~290
//          observable outputs) -> decimation -> 128-lag preamble correlation
//          -> argmax -> equalizer window dec[mi .. mi+162] to HBM.
//   back   (lane per channel):  128 train_eq + 31 data_eq steps of the
//          square-root Kalman equalizer, slicer, descrambler.
// The front of frame n+1 needs only rx_timing of frame n, so one launch runs
// front(n+1) and back(n) side by side; both are roles of one kernel.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "qpsk_batch.h"
#include "qpsk_consts.h"

#pragma clang fp contract(off)

namespace {

constexpr int kBlock = 256;            // 4 waves
constexpr int kWaves = kBlock / 64;
constexpr int kChPerWave = QK_GROUP / kWaves;   // front: 16 channels per wave
// front LDS per wave (float2 units): M1 = m_{n-2}[1832..1879] ++ m_{n-1}[0..1191],
// M2 = m_{n-1}[1832..1879] ++ m_n[0..103], dec[0..289], TU[0..255]
constexpr int kM1 = 48 + 1192, kM2 = 48 + 104, kDec = 296, kTU = 256;
constexpr int kLdsWave = kM1 + kM2 + kDec + kTU;

constexpr unsigned long long pre_mask(int half) {
    unsigned long long m = 0;
    for (int i = 0; i < 64; i++)
        if (QK_PRE[half * 64 + i] > 0) m |= 1ull << i;
    return m;
}
constexpr unsigned long long kPreLo = pre_mask(0), kPreHi = pre_mask(1);

struct StepArgs {
    const int16_t* in;       // [nch][F][1880]
    const int16_t* hist;     // [nch][2][1880]: frames -2, -1 of this call
    const float2* ptab;      // [1880] mixer table P[t] * 2^-14
    const float2* win_rd;    // [ngroup][163][64] equalizer window of frame n
    float2* win_wr;          // ... of frame n+1
    const int* mi_rd;
    int* mi_wr;
    const int* rt_rd;
    int* rt_wr;
    uint8_t* bits;           // [nch][F][62]
    uint8_t* valid;          // [nch][F]
    int32_t* trace;          // [nch][F][4] or null
    float2* soft;            // [nch][F][31] or null
    unsigned long long ks;   // keystream bits 62g .. 62g+61 of frame g
    int nch, F, n, nb_back;
    unsigned g;              // global frame index of frame n
};

__device__ __forceinline__ const int16_t* frame_ptr(const StepArgs& a, int ch, int k) {
    return k >= 0 ? a.in + ((size_t)ch * a.F + k) * QK_FRAME
                  : a.hist + ((size_t)ch * 2 + (k + 2)) * QK_FRAME;
}

// 8 samples of one frame -> mixed cf32 (src/qpsk.c:139-144 as (-1)^G P[t] x 2^-14)
__device__ __forceinline__ void mix8(const int16_t* x, int t0, bool neg, const float2* ptab,
                                     float2* dst) {
    const int4 raw = *reinterpret_cast<const int4*>(x + t0);
    const int w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
    for (int e = 0; e < 8; e++) {
        const float v = (float)(int16_t)((e & 1) ? (w[e >> 1] >> 16) : (w[e >> 1] & 0xffff));
        float2 p = ptab[t0 + e];
        if (neg) { p.x = -p.x; p.y = -p.y; }
        dst[e] = make_float2(p.x * v, p.y * v);
    }
}

// one RRC output, src/fir.c:36-42 (M points at the sample under tap 0)
__device__ __forceinline__ float2 fir_at(const float2* M) {
    float yr = 0.0f, yi = 0.0f;
#pragma unroll
    for (int k = 0; k < QK_NTAPS; k++) {
        const float2 m = M[k];
        yr = yr + m.x * QK_RRC[k];
        yi = yi + m.y * QK_RRC[k];
    }
    return make_float2(yr * QK_GAIN, yi * QK_GAIN);
}

// ---------------------------------------------------------------- front role
__device__ void front_group(const StepArgs& a, int grp, float2* lds) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float2* M1 = lds + w * kLdsWave;
    float2* M2 = M1 + kM1;
    float2* dec = M2 + kM2;
    float2* TU = dec + kDec;
    const int n = a.n;
    const bool neg_m1 = ((a.g - 1u) & 1u) != 0;   // frame g-1
    const bool neg_02 = (a.g & 1u) != 0;          // frames g and g-2

    for (int c = 0; c < kChPerWave; c++) {
        const int col = w * kChPerWave + c;
        const int ch = grp * QK_GROUP + col;
        const bool live = ch < a.nch;
        if (live) {
            // 1. load + mix: 149 + 6 + 13 + 6 eight-sample items
            const int16_t* xm1 = frame_ptr(a, ch, n - 1);
            const int16_t* xm2 = frame_ptr(a, ch, n - 2);
            const int16_t* x0 = frame_ptr(a, ch, n);
            for (int it = lane; it < 174; it += 64) {
                if (it < 149) mix8(xm1, 8 * it, neg_m1, a.ptab, M1 + 48 + 8 * it);
                else if (it < 155) mix8(xm2, 1832 + 8 * (it - 149), neg_02, a.ptab, M1 + 8 * (it - 149));
                else if (it < 168) mix8(x0, 8 * (it - 155), neg_02, a.ptab, M2 + 48 + 8 * (it - 155));
                else mix8(xm1, 1832 + 8 * (it - 168), neg_m1, a.ptab, M2 + 8 * (it - 168));
            }
        }
        __syncthreads();
        if (live) {
            // 2. FIR: D_n[i] = fir_out[5i + rt] (decimation, model A) and
            //    F_{n+1}[j] = fir_out'[j], j < 102 -> dec_{n+1} = [D_n, F_{n+1}]
            const int rt = a.rt_rd[ch];
            for (int o = lane; o < QK_NDECOBS; o += 64) {
                const float2* base = o < QK_NDEC ? M1 + 5 * o + rt : M2 + (o - QK_NDEC);
                dec[o] = fir_at(base);
            }
        }
        __syncthreads();
        if (live) {
            // 3. p*(dr-di, di+dr) == preambletable[i]*dec (p = +-1, exact)
            for (int j = lane; j < 255; j += 64) {
                const float2 d = dec[j];
                TU[j] = make_float2(d.x - d.y, d.y + d.x);
            }
        }
        __syncthreads();
        if (live) {
            // 4. correlate lags 2*lane and 2*lane+1, terms in index order
            float r0 = 0.0f, i0 = 0.0f, r1 = 0.0f, i1 = 0.0f;
            const float2* tu = TU + 2 * lane;
#pragma unroll
            for (int s = 0; s <= QK_NPRE; s++) {
                const float2 v = tu[s];
                if (s < QK_NPRE) {
                    if (QK_PRE[s] > 0) { r0 = r0 + v.x; i0 = i0 + v.y; }
                    else { r0 = r0 - v.x; i0 = i0 - v.y; }
                }
                if (s >= 1) {
                    if (QK_PRE[s - 1] > 0) { r1 = r1 + v.x; i1 = i1 + v.y; }
                    else { r1 = r1 - v.x; i1 = i1 - v.y; }
                }
            }
            float c0 = r0 * r0 + i0 * i0;          // cnormf, src/qpsk.c:75-80
            float c1 = r1 * r1 + i1 * i1;
            // 5. first strict maximum over lags (src/qpsk.c:176-183); NaN never wins
            c0 = (c0 == c0) ? c0 : -1.0f;
            c1 = (c1 == c1) ? c1 : -1.0f;
            float best = c0;
            int idx = 2 * lane;
            if (c1 > best) { best = c1; idx = 2 * lane + 1; }
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const float ob = __shfl_xor(best, off);
                const int oi = __shfl_xor(idx, off);
                if (ob > best || (ob == best && oi < idx)) { best = ob; idx = oi; }
            }
            const int mi = best > 0.0f ? idx : 0;
            // 6. equalizer window of frame n+1, layout [grp][k][64 channels]
            float2* wo = a.win_wr + (size_t)grp * QK_NWIN * QK_GROUP + col;
            for (int k = lane; k < QK_NWIN; k += 64) wo[(size_t)k * QK_GROUP] = dec[mi + k];
            if (lane == 0) a.mi_wr[ch] = mi;
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------- back role
struct Kal {
    float eqr[5], eqi[5];    // eq_coeff     src/kalman.c:19
    float gr[5], gi[5];      // kalman_gain  src/kalman.c:20
    float ur[5][5], ui[5][5];// u (upper triangle used)  src/kalman.c:25
    float d[5];              // src/kalman.c:29
};

// kalman_calculate (src/kalman.c:85-141) then update_eq (src/equalizer.c:25-40)
__device__ __forceinline__ void update_eq(Kal& k, const float (&xr)[5], const float (&xi)[5],
                                          float er, float ei) {
    const float E = QK_KAL_E, q = QK_KAL_Q;
    float fr[5], fi[5], a[5];
    fr[0] = xr[0];                              // 6.2  f0 = conj(x0)
    fi[0] = -xi[0];
#pragma unroll
    for (int j = 1; j < 5; j++) {
        // u0j*conj(x0) + conj(xj) (the double conj() sum rounds to the fp32 sum)
        float pr = k.ur[0][j] * xr[0] - k.ui[0][j] * (-xi[0]);
        float pi = k.ur[0][j] * (-xi[0]) + k.ui[0][j] * xr[0];
        fr[j] = pr + xr[j];
        fi[j] = pi + (-xi[j]);
#pragma unroll
        for (int i = 1; i < j; i++) {
            pr = k.ur[i][j] * xr[i] - k.ui[i][j] * (-xi[i]);
            pi = k.ur[i][j] * (-xi[i]) + k.ui[i][j] * xr[i];
            fr[j] = fr[j] + pr;
            fi[j] = fi[j] + pi;
        }
    }
#pragma unroll
    for (int j = 0; j < 5; j++) {               // 6.4  g = f*d
        k.gr[j] = fr[j] * k.d[j];
        k.gi[j] = fi[j] * k.d[j];
    }
    a[0] = E + (k.gr[0] * fr[0] - k.gi[0] * (-fi[0]));   // 6.5
#pragma unroll
    for (int j = 1; j < 5; j++) a[j] = a[j - 1] + (k.gr[j] * fr[j] - k.gi[j] * (-fi[j]));
    const float hq = 1.0f + q;                  // 6.7
    const float ht = a[4] * q;
    float y = 1.0f / (a[0] + ht);               // 6.19 (correctly rounded)
    k.d[0] = k.d[0] * ((hq * (E + ht)) * y);    // 6.20
#pragma unroll
    for (int j = 1; j < 5; j++) {
        const float B = a[j - 1] + ht;          // 6.21
        const float hr = (-fr[j]) * y;          // 6.11
        const float hi = (-fi[j]) * y;
        y = 1.0f / (a[j] + ht);                 // 6.22
        k.d[j] = k.d[j] * ((hq * B) * y);       // 6.13
#pragma unroll
        for (int i = 0; i < j; i++) {
            const float b1r = k.ur[i][j], b1i = k.ui[i][j];
            const float cgr = k.gr[i], cgi = -k.gi[i];
            k.ur[i][j] = b1r + (hr * cgr - hi * cgi);           // 6.15
            k.ui[i][j] = b1i + (hr * cgi + hi * cgr);
            k.gr[i] = k.gr[i] + (k.gr[j] * b1r - k.gi[j] * (-b1i));  // 6.16
            k.gi[i] = k.gi[i] + (k.gr[j] * (-b1i) + k.gi[j] * b1r);
        }
    }
    // update_eq: error *= kalman_y; eq += error * conj(g)
    er = er * y;
    ei = ei * y;
#pragma unroll
    for (int i = 0; i < 5; i++) {
        const float cgr = k.gr[i], cgi = -k.gi[i];
        k.eqr[i] = k.eqr[i] + (er * cgr - ei * cgi);
        k.eqi[i] = k.eqi[i] + (er * cgi + ei * cgr);
    }
}

__device__ void back_group(const StepArgs& a, int grp) {
    const int lane = threadIdx.x & 63;
    const int ch = grp * QK_GROUP + lane;
    const bool live = ch < a.nch;
    const int chs = live ? ch : 0;
    const int mi = a.mi_rd[chs];
    const int rt = a.rt_rd[chs];
    const float2* wp = a.win_rd + (size_t)grp * QK_NWIN * QK_GROUP + lane;

    Kal k;                                         // kalman_reset, src/kalman.c:42-55
#pragma unroll
    for (int i = 0; i < 5; i++) {
        k.eqr[i] = k.eqi[i] = k.gr[i] = k.gi[i] = 0.0f;
        k.d[i] = 1.0f;
#pragma unroll
        for (int j = 0; j < 5; j++) k.ur[i][j] = k.ui[i][j] = 0.0f;
    }
    float xr[5], xi[5];
#pragma unroll
    for (int i = 0; i < 5; i++) {
        const float2 v = wp[(size_t)i * QK_GROUP];
        xr[i] = v.x;
        xi[i] = v.y;
    }
    // equalize(): 128 x train_eq (src/qpsk.c:111-123, src/equalizer.c:45-58)
    int matches = 0;
    for (int i = 0; i < QK_NPRE; i++) {
        const float2 nx = wp[(size_t)(i + 5) * QK_GROUP];  // next window sample
        const unsigned long long m = i < 64 ? kPreLo : kPreHi;
        const float ref = ((m >> (i & 63)) & 1ull) ? 1.0f : -1.0f;
        float vr = 0.0f, vi = 0.0f;
#pragma unroll
        for (int t = 0; t < 5; t++) {
            vr = vr + (xr[t] * k.eqr[t] - xi[t] * k.eqi[t]);
            vi = vi + (xr[t] * k.eqi[t] + xi[t] * k.eqr[t]);
        }
        const float er = ref - vr;                 // conjf(ref - val) = (ref-vr, vi)
        update_eq(k, xr, xi, er, vi);
        if (er * ref > 0.0f) matches++;
#pragma unroll
        for (int t = 0; t < 4; t++) { xr[t] = xr[t + 1]; xi[t] = xi[t + 1]; }
        xr[4] = nx.x;
        xi[4] = nx.y;
    }
    const bool valid = live && matches > QK_MATCH_MIN;   // src/qpsk.c:196
    const size_t cf = (size_t)chs * a.F + a.n;
    uint16_t* bo = reinterpret_cast<uint16_t*>(a.bits + cf * QK_NBITS);
    float2* so = a.soft ? a.soft + cf * QK_NDSYM : nullptr;
    // data symbols (src/qpsk.c:204-215): data_eq + qpsk_demod + scramble
    for (int s = 0; s < QK_NDSYM; s++) {
        uint16_t out = 0;
        float sr = 0.0f, si = 0.0f;
        if (valid) {
            const float2 nx = wp[(size_t)(QK_NPRE + s + 5 < QK_NWIN ? QK_NPRE + s + 5 : QK_NWIN - 1) * QK_GROUP];
#pragma unroll
            for (int t = 0; t < 5; t++) {          // symbol = sum x * conj(eq)
                sr = sr + (xr[t] * k.eqr[t] - xi[t] * (-k.eqi[t]));
                si = si + (xr[t] * (-k.eqi[t]) + xi[t] * k.eqr[t]);
            }
            const int dI = sr < 0.0f, dQ = si < 0.0f;
            const float cr = dI ? -1.0f : 1.0f, cq = dQ ? -1.0f : 1.0f;
            update_eq(k, xr, xi, (cr - sr) * 0.1f, (cq - si) * 0.1f);
            const int q = dQ ^ (int)((a.ks >> (2 * s)) & 1ull);
            const int ib = dI ^ (int)((a.ks >> (2 * s + 1)) & 1ull);
            out = (uint16_t)(q | (ib << 8));       // bits[2s] = Q, bits[2s+1] = I
#pragma unroll
            for (int t = 0; t < 4; t++) { xr[t] = xr[t + 1]; xi[t] = xi[t + 1]; }
            xr[4] = nx.x;
            xi[4] = nx.y;
        }
        if (live) {
            bo[s] = out;
            if (so) so[s] = make_float2(sr, si);
        }
    }
    if (live) {
        const int rt_next = valid ? mi + QK_NPRE : rt;  // src/qpsk.c:219
        a.rt_wr[ch] = rt_next;
        a.valid[cf] = valid ? 1 : 0;
        if (a.trace) {
            int4* tp = reinterpret_cast<int4*>(a.trace + cf * 4);
            *tp = make_int4(mi, matches, valid ? 1 : 0, rt_next);
        }
    }
}

__global__ void __launch_bounds__(kBlock) rx_step_kernel(StepArgs a) {
    __shared__ float2 lds[kWaves * kLdsWave];
    const int b = blockIdx.x;
    if (b < a.nb_back) {
        const int grp = b * kWaves + (threadIdx.x >> 6);
        if (grp * QK_GROUP < a.nch) back_group(a, grp);
    } else {
        front_group(a, b - a.nb_back, lds);
    }
}

// carry the samples the next call needs: x_{N-1}[0..1191], x_{N-1}[1832..1879],
// x_{N-2}[1832..1879] (eight-sample units)
__global__ void hist_kernel(const int16_t* in, int16_t* hist, int nch, int F) {
    const int ch = blockIdx.x;
    if (ch >= nch) return;
    int16_t* h0 = hist + (size_t)ch * 2 * QK_FRAME;
    int16_t* h1 = h0 + QK_FRAME;
    const int16_t* last = in + ((size_t)ch * F + (F - 1)) * QK_FRAME;
    const int16_t* prev = F >= 2 ? in + ((size_t)ch * F + (F - 2)) * QK_FRAME : h1;
    for (int u = threadIdx.x; u < 6; u += blockDim.x) {
        const int t = 1832 + 8 * u;
        *reinterpret_cast<int4*>(h0 + t) = *reinterpret_cast<const int4*>(prev + t);
    }
    __syncthreads();  // F == 1 reads h1 before it is overwritten
    for (int u = threadIdx.x; u < 155; u += blockDim.x) {
        const int t = u < 149 ? 8 * u : 1832 + 8 * (u - 149);
        *reinterpret_cast<int4*>(h1 + t) = *reinterpret_cast<const int4*>(last + t);
    }
}

// ---------------------------------------------------------------- host side

float bits2f(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}

}  // namespace

struct qpsk_ctx {
    int device = 0, nch = 0, ngroup = 0;
    uint64_t frames = 0;
    hipStream_t stream = nullptr;
    float2* d_ptab = nullptr;
    int16_t* d_hist = nullptr;
    float2* d_win[2] = {nullptr, nullptr};
    int* d_mi[2] = {nullptr, nullptr};
    int* d_rt[2] = {nullptr, nullptr};
    unsigned long long ks[QK_KS_FRAMES];
    // staging for the host-memory entry point
    int16_t* s_in = nullptr;
    uint8_t* s_bits = nullptr;
    uint8_t* s_valid = nullptr;
    int32_t* s_trace = nullptr;
    float* s_soft = nullptr;
    size_t s_frames = 0;
    // kernel-span accounting: events around each call's step-kernel sequence
    static constexpr int kEv = 64;
    hipEvent_t ev[kEv][2] = {};
    int ev_launches[kEv] = {};
    int ev_n = 0;
    bool timing = false;
    float pend_ms = 0.0f;
    int pend_launches = 0;
};

extern "C" int qpsk_rx_timing_collect(qpsk_ctx* c, float* ms, int* launches);

static int herr(hipError_t e) { return e == hipSuccess ? QPSK_OK : QPSK_EHIP - (int)e; }
#define HCHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return herr(e_); } while (0)

static void build_tables(qpsk_ctx* c, float2* ptab) {
    // P[t] = R^(t+1): fbb_rx_phase *= fbb_rx_rect (src/qpsk.c:139), fp32, host
    const float rr = bits2f(QK_RX_RECT_RE_BITS), ri = bits2f(QK_RX_RECT_IM_BITS);
    volatile float pr = 1.0f, pi = 0.0f;  // volatile: keep every op a rounded fp32 op
    for (int t = 0; t < QK_FRAME; t++) {
        const float a = pr * rr - pi * ri;
        const float b = pr * ri + pi * rr;
        pr = a;
        pi = b;
        ptab[t] = make_float2(a * 0x1p-14f, b * 0x1p-14f);  // exact power-of-two scale
    }
    // keystream of the RX descrambler (src/scramble.c:57-69), 62 bits per frame
    static uint8_t ks[QK_KS_PERIOD];
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
        c->ks[f] = w;
    }
}

static int ctx_alloc(qpsk_ctx* c) {
    const size_t nslot = (size_t)c->ngroup * QK_GROUP;
    HCHECK(hipMalloc(&c->d_ptab, sizeof(float2) * QK_FRAME));
    HCHECK(hipMalloc(&c->d_hist, sizeof(int16_t) * nslot * 2 * QK_FRAME));
    for (int p = 0; p < 2; p++) {
        HCHECK(hipMalloc(&c->d_win[p], sizeof(float2) * (size_t)c->ngroup * QK_NWIN * QK_GROUP));
        HCHECK(hipMalloc(&c->d_mi[p], sizeof(int) * nslot));
        HCHECK(hipMalloc(&c->d_rt[p], sizeof(int) * nslot));
    }
    return QPSK_OK;
}

extern "C" int qpsk_rx_reset(qpsk_ctx* c) {
    if (!c) return QPSK_EINVAL;
    HCHECK(hipSetDevice(c->device));
    const size_t nslot = (size_t)c->ngroup * QK_GROUP;
    HCHECK(hipMemsetAsync(c->d_hist, 0, sizeof(int16_t) * nslot * 2 * QK_FRAME, c->stream));
    for (int p = 0; p < 2; p++) {
        HCHECK(hipMemsetAsync(c->d_win[p], 0, sizeof(float2) * (size_t)c->ngroup * QK_NWIN * QK_GROUP,
                              c->stream));
        HCHECK(hipMemsetAsync(c->d_mi[p], 0, sizeof(int) * nslot, c->stream));
    }
    int* rt0 = (int*)malloc(sizeof(int) * nslot);
    if (!rt0) return QPSK_ENOMEM;
    for (size_t i = 0; i < nslot; i++) rt0[i] = QK_RT0;
    hipError_t e = hipMemcpy(c->d_rt[0], rt0, sizeof(int) * nslot, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(c->d_rt[1], rt0, sizeof(int) * nslot, hipMemcpyHostToDevice);
    free(rt0);
    HCHECK(e);
    HCHECK(hipStreamSynchronize(c->stream));
    c->frames = 0;
    return QPSK_OK;
}

static void ctx_free(qpsk_ctx* c) {
    for (int i = 0; i < qpsk_ctx::kEv; i++)
        for (int j = 0; j < 2; j++)
            if (c->ev[i][j]) (void)hipEventDestroy(c->ev[i][j]);
    (void)hipFree(c->d_ptab);
    (void)hipFree(c->d_hist);
    for (int p = 0; p < 2; p++) {
        (void)hipFree(c->d_win[p]);
        (void)hipFree(c->d_mi[p]);
        (void)hipFree(c->d_rt[p]);
    }
    (void)hipFree(c->s_in);
    (void)hipFree(c->s_bits);
    (void)hipFree(c->s_valid);
    (void)hipFree(c->s_trace);
    (void)hipFree(c->s_soft);
    if (c->stream) (void)hipStreamDestroy(c->stream);
}

extern "C" qpsk_ctx* qpsk_rx_create(int device, int nch, int* err) {
    int dummy;
    if (!err) err = &dummy;
    if (nch < 1) { *err = QPSK_EINVAL; return nullptr; }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
        *err = QPSK_ENODEV;
        return nullptr;
    }
    qpsk_ctx* c = new (std::nothrow) qpsk_ctx();
    if (!c) { *err = QPSK_ENOMEM; return nullptr; }
    c->device = device;
    c->nch = nch;
    c->ngroup = (nch + QK_GROUP - 1) / QK_GROUP;
    int r = herr(hipSetDevice(device));
    if (r == QPSK_OK) r = herr(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    if (r == QPSK_OK) r = ctx_alloc(c);
    if (r == QPSK_OK) {
        float2 ptab[QK_FRAME];
        build_tables(c, ptab);
        r = herr(hipMemcpy(c->d_ptab, ptab, sizeof ptab, hipMemcpyHostToDevice));
    }
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

extern "C" void qpsk_rx_destroy(qpsk_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    ctx_free(c);
    delete c;
}

extern "C" int qpsk_rx_channels(const qpsk_ctx* c) { return c ? c->nch : 0; }
extern "C" uint64_t qpsk_rx_frames(const qpsk_ctx* c) { return c ? c->frames : 0; }

extern "C" int qpsk_rx_batch_device(qpsk_ctx* c, const int16_t* d_in, int F, uint8_t* d_bits,
                                    uint8_t* d_valid, int32_t* d_trace, float* d_soft,
                                    void* stream) {
    if (!c || F < 0 || (F > 0 && (!d_in || !d_bits || !d_valid))) return QPSK_EINVAL;
    if (F == 0) return QPSK_OK;
    HCHECK(hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)stream;
    const int nb_back = (c->ngroup + kWaves - 1) / kWaves;
    StepArgs a{};
    a.in = d_in;
    a.hist = c->d_hist;
    a.ptab = c->d_ptab;
    a.bits = d_bits;
    a.valid = d_valid;
    a.trace = d_trace;
    a.soft = reinterpret_cast<float2*>(d_soft);
    a.nch = c->nch;
    a.F = F;
    a.nb_back = nb_back;
    int slot = -1;
    if (c->timing) {
        if (c->ev_n == qpsk_ctx::kEv) {   // pool full: fold pending spans into the totals
            float ms;
            int l;
            int r = qpsk_rx_timing_collect(c, &ms, &l);
            if (r != QPSK_OK) return r;
            c->pend_ms += ms;
            c->pend_launches += l;
        }
        slot = c->ev_n++;
        for (int j = 0; j < 2; j++)
            if (!c->ev[slot][j]) HCHECK(hipEventCreate(&c->ev[slot][j]));
        HCHECK(hipEventRecord(c->ev[slot][0], s));
        c->ev_launches[slot] = F;
    }
    for (int n = 0; n < F; n++) {
        const uint64_t g = c->frames + (uint64_t)n;
        const int p = (int)(g & 1u);
        a.n = n;
        a.g = (unsigned)(g & 0xffffffffu);
        a.ks = c->ks[g % QK_KS_FRAMES];
        a.win_rd = c->d_win[p];
        a.win_wr = c->d_win[p ^ 1];
        a.mi_rd = c->d_mi[p];
        a.mi_wr = c->d_mi[p ^ 1];
        a.rt_rd = c->d_rt[p];
        a.rt_wr = c->d_rt[p ^ 1];
        hipLaunchKernelGGL(rx_step_kernel, dim3(nb_back + c->ngroup), dim3(kBlock), 0, s, a);
        HCHECK(hipGetLastError());
    }
    if (slot >= 0) HCHECK(hipEventRecord(c->ev[slot][1], s));
    hipLaunchKernelGGL(hist_kernel, dim3(c->nch), dim3(64), 0, s, d_in, c->d_hist, c->nch, F);
    HCHECK(hipGetLastError());
    c->frames += (uint64_t)F;
    return QPSK_OK;
}

extern "C" int qpsk_rx_timing_enable(qpsk_ctx* c, int on) {
    if (!c) return QPSK_EINVAL;
    c->timing = on != 0;
    return QPSK_OK;
}

extern "C" int qpsk_rx_timing_collect(qpsk_ctx* c, float* ms, int* launches) {
    if (!c || !ms || !launches) return QPSK_EINVAL;
    HCHECK(hipSetDevice(c->device));
    float tot = c->pend_ms;
    int nl = c->pend_launches;
    for (int i = 0; i < c->ev_n; i++) {
        HCHECK(hipEventSynchronize(c->ev[i][1]));
        float t = 0.0f;
        HCHECK(hipEventElapsedTime(&t, c->ev[i][0], c->ev[i][1]));
        tot += t;
        nl += c->ev_launches[i];
    }
    c->ev_n = 0;
    c->pend_ms = 0.0f;
    c->pend_launches = 0;
    *ms = tot;
    *launches = nl;
    return QPSK_OK;
}

static int stage_grow(qpsk_ctx* c, size_t F) {
    if (F <= c->s_frames) return QPSK_OK;
    (void)hipFree(c->s_in);
    (void)hipFree(c->s_bits);
    (void)hipFree(c->s_valid);
    (void)hipFree(c->s_trace);
    (void)hipFree(c->s_soft);
    c->s_in = nullptr; c->s_bits = nullptr; c->s_valid = nullptr; c->s_trace = nullptr; c->s_soft = nullptr;
    c->s_frames = 0;
    const size_t cf = (size_t)c->nch * F;
    HCHECK(hipMalloc(&c->s_in, sizeof(int16_t) * cf * QK_FRAME));
    HCHECK(hipMalloc(&c->s_bits, cf * QK_NBITS));
    HCHECK(hipMalloc(&c->s_valid, cf));
    HCHECK(hipMalloc(&c->s_trace, sizeof(int32_t) * cf * 4));
    HCHECK(hipMalloc(&c->s_soft, sizeof(float) * cf * QK_NDSYM * 2));
    c->s_frames = F;
    return QPSK_OK;
}

extern "C" int qpsk_rx_batch(qpsk_ctx* c, const int16_t* in, int F, uint8_t* bits, uint8_t* valid,
                             int32_t* trace, float* soft) {
    if (!c || F < 0 || (F > 0 && (!in || !bits || !valid))) return QPSK_EINVAL;
    if (F == 0) return QPSK_OK;
    HCHECK(hipSetDevice(c->device));
    int r = stage_grow(c, (size_t)F);
    if (r != QPSK_OK) return r;
    const size_t cf = (size_t)c->nch * F;
    HCHECK(hipMemcpyAsync(c->s_in, in, sizeof(int16_t) * cf * QK_FRAME, hipMemcpyHostToDevice,
                          c->stream));
    r = qpsk_rx_batch_device(c, c->s_in, F, c->s_bits, c->s_valid, trace ? c->s_trace : nullptr,
                             soft ? c->s_soft : nullptr, c->stream);
    if (r != QPSK_OK) return r;
    HCHECK(hipMemcpyAsync(bits, c->s_bits, cf * QK_NBITS, hipMemcpyDeviceToHost, c->stream));
    HCHECK(hipMemcpyAsync(valid, c->s_valid, cf, hipMemcpyDeviceToHost, c->stream));
    if (trace)
        HCHECK(hipMemcpyAsync(trace, c->s_trace, sizeof(int32_t) * cf * 4, hipMemcpyDeviceToHost,
                              c->stream));
    if (soft)
        HCHECK(hipMemcpyAsync(soft, c->s_soft, sizeof(float) * cf * QK_NDSYM * 2,
                              hipMemcpyDeviceToHost, c->stream));
    HCHECK(hipStreamSynchronize(c->stream));
    return QPSK_OK;
}

extern "C" const char* qpsk_strerror(int err) {
    switch (err) {
        case QPSK_OK: return "success";
        case QPSK_EINVAL: return "invalid argument";
        case QPSK_ENOMEM: return "out of memory";
        case QPSK_ENODEV: return "no such HIP device";
        default: break;
    }
    if (err <= QPSK_EHIP) return hipGetErrorString((hipError_t)(QPSK_EHIP - err));
    return "unknown error";
}
