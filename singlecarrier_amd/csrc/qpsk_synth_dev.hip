// qpsk_synth_dev.hip -- the synthetic multi-channel input of include/qpsk_synth.h
// generated on the GPU (qpsk_synth_device), identical to the host generator
// qpsk_synth_batch() (qpsk_synth.c), whose transmitter qpsk_tx_frame_state()
// reproduces the reference's qpsk_tx_frame (src/qpsk.c:278-322) bit for bit.
//
// The host generator walks each channel's stream with an explicit transmitter
// state.  Here every TX sample is computed independently, so the work spreads
// over (channel, block of 40 TX samples):
//   * the TX samples of channel c are the concatenation of its packets'
//     transmitter calls (preamble 640, then 8 x 155 data samples = 1880 per
//     packet); TX sample t lands at output position delay_c + 2783*(t/1880) +
//     t%1880 (the 903 zero samples after each packet are not transmitted);
//   * its FIR input (src/fir.c:29-43 over the zero-stuffed symbol stream) is
//     nonzero only at symbol instants, so y(t) = sum over the <= 10 symbols
//     u = t/5 - 9 .. t/5 of sym_u * c[5u - t + 48], i ascending.  Every
//     product is +-c exactly (symbols are +-1); the skipped zero-stuffed terms
//     add +-0, which changes at most the sign of a zero sum, and that cannot
//     reach the int16 output;
//   * symbol u of packet k = u/376 is the preamble value p_{u%376} (both
//     components) or data symbol d = u%376 - 128, whose dibit is draw
//     2 + 248k + d of the channel's splitmix64 stream (counter based:
//     draw n = mix(seed ^ c*K + n*K)), so no symbol depends on another;
//   * the carrier phase depends only on the sequence of transmitter calls,
//     the same for every channel: the host computes it once per call with the
//     reference's fp32 recurrence and per-call renormalisation.
// Positions no TX sample reaches (the leading delay, the gaps, the tail) are
// zero (a memset), and AWGN is added by a second, per-sample kernel with the
// host generator's counter-based Box-Muller.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <string.h>

#include "qpsk_consts.h"
#include "qpsk_synth.h"

#pragma clang fp contract(off)

namespace {

constexpr int kPacket = 2783;       // 640 + 8*155 + 903 output samples
constexpr int kTxPacket = 1880;     // transmitted samples per packet
constexpr int kSymPacket = 376;     // 128 + 8*31 symbols per packet
constexpr int kBlk = 40;            // TX samples per thread (8 symbol periods)
constexpr int kSyms = kBlk / 5 + 9; // symbols a block's FIR outputs touch (17)
constexpr uint64_t kGolden = 0x9E3779B97F4A7C15ull;
constexpr double kPData = 5.19e7;   // mean square of noiseless data samples

__host__ __device__ inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

constexpr unsigned long long pre_bits(int half) {
    unsigned long long m = 0;
    for (int i = 0; i < 64; i++)
        if (QK_PRE[half * 64 + i] > 0) m |= 1ull << i;
    return m;
}

// symbol u of channel stream s0 (draw n = mix(s0 + n*K)) as (re, im) = +-1, or
// 0 before the stream starts
__device__ inline float2 symbol(uint64_t s0, long u) {
    if (u < 0) return make_float2(0.0f, 0.0f);
    const long k = u / kSymPacket;
    const int d = (int)(u - k * kSymPacket);
    if (d < QK_NPRE) {
        constexpr unsigned long long lo = pre_bits(0), hi = pre_bits(1);
        const unsigned long long m = d < 64 ? lo : hi;
        const float p = ((m >> (d & 63)) & 1ull) ? 1.0f : -1.0f;
        return make_float2(p, p);
    }
    const uint64_t n = 2u + 248u * (uint64_t)k + (uint64_t)(d - QK_NPRE);
    const uint64_t dib = mix64(s0 + n * kGolden) & 3u;   // qpsk_mod, src/qpsk.c:251-256
    return make_float2((dib >> 1) ? -1.0f : 1.0f, (dib & 1u) ? -1.0f : 1.0f);
}

// grid: x = TX block, y = channel group of 64 (lane = channel)
__global__ void __launch_bounds__(64) tx_kernel(uint64_t seed, uint32_t c0, int nch,
                                                const float2* phase, long ntx, int16_t* out,
                                                long ns) {
    const int c = blockIdx.y * 64 + threadIdx.x;
    const long t0 = (long)blockIdx.x * kBlk;
    if (c >= nch || t0 >= ntx) return;
    const uint64_t s0 = seed ^ ((uint64_t)(c0 + (uint32_t)c) * kGolden);
    long delay = (long)(mix64(s0 + kGolden) % (uint64_t)kPacket);
    if (delay > ns) delay = ns;
    const long u0 = t0 / 5;
    float2 sym[kSyms];   // symbols u0-9 .. u0+7
#pragma unroll
    for (int v = 0; v < kSyms; v++) sym[v] = symbol(s0, u0 - 9 + v);
    int16_t* o = out + (size_t)c * ns;
#pragma unroll
    for (int j = 0; j < kBlk; j++) {
        const long t = t0 + j;
        const long k = t / kTxPacket;
        const long r = t - k * kTxPacket;
        const long p = delay + k * kPacket + r;
        // fir(): y = sum_i mem[i]*c[i], i ascending (src/fir.c:36-42), then GAIN
        float yr = 0.0f, yi = 0.0f;
#pragma unroll
        for (int v = j / 5 - 9; v <= j / 5; v++) {
            const int i = 5 * v - j + 48;
            if (i < 0 || i > 48) continue;
            yr = yr + sym[v + 9].x * QK_RRC[i];
            yi = yi + sym[v + 9].y * QK_RRC[i];
        }
        yr = yr * QK_GAIN;
        yi = yi * QK_GAIN;
        const float2 ph = phase[t];                            // src/qpsk.c:301-304
        const float sr = yr * ph.x - yi * ph.y;                // crealf(signal * phase)
        const float scale = r < 5 * QK_NPRE ? 8192.0f : 16384.0f;   // src/qpsk.c:313-319
        if (p < ns) o[p] = (int16_t)(int)(sr * scale);
    }
}

// AWGN of qpsk_synth.c: per output sample, counter-based Box-Muller in double
__global__ void __launch_bounds__(256) noise_kernel(uint64_t seed, uint32_t c0, int nch,
                                                    double sigma, int16_t* out, long ns) {
    const long total = (long)nch * ns;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
         i += (long)gridDim.x * blockDim.x) {
        const long c = i / ns, t = i - c * ns;
        uint64_t k = seed ^ 0x5851F42D4C957F2Dull;
        k ^= ((uint64_t)(c0 + (uint32_t)c) << 32) ^ (uint64_t)t;
        const uint64_t h1 = mix64(k + kGolden), h2 = mix64(k + 2 * kGolden);
        const double u1 = ((double)(h1 >> 11) + 1.0) * 0x1p-53;
        const double u2 = (double)(h2 >> 11) * 0x1p-53;
        const double z = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
        double v = rint((double)out[i] + sigma * z);
        if (v > 32767.0) v = 32767.0;
        if (v < -32768.0) v = -32768.0;
        out[i] = (int16_t)v;
    }
}

}  // namespace

// Carrier phase of TX samples [0, ntx): qpsk_tx_frame's fbb_tx_phase *=
// fbb_tx_rect per sample and /= cabsf() per call (src/qpsk.c:301-306), calls of
// 640 (preamble) and 155 (data) samples in packet order.  Same fp32 operations
// as qpsk_tx_frame_state() (qpsk_surface.c).
extern "C" void qpsk_tx_phase_table(float* out2, long ntx) {
    const float arg = (float)(2.0f * 3.14159265358979323846 * 1100.0f / 8000.0f);
    const float rr = cosf(arg), ri = sinf(arg);
    float pr = 1.0f, pi = 0.0f;
    long t = 0;
    for (int call = 0; t < ntx; call = (call + 1) % 9) {
        const int len = call == 0 ? 5 * QK_NPRE : 5 * QK_NDSYM;
        for (int j = 0; j < len && t < ntx; j++, t++) {
            const float a = pr * rr - pi * ri;
            const float b = pr * ri + pi * rr;
            pr = a;
            pi = b;
            out2[2 * t] = a;
            out2[2 * t + 1] = b;
        }
        const float mag = (float)sqrt((double)pr * pr + (double)pi * pi);
        pr = pr / mag;
        pi = pi / mag;
    }
}

extern "C" int qpsk_synth_device(uint64_t seed, uint32_t c0, int nch, double ebn0_db,
                                 int16_t* d_out, long nsamples, void* stream) {
    if (nch < 1 || nsamples < 0 || (nsamples > 0 && !d_out)) return -1;
    if (nsamples == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    // TX samples reaching [0, nsamples) of the channel with the smallest delay (0)
    const long np = nsamples / kPacket;
    long ntx = np * kTxPacket + (nsamples - np * kPacket < kTxPacket ? nsamples - np * kPacket
                                                                   : kTxPacket);
    ntx = (ntx + kBlk - 1) / kBlk * kBlk;
    float* h_ph = (float*)malloc(sizeof(float) * 2 * (size_t)ntx);
    if (!h_ph) return -2;
    qpsk_tx_phase_table(h_ph, ntx);
    float2* d_ph = nullptr;
    hipError_t e = hipMallocAsync((void**)&d_ph, sizeof(float2) * (size_t)ntx, s);
    if (e == hipSuccess)
        e = hipMemcpyAsync(d_ph, h_ph, sizeof(float2) * (size_t)ntx, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);   // h_ph is pageable and freed below
    free(h_ph);
    if (e == hipSuccess)
        e = hipMemsetAsync(d_out, 0, sizeof(int16_t) * (size_t)nch * (size_t)nsamples, s);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(tx_kernel, dim3((unsigned)(ntx / kBlk), (unsigned)((nch + 63) / 64)),
                           dim3(64), 0, s, seed, c0, nch, d_ph, ntx, d_out, nsamples);
        e = hipGetLastError();
    }
    if (e == hipSuccess && ebn0_db < 100.0) {
        const double sigma = sqrt(1.25 * kPData / pow(10.0, ebn0_db / 10.0));
        hipLaunchKernelGGL(noise_kernel, dim3(8192), dim3(256), 0, s, seed, c0, nch, sigma, d_out,
                           nsamples);
        e = hipGetLastError();
    }
    if (d_ph) {
        const hipError_t e2 = hipFreeAsync(d_ph, s);
        if (e == hipSuccess) e = e2;
    }
    return e == hipSuccess ? 0 : -1000 - (int)e;
}
