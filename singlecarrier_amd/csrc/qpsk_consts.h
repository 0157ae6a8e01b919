// qpsk_consts.h -- fixed modem constants shared by the HIP kernels and the host
// library.  Values are the reference's (file:line cited); nothing here is code.
#pragma once
#include <stdint.h>

#ifdef __cplusplus
#define QK_CONSTEXPR constexpr
#else
#define QK_CONSTEXPR static const
#endif

enum {
    QK_FRAME = 1880,    // FRAME_SIZE            headers/qpsk_internal.h:45
    QK_CYCLES = 5,      // CYCLES (FS/RS)        headers/qpsk_internal.h:30
    QK_NPRE = 128,      // PREAMBLE_LENGTH       headers/qpsk_internal.h:50
    QK_NDSYM = 31,      // DATA_SYMBOLS          headers/qpsk_internal.h:37
    QK_NBITS = 62,      // bits per valid frame  src/qpsk.c:206-215
    QK_NTAPS = 49,      // NTAPS                 headers/fir.h:16
    QK_NDEC = 188,      // decimated symbols carried to the next frame (App. A.4)
    QK_NHEAD = 102,     // observable undecimated FIR outputs dec[188..289] (App. A.6)
    QK_NDECOBS = 290,   // observable dec[0..289]
    QK_NWIN = 163,      // equalizer window dec[mi .. mi+162] (128 + 31 + 4)
    QK_NLAG = 128,      // preamble hunt lags    src/qpsk.c:176
    QK_MATCH_MIN = 98,  // valid iff matches > PREAMBLE_LENGTH - 30  src/qpsk.c:196
    QK_RT0 = 3,         // FINE_TIMING_OFFSET    headers/qpsk_internal.h:23
    QK_KS_PERIOD = 32767,   // 1 + x^14 + x^15 LFSR period
    QK_KS_FRAMES = 1057,    // period of the 62-bit-per-frame keystream window
    QK_GROUP = 64,      // channels per wave in the lane-per-channel stages
};

// PN preamble, src/constants.c:25-42 (preamblevalues)
QK_CONSTEXPR int8_t QK_PRE[QK_NPRE] = {
    -1, 1, 1, -1, -1, 1, 1, 1, -1, 1, -1, -1, 1, 1, -1, -1,
    1, 1, -1, 1, -1, -1, 1, -1, 1, -1, 1, -1, 1, -1, 1, 1,
    1, -1, 1, 1, 1, 1, -1, -1, 1, -1, -1, 1, 1, -1, 1, -1,
    1, 1, -1, 1, -1, -1, 1, -1, -1, -1, -1, 1, 1, -1, 1, -1,
    1, 1, 1, -1, -1, 1, 1, -1, 1, 1, -1, -1, 1, 1, -1, 1,
    1, -1, 1, 1, -1, -1, -1, 1, -1, 1, -1, 1, -1, -1, -1, 1,
    -1, -1, 1, -1, 1, 1, -1, -1, -1, -1, -1, 1, 1, 1, -1, 1,
    1, -1, 1, 1, -1, -1, 1, 1, -1, 1, -1, 1, -1, -1, -1, 1};

// RRC alpha=0.35 taps, src/constants.c:106-156 (alpha35_root; RX and TX use
// it because firwide == false, src/qpsk.c:60)
QK_CONSTEXPR float QK_RRC[QK_NTAPS] = {
    -0.00024537f, -0.00220636f, -0.00291493f, -0.00175708f, 0.00068764f,
    0.00282391f,  0.00297883f,  0.00059170f,  -0.00311265f, -0.00553670f,
    -0.00418297f, 0.00153693f,  0.00925400f,  0.01422443f,  0.01161151f,
    -0.00045943f, -0.01864749f, -0.03439334f, -0.03667604f, -0.01667595f,
    0.02761997f,  0.08908617f,  0.15279058f,  0.20079911f,  0.21864582f,
    0.20079911f,  0.15279058f,  0.08908617f,  0.02761997f,  -0.01667595f,
    -0.03667604f, -0.03439334f, -0.01864749f, -0.00045943f, 0.01161151f,
    0.01422443f,  0.00925400f,  0.00153693f,  -0.00418297f, -0.00553670f,
    -0.00311265f, 0.00059170f,  0.00297883f,  0.00282391f,  0.00068764f,
    -0.00175708f, -0.00291493f, -0.00220636f, -0.00024537f};

// GAIN headers/fir.h:17; E, q src/kalman.c:61-62
#define QK_GAIN 2.2f
#define QK_KAL_E 0.1f
#define QK_KAL_Q 0.08f
// fbb_rx_rect = cmplx(TAU*(-CENTER+FOFFSET)/FS) (src/qpsk.c:428) as fp32 bits
#define QK_RX_RECT_RE_BITS 0x3f26423au
#define QK_RX_RECT_IM_BITS 0xbf42a9f7u
#define QK_SEED 0x4A80  // headers/scramble.h:16
