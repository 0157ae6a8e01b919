/*
 * cpu_ref.c -- TEST INFRASTRUCTURE ONLY (oracle): clean-room C restatement of
 * the reference receive path, see cpu_ref.h.
 *
 * Arithmetic contract: IEEE fp32, round-to-nearest, every
 * product and sum rounded separately (built with -ffp-contract=off), sums in
 * the reference's index order starting from 0.0f, complex products written out
 * as (ac - bd, ad + bc) exactly as gcc expands them for finite operands.
 *
 * Minimal form, each step proved equal to the reference:
 *  - mixer: frame n uses (-1)^n * P[t] (A.2), P[t] = R^(t+1) by the fp32
 *    recurrence of src/qpsk.c:139; the per-frame renormalisation
 *    (src/qpsk.c:147) maps P[1879] to exactly -1+0i, so the phase alternates.
 *  - FIR (src/fir.c:22-44): call n filters the PREVIOUS frame's mixed samples
 *    (input_frame[0..1879] holds them, src/qpsk.c:143); only outputs
 *    [0..101] and {5i+rt} are observable (A.6) and only those are computed.
 *  - decimation with the gcc -O2 overflow semantics ("model A", A.4):
 *    dec[0..187] = D_{n-1}, dec[188..] = fir_out_n[0..], D_n[i] = fir_out_n[5i+rt].
 *    QC_MODE_DEC752 instead gives decimated_frame the 752 entries the loop at
 *    src/qpsk.c:157-162 writes: dec[0..375] = D_{n-1}[0..375] and nothing of
 *    frame n's own decimation is read before frame n+1, so the observable
 *    dec[0..289] = D_{n-1}[0..289], D_n[i] = fir_out_n[5i+rt] (5i+rt <= 1700 <
 *    1880: always a filtered sample).
 *  - correlator (src/qpsk.c:88-96): preamble symbols are p+pj with p = +-1, so
 *    each product is p*(dr-di, di+dr) exactly (A.3).
 *  - invalid frames skip data_eq (unobservable, A.6) but advance the keystream
 *    by 62 bits, i.e. frame n always uses keystream bits [62n, 62n+62).
 */
#include "cpu_ref.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* src/constants.c:25-42 (preamblevalues) */
static const int8_t k_pre[QC_PRE] = {
    -1, 1, 1, -1, -1, 1, 1, 1, -1, 1, -1, -1, 1, 1, -1, -1,
    1, 1, -1, 1, -1, -1, 1, -1, 1, -1, 1, -1, 1, -1, 1, 1,
    1, -1, 1, 1, 1, 1, -1, -1, 1, -1, -1, 1, 1, -1, 1, -1,
    1, 1, -1, 1, -1, -1, 1, -1, -1, -1, -1, 1, 1, -1, 1, -1,
    1, 1, 1, -1, -1, 1, 1, -1, 1, 1, -1, -1, 1, 1, -1, 1,
    1, -1, 1, 1, -1, -1, -1, 1, -1, 1, -1, 1, -1, -1, -1, 1,
    -1, -1, 1, -1, 1, 1, -1, -1, -1, -1, -1, 1, 1, 1, -1, 1,
    1, -1, 1, 1, -1, -1, 1, 1, -1, 1, -1, 1, -1, -1, -1, 1};

/* src/constants.c:106-156 (alpha35_root; rx uses it, firwide=false src/qpsk.c:60) */
static const float k_rrc[QC_NTAPS] = {
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

#define GAIN_F 2.2f    /* headers/fir.h:17 */
#define KAL_E 0.1f     /* src/kalman.c:61  */
#define KAL_Q 0.08f    /* src/kalman.c:62  */

static float bits2f(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}

/* ------------------------------------------------------------------ tables */

static float g_p[QC_FRAME][2];       /* mixer table P[t] * 2^-14 */
static uint8_t g_ks[32767 + 64];     /* RX keystream, one period + slack */
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

/* fbb_rx_rect = cmplx(TAU*(-CENTER+FOFFSET)/FS), src/qpsk.c:428; the bits of
 * glibc's cosf/sinf at that float argument (pinned by test_oracle.py). */
static void rx_rect(float r[2]) {
    r[0] = bits2f(0x3f26423au);
    r[1] = bits2f(0xbf42a9f7u);
}

void qc_mixer_table(float p[QC_FRAME][2]) {
    float r[2], ph[2] = {1.0f, 0.0f};  /* fbb_rx_phase = cmplx(0) src/qpsk.c:427 */
    rx_rect(r);
    for (int t = 0; t < QC_FRAME; t++) { /* fbb_rx_phase *= fbb_rx_rect :139 */
        float a = ph[0] * r[0] - ph[1] * r[1];
        float b = ph[0] * r[1] + ph[1] * r[0];
        ph[0] = a;
        ph[1] = b;
        p[t][0] = a;
        p[t][1] = b;
    }
}

void qc_keystream(uint8_t *ks, int n) {
    uint16_t m = 0x4A80; /* SEED headers/scramble.h:16 */
    for (int k = 0; k < n; k++) { /* scramble_internal, src/scramble.c:57-69 */
        uint16_t o = (uint16_t)(((m & 0x2) >> 1) ^ (m & 0x1));
        ks[k] = (uint8_t)o;
        m = (uint16_t)((m >> 1) | (o << 14));
    }
}

static void init_tables(void) {
    float p[QC_FRAME][2];
    qc_mixer_table(p);
    for (int t = 0; t < QC_FRAME; t++) {  /* (float)in/16384 folded into P: exact */
        g_p[t][0] = p[t][0] * 0x1p-14f;
        g_p[t][1] = p[t][1] * 0x1p-14f;
    }
    qc_keystream(g_ks, (int)sizeof g_ks);
}

/* ------------------------------------------------------------------ RX */

void qc_chan_init_mode(qc_chan_t *ch, int mode) {
    pthread_once(&g_once, init_tables);
    memset(ch, 0, sizeof(*ch));
    ch->rx_timing = 3;  /* FINE_TIMING_OFFSET, headers/qpsk_internal.h:23 */
    ch->mode = mode;
}

void qc_chan_init(qc_chan_t *ch) { qc_chan_init_mode(ch, QC_MODE_REF); }

/* mixed sample m_k[t] (src/qpsk.c:139-144) of frame k with parity sign */
static inline void mix(const int16_t *x, uint32_t k, int t, float out[2]) {
    float v = (float)x[t];
    float pr = g_p[t][0], pi = g_p[t][1];
    if (k & 1u) {
        pr = -pr;
        pi = -pi;
    }
    out[0] = pr * v;
    out[1] = pi * v;
}

/* one RRC output (src/fir.c:36-42): M points at the sample aligned with tap 0 */
static inline void fir_at(const float (*M)[2], float out[2]) {
    float yr = 0.0f, yi = 0.0f;
    for (int i = 0; i < QC_NTAPS; i++) {
        yr = yr + M[i][0] * k_rrc[i];
        yi = yi + M[i][1] * k_rrc[i];
    }
    out[0] = yr * GAIN_F;
    out[1] = yi * GAIN_F;
}

typedef struct {
    float eq[5][2];          /* eq_coeff   src/kalman.c:19 */
    float g[5][2];           /* kalman_gain src/kalman.c:20 */
    float u[5][5][2];        /* src/kalman.c:25 */
    float d[5];              /* src/kalman.c:29 */
    float y;                 /* kalman_y */
} kal_t;

static void kal_reset(kal_t *k) {  /* kalman_reset, src/kalman.c:42-55 */
    memset(k, 0, sizeof(*k));
    for (int i = 0; i < 5; i++) k->d[i] = 1.0f;
}

/* kalman_calculate, src/kalman.c:85-141, on x[0..4] = dec[index..index+4] */
static void kal_calc(kal_t *k, const float (*x)[2]) {
    float f[5][2], a[5];
    const float E = KAL_E, q = KAL_Q;
    f[0][0] = x[0][0];                         /* 6.2 f0 = conj(x0) */
    f[0][1] = -x[0][1];
    for (int j = 1; j < 5; j++) {
        /* u0j*conj(x0) + conj(xj): the double-precision conj() sum rounds to
         * the fp32 sum (2p+2 <= 53), so it is an fp32 add. */
        float ur = k->u[0][j][0], ui = k->u[0][j][1];
        float cr = x[0][0], ci = -x[0][1];
        float pr = ur * cr - ui * ci;
        float pi = ur * ci + ui * cr;
        f[j][0] = pr + x[j][0];
        f[j][1] = pi + (-x[j][1]);
        for (int i = 1; i < j; i++) {
            ur = k->u[i][j][0];
            ui = k->u[i][j][1];
            cr = x[i][0];
            ci = -x[i][1];
            pr = ur * cr - ui * ci;
            pi = ur * ci + ui * cr;
            f[j][0] = f[j][0] + pr;
            f[j][1] = f[j][1] + pi;
        }
    }
    for (int j = 0; j < 5; j++) {              /* 6.4 g = f*d */
        k->g[j][0] = f[j][0] * k->d[j];
        k->g[j][1] = f[j][1] * k->d[j];
    }
    /* 6.5/6.6 a_j = a_{j-1} + Re(g_j * conj(f_j)) */
    a[0] = E + (k->g[0][0] * f[0][0] - k->g[0][1] * (-f[0][1]));
    for (int j = 1; j < 5; j++)
        a[j] = a[j - 1] + (k->g[j][0] * f[j][0] - k->g[j][1] * (-f[j][1]));
    const float hq = 1.0f + q;                 /* 6.7 */
    const float ht = a[4] * q;
    float y = 1.0f / (a[0] + ht);              /* 6.19 */
    k->d[0] = k->d[0] * ((hq * (E + ht)) * y); /* 6.20 */
    for (int j = 1; j < 5; j++) {
        float B = a[j - 1] + ht;               /* 6.21 */
        float hr = (-f[j][0]) * y;             /* 6.11 h = -f*y */
        float hi = (-f[j][1]) * y;
        y = 1.0f / (a[j] + ht);                /* 6.22 */
        k->d[j] = k->d[j] * ((hq * B) * y);    /* 6.13 */
        for (int i = 0; i < j; i++) {
            float b1r = k->u[i][j][0], b1i = k->u[i][j][1];
            float gr = k->g[i][0], gi = -k->g[i][1];       /* conj(g_i) */
            k->u[i][j][0] = b1r + (hr * gr - hi * gi);     /* 6.15 */
            k->u[i][j][1] = b1i + (hr * gi + hi * gr);
            float jr = k->g[j][0], ji = k->g[j][1];
            float cr = b1r, ci = -b1i;                     /* conj(B1) */
            k->g[i][0] = k->g[i][0] + (jr * cr - ji * ci); /* 6.16 */
            k->g[i][1] = k->g[i][1] + (jr * ci + ji * cr);
        }
    }
    k->y = y;
}

/* update_eq, src/equalizer.c:25-40 */
static void update_eq(kal_t *k, const float (*x)[2], float er, float ei) {
    kal_calc(k, x);
    er = er * k->y;
    ei = ei * k->y;
    for (int i = 0; i < 5; i++) {
        float gr = k->g[i][0], gi = -k->g[i][1];
        k->eq[i][0] = k->eq[i][0] + (er * gr - ei * gi);
        k->eq[i][1] = k->eq[i][1] + (er * gi + ei * gr);
    }
}

/* train_eq, src/equalizer.c:45-58; returns crealf(error) = ref - Re(val) */
static float train_eq(kal_t *k, const float (*x)[2], float ref) {
    float vr = 0.0f, vi = 0.0f;
    for (int i = 0; i < 5; i++) {
        float a = x[i][0], b = x[i][1], c = k->eq[i][0], d = k->eq[i][1];
        vr = vr + (a * c - b * d);
        vi = vi + (a * d + b * c);
    }
    float er = ref - vr;   /* conjf(ref - val) = (ref - vr, vi) */
    float ei = vi;
    update_eq(k, x, er, ei);
    return er;
}

/* data_eq + qpsk_demod, src/equalizer.c:64-90, src/qpsk.c:268-271;
 * returns the dibit (I<<1)|Q before descrambling */
static int data_eq(kal_t *k, const float (*x)[2], float soft[2]) {
    float sr = 0.0f, si = 0.0f;
    for (int i = 0; i < 5; i++) {
        float a = x[i][0], b = x[i][1], c = k->eq[i][0], d = -k->eq[i][1];
        sr = sr + (a * c - b * d);
        si = si + (a * d + b * c);
    }
    int dI = sr < 0.0f;
    int dQ = si < 0.0f;
    float cr = dI ? -1.0f : 1.0f;
    float ci = dQ ? -1.0f : 1.0f;
    update_eq(k, x, (cr - sr) * 0.1f, (ci - si) * 0.1f);
    if (soft) {
        soft[0] = sr;
        soft[1] = si;
    }
    return (dI << 1) | dQ;
}

static int rx_frame(qc_chan_t *ch, const int16_t in[QC_FRAME], uint8_t bits[QC_BITS],
                    qc_trace_t *tr, float (*dec_out)[2]);

_Thread_local int qc_decision_step;
int qc_poison_unobservable;

int qc_rx_frame(qc_chan_t *ch, const int16_t in[QC_FRAME], uint8_t bits[QC_BITS],
                qc_trace_t *tr) {
    return rx_frame(ch, in, bits, tr, NULL);
}

long qc_rx_stages(const int16_t *in, int nframes, int mode, float *dec_out) {
    qc_chan_t *ch = (qc_chan_t *)malloc(sizeof(qc_chan_t));
    uint8_t bits[QC_BITS];
    long nvalid = 0;
    qc_chan_init_mode(ch, mode);
    for (int n = 0; n < nframes; n++)
        nvalid += rx_frame(ch, in + (size_t)n * QC_FRAME, bits, NULL,
                           (float (*)[2])(dec_out + (size_t)n * QC_DEC752 * 2));
    free(ch);
    return nvalid;
}

static int rx_frame(qc_chan_t *ch, const int16_t in[QC_FRAME], uint8_t bits[QC_BITS],
                    qc_trace_t *tr, float (*dec_out)[2]) {
    const uint32_t n = ch->frame;
    const int rt = ch->rx_timing;
    const int d752 = (ch->mode & QC_MODE_DEC752) != 0;
    /* M[-48..hi]: m_{n-2}[1832..1879] ++ m_{n-1}[0..hi] (zero before frame 0);
     * hi = 1190 (model A, D_n[0..187]) or 1700 (dec752, D_n[0..289]) */
    enum { LO = QC_NTAPS - 1, HIMAX = 5 * (QC_DEC752 - 1) + 255 };
    const int HI = d752 ? HIMAX : 5 * (QC_DEC - 1) + 255;
    float Mbuf[LO + HIMAX + 1][2];
    float (*M)[2] = Mbuf + LO;
    for (int t = -LO; t <= HI; t++) {
        if (t < 0) {
            if (n >= 2) mix(ch->hist[0], n - 2, QC_FRAME + t, M[t]);
            else M[t][0] = M[t][1] = 0.0f;
        } else {
            if (n >= 1) mix(ch->hist[1], n - 1, t, M[t]);
            else M[t][0] = M[t][1] = 0.0f;
        }
    }
    /* dec[0..289] */
    float dec[QC_DEC752][2];
    if (d752) {   /* dec = D_{n-1}[0..289] */
        memcpy(dec, ch->dprev, sizeof ch->dprev);
        for (int i = 0; i < QC_DEC752; i++) fir_at(M + 5 * i + rt - LO, ch->dprev[i]);
    } else {      /* model A: dec = D_{n-1}[0..187] ++ fir_out_n[0..101] */
        memcpy(dec, ch->dprev, sizeof(float[QC_DEC][2]));
        for (int j = 0; j < 102; j++) fir_at(M + j - LO, dec[QC_DEC + j]);
        for (int i = 0; i < QC_DEC; i++) fir_at(M + 5 * i + rt - LO, ch->dprev[i]);
    }

    if (dec_out) memcpy(dec_out, dec, sizeof dec);   /* decimated_frame[0..289] */

    /* preamble hunt, src/qpsk.c:172-183 */
    int mi = 0;
    if (ch->mode & QC_MODE_FFT_HUNT) {
        mi = qc_fft_hunt(&dec[0][0]);
    } else {
    float T[255], U[255];
    for (int j = 0; j < 255; j++) {
        T[j] = dec[j][0] - dec[j][1];
        U[j] = dec[j][1] + dec[j][0];
    }
    float max_value = 0.0f;
    for (int L = 0; L < QC_PRE; L++) {
        float sr = 0.0f, si = 0.0f;
        for (int i = 0; i < QC_PRE; i++) {
            if (k_pre[i] > 0) {
                sr = sr + T[L + i];
                si = si + U[L + i];
            } else {
                sr = sr - T[L + i];
                si = si - U[L + i];
            }
        }
        float c = sr * sr + si * si;  /* cnormf, src/qpsk.c:75-80 */
        if (c > max_value) {
            max_value = c;
            mi = L;
        }
    }
    }

    if (qc_poison_unobservable) {   /* test switch, cpu_ref.h */
        const float nan = bits2f(0x7fc00000u);
        for (int j = 0; j < QC_DEC752; j++)
            if (j < mi || j > mi + QC_PRE + QC_DSYM + 3) dec[j][0] = dec[j][1] = nan;
    }
    /* equalize(), src/qpsk.c:111-123 */
    kal_t k;
    kal_reset(&k);
    int matches = 0;
    int dstep = QC_PRE;
    for (int i = 0; i < QC_PRE; i++) {
        float ref = (float)k_pre[i];
        if (train_eq(&k, dec + mi + i, ref) * ref > 0.0f) matches++;
        /* diagnostics: first step at which the decision below is certain */
        if (dstep == QC_PRE && (matches > QC_PRE - 30 || i + 1 - matches >= 30)) dstep = i + 1;
    }
    qc_decision_step = dstep;
    const int valid = matches > QC_PRE - 30;  /* src/qpsk.c:196 */
    memset(bits, 0, QC_BITS);
    if (tr) memset(tr, 0, sizeof(*tr));
    if (valid) {
        const uint8_t *ks = g_ks + (size_t)(((uint64_t)n * 62u) % 32767u);
        for (int s = 0; s < QC_DSYM; s++) {
            float soft[2];
            int dib = data_eq(&k, dec + mi + QC_PRE + s, soft);
            bits[2 * s] = (uint8_t)((dib & 1) ^ ks[2 * s]);            /* Q */
            bits[2 * s + 1] = (uint8_t)(((dib >> 1) & 1) ^ ks[2 * s + 1]); /* I */
            if (tr) {
                tr->soft[s][0] = soft[0];
                tr->soft[s][1] = soft[1];
            }
        }
        ch->rx_timing = mi + QC_PRE;  /* src/qpsk.c:219 */
    }
    if (tr) {
        tr->max_index = mi;
        tr->matches = matches;
        tr->valid = valid;
        tr->rx_timing = ch->rx_timing;
    }
    memcpy(ch->hist[0], ch->hist[1], sizeof ch->hist[0]);
    memcpy(ch->hist[1], in, sizeof ch->hist[1]);
    ch->frame = n + 1;
    return valid;
}

typedef struct {
    const int16_t *in;
    int nch, nframes, c0, c1, mode;
    uint8_t *bits, *valid;
    qc_trace_t *tr;
    long nvalid;
} batch_job_t;

static void *batch_worker(void *arg) {
    batch_job_t *j = (batch_job_t *)arg;
    qc_chan_t *ch = (qc_chan_t *)malloc(sizeof(qc_chan_t));
    j->nvalid = 0;
    for (int c = j->c0; c < j->c1; c++) {
        qc_chan_init_mode(ch, j->mode);
        for (int n = 0; n < j->nframes; n++) {
            size_t cf = (size_t)c * j->nframes + n;
            int v = qc_rx_frame(ch, j->in + cf * QC_FRAME, j->bits + cf * QC_BITS,
                                j->tr ? j->tr + cf : NULL);
            if (j->valid) j->valid[cf] = (uint8_t)v;
            j->nvalid += v;
        }
    }
    free(ch);
    return NULL;
}

long qc_rx_batch(const int16_t *in, int nch, int nframes, uint8_t *bits,
                 uint8_t *valid, qc_trace_t *tr, int nthreads) {
    return qc_rx_batch_mode(in, nch, nframes, bits, valid, tr, nthreads, QC_MODE_REF);
}

long qc_rx_batch_mode(const int16_t *in, int nch, int nframes, uint8_t *bits,
                      uint8_t *valid, qc_trace_t *tr, int nthreads, int mode) {
    pthread_once(&g_once, init_tables);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > nch) nthreads = nch > 0 ? nch : 1;
    batch_job_t *jobs = (batch_job_t *)calloc((size_t)nthreads, sizeof(batch_job_t));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (batch_job_t){in, nch, nframes, (int)((long)nch * t / nthreads),
                                (int)((long)nch * (t + 1) / nthreads), mode, bits, valid, tr, 0};
        if (nthreads > 1) pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
        else batch_worker(&jobs[t]);
    }
    long total = 0;
    for (int t = 0; t < nthreads; t++) {
        if (nthreads > 1) pthread_join(th[t], NULL);
        total += jobs[t].nvalid;
    }
    free(jobs);
    free(th);
    return total;
}

/* ------------------------------------------------------------------ FFT */
/* Restatement of the reference's kiss_fft (src/fft.c, Borgerding's kiss_fft
 * as modified by the reference author).  Complex values are (re, im) float
 * pairs; every operation below is the one gcc -O2 emits for the reference's
 * C99 complex expressions with finite operands: a complex product is
 * (ac - bd, ad + bc), complex * real is componentwise, and `x + y * I` is
 * (x + y * 0.0f, y), `x - y * I` is (x - y * 0.0f, -y) (the y * 0.0f only
 * decides the sign of a zero real part; checked on gcc 11.4's output).  Pinned bit for bit against the compiled reference
 * (oracle/_ref/libkissfft_ref.so) by tests/test_oracle.py. */

typedef struct { float r, i; } qc_cf;

static inline qc_cf cf_mul(qc_cf a, qc_cf b) {
    qc_cf o = {a.r * b.r - a.i * b.i, a.r * b.i + a.i * b.r};
    return o;
}
static inline qc_cf cf_add(qc_cf a, qc_cf b) { qc_cf o = {a.r + b.r, a.i + b.i}; return o; }
static inline qc_cf cf_sub(qc_cf a, qc_cf b) { qc_cf o = {a.r - b.r, a.i - b.i}; return o; }
static inline qc_cf cf_mk(float x, float y) { qc_cf o = {x + y * 0.0f, y}; return o; }     /* x + y*I */
static inline qc_cf cf_mkm(float x, float y) { qc_cf o = {x - y * 0.0f, -y}; return o; }   /* x - y*I */

typedef struct {
    int nfft, inverse;
    int factors[64];
    qc_cf *tw;
} qc_fft_t;

void qc_fft_twiddles(int nfft, int inverse, float *tw) {   /* src/fft.c:67-74 */
    /* TAU (headers/qpsk_internal.h:60) is 2.0f * M_PI, and M_PI is math.h's
     * double constant (the header's float fallback is #ifndef'd away), so the
     * phase is evaluated in double and rounded once to the float variable. */
    const double tau = 2.0f * 3.14159265358979323846;
    for (int i = 0; i < nfft; i++) {
        float phase = (float)(-tau * (float)i / (float)nfft);
        if (inverse) phase *= -1.0f;
        tw[2 * i] = cosf(phase);                             /* cmplx() :67 */
        tw[2 * i + 1] = sinf(phase);
    }
}

static void qc_kf_factor(int n, int *fac) {                  /* src/fft.c:433-459 */
    int p = 4;
    const float floor_sqrt = floorf(sqrtf((float)n));
    do {
        while (n % p) {
            p = p == 4 ? 2 : p == 2 ? 3 : p + 2;
            if (p > floor_sqrt) p = n;
        }
        n /= p;
        *fac++ = p;
        *fac++ = n;
    } while (n > 1);
}

static void qc_bfly2(qc_cf *F, size_t fs, const qc_fft_t *st, int m) {   /* :190-211 */
    const qc_cf *tw = st->tw;
    for (int k = 0; k < m; k++, tw += fs) {
        const qc_cf t = cf_mul(F[m + k], *tw);
        F[m + k] = cf_sub(F[k], t);
        F[k] = cf_add(F[k], t);
    }
}

static void qc_bfly4(qc_cf *F, size_t fs, const qc_fft_t *st, size_t m) {   /* :213-255 */
    for (size_t k = 0; k < m; k++) {
        qc_cf *f = F + k;
        const qc_cf s0 = cf_mul(f[m], st->tw[k * fs]);
        const qc_cf s1 = cf_mul(f[2 * m], st->tw[2 * k * fs]);
        const qc_cf s2 = cf_mul(f[3 * m], st->tw[3 * k * fs]);
        const qc_cf s5 = cf_sub(f[0], s1);
        f[0] = cf_add(f[0], s1);
        const qc_cf s3 = cf_add(s0, s2);
        const qc_cf s4 = cf_sub(s0, s2);
        f[2 * m] = cf_sub(f[0], s3);
        f[0] = cf_add(f[0], s3);
        if (st->inverse) {
            f[m] = cf_mk(s5.r - s4.i, s5.i + s4.r);
            f[3 * m] = cf_mk(s5.r + s4.i, s5.i - s4.r);
        } else {
            f[m] = cf_mk(s5.r + s4.i, s5.i - s4.r);
            f[3 * m] = cf_mk(s5.r - s4.i, s5.i + s4.r);
        }
    }
}

static void qc_bfly3(qc_cf *F, size_t fs, const qc_fft_t *st, size_t m) {   /* :257-290 */
    const qc_cf epi3 = st->tw[fs * m];
    for (size_t k = 0; k < m; k++) {
        qc_cf *f = F + k;
        const qc_cf s1 = cf_mul(f[m], st->tw[k * fs]);
        const qc_cf s2 = cf_mul(f[2 * m], st->tw[2 * k * fs]);
        const qc_cf s3 = cf_add(s1, s2);
        qc_cf s0 = cf_sub(s1, s2);
        f[m] = cf_mk(f[0].r - s3.r * .5f, f[0].i - s3.i * .5f);
        s0 = (qc_cf){s0.r * epi3.i, s0.i * epi3.i};
        f[0] = cf_add(f[0], s3);
        f[2 * m] = cf_mk(f[m].r + s0.i, f[m].i - s0.r);
        f[m] = cf_mk(f[m].r - s0.i, f[m].i + s0.r);
    }
}

static void qc_bfly5(qc_cf *F, size_t fs, const qc_fft_t *st, int m) {   /* :292-344 */
    const qc_cf ya = st->tw[fs * m], yb = st->tw[fs * m * 2];
    for (int u = 0; u < m; u++) {
        qc_cf *f0 = F + u, *f1 = f0 + m, *f2 = f0 + 2 * m, *f3 = f0 + 3 * m, *f4 = f0 + 4 * m;
        const qc_cf s0 = *f0;
        const qc_cf s1 = cf_mul(*f1, st->tw[fs * u]);
        const qc_cf s2 = cf_mul(*f2, st->tw[fs * 2 * u]);
        const qc_cf s3 = cf_mul(*f3, st->tw[fs * 3 * u]);
        const qc_cf s4 = cf_mul(*f4, st->tw[fs * 4 * u]);
        const qc_cf s7 = cf_add(s1, s4), s10 = cf_sub(s1, s4);
        const qc_cf s8 = cf_add(s2, s3), s9 = cf_sub(s2, s3);
        *f0 = cf_add(*f0, cf_mk(s7.r + s8.r, s7.i + s8.i));
        const qc_cf s5 = cf_mk((s0.r + s7.r * ya.r) + s8.r * yb.r, (s0.i + s7.i * ya.r) + s8.i * yb.r);
        const qc_cf s6 = cf_mkm(-(s10.i * ya.i + s9.i * yb.i), s10.r * ya.i - s9.r * yb.i);
        *f1 = cf_sub(s5, s6);
        *f4 = cf_add(s5, s6);
        const qc_cf s11 = cf_mk((s0.r + s7.r * yb.r) + s8.r * ya.r, (s0.i + s7.i * yb.r) + s8.i * ya.r);
        /* as written at :327 (upstream kiss_fft has -a + b here, not -(a + b)) */
        const qc_cf s12 = cf_mk(-(s10.i * yb.i + s9.i * ya.i), s10.r * yb.i - s9.r * ya.i);
        *f2 = cf_add(s11, s12);
        *f3 = cf_sub(s11, s12);
    }
}

static void qc_bfly_generic(qc_cf *F, size_t fs, const qc_fft_t *st, int m, int p) {   /* :346-386 */
    qc_cf *scratch = (qc_cf *)malloc(sizeof(qc_cf) * (size_t)p);
    for (int u = 0; u < m; u++) {
        int k = u;
        for (int q1 = 0; q1 < p; q1++, k += m) scratch[q1] = F[k];
        k = u;
        for (int q1 = 0; q1 < p; q1++, k += m) {
            int twidx = 0;
            F[k] = scratch[0];
            for (int q = 1; q < p; q++) {
                twidx += (int)fs * k;
                if (twidx >= st->nfft) twidx -= st->nfft;
                F[k] = cf_add(F[k], cf_mul(scratch[q], st->tw[twidx]));
            }
        }
    }
    free(scratch);
}

static void qc_kf_work(qc_cf *Fout, const qc_cf *f, size_t fs, const int *fac,
                       const qc_fft_t *st) {                 /* :388-431 */
    const int p = fac[0], m = fac[1];
    if (m == 1) {
        for (int j = 0; j < p; j++) Fout[j] = f[(size_t)j * fs];
    } else {
        for (int j = 0; j < p; j++) qc_kf_work(Fout + (size_t)j * m, f + (size_t)j * fs, fs * p, fac + 2, st);
    }
    switch (p) {
        case 2: qc_bfly2(Fout, fs, st, m); break;
        case 3: qc_bfly3(Fout, fs, st, (size_t)m); break;
        case 4: qc_bfly4(Fout, fs, st, (size_t)m); break;
        case 5: qc_bfly5(Fout, fs, st, m); break;
        default: qc_bfly_generic(Fout, fs, st, m, p);
    }
}

int qc_fft(int nfft, int inverse, const float *in, float *out) {
    if (nfft < 1) return -1;
    qc_fft_t st;
    st.nfft = nfft;
    st.inverse = inverse;
    st.tw = (qc_cf *)malloc(sizeof(qc_cf) * (size_t)nfft);
    qc_fft_twiddles(nfft, inverse, (float *)st.tw);
    qc_kf_factor(nfft, st.factors);
    qc_cf *tmp = (qc_cf *)malloc(sizeof(qc_cf) * (size_t)nfft);   /* fft_stride(): in may == out */
    qc_kf_work(tmp, (const qc_cf *)in, 1, st.factors, &st);
    memcpy(out, tmp, sizeof(qc_cf) * (size_t)nfft);
    free(tmp);
    free(st.tw);
    return 0;
}

static float g_fftq[256][2];
static pthread_once_t g_fftq_once = PTHREAD_ONCE_INIT;

static void init_fftq(void) {
    float c[256][2];
    memset(c, 0, sizeof c);
    for (int i = 0; i < QC_PRE; i++) {   /* conj(preambletable[i]) = (p, -p) */
        c[i][0] = (float)k_pre[i];
        c[i][1] = -(float)k_pre[i];
    }
    float C[256][2];
    qc_fft(256, 0, &c[0][0], &C[0][0]);
    for (int k = 0; k < 256; k++) {
        g_fftq[k][0] = C[k][0];
        g_fftq[k][1] = -C[k][1];
    }
}

void qc_fft_hunt_spectrum(float *q) {
    pthread_once(&g_fftq_once, init_fftq);
    memcpy(q, g_fftq, sizeof g_fftq);
}

int qc_fft_hunt(const float *dec) {
    pthread_once(&g_fftq_once, init_fftq);
    float X[256][2], Y[256][2], S[256][2];
    qc_fft(256, 0, dec, &X[0][0]);
    for (int k = 0; k < 256; k++) {   /* complex product, (ac - bd, ad + bc) */
        const qc_cf p = cf_mul((qc_cf){X[k][0], X[k][1]}, (qc_cf){g_fftq[k][0], g_fftq[k][1]});
        Y[k][0] = p.r;
        Y[k][1] = p.i;
    }
    qc_fft(256, 1, &Y[0][0], &S[0][0]);
    float max_value = 0.0f;
    int mi = 0;
    for (int L = 0; L < QC_PRE; L++) {   /* src/qpsk.c:172-183 */
        const float c = S[L][0] * S[L][0] + S[L][1] * S[L][1];   /* cnormf :75-80 */
        if (c > max_value) {
            max_value = c;
            mi = L;
        }
    }
    return mi;
}

/* ------------------------------------------------------------------ TX */

void qc_tx_init(qc_tx_t *tx) {
    pthread_once(&g_once, init_tables);
    memset(tx, 0, sizeof(*tx));
    tx->phase[0] = 1.0f;  /* fbb_tx_phase = cmplx(0.0f), src/qpsk.c:375 */
}

/* fbb_tx_rect = cmplx(TAU*CENTER/FS), src/qpsk.c:376 (argument rounded to float) */
static void tx_rect(float r[2]) {
    const float arg = (float)(2.0f * 3.14159265358979323846 * 1100.0f / 8000.0f);
    r[0] = cosf(arg);
    r[1] = sinf(arg);
}

int qc_tx_frame(qc_tx_t *tx, int16_t *out, const float (*sym)[2], int len,
                int preamble) {
    const int n = len * 5;
    float (*sig)[2] = (float (*)[2])calloc((size_t)n, sizeof(float[2]));
    for (int i = 0; i < len; i++) {   /* zero-stuff x5, src/qpsk.c:285-291 */
        sig[5 * i][0] = sym[i][0];
        sig[5 * i][1] = sym[i][1];
    }
    for (int j = 0; j < n; j++) {      /* fir(tx_filter, ...), src/fir.c:29-43 */
        memmove(tx->fir_mem[0], tx->fir_mem[1], sizeof(float[2]) * (QC_NTAPS - 1));
        tx->fir_mem[QC_NTAPS - 1][0] = sig[j][0];
        tx->fir_mem[QC_NTAPS - 1][1] = sig[j][1];
        fir_at((const float (*)[2])tx->fir_mem, sig[j]);
    }
    float r[2];
    tx_rect(r);
    for (int i = 0; i < n; i++) {      /* mix up, src/qpsk.c:301-304 */
        float a = tx->phase[0] * r[0] - tx->phase[1] * r[1];
        float b = tx->phase[0] * r[1] + tx->phase[1] * r[0];
        tx->phase[0] = a;
        tx->phase[1] = b;
        float sr = sig[i][0] * a - sig[i][1] * b;
        float si = sig[i][0] * b + sig[i][1] * a;
        sig[i][0] = sr;
        sig[i][1] = si;
    }
    /* fbb_tx_phase /= cabsf(...), src/qpsk.c:306; glibc hypotf is the
     * correctly rounded double-evaluated norm */
    float mag = (float)sqrt((double)tx->phase[0] * tx->phase[0] +
                            (double)tx->phase[1] * tx->phase[1]);
    tx->phase[0] = tx->phase[0] / mag;
    tx->phase[1] = tx->phase[1] / mag;
    for (int i = 0; i < n; i++)        /* src/qpsk.c:313-319 */
        out[i] = (int16_t)(sig[i][0] * (preamble ? 8192.0f : 16384.0f));
    free(sig);
    return n;
}

static uint64_t sm64(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* mean square of noiseless data samples (data RMS ~7,200) */
#define QC_PDATA 5.19e7

void qc_synth_channel(uint64_t seed, uint32_t c, double ebn0_db, int16_t *out,
                      long nsamples, uint8_t *unused) {
    (void)unused;
    uint64_t s = seed ^ ((uint64_t)c * 0x9E3779B97F4A7C15ull);
    qc_tx_t tx;
    qc_tx_init(&tx);
    long pos = (long)(sm64(&s) % QC_PACKET);  /* leading delay d_c */
    if (pos > nsamples) pos = nsamples;
    memset(out, 0, sizeof(int16_t) * (size_t)pos);
    float pre[QC_PRE][2], dsym[QC_DSYM][2];
    for (int i = 0; i < QC_PRE; i++) pre[i][0] = pre[i][1] = (float)k_pre[i];
    int16_t buf[640];
    while (pos < nsamples) {
        int m = qc_tx_frame(&tx, buf, (const float (*)[2])pre, QC_PRE, 1);
        for (int i = 0; i < m && pos < nsamples; i++) out[pos++] = buf[i];
        for (int f = 0; f < 8; f++) {
            for (int i = 0; i < QC_DSYM; i++) {  /* qpsk_mod, src/qpsk.c:251-256 */
                uint64_t dib = sm64(&s) & 3u;
                dsym[i][0] = (dib >> 1) ? -1.0f : 1.0f;  /* I odd bit  */
                dsym[i][1] = (dib & 1) ? -1.0f : 1.0f;   /* Q even bit */
            }
            m = qc_tx_frame(&tx, buf, (const float (*)[2])dsym, QC_DSYM, 0);
            for (int i = 0; i < m && pos < nsamples; i++) out[pos++] = buf[i];
        }
        for (int i = 0; i < 903 && pos < nsamples; i++) out[pos++] = 0;
    }
    if (ebn0_db >= 100.0) return;
    /* AWGN: sigma^2 = P_data * Fs / (2 * Rb * 10^(EbN0/10)), Rb = 3200 b/s */
    const double sigma = sqrt(1.25 * QC_PDATA / pow(10.0, ebn0_db / 10.0));
    for (long t = 0; t < nsamples; t++) {
        uint64_t k = seed ^ 0x5851F42D4C957F2Dull;
        k ^= ((uint64_t)c << 32) ^ (uint64_t)t;
        uint64_t h1 = sm64(&k), h2 = sm64(&k);
        double u1 = ((double)(h1 >> 11) + 1.0) * 0x1p-53;
        double u2 = (double)(h2 >> 11) * 0x1p-53;
        double z = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
        double v = nearbyint((double)out[t] + sigma * z);
        if (v > 32767.0) v = 32767.0;
        if (v < -32768.0) v = -32768.0;
        out[t] = (int16_t)v;
    }
}

typedef struct {
    uint64_t seed;
    uint32_t c0;
    int lo, hi;
    double ebn0;
    int16_t *out;
    long ns;
} synth_job_t;

static void *synth_worker(void *arg) {
    synth_job_t *j = (synth_job_t *)arg;
    for (int c = j->lo; c < j->hi; c++)
        qc_synth_channel(j->seed, j->c0 + (uint32_t)c, j->ebn0, j->out + (size_t)c * j->ns,
                         j->ns, NULL);
    return NULL;
}

void qc_synth_batch(uint64_t seed, uint32_t c0, int nch, double ebn0_db,
                    int16_t *out, long nsamples, int nthreads) {
    pthread_once(&g_once, init_tables);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > nch) nthreads = nch > 0 ? nch : 1;
    synth_job_t *jobs = (synth_job_t *)calloc((size_t)nthreads, sizeof(synth_job_t));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (synth_job_t){seed, c0, (int)((long)nch * t / nthreads),
                                (int)((long)nch * (t + 1) / nthreads), ebn0_db, out, nsamples};
        pthread_create(&th[t], NULL, synth_worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(jobs);
    free(th);
}
