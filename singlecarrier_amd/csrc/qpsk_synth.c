/*
 * qpsk_synth.c -- multi-channel synthetic input generator (include/qpsk_synth.h).
 * Host C over the reentrant transmitter qpsk_tx_frame_state(); pthreads over
 * channels.
 */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "qpsk_consts.h"
#include "qpsk_synth.h"

#define PACKET 2783          /* 640 + 8*155 + 903 samples */
#define P_DATA 5.19e7        /* mean square of noiseless data samples */

static uint64_t sm64(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static void synth_channel(uint64_t seed, uint32_t c, double ebn0_db, int16_t *out, long ns) {
    uint64_t s = seed ^ ((uint64_t)c * 0x9E3779B97F4A7C15ull);
    qpsk_tx_state tx;
    qpsk_tx_state_init(&tx);
    long pos = (long)(sm64(&s) % PACKET);
    if (pos > ns) pos = ns;
    memset(out, 0, sizeof(int16_t) * (size_t)pos);
    float pre[QK_NPRE * 2], dsym[QK_NDSYM * 2];
    for (int i = 0; i < QK_NPRE; i++) pre[2 * i] = pre[2 * i + 1] = (float)QK_PRE[i];
    int16_t buf[QK_NPRE * 5];
    while (pos < ns) {
        int m = qpsk_tx_frame_state(&tx, buf, pre, QK_NPRE, true);
        for (int i = 0; i < m && pos < ns; i++) out[pos++] = buf[i];
        for (int f = 0; f < 8; f++) {
            for (int i = 0; i < QK_NDSYM; i++) {   /* qpsk_mod, src/qpsk.c:251-256 */
                uint64_t dib = sm64(&s) & 3u;
                dsym[2 * i] = (dib >> 1) ? -1.0f : 1.0f;
                dsym[2 * i + 1] = (dib & 1) ? -1.0f : 1.0f;
            }
            m = qpsk_tx_frame_state(&tx, buf, dsym, QK_NDSYM, false);
            for (int i = 0; i < m && pos < ns; i++) out[pos++] = buf[i];
        }
        for (int i = 0; i < 903 && pos < ns; i++) out[pos++] = 0;
    }
    if (ebn0_db >= 100.0) return;
    const double sigma = sqrt(1.25 * P_DATA / pow(10.0, ebn0_db / 10.0));
    for (long t = 0; t < ns; t++) {
        uint64_t k = seed ^ 0x5851F42D4C957F2Dull;
        k ^= ((uint64_t)c << 32) ^ (uint64_t)t;
        const uint64_t h1 = sm64(&k), h2 = sm64(&k);
        const double u1 = ((double)(h1 >> 11) + 1.0) * 0x1p-53;
        const double u2 = (double)(h2 >> 11) * 0x1p-53;
        const double z = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
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
} job_t;

static void *worker(void *arg) {
    job_t *j = (job_t *)arg;
    for (int c = j->lo; c < j->hi; c++)
        synth_channel(j->seed, j->c0 + (uint32_t)c, j->ebn0, j->out + (size_t)c * j->ns, j->ns);
    return NULL;
}

void qpsk_synth_batch(uint64_t seed, uint32_t c0, int nch, double ebn0_db, int16_t *out,
                      long nsamples, int nthreads) {
    if (nch < 1) return;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > nch) nthreads = nch;
    job_t *jobs = (job_t *)calloc((size_t)nthreads, sizeof(job_t));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (job_t){seed, c0, (int)((long)nch * t / nthreads),
                          (int)((long)nch * (t + 1) / nthreads), ebn0_db, out, nsamples};
        pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(jobs);
    free(th);
}
