/*
 * threads_caller.c -- the batched C-ABI (include/qpsk_batch.h) from several
 * host threads at once, as a C integrator would drive it: one context per
 * thread, created concurrently behind a barrier, each demodulating its own
 * channel batch in three calls.  Test-only (tests/test_gpu_threads.py).
 *
 * The reference receiver is not reentrant (its state is file-scope statics,
 * /root/reference/src/qpsk.c:34-53); SURVEY.md 8b asks the replacement to be
 * thread-safe across contexts.
 *
 *   threads_caller DEVICES  IN_0 NCH_0 NF_0 MODE_0 OUT_0  [IN_1 ...]
 * IN_t: int16 [nch][nf][1880]; OUT_t: bits uint8 [nch][nf][62] then valid
 * uint8 [nch][nf].  Thread t uses device t % DEVICES.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "qpsk_batch.h"

#define FRAME 1880
#define NBITS 62

typedef struct {
    const char *in, *out;
    int nch, nf, mode, device;
    int rc;
} job;

static pthread_barrier_t start;

static void *run(void *arg) {
    job *j = (job *)arg;
    const size_t cf = (size_t)j->nch * (size_t)j->nf;
    int16_t *x = malloc(cf * FRAME * sizeof(int16_t));
    uint8_t *bits = calloc(cf * NBITS, 1), *valid = calloc(cf, 1);
    int16_t *part = malloc(cf * FRAME * sizeof(int16_t));
    uint8_t *pb = malloc(cf * NBITS), *pv = malloc(cf);
    j->rc = -100;
    FILE *f = fopen(j->in, "rb");
    const int ok = x && bits && valid && part && pb && pv && f && fread(x, 2, cf * FRAME, f) == cf * FRAME;
    if (f) fclose(f);
    pthread_barrier_wait(&start);   /* every thread creates its context at once */
    int err = 0;
    qpsk_ctx *c = ok ? qpsk_rx_create_mode(j->device, j->nch, j->mode, &err) : NULL;
    if (!c) {
        if (ok) j->rc = err;
        free(x); free(bits); free(valid); free(part); free(pb); free(pv);
        return NULL;
    }
    /* frames [0, a), [a, b), [b, nf): per-channel state carries across calls */
    const int cut[4] = {0, j->nf / 3, (2 * j->nf) / 3, j->nf};
    int rc = 0;
    for (int k = 0; k < 3 && rc == 0; k++) {
        const int a = cut[k], n = cut[k + 1] - cut[k];
        if (n == 0) continue;
        for (int ch = 0; ch < j->nch; ch++)   /* [nch][n][1880] slice of the stream */
            for (int i = 0; i < n; i++)
                for (int t = 0; t < FRAME; t++)
                    part[((size_t)ch * n + i) * FRAME + t] = x[((size_t)ch * j->nf + a + i) * FRAME + t];
        rc = qpsk_rx_batch(c, part, n, pb, pv, NULL, NULL);
        for (int ch = 0; ch < j->nch; ch++)
            for (int i = 0; i < n; i++) {
                const size_t d = (size_t)ch * j->nf + a + i, s = (size_t)ch * n + i;
                valid[d] = pv[s];
                for (int b = 0; b < NBITS; b++) bits[d * NBITS + b] = pb[s * NBITS + b];
            }
    }
    if (rc == 0 && qpsk_rx_frames(c) != (uint64_t)j->nf) rc = -101;
    qpsk_rx_destroy(c);
    if (rc == 0) {
        FILE *o = fopen(j->out, "wb");
        if (!o || fwrite(bits, 1, cf * NBITS, o) != cf * NBITS || fwrite(valid, 1, cf, o) != cf) rc = -102;
        if (o) fclose(o);
    }
    j->rc = rc;
    free(x); free(bits); free(valid); free(part); free(pb); free(pv);
    return NULL;
}

int main(int argc, char **argv) {
    if (argc < 7 || (argc - 2) % 5 != 0) {
        fprintf(stderr, "usage: %s DEVICES IN NCH NF MODE OUT [...]\n", argv[0]);
        return 2;
    }
    const int ndev = atoi(argv[1]), nt = (argc - 2) / 5;
    job *jobs = calloc((size_t)nt, sizeof(job));
    pthread_t *th = calloc((size_t)nt, sizeof(pthread_t));
    pthread_barrier_init(&start, NULL, (unsigned)nt);
    for (int t = 0; t < nt; t++) {
        char **a = argv + 2 + 5 * t;
        jobs[t] = (job){a[0], a[4], atoi(a[1]), atoi(a[2]), atoi(a[3]), t % (ndev > 0 ? ndev : 1), 0};
        pthread_create(&th[t], NULL, run, &jobs[t]);
    }
    int bad = 0;
    for (int t = 0; t < nt; t++) {
        pthread_join(th[t], NULL);
        if (jobs[t].rc != 0) {
            fprintf(stderr, "thread %d: %d %s\n", t, jobs[t].rc, qpsk_strerror(jobs[t].rc));
            bad = 1;
        }
    }
    pthread_barrier_destroy(&start);
    free(jobs);
    free(th);
    return bad;
}
