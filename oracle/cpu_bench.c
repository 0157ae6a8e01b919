/*
 * cpu_bench.c -- TEST INFRASTRUCTURE ONLY (oracle).
 * Times the clean-room restatement on synthetic channels:
 *   qpsk_cpu_bench NCH NFRAMES THREADS [SEED] [EBN0_DB]
 * prints one JSON line {msamples_per_s, seconds, valid, ...}.
 */
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "cpu_ref.h"

static double now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

int main(int argc, char **argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s NCH NFRAMES THREADS [SEED] [EBN0_DB]\n", argv[0]);
        return 2;
    }
    int nch = atoi(argv[1]), nf = atoi(argv[2]), th = atoi(argv[3]);
    unsigned long long seed = argc > 4 ? strtoull(argv[4], NULL, 0) : 1;
    double ebn0 = argc > 5 ? atof(argv[5]) : 1000.0;
    long ns = (long)nf * QC_FRAME;
    int16_t *in = malloc(sizeof(int16_t) * (size_t)nch * ns);
    uint8_t *bits = malloc((size_t)nch * nf * QC_BITS);
    uint8_t *valid = malloc((size_t)nch * nf);
    qc_synth_batch(seed, 0, nch, ebn0, in, ns, th);
    double t0 = now();
    long nv = qc_rx_batch(in, nch, nf, bits, valid, NULL, th);
    double dt = now() - t0;
    printf("{\"msamples_per_s\": %.3f, \"seconds\": %.4f, \"valid\": %ld, \"nch\": %d, "
           "\"nframes\": %d, \"threads\": %d}\n",
           (double)nch * ns / dt / 1e6, dt, nv, nch, nf, th);
    free(in);
    free(bits);
    free(valid);
    return 0;
}
