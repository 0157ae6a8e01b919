/* Block decision steps of the bench workload (profiles/r03_early_decision_ab.txt):
 *   gcc -O2 -std=gnu11 -ffp-contract=off -Ioracle -o /tmp/dsteps profiles/decision_steps_drv.c oracle/cpu_ref.c -lm -lpthread
 *   /tmp/dsteps NCH FRAMES BLOCK [EBN0] */
#include <stdio.h>
#include <stdlib.h>
#include "cpu_ref.h"
int main(int argc, char** argv) {
    int nch = atoi(argv[1]), nf = atoi(argv[2]), blk = atoi(argv[3]);
    double eb = argc > 4 ? atof(argv[4]) : 1000.0;
    int16_t* x = malloc((size_t)nch * nf * QC_FRAME * 2);
    qc_synth_batch(3, 0, nch, eb, x, (long)nf * QC_FRAME, 8);
    int* ds = malloc(sizeof(int) * nch * nf);
    int* vd = malloc(sizeof(int) * nch * nf);
    for (int c = 0; c < nch; c++) {
        qc_chan_t ch; qc_chan_init(&ch);
        uint8_t bits[QC_BITS];
        for (int n = 0; n < nf; n++) {
            vd[c * nf + n] = qc_rx_frame(&ch, x + ((size_t)c * nf + n) * QC_FRAME, bits, NULL);
            ds[c * nf + n] = qc_decision_step;
        }
    }
    /* per block of blk channels and frame: max decision step */
    long hist[130] = {0}, chist[130] = {0}; long nb = 0, sum = 0, nvalid = 0;
    for (int b = 0; b < nch / blk; b++)
        for (int n = 0; n < nf; n++) {
            int m = 0;
            for (int c = b * blk; c < (b + 1) * blk; c++) { if (ds[c * nf + n] > m) m = ds[c * nf + n]; chist[ds[c*nf+n]]++; nvalid += vd[c*nf+n]; }
            hist[m]++; nb++; sum += m;
        }
    printf("blocks %ld mean block decision step %.1f, valid %.3f\n", nb, (double)sum / nb, (double)nvalid / nch / nf);
    long acc = 0;
    for (int s = 0; s <= 128; s++) { acc += hist[s]; if (hist[s]) printf("step<=%d: %.3f\n", s, (double)acc / nb); }
    return 0;
}
