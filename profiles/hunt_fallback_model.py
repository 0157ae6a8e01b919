"""Model of the filtered hunt's exact-fallback rate (qhunt::pick_h) against its error bound
d = W * 2^-13 scaled by a factor, on oracle dec images (float64 correlations): the rate a
wider bound (e.g. a filter FIR feeding the hunt) would cause.  CPU only:
    python3 profiles/hunt_fallback_model.py"""
import sys, re; sys.path.insert(0,'/root/repo')
import numpy as np, oracle
src = open('/root/repo/singlecarrier_amd/csrc/qpsk_consts.h').read()
pre = np.array([int(v) for v in re.search(r'QK_PRE\[QK_NPRE\] = \{([^}]*)\}', src).group(1).replace('\n',' ').split(',') if v.strip()], np.float64)
idx = np.arange(128)[:,None] + np.arange(128)[None,:]
def rates(x, factors):
    nch, nf = x.shape[:2]
    cnt = np.zeros(len(factors)); tot = 0; zero = 0; gaps = []
    for c in range(nch):
        dec = oracle.cpu_stages(x[c]).astype(np.float64)
        for n in range(nf):
            d = dec[n]
            Tr = d[:255,0] - d[:255,1]; Ti = d[:255,1] + d[:255,0]
            W = np.abs(Tr).sum() + np.abs(Ti).sum()
            if W == 0: zero += 1; continue
            Sr = (Tr[idx] * pre[None,:]).sum(1); Si = (Ti[idx] * pre[None,:]).sum(1)
            ar, ai = np.abs(Sr), np.abs(Si)
            cn = ar**2 + ai**2
            s = np.sort(cn); gaps.append((s[-1]-s[-2]) / (W*W))
            tot += 1
            for k, f in enumerate(factors):
                dd = W * 2.0**-13 * f
                U = (ar+dd)**2 + (ai+dd)**2
                L = np.maximum(ar-dd,0)**2 + np.maximum(ai-dd,0)**2
                if (U >= L.max()).sum() != 1: cnt[k] += 1
    return cnt / tot, tot, zero, np.array(gaps)
F = [1/64, 1/16, 1/4, 1, 4, 16]
for eb in (1000.0, 5.0):
    x = oracle.synth(5, 64, 8, eb)
    r, tot, zero, gaps = rates(x, F)
    print(f"EbN0 {eb}: {tot} nonzero channel-frames (+{zero} silent); fallback rate at bound x{[round(f,4) for f in F]}:", np.round(r, 3))
    print("  exact ties (gap 0):", int((gaps == 0).sum()), " gap/W^2 quantiles:", np.quantile(gaps, [0.05, 0.1, 0.3, 0.5]))
