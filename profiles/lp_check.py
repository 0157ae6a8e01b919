"""Quick exactness check of the lane-parallel front (QPSK_SHAPE=lp) against
the oracle on a few batch shapes and call splits (A/B tool; the pytest GPU
suite is the real gate)."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle
import singlecarrier_amd as sc


def check(nch, nf, ebn0, seed, splits=None):
    x = oracle.synth(seed, nch, nf, ebn0)
    bits, valid, tr = oracle.cpu_rx(x, trace=True)
    rx = sc.Receiver(nch)
    parts, a = [], 0
    for b in (splits or []) + [nf]:
        parts.append(rx.demod(np.ascontiguousarray(x[:, a:b]), trace=True, soft=True))
        a = b
    out = {k: np.concatenate([p[k] for p in parts], axis=1) for k in ("bits", "valid", "trace", "soft")}
    t = out["trace"]
    res = {
        "valid": int((out["valid"] != valid).sum()),
        "bits": int((out["bits"] != bits).sum()),
        "mi": int((t[..., 0] != tr["max_index"]).sum()),
        "matches": int((t[..., 1] != tr["matches"]).sum()),
        "rt": int((t[..., 3] != tr["rx_timing"]).sum()),
    }
    vm = valid.astype(bool)
    res["soft"] = int((out["soft"][vm] != tr["soft"][vm]).sum())
    ok = all(v == 0 for v in res.values())
    print(f"nch={nch} nf={nf} ebn0={ebn0} splits={splits}: {'OK' if ok else 'DIFF'} {res}", flush=True)
    if not ok:
        bad = np.argwhere(t[..., 0] != tr["max_index"])[:5]
        print("  first mi diffs (ch, frame):", bad.tolist(), flush=True)
    return ok


if __name__ == "__main__":
    ok = True
    ok &= check(64, 4, 1000.0, 5)
    ok &= check(300, 9, 4.0, 6, [1, 2, 5])
    ok &= check(1000, 12, 1000.0, 7, [3])
    ok &= check(4096, 16, 6.0, 8)
    sys.exit(0 if ok else 1)
