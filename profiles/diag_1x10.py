import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np, oracle, singlecarrier_amd as sc
for split in ("7", "6", "8"):
    for nch, nf in ((64, 4), (128, 4), (300, 12)):
        os.environ["QPSK_SHAPE"] = "1x10"; os.environ["QPSK_SPLIT10"] = split
        x = oracle.synth(61, nch, nf, 5.0)
        rx = sc.Receiver(nch)
        try:
            out = rx.demod(x)
            bits, valid, _ = oracle.cpu_rx(x)
            print(split, nch, nf, "ok", bool((out["bits"] == bits).all() and (out["valid"] == valid).all()), flush=True)
        except sc.QpskError as e:
            print(split, nch, nf, "error", e.code, flush=True)
        rx.close()
