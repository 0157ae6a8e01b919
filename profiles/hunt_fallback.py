"""How often the filtered hunt hands a channel-frame to the exact chain
(qpsk_hunt.h hunt_index), from the diagnostic build's counters
(`make -C singlecarrier_amd/csrc stamps`: stamp slots 2 = hunts, 3 = exact
chain runs).  One line per workload.

    python profiles/hunt_fallback.py
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import singlecarrier_amd as sc  # noqa: E402

sc.LIB_PATH = os.path.join(ROOT, "singlecarrier_amd", "csrc", "build", "libqpsk_hip_stamps.so")
lib = sc.lib()
lib.qpsk_debug_stamps.argtypes = [C.c_void_p, C.c_int]
import torch  # noqa: E402

st = np.zeros(16, np.uint64)
for nch, ebn0 in ((65536, 1000.0), (65536, 10.0), (65536, 5.0), (65536, 0.0), (8192, 1000.0)):
    nf = 32
    x = sc.synth_device(3, nch, nf, ebn0)
    bits = torch.empty((nch, nf, 62), dtype=torch.uint8, device="cuda")
    valid = torch.empty((nch, nf), dtype=torch.uint8, device="cuda")
    rx = sc.Receiver(nch)
    lib.qpsk_debug_stamps(st.ctypes.data, 1)
    rx.demod_device(x, bits, valid)
    torch.cuda.synchronize()
    lib.qpsk_debug_stamps(st.ctypes.data, 1)
    hunts, exact = int(st[2]), int(st[3])
    print(json.dumps({"channels": nch, "frames": nf, "ebn0_db": ebn0 if ebn0 < 100 else None,
                      "hunts": hunts, "exact_chain": exact,
                      "exact_share": round(exact / max(hunts, 1), 5),
                      "valid_share": round(float(valid.float().mean()), 4)}), flush=True)
    del x, bits, valid, rx
