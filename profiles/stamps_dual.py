"""Role breakdown of the dual-chain kernel from the diagnostic build (in-kernel
s_memtime stamps, singlecarrier_amd/csrc/build/libqpsk_hip_stamps.so; `make
stamps`).  Stamps perturb timing: read the SHARES and the per-role balance, not
the absolute times.

    python profiles/stamps_dual.py NCH [FRAMES]      (QPSK_QUAD / QPSK_WIDTH as usual)

Per back wave and frame it trains: frame work (13: 128 train_eq steps, job,
outputs), wait for the fronts (14), wait for the other chain's decision (15).
Per front wave and frame: wait for the backs (7), per channel: mix (0), window
store + prefetch (1), front_channel + tail (6, of which 8-12 are its phases).
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import singlecarrier_amd as sc  # noqa: E402

nch = int(sys.argv[1])
nf = int(sys.argv[2]) if len(sys.argv) > 2 else 32
sc.LIB_PATH = os.environ.get("QPSK_STAMPS_LIB") or os.path.join(ROOT, "singlecarrier_amd", "csrc", "build",
                                                                 "libqpsk_hip_stamps.so")
lib = sc.lib()
lib.qpsk_debug_stamps.argtypes = [C.c_void_p, C.c_int]
import torch  # noqa: E402

ncu = torch.cuda.get_device_properties(0).multi_processor_count
W = int(os.environ.get("QPSK_WIDTH", "0")) or (16 if nch <= 16 * ncu else 32 if nch <= 32 * ncu else 64)
quad = int(os.environ.get("QPSK_QUAD", "1" if (W <= 32 or os.environ.get("QPSK_FRONTS") == "4") else "0"))
nwg = (nch + W - 1) // W
back_waves = nwg * 2 * (W // (16 * quad) if quad else 1)
front_waves = nwg * (4 if os.environ.get("QPSK_FRONTS") == "4" and quad else 8)
x = torch.from_numpy(sc.synth(3, nch, nf)).cuda()
bits = torch.empty((nch, nf, 62), dtype=torch.uint8, device="cuda")
valid = torch.empty((nch, nf), dtype=torch.uint8, device="cuda")
rx = sc.Receiver(nch)
st = np.zeros(16, np.uint64)
rx.demod_device(x, bits, valid)
torch.cuda.synchronize()
lib.qpsk_debug_stamps(st.ctypes.data, 1)
rx.demod_device(x, bits, valid)
torch.cuda.synchronize()
lib.qpsk_debug_stamps(st.ctypes.data, 1)
v = [int(t) for t in st]
bf = back_waves * nf / 2          # back-wave frames
ff = front_waves * nf             # front-wave frames
fc = nch * nf                     # front channel iterations
out = {
    "channels": nch, "frames": nf, "W": W, "quad": quad,
    "back_cycles_per_frame": {"work (13)": round(v[13] / bf), "wait fronts (14)": round(v[14] / bf),
                              "wait other chain (15)": round(v[15] / bf)},
    "front_cycles_per_frame": {"wait backs (7)": round(v[7] / ff), "signal (5)": round(v[5] / ff),
                               "channels (0+1+4+6)": round((v[0] + v[1] + v[4] + v[6]) / ff)},
    "front_cycles_per_channel": {"mix (0)": round(v[0] / fc), "window store (4)": round(v[4] / fc),
                                 "prefetch+sync (1)": round(v[1] / fc),
                                 "front_channel+tail (6)": round(v[6] / fc),
                                 "FIR D (8)": round(v[8] / fc), "FIR head (9)": round(v[9] / fc),
                                 "T image (10)": round(v[10] / fc), "MFMA (11)": round(v[11] / fc),
                                 "argmax (12)": round(v[12] / fc)},
}
out["back_steps_cycles"] = round(v[13] / bf / 128)
print(json.dumps(out, indent=1))
