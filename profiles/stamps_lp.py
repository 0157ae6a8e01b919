"""Role breakdown of rx_lp_kernel (QPSK_SHAPE=lp) from the diagnostic build
(in-kernel s_memtime stamps; `make -C singlecarrier_amd/csrc stamps`).
Stamps perturb timing: read the shares, not the absolute times.
Cycles per wave per frame: back work / barrier; FIR D_n / signal / F_{n+2} /
barrier; hunt wait for D_n / hunts / barrier.

    python profiles/stamps_lp.py NCH [FRAMES]
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
os.environ["QPSK_SHAPE"] = "lp"
sc.LIB_PATH = os.path.join(ROOT, "singlecarrier_amd", "csrc", "build", "libqpsk_hip_stamps.so")
lib = sc.lib()
lib.qpsk_debug_stamps.argtypes = [C.c_void_p, C.c_int]
import torch  # noqa: E402

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
nwg = (nch + 255) // 256
wf = nwg * 4 * nf          # wave-frames per role (4 groups per workgroup)
print(json.dumps({
    "channels": nch, "frames": nf,
    "back": {"work": round(v[0] / wf), "barrier": round(v[1] / wf)},
    "fir": {"D": round(v[2] / wf), "signal": round(v[3] / wf), "head": round(v[4] / wf),
            "barrier": round(v[5] / wf)},
    "hunt": {"wait D": round(v[6] / wf), "hunts": round(v[7] / wf), "barrier": round(v[8] / wf)},
}, indent=1))
