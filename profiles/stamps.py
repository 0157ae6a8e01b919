"""Front-wave phase breakdown from the diagnostic build (in-kernel s_memtime
stamps, singlecarrier_amd/csrc/build/libqpsk_hip_stamps.so; `make stamps`).
Stamps perturb timing: read the SHARES, not the absolute times.

    python profiles/stamps.py [front|both]
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import singlecarrier_amd as sc  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "both"
if mode == "front":
    os.environ["QPSK_ABLATE"] = "front"
sc.LIB_PATH = os.path.join(ROOT, "singlecarrier_amd", "csrc", "build", "libqpsk_hip_stamps.so")
lib = sc.lib()
lib.qpsk_debug_stamps.argtypes = [C.c_void_p, C.c_int]
import torch  # noqa: E402

nch, nf = 65536, 32
x = torch.from_numpy(sc.synth(3, nch, nf)).cuda()
bits = torch.empty((nch, nf, 62), dtype=torch.uint8, device="cuda")
valid = torch.empty((nch, nf), dtype=torch.uint8, device="cuda")
rx = sc.Receiver(nch)
rx.demod_device(x, bits, valid)
torch.cuda.synchronize()
st = np.zeros(16, np.uint64)
lib.qpsk_debug_stamps(st.ctypes.data, 1)
rx.demod_device(x, bits, valid)
torch.cuda.synchronize()
lib.qpsk_debug_stamps(st.ctypes.data, 1)
names = {0: "mix", 1: "store_window+prefetch+sync", 6: "front_channel+mi+sync (total)",
         7: "frame barrier wait", 8: "FIR decimated (D)", 9: "FIR head (F)+sync",
         10: "T image+sync", 11: "correlate (MFMA)", 12: "argmax (DPP max)"}
bnames = {13: "back: frame (128 train steps + job/outputs)", 14: "back: frame barrier wait"}
ch_iters = nch * nf  # front-wave channel iterations (each wave does 32 per frame)
waves = nch // 32
out = {"mode": mode, "cycles_per_channel": {}}
tot = sum(int(st[i]) for i in (0, 1, 6, 7))
for i, nm in names.items():
    v = int(st[i]) / ch_iters  # lane-0 sums: cycles per channel iteration
    out["cycles_per_channel"][nm] = round(v, 1)
out["share_of_loop"] = {names[i]: round(int(st[i]) / tot, 3) for i in (0, 1, 6, 7)}
bw = nch // 64   # back waves
btot = int(st[13]) + int(st[14])
out["back_cycles_per_frame"] = {bnames[i]: round(int(st[i]) / (bw * nf), 1) for i in (13, 14)}
out["back_share"] = {bnames[i]: round(int(st[i]) / max(btot, 1), 3) for i in (13, 14)}
# round 6 (4x2 only): the back wave's arrival at the frame barrier minus the
# last arrival of the fronts on its SIMD (stamp 15), over the frames where the
# back arrived last (stamp 5): the cycles it trains alone at each frame's end
fr = bw * nf
out["back_alone_tail"] = {
    "frames_back_last_share": round(int(st[5]) / fr, 3),
    "tail_cycles_per_frame_all": round(int(st[15]) / fr, 1),
    "tail_cycles_per_frame_when_last": round(int(st[15]) / max(int(st[5]), 1), 1),
    "frame_cycles": round(btot / fr, 1),
    "tail_share_of_frame": round(int(st[15]) / max(btot, 1), 3)}
print(json.dumps(out, indent=1))
