"""Summarise a profiles/profile.sh run: per-kernel average duration and
per-dispatch PMC averages for rx_kernel / rx_data_kernel, HBM traffic per
launch with the gfx950 FETCH_SIZE correction (MI355X_MICROARCH.md 'HBM':
FETCH_SIZE counts half the bytes of wide coalesced reads -> x2), the VALU
instruction count per launch (SQ_INSTS_VALU) and the LDS bank-conflict share;
writes profiles/<tag>_summary.md, profiles/pmc_traffic.json and
profiles/pmc_valu.json (bench.py reads the last two when the workload AND the
kernel hash match: the run directory's kernel_hash.txt, written by profile.sh
from the profiled library's qpsk_kernel_hash()).

    python profiles/summarize.py gpurun_out/prof_v1 TAG CHANNELS FRAMES [SKIP [COUNT]]

Only the bench's timed launches are summarised: per kernel, the launches
SKIP .. SKIP+COUNT-1 in dispatch order (default 2 and 5 = bench.py's
--warmup 2 --steps 5 as profile.sh runs it).  Later launches of the same
kernels (other batch sizes) and the cold warmup launches are excluded.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

d, tag, nch, nfr = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
SKIP = int(sys.argv[5]) if len(sys.argv) > 5 else 2
COUNT = int(sys.argv[6]) if len(sys.argv) > 6 else 5
K, KD = "rx_kernel", "rx_data_kernel"


def rows(pattern):
    out = []
    for f in glob.glob(os.path.join(d, pattern), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def short(name):
    name = re.sub(r"<[^<>]*>", "", name.replace("(anonymous namespace)", "anon"))   # template args
    m = re.search(r"(\w+)\(", name)
    return m.group(1) if m else name


def launches(run):
    """{kernel: [(dispatch_id, duration ns)]} of the selected launches"""
    per = defaultdict(list)
    for x in rows(f"{run}/**/*kernel_trace.csv"):
        per[short(x["Kernel_Name"])].append(
            (int(x["Dispatch_Id"]), int(x["End_Timestamp"]) - int(x["Start_Timestamp"])))
    return {k: sorted(v)[SKIP:SKIP + COUNT] for k, v in per.items()}


def avg_ns(run, kern):
    sel = launches(run).get(kern, [])
    return sum(t for _, t in sel) / len(sel) if sel else 0.0


def counters(run, kern):
    ids = {i for i, _ in launches(run).get(kern, [])}
    acc = defaultdict(lambda: defaultdict(float))   # counter -> dispatch -> sum over agents/dims
    for x in rows(f"{run}/**/*counter_collection.csv"):
        if short(x["Kernel_Name"]) == kern and int(x["Dispatch_Id"]) in ids:
            acc[x["Counter_Name"]][int(x["Dispatch_Id"])] += float(x["Counter_Value"])
    return {k: sum(v.values()) / len(v) for k, v in acc.items()}


lines = [f"# rocprofv3 summary: {tag} ({nch} channels x {nfr} frames per launch)", "",
         f"Launches {SKIP}..{SKIP + COUNT - 1} of each kernel (the bench's timed steps; "
         f"the first {SKIP} are its untimed warmup).", ""]
t_ns, t_dns = avg_ns("stats", K), avg_ns("stats", KD)
lines += ["## Kernel durations (kernel-trace)", "", "| kernel | launches | avg us |", "|---|---|---|",
          f"| {K} | {COUNT} | {t_ns / 1e3:.1f} |", f"| {KD} | {COUNT} | {t_dns / 1e3:.1f} |"]
for ab in ("abl_back", "abl_front"):
    if glob.glob(os.path.join(d, ab)):
        lines.append(f"| {K} [{ab}: only the {ab[4:]} role runs] | {COUNT} | {avg_ns(ab, K) / 1e3:.1f} |")
c, cd = {}, {}
for p in ("fetch", "write", "sq", "lds"):
    c.update(counters(p, K))
    cd.update(counters(p, KD))
# per step: rx_kernel + rx_data_kernel (the data symbols of the valid frames)
fetch_b = (c.get("FETCH_SIZE", 0) + cd.get("FETCH_SIZE", 0)) * 1024 * 2   # KB, x2 gfx950 correction
write_b = (c.get("WRITE_SIZE", 0) + cd.get("WRITE_SIZE", 0)) * 1024
alg = nch * nfr * 3823
t_step = t_ns + t_dns
lines += ["", "## Counters per dispatch (averages)", "", f"| counter | {K} | {KD} |", "|---|---|---|"]
for k in sorted(c):
    lines.append(f"| {k} | {c[k]:.4g} | {cd.get(k, float('nan')):.4g} |")
lines += ["", "## Derived (per step = one rx_kernel + one rx_data_kernel launch)", "",
          f"- HBM read bytes/step (2 x FETCH_SIZE): {fetch_b / 1e6:.1f} MB; written (WRITE_SIZE): {write_b / 1e6:.1f} MB",
          f"- algorithmic bytes/step: {alg / 1e6:.1f} MB (3823 B per channel-frame, {nch} x {nfr})",
          f"- traffic / algorithmic = {(fetch_b + write_b) / alg:.2f}",
          f"- kernel time/step: {t_ns / 1e3:.1f} + {t_dns / 1e3:.1f} us; achieved algorithmic GB/s = {alg / t_step:.1f}; physical GB/s = {(fetch_b + write_b) / t_step:.1f}"]
if "SQ_WAVE_CYCLES" in c and "SQ_BUSY_CYCLES" in c:
    lines.append(f"- VALU instructions per wave-cycle: {c['SQ_INSTS_VALU'] / max(c['SQ_WAVE_CYCLES'], 1):.3f}; "
                 f"SQ_ACTIVE_INST_VALU/SQ_WAVE_CYCLES = {c['SQ_ACTIVE_INST_VALU'] / c['SQ_WAVE_CYCLES']:.3f}")
clock = None
if "GRBM_GUI_ACTIVE" in c:
    clock = c['GRBM_GUI_ACTIVE'] / 8 / t_ns
    lines.append(f"- effective clock ~ GRBM_GUI_ACTIVE/8/t = {clock:.2f} GHz")
if "SQ_LDS_BANK_CONFLICT" in c and "SQ_ACTIVE_INST_LDS" in c:
    lines.append(f"- LDS bank conflicts: SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS = "
                 f"{c['SQ_LDS_BANK_CONFLICT'] / max(c['SQ_ACTIVE_INST_LDS'], 1):.3f}"
                 + (f"; / SQ_LDS_IDX_ACTIVE = {c['SQ_LDS_BANK_CONFLICT'] / max(c['SQ_LDS_IDX_ACTIVE'], 1):.3f}"
                    if "SQ_LDS_IDX_ACTIVE" in c else ""))
valu_insts = c.get("SQ_INSTS_VALU", 0) + cd.get("SQ_INSTS_VALU", 0)
if valu_insts:
    lines.append(f"- VALU wave-instructions per step (SQ_INSTS_VALU, both kernels): {valu_insts:.4g}; "
                 f"issue rate {valu_insts / t_step:.4g} per ns vs peak 1,024 SIMDs / 2 cycles x 2.4 GHz "
                 f"= 1228.8 per ns: {valu_insts / t_step / 1228.8:.3f}")
# the profiled library's qpsk_kernel_hash() (profile.sh writes it next to the
# runs): bench.py reports these counters only for a library with that hash
khash = None
kh_path = os.path.join(d, "kernel_hash.txt")
if os.path.exists(kh_path):
    khash = open(kh_path).read().strip() or None
lines.append(f"- kernel hash (qpsk_kernel_hash of the profiled library): {khash}")
open(os.path.join("profiles", f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
json.dump({"channels": nch, "frames": nfr, "hbm_bytes_per_launch": int(fetch_b + write_b),
           "kernels": [K, KD],
           "fetch_bytes": int(fetch_b), "write_bytes": int(write_b), "kernel_hash": khash,
           "source": f"profiles/{tag}_summary.md (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes)"},
          open(os.path.join("profiles", "pmc_traffic.json"), "w"), indent=1)
if valu_insts:
    json.dump({"channels": nch, "frames": nfr, "kernels": [K, KD],
               "valu_insts_per_launch": int(valu_insts),
               "active_valu_frac": (round(c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"], 4)
                                    if "SQ_ACTIVE_INST_VALU" in c and "SQ_WAVE_CYCLES" in c else None),
               "clock_ghz": round(clock, 3) if clock else None, "kernel_hash": khash,
               "source": f"profiles/{tag}_summary.md (rocprofv3 --pmc SQ_INSTS_VALU pass)"},
              open(os.path.join("profiles", "pmc_valu.json"), "w"), indent=1)
print("\n".join(lines))
