"""Per-kernel averages of a rocprofv3 --pmc run (counter_collection.csv), the
bench's timed launches only (launches SKIP .. SKIP+COUNT-1 of rx_kernel).
    python profiles/pmc_table.py DIR [DIR ...]"""
import csv
import glob
import sys
from collections import defaultdict

SKIP, COUNT = 2, 5
for d in sys.argv[1:]:
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    if not f:
        print(d, "no counters")
        continue
    per = defaultdict(lambda: defaultdict(float))   # dispatch -> counter -> value
    name = {}
    for row in csv.DictReader(open(f[0])):
        if "rx_kernel" not in row["Kernel_Name"]:
            continue
        k = int(row["Dispatch_Id"])
        per[k][row["Counter_Name"]] += float(row["Counter_Value"])
        name[k] = row["Kernel_Name"]
    ks = sorted(per)[SKIP:SKIP + COUNT]
    avg = {c: sum(per[k][c] for k in ks) / len(ks) for c in per[ks[0]]}
    wc = avg.get("SQ_WAVE_CYCLES", 0)
    out = [f"{d.rstrip('/').split('/')[-1]:>10}"]
    for c in sorted(avg):
        out.append(f"{c}={avg[c]:.4g}")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS"):
            if c in avg:
                out.append(f"{c}/WAVE_CYCLES={avg[c] / wc:.3f}")
    print("  ".join(out))
