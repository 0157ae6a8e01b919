"""Per-kernel register / spill / occupancy summary of a -Rpass-analysis=kernel-resource-usage log.
    python profiles/resources.py resource.txt [name-substring ...]"""
import re
import sys

cur, out = None, {}
for line in open(sys.argv[1]):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        out[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+(?:\[[^\]]*\])?):\s*(\d+)", line)
    if cur and m:
        out[cur][m.group(1).strip()] = int(m.group(2))
pats = sys.argv[2:] or [""]
for f, d in out.items():
    if any(p in f for p in pats):
        print(f[:70], {k: d.get(k) for k in ("VGPRs", "AGPRs", "VGPRs Spill", "SGPRs Spill",
                                             "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]")})
