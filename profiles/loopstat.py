"""Instruction mix of every loop in a kernel's assembly (hipcc -S output):
for each loop header label, the instructions between it and the branch back to
it.  python profiles/loopstat.py file.s [kernel-substring]"""
import collections
import re
import sys

lines = open(sys.argv[1]).read().splitlines()
kern = sys.argv[2] if len(sys.argv) > 2 else None
off = 1
if kern:
    a = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + kern + r"\S*:", l))
    b = next(i for i in range(a, len(lines)) if "s_endpgm" in lines[i])
    lines = lines[a:b + 1]
    off = a + 1
labels = {}
for i, l in enumerate(lines):
    m = re.match(r"^(\.LBB\d+_\d+):", l)
    if m:
        labels[m.group(1)] = i
for i, l in enumerate(lines):
    m = re.search(r"s_cbranch_\w+\s+(\.LBB\d+_\d+)|s_branch\s+(\.LBB\d+_\d+)", l)
    if not m:
        continue
    tgt = m.group(1) or m.group(2)
    if tgt in labels and labels[tgt] < i:
        body = [x.split()[0] for x in lines[labels[tgt]:i + 1]
                if x.strip() and not x.strip().startswith((";", ".")) and not x.startswith(".")]
        c = collections.Counter(body)
        valu = sum(v for k, v in c.items() if k.startswith("v_"))
        print(f"{tgt} lines {labels[tgt] + off}-{i + off}: {len(body)} instr, {valu} VALU, "
              f"pk {sum(v for k, v in c.items() if k.startswith('v_pk'))}, "
              f"mov {sum(v for k, v in c.items() if k.startswith('v_mov'))}, "
              f"mfma {sum(v for k, v in c.items() if 'mfma' in k)}, "
              f"ds {sum(v for k, v in c.items() if k.startswith('ds_'))}, "
              f"vmem {sum(v for k, v in c.items() if k.startswith(('global_', 'buffer_')))}")
