"""In-order issue model of one wave's loop body (hipcc -S output), to price a
schedule before spending GPU time on it.

    python profiles/depsim.py file.s START END [--detail]

START/END are line numbers of the loop (profiles/loopstat.py prints them).
Model (profiles/calib/valu_rate_r01.txt, MI355X_MICROARCH.md constants):
one wave issues an independent VALU instruction every 4.64 cycles (packed
fp32 5.0, v_rcp 8.57, a DPP add 6.68), a dependent one no earlier than 9.7
cycles after its producer issued (14 for a DPP read of a VALU result); every
other instruction (SALU, waits, branches, s_nop 0) takes one issue slot of 4
cycles, s_nop N 4(N+1).  calib/valu_rate_r01.txt, calib/dpp_rate_r04.txt.  The body is iterated twice
and the second pass is reported (loop-carried latency included).
"""
import re
import sys

ISSUE = {"pk": 5.0, "trans": 8.57, "valu": 4.64, "dpp_alu": 6.68, "scalar": 4.0}
LAT = 9.7
DPP_LAT = 14.0   # VALU write -> DPP read of it, issue to issue (calib/dpp_rate: 14.0-14.2)
TRANS = ("v_rcp_", "v_rsq_", "v_sqrt_", "v_exp_", "v_log_", "v_sin_", "v_cos_")


def regs(tok):
    """VGPR numbers named by one operand token."""
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return list(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    if m:
        return [int(m.group(1))]
    return []


def parse(lines):
    out = []
    for l in lines:
        s = l.strip()
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        s = s.split(";")[0]
        op = s.split()[0]
        rest = s[len(op):]
        toks = [t.strip() for t in re.split(r",\s*", rest.strip()) if t.strip()]
        toks = [t.split()[0] for t in toks]
        dst, src = [], []
        if op.startswith("v_pk_") and toks:
            # packed: source i's low register feeds the low result unless
            # op_sel[i], its high register the high result unless op_sel_hi[i] = 0
            def bits(name, k, dflt):
                m = re.search(name + r":\[([0-9,]+)\]", s)
                v = [int(x) for x in m.group(1).split(",")] if m else []
                return [v[i] if i < len(v) else dflt for i in range(k)]
            srcs = toks[1:]
            osel = bits(r"(?<!_)op_sel", len(srcs), 0)
            oshi = bits("op_sel_hi", len(srcs), 1)
            dst = regs(toks[0])
            for i, t in enumerate(srcs):
                rr = regs(t)
                if len(rr) == 2:
                    src += [rr[1] if osel[i] else rr[0], rr[1] if oshi[i] else rr[0]]
                else:
                    src += rr
        elif op.startswith("v_") and toks:
            if op.startswith(("v_cmp", "v_readfirstlane", "v_readlane")):
                src = [r for t in toks[1:] for r in regs(t)]
            else:
                dst = regs(toks[0])
                src = [r for t in toks[1:] for r in regs(t)]
        elif op.startswith(("ds_write", "global_store", "buffer_store")):
            src = [r for t in toks for r in regs(t)]
        elif op.startswith(("ds_read", "global_load", "buffer_load")):
            dst = regs(toks[0]) if toks else []
            src = [r for t in toks[1:] for r in regs(t)]
        out.append((op, dst, src, "dpp" in s, s))
    return out


def cost(op, dpp=False):
    if op.startswith("v_pk_"):
        return ISSUE["pk"]
    if op.startswith(TRANS):
        return ISSUE["trans"]
    if dpp and not op.startswith("v_mov"):
        return ISSUE["dpp_alu"]
    if op.startswith("v_"):
        return ISSUE["valu"]
    return ISSUE["scalar"]   # one issue slot of the wave: SALU, waits, branches, s_nop 0


def simulate(ins, passes=2, detail=False):
    ready = {}       # vgpr -> cycle its value can be read
    written = {}     # vgpr -> cycle written (for DPP wait states)
    t = 0.0
    starts = []
    stall_by = {}
    for p in range(passes):
        t0 = t
        for op, dst, src, dpp, text in ins:
            r = max([ready.get(x, 0.0) for x in src] + [0.0])
            if dpp:
                r = max([r] + [written.get(x, 0.0) + DPP_LAT for x in src[:1]])
            issue = max(t, r)
            if p == passes - 1:
                stall_by[op] = stall_by.get(op, 0.0) + (issue - t)
                if detail:
                    print(f"{issue - t0:8.1f} +{issue - t:5.1f}  {text}")
            c = cost(op, dpp)
            if op.startswith("s_nop"):
                m = re.search(r"s_nop\s+(\d+)", text)
                c = 4.0 * (int(m.group(1)) + 1) if m else 4.0
            t = issue + c
            lat = LAT if op.startswith("v_") else (60.0 if op.startswith("ds_") else 0.0)
            for x in dst:
                ready[x] = issue + lat
                written[x] = issue
        starts.append(t - t0)
    return starts[-1], stall_by


def main():
    f, a, b = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    lines = open(f).read().splitlines()[a - 1:b]
    ins = parse(lines)
    nvalu = sum(1 for i in ins if i[0].startswith("v_"))
    issue_only = sum(cost(i[0], i[3]) for i in ins)
    cyc, stalls = simulate(ins, detail="--detail" in sys.argv)
    print(f"{len(ins)} instr, {nvalu} VALU; issue-only {issue_only:.0f} cyc; modelled {cyc:.0f} cyc")
    top = sorted(stalls.items(), key=lambda kv: -kv[1])[:12]
    print("stall cycles by the stalled instruction's opcode:", ", ".join(f"{k} {v:.0f}" for k, v in top))


if __name__ == "__main__":
    main()
