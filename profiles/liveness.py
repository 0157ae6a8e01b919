"""VGPR pressure along a loop body of a kernel's assembly (hipcc -S output):
which registers are live where, to find what holds a kernel above a
register budget.  Straight-line approximation: the body is treated as one
block executed in order (branches inside are ignored); a register read before
its first write in the body is loop-carried (live from the top), one written
and read again at the top of the next iteration is live to the bottom.

    python profiles/liveness.py file.s START END [top]
"""
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
from depsim import parse  # noqa: E402


def main():
    f, a, b = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 12
    lines = open(f).read().splitlines()[a - 1:b]
    ins = parse(lines)
    n = len(ins)
    # backward liveness over the body as straight-line code, loop-carried values
    # (live into the top) live out of the bottom; two passes reach the fixpoint
    live_top = set()
    for _ in range(3):
        live = set(live_top)
        count = [0] * n
        live_at = [None] * n
        for i in range(n - 1, -1, -1):
            op, dst, src, _, _ = ins[i]
            live = (live - set(dst)) | set(src)
            count[i] = len(live)
            live_at[i] = live
        live_top = live
    peak = max(range(n), key=lambda i: count[i])
    print(f"{n} instructions; peak {count[peak]} live VGPRs before body instruction {peak}: {ins[peak][4]}")
    print(f"live into the top (loop-carried): {len(live_top)}")
    # for each register live at the peak: its defining instruction (last def at or
    # before the peak) and its next use after the peak
    for r in sorted(live_at[peak])[:top]:
        d = next((i for i in range(peak, -1, -1) if r in ins[i][1]), None)
        u = next((i for i in range(peak, n) if r in ins[i][2]), None)
        print(f"  v{r}: def {d if d is not None else 'carried'}: "
              f"{(ins[d][4][:55] if d is not None else '')!r} -> use {u}: {(ins[u][4][:55] if u is not None else '')!r}")
    step = max(1, n // 40)
    print("live VGPRs along the body:", " ".join(str(max(count[i:i + step])) for i in range(0, n, step)))


if __name__ == "__main__":
    main()
