"""Generate the golden fixtures in tests/golden/ from the UNMODIFIED reference.

Runs in the build container only (needs /root/reference and oracle/_ref, built
by `make -C oracle ref`).  Inputs are either the reference's own data file
(preamble_qpsk_8k.raw, copied here as a data fixture) or synthetic channel
streams regenerated from a seed by the oracle's TX restatement (the input's
sha256 is stored so the generator itself is pinned).  Every expected output
below comes from oracle/_ref/libqpsk_ref.so, i.e. the reference's own code.

    python tests/golden/make_golden.py            # everything
    python tests/golden/make_golden.py --dec752   # only the dec752-mode fixtures

The dec752 fixtures ("intended semantics"; NOT reference
parity) come from oracle/_ref/libqpsk_ref752.so: the same unmodified reference
sources, linked so that decimated_frame owns the 752 entries its decimation
loop writes (oracle/ref/dec752.ld).
"""
import hashlib
import json
import os
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import oracle  # noqa: E402

SYNTH_CASES = [  # (name, seed, nch, nframes, ebn0_db)
    ("synth_s1_clean", 1, 64, 16, 1000.0),
    ("synth_s2_eb8", 2, 64, 16, 8.0),
    ("synth_s3_eb4", 3, 64, 16, 4.0),
    ("synth_s4_eb0", 4, 64, 16, 0.0),
]


# src/constants.c:25-42
PREAMBLE = [-1, 1, 1, -1, -1, 1, 1, 1, -1, 1, -1, -1, 1, 1, -1, -1, 1, 1, -1, 1, -1, -1, 1, -1,
            1, -1, 1, -1, 1, -1, 1, 1, 1, -1, 1, 1, 1, 1, -1, -1, 1, -1, -1, 1, 1, -1, 1, -1,
            1, 1, -1, 1, -1, -1, 1, -1, -1, -1, -1, 1, 1, -1, 1, -1, 1, 1, 1, -1, -1, 1, 1, -1,
            1, 1, -1, -1, 1, 1, -1, 1, 1, -1, 1, 1, -1, -1, -1, 1, -1, 1, -1, 1, -1, -1, -1, 1,
            -1, -1, 1, -1, 1, 1, -1, -1, -1, -1, -1, 1, 1, 1, -1, 1, 1, -1, 1, 1, -1, -1, 1, 1,
            -1, 1, -1, 1, -1, -1, -1, 1]


DEC752_CASES = [  # (name, seed, nch, nframes, ebn0_db)
    ("synth_d752_s1_clean", 11, 48, 16, 1000.0),
    ("synth_d752_s2_eb4", 12, 48, 16, 4.0),
]


def bitstr(b):
    return "".join(str(int(v)) for v in b)


def _synth_golden(name, seed, nch, nfr, eb, mode):
    xs = oracle.synth(seed, nch, nfr, eb)
    b, v, t = oracle.ref_rx(xs, trace=True, mode=mode)
    soft = np.where(v[..., None, None].astype(bool), t["soft"], 0).astype(np.float32)
    np.savez_compressed(
        os.path.join(HERE, name + ".npz"), seed=seed, nch=nch, nframes=nfr, ebn0_db=eb,
        mode=mode, input_sha256=hashlib.sha256(xs.tobytes()).hexdigest(),
        bits=np.packbits(b, axis=-1), valid=v, max_index=t["max_index"],
        matches=t["matches"], rx_timing=t["rx_timing"], soft=soft)
    print(name, "valid frac %.3f" % v.mean())


def dec752():
    """Fixtures of the dec752 mode from the layout-padded reference build."""
    assert oracle.ref_available(oracle.MODE_DEC752)
    raw = np.fromfile(os.path.join(HERE, "preamble_qpsk_8k.raw"), np.int16)
    nf = raw.size // oracle.FRAME
    x = raw[: nf * oracle.FRAME].reshape(1, nf, oracle.FRAME)
    bits, valid, tr = oracle.ref_rx(x, trace=True, mode=oracle.MODE_DEC752)
    recs = b"".join(np.concatenate([bits[0, n], np.zeros(496 - 62, np.uint8)]).tobytes()
                    for n in range(nf) if valid[0, n])
    exp = {
        "mode": "dec752 (decimated_frame[752]; not reference parity)",
        "input": "preamble_qpsk_8k.raw",
        "input_md5": hashlib.md5(raw.tobytes()).hexdigest(),
        "frames": int(nf),
        "output_bytes": len(recs),
        "output_md5": hashlib.md5(recs).hexdigest(),
        "trace": [{k: int(tr[0, n][k]) for k in ("max_index", "matches", "valid", "rx_timing")}
                  for n in range(nf)],
        "soft": {str(n): tr[0, n]["soft"].tolist() for n in range(nf) if valid[0, n]},
    }
    with open(os.path.join(HERE, "sample_expected_dec752.json"), "w") as f:
        json.dump(exp, f, indent=1)
    for name, seed, nch, nfr, eb in DEC752_CASES:
        _synth_golden(name, seed, nch, nfr, eb, oracle.MODE_DEC752)
    print("sample (dec752):", exp["output_md5"], exp["output_bytes"], "B")


def main():
    oracle.build(ref=True)
    if "--dec752" in sys.argv[1:]:
        return dec752()
    assert oracle.ref_available()
    # 1. the reference's sample capture, through the reference driver semantics
    src = "/root/reference/preamble_qpsk_8k.raw"
    dst = os.path.join(HERE, "preamble_qpsk_8k.raw")
    shutil.copyfile(src, dst)
    raw = np.fromfile(dst, np.int16)
    nf = raw.size // oracle.FRAME
    x = raw[: nf * oracle.FRAME].reshape(1, nf, oracle.FRAME)
    bits, valid, tr, log = oracle.ref_rx(x, trace=True, log=True)
    recs = b"".join(np.concatenate([bits[0, n], np.zeros(496 - 62, np.uint8)]).tobytes()
                    for n in range(nf) if valid[0, n])
    dec, mixed, _, _ = oracle.ref_stages(x)
    exp = {
        "input": "preamble_qpsk_8k.raw",
        "input_md5": hashlib.md5(raw.tobytes()).hexdigest(),
        "frames": int(nf),
        "output_bytes": len(recs),
        "output_md5": hashlib.md5(recs).hexdigest(),
        "trace": [{k: int(tr[0, n][k]) for k in ("max_index", "matches", "valid", "rx_timing")}
                  for n in range(nf)],
        "valid_bits": {str(n): bitstr(bits[0, n]) for n in range(nf) if valid[0, n]},
        "debug2": log.splitlines(),
    }
    with open(os.path.join(HERE, "sample_expected.json"), "w") as f:
        json.dump(exp, f, indent=1)
    np.savez_compressed(os.path.join(HERE, "sample_stages.npz"), dec=dec,
                        soft=tr[0]["soft"], valid=valid[0])

    # 2. KATs straight from the reference: mixer table and keystream
    ones = np.full((1, 2, oracle.FRAME), 16384, np.int16)   # x/16384 == 1
    _, mixed1, _, _ = oracle.ref_stages(ones)
    nz = 530                                                 # 530*62 > 32767 + 62
    zb, zv, _ = oracle.ref_rx(np.zeros((1, nz, oracle.FRAME), np.int16))
    assert zv.all(), "all-zero frames are always valid (matches == 128)"
    np.savez_compressed(os.path.join(HERE, "kat.npz"), mixer_frame0=mixed1[0],
                        mixer_frame1=mixed1[1], keystream=zb[0].reshape(-1))

    # 3. seeded synthetic channels (noiseless and AWGN)
    for name, seed, nch, nfr, eb in SYNTH_CASES:
        _synth_golden(name, seed, nch, nfr, eb, oracle.MODE_REF)
    # 4. reference transmitter (src/qpsk.c:278-342): 3 packets, seeded dibits
    pre = np.array([complex(p, p) for p in PREAMBLE], np.complex64)
    rng = np.random.default_rng(42)
    syms = []
    for _ in range(3):
        syms.append((pre, True))
        for _ in range(8):
            d = rng.integers(0, 4, 31)
            syms.append((np.array([complex(-1 if v >> 1 else 1, -1 if v & 1 else 1) for v in d],
                                  np.complex64), False))
    out = oracle.ref_tx(syms)
    np.savez_compressed(os.path.join(HERE, "tx_golden.npz"),
                        symbols=np.concatenate([s for s, _ in syms]),
                        preamble=np.array([p for _, p in syms]),
                        lengths=np.array([len(s) for s, _ in syms]), samples=np.concatenate(out))
    print("sample:", exp["output_md5"], exp["output_bytes"], "B")
    dec752()


if __name__ == "__main__":
    main()
