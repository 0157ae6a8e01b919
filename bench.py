#!/usr/bin/env python3
"""bench.py -- demodulated Msamples/s of the MI355X QPSK receive path.

One "step" = demodulating one batch: every channel of the workload advances by
`--frames` 1880-sample frames (C3: 65536 channels x 32 frames = 3.94e9 int16
samples, 7.88 GB, resident in HBM before timing).

N GPUs (C4): the 65536-channel batch is split into N channel
shards, shard g = channels [g*C/N, (g+1)*C/N) on GPU g, one process per GPU,
no collective on the data path ("scaling": "strong"; --weak gives every GPU
its own 65536-channel batch instead).  The barrier around the timed region and
the MAX-over-ranks time reduction run over gloo on the host, not RCCL.

    python bench.py [--gpus N] [--steps K] [--warmup W]     (spawns N ranks itself)
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Rank 0 prints ONE JSON line.  See DESIGN.md "Measurement" for every field.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "demodulated Msamples/sec (whole node), 65536-channel 8 kHz batch; BER vs ref"
FRAME = 1880
ALG_BYTES_PER_FRAME = 3760 + 63     # int16 in + 62 bit-bytes + valid byte
HBM_PEAK_GBS = 8000.0               # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
VALU_SIMDS = 256 * 4                 # MI355X: 256 CUs x 4 SIMD-32
VALU_CLOCK_GHZ = 2.4                 # max engine clock (MI355X_MICROARCH.md)


# receiver semantics (include/qpsk_batch.h QPSK_MODE_*): reference parity, the
# dec752 buffer, the kiss_fft hunt, both (not parity)
MODES = {"reference": 0, "dec752": 1, "fft": 2, "dec752fft": 3}


def shard(channels: int, world: int, rank: int, strong: bool = True):
    """(channels on this rank, first global channel id).  Strong (C4, default):
    one `channels`-channel batch split across the ranks, shard g = channels
    [g*C/N, (g+1)*C/N) (src/qpsk.c:436-458 is the per-channel
    loop being split); weak: every rank demodulates its own `channels`-channel
    batch (distinct channel ids)."""
    if strong:
        base, rem = divmod(channels, world)
        return base + (1 if rank < rem else 0), rank * base + min(rank, rem)
    return channels, rank * channels


def reduce_step(dist, wall: float, nch: int):
    """Job time = MAX over ranks of the timed region; channels = SUM.  Host
    tensors over the gloo group: no collective touches the GPUs."""
    import torch
    if dist is None:
        return wall, nch
    tmax = torch.tensor([wall], dtype=torch.float64)
    dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    tot = torch.tensor([nch], dtype=torch.int64)
    dist.all_reduce(tot)
    return float(tmax.item()), int(tot.item())


def init_host_group(rank: int, world: int):
    """The ranks' host-side gloo group (barrier and time reduction only).
    gloo's native code announces its peer connections on fd 1; the driver
    reads rank 0's stdout as the one JSON line, so fd 1 points at stderr
    while the group forms."""
    import datetime

    import torch.distributed as dist
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        # a bounded rendezvous/collective timeout: a rank that dies outside the
        # launcher's watch (torch.distributed.run) cannot hold the others for
        # gloo's default 30 minutes
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=300))
    finally:
        os.dup2(saved, 1)
        os.close(saved)
    return dist


def free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(nproc: int, argv, script: str = None, env=None, poll_s: float = 0.2,
           grace_s: float = 10.0) -> int:
    """Run `script argv` as `nproc` ranks (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*
    as torch.distributed.run sets them), one per GPU, and wait for all of
    them.  The launcher itself makes no GPU call (children are started before
    anything here touches HIP, and by Popen, never exec).  Every child is
    watched: the first one to exit non-zero gets its peers terminated (they
    would otherwise block in gloo's rendezvous or barrier until its timeout),
    killed if they are still alive `grace_s` later, and its status is returned
    (128 + signal for a rank ended by a signal); 0 when every rank succeeds."""
    import subprocess
    script = script or os.path.abspath(__file__)
    port = free_port()
    procs = []
    for r in range(nproc):
        e = dict(os.environ if env is None else env)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nproc), LOCAL_WORLD_SIZE=str(nproc),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script, *argv], env=e))
    first_bad = 0
    killed_at = None                    # when the peers of a failed rank were terminated
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and first_bad == 0:
                # a rank killed by a signal reports -signum: as a shell would, 128 + signum
                first_bad = rc if rc > 0 else 128 - rc
                killed_at = time.monotonic()
                for q in live:          # exact children of this launcher, by handle
                    q.terminate()
        if live and killed_at is not None and time.monotonic() - killed_at > grace_s:
            for q in live:              # a peer that ignored SIGTERM
                q.kill()
            killed_at = float("inf")
        if live:
            time.sleep(poll_s)
    return first_bad


def cpu_info() -> dict:
    """Host-core provenance for the CPU baselines (BASELINE.md plan)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = None
    # the CPU time this job may use: cgroup v2 cpu.max ("quota period", or
    # "max" for no limit), as CPUs
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"nproc": os.cpu_count(), "affinity_cpus": aff, "cgroup_cpu_quota": quota,
            "cpu_model": model, "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def host_cpus() -> int:
    """CPUs this job may run on at once: the affinity set, capped by the cgroup
    CPU quota (on the GPU boxes the affinity set is the node's 256 CPUs while
    cpu.max grants 16: more workers than that only time-share them)."""
    info = cpu_info()
    n = info["affinity_cpus"] or os.cpu_count() or 1
    if info["cgroup_cpu_quota"]:
        n = min(n, max(1, int(info["cgroup_cpu_quota"])))
    return n


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--channels", type=int, default=65536,
                    help="channels of the batch (split over the GPUs; per GPU with --weak)")
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--ebn0", type=float, default=1000.0, help=">= 100: noiseless")
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--weak", action="store_true",
                    help="every GPU demodulates its own --channels batch (default: C4's split)")
    ap.add_argument("--strong", action="store_true", help="(the default) split --channels across GPUs")
    ap.add_argument("--mode", choices=tuple(MODES), default="reference",
                    help="receiver semantics: reference parity (default); dec752 "
                         "(decimated_frame[752]), fft (kiss_fft hunt) or both: SURVEY.md 8f "
                         "rank 3 variants, not reference parity")
    ap.add_argument("--cpu-channels", type=int, default=4096,
                    help="channels of the bounded CPU-baseline sample (0: skip)")
    ap.add_argument("--verify", type=int, default=256,
                    help="channels checked against the oracle after timing (0: skip)")
    ap.add_argument("--stream-chunks", type=int, default=12,
                    help="chunks through the streaming-ingest pipeline after timing (0: skip)")
    ap.add_argument("--stream-frames", type=int, default=4, help="frames per stream chunk")
    ap.add_argument("--frame-latency", type=int, default=512,
                    help="frames of one synthetic channel timed through the per-frame drop-in "
                         "qpsk_rx_frame() (rank 0; 0: skip)")
    ap.add_argument("--sweep", action="store_true",
                    help="C5: AWGN Eb/N0 sweep (GPU vs the reference C on host cores)")
    ap.add_argument("--sweep-frames", type=int, default=16)
    ap.add_argument("--sweep-points", type=str, default="0,1,2,3,4,5,6,7,8,9,10")
    ap.add_argument("--cpu-procs", type=int, default=0,
                    help="host processes for the all-cores reference baseline and the sweep "
                         "(0: every CPU this job may use, host_cpus())")
    ap.add_argument("--cpu-all-channels", type=int, default=32768,
                    help="channels of the multi-core reference sample (0: skip)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher/sharding rehearsal: every rank forms the host group, takes "
                         "its shard and reduces a zero time, rank 0 prints the shards; no GPU use")
    return ap.parse_args(argv)


# ----------------------------------------------------------------- C5 sweep
_SM_K = 0x9E3779B97F4A7C15
_M64 = (1 << 64) - 1


def _sm64_next(s):
    """splitmix64 over a uint64 numpy array (wrapping), as qpsk_synth.c."""
    s = s + np.uint64(_SM_K)
    z = s.copy()
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return s, z ^ (z >> np.uint64(31))


def tx_frames(seed: int, c0: int, nch: int, nsamples: int):
    """TX data-frame bits of every channel, regenerated from the generator's RNG
    stream (include/qpsk_synth.h): uint64 [nch][nframes_tx] with bit 2s = Q,
    bit 2s+1 = I of data symbol s (the reference's bits[] order)."""
    with np.errstate(over="ignore"):
        c = np.arange(c0, c0 + nch, dtype=np.uint64)
        s = np.uint64(seed) ^ (c * np.uint64(_SM_K))
        s, z = _sm64_next(s)
        delay = (z % np.uint64(2783)).astype(np.int64)
        npk = int(np.max((nsamples - delay + 2782) // 2783)) + 1
        frames = np.zeros((nch, npk * 8), np.uint64)
        for f in range(npk * 8):
            w = np.zeros(nch, np.uint64)
            for i in range(31):
                s, z = _sm64_next(s)
                dib = z & np.uint64(3)
                w |= (dib & np.uint64(1)) << np.uint64(2 * i)           # Q
                w |= (dib >> np.uint64(1)) << np.uint64(2 * i + 1)      # I
            frames[:, f] = w
    return frames


def _pack62(bits):
    w = np.zeros(bits.shape[:-1], np.uint64)
    for k in range(62):
        w |= bits[..., k].astype(np.uint64) << np.uint64(k)
    return w


def _ref_name(mode: int) -> str:
    return ("unmodified reference (oracle/_ref, gcc -O2)" if mode == 0 else
            "unmodified reference sources, dec752 layout (oracle/_ref/libqpsk_ref752.so)")


def _ref_timed(args):
    """One host process of the all-cores baseline: regenerate its channels of
    the benchmark workload (oracle.synth == the bench generator) and time the
    unmodified reference over them, one channel after another."""
    import oracle
    seed, c0, n, nf, ebn0, mode = args
    x = oracle.synth(seed, n, nf, ebn0, c0=c0, threads=1)
    t = time.perf_counter()
    oracle.ref_rx(x, mode=mode)
    return n * nf * FRAME, time.perf_counter() - t


def _ref_chunk(args):
    import oracle
    x, = args
    b, v, _ = oracle.ref_rx(x)
    return b, v


def sweep(args):
    """C5 (BASELINE.json configs[4]): AWGN Eb/N0 sweep over the channel batch.
    Per point: GPU demod vs the unmodified reference C receiver on host cores
    (disagreements must be 0) and BER against the transmitted bits, taken as
    each valid frame's best match over that channel's TX data frames (the
    reference modem does not recover TX data, SURVEY.md 0.6: BER ~ chance)."""
    import multiprocessing as mp
    import oracle
    ctx = mp.get_context("spawn")
    pool = ctx.Pool(args.cpu_procs)   # before any GPU use
    import torch  # noqa: F401
    import singlecarrier_amd as sc
    nch, nf = args.channels, args.sweep_frames
    ks = oracle.keystream(32767 + 62 * nf + 64)
    ksw = np.array([int("".join(map(str, ks[62 * n:62 * n + 62][::-1])), 2) for n in range(nf)],
                   np.uint64)
    rows = []
    for eb in [float(v) for v in args.sweep_points.split(",")]:
        t0 = time.perf_counter()
        x = sc.synth_device(args.seed, nch, nf, eb).cpu().numpy()   # == host generator
        t_syn = time.perf_counter() - t0
        rx = sc.Receiver(nch)
        t0 = time.perf_counter()
        out = rx.demod(x)
        t_gpu = time.perf_counter() - t0
        rx.close()
        chunks = np.array_split(np.arange(nch), args.cpu_procs * 4)
        t0 = time.perf_counter()
        res = pool.map(_ref_chunk, [(np.ascontiguousarray(x[c]),) for c in chunks])
        t_cpu = time.perf_counter() - t0
        rbits = np.concatenate([r[0] for r in res])
        rvalid = np.concatenate([r[1] for r in res])
        dis_bits = int((out["bits"] != rbits).sum())
        dis_valid = int((out["valid"] != rvalid).sum())
        tx = tx_frames(args.seed, 0, nch, nf * FRAME)
        vm = out["valid"].astype(bool)
        w = _pack62(out["bits"])
        raw = w ^ ksw[None, :]            # before descrambling
        best = np.full(w.shape, 62, np.int64)
        best_raw = np.full(w.shape, 62, np.int64)
        best_ctl = np.full(w.shape, 62, np.int64)      # control: another channel's TX
        txo = np.roll(tx, 1, axis=0)
        for f in range(tx.shape[1]):
            best = np.minimum(best, np.bitwise_count(w ^ tx[:, f:f + 1]).astype(np.int64))
            best_raw = np.minimum(best_raw, np.bitwise_count(raw ^ tx[:, f:f + 1]).astype(np.int64))
            best_ctl = np.minimum(best_ctl, np.bitwise_count(w ^ txo[:, f:f + 1]).astype(np.int64))
        nvalid = int(vm.sum())
        row = {"ebn0_db": eb, "frames": int(nch * nf), "valid_frames": nvalid,
               "valid_frac": round(nvalid / (nch * nf), 4),
               "disagree_bits_vs_ref": dis_bits, "disagree_valid_vs_ref": dis_valid,
               "ber_best_tx_match": round(float(best[vm].mean()) / 62, 4) if nvalid else None,
               "ber_best_tx_match_raw": round(float(best_raw[vm].mean()) / 62, 4) if nvalid else None,
               "ber_control_other_channel": round(float(best_ctl[vm].mean()) / 62, 4) if nvalid else None,
               "gpu_s_incl_h2d": round(t_gpu, 3), "ref_cpu_s": round(t_cpu, 2),
               "ref_cpu_msamples_s": round(nch * nf * FRAME / t_cpu / 1e6, 1),
               "cpu_procs": args.cpu_procs, "synth_s": round(t_syn, 1)}
        rows.append(row)
        print(json.dumps(row), flush=True)
    pool.close()
    print(json.dumps({"sweep": "C5 AWGN Eb/N0", "channels": nch, "frames": nf,
                      "kernel_hash": sc.kernel_hash(), "reference": "unmodified reference C "
                      "(oracle/_ref, gcc -O2) on host cores",
                      "all_identical_to_reference": all(r["disagree_bits_vs_ref"] == 0 and
                                                       r["disagree_valid_vs_ref"] == 0
                                                       for r in rows)}), flush=True)


SAMPLE_MD5 = "b56a4d3609d0312934aaef69903c5298"   # reference output of preamble_qpsk_8k.raw


def frame_latency(nframes: int, seed: int) -> dict:
    """The per-frame drop-in (qpsk_rx_frame, src/qpsk.c:447's call), timed call
    by call from the host: the sample capture (its 496-byte records must give
    the reference output file) and a synthetic one-channel stream of `nframes`
    frames.  Each call is a full GPU round trip (H2D, two launches, D2H, sync):
    latency-bound, reported next to the reference's time per frame on one core."""
    import singlecarrier_amd as sc
    L = sc.lib()
    raw = np.fromfile(os.path.join(ROOT, "tests", "golden", "preamble_qpsk_8k.raw"), dtype="<i2")
    frames = raw[: len(raw) // FRAME * FRAME].reshape(-1, FRAME)
    L.qpsk_rx_init()
    recs = b""
    bits = np.zeros(496, np.uint8)
    for fr in frames:
        bits[:] = 0
        if L.qpsk_rx_frame(fr.ctypes.data, bits.ctypes.data):
            recs += bits.tobytes()
    import hashlib
    sample_ok = hashlib.md5(recs).hexdigest() == SAMPLE_MD5 and L.qpsk_surface_error() == 0
    x = np.ascontiguousarray(sc.synth(seed, 1, nframes)[0])
    L.qpsk_rx_init()
    for fr in x[:8]:                         # untimed: first-call allocations
        L.qpsk_rx_frame(fr.ctypes.data, bits.ctypes.data)
    L.qpsk_rx_init()
    us = np.empty(nframes)
    nvalid = 0
    for i, fr in enumerate(x):
        t = time.perf_counter_ns()
        nvalid += L.qpsk_rx_frame(fr.ctypes.data, bits.ctypes.data)
        us[i] = (time.perf_counter_ns() - t) / 1e3
    if L.qpsk_surface_error() != 0:
        raise sc.QpskError(f"qpsk_rx_frame failed: {L.qpsk_surface_error()}")
    return {"p50_us": round(float(np.percentile(us, 50)), 1),
            "p99_us": round(float(np.percentile(us, 99)), 1),
            "mean_us": round(float(us.mean()), 1), "frames": nframes, "valid_frames": nvalid,
            "sample_file_md5_ok": bool(sample_ok),
            "what": "qpsk_rx_frame() per call, host wall time, one synthetic channel "
                    "(include/qpsk_internal.h, one-channel context on device 0)"}


def pmc_record(name: str, nch: int, nf: int, mode: str, khash: str, root: str = ROOT):
    """A committed rocprofv3 counter record (profiles/pmc_traffic.json or
    pmc_valu.json, written by profiles/summarize.py) when it describes THIS
    workload and THIS build: same channels/frames/mode and the same
    qpsk_kernel_hash() as the running library (the hash of the kernels'
    sources and build rules).  Counters of another build are never reported."""
    path = os.path.join(root, "profiles", name)
    if not os.path.exists(path):
        return None
    p = json.load(open(path))
    if p.get("channels") != nch or p.get("frames") != nf or p.get("mode", "reference") != mode:
        return None
    if not khash or p.get("kernel_hash") != khash:
        return None
    return p


def valu_from_counters(p, t_launch: float):
    """VALU issue rate of rx_kernel + rx_data_kernel from MEASURED counters:
    SQ_INSTS_VALU (wave-instructions, every pass summed over the chip) per
    launch, from the rocprofv3 --pmc pass of this build (pmc_record), over the
    kernel time measured live here.  Peak: one wave64 VALU instruction per
    SIMD-32 per 2 cycles (MI355X_MICROARCH.md "Wave scheduling"), 1,024 SIMDs at
    2.4 GHz = 1.229e12 wave-instr/s; packed fp32 (v_pk_*) measured at 3.47
    cycles per wave-instruction per SIMD with two waves per SIMD
    (profiles/calib/valu_rate_r01.txt), i.e. 0.708e12 wave-instr/s."""
    if p is None:
        return None
    insts = p["valu_insts_per_launch"]
    peak = VALU_SIMDS * VALU_CLOCK_GHZ * 1e9 / 2.0
    peak_pk = VALU_SIMDS * VALU_CLOCK_GHZ * 1e9 / 3.47
    ach = insts / t_launch
    out = {"valu_insts_per_launch": insts, "achieved_winst_s": round(ach / 1e12, 4),
           "peak_winst_s": round(peak / 1e12, 4), "frac": round(ach / peak, 4),
           "packed_peak_winst_s": round(peak_pk / 1e12, 4), "frac_packed": round(ach / peak_pk, 4),
           "unit": "1e12 wave64 VALU instructions/s", "source": p.get("source"),
           "kernel_hash": p.get("kernel_hash")}
    if p.get("active_valu_frac") is not None:
        out["sq_active_inst_valu_per_wave_cycle"] = p["active_valu_frac"]
    if p.get("clock_ghz") is not None:
        out["clock_ghz_under_profiler"] = p["clock_ghz"]
    return out


def dry_run(args, world: int, rank: int, local: int, strong: bool) -> None:
    """The multi-rank path up to the first GPU call: host group, shard,
    timing reduction, gather of the per-rank records; rank 0 prints one JSON
    line.  Lets a CPU test run `bench.py --gpus N --dry-run` end to end."""
    dist = init_host_group(rank, world) if world > 1 else None
    nch, c0 = shard(args.channels, world, rank, strong)
    tmax, total = reduce_step(dist, 0.001 * (rank + 1), nch)
    rec = {"rank": rank, "local_rank": local, "channels": [c0, c0 + nch]}
    recs = [rec]
    if dist:
        recs = [None] * world
        dist.all_gather_object(recs, rec)
    if rank == 0:
        print(json.dumps({"dry_run": True, "world": world, "channels_total": total,
                          "max_time_s": tmax, "shards": recs,
                          "scaling": "strong" if strong else "weak"}), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def main():
    args = parse()
    if args.cpu_procs <= 0:
        args.cpu_procs = host_cpus()
    if args.sweep:
        return sweep(args)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # one process per GPU, started before this process touches HIP
        sys.exit(launch(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    strong = not args.weak
    if args.dry_run:
        return dry_run(args, world, rank, local, strong)
    pool = None
    if rank == 0 and args.cpu_all_channels > 0 and args.cpu_procs > 1:
        import multiprocessing as mp
        import oracle
        if oracle.ref_available(MODES[args.mode]):
            pool = mp.get_context("spawn").Pool(args.cpu_procs)   # before any GPU use

    dist = None
    if world > 1:
        # host-side group: the timing barrier and the reductions only (the
        # data path has no collective)
        dist = init_host_group(rank, world)

    import torch
    import singlecarrier_amd as sc

    # one GPU per rank; ranks beyond the visible devices share them (only a
    # launcher rehearsal on a one-GPU box does that: its timing means nothing)
    ndev = torch.cuda.device_count()
    local = local % ndev if ndev > 0 else local
    torch.cuda.set_device(local)
    nch, c0 = shard(args.channels, world, rank, strong)
    nf = args.frames

    # input: generated on the GPU (qpsk_synth_device == the oracle's generator,
    # tests/test_gpu_synth.py), resident in HBM before timing
    t = time.perf_counter()
    x = sc.synth_device(args.seed, nch, nf, args.ebn0, c0=c0, device=local)
    torch.cuda.synchronize()
    t_synth = time.perf_counter() - t
    # PCIe-inclusive reference point (never `value`), rank 0 only: the same
    # batch copied in from pageable host memory.  Other ranks keep only the
    # channels they verify.
    x_host, t_h2d = None, None
    if rank == 0:
        x_host = x.cpu().numpy()
        t = time.perf_counter()
        x2 = torch.from_numpy(x_host).to(x.device)
        torch.cuda.synchronize()
        t_h2d = time.perf_counter() - t
        del x2
    elif args.verify:
        x_host = x[:min(args.verify, nch)].cpu().numpy()
    bits = torch.empty((nch, nf, 62), dtype=torch.uint8, device=x.device)
    valid = torch.empty((nch, nf), dtype=torch.uint8, device=x.device)
    mode = MODES[args.mode]
    rx = sc.Receiver(nch, device=local, mode=mode)

    for _ in range(args.warmup):
        rx.demod_device(x, bits, valid)
    rx.sync()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    rx.timing(True)
    rx.collect_timing()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        rx.demod_device(x, bits, valid)
    ev1.record()
    torch.cuda.synchronize()
    # this rank's time ends when its GPU is done; the closing barrier stays
    # outside it (a gloo round trip is ~0.1-1 ms, a step at N = 8 ~1.5 ms),
    # and the MAX over ranks below is the slowest GPU
    wall = time.perf_counter() - t0
    if dist:
        dist.barrier()
    rx.sync()   # a device-side failure of any timed call raises here
    rx_ms, data_ms, kern_frames = rx.collect_timing_split()
    kern_ms = rx_ms + data_ms
    rx.timing(False)
    region_ms = ev0.elapsed_time(ev1)

    tmax, total_ch = reduce_step(dist, wall, nch)
    samples = float(total_ch) * nf * FRAME * args.steps
    value = samples / tmax / 1e6

    # roofline of the path's kernels per step: rx_kernel (one persistent launch,
    # all `frames` frames of all channels; dominant) + rx_data_kernel (data
    # symbols of the valid frames).  Durations from HIP events on their stream;
    # the algorithmic bytes of the step are divided by the SUM of both.
    t_launch = kern_ms / 1e3 / args.steps
    alg_bytes = nch * nf * ALG_BYTES_PER_FRAME
    achieved = alg_bytes / t_launch / 1e9
    roofline = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                "kernel": "rx_kernel + rx_data_kernel", "launch_us": round(t_launch * 1e6, 2),
                "kernels_us": {"rx_kernel": round(rx_ms / args.steps * 1e3, 2),
                               "rx_data_kernel": round(data_ms / args.steps * 1e3, 2)},
                "alg_bytes_per_launch": alg_bytes}
    khash = sc.kernel_hash()
    roofline["kernel_hash"] = khash
    p = pmc_record("pmc_traffic.json", nch, nf, args.mode, khash)
    if p is not None:
        roofline["traffic"] = p["hbm_bytes_per_launch"]
        roofline["traffic_source"] = p.get("source")
    valu = valu_from_counters(pmc_record("pmc_valu.json", nch, nf, args.mode, khash), t_launch)
    # the minimal bit-exact formulation is ~96 fp32 ops per
    # sample, 8.2e11 samples/s per GPU at 78.6e12 non-FMA packed ops/s
    bound = {"samples_s_per_gpu": 8.2e11, "source": "SURVEY.md 8d (96 ops/sample minimal form)",
             "frac": round(nch * nf * FRAME / t_launch / 8.2e11, 4)}
    if valu is None:
        valu = {}
    valu["survey_minimal_form_bound"] = bound

    # parity spot check of the timed outputs on every rank (checker only; not
    # timed): the first k channels of the rank's shard
    verified = None
    if args.verify:
        import oracle
        k = min(args.verify, nch)
        # the timed context advanced (warmup + steps) batches of the same
        # input: the oracle replays that whole stream for the first k channels
        reps = args.warmup + args.steps
        exp_bits, exp_valid, _ = oracle.cpu_rx(np.concatenate([x_host[:k]] * reps, axis=1),
                                               mode=mode)
        same_input = bool((oracle.synth(args.seed, k, nf, args.ebn0, c0=c0) == x_host[:k]).all())
        ok = bool(same_input and (bits[:k].cpu().numpy() == exp_bits[:, -nf:]).all()
                  and (valid[:k].cpu().numpy() == exp_valid[:, -nf:]).all())
        verified = {"rank": rank, "channels": [c0, c0 + k], "ok": ok}
    per_rank = [verified]
    if dist:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, verified)

    # streaming ingest (include/qpsk_stream.h): host chunks through pinned slots,
    # H2D / receive / D2H overlapped.  PCIe-inclusive; reported, never `value`.
    stream = None
    if args.stream_chunks > 0 and rank == 0 and mode == sc.MODE_REFERENCE:
        fpc = min(args.stream_frames, nf)
        st = sc.Stream(nch, fpc, nslot=3, device=local)
        for _ in range(3):   # untimed: fill every slot's pinned buffer once
            st.acquire()[...] = x_host[:, :fpc]
            st.submit()
        while st.pending:
            st.retrieve(copy=False)
        t = time.perf_counter()
        for _ in range(args.stream_chunks):
            if st.pending == 3:
                st.retrieve(copy=False)
            st.acquire()
            st.submit()
        while st.pending:
            st.retrieve(copy=False)
        dt = time.perf_counter() - t
        st.close()
        ns = nch * fpc * FRAME * args.stream_chunks
        stream = {"msamples_s": round(ns / dt / 1e6, 1), "input_gb_s": round(2 * ns / dt / 1e9, 2),
                  "chunk": f"{nch} channels x {fpc} frames", "chunks": args.stream_chunks,
                  "slots": 3}

    drop_in = None
    if args.frame_latency > 0 and rank == 0 and mode == sc.MODE_REFERENCE:
        drop_in = frame_latency(args.frame_latency, args.seed)

    # CPU baselines, rank 0, after the timed region (the other ranks wait at
    # the final barrier): the C3 workload's channels 0.. regenerated on the host
    cpu = cpu_all = None
    host = cpu_info()
    if rank == 0 and args.cpu_channels > 0:
        import oracle
        k = min(args.cpu_channels, nch)
        sample = x_host[:k] if c0 == 0 else oracle.synth(args.seed, k, nf, args.ebn0)
        if oracle.ref_available(mode):
            t = time.perf_counter()
            oracle.ref_rx(sample, mode=mode)
            dt = time.perf_counter() - t
            cpu = {"value": round(k * nf * FRAME / dt / 1e6, 3), "unit": "Msamples/s",
                   "cores": 1, "kind": "reference",
                   "sample": f"channels 0..{k - 1} of the {args.channels}-channel batch x {nf} "
                             f"frames, {_ref_name(mode)}, one channel after another, {dt:.1f} s",
                   **host}
        else:
            t = time.perf_counter()
            oracle.cpu_rx(sample, threads=1, mode=mode)
            dt = time.perf_counter() - t
            cpu = {"value": round(k * nf * FRAME / dt / 1e6, 3), "unit": "Msamples/s",
                   "cores": 1, "kind": "port",
                   "sample": f"{k} channels x {nf} frames, oracle/cpu_ref.c, 1 thread, {dt:.1f} s",
                   **host}
    if pool is not None:
        k = min(args.cpu_all_channels, args.channels)
        bounds = np.linspace(0, k, args.cpu_procs + 1).astype(int)
        jobs = [(args.seed, int(a), int(b - a), nf, args.ebn0, mode)
                for a, b in zip(bounds[:-1], bounds[1:]) if b > a]
        res = pool.map(_ref_timed, jobs)
        pool.close()
        tot = sum(r[0] for r in res)
        tmx = max(r[1] for r in res)
        cpu_all = {"value": round(tot / tmx / 1e6, 3), "unit": "Msamples/s",
                   "cores": len(jobs), "kind": "reference",
                   "sample": f"channels 0..{k - 1} of the {args.channels}-channel batch x {nf} "
                             f"frames, {_ref_name(mode)}, {len(jobs)} host processes (every CPU "
                             f"this job may use: affinity {host['affinity_cpus']}, cgroup quota "
                             f"{host['cgroup_cpu_quota']}), slowest {tmx:.1f} s", **host}

    if drop_in is not None and cpu is not None:
        # the CPU receiver's time per frame on one core, from the baseline just
        # timed, under the name of what was timed: the unmodified reference, or
        # (reference not built) the oracle's port
        key = "reference_us_per_frame" if cpu["kind"] == "reference" else "port_us_per_frame"
        drop_in[key] = round(FRAME / cpu["value"], 1)
    if rank == 0:
        ch_total = total_ch
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "Msamples/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(tmax / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "strong" if strong else "weak", "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic, generated on the GPU: reference TX packets, splitmix64 dibits, "
                    "per-channel delay"
                    + ("" if args.ebn0 >= 100 else f", AWGN Eb/N0 {args.ebn0} dB"),
            "config": {"workload": (f"{ch_total} channels x {nf} frames x 1880 samples"
                                    + (f", {world} channel shards of {nch}" if world > 1 and strong
                                       else f" ({nch} per GPU)" if world > 1 else "")
                                    + (" (C4)" if world > 1 and strong
                                       else " (C3)" if ch_total == 65536 and nf == 32 else "")),
                       "channels_per_gpu": nch, "channels_total": ch_total, "frames": nf,
                       "samples_per_step": int(ch_total * nf * FRAME),
                       "parallelism": f"{world} channel shard(s), one process per GPU, no "
                                      f"collective (host gloo barrier/time reduction)",
                       "mode": args.mode},
            "roofline": roofline, "valu": valu, "cpu_baseline": cpu,
            "cpu_baseline_all_cores": cpu_all,
            "rank0_region_ms_per_step": round(region_ms / args.steps, 3),
            "synth_s": round(t_synth, 2), "h2d_s": round(t_h2d, 2),
            "h2d_incl_msamples_s": round(nch * nf * FRAME / (t_h2d + tmax / args.steps) / 1e6, 1),
            "stream_pcie_note": "rank 0 only, after the timed region",
            "verified_vs_oracle": all(v is not None and v["ok"] for v in per_rank) if args.verify else None,
            "verified_per_rank": per_rank if args.verify else None,
            "stream_pcie": stream,
            "drop_in_frame_latency": drop_in,
            "gpus_visible": ndev,
            "shared_gpus": world > ndev,   # a launcher rehearsal: not a scaling figure
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
    rx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
