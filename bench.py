"""Benchmark: device-resident batched CRC32C (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config NAME]

Configs (BASELINE.json "configs"; the default line is the headline):
  headline        10,000 x 4 KiB blocks per GPU per step (the metric's
                  workload); the line also carries `split`, config 5 measured
                  in the same run.
  blocks1m_split  config 5: ONE batch of 1M x 4 KiB blocks split across the
                  ranks (shard.shard_range), aggregate GiB/s.
  blocks1m        config 4: 1M x 4 KiB blocks per GPU per step.
  wal32k          config 3: 16,384 x 32 KiB WAL blocks, CRC over [6, 32768)
                  (the engine's general walk, lvkv_ek_ragged).

One step = one batch submitted to the AQL engine (lvkv_engine_crc32c_uniform,
include/lvkv_crc32c.h) over blocks already resident in HBM. Consecutive steps
read different windows of a >= 1.25 GiB rotation, so every batch is cold in
the 256 MiB Infinity Cache; consecutive batches overlap on the device (the
engine's queues), as in a checksum service with batches in flight.

Ranks: one process per GPU. Under torch.distributed.run (WORLD_SIZE set) the
launcher's ranks are used and must number --gpus; `python bench.py --gpus N`
without a launcher starts the N ranks itself (a torch.distributed.run child
process, before any GPU call). Config 5 below 1 GiB per slice keeps several
copies of the slice per rank and rotates over them (MALL-cold every step).

Timed region (every config, every rank; `timed_region`): time-based warm-up
(>= --warmup-ms and >= W steps), barrier, synchronize, t0, K steps, engine
wait, synchronize, t1, barrier; elapsed = max over ranks of t1 - t0 (common
start to last completion). value = all ranks' bytes / elapsed.

roofline: algorithmic bytes per launch (nblocks x (block + 4 B CRC out),
SURVEY.md §8(d)) / the launch's duration, from the packet processor's
start/end timestamps of each dispatch (HSA profiling, the engine's HIP-event
counterpart): `achieved` prices a launch running alone (ordered dispatches,
the same kernel a rocprofv3 kernel trace of `--isolated` times); `pipelined`
prices the device span of K overlapped launches / K. `traffic`: HBM-side
bytes per isolated launch from a rocprofv3 FETCH_SIZE pass over this run's
own code (a child profiler process, N = 1 headline only; --no-pmc skips it).
cpu_baseline: the reference's util/crc32c.cc (compiled in place into
oracle/_ref) on this host.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
GIB = float(1 << 30)
BLOCK = 4096
SPLIT_TOTAL = 1_000_000
METRIC = "device-resident CRC32C GiB/s over 10k×4KiB blocks; % of MI355X HBM peak"
# each config's own line names its own workload (the headline's is BASELINE.json's)
METRICS = {
    "headline": METRIC,
    "blocks1m": "device-resident CRC32C GiB/s over 1M×4KiB blocks per GPU (config 4); "
                "% of MI355X HBM peak",
    "blocks1m_split": "device-resident CRC32C GiB/s over 1M×4KiB blocks split across the GPUs "
                      "(config 5), aggregate; % of MI355X HBM peak per GPU",
    "wal32k": "device-resident CRC32C GiB/s over 16384×32KiB WAL blocks, CRC over [6, 32768) "
              "(config 3); % of MI355X HBM peak",
}

CONFIGS = {
    # name: (nblocks, block_bytes, stride, crc_offset_in_block, description)
    "headline": (10_000, 4096, 4096, 0, "10k x 4 KiB blocks per GPU per step (BASELINE headline)"),
    "blocks1m": (1_000_000, 4096, 4096, 0, "1M x 4 KiB blocks per GPU per step (config 4)"),
    "blocks1m_split": (SPLIT_TOTAL, 4096, 4096, 0,
                       "1M x 4 KiB blocks split across the ranks (config 5)"),
    "wal32k": (16_384, 32762, 32768, 6, "16384 x 32 KiB WAL blocks, CRC over [6, 32768) (config 3)"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


def _load_shard():
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "lvkv_shard", REPO / "leveldb-kv-separation_amd" / "shard.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


# --------------------------------------------------------------------------
# the timed region (shared by every config and by tests/test_dist.py)


class Comm:
    """Barrier and max-over-ranks on the process group (RCCL on the GPU box,
    gloo in the CPU tests); no-ops at world 1. `device` is where the max's
    one-element tensor lives: the rank's GPU under RCCL, None (host) under
    gloo."""

    def __init__(self, world: int, device=None):
        self.world = world
        self.device = device

    def barrier(self):
        if self.world > 1:
            import torch.distributed as dist
            dist.barrier()

    def gather(self, obj):
        """Every rank's `obj`, in rank order (all_gather_object; [obj] at world 1)."""
        if self.world == 1:
            return [obj]
        import torch.distributed as dist
        out = [None] * self.world
        dist.all_gather_object(out, obj)
        return out

    def max(self, x: float) -> float:
        if self.world == 1:
            return x
        import torch
        import torch.distributed as dist
        t = torch.tensor([x], dtype=torch.float64, device=self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())


def timed_region(runner, comm: Comm, steps: int, warmup: int, warmup_s: float,
                 first: int = 0):
    """Warm-up (>= warmup steps and >= warmup_s seconds), then K steps timed
    from a common start (barrier + sync) to this rank's last completion
    (finish + sync); returns (max over ranks in seconds, next step index).
    `runner` has step(i), finish() and sync(). Step indices continue from `first` so the
    timed steps read windows the warm-up did not just leave in the cache."""
    i = first
    t_end = time.perf_counter() + warmup_s
    n = 0
    while n < warmup or time.perf_counter() < t_end:
        runner.step(i)
        i += 1
        n += 1
        if n % 16 == 0:
            runner.finish()
    runner.finish()
    runner.sync()
    comm.barrier()
    runner.sync()
    t0 = time.perf_counter()
    fw = getattr(runner, "final_window", 0)
    for k in range(steps):
        if k >= steps - fw:
            runner.step(i + k, final=True)
        else:
            runner.step(i + k)
    runner.finish()
    runner.sync()
    elapsed = time.perf_counter() - t0
    comm.barrier()
    return comm.max(elapsed), i + steps


def split_measure(make_runner, comm: Comm, rank: int, world: int, steps: int, warmup: int,
                  warmup_s: float, total: int = SPLIT_TOTAL, block: int = BLOCK):
    """Config 5: one batch of `total` blocks split into contiguous slices, one
    per rank (shard.shard_range, no collective on the data path); every step
    checksums the rank's whole slice. Returns the runner and the aggregate
    record (GiB/s of the whole batch over the max-over-ranks time)."""
    shard = _load_shard()
    start, count = shard.shard_range(total, rank, world)
    runner = make_runner(start, count)
    elapsed, _ = timed_region(runner, comm, steps, warmup, warmup_s)
    value = total * block * steps / elapsed / GIB
    # every rank's slice and how many of its blocks were checked against the
    # oracle (the whole slice, before the timed region)
    slices = comm.gather({"rank": rank, "start": start, "blocks": count,
                          "parity_blocks": getattr(runner, "parity_blocks", None)})
    rec = {"workload": CONFIGS["blocks1m_split"][4], "total_blocks": total,
           "block_bytes": block, "ranks": world, "slice_blocks_rank0": shard.shard_range(total, 0, world)[1],
           "slice_copies": getattr(runner, "nrot", 1),
           "steps": steps, "ms_per_step": round(elapsed / steps * 1e3, 5),
           "value": round(value, 4), "unit": "GiB/s",
           "pct_hbm_peak_per_gpu": round(100.0 * value * GIB / 1e9 / HBM_PEAK_GBS / world, 2),
           "timing": "common start barrier to the last rank's completion (max over ranks)",
           "slices": slices}
    return runner, rec


# --------------------------------------------------------------------------
# GPU runners


class EngineRunner:
    """Steps through the AQL engine over rotating HBM windows."""

    def __init__(self, lvkv, eng, buf, nb, L, stride, crc_off, nrot, window, outs):
        import torch
        self.torch = torch
        self.eng = eng
        self.submit = eng.submit_ptr
        self.h = eng.handle
        self.nb, self.L, self.stride = nb, L, stride
        self.bases = [buf.data_ptr() + w * window + crc_off for w in range(nrot)]
        self.outs = [o.data_ptr() for o in outs]
        self.outs_t = outs
        self.nrot = nrot
        self.flags = 0
        # the engine does not follow HIP streams: the kernels that wrote the
        # blocks (torch.randint) must be complete before the first submit
        torch.cuda.synchronize()

    # the last submits before a wait, one per queue, carry LVKV_FLAG_FINAL
    # (their completion releases the results, so the wait needs no barrier
    # packets); the engine's default is three queues
    final_window = 3

    def step(self, i, final=False):
        rc = self.submit(self.h, self.bases[i % self.nrot], self.stride, self.L, 0,
                         self.outs[i % len(self.outs)], self.nb,
                         self.flags | (8 if final else 0))  # LVKV_FLAG_FINAL
        if rc != 0:
            raise SystemExit(f"bench: lvkv_engine_crc32c_uniform failed ({rc})")

    def finish(self):
        self.eng.wait()

    def sync(self):
        self.torch.cuda.synchronize()


def make_buffers(torch, dev, rank, nb, stride, rotate_bytes, extra=64):
    window = nb * stride
    nrot = max(1, int(np.ceil(rotate_bytes / window)))
    gen = torch.Generator(device=dev).manual_seed(0x1EDC6F41 + 17 * rank)
    buf = torch.randint(0, 256, (nrot * window + extra,), dtype=torch.uint8, device=dev,
                        generator=gen)
    return buf, nrot, window


def parity_check(buf, outs0, nb, L, stride, crc_off, rank, what, chunk=1 << 18):
    """Every block of the batch (a rank's whole slice) against the oracle
    (checker), once, outside the timed region; in chunks of `chunk` blocks so
    the host copy stays bounded."""
    sys.path.insert(0, str(REPO / "oracle"))
    import oracle
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    got_all = outs0[:nb].cpu().numpy().view(np.uint32)
    for b0 in range(0, nb, chunk):
        n = min(chunk, nb - b0)
        lo = crc_off + b0 * stride
        host = buf[lo: lo + (n - 1) * stride + L].cpu().numpy()
        want = oracle.uniform(host, n, L, stride, threads=threads)
        if not np.array_equal(got_all[b0:b0 + n], want):
            bad = int(np.flatnonzero(got_all[b0:b0 + n] != want)[0]) + b0
            raise SystemExit(f"bench: parity check FAILED on rank {rank} ({what}): "
                             f"block {bad} of {nb}")
    return nb


def profile_launches(runner, eng, n, ordered, first):
    """Packet-processor start/end of n dispatches (HSA profiling)."""
    runner.flags = 2 if ordered else 0  # LVKV_FLAG_ORDERED
    eng.profile(True)
    for k in range(n):
        runner.step(first + k)
    eng.wait()
    spans = eng.profile_read(4096)
    eng.profile(False)
    runner.flags = 0
    return spans


# --------------------------------------------------------------------------
# CPU baseline (rank 0, N = 1)


def cpu_baseline(seconds: float = 8.0):
    """The reference's util/crc32c.cc (oracle/_ref, kind 'reference'), or the
    oracle restatement (kind 'port') if the reference build is absent, on a
    bounded sample of the headline workload."""
    sys.path.insert(0, str(REPO / "oracle"))
    import oracle  # checker / baseline only

    nb, L = 10_000, 4096
    data = oracle.splitmix_bytes(0x1EDC6F41, nb * L)
    if oracle.reference_available():
        ref = oracle.Reference()
        fn = lambda: ref.uniform(data, nb, L, threads=1)  # noqa: E731
        kind = "reference"
    else:
        fn = lambda: oracle.uniform(data, nb, L, threads=1)  # noqa: E731
        kind = "port"

    def best_of(f, secs):
        f()
        best, t_end, passes = float("inf"), time.perf_counter() + secs, 0
        while time.perf_counter() < t_end or passes < 3:
            t0 = time.perf_counter()
            f()
            best = min(best, time.perf_counter() - t0)
            passes += 1
        return nb * L / best / GIB, passes

    gibs, passes = best_of(fn, seconds)
    # Static contiguous partition over the host threads this job may use
    # (SURVEY.md §8(d)); the box grants 16 CPUs to one GPU.
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    if kind == "reference":
        fn_mt = lambda: ref.uniform(data, nb, L, threads=threads)  # noqa: E731
    else:
        fn_mt = lambda: oracle.uniform(data, nb, L, threads=threads)  # noqa: E731
    gibs_mt, passes_mt = best_of(fn_mt, max(1.0, seconds / 4))
    return {"value": round(gibs, 3), "unit": "GiB/s", "cores": 1, "kind": kind,
            "sample": f"{nb} x {L} B splitmix64 blocks, 1 thread, best of {passes} passes "
                      f"over {seconds:.0f} s (util/crc32c.cc -O3 -DNDEBUG)",
            "multi_thread": {"value": round(gibs_mt, 3), "cores": threads,
                             "passes": passes_mt},
            "cpu_model": _cpu_model()}


def _cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def live_pmc_traffic(launches: int = 16, timeout_s: float = 90.0):
    """HBM-side bytes per launch of the roofline kernel, measured for the code
    being benched: a child `rocprofv3 --pmc FETCH_SIZE -- python3 bench.py
    --isolated N` (the profiler starts its own process; this one never
    execs), FETCH_SIZE per dispatch of lvkv_ek_uniform_pair, median, KiB x
    1024 x 2 (gfx950 counts a wide streaming read's bytes at half, per the
    MI355X guide). None when the profiler is absent or the pass fails."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None
    out = tempfile.mkdtemp(prefix="lvkv_pmc_", dir="/tmp")
    cmd = [prof, "--pmc", "FETCH_SIZE", "--output-format", "csv", "-d", out, "-o", "run", "--",
           sys.executable, str(REPO / "bench.py"), "--isolated", str(launches), "--gpus", "1"]
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    env["TMPDIR"] = "/tmp"
    try:
        subprocess.run(cmd, cwd="/tmp", env=env, timeout=timeout_s, capture_output=True, check=True)
        vals = []
        for f in glob.glob(out + "/**/run_counter_collection.csv", recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    if "lvkv_ek_uniform_pair" in r.get("Kernel_Name", "") and \
                            r.get("Counter_Name") == "FETCH_SIZE":
                        vals.append(float(r["Counter_Value"]))
        if not vals:
            return None
        return {"bytes": int(statistics.median(vals) * 1024 * 2), "dispatches": len(vals),
                "source": f"rocprofv3 --pmc FETCH_SIZE over {len(vals)} isolated launches of "
                          "this run's code (KiB x 1024 x 2, gfx950 half-count)"}
    except (subprocess.SubprocessError, OSError, ValueError, KeyError):
        return None
    finally:
        shutil.rmtree(out, ignore_errors=True)


# --------------------------------------------------------------------------


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--warmup-ms", type=float, default=150.0,
                    help="warm-up lasts at least this long, whatever --warmup says")
    ap.add_argument("--config", default="headline", choices=sorted(CONFIGS))
    ap.add_argument("--rotate-bytes", type=float, default=1.25 * GIB)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-split", action="store_true", help="skip config 5 in the headline line")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the rocprofv3 FETCH_SIZE pass behind roofline.traffic")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--ceiling-trace", type=int, default=0,
                    help="only run K launches of the production and read-ceiling kernels "
                         "(the command a rocprofv3 kernel trace of the ceiling wraps)")
    ap.add_argument("--no-ceiling", action="store_true",
                    help="skip the read-only ceiling kernels behind roofline.ceiling")
    ap.add_argument("--isolated", type=int, default=0,
                    help="only run N ordered (one-at-a-time) launches and exit: the "
                         "command a rocprofv3 kernel trace of the roofline kernel wraps")
    ap.add_argument("--split-total", type=int, default=SPLIT_TOTAL,
                    help="blocks of the config-5 batch (1M; smaller only for plumbing tests)")
    ap.add_argument("--plumbing-cpu", action="store_true",
                    help="test only: gloo process group and the library's per-call CPU "
                         "CRC in place of the device (no GPU touched); exercises the "
                         "--gpus launch, the slicing and the timed region")
    args = ap.parse_args()

    # --gpus N > 1 outside a launcher: start one rank per GPU here, before
    # anything touches the GPU, as a child torch.distributed.run (never an
    # exec), and exit with its status.
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(_launch_ranks(args.gpus))
    world, rank, local = dist_env()
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but the launcher started {world} rank(s)")

    import torch
    warm_s = args.warmup_ms / 1e3
    import __graft_entry__ as g
    lvkv = g.load_package()

    if args.plumbing_cpu:
        _plumbing_cpu(args, lvkv, world, rank, warm_s)
        return

    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
    comm = Comm(world, dev)

    if args.config == "blocks1m_split":
        eng = lvkv.Engine(local)
        runner, rec = split_measure(
            lambda s, c: _split_runner(torch, lvkv, eng, dev, rank, s, c), comm, rank, world,
            args.steps, args.warmup, warm_s, total=args.split_total)
        if rank == 0:
            line = _line_base(args, world, rec["value"], rec["ms_per_step"] / 1e3,
                              {"workload": rec["workload"], "total_blocks": args.split_total,
                               "block_bytes": BLOCK,
                               "parallelism": f"{world} contiguous slices (no collective)"})
            line["split"] = rec
            print(json.dumps(line), flush=True)
        _end(world)
        return

    nb, L, stride, crc_off, desc = CONFIGS[args.config]
    # every config runs on the AQL engine: the burst kernel for the 4 KiB
    # blocks, the general walk (lvkv_ek_ragged) for config 3's 32 KiB blocks
    burst = L <= 16 * 256 and stride % 4 == 0 and (crc_off + L) % 4 == 0
    buf, nrot, window = make_buffers(torch, dev, rank, nb, stride, args.rotate_bytes)
    outs = [torch.empty(nb, dtype=torch.int32, device=dev) for _ in range(4)]
    eng = lvkv.Engine(local)
    runner = EngineRunner(lvkv, eng, buf, nb, L, stride, crc_off, nrot, window, outs)
    runner.step(0)
    runner.finish()
    runner.sync()
    checked = parity_check(buf, outs[0], nb, L, stride, crc_off, rank, args.config)

    if args.isolated:
        runner.flags = 2
        for k in range(args.isolated):
            runner.step(1 + k)
        eng.wait()
        return
    if args.ceiling_trace:
        _ceiling_trace(torch, lvkv, eng, runner, dev, rank, args.ceiling_trace)
        return

    elapsed, nxt = timed_region(runner, comm, args.steps, args.warmup, warm_s, first=1)
    ms_per_step = elapsed / args.steps * 1e3
    value = world * nb * L * args.steps / elapsed / GIB
    algo_bytes = nb * (L + 4)

    # every rank prices its own launches (its own GPU's packet-processor times)
    roof = {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": None, "traffic": None, "algo_bytes_per_launch": algo_bytes}
    # one launch alone (ordered: the engine drains, then the whole-chip kernel)
    iso = profile_launches(runner, eng, 64, True, nxt)
    # a batch beyond one dispatch's capacity is several dispatches: its
    # duration is first start to last end of its group
    per = max(1, len(iso) // 64)
    d = [iso[i + per - 1][1] - iso[i][0] for i in range(0, per * 64, per)]
    kern_us = statistics.mean(d)
    achieved = algo_bytes / (kern_us * 1e-6) / 1e9
    # K overlapped launches: device span (first start -> last end) / K
    runner.step(nxt + 64)
    eng.wait()
    pipe = profile_launches(runner, eng, args.steps, False, nxt + 65)
    nxt += 65 + args.steps
    span = (max(b for _, b in pipe) - min(a for a, _ in pipe)) / args.steps
    w, c, gr = eng.shape()
    roof.update({
        "achieved": round(achieved, 1), "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": None,
        "kernel": ("lvkv_ek_uniform_pair (ordered launch, 2 workgroups x 8 waves per CU)"
                   if burst else
                   "lvkv_ek_ragged (ordered launch, 2 workgroups x 8 waves x 2 chains per CU)"),
        "kernel_us_avg": round(kern_us, 3), "kernel_us_median": round(statistics.median(d), 3),
        "kernel_us_min": round(min(d), 3), "launches": len(d), "dispatches_per_launch": per,
        "timing": "HSA packet-processor start/end per dispatch (engine profiling)",
        "pipelined": {"kernel": (f"lvkv_ek_uniform ({w} waves x {c} chains, {gr} workgroups, "
                                 f"{eng.queues()} queues)" if burst else
                                 f"lvkv_ek_ragged ({eng.queues()} queues)"),
                      "launches": args.steps, "dispatches": len(pipe),
                      "period_us": round(span, 3),
                      "achieved": round(algo_bytes / (span * 1e-6) / 1e9, 1),
                      "frac": round(algo_bytes / (span * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                      "dispatch_us_avg": round(statistics.mean(b - a for a, b in pipe), 3)}})
    if burst and not args.no_ceiling:
        roof["ceiling"] = measure_ceiling(torch, eng, runner, comm, args.steps, args.warmup,
                                          warm_s, nxt, algo_bytes, roof)

    rank_rec = {"rank": rank, "device": local, "nblocks": nb, "parity_blocks": checked,
                "kernel_us_avg": roof["kernel_us_avg"], "frac": roof["frac"],
                "pipelined_period_us": roof["pipelined"]["period_us"],
                "pipelined_frac": roof["pipelined"]["frac"],
                "ceiling_frac": (roof.get("ceiling") or {}).get("frac")}

    split = None
    if args.config == "headline" and not args.no_split:
        del buf, outs
        torch.cuda.empty_cache()
        split_runner, split = split_measure(
            lambda s, c: _split_runner(torch, lvkv, eng, dev, rank, s, c), comm, rank, world,
            min(args.steps, 20), 2, warm_s, total=args.split_total)
        del split_runner
        torch.cuda.empty_cache()

    ranks = comm.gather(rank_rec)
    if rank == 0 and args.config == "headline" and not args.no_pmc:
        # rank 0's GPU (device 0 of the node); the other ranks are done with theirs
        t = live_pmc_traffic()
        if t is not None:
            roof["traffic"] = t["bytes"]
            roof["traffic_source"] = t["source"] + (f"; rank 0 of {world}" if world > 1 else "")

    if rank == 0:
        line = _line_base(args, world, value, ms_per_step / 1e3, {
            "workload": desc, "nblocks_per_gpu": nb, "block_bytes": L, "stride": stride,
            "rotation_buffers": nrot, "rotation_bytes": nrot * window,
            "path": "AQL engine, batches overlapped" + ("" if burst else ", general walk"),
            "parallelism": f"{world} independent block batches (no collective)",
            "parity_blocks": sum(r["parity_blocks"] for r in ranks)})
        line["pct_hbm_peak"] = round(100.0 * value * GIB / 1e9 / HBM_PEAK_GBS / world, 2)
        line["roofline"] = roof
        if world > 1:
            line["roofline"]["per_rank"] = ranks
        line["split"] = split
        line["cpu_baseline"] = None if args.no_cpu_baseline else cpu_baseline(
            args.cpu_seconds if world == 1 else min(args.cpu_seconds, 4.0))
        if line["cpu_baseline"] is not None and world > 1:
            line["cpu_baseline"]["note"] = (f"rank 0's host after every rank's GPU work "
                                            f"({world} ranks on this node)")
        print(json.dumps(line), flush=True)
    _end(world)


CEILING_CO = REPO / "tools" / "probe" / "ceiling_kernels.co"


def _ceiling_trace(torch, lvkv, eng, runner, dev, rank, k):
    """The command a rocprofv3 kernel trace of the read ceiling wraps
    (--ceiling-trace K): the production kernel, then ck_burst_bare and
    ck_stream, K overlapped launches each over the headline rotation (after
    a warm-up of 2K), then ck_burst_bare over the 4 GB config-5 buffer (1M
    blocks a step, K // 10 + 1 steps). Each dispatch's start/end is in the
    trace; tools/trace_period.py reads the period per kernel."""
    co = CEILING_CO.read_bytes()
    i = 1
    for kern in (None, "ck_burst_bare", "ck_stream"):
        if kern is not None:
            eng.load_probe(co, kern, 8, 5, 1, overlapped=True)
        for _ in range(2 * k):
            runner.step(i)
            i += 1
        eng.wait()
        for n in range(k):
            runner.step(i, final=n >= k - 3)
            i += 1
        eng.wait()
    eng.load_probe(None)  # the split runner checks its first step against the oracle
    del runner
    torch.cuda.empty_cache()
    r = _split_runner(torch, lvkv, eng, dev, rank, 0, SPLIT_TOTAL)
    eng.load_probe(co, "ck_burst_bare", 8, 5, 1, overlapped=True)
    for n in range(k // 10 + 1):
        r.step(n)
    eng.wait()
    eng.load_probe(None)


def measure_ceiling(torch, eng, runner, comm, steps, warmup, warm_s, first, algo_bytes, roof):
    """What the chip gives a kernel that only reads, measured the way the
    headline is ('a measured copy-kernel ceiling'): the
    engine dispatches read-only kernels (tools/probe/ceiling_kernels.hip) in
    place of the CRC kernel over the same rotating windows, K overlapped
    launches on the same queues, priced with the same algorithmic bytes.
      burst_bare  the production overlapped kernel's own loads, no tables/walk
      stream      a plain 16 B/lane streaming read of each window
      ordered     the ordered kernel's loads, one launch alone
      warm_mall   the production kernel over 4 windows (164 MB: resident in
                  the 256 MiB Infinity Cache), to show what a MALL-served
                  rate looks like next to the cold rotation
      copy_d2d    torch's device copy of 512 MiB (read + write bytes)."""
    if not CEILING_CO.exists():
        return None
    co = CEILING_CO.read_bytes()
    i = first
    out = {"unit": "GB/s", "peak": HBM_PEAK_GBS,
           "source": "AQL engine dispatching tools/probe/ceiling_kernels.co (lvkv_engine_load_probe)"}

    def pipelined(tag):
        nonlocal i
        el, i = timed_region(runner, comm, steps, warmup, warm_s, first=i)
        spans = profile_launches(runner, eng, steps, False, i)
        i += steps
        period = (max(b for _, b in spans) - min(a for a, _ in spans)) / steps
        return {"kernel": tag, "launches": steps, "period_us": round(period, 3),
                "achieved": round(algo_bytes / (period * 1e-6) / 1e9, 1),
                "timed_region_GBs": round(algo_bytes * steps / el / 1e9, 1)}

    try:
        eng.load_probe(co, "ck_burst_bare", 8, 5, 1, overlapped=True)
        out["burst_bare"] = pipelined("ck_burst_bare (8 waves x 5 chains, 1 per CU, 3 queues)")
        eng.load_probe(co, "ck_stream", 8, 5, 1, overlapped=True)
        out["stream"] = pipelined("ck_stream (16 B/lane, 8 loads in flight, 1 per CU, 3 queues)")
        eng.load_probe(co, "ck_pair_bare", 8, 3, 2, overlapped=False)
        iso = profile_launches(runner, eng, 64, True, i)
        i += 64
        per = max(1, len(iso) // 64)
        d = [iso[k + per - 1][1] - iso[k][0] for k in range(0, per * 64, per)]
        out["ordered"] = {"kernel": "ck_pair_bare (8 x 3, 2 per CU), one launch alone",
                          "kernel_us_avg": round(statistics.mean(d), 3),
                          "achieved": round(algo_bytes / (statistics.mean(d) * 1e-6) / 1e9, 1)}
    finally:
        eng.load_probe(None)
    nrot = runner.nrot
    runner.nrot = min(4, nrot)
    try:
        out["warm_mall"] = pipelined(f"production lvkv_ek_uniform over {runner.nrot} windows "
                                     f"({runner.nrot * runner.nb * runner.stride / 1e6:.0f} MB)")
    finally:
        runner.nrot = nrot
    n = 1 << 29
    src = torch.empty(n, dtype=torch.uint8, device=runner.outs_t[0].device)
    dst = torch.empty_like(src)
    best = float("inf")
    for _ in range(6):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        dst.copy_(src)
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e-3)
    out["copy_d2d"] = {"bytes": 2 * n, "achieved": round(2 * n / best / 1e9, 1),
                       "timing": "torch copy_ of 512 MiB, best of 6, HIP events"}
    del src, dst
    best_bare = max(out["burst_bare"]["achieved"], out["stream"]["achieved"])
    out["achieved"] = best_bare
    out["frac"] = round(best_bare / HBM_PEAK_GBS, 4)
    out["production_over_ceiling"] = round(roof["pipelined"]["achieved"] / best_bare, 4)
    return out


SPLIT_ROTATE_BYTES = 1 << 30  # a rank's slice copies span at least this much


def _split_runner(torch, lvkv, eng, dev, rank, start, count):
    """This rank's slice [start, start + count) of the config-5 batch,
    resident in its HBM, checksummed through the engine. Below 1 GiB per
    slice (4+ ranks) the rank holds several copies of its slice and steps
    rotate over them, so every step reads its slice cold from HBM (2x the
    256 MiB Infinity Cache would still be half warm)."""
    slice_bytes = max(count, 1) * BLOCK
    nrot = max(1, -(-SPLIT_ROTATE_BYTES // slice_bytes))
    gen = torch.Generator(device=dev).manual_seed(0x5EED + start)
    buf = torch.randint(0, 256, (nrot * slice_bytes,), dtype=torch.uint8, device=dev,
                        generator=gen)
    outs = [torch.empty(max(count, 1), dtype=torch.int32, device=dev) for _ in range(2)]
    r = EngineRunner(lvkv, eng, buf, count, BLOCK, BLOCK, 0, nrot, slice_bytes, outs)
    r.step(0)
    r.finish()
    r.sync()
    r.parity_blocks = parity_check(buf, outs[0], count, BLOCK, BLOCK, 0, rank, "split") if count else 0
    r.buf = buf
    return r


def _launch_ranks(n: int) -> int:
    """One process per GPU: this script again under torch.distributed.run
    (rendezvous on 127.0.0.1), as a child process; returns its exit status."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1", f"--master-port={port}",
           str(Path(__file__).resolve()), *sys.argv[1:]]
    log(f"bench: --gpus {n}: launching {n} ranks: {' '.join(cmd)}")
    return subprocess.run(cmd).returncode


class CpuPlumbingRunner:
    """Test-only stand-in for the engine (--plumbing-cpu): the library's
    per-call CPU CRC32C (lvkv_crc32c_value, the drop-in symbol) over this
    rank's slice, so a CPU-only run exercises the rank launch, the slicing,
    the parity count, the per-rank records and the timed region end to end.
    Never a measured line."""

    def __init__(self, lvkv, start, count):
        self.value = lvkv.Value
        self.data = np.frombuffer(np.random.default_rng(start).bytes(max(count, 1) * BLOCK),
                                  np.uint8)
        self.blocks = [self.data[i * BLOCK:(i + 1) * BLOCK].tobytes() for i in range(count)]
        self.count = count
        self.crc = None
        self.step(0)
        self.parity_blocks = self.parity()

    def parity(self):
        """This rank's CRCs against the oracle (checker), as parity_check does."""
        sys.path.insert(0, str(REPO / "oracle"))
        import oracle
        want = oracle.uniform(self.data, self.count, BLOCK, threads=1)
        if [int(x) for x in want] != self.crc:
            raise SystemExit("bench: plumbing parity FAILED")
        return self.count

    def step(self, i, final=False):
        self.crc = [self.value(b) for b in self.blocks]

    def finish(self):
        pass

    def sync(self):
        pass


def _plumbing_cpu(args, lvkv, world, rank, warm_s):
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    comm = Comm(world, None)
    runner, rec = split_measure(lambda s, c: CpuPlumbingRunner(lvkv, s, c), comm, rank, world,
                                args.steps, args.warmup, warm_s, total=args.split_total)
    ranks = comm.gather({"rank": rank, "device": None, "nblocks": runner.count,
                         "parity_blocks": runner.parity_blocks})
    if rank == 0:
        line = _line_base(args, world, rec["value"], rec["ms_per_step"] / 1e3,
                          {"workload": "plumbing test (CPU per-call CRC, not a measurement)",
                           "total_blocks": args.split_total, "block_bytes": BLOCK,
                           "parallelism": f"{world} contiguous slices (no collective)",
                           "parity_blocks": sum(r["parity_blocks"] for r in ranks)})
        line["split"] = rec
        line["rank_counts"] = [r["nblocks"] for r in ranks]
        line["roofline"] = {"per_rank": ranks}
        line["cpu_baseline"] = None if args.no_cpu_baseline else cpu_baseline(args.cpu_seconds)
        line["data"] = "plumbing-cpu: NOT a device measurement"
        print(json.dumps(line), flush=True)
    _end(world)


def _line_base(args, world, value, sec_per_step, config):
    return {"metric": METRICS[args.config], "value": round(value, 2), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(sec_per_step * 1e3, 5), "higher_is_better": True,
            "scaling": "weak" if args.config != "blocks1m_split" else "strong",
            "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (uniform random bytes, device-generated), resident in HBM",
            "warmup_ms_min": args.warmup_ms, "config": config}


def _end(world):
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
