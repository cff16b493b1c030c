"""Benchmark: device-resident batched CRC32C (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config headline|wal32k|blocks1m|host]

One step = one launch of the batch kernel over one batch of blocks already
resident in HBM (the headline batch: 10,000 x 4096 B). Consecutive steps read
different windows of a >= 1 GiB rotation so every launch is cold in the
256 MiB Infinity Cache. Steps are independent batches: step i is issued on
stream i % S (--streams, default 2), so one batch's kernel can start on the
CUs the previous batch's kernel has released (a checksum service with two
batches in flight); --streams 1 serialises them. N > 1: one process per GPU
(torchrun), every rank checksums its own 10k-block batch (independent slices,
weak scaling, no collective on the data path); time = max over ranks of the
barrier-bracketed K steps. Rank 0 prints ONE JSON line.

value = whole-job GiB/s of the K steps (all streams, barrier + synchronize
on both sides). roofline.achieved = algorithmic bytes per launch (nblocks x
(block + 4 B CRC out)) / the kernel's own average launch
duration, measured by a HIP event pair around K launches issued back to back
on ONE stream (so it agrees with a rocprofv3 kernel trace of --streams 1);
roofline.pipelined prices the same bytes on the S-stream launch period.
cpu_baseline = the reference's own util/crc32c.cc (compiled in place into
oracle/_ref) timed on this host.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
GIB = float(1 << 30)

CONFIGS = {
    # name: (nblocks, block_bytes, stride, crc_offset_in_block, description)
    "headline": (10_000, 4096, 4096, 0, "10k x 4 KiB blocks (BASELINE headline)"),
    "wal32k": (16_384, 32762, 32768, 6, "16384 x 32 KiB WAL blocks, CRC over [6, 32768) (config 3)"),
    "blocks1m": (1_000_000, 4096, 4096, 0, "1M x 4 KiB blocks (config 4)"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


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


def load_pmc_traffic():
    p = REPO / "profiles" / "pmc_traffic.json"
    if p.exists():
        try:
            return json.loads(p.read_text()).get("hbm_bytes_per_launch")
        except (ValueError, OSError):
            return None
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", default="headline", choices=sorted(CONFIGS))
    ap.add_argument("--rotate-bytes", type=float, default=1.25 * GIB)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--streams", type=int, default=2,
                    help="independent batches in flight: step i runs on stream i %% S")
    args = ap.parse_args()

    world, rank, local = dist_env()
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    import __graft_entry__ as g
    lvkv = g.load_package()

    nb, L, stride, crc_off, desc = CONFIGS[args.config]
    batch_bytes = nb * stride
    nrot = max(1, int(np.ceil(args.rotate_bytes / batch_bytes)))
    gen = torch.Generator(device=dev).manual_seed(0x1EDC6F41 + 17 * rank)
    buf = torch.randint(0, 256, (nrot * batch_bytes + 64,), dtype=torch.uint8,
                        device=dev, generator=gen)
    nstreams = max(1, args.streams)
    outs = [torch.empty(nb, dtype=torch.int32, device=dev) for _ in range(2 * nstreams)]
    stream = torch.cuda.current_stream(dev)
    side = [torch.cuda.Stream(dev) for _ in range(nstreams - 1)]
    hstreams = [stream.cuda_stream] + [s.cuda_stream for s in side]

    # Steps call the C-ABI entry point directly (lvkv_crc32c_uniform_device,
    # include/lvkv_crc32c.h) with pre-computed device pointers, so the host
    # issues launches faster than the GPU retires them.
    c_uniform = lvkv.lib.lvkv_crc32c_uniform_device
    bases = [buf.data_ptr() + w * batch_bytes + crc_off for w in range(nrot)]
    out_ptrs = [o.data_ptr() for o in outs]
    hstream = stream.cuda_stream

    def launch(i):
        rc = c_uniform(bases[i % nrot], stride, L, 0, out_ptrs[i % len(out_ptrs)], nb, 0,
                       hstreams[i % nstreams])
        if rc != 0:
            raise SystemExit(f"bench: lvkv_crc32c_uniform_device failed ({rc})")

    # correctness spot check (outside the timed region) against the oracle
    sys.path.insert(0, str(REPO / "oracle"))
    import oracle
    launch(0)
    torch.cuda.synchronize()
    check_n = min(nb, 2000)
    host = buf[crc_off: crc_off + (check_n - 1) * stride + L].cpu().numpy()
    want = oracle.uniform(host, check_n, L, stride, threads=8)
    got = outs[0][:check_n].cpu().numpy().view(np.uint32)
    if not np.array_equal(got, want):
        raise SystemExit(f"bench: parity check FAILED on rank {rank}")

    # The kernel's own launch duration (roofline): K launches issued back to
    # back on ONE stream, before any side stream is used (a process whose
    # side streams have run measured ~10 % longer single-stream launches).
    for i in range(args.warmup):
        c_uniform(bases[(i + 1) % nrot], stride, L, 0, out_ptrs[i & 1], nb, 0, hstream)
    k0 = torch.cuda.Event(enable_timing=True)
    k1 = torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    k0.record(stream)
    for i in range(args.steps):
        c_uniform(bases[(i + 5) % nrot], stride, L, 0, out_ptrs[i & 1], nb, 0, hstream)
    k1.record(stream)
    torch.cuda.synchronize()
    kern_ms = k0.elapsed_time(k1) / args.steps

    # Labelled secondary figure: the same batch re-read while resident in the
    # 256 MiB MALL (not the headline; the headline rotates >= 1.25 GiB).
    warm_us = None
    if args.config == "headline":
        torch.cuda.synchronize()
        w0 = torch.cuda.Event(enable_timing=True)
        w1 = torch.cuda.Event(enable_timing=True)
        for _ in range(5):
            c_uniform(bases[0], stride, L, 0, out_ptrs[0], nb, 0, hstream)
        w0.record(stream)
        for _ in range(100):
            c_uniform(bases[0], stride, L, 0, out_ptrs[0], nb, 0, hstream)
        w1.record(stream)
        torch.cuda.synchronize()
        warm_us = w0.elapsed_time(w1) * 10.0

    for i in range(args.warmup):
        launch(i + 1)
    torch.cuda.synchronize()

    # timed region: K back-to-back steps over S streams, barrier + sync on
    # both sides; an event pair on the default stream (the side streams fork
    # from and join into it) gives the device-side launch period.
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for s in side:
        s.wait_stream(stream)
    for i in range(args.steps):
        launch(i + 3)
    for s in side:
        stream.wait_stream(s)
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    period_ms = ev0.elapsed_time(ev1) / args.steps
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())

    ms_per_step = elapsed / args.steps * 1e3
    data_bytes = nb * L
    value = world * data_bytes * args.steps / elapsed / GIB
    algo_bytes = nb * (L + 4)
    achieved = algo_bytes / (kern_ms * 1e-3) / 1e9
    achieved_pipe = algo_bytes / (period_ms * 1e-3) / 1e9

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args.cpu_seconds)
        traffic = load_pmc_traffic() if args.config == "headline" else None
        line = {
            "metric": "device-resident CRC32C GiB/s over 10k×4KiB blocks; % of MI355X HBM peak",
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (uniform random bytes, device-generated), resident in HBM",
            "pct_hbm_peak": round(100.0 * value * GIB / 1e9 / HBM_PEAK_GBS, 2),
            "config": {"workload": desc, "nblocks_per_gpu": nb, "block_bytes": L,
                       "stride": stride, "rotation_buffers": nrot,
                       "rotation_bytes": nrot * batch_bytes,
                       "streams": nstreams,
                       "parallelism": f"{world} independent block slices (no collective)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "kernel_us_avg": round(kern_ms * 1e3, 3),
                         "pipelined": {"streams": nstreams,
                                       "period_us": round(period_ms * 1e3, 3),
                                       "achieved": round(achieved_pipe, 1),
                                       "frac": round(achieved_pipe / HBM_PEAK_GBS, 4)},
                         "warm_mall_us_avg": None if warm_us is None else round(warm_us, 3),
                         "algo_bytes_per_launch": algo_bytes},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
