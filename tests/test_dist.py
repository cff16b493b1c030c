"""Multi-process plumbing of the N>1 path on CPU (gloo, world_size 2).

The device work per rank is the same batch call as at N=1 (covered by the GPU
tests). Here two real processes run bench.py's own config-5 code
(bench.split_measure -> shard.shard_range -> bench.timed_region ->
bench.Comm) with a CPU runner in place of the engine: every block is
checksummed exactly once, the gathered slices equal the oracle over the whole
batch, and the reported time is the slowest rank's (common start barrier to
the last completion).
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import REPO


def _load_shard():
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "lvkv_shard", REPO / "leveldb-kv-separation_amd" / "shard.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("n,world", [(0, 2), (1, 2), (7, 2), (10_000, 8), (1_000_000, 8), (13, 5)])
def test_shard_ranges_partition(n, world):
    shard = _load_shard()
    ranges = shard.all_ranges(n, world)
    seen = np.zeros(n, np.int32)
    prev_end = 0
    for start, count in ranges:
        assert start == prev_end
        seen[start:start + count] += 1
        prev_end = start + count
    assert prev_end == n and (seen == 1).all()
    counts = [c for _, c in ranges]
    assert max(counts) - min(counts) <= 1 and counts == sorted(counts, reverse=True)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, slow_rank, q):
    import sys
    import time

    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, str(REPO))
    sys.path.insert(0, str(REPO / "oracle"))
    import bench
    import oracle

    block = 4096
    data = oracle.splitmix_bytes(0xC0FFEE, total * block)

    class CpuSliceRunner:
        """bench.EngineRunner's interface over this rank's slice, on the CPU."""

        def __init__(self, start, count):
            self.view = data[start * block:(start + count) * block]
            self.count = count
            self.crc = None
            self.steps = 0

        def step(self, i):
            self.crc = oracle.uniform(self.view, self.count, block, threads=1)
            self.steps += 1
            if rank == slow_rank:
                time.sleep(0.02)

        def finish(self):
            pass

        def sync(self):
            pass

    comm = bench.Comm(world)
    runner, rec = bench.split_measure(CpuSliceRunner, comm, rank, world, steps=3, warmup=1,
                                      warmup_s=0.0, total=total, block=block)
    shard = _load_shard()
    local = torch.from_numpy(runner.crc.view(np.int32).copy())
    full = shard.gather_slices(local, total)
    if rank == 0:
        q.put((full.numpy().view(np.uint32).tolist(), rec, runner.count))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("total,slow_rank", [(11, 1), (64, 0), (97, 1)])
def test_gloo_world2_split_bench(total, slow_rank):
    import sys
    sys.path.insert(0, str(REPO / "oracle"))
    import oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, total, slow_rank, q))
             for r in range(2)]
    for p in procs:
        p.start()
    full, rec, count0 = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    data = oracle.splitmix_bytes(0xC0FFEE, total * 4096)
    want = oracle.uniform(data, total, 4096, threads=1)
    assert full == [int(x) for x in want]
    assert count0 == (total + 1) // 2
    assert rec["total_blocks"] == total and rec["ranks"] == 2 and rec["steps"] == 3
    # max over ranks: the slow rank's 3 x 20 ms is the reported time on rank 0
    assert rec["ms_per_step"] >= 20.0
    assert rec["value"] == pytest.approx(total * 4096 / (rec["ms_per_step"] * 1e-3) / 2**30,
                                         rel=1e-3, abs=1e-3)


def _bench(args, env_extra=None, timeout=240):
    import json
    import subprocess
    import sys
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, str(REPO / "bench.py"), *args], env=env,
                       capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr


def test_bench_gpus2_launches_two_ranks():
    """`bench.py --gpus 2` with no launcher around it starts two ranks itself
    (torch.distributed.run child, before any GPU call) and the line reports
    both: n_gpus, the split's ranks and each rank's slice."""
    rc, line, err = _bench(["--gpus", "2", "--plumbing-cpu", "--config", "blocks1m_split",
                            "--split-total", "65", "--steps", "3", "--warmup", "1",
                            "--warmup-ms", "0", "--cpu-seconds", "0.3"])
    assert rc == 0, err[-2000:]
    assert line["n_gpus"] == 2
    assert line["split"]["ranks"] == 2 and line["split"]["total_blocks"] == 65
    assert line["rank_counts"] == [33, 32]
    # the N > 1 line: the config's own metric, every rank's slice
    # and parity count, per-rank records, and rank 0's CPU baseline
    import sys
    sys.path.insert(0, str(REPO))
    import bench
    assert line["metric"] == bench.METRICS["blocks1m_split"] != bench.METRIC
    assert line["split"]["slices"] == [
        {"rank": 0, "start": 0, "blocks": 33, "parity_blocks": 33},
        {"rank": 1, "start": 33, "blocks": 32, "parity_blocks": 32}]
    assert [r["rank"] for r in line["roofline"]["per_rank"]] == [0, 1]
    assert line["config"]["parity_blocks"] == 65
    cb = line["cpu_baseline"]
    assert cb["kind"] in ("reference", "port") and cb["cores"] == 1 and cb["value"] > 0
    assert cb["multi_thread"]["cores"] >= 1


def test_bench_refuses_world_mismatch():
    """A launcher that started a different number of ranks than --gpus asks
    for is an error, not a one-GPU line."""
    rc, line, err = _bench(["--gpus", "2", "--plumbing-cpu", "--config", "blocks1m_split",
                            "--split-total", "8", "--steps", "1", "--warmup", "1",
                            "--warmup-ms", "0"],
                           env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert rc != 0 and line is None
    assert "--gpus 2" in err
