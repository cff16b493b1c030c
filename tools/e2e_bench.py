"""End-to-end (host memory in, host memory out) CRC32C rate through
lvkv_crc32c_batch_host: pageable user buffer -> packed into pinned staging ->
hipMemcpyAsync H2D -> batch kernel -> D2H of N x 4 B, two stages overlapped;
and through the AQL engine from pinned host memory (chunked H2D copies on a
side stream, each chunk submitted to the engine when its copy completes).
Also measures the raw pinned H2D copy rate (the ceiling for this path) and
checks every result against the oracle. Prints one JSON object.

    python tools/e2e_bench.py [--blocks N] [--block-bytes L] [--reps R]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "oracle"))
import __graft_entry__ as g  # noqa: E402

GIB = float(1 << 30)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, nargs="+", default=[10_000, 250_000])
    ap.add_argument("--block-bytes", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--chunk-mib", type=int, default=8,
                    help="engine path: bytes per H2D copy + engine submit")
    a = ap.parse_args()
    lvkv = g.load_package()
    import oracle

    torch.cuda.init()
    res = {"block_bytes": a.block_bytes, "runs": []}
    L = a.block_bytes
    for nb in a.blocks:
        data = np.frombuffer(np.random.default_rng(nb).bytes(nb * L), dtype=np.uint8)
        offs = np.arange(nb, dtype=np.uint64) * L
        lens = np.full(nb, L, dtype=np.uint32)
        got = lvkv.crc32c_batch_host(data, offs, lens)  # warm: staging alloc
        want = oracle.uniform(data, nb, L, threads=8)
        assert np.array_equal(got, want), "e2e parity"
        best = float("inf")
        for _ in range(a.reps):
            t0 = time.perf_counter()
            lvkv.crc32c_batch_host(data, offs, lens)
            best = min(best, time.perf_counter() - t0)
        # raw pinned H2D ceiling for the same bytes (one copy, and the engine
        # path's own chunked copies with no engine): measured interleaved with
        # the engine path below, in the same process, on the same buffers
        pinned = torch.empty(nb * L, dtype=torch.uint8).pin_memory()
        dev = torch.empty(nb * L, dtype=torch.uint8, device="cuda")
        dev.copy_(pinned, non_blocking=True)
        torch.cuda.synchronize()

        def h2d_run():
            dev.copy_(pinned, non_blocking=True)
            torch.cuda.synchronize()
        # engine path from pinned host memory (a reader that pread()s into a
        # pinned buffer, table/format.cc:69-100): chunks copied H2D on a side
        # stream (SDMA), each submitted to the AQL engine as soon as its copy
        # event completes (system-scope acquire: a copy engine wrote it) while
        # the next chunk's copy runs; the CRCs come back D2H at the end
        pinned.copy_(torch.from_numpy(data))
        eng = lvkv.Engine(0)
        out = torch.empty(nb, dtype=torch.int32, device="cuda")
        hout = torch.empty(nb, dtype=torch.int32).pin_memory()
        chunk_blocks = max(1, min(nb, (a.chunk_mib << 20) // L))
        side = torch.cuda.Stream()

        def chunked_h2d_run():
            with torch.cuda.stream(side):
                for b0 in range(0, nb, chunk_blocks):
                    n = min(chunk_blocks, nb - b0)
                    dev[b0 * L:(b0 + n) * L].copy_(pinned[b0 * L:(b0 + n) * L], non_blocking=True)
            side.synchronize()

        def engine_run():
            evs = []
            with torch.cuda.stream(side):
                for b0 in range(0, nb, chunk_blocks):
                    n = min(chunk_blocks, nb - b0)
                    dev[b0 * L:(b0 + n) * L].copy_(pinned[b0 * L:(b0 + n) * L], non_blocking=True)
                    e = torch.cuda.Event()
                    e.record(side)
                    evs.append((b0, n, e))
            for b0, n, e in evs:
                e.synchronize()
                rc = eng.submit_ptr(eng.handle, dev.data_ptr() + b0 * L, L, L, 0,
                                    out.data_ptr() + 4 * b0, n, lvkv.LVKV_FLAG_SYSTEM_ACQUIRE)
                assert rc == 0
            eng.wait()
            hout.copy_(out)  # D2H of N x 4 B
        engine_run()
        assert np.array_equal(hout.numpy().view(np.uint32), want), "engine e2e parity"
        times = {"h2d": [], "chunked": [], "engine": []}
        for _ in range(a.reps):
            for name, fn in (("h2d", h2d_run), ("chunked", chunked_h2d_run), ("engine", engine_run)):
                t0 = time.perf_counter()
                fn()
                times[name].append(time.perf_counter() - t0)
        h2d, eng_best = min(times["h2d"]), min(times["engine"])
        med = {k: sorted(v)[len(v) // 2] for k, v in times.items()}
        res["runs"].append({
            "nblocks": nb, "bytes": nb * L,
            "e2e_gibs": round(nb * L / best / GIB, 3), "e2e_ms": round(best * 1e3, 3),
            "engine_pinned_e2e_gibs": round(nb * L / eng_best / GIB, 3),
            "engine_pinned_e2e_ms": round(eng_best * 1e3, 3),
            "engine_chunk_blocks": chunk_blocks,
            "pinned_h2d_gibs": round(nb * L / h2d / GIB, 3),
            "chunked_h2d_gibs": round(nb * L / min(times["chunked"]) / GIB, 3),
            "median_gibs": {k: round(nb * L / v / GIB, 3) for k, v in med.items()},
            "reps": a.reps, "timing": "best and median of reps, the three runs interleaved",
            "parity": "bit-exact vs oracle (both paths)"})
        del pinned, dev, out, hout, eng
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
