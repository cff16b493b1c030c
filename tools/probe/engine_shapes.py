"""Per-shape timing of the engine's general walk (GPU box). Not part of the
product.

    python tools/probe/engine_shapes.py [--cases a,b] [--reps 40]

Each case is one batch submitted to the AQL engine (lvkv_engine_crc32c_batch,
or lvkv_engine_crc32c_uniform for the uniform cases): checked once against
the oracle, then `reps` ordered launches (one alone on the chip, HSA
packet-processor start/end per dispatch) and `reps` overlapped ones (device
span / reps). Algorithmic bytes: sum(length) + 4 per block.
Run under rocprofv3 --kernel-trace --stats for the kernel durations (one
case per run keeps the rows apart)."""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "oracle"))
import __graft_entry__ as g  # noqa: E402

# name: (nblocks, length | max length, stride | 0 = packed random lengths, first offset | seed, uniform)
CASES = {
    "sst4271_16k": (16384, 4271, 4272, 0, False),     # SST-sized, ends unaligned
    "sst4106_16k": (16384, 4106, 4106, 3, False),     # 4105 B + type byte, any alignment
    "rand2000_62k": (62000, 2000, 0, 7, False),       # WAL-record-sized, packed (LVKV_FLAG_SMALL_BLOCKS)
    "eq1000_62k": (62000, -1000, 0, 7, False),        # packed, every record 1000 B
    "eq200_300k": (300000, -200, 0, 7, False),        # packed, every record 200 B
    "wal32k_16k": (16384, 32762, 32768, 6, True),     # config 3 (512 MiB)
    "wal32k_2k": (2048, 32762, 32768, 6, True),
    "u4096_65k": (65536, 4096, 4096, 0, False),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default=",".join(CASES))
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--specs", default="-1,2,3,4,5",
                    help="lvkv_debug_engine_ragged_spec values (-1: the engine's choice)")
    args = ap.parse_args()
    lvkv = g.load_package()
    import oracle
    dev = torch.device("cuda:0")
    eng = lvkv.Engine(0)
    import ctypes
    lvkv.lib.lvkv_debug_engine_ragged_spec.argtypes = [ctypes.c_void_p, ctypes.c_int]
    res = {}
    for name in args.cases.split(","):
        n, length, stride, first, uniform = CASES[name]
        rng = np.random.default_rng(n + length)
        if stride:
            lens = np.full(n, length, np.uint32)
            offs = (np.arange(n, dtype=np.uint64) * stride + first).astype(np.uint64)
            size = int(offs[-1]) + length + 8
        else:
            lens = (np.full(n, -length, np.uint32) if length < 0 else
                    rng.integers(0, length, n).astype(np.uint32))
            offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
            size = int(offs[-1]) + int(lens[-1]) + 8
        host = rng.integers(0, 256, size, dtype=np.uint8)
        buf = torch.from_numpy(host).to(dev)
        d_off = torch.from_numpy(offs.astype(np.int64)).to(dev)
        d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()

        def submit(ordered=False):
            if uniform:
                eng.crc32c_uniform(buf[first:], n, length, stride, ordered=ordered, fresh=False,
                                   out=out)
            else:
                # (the small-record case passes the caller's hint)
                eng.crc32c_batch(buf, d_off, d_len, ordered=ordered, fresh=False, out=out,
                                 small=name.startswith(("rand", "eq")))
        want = (oracle.uniform(host[first:], n, length, stride, threads=16) if uniform else
                oracle.batch(host, offs, lens, threads=16))
        algo = int(lens.sum()) + 4 * n
        for spec in (int(x) for x in args.specs.split(",")):
            assert lvkv.lib.lvkv_debug_engine_ragged_spec(eng.handle, spec) == 0
            out.zero_()
            torch.cuda.synchronize()
            submit()
            eng.wait()
            ok = bool(np.array_equal(out.cpu().numpy().view(np.uint32), want))
            for _ in range(5):
                submit()
            eng.wait()
            eng.profile(True)
            for _ in range(args.reps):
                submit(ordered=True)
            eng.wait()
            iso = eng.profile_read()
            for _ in range(args.reps):
                submit()
            eng.wait()
            pipe = eng.profile_read()
            eng.profile(False)
            per = max(1, len(iso) // args.reps)  # dispatches per batch
            d = [iso[i + per - 1][1] - iso[i][0] for i in range(0, per * args.reps, per)]
            span = (max(b for _, b in pipe) - min(a for a, _ in pipe)) / args.reps
            r = {"spec": spec, "parity": ok, "blocks": n, "algo_bytes": algo,
                 "dispatches": per,
                 "iso_us_avg": round(statistics.mean(d), 2), "iso_us_min": round(min(d), 2),
                 "iso_frac": round(algo / (statistics.mean(d) * 1e-6) / 8e12, 4),
                 "pipe_period_us": round(span, 2),
                 "pipe_frac": round(algo / (span * 1e-6) / 8e12, 4)}
            res[f"{name}/{spec}"] = r
            print(name, json.dumps(r), flush=True)
        assert lvkv.lib.lvkv_debug_engine_ragged_spec(eng.handle, -1) == 0
        del buf, d_off, d_len, out
        torch.cuda.empty_cache()
    (REPO / "gpurun_out").mkdir(exist_ok=True)
    (REPO / "gpurun_out" / "engine_shapes.json").write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
