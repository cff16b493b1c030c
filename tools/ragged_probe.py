"""Timing probe for the general-layout kernels (crc32c_ragged.hip and
crc32c_kernel.hip) on synthetic batches that isolate one factor each:
end alignment, block length, block count. Compute mode through
lvkv_crc32c_batch_device; every result checked against the oracle once.

    python tools/ragged_probe.py [--kernels=-1,0,4] [--reps 50]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "oracle"))
import __graft_entry__ as g  # noqa: E402

# name: (nblocks, length, stride, first offset)
CASES = {
    "4096_aligned": (16384, 4096, 4096, 0),
    "4272_aligned": (16384, 4272, 4272, 0),
    "4271_end_unaligned": (16384, 4271, 4272, 0),
    "4270_start_end_unaligned": (16384, 4270, 4272, 1),
    "4272_stride4275": (16384, 4272, 4275, 0),
    "8192_aligned": (8192, 8192, 8192, 0),
    "2048_aligned": (32768, 2048, 2048, 0),
    "4096_aligned_65k": (65536, 4096, 4096, 0),
    # (n, max length, 0, seed): lengths uniform in [0, max), packed back to back
    "rand2000_62k": (62000, 2000, 0, 7),
    "rand8000_16k": (16384, 8000, 0, 8),
    "4271_end_unaligned_65k": (65536, 4271, 4272, 0),
    "rand8000_65k": (65536, 8000, 0, 9),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernels", default="-1,0,4")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--cases", default=",".join(CASES))
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    lvkv = g.load_package()
    import oracle
    dev = torch.device("cuda:0")
    L = lvkv.lib
    vp = ctypes.c_void_p
    h = vp(torch.cuda.current_stream().cuda_stream)
    rng = np.random.default_rng(1)
    data = torch.from_numpy(rng.integers(0, 256, 300 << 20, dtype=np.uint8)).to(dev)
    host = None
    res = {}
    for name in args.cases.split(","):
        n, length, stride, first = CASES[name]
        want = None
        if stride == 0:
            lens = np.random.default_rng(first).integers(0, length, n).astype(np.uint32)
            offs = np.concatenate([[0], np.cumsum(lens[:-1].astype(np.uint64))]).astype(np.uint64)
            length = float(lens.mean())
        else:
            offs = (first + stride * np.arange(n, dtype=np.uint64)).astype(np.uint64)
            lens = np.full(n, length, dtype=np.uint32)
        d_off = torch.from_numpy(offs.astype(np.int64)).to(dev)
        d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        row = {}
        for k in [int(x) for x in args.kernels.split(",")]:
            assert L.lvkv_debug_set_general_kernel(k) == 0

            def call():
                rc = L.lvkv_crc32c_batch_device(vp(data.data_ptr()), vp(d_off.data_ptr()),
                                                vp(d_len.data_ptr()), None, 0, vp(out.data_ptr()),
                                                n, 0, h)
                assert rc == 0
            call()
            torch.cuda.synchronize()
            if host is None:
                host = data.cpu().numpy()
            if want is None:
                want = oracle.batch(host, offs, lens, None, threads=8)
            if True:  # every kernel against the oracle
                assert np.array_equal(out.cpu().numpy().view(np.uint32), want), (name, k)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.reps):
                call()
            b.record()
            torch.cuda.synchronize()
            us = a.elapsed_time(b) * 1e3 / args.reps
            row[str(k)] = {"us": round(us, 2), "TBps": round(n * length / us / 1e6, 2)}
        L.lvkv_debug_set_general_kernel(0)
        res[name] = row
        print(name, json.dumps(row), flush=True)
    if args.json:
        Path(args.json).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
