"""Per-kernel profile of the WAL path: run under
`rocprofv3 --kernel-trace -d gpurun_out/x -o run -- python tools/log_prof.py`.
Builds the synthetic log (tests/log_synth.py) and calls
lvkv_log_verify_blocks_device and lvkv_log_fill_headers_device --reps times.
"""
from __future__ import annotations

import argparse
import ctypes
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "oracle"))
sys.path.insert(0, str(REPO / "tests"))
import __graft_entry__ as g  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--nrec", type=int, default=60000)
    ap.add_argument("--big-every", type=int, default=997)
    ap.add_argument("--kernels", default="0")
    ap.add_argument("--log-kernels", default="8")
    args = ap.parse_args()
    lvkv = g.load_package()
    import log_synth
    dev = torch.device("cuda:0")
    img = log_synth.build_log(args.nrec, seed=args.nrec, max_len=2000, big_every=args.big_every)
    buf = torch.from_numpy(np.frombuffer(img, dtype=np.uint8).copy()).to(dev)
    rep, hdr, actual, rst, bst, bdrop = lvkv.log_verify_blocks(buf)
    cap, nb = rep["nrecords"], rep["nblocks"]
    L = lvkv.lib
    vp = ctypes.c_void_p
    h = vp(torch.cuda.current_stream().cuda_stream)
    hdr2 = torch.empty(cap, dtype=torch.int64, device=dev)
    act2 = torch.empty(cap, dtype=torch.int32, device=dev)
    rst2 = torch.empty(cap, dtype=torch.uint8, device=dev)
    bst2 = torch.empty(nb, dtype=torch.uint8, device=dev)
    bd2 = torch.empty(nb, dtype=torch.int32, device=dev)
    rp = torch.zeros(64, dtype=torch.uint8, device=dev)
    for k, lk in [(int(x), int(y)) for x in args.kernels.split(",")
                  for y in args.log_kernels.split(",")]:
        assert L.lvkv_debug_set_general_kernel(k) == 0
        assert L.lvkv_debug_set_log_kernel(lk) == 0
        for _ in range(args.reps):
            assert L.lvkv_log_verify_blocks_device(vp(buf.data_ptr()), len(img), vp(hdr2.data_ptr()),
                                                   vp(act2.data_ptr()), vp(rst2.data_ptr()), cap,
                                                   vp(bst2.data_ptr()), vp(bd2.data_ptr()),
                                                   vp(rp.data_ptr()), h) == 0
        for _ in range(args.reps):
            assert L.lvkv_log_fill_headers_device(vp(buf.data_ptr()), vp(hdr.data_ptr()), None,
                                                  cap, h) == 0
    L.lvkv_debug_set_general_kernel(0)
    L.lvkv_debug_set_log_kernel(8)
    torch.cuda.synchronize()
    assert bytes(buf.cpu().numpy()) == img
    print("ok", flush=True)


if __name__ == "__main__":
    main()
