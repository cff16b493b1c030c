"""Per-kernel profile of the §8f SST paths: run under
`rocprofv3 --kernel-trace --stats -d gpurun_out/sst -- python tools/sst_prof.py`.

Builds the 16,384-block synthetic table (tests/sst_synth.py), then calls
  - lvkv_sst_verify_table_device        (the eight-launch pipeline)
  - lvkv_sst_fill_trailers_device       (general batch + long-block kernel)
  - lvkv_sst_verify_device on the data blocks only (no index/filter: the
    general batch kernel alone, no long block)
`--reps` times each, for every general-layout kernel given with --kernels.
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
    ap.add_argument("--kernels", default="0")
    ap.add_argument("--nblocks", type=int, default=16384)
    args = ap.parse_args()
    lvkv = g.load_package()
    import sst_synth
    import sst_table
    dev = torch.device("cuda:0")
    img = sst_synth.build_sst(args.nblocks, 4096, seed=args.nblocks, ragged=True)
    want = sst_table.verify_table(img)
    buf = torch.from_numpy(np.frombuffer(img, dtype=np.uint8).copy()).to(dev)
    L = lvkv.lib
    vp = ctypes.c_void_p
    h = vp(torch.cuda.current_stream().cuda_stream)
    cap = args.nblocks + 8
    o2 = torch.empty(cap, dtype=torch.int64, device=dev)
    s2 = torch.empty(cap, dtype=torch.int32, device=dev)
    a2 = torch.empty(cap, dtype=torch.int32, device=dev)
    st2 = torch.empty(cap, dtype=torch.uint8, device=dev)
    rp = torch.zeros(ctypes.sizeof(lvkv.SstReport), dtype=torch.uint8, device=dev)
    handles = want.handles + [want.meta, want.index]
    offs = torch.tensor([x for x, _ in handles], dtype=torch.int64, device=dev)
    sizes = torch.tensor([s for _, s in handles], dtype=torch.int32, device=dev)
    crc = torch.empty(len(handles), dtype=torch.int32, device=dev)
    ndata = want.ndata
    for k in [int(x) for x in args.kernels.split(",")]:
        assert L.lvkv_debug_set_general_kernel(k) == 0
        for _ in range(args.reps):
            assert L.lvkv_sst_verify_table_device(vp(buf.data_ptr()), len(img), vp(o2.data_ptr()),
                                                  vp(s2.data_ptr()), vp(a2.data_ptr()),
                                                  vp(st2.data_ptr()), cap, vp(rp.data_ptr()),
                                                  h) == 0
        for _ in range(args.reps):
            assert L.lvkv_sst_fill_trailers_device(vp(buf.data_ptr()), vp(offs.data_ptr()),
                                                   vp(sizes.data_ptr()), vp(crc.data_ptr()),
                                                   len(handles), h) == 0
        for _ in range(args.reps):
            assert L.lvkv_sst_verify_device(vp(buf.data_ptr()), vp(offs.data_ptr()),
                                            vp(sizes.data_ptr()), vp(a2.data_ptr()),
                                            vp(st2.data_ptr()), ndata, h) == 0
        torch.cuda.synchronize()
        assert int(st2[:ndata].sum()) == 0
    L.lvkv_debug_set_general_kernel(0)
    assert bytes(buf.cpu().numpy()) == img
    print("ok", flush=True)


if __name__ == "__main__":
    main()
