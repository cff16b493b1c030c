"""Whole-SSTable verify timing (GPU box). Not part of the product.

    python tools/probe/sst_probe.py [nblocks]

A synthetic table (tests/sst_synth.py) through lvkv_sst_verify_table_device,
back to back on one stream; with rocprofv3 around it, the two launches' own
durations.
"""
import ctypes
import sys
import time
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests"))
sys.path.insert(0, str(REPO / "oracle"))
import __graft_entry__ as g  # noqa: E402
import sst_synth  # noqa: E402

lvkv = g.load_package()


def main():
    nblocks = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    img = sst_synth.build_sst(nblocks, 4096, seed=nblocks, ragged=True)
    dev = torch.device("cuda:0")
    buf = torch.from_numpy(np.frombuffer(img, dtype=np.uint8).copy()).to(dev)
    rep, *_ = lvkv.sst_verify_table(buf)
    cap = rep["nblocks"] + 1
    o = torch.empty(cap, dtype=torch.int64, device=dev)
    sz = torch.empty(cap, dtype=torch.int32, device=dev)
    ac = torch.empty(cap, dtype=torch.int32, device=dev)
    st = torch.empty(cap, dtype=torch.uint8, device=dev)
    rp = torch.zeros(ctypes.sizeof(lvkv.SstReport), dtype=torch.uint8, device=dev)
    vp = ctypes.c_void_p
    h = vp(torch.cuda.current_stream().cuda_stream)
    L = lvkv.lib
    pol = lvkv.BLOOM_POLICY.encode()

    def call():
        rc = L.lvkv_sst_verify_table_device(vp(buf.data_ptr()), len(img), vp(o.data_ptr()),
                                            vp(sz.data_ptr()), vp(ac.data_ptr()),
                                            vp(st.data_ptr()), cap, pol, vp(rp.data_ptr()), h)
        assert rc == 0
    for _ in range(5):
        call()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        call()
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / 50 * 1e6
    print(f"sst_verify {nblocks} blocks, {len(img)} bytes: {us:.1f} us/call", flush=True)


if __name__ == "__main__":
    main()
