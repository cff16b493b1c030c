"""Throughput of the §8f paths on one GPU (device-resident inputs), next to
the reference's util/crc32c.cc on the same blocks (oracle/_ref, 1 thread).

    python tools/paths_bench.py [--reps R] [--json out.json]

  sst_verify_table   lvkv_sst_verify_table_device on a synthetic SSTable
                     (reference format, tests/sst_synth.py), 5 launches/call
  log_verify_blocks  lvkv_log_verify_blocks_device on a synthetic log
                     (tests/log_synth.py), 5 launches/call
  sst_fill_trailers  lvkv_sst_fill_trailers_device over the same table
  log_fill_headers   lvkv_log_fill_headers_device over the same log

GB/s = file bytes / device time per call (HIP events around R calls issued
back to back on one stream). Every result is checked against the oracle.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "oracle"))
sys.path.insert(0, str(REPO / "tests"))
import __graft_entry__ as g  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps  # us per call


def cpu_rate(ref, img: np.ndarray, offs, lens, seconds=2.0):
    """The reference's Value() over the same covered ranges, 1 thread."""
    o = np.asarray(offs, dtype=np.uint64)
    n = np.asarray(lens, dtype=np.uint32)
    best, t_end = float("inf"), time.perf_counter() + seconds
    while time.perf_counter() < t_end:
        t0 = time.perf_counter()
        ref.batch(img, o, n)
        best = min(best, time.perf_counter() - t0)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    lvkv = g.load_package()
    import oracle
    import log_synth
    import log_walk
    import sst_synth
    import sst_table
    dev = torch.device("cuda:0")
    ref = oracle.Reference() if oracle.reference_available() else None
    res = {}

    def report(name, nbytes, us, cpu_s, note):
        line = {"bytes": nbytes, "us_per_call": round(us, 2),
                "GBps": round(nbytes / us / 1e3, 1), "pct_hbm_peak": round(nbytes / us / 1e3 / 80.0, 2),
                "cpu_ref_1t_GBps": None if cpu_s is None else round(nbytes / cpu_s / 1e9, 2),
                "note": note}
        res[name] = line
        print(name, json.dumps(line), flush=True)

    for nblocks in (512, 16384):
        img = sst_synth.build_sst(nblocks, 4096, seed=nblocks, ragged=True)
        want = sst_table.verify_table(img)
        buf = torch.from_numpy(np.frombuffer(img, dtype=np.uint8).copy()).to(dev)
        rep, off, size, actual, status = lvkv.sst_verify_table(buf)
        assert rep["status"] == 0 and rep["nbad"] == 0 and rep["ndata"] == nblocks
        cap = rep["nblocks"] + 1
        o2 = torch.empty(cap, dtype=torch.int64, device=dev)
        s2 = torch.empty(cap, dtype=torch.int32, device=dev)
        a2 = torch.empty(cap, dtype=torch.int32, device=dev)
        st2 = torch.empty(cap, dtype=torch.uint8, device=dev)
        rp = torch.zeros(ctypes.sizeof(lvkv.SstReport), dtype=torch.uint8, device=dev)
        L = lvkv.lib
        vp = ctypes.c_void_p
        h = vp(torch.cuda.current_stream().cuda_stream)

        def call():
            rc = L.lvkv_sst_verify_table_device(vp(buf.data_ptr()), len(img), vp(o2.data_ptr()),
                                                vp(s2.data_ptr()), vp(a2.data_ptr()),
                                                vp(st2.data_ptr()), cap, lvkv.BLOOM_POLICY.encode(),
                                                vp(rp.data_ptr()), h)
            assert rc == 0
        us = timed(call, args.reps)
        handles = want.handles + [want.meta, want.index]
        cpu = cpu_rate(ref, np.frombuffer(img, dtype=np.uint8), [x for x, _ in handles],
                       [s + 1 for _, s in handles]) if ref else None
        report(f"sst_verify_table_{nblocks}x4KiB", len(img), us, cpu,
               "footer + index/metaindex verify + index parse + block verify + merge")
        # write side: wipe and refill every trailer of the same table
        offs = torch.tensor([x for x, _ in handles], dtype=torch.int64, device=dev)
        sizes = torch.tensor([s for _, s in handles], dtype=torch.int32, device=dev)
        crc = torch.empty(len(handles), dtype=torch.int32, device=dev)

        def fill():
            rc = L.lvkv_sst_fill_trailers_device(vp(buf.data_ptr()), vp(offs.data_ptr()),
                                                 vp(sizes.data_ptr()), vp(crc.data_ptr()),
                                                 len(handles), h)
            assert rc == 0
        us = timed(fill, args.reps)
        assert bytes(buf.cpu().numpy()) == img
        report(f"sst_fill_trailers_{nblocks}x4KiB", len(img), us, cpu,
               "Mask(CRC32C(contents + type)) written into every trailer")
        if nblocks == 16384:
            # the general-layout kernels side by side on the same table
            ab = {}
            for k in (-1, 0, 1, 2, 3, 4, 5, 6, 7):
                assert L.lvkv_debug_set_general_kernel(k) == 0
                ab[k] = (round(timed(call, args.reps), 2), round(timed(fill, args.reps), 2))
                assert bytes(buf.cpu().numpy()) == img
            L.lvkv_debug_set_general_kernel(0)
            res["general_kernel_ab_70MB_table"] = {
                "us_verify_table_fill": {str(k): v for k, v in ab.items()},
                "note": "-1 crc32c_kernel.hip; 0-3 crc32c_ragged.hip shapes (8x2x24, 8x3x16, 8x2x32, 8x3x24), +4: one round per workgroup"}
            print("general_kernel_ab", json.dumps(ab), flush=True)

    # compaction-input shape: 32 tables of ~2 MiB, one multi-table call vs
    # 32 single-table calls on one stream
    imgs = [sst_synth.build_sst(512, 4096, seed=100 + t) for t in range(32)]
    offs, pos = [], 0
    for im in imgs:
        offs.append(pos)
        pos += (len(im) + 255) // 256 * 256
    host = np.zeros(pos, dtype=np.uint8)
    for o_, im in zip(offs, imgs):
        host[o_: o_ + len(im)] = np.frombuffer(im, dtype=np.uint8)
    buf = torch.from_numpy(host).to(dev)
    sizes_t = [len(im) for im in imgs]
    tabs = lvkv.sst_verify_tables(buf, offs, sizes_t)
    assert all(r[0]["status"] == 0 and r[0]["nbad"] == 0 for r in tabs)
    L = lvkv.lib
    vp = ctypes.c_void_p
    h = vp(torch.cuda.current_stream().cuda_stream)
    d_toff = torch.tensor(offs, dtype=torch.int64, device=dev)
    d_tsz = torch.tensor(sizes_t, dtype=torch.int64, device=dev)
    tot = 32 * 600
    o3 = torch.empty(tot, dtype=torch.int64, device=dev)
    s3 = torch.empty(tot, dtype=torch.int32, device=dev)
    a3 = torch.empty(tot, dtype=torch.int32, device=dev)
    st3 = torch.empty(tot, dtype=torch.uint8, device=dev)
    rp3 = torch.zeros(32 * ctypes.sizeof(lvkv.SstReport), dtype=torch.uint8, device=dev)

    def multi():
        rc = L.lvkv_sst_verify_tables_device(
            vp(buf.data_ptr()), vp(d_toff.data_ptr()), vp(d_tsz.data_ptr()), 32,
            vp(o3.data_ptr()), vp(s3.data_ptr()), vp(a3.data_ptr()), vp(st3.data_ptr()), tot,
            lvkv.BLOOM_POLICY.encode(), vp(rp3.data_ptr()), h)
        assert rc == 0

    def single():
        for t in range(32):
            f = 600 * t
            rc = L.lvkv_sst_verify_table_device(
                vp(buf.data_ptr() + offs[t]), sizes_t[t], vp(o3.data_ptr() + 8 * f),
                vp(s3.data_ptr() + 4 * f), vp(a3.data_ptr() + 4 * f), vp(st3.data_ptr() + f),
                600, lvkv.BLOOM_POLICY.encode(),
                vp(rp3.data_ptr() + t * ctypes.sizeof(lvkv.SstReport)), h)
            assert rc == 0
    nbytes = sum(sizes_t)
    us_m = timed(multi, max(5, args.reps // 5))
    us_s = timed(single, max(5, args.reps // 5))
    report("sst_verify_tables_32x2MiB", nbytes, us_m, None,
           f"one multi-table call (2 launches); 32 single-table calls: {us_s:.1f} us")

    for nrec in (2000, 60000):
        img = log_synth.build_log(nrec, seed=nrec, max_len=2000, big_every=997)
        v = log_walk.block_verdicts(img)
        buf = torch.from_numpy(np.frombuffer(img, dtype=np.uint8).copy()).to(dev)
        rep, hdr, actual, rst, bst, bdrop = lvkv.log_verify_blocks(buf)
        assert rep["status"] == 0 and rep["ncorrupt"] == 0 and rep["nrecords"] == len(v.hdrs)
        cap = rep["nrecords"]
        nb = rep["nblocks"]
        vp = ctypes.c_void_p
        L = lvkv.lib
        h = vp(torch.cuda.current_stream().cuda_stream)
        hdr2 = torch.empty(cap, dtype=torch.int64, device=dev)
        act2 = torch.empty(cap, dtype=torch.int32, device=dev)
        rst2 = torch.empty(cap, dtype=torch.uint8, device=dev)
        bst2 = torch.empty(nb, dtype=torch.uint8, device=dev)
        bd2 = torch.empty(nb, dtype=torch.int32, device=dev)
        rp = torch.zeros(64, dtype=torch.uint8, device=dev)

        def call():
            rc = L.lvkv_log_verify_blocks_device(vp(buf.data_ptr()), len(img), vp(hdr2.data_ptr()),
                                                 vp(act2.data_ptr()), vp(rst2.data_ptr()), cap,
                                                 vp(bst2.data_ptr()), vp(bd2.data_ptr()),
                                                 vp(rp.data_ptr()), h)
            assert rc == 0
        us = timed(call, args.reps)
        lens = [1 + (img[x + 4] | img[x + 5] << 8) for x in v.hdrs]
        cpu = cpu_rate(ref, np.frombuffer(img, dtype=np.uint8), [x + 6 for x in v.hdrs],
                       lens) if ref else None
        report(f"log_verify_blocks_{nrec}rec", len(img), us, cpu,
               f"{nb} blocks, {cap} records: one launch: stage, walk, place, checksum, merge")

        def fill():
            rc = L.lvkv_log_fill_headers_device(vp(buf.data_ptr()), vp(hdr.data_ptr()), None,
                                                cap, h)
            assert rc == 0
        us = timed(fill, args.reps)
        assert bytes(buf.cpu().numpy()) == img
        report(f"log_fill_headers_{nrec}rec", len(img), us, cpu,
               "Mask(CRC32C(type + payload)) written into every header")

    if args.json:
        Path(args.json).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
