"""WAL verify timing (GPU box). Not part of the product.

    python tools/probe/log_probe.py [nrec]

The synthetic 60k-record log of tools/paths_bench.py through
lvkv_log_verify_blocks_device: host time per call (back to back, one stream)
and, with rocprofv3 around it, the kernels' own durations.
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
import log_synth  # noqa: E402

lvkv = g.load_package()


def main():
    nrec = int(sys.argv[1]) if len(sys.argv) > 1 else 60000
    img = log_synth.build_log(nrec, seed=nrec, max_len=2000, big_every=997)
    dev = torch.device("cuda:0")
    buf = torch.from_numpy(np.frombuffer(img, dtype=np.uint8).copy()).to(dev)
    rep, *_ = lvkv.log_verify_blocks(buf)
    cap = rep["nrecords"] + 1
    nb = rep["nblocks"]
    hdr = torch.empty(cap, dtype=torch.int64, device=dev)
    act = torch.empty(cap, dtype=torch.int32, device=dev)
    rst = torch.empty(cap, dtype=torch.uint8, device=dev)
    bst = torch.empty(nb, dtype=torch.uint8, device=dev)
    bdr = torch.empty(nb, dtype=torch.int32, device=dev)
    rp = torch.zeros(64, dtype=torch.uint8, device=dev)
    vp = ctypes.c_void_p
    h = vp(torch.cuda.current_stream().cuda_stream)
    L = lvkv.lib

    def call():
        rc = L.lvkv_log_verify_blocks_device(vp(buf.data_ptr()), len(img), vp(hdr.data_ptr()),
                                             vp(act.data_ptr()), vp(rst.data_ptr()), cap,
                                             vp(bst.data_ptr()), vp(bdr.data_ptr()),
                                             vp(rp.data_ptr()), h)
        assert rc == 0
    for _ in range(5):
        call()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        call()
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / 50 * 1e6
    if "--stamps" in sys.argv:
        # phase stamps from the probe build of the library
        P = ctypes.CDLL(str(HERE / "liblvkv_probe.so"))
        P.lvkv_debug_log_stamps.argtypes = [vp]
        st = torch.zeros(256 * 16 * 8, dtype=torch.int64, device=dev)
        P.lvkv_debug_log_stamps(vp(st.data_ptr()))
        P.lvkv_log_verify_blocks_device.argtypes = [vp, ctypes.c_uint64, vp, vp, vp,
                                                    ctypes.c_size_t, vp, vp, vp, vp]
        knobs = int(next((x.split("=")[1] for x in sys.argv if x.startswith("--knobs=")), 0))
        P.lvkv_debug_log_knobs.argtypes = [ctypes.c_uint32]
        P.lvkv_debug_log_knobs(knobs)
        print("knobs", knobs, flush=True)
        for _ in range(3):
            st.zero_()
            torch.cuda.synchronize()
            rc = P.lvkv_log_verify_blocks_device(vp(buf.data_ptr()), len(img), vp(hdr.data_ptr()),
                                                 vp(act.data_ptr()), vp(rst.data_ptr()), cap,
                                                 vp(bst.data_ptr()), vp(bdr.data_ptr()),
                                                 vp(rp.data_ptr()), h)
            assert rc == 0
            torch.cuda.synchronize()
        # A/B in this process: the probe library with the knob, unstamped
        P.lvkv_debug_log_stamps(None)
        for kn in (0, knobs):
            P.lvkv_debug_log_knobs(kn)
            for _ in range(5):
                P.lvkv_log_verify_blocks_device(vp(buf.data_ptr()), len(img), vp(hdr.data_ptr()),
                                                vp(act.data_ptr()), vp(rst.data_ptr()), cap,
                                                vp(bst.data_ptr()), vp(bdr.data_ptr()),
                                                vp(rp.data_ptr()), h)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(50):
                P.lvkv_log_verify_blocks_device(vp(buf.data_ptr()), len(img), vp(hdr.data_ptr()),
                                                vp(act.data_ptr()), vp(rst.data_ptr()), cap,
                                                vp(bst.data_ptr()), vp(bdr.data_ptr()),
                                                vp(rp.data_ptr()), h)
            torch.cuda.synchronize()
            ab = (time.perf_counter() - t1) / 50 * 1e6
            a_ = act.cpu().numpy().copy() if kn == 0 else None
            if kn == 0:
                ref_act, ref_rst = act.cpu().numpy().copy(), rst.cpu().numpy().copy()
            else:
                same = (np.array_equal(ref_act, act.cpu().numpy()) and
                        np.array_equal(ref_rst, rst.cpu().numpy()))
                print(f"  outputs equal to knob 0: {same}", flush=True)
            print(f"  probe lib knobs {kn}: {ab:.1f} us/call", flush=True)
        P.lvkv_debug_log_knobs(knobs)
        x = st.cpu().numpy().reshape(256, 16, 8).astype(np.int64)
        t0 = x[:, 0, 0][x[:, 0, 0] > 0].min()
        for k in range(9):
            row = x[:, k, :]
            ok = row[:, 0] > 0
            if not ok.any():
                break
            rel = (row[ok] - t0) / 100.0
            med = np.median(rel, axis=0)
            print(f"iter {k}: start {med[0]:.2f} placed {med[1]:.2f} walked {med[2]:.2f} "
                  f"w2first {med[7]:.2f} w2done {med[3]:.2f} recs {med[4]:.2f} long {med[5]:.2f} merged {med[6]:.2f} "
                  f"(max merged {rel[:, 6].max():.2f})", flush=True)
    print(f"log_verify {nrec} records, {len(img)} bytes, {nb} blocks: {us:.1f} us/call, "
          f"{len(img) / us / 1e3:.1f} GB/s", flush=True)
    if "--read" in sys.argv:
        # verify + the logical layer (lvkv_log_read_device)
        recs = torch.zeros(cap * 24, dtype=torch.uint8, device=dev)
        reps = torch.zeros((cap + nb) * 16, dtype=torch.uint8, device=dev)
        rd = torch.zeros(64, dtype=torch.uint8, device=dev)

        def read():
            rc = L.lvkv_log_read_device(vp(buf.data_ptr()), len(img), vp(hdr.data_ptr()),
                                        vp(act.data_ptr()), vp(rst.data_ptr()), cap,
                                        vp(bst.data_ptr()), vp(bdr.data_ptr()), vp(rp.data_ptr()),
                                        vp(recs.data_ptr()), cap, vp(reps.data_ptr()), cap + nb,
                                        0, vp(rd.data_ptr()), h)
            assert rc == 0
        for _ in range(5):
            read()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(50):
            read()
        torch.cuda.synchronize()
        us2 = (time.perf_counter() - t0) / 50 * 1e6
        print(f"log_read {nrec} records: {us2:.1f} us/call (verify + ReadRecord)", flush=True)


if __name__ == "__main__":
    main()
