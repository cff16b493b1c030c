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
        # manager phase stamps from the probe build of the library: per
        # (workgroup, slot, block k) 0 claimed, 1 in LDS, 2 walked, 3 placed,
        # 4 CRCs done, 5 emitted (s_memrealtime, 100 MHz)
        P = ctypes.CDLL(str(HERE / "liblvkv_probe.so"))
        P.lvkv_debug_log_stamps.argtypes = [vp]
        nsl = int(next((x.split('=')[1] for x in sys.argv if x.startswith('--slots=')), 3))
        st = torch.zeros(256 * 4 * 16 * 8, dtype=torch.int64, device=dev)
        P.lvkv_debug_log_stamps(vp(st.data_ptr()))
        P.lvkv_log_verify_blocks_device.argtypes = [vp, ctypes.c_uint64, vp, vp, vp,
                                                    ctypes.c_size_t, vp, vp, vp, vp]
        P.lvkv_debug_log_knobs.argtypes = [ctypes.c_uint32]
        knobs = int(next((x.split("=")[1] for x in sys.argv if x.startswith("--knobs=")), 0))
        P.lvkv_debug_log_knobs(knobs)
        for _ in range(3):
            st.zero_()
            torch.cuda.synchronize()
            rc = P.lvkv_log_verify_blocks_device(vp(buf.data_ptr()), len(img), vp(hdr.data_ptr()),
                                                 vp(act.data_ptr()), vp(rst.data_ptr()), cap,
                                                 vp(bst.data_ptr()), vp(bdr.data_ptr()),
                                                 vp(rp.data_ptr()), h)
            assert rc == 0
            torch.cuda.synchronize()
        P.lvkv_debug_log_stamps(None)
        # unstamped A/B in this process: knob 0 against the knobs asked for
        for kn in sorted({0, knobs}):
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
            print(f"  probe lib knobs {kn}: {(time.perf_counter() - t1) / 50 * 1e6:.1f} us/call",
                  flush=True)
        P.lvkv_debug_log_knobs(0)
        print(f"stamps below: knobs {knobs}", flush=True)
        x = st.cpu().numpy()[:256 * nsl * 16 * 8].reshape(256, nsl, 16, 8).astype(np.int64)
        t0 = x[:, 0, 15, 0][x[:, 0, 15, 0] > 0].min()
        w = x[:, 0, 15, :]
        ok = w[:, 0] > 0
        rel = (w[ok] - t0) / 100.0
        print("workgroups: start min/med/max %.2f/%.2f/%.2f, image built med %.2f, "
              "done min/med/max %.2f/%.2f/%.2f" % (
                  rel[:, 0].min(), np.median(rel[:, 0]), rel[:, 0].max(), np.median(rel[:, 1]),
                  rel[:, 2].min(), np.median(rel[:, 2]), rel[:, 2].max()), flush=True)
        names = ["claim", "dma", "walk", "crcs", "staged"]
        for k in range(6):
            row = x[:, :, k, :].reshape(-1, 8)
            ok = row[:, 0] > 0
            if not ok.any():
                break
            rel = (row[ok] - t0) / 100.0
            med = np.median(rel, axis=0)
            d = np.median(np.diff(rel[:, :5], axis=1), axis=0)
            wl = row[ok][:, 5] > 0
            if wl.any():
                r5 = (row[ok][wl] - t0) / 100.0
                print(f"   walk split: window {np.median(r5[:, 5] - r5[:, 1]):.2f} loop "
                      f"{np.median(r5[:, 6] - r5[:, 5]):.2f} tail {np.median(r5[:, 2] - r5[:, 6]):.2f}",
                      flush=True)
            print(f"block {k}: claimed at {med[0]:.2f} us; phases " +
                  " ".join(f"{n}+{v:.2f}" for n, v in zip(names[1:], d)) +
                  f"; staged at {med[4]:.2f} (max {rel[:, 4].max():.2f}, n {ok.sum()})", flush=True)
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
        if "--asm-stamps" in sys.argv:
            # log_asm_emit phases per workgroup (probe build; s_memrealtime,
            # 100 MHz): 0 start, 1 shares and items summed, 2 barrier 1, 3 counts
            # (barrier 2), 5 written
            P = ctypes.CDLL(str(HERE / "liblvkv_probe.so"))
            P.lvkv_debug_asm_stamps.argtypes = [vp]
            P.lvkv_log_read_device.argtypes = L.lvkv_log_read_device.argtypes
            st = torch.zeros(4096 * 8, dtype=torch.int64, device=dev)
            P.lvkv_debug_asm_stamps(vp(st.data_ptr()))
            for _ in range(3):
                st.zero_()
                torch.cuda.synchronize()
                assert P.lvkv_log_read_device(vp(buf.data_ptr()), len(img), vp(hdr.data_ptr()),
                                              vp(act.data_ptr()), vp(rst.data_ptr()), cap,
                                              vp(bst.data_ptr()), vp(bdr.data_ptr()),
                                              vp(rp.data_ptr()), vp(recs.data_ptr()), cap,
                                              vp(reps.data_ptr()), cap + nb, 0, vp(rd.data_ptr()),
                                              h) == 0
                torch.cuda.synchronize()
            P.lvkv_debug_asm_stamps(None)
            x = st.cpu().numpy().reshape(-1, 8)
            x = x[x[:, 0] > 0]
            t0s = x[:, 0].min()
            rel = (x - t0s) / 100.0
            print(f"asm emit workgroups {len(x)}: start max {rel[:, 0].max():.2f}; med phases "
                  f"shares+items {np.median(rel[:, 1] - rel[:, 0]):.2f}, barrier 1 "
                  f"+{np.median(rel[:, 2] - rel[:, 1]):.2f}, counts+barrier 2 "
                  f"+{np.median(rel[:, 3] - rel[:, 2]):.2f}, step+write "
                  f"+{np.median(rel[:, 5] - rel[:, 3]):.2f}; end max {rel[:, 5].max():.2f}",
                  flush=True)
        # + the records' bytes laid end to end (lvkv_log_gather_device)
        payload = torch.empty(len(img), dtype=torch.uint8, device=dev)
        rpos = torch.empty(cap, dtype=torch.int64, device=dev)
        L.lvkv_log_gather_device.argtypes = [vp, vp, ctypes.c_size_t, vp, vp, ctypes.c_size_t, vp,
                                             vp, ctypes.c_uint64, vp, vp]

        def gather():
            rc = L.lvkv_log_gather_device(vp(buf.data_ptr()), vp(hdr.data_ptr()), cap,
                                          vp(rp.data_ptr()), vp(recs.data_ptr()), cap,
                                          vp(rd.data_ptr()), vp(payload.data_ptr()), len(img),
                                          vp(rpos.data_ptr()), h)
            assert rc == 0
        for _ in range(5):
            gather()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(50):
            gather()
        torch.cuda.synchronize()
        us3 = (time.perf_counter() - t0) / 50 * 1e6
        print(f"log_gather {nrec} records: {us3:.1f} us/call", flush=True)


if __name__ == "__main__":
    main()
