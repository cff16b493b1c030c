"""Whole-SSTable verify timing (GPU box). Not part of the product.

    python tools/probe/sst_probe.py [nblocks] [--form=0|1|2] [--tables=K]

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


def opt(name, default):
    return int(next((x.split("=")[1] for x in sys.argv if x.startswith(f"--{name}=")), default))


def multi(nblocks, k):
    # k copies of one table in one buffer, back-to-back lvkv_sst_verify_tables_device calls
    img = sst_synth.build_sst(nblocks, 4096, seed=nblocks, ragged=True)
    dev = torch.device("cuda:0")
    offs = [i * (len(img) + 13) for i in range(k)]
    raw = bytearray(offs[-1] + len(img))
    for o in offs:
        raw[o: o + len(img)] = img
    buf = torch.from_numpy(np.frombuffer(bytes(raw), dtype=np.uint8).copy()).to(dev)
    res = lvkv.sst_verify_tables(buf, offs, [len(img)] * k)
    assert all(r[0]["status"] == 0 and r[0]["nbad"] == 0 for r in res)
    cap = k * (res[0][0]["nblocks"] + 1)
    toff = torch.tensor(offs, dtype=torch.int64, device=dev)
    tsz = torch.tensor([len(img)] * k, dtype=torch.int64, device=dev)
    o = torch.empty(cap, dtype=torch.int64, device=dev)
    sz = torch.empty(cap, dtype=torch.int32, device=dev)
    ac = torch.empty(cap, dtype=torch.int32, device=dev)
    st = torch.empty(cap, dtype=torch.uint8, device=dev)
    rp = torch.zeros(k * ctypes.sizeof(lvkv.SstReport), dtype=torch.uint8, device=dev)
    vp = ctypes.c_void_p
    h = vp(torch.cuda.current_stream().cuda_stream)
    pol = lvkv.BLOOM_POLICY.encode()

    def call():
        rc = lvkv.lib.lvkv_sst_verify_tables_device(
            vp(buf.data_ptr()), vp(toff.data_ptr()), vp(tsz.data_ptr()), k, vp(o.data_ptr()),
            vp(sz.data_ptr()), vp(ac.data_ptr()), vp(st.data_ptr()), cap, pol, vp(rp.data_ptr()), h)
        assert rc == 0
    for _ in range(5):
        call()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        call()
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / 50 * 1e6
    print(f"sst_verify_tables form {opt('form', 0)}, {k} x {nblocks} blocks, {len(raw)} bytes: "
          f"{us:.1f} us/call", flush=True)
    if "--stamps" in sys.argv:
        P = probe_lib(opt("form", 0))
        P.lvkv_sst_verify_tables_device.argtypes = L_TABLES_ARGS
        stz = torch.zeros(16 * k, dtype=torch.int64, device=dev)
        P.lvkv_debug_sst_stamps(vp(stz.data_ptr()))
        rows = []
        for _ in range(8):
            stz.zero_()
            torch.cuda.synchronize()
            assert P.lvkv_sst_verify_tables_device(
                vp(buf.data_ptr()), vp(toff.data_ptr()), vp(tsz.data_ptr()), k, vp(o.data_ptr()),
                vp(sz.data_ptr()), vp(ac.data_ptr()), vp(st.data_ptr()), cap, pol,
                vp(rp.data_ptr()), h) == 0
            torch.cuda.synchronize()
            x = stz.cpu().numpy().astype(np.int64).reshape(k, 16)
            t0 = x[:, 0][x[:, 0] > 0].min()
            rows.append(np.where(x > 0, (x - t0) / 100.0, np.nan))
        r = np.array(rows)  # runs x tables x slots
        med0 = np.nanmedian(r[:, 0, :], axis=0)
        print("  table 0: " + "  ".join(f"{n} {v:.2f}" for n, v in zip(STAMP_NAMES, med0)
                                         if not np.isnan(v)), flush=True)
        mx = np.nanmedian(np.nanmax(r, axis=1), axis=0)
        print("  max over tables: " + "  ".join(f"{n} {v:.2f}" for n, v in zip(STAMP_NAMES, mx)
                                                 if not np.isnan(v)), flush=True)
        P.lvkv_debug_sst_stamps(None)


# phase stamps (tools/probe build): head slots 0-7; the CRC workgroups' 8-12
# (speculative form: table t's first CRC workgroup; fused: the first one)
STAMP_NAMES = ["start", "footer", "crcs", "verdicts", "staged", "filter", "placed", "done",
               "crc_share", "crc_decoded", "crc_walked", "crc_head_seen", "crc_stored"]
L_TABLES_ARGS = [ctypes.c_void_p] * 3 + [ctypes.c_size_t] + [ctypes.c_void_p] * 4 + [
    ctypes.c_size_t, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p]


def probe_lib(form):
    vp = ctypes.c_void_p
    P = ctypes.CDLL(str(HERE / "liblvkv_probe.so"))
    P.lvkv_debug_sst_stamps.argtypes = [vp]
    P.lvkv_debug_set_sst_form.argtypes = [ctypes.c_int]
    P.lvkv_debug_set_sst_form(form)
    return P


def main():
    nblocks = int(sys.argv[1]) if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else 16384
    form = opt("form", 0)
    assert lvkv.lib.lvkv_debug_set_sst_form(form) == 0
    if opt("tables", 0):
        return multi(nblocks, opt("tables", 0))
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
    print(f"sst_verify form {form}, {nblocks} blocks, {len(img)} bytes: {us:.1f} us/call",
          flush=True)
    if "--stamps" in sys.argv:
        # phase stamps from the probe build (10 ns units -> us from the head's start)
        P = probe_lib(form)
        P.lvkv_sst_verify_table_device.argtypes = [vp, ctypes.c_uint64, vp, vp, vp, vp,
                                                   ctypes.c_size_t, ctypes.c_char_p, vp, vp]
        stz = torch.zeros(16, dtype=torch.int64, device=dev)
        P.lvkv_debug_sst_stamps(vp(stz.data_ptr()))
        rows = []
        for _ in range(8):
            stz.zero_()
            torch.cuda.synchronize()
            rc = P.lvkv_sst_verify_table_device(vp(buf.data_ptr()), len(img), vp(o.data_ptr()),
                                                vp(sz.data_ptr()), vp(ac.data_ptr()),
                                                vp(st.data_ptr()), cap, pol, vp(rp.data_ptr()), h)
            assert rc == 0
            torch.cuda.synchronize()
            x = stz.cpu().numpy().astype(np.int64)
            rows.append([(v - x[0]) / 100.0 if v else float("nan") for v in x[:13]])
        med = np.nanmedian(np.array(rows), axis=0)
        names = STAMP_NAMES if form == 3 else STAMP_NAMES[:8] + [
            "crc_wg_waited", "crc_wg_end", "crc_wg_image"]
        print("  " + "  ".join(f"{n} {v:.2f}" for n, v in zip(names, med) if not np.isnan(v)),
              flush=True)
        P.lvkv_debug_sst_stamps(None)


if __name__ == "__main__":
    main()
