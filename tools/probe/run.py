"""Run the headline-kernel timing probes (GPU box). Not part of the product.

    python tools/probe/run.py [cfg ...] [--streams=S] [--K=N] [--warm=MS]

For every cfg: a parity check against the product entry (burst variants that
compute CRCs), then probe_time (see probe.hip). Writes gpurun_out/probe.json.
"""
from __future__ import annotations

import ctypes
import json
import sys
from pathlib import Path

import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO))
import __graft_entry__ as g  # noqa: E402

lvkv = g.load_package()
P = ctypes.CDLL(str(HERE / "libprobe.so"))
vp = ctypes.c_void_p
P.probe_time.argtypes = [ctypes.c_int, ctypes.c_int, vp, ctypes.c_uint64, ctypes.c_int,
                         ctypes.c_uint32, ctypes.c_uint32, vp, ctypes.c_int, ctypes.c_int,
                         ctypes.c_double, ctypes.POINTER(ctypes.c_double)]
P.probe_launch.argtypes = [ctypes.c_int, ctypes.c_int, vp, ctypes.c_uint32, ctypes.c_uint32, vp,
                           vp, vp]

NAMES = {0: "burst 8x3x2", 1: "burst late (compact order)", 2: "bare 8x3x2", 3: "no build",
         4: "no walk", 5: "rows from HBM", 6: "default policy", 7: "burst 8x5 (1 WG/CU)",
         8: "bare 8x5", 9: "burst 16x3x1", 10: "bare 16x3x1", 11: "stamps",
         12: "no build, no walk", 13: "burst 8x4x2", 14: "late 8x4x2",
         15: "split2 8x3x2", 16: "split4 8x3x2", 17: "split2 8x5 (1 WG/CU)",
         18: "split4 8x5", 19: "split2 late",
         100: "product lvkv_crc32c_uniform_device", 101: "read-only x4 kernel"}
CORRECT = {0, 1, 5, 6, 7, 9, 11, 13, 14, 15, 16, 17, 18, 19, 100}


def arg(name, default):
    for a in sys.argv[1:]:
        if a.startswith(f"--{name}="):
            return type(default)(a.split("=", 1)[1])
    return default


def main():
    cfgs = [int(a) for a in sys.argv[1:] if not a.startswith("--")] or [100, 0, 1, 2, 101]
    S, K, warm = arg("streams", 2), arg("K", 400), arg("warm", 150.0)
    nb, L = arg("nb", 10_000), arg("len", 4096)
    groups = arg("groups", 0)
    dev = torch.device("cuda:0")
    win = nb * L
    nrot = max(2, -(-int(1.25 * (1 << 30)) // win))
    buf = torch.randint(0, 256, (nrot * win,), dtype=torch.uint8, device=dev)
    out = torch.zeros(2 * nb, dtype=torch.int32, device=dev)
    ref = torch.zeros(nb, dtype=torch.int32, device=dev)
    lvkv.lib.lvkv_crc32c_uniform_device(vp(buf.data_ptr()), L, L, 0, vp(ref.data_ptr()), nb, 0,
                                        vp(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    if "--single" in sys.argv:  # profiling: K launches per cfg on one stream
        P.probe_single.argtypes = [ctypes.c_int, ctypes.c_int, vp, ctypes.c_uint64, ctypes.c_int,
                                   ctypes.c_uint32, ctypes.c_uint32, vp, ctypes.c_int]
        for cfg in cfgs:
            assert P.probe_single(cfg, groups, vp(buf.data_ptr()), win, nrot, L, nb,
                                  vp(out.data_ptr()), K) == 0
        return
    res = {}
    for cfg in cfgs:
        if cfg in CORRECT and cfg < 100:
            out.zero_()
            rc = P.probe_launch(cfg, groups, vp(buf.data_ptr()), L, nb, vp(out.data_ptr()), None,
                                vp(torch.cuda.current_stream().cuda_stream))
            torch.cuda.synchronize()
            assert rc == 0, (cfg, rc)
            ok = bool(torch.equal(out[:nb], ref))
            assert ok, f"cfg {cfg}: parity FAILED"
        r = (ctypes.c_double * 4)()
        rc = P.probe_time(cfg, groups, vp(buf.data_ptr()), win, nrot, L, nb, vp(out.data_ptr()), K,
                          S, warm, r)
        assert rc == 0, (cfg, rc)
        algo = nb * (L + 4)
        row = {"name": NAMES.get(cfg, str(cfg)), "single_us": round(r[0], 3),
               f"period_{S}s_us": round(r[1], 3), "host20_us": round(r[2], 3),
               f"host{K}_us": round(r[3], 3),
               "single_frac": round(algo / (r[0] * 1e-6) / 8e12, 4),
               "period_frac": round(algo / (r[1] * 1e-6) / 8e12, 4),
               "host20_pct": round(100 * nb * L / (r[2] * 1e-6) / 8e12, 2)}
        res[cfg] = row
        print(cfg, json.dumps(row), flush=True)
    outp = REPO / "gpurun_out"
    outp.mkdir(exist_ok=True)
    tag = arg("tag", "probe")
    (outp / f"{tag}.json").write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
