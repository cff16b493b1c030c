"""Host-timed region overhead vs K (GPU box). Not part of the product.

    python tools/probe/host_sweep.py [--spin] [cfg]
--spin: hipSetDeviceFlags(hipDeviceScheduleSpin) before the HIP context exists.
"""
import ctypes
import json
import os
import sys
from pathlib import Path

if "--spin" in sys.argv:
    hip = ctypes.CDLL("libamdhip64.so")
    print("hipSetDeviceFlags(spin) ->", hip.hipSetDeviceFlags(1), flush=True)

import torch  # noqa: E402

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO))
import __graft_entry__ as g  # noqa: E402

lvkv = g.load_package()
P = ctypes.CDLL(str(HERE / "libprobe.so"))
vp = ctypes.c_void_p
P.probe_host_sweep.argtypes = [ctypes.c_int, ctypes.c_int, vp, ctypes.c_uint64, ctypes.c_int,
                               ctypes.c_uint32, ctypes.c_uint32, vp, ctypes.c_int, ctypes.c_int,
                               ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                               ctypes.POINTER(ctypes.c_double)]
P.probe_latency.argtypes = [ctypes.POINTER(ctypes.c_double)]
lat = (ctypes.c_double * 6)()
assert P.probe_latency(lat) == 0
print("latency us: devsync_idle %.1f streamsync_idle %.1f empty_spin %.1f empty_devsync %.1f "
      "launch_call %.1f empty_streamsync %.1f" % tuple(lat), flush=True)
cfgs = [int(a) for a in sys.argv[1:] if not a.startswith("--")] or [100]
nb, L = 10_000, 4096
win = nb * L
nrot = 33
dev = torch.device("cuda:0")
buf = torch.randint(0, 256, (nrot * win,), dtype=torch.uint8, device=dev)
out = torch.zeros(2 * nb, dtype=torch.int32, device=dev)
P.probe_region.argtypes = [ctypes.c_int, ctypes.c_int, vp, ctypes.c_uint64, ctypes.c_int,
                           ctypes.c_uint32, ctypes.c_uint32, vp, ctypes.c_int,
                           ctypes.POINTER(ctypes.c_double)]
for cfg in cfgs:
    for K in (1, 20):
        rr = (ctypes.c_double * 16)()
        assert P.probe_region(cfg, 0, vp(buf.data_ptr()), win, nrot, L, nb, vp(out.data_ptr()), K,
                              rr) == 0
        for prep, name in enumerate(["none", "warm", "warm+prime", "warm+2ms"]):
            print(f"region cfg {cfg} K {K} prep {name}: total %.1f issue %.1f device %.1f "
                  f"wait %.1f" % tuple(rr[prep * 4: prep * 4 + 4]), flush=True)
P.probe_graph.argtypes = [ctypes.c_int, ctypes.c_int, vp, ctypes.c_uint64, ctypes.c_int,
                          ctypes.c_uint32, ctypes.c_uint32, vp, ctypes.c_int, ctypes.c_int,
                          ctypes.POINTER(ctypes.c_double)]
for cfg in cfgs:
    for K in (20, 100):
        for S in (1, 2, 3):
            rr = (ctypes.c_double * 4)()
            rc = P.probe_graph(cfg, 0, vp(buf.data_ptr()), win, nrot, L, nb, vp(out.data_ptr()),
                               K, S, rr)
            print(f"graph cfg {cfg} K {K} streams {S}: rc {rc} host/step %.2f device/step %.2f "
                  f"launch_call %.1f inst_ms %.2f" % tuple(rr), flush=True)
if "--graph-only" in sys.argv:
    sys.exit(0)
ks = [1, 2, 5, 10, 20, 40, 100]
karr = (ctypes.c_int * len(ks))(*ks)
res = {}
for cfg in cfgs:
    for mode in (0, 1):
        r = (ctypes.c_double * len(ks))()
        rc = P.probe_host_sweep(cfg, 0, vp(buf.data_ptr()), win, nrot, L, nb, vp(out.data_ptr()),
                                2, mode, karr, len(ks), r)
        assert rc == 0, rc
        row = {k: round(v, 2) for k, v in zip(ks, r)}
        res[f"{cfg}/{mode}"] = row
        print(cfg, mode, json.dumps(row), flush=True)
tag = ("spin" if "--spin" in sys.argv else "default") + os.environ.get("SWEEP_TAG", "")
(REPO / "gpurun_out").mkdir(exist_ok=True)
(REPO / "gpurun_out" / f"host_sweep_{tag}.json").write_text(json.dumps(res, indent=1))
