"""Does a queue parked on a barrier packet start the next dispatch sooner?
(GPU box; not part of the product.)

    python tools/probe/gate_probe.py

The K = 20 region of tools/probe/edges.py, twice, interleaved: as bench.py
runs it, and with every engine queue first parked on a barrier-AND packet
that waits on a signal (lvkv_debug_engine_stall(1)); the first submit goes
behind it, then the signal opens the queues (stall(0)) and the other submits
follow. Reports t0 -> first dispatch start and the host time of the region
(HSA clock), medians of 15 each. Writes gpurun_out/gate_probe.json.
"""
import ctypes
import json
import statistics
import sys
import time
from pathlib import Path

import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO))
import __graft_entry__ as g  # noqa: E402

lvkv = g.load_package()
hsa = ctypes.CDLL("libhsa-runtime64.so.1")
hsa.hsa_system_get_info.argtypes = [ctypes.c_int, ctypes.c_void_p]
lvkv.lib.lvkv_debug_engine_stall.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_double]
lvkv.lib.lvkv_engine_set_final_variant.argtypes = [ctypes.c_void_p, ctypes.c_int]


def now_us():
    v = ctypes.c_uint64()
    hsa.hsa_system_get_info(2, ctypes.byref(v))
    return v.value * 1e-3


def main():
    nb, Lb, nrot = 10_000, 4096, 33
    dev = torch.device("cuda:0")
    win = nb * Lb
    buf = torch.randint(0, 256, (nrot * win,), dtype=torch.uint8, device=dev)
    out = torch.zeros(nb, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    eng = lvkv.Engine(0)
    sub, h = eng.submit_ptr, eng.handle
    stall = lvkv.lib.lvkv_debug_engine_stall
    rot = [0]

    def step(final=False):
        rot[0] += 1
        rc = sub(h, buf.data_ptr() + (rot[0] % nrot) * win, Lb, Lb, 0, out.data_ptr(), nb,
                 8 if final else 0)
        assert rc == 0

    K = 20
    modes = ["plain", "gated", "final_pair", "gated_final_pair"]
    res = {m: [] for m in modes}
    for rep in range(60):
        mode = modes[rep % 4]
        gated = mode.startswith("gated")
        assert lvkv.lib.lvkv_engine_set_final_variant(h, 1 if "final_pair" in mode else -1) == 0
        for _ in range(40):
            step()
        eng.wait()
        torch.cuda.synchronize()
        for prof in (False, True):
            if prof:
                eng.profile(True)
            if gated:
                assert stall(h, 1, 60.0) == 0
                time.sleep(0.0002)  # the packet processors reach the barriers
            torch.cuda.synchronize()
            t0 = now_us()
            step()
            if gated:
                stall(h, 0, 60.0)
            for k in range(1, K):
                step(final=k >= K - 3)
            eng.wait()
            torch.cuda.synchronize()
            t1 = now_us()
            if prof:
                sp = eng.profile_read()
                eng.profile(False)
                res[mode][-1].update({"t0_to_first_start": sp[0][0] - t0, "span": max(b for _, b in sp) - sp[0][0],
                                      "last_dur": sp[-1][1] - sp[-1][0]})
            else:
                res[mode].append({"host_us": t1 - t0})
    agg = {k: {f: round(statistics.median(r[f] for r in v), 3) for f in v[0]} for k, v in res.items()}
    print(json.dumps(agg), flush=True)
    (REPO / "gpurun_out").mkdir(exist_ok=True)
    (REPO / "gpurun_out" / "gate_probe.json").write_text(json.dumps({"median": agg, "runs": res}, indent=1))
    eng.close()


if __name__ == "__main__":
    main()
