"""Where the edges of a short bench region go (GPU box). Not part of the
product.

    python tools/probe/edges.py

The bench's timed region (sync, t0, K engine submits, wait, sync, t1) with
the HSA system clock read on the host at each point, next to the packet
processor's start/end of every dispatch (the same clock): host submit time,
t0 -> first dispatch start, last dispatch end -> wait return -> sync return.
Writes gpurun_out/edges.json.
"""
import ctypes
import json
import statistics
import sys
from pathlib import Path

import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO))
import __graft_entry__ as g  # noqa: E402

lvkv = g.load_package()
hsa = ctypes.CDLL("libhsa-runtime64.so.1")
hsa.hsa_system_get_info.argtypes = [ctypes.c_int, ctypes.c_void_p]


def now_us():
    v = ctypes.c_uint64()
    hsa.hsa_system_get_info(2, ctypes.byref(v))  # HSA_SYSTEM_INFO_TIMESTAMP
    return v.value * 1e-3  # 1 GHz system timestamp -> us


def main():
    nb, Lb = 10_000, 4096
    dev = torch.device("cuda:0")
    win = nb * Lb
    nrot = 33
    buf = torch.randint(0, 256, (nrot * win,), dtype=torch.uint8, device=dev)
    out = torch.zeros(nb, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    eng = lvkv.Engine(0)
    f = ctypes.c_uint64()
    hsa.hsa_system_get_info(3, ctypes.byref(f))
    assert f.value == 1_000_000_000, f.value
    sub, h = eng.submit_ptr, eng.handle
    rot = [0]

    fin = [0]

    def step(n=nb, final=False):
        rot[0] += 1
        sub(h, buf.data_ptr() + (rot[0] % nrot) * win, Lb, Lb, 0, out.data_ptr(), n,
            8 if (final and fin[0]) else 0)  # LVKV_FLAG_FINAL on the last submit per queue

    res = {}
    lvkv.lib.lvkv_engine_set_scopes.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                 ctypes.c_int]
    scopes = [tuple(int(x) for x in a.split("=", 1)[1].split(","))
              for a in sys.argv if a.startswith("--scopes=")] or [(2, 2, 2)]
    lvkv.lib.lvkv_engine_set_priority.argtypes = [ctypes.c_void_p, ctypes.c_int]
    for sc in scopes:
        assert lvkv.lib.lvkv_engine_set_priority(h, sc[3] if len(sc) > 3 else 1) == 0
        assert lvkv.lib.lvkv_engine_set_scopes(h, *sc[:3]) == 0
        for f in (0, 1):
            fin[0] = f
            res[f"scopes_{sc}_final{f}"] = run_set(eng, step, (sc, f"final={f}"))
    (REPO / "gpurun_out").mkdir(exist_ok=True)
    (REPO / "gpurun_out" / "edges.json").write_text(json.dumps(res, indent=1))


def run_set(eng, step, sc):
    res = {}
    # idle costs
    ts = []
    for _ in range(50):
        a = now_us()
        torch.cuda.synchronize()
        ts.append(now_us() - a)
    res["sync_idle_us"] = statistics.median(ts)
    ts = []
    for _ in range(50):
        a = now_us()
        eng.wait()
        ts.append(now_us() - a)
    res["wait_idle_us"] = statistics.median(ts)
    rt = []
    for _ in range(50):
        a = now_us()
        step(256)
        eng.wait()
        rt.append(now_us() - a)
    res["roundtrip_256_blocks_us"] = statistics.median(rt)
    for K in (20, 200):
        rows = []
        for rep in range(9):
            for _ in range(40):
                step()
            eng.wait()
            eng.profile(True)
            torch.cuda.synchronize()
            t0 = now_us()
            step(final=K <= 3)
            t_first = now_us()
            for k in range(1, K):
                step(final=k >= K - 3)
            t_sub = now_us()
            eng.wait()
            t_wait = now_us()
            torch.cuda.synchronize()
            t1 = now_us()
            sp = eng.profile_read()
            eng.profile(False)
            first, last = sp[0][0], max(b for _, b in sp)
            rows.append({"host_us": t1 - t0, "submit_us": t_sub - t0,
                         "first_submit_us": t_first - t0,
                         "t0_to_first_start": first - t0, "device_span": last - first,
                         "last_end_to_wait": t_wait - last, "wait_to_sync": t1 - t_wait,
                         "first_dispatch_us": sp[0][1] - sp[0][0],
                         "steady_period": (sp[-1][0] - sp[1][0]) / (K - 2)})
        agg = {k: round(statistics.median(r[k] for r in rows), 3) for k in rows[0]}
        res[f"K{K}"] = agg
        print(sc, K, json.dumps(agg), flush=True)
        # unprofiled host time of the same region
        ts = []
        for rep in range(9):
            for _ in range(40):
                step()
            eng.wait()
            torch.cuda.synchronize()
            t0 = now_us()
            for k in range(K):
                step(final=k >= K - 3)
            eng.wait()
            torch.cuda.synchronize()
            ts.append((now_us() - t0) / K)
        res[f"K{K}_plain_us_per_step"] = round(statistics.median(ts), 3)
        print(sc, K, "plain", res[f"K{K}_plain_us_per_step"], flush=True)
    print(sc, json.dumps({k: v for k, v in res.items() if not k.startswith("K")}), flush=True)
    print(sc, "kernarg cache (hits, misses)", eng.kernarg_cache(), flush=True)
    return res


if __name__ == "__main__":
    main()
