"""Isolated (ordered) launch time of engine kernel variants (GPU box). Not
part of the product.

    bash tools/probe/build.sh && python tools/probe/iso_probe.py [names...]

Every probe kernel of engine_probe_kernels.co is loaded as the engine's
ordered kernel (lvkv_engine_load_probe), checked against the HIP path where
it computes CRCs, then timed over 64 ordered dispatches on MALL-cold windows
of the headline batch (packet-processor start/end, HSA profiling).
Writes gpurun_out/iso_probe.json.
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
L = lvkv.lib
vp = ctypes.c_void_p
L.lvkv_engine_load_probe.argtypes = [vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                     ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                     ctypes.c_int]
L.lvkv_engine_load_probe.restype = ctypes.c_int
L.lvkv_engine_set_stamps.argtypes = [vp, vp, ctypes.c_uint64]

# name: (waves, chains, workgroups per CU, computes CRCs)
KERNELS = {
    "pk_pair": (8, 3, 2, True), "pk_pair_bare": (8, 3, 2, False),
    "pk_pair_nobuild": (8, 3, 2, False), "pk_pair_nowalk": (8, 3, 2, False),
    "pk_pair_late": (8, 3, 2, True), "pk_pair_split2": (8, 3, 2, True),
    "pk_pair_dp": (8, 3, 2, True), "pk_pair_bare_dp": (8, 3, 2, False),
    "pk_pair_pipe1": (8, 3, 2, True), "pk_pair_pipe2": (8, 3, 2, True),
    "pk_one_pipe1": (8, 5, 1, True), "pk_one_pipe2": (8, 5, 1, True),
    "pk_w16_pipe1": (16, 3, 1, True),
    "pk_pair_pipe1_s2": (8, 3, 2, True), "pk_pair_pipe1_s4": (8, 3, 2, True),
    "pk_pair_pipe2_s2": (8, 3, 2, True), "pk_one_pipe2_s2": (8, 5, 1, True),
    "pk_w16": (16, 3, 1, True), "pk_w16_bare": (16, 3, 1, False),
    "pk_one": (8, 5, 1, True), "pk_one_bare": (8, 5, 1, False),
    "pk_w10c2_pipe1": (10, 2, 2, True), "pk_w10c2": (10, 2, 2, True),
    "pk_w12c2_pipe1": (12, 2, 2, True), "pk_w10c2_pipe1_s2": (10, 2, 2, True),
}


def main():
    names = [a for a in sys.argv[1:] if not a.startswith("--")] or list(KERNELS)
    co = (HERE / "engine_probe_kernels.co").read_bytes()
    nb, Lb = 10_000, 4096
    dev = torch.device("cuda:0")
    win = nb * Lb
    nrot = 33
    buf = torch.randint(0, 256, (nrot * win,), dtype=torch.uint8, device=dev)
    ref = lvkv.crc32c_uniform(buf, nb, Lb)
    out = torch.zeros(nb, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    eng = lvkv.Engine(0)
    sub = eng.submit_ptr
    res = {}
    rot = 0
    for name in ["(engine ordered default)"] + names:
        if name in KERNELS:
            w, c, per_cu, computes = KERNELS[name]
            rc = L.lvkv_engine_load_probe(eng.handle, co, len(co), (name + ".kd").encode(), w, c,
                                          per_cu, 0)
            assert rc == 0, (name, rc)
        else:
            computes = True
        out.zero_()
        torch.cuda.synchronize()  # the engine does not follow torch's stream
        assert sub(eng.handle, buf.data_ptr(), Lb, Lb, 0, out.data_ptr(), nb, 2) == 0
        eng.wait()
        ok = bool(torch.equal(out, ref)) if computes else None
        ts = []
        for rep in range(3):
            eng.profile(True)
            for _ in range(64):
                rot += 1
                sub(eng.handle, buf.data_ptr() + (rot % nrot) * win, Lb, Lb, 0, out.data_ptr(),
                    nb, 2)
            eng.wait()
            ts += [b - a for a, b in eng.profile_read()]
            eng.profile(False)
        row = {"parity": ok, "us_mean": round(statistics.mean(ts), 3),
               "us_median": round(statistics.median(ts), 3), "us_min": round(min(ts), 3),
               "frac_median": round(nb * (Lb + 4) / (statistics.median(ts) * 1e-6) / 8e12, 4)}
        res[name] = row
        print(name, json.dumps(row), flush=True)
    if "--sweep" in sys.argv:
        # launch time against batch size: slope = streaming rate, intercept =
        # the fixed cost of a launch (dispatch, ramp, drain)
        big = torch.randint(0, 256, (16 * 40_000 * Lb,), dtype=torch.uint8, device=dev)
        bout = torch.zeros(40_000, dtype=torch.int32, device=dev)
        for name in names:
            w, c, per_cu, _ = KERNELS[name]
            L.lvkv_engine_load_probe(eng.handle, co, len(co), (name + ".kd").encode(), w, c, per_cu, 0)
            cap = 256 * per_cu * w * c
            for n in (256, 1024, 2500, 5000, 7500, 10_000, min(cap, 12_000)):
                if n > cap:
                    continue
                ts = []
                eng.profile(True)
                for k in range(96):
                    sub(eng.handle, big.data_ptr() + (k % 16) * 40_000 * Lb, Lb, Lb, 0,
                        bout.data_ptr(), n, 2)
                eng.wait()
                ts = [b - a for a, b in eng.profile_read()]
                eng.profile(False)
                med = statistics.median(ts)
                key = f"sweep_{name}_{n}"
                res[key] = {"us_median": round(med, 3), "bytes": n * Lb}
                print(key, json.dumps(res[key]), flush=True)
    for name in [a.split("=", 1)[1] for a in sys.argv if a.startswith("--stamps=")]:
        # per-wave phases (s_memrealtime, 100 MHz) of ordered launches
        L.lvkv_engine_load_probe(eng.handle, co, len(co), (name + ".kd").encode(), 8, 3, 2, 0)
        K, waves = 32, 512 * 8
        st = torch.zeros(K * waves * 8, dtype=torch.int64, device=dev)
        assert L.lvkv_engine_set_stamps(eng.handle, st.data_ptr(), K) == 0
        eng.profile(True)
        for k in range(K):
            sub(eng.handle, buf.data_ptr() + ((rot + k) % nrot) * win, Lb, Lb, 0, out.data_ptr(),
                nb, 2)
        eng.wait()
        cp = [b - a for a, b in eng.profile_read()]
        eng.profile(False)
        L.lvkv_engine_set_stamps(eng.handle, None, 0)
        import numpy as np
        s = st.cpu().numpy().reshape(K, waves, 8).astype(np.int64)
        rows = []
        for k in range(K):
            v = s[k]
            ok = v[:, 0] > 0
            t0 = v[ok, 0].min()
            rel = (v[ok] - t0) / 100.0
            rows.append({"cp_us": cp[k], "waves_span_us": float(rel[:, 4].max()),
                         "start_spread_us": float(rel[:, 0].max()),
                         "p50_start": float(np.median(rel[:, 0])),
                         "p50_loads_issued": float(np.median(rel[:, 1])),
                         "p50_image": float(np.median(rel[:, 2])),
                         "p50_rowtabs": float(np.median(rel[:, 3])),
                         "p50_lanetabs": float(np.median(rel[:, 5])),
                         "p50_chain0": float(np.median(rel[:, 6])),
                         "p50_chain1": float(np.median(rel[:, 7])),
                         "p50_end": float(np.median(rel[:, 4])),
                         "p90_end": float(np.percentile(rel[:, 4], 90)),
                         "p50_wave_life": float(np.median(rel[:, 4] - rel[:, 0]))})
        agg = {key: round(float(np.median([r[key] for r in rows])), 3) for key in rows[0]}
        res[f"stamps_{name}"] = agg
        print(f"stamps_{name}", json.dumps(agg), flush=True)
    for spec in [a.split("=", 1)[1] for a in sys.argv if a.startswith("--overlap=")]:
        # steady-state period of overlapped dispatches: name:nq
        name, nq = spec.split(":")
        w, c, per_cu, _ = KERNELS[name]
        L.lvkv_engine_load_probe(eng.handle, co, len(co), (name + ".kd").encode(), w, c, per_cu,
                                 1)
        eng.queues(int(nq))
        out.zero_()
        torch.cuda.synchronize()  # the engine does not follow torch's stream
        assert sub(eng.handle, buf.data_ptr(), Lb, Lb, 0, out.data_ptr(), nb, 0) == 0
        eng.wait()
        ok = bool(torch.equal(out, ref))
        row = {"parity": ok}
        for K in (20, 400):
            spans = []
            for rep in range(5):
                t_end = time.perf_counter() + 0.1
                while time.perf_counter() < t_end:
                    for _ in range(16):
                        rot += 1
                        sub(eng.handle, buf.data_ptr() + (rot % nrot) * win, Lb, Lb, 0,
                            out.data_ptr(), nb, 0)
                    eng.wait()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(K):
                    rot += 1
                    sub(eng.handle, buf.data_ptr() + (rot % nrot) * win, Lb, Lb, 0,
                        out.data_ptr(), nb, 0)
                eng.wait()
                torch.cuda.synchronize()
                spans.append((time.perf_counter() - t0) / K * 1e6)
            row[f"K{K}_us"] = round(statistics.median(spans), 3)
            row[f"K{K}_pct"] = round(100 * nb * Lb / (statistics.median(spans) * 1e-6) / 8e12, 2)
        res[f"overlap_{name}_nq{nq}"] = row
        print(f"overlap_{name}_nq{nq}", json.dumps(row), flush=True)
        eng.queues(3)
    L.lvkv_engine_load_probe(eng.handle, None, 0, None, 0, 0, 0, 0)
    (REPO / "gpurun_out").mkdir(exist_ok=True)
    (REPO / "gpurun_out" / "iso_probe.json").write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
