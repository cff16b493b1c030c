"""Device timeline of a 20-step engine region (GPU box). Not part of the product.

    python tools/probe/timeline.py [--variant=V] [--nq=Q] [--K=K]

The bench-style region (sync, t0, 20 engine submits, wait, sync, t1) with the
timestamp build of the engine kernel: per dispatch the first wave start and
the last wave end (s_memrealtime, 100 MHz), against the host's t1 - t0.
Writes gpurun_out/timeline.json.
"""
import ctypes
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO))
import __graft_entry__ as g  # noqa: E402

lvkv = g.load_package()
L = lvkv.lib
vp = ctypes.c_void_p
L.lvkv_engine_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
L.lvkv_engine_crc32c_uniform.argtypes = [vp, vp, ctypes.c_uint64, ctypes.c_uint32,
                                         ctypes.c_uint32, vp, ctypes.c_size_t, ctypes.c_uint32]
L.lvkv_engine_wait.argtypes = [vp]
L.lvkv_engine_set_variant.argtypes = [vp, ctypes.c_int, ctypes.c_int]
L.lvkv_engine_set_stamps.argtypes = [vp, vp, ctypes.c_uint64]


def arg(name, default):
    for a in sys.argv[1:]:
        if a.startswith(f"--{name}="):
            return type(default)(a.split("=", 1)[1])
    return default


def main():
    nb, Lb, K = 10_000, 4096, arg("K", 20)
    dev = torch.device("cuda:0")
    win = nb * Lb
    nrot = 33
    buf = torch.randint(0, 256, (nrot * win,), dtype=torch.uint8, device=dev)
    outs = [torch.zeros(nb, dtype=torch.int32, device=dev) for _ in range(4)]
    ptrs = [buf.data_ptr() + w * win for w in range(nrot)]
    optr = [o.data_ptr() for o in outs]
    eng = vp()
    assert L.lvkv_engine_create(0, ctypes.byref(eng)) == 0
    variant = arg("variant", 0)
    assert L.lvkv_engine_queues(eng, arg("nq", 3)) == arg("nq", 3)
    assert L.lvkv_engine_set_variant(eng, variant, variant) == 0
    w, c, gr = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    L.lvkv_engine_shape(eng, ctypes.byref(w), ctypes.byref(c), ctypes.byref(gr))
    waves = gr.value * w.value
    stamps = torch.zeros(K * waves * 8, dtype=torch.int64, device=dev)
    sub = L.lvkv_engine_crc32c_uniform
    res = {}
    rot = 0
    for flags, name in ((0, "overlap"), (2, "ordered")):
        runs = []
        for rep in range(8):
            L.lvkv_engine_set_stamps(eng, None, 0)
            t_end = time.perf_counter() + 0.05
            while time.perf_counter() < t_end:
                for _ in range(8):
                    sub(eng, ptrs[rot % nrot], Lb, Lb, 0, optr[rot % 4], nb, 0)
                    rot += 1
                L.lvkv_engine_wait(eng)
            stamps.zero_()
            assert L.lvkv_engine_set_stamps(eng, vp(stamps.data_ptr()), K) == 0
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(K):
                sub(eng, ptrs[rot % nrot], Lb, Lb, 0, optr[rot % 4], nb, flags)
                rot += 1
            t_sub = time.perf_counter()
            L.lvkv_engine_wait(eng)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            s = stamps.cpu().numpy().reshape(K, waves, 8).astype(np.int64)
            start = np.where(s[:, :, 0] > 0, s[:, :, 0], np.iinfo(np.int64).max).min(axis=1)
            end = s[:, :, 4].max(axis=1)
            t_base = start[0]
            runs.append({"host_us": (t1 - t0) * 1e6, "submit_us": (t_sub - t0) * 1e6,
                         "device_span_us": (end.max() - t_base) / 100.0,
                         "start_us": ((start - t_base) / 100.0).round(2).tolist(),
                         "end_us": ((end - t_base) / 100.0).round(2).tolist(),
                         # per wave: stamp slots relative to its own start
                         "spread": [float(x) for x in np.percentile(
                             (s[10, :, 0][s[10, :, 0] > 0] - start[10]) / 100.0, [0, 50, 100])],
                         "wave_phase_us": {str(sl): float(np.median((s[:, :, sl] - s[:, :, 0])[s[:, :, 0] > 0]) / 100.0)
                                           for sl in (1, 2, 3, 4)}})
        best = sorted(runs, key=lambda r: r["host_us"])[len(runs) // 2]
        res[name] = best
        print(name, "host %.1f us, device span %.1f us, submit %.1f us" %
              (best["host_us"], best["device_span_us"], best["submit_us"]), flush=True)
        print("  starts", best["start_us"])
        print("  ends  ", best["end_us"])
        print("  wave phases (median us after wave start): ", best["wave_phase_us"])
        print("  wave start spread in kernel 10 (p0/p50/p100 us from its first):",
              best["spread"])
    (REPO / "gpurun_out").mkdir(exist_ok=True)
    (REPO / "gpurun_out" / f"timeline_v{variant}_nq{arg('nq', 3)}.json").write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
