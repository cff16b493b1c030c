"""What a 20-step bench region costs (GPU box). Not part of the product.

    python tools/probe/k20.py

The bench's timed region (sync, t0, K launches, wait, sync, t1) for K = 20,
through the AQL engine (overlapped dispatches) and through HIP (2 streams),
after different warm-ups (0, 5, 50, 200 ms of back-to-back batches) and idle
gaps before t0 (0, 1, 10 ms). Medians of 15 repetitions, us per step.
Writes gpurun_out/k20.json.
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
L.lvkv_engine_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
L.lvkv_engine_crc32c_uniform.argtypes = [vp, vp, ctypes.c_uint64, ctypes.c_uint32,
                                         ctypes.c_uint32, vp, ctypes.c_size_t, ctypes.c_uint32]
L.lvkv_engine_wait.argtypes = [vp]


def main():
    nb, Lb, K = 10_000, 4096, 20
    dev = torch.device("cuda:0")
    win = nb * Lb
    nrot = 33
    buf = torch.randint(0, 256, (nrot * win,), dtype=torch.uint8, device=dev)
    outs = [torch.zeros(nb, dtype=torch.int32, device=dev) for _ in range(4)]
    ptrs = [buf.data_ptr() + w * win for w in range(nrot)]
    optr = [o.data_ptr() for o in outs]
    eng = vp()
    assert L.lvkv_engine_create(0, ctypes.byref(eng)) == 0
    sub = L.lvkv_engine_crc32c_uniform
    uni = L.lvkv_crc32c_uniform_device
    side = torch.cuda.Stream()
    main_s = torch.cuda.current_stream()
    hs = [main_s.cuda_stream, side.cuda_stream]
    rot = [0]

    def eng_steps(n):
        for _ in range(n):
            i = rot[0]
            rot[0] += 1
            sub(eng, ptrs[i % nrot], Lb, Lb, 0, optr[i % 4], nb, 0)

    def hip_steps(n):
        for k in range(n):
            i = rot[0]
            rot[0] += 1
            uni(ptrs[i % nrot], Lb, Lb, 0, optr[i % 4], nb, 0, hs[k % 2])

    res = {}
    for mode in ("engine", "hip2"):
        for warm_ms in (0, 5, 50, 200):
            for gap_ms in (0, 1, 10):
                ts = []
                for _ in range(15):
                    t_end = time.perf_counter() + warm_ms / 1000
                    while time.perf_counter() < t_end:
                        if mode == "engine":
                            eng_steps(8)
                        else:
                            hip_steps(8)
                    if mode == "engine":
                        L.lvkv_engine_wait(eng)
                    torch.cuda.synchronize()
                    if gap_ms:
                        time.sleep(gap_ms / 1000)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    if mode == "engine":
                        eng_steps(K)
                        L.lvkv_engine_wait(eng)
                    else:
                        side.wait_stream(main_s)
                        hip_steps(K)
                        main_s.wait_stream(side)
                    torch.cuda.synchronize()
                    ts.append((time.perf_counter() - t0) / K * 1e6)
                us = statistics.median(ts)
                key = f"{mode}_warm{warm_ms}_gap{gap_ms}"
                res[key] = {"us": round(us, 3), "pct": round(100 * nb * Lb / (us * 1e-6) / 8e12, 2),
                            "min_us": round(min(ts), 3)}
                print(key, json.dumps(res[key]), flush=True)
    (REPO / "gpurun_out").mkdir(exist_ok=True)
    (REPO / "gpurun_out" / "k20.json").write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
