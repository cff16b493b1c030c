"""AQL engine timing (GPU box). Not part of the product.

    python tools/probe/engine_probe.py [--K=N] [--variant=V]

Parity of lvkv_engine_crc32c_uniform against lvkv_crc32c_uniform_device on
the headline batch, then host-timed regions (Python submit loop, as bench.py):
ordered (barrier bit: one batch at a time) and overlapped, K = 20 and K = N,
each after a 100 ms warm-up. Writes gpurun_out/engine_probe.json.
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
L.lvkv_engine_destroy.argtypes = [vp]
L.lvkv_engine_set_variant.argtypes = [vp, ctypes.c_int, ctypes.c_int]


def arg(name, default):
    for a in sys.argv[1:]:
        if a.startswith(f"--{name}="):
            return type(default)(a.split("=", 1)[1])
    return default


def main():
    K = arg("K", 400)
    nb, Lb = arg("nb", 10_000), 4096
    dev = torch.device("cuda:0")
    win = nb * Lb
    nrot = max(2, -(-int(1.25 * (1 << 30)) // win))
    buf = torch.randint(0, 256, (nrot * win,), dtype=torch.uint8, device=dev)
    outs = [torch.zeros(nb, dtype=torch.int32, device=dev) for _ in range(4)]
    ref = torch.zeros(nb, dtype=torch.int32, device=dev)
    L.lvkv_crc32c_uniform_device(vp(buf.data_ptr()), Lb, Lb, 0, vp(ref.data_ptr()), nb, 0,
                                 vp(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    eng = vp()
    rc = L.lvkv_engine_create(0, ctypes.byref(eng))
    assert rc == 0, f"engine create {rc}"
    res = {}
    combos = [(v, q) for v in (0, 1) for q in (1, 2, 3, 4)]
    if "--one" in sys.argv:
        combos = [(0, 3)]
    for variant, nq in combos:
        assert L.lvkv_engine_queues(eng, nq) == nq
        assert L.lvkv_engine_set_variant(eng, variant, variant) == 0
        tag = f"v{variant}_nq{nq}"
        rc = L.lvkv_engine_crc32c_uniform(eng, vp(buf.data_ptr()), Lb, Lb, 0,
                                          vp(outs[0].data_ptr()), nb, 0)
        assert rc == 0, rc
        assert L.lvkv_engine_wait(eng) == 0
        assert torch.equal(outs[0], ref), f"{tag}: engine parity FAILED"
        ptrs = [buf.data_ptr() + w * win for w in range(nrot)]
        optr = [o.data_ptr() for o in outs]
        sub = L.lvkv_engine_crc32c_uniform
        rot = [0]

        def submit(n, flags):
            for _ in range(n):
                i = rot[0]
                rot[0] += 1
                sub(eng, ptrs[i % nrot], Lb, Lb, 0, optr[i % 4], nb, flags)

        def warm():
            t_end = time.perf_counter() + 0.1
            while time.perf_counter() < t_end:
                submit(16, 0)
                L.lvkv_engine_wait(eng)

        row = {}
        for flags, name in ((2, "ordered"), (0, "overlap")):
            for n in (20, K):
                ts = []
                for _ in range(7):
                    warm()
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    submit(n, flags)
                    L.lvkv_engine_wait(eng)
                    torch.cuda.synchronize()
                    ts.append((time.perf_counter() - t0) / n * 1e6)
                us = statistics.median(ts)
                row[f"{name}_{n}_us"] = round(us, 3)
                row[f"{name}_{n}_pct"] = round(100 * nb * Lb / (us * 1e-6) / 8e12, 2)
        # device time of isolated dispatches (HSA profiling, one queue, ordered)
        L.lvkv_engine_queues(eng, 1)
        L.lvkv_engine_profile(eng, 1)
        submit(64, 2)
        L.lvkv_engine_wait(eng)
        t0s, t1s = (ctypes.c_double * 64)(), (ctypes.c_double * 64)()
        k = L.lvkv_engine_profile_read(eng, t0s, t1s, 64)
        dts = [b - a for a, b in zip(t0s[:k], t1s[:k])]
        L.lvkv_engine_profile(eng, 0)
        L.lvkv_engine_queues(eng, nq)
        dt = statistics.median(dts[:k])
        row["single_dispatch_us"] = round(dt, 3)
        row["single_dispatch_pct"] = round(100 * nb * Lb / (dt * 1e-6) / 8e12, 2)
        # submit cost alone (host)
        t0 = time.perf_counter()
        submit(64, 0)
        t_sub = (time.perf_counter() - t0) / 64 * 1e6
        L.lvkv_engine_wait(eng)
        row["submit_call_us"] = round(t_sub, 2)
        res[tag] = row
        print(tag, json.dumps(row), flush=True)
    L.lvkv_engine_destroy(eng)
    # the HIP path on the same box: 1 and 2 streams, Python launch loop
    side = torch.cuda.Stream()
    hs = [torch.cuda.current_stream().cuda_stream, side.cuda_stream]
    uni = L.lvkv_crc32c_uniform_device
    for S in (1, 2):
        row = {}
        for n in (20, K):
            ts = []
            for _ in range(7):
                t_end = time.perf_counter() + 0.1
                i = 0
                while time.perf_counter() < t_end:
                    uni(ptrs[i % nrot], Lb, Lb, 0, optr[i % 4], nb, 0, hs[i % S])
                    i += 1
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for k in range(n):
                    uni(ptrs[(i + k) % nrot], Lb, Lb, 0, optr[k % 4], nb, 0, hs[k % S])
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t0) / n * 1e6)
            us = statistics.median(ts)
            row[f"hip_{n}_us"] = round(us, 3)
            row[f"hip_{n}_pct"] = round(100 * nb * Lb / (us * 1e-6) / 8e12, 2)
        res[f"hip_{S}streams"] = row
        print(f"hip_{S}streams", json.dumps(row), flush=True)
    (REPO / "gpurun_out").mkdir(exist_ok=True)
    (REPO / "gpurun_out" / "engine_probe.json").write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
