"""Per-wave timeline of the batch kernel (variant 96 = uniform + stamps)."""
import ctypes, json, sys
from pathlib import Path
import numpy as np
import torch
REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
import __graft_entry__ as g
lvkv = g.load_package()
L = lvkv.lib
vp = ctypes.c_void_p
L.lvkv_debug_uniform_variant.argtypes = [ctypes.c_int, ctypes.c_int, vp, ctypes.c_uint64, ctypes.c_uint32, vp, ctypes.c_size_t, vp]
L.lvkv_debug_set_stamps.argtypes = [vp]
NB, BL = 10_000, 4096
dev = torch.device("cuda:0")
nrot = 33
buf = torch.randint(0, 256, (nrot * NB * BL,), dtype=torch.uint8, device=dev)
out = torch.empty(NB, dtype=torch.int32, device=dev)
cu = lvkv.device_groups()
st = torch.zeros(cu * 16 * 8, dtype=torch.int64, device=dev)
L.lvkv_debug_set_stamps(vp(st.data_ptr()))
s = torch.cuda.current_stream()
res = {}
for variant in [int(x) for x in (sys.argv[1:] or ["96", "97"])]:
    runs = []
    for i in range(12):
        st.zero_()
        # a preceding launch keeps the pipeline in its steady state
        L.lvkv_debug_uniform_variant((variant & 768) if variant & 256 else 32, 0, vp(buf.data_ptr() + ((2 * i) % nrot) * NB * BL), BL, BL, vp(out.data_ptr()), NB, vp(s.cuda_stream))
        L.lvkv_debug_uniform_variant(variant, 0, vp(buf.data_ptr() + ((2 * i + 1) % nrot) * NB * BL), BL, BL, vp(out.data_ptr()), NB, vp(s.cuda_stream))
        torch.cuda.synchronize()
        a = st.cpu().numpy().reshape(-1, 8).astype(np.int64)
        t0 = a[:, 0].min()
        rel = np.where(a > 0, (a - t0) * 10, -1)  # ns (100 MHz clock)
        runs.append(rel)
    # per-workgroup tails: the launch ends with its slowest workgroup
    wg_exit = np.stack([r[:, 7].reshape(-1, 16).max(axis=1) for r in runs[2:]])  # [run, wg]
    wg_rows = np.stack([r[:, 2].reshape(-1, 16).max(axis=1) for r in runs[2:]])
    ng = wg_exit.shape[1]
    xcd = np.arange(ng) % 8
    print(f"variant {variant}: per-WG exit (max over its waves), mean over runs; by XCD (g % 8):")
    print("   ", " ".join(f"x{x}:{int(wg_exit[:, xcd == x].mean())}" for x in range(8)))
    print("    by g-octile:", " ".join(str(int(wg_exit[:, k * ng // 8:(k + 1) * ng // 8].mean())) for k in range(8)))
    slow = np.argsort(-wg_exit.mean(axis=0))[:8]
    print("    slowest WGs:", " ".join(f"g{g}:{int(wg_exit[:, g].mean())}/{int(wg_rows[:, g].mean())}" for g in slow))
    per_run_end = wg_exit.max(axis=1)
    print("    launch end (max WG exit) per run:", [int(x) for x in per_run_end])
    rel = np.concatenate(runs[2:])
    def pct(col):
        v = rel[:, col]; v = v[v >= 0]
        return [int(x) for x in np.percentile(v, [0, 10, 50, 90, 100])] if v.size else None
    res[variant] = {k: pct(c) for k, c in [("entry", 0), ("pre_fill", 3), ("fill_issued", 4), ("barrier", 1), ("bc_issued", 5), ("rows_done", 2), ("exit", 7)]}
    print("variant", variant, "percentiles [0,10,50,90,100] ns from first wave entry")
    for k, v in res[variant].items():
        print(f"  {k:10s} {v}")
(REPO / "gpurun_out").mkdir(exist_ok=True)
(REPO / "gpurun_out" / "timeline.json").write_text(json.dumps(res))
