"""Timing probes of the batch kernel's parts (GPU box).

Runs kernel variants (see include/lvkv_crc32c_debug.h) and the read-bandwidth
ceiling on the headline layout (10k x 4 KiB per launch, MALL-cold rotation over
> 1 GiB), interleaved in one process, HIP events per launch. Prints a table and
writes gpurun_out/probe.json.
"""
from __future__ import annotations

import ctypes
import json
import statistics
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
import __graft_entry__ as g  # noqa: E402

lvkv = g.load_package()
# schedule variants and the read-bandwidth kernel: the probe build
L = ctypes.CDLL(str(Path(__file__).resolve().parent / "probe" / "liblvkv_probe.so"))
vp = ctypes.c_void_p
L.lvkv_debug_uniform_variant.argtypes = [ctypes.c_int, ctypes.c_int, vp, ctypes.c_uint64,
                                         ctypes.c_uint32, vp, ctypes.c_size_t, vp]
L.lvkv_debug_uniform_variant.restype = ctypes.c_int
L.lvkv_debug_read_bw.argtypes = [vp, ctypes.c_uint64, vp, ctypes.c_int, vp]
L.lvkv_debug_read_bw.restype = ctypes.c_int

NB, BL = 10_000, 4096
BATCH = NB * BL
dev = torch.device("cuda:0")
nrot = 33
buf = torch.randint(0, 256, (nrot * BATCH,), dtype=torch.uint8, device=dev)
out = torch.empty(NB, dtype=torch.int32, device=dev)
stream = torch.cuda.current_stream()
# --streams S: launch i goes to stream i % S (independent batches in flight,
# as bench.py --streams); timing brackets all streams.
NSTREAMS = next((int(a.split("=")[1]) for a in sys.argv[1:] if a.startswith("--streams=")), 1)
side = [torch.cuda.Stream() for _ in range(NSTREAMS - 1)]
handles = [vp(stream.cuda_stream)] + [vp(x.cuda_stream) for x in side]
sh = handles[0]
cu = lvkv.device_groups()


def run_variant(variant, groups, i, warm=False):
    w = 0 if warm else i % nrot
    rc = L.lvkv_debug_uniform_variant(variant, groups, vp(buf.data_ptr() + w * BATCH), BL, BL,
                                      vp(out.data_ptr()), NB, handles[i % NSTREAMS])
    assert rc == 0, rc


def run_readbw(groups, i, nbytes=BATCH, warm=False):
    w = 0 if warm else i % nrot
    rc = L.lvkv_debug_read_bw(vp(buf.data_ptr() + w * BATCH), nbytes, vp(out.data_ptr()), groups,
                              handles[i % NSTREAMS])
    assert rc == 0, rc


def small_variant(kernel_bits):
    """Small-kernel schedule flags (crc32c_uniform.hip enum) via the debug entry."""
    return (kernel_bits << 16) | 768


SMALL_CASES = {}  # e.g. {12: "production"}: kernel bits of crc32c_uniform.hip's small kernel
SMALL_CORRECT = ()


def compact_variant(cfg):
    return (cfg << 16) | 2048 | 256


COMPACT_CASES = {0: "16w x3 occ1", 1: "8w x3 occ2", 2: "16w x2 occ2", 4: "16w x3 occ1 bare",
                 5: "8w x3 occ2 bare", 6: "16w x2 occ2 bare", 8: "16w x3 occ1 genlane",
                 9: "8w x3 occ2 genlane"}
COMPACT_CORRECT = (0, 1, 2, 8, 9)

GRAPH = "--graph" in sys.argv


def timed(fn, n=60):
    """Average per launch over n back-to-back launches (events only around
    the whole run, as in bench.py's timed region), repeated 5 times.
    --graph: the n launches (over all streams) are captured once into a HIP
    graph and replayed, so the host launch rate drops out."""
    if GRAPH:
        return timed_graph(fn, n)
    out = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for x in side:
            x.wait_stream(stream)
        for i in range(n):
            fn(i + 1)
        for x in side:
            stream.wait_stream(x)
        b.record(stream)
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b) * 1e3 / n)
    return out


def timed_graph(fn, n):
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream()
    cap.wait_stream(stream)
    global handles, side
    saved = (handles, side)
    with torch.cuda.stream(cap):
        cside = [torch.cuda.Stream() for _ in range(NSTREAMS - 1)]
        handles = [vp(cap.cuda_stream)] + [vp(x.cuda_stream) for x in cside]
        side = cside
        g.capture_begin()
        for x in cside:
            x.wait_stream(cap)
        for i in range(n):
            fn(i + 1)
        for x in cside:
            cap.wait_stream(x)
        g.capture_end()
    handles, side = saved
    torch.cuda.synchronize()
    out = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        g.replay()
        b.record(stream)
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b) * 1e3 / n)
    return out


cases = {
    "v256 uniform kernel": lambda i: run_variant(256, 0, i),
    "v768 small kernel loads-first": lambda i: run_variant(768, 0, i),
    "v772 small lane-early": lambda i: run_variant(772, 0, i),
    "v776 small early-A": lambda i: run_variant(776, 0, i),
    "v780 small early-A lane-early": lambda i: run_variant(780, 0, i),
    "v780 warm(MALL)": lambda i: run_variant(780, 0, i, warm=True),
    **{f"k{kb} {d}": (lambda i, kb=kb: run_variant(small_variant(kb), 0, i))
       for kb, d in SMALL_CASES.items()},
    **{f"c{cf} compact {d}": (lambda i, cf=cf: run_variant(compact_variant(cf), 0, i))
       for cf, d in COMPACT_CASES.items()},
    "v784 small one-barrier": lambda i: run_variant(784, 0, i),
    "v1804 small half-early-A": lambda i: run_variant(1804, 0, i),
    "v17152 small bare loads": lambda i: run_variant(17152, 0, i),
    "v781 small 12 no-walk": lambda i: run_variant(781, 0, i),
    "v782 small 12 no-loads": lambda i: run_variant(782, 0, i),
    "v812 small 12 no-fill": lambda i: run_variant(812, 0, i),
    "v783 small 12 no-loads no-walk": lambda i: run_variant(783, 0, i),
    "v896 small fill-first": lambda i: run_variant(896, 0, i),
    "v900 small fill-first lane-early": lambda i: run_variant(900, 0, i),
    "v384 uniform fill-first": lambda i: run_variant(384, 0, i),
    "v257 uniform no-compute": lambda i: run_variant(257, 0, i),
    "v258 uniform no-loads": lambda i: run_variant(258, 0, i),
    "v385 uniform fill-first no-compute": lambda i: run_variant(385, 0, i),
    "v386 uniform fill-first no-loads": lambda i: run_variant(386, 0, i),
    "v32 uniform": lambda i: run_variant(32, 0, i),
    "v160 uniform late-loads": lambda i: run_variant(160, 0, i),
    "v33 uniform no-compute": lambda i: run_variant(33, 0, i),
    "v38 uniform no-loads no-fill": lambda i: run_variant(38, 0, i),
    "v0 full": lambda i: run_variant(0, 0, i),
    "v8 shfl-reduce": lambda i: run_variant(8, 0, i),
    "v1 no-compute": lambda i: run_variant(1, 0, i),
    "v2 no-loads": lambda i: run_variant(2, 0, i),
    "v4 no-fill": lambda i: run_variant(4, 0, i),
    "v3 fill+loop only": lambda i: run_variant(3, 0, i),
    "v6 no-loads no-fill": lambda i: run_variant(6, 0, i),
    "v0 full groups=128": lambda i: run_variant(0, cu // 2, i),
    "v0 full warm(MALL)": lambda i: run_variant(0, 0, i, warm=True),
    "v16 empty kernel": lambda i: run_variant(16, 0, i),
    "readbw 41MB cold dword 8/CU": lambda i: run_readbw(-8 * cu, i),
    "readbw 41MB cold 8/CU": lambda i: run_readbw(8 * cu, i),
    "readbw 41MB cold 4/CU": lambda i: run_readbw(4 * cu, i),
    "readbw 41MB cold 16/CU": lambda i: run_readbw(16 * cu, i),
    "readbw 41MB warm": lambda i: run_readbw(8 * cu, i, warm=True),
    "readbw 1.3GB": lambda i: run_readbw(8 * cu, 0, nbytes=nrot * BATCH - 16 * 1024),
}

FILTERS = [a for a in sys.argv[1:] if not a.startswith("--")]
if FILTERS:  # optional substring filter, e.g. "v0 full" "v6"
    cases = {k: v for k, v in cases.items() if any(f in k for f in FILTERS)}

# correctness of the production variant first
for v in (0, 8, 32, 256, 768, 772, 776, 780, 784, 896, 900, 1804,
          *[small_variant(kb) for kb in SMALL_CORRECT],
          *[compact_variant(cf) for cf in COMPACT_CORRECT]):
    run_variant(v, 0, 0)  # stream 0
    torch.cuda.synchronize()
    ref = lvkv.crc32c_uniform(buf, NB, BL)
    torch.cuda.synchronize()
    assert torch.equal(out, ref), f"variant {v} differs from the production launch"

for fn in cases.values():  # warmup
    for i in range(3):
        fn(i)
torch.cuda.synchronize()

res = {k: [] for k in cases}
for rnd in range(3):
    for k, fn in cases.items():
        res[k] += timed(fn, 60 if "1.3GB" not in k else 3)

summary = {}
print(f"{'case':28s} {'median_us':>10s} {'min_us':>10s} {'GB/s(med)':>10s}")
for k, v in res.items():
    med, mn = statistics.median(v), min(v)
    nbytes = (nrot * BATCH - 16 * 1024) if "1.3GB" in k else BATCH
    summary[k] = {"median_us": med, "min_us": mn, "GBps_median": nbytes / med / 1e3}
    print(f"{k:28s} {med:10.2f} {mn:10.2f} {nbytes / med / 1e3:10.1f}")
(REPO / "gpurun_out").mkdir(exist_ok=True)
(REPO / "gpurun_out" / "probe.json").write_text(json.dumps(summary, indent=1))
