"""Where a block's zstd compression time goes (GPU box; not part of the
product).

    python tools/probe/zstdc_probe.py [blocks]

The probe library (tools/probe/liblvkv_probe.so) stamps s_memtime at the
compressor's phases (tools/probe/lvkv_probe.h, lvkv_debug_zstdc_stamps).
Compresses `blocks` db_bench blocks of 4 KiB at level 1 and prints the
median ticks of each phase, and the launch time with and without stamps.
"""
import ctypes
import json
import sys
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO))
from tools.db_bench_data import block_batch  # noqa: E402


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    libpath = REPO / "tools" / "probe" / "liblvkv_probe.so"
    if len(sys.argv) > 2 and sys.argv[2] == "product":
        libpath = REPO / "leveldb-kv-separation_amd" / "liblvkv_crc32c.so"
    elif len(sys.argv) > 2:
        libpath = Path(sys.argv[2])
    print("lib", libpath.name, flush=True)
    L = 4096
    dev = torch.device("cuda:0")
    src = torch.from_numpy(block_batch(nb, L)).to(dev)
    off = torch.arange(nb, dtype=torch.int64, device=dev) * L
    ln = torch.full((nb,), L, dtype=torch.int32, device=dev)
    zb = L + (L >> 8) + ((131072 - L) >> 11)
    dst = torch.empty(nb * zb, dtype=torch.uint8, device=dev)
    doff = torch.arange(nb, dtype=torch.int64, device=dev) * zb
    dl = torch.empty(nb, dtype=torch.int32, device=dev)
    st = torch.empty(nb, dtype=torch.uint8, device=dev)
    stamps = torch.zeros(nb * 16, dtype=torch.int64, device=dev)
    lib = ctypes.CDLL(str(libpath))
    vp = ctypes.c_void_p
    has_stamps = hasattr(lib, "lvkv_debug_zstdc_stamps")
    if has_stamps:
        lib.lvkv_debug_zstdc_stamps.argtypes = [vp]
    lib.lvkv_zstd_compress_device.argtypes = [vp] * 7 + [ctypes.c_size_t, ctypes.c_uint32,
                                                         ctypes.c_int, vp]
    stream = torch.cuda.current_stream()
    args = [src.data_ptr(), off.data_ptr(), ln.data_ptr(), dst.data_ptr(), doff.data_ptr(),
            dl.data_ptr(), st.data_ptr(), nb, L, 1, stream.cuda_stream]

    def timed(k=5):
        assert lib.lvkv_zstd_compress_device(*args) == 0
        print("launched", flush=True)
        torch.cuda.synchronize()
        print("first done", flush=True)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(k):
            assert lib.lvkv_zstd_compress_device(*args) == 0
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / k

    t_plain = timed()
    print("plain", t_plain, flush=True)
    if not has_stamps:
        return
    lib.lvkv_debug_zstdc_stamps(stamps.data_ptr())
    t_stamped = timed(1)
    lib.lvkv_debug_zstdc_stamps(None)
    assert int(st.max()) == 0
    s = stamps.view(nb, 16).cpu().numpy().astype(np.float64)
    seg = {"stage+zero": (0, 1), "match": (1, 2), "lit count": (2, 8), "tree": (8, 9),
           "weights": (9, 10), "stream sizes": (10, 11), "streams packed": (11, 3),
           "seq tables": (3, 4), "seq bits": (4, 5), "tail+out": (5, 6), "total": (0, 6)}
    med = {k: float(np.median(s[:, b] - s[:, a])) for k, (a, b) in seg.items()}
    res = {"blocks": nb, "us_per_launch": round(t_plain, 1), "us_stamped": round(t_stamped, 1),
           "ticks_median": med}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
