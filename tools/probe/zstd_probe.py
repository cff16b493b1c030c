"""Where a zstd frame's decode time goes (GPU box; not part of the product).

    python tools/probe/zstd_probe.py [frames.bin]

The probe library (tools/probe/liblvkv_probe.so) stamps s_memtime at the
decoder's phases: start, frame staged, literals decoded (weights, Huffman
table, four streams), sequence tables built, sequences executed, output
written. Decodes 65,536 db_bench frames (libzstd level 1, from
tools/snappy_bench.py --write-zstd-frames) and prints the median of each
phase, in shader-clock ticks.
"""
import ctypes
import sys
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO))


def main():
    blob = Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r05/zframes.bin").read_bytes()
    frames, p = [], 0
    while p < len(blob):
        n = int.from_bytes(blob[p:p + 4], "little")
        frames.append(blob[p + 4:p + 4 + n])
        p += 4 + n
    nb = 65536
    fr = [frames[i % len(frames)] for i in range(nb)]
    off = np.zeros(nb, dtype=np.int64)
    off[1:] = np.cumsum([len(f) for f in fr[:-1]])
    dev = torch.device("cuda:0")
    src = torch.from_numpy(np.frombuffer(b"".join(fr), dtype=np.uint8).copy()).to(dev)
    so = torch.from_numpy(off).to(dev)
    sl = torch.tensor([len(f) for f in fr], dtype=torch.int32, device=dev)
    dst = torch.empty(nb * 4096, dtype=torch.uint8, device=dev)
    doff = torch.arange(nb, dtype=torch.int64, device=dev) * 4096
    cap = torch.full((nb,), 4096, dtype=torch.int32, device=dev)
    ol = torch.empty(nb, dtype=torch.int32, device=dev)
    st = torch.empty(nb, dtype=torch.uint8, device=dev)
    stamps = torch.zeros(nb * 16, dtype=torch.int64, device=dev)
    lib = ctypes.CDLL(str(REPO / "tools" / "probe" / "liblvkv_probe.so"))
    vp = ctypes.c_void_p
    lib.lvkv_debug_zstd_stamps.argtypes = [vp]
    lib.lvkv_zstd_uncompress_device.argtypes = [vp] * 8 + [ctypes.c_size_t, ctypes.c_uint32, vp]
    args = [src.data_ptr(), so.data_ptr(), sl.data_ptr(), dst.data_ptr(), doff.data_ptr(),
            cap.data_ptr(), ol.data_ptr(), st.data_ptr(), nb, 4096,
            torch.cuda.current_stream().cuda_stream]
    lib.lvkv_debug_zstd_stamps(stamps.data_ptr())
    assert lib.lvkv_zstd_uncompress_device(*args) == 0
    torch.cuda.synchronize()
    assert int(st.max()) == 0
    s = stamps.view(nb, 16).cpu().numpy().astype(np.float64)
    names = ["stage", "literals", "seq tables", "sequences", "out"]
    d = np.diff(s[:, :6], axis=1)
    med = {n: float(np.median(d[:, i])) for i, n in enumerate(names)}
    tot = float(np.median(s[:, 5] - s[:, 0]))
    med["weights"] = float(np.median(s[:, 6] - s[:, 1]))
    med["huf table"] = float(np.median(s[:, 7] - s[:, 6]))
    med["streams"] = float(np.median(s[:, 2] - s[:, 7]))
    fse = s[:, 11] > 0  # frames whose first tree has FSE-coded weights
    for name, a, b in (("to weights", 1, 8), ("ncount", 8, 9), ("fse build", 9, 10),
                       ("weight decode", 10, 11), ("weight checks", 11, 6)):
        med[name] = float(np.median(s[fse, b] - s[fse, a])) if fse.any() else None
    med["fse frames"] = int(fse.sum())
    print({"ticks_median": med, "total": tot})


if __name__ == "__main__":
    main()
