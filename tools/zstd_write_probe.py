"""Dump the device Zstd compressor's frames for the write fixtures' inputs
(and a ragged fuzz set) so that they can be compared, section by section,
with the oracle's on the CPU (tools/zstd_write_diff.py).

    python tools/zstd_write_probe.py OUT_DIR [level]
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests"))


def main():
    import torch
    import __graft_entry__ as g
    lvkv = g.load_package()
    out = Path(sys.argv[1])
    level = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    out.mkdir(parents=True, exist_ok=True)
    gold = REPO / "tests" / "golden"
    spec = json.loads((gold / "zstd_write.json").read_text())
    blob = (gold / "zstd_write_inputs.bin").read_bytes()
    ins, p = [], 0
    for n in spec["inputs"]:
        ins.append(blob[p:p + n])
        p += n
    ins = [x for x in ins if len(x) <= lvkv.ZSTD_COMPRESS_MAX_BLOCK]
    dev = torch.device("cuda:0")
    offs, q = [], 1
    for x in ins:
        offs.append(q)
        q += len(x) + 1
    buf = np.zeros(q, dtype=np.uint8)
    for o, x in zip(offs, ins):
        buf[o:o + len(x)] = np.frombuffer(x, dtype=np.uint8)
    src = torch.from_numpy(buf).to(dev)
    off = torch.tensor(offs, dtype=torch.int64, device=dev)
    ln = torch.tensor([len(x) for x in ins], dtype=torch.int32, device=dev)
    dst, doff, dlen, st = lvkv.zstd_compress(src, off, ln, level=level, max_len=20480)
    torch.cuda.synchronize()
    d = dst.cpu().numpy()
    frames = [d[o:o + n].tobytes() for o, n in zip(doff.cpu().tolist(), dlen.cpu().tolist())]
    (out / f"zw_inputs_{level}.bin").write_bytes(b"".join(ins))
    (out / f"zw_frames_{level}.bin").write_bytes(b"".join(frames))
    (out / f"zw_{level}.json").write_text(json.dumps({
        "inputs": [len(x) for x in ins], "frames": [len(f) for f in frames],
        "status": st.cpu().tolist()}))
    print("dumped", len(ins), "frames at level", level)


if __name__ == "__main__":
    main()
