"""Generates tests/golden/zstd_{inputs,frames,damaged}.bin + zstd.json from
libzstd 1.4.9 (/opt/conda/lib, the zstd this image carries; the reference
leaves Zstd to that library, port/port_stdcxx.h:133-199).

    python tests/golden/gen_zstd.py

inputs  : db_bench's 4 KiB blocks, text, random and few-symbol bytes, runs,
          empty / one-byte inputs, and inputs past one 128 KiB block;
frames  : ZSTD_compress of each input at levels 1 (LevelDB's default
          zstd_compression_level), 3, 19 and -5;
damaged : frames with bytes flipped, replaced, cut or extended, with the
          library's verdict through port::Zstd_Uncompress (1 decoded, 0
          failed, 2 content size unknown or huge) and the sha256 of the
          bytes when it decodes.
"""
from __future__ import annotations

import hashlib
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO))
from oracle import zstd_oracle as zo  # noqa: E402
from tools.db_bench_data import block_batch  # noqa: E402

LEVELS = (1, 3, 19, -5)


def inputs():
    rng = np.random.default_rng(20261018)
    bb = block_batch(16).tobytes()
    out = [b"", b"x", bytes(100), bytes([7]) * 5000]
    for i in range(8):
        out.append(bb[i * 4096:(i + 1) * 4096])
    for n in (10, 100, 1000, 4096, 9000):
        out.append(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        out.append(rng.integers(0, 5, n, dtype=np.uint8).tobytes())
    text = (b"LevelDB is a fast key-value storage library written at Google that provides"
            b" an ordered mapping from string keys to string values. ")
    for n in (50, 700, 4096, 20000):
        out.append((text * (n // len(text) + 1))[:n])
    out.append((bb * 4)[:200000])  # two blocks at 128 KiB
    return out


def main():
    lib = zo.system_zstd()
    if lib is None:
        raise SystemExit("libzstd 1.4.9 not found")
    ins = inputs()
    frames, meta = [], []
    for i, x in enumerate(ins):
        for lvl in LEVELS:
            frames.append(zo.lib_compress(lib, x, lvl))
            meta.append([i, lvl])
    rng = np.random.default_rng(5)
    small = [f for f in frames if len(f) < 1500]
    dam, verdicts = [], []
    for k in range(1000):
        f = bytearray(small[k % len(small)])
        for _ in range(int(rng.integers(1, 4))):
            j = int(rng.integers(0, len(f)))
            if k % 2:
                f[j] ^= 1 << int(rng.integers(0, 8))
            else:
                f[j] = int(rng.integers(0, 256))
        if k % 5 == 0:
            f = f[: int(rng.integers(1, len(f) + 1))]
        if k % 7 == 0:
            f += rng.integers(0, 256, int(rng.integers(1, 6)), dtype=np.uint8).tobytes()
        dam.append(bytes(f))
    # hand-made: literals under a 12-bit single-stream Huffman tree
    # (HUF_TABLELOG_MAX; libzstd decodes it to four zero bytes)
    dam.append(bytes.fromhex("28b52ffd20047500004280028cbbba9876543210550100"))
    for f in dam:
        ok, out = zo.lib_uncompress(lib, f)
        verdicts.append({"ok": 2 if ok is None else int(ok), "n": len(out),
                         "sha256": hashlib.sha256(out).hexdigest() if ok else None})
    blob = {"inputs": [len(x) for x in ins], "frames": [len(f) for f in frames], "meta": meta,
            "damaged": [len(d) for d in dam], "verdicts": verdicts,
            "sha256_inputs": [hashlib.sha256(x).hexdigest() for x in ins],
            "source": "libzstd 1.4.9 (/opt/conda/lib/libzstd.so.1.4.9), ZSTD_compress / "
                      "ZSTD_getFrameContentSize / ZSTD_decompress"}
    (HERE / "zstd_inputs.bin").write_bytes(b"".join(ins))
    (HERE / "zstd_frames.bin").write_bytes(b"".join(frames))
    (HERE / "zstd_damaged.bin").write_bytes(b"".join(dam))
    (HERE / "zstd.json").write_text(json.dumps(blob, indent=0))
    c = [v["ok"] for v in verdicts]
    print(len(ins), "inputs,", len(frames), "frames,", len(dam), "damaged:",
          {k: c.count(k) for k in (0, 1, 2)})


if __name__ == "__main__":
    main()
