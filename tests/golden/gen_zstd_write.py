"""Generates tests/golden/zstd_write_{inputs,frames}.bin + zstd_write.json from
libzstd 1.4.9 (/opt/conda/lib, the zstd this image carries) driven the way
port::Zstd_Compress drives it (port/port_stdcxx.h:133-161):

    ctx = ZSTD_createCCtx()
    p = ZSTD_getCParams(level, max(n, 1), 0)
    ZSTD_CCtx_setCParams(ctx, p)      # 1.5.x's definition: seven
                                      # ZSTD_CCtx_setParameter calls (1.4.9
                                      # has no ZSTD_CCtx_setCParams)
    ZSTD_compress2(ctx, dst, ZSTD_compressBound(n), src, n)

(oracle/zstd_encoder.lib_port_compress). TableBuilder::WriteBlock calls it
with options.zstd_compression_level (default 1, include/leveldb/options.h:141).

    python tests/golden/gen_zstd_write.py

inputs : db_bench's blocks (4096 and LevelDB-sized 4096 + a record), edge
         sizes 0-20, 63-65, 255-257, 1023-1025, 4105, incompressible bytes,
         few-symbol bytes, text, runs (RLE literals, later RLE blocks),
         skewed symbol counts (Huffman trees past 11 bits), key/value
         entries, and inputs past one 128 KiB block;
frames : at levels 1 (the default), 2, -1 and -5 (the negative levels share
         ZSTD_fast with literal compression off).
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
from oracle import zstd_encoder as ze  # noqa: E402
from tools.db_bench_data import block_batch  # noqa: E402

LEVELS = (1, 2, -1, -5)


def inputs():
    rng = np.random.default_rng(20261018)
    bb = block_batch(64).tobytes()
    out = [bb[i * 4096:(i + 1) * 4096] for i in range(6)]
    out += [bb[10 + i * 4105: 10 + (i + 1) * 4105] for i in range(4)]  # 4096 + a record
    out += [bb[:n] for n in list(range(0, 21)) + [63, 64, 65, 255, 256, 257, 1023, 1024, 1025,
                                                 8191, 8192, 8193, 16384, 16385, 20480]]
    for n in (100, 1000, 4096):
        out.append(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        out.append(rng.integers(0, 3, n, dtype=np.uint8).tobytes())
        out.append(rng.integers(60, 70, n, dtype=np.uint8).tobytes())
    text = (b"LevelDB is a fast key-value storage library written at Google that provides"
            b" an ordered mapping from string keys to string values. ")
    for n in (70, 700, 4096, 12000):
        out.append((text * (n // len(text) + 1))[:n])
    out += [bytes(4096), bytes([7]) * 300, b"ab" * 2000, bytes(range(256)) * 16]
    # one symbol of literals between matches (RLE literals)
    out.append((b"x" * 40 + bytes(rng.integers(0, 256, 16, dtype=np.uint8))) * 70)
    for p in (0.3, 0.45, 0.6):  # skewed counts: deep trees, HUF_setMaxHeight
        g = np.minimum(rng.geometric(p, 4096) - 1, 255).astype(np.uint8)
        out.append(g.tobytes())
    fib, a, b, s = bytearray(), 1, 1, 0
    while len(fib) < 6000:
        fib += bytes([s]) * a
        a, b, s = b, a + b, s + 1
    arr = np.frombuffer(bytes(fib[:6000]), dtype=np.uint8).copy()
    rng.shuffle(arr)
    out.append(arr.tobytes())
    ent = bytearray()
    for i in range(150):
        ent += bytes([0, 16, 40]) + f"key{i:013d}".encode() + rng.integers(0, 256, 40,
                                                                           dtype=np.uint8).tobytes()
    out.append(bytes(ent))
    # past one block: 128 KiB blocks, HUF repeat, later RLE blocks
    out.append((bb * 3)[:200000])
    out.append(bytes(140000) + bb[:5000])
    out.append(bytes(270000))  # later blocks of one byte: RLE blocks
    # RLE literals: a second block whose every literal is one byte (each
    # 'x' + R_i, R_i met only in the first block)
    rs = [bytes(rng.integers(0, 256, 48, dtype=np.uint8)).replace(b"x", b"y") for _ in range(120)]
    first = (b"".join(r + r for r in rs) * 14)[:131072]
    out.append(first + b"".join(b"x" + rs[int(i)] for i in rng.permutation(120)))
    return out


def main():
    lib = ze.system_zstd_writer()
    if lib is None:
        raise SystemExit("libzstd 1.4.9 not found")
    ins = inputs()
    frames, meta = [], []
    for i, x in enumerate(ins):
        for lvl in LEVELS:
            if not ze.supported(lvl, len(x)):
                continue
            frames.append(ze.lib_port_compress(lib, x, lvl))
            meta.append([i, lvl])
    # the parameters ZSTD_getCParams gives (the oracle's table is pinned to them)
    grid = []
    for lvl in (1, 2, 3, 0, -1, -5, -131072, -200000, 22):
        for n in (1, 2, 63, 64, 65, 100, 1000, 1024, 1025, 4096, 4097, 16384, 16385, 131072,
                  131073, 262144, 262145, 1 << 20):
            p = lib.ZSTD_getCParams(lvl, n, 0)
            grid.append([lvl, n, [p.windowLog, p.chainLog, p.hashLog, p.searchLog, p.minMatch,
                                  p.targetLength, p.strategy]])
    blob = {"inputs": [len(x) for x in ins], "frames": [len(f) for f in frames], "meta": meta,
            "sha256_inputs": [hashlib.sha256(x).hexdigest() for x in ins], "cparams": grid,
            "source": "libzstd 1.4.9 (/opt/conda/lib/libzstd.so.1.4.9): ZSTD_createCCtx, "
                      "ZSTD_getCParams(level, max(n,1), 0), seven ZSTD_CCtx_setParameter "
                      "(= ZSTD_CCtx_setCParams), ZSTD_compress2"}
    (HERE / "zstd_write_inputs.bin").write_bytes(b"".join(ins))
    (HERE / "zstd_write_frames.bin").write_bytes(b"".join(frames))
    (HERE / "zstd_write.json").write_text(json.dumps(blob, indent=0))
    print(len(ins), "inputs", sum(map(len, ins)), "bytes;", len(frames), "frames",
          sum(map(len, frames)), "bytes")


if __name__ == "__main__":
    main()
