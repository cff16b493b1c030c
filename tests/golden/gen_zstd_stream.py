"""Generates tests/golden/zstd_stream_{inputs,frames}.bin + zstd_stream.json:
multi-block zstd frames of at most 48 KiB of content, written by libzstd
1.4.9 (/opt/conda/lib) through ZSTD_compressStream2 with a flush every
`chunk` bytes, so that one frame holds several small blocks.

    python tests/golden/gen_zstd_stream.py

A single ZSTD_compress frame of that size is one block, so the whole-frame
fixtures (gen_zstd.py) never reach what only a later block can use: a
Huffman tree kept from the block before (treeless literals), FSE tables kept
from it (repeat mode), repeat offsets carried across blocks, and matches
reaching into an earlier block's output. These frames do; the script counts
how many of each occur (through the oracle) and stores the counts with the
fixtures, and every frame is checked to decode back to its input through the
library and through oracle/zstd_oracle.py.
"""
from __future__ import annotations

import ctypes
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO))
from oracle import zstd_oracle as zo  # noqa: E402
from tools.db_bench_data import block_batch  # noqa: E402

# zstd.h 1.4.x: ZSTD_cParameter / ZSTD_EndDirective values
C_LEVEL, C_CONTENT_SIZE, C_CHECKSUM = 100, 200, 201
E_FLUSH, E_END = 1, 2


class _Buf(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("size", ctypes.c_size_t), ("pos", ctypes.c_size_t)]


def _bind(lib):
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    lib.ZSTD_createCCtx.restype = vp
    lib.ZSTD_freeCCtx.argtypes = [vp]
    lib.ZSTD_CCtx_setParameter.restype = sz
    lib.ZSTD_CCtx_setParameter.argtypes = [vp, ctypes.c_int, ctypes.c_int]
    lib.ZSTD_CCtx_setPledgedSrcSize.restype = sz
    lib.ZSTD_CCtx_setPledgedSrcSize.argtypes = [vp, ctypes.c_ulonglong]
    lib.ZSTD_compressStream2.restype = sz
    lib.ZSTD_compressStream2.argtypes = [vp, ctypes.POINTER(_Buf), ctypes.POINTER(_Buf), ctypes.c_int]


def stream_compress(lib, data: bytes, level: int, chunk: int, checksum: bool) -> bytes:
    cctx = lib.ZSTD_createCCtx()
    try:
        for p, v in ((C_LEVEL, level), (C_CONTENT_SIZE, 1), (C_CHECKSUM, int(checksum))):
            assert not lib.ZSTD_isError(lib.ZSTD_CCtx_setParameter(cctx, p, v))
        assert not lib.ZSTD_isError(lib.ZSTD_CCtx_setPledgedSrcSize(cctx, len(data)))
        cap = lib.ZSTD_compressBound(len(data)) + 64 * (len(data) // max(chunk, 1) + 2)
        out = ctypes.create_string_buffer(cap)
        ob = _Buf(ctypes.cast(out, ctypes.c_void_p), cap, 0)
        src = ctypes.create_string_buffer(data, max(len(data), 1))
        pos = 0
        while True:
            end = min(pos + chunk, len(data))
            last = end == len(data)
            ib = _Buf(ctypes.cast(ctypes.addressof(src) + pos, ctypes.c_void_p), end - pos, 0)
            while True:
                r = lib.ZSTD_compressStream2(cctx, ctypes.byref(ob), ctypes.byref(ib),
                                             E_END if last else E_FLUSH)
                assert not lib.ZSTD_isError(r)
                if r == 0 and ib.pos == ib.size:
                    break
            pos = end
            if last:
                break
        return out.raw[:ob.pos]
    finally:
        lib.ZSTD_freeCCtx(cctx)


def inputs():
    rng = np.random.default_rng(20261019)
    bb = block_batch(16).tobytes()
    text = (b"LevelDB is a fast key-value storage library written at Google that provides"
            b" an ordered mapping from string keys to string values. ")
    out = []
    for n in (6000, 12288, 30000, 49152):
        out.append(bb[:n])
        out.append((text * (n // len(text) + 1))[:n])
    for n in (9000, 40000):
        x = bytearray(bb[4096:4096 + n])
        x[n // 3:n // 3 + 700] = rng.integers(0, 256, 700, dtype=np.uint8).tobytes()
        out.append(bytes(x))
        out.append(rng.integers(0, 7, n, dtype=np.uint8).tobytes())
    return out


def modes(frame: bytes):
    """Counts of the later-block features in a frame (through the oracle)."""
    seen = {"blocks": 0, "treeless": 0, "fse_repeat": 0}
    orig_lit, orig_st = zo._literals, zo._seq_table

    def lit(data, p, end, st):
        seen["blocks"] += 1
        if data[p] & 3 == 3:
            seen["treeless"] += 1
        return orig_lit(data, p, end, st)

    def st(data, p, end, mode, *a):
        if mode == 3:
            seen["fse_repeat"] += 1
        return orig_st(data, p, end, mode, *a)

    zo._literals, zo._seq_table = lit, st
    try:
        ok, got = zo.uncompress(frame)
    finally:
        zo._literals, zo._seq_table = orig_lit, orig_st
    return ok, got, seen


def main():
    lib = zo.system_zstd()
    if lib is None:
        raise SystemExit("libzstd 1.4.9 not found")
    _bind(lib)
    ins = inputs()
    frames, meta, total = [], [], {"blocks": 0, "treeless": 0, "fse_repeat": 0}
    for i, x in enumerate(ins):
        for lvl, chunk, ck in ((1, 1024, False), (1, 4096, True), (3, 2000, False), (19, 3000, True)):
            f = stream_compress(lib, x, lvl, chunk, ck)
            ok, got = zo.lib_uncompress(lib, f)
            assert ok and got == x, (i, lvl, chunk)
            ok2, got2, seen = modes(f)
            assert ok2 and got2 == x, (i, lvl, chunk, "oracle")
            for k in total:
                total[k] += seen[k]
            frames.append(f)
            meta.append([i, lvl, chunk, int(ck), seen["blocks"]])
    (HERE / "zstd_stream_inputs.bin").write_bytes(b"".join(ins))
    (HERE / "zstd_stream_frames.bin").write_bytes(b"".join(frames))
    spec = {"inputs": [len(x) for x in ins], "frames": [len(f) for f in frames],
            "meta": meta, "meta_fields": ["input", "level", "chunk", "checksum", "blocks"],
            "counts": total}
    (HERE / "zstd_stream.json").write_text(json.dumps(spec, indent=0))
    print(len(frames), "frames,", total)


if __name__ == "__main__":
    main()
