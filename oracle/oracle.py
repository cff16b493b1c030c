"""TEST INFRASTRUCTURE ONLY — Python access to the CPU oracle.

Loads oracle/liboracle_crc32c.so (the C restatement of the reference's
util/crc32c.cc:276-377, see crc32c_oracle.c) and, when present,
oracle/_ref/libref_crc32c.so (the reference's own util/crc32c.cc compiled in
place). Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
use this module — as the checker, never as the product path.

Also provides splitmix64 byte generation identical to oracle/gen_golden.cc so
golden fixtures can be regenerated from their seeds.
"""
from __future__ import annotations

import ctypes
from pathlib import Path
from typing import Optional

import numpy as np

HERE = Path(__file__).resolve().parent
ORACLE_LIB = HERE / "liboracle_crc32c.so"
REF_LIB = HERE / "_ref" / "libref_crc32c.so"

_u32, _u64, _sz, _vp, _int = (ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t,
                              ctypes.c_void_p, ctypes.c_int)


def _load_oracle() -> ctypes.CDLL:
    if not ORACLE_LIB.exists():
        raise ImportError(f"{ORACLE_LIB} missing: run `make -C oracle`")
    L = ctypes.CDLL(str(ORACLE_LIB))
    L.oracle_crc32c_extend.argtypes = [_u32, ctypes.c_char_p, _sz]
    L.oracle_crc32c_extend.restype = _u32
    L.oracle_crc32c_value.argtypes = [ctypes.c_char_p, _sz]
    L.oracle_crc32c_value.restype = _u32
    L.oracle_crc32c_mask.argtypes = [_u32]
    L.oracle_crc32c_mask.restype = _u32
    L.oracle_crc32c_unmask.argtypes = [_u32]
    L.oracle_crc32c_unmask.restype = _u32
    L.oracle_crc32c_table.argtypes = [_int, _vp]
    L.oracle_crc32c_table.restype = _int
    L.oracle_crc32c_batch_mt.argtypes = [_vp, _vp, _vp, _vp, _vp, _sz, _int, _int]
    L.oracle_crc32c_batch_mt.restype = None
    L.oracle_crc32c_uniform.argtypes = [_vp, _u64, _u32, _u32, _vp, _sz, _int, _int]
    L.oracle_crc32c_uniform.restype = None
    return L


_L = _load_oracle()


def extend(init: int, data: bytes) -> int:
    return int(_L.oracle_crc32c_extend(init & 0xFFFFFFFF, bytes(data), len(data)))


def value(data: bytes) -> int:
    return extend(0, data)


def mask(c: int) -> int:
    return int(_L.oracle_crc32c_mask(c & 0xFFFFFFFF))


def unmask(c: int) -> int:
    return int(_L.oracle_crc32c_unmask(c & 0xFFFFFFFF))


def table(which: int) -> np.ndarray:
    out = np.zeros(256, dtype=np.uint32)
    assert _L.oracle_crc32c_table(which, out.ctypes.data) == 0
    return out


def batch(buf: np.ndarray, offsets, lengths, inits=None, mask: bool = False,
          threads: int = 1) -> np.ndarray:
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
    n = offsets.size
    out = np.empty(n, dtype=np.uint32)
    ip = None
    if inits is not None:
        inits = np.ascontiguousarray(inits, dtype=np.uint32)
        ip = inits.ctypes.data
    _L.oracle_crc32c_batch_mt(buf.ctypes.data, offsets.ctypes.data, lengths.ctypes.data,
                              ip, out.ctypes.data, n, int(mask), threads)
    return out


def uniform(buf: np.ndarray, nblocks: int, length: int, stride: Optional[int] = None,
            init: int = 0, mask: bool = False, threads: int = 1) -> np.ndarray:
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    stride = length if stride is None else stride
    assert nblocks == 0 or (nblocks - 1) * stride + length <= buf.size
    out = np.empty(nblocks, dtype=np.uint32)
    _L.oracle_crc32c_uniform(buf.ctypes.data, stride, length, init & 0xFFFFFFFF,
                             out.ctypes.data, nblocks, int(mask), threads)
    return out


# ---- the reference itself (oracle/_ref), when built -----------------------

class Reference:
    """The reference's own leveldb::crc32c::Extend, compiled from
    /root/reference/util/crc32c.cc by oracle/Makefile (target `ref`)."""

    def __init__(self, path: Path = REF_LIB):
        L = ctypes.CDLL(str(path))
        L.ref_crc32c_extend.argtypes = [_u32, ctypes.c_char_p, _sz]
        L.ref_crc32c_extend.restype = _u32
        L.ref_crc32c_mask.argtypes = [_u32]
        L.ref_crc32c_mask.restype = _u32
        L.ref_crc32c_uniform.argtypes = [_vp, _u64, _u32, _u32, _vp, _sz, _int]
        L.ref_crc32c_uniform.restype = None
        L.ref_crc32c_batch.argtypes = [_vp, _vp, _vp, _vp, _sz]
        L.ref_crc32c_batch.restype = None
        self._L = L

    def extend(self, init: int, data: bytes) -> int:
        return int(self._L.ref_crc32c_extend(init & 0xFFFFFFFF, bytes(data), len(data)))

    def mask(self, c: int) -> int:
        return int(self._L.ref_crc32c_mask(c & 0xFFFFFFFF))

    def uniform(self, buf: np.ndarray, nblocks: int, length: int,
                stride: Optional[int] = None, init: int = 0, threads: int = 1) -> np.ndarray:
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        stride = length if stride is None else stride
        assert nblocks == 0 or (nblocks - 1) * stride + length <= buf.size
        out = np.empty(nblocks, dtype=np.uint32)
        self._L.ref_crc32c_uniform(buf.ctypes.data, stride, length, init & 0xFFFFFFFF,
                                   out.ctypes.data, nblocks, threads)
        return out


    def batch(self, buf: np.ndarray, offsets, lengths) -> np.ndarray:
        """Value() over block i = buf[offsets[i], + lengths[i]), 1 thread."""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
        assert offsets.size == lengths.size
        assert offsets.size == 0 or int((offsets + lengths).max()) <= buf.size
        out = np.empty(offsets.size, dtype=np.uint32)
        self._L.ref_crc32c_batch(buf.ctypes.data, offsets.ctypes.data, lengths.ctypes.data,
                                 out.ctypes.data, offsets.size)
        return out


def reference_available() -> bool:
    return REF_LIB.exists()


# ---- splitmix64 (same stream as oracle/gen_golden.cc) -----------------------

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix_bytes(seed: int, n: int) -> np.ndarray:
    """n bytes: 8 little-endian bytes per splitmix64 output, state starting at
    `seed` and advancing by the golden gamma before each output."""
    nw = (n + 7) // 8
    with np.errstate(over="ignore"):
        i = np.arange(1, nw + 1, dtype=np.uint64)
        z = np.uint64(seed) + i * _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").view(np.uint8)[:n].copy()
