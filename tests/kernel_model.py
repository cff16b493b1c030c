"""A line-by-line numpy model of crc32c_kernel.hip's per-block decomposition.

It runs the same geometry (end-aligned word grid, buffer window with
out-of-bounds-reads-as-zero, row-0 fix-ups, v_alignbyte re-alignment with the
lane+1 neighbour, Horner over rows with the Z_256 tables, per-lane Z_{256-4s}
nibble tables, wave xor-reduce) on the CPU with the library's own tables
(lvkv_debug_tables), so the math can be checked against the oracle without a
GPU. It is test infrastructure: it checks the design, the GPU tests check the
kernel.
"""
from __future__ import annotations

import numpy as np

POLY = 0x82F63B78  # reflected Castagnoli
M32 = 0xFFFFFFFF
LANES = np.arange(64, dtype=np.int64)


def _le32(mem: np.ndarray, a: int) -> int:
    return int(mem[a]) | int(mem[a + 1]) << 8 | int(mem[a + 2]) << 16 | int(mem[a + 3]) << 24


class KernelModel:
    def __init__(self, row_tab: np.ndarray, lane_tab: np.ndarray):
        self.A = row_tab.reshape(4, 256).astype(np.uint64)
        self.N = lane_tab.reshape(8, 16, 64).astype(np.uint64)

    def _row_adv(self, s: np.ndarray) -> np.ndarray:
        A = self.A
        return (A[0][s & 255] ^ A[1][(s >> 8) & 255] ^ A[2][(s >> 16) & 255]
                ^ A[3][(s >> 24) & 255])

    def _lane_shift(self, s: np.ndarray) -> np.ndarray:
        r = np.zeros(64, dtype=np.uint64)
        for k in range(8):
            nib = (s >> np.uint64(4 * k)) & np.uint64(15)
            r ^= self.N[k][nib.astype(np.int64), LANES]
        return r

    def block(self, mem: np.ndarray, ptr: int, length: int, init: int) -> int:
        s0 = (init ^ M32) & M32
        if length < 4:
            reg = s0
            for i in range(length):
                reg ^= int(mem[ptr + i])
                for _ in range(8):
                    reg = (reg >> 1) ^ (POLY if reg & 1 else 0)
            return reg ^ M32
        q = (length + 3) >> 2
        rows = (q + 63) >> 6
        delta = 4 * q - length
        s0l = 64 * rows - q
        spill = (s0 >> (32 - 8 * delta)) if delta else 0
        m = ptr & 3
        d = m - delta
        e = d & 3
        f = d >> 2
        b4 = ptr - m
        nrec = ((ptr + length + 3) & ~3) - b4
        vb0 = 4 * f - 4 * s0l

        def load(off: int) -> int:  # raw buffer load: u32 offset, OOB -> 0
            o = off & M32
            if o >= nrec:
                return 0
            return _le32(mem, b4 + o)

        nchunks = (rows + 15) // 16
        s = np.zeros(64, dtype=np.uint64)
        for c in range(nchunks):
            row0 = vb0 + 4096 * c
            buf = np.array([[load(row0 + 4 * ln + 256 * j) for ln in range(64)]
                            for j in range(16)], dtype=np.uint64)
            extra = np.zeros(64, dtype=np.uint64)
            extra[0] = load(row0 + 4096) if row0 + 4096 >= 0 else 0
            rowsets = np.vstack([buf, extra[None, :]])
            left = rows - 16 * c
            for j in range(min(16, left)):
                if e == 0:
                    w = rowsets[j].copy()
                else:
                    src = rowsets[j].copy()
                    src[0] = rowsets[j + 1][0]
                    hi = src[(LANES + 1) & 63]
                    w = ((hi << np.uint64(32) | rowsets[j]) >> np.uint64(8 * e)) & np.uint64(M32)
                if c == 0 and j == 0:
                    sh = 8 * delta
                    w = np.where(LANES < s0l, np.uint64(0), w)
                    first = (int(w[s0l]) & ((M32 << sh) & M32)) ^ ((s0 << sh) & M32)
                    w[s0l] = first
                    if s0l + 1 < 64:
                        w[s0l + 1] ^= np.uint64(spill)
                    s = w
                    continue
                if c == 0 and j == 1 and s0l == 63:
                    w[0] ^= np.uint64(spill)
                s = self._row_adv(s) ^ w
        tot = int(np.bitwise_xor.reduce(self._lane_shift(s)))
        return (tot ^ M32) & M32
