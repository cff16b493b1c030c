"""Test helper: log images in the reference's WAL format.

Restates log::Writer::AddRecord / EmitPhysicalRecord (db/log_writer.cc:34-108):
records are fragmented over 32 KiB blocks as FULL / FIRST / MIDDLE / LAST
physical records, a block tail shorter than the 7-byte header is zero-filled,
and each header is [Mask(CRC32C(type + payload)) u32][length u16][type u8].
The golden tests/golden/wal.log written by the reference pins the format;
this generator scales it for the GPU tests.
"""
from __future__ import annotations

import struct

import numpy as np

import oracle

K_BLOCK, K_HEADER = 32768, 7
FULL, FIRST, MIDDLE, LAST = 1, 2, 3, 4


class LogWriter:
    def __init__(self):
        self.buf = bytearray()
        self.block_offset = 0

    def emit(self, rtype: int, payload: bytes) -> None:
        crc = oracle.mask(oracle.value(bytes([rtype]) + payload))
        self.buf += struct.pack("<IHB", crc, len(payload), rtype) + payload
        self.block_offset += K_HEADER + len(payload)

    def add_record(self, data: bytes) -> None:
        left, pos, begin = len(data), 0, True
        while True:
            leftover = K_BLOCK - self.block_offset
            if leftover < K_HEADER:
                self.buf += b"\0" * leftover
                self.block_offset = 0
            avail = K_BLOCK - self.block_offset - K_HEADER
            frag = min(left, avail)
            end = left == frag
            rtype = FULL if begin and end else FIRST if begin else LAST if end else MIDDLE
            self.emit(rtype, data[pos: pos + frag])
            pos += frag
            left -= frag
            begin = False
            if left <= 0:
                break


def build_log(nrecords: int, seed: int = 1, max_len: int = 3000, big_every: int = 0) -> bytes:
    rng = np.random.default_rng(seed)
    w = LogWriter()
    for i in range(nrecords):
        n = int(rng.integers(0, max_len))
        if big_every and i % big_every == big_every - 1:
            n = 100_000  # spans several blocks: FIRST, MIDDLE..., LAST
        w.add_record(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
    return bytes(w.buf)


def fix_header_crc(img: bytearray, hdr: int) -> None:
    length = img[hdr + 4] | (img[hdr + 5] << 8)
    crc = oracle.mask(oracle.value(bytes(img[hdr + 6: hdr + 7 + length])))
    img[hdr: hdr + 4] = struct.pack("<I", crc)
