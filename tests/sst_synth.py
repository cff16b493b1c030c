"""Test helper: synthetic SSTable images in the reference's on-disk format.

Restates the layout TableBuilder writes (table/table_builder.cc:141-265,
table/format.cc:16-41, table/block_builder.cc): data blocks, an optional
filter block, the metaindex block (one "filter.<name>" entry), the index
block (block_restart_interval = 1, one entry per data block: separator key ->
BlockHandle), each followed by the 5-byte trailer [type][Mask(CRC32C(contents
+ type))], then the 48-byte footer [metaindex handle][index handle][padding]
[kTableMagicNumber LE]. Data-block contents are random bytes: the verify path
checks trailers and handles, never parses data entries. The golden
tests/golden/table.sst written by the reference itself pins the format; this
generator only scales it (thousands of blocks) for the GPU tests.
"""
from __future__ import annotations

import struct

import numpy as np

import oracle

MAGIC = 0xDB4775248B80FB57


def varint(v: int) -> bytes:
    out = bytearray()
    while v >= 128:
        out.append((v & 127) | 128)
        v >>= 7
    out.append(v)
    return bytes(out)


def handle(off: int, size: int) -> bytes:
    return varint(off) + varint(size)


def block(entries, restart_interval: int = 1) -> bytes:
    """BlockBuilder: prefix-compressed entries + restart array."""
    out, restarts, last = bytearray(), [], b""
    for i, (k, v) in enumerate(entries):
        if i % restart_interval == 0:
            restarts.append(len(out))
            shared = 0
        else:
            shared = 0
            while shared < min(len(k), len(last)) and k[shared] == last[shared]:
                shared += 1
        out += varint(shared) + varint(len(k) - shared) + varint(len(v)) + k[shared:] + v
        last = k
    if not restarts:
        restarts = [0]
    for r in restarts:
        out += struct.pack("<I", r)
    out += struct.pack("<I", len(restarts))
    return bytes(out)


def trailer(contents: bytes, btype: int = 0) -> bytes:
    return bytes([btype]) + struct.pack("<I", oracle.mask(oracle.value(contents + bytes([btype]))))


def build_sst(nblocks: int, block_bytes: int = 4096, seed: int = 1, with_filter: bool = True,
              ragged: bool = True, index_values=None, block_types=None) -> bytes:
    """index_values: {entry: raw value bytes} replacing an index entry's
    BlockHandle; block_types: {block: type byte} (trailer CRC still valid)."""
    index_values = index_values or {}
    block_types = block_types or {}
    rng = np.random.default_rng(seed)
    img = bytearray()
    index_entries = []
    for i in range(nblocks):
        n = block_bytes + (int(rng.integers(0, 300)) if ragged else 0)
        contents = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        off = len(img)
        img += contents + trailer(contents, block_types.get(i, 0))
        index_entries.append((b"key%08d" % i, index_values.get(i, handle(off, n))))
    meta_entries = []
    if with_filter:
        f = rng.integers(0, 256, 64 + nblocks // 4, dtype=np.uint8).tobytes()
        off = len(img)
        img += f + trailer(f)
        meta_entries.append((b"filter.leveldb.BuiltinBloomFilter2", handle(off, len(f))))
    meta = block(meta_entries, 16)
    meta_off = len(img)
    img += meta + trailer(meta)
    idx = block(index_entries, 1)
    idx_off = len(img)
    img += idx + trailer(idx)
    footer = handle(meta_off, len(meta)) + handle(idx_off, len(idx))
    footer = footer.ljust(40, b"\0") + struct.pack("<Q", MAGIC)
    return bytes(img + footer)


def fix_trailer(img: bytearray, off: int, size: int) -> None:
    """Recompute the masked CRC of block (off, size) after an edit."""
    c = oracle.mask(oracle.value(bytes(img[off: off + size + 1])))
    img[off + size + 1: off + size + 5] = struct.pack("<I", c)
