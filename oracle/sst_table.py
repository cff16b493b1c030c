"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's SSTable
walk, the checker for lvkv_sst_verify_table_device.

Restates, from the reference snapshot:
  * Table::Open's size check and footer read (table/table.cc:38-58);
  * Footer::DecodeFrom (table/format.cc:43-67) with kTableMagicNumber and
    kEncodedLength (table/format.h:53, :76);
  * BlockHandle::DecodeFrom = two GetVarint64 (table/format.cc:24-30,
    util/coding.cc GetVarint64Ptr);
  * ReadBlock's short-read, checksum and type checks (table/format.cc:69-160,
    kBlockTrailerSize table/format.h:79);
  * Block::Block's restart-array sanity and DecodeEntry (table/block.cc:25-75),
    walked entry by entry like Block::Iter::ParseNextKey (:252-280);
  * Table::ReadMeta's exact Seek("filter." + policy name) in the metaindex
    and ReadFilter (table/table.cc:81-124);
  * ReadBlock's size_t arithmetic for handles near 2^64 (format.cc:77-87).

Pinned by tests/golden/damage_sst.json: verdicts the reference's own
Table::Open / ReadBlock / Block::Iter / ReadMeta steps gave on damaged copies
of the reference-written table (oracle/gen_damage.cc).

Only tests/ import this module. Status codes are the ones
include/lvkv_crc32c.h defines for the device path.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import oracle

K_TABLE_MAGIC = 0xDB4775248B80FB57   # table/format.h:76
K_FOOTER_LEN = 48                    # table/format.h:53: 2 * 20 + 8
K_TRAILER = 5                        # table/format.h:79

# report.status (include/lvkv_crc32c.h, LVKV_SST_*)
SST_OK, SST_TOO_SHORT, SST_BAD_MAGIC, SST_BAD_HANDLE = 0, 1, 2, 3
SST_INDEX_TRUNCATED, SST_INDEX_CHECKSUM, SST_INDEX_TYPE = 4, 5, 6
SST_INDEX_CORRUPT, SST_CAPACITY = 7, 8
# per-block status (LVKV_BLOCK_*)
BLK_OK, BLK_CHECKSUM, BLK_TRUNCATED, BLK_BAD_TYPE, BLK_BAD_HANDLE, BLK_BAD_ENTRY = 0, 1, 2, 3, 4, 5
BLK_COMPRESSED, BLK_NOT_READ = 6, 7
BLOOM_POLICY = "leveldb.BuiltinBloomFilter2"   # util/bloom.cc BloomFilterPolicy::Name()
U64_MAX = (1 << 64) - 1


def get_varint(buf: bytes, pos: int, limit: int, max_shift: int) -> Tuple[Optional[int], int]:
    """GetVarint32Ptr / GetVarint64Ptr (util/coding.cc): (value, next pos) or
    (None, pos) when the varint runs past `limit` or is too long."""
    result, shift = 0, 0
    while shift <= max_shift and pos < limit:
        b = buf[pos]
        pos += 1
        if b & 128:
            result |= (b & 127) << shift
        else:
            return result | (b << shift), pos
        shift += 7
    return None, pos


def decode_handle(buf: bytes, pos: int, limit: int):
    """BlockHandle::DecodeFrom (table/format.cc:24-30)."""
    off, pos = get_varint(buf, pos, limit, 63)
    if off is None:
        return None, pos
    size, pos = get_varint(buf, pos, limit, 63)
    if size is None:
        return None, pos
    return (off, size), pos


def block_status(img: bytes, off: int, size: int) -> Tuple[int, int]:
    """ReadBlock with verify_checksums (table/format.cc:69-158) as built
    (no snappy/zstd): (status, crc of contents + type byte; 0 if none).

    n + kBlockTrailerSize is size_t arithmetic (:77-80): n = 2^64-1 reads
    4 bytes, passes the length test and compares Unmask of them with the CRC
    of zero bytes (0). n in [2^64-5, 2^64-2] reads before the reference's
    buffer (undefined): reported as a short read, as the device does."""
    avail = len(img) - off if off <= len(img) else -1
    if size == U64_MAX and avail >= 4:
        stored = oracle.unmask(struct.unpack_from("<I", img, off)[0])
        return (BLK_CHECKSUM if stored != 0 else BLK_TRUNCATED), 0
    if avail < 0 or size > 0xFFFFFFFE or avail < K_TRAILER or avail - K_TRAILER < size:
        return BLK_TRUNCATED, 0
    actual = oracle.value(img[off: off + size + 1])
    stored = oracle.unmask(struct.unpack_from("<I", img, off + size + 1)[0])
    if actual != stored:
        return BLK_CHECKSUM, actual
    t = img[off + size]
    if t in (1, 2):   # kSnappyCompression / kZstdCompression: no codec as built
        return BLK_COMPRESSED, actual
    if t > 2:
        return BLK_BAD_TYPE, actual
    return BLK_OK, actual


def decode_entry(img: bytes, p: int, limit: int):
    """DecodeEntry (table/block.cc:55-75): (shared, non_shared, value_len, p)."""
    if limit - p < 3:
        return None
    sh, ns, vl = img[p], img[p + 1], img[p + 2]
    if (sh | ns | vl) < 128:
        p += 3
    else:
        sh, p = get_varint(img, p, limit, 28)
        if sh is None:
            return None
        ns, p = get_varint(img, p, limit, 28)
        if ns is None:
            return None
        vl, p = get_varint(img, p, limit, 28)
        if vl is None:
            return None
    if limit - p < ns + vl:
        return None
    return sh, ns, vl, p


def restart_array(img: bytes, off: int, size: int):
    """Block::Block (table/block.cc:25-39): (restart_offset, [restarts]) or None."""
    if size < 4:
        return None
    n = struct.unpack_from("<I", img, off + size - 4)[0]
    if n > (size - 4) // 4:
        return None
    ro = size - (1 + n) * 4
    return ro, list(struct.unpack_from(f"<{n}I", img, off + ro))


@dataclass
class TableReport:
    status: int = SST_OK
    ndata: int = 0
    has_filter: int = 0
    index: Tuple[int, int] = (0, 0)
    meta: Tuple[int, int] = (0, 0)
    index_status: int = BLK_NOT_READ
    meta_status: int = BLK_NOT_READ
    index_crc: int = 0
    meta_crc: int = 0
    handles: List[Tuple[int, int]] = field(default_factory=list)  # data..., filter
    status_per_block: List[int] = field(default_factory=list)
    crc_per_block: List[int] = field(default_factory=list)

    @property
    def nblocks(self) -> int:
        return len(self.handles)

    @property
    def nbad(self) -> int:
        return sum(1 for s in self.status_per_block if s)


def _entry(r: TableReport, img: bytes, h) -> None:
    st, crc = block_status(img, *h)
    r.handles.append(h if st in (BLK_OK, BLK_CHECKSUM, BLK_BAD_TYPE, BLK_COMPRESSED)
                     and h[1] != U64_MAX else (0, 0))
    r.status_per_block.append(st)
    r.crc_per_block.append(crc if r.handles[-1] != (0, 0) or st == BLK_OK else None)


def find_filter(img: bytes, moff: int, msize: int, key: bytes):
    """Table::ReadMeta's Seek(key) + exact test (table.cc:95-102) on a
    well-formed, CRC-verified metaindex: the value of the entry whose key is
    exactly `key`, else None."""
    mra = restart_array(img, moff, msize)
    if mra is None:
        return None
    mro = mra[0]
    p, k = moff, b""
    while p < moff + mro:
        e = decode_entry(img, p, moff + mro)
        if e is None or e[0] > len(k):
            return None
        sh, ns, vl, q = e
        k = k[:sh] + img[q: q + ns]
        if k == key:
            return q + ns, q + ns + vl
        p = q + ns + vl
    return None


def verify_table(img: bytes, capacity: int = 1 << 30,
                 filter_policy: Optional[str] = BLOOM_POLICY) -> TableReport:
    r = TableReport()
    if len(img) < K_FOOTER_LEN:                           # table/table.cc:40-42
        r.status = SST_TOO_SHORT
        return r
    fo = len(img) - K_FOOTER_LEN
    magic = struct.unpack_from("<Q", img, fo + 40)[0]     # format.cc:48-53
    if magic != K_TABLE_MAGIC:
        r.status = SST_BAD_MAGIC
        return r
    meta, p = decode_handle(img, fo, fo + K_FOOTER_LEN)   # format.cc:58-61
    index, p = decode_handle(img, p, fo + K_FOOTER_LEN) if meta else (None, p)
    if meta is None or index is None:
        r.status = SST_BAD_HANDLE
        return r
    r.meta, r.index = meta, index
    r.index_status, r.index_crc = block_status(img, *index)
    r.meta_status, r.meta_crc = block_status(img, *meta)
    if r.index_status == BLK_TRUNCATED:
        r.status = SST_INDEX_TRUNCATED
        return r
    if r.index_status == BLK_CHECKSUM:
        r.status = SST_INDEX_CHECKSUM
        return r
    if r.index_status != BLK_OK:   # compressed (no codec as built) or bad type
        r.status = SST_INDEX_TYPE
        return r
    ioff, isize = index
    ra = restart_array(img, ioff, isize)
    if ra is None:
        r.status = SST_INDEX_CORRUPT   # Table::Open is OK; the index iterator fails
    else:
        ro, restarts = ra
        r.ndata = len(restarts)
        # The index is written with block_restart_interval = 1
        # (table/table_builder.cc:35, :90): one entry per restart point, shared 0.
        for i, rs in enumerate(restarts):
            end = restarts[i + 1] if i + 1 < len(restarts) else ro
            e = decode_entry(img, ioff + rs, ioff + ro) if rs < ro and end <= ro else None
            if e is None or e[0] != 0 or e[3] + e[1] + e[2] != ioff + end:
                r.handles.append((0, 0))
                r.status_per_block.append(BLK_BAD_ENTRY)
                r.crc_per_block.append(None)
                continue
            _, ns, vl, q = e
            h, _ = decode_handle(img, q + ns, q + ns + vl)
            if h is None:
                r.handles.append((0, 0))
                r.status_per_block.append(BLK_BAD_HANDLE)
                r.crc_per_block.append(None)
                continue
            _entry(r, img, h)
    # Table::ReadMeta + ReadFilter (table.cc:81-124): Open succeeded
    if filter_policy is not None and r.meta_status == BLK_OK:
        moff, msize = meta
        v = find_filter(img, moff, msize, b"filter." + filter_policy.encode())
        if v is not None:
            h, _ = decode_handle(img, v[0], v[1])
            if h is not None:
                _entry(r, img, h)
                r.has_filter = 1
    if r.nblocks > capacity:
        r.status = SST_CAPACITY
    return r
