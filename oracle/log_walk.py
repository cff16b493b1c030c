"""TEST INFRASTRUCTURE ONLY — CPU restatement of log::Reader's physical
record walk, the checker for lvkv_log_verify_blocks_device (SURVEY.md §8f
row 2).

Restates log::Reader::ReadPhysicalRecord (db/log_reader.cc:189-271) with
checksum = true and initial_offset = 0 over a whole log image: 32 KiB reads
(db/log_format.h kBlockSize), the short-read EOF rule, the 7-byte header
[masked crc u32][length u16][type u8] (kHeaderSize), "bad record length"
(reported unless at EOF), the zero-type/zero-length skip (silent), "checksum
mismatch" (always reported, drops the rest of the block), ReportDrop's byte
counts (:182-187), and the trailer / truncated-header EOF cases.

Only tests/ import this module.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import List, Tuple

import oracle

K_BLOCK = 32768
K_HEADER = 7

# per-record status (include/lvkv_crc32c.h LVKV_REC_*)
REC_OK, REC_CHECKSUM, REC_DROPPED = 0, 1, 2
# per-block status (LVKV_LOGBLK_*)
BLK_OK, BLK_CHECKSUM, BLK_BAD_LENGTH, BLK_ZERO, BLK_EOF = 0, 1, 2, 3, 4


@dataclass
class LogWalk:
    records: List[Tuple[int, int, int]] = field(default_factory=list)  # returned: (hdr, len, type)
    corruptions: List[Tuple[int, str]] = field(default_factory=list)   # reported: (bytes, reason)


def read_physical_records(img: bytes) -> LogWalk:
    """The sequence ReadPhysicalRecord produces until kEof."""
    out = LogWalk()
    pos, eof = 0, False
    buf_start, buf_end = 0, 0   # the current buffer_ = img[buf_start:buf_end]
    while True:
        if buf_end - buf_start < K_HEADER:
            if not eof:                                   # :191-205
                buf_start = pos
                buf_end = min(len(img), pos + K_BLOCK)
                pos = buf_end
                if buf_end - buf_start < K_BLOCK:
                    eof = True
                continue
            return out                                    # :206-213
        h = buf_start
        length = img[h + 4] | (img[h + 5] << 8)           # :216-220
        rtype = img[h + 6]
        if K_HEADER + length > buf_end - buf_start:       # :221-232
            drop = buf_end - buf_start
            buf_start = buf_end
            if not eof:
                out.corruptions.append((drop, "bad record length"))
                continue
            return out
        if rtype == 0 and length == 0:                    # :234-240
            buf_start = buf_end
            continue
        expected = oracle.unmask(struct.unpack_from("<I", img, h)[0])  # :243-255
        actual = oracle.value(img[h + 6: h + 7 + length])
        if actual != expected:
            drop = buf_end - buf_start
            buf_start = buf_end
            out.corruptions.append((drop, "checksum mismatch"))
            continue
        buf_start += K_HEADER + length                    # :258
        out.records.append((h, length, rtype))


@dataclass
class BlockVerdicts:
    """Per 32 KiB block and per candidate record, the form the device path
    reports (derived from the sequential walk above)."""
    hdrs: List[int] = field(default_factory=list)          # candidate records, file order
    rec_status: List[int] = field(default_factory=list)
    block_status: List[int] = field(default_factory=list)
    block_drop: List[int] = field(default_factory=list)    # reported drop bytes


def block_verdicts(img: bytes) -> BlockVerdicts:
    """Per-block restatement of the same rules: a block's walk never depends
    on another block (headers do not straddle blocks, log_writer.cc:44-55)."""
    v = BlockVerdicts()
    nblocks = (len(img) + K_BLOCK - 1) // K_BLOCK
    for b in range(nblocks):
        start, end = b * K_BLOCK, min(len(img), (b + 1) * K_BLOCK)
        eof = end - start < K_BLOCK
        pos, status, drop, mismatch = start, BLK_OK, 0, False
        while end - pos >= K_HEADER:
            length = img[pos + 4] | (img[pos + 5] << 8)
            rtype = img[pos + 6]
            if K_HEADER + length > end - pos:
                if not mismatch:
                    status = BLK_EOF if eof else BLK_BAD_LENGTH
                    drop = 0 if eof else end - pos
                break
            if rtype == 0 and length == 0:
                if not mismatch:
                    status = BLK_ZERO
                break
            v.hdrs.append(pos)
            if mismatch:
                v.rec_status.append(REC_DROPPED)
            else:
                expected = oracle.unmask(struct.unpack_from("<I", img, pos)[0])
                if oracle.value(img[pos + 6: pos + 7 + length]) != expected:
                    mismatch, status, drop = True, BLK_CHECKSUM, end - pos
                    v.rec_status.append(REC_CHECKSUM)
                else:
                    v.rec_status.append(REC_OK)
            pos += K_HEADER + length
        else:
            if eof and pos < end and not mismatch:
                status = BLK_EOF  # truncated header at the end of the file
        v.block_status.append(status)
        v.block_drop.append(drop)
    return v
