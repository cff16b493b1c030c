"""TEST INFRASTRUCTURE ONLY — CPU restatement of log::Reader's physical
record walk, the checker for lvkv_log_verify_blocks_device (SURVEY.md §8f
row 2).

Restates log::Reader::ReadPhysicalRecord (db/log_reader.cc:189-271) with
checksum = true over a whole log image (initial_offset = 0; class Reader
restates the whole reader with an initial offset): 32 KiB reads
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


# ---- the logical layer: log::Reader::ReadRecord (db/log_reader.cc:55-176) ----
# Physical events, in file order, as ReadPhysicalRecord hands them over:
#   ("rec", header_offset, length, type)   a record whose checksum passed
#   ("bad", drop_bytes, reason)            kBadRecord; reason None = silent
#                                          (the zero-type zero-length skip)
#   ("eof",)                               kEof
K_FULL, K_FIRST, K_MIDDLE, K_LAST = 1, 2, 3, 4
K_EOF, K_BAD_RECORD = 5, 6  # log_reader.h: kMaxRecordType + 1, + 2


def physical_events(img: bytes):
    """The events the sequential walk above produces (ReadPhysicalRecord
    with checksum = true from offset 0)."""
    ev = []
    pos, eof = 0, False
    buf_start, buf_end = 0, 0
    while True:
        if buf_end - buf_start < K_HEADER:
            if not eof:
                buf_start = pos
                buf_end = min(len(img), pos + K_BLOCK)
                pos = buf_end
                if buf_end - buf_start < K_BLOCK:
                    eof = True
                continue
            ev.append(("eof",))
            return ev
        h = buf_start
        length = img[h + 4] | (img[h + 5] << 8)
        rtype = img[h + 6]
        if K_HEADER + length > buf_end - buf_start:
            drop = buf_end - buf_start
            buf_start = buf_end
            if not eof:
                ev.append(("bad", drop, "bad record length"))
                continue
            ev.append(("eof",))
            return ev
        if rtype == 0 and length == 0:
            buf_start = buf_end
            ev.append(("bad", 0, None))
            continue
        expected = oracle.unmask(struct.unpack_from("<I", img, h)[0])
        if oracle.value(img[h + 6: h + 7 + length]) != expected:
            drop = buf_end - buf_start
            buf_start = buf_end
            ev.append(("bad", drop, "checksum mismatch"))
            continue
        buf_start += K_HEADER + length
        ev.append(("rec", h, length, rtype))


def assemble(img: bytes, events):
    """ReadRecord over the physical events: the logical records it returns
    as (LastRecordOffset, length, CRC32C of the contents) and every
    Reporter::Corruption(bytes, reason) in order (physical and logical)."""
    records, reports = [], []
    it = iter(events)
    while True:
        in_frag, scratch, prospective = False, b"", 0
        done = False
        for e in it:
            if e[0] == "eof":
                return records, reports
            if e[0] == "bad":
                if e[2] is not None:
                    reports.append((e[1], e[2]))
                if in_frag:
                    reports.append((len(scratch), "error in middle of record"))
                    in_frag, scratch = False, b""
                continue
            _, h, length, rtype = e
            frag = img[h + K_HEADER: h + K_HEADER + length]
            # a header's own type byte 5 / 6 IS kEof / kBadRecord to ReadRecord
            # (ReadPhysicalRecord returns the byte as is, log_reader.cc:258-262;
            # switch at :143-161)
            if rtype == K_EOF:
                return records, reports
            if rtype == K_BAD_RECORD:
                if in_frag:
                    reports.append((len(scratch), "error in middle of record"))
                    in_frag, scratch = False, b""
                continue
            if rtype == K_FULL:
                if in_frag and scratch:
                    reports.append((len(scratch), "partial record without end(1)"))
                records.append((h, len(frag), oracle.value(frag)))
                done = True
                break
            if rtype == K_FIRST:
                if in_frag and scratch:
                    reports.append((len(scratch), "partial record without end(2)"))
                prospective, scratch, in_frag = h, frag, True
            elif rtype == K_MIDDLE:
                if not in_frag:
                    reports.append((len(frag), "missing start of fragmented record(1)"))
                else:
                    scratch += frag
            elif rtype == K_LAST:
                if not in_frag:
                    reports.append((len(frag), "missing start of fragmented record(2)"))
                else:
                    scratch += frag
                    records.append((prospective, len(scratch), oracle.value(scratch)))
                    done = True
                    break
            else:
                reports.append((len(frag) + (len(scratch) if in_frag else 0),
                                f"unknown record type {rtype}"))
                in_frag, scratch = False, b""
        if not done:
            return records, reports


class Reader:
    """log::Reader(file, reporter, checksum = true, initial_offset) as the
    reference has it (db/log_reader.cc:18-271), statement by statement, over
    an in-memory image whose Skip clamps at the end like a posix file: the
    restatement the initial-offset paths are checked against (resync, the
    trailer rule, ReportDrop's filter, physical records before the offset)."""

    def __init__(self, img: bytes, initial_offset: int = 0):
        self.img = img
        self.pos = 0                       # SequentialFile position
        self.buf = (0, 0)                  # buffer_ = img[buf[0]:buf[1]]
        self.eof = False
        self.last_record_offset = 0
        self.end_of_buffer_offset = 0
        self.initial_offset = initial_offset
        self.resyncing = initial_offset > 0  # :29
        self.reports = []
        self.stopped5 = False              # a header of type kEof ended ReadRecord

    def _bufsize(self):
        return self.buf[1] - self.buf[0]

    def _report_drop(self, nbytes, reason):  # :182-187 (unsigned arithmetic)
        if (self.end_of_buffer_offset - self._bufsize() - nbytes) % (1 << 64) >= self.initial_offset:
            self.reports.append((nbytes, reason))

    def _skip_to_initial_block(self):  # :33-54
        in_block = self.initial_offset % K_BLOCK
        start = self.initial_offset - in_block
        if in_block > K_BLOCK - 6:
            start += K_BLOCK
        self.end_of_buffer_offset = start
        if start > 0:
            self.pos = min(len(self.img), self.pos + start)
        return True

    def _read_physical(self):  # :189-271 -> (type, fragment offset, fragment length)
        img = self.img
        while True:
            if self._bufsize() < K_HEADER:
                if not self.eof:
                    end = min(len(img), self.pos + K_BLOCK)
                    self.buf = (self.pos, end)
                    self.end_of_buffer_offset += end - self.pos
                    if end - self.pos < K_BLOCK:
                        self.eof = True
                    self.pos = end
                    continue
                self.buf = (self.buf[1], self.buf[1])
                return K_EOF, 0, 0
            h = self.buf[0]
            length = img[h + 4] | (img[h + 5] << 8)
            rtype = img[h + 6]
            if K_HEADER + length > self._bufsize():
                drop = self._bufsize()
                self.buf = (self.buf[1], self.buf[1])
                if not self.eof:
                    self._report_drop(drop, "bad record length")
                    return K_BAD_RECORD, 0, 0
                return K_EOF, 0, 0
            if rtype == 0 and length == 0:
                self.buf = (self.buf[1], self.buf[1])
                return K_BAD_RECORD, 0, 0
            expected = oracle.unmask(struct.unpack_from("<I", img, h)[0])
            if oracle.value(img[h + 6: h + 7 + length]) != expected:
                drop = self._bufsize()
                self.buf = (self.buf[1], self.buf[1])
                self._report_drop(drop, "checksum mismatch")
                return K_BAD_RECORD, 0, 0
            self.buf = (h + K_HEADER + length, self.buf[1])
            if self.end_of_buffer_offset - self._bufsize() - K_HEADER - length < self.initial_offset:
                return K_BAD_RECORD, 0, 0   # :261-266, an empty fragment
            return rtype, h + K_HEADER, length

    def read_record(self):  # :56-174 -> bytes, or None when it returns false
        if self.last_record_offset < self.initial_offset:
            if not self._skip_to_initial_block():
                return None
        scratch = b""
        in_frag = False
        prospective = 0
        while True:
            rtype, fo, flen = self._read_physical()
            frag = self.img[fo: fo + flen]
            physical = self.end_of_buffer_offset - self._bufsize() - K_HEADER - flen
            if self.resyncing:                  # :80-89
                if rtype == K_MIDDLE:
                    continue
                if rtype == K_LAST:
                    self.resyncing = False
                    continue
                self.resyncing = False
            if rtype == K_FULL:
                if in_frag and scratch:
                    self._report_drop(len(scratch), "partial record without end(1)")
                self.last_record_offset = physical
                return frag
            if rtype == K_FIRST:
                if in_frag and scratch:
                    self._report_drop(len(scratch), "partial record without end(2)")
                prospective, scratch, in_frag = physical, frag, True
            elif rtype == K_MIDDLE:
                if not in_frag:
                    self._report_drop(len(frag), "missing start of fragmented record(1)")
                else:
                    scratch += frag
            elif rtype == K_LAST:
                if not in_frag:
                    self._report_drop(len(frag), "missing start of fragmented record(2)")
                else:
                    scratch += frag
                    self.last_record_offset = prospective
                    return scratch
            elif rtype == K_EOF:
                # a real kEof, or a header whose own type byte is 5
                self.stopped5 = fo != 0
                return None
            elif rtype == K_BAD_RECORD:
                if in_frag:
                    self._report_drop(len(scratch), "error in middle of record")
                    in_frag, scratch = False, b""
            else:
                self._report_drop(len(frag) + (len(scratch) if in_frag else 0),
                                  f"unknown record type {rtype}")
                in_frag, scratch = False, b""


def read_all(img: bytes, initial_offset: int = 0):
    """log::Reader(checksum = true, initial_offset) over the whole image:
    (LastRecordOffset, length, CRC32C of the contents) of every record
    ReadRecord returns, every Reporter::Corruption(bytes, reason), and
    whether a header of type kEof ended the reading."""
    r = Reader(img, initial_offset)
    records = []
    while True:
        rec = r.read_record()
        if rec is None:
            return records, r.reports, r.stopped5
        records.append((r.last_record_offset, len(rec), oracle.value(rec)))


def read_records(img: bytes, initial_offset: int = 0):
    """read_all's records and reports."""
    return read_all(img, initial_offset)[:2]


def events_from_blocks(img: bytes, hdrs, rec_status, block_status, block_drop):
    """The same physical events rebuilt from the per-block / per-record
    verdicts of the block form (and of lvkv_log_verify_blocks_device): a
    block's records up to its first mismatch, then its error, block by block;
    kEof after the last block (or at a truncated end)."""
    ev = []
    nblocks = (len(img) + K_BLOCK - 1) // K_BLOCK
    j = 0
    for b in range(nblocks):
        start, end = b * K_BLOCK, min(len(img), (b + 1) * K_BLOCK)
        while j < len(hdrs) and hdrs[j] < end:
            h = hdrs[j]
            if rec_status[j] == REC_OK:
                length = img[h + 4] | (img[h + 5] << 8)
                ev.append(("rec", h, length, img[h + 6]))
            j += 1
        st = block_status[b]
        if st == BLK_CHECKSUM:
            ev.append(("bad", int(block_drop[b]), "checksum mismatch"))
        elif st == BLK_BAD_LENGTH:
            ev.append(("bad", int(block_drop[b]), "bad record length"))
        elif st == BLK_ZERO:
            ev.append(("bad", 0, None))
        elif st == BLK_EOF:
            ev.append(("eof",))
            return ev
    ev.append(("eof",))
    return ev
