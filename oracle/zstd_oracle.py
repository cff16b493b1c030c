"""CPU restatement of the Zstd frame decoder (TEST INFRASTRUCTURE ONLY: the
checker of the device decoder, never the thing measured or shipped).

LevelDB's kZstdCompression blocks are read through
port::Zstd_GetUncompressedLength / Zstd_Uncompress (port/port_stdcxx.h:163-199):
ZSTD_getFrameContentSize, then ZSTD_decompressDCtx into exactly that many
bytes, in ReadBlock (table/format.cc:138-155). The as-built reference has
HAVE_ZSTD=0. Zstd is a third-party dependency absent from /root/reference;
the image carries /opt/conda/lib/libzstd.so.1.4.9 (no headers; its C ABI is
bound here with ctypes). This module restates the published format (RFC 8878,
"Zstandard Compression and the application/zstd Media Type") the way that
library decodes it:

  frame     = magic 0xFD2FB528, descriptor, [window], [dict id], [content
              size], blocks (raw / RLE / compressed, <= 128 KiB each), [XXH64
              low 32 bits of the content]
  compressed block = literals section (raw / RLE / Huffman with its tree /
              Huffman with the previous tree; 1 or 4 streams) + sequences
              section (count, LL / OF / ML modes: predefined / RLE / FSE
              table / repeat; one backward bitstream of three FSE states)
  execution = literals then match copies, offsets from three repeat
              offsets (1, 4, 8 at the frame's start)

Pinned by tests/test_zstd.py against the library itself (frames it writes
at several levels decode to the same bytes here, and every frame the
library accepts this accepts). Verdicts on damaged frames are checked for
agreement on a corpus; libzstd's exact error boundaries (which malformed
inputs it still decodes) are followed where the tests reach them
(`corrupt` below), not claimed in general.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

MAGIC = 0xFD2FB528
BLOCK_MAX = 128 * 1024
CONTENTSIZE_UNKNOWN = (1 << 64) - 1
CONTENTSIZE_ERROR = (1 << 64) - 2


class Corrupt(Exception):
    """A frame libzstd rejects (any ZSTD_isError result)."""


# ---- backward bitstreams (RFC 8878 §4.1.1.1, zstd's BIT_DStream) ---------

class BackBits:
    """Bits read from the end of `data[lo:hi]` toward its start, below the
    highest set bit of the last byte (the end marker)."""

    def __init__(self, data: bytes, lo: int, hi: int):
        if hi <= lo:
            raise Corrupt("empty bitstream")
        last = data[hi - 1]
        if last == 0:
            raise Corrupt("no end marker")
        self.x = int.from_bytes(data[lo:hi], "little")
        self.pos = 8 * (hi - lo - 1) + last.bit_length() - 1  # bits left

    def read(self, n: int) -> int:
        if n == 0:
            return 0
        self.pos -= n
        if self.pos >= 0:
            return (self.x >> self.pos) & ((1 << n) - 1)
        return (self.x << -self.pos) & ((1 << n) - 1)  # zeros past the start

    def peek(self, n: int) -> int:
        p = self.pos - n
        return (self.x >> p) & ((1 << n) - 1) if p >= 0 else (self.x << -p) & ((1 << n) - 1)

    def done_exact(self) -> bool:
        return self.pos == 0

    def overflowed(self) -> bool:
        return self.pos < 0


# ---- FSE (RFC 8878 §4.1) -------------------------------------------------

def read_ncount(data: bytes, p: int, end: int, max_symbol: int, max_log: int):
    """FSE table description at data[p:end]: (normalized counts, accuracy
    log, bytes used). Follows FSE_readNCount."""
    buf = bytes(data[p:end]) + bytes(8)
    if end - p < 1:
        raise Corrupt("ncount: no bytes")

    def rd32(i):
        return int.from_bytes(buf[i:i + 4], "little")

    ip = 0
    bits = rd32(0)
    log = (bits & 0xF) + 5
    if log > max_log:
        raise Corrupt("ncount: table log too large")
    bits >>= 4
    bit_count = 4
    nb = log + 1
    remaining = (1 << log) + 1
    threshold = 1 << log
    counts: List[int] = []
    prev0 = False
    s = 0
    while remaining > 1 and s <= max_symbol:
        if prev0:
            n0 = s
            while (bits & 0xFFFF) == 0xFFFF:
                n0 += 24
                ip += 2
                bits = rd32(ip) >> bit_count
            while (bits & 3) == 3:
                n0 += 3
                bits >>= 2
                bit_count += 2
            n0 += bits & 3
            bit_count += 2
            if n0 > max_symbol:
                raise Corrupt("ncount: too many zeros")
            while s < n0:
                counts.append(0)
                s += 1
            ip += bit_count >> 3
            bit_count &= 7
            bits = rd32(ip) >> bit_count
        mx = (2 * threshold - 1) - remaining
        if (bits & (threshold - 1)) < mx:
            count = bits & (threshold - 1)
            bit_count += nb - 1
        else:
            count = bits & (2 * threshold - 1)
            if count >= threshold:
                count -= mx
            bit_count += nb
        count -= 1
        remaining -= -count if count < 0 else count
        counts.append(count)
        s += 1
        prev0 = count == 0
        while remaining < threshold:
            nb -= 1
            threshold >>= 1
        ip += bit_count >> 3
        bit_count &= 7
        bits = rd32(ip) >> bit_count
    if remaining != 1 or bit_count > 32:
        raise Corrupt("ncount: counts do not sum")
    used = ip + ((bit_count + 7) >> 3)
    if used > end - p:
        raise Corrupt("ncount: past the end")
    return counts, log, used


def build_fse(counts: List[int], log: int):
    """FSE decoding table: [(symbol, nbBits, baseline)] (FSE_buildDTable)."""
    size = 1 << log
    high = size - 1
    sym = [0] * size
    nxt = [0] * len(counts)
    for s, c in enumerate(counts):
        if c == -1:
            sym[high] = s
            high -= 1
            nxt[s] = 1
        else:
            nxt[s] = c
    step = (size >> 1) + (size >> 3) + 3
    pos = 0
    for s, c in enumerate(counts):
        for _ in range(max(c, 0)):
            sym[pos] = s
            pos = (pos + step) & (size - 1)
            while pos > high:
                pos = (pos + step) & (size - 1)
    if pos != 0:
        raise Corrupt("fse: bad spread")
    table = []
    for u in range(size):
        s = sym[u]
        ns = nxt[s]
        nxt[s] += 1
        nbits = log - (ns.bit_length() - 1)
        table.append((s, nbits, (ns << nbits) - size))
    return table, log


LL_DEFAULT = ([4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 3, 2, 1,
               1, 1, 1, 1, -1, -1, -1, -1], 6)
ML_DEFAULT = ([1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
               1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1], 6)
OF_DEFAULT = ([1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1,
               -1, -1, -1], 5)

LL_BASE = list(range(16)) + [16, 18, 20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048,
                             4096, 8192, 16384, 32768, 65536]
LL_BITS = [0] * 16 + [1, 1, 1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16]
ML_BASE = list(range(3, 35)) + [35, 37, 39, 41, 43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027,
                                2051, 4099, 8195, 16387, 32771, 65539]
ML_BITS = [0] * 32 + [1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16]


# ---- Huffman literals (RFC 8878 §4.2) ------------------------------------

def huf_weights(data: bytes, p: int, end: int):
    """Huffman_Tree_Description at data[p:]: (weights incl. the last, bytes)."""
    if p >= end:
        raise Corrupt("huf: no header")
    hb = data[p]
    if hb >= 128:  # direct 4-bit weights
        n = hb - 127
        nbytes = (n + 1) // 2
        if p + 1 + nbytes > end:
            raise Corrupt("huf: weights past the end")
        w = []
        for i in range(n):
            b = data[p + 1 + i // 2]
            w.append(b >> 4 if i % 2 == 0 else b & 15)
        used = 1 + nbytes
    else:  # FSE-compressed weights (HUF_readStats -> FSE_decompress_wksp)
        if p + 1 + hb > end or hb == 0:
            raise Corrupt("huf: weights past the end")
        counts, log, nc = read_ncount(data, p + 1, p + 1 + hb, 255, 6)
        table, _ = build_fse(counts, log)
        bs = BackBits(data, p + 1 + nc, p + 1 + hb)
        s1 = bs.read(log)
        s2 = bs.read(log)
        w = []
        omax = 255

        def getsym(state):
            sym, nbits, base = table[state]
            return sym, base + bs.read(nbits)

        while True:
            if len(w) > omax - 2:
                raise Corrupt("huf: too many weights")
            sym, s1 = getsym(s1)
            w.append(sym)
            if bs.overflowed():
                w.append(table[s2][0])
                break
            if len(w) > omax - 2:
                raise Corrupt("huf: too many weights")
            sym, s2 = getsym(s2)
            w.append(sym)
            if bs.overflowed():
                w.append(table[s1][0])
                break
        used = 1 + hb
    if any(x > 11 for x in w):
        raise Corrupt("huf: weight > 11")
    total = sum((1 << x) >> 1 for x in w)
    if total == 0:
        raise Corrupt("huf: no weights")
    maxbits = total.bit_length()  # highbit(total) + 1
    if maxbits > 12:  # HUF_TABLELOG_MAX (weights stay <= 11)
        raise Corrupt("huf: tree too deep")
    rest = (1 << maxbits) - total
    if rest & (rest - 1):
        raise Corrupt("huf: last weight not a power of two")
    w.append(rest.bit_length())  # log2(rest) + 1
    # rank 1 must hold at least 2 symbols (an even count), HUF_readStats
    if sum(1 for x in w if x == 1) < 2 or sum(1 for x in w if x == 1) & 1:
        raise Corrupt("huf: bad rank 1")
    return w, maxbits, used


def huf_table(w: List[int], maxbits: int):
    """Decoding table of 2^maxbits entries: (symbol, nbBits)."""
    size = 1 << maxbits
    table = [None] * size
    pos = 0
    for weight in range(1, maxbits + 1):
        for s, x in enumerate(w):
            if x == weight:
                nb = maxbits + 1 - x
                span = 1 << (maxbits - nb)
                for i in range(span):
                    table[pos + i] = (s, nb)
                pos += span
    if pos != size:
        raise Corrupt("huf: table not full")
    return table, maxbits


def huf_stream(data: bytes, lo: int, hi: int, n: int, ht) -> bytes:
    table, mb = ht
    bs = BackBits(data, lo, hi)
    out = bytearray()
    for _ in range(n):
        s, nb = table[bs.peek(mb)]
        bs.pos -= nb
        out.append(s)
    if not bs.done_exact():
        raise Corrupt("huf: stream not consumed exactly")
    return bytes(out)


# ---- frames --------------------------------------------------------------

class FrameHeader:
    pass


def frame_header(src: bytes) -> FrameHeader:
    if len(src) < 5:
        raise Corrupt("frame: too short")
    if int.from_bytes(src[0:4], "little") != MAGIC:
        raise Corrupt("frame: bad magic")
    fhd = src[4]
    fcs_flag = fhd >> 6
    single = (fhd >> 5) & 1
    if (fhd >> 3) & 1:
        raise Corrupt("frame: reserved bit")
    checksum = (fhd >> 2) & 1
    did_flag = fhd & 3
    p = 5
    h = FrameHeader()
    h.window = None
    if not single:
        if p >= len(src):
            raise Corrupt("frame: header cut")
        wd = src[p]
        p += 1
        exp, mant = wd >> 3, wd & 7
        if 10 + exp > 31:
            raise Corrupt("frame: window too large")
        base = 1 << (10 + exp)
        h.window = base + (base >> 3) * mant
    did_size = [0, 1, 2, 4][did_flag]
    fcs_size = [1 if single else 0, 2, 4, 8][fcs_flag]
    if p + did_size + fcs_size > len(src):
        raise Corrupt("frame: header cut")
    h.dict_id = int.from_bytes(src[p:p + did_size], "little")
    p += did_size
    if fcs_size:
        fcs = int.from_bytes(src[p:p + fcs_size], "little")
        if fcs_size == 2:
            fcs += 256
        h.content_size = fcs
    else:
        h.content_size = CONTENTSIZE_UNKNOWN
    p += fcs_size
    if single:
        h.window = h.content_size
    h.checksum = checksum
    h.size = p
    return h


def frame_content_size(src: bytes) -> int:
    """ZSTD_getFrameContentSize: the size, UNKNOWN or ERROR (a skippable
    frame gives 0)."""
    if len(src) >= 4 and (int.from_bytes(src[0:4], "little") & 0xFFFFFFF0) == 0x184D2A50:
        return 0 if len(src) >= 8 else CONTENTSIZE_ERROR
    try:
        return frame_header(src).content_size
    except Corrupt:
        return CONTENTSIZE_ERROR


def _literals(data: bytes, p: int, end: int, st) -> Tuple[bytes, int]:
    b0 = data[p]
    ltype, sf = b0 & 3, (b0 >> 2) & 3
    if ltype in (0, 1):  # raw / RLE
        if sf in (0, 2):
            n, hs = b0 >> 3, 1
        elif sf == 1:
            if p + 2 > end:
                raise Corrupt("lit: header cut")
            n, hs = (b0 >> 4) + (data[p + 1] << 4), 2
        else:
            if p + 3 > end:
                raise Corrupt("lit: header cut")
            n, hs = (b0 >> 4) + (data[p + 1] << 4) + (data[p + 2] << 12), 3
        if n > BLOCK_MAX:
            raise Corrupt("lit: too large")
        if ltype == 0:
            if p + hs + n > end:
                raise Corrupt("lit: raw past the end")
            return bytes(data[p + hs:p + hs + n]), hs + n
        if p + hs + 1 > end:
            raise Corrupt("lit: rle past the end")
        return bytes([data[p + hs]]) * n, hs + 1
    # compressed / treeless
    hs = [3, 3, 4, 5][sf]
    if p + hs > end:
        raise Corrupt("lit: header cut")
    hv = int.from_bytes(data[p:p + hs], "little")
    bits = [10, 10, 14, 18][sf]
    n = (hv >> 4) & ((1 << bits) - 1)
    csize = (hv >> (4 + bits)) & ((1 << bits) - 1)
    streams = 1 if sf == 0 else 4
    if n > BLOCK_MAX:
        raise Corrupt("lit: too large")
    if p + hs + csize > end:
        raise Corrupt("lit: compressed past the end")
    q, qend = p + hs, p + hs + csize
    if ltype == 2:
        w, mb, used = huf_weights(data, q, qend)
        st["huf"] = huf_table(w, mb)
        q += used
    elif st.get("huf") is None:
        raise Corrupt("lit: treeless without a tree")
    ht = st["huf"]
    if streams == 1:
        out = huf_stream(data, q, qend, n, ht)
    else:
        if qend - q < 10:
            raise Corrupt("lit: jump table")
        s1 = int.from_bytes(data[q:q + 2], "little")
        s2 = int.from_bytes(data[q + 2:q + 4], "little")
        s3 = int.from_bytes(data[q + 4:q + 6], "little")
        a = q + 6
        b, c, d = a + s1, a + s1 + s2, a + s1 + s2 + s3
        if d > qend:
            raise Corrupt("lit: jump table past the end")
        seg = (n + 3) // 4
        if 3 * seg > n:
            raise Corrupt("lit: too few literals for 4 streams")
        out = (huf_stream(data, a, b, seg, ht) + huf_stream(data, b, c, seg, ht) +
               huf_stream(data, c, d, seg, ht) + huf_stream(data, d, qend, n - 3 * seg, ht))
    return out, hs + csize


def _seq_table(data, p, end, mode, default, max_sym, max_log, st, key):
    if mode == 0:
        st[key] = build_fse(*default)
        return 0
    if mode == 1:
        if p >= end:
            raise Corrupt("seq: rle cut")
        s = data[p]
        if s > max_sym:
            raise Corrupt("seq: rle symbol")
        st[key] = ([(s, 0, 0)], 0)
        return 1
    if mode == 2:
        counts, log, used = read_ncount(data, p, end, max_sym, max_log)
        st[key] = build_fse(counts, log)
        return used
    if st.get(key) is None:
        raise Corrupt("seq: repeat without a table")
    return 0


def _block(data: bytes, p: int, end: int, out: bytearray, st, frame_start: int, window: int):
    lits, used = _literals(data, p, end, st)
    q = p + used
    if q >= end:
        raise Corrupt("seq: missing")
    b0 = data[q]
    if b0 == 0:
        nseq, q = 0, q + 1
    elif b0 < 128:
        nseq, q = b0, q + 1
    elif b0 < 255:
        if q + 2 > end:
            raise Corrupt("seq: count cut")
        nseq, q = ((b0 - 128) << 8) + data[q + 1], q + 2
    else:
        if q + 3 > end:
            raise Corrupt("seq: count cut")
        nseq, q = data[q + 1] + (data[q + 2] << 8) + 0x7F00, q + 3
    if nseq == 0:
        if q != end:
            raise Corrupt("seq: bytes after an empty section")
        out += lits
        return
    if q >= end:
        raise Corrupt("seq: modes cut")
    modes = data[q]
    q += 1
    q += _seq_table(data, q, end, modes >> 6, LL_DEFAULT, 35, 9, st, "ll")
    q += _seq_table(data, q, end, (modes >> 4) & 3, OF_DEFAULT, 31, 8, st, "of")
    q += _seq_table(data, q, end, (modes >> 2) & 3, ML_DEFAULT, 52, 9, st, "ml")
    ll_t, ll_log = st["ll"]
    of_t, of_log = st["of"]
    ml_t, ml_log = st["ml"]
    bs = BackBits(data, q, end)
    sl, so_, sm = bs.read(ll_log), bs.read(of_log), bs.read(ml_log)
    lp = 0
    rep = st["rep"]
    for i in range(nseq):
        llc, mlc, ofc = ll_t[sl][0], ml_t[sm][0], of_t[so_][0]
        if ofc > 31:
            raise Corrupt("seq: offset code")
        ofv = (1 << ofc) + bs.read(ofc)
        ml = ML_BASE[mlc] + bs.read(ML_BITS[mlc])
        ll = LL_BASE[llc] + bs.read(LL_BITS[llc])
        if ofv > 3:
            off = ofv - 3
            rep[:] = [off, rep[0], rep[1]]
        else:
            idx = ofv - 1 + (1 if ll == 0 else 0)
            if idx == 0:
                off = rep[0]
            elif idx == 1:
                off = rep[1]
                rep[:] = [off, rep[0], rep[2]]
            elif idx == 2:
                off = rep[2]
                rep[:] = [off, rep[0], rep[1]]
            else:
                off = rep[0] - 1
                rep[:] = [off, rep[0], rep[1]]
            if off == 0:  # (1.4.9 forces a zero repeat offset to 1)
                off = rep[0] = 1
        # the states, LL then ML then OF (1.4.9 updates them after the last
        # sequence too, reading zeros past the stream's start)
        s, nb, base = ll_t[sl]
        sl = base + bs.read(nb)
        s, nb, base = ml_t[sm]
        sm = base + bs.read(nb)
        s, nb, base = of_t[so_]
        so_ = base + bs.read(nb)
        if lp + ll > len(lits):
            raise Corrupt("seq: literals overrun")
        out += lits[lp:lp + ll]
        lp += ll
        produced = len(out) - frame_start
        if off > produced:
            raise Corrupt("seq: offset before the frame")
        for _ in range(ml):
            out.append(out[-off])
    if bs.pos > 0:  # (past the start is accepted, as 1.4.9 does)
        raise Corrupt("seq: bits left")
    out += lits[lp:]


def decompress(src: bytes, capacity: int) -> bytes:
    """ZSTD_decompressDCtx(dst, capacity, src): the bytes, or Corrupt.
    Frames one after another (skippable frames skipped), as the library."""
    src = bytes(src)
    out = bytearray()
    p = 0
    if len(src) == 0:
        raise Corrupt("empty input")
    while p < len(src):
        rem = src[p:]
        if len(rem) >= 4 and (int.from_bytes(rem[0:4], "little") & 0xFFFFFFF0) == 0x184D2A50:
            if len(rem) < 8:
                raise Corrupt("skippable: cut")
            n = int.from_bytes(rem[4:8], "little")
            if 8 + n > len(rem):
                raise Corrupt("skippable: cut")
            p += 8 + n
            continue
        if len(rem) < 9:
            raise Corrupt("frame: shorter than a header and a block header")
        h = frame_header(rem)
        if h.dict_id:
            raise Corrupt("frame: dictionary required")
        q = p + h.size
        start = len(out)
        st = {"huf": None, "ll": None, "of": None, "ml": None, "rep": [1, 4, 8]}
        while True:
            if q + 3 > len(src):
                raise Corrupt("block: header cut")
            bh = int.from_bytes(src[q:q + 3], "little")
            q += 3
            last, btype, bsize = bh & 1, (bh >> 1) & 3, bh >> 3
            if btype == 3:
                raise Corrupt("block: reserved type")
            if btype == 1:
                if q + 1 > len(src):
                    raise Corrupt("block: rle cut")
                if len(out) + bsize > capacity:
                    raise Corrupt("dst too small")
                out += bytes([src[q]]) * bsize
                q += 1
            else:
                if btype == 2 and bsize >= BLOCK_MAX:
                    raise Corrupt("block: too large")
                if q + bsize > len(src):
                    raise Corrupt("block: cut")
                if btype == 0:
                    out += src[q:q + bsize]
                else:
                    if bsize < 3:
                        raise Corrupt("block: compressed block under 3 bytes")
                    _block(src, q, q + bsize, out, st, start, h.window)
                q += bsize
            if len(out) > capacity:
                raise Corrupt("dst too small")
            if last:
                break
        if h.content_size != CONTENTSIZE_UNKNOWN and len(out) - start != h.content_size:
            raise Corrupt("frame: content size mismatch")
        if h.checksum:
            if q + 4 > len(src):
                raise Corrupt("frame: checksum cut")
            import xxhash
            want = xxhash.xxh64(bytes(out[start:]), seed=0).intdigest() & 0xFFFFFFFF
            if int.from_bytes(src[q:q + 4], "little") != want:
                raise Corrupt("frame: checksum")
            q += 4
        p = q
    return bytes(out)


# ---- ReadBlock's use (port/port_stdcxx.h:163-199) -------------------------

def get_uncompressed_length(src: bytes) -> Optional[int]:
    """port::Zstd_GetUncompressedLength: ZSTD_getFrameContentSize, false on 0
    (UNKNOWN and ERROR pass through as huge values, as the port does)."""
    v = frame_content_size(src)
    return None if v == 0 else v


HUGE = 1 << 26  # a content size past any block: the caller's (device: CAPACITY)


def uncompress(src: bytes) -> Tuple[Optional[bool], bytes]:
    """port::Zstd_Uncompress into a buffer of the content size: (True,
    bytes), (False, b"") when it fails, (None, b"") when the frame's content
    size is unknown or past HUGE (the port would allocate that much)."""
    n = get_uncompressed_length(src)
    if n is None:
        return False, b""
    if n >= HUGE:
        return None, b""
    try:
        return True, decompress(src, n)
    except Corrupt:
        return False, b""


# ---- the system library (the pin), where the image has it ----------------

def system_zstd():
    import ctypes
    import os
    for p in ("/opt/conda/lib/libzstd.so.1.4.9", "/opt/conda/lib/libzstd.so.1"):
        if os.path.exists(p):
            try:
                lib = ctypes.CDLL(p)
            except OSError:
                continue
            sz, vp = ctypes.c_size_t, ctypes.c_void_p
            lib.ZSTD_compressBound.restype = sz
            lib.ZSTD_compressBound.argtypes = [sz]
            lib.ZSTD_compress.restype = sz
            lib.ZSTD_compress.argtypes = [vp, sz, ctypes.c_char_p, sz, ctypes.c_int]
            lib.ZSTD_decompress.restype = sz
            lib.ZSTD_decompress.argtypes = [vp, sz, ctypes.c_char_p, sz]
            lib.ZSTD_isError.restype = ctypes.c_uint
            lib.ZSTD_isError.argtypes = [sz]
            lib.ZSTD_getFrameContentSize.restype = ctypes.c_ulonglong
            lib.ZSTD_getFrameContentSize.argtypes = [ctypes.c_char_p, sz]
            return lib
    return None


def lib_compress(lib, data: bytes, level: int = 1) -> bytes:
    import ctypes
    cap = lib.ZSTD_compressBound(len(data))
    out = ctypes.create_string_buffer(max(cap, 1))
    n = lib.ZSTD_compress(out, cap, data, len(data), level)
    assert not lib.ZSTD_isError(n)
    return out.raw[:n]


def lib_uncompress(lib, src: bytes) -> Tuple[Optional[bool], bytes]:
    """port::Zstd_Uncompress through the library."""
    import ctypes
    n = lib.ZSTD_getFrameContentSize(src, len(src))
    if n == 0:
        return False, b""
    if n >= HUGE:
        return None, b""  # (the port would try to allocate that much)
    out = ctypes.create_string_buffer(max(n, 1))
    r = lib.ZSTD_decompress(out, n, src, len(src))
    if lib.ZSTD_isError(r):
        return False, b""
    return True, out.raw[:r]
