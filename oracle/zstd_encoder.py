"""CPU restatement of the Zstd block compressor as LevelDB calls it (TEST
INFRASTRUCTURE ONLY: the checker of the device compressor, never the thing
measured or shipped).

What it restates. TableBuilder::WriteBlock's kZstdCompression case
(table/table_builder.cc:172-185) calls port::Zstd_Compress
(port/port_stdcxx.h:133-161):

    ctx = ZSTD_createCCtx()
    p   = ZSTD_getCParams(level, max(n, 1), 0)     # level = options.
    ZSTD_CCtx_setCParams(ctx, p)                   #  zstd_compression_level
    out = ZSTD_compress2(ctx, dst, ZSTD_compressBound(n), src, n)   # (= 1)

Zstd is a third-party dependency absent from /root/reference. The image
carries libzstd 1.4.9 (/opt/conda/lib/libzstd.so.1.4.9, zstd.h in
/opt/conda/include), the library port_stdcxx.h would link. 1.4.9 has no
ZSTD_CCtx_setCParams (it arrived in 1.5.x, defined there as the seven
ZSTD_CCtx_setParameter calls windowLog, chainLog, hashLog, searchLog,
minMatch, targetLength, strategy), so the fixtures make exactly those seven
calls (tests/golden/gen_zstd_write.py). The context keeps its default
compression level (3) underneath, whose parameters the seven calls override
field by field (a zero field, e.g. targetLength 0, does not override: level
3's is 0 too).

This module restates libzstd 1.4.9's code for the parameters that sequence
produces when the strategy is ZSTD_fast (levels <= 1 at every size, level 2
below 128 KiB; LevelDB's default level is 1):

  cparams      ZSTD_getCParams rows for those levels + ZSTD_adjustCParams'
               size fit (pinned to the library on a grid)
  frame        ZSTD_writeFrameHeader (content size always, single segment
               when the window covers it, no checksum, no dictionary), the
               128 KiB blocks of ZSTD_compress_frameChunk, raw / RLE /
               compressed block headers, the empty frame's last raw block
  matcher      ZSTD_compressBlock_fast_generic (two positions a step, the
               repcode test at ip+2, step = (ip - anchor) >> 7 + stepSize,
               the two hash-table fills and the offset_2 loop after a match)
  literals     ZSTD_compressLiterals: raw below 64 bytes or when disabled
               (fast with targetLength > 0), HUF_compress_internal (count,
               RLE, "not compressible enough", HUF_optimalTableLog,
               HUF_buildCTable with HUF_setMaxHeight, HUF_writeCTable with
               FSE-compressed or 4-bit weights, 1 or 4 streams), minGain
  sequences    ZSTD_seqToCodes, ZSTD_selectEncodingType (fast: predefined,
               RLE or new table; never the cost search), ZSTD_buildCTable
               (FSE_optimalTableLog, FSE_normalizeCount + FSE_normalizeM2,
               FSE_writeNCount, FSE_buildCTable), ZSTD_encodeSequences
  block rules  MIN_CBLOCK_SIZE (< 7 bytes: raw), minGain (cSize >= n -
               (n >> 6) - 2: raw), the 1.3.4-decoder guard (a last NCount
               within 4 bytes of the end: raw), RLE for a later block of
               one byte, entropy tables and repcodes carried only past a
               compressed block (HUF repeat: HUF_validateCTable, preferRepeat
               under 1 KiB of literals, HUF_estimateCompressedSize)

Pinned by tests/test_zstd_write.py: byte for byte against the committed
fixtures (tests/golden/zstd_write*.bin, the library's own frames through the
port's call sequence) and, where the library is present, against it on fuzz
inputs.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

MAGIC = 0xFD2FB528
BLOCKSIZE_MAX = 128 * 1024
MIN_CBLOCK_SIZE = 3
BLOCK_HEADER = 3
HASH_READ_SIZE = 8
K_SEARCH_STRENGTH = 8
REP_MOVE = 2
MINMATCH = 3
HUF_TABLELOG_DEFAULT = 11
HUF_TABLELOG_MAX = 12
FSE_MIN_TABLELOG = 5
FSE_MAX_TABLELOG = 12
MAX_FSE_TABLELOG_FOR_HUFF_HEADER = 6
LONGNBSEQ = 0x7F00
MAX_LL, MAX_ML, MAX_OFF, DEFAULT_MAX_OFF = 35, 52, 31, 28
LL_FSELOG, ML_FSELOG, OFF_FSELOG = 9, 9, 8
STRAT_FAST = 1

# predefined distributions (zstd_internal.h; RFC 8878 §3.1.1.3.2.2)
LL_DEFAULT_NORM = [4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 3,
                   2, 1, 1, 1, 1, 1, -1, -1, -1, -1]
ML_DEFAULT_NORM = [1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                   1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1,
                   -1, -1]
OF_DEFAULT_NORM = [1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1,
                   -1, -1, -1, -1]
LL_DEFAULT_LOG, ML_DEFAULT_LOG, OF_DEFAULT_LOG = 6, 6, 5

LL_BITS = [0] * 16 + [1, 1, 1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16]
ML_BITS = [0] * 32 + [1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16]
_LL_CODE = (list(range(16)) + [16, 16, 17, 17, 18, 18, 19, 19] + [20] * 4 + [21] * 4 +
            [22] * 8 + [23] * 8 + [24] * 16)
_ML_CODE = (list(range(32)) + [32, 32, 33, 33, 34, 34, 35, 35] + [36] * 4 + [37] * 4 +
            [38] * 8 + [39] * 8 + [40] * 16 + [41] * 16 + [42] * 32)

PRIME = {4: 2654435761, 5: 889523592379, 6: 227718039650203, 7: 58295818150454627,
         8: 0xCF1BBCDCB7A56463}
M64 = (1 << 64) - 1


class Unsupported(Exception):
    """Parameters outside the fast strategy (not restated here)."""


def highbit(v: int) -> int:
    return v.bit_length() - 1


def ll_code(ll: int) -> int:
    return highbit(ll) + 19 if ll > 63 else _LL_CODE[ll]


def ml_code(mlbase: int) -> int:
    return highbit(mlbase) + 36 if mlbase > 127 else _ML_CODE[mlbase]


# ---- parameters (ZSTD_getCParams / ZSTD_adjustCParams_internal) -----------

# (W, C, H, S, L, TL, strategy) rows of ZSTD_defaultCParameters for the
# levels whose strategy is ZSTD_fast; [table][level] with level 0 = the
# base row for negative levels. Tables: > 256 KiB, <= 256 KiB, <= 128 KiB,
# <= 16 KiB. (Level 2 at <= 256 KiB is ZSTD_dfast: not restated.)
_ROWS = {
    0: {0: (19, 12, 13, 1, 6, 1, 1), 1: (19, 13, 14, 1, 7, 0, 1), 2: (20, 15, 16, 1, 6, 0, 1)},
    1: {0: (18, 12, 13, 1, 5, 1, 1), 1: (18, 13, 14, 1, 6, 0, 1)},
    2: {0: (17, 12, 12, 1, 5, 1, 1), 1: (17, 12, 13, 1, 6, 0, 1), 2: (17, 13, 15, 1, 5, 0, 1)},
    3: {0: (14, 12, 13, 1, 5, 1, 1), 1: (14, 14, 15, 1, 5, 0, 1), 2: (14, 14, 15, 1, 4, 0, 1)},
}
MIN_CLEVEL = -(1 << 17)


def _table_id(size: int) -> int:
    # ZSTD_getCParams_internal: tableID = (rSize <= 256K) + (<= 128K) + (<= 16K)
    return (size <= 256 * 1024) + (size <= 128 * 1024) + (size <= 16 * 1024)


def get_cparams(level: int, size_hint: int) -> Tuple[int, ...]:
    """ZSTD_getCParams(level, size_hint, 0) for a fast-strategy level."""
    if level == 0:
        level = 3
    row_level = 0 if level < 0 else level
    rows = _ROWS[_table_id(size_hint)]
    if row_level not in rows:
        raise Unsupported(f"level {level} at {size_hint} bytes is not ZSTD_fast")
    w, c, h, s, l_, tl, st = rows[row_level]
    if level < 0:
        tl = -max(MIN_CLEVEL, level)
    return adjust_cparams((w, c, h, s, l_, tl, st), size_hint)


def adjust_cparams(cp, src_size: int):
    """ZSTD_adjustCParams_internal(cPar, srcSize, dictSize = 0)."""
    w, c, h, s, l_, tl, st = cp
    max_window_resize = 1 << 30  # 1ULL << (ZSTD_WINDOWLOG_MAX - 1) on 64-bit
    if src_size < max_window_resize:
        src_log = 6 if src_size < 64 else highbit(src_size - 1) + 1
        if w > src_log:
            w = src_log
    if h > w + 1:
        h = w + 1
    cycle = c - (1 if st >= 6 else 0)  # ZSTD_cycleLog (btlazy2 and up)
    if cycle > w:
        c -= cycle - w
    if w < 10:  # ZSTD_WINDOWLOG_ABSOLUTEMIN
        w = 10
    return (w, c, h, s, l_, tl, st)


def port_cparams(level: int, n: int):
    """The parameters ZSTD_compress2 runs with after port::Zstd_Compress's
    getCParams(level, max(n, 1)) + setCParams: the set fields override the
    context's level-3 row, then ZSTD_getCParamsFromCCtxParams adjusts them
    to the pledged size n again."""
    cp = get_cparams(level, max(n, 1))
    if n == 0:
        return cp  # (srcSize 0: no resize; the frame is empty either way)
    return adjust_cparams(cp, n)


# ---- bit output (BIT_CStream: LSB first) ----------------------------------

class BitOut:
    __slots__ = ("v", "n")

    def __init__(self):
        self.v = 0
        self.n = 0

    def add(self, value: int, nbits: int):
        if nbits:
            self.v |= (value & ((1 << nbits) - 1)) << self.n
            self.n += nbits

    def close(self) -> bytes:
        """BIT_closeCStream: the end mark, then whole bytes."""
        self.add(1, 1)
        return self.v.to_bytes((self.n + 7) // 8, "little")


# ---- FSE (fse_compress.c) -------------------------------------------------

def fse_min_table_log(src_size: int, max_sym: int) -> int:
    return min(highbit(src_size) + 1, highbit(max_sym) + 2)


def fse_optimal_table_log(max_log: int, src_size: int, max_sym: int, minus: int = 2) -> int:
    max_bits_src = highbit(src_size - 1) - minus
    tl = max_log if max_log else 11
    if max_bits_src < tl:
        tl = max_bits_src
    mb = fse_min_table_log(src_size, max_sym)
    if mb > tl:
        tl = mb
    return min(max(tl, FSE_MIN_TABLELOG), FSE_MAX_TABLELOG)


_RTB = [0, 473195, 504333, 520860, 550000, 700000, 750000, 830000]


def fse_normalize_count(count: List[int], tl: int, total: int, max_sym: int,
                        low_prob: bool) -> List[int]:
    """FSE_normalizeCount (useLowProbCount: -1 for the rarest symbols)."""
    low = -1 if low_prob else 1
    scale = 62 - tl
    step = (1 << 62) // total
    vstep = 1 << (scale - 20)
    still = 1 << tl
    largest, largest_p = 0, 0
    low_threshold = total >> tl
    norm = [0] * (max_sym + 1)
    for s in range(max_sym + 1):
        c = count[s]
        if c == total:
            raise AssertionError("rle in normalize")
        if c == 0:
            continue
        if c <= low_threshold:
            norm[s] = low
            still -= 1
        else:
            p = (c * step) >> scale
            if p < 8:
                rest = vstep * _RTB[p]
                p += 1 if (c * step) - (p << scale) > rest else 0
            if p > largest_p:
                largest_p, largest = p, s
            norm[s] = p
            still -= p
    if -still >= (norm[largest] >> 1):
        return _fse_normalize_m2(norm, tl, count, total, max_sym, low)
    norm[largest] += still
    return norm


def _fse_normalize_m2(norm, tl, count, total, max_sym, low):
    NA = -2
    distributed = 0
    low_threshold = total >> tl
    low_one = (total * 3) >> (tl + 1)
    for s in range(max_sym + 1):
        c = count[s]
        if c == 0:
            norm[s] = 0
        elif c <= low_threshold:
            norm[s] = low
            distributed += 1
            total -= c
        elif c <= low_one:
            norm[s] = 1
            distributed += 1
            total -= c
        else:
            norm[s] = NA
    to_dist = (1 << tl) - distributed
    if to_dist == 0:
        return norm
    if total // to_dist > low_one:
        low_one = (total * 3) // (to_dist * 2)
        for s in range(max_sym + 1):
            if norm[s] == NA and count[s] <= low_one:
                norm[s] = 1
                distributed += 1
                total -= count[s]
        to_dist = (1 << tl) - distributed
    if distributed == max_sym + 1:
        max_v, max_c = 0, 0
        for s in range(max_sym + 1):
            if count[s] > max_c:
                max_v, max_c = s, count[s]
        norm[max_v] += to_dist
        return norm
    if total == 0:
        s = 0
        while to_dist > 0:
            if norm[s] > 0:
                to_dist -= 1
                norm[s] += 1
            s = (s + 1) % (max_sym + 1)
        return norm
    vlog = 62 - tl
    mid = (1 << (vlog - 1)) - 1
    rstep = (((1 << vlog) * to_dist) + mid) // total
    tmp = mid
    for s in range(max_sym + 1):
        if norm[s] == NA:
            end = tmp + count[s] * rstep
            w = (end >> vlog) - (tmp >> vlog)
            if w < 1:
                raise AssertionError("normalizeM2: zero weight")
            norm[s] = w
            tmp = end
    return norm


def fse_write_ncount(norm: List[int], max_sym: int, tl: int) -> bytes:
    """FSE_writeNCount_generic."""
    out = bytearray()
    bit_stream = (tl - FSE_MIN_TABLELOG)
    bit_count = 4
    remaining = (1 << tl) + 1
    threshold = 1 << tl
    nb = tl + 1
    s = 0
    alphabet = max_sym + 1
    prev0 = False
    while s < alphabet and remaining > 1:
        if prev0:
            start = s
            while s < alphabet and norm[s] == 0:
                s += 1
            if s == alphabet:
                break
            while s >= start + 24:
                start += 24
                bit_stream += 0xFFFF << bit_count
                out += bytes([bit_stream & 255, (bit_stream >> 8) & 255])
                bit_stream >>= 16
            while s >= start + 3:
                start += 3
                bit_stream += 3 << bit_count
                bit_count += 2
            bit_stream += (s - start) << bit_count
            bit_count += 2
            if bit_count > 16:
                out += bytes([bit_stream & 255, (bit_stream >> 8) & 255])
                bit_stream >>= 16
                bit_count -= 16
        count = norm[s]
        s += 1
        mx = (2 * threshold - 1) - remaining
        remaining -= -count if count < 0 else count
        count += 1
        if count >= threshold:
            count += mx
        bit_stream += count << bit_count
        bit_count += nb
        bit_count -= 1 if count < mx else 0
        prev0 = count == 1
        if remaining < 1:
            raise AssertionError("ncount: negative remaining")
        while remaining < threshold:
            nb -= 1
            threshold >>= 1
        if bit_count > 16:
            out += bytes([bit_stream & 255, (bit_stream >> 8) & 255])
            bit_stream >>= 16
            bit_count -= 16
    if remaining != 1:
        raise AssertionError("ncount: bad distribution")
    out += bytes([bit_stream & 255, (bit_stream >> 8) & 255])[: (bit_count + 7) // 8]
    return bytes(out)


class FseCTable:
    """FSE_buildCTable_wksp: next-state table + per-symbol transforms."""

    def __init__(self, norm: List[int], max_sym: int, tl: int):
        size = 1 << tl
        mask = size - 1
        step = (size >> 1) + (size >> 3) + 3
        high = size - 1
        cumul = [0] * (max_sym + 2)
        table_sym = [0] * size
        for u in range(1, max_sym + 2):
            if norm[u - 1] == -1:
                cumul[u] = cumul[u - 1] + 1
                table_sym[high] = u - 1
                high -= 1
            else:
                cumul[u] = cumul[u - 1] + norm[u - 1]
        cumul[max_sym + 1] = size + 1
        pos = 0
        for s in range(max_sym + 1):
            for _ in range(max(norm[s], 0)):
                table_sym[pos] = s
                pos = (pos + step) & mask
                while pos > high:
                    pos = (pos + step) & mask
        assert pos == 0
        self.state = [0] * size
        for u in range(size):
            s = table_sym[u]
            self.state[cumul[s]] = size + u
            cumul[s] += 1
        self.dnb = [0] * (max_sym + 1)
        self.dfs = [0] * (max_sym + 1)
        total = 0
        for s in range(max_sym + 1):
            c = norm[s]
            if c == 0:
                self.dnb[s] = ((tl + 1) << 16) - (1 << tl)
            elif c in (-1, 1):
                self.dnb[s] = (tl << 16) - (1 << tl)
                self.dfs[s] = total - 1
                total += 1
            else:
                mbo = tl - highbit(c - 1)
                self.dnb[s] = (mbo << 16) - (c << mbo)
                self.dfs[s] = total - c
                total += c
        self.log = tl

    @classmethod
    def rle(cls, sym: int):
        t = cls.__new__(cls)
        t.state = [0, 0]
        t.dnb = [0] * (sym + 1)
        t.dfs = [0] * (sym + 1)
        t.log = 0
        return t

    def init_state(self, sym: int) -> int:
        """FSE_initCState2."""
        nbo = (self.dnb[sym] + (1 << 15)) >> 16
        v = (nbo << 16) - self.dnb[sym]
        return self.state[(v >> nbo) + self.dfs[sym]]

    def encode(self, bits: BitOut, st: int, sym: int) -> int:
        nbo = (st + self.dnb[sym]) >> 16
        bits.add(st, nbo)
        return self.state[(st >> nbo) + self.dfs[sym]]

    def flush(self, bits: BitOut, st: int):
        bits.add(st, self.log)


def fse_compress_using_ctable(src: List[int], ct: FseCTable) -> bytes:
    """FSE_compress_usingCTable (two interleaved states, from the end)."""
    n = len(src)
    if n <= 2:
        return b""
    bits = BitOut()
    ip = n
    if n & 1:
        ip -= 1
        s1 = ct.init_state(src[ip])
        ip -= 1
        s2 = ct.init_state(src[ip])
        ip -= 1
        s1 = ct.encode(bits, s1, src[ip])
    else:
        ip -= 1
        s2 = ct.init_state(src[ip])
        ip -= 1
        s1 = ct.init_state(src[ip])
    rem = n - 2
    if rem & 2:
        ip -= 1
        s2 = ct.encode(bits, s2, src[ip])
        ip -= 1
        s1 = ct.encode(bits, s1, src[ip])
    while ip > 0:
        ip -= 1
        s2 = ct.encode(bits, s2, src[ip])
        ip -= 1
        s1 = ct.encode(bits, s1, src[ip])
        ip -= 1
        s2 = ct.encode(bits, s2, src[ip])
        ip -= 1
        s1 = ct.encode(bits, s1, src[ip])
    ct.flush(bits, s2)
    ct.flush(bits, s1)
    return bits.close()


# ---- Huffman (huf_compress.c) ---------------------------------------------

def huf_build_ctable(count: List[int], max_sym: int, max_nb: int):
    """HUF_buildCTable_wksp: (nbBits per symbol, code per symbol, maxNbBits)."""
    # HUF_sort: decreasing count, ties in symbol order
    order = sorted(range(max_sym + 1), key=lambda s: -count[s])
    STARTNODE = 256
    # huffNode[-1] is the barrier: index shift by one
    size = 2 * 256 + 2
    cnt = [0] * size
    parent = [0] * size
    nbits = [0] * size
    sym = [0] * size
    for i, s in enumerate(order):
        cnt[i + 1] = count[s]
        sym[i + 1] = s

    def C(i):
        return cnt[i + 1]

    non_null = max_sym
    while C(non_null) == 0:
        non_null -= 1
    low_s = non_null
    node_nb = STARTNODE
    node_root = node_nb + low_s - 1
    low_n = node_nb
    cnt[node_nb + 1] = C(low_s) + C(low_s - 1)
    parent[low_s + 1] = parent[low_s - 1 + 1] = node_nb
    node_nb += 1
    low_s -= 2
    for n in range(node_nb, node_root + 1):
        cnt[n + 1] = 1 << 30
    cnt[0] = 1 << 31
    while node_nb <= node_root:
        if C(low_s) < C(low_n):
            n1 = low_s
            low_s -= 1
        else:
            n1 = low_n
            low_n += 1
        if C(low_s) < C(low_n):
            n2 = low_s
            low_s -= 1
        else:
            n2 = low_n
            low_n += 1
        cnt[node_nb + 1] = C(n1) + C(n2)
        parent[n1 + 1] = parent[n2 + 1] = node_nb
        node_nb += 1
    nbits[node_root + 1] = 0
    for n in range(node_root - 1, STARTNODE - 1, -1):
        nbits[n + 1] = nbits[parent[n + 1] + 1] + 1
    for n in range(0, non_null + 1):
        nbits[n + 1] = nbits[parent[n + 1] + 1] + 1
    node = [[cnt[i + 1], nbits[i + 1]] for i in range(non_null + 1)]
    max_nb = _huf_set_max_height(node, non_null, max_nb)
    nb_per_rank = [0] * (HUF_TABLELOG_MAX + 1)
    val_per_rank = [0] * (HUF_TABLELOG_MAX + 1)
    for n in range(non_null + 1):
        nb_per_rank[node[n][1]] += 1
    mn = 0
    for n in range(max_nb, 0, -1):
        val_per_rank[n] = mn
        mn += nb_per_rank[n]
        mn >>= 1
    sym_nb = [0] * (max_sym + 1)
    for n in range(max_sym + 1):
        sym_nb[sym[n + 1]] = node[n][1] if n <= non_null else 0
    code = [0] * (max_sym + 1)
    for s in range(max_sym + 1):
        code[s] = val_per_rank[sym_nb[s]] & 0xFFFF
        val_per_rank[sym_nb[s]] += 1
    return sym_nb, code, max_nb


def _huf_set_max_height(node, last_non_null: int, max_nb: int) -> int:
    """HUF_setMaxHeight over node[i] = [count, nbBits] (sorted, decreasing)."""
    largest = node[last_non_null][1]
    if largest <= max_nb:
        return largest

    def bits_at(i):  # huffNode[-1] is the zeroed barrier entry
        return node[i][1] if i >= 0 else 0
    total_cost = 0
    base_cost = 1 << (largest - max_nb)
    n = last_non_null
    while node[n][1] > max_nb:
        total_cost += base_cost - (1 << (largest - node[n][1]))
        node[n][1] = max_nb
        n -= 1
    while bits_at(n) == max_nb:
        n -= 1
    total_cost >>= (largest - max_nb)
    NOSYM = 0xF0F0F0F0
    rank_last = [NOSYM] * (HUF_TABLELOG_MAX + 2)
    cur = max_nb
    for pos in range(n, -1, -1):
        if node[pos][1] >= cur:
            continue
        cur = node[pos][1]
        rank_last[max_nb - cur] = pos
    while total_cost > 0:
        nb_dec = highbit(total_cost) + 1
        while nb_dec > 1:
            hi = rank_last[nb_dec]
            lo = rank_last[nb_dec - 1]
            if hi == NOSYM:
                nb_dec -= 1
                continue
            if lo == NOSYM:
                break
            if node[hi][0] <= 2 * node[lo][0]:
                break
            nb_dec -= 1
        while nb_dec <= HUF_TABLELOG_MAX and rank_last[nb_dec] == NOSYM:
            nb_dec += 1
        total_cost -= 1 << (nb_dec - 1)
        if rank_last[nb_dec - 1] == NOSYM:
            rank_last[nb_dec - 1] = rank_last[nb_dec]
        node[rank_last[nb_dec]][1] += 1
        if rank_last[nb_dec] == 0:
            rank_last[nb_dec] = NOSYM
        else:
            rank_last[nb_dec] -= 1
            if node[rank_last[nb_dec]][1] != max_nb - nb_dec:
                rank_last[nb_dec] = NOSYM
    while total_cost < 0:
        if rank_last[1] == NOSYM:
            while bits_at(n) == max_nb:
                n -= 1
            node[n + 1][1] -= 1
            rank_last[1] = n + 1
            total_cost += 1
            continue
        node[rank_last[1] + 1][1] -= 1
        rank_last[1] += 1
        total_cost += 1
    return max_nb


def _huf_compress_weights(weights: List[int]) -> Optional[bytes]:
    """HUF_compressWeights: the FSE form, or None (raw), or b"\\x01"-like
    sentinels returned as their size only (1 = rle, 0 = incompressible)."""
    ws = len(weights)
    if ws <= 1:
        return None
    count = [0] * (HUF_TABLELOG_MAX + 1)
    for w in weights:
        count[w] += 1
    max_sym = HUF_TABLELOG_MAX
    while count[max_sym] == 0:
        max_sym -= 1
    max_count = max(count)
    if max_count == ws or max_count == 1:
        return None  # (sizes 1 / 0: neither is kept, the 4-bit form follows)
    tl = fse_optimal_table_log(MAX_FSE_TABLELOG_FOR_HUFF_HEADER, ws, max_sym)
    norm = fse_normalize_count(count, tl, ws, max_sym, False)
    head = fse_write_ncount(norm, max_sym, tl)
    ct = FseCTable(norm, max_sym, tl)
    body = fse_compress_using_ctable(weights, ct)
    if not body:
        return None
    return head + body


def huf_write_ctable(sym_nb: List[int], max_sym: int, huf_log: int) -> bytes:
    """HUF_writeCTable."""
    to_w = [0] + [huf_log + 1 - n for n in range(1, huf_log + 1)]
    weights = [to_w[sym_nb[s]] for s in range(max_sym)]
    fse = _huf_compress_weights(weights)
    if fse is not None and 1 < len(fse) < max_sym // 2:
        return bytes([len(fse)]) + fse
    if max_sym > 128:
        raise AssertionError("huf: 4-bit weights past 128 symbols")
    weights.append(0)
    out = bytearray([128 + (max_sym - 1)])
    for n in range(0, max_sym, 2):
        out.append((weights[n] << 4) + weights[n + 1])
    return bytes(out)


def _huf_1x(src: bytes, nb: List[int], code: List[int]) -> bytes:
    """HUF_compress1X_usingCTable: symbols from the last to the first."""
    bits = BitOut()
    for i in range(len(src) - 1, -1, -1):
        s = src[i]
        bits.add(code[s], nb[s])
    return bits.close()


def huf_compress_ctable(src: bytes, streams: int, nb, code, head: bytes = b"") -> Optional[bytes]:
    """HUF_compressCTable_internal: head + streams, None when that does not
    pay (>= n - 1 bytes) or a stream is empty."""
    n = len(src)
    if streams == 1:
        out = _huf_1x(src, nb, code)
    else:
        if n < 12:
            return None
        seg = (n + 3) // 4
        parts = [src[0:seg], src[seg:2 * seg], src[2 * seg:3 * seg], src[3 * seg:]]
        enc = [_huf_1x(p, nb, code) for p in parts]
        if any(len(e) == 0 for e in enc):
            return None
        out = (len(enc[0]).to_bytes(2, "little") + len(enc[1]).to_bytes(2, "little") +
               len(enc[2]).to_bytes(2, "little") + b"".join(enc))
    if len(head) + len(out) >= n - 1:
        return None
    return head + out


class HufState:
    """ZSTD_hufCTables_t: the table a later block may repeat."""

    def __init__(self):
        self.repeat = "none"  # HUF_repeat_none / check
        self.nb = [0] * 256
        self.code = [0] * 256


def huf_compress(src: bytes, streams: int, prev: HufState, prefer_repeat: bool):
    """HUF_compress{1,4}X_repeat as ZSTD_compressLiterals calls it. Returns
    (payload or None for 'not compressed', 1-byte RLE marker, kind) where
    kind is 'new', 'repeat' or 'none'; prev is updated like *repeat and
    oldHufTable."""
    n = len(src)
    if n == 0:
        return None, "none"
    count = [0] * 256
    for b in src:
        count[b] += 1
    max_sym = 255
    while count[max_sym] == 0:
        max_sym -= 1
    largest = max(count)
    if largest == n:
        return bytes([src[0]]), "rle"
    if largest <= (n >> 7) + 4:
        return None, "none"
    if prev.repeat == "check" and any(count[s] and prev.nb[s] == 0 for s in range(max_sym + 1)):
        prev.repeat = "none"
    if prefer_repeat and prev.repeat != "none":
        return huf_compress_ctable(src, streams, prev.nb, prev.code), "repeat"
    huf_log = fse_optimal_table_log(HUF_TABLELOG_DEFAULT, n, max_sym, minus=1)
    nb, code, max_nb = huf_build_ctable(count, max_sym, huf_log)
    nb = nb + [0] * (256 - len(nb))
    code = code + [0] * (256 - len(code))
    head = huf_write_ctable(nb, max_sym, max_nb)
    if prev.repeat != "none":
        old = sum(count[s] * prev.nb[s] for s in range(max_sym + 1)) >> 3
        new = sum(count[s] * nb[s] for s in range(max_sym + 1)) >> 3
        if old <= len(head) + new or len(head) + 12 >= n:
            return huf_compress_ctable(src, streams, prev.nb, prev.code), "repeat"
    if len(head) + 12 >= n:
        return None, "none"
    prev.repeat = "none"
    prev.nb, prev.code = nb, code  # (oldHufTable overwritten: the new table)
    return huf_compress_ctable(src, streams, nb, code, head), "new"


def raw_literals(src: bytes) -> bytes:
    n = len(src)
    fl = 1 + (n > 31) + (n > 4095)
    if fl == 1:
        h = (n << 3).to_bytes(1, "little")
    elif fl == 2:
        h = ((1 << 2) + (n << 4)).to_bytes(2, "little")
    else:
        h = ((3 << 2) + (n << 4)).to_bytes(3, "little")
    return h + src


def rle_literals(src: bytes) -> bytes:
    n = len(src)
    fl = 1 + (n > 31) + (n > 4095)
    if fl == 1:
        h = (1 + (n << 3)).to_bytes(1, "little")
    elif fl == 2:
        h = (1 + (1 << 2) + (n << 4)).to_bytes(2, "little")
    else:
        h = (1 + (3 << 2) + (n << 4)).to_bytes(3, "little")
    return h + src[:1]


def compress_literals(lits: bytes, prev: HufState, disable: bool) -> Tuple[bytes, HufState]:
    """ZSTD_compressLiterals (strategy fast). Returns (section, next huf)."""
    n = len(lits)
    nxt = HufState()
    nxt.repeat, nxt.nb, nxt.code = prev.repeat, list(prev.nb), list(prev.code)
    if disable:
        return raw_literals(lits), nxt
    if n <= 63:  # COMPRESS_LITERALS_SIZE_MIN (repeat never 'valid' here)
        return raw_literals(lits), nxt
    min_gain = (n >> 6) + 2
    lh = 3 + (n >= 1024) + (n >= 16384)
    single = n < 256
    prefer = n <= 1024
    work = HufState()
    work.repeat, work.nb, work.code = nxt.repeat, nxt.nb, nxt.code
    payload, kind = huf_compress(lits, 1 if single else 4, work, prefer)
    if kind == "rle":
        return rle_literals(lits), nxt
    if payload is None or len(payload) >= n - min_gain:
        return raw_literals(lits), nxt
    if len(payload) == 1:
        return rle_literals(lits), nxt
    if kind == "repeat":
        htype = 3
    else:
        htype = 2
        nxt.repeat = "check"
        nxt.nb, nxt.code = work.nb, work.code
    c = len(payload)
    if lh == 3:
        h = (htype + ((not single) << 2) + (n << 4) + (c << 14)).to_bytes(3, "little")
    elif lh == 4:
        h = (htype + (2 << 2) + (n << 4) + (c << 18)).to_bytes(4, "little")
    else:
        h = ((htype + (3 << 2) + (n << 4) + (c << 22)) & 0xFFFFFFFF).to_bytes(4, "little") + \
            bytes([c >> 10])
    return h + payload, nxt


# ---- sequences (zstd_compress_sequences.c) --------------------------------

def select_encoding_type(count, max_sym, most_frequent, nbseq, default_log, default_allowed):
    """ZSTD_selectEncodingType for strategy < ZSTD_lazy, repeat mode none:
    0 basic, 1 rle, 2 compressed."""
    if most_frequent == nbseq:
        if default_allowed and nbseq <= 2:
            return 0
        return 1
    if default_allowed:
        mult = 10 - STRAT_FAST
        dyn_min = ((1 << default_log) * mult) >> 3
        if nbseq < dyn_min or most_frequent < (nbseq >> (default_log - 1)):
            return 0
    return 2


def build_ctable(kind, count, max_sym, codes, fse_log, default_norm, default_log, default_max):
    """ZSTD_buildCTable: (table description bytes, FseCTable)."""
    nbseq = len(codes)
    if kind == 1:
        return bytes([codes[0]]), FseCTable.rle(max_sym)
    if kind == 0:
        return b"", FseCTable(default_norm, default_max, default_log)
    count = list(count)
    tl = fse_optimal_table_log(fse_log, nbseq, max_sym)
    n1 = nbseq
    if count[codes[-1]] > 1:
        count[codes[-1]] -= 1
        n1 -= 1
    norm = fse_normalize_count(count, tl, n1, max_sym, n1 >= 2048)
    head = fse_write_ncount(norm, max_sym, tl)
    return head, FseCTable(norm, max_sym, tl)


def encode_sequences(seqs, llc, ofc, mlc, ct_ll, ct_of, ct_ml) -> bytes:
    """ZSTD_encodeSequences (64-bit; no long offsets below 2^57 windows)."""
    n = len(seqs)
    bits = BitOut()
    sm = ct_ml.init_state(mlc[n - 1])
    so = ct_of.init_state(ofc[n - 1])
    sl = ct_ll.init_state(llc[n - 1])
    ll, off, ml = seqs[n - 1]
    bits.add(ll, LL_BITS[llc[n - 1]])
    bits.add(ml, ML_BITS[mlc[n - 1]])
    bits.add(off, ofc[n - 1])
    for i in range(n - 2, -1, -1):
        ll, off, ml = seqs[i]
        so = ct_of.encode(bits, so, ofc[i])
        sm = ct_ml.encode(bits, sm, mlc[i])
        sl = ct_ll.encode(bits, sl, llc[i])
        bits.add(ll, LL_BITS[llc[i]])
        bits.add(ml, ML_BITS[mlc[i]])
        bits.add(off, ofc[i])
    ct_ml.flush(bits, sm)
    ct_of.flush(bits, so)
    ct_ll.flush(bits, sl)
    return bits.close()


def entropy_compress(lits: bytes, seqs, prev_huf: HufState, disable_lit: bool):
    """ZSTD_entropyCompressSequences_internal: (block body or None for
    'emit raw', next huf)."""
    out, nxt = compress_literals(lits, prev_huf, disable_lit)
    out = bytearray(out)
    nbseq = len(seqs)
    if nbseq < 128:
        out.append(nbseq)
    elif nbseq < LONGNBSEQ:
        out += bytes([(nbseq >> 8) + 0x80, nbseq & 255])
    else:
        out += bytes([0xFF]) + (nbseq - LONGNBSEQ).to_bytes(2, "little")
    if nbseq == 0:
        return bytes(out), nxt
    llc, ofc, mlc = [], [], []
    for ll, off, ml in seqs:
        llc.append(MAX_LL if ll >= 65536 else ll_code(ll))
        ofc.append(highbit(off))
        mlc.append(MAX_ML if ml >= 65536 else ml_code(ml))
    seq_head = len(out)
    out.append(0)
    last_ncount = None
    types = []
    tables = []
    for codes, mx, fse_log, dnorm, dlog, dmax, is_of in (
            (llc, MAX_LL, LL_FSELOG, LL_DEFAULT_NORM, LL_DEFAULT_LOG, MAX_LL, False),
            (ofc, MAX_OFF, OFF_FSELOG, OF_DEFAULT_NORM, OF_DEFAULT_LOG, DEFAULT_MAX_OFF, True),
            (mlc, MAX_ML, ML_FSELOG, ML_DEFAULT_NORM, ML_DEFAULT_LOG, MAX_ML, False)):
        count = [0] * (mx + 1)
        for c in codes:
            count[c] += 1
        m = mx
        while m > 0 and count[m] == 0:
            m -= 1
        most = max(count)
        allowed = (m <= DEFAULT_MAX_OFF) if is_of else True
        kind = select_encoding_type(count, m, most, nbseq, dlog, allowed)
        head, ct = build_ctable(kind, count, m, codes, fse_log, dnorm, dlog, dmax)
        if kind == 2:
            last_ncount = len(out)
        out += head
        types.append(kind)
        tables.append(ct)
    out[seq_head] = (types[0] << 6) + (types[1] << 4) + (types[2] << 2)
    # (the sequences' stored lengths are the low 16 bits of a long length)
    sq = [(ll & 0xFFFF, off, ml & 0xFFFF) for ll, off, ml in seqs]
    out += encode_sequences(sq, llc, ofc, mlc, tables[0], tables[1], tables[2])
    if last_ncount is not None and len(out) - last_ncount < 4:
        return None, nxt  # (zstd <= 1.3.4 decoder guard: emit raw)
    return bytes(out), nxt


# ---- the matcher (zstd_fast.c) --------------------------------------------

def _r32(b, i):
    return b[i] | (b[i + 1] << 8) | (b[i + 2] << 16) | (b[i + 3] << 24)


def _hash(b, i, hlog, mls):
    if mls == 4:
        return ((_r32(b, i) * PRIME[4]) & 0xFFFFFFFF) >> (32 - hlog)
    v = int.from_bytes(b[i:i + 8], "little")
    if mls < 8:
        v = (v << (64 - 8 * mls)) & M64
    return ((v * PRIME[mls]) & M64) >> (64 - hlog)


def _count(b, a, m, end):
    """ZSTD_count: equal bytes at a and m, a bounded by end."""
    n = 0
    while a + n < end and b[a + n] == b[m + n]:
        n += 1
    return n


class MatchState:
    """The frame's window: positions are indices into the frame's source
    plus 1 (window.base = src - 1, dictLimit = 1 after the first update)."""

    def __init__(self, hlog: int, mls: int, wlog: int, step_size: int):
        self.table = [0] * (1 << hlog)
        self.hlog = hlog
        self.mls = mls
        self.wlog = wlog
        self.step_size = step_size


def compress_block_fast(ms: MatchState, src: bytes, start: int, end: int, rep: List[int]):
    """ZSTD_compressBlock_fast_generic over src[start:end] (the frame's
    bytes before `start` are the window). Returns (sequences [(litLength,
    offset code + 1, matchLength - 3)], literals, last literals length);
    rep is updated in place as rep[0..1]."""
    hlog, mls, table = ms.hlog, ms.mls, ms.table
    b = src  # index i in b <-> window index i + 1
    istart, iend = start, end
    ilimit = iend - HASH_READ_SIZE
    end_index = iend + 1
    max_dist = 1 << ms.wlog
    prefix_start_index = end_index - max_dist if end_index - 1 > max_dist else 1
    prefix_start = prefix_start_index - 1  # as a position in b
    seqs = []
    lits = bytearray()
    anchor = istart
    ip0 = istart + (1 if istart == prefix_start else 0)
    ip1 = ip0 + 1
    off1, off2 = rep[0], rep[1]
    saved = 0
    cur = ip0 + 1
    wlow = cur - max_dist if cur - 1 > max_dist else 1
    max_rep = cur - wlow
    if off2 > max_rep:
        saved, off2 = off2, 0
    if off1 > max_rep:
        saved, off1 = off1, 0
    step_size = ms.step_size

    def store(litlen, anchor_pos, offcode, mlbase):
        lits.extend(b[anchor_pos:anchor_pos + litlen])
        seqs.append((litlen, offcode + 1, mlbase))

    while ip1 < ilimit:
        ip2 = ip0 + 2
        h0 = _hash(b, ip0, hlog, mls)
        val0 = _r32(b, ip0)
        h1 = _hash(b, ip1, hlog, mls)
        val1 = _r32(b, ip1)
        cur0 = ip0 + 1
        cur1 = ip1 + 1
        mi0 = table[h0]
        mi1 = table[h1]
        rep_match = ip2 - off1
        table[h0] = cur0
        table[h1] = cur1
        if off1 > 0 and _r32(b, rep_match) == _r32(b, ip2):
            ml = 1 if b[ip2 - 1] == b[rep_match - 1] else 0
            ip0 = ip2 - ml
            m0 = rep_match - ml
            ml += 4
            offcode = 0
        else:
            if mi0 > prefix_start_index and _r32(b, mi0 - 1) == val0:
                m0 = mi0 - 1
            elif mi1 > prefix_start_index and _r32(b, mi1 - 1) == val1:
                ip0 = ip1
                m0 = mi1 - 1
            else:
                step = ((ip0 - anchor) >> (K_SEARCH_STRENGTH - 1)) + step_size
                ip0 += step
                ip1 += step
                continue
            off2 = off1
            off1 = ip0 - m0
            offcode = off1 + REP_MOVE
            ml = 4
            while ip0 > anchor and m0 > prefix_start and b[ip0 - 1] == b[m0 - 1]:
                ip0 -= 1
                m0 -= 1
                ml += 1
        ml += _count(b, ip0 + ml, m0 + ml, iend)
        store(ip0 - anchor, anchor, offcode, ml - MINMATCH)
        ip0 += ml
        anchor = ip0
        if ip0 <= ilimit:
            table[_hash(b, cur0 + 2 - 1, hlog, mls)] = cur0 + 2
            table[_hash(b, ip0 - 2, hlog, mls)] = ip0 - 2 + 1
            if off2 > 0:
                while ip0 <= ilimit and _r32(b, ip0) == _r32(b, ip0 - off2):
                    rl = _count(b, ip0 + 4, ip0 + 4 - off2, iend) + 4
                    off1, off2 = off2, off1
                    table[_hash(b, ip0, hlog, mls)] = ip0 + 1
                    ip0 += rl
                    store(0, anchor, 0, rl - MINMATCH)
                    anchor = ip0
        ip1 = ip0 + 1
    rep[0] = off1 if off1 else saved
    rep[1] = off2 if off2 else saved
    last = iend - anchor
    lits.extend(b[anchor:iend])
    return seqs, bytes(lits), last


# ---- frame (zstd_compress.c) ----------------------------------------------

def frame_header(wlog: int, n: int) -> bytes:
    """ZSTD_writeFrameHeader: content size on, checksum off, no dict id."""
    window = 1 << wlog
    single = window >= n
    fcs = (n >= 256) + (n >= 65536 + 256) + (n >= 0xFFFFFFFF)
    fhd = (single << 5) + (fcs << 6)
    out = bytearray(MAGIC.to_bytes(4, "little"))
    out.append(fhd)
    if not single:
        out.append((wlog - 10) << 3)
    if fcs == 0:
        if single:
            out.append(n & 255)
    elif fcs == 1:
        out += (n - 256).to_bytes(2, "little")
    elif fcs == 2:
        out += n.to_bytes(4, "little")
    else:
        out += n.to_bytes(8, "little")
    return bytes(out)


def compress_bound(n: int) -> int:
    return n + (n >> 8) + (((128 << 10) - n) >> 11 if n < (128 << 10) else 0)


def compress(data: bytes, level: int = 1) -> bytes:
    """port::Zstd_Compress(level, data): the frame ZSTD_compress2 writes
    (libzstd 1.4.9) after getCParams(level, max(n, 1)) + setCParams."""
    data = bytes(data)
    n = len(data)
    w, c, h, s, mml, tl, strat = port_cparams(level, n)
    if strat != STRAT_FAST:
        raise Unsupported(f"strategy {strat}")
    out = bytearray(frame_header(w, n))
    if n == 0:
        out += (1).to_bytes(3, "little")  # the last (empty) raw block
        return bytes(out)
    mls = min(max(mml, 4), 7)  # ZSTD_compressBlock_fast: 3 -> 4, 4..7
    ms = MatchState(h, mls, w, tl + (0 if tl else 1) + 1)
    disable_lit = tl > 0  # ZSTD_disableLiteralsCompression (fast, TL > 0)
    block_size = min(BLOCKSIZE_MAX, 1 << w)
    rep = [1, 4, 8]
    huf = HufState()
    pos = 0
    first = True
    while pos < n:
        bs = min(block_size, n - pos)
        last = 1 if pos + bs >= n else 0
        body = None
        if bs >= MIN_CBLOCK_SIZE + BLOCK_HEADER + 1:
            nrep = list(rep)
            seqs, lits, _ = compress_block_fast(ms, data, pos, pos + bs, nrep)
            body, nhuf = entropy_compress(lits, seqs, huf, disable_lit)
            if body is not None and len(body) >= bs - ((bs >> 6) + 2):
                body = None
            blk = data[pos:pos + bs]
            # (a block not worth compressing has cSize 0, also < 25)
            if (not first and (0 if body is None else len(body)) < 25 and
                    blk.count(blk[0]) == bs):
                body = blk[:1]
            if body is not None and len(body) > 1:
                rep, huf = nrep, nhuf  # ZSTD_confirmRepcodesAndEntropyTables
        if body is None:
            out += (last + (0 << 1) + (bs << 3)).to_bytes(3, "little") + data[pos:pos + bs]
        elif len(body) == 1:
            out += (last + (1 << 1) + (bs << 3)).to_bytes(3, "little") + body
        else:
            out += (last + (2 << 1) + (len(body) << 3)).to_bytes(3, "little") + body
        pos += bs
        first = False
    return bytes(out)


def supported(level: int, n: int) -> bool:
    """Whether port::Zstd_Compress(level, n bytes) runs ZSTD_fast."""
    try:
        return port_cparams(level, n)[6] == STRAT_FAST
    except Unsupported:
        return False


# ---- the library through the port's exact calls (the pin) -----------------

class _CParams:
    pass


def system_zstd_writer():
    """libzstd 1.4.9 bound for port::Zstd_Compress's call sequence, or None."""
    import ctypes
    try:
        from oracle import zstd_oracle as zo
    except ImportError:  # (oracle/ itself on sys.path)
        import zstd_oracle as zo
    lib = zo.system_zstd()
    if lib is None:
        return None

    class CP(ctypes.Structure):
        _fields_ = [(f, ctypes.c_uint) for f in ("windowLog", "chainLog", "hashLog",
                                                 "searchLog", "minMatch", "targetLength",
                                                 "strategy")]
    lib.ZSTD_getCParams.restype = CP
    lib.ZSTD_getCParams.argtypes = [ctypes.c_int, ctypes.c_ulonglong, ctypes.c_size_t]
    lib.ZSTD_createCCtx.restype = ctypes.c_void_p
    lib.ZSTD_freeCCtx.argtypes = [ctypes.c_void_p]
    lib.ZSTD_CCtx_setParameter.restype = ctypes.c_size_t
    lib.ZSTD_CCtx_setParameter.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    lib.ZSTD_compress2.restype = ctypes.c_size_t
    lib.ZSTD_compress2.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                   ctypes.c_char_p, ctypes.c_size_t]
    lib._CP = CP
    return lib


def lib_port_compress(lib, data: bytes, level: int = 1) -> bytes:
    """port::Zstd_Compress (port/port_stdcxx.h:133-161) through the library:
    ZSTD_createCCtx; ZSTD_getCParams(level, max(n, 1), 0); ZSTD_CCtx_setCParams
    as 1.5.x defines it (seven ZSTD_CCtx_setParameter calls: windowLog 101,
    chainLog 103, hashLog 102, searchLog 104, minMatch 105, targetLength 106,
    strategy 107); ZSTD_compress2 into ZSTD_compressBound(n) bytes."""
    import ctypes
    n = len(data)
    cap = lib.ZSTD_compressBound(n)
    out = ctypes.create_string_buffer(max(cap, 1))
    ctx = lib.ZSTD_createCCtx()
    try:
        p = lib.ZSTD_getCParams(level, max(n, 1), 0)
        for param, field in ((101, "windowLog"), (103, "chainLog"), (102, "hashLog"),
                             (104, "searchLog"), (105, "minMatch"), (106, "targetLength"),
                             (107, "strategy")):
            r = lib.ZSTD_CCtx_setParameter(ctx, param, getattr(p, field))
            assert not lib.ZSTD_isError(r), (param, getattr(p, field))
        r = lib.ZSTD_compress2(ctx, out, cap, data, n)
        assert not lib.ZSTD_isError(r)
    finally:
        lib.ZSTD_freeCCtx(ctx)
    return out.raw[:r]
