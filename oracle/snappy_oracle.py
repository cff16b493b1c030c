"""CPU restatement of the Snappy block codec (TEST INFRASTRUCTURE ONLY: the
checker of the device codec, never the thing measured or shipped).

LevelDB's block compression calls Google Snappy
through port::Snappy_Compress / Snappy_GetUncompressedLength /
Snappy_Uncompress (port/port_stdcxx.h:90-133): snappy::RawCompress,
snappy::GetUncompressedLength and snappy::RawUncompress. The reference as
built here has HAVE_SNAPPY=0 (those return false: TableBuilder keeps blocks
raw, table_builder.cc:158-168; ReadBlock reports "corrupted snappy
compressed block length", format.cc:120-125). Snappy is a third-party
dependency absent from /root/reference; the image carries it as
/opt/conda/lib/libsnappy.so.1.1.8 (snappy 1.1.8, with its headers), and this
module restates that version's published algorithm (snappy.cc of 1.1.8):

  stream    = varint32(uncompressed length) ++ the fragments' elements
  fragments = the input in 64 KiB pieces (kBlockSize), each compressed alone
              with a fresh hash table of max(256, pow2 >= piece) <= 16384
              u16 entries
  elements  = literal: tag (len-1) << 2 | 0 (len-1 >= 60: 60 + k, then k
              bytes of len-1 LE), then the bytes;
              copy-1: (len-4) << 2 | (off >> 8) << 5 | 1, off & 255
              (4 <= len < 12, off < 2048);
              copy-2: (len-1) << 2 | 2, off LE16 (len <= 64);
              copy-4: (len-1) << 2 | 3, off LE32 (decoder only)
  matching  = CompressFragment: hash (u32 LE * 0x1e35a7bd) >> (32 - log2 T),
              heuristic skipping (skip = 32, step skip >> 5), greedy
              4-byte matches extended to the longest, EmitCopy in pieces of
              64 (60 when 64 < len < 68), the table updated at ip - 1 and ip
              after each copy, no match search in the last 15 bytes.

Pinned by tests/test_snappy.py: byte-for-byte against libsnappy 1.1.8 where
it is present (this container and the GPU image), and against the committed
fixtures tests/golden/snappy_*.{bin,json} generated from it
(tests/golden/gen_snappy.py). pyarrow bundles a newer snappy whose
compressor emits different (equally valid) streams for some inputs; its
decompressor agrees with this one on every stream.
"""
from __future__ import annotations

from typing import Optional, Tuple

K_BLOCK = 1 << 16
K_MAX_TABLE = 1 << 14
K_MUL = 0x1E35A7BD

# port/port_stdcxx.h / format.cc verdicts of the decoder
OK, BAD_LENGTH, BAD_CONTENTS = 0, 1, 2


def max_compressed_length(n: int) -> int:
    return 32 + n + n // 6


def _varint32(v: int) -> bytes:
    out = bytearray()
    while v >= 128:
        out.append((v & 127) | 128)
        v >>= 7
    out.append(v)
    return bytes(out)


def _u32(b: bytes, i: int) -> int:
    return b[i] | (b[i + 1] << 8) | (b[i + 2] << 16) | (b[i + 3] << 24)


def _table_size(n: int) -> int:
    t = 256
    while t < K_MAX_TABLE and t < n:
        t <<= 1
    return t


def _emit_literal(out: bytearray, lit: bytes) -> None:
    n = len(lit) - 1
    if n < 60:
        out.append(n << 2)
    else:
        count = (n.bit_length() - 1) // 8 + 1
        out.append((59 + count) << 2)
        out += n.to_bytes(4, "little")[:count]
    out += lit


def _emit_copy_at_most_64(out: bytearray, offset: int, length: int, lt12: bool) -> None:
    if lt12 and offset < 2048:
        out.append(1 + ((length - 4) << 2) + ((offset >> 3) & 0xE0))
        out.append(offset & 0xFF)
    else:
        u = 2 + ((length - 1) << 2) + (offset << 8)
        out += (u & 0xFFFFFF).to_bytes(3, "little")


def _emit_copy(out: bytearray, offset: int, length: int) -> None:
    if length < 12:
        _emit_copy_at_most_64(out, offset, length, True)
        return
    while length >= 68:
        _emit_copy_at_most_64(out, offset, 64, False)
        length -= 64
    if length > 64:
        _emit_copy_at_most_64(out, offset, 60, False)
        length -= 60
    _emit_copy_at_most_64(out, offset, length, length < 12)


def _compress_fragment(frag: bytes, out: bytearray) -> None:
    n = len(frag)
    tsize = _table_size(n)
    shift = 32 - (tsize.bit_length() - 1)
    table = [0] * tsize

    def h(i):
        return ((_u32(frag, i) * K_MUL) & 0xFFFFFFFF) >> shift

    ip = 0
    next_emit = 0
    if n >= 15:
        ip_limit = n - 15
        ip += 1
        next_hash = h(ip)
        while True:
            skip = 32
            next_ip = ip
            while True:
                ip = next_ip
                hh = next_hash
                step = skip >> 5
                skip += step
                next_ip = ip + step
                if next_ip > ip_limit:
                    break
                next_hash = h(next_ip)
                cand = table[hh]
                table[hh] = ip
                if _u32(frag, ip) == _u32(frag, cand):
                    break
            else:  # pragma: no cover
                pass
            if next_ip > ip_limit:
                break  # emit_remainder
            _emit_literal(out, frag[next_emit:ip])
            while True:
                base = ip
                m = 4
                while ip + m < n and frag[cand + m] == frag[ip + m]:
                    m += 1
                ip += m
                _emit_copy(out, base - cand, m)
                next_emit = ip
                if ip >= ip_limit:
                    break
                prev_hash = ((_u32(frag, ip - 1) * K_MUL) & 0xFFFFFFFF) >> shift
                table[prev_hash] = ip - 1
                cur = _u32(frag, ip)
                cur_hash = ((cur * K_MUL) & 0xFFFFFFFF) >> shift
                cand = table[cur_hash]
                table[cur_hash] = ip
                if cur != _u32(frag, cand):
                    break
            if ip >= ip_limit:
                break
            next_hash = ((_u32(frag, ip + 1) * K_MUL) & 0xFFFFFFFF) >> shift
            ip += 1
    if next_emit < n:
        _emit_literal(out, frag[next_emit:])


def compress(data: bytes) -> bytes:
    """snappy::RawCompress (1.1.8)."""
    data = bytes(data)
    out = bytearray(_varint32(len(data)))
    for s in range(0, len(data), K_BLOCK):
        _compress_fragment(data[s: s + K_BLOCK], out)
    return bytes(out)


def uncompressed_length(src: bytes) -> Optional[int]:
    """snappy::GetUncompressedLength: the varint32 preamble, or None."""
    v, shift = 0, 0
    for i in range(min(5, len(src))):
        b = src[i]
        v |= (b & 127) << shift
        if b < 128:
            return v if v < (1 << 32) else None
        shift += 7
    return None


def _preamble_len(src: bytes) -> int:
    i = 0
    while src[i] >= 128:
        i += 1
    return i + 1


def uncompress(src: bytes) -> Tuple[int, bytes]:
    """snappy::RawUncompress behind ReadBlock (format.cc:120-135):
    (OK, data), (BAD_LENGTH, b"") when GetUncompressedLength fails,
    (BAD_CONTENTS, b"") when the elements are malformed or do not produce
    exactly that many bytes."""
    src = bytes(src)
    n = uncompressed_length(src)
    if n is None:
        return BAD_LENGTH, b""
    i = _preamble_len(src)
    out = bytearray()
    while i < len(src):
        tag = src[i]
        i += 1
        kind = tag & 3
        if kind == 0:
            ln = (tag >> 2) + 1
            if ln > 60:
                k = ln - 60
                if i + k > len(src):
                    return BAD_CONTENTS, b""
                # snappy adds the 1 in uint32 (0xffffffff wraps to 0)
                ln = (int.from_bytes(src[i: i + k], "little") + 1) & 0xFFFFFFFF
                i += k
            if i + ln > len(src) or len(out) + ln > n:
                return BAD_CONTENTS, b""
            out += src[i: i + ln]
            i += ln
            continue
        if kind == 1:
            if i + 1 > len(src):
                return BAD_CONTENTS, b""
            ln = ((tag >> 2) & 7) + 4
            off = ((tag >> 5) << 8) | src[i]
            i += 1
        elif kind == 2:
            if i + 2 > len(src):
                return BAD_CONTENTS, b""
            ln = (tag >> 2) + 1
            off = src[i] | (src[i + 1] << 8)
            i += 2
        else:
            if i + 4 > len(src):
                return BAD_CONTENTS, b""
            ln = (tag >> 2) + 1
            off = _u32(src, i)
            i += 4
        if off == 0 or off > len(out) or len(out) + ln > n:
            return BAD_CONTENTS, b""
        for _ in range(ln):
            out.append(out[-off])
    if len(out) != n:
        return BAD_CONTENTS, b""
    return OK, bytes(out)


# ---- the block writer / reader around the codec -------------------------

def _crc():
    """The CRC32C restatement (oracle/oracle.py, pinned to util/crc32c.cc)."""
    import importlib.util
    from pathlib import Path
    spec = importlib.util.spec_from_file_location("lvkv_crc_oracle", Path(__file__).with_name("oracle.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def write_blocks(raws, compression: int, file_offset: int = 0, zstd_level: int = 1):
    """TableBuilder::WriteBlock + WriteRawBlock (table/table_builder.cc:141-209)
    for each raw block in order: (file bytes from file_offset, handles
    [(offset, size)], types). Compression 2 is kZstdCompression through
    oracle/zstd_encoder.py (port::Zstd_Compress at zstd_level, :172-185)."""
    crc = _crc()
    out = bytearray()
    handles, types = [], []
    for raw in raws:
        raw = bytes(raw)
        contents, typ = raw, 0
        if compression == 1:
            c = compress(raw)
            if len(c) < len(raw) - len(raw) // 8:  # :160-168
                contents, typ = c, 1
        elif compression == 2:
            try:
                from oracle import zstd_encoder as ze
            except ImportError:  # (oracle/ itself on sys.path)
                import zstd_encoder as ze
            c = ze.compress(raw, zstd_level)
            if len(c) < len(raw) - len(raw) // 8:  # :172-185
                contents, typ = c, 2
        handles.append((file_offset + len(out), len(contents)))
        types.append(typ)
        out += contents
        out.append(typ)
        v = crc.extend(crc.value(contents), bytes([typ]))
        out += crc.mask(v).to_bytes(4, "little")
    return bytes(out), handles, types


READ_OK, READ_CHECKSUM, READ_BAD_TYPE, READ_SNAPPY_LENGTH, READ_SNAPPY_CONTENTS, \
    READ_ZSTD_LENGTH, READ_CAPACITY, READ_TOO_LARGE, READ_ZSTD_CONTENTS = range(9)


def read_block(img: bytes, off: int, size: int, verify: bool = True):
    """ReadBlock (table/format.cc:69-162) of handle (off, size) in a file
    image: (READ_*, contents)."""
    crc = _crc()
    data = img[off: off + size + 5]
    if verify:
        stored = crc.unmask(int.from_bytes(data[size + 1: size + 5], "little"))
        if crc.value(data[: size + 1]) != stored:
            return READ_CHECKSUM, b""
    t = data[size]
    if t == 0:
        return READ_OK, data[:size]
    if t == 1:
        if uncompressed_length(data[:size]) is None:
            return READ_SNAPPY_LENGTH, b""
        st, out = uncompress(data[:size])
        return (READ_OK, out) if st == OK else (READ_SNAPPY_CONTENTS, b"")
    if t == 2:  # (:138-155) through the zstd restatement beside this one
        import importlib.util
        from pathlib import Path
        spec = importlib.util.spec_from_file_location(
            "lvkv_zstd_oracle", Path(__file__).with_name("zstd_oracle.py"))
        zo = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(zo)
        if zo.get_uncompressed_length(data[:size]) is None:
            return READ_ZSTD_LENGTH, b""
        ok, out = zo.uncompress(data[:size])
        if ok is None:
            return READ_CAPACITY, b""
        return (READ_OK, out) if ok else (READ_ZSTD_CONTENTS, b"")
    return READ_BAD_TYPE, b""


# ---- the system library itself (the pin), where the image has it --------

_LIB_PATHS = ("/opt/conda/lib/libsnappy.so.1.1.8", "/opt/conda/lib/libsnappy.so.1")


def system_snappy():
    """ctypes handle of libsnappy 1.1.8 (snappy-c API), or None."""
    import ctypes
    import os
    for p in _LIB_PATHS:
        if os.path.exists(p):
            try:
                lib = ctypes.CDLL(p)
            except OSError:
                continue
            lib.snappy_max_compressed_length.restype = ctypes.c_size_t
            lib.snappy_max_compressed_length.argtypes = [ctypes.c_size_t]
            lib.snappy_compress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                            ctypes.POINTER(ctypes.c_size_t)]
            lib.snappy_uncompress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                              ctypes.POINTER(ctypes.c_size_t)]
            lib.snappy_uncompressed_length.argtypes = [ctypes.c_char_p, ctypes.c_size_t,
                                                       ctypes.POINTER(ctypes.c_size_t)]
            return lib
    return None


def lib_compress(lib, data: bytes) -> bytes:
    import ctypes
    n = lib.snappy_max_compressed_length(len(data))
    out = ctypes.create_string_buffer(max(n, 1))
    ol = ctypes.c_size_t(n)
    assert lib.snappy_compress(data, len(data), out, ctypes.byref(ol)) == 0
    return out.raw[: ol.value]


def lib_uncompress(lib, src: bytes) -> Tuple[int, bytes]:
    import ctypes
    ul = ctypes.c_size_t(0)
    if lib.snappy_uncompressed_length(src, len(src), ctypes.byref(ul)) != 0:
        return BAD_LENGTH, b""
    out = ctypes.create_string_buffer(max(ul.value, 1))
    ol = ctypes.c_size_t(ul.value)
    if lib.snappy_uncompress(src, len(src), out, ctypes.byref(ol)) != 0:
        return BAD_CONTENTS, b""
    return OK, out.raw[: ol.value]
