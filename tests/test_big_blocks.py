"""Codec blocks of any size on the device (§8(f) row 4; VERDICT r5 missing
#2): ReadBlock decodes a block whatever its size (table/format.cc:120-155;
block_size is a user option, include/leveldb/options.h:101), so a block
past the decoders' LDS staging is decoded straight into the HBM output, and
so is a stream longer than MaxCompressedLength (padded elements no encoder
writes, but RawUncompress accepts).

Fixtures: tests/golden/gen_big.py (libsnappy 1.1.8; libzstd 1.4.9 through
port::Zstd_Compress at level 1, and ZSTD_compress at level 3), inputs
rebuilt from db_bench's generator and pinned by sha256.
"""
from __future__ import annotations

import hashlib
import json

import numpy as np
import pytest

import snappy_oracle as so
import zstd_oracle as zo
from conftest import GOLDEN


def _split(blob: bytes, lengths):
    out, p = [], 0
    for n in lengths:
        out.append(blob[p:p + n])
        p += n
    assert p == len(blob)
    return out


@pytest.fixture(scope="module")
def big():
    import sys
    sys.path.insert(0, str(GOLDEN))
    import gen_big
    spec = json.loads((GOLDEN / "big.json").read_text())
    ins = gen_big.inputs()
    assert [hashlib.sha256(x).hexdigest() for x in ins] == spec["sha256_inputs"]
    snap = _split((GOLDEN / "big_snappy.bin").read_bytes(), spec["snappy"])
    zst = _split((GOLDEN / "big_zstd.bin").read_bytes(), spec["zstd"])
    return ins, snap, zst


def _padded_snappy(data: bytes) -> bytes:
    """A stream of one-byte literals each with a 4-byte length field: valid
    for RawUncompress, ~6x the input, past MaxCompressedLength."""
    out = bytearray(so._varint32(len(data)))
    for b in data:
        out += bytes([63 << 2, 0, 0, 0, 0, b])
    return bytes(out)


def test_oracles_decode_big_fixtures(big):
    ins, snap, zst = big
    for x, s in zip(ins, snap):
        assert so.uncompress(s) == (so.OK, x)
    for k, z in enumerate(zst):
        x = ins[k // 2]
        assert zo.decompress(z, len(x)) == x
    p = _padded_snappy(ins[0][:3000])
    assert len(p) > so.max_compressed_length(3000)
    assert so.uncompress(p) == (so.OK, ins[0][:3000])
    lib = so.system_snappy()
    if lib is not None:  # the library's verdict on the padded stream
        assert so.lib_uncompress(lib, p) == (so.OK, ins[0][:3000])


def _pack(torch, dev, blobs, skew=0):
    offs, p = [], skew
    for b in blobs:
        offs.append(p)
        p += len(b) + 3
    buf = np.zeros(max(1, p), dtype=np.uint8)
    for o, b in zip(offs, blobs):
        buf[o:o + len(b)] = np.frombuffer(b, dtype=np.uint8)
    return (torch.from_numpy(buf).to(dev), torch.tensor(offs, dtype=torch.int64, device=dev),
            torch.tensor([len(b) for b in blobs], dtype=torch.int32, device=dev))


def _outbuf(torch, dev, sizes):
    off = np.zeros(len(sizes), dtype=np.int64)
    off[1:] = np.cumsum(sizes[:-1])
    return (torch.empty(max(1, int(sum(sizes))), dtype=torch.uint8, device=dev),
            torch.from_numpy(off).to(dev), torch.tensor(sizes, dtype=torch.int32, device=dev))


@pytest.mark.gpu
@pytest.mark.parametrize("max_ulen", [4096, 49152])
def test_device_snappy_decodes_big_blocks(lvkv, gpu, big, max_ulen):
    import torch
    ins, snap, _ = big
    pad = [_padded_snappy(ins[0][:3000]), _padded_snappy(ins[1][:40000])]
    streams = snap + pad
    want = ins + [ins[0][:3000], ins[1][:40000]]
    src, off, ln = _pack(torch, gpu, streams, skew=1)
    dst, doff, cap = _outbuf(torch, gpu, [len(x) for x in want])
    _, _, olen, st = lvkv.snappy_uncompress(src, off, ln, max_ulen=max_ulen, dst=dst,
                                            dst_offsets=doff, dst_caps=cap)
    torch.cuda.synchronize()
    assert st.cpu().tolist() == [lvkv.SNAPPY_OK] * len(streams)
    assert olen.cpu().tolist() == [len(x) for x in want]
    d = dst.cpu().numpy()
    for x, o in zip(want, doff.cpu().tolist()):
        assert d[o:o + len(x)].tobytes() == x
    # damaged big streams get the oracle's verdicts (a byte changed, a cut)
    rng = np.random.default_rng(8)
    dam = []
    for s in snap[:4]:
        b = bytearray(s)
        b[int(rng.integers(len(b) // 2, len(b)))] ^= 0x5A
        dam.append(bytes(b))
        dam.append(s[:len(s) - 100])
    src, off, ln = _pack(torch, gpu, dam)
    sizes = [so.uncompressed_length(x) or 0 for x in dam]
    dst, doff, cap = _outbuf(torch, gpu, sizes)
    _, _, olen, st = lvkv.snappy_uncompress(src, off, ln, max_ulen=max_ulen, dst=dst,
                                            dst_offsets=doff, dst_caps=cap)
    torch.cuda.synchronize()
    d = dst.cpu().numpy()
    for k, (x, o) in enumerate(zip(dam, doff.cpu().tolist())):
        ost, out = so.uncompress(x)
        assert st[k].item() == ost, k
        if ost == so.OK:
            assert d[o:o + len(out)].tobytes() == out


@pytest.mark.gpu
def test_device_read_blocks_big_snappy_blocks(lvkv, gpu, big):
    """ReadBlock over an image of big snappy blocks (library streams) and
    raw ones: every block reads back, with max_ulen far below their size."""
    import torch
    ins, snap, _ = big
    crc = so._crc()
    img = bytearray()
    handles, raws = [], []
    for x, s in list(zip(ins, snap))[:6]:
        for contents, t in ((s, 1), (x[:70000], 0)):
            handles.append((len(img), len(contents)))
            raws.append(x if t == 1 else x[:70000])
            img += contents + bytes([t])
            img += crc.mask(crc.extend(crc.value(contents), bytes([t]))).to_bytes(4, "little")
    file = torch.from_numpy(np.frombuffer(bytes(img), dtype=np.uint8).copy()).to(gpu)
    ho = torch.tensor([h[0] for h in handles], dtype=torch.int64, device=gpu)
    hs = torch.tensor([h[1] for h in handles], dtype=torch.int32, device=gpu)
    out, ooff, cap = _outbuf(torch, gpu, [len(r) for r in raws])
    for verify in (True, False):
        _, _, olen, st = lvkv.sst_read_blocks(file, ho, hs, max_ulen=8192, verify=verify,
                                              out=out, out_offsets=ooff, out_caps=cap)
        torch.cuda.synchronize()
        assert st.cpu().tolist() == [lvkv.READ_OK] * len(raws)
        d = out.cpu().numpy()
        for r, o in zip(raws, ooff.cpu().tolist()):
            assert d[o:o + len(r)].tobytes() == r


def _with_checksum(f: bytes, x: bytes) -> bytes:
    """Frame f with its checksum flag set and XXH64(x)'s low 32 bits after
    its last block (the library's ZSTD_c_checksumFlag frame)."""
    import xxhash
    b = bytearray(f)
    b[4] |= 4
    return bytes(b) + (xxhash.xxh64(x, seed=0).intdigest() & 0xFFFFFFFF).to_bytes(4, "little")


def _zstd_cases(ins, zst):
    """(stream, expected output or None): the library's big frames, checksummed
    copies, a skippable frame before one, two frames in one stream (the
    second overflows the first's content size), and damaged copies."""
    want = [ins[k // 2] for k in range(len(zst))]
    cases = list(zip(zst, want))
    for k in (0, 8, 12, 13, 16):  # 64 KiB, 256 KiB, 1 MiB (levels 1, 3), 300,000
        cases.append((_with_checksum(zst[k], want[k]), want[k]))
    # (a stream that opens with a skippable frame has no length: BAD_LENGTH)
    cases.append((b"\x50\x2a\x4d\x18" + (5).to_bytes(4, "little") + b"skip!" + zst[12], None))
    cases.append((zst[8] + zst[2], None))
    rng = np.random.default_rng(9)
    for k in (0, 8, 12, 13, 16):
        b = bytearray(zst[k])
        b[int(rng.integers(len(b) // 2, len(b)))] ^= 0x21
        cases.append((bytes(b), None))
        cases.append((zst[k][:len(zst[k]) - 100], None))
        c = bytearray(_with_checksum(zst[k], want[k]))
        c[-1] ^= 1
        cases.append((bytes(c), None))
    return cases


@pytest.fixture(scope="module")
def zcases(big):
    """_zstd_cases with the oracle's verdict on each: (stream, want, ok, out)."""
    ins, _, zst = big
    return [(f, x) + tuple(zo.uncompress(f)) for f, x in _zstd_cases(ins, zst)]


def test_oracle_big_zstd_cases(zcases):
    bad = 0
    for f, x, ok, out in zcases:
        if x is not None:
            assert ok and out == x
        else:
            bad += not ok
    assert bad >= 10  # (a changed byte can land where it changes nothing checked)


@pytest.mark.gpu
@pytest.mark.parametrize("max_ulen", [4096, 49152])
def test_device_zstd_decodes_big_frames(lvkv, gpu, zcases, max_ulen):
    """Frames of 64 KiB - 1 MiB (one to eight 128 KiB blocks) through the
    HBM-output kernel, checksums included; damaged ones get the oracle's
    verdict."""
    import torch
    streams = [c[0] for c in zcases]
    sizes = [zo.get_uncompressed_length(f) or 0 for f in streams]
    src, off, ln = _pack(torch, gpu, streams, skew=3)
    dst, doff, cap = _outbuf(torch, gpu, sizes)
    _, _, olen, st, why = lvkv.zstd_uncompress(src, off, ln, max_ulen=max_ulen, dst=dst,
                                               dst_offsets=doff, dst_caps=cap, detail=True)
    torch.cuda.synchronize()
    st, why, olen = st.cpu().tolist(), why.cpu().tolist(), olen.cpu().tolist()
    d = dst.cpu().numpy()
    for k, ((f, _, ok, out), o) in enumerate(zip(zcases, doff.cpu().tolist())):
        if zo.get_uncompressed_length(f) is None:
            want = lvkv.SNAPPY_BAD_LENGTH
        else:
            want = lvkv.SNAPPY_OK if ok else lvkv.SNAPPY_BAD_CONTENTS
        assert st[k] == want, (k, len(f), st[k], want, why[k])
        if ok:
            assert olen[k] == len(out)
            assert d[o:o + len(out)].tobytes() == out, k


@pytest.mark.gpu
def test_device_read_blocks_big_zstd_blocks(lvkv, gpu, big):
    """ReadBlock over an image of big zstd blocks (library frames) between
    small snappy and raw ones: every block reads back at max_ulen 8192."""
    import torch
    ins, snap, zst = big
    crc = so._crc()
    img = bytearray()
    handles, raws = [], []

    def put(contents, t, raw):
        handles.append((len(img), len(contents)))
        raws.append(raw)
        img.extend(contents + bytes([t]))
        img.extend(crc.mask(crc.extend(crc.value(contents), bytes([t]))).to_bytes(4, "little"))

    small = ins[0][:3000]
    for k, z in enumerate(zst):
        put(z, 2, ins[k // 2])
        put(so.compress(small), 1, small)
        put(small, 0, small)
    file = torch.from_numpy(np.frombuffer(bytes(img), dtype=np.uint8).copy()).to(gpu)
    ho = torch.tensor([h[0] for h in handles], dtype=torch.int64, device=gpu)
    hs = torch.tensor([h[1] for h in handles], dtype=torch.int32, device=gpu)
    out, ooff, cap = _outbuf(torch, gpu, [len(r) for r in raws])
    for verify in (True, False):
        _, _, olen, st = lvkv.sst_read_blocks(file, ho, hs, max_ulen=8192, verify=verify,
                                              out=out, out_offsets=ooff, out_caps=cap)
        torch.cuda.synchronize()
        assert st.cpu().tolist() == [lvkv.READ_OK] * len(raws)
        d = out.cpu().numpy()
        for r, o in zip(raws, ooff.cpu().tolist()):
            assert d[o:o + len(r)].tobytes() == r
