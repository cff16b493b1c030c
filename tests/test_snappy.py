"""§8(f) row 4: the Snappy block codec LevelDB wraps around the block CRC
(port::Snappy_* , port/port_stdcxx.h:90-133; TableBuilder::WriteBlock,
table/table_builder.cc:158-168; ReadBlock, table/format.cc:120-135).

Pins: the oracle (oracle/snappy_oracle.py) is checked byte-for-byte against
the fixtures libsnappy 1.1.8 wrote (tests/golden/gen_snappy.py) and, where
the library is present, against the library itself on fuzzed inputs. The
device codec is then checked against the fixtures and the library/oracle:
compressed bytes identical, decoded bytes identical, every damaged stream
given the library's verdict.
"""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

import snappy_oracle as so
from conftest import GOLDEN


def _split(blob: bytes, lengths):
    out, p = [], 0
    for n in lengths:
        out.append(blob[p:p + n])
        p += n
    assert p == len(blob)
    return out


@pytest.fixture(scope="module")
def fx():
    import json
    spec = json.loads((GOLDEN / "snappy.json").read_text())
    ins = _split((GOLDEN / "snappy_inputs.bin").read_bytes(), spec["inputs"])
    streams = _split((GOLDEN / "snappy_streams.bin").read_bytes(), spec["streams"])
    dam = _split((GOLDEN / "snappy_damaged.bin").read_bytes(), spec["damaged"])
    for x, h in zip(ins, spec["sha256_inputs"]):
        assert hashlib.sha256(x).hexdigest() == h
    return ins, streams, dam, spec["verdicts"]


# ---- the oracle against the library's fixtures (CPU) -----------------------

def test_oracle_compress_matches_fixtures(fx):
    ins, streams, _, _ = fx
    bad = [i for i, (x, s) in enumerate(zip(ins, streams)) if so.compress(x) != s]
    assert not bad, f"oracle differs from libsnappy 1.1.8 on inputs {bad}"


def test_oracle_uncompress_roundtrips_fixtures(fx):
    ins, streams, _, _ = fx
    for x, s in zip(ins, streams):
        assert so.uncompressed_length(s) == len(x)
        assert so.uncompress(s) == (so.OK, x)


def test_oracle_damaged_verdicts_match_fixtures(fx):
    _, _, dam, verdicts = fx
    assert {v["status"] for v in verdicts} == {0, 1, 2}
    for d, v in zip(dam, verdicts):
        st, out = so.uncompress(d)
        assert st == v["status"], d[:16].hex()
        if st == so.OK:
            assert hashlib.sha256(out).hexdigest() == v["sha256"]


def test_oracle_matches_library_on_fuzz():
    lib = so.system_snappy()
    if lib is None:
        pytest.skip("libsnappy 1.1.8 not present")
    rng = np.random.default_rng(5)
    for k in range(120):
        n = int(rng.integers(0, 3000))
        alpha = int(rng.integers(1, 257))
        x = rng.integers(0, alpha, n, dtype=np.uint16).astype(np.uint8).tobytes()
        s = so.lib_compress(lib, x)
        assert so.compress(x) == s
        d = bytearray(s)
        if d:
            d[int(rng.integers(0, len(d)))] ^= 0x20
        assert so.uncompress(bytes(d))[0] == so.lib_uncompress(lib, bytes(d))[0]


def test_max_compressed_length(lvkv):
    for n in (0, 1, 6, 4096, 65536, 1 << 20):
        assert lvkv.snappy_max_compressed_length(n) == so.max_compressed_length(n) == 32 + n + n // 6


def test_db_bench_generator_is_compressible():
    from tools.db_bench_data import block_batch, Random
    r = Random(301)
    M = 2 ** 31 - 1  # Park-Miller: 301 * 16807^k mod (2^31 - 1)
    assert [r.next() for _ in range(3)] == [301 * pow(16807, k, M) % M for k in (1, 2, 3)]
    b = block_batch(4).tobytes()
    ratio = len(so.compress(b[:4096])) / 4096
    assert 0.45 < ratio < 0.65  # compression_ratio 0.5 (db_bench.cc:189)


# ---- the device codec (GPU) ------------------------------------------------

def _pack(torch, dev, blobs, align=1, skew=0):
    offs, p = [], skew
    for b in blobs:
        offs.append(p)
        p += len(b) + (-(len(b)) % align)
    buf = np.zeros(max(1, p), dtype=np.uint8)
    for o, b in zip(offs, blobs):
        buf[o:o + len(b)] = np.frombuffer(b, dtype=np.uint8)
    return (torch.from_numpy(buf).to(dev), torch.tensor(offs, dtype=torch.int64, device=dev),
            torch.tensor([len(b) for b in blobs], dtype=torch.int32, device=dev))


def _unpack(dst, offs, lens):
    d = dst.cpu().numpy()
    return [d[o:o + n].tobytes() for o, n in zip(offs.cpu().tolist(), lens.cpu().tolist())]


@pytest.mark.gpu
@pytest.mark.parametrize("skew", [0, 3])
def test_device_compress_matches_fixtures(lvkv, gpu, fx, skew):
    import torch
    ins, streams, _, _ = fx
    src, off, ln = _pack(torch, gpu, ins, skew=skew)
    dst, doff, dlen, st = lvkv.snappy_compress(src, off, ln)
    torch.cuda.synchronize()
    assert st.cpu().tolist() == [0] * len(ins)
    got = _unpack(dst, doff, dlen)
    bad = [i for i, (g, s) in enumerate(zip(got, streams)) if g != s]
    assert not bad, f"device stream differs from libsnappy on inputs {bad}"


@pytest.mark.gpu
def test_device_compress_small_max_len_reports_too_large(lvkv, gpu, fx):
    import torch
    ins, streams, _, _ = fx
    src, off, ln = _pack(torch, gpu, ins)
    dst, doff, dlen, st = lvkv.snappy_compress(src, off, ln, max_len=4096)
    torch.cuda.synchronize()
    st = st.cpu().tolist()
    got = _unpack(dst, doff, dlen)
    for x, s, g, t in zip(ins, streams, got, st):
        if len(x) > 4096:
            assert t == lvkv.SNAPPY_TOO_LARGE
        else:
            assert t == 0 and g == s


@pytest.mark.gpu
def test_device_uncompress_matches_fixtures(lvkv, gpu, fx):
    import torch
    ins, streams, _, _ = fx
    src, off, ln = _pack(torch, gpu, streams, skew=1)
    cap = lvkv.SNAPPY_MAX_BLOCK
    dst, doff, dlen, st = lvkv.snappy_uncompress(src, off, ln, max_ulen=cap)
    ul, ust = lvkv.snappy_uncompressed_length(src, off, ln)
    torch.cuda.synchronize()
    st = st.cpu().tolist()
    assert ust.cpu().tolist() == [0] * len(ins)
    assert ul.cpu().tolist() == [len(x) for x in ins]
    got = _unpack(dst, doff, dlen)
    for x, g, t in zip(ins, got, st):
        if len(x) > cap:
            assert t == lvkv.SNAPPY_CAPACITY
        else:
            assert t == 0 and g == x


def _expected_device_verdict(lvkv, d, v, cap):
    if v["status"] == so.BAD_LENGTH:
        return so.BAD_LENGTH
    ulen = so.uncompressed_length(d)
    if ulen > cap:
        return lvkv.SNAPPY_CAPACITY
    # (a stream past the LDS staging is decoded by the HBM-output kernel)
    return v["status"]


@pytest.mark.gpu
@pytest.mark.parametrize("cap", [4096, 49152])
def test_device_uncompress_damaged_verdicts(lvkv, gpu, fx, cap):
    import torch
    _, _, dam, verdicts = fx
    src, off, ln = _pack(torch, gpu, dam)
    dst, doff, dlen, st = lvkv.snappy_uncompress(src, off, ln, max_ulen=cap)
    ul, ust = lvkv.snappy_uncompressed_length(src, off, ln)
    torch.cuda.synchronize()
    st, ust, ul = st.cpu().tolist(), ust.cpu().tolist(), ul.cpu().tolist()
    got = _unpack(dst, doff, dlen)
    for i, (d, v) in enumerate(zip(dam, verdicts)):
        exp = _expected_device_verdict(lvkv, d, v, cap)
        assert st[i] == exp, (i, d[:12].hex(), st[i], exp)
        assert ust[i] == (so.BAD_LENGTH if v["status"] == so.BAD_LENGTH else 0)
        if ust[i] == 0:
            assert ul[i] & 0xFFFFFFFF == so.uncompressed_length(d)
        if exp == 0:
            assert hashlib.sha256(got[i]).hexdigest() == v["sha256"]


@pytest.mark.gpu
def test_device_codec_ragged_batch_against_library(lvkv, gpu):
    """Thousands of blocks of ragged lengths and kinds, unaligned offsets:
    device compress == libsnappy (or the oracle on a sample without it),
    device uncompress == the inputs."""
    import torch
    rng = np.random.default_rng(11)
    from tools.db_bench_data import block_batch
    bench = block_batch(256).tobytes()
    blobs = []
    for k in range(3000):
        kind = k % 4
        n = int(rng.integers(0, 9000))
        if kind == 0:
            s = int(rng.integers(0, len(bench) - n))
            blobs.append(bench[s:s + n])
        elif kind == 1:
            blobs.append(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        elif kind == 2:
            blobs.append(rng.integers(0, 3, n, dtype=np.uint8).tobytes())
        else:
            blobs.append((rng.integers(0, 256, int(rng.integers(1, 300)), dtype=np.uint8)
                          .tobytes() * 40)[:n])
    lib = so.system_snappy()
    check = range(len(blobs)) if lib is not None else range(0, len(blobs), 25)
    src, off, ln = _pack(torch, gpu, blobs, skew=5)
    dst, doff, dlen, st = lvkv.snappy_compress(src, off, ln, max_len=9000)
    torch.cuda.synchronize()
    assert st.cpu().tolist() == [0] * len(blobs)
    got = _unpack(dst, doff, dlen)
    for i in check:
        want = so.lib_compress(lib, blobs[i]) if lib is not None else so.compress(blobs[i])
        assert got[i] == want, i
    # and back, from the device's own streams where they lie
    out, ooff, olen, ost = lvkv.snappy_uncompress(dst, doff, dlen.clone(), max_ulen=9000)
    torch.cuda.synchronize()
    assert ost.cpu().tolist() == [0] * len(blobs)
    assert _unpack(out, ooff, olen) == blobs


@pytest.mark.gpu
def test_device_codec_empty_batch(lvkv, gpu):
    import torch
    z8 = torch.zeros(1, dtype=torch.uint8, device=gpu)
    e64 = torch.zeros(0, dtype=torch.int64, device=gpu)
    e32 = torch.zeros(0, dtype=torch.int32, device=gpu)
    _, _, dl, st = lvkv.snappy_compress(z8, e64, e32, max_len=0)
    assert dl.numel() == 0 and st.numel() == 0
    _, _, dl, st = lvkv.snappy_uncompress(z8, e64, e32, max_ulen=4096)
    assert dl.numel() == 0 and st.numel() == 0
    for comp in (0, 1):  # no blocks: Rep::offset stays where it was
        _, _, _, _, end = lvkv.sst_write_blocks(z8, e64, e32, compression=comp,
                                                file_offset=987654321)
        torch.cuda.synchronize()
        assert int(end.item()) == 987654321


# ---- WriteBlock / ReadBlock around the codec -------------------------------

def _block_set(n=300, seed=3):
    from tools.db_bench_data import block_batch
    rng = np.random.default_rng(seed)
    bench = block_batch(64).tobytes()
    out = []
    for k in range(n):
        L = int(rng.integers(0, 6000))
        kind = k % 3
        if kind == 0:
            s = int(rng.integers(0, len(bench) - L))
            out.append(bench[s:s + L])
        elif kind == 1:
            out.append(rng.integers(0, 256, L, dtype=np.uint8).tobytes())
        else:  # barely compressible: around the 12.5% rule
            a = rng.integers(0, 256, L, dtype=np.uint8)
            a[: L // 7] = 7
            out.append(a.tobytes())
    return out


def test_oracle_write_then_read_blocks():
    raws = _block_set(60)
    img, handles, types = so.write_blocks(raws, 1, file_offset=0)
    assert 1 in types and 0 in types
    for raw, (off, size), t in zip(raws, handles, types):
        assert so.read_block(img, off, size) == (so.READ_OK, raw)
        assert img[off + size] == t
    off, size = handles[0]
    bad = bytearray(img)
    bad[off] ^= 1
    assert so.read_block(bytes(bad), off, size)[0] == so.READ_CHECKSUM


@pytest.mark.gpu
@pytest.mark.parametrize("compression,file_offset", [(1, 0), (1, 1234567), (0, 17)])
def test_device_write_blocks_matches_oracle(lvkv, gpu, compression, file_offset):
    import torch
    raws = _block_set()
    src, off, ln = _pack(torch, gpu, raws, skew=1)
    file, hoff, hsize, typ, end = lvkv.sst_write_blocks(src, off, ln, compression=compression,
                                                        file_offset=file_offset)
    torch.cuda.synchronize()
    img, handles, types = so.write_blocks(raws, compression, file_offset)
    assert hoff.cpu().tolist() == [h[0] for h in handles]
    assert hsize.cpu().tolist() == [h[1] for h in handles]
    assert typ.cpu().tolist() == types
    assert int(end.item()) == file_offset + len(img)
    got = file.cpu().numpy()[file_offset:file_offset + len(img)].tobytes()
    assert got == img


@pytest.mark.gpu
def test_device_write_blocks_longer_than_max_len_stay_raw(lvkv, gpu):
    """A block longer than the call's max_len (here >= 64 KiB, so the LDS
    would take it) must not run past its fixed-stride scratch slot: it is
    TOO_LARGE for the compressor and the layout keeps it raw.
    Every block still reads back to its bytes."""
    import torch
    from tools.db_bench_data import block_batch
    bench = block_batch(40).tobytes()
    raws = [bench[:5000], bench[7:7 + 70000], bench[100:4196], bench[:65536]]
    src, off, ln = _pack(torch, gpu, raws, skew=1)
    file, hoff, hsize, typ, end = lvkv.sst_write_blocks(src, off, ln, compression=1,
                                                        max_len=65536)
    torch.cuda.synchronize()
    types = typ.cpu().tolist()
    assert types[1] == 0 and types[0] == types[2] == types[3] == 1
    img = file.cpu().numpy().tobytes()
    for raw, o, s in zip(raws, hoff.cpu().tolist(), hsize.cpu().tolist()):
        assert so.read_block(img, o, s) == (so.READ_OK, raw)
    assert int(end.item()) == sum(hsize.cpu().tolist()) + 5 * len(raws)


@pytest.mark.gpu
def test_device_read_blocks_roundtrip_and_verdicts(lvkv, gpu):
    import torch
    raws = _block_set(200, seed=9)
    img, handles, types = so.write_blocks(raws, 1)
    buf = bytearray(img)
    rng = np.random.default_rng(4)
    hurt = {}
    for i in rng.choice(len(raws), 40, replace=False).tolist():
        off, size = handles[i]
        kind = len(hurt) % 4
        if kind == 0 and size:  # contents flipped: checksum mismatch
            buf[off + int(rng.integers(0, size))] ^= 0x10
        elif kind == 1:  # type 2 (zstd) or 9 (bad), CRC refilled to match
            buf[off + size] = 2 if i % 2 else 9
        elif kind == 2 and size:  # snappy bytes damaged, CRC refilled
            buf[off + int(rng.integers(0, min(size, 8)))] ^= 0x80
        else:  # trailer damaged
            buf[off + size + 2] ^= 1
        hurt[i] = kind
    crc = so._crc()
    for i, kind in hurt.items():
        if kind in (1, 2):
            off, size = handles[i]
            v = crc.mask(crc.value(bytes(buf[off:off + size + 1])))
            buf[off + size + 1: off + size + 5] = v.to_bytes(4, "little")
    img2 = bytes(buf)
    file = torch.from_numpy(np.frombuffer(img2, dtype=np.uint8).copy()).to(gpu)
    ho = torch.tensor([h[0] for h in handles], dtype=torch.int64, device=gpu)
    hs = torch.tensor([h[1] for h in handles], dtype=torch.int32, device=gpu)
    for verify in (True, False):
        out, ooff, olen, st = lvkv.sst_read_blocks(file, ho, hs, max_ulen=8192, verify=verify)
        torch.cuda.synchronize()
        st, olen = st.cpu().tolist(), olen.cpu().tolist()
        got = _unpack(out, ooff, torch.tensor(olen))
        for i, (off, size) in enumerate(handles):
            want_st, want = so.read_block(img2, off, size, verify)
            ul = so.uncompressed_length(img2[off:off + size])
            if want_st in (so.READ_OK, so.READ_SNAPPY_CONTENTS) and img2[off + size] == 1 \
                    and ul is not None and ul > 8192:
                want_st = lvkv.READ_CAPACITY  # a damaged preamble asks for more than the cap
            assert st[i] == want_st, (i, hurt.get(i), st[i], want_st)
            if want_st == so.READ_OK:
                assert got[i] == want
                if i not in hurt:
                    assert want == raws[i]


@pytest.mark.gpu
def test_device_uncompress_fuzz_against_oracle(lvkv, gpu):
    """Random byte strings and lightly-mutated valid streams, 6,000 of them:
    the device's verdict and bytes equal the oracle's (the oracle is pinned
    to libsnappy's verdicts above)."""
    import torch
    rng = np.random.default_rng(23)
    from tools.db_bench_data import block_batch
    base = [so.compress(block_batch(1, 4096, r).tobytes()) for r in (0.2, 0.5, 0.9)]
    streams = []
    for k in range(6000):
        kind = k % 3
        if kind == 0:  # random bytes behind a plausible preamble
            n = int(rng.integers(1, 300))
            body = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            streams.append(so._varint32(int(rng.integers(0, 600))) + body)
        else:  # a valid stream with 1-3 bytes changed or a cut
            s = bytearray(base[k % 3])
            for _ in range(int(rng.integers(1, 4))):
                s[int(rng.integers(0, len(s)))] = int(rng.integers(0, 256))
            if kind == 2:
                s = s[: int(rng.integers(1, len(s) + 1))]
            streams.append(bytes(s))
    src, off, ln = _pack(torch, gpu, streams, skew=2)
    cap = 4096
    dst, doff, dlen, st = lvkv.snappy_uncompress(src, off, ln, max_ulen=cap)
    torch.cuda.synchronize()
    st, dl = st.cpu().tolist(), dlen.cpu().tolist()
    got = _unpack(dst, doff, torch.tensor(dl))
    for i, s in enumerate(streams):
        ost, out = so.uncompress(s)
        ul = so.uncompressed_length(s)
        if ost != so.BAD_LENGTH and ul is not None and ul > cap:
            want = lvkv.SNAPPY_CAPACITY
        else:
            want = ost
        assert st[i] == want, (i, s[:12].hex(), st[i], want)
        if want == so.OK:
            assert got[i] == out
