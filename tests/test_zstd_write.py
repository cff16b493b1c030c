"""§8(f) row 4, the write side of kZstdCompression: TableBuilder::WriteBlock's
zstd case (table/table_builder.cc:172-185) through port::Zstd_Compress
(port/port_stdcxx.h:133-161): ZSTD_getCParams(level, max(n, 1), 0),
ZSTD_CCtx_setCParams, ZSTD_compress2, at options.zstd_compression_level
(default 1, include/leveldb/options.h:141).

Pins: the oracle (oracle/zstd_encoder.py, a restatement of libzstd 1.4.9's
fast-strategy compressor) byte for byte against the frames the library wrote
through that exact call sequence (tests/golden/gen_zstd_write.py), its
parameter table against the library's ZSTD_getCParams, and, where the library
is present, against the library on fresh fuzz. The device compressor is then
held to the fixtures and the oracle.
"""
from __future__ import annotations

import hashlib
import json

import numpy as np
import pytest

import zstd_encoder as ze
import zstd_oracle as zo
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
def wfx():
    spec = json.loads((GOLDEN / "zstd_write.json").read_text())
    ins = _split((GOLDEN / "zstd_write_inputs.bin").read_bytes(), spec["inputs"])
    frames = _split((GOLDEN / "zstd_write_frames.bin").read_bytes(), spec["frames"])
    for x, h in zip(ins, spec["sha256_inputs"]):
        assert hashlib.sha256(x).hexdigest() == h
    return ins, frames, spec["meta"], spec["cparams"]


# ---- the oracle, pinned ----------------------------------------------------

def test_oracle_matches_every_library_frame(wfx):
    ins, frames, meta, _ = wfx
    assert {lvl for _, lvl in meta} == {1, 2, -1, -5}
    bad = [(i, lvl) for f, (i, lvl) in zip(frames, meta) if ze.compress(ins[i], lvl) != f]
    assert not bad, f"oracle differs from libzstd 1.4.9 on {bad}"


def test_library_frames_decode(wfx):
    ins, frames, meta, _ = wfx
    for f, (i, lvl) in zip(frames, meta):
        assert zo.decompress(f, len(ins[i])) == ins[i]


def test_oracle_parameters_match_getcparams(wfx):
    *_, grid = wfx
    checked = 0
    for lvl, n, p in grid:
        if not ze.supported(lvl, n):
            assert lvl in (0, 3, 22) or (lvl == 2 and 131072 < n <= 262144), (lvl, n)
            continue
        assert list(ze.get_cparams(lvl, n)) == p, (lvl, n)
        checked += 1
    assert checked >= 100


def test_fixtures_reach_the_rare_paths(wfx):
    """The committed frames exercise what a 4 KiB db_bench block does not:
    RLE literals, 4-bit and FSE tree descriptions, trees cut to 11 bits,
    raw blocks, later RLE blocks, predefined / RLE / new sequence tables."""
    ins, frames, meta, _ = wfx
    kinds = set()
    for f, (i, lvl) in zip(frames, meta):
        h = zo.frame_header(f)
        q = h.size
        while True:
            bh = int.from_bytes(f[q:q + 3], "little")
            last, bt, bs = bh & 1, (bh >> 1) & 3, bh >> 3
            kinds.add(("block", bt))
            q += 3
            if bt == 2:
                lt = f[q] & 3
                kinds.add(("lit", lt))
                if lt == 2:
                    sf = (f[q] >> 2) & 3
                    hs = [3, 3, 4, 5][sf]
                    kinds.add(("tree", "fse" if f[q + hs] < 128 else "4bit"))
            q += 1 if bt == 1 else bs
            if last:
                break
    for k in [("block", 0), ("block", 1), ("block", 2), ("lit", 0), ("lit", 1), ("lit", 2),
              ("tree", "fse"), ("tree", "4bit")]:
        assert k in kinds, k


def _fuzz_inputs(rng, count, max_n):
    from tools.db_bench_data import block_batch
    bb = block_batch(64).tobytes()
    out = []
    for k in range(count):
        n = int(rng.integers(0, max_n))
        kind = k % 6
        if kind == 0:
            s = int(rng.integers(0, len(bb) - n))
            out.append(bb[s:s + n])
        elif kind == 1:
            out.append(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        elif kind == 2:
            out.append(rng.integers(0, int(rng.integers(1, 20)), n, dtype=np.uint8).tobytes())
        elif kind == 3:
            p = float(rng.uniform(0.3, 0.7))
            out.append(np.minimum(rng.geometric(p, n) - 1, 255).astype(np.uint8).tobytes())
        elif kind == 4:
            base = rng.integers(0, 256, int(rng.integers(1, 64)), dtype=np.uint8).tobytes()
            x = bytearray((base * (n // len(base) + 1))[:n])
            for _ in range(int(rng.integers(0, 20))):
                if n:
                    x[int(rng.integers(0, n))] = int(rng.integers(0, 256))
            out.append(bytes(x))
        else:
            ent = bytearray()
            i = 0
            while len(ent) < n:
                ent += bytes([0, 16, int(rng.integers(1, 100))]) + f"key{i:013d}".encode() + \
                    rng.integers(0, 256, int(rng.integers(0, 100)), dtype=np.uint8).tobytes()
                i += 1
            out.append(bytes(ent[:n]))
    return out


def test_oracle_matches_library_fuzz():
    """400 fresh inputs at levels 1, 2, -1, -3: the oracle's frame is the
    library's (skipped where libzstd 1.4.9 is absent)."""
    lib = ze.system_zstd_writer()
    if lib is None:
        pytest.skip("libzstd 1.4.9 not present")
    rng = np.random.default_rng(611)
    ins = _fuzz_inputs(rng, 400, 9000)
    for k, x in enumerate(ins):
        lvl = (1, 1, 2, -1, -3)[k % 5]
        assert ze.compress(x, lvl) == ze.lib_port_compress(lib, x, lvl), (k, lvl, len(x))


def test_oracle_write_blocks_zstd_reads_back():
    from tools.db_bench_data import block_batch
    bb = block_batch(8).tobytes()
    raws = [bb[:4096], bb[5:4105], bytes(np.random.default_rng(1).integers(0, 256, 3000,
                                                                           dtype=np.uint8)), b""]
    img, handles, types = so.write_blocks(raws, 2)
    assert types == [2, 2, 0, 0]
    for raw, (off, size) in zip(raws, handles):
        assert so.read_block(img, off, size) == (so.READ_OK, raw)


# ---- the device ------------------------------------------------------------

def _pack(torch, dev, blobs, skew=0):
    offs, p = [], skew
    for b in blobs:
        offs.append(p)
        p += len(b) + 1  # (one byte apart: every alignment)
    buf = np.zeros(max(1, p), dtype=np.uint8)
    for o, b in zip(offs, blobs):
        buf[o:o + len(b)] = np.frombuffer(b, dtype=np.uint8)
    return (torch.from_numpy(buf).to(dev), torch.tensor(offs, dtype=torch.int64, device=dev),
            torch.tensor([len(b) for b in blobs], dtype=torch.int32, device=dev))


def _unpack(dst, offs, lens):
    d = dst.cpu().numpy()
    return [d[o:o + n].tobytes() for o, n in zip(offs.cpu().tolist(), lens.cpu().tolist())]


@pytest.mark.gpu
@pytest.mark.parametrize("level", [1, 2, -1, -5])
def test_device_compress_matches_library_fixtures(lvkv, gpu, wfx, level):
    import torch
    ins, frames, meta, _ = wfx
    cap = lvkv.ZSTD_COMPRESS_MAX_BLOCK
    pick = [(i, f) for f, (i, lvl) in zip(frames, meta) if lvl == level and len(ins[i]) <= cap]
    assert len(pick) >= 50
    blobs = [ins[i] for i, _ in pick]
    src, off, ln = _pack(torch, gpu, blobs, skew=3)
    dst, doff, dlen, st = lvkv.zstd_compress(src, off, ln, level=level, max_len=cap)
    torch.cuda.synchronize()
    assert st.cpu().tolist() == [lvkv.ZSTD_OK] * len(pick)
    got = _unpack(dst, doff, dlen)
    bad = [i for (i, f), g in zip(pick, got) if g != f]
    assert not bad, f"device frame differs from libzstd on inputs {bad}"


@pytest.mark.gpu
def test_device_compress_ragged_against_oracle(lvkv, gpu):
    """3,000 blocks of 0-20 KiB at every alignment (db_bench slices, random,
    few-symbol, skewed, repeats, key/value entries): the device's frame is the
    oracle's, and it decodes back (device decoder) to the block."""
    import torch
    rng = np.random.default_rng(99)
    blobs = _fuzz_inputs(rng, 2700, 6000) + _fuzz_inputs(rng, 300, 20481)
    src, off, ln = _pack(torch, gpu, blobs, skew=1)
    dst, doff, dlen, st = lvkv.zstd_compress(src, off, ln, level=1, max_len=20480)
    torch.cuda.synchronize()
    assert st.cpu().tolist() == [lvkv.ZSTD_OK] * len(blobs)
    got = _unpack(dst, doff, dlen)
    bad = [k for k, (x, g) in enumerate(zip(blobs, got)) if g != ze.compress(x, 1)]
    assert not bad, f"device frame differs from the oracle on {bad[:20]} ({len(bad)})"
    # the device decoder reads them back
    small = [k for k, x in enumerate(blobs) if 0 < len(x) <= lvkv.ZSTD_MAX_BLOCK]
    fr = [got[k] for k in small]
    s2, o2, l2 = _pack(torch, gpu, fr)
    out, ooff, olen, st2 = lvkv.zstd_uncompress(s2, o2, l2, max_ulen=20480)
    torch.cuda.synchronize()
    assert st2.cpu().tolist() == [lvkv.ZSTD_OK] * len(small)
    back = _unpack(out, ooff, olen)
    assert all(back[j] == blobs[k] for j, k in enumerate(small))


@pytest.mark.gpu
@pytest.mark.parametrize("level", [2, -1, -5])
def test_device_compress_ragged_other_levels(lvkv, gpu, level):
    """400 blocks of 0-20 KiB at levels 2 (the fast strategy below 128 KiB)
    and -1, -5 (literal compression off): the device's frame is the oracle's
    at every one."""
    import torch
    rng = np.random.default_rng(400 + level)
    blobs = _fuzz_inputs(rng, 340, 6000) + _fuzz_inputs(rng, 60, 20481)
    src, off, ln = _pack(torch, gpu, blobs, skew=3)
    dst, doff, dlen, st = lvkv.zstd_compress(src, off, ln, level=level, max_len=20480)
    torch.cuda.synchronize()
    assert st.cpu().tolist() == [lvkv.ZSTD_OK] * len(blobs)
    got = _unpack(dst, doff, dlen)
    bad = [k for k, (x, g) in enumerate(zip(blobs, got)) if g != ze.compress(x, level)]
    assert not bad, f"level {level}: device frame differs from the oracle on {bad[:20]} ({len(bad)})"


@pytest.mark.gpu
def test_device_compress_statuses(lvkv, gpu):
    import torch
    from tools.db_bench_data import block_batch
    bb = block_batch(8).tobytes()
    blobs = [bb[:4096], bb[:5000], b"", b"abc"]
    src, off, ln = _pack(torch, gpu, blobs)
    # a block past max_len
    _, _, dl, st = lvkv.zstd_compress(src, off, ln, level=1, max_len=4096)
    torch.cuda.synchronize()
    assert st.cpu().tolist() == [lvkv.ZSTD_OK, lvkv.ZSTD_TOO_LARGE, lvkv.ZSTD_OK, lvkv.ZSTD_OK]
    # level 3 (ZSTD_dfast) and 0 (= 3) are the host library's
    for lvl in (3, 0, 19):
        _, _, dl, st = lvkv.zstd_compress(src, off, ln, level=lvl, max_len=5000)
        torch.cuda.synchronize()
        assert set(st.cpu().tolist()) == {lvkv.ZSTD_UNSUPPORTED}
    # the empty and tiny frames
    dst, doff, dl, st = lvkv.zstd_compress(src, off, ln, level=1, max_len=5000)
    torch.cuda.synchronize()
    got = _unpack(dst, doff, dl)
    assert got[2] == ze.compress(b"", 1) and got[3] == ze.compress(b"abc", 1)
    with pytest.raises(RuntimeError):
        lvkv.zstd_compress(src, off, ln, level=1, max_len=lvkv.ZSTD_COMPRESS_MAX_BLOCK + 1)


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
        else:  # around the 12.5% rule
            a = rng.integers(0, 256, L, dtype=np.uint8)
            a[: L // 7] = 7
            out.append(a.tobytes())
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("level,file_offset", [(1, 0), (1, 777), (-1, 5), (2, 0)])
def test_device_write_blocks_zstd_matches_oracle(lvkv, gpu, level, file_offset):
    import torch
    raws = _block_set()
    src, off, ln = _pack(torch, gpu, raws, skew=1)
    file, hoff, hsize, typ, end = lvkv.sst_write_blocks(src, off, ln, compression=2,
                                                        zstd_level=level, file_offset=file_offset)
    torch.cuda.synchronize()
    img, handles, types = so.write_blocks(raws, 2, file_offset, zstd_level=level)
    assert typ.cpu().tolist() == types and 2 in types and 0 in types
    assert hoff.cpu().tolist() == [h[0] for h in handles]
    assert hsize.cpu().tolist() == [h[1] for h in handles]
    assert int(end.item()) == file_offset + len(img)
    assert file.cpu().numpy()[file_offset:file_offset + len(img)].tobytes() == img
    # ReadBlock on the device reads every block back
    out, ooff, olen, st = lvkv.sst_read_blocks(file, hoff, hsize, max_ulen=8192)
    torch.cuda.synchronize()
    assert st.cpu().tolist() == [lvkv.READ_OK] * len(raws)
    assert _unpack(out, ooff, olen) == raws


@pytest.mark.gpu
def test_device_write_blocks_zstd_rejects_host_levels(lvkv, gpu):
    import torch
    src, off, ln = _pack(torch, gpu, [b"x" * 100])
    for lvl in (0, 3):
        with pytest.raises(RuntimeError):
            lvkv.sst_write_blocks(src, off, ln, compression=2, zstd_level=lvl)
