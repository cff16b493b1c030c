"""§8(f) row 4, the read side of kZstdCompression: ReadBlock's zstd case
(table/format.cc:138-155) through port::Zstd_GetUncompressedLength /
Zstd_Uncompress (port/port_stdcxx.h:163-199).

Pins: the oracle (oracle/zstd_oracle.py, an RFC 8878 decoder) against the
fixtures libzstd 1.4.9 wrote (tests/golden/gen_zstd.py): every frame decodes
to its input, and every damaged frame gets the library's verdict; where the
library is present, also against it on fresh fuzz. The device decoder is
then held to the fixtures and the oracle.
"""
from __future__ import annotations

import hashlib
import json

import numpy as np
import pytest

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
def fx():
    spec = json.loads((GOLDEN / "zstd.json").read_text())
    ins = _split((GOLDEN / "zstd_inputs.bin").read_bytes(), spec["inputs"])
    frames = _split((GOLDEN / "zstd_frames.bin").read_bytes(), spec["frames"])
    dam = _split((GOLDEN / "zstd_damaged.bin").read_bytes(), spec["damaged"])
    for x, h in zip(ins, spec["sha256_inputs"]):
        assert hashlib.sha256(x).hexdigest() == h
    return ins, frames, spec["meta"], dam, spec["verdicts"]


def _verdict(ok):
    return 2 if ok is None else int(ok)


def test_oracle_decodes_every_library_frame(fx):
    ins, frames, meta, _, _ = fx
    assert {lvl for _, lvl in meta} == {1, 3, 19, -5}
    for f, (i, lvl) in zip(frames, meta):
        assert zo.get_uncompressed_length(f) == len(ins[i]) or len(ins[i]) == 0
        assert zo.decompress(f, len(ins[i])) == ins[i], (i, lvl)


def test_oracle_damaged_verdicts_match_fixtures(fx):
    _, _, _, dam, verdicts = fx
    assert {v["ok"] for v in verdicts} == {0, 1, 2}
    for d, v in zip(dam, verdicts):
        ok, out = zo.uncompress(d)
        assert _verdict(ok) == v["ok"], d[:16].hex()
        if ok:
            assert hashlib.sha256(out).hexdigest() == v["sha256"]


def test_oracle_matches_library_on_fuzz():
    lib = zo.system_zstd()
    if lib is None:
        pytest.skip("libzstd 1.4.9 not present")
    from tools.db_bench_data import block_batch
    rng = np.random.default_rng(31)
    bb = block_batch(8).tobytes()
    for k in range(400):
        n = int(rng.integers(0, 3000))
        s = int(rng.integers(0, len(bb) - n))
        x = bb[s:s + n] if k % 2 else rng.integers(0, int(rng.integers(2, 256)), n,
                                                     dtype=np.uint8).tobytes()
        f = zo.lib_compress(lib, x, (1, 3, 19)[k % 3])
        assert zo.decompress(f, len(x)) == x
        d = bytearray(f)
        d[int(rng.integers(0, len(d)))] ^= 1 << int(rng.integers(0, 8))
        assert zo.uncompress(bytes(d)) == zo.lib_uncompress(lib, bytes(d))


# ---- the device decoder (GPU) ---------------------------------------------

def _pack(torch, dev, blobs, skew=0):
    offs, p = [], skew
    for b in blobs:
        offs.append(p)
        p += len(b)
    buf = np.zeros(max(1, p), dtype=np.uint8)
    for o, b in zip(offs, blobs):
        buf[o:o + len(b)] = np.frombuffer(b, dtype=np.uint8)
    return (torch.from_numpy(buf).to(dev), torch.tensor(offs, dtype=torch.int64, device=dev),
            torch.tensor([len(b) for b in blobs], dtype=torch.int32, device=dev))


def _unpack(dst, offs, lens):
    d = dst.cpu().numpy()
    return [d[o:o + n].tobytes() for o, n in zip(offs.cpu().tolist(), lens.cpu().tolist())]


def _in_cap(cap):  # ZSTD_compressBound (1.4.9)
    return cap + (cap >> 8) + (((128 << 10) - cap) >> 11 if cap < (128 << 10) else 0)


def _want(lvkv, f, cap, ok=None):
    """The device's status for stream f at capacity cap, from the oracle."""
    n = zo.get_uncompressed_length(f)
    if n is None:
        return lvkv.SNAPPY_BAD_LENGTH
    if n > cap:
        return lvkv.SNAPPY_CAPACITY
    # (a stream past the LDS staging, len(f) > _in_cap(max_ulen), is decoded
    # by the HBM-output kernel: the same verdict)
    if ok is None:
        ok, _ = zo.uncompress(f)
    return lvkv.SNAPPY_OK if ok else lvkv.SNAPPY_BAD_CONTENTS


@pytest.mark.gpu
def test_device_decodes_every_library_frame(lvkv, gpu, fx):
    import torch
    ins, frames, meta, _, _ = fx
    cap = lvkv.SNAPPY_MAX_BLOCK
    src, off, ln = _pack(torch, gpu, frames, skew=3)
    dst, doff, dlen, st, why = lvkv.zstd_uncompress(src, off, ln, max_ulen=cap, detail=True)
    ul, ust = lvkv.zstd_uncompressed_length(src, off, ln)
    torch.cuda.synchronize()
    st, why, ul, ust = st.cpu().tolist(), why.cpu().tolist(), ul.cpu().tolist(), ust.cpu().tolist()
    got = _unpack(dst, doff, dlen)
    for k, (f, (i, lvl)) in enumerate(zip(frames, meta)):
        x = ins[i]
        want = _want(lvkv, f, cap, ok=True)
        assert st[k] == want, (k, i, lvl, len(x), st[k], want, why[k])
        if want == 0:
            assert got[k] == x, (k, i, lvl)
        assert ust[k] == (lvkv.SNAPPY_BAD_LENGTH if len(x) == 0 else 0)
        if len(x):
            assert ul[k] == len(x)


@pytest.mark.gpu
@pytest.mark.parametrize("cap", [4096, 49152])
def test_device_damaged_verdicts_match_fixtures(lvkv, gpu, fx, cap):
    import torch
    _, _, _, dam, verdicts = fx
    src, off, ln = _pack(torch, gpu, dam)
    dst, doff, dlen, st, why = lvkv.zstd_uncompress(src, off, ln, max_ulen=cap, detail=True)
    torch.cuda.synchronize()
    st, why = st.cpu().tolist(), why.cpu().tolist()
    got = _unpack(dst, doff, dlen)
    for k, (d, v) in enumerate(zip(dam, verdicts)):
        want = _want(lvkv, d, cap, ok=None if v["ok"] == 2 else bool(v["ok"]))
        assert st[k] == want, (k, d[:12].hex(), st[k], want, why[k])
        if want == 0:
            assert hashlib.sha256(got[k]).hexdigest() == v["sha256"]


@pytest.mark.gpu
def test_device_fuzz_against_oracle(lvkv, gpu):
    """5,000 frames of db_bench-like, text and few-symbol bytes, written by
    the library where present (else the fixtures' frames), 1-4 bytes changed
    or cut: the device's verdict and bytes equal the oracle's."""
    import torch
    from tools.db_bench_data import block_batch
    lib = zo.system_zstd()
    rng = np.random.default_rng(41)
    bb = block_batch(16).tobytes()
    if lib is not None:
        base = []
        for k in range(60):
            n = int(rng.integers(1, 4096))
            s = int(rng.integers(0, len(bb) - n))
            x = bb[s:s + n] if k % 3 else rng.integers(0, 6, n, dtype=np.uint8).tobytes()
            base.append(zo.lib_compress(lib, x, (1, 3, 19)[k % 3]))
    else:
        spec = json.loads((GOLDEN / "zstd.json").read_text())
        base = [f for f in _split((GOLDEN / "zstd_frames.bin").read_bytes(), spec["frames"])
                if len(f) < 4000]
    frames = []
    for k in range(5000):
        f = bytearray(base[k % len(base)])
        if k % 10:  # (one in ten left whole)
            for _ in range(int(rng.integers(1, 5))):
                j = int(rng.integers(0, len(f)))
                f[j] = int(rng.integers(0, 256)) if k % 2 else f[j] ^ (1 << int(rng.integers(0, 8)))
            if k % 7 == 0:
                f = f[: int(rng.integers(1, len(f) + 1))]
        frames.append(bytes(f))
    cap = 8192
    src, off, ln = _pack(torch, gpu, frames, skew=1)
    dst, doff, dlen, st, why = lvkv.zstd_uncompress(src, off, ln, max_ulen=cap, detail=True)
    torch.cuda.synchronize()
    st, why = st.cpu().tolist(), why.cpu().tolist()
    got = _unpack(dst, doff, dlen)
    for k, f in enumerate(frames):
        want = _want(lvkv, f, cap)
        assert st[k] == want, (k, f[:12].hex(), st[k], want, why[k])
        if want == 0:
            assert got[k] == zo.uncompress(f)[1]


@pytest.mark.gpu
def test_device_read_blocks_with_zstd_blocks(lvkv, gpu):
    """ReadBlock over a file image whose blocks are raw, snappy and zstd
    (the zstd ones written by the library: TableBuilder's kZstdCompression
    case, table_builder.cc:172-185, under the same 12.5 % rule)."""
    import torch
    import snappy_oracle as so
    lib = zo.system_zstd()
    if lib is None:
        pytest.skip("libzstd 1.4.9 not present (the writer of the zstd blocks)")
    from tools.db_bench_data import block_batch
    crc = so._crc()
    rng = np.random.default_rng(8)
    bb = block_batch(32).tobytes()
    img = bytearray()
    handles, raws, types = [], [], []
    for k in range(300):
        n = int(rng.integers(0, 6000))
        s = int(rng.integers(0, len(bb) - n))
        raw = bb[s:s + n] if k % 4 else rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        t = k % 3
        contents = raw
        if t == 1:
            c = so.compress(raw)
            contents, t = (c, 1) if len(c) < len(raw) - len(raw) // 8 else (raw, 0)
        elif t == 2:
            c = zo.lib_compress(lib, raw, 1)
            contents, t = (c, 2) if len(c) < len(raw) - len(raw) // 8 else (raw, 0)
        handles.append((len(img), len(contents)))
        raws.append(raw)
        types.append(t)
        img += contents + bytes([t])
        img += crc.mask(crc.extend(crc.value(contents), bytes([t]))).to_bytes(4, "little")
    assert {0, 1, 2} <= set(types)
    bad = bytearray(img)
    hurt = set()
    for i in rng.choice(len(handles), 20, replace=False).tolist():
        o, sz = handles[i]
        if sz:
            bad[o + int(rng.integers(0, sz))] ^= 0x41
            hurt.add(i)
    file = torch.from_numpy(np.frombuffer(bytes(bad), dtype=np.uint8).copy()).to(gpu)
    ho = torch.tensor([h[0] for h in handles], dtype=torch.int64, device=gpu)
    hs = torch.tensor([h[1] for h in handles], dtype=torch.int32, device=gpu)
    for verify in (True, False):
        out, ooff, olen, st = lvkv.sst_read_blocks(file, ho, hs, max_ulen=8192, verify=verify)
        torch.cuda.synchronize()
        st, olen = st.cpu().tolist(), olen.cpu().tolist()
        got = _unpack(out, ooff, torch.tensor(olen))
        for i, (o, sz) in enumerate(handles):
            want_st, want = so.read_block(bytes(bad), o, sz, verify)
            if types[i] == 2 and want_st in (so.READ_OK, so.READ_ZSTD_CONTENTS):
                n = zo.get_uncompressed_length(bytes(bad[o:o + sz]))
                if n is not None and n > 8192:
                    want_st = lvkv.READ_CAPACITY
            assert st[i] == want_st, (i, types[i], verify, st[i], want_st)
            if want_st == so.READ_OK:
                assert got[i] == want
                if i not in hurt:
                    assert want == raws[i]


def test_predefined_tables_header_matches_oracle():
    """csrc/lvkv_zstd_tables.h (tools/gen_zstd_tables.py) holds the oracle's
    decode tables of the predefined distributions."""
    import re
    from conftest import REPO
    text = (REPO / "leveldb-kv-separation_amd" / "csrc" / "lvkv_zstd_tables.h").read_text()
    for name, dist in (("LL", zo.LL_DEFAULT), ("ML", zo.ML_DEFAULT), ("OF", zo.OF_DEFAULT)):
        table, log = zo.build_fse(*dist)
        m = re.search(rf"kPredef{name}\[\d+\] = \{{([^}}]*)\}}", text)
        got = [int(x.strip().rstrip("u"), 16) for x in m.group(1).split(",")]
        assert got == [s | (nb << 8) | (b << 16) for s, nb, b in table]
        assert f"kPredef{name}Log = {log};" in text


# ---- multi-block frames (tests/golden/gen_zstd_stream.py) -----------------

@pytest.fixture(scope="module")
def sfx():
    spec = json.loads((GOLDEN / "zstd_stream.json").read_text())
    ins = _split((GOLDEN / "zstd_stream_inputs.bin").read_bytes(), spec["inputs"])
    frames = _split((GOLDEN / "zstd_stream_frames.bin").read_bytes(), spec["frames"])
    return ins, frames, spec


def test_oracle_decodes_streamed_frames(sfx):
    """Frames of several small blocks (a flush every 1-4 KiB): the later
    blocks reuse the earlier one's Huffman tree (treeless literals) and FSE
    tables (repeat mode), carry repeat offsets and reach back into earlier
    blocks' output."""
    ins, frames, spec = sfx
    assert spec["counts"]["treeless"] > 100 and spec["counts"]["fse_repeat"] > 10
    assert min(m[4] for m in spec["meta"]) >= 2
    for f, m in zip(frames, spec["meta"]):
        x = ins[m[0]]
        assert zo.get_uncompressed_length(f) == len(x)
        ok, got = zo.uncompress(f)
        assert ok and got == x, m
    lib = zo.system_zstd()
    if lib is not None:
        for f, m in zip(frames, spec["meta"]):
            assert zo.lib_uncompress(lib, f) == (True, ins[m[0]])


@pytest.mark.gpu
def test_device_decodes_streamed_frames(lvkv, gpu, sfx):
    import torch
    ins, frames, spec = sfx
    src, off, ln = _pack(torch, gpu, frames, skew=1)
    dst, doff, dlen, st, why = lvkv.zstd_uncompress(src, off, ln, max_ulen=lvkv.SNAPPY_MAX_BLOCK,
                                                    detail=True)
    torch.cuda.synchronize()
    st, why = st.cpu().tolist(), why.cpu().tolist()
    got = _unpack(dst, doff, dlen)
    for k, m in enumerate(spec["meta"]):
        assert st[k] == lvkv.SNAPPY_OK, (k, m, st[k], why[k])
        assert got[k] == ins[m[0]], (k, m)


@pytest.mark.gpu
def test_device_streamed_frames_damaged_against_oracle(lvkv, gpu, sfx):
    """Bytes flipped in the multi-block frames: the device's verdict and bytes
    are the oracle's (damage in a later block lands in the repeat paths)."""
    import torch
    _, frames, _ = sfx
    rng = np.random.default_rng(77)
    cap = lvkv.SNAPPY_MAX_BLOCK
    blobs = []
    for k in range(1500):
        d = bytearray(frames[k % len(frames)])
        for _ in range(int(rng.integers(1, 3))):
            d[int(rng.integers(6, len(d)))] ^= 1 << int(rng.integers(0, 8))
        blobs.append(bytes(d))
    src, off, ln = _pack(torch, gpu, blobs, skew=2)
    dst, doff, dlen, st, why = lvkv.zstd_uncompress(src, off, ln, max_ulen=cap, detail=True)
    torch.cuda.synchronize()
    st, why = st.cpu().tolist(), why.cpu().tolist()
    got = _unpack(dst, doff, dlen)
    for k, b in enumerate(blobs):
        ok, want = zo.uncompress(b)
        want_st = _want(lvkv, b, cap, ok=ok)
        assert st[k] == want_st, (k, st[k], want_st, why[k])
        if want_st == lvkv.SNAPPY_OK:
            assert got[k] == want, k
