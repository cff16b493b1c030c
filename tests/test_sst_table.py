"""Whole-SSTable verify: the CPU restatement
(oracle/sst_table.py) pinned by the reference-written golden table, and the
device path lvkv_sst_verify_table_device checked against it.

Corruption cases follow the reference's own tests: corruption_test.cc
TableFile (:227-252: any flipped byte of a table is caught) and the Status
strings of table/format.cc and table/table.cc.
"""
from __future__ import annotations

import ctypes
import json
import struct
import subprocess
import textwrap

import numpy as np
import pytest

import sst_synth
import sst_table as st
from conftest import GOLDEN, REPO


def _golden_img() -> bytes:
    return (GOLDEN / "table.sst").read_bytes()


def _golden_blocks():
    return json.loads((GOLDEN / "table_blocks.json").read_text())["blocks"]


# ---------------------------------------------------------------- CPU -----

def test_oracle_walk_matches_reference_table():
    # The reference's TableBuilder wrote table.sst and listed its blocks in
    # file order (oracle/gen_golden.cc): data..., filter, metaindex, index.
    r = st.verify_table(_golden_img())
    blocks = _golden_blocks()
    assert r.status == st.SST_OK and r.has_filter == 1 and r.nbad == 0
    assert r.handles + [r.meta, r.index] == [(b["offset"], b["size"]) for b in blocks]
    crcs = [b["crc"] for b in blocks]
    assert r.crc_per_block + [r.meta_crc, r.index_crc] == crcs


def test_oracle_footer_errors():
    img = bytearray(_golden_img())
    assert st.verify_table(bytes(img[:47])).status == st.SST_TOO_SHORT
    bad = bytearray(img)
    bad[-1] ^= 0x40
    assert st.verify_table(bytes(bad)).status == st.SST_BAD_MAGIC
    bad = bytearray(img)
    bad[-48:-8] = b"\xff" * 40  # no varint terminates inside the footer
    assert st.verify_table(bytes(bad)).status == st.SST_BAD_HANDLE


def test_oracle_every_block_kind_detects_a_flip():
    img = _golden_img()
    r0 = st.verify_table(img)
    nd = r0.ndata
    # a data block, the filter, the metaindex, the index
    for (off, size), expect in [(r0.handles[3], "data"), (r0.handles[nd], "filter"),
                                (r0.meta, "meta"), (r0.index, "index")]:
        bad = bytearray(img)
        bad[off + size // 2] ^= 1
        r = st.verify_table(bytes(bad))
        if expect == "data":
            assert r.status == st.SST_OK and r.status_per_block[3] == st.BLK_CHECKSUM
            assert r.nbad == 1
        elif expect == "filter":
            assert r.status_per_block[nd] == st.BLK_CHECKSUM and r.nbad == 1
        elif expect == "meta":
            assert r.status == st.SST_OK and r.meta_status == st.BLK_CHECKSUM
            assert r.has_filter == 0 and r.nbad == 0  # ReadMeta drops the filter
        else:
            assert r.status == st.SST_INDEX_CHECKSUM


def test_oracle_synthetic_tables_round_trip():
    for n, filt in ((1, False), (7, True), (300, True)):
        img = sst_synth.build_sst(n, 1024, seed=n, with_filter=filt)
        r = st.verify_table(img)
        assert r.status == st.SST_OK and r.ndata == n and r.has_filter == int(filt)
        assert r.nbad == 0


def test_report_struct_layout_matches_header(tmp_path, lvkv):
    # The Python mirror of lvkv_sst_report must match the C header byte for byte.
    src = tmp_path / "layout.c"
    src.write_text(textwrap.dedent("""
        #include <stddef.h>
        #include <stdio.h>
        #include "lvkv_crc32c.h"
        #define F(x) printf("%s %zu\\n", #x, offsetof(lvkv_sst_report, x));
        int main(void) {
          printf("size %zu\\n", sizeof(lvkv_sst_report));
          F(status) F(nblocks) F(ndata) F(has_filter) F(nbad) F(first_bad) F(index_crc)
          F(meta_crc) F(index_status) F(meta_status) F(first) F(index_offset) F(index_size)
          F(meta_offset) F(meta_size) F(link_) F(total_) F(done_)
          return 0;
        }"""))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", str(REPO / "include"), str(src), "-o", str(exe)], check=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                  check=True).stdout.splitlines())
    S = lvkv.SstReport
    assert int(got.pop("size")) == ctypes.sizeof(S)
    for name, off in got.items():
        assert getattr(S, name).offset == int(off), name


# ---------------------------------------------------------------- GPU -----

def _device_verify(lvkv, img: bytes, gpu, capacity=None):
    import torch
    buf = torch.from_numpy(np.frombuffer(img, dtype=np.uint8).copy()).to(gpu)
    rep, off, size, actual, status = lvkv.sst_verify_table(buf, capacity=capacity)
    torch.cuda.synchronize()
    return (rep, off.cpu().numpy(), size.cpu().numpy().view(np.uint32),
            actual.cpu().numpy().view(np.uint32), status.cpu().numpy())


def _assert_matches_oracle(lvkv, img: bytes, gpu, capacity=None, got=None, base=0):
    want = st.verify_table(img)
    rep, off, size, actual, status = got if got is not None else _device_verify(
        lvkv, img, gpu, capacity)
    # handles come back as offsets into the device buffer, unreadable entries
    # as (table start, 0)
    off = np.array([int(x) - base for x in off], dtype=np.int64)
    assert rep["status"] == want.status
    assert rep["index_status"] == want.index_status and rep["meta_status"] == want.meta_status
    if want.status in (st.SST_TOO_SHORT, st.SST_BAD_MAGIC, st.SST_BAD_HANDLE):
        assert rep["nblocks"] == 0
        return rep, want
    assert (rep["index_offset"], rep["index_size"]) == want.index
    assert (rep["meta_offset"], rep["meta_size"]) == want.meta
    assert rep["index_crc"] == want.index_crc
    assert rep["meta_crc"] == want.meta_crc
    if want.status == st.SST_CAPACITY:
        assert rep["nblocks"] == 0 and rep["ndata"] == want.ndata
        return rep, want
    assert rep["ndata"] == want.ndata and rep["has_filter"] == want.has_filter
    assert rep["nblocks"] == want.nblocks
    assert [tuple(int(x) for x in h) for h in zip(off, size)] == want.handles
    assert list(status) == want.status_per_block
    for i, c in enumerate(want.crc_per_block):
        assert int(actual[i]) == (c if c is not None else 0), i
    assert rep["nbad"] == want.nbad
    bad = [i for i, s in enumerate(want.status_per_block) if s]
    assert rep["first_bad"] == (bad[0] if bad else 0xFFFFFFFF)
    return rep, want


@pytest.mark.gpu
def test_device_table_verify_golden(lvkv, gpu, sst_form):
    rep, want = _assert_matches_oracle(lvkv, _golden_img(), gpu)
    assert rep["status"] == 0 and rep["nbad"] == 0 and rep["ndata"] == 49


@pytest.mark.gpu
def test_device_table_verify_footer_and_index_errors(lvkv, gpu, sst_form):
    img = _golden_img()
    r0 = st.verify_table(img)
    cases = [img[:40]]
    bad = bytearray(img); bad[-3] ^= 0x10; cases.append(bytes(bad))          # magic
    bad = bytearray(img); bad[-48:-8] = b"\xff" * 40; cases.append(bytes(bad))  # handles
    off, size = r0.index
    bad = bytearray(img); bad[off + 7] ^= 4; cases.append(bytes(bad))        # index crc
    bad = bytearray(img); bad[off + size] = 1                                # snappy index
    sst_synth.fix_trailer(bad, off, size); cases.append(bytes(bad))
    bad = bytearray(img); bad[off + size - 4: off + size] = struct.pack("<I", 10 ** 6)
    sst_synth.fix_trailer(bad, off, size); cases.append(bytes(bad))          # restarts
    for c in cases:
        rep, want = _assert_matches_oracle(lvkv, c, gpu)
        assert rep["status"] != 0


@pytest.mark.gpu
def test_device_table_verify_detects_every_block_kind(lvkv, gpu, sst_form):
    img = _golden_img()
    r0 = st.verify_table(img)
    nd = r0.ndata
    targets = [r0.handles[0], r0.handles[nd // 2], r0.handles[nd - 1], r0.handles[nd],
               r0.meta]
    for off, size in targets:
        for pos in (off, off + size - 1, off + size, off + size + 2):  # contents, type, crc
            bad = bytearray(img)
            bad[pos] ^= 0x80
            _assert_matches_oracle(lvkv, bytes(bad), gpu)


@pytest.mark.gpu
def test_device_table_verify_bad_type_and_handles(lvkv, gpu, sst_form):
    # block 5: type byte 9 under a valid CRC -> "bad block type"; index entry 7
    # points past the file -> "truncated block read"; entry 9's value is not
    # a varint pair -> "bad block handle"; entry 11 has a trailing byte after
    # its handle, which DecodeFrom ignores (format.cc:24-30): the handle (0,
    # 512) is decoded and then misses the real block end -> checksum mismatch.
    img = sst_synth.build_sst(40, 512, seed=3, block_types={5: 9},
                              index_values={7: sst_synth.handle(10 ** 9, 100),
                                            9: b"\xff\xff\xff",
                                            11: sst_synth.handle(0, 512) + b"\x00"})
    rep, want = _assert_matches_oracle(lvkv, img, gpu)
    assert want.status_per_block[5] == st.BLK_BAD_TYPE
    assert want.status_per_block[7] == st.BLK_TRUNCATED
    assert want.status_per_block[9] == st.BLK_BAD_HANDLE
    assert want.status_per_block[11] == st.BLK_CHECKSUM
    assert rep["nbad"] == 4


@pytest.mark.gpu
@pytest.mark.parametrize("n,bs,filt", [(1, 100, False), (257, 1000, True), (5000, 4096, True)])
def test_device_table_verify_synthetic(lvkv, gpu, sst_form, n, bs, filt):
    img = sst_synth.build_sst(n, bs, seed=n, with_filter=filt)
    rep, _ = _assert_matches_oracle(lvkv, img, gpu)
    assert rep["ndata"] == n and rep["nbad"] == 0
    # capacity too small: reported, then the wrapper's retry succeeds
    if n > 1:
        rep2, *_ = _device_verify(lvkv, img, gpu, capacity=n // 2)
        assert rep2["status"] == st.SST_CAPACITY and rep2["ndata"] == n


@pytest.mark.gpu
def test_device_table_verify_wide_index(lvkv, gpu, sst_form):
    # An index over 64 KiB: under the two-launch form a one-table call hands
    # it to sst_index_kernel (CRC cut over the grid, entries decoded by every
    # thread, the verdict settled by the last workgroup). Clean, then every
    # way the index can fail in ReadBlock's / Block::Block's order, a bad
    # entry, a bad data block and a short capacity, each against the oracle.
    img = sst_synth.build_sst(4000, 200, seed=41, index_values={17: b"\xff\xff\xff"})
    r0 = st.verify_table(img)
    off, size = r0.index
    assert size + 1 > 64 * 1024
    cases = [img]
    for pos in (off, off + 1, off + size // 2, off + size - 9, off + size - 1):
        bad = bytearray(img); bad[pos] ^= 0x21; cases.append(bytes(bad))     # index crc
    bad = bytearray(img); bad[off + size + 2] ^= 1; cases.append(bytes(bad))  # stored crc
    for t in (1, 2, 7):                                                       # index type
        bad = bytearray(img); bad[off + size] = t
        sst_synth.fix_trailer(bad, off, size); cases.append(bytes(bad))
    bad = bytearray(img); bad[off + size - 4: off + size] = struct.pack("<I", 10 ** 7)
    sst_synth.fix_trailer(bad, off, size); cases.append(bytes(bad))          # restarts
    bad = bytearray(img); bad[off + size - 4: off + size] = struct.pack("<I", 10 ** 7)
    cases.append(bytes(bad))                                                  # restarts, crc bad
    d_off, d_size = r0.handles[100]
    bad = bytearray(img); bad[d_off + 3] ^= 1; cases.append(bytes(bad))      # data block
    for c in cases:
        _assert_matches_oracle(lvkv, c, gpu)
    rep, *_ = _device_verify(lvkv, img, gpu, capacity=1000)
    assert rep["status"] == st.SST_CAPACITY and rep["ndata"] == 4000
    bad = bytearray(img); bad[off + 5] ^= 1
    rep, *_ = _device_verify(lvkv, bytes(bad), gpu, capacity=1000)
    assert rep["status"] == st.SST_INDEX_CHECKSUM and rep["nblocks"] == 0


# --------------------------------------------- write side (§8f row 3) -----

@pytest.mark.gpu
@pytest.mark.parametrize("source", ["golden", "synthetic"])
def test_device_fill_trailers_rebuilds_the_table(lvkv, gpu, source):
    # TableBuilder::WriteRawBlock (table_builder.cc:192-209) wrote these
    # trailers; wipe every CRC (types kept) and let the device refill them.
    import torch
    if source == "golden":
        img = _golden_img()
        blocks = [(b["offset"], b["size"]) for b in _golden_blocks()]
    else:
        img = sst_synth.build_sst(3000, 4096, seed=21)
        r = st.verify_table(img)
        blocks = r.handles + [r.meta, r.index]
    wiped = bytearray(img)
    for off, size in blocks:
        wiped[off + size + 1: off + size + 5] = b"\0\0\0\0"
    buf = torch.from_numpy(np.frombuffer(bytes(wiped), dtype=np.uint8).copy()).to(gpu)
    offs = torch.tensor([o for o, _ in blocks], dtype=torch.int64, device=gpu)
    sizes = torch.tensor([s for _, s in blocks], dtype=torch.int32, device=gpu)
    crc = lvkv.sst_fill_trailers(buf, offs, sizes)
    torch.cuda.synchronize()
    assert bytes(buf.cpu().numpy()) == img
    import oracle
    want = [oracle.value(img[o: o + s + 1]) for o, s in blocks]
    assert list(crc.cpu().numpy().view(np.uint32)) == want


@pytest.mark.gpu
def test_device_table_with_long_blocks(lvkv, gpu, sst_form):
    # Data blocks far beyond kLongBytes (one huge value per block, as a table
    # with big values gets): verify, a corrupted long block, and the refill.
    import torch
    img = sst_synth.build_sst(24, 300_000, seed=8)
    rep, want = _assert_matches_oracle(lvkv, img, gpu)
    assert rep["nbad"] == 0
    r0 = st.verify_table(img)
    off, size = r0.handles[7]
    bad = bytearray(img)
    bad[off + size - 3] ^= 0x20
    rep, want = _assert_matches_oracle(lvkv, bytes(bad), gpu)
    assert rep["nbad"] == 1 and rep["first_bad"] == 7
    blocks = r0.handles + [r0.meta, r0.index]
    wiped = bytearray(img)
    for o, s in blocks:
        wiped[o + s + 1: o + s + 5] = b"\0\0\0\0"
    buf = torch.from_numpy(np.frombuffer(bytes(wiped), dtype=np.uint8).copy()).to(gpu)
    lvkv.sst_fill_trailers(buf, torch.tensor([o for o, _ in blocks], dtype=torch.int64, device=gpu),
                           torch.tensor([s for _, s in blocks], dtype=torch.int32, device=gpu))
    torch.cuda.synchronize()
    assert bytes(buf.cpu().numpy()) == img


@pytest.mark.gpu
def test_device_many_small_tables(lvkv, gpu, sst_form):
    # 120 tables of 1-40 blocks in one call (the speculative form shares its
    # CRC workgroups out by table size, at least one per table; 120 is under
    # half the CUs), two of them damaged: each exactly as the oracle says.
    import torch
    rng = np.random.default_rng(77)
    imgs = []
    for t in range(120):
        im = bytearray(sst_synth.build_sst(int(rng.integers(1, 41)), int(rng.integers(64, 5000)),
                                           seed=1000 + t, with_filter=bool(t % 3)))
        if t in (17, 90):
            im[int(rng.integers(0, len(im) // 2))] ^= 0x20
        imgs.append(bytes(im))
    offs, pos = [], 0
    for im in imgs:
        offs.append(pos)
        pos += len(im) + 7
    buf = bytearray(pos)
    for o_, im in zip(offs, imgs):
        buf[o_: o_ + len(im)] = im
    dbuf = torch.from_numpy(np.frombuffer(bytes(buf), dtype=np.uint8).copy()).to(gpu)
    res = lvkv.sst_verify_tables(dbuf, offs, [len(im) for im in imgs])
    torch.cuda.synchronize()
    for o_, im, (rep, off, size, actual, status) in zip(offs, imgs, res):
        got = (rep, off.cpu().numpy(), size.cpu().numpy().view(np.uint32),
               actual.cpu().numpy().view(np.uint32), status.cpu().numpy())
        _assert_matches_oracle(lvkv, im, gpu, got=got, base=o_)


@pytest.mark.gpu
def test_device_multi_table_verify(lvkv, gpu, sst_form):
    # Compaction-input shape: many tables in one buffer, each checked exactly
    # as the single-table call would (lvkv_sst_verify_tables_device).
    import torch
    gold = _golden_img()
    r0 = st.verify_table(gold)
    bad = bytearray(gold)
    o, n = r0.handles[11]
    bad[o + n // 3] ^= 4
    imgs = [gold, sst_synth.build_sst(300, 4096, seed=30), bytes(bad),
            b"\x07" * 2000, sst_synth.build_sst(1, 50, seed=31, with_filter=False),
            sst_synth.build_sst(6, 200_000, seed=32)] * 3
    offs, pos = [], 0
    for im in imgs:
        offs.append(pos)
        pos += len(im) + 13  # unaligned table starts
    buf = bytearray(pos)
    for o_, im in zip(offs, imgs):
        buf[o_: o_ + len(im)] = im
    dbuf = torch.from_numpy(np.frombuffer(bytes(buf), dtype=np.uint8).copy()).to(gpu)
    res = lvkv.sst_verify_tables(dbuf, offs, [len(im) for im in imgs])
    torch.cuda.synchronize()
    assert len(res) == len(imgs)
    for o_, im, (rep, off, size, actual, status) in zip(offs, imgs, res):
        got = (rep, off.cpu().numpy(), size.cpu().numpy().view(np.uint32),
               actual.cpu().numpy().view(np.uint32), status.cpu().numpy())
        _assert_matches_oracle(lvkv, im, gpu, got=got, base=o_)
    # a shared capacity too small for all: the tables that fit are verified,
    # the first that does not and every later one report LVKV_SST_CAPACITY
    small = lvkv.sst_verify_tables(dbuf, offs, [len(im) for im in imgs], capacity=400)
    torch.cuda.synchronize()
    stats = [r[0]["status"] for r in small]
    assert stats[0] == 0 and st.SST_CAPACITY in stats
    k = stats.index(st.SST_CAPACITY)
    assert all(s_ in (st.SST_CAPACITY, st.SST_BAD_MAGIC) for s_ in stats[k:])
    assert res[2][0]["nbad"] == 1 and res[3][0]["status"] == st.SST_BAD_MAGIC


@pytest.mark.gpu
def test_device_table_shares_over_one_pass(lvkv, gpu, sst_form):
    # 150k tiny blocks: the speculative form's CRC workgroups (2 x CUs - 1 for
    # one table) each own ~290 index entries, more than one pass of 256, and
    # the shares at the index's end took their restart offsets from the
    # staged tail on the first pass (later passes must not read it
    # back after the window overwrote it). One table, then three in one call,
    # each with a damaged block in the last entries.
    import torch
    img = bytearray(sst_synth.build_sst(150_000, 16, seed=5, ragged=False))
    r0 = st.verify_table(bytes(img))
    for e in (149_999, 149_800, 149_300):
        o, n = r0.handles[e]
        img[o + 3] ^= 0x40
    img = bytes(img)
    rep, _ = _assert_matches_oracle(lvkv, img, gpu)
    assert rep["ndata"] == 150_000 and rep["nbad"] == 3 and rep["first_bad"] == 149_300
    imgs = [img, sst_synth.build_sst(120_000, 24, seed=6, ragged=False), img]
    offs, pos = [], 0
    for im in imgs:
        offs.append(pos)
        pos += len(im) + 5
    buf = bytearray(pos)
    for o_, im in zip(offs, imgs):
        buf[o_: o_ + len(im)] = im
    dbuf = torch.from_numpy(np.frombuffer(bytes(buf), dtype=np.uint8).copy()).to(gpu)
    res = lvkv.sst_verify_tables(dbuf, offs, [len(im) for im in imgs], capacity=430_000)
    torch.cuda.synchronize()
    for o_, im, (rep, off, size, actual, status) in zip(offs, imgs, res):
        got = (rep, off.cpu().numpy(), size.cpu().numpy().view(np.uint32),
               actual.cpu().numpy().view(np.uint32), status.cpu().numpy())
        _assert_matches_oracle(lvkv, im, gpu, got=got, base=o_)
