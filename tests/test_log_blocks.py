"""WAL / MANIFEST block verify: the CPU restatement of
log::Reader::ReadPhysicalRecord (oracle/log_walk.py) pinned by the
reference-written golden log and the reference's own log_test.cc cases, and
the device path lvkv_log_verify_blocks_device checked against it.
"""
from __future__ import annotations

import ctypes
import json
import random
import subprocess
import textwrap

import numpy as np
import pytest

import log_synth
import log_walk as lw
from conftest import GOLDEN, REPO


def _golden_log() -> bytes:
    return (GOLDEN / "wal.log").read_bytes()


def _check_equivalent(img: bytes) -> None:
    """The per-block form (what the device computes) yields exactly the
    sequential reader's returned records and reported corruptions."""
    w = lw.read_physical_records(img)
    v = lw.block_verdicts(img)
    assert [h for h, s in zip(v.hdrs, v.rec_status) if s == lw.REC_OK] == [r[0] for r in w.records]
    reported = [(d, "checksum mismatch" if s == lw.BLK_CHECKSUM else "bad record length")
                for s, d in zip(v.block_status, v.block_drop)
                if s in (lw.BLK_CHECKSUM, lw.BLK_BAD_LENGTH)]
    assert reported == w.corruptions


# ---------------------------------------------------------------- CPU -----

def test_oracle_reads_reference_log():
    # oracle/gen_golden.cc wrote wal.log with log::Writer and listed every
    # physical record log::Reader returned.
    fx = json.loads((GOLDEN / "wal_records.json").read_text())
    w = lw.read_physical_records(_golden_log())
    assert w.records == [(r["offset"], r["length"], r["type"]) for r in fx["records"]]
    assert w.corruptions == []
    v = lw.block_verdicts(_golden_log())
    assert v.hdrs == [r["offset"] for r in fx["records"]]


def test_oracle_log_test_cases():
    # db/log_test.cc, restated on images built like its Writer does.
    def one(payload):
        wr = log_synth.LogWriter()
        wr.add_record(payload)
        return bytearray(wr.buf)
    img = one(b"foo")                                  # ChecksumMismatch (:412-418)
    img[0] = (img[0] + 10) & 0xFF
    w = lw.read_physical_records(bytes(img))
    assert w.records == [] and w.corruptions == [(10, "checksum mismatch")]
    wr = log_synth.LogWriter()                         # BadLength (:393-402)
    wr.add_record(b"b" * (32768 - 7))
    wr.add_record(b"foo")
    img = bytearray(wr.buf)
    img[4] = (img[4] + 1) & 0xFF
    w = lw.read_physical_records(bytes(img))
    assert [r[1] for r in w.records] == [3] and w.corruptions == [(32768, "bad record length")]
    img = one(b"foo")[:-1]                             # BadLengthAtEndIsIgnored (:404-410)
    assert lw.read_physical_records(bytes(img)).corruptions == []
    img = one(b"foo")[:-4]                             # TruncatedTrailingRecordIsIgnored
    w = lw.read_physical_records(bytes(img))
    assert w.records == [] and w.corruptions == []
    wr = log_synth.LogWriter()                         # MarginalTrailer (:296-307)
    wr.add_record(b"a" * (32768 - 2 * 7))
    wr.add_record(b"")
    wr.add_record(b"bar")
    w = lw.read_physical_records(bytes(wr.buf))
    assert [r[1] for r in w.records] == [32768 - 14, 0, 3]
    for img in (_golden_log(), log_synth.build_log(200, seed=2, big_every=37)):
        _check_equivalent(img)


def test_oracle_block_form_equivalent_under_random_damage():
    img = log_synth.build_log(300, seed=5, max_len=4000, big_every=53)
    rng = random.Random(7)
    for _ in range(200):
        b = bytearray(img)
        for _ in range(rng.randint(1, 4)):
            p = rng.randrange(len(b))
            b[p] ^= 1 << rng.randrange(8)
        if rng.random() < 0.3:
            b = b[: rng.randrange(len(b))]
        if rng.random() < 0.2:  # a preallocated zero region
            p = rng.randrange(len(b))
            b[p: p + 64] = b"\0" * len(b[p: p + 64])
        _check_equivalent(bytes(b))


def test_log_report_struct_layout(tmp_path, lvkv):
    src = tmp_path / "layout.c"
    src.write_text(textwrap.dedent("""
        #include <stddef.h>
        #include <stdio.h>
        #include "lvkv_crc32c.h"
        #define F(x) printf("%s %zu\\n", #x, offsetof(lvkv_log_report, x));
        int main(void) {
          printf("size %zu\\n", sizeof(lvkv_log_report));
          F(status) F(nblocks) F(nrecords) F(ngood) F(ncorrupt) F(first_bad_block)
          F(dropped_bytes) F(count_)
          return 0;
        }"""))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", str(REPO / "include"), str(src), "-o", str(exe)], check=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                  check=True).stdout.splitlines())
    S = lvkv.LogReport
    assert int(got.pop("size")) == ctypes.sizeof(S)
    for name, off in got.items():
        assert getattr(S, name).offset == int(off), name


def test_log_read_struct_layouts(tmp_path, lvkv):
    # lvkv_log_read_device's outputs as the Python log_read() decodes them:
    # lvkv_log_read_report (ctypes mirror), lvkv_log_record (24 bytes: offset,
    # length, first | nfrags << 32) and lvkv_log_corruption (16 bytes: bytes,
    # reason | type << 32), and the reason codes the wrapper names.
    src = tmp_path / "layout.c"
    src.write_text(textwrap.dedent("""
        #include <stddef.h>
        #include <stdio.h>
        #include "lvkv_crc32c.h"
        #define R(x) printf("r.%s %zu\\n", #x, offsetof(lvkv_log_read_report, x));
        int main(void) {
          printf("r.size %zu\\n", sizeof(lvkv_log_read_report));
          R(status) R(nrecords) R(nreports) R(stopped) R(bytes)
          printf("rec %zu %zu %zu %zu %zu\\n", sizeof(lvkv_log_record),
                 offsetof(lvkv_log_record, offset), offsetof(lvkv_log_record, length),
                 offsetof(lvkv_log_record, first), offsetof(lvkv_log_record, nfrags));
          printf("cor %zu %zu %zu %zu\\n", sizeof(lvkv_log_corruption),
                 offsetof(lvkv_log_corruption, bytes), offsetof(lvkv_log_corruption, reason),
                 offsetof(lvkv_log_corruption, type));
          printf("why %d %d %d %d %d %d %d %d\\n", LVKV_LOGR_CHECKSUM, LVKV_LOGR_BAD_LENGTH,
                 LVKV_LOGR_PARTIAL_1, LVKV_LOGR_PARTIAL_2, LVKV_LOGR_MISSING_1,
                 LVKV_LOGR_MISSING_2, LVKV_LOGR_MIDDLE, LVKV_LOGR_UNKNOWN_TYPE);
          return 0;
        }"""))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", str(REPO / "include"), str(src), "-o", str(exe)], check=True)
    lines = subprocess.run([str(exe)], capture_output=True, text=True,
                           check=True).stdout.splitlines()
    got = {l.split()[0]: l.split()[1:] for l in lines}
    S = lvkv.LogReadReport
    assert int(got.pop("r.size")[0]) == ctypes.sizeof(S)
    for name in ("status", "nrecords", "nreports", "stopped", "bytes"):
        assert getattr(S, name).offset == int(got["r." + name][0]), name
    assert [int(x) for x in got["rec"]] == [24, 0, 8, 16, 20]
    assert [int(x) for x in got["cor"]] == [16, 0, 8, 12]
    codes = [int(x) for x in got["why"]]
    assert sorted(lvkv.LOG_REASONS) == codes
    assert lvkv.LOG_REASONS[1] == "checksum mismatch"
    assert lvkv.LOG_REASONS[7] == "error in middle of record"


# ---------------------------------------------------------------- GPU -----

def _device(lvkv, img: bytes, gpu, capacity=None):
    import torch
    buf = torch.from_numpy(np.frombuffer(img, dtype=np.uint8).copy()).to(gpu)
    rep, hdr, actual, rst, bst, bdrop = lvkv.log_verify_blocks(buf, capacity=capacity)
    torch.cuda.synchronize()
    return (rep, hdr.cpu().numpy(), actual.cpu().numpy().view(np.uint32), rst.cpu().numpy(),
            bst.cpu().numpy(), bdrop.cpu().numpy().view(np.uint32))


def _assert_matches(lvkv, img: bytes, gpu):
    import oracle
    v = lw.block_verdicts(img)
    w = lw.read_physical_records(img)
    rep, hdr, actual, rst, bst, bdrop = _device(lvkv, img, gpu)
    assert rep["status"] == 0
    assert rep["nrecords"] == len(v.hdrs) and list(hdr) == v.hdrs
    assert list(rst) == v.rec_status
    assert list(bst) == v.block_status and list(bdrop) == v.block_drop
    assert rep["ngood"] == len(w.records) and rep["ncorrupt"] == len(w.corruptions)
    assert rep["dropped_bytes"] == sum(d for d, _ in w.corruptions)
    bad = [i for i, s in enumerate(v.block_status) if s in (lw.BLK_CHECKSUM, lw.BLK_BAD_LENGTH)]
    assert rep["first_bad_block"] == (bad[0] if bad else 0xFFFFFFFF)
    for i, (h, s) in enumerate(zip(v.hdrs, v.rec_status)):
        if s != lw.REC_DROPPED:
            n = img[h + 4] | (img[h + 5] << 8)
            assert int(actual[i]) == oracle.value(img[h + 6: h + 7 + n]), i
    return rep


@pytest.mark.gpu
def test_device_log_golden(lvkv, gpu):
    rep = _assert_matches(lvkv, _golden_log(), gpu)
    assert rep["ngood"] == 18 and rep["ncorrupt"] == 0


@pytest.mark.gpu
def test_device_log_reference_cases(lvkv, gpu):
    def one(payload):
        wr = log_synth.LogWriter()
        wr.add_record(payload)
        return bytearray(wr.buf)
    cases = []
    img = one(b"foo"); img[0] = (img[0] + 10) & 0xFF; cases.append(img)
    wr = log_synth.LogWriter(); wr.add_record(b"b" * (32768 - 7)); wr.add_record(b"foo")
    img = bytearray(wr.buf); img[4] = (img[4] + 1) & 0xFF; cases.append(img)
    cases += [one(b"foo")[:-1], one(b"foo")[:-4], bytearray()]
    wr = log_synth.LogWriter(); wr.add_record(b"a" * (32768 - 14)); wr.add_record(b"")
    wr.add_record(b"bar"); cases.append(bytearray(wr.buf))
    wr = log_synth.LogWriter(); wr.add_record(b"c" * (32768 - 7)); cases.append(bytearray(wr.buf))
    img = one(b"foo"); img[6] = 100; log_synth.fix_header_crc(img, 0); cases.append(img)
    for c in cases:
        _assert_matches(lvkv, bytes(c), gpu)


@pytest.mark.gpu
def test_device_log_random_damage(lvkv, gpu):
    img = log_synth.build_log(400, seed=9, max_len=5000, big_every=61)
    rng = random.Random(11)
    for _ in range(40):
        b = bytearray(img)
        for _ in range(rng.randint(1, 4)):
            p = rng.randrange(len(b))
            b[p] ^= 1 << rng.randrange(8)
        if rng.random() < 0.3:
            b = b[: rng.randrange(len(b))]
        if rng.random() < 0.2:
            p = rng.randrange(len(b))
            b[p: p + 64] = b"\0" * len(b[p: p + 64])
        _assert_matches(lvkv, bytes(b), gpu)


@pytest.mark.gpu
def test_device_log_large_and_capacity(lvkv, gpu):
    img = log_synth.build_log(20_000, seed=3, max_len=600, big_every=997)  # ~6 MB, ~190 blocks
    rep = _assert_matches(lvkv, img, gpu)
    assert rep["ncorrupt"] == 0 and rep["nblocks"] == (len(img) + 32767) // 32768
    rep2, *_ = _device(lvkv, img, gpu, capacity=100)
    assert rep2["status"] == 1 and rep2["nrecords"] == rep["nrecords"]


@pytest.mark.gpu
def test_device_log_many_blocks_tiled(lvkv, gpu):
    """Past 4096 blocks the emit launch takes every block's first record from
    log_scan_kernel instead of summing the counts before it. A damaged ~1 MB
    log padded to whole 32 KiB blocks (zero trailers, skipped silently) and
    tiled: each block's verdict depends on that block alone, so the oracle's
    answer for the base tiles too."""
    import oracle
    base = bytearray(log_synth.build_log(1500, seed=41, max_len=1200, big_every=89))
    base += bytes(-len(base) % 32768)
    for p in (5000, 200_001, len(base) // 2 + 7):
        base[p] ^= 0x20
    base = bytes(base)
    nb = len(base) // 32768
    tiles = 4096 // nb + 2
    v = lw.block_verdicts(base)
    img = base * tiles
    rep, hdr, actual, rst, bst, bdrop = _device(lvkv, img, gpu)
    assert rep["status"] == 0 and rep["nblocks"] == nb * tiles > 4096
    assert rep["nrecords"] == len(v.hdrs) * tiles
    assert np.array_equal(hdr, np.array([t * len(base) + h for t in range(tiles) for h in v.hdrs]))
    assert list(rst) == v.rec_status * tiles
    assert list(bst) == v.block_status * tiles and list(bdrop) == v.block_drop * tiles
    bad = [i for i, s in enumerate(v.block_status) if s in (lw.BLK_CHECKSUM, lw.BLK_BAD_LENGTH)]
    assert bad and rep["first_bad_block"] == bad[0]
    assert rep["ncorrupt"] == len(bad) * tiles
    assert rep["ngood"] == v.rec_status.count(lw.REC_OK) * tiles
    assert rep["dropped_bytes"] == sum(v.block_drop[i] for i in bad) * tiles
    want = np.array([oracle.value(base[h + 6: h + 7 + (base[h + 4] | base[h + 5] << 8)])
                     for h in v.hdrs], dtype=np.uint32)
    keep = np.tile(np.array(v.rec_status) != lw.REC_DROPPED, tiles)
    assert np.array_equal(actual[keep], np.tile(want, tiles)[keep])


@pytest.mark.gpu
@pytest.mark.parametrize("source", ["golden", "synthetic"])
def test_device_fill_headers_rebuilds_the_log(lvkv, gpu, source):
    # log::Writer::EmitPhysicalRecord (log_writer.cc:82-108) wrote these
    # headers; wipe every header CRC and let the device refill them.
    import torch
    import oracle
    img = _golden_log() if source == "golden" else log_synth.build_log(3000, seed=4,
                                                                         big_every=101)
    hdrs = lw.block_verdicts(img).hdrs
    wiped = bytearray(img)
    for h in hdrs:
        wiped[h: h + 4] = b"\0\0\0\0"
    buf = torch.from_numpy(np.frombuffer(bytes(wiped), dtype=np.uint8).copy()).to(gpu)
    crc = lvkv.log_fill_headers(buf, torch.tensor(hdrs, dtype=torch.int64, device=gpu))
    torch.cuda.synchronize()
    assert bytes(buf.cpu().numpy()) == img
    want = [oracle.value(img[h + 6: h + 7 + (img[h + 4] | img[h + 5] << 8)]) for h in hdrs]
    assert list(crc.cpu().numpy().view(np.uint32)) == want


@pytest.mark.gpu
def test_device_log_two_streams_at_once(lvkv, gpu):
    """Two WAL verifies in flight on two streams (and back to back on each):
    blocks are claimed by ticket and each call has its own scratch, so the
    calls neither deadlock nor share counters; every result equals the
    one-call result."""
    import torch
    L = lvkv.lib
    vp = ctypes.c_void_p
    imgs = [log_synth.build_log(6000, seed=21, max_len=3000, big_every=211),
            log_synth.build_log(9000, seed=22, max_len=1500, big_every=0)]
    want = [_device(lvkv, img, gpu) for img in imgs]
    streams = [torch.cuda.Stream(gpu), torch.cuda.Stream(gpu)]
    outs = []
    for rep_i in range(3):
        for k, img in enumerate(imgs):
            buf = torch.from_numpy(np.frombuffer(img, dtype=np.uint8).copy()).to(gpu)
            torch.cuda.synchronize()
            cap = want[k][0]["nrecords"] + 1
            nb = (len(img) + 32767) // 32768
            o = dict(buf=buf, hdr=torch.empty(cap, dtype=torch.int64, device=gpu),
                     act=torch.empty(cap, dtype=torch.int32, device=gpu),
                     rst=torch.empty(cap, dtype=torch.uint8, device=gpu),
                     bst=torch.empty(nb, dtype=torch.uint8, device=gpu),
                     bdr=torch.empty(nb, dtype=torch.int32, device=gpu),
                     rep=torch.zeros(ctypes.sizeof(lvkv.LogReport), dtype=torch.uint8, device=gpu),
                     k=k)
            outs.append(o)
    # launch everything without a host sync in between, alternating streams
    for i, o in enumerate(outs):
        s = streams[i % 2]
        rc = L.lvkv_log_verify_blocks_device(
            vp(o["buf"].data_ptr()), o["buf"].numel(), vp(o["hdr"].data_ptr()),
            vp(o["act"].data_ptr()), vp(o["rst"].data_ptr()), o["hdr"].numel(),
            vp(o["bst"].data_ptr()), vp(o["bdr"].data_ptr()), vp(o["rep"].data_ptr()),
            vp(s.cuda_stream))
        assert rc == 0
    torch.cuda.synchronize()
    for o in outs:
        rep, hdr, actual, rst, bst, bdrop = want[o["k"]]
        r = lvkv.LogReport.from_buffer_copy(bytes(o["rep"].cpu().numpy())).as_dict()
        assert r == rep
        n = rep["nrecords"]
        assert np.array_equal(o["hdr"][:n].cpu().numpy(), hdr)
        assert np.array_equal(o["act"][:n].cpu().numpy().view(np.uint32), actual)
        assert np.array_equal(o["rst"][:n].cpu().numpy(), rst)
        assert np.array_equal(o["bst"].cpu().numpy(), bst)


@pytest.mark.gpu
def test_device_log_refuses_stream_capture(lvkv, gpu):
    """The verify's scratch counters are zeroed once and left at 0 by each
    call: a captured graph would replay them unzeroed, so capture is refused
    (LVKV_ERR_INVALID) instead of recorded."""
    import torch
    img = log_synth.build_log(50, seed=5)
    buf = torch.from_numpy(np.frombuffer(img, dtype=np.uint8).copy()).to(gpu)
    L = lvkv.lib
    vp = ctypes.c_void_p
    hdr = torch.empty(64, dtype=torch.int64, device=gpu)
    act = torch.empty(64, dtype=torch.int32, device=gpu)
    rst = torch.empty(64, dtype=torch.uint8, device=gpu)
    bst = torch.empty(4, dtype=torch.uint8, device=gpu)
    bdr = torch.empty(4, dtype=torch.int32, device=gpu)
    rep = torch.zeros(ctypes.sizeof(lvkv.LogReport), dtype=torch.uint8, device=gpu)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(gpu)
    rcs = []
    with torch.cuda.stream(s):
        g.capture_begin()
        rcs.append(L.lvkv_log_verify_blocks_device(
            vp(buf.data_ptr()), len(img), vp(hdr.data_ptr()), vp(act.data_ptr()),
            vp(rst.data_ptr()), 64, vp(bst.data_ptr()), vp(bdr.data_ptr()), vp(rep.data_ptr()),
            vp(s.cuda_stream)))
        hdr.add_(0)  # capture something so the graph is not empty
        g.capture_end()
    assert rcs == [lvkv.LVKV_ERR_INVALID]


@pytest.mark.gpu
@pytest.mark.parametrize("max_len", [1, 24])
def test_device_log_dense_blocks(lvkv, gpu, max_len):
    """Blocks of thousands of tiny records (7-30 bytes each: up to 4681 in a
    block), past what a slot keeps in LDS: the positions beyond it go
    through the slot's scratch overflow. Also a few damaged ones."""
    img = log_synth.build_log(12_000, seed=31 + max_len, max_len=max_len)
    _assert_matches(lvkv, img, gpu)
    b = bytearray(img)
    for p in (40_000, 70_001, len(b) // 2 + 3):
        b[p] ^= 0x10
    _assert_matches(lvkv, bytes(b), gpu)
