"""Damaged images against the reference itself.

tests/golden/damage_sst.json and damage_wal.json hold what the reference's
own readers reported on seeded damaged copies of the reference-written table
and log (oracle/gen_damage.cc, built from /root/reference where it lies):
Table::Open(paranoid_checks) + ReadBlock(verify_checksums) over every index
entry + the ReadMeta steps (table/table.cc:38-124, table/format.cc:69-160),
and log::Reader(checksum = true) with a recording Reporter
(db/log_reader.cc:55-271).

CPU: the oracles (oracle/sst_table.py, oracle/log_walk.py) reproduce every
case. GPU: the device paths reproduce every case — the whole-SSTable verify
directly, the WAL verify through its per-block verdicts fed to the logical
record assembly (records, offsets, CRCs and every report, in order).
"""
from __future__ import annotations

import numpy as np
import pytest

import damage_fixtures as df
import log_walk as lw
import sst_table as st

SST_CASES = df.sst_cases()
WAL_CASES = df.wal_cases()


def _entries_want(exp):
    return [(o if df.readable(o, s, t) else 0, s if df.readable(o, s, t) else 0, t)
            for o, s, t in exp["entries"]]


# ---------------------------------------------------------------- CPU -----

def test_fixtures_cover_the_cases_the_verdict_names():
    names = {c["name"] for c in SST_CASES}
    assert {"data_type_1_crc_fixed", "data_type_2_crc_fixed", "index_type_1_crc_fixed",
            "filter_policy_other_name", "two_filter_keys_bloom", "footer_index_size_max",
            "footer_meta_size_max", "index_restart_count_crc_fixed"} <= names
    assert len(SST_CASES) >= 50 and len(WAL_CASES) >= 40
    # the reference's verdicts the device path must follow
    by = {c["name"]: c for c in SST_CASES}
    assert "snappy" in by["data_type_1_crc_fixed"]["entries"][24][2]
    assert by["filter_policy_other_name"]["filter_found"] is False
    assert by["footer_index_size_max"]["open"] == "Corruption: block checksum mismatch"


@pytest.mark.parametrize("case", SST_CASES, ids=[c["name"] for c in SST_CASES])
def test_oracle_sst_matches_reference(case):
    r = st.verify_table(df.image(case), filter_policy=case["filter_policy"])
    exp = df.sst_expected(case)
    assert r.status == exp["status"]
    assert (r.index_status, r.meta_status) == (exp["index_status"], exp["meta_status"])
    assert r.has_filter == exp["has_filter"]
    got = [(h[0], h[1], s) for h, s in zip(r.handles, r.status_per_block)]
    assert got == _entries_want(exp)


@pytest.mark.parametrize("case", WAL_CASES, ids=[c["name"] for c in WAL_CASES])
def test_oracle_wal_matches_reference(case):
    img = df.image(case, "wal.log")
    recs, reps = df.wal_expected(case)
    assert lw.read_records(img, case["initial_offset"]) == (recs, reps)
    if case["initial_offset"]:
        return  # the block form below is the physical layer from offset 0
    v = lw.block_verdicts(img)
    ev = lw.events_from_blocks(img, v.hdrs, v.rec_status, v.block_status, v.block_drop)
    assert lw.assemble(img, ev) == (recs, reps)


# ---------------------------------------------------------------- GPU -----

@pytest.mark.gpu
def test_device_sst_matches_reference(lvkv, gpu, sst_form):
    import torch
    for case in SST_CASES:
        img = df.image(case)
        buf = torch.from_numpy(np.frombuffer(img, dtype=np.uint8).copy()).to(gpu)
        rep, off, size, actual, status = lvkv.sst_verify_table(
            buf, filter_policy=case["filter_policy"])
        torch.cuda.synchronize()
        exp = df.sst_expected(case)
        name = case["name"]
        assert rep["status"] == exp["status"], name
        assert (rep["index_status"], rep["meta_status"]) == (
            exp["index_status"], exp["meta_status"]), name
        assert rep["has_filter"] == exp["has_filter"], name
        got = [(int(o), int(s), int(t)) for o, s, t in
               zip(off.cpu().numpy(), size.cpu().numpy().view(np.uint32), status.cpu().numpy())]
        assert got == _entries_want(exp), name
        nbad = sum(1 for *_, t in exp["entries"] if t)
        assert rep["nbad"] == nbad, name


@pytest.mark.gpu
def test_device_wal_matches_reference(lvkv, gpu):
    import torch
    for case in WAL_CASES:
        if case["initial_offset"]:
            continue  # the physical layer does not depend on it
        img = df.image(case, "wal.log")
        buf = torch.from_numpy(np.frombuffer(img, dtype=np.uint8).copy()).to(gpu)
        rep, hdr, actual, rst, bst, bdrop = lvkv.log_verify_blocks(buf)
        torch.cuda.synchronize()
        ev = lw.events_from_blocks(img, [int(x) for x in hdr.cpu().numpy()],
                                   list(rst.cpu().numpy()), list(bst.cpu().numpy()),
                                   list(bdrop.cpu().numpy()))
        assert lw.assemble(img, ev) == df.wal_expected(case), case["name"]


def _device_log_records(img, records, hdrs, gathered):
    """(LastRecordOffset, length, CRC32C of the contents) of each device
    record, the contents taken from the device's own gather
    (lvkv_log_gather_device: the records end to end); the CRC is the
    checker's (oracle). The fragment list is cross-checked against the
    image, and the gathered bytes byte for byte against the fragments'
    payloads sliced from the image (ReadRecord's scratch->append of each
    fragment, db/log_reader.cc:92-137), so the CRC comparison with the
    reference rides on top of an exact one."""
    import oracle
    payload, pos = gathered
    pl = payload.cpu().numpy().tobytes()
    pos = [int(x) for x in pos.cpu().numpy()]
    assert len(pos) == len(records)
    out, at = [], 0
    for (off, length, first, nfrags), p in zip(records, pos):
        frags = hdrs[first: first + nfrags]
        want = b"".join(img[h + 7: h + 7 + (img[h + 4] | img[h + 5] << 8)] for h in frags)
        assert hdrs[first] == off and len(want) == length and p == at
        assert pl[p: p + length] == want, ("gathered bytes differ", off)
        at += length
        out.append((off, length, oracle.value(pl[p: p + length])))
    return out


@pytest.mark.gpu
def test_device_log_read_matches_reference(lvkv, gpu):
    # The logical layer on the device (lvkv_log_read_device): records and
    # every Reporter call, against the reference's own log::Reader run on
    # the same damaged images (oracle/gen_damage.cc), from offset 0 and from
    # the cases' initial offsets.
    import torch
    for case in WAL_CASES:
        img = df.image(case, "wal.log")
        buf = torch.from_numpy(np.frombuffer(img, dtype=np.uint8).copy()).to(gpu)
        rd, records, reports, phys, gathered = lvkv.log_read(
            buf, initial_offset=case["initial_offset"], gather=True)
        torch.cuda.synchronize()
        assert rd["status"] == 0, case["name"]
        hdrs = [int(x) for x in phys[1].cpu().numpy()]
        want_recs, want_reps = df.wal_expected(case)
        assert _device_log_records(img, records, hdrs, gathered) == want_recs, case["name"]
        assert reports == want_reps, case["name"]
        assert rd["bytes"] == sum(r[1] for r in want_recs), case["name"]
        stopped = lw.read_all(img, case["initial_offset"])[2]
        assert rd["stopped"] == int(stopped), case["name"]
        if not case["initial_offset"]:
            assert stopped == case["name"].endswith("_to_eof"), case["name"]


@pytest.mark.gpu
def test_device_log_read_large_and_capacity(lvkv, gpu):
    # A synthetic 20k-record log with fragmented records across blocks and
    # random damage: device ReadRecord = the oracle's; too-small capacities
    # are reported with exact counts.
    import torch
    import log_synth
    rng = np.random.default_rng(7)
    base = log_synth.build_log(20000, seed=11, max_len=2000, big_every=97)
    for trial in range(6):
        img = bytearray(base)
        for _ in range(trial * 3):
            img[int(rng.integers(0, len(img)))] ^= int(rng.integers(1, 256))
        if trial % 2:  # retyped headers under fixed CRCs (types 0..7)
            hdrs0 = lw.block_verdicts(base).hdrs
            for h in rng.choice(hdrs0, 12, replace=False):
                img[int(h) + 6] = int(rng.integers(0, 8))
                log_synth.fix_header_crc(img, int(h))
        if trial == 5:  # a kEof-type header early on: nothing after it is read
            h = int(lw.block_verdicts(base).hdrs[1500])
            img[h + 6] = 5
            log_synth.fix_header_crc(img, h)
        img = bytes(img)
        buf = torch.from_numpy(np.frombuffer(img, dtype=np.uint8).copy()).to(gpu)
        rd, records, reports, phys, gathered = lvkv.log_read(buf, gather=True)
        hdrs = [int(x) for x in phys[1].cpu().numpy()]
        want_recs, want_reps = lw.read_records(img)
        assert _device_log_records(img, records, hdrs, gathered) == want_recs, trial
        assert reports == want_reps, trial
        assert rd["bytes"] == sum(r[1] for r in want_recs), trial
        # from initial offsets: block starts (resync), the trailer rule,
        # inside fragmented records, past the end
        offs = [32768 * 3, 32768 * 7 - 5, 32768 * 7 - 6, len(img), len(img) + 40000]
        offs += [int(h) + d for h in rng.choice(hdrs, 4, replace=False) for d in (0, 1)]
        offs += [int(x) for x in rng.integers(1, len(img), 3)]
        for off in offs:
            rd, records, reports, phys, gathered = lvkv.log_read(buf, initial_offset=off,
                                                                 gather=True)
            o_recs, o_reps, stopped = lw.read_all(img, off)
            assert _device_log_records(img, records, hdrs, gathered) == o_recs, (trial, off)
            assert reports == o_reps, (trial, off)
            assert rd["stopped"] == int(stopped), (trial, off)
            assert rd["bytes"] == sum(r[1] for r in o_recs), (trial, off)
    rd, records, reports, _, gathered = lvkv.log_read(buf, record_capacity=5, report_capacity=1,
                                                      gather=True)
    assert rd["status"] == 1 and rd["nrecords"] == len(want_recs)
    assert rd["nreports"] == len(want_reps) and len(records) == 5
    # the first five records' bytes are still gathered
    assert _device_log_records(img, records, hdrs, gathered) == want_recs[:5]


@pytest.mark.gpu
def test_device_log_read_dense_blocks(lvkv, gpu):
    """Blocks of hundreds of tiny records (over a thousand items a block, so
    ReadRecord's 256-item workgroups fall many to a block), fragmented
    records between them (big_every), damage, initial offsets."""
    import torch
    import log_synth
    rng = np.random.default_rng(3)
    base = log_synth.build_log(60_000, seed=5, max_len=40, big_every=1999)
    for trial in range(3):
        img = bytearray(base)
        for _ in range(trial * 4):
            img[int(rng.integers(0, len(img)))] ^= int(rng.integers(1, 256))
        img = bytes(img)
        buf = torch.from_numpy(np.frombuffer(img, dtype=np.uint8).copy()).to(gpu)
        for off in [0, 32768 * 2 + 100, int(rng.integers(1, len(img)))]:
            rd, records, reports, phys, gathered = lvkv.log_read(buf, initial_offset=off,
                                                                 gather=True)
            hdrs = [int(x) for x in phys[1].cpu().numpy()]
            o_recs, o_reps, stopped = lw.read_all(img, off)
            assert rd["status"] == 0, (trial, off)
            assert _device_log_records(img, records, hdrs, gathered) == o_recs, (trial, off)
            assert reports == o_reps, (trial, off)
            assert rd["stopped"] == int(stopped), (trial, off)
            assert rd["bytes"] == sum(r[1] for r in o_recs), (trial, off)


def _windowed_log(target_items: int, seed: int, window: int = 64 * 256):
    """Tiny records, plus a 100 KB record (FIRST, MIDDLEs, LAST over four
    blocks) whose fragments straddle every multiple of `window` ReadRecord
    items (one item per physical record and one per block, in file order)."""
    import log_synth
    rng = np.random.default_rng(seed)
    w = log_synth.LogWriter()
    emitted = [0]
    emit = w.emit

    def counted(rtype, payload):
        emitted[0] += 1
        emit(rtype, payload)
    w.emit = counted
    nxt = window - 3
    while emitted[0] + len(w.buf) // 32768 < target_items:
        if emitted[0] + len(w.buf) // 32768 >= nxt:
            w.add_record(rng.integers(0, 256, 100_000, dtype=np.uint8).tobytes())
            nxt += window
        else:
            w.add_record(rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8).tobytes())
    return bytes(w.buf)


@pytest.mark.gpu
def test_device_log_read_scanned_windows(lvkv, gpu):
    """Over 1,024 ReadRecord workgroups (> 262k items) the emit launch takes
    its window's prefix from log_asm_scan instead of folding every earlier
    aggregate: fragmented records across every 64-workgroup
    window boundary, damage (a flipped byte, a retyped header, a kEof-type
    header late in the log), and initial offsets inside and between those
    records, each against the oracle's log::Reader."""
    import torch
    import log_synth
    rng = np.random.default_rng(17)
    base = _windowed_log(300_000, seed=19)
    hdrs0 = lw.block_verdicts(base).hdrs
    assert len(hdrs0) + len(base) // 32768 > 262_144
    big = [off for off, n, _ in lw.read_records(base)[0] if n == 100_000]  # their FIRSTs
    assert len(big) >= 17
    for trial in range(3):
        img = bytearray(base)
        if trial >= 1:
            for _ in range(6):
                img[int(rng.integers(0, len(img)))] ^= int(rng.integers(1, 256))
            h = big[5] + 7 + 32768  # inside a MIDDLE
            img[h] ^= 0x11
            for h in rng.choice(hdrs0, 8, replace=False):
                img[int(h) + 6] = int(rng.integers(0, 8))
                log_synth.fix_header_crc(img, int(h))
        if trial == 2:
            h = int(hdrs0[len(hdrs0) - 5000])
            img[h + 6] = 5
            log_synth.fix_header_crc(img, h)
        img = bytes(img)
        buf = torch.from_numpy(np.frombuffer(img, dtype=np.uint8).copy()).to(gpu)
        offs = [0, big[3] + 1, big[9] + 40_000, (big[12] // 32768) * 32768 + 32768,
                int(rng.integers(1, len(img)))]
        for off in offs:
            rd, records, reports, phys, gathered = lvkv.log_read(buf, initial_offset=off,
                                                                 gather=True)
            hdrs = [int(x) for x in phys[1].cpu().numpy()]
            o_recs, o_reps, stopped = lw.read_all(img, off)
            assert rd["status"] == 0, (trial, off)
            assert _device_log_records(img, records, hdrs, gathered) == o_recs, (trial, off)
            assert reports == o_reps, (trial, off)
            assert rd["stopped"] == int(stopped), (trial, off)
            assert rd["bytes"] == sum(r[1] for r in o_recs), (trial, off)


@pytest.mark.gpu
def test_device_log_gather_large_image_default_capacity(lvkv, gpu):
    """A ~650 MB log (a clean 20k-record, 40 MB log padded to whole 32 KiB blocks
    with zeros — zero-type zero-length trailers, skipped silently, as
    log_reader.cc:234-240 has them — tiled 16 times) read and gathered with
    the default capacities (size // 7 + blocks candidates): the gather's copy
    grid is bounded (a grid sized by that capacity passed 2^32 work-items
    above ~470 MB), and every record's bytes are exact."""
    import torch
    import log_synth
    base = log_synth.build_log(20000, seed=23, max_len=2000, big_every=97)
    base += bytes(-len(base) % 32768)
    b_recs, b_reps = lw.read_records(base)
    assert not b_reps
    hdrs_b = lw.block_verdicts(base).hdrs
    at = {h: k for k, h in enumerate(hdrs_b)}
    tiles = 16
    img = base * tiles
    payload_b = []
    for (off, length, _crc) in b_recs:
        # a record's fragments: consecutive headers from its first one
        k = at[off]
        got, parts = 0, []
        while got < length:
            h = hdrs_b[k]
            n = base[h + 4] | base[h + 5] << 8
            parts.append(base[h + 7: h + 7 + n])
            got += n
            k += 1
        payload_b.append(b"".join(parts))
    want_payload = b"".join(payload_b) * tiles
    buf = torch.from_numpy(np.frombuffer(img, dtype=np.uint8)).to(gpu)
    rd, records, reports, _, (payload, pos) = lvkv.log_read(buf, gather=True)
    torch.cuda.synchronize()
    assert rd["status"] == 0 and not reports
    assert rd["nrecords"] == len(b_recs) * tiles
    assert rd["bytes"] == len(want_payload)
    want_offs = [t * len(base) + r[0] for t in range(tiles) for r in b_recs]
    assert [r[0] for r in records] == want_offs
    assert payload[:len(want_payload)].cpu().numpy().tobytes() == want_payload
    starts = np.cumsum([0] + [len(p) for p in payload_b] * tiles)[:-1]
    assert np.array_equal(pos.cpu().numpy(), starts)
