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
    assert lw.read_records(img) == (recs, reps)
    v = lw.block_verdicts(img)
    ev = lw.events_from_blocks(img, v.hdrs, v.rec_status, v.block_status, v.block_drop)
    assert lw.assemble(img, ev) == (recs, reps)


# ---------------------------------------------------------------- GPU -----

@pytest.mark.gpu
def test_device_sst_matches_reference(lvkv, gpu):
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
        img = df.image(case, "wal.log")
        buf = torch.from_numpy(np.frombuffer(img, dtype=np.uint8).copy()).to(gpu)
        rep, hdr, actual, rst, bst, bdrop = lvkv.log_verify_blocks(buf)
        torch.cuda.synchronize()
        ev = lw.events_from_blocks(img, [int(x) for x in hdr.cpu().numpy()],
                                   list(rst.cpu().numpy()), list(bst.cpu().numpy()),
                                   list(bdrop.cpu().numpy()))
        assert lw.assemble(img, ev) == df.wal_expected(case), case["name"]
