"""Helpers for the reference-run damage fixtures (tests/golden/damage_*.json,
written by oracle/gen_damage.cc from the reference's own Table::Open,
ReadBlock, Block::Iter, ReadMeta steps and log::Reader). Test code only."""
from __future__ import annotations

import json

from conftest import GOLDEN

# ReadBlock / Footer / BlockHandle status strings -> LVKV_BLOCK_*
BLOCK_OF = {
    "OK": 0,
    "Corruption: block checksum mismatch": 1,
    "Corruption: truncated block read": 2,
    "Corruption: bad block type": 3,
    "Corruption: bad block handle": 4,
    "Corruption: corrupted snappy compressed block length": 6,
    "Corruption: corrupted zstd compressed block length": 6,
}
# Table::Open / footer failures -> LVKV_SST_*
FOOTER_OF = {
    "Corruption: file is too short to be an sstable": 1,
    "Corruption: not an sstable (bad magic number)": 2,
    "Corruption: bad block handle": 3,
}
INDEX_SST_OF = {1: 5, 2: 4, 3: 6, 6: 6}  # index ReadBlock verdict -> LVKV_SST_*
NOT_READ = 7
U64_MAX = (1 << 64) - 1


def sst_cases():
    return json.loads((GOLDEN / "damage_sst.json").read_text())["cases"]


def wal_cases():
    return json.loads((GOLDEN / "damage_wal.json").read_text())["cases"]


def image(case, golden_name="table.sst") -> bytes:
    img = bytearray((GOLDEN / case.get("base", golden_name)).read_bytes())
    for off, hx in case["patches"]:
        b = bytes.fromhex(hx)
        img[off: off + len(b)] = b
    return bytes(img[: case["truncate_to"]])


def sst_expected(case) -> dict:
    """What the device report / oracle must say for this case: status,
    index / meta verdicts, has_filter and the per-entry (offset, size,
    status) list (data blocks, then the filter block)."""
    if case["footer"] != "OK":
        return {"status": FOOTER_OF[case["footer"]], "index_status": NOT_READ,
                "meta_status": NOT_READ, "has_filter": 0, "entries": []}
    idx = BLOCK_OF[case["index"]]
    exp = {"index_status": idx, "meta_status": BLOCK_OF[case["meta"]],
           "has_filter": int(case.get("filter_found", False)), "entries": []}
    if idx != 0:
        exp["status"] = INDEX_SST_OF[idx]
        exp["has_filter"] = 0
        return exp
    exp["status"] = 0 if case["index_iter"] == "OK" else 7
    ents = [(o, s, BLOCK_OF[t]) for o, s, t in case["entries"]]
    if case.get("filter_found"):
        o, s, t = case["filter"]
        ents.append((o, s, BLOCK_OF[t]))
    exp["entries"] = ents
    return exp


def readable(off: int, size: int, status: int) -> bool:
    """Entries whose handle the report keeps (others come back as 0/0)."""
    return status in (0, 1, 3, 6) and size != U64_MAX


def wal_expected(case):
    recs = [tuple(r) for r in case["records"]]
    reps = [(b, r.replace("Corruption: ", "")) for b, r in case["reports"]]
    return recs, reps
