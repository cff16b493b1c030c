"""Link-level drop-in (CPU, needs /root/reference — this container only).

The reference's own callers — TableBuilder::WriteRawBlock, ReadBlock,
log::Writer, log::Reader (+ everything they pull in) — are compiled in place
and linked against liblvkv_crc32c.so in two ways, then rerun the fixture
generator; the SST, WAL and every vector must come out byte-identical to the
fixtures the reference produced with its own util/crc32c.cc:

* linktest: util/crc32c.cc removed; leveldb::crc32c::Extend comes from the
  shim (the callers link unchanged).
* hooktest: stock util/crc32c.cc built with HAVE_CRC32C=1 against
  include/crc32c/crc32c.h, so port::AcceleratedCRC32C (port_stdcxx.h:208-210)
  binds to the library and passes CanAccelerateCRC32C.
"""
from __future__ import annotations

import subprocess
from pathlib import Path

import pytest

from conftest import GOLDEN, REPO

REFERENCE = Path("/root/reference")
FILES = ["kat.json", "corpus.json", "blocks1000_crc.bin", "table.sst",
         "table_blocks.json", "wal.log", "wal_records.json"]

pytestmark = pytest.mark.skipif(not REFERENCE.is_dir(), reason="reference tree not present")


@pytest.mark.parametrize("target", ["linktest", "hooktest"])
def test_reference_callers_linked_against_library(target, lvkv):
    subprocess.run(["make", "-s", "-C", str(REPO / "oracle"), target], check=True,
                   capture_output=True, timeout=600)
    out = REPO / "oracle" / "_ref" / target
    for f in FILES:
        assert (out / f).read_bytes() == (GOLDEN / f).read_bytes(), f
    if target == "linktest":
        nm = subprocess.run(["nm", str(REPO / "oracle" / "_ref" / "gen_golden_lvkv")],
                            capture_output=True, text=True, check=True).stdout
        # Extend is imported, not defined: it comes from the library.
        assert " U _ZN7leveldb6crc32c6ExtendEjPKcm" in nm
