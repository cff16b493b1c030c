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
