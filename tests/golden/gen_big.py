"""Generates tests/golden/big_{snappy,zstd}.bin + big.json: codec streams of
blocks past the decoders' LDS staging (64 KiB, 256 KiB, 1 MiB: LevelDB's
block_size is a user option, include/leveldb/options.h:101, and ReadBlock
decodes any size, table/format.cc:120-155), written by the libraries the
reference would link (libsnappy 1.1.8; libzstd 1.4.9 through
port::Zstd_Compress's calls at level 1, and ZSTD_compress at level 3).

The inputs are not stored: `inputs()` rebuilds them from db_bench's
generator (tools/db_bench_data.py) and a fixed seed; big.json keeps their
sha256.

    python tests/golden/gen_big.py
"""
from __future__ import annotations

import hashlib
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO))
from tools.db_bench_data import block_batch  # noqa: E402

SIZES = (65536, 65600, 262144, 1 << 20)


def inputs():
    rng = np.random.default_rng(424242)
    bb = block_batch(300).tobytes()  # 1.2 MB of db_bench values
    text = (b"LevelDB is a fast key-value storage library written at Google that provides"
            b" an ordered mapping from string keys to string values. ") * 9000
    out = []
    for n in SIZES:
        out.append(bb[:n])
        out.append(text[7:7 + n])
    a = rng.integers(0, 256, 300000, dtype=np.uint8)  # barely compressible, long literals
    a[::3] = 0
    out.append(a.tobytes())
    return out


def main():
    from oracle import snappy_oracle as so
    from oracle import zstd_encoder as ze
    from oracle import zstd_oracle as zo
    sl, zl = so.system_snappy(), ze.system_zstd_writer()
    if sl is None or zl is None:
        raise SystemExit("libsnappy 1.1.8 / libzstd 1.4.9 not found")
    ins = inputs()
    snap = [so.lib_compress(sl, x) for x in ins]
    zst = []
    for x in ins:
        zst.append(ze.lib_port_compress(zl, x, 1))
        zst.append(zo.lib_compress(zl, x, 3))
    for x, s in zip(ins, snap):
        assert so.uncompress(s) == (so.OK, x)
    blob = {"inputs": [len(x) for x in ins], "sha256_inputs": [hashlib.sha256(x).hexdigest()
                                                              for x in ins],
            "snappy": [len(s) for s in snap], "zstd": [len(z) for z in zst],
            "zstd_levels": [1, 3],
            "source": "libsnappy 1.1.8 RawCompress; libzstd 1.4.9 port::Zstd_Compress(1) "
                      "and ZSTD_compress(3)"}
    (HERE / "big_snappy.bin").write_bytes(b"".join(snap))
    (HERE / "big_zstd.bin").write_bytes(b"".join(zst))
    (HERE / "big.json").write_text(json.dumps(blob, indent=0))
    print(len(ins), "inputs", sum(map(len, ins)), "bytes; snappy", sum(map(len, snap)),
          "zstd", sum(map(len, zst)))


if __name__ == "__main__":
    main()
