"""Generates tests/golden/snappy_{inputs,streams,damaged}.bin + snappy.json
from libsnappy 1.1.8 (/opt/conda/lib, the snappy this image carries; the
reference leaves Snappy to that library, port/port_stdcxx.h:90-133).

    python tests/golden/gen_snappy.py

inputs  : the edge sizes of the format (empty, < 15 bytes with no match
          search, the 60-byte literal-tag boundary, copies of 4/11/12/64/65/
          67/68 bytes, offsets across 2048, whole 64 KiB fragments and more),
          random and repetitive bytes, and db_bench's 4 KiB blocks
          (tools/db_bench_data.py);
streams : libsnappy's RawCompress of each input;
damaged : streams with bytes flipped, cut or extended, with libsnappy's
          verdict (0 ok, 1 bad length, 2 bad contents) and, when it
          decodes, the sha256 of what it decodes to.
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
from oracle import snappy_oracle as so  # noqa: E402
from tools.db_bench_data import block_batch  # noqa: E402


def inputs():
    rng = np.random.default_rng(20260501)
    out = []
    for n in (0, 1, 2, 3, 4, 5, 14, 15, 16, 17, 20, 59, 60, 61, 62, 63, 64, 65, 100, 255, 256,
              257, 1000):
        out.append(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
    for n in (15, 16, 17, 18, 30, 64, 65, 67, 68, 69, 75, 128, 1000, 5000):
        out.append(b"a" * n)
    out.append(b"ab" * 3000)
    for L in (4, 5, 11, 12, 13, 63, 64, 65, 66, 67, 68, 69, 70, 131, 132):
        pat = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        gap = rng.integers(0, 256, 37, dtype=np.uint8).tobytes()
        out.append(gap + pat + gap[:5] + pat + gap)
    for off in (2000, 2047, 2048, 2049, 4000, 40000, 65000):
        pat = rng.integers(0, 256, 40, dtype=np.uint8).tobytes()
        mid = rng.integers(0, 256, off - 40, dtype=np.uint8).tobytes()
        out.append(pat + mid + pat + b"tail-bytes-here-xx")
    text = (b"LevelDB is a fast key-value storage library written at Google that provides"
            b" an ordered mapping from string keys to string values. ")
    for n in (4096, 65535, 65536, 65537, 70000, 140000):
        out.append((text * (n // len(text) + 1))[:n])
    lo = rng.integers(0, 4, 70000, dtype=np.uint8)
    out.append(lo.tobytes())
    out.append(rng.integers(0, 256, 65536 + 100, dtype=np.uint8).tobytes())
    blocks = block_batch(24)
    for i in range(24):
        out.append(blocks[i * 4096:(i + 1) * 4096].tobytes())
    for ratio in (0.1, 0.25, 0.9, 1.0):
        out.append(block_batch(1, 4096, ratio).tobytes())
    # key/value entries in a block (shared key prefixes, 16-byte keys)
    ent = bytearray()
    for i in range(150):
        ent += bytes([8, 8, 10]) + f"{i:08d}".encode() + rng.integers(0, 256, 10, dtype=np.uint8).tobytes()
    out.append(bytes(ent))
    return out


def damaged(streams):
    rng = np.random.default_rng(77)
    small = [s for s in streams if 0 < len(s) < 6000]
    cases = []
    for k in range(600):
        s = bytearray(small[k % len(small)])
        kind = k % 5
        if kind == 0 and len(s) > 0:
            i = int(rng.integers(0, len(s)))
            s[i] ^= 1 << int(rng.integers(0, 8))
        elif kind == 1:
            s = s[: int(rng.integers(0, len(s) + 1))]
        elif kind == 2:
            s += rng.integers(0, 256, int(rng.integers(1, 9)), dtype=np.uint8).tobytes()
        elif kind == 3 and len(s) > 1:
            i = int(rng.integers(1, len(s)))
            s[i] = int(rng.integers(0, 256))
        else:
            s[0:1] = rng.integers(0, 256, 1, dtype=np.uint8).tobytes()
        cases.append(bytes(s))
    # hand-made: copy-4 elements, padded literal lengths, offset 0
    cases += [bytes([5, 0x10]) + b"abcde",          # literal, length 5
              bytes([5, 0xF0, 4]) + b"abcde",       # literal, 1-byte length field
              bytes([5, 0xFC, 4, 0, 0, 0]) + b"abcde",
              bytes([8, 0x0C]) + b"abcd" + bytes([0x0F, 4, 0, 0, 0]),   # copy-4 off 4 len 4
              bytes([8, 0x0C]) + b"abcd" + bytes([0x0E, 4, 0]),          # copy-2
              bytes([8, 0x0C]) + b"abcd" + bytes([0x0E, 0, 0]),          # offset 0
              bytes([8, 0x0C]) + b"abcd" + bytes([0x0E, 5, 0]),          # offset past start
              bytes([0xFF, 0xFF, 0xFF, 0xFF, 0x0F]),                     # 2^32 - 1, no data
              bytes([0xFF, 0xFF, 0xFF, 0xFF, 0x10]),                     # varint too long
              bytes([0x80, 0x80, 0x80, 0x80, 0x80, 0x00]),
              bytes([3, 0xFC, 0xFF, 0xFF, 0xFF, 0xFF]) + b"abc",         # literal of 2^32
              bytes([0]), b"", bytes([1]), bytes([2, 0x04]) + b"xy" + bytes([0x00]) + b"z",
              # 4-byte literal length 0xffffffff: + 1 wraps in uint32 to an
              # empty literal (libsnappy decodes this to b"abc", status 0)
              bytes([3, 0xFC, 0xFF, 0xFF, 0xFF, 0xFF, 0x08]) + b"abc"]
    return cases


def main():
    lib = so.system_snappy()
    if lib is None:
        raise SystemExit("libsnappy 1.1.8 not found")
    ins = inputs()
    streams = [so.lib_compress(lib, x) for x in ins]
    dam = damaged(streams)
    verdicts = []
    for d in dam:
        st, out = so.lib_uncompress(lib, d)
        verdicts.append({"status": st, "ulen": len(out),
                         "sha256": hashlib.sha256(out).hexdigest() if st == 0 else None})
    blob = {"inputs": [len(x) for x in ins], "streams": [len(s) for s in streams],
            "damaged": [len(d) for d in dam], "verdicts": verdicts,
            "sha256_inputs": [hashlib.sha256(x).hexdigest() for x in ins],
            "source": "libsnappy 1.1.8 (/opt/conda/lib/libsnappy.so.1.1.8), snappy-c API"}
    (HERE / "snappy_inputs.bin").write_bytes(b"".join(ins))
    (HERE / "snappy_streams.bin").write_bytes(b"".join(streams))
    (HERE / "snappy_damaged.bin").write_bytes(b"".join(dam))
    (HERE / "snappy.json").write_text(json.dumps(blob, indent=0))
    print(len(ins), "inputs", sum(map(len, ins)), "bytes;", len(dam), "damaged")


if __name__ == "__main__":
    main()
