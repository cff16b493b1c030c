"""The bytes db_bench compresses (synthetic workload, not the product).

db_bench's snappycomp / snappyuncomp (benchmarks/db_bench.cc:384-433)
compress one Options().block_size (4096-byte) slice of RandomGenerator's
data (db_bench.cc:174-203): 1 MiB of 100-byte pieces from
test::CompressibleString(&rnd, FLAGS_compression_ratio = 0.5, 100)
(util/testutil.cc:14-48), rnd = leveldb::Random(301) (util/random.h). This
restates those generators so the device codec runs on the same bytes.
"""
from __future__ import annotations

import numpy as np


class Random:
    """leveldb::Random (util/random.h): Park-Miller, seed_ = seed & 0x7fffffff."""

    def __init__(self, s: int):
        self.seed = s & 0x7FFFFFFF
        if self.seed in (0, 2147483647):
            self.seed = 1

    def next(self) -> int:
        M, A = 2147483647, 16807
        product = self.seed * A
        self.seed = (product >> 31) + (product & M)
        if self.seed > M:
            self.seed -= M
        return self.seed

    def uniform(self, n: int) -> int:
        return self.next() % n


def compressible_string(rnd: Random, fraction: float, length: int) -> bytes:
    raw = max(1, int(length * fraction))
    piece = bytes(32 + rnd.uniform(95) for _ in range(raw))
    return (piece * (length // raw + 1))[:length]


def random_generator_data(ratio: float = 0.5, size: int = 1 << 20) -> bytes:
    """RandomGenerator::data_ (db_bench.cc:180-193)."""
    rnd = Random(301)
    out = bytearray()
    while len(out) < size:
        out += compressible_string(rnd, ratio, 100)
    return bytes(out)


def block_batch(nblocks: int, block: int = 4096, ratio: float = 0.5) -> np.ndarray:
    """nblocks consecutive Generate(block) slices (db_bench.cc:195-202),
    as one uint8 array of nblocks * block bytes."""
    data = random_generator_data(ratio)
    out = np.empty(nblocks * block, dtype=np.uint8)
    src = np.frombuffer(data, dtype=np.uint8)
    pos = 0
    for i in range(nblocks):
        if pos + block > len(data):
            pos = 0
        out[i * block:(i + 1) * block] = src[pos:pos + block]
        pos += block
    return out
