"""CPU check of the kernel's decomposition (tests/kernel_model.py) and of the
device tables it uses, against the oracle. No GPU needed."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

from kernel_model import KernelModel


def _zero_adv(v: int, nbytes: int) -> int:
    for _ in range(8 * nbytes):
        v = (v >> 1) ^ (0x82F63B78 if v & 1 else 0)
    return v


@pytest.fixture(scope="module")
def tables(lvkv):
    row = np.zeros(1024, dtype=np.uint32)
    lane = np.zeros(8192, dtype=np.uint32)
    lvkv.lib.lvkv_debug_tables.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lvkv.lib.lvkv_debug_tables.restype = None
    lvkv.lib.lvkv_debug_tables(row.ctypes.data, lane.ctypes.data)
    return row, lane


def test_row_table_is_z256(tables):
    row, _ = tables
    rng = np.random.default_rng(1)
    for t in range(4):
        for i in list(range(4)) + list(rng.integers(0, 256, 6)):
            assert row[t * 256 + i] == _zero_adv(int(i) << (8 * t), 256)


def test_lane_table_is_z_256_minus_4s(tables):
    _, lane = tables
    for s in (0, 1, 31, 32, 63):
        for k in (0, 3, 7):
            for nib in (1, 9, 15):
                assert lane[(k * 16 + nib) * 64 + s] == _zero_adv(nib << (4 * k), 256 - 4 * s)


@pytest.fixture(scope="module")
def model(tables):
    return KernelModel(*tables)


def test_model_matches_oracle_on_corpus(model, oracle, golden, corpus_buf):
    spec = golden("corpus.json")
    mem = np.concatenate([np.zeros(64, np.uint8), corpus_buf, np.zeros(64, np.uint8)])
    for length, off, init, crc in spec["entries"]:
        if length > 9000:
            continue  # long entries are covered by the GPU tests; keep CPU time small
        assert model.block(mem, 64 + off, length, init) == crc, (length, off, init)


def test_model_ragged_random(model, oracle):
    rng = np.random.default_rng(11)
    mem = rng.integers(0, 256, 40000, dtype=np.uint8)
    cases = [(L, a) for L in [4, 5, 6, 7, 8, 252, 253, 255, 256, 257, 259, 260, 1020, 4092,
                               4093, 4094, 4095, 4096, 4100, 4106, 4352, 4353, 8192, 8193]
             for a in range(4)]
    for L, a in cases:
        ptr = 256 + 64 * int(rng.integers(0, 100)) + a
        init = int(rng.integers(0, 2**32))
        want = oracle.extend(init, mem[ptr:ptr + L].tobytes())
        assert model.block(mem, ptr, L, init) == want, (L, a)


def test_model_tiny(model, oracle):
    mem = np.arange(64, dtype=np.uint8)
    for L in range(4):
        for a in range(4):
            for init in (0, 0xFFFFFFFF, 0x12345678):
                assert model.block(mem, 8 + a, L, init) == oracle.extend(init, mem[8 + a:8 + a + L].tobytes())
