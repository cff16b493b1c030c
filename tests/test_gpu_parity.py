"""GPU parity: the gfx950 kernel through the C-ABI vs the oracle, bit-exact.

Covers the reference's fixtures (KAT corpus, 1000 x 4 KiB, a real SST and a
real WAL written by the reference), ragged lengths 0..70000 at every
alignment with random inits, the BASELINE configs (2: 1k x 4 KiB, 3: 32 KiB
WAL blocks misaligned by 2, 4: 1M x 4 KiB over > 4 GiB of device memory),
mask/verify variants, corruption detection (log_test ChecksumMismatch,
corruption_test TableFile) and the host-staged pipeline.
"""
from __future__ import annotations

import numpy as np
import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


def _to_dev(torch, arr, dev, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(arr))
    if dtype is not None:
        t = t.view(dtype)
    return t.to(dev)


def _u32(t):
    return t.cpu().numpy().view(np.uint32)


def test_corpus_fixture_on_gpu(lvkv, golden, corpus_buf, gpu):
    import torch
    spec = golden("corpus.json")
    pad = 256  # base of the device buffer is 256-aligned: offset o => misalignment o % 4
    mem = np.concatenate([np.zeros(pad, np.uint8), corpus_buf])
    ent = np.array(spec["entries"], dtype=np.uint64)
    offs = (ent[:, 1] + pad).astype(np.int64)
    lens = ent[:, 0].astype(np.uint32)
    inits = ent[:, 2].astype(np.uint32)
    got = lvkv.crc32c_batch(_to_dev(torch, mem, gpu), _to_dev(torch, offs, gpu),
                            _to_dev(torch, lens.view(np.int32), gpu),
                            inits=_to_dev(torch, inits.view(np.int32), gpu))
    assert np.array_equal(_u32(got), ent[:, 3].astype(np.uint32))


def test_config2_blocks1000(lvkv, golden, oracle, gpu):
    import torch
    want = golden("blocks1000_crc.bin").view("<u4")
    data = oracle.splitmix_bytes(0x1EDC6F41 + 2, 1000 * 4096)
    d = _to_dev(torch, data, gpu)
    got = lvkv.crc32c_uniform(d, 1000, 4096)
    assert np.array_equal(_u32(got), want)
    gm = lvkv.crc32c_uniform(d, 1000, 4096, mask=True)
    assert np.array_equal(_u32(gm), oracle.uniform(data, 1000, 4096, mask=True))


def test_exhaustive_short_lengths_all_alignments(lvkv, oracle, gpu):
    import torch
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    L = np.repeat(np.arange(0, 1100, dtype=np.uint32), 4)
    a = np.tile(np.arange(4, dtype=np.uint64), 1100)
    offs = (rng.integers(0, 200, L.size).astype(np.uint64) * 4096 + a).astype(np.uint64)
    inits = rng.integers(0, 2**32, L.size, dtype=np.uint64).astype(np.uint32)
    want = oracle.batch(data, offs, L, inits)
    got = lvkv.crc32c_batch(_to_dev(torch, data, gpu), _to_dev(torch, offs.astype(np.int64), gpu),
                            _to_dev(torch, L.view(np.int32), gpu),
                            inits=_to_dev(torch, inits.view(np.int32), gpu))
    bad = np.nonzero(_u32(got) != want)[0]
    assert bad.size == 0, [(int(L[i]), int(offs[i] % 4)) for i in bad[:10]]


def test_ragged_random_long(lvkv, oracle, gpu):
    import torch
    rng = np.random.default_rng(6)
    data = rng.integers(0, 256, 48 << 20, dtype=np.uint8)
    n = 3000
    L = rng.integers(0, 70000, n).astype(np.uint32)
    L[:6] = [65535, 65536, 65537, 32762, 4105, 4106]
    offs = rng.integers(0, data.size - 70000, n).astype(np.uint64)
    inits = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    want = oracle.batch(data, offs, L, inits, threads=8)
    got = lvkv.crc32c_batch(_to_dev(torch, data, gpu), _to_dev(torch, offs.astype(np.int64), gpu),
                            _to_dev(torch, L.view(np.int32), gpu),
                            inits=_to_dev(torch, inits.view(np.int32), gpu))
    assert np.array_equal(_u32(got), want)
    # Same blocks, uniform init and masked output.
    gm = lvkv.crc32c_batch(_to_dev(torch, data, gpu), _to_dev(torch, offs.astype(np.int64), gpu),
                           _to_dev(torch, L.view(np.int32), gpu), init=0x12345678, mask=True)
    wm = oracle.batch(data, offs, L, np.full(n, 0x12345678, np.uint32), mask=True, threads=8)
    assert np.array_equal(_u32(gm), wm)


def test_sst_fixture_verify_and_corruption(lvkv, golden, gpu):
    # table/format.cc:92-99 over a real SST written by the reference.
    import torch
    img = golden("table.sst")
    meta = golden("table_blocks.json")
    offs = np.array([b["offset"] for b in meta["blocks"]], np.int64)
    sizes = np.array([b["size"] for b in meta["blocks"]], np.int32)
    d_img = _to_dev(torch, img, gpu)
    actual, status = lvkv.sst_verify(d_img, _to_dev(torch, offs, gpu), _to_dev(torch, sizes, gpu))
    assert np.array_equal(_u32(actual), np.array([b["crc"] for b in meta["blocks"]], np.uint32))
    assert not status.any().item()
    # corruption_test TableFile: flip a covered byte (contents or type) of
    # some blocks; exactly those report a mismatch.
    bad = img.copy()
    hit = [1, 7, len(offs) - 1]
    for j, i in enumerate(hit):
        pos = int(offs[i]) + (int(sizes[i]) if j == 2 else int(sizes[i]) // 2)  # j==2: the type byte
        bad[pos] ^= 0x40
    _, st = lvkv.sst_verify(_to_dev(torch, bad, gpu), _to_dev(torch, offs, gpu), _to_dev(torch, sizes, gpu))
    assert sorted(np.nonzero(st.cpu().numpy())[0].tolist()) == hit


def test_wal_fixture_verify_and_corruption(lvkv, golden, gpu):
    # db/log_reader.cc:243-257 over a real WAL written by the reference.
    import torch
    img = golden("wal.log")
    recs = golden("wal_records.json")["records"]
    hdr = np.array([r["offset"] for r in recs], np.int64)
    actual, status = lvkv.log_verify(_to_dev(torch, img, gpu), _to_dev(torch, hdr, gpu))
    assert np.array_equal(_u32(actual), np.array([r["crc"] for r in recs], np.uint32))
    assert not status.any().item()
    # log_test ChecksumMismatch / BadRecordType: payload byte and type byte
    # are both inside the CRC.
    bad = img.copy()
    big = [i for i, r in enumerate(recs) if r["length"] > 10]
    bad[recs[big[0]]["offset"] + 7 + 3] ^= 1   # payload
    bad[recs[big[1]]["offset"] + 6] ^= 0x10    # type byte
    _, st = lvkv.log_verify(_to_dev(torch, bad, gpu), _to_dev(torch, hdr, gpu))
    assert sorted(np.nonzero(st.cpu().numpy())[0].tolist()) == sorted([big[0], big[1]])


def test_config3_wal_32k_blocks(lvkv, oracle, gpu):
    # BASELINE config 3: 32 KiB log blocks, each one FULL record of 32761 B
    # payload; CRC domain = bytes [6, 32768) (2-mod-4 misaligned starts).
    import torch
    nblk = 2048  # 64 MiB here; the bench runs the 16384-block (512 MiB) shape
    g = torch.Generator(device=gpu).manual_seed(3)
    d = torch.randint(0, 256, (nblk * 32768,), dtype=torch.uint8, device=gpu, generator=g)
    h = d.cpu().numpy()
    blocks = h.reshape(nblk, 32768)
    blocks[:, 4] = 32761 & 0xFF
    blocks[:, 5] = 32761 >> 8
    blocks[:, 6] = 1  # kFullType
    crcs = oracle.uniform(h[6:], nblk, 32762, stride=32768, threads=8)
    masked = np.array([oracle.mask(int(c)) for c in crcs], dtype="<u4")
    blocks[:, 0:4] = masked.view(np.uint8).reshape(nblk, 4)
    d = torch.from_numpy(h).to(gpu)
    hdr = torch.arange(nblk, dtype=torch.int64, device=gpu) * 32768
    actual, status = lvkv.log_verify(d, hdr)
    assert np.array_equal(_u32(actual), crcs)
    assert not status.any().item()
    got = lvkv.crc32c_uniform(d[6:], nblk, 32762, stride=32768)
    assert np.array_equal(_u32(got), crcs)


def test_config4_1m_blocks_above_4gib(lvkv, oracle, gpu):
    # BASELINE config 4: 1M x 4 KiB (4 GiB) in one device buffer, plus blocks
    # at byte offsets >= 2^32; checked block-for-block against the oracle.
    import torch
    n = 1 << 20
    extra = 1 << 20
    g = torch.Generator(device=gpu).manual_seed(4)
    d = torch.randint(0, 256, (n * 4096 + extra,), dtype=torch.uint8, device=gpu, generator=g)
    got = lvkv.crc32c_uniform(d, n, 4096)
    h = d.cpu().numpy()
    want = oracle.uniform(h, n, 4096, threads=16)
    assert np.array_equal(_u32(got), want)
    del want
    offs = np.array([n * 4096 + 1, (1 << 32) - 3, (1 << 32) + 12345, n * 4096 + extra - 5000], np.uint64)
    lens = np.array([4096, 4105, 32762, 5000], np.uint32)
    got2 = lvkv.crc32c_batch(d, _to_dev(torch, offs.astype(np.int64), gpu), _to_dev(torch, lens.view(np.int32), gpu))
    assert np.array_equal(_u32(got2), oracle.batch(h, offs, lens))


def test_repeat_launches_are_deterministic(lvkv, gpu):
    import torch
    g = torch.Generator(device=gpu).manual_seed(9)
    d = torch.randint(0, 256, (10000 * 4096,), dtype=torch.uint8, device=gpu, generator=g)
    a = lvkv.crc32c_uniform(d, 10000, 4096)
    s = torch.cuda.Stream(gpu)
    with torch.cuda.stream(s):
        b = lvkv.crc32c_uniform(d, 10000, 4096, stream=s)
    s.synchronize()
    assert torch.equal(a, b)


def test_host_pipeline(lvkv, oracle, gpu):
    rng = np.random.default_rng(12)
    data = rng.integers(0, 256, 96 << 20, dtype=np.uint8)
    n = 30000
    L = rng.integers(0, 9000, n).astype(np.uint32)
    offs = rng.integers(0, data.size - 9000, n).astype(np.uint64)
    inits = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    got = lvkv.crc32c_batch_host(data, offs, L, inits=inits)
    assert np.array_equal(got, oracle.batch(data, offs, L, inits, threads=8))
    # > one staging buffer (64 MiB) of 4 KiB blocks, masked
    got = lvkv.crc32c_batch_host(data, np.arange(20000, dtype=np.uint64) * 4096,
                                 np.full(20000, 4096, np.uint32), mask=True)
    assert np.array_equal(got, oracle.uniform(data, 20000, 4096, mask=True, threads=8))


def test_all_zero_and_x_blocks(lvkv, oracle, gpu):
    # db_bench_new.cc:786 hashes a 4 KiB 'x' buffer; RFC zeros/ones too.
    import torch
    for fill in (0x00, 0xFF, ord("x")):
        h = np.full(64 * 4096, fill, np.uint8)
        got = lvkv.crc32c_uniform(torch.from_numpy(h).to(gpu), 64, 4096)
        assert np.array_equal(_u32(got), oracle.uniform(h, 64, 4096))
    z = torch.zeros(64, dtype=torch.uint8, device=gpu)
    assert _u32(lvkv.crc32c_uniform(z, 1, 32))[0] == 0x8A9136AA


@pytest.mark.parametrize("length,nblocks", [
    (4, 5000), (5, 1), (7, 777), (8, 33), (255, 20000), (256, 9000), (257, 4097),
    (259, 300), (1021, 1000), (4093, 2500), (4096, 20000), (4097, 10001), (4100, 123),
    (8188, 700), (32762, 300), (65536, 64), (70001, 50)])
def test_uniform_kernel_shapes(lvkv, oracle, gpu, length, nblocks):
    # The dedicated uniform kernel (block END 4-byte aligned): every residue of
    # length mod 4 (front padding + init spill, incl. the s0l == 63 case at
    # 257), multi-chunk blocks, batches of 1..5 rounds per wave.
    import torch
    stride = (length + 3) // 4 * 4 + 4 * (length % 3)
    pad = (-length) % 4            # base + pad + length is 4-aligned
    nbytes = pad + (nblocks - 1) * stride + length
    g = torch.Generator(device=gpu).manual_seed(length * 31 + nblocks)
    d = torch.randint(0, 256, (nbytes + 64,), dtype=torch.uint8, device=gpu, generator=g)
    init = (length * 2654435761) & 0xFFFFFFFF
    got = lvkv.crc32c_uniform(d[pad:], nblocks, length, stride, init=init, mask=bool(length & 1))
    h = d.cpu().numpy()[pad:]
    want = oracle.uniform(h, nblocks, length, stride, init=init, mask=bool(length & 1), threads=8)
    assert np.array_equal(_u32(got), want)


@pytest.mark.parametrize("length,nblocks,groups", [
    (4, 700, 0), (6, 3000, 64), (255, 12288, 0), (1021, 999, 3), (4093, 48, 1),
    (4096, 10000, 0), (4096, 3 * 16 * 17, 17)])
def test_every_uniform_variant(lvkv, oracle, gpu, length, nblocks, groups):
    # Force each kernel that can serve a uniform end-aligned batch (the general
    # kernel's uniform specialisation, the two-stream uniform kernel loads-first
    # and fill-first, the one-round small kernel both ways) onto the same input
    # and grid; all must match the oracle bit for bit.
    import ctypes
    import torch
    # the alternative schedules are compiled into the probe build only
    L = ctypes.CDLL(str(REPO / "tools" / "probe" / "liblvkv_probe.so"))
    L.lvkv_debug_uniform_variant.argtypes = [
        ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
        ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    L.lvkv_debug_uniform_variant.restype = ctypes.c_int
    stride = (length + 3) // 4 * 4
    pad = (-length) % 4
    g = torch.Generator(device=gpu).manual_seed(length + 7 * nblocks)
    d = torch.randint(0, 256, (pad + nblocks * stride + 64,), dtype=torch.uint8,
                      device=gpu, generator=g)
    want = oracle.uniform(d.cpu().numpy()[pad:], nblocks, length, stride, threads=8)
    waves = 16 * (groups or lvkv.device_groups())
    small_fits = length <= 4096 and nblocks <= 3 * waves
    # compact-LDS kernel shapes (crc32c_compact.hip): (cfg, blocks per group, groups per CU)
    compact = tuple((cfg << 16) | 2048 | 256 for cfg, cap, occ in ((0, 48, 1), (1, 24, 2), (2, 32, 2),
                                                                   (8, 48, 1), (9, 24, 2))
                    if length <= 4096 and nblocks <= cap * (groups or occ * lvkv.device_groups()))
    for variant in ((32, 256, 384) + ((768, 772, 776, 780, 784, 896, 900, 1804) if small_fits else ())
                    + compact):
        out = torch.full((nblocks,), -1, dtype=torch.int32, device=gpu)
        rc = L.lvkv_debug_uniform_variant(variant, groups, d.data_ptr() + pad, stride, length,
                                          out.data_ptr(), nblocks, None)
        assert rc == 0, (variant, rc)
        torch.cuda.synchronize()
        assert np.array_equal(_u32(out), want), variant


def test_long_blocks_split_over_workgroups(lvkv, oracle, gpu):
    # Blocks past kLongBytes (64 KiB) are cut into 16 KiB segments on 4-byte
    # boundaries and combined with Z_{2^j} shifts (crc32c_long_kernel): every
    # start and end alignment, segment-boundary lengths, mixed with short ones.
    import torch
    rng = np.random.default_rng(12)
    data = rng.integers(0, 256, 24 << 20, dtype=np.uint8)
    lens = [65536, 65537, 65538, 65539, 65540, 16384 * 5, 16384 * 5 + 1, 100003,
            (1 << 20) + 1, (3 << 20) + 2, 7, 4096, 70000]
    L = np.array([l for l in lens for _ in range(4)], dtype=np.uint32)
    offs = np.array([rng.integers(0, (data.size - l) // 8) * 4 + k
                     for l in lens for k in range(4)], dtype=np.uint64)
    inits = rng.integers(0, 2**32, L.size, dtype=np.uint64).astype(np.uint32)
    want = oracle.batch(data, offs, L, inits, threads=8)
    got = lvkv.crc32c_batch(_to_dev(torch, data, gpu), _to_dev(torch, offs.astype(np.int64), gpu),
                            _to_dev(torch, L.view(np.int32), gpu),
                            inits=_to_dev(torch, inits.view(np.int32), gpu))
    bad = np.nonzero(_u32(got) != want)[0]
    assert bad.size == 0, [(int(L[i]), int(offs[i] % 4)) for i in bad[:10]]


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", [-1, 0, 1, 2, 3, 4, 7, 8, 16, 24])
def test_general_layout_kernels(lvkv, oracle, gpu, kernel):
    # Every general-layout kernel (crc32c_kernel.hip: -1; crc32c_ragged.hip
    # shapes 0-2) on every start/end alignment, lengths at and around the
    # 16/24/32-row chunk edges, idle chains (batch sizes not a multiple of
    # a round) and blocks up to 64 KiB + a few.
    import torch
    L_ = lvkv.lib
    assert L_.lvkv_debug_set_general_kernel(kernel) == 0
    try:
        rng = np.random.default_rng(40 + kernel)
        data = rng.integers(0, 256, 8 << 20, dtype=np.uint8)
        edges = [r * 256 + d for r in (1, 15, 16, 17, 23, 24, 25, 31, 32, 33, 48, 64, 255, 256)
                 for d in (-4, -3, -2, -1, 0, 1, 2, 3, 4)]
        lens = np.array([0, 1, 2, 3, 4, 5, 7, 8] + edges + [65535, 65536, 65537, 70001],
                        dtype=np.uint32)
        L = np.repeat(lens, 4)
        a = np.tile(np.arange(4, dtype=np.uint64), lens.size)
        offs = (rng.integers(0, (data.size - 80000) // 4096, L.size).astype(np.uint64) * 4096
                + a).astype(np.uint64)
        inits = rng.integers(0, 2**32, L.size, dtype=np.uint64).astype(np.uint32)
        for n in (L.size, 1, 5, 17, 33):
            want = oracle.batch(data, offs[:n], L[:n], inits[:n])
            got = lvkv.crc32c_batch(_to_dev(torch, data, gpu),
                                    _to_dev(torch, offs[:n].astype(np.int64), gpu),
                                    _to_dev(torch, L[:n].view(np.int32), gpu),
                                    inits=_to_dev(torch, inits[:n].view(np.int32), gpu))
            bad = np.nonzero(_u32(got) != want)[0]
            assert bad.size == 0, [(int(L[i]), int(offs[i] % 4)) for i in bad[:10]]
        # many rounds per workgroup: 20k random blocks of 0..9 KiB, masked
        n = 20000
        L2 = rng.integers(0, 9000, n).astype(np.uint32)
        o2 = rng.integers(0, data.size - 9000, n).astype(np.uint64)
        want = oracle.batch(data, o2, L2, np.full(n, 7, np.uint32), mask=True, threads=8)
        got = lvkv.crc32c_batch(_to_dev(torch, data, gpu), _to_dev(torch, o2.astype(np.int64), gpu),
                                _to_dev(torch, L2.view(np.int32), gpu), init=7, mask=True)
        assert np.array_equal(_u32(got), want)
    finally:
        L_.lvkv_debug_set_general_kernel(0)


@pytest.mark.gpu
def test_kat_vectors_through_the_batch_kernels(lvkv, gpu, golden):
    # tests/golden/kat.json (util/crc32c_test.cc's known answers) as one
    # batch: every vector a block with its own init, at every start
    # alignment, through the general-layout kernel; masked values too.
    import torch
    vecs = golden("kat.json")["vectors"]
    blob, offs, lens, inits, want, wmask = bytearray(), [], [], [], [], []
    for a in range(4):
        for v in vecs:
            data = bytes.fromhex(v["hex"])
            blob += b"\0" * ((a - len(blob)) % 8)
            offs.append(len(blob))
            blob += data
            lens.append(len(data))
            inits.append(v["init"])
            want.append(v["crc"])
            wmask.append(v["masked"])
    data = np.frombuffer(bytes(blob) + b"\0" * 64, dtype=np.uint8)
    d = _to_dev(torch, data, gpu)
    o = _to_dev(torch, np.array(offs, np.int64), gpu)
    n = _to_dev(torch, np.array(lens, np.uint32).view(np.int32), gpu)
    i = _to_dev(torch, np.array(inits, np.uint32).view(np.int32), gpu)
    got = lvkv.crc32c_batch(d, o, n, inits=i)
    torch.cuda.synchronize()
    assert _u32(got).tolist() == want
    got_m = lvkv.crc32c_batch(d, o, n, inits=i, mask=True)
    torch.cuda.synchronize()
    assert _u32(got_m).tolist() == wmask
