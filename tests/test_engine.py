"""The AQL engine (lvkv_engine_*, include/lvkv_crc32c.h) against the oracle
and the HIP launch path: same contract as lvkv_crc32c_uniform_device for
blocks of 4..4096 bytes, over batches of one and of several dispatches,
overlapped and ordered, with init/mask, and its profiling log."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng(lvkv, gpu):
    e = lvkv.Engine(gpu)
    yield e
    e.close()


def _data(torch, gpu, n, seed):
    g = torch.Generator(device=gpu).manual_seed(seed)
    return torch.randint(0, 256, (n,), dtype=torch.uint8, device=gpu, generator=g)


@pytest.mark.parametrize("nblocks,length,stride", [
    (1, 4096, 4096), (2, 4096, 4096), (3, 4096, 4096), (10_000, 4096, 4096),
    (10_241, 4096, 4096), (25_000, 4096, 4096), (777, 4, 4), (500, 100, 104),
    (4000, 1024, 1024), (333, 2048, 4096), (100, 260, 260), (64, 3996, 4000)])
def test_engine_matches_oracle(lvkv, oracle, eng, gpu, nblocks, length, stride):
    import torch
    buf = _data(torch, gpu, (nblocks - 1) * stride + length, nblocks * 7 + length)
    got = eng.crc32c_uniform(buf, nblocks, length, stride)
    eng.wait()
    want = oracle.uniform(buf.cpu().numpy(), nblocks, length, stride, threads=8)
    assert np.array_equal(got.cpu().numpy().view(np.uint32), want)
    hip = lvkv.crc32c_uniform(buf, nblocks, length, stride)
    torch.cuda.synchronize()
    assert torch.equal(hip, got)


def test_engine_init_mask_ordered(lvkv, oracle, eng, gpu):
    import torch
    nb, L = 3000, 4096
    buf = _data(torch, gpu, nb * L, 5)
    host = buf.cpu().numpy()
    a = eng.crc32c_uniform(buf, nb, L, init=0xDEADBEEF, mask=True)
    b = eng.crc32c_uniform(buf, nb, L, ordered=True)
    eng.wait()
    want = oracle.uniform(host, nb, L, threads=8)
    assert np.array_equal(b.cpu().numpy().view(np.uint32), want)
    hip = lvkv.crc32c_uniform(buf, nb, L, init=0xDEADBEEF, mask=True)
    torch.cuda.synchronize()
    assert torch.equal(a, hip)


def test_engine_kernarg_cache(oracle, eng, gpu):
    """Batches with the same arguments reuse the cached kernel-argument copy
    (only the pointers are cached: each run reads the blocks as they are
    then); more distinct argument sets than the cache holds, all in flight
    at once, fall back to the ring and stay intact."""
    import torch
    nb, L = 300, 4096
    buf = _data(torch, gpu, nb * L, 41)
    out = torch.zeros(nb, dtype=torch.int32, device=gpu)
    h0, _ = eng.kernarg_cache()
    for rep in range(3):
        eng.crc32c_uniform(buf, nb, L, out=out, fresh=False)
        eng.wait()
        want = oracle.uniform(buf.cpu().numpy(), nb, L, threads=8)
        assert np.array_equal(out.cpu().numpy().view(np.uint32), want), rep
        buf.add_(1)  # new contents under the same pointers
        torch.cuda.synchronize()
    h1, _ = eng.kernarg_cache()
    assert h1 - h0 >= 2
    # 1,200 distinct argument sets (the cache holds 1,024), none waited for
    n, small = 1200, 4
    data = _data(torch, gpu, n * small * L, 43)
    outs = torch.zeros(n * small, dtype=torch.int32, device=gpu)
    for i in range(n):
        eng.crc32c_uniform(data[i * small * L:], small, L, out=outs[i * small:], fresh=False)
    eng.wait()
    want = oracle.uniform(data.cpu().numpy(), n * small, L, threads=8)
    assert np.array_equal(outs.cpu().numpy().view(np.uint32), want)


def test_engine_many_batches_in_flight(oracle, eng, gpu):
    """More dispatches than kernarg slots between waits: the engine fences
    itself; every batch's result is intact."""
    import torch
    nb, L, K = 64, 4096, 1500
    buf = _data(torch, gpu, 8 * nb * L, 11)
    outs = torch.zeros(K, nb, dtype=torch.int32, device=gpu)
    for k in range(K):
        eng.crc32c_uniform(buf[(k % 8) * nb * L:], nb, L, out=outs[k])
    eng.wait()
    host = buf.cpu().numpy()
    want = [oracle.uniform(host[w * nb * L:(w + 1) * nb * L], nb, L, threads=8) for w in range(8)]
    got = outs.cpu().numpy().view(np.uint32)
    for k in range(K):
        assert np.array_equal(got[k], want[k % 8]), k


def test_engine_queues_and_profile(oracle, eng, gpu):
    import torch
    nb, L = 10_000, 4096
    buf = _data(torch, gpu, nb * L, 3)
    want = oracle.uniform(buf.cpu().numpy(), nb, L, threads=8)
    assert eng.queues() == 3
    for nq in (1, 2, 4, 3):
        assert eng.queues(nq) == nq
        out = eng.crc32c_uniform(buf, nb, L)
        eng.wait()
        assert np.array_equal(out.cpu().numpy().view(np.uint32), want)
    eng.profile(True)
    for _ in range(5):
        eng.crc32c_uniform(buf, nb, L, ordered=True)
    eng.wait()
    spans = eng.profile_read()
    eng.profile(False)
    assert len(spans) == 5
    for (a, b), (c, _) in zip(spans, spans[1:]):
        assert 0.5 < b - a < 1000.0   # us
        assert c >= b - 1e-3          # ordered: one after the other
    assert eng.profile_read() == []


def test_engine_rejects_bad_arguments(lvkv, eng, gpu):
    """Null pointers are LVKV_ERR_INVALID; an empty batch is a no-op. (Every
    block shape is accepted: the burst kernel's 16-row, end-aligned blocks go
    to it, the rest to the general walk, tests/test_engine_general.py.)"""
    import ctypes

    import torch
    buf = _data(torch, gpu, 1 << 16, 1)
    L = lvkv.lib
    vp = ctypes.c_void_p
    assert L.lvkv_engine_crc32c_uniform(eng.handle, vp(buf.data_ptr()), 4096, 4096, 0, None,
                                        2, 0) == -1
    assert L.lvkv_engine_crc32c_uniform(eng.handle, None, 4096, 4096, 0, vp(buf.data_ptr()),
                                        2, 0) == -1
    assert L.lvkv_engine_crc32c_batch(eng.handle, vp(buf.data_ptr()), None, None, None, 0,
                                      vp(buf.data_ptr()), 2, 0) == -1
    assert L.lvkv_engine_sst_verify(None, None, None, None, None, None, 1, 0) == -1
    out = eng.crc32c_uniform(buf, 0, 4096)
    assert out.numel() == 0


def test_engine_reads_a_reused_buffer_after_a_host_copy(oracle, eng, gpu):
    """A buffer the device has read, overwritten by a host-to-device copy,
    checksummed again with LVKV_FLAG_SYSTEM_ACQUIRE (the wrapper's default):
    the new bytes, not lines left in the L2."""
    import torch
    nb, L = 2000, 4096
    buf = _data(torch, gpu, nb * L, 21)
    first = eng.crc32c_uniform(buf, nb, L, fresh=False)
    eng.wait()
    host = np.random.default_rng(5).integers(0, 256, nb * L, dtype=np.uint8)
    buf.copy_(torch.from_numpy(host))
    torch.cuda.synchronize()
    again = eng.crc32c_uniform(buf, nb, L)  # fresh=True
    eng.wait()
    assert np.array_equal(again.cpu().numpy().view(np.uint32),
                          oracle.uniform(host, nb, L, threads=8))
    assert not torch.equal(first, again)


def test_engine_wait_gives_up_on_a_stuck_queue(lvkv, gpu):
    """The no-hang contract (SURVEY.md §8(b) Errors): queues blocked behind a
    packet that never completes (lvkv_debug_engine_stall, as a faulted or
    endless dispatch would block them) make wait() return LVKV_ERR_HIP after
    the stuck timeout instead of spinning forever; the engine then refuses
    work, and closes cleanly once the queues drain."""
    import time

    import torch
    e = lvkv.Engine(gpu)
    try:
        buf = _data(torch, gpu, 64 * 4096, 11)
        assert lvkv.lib.lvkv_debug_engine_stall(e.handle, 1, 1.0) == 0
        e.crc32c_uniform(buf, 64, 4096)  # queued behind the stall
        t0 = time.perf_counter()
        with pytest.raises(lvkv.LvkvError):
            e.wait()
        assert 0.9 < time.perf_counter() - t0 < 30
        with pytest.raises(lvkv.LvkvError):
            e.crc32c_uniform(buf, 64, 4096)
    finally:
        lvkv.lib.lvkv_debug_engine_stall(e.handle, 0, 60.0)
        time.sleep(0.2)
        e._inflight.clear()
        e.close()


# ---- config 4 / 5 scale (db_bench_new.cc:782-799 as a
# batch): the paths behind bench.py's `split` figure, checked block for block

def _oracle_threads():
    import os
    return max(1, min(16, len(os.sched_getaffinity(0))))


def test_engine_1m_blocks_overlapped_and_ordered(lvkv, oracle, eng, gpu):
    """Config 4: ONE submit of 1M x 4 KiB (4.1 GB, ~98 dispatches rotating
    over the queues), overlapped and then LVKV_FLAG_ORDERED; every block
    against the oracle. Ordered: all of the batch's dispatches on one queue,
    one after another (profiled start/end never overlap)."""
    import torch
    nb, L = 1_000_000, 4096
    buf = _data(torch, gpu, nb * L, 0x1EDC6F41 + 4)
    host = buf.cpu().numpy()
    want = oracle.uniform(host, nb, L, threads=_oracle_threads())
    del host
    _, chains, groups = eng.shape()
    over = eng.crc32c_uniform(buf, nb, L, fresh=False)
    eng.wait()
    assert np.array_equal(over.cpu().numpy().view(np.uint32), want)
    eng.profile(True)
    ordered = eng.crc32c_uniform(buf, nb, L, fresh=False, ordered=True)
    eng.wait()
    spans = eng.profile_read()
    eng.profile(False)
    assert np.array_equal(ordered.cpu().numpy().view(np.uint32), want)
    assert len(spans) > 1  # several dispatches
    for (a, b), (c, _) in zip(spans, spans[1:]):
        assert c >= b - 1e-3, "dispatches of one ordered batch overlapped"


def test_engine_config3_wal_blocks_at_surveyed_size(lvkv, oracle, eng, gpu):
    """Config 3 at its surveyed size: 16,384 log blocks of
    32 KiB (512 MiB, beyond the 256 MiB Infinity Cache), each CRC over bytes
    [6, 32768) -- type + 32761-byte payload, what log::Reader checks
    (db/log_reader.cc:243-247; kBlockSize / kHeaderSize, db/log_format.h:27,30)
    -- built as `bench.py --config wal32k` builds them (make_buffers, base + 6,
    stride 32768) and submitted through lvkv_engine_crc32c_uniform, overlapped
    and then LVKV_FLAG_ORDERED; every CRC against the oracle."""
    import torch

    import bench
    nb, L, stride, crc_off, _ = bench.CONFIGS["wal32k"]
    assert (nb, L, stride, crc_off) == (16_384, 32762, 32768, 6)
    buf, nrot, window = bench.make_buffers(torch, gpu, 0, nb, stride, 0)
    assert nrot == 1 and window == 512 << 20
    torch.cuda.synchronize()
    host = buf.cpu().numpy()
    want = oracle.uniform(host[crc_off:], nb, L, stride, threads=_oracle_threads())
    del host
    over = eng.crc32c_uniform(buf[crc_off:], nb, L, stride, fresh=False)
    eng.wait()
    assert np.array_equal(over.cpu().numpy().view(np.uint32), want)
    ordered = eng.crc32c_uniform(buf[crc_off:], nb, L, stride, fresh=False, ordered=True,
                                 mask=True)
    eng.wait()
    want_masked = np.array([oracle.mask(int(c)) for c in want], dtype=np.uint32)
    assert np.array_equal(ordered.cpu().numpy().view(np.uint32), want_masked)


def test_engine_config5_slice_as_bench_builds_it(lvkv, oracle, eng, gpu):
    """Config 5: rank 3 of 8's slice of the 1M-block batch (125,000 blocks
    at a non-zero start), built by bench.py's own _split_runner (which checks
    window 0 block for block), then every rotation window stepped through the
    engine and compared in full."""
    import torch

    import bench
    shard = bench._load_shard()
    start, count = shard.shard_range(bench.SPLIT_TOTAL, 3, 8)
    assert start > 0 and count == 125_000
    r = bench._split_runner(torch, lvkv, eng, gpu, 3, start, count)
    assert r.nrot >= 2
    for i in range(1, r.nrot + 1):
        r.step(i)
        r.finish()
        r.sync()
        w = i % r.nrot
        host = r.buf[w * count * 4096:(w + 1) * count * 4096].cpu().numpy()
        want = oracle.uniform(host, count, 4096, threads=_oracle_threads())
        got = r.outs_t[i % len(r.outs_t)].cpu().numpy().view(np.uint32)
        assert np.array_equal(got, want), i
    del r


def test_bench_parity_check_catches_a_wrong_block(lvkv, oracle, gpu):
    """bench.parity_check compares every block, not a prefix: a wrong CRC at
    the last block of a slice fails it."""
    import torch

    import bench
    nb, L = 50_000, 4096
    buf = _data(torch, gpu, nb * L, 77)
    out = lvkv.crc32c_uniform(buf, nb, L)
    torch.cuda.synchronize()
    assert bench.parity_check(buf, out, nb, L, L, 0, 0, "test", chunk=8192) == nb
    out[nb - 1] ^= 1
    with pytest.raises(SystemExit, match="block 49999"):
        bench.parity_check(buf, out, nb, L, L, 0, 0, "test", chunk=8192)


@pytest.mark.parametrize("nq,finals", [(3, 3), (3, 1), (1, 1), (4, 2)])
def test_engine_final_flag_fence(lvkv, oracle, eng, gpu, nq, finals):
    """LVKV_FLAG_FINAL on the last `finals` submits before a wait: queues
    whose last dispatch is FINAL are fenced by its own completion (system
    release), the others by barrier packets; every result is intact and
    visible after wait(), for any mix, over several rounds."""
    import torch
    nb, L, K = 3000, 4096, 12
    buf = _data(torch, gpu, 6 * nb * L, 31)
    host = buf.cpu().numpy()
    want = [oracle.uniform(host[w * nb * L:(w + 1) * nb * L], nb, L, threads=8) for w in range(6)]
    assert eng.queues(nq) == nq
    try:
        for rnd in range(3):
            outs = torch.zeros(K, nb, dtype=torch.int32, device=gpu)
            for k in range(K):
                w = (k + rnd) % 6
                eng.crc32c_uniform(buf[w * nb * L:], nb, L, out=outs[k], fresh=False,
                                   final=k >= K - finals)
            eng.wait()
            got = outs.cpu().numpy().view(np.uint32)
            for k in range(K):
                assert np.array_equal(got[k], want[(k + rnd) % 6]), (rnd, k)
    finally:
        eng.queues(3)
