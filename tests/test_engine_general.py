"""The engine's general-layout submits (lvkv_engine_crc32c_batch,
lvkv_engine_sst_verify / _log_verify / _sst_fill_trailers /
_log_fill_headers, and lvkv_engine_crc32c_uniform beyond the burst kernel's
shapes) against the oracle and the HIP launch path: the ragged walk
(crc32c_ragged_body.h) dispatched into the engine's queues. Reference:
util/crc32c.cc:276-377, table/format.cc:92-99, table/table_builder.cc:192-209,
db/log_reader.cc:243-247, db/log_writer.cc:82-108."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng(lvkv, gpu):
    e = lvkv.Engine(gpu)
    yield e
    e.close()


def _dev(torch, arr, gpu):
    return torch.from_numpy(np.ascontiguousarray(arr)).to(gpu)


def _u32(t):
    return t.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("ordered,small", [(False, False), (True, False), (False, True)])
def test_engine_batch_ragged_random(lvkv, oracle, eng, gpu, ordered, small):
    """Random offsets (every alignment), lengths 0..70,000 (blocks over
    64 KiB walked by a whole workgroup in the same dispatch, tiny blocks
    bitwise), per-block inits; then uniform init with Mask. `small`: the
    LVKV_FLAG_SMALL_BLOCKS hint (another walk, the same results)."""
    import torch
    rng = np.random.default_rng(41)
    data = rng.integers(0, 256, 48 << 20, dtype=np.uint8)
    n = 5000
    L = rng.integers(0, 9000, n).astype(np.uint32)
    L[::97] = rng.integers(0, 70000, L[::97].size)
    L[:8] = [0, 1, 2, 3, 65535, 65536, 65537, 4106]
    offs = rng.integers(0, data.size - 70000, n).astype(np.uint64)
    inits = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    d = _dev(torch, data, gpu)
    do, dl = _dev(torch, offs.astype(np.int64), gpu), _dev(torch, L.view(np.int32), gpu)
    di = _dev(torch, inits.view(np.int32), gpu)
    got = eng.crc32c_batch(d, do, dl, inits=di, ordered=ordered, small=small)
    gm = eng.crc32c_batch(d, do, dl, init=0x12345678, mask=True, ordered=ordered, small=small)
    eng.wait()
    assert np.array_equal(_u32(got), oracle.batch(data, offs, L, inits, threads=8))
    want_m = oracle.batch(data, offs, L, np.full(n, 0x12345678, np.uint32), mask=True, threads=8)
    assert np.array_equal(_u32(gm), want_m)
    hip = lvkv.crc32c_batch(d, do, dl, inits=di)
    torch.cuda.synchronize()
    assert torch.equal(hip, got)


@pytest.mark.parametrize("nblocks,length,stride,shift", [
    (2, 8192, 8192, 0),        # beyond the burst kernel's 16 rows
    (5, 3, 4, 0),              # < 4 bytes: bitwise
    (7, 8, 8, 1),              # ends not 4-byte aligned
    (333, 4271, 4271, 0),      # SST-sized, odd stride
    (100, 70000, 70001, 3),    # over 64 KiB: whole-workgroup walk
    (512, 32762, 32768, 6),    # config 3's WAL blocks at +6
    (1000, 0, 16, 0),          # empty blocks: Extend(init, "", 0) = init
])
def test_engine_uniform_any_shape(lvkv, oracle, eng, gpu, nblocks, length, stride, shift):
    import torch
    rng = np.random.default_rng(nblocks + length)
    host = rng.integers(0, 256, (nblocks - 1) * stride + length + shift + 8, dtype=np.uint8)
    d = _dev(torch, host, gpu)
    got = eng.crc32c_uniform(d[shift:], nblocks, length, stride, init=0xA5A5A5A5)
    eng.wait()
    want = oracle.uniform(host[shift:], nblocks, length, stride, init=0xA5A5A5A5, threads=8)
    assert np.array_equal(_u32(got), want)


def test_engine_sst_verify_and_fill_golden(lvkv, golden, eng, gpu):
    """The reference-written table (tests/golden/table.sst): verify every
    block (format.cc:92-99), then with covered bytes flipped, then wipe every
    trailer CRC and refill it on the engine (table_builder.cc:192-209): the
    image comes back byte for byte."""
    import torch
    img = golden("table.sst")
    meta = golden("table_blocks.json")
    offs = np.array([b["offset"] for b in meta["blocks"]], np.int64)
    sizes = np.array([b["size"] for b in meta["blocks"]], np.int32)
    do, ds = _dev(torch, offs, gpu), _dev(torch, sizes, gpu)
    actual, status = eng.sst_verify(_dev(torch, img, gpu), do, ds)
    eng.wait()
    assert np.array_equal(_u32(actual), np.array([b["crc"] for b in meta["blocks"]], np.uint32))
    assert not status.any().item()
    bad = img.copy()
    hit = [1, 7, len(offs) - 1]
    for j, i in enumerate(hit):
        bad[int(offs[i]) + (int(sizes[i]) if j == 2 else int(sizes[i]) // 2)] ^= 0x40
    _, st = eng.sst_verify(_dev(torch, bad, gpu), do, ds, ordered=True)
    eng.wait()
    assert sorted(np.nonzero(st.cpu().numpy())[0].tolist()) == hit
    wiped = img.copy()
    for o, s in zip(offs, sizes):
        wiped[int(o) + int(s) + 1: int(o) + int(s) + 5] = 0
    buf = _dev(torch, wiped, gpu)
    crc = eng.sst_fill_trailers(buf, do, ds)
    eng.wait()
    assert np.array_equal(_u32(crc), np.array([b["crc"] for b in meta["blocks"]], np.uint32))
    assert np.array_equal(buf.cpu().numpy(), img)


def test_engine_log_verify_and_fill_golden(lvkv, golden, eng, gpu):
    """The reference-written WAL (tests/golden/wal.log): verify every record
    (log_reader.cc:243-247), catch a payload and a type-byte flip, refill
    every wiped header CRC (log_writer.cc:82-108) byte for byte."""
    import torch
    img = golden("wal.log")
    recs = golden("wal_records.json")["records"]
    hdr = _dev(torch, np.array([r["offset"] for r in recs], np.int64), gpu)
    actual, status = eng.log_verify(_dev(torch, img, gpu), hdr)
    eng.wait()
    assert np.array_equal(_u32(actual), np.array([r["crc"] for r in recs], np.uint32))
    assert not status.any().item()
    bad = img.copy()
    big = [i for i, r in enumerate(recs) if r["length"] > 10]
    bad[recs[big[0]]["offset"] + 7 + 3] ^= 1
    bad[recs[big[1]]["offset"] + 6] ^= 0x10
    _, st = eng.log_verify(_dev(torch, bad, gpu), hdr)
    eng.wait()
    assert sorted(np.nonzero(st.cpu().numpy())[0].tolist()) == sorted([big[0], big[1]])
    wiped = img.copy()
    for r in recs:
        wiped[r["offset"]: r["offset"] + 4] = 0
    buf = _dev(torch, wiped, gpu)
    eng.log_fill_headers(buf, hdr)
    eng.wait()
    assert np.array_equal(buf.cpu().numpy(), img)


def test_engine_general_many_in_flight(oracle, eng, gpu):
    """Hundreds of general submits between waits, rotating over the queues
    and through the kernarg ring: every batch's result intact."""
    import torch
    rng = np.random.default_rng(9)
    data = rng.integers(0, 256, 8 << 20, dtype=np.uint8)
    d = _dev(torch, data, gpu)
    K, n = 1200, 200
    offs = [rng.integers(0, data.size - 6000, n).astype(np.int64) for _ in range(8)]
    lens = [rng.integers(0, 6000, n).astype(np.int32) for _ in range(8)]
    do = [_dev(torch, o, gpu) for o in offs]
    dl = [_dev(torch, x, gpu) for x in lens]
    outs = torch.zeros(K, n, dtype=torch.int32, device=gpu)
    for k in range(K):
        eng.crc32c_batch(d, do[k % 8], dl[k % 8], out=outs[k], fresh=False)
    eng.wait()
    want = [oracle.batch(data, offs[w].astype(np.uint64), lens[w].view(np.uint32)) for w in range(8)]
    got = outs.cpu().numpy().view(np.uint32)
    for k in range(K):
        assert np.array_equal(got[k], want[k % 8]), k


@pytest.mark.parametrize("spec", [2, 3, 4, 5])
def test_engine_every_general_kernel(lvkv, oracle, eng, gpu, spec):
    """Each of the engine's general-layout kernels forced in turn
    (lvkv_debug_engine_ragged_spec): persistent and one-round burst walks of
    both shapes, on blocks of every start alignment and lengths 0..12,000
    (some over the lane walk's 4 KiB and over 64 KiB), with per-block inits;
    compute, masked compute, SST verify, and a synthetic WAL's verify and
    header refill."""
    import ctypes

    import torch
    lvkv.lib.lvkv_debug_engine_ragged_spec.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert lvkv.lib.lvkv_debug_engine_ragged_spec(eng.handle, spec) == 0
    try:
        rng = np.random.default_rng(100 + spec)
        data = rng.integers(0, 256, 24 << 20, dtype=np.uint8)
        n = 6000
        L = rng.integers(0, 2500, n).astype(np.uint32)
        L[::53] = rng.integers(2500, 12000, L[::53].size)
        L[:12] = [0, 1, 2, 3, 4, 15, 16, 17, 4095, 4096, 4097, 70000]
        offs = rng.integers(0, data.size - 70008, n).astype(np.uint64)
        inits = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        d = _dev(torch, data, gpu)
        do, dl = _dev(torch, offs.astype(np.int64), gpu), _dev(torch, L.view(np.int32), gpu)
        got = eng.crc32c_batch(d, do, dl, inits=_dev(torch, inits.view(np.int32), gpu))
        gm = eng.crc32c_batch(d, do, dl, init=0x0BADF00D, mask=True, ordered=True)
        eng.wait()
        assert np.array_equal(_u32(got), oracle.batch(data, offs, L, inits, threads=8))
        want_m = oracle.batch(data, offs, L, np.full(n, 0x0BADF00D, np.uint32), mask=True,
                              threads=8)
        assert np.array_equal(_u32(gm), want_m)
        # SST verify: trailers written from the oracle, some corrupted
        host = data.copy()
        so = (np.arange(800, dtype=np.uint64) * 7001 + rng.integers(0, 4, 800)).astype(np.uint64)
        ss = rng.integers(0, 6000, 800).astype(np.uint32)
        crc = oracle.batch(host, so, ss + 1, threads=8)
        for i in range(800):
            o = int(so[i]) + int(ss[i]) + 1
            host[o:o + 4] = np.frombuffer(np.uint32(oracle.mask(int(crc[i]))).tobytes(), np.uint8)
        bad = rng.choice(800, 40, replace=False)
        for i in bad:
            host[int(so[i]) + int(ss[i]) // 2] ^= 0x10
        act, st = eng.sst_verify(_dev(torch, host, gpu), _dev(torch, so.astype(np.int64), gpu),
                                 _dev(torch, ss.view(np.int32), gpu))
        eng.wait()
        assert sorted(np.nonzero(st.cpu().numpy())[0].tolist()) == sorted(bad.tolist())
        # WAL records (log_reader.cc:243-247, log_writer.cc:94-96): every
        # fragment kind, records of 0..2999 bytes and 100 KB ones, a few
        # payload bytes flipped; verify, then refill the wiped header CRCs
        import log_synth
        import log_walk as lw
        img = np.frombuffer(log_synth.build_log(3000, seed=spec, max_len=3000, big_every=211),
                            np.uint8).copy()
        hdrs = np.array(lw.block_verdicts(bytes(img)).hdrs, np.int64)
        lens = np.array([1 + int(img[h + 4]) + 256 * int(img[h + 5]) for h in hdrs], np.uint32)
        want = oracle.batch(img, (hdrs + 6).astype(np.uint64), lens, threads=8)
        flip = rng.choice(len(hdrs), 25, replace=False)
        badimg = img.copy()
        for i in flip:
            badimg[int(hdrs[i]) + 6 + int(lens[i]) // 2] ^= 0x08
        dh = _dev(torch, hdrs, gpu)
        act, st = eng.log_verify(_dev(torch, img, gpu), dh)
        act2, st2 = eng.log_verify(_dev(torch, badimg, gpu), dh)
        eng.wait()
        assert np.array_equal(_u32(act), want)
        assert not st.any().item()
        assert sorted(np.nonzero(st2.cpu().numpy())[0].tolist()) == sorted(flip.tolist())
        wiped = img.copy()
        for h in hdrs:
            wiped[int(h): int(h) + 4] = 0
        wb = _dev(torch, wiped, gpu)
        eng.log_fill_headers(wb, dh)
        eng.wait()
        assert np.array_equal(wb.cpu().numpy(), img)
    finally:
        lvkv.lib.lvkv_debug_engine_ragged_spec(eng.handle, -1)
