"""Device Snappy codec throughput on db_bench's workload (GPU box).

    python tools/snappy_bench.py [--blocks 65536] [--steps 20]

db_bench's snappycomp / snappyuncomp (benchmarks/db_bench.cc:384-433)
compress one 4096-byte block of RandomGenerator data (compression ratio 0.5)
over and over, one thread, and report MB/s of uncompressed bytes. Here a
batch of `--blocks` such blocks (the generator's consecutive 4 KiB slices,
db_bench.cc:195-202) sits in HBM; one step compresses (or uncompresses) the
whole batch in one launch, timed with HIP events on the launch stream. The
CPU lines run libsnappy 1.1.8 (the library the reference would link) the
db_bench way on one thread, and in 16 processes over distinct blocks (run
before the GPU is initialised: the pool forks).
Prints one JSON line; writes gpurun_out/snappy_bench.json.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "oracle"))
from tools.db_bench_data import block_batch  # noqa: E402


def cpu_lines(blocks: np.ndarray, seconds: float = 2.0, procs: int = 16):
    import snappy_oracle as so  # libsnappy 1.1.8 handle (test infrastructure)
    lib = so.system_snappy()
    if lib is None:
        return None
    import ctypes
    blk = blocks[:4096].tobytes()
    comp = so.lib_compress(lib, blk)
    out = ctypes.create_string_buffer(lib.snappy_max_compressed_length(4096))
    unc = ctypes.create_string_buffer(4096)

    def loop_comp(b, secs):
        n, t0 = 0, time.perf_counter()
        ol = ctypes.c_size_t()
        o = ctypes.create_string_buffer(lib.snappy_max_compressed_length(4096))
        while time.perf_counter() - t0 < secs:
            for _ in range(64):
                ol.value = len(o)
                lib.snappy_compress(b, 4096, o, ctypes.byref(ol))
            n += 64
        return n * 4096 / (time.perf_counter() - t0)

    def loop_unc(c, secs):
        n, t0 = 0, time.perf_counter()
        ol = ctypes.c_size_t()
        o = ctypes.create_string_buffer(4096)
        while time.perf_counter() - t0 < secs:
            for _ in range(64):
                ol.value = 4096
                lib.snappy_uncompress(c, len(c), o, ctypes.byref(ol))
            n += 64
        return n * 4096 / (time.perf_counter() - t0)

    del out, unc
    res = {"comp_1t_MBps": loop_comp(blk, seconds) / 1e6, "uncomp_1t_MBps": loop_unc(comp, seconds) / 1e6,
           "output_pct": round(100.0 * len(comp) / 4096, 1)}
    if procs > 1:  # one process a core (no GIL between them), distinct blocks
        import multiprocessing as mp
        with mp.get_context("fork").Pool(procs) as pool:
            r = pool.map(_cpu_worker, [(blocks[i * 4096:(i + 1) * 4096].tobytes(), seconds)
                                       for i in range(procs)])
        res[f"comp_{procs}p_MBps"] = sum(a for a, _ in r) / 1e6
        res[f"uncomp_{procs}p_MBps"] = sum(b for _, b in r) / 1e6
    return {k: round(v, 1) for k, v in res.items()}


def zstd_cpu_lines(frames, seconds: float = 2.0, procs: int = 16):
    """libzstd 1.4.9 decompressing the same frames: one core, and `procs`
    processes (port::Zstd_Uncompress: ZSTD_decompress into the content size)."""
    import zstd_oracle as zo
    if zo.system_zstd() is None:
        return None
    import multiprocessing as mp
    one = _zstd_worker((frames[:256], seconds))
    res = {"uncomp_1t_MBps": one / 1e6}
    if procs > 1:
        with mp.get_context("fork").Pool(procs) as pool:
            r = pool.map(_zstd_worker, [(frames[i * 16:(i + 1) * 16], seconds)
                                        for i in range(procs)])
        res[f"uncomp_{procs}p_MBps"] = sum(r) / 1e6
    return {k: round(v, 1) for k, v in res.items()}


def zstd_compress_cpu_lines(blocks: np.ndarray, seconds: float = 2.0, procs: int = 16):
    """libzstd 1.4.9 through port::Zstd_Compress's calls, per 4 KiB block at
    level 1 (oracle/zstd_port_bench, a C harness): one core and `procs`
    processes."""
    import subprocess
    import tempfile
    exe = REPO / "oracle" / "zstd_port_bench"
    if not exe.exists():
        return None
    with tempfile.NamedTemporaryFile(suffix=".bin") as f:
        f.write(blocks.tobytes())
        f.flush()
        res = {}
        for p in (1, procs):
            out = subprocess.run([str(exe), f.name, "4096", "1", str(seconds), str(p)],
                                 capture_output=True, text=True, check=True).stdout
            r = json.loads(out)
            res[f"comp_{'1t' if p == 1 else f'{p}p'}_MBps"] = r["MBps"]
            res["output_pct"] = r["output_pct"]
    return res


def _zstd_worker(arg):
    frames, seconds = arg
    import ctypes
    import zstd_oracle as zo
    lib = zo.system_zstd()
    o = ctypes.create_string_buffer(4096)
    n, t0, k = 0, time.perf_counter(), 0
    while time.perf_counter() - t0 < seconds:
        for _ in range(256):
            f = frames[k % len(frames)]
            k += 1
            lib.ZSTD_decompress(o, 4096, f, len(f))
        n += 256
    return n * 4096 / (time.perf_counter() - t0)


def _cpu_worker(arg):
    blk, seconds = arg
    import ctypes
    import snappy_oracle as so
    lib = so.system_snappy()
    comp = so.lib_compress(lib, blk)
    o = ctypes.create_string_buffer(lib.snappy_max_compressed_length(4096))
    ol = ctypes.c_size_t()
    rates = []
    for fn, src, cap in ((lib.snappy_compress, blk, len(o)), (lib.snappy_uncompress, comp, 4096)):
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            for _ in range(256):
                ol.value = cap
                fn(src, len(src), o, ctypes.byref(ol))
            n += 256
        rates.append(n * 4096 / (time.perf_counter() - t0))
    return tuple(rates)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--zstd-frames", default=None,
                    help="read the zstd frames from this file instead of libzstd (profiled "
                         "runs: the profiler's own zstd clashes with the library)")
    ap.add_argument("--write-zstd-frames", default=None,
                    help="write the zstd frames to this file and exit")
    args = ap.parse_args()
    cpu = None if args.no_cpu else cpu_lines(block_batch(64))
    # the same blocks as zstd frames (libzstd level 1, LevelDB's default
    # zstd_compression_level), for the device decoder
    import zstd_oracle as zo
    zframes = None
    if args.zstd_frames:
        blob = Path(args.zstd_frames).read_bytes()
        zframes, p = [], 0
        while p < len(blob):
            n = int.from_bytes(blob[p:p + 4], "little")
            zframes.append(blob[p + 4:p + 4 + n])
            p += 4 + n
        args.no_cpu = True
    else:
        zlib = zo.system_zstd()
        if zlib is not None:
            h = block_batch(256)
            zframes = [zo.lib_compress(zlib, h[i * 4096:(i + 1) * 4096].tobytes(), 1)
                       for i in range(256)]
    if args.write_zstd_frames:
        Path(args.write_zstd_frames).write_bytes(
            b"".join(len(f).to_bytes(4, "little") + f for f in zframes))
        return
    zcpu = None if args.no_cpu or zframes is None else zstd_cpu_lines(zframes)
    zccpu = None if args.no_cpu else zstd_compress_cpu_lines(block_batch(256))
    import torch
    import __graft_entry__ as g
    lvkv = g.load_package()
    dev = torch.device("cuda:0")
    nb, L = args.blocks, 4096
    host = block_batch(nb, L)
    src = torch.from_numpy(host).to(dev)
    off = torch.arange(nb, dtype=torch.int64, device=dev) * L
    ln = torch.full((nb,), L, dtype=torch.int32, device=dev)
    dst, doff, dlen, st = lvkv.snappy_compress(src, off, ln, max_len=L)
    torch.cuda.synchronize()
    assert int(st.max()) == 0
    # parity on a sample: the device streams decode to the inputs and match
    # libsnappy / the oracle (tests/test_snappy.py covers the rest)
    import snappy_oracle as so
    lib = so.system_snappy()
    d_host = dst.cpu().numpy()
    for i in range(0, nb, max(1, nb // 64)):
        s = d_host[int(doff[i]):int(doff[i]) + int(dlen[i])].tobytes()
        want = so.lib_compress(lib, host[i * L:(i + 1) * L].tobytes()) if lib else \
            so.compress(host[i * L:(i + 1) * L].tobytes())
        assert s == want, i
    comp_bytes = int(dlen.to(torch.int64).sum())
    stream = torch.cuda.current_stream(dev)

    def timed(fn):
        for _ in range(args.warmup):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.steps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e-3 / args.steps

    out_len, out_st = torch.empty_like(dlen), torch.empty_like(st)
    t_comp = timed(lambda: lvkv.lib.lvkv_snappy_compress_device(
        src.data_ptr(), off.data_ptr(), ln.data_ptr(), dst.data_ptr(), doff.data_ptr(),
        out_len.data_ptr(), out_st.data_ptr(), nb, L, stream.cuda_stream))
    cap = torch.full((nb,), L, dtype=torch.int32, device=dev)
    udst = torch.empty(nb * L, dtype=torch.uint8, device=dev)
    ulen, ust = torch.empty_like(dlen), torch.empty_like(st)
    t_unc = timed(lambda: lvkv.lib.lvkv_snappy_uncompress_device(
        dst.data_ptr(), doff.data_ptr(), dlen.data_ptr(), udst.data_ptr(), off.data_ptr(),
        cap.data_ptr(), ulen.data_ptr(), ust.data_ptr(), nb, L, stream.cuda_stream))
    torch.cuda.synchronize()
    assert int(ust.max()) == 0 and torch.equal(udst, src)
    assert torch.equal(out_len, dlen)
    raw = nb * L
    res = {
        "workload": f"db_bench snappycomp/snappyuncomp blocks: {nb} x {L} B (RandomGenerator, ratio 0.5)",
        "blocks": nb, "block_bytes": L, "output_pct": round(100.0 * comp_bytes / raw, 2),
        "compress": {"us_per_launch": round(t_comp * 1e6, 1), "GBps_uncompressed": round(raw / t_comp / 1e9, 2),
                     "hbm_GBps": round((raw + comp_bytes) / t_comp / 1e9, 2)},
        "uncompress": {"us_per_launch": round(t_unc * 1e6, 1), "GBps_uncompressed": round(raw / t_unc / 1e9, 2),
                       "hbm_GBps": round((raw + comp_bytes) / t_unc / 1e9, 2)},
    }
    if cpu is not None:
        res["cpu_libsnappy_1_1_8"] = cpu
    if zframes is not None:  # zstd: the device decoder over the 256 distinct frames, cycled
        zf = [zframes[i % 256] for i in range(nb)]
        zoff = np.zeros(nb, dtype=np.int64)
        zoff[1:] = np.cumsum([len(f) for f in zf[:-1]])
        zbuf = torch.from_numpy(np.frombuffer(b"".join(zf), dtype=np.uint8).copy()).to(dev)
        zo_t = torch.from_numpy(zoff).to(dev)
        zl_t = torch.tensor([len(f) for f in zf], dtype=torch.int32, device=dev)
        zbytes = int(zl_t.to(torch.int64).sum())
        t_z = timed(lambda: lvkv.lib.lvkv_zstd_uncompress_device(
            zbuf.data_ptr(), zo_t.data_ptr(), zl_t.data_ptr(), udst.data_ptr(), off.data_ptr(),
            cap.data_ptr(), ulen.data_ptr(), ust.data_ptr(), nb, L, stream.cuda_stream))
        torch.cuda.synchronize()
        assert int(ust.max()) == 0 and torch.equal(udst, src)
        res["zstd_uncompress"] = {"us_per_launch": round(t_z * 1e6, 1),
                                  "GBps_uncompressed": round(raw / t_z / 1e9, 2),
                                  "hbm_GBps": round((raw + zbytes) / t_z / 1e9, 2),
                                  "output_pct": round(100.0 * zbytes / raw, 2)}
        if zcpu is not None:
            res["cpu_libzstd_1_4_9"] = zcpu
    # zstd compress (port::Zstd_Compress at level 1, LevelDB's default): the
    # device compressor over the nb blocks, one launch
    zb = L + (L >> 8) + ((131072 - L) >> 11)
    zdst = torch.empty(nb * zb, dtype=torch.uint8, device=dev)
    zdoff = torch.arange(nb, dtype=torch.int64, device=dev) * zb
    zlen, zst = torch.empty_like(dlen), torch.empty_like(st)
    t_zc = timed(lambda: lvkv.lib.lvkv_zstd_compress_device(
        src.data_ptr(), off.data_ptr(), ln.data_ptr(), zdst.data_ptr(), zdoff.data_ptr(),
        zlen.data_ptr(), zst.data_ptr(), nb, L, 1, stream.cuda_stream))
    torch.cuda.synchronize()
    assert int(zst.max()) == 0
    zc_bytes = int(zlen.to(torch.int64).sum())
    # parity on a sample (tests/test_zstd_write.py covers the rest): the
    # library's own frame through the port's calls, or the oracle's
    import zstd_encoder as ze
    zlib_w = None if args.zstd_frames else ze.system_zstd_writer()  # (profiled: no libzstd)
    zh = zdst.cpu().numpy()
    for i in range(0, nb, max(1, nb // (64 if zlib_w else 8))):
        blk = host[i * L:(i + 1) * L].tobytes()
        want = ze.lib_port_compress(zlib_w, blk, 1) if zlib_w else ze.compress(blk, 1)
        assert zh[i * zb:i * zb + int(zlen[i])].tobytes() == want, i
    res["zstd_compress"] = {"us_per_launch": round(t_zc * 1e6, 1),
                            "GBps_uncompressed": round(raw / t_zc / 1e9, 2),
                            "hbm_GBps": round((raw + zc_bytes) / t_zc / 1e9, 2),
                            "output_pct": round(100.0 * zc_bytes / raw, 2), "level": 1}
    if zccpu is not None:
        res["cpu_libzstd_1_4_9_port_compress"] = zccpu
    print(json.dumps(res), flush=True)
    (REPO / "gpurun_out").mkdir(exist_ok=True)
    (REPO / "gpurun_out" / "snappy_bench.json").write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
