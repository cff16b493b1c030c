"""Sweep of the any-size decode paths (GPU box; evidence, not a test): M
blocks of 5 KiB - 1.5 MiB (db_bench's generator, text, runs, random bytes),
each compressed by libsnappy 1.1.8 and by libzstd 1.4.9 at levels 1, 3 and
19 (the host libraries ReadBlock would meet), decoded on the device with
max_ulen 4,096 so that nearly every block takes the HBM-output kernels, and
compared with its input. Prints one JSON line; writes
gpurun_out/big_blocks_fuzz.json.

    python tests/sweeps/big_blocks_fuzz.py [M] [seed]
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "oracle"))


def inputs(m, seed):
    from tools.db_bench_data import block_batch
    rng = np.random.default_rng(seed)
    bb = block_batch(512).tobytes()  # 2 MiB of db_bench data
    text = (b"LevelDB is a fast key-value storage library written at Google that provides"
            b" an ordered mapping from string keys to string values. ") * 20000
    out = []
    for k in range(m):
        n = int(np.exp(rng.uniform(np.log(5 << 10), np.log(1536 << 10))))
        kind = k % 4
        if kind == 0:
            s = int(rng.integers(0, max(1, len(bb) - n)))
            x = (bb * (n // len(bb) + 2))[s:s + n]
        elif kind == 1:
            s = int(rng.integers(0, 1000))
            x = text[s:s + n]
        elif kind == 2:
            x = rng.integers(0, int(rng.integers(2, 12)), n, dtype=np.uint8).tobytes()
        else:
            x = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        out.append(x)
    return out


def main():
    import torch
    import __graft_entry__ as g
    import snappy_oracle as so
    import zstd_oracle as zo
    lvkv = g.load_package()
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 120
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    ins = inputs(m, seed)
    slib, zlib = so.system_snappy(), zo.system_zstd()
    dev = torch.device("cuda:0")
    res = {"blocks": m, "seed": seed, "bytes": int(sum(map(len, ins))), "cases": {}}

    def run(name, streams, decode):
        offs = np.zeros(len(streams), dtype=np.int64)
        offs[1:] = np.cumsum([len(s) for s in streams[:-1]])
        src = torch.from_numpy(np.frombuffer(b"".join(streams), dtype=np.uint8).copy()).to(dev)
        off = torch.from_numpy(offs).to(dev)
        ln = torch.tensor([len(s) for s in streams], dtype=torch.int32, device=dev)
        sizes = [len(x) for x in ins]
        doff = np.zeros(len(sizes), dtype=np.int64)
        doff[1:] = np.cumsum(sizes[:-1])
        dst = torch.empty(int(sum(sizes)), dtype=torch.uint8, device=dev)
        d_off = torch.from_numpy(doff).to(dev)
        cap = torch.tensor(sizes, dtype=torch.int32, device=dev)
        _, _, olen, st = decode(src, off, ln, max_ulen=4096, dst=dst, dst_offsets=d_off, dst_caps=cap)
        torch.cuda.synchronize()
        d = dst.cpu().numpy()
        bad = [k for k, (x, o) in enumerate(zip(ins, doff.tolist()))
               if int(st[k]) != 0 or d[o:o + len(x)].tobytes() != x]
        res["cases"][name] = {"streams": len(streams), "stream_bytes": int(sum(map(len, streams))),
                              "mismatches": len(bad), "first_bad": bad[:10]}
        print(name, res["cases"][name], flush=True)

    if slib is not None:
        run("snappy", [so.lib_compress(slib, x) for x in ins], lvkv.snappy_uncompress)
    if zlib is not None:
        for lvl in (1, 3, 19):
            run(f"zstd_level{lvl}", [zo.lib_compress(zlib, x, lvl) for x in ins], lvkv.zstd_uncompress)
    print(json.dumps(res), flush=True)
    (REPO / "gpurun_out").mkdir(exist_ok=True)
    (REPO / "gpurun_out" / "big_blocks_fuzz.json").write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
