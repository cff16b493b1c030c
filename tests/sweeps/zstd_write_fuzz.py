"""Large parity sweep of the device Zstd compressor against the oracle
(GPU box; evidence, not a test): N ragged blocks per level from
tests/test_zstd_write.py's generator (db_bench slices, random, few-symbol,
skewed, repeats, key/value entries; 0-20 KiB), every device frame compared
byte for byte with oracle/zstd_encoder.py and decoded back by the device
decoder. Prints one JSON line; writes gpurun_out/zstd_write_fuzz.json.

    python tests/sweeps/zstd_write_fuzz.py [N] [seed] [levels, comma-separated; default 1,-1]
"""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests"))
sys.path.insert(0, str(REPO / "oracle"))


def main():
    import torch
    import __graft_entry__ as g
    import test_zstd_write as t
    import zstd_encoder as ze
    lvkv = g.load_package()
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 2026
    dev = torch.device("cuda:0")
    res = {"blocks_per_level": n, "seed": seed, "levels": {}}
    levels = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [1, -1]
    for level in levels:
        rng = np.random.default_rng(seed + level)
        blobs = t._fuzz_inputs(rng, n - n // 10, 6000) + t._fuzz_inputs(rng, n // 10, 20481)
        src, off, ln = t._pack(torch, dev, blobs, skew=5)
        dst, doff, dlen, st = lvkv.zstd_compress(src, off, ln, level=level, max_len=20480)
        torch.cuda.synchronize()
        got = t._unpack(dst, doff, dlen)
        t0 = time.time()
        bad = [k for k, (x, f) in enumerate(zip(blobs, got)) if f != ze.compress(x, level)]
        small = [k for k, x in enumerate(blobs) if 0 < len(x)]
        s2, o2, l2 = t._pack(torch, dev, [got[k] for k in small])
        out, ooff, olen, st2 = lvkv.zstd_uncompress(s2, o2, l2, max_ulen=20480)
        torch.cuda.synchronize()
        back = t._unpack(out, ooff, olen)
        rt_bad = sum(1 for j, k in enumerate(small) if back[j] != blobs[k])
        res["levels"][str(level)] = {
            "blocks": len(blobs), "bytes": int(sum(map(len, blobs))),
            "statuses_ok": int((st.cpu() == 0).sum()), "frames_differing_from_oracle": len(bad),
            "first_bad": bad[:10], "device_roundtrip_mismatches": rt_bad,
            "oracle_seconds": round(time.time() - t0, 1)}
        print(level, res["levels"][str(level)], flush=True)
    print(json.dumps(res), flush=True)
    (REPO / "gpurun_out").mkdir(exist_ok=True)
    (REPO / "gpurun_out" / "zstd_write_fuzz.json").write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
