"""Pins oracle/zstd_encoder.py to libzstd 1.4.9 (this container's
/opt/conda/lib) on many fresh inputs, driven as port::Zstd_Compress drives
the library (CPU; evidence beside tests/test_zstd_write.py's 400-input fuzz; writes
gpurun_out/zstd_oracle_pin.json).

    python tests/sweeps/zstd_oracle_pin.py [N] [seed] [levels, comma-separated]
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests"))
sys.path.insert(0, str(REPO / "oracle"))


def main():
    import test_zstd_write as t
    import zstd_encoder as ze
    lib = ze.system_zstd_writer()
    if lib is None:
        raise SystemExit("libzstd 1.4.9 not found")
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 11
    levels = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [1, 2, -1, -5]
    res = {"inputs_per_level": n, "seed": seed, "library": "libzstd 1.4.9 (port::Zstd_Compress calls)",
           "levels": {}}
    for level in levels:
        rng = np.random.default_rng(seed * 10 + level)
        blobs = t._fuzz_inputs(rng, n - n // 10, 6000) + t._fuzz_inputs(rng, n // 10, 20481)
        bad = [k for k, x in enumerate(blobs) if ze.compress(x, level) != ze.lib_port_compress(lib, x, level)]
        res["levels"][str(level)] = {"inputs": len(blobs), "bytes": int(sum(map(len, blobs))),
                                     "oracle_differs_from_library": len(bad), "first_bad": bad[:10]}
        print(level, res["levels"][str(level)], flush=True)
    print(json.dumps(res))
    return res


if __name__ == "__main__":
    r = main()
    (REPO / "gpurun_out").mkdir(exist_ok=True)
    (REPO / "gpurun_out" / "zstd_oracle_pin.json").write_text(json.dumps(r, indent=1))
