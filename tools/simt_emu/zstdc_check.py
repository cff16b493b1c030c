"""Run the emulated device Zstd compressor (tools/simt_emu/emu_build.sh) on
blocks and compare every frame with the oracle's (CPU debugging aid).

    python tools/simt_emu/zstdc_check.py [fixtures|bench N|fuzz N SEED] [level]
"""
from __future__ import annotations

import json
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests"))
sys.path.insert(0, str(REPO / "oracle"))
import zstd_encoder as ze  # noqa: E402


def blocks(kind, args):
    if kind == "fixtures":
        spec = json.loads((REPO / "tests/golden/zstd_write.json").read_text())
        blob = (REPO / "tests/golden/zstd_write_inputs.bin").read_bytes()
        out, p = [], 0
        for n in spec["inputs"]:
            out.append(blob[p:p + n])
            p += n
        return [x for x in out if len(x) <= 20480]
    if kind == "bench":
        from tools.db_bench_data import block_batch
        n = int(args[0])
        h = block_batch(n).tobytes()
        return [h[i * 4096:(i + 1) * 4096] for i in range(n)]
    import test_zstd_write as t
    rng = np.random.default_rng(int(args[1]) if len(args) > 1 else 1)
    return t._fuzz_inputs(rng, int(args[0]), 6000)


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "bench"
    rest = sys.argv[2:]
    level = 1
    if rest and rest[-1].lstrip("-").isdigit() and kind == "fixtures":
        level = int(rest[-1])
    ins = blocks(kind, rest)
    exe = REPO / "build" / "simt_emu" / "zstdc_emu"
    with tempfile.TemporaryDirectory() as d:
        d = Path(d)
        (d / "in.bin").write_bytes(b"".join(ins))
        (d / "lens.u32").write_bytes(np.array([len(x) for x in ins], dtype=np.uint32).tobytes())
        mx = max(16, max(len(x) for x in ins))
        r = subprocess.run([str(exe), str(d / "in.bin"), str(d / "lens.u32"), str(level), str(mx),
                            str(d / "out.bin"), str(d / "ol.u32")], capture_output=True, text=True)
        if r.returncode:
            print(r.stderr[-4000:])
            raise SystemExit(f"emulator failed: {r.returncode}")
        ob = (d / "out.bin").read_bytes()
        rec = np.frombuffer((d / "ol.u32").read_bytes(), dtype=np.uint32).reshape(-1, 2)
    bad, p = [], 0
    for k, (x, (n, st)) in enumerate(zip(ins, rec)):
        f = ob[p:p + n]
        p += n
        if st != 0 or f != ze.compress(x, level):
            bad.append(k)
    print(f"{len(ins)} blocks, {len(bad)} differ from the oracle: {bad[:20]}")


if __name__ == "__main__":
    main()
