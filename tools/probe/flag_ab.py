"""A/B of the engine's device-written completion (lvkv_engine_set_flag_wait)
on the bench's headline region (GPU box). Not part of the product.

    python tools/probe/flag_ab.py [--reps 7] [--steps 20]

Interleaved runs of bench.timed_region (sync, t0, K submits with the last 3
FINAL, wait, sync, t1) with the flag wait off and on, on one engine over the
bench's 1.25 GiB rotation; the results of the last flagged steps are checked
against ordered recomputation. Writes gpurun_out/flag_ab.json.
"""
import json
import statistics
import sys
from pathlib import Path

import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO))
import __graft_entry__ as g  # noqa: E402
import bench  # noqa: E402


def main():
    reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 7
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 20
    lvkv = g.load_package()
    dev = torch.device("cuda:0")
    nb, L, stride, off, _ = bench.CONFIGS["headline"]
    buf, nrot, window = bench.make_buffers(torch, dev, 0, nb, stride, 1.25 * bench.GIB)
    outs = [torch.empty(nb, dtype=torch.int32, device=dev) for _ in range(4)]
    eng = lvkv.Engine(0)
    runner = bench.EngineRunner(lvkv, eng, buf, nb, L, stride, off, nrot, window, outs)
    comm = bench.Comm(1)
    nxt = 1
    res = {"off": [], "on": []}
    for rep in range(reps):
        for mode in ("off", "on") if rep % 2 == 0 else ("on", "off"):
            eng.set_flag_wait(mode == "on")
            el, nxt = bench.timed_region(runner, comm, steps, 5, 0.15, first=nxt)
            gibs = nb * L * steps / el / bench.GIB
            res[mode].append(round(100.0 * gibs * bench.GIB / 1e9 / bench.HBM_PEAK_GBS, 3))
            if mode == "on":
                # the last 4 steps' outputs (3 of them flagged) against ordered submits
                last = [nxt - 4 + k for k in range(4)]
                want = [outs[i % 4].clone() for i in last]
                eng.set_flag_wait(False)
                chk = torch.empty(nb, dtype=torch.int32, device=dev)
                for i, w in zip(last, want):
                    runner.submit(runner.h, runner.bases[i % nrot], stride, L, 0, chk.data_ptr(),
                                  nb, 2)
                    eng.wait()
                    assert torch.equal(chk, w), ("flagged outputs differ", i)
            print(rep, mode, res[mode][-1], flush=True)
    summary = {m: {"pct_hbm_peak": v, "median": statistics.median(v)} for m, v in res.items()}
    summary["flag_stats"] = eng.flag_stats()
    summary["steps"] = steps
    print(json.dumps(summary), flush=True)
    (REPO / "gpurun_out").mkdir(exist_ok=True)
    (REPO / "gpurun_out" / "flag_ab.json").write_text(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
