"""Copy the rocprofv3 summaries of tools/prof_engine.sh into profiles/.

    python tools/collect_engine_profiles.py r02 [gpurun_out/prof_engine]

Writes profiles/<tag>_engine_iso_kernel_stats.csv and
<tag>_engine_pipe_kernel_stats.csv (kernel-trace --stats, lvkv kernels only;
the one torch RNG launch that fills the input is dropped), <tag>_engine_pmc.json
(per-dispatch means of every counter over the isolated launches, first
quarter dropped) and pmc_traffic.json (HBM bytes per headline launch,
bench.py's roofline.traffic).

FETCH_SIZE is in KiB and, on gfx950, counts half the bytes of a coalesced
streaming read (MI355X_MICROARCH.md, HBM/rocprofv3 section): bytes =
FETCH_SIZE x 1024 x 2. WRITE_SIZE (KiB) is exact for dword stores.
"""
import collections
import csv
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
KERNEL = "lvkv_ek_uniform_pair"


def main():
    tag = sys.argv[1]
    src = Path(sys.argv[2] if len(sys.argv) > 2 else REPO / "gpurun_out" / "prof_engine")
    dst = REPO / "profiles"
    for run in ("iso", "pipe"):
        rows = list(csv.reader(open(src / run / "run_kernel_stats.csv")))
        keep = [rows[0]] + [r for r in rows[1:] if r[0].startswith("lvkv_") or
                            r[0].startswith("__amd")]
        with open(dst / f"{tag}_engine_{run}_kernel_stats.csv", "w", newline="") as f:
            csv.writer(f, quoting=csv.QUOTE_NONNUMERIC).writerows(keep)
    vals = collections.defaultdict(list)
    for p in sorted(src.glob("pmc*/run_counter_collection.csv")):
        for r in csv.DictReader(open(p)):
            if r["Kernel_Name"].startswith("lvkv_"):
                vals[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    pmc = {}
    for (k, c), v in sorted(vals.items()):
        v = v[len(v) // 4:] if len(v) > 4 else v
        pmc.setdefault(k, {})[c] = {"mean": round(sum(v) / len(v), 3), "dispatches": len(v)}
    (dst / f"{tag}_engine_pmc.json").write_text(json.dumps(pmc, indent=1) + "\n")
    m = pmc[KERNEL]
    fetch = m["FETCH_SIZE"]["mean"] * 1024 * 2
    write = m["WRITE_SIZE"]["mean"] * 1024
    traffic = {"kernel": KERNEL, "source": f"profiles/{tag}_engine_pmc.json",
               "fetch_bytes_per_launch": int(fetch), "write_bytes_per_launch": int(write),
               "hbm_bytes_per_launch": int(fetch + write),
               "algo_bytes_per_launch": 10_000 * (4096 + 4),
               "correction": "FETCH_SIZE KiB x 1024 x 2 (gfx950 half-count), WRITE_SIZE KiB x 1024",
               "note": "isolated (ordered) launches of bench.py --isolated; the 40 KB of CRC "
                       "stores stay in L2 until the engine's system-scope fence (WRITE_SIZE ~0)"}
    (dst / "pmc_traffic.json").write_text(json.dumps(traffic, indent=1) + "\n")
    print(json.dumps(traffic))


if __name__ == "__main__":
    main()
