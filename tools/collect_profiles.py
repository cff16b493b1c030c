"""Copy the rocprofv3 summaries of a gpu_prof.sh run into profiles/.

    python tools/collect_profiles.py r01 [gpurun_out/prof]

Writes profiles/<tag>_bench_kernel_stats.csv (kernel-trace --stats of the
bench command), <tag>_probe_kernel_stats.csv, <tag>_pmc.json (per-kernel
FETCH_SIZE / WRITE_SIZE means, separate --pmc passes) and pmc_traffic.json
(the HBM bytes per headline launch bench.py reports as roofline.traffic).

FETCH_SIZE is in KiB and, on gfx950, reports half the bytes of a coalesced
streaming read (MI355X_MICROARCH.md, HBM/rocprofv3 section): bytes =
FETCH_SIZE x 1024 x 2. The x2 was checked on this pool with the dword
read-bandwidth kernel, whose byte count is known (tools/probe.py readbw).
WRITE_SIZE (KiB) is exact for the dword result stores.
"""
import collections
import csv
import json
import shutil
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
HEADLINE = "crc32c_compact_kernel"


def short(name):
    if "lvkv::" not in name:
        return None
    return name.split("lvkv::")[1].split("(")[0]


def pmc_means(path):
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        if k:
            vals[k].append(float(r["Counter_Value"]))
    # drop the first quarter (warm-up, table upload) of each kernel's dispatches
    return {k: sum(v[len(v) // 4:]) / len(v[len(v) // 4:]) for k, v in vals.items()}


def main():
    tag = sys.argv[1]
    src = Path(sys.argv[2] if len(sys.argv) > 2 else REPO / "gpurun_out" / "prof")
    dst = REPO / "profiles"
    dst.mkdir(exist_ok=True)
    for name, sub in (("bench", "bench/bench_kernel_stats.csv"),
                      ("probe", "probe/probe_kernel_stats.csv")):
        if (src / sub).exists():
            shutil.copy(src / sub, dst / f"{tag}_{name}_kernel_stats.csv")
    pmc = {}
    for run in ("bench", "readbw"):
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            p = src / f"pmc_{run}_{ctr}" / "run_counter_collection.csv"
            if p.exists():
                for k, v in pmc_means(p).items():
                    pmc.setdefault(run, {}).setdefault(k, {})[ctr + "_KiB"] = round(v, 3)
    (dst / f"{tag}_pmc.json").write_text(json.dumps(pmc, indent=1) + "\n")
    bench = pmc.get("bench", {})
    head = [k for k in bench if HEADLINE in k]
    if head:
        c = bench[head[0]]
        fetch = c.get("FETCH_SIZE_KiB", 0.0) * 1024 * 2
        write = c.get("WRITE_SIZE_KiB", 0.0) * 1024
        (dst / "pmc_traffic.json").write_text(json.dumps({
            "kernel": head[0], "source": f"profiles/{tag}_pmc.json",
            "fetch_bytes_per_launch": round(fetch), "write_bytes_per_launch": round(write),
            "hbm_bytes_per_launch": round(fetch + write),
            "correction": "FETCH_SIZE KiB x 1024 x 2 (gfx950 half-count), WRITE_SIZE KiB x 1024",
        }, indent=1) + "\n")
    print(json.dumps(pmc, indent=1))


if __name__ == "__main__":
    main()
