#!/bin/bash
# rocprofv3 kernel-trace of selected probe cases (device durations, no host
# launch-rate effects). Usage: PROBES="v780 v782" bash tools/gpu_probe_prof.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT="$R/gpurun_out/pprof"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o p -- \
  python3 "$R/tools/probe.py" $PROBES > "$OUT/stdout.txt" 2>&1 || { echo "probe trace failed"; tail -20 "$OUT/stdout.txt"; exit 1; }
python3 - "$OUT/p_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "lvkv" in n:
        print(f'{n.split("lvkv::")[1].split("(")[0]:45s} calls={r["Calls"]:>6s} avg_ns={float(r["AverageNs"]):9.1f} min_ns={r["MinNs"]}')
PY
