#!/bin/bash
# Profiles for profiles/: rocprofv3 kernel-trace + stats of the bench command
# and of the probe variants, then separate PMC passes (FETCH_SIZE, WRITE_SIZE)
# over the bench and over the dword read-bandwidth kernel (known byte count:
# calibrates FETCH_SIZE for this access width).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT="$R/gpurun_out/prof"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bench" -o bench -- \
  python3 "$R/bench.py" --streams 1 --steps 200 --warmup 20 --no-cpu-baseline > "$OUT/bench_stdout.json" 2> "$OUT/bench_stderr.log" \
  || { echo "bench trace failed"; tail -20 "$OUT/bench_stderr.log"; exit 1; }
echo "bench trace ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/probe" -o probe -- \
  python3 "$R/tools/probe.py" ${PROBES:-c1 v780 "readbw 41MB cold dword" "readbw 41MB cold 16" "v16 empty"} > "$OUT/probe_stdout.txt" 2>&1 \
  || { echo "probe trace failed"; tail -20 "$OUT/probe_stdout.txt"; exit 1; }
echo "probe trace ok"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_bench_$c" -o run -- \
    python3 "$R/bench.py" --streams 1 --steps 40 --warmup 5 --no-cpu-baseline > "$OUT/pmc_bench_$c.log" 2>&1 \
    || { echo "pmc bench $c failed"; tail -20 "$OUT/pmc_bench_$c.log"; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_readbw_$c" -o run -- \
    python3 "$R/tools/probe.py" "readbw 41MB cold dword" > "$OUT/pmc_readbw_$c.log" 2>&1 \
    || { echo "pmc readbw $c failed"; tail -20 "$OUT/pmc_readbw_$c.log"; exit 1; }
done
echo "pmc ok"
find "$OUT" -name "*.csv" | head -40
