#!/bin/bash
# Round 3 SST verify: GPU tests, per-call timings of the three shapes under
# the default form choice, and kernel traces of the 70 MB table.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_sst_table.py tests/test_damage.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_sst_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/r03_sst_tests.log; exit 1; }
tail -2 gpurun_out/r03_sst_tests.log
for a in "512" "16384" "512 --tables=32"; do timeout -k 10 60 python tools/probe/sst_probe.py $a 2>&1 | grep -v amdgpu.ids || exit 1; done
for a in 16384 512; do
  rm -rf gpurun_out/r03_sstprof_$a
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_sstprof_$a -o run -- python3 tools/probe/sst_probe.py $a > gpurun_out/r03_sstprof_$a.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r03_sstprof_$a.log; exit 1; }
  python3 -c "
import csv,sys
for r in csv.DictReader(open('gpurun_out/r03_sstprof_$a/run_kernel_stats.csv')):
    print('$a', r['Name'].split('(')[0][-34:], r['Calls'], r['AverageNs'], r['MinNs'])
"
done
mkdir -p /tmp/wp && hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe/walk_probe.hip -o /tmp/wp/walk_probe 2>/dev/null && timeout -k 5 60 /tmp/wp/walk_probe 2048
