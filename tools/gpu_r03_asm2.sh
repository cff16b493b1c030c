#!/bin/bash
# ReadRecord and gather look-backs: the log tests and the read path's kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_damage.py tests/test_log_blocks.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/asm_tests.log 2>&1 \
  || { echo "log tests failed"; tail -30 gpurun_out/asm_tests.log; exit 1; }
tail -2 gpurun_out/asm_tests.log
rm -rf gpurun_out/r03_asm_prof
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_asm_prof -o run -- python3 tools/probe/log_probe.py 60000 --read > gpurun_out/r03_asm_prof.log 2>&1 \
  || { echo "log prof failed"; tail -20 gpurun_out/r03_asm_prof.log; exit 1; }
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/r03_asm_prof/run_kernel_stats.csv')):
    print(r['Name'][:60], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])
"
timeout -k 10 200 python3 tools/probe/log_probe.py 60000 --read --asm-stamps > gpurun_out/asm_stamps.log 2>&1 && tail -13 gpurun_out/asm_stamps.log
