#!/bin/bash
# WAL verify iteration on one GPU: the log tests, then timing, phase stamps
# and a kernel trace of the read path (62k-record log).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_damage.py tests/test_log_blocks.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_log_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/r03_log_tests.log; exit 1; }
tail -2 gpurun_out/r03_log_tests.log
timeout -k 10 60 python tools/probe/log_probe.py 60000 --stamps --slots=2 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_logread_prof -o run -- python3 tools/probe/log_probe.py 60000 --read > gpurun_out/r03_logread_prof.log 2>&1 || { echo "log prof failed"; tail gpurun_out/r03_logread_prof.log; exit 1; }
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/r03_logread_prof/run_kernel_stats.csv')):
    print(r['Name'].split('(')[0][-40:], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])
"
