#!/bin/bash
# Round 3 iteration: SST tests + timings, WAL tests + timings (+ gather), walk probe.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_sst_table.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_sst_tests.log 2>&1 || { echo SST TESTS FAILED; tail -30 gpurun_out/r03_sst_tests.log; exit 1; }
tail -1 gpurun_out/r03_sst_tests.log
for a in "512" "16384" "512 --tables=32"; do timeout -k 10 60 python tools/probe/sst_probe.py $a 2>&1 | grep -v amdgpu.ids || exit 1; done
rm -rf gpurun_out/r03_sstprof_16384
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_sstprof_16384 -o run -- python3 tools/probe/sst_probe.py 16384 > gpurun_out/r03_sstprof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r03_sstprof.log; exit 1; }
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/r03_sstprof_16384/run_kernel_stats.csv')):
    print('16384', r['Name'].split('(')[0][-34:], r['Calls'], r['AverageNs'], r['MinNs'])
"
timeout -k 10 300 python -u -m pytest tests/test_log_blocks.py tests/test_damage.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_log_tests.log 2>&1 || { echo LOG TESTS FAILED; tail -40 gpurun_out/r03_log_tests.log; exit 1; }
tail -1 gpurun_out/r03_log_tests.log
timeout -k 10 60 python tools/probe/log_probe.py 60000 --stamps --slots=4 2>&1 | grep -v amdgpu.ids || exit 1
rm -rf gpurun_out/r03_logread_prof
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_logread_prof -o run -- python3 tools/probe/log_probe.py 60000 --read > gpurun_out/r03_logread_prof.log 2>&1 || { echo "log prof failed"; tail gpurun_out/r03_logread_prof.log; exit 1; }
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/r03_logread_prof/run_kernel_stats.csv')):
    print(r['Name'].split('(')[0][-40:], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])
"
mkdir -p /tmp/wp && hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe/walk_probe.hip -o /tmp/wp/walk_probe 2>/dev/null && timeout -k 5 60 /tmp/wp/walk_probe 2048
