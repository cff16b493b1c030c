#!/bin/bash
# SST verify forms + WAL ReadRecord: GPU tests, timings, kernel durations.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_sst_table.py tests/test_damage.py tests/test_log_blocks.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sst_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/sst_tests.log; exit 1; }
tail -2 gpurun_out/sst_tests.log
for f in 1 2; do for n in 512 16384; do timeout -k 10 60 python tools/probe/sst_probe.py $n --form=$f 2>&1 | grep -v amdgpu.ids || exit 1; done; timeout -k 10 60 python tools/probe/sst_probe.py 512 --form=$f --tables=32 2>&1 | grep -v amdgpu.ids || exit 1; done
timeout -k 10 60 python tools/probe/log_probe.py 60000 --read 2>&1 | grep -v amdgpu.ids || exit 1
for f in 1 2; do
  n=512
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sstprof_f${f}_$n -o run -- python3 tools/probe/sst_probe.py $n --form=$f > gpurun_out/sstprof_f${f}_$n.log 2>&1 || { echo "prof $f $n failed"; tail -20 gpurun_out/sstprof_f${f}_$n.log; exit 1; }
  find gpurun_out/sstprof_f${f}_$n -name '*kernel_stats.csv' -exec cat {} \; | cut -d, -f1-4 | cut -c1-50,200-
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/logread_prof -o run -- python3 tools/probe/log_probe.py 60000 --read > gpurun_out/logread_prof.log 2>&1 || { echo "log prof failed"; exit 1; }
find gpurun_out/logread_prof -name '*kernel_stats.csv' -exec cat {} \; | cut -d, -f1-4 | cut -c1-50,200-
