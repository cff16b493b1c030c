#!/bin/bash
# Round-4 SST iteration: the SST and WAL device tests (verbose, per-test
# timeouts), then whole-table verify timings per form (1 fused, 2 two
# launches, 3 speculative) for one 2 MiB table and 32 of them, with a kernel
# trace of the speculative form.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${T:-"tests/test_sst_table.py tests/test_damage.py tests/test_log_blocks.py"}
timeout -k 10 600 python -u -m pytest $T -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_sst.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/pytest_sst.log; exit 1; }
tail -2 gpurun_out/pytest_sst.log
for F in 1 2 3; do
  timeout -k 10 120 python tools/probe/sst_probe.py 512 --form=$F >> gpurun_out/sst_forms.log 2>&1 || { echo probe failed; tail -20 gpurun_out/sst_forms.log; exit 1; }
  timeout -k 10 120 python tools/probe/sst_probe.py 512 --form=$F --tables=32 >> gpurun_out/sst_forms.log 2>&1 || { echo probe failed; tail -20 gpurun_out/sst_forms.log; exit 1; }
done
timeout -k 10 120 python tools/probe/sst_probe.py 16384 --form=0 >> gpurun_out/sst_forms.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/sst_forms.log
rm -rf gpurun_out/r04_sst_spec
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_sst_spec -o run -- python tools/probe/sst_probe.py 512 --form=3 --tables=32 > gpurun_out/r04_sst_spec.log 2>&1 || { echo prof failed; tail -20 gpurun_out/r04_sst_spec.log; exit 1; }
find gpurun_out/r04_sst_spec -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200
rm -rf gpurun_out/r04_sst_spec1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_sst_spec1 -o run -- python tools/probe/sst_probe.py 512 --form=3 > gpurun_out/r04_sst_spec1.log 2>&1 || { echo prof failed; exit 1; }
find gpurun_out/r04_sst_spec1 -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200
