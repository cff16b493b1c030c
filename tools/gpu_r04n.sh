#!/bin/bash
# Round-4: ReadRecord by block groups, the aggregates left by the WAL emit:
# the log tests, then kernel traces of the WAL read path and the emit stamps.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} && mkdir -p gpurun_out && export TMPDIR=/tmp
. tools/gpu_r04_prof.sh none
T="tests/test_damage.py tests/test_log_blocks.py"
timeout -k 10 600 python -u -m pytest $T -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_n.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/pytest_n.log; exit 1; }
tail -2 gpurun_out/pytest_n.log
D=gpurun_out/n_logread; rm -rf $D
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 tools/probe/log_probe.py 60000 --read > $D.log 2>&1 \
  || { echo "log prof failed"; tail -20 $D.log; exit 1; }
grep "us/call" $D.log; stats $D
timeout -k 10 200 python tools/probe/log_probe.py 60000 --read --asm-stamps > gpurun_out/n_asm_stamps.log 2>&1 || { tail -20 gpurun_out/n_asm_stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/n_asm_stamps.log | tail -6
