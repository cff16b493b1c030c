#!/bin/bash
# Round-4: the WAL walk's tests and branches on the scalar unit: log tests,
# then the verify's phase stamps and kernel trace.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} && mkdir -p gpurun_out && export TMPDIR=/tmp
. tools/gpu_r04_prof.sh none
T="tests/test_damage.py tests/test_log_blocks.py"
timeout -k 10 600 python -u -m pytest $T -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_q.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/pytest_q.log; exit 1; }
tail -2 gpurun_out/pytest_q.log
timeout -k 10 200 python tools/probe/log_probe.py 60000 --stamps --slots=2 > gpurun_out/q_stamps.log 2>&1 || { tail -20 gpurun_out/q_stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/q_stamps.log | tail -14
D=gpurun_out/q_logread; rm -rf $D
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 tools/probe/log_probe.py 60000 --read > $D.log 2>&1 \
  || { echo "log prof failed"; tail -20 $D.log; exit 1; }
grep "us/call" $D.log; stats $D
