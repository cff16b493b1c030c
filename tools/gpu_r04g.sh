#!/bin/bash
# Round-4: WAL read/gather tests, then the WAL read path's kernel trace.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${T:-"tests/test_damage.py tests/test_log_blocks.py"}
timeout -k 10 600 python -u -m pytest $T -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_g.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/pytest_g.log; exit 1; }
tail -2 gpurun_out/pytest_g.log
bash tools/gpu_r04.sh logprof
