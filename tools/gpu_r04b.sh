#!/bin/bash
# Round-4 iteration: engine + WAL tests, the engine's ragged shapes A/B, the
# WAL read path's kernel trace. Arguments: pytest files (default: engine,
# damage, log).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${T:-"tests/test_engine.py tests/test_engine_general.py tests/test_damage.py tests/test_log_blocks.py"}
timeout -k 10 600 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/pytest_iter.log; exit 1; }
tail -2 gpurun_out/pytest_iter.log
timeout -k 10 400 python tools/probe/engine_shapes.py ${SHAPES:+--cases $SHAPES} > gpurun_out/engine_shapes.log 2>&1 || { echo shapes failed; tail -20 gpurun_out/engine_shapes.log; exit 1; }
grep -v amdgpu.ids gpurun_out/engine_shapes.log
bash tools/gpu_r04.sh logprof
