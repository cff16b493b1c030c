#!/bin/bash
# Round-4: engine tests after the ordered-shape rule, auto shapes.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine.py tests/test_engine_general.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_i.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/pytest_i.log; exit 1; }
tail -2 gpurun_out/pytest_i.log
timeout -k 10 300 python tools/probe/engine_shapes.py --specs=-1 > gpurun_out/shapes_i.log 2>&1 || { tail -20 gpurun_out/shapes_i.log; exit 1; }
cp gpurun_out/engine_shapes.json gpurun_out/engine_shapes_auto.json
grep -v amdgpu.ids gpurun_out/shapes_i.log | cut -c1-220
