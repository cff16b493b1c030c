#!/bin/bash
# Round-4: engine general tests, WAL verify phase stamps, auto engine shapes.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_general.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_h.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/pytest_h.log; exit 1; }
tail -2 gpurun_out/pytest_h.log
timeout -k 10 200 python tools/probe/log_probe.py 60000 --stamps --slots=2 > gpurun_out/log_stamps.log 2>&1 || { tail -20 gpurun_out/log_stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/log_stamps.log
timeout -k 10 300 python tools/probe/engine_shapes.py --cases rand2000_62k,sst4271_16k --specs=-1 > gpurun_out/shapes_h.log 2>&1 || { tail -20 gpurun_out/shapes_h.log; exit 1; }
grep -v amdgpu.ids gpurun_out/shapes_h.log | cut -c1-220
