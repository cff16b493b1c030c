#!/bin/bash
# Round-4: vector-loaded descriptors in the ragged walk: every ragged user's
# tests, then the engine shapes and the SST forms.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} && mkdir -p gpurun_out && export TMPDIR=/tmp
T="tests/test_engine_general.py tests/test_gpu_parity.py tests/test_sst_table.py tests/test_damage.py tests/test_log_blocks.py tests/test_engine.py"
timeout -k 10 600 python -u -m pytest $T -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_l.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/pytest_l.log; exit 1; }
tail -2 gpurun_out/pytest_l.log
timeout -k 10 400 python tools/probe/engine_shapes.py --cases sst4271_16k,rand2000_62k,u4096_65k,wal32k_2k > gpurun_out/shapes_l.log 2>&1 || { tail -20 gpurun_out/shapes_l.log; exit 1; }
grep -v amdgpu.ids gpurun_out/shapes_l.log | cut -c1-200
for A in "512 --form=2 --tables=32" "512 --form=1" "512 --form=3 --tables=32"; do
  timeout -k 10 120 python tools/probe/sst_probe.py $A 2>&1 | grep "us/call" || exit 1
done
