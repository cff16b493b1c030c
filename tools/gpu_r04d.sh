#!/bin/bash
# Round-4: WAL/SST device tests, SST phase stamps of the speculative form, the
# WAL read path's kernel traces under both verify paths.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${T:-"tests/test_log_blocks.py tests/test_damage.py tests/test_sst_table.py"}
timeout -k 10 600 python -u -m pytest $T -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_d.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/pytest_d.log; exit 1; }
tail -2 gpurun_out/pytest_d.log
rm -f gpurun_out/sst_stamps.log
timeout -k 10 120 python tools/probe/sst_probe.py 512 --form=3 --stamps >> gpurun_out/sst_stamps.log 2>&1 || { tail -20 gpurun_out/sst_stamps.log; exit 1; }
timeout -k 10 120 python tools/probe/sst_probe.py 512 --form=3 --tables=32 --stamps >> gpurun_out/sst_stamps.log 2>&1 || { tail -20 gpurun_out/sst_stamps.log; exit 1; }
timeout -k 10 120 python tools/probe/sst_probe.py 512 --form=1 --stamps >> gpurun_out/sst_stamps.log 2>&1 || { tail -20 gpurun_out/sst_stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/sst_stamps.log
bash tools/gpu_r04.sh logprof
