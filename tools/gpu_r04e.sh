#!/bin/bash
# Round-4: SST/engine/parity device tests after the deferred-trailer walk,
# then the SST forms' timings and the speculative form's phase stamps.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${T:-"tests/test_sst_table.py tests/test_damage.py tests/test_engine_general.py tests/test_gpu_parity.py"}
timeout -k 10 600 python -u -m pytest $T -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_e.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/pytest_e.log; exit 1; }
tail -2 gpurun_out/pytest_e.log
rm -f gpurun_out/sst_e.log
for A in "512 --form=3 --stamps" "512 --form=3 --tables=32 --stamps" "512 --form=2" "512 --form=2 --tables=32" "16384 --form=0"; do
  timeout -k 10 120 python tools/probe/sst_probe.py $A >> gpurun_out/sst_e.log 2>&1 || { tail -20 gpurun_out/sst_e.log; exit 1; }
done
grep -v -e amdgpu.ids -e Warning -e nanmedian gpurun_out/sst_e.log
