#!/bin/bash
# Round-4: the SST heads' filter lookup beside the index CRC: every SST test
# (all forms, the reference damage cases), then the forms' timings.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} && mkdir -p gpurun_out && export TMPDIR=/tmp
. tools/gpu_r04_prof.sh none
T="tests/test_sst_table.py tests/test_damage.py tests/test_gpu_parity.py tests/test_engine_general.py"
timeout -k 10 600 python -u -m pytest $T -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_r.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/pytest_r.log; exit 1; }
tail -2 gpurun_out/pytest_r.log
for A in "512 --form=3" "512 --form=3 --tables=32" "512 --form=1" "512 --form=2 --tables=32"; do
  N=$(echo "$A" | tr -d ' =-' ); D=gpurun_out/r_sst_$N; rm -rf $D
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 tools/probe/sst_probe.py $A > $D.log 2>&1 \
    || { echo "sst prof failed"; tail -20 $D.log; exit 1; }
  grep "us/call" $D.log; stats $D
done
timeout -k 10 120 python tools/probe/sst_probe.py 512 --form=3 --stamps > gpurun_out/r_sst_stamps.log 2>&1 || { tail -20 gpurun_out/r_sst_stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r_sst_stamps.log | tail -12
