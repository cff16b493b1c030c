#!/bin/bash
# One-item-per-thread ReadRecord: the log tests, its kernel trace, the engine
# shape probe, then the round-3 check.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_damage.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/asm_tests.log 2>&1 \
  || { echo "damage tests failed"; tail -30 gpurun_out/asm_tests.log; exit 1; }
tail -2 gpurun_out/asm_tests.log
rm -rf gpurun_out/r03_asm_prof
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_asm_prof -o run -- python3 tools/probe/log_probe.py 60000 --read > gpurun_out/r03_asm_prof.log 2>&1 \
  || { echo "log prof failed"; tail -20 gpurun_out/r03_asm_prof.log; exit 1; }
find gpurun_out/r03_asm_prof -name '*kernel_stats.csv' -exec cat {} \; | cut -d, -f1-4 | cut -c1-60,200-
timeout -k 10 180 python -u tools/probe/iso_probe.py pk_pair_pipe1 pk_w10c2_pipe1 pk_w10c2 pk_w12c2_pipe1 pk_w10c2_pipe1_s2 pk_pair_pipe1 > gpurun_out/iso_w10.log 2>&1 \
  || { echo "iso probe failed"; tail -20 gpurun_out/iso_w10.log; exit 1; }
cat gpurun_out/iso_w10.log
bash tools/gpu_r03_check.sh
