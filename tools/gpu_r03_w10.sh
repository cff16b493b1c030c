#!/bin/bash
# Engine pair-kernel shapes (8x3 vs 10x2 / 12x2 waves x chains) in isolation,
# then the round-3 check.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 180 python -u tools/probe/iso_probe.py pk_pair_pipe1 pk_w10c2_pipe1 pk_w10c2 pk_w12c2_pipe1 pk_w10c2_pipe1_s2 pk_pair_pipe1 > gpurun_out/iso_w10.log 2>&1 \
  || { echo "iso probe failed"; tail -20 gpurun_out/iso_w10.log; exit 1; }
cat gpurun_out/iso_w10.log
bash tools/gpu_r03_check.sh
