#!/bin/bash
# Round-4: WAL verify against the number of record (worker) waves per CU
# (probe knob bits 8-11 idle that many of the 14), A/B in one process each.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} && mkdir -p gpurun_out && export TMPDIR=/tmp
rm -f gpurun_out/workers_ab.log
for K in 512 1024 1536 2048; do
  timeout -k 10 200 python tools/probe/log_probe.py 60000 --stamps --slots=2 --knobs=$K > gpurun_out/wk_$K.log 2>&1 || { tail -20 gpurun_out/wk_$K.log; exit 1; }
  grep -E "probe lib knobs|slot" gpurun_out/wk_$K.log | head -8 >> gpurun_out/workers_ab.log
done
cat gpurun_out/workers_ab.log
