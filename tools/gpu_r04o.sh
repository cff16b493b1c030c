#!/bin/bash
# Round-4: the K=20 headline and the t0 -> first dispatch edge against the
# number of HIP hardware queues of the process (HIP's default 4 beside the
# engine's own 3 HSA queues), interleaved A/B on one box.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} && mkdir -p gpurun_out && export TMPDIR=/tmp
rm -f gpurun_out/hwq_ab.log
for rep in 1 2 3; do
  for Q in 4 1 2; do
    GPU_MAX_HW_QUEUES=$Q timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-pmc --no-split > gpurun_out/hq.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/hq.json')); print('Q', sys.argv[1], round(d['value']/ (8000/1.073741824)*100, 2), d['ms_per_step'])" $Q >> gpurun_out/hwq_ab.log
  done
done
cat gpurun_out/hwq_ab.log
for Q in 4 1; do
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 120 python tools/probe/edges.py > gpurun_out/edges_q$Q.log 2>&1 || { tail -5 gpurun_out/edges_q$Q.log; exit 1; }
  echo "Q=$Q"; grep -v amdgpu.ids gpurun_out/edges_q$Q.log | grep -E "^[a-z_]+ 20 " | cut -c1-300
done
