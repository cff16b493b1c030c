#!/bin/bash
# Round-4: the K=20 headline's sensitivity to the warm-up length (A/B, one box).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} && mkdir -p gpurun_out && export TMPDIR=/tmp
rm -f gpurun_out/warm_ab.log
for rep in 1 2 3; do
  for W in 150 20 2; do
    timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --warmup-ms $W --no-cpu-baseline --no-pmc --no-split > gpurun_out/wab.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/wab.json')); print(sys.argv[1], round(d['value']/ (8000/1.073741824)*100, 2), d['ms_per_step'])" $W >> gpurun_out/warm_ab.log
  done
done
cat gpurun_out/warm_ab.log
