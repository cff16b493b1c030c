#!/bin/bash
# Iteration pass: GPU parity tests, probe table, per-wave timeline, bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/probe.py ${PROBES:-"v256" "v768" "v896" "readbw 41MB cold 16"} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/probe_iter.txt
timeout -k 10 300 python tools/timeline.py ${TIMELINE:-320 832 960} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/timeline_iter.txt
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 2 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench failed; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
[ -n "$E2E" ] && { timeout -k 10 300 python tools/e2e_bench.py > gpurun_out/e2e.json 2> gpurun_out/e2e.err || { echo e2e failed; tail -20 gpurun_out/e2e.err; exit 1; }; cat gpurun_out/e2e.json; }
exit 0
