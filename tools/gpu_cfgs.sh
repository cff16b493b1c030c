#!/bin/bash
# Parity tests, probe subset, and bench lines for every config.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/probe.py ${PROBES:-v780 v1804 v17152 "readbw 41MB cold 16"} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/probe_iter.txt
for c in headline wal32k blocks1m; do
  timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-100} --warmup 10 --no-cpu-baseline > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { echo "bench $c failed"; tail -20 gpurun_out/bench_$c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$c.json'));print('$c', d['value'], d['unit'], d['roofline']['kernel_us_avg'], 'us', d['roofline']['frac'])"
done
