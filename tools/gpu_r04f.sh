#!/bin/bash
# Round-4 headline: the driver's bench command twice, the engine edges probe.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine.py tests/test_engine_general.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_f.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/pytest_f.log; exit 1; }
tail -2 gpurun_out/pytest_f.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_k20_$i.json 2> gpurun_out/bench_k20_$i.err \
    || { echo "bench failed"; tail -20 gpurun_out/bench_k20_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('pipelined'))" gpurun_out/bench_k20_$i.json
done
timeout -k 10 200 python tools/probe/edges.py > gpurun_out/edges.log 2>&1 || { tail -20 gpurun_out/edges.log; exit 1; }
grep -v amdgpu.ids gpurun_out/edges.log | tail -30
