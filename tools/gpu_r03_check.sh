#!/bin/bash
# Round-3 check on one GPU: GPU tests, smoke, the driver's bench command, and a
# kernel trace of the WAL read path (62k-record log).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
  || { echo "gpu tests failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
  || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_k20.json 2> gpurun_out/bench_k20.err \
  || { echo "bench failed"; tail -20 gpurun_out/bench_k20.err; exit 1; }
cat gpurun_out/bench_k20.json
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_logread_prof -o run -- python3 tools/probe/log_probe.py 60000 --read > gpurun_out/r03_logread_prof.log 2>&1 \
  || { echo "log prof failed"; tail -20 gpurun_out/r03_logread_prof.log; exit 1; }
find gpurun_out/r03_logread_prof -name '*kernel_stats.csv' -exec cat {} \; | cut -d, -f1-4 | cut -c1-60,200-
timeout -k 10 60 rocprofv3 -L > gpurun_out/r03_counters.txt 2>&1 || true
grep -o "TCC_EA0_RDREQ[A-Z_0-9]*\|TCC_EA_RDREQ[A-Z_0-9]*\|TCC_BUBBLE[A-Z_0-9]*\|MALL[A-Z_0-9]*\|TCC_EA0_RD[A-Z_0-9]*" gpurun_out/r03_counters.txt | sort -u | head -20 || true
timeout -k 10 240 python tools/e2e_bench.py --blocks 10000 250000 > gpurun_out/r03_e2e.json 2> gpurun_out/r03_e2e.err || { echo "e2e failed"; tail -5 gpurun_out/r03_e2e.err; exit 1; }
cat gpurun_out/r03_e2e.json
