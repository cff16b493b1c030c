#!/bin/bash
# Round-4 check on one GPU: GPU tests, smoke, the driver's bench command and a
# kernel trace of the WAL read path (62k-record log). Every GPU step has its
# own time limit; the first failure ends the script.
#   bash tools/gpu_r04.sh [tests|bench|logprof|all]...
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
steps=${*:-all}
want() { [[ " $steps " == *" $1 "* || " $steps " == *" all "* ]]; }
if want tests; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
    || { echo "gpu tests failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
    || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
  tail -1 gpurun_out/smoke.log
fi
if want bench; then
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_k20.json 2> gpurun_out/bench_k20.err \
    || { echo "bench failed"; tail -20 gpurun_out/bench_k20.err; exit 1; }
  cat gpurun_out/bench_k20.json
fi
if want logprof; then
  for P in 0; do
    D=gpurun_out/r04_logread_prof
    rm -rf $D
    timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 tools/probe/log_probe.py 60000 --read > $D.log 2>&1 \
      || { echo "log prof failed"; tail -20 $D.log; exit 1; }
    grep -v amdgpu.ids $D.log | grep "log_" | tail -4
    python3 -c "
import csv,glob,sys
for f in glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        n = r['Name'].split('(')[0] if '(anonymous' not in r['Name'] else r['Name'].split('::')[2].split('(')[0]
        print('  ', n[-44:], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])
" $D
  done
fi
