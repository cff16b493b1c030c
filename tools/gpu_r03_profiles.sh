#!/bin/bash
# Round-3 profile set (one GPU): rocprofv3 kernel traces of the headline
# kernel alone and overlapped, the SST shapes, the ragged shapes, and the PMC
# passes of the WAL verify. Summaries land in gpurun_out/r03_prof/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" && export TMPDIR=/tmp
O=gpurun_out/r03_prof; rm -rf $O; mkdir -p $O
kt() {  # name, command...
  local n=$1; shift
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- "$@" > $O/$n.log 2>&1 \
    || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }
  cp $O/$n/run_kernel_stats.csv $O/${n}_kernel_stats.csv
  python3 -c "
import csv
for r in csv.DictReader(open('$O/${n}_kernel_stats.csv')):
    print('$n', r['Name'].split('(')[0][-36:], r['Calls'], r['AverageNs'], r['MinNs'])"
}
kt engine_iso python3 bench.py --isolated 200
kt engine_pipe python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-split --no-pmc
kt sst512 python3 tools/probe/sst_probe.py 512
kt sst32x512 python3 tools/probe/sst_probe.py 512 --tables=32
kt ragged python3 tools/ragged_probe.py --reps 20
KNOBS=0 timeout -k 10 600 bash tools/gpu_r03_logpmc.sh > $O/log_pmc.txt 2>&1 || { echo "log pmc failed"; tail -5 $O/log_pmc.txt; exit 1; }
cat $O/log_pmc.txt
