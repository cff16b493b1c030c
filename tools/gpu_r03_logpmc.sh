#!/bin/bash
# PMC passes over the WAL verify kernel (tools/probe/log_probe.py, 60k-record log).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT="$R/gpurun_out/r03_pmc_log"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU" \
           "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- python3 "$R/tools/probe/log_probe.py" 60000 > "$OUT/p$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 - "$OUT" <<'PY'
import collections, csv, glob, sys
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(sys.argv[1] + '/p*/run_counter_collection.csv')):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name']
        name = k.split('::')[-1].split('(')[0]
        agg[name][r['Counter_Name']].append(float(r['Counter_Value']))
for name in sorted(agg):
    d = {c: sorted(v)[len(v) // 2] for c, v in agg[name].items()}
    print(name, ' '.join(f"{c}={x:.5g}" for c, x in sorted(d.items())))
PY
