#!/bin/bash
# rocprofv3 over the engine bench (GPU box): kernel traces of the isolated
# (ordered) and the pipelined headline, then PMC passes, one counter group per
# run, over isolated launches. Outputs under gpurun_out/prof_engine/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
OUT="$R/gpurun_out/prof_engine"
mkdir -p "$OUT"
run() {  # name, rocprofv3 args..., -- cmd
  local name=$1; shift
  timeout -k 10 240 rocprofv3 "$@" > "$OUT/$name.log" 2>&1 || { echo "rocprofv3 $name failed"; tail -20 "$OUT/$name.log"; exit 1; }
}
run iso --kernel-trace --stats --output-format csv -d "$OUT/iso" -o run -- python3 "$R/bench.py" --isolated 200
run pipe --kernel-trace --stats --output-format csv -d "$OUT/pipe" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-split
i=0
for grp in "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAVES" \
           "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VMEM SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  run pmc$i --pmc $grp --output-format csv -d "$OUT/pmc$i" -o run -- python3 "$R/bench.py" --isolated 64
done
echo done
