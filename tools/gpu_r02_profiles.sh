#!/bin/bash
# Round-2 kernel traces of the SST forms and the WAL read path (rocprofv3).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
run() {  # name, command...
  local name=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_$name -o run -- "$@" > gpurun_out/p_$name.log 2>&1 || { echo "prof $name failed"; tail -5 gpurun_out/p_$name.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/p_$name.log | grep "us/call" || true
}
run sst512_fused python3 tools/probe/sst_probe.py 512 --form=1
run sst512_two python3 tools/probe/sst_probe.py 512 --form=2
run sst16384_two python3 tools/probe/sst_probe.py 16384 --form=2
run sst32x512_two python3 tools/probe/sst_probe.py 512 --form=2 --tables=32
run logread python3 tools/probe/log_probe.py 60000 --read
