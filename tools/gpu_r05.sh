#!/bin/bash
# Round-5 evidence on one GPU. Every GPU step has its own time limit; the
# first failure ends the script.
#   bash tools/gpu_r05.sh [tests|bench|prof|logpmc|shapes|sst|edges]...
#   tests   every -m gpu test, then smoke()
#   bench   the driver's command (K = 20) and the default (K = 200) lines
#   prof    rocprofv3 kernel trace of isolated headline launches and of the
#           WAL read path
#   logpmc  PMC passes over the WAL verify (one counter group per run)
#   shapes  the engine's general shapes (tools/probe/engine_shapes.py)
#   sst     kernel traces of the SST forms
#   ceiling kernel trace of the production and read-ceiling kernels, overlapped
#   edges   the K = 20 region's edges (tools/probe/edges.py)
#   e2e     host-memory rates (tools/e2e_bench.py)
#   gate    parked queues / pair kernel for the last batches (tools/probe/gate_probe.py)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} && mkdir -p gpurun_out && export TMPDIR=/tmp
steps=${*:-tests bench}
want() { [[ " $steps " == *" $1 "* ]]; }
O=gpurun_out/r05
mkdir -p $O
stats() {  # kernel stats of a rocprofv3 csv output dir, short names
  python3 -c "
import csv,glob,sys
for f in glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        n = r['Name'].split('(')[0] if '(anonymous' not in r['Name'] else r['Name'].split('::')[2].split('(')[0]
        print('  ', n[-44:], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])
" $1
}
if want tests; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
    || { echo "gpu tests failed"; tail -40 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
    || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
if want bench; then
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20.json 2> $O/bench_k20.err \
    || { echo "bench failed"; tail -20 $O/bench_k20.err; exit 1; }
  cat $O/bench_k20.json
  timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err \
    || { echo "bench failed"; tail -20 $O/bench_default.err; exit 1; }
  cat $O/bench_default.json
fi
if want ceiling; then
  D=$O/ceiling_prof; rm -rf $D
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --ceiling-trace 200 --no-cpu-baseline --no-split --no-pmc > $D.log 2>&1 \
    || { echo "ceiling prof failed"; tail -20 $D.log; exit 1; }
  stats $D
  python3 tools/trace_period.py $D > $O/ceiling_periods.json && cat $O/ceiling_periods.json | head -80
fi
if want edges; then
  timeout -k 10 300 python tools/probe/edges.py --scopes=1,0,2 --scopes=0,0,2 --scopes=2,2,2 > $O/edges.log 2>&1 || { tail -20 $O/edges.log; exit 1; }
fi
if want edgesdev; then  # AQL rings in device memory (ROCr HSA_ALLOCATE_QUEUE_DEV_MEM)
  HSA_ALLOCATE_QUEUE_DEV_MEM=1 timeout -k 10 300 python tools/probe/edges.py --scopes=1,0,2 > $O/edgesdev.log 2>&1 || { tail -20 $O/edgesdev.log; exit 1; }
  grep -v amdgpu.ids $O/edgesdev.log | tail -12
  HSA_ALLOCATE_QUEUE_DEV_MEM=1 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > $O/bench_k20_devq.json 2> $O/bench_k20_devq.err || { tail -20 $O/bench_k20_devq.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_k20_devq.json')); print('devq k20', d['pct_hbm_peak'], d['roofline']['kernel_us_avg'], d['roofline']['pipelined']['period_us'])"
fi
if want edges; then
  cp gpurun_out/edges.json $O/edges.json
  grep -v amdgpu.ids $O/edges.log | tail -12
fi
if want prof; then
  D=$O/iso_prof; rm -rf $D
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --isolated 200 --no-cpu-baseline --no-split --no-pmc > $D.log 2>&1 \
    || { echo "iso prof failed"; tail -20 $D.log; exit 1; }
  stats $D
  D=$O/logread_prof; rm -rf $D
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 tools/probe/log_probe.py 60000 --read > $D.log 2>&1 \
    || { echo "log prof failed"; tail -20 $D.log; exit 1; }
  grep "us/call" $D.log; stats $D
fi
if want logpmc; then
  i=0; mkdir -p $O/logpmc
  for grp in "FETCH_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU" \
             "SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE"; do
    i=$((i+1)); D=$O/logpmc/p$i; rm -rf $D
    timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d $D -o run -- python3 tools/probe/log_probe.py 60000 > $D.log 2>&1 \
      || { echo "log pmc pass $i failed"; tail -5 $D.log; exit 1; }
  done
  python3 tools/pmc_table.py $O/logpmc > $O/logpmc.txt 2>&1 || true
  cat $O/logpmc.txt | head -40
fi
if want smallpmc; then
  i=0; mkdir -p $O/smallpmc
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
             "FETCH_SIZE GRBM_GUI_ACTIVE"; do
    i=$((i+1)); D=$O/smallpmc/p$i; rm -rf $D
    timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d $D -o run -- python3 tools/probe/engine_shapes.py --cases rand2000_62k --specs ${SMALL_SPECS:-3,2} --reps 4 > $D.log 2>&1 \
      || { echo "small pmc pass $i failed"; tail -5 $D.log; exit 1; }
  done
  python3 tools/pmc_table.py $O/smallpmc > $O/smallpmc.txt 2>&1 || true
  cat $O/smallpmc.txt | head -40
fi
if want group; then  # the grouped small-record walk: parity, then timing by spec
  timeout -k 10 400 python -u -m pytest tests/test_engine_general.py -x -v --timeout 150 --timeout-method thread -k "every_general or golden" > $O/group_tests.log 2>&1 \
    || { echo "group tests failed"; tail -60 $O/group_tests.log; exit 1; }
  tail -3 $O/group_tests.log
  timeout -k 10 300 python tools/probe/engine_shapes.py --cases rand2000_62k,sst4106_16k --specs 3,6,7,8 --reps 20 > $O/group_shapes.log 2>&1 || { echo shapes failed; tail -20 $O/group_shapes.log; exit 1; }
  grep -v amdgpu.ids $O/group_shapes.log | tail -12
fi
if want e2e; then  # the host-memory rates of DESIGN §8
  timeout -k 10 300 python tools/e2e_bench.py > $O/e2e.json 2> $O/e2e.err || { tail -20 $O/e2e.err; exit 1; }
  cat $O/e2e.json
fi
if want gate; then
  timeout -k 10 200 python tools/probe/gate_probe.py > $O/gate.log 2>&1 || { tail -20 $O/gate.log; exit 1; }
  grep -v amdgpu.ids $O/gate.log | tail -3
fi
if want snappy; then  # the device codecs (Snappy, Zstd decode): parity, throughput, kernel trace
  timeout -k 10 300 python -u -m pytest tests/test_snappy.py tests/test_zstd.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/snappy_tests.log 2>&1 \
    || { echo "snappy tests failed"; tail -40 $O/snappy_tests.log; exit 1; }
  tail -2 $O/snappy_tests.log
  timeout -k 10 200 python tools/snappy_bench.py > $O/snappy_bench.log 2>&1 || { tail -20 $O/snappy_bench.log; exit 1; }
  grep -v amdgpu.ids $O/snappy_bench.log | tail -2
  timeout -k 10 120 python3 tools/snappy_bench.py --write-zstd-frames $O/zframes.bin > /dev/null 2>&1 || { echo "zstd frames failed"; exit 1; }
  D=$O/snappy_prof; rm -rf $D
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 tools/snappy_bench.py --no-cpu --zstd-frames $O/zframes.bin > $D.log 2>&1 \
    || { echo "snappy prof failed"; tail -20 $D.log; exit 1; }
  stats $D
fi
if want snappypmc; then
  i=0; mkdir -p $O/snappypmc
  timeout -k 10 120 python3 tools/snappy_bench.py --write-zstd-frames $O/zframes.bin > /dev/null 2>&1 || { echo "zstd frames failed"; exit 1; }
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
             "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM" \
             "FETCH_SIZE GRBM_GUI_ACTIVE"; do
    i=$((i+1)); D=$O/snappypmc/p$i; rm -rf $D
    timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d $D -o run -- python3 tools/snappy_bench.py --no-cpu --steps 4 --warmup 1 --zstd-frames $O/zframes.bin > $D.log 2>&1 \
      || { echo "snappy pmc pass $i failed"; tail -5 $D.log; exit 1; }
  done
  python3 tools/pmc_table.py $O/snappypmc > $O/snappypmc.txt 2>&1 || true
  cat $O/snappypmc.txt | head -40
fi
if want shapes; then
  timeout -k 10 400 python tools/probe/engine_shapes.py > $O/engine_shapes.log 2>&1 || { echo shapes failed; tail -20 $O/engine_shapes.log; exit 1; }
  cp gpurun_out/engine_shapes.json $O/engine_shapes.json 2>/dev/null
  grep -v amdgpu.ids $O/engine_shapes.log | tail -40
fi
if want sst; then
  for A in "512 --form=3" "512 --form=3 --tables=32" "512 --form=2 --tables=32" "16384 --form=0"; do
    N=$(echo "$A" | tr -d ' =-' ); D=$O/sst_$N; rm -rf $D
    timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 tools/probe/sst_probe.py $A > $D.log 2>&1 \
      || { echo "sst prof failed"; tail -20 $D.log; exit 1; }
    grep "us/call" $D.log; stats $D
  done
fi
