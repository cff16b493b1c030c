# Round 3: WAL verify tests + timing (+ engine tests) on one GPU.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_damage.py tests/test_log_blocks.py tests/test_engine.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_log_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/r03_log_tests.log; exit 1; }
tail -2 gpurun_out/r03_log_tests.log
timeout -k 10 60 python tools/probe/log_probe.py 60000 --read 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_logread_prof -o run -- python3 tools/probe/log_probe.py 60000 --read > gpurun_out/r03_logread_prof.log 2>&1 || { echo "log prof failed"; exit 1; }
find gpurun_out/r03_logread_prof -name '*kernel_stats.csv' -exec cat {} \; | cut -d, -f1-4 | cut -c1-60,200-
