#!/bin/bash
# WAL verify: GPU tests, per-iteration phase stamps (probe build), knob variants.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_log_blocks.py tests/test_damage.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/log_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/log_tests.log; exit 1; }
tail -1 gpurun_out/log_tests.log
for k in ${KNOBS:-0 1}; do timeout -k 10 60 python tools/probe/log_probe.py 60000 --stamps --knobs=$k 2>&1 | grep -v "amdgpu.ids" || exit 1; done
timeout -k 10 60 python tools/probe/log_probe.py 2000 2>&1 | grep -v "amdgpu.ids" || exit 1
