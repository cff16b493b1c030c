#!/bin/bash
# Whole-SSTable verify: GPU tests of both forms, then phase stamps.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_sst_table.py tests/test_damage.py tests/test_log_blocks.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sst_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/sst_tests.log; exit 1; }
tail -1 gpurun_out/sst_tests.log
for f in 1 2; do for n in 512 16384; do timeout -k 10 60 python tools/probe/sst_probe.py $n --form=$f --stamps 2>&1 | grep -v "amdgpu.ids\|RuntimeWarning\|nanmedian" || exit 1; done; timeout -k 10 60 python tools/probe/sst_probe.py 512 --form=$f --tables=32 2>&1 | grep -v amdgpu.ids || exit 1; done
