#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" && mkdir -p gpurun_out build
hipcc --offload-arch=gfx950 -O3 tools/launch_probe.hip -o build/launch_probe 2>/dev/null
timeout -k 10 60 ./build/launch_probe | tee gpurun_out/launch_probe.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/lprof" -o run --output-format csv -- "$R/build/launch_probe" > /dev/null 2>&1
cat "$R"/gpurun_out/lprof/run_kernel_stats.csv | cut -d, -f1-4,6-7
