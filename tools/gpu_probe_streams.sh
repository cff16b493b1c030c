#!/bin/bash
# probe.py cases at 1 and 2 streams. Usage: PROBES="v780 k8204" bash tools/gpu_probe_streams.sh
set -o pipefail
mkdir -p gpurun_out
P=${PROBES:-"v780 v781 v782 v812 v783 v768 v17152 v16 16/CU readbw 41MB warm"}
timeout -k 10 200 python tools/probe.py $P > gpurun_out/ps1.txt 2>&1 && \
timeout -k 10 200 python tools/probe.py --streams=2 $P > gpurun_out/ps2.txt 2>&1; rc=$?
cat gpurun_out/ps1.txt gpurun_out/ps2.txt; exit $rc
