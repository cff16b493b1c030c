#!/bin/bash
cd ${GRAFT_REPO_ROOT:-/root/repo} && mkdir -p gpurun_out
timeout -k 10 120 python tools/diag_hip.py lib-first 2>&1 | grep -v amdgpu.ids
timeout -k 10 120 python tools/diag_hip.py torch-first 2>&1 | grep -v amdgpu.ids
