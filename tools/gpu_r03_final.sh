#!/bin/bash
# Round-3 close: the log tests with ReadRecord's profile and stamps, then the full check.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" && bash tools/gpu_r03_asm2.sh && bash tools/gpu_r03_check.sh
