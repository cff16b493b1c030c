cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for k in 1 4 5; do timeout -k 10 60 python tools/probe/log_probe.py 60000 --stamps --knobs=$k 2>&1 | grep -v amdgpu.ids || exit 1; done
