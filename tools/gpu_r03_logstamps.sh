cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for k in ${KNOBS:-0}; do
timeout -k 5 25 python tools/probe/log_probe.py 60000 --stamps --slots=${SLOTS:-2} --knobs=$k 2>&1 | grep -v amdgpu.ids || exit 1
done
