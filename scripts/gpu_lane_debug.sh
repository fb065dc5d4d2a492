cd $GRAFT_REPO_ROOT && for m in 0 1 2; do WVG_LANE_KERNEL=$m timeout -k 10 120 python scripts/lane_debug.py 2>&1 | grep -v amdgpu.ids || exit 1; done
