#!/bin/bash
# Recorder host-phase timing on the GPU box's CPUs (no GPU used):
#   bash tools/rec_host_ab.sh [VARIANT...]     (base = the product build)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for v in base "$@" base "$@"; do
    if [ "$v" = base ]; then unset DAV1D_GPU_LIB_VARIANT; else export DAV1D_GPU_LIB_VARIANT=$v; fi
    echo "== $v (nproc $(nproc))"
    DAV1D_GPU_REC_HOSTONLY=1 DAV1D_GPU_REC_TIMING=1 timeout -k 10 300 python3 tools/rec_host_time.py --reps 4 2>&1 | tail -9 || exit 1
done
