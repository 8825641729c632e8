#!/bin/bash
# Round-4 profiles (through gpurun): kernel trace + PMC passes of the 8-bit
# headline with the CDEF / LR legs, the 10-bit config, then the intra
# wavefront's per-class flow trace and the recorder's host laps.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
FAST="--steps 10 --warmup 2 --no-families --no-configs --no-tiles --no-intra --no-recorder --no-grain --no-superres --no-lpf --no-check"
bash tools/prof.sh r4 $FAST || exit 1
bash tools/prof.sh r4_10bit --config 4k-10bit $FAST --no-cdef --no-lr || exit 1
mkdir -p gpurun_out/r4m
DAV1D_GPU_LIB_VARIANT=ftrace timeout -k 10 200 python -u tools/flow_trace.py > gpurun_out/r4m/flow_trace.json 2> gpurun_out/r4m/flow_trace.log || exit 1
DAV1D_GPU_REC_THREADS=8 bash tools/rec_host_ab.sh > gpurun_out/r4m/rec_host.log 2>&1
echo "[r4_prof] done"
