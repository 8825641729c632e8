#!/bin/bash
# WRITE_SIZE / FETCH_SIZE of the headline kernel per unit sort variant (GPU box):
#   bash tools/write_amp.sh  ->  gpurun_out/wa_<variant>/{write,fetch,trace}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
A="--steps 10 --warmup 2 --no-cpu --no-families --no-configs --no-tiles --no-intra --no-recorder --no-grain --no-cdef --no-lpf --no-lr"
for v in ${VARIANTS:-b16 b8 b32 b64 raster}; do
    case $v in
    b*) export DAV1D_GPU_SORT_BANDS=${v#b}; export DAV1D_GPU_SORT_MODE=txtp ;;
    *) export DAV1D_GPU_SORT_BANDS=16; export DAV1D_GPU_SORT_MODE=$v ;;
    esac
    O=$R/gpurun_out/wa_$v
    mkdir -p "$O"
    timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d "$O/write" -o run --output-format csv -- python3 "$R/bench.py" $A > "$O/write.log" 2>&1 || exit 1
    timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d "$O/fetch" -o run --output-format csv -- python3 "$R/bench.py" $A > "$O/fetch.log" 2>&1 || exit 1
    timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- python3 "$R/bench.py" $A > "$O/trace.log" 2>&1 || exit 1
    echo "[wa] $v done" >&2
done
