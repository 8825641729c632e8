#!/bin/bash
# Kernel time per unit sort order (workload.SORT_MODE), GPU box.
R=${GRAFT_REPO_ROOT:-$(pwd)}
for m in ${MODES:-txtp block raster txblk txtp}; do
    DAV1D_GPU_SORT_MODE=$m timeout -k 10 300 python3 "$R/bench.py" --no-cpu --no-families --steps 30 --warmup 3 --check $BENCH_ARGS > "$R/gpurun_out/sort_$m.json" 2> "$R/gpurun_out/sort_$m.err" || exit 1
    echo "$m $(grep -o '"kernel_us": [0-9.]*' "$R/gpurun_out/sort_$m.json") $(grep -o '"bit_exact_vs_oracle": [a-z]*' "$R/gpurun_out/sort_$m.json")"
done
