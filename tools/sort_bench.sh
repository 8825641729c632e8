#!/bin/bash
# bench.py kernel time for several unit-sort band counts (GPU box).
R=${GRAFT_REPO_ROOT:-$(pwd)}
for b in ${BANDS:-16 8 4}; do
    DAV1D_GPU_SORT_BANDS=$b timeout -k 10 300 python3 "$R/bench.py" --no-cpu --steps 30 --warmup 3 > "$R/gpurun_out/sbench_$b.json" 2>/dev/null || exit 1
    echo "bands $b $(grep -o '"kernel_us": [0-9.]*' "$R/gpurun_out/sbench_$b.json")"
done
