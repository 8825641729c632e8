#!/bin/bash
# bench.py kernel time for the product build and each variant (GPU box).
R=${GRAFT_REPO_ROOT:-$(pwd)}
for v in base ${VARIANTS} base; do
    if [ "$v" = base ]; then unset DAV1D_GPU_LIB_VARIANT; else export DAV1D_GPU_LIB_VARIANT=$v; fi
    timeout -k 10 300 python3 "$R/bench.py" --no-cpu --steps 30 --warmup 3 --no-families $BENCH_ARGS > "$R/gpurun_out/vbench_$v.json" 2> "$R/gpurun_out/vbench_$v.err" || exit 1
    echo "$v $(grep -o '"kernel_us": [0-9.]*' "$R/gpurun_out/vbench_$v.json")"
done
