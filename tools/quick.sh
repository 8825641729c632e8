#!/bin/bash
# Quick GPU check of the product build: bench kernel time (8 and 10 bit)
# with the oracle check of rank 0's frame.
R=${GRAFT_REPO_ROOT:-$(pwd)}
for c in ${CONFIGS:-4k 4k-10bit}; do
    timeout -k 10 300 python3 "$R/bench.py" --no-cpu --no-families --steps 30 --warmup 3 --check --config $c > "$R/gpurun_out/q_$c.json" 2> "$R/gpurun_out/q_$c.err" || exit 1
    echo "$c $(grep -o '"kernel_us": [0-9.]*' "$R/gpurun_out/q_$c.json") $(grep -o '"bit_exact_vs_oracle": [a-z]*' "$R/gpurun_out/q_$c.json")"
done
