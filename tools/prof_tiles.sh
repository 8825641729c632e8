#!/bin/bash
# PMC passes over the tile kernel (run on the GPU box): bash tools/prof_tiles.sh TAG [tile_time args]
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
O=$R/gpurun_out/ptile_$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
run() {
    local name=$1; shift
    timeout -k 10 120 rocprofv3 "$@" -d "$O/$name" -o run --output-format csv -- \
        python3 "$R/tools/tile_time.py" --only-tiles --iters 5 $ARGS > "$O/$name.log" 2>&1 || echo "pass $name failed" >&2
}
ARGS="$*"
run trace --kernel-trace --stats
run sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES
run sq2 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_BRANCH
run sq3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ SQ_IFETCH
run ta --pmc TA_BUSY_avr TA_TA_BUSY_sum
rocprofv3 -L > "$O/counters.txt" 2>&1 || true
