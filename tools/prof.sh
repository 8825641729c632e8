#!/bin/bash
# Profiling recipe for the batch kernels (run ON the GPU box via gpurun):
#   bash tools/prof.sh TAG [bench.py args...]
# One kernel-trace pass plus separate PMC passes (FETCH_SIZE and WRITE_SIZE
# cannot share a pass), each its own rocprofv3 run with the program directly
# after `--`.  Output: gpurun_out/prof_TAG/<pass>/run_*.csv; summarise with
# tools/pmc_summary.py.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
shift
ARGS=${*:-"--steps 10 --warmup 2"}
O=$R/gpurun_out/prof_$TAG
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
run() {
    local name=$1
    shift
    echo "[prof] $name" >&2
    timeout -k 10 300 rocprofv3 "$@" -d "$O/$name" -o run --output-format csv -- \
        python3 "$R/bench.py" --no-cpu $ARGS > "$O/$name.log" 2>&1
}
run trace --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES
run sq2 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES
echo "[prof] done" >&2
