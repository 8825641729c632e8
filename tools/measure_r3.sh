#!/bin/bash
# Round-3 GPU pass (GPU box):  bash tools/measure_r3.sh TAG [tests|bench|prof]...
#   tests: every -m gpu parity test, then smoke()
#   bench: the default bench line (headline + configs legs + breakdowns)
#   prof:  rocprofv3 kernel-trace + FETCH/WRITE PMC passes of the headline
#          kernel, 8-bit and 10-bit 4K (tools/prof.sh)
#   lrprof: kernel trace + SQ / FETCH / WRITE passes of k_lr_frame and k_cdef
# Each step has its own time limit; the script stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r3}
shift
STEPS=${*:-"tests bench prof"}
O=$R/gpurun_out/m_$TAG
mkdir -p "$O"
cd "$R"
for s in $STEPS; do
    case $s in
    tests)
        echo "[m] tests" >&2
        timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
            > "$O/gputest.log" 2>&1 || { echo "tests failed" >&2; tail -30 "$O/gputest.log"; exit 1; }
        tail -2 "$O/gputest.log"
        timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
            || { echo "smoke failed" >&2; cat "$O/smoke.log"; exit 1; }
        ;;
    bench)
        echo "[m] bench" >&2
        timeout -k 10 600 python3 bench.py > "$O/bench.json" 2> "$O/bench.err" \
            || { echo "bench failed" >&2; tail -20 "$O/bench.err"; exit 1; }
        ;;
    prof)
        echo "[m] prof" >&2
        P="--steps 20 --warmup 3 --no-families --no-configs --no-tiles --no-intra --no-recorder --no-grain --no-cdef --no-superres --no-lpf --no-lr"
        timeout -k 10 600 bash tools/prof.sh "$TAG" $P || exit 1
        timeout -k 10 600 bash tools/prof.sh "${TAG}_10bit" $P --config 4k-10bit || exit 1
        ;;
    lrprof)   # the post-filter frame kernels' SQ counters (two passes) and kernel trace
        echo "[m] lrprof" >&2
        cd /tmp && export TMPDIR=/tmp
        for t in lr cdef; do
            timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/pf_${TAG}_$t/trace" -o run --output-format csv \
                -- python3 "$R/tools/${t}_time.py" --no-check --iters 10 > "$O/pf_$t.trace.log" 2>&1 || exit 1
            timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
                -d "$R/gpurun_out/pf_${TAG}_$t/sq1" -o run --output-format csv \
                -- python3 "$R/tools/${t}_time.py" --no-check --iters 5 > "$O/pf_$t.sq1.log" 2>&1 || exit 1
            timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM \
                -d "$R/gpurun_out/pf_${TAG}_$t/sq2" -o run --output-format csv \
                -- python3 "$R/tools/${t}_time.py" --no-check --iters 5 > "$O/pf_$t.sq2.log" 2>&1 || exit 1
            timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pf_${TAG}_$t/fetch" -o run --output-format csv \
                -- python3 "$R/tools/${t}_time.py" --no-check --iters 5 > "$O/pf_$t.fetch.log" 2>&1 || exit 1
            timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/pf_${TAG}_$t/write" -o run --output-format csv \
                -- python3 "$R/tools/${t}_time.py" --no-check --iters 5 > "$O/pf_$t.write.log" 2>&1 || exit 1
        done
        cd "$R"
        ;;
    esac
done
echo "[m] done" >&2
