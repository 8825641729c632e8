#!/bin/bash
# One iteration on the GPU box:  bash tools/iter.sh TAG [STEP...]
#   tests:  the -m gpu parity suite (stops at the first failure)
#   quick:  headline kernel time (configs 3 / 2 / 4 and families, no other legs)
#   trace:  rocprofv3 kernel-trace summary of the quick bench
#   cls:    per-class profile (tools/class_prof.sh)
#   var:    quick bench per DAV1D_GPU_LIB_VARIANT in $VARIANTS
# Every step has its own time limit; the script stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-it}
shift
STEPS=${*:-"tests quick"}
O=$R/gpurun_out/it_$TAG
mkdir -p "$O"
cd "$R"
Q="--no-cpu --steps 30 --warmup 3 --no-tiles --no-intra --no-recorder --no-grain --no-cdef --no-superres --no-lpf --no-lr"
for s in $STEPS; do
    case $s in
    tests)
        echo "[it] tests" >&2
        timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
            > "$O/gputest.log" 2>&1 || { echo "tests failed" >&2; tail -30 "$O/gputest.log"; exit 1; }
        tail -2 "$O/gputest.log"
        ;;
    quick)
        echo "[it] quick" >&2
        timeout -k 10 300 python3 bench.py $Q > "$O/quick.json" 2> "$O/quick.err" \
            || { echo "bench failed" >&2; tail -20 "$O/quick.err"; exit 1; }
        python3 -c "import json,sys; d=json.load(open('$O/quick.json')); r=d['roofline']; print('4k', r['kernel_us'], r['frac'], {k: v['kernel_us'] for k, v in d.get('configs', {}).items()}, {k: v['kernel_us'] for k, v in d.get('families', {}).items()})"
        ;;
    trace)
        echo "[it] trace" >&2
        cd /tmp && export TMPDIR=/tmp
        timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv \
            -- python3 "$R/bench.py" $Q --no-families > "$O/trace.log" 2>&1 || { echo "trace failed" >&2; exit 1; }
        cd "$R"
        head -12 "$O/trace/run_kernel_stats.csv"
        ;;
    cls)
        echo "[it] cls" >&2
        timeout -k 10 800 bash tools/class_prof.sh "$TAG" > "$O/cls.log" 2>&1 || { echo "cls failed" >&2; tail -20 "$O/cls.log"; exit 1; }
        cat "$O/cls.log" | tail -60
        ;;
    rec)
        echo "[it] rec" >&2
        DAV1D_GPU_REC_TIMING=1 timeout -k 10 300 python3 bench.py --no-cpu --steps 5 --warmup 1 --no-families --no-configs --no-tiles --no-intra \
            --no-grain --no-cdef --no-superres --no-lpf --no-lr > "$O/rec.json" 2> "$O/rec.err" || { echo "rec failed" >&2; tail -20 "$O/rec.err"; exit 1; }
        python3 -c "import json; d=json.load(open('$O/rec.json')); print(json.dumps(d['recorder']))"
        grep "^recorder" "$O/rec.err" | tail -14
        ;;
    recpin)   # the recorder's staging allocation (DAV1D_GPU_REC_PIN), bench recorder leg each
        for m in default nc; do
            DAV1D_GPU_REC_PIN=$m timeout -k 10 300 python3 bench.py --no-cpu --steps 5 --warmup 1 --no-families --no-configs --no-tiles --no-intra \
                --no-grain --no-cdef --no-superres --no-lpf --no-lr > "$O/recpin_$m.json" 2> "$O/recpin_$m.err" || { echo "recpin $m failed" >&2; tail -20 "$O/recpin_$m.err"; exit 1; }
            python3 -c "import json; d=json.load(open('$O/recpin_$m.json'))['recorder']; print('$m', d['flush_host_ms'], d['flush_device_ms'], d['frame_threads']['flush_host_ms_per_frame'], d['bit_exact_vs_oracle'], d['frame_threads']['bit_exact_vs_oracle'])"
        done
        ;;
    intra)   # the intra wavefront leg for the product build and each of $IVARIANTS
        for v in base $IVARIANTS; do
            if [ "$v" = base ]; then unset DAV1D_GPU_LIB_VARIANT; else export DAV1D_GPU_LIB_VARIANT=$v; fi
            timeout -k 10 400 python3 bench.py --no-cpu --steps 5 --warmup 1 --no-families --no-configs --no-tiles \
                --no-recorder --no-grain --no-cdef --no-superres --no-lpf --no-lr > "$O/intra_$v.json" 2> "$O/intra_$v.err" \
                || { echo "intra $v failed" >&2; tail -5 "$O/intra_$v.err"; exit 1; }
            python3 -c "import json; d=json.load(open('$O/intra_$v.json'))['intra_wavefront']; print('$v', {k: (x['ms_per_frame'], x['us_per_level'], x['bit_exact_vs_oracle']) for k, x in d.items()})"
        done
        unset DAV1D_GPU_LIB_VARIANT
        ;;
    vtests)   # the intra wavefront / recorder / chain GPU tests against each of $IVARIANTS
        for v in $IVARIANTS; do
            DAV1D_GPU_LIB_VARIANT=$v timeout -k 10 900 python3 -u -m pytest tests/test_gpu_intra_frame.py tests/test_gpu_recorder.py \
                tests/test_gpu_chain.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/vtests_$v.log" 2>&1 \
                || { echo "vtests $v failed" >&2; tail -30 "$O/vtests_$v.log"; exit 1; }
            echo "$v $(tail -1 "$O/vtests_$v.log")"
        done
        ;;
    superres)   # the super-res frame tier's GPU tests and its bench leg
        timeout -k 10 600 python3 -u -m pytest tests/test_gpu_superres.py -m gpu -x -q --timeout 300 --timeout-method thread \
            > "$O/superres_tests.log" 2>&1 || { echo "superres tests failed" >&2; tail -30 "$O/superres_tests.log"; exit 1; }
        tail -1 "$O/superres_tests.log"
        timeout -k 10 300 python3 bench.py --no-cpu --steps 20 --warmup 2 --no-families --no-configs --no-tiles --no-intra \
            --no-recorder --no-grain --no-cdef --no-lpf --no-lr > "$O/superres.json" 2> "$O/superres.err" \
            || { echo "superres bench failed" >&2; tail -20 "$O/superres.err"; exit 1; }
        python3 -c "import json; print(json.dumps(json.load(open('$O/superres.json'))['superres']))"
        ;;
    var)
        for v in base $VARIANTS; do
            if [ "$v" = base ]; then unset DAV1D_GPU_LIB_VARIANT; else export DAV1D_GPU_LIB_VARIANT=$v; fi
            timeout -k 10 300 python3 bench.py $Q --no-families --no-configs > "$O/var_$v.json" 2> "$O/var_$v.err" \
                || { echo "variant $v failed" >&2; tail -5 "$O/var_$v.err"; exit 1; }
            echo "$v $(grep -o '"kernel_us": [0-9.]*' "$O/var_$v.json" | head -1)"
        done
        unset DAV1D_GPU_LIB_VARIANT
        ;;
    esac
done
echo "[it] done" >&2
