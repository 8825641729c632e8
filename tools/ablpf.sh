#!/bin/bash
# deblocking A/B per variant library (ABV): the LPF and chain GPU tests, then the bench's loop_filter leg
O=gpurun_out/${1:-ablpf}; mkdir -p $O
F="--steps 100 --no-families --no-configs --no-tiles --no-intra --no-recorder --no-grain --no-cdef --no-lr --no-superres --no-cpu"
for v in base $ABV; do
    if [ "$v" = base ]; then unset DAV1D_GPU_LIB_VARIANT; else export DAV1D_GPU_LIB_VARIANT=$v; fi
    timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu -x tests/test_gpu_lpf.py tests/test_gpu_chain.py > $O/test_$v.log 2>&1 \
        || { echo "ablpf tests $v failed"; tail -n 5 $O/test_$v.log; exit 1; }
    timeout -k 10 300 python -u bench.py $F > $O/bench_$v.json 2> $O/bench_$v.log || { echo "ablpf bench $v failed"; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_$v.json'))['loop_filter']; print('ablpf $v', d['us_per_frame'], d['bit_exact_vs_oracle'], '$(tail -n 1 $O/test_$v.log | tr -d =)')"
done
