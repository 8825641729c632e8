#!/bin/bash
# super-res A/B per variant library (ABV): the super-res and chain GPU tests, then the bench's superres leg
O=gpurun_out/${1:-absr}; mkdir -p $O
F="--steps 100 --no-families --no-configs --no-tiles --no-intra --no-recorder --no-grain --no-cdef --no-lr --no-lpf --no-cpu"
for v in base $ABV; do
    if [ "$v" = base ]; then unset DAV1D_GPU_LIB_VARIANT; else export DAV1D_GPU_LIB_VARIANT=$v; fi
    timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu -x tests/test_gpu_superres.py tests/test_gpu_chain.py > $O/test_$v.log 2>&1 \
        || { echo "absr tests $v failed"; tail -n 5 $O/test_$v.log; exit 1; }
    timeout -k 10 300 python -u bench.py $F > $O/bench_$v.json 2> $O/bench_$v.log || { echo "absr bench $v failed"; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_$v.json'))['superres']; print('absr $v', d['us_per_frame'], d['bit_exact_vs_oracle'], '$(tail -n 1 $O/test_$v.log | tr -d =)')"
done
