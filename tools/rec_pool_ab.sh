mkdir -p gpurun_out/r5t
F="--steps 20 --no-families --no-configs --no-tiles --no-intra --no-grain --no-cdef --no-superres --no-lpf --no-lr --no-cpu"
for i in 1 2; do
  DAV1D_GPU_REC_THREADS=8 timeout -k 10 300 python -u bench.py $F > gpurun_out/r5t/rec8_$i.json 2> gpurun_out/r5t/rec8_$i.log || exit 1
  timeout -k 10 300 python -u bench.py $F > gpurun_out/r5t/recauto_$i.json 2> gpurun_out/r5t/recauto_$i.log || exit 1
  for v in rec8_$i recauto_$i; do python3 -c "import json; r=json.load(open('gpurun_out/r5t/$v.json'))['recorder']; print('$v', r['flush_host_ms'], r['flush_device_ms'], r['frame_threads']['wall_ms'], r['frame_threads']['flush_host_ms_per_frame'], r['bit_exact_vs_oracle'], r['frame_threads']['bit_exact_vs_oracle'])"; done
done
python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"
