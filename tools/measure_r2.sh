#!/bin/bash
# Round-2 GPU pass: GPU parity tests, the bench line of every config (with
# the tile batch beside the headline), and rocprofv3 kernel-trace + PMC
# passes of the metric's config (GPU box):  bash tools/measure_r2.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r2}
O=$R/gpurun_out/m_$TAG
mkdir -p "$O"
cd "$R"
echo "[m] tests" >&2
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/gputest.log" 2>&1 || { echo "tests failed" >&2; exit 1; }
for c in 4k 1080p-mc 4k-10bit; do
    echo "[m] bench $c" >&2
    timeout -k 10 300 python3 bench.py --config $c > "$O/bench_$c.json" 2> "$O/bench_$c.err" || exit 1
done
echo "[m] prof" >&2
timeout -k 10 900 bash tools/prof.sh "$TAG" --steps 10 --warmup 2 --no-families || exit 1
timeout -k 10 600 bash tools/prof.sh "${TAG}_10bit" --steps 10 --warmup 2 --config 4k-10bit --no-families || exit 1
echo "[m] done" >&2
