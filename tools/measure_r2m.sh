#!/bin/bash
# Round-2 closing GPU pass (GPU box): every GPU parity test, smoke(), the
# default bench line (with the CDEF and deblocking legs), and a rocprofv3
# kernel-trace of the bench:  bash tools/measure_r2m.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r2m}
O=$R/gpurun_out/m_$TAG
mkdir -p "$O"
cd "$R"
echo "[m] tests" >&2
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/gputest.log" 2>&1 || { echo "tests failed" >&2; exit 1; }
echo "[m] smoke" >&2
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "smoke failed" >&2; exit 1; }
echo "[m] bench" >&2
timeout -k 10 600 python3 bench.py > "$O/bench_4k.json" 2> "$O/bench_4k.err" || { echo "bench failed" >&2; exit 1; }
echo "[m] trace" >&2
cd /tmp
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- \
    python3 "$R/bench.py" --no-cpu --steps 10 --warmup 2 --no-families --no-intra --no-recorder > "$O/trace.log" 2>&1 || { echo "trace failed" >&2; exit 1; }
echo "[m] done" >&2
