#!/bin/bash
# Instruction-cache counters for the full-frame bench and per class (GPU box).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d $R/gpurun_out/ic_full -o run --output-format csv -- python3 $R/bench.py --no-cpu --steps 5 --warmup 1 > $R/gpurun_out/ic_full.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d $R/gpurun_out/ic_cls -o run --output-format csv -- python3 $R/tools/class_pmc.py > $R/gpurun_out/ic_cls.log 2>&1
