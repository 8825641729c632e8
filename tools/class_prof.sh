#!/bin/bash
# Per-class profile of the batch kernel on the config-3 frame (GPU box):
#   bash tools/class_prof.sh TAG
# One kernel-trace pass (durations per class) and two SQ counter passes
# (tools/class_pmc.py launches the frame once per class with
# DAV1D_GPU_CLASSMASK).  Summaries go to gpurun_out/cls_TAG/*.txt.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r3}
O=$R/gpurun_out/cls_$TAG
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace -d "$O/trace" -o run --output-format csv \
    -- python3 "$R/tools/class_pmc.py" > "$O/trace.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    -d "$O/sq1" -o run --output-format csv -- python3 "$R/tools/class_pmc.py" > "$O/sq1.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS \
    -d "$O/sq2" -o run --output-format csv -- python3 "$R/tools/class_pmc.py" > "$O/sq2.log" 2>&1
cd "$R"
python3 tools/class_pmc.py --durations "$O/trace/run_kernel_trace.csv" > "$O/durations.txt"
python3 tools/class_pmc.py --summarise "$O/sq1/run_counter_collection.csv" > "$O/sq1.txt"
python3 tools/class_pmc.py --summarise "$O/sq2/run_counter_collection.csv" > "$O/sq2.txt"
cat "$O/durations.txt" "$O/sq1.txt" "$O/sq2.txt"
