#!/bin/bash
# Per-class PMC for the product build and each ablation variant (GPU box).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp
export TMPDIR=/tmp
for v in base ${VARIANTS:-nomc noitx nointra}; do
    if [ "$v" = base ]; then unset DAV1D_GPU_LIB_VARIANT; else export DAV1D_GPU_LIB_VARIANT=$v; fi
    timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
        -d "$R/gpurun_out/vpmc_$v" -o run --output-format csv -- python3 "$R/tools/class_pmc.py" > "$R/gpurun_out/vpmc_$v.log" 2>&1
done
