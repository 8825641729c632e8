#!/bin/bash
# SQ counters of the unit kernel, product build and ablation variants (GPU box)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in "" nostore nomc noitx nointra none; do
  O=$R/gpurun_out/pu_${v:-prod}
  mkdir -p $O
  DAV1D_GPU_LIB_VARIANT=$v timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY -d $O -o run --output-format csv -- python3 $R/tools/unit_time.py --iters 3 > $O/log 2>&1 || echo "fail $v"
done
