cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in "" t1 t2 t4 t7; do
  O=$R/gpurun_out/pv_${v:-prod}
  mkdir -p $O
  DAV1D_GPU_LIB_VARIANT=$v timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $O -o run --output-format csv -- python3 $R/tools/tile_time.py --only-tiles --iters 3 > $O/log 2>&1 || echo "fail $v"
done
