R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE TA_BUSY_avr TA_BUSY_max SQ_WAVES -d $R/gpurun_out/ta1 -o run --output-format csv -- python3 $R/tools/class_pmc.py > $R/gpurun_out/ta1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE -d $R/gpurun_out/ta2 -o run --output-format csv -- python3 $R/tools/class_pmc.py > $R/gpurun_out/ta2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc TCP_PENDING_STALL_CYCLES_sum TCP_TAGRAM0_REQ_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum GRBM_GUI_ACTIVE -d $R/gpurun_out/ta3 -o run --output-format csv -- python3 $R/tools/class_pmc.py > $R/gpurun_out/ta3.log 2>&1
