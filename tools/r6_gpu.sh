#!/bin/bash
# Round-6 GPU check (run through gpurun from the repo root):
#   bash tools/r6_gpu.sh <tag> [steps...]
# steps: tests (full -m gpu suite), stests (the same with every kernel
# serialized, AMD_SERIALIZE_KERNEL=3, so a fault is reported at its launch), bounds (the recorder tests on the
# DGPU_BOUNDS build, tools/build_variants.sh bounds), smoke, bench (headline
# line), prof (rocprofv3 kernel trace of the headline), pmc (FETCH / WRITE
# passes), intra / cdef (those GPU test files), benchpart (the intra,
# CDEF, LR and recorder bench legs), cdefpmc (CDEF / LR counters).  Every step has its own time limit; the first failure ends the run.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
T=${1:-r6}
shift
O=$R/gpurun_out/$T
mkdir -p "$O"
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
BENCH_FAST="--no-families --no-configs --no-tiles --no-intra --no-recorder --no-grain --no-cdef --no-superres --no-lpf --no-lr --no-cpu --no-check"
for s in "${@:-tests}"; do
    echo "[r6] $s start $(date +%T)"
    case $s in
    tests) timeout -k 10 900 $PYT -m gpu -x ${PYK:+-k "$PYK"} tests > "$O/gputest.log" 2>&1 || { echo "[r6] tests failed"; tail -5 "$O/gputest.log"; exit 1; } ;;
    topedge) # the recorder's top_edge / post-filter interleave tests (no -x: every case reported)
        timeout -k 10 300 $PYT -m gpu tests/test_gpu_recorder.py -k top_edge > "$O/topedge.log" 2>&1; echo "[r6] topedge rc=$? $(tail -1 "$O/topedge.log")" ;;
    stests) AMD_SERIALIZE_KERNEL=3 timeout -k 10 1200 $PYT -m gpu -x tests > "$O/gputest.log" 2>&1 || { echo "[r6] stests failed"; exit 1; } ;;
    rectests) timeout -k 10 600 $PYT -m gpu -x tests/test_gpu_recorder.py tests/test_gpu_batch.py > "$O/rectest.log" 2>&1 || { echo "[r6] rectests failed"; exit 1; } ;;
    bounds) # -s: the device printf reports must not be captured by pytest
            DAV1D_GPU_LIB_VARIANT=bounds timeout -k 10 600 $PYT -s -m gpu tests/test_gpu_recorder.py > "$O/bounds.log" 2>&1
            rc=$?; echo "[r6] bounds rc=$rc reports=$(grep -c 'DGPU_BOUNDS line' "$O/bounds.log")"; [ $rc -le 1 ] || exit 1
            # positive control: the coefficient pool registered 64 bytes short must be reported
            DAV1D_GPU_BND_SELFTEST=1 DAV1D_GPU_LIB_VARIANT=bounds timeout -k 10 300 $PYT -s -m gpu \
                "tests/test_gpu_recorder.py::test_recorder_mixed" > "$O/bounds_selftest.log" 2>&1
            echo "[r6] bounds selftest rc=$? reports=$(grep -c 'DGPU_BOUNDS line' "$O/bounds_selftest.log")" ;;
    tbounds) # the tile batch under the bounds build: every record / coefficient / edge / aux access against the
             # exact buffers, record indices against the tile's counts; then the round-3 lane maps restored
             # (DAV1D_GPU_BND_NOCLAMP: no padding init, raw indices) as the positive control
            DAV1D_GPU_LIB_VARIANT=bounds timeout -k 10 600 $PYT -s -m gpu tests/test_gpu_tiles.py > "$O/tbounds.log" 2>&1
            rc=$?; echo "[r6] tbounds rc=$rc range=$(grep -c 'DGPU_BOUNDS line' "$O/tbounds.log") index=$(grep -c 'DGPU_TILE_INDEX' "$O/tbounds.log")"
            [ $rc -le 1 ] || exit 1
            DAV1D_GPU_BND_NOCLAMP=1 DAV1D_GPU_LIB_VARIANT=bounds timeout -k 10 600 $PYT -s -m gpu tests/test_gpu_tiles.py > "$O/tbounds_noclamp.log" 2>&1
            rc=$?; echo "[r6] tbounds noclamp rc=$rc range=$(grep -c 'DGPU_BOUNDS line' "$O/tbounds_noclamp.log") index=$(grep -c 'DGPU_TILE_INDEX' "$O/tbounds_noclamp.log")"
            [ $rc -le 1 ] || exit 1 ;;
    intra) timeout -k 10 600 $PYT -m gpu -x tests/test_gpu_intra_frame.py > "$O/intra.log" 2>&1 || { echo "[r6] intra failed"; exit 1; } ;;
    benchpart) # the intra wavefront, CDEF, LR and recorder legs only (recorder host laps on stderr)
            DAV1D_GPU_REC_TIMING=1 timeout -k 10 600 python -u bench.py --steps 50 --no-families --no-configs --no-tiles \
                --no-grain --no-superres --no-lpf --no-cpu --no-check > "$O/benchpart.json" 2> "$O/benchpart.log" \
                || { echo "[r6] benchpart failed"; exit 1; } ;;
    recbench) # the recorder leg alone (host laps on stderr), with the headline
            DAV1D_GPU_REC_TIMING=1 timeout -k 10 300 python -u bench.py --steps 20 --no-families --no-configs --no-tiles \
                --no-intra --no-grain --no-cdef --no-superres --no-lpf --no-lr --no-cpu --no-check > "$O/recbench.json" \
                2> "$O/recbench.log" || { echo "[r6] recbench failed"; exit 1; } ;;
    recprep) # the recorder flush alone: host / prep / stream times, laps, then its kernels under rocprofv3
            DAV1D_GPU_REC_TIMING=1 timeout -k 10 300 python -u tools/rec_prep_time.py --reps 5 --threads 4 > "$O/recprep.log" 2>&1 \
                || { echo "[r6] recprep failed"; exit 1; }
            tail -3 "$O/recprep.log"
            timeout -k 10 300 python -u tools/rec_prep_time.py --reps 2 --threads 4 --busy > "$O/recprep_busy.log" 2>&1 \
                || { echo "[r6] recprep busy failed"; exit 1; }
            tail -3 "$O/recprep_busy.log"
            cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/recprof" -o rec \
                -- python3 -u "$R/tools/rec_prep_time.py" --reps 3 > "$O/recprof.log" 2>&1 || { echo "[r6] recprof failed"; exit 1; }
            cd "$R" ;;
    leadab) # the recorder flush's leading-level threshold (DAV1D_GPU_LEAD_UNITS), stream / host / prep times
            for L in ${LEADU:-1000000000 8192 4096 2048 1024 512}; do
                DAV1D_GPU_LEAD_UNITS=$L timeout -k 10 300 python -u tools/rec_prep_time.py --reps 5 > "$O/leadab_$L.log" 2>&1 \
                    || { echo "[r6] leadab $L failed"; exit 1; }
                echo "leadab $L $(tail -1 "$O/leadab_$L.log")"
            done ;;
    checkasm) # the full checkasm-style space (no --quick), one pass per table and bitdepth
            for t in ${CKT:-mc ipred itx cdef lpf lr}; do for b in 8 16; do
                timeout -k 10 1200 ./tests/checkasm_gpu --test=$t --bpc=$b --seed=1 > "$O/checkasm_full_${t}_${b}.log" 2>&1 \
                    || { echo "[r6] checkasm $t $b failed"; tail -5 "$O/checkasm_full_${t}_${b}.log"; exit 1; }
                tail -1 "$O/checkasm_full_${t}_${b}.log"
            done; done ;;
    ab) # headline-frame A/B of variant libraries (ABV="persist persist2"): kernel us per variant, bit-exact check on
        for v in base $ABV; do
            if [ "$v" = base ]; then unset DAV1D_GPU_LIB_VARIANT; else export DAV1D_GPU_LIB_VARIANT=$v; fi
            timeout -k 10 300 python -u bench.py --no-families --no-configs --no-tiles --no-intra --no-recorder --no-grain \
                --no-cdef --no-superres --no-lpf --no-lr --no-cpu --steps ${ABSTEPS:-200} > "$O/ab_$v.json" 2> "$O/ab_$v.log" \
                || { echo "[r6] ab $v failed"; tail -5 "$O/ab_$v.log"; exit 1; }
            python3 -c "import json; d=json.load(open('$O/ab_$v.json')); r=d['roofline']; print('ab $v', r['kernel_us'], r.get('stream_us_per_step'), d['ms_per_step'], d['config'].get('bit_exact_vs_oracle'))"
        done
        unset DAV1D_GPU_LIB_VARIANT ;;
    abpmc) # FETCH_SIZE / WRITE_SIZE of the headline kernel per variant library (ABV)
        for v in base $ABV; do
            if [ "$v" = base ]; then unset DAV1D_GPU_LIB_VARIANT; else export DAV1D_GPU_LIB_VARIANT=$v; fi
            for c in FETCH_SIZE WRITE_SIZE; do
                (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --pmc $c -d "$O/abpmc_${v}_$c" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 2 $BENCH_FAST) > "$O/abpmc_${v}_$c.log" 2>&1 || { echo "[r6] abpmc $v $c failed"; exit 1; }
            done
        done
        unset DAV1D_GPU_LIB_VARIANT ;;
    post) # CDEF, LR, super-res and deblocking bench legs (the headline leg runs too)
        timeout -k 10 400 python -u bench.py --steps 50 --no-families --no-configs --no-tiles --no-intra --no-recorder \
            --no-grain --no-cpu --no-check > "$O/post.json" 2> "$O/post.log" || { echo "[r6] post failed"; exit 1; }
        python3 -c "import json; d=json.load(open('$O/post.json')); print('post', {k: (d[k]['us_per_frame'], d[k]['bit_exact_vs_oracle']) for k in ('cdef','loop_restoration','superres','loop_filter')})" ;;
    lr) timeout -k 10 600 $PYT -m gpu -x tests/test_gpu_lr.py "tests/test_gpu_checkasm.py::test_checkasm[lr]" tests/test_gpu_chain.py > "$O/lr.log" 2>&1 || { echo "[r6] lr failed"; tail -5 "$O/lr.log"; exit 1; }
        tail -1 "$O/lr.log"
        timeout -k 10 300 python -u bench.py --steps 50 --no-families --no-configs --no-tiles --no-intra --no-recorder \
            --no-grain --no-cdef --no-superres --no-lpf --no-cpu --no-check > "$O/lrbench.json" 2> "$O/lrbench.log" \
            || { echo "[r6] lr bench failed"; exit 1; }
        python3 -c "import json; d=json.load(open('$O/lrbench.json'))['loop_restoration']; print('lr', d['us_per_frame'], d['bit_exact_vs_oracle'])" ;;
    varintra) # the intra-frame and recorder GPU tests on each variant library (ABV)
        for v in $ABV; do
            DAV1D_GPU_LIB_VARIANT=$v timeout -k 10 600 $PYT -m gpu -x -k "not lossless" tests/test_gpu_intra_frame.py tests/test_gpu_recorder.py > "$O/varintra_$v.log" 2>&1 \
                || { echo "[r6] varintra $v failed"; tail -5 "$O/varintra_$v.log"; exit 1; }
            echo "varintra $v $(tail -1 "$O/varintra_$v.log")"
        done ;;
    ablr) # the LR frame tests and bench leg per variant library (ABV), base first
        for v in base $ABV; do
            if [ "$v" = base ]; then unset DAV1D_GPU_LIB_VARIANT; else export DAV1D_GPU_LIB_VARIANT=$v; fi
            timeout -k 10 400 $PYT -m gpu -x tests/test_gpu_lr.py tests/test_gpu_chain.py > "$O/ablr_test_$v.log" 2>&1 \
                || { echo "[r6] ablr tests $v failed"; tail -5 "$O/ablr_test_$v.log"; exit 1; }
            timeout -k 10 300 python -u bench.py --steps 100 --no-families --no-configs --no-tiles --no-intra --no-recorder \
                --no-grain --no-cdef --no-superres --no-lpf --no-cpu > "$O/ablr_$v.json" 2> "$O/ablr_$v.log" \
                || { echo "[r6] ablr bench $v failed"; exit 1; }
            python3 -c "import json; d=json.load(open('$O/ablr_$v.json'))['loop_restoration']; print('ablr $v', d['us_per_frame'], d['bit_exact_vs_oracle'], '$(tail -1 "$O/ablr_test_$v.log" | tr -d =)')"
        done
        unset DAV1D_GPU_LIB_VARIANT ;;
    abcdef) # the CDEF frame tests and bench leg per variant library (ABV), base first
        for v in base $ABV; do
            if [ "$v" = base ]; then unset DAV1D_GPU_LIB_VARIANT; else export DAV1D_GPU_LIB_VARIANT=$v; fi
            timeout -k 10 400 $PYT -m gpu -x tests/test_gpu_cdef.py > "$O/abcdef_test_$v.log" 2>&1 \
                || { echo "[r6] abcdef tests $v failed"; tail -5 "$O/abcdef_test_$v.log"; exit 1; }
            timeout -k 10 300 python -u bench.py --steps 100 --no-families --no-configs --no-tiles --no-intra --no-recorder \
                --no-grain --no-lr --no-superres --no-lpf --no-cpu > "$O/abcdef_$v.json" 2> "$O/abcdef_$v.log" \
                || { echo "[r6] abcdef bench $v failed"; exit 1; }
            python3 -c "import json; d=json.load(open('$O/abcdef_$v.json'))['cdef']; print('abcdef $v', d['us_per_frame'], d['bit_exact_vs_oracle'], '$(tail -1 "$O/abcdef_test_$v.log" | tr -d =)')"
        done
        unset DAV1D_GPU_LIB_VARIANT ;;
    flowunits) # the wavefront's units-per-task cap above level 0 (DAV1D_GPU_FLOW_UNITS), 4K intra frames
        for U in ${FLOWU:-4 8 16}; do
            DAV1D_GPU_FLOW_UNITS=$U timeout -k 10 300 python -u bench.py --steps 20 --no-families --no-configs --no-tiles --no-recorder --no-grain \
                --no-cdef --no-superres --no-lpf --no-lr --no-cpu --no-check > "$O/flowunits_$U.json" 2> "$O/flowunits_$U.log" \
                || { echo "[r6] flowunits $U failed"; exit 1; }
            python3 -c "import json; d=json.load(open('$O/flowunits_$U.json'))['intra_wavefront']; print('flowunits $U', d['1_tile']['ms_per_frame'], d['1_tile']['bit_exact_vs_oracle'], d['2x2_tiles']['ms_per_frame'], d['2x2_tiles']['bit_exact_vs_oracle'])"
        done ;;
    abintra) # the intra wavefront bench leg per variant library (ABV): 1-tile / 2x2 ms per 4K frame, bit-exact
        for v in base $ABV; do
            if [ "$v" = base ]; then unset DAV1D_GPU_LIB_VARIANT; else export DAV1D_GPU_LIB_VARIANT=$v; fi
            timeout -k 10 400 python -u bench.py --steps 20 --no-families --no-configs --no-tiles --no-recorder --no-grain \
                --no-cdef --no-superres --no-lpf --no-lr --no-cpu --no-check > "$O/abintra_$v.json" 2> "$O/abintra_$v.log" \
                || { echo "[r6] abintra $v failed"; tail -5 "$O/abintra_$v.log"; exit 1; }
            python3 -c "import json; d=json.load(open('$O/abintra_$v.json'))['intra_wavefront']; print('abintra $v', d['1_tile']['ms_per_frame'], d['1_tile']['bit_exact_vs_oracle'], d['2x2_tiles']['ms_per_frame'], d['2x2_tiles']['bit_exact_vs_oracle'])"
        done
        unset DAV1D_GPU_LIB_VARIANT ;;
    cdef) timeout -k 10 600 $PYT -m gpu -x tests/test_gpu_cdef.py "tests/test_gpu_checkasm.py::test_checkasm[cdef]" > "$O/cdef.log" 2>&1 || { echo "[r6] cdef failed"; tail -5 "$O/cdef.log"; exit 1; }
        tail -1 "$O/cdef.log"
        timeout -k 10 300 python -u bench.py --steps 50 --no-families --no-configs --no-tiles --no-intra --no-recorder \
            --no-grain --no-lr --no-superres --no-lpf --no-cpu --no-check > "$O/cdefbench.json" 2> "$O/cdefbench.log" \
            || { echo "[r6] cdef bench failed"; exit 1; }
        python3 -c "import json; d=json.load(open('$O/cdefbench.json'))['cdef']; print('cdef', d['us_per_frame'], d['bit_exact_vs_oracle'])" ;;
    new) # this round's new GPU tests (LR last stripe, per-row chain heights, the two-pass split)
        timeout -k 10 900 $PYT -m gpu -x tests/test_gpu_lr.py tests/test_gpu_chain.py "tests/test_gpu_batch.py::test_batch_split_two_pass" > "$O/new.log" 2>&1 || { echo "[r6] new failed"; tail -5 "$O/new.log"; exit 1; }
        tail -1 "$O/new.log" ;;
    split) # fused vs two-pass A/B on config 3 (and 10-bit), stream time per frame, pictures compared
        for cfg in 4k 4k-10bit; do
            timeout -k 10 300 python -u tools/split_ab.py --config $cfg --steps 100 --rounds 3 ${SPLITARGS} > "$O/split_$cfg.json" 2> "$O/split_$cfg.log" || { echo "[r6] split $cfg failed"; tail -5 "$O/split_$cfg.log"; exit 1; }
            cat "$O/split_$cfg.json"
        done ;;
    splitprof) # rocprofv3 kernel trace + FETCH / WRITE / SQ passes of the two forms (each alone)
        for f in fused split; do
            (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/splitprof_$f" -o run --output-format csv -- python3 "$R/tools/split_ab.py" --only $f --steps 50 --rounds 1) > "$O/splitprof_$f.log" 2>&1 || { echo "[r6] splitprof $f failed"; exit 1; }
            for c in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS"; do
                n=$(echo $c | cut -d' ' -f1)
                (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --pmc $c -d "$O/splitpmc_${f}_$n" -o run --output-format csv -- python3 "$R/tools/split_ab.py" --only $f --steps 10 --rounds 1) > "$O/splitpmc_${f}_$n.log" 2>&1 || { echo "[r6] splitpmc $f $n failed"; exit 1; }
            done
        done ;;
    fam) # the headline plus the per-family legs (mc / ipred / itx / ext) and configs 2 / 4
        timeout -k 10 400 python -u bench.py --steps 100 --no-tiles --no-intra --no-recorder --no-grain --no-cdef --no-superres \
            --no-lpf --no-lr --no-cpu > "$O/fam.json" 2> "$O/fam.log" || { echo "[r6] fam failed"; tail -5 "$O/fam.log"; exit 1; }
        python3 -c "import json; d=json.load(open('$O/fam.json')); print('fam', d['roofline']['kernel_us'], {k: v['kernel_us'] for k, v in d['families'].items()}, {k: v['kernel_us'] for k, v in d['configs'].items()}, d['config'].get('bit_exact_vs_oracle'))" ;;
    fphase) # the intra wavefront's per-task / per-phase trace (diagnostics library fphase)
        DAV1D_GPU_LIB_VARIANT=${FTV:-fphase} timeout -k 10 300 python -u tools/flow_trace.py > "$O/fphase_${FTV:-fphase}.json" 2> "$O/fphase.log" || { echo "[r6] fphase failed"; tail -5 "$O/fphase.log"; exit 1; }
        head -c 3000 "$O/fphase_${FTV:-fphase}.json"; echo ;;
    flowab) # the wavefront's units-per-task cap x coded-mode task groups (tools/flow_units_ab.py, one process each)
        for U in ${FLOWU:-4 8 16}; do for TG in 0 1; do
            DAV1D_GPU_FLOW_UNITS=$U FLOW_TASK_GROUPS=$TG timeout -k 10 300 python -u tools/flow_units_ab.py >> "$O/flowab.jsonl" 2>> "$O/flowab.log" \
                || { echo "[r6] flowab $U $TG failed"; tail -5 "$O/flowab.log"; exit 1; }
        done; done
        cat "$O/flowab.jsonl" ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "[r6] smoke failed"; exit 1; } ;;
    bench) timeout -k 10 900 python -u bench.py > "$O/bench.json" 2> "$O/bench.log" || { echo "[r6] bench failed"; exit 1; } ;;
    benchfast) timeout -k 10 300 python -u bench.py $BENCH_FAST > "$O/benchfast.json" 2> "$O/benchfast.log" || { echo "[r6] benchfast failed"; exit 1; } ;;
    prof) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 50 $BENCH_FAST) > "$O/prof.log" 2>&1 || { echo "[r6] prof failed"; exit 1; } ;;
    prof10) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof10" -o run --output-format csv -- python3 "$R/bench.py" --config 4k-10bit --steps 50 $BENCH_FAST) > "$O/prof10.log" 2>&1 || { echo "[r6] prof10 failed"; exit 1; }
            for c in FETCH_SIZE WRITE_SIZE; do
                (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --pmc $c -d "$O/pmc10_$c" -o run --output-format csv -- python3 "$R/bench.py" --config 4k-10bit --steps 10 --warmup 2 $BENCH_FAST) > "$O/pmc10_$c.log" 2>&1 || { echo "[r6] pmc10 $c failed"; exit 1; }
            done ;;
    sqpmc) # SQ counters of the headline kernel (one pass: 8 SQ counters at most)
        (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d "$O/sqpmc" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 2 $BENCH_FAST) > "$O/sqpmc.log" 2>&1 || { echo "[r6] sqpmc failed"; exit 1; } ;;
    pmc) for c in FETCH_SIZE WRITE_SIZE; do
             (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --pmc $c -d "$O/pmc_$c" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 2 $BENCH_FAST) > "$O/pmc_$c.log" 2>&1 || { echo "[r6] pmc $c failed"; exit 1; }
         done ;;
    cdefpmc) # CDEF / LR counters: the bench with only those legs (the headline frame runs too; filter by kernel)
         for c in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS"; do
             n=$(echo $c | cut -d' ' -f1)
             (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --pmc $c -d "$O/cdefpmc_$n" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-families --no-configs --no-tiles --no-intra --no-recorder --no-grain --no-superres --no-lpf --no-cpu --no-check) > "$O/cdefpmc_$n.log" 2>&1 || { echo "[r6] cdefpmc $n failed"; exit 1; }
         done ;;
    esac
    echo "[r6] $s done $(date +%T)"
done
