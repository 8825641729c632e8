#!/bin/bash
# Profiling builds: libdav1d_gpu.<name>.so with one phase of the batch
# kernel ablated (DGPU_ABL_* in csrc/recon_kernel.hpp), or a tunable changed.  Select one with
# DAV1D_GPU_LIB_VARIANT=<name>.  Outputs of these builds are wrong by design.
set -e
cd "$(dirname "$0")/../dav1d-mirror_amd"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../include -Icsrc"
mkdir -p build/var
build() {
    local name=$1; shift
    # only the batch TUs differ; the per-call TUs come from the product build
    for s in ${TUS:-recon8 recon16}; do
        $HIPCC $F "$@" -c csrc/$s.hip -o build/var/$name.$s.o &
    done
    wait
    local objs=""
    for s in runtime mc ipred itx recon8 recon16 tile8 tile16 edges recon_ie8 recon_ie16 recon_sb8 recon_sb16 recorder grain cdef lpf lr picture; do
        if [ -f build/var/$name.$s.o ] && [[ " ${TUS:-recon8 recon16} " == *" $s "* ]]; then objs="$objs build/var/$name.$s.o"; else objs="$objs build/$s.o"; fi
    done
    $HIPCC $F -shared -o libdav1d_gpu.$name.so $objs build/stamp.o
}
for v in ${VARIANTS:-nomc noitx nointra}; do
    case $v in
        vodd) TUS=recon8 build vodd -DDGPU_VODD_ALIGN=1 ;;
        nod2) TUS=recon8 build nod2 -DDGPU_ITX_D2=0 ;;
        notall) TUS=recon8 build notall -DDGPU_TALL_LANES=0 ;;
        salu200) build salu200 -DDGPU_PAD_SALU=200 ;;
        al16) build al16 -DDGPU_ALIGNED_ROWS16=1 ;;
        ch16) build ch16 -DDGPU_CH16=1 ;;
        vmem8) build vmem8 -DDGPU_PAD_VMEM=8 ;;
        vmem1x8) build vmem1x8 -DDGPU_PAD_VMEM1=8 ;;
        fakecoal) build fakecoal -DDGPU_FAKE_COALESCE=1 ;;
        valu200) build valu200 -DDGPU_PAD_VALU=200 ;;
        t1|t2|t4|t8|t16|t3|t6|t7|t15|t31) TUS=tile8 build $v -DDGPU_TILE_ABL=${v#t} ;;
        ttrace) TUS=tile8 build ttrace -DDGPU_TILE_TRACE=1 ;;
        twpe2|twpe4|twpe5) TUS=tile8 build $v -DDGPU_TILE_WPE=${v#twpe} ;;
        cdefw6|cdefw7|cdefw8) TUS=cdef build $v -DDGPU_CDEF_WPE=${v#cdefw} ;;
        cdefa1|cdefa2|cdefa3) TUS=cdef build $v -DDGPU_CDEF_ABL=${v#cdefa} ;;
        lra1|lra2|lra3) TUS=lr build $v -DDGPU_LR_ABL=${v#lra} ;;
        lrv1|lrv2|lrv3|lrv4|lrv5|lrv6|lrv7) TUS=lr build $v -DDGPU_LR_VEC=${v#lrv} ;;
        lrpf1|lrpf2|lrpf3) TUS=lr build $v -DDGPU_LR_PF=${v#lrpf} ;;
        st8) TUS=recon8 build st8 -DDGPU_ST8=1 ;;
        lpfb) TUS=lpf build lpfb -DDGPU_LPF_BATCH=1 ;;
        rzvec) TUS=mc build rzvec -DDGPU_RZ_VEC=1 ;;
        bounds) TUS="recon8 recon_ie8 recon_sb8 recorder tile8 tile16" build bounds -DDGPU_BOUNDS=1 ;;
        fnofence) TUS="recon_ie8" build fnofence -DDGPU_FLOW_NOFENCE=1 ;;
        fsc1) TUS="recon_ie8" build fsc1 -DDGPU_FLOW_SC1=1 ;;
        fsleep1) TUS="recon_ie8" build fsleep1 -DDGPU_FLOW_SLEEP=1 ;;
        ftrace) TUS="recon_ie8" build ftrace -DDGPU_FLOW_TRACE=1 ;;
        fprio) TUS="recon_ie8" build fprio -DDGPU_FLOW_PRIO=1 ;;
        ielanes) TUS="recon_ie8" build ielanes -DDGPU_IE_SMALL_LANES=8 ;;
        ielanes16) TUS="recon_ie8" build ielanes16 -DDGPU_IE_SMALL_LANES=16 ;;
        sbdiag) TUS="recon_sb8" build sbdiag -DDGPU_DIAG=1 ;;   # tools/sb_debug.py
        fphase) TUS="recon_ie8" build fphase -DDGPU_FLOW_TRACE=1 -DDGPU_TRACE=1 -DDGPU_TRACE_RT=1 ;;
        ftrace127) TUS="recon_ie8" build ftrace127 -DDGPU_FLOW_TRACE=1 -DDGPU_FLOW_SLEEP=127 ;;
        fsleep32) TUS="recon_ie8" build fsleep32 -DDGPU_FLOW_SLEEP=32 ;;
        fsleep127) TUS="recon_ie8" build fsleep127 -DDGPU_FLOW_SLEEP=127 ;;
        nomc) build nomc -DDGPU_ABL_MC=1 ;;
        nostore) build nostore -DDGPU_ABL_STORE=1 ;;
        noitx) build noitx -DDGPU_ABL_ITX=1 ;;
        nointra) build nointra -DDGPU_ABL_INTRA=1 ;;
        none) build none -DDGPU_ABL_MC=1 -DDGPU_ABL_ITX=1 -DDGPU_ABL_INTRA=1 ;;
        noseq) build noseq -DDGPU_SEQREF_MAX_TPL=0 ;;
        seg4) build seg4 -DDGPU_SEGMENTS=4 ;;
        seg64) build seg64 -DDGPU_SEGMENTS=64 ;;
        seg1) build seg1 -DDGPU_SEGMENTS=1 ;;
        trace) build trace -DDGPU_TRACE=1 ;;
        persist) TUS=recon8 build persist -DDGPU_PERSIST=1 -DDGPU_LANE_OPAQUE=1 ;;
        persist2) TUS=recon8 build persist2 -DDGPU_PERSIST=2 -DDGPU_LANE_OPAQUE=1 ;;
        persistn) TUS=recon8 build persistn -DDGPU_PERSIST=1 ;;
        persist3) TUS=recon8 build persist3 -DDGPU_PERSIST=3 -DDGPU_LANE_OPAQUE=1 ;;
        persist3n) TUS=recon8 build persist3n -DDGPU_PERSIST=3 ;;
        ntload) TUS=recon8 build ntload -DDGPU_NT_STREAM=1 ;;
        respad) TUS=recon8 build respad -DDGPU_RES_PAD=1 ;;
        persist4) TUS=recon8 build persist4 -DDGPU_PERSIST=4 -DDGPU_LANE_OPAQUE=1 -DDGPU_PERSIST_WPE=4 ;;
        merge) build merge -DDGPU_MERGE_GROUPS=1 ;;
        sl2) build sl2 -DDGPU_SEG_INNER=2 ;;
        early1) build early1 -DDGPU_EARLY_REF1=1 ;;
        early1w4) build early1w4 -DDGPU_EARLY_REF1=1 -DDGPU_WPE_SMALL8=4 ;;
        sl4) build sl4 -DDGPU_SEG_INNER=4 ;;
        sl2s32) build sl2s32 -DDGPU_SEG_INNER=2 -DDGPU_SEGMENTS=32 ;;
        merge5) build merge5 -DDGPU_MERGE_GROUPS=1 -DDGPU_WPE_SMALL8=5 ;;
        merge4) build merge4 -DDGPU_MERGE_GROUPS=1 -DDGPU_WPE_SMALL8=1 ;;
        merge6) build merge6 -DDGPU_MERGE_GROUPS=1 -DDGPU_WPE_SMALL8=6 ;;
        seg8) build seg8 -DDGPU_SEGMENTS=8 ;;
        noskip) build noskip -DDGPU_ROWSKIP=0 ;;
        seg32) build seg32 -DDGPU_SEGMENTS=32 ;;
        m5seg8) build m5seg8 -DDGPU_MERGE_GROUPS=1 -DDGPU_WPE_SMALL8=5 -DDGPU_SEGMENTS=8 ;;
        m5seg32) build m5seg32 -DDGPU_MERGE_GROUPS=1 -DDGPU_WPE_SMALL8=5 -DDGPU_SEGMENTS=32 ;;
    esac
done
