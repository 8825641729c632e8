#!/bin/bash
# Diagnostics builds: libdav1d_gpu.<name>.so with bounds checks or trace
# stamps compiled in.  Select one with DAV1D_GPU_LIB_VARIANT=<name>.
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
# Round 6: the measured-slower and probe variants (ablations, row skipping,
# persistent waves, paired stores, nontemporal streams, ...) were deleted from
# the sources; their A/B results stay under profiles/r1..r5.  What is left are
# the diagnostics builds.
for v in ${VARIANTS:-bounds}; do
    case $v in
        ttrace) TUS=tile8 build ttrace -DDGPU_TILE_TRACE=1 ;;
        bounds) TUS="recon8 recon_ie8 recon_sb8 recorder tile8 tile16" build bounds -DDGPU_BOUNDS=1 ;;
        ftrace) TUS="recon_ie8" build ftrace -DDGPU_FLOW_TRACE=1 ;;
        ielanes16) TUS="recon_ie8" build ielanes16 -DDGPU_IE_SMALL_LANES=16 ;;
        ienarrow) TUS="recon_ie8" build ienarrow -DDGPU_IE_WIDE_LANES=0 ;;   # the round-5 lanes
        sbdiag) TUS="recon_sb8" build sbdiag -DDGPU_DIAG=1 ;;   # tools/sb_debug.py
        fphase) TUS="recon_ie8" build fphase -DDGPU_FLOW_TRACE=1 -DDGPU_TRACE=1 -DDGPU_TRACE_RT=1 ;;
        trace) build trace -DDGPU_TRACE=1 ;;
        *) echo "unknown variant $v" >&2; exit 2 ;;
    esac
done
