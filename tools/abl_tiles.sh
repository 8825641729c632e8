#!/bin/bash
# Tile-kernel timing of the product build and the ablation variants
# (tools/build_variants.sh t*), then PMC passes of the product: GPU box only.
#   bash tools/abl_tiles.sh TAG "variants" [tile_time args]
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; VARS=$2; shift 2
O=$R/gpurun_out/abl_$TAG
mkdir -p "$O"
for v in "" $VARS; do
  echo "== variant ${v:-product}" >> "$O/time.log"
  DAV1D_GPU_LIB_VARIANT=$v timeout -k 10 100 python3 "$R/tools/tile_time.py" --only-tiles "$@" >> "$O/time.log" 2>&1 || echo "variant $v failed" >> "$O/time.log"
done
bash "$R/tools/prof_tiles.sh" "$TAG" "$@"
