for sp in 8 16 32; do DAV1D_GPU_MC_SPLIT=$sp CONFIGS="1080p-mc" bash tools/quick.sh | sed "s/^/split $sp /"; done
