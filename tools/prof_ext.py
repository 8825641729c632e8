#!/usr/bin/env python3
"""Profiling aid: launch the 4K `ext` family frame (w_avg / mask / palette /
warp mix) REPS times; run under rocprofv3 --kernel-trace --stats to split
the main and warp launches."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402


def main():
    ge.load_package()
    import torch
    import dav1d_mirror_amd.workload as wl
    import dav1d_mirror_amd.batch as bt
    bpc = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    cfg = wl.FrameConfig(kind="ext", bpc=bpc, bitdepth_max=255 if bpc == 8 else 1023)
    fd = wl.make_frame(cfg)
    print("units", fd.n_units, "warp units", fd.stats["n_warp"], "class_warp", list(fd.class_warp), flush=True)
    dev = bt.DeviceFrame(fd, "cuda:0")
    for _ in range(20):
        dev.launch()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
