#!/usr/bin/env python3
"""Profiling aid: time the fused recon kernel with phases disabled through
the debug-only DAV1D_GPU_ABLATE mask (1 footprint loads, 2 inter filter
math, 4 intra prediction, 8 inverse transforms).  Outputs are wrong in the
ablated runs; only the timings matter."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402


def main():
    import torch
    ge.load_package()
    import dav1d_mirror_amd.workload as wl
    import dav1d_mirror_amd.batch as bt
    cfg = sys.argv[1] if len(sys.argv) > 1 else "4k"
    kw = dict(width=1920, height=1080, kind="mc") if cfg == "1080p-mc" else {}
    fd = wl.make_frame(wl.FrameConfig(**kw))
    dev = bt.DeviceFrame(fd, "cuda:0")
    s = torch.cuda.current_stream()
    for mask in [0, 1, 2, 4, 8, 3, 15]:
        os.environ["DAV1D_GPU_ABLATE"] = str(mask)
        for _ in range(3):
            dev.launch(s)
        torch.cuda.synchronize()
        ts = []
        for _ in range(20):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            dev.launch(s)
            b.record(s)
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        print(f"ablate={mask:2d}  median {np.median(ts):8.1f} us  min {np.min(ts):8.1f} us", flush=True)
    os.environ["DAV1D_GPU_ABLATE"] = "0"


if __name__ == "__main__":
    main()
