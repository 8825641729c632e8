#!/usr/bin/env python3
"""Profiling aid: time the fused recon kernel one transform class at a time
(debug-only DAV1D_GPU_CLASSMASK), reporting us, units and ns per pixel."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402


def timeit(dev, s, n=20):
    import torch
    for _ in range(3):
        dev.launch(s)
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        dev.launch(s)
        b.record(s)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return float(np.median(ts))


def main():
    import torch
    pkg = ge.load_package()
    import dav1d_mirror_amd.workload as wl
    import dav1d_mirror_amd.batch as bt
    fd = wl.make_frame(wl.FrameConfig())
    dev = bt.DeviceFrame(fd, "cuda:0")
    s = torch.cuda.current_stream()
    cnt = np.diff(fd.class_start)
    os.environ["DAV1D_GPU_CLASSMASK"] = hex((1 << 19) - 1)
    print(f"all classes: {timeit(dev, s):8.1f} us", flush=True)
    for t in range(19):
        if not cnt[t]:
            continue
        os.environ["DAV1D_GPU_CLASSMASK"] = hex(1 << t)
        us = timeit(dev, s)
        w, h = pkg.abi.TX_WH[t]
        px = cnt[t] * w * h
        print(f"{w:2d}x{h:<2d} units {cnt[t]:7d}  {us:8.1f} us  {us * 1e3 / px:6.2f} ns/px  "
              f"{us * 1e3 / cnt[t]:6.2f} ns/unit", flush=True)
    os.environ.pop("DAV1D_GPU_CLASSMASK")


if __name__ == "__main__":
    main()
