"""Time dav1d_gpu_lr_frame_* on a synthetic CDEF output (HIP events on
the launch stream) and check it against the oracle.

  python tools/lr_time.py [--width 3840 --height 2160 --bpc 8 --iters 50]
"""
import argparse
import json
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--bpc", type=int, default=8)
    ap.add_argument("--bdmax", type=int, default=1023)
    ap.add_argument("--layout", type=int, default=1)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--no-check", action="store_true")
    args = ap.parse_args()
    import numpy as np
    import torch
    import __graft_entry__ as ge
    ge.load_package()
    import dav1d_mirror_amd.lr as lr
    c = lr.make_lr_case(seed=11, unit_log2=(6, 5), width=args.width, height=args.height, bpc=args.bpc, bitdepth_max=args.bdmax,
                            layout=args.layout)
    dev = lr.DeviceLr(c)
    s = torch.cuda.current_stream()
    for _ in range(3):
        dev.launch(s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(args.iters):
        dev.launch(s)
    e1.record(s)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / args.iters
    nbytes = lr.algorithmic_bytes(c)
    out = {"width": args.width, "height": args.height, "bpc": args.bpc, "layout": args.layout,
           "us_per_frame": round(us, 2), "algorithmic_MB": round(nbytes / 1e6, 2),
           "GBps": round(nbytes / us / 1e3, 1), "frac_of_8TBps": round(nbytes / us / 1e3 / 8000, 4)}
    if not args.no_check:
        orc = ge.load_oracle()
        t = time.perf_counter()
        want = orc.lr_frame(c)
        out["oracle_ms_1core"] = round((time.perf_counter() - t) * 1e3, 1)
        out["bit_exact"] = all(np.array_equal(a, b) for a, b in zip(dev.outputs_host(), want))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
