#!/usr/bin/env python3
"""A/B of the fused unit batch against its two-pass form (workload.
split_frame: prediction blocks, then residuals onto the picture) on one
frame: K back-to-back launches of each, timed by one HIP event pair on the
launch stream, alternated `--rounds` times; both pictures checked equal.
Run under rocprofv3 --kernel-trace --stats / --pmc for the per-launch
counters (the kernels appear in launch order: fused, then pred / res).

    python tools/split_ab.py [--config 4k|4k-10bit] [--steps K] [--rounds R] [--piece 32]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="4k")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--piece", type=int, default=32)
    ap.add_argument("--only", default="", help="fused|split: launch only one form (profiling)")
    args = ap.parse_args()
    import numpy as np
    import torch
    import bench
    import __graft_entry__ as ge
    ge.load_package()
    import dav1d_mirror_amd.batch as bt
    import dav1d_mirror_amd.workload as wl
    c = dict(bench.CONFIGS[args.config])
    c.pop("label")
    fd = wl.make_frame(wl.FrameConfig(**c))
    pf, rf = wl.split_frame(fd, piece=args.piece)
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev)
    fused = bt.DeviceFrame(fd, dev)
    a = bt.DeviceFrame(pf, dev)
    b = bt.DeviceFrame(rf, dev, dst_planes=a.dst)

    def run_fused():
        fused.launch(s)

    def run_split():
        a.launch(s)
        b.launch(s)

    def timed(fn, n):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(n):
            fn()
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / n

    res = {"config": args.config, "units_fused": fd.n_units, "units_pred": pf.n_units, "units_res": rf.n_units,
           "piece": args.piece, "algorithmic_bytes": fd.stats["total_bytes"], "fused_us": [], "split_us": [],
           "pred_us": [], "res_us": []}
    for _ in range(args.rounds):
        if args.only != "split":
            res["fused_us"].append(round(timed(run_fused, args.steps), 2))
        if args.only != "fused":
            res["split_us"].append(round(timed(run_split, args.steps), 2))
            res["pred_us"].append(round(timed(lambda: a.launch(s), args.steps), 2))
            res["res_us"].append(round(timed(lambda: b.launch(s), args.steps), 2))
    run_split()
    run_fused()
    torch.cuda.synchronize()
    if not args.only:
        res["identical"] = all(np.array_equal(x, y) for x, y in zip(fused.planes_host(), b.planes_host()))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
