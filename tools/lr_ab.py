#!/usr/bin/env python3
"""A/B of the LR frame kernel's workgroup order (DAV1D_GPU_LR_ORDER=linear:
the dispatcher's round-robin order; default: XCD-contiguous runs of
stripes) on the bench's 4K 8-bit frame: K launches per mode, alternated
`--rounds` times, HIP events on the launch stream; outputs compared.

    python tools/lr_ab.py [--steps K] [--rounds R] [--only xcd|linear]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", default="")
    ap.add_argument("--bpc", type=int, default=8)
    args = ap.parse_args()
    import numpy as np
    import torch
    import __graft_entry__ as ge
    ge.load_package()
    import dav1d_mirror_amd.lr as lr
    c = lr.make_lr_case(seed=11, width=3840, height=2160, bpc=args.bpc, bitdepth_max=255 if args.bpc == 8 else 1023,
                        layout=1, unit_log2=(6, 5))
    dev = torch.device("cuda:0")
    d = lr.DeviceLr(c, dev)
    s = torch.cuda.current_stream(dev)
    modes = [args.only] if args.only else ["xcd", "linear"]
    out = {m: [] for m in modes}
    pics = {}
    for _ in range(args.rounds):
        for m in modes:
            if m == "linear":
                os.environ["DAV1D_GPU_LR_ORDER"] = "linear"
            else:
                os.environ.pop("DAV1D_GPU_LR_ORDER", None)
            d.launch(s)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(args.steps):
                d.launch(s)
            e1.record(s)
            torch.cuda.synchronize()
            out[m].append(round(e0.elapsed_time(e1) * 1e3 / args.steps, 2))
            pics[m] = [a.copy() for a in d.outputs_host()]
    if len(modes) == 2:
        out["identical"] = all(np.array_equal(a, b) for a, b in zip(pics["xcd"], pics["linear"]))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
