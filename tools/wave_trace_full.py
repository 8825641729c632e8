#!/usr/bin/env python3
"""Debug aid: per-wave phase timeline of the whole-frame launch (all
classes in one grid) from the DGPU_TRACE build:

    DAV1D_GPU_LIB_VARIANT=trace python tools/wave_trace_full.py

Prints the launch span, how many waves are resident over time and in which
phase, and per-class medians of each phase (s_memtime shader cycles; marks
as in tools/wave_trace.py: 15 entry, 0 unit start, 1 descriptor, 2 staged,
3 h-pass, 4 rows, 5 cols, 6/7 second ref, 8 stores issued)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402
from tools.wave_trace import read  # noqa: E402

PH = [(15, 13, "table+bar"), (13, 14, "schedule"), (14, 0, "dispatch"), (0, 1, "desc"), (1, 2, "stage"), (2, 3, "hpass"), (3, 4, "rows"), (4, 5, "cols"),
      (5, 8, "pred+store")]


def main():
    pkg = ge.load_package()
    import torch
    import dav1d_mirror_amd.workload as wl
    import dav1d_mirror_amd.batch as bt
    fd = wl.make_frame(wl.FrameConfig())
    dev = bt.DeviceFrame(fd, "cuda:0")
    path = "/tmp/dgpu_trace_full.bin"
    for _ in range(3):
        dev.launch()
    torch.cuda.synchronize()
    if os.path.exists(path):
        os.remove(path)
    os.environ["DAV1D_GPU_TRACE_FILE"] = path
    dev.launch()
    torch.cuda.synchronize()
    os.environ.pop("DAV1D_GPU_TRACE_FILE")
    for g, a in read(path):
        a = a[a[:, 15] > 0]
        if not len(a):
            continue
        t0 = a[:, 15].min()
        ent, end = a[:, 15] - t0, a[:, 8] - t0
        span = end.max()
        life = end - ent
        print(f"group {g}: {len(a)} waves, span {span} cycles; life p10/50/90 "
              f"{np.percentile(life, 10):.0f}/{np.median(life):.0f}/{np.percentile(life, 90):.0f}; "
              f"entry p10/50/90 {np.percentile(ent, 10):.0f}/{np.median(ent):.0f}/{np.percentile(ent, 90):.0f}")
        # residency over time by phase
        nb = 20
        edges = np.linspace(0, span, nb + 1)
        print(" time-slice   resident  " + "  ".join(f"{n:>10s}" for _, _, n in PH))
        for i in range(nb):
            tm = (edges[i] + edges[i + 1]) / 2
            row = []
            for s, e, _ in PH:
                ts = a[:, s] - t0
                te = a[:, e] - t0
                ok = (a[:, s] > 0) & (a[:, e] > 0)
                row.append(int(((ts <= tm) & (te > tm) & ok).sum()))
            res = int(((ent <= tm) & (end > tm)).sum())
            print(f" {tm / span:9.2f}   {res:8d}  " + "  ".join(f"{r:10d}" for r in row))
        # per-phase medians over all waves, and early vs late waves
        for label, sel in (("all", np.ones(len(a), bool)), ("first 20%", ent < 0.2 * span),
                           ("last 50%", ent > 0.5 * span)):
            parts = []
            for s, e, n in PH:
                ok = sel & (a[:, s] > 0) & (a[:, e] > 0)
                if ok.sum():
                    parts.append(f"{n} {np.median(a[ok, e] - a[ok, s]):.0f}")
            print(f" {label:10s} ({sel.sum():5d} waves): " + ", ".join(parts))


if __name__ == "__main__":
    main()
