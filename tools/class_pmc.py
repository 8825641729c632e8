#!/usr/bin/env python3
"""Profiling aid: per-class PMC counters of the batch kernel.

Run under rocprofv3 --pmc ... (program directly after `--`): launches the
4K frame REPS times per transform class with the debug-only
DAV1D_GPU_CLASSMASK, in class order.  Then summarise with

    python tools/class_pmc.py --summarise gpurun_out/<dir>/run_counter_collection.csv
"""
import argparse
import collections
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

REPS = 3


def classes_with_units():
    pkg = ge.load_package()
    import dav1d_mirror_amd.workload as wl
    fd = wl.make_frame(wl.FrameConfig())
    import numpy as np
    cnt = np.diff(fd.class_start)
    return pkg, fd, [t for t in range(19) if cnt[t]], cnt


def run():
    import torch
    pkg, fd, cls, _ = classes_with_units()
    import dav1d_mirror_amd.batch as bt
    dev = bt.DeviceFrame(fd, "cuda:0")
    s = torch.cuda.current_stream()
    for t in cls:
        os.environ["DAV1D_GPU_CLASSMASK"] = hex(1 << t)
        for _ in range(REPS):
            dev.launch(s)
        torch.cuda.synchronize()
    os.environ.pop("DAV1D_GPU_CLASSMASK")


def summarise(path):
    pkg, fd, cls, cnt = classes_with_units()
    rows = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        if "k_recon" not in r["Kernel_Name"]:
            continue
        rows.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    disp = [rows[k] for k in sorted(rows)]
    assert len(disp) == REPS * len(cls), (len(disp), len(cls))
    names = sorted(disp[0])
    print("class   units  " + "  ".join(f"{n[:14]:>14}" for n in names) + "   VALU/px  VALU/wave")
    for i, t in enumerate(cls):
        d = disp[i * REPS:(i + 1) * REPS]
        m = {n: sum(x[n] for x in d) / REPS for n in names}
        w, h = pkg.abi.TX_WH[t]
        px = cnt[t] * w * h
        extra = ""
        if "SQ_INSTS_VALU" in m:
            extra = f"  {m['SQ_INSTS_VALU'] * 64 / px:8.1f}"
            if "SQ_WAVES" in m:
                extra += f"  {m['SQ_INSTS_VALU'] / max(m['SQ_WAVES'], 1):9.0f}"
        print(f"{w:2d}x{h:<2d} {cnt[t]:7d}  " + "  ".join(f"{m[n]:14.0f}" for n in names) + extra)


def durations(path):
    """Kernel-trace durations per class (rocprofv3 --kernel-trace run of this script)."""
    pkg, fd, cls, cnt = classes_with_units()
    rows = []
    for r in csv.DictReader(open(path)):
        if "k_recon" in r["Kernel_Name"]:
            rows.append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3))
    rows.sort()
    assert len(rows) == REPS * len(cls)
    for i, t in enumerate(cls):
        d = sorted(x[1] for x in rows[i * REPS:(i + 1) * REPS])
        w, h = pkg.abi.TX_WH[t]
        print(f"{w:2d}x{h:<2d} {cnt[t]:7d} units  kernel {d[len(d) // 2]:7.1f} us")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--summarise")
    ap.add_argument("--durations")
    a = ap.parse_args()
    if a.durations:
        durations(a.durations)
    elif a.summarise:
        summarise(a.summarise)
    else:
        run()
