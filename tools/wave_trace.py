#!/usr/bin/env python3
"""Debug aid: per-wave phase timeline of the batch kernel, one class at a
time, from the DGPU_TRACE build (tools/build_variants.sh trace).

    DAV1D_GPU_LIB_VARIANT=trace python tools/wave_trace.py [class ...]

Marks (s_memtime shader cycles, each taken after draining the wave's memory
operations): 15 kernel entry, 0 unit start, 1 descriptor in, 2 coefs/edges
staged, 3 mc h-pass done, 4 row transforms, 5 column transforms, 6/7 second
ref h-pass of a compound unit, 8 stores issued."""
import os
import struct
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

NAMES = {1: "descriptor", 2: "stage", 3: "hpass", 4: "rows", 5: "cols", 7: "hpass2", 8: "emit"}


def read(path):
    out = []
    data = open(path, "rb").read()
    o = 0
    while o < len(data):
        g, n = struct.unpack_from("<ii", data, o)
        o += 8
        a = np.frombuffer(data, np.uint64, n * 16, o).reshape(n, 16).astype(np.int64)
        o += n * 16 * 8
        out.append((g, a))
    return out


def main():
    pkg = ge.load_package()
    import torch
    import dav1d_mirror_amd.workload as wl
    import dav1d_mirror_amd.batch as bt
    fd = wl.make_frame(wl.FrameConfig())
    dev = bt.DeviceFrame(fd, "cuda:0")
    cnt = np.diff(fd.class_start)
    classes = [int(c) for c in sys.argv[1:]] or [t for t in range(19) if cnt[t]]
    path = "/tmp/dgpu_trace.bin"
    for t in classes:
        os.environ["DAV1D_GPU_CLASSMASK"] = hex(1 << t)
        for rep in range(3):
            if os.path.exists(path):
                os.remove(path)
            os.environ["DAV1D_GPU_TRACE_FILE"] = path
            dev.launch()
            torch.cuda.synchronize()
        recs = read(path)
        w, h = pkg.abi.TX_WH[t]
        for g, a in recs:
            valid = a[:, 15] > 0
            a = a[valid]
            t0 = a[:, 15].min()
            ent = a[:, 15] - t0
            end = a[:, 8] - t0
            line = [f"{w:2d}x{h:<2d} grp{g} waves {len(a):5d}  entry p50 {np.median(ent):7.0f} p90 "
                    f"{np.percentile(ent, 90):7.0f}  end p50 {np.median(end):7.0f} max {end.max():7.0f}  |"]
            prev = a[:, 0]
            line.append(f" start {np.median(a[:, 0] - a[:, 15]):6.0f}")
            for i in (1, 2, 3, 4, 5, 7, 8):
                ok = a[:, i] > 0
                if ok.sum() == 0:
                    continue
                d = a[ok, i] - np.where(a[ok, i - 1] > 0, a[ok, i - 1], prev[ok]) if i != 7 else a[ok, 7] - a[ok, 5]
                line.append(f" {NAMES[i]} {np.median(d):6.0f}")
                prev = np.where(a[:, i] > 0, a[:, i], prev)
            print("".join(line), flush=True)
    os.environ.pop("DAV1D_GPU_CLASSMASK", None)


if __name__ == "__main__":
    main()
