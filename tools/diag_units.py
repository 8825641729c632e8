#!/usr/bin/env python3
"""Debug aid: run a small frame on the GPU, compare with the oracle and
tabulate the mismatching units by prediction kind / class / filter / mv
fraction, so a parity break can be localised without a debugger."""
import collections
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402


def main():
    pkg = ge.load_package()
    orc = ge.load_oracle()
    import dav1d_mirror_amd.workload as wl
    import dav1d_mirror_amd.batch as bt
    kw = dict(width=512, height=256, seed=int(sys.argv[1]) if len(sys.argv) > 1 else 1)
    if len(sys.argv) > 2 and int(sys.argv[2]) > 255:
        kw.update(bpc=16, bitdepth_max=int(sys.argv[2]))
    if len(sys.argv) > 3:
        kw.update(kind=sys.argv[3])
    fd = wl.make_frame(wl.FrameConfig(**kw))
    dev = bt.DeviceFrame(fd, "cuda:0")
    dev.launch()
    import torch
    torch.cuda.synchronize()
    got = dev.planes_host()
    hf = orc.HostFrame(fd)
    hf.run(threads=4)
    stats = collections.Counter()
    tot = collections.Counter()
    shown = 0
    for u in fd.units:
        p = int(u["plane"])
        w, h = pkg.abi.TX_WH[int(u["tx"])]
        pw = fd.plane_wh[p][0]
        y0, x0 = divmod(int(u["dst_off"]), pw)
        a = got[p][y0:y0 + h, x0:x0 + w]
        b = hf.dst[p][y0:y0 + h, x0:x0 + w]
        pred = int(u["pred"])
        key = [f"pred{pred}", f"{w}x{h}"]
        if pred in (1, 2, 9):
            key += [f"f{int(u['filter2d'])}", f"mx0={int(u['mx0']) > 0}", f"my0={int(u['my0']) > 0}",
                    f"bw{int(u['bw4']) * 4}"]
        elif pred == 3:
            key += [f"mode{int(u['mode'])}"]
        key += ["nores" if int(u["txtp"]) == 255 else ("dc" if int(u["nzw"]) == 0 else "res")]
        bad = not np.array_equal(a, b)
        for k in key:
            tot[k] += 1
            if bad:
                stats[k] += 1
        if bad and shown < 3:
            shown += 1
            print("unit", {n: int(u[n]) for n in u.dtype.names if not n.startswith("pad")})
            print(" got\n", a.astype(int))
            print(" want\n", b.astype(int))
    for k in sorted(tot):
        print(f"{k:16s} bad {stats[k]:6d} / {tot[k]:6d}")


if __name__ == "__main__":
    main()
