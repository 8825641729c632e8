#!/usr/bin/env python3
"""Debug aid: inter-intra units as pure put (mask 0, no residual): the GPU's
block vs the oracle's put with each Filter2d, for a few units."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402


def main():
    pkg = ge.load_package()
    orc = ge.load_oracle()
    import torch
    import dav1d_mirror_amd.workload as wl
    import dav1d_mirror_amd.batch as bt
    abi = pkg.abi
    fd = wl.make_frame(wl.FrameConfig(width=512, height=256, kind="ext", seed=21))
    u = fd.units.copy()
    ii = np.nonzero(u["pred"] == abi.PRED_INTER_INTRA)[0]
    pool = fd.aux_pool.copy()
    for i in ii:
        moff = int(pool[fd.aux[i] + 8:fd.aux[i] + 12].view("<i4")[0])
        w, h = abi.TX_WH[int(u["tx"][i])]
        bw = int(u["bw4"][i]) * 4
        for y in range(h):
            pool[moff + y * bw:moff + y * bw + w] = 0
    u["txtp"] = 255
    fd.aux_pool = pool
    fd.units = u
    dev = bt.DeviceFrame(fd, "cuda:0")
    dev.launch()
    torch.cuda.synchronize()
    got = dev.planes_host()
    shown = 0
    for i in ii:
        p = int(u["plane"][i])
        w, h = abi.TX_WH[int(u["tx"][i])]
        y0, x0 = divmod(int(u["dst_off"][i]), fd.plane_wh[p][0])
        g = got[p][y0:y0 + h, x0:x0 + w].astype(int)
        match = []
        for f in range(10):
            sub = wl.FrameData(**{k: getattr(fd, k) for k in fd.__dataclass_fields__})
            uu = u[i:i + 1].copy()
            uu["pred"] = abi.PRED_INTER
            uu["filter2d"] = f
            sub.units = uu
            sub.aux = None
            sub.class_start = np.concatenate([[0], np.cumsum(np.bincount(uu["tx"], minlength=19))]).astype(np.int32)
            sub.class_warp = np.zeros(19, np.int32)
            hf = orc.HostFrame(sub)
            hf.run()
            o = hf.dst[p][y0:y0 + h, x0:x0 + w].astype(int)
            match.append(int(np.abs(o - g).max()))
        print("unit f2d", int(u["filter2d"][i]), "mx", int(u["mx0"][i]), "my", int(u["my0"][i]), "bw", int(u["bw4"][i]) * 4,
              "max|gpu - oracle put(f)| for f=0..9:", match, flush=True)
        shown += 1
        if shown >= 8:
            break


if __name__ == "__main__":
    main()
