#!/usr/bin/env python3
"""Debug aid: inter-intra units with their masks forced to 0 (pure inter)
and to 64 (pure intra), GPU vs oracle, to localise a parity break."""
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
    for mval in (None, 0, 64):
        fd = wl.make_frame(wl.FrameConfig(width=512, height=256, kind="ext", seed=21))
        u = fd.units
        ii = np.nonzero(u["pred"] == abi.PRED_INTER_INTRA)[0]
        if mval is not None:
            pool = fd.aux_pool.copy()
            for i in ii:
                moff = int(pool[fd.aux[i] + 8:fd.aux[i] + 12].view("<i4")[0])
                w, h = abi.TX_WH[int(u["tx"][i])]
                bw = int(u["bw4"][i]) * 4
                for y in range(h):
                    pool[moff + y * bw:moff + y * bw + w] = mval
            fd.aux_pool = pool
        dev = bt.DeviceFrame(fd, "cuda:0")
        dev.launch()
        torch.cuda.synchronize()
        got = dev.planes_host()
        hf = orc.HostFrame(fd)
        hf.run()
        bad = 0
        for i in ii:
            p = int(u["plane"][i])
            w, h = abi.TX_WH[int(u["tx"][i])]
            y0, x0 = divmod(int(u["dst_off"][i]), fd.plane_wh[p][0])
            if not np.array_equal(got[p][y0:y0 + h, x0:x0 + w], hf.dst[p][y0:y0 + h, x0:x0 + w]):
                bad += 1
        print(f"mask {mval}: {bad} / {len(ii)} inter-intra units differ", flush=True)


if __name__ == "__main__":
    main()
