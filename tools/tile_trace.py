"""Per-phase timing of the tile kernel from a DGPU_TILE_TRACE build
(tools/build_variants.sh ttrace), run on the GPU box:
   DAV1D_GPU_LIB_VARIANT=ttrace python tools/tile_trace.py [tile_time-like args]
Phases (s_memtime ticks, shader clock): 0 start, 1 staging issued+LDS
written, 2 after barrier, 3 transforms done, 4 after barrier, 5 preds done,
6 after barrier, 7 stored."""
import argparse
import os
import sys
import pathlib
import numpy as np
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import __graft_entry__ as ge  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="full")
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    a = ap.parse_args()
    ge.load_package()
    import torch
    import dav1d_mirror_amd.workload as wl
    import dav1d_mirror_amd.tiles as tl
    import dav1d_mirror_amd.batch as bt
    fd = wl.make_frame(wl.FrameConfig(width=a.width, height=a.height, kind=a.kind))
    td = tl.build_tiles(fd)
    dev = bt.DeviceTiles(fd, td, "cuda:0")
    dev.launch()
    torch.cuda.synchronize()
    f = "/tmp/tile_trace.bin"
    os.environ["DAV1D_GPU_TRACE_FILE"] = f
    dev.launch()
    torch.cuda.synchronize()
    t = np.fromfile(f, np.uint64).reshape(-1, 4, 8).astype(np.int64)
    t0 = t[:, :, 0].min()
    tt = t - t0
    ph = np.diff(t, axis=2)   # [tile][wave][7]
    names = ["stage", "bar1", "itx", "bar2", "pred", "bar3", "store"]
    print("kernel span (ticks): %d" % (t[:, :, 7].max() - t0))
    for i, n in enumerate(names):
        v = ph[:, :, i]
        print(f"{n:6s} mean {v.mean():8.0f}  median {np.median(v):8.0f}  p90 {np.percentile(v, 90):8.0f}")
    life = t[:, :, 7] - t[:, :, 0]
    print(f"tile life mean {life.mean():.0f} median {np.median(life):.0f}")
    st = np.sort(tt[:, 0, 0])
    print("tile start quantiles:", [int(st[int(q * (len(st) - 1))]) for q in (0, .1, .25, .5, .75, .9, 1)])
    T = td.tiles
    for p in range(3):
        sel = T["plane"] == p
        print(f"plane {p}: life mean {life[sel].mean():.0f}, itx {ph[sel, :, 2].mean():.0f}, pred {ph[sel, :, 4].mean():.0f}")


if __name__ == "__main__":
    main()
