"""Quick timing of the tile batch vs the unit batch on one config (GPU box).
   python tools/tile_time.py [--kind full] [--width 3840 --height 2160] [--bpc 8]"""
import argparse
import sys
import pathlib
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import __graft_entry__ as ge  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="full")
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--bpc", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only-tiles", action="store_true")
    a = ap.parse_args()
    ge.load_package()
    import torch
    import dav1d_mirror_amd.workload as wl
    import dav1d_mirror_amd.tiles as tl
    import dav1d_mirror_amd.batch as bt
    cfg = wl.FrameConfig(width=a.width, height=a.height, kind=a.kind, bpc=a.bpc,
                         bitdepth_max=255 if a.bpc == 8 else 1023)
    fd = wl.make_frame(cfg)
    td = tl.build_tiles(fd)
    out = {}
    devs = [("tiles", bt.DeviceTiles(fd, td, "cuda:0"))]
    if not a.only_tiles:
        devs.insert(0, ("units", bt.DeviceFrame(fd, "cuda:0")))
    for name, dev in devs:
        for _ in range(3):
            dev.launch()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            dev.launch()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) * 1000 / a.iters
        out[name] = us
        print(f"{name}: {us:.1f} us/frame  {fd.stats['pixels'] / us / 1e3:.1f} Gpix/s", flush=True)
    print("tile stats:", {k: td.stats[k] for k in ("n_tiles", "n_preds", "n_txs", "desc_bytes", "total_bytes")})
    print(f"tiles algorithmic GB/s: {td.stats['total_bytes'] / out['tiles'] / 1e3:.1f}")


if __name__ == "__main__":
    main()
