"""Quick timing of the unit batch (dav1d_gpu_recon_*) on one config, GPU box:
   DAV1D_GPU_LIB_VARIANT=<v> python tools/unit_time.py [--kind full]"""
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
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    ge.load_package()
    import torch
    import dav1d_mirror_amd.workload as wl
    import dav1d_mirror_amd.batch as bt
    fd = wl.make_frame(wl.FrameConfig(width=a.width, height=a.height, kind=a.kind))
    dev = bt.DeviceFrame(fd, "cuda:0")
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
    print(f"units {a.kind}: {us:.1f} us/frame  {fd.stats['pixels'] / us / 1e3:.1f} Gpix/s", flush=True)


if __name__ == "__main__":
    main()
