"""Time film grain on the device (dav1d_gpu_apply_grain_*): HIP events
around K back-to-back applications (prep + apply launches) of a 4K picture,
and the oracle's whole-picture time on one core."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--bpc", type=int, default=8)
    ap.add_argument("--bdmax", type=int, default=1023)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--lag", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    import torch
    import __graft_entry__ as ge
    ge.load_package()
    import dav1d_mirror_amd.grain as grain
    c = grain.make_grain_case(seed=5, width=a.width, height=a.height, bpc=a.bpc, bitdepth_max=a.bdmax,
                              lag=a.lag, num_y=8, csfl=False, num_uv=(6, 6), overlap=True)
    dev = grain.DeviceGrain(c)
    s = torch.cuda.current_stream()
    for _ in range(3):
        dev.launch(s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(a.steps):
        dev.launch(s)
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.steps
    t0 = time.perf_counter()
    outs, _, _ = ge.load_oracle().apply_grain(c)
    cpu = time.perf_counter() - t0
    px = sum(w * h for w, h in c.plane_wh)
    bpp = 1 if a.bpc == 8 else 2
    print(json.dumps({"frame": f"{a.width}x{a.height}", "bpc": a.bpc, "ms_per_frame": round(ms, 4),
                      "gpix_s": round(px / ms / 1e6, 2), "io_bytes": 2 * px * bpp,
                      "io_gbs": round(2 * px * bpp / ms / 1e6, 1), "oracle_1core_ms": round(cpu * 1e3, 1),
                      "bit_exact": all(bool(np.array_equal(x, y)) for x, y in zip(dev.outputs_host(), outs))}))


if __name__ == "__main__":
    main()
