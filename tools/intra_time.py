"""Time the intra wavefront (dav1d_gpu_recon_intra_frame_*) on one frame:
HIP events around K back-to-back launches (each relaunch is idempotent:
the edge stage rewrites the unit modes from the records and every pixel is
predicted afresh), plus the oracle's decoder-order walk on the host."""
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
    ap.add_argument("--bdmax", type=int, default=255)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--graph", action="store_true", help="capture one frame in a HIP graph, time replays")
    ap.add_argument("--mode", default="persistent", choices=["persistent", "levels", "fused", "staged"])
    ap.add_argument("--tiles", default="1x1", help="tile columns x rows")
    a = ap.parse_args()
    import __graft_entry__ as ge
    ge.load_package()
    import numpy as np
    import torch
    import dav1d_mirror_amd.intra as intra
    t0 = time.time()
    tc, tr = (int(v) for v in a.tiles.split("x"))
    fr = intra.make_intra_frame(intra.IntraConfig(width=a.width, height=a.height, bpc=a.bpc,
                                                  bitdepth_max=a.bdmax, tile_cols=tc, tile_rows=tr))
    gen_s = time.time() - t0
    dev = intra.DeviceIntraFrame(fr, mode=a.mode)
    s = torch.cuda.current_stream()
    for _ in range(2):
        dev.launch(s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if a.graph:
        g = torch.cuda.CUDAGraph()
        cs = torch.cuda.Stream()
        with torch.cuda.stream(cs):
            g.capture_begin()
            dev.launch(cs)
            g.capture_end()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        run = g.replay
    else:
        run = lambda: dev.launch(s)   # noqa: E731
    t0 = time.perf_counter()
    e0.record(s)
    for _ in range(a.steps):
        run()
    e1.record(s)
    host_enqueue = (time.perf_counter() - t0) / a.steps
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.steps
    px = sum(w * h for w, h in fr.plane_wh)
    out = {"frame": f"{a.width}x{a.height}", "bpc": a.bpc, "units": len(fr.units), "levels": fr.n_levels,
           "ms_per_frame": ms, "gpix_s": px / ms / 1e6, "host_enqueue_ms": host_enqueue * 1e3,
           "gen_s": gen_s, "graph": a.graph, "mode": a.mode, "tiles": a.tiles}
    oracle = ge.load_oracle()
    ho = oracle.HostIntraFrame(fr)
    t0 = time.perf_counter()
    ho.run()
    out["oracle_ms"] = (time.perf_counter() - t0) * 1e3
    if a.check:
        got = dev.planes_host()
        out["bit_exact"] = all(bool(np.array_equal(g, o)) for g, o in zip(got, ho.dst))
        out["flow_error"] = dev.flow_error()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
