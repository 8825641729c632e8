#!/usr/bin/env python3
"""Benchmark of the fused reconstruction hot path (BASELINE.json metric).

One step = one reconstruction of one synthetic 8-bit 4K 4:2:0 frame batch
(mc put / mct+avg, all 14 intra_pred modes, inv_txfm_add 4x4..32x32) with
every input already resident in HBM: one launch of libdav1d_gpu.so's fused
kernel.  N GPUs = N independent frames, one per rank (frame sharding, no
collective on the data path; weak scaling).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 4k|1080p-mc|4k-10bit]

Rank 0 prints one JSON line.  See DESIGN.md for the roofline accounting.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

CONFIGS = {
    # BASELINE.json configs[2]: the metric's config
    "4k": dict(width=3840, height=2160, bpc=8, kind="full",
               label="8-bit 4K 4:2:0 synthetic block batch, full mc + ipred + inv_txfm_add 4x4..32x32"),
    # configs[1]
    "1080p-mc": dict(width=1920, height=1080, bpc=8, kind="mc",
                     label="8-bit 1080p 4:2:0 synthetic block batch, mc.put/mc.avg 8-tap only"),
    # configs[3]
    "4k-10bit": dict(width=3840, height=2160, bpc=16, bitdepth_max=1023, kind="full",
                     label="10-bit 4K 4:2:0 synthetic block batch, full mc + ipred + inv_txfm_add"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(fd, budget_s=12.0):
    """The oracle (C restatement of dav1d's C DSP) on this host's cores,
    single thread, over whole frames until ~budget_s of CPU work."""
    orc = ge.load_oracle()
    hf = orc.HostFrame(fd)
    frames = 0
    t0 = time.perf_counter()
    while True:
        hf.run(threads=1)
        frames += 1
        el = time.perf_counter() - t0
        if el > budget_s or frames >= 64:
            break
    px = fd.stats["pixels"] * frames
    return {"value": round(px / el / 1e9, 5), "unit": "Gpixels/s", "cores": 1, "kind": "port",
            "sample": f"{frames} full frame(s) of the same batch ({fd.stats['pixels']} px each), "
                      f"{el:.1f} s single-thread, oracle/dsp_ref.c -O2 (restatement of dav1d C, not dav1d)"}


PMC_SUMMARY = os.path.join(ROOT, "profiles", "r1", "v3i_pmc_summary.json")


def pmc_traffic(bpc):
    """HBM bytes per launch of the same kernels from the committed rocprofv3
    PMC summary (FETCH_SIZE and WRITE_SIZE, separate --pmc passes, KB as
    rocprofv3 reports them).  PMC needs rocprofv3 around the process, so a
    plain bench run cannot re-measure it; the source file is named."""
    try:
        d = json.load(open(PMC_SUMMARY))
    except (OSError, ValueError):
        return None, None
    tot = 0.0
    for k, v in d.items():
        if k.startswith(f"k_recon<{bpc},") and "FETCH_SIZE" in v and "WRITE_SIZE" in v:
            tot += (v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024
    if not tot:
        return None, None
    return int(tot), (f"FETCH_SIZE+WRITE_SIZE per frame from {os.path.relpath(PMC_SUMMARY, ROOT)} "
                      "(uncorrected: the gfx950 x2 FETCH factor holds for wide coalesced reads, "
                      "not these scattered row loads)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="4k", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--check", action="store_true", help="verify rank 0's frame against the oracle")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")

    pkg = ge.load_package()
    import dav1d_mirror_amd.workload as wl
    import dav1d_mirror_amd.batch as bt
    import dav1d_mirror_amd.shard as sh

    c = dict(CONFIGS[args.config])
    label = c.pop("label")
    cfg = sh.rank_config(wl.FrameConfig(**c), rank)
    t0 = time.perf_counter()
    fd = wl.make_frame(cfg)
    log(f"[rank {rank}] frame: {fd.n_units} units, {fd.stats['pixels']} px, "
        f"{fd.stats['total_bytes'] / 1e6:.1f} MB algorithmic, generated in {time.perf_counter() - t0:.1f}s")
    frame = bt.DeviceFrame(fd, dev)
    stream = torch.cuda.current_stream(dev)

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        frame.launch(stream)
    torch.cuda.synchronize(dev)

    # timed region: exactly K steps, barrier + synchronize on both sides
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        frame.launch(stream)
    torch.cuda.synchronize(dev)
    barrier()
    el = sh.max_over_ranks(time.perf_counter() - t0, dist, dev)

    # per-launch kernel duration with HIP events on the launch stream
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    for a, b in evs:
        a.record(stream)
        frame.launch(stream)
        b.record(stream)
    torch.cuda.synchronize(dev)
    durs = np.array([a.elapsed_time(b) for a, b in evs]) * 1e-3   # s
    kern_s = float(np.mean(durs))

    check = None
    if args.check and rank == 0:
        orc = ge.load_oracle()
        hf = orc.HostFrame(fd)
        hf.run(threads=4)
        got = frame.planes_host()
        check = all(np.array_equal(got[p], hf.dst[p]) for p in range(3))
        log(f"[rank 0] bit-exact vs oracle: {check}")

    if rank == 0:
        traffic, traffic_note = pmc_traffic(cfg.bpc) if args.config == "4k" else (None, None)
        value = sh.aggregate_gpix_per_s(fd.stats["pixels"], args.steps, world, el)
        bytes_launch = fd.stats["total_bytes"]
        achieved = bytes_launch / kern_s / 1e9
        out = {
            "metric": "Gpixels/s (mc+ipred+itx block batch) + achieved HBM GB/s vs peak, 8-bit 4K, 1/8 GPU",
            "value": round(value, 3),
            "unit": "Gpixels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8" if cfg.bpc == 8 else "u16",
            "data": "synthetic (seeded block batch; random reference frames, edges, coefficients from a forward transform of random residuals)",
            "config": {
                "workload": label,
                "frame": f"{cfg.width}x{cfg.height} 4:2:0",
                "units_per_frame": fd.n_units,
                "pixels_per_frame": fd.stats["pixels"],
                "frames_per_step_per_gpu": 1,
                "parallelism": f"frame-sharded x{world}",
                "zero_coefs": False,
                "launches_per_step": 1,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_note": traffic_note,
                "kernel": f"k_recon<{cfg.bpc},*> (main group: all classes up to 32x32 in one launch; "
                          "the 64-point group launches only when such units exist; events bracket the step)",
                "kernel_us": round(kern_s * 1e6, 2),
                "algorithmic_bytes_per_launch": bytes_launch,
                "bytes_breakdown": {k: fd.stats[k] for k in
                                    ("ref_bytes", "edge_bytes", "coef_bytes", "dst_bytes", "desc_bytes")},
            },
        }
        if check is not None:
            out["config"]["bit_exact_vs_oracle"] = check
        if not args.no_cpu and world == 1:
            out["cpu_baseline"] = cpu_baseline(fd)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
