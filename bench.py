#!/usr/bin/env python3
"""Benchmark of the fused reconstruction hot path (BASELINE.json metric).

One step = one reconstruction of one synthetic 8-bit 4K 4:2:0 frame batch
(mc put / mct+avg, all 14 intra_pred modes, inv_txfm_add 4x4..32x32) with
every input already resident in HBM: one launch of libdav1d_gpu.so's fused
kernel.  N GPUs = N independent frames, one per rank (frame sharding, no
collective on the data path; weak scaling).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 4k|1080p-mc|4k-10bit]
                    [--feed local|rccl] [--no-families] [--no-cpu]

--feed rccl: rank 0 generates every rank's frame and scatters them over RCCL
point-to-point before the timed region (config 5's coded-block feed over
xGMI); the feed's time and bytes are reported on their own ("feed").
At N=1 the line also carries a per-family breakdown ("families": mc-only,
intra-only and itx-only 4K frames of the same bitdepth, one launch each).

Rank 0 prints one JSON line.  See DESIGN.md for the roofline accounting.
"""
import argparse
import dataclasses
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
    """The oracle (C restatement of dav1d's C DSP) on this host's cores over
    whole frames: first on every usable core (the box's CPU share: at most 16
    threads, units split into contiguous ranges), then single-thread beside
    it, each for about budget_s / 2 of wall time."""
    orc = ge.load_oracle()
    hf = orc.HostFrame(fd)

    def timed(threads, budget):
        frames = 0
        t0 = time.perf_counter()
        while True:
            hf.run(threads=threads)
            frames += 1
            el = time.perf_counter() - t0
            if el > budget or frames >= 64:
                return frames, el

    nthr = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count() or 1))
    fm, em = timed(nthr, budget_s / 2)
    f1, e1 = timed(1, budget_s / 2)
    px = fd.stats["pixels"]
    return {"value": round(px * fm / em / 1e9, 5), "unit": "Gpixels/s", "cores": nthr, "kind": "port",
            "sample": f"{fm} full frame(s) of the same batch ({px} px each), {em:.1f} s on {nthr} threads "
                      f"(unit ranges split per thread), oracle/dsp_ref.c -O2 (restatement of dav1d C, not dav1d; "
                      f"AVX2 baseline unavailable: no nasm/meson)",
            "single_thread": {"value": round(px * f1 / e1 / 1e9, 5), "cores": 1,
                              "sample": f"{f1} full frame(s), {e1:.1f} s single-thread"}}


# rocprofv3 summaries of the current kernels (tools/prof.sh + tools/pmc_summary.py):
# the kernel-trace averages (cross-check of the event timing below) and the
# PMC traffic of separate FETCH_SIZE / WRITE_SIZE passes
def _latest_profile(fmt):
    """The newest round's committed summary (profiles/rN/rN_<fmt>), so a line
    never cites an older kernel's profile once the current one is in."""
    for rnd in ("r6", "r5", "r4", "r3"):
        path = os.path.join(ROOT, "profiles", rnd, f"{rnd}_{fmt}")
        if os.path.exists(path):
            return path
    return os.path.join(ROOT, "profiles", "r4", f"r4_{fmt}")


PMC_SUMMARY = {8: _latest_profile("pmc_summary.json"), 16: _latest_profile("10bit_pmc_summary.json")}
KERNEL_STATS = {8: _latest_profile("kernel_stats.csv"), 16: _latest_profile("10bit_kernel_stats.csv")}


def pmc_traffic(bpc):
    """HBM bytes per launch of the same kernels from the committed rocprofv3
    PMC summary (FETCH_SIZE and WRITE_SIZE, separate --pmc passes, KB as
    rocprofv3 reports them).  PMC needs rocprofv3 around the process, so a
    plain bench run cannot re-measure it; the source file is named."""
    path = PMC_SUMMARY[bpc]
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    tot = 0.0
    for k, v in d.items():
        if k.startswith(f"k_recon<{bpc},") and "FETCH_SIZE" in v and "WRITE_SIZE" in v:
            tot += (v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024
    if not tot:
        return None, None
    return int(tot), (f"FETCH_SIZE+WRITE_SIZE per frame from {os.path.relpath(path, ROOT)} "
                      "(uncorrected: the gfx950 x2 FETCH factor holds for wide coalesced reads, "
                      "not these scattered row loads)")


def rocprof_kernel_us(bpc):
    """Average duration (us) of the frame's k_recon launches in the committed
    rocprofv3 --kernel-trace --stats summary (sum over the launch groups of
    one frame), or None."""
    import csv
    try:
        rows = list(csv.DictReader(open(KERNEL_STATS[bpc])))
    except OSError:
        return None
    us = 0.0
    for r in rows:
        name = r.get("Name", "")
        if f"k_recon<{bpc}," in name or f"k_reconILi{bpc}E" in name:
            us += float(r["AverageNs"]) / 1e3
    return round(us, 2) if us else None


FAMILIES = {
    # per-family frames ("also report per-family Gpix/s")
    "mc": "inter only: mc put / mct x2 + avg per block, no residual",
    "ipred": "intra only: the 14 intra_pred modes + CfL per transform block, no residual",
    "itx": "inv_txfm_add only: residual 4x4..32x32 onto an existing picture (dst read + write)",
    "ext": "the other batch kinds with residual: mc put / avg / w_avg / mask compound and pal_pred blocks",
}


def kernel_seconds(frame, stream, n):
    """Mean launch duration over n back-to-back launches: one pair of HIP
    events on the launch stream around all of them (an event pair around
    every launch adds the event packets' own dispatch latency, ~2-3 us, to
    each: measured 60.7 us against rocprofv3's 58.1 us for the same kernel)."""
    import torch
    frame.launch(stream)   # warm
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for _ in range(n):
        frame.launch(stream)
    b.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e-3 / n


def config_legs(dev, stream, steps):
    """BASELINE.json configs[1] and configs[3] at N=1 beside the headline:
    the 1080p mc-only frame and the 10-bit 4K full frame, one launch each
    (kernel time by HIP events on the launch stream)."""
    import dav1d_mirror_amd.workload as wl
    import dav1d_mirror_amd.batch as bt
    out = {}
    for name in ("1080p-mc", "4k-10bit"):
        c = dict(CONFIGS[name])
        label = c.pop("label")
        fd = wl.make_frame(wl.FrameConfig(**c))
        frame = bt.DeviceFrame(fd, dev)
        for _ in range(3):
            frame.launch(stream)
        ks = kernel_seconds(frame, stream, max(steps, 10))
        b = fd.stats["total_bytes"]
        out[name] = {"workload": label, "units": fd.n_units, "pixels": fd.stats["pixels"],
                     "kernel_us": round(ks * 1e6, 2), "gpix_s": round(fd.stats["pixels"] / ks / 1e9, 2),
                     "algorithmic_bytes": b, "achieved_gbs": round(b / ks / 1e9, 1),
                     "frac": round(b / ks / 1e9 / HBM_PEAK_GBS, 4), "desc_bytes": fd.stats["desc_bytes"],
                     "rocprof_kernel_us": rocprof_kernel_us(c.get("bpc", 8)) if name == "4k-10bit" else None}
        del frame
    return out


def cold_mall_leg(fd, dev, stream, steps, copies=6):
    """The headline frame with the 256 MB MALL (Infinity Cache) cold: launches
    rotate over `copies` device-resident copies of the frame (distinct
    buffers, > 256 MB together), so each launch's reads miss the MALL left
    by the previous one and FETCH_SIZE-style accounting measures HBM."""
    import dav1d_mirror_amd.batch as bt
    frames = [bt.DeviceFrame(fd, dev) for _ in range(copies)]
    foot = sum(sum(t.numel() * t.element_size() for t in f.device_tensors()) for f in frames)
    for f in frames:
        f.launch(stream)
    n = max(steps, 12)
    n -= n % copies
    a, b = torch_event(), torch_event()
    a.record(stream)
    for i in range(n):
        frames[i % copies].launch(stream)
    b.record(stream)
    import torch
    torch.cuda.synchronize()
    ks = a.elapsed_time(b) * 1e-3 / n
    b = fd.stats["total_bytes"]
    del frames
    return {"copies": copies, "footprint_bytes": int(foot), "kernel_us": round(ks * 1e6, 2),
            "gpix_s": round(fd.stats["pixels"] / ks / 1e9, 2), "achieved_gbs": round(b / ks / 1e9, 1),
            "frac": round(b / ks / 1e9 / HBM_PEAK_GBS, 4)}


def torch_event():
    import torch
    return torch.cuda.Event(enable_timing=True)


def family_breakdown(base_cfg, dev, stream, steps):
    import dav1d_mirror_amd.workload as wl
    import dav1d_mirror_amd.batch as bt
    out = {}
    for kind, what in FAMILIES.items():
        fd = wl.make_frame(dataclasses.replace(base_cfg, kind=kind))
        frame = bt.DeviceFrame(fd, dev)
        for _ in range(3):
            frame.launch(stream)
        ks = kernel_seconds(frame, stream, max(steps, 10))
        out[kind] = {"workload": what, "units": fd.n_units, "pixels": fd.stats["pixels"],
                     "kernel_us": round(ks * 1e6, 2), "gpix_s": round(fd.stats["pixels"] / ks / 1e9, 2),
                     "algorithmic_bytes": fd.stats["total_bytes"],
                     "achieved_gbs": round(fd.stats["total_bytes"] / ks / 1e9, 1),
                     "frac": round(fd.stats["total_bytes"] / ks / 1e9 / HBM_PEAK_GBS, 4)}
        del frame
    return out


def tile_breakdown(fd, dev, stream, steps):
    """The same frame through the superblock-tile batch (dav1d_gpu_recon_tiles_*):
    block-level mc with clamped (emu_edge) footprints, one workgroup per
    64x64 luma / 32x32 chroma tile.  Reported beside the headline unit batch."""
    import dav1d_mirror_amd.tiles as tl
    import dav1d_mirror_amd.batch as bt
    td = tl.build_tiles(fd)
    frame = bt.DeviceTiles(fd, td, dev)
    for _ in range(3):
        frame.launch(stream)
    ks = kernel_seconds(frame, stream, max(steps, 10))
    b = td.stats["total_bytes"]
    out = {"kernel": "k_tiles<bpc, huge=false/true>", "tiles": int(len(td.tiles)), "preds": int(len(td.preds)),
           "txs": int(len(td.txs)), "kernel_us": round(ks * 1e6, 2),
           "gpix_s": round(fd.stats["pixels"] / ks / 1e9, 2), "algorithmic_bytes": b,
           "achieved_gbs": round(b / ks / 1e9, 1), "frac": round(b / ks / 1e9 / HBM_PEAK_GBS, 4)}
    del frame
    return out


def intra_breakdown(cfg, dev, stream, steps):
    """an all-intra frame of the config's size and
    bitdepth reconstructed on the device by the intra wavefront
    (dav1d_gpu_recon_intra_frame_*: persistent -- the headline ms_per_frame --
    one launch per frame whose waves wait on their producers' tasks; sb, one
    launch per frame, a workgroup per superblock (DGPU_IS_SB); levels,
    the same launch waiting on per-level counters; and fused, one launch per
    level), one
    tile and 2x2 tiles; beside it the oracle in the decoder's own order on
    one host core.  Reported beside the headline, not part of it."""
    import dav1d_mirror_amd.intra as intra
    out = {}
    orc = ge.load_oracle()
    for name, tiles in (("1_tile", (1, 1)), ("2x2_tiles", (2, 2))):
        fr = intra.make_intra_frame(intra.IntraConfig(width=cfg.width, height=cfg.height, bpc=cfg.bpc,
                                                      bitdepth_max=cfg.bitdepth_max, tile_cols=tiles[0],
                                                      tile_rows=tiles[1]))
        ms, got, flow_error = {}, {}, 0
        for mode in ("sb", "persistent", "levels", "fused"):
            frame = intra.DeviceIntraFrame(fr, dev, mode=mode)
            for _ in range(2):
                frame.launch(stream)
            ms[mode] = kernel_seconds(frame, stream, max(3, min(steps, 5)))
            if mode in ("sb", "persistent"):
                flow_error |= frame.flow_error()
                got[mode] = frame.planes_host()
            del frame
        ks = ms["persistent"]
        ho = orc.HostIntraFrame(fr)
        t0 = time.perf_counter()
        ho.run()
        cpu_s = time.perf_counter() - t0
        px = sum(w * h for w, h in fr.plane_wh)
        n_sb = len(intra.sb_schedule(fr)[3]) - 1
        out[name] = {"units": int(len(fr.units)), "levels": int(fr.n_levels), "superblocks": n_sb,
                     "ms_per_frame": round(ks * 1e3, 3), "gpix_s": round(px / ks / 1e9, 4),
                     "us_per_level": round(ks * 1e6 / fr.n_levels, 2),
                     "sb_ms_per_frame": round(ms["sb"] * 1e3, 3),
                     "levels_ms_per_frame": round(ms["levels"] * 1e3, 3),
                     "fused_ms_per_frame": round(ms["fused"] * 1e3, 3),
                     "oracle_1core_ms": round(cpu_s * 1e3, 2), "flow_error": flow_error,
                     "bit_exact_vs_oracle": all(bool(np.array_equal(g, o)) for m in got for g, o in zip(got[m], ho.dst))}
    return out


def recorder_breakdown(cfg, dev):
    """a 4K mixed frame (70% inter blocks) handed to the
    native batch recorder block by block and residual by residual
    (dav1d_gpu_rec_*), then one flush: the flush's host time (the call's wall
    time: uploading the recording and waiting for the device-side cut and
    schedule on the recorder's stream, then the launches), the device time
    of that prep (HIP events on the recorder's stream) and of the picture's
    work on the caller's stream (HIP events with the GPU kept busy while the
    host builds), their sum the flush's device time, checked against the
    oracle."""
    import torch
    import dav1d_mirror_amd.intra as intra
    fr = intra.make_intra_frame(intra.IntraConfig(width=cfg.width, height=cfg.height, bpc=cfg.bpc,
                                                  bitdepth_max=cfg.bitdepth_max, inter_frac=0.7,
                                                  sb_edge_backup=False))
    hbd = cfg.bpc != 8
    pdt = torch.int16 if hbd else torch.uint8
    dst = [torch.zeros((h, w), dtype=pdt, device=dev) for (w, h) in fr.plane_wh]
    refs = [[(torch.from_numpy((x.view(np.int16) if hbd else x).copy()).to(dev), fr.ref_origin_offset(p),
              fr.plane_wh[p][0], fr.plane_wh[p][1]) for p, x in enumerate(rp)] for rp in fr.refs]
    rec = intra.Recorder(cfg.bpc, cfg.bitdepth_max, cfg.width, cfg.height, dev.index or 0)
    s = torch.cuda.current_stream(dev)
    host, devt, prep = [], [], []
    for _ in range(2):
        intra.replay(rec, fr)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(int(0.2 * 2.0e9))
        e0.record(s)
        t0 = time.perf_counter()
        rec.flush(dst, refs, s)
        host.append(time.perf_counter() - t0)
        e1.record(s)
        torch.cuda.synchronize(dev)
        devt.append(e0.elapsed_time(e1) * 1e-3)
        prep.append(rec.prep_ms() * 1e-3)
    n_units, n_levels = rec.stats()
    rec.close()
    ho = ge.load_oracle().HostIntraFrame(fr)
    ho.run()
    got = [(t.cpu().numpy().view(np.uint16) if hbd else t.cpu().numpy()) for t in dst]
    px = sum(w * h for w, h in fr.plane_wh)
    ok = all(bool(np.array_equal(g, o)) for g, o in zip(got, ho.dst))
    # frame threads: F recorders (one per frame, as dav1d's frame threads
    # would own them) flushing at once from F host threads on F streams;
    # host time per frame = the wall time of the concurrent flushes / F
    import threading
    nf = max(1, min(4, len(os.sched_getaffinity(0)) // 2 if hasattr(os, "sched_getaffinity") else 2))
    recs = [intra.Recorder(cfg.bpc, cfg.bitdepth_max, cfg.width, cfg.height, dev.index or 0) for _ in range(nf)]
    dsts = [[torch.zeros((h, w), dtype=pdt, device=dev) for (w, h) in fr.plane_wh] for _ in range(nf)]
    streams = [torch.cuda.Stream(dev) for _ in range(nf)]
    # one untimed flush per recorder first: a frame thread reuses its
    # recorder frame after frame, so the timed flushes are warm ones (the
    # first flush of a recorder also allocates its staging and device
    # buffers, and page-locking memory serialises across threads)
    for r_, d_, s_ in zip(recs, dsts, streams):
        intra.replay(r_, fr)
        r_.flush(d_, refs, s_)
    torch.cuda.synchronize(dev)
    for r_ in recs:
        intra.replay(r_, fr)
    torch.cuda.synchronize(dev)
    torch.cuda._sleep(int(0.3 * 2.0e9))   # the device busy: host time only
    go = threading.Barrier(nf + 1)

    def flush_one(i):
        go.wait()
        recs[i].flush(dsts[i], refs, streams[i])
    ths = [threading.Thread(target=flush_one, args=(i,)) for i in range(nf)]
    for t in ths:
        t.start()
    go.wait()
    t0 = time.perf_counter()
    for t in ths:
        t.join()
    wall = time.perf_counter() - t0
    torch.cuda.synchronize(dev)
    ok_par = all(bool(np.array_equal((t.cpu().numpy().view(np.uint16) if hbd else t.cpu().numpy()), o))
                 for d in dsts for t, o in zip(d, ho.dst))
    for r_ in recs:
        r_.close()
    return {"frame": f"{cfg.width}x{cfg.height}, 70% inter blocks", "units": n_units, "levels": n_levels,
            # the flush's device time is all the device work it queues: the
            # prep on the recorder's stream (the call waits for it, so it is
            # inside flush_host_ms too) and the picture's work on the caller's
            "flush_host_ms": round(host[-1] * 1e3, 2), "flush_device_ms": round((devt[-1] + prep[-1]) * 1e3, 3),
            "flush_prep_device_ms": round(prep[-1] * 1e3, 3), "flush_picture_device_ms": round(devt[-1] * 1e3, 3),
            "device_gpix_s": round(px / (devt[-1] + prep[-1]) / 1e9, 3), "bit_exact_vs_oracle": ok,
            "frame_threads": {"frames": nf, "host_threads": nf, "wall_ms": round(wall * 1e3, 2), "warm": True,
                              "flush_host_ms_per_frame": round(wall * 1e3 / nf, 2), "bit_exact_vs_oracle": ok_par}}


def grain_breakdown(cfg, dev, steps):
    """film grain (dav1d_gpu_apply_grain_*) on a picture
    of the config's size and bitdepth, lag-3 auto-regression, overlap on,
    grain on all planes: ms per picture (prep + apply launches) by HIP
    events, and the oracle's time on one core, bit-exact check."""
    import torch
    import dav1d_mirror_amd.grain as grain
    c = grain.make_grain_case(seed=5, width=cfg.width, height=cfg.height, bpc=cfg.bpc,
                              bitdepth_max=cfg.bitdepth_max, lag=3, num_y=8, csfl=False, num_uv=(6, 6),
                              overlap=True)
    g = grain.DeviceGrain(c, dev)
    s = torch.cuda.current_stream(dev)
    for _ in range(3):
        g.launch(s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = max(steps, 10)
    e0.record(s)
    for _ in range(n):
        g.launch(s)
    e1.record(s)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / n
    t0 = time.perf_counter()
    outs, _, _ = ge.load_oracle().apply_grain(c)
    cpu = time.perf_counter() - t0
    px = sum(w * h for w, h in c.plane_wh)
    bpp = 1 if cfg.bpc == 8 else 2
    return {"picture": f"{cfg.width}x{cfg.height} 4:2:0", "ms_per_picture": round(ms, 4),
            "gpix_s": round(px / ms / 1e6, 2), "picture_io_bytes": 2 * px * bpp,
            "oracle_1core_ms": round(cpu * 1e3, 1),
            "bit_exact_vs_oracle": all(bool(np.array_equal(a, b)) for a, b in zip(g.outputs_host(), outs))}


def cdef_breakdown(cfg, dev, steps):
    """CDEF (dav1d_gpu_cdef_frame_*, dav1d_cdef_brow over
    a whole deblocked frame) on a synthetic picture of the config's size and
    bitdepth, 4:2:0, random strengths, 10% of superblocks and 15% of 8x8
    blocks skipped: us per frame by HIP events, algorithmic GB/s (picture
    read once and written once) against the HBM peak, the oracle's walker on
    one core, bit-exact check."""
    import torch
    import dav1d_mirror_amd.cdef as cdef
    c = cdef.make_cdef_case(seed=11, width=cfg.width, height=cfg.height, bpc=cfg.bpc,
                            bitdepth_max=cfg.bitdepth_max, layout=1)
    d = cdef.DeviceCdef(c, dev)
    s = torch.cuda.current_stream(dev)
    for _ in range(3):
        d.launch(s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = max(steps, 20)
    e0.record(s)
    for _ in range(n):
        d.launch(s)
    e1.record(s)
    torch.cuda.synchronize(dev)
    us = e0.elapsed_time(e1) * 1e3 / n
    t0 = time.perf_counter()
    want = ge.load_oracle().cdef_frame(c)
    cpu = time.perf_counter() - t0
    nbytes = cdef.algorithmic_bytes(c)
    px = sum(w * h for w, h in (c.plane_wh(p) for p in range(3)))
    return {"frame": f"{cfg.width}x{cfg.height} 4:2:0", "us_per_frame": round(us, 2),
            "gpix_s": round(px / us / 1e3, 2), "algorithmic_bytes": nbytes,
            "achieved_gbs": round(nbytes / us / 1e3, 1), "frac_of_hbm_peak": round(nbytes / us / 1e3 / HBM_PEAK_GBS, 4),
            "kernel": f"k_cdef<{cfg.bpc},1>", "oracle_1core_ms": round(cpu * 1e3, 1),
            "bit_exact_vs_oracle": all(bool(np.array_equal(a, b)) for a, b in zip(d.outputs_host(), want))}


def superres_breakdown(cfg, dev, steps):
    """super-res (dav1d_gpu_resize_frame_*, dav1d_filter_
    sbrow_resize over a whole frame) of a picture upscaled to the config's
    size from half its width (denominator 16), 4:2:0: us per frame by HIP
    events, algorithmic GB/s (source read once, output written once), the
    oracle's superblock-row walk on one core, bit-exact check."""
    import torch
    import dav1d_mirror_amd.superres as sr
    c = sr.make_case(cfg.width, cfg.height, 16, layout=1, bpc=cfg.bpc, bitdepth_max=cfg.bitdepth_max, seed=11)
    d = sr.DeviceResize(c, dev)
    s = torch.cuda.current_stream(dev)
    for _ in range(3):
        d.launch(s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = max(steps, 20)
    e0.record(s)
    for _ in range(n):
        d.launch(s)
    e1.record(s)
    torch.cuda.synchronize(dev)
    us = e0.elapsed_time(e1) * 1e3 / n
    t0 = time.perf_counter()
    want = ge.load_oracle().resize_frame(c)
    cpu = time.perf_counter() - t0
    nbytes = sr.algorithmic_bytes(c)
    px = sum(a.shape[0] * c.dst_w[p] for p, a in enumerate(c.ins))
    return {"frame": f"{c.w}x{cfg.height} -> {cfg.width}x{cfg.height} 4:2:0", "us_per_frame": round(us, 2),
            "gpix_s": round(px / us / 1e3, 2), "algorithmic_bytes": nbytes,
            "achieved_gbs": round(nbytes / us / 1e3, 1), "frac_of_hbm_peak": round(nbytes / us / 1e3 / HBM_PEAK_GBS, 4),
            "kernel": f"k_resize_frame<{cfg.bpc}>", "oracle_1core_ms": round(cpu * 1e3, 1),
            "bit_exact_vs_oracle": all(bool(np.array_equal(a, b)) for a, b in zip(d.outputs_host(), want))}


def lpf_breakdown(cfg, dev, steps):
    """the deblocking loop filter (dav1d_gpu_loopfilter_
    frame_*: every column edge, then every row edge) on a synthetic frame of
    the config's size and bitdepth, 4:2:0, random transform quadtree per 64x64
    with the edge masks and levels it implies: us per frame (both launches)
    by HIP events over repeated in-place launches, algorithmic GB/s (each
    pass reads and writes the picture once), the oracle's superblock-row
    walker on one core, bit-exact check from the unfiltered picture."""
    import torch
    import dav1d_mirror_amd.lpf as lpf
    c = lpf.make_lpf_case(seed=11, width=cfg.width, height=cfg.height, bpc=cfg.bpc,
                          bitdepth_max=cfg.bitdepth_max, layout=1)
    d = lpf.DeviceLpf(c, dev)
    s = torch.cuda.current_stream(dev)
    for _ in range(3):
        d.launch(s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = max(steps, 20)
    e0.record(s)
    for _ in range(n):
        d.launch(s)
    e1.record(s)
    torch.cuda.synchronize(dev)
    us = e0.elapsed_time(e1) * 1e3 / n
    d.reset()
    d.launch(s)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    want = ge.load_oracle().loopfilter_frame(c)
    cpu = time.perf_counter() - t0
    nbytes = lpf.algorithmic_bytes(c)
    px = sum(w * h for w, h in (c.plane_wh(p) for p in range(3)))
    return {"frame": f"{cfg.width}x{cfg.height} 4:2:0", "us_per_frame": round(us, 2),
            "gpix_s": round(px / us / 1e3, 2), "algorithmic_bytes": nbytes,
            "achieved_gbs": round(nbytes / us / 1e3, 1), "frac_of_hbm_peak": round(nbytes / us / 1e3 / HBM_PEAK_GBS, 4),
            "kernel": f"k_lpf<{cfg.bpc},0> + k_lpf<{cfg.bpc},1>", "oracle_1core_ms": round(cpu * 1e3, 1),
            "bit_exact_vs_oracle": all(bool(np.array_equal(a, b)) for a, b in zip(d.outputs_host(), want))}


def lr_breakdown(cfg, dev, steps):
    """loop restoration (dav1d_gpu_lr_frame_*:
    dav1d_lr_sbrow over a frame) on a synthetic CDEF output of the config's
    size and bitdepth, 4:2:0, 64-px luma / 32-px chroma units, a mix of
    Wiener, self-guided and unrestored units: us per frame by HIP events,
    algorithmic GB/s (picture read once, written once), the oracle's walker on
    one core, bit-exact check."""
    import torch
    import dav1d_mirror_amd.lr as lr
    c = lr.make_lr_case(seed=11, width=cfg.width, height=cfg.height, bpc=cfg.bpc, bitdepth_max=cfg.bitdepth_max,
                        layout=1, unit_log2=(6, 5))
    d = lr.DeviceLr(c, dev)
    s = torch.cuda.current_stream(dev)
    for _ in range(3):
        d.launch(s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = max(steps, 20)
    e0.record(s)
    for _ in range(n):
        d.launch(s)
    e1.record(s)
    torch.cuda.synchronize(dev)
    us = e0.elapsed_time(e1) * 1e3 / n
    t0 = time.perf_counter()
    want = ge.load_oracle().lr_frame(c)
    cpu = time.perf_counter() - t0
    nbytes = lr.algorithmic_bytes(c)
    px = sum(w * h for w, h in (c.plane_wh(p) for p in range(3)))
    return {"frame": f"{cfg.width}x{cfg.height} 4:2:0", "us_per_frame": round(us, 2),
            "gpix_s": round(px / us / 1e3, 2), "algorithmic_bytes": nbytes,
            "achieved_gbs": round(nbytes / us / 1e3, 1), "frac_of_hbm_peak": round(nbytes / us / 1e3 / HBM_PEAK_GBS, 4),
            "kernel": f"k_lr_frame<{cfg.bpc}>", "oracle_1core_ms": round(cpu * 1e3, 1),
            "bit_exact_vs_oracle": all(bool(np.array_equal(a, b)) for a, b in zip(d.outputs_host(), want))}


def spawn_ranks(n, argv):
    """`bench.py --gpus N` without a launcher (WORLD_SIZE unset): start N
    rank processes of this script with the rank environment torchrun would
    set (one per GPU, RCCL rendezvous on 127.0.0.1), before this process has
    touched the GPU, and exit with the first failing rank's status.  Rank 0
    prints the JSON line; the others' stdout goes to stderr."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=None if r == 0 else sys.stderr))
    return wait_ranks(procs)


def wait_ranks(procs, poll_s=0.2):
    """Poll every rank (waiting in rank order blocks forever when a
    later rank dies while rank 0 sits in a rendezvous or barrier).  On the
    first non-zero exit the other ranks are terminated (then killed) and that
    status is returned; 0 when every rank exits cleanly."""
    import time as _t
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad:
            log(f"bench: rank exit codes {codes}: stopping the others")
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            t_end = _t.time() + 10
            for p in procs:
                try:
                    p.wait(timeout=max(0.1, t_end - _t.time()))
                except Exception:
                    p.kill()
                    p.wait()
            return bad[0]
        if all(c == 0 for c in codes):
            return 0
        _t.sleep(poll_s)


def per_rank_fields(kernel_us, ms_per_step):
    """The N>1 line's per-rank view: each rank's kernel time
    and time per step, in rank order, with the max over ranks (the rank that
    sets the aggregate's clock)."""
    return {"kernel_us": [round(v, 2) for v in kernel_us], "kernel_us_max": round(max(kernel_us), 2),
            "ms_per_step": [round(v, 4) for v in ms_per_step], "ms_per_step_max": round(max(ms_per_step), 4),
            "slowest_rank": int(np.argmax(ms_per_step))}


def dry_run(world, rank, local):
    """--dry-run: the N-rank wiring without a GPU (gloo): every rank joins the
    process group, passes the barrier and the max-over-ranks reduction the
    timed region uses; rank 0 prints what it saw.  No bench number."""
    import torch.distributed as dist
    import dav1d_mirror_amd.shard as sh
    if world > 1:
        dist.init_process_group("gloo")
        dist.barrier()
    got = sh.max_over_ranks(float(rank), dist, "cpu")
    total = sh.sum_over_ranks(1, dist, "cpu")
    per_rank = sh.gather_over_ranks(10.0 + rank, dist, "cpu")   # stands in for each rank's kernel_us
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "ranks_joined": total, "max_rank": got,
                          "local_rank": local, "per_rank": per_rank_fields(per_rank, per_rank)}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="4k", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--no-check", action="store_true",
                    help="skip the bit-exact check of rank 0's timed frame against the oracle (on by default)")
    ap.add_argument("--feed", default="local", choices=["local", "rccl"],
                    help="local: each rank generates its frame; rccl: rank 0 generates all and scatters")
    ap.add_argument("--no-families", action="store_true", help="skip the per-family breakdown (N=1)")
    ap.add_argument("--no-configs", action="store_true", help="skip the 1080p-mc / 4k-10bit legs (N=1)")
    ap.add_argument("--no-tiles", action="store_true", help="skip the tile-batch measurement (N=1)")
    ap.add_argument("--no-intra", action="store_true", help="skip the intra-wavefront measurement (N=1)")
    ap.add_argument("--no-recorder", action="store_true", help="skip the batch-recorder measurement (N=1)")
    ap.add_argument("--no-grain", action="store_true", help="skip the film-grain measurement (N=1)")
    ap.add_argument("--no-cdef", action="store_true", help="skip the CDEF measurement (N=1)")
    ap.add_argument("--no-superres", action="store_true", help="skip the super-res measurement (N=1)")
    ap.add_argument("--no-lpf", action="store_true", help="skip the deblocking measurement (N=1)")
    ap.add_argument("--no-lr", action="store_true", help="skip the loop-restoration measurement (N=1)")
    ap.add_argument("--dry-run", action="store_true",
                    help="check the N-rank wiring only (gloo, no GPU, no bench number)")
    args = ap.parse_args()

    # --gpus N is honoured: without a launcher this process starts the N
    # ranks itself (before any GPU call); under a launcher its WORLD_SIZE must
    # agree.  A 1-rank number is never reported under --gpus N > 1
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        ap.error(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N ranks for --gpus N")
    if args.dry_run:
        ge.load_package()
        dry_run(world, rank, local)
        return

    import torch
    import torch.distributed as dist

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
    base = wl.FrameConfig(**c)
    cfg = sh.rank_config(base, rank)
    t0 = time.perf_counter()
    feed = None
    if args.feed == "rccl" and world > 1:
        fd, feed_s, feed_bytes = sh.feed_frame(lambda r: sh.rank_config(base, r), rank, world, dist, dev)
        feed_s = sh.max_over_ranks(feed_s, dist, dev)
        feed_bytes = sh.sum_over_ranks(feed_bytes if rank else 0, dist, dev)
        feed = {"kind": "rccl send/recv from rank 0 (scatter of independent frames)",
                "bytes": feed_bytes, "ms": round(feed_s * 1e3, 3),
                "gbs": round(feed_bytes / feed_s / 1e9, 2) if feed_s > 0 else None,
                "note": "outside the timed region; kernel-phase scaling excludes it (SURVEY 8(e))"}
    else:
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

    # timed region: exactly K steps, barrier + synchronize on both sides.
    # One HIP event pair on the launch stream brackets the same K launches
    # inside it; the kernel time per launch is that stream time / K, which
    # sits inside the wall-clock bracket and so never exceeds the time per
    # step (frac comes from it; the launches are back to back,
    # so it matches rocprofv3's per-launch duration)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        frame.launch(stream)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    barrier()
    my_el = time.perf_counter() - t0
    el = sh.max_over_ranks(my_el, dist, dev)
    stream_s = ev0.elapsed_time(ev1) * 1e-3 / args.steps
    kern_s = stream_s
    assert kern_s <= my_el / args.steps * (1 + 1e-6), (kern_s, my_el / args.steps)

    # diagnostic only (outside the timed region, not used for frac): an event
    # pair around each launch; the pairs add their own packets' latency
    nk = min(args.steps, 100)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(nk)]
    for a, b in evs:
        a.record(stream)
        frame.launch(stream)
        b.record(stream)
    torch.cuda.synchronize(dev)
    pair_s = sum(a.elapsed_time(b) for a, b in evs) * 1e-3 / nk
    per_rank = None
    if world > 1:
        per_rank = per_rank_fields([v * 1e6 for v in sh.gather_over_ranks(kern_s, dist, dev)],
                                   [v * 1e3 / args.steps for v in sh.gather_over_ranks(my_el, dist, dev)])

    # the timed frame's pixels against the oracle (outside the timed region;
    # the launches are idempotent, so the picture is the last step's)
    check = None
    if not args.no_check and rank == 0:
        orc = ge.load_oracle()
        hf = orc.HostFrame(fd)
        nthr = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else 4))
        t1 = time.perf_counter()
        hf.run(threads=nthr)
        got = frame.planes_host()
        check = all(np.array_equal(got[p], hf.dst[p]) for p in range(3))
        log(f"[rank 0] bit-exact vs oracle: {check} ({time.perf_counter() - t1:.1f} s on {nthr} threads)")

    if rank == 0:
        traffic, traffic_note = pmc_traffic(cfg.bpc) if args.config in ("4k", "4k-10bit") else (None, None)
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
            "ms_per_step": round(el / args.steps * 1e3, 5),
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
                "library_sources": dict(zip(("built_from", "tree", "matches_tree"), pkg.abi.build_stamp())),
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
                          "the 64-point group launches only when such units exist)",
                "kernel_us": round(kern_s * 1e6, 2),
                "kernel_us_note": "one HIP event pair on the launch stream around the K timed launches "
                                  "(inside the wall-clock bracket, so <= ms_per_step), / K; frac uses it",
                "event_pair_us_diag": round(pair_s * 1e6, 2),
                "event_pair_note": f"diagnostic only: mean of {nk} launches each bracketed by its own event "
                                   "pair (adds the event packets' latency; not used for frac)",
                "rocprof_kernel_us": rocprof_kernel_us(cfg.bpc) if args.config != "1080p-mc" else None,
                "frac_rocprof": (round(bytes_launch / (rocprof_kernel_us(cfg.bpc) * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
                                 if args.config != "1080p-mc" and rocprof_kernel_us(cfg.bpc) else None),
                "rocprof_source": os.path.relpath(KERNEL_STATS[cfg.bpc], ROOT),
                "algorithmic_bytes_per_launch": bytes_launch,
                "bytes_breakdown": {k: fd.stats[k] for k in
                                    ("ref_bytes", "edge_bytes", "coef_bytes", "dst_bytes", "dst_read_bytes",
                                     "aux_bytes")},
                "desc_bytes": fd.stats["desc_bytes"],
                "accounting": "achieved = algorithmic bytes per launch (SURVEY 8(d): per-block reference "
                              "footprints + edges + stored coefficients + output, no descriptors) / mean "
                              "launch duration by HIP events on the launch stream",
            },
        }
        if check is not None:
            out["config"]["bit_exact_vs_oracle"] = check
        if feed is not None:
            out["feed"] = feed
        if per_rank is not None:
            out["per_rank"] = per_rank
        if not args.no_configs and world == 1 and args.config == "4k":
            out["configs"] = config_legs(dev, stream, args.steps)
        if not args.no_configs and world == 1 and args.config == "4k":
            out["cold_mall"] = cold_mall_leg(fd, dev, stream, args.steps)
        if not args.no_families and world == 1 and c.get("kind") == "full":
            out["families"] = family_breakdown(cfg, dev, stream, args.steps)
        if not args.no_tiles and world == 1:
            out["tile_batch"] = tile_breakdown(fd, dev, stream, args.steps)
        if not args.no_intra and world == 1 and c.get("kind") == "full":
            out["intra_wavefront"] = intra_breakdown(cfg, dev, stream, args.steps)
        if not args.no_recorder and world == 1 and c.get("kind") == "full":
            out["recorder"] = recorder_breakdown(cfg, dev)
        if not args.no_grain and world == 1:
            out["film_grain"] = grain_breakdown(cfg, dev, args.steps)
        if not args.no_cdef and world == 1:
            out["cdef"] = cdef_breakdown(cfg, dev, args.steps)
        if not args.no_superres and world == 1:
            out["superres"] = superres_breakdown(cfg, dev, args.steps)
        if not args.no_lpf and world == 1:
            out["loop_filter"] = lpf_breakdown(cfg, dev, args.steps)
        if not args.no_lr and world == 1:
            out["loop_restoration"] = lr_breakdown(cfg, dev, args.steps)
        if not args.no_cpu and world == 1:
            out["cpu_baseline"] = cpu_baseline(fd)
        # (on the unrounded values: the stream events sit inside the wall-clock bracket)
        assert kern_s <= el / args.steps * (1 + 1e-6), "kernel time exceeds the step time"
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
