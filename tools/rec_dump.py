"""Recorder flushes of several frames with the upload image and schedule
dumped (DAV1D_GPU_REC_DUMP): host-only (DAV1D_GPU_REC_HOSTONLY, the cut and
schedule steps run serially on the host, no GPU needed) or, with --device,
built by the device steps on the GPU and read back (nothing is launched on
the pictures, whose addresses are dummies).  Compares builds, and the device
against the host, byte for byte (tests/golden/rec_dump_md5.json).

  python tools/rec_dump.py OUT.bin [--only I] [--device] [--twice]   (prints one md5 per frame and flush)"""
import ctypes
import hashlib
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

FRAMES = [
    dict(width=3840, height=2160, inter_frac=0.7, sb_edge_backup=False),
    dict(width=1024, height=512, tile_cols=2, tile_rows=2, cfl_frac=0.6, sb_edge_backup=False),
    dict(width=992, height=552, inter_frac=0.6, ext_frac=0.5, overhang=True, tile_cols=2, sb_edge_backup=False),
    dict(width=512, height=256, bpc=16, bitdepth_max=1023, inter_frac=0.5, ext_frac=0.4, sb_edge_backup=False),
    dict(width=1920, height=1080, inter_frac=0.3, overhang=True, sb_log2=7, sb_edge_backup=False),
    # with top_edge (dav1d_gpu_recorder_set_top_edge): TOP_SB_EDGE flags and
    # the launch-ahead units' backup runs
    dict(seed=71, width=512, height=320, inter_frac=0.6, ext_frac=0.6, tile_cols=2, tile_rows=2, top=True),
    dict(seed=72, width=640, height=384, sb_log2=7, inter_frac=0.5, ext_frac=0.5, overhang=True, bpc=16,
         bitdepth_max=4095, top=True),
]


def main():
    out = sys.argv[1]
    only = int(sys.argv[sys.argv.index("--only") + 1]) if "--only" in sys.argv else None
    if "--device" not in sys.argv:
        os.environ["DAV1D_GPU_REC_HOSTONLY"] = "1"
    os.environ["DAV1D_GPU_REC_DUMP"] = out
    import __graft_entry__ as ge
    ge.load_package()
    import dav1d_mirror_amd.abi as abi
    import dav1d_mirror_amd.intra as intra
    for i, kw in enumerate(FRAMES):
        if only is not None and i != only:
            continue
        if os.path.exists(out):
            os.remove(out)
        kw = dict(kw)
        top = kw.pop("top", False)
        fr = intra.make_intra_frame(intra.IntraConfig(**(dict(kw, sb_edge_backup=True) if top else kw)))
        rec = intra.Recorder(fr.cfg.bpc, fr.cfg.bitdepth_max, fr.cfg.width, fr.cfg.height)
        if top:   # planes at a dummy address (nothing is uploaded host-only)
            t = (abi.Plane * 3)()
            sbl = fr.cfg.sb_log2
            for p, (w, h) in enumerate(fr.plane_wh):
                sh = sbl - (p > 0)
                t[p].data, t[p].w, t[p].h = 0x1000, ((w + (1 << sh) - 1) >> sh) << sh, ((h + (1 << sh) - 1) >> sh) - 1
                t[p].stride = t[p].w * (fr.cfg.bpc // 8)
            assert rec.lib.dav1d_gpu_recorder_set_top_edge(rec.h, ctypes.byref(t), int(sbl == 7)) == 0
        d = (abi.Plane * 3)()
        for p, (w, h) in enumerate(fr.plane_wh):
            pad = getattr(fr, "dst_pad", 0)
            d[p].data, d[p].stride, d[p].w, d[p].h = 0x1000, (w + pad) * (fr.cfg.bpc // 8), w, h
        r = ((abi.Plane * 3) * abi.MAX_REFS)()
        for k in range(2):
            for p, (w, h) in enumerate(fr.plane_wh):
                st = (w + 2 * fr.cfg.ref_pad) * (fr.cfg.bpc // 8)
                r[k][p].data, r[k][p].stride, r[k][p].w, r[k][p].h = 0x1000, st, w, h
        # --twice: the same recording flushed again on the same recorder (its
        # records then stream to the device while they are made)
        for rep in range(2 if "--twice" in sys.argv else 1):
            if os.path.exists(out):
                os.remove(out)
            intra.replay(rec, fr)
            t0 = time.perf_counter()
            rc = rec.lib.dav1d_gpu_recorder_flush(rec.h, ctypes.byref(d), ctypes.byref(r), None)
            t1 = time.perf_counter()
            md5 = hashlib.md5(open(out, "rb").read()).hexdigest() if os.path.exists(out) else None
            tag = f"frame {i}" if not rep else f"again {i}"
            print(f"{tag} rc {rc} units {rec.stats()[0]} flush {1e3 * (t1 - t0):.2f} ms md5 {md5}", flush=True)
        rec.close()


if __name__ == "__main__":
    main()
