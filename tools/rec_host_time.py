"""Host-only timing of the batch recorder's flush (no GPU needed): the
frame is replayed into a recorder and flushed with DAV1D_GPU_REC_HOSTONLY=1
(cutting, edge records, levels, sort, fill; nothing uploaded) and
DAV1D_GPU_REC_TIMING=1 (per-phase times on stderr).

  DAV1D_GPU_REC_HOSTONLY=1 DAV1D_GPU_REC_TIMING=1 python tools/rec_host_time.py [--width 3840 --height 2160]
"""
import argparse
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--inter", type=float, default=0.7)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    assert os.environ.get("DAV1D_GPU_REC_HOSTONLY"), "set DAV1D_GPU_REC_HOSTONLY=1"
    import __graft_entry__ as ge
    ge.load_package()
    import dav1d_mirror_amd.abi as abi
    import dav1d_mirror_amd.intra as intra
    fr = intra.make_intra_frame(intra.IntraConfig(width=a.width, height=a.height, inter_frac=a.inter,
                                                  sb_edge_backup=False))
    rec = intra.Recorder(8, 255, a.width, a.height)
    L = rec.lib
    d = (abi.Plane * 3)()
    for p, (w, h) in enumerate(fr.plane_wh):
        d[p].data, d[p].stride, d[p].w, d[p].h = 0x1000, w, w, h
    r = ((abi.Plane * 3) * abi.MAX_REFS)()
    for k in range(2):
        for p, (w, h) in enumerate(fr.plane_wh):
            r[k][p].data, r[k][p].stride, r[k][p].w, r[k][p].h = 0x1000, w + 2 * fr.cfg.ref_pad, w, h
    for _ in range(a.reps):
        intra.replay(rec, fr)
        t0 = time.perf_counter()
        rc = L.dav1d_gpu_recorder_flush(rec.h, ctypes.byref(d), ctypes.byref(r), None)
        t1 = time.perf_counter()
        print(f"flush rc {rc}: {1e3 * (t1 - t0):.2f} ms, units {rec.stats()[0]}", flush=True)


if __name__ == "__main__":
    main()
