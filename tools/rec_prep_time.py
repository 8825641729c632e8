"""The recorder's flush on the GPU, 4K mixed frame (bench.py's recorder leg
without the oracle): per flush the call's host time, the prep's device time
(dav1d_gpu_recorder_prep_ms) and the caller stream's device time, warm
flushes.  DAV1D_GPU_REC_TIMING=1 adds the host laps on stderr; run under
rocprofv3 --kernel-trace --stats for the prep's kernels.

  python tools/rec_prep_time.py [--reps 5] [--width 3840 --height 2160]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--inter", type=float, default=0.7)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--threads", type=int, default=0, help="also: N recorders flushing at once from N threads")
    ap.add_argument("--busy", action="store_true",
                    help="threads: the device kept busy by a 0.3 s kernel on the default stream meanwhile (as bench.py)")
    a = ap.parse_args()
    import torch
    import __graft_entry__ as ge
    ge.load_package()
    import dav1d_mirror_amd.intra as intra
    fr = intra.make_intra_frame(intra.IntraConfig(width=a.width, height=a.height, inter_frac=a.inter,
                                                  sb_edge_backup=False))
    dev = torch.device("cuda:0")
    dst = [torch.zeros((h, w), dtype=torch.uint8, device=dev) for (w, h) in fr.plane_wh]
    refs = [[(torch.from_numpy(x.copy()).to(dev), fr.ref_origin_offset(p), fr.plane_wh[p][0], fr.plane_wh[p][1])
             for p, x in enumerate(rp)] for rp in (fr.refs or [])]
    rec = intra.Recorder(8, 255, a.width, a.height)
    s = torch.cuda.current_stream(dev)
    rows = []
    for i in range(a.reps + 1):
        intra.replay(rec, fr)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        t0 = time.perf_counter()
        rec.flush(dst, refs, s)
        t1 = time.perf_counter()
        e1.record(s)
        torch.cuda.synchronize(dev)
        row = dict(host_ms=round(1e3 * (t1 - t0), 3), prep_ms=round(rec.prep_ms(), 3),
                   stream_ms=round(e0.elapsed_time(e1), 3))
        print(("warm-up " if i == 0 else "") + str(row), flush=True)
        if i:
            rows.append(row)
    print({k: round(float(np.median([r[k] for r in rows])), 3) for k in rows[0]}, "median units", rec.stats())
    rec.close()
    if a.threads:   # frame threads: one recorder and stream per thread, flushed together (warm)
        import threading
        nf = a.threads
        recs = [intra.Recorder(8, 255, a.width, a.height) for _ in range(nf)]
        dsts = [[torch.zeros((h, w), dtype=torch.uint8, device=dev) for (w, h) in fr.plane_wh] for _ in range(nf)]
        sts = [torch.cuda.Stream(dev) for _ in range(nf)]
        for rep in range(3):
            for r_ in recs:
                intra.replay(r_, fr)
            torch.cuda.synchronize(dev)
            if a.busy:
                torch.cuda._sleep(int(0.3 * 2.0e9))
            go = threading.Barrier(nf + 1)
            hms = [0.0] * nf

            def one(i):
                go.wait()
                t0 = time.perf_counter()
                recs[i].flush(dsts[i], refs, sts[i])
                hms[i] = 1e3 * (time.perf_counter() - t0)
            ths = [threading.Thread(target=one, args=(i,)) for i in range(nf)]
            for t in ths:
                t.start()
            go.wait()
            t0 = time.perf_counter()
            for t in ths:
                t.join()
            wall = 1e3 * (time.perf_counter() - t0)
            torch.cuda.synchronize(dev)
            print(f"threads {nf} rep {rep}: wall {wall:.2f} ms, per frame {wall / nf:.2f} ms, host ms "
                  f"{[round(h, 2) for h in hms]}, prep ms {[round(r_.prep_ms(), 2) for r_ in recs]}", flush=True)
        for r_ in recs:
            r_.close()


if __name__ == "__main__":
    main()
