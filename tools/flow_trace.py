"""Per-task timeline of the persistent intra wavefront (DGPU_FLOW_TRACE
build: DAV1D_GPU_LIB_VARIANT=ftrace).  Prints, per level, the wake latency
(first task ready after the previous level's last release), the slowest
task's compute time and the release time, averaged over levels."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    import __graft_entry__ as ge
    ge.load_package()
    import dav1d_mirror_amd.intra as intra
    import dav1d_mirror_amd.abi as abi
    w, h = (int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "3840x2160").split("x"))
    fr = intra.make_intra_frame(intra.IntraConfig(width=w, height=h))
    dev = intra.DeviceIntraFrame(fr, mode="persistent")
    phases = None
    if os.environ.get("DAV1D_GPU_LIB_VARIANT") == "fphase":   # + the class code's marks per task (group 8)
        phases = torch.zeros(9 << 20, dtype=torch.int64, device="cuda:0")
        os.environ["DAV1D_GPU_FLOW_PHASES"] = str(phases.data_ptr())
    for _ in range(3):
        dev.launch()
    torch.cuda.synchronize()
    # the task list as the library builds it (levels, classes largest first)
    order = [3, 9, 10, 2, 15, 16, 7, 8, 1, 13, 14, 5, 6, 0, 4, 11, 12, 17, 18]
    lanes = {}
    for t, (tw, th) in enumerate(abi.TX_WH):
        # lanes_per_unit, csrc/recon_kernel.hpp
        lanes[t] = 64 if tw * th >= 1024 else min(max(min(tw * th // 8, max(tw, min(th, 32))), 2), 64)
        lanes[t] = {(8, 16): 8, (4, 16): 4, (8, 32): 16}.get((tw, th), lanes[t])   # the tall classes
        if os.environ.get("DGPU_IE_WIDE_LANES", "1") == "1":   # the wavefront TUs since round 6
            lanes[t] = min(max(tw * th // 8, 2), 64)
        if tw * th <= 32:   # the wavefront TUs: DGPU_IE_SMALL_LANES (recon_ie{8,16}.hip)
            lanes[t] = int(os.environ.get("DGPU_IE_SMALL_LANES", "8"))
    levels, classes, firsts = [], [], []
    tg_all = intra.task_group_bytes(fr)
    for l in range(fr.n_levels):
        cs = fr.class_start[l]
        for c in order:
            n = int(cs[c + 1] - cs[c])
            U = min(64 // lanes[c], int(os.environ.get("DAV1D_GPU_FLOW_UNITS", "8"))) if l else 64 // lanes[c]
            tg = tg_all if (l and os.environ.get("FLOW_TASK_GROUPS", "0") == "1") else None   # (the library's cut)
            i, e_ = int(fr.unit_start[l] + cs[c]), int(fr.unit_start[l] + cs[c + 1])
            while i < e_:
                e = min(i + U, e_)
                if tg is not None:
                    k = i + 1
                    while k < e and tg[k] == tg[i]:
                        k += 1
                    e = k
                levels.append(l)
                classes.append(c)
                firsts.append(i)
                i = e
    nt = len(levels)
    ws = dev.workspace.cpu().numpy()
    # the trace is the workspace's last part (flow_layout: counters, done
    # flags, tasks, level counts, producer lists, trace)
    n, nd = len(fr.units), len(fr.deps)
    base = (32 + 16 * fr.n_levels) * 4 + ((n * 4 + 15) & ~15) + nt * 16 + fr.n_levels * 4 + (n + 1) * 4 + nd * 4
    base = (base + 15) & ~15
    assert base + nt * 32 == len(ws), (base + nt * 32, len(ws))   # same task list as the library
    tr = ws[base:base + nt * 32].view(np.uint64).reshape(nt, 4).astype(np.int64)
    lv = np.array(levels)
    ready_first = np.full(fr.n_levels, np.iinfo(np.int64).max)
    rel_last = np.zeros(fr.n_levels, np.int64)
    comp_max = np.zeros(fr.n_levels, np.int64)
    np.minimum.at(ready_first, lv, tr[:, 1])
    np.maximum.at(rel_last, lv, tr[:, 3])
    np.maximum.at(comp_max, lv, tr[:, 2] - tr[:, 1])
    wake = ready_first[1:] - rel_last[:-1]
    rel = tr[:, 3] - tr[:, 2]
    span = (rel_last[-1] - tr[:, 0].min())
    out = {"levels": int(fr.n_levels), "tasks": int(nt), "frame_us": span / 100.0,
           "per_level_us": span / 100.0 / fr.n_levels,
           "wake_us_mean": float(wake.mean()) / 100.0, "wake_us_p50": float(np.median(wake)) / 100.0,
           "slowest_task_compute_us_mean": float(comp_max.mean()) / 100.0,
           "task_compute_us_p50": float(np.median(tr[:, 2] - tr[:, 1])) / 100.0,
           "release_us_p50": float(np.median(rel)) / 100.0,
           "ticket_to_ready_us_p50": float(np.median(tr[:, 1] - tr[:, 0])) / 100.0}
    # per class: the post-wait part (ready -> computed) and how often a task
    # of the class is its level's slowest; per prediction kind of the
    # slowest tasks
    comp = tr[:, 2] - tr[:, 1]
    cl = np.array(classes)
    slow = np.zeros(nt, bool)
    for l in range(fr.n_levels):
        idx = np.nonzero(lv == l)[0]
        slow[idx[np.argmax(comp[idx])]] = True
    per = {}
    for c in sorted(set(classes)):
        m = cl == c
        tw, th = abi.TX_WH[c]
        per[f"{tw}x{th}"] = {"tasks": int(m.sum()), "p50_us": round(float(np.median(comp[m])) / 100.0, 2),
                             "p90_us": round(float(np.percentile(comp[m], 90)) / 100.0, 2),
                             "slowest_of_level": int((slow & m).sum())}
    out["per_class"] = per
    kinds = {}
    fi = np.array(firsts)
    for t in np.nonzero(slow)[0]:
        u = fr.units[fi[t]]
        k = "cfl" if u["pred"] == abi.PRED_CFL else f"mode{int(u['mode']) & 15}"
        kinds[k] = kinds.get(k, 0) + 1
    out["slowest_task_kind"] = dict(sorted(kinds.items(), key=lambda kv: -kv[1]))
    if phases is not None:
        # marks (recon_kernel.hpp mark(i)): 0 entry, 2 loads committed, 4 row
        # transforms done, 5 after the wait and the edge gather, 8 stored;
        # tr[:, 1] is the end of the wait (same 100 MHz clock)
        m = phases.cpu().numpy()[8 << 20:(8 << 20) + nt * 16].reshape(nt, 16).astype(np.int64)
        ok = (m[:, 0] > 0) & (m[:, 5] > 0) & (m[:, 8] > 0)
        ph = {}
        for c in sorted(set(classes)):
            sel = ok & (cl == c)
            if not sel.any():
                continue
            tw, th = abi.TX_WH[c]
            f = lambda v: round(float(np.median(v)) / 100.0, 2)   # noqa: E731
            ph[f"{tw}x{th}"] = {"loads_us": f(m[sel, 2] - m[sel, 0]), "to_row_tx_us": f(m[sel, 4] - m[sel, 2]),
                                "wait_end_to_gathered_us": f(m[sel, 5] - tr[sel, 1]),
                                "gathered_to_stored_us": f(m[sel, 8] - m[sel, 5]),
                                "stored_to_released_us": f(tr[sel, 3] - m[sel, 8])}
        out["phases_p50"] = ph
        # 4x4 tasks by the intra modes of their units (device-rewritten modes:
        # the remapped mode the prediction ran), the post-gather phase
        uu = dev.units.cpu().numpy().view(fr.units.dtype)
        c44 = [c for c in set(classes) if tuple(abi.TX_WH[c]) == (4, 4)][0]
        cnt = np.array([min(64 // lanes[c_], int(os.environ.get("DAV1D_GPU_FLOW_UNITS", "8"))) if lv[t] else 64 // lanes[c_]
                        for t, c_ in enumerate(classes)])
        bym, bynm = {}, {}
        for t in np.nonzero(ok & (cl == c44))[0]:
            f0 = fi[t]
            n_ = min(cnt[t], int(fr.unit_start[lv[t] + 1]) - f0)
            mset = sorted(set(int(x) for x in (uu["mode"][f0:f0 + n_] & 15)))
            key = "pal" if uu["pred"][f0] == abi.PRED_PAL else "cfl" if uu["pred"][f0] == abi.PRED_CFL else str(mset[0])
            bym.setdefault(key, []).append(m[t, 8] - m[t, 5])
            bynm.setdefault(len(mset), []).append(m[t, 8] - m[t, 5])
        out["4x4_gathered_to_stored_p50_by_first_mode"] = {k: [len(v), round(float(np.median(v)) / 100.0, 2)]
                                                           for k, v in sorted(bym.items())}
        out["4x4_gathered_to_stored_p50_by_modes_in_task"] = {k: [len(v), round(float(np.median(v)) / 100.0, 2)]
                                                              for k, v in sorted(bynm.items())}
        sl = ok & slow
        out["slowest_tasks_phases_mean_us"] = {
            "wait_end_to_gathered": round(float((m[sl, 5] - tr[sl, 1]).mean()) / 100.0, 2),
            "gathered_to_stored": round(float((m[sl, 8] - m[sl, 5]).mean()) / 100.0, 2),
            "stored_to_released": round(float((tr[sl, 3] - m[sl, 8]).mean()) / 100.0, 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
