"""CPU tests of the intra wavefront: the scheduler's
dependency levels replayed by the oracle in level order must give the
pixels of the decoder's own order (per transform block: prepare edges,
predict, add the residual; top_edge backed up at superblock-row ends,
src/recon_tmpl.c:1195-1596, :2162, src/decode.c:2677), plus the schedule's
structural invariants."""
import numpy as np
import pytest


def _frame(**kw):
    import dav1d_mirror_amd.intra as intra
    return intra.make_intra_frame(intra.IntraConfig(**kw))


@pytest.mark.parametrize("kw", [dict(), dict(seed=2, cfl_frac=1.0), dict(seed=3, filter_edge=False, tx64=False),
                                dict(seed=4, bpc=16, bitdepth_max=1023), dict(seed=5, bpc=16, bitdepth_max=4095),
                                dict(seed=6, width=480, height=264),
                                dict(seed=8, width=640, height=384, tile_cols=3, tile_rows=2),
                                dict(seed=9, tile_cols=2, sb_edge_backup=False),
                                dict(seed=10, inter_frac=0.5), dict(seed=11, inter_frac=0.8, bpc=16, bitdepth_max=1023)])
def test_level_order_equals_decode_order(pkg, oracle, kw):
    fr = _frame(**kw)
    a = oracle.HostIntraFrame(fr)
    a.run()
    b = oracle.HostIntraFrame(fr)
    b.run_levels()
    for p in range(3):
        assert np.array_equal(a.dst[p], b.dst[p]), p
        assert np.array_equal(a.top[p][:-1], b.top[p][:-1]), p   # (the last sb row is never backed up)
    assert np.array_equal(a.units, b.units)


@pytest.mark.parametrize("kw", [dict(seed=21), dict(seed=22, cfl_frac=1.0, bpc=16, bitdepth_max=1023),
                                dict(seed=23, width=640, height=384, tile_cols=3, tile_rows=2),
                                dict(seed=24, tile_cols=2, sb_edge_backup=False), dict(seed=25, inter_frac=0.5)])
def test_dataflow_order_equals_decode_order(pkg, oracle, kw):
    """Any order the producer lists allow (the persistent kernel's dataflow
    waits) gives the decoder's pixels."""
    fr = _frame(**kw)
    a = oracle.HostIntraFrame(fr)
    a.run()
    for seed in (1, 2):
        b = oracle.HostIntraFrame(fr)
        b.run_dataflow(seed)
        for p in range(3):
            assert np.array_equal(a.dst[p], b.dst[p]), (seed, p)
            assert np.array_equal(a.top[p][:-1], b.top[p][:-1]), (seed, p)
        assert np.array_equal(a.units, b.units)


def test_producer_lists(pkg):
    """A unit's level is one more than its highest producer's (0 without
    producers), producers sit at lower levels, lists are duplicate-free."""
    fr = _frame(seed=26, inter_frac=0.3)
    n = len(fr.units)
    lvl = np.repeat(np.arange(fr.n_levels), np.diff(fr.unit_start))
    assert fr.dep_start[0] == 0 and fr.dep_start[-1] == len(fr.deps) and len(fr.dep_start) == n + 1
    for u in range(n):
        d = fr.deps[fr.dep_start[u]:fr.dep_start[u + 1]]
        assert len(np.unique(d)) == len(d)
        assert lvl[u] == (lvl[d].max() + 1 if len(d) else 0)
        if fr.units["pred"][u] not in (pkg.abi.PRED_INTRA, pkg.abi.PRED_CFL):
            assert len(d) == 0                                  # inter units read only references


def test_schedule_invariants(pkg):
    abi = pkg.abi
    fr = _frame(seed=7)
    n = len(fr.units)
    assert fr.unit_start[0] == 0 and fr.unit_start[-1] == n
    assert fr.rec_start[-1] == len(fr.recs) == n          # every unit is intra or CfL here
    assert fr.run_start[-1] == len(fr.runs)
    assert np.array_equal(np.sort(fr.recs["unit"]), np.arange(n))
    for lv in range(fr.n_levels):
        u0, u1 = fr.unit_start[lv], fr.unit_start[lv + 1]
        assert u1 > u0                                      # no empty level
        t = fr.units["tx"][u0:u1]
        assert np.all(np.diff(t.astype(int)) >= 0)          # size classes contiguous
        assert np.array_equal(fr.class_start[lv], np.concatenate([[0], np.cumsum(np.bincount(t, minlength=abi.N_TX))]))
        r = fr.recs["unit"][fr.rec_start[lv]:fr.rec_start[lv + 1]]
        assert np.all((r >= u0) & (r < u1))                 # a level's records serve its units
    # every pixel of every plane is written by exactly one unit
    for p, (w, h) in enumerate(fr.plane_wh):
        cov = np.zeros((h, w), np.int32)
        for u in fr.units[fr.units["plane"] == p]:
            tw, th = abi.TX_WH[u["tx"]]
            y, x = divmod(int(u["dst_off"]), w)
            cov[y:y + th, x:x + tw] += 1
        assert np.all(cov == 1)
    # the wavefront is much shorter than the unit count
    assert fr.n_levels < n / 8


def test_intra_frame_launch_validation(pkg):
    import ctypes
    L = pkg.abi.load_lib()
    for bpc in (8, 16):
        fn = getattr(L, f"dav1d_gpu_recon_intra_frame_{bpc}bpc")
        rb, eb, s = pkg.abi.FrameBatch(), pkg.abi.IntraEdgeBatch(), pkg.abi.IntraSchedule()
        assert fn(None, None, None, None) == -1
        s.n_levels = 1
        assert fn(ctypes.byref(rb), ctypes.byref(eb), ctypes.byref(s), None) == -1   # NULL tables
        us = (ctypes.c_int32 * 2)(0, 5)
        cs = (ctypes.c_int32 * (pkg.abi.N_TX + 1))()
        z = (ctypes.c_int32 * 2)(0, 0)
        s.unit_start, s.class_start, s.rec_start, s.run_start = (ctypes.addressof(us), ctypes.addressof(cs),
                                                                  ctypes.addressof(z), ctypes.addressof(z))
        assert fn(ctypes.byref(rb), ctypes.byref(eb), ctypes.byref(s), None) == -2   # class_start != level size
        s.n_levels = 0
        assert fn(ctypes.byref(rb), ctypes.byref(eb), ctypes.byref(s), None) == 0
        bk = getattr(L, f"dav1d_gpu_backup_ipred_edge_{bpc}bpc")
        assert bk(None, None, 0, None) == -1
        assert bk(ctypes.byref(eb), None, 3, None) == -1
        assert bk(ctypes.byref(eb), None, 0, None) == 0


@pytest.mark.parametrize("kw", [dict(seed=27), dict(seed=28, sb_log2=7, width=512, height=384),
                                dict(seed=29, width=640, height=384, tile_cols=3, tile_rows=2, inter_frac=0.3),
                                dict(seed=30, bpc=16, bitdepth_max=1023, cfl_frac=1.0)])
def test_sb_schedule(pkg, kw):
    """The superblock schedule (DGPU_IS_SB, intra.sb_schedule): a
    permutation whose groups are (superblock, level) runs in superblock
    order, size classes inside a group; every producer of a unit sits in an
    earlier superblock the unit's superblock waits for, or in an earlier
    group of its own superblock."""
    abi = pkg.abi
    fr = _frame(**kw)
    n = len(fr.units)
    perm, cut, cls, sls, sds, sdeps = pkg.intra.sb_schedule(fr)
    assert np.array_equal(np.sort(perm), np.arange(n))
    inv = np.empty(n, np.int64)
    inv[perm] = np.arange(n)
    n_g, n_sb = len(cut) - 1, len(sls) - 1
    assert cut[0] == 0 and cut[-1] == n and np.all(np.diff(cut) > 0)
    assert sls[0] == 0 and sls[-1] == n_g and np.all(np.diff(sls) > 0)
    grp = np.repeat(np.arange(n_g), np.diff(cut))             # group of each position
    sb_of_g = np.repeat(np.arange(n_sb), np.diff(sls))
    for g in range(n_g):
        t = fr.units["tx"][perm[cut[g]:cut[g + 1]]]
        assert np.all(np.diff(t.astype(int)) >= 0)
        assert np.array_equal(cls[g], np.concatenate([[0], np.cumsum(np.bincount(t, minlength=abi.N_TX))]))
    for b in range(n_sb):
        d = sdeps[sds[b]:sds[b + 1]]
        assert np.all(d < b) and len(np.unique(d)) == len(d)
    for u in range(n):
        gu = grp[inv[u]]
        for q in fr.deps[fr.dep_start[u]:fr.dep_start[u + 1]]:
            gq = grp[inv[q]]
            if sb_of_g[gq] == sb_of_g[gu]:
                assert gq < gu
            else:
                b = sb_of_g[gu]
                assert sb_of_g[gq] in sdeps[sds[b]:sds[b + 1]]
    # far fewer steps on the critical path than levels: a superblock waits
    # for at most its left, top-left, top and top-right neighbours
    assert np.all(np.diff(sds) <= 4)


def _flow_tasks_py(pkg, fr, groups, cap=8, first_level=0):
    """The wave tasks flow_impl.hpp's flow_tasks cuts (classes largest first
    per level; above level 0 at most `cap` units, and with task groups never
    across a change of the group byte); levels below first_level left out
    (DGPU_IS_LEVEL0_BATCH)."""
    abi = pkg.abi
    order = [3, 9, 10, 2, 15, 16, 7, 8, 1, 13, 14, 5, 6, 0, 4, 11, 12, 17, 18]
    # the wavefront TUs (recon_ie{8,16}.hip): 4x4 / 4x8 / 8x4 units get 8
    # lanes (DGPU_IE_SMALL_LANES), every other class one 4x2 output task per
    # lane (DGPU_IE_WIDE_LANES: w * h / 8 lanes, 2..64)
    lanes = {}
    for t, (tw, th) in enumerate(abi.TX_WH):
        lanes[t] = 8 if tw * th <= 32 else min(max(tw * th // 8, 2), 64)
    n = 0
    for lv in range(first_level, fr.n_levels):
        cs = fr.class_start[lv]
        for c in order:
            full = 64 // lanes[c]
            U = min(full, cap) if lv else full
            i, e_ = int(fr.unit_start[lv] + cs[c]), int(fr.unit_start[lv] + cs[c + 1])
            while i < e_:
                e = min(i + U, e_)
                if groups is not None and lv:
                    k = i + 1
                    while k < e and groups[k] == groups[i]:
                        k += 1
                    e = k
                n += 1
                i = e
    return n


def test_flow_task_cut(pkg):
    """dav1d_gpu_intra_workspace_bytes (host code) sizes the persistent
    kernel's workspace from the tasks it cuts: with and without the
    schedule's task_group bytes it matches the Python restatement of the
    cut (size cap above level 0, then one group per task)."""
    import ctypes
    abi = pkg.abi
    fr = _frame(seed=42, width=512, height=256, inter_frac=0.3)
    L = abi.load_lib()
    n, nl = len(fr.units), fr.n_levels
    keep = [np.ascontiguousarray(a, np.int32) for a in (fr.unit_start, fr.class_start, fr.dep_start, fr.deps)]
    tg = pkg.intra.task_group_bytes(fr)
    for groups in (None, tg):
        s = abi.IntraSchedule()
        s.n_levels = nl
        s.flags = abi.IS_FUSED | abi.IS_PERSISTENT
        s.unit_start, s.class_start = keep[0].ctypes.data, keep[1].ctypes.data
        s.rec_start, s.run_start = keep[0].ctypes.data, keep[0].ctypes.data
        s.dep_start, s.deps = keep[2].ctypes.data, keep[3].ctypes.data
        if groups is not None:
            s.task_group = groups.ctypes.data
        nt = _flow_tasks_py(pkg, fr, groups)
        want = (32 + 16 * nl) * 4 + ((n * 4 + 15) & ~15) + nt * 16 + nl * 4 + (n + 1) * 4 + len(fr.deps) * 4
        assert L.dav1d_gpu_intra_workspace_bytes(ctypes.byref(s), n) == want, groups is not None
    assert _flow_tasks_py(pkg, fr, tg) > _flow_tasks_py(pkg, fr, None)
    # DGPU_IS_LEVEL0_BATCH (lead_levels.hpp): level 0 and each next level of
    # >= 2048 units run as launches of their own, out of the task list
    sizes = np.diff(np.asarray(fr.unit_start))
    lead = 1
    while lead < nl and sizes[lead] >= 2048:
        lead += 1
    s = abi.IntraSchedule()
    s.n_levels = nl
    s.flags = abi.IS_FUSED | abi.IS_PERSISTENT | abi.IS_LEVEL0_BATCH
    s.unit_start, s.class_start = keep[0].ctypes.data, keep[1].ctypes.data
    s.rec_start, s.run_start = keep[0].ctypes.data, keep[0].ctypes.data
    s.dep_start, s.deps = keep[2].ctypes.data, keep[3].ctypes.data
    nt = _flow_tasks_py(pkg, fr, None, first_level=lead)
    want = (32 + 16 * nl) * 4 + ((n * 4 + 15) & ~15) + nt * 16 + nl * 4 + (n + 1) * 4 + len(fr.deps) * 4
    assert L.dav1d_gpu_intra_workspace_bytes(ctypes.byref(s), n) == want
    assert nt < _flow_tasks_py(pkg, fr, None)
