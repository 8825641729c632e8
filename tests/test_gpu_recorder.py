"""GPU parity of the batch recorder (dav1d_gpu_recorder_*): frames handed
over block by block and residual by residual, as recon_b_inter /
recon_b_intra would (dav1d_mirror_amd.intra.replay), cut into units,
scheduled and reconstructed natively, against the oracle's decoder-order
walk of the same frame.  Bit-exact bar."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(oracle, **kw):
    import torch
    import dav1d_mirror_amd.intra as intra
    fr = intra.make_intra_frame(intra.IntraConfig(**kw))
    hbd = fr.cfg.bpc != 8
    pdt = torch.int16 if hbd else torch.uint8
    dst = [torch.zeros((h, w), dtype=pdt, device="cuda:0") for (w, h) in fr.plane_wh]
    refs = []
    for rp in fr.refs or []:
        planes = []
        for p, a in enumerate(rp):
            t = torch.from_numpy((a.view(np.int16) if hbd else a).copy()).to("cuda:0")
            planes.append((t, fr.ref_origin_offset(p), fr.plane_wh[p][0], fr.plane_wh[p][1]))
        refs.append(planes)
    rec = intra.Recorder(fr.cfg.bpc, fr.cfg.bitdepth_max, fr.cfg.width, fr.cfg.height)
    intra.replay(rec, fr)
    rec.flush(dst, refs, torch.cuda.current_stream())
    torch.cuda.synchronize()
    n_units, n_levels = rec.stats()
    assert n_units == len(fr.units)
    ho = oracle.HostIntraFrame(fr)
    ho.run()
    for p in range(3):
        got = dst[p].cpu().numpy()
        got = got.view(np.uint16) if hbd else got
        diff = np.argwhere(got != ho.dst[p])
        assert len(diff) == 0, f"plane {p}: {len(diff)} pixels differ, first {diff[:5].tolist()}"
    rec.close()
    return fr, n_levels


@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023), (16, 4095)])
def test_recorder_intra_frame(oracle, bpc, bdmax):
    fr, n_levels = _run(oracle, seed=51, bpc=bpc, bitdepth_max=bdmax, sb_edge_backup=False)
    assert n_levels == fr.n_levels   # the native scheduler finds the same levels


@pytest.mark.parametrize("kw", [dict(seed=52, inter_frac=0.5, tile_cols=2),
                                dict(seed=53, inter_frac=0.3, bpc=16, bitdepth_max=1023),
                                dict(seed=54, inter_frac=1.0),
                                dict(seed=55, cfl_frac=1.0, tile_cols=3, tile_rows=2, width=640, height=384),
                                dict(seed=56, width=1920, height=1080, inter_frac=0.3)])
def test_recorder_mixed(oracle, kw):
    _run(oracle, sb_edge_backup=False, **kw)


def _setup(fr):
    import torch
    hbd = fr.cfg.bpc != 8
    pdt = torch.int16 if hbd else torch.uint8
    pad = getattr(fr, "dst_pad", 0)   # room for transform blocks overhanging the picture
    dst = [torch.zeros((h + pad, w + pad), dtype=pdt, device="cuda:0") for (w, h) in fr.plane_wh]
    refs = []
    for rp in fr.refs or []:
        planes = []
        for p, a in enumerate(rp):
            t = torch.from_numpy((a.view(np.int16) if hbd else a).copy()).to("cuda:0")
            planes.append((t, fr.ref_origin_offset(p), fr.plane_wh[p][0], fr.plane_wh[p][1]))
        refs.append(planes)
    return dst, refs


def _compare(fr, dst, oracle):
    ho = oracle.HostIntraFrame(fr)
    ho.run()
    hbd = fr.cfg.bpc != 8
    for p in range(3):
        w, h = fr.plane_wh[p]
        got = dst[p][:h, :w].cpu().numpy()
        got = got.view(np.uint16) if hbd else got
        diff = np.argwhere(got != ho.dst[p])
        assert len(diff) == 0, f"plane {p}: {len(diff)} pixels differ, first {diff[:5].tolist()}"


@pytest.mark.parametrize("inter_frac", [0.0, 0.4])
def test_recorder_flush_per_superblock_row(oracle, inter_frac):
    """One flush per 64-px superblock row: intra units of a row
    read edges and CfL luma that an earlier flush reconstructed on the same
    stream; those pixels have no producer in the current flush."""
    import torch
    import dav1d_mirror_amd.intra as intra
    fr = intra.make_intra_frame(intra.IntraConfig(seed=57, width=512, height=320, inter_frac=inter_frac,
                                                  sb_edge_backup=False))
    dst, refs = _setup(fr)
    rec = intra.Recorder(fr.cfg.bpc, fr.cfg.bitdepth_max, fr.cfg.width, fr.cfg.height)
    s = torch.cuda.current_stream()
    total = 0
    for y0 in range(0, fr.cfg.height, 64):
        intra.replay(rec, fr, rows=(y0, y0 + 64))
        rec.flush(dst, refs, s)
        total += rec.stats()[0]
    assert rec.status() == 0
    torch.cuda.synchronize()
    assert total == len(fr.units)
    _compare(fr, dst, oracle)
    rec.close()


def test_recorder_reports_wavefront_stall(oracle, monkeypatch):
    """A wavefront that gives up waiting (forced: DAV1D_GPU_FLOW_SPIN_LIMIT=0)
    is reported by dav1d_gpu_recorder_status, once; the next flush then runs
    normally and the picture is right again."""
    import torch
    import dav1d_mirror_amd.intra as intra
    fr = intra.make_intra_frame(intra.IntraConfig(seed=58, width=512, height=256, sb_edge_backup=False))
    dst, refs = _setup(fr)
    rec = intra.Recorder(fr.cfg.bpc, fr.cfg.bitdepth_max, fr.cfg.width, fr.cfg.height)
    s = torch.cuda.current_stream()
    monkeypatch.setenv("DAV1D_GPU_FLOW_SPIN_LIMIT", "0")
    intra.replay(rec, fr)
    rec.flush(dst, refs, s)
    monkeypatch.delenv("DAV1D_GPU_FLOW_SPIN_LIMIT")
    assert rec.status() == -6
    assert rec.status() == 0   # reported once
    # the same stall not read through status() comes back from the next flush,
    # which then launches nothing and keeps its recording
    monkeypatch.setenv("DAV1D_GPU_FLOW_SPIN_LIMIT", "0")
    intra.replay(rec, fr)
    rec.flush(dst, refs, s)
    monkeypatch.delenv("DAV1D_GPU_FLOW_SPIN_LIMIT")
    intra.replay(rec, fr)
    assert rec.flush_rc(dst, refs, s) == -6
    for t in dst:
        t.zero_()
    assert rec.flush_rc(dst, refs, s) == 0   # the kept recording, run normally
    assert rec.status() == 0
    torch.cuda.synchronize()
    _compare(fr, dst, oracle)
    rec.close()


def test_recorder_rejects_missing_reference(oracle):
    """An inter block naming a reference plane the flush does not give is
    an error (-1), not a read through a NULL pointer."""
    import torch
    import dav1d_mirror_amd.intra as intra
    fr = intra.make_intra_frame(intra.IntraConfig(seed=59, width=256, height=128, inter_frac=1.0,
                                                  sb_edge_backup=False))
    dst, refs = _setup(fr)
    rec = intra.Recorder(fr.cfg.bpc, fr.cfg.bitdepth_max, fr.cfg.width, fr.cfg.height)
    intra.replay(rec, fr)
    assert rec.flush_rc(dst, None, torch.cuda.current_stream()) == -1
    rec.close()


@pytest.mark.parametrize("bpc,bdmax,seed,ext", [(8, 255, 61, 0.0), (16, 1023, 62, 0.0), (16, 4095, 63, 0.0),
                                                  (8, 255, 64, 0.8), (16, 1023, 65, 0.8), (16, 4095, 66, 0.8)])
def test_recorder_unpadded_references(oracle, bpc, bdmax, seed, ext):
    """References without padding and MVs up to 200 px past the picture
    (VERDICT r2): every read is clamped to the picture, as mc()'s emu_edge
    copy makes it (src/recon_tmpl.c:986-999).  The device gets exact-size
    reference planes (stride = width, so an unclamped read lands on another
    row); the oracle reads edge-replicated copies padded past every MV.
    With ext: the launch-ahead kinds too: WARP 8x8 origins,
    INTER_WMASK / OBMC lap MVs and scaled positions up to 200 px outside
    (scaled :1036-1046, warp :1168-1177)."""
    import torch
    import dav1d_mirror_amd.abi as abi
    import dav1d_mirror_amd.intra as intra
    fr = intra.make_intra_frame(intra.IntraConfig(seed=seed, width=384, height=256, bpc=bpc, bitdepth_max=bdmax,
                                                  inter_frac=0.8, mv_range=200, ref_pad=288, ext_frac=ext,
                                                  sb_edge_backup=False))
    if ext:
        kinds = set(int(k) for k in fr.units["pred"])
        assert {abi.PRED_WARP, abi.PRED_INTER_WMASK, abi.PRED_INTER_OBMC, abi.PRED_INTER_SCALED} <= kinds
    hbd = bpc != 8
    dst = [torch.zeros((h, w), dtype=torch.int16 if hbd else torch.uint8, device="cuda:0") for (w, h) in fr.plane_wh]
    pad = fr.cfg.ref_pad
    refs = []
    for rp in fr.refs:
        planes = []
        for p, a in enumerate(rp):
            w, h = fr.plane_wh[p]
            crop = np.ascontiguousarray(a[pad:pad + h, pad:pad + w])
            t = torch.from_numpy(crop.view(np.int16) if hbd else crop).to("cuda:0")
            planes.append((t, 0, w, h))
        refs.append(planes)
    rec = intra.Recorder(fr.cfg.bpc, fr.cfg.bitdepth_max, fr.cfg.width, fr.cfg.height)
    intra.replay(rec, fr)
    rec.flush(dst, refs, torch.cuda.current_stream())
    torch.cuda.synchronize()
    assert rec.status() == 0
    _compare(fr, dst, oracle)
    rec.close()


@pytest.mark.parametrize("bpc,bdmax,seed", [(8, 255, 81), (16, 1023, 82), (16, 4095, 83)])
def test_recorder_block_data_kinds(oracle, bpc, bdmax, seed):
    """Blocks recorded with their data (dav1d_gpu_rec_block_aux): INTER_MASK
    (caller masks, and COMPOUND_SEG chroma on the luma's w_mask output),
    palette, WARP, INTER_WMASK, INTER_OBMC, INTER_SCALED and inter-intra (its
    intra edges gathered in the wavefront), beside intra /
    CfL / inter blocks whose edges read them.  The recorder cuts the
    launch-ahead kinds into prediction units and adds their residuals in the
    wavefront; the oracle walks its own cut of the same blocks in decoder
    order (dav1d_mirror_amd.intra._ExtBuilder)."""
    import torch
    import dav1d_mirror_amd.intra as intra
    fr = intra.make_intra_frame(intra.IntraConfig(seed=seed, width=384, height=256, bpc=bpc, bitdepth_max=bdmax,
                                                  inter_frac=0.6, ext_frac=0.7, sb_edge_backup=False))
    kinds = set(int(k) for k in fr.units["pred"])
    import dav1d_mirror_amd.abi as abi
    assert {abi.PRED_INTER_MASK, abi.PRED_PAL, abi.PRED_WARP, abi.PRED_INTER_WMASK, abi.PRED_INTER_OBMC,
            abi.PRED_INTER_SCALED, abi.PRED_INTER_INTRA} <= kinds
    dst, refs = _setup(fr)
    rec = intra.Recorder(fr.cfg.bpc, fr.cfg.bitdepth_max, fr.cfg.width, fr.cfg.height)
    intra.replay(rec, fr)
    rec.flush(dst, refs, torch.cuda.current_stream())
    torch.cuda.synchronize()
    assert rec.status() == 0
    _compare(fr, dst, oracle)
    rec.close()


def test_recorder_block_data_per_superblock_row(oracle):
    """The same kinds flushed per 64-px superblock row: a COMPOUND_SEG chroma
    block finds its luma's mask in the same flush; flushes with only
    launch-ahead work are valid."""
    import torch
    import dav1d_mirror_amd.intra as intra
    fr = intra.make_intra_frame(intra.IntraConfig(seed=84, width=384, height=256, inter_frac=0.7, ext_frac=0.8,
                                                  sb_edge_backup=False))
    dst, refs = _setup(fr)
    rec = intra.Recorder(fr.cfg.bpc, fr.cfg.bitdepth_max, fr.cfg.width, fr.cfg.height)
    s = torch.cuda.current_stream()
    for y0 in range(0, fr.cfg.height, 64):
        intra.replay(rec, fr, rows=(y0, y0 + 64))
        rec.flush(dst, refs, s)
    assert rec.status() == 0
    torch.cuda.synchronize()
    _compare(fr, dst, oracle)
    rec.close()


@pytest.mark.parametrize("kw", [dict(width=1920, height=1080, seed=95, inter_frac=0.4),
                                dict(width=992, height=552, seed=96, inter_frac=0.3, bpc=16, bitdepth_max=1023),
                                dict(width=992, height=552, seed=97, inter_frac=0.6, ext_frac=0.6, tile_cols=2)])
def test_recorder_overhanging_blocks(oracle, kw):
    """Blocks that run past the right / bottom edge, as AV1's partition allows
    (ADVICE r2): 1080 rows (not a multiple of 64) and a 992 x 552 picture.
    The recorder cuts only the part inside the 8-aligned grid into transform
    blocks (recon_tmpl.c:1208 w4 / h4), which may overhang into the plane's
    padding; TOP_HAS_RIGHT / LEFT_HAS_BOTTOM follow the clipped block, intra
    max_w / max_h the grid, CfL's cfl_ac pads the luma past the edge."""
    import torch
    import dav1d_mirror_amd.intra as intra
    fr = intra.make_intra_frame(intra.IntraConfig(overhang=True, sb_edge_backup=False, **kw))
    assert any(y + s_ > fr.cfg.height or x + s_ > fr.cfg.width for (p, x, y, s_, *_r) in fr.blocks if p == 0)
    dst, refs = _setup(fr)
    rec = intra.Recorder(fr.cfg.bpc, fr.cfg.bitdepth_max, fr.cfg.width, fr.cfg.height)
    intra.replay(rec, fr)
    rec.flush(dst, refs, torch.cuda.current_stream())
    torch.cuda.synchronize()
    assert rec.status() == 0
    _compare(fr, dst, oracle)
    rec.close()


@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023)])
def test_recorder_lossless(oracle, bpc, bdmax):
    """Lossless (WHT_WHT) residuals handed to the recorder as
    dav1d_gpu_rec_residual calls with txtp 16."""
    fr, _ = _run(oracle, seed=57, inter_frac=0.4, bpc=bpc, bitdepth_max=bdmax, lossless=0.8,
                 sb_edge_backup=False)
    assert (fr.units["txtp"] == 16).sum() > 100


@pytest.mark.parametrize("kw", [dict(seed=58, inter_frac=0.4),
                                dict(seed=59, inter_frac=0.4, ext_frac=0.4, tile_cols=2),
                                dict(seed=60, inter_frac=0.3, bpc=16, bitdepth_max=1023, lossless=0.3)])
def test_recorder_top_edge_post_filter_interleave(oracle, kw):
    """dav1d_gpu_recorder_set_top_edge (f->ipred_edge, src/recon_tmpl.c:2162-2186
    and the top_sb_edge reads :1275-1279 / :1394-1398 / :1664-1668): one flush
    per superblock row, and after each flush the rows just reconstructed are
    checked and then overwritten in the picture, standing in for the
    decoder's in-place post-filters of that row (src/decode.c:3277).  Every
    later row must come out exact, so nothing read a superblock-top row from
    the picture; the backed-up rows equal the oracle's top_edge (launch-ahead
    predictions at superblock bottoms included, ext_frac)."""
    import torch
    import dav1d_mirror_amd.intra as intra
    fr = intra.make_intra_frame(intra.IntraConfig(width=512, height=320, sb_edge_backup=True, **kw))
    ho = oracle.HostIntraFrame(fr)
    ho.run()
    dst, refs = _setup(fr)
    hbd = fr.cfg.bpc != 8
    pdt = torch.int16 if hbd else torch.uint8
    sbl = [6, 5, 5]
    tops = [torch.full(((h + (1 << s) - 1 >> s) - 1, (w + (1 << s) - 1 >> s << s)), 0x5A, dtype=pdt, device="cuda:0")
            for (w, h), s in zip(fr.plane_wh, sbl)]
    rec = intra.Recorder(fr.cfg.bpc, fr.cfg.bitdepth_max, fr.cfg.width, fr.cfg.height)
    rec.set_top_edge(tops)
    s = torch.cuda.current_stream()
    gen = torch.Generator(device="cuda:0").manual_seed(5)
    for y0 in range(0, fr.cfg.height, 64):
        intra.replay(rec, fr, rows=(y0, y0 + 64))
        rec.flush(dst, refs, s)
        assert rec.status() == 0
        torch.cuda.synchronize()
        for p in range(3):
            w, h = fr.plane_wh[p]
            r0, r1 = y0 >> (p > 0), min(h, (y0 + 64) >> (p > 0))
            got = dst[p][r0:r1, :w].cpu().numpy()
            got = got.view(np.uint16) if hbd else got
            diff = np.argwhere(got != ho.dst[p][r0:r1])
            assert len(diff) == 0, f"rows {y0}+ plane {p}: {len(diff)} pixels differ, first {diff[:5].tolist()}"
            # the "post-filter": this row's pixels change in place
            dst[p][r0:r1] = torch.randint(0, fr.cfg.bitdepth_max + 1, dst[p][r0:r1].shape, generator=gen,
                                          device="cuda:0").to(pdt)
    for p in range(3):
        rows = tops[p].shape[0]
        w = fr.plane_wh[p][0]
        got = tops[p][:, :w].cpu().numpy()
        got = got.view(np.uint16) if hbd else got
        assert np.array_equal(got, ho.top[p][:rows, :w]), p
    rec.close()


def test_recorder_device_image_golden(tmp_path):
    """The flush's cut and schedule built on the device (csrc/rec_cut.hpp,
    csrc/recorder.hip) and read back: the upload image and schedule of
    tools/rec_dump.py's seven frames byte for byte as the round-6 host
    implementation made them (tests/golden/rec_dump_md5.json; the same
    frames' host-only steps are checked in test_cpu_recorder_golden.py).
    Dump mode launches nothing on the (dummy) pictures.  Every frame is
    flushed twice on one recorder, so the second recording streams to the
    device while it is made."""
    import json
    import os
    import re
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    want = json.load(open(os.path.join(root, "tests", "golden", "rec_dump_md5.json")))["frames"]
    env = dict(os.environ)
    env.pop("DAV1D_GPU_REC_HOSTONLY", None)
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "rec_dump.py"), str(tmp_path / "d.bin"),
                        "--device", "--twice"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    # each frame flushed twice on one recorder: the second recording's records
    # stream to the device while they are made (kStreamChunk pieces)
    for tag in ("frame", "again"):
        got = {m.group(1): (int(m.group(3)), m.group(4)) for m in
               re.finditer(tag + r" (\d+) rc (\S+) units (\d+) .* md5 (\w+)", r.stdout)}
        assert set(got) == set(want), r.stdout
        for k, w in want.items():
            assert got[k] == (w["units"], w["md5"]), (tag, k, got[k], w)
