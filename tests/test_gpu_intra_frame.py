"""GPU parity of the intra wavefront (dav1d_gpu_recon_intra_frame_*): a
whole all-intra frame reconstructed on the device level by level (edge
preparation -> unit batch -> top_edge backup runs) against the oracle in
the decoder's own order (oracle_recon_intra_frame).  Bit-exact bar: planes,
backed-up top_edge rows and the rewritten unit records."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _check(oracle, fr, mode="persistent"):
    import torch
    import dav1d_mirror_amd.intra as intra
    dev = intra.DeviceIntraFrame(fr, mode=mode)
    dev.launch()
    torch.cuda.synchronize()
    assert dev.flow_error() == 0
    got = dev.planes_host()
    ho = oracle.HostIntraFrame(fr)
    ho.run()
    for p in range(3):
        diff = np.argwhere(got[p] != ho.dst[p])
        assert len(diff) == 0, f"plane {p}: {len(diff)} pixels differ, first {diff[:5].tolist()}"
        top = dev.top[p].cpu().numpy()
        top = top if fr.cfg.bpc == 8 else top.view(np.uint16)
        assert np.array_equal(top[:-1], ho.top[p][:-1]), p
    assert np.array_equal(dev.units_frame_order(), ho.units)
    return dev, ho


def _frame(**kw):
    import dav1d_mirror_amd.intra as intra
    return intra.make_intra_frame(intra.IntraConfig(**kw))


@pytest.mark.parametrize("mode", ["persistent", "levels", "fused", "staged", "sb"])
@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023), (16, 4095)])
def test_intra_frame(oracle, bpc, bdmax, mode):
    """persistent: one launch per frame, waves wait on their producers'
    task flags; levels: the same, waiting on per-level counters; sb: one
    launch per frame, a workgroup per superblock (DGPU_IS_SB); fused: one launch per level (edges gathered in the reconstruction
    kernel, backups with the stores); staged: edge stage, unit batch and
    backup runs as three launches per level."""
    _check(oracle, _frame(seed=31, bpc=bpc, bitdepth_max=bdmax), mode=mode)


@pytest.mark.parametrize("kw", [dict(seed=32, cfl_frac=1.0), dict(seed=33, filter_edge=False, tx64=False),
                                dict(seed=34, width=480, height=264), dict(seed=35, sb_log2=7, width=512, height=384),
                                dict(seed=38, width=640, height=384, tile_cols=3, tile_rows=2),
                                dict(seed=39, tile_cols=2, sb_edge_backup=False)])
@pytest.mark.parametrize("mode", ["persistent", "sb"])
def test_intra_frame_variants(oracle, kw, mode):
    _check(oracle, _frame(**kw), mode=mode)


@pytest.mark.parametrize("mode", ["persistent", "levels", "fused", "staged", "sb", "lead"])
@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023)])
def test_mixed_frame(oracle, mode, bpc, bdmax):
    """Inter blocks (put / compound avg from padded references) among the
    intra ones: inter units sit at level 0, intra neighbours read their
    reconstructed pixels; the edge stage skips records of non-intra units."""
    _check(oracle, _frame(seed=41, inter_frac=0.5, bpc=bpc, bitdepth_max=bdmax, tile_cols=2), mode=mode)


@pytest.mark.parametrize("mode", ["persistent", "sb"])
def test_intra_frame_relaunch(oracle, mode):
    """reset() + launch again: the same pixels (the wavefront is repeatable)."""
    import torch
    dev, ho = _check(oracle, _frame(seed=36), mode=mode)
    first = [a.copy() for a in dev.planes_host()]
    dev.reset()
    dev.launch()
    torch.cuda.synchronize()
    for a, b in zip(first, dev.planes_host()):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("mode", ["persistent", "levels", "fused", "staged", "sb"])
def test_intra_frame_1080p(oracle, mode):
    """A 1080p intra frame (partial superblock row at the bottom)."""
    _check(oracle, _frame(seed=37, width=1920, height=1080), mode=mode)


@pytest.mark.parametrize("mode", ["persistent", "levels", "sb"])
def test_intra_frame_4k_persistent(oracle, mode):
    """A 4K intra frame (1603 levels) through the persistent kernel, twice."""
    import torch
    dev, ho = _check(oracle, _frame(seed=40, width=3840, height=2160), mode=mode)
    dev.reset()
    dev.launch()
    torch.cuda.synchronize()
    assert dev.flow_error() == 0
    for a, b in zip(dev.planes_host(), ho.dst):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("mode", ["persistent", "staged", "sb"])
@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023)])
def test_lossless_frame(oracle, mode, bpc, bdmax):
    """WHT_WHT (lossless 4x4) residuals on intra and inter units of a mixed
    frame, through the wavefront's class code."""
    fr = _frame(seed=42, inter_frac=0.4, bpc=bpc, bitdepth_max=bdmax, lossless=0.8)
    assert (fr.units["txtp"] == 16).sum() > 100
    _check(oracle, fr, mode=mode)


@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023)])
def test_mixed_frame_lead_levels(oracle, bpc, bdmax):
    """DGPU_IS_LEVEL0_BATCH on a caller's schedule: a 1080p mixed frame whose
    first levels hold >= 2048 units each, so several leading levels run as
    fused launches (units, records and per-unit aux offset to the level)
    before the persistent kernel takes the rest; bit-exact."""
    import numpy as np
    fr = _frame(seed=42, width=1920, height=1080, inter_frac=0.7, bpc=bpc, bitdepth_max=bdmax)
    sizes = np.diff(np.asarray(fr.unit_start))
    assert sizes[0] >= 2048 and sizes[1] >= 2048   # more than level 0 leads
    _check(oracle, fr, mode="lead")
