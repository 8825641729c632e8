"""GPU parity of dav1d_gpu_cdef_frame_* (bytefn(dav1d_cdef_brow) over a
frame, src/cdef_apply_tmpl.c:97-309, driven as dav1d_filter_sbrow_cdef,
src/recon_tmpl.c:2076-2102) against the oracle's walker: every pixel of the
frame's 8x8 grid, bit-exact."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _check(oracle, c, sb128=0, step=None):
    import torch
    import dav1d_mirror_amd.cdef as cdef
    dev = cdef.DeviceCdef(c)
    if step is None:
        dev.launch()
    else:   # one call per superblock row, last row first (the input is read-only), and one past the picture
        for y in reversed(range(0, c.height + step, step)):
            dev.launch(rows=(y, y + step))
    torch.cuda.synchronize()
    want = oracle.cdef_frame(c, sb128)
    for p, (a, b) in enumerate(zip(dev.outputs_host(), want)):
        bad = np.argwhere(a != b)
        assert len(bad) == 0, f"plane {p}: {len(bad)} pixels differ, first {bad[:5].tolist()}"
    return dev


@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023), (16, 4095)])
@pytest.mark.parametrize("layout", [0, 1, 2, 3])
def test_cdef(oracle, bpc, bdmax, layout):
    import dav1d_mirror_amd.cdef as cdef
    _check(oracle, cdef.make_cdef_case(seed=10 * layout + bpc, width=320, height=192, bpc=bpc, bitdepth_max=bdmax,
                                       layout=layout))


@pytest.mark.parametrize("seed", range(8))
def test_cdef_random_sizes(oracle, seed):
    """Sizes that are not multiples of 8 or 64 (odd 4x4 grids), random damping / strengths."""
    import dav1d_mirror_amd.cdef as cdef
    rng = np.random.default_rng(seed)
    w, h = int(rng.integers(1, 40)) * 4 + 4 * int(rng.integers(0, 2)), int(rng.integers(1, 30)) * 4
    bpc = 8 if seed % 2 else 16
    _check(oracle, cdef.make_cdef_case(seed=700 + seed, width=w, height=h, bpc=bpc,
                                       bitdepth_max=[1023, 4095][seed % 3 == 0], layout=1 + seed % 3),
           sb128=seed % 2)


@pytest.mark.parametrize("kw", [dict(p_skip_sb=1.0), dict(p_noskip=0.0), dict(p_skip_sb=0.0, p_noskip=1.0),
                                dict(strengths=([0] * 8, [63] * 8)), dict(strengths=([63] * 8, [0] * 8)),
                                dict(strengths=([3] * 8, [60] * 8)), dict(damping=3), dict(damping=6)])
def test_cdef_paths(oracle, kw):
    """Whole-frame skip, no coded blocks, everything filtered, chroma- / luma-only,
    secondary- / primary-only strengths, damping extremes."""
    import dav1d_mirror_amd.cdef as cdef
    _check(oracle, cdef.make_cdef_case(seed=900 + len(str(kw)), width=256, height=136, **kw))


def test_cdef_relaunch_idempotent(oracle):
    import torch
    import dav1d_mirror_amd.cdef as cdef
    dev = _check(oracle, cdef.make_cdef_case(seed=31, width=200, height=100))
    first = dev.outputs_host()
    dev.launch()
    torch.cuda.synchronize()
    for a, b in zip(first, dev.outputs_host()):
        assert np.array_equal(a, b)


def test_cdef_1080p(oracle):
    import dav1d_mirror_amd.cdef as cdef
    _check(oracle, cdef.make_cdef_case(seed=7, width=1920, height=1080))


def test_cdef_4k_10bit(oracle):
    import dav1d_mirror_amd.cdef as cdef
    _check(oracle, cdef.make_cdef_case(seed=8, width=3840, height=2160, bpc=16, bitdepth_max=1023))


@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023)])
@pytest.mark.parametrize("layout", [1, 2])
@pytest.mark.parametrize("sb128", [0, 1])
def test_cdef_per_superblock_row(oracle, bpc, bdmax, layout, sb128):
    """Row ranges (round 5): one call per superblock row (dav1d_cdef_brow
    per row), in reverse order, equal the oracle's frame walk."""
    import dav1d_mirror_amd.cdef as cdef
    c = cdef.make_cdef_case(seed=90 + layout + bpc, width=328, height=264, bpc=bpc, bitdepth_max=bdmax,
                            layout=layout)
    dev = _check(oracle, c, sb128=sb128, step=64 << sb128)
    with pytest.raises(RuntimeError):
        dev.launch(rows=(64, 64))
