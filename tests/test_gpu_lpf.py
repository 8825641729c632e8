"""GPU parity of dav1d_gpu_loopfilter_frame_* (dav1d_loopfilter_sbrow_cols /
_rows over a frame, src/lf_apply_tmpl.c:314-466, driven as
dav1d_filter_sbrow_deblock_cols / _rows, src/recon_tmpl.c:2037-2069)
against the oracle's superblock-row walker: every pixel of the picture's
allocation, bit-exact."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _check(oracle, c, step=None):
    import torch
    import dav1d_mirror_amd.lpf as lpf
    dev = lpf.DeviceLpf(c)
    if step is None:
        dev.launch()
    else:   # one call per superblock row, in decoding order (row_start / row_end), and one past the picture
        for y in range(0, c.height + step, step):
            dev.launch(rows=(y, y + step))
    torch.cuda.synchronize()
    want = oracle.loopfilter_frame(c)
    for p, (a, b) in enumerate(zip(dev.outputs_host(), want)):
        bad = np.argwhere(a != b)
        assert len(bad) == 0, f"plane {p}: {len(bad)} pixels differ, first {bad[:5].tolist()}"
    return dev


@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023), (16, 4095)])
@pytest.mark.parametrize("layout", [0, 1, 2, 3])
@pytest.mark.parametrize("sb128", [0, 1])
def test_lpf(oracle, bpc, bdmax, layout, sb128):
    import dav1d_mirror_amd.lpf as lpf
    _check(oracle, lpf.make_lpf_case(seed=10 * layout + bpc + sb128, width=328, height=200, bpc=bpc,
                                     bitdepth_max=bdmax, layout=layout, sb128=sb128))


@pytest.mark.parametrize("seed", range(6))
def test_lpf_random_sizes(oracle, seed):
    import dav1d_mirror_amd.lpf as lpf
    rng = np.random.default_rng(seed)
    w, h = int(rng.integers(2, 80)) * 4 + int(rng.integers(0, 4)), int(rng.integers(2, 70)) * 4 + int(rng.integers(0, 4))
    _check(oracle, lpf.make_lpf_case(seed=300 + seed, width=w, height=h, bpc=8 if seed % 2 else 16,
                                     bitdepth_max=[1023, 4095][seed % 3 == 0], layout=1 + seed % 3, sb128=seed % 2,
                                     p_split=float(rng.uniform(0.2, 0.8))))


@pytest.mark.parametrize("kw", [dict(p_zero_level=1.0), dict(filter_uv=0), dict(sharp=0), dict(sharp=7),
                                dict(p_split=0.0), dict(p_split=1.0)])
def test_lpf_paths(oracle, kw):
    """No levels, luma only, sharpness extremes, all-64x64 (long filters) and all-4x4 partitions."""
    import dav1d_mirror_amd.lpf as lpf
    _check(oracle, lpf.make_lpf_case(seed=40 + len(str(kw)), width=264, height=136, **kw))


def test_lpf_1080p(oracle):
    import dav1d_mirror_amd.lpf as lpf
    _check(oracle, lpf.make_lpf_case(seed=5, width=1920, height=1080))


@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023)])
@pytest.mark.parametrize("layout", [1, 3])
@pytest.mark.parametrize("sb128", [0, 1])
def test_lpf_per_superblock_row(oracle, bpc, bdmax, layout, sb128):
    """Row ranges (round 5): one call per superblock row, in order, as
    dav1d_filter_sbrow_deblock_cols / _rows run (src/recon_tmpl.c:2037-2069),
    equal the oracle's frame walk; a range past the picture does nothing and
    a range off the 64-row grid is refused."""
    import ctypes
    import dav1d_mirror_amd.lpf as lpf
    c = lpf.make_lpf_case(seed=77 + layout + sb128, width=328, height=264, bpc=bpc, bitdepth_max=bdmax,
                          layout=layout, sb128=sb128)
    dev = _check(oracle, c, step=64 << sb128)
    with pytest.raises(RuntimeError):
        dev.launch(rows=(32, 96))
