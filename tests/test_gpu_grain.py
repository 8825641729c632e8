"""GPU parity of dav1d_gpu_apply_grain_* (device bitfn(dav1d_apply_grain),
src/fg_apply_tmpl.c:222-241) against the oracle: the grain and scaling LUTs
the prep kernel builds and every output pixel.  Bit-exact bar."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _check(oracle, c):
    import torch
    import dav1d_mirror_amd.grain as grain
    dev = grain.DeviceGrain(c)
    dev.launch()
    torch.cuda.synchronize()
    outs, g, sc = oracle.apply_grain(c)
    dg, dsc = dev.luts_host()
    assert np.array_equal(dg[0], g[0]), "luma grain LUT"
    d = c.data
    for uv in range(2):
        if d.num_uv_points[uv] or d.chroma_scaling_from_luma:
            assert np.array_equal(dg[1 + uv], g[1 + uv]), f"chroma grain LUT {uv}"
    assert np.array_equal(dsc, sc), "scaling LUTs"
    for p, (a, b) in enumerate(zip(dev.outputs_host(), outs)):
        bad = np.argwhere(a != b)
        assert len(bad) == 0, f"plane {p}: {len(bad)} pixels differ, first {bad[:5].tolist()}"


@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023), (16, 4095)])
@pytest.mark.parametrize("layout", [1, 2, 3])
@pytest.mark.parametrize("lag", [0, 3])
def test_grain(oracle, bpc, bdmax, layout, lag):
    import dav1d_mirror_amd.grain as grain
    _check(oracle, grain.make_grain_case(seed=100 * layout + 10 * lag + bpc, width=160, height=96, bpc=bpc,
                                         bitdepth_max=bdmax, layout=layout, lag=lag))


@pytest.mark.parametrize("seed", range(8))
def test_grain_random(oracle, seed):
    """Random parameters (checkasm's ranges), sizes not multiples of 32."""
    import dav1d_mirror_amd.grain as grain
    rng = np.random.default_rng(seed)
    w, h = int(rng.integers(1, 12)) * 16 + 2 * int(rng.integers(0, 8)), int(rng.integers(1, 8)) * 16 + 2
    bpc = 8 if seed % 2 else 16
    _check(oracle, grain.make_grain_case(seed=500 + seed, width=w, height=h, bpc=bpc,
                                         bitdepth_max=[1023, 4095][seed % 3 == 0], layout=1 + seed % 3))


@pytest.mark.parametrize("kw", [dict(csfl=True, overlap=True), dict(num_y=0, num_uv=(0, 5), overlap=True),
                                dict(num_y=6, num_uv=(0, 0)), dict(num_y=0, num_uv=(0, 0))])
def test_grain_plane_mixes(oracle, kw):
    import dav1d_mirror_amd.grain as grain
    _check(oracle, grain.make_grain_case(seed=900 + len(kw), width=200, height=120, **kw))


def test_grain_1080p(oracle):
    import dav1d_mirror_amd.grain as grain
    _check(oracle, grain.make_grain_case(seed=7, width=1920, height=1080, overlap=True))


def test_grain_4k_10bit(oracle):
    import dav1d_mirror_amd.grain as grain
    _check(oracle, grain.make_grain_case(seed=8, width=3840, height=2160, bpc=16, bitdepth_max=1023,
                                         overlap=True))
