"""CPU checks of the super-res restatement: the oracle's
walk of bytefn(dav1d_filter_sbrow_resize) (src/recon_tmpl.c:2104-2137),
superblock row by superblock row with its 8-row lag, against a second,
numpy restatement of resize_c (src/mc_tmpl.c:877-903) applied to every row
at once -- so the walk's row ranges tile each plane exactly, which is what
lets the device run the whole frame in one launch.  Also dav1d's super-res
parameters (src/decode.c:3365-3369, 3517-3518, 3575-3583)."""
import numpy as np
import pytest


@pytest.mark.parametrize("layout", [0, 1, 2, 3])
@pytest.mark.parametrize("sb128", [0, 1])
@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023), (16, 4095)])
def test_walk_equals_rows(oracle, layout, sb128, bpc, bdmax):
    import dav1d_mirror_amd.superres as sr
    for i, (W, H, d) in enumerate([(256, 200, 16), (333, 131, 9), (130, 70, 13), (64, 16, 11), (520, 300, 15)]):
        c = sr.make_case(W, H, d, layout=layout, bpc=bpc, bitdepth_max=bdmax, sb128=sb128, seed=i + 7 * layout)
        for p, (a, b) in enumerate(zip(oracle.resize_frame(c), sr.restate_rows(c))):
            assert np.array_equal(a, b), (W, H, d, p)


def test_parameters():
    """Known answers: a 2x super-res frame steps half a pixel (8192 in Q14);
    a coded width equal to the upscaled one steps exactly one; coded widths
    follow (W * 8 + d / 2) / d with a floor of min(W, 16); starts are 14-bit."""
    import dav1d_mirror_amd.superres as sr
    assert sr.coded_width(3840, 16) == 1920 and sr.coded_width(3840, 9) == 3413
    assert sr.coded_width(20, 16) == 16 and sr.coded_width(8, 16) == 8
    assert sr.scale_fac(1920, 3840) == 8192 and sr.scale_fac(3840, 3840) == 16384
    for W in (64, 333, 1920, 3840):
        for d in range(9, 17):
            w = sr.coded_width(W, d)
            st = sr.scale_fac(w, W)
            x0 = sr.upscale_x0(w, W, st)
            assert 0 <= x0 < 1 << 14
            # the last output's source position stays within one pixel of the coded width
            assert ((x0 + (W - 1) * st) >> 14) <= w


def test_superres_rejects(pkg):
    """Validation before any device call (no GPU needed)."""
    import ctypes
    import dav1d_mirror_amd.abi as abi
    L = abi.load_lib()
    assert L.dav1d_gpu_resize_frame_8bpc(None, None) == -1
    f = abi.ResizeFrame()
    f.layout = 5
    assert L.dav1d_gpu_resize_frame_8bpc(ctypes.byref(f), None) == -1
    f.layout = 1   # planes missing
    assert L.dav1d_gpu_resize_frame_16bpc(ctypes.byref(f), None) == -1
