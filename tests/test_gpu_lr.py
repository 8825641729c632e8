"""GPU parity of dav1d_gpu_lr_frame_* (bytefn(dav1d_lr_sbrow) over a frame,
src/lr_apply_tmpl.c:99-202) against the oracle's walker: every pixel,
bit-exact."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _check(oracle, c, step=None, exact=False):
    import torch
    import dav1d_mirror_amd.lr as lr
    dev = lr.DeviceLr(c)
    if step is None:
        dev.launch()
    elif exact:   # sby = 0 .. sbh - 1 only, in decoding order, as dav1d_filter_sbrow_lr calls it
        for y in range(0, (c.height + step - 1) // step * step, step):
            dev.launch(rows=(y, y + step))
    else:   # one call per superblock row, last row first (in, lpf read-only), and one past the picture
        for y in reversed(range(0, c.height + step, step)):
            dev.launch(rows=(y, y + step))
    torch.cuda.synchronize()
    want = oracle.lr_frame(c)
    for p, (a, b) in enumerate(zip(dev.outputs_host(), want)):
        bad = np.argwhere(a != b)
        assert len(bad) == 0, f"plane {p}: {len(bad)} pixels differ, first {bad[:5].tolist()}"


@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023), (16, 4095)])
@pytest.mark.parametrize("layout", [0, 1, 2, 3])
@pytest.mark.parametrize("sb128", [0, 1])
def test_lr(oracle, bpc, bdmax, layout, sb128):
    import dav1d_mirror_amd.lr as lr
    _check(oracle, lr.make_lr_case(seed=20 * layout + bpc + sb128, width=336, height=250, bpc=bpc,
                                   bitdepth_max=bdmax, layout=layout, sb128=sb128,
                                   unit_log2=(6 + sb128, 5 + sb128 if layout == 1 else 6 + sb128)))


@pytest.mark.parametrize("seed", range(6))
def test_lr_random(oracle, seed):
    """Random sizes, unit sizes 32..256, plane mixes."""
    import dav1d_mirror_amd.lr as lr
    rng = np.random.default_rng(seed)
    w, h = int(rng.integers(40, 500)), int(rng.integers(30, 300))
    _check(oracle, lr.make_lr_case(seed=60 + seed, width=w, height=h, bpc=8 if seed % 2 else 16,
                                   bitdepth_max=[1023, 4095][seed % 3 == 0], layout=1 + seed % 3, sb128=seed % 2,
                                   restore_planes=int(rng.integers(1, 8))))


def test_lr_1080p(oracle):
    import dav1d_mirror_amd.lr as lr
    _check(oracle, lr.make_lr_case(seed=9, width=1920, height=1080, unit_log2=(6, 5)))


@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023)])
@pytest.mark.parametrize("layout", [1, 3])
@pytest.mark.parametrize("sb128", [0, 1])
def test_lr_per_superblock_row(oracle, bpc, bdmax, layout, sb128):
    """Row ranges (round 5): one call per superblock row, the stripes
    dav1d_lr_sbrow filters for it (src/lr_apply_tmpl.c:169-202), in reverse
    order, equal the oracle's frame walk."""
    import dav1d_mirror_amd.lr as lr
    c = lr.make_lr_case(seed=120 + layout + sb128 + bpc, width=336, height=264, bpc=bpc, bitdepth_max=bdmax,
                        layout=layout, sb128=sb128, unit_log2=(6 + sb128, 5 + sb128 if layout == 1 else 6 + sb128))
    _check(oracle, c, step=64 << sb128)


@pytest.mark.parametrize("height", [256, 1024, 250, 1080])
@pytest.mark.parametrize("sb128", [0, 1])
@pytest.mark.parametrize("layout", [1, 3])
def test_lr_per_row_last_stripe(oracle, height, sb128, layout):
    """the call for the last superblock row filters down to
    the picture's bottom (dav1d_lr_sbrow: not_last = 0, row_h = h,
    src/lr_apply_tmpl.c:174-191), also when h % 64 is 0 or 57..63 and the
    last stripe starts 8 rows above a 64-row multiple.  Only sby = 0 ..
    sbh - 1 are called, no range past the picture."""
    import dav1d_mirror_amd.lr as lr
    c = lr.make_lr_case(seed=300 + height + sb128 + layout, width=200, height=height, bpc=8, layout=layout,
                        sb128=sb128, unit_log2=(6 + sb128, 5 + sb128 if layout == 1 else 6 + sb128))
    _check(oracle, c, step=64 << sb128, exact=True)
