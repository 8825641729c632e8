"""GPU parity of the superblock-tile batch (dav1d_gpu_recon_tiles_*) against
the oracle's tile walker (oracle_recon_tiles: the reference's DSP calls per
block, mc with recon_tmpl.c's emu_edge condition), through the C ABI.
Bit-exact bar."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _frame(**kw):
    import dav1d_mirror_amd.workload as wl
    return wl.make_frame(wl.FrameConfig(**kw))


def _check(fd, oracle, threads=4, zero_coefs=False, td=None):
    import torch
    import dav1d_mirror_amd.batch as bt
    import dav1d_mirror_amd.tiles as tl
    td = td if td is not None else tl.build_tiles(fd)
    dev = bt.DeviceTiles(fd, td, "cuda:0", zero_coefs=zero_coefs)
    dev.launch()
    torch.cuda.synchronize()
    got = dev.planes_host()
    ht = oracle.HostTiles(fd, td, zero_coefs=zero_coefs)
    ht.run(threads=threads)
    for p in range(3):
        diff = np.argwhere(got[p] != ht.dst[p])
        assert len(diff) == 0, f"plane {p}: {len(diff)} pixels differ, first {diff[:5].tolist()}"
    return dev, ht


@pytest.mark.parametrize("kind", ["full", "mc", "ipred", "itx", "ext"])
@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023), (16, 4095)])
def test_tiles_kinds(oracle, kind, bpc, bdmax):
    _check(_frame(width=512, height=256, seed=21, kind=kind, bpc=bpc, bitdepth_max=bdmax), oracle)


@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023), (16, 4095)])
def test_tiles_tx64(oracle, bpc, bdmax):
    """64-point transforms: the tiles holding them run in the second kernel."""
    fd = _frame(width=1024, height=512, seed=23, tx64=True, bpc=bpc, bitdepth_max=bdmax)
    import dav1d_mirror_amd.tiles as tl
    td = tl.build_tiles(fd)
    assert td.n_tiles_huge > 0
    _check(fd, oracle, td=td)


@pytest.mark.parametrize("kind", ["full", "ext"])
@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023)])
def test_tiles_edge_clamp(oracle, kind, bpc, bdmax):
    """MVs far past the picture (+-200 px): every clamped footprint (mc and
    warp) must equal the reference's emu_edge results."""
    fd = _frame(width=512, height=256, seed=25, kind=kind, mv_range=200, bpc=bpc, bitdepth_max=bdmax)
    _check(fd, oracle)


def test_tiles_odd_size(oracle):
    """A 1080p-like height (partial superblock row: 56-row luma / 28-row
    chroma tiles) and a width that is not a multiple of 64."""
    _check(_frame(width=480, height=248, seed=27, kind="full"), oracle)
    _check(_frame(width=480, height=248, seed=28, kind="ext", bpc=16, bitdepth_max=1023), oracle)


def test_tiles_zero_coefs(oracle):
    """The coefficient-zeroing contract (src/itx_tmpl.c:55/89) on device."""
    import torch
    fd = _frame(width=512, height=256, seed=29)
    dev, ht = _check(fd, oracle, zero_coefs=True)
    torch.cuda.synchronize()
    assert not dev.coefs.any().item()
    assert not np.any(ht.coefs)


def test_tiles_full_4k(oracle):
    """The full 4K config-3 frame through the tile batch."""
    _check(_frame(), oracle, threads=8)


def test_tiles_full_1080p_mc(oracle):
    """The 1080p config-2 frame (mc put / avg only)."""
    _check(_frame(width=1920, height=1080, kind="mc"), oracle, threads=8)


def test_tiles_idempotent(oracle):
    """Re-launching over the same inputs gives the same pixels."""
    import torch
    fd = _frame(width=512, height=256, seed=31, kind="ext")
    dev, ht = _check(fd, oracle)
    first = [p.copy() for p in dev.planes_host()]
    dev.launch()
    torch.cuda.synchronize()
    for a, b in zip(first, dev.planes_host()):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("kind,bpc,bdmax", [("full", 8, 255), ("ext", 8, 255), ("full", 16, 1023)])
def test_tiles_equal_unit_batch(oracle, kind, bpc, bdmax):
    """Both batch tiers on one frame whose MVs reach 200 px past the picture:
    the unit batch reads the edge-replicated reference padding (the caller's
    emu_edge, as dav1d's DSP functions expect), the tile batch clamps
    (recon_tmpl.c's mc() emu_edge); the pictures are identical."""
    import torch
    import dav1d_mirror_amd.batch as bt
    import dav1d_mirror_amd.tiles as tl
    fd = _frame(width=512, height=256, seed=33, kind=kind, mv_range=200, bpc=bpc, bitdepth_max=bdmax)
    du = bt.DeviceFrame(fd, "cuda:0")
    du.launch()
    dt = bt.DeviceTiles(fd, tl.build_tiles(fd), "cuda:0")
    dt.launch()
    torch.cuda.synchronize()
    for a, b in zip(du.planes_host(), dt.planes_host()):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023), (16, 4095)])
def test_tiles_lossless(oracle, bpc, bdmax):
    """WHT_WHT (lossless 4x4) transform blocks in the tile batch, full-range
    coefficients (VERDICT r4 missing #5)."""
    fd = _frame(width=512, height=256, seed=94, bpc=bpc, bitdepth_max=bdmax, lossless=0.6)
    assert (fd.units["txtp"] == 16).sum() > 100
    _check(fd, oracle)
