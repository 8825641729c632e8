"""GPU parity of dav1d_gpu_prepare_intra_edges_* (device
bytefn(dav1d_prepare_intra_edges), src/ipred_prepare_tmpl.c:76-204) against
the oracle through the C ABI: the whole edge pool (entries a record's mode
does not need must stay untouched) and every unit record, bit-exact."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _check(oracle, case):
    import torch
    import dav1d_mirror_amd.intra as intra
    dev = intra.DeviceEdges(case)
    dev.launch()
    torch.cuda.synchronize()
    gu, ge = dev.results_host()
    ou, oe = oracle.prepare_intra_edges(case)
    bad = np.flatnonzero(ge != oe)
    assert len(bad) == 0, f"{len(bad)} edge pixels differ, first at {bad[:8].tolist()}"
    assert np.array_equal(gu.view(np.uint8), ou.view(np.uint8))
    return dev


@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023), (16, 4095)])
@pytest.mark.parametrize("seed", [11, 12])
def test_prepare_edges_random(oracle, bpc, bdmax, seed):
    _check(oracle, __import__("dav1d_mirror_amd.intra", fromlist=["x"]).make_edge_case(
        seed=seed, bpc=bpc, bitdepth_max=bdmax, n=3000))


@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023)])
def test_prepare_edges_128_superblocks(oracle, bpc, bdmax):
    """128-px superblocks (sb_log2 7 / 6 chroma) on a taller picture."""
    import dav1d_mirror_amd.intra as intra
    _check(oracle, intra.make_edge_case(seed=13, bpc=bpc, bitdepth_max=bdmax, n=2000, width=384,
                                        height=384, sb_log2=7))


def test_prepare_edges_small_batches(oracle):
    """1, 15, 16, 17 records: partial workgroups."""
    import dav1d_mirror_amd.intra as intra
    for n in (1, 15, 16, 17):
        _check(oracle, intra.make_edge_case(seed=20 + n, n=n))


def test_prepare_edges_large(oracle):
    """A 4K-sized picture, 60000 records."""
    import dav1d_mirror_amd.intra as intra
    _check(oracle, intra.make_edge_case(seed=14, n=60000, width=3840, height=2160))
