"""The two-pass form of a frame (workload.split_frame):
prediction blocks first (mc() once per block and reference,
src/recon_tmpl.c:957-1060), then every transform block's residual added to
the predicted picture (inv_txfm_add's dst read + clip, src/itx_tmpl.c:
40-100).  On the CPU the oracle runs both passes one after the other on one
picture and must give the fused walk's picture exactly."""
import dataclasses

import numpy as np
import pytest


@pytest.mark.parametrize("w,h,bpc,bdmax,seed", [(256, 128, 8, 255, 3), (320, 192, 16, 1023, 5),
                                                 (384, 256, 16, 4095, 8), (640, 384, 8, 255, 11)])
def test_split_frame_equals_fused(pkg, oracle, w, h, bpc, bdmax, seed):
    import dav1d_mirror_amd.workload as wl
    import dav1d_mirror_amd.abi as abi
    fd = wl.make_frame(wl.FrameConfig(width=w, height=h, bpc=bpc, bitdepth_max=bdmax, seed=seed))
    pf, rf = wl.split_frame(fd)
    # every inter transform unit's residual is in the residual pass, as PRED_NONE
    assert (pf.units["txtp"] == abi.NO_RESIDUAL).all()
    assert not np.isin(rf.units["pred"], abi.INTER_KINDS).any()
    n_inter = int(np.isin(fd.units["pred"], abi.INTER_KINDS).sum())
    assert int((rf.units["pred"] == abi.PRED_NONE).sum()) == n_inter
    assert rf.n_units == fd.n_units
    # prediction pieces tile the inter area exactly once
    px = lambda f, m: int(sum(abi.TX_WH[t][0] * abi.TX_WH[t][1] for t in f.units["tx"][m]))  # noqa: E731
    assert px(pf, slice(None)) == px(fd, np.isin(fd.units["pred"], abi.INTER_KINDS))
    # class ranges are consistent with the sort
    for f in (pf, rf):
        for c in range(abi.N_TX):
            assert (f.units["tx"][f.class_start[c]:f.class_start[c + 1]] == c).all()
    want = oracle.HostFrame(fd)
    want.run()
    a = oracle.HostFrame(pf)
    a.run()
    b = oracle.HostFrame(dataclasses.replace(rf, dst_init=[p.copy() for p in a.dst]))
    b.run()
    for p in range(3):
        assert np.array_equal(b.dst[p], want.dst[p]), f"plane {p}"


def test_split_frame_refuses_block_data_kinds(pkg):
    import dav1d_mirror_amd.workload as wl
    fd = wl.make_frame(wl.FrameConfig(width=256, height=128, kind="ext"))
    with pytest.raises(ValueError):
        wl.split_frame(fd)
