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
