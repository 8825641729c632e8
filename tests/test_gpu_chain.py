"""The frame pipeline chained on one stream with every picture resident in
HBM (dav1d_mirror_amd.chain): reconstruction, deblocking, CDEF, loop
restoration and film grain, in dav1d_filter_sbrow's order (src/recon_tmpl.c:
2104-2160), against the oracle walkers chained the same way.  Every stage's
picture is compared, bit-exact."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("w,h,bpc,bdmax,per_row", [(1920, 1080, 8, 255, False), (3840, 2160, 8, 255, False),
                                                   (1920, 1080, 16, 1023, False), (1920, 1080, 8, 255, True),
                                                   (1920, 1080, 16, 1023, True),
                                                   (1920, 1024, 8, 255, True), (1280, 256, 8, 255, True)])
def test_chain_recon_postfilters_grain(pkg, oracle, w, h, bpc, bdmax, per_row):
    """per_row: the post-filters run per superblock row, interleaved as a
    decoder runs them (DeviceChain.launch_per_row), against the same
    whole-frame oracle chain."""
    import torch
    import dav1d_mirror_amd.chain as ch
    import dav1d_mirror_amd.workload as wl
    fd = wl.make_frame(wl.FrameConfig(width=w, height=h, bpc=bpc, bitdepth_max=bdmax, seed=81))
    cases = ch.make_cases(fd, seed=17)
    dev = ch.DeviceChain(fd, cases, "cuda:0")
    if per_row:
        dev.launch_per_row(torch.cuda.current_stream())
    else:
        dev.launch(torch.cuda.current_stream())
    torch.cuda.synchronize()
    got = [dev.stage_host(P) for P in (dev.A, dev.B, dev.C, dev.D)]
    want = ch.host_chain(fd, cases, oracle, threads=8)
    # A holds the deblocked picture after the chain; the stages after it
    for name, g, o in zip(("deblock", "cdef", "lr", "grain"), got, want[1:]):
        for p in range(3):
            diff = np.argwhere(g[p] != o[p])
            assert len(diff) == 0, f"{name} plane {p}: {len(diff)} pixels differ, first {diff[:4].tolist()}"
