"""Device-visible pictures: pictures from the HBM
Dav1dPicAllocator have dav1d_default_picture_alloc's geometry
(src/picture.c:46-83), are reused from the pool once released, and the
frame tier reconstructs straight into them (here the unit batch; the
oracle checks the pixels after a copy back)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _hip():
    L = ctypes.CDLL("libamdhip64.so")
    L.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    L.hipMemcpy2D.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                              ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int]
    return L


@pytest.mark.parametrize("w,h,bpc,layout,flags", [(3840, 2160, 8, 1, 0), (1920, 1080, 10, 1, 0), (1024, 512, 8, 3, 0),
                                                  (640, 360, 8, 1, 1)])
def test_allocator_geometry_and_pool(pkg, w, h, bpc, layout, flags):
    abi, L = pkg.abi, pkg.abi.load_lib()
    a = abi.PicAllocator()
    assert L.dav1d_gpu_pic_allocator_init(ctypes.byref(a), 0, flags) == 0
    pic = abi.Picture()
    pic.p.w, pic.p.h, pic.p.layout, pic.p.bpc = w, h, layout, bpc
    assert a.alloc_picture_callback(ctypes.byref(pic), a.cookie) == 0
    hbd = bpc > 8
    ys = ((w + 127) & ~127) << hbd
    ss_hor = layout != 3
    uvs = ys >> ss_hor
    ys += 64 if not ys & 1023 else 0
    uvs += 64 if not uvs & 1023 else 0
    assert (pic.stride[0], pic.stride[1]) == (ys, uvs)
    assert all(pic.data[p] % 64 == 0 for p in range(3))
    pl = abi.Plane()
    assert L.dav1d_gpu_picture_plane(ctypes.byref(pic), 1, ctypes.byref(pl)) == 0
    assert pl.w == (w + ss_hor) >> ss_hor and pl.stride == uvs
    first = pic.data[0]
    a.release_picture_callback(ctypes.byref(pic), a.cookie)
    pic2 = abi.Picture()
    pic2.p = pic.p
    assert a.alloc_picture_callback(ctypes.byref(pic2), a.cookie) == 0
    assert pic2.data[0] == first   # reused from the pool
    assert L.dav1d_gpu_pic_allocator_close(ctypes.byref(a)) == 1   # one outstanding
    a.release_picture_callback(ctypes.byref(pic2), a.cookie)
    assert L.dav1d_gpu_pic_allocator_close(ctypes.byref(a)) == 0


@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023)])
def test_recon_into_allocator_picture(pkg, oracle, bpc, bdmax):
    import torch
    import dav1d_mirror_amd.batch as bt
    import dav1d_mirror_amd.workload as wl
    abi, L = pkg.abi, pkg.abi.load_lib()
    fd = wl.make_frame(wl.FrameConfig(width=1920, height=1080, bpc=bpc, bitdepth_max=bdmax, seed=91))
    a = abi.PicAllocator()
    assert L.dav1d_gpu_pic_allocator_init(ctypes.byref(a), 0, abi.PIC_DEVICE) == 0
    pic = abi.Picture()
    pic.p.w, pic.p.h, pic.p.layout, pic.p.bpc = 1920, 1080, 1, 8 if bpc == 8 else 10
    assert a.alloc_picture_callback(ctypes.byref(pic), a.cookie) == 0
    dev = bt.DeviceFrame(fd, "cuda:0")
    for p in range(3):
        pl = abi.Plane()
        assert L.dav1d_gpu_picture_plane(ctypes.byref(pic), p, ctypes.byref(pl)) == 0
        dev.batch.dst[p] = pl
    dev.launch()
    torch.cuda.synchronize()
    hf = oracle.HostFrame(fd)
    hf.run(threads=8)
    hip = _hip()
    bpp = 1 if bpc == 8 else 2
    for p in range(3):
        w, h = fd.plane_wh[p]
        out = np.zeros((h, w), np.uint8 if bpc == 8 else np.uint16)
        assert hip.hipMemcpy2D(out.ctypes.data, w * bpp, pic.data[p], pic.stride[1 if p else 0], w * bpp, h, 2) == 0
        assert np.array_equal(out, hf.dst[p]), f"plane {p}"
    a.release_picture_callback(ctypes.byref(pic), a.cookie)
    assert L.dav1d_gpu_pic_allocator_close(ctypes.byref(a)) == 0
