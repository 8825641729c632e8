"""The HBM picture allocator's ABI (include/dav1d_gpu.h, Dav1dGpuPicAllocator
== Dav1dPicAllocator, include/dav1d/picture.h:107-145): the struct layouts
match dav1d's, and without a usable device an allocation fails cleanly with
-ENOMEM (as dav1d's own allocator reports exhaustion) instead of aborting."""
import ctypes
import errno


def test_picture_struct_layout(pkg):
    abi = pkg.abi
    assert ctypes.sizeof(abi.Picture) == 272
    assert abi.Picture.data.offset == 16 and abi.Picture.stride.offset == 40
    assert abi.Picture.p.offset == 56 and abi.Picture.allocator_data.offset == 264
    assert ctypes.sizeof(abi.PicAllocator) == 24


def test_allocator_lifecycle_without_device(pkg):
    L = pkg.abi.load_lib()
    if L.dav1d_gpu_device_count() > 0:
        return   # covered by tests/test_gpu_picture.py
    a = pkg.abi.PicAllocator()
    assert L.dav1d_gpu_pic_allocator_init(ctypes.byref(a), 0, pkg.abi.PIC_DEVICE) == 0
    pic = pkg.abi.Picture()
    pic.p.w, pic.p.h, pic.p.layout, pic.p.bpc = 640, 360, 1, 8
    assert a.alloc_picture_callback(ctypes.byref(pic), a.cookie) == -errno.ENOMEM
    assert not pic.allocator_data
    assert L.dav1d_gpu_pic_allocator_close(ctypes.byref(a)) == 0
    assert L.dav1d_gpu_pic_allocator_init(ctypes.byref(a), 0, 7) == -1
