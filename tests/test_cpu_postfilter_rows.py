"""The superblock-row ranges of the post-filter frame entries (round 5,
include/dav1d_gpu.h: row_start / row_end of Dav1dGpuLoopFilterFrame,
Dav1dGpuCdefFrame and Dav1dGpuLrFrame) are validated on the host before
anything is launched: a range off the 64-row grid, negative, or empty
returns -1.  No device is touched (fake plane addresses); the per-row
results themselves are GPU tests (test_gpu_{lpf,cdef,lr}.py::*per_superblock_row,
test_gpu_chain.py)."""
import ctypes

import pytest

BAD = [(32, 96), (0, 32), (-64, 64), (128, 64), (64, 64), (0, 100)]
FAKE = 0x10000


def _call(lib, name, frame):
    return getattr(lib, name)(ctypes.byref(frame), None)


@pytest.mark.parametrize("rows", BAD)
def test_lpf_rows_refused(pkg, rows):
    import dav1d_mirror_amd.lpf as lpf
    c = lpf.make_lpf_case(seed=1, width=256, height=192)
    f = lpf.fill_frame(pkg.abi.LoopFilterFrame(), c, [(FAKE, w) for (w, h) in (c.plane_wh(p) for p in range(3))],
                       FAKE, FAKE)
    f.row_start, f.row_end = rows
    assert _call(pkg.abi.load_lib(), "dav1d_gpu_loopfilter_frame_8bpc", f) == -1


@pytest.mark.parametrize("rows", BAD)
def test_cdef_rows_refused(pkg, rows):
    import dav1d_mirror_amd.cdef as cdef
    c = cdef.make_cdef_case(seed=1, width=256, height=192)
    planes = [(FAKE, (w + 15) // 16 * 16) for (w, h) in (c.plane_wh(p) for p in range(3))]
    f = cdef.fill_frame(pkg.abi.CdefFrame(), c, planes, [(FAKE * 2, s) for _, s in planes], FAKE, FAKE)
    f.row_start, f.row_end = rows
    assert _call(pkg.abi.load_lib(), "dav1d_gpu_cdef_frame_8bpc", f) == -1


@pytest.mark.parametrize("rows", BAD)
def test_lr_rows_refused(pkg, rows):
    import dav1d_mirror_amd.lr as lr
    c = lr.make_lr_case(seed=1, width=256, height=192, unit_log2=(6, 5))
    planes = [(FAKE, w) for (w, h) in (c.plane_wh(p) for p in range(3))]
    f = lr.fill_frame(pkg.abi.LrFrame(), c, planes, [(FAKE * 2, s) for _, s in planes],
                      [(FAKE * 3, s) for _, s in planes], [FAKE] * 3)
    f.row_start, f.row_end = rows
    assert _call(pkg.abi.load_lib(), "dav1d_gpu_lr_frame_8bpc", f) == -1


def test_rows_past_the_picture_launch_nothing(pkg):
    """A well-formed range below the picture is a no-op (0, nothing launched)
    for CDEF and LR -- which also shows the -1 above comes from the range
    check, the frames being otherwise valid."""
    import dav1d_mirror_amd.cdef as cdef
    import dav1d_mirror_amd.lr as lr
    lib = pkg.abi.load_lib()
    c = cdef.make_cdef_case(seed=1, width=256, height=192)
    planes = [(FAKE, (w + 15) // 16 * 16) for (w, h) in (c.plane_wh(p) for p in range(3))]
    f = cdef.fill_frame(pkg.abi.CdefFrame(), c, planes, [(FAKE * 2, s) for _, s in planes], FAKE, FAKE)
    f.row_start, f.row_end = 256, 320
    assert _call(lib, "dav1d_gpu_cdef_frame_8bpc", f) == 0
    c = lr.make_lr_case(seed=1, width=256, height=192, unit_log2=(6, 5))
    planes = [(FAKE, w) for (w, h) in (c.plane_wh(p) for p in range(3))]
    f = lr.fill_frame(pkg.abi.LrFrame(), c, planes, [(FAKE * 2, s) for _, s in planes],
                      [(FAKE * 3, s) for _, s in planes], [FAKE] * 3)
    f.row_start, f.row_end = 320, 384
    assert _call(lib, "dav1d_gpu_lr_frame_8bpc", f) == 0
