"""The per-call tier's error contract: a HIP failure inside a
table entry must not abort the decoder and must not write part of the
entry's outputs; it latches a sticky error the caller reads at a flush point
(the reference latches task errors the same way, src/thread_task.c:453 and
src/lib.c:715) and, when the *_gpu_* hook replaced a caller's entries, the
failed call runs the caller's previous (C default) entry instead.

The checks run in a child process (the latch is process-wide).  Without a
GPU the failure is the missing device; with one, DAV1D_GPU_FAIL_AFTER=0
fails the tier's first HIP call.  Either way no kernel runs.
"""
import os
import subprocess
import sys
import textwrap

import pytest

CHILD = textwrap.dedent(r"""
    import ctypes, os, sys
    sys.path.insert(0, os.environ["DGPU_ROOT"])
    import __graft_entry__ as ge
    L = ge.load_package().abi.load_lib()
    L.dav1d_gpu_get_error.restype = ctypes.c_int
    L.dav1d_gpu_clear_error.restype = ctypes.c_int
    VP = ctypes.c_void_p
    McTab = VP * 53        # Dav1dMCDSPContext: 4 x 10 + avg, w_avg, mask, w_mask[3], blend x3, warp x2, emu_edge, resize
    ItxTab = VP * (19 * 17)
    PUT8 = ctypes.CFUNCTYPE(None, VP, ctypes.c_ssize_t, VP, ctypes.c_ssize_t, ctypes.c_int, ctypes.c_int,
                            ctypes.c_int, ctypes.c_int)
    ITX8 = ctypes.CFUNCTYPE(None, VP, ctypes.c_ssize_t, VP, ctypes.c_int)
    assert L.dav1d_gpu_get_error() == 0

    # 1. whole-table replacement: no fallback exists, the outputs stay untouched
    t = McTab()
    L.dav1d_mc_dsp_init_8bpc(ctypes.byref(t))
    put = PUT8(t[0])
    src = (ctypes.c_uint8 * (64 * 64))(*[(i * 37) & 255 for i in range(64 * 64)])
    dst = (ctypes.c_uint8 * (32 * 16))(*([0xAB] * (32 * 16)))
    put(ctypes.addressof(dst), 32, ctypes.addressof(src) + 16 * 64 + 16, 64, 8, 8, 3, 5)
    assert all(v == 0xAB for v in dst), "partial write after a failed call"
    err = L.dav1d_gpu_get_error()
    assert err != 0, "no sticky error latched"
    it = ItxTab()
    L.dav1d_itx_dsp_init_8bpc(ctypes.byref(it), 8)
    coef = (ctypes.c_int16 * 16)(*range(1, 17))
    pix = (ctypes.c_uint8 * 64)(*([7] * 64))
    ITX8(it[0])(ctypes.addressof(pix), 16, ctypes.addressof(coef), 15)
    assert list(coef) == list(range(1, 17)) and all(v == 7 for v in pix), "itx wrote after a failure"
    assert L.dav1d_gpu_get_error() == err, "the first error must stay latched"
    assert L.dav1d_gpu_clear_error() == err and L.dav1d_gpu_get_error() == 0

    # 2. the _gpu_ hook over a caller's table: the failed call runs the
    #    caller's previous entry (a second hook call must not replace it)
    calls = []
    def c_put(d, ds, s, ss, w, h, mx, my):
        calls.append((w, h, mx, my))
        for y in range(h):
            ctypes.memset(d + y * ds, 0x11, w)
    cb = PUT8(c_put)
    t2 = McTab()
    t2[0] = ctypes.cast(cb, VP).value
    L.dav1d_mc_dsp_init_gpu_8bpc(ctypes.byref(t2))
    L.dav1d_mc_dsp_init_gpu_8bpc(ctypes.byref(t2))
    assert t2[0] != ctypes.cast(cb, VP).value, "hook did not install the GPU entry"
    dst2 = (ctypes.c_uint8 * (32 * 16))(*([0xAB] * (32 * 16)))
    PUT8(t2[0])(ctypes.addressof(dst2), 32, ctypes.addressof(src) + 16 * 64 + 16, 64, 8, 8, 3, 5)
    assert calls == [(8, 8, 3, 5)], calls
    assert all(dst2[y * 32 + x] == 0x11 for y in range(8) for x in range(8))
    assert all(dst2[y * 32 + x] == 0xAB for y in range(8, 16) for x in range(32))
    assert L.dav1d_gpu_get_error() != 0
    # latched: the next call goes straight to the fallback, no GPU attempt
    PUT8(t2[0])(ctypes.addressof(dst2), 32, ctypes.addressof(src), 64, 4, 2, 0, 0)
    assert calls[-1] == (4, 2, 0, 0)
    print("ERRORS-OK", err)
""")


def test_per_call_error_contract():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, DGPU_ROOT=root, DAV1D_GPU_FAIL_AFTER="0")
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, f"child failed (rc {r.returncode}):\n{r.stdout}\n{r.stderr}"
    assert "ERRORS-OK" in r.stdout
    assert "failed (error" in r.stderr   # the readable message of the latch
