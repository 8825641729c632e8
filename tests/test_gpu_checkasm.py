"""The checkasm-style harness (tests/checkasm_gpu.c): every per-call DSP
table entry (mc/mct/scaled/avg/w_avg/mask/w_mask/blend*/warp/emu_edge/resize,
14 intra modes + cfl + pal, 156 itx entries, cdef dir + fb[3], loop_filter_sb[2][2],
wiener[2] + sgr[3]) at 8 and 16 bpc, byte-exact
against the oracle with 8-px guard bands and coefficient-zeroing checks."""
import os
import re
import subprocess

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("test", ["mc", "ipred", "itx", "cdef", "lpf", "lr"])
def test_checkasm(test):
    exe = os.path.join(HERE, "checkasm_gpu")
    assert os.path.exists(exe), "build with __graft_entry__.build()"
    r = subprocess.run([exe, f"--test={test}", "--seed=1", "--quick"], capture_output=True, text=True,
                       timeout=900)
    print(r.stdout[-4000:])
    m = re.search(r"TOTAL fail=(\d+)", r.stdout)
    assert m and int(m.group(1)) == 0 and r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
