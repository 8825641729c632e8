#!/usr/bin/env python3
"""Generate tests/golden/recon_golden.npz from the CPU oracle.

The reference (dav1d C) cannot be built in this image (its sources need the
meson-generated config.h) and ships no known-answer vectors for the DSP, so
these fixtures pin the oracle against regressions only ("parity unpinned"
vs the reference binary).  Inputs are regenerated from the
seeded workload generator; the fixture holds the sha256 of every output
plane plus the full planes of the smallest batch.
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

CASES = [
    ("full8_s1", dict(width=128, height=64, seed=1)),
    ("full8_s2", dict(width=256, height=128, seed=2)),
    ("mc8", dict(width=256, height=128, kind="mc", seed=3, mc_split=64)),
    ("full10", dict(width=128, height=64, bpc=16, bitdepth_max=1023, seed=4)),
    ("full12", dict(width=128, height=64, bpc=16, bitdepth_max=4095, seed=5)),
    ("full8_tx64", dict(width=256, height=128, seed=6, tx64=True)),
    ("ext8", dict(width=256, height=128, seed=7, kind="ext")),
    ("ext12", dict(width=256, height=128, seed=8, kind="ext", bpc=16, bitdepth_max=4095)),
    # MVs far past the picture on edge-replicated references: the unit walker
    # reads the replicated padding, the tile walker clamps (emu_edge)
    ("edge8", dict(width=256, height=128, seed=9, kind="ext", mv_range=200)),
]


def run_case(kw):
    ge.load_package()
    import dav1d_mirror_amd.workload as wl
    orc = ge.load_oracle()
    fd = wl.make_frame(wl.FrameConfig(**kw))
    hf = orc.HostFrame(fd)
    hf.run()
    return fd, hf.dst


def main():
    out = {}
    for name, kw in CASES:
        fd, planes = run_case(kw)
        for p, a in enumerate(planes):
            out[f"{name}_p{p}_sha256"] = np.frombuffer(hashlib.sha256(a.tobytes()).digest(), np.uint8)
            if name == "full8_s1":
                out[f"{name}_p{p}"] = a
        out[f"{name}_units"] = np.array([fd.n_units])
    path = os.path.join(ROOT, "tests", "golden", "recon_golden.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, len(out), "arrays")


if __name__ == "__main__":
    main()
