"""The recorder's flush steps (the cut per block, the level pass, the sort,
the scatter; csrc/rec_cut.hpp, csrc/recorder.hip) give the upload image and
schedule of tools/rec_dump.py's seven frames byte for byte as the round-6
host implementation did (tests/golden/rec_dump_md5.json, recorded from its
host-only dumps before the cut moved to the device): 4K / 1080p mixed
frames, 2x2 tiles, all-CfL, overhanging blocks, 128-px superblocks, 10 / 12
bit, every launch-ahead kind, and top_edge with its backup runs.  Host-only
flushes (DAV1D_GPU_REC_HOSTONLY: the same step functions run serially on
the host), no device; tests/test_gpu_recorder.py checks the device's."""
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_flush_image_golden(pkg, tmp_path):
    want = json.load(open(os.path.join(ROOT, "tests", "golden", "rec_dump_md5.json")))["frames"]
    env = dict(os.environ)
    env.pop("DAV1D_GPU_REC_HOSTONLY", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rec_dump.py"), str(tmp_path / "d.bin")],
                       env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-2000:]
    got = {m.group(1): (int(m.group(3)), m.group(4)) for m in
           re.finditer(r"frame (\d+) rc (\S+) units (\d+) .* md5 (\w+)", r.stdout)}
    assert set(got) == set(want), r.stdout
    for k, w in want.items():
        assert got[k] == (w["units"], w["md5"]), (k, got[k], w)
