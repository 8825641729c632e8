"""The recorder's flush on its worker pool (cells cut per run of blocks, the
level pass split into parallel stamping / producer lookup and a sequential
walk, the sort's key, rank and boundary passes, the fill) gives the same
upload image and schedule, byte for byte, with 1 and with 8 workers
(host-only flushes dumped by tools/rec_dump.py; a 1080p mixed frame with
overhanging blocks and 128-px superblocks, ~60 k cells, above the size at
which the passes go parallel)."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _dump(tmp_path, threads):
    env = dict(os.environ, DAV1D_GPU_REC_THREADS=str(threads))
    out = str(tmp_path / f"dump{threads}.bin")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rec_dump.py"), out, "--only", "4"],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    m = re.search(r"rc (\S+) units (\d+) .* md5 (\w+)", r.stdout)
    assert m and m.group(1) == "0", r.stdout
    return int(m.group(2)), m.group(3)


def test_flush_threads_byte_identical(pkg, tmp_path):
    n1, h1 = _dump(tmp_path, 1)
    n8, h8 = _dump(tmp_path, 8)
    assert n1 == n8 and n1 > 32768
    assert h1 == h8
