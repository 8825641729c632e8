"""bench.py --gpus N runs N ranks: without a launcher it
spawns the N rank processes itself, under a launcher its WORLD_SIZE must
agree.  The wiring is checked with --dry-run (gloo on the CPU, no GPU, no
bench number): every rank joins, the barrier and the max-over-ranks
reduction of the timed region run, and rank 0 reports world size N."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                          "MASTER_PORT")}
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=e,
                          capture_output=True, text=True, timeout=300)


def test_bench_spawns_n_ranks():
    for n in (2, 3):
        r = _run(["--gpus", str(n), "--dry-run"])
        assert r.returncode == 0, r.stdout + r.stderr
        lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
        assert len(lines) == 1, r.stdout   # rank 0 alone prints
        d = json.loads(lines[0])
        assert d["dry_run"] and d["n_gpus"] == n and d["ranks_joined"] == n and d["max_rank"] == n - 1
        # the N>1 line's per-rank fields: every rank's value in rank order and the max
        pr = d["per_rank"]
        assert pr["kernel_us"] == [10.0 + r for r in range(n)] and pr["kernel_us_max"] == 10.0 + n - 1
        assert pr["slowest_rank"] == n - 1


def test_bench_single_rank_default():
    r = _run(["--dry-run"])
    assert r.returncode == 0, r.stdout + r.stderr
    assert json.loads(r.stdout.strip().splitlines()[-1])["n_gpus"] == 1


def test_bench_world_mismatch_fails():
    """A launcher's WORLD_SIZE that disagrees with --gpus is an error, never
    a number for the wrong GPU count."""
    r = _run(["--gpus", "8", "--dry-run"], WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_wait_ranks_stops_on_first_failure():
    """a later rank dying while rank 0 still runs (e.g. in a
    rendezvous) ends the bench with that rank's status, the others stopped."""
    import time
    sys.path.insert(0, ROOT)
    import bench
    procs = [subprocess.Popen([sys.executable, "-c", "import time; time.sleep(120)"]),
             subprocess.Popen([sys.executable, "-c", "import sys; sys.exit(3)"])]
    t0 = time.time()
    assert bench.wait_ranks(procs) == 3
    assert time.time() - t0 < 30
    assert procs[0].poll() is not None
    ok = [subprocess.Popen([sys.executable, "-c", "pass"]) for _ in range(2)]
    assert bench.wait_ranks(ok) == 0
