"""bench.py's multi-GPU launch path on CPU: `python bench.py --gpus 2` starts
torchrun with two ranks by itself (reference fan-out: misc/p_sweep.py:17-29
splits shots over Pool workers), each rank decodes its own shot range, and rank
0 merges the failure counts and reports the max-over-ranks time.  The decode is
replaced by a stand-in (--fake-device) whose failures are a known function of
the global shot index, so the merged counts are checked exactly."""
import json
import os
import subprocess
import sys

from conftest import REPO


def test_bench_gpus2_self_launches_two_ranks_and_merges():
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--fake-device",
                          "--batch", "1000", "--steps", "2", "--points", "3", "--no-cpu-baseline"],
                         capture_output=True, text=True, timeout=300, env=env, cwd="/tmp")
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), out.stdout[-2000:]  # stdout: rank 0's one JSON line only
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["steps"] == 2 and r["scaling"] == "weak"
    assert r["config"]["global_batch"] == 1000 * 3 * 2
    # shots per point: 2 steps x 1000 x 2 ranks, disjoint index ranges; the
    # stand-in fails shot s of point i iff s + i is odd: exactly half
    for row in r["ler"].values():
        assert row["shots"] == 4000
        assert row["failures"] == 2000
    assert r["value"] > 0 and r["ms_per_step"] > 0
    # per-rank record: every rank seen once, its own timing and shot count
    assert r["ranks_seen"] == 2 and [x["rank"] for x in r["ranks"]] == [0, 1]
    for x in r["ranks"]:
        assert x["device"] == -1 and x["shots"] == 2 * 1000 * 3 and x["timed_s"] > 0
    assert max(x["timed_s"] for x in r["ranks"]) <= r["ms_per_step"] * r["steps"] / 1e3 * 1.0001
