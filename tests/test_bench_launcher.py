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
    assert r["ler"]["shots"] == 4000 and r["ler"]["failures"] == [2000, 2000, 2000]
    assert r["value"] > 0 and r["ms_per_step"] > 0
    # per-rank record: every rank seen once, its own timing and shot count
    assert r["ranks_seen"] == 2 and [x["rank"] for x in r["ranks"]] == [0, 1]
    for x in r["ranks"]:
        assert x["device"] == -1 and x["shots"] == 2 * 1000 * 3 and x["timed_s"] > 0
    assert max(x["timed_s"] for x in r["ranks"]) <= r["ms_per_step"] * r["steps"] / 1e3 * 1.001


def _run_fake(tmp_path, *extra):
    env = dict(os.environ, OMP_NUM_THREADS="2")
    env.pop("WORLD_SIZE", None)
    detail = tmp_path / "detail.json"
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--fake-device", "--batch", "512",
                          "--steps", "2", "--detail-out", str(detail)] + list(extra),
                         capture_output=True, text=True, timeout=600, env=env, cwd="/tmp")
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1
    return lines[0], detail


def test_bench_line_is_bounded_and_carries_roofline_and_cpu_baseline(tmp_path):
    """Round 5's 20 KB line was not parsed by the driver: the stdout line stays
    under LINE_MAX_BYTES and still carries the roofline and CPU-baseline blocks
    (the CPU leg is the real oracle on a small sample); the full record goes to
    the side file the line names."""
    sys.path.insert(0, REPO)
    import bench
    raw, detail = _run_fake(tmp_path, "--cpu-shots", "64")
    assert len(raw) < bench.LINE_MAX_BYTES
    r = json.loads(raw)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype", "config", "ranks_seen"):
        assert k in r
    for k in ("bound", "achieved", "peak", "frac", "traffic", "kernel", "avg_launch_ms"):
        assert k in r["roofline"]
    assert "frac" in r["roofline"]["hbm"] and "achieved" in r["roofline"]["triage"]
    assert r["cpu_baseline"]["value"] > 0 and r["cpu_baseline"]["cores"] == 2 and r["cpu_baseline"]["kind"] == "port"
    assert "ler_overlap_all" in r and len(r["ler"]["cpu_f64_failures"]) == 9
    assert r["detail"] == str(detail) and detail.exists()
    full = json.loads(detail.read_text())
    assert full["value"] == r["value"] or abs(full["value"] - r["value"]) <= 1e-5 * full["value"]
    assert len(full["ler"]) == 9 and "per_point" in full["roofline"]


def test_compact_line_bound_with_every_config_block(tmp_path):
    """The GPU run adds the C3 / C4 / C5 / reference-default blocks: fill them
    at their real sizes (and long strings) and check the bound still holds."""
    sys.path.insert(0, REPO)
    import bench
    raw, detail = _run_fake(tmp_path, "--no-cpu-baseline")
    full = json.loads(detail.read_text())
    kern = "qdec::bp_ms_cmp_kernel<double, 2, 4, 7, true, 2, 0>" + "x" * 200
    roof = {"bound": "lds", "achieved": 1.0, "peak": 2.0, "unit": "GB/s", "frac": 0.5, "traffic": 1e6,
            "algorithmic_bytes_per_launch": 1e9, "bytes_model": "y" * 1000}
    full["c3_line"] = {"lines": [{"p": p, "shots_per_s": 1e8, "ler": 1e-3, "bp_kernel": kern, "roofline": roof}
                                 for p in (0.001, 0.003, 0.01)]}
    full["c4_line"] = {"lines": [{"precision": pr, "p": p, "shots_per_s": 1e6, "bp_kernel": kern, "roofline": roof}
                                 for pr in ("f32", "f64") for p in (0.005, 0.01, 0.03)]}
    full["large_code_roofline"] = {"kernel": kern, "lines": [{"p": p, "shots_per_s": 1e5, "ler": 0.5, "roofline": roof}
                                                             for p in (0.002, 0.005)]}
    full["reference_default"] = {"shots_per_s": 1e6, "ler": 1e-3, "kernel": kern,
                                 "cpu_baseline": {"value": 1e3, "cores": 64, "osd_impl": "c", "fail_flags_identical": True}}
    full["cpu_baseline"] = {"value": 1e6, "unit": "shots/s", "cores": 64, "kind": "port", "dtype": "f64",
                            "sample": "z" * 5000}
    full["variants"] = [{"dtype": "f32", "value": 1e8, "ms_per_step": 10.0}]
    for row in full["ler"].values():
        row["cpu_f64"] = {"failures": 10 ** 6, "shots": 10 ** 7}
        row["f32"] = {"failures": 10 ** 6}
    full["ranks"] = full["ranks"] * 8
    full["roofline"]["frac"] = float("nan")  # a non-finite value never reaches the line
    full["value"] = float("inf")
    line = json.dumps(bench._finite(bench.compact_line(full, "gpurun_out/bench_detail.json")), allow_nan=False)
    assert len(line) < bench.LINE_MAX_BYTES, len(line)
    r = json.loads(line)
    assert set(r["configs"]) == {"c3", "c4_f32", "c4_f64", "c5", "reference_default"}
    assert r["roofline"]["frac"] is None and r["value"] is None
