"""bench.py's output contract on the GPU: one JSON line on stdout with the driver's fields, the
roofline object (bound, achieved, peak, unit, frac, traffic) of the dominant kernel and the
cpu_baseline object (value, unit, cores, kind, sample), at small sizes (a few seconds). The full
default run is the driver's; this guards the shape of the line and its arithmetic."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def test_bench_line_has_the_contract_fields():
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--envs", "4096", "--steps", "40",
           "--warmup", "4", "--graph-chunk", "20", "--train-steps", "120", "--eval-mazes", "32",
           "--curriculum-steps", "0", "--config-legs", "", "--cpu-seconds", "1"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout[-2000:]  # ONE JSON line, nothing else on stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 40 and d["warmup"] == 4
    assert d["higher_is_better"] is True and d["scaling"] == "weak" and d["vs_baseline"] is None
    assert "workload" in d["config"]
    assert d["value"] > 0 and d["value"] == pytest.approx(4096 * 1e3 / d["ms_per_step"], rel=1e-6)
    r = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], rel=1e-9)
    # achieved = algorithmic bytes per launch / the launch's average duration
    assert r["achieved"] == pytest.approx(r["alg_bytes_per_instance_step"] * 4096
                                          / (r["avg_kernel_ms"] * 1e-3) / 1e9, rel=1e-6)
    assert 0.0 < r["frac"] < 1.0
    c = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in c, k
    assert c["kind"] in ("port", "reference") and c["value"] > 0 and c["cores"] >= 1
    w = d["win_rate"]
    assert 0.0 <= w["greedy"] <= 1.0 and w["train_vector_steps"] >= 120


def test_bench_self_launched_two_ranks_rehearsal():
    """`bench.py --gpus 2` starts its own 2 ranks (no torchrun); on a one-GPU box both share the
    card over gloo (MZ_DIST_BACKEND=gloo): rank 0's line reports both ranks and the whole-job
    value (the sum over ranks of instances x steps / the max-over-ranks wall time)."""
    env = dict(os.environ, MZ_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--envs", "2048",
           "--steps", "20", "--warmup", "2", "--graph-chunk", "10", "--train-steps", "60",
           "--eval-mazes", "16", "--curriculum-steps", "0", "--config-legs", "",
           "--launch-timeout", "400"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks_seen"] == 2 and d["backend"] == "gloo"
    assert d["launch"].startswith("bench.py --gpus N")
    assert d["value"] == pytest.approx(2 * 2048 * 1e3 / d["ms_per_step"], rel=1e-6)
    assert "cpu_baseline" not in d  # rank 0 at N = 1 only
    assert d["win_rate"]["ranks"] == 2
