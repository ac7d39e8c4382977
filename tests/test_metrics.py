"""The maze-metric suite (metrics_calculator.py + the McClendon complexity, as
generation_algos_metrics_evaluations.py uses them) against the reference's own values on the
120 golden euclidean mazes (tests/golden/metrics.npz, make_golden_metrics.py).

CPU part: the oracle restatement (oracle/mzmetrics.c) and libmazerl's host McClendon
(mz_maze_complexity). GPU part: mz_maze_metrics (csrc/mz_metrics.hip) on the same mazes."""
import ctypes as C
import math

import numpy as np
import pytest

import golden_io as G
import pyoracle as O


@pytest.fixture(scope="module")
def fx():
    z = G.load("metrics.npz")
    ms = G.mazes("gen_euclid.npz")
    return [(ms[int(i)], {k: float(z[k][j]) for k in ("L", "DE", "D", "AC", "FDE", "BDE",
                                                       "difficulty", "complexity")})
            for j, i in enumerate(z["idx"])]


def test_oracle_metrics_match_reference(fx):
    for m, ref in fx:
        got = O.metrics(m["grid"], m["start"], m["goal"])
        key = (m["algo"], m["n"], m["seed"])
        for name, v in zip(("L", "DE", "D", "AC", "FDE", "BDE"), got):
            assert v == ref[name], (key, name, v, ref[name])


def test_native_complexity_matches_reference(fx):
    from mazerl import _native as N
    L = N.load()
    checked = 0
    for m, ref in fx:
        if math.isnan(ref["complexity"]):
            continue
        g = np.ascontiguousarray(m["grid"], np.uint8)
        d, c = C.c_double(), C.c_double()
        N.check(L.mz_maze_complexity(g.ctypes.data, g.shape[0], g.shape[1], *m["start"], *m["goal"],
                                     C.byref(d), C.byref(c)))
        # bit-exact: the hallway sums follow the networkx subgraph views' set order
        assert c.value == ref["complexity"], (m["n"], m["seed"])
        assert d.value == ref["difficulty"], (m["n"], m["seed"])
        checked += 1
    assert checked >= 100


@pytest.mark.gpu
def test_gpu_metrics_match_reference(fx):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import mazerl
    maxn = max(m["n"] for m, _ in fx)
    env = mazerl.VectorMazeEnv(len(fx), maxn, enrich=False, generate=False)
    for i, (m, _) in enumerate(fx):
        env.load_mazes(m["grid"][None], np.array([[*m["start"], *m["goal"]]]), env_ids=[i])
    out = env.maze_metrics().cpu().numpy()
    for i, (m, ref) in enumerate(fx):
        for k, name in enumerate(("L", "DE", "D", "AC", "FDE", "BDE")):
            assert out[i, k] == ref[name], ((m["algo"], m["n"], m["seed"]), name, out[i, k], ref[name])
    env.close()
