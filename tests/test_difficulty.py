"""Native McClendon difficulty (libmazerl mz_difficulty, host C++) vs the reference's
ComplexityEvaluation values stored in the golden fixtures (maze_complexity_evaluation.py:319-329).
CPU-only: mz_difficulty makes no HIP call. Tolerance: 1e-15 relative (the reference sums a
hallway's 1/(2d) terms in Python-set order inside networkx subgraph views; where that order differs
from insertion order the last bit can differ); at least 95% of the fixtures must match exactly."""
import math

import pytest

import golden_io as G


@pytest.fixture(scope="module")
def diff():
    from mazerl import difficulty
    from mazerl import _build
    _build.build()
    return difficulty


def test_difficulty_matches_reference(diff):
    exact = total = 0
    for name, fn in (("gen_euclid.npz", diff.maze_difficulty), ("gen_toroid.npz", diff.toroidal_difficulty)):
        for m in G.mazes(name):
            if math.isnan(m["difficulty"]):
                continue
            d = fn(m["grid"], m["start"], m["goal"])
            assert d == pytest.approx(m["difficulty"], rel=1e-15, abs=0), (name, m["algo"], m["n"], m["seed"])
            exact += d == m["difficulty"]
            total += 1
    assert total >= 200 and exact >= 0.95 * total


def test_complexity_evaluation_dropin_matches_reference(diff):
    """mazerl.lib...ComplexityEvaluation (the reference's class name and methods,
    maze_complexity_evaluation.py:38-329) on the golden euclidean mazes: difficulty_of_maze()
    == the reference's value (same tolerance as above); complexity_of_maze() is finite."""
    from mazerl.lib.maze_difficulty_evaluation.maze_complexity_evaluation import ComplexityEvaluation
    n = 0
    for m in G.mazes("gen_euclid.npz"):
        if math.isnan(m["difficulty"]):
            continue
        ce = ComplexityEvaluation(m["grid"].astype(int).tolist(), m["start"], m["goal"])
        assert ce.difficulty_of_maze() == pytest.approx(m["difficulty"], rel=1e-15, abs=0)
        assert math.isfinite(ce.complexity_of_maze())
        n += 1
    assert n >= 90  # the euclidean fixtures with a reference difficulty (N <= 41)


def test_difficulty_81x81_matches_reference(diff):
    """The headline size: the 24 reference 81x81 mazes of gen_euclid.npz against the values the
    reference's ComplexityEvaluation computed for them (tests/golden/difficulty81.npz, made by
    tests/golden/make_golden_difficulty81.py) — difficulty and complexity, same tolerance."""
    z = G.load("difficulty81.npz")
    allm = G.mazes("gen_euclid.npz")
    exact = 0
    for k, i in enumerate(z["index"]):
        m = allm[int(i)]
        assert m["n"] == 81
        d, c = diff.maze_complexity(m["grid"], m["start"], m["goal"])
        assert d == pytest.approx(float(z["difficulty"][k]), rel=1e-15, abs=0), k
        assert c == pytest.approx(float(z["complexity"][k]), rel=1e-15, abs=0), k
        exact += int(d == z["difficulty"][k]) + int(c == z["complexity"][k])
    assert len(z["index"]) == 24 and exact >= 40
