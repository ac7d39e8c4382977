"""Native McClendon difficulty (libmazerl mz_difficulty, host C++) vs the reference's
ComplexityEvaluation values stored in the golden fixtures (maze_complexity_evaluation.py:319-329),
bit for bit: the reference sums each hallway's 1/(2d) terms in the order networkx 3.4's subgraph
view iterates a CPython 3.10 set (:217-218, 283-295), which the host restatement rebuilds (PySetEm
in csrc/mz_difficulty.hip); oracle/mcclendon.py restates the same in Python (oracle/pyset.py,
checked here against the interpreter's own sets). CPU-only: mz_difficulty makes no HIP call."""
import math
import os
import random
import sys

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
            assert d == m["difficulty"], (name, m["algo"], m["n"], m["seed"])
            total += 1
    assert total >= 200


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
        assert ce.difficulty_of_maze() == m["difficulty"]
        assert math.isfinite(ce.complexity_of_maze())
        n += 1
    assert n >= 90  # the euclidean fixtures with a reference difficulty (N <= 41)


def test_difficulty_81x81_matches_reference(diff):
    """The headline size: the 24 reference 81x81 mazes of gen_euclid.npz against the values the
    reference's ComplexityEvaluation computed for them (tests/golden/difficulty81.npz, made by
    tests/golden/make_golden_difficulty81.py) — difficulty and complexity, same tolerance."""
    z = G.load("difficulty81.npz")
    allm = G.mazes("gen_euclid.npz")
    for k, i in enumerate(z["index"]):
        m = allm[int(i)]
        assert m["n"] == 81
        d, c = diff.maze_complexity(m["grid"], m["start"], m["goal"])
        assert d == z["difficulty"][k] and c == z["complexity"][k], k
    assert len(z["index"]) == 24


def _mcclendon_fixture():
    z = G.load("mcclendon.npz")
    for i in range(len(z["n"])):
        n = int(z["n"][i])
        yield (z["grid"][i, :n, :n], tuple(int(x) for x in z["start"][i]),
               tuple(int(x) for x in z["goal"][i]), float(z["difficulty"][i]),
               float(z["complexity"][i]), int(z["toroidal"][i]))


def test_difficulty_set_order_fixture_matches_reference(diff):
    """tests/golden/mcclendon.npz (make_golden_mcclendon.py): 228 more reference mazes, euclidean
    9..61 and re-bordered toroidal 9..41, 3 algorithms — difficulty and complexity bit for bit."""
    n = 0
    for grid, s, t, d0, c0, _ in _mcclendon_fixture():
        if math.isnan(d0):
            continue
        d, c = diff.maze_complexity(grid, s, t)
        assert d == d0 and c == c0, (grid.shape, s, t)
        n += 1
    assert n >= 220


ORACLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")


def test_pyset_emulation_matches_the_interpreter():
    """oracle/pyset.py == CPython's own set iteration order for the operations the reference's
    hallway views go through: add() sequences with growth, set(s), s.union(t), set(generator)."""
    sys.path.insert(0, ORACLE)
    from pyset import PySet
    rng = random.Random(7)
    for _ in range(3000):
        n = rng.choice([rng.randint(0, 12), rng.randint(0, 80), rng.randint(0, 400)])
        hi = rng.choice([64, 2000, 33000])
        keys = [rng.randrange(1, hi) for _ in range(n)]
        real, em = set(), PySet.from_iter(keys)
        for k in keys:
            real.add(k)
        assert list(real) == list(em)
        other = [rng.randrange(1, hi) for _ in range(rng.randint(0, 4))]
        r2, e2 = set(real).union(set(other)), em.copy().union(PySet.from_iter(other))
        assert list(r2) == list(e2)
        assert list(set(k for k in r2)) == list(PySet.from_iter(iter(e2)))


def test_python_oracle_matches_reference_fixtures():
    """oracle/mcclendon.py (the Python restatement with the set emulation) == the reference's
    values on every fixture maze: it pins the restatement the GPU kernel is checked against."""
    sys.path.insert(0, ORACLE)
    import mcclendon as M
    n = 0
    for grid, s, t, d0, c0, _ in _mcclendon_fixture():
        if math.isnan(d0) or grid.shape[0] > 41:
            continue
        assert M.evaluate(grid, s, t) == (d0, c0)
        n += 1
    z = G.load("difficulty81.npz")
    allm = G.mazes("gen_euclid.npz")
    for k in (0, 9, 18):  # one per algorithm at 81x81
        m = allm[int(z["index"][k])]
        assert M.evaluate(m["grid"], m["start"], m["goal"]) == (z["difficulty"][k], z["complexity"][k])
    assert n >= 150
