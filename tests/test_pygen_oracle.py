"""CPython-exact generation: the oracle's restatement (oracle/mzpygen.c) of
gen_maze / gen_maze_no_border as CPython 3.10 runs them — MT19937 draws and set iteration order —
pinned against the reference's own mazes (tests/golden/gen_*.npz: random.seed(s) + gen_maze) and
env constructors (tests/golden/envs.npz: random.seed(s) + best-of-6 + the stream position after).

CPU-only. The selection among the six candidates uses libmazerl's native McClendon difficulty
(host C++, mz_difficulty — the product's best-of-6 rule), so the envs.npz check also pins that.
"""
import random

import numpy as np
import pytest

import golden_io as G
import pyoracle as O


def test_tuple_hash_and_mt_state_match_cpython():
    for t in [(0, 0), (1, 2), (3, 5), (80, 79), (128, 1), (127, 127)]:
        h = O.lib().mzo_tuple_hash(*t)
        assert (h - (1 << 64) if h >= 1 << 63 else h) == hash(t)
    for s in [0, 1, 1000, 2**32 - 1, 2**32, 2**40 + 3]:
        assert list(O.mt_state(s)) == list(random.Random(s).getstate()[1]), s
    st = O.mt_state(7)
    r = random.Random(7)
    for n in [1, 2, 3, 7, 40, 41, 1600, 2**20 + 3]:
        for _ in range(50):
            assert int(O.lib().mzo_mt_below(st.ctypes.data_as(O.C.POINTER(O.C.c_uint32)), n)) == r._randbelow(n)


@pytest.mark.parametrize("name,tor", [("gen_euclid.npz", False), ("gen_toroid.npz", True)])
def test_generate_py_reproduces_reference_mazes(name, tor):
    """All 240 golden mazes (3 algorithms x 5 sizes x 8 seeds, euclidean 9..81, toroidal 9..41)."""
    for m in G.mazes(name):
        s, g, grid = O.generate_py(m["n"], m["algo"], m["seed"], tor)
        assert s == m["start"] and g == m["goal"], (name, m["algo"], m["n"], m["seed"])
        np.testing.assert_array_equal(grid, m["grid"])


def test_generate_py_largest_grids_fit():
    """The set tables stay within their capacity up to the largest pitch (127)."""
    for algo in (0, 1, 2):
        for n, tor in ((127, False), (125, True)):
            s, g, grid = O.generate_py(n, algo, 12345 + algo, tor)
            assert grid[g] == 2 and grid[s] == 1


KIND_TOR = {"simple": False, "simple_enrich": False, "simple_variable": False,
            "toroidal": True, "toroidal_enrich": True, "toroidal_variable": True}


def test_env_constructor_best_of_six_and_stream_position():
    """random.seed(s); Env(shape): six candidates from the global stream, the first with the
    smallest difficulty kept; afterwards the stream is where the reference left it."""
    from mazerl.difficulty import maze_difficulty, toroidal_difficulty
    for e in G.envs():
        tor = KIND_TOR[e["kind"]]
        st = O.mt_state(e["seed"])
        best = None
        for _ in range(6):
            s, g, grid = O.generate_py(e["n"], e["algo"], st, tor)
            d = (toroidal_difficulty if tor else maze_difficulty)(grid, s, g)
            if best is None or d < best[0]:
                best = (d, s, g, grid)
        assert best[1] == e["start"] and best[2] == e["goal"], (e["kind"], e["algo"], e["seed"])
        np.testing.assert_array_equal(best[3], e["grid"])
        r = random.Random()
        r.setstate((3, tuple(int(x) for x in st), None))
        assert r.getrandbits(32) == e["probe"]
        assert O.max_steps(e["grid"], e["start"], e["goal"], tor) == e["max_steps"]
