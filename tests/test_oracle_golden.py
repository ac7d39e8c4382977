"""Pin the CPU oracle (oracle/mzoracle.c) against the reference's own outputs (tests/golden/).

CPU-only. The fixtures were produced by running the reference Python (make_golden.py); this file
only reads them. Every assertion is bit-exact (integers, bools, and float64 rewards compared with
==), which is the parity bar for this integer/byte path.
"""
import numpy as np
import pytest

import golden_io as G
import pyoracle as O


@pytest.fixture(scope="module")
def euclid():
    return G.mazes("gen_euclid.npz")


@pytest.fixture(scope="module")
def toroid():
    return G.mazes("gen_toroid.npz")


@pytest.fixture(scope="module")
def traces():
    return G.traces()


def test_philox_known_answer():
    # Random123 philox4x32_10 KAT: ctr = 0, key = 0
    assert O.philox(0, 0, 0) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]


def test_goal_selection_euclid(euclid):
    """find_random_position (maze_generation.py:187-218) on every reference maze."""
    for m in euclid:
        g = m["grid"].copy()
        assert g[m["goal"]] == 2
        g[g == 2] = 1
        assert O.goal_select(g, m["start"]) == m["goal"], (m["algo"], m["n"], m["seed"])


def test_goal_selection_toroid(toroid):
    """gen_maze_no_border selects the goal on the bordered (N+2) maze, then crops."""
    for m in toroid:
        g = np.pad(m["grid"], 1)  # cropped border is all wall
        g[g == 2] = 1
        s = (m["start"][0] + 1, m["start"][1] + 1)
        got = O.goal_select(g, s)
        assert got == (m["goal"][0] + 1, m["goal"][1] + 1), (m["algo"], m["n"], m["seed"])


def test_max_steps(euclid, toroid):
    for m in euclid:
        assert O.max_steps(m["grid"], m["start"], m["goal"], False) == m["max_steps"]
    for m in toroid:
        assert O.max_steps(m["grid"], m["start"], m["goal"], True) == m["max_steps"]


def test_astar_len_equals_bfs_field(euclid, toroid):
    """a5: len(astar_limited_partial(src, goal, depth)) == min(D[src], depth) + 1."""
    rng = np.random.default_rng(0)
    for tor, mazes in ((False, euclid), (True, toroid)):
        for m in mazes[:: 3]:
            D = O.bfs(m["grid"], m["goal"], tor)
            cells = np.argwhere(m["grid"] != 0)
            n = m["n"]
            for r, c in cells[rng.choice(len(cells), size=min(40, len(cells)), replace=False)]:
                for depth in (-1, 2 * n):
                    want = D[r, c] + 1 if depth < 0 else min(D[r, c], depth) + 1
                    assert O.astar_len(m["grid"], (r, c), m["goal"], tor, depth) == want


def test_perfect_mazes(euclid):
    """Every reference generator builds a spanning tree: open squares form a tree."""
    for m in euclid:
        g = m["grid"]
        n_open = int((g != 0).sum())
        edges = int(((g[1:, :] != 0) & (g[:-1, :] != 0)).sum() + ((g[:, 1:] != 0) & (g[:, :-1] != 0)).sum())
        D = O.bfs(g, m["start"])
        assert (D[g != 0] >= 0).all()
        assert edges == n_open - 1


@pytest.mark.parametrize("astar_mode", [False, True])
def test_traces_bit_exact(traces, astar_mode):
    """Replay every reference op trace through the oracle env; compare every output."""
    for t in traces:
        env = O.Env(t["grid"], t["start"], t["goal"], t["toroidal"], t["enrich"], astar_mode)
        assert env.max_steps == t["max_steps"]
        env.reset()
        n = t["n"]
        for i, op in enumerate(t["op"]):
            ctx = (t["kind"], n, i, int(op))
            np.testing.assert_array_equal(env.mask(False), t["mask_int"][i].astype(np.float32), err_msg=str(ctx))
            np.testing.assert_array_equal(env.mask(True), t["mask_prob"][i], err_msg=str(ctx))
            o = env.reset() if op == 4 else env.step(int(op))
            assert o["reward"] == t["reward"][i], ctx
            assert o["truncated"] == bool(t["truncated"][i]), ctx
            assert o["terminated"] == bool(t["terminated"][i]), ctx
            assert o["pos"] == tuple(t["pos"][i]), ctx
            assert o["best_dir"] == tuple(t["best_dir"][i]), ctx
            assert o["distance"] == t["distance"][i], ctx
            if t["enrich"]:
                np.testing.assert_array_equal(np.array(o["pos"], np.float64) / np.array([n, n]),
                                              t["agent"][i])
                np.testing.assert_array_equal(o["window"], t["window"][i], err_msg=str(ctx))
            else:
                np.testing.assert_array_equal(np.array(o["pos"], np.float64), t["agent"][i])


def test_oracle_generators_structure():
    """Oracle generators (Philox stream) build perfect mazes with the reference goal rule."""
    for algo in range(3):
        for n in (9, 15, 21, 41):
            for seed in range(4):
                s, gl, g = O.generate(n, algo, 0x5EED0000 + seed)
                assert g[s] == 1 and g[gl] == 2
                n_open = int((g != 0).sum())
                edges = int(((g[1:, :] != 0) & (g[:-1, :] != 0)).sum() + ((g[:, 1:] != 0) & (g[:, :-1] != 0)).sum())
                assert edges == n_open - 1
                h = g.copy(); h[h == 2] = 1
                assert O.goal_select(h, s) == gl
                # every odd cell open, every even/even square wall
                assert (g[1::2, 1::2] != 0).all() and (g[::2, ::2] == 0).all()
