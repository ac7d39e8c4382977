"""GPU McClendon difficulty (mz_difficulty_batch, csrc/mz_mcclendon.hip) vs the reference's values
and the host restatement (mz_difficulty / mz_maze_complexity, maze_complexity_evaluation.py:38-329).

- the 24 reference 81x81 mazes of gen_euclid.npz: difficulty and complexity equal the values the
  reference's ComplexityEvaluation computed (tests/golden/difficulty81.npz, rel 1e-15 as
  tests/test_difficulty.py) and the host restatement's bit for bit;
- every golden euclidean maze of 15..81 squares and 1,152 GPU-generated mazes (3 algorithms x 6 sizes):
  status 0 and bit-exact with the host restatement;
- the kernel's declines: a maze with a cycle (status 1), toroidal instances (status 4); the
  Python wrapper computes those on the host, equal to the host calls.
"""
import math

import numpy as np
import pytest

import golden_io as G

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mods():
    import torch
    from mazerl import VectorMazeEnv, difficulty
    from mazerl import _native as N
    return torch, VectorMazeEnv, difficulty, N


def _raw(mods, env):
    torch, _, _, N = mods
    n = env.num_envs
    out = torch.empty(n, 2, dtype=torch.float64, device=env.device)
    st = torch.full((n,), -7, dtype=torch.int32, device=env.device)
    N.check(N.load().mz_difficulty_batch(env._h, None, n, out.data_ptr(), st.data_ptr(),
                                         env._stream()))
    return out.cpu().numpy(), st.cpu().numpy()


def _loaded(mods, ms, toroidal=False):
    _, VectorMazeEnv, _, _ = mods
    dim = max(m["n"] for m in ms)
    env = VectorMazeEnv(len(ms), dim, enrich=True, device="cuda:0", generate=False,
                        toroidal=toroidal, done_list=False)
    for n in sorted({m["n"] for m in ms}):  # one load per size (a load sets N = the grid size)
        ids = [k for k, m in enumerate(ms) if m["n"] == n]
        grids = np.stack([ms[k]["grid"] for k in ids]).astype(np.uint8)
        sg = np.array([ms[k]["start"] + ms[k]["goal"] for k in ids], np.int32)
        env.load_mazes(grids, sg, env_ids=np.array(ids, np.int32))
    return env


def test_reference_81x81_values(mods):
    _, _, D, _ = mods
    z = G.load("difficulty81.npz")
    allm = G.mazes("gen_euclid.npz")
    ms = [allm[int(i)] for i in z["index"]]
    assert all(m["n"] == 81 for m in ms) and len(ms) == 24
    env = _loaded(mods, ms)
    pw, st = _raw(mods, env)
    assert (st == 0).all(), st
    d, c = D.difficulty_batch(env, complexity=True)
    exact = 0
    for k, m in enumerate(ms):
        hd, hc = D.maze_complexity(m["grid"], m["start"], m["goal"])
        assert d[k] == hd and c[k] == hc, (k, d[k], hd, c[k], hc)  # bit-exact vs the host
        assert d[k] == math.log(pw[k, 0])
        assert d[k] == pytest.approx(float(z["difficulty"][k]), rel=1e-15, abs=0)
        assert c[k] == pytest.approx(float(z["complexity"][k]), rel=1e-15, abs=0)
        exact += d[k] == z["difficulty"][k]
    assert exact >= 20
    env.close()


def test_golden_euclidean_mazes_bit_exact_with_host(mods):
    _, _, D, _ = mods
    ms = [m for m in G.mazes("gen_euclid.npz") if m["n"] >= 15]  # the env's window needs N >= 15
    env = _loaded(mods, ms)
    pw, st = _raw(mods, env)
    assert (st == 0).all(), np.nonzero(st)[0]
    d, c = D.difficulty_batch(env, complexity=True)
    for k, m in enumerate(ms):
        assert (d[k], c[k]) == D.maze_complexity(m["grid"], m["start"], m["goal"]), k
        if not math.isnan(m["difficulty"]):
            assert d[k] == pytest.approx(m["difficulty"], rel=1e-15, abs=0)
    env.close()


@pytest.mark.parametrize("algo", ["r-prim", "dfs", "prim&kill"])
def test_generated_mazes_bit_exact_with_host(mods, algo):
    _, _, D, _ = mods
    from mazerl.trainers.vector_trainer import make_env
    dims = [15, 21, 33, 41, 61, 81]
    n = 64 * len(dims)
    env = make_env(n, dims, algorithm=algo, seed=0xD1FF, device="cuda:0", done_list=False)
    pw, st = _raw(mods, env)
    assert (st == 0).all(), np.nonzero(st)[0]
    d, c = D.difficulty_batch(env, complexity=True)
    for i in range(n):
        q = env.query(i)
        h = D.maze_complexity(env.grid(i), (q["start_r"], q["start_c"]), (q["goal_r"], q["goal_c"]))
        assert (d[i], c[i]) == h, (i, q["n"], d[i], c[i], h)
    env.close()


def test_declined_mazes_fall_back_to_the_host(mods):
    _, _, D, _ = mods
    ms = [m for m in G.mazes("gen_euclid.npz") if m["n"] == 21][:2]
    cyc = dict(ms[0])
    g = cyc["grid"].copy()
    # open one interior wall between two floor squares of different rows: a cycle
    r, c = next((r, c) for r in range(2, 19, 2) for c in range(1, 20, 2)
                if g[r, c] == 0 and g[r - 1, c] and g[r + 1, c])
    g[r, c] = 1
    cyc["grid"] = g
    env = _loaded(mods, [cyc, ms[1]])
    _, st = _raw(mods, env)
    assert st[0] == 1 and st[1] == 0, st
    d = D.difficulty_batch(env)
    assert d[0] == D.maze_difficulty(g, cyc["start"], cyc["goal"])
    assert d[1] == D.maze_difficulty(ms[1]["grid"], ms[1]["start"], ms[1]["goal"])
    env.close()
    tor = [m for m in G.mazes("gen_toroid.npz") if m["n"] >= 15][:3]
    env = _loaded(mods, tor, toroidal=True)
    _, st = _raw(mods, env)
    assert (st == 4).all()
    d = D.difficulty_batch(env)
    for k, m in enumerate(tor):
        assert d[k] == D.toroidal_difficulty(m["grid"], m["start"], m["goal"])
    env.close()


def test_subset_ids(mods):
    """env_ids lists a subset in any order: out[i] belongs to env_ids[i]."""
    _, VectorMazeEnv, D, _ = mods
    env = VectorMazeEnv(40, 41, enrich=True, device="cuda:0", algorithm="dfs", seed=5,
                        done_list=False)
    full = D.difficulty_batch(env)
    ids = np.array([37, 2, 2, 19, 0], np.int32)
    assert np.array_equal(D.difficulty_batch(env, ids), full[ids])
    env.close()
