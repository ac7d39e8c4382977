"""GPU McClendon difficulty (mz_difficulty_batch, csrc/mz_mcclendon.hip) vs the reference's values
and the host restatement (mz_difficulty / mz_maze_complexity, maze_complexity_evaluation.py:38-329).

- the 24 reference 81x81 mazes of gen_euclid.npz: difficulty and complexity equal the values the
  reference's ComplexityEvaluation computed (tests/golden/difficulty81.npz) and the host
  restatement's, bit for bit (hallway sums in networkx's subgraph-view set order);
- every golden euclidean maze of 15..81 squares, the toroidal golden mazes (scored on their
  bordered grid, as the reference scores them) and tests/golden/mcclendon.npz: status 0 and
  bit-exact with the reference's values and the host restatement;
- 1,152 GPU-generated euclidean and 768 toroidal mazes (3 algorithms x sizes): bit-exact with the
  host restatement;
- the kernel's declines: a maze with a cycle (status 1); the Python wrapper computes it on the
  host, equal to the host call.
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
    for k, m in enumerate(ms):
        hd, hc = D.maze_complexity(m["grid"], m["start"], m["goal"])
        assert d[k] == hd and c[k] == hc, (k, d[k], hd, c[k], hc)  # bit-exact vs the host
        assert d[k] == math.log(pw[k, 0])
        assert d[k] == z["difficulty"][k] and c[k] == z["complexity"][k], k  # and the reference
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
            assert d[k] == m["difficulty"], k
    env.close()


def test_golden_toroidal_mazes_on_the_gpu(mods):
    """Toroidal handles: the kernel scores the bordered maze (wall ring, start / goal + 1) —
    status 0, == the reference's gen_maze_no_border difficulty and the host restatement."""
    _, _, D, _ = mods
    ms = [m for m in G.mazes("gen_toroid.npz") if m["n"] >= 17]
    env = _loaded(mods, ms, toroidal=True)
    _, st = _raw(mods, env)
    assert (st == 0).all(), np.nonzero(st)[0]
    d, c = D.difficulty_batch(env, complexity=True)
    for k, m in enumerate(ms):
        assert d[k] == D.toroidal_difficulty(m["grid"], m["start"], m["goal"]), k
        assert c[k] == D.toroidal_complexity(m["grid"], m["start"], m["goal"]), k
        if not math.isnan(m["difficulty"]):
            assert d[k] == m["difficulty"], k
    env.close()


def test_set_order_fixture_on_the_gpu(mods):
    """tests/golden/mcclendon.npz (228 reference mazes, euclidean 9..61 and re-bordered toroidal
    9..41): the euclidean ones of >= 15 squares in a euclidean handle, the toroidal ones cropped
    back into a toroidal handle — GPU == the reference's difficulty and complexity."""
    _, _, D, _ = mods
    z = G.load("mcclendon.npz")
    eu, to = [], []
    for i in range(len(z["n"])):
        n = int(z["n"][i])
        m = dict(grid=z["grid"][i, :n, :n], start=tuple(int(x) for x in z["start"][i]),
                 goal=tuple(int(x) for x in z["goal"][i]), difficulty=float(z["difficulty"][i]),
                 complexity=float(z["complexity"][i]), n=n)
        if math.isnan(m["difficulty"]):
            continue
        if z["toroidal"][i]:
            if n - 2 >= 17:
                to.append(dict(m, grid=m["grid"][1:-1, 1:-1], n=n - 2,
                               start=(m["start"][0] - 1, m["start"][1] - 1),
                               goal=(m["goal"][0] - 1, m["goal"][1] - 1)))
        elif n >= 15:
            eu.append(m)
    assert len(eu) >= 100 and len(to) >= 40
    for ms, tor in ((eu, False), (to, True)):
        env = _loaded(mods, ms, toroidal=tor)
        _, st = _raw(mods, env)
        assert (st == 0).all(), (tor, np.nonzero(st)[0])
        d, c = D.difficulty_batch(env, complexity=True)
        for k, m in enumerate(ms):
            assert d[k] == m["difficulty"] and c[k] == m["complexity"], (tor, k, m["n"])
        env.close()


@pytest.mark.parametrize("algo", ["r-prim", "dfs", "prim&kill"])
def test_generated_toroidal_mazes_bit_exact_with_host(mods, algo):
    _, _, D, _ = mods
    from mazerl.trainers.vector_trainer import make_env
    dims = [17, 29, 41, 53, 65, 79, 23, 35]
    n = 32 * len(dims)
    env = make_env(n, dims, toroidal=True, algorithm=algo, seed=0x70D1FF, device="cuda:0",
                   done_list=False)
    pw, st = _raw(mods, env)
    assert (st == 0).all(), np.nonzero(st)[0]
    d, c = D.difficulty_batch(env, complexity=True)
    for i in range(n):
        q = env.query(i)
        g, s, t = env.grid(i), (q["start_r"], q["start_c"]), (q["goal_r"], q["goal_c"])
        h = (D.toroidal_difficulty(g, s, t), D.toroidal_complexity(g, s, t))
        assert (d[i], c[i]) == h, (i, q["n"], d[i], c[i], h)
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


def test_subset_ids(mods):
    """env_ids lists a subset in any order: out[i] belongs to env_ids[i]."""
    _, VectorMazeEnv, D, _ = mods
    env = VectorMazeEnv(40, 41, enrich=True, device="cuda:0", algorithm="dfs", seed=5,
                        done_list=False)
    full = D.difficulty_batch(env)
    ids = np.array([37, 2, 2, 19, 0], np.int32)
    assert np.array_equal(D.difficulty_batch(env, ids), full[ids])
    env.close()
