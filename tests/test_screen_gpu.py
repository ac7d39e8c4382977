"""The order-free McClendon screen (mz_screen_batch, csrc/mz_screen.hip) — the first stage of the
best-of-C selection (BaseMazeEnv.generate_maze, base_maze_env.py:78-97).

The screen forms the reference's product prod_b (C_b + 1) * C_0 (maze_complexity_evaluation.py:
319-329) with its sums in an order of its own, and reports a bound e on its relative distance from
the reference's float64 evaluation. Checked here against the order-exact kernel
(mz_difficulty_batch, bit-exact with the reference — tests/test_mcclendon_gpu.py) and the
reference's own values:
- every golden euclidean maze (gen_euclid.npz >= 15 squares, the euclidean mazes of
  mcclendon.npz, the 24 81 x 81 mazes of difficulty81.npz): status 0, |prod - prod_ref| <= e prod;
- 1,152 GPU-generated mazes per algorithm, 15 .. 81 squares: the same against the exact kernel;
- the bound itself stays small (< 2^-30), so a group is sent to the exact kernel only when two
  candidates' difficulties agree to ~9 digits;
- a maze with a cycle is declined (status 2); toroidal handles are refused.
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


def _exact(mods, env):
    torch, _, _, N = mods
    n = env.num_envs
    out = torch.empty(n, 2, dtype=torch.float64, device=env.device)
    st = torch.full((n,), -7, dtype=torch.int32, device=env.device)
    N.check(N.load().mz_difficulty_batch(env._h, None, n, out.data_ptr(), st.data_ptr(),
                                         env._stream()))
    return out.cpu().numpy()[:, 0], st.cpu().numpy()


def _loaded(mods, ms):
    _, VectorMazeEnv, _, _ = mods
    dim = max(m["n"] for m in ms)
    env = VectorMazeEnv(len(ms), dim, enrich=True, device="cuda:0", generate=False,
                        done_list=False)
    for n in sorted({m["n"] for m in ms}):
        ids = [k for k, m in enumerate(ms) if m["n"] == n]
        grids = np.stack([ms[k]["grid"] for k in ids]).astype(np.uint8)
        sg = np.array([ms[k]["start"] + ms[k]["goal"] for k in ids], np.int32)
        env.load_mazes(grids, sg, env_ids=np.array(ids, np.int32))
    return env


def _check_bounds(p, e, st, px, sx):
    assert (st == 0).all(), np.nonzero(st)[0]
    assert (e > 0).all() and (e < 2.0 ** -30).all(), e.max()
    ok = sx == 0
    assert ok.mean() > 0.99
    rel = np.abs(p[ok] - px[ok]) / p[ok]
    assert (rel <= e[ok]).all(), (rel.max(), e[ok][np.argmax(rel / e[ok])])
    return rel


def test_screen_golden_mazes_within_bound_of_the_reference(mods):
    _, _, D, _ = mods
    ms = [m for m in G.mazes("gen_euclid.npz") if m["n"] >= 15]
    z = G.load("mcclendon.npz")
    for i in range(len(z["n"])):
        n = int(z["n"][i])
        if z["toroidal"][i] or n < 15 or math.isnan(float(z["difficulty"][i])):
            continue
        ms.append(dict(grid=z["grid"][i, :n, :n], start=tuple(int(x) for x in z["start"][i]),
                       goal=tuple(int(x) for x in z["goal"][i]),
                       difficulty=float(z["difficulty"][i]), n=n))
    env = _loaded(mods, ms)
    p, e, st = D.screen_batch(env)
    px, sx = _exact(mods, env)
    assert (sx == 0).all()
    _check_bounds(p, e, st, px, sx)
    for k, m in enumerate(ms):  # and the reference's own logs: within the bound + log rounding
        if not math.isnan(m["difficulty"]):
            d = m["difficulty"]
            assert abs(math.log(p[k]) - d) <= e[k] * 1.01 + 4 * math.ulp(d), (k, m["n"])
    env.close()


def test_screen_81x81_reference_values(mods):
    _, _, D, _ = mods
    z = G.load("difficulty81.npz")
    allm = G.mazes("gen_euclid.npz")
    ms = [allm[int(i)] for i in z["index"]]
    env = _loaded(mods, ms)
    p, e, st = D.screen_batch(env)
    assert (st == 0).all()
    for k in range(len(ms)):
        d = float(z["difficulty"][k])
        assert abs(math.log(p[k]) - d) <= e[k] * 1.01 + 4 * math.ulp(d), k
    env.close()


@pytest.mark.parametrize("algo", ["r-prim", "dfs", "prim&kill"])
def test_screen_generated_mazes_within_bound_of_exact(mods, algo):
    _, _, D, _ = mods
    from mazerl.trainers.vector_trainer import make_env
    dims = [15, 21, 33, 41, 61, 81]
    n = 192 * len(dims)
    env = make_env(n, dims, algorithm=algo, seed=0x5C4EE7, device="cuda:0", done_list=False)
    p, e, st = D.screen_batch(env)
    px, sx = _exact(mods, env)
    rel = _check_bounds(p, e, st, px, sx)
    # the screen is the same sums in another order: most products agree to the last bits
    assert np.median(rel) < 1e-14
    # subset ids in any order
    ids = np.array([n - 1, 3, 3, 100], np.int32)
    p2, e2, st2 = D.screen_batch(env, ids)
    assert np.array_equal(p2, p[ids]) or np.allclose(p2, p[ids], rtol=4 * e[ids].max(), atol=0)
    env.close()


def test_screen_declines_a_cycle_and_refuses_toroidal(mods):
    torch, VectorMazeEnv, D, N = mods
    m = [m for m in G.mazes("gen_euclid.npz") if m["n"] == 21][0]
    cyc = dict(m)
    g = cyc["grid"].copy()
    r, c = next((r, c) for r in range(2, 19, 2) for c in range(1, 20, 2)
                if g[r, c] == 0 and g[r - 1, c] and g[r + 1, c])
    g[r, c] = 1
    cyc["grid"] = g
    env = _loaded(mods, [cyc, m])
    _, _, st = D.screen_batch(env)
    assert st[0] == 2 and st[1] == 0, st
    env.close()
    tor = VectorMazeEnv(4, 21, enrich=True, device="cuda:0", toroidal=True, done_list=False)
    out = torch.zeros(4, 2, dtype=torch.float64, device="cuda:0")
    stt = torch.zeros(4, dtype=torch.int32, device="cuda:0")
    assert N.load().mz_screen_batch(tor._h, None, 4, out.data_ptr(), stt.data_ptr(), None) != 0
    tor.close()
