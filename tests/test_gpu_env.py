"""GPU parity of libmazerl.so (HIP, gfx950) against the reference fixtures and the CPU oracle.

Every comparison is bit-exact: integer state, bools, float64 rewards (==) and the float32
observation tensors. All compute goes through the C ABI (mazerl.VectorMazeEnv -> libmazerl.so).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import golden_io as G  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mazerl():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import mazerl as M
    return M


def _group_traces():
    groups = {}
    for t in G.traces():
        groups.setdefault((t["toroidal"], t["enrich"]), []).append(t)
    return groups


@pytest.mark.parametrize("key", [(False, False), (False, True), (True, False), (True, True)])
def test_reference_traces_bit_exact(mazerl, key):
    """Replay the reference's own op traces (tests/golden/traces.npz) through the batched GPU env."""
    ts = _group_traces()[key]
    tor, enrich = key
    B = len(ts)
    maxn = max(t["n"] for t in ts)
    env = mazerl.VectorMazeEnv(B, maxn, toroidal=tor, enrich=enrich, generate=False, reward64=True)
    for i, t in enumerate(ts):
        env.load_mazes(t["grid"][None], np.array([[*t["start"], *t["goal"]]]), env_ids=[i])
    for i, t in enumerate(ts):
        assert env.query(i)["max_steps"] == t["max_steps"]
        np.testing.assert_array_equal(env.grid(i), t["grid"])
    env.reset()
    T = max(len(t["op"]) for t in ts)
    for step in range(T):
        active = [i for i, t in enumerate(ts) if step < len(t["op"])]
        ops = np.full(B, -1, np.int32)
        for i in active:
            ops[i] = ts[i]["op"][step]
        mi = env.direction_mask(False).cpu().numpy()
        mp = env.direction_mask(True).cpu().numpy()
        for i in active:
            np.testing.assert_array_equal(mi[i], ts[i]["mask_int"][step].astype(np.float32))
            np.testing.assert_array_equal(mp[i], ts[i]["mask_prob"][step])
        acts = np.where(ops == 4, -1, ops).astype(np.int32)
        env.step(torch.from_numpy(acts).cuda())
        resets = [i for i in active if ops[i] == 4]
        if resets:
            env.reset_list(torch.tensor(resets, dtype=torch.int32))
        r64 = env.reward64.cpu().numpy()
        r32 = env.reward.cpu().numpy()
        te = env.terminated.cpu().numpy()
        tr = env.truncated.cpu().numpy()
        pos = env.pos.cpu().numpy()
        bd = env.best_dir.cpu().numpy()
        o6 = env.obs6.cpu().numpy()
        win = env.window.cpu().numpy() if enrich else None
        wb = env.window_bits.cpu().numpy() if enrich else None
        for i in active:
            t, n = ts[i], ts[i]["n"]
            ctx = (key, t["n"], step, int(ops[i]))
            assert r64[i] == t["reward"][step], ctx
            assert r32[i] == np.float32(t["reward"][step]), ctx
            assert bool(te[i]) == bool(t["terminated"][step]), ctx
            assert bool(tr[i]) == bool(t["truncated"][step]), ctx
            np.testing.assert_array_equal(pos[i], t["pos"][step], err_msg=str(ctx))
            np.testing.assert_array_equal(bd[i], t["best_dir"][step], err_msg=str(ctx))
            want6 = np.concatenate([t["agent"][step], t["target"][step], t["best_dir"][step]]).astype(np.float32)
            np.testing.assert_array_equal(o6[i], want6, err_msg=str(ctx))
            if enrich:
                np.testing.assert_array_equal(win[i], t["window"][step].astype(np.float32), err_msg=str(ctx))
                bits = np.unpackbits(wb[i].view(np.uint8), bitorder="little")[:675]
                np.testing.assert_array_equal(bits.reshape(3, 15, 15), t["window"][step], err_msg=str(ctx))
    env.close()


@pytest.mark.parametrize("tor,dims", [(False, (15, 21, 41, 81)), (True, (9, 17, 29, 41))])
def test_generation_matches_oracle(mazerl, tor, dims):
    """GPU generators (r-prim / dfs / prim&kill + goal + crop) == oracle restatement, same Philox stream."""
    import pyoracle as O
    B = 24
    algos = np.arange(B) % 3
    for dim in dims:
        env = mazerl.VectorMazeEnv(B, dim, toroidal=tor, enrich=False, generate=False)
        env.generate(algorithm=algos, dim=dim, seed=0x5EED0000 + dim)
        torch.cuda.synchronize()
        for i in range(B):
            (sr, sc), (gr, gc), g = O.generate(dim, int(algos[i]), 0x5EED0000 + dim + i, tor)
            q = env.query(i)
            np.testing.assert_array_equal(env.grid(i), g, err_msg=f"dim {dim} env {i}")
            assert (q["start_r"], q["start_c"], q["goal_r"], q["goal_c"]) == (sr, sc, gr, gc)
            assert q["max_steps"] == O.max_steps(g, (sr, sc), (gr, gc), tor)
        env.close()


def _cell_words(env):
    """The handle's cell words [B, P, P] (the first section of mz_state_save's blob)."""
    blob = env.state_dict()["device_state"].cpu().numpy()
    B, P = env.num_envs, env.max_dim
    return blob[256:256 + B * P * P * 4].view(np.uint32).reshape(B, P, P)


@pytest.mark.parametrize("tor,dims", [(False, (15, 21, 41, 81, 127)), (True, (17, 41, 79, 125))])
def test_generated_distance_field_matches_bfs(mazerl, tor, dims):
    """The distance-to-goal field in the cell words (len(find_path(p)) = D[p] + 1, a5) of
    Philox-generated mazes — derived from the carved tree for euclidean mazes (mz_cs_dist of the
    cell-space build), by the row-mask BFS on the torus — == the oracle's BFS from the goal on
    every open cell, and the
    open / open-neighbour bits == the grid, for all three generators."""
    import pyoracle as O
    B = 48
    algos = np.arange(B) % 3
    for dim in dims:
        env = mazerl.VectorMazeEnv(B, dim, toroidal=tor, enrich=False, generate=False)
        env.generate(algorithm=algos, dim=dim, seed=0xD15700 + dim)
        torch.cuda.synchronize()
        cw = _cell_words(env)
        for i in range(B):
            g = env.grid(i)
            q = env.query(i)
            want = O.bfs(g, (q["goal_r"], q["goal_c"]), tor)
            w = cw[i, :dim, :dim]
            open_ = g != 0
            np.testing.assert_array_equal((w >> 16) & 1, open_.astype(np.uint32), err_msg=f"dim {dim} env {i}")
            np.testing.assert_array_equal((w & 0x1FFF)[open_], want[open_], err_msg=f"dim {dim} env {i} algo {algos[i]}")
        env.close()


@pytest.mark.parametrize("tor,dims", [(False, (81, 127)), (True, (79, 125))])
def test_primkill_restart_pick_matches_oracle(mazerl, tor, dims):
    """prim&kill's restart pick (maze_generation.py:151: the k-th marked cell with an unmarked
    neighbour, row-major) from the candidate bits the walk keeps current == the oracle's full
    rescan, over many seeds and up to the largest pitch (127)."""
    import pyoracle as O
    B, algo = 128, 2
    for dim in dims:
        env = mazerl.VectorMazeEnv(B, dim, toroidal=tor, enrich=False, generate=False)
        env.generate(algorithm="prim&kill", dim=dim, seed=0x9C0000 + dim)
        torch.cuda.synchronize()
        for i in range(B):
            (sr, sc), (gr, gc), g = O.generate(dim, algo, 0x9C0000 + dim + i, tor)
            q = env.query(i)
            np.testing.assert_array_equal(env.grid(i), g, err_msg=f"dim {dim} env {i}")
            assert (q["start_r"], q["start_c"], q["goal_r"], q["goal_c"]) == (sr, sc, gr, gc)
        env.close()


def test_full_size_vs_oracle_sample(mazerl):
    """65,536 x 81x81 r-prim (the headline config): step with the fused exploration kernel; a
    sample of instances is replayed through the oracle with the same actions; size-independent
    invariants are checked on all instances."""
    import pyoracle as O
    B, dim, K = 65536, 81, 60
    env = mazerl.VectorMazeEnv(B, dim, enrich=True, reward64=True)
    sample = list(range(0, B, B // 64))
    oracles = {}
    for i in sample:
        q = env.query(i)
        oracles[i] = O.Env(env.grid(i), (q["start_r"], q["start_c"]), (q["goal_r"], q["goal_c"]),
                           False, True)
        oracles[i].reset()
        assert oracles[i].max_steps == q["max_steps"]
    for k in range(K):
        acts = env.act(eps=1.0, seed=7, counter=k)
        a_host = acts.cpu().numpy()
        env.step(acts)
        te, tr = env.terminated.bool(), env.truncated.bool()
        done = te | tr
        cnt = int(env.done_count.item())
        assert cnt == int(done.sum().item())
        idx = set(env.done_idx[:cnt].cpu().tolist())
        assert idx == set(torch.nonzero(done).flatten().cpu().tolist())
        r64 = env.reward64.cpu().numpy()
        pos = env.pos.cpu().numpy()
        win = env.window[sample].cpu().numpy()
        for j, i in enumerate(sample):
            o = oracles[i].step(int(a_host[i]))
            assert o["reward"] == r64[i]
            assert tuple(pos[i]) == o["pos"]
            np.testing.assert_array_equal(win[j], o["window"].astype(np.float32))
            if o["terminated"] or o["truncated"]:
                oracles[i].reset()
        # window invariants on every instance: channels are disjoint indicator planes
        w = env.window
        assert torch.all((w[:, 0] + w[:, 1]) <= 1)
        assert torch.all(w[:, 2] <= 1 - w[:, 0])
        # expand(bits) == f32 window
        torch.testing.assert_close(env.expand_window(env.window_bits), w, rtol=0, atol=0)
        env.reset_done()
    env.close()


def test_act_kernel(mazerl):
    env = mazerl.VectorMazeEnv(4096, 21, enrich=True)
    a1 = env.act(eps=1.0, seed=3, counter=5).clone()
    a2 = env.act(eps=1.0, seed=3, counter=5).clone()
    assert torch.equal(a1, a2)
    m = env.direction_mask(True)
    assert torch.all(m.gather(1, a1.long()[:, None]) > 0)  # only open / 0.25-weighted moves
    g = torch.randint(0, 4, (4096,), device="cuda")
    a3 = env.act(eps=0.0, greedy=g, seed=3, counter=6)
    assert torch.equal(a3.long(), g)
    env.close()


def test_rejects_reference_crash_shapes(mazerl):
    with pytest.raises(ValueError):
        mazerl.VectorMazeEnv(4, 40, enrich=False)  # even N: reference IndexError (Q4)
    with pytest.raises(ValueError):
        mazerl.VectorMazeEnv(4, 9, enrich=True)  # euclidean window with N < 15 (Q7)


@pytest.mark.parametrize("tor,dim", [(False, 41), (True, 29)])
def test_fused_step_act_matches_separate(mazerl, tor, dim):
    """mz_step_act (one launch) == mz_act + mz_step, including done lists and auto-resets."""
    B = 3000
    e1 = mazerl.VectorMazeEnv(B, dim, toroidal=tor, enrich=True, reward64=True, seed=99)
    e2 = mazerl.VectorMazeEnv(B, dim, toroidal=tor, enrich=True, reward64=True, seed=99)
    for k in range(120):
        a = e1.act(eps=1.0, seed=5, counter=k).clone()
        e1.step(a)
        e2.step_act(eps=1.0, seed=5, counter=k)
        assert torch.equal(e2.actions, a)
        for name in ("reward64", "terminated", "truncated", "pos", "best_dir", "obs6", "window",
                     "window_bits"):
            assert torch.equal(getattr(e1, name), getattr(e2, name)), (k, name)
        c1, c2 = int(e1.done_count.item()), int(e2.done_count.item())
        assert c1 == c2
        assert sorted(e1.done_idx[:c1].tolist()) == sorted(e2.done_idx[:c2].tolist())
        e1.reset_done()        # flag-scan auto-reset
        e2.reset_done_list()   # device-list auto-reset (consumes the count)
        assert int(e2.done_count.item()) == 0
        for name in ("obs6", "window", "window_bits"):
            assert torch.equal(getattr(e1, name), getattr(e2, name)), (k, name)
    e1.close(); e2.close()


def test_regen_on_win(mazerl):
    """win -> new maze (regen_won): a won instance gets a different maze of the same size whose
    tables are consistent (oracle goal/max_steps), others keep theirs."""
    import pyoracle as O
    B, dim = 256, 15
    env = mazerl.VectorMazeEnv(B, dim, enrich=True, seed=1234)
    grids0 = [env.grid(i) for i in range(B)]
    won = set()
    for k in range(400):
        # follow "best dir" greedily: a = action whose delta == -best_dir
        bd = env.best_dir.long()
        dr, dc = -bd[:, 0], -bd[:, 1]
        greedy = torch.where(dr == 1, 0, torch.where(dr == -1, 1, torch.where(dc == 1, 2, 3)))
        env.step_act(eps=0.0, greedy=greedy, seed=1, counter=k)
        won |= set(torch.nonzero(env.terminated).flatten().tolist())
        env.reset_done(regen_won=True)
        if len(won) >= 32:
            break
    assert len(won) >= 32
    torch.cuda.synchronize()
    changed = 0
    for i in range(B):
        g = env.grid(i)
        if i in won:
            changed += not np.array_equal(g, grids0[i])
            q = env.query(i)
            h = g.copy(); h[h == 2] = 1
            assert O.goal_select(h, (q["start_r"], q["start_c"])) == (q["goal_r"], q["goal_c"])
            assert q["max_steps"] == O.max_steps(g, (q["start_r"], q["start_c"]), (q["goal_r"], q["goal_c"]))
    assert changed >= len(won) - 1
    env.close()


@pytest.mark.parametrize("tor,dim,B", [(False, 15, 192), (False, 21, 192), (True, 17, 192),
                                       (True, 29, 128)])
def test_autoreset_step_vs_oracle(mazerl, tor, dim, B):
    """MZ_STEP_AUTORESET (one launch per vector step): an instance whose previous step ended is
    reset by the next launch (action ignored, reported as -1, reward 0, reset observation);
    every other instance steps with its sampled action. Replayed through the oracle, which
    calls reset() exactly where the reference trainer does (off_policy_trainer.py:153)."""
    import pyoracle as O
    env = mazerl.VectorMazeEnv(B, dim, toroidal=tor, enrich=True, reward64=True, seed=4242)
    ors = []
    for i in range(B):
        q = env.query(i)
        o = O.Env(env.grid(i), (q["start_r"], q["start_c"]), (q["goal_r"], q["goal_c"]), tor, True)
        o.reset()
        ors.append(o)
    was_done = np.zeros(B, bool)
    resets = 0
    for k in range(400):
        env.step_act(eps=1.0, seed=21, counter=k, autoreset=True)
        a = env.actions.cpu().numpy()
        r64 = env.reward64.cpu().numpy()
        te, tr = env.terminated.cpu().numpy(), env.truncated.cpu().numpy()
        pos, bd = env.pos.cpu().numpy(), env.best_dir.cpu().numpy()
        win = env.window.cpu().numpy()
        bits = env.expand_window(env.window_bits).cpu().numpy()
        for i in range(B):
            if was_done[i]:
                assert a[i] == -1, (k, i)
                o = ors[i].reset()
                resets += 1
            else:
                assert 0 <= a[i] < 4, (k, i)
                o = ors[i].step(int(a[i]))
            assert r64[i] == o["reward"], (k, i)
            assert bool(te[i]) == o["terminated"] and bool(tr[i]) == o["truncated"], (k, i)
            assert tuple(pos[i]) == o["pos"] and tuple(bd[i]) == o["best_dir"], (k, i)
            np.testing.assert_array_equal(win[i], o["window"].astype(np.float32))
            np.testing.assert_array_equal(bits[i], win[i])
            was_done[i] = o["terminated"] or o["truncated"]
    assert resets > 0
    env.close()


@pytest.mark.parametrize("name,tor", [("gen_euclid.npz", False), ("gen_toroid.npz", True)])
def test_cpython_generation_matches_reference_mazes(mazerl, name, tor):
    """rng="cpython": instance i gets the maze of random.seed(seed + i); gen_maze(...) — checked
    against the reference's own 240 golden mazes (3 algorithms x 5 sizes x 8 seeds)."""
    ms = G.mazes(name)
    maxn = max(m["n"] for m in ms)
    env = mazerl.VectorMazeEnv(len(ms), maxn, toroidal=tor, enrich=False, generate=False)
    for i, m in enumerate(ms):
        env.generate(env_ids=[i], algorithm=m["algo"], dim=m["n"],
                     seed=(m["seed"] - i) & 0xFFFFFFFFFFFFFFFF, rng="cpython")
    for i, m in enumerate(ms):
        q = env.query(i)
        key = (m["algo"], m["n"], m["seed"])
        np.testing.assert_array_equal(env.grid(i), m["grid"], err_msg=str(key))
        assert (q["start_r"], q["start_c"]) == m["start"] and (q["goal_r"], q["goal_c"]) == m["goal"], key
        assert q["max_steps"] == m["max_steps"], key
    env.close()


@pytest.mark.parametrize("tor,dim,B", [(False, 81, 192), (True, 41, 96), (False, 127, 12)])
def test_cpython_generation_bulk_vs_oracle(mazerl, tor, dim, B):
    """One launch, B instances per algorithm at the headline size (and the largest pitch):
    every maze == the oracle's CPython restatement from random.seed(seed + i)."""
    import pyoracle as O
    for algo in (0, 1, 2):
        env = mazerl.VectorMazeEnv(B, dim, toroidal=tor, enrich=False, generate=False)
        seed = 777 + 1000 * algo
        env.generate(algorithm=algo, seed=seed, rng="cpython")
        for i in range(B):
            s, g, grid = O.generate_py(dim, algo, seed + i, tor)
            q = env.query(i)
            np.testing.assert_array_equal(env.grid(i), grid, err_msg=str((algo, i)))
            assert (q["start_r"], q["start_c"]) == s and (q["goal_r"], q["goal_c"]) == g
        env.close()


def test_generate_from_random_advances_python_stream(mazerl):
    """generate_from_random consumes a random.Random exactly like gen_maze would."""
    import random
    import pyoracle as O
    env = mazerl.VectorMazeEnv(2, 41, enrich=False, generate=False)
    for algo in (0, 1, 2):
        r = random.Random(99 + algo)
        st = O.mt_state(99 + algo)
        for k in range(3):
            env.generate_from_random(k % 2, algo, dim=41, rnd=r)
            s, g, grid = O.generate_py(41, algo, st)
            np.testing.assert_array_equal(env.grid(k % 2), grid)
            assert list(st) == list(r.getstate()[1])
    env.close()


@pytest.mark.parametrize("tor,dim,ar", [(False, 15, False), (True, 17, False), (False, 15, True),
                                        (True, 17, True)])
def test_many_episodes_reset_done_vs_oracle(mazerl, tor, dim, ar):
    """Visit counts live in the cell words under a 3-bit episode tag that wraps every 8 resets
    (then the counts are cleared). Replay 25+ episodes per instance — through step + k_reset_done (flag-scan
    auto-reset) or through k_step's fused autoreset — against the oracle, rewards compared as
    float64 ==."""
    import pyoracle as O
    B = 96
    env = mazerl.VectorMazeEnv(B, dim, toroidal=tor, enrich=True, reward64=True, seed=777)
    ors = []
    for i in range(B):
        q = env.query(i)
        o = O.Env(env.grid(i), (q["start_r"], q["start_c"]), (q["goal_r"], q["goal_c"]), tor, True)
        o.reset()
        ors.append(o)
    episodes = np.zeros(B, np.int64)
    was_done = np.zeros(B, bool)
    for k in range(1500):
        env.step_act(eps=1.0, seed=5, counter=k, autoreset=ar)
        a = env.actions.cpu().numpy()
        r64 = env.reward64.cpu().numpy()
        win = env.window.cpu().numpy()
        done = (env.terminated | env.truncated).cpu().numpy().astype(bool)
        for i in range(B):
            if ar and was_done[i]:
                assert a[i] == -1, (k, i)
                o = ors[i].reset()
            else:
                o = ors[i].step(int(a[i]))
            assert r64[i] == o["reward"], (k, i)
            assert bool(done[i]) == (o["terminated"] or o["truncated"]), (k, i)
            np.testing.assert_array_equal(win[i], o["window"].astype(np.float32))
            if done[i]:
                if not ar:
                    ors[i].reset()
                episodes[i] += 1
            was_done[i] = done[i]
        if not ar:
            env.reset_done()
    assert episodes.min() >= 9, episodes.min()  # every instance wrapped its tag at least once
    env.close()


@pytest.mark.parametrize("tor,dim,B", [(False, 127, 64), (True, 127, 48), (True, 5, 64),
                                       (False, 15, 1), (True, 15, 33)])
def test_extreme_sizes_vs_oracle(mazerl, tor, dim, B):
    """Largest pitch (127: three plane word pairs + a fourth, 13-bit D), the smallest toroidal
    grid (5 < window: rows and columns wrap several times), N = 15 (window == maze; toroidal
    15 is the reference's Q8 crash, generic wrapped window here), a single instance and a
    batch that is not a multiple of 32: stepping with autoreset vs the oracle."""
    import pyoracle as O
    env = mazerl.VectorMazeEnv(B, dim, toroidal=tor, enrich=True, reward64=True, seed=31337,
                               algorithm="dfs")
    ors = []
    for i in range(B):
        q = env.query(i)
        o = O.Env(env.grid(i), (q["start_r"], q["start_c"]), (q["goal_r"], q["goal_c"]), tor, True)
        o.reset()
        ors.append(o)
        assert o.max_steps == q["max_steps"]
    was_done = np.zeros(B, bool)
    for k in range(150):
        env.step_act(eps=1.0, seed=9, counter=k, autoreset=True)
        a = env.actions.cpu().numpy()
        r64 = env.reward64.cpu().numpy()
        pos, bd = env.pos.cpu().numpy(), env.best_dir.cpu().numpy()
        win = env.window.cpu().numpy()
        te, trn = env.terminated.cpu().numpy(), env.truncated.cpu().numpy()
        for i in range(B):
            o = ors[i].reset() if was_done[i] else ors[i].step(int(a[i]))
            assert r64[i] == o["reward"], (k, i)
            assert tuple(pos[i]) == o["pos"] and tuple(bd[i]) == o["best_dir"], (k, i)
            np.testing.assert_array_equal(win[i], o["window"].astype(np.float32))
            was_done[i] = bool(te[i]) or bool(trn[i])
    env.close()


def test_host_scalars_match_device_outputs(mazerl):
    """VectorMazeEnv(host_scalars=True) — action and scalar outputs in mapped host memory
    (mz_host_alloc) — gives the same actions, rewards, flags, positions and windows as the
    device-output env on the same mazes and seeds, fused act + step with autoreset."""
    import torch
    B = 37
    A = mazerl.VectorMazeEnv(B, 21, enrich=True, reward64=True, seed=99)
    H = mazerl.VectorMazeEnv(B, 21, enrich=True, reward64=True, seed=99, host_scalars=True)
    assert H.reward64.device.type == "cpu" and H.obs6.is_cuda
    for k in range(120):
        A.step_act(eps=1.0, seed=4, counter=k, autoreset=True)
        H.step_act(eps=1.0, seed=4, counter=k, autoreset=True)
        H.sync()
        assert torch.equal(A.actions.cpu(), H.actions)
        assert torch.equal(A.reward64.cpu(), H.reward64)
        assert torch.equal(A.terminated.cpu(), H.terminated) and torch.equal(A.truncated.cpu(), H.truncated)
        assert torch.equal(A.pos.cpu(), H.pos) and torch.equal(A.best_dir.cpu(), H.best_dir)
        assert torch.equal(A.window, H.window) and torch.equal(A.obs6, H.obs6)
    for k in range(20):  # one instance through step_host (the drop-ins' path)
        a = int(k % 4)
        acts = torch.full((B,), -1, dtype=torch.int32, device="cuda")
        acts[0] = a
        A.step(acts)
        H.actions.fill_(-1)
        H.step_host(a)
        assert float(A.reward64[0]) == float(H.reward64[0]) and A.pos[0].tolist() == H.pos[0].tolist()
    A.close()
    H.close()


@pytest.mark.parametrize("B", [32768, 16400])
def test_large_batch_fused_autoreset_every_lane_vs_oracle(mazerl, B):
    """Batches above 16,384 step with 16 instances per wave, the bench's path (fused act + step +
    autoreset); 32,768 also takes the XCD-aware group map (grid a multiple of 8), 16,400 ends in
    a partial group without it. Every lane of several whole groups (first, middle, last) is
    replayed through the oracle, rewards as float64 ==, windows and positions exactly."""
    import pyoracle as O
    dim = 21
    env = mazerl.VectorMazeEnv(B, dim, enrich=True, reward64=True, seed=0xC0FFEE)
    groups = sorted({0, 1, (B // 16) // 2, (B - 1) // 16})
    sample = [i for g in groups for i in range(16 * g, min(B, 16 * g + 16))]
    ors = {}
    for i in sample:
        q = env.query(i)
        ors[i] = O.Env(env.grid(i), (q["start_r"], q["start_c"]), (q["goal_r"], q["goal_c"]), False, True)
        ors[i].reset()
    was_done = {i: False for i in sample}
    resets = 0
    for k in range(150):
        env.step_act(eps=1.0, seed=17, counter=k, autoreset=True)
        a = env.actions.cpu().numpy()
        r64 = env.reward64.cpu().numpy()
        pos, bd = env.pos.cpu().numpy(), env.best_dir.cpu().numpy()
        te, tr = env.terminated.cpu().numpy(), env.truncated.cpu().numpy()
        win = env.window[sample].cpu().numpy()
        for j, i in enumerate(sample):
            if was_done[i]:
                assert a[i] == -1, (k, i)
                o = ors[i].reset()
                resets += 1
            else:
                o = ors[i].step(int(a[i]))
            assert r64[i] == o["reward"], (k, i)
            assert tuple(pos[i]) == o["pos"] and tuple(bd[i]) == o["best_dir"], (k, i)
            assert bool(te[i]) == o["terminated"] and bool(tr[i]) == o["truncated"], (k, i)
            np.testing.assert_array_equal(win[j], o["window"].astype(np.float32))
            was_done[i] = o["terminated"] or o["truncated"]
    assert resets > 0
    env.close()


def test_headline_config_every_lane_autoreset_vs_oracle(mazerl):
    """The bench's kernel instantiation (k_step<16, euclidean, Enrich, fused act, autoreset) at
    the headline config, 65,536 x 81x81 r-prim: every lane of 9 whole 16-instance groups — one
    in each XCD's slice of the group map (mz_env.hip k_step: workgroup b steps group
    (b & 7) * grid/8 + (b >> 3)) plus the last group — replayed through the oracle for 400 vector
    steps, rewards as float64 ==, flags, positions, best dirs and f32 windows exactly. Actions:
    epsilon-mixed best-dir following (eps 0.3: episodes end in wins across multi-strip windows);
    two groups play loaded copies of their mazes with the start two cells from the goal
    (max_steps 7) at eps 1.0, so truncation resets come often too. >= 100 resets must occur in
    the sampled lanes, of both kinds."""
    import pyoracle as O
    B, dim, K = 65536, 81, 400
    env = mazerl.VectorMazeEnv(B, dim, enrich=True, reward64=True, seed=0x5EED0000)
    per_xcd = (B // 16) // 8
    groups = [x * per_xcd + (61 * x) % per_xcd for x in range(8)] + [B // 16 - 1]
    sample = [i for g in groups for i in range(16 * g, 16 * g + 16)]
    short = [i for g in (groups[3], groups[8]) for i in range(16 * g, 16 * g + 16)]
    grids, sg = [], []
    for i in short:
        g = env.grid(i)
        q = env.query(i)
        gr, gc = q["goal_r"], q["goal_c"]
        for dr, dc in ((1, 0), (-1, 0), (0, 1), (0, -1)):
            if 0 < gr + 2 * dr < dim - 1 and 0 < gc + 2 * dc < dim - 1 and g[gr + dr, gc + dc]:
                sg.append((gr + 2 * dr, gc + 2 * dc, gr, gc))
                break
        grids.append(g)
    env.load_mazes(np.stack(grids), np.array(sg), env_ids=short)
    env.reset()
    eps = torch.full((B,), 0.3, device="cuda")
    eps[torch.tensor(short, device="cuda")] = 1.0
    ors = {}
    for i in sample:
        q = env.query(i)
        ors[i] = O.Env(env.grid(i), (q["start_r"], q["start_c"]), (q["goal_r"], q["goal_c"]), False, True)
        ors[i].reset()
        if i in short:
            assert q["max_steps"] == ors[i].max_steps == 7
    idx = torch.tensor(sample, device="cuda")
    was_done = {i: False for i in sample}
    short_set = set(short)
    wins = truncs = resets = long_wins = 0
    for k in range(K):
        bd = env.best_dir.long()
        dr, dc = -bd[:, 0], -bd[:, 1]
        greedy = torch.where(dr == 1, 0, torch.where(dr == -1, 1, torch.where(dc == 1, 2, 3)))
        env.step_act(eps=eps, greedy=greedy, seed=0xB16, counter=k, autoreset=True)
        a = env.actions[idx].cpu().numpy()
        r64 = env.reward64[idx].cpu().numpy()
        te, tr = env.terminated[idx].cpu().numpy(), env.truncated[idx].cpu().numpy()
        pos, bdir = env.pos[idx].cpu().numpy(), env.best_dir[idx].cpu().numpy()
        win = env.window[idx].cpu().numpy()
        bits = env.expand_window(env.window_bits[idx].contiguous()).cpu().numpy()
        for j, i in enumerate(sample):
            if was_done[i]:
                assert a[j] == -1, (k, i)
                o = ors[i].reset()
                resets += 1
            else:
                assert 0 <= a[j] < 4, (k, i)
                o = ors[i].step(int(a[j]))
            assert r64[j] == o["reward"], (k, i)
            assert bool(te[j]) == o["terminated"] and bool(tr[j]) == o["truncated"], (k, i)
            assert tuple(pos[j]) == o["pos"] and tuple(bdir[j]) == o["best_dir"], (k, i)
            np.testing.assert_array_equal(win[j], o["window"].astype(np.float32), err_msg=f"{k} {i}")
            np.testing.assert_array_equal(bits[j], win[j])
            wins += bool(te[j])
            long_wins += bool(te[j]) and i not in short_set
            truncs += bool(tr[j]) and not bool(te[j])
            was_done[i] = o["terminated"] or o["truncated"]
    assert resets >= 100 and wins >= 20 and truncs >= 20, (resets, wins, truncs)
    assert long_wins >= 8, long_wins  # wins on the generated 81x81 mazes too (long paths)
    env.close()


@pytest.mark.parametrize("tor,dim", [(False, 21), (True, 17), (False, 81), (True, 29)])
def test_act_draw_follows_reference_exploration_distribution(mazerl, tor, dim):
    """The fused act's exploration draw (act_draw, csrc/mz_env.hip) against the reference's
    np.random.choice(4, p=mask / mask.sum()) (dqn_agent.py:109-112) with the 0.25 weight on the
    step back after >= 2 moves — on the torus on the transposed direction (Q6,
    toroidal_maze_env.py:64-68); the masks themselves are pinned bit-exactly to the reference
    by the traces (get_mask_direction(probs=True)). 4,096 instances in mid-episode states x 256
    draws each, pooled per distinct mask row: chi-square p-value > 1e-6, zero-probability
    directions never drawn. Then epsilon: with a greedy action the mask forbids, the greedy
    fraction is binomial(1 - eps)."""
    from scipy.stats import chi2, norm
    B, K = 4096, 256
    env = mazerl.VectorMazeEnv(B, dim, toroidal=tor, enrich=True, seed=99)
    for k in range(12):  # most instances now have >= 2 moves: the 0.25 weight is live
        env.step_act(eps=1.0, seed=5, counter=k)
        env.reset_done()
    m = env.direction_mask(True).clone()
    assert int(((m == 0.25).sum(1) == 1).sum()) > B // 4
    assert bool(((m == 0) | (m == 0.25) | (m == 1)).all())
    counts = torch.zeros(B, 4, dtype=torch.int64, device="cuda")
    ar = torch.arange(B, device="cuda")
    for c in range(K):
        a = env.act(eps=1.0, seed=123, counter=c).long()
        counts[ar, a] += 1
    key = (m * 4).round().long()
    key = key[:, 0] + 5 * key[:, 1] + 25 * key[:, 2] + 125 * key[:, 3]
    stat, dof = 0.0, 0
    for kv in torch.unique(key).tolist():
        sel = key == kv
        row = m[sel][0].double()
        p = (row / row.sum()).cpu().numpy()
        n = counts[sel].sum(0).cpu().numpy().astype(np.float64)
        live = p > 0
        assert n[~live].sum() == 0, (row, n)
        exp = p[live] * n.sum()
        stat += float(((n[live] - exp) ** 2 / exp).sum())
        dof += int(live.sum()) - 1
    assert dof > 0 and chi2.sf(stat, dof) > 1e-6, (stat, dof)
    # epsilon-greedy: sample < eps explores, else the greedy action (dqn_agent.py:104-116)
    blocked = (m == 0).any(1)
    g = torch.argmin(m, 1)  # a direction the exploration never draws where blocked
    eps, hits, tot = 0.37, 0, 0
    for c in range(64):
        a = env.act(eps=eps, greedy=g, seed=321, counter=c).long()
        hits += int((a[blocked] == g[blocked]).sum())
        tot += int(blocked.sum())
    z = (hits - tot * (1 - eps)) / np.sqrt(tot * eps * (1 - eps))
    assert 2 * norm.sf(abs(z)) > 1e-6, (hits, tot)
    env.close()
