"""Best-of-C mazes on the GPU for the vectorised trainers: the reference hands
its agent the easiest of six candidates by McClendon difficulty for every new maze
(BaseMazeEnv.generate_maze, base_maze_env.py:78-97; toroidal_maze_env.py:40-54, scored on the
bordered maze) — the env's first maze and every win's update_maze (off_policy_trainer.py:202,
ppo_trainer.py:96). Here both the initial mazes (mz_generate_best) and a maze bank's refilled
slots (mz_bank_create_ex, candidates = 6) are chosen by k_mcclendon + k_cand_select inside the
launch sequence, and checked against best_of_mazes — the same candidates scored with the host's
glibc log, argmin = the reference's first minimum (tests/test_greedy_rows.py pins best_of_mazes
to the host restatement, which tests/test_difficulty.py pins to the reference's values)."""
import numpy as np
import pytest
import torch

from test_bank import Solver

pytestmark = pytest.mark.gpu


def bank_key(seed, bank, algo, di=0):
    """mz_bank_fill's Philox key of a (bank, algorithm, size index) block."""
    return (seed ^ ((3 * bank + algo + 1) << 56) ^ (di << 48)) & 0xFFFFFFFFFFFFFFFF


def assert_bank_block(env, bank, algo, dim, di, slots, seed, epoch, toroidal=False):
    from mazerl.trainers.vector_trainer import best_of_mazes
    from mazerl.vector_env import ALGOS
    a = ALGOS[algo]
    key = (bank_key(seed, bank, a, di) + (epoch << 32)) & 0xFFFFFFFFFFFFFFFF
    grids, sg, _ = best_of_mazes(len(slots), dim, algo, seed=key, device="cuda:0", candidates=6,
                                 toroidal=toroidal)
    for k, j in enumerate(slots):
        g, info = env.bank_slot(bank, algo, dim, j)
        assert np.array_equal(g, grids[k, :dim, :dim]), (bank, algo, dim, j)
        assert info == tuple(int(x) for x in sg[k]), (bank, algo, dim, j)


def test_generate_best_matches_best_of_mazes():
    """VectorMazeEnv(candidates=6): instance e holds best_of_mazes' maze e (candidate c of maze e
    = Philox seed + 6 e + c), euclidean 21 x 21 and 81 x 81 (the headline's size)."""
    from mazerl import VectorMazeEnv
    from mazerl.trainers.vector_trainer import best_of_mazes
    for n, dim, algo in ((24, 21, "dfs"), (12, 81, "r-prim"), (12, 41, "prim&kill")):
        env = VectorMazeEnv(n, dim, enrich=True, device="cuda:0", seed=0x5EED0077, algorithm=algo,
                            done_list=False, candidates=6)
        grids, sg, _ = best_of_mazes(n, dim, algo, seed=0x5EED0077, device="cuda:0", candidates=6)
        for e in range(n):
            q = env.query(e)
            assert np.array_equal(env.grid(e), grids[e]), (dim, e)
            assert (q["start_r"], q["start_c"], q["goal_r"], q["goal_c"]) == tuple(sg[e])
            assert (q["r"], q["c"]) == (q["start_r"], q["start_c"]) and q["steps"] == 0
        st = env.select_stats()
        assert st["groups"] == n and st["unresolved"] == 0 and st["near_ties"] == 0
        env.close()


def test_generate_best_variable_size_toroidal_make_env():
    """make_env(candidates=6) over toroidal sizes (config 5's variable-size envs): instance i of
    size dims[i % 3] holds best_of_mazes' maze i (scored as the bordered maze)."""
    from mazerl.trainers.vector_trainer import best_of_mazes, make_env
    n, dims = 18, [17, 21, 29]
    env = make_env(n, dims, toroidal=True, algorithm="prim&kill", seed=0x5EED0100,
                   device="cuda:0", done_list=False, candidates=6)
    grids, sg, sizes = best_of_mazes(n, dims, "prim&kill", seed=0x5EED0100, device="cuda:0",
                                     candidates=6, toroidal=True)
    for e in range(n):
        m = int(sizes[e])
        q = env.query(e)
        assert q["n"] == m
        assert np.array_equal(env.grid(e), grids[e, :m, :m]), e
        assert (q["start_r"], q["start_c"], q["goal_r"], q["goal_c"]) == tuple(sg[e])
    assert env.select_stats()["unresolved"] == 0
    env.close()


def test_best_of_bank_first_fill_matches_best_of_mazes():
    """enable_bank(candidates=6): slot j of every (bank, algorithm) block's first fill is
    best_of_mazes' maze j for the block's Philox key (the candidates a C = 1 bank would build for
    slots 6 j .. 6 j + 5)."""
    from mazerl import VectorMazeEnv
    B, K, dim, seed = 32, 10, 21, 0xBA4C0011
    env = VectorMazeEnv(B, dim, enrich=True, device="cuda:0", seed=7, algorithm="r-prim",
                        done_list=False)
    env.enable_bank(slots=K, swap_every=10 ** 9, algorithms=["r-prim", "dfs", "prim&kill"],
                    seed=seed, candidates=6)
    torch.cuda.synchronize()
    for bank in (0, 1):
        for algo in ("r-prim", "dfs", "prim&kill"):
            assert_bank_block(env, bank, algo, dim, 0, range(K), seed, 0)
    st = env.select_stats()
    assert st["groups"] == 2 * 3 * K and st["unresolved"] == 0 and st["near_ties"] == 0
    env.close()


def test_best_of_bank_refill_rebuilds_consumed_slots_only():
    """A refill (epoch 1) rebuilds exactly the consumed slots [0, used) as best-of-6 mazes of the
    epoch-1 keys (the difficulty launch and the selection read the consumed count on the device)
    and leaves the others; winners receive the slots in instance order."""
    from mazerl import VectorMazeEnv
    from mazerl.vector_env import _ptr
    import mazerl._native as N
    B, K, dim, seed = 48, 40, 15, 0xBA4C0022
    env = VectorMazeEnv(B, dim, enrich=True, device="cuda:0", seed=9, algorithm="dfs",
                        done_list=False)
    env.enable_bank(slots=K, swap_every=10 ** 9, algorithms=["dfs"], seed=seed, candidates=6)
    torch.cuda.synchronize()
    before = [env.bank_slot(0, "dfs", dim, j) for j in range(K)]
    solver = Solver(env)
    used = 0
    for _ in range(400):
        env.step(solver.actions())
        env.reset_done(regen_won=True)
        used = int(env.bank_consumed()[1])
        if used >= 3:
            break
    assert 0 < used < K
    N.check(env.lib.mz_bank_fill(env._h, 0, seed, env._stream()))
    torch.cuda.synchronize()
    assert_bank_block(env, 0, "dfs", dim, 0, range(used), seed, 1)
    for j in range(used, K):
        g, info = env.bank_slot(0, "dfs", dim, j)
        assert np.array_equal(g, before[j][0]) and info == before[j][1]
    assert int(env.bank_consumed()[1]) == 0
    env.close()


def test_best_of_bank_multi_size_toroidal():
    """A toroidal bank over several sizes with best-of-6 slots (config 5's variable-size envs):
    size index di keys its slots with di << 48 and scores the bordered mazes."""
    from mazerl.trainers.vector_trainer import make_env
    dims, K, seed = [17, 25], 6, 0xBA4C0033
    env = make_env(16, dims, toroidal=True, algorithm="r-prim", seed=5, device="cuda:0",
                   done_list=False)
    env.enable_bank(slots=K, swap_every=10 ** 9, algorithms=["r-prim"], seed=seed, dims=dims,
                    candidates=6)
    torch.cuda.synchronize()
    for di, dim in enumerate(dims):
        assert_bank_block(env, 0, "r-prim", dim, di, range(K), seed, 0, toroidal=True)
    env.close()


def test_best_of_bank_rejects_bad_candidates():
    from mazerl import VectorMazeEnv, _native as N
    env = VectorMazeEnv(8, 21, enrich=True, device="cuda:0", seed=1)
    arr = (N.C.c_int32 * 1)(21)
    assert env.lib.mz_bank_create_ex(env._h, 4, arr, 1, 1, 0) != 0
    assert env.lib.mz_bank_create_ex(env._h, 4, arr, 1, 1, 65) != 0
    assert env.lib.mz_generate_best(env._h, None, 8, None, 0, 21, 1, 0, None) != 0
    assert env.lib.mz_bank_create_ex(env._h, 4, arr, 1, 1, 6) == 0
    env.close()
    big = VectorMazeEnv(4, 101, enrich=True, device="cuda:0", seed=1, generate=False)
    arr = (N.C.c_int32 * 1)(101)
    assert big.lib.mz_bank_create_ex(big._h, 4, arr, 1, 1, 6) == -2  # beyond the LDS plan
    assert big.lib.mz_bank_create_ex(big._h, 4, arr, 1, 1, 1) == 0   # one candidate: no scoring
    big.close()


# ---- the screen -> exact -> host pipeline (mz_screen.hip, k_cand_pick, k_cand_select) ---------
def _gen(n, dim, algo, seed, dbg):
    from mazerl import VectorMazeEnv
    env = VectorMazeEnv(n, dim, enrich=True, device="cuda:0", seed=seed, generate=False,
                        done_list=False)
    env.set_debug(dbg)
    env.select_stats(reset=True)
    env.generate(algorithm=algo, dim=dim, seed=seed, candidates=6)
    torch.cuda.synchronize()
    return env


def test_screen_decides_and_matches_exact_path():
    """The screen's picks == every group through the order-exact kernel (debug flag 1) == the
    host-log argmin of best_of_mazes; without the flag no group needs the exact kernel."""
    from mazerl.trainers.vector_trainer import best_of_mazes
    for n, dim, algo in ((40, 81, "r-prim"), (40, 81, "dfs"), (40, 41, "prim&kill")):
        seed = 0x5C2EE0 + dim
        a = _gen(n, dim, algo, seed, 0)
        b = _gen(n, dim, algo, seed, 1)
        grids, sg, _ = best_of_mazes(n, dim, algo, seed=seed, device="cuda:0", candidates=6)
        for e in range(n):
            assert np.array_equal(a.grid(e), grids[e]) and np.array_equal(b.grid(e), grids[e]), e
            qa, qb = a.query(e), b.query(e)
            assert qa == qb and (qa["start_r"], qa["start_c"], qa["goal_r"], qa["goal_c"]) == tuple(sg[e])
        sa, sb = a.select_stats(), b.select_stats()
        assert sa["groups"] == n and sa["exact"] == 0 and sa["unresolved"] == 0, sa
        assert sb["groups"] == n and sb["exact"] == n and sb["unresolved"] == 0, sb
        a.close()
        b.close()


def test_screen_cannot_decide_identical_candidates_exact_path_keeps_the_first():
    """All six candidates of a group from one seed (debug flag 4): equal difficulties, which no
    bound can separate — the group goes to the exact kernel, whose first-minimum rule keeps
    candidate 0 (the reference replaces only on a strict `<`): the maze of seed + 6 e."""
    from mazerl import VectorMazeEnv
    n, dim, seed = 24, 41, 0x71A5
    env = _gen(n, dim, "r-prim", seed, 4)
    ref = VectorMazeEnv(6 * n, dim, enrich=True, device="cuda:0", seed=seed, algorithm="r-prim",
                        done_list=False)
    for e in range(n):
        assert np.array_equal(env.grid(e), ref.grid(6 * e)), e
    st = env.select_stats()
    assert st["exact"] == n and st["unresolved"] == 0 and st["near_ties"] == 0, st
    env.close()
    ref.close()


def test_declined_candidates_are_scored_on_the_host():
    """Candidates the exact kernel declines (forced for every even-numbered one, debug flags
    1 | 2) are scored by the host restatement inside the stream: the selection is still the
    first minimum over all six (best_of_mazes), none unresolved."""
    from mazerl.trainers.vector_trainer import best_of_mazes
    n, dim, seed = 30, 33, 0xDEC1
    env = _gen(n, dim, "dfs", seed, 3)
    grids, sg, _ = best_of_mazes(n, dim, "dfs", seed=seed, device="cuda:0", candidates=6)
    for e in range(n):
        assert np.array_equal(env.grid(e), grids[e]), e
    st = env.select_stats()
    assert st["exact"] == n and st["host_scored"] == 3 * n and st["unresolved"] == 0, st
    env.close()


def test_bank_slots_with_host_scored_candidates():
    """A best-of-6 bank whose refill has its even candidates declined (host-scored): every slot
    equals the reference's first minimum over the six candidates (best_of_mazes)."""
    from mazerl import VectorMazeEnv
    B, K, dim, seed = 32, 12, 21, 0xBA4C0044
    env = VectorMazeEnv(B, dim, enrich=True, device="cuda:0", seed=3, algorithm="r-prim",
                        done_list=False)
    env.set_debug(3)
    env.select_stats(reset=True)
    env.enable_bank(slots=K, swap_every=10 ** 9, algorithms=["r-prim", "prim&kill"], seed=seed,
                    candidates=6)
    torch.cuda.synchronize()
    for algo in ("r-prim", "prim&kill"):
        assert_bank_block(env, 0, algo, dim, 0, range(K), seed, 0)
        assert_bank_block(env, 1, algo, dim, 0, range(K), seed, 0)
    st = env.select_stats()
    assert st["groups"] == 4 * K and st["host_scored"] == 4 * K * 3 and st["unresolved"] == 0, st
    env.close()
