"""Maze bank (mz_bank_*): regeneration on win (update_maze, simple_maze_env.py:81-94, driven by
off_policy_trainer.py:190-202) copies mazes generated ahead of time.

Checked bit-exactly: every maze a winner receives is one of the bank's slot mazes, and slot j of
(bank b, algorithm a, first fill) is exactly the maze k_build makes for instance j with seed
bank_seed ^ ((3b + a + 1) << 56) (same generator, same tables); start / goal / max_steps come
with it. Every instance wins after D[start] steps (shortest-path actions from the oracle's BFS
field). Exhausting a bank falls back to building in place; the swap + side-stream refill keeps
serving fresh mazes."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DIM = 21


class Solver:
    """Shortest-path actions from the oracle's BFS distance-to-goal field (test infrastructure),
    recomputed whenever an instance's maze changes; every instance wins after D[start] steps."""

    def __init__(self, env):
        self.env, self.sig, self.dist = env, {}, {}

    def actions(self):
        import pyoracle as O
        env = self.env
        pos = env.pos.cpu().numpy()
        acts = np.zeros(env.num_envs, np.int32)
        for i in range(env.num_envs):
            s = signature(env, i)
            if self.sig.get(i) != s:
                q = env.query(i)
                self.sig[i] = s
                self.dist[i] = O.bfs(env.grid(i), (q["goal_r"], q["goal_c"]))
            d = self.dist[i]
            r, c = pos[i]
            for a, (dr, dc) in enumerate(((1, 0), (-1, 0), (0, 1), (0, -1))):  # ACTIONS order
                nr, nc = r + dr, c + dc
                if 0 <= nr < d.shape[0] and 0 <= nc < d.shape[1] and 0 <= d[nr, nc] < d[r, c]:
                    acts[i] = a
                    break
        return torch.from_numpy(acts).cuda()


def signature(env, i):
    q = env.query(i)
    return env.grid(i).tobytes(), (q["start_r"], q["start_c"], q["goal_r"], q["goal_c"], q["max_steps"])


def slot_mazes(K, key, algo):
    from mazerl import VectorMazeEnv
    ref = VectorMazeEnv(K, DIM, enrich=True, device="cuda", seed=key, algorithm=algo)
    sigs = [signature(ref, j) for j in range(K)]
    ref.close()
    return sigs


def test_bank_serves_generated_slots():
    from mazerl import VectorMazeEnv
    B, K, seed = 48, 64, 0xBA4C0000
    env = VectorMazeEnv(B, DIM, enrich=True, device="cuda", seed=11, algorithm="dfs",
                        done_list=False)
    env.enable_bank(slots=K, swap_every=10 ** 9, algorithms=["dfs"], seed=seed)
    before = [signature(env, i) for i in range(B)]
    won = np.zeros(B, bool)
    solver = Solver(env)
    for _ in range(2000):
        env.step(solver.actions())
        term = env.terminated.cpu().numpy().astype(bool)
        won |= term
        env.reset_done(regen_won=True)
        if won.all():
            break
    assert won.all()
    torch.cuda.synchronize()
    consumed = env.bank_consumed().cpu().numpy()
    assert consumed[1] >= B and consumed[0] == 0 and consumed[2] == 0
    n = int(min(consumed[1], K))
    slots = slot_mazes(K, seed ^ ((3 * 0 + 1 + 1) << 56), "dfs")
    slot_set = {s: j for j, s in enumerate(slots[:n])}
    after = [signature(env, i) for i in range(B)]
    got = set()
    for i in range(B):
        assert after[i] != before[i]
        if consumed[1] <= K:  # no fallback builds: every current maze is a consumed slot
            assert after[i] in slot_set, i
            got.add(slot_set[after[i]])
    if consumed[1] <= K:
        assert len(got) == B  # each slot is handed out once
    env.close()


def test_bank_slots_go_to_winners_in_instance_order():
    """The winners of one reset_done launch take consecutive slots in instance order (k_bank_count
    / k_bank_scan), so the maze each winner receives does not depend on wave scheduling: runs
    from the same seeds are reproducible (and a resumed checkpoint continues exactly)."""
    from mazerl import VectorMazeEnv
    B, K, seed = 48, 64, 0xBA4C0000
    env = VectorMazeEnv(B, DIM, enrich=True, device="cuda", seed=12, algorithm="dfs",
                        done_list=False)
    env.enable_bank(slots=K, swap_every=10 ** 9, algorithms=["dfs"], seed=seed)
    slots = slot_mazes(K, seed ^ ((3 * 0 + 1 + 1) << 56), "dfs")
    solver = Solver(env)
    multi = 0
    for _ in range(2000):
        env.step(solver.actions())
        winners = torch.nonzero(env.terminated).flatten().tolist()
        c0 = int(env.bank_consumed()[1])
        env.reset_done(regen_won=True)
        if winners:
            multi += len(winners) > 1
            for k, i in enumerate(winners):
                if c0 + k < K:
                    assert signature(env, i) == slots[c0 + k], (i, c0 + k)
        if c0 >= K:
            break
    assert multi > 0  # some launch had several winners racing for slots
    env.close()


def test_bank_exhaustion_and_swap_keep_valid_mazes():
    """Tiny banks: most wins fall back to in-place builds; swaps refill on the side stream."""
    from mazerl import VectorMazeEnv
    B = 64
    env = VectorMazeEnv(B, DIM, enrich=True, device="cuda", seed=3, done_list=False)
    env.enable_bank(slots=4, swap_every=3)
    wins = 0
    solver = Solver(env)
    for _ in range(300):
        env.step(solver.actions())
        wins += int(env.terminated.sum())
        env.reset_done(regen_won=True)
    torch.cuda.synchronize()
    assert wins > 2 * B
    for i in range(0, B, 7):
        g = env.grid(i)
        q = env.query(i)
        assert g.shape == (DIM, DIM)
        assert g[q["goal_r"], q["goal_c"]] == 2 and g[q["start_r"], q["start_c"]] != 0
        # perfect maze on the odd lattice: open cells form a tree
        open_ = g != 0
        n_open = int(open_.sum())
        n_edges = int((open_[1:, :] & open_[:-1, :]).sum() + (open_[:, 1:] & open_[:, :-1]).sum())
        assert n_edges == n_open - 1
    env.close()


def test_bank_rejects_bad_arguments():
    from mazerl import VectorMazeEnv, _native as N
    env = VectorMazeEnv(8, DIM, enrich=True, device="cuda", seed=1)
    L = env.lib
    assert L.mz_bank_fill(env._h, 0, 0, None) != 0           # no bank yet
    assert L.mz_bank_create(env._h, 4, 20, 1) != 0           # even size (IndexError in the reference)
    assert L.mz_bank_create(env._h, 4, DIM, 0) != 0          # no algorithm
    assert L.mz_bank_create(env._h, 4, DIM, 1) == 0
    assert L.mz_bank_create(env._h, 4, DIM, 1) != 0          # one bank per handle
    assert L.mz_bank_use(env._h, 2) != 0
    assert L.mz_bank_use(env._h, -1) == 0
    env.close()


def test_multi_size_bank_serves_each_size_its_slots():
    """A bank over several maze sizes (mz_bank_create_dims, the variable-size configs): a winner
    gets a slot maze of its own size — slot j of size index di is exactly the maze k_build makes
    for instance j with seed bank_seed ^ ((3b + a + 1) << 56) ^ (di << 48)."""
    from mazerl.trainers.vector_trainer import make_env
    dims = [15, 19, 23]
    B, K, seed = 48, 32, 0xBA4C0000
    env = make_env(B, dims, algorithm="dfs", seed=5, device="cuda", done_list=False)
    env.enable_bank(slots=K, swap_every=10 ** 9, algorithms=["dfs"], seed=seed, dims=dims)
    size = [env.query(i)["n"] for i in range(B)]
    assert size == [dims[i % 3] for i in range(B)]
    won = np.zeros(B, bool)
    solver = Solver(env)
    for _ in range(3000):
        env.step(solver.actions())
        won |= env.terminated.cpu().numpy().astype(bool)
        env.reset_done(regen_won=True)
        if won.all():
            break
    assert won.all()
    torch.cuda.synchronize()
    consumed = env.bank_consumed().cpu().numpy()
    assert consumed.shape == (3, 3) and consumed[0].sum() == 0 and consumed[2].sum() == 0
    assert (consumed[1] >= B // 3).all()
    for di, dim in enumerate(dims):
        n = int(min(consumed[1, di], K))
        from mazerl import VectorMazeEnv
        ref = VectorMazeEnv(K, dim, enrich=True, device="cuda",
                            seed=seed ^ ((3 * 0 + 1 + 1) << 56) ^ (di << 48), algorithm="dfs")
        slots = {signature(ref, j): j for j in range(n)}
        ref.close()
        for i in range(di, B, 3):
            assert env.query(i)["n"] == dim  # same size after the win (bank or fallback build)
            if consumed[1, di] <= K:
                assert signature(env, i) in slots, (dim, i)
    env.close()


def test_multi_size_bank_rejects_bad_sizes():
    from mazerl import VectorMazeEnv, _native as N
    env = VectorMazeEnv(8, 31, enrich=True, device="cuda", seed=1)
    L = env.lib

    def create(dims):
        arr = (N.C.c_int32 * len(dims))(*dims)
        return L.mz_bank_create_dims(env._h, 4, arr, len(dims), 1)
    assert create([15, 20]) != 0    # even size
    assert create([15, 15]) != 0    # listed twice
    assert create([15, 33]) != 0    # larger than the handle's pitch
    assert create([15, 21, 31]) == 0
    env.close()
