"""Greedy-row acting (mz_greedy_rows + mz_q_front_rows, agents/fused.py GreedyRows).

The reference draws `sample = random.random()` first and evaluates source_net(state) only when
sample >= eps (dqn_agent.py:104-116). The vectorised learner builds the list of instances whose
epsilon draw of the coming fused act says "greedy" and runs the acting forward over those rows
only. Checked here:
  * the list is exactly the set of instances the fused act (mz_step_act, same eps / seed /
    counter) takes greedy_dev[i] for: every greedy entry is set to a sentinel action (7 — the
    step uses 7 & 3, act_out reports 7), so act_out == 7 marks the greedy branch; sorted, no
    duplicates, count on the device == host count; partial last block (B not a multiple of 1024),
    scalar eps, eps 0 / 1;
  * the row-indexed stem writes, bit for bit, the listed rows of the full stem (no dropout: the
    DQN stem; the per-row computation does not depend on the row's position);
  * GreedyRows' argmax equals the argmax of the full forward on the listed rows wherever the Q
    margin exceeds bf16 GEMM rounding (the GEMM row count differs, so accumulation order may).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _env(B, dim=21, seed=0x5EED0000):
    import mazerl
    return mazerl.VectorMazeEnv(B, dim, enrich=True, device="cuda:0", seed=seed, window=False,
                                window_bits=True, done_list=False)


def _rows(eps, seed, counter, n):
    from mazerl.agents.fused import GreedyRows
    gr = GreedyRows(n, torch.device("cuda", 0))
    k = gr.select(eps, seed, counter)
    torch.cuda.synchronize()
    return gr, k


@pytest.mark.parametrize("B", [1, 1000, 5000, 32768])
def test_list_is_the_fused_act_greedy_branch(B):
    env = _env(B)
    g = torch.Generator(device="cuda").manual_seed(B)
    for t, eps in enumerate([torch.rand(B, generator=g, device="cuda"), 0.3, 0.0, 1.0]):
        seed, counter = 0xC0FFEE + t, 17 * t + 3
        gr, k = _rows(eps, seed, counter, B)
        rows = gr.rows[:k].long()
        assert int(gr.count.item()) == k
        if k > 1:
            assert bool((rows[1:] > rows[:-1]).all())  # increasing: sorted, unique
        sentinel = torch.full((B,), 7, dtype=torch.int64, device="cuda")
        env.step_act(eps=eps, greedy=sentinel, seed=seed, counter=counter)
        torch.cuda.synchronize()
        took = (env.actions == 7).nonzero().flatten()
        assert torch.equal(took, rows), (B, t, k, took.numel())
        if not torch.is_tensor(eps):
            if eps == 0.0:
                assert k == B
            if eps == 1.0:
                assert k == 0
    env.close()


def test_row_stem_equals_full_stem_rows():
    from mazerl.agents.fused import FusedQ
    from mazerl.agents.nets import QNet
    B = 3000
    env = _env(B)
    for k in range(5):  # some visited cells in the windows
        env.step_act(eps=1.0, seed=5, counter=k)
    torch.manual_seed(0)
    net = QNet(variant="dqn").cuda()
    fq = FusedQ(net, seed=3)
    eps = torch.rand(B, generator=torch.Generator(device="cuda").manual_seed(1), device="cuda")
    gr, k = _rows(eps, 9, 9, B)
    assert 0 < k < B
    full = fq.stem(env.obs6, env.window_bits)
    part = fq.stem(env.obs6, env.window_bits, gr.rows, k)
    torch.cuda.synchronize()
    assert torch.equal(part, full[gr.rows[:k].long()])
    env.close()


def test_greedy_rows_argmax_matches_full_forward():
    from mazerl.agents.fused import FusedQ, GreedyRows
    from mazerl.agents.nets import QNet
    B = 8192
    env = _env(B, dim=41)
    for k in range(7):
        env.step_act(eps=1.0, seed=6, counter=k)
    torch.manual_seed(1)
    net = QNet(variant="dqn").cuda()
    fq = FusedQ(net, seed=3)
    eps = torch.rand(B, generator=torch.Generator(device="cuda").manual_seed(2), device="cuda")
    gr = GreedyRows(B, torch.device("cuda", 0))
    greedy = gr(fq, env.obs6, env.window_bits, eps, 21, 4)
    k = gr.last_count
    rows = gr.rows[:k].long()
    q = fq(env.obs6, env.window_bits).float()[rows]
    top2 = q.topk(2, dim=1).values
    clear = (top2[:, 0] - top2[:, 1]) > 0.02 * top2[:, 0].abs().clamp_min(1e-3)
    assert clear.float().mean() > 0.5
    assert torch.equal(greedy[rows][clear], q.argmax(1)[clear])
    env.close()


def test_trainer_step_uses_greedy_rows():
    """One training vector step through VectorOffPolicyTrainer with the row-list acting path."""
    from mazerl.agents.dqn import VectorDQNLearner
    from mazerl.trainers.vector_trainer import VectorOffPolicyTrainer
    B = 2048
    env = _env(B)
    L = VectorDQNLearner(B, "cuda:0", variant="ddqn", batch_size=256, capacity=1 << 16,
                         eps_decay=50.0)
    tr = VectorOffPolicyTrainer(env, L, seed=3)
    for _ in range(3):
        tr.vector_step()
    torch.cuda.synchronize()
    assert L._rows is not None and 0 < int(L._rows.count[0]) <= B
    assert int((env.actions < 0).sum()) == 0 and int((env.actions > 3).sum()) == 0
    env.close()


def test_best_of_mazes_picks_the_easiest_candidate():
    """best_of_mazes == the reference's generate_maze selection (base_maze_env.py:78-97) over the
    same candidates: min McClendon difficulty, first minimum; evaluate() plays the loaded mazes."""
    import numpy as np
    from mazerl import VectorMazeEnv
    from mazerl.difficulty import maze_difficulty
    from mazerl.trainers.vector_trainer import best_of_mazes
    n, dim, c = 5, 21, 6
    grids, sg, sizes = best_of_mazes(n, dim, "dfs", seed=77, device="cuda:0", candidates=c)
    assert sizes.tolist() == [dim] * n
    ref = VectorMazeEnv(n * c, dim, enrich=True, device="cuda:0", algorithm="dfs", seed=77)
    for k in range(n):
        ds = []
        for j in range(c):
            q = ref.query(k * c + j)
            ds.append(maze_difficulty(ref.grid(k * c + j), (q["start_r"], q["start_c"]),
                                      (q["goal_r"], q["goal_c"])))
        j = int(np.argmin(ds))  # first minimum
        q = ref.query(k * c + j)
        assert np.array_equal(grids[k], ref.grid(k * c + j))
        assert tuple(sg[k]) == (q["start_r"], q["start_c"], q["goal_r"], q["goal_c"])
    ref.close()
    env = VectorMazeEnv(n, dim, enrich=True, device="cuda:0", generate=False, done_list=False)
    env.load_mazes(grids, sg)
    env.reset()
    for k in range(n):
        assert np.array_equal(env.grid(k), grids[k])
    env.close()


def test_best_of_mazes_mixed_algorithms_toroidal_variable_sizes():
    """test(new=True)'s per-maze random algorithm (off_policy_trainer.py:231-233) and the toroidal
    variable-size envs (toroidal_maze_env.py:40-54): each maze's 6 candidates share its size and
    algorithm; the pick is the first minimum of the difficulty of the bordered maze (the host
    restatement here, candidates regenerated one by one); evaluate() loads and plays them."""
    import numpy as np
    import torch
    from mazerl import VectorMazeEnv
    from mazerl.difficulty import toroidal_difficulty
    from mazerl.trainers.vector_trainer import best_of_mazes, load_selected, maze_algorithms
    n, c, dims = 6, 6, [17, 21, 25]
    algos = maze_algorithms(n, seed=5)
    assert algos == maze_algorithms(n, seed=5) and set(algos) <= {"r-prim", "prim&kill", "dfs"}
    grids, sg, sizes = best_of_mazes(n, dims, algos, seed=91, device="cuda:0", candidates=c,
                                     toroidal=True)
    assert sizes.tolist() == [dims[k % 3] for k in range(n)]
    ref = VectorMazeEnv(n * c, 17, toroidal=True, enrich=True, device="cuda:0", max_dim=25,
                        generate=False, done_list=False)
    for k in range(n):
        ds = []
        for j in range(c):
            i = k * c + j
            ref.generate(env_ids=torch.tensor([i], dtype=torch.int32, device="cuda:0"),
                         algorithm=algos[k], dim=int(sizes[k]), seed=91)
            q = ref.query(i)
            assert q["n"] == sizes[k]
            ds.append(toroidal_difficulty(ref.grid(i), (q["start_r"], q["start_c"]),
                                          (q["goal_r"], q["goal_c"])))
        j = int(np.argmin(ds))
        q = ref.query(k * c + j)
        m = int(sizes[k])
        assert np.array_equal(grids[k, :m, :m], ref.grid(k * c + j))
        assert tuple(sg[k]) == (q["start_r"], q["start_c"], q["goal_r"], q["goal_c"])
    ref.close()
    env = VectorMazeEnv(n, 17, toroidal=True, enrich=True, device="cuda:0", max_dim=25,
                        generate=False, done_list=False)
    load_selected(env, (grids, sg, sizes))
    for k in range(n):
        m = int(sizes[k])
        assert np.array_equal(env.grid(k), grids[k, :m, :m])
    env.close()


def test_curriculum_change_algorithm_per_instance():
    """VectorOffPolicyTrainer(curriculum="per-instance"): NeuralOffPolicyTrainer.change_algorithm
    (off_policy_trainer.py:302-310, on every win) per instance — epsilon_decay * 3 at the 5th win
    and * 4 at the 10th, the algorithm prim&kill from the 5th win and dfs from the 10th; steps_done
    = 0 on every win. Wins are recounted here from each step's terminated flags."""
    from mazerl.agents.dqn import VectorDQNLearner
    from mazerl.trainers.vector_trainer import VectorOffPolicyTrainer
    from mazerl.vector_env import ALGOS
    B, base = 1024, 40.0
    env = _env(B, dim=15)
    L = VectorDQNLearner(B, "cuda:0", variant="dqn", batch_size=128, capacity=1 << 15,
                         eps_decay=base, eps_start=1.0, eps_final=1.0)  # random walks: many wins
    tr = VectorOffPolicyTrainer(env, L, seed=5, curriculum="per-instance")
    wins = torch.zeros(B, dtype=torch.int32, device="cuda:0")
    last = {}
    step_act = env.step_act

    def hooked(*a, **k):  # the step's flags (the auto-reset that follows clears them)
        r = step_act(*a, **k)
        last["term"] = env.terminated.bool().clone()
        return r
    env.step_act = hooked
    for _ in range(400):
        tr.vector_step()
        term = last["term"]
        wins += term.to(torch.int32)
        assert torch.equal(L.steps_done[term], torch.zeros_like(L.steps_done[term]))
    torch.cuda.synchronize()
    assert torch.equal(tr.inst_wins, wins) and int(wins.sum()) > 0
    assert torch.equal(tr.schedule.inst_wins, wins)

    def expect(w):
        mult = torch.where(w >= 10, 12.0, torch.where(w >= 5, 3.0, 1.0))
        algo = torch.where(w >= 10, ALGOS["dfs"], torch.where(w >= 5, ALGOS["prim&kill"],
                                                              ALGOS["r-prim"]))
        return base * mult, algo.long()
    d, a = expect(wins)
    assert torch.equal(L.eps_decay, d) and torch.equal(tr.algo.long(), a)
    # the thresholds themselves, on scripted wins: instance i wins in round k iff k < i % 13
    sch = tr.schedule
    sch.inst_wins.zero_()
    sch.algo.fill_(ALGOS["r-prim"])
    sch.maze_algo.fill_(ALGOS["r-prim"])
    L.eps_decay = base
    idx = torch.arange(B, device="cuda:0")
    for k in range(12):
        won = k < idx % 13
        sch.before_reset(won)
        sch.after_reset(won)
    w = (idx % 13).clamp(max=12).to(torch.int32)
    d, a = expect(w)
    assert torch.equal(sch.inst_wins, w) and torch.equal(L.eps_decay, d)
    assert torch.equal(tr.algo.long(), a)
    env.close()
