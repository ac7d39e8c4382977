"""The reference trainers' win branch in the vectorised trainers (mazerl/trainers/schedule.py,
VERDICT r4 next 2): change_algorithm (off_policy_trainer.py:302-310, ppo_trainer.py:137-141), the
variable-size envs' +4 growth (simple_variable_maze_env.py:93-112,
toroidal_variable_maze_env.py:113-131) and the max-shape stop (off_policy_trainer.py:210-212,
ppo_trainer.py:104-105).

CPU: the rules on scripted win sequences (a stand-in env records what the schedule hands it).
GPU: the mazes the winners actually receive — their algorithm (each winner's new maze equals the
maze of the expected algorithm built from the same Philox seed), their size (the handle's meta),
an unchanged maze past max_shape, and the trainers stopping once every instance retired."""
import numpy as np
import pytest
import torch


class FakeEnv:
    """What WinSchedule needs of a VectorMazeEnv (CPU tensors)."""

    def __init__(self, B, max_dim=81):
        self.device, self.num_envs, self.max_dim = torch.device("cpu"), B, max_dim
        self.algo_set, self.regen = None, None

    def set_algorithm(self, a):
        self.algo_set = a.clone()

    def set_regen_dims(self, d):
        self.regen = d


def test_global_rule_ranks_wins_in_instance_order():
    from mazerl.trainers.schedule import WinSchedule
    from mazerl.vector_env import ALGOS

    class L:
        eps_decay = 100.0
    env, lr = FakeEnv(8), L()
    s = WinSchedule(env, "global", learner=lr)
    steps = [[0, 1, 0, 1, 0, 0, 0, 0],   # wins 1, 2
             [1, 1, 1, 1, 0, 0, 1, 0],   # wins 3 .. 7: the 5th win (instance 2) -> prim&kill
             [0, 0, 0, 0, 1, 1, 1, 1],   # wins 8 .. 11: the 10th (instance 6) -> dfs
             [1, 0, 0, 0, 0, 0, 0, 0]]   # win 12
    seq = []
    for k, st in enumerate(steps):
        t = torch.tensor(st, dtype=torch.bool)
        s.before_reset(t)
        s.after_reset(t)
        seq.append(s.algo.clone())
    R, P, D = ALGOS["r-prim"], ALGOS["prim&kill"], ALGOS["dfs"]
    assert seq[0].tolist() == [R, R, R, R, R, R, R, R]
    assert seq[1].tolist() == [R, R, P, P, R, R, P, R]
    assert seq[2].tolist() == [R, R, P, P, P, P, D, D]
    assert seq[3].tolist() == [D, R, P, P, P, P, D, D]
    assert int(s.total_wins) == 12 and torch.equal(env.algo_set, seq[3])
    assert float(lr.eps_decay) == 100.0 * 3 * 4
    sm = s.summary()
    assert sm["total_wins"] == 12 and sm["instances_per_algorithm"] == {"r-prim": 1, "dfs": 3,
                                                                         "prim&kill": 4}


def test_global_rule_both_thresholds_in_one_step():
    from mazerl.trainers.schedule import WinSchedule

    class L:
        eps_decay = 10.0
    env, lr = FakeEnv(16), L()
    s = WinSchedule(env, True, learner=lr)
    t = torch.ones(16, dtype=torch.bool)
    s.before_reset(t)
    assert s.algo.tolist() == [0] * 4 + [2] * 5 + [1] * 7  # ids: r-prim 0, dfs 1, prim&kill 2
    assert float(lr.eps_decay) == 120.0


def test_growth_rule_sizes_keep_and_retire():
    """start 15, max 25: 15 -> 19 -> 23; a win at 23 keeps the maze (27 > 25) and never retires;
    start 15, max 23: the win that reaches 23 retires the instance."""
    from mazerl.trainers.schedule import WinSchedule, growth_sizes
    assert growth_sizes(15, 25) == [15, 19, 23] and growth_sizes(17, 79)[-1] == 77
    env = FakeEnv(3, max_dim=25)
    s = WinSchedule(env, None, growth=(15, 25))
    assert env.regen is s.next_dim and s.next_dim.tolist() == [19, 19, 19]
    for won in ([1, 0, 0], [1, 1, 0], [1, 0, 0], [1, 0, 0]):
        t = torch.tensor(won, dtype=torch.bool)
        s.before_reset(t)
        s.after_reset(t)
    assert s.dim.tolist() == [23, 19, 15] and s.next_dim.tolist() == [0, 23, 19]
    assert not s.retired.any() and not s.all_retired()
    # growth without a curriculum rule still counts the wins (summary()["total_wins"])
    assert int(s.total_wins) == 5 and s.inst_wins.tolist() == [4, 1, 0]
    assert s.summary()["total_wins"] == 5
    env2 = FakeEnv(2, max_dim=23)
    s2 = WinSchedule(env2, None, growth=(15, 23))
    for won in ([1, 1], [1, 0]):
        t = torch.tensor(won, dtype=torch.bool)
        s2.before_reset(t)
        s2.after_reset(t)
    assert s2.dim.tolist() == [23, 19] and s2.retired.tolist() == [True, False]
    with pytest.raises(ValueError):
        WinSchedule(FakeEnv(2, 21), None, growth=(15, 22))
    with pytest.raises(ValueError):
        WinSchedule(FakeEnv(2, 21), None, growth=(15, 25))  # beyond the env's pitch
    with pytest.raises(ValueError):
        WinSchedule(FakeEnv(2), "sometimes")


# ------------------------------------------------------------------------------------------ GPU
def _dqn(B, **kw):
    from mazerl.agents.dqn import VectorDQNLearner
    return VectorDQNLearner(B, "cuda:0", variant="dqn", batch_size=128, capacity=1 << 15,
                            eps_decay=40.0, eps_start=1.0, eps_final=1.0, **kw)  # random walks


def _hook(env):
    last = {}
    step_act = env.step_act

    def hooked(*a, **k):
        r = step_act(*a, **k)
        last["term"] = env.terminated.bool().clone()
        last["epoch"] = env.epoch
        return r
    env.step_act = hooked
    return last


@pytest.mark.gpu
def test_global_curriculum_winners_get_the_ranked_algorithm():
    """bank=False: a winner's new maze is built in place from Philox seed env.seed + e +
    (epoch << 32) with its scheduled algorithm — equal to generate() of that algorithm from the
    same seed, for the winners ranked around the 5th and 10th wins."""
    import mazerl
    from mazerl.trainers.vector_trainer import VectorOffPolicyTrainer
    from mazerl.vector_env import ALGOS
    B, dim = 512, 15
    env = mazerl.VectorMazeEnv(B, dim, enrich=True, device="cuda:0", seed=0x5EED0300,
                               window=False, window_bits=True, done_list=False)
    L = _dqn(B)
    tr = VectorOffPolicyTrainer(env, L, seed=5, curriculum="global", bank=False)
    last = _hook(env)
    name = {v: k for k, v in ALGOS.items()}
    total, checked = 0, 0
    for _ in range(200):
        tr.vector_step()
        term = last["term"]
        nw = int(term.sum())
        if nw == 0:
            continue
        winners = torch.nonzero(term).flatten().tolist()
        ranks = list(range(total + 1, total + nw + 1))
        total += nw
        epoch = env.epoch  # reset_done(regen_won) advanced it before building
        for e, k in list(zip(winners, ranks))[:12]:
            want = "dfs" if k >= 10 else ("prim&kill" if k >= 5 else "r-prim")
            assert name[int(tr.algo[e])] == want
            ref = mazerl.VectorMazeEnv(1, dim, enrich=True, device="cuda:0", generate=False,
                                       done_list=False)
            # k_reset_done builds instance e from seed + e + (epoch << 32); generate() builds
            # instance 0 from its seed + 0: pass the whole offset in the seed
            ref.generate(env_ids=[0], algorithm=want,
                         seed=(env.seed + e + (epoch << 32)) & 0xFFFFFFFFFFFFFFFF)
            assert np.array_equal(env.grid(e), ref.grid(0)), (e, k, want)
            ref.close()
            checked += 1
        if total >= 12:
            break
    assert total >= 12 and checked >= 10
    assert int(tr.schedule.total_wins) == total
    assert float(L.eps_decay) == 40.0 * 12
    env.close()


def _solve_step(env, solver, sch):
    """One vector step of the trainers' win branch with shortest-path actions (every instance
    wins after D[start] moves): step, change_algorithm / sizes, reset_done(regen), after_reset."""
    env.step(solver.actions())
    won = env.terminated.bool().clone()
    sch.before_reset(won)
    env.reset_done(regen_won=True)
    sch.after_reset(won)
    return won


@pytest.mark.gpu
def test_growth_sizes_bank_and_max_shape_stop():
    """DQN trainer's schedule, euclidean growth 15 -> 19 -> 23 (max 23) with the maze bank holding
    every size; shortest-path actions so that every instance keeps winning: each instance's
    handle size == the schedule's after every vector step, every instance walks 15, 19, 23 and
    retires on reaching 23; train() stops at its first check once all have retired (the
    reference returns at max shape)."""
    from test_bank import Solver
    from mazerl.trainers.vector_trainer import VectorOffPolicyTrainer, make_env
    B = 48
    env = make_env(B, 15, max_dim=23, seed=0x5EED0400, device="cuda:0", done_list=False,
                   window=False, window_bits=True)
    tr = VectorOffPolicyTrainer(env, _dqn(B), seed=6, growth=(15, 23))
    sch = tr.schedule
    assert env._bank["dims"] == [15, 19, 23]
    solver = Solver(env)
    seen = {i: [15] for i in range(B)}
    for _ in range(3000):
        _solve_step(env, solver, sch)
        n = env.meta()[:, 0]
        assert torch.equal(n, sch.dim), "handle sizes follow the schedule"
        for i, x in enumerate(n.tolist()):
            if seen[i][-1] != x:
                seen[i].append(x)
        if sch.all_retired():
            break
    assert sch.all_retired() and all(v == [15, 19, 23] for v in seen.values())
    tr.train(100)
    assert tr.stopped_at == 32
    env.close()


@pytest.mark.gpu
def test_growth_past_max_keeps_the_maze():
    """max 21 from 15: 15 -> 19, then 23 > 21: a win at 19 keeps the same maze (update_maze's
    `random.shuffle(self.mazes)` branch) and the instance never retires."""
    from test_bank import Solver
    from mazerl.trainers.vector_trainer import VectorOffPolicyTrainer, make_env
    B = 32
    env = make_env(B, 15, max_dim=21, seed=0x5EED0500, device="cuda:0", done_list=False,
                   window=False, window_bits=True)
    tr = VectorOffPolicyTrainer(env, _dqn(B), seed=7, growth=(15, 21))
    sch = tr.schedule
    solver = Solver(env)
    grids, kept = {}, 0
    for _ in range(3000):
        at19 = (sch.dim == 19).cpu().numpy()
        for e in np.nonzero(at19)[0]:
            grids.setdefault(int(e), env.grid(int(e)))
        won = _solve_step(env, solver, sch).cpu().numpy()
        for e, g in grids.items():
            if won[e]:
                assert np.array_equal(env.grid(e), g)  # same maze after the win
                assert int(env.meta()[e, 0]) == 19
                kept += 1
        if kept >= 2 * B:
            break
    assert kept >= 2 * B and not sch.retired.any()
    env.close()


@pytest.mark.gpu
def test_ppo_growth_and_curriculum_config5_shape():
    """VectorPPOTrainer on config 5's toroidal envs in growth mode (17 -> 21 -> 25, every size in a
    best-of-6 bank) with the global curriculum: sizes follow the schedule, every algorithm's
    mazes appear, and the trainer checkpoints and resumes the schedule."""
    from mazerl.trainers.ppo_trainer import VectorPPOTrainer
    from mazerl.trainers.vector_trainer import make_env
    B = 512
    env = make_env(B, 17, max_dim=25, toroidal=True, seed=0x5EED0600, device="cuda:0",
                   done_list=False, reward64=True, window=False, window_bits=True, candidates=6)
    tr = VectorPPOTrainer(env, "cuda:0", batch_size=512, ppo_steps=1, pool_size=4096, seed=3,
                          curriculum="global", growth=(17, 25), bank_candidates=6)
    for _ in range(200):
        tr.vector_step()
        assert torch.equal(env.meta()[:, 0], tr.schedule.dim)
    sm = tr.schedule.summary()
    assert sm["total_wins"] >= 10 and sm["instances_per_algorithm"]["dfs"] > 0
    assert sum(sm["instances_per_size"].values()) == B
    sd = tr.state_dict()
    assert sd["format"] == "mazerl.VectorPPOTrainer/2" and sd["schedule"]["rule"] == "global"
    assert env.select_stats()["unresolved"] == 0
    env.close()
