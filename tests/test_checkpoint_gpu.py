"""Checkpoint / resume on the GPU (mz_state_save / mz_state_load, mazerl/checkpoint.py).

* env: a VectorMazeEnv saved mid-run (mazes, BFS tables, visit counts and tags, visited planes,
  per-instance state, both maze banks mid-rotation) and loaded into an env built from other seeds
  steps on bit-identically: observations, window bits, rewards, flags, regenerated mazes.
* trainer: a DDQN VectorOffPolicyTrainer checkpointed to a file between two train() calls and
  resumed in a fresh trainer (other seeds, other construction order, no captured graphs yet)
  continues exactly as the saved one: same Q-net parameters, counters and env state after the
  next vector steps (side-stream updates, graph replays, greedy-row acting, maze bank included).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _best_action(env):
    """The action toward the cell the env's "best dir" points at (best_dir = agent - next)."""
    dr, dc = -env.best_dir[:, 0], -env.best_dir[:, 1]
    return torch.where(dr == 1, 0, torch.where(dr == -1, 1, torch.where(dc == 1, 2, 3)))


def _env(seed):
    from mazerl import VectorMazeEnv
    env = VectorMazeEnv(512, 21, enrich=True, device="cuda", seed=seed, done_list=False,
                        window=True, window_bits=True)
    env.enable_bank(slots=48, swap_every=4)
    return env


def _run(env, k0, n, record):
    out = []
    for k in range(k0, k0 + n):
        env.step_act(eps=0.3, greedy=_best_action(env), seed=9, counter=k)
        if record:  # the step's outputs (reset_done clears the flags of the instances it resets)
            out.append([t.clone() for t in (env.reward, env.terminated, env.truncated, env.actions)])
        env.reset_done(regen_won=True)
        if record:
            out[-1] += [t.clone() for t in (env.obs6, env.window_bits, env.window)]
    torch.cuda.synchronize()
    return out


def test_env_resume_is_bit_exact():
    A = _env(0x5EED0000)
    _run(A, 0, 30, False)
    sd = A.state_dict()
    ra = _run(A, 30, 45, True)
    wins = sum(int(r[1].sum()) for r in ra)
    assert wins > 50  # maze regenerations (bank copies, rotations, refills) happen in the window
    B = _env(0xB0B)
    assert not torch.equal(A.obs6, B.obs6)
    B.load_state_dict(sd)
    rb = _run(B, 30, 45, True)
    for k, (x, y) in enumerate(zip(ra, rb)):
        for i, (u, v) in enumerate(zip(x, y)):
            assert torch.equal(u, v), (k, i)
    for i in (0, 7, 311, 511):
        assert A.query(i) == B.query(i)
        assert (A.grid(i) == B.grid(i)).all()
    assert A._bank["calls"] == B._bank["calls"] and A._bank["cur"] == B._bank["cur"]
    assert torch.equal(A.bank_consumed(), B.bank_consumed())
    A.close()
    B.close()


def test_env_state_rejects_another_shape():
    from mazerl import VectorMazeEnv
    A = _env(1)
    sd = A.state_dict()
    C = VectorMazeEnv(256, 21, enrich=True, device="cuda", seed=2)
    C.enable_bank(slots=48, swap_every=4)
    with pytest.raises(ValueError):
        C.load_state_dict(sd)
    D = VectorMazeEnv(512, 21, enrich=True, device="cuda", seed=2)  # no bank
    with pytest.raises(ValueError):
        D.load_state_dict(sd)
    for e in (A, C, D):
        e.close()


def _trainer(env_seed, seed):
    from mazerl import VectorMazeEnv
    from mazerl.agents.dqn import VectorDQNLearner
    from mazerl.trainers.vector_trainer import VectorOffPolicyTrainer
    B = 2048
    env = VectorMazeEnv(B, 21, enrich=True, device="cuda", seed=env_seed, done_list=False,
                        window=False, window_bits=True)
    L = VectorDQNLearner(B, "cuda:0", variant="ddqn", batch_size=128, capacity=1 << 15,
                         eps_decay=60.0, target_every=5, updates_per_epoch=7, overlap=True,
                         seed=seed)
    return VectorOffPolicyTrainer(env, L, seed=seed + 1)


def test_trainer_resume_is_bit_exact(tmp_path):
    from mazerl.checkpoint import load_checkpoint, save_checkpoint
    A = _trainer(0xA11CE, 3)
    A.train(25)
    path = save_checkpoint(str(tmp_path / "run.pt"), A)
    A.train(15)
    B = _trainer(0x5EED, 8)
    load_checkpoint(path, B)
    B.train(15)
    torch.cuda.synchronize()
    assert A.learner.n_updates == B.learner.n_updates > 30
    assert A.counter == B.counter == 40
    assert int(A.wins) == int(B.wins) and int(A.episodes) == int(B.episodes)
    for (ka, pa), (kb, pb) in zip(A.learner.source.state_dict().items(),
                                  B.learner.source.state_dict().items()):
        assert torch.equal(pa, pb), ka
    for pa, pb in zip(A.learner.target.parameters(), B.learner.target.parameters()):
        assert torch.equal(pa, pb)
    assert torch.equal(A.learner.steps_done, B.learner.steps_done)
    assert torch.equal(A.env.obs6, B.env.obs6) and torch.equal(A.env.window_bits, B.env.window_bits)
    ra, rb = A.learner.replay, B.learner.replay
    assert (ra.ptr, ra.size) == (rb.ptr, rb.size)
    assert torch.equal(ra.sw[:ra.size], rb.sw[:rb.size]) and torch.equal(ra.a[:ra.size], rb.a[:rb.size])
    A.env.close()
    B.env.close()


def _ppo(seed):
    from mazerl.trainers.ppo_trainer import VectorPPOTrainer
    from mazerl.trainers.vector_trainer import make_env
    env = make_env(512, [17, 21, 25, 29], toroidal=True, device="cuda", seed=0x70500000 + seed,
                   done_list=False, reward64=True, window=False, window_bits=True)
    return VectorPPOTrainer(env, "cuda", hidden_dim=256, batch_size=512, ppo_steps=2,
                            pool_size=4096, seed=seed)


def test_ppo_trainer_resume_is_bit_exact(tmp_path):
    """Config 5's trainer (on-device rollout, episode records, the update pool, the captured
    minibatch step, a maze bank per size) resumed from a file continues exactly."""
    from mazerl.checkpoint import load_checkpoint, save_checkpoint
    A = _ppo(1)
    A.train(40)
    assert A.updates > 0
    path = save_checkpoint(str(tmp_path / "ppo.pt"), A)
    A.train(30)
    B = _ppo(2)
    load_checkpoint(path, B)
    B.train(30)
    torch.cuda.synchronize()
    assert A.updates == B.updates and A.counter == B.counter and A.consumed == B.consumed
    assert torch.equal(A.stats, B.stats) and torch.equal(A.t, B.t)
    for (ka, pa), (kb, pb) in zip(A.net.state_dict().items(), B.net.state_dict().items()):
        assert torch.equal(pa, pb), ka
    assert torch.equal(A.env.obs6, B.env.obs6) and torch.equal(A.env.window_bits, B.env.window_bits)
    fill = int(A.pool_fill)
    assert fill == int(B.pool_fill) and torch.equal(A.p_w[:fill], B.p_w[:fill])
    A.env.close()
    B.env.close()
