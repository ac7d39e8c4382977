#!/usr/bin/env python3
"""Fixtures for the tabular Q-agent (config 1) and PPO (config 5) from the reference's own code:
agents/q_agent.py:8-79 driven by gymnasium_env SimpleMazeEnv on a golden 9x9 maze, and
agents/ppo_agent.py:13-237 (returns, advantages, evaluate, optimize_model on a small net).

Test infrastructure only (build container). Writes tests/golden/agents.npz (data only).
"""
import contextlib
import io
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import golden_io as G  # noqa: E402
import learner_util as U  # noqa: E402

PPO_T, PPO_BATCH, PPO_STEPS, PPO_COEF = 8, 4, 2, 0.01
PPO_REWARDS = [0.45, -0.55, -0.05, -0.18126924692201818, 0.45, 0.45, -1, 1]


def ppo_inputs():
    rng = np.random.default_rng(77)
    s6 = rng.random((PPO_T, 6)).astype(np.float32)
    w = rng.integers(0, 2, (PPO_T, 3, 15, 15)).astype(np.float32)
    a = rng.integers(0, 4, (PPO_T, 1)).astype(np.int64)
    lp = (-rng.random((PPO_T, 1)) * 2).astype(np.float32)
    adv = rng.standard_normal(PPO_T).astype(np.float32)
    ret = rng.standard_normal(PPO_T).astype(np.float32)
    vals = rng.standard_normal(PPO_T).astype(np.float32)
    return s6, w, a, lp, adv, ret, vals


# a pool of whole episodes for the vectorised trainer's on-device finishing (mz_ppo_scan /
# mz_ppo_finish): lengths incl. 1-step episodes (NaN returns in the reference: torch.std of one
# element) and one longer than the kernel's 2,048-reward LDS chunk
POOL_LENS = [1, 2, 3, 7, 1, 40, 12, 2, 150, 5, 2600, 9]


def pool_episodes():
    """Rewards from the env's reward set (base_maze_env.py:183-208: new cell 0.45 / -0.55 /
    toroidal -0.05, revisit -(1 - exp(-0.2 k)), invalid move -(1 - exp(-0.15 k)), win 1,
    truncation -1) and critic values per episode."""
    import math
    rng = np.random.default_rng(2024)
    eps = []
    for n in POOL_LENS:
        r = []
        for t in range(n):
            c = rng.integers(0, 6)
            if c == 0:
                r.append(0.45)
            elif c == 1:
                r.append(-0.55)
            elif c == 2:
                r.append(-0.05)
            elif c == 3:
                r.append(0.0 - (1 - math.exp(-0.2 * int(rng.integers(1, 300)))))
            elif c == 4:
                r.append(0.0 - (1 - math.exp(-0.15 * int(rng.integers(1, 300)))))
            else:
                r.append(0.45)
        r[-1] = 1 if rng.random() < 0.5 else -1  # the last step: a win or a truncation
        v = rng.standard_normal(n).astype(np.float32)
        eps.append((r, v))
    return eps


def main(ref="/root/reference"):
    sys.path.insert(0, HERE)
    import _refstubs
    _refstubs.install()
    sys.dont_write_bytecode = True
    sys.path.insert(0, ref)
    from agents import ppo_agent, q_agent
    from gymnasium_env.envs import simple_maze_env
    torch.set_num_threads(1)
    out = {}

    # ---- Q-agent on a golden 9x9 plain trace ---------------------------------------------
    t = [t for t in G.traces() if t["kind"] == G.KIND_SIMPLE][0]
    grid = [list(map(int, r)) for r in t["grid"]]
    fixed = lambda self, shape: (t["start"], t["goal"], [r[:] for r in grid])  # noqa: E731
    Env = type("FixedEnv", (simple_maze_env.SimpleMazeEnv,), {"generate_maze": fixed})
    env = Env((t["n"], t["n"]))
    agent = q_agent.QAgent(env, learning_rate=0.1, initial_epsilon=0.95, epsilon_decay=40,
                           final_epsilon=0.05, discount_factor=0.7, eta=0.01)
    obs, _ = env.reset()
    seq = {"obs": [], "act": [], "rew": [], "term": [], "next": []}
    for op in t["op"][:600]:
        if op == 4:
            obs, _ = env.reset()
            continue
        nobs, r, tr, te, _ = env.step(int(op))
        agent.update(obs, int(op), r, te, nobs)
        seq["obs"].append(str(obs)); seq["act"].append(int(op)); seq["rew"].append(float(r))
        seq["term"].append(bool(te)); seq["next"].append(str(nobs))
        obs = nobs
    keys = sorted(agent.q_values)
    out["q.trace_index"] = np.int64(0)
    out["q.obs"] = np.array(seq["obs"]); out["q.next"] = np.array(seq["next"])
    out["q.act"] = np.array(seq["act"]); out["q.rew"] = np.array(seq["rew"])
    out["q.term"] = np.array(seq["term"])
    out["q.keys"] = np.array(keys)
    out["q.values"] = np.stack([agent.q_values[k] for k in keys])

    # ---- PPO -------------------------------------------------------------------------------
    s6, w, a, lp, adv, ret, vals = ppo_inputs()
    net = ppo_agent.ActorCriticNet(3, 6, 4, 4, hidden_dim=8)
    U.fill_params(net, 101)

    class Holder:  # the parts of PPOAgent that optimize_model/calculate_* use
        pass
    h = Holder()
    h.gamma, h.batch_size, h.ppo_steps, h.agent = 0.9, PPO_BATCH, PPO_STEPS, net
    h.actor_lr, h.critic_lr = 3e-4, 1e-4
    h.optimizer = torch.optim.AdamW([
        {"params": net.actor_head.parameters(), "lr": h.actor_lr},
        {"params": net.critic_head.parameters(), "lr": h.critic_lr},
        {"params": net.conv.parameters(), "lr": (h.actor_lr + h.critic_lr) / 2}])
    P = ppo_agent.PPOAgent
    out["ppo.returns"] = P.calculate_returns(h, PPO_REWARDS).numpy()
    out["ppo.advantages"] = P.calculate_advantages(h, torch.from_numpy(ret), torch.from_numpy(vals)).numpy()
    st = (torch.from_numpy(s6), torch.from_numpy(w))
    lpn, val, ent = net.evaluate(st, torch.from_numpy(a))
    out["ppo.eval_logp"] = lpn.detach().numpy()
    out["ppo.eval_value"] = val.detach().numpy()
    out["ppo.eval_entropy"] = ent.detach().numpy()
    h.calculate_surrogate_loss = lambda *x, **k: P.calculate_surrogate_loss(h, *x, **k)
    h.calculate_loss = lambda *x, **k: P.calculate_loss(h, *x, **k)
    with contextlib.redirect_stdout(io.StringIO()):
        P.optimize_model(h, st, torch.from_numpy(a), torch.from_numpy(lp), torch.from_numpy(adv),
                         torch.from_numpy(ret), PPO_COEF)
    for k, p in sorted(net.named_parameters()):
        out[f"ppo.param.{k}"] = p.data.numpy().copy()
    # per-episode returns / advantages of the pool episodes (do_episode's tail, :166-167)
    rew, val, rets, advs = [], [], [], []
    for r, v in pool_episodes():
        R = P.calculate_returns(h, r)
        A = P.calculate_advantages(h, R, torch.from_numpy(v))
        rew.append(np.array(r, np.float64)); val.append(v)
        rets.append(R.numpy().astype(np.float32)); advs.append(A.numpy().astype(np.float32))
    out["ppo.pool.lens"] = np.array(POOL_LENS, np.int64)
    out["ppo.pool.rewards"] = np.concatenate(rew)
    out["ppo.pool.values"] = np.concatenate(val)
    out["ppo.pool.returns"] = np.concatenate(rets)
    out["ppo.pool.advantages"] = np.concatenate(advs)
    out["ppo.pool.gamma"] = np.float64(h.gamma)
    np.savez_compressed(os.path.join(HERE, "agents.npz"), **out)
    print("q keys", len(keys), "ppo returns", out["ppo.returns"][:3])


if __name__ == "__main__":
    main(*sys.argv[1:])
