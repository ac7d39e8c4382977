#!/usr/bin/env python3
"""Q-loss parity fixtures from the reference's own DQNAgent/DDQNAgent.optimize_model
(agents/dqn_agent.py:121-157, agents/ddqn_agent.py:113-152), run here on CPU with fp32.

Test infrastructure only (build container). Writes tests/golden/learner.npz (outputs only; the
inputs are regenerated from seeds by tests/learner_util.py):
  <case>.loss, <case>.grad_sum/grad_abs (per parameter, after clamp_(-1,1)),
  <case>.param_sum/param_abs (after one AdamW step), and for the small nets the full tensors.
"""
import os
import random
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))  # tests/
import learner_util as U  # noqa: E402


class FakeEnv:
    """What the agents read from an env at construction: action_space.n and reset()."""

    class _A:
        n = 4

    action_space = _A()

    def reset(self):
        return {"agent": np.zeros(2), "target": np.zeros(2), "best dir": np.zeros(2)}, {}


def main(ref="/root/reference"):
    sys.path.insert(0, HERE)
    import _refstubs
    _refstubs.install()
    sys.dont_write_bytecode = True
    sys.path.insert(0, ref)
    from agents import dqn_agent, ddqn_agent
    torch.set_num_threads(1)
    out = {}
    for name, (variant, h, hid, n, gamma, lr, train) in U.CASES.items():
        mod = dqn_agent if variant == "dqn" else ddqn_agent
        Agent = mod.DQNAgent if variant == "dqn" else mod.DDQNAgent
        torch.manual_seed(0)
        agent = Agent(FakeEnv(), learning_rate=lr, starting_epsilon=0.9, final_epsilon=0.1,
                      epsilon_decay=100, discount_factor=gamma, eta=0.01, batch_size=n,
                      memory_size=1000, target_update_frequency=1, device="cpu")
        agent.source_net = mod.DQN(3, 6, 4, h, hidden_dim=hid)
        agent.target_net = mod.DQN(3, 6, 4, h, hidden_dim=hid)
        agent.optimizer = torch.optim.AdamW(agent.source_net.parameters(), lr)
        U.fill_params(agent.source_net, 11)
        U.fill_params(agent.target_net, 22)
        if not train:
            agent.source_net.eval()
            agent.target_net.eval()
        s6, w, a, r, s6n, wn = U.make_batch(n, 33)
        for i in range(n):
            st = (torch.from_numpy(s6[i:i + 1]), torch.from_numpy(w[i:i + 1]))
            nx = (torch.from_numpy(s6n[i:i + 1]), torch.from_numpy(wn[i:i + 1]))
            agent.memorize(st, torch.tensor(int(a[i])), float(r[i]), nx)
        random.seed(44)
        torch.manual_seed(55)
        loss = agent.optimize_model()
        out[f"{name}.loss"] = np.float64(loss)
        gs = U.param_stats(agent.source_net, grads=True)
        ps = U.param_stats(agent.source_net)
        names = sorted(gs)
        out[f"{name}.names"] = np.array(names)
        out[f"{name}.grad_sum"] = np.array([gs[k][0] for k in names])
        out[f"{name}.grad_abs"] = np.array([gs[k][1] for k in names])
        out[f"{name}.param_sum"] = np.array([ps[k][0] for k in names])
        out[f"{name}.param_abs"] = np.array([ps[k][1] for k in names])
        if hid <= 8:
            for k, p in sorted(agent.source_net.named_parameters()):
                out[f"{name}.grad.{k}"] = p.grad.numpy().copy()
                out[f"{name}.param.{k}"] = p.data.numpy().copy()
        print(name, "loss", loss)
    np.savez_compressed(os.path.join(HERE, "learner.npz"), **out)


if __name__ == "__main__":
    main(*sys.argv[1:])
