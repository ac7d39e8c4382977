"""Config-1 tabular Q-agent and config-5 PPO vs the reference's own outputs (tests/golden/agents.npz,
made by make_golden_agents.py from agents/q_agent.py and agents/ppo_agent.py).
Q-table: exact (float64). PPO: returns/advantages exact in float32, evaluate() rtol 1e-6,
parameters after optimize_model rtol 1e-5 (fp32)."""
import numpy as np
import pytest
import torch

import golden_io as G
import learner_util as U


@pytest.fixture(scope="module")
def fx():
    return G.load("agents.npz")


class _Env:
    class action_space:
        n = 4


def test_q_agent_table_matches_reference(fx):
    from mazerl.agents.q_agent import QAgent
    ag = QAgent(_Env(), learning_rate=0.1, initial_epsilon=0.95, epsilon_decay=40,
                final_epsilon=0.05, discount_factor=0.7, eta=0.01)
    for o, a, r, te, n in zip(fx["q.obs"], fx["q.act"], fx["q.rew"], fx["q.term"], fx["q.next"]):
        ag.update(str(o), int(a), float(r), bool(te), str(n))
    assert sorted(ag.q_values) == list(fx["q.keys"])
    for k, v in zip(fx["q.keys"], fx["q.values"]):
        np.testing.assert_array_equal(ag.q_values[str(k)], v)


def _ppo_net():
    from mazerl.agents.ppo import ActorCriticNet
    net = ActorCriticNet(3, 6, 4, 4, hidden_dim=8)
    U.fill_params(net, 101)
    return net


def test_ppo_returns_advantages_evaluate(fx):
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_golden_agents import PPO_REWARDS, ppo_inputs
    from mazerl.agents.ppo import calculate_advantages, calculate_returns
    np.testing.assert_array_equal(calculate_returns(PPO_REWARDS, 0.9).numpy(), fx["ppo.returns"])
    s6, w, a, lp, adv, ret, vals = ppo_inputs()
    np.testing.assert_array_equal(
        calculate_advantages(torch.from_numpy(ret), torch.from_numpy(vals)).numpy(), fx["ppo.advantages"])
    net = _ppo_net()
    lpn, val, ent = net.evaluate((torch.from_numpy(s6), torch.from_numpy(w)), torch.from_numpy(a))
    np.testing.assert_allclose(lpn.detach().numpy(), fx["ppo.eval_logp"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(val.detach().numpy(), fx["ppo.eval_value"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(ent.detach().numpy(), fx["ppo.eval_entropy"], rtol=1e-6, atol=1e-7)


def test_ppo_optimize_model_matches_reference(fx):
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_golden_agents import PPO_BATCH, PPO_COEF, PPO_STEPS, ppo_inputs
    from mazerl.agents.ppo import make_optimizer, optimize_model
    torch.set_num_threads(1)
    s6, w, a, lp, adv, ret, vals = ppo_inputs()
    net = _ppo_net()
    opt = make_optimizer(net, 3e-4, 1e-4)
    optimize_model(net, opt, (torch.from_numpy(s6), torch.from_numpy(w)), torch.from_numpy(a),
                   torch.from_numpy(lp), torch.from_numpy(adv), torch.from_numpy(ret), PPO_COEF,
                   PPO_BATCH, PPO_STEPS)
    for k, p in sorted(net.named_parameters()):
        np.testing.assert_allclose(p.data.numpy(), fx[f"ppo.param.{k}"], rtol=1e-5, atol=1e-7, err_msg=k)


def test_ppo_pool_episode_returns_advantages(fx):
    """The pool fixture (per-episode calculate_returns / calculate_advantages of the reference,
    ppo_agent.py:171-186, incl. 1-step episodes whose unbiased std is NaN) against this package's
    CPU restatement, exactly — the fixture the GPU finishing kernel is checked against."""
    from mazerl.agents.ppo import calculate_advantages, calculate_returns
    lens = fx["ppo.pool.lens"]
    off = np.concatenate([[0], np.cumsum(lens)])
    for k, n in enumerate(lens):
        sl = slice(off[k], off[k + 1])
        R = calculate_returns([float(x) for x in fx["ppo.pool.rewards"][sl]],
                              float(fx["ppo.pool.gamma"]))  # Python floats, as the reference
        A = calculate_advantages(R, torch.from_numpy(fx["ppo.pool.values"][sl]))
        np.testing.assert_array_equal(R.numpy(), fx["ppo.pool.returns"][sl])
        np.testing.assert_array_equal(A.numpy(), fx["ppo.pool.advantages"][sl])
        assert np.isnan(R.numpy()).all() == (n == 1)


def test_ppo_episode_bound_covers_max_steps():
    """VectorPPOTrainer's record buffers hold L = episode_bound(max_dim, toroidal) steps per
    instance: more than any episode (max_steps + 1 steps, base_maze_env.py:205-208). On the torus
    len / CE exceeds 1 for some mazes, so (N-1)^2 + 2 is not a bound there; the oracle's max_steps
    of generated mazes (17..79 toroidal, 15..81 euclidean, 3 algorithms) stay below L, and the
    formula's worst case (every open square on the solution) is what L is sized for."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import pyoracle as O
    from mazerl.trainers.ppo_trainer import episode_bound
    for tor, sizes in ((True, range(17, 80, 6)), (False, range(15, 82, 6))):
        L = episode_bound(max(sizes), tor)
        for n in sizes:
            for algo in range(3):
                for s in range(3):
                    start, goal, g = O.generate(n, algo, 0x5EED + 97 * n + s, toroidal=tor)
                    assert O.max_steps(g, start, goal, tor) + 1 < L
        # the formula's worst case at the largest size: len = every open square
        n = max(sizes)
        c = ((n + 1) // 2) ** 2 if tor else ((n - 1) // 2) ** 2
        worst = -(-((n - 1) ** 2 - 1) * (2 * c - 1) // ((n - 1) * ((n - 1) // 2) - 1))
        assert worst + 1 < L
    assert episode_bound(79, True) > (79 - 1) ** 2 + 2  # the old bound was short on the torus
