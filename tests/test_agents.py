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
