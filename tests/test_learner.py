"""Q-loss parity of mazerl's DQN/DDQN update against the reference's optimize_model outputs
(tests/golden/learner.npz, produced by make_golden_learner.py from agents/dqn_agent.py:121-157 and
agents/ddqn_agent.py:113-152). Tolerances (fp32): loss rtol 1e-5 on CPU / 1e-4 on GPU; gradients
rtol 1e-4 + atol 1e-6 elementwise (small nets) or on per-parameter sums (full 2.1M-param nets)."""
import os
import random

import numpy as np
import pytest
import torch

import golden_io as G
import learner_util as U
from mazerl.agents.dqn import learner_update, q_loss
from mazerl.agents.nets import QNet, count_params, forward_flops


@pytest.fixture(scope="module")
def fx():
    return G.load("learner.npz")


def run_ours(case, device):
    variant, h, hid, n, gamma, lr, train = U.CASES[case]
    src = QNet(3, 6, 4, h, hid, variant)
    tgt = QNet(3, 6, 4, h, hid, variant)
    U.fill_params(src, 11)
    U.fill_params(tgt, 22)
    src.to(device)
    tgt.to(device)
    if not train:
        src.eval()
        tgt.eval()
    opt = torch.optim.AdamW(src.parameters(), lr)
    s6, w, a, r, s6n, wn = U.make_batch(n, 33)
    random.seed(44)
    perm = random.sample(range(n), n)  # the reference's random.sample order (replay_memory.py:18)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x[perm])).to(device)  # noqa: E731
    torch.manual_seed(55)
    reward = torch.tensor(tuple(float(x) for x in r[perm])).to(device)
    loss = q_loss(src, tgt, (t(s6), t(w)), t(a), reward, (t(s6n), t(wn)), gamma, variant == "ddqn")
    lv = float(loss.item())
    learner_update(src, opt, loss)
    return src, lv


def _compare(fx, case, src, loss, device):
    rt = 1e-5 if device == "cpu" else 1e-4
    assert loss == pytest.approx(float(fx[f"{case}.loss"]), rel=rt)
    names = list(fx[f"{case}.names"])
    gs = U.param_stats(src, grads=True)
    ps = U.param_stats(src)
    assert sorted(gs) == names
    for i, k in enumerate(names):
        ga = float(fx[f"{case}.grad_abs"][i])
        assert gs[k][1] == pytest.approx(ga, rel=1e-4, abs=1e-6), k
        assert gs[k][0] == pytest.approx(float(fx[f"{case}.grad_sum"][i]), abs=1e-4 * ga + 1e-6), k
        pa = float(fx[f"{case}.param_abs"][i])
        assert ps[k][1] == pytest.approx(pa, rel=1e-5), k
        assert ps[k][0] == pytest.approx(float(fx[f"{case}.param_sum"][i]), abs=1e-5 * pa + 1e-6), k
    if f"{case}.grad.{names[0]}" in fx:
        for k, p in src.named_parameters():
            np.testing.assert_allclose(p.grad.cpu().numpy(), fx[f"{case}.grad.{k}"], rtol=1e-4, atol=1e-6)
            np.testing.assert_allclose(p.data.cpu().numpy(), fx[f"{case}.param.{k}"], rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("case", list(U.CASES))
def test_q_loss_matches_reference_cpu(fx, case):
    torch.set_num_threads(1)
    src, loss = run_ours(case, "cpu")
    _compare(fx, case, src, loss, "cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("case", [c for c in U.CASES if not U.CASES[c][6]])
def test_q_loss_matches_reference_gpu(fx, case):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    src, loss = run_ours(case, "cuda")
    _compare(fx, case, src, loss, "cuda")


def test_architecture_counts():
    """2,140,548 parameters, 4,665,024 FLOP per sample forward."""
    assert count_params(QNet(variant="dqn")) == 2_140_548
    assert count_params(QNet(variant="ddqn")) == 2_140_548
    assert forward_flops() == 4_665_024
    sd = QNet(variant="ddqn").state_dict()
    assert list(sd) == ["conv.0.weight", "conv.0.bias", "fc.0.weight", "fc.0.bias", "fc.2.weight",
                        "fc.2.bias", "fc.4.weight", "fc.4.bias"]


def test_device_replay_ring_cpu():
    from mazerl.replay import DeviceReplay
    rb = DeviceReplay(10, "cpu")
    for k in range(3):
        n = 4
        s6 = torch.full((n, 6), float(k))
        sw = torch.full((n, 22), k, dtype=torch.int32)
        rb.push(s6, sw, torch.arange(n), torch.ones(n), s6 + 1, sw + 1)
    assert len(rb) == 10 and rb.ptr == 2
    assert rb.s6[0, 0] == 2 and rb.s6[1, 0] == 2 and rb.s6[2, 0] == 0 and rb.s6[8, 0] == 2
    expand = lambda b: torch.zeros(b.shape[0], 3, 15, 15)  # noqa: E731
    (s, w), a, r, (sn, wn) = rb.sample(5, expand)
    assert s.shape == (5, 6) and w.shape == (5, 3, 15, 15) and torch.all(sn == s + 1)
