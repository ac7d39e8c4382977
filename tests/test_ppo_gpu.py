"""Config-5 PPO update on the GPU (agents/ppo.py) against the eager torch path it replaces
(ppo_agent.py:13-95 ActorCriticNet, :206-237 optimize_model).

1. ActorCriticNet from packed windows (the HIP f32 stem, csrc/mz_stem.hip) == from the f32
   window through Conv2d / LeakyReLU / MaxPool2d: outputs rtol 1e-5, parameter gradients rtol
   1e-4 (the conv sums associate differently, f32).
2. optimize_model with the captured minibatch step (PPOMinibatchGraph: 3 eager warm-up steps,
   capture, replays) == the same loop run eagerly with the same fused AdamW, over full and short
   minibatches and three passes: params within rtol 1e-5 + atol 1e-5, losses rel 1e-4."""
import copy

import pytest
import torch

from test_stem import _bits, _window

pytestmark = pytest.mark.gpu


def _close(a, b, rtol, atol):
    scale = float(b.detach().abs().max()) or 1.0
    return torch.allclose(a, b, rtol=rtol, atol=atol * scale)


def test_actor_critic_bits_match_f32_window():
    from mazerl.agents.ppo import ActorCriticNet
    torch.manual_seed(0)
    net = ActorCriticNet(3, 6, 4, 32, 1024).cuda()
    n = 130
    bits = _bits(n, 7).cuda()
    s6 = torch.randn(n, 6).cuda()
    win = _window(bits.cpu()).cuda()
    la, va = net((s6, bits))
    lb, vb = net((s6, win))
    assert _close(la, lb, 1e-5, 1e-6) and _close(va, vb, 1e-5, 1e-6)
    R1, R2 = torch.randn_like(la), torch.randn_like(va)
    ga = torch.autograd.grad((la * R1).sum() + (va * R2).sum(), list(net.parameters()))
    gb = torch.autograd.grad((lb * R1).sum() + (vb * R2).sum(), list(net.parameters()))
    for (name, _), x, y in zip(net.named_parameters(), ga, gb):
        assert _close(x, y, 1e-4, 1e-5), name


@pytest.mark.parametrize("hidden,bs,full", [(256, 64, 5), (1024, 2048, 4)])
def test_ppo_graph_minibatches_track_eager(hidden, bs, full):
    from mazerl.agents.ppo import ActorCriticNet, PPOMinibatchGraph, make_optimizer, optimize_model
    torch.manual_seed(1)
    A = ActorCriticNet(3, 6, 4, 32, hidden).cuda()
    B = copy.deepcopy(A)
    oa = make_optimizer(A, 3e-4, 1e-4, capturable=True)
    ob = make_optimizer(B, 3e-4, 1e-4, capturable=True)  # the same fused AdamW, run eagerly
    graph = PPOMinibatchGraph(A, oa, bs)
    g = torch.Generator().manual_seed(2)
    n = full * bs + 17  # full minibatches and a short one per pass
    bits = _bits(n, 3).cuda()
    s6 = torch.randn(n, 6, generator=g).cuda()
    act = torch.randint(0, 4, (n, 1), generator=g).cuda()
    lp = -torch.rand(n, 1, generator=g).cuda()
    adv = torch.randn(n, generator=g).cuda()
    ret = torch.randn(n, generator=g).cuda()
    for k in range(3):
        la = optimize_model(A, oa, (s6, bits), act, lp, adv, ret, 1e-2, bs, 2, graph=graph)
        lb = optimize_model(B, ob, (s6, bits), act, lp, adv, ret, 1e-2, bs, 2)
        torch.cuda.synchronize()
        assert float(la) == pytest.approx(float(lb), rel=1e-4, abs=1e-6), k
    assert graph.graphs is not None  # captured after the warm-up steps
    for (name, pa), pb in zip(A.named_parameters(), B.parameters()):
        assert torch.allclose(pa, pb, rtol=1e-5, atol=1e-5), name


def test_pair_surrogate_matches_torch_broadcast():
    """_PairSurrogate (the reference's [b,b] clipped surrogate with a written-out backward)
    against the torch expression it replaces, forward and gradient, incl. ratios on and outside
    the clip boundaries and zero advantages."""
    from mazerl.agents.ppo import _PairSurrogate
    torch.manual_seed(4)
    b = 300
    lp_new = (torch.randn(b, device="cuda") * 0.4).requires_grad_()
    lp_old = lp_new.detach()[torch.randperm(b, device="cuda")].reshape(b, 1) + 0.1 * torch.randn(b, 1, device="cuda")
    lp_old[:5, 0] = lp_new.detach()[:5] - torch.log(torch.tensor(1.3, device="cuda"))  # r == 1.3 at (j, j)
    adv = torch.randn(b, device="cuda")
    adv[::17] = 0.0
    out = _PairSurrogate.apply(lp_new, lp_old, adv, 0.3)
    (g,) = torch.autograd.grad(out, lp_new)
    lp2 = lp_new.detach().clone().requires_grad_()
    ratio = (lp2 - lp_old).exp()
    ref = torch.min(ratio * adv, torch.clamp(ratio, min=0.7, max=1.3) * adv).mean()
    (g2,) = torch.autograd.grad(ref, lp2)
    assert float(out) == pytest.approx(float(ref), rel=1e-5, abs=1e-7)
    assert torch.allclose(g, g2, rtol=1e-4, atol=1e-6 * float(g2.abs().max()))


def test_flat_adamw_groups_matches_torch_clip_and_adamw():
    """FlatAdamWGroups (mz_adamw_groups: clip_grad_norm_ + 3-group AdamW in three launches) ==
    torch.nn.utils.clip_grad_norm_(0.5) + torch.optim.AdamW(fused) with the same groups, over
    steps with the clip active and inactive (ppo_agent.py:232-236)."""
    from mazerl.agents.flat import FlatAdamWGroups
    from mazerl.agents.ppo import ActorCriticNet
    torch.manual_seed(9)
    A = ActorCriticNet(3, 6, 4, 32, 256).cuda()
    B = copy.deepcopy(A)

    def groups(n):
        return [(n.actor_head.parameters(), 3e-4), (n.critic_head.parameters(), 1e-4),
                (n.conv.parameters(), 2e-4)]
    oa = FlatAdamWGroups(A, groups(A), max_norm=0.5)
    ob = torch.optim.AdamW([{"params": list(ps), "lr": lr} for ps, lr in groups(B)], fused=True)
    g = torch.Generator(device="cuda").manual_seed(10)
    for k, scale in enumerate([1.0, 1e-4, 3.0, 1e-5, 1.0]):
        grads = [torch.randn(p.shape, generator=g, device="cuda") * scale for p in A.parameters()]
        for pa, pb, gr in zip(A.parameters(), B.parameters(), grads):
            pa.grad = gr.clone()
            pb.grad = gr.clone()
        oa.step()
        torch.nn.utils.clip_grad_norm_(B.parameters(), max_norm=0.5)
        ob.step()
        torch.cuda.synchronize()
        for (name, pa), pb in zip(A.named_parameters(), B.parameters()):
            assert torch.allclose(pa.grad, pb.grad, rtol=1e-5, atol=1e-9), (k, name)
            assert torch.allclose(pa, pb, rtol=1e-5, atol=1e-6), (k, name)
