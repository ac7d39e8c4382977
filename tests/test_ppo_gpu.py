"""Config-5 PPO update on the GPU (agents/ppo.py) against the eager torch path it replaces
(ppo_agent.py:13-95 ActorCriticNet, :206-237 optimize_model).

1. ActorCriticNet from packed windows (the HIP f32 stem, csrc/mz_stem.hip) == from the f32
   window through Conv2d / LeakyReLU / MaxPool2d: outputs rtol 1e-5, parameter gradients rtol
   1e-4 (the conv sums associate differently, f32).
2. optimize_model with the captured minibatch step (PPOMinibatchGraph: 3 eager warm-up steps,
   capture, replays) == the same loop run eagerly with the same fused AdamW, over full and short
   minibatches and three passes: params within rtol 1e-5 + atol 1e-5, losses rel 1e-4."""
import copy

import numpy as np
import pytest
import torch
import torch.nn.functional as F

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


@pytest.mark.parametrize("b", [37, 2048])
def test_fused_head_loss_matches_torch(b):
    """_PPOHeadLoss (mz_ppo_head_loss) == evaluate() + ppo_losses() + total = pl + 0.5 vl in torch
    (ppo_agent.py:55-66, 188-203): the loss to 1e-5 relative and every parameter gradient of the
    actor-critic to 1e-4, with the entropy coefficient as a device scalar (the captured step's)."""
    import torch.nn.functional as F
    from mazerl.agents.ppo import ActorCriticNet, _PPOHeadLoss, ppo_losses
    torch.manual_seed(3)
    net = ActorCriticNet(3, 6, 4, 32, 256).cuda()
    g = torch.Generator().manual_seed(4)
    bits = _bits(b, 5).cuda()
    s6 = torch.randn(b, 6, generator=g).cuda()
    act = torch.randint(0, 4, (b, 1), generator=g).cuda()
    lp_old = (-torch.rand(b, 1, generator=g) * 2).cuda()
    adv = torch.randn(b, generator=g).cuda()
    ret = torch.randn(b, generator=g).cuda()
    coef = torch.tensor(7e-3, device="cuda")
    out = {}
    for fused in (False, True):
        net.zero_grad()
        logits, value = net((s6, bits))
        if fused:
            total = _PPOHeadLoss.apply(logits, value, act, lp_old, adv, ret, coef, 0.3)
        else:
            prob = F.softmax(logits, dim=-1)
            lp_new = F.log_softmax(logits, dim=-1).gather(1, act).squeeze(1)
            ent = -torch.sum(prob * torch.log(prob + 1e-8), dim=1)
            pl, vl = ppo_losses(lp_old, lp_new, adv, ent, ret, value, coef)
            total = pl + 0.5 * vl
        total.backward()
        out[fused] = (float(total), [p.grad.clone() for p in net.parameters()])
    assert out[True][0] == pytest.approx(out[False][0], rel=1e-5, abs=1e-7)
    for (name, _), x, y in zip(net.named_parameters(), out[False][1], out[True][1]):
        assert _close(y, x, 1e-4, 1e-6), name


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


# ---- the on-device rollout path of VectorPPOTrainer (csrc/mz_ppo.hip) -----------------------
def _ppo_trainer(B, dims, hidden=256, **kw):
    from mazerl.trainers.ppo_trainer import VectorPPOTrainer
    from mazerl.trainers.vector_trainer import make_env
    env = make_env(B, list(dims), toroidal=True, device="cuda", done_list=False, reward64=True,
                   window=False, window_bits=True)
    kw.setdefault("bank", False)
    return env, VectorPPOTrainer(env, "cuda", hidden_dim=hidden, **kw)


def _pool_fixture():
    import golden_io as G
    fx = G.load("agents.npz")
    lens = [int(n) for n in fx["ppo.pool.lens"]]
    off = np.concatenate([[0], np.cumsum(lens)]).astype(int)
    return fx, lens, off


def test_episode_finish_matches_reference_returns_advantages():
    """mz_ppo_scan + mz_ppo_finish on recorded episodes vs the reference's calculate_returns /
    calculate_advantages (ppo_agent.py:171-186; tests/golden/agents.npz "ppo.pool.*": 12
    episodes of 1..2,600 steps). Returns and advantages within rtol 1e-5 / atol 2e-6 (the
    reference normalises with float32 reductions, the kernel sums in float64); 1-step episodes
    (NaN in the reference) are dropped and counted; every other pool column is the record,
    bit-exact; rows land in instance order after the rows already pooled; a second round of
    finished episodes appends behind the first."""
    fx, lens, off = _pool_fixture()
    E = len(lens)
    B = E + 2
    env, tr = _ppo_trainer(B, [55], pool_size=1 << 20)  # L = 54^2 + 2 >= 2,600
    assert tr.L > max(lens)
    tr.gamma = float(fx["ppo.pool.gamma"])
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(5)
    tr.b_s6.copy_(torch.rand(tr.b_s6.shape, generator=g, device=dev))
    tr.b_w.copy_(torch.randint(-2**31, 2**31 - 1, tr.b_w.shape, generator=g, device=dev, dtype=torch.int32))
    tr.b_a.copy_(torch.randint(0, 4, tr.b_a.shape, generator=g, device=dev))
    tr.b_lp.copy_(-torch.rand(tr.b_lp.shape, generator=g, device=dev))
    rew = torch.from_numpy(fx["ppo.pool.rewards"]).to(dev)
    val = torch.from_numpy(fx["ppo.pool.values"]).to(dev)

    def round_(episodes):
        r64 = torch.zeros(B, dtype=torch.float64, device=dev)
        term = torch.zeros(B, dtype=torch.uint8, device=dev)
        trunc = torch.zeros(B, dtype=torch.uint8, device=dev)
        t0 = torch.zeros(B, dtype=torch.int32)
        for i, k in episodes:
            n, sl = lens[k], slice(off[k], off[k + 1])
            tr.b_r[i, :n - 1] = rew[sl][:-1]
            tr.b_v[i, :n] = val[sl]
            t0[i] = n - 1
            r64[i] = rew[sl][-1]
            win = float(fx["ppo.pool.rewards"][off[k + 1] - 1]) == 1.0
            (term if win else trunc)[i] = 1
        t0[E], t0[E + 1] = 5, 0  # two instances mid-episode
        r64[E] = r64[E + 1] = 0.45
        tr.t.copy_(t0)
        tr._scan_finish(r64, term, trunc)
        torch.cuda.synchronize()
        t1 = tr.t.cpu()
        for i, _ in episodes:
            assert t1[i] == 0
        assert t1[E] == 6 and t1[E + 1] == 1 and float(tr.b_r[E, 5]) == 0.45

    def check(episodes, base):
        o = base
        for i, k in episodes:
            n, sl = lens[k], slice(off[k], off[k + 1])
            if n == 1:
                continue
            rows = slice(o, o + n)
            torch.testing.assert_close(tr.p_ret[rows].cpu(), torch.from_numpy(fx["ppo.pool.returns"][sl]),
                                       rtol=1e-5, atol=2e-6)
            torch.testing.assert_close(tr.p_adv[rows].cpu(), torch.from_numpy(fx["ppo.pool.advantages"][sl]),
                                       rtol=1e-5, atol=2e-6)
            assert torch.equal(tr.p_s6[rows], tr.b_s6[i, :n]) and torch.equal(tr.p_w[rows], tr.b_w[i, :n])
            assert torch.equal(tr.p_a[rows], tr.b_a[i, :n]) and torch.equal(tr.p_lp[rows], tr.b_lp[i, :n])
            o += n
        return o

    first = [(k, k) for k in range(E)]
    round_(first)
    fill = check(first, 0)
    assert int(tr.pool_fill) == fill == sum(n for n in lens if n > 1) == int(tr.pool_total)
    wins = sum(float(fx["ppo.pool.rewards"][off[k + 1] - 1]) == 1.0 for k in range(E))
    assert tr.stats.tolist() == [E, wins, sum(n == 1 for n in lens), 0]
    second = [(3, 6), (0, 9), (7, 4), (10, 2)]  # instance order differs from fixture order
    round_(second)
    end = check(sorted(second), fill)
    assert int(tr.pool_fill) == end == int(tr.pool_total)
    env.close()


def test_ppo_act_records_the_f32_policy():
    """mz_ppo_act after the f32 forward: the recorded log-prob is bit-identical to
    ActorCriticNet.act's torch.log(softmax(logits).gather(action)) in f32 (ppo_agent.py:55-68),
    the value is the critic's output, obs6 / window bits are the env's, and the action the env
    steps with is the recorded one."""
    env, tr = _ppo_trainer(512, [17, 21, 29])
    for step in range(3):
        t = tr.t.clone().long()
        logits, value = tr._act()
        torch.cuda.synchronize()
        ar = torch.arange(512, device="cuda")
        a = tr.b_a[ar, t]
        ref_lp = torch.log(F.softmax(logits, dim=-1).gather(1, a[:, None]).squeeze(1))
        assert torch.equal(tr.b_lp[ar, t], ref_lp)
        assert torch.equal(tr.b_v[ar, t], value[:, 0])
        assert torch.equal(tr.b_s6[ar, t], env.obs6) and torch.equal(tr.b_w[ar, t], env.window_bits)
        assert torch.equal(tr.act_out.long(), a)
        l2, v2 = tr.net((env.obs6, env.window_bits))  # the acting forward is the f32 net's
        assert torch.equal(l2, logits) and torch.equal(v2, value)
        env.step(tr.act_out)
        tr._scan_finish()
        env.reset_done(regen_won=True)
    env.close()


def test_ppo_draws_follow_softmax_probabilities():
    """P(a) of mz_ppo_act's draw == softmax(logits)[a] (torch.multinomial's distribution,
    ppo_agent.py:63): 2^20 draws per logits row, chi-square against the softmax probabilities
    (p-value > 1e-6), including a near-zero-probability action that must never be drawn."""
    from scipy.stats import chi2
    from mazerl import _native as N
    lib = N.load()
    rows = torch.tensor([[0.0, 0.5, -1.0, 2.0], [3.0, 3.0, -200.0, 0.1], [-0.3, -0.3, -0.3, -0.3]],
                        device="cuda")
    B, K = 65536, 16
    for r in rows:
        logits = r.repeat(B, 1).contiguous()
        value = torch.zeros(B, device="cuda")
        t = torch.zeros(B, dtype=torch.int32, device="cuda")
        s6 = torch.zeros(B, 6, device="cuda")
        bits = torch.zeros(B, 22, dtype=torch.int32, device="cuda")
        rs6, rw = torch.zeros(B, 6, device="cuda"), torch.zeros(B, 22, dtype=torch.int32, device="cuda")
        ra, rlp, rv = (torch.zeros(B, dtype=torch.int64, device="cuda"), torch.zeros(B, device="cuda"),
                       torch.zeros(B, device="cuda"))
        out = torch.zeros(B, dtype=torch.int32, device="cuda")
        counts = torch.zeros(4, dtype=torch.int64, device="cuda")
        for c in range(K):
            N.check(lib.mz_ppo_act(logits.data_ptr(), 4, value.data_ptr(), 1, s6.data_ptr(),
                                   bits.data_ptr(), B, 1, 77, c, t.data_ptr(), rs6.data_ptr(),
                                   rw.data_ptr(), ra.data_ptr(), rlp.data_ptr(), rv.data_ptr(),
                                   out.data_ptr(), torch.cuda.current_stream().cuda_stream))
            counts += torch.bincount(out.long(), minlength=4)
        p = F.softmax(r.double(), dim=-1).cpu().numpy()
        n = counts.cpu().numpy().astype(np.float64)
        live = p > 1e-12
        assert n[~live].sum() == 0
        exp = p[live] * n.sum()
        stat = ((n[live] - exp) ** 2 / exp).sum()
        assert chi2.sf(stat, live.sum() - 1) > 1e-6, (r.tolist(), n, exp)


def test_vector_ppo_trains_with_device_pool():
    """VectorPPOTrainer end to end on a small toroidal config: updates fire from the host's
    one-step-late view of the device pool total, each consumes exactly pool_size rows (none
    non-finite), the remainder stays in the pool, counters match the pool's rows, and
    evaluation runs greedy in f32."""
    from mazerl.trainers.vector_trainer import evaluate
    env, tr = _ppo_trainer(256, [17, 21], pool_size=2048, batch_size=256, ppo_steps=1, use_graph=True)
    tr.train(300)
    fill = int(tr.pool_fill)
    assert tr.updates >= 1 and tr.consumed == tr.updates * 2048 == tr.rows_trained
    assert 0 <= fill < 2048 + 2 * 256 * tr.L
    assert int(tr.pool_total) == tr.consumed + fill
    assert tr.episodes > 0 and int(tr.stats[2]) >= 0
    rate, _ = evaluate(tr, 64, [17, 21], toroidal=True, device="cuda", seed=5)
    assert 0.0 <= rate <= 1.0
    env.close()
