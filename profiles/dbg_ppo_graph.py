"""Debug: PPOMinibatchGraph replays vs eager recomputation (variants monkeypatch the step)."""
import copy
import os
import sys

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import mazerl.agents.ppo as P  # noqa: E402
from test_stem import _bits  # noqa: E402

variant = sys.argv[1]
bs = int(sys.argv[2])
orig = P.ppo_minibatch


def losses(net, pos, win, act, lp_old, adv, ret, coef, flat):
    lp_new, value, ent = net.evaluate((pos, win), act)
    if flat:  # elementwise ratio instead of the [b,b] broadcast
        ratio = (lp_new - lp_old.squeeze(1)).exp()
        s1 = ratio * adv
        s2 = torch.clamp(ratio, 0.7, 1.3) * adv
        pl = -(torch.min(s1, s2).mean() + ent * coef).mean()
        vl = F.mse_loss(ret.unsqueeze(1), value)
        return pl, vl
    return P.ppo_losses(lp_old, lp_new, adv, ent, ret, value, coef)


def mb_variant(net, opt, pos, win, act, lp_old, adv, ret, coef, allreduce=None, phase=None):
    pl, vl = losses(net, pos, win, act, lp_old, adv, ret, coef, "flat" in variant)
    total = pl + 0.5 * vl
    opt.zero_grad()
    total.backward()
    if "noclip" not in variant:
        torch.nn.utils.clip_grad_norm_(net.parameters(), max_norm=0.5)
    opt.step()
    return total.detach()


P.ppo_minibatch = mb_variant
torch.manual_seed(1)
A = P.ActorCriticNet(3, 6, 4, 32, 1024).cuda()
if "nofused" in variant:
    oa = torch.optim.AdamW([{"params": A.actor_head.parameters(), "lr": 3e-4},
                            {"params": A.critic_head.parameters(), "lr": 1e-4},
                            {"params": A.conv.parameters(), "lr": 2e-4}], capturable=True)
else:
    oa = P.make_optimizer(A, 3e-4, 1e-4, capturable=True)
G = P.PPOMinibatchGraph(A, oa, bs)


def mb(seed):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(bs, 6, generator=g).cuda(), _bits(bs, seed).cuda(),
            torch.randint(0, 4, (bs, 1), generator=g).cuda(), -torch.rand(bs, 1, generator=g).cuda(),
            torch.randn(bs, generator=g).cuda(), torch.randn(bs, generator=g).cuda()]


for k in range(4):
    G.step(mb(k), 1e-2)
torch.cuda.synchronize()
bad_loss = bad_grad = 0
deferred = "defer" in variant
saved = []
for k in range(4, 10):
    x = mb(k)
    if deferred:  # no eager work between replays: keep param snapshots, check afterwards
        snap = [p.detach().clone() for p in A.parameters()]
        out = G.step(x, 1e-2)
        torch.cuda.synchronize()
        saved.append((k, x, snap, float(out), [p.grad.clone() for p in A.parameters()]))
        continue
    B = copy.deepcopy(A)
    for p in B.parameters():
        p.grad = None
    pl, vl = losses(B, *x, 1e-2, "flat" in variant)
    ref = float(pl + 0.5 * vl)
    (pl + 0.5 * vl).backward()
    if "noclip" not in variant:
        torch.nn.utils.clip_grad_norm_(B.parameters(), max_norm=0.5)
    out = G.step(x, 1e-2)
    torch.cuda.synchronize()
    bad_loss += abs(float(out) - ref) > 1e-5 * abs(ref)
    for (nm, pa), pb in zip(A.named_parameters(), B.parameters()):
        e = float((pa.grad - pb.grad).abs().max()) / (float(pb.grad.abs().max()) + 1e-30)
        if e > 1e-3:
            bad_grad += 1
            if k < 6:
                print(f"   replay {k}: {nm} rel err {e:.3g}")
for k, x, snap, out, grads in saved:
    B = copy.deepcopy(A)
    with torch.no_grad():
        for p, q in zip(B.parameters(), snap):
            p.copy_(q)
    for p in B.parameters():
        p.grad = None
    pl, vl = losses(B, *x, 1e-2, "flat" in variant)
    ref = float(pl + 0.5 * vl)
    (pl + 0.5 * vl).backward()
    torch.nn.utils.clip_grad_norm_(B.parameters(), max_norm=0.5)
    bad_loss += abs(out - ref) > 1e-5 * abs(ref)
    for (nm, pb), ga in zip(B.named_parameters(), grads):
        e = float((ga - pb.grad).abs().max()) / (float(pb.grad.abs().max()) + 1e-30)
        if e > 1e-3:
            bad_grad += 1
            if k < 6:
                print(f"   replay {k}: {nm} rel err {e:.3g}")
print(f"{variant:24s} bs {bs}: replays with wrong loss {bad_loss}/6, wrong param grads {bad_grad}/{6 * 14}")
