"""The fused Q head + loss (agents/dqn.py _HeadLossFn: mz_head_loss / mz_head_loss_backward, one
launch forward for both nets' last activation, fc3 and the loss; one launch + a column sum
backward) against the unfused path (the nets' own fc3 / activation launches, then mz_q_loss):
the loss and every source gradient agree to f32 tolerance (the dot products associate
differently), for DQN (LeakyReLU, max over the target's row) and DDQN (ReLU, the stacked [s; s']
pass and the argmax of the source's s' rows), with and without the flat gradient buffer
(agents/flat.py: fc3's weight and bias gradients land in their segments with one column sum)."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _batch(b, seed):
    g = torch.Generator().manual_seed(seed)
    s6 = torch.rand(b, 6, generator=g).cuda()
    sw = torch.randint(0, 2 ** 31, (b, 22), generator=g, dtype=torch.int64)
    sw[:, 21] &= 7
    sw = sw.to(torch.int32).cuda()
    s6n = torch.rand(b, 6, generator=g).cuda()
    swn = torch.roll(sw, 1, 0).contiguous()
    a = torch.randint(0, 4, (b,), generator=g).cuda()
    r = (torch.rand(b, generator=g) - 0.5).cuda()
    return (s6, sw), a, r, (s6n, swn)


@pytest.mark.parametrize("flat", [False, True], ids=["grads", "flat-grads"])
@pytest.mark.parametrize("variant", ["dqn", "ddqn"])
@pytest.mark.parametrize("b", [200, 1024])
def test_fused_head_matches_unfused(variant, flat, b):
    import mazerl.agents.dqn as D
    from mazerl.agents.flat import flatten_grads
    from mazerl.agents.nets import QNet
    torch.manual_seed(3)
    src0 = QNet(3, 6, 4, 32, 1024, variant).cuda()
    tgt0 = QNet(3, 6, 4, 32, 1024, variant).cuda()
    state, a, r, nxt = _batch(b, 11)
    out = {}
    for fused in (True, False):
        src, tgt = copy.deepcopy(src0), copy.deepcopy(tgt0)
        src.eval(); tgt.eval()  # Dropout(0.2) (DDQN) would draw per-net masks
        if flat:
            flatten_grads(src)
        D.FUSED_HEAD = fused
        try:
            loss = D.q_loss(src, tgt, state, a, r, nxt, 0.7, variant == "ddqn")
            src.zero_grad(set_to_none=True)
            loss.backward()
        finally:
            D.FUSED_HEAD = True
        torch.cuda.synchronize()
        out[fused] = (float(loss), [p.grad.detach().clone() for p in src.parameters()])
    (lf, gf), (lu, gu) = out[True], out[False]
    assert lf == pytest.approx(lu, rel=2e-5)
    names = [n for n, _ in src0.named_parameters()]
    for n, x, y in zip(names, gf, gu):
        torch.testing.assert_close(x, y, rtol=2e-4, atol=1e-6, msg=n)


def test_fused_head_loss_is_deterministic():
    """Two launches on the same rows give the same loss and gradients bit for bit (the loss and
    the fc3 gradient sums run in a fixed order: per block, then over blocks)."""
    import mazerl.agents.dqn as D
    from mazerl.agents.nets import QNet
    torch.manual_seed(4)
    src = QNet(3, 6, 4, 32, 1024, "ddqn").cuda().eval()
    tgt = QNet(3, 6, 4, 32, 1024, "ddqn").cuda().eval()
    state, a, r, nxt = _batch(1024, 12)
    res = []
    for _ in range(2):
        loss = D.q_loss(src, tgt, state, a, r, nxt, 0.7, True)
        src.zero_grad(set_to_none=True)
        loss.backward()
        res.append((loss.detach().clone(), [p.grad.clone() for p in src.parameters()]))
    assert torch.equal(res[0][0], res[1][0])
    for x, y in zip(res[0][1], res[1][1]):
        assert torch.equal(x, y)
