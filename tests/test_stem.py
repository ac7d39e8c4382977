"""The learner's packed-window conv stem (csrc/mz_stem.hip, agents/stem.py) against the torch
stem it replaces (dqn_agent.py:47-57, ddqn_agent.py:18-52: Conv2d(3->32, 3x3, pad 1) ->
LeakyReLU -> [Dropout(0.2)] -> MaxPool2d(2) -> flatten || obs6), forward and backward, in f32.

Dropout: the kernel's masks come from its counter hash; the test regenerates them in numpy
(same hash, same key mixing) and applies them in the torch pipeline, so the DDQN train-mode stem
is checked element for element too. Tolerances: the conv sums and the weight-gradient sums
associate differently from MIOpen's (f32): features rtol 1e-5 / atol 1e-6, gradients rtol 1e-4
/ atol 1e-5 (relative to each tensor's scale)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

M32 = np.uint64(0xFFFFFFFF)


def _hash32(x):
    x = x.astype(np.uint64) & M32
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & M32
    x ^= x >> np.uint64(16)
    return x


def _masks(n, key, salt, p):
    """keep mask [n, 32, 15, 15] (float) the kernel draws for rng value `key` and `salt`."""
    thresh = int(p * 65536.0 + 0.5)
    k0 = (np.uint64(key) & M32) ^ (np.uint64((salt * 0x9E3779B9) & 0xFFFFFFFF))
    k1 = (np.uint64(key >> 32) + _hash32(np.array([salt]))[0]) & M32
    nn, j = np.meshgrid(np.arange(n, dtype=np.uint64), np.arange(1568, dtype=np.uint64), indexing="ij")
    gid = np.uint64(2) * (nn * np.uint64(1568) + j)
    h0 = _hash32((_hash32(gid ^ k0) + k1) & M32)
    h1 = _hash32((_hash32((gid + np.uint64(1)) ^ k0) + k1) & M32)
    keep = np.ones((n, 32, 15, 15), dtype=np.float32)
    c, q = j.astype(np.int64) // 49, j.astype(np.int64) % 49
    py, px = q // 7, q % 7
    ni = nn.astype(np.int64)
    for r in range(4):
        h = h0 if r < 2 else h1
        u = (h >> np.uint64(16 * (r & 1))) & np.uint64(0xFFFF)
        keep[ni, c, 2 * py + (r >> 1), 2 * px + (r & 1)] = (u >= np.uint64(thresh)).astype(np.float32)
    return keep


def _bits(n, seed):
    g = torch.Generator().manual_seed(seed)
    b = torch.randint(0, 2**31, (n, 22), generator=g, dtype=torch.int64)
    b[:, 21] &= (1 << (675 - 21 * 32)) - 1
    return b.to(torch.int32)


def _window(bits):
    i = torch.arange(675)
    w = (bits.to(torch.int64)[:, i // 32] >> (i % 32)) & 1
    return w.to(torch.float32).view(-1, 3, 15, 15)


def _torch_stem(net, s6, win, keep=None, p=0.0):
    conv = net.conv[0]
    a = F.conv2d(win, conv.weight, conv.bias, padding=1)
    x = F.leaky_relu(a)
    if keep is not None:
        x = x * keep * (1.0 / (1.0 - p))
    x = F.max_pool2d(x, 2, 2)
    return torch.cat((x.flatten(1), s6), 1)


def _close(a, b, rtol, atol):
    scale = float(b.detach().abs().max()) or 1.0
    return torch.allclose(a, b, rtol=rtol, atol=atol * scale)


@pytest.mark.parametrize("variant", ["dqn", "ddqn"])
def test_stem_forward_backward_no_dropout(variant):
    from mazerl.agents.nets import QNet
    torch.manual_seed(1)
    net = QNet(variant=variant).cuda().eval()  # eval: no dropout
    n = 300
    bits = _bits(n, 2).cuda()
    s6 = torch.randn(n, 6).cuda()
    win = _window(bits.cpu()).cuda()
    R = torch.randn(n, 4).cuda()
    out_b = net((s6, bits))
    gb = torch.autograd.grad((out_b * R).sum(), list(net.parameters()))
    out_t = net((s6, win))
    gt = torch.autograd.grad((out_t * R).sum(), list(net.parameters()))
    assert _close(out_b, out_t, 1e-5, 1e-6)
    for (name, _), a, b in zip(net.named_parameters(), gb, gt):
        assert _close(a, b, 1e-4, 1e-5), name
    feat = net._bit_stem(s6, bits)
    with torch.no_grad():
        ref = _torch_stem(net, s6, win)
    assert _close(feat, ref, 1e-5, 1e-6)


def test_stem_dropout_matches_torch_with_same_masks():
    from mazerl.agents.nets import QNet
    torch.manual_seed(3)
    net = QNet(variant="ddqn").cuda().train()  # Dropout(0.2) active
    n = 256
    bits = _bits(n, 4).cuda()
    s6 = torch.randn(n, 6).cuda()
    win = _window(bits.cpu()).cuda()
    net._stem_rng = torch.tensor([0x123456789AB], dtype=torch.int64, device="cuda")
    key = 0x123456789AB
    feat = net._bit_stem(s6, bits)
    assert int(net._stem_rng.item()) == key + 1  # advanced for the next call
    keep = torch.from_numpy(_masks(n, key, net._salt, 0.2)).cuda()
    frac = 1.0 - float(keep[:, :, :14, :14].mean())
    assert abs(frac - 13107 / 65536) < 0.01
    ref = _torch_stem(net, s6, win, keep, 0.2)
    assert _close(feat, ref.detach(), 1e-5, 1e-6)
    # backward with the same masks
    R = torch.randn(n, 1574).cuda()
    net._stem_rng.fill_(key)
    fb = net._bit_stem(s6, bits)
    gb = torch.autograd.grad((fb * R).sum(), [net.conv[0].weight, net.conv[0].bias])
    ft = _torch_stem(net, s6, win, keep, 0.2)
    gt = torch.autograd.grad((ft * R).sum(), [net.conv[0].weight, net.conv[0].bias])
    for a, b in zip(gb, gt):
        assert _close(a, b, 1e-4, 1e-5)
    # a second call draws different masks
    f2 = net._bit_stem(s6, bits)
    assert not torch.equal(f2, feat)


def test_stem_edge_sizes():
    from mazerl.agents.nets import QNet
    net = QNet(variant="dqn").cuda().eval()
    for n in (1, 3, 65):
        bits = _bits(n, 10 + n).cuda()
        s6 = torch.randn(n, 6).cuda()
        win = _window(bits.cpu()).cuda()
        out_b = net((s6, bits))
        g_b = torch.autograd.grad(out_b.sum(), [net.conv[0].weight])[0]
        out_t = net((s6, win))
        g_t = torch.autograd.grad(out_t.sum(), [net.conv[0].weight])[0]
        assert _close(out_b, out_t, 1e-5, 1e-6), n
        assert _close(g_b, g_t, 1e-4, 1e-5), n
    # all-zero and all-one windows (ties in the pool, every conv term on)
    for fill in (0, -1):
        bits = torch.full((4, 22), fill, dtype=torch.int32)
        bits[:, 21] &= (1 << (675 - 21 * 32)) - 1
        s6 = torch.zeros(4, 6).cuda()
        win = _window(bits).cuda()
        bits = bits.cuda()
        assert _close(net((s6, bits)), net((s6, win)), 1e-5, 1e-6)


def test_learner_bit_stem_tracks_f32_stem():
    """VectorDQNLearner with the HIP stem vs the torch stem on the same replay (DQN, no dropout):
    losses and parameters track each other over several graph-replayed updates."""
    from mazerl import VectorMazeEnv
    from mazerl.agents.dqn import VectorDQNLearner
    env = VectorMazeEnv(64, 21, enrich=True, device="cuda", seed=1, window=False, window_bits=True)
    mk = lambda bs: VectorDQNLearner(64, "cuda", variant="dqn", batch_size=64, capacity=256,  # noqa: E731
                                     updates_per_step=1, target_every=4, seed=5, bit_stem=bs)
    A, B = mk(True), mk(False)
    B.source.load_state_dict(A.source.state_dict())
    B.target.load_state_dict(A.target.state_dict())
    for k in range(4):
        s6, sw = env.obs6.clone(), env.window_bits.clone()
        env.step_act(eps=1.0, seed=2, counter=k)
        for L in (A, B):
            L.replay.push(s6, sw, env.actions, env.reward, env.obs6, env.window_bits)
    A.replay._gen.manual_seed(9)
    B.replay._gen.manual_seed(9)
    for k in range(8):
        torch.manual_seed(100 + k)  # graph-captured sampling draws from the default generator
        la = A.update(env.expand_window)
        torch.manual_seed(100 + k)
        lb = B.update(env.expand_window)
        torch.cuda.synchronize()
        assert float(la) == pytest.approx(float(lb), rel=1e-3, abs=1e-6), k
    # AdamW normalises each element's step, so near-zero gradient elements whose f32 rounding
    # differs can move by up to lr per update in either direction: bound by 8 updates x lr
    for (name, pa), pb in zip(A.source.named_parameters(), B.source.parameters()):
        assert float((pa - pb).abs().max()) <= 8 * 1e-3 + 1e-6, name
    env.close()


@pytest.mark.parametrize("overlap", [False, True], ids=["sequential", "overlapped"])
def test_learner_counter_advanced_by_backward_draws_the_same_masks(overlap):
    """VectorDQNLearner (DDQN, packed windows) gives its two nets ONE dropout counter and moves it
    on from the source stem's backward (mz_stem_backward_ex; no add launch per forward). Each net
    still draws keys 0, 1, 2, ... per update, as with its own counter advanced after every
    forward — so, dropout active, the same weights bit for bit over eager and graph-captured
    updates."""
    from mazerl import VectorMazeEnv
    from mazerl.agents.dqn import VectorDQNLearner
    from test_learner_graph import _fill
    env = VectorMazeEnv(4, 21, enrich=True, device="cuda", seed=1)
    mk = lambda: VectorDQNLearner(4, "cuda", variant="ddqn", batch_size=64, capacity=256,  # noqa: E731
                                  updates_per_step=1, target_every=4, updates_per_epoch=2, seed=5,
                                  use_graph=True, overlap=overlap)
    A, B = mk(), mk()
    assert A.source._stem_rng is A.target._stem_rng
    assert (A.source._stem_advance, A.target._stem_advance) == ("backward", "none")
    # B: the per-forward scheme — a counter per net, an add after every forward
    for ma, mb in ((A.source, B.source), (A.target, B.target)):
        mb._stem_rng = torch.zeros(1, dtype=torch.int64, device="cuda")
        mb._stem_advance = "add"
        mb._salt = ma._salt  # the construction-order salts (before any capture bakes them in)
        mb.load_state_dict(ma.state_dict())
    assert A.source.training and A.target.training  # Dropout(0.2) active
    for L in (A, B):
        for k in range(4):
            _fill(L, n=64, seed=k)
    n = 10
    # one learner after the other, each from the same CUDA generator state: the sequential graph
    # learner samples its rows from the default generator, so interleaved updates would draw
    # different rows
    for L in (A, B):
        torch.cuda.manual_seed(123)
        for _ in range(n):
            L.update(env.expand_window, reserve=0)
        if overlap:
            L.finish()
        torch.cuda.synchronize()
    assert int(A.source._stem_rng.item()) == n
    assert int(B.source._stem_rng.item()) == n and int(B.target._stem_rng.item()) == n
    for pa, pb in zip(A.source.parameters(), B.source.parameters()):
        assert torch.equal(pa, pb)
    env.close()
