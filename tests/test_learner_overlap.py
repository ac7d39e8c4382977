"""The overlapped learner (env -> learner handoff on a side HIP stream, agents/dqn.py
VectorDQNLearner(overlap=True)) against the eager learner (q_loss / learner_update,
dqn_agent.py:121-157).

Same replay trick as test_learner_graph.py: one transition repeated, so every batch is the same
whatever rows are drawn, and the side-stream graph replays must track the eager updates update
for update (tolerance as there: capturable AdamW, rtol 1e-5 + atol 1e-5 on params, rel 1e-4 on
losses). The acting snapshot greedy() reads must be the source net one update behind (the
documented lag of the overlapped schedule), and the sampled rows must avoid the `reserve` rows
the next push overwrites."""
import pytest
import torch
import torch.nn.functional as F

from test_learner_graph import _fill

pytestmark = pytest.mark.gpu


def _mk(overlap, **kw):
    from mazerl.agents.dqn import VectorDQNLearner
    args = dict(variant="dqn", batch_size=32, capacity=64, updates_per_step=1, target_every=4,
                updates_per_epoch=2, seed=5)
    args.update(kw)
    return VectorDQNLearner(4, "cuda", overlap=overlap, use_graph=overlap, **args)


def _params(net):
    return [p.detach().clone() for p in net.parameters()]


def test_overlapped_updates_track_eager_and_acting_lags_one_update():
    from mazerl import VectorMazeEnv
    env = VectorMazeEnv(4, 21, enrich=True, device="cuda", seed=1)
    A, B = _mk(True), _mk(False)
    assert A.overlap and not B.overlap
    B.source.load_state_dict(A.source.state_dict())
    B.target.load_state_dict(A.target.state_dict())
    _fill(A)
    _fill(B)
    bits, obs6 = A.replay.sw[:8].contiguous(), A.replay.s6[:8].contiguous()
    after = [_params(B.source)]  # B's params after j updates
    for k in range(12):
        A.greedy(obs6, None, bits)
        if A._async and k >= 5:
            slot = A._acting
            torch.cuda.synchronize()
            for pa, pb in zip(A.actors[slot].parameters(), after[k - 1]):
                assert torch.allclose(pa, pb, rtol=1e-5, atol=1e-5), k
        la = A.update(env.expand_window, reserve=0)
        lb = B.update(env.expand_window)
        after.append(_params(B.source))
        torch.cuda.synchronize()
        assert float(la) == pytest.approx(float(lb), rel=1e-4, abs=1e-7), k
    assert A._async  # the graph replays went to the side stream
    A.finish()
    torch.cuda.synchronize()
    assert A.n_updates == B.n_updates == 12
    assert float(A.opt.param_groups[0]["lr"]) == pytest.approx(B.opt.param_groups[0]["lr"], rel=1e-6)
    for (na, pa), (nb, pb) in zip(A.source.named_parameters(), B.source.named_parameters()):
        assert torch.allclose(pa, pb, rtol=1e-5, atol=1e-5), na
    for pa, pb in zip(A.target.parameters(), B.target.parameters()):
        assert torch.allclose(pa, pb, rtol=1e-5, atol=1e-5)
    # after finish() acting reads the source net again
    assert not A._async
    q = A.fused(obs6, bits).float()
    qs = A.greedy(obs6, None, bits)
    assert torch.equal(qs, q.argmax(1))
    env.close()


def test_overlapped_sampling_avoids_the_next_push():
    from mazerl import VectorMazeEnv
    env = VectorMazeEnv(4, 21, enrich=True, device="cuda", seed=1)
    A = _mk(True, capacity=64)
    _fill(A, n=64)
    _fill(A, n=40)  # wrap: ptr = 40, full
    rp, reserve = A.replay, 16
    for k in range(10):
        A.update(env.expand_window, reserve=reserve)
        if A._async:
            slot = A._par ^ 1  # the buffer the update just issued reads
            torch.cuda.synchronize()
            idx = A._idx[slot].flatten().cpu()
            ahead = (idx - rp.ptr) % rp.capacity  # 0 .. reserve-1 = rows the next push writes
            assert int(ahead.min()) >= reserve, k
            assert len(set(idx.tolist())) > 16  # spread over the allowed rows
    A.finish()
    with pytest.raises(ValueError):
        A.update(env.expand_window, reserve=64 - 8)  # fewer rows left than a batch
    A.finish()
    env.close()


def test_overlapped_updates_on_distinct_rows_match_a_reference_update():
    """Distinct transitions in the replay: each side-stream graph replay must equal q_loss +
    learner_update (the reference's optimize_model, dqn_agent.py:121-157) computed eagerly on the
    rows the update drew: loss and clamped gradients, one update at a time (a repeated transition
    would hide a gradient that goes stale between replays)."""
    from mazerl import VectorMazeEnv
    from mazerl.agents.dqn import q_loss
    env = VectorMazeEnv(4, 21, enrich=True, device="cuda", seed=1)
    A, B = _mk(True, batch_size=1024, capacity=4096), _mk(False, batch_size=1024, capacity=4096)
    B.source.load_state_dict(A.source.state_dict())
    B.target.load_state_dict(A.target.state_dict())
    g = torch.Generator(device="cuda").manual_seed(3)
    n = 4096
    s6, s6n = (torch.randn(n, 6, device="cuda", generator=g) for _ in range(2))
    sw, swn = (torch.randint(0, 2**31 - 1, (n, 22), device="cuda", generator=g, dtype=torch.int32)
               for _ in range(2))
    a = torch.randint(0, 4, (n,), device="cuda", generator=g)
    r = torch.randn(n, device="cuda", generator=g)
    for L in (A, B):
        L.replay.push(s6, sw, a, r, s6n, swn)
    for k in range(8):
        B.source.load_state_dict(A.source.state_dict())  # A's nets before this update
        B.target.load_state_dict(A.target.state_dict())
        A.update(env.expand_window, reserve=0)
        torch.cuda.synchronize()
        if not A._async:  # eager warm-up and capture updates draw their own rows
            continue
        idx = A._idx[A._par ^ 1][0]  # the rows this side-stream update read
        rp = B.replay
        loss = q_loss(B.source, B.target, (rp.s6[idx], rp.sw[idx]), rp.a[idx], rp.r[idx],
                      (rp.s6n[idx], rp.swn[idx]), B.gamma, False)
        B.opt.zero_grad()
        loss.backward()
        for (name, pa), pb in zip(A.source.named_parameters(), B.source.parameters()):
            ref = pb.grad.clamp(-1, 1)  # A's FlatAdamW leaves the clamped gradient in place
            assert torch.allclose(pa.grad, ref, rtol=1e-3, atol=1e-4 * float(ref.abs().max())), (k, name)
        assert float(A.last_loss) == pytest.approx(float(loss.detach()), rel=1e-4), k
    A.finish()
    env.close()


def test_replay_gather_matches_index_select():
    """DeviceReplay.sample on the GPU (one mz_replay_gather launch into stacked [2b] buffers)
    returns exactly the rows index_select gives, and q_loss reads the stacked buffer in place."""
    from mazerl.agents.dqn import _stacked
    from mazerl.replay import DeviceReplay
    rp = DeviceReplay(1000, "cuda")
    g = torch.Generator(device="cuda").manual_seed(7)
    n = 700
    s6, s6n = (torch.randn(n, 6, device="cuda", generator=g) for _ in range(2))
    sw, swn = (torch.randint(-2**31, 2**31 - 1, (n, 22), device="cuda", generator=g,
                             dtype=torch.int32) for _ in range(2))
    a = torch.randint(0, 4, (n,), device="cuda", generator=g)
    r = torch.randn(n, device="cuda", generator=g)
    rp.push(s6, sw, a, r, s6n, swn)
    rp.push(s6[:500], sw[:500], a[:500], r[:500], s6n[:500], swn[:500])  # wraps the ring
    for b in (1, 37, 512):
        rp.idx_static = torch.randint(0, rp.size, (b,), device="cuda", generator=g)
        (x6, xw), xa, xr, (y6, yw) = rp.sample(b, None, idx_static=True)
        i = rp.idx_static
        assert torch.equal(x6, rp.s6[i]) and torch.equal(xw, rp.sw[i])
        assert torch.equal(y6, rp.s6n[i]) and torch.equal(yw, rp.swn[i])
        assert torch.equal(xa, rp.a[i]) and torch.equal(xr, rp.r[i])
        st = _stacked(x6, y6)
        assert st.data_ptr() == x6.data_ptr() and st.shape == (2 * b, 6)
        assert torch.equal(_stacked(xw, yw), torch.cat((rp.sw[i], rp.swn[i])))


def test_stacked_ddqn_pass_matches_two_passes():
    """q_loss's stacked DDQN pass (source over [s; s'] in one 2b-row pass, backward over the
    first b rows: QNet.forward_rows) against the two-pass form (source(s), then source(s') under
    no_grad: ddqn_agent.py:113-152) on distinct rows: same loss and gradients (f32 tolerance:
    the GEMMs run at other shapes)."""
    import copy

    from mazerl.agents import dqn as D
    from mazerl.agents.nets import QNet
    torch.manual_seed(4)
    src, tgt = QNet(variant="ddqn").cuda().eval(), QNet(variant="ddqn").cuda().eval()
    g = torch.Generator(device="cuda").manual_seed(9)
    b = 1024
    s = (torch.randn(b, 6, device="cuda", generator=g),
         torch.randint(-2**31, 2**31 - 1, (b, 22), device="cuda", generator=g, dtype=torch.int32))
    nx = (torch.randn(b, 6, device="cuda", generator=g),
          torch.randint(-2**31, 2**31 - 1, (b, 22), device="cuda", generator=g, dtype=torch.int32))
    a = torch.randint(0, 4, (b,), device="cuda", generator=g)
    r = torch.randn(b, device="cuda", generator=g)
    out = {}
    for stack in (False, True):
        net = copy.deepcopy(src)
        old, D.STACK_ROWS = D.STACK_ROWS, stack
        try:
            loss = D.q_loss(net, tgt, s, a, r, nx, 0.7, True)
        finally:
            D.STACK_ROWS = old
        loss.backward()
        out[stack] = (float(loss), [p.grad.clone() for p in net.parameters()])
    assert out[True][0] == pytest.approx(out[False][0], rel=1e-5)
    for g1, g0 in zip(out[True][1], out[False][1]):
        assert torch.allclose(g1, g0, rtol=1e-4, atol=1e-5 * float(g0.abs().max()) + 1e-12)


def test_stacked_ddqn_pass_train_mode_matches_torch_with_same_masks():
    """The stacked pass in TRAIN mode (Dropout(0.2) on, as DDQN always runs: SURVEY Q13): the
    forward over [s; s'] and the row-limited backward against the torch pipeline (Conv2d ->
    LeakyReLU -> dropout with the kernel's masks regenerated in numpy -> MaxPool2d -> fc) over
    the same 2b rows, the gradient taken through the first b rows only. f32 tolerances as in
    test_stem.py."""
    import copy

    from test_stem import _bits, _close, _masks, _torch_stem, _window

    from mazerl.agents.nets import QNet
    torch.manual_seed(6)
    net = QNet(variant="ddqn").cuda().train()
    # the reference in float64: an f32 torch reference's MIOpen conv algorithm (and so its max-pool
    # near ties) can change from run to run
    ref = copy.deepcopy(net).double()
    b = 384
    bits = _bits(2 * b, 21)
    win = _window(bits).cuda()
    bits = bits.cuda()
    s6 = torch.randn(2 * b, 6).cuda()
    key = 0x5151_0000_2222
    net._stem_rng = torch.tensor([key], dtype=torch.int64, device="cuda")
    q = net.forward_rows((s6, bits), b)
    assert int(net._stem_rng.item()) == key + 1
    keep = torch.from_numpy(_masks(2 * b, key, net._salt, 0.2)).cuda()
    q_ref = ref.fc(_torch_stem(ref, s6.double(), win.double(), keep.double(), 0.2))
    # the stem's features agree to ~1.3e-7 x scale; the f32 fc GEMMs (K = 1,574, then 1,024)
    # against float64 add ~1.0-1.6e-6 x scale, which an atol of 1e-6 x scale failed by chance
    # for some dropout salts (profiles/dbg_stem_salt.py: worst ratio 0.67-1.04 over salts 1..40)
    assert _close(q, q_ref.detach().float(), 1e-5, 1e-5)
    R = torch.randn(b, 4).cuda()
    # Rows holding a pool window whose two largest (kept, non-zero) activations lie within f32
    # reassociation noise of each other get zero weight: there the argmax — and so which conv
    # position receives the gradient — depends on the conv's summation order (MFMA chain here,
    # MIOpen there), not on the row limiting under test.
    with torch.no_grad():
        cw = ref.conv[0]
        a64 = F.conv2d(win.double(), cw.weight.double(), cw.bias.double(), padding=1)
        v = F.leaky_relu(a64, 0.01) * keep.double() * 1.25
        v = v[:, :, :14, :14].reshape(2 * b, 32, 7, 2, 7, 2).permute(0, 1, 2, 4, 3, 5)
        top = v.reshape(2 * b, 32, 7, 7, 4).topk(2, dim=-1).values
        near = (top[..., 0] != 0) & ((top[..., 0] - top[..., 1]) <= 1e-5 * top[..., 0].abs())
        bad = near.flatten(1).any(1)[:b]
    assert int(bad.sum()) < b // 8
    R[bad] = 0
    g = torch.autograd.grad((q[:b] * R).sum(), list(net.parameters()))
    g_ref = torch.autograd.grad((q_ref[:b] * R.double()).sum(), list(ref.parameters()))
    for (name, _), a, c in zip(net.named_parameters(), g, g_ref):
        assert _close(a, c.float(), 1e-4, 1e-5), name


def test_k_update_block_graph_matches_per_update_replays():
    """K = 4 updates per vector step as one captured graph per index slot (agents/dqn.py
    _capture_k_block) against the K single-update replays (MZ_K_BLOCK off): the same kernels in
    the same order, so parameters, optimizer state and losses agree bit for bit over vector steps
    where the target sync falls at a block's end, strictly inside one (the per-update fallback) and
    between blocks."""
    from mazerl import VectorMazeEnv
    from mazerl.agents import dqn as D
    env = VectorMazeEnv(4, 21, enrich=True, device="cuda", seed=1)
    kw = dict(batch_size=256, capacity=4096, updates_per_step=4, target_every=13,
              updates_per_epoch=100)
    A, B = _mk(True, **kw), _mk(True, **kw)
    B.source.load_state_dict(A.source.state_dict())
    B.target.load_state_dict(A.target.state_dict())
    g = torch.Generator(device="cuda").manual_seed(11)
    n = 4096
    s6, s6n = (torch.randn(n, 6, device="cuda", generator=g) for _ in range(2))
    sw, swn = (torch.randint(0, 2**31 - 1, (n, 22), device="cuda", generator=g, dtype=torch.int32)
               for _ in range(2))
    a = torch.randint(0, 4, (n,), device="cuda", generator=g)
    r = torch.randn(n, device="cuda", generator=g)
    for L in (A, B):
        L.replay.push(s6, sw, a, r, s6n, swn)
    blocks = 0
    for k in range(14):
        old = D.K_BLOCK
        try:
            D.K_BLOCK = True
            blocks += int(A._async and A._k_block_ok())
            la = A.update(env.expand_window, reserve=0)
            D.K_BLOCK = False
            lb = B.update(env.expand_window, reserve=0)
        finally:
            D.K_BLOCK = old
        torch.cuda.synchronize()
        assert A.n_updates == B.n_updates
        assert float(la) == float(lb), k
        for (name, pa), pb in zip(A.source.named_parameters(), B.source.parameters()):
            assert torch.equal(pa, pb), (k, name)
        for pa, pb in zip(A.target.parameters(), B.target.parameters()):
            assert torch.equal(pa, pb), k
    assert torch.equal(A.opt.exp_avg, B.opt.exp_avg) and torch.equal(A.opt.exp_avg_sq, B.opt.exp_avg_sq)
    assert blocks >= 5 and all(gk is not None for gk in A._graphK)
    assert all(gk is None for gk in B._graphK)
    A.finish()
    B.finish()
    env.close()
