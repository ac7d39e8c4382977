"""Trainer bookkeeping kernels (csrc/mz_trainer.hip) against the torch expressions they replace.

  mz_trainer_tick      steps_done += 1 / = 0 on a win (off_policy_trainer.py:192), the epsilon of
                       dqn_agent.py:118-119 as VectorDQNLearner.epsilon() computes it (f32, bit for
                       bit), wins / episodes counters, and the next act's greedy-row list (== the
                       list mz_greedy_rows builds from the same epsilon)
  mz_greedy_scatter    == torch.argmax over the bf16 Q rows, scattered to the listed instances
  mz_head_bf16         == the torch bf16 conversion (permuted, padded fc1; .to(bfloat16)) bit for bit
  mz_replay_push       == ring slice copies (state half before the step, the rest after; wrap)
  mz_replay_sample_idx rows inside the newest n_avail ring rows, roughly uniform
and the trainer's vector step with these kernels == the torch bookkeeping path, step for step.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _lib():
    from mazerl import _native as N
    return N, N.load()


def _stream():
    return torch.cuda.current_stream().cuda_stream


def test_tick_matches_torch_bookkeeping():
    from mazerl.agents.fused import GreedyRows
    B = 70000  # partial last block
    g = torch.Generator(device=DEV).manual_seed(3)
    term = (torch.rand(B, generator=g, device=DEV) < 0.05).to(torch.uint8)
    trunc = ((torch.rand(B, generator=g, device=DEV) < 0.05) & (term == 0)).to(torch.uint8)
    sd0 = torch.randint(0, 3000, (B,), generator=g, device=DEV).to(torch.float32)
    e0, ef, decay = 0.95, 0.1, 400.0
    sd = sd0.clone()
    wins = torch.zeros((), dtype=torch.int64, device=DEV)
    eps_n = torch.zeros((), dtype=torch.int64, device=DEV) + 5
    gr = GreedyRows(B, torch.device(DEV))
    eps = gr.tick(term, trunc, sd, e0, ef, decay, wins, eps_n, 77, 12)
    torch.cuda.synchronize()
    ref_sd = (sd0 + 1).masked_fill(term.bool(), 0)
    ref_eps = ef + (e0 - ef) * torch.exp(-ref_sd / decay)  # VectorDQNLearner.epsilon()
    assert torch.equal(sd, ref_sd)
    assert torch.equal(eps, ref_eps)
    assert int(wins) == int(term.sum()) and int(eps_n) == 5 + int((term | trunc).sum())
    k = gr.select(eps, 77, 12)  # issued by tick: no second launch
    rows_tick = gr.rows[:k].clone()
    gr2 = GreedyRows(B, torch.device(DEV))
    k2 = gr2.select(ref_eps, 77, 12)
    assert k == k2 and torch.equal(rows_tick, gr2.rows[:k2])


def test_greedy_scatter_is_argmax():
    N, L = _lib()
    m, B = 5000, 9000
    g = torch.Generator(device=DEV).manual_seed(4)
    q = torch.randn(m, 4, generator=g, device=DEV).to(torch.bfloat16)
    q[:100, 2] = q[:100, 0]  # ties: first maximum
    rows = torch.randperm(B, generator=g, device=DEV)[:m].to(torch.int32)
    for k in (0, 1, 4321, m):
        cnt = torch.tensor([k], dtype=torch.int32, device=DEV)
        greedy = torch.full((B,), -7, dtype=torch.int64, device=DEV)
        N.check(L.mz_greedy_scatter(q.data_ptr(), 4, rows.data_ptr(), cnt.data_ptr(), m,
                                    greedy.data_ptr(), _stream()))
        ref = torch.full((B,), -7, dtype=torch.int64, device=DEV)
        ref[rows[:k].long()] = q[:k].float().argmax(1)
        torch.cuda.synchronize()
        assert torch.equal(greedy, ref), k


@pytest.mark.parametrize("variant", ["dqn", "ddqn"])
def test_head_bf16_matches_torch_conversion(variant):
    from mazerl.agents.fused import CONV_OUT, LD, _Head, feature_perm
    from mazerl.agents.nets import QNet
    torch.manual_seed(5)
    net = QNet(variant=variant).to(DEV)
    h = _Head(net.fc)
    h.refresh()
    torch.cuda.synchronize()
    l0, l1, l2 = h.lin
    w0 = torch.zeros(l0.out_features, LD, dtype=torch.bfloat16, device=DEV)
    w0[:, :CONV_OUT] = l0.weight.detach().index_select(1, feature_perm(DEV)).to(torch.bfloat16)
    w0[:, CONV_OUT:l0.in_features] = l0.weight.detach()[:, CONV_OUT:].to(torch.bfloat16)
    ref = [(w0, l0.bias), (l1.weight, l1.bias), (l2.weight, l2.bias)]
    for (dw, db), (rw, rb) in zip(h._w, ref):
        assert torch.equal(dw, rw.detach().to(torch.bfloat16))
        assert torch.equal(db, rb.detach().to(torch.bfloat16))


def test_replay_push_state_rest_wraps():
    from mazerl.replay import DeviceReplay
    C, n = 1000, 384
    a = DeviceReplay(C, DEV)
    b = DeviceReplay(C, DEV)
    g = torch.Generator(device=DEV).manual_seed(6)
    for it in range(4):  # ptr 0, 384, 768 (wraps), 152
        s6 = torch.randn(n, 6, generator=g, device=DEV)
        sw = torch.randint(-2**31, 2**31 - 1, (n, 22), generator=g, device=DEV, dtype=torch.int32)
        act = torch.randint(0, 4, (n,), generator=g, device=DEV, dtype=torch.int32)
        r = torch.randn(n, generator=g, device=DEV)
        s6n = torch.randn(n, 6, generator=g, device=DEV)
        swn = torch.randint(-2**31, 2**31 - 1, (n, 22), generator=g, device=DEV, dtype=torch.int32)
        a.push_state(s6, sw)
        a.push_rest(act, r, s6n, swn)
        b.push(s6, sw, act, r, s6n, swn)
        assert a.ptr == b.ptr and a.size == b.size
    torch.cuda.synchronize()
    for x, y in ((a.s6, b.s6), (a.sw, b.sw), (a.a, b.a), (a.r, b.r), (a.s6n, b.s6n), (a.swn, b.swn)):
        assert torch.equal(x, y)
    assert float(a.size_dev) == float(b.size_dev)


def test_replay_sample_idx_range():
    N, L = _lib()
    C, n = 100000, 1 << 16
    out = torch.empty(n, dtype=torch.int64, device=DEV)
    for newest, avail in ((99999, 100000), (10, 5000), (70000, 1)):
        N.check(L.mz_replay_sample_idx(9, 3, newest, avail, C, out.data_ptr(), n, _stream()))
        torch.cuda.synchronize()
        back = (newest - out) % C  # 0 .. avail - 1
        assert int(back.min()) >= 0 and int(back.max()) < avail
        assert bool(((out >= 0) & (out < C)).all())
        if avail > 1000:
            h = torch.histc(back.double(), bins=10, min=0, max=avail)
            assert float(h.min()) > 0.9 * n / 10 and float(h.max()) < 1.1 * n / 10


def test_vector_step_kernels_match_torch_bookkeeping():
    """Two trainers on identical envs (no learner updates: batch > pushes): the bookkeeping kernels
    + ring push vs the torch path give the same actions, replay rows and counters."""
    from mazerl import VectorMazeEnv
    from mazerl.agents.dqn import VectorDQNLearner
    from mazerl.trainers.vector_trainer import VectorOffPolicyTrainer
    B = 3000
    runs = []
    for fast in (True, False):
        env = VectorMazeEnv(B, 15, enrich=True, device=DEV, seed=0x5EED0000, window=False,
                            window_bits=True, done_list=False)
        L = VectorDQNLearner(B, DEV, variant="dqn", batch_size=10**6, capacity=1 << 15,
                             eps_decay=30.0, seed=1)
        tr = VectorOffPolicyTrainer(env, L, seed=3, bank=False, fused=fast)
        acts = []
        for _ in range(120):
            tr.vector_step()
            acts.append(env.actions.clone())
        torch.cuda.synchronize()
        runs.append((torch.stack(acts), L.replay, L.steps_done.clone(), int(tr.wins),
                     int(tr.episodes)))
        env.close()
    (a0, r0, s0, w0, e0), (a1, r1, s1, w1, e1) = runs
    assert torch.equal(a0, a1)
    assert torch.equal(s0, s1) and (w0, e0) == (w1, e1) and e0 > 0
    for x, y in ((r0.s6, r1.s6), (r0.sw, r1.sw), (r0.a, r1.a), (r0.r, r1.r), (r0.s6n, r1.s6n),
                 (r0.swn, r1.swn)):
        assert torch.equal(x, y)


@pytest.mark.parametrize("variant", ["ddqn", "dqn"])
def test_fused_q_loss_matches_torch_loss(variant):
    """mz_q_loss / mz_q_loss_backward (agents/dqn.py _QLossFn) == gather / max / mse_loss and their
    autograd backward: loss and every parameter gradient, on packed-window replay rows (f32)."""
    from mazerl.agents import dqn as D
    from mazerl.agents.nets import QNet
    torch.manual_seed(7)
    src = QNet(variant=variant).to(DEV).eval()  # dropout off: both paths see the same stem
    tgt = QNet(variant=variant).to(DEV).eval()
    b = 512
    g = torch.Generator(device=DEV).manual_seed(8)

    def bits():
        x = torch.randint(-2**31, 2**31 - 1, (b, 22), generator=g, device=DEV, dtype=torch.int32)
        x[:, 21] &= (1 << (675 - 21 * 32)) - 1
        return x
    s = (torch.rand(b, 6, generator=g, device=DEV), bits())
    sn = (torch.rand(b, 6, generator=g, device=DEV), bits())
    a = torch.randint(0, 4, (b,), generator=g, device=DEV)
    r = torch.randn(b, generator=g, device=DEV)
    out = []
    for fused in (True, False):
        D.FUSED_LOSS = fused
        try:
            src.zero_grad(set_to_none=True)
            loss = D.q_loss(src, tgt, s, a, r, sn, 0.7, variant == "ddqn")
            loss.backward()
        finally:
            D.FUSED_LOSS = True
        out.append((loss.detach().clone(), [p.grad.clone() for p in src.parameters()]))
    (l0, g0), (l1, g1) = out
    torch.testing.assert_close(l0, l1, rtol=1e-6, atol=0)
    for x, y in zip(g0, g1):
        torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("ddqn", [True, False])
def test_fused_q_loss_propagates_nan_like_torch(ddqn):
    """mz_q_loss on rows holding NaN: torch's argmax takes the first NaN as the maximum
    (DDQN's target column) and max(1)[0] propagates NaN (DQN), so the per-row diff — and the
    loss — are NaN exactly where the torch expression's are (a diverging net must not report a
    finite loss)."""
    from mazerl.agents.dqn import _QLossFn
    nan = float("nan")
    q = torch.tensor([[1., 2., 3., 4.], [0.5, nan, 0.1, 0.2], [1., 1., 1., 1.], [2., 0., 0., 0.]],
                     device=DEV)
    qn = torch.tensor([[0., nan, 5., nan], [1., 2., 3., 4.], [nan, 0., 0., 0.], [3., 1., 9., 2.]],
                      device=DEV)
    qt = torch.tensor([[1., nan, 3., 4.], [1., nan, 0., 0.], [5., 6., 7., 8.], [1., 2., 3., nan]],
                      device=DEV)
    a = torch.tensor([0, 2, 1, 3], device=DEV)
    r = torch.tensor([0.5, -0.05, 1.0, 0.45], device=DEV)
    diff_ref = []
    for i in range(4):
        v = qt[i, torch.argmax(qn[i])] if ddqn else qt[i].max()
        diff_ref.append(q[i, a[i]] - (v * 0.7 + r[i]))
    diff_ref = torch.stack(diff_ref)
    loss = _QLossFn.apply(q, qn if ddqn else None, qt, a, r, 0.7, 4)
    torch.cuda.synchronize()
    assert torch.isnan(loss) and torch.isnan((diff_ref ** 2).mean())
    # row by row: the kernel's diff has NaN in the rows torch's has
    from mazerl import _native as N
    diff = torch.empty(4, device=DEV)
    out = torch.empty((), device=DEV)
    N.check(N.load().mz_q_loss(q.data_ptr(), 4, qn.data_ptr() if ddqn else None, 4 if ddqn else 0,
                               qt.data_ptr(), 4, a.data_ptr(), r.data_ptr(), 0.7, 4, out.data_ptr(),
                               diff.data_ptr(), torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    assert torch.equal(torch.isnan(diff), torch.isnan(diff_ref)), (diff, diff_ref)
    fin = ~torch.isnan(diff_ref)
    assert torch.equal(diff[fin], diff_ref[fin])
