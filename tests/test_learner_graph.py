"""VectorDQNLearner's HIP-graph update path against its eager path (same q_loss /
learner_update, dqn_agent.py:121-157, ddqn_agent.py:113-152).

The replay holds one transition repeated, so every sampled batch is the same whatever indices
either path draws; the graph path (3 eager warm-up updates on a side stream, capture, replays,
capturable AdamW with a device-side lr, cosine schedule stepping between replays) must then
track the eager path update for update. Tolerance: capturable AdamW forms its bias corrections
on the device in f32 and rearranges the denominator (the eager path: Python double), which moves
a few elements whose gradient is near eps by a few 1e-6 after 9 steps of lr 1e-3: params agree
within rtol 1e-5 + atol 1e-5 (1 % of one step), losses within rel 1e-4."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _fill(L, n=64, seed=0):
    g = torch.Generator().manual_seed(seed)
    s6 = torch.randn(1, 6, generator=g).repeat(n, 1).cuda()
    sw = torch.randint(0, 2**31, (1, 22), generator=g, dtype=torch.int64)
    sw[:, 21] &= 7
    sw = sw.to(torch.int32).repeat(n, 1).cuda()
    a = torch.full((n,), 2, dtype=torch.int64, device="cuda")
    r = torch.full((n,), 0.45, device="cuda")
    s6n = torch.randn(1, 6, generator=g).repeat(n, 1).cuda()
    swn = torch.roll(sw, 1, 1).contiguous()
    L.replay.push(s6, sw, a, r, s6n, swn)


def test_graph_update_tracks_eager():
    from mazerl import VectorMazeEnv
    from mazerl.agents.dqn import VectorDQNLearner
    env = VectorMazeEnv(4, 21, enrich=True, device="cuda", seed=1)
    mk = lambda g: VectorDQNLearner(4, "cuda", variant="dqn", batch_size=32, capacity=64,  # noqa: E731
                                    updates_per_step=1, target_every=4, updates_per_epoch=2,
                                    seed=5, use_graph=g)
    A, B = mk(True), mk(False)
    assert A.use_graph and not B.use_graph
    B.source.load_state_dict(A.source.state_dict())
    B.target.load_state_dict(A.target.state_dict())
    _fill(A)
    _fill(B)
    for k in range(9):
        la = A.update(env.expand_window)
        lb = B.update(env.expand_window)
        torch.cuda.synchronize()
        assert float(la) == pytest.approx(float(lb), rel=1e-4, abs=1e-7), k
    assert A._graph is not None  # captured after the warm-up updates
    assert float(A.opt.param_groups[0]["lr"]) == pytest.approx(B.opt.param_groups[0]["lr"], rel=1e-6)
    for (na, pa), (nb, pb) in zip(A.source.named_parameters(), B.source.named_parameters()):
        assert torch.allclose(pa, pb, rtol=1e-5, atol=1e-5), na
    for pa, pb in zip(A.target.parameters(), B.target.parameters()):
        assert torch.allclose(pa, pb, rtol=1e-5, atol=1e-5)
    # the fused acting forward sees the graph-updated weights
    from test_qfront import bits_to_window
    bits, obs6 = A.replay.sw[:8].contiguous(), A.replay.s6[:8].contiguous()
    q = A.fused(obs6, bits).float()
    with torch.no_grad():
        ref = A.source((obs6, bits_to_window(bits)))
    assert float((q - ref).abs().max()) <= 0.03 * float(ref.abs().max()) + 1e-3
    env.close()
