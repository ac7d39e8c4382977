"""FlatAdamW (agents/flat.py, csrc/mz_optim.hip: the reference's per-parameter
grad.clamp_(-1, 1) + torch.optim.AdamW step, dqn_agent.py:152-157, as one launch over a flat
buffer) against torch.optim.AdamW (single-tensor path) + clamp_ on the same QNet, with a cosine
schedule stepping the device-side lr. Same formula and operation order; torch's kernels may
contract multiply-adds, so params agree within rtol 1e-5 / atol 1e-6 after 25 steps and the
moments within rtol 1e-4 (relative to each tensor's scale)."""
import copy

import pytest
import torch
from torch.optim import lr_scheduler

pytestmark = pytest.mark.gpu


def test_flat_adamw_matches_torch_adamw_with_clamp():
    from mazerl.agents.flat import FlatAdamW
    from mazerl.agents.nets import QNet
    torch.manual_seed(0)
    A = QNet(variant="ddqn").cuda()
    B = copy.deepcopy(A)
    oa = FlatAdamW(A, lr=1e-3)
    ob = torch.optim.AdamW(B.parameters(), lr=1e-3, foreach=False)
    sa = lr_scheduler.CosineAnnealingLR(oa, T_max=7, eta_min=1e-5)
    sb = lr_scheduler.CosineAnnealingLR(ob, T_max=7, eta_min=1e-5)
    assert all(p.data_ptr() >= A._flat_params.data_ptr() for p in A.parameters())
    g = torch.Generator(device="cuda").manual_seed(1)
    for k in range(25):
        for pa, pb in zip(A.parameters(), B.parameters()):
            gr = torch.randn(pa.shape, device="cuda", generator=g) * (0.5 if k % 3 else 3.0)
            pa.grad = gr.clone()
            pb.grad = gr.clone()
        oa.step()
        for p in B.parameters():
            p.grad.data.clamp_(-1, 1)
        ob.step()
        if k % 4 == 3:
            sa.step()
            sb.step()
    torch.cuda.synchronize()
    assert float(oa.param_groups[0]["lr"]) == pytest.approx(ob.param_groups[0]["lr"], rel=1e-6)
    assert float(oa.step_t) == 25.0
    for (n, pa), pb in zip(A.named_parameters(), B.parameters()):
        assert torch.allclose(pa, pb, rtol=1e-5, atol=1e-6), n
        assert torch.equal(pa.grad, pb.grad), n  # clamped in place, like clamp_
    off = 0
    for pb, n in zip(B.parameters(), oa.sizes):
        st = ob.state[pb]
        m = oa.exp_avg[off:off + pb.numel()].view_as(pb)
        v = oa.exp_avg_sq[off:off + pb.numel()].view_as(pb)
        assert torch.allclose(m, st["exp_avg"], rtol=1e-4, atol=1e-4 * float(st["exp_avg"].abs().max()))
        assert torch.allclose(v, st["exp_avg_sq"], rtol=1e-4, atol=1e-4 * float(st["exp_avg_sq"].abs().max()))
        off += n


def test_flat_params_survive_state_dict_and_copy():
    from mazerl.agents.flat import copy_flat, flatten_params
    from mazerl.agents.nets import QNet
    torch.manual_seed(0)
    A, B = QNet(variant="dqn").cuda(), QNet(variant="dqn").cuda()
    ref = {k: v.clone() for k, v in A.state_dict().items()}
    fa, fb = flatten_params(A), flatten_params(B)
    assert flatten_params(A) is fa  # idempotent
    for k, v in A.state_dict().items():
        assert torch.equal(v, ref[k]), k
    copy_flat(B, A)
    for (k, v), w in zip(B.state_dict().items(), A.state_dict().values()):
        assert torch.equal(v, w), k
    C = copy.deepcopy(A)  # deepcopy clones the parameters apart from the buffer
    fc = flatten_params(C)
    assert fc.data_ptr() != fa.data_ptr()
    assert all(torch.equal(x, y) for x, y in zip(C.parameters(), A.parameters()))


def test_flat_adamw_step_counts_are_independent_and_graph_safe():
    """The step count is a plain f32 [1] (include/mazerl.h mz_adamw_flat), advanced by a
    one-thread launch behind the update on the caller's stream. Two optimizers interleaved on
    two streams, eagerly and as captured-graph replays, each advance their own count by exactly
    one per step."""
    from mazerl.agents.flat import FlatAdamW
    from mazerl.agents.nets import QNet
    torch.manual_seed(3)
    A, B = QNet(variant="dqn").cuda(), QNet(variant="ddqn").cuda()
    oa, ob = FlatAdamW(A, lr=1e-3), FlatAdamW(B, lr=1e-3)
    assert oa._step_buf.numel() == 1 and ob._step_buf.numel() == 1
    for p in list(A.parameters()) + list(B.parameters()):
        p.grad = torch.randn_like(p) * 1e-3
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for k in range(7):
        with torch.cuda.stream(s1):
            oa.step()
        with torch.cuda.stream(s2):
            ob.step()
            ob.step()
    torch.cuda.synchronize()
    assert float(oa.step_t) == 7.0 and float(ob.step_t) == 14.0
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            oa.step()
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(5):
        g.replay()
    ob.step()
    torch.cuda.synchronize()
    assert float(oa.step_t) == 12.0 and float(ob.step_t) == 15.0


def test_learner_gradients_land_in_the_flat_buffer():
    """VectorDQNLearner's backward writes every source-net gradient into its segment of ONE flat
    buffer (agents/flat.py flatten_grads: GraphSafeLinear's GEMM / column-sum outputs and the HIP
    stem's weight gradients, kept by autograd as .grad without a copy) — eager and captured — so
    FlatAdamW reads one contiguous gradient and a gradient all-reduce runs on it in place."""
    from mazerl import VectorMazeEnv
    from mazerl.agents.dqn import VectorDQNLearner
    from mazerl.agents.flat import grads_are_flat
    from test_learner_graph import _fill
    env = VectorMazeEnv(4, 21, enrich=True, device="cuda", seed=1)
    L = VectorDQNLearner(4, "cuda", variant="ddqn", batch_size=32, capacity=64, seed=3)
    _fill(L)
    for _ in range(5):  # 3 eager warm-up updates, the capture, a replay
        L.update(env.expand_window)
        torch.cuda.synchronize()
        assert grads_are_flat(L.source)
        g = L.source._flat_grads
        assert float(g.abs().sum()) > 0
        off = 0
        for p, n in zip(L.source.parameters(), L.source._flat_sizes):
            assert p.grad.data_ptr() == g.data_ptr() + 4 * off
            off += n
    assert L._graph is not None
    env.close()
