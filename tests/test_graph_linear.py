"""GraphSafeLinear (agents/linear.py) inside a captured HIP graph: forward + backward replayed on
fresh inputs every time must give the eager gradients (rtol 1e-4 of each tensor's scale: the
GEMMs may pick different tilings). The learners' updates are such graphs; torch's own Linear
loses its bias gradient there on PyTorch-ROCm at batch >= 512 (profiles/dbg_graph_linear.py)."""
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("bs", [64, 2048])
def test_graph_safe_linear_replays_match_eager(bs):
    from mazerl.agents.linear import GraphSafeLinear
    torch.manual_seed(0)
    net = nn.Sequential(GraphSafeLinear(1574, 1024), nn.LeakyReLU(), GraphSafeLinear(1024, 512),
                        nn.ReLU(), GraphSafeLinear(512, 4)).cuda()
    X = torch.zeros(bs, 1574, device="cuda")

    def loss():
        return net(X).pow(2).sum()

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for k in range(3):
            X.normal_()
            net.zero_grad(set_to_none=True)
            loss().backward()
    torch.cuda.current_stream().wait_stream(s)
    net.zero_grad(set_to_none=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        loss().backward()
    grads = [p.grad for p in net.parameters()]
    for k in range(5):
        X.normal_()
        g.replay()
        torch.cuda.synchronize()
        got = [x.clone() for x in grads]
        ref = torch.autograd.grad(loss(), list(net.parameters()))
        for (name, _), a, b in zip(net.named_parameters(), got, ref):
            assert torch.allclose(a, b, rtol=1e-4, atol=1e-4 * float(b.abs().max())), (k, name)


def test_graph_safe_linear_is_a_linear():
    from mazerl.agents.linear import GraphSafeLinear
    torch.manual_seed(1)
    a = nn.Linear(7, 3)
    torch.manual_seed(1)
    b = GraphSafeLinear(7, 3)
    assert isinstance(b, nn.Linear)
    assert all(torch.equal(x, y) for x, y in zip(a.parameters(), b.parameters()))
    assert list(a.state_dict()) == list(b.state_dict())


@pytest.mark.gpu
@pytest.mark.parametrize("n,m,ld", [(2048, 1024, 1024), (4096, 512, 512), (37, 4, 4), (1, 64, 68),
                                    (0, 8, 8), (3000, 1028, 1100)])
def test_colsum_matches_torch_sum(n, m, ld):
    """mz_colsum_f32 (the bias gradient of GraphSafeLinear's backward) against torch's f32
    column sum, including a row pitch wider than the columns summed and an empty matrix."""
    from mazerl import _native as N
    g = torch.Generator(device="cuda").manual_seed(n + m)
    full = torch.randn(max(n, 1), ld, device="cuda", generator=g)
    out = torch.full((m,), float("nan"), device="cuda")
    N.check(N.load().mz_colsum_f32(full.data_ptr(), n, m, ld, out.data_ptr(),
                                   torch.cuda.current_stream().cuda_stream))
    ref = full[:n, :m].double().sum(0).float()
    assert torch.allclose(out, ref, rtol=1e-5, atol=1e-4 * max(1.0, n ** 0.5))
    bad = N.load().mz_colsum_f32(full.data_ptr(), n, 6, ld, out.data_ptr(),
                                 torch.cuda.current_stream().cuda_stream)
    assert bad != 0  # m not a multiple of 4
