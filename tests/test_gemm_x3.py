"""Split-precision learner GEMM (mz_gemm_x3, csrc/mz_gemm.hip) vs float64 references.

- every operand layout (k-contiguous / row-contiguous A and B), edge tiles (M, N not multiples of
  128, K not a multiple of 32), split-K and single-pass grids, bias and both activations: the
  result equals the bf16x3 product (hi*hi + hi*lo + lo*hi of the operands' bf16 halves) computed in
  float64 to 2e-6 of max|C| (f32 accumulation order only), and the f32 product to 3e-5 of max|C|;
- deterministic (bit-identical repeat), strided views (no copies), captured in a HIP graph;
- GraphSafeLinear(gemm="x3") forward / dX / dW / db of a two-layer head track the f32 layer to
  1e-4 relative (the reference's optimize_model arithmetic, dqn_agent.py:121-157);
- any alignment, odd K and odd strides (the operand images are built with scalar loads).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _bf(x):
    return x.to(torch.bfloat16).to(torch.float64)


def _x3_ref(a, b):
    a, b = a.double(), b.double()
    ah, bh = _bf(a), _bf(b)
    al, bl = _bf(a - ah), _bf(b - bh)
    return ah @ bh.t() + ah @ bl.t() + al @ bh.t()


def _layout(x, kc):
    """x [R, K] as a view with unit stride along k (kc) or along rows (a transposed copy)."""
    return x.contiguous() if kc else x.t().contiguous().t()


@pytest.mark.parametrize("M,N,K", [(2048, 1024, 1574), (2048, 512, 1024), (1024, 1574, 2048),
                                   (300, 200, 96), (130, 2, 64), (4096, 1024, 1574)])
@pytest.mark.parametrize("ak,bk", [(True, True), (True, False), (False, True), (False, False)])
def test_x3_matches_split_reference(M, N, K, ak, bk):
    from mazerl.agents.linear import mm_x3
    g = torch.Generator(device="cuda:0").manual_seed(M * 7 + N * 3 + K + 2 * ak + bk)
    a = torch.randn(M, K, device="cuda:0", generator=g)
    b = torch.randn(N, K, device="cuda:0", generator=g) * 0.05
    c = mm_x3(_layout(a, ak), _layout(b, bk))
    ref3 = _x3_ref(a, b)
    ref = a.double() @ b.double().t()
    s = ref.abs().max()
    assert float((c.double() - ref3).abs().max() / s) < 2e-6
    assert float((c.double() - ref).abs().max() / s) < 3e-5
    c2 = mm_x3(_layout(a, ak), _layout(b, bk))
    assert torch.equal(c, c2)


@pytest.mark.parametrize("act", [0, 1, 2])
def test_bias_and_activation(act):
    from mazerl.agents.linear import mm_x3
    g = torch.Generator(device="cuda:0").manual_seed(act)
    a = torch.randn(777, 512, device="cuda:0", generator=g)
    b = torch.randn(300, 512, device="cuda:0", generator=g) * 0.05
    bias = torch.randn(300, device="cuda:0", generator=g)
    c = mm_x3(a, b, bias=bias, act=act)
    y = _x3_ref(a, b) + bias.double()
    if act == 1:
        y = torch.where(y > 0, y, y * 0.01)
    elif act == 2:
        y = y.clamp_min(0)
    assert float((c.double() - y).abs().max() / y.abs().max()) < 2e-6


def test_strided_out_and_graph_capture():
    from mazerl.agents.linear import mm_x3
    a = torch.randn(2048, 1600, device="cuda:0")[:, :1574]  # a padded-row view, as the stem writes
    b = torch.randn(1024, 1574, device="cuda:0") * 0.03
    out = torch.zeros(2048, 1100, device="cuda:0")
    eager = mm_x3(a, b).clone()
    mm_x3(a, b, out=out[:, 50:1074])
    assert torch.equal(out[:, 50:1074], eager) and float(out[:, :50].abs().max()) == 0.0
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        mm_x3(a, b)
    torch.cuda.current_stream().wait_stream(st)
    gph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gph):
        c = mm_x3(a, b)
    a.mul_(2.0)  # exact: every split half, product and partial sum doubles
    gph.replay()
    torch.cuda.synchronize()
    assert torch.equal(c, 2.0 * eager)


def test_unaligned_odd_views():
    """Operands at 4-B offsets with odd K and odd strides: the images are built with scalar loads,
    so any view of f32 memory works."""
    from mazerl.agents.linear import mm_x3
    a = torch.randn(301, 167, device="cuda:0")
    b = torch.randn(77, 167, device="cuda:0")
    av, bv = a[:, 1:166], b[:, 1:166]  # K = 165, bases 4-B aligned
    c = mm_x3(av, bv)
    ref = _x3_ref(av, bv)
    assert float((c.double() - ref).abs().max() / ref.abs().max()) < 2e-6
    ct = mm_x3(av.t().contiguous().t(), bv)
    assert torch.equal(c, ct)


def test_linear_layer_x3_tracks_f32():
    """One GraphSafeLinear, the same upstream gradient: y, dX, dW, db within 3e-5 of max|.| of the
    f32 layer's (a deeper head also differs where a LeakyReLU's sign flips between the two
    precisions — the learners are checked against the reference's fixtures instead,
    tests/test_learner.py::test_q_loss_matches_reference_gpu_x3)."""
    from mazerl.agents.linear import GraphSafeLinear, set_learner_gemm
    torch.manual_seed(0)
    for fin, fout in ((1574, 1024), (1024, 512)):
        lin = GraphSafeLinear(fin, fout).cuda()
        x = torch.randn(2048, fin, device="cuda:0", requires_grad=True)
        gy = torch.randn(2048, fout, device="cuda:0") * 1e-3
        outs = {}
        for mode in ("f32", "x3"):
            set_learner_gemm(lin, mode)
            lin.zero_grad()
            x.grad = None
            y = lin(x)
            y.backward(gy)
            outs[mode] = [y.detach().clone(), x.grad.clone(), lin.weight.grad.clone(),
                          lin.bias.grad.clone()]
        assert lin.gemm == "x3"
        for u, v in zip(outs["f32"], outs["x3"]):
            assert float((u - v).abs().max() / u.abs().max()) < 3e-5
