"""Acting-head kernels: mz_leaky_relu_bf16 against F.leaky_relu (bit-exact on bf16, edge values
and ragged sizes) and the fc2 bias + ReLU epilogue (torch._addmm_activation) against
relu(linear) as used by agents/fused.py _Head."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _lib():
    from mazerl import _native as N
    return N, N.load()


def _leaky_hip(x, slope):
    N, lib = _lib()
    N.check(lib.mz_leaky_relu_bf16(x.data_ptr(), x.numel(), float(slope),
                                   torch.cuda.current_stream().cuda_stream))
    return x


@pytest.mark.parametrize("n", [8, 136, 1000 * 8, 4096 * 1024])
def test_leaky_bf16_bit_exact(n):
    g = torch.Generator(device="cuda").manual_seed(n)
    x = (torch.randn(n, device="cuda", generator=g) * 10).to(torch.bfloat16)
    edge = torch.tensor([0.0, -0.0, 1e-38, -1e-38, -3e38, 3e38, float("inf"), float("-inf"),
                         -1.0, 1.0], device="cuda").to(torch.bfloat16)
    k = min(n, edge.numel())
    x[:k] = edge[:k]
    ref = F.leaky_relu(x, 0.01)
    got = _leaky_hip(x.clone(), 0.01)
    torch.cuda.synchronize()
    assert torch.equal(got.view(torch.int16), ref.view(torch.int16))


def test_leaky_bf16_rejects_ragged():
    _, lib = _lib()
    x = torch.zeros(1008, device="cuda", dtype=torch.bfloat16)
    st = torch.cuda.current_stream().cuda_stream
    assert lib.mz_leaky_relu_bf16(x.data_ptr(), 1003, 0.01, st) != 0       # n % 8
    assert lib.mz_leaky_relu_bf16(x.data_ptr() + 2, 1000, 0.01, st) != 0   # 16-B alignment


def test_head_leaky_routes_agree():
    """_leaky_ sends multiples of 8 to the kernel and the rest to torch; same values."""
    from mazerl.agents.fused import _leaky_
    for n in (1003, 1000):
        x = torch.randn(n, device="cuda").to(torch.bfloat16)
        assert torch.equal(_leaky_(x.clone(), 0.01).view(torch.int16),
                           F.leaky_relu(x, 0.01).view(torch.int16))


def test_addmm_activation_matches_relu_linear():
    g = torch.Generator(device="cuda").manual_seed(3)
    h = torch.randn(4096, 1024, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(512, 1024, device="cuda", generator=g) * 0.03).to(torch.bfloat16)
    b = torch.randn(512, device="cuda", generator=g).to(torch.bfloat16)
    ref = F.relu(F.linear(h, w, b))
    got = torch._addmm_activation(b, h, w.t())
    # same GEMM with the epilogue fused: measured bit-identical (profiles/exp_epilogue.py);
    # the bound leaves one bf16 ulp in case the library picks another accumulation order
    diff = (ref.float() - got.float()).abs()
    assert float(diff.max()) <= float(ref.float().abs().max()) * 2 ** -7
    assert bool((got >= 0).all())
