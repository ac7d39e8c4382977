"""nn.Linear whose backward is safe to capture in a HIP graph on PyTorch-ROCm.

Replaying a captured forward + backward of torch's own Linear at batch >= 512 gives a wrong bias
gradient for a Linear whose input needs no gradient (the first layer of every head here) from the
second replay on — the weight and input gradients and every other layer are right, and eager
execution is right (profiles/dbg_graph_linear.py reproduces it: 5 of 6 replays wrong at batch
2,048, 0 of 6 at 256; torch 2.10.0+rocm7.0, hipBLASLt or rocBLAS alike). The learners' updates
are captured graphs (agents/dqn.py, agents/ppo.py), so on the GPU their Linear layers compute the
same three products explicitly: dX = dY W, dW = dY^T X (GEMMs) and db = dY^T 1 (a GEMV) — the
same arithmetic class as torch's, and correct under replay (tests/test_graph_linear.py).
Module and parameter names are nn.Linear's, so state_dicts interchange with the reference's.

`n_grad` (QNet.forward_rows): only the first n_grad rows of the input carry a gradient — the
rest are rows stacked under them for the forward only (DDQN's source(s') beside source(s)). The
backward then reads those rows only: dW and db over n_grad rows, dX for them alone. db is one
HIP column-sum launch (mz_colsum_f32) instead of rocBLAS's GEMV against a ones vector.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


_WS = {}


def mm_x3(a, b, bias=None, act=0, out=None):
    """a @ b.T (+ bias, act 0 / 1 LeakyReLU(0.01) / 2 ReLU) for f32 2-D views a [M, K], b [N, K]
    with one unit stride each, on the bf16 MFMA in split precision (mz_gemm_x3: hi*hi + hi*lo +
    lo*hi, f32 accumulate). out: [M, N] with unit column stride (default: a new tensor)."""
    from .. import _native as N
    M, K = a.shape
    Nn = b.shape[0]
    if out is None:
        out = torch.empty(M, Nn, dtype=torch.float32, device=a.device)
    lib = N.load()
    key = (M, Nn, K)
    if key not in _WS:
        f = N.C.c_int64()
        N.check(lib.mz_gemm_x3_workspace(M, Nn, K, N.C.byref(f)))
        _WS[key] = f.value
    ws = torch.empty(_WS[key], dtype=torch.float32, device=a.device)
    N.check(lib.mz_gemm_x3(a.data_ptr(), a.stride(0), a.stride(1), b.data_ptr(), b.stride(0),
                           b.stride(1), out.data_ptr(), out.stride(0),
                           bias.data_ptr() if bias is not None else None, M, Nn, K, int(act),
                           ws.data_ptr(),
                           torch.cuda.current_stream(a.device).cuda_stream))
    return out


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, n_grad=None, x3=False):
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        ctx.n_grad = n_grad
        ctx.x3 = x3
        if x3:
            return mm_x3(x, w, b.detach() if b is not None else None)
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        n = ctx.n_grad
        part = n is not None and n < gy.shape[0]
        gy_n, x_n = (gy[:n], x[:n]) if part else (gy, x)
        x3 = ctx.x3
        gx = None
        if ctx.needs_input_grad[0]:
            if part:
                # rows >= n are left unwritten: every consumer below a forward_rows pass (the
                # activation, this class and the stem with the same n_grad) reads rows < n only
                gx = torch.empty(x.shape, dtype=gy.dtype, device=gy.device)
                if x3:
                    mm_x3(gy_n, w.t(), out=gx[:n])
                else:
                    torch.mm(gy_n, w, out=gx[:n])
            else:
                gx = mm_x3(gy, w.t()) if x3 else gy @ w
        gw = None
        if ctx.needs_input_grad[1]:
            gw = mm_x3(gy_n.t(), x_n.t()) if x3 else gy_n.t() @ x_n
        gb = None
        if ctx.has_bias and ctx.needs_input_grad[2]:
            gb = _bias_grad(gy_n)
        return gx, gw, gb, None, None


def _bias_grad(gy):
    """db = dY^T 1: one HIP column-sum launch (mz_colsum_f32) for f32 rows whose width is a
    multiple of 4; else a GEMV against ones."""
    m = gy.shape[1]
    if gy.dtype == torch.float32 and m % 4 == 0:
        from .. import _native as N
        g = gy if gy.is_contiguous() and gy.data_ptr() % 16 == 0 else gy.contiguous()
        out = torch.empty(m, dtype=torch.float32, device=gy.device)
        N.check(N.load().mz_colsum_f32(g.data_ptr(), g.shape[0], m, m, out.data_ptr(),
                                       torch.cuda.current_stream(gy.device).cuda_stream))
        return out
    return torch.mv(gy.t(), torch.ones(gy.shape[0], dtype=gy.dtype, device=gy.device))


class GraphSafeLinear(nn.Linear):
    """`gemm = "x3"` (set by the learners on their large layers, LEARNER_GEMM): forward, dX and dW
    through mz_gemm_x3 (bf16x3 split precision) instead of f32 hipBLASLt GEMMs."""
    gemm = "f32"

    def _x3(self, x):
        return self.gemm == "x3" and x.is_cuda and x.dtype == torch.float32 and \
            self.in_features % 2 == 0 and self.out_features % 2 == 0

    def forward(self, x, n_grad=None):
        if x.is_cuda and x.dim() == 2 and torch.is_grad_enabled() and self.weight.requires_grad:
            return _LinearFn.apply(x, self.weight, self.bias, n_grad, self._x3(x))
        if x.dim() == 2 and self._x3(x):
            return mm_x3(x, self.weight.detach(), self.bias.detach() if self.bias is not None else None)
        return F.linear(x, self.weight, self.bias)


def set_learner_gemm(net, mode, min_features=64):
    """Route the GEMMs of `net`'s GraphSafeLinear layers with both dimensions >= min_features
    (fc1 / fc2 of the reference's heads; the 4- and 1-wide output layers stay f32) through
    mode "x3" (mz_gemm_x3) or "f32" (torch / hipBLASLt)."""
    for m in net.modules():
        if isinstance(m, GraphSafeLinear):
            big = m.in_features >= min_features and m.out_features >= min_features
            m.gemm = mode if big else "f32"
    return net
