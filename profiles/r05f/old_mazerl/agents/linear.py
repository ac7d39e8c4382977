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


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, n_grad=None):
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        ctx.n_grad = n_grad
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        n = ctx.n_grad
        part = n is not None and n < gy.shape[0]
        gy_n, x_n = (gy[:n], x[:n]) if part else (gy, x)
        gx = None
        if ctx.needs_input_grad[0]:
            if part:
                # rows >= n are left unwritten: every consumer below a forward_rows pass (the
                # activation, this class and the stem with the same n_grad) reads rows < n only
                gx = torch.empty(x.shape, dtype=gy.dtype, device=gy.device)
                torch.mm(gy_n, w, out=gx[:n])
            else:
                gx = gy @ w
        gw = gy_n.t() @ x_n if ctx.needs_input_grad[1] else None
        gb = None
        if ctx.has_bias and ctx.needs_input_grad[2]:
            gb = _bias_grad(gy_n)
        return gx, gw, gb, None


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
    def forward(self, x, n_grad=None):
        if x.is_cuda and x.dim() == 2 and torch.is_grad_enabled() and self.weight.requires_grad:
            return _LinearFn.apply(x, self.weight, self.bias, n_grad)
        return F.linear(x, self.weight, self.bias)
