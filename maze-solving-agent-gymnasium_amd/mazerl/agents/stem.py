"""The Q-network's conv stem for the learner update, from packed window bits (HIP, f32).

QNet.forward((obs6, window)) with `window` an int32 [n, 22] tensor of packed windows (the
replay's storage, DeviceReplay.sw) on the GPU runs this instead of Conv2d -> LeakyReLU ->
[Dropout] -> MaxPool2d -> flatten -> cat (dqn_agent.py:47-57, ddqn_agent.py:18-52):

  forward   mz_stem_forward (csrc/mz_stem.hip): fc.0's f32 input row [n, 1574] in torch's
            flatten order, plus one code byte per feature (pool argmax + gradient class) when
            autograd needs the backward;
  backward  mz_stem_backward: the conv weight / bias gradients (the window is data: no input
            gradient); the obs6 columns' gradient is not needed either. With `n_grad` only the
            first n_grad rows carry a gradient (QNet.forward_rows) and only they are read.

Dropout (DDQN, train mode: SURVEY Q13) draws its masks from a counter hash keyed by a device-side
u64 that is advanced after every call (an in-graph add), so a captured HIP graph replays fresh
masks; P(drop) = round(p * 65536) / 65536. `advance`: "add" (that add), "backward" (the stem's
backward advances the counter instead — one launch fewer per forward; the learner shares one
counter between its source and target nets and moves it on from the source's backward, so each
net's key sequence is the same 0, 1, 2, ... per update as with an add per forward) or "none". Same f32 arithmetic as the torch stem element by
element; the conv and weight-gradient sums associate differently (f32 tolerance).
"""
import torch

from .. import _native as N

FEAT = 1568
IN_DIM = FEAT + 6


class _StemFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, bits, obs6, weight, bias, p, rng, salt, n_grad=None, advance=None):
        n = bits.shape[0]
        L = N.load()
        feat = torch.empty(n, IN_DIM, dtype=torch.float32, device=bits.device)
        need = ctx.needs_input_grad[2] or ctx.needs_input_grad[3]
        code = torch.empty(n, FEAT, dtype=torch.uint8, device=bits.device) if need else None
        st = torch.cuda.current_stream(bits.device).cuda_stream
        N.check(L.mz_stem_forward(bits.data_ptr(), obs6.data_ptr(), n, weight.data_ptr(),
                                  bias.data_ptr(), float(p), rng.data_ptr() if rng is not None else None,
                                  salt, feat.data_ptr(), IN_DIM,
                                  code.data_ptr() if code is not None else None, st))
        if need:
            ctx.save_for_backward(bits, code)
        ctx.p = float(p)
        ctx.n_grad = n if n_grad is None else max(0, min(int(n_grad), n))
        ctx.wp, ctx.bp = weight, bias  # flat gradient segments (agents/flat.py), if any
        ctx.advance = advance  # the dropout counter the backward advances (None: none)
        return feat

    @staticmethod
    def backward(ctx, gfeat):
        bits, code = ctx.saved_tensors
        n = ctx.n_grad  # rows >= n_grad carry no gradient
        bits, code = bits[:n], code[:n]
        L = N.load()
        gfeat = gfeat[:n].contiguous()
        dev = gfeat.device
        ws = torch.empty(max(1, L.mz_stem_workspace_floats(n)), dtype=torch.float32, device=dev)
        from .flat import grad_segment
        dw = grad_segment(ctx.wp, (32, 3, 3, 3))
        db = grad_segment(ctx.bp, (32,))
        ctx.wp = ctx.bp = None
        if dw is None or db is None:
            dw = torch.empty(32, 3, 3, 3, dtype=torch.float32, device=dev)
            db = torch.empty(32, dtype=torch.float32, device=dev)
        st = torch.cuda.current_stream(dev).cuda_stream
        adv = ctx.advance
        ctx.advance = None
        if adv is not None:
            N.check(L.mz_stem_backward_ex(bits.data_ptr(), code.data_ptr(), gfeat.data_ptr(), IN_DIM,
                                          n, ctx.p, ws.data_ptr(), dw.data_ptr(), db.data_ptr(),
                                          adv.data_ptr(), st))
        else:
            N.check(L.mz_stem_backward(bits.data_ptr(), code.data_ptr(), gfeat.data_ptr(), IN_DIM,
                                       n, ctx.p, ws.data_ptr(), dw.data_ptr(), db.data_ptr(), st))
        return None, None, dw, db, None, None, None, None, None


def stem_features(bits, obs6, conv, p, rng, salt, n_grad=None, advance="add"):
    """fc.0 input [n, 1574] f32 from packed windows; `conv` is the stem's nn.Conv2d(3, 32, 3).
    advance: how the dropout counter `rng` moves on (module docstring)."""
    if conv.weight.shape != (32, 3, 3, 3) or conv.bias is None:
        raise ValueError("the bit stem implements Conv2d(3, 32, 3, padding=1) with bias")
    if not bits.is_cuda:
        raise RuntimeError("the packed-window stem runs on the GPU (HIP); use f32 windows on CPU")
    bits = bits.contiguous()
    obs6 = obs6.contiguous().float()
    w = conv.weight.contiguous()
    by_backward = (advance == "backward" and p > 0 and torch.is_grad_enabled()
                   and (w.requires_grad or conv.bias.requires_grad))
    feat = _StemFn.apply(bits, obs6, w, conv.bias, p, rng, salt, n_grad,
                         rng if by_backward else None)
    if p > 0 and (advance == "add" or (advance == "backward" and not by_backward)):
        rng.add_(1)  # next call (or graph replay) draws new masks
    return feat
