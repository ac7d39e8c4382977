"""Flat parameter buffers and the one-launch clamp + AdamW of the learner update.

`flatten_params(net)` moves every parameter of `net` into ONE contiguous f32 buffer (the
parameters become views of it; autograd, state_dict and load_state_dict see ordinary leaf
tensors). Whole-net copies — the target sync `target.load_state_dict(source.state_dict())`
(dqn_agent.py update_target) and the overlapped learner's actor snapshots — are then one
device copy (`copy_flat`) instead of one per tensor.

`FlatAdamW` is the reference's optimizer step with its gradient clamp
(dqn_agent.py:152-157, ddqn_agent.py:148-152: `param.grad.data.clamp_(-1, 1)` for every
parameter, then `torch.optim.AdamW(lr)` with default betas / eps / weight decay) as one HIP
launch over the flat buffer (`mz_adamw_flat`, csrc/mz_optim.hip): torch's multi-tensor kernels
size their grids by tensor chunks and keep ~15 % of the CUs busy on this 8-tensor net. It is a
torch.optim.Optimizer (one param group over the net's parameters) so the LR schedulers drive
it; lr and the step counter live on the device, so the step can be captured in a HIP graph.
"""
import ctypes as C

import torch

from .. import _native as N


FLAT_ALIGN = 256


def flatten_params(net):
    """Make `net`'s parameters views of one flat f32 buffer (idempotent); returns the buffer."""
    flat = getattr(net, "_flat_params", None)
    params = list(net.parameters())
    if flat is not None and _aliases(flat, params, net._flat_sizes):
        return flat  # (a deepcopy clones parameters apart from the buffer: flatten again)
    if not params:
        raise ValueError("net has no parameters")
    dev, dt = params[0].device, params[0].dtype
    if any(p.device != dev or p.dtype != torch.float32 for p in params):
        raise ValueError("flatten_params needs f32 parameters on one device")
    sizes = [(p.numel() + 3) // 4 * 4 for p in params]  # 16-B aligned segments
    # the buffer's length a multiple of FLAT_ALIGN floats (zero tail): it splits into equal,
    # 16-B aligned shards over 2, 4, ... 64 ranks (distributed.GradAllReduce's sharded step)
    flat = torch.zeros(-(-sum(sizes) // FLAT_ALIGN) * FLAT_ALIGN, dtype=dt, device=dev)
    off = 0
    with torch.no_grad():
        for p, n in zip(params, sizes):
            view = flat[off:off + p.numel()].view_as(p)
            view.copy_(p)
            p.data = view
            off += n
    net._flat_params = flat
    net._flat_sizes = sizes
    return flat


def _aliases(flat, params, sizes):
    off = 0
    for p, n in zip(params, sizes):
        if p.data_ptr() != flat.data_ptr() + 4 * off:
            return False
        off += n
    return len(params) == len(sizes)


def flatten_grads(net):
    """Lay the net's parameter gradients out as views of ONE flat f32 buffer shaped like its flat
    parameter buffer (`net._flat_grads`). The learner's backward kernels (GraphSafeLinear's GEMMs
    and column sums, the HIP stem's weight gradients) write each gradient straight into its
    segment and hand autograd a fresh view of it, which becomes `.grad` without a copy. Then the
    optimizer reads one contiguous gradient, and the gradient all-reduce runs on the buffer in
    place: no pack / unpack copies, the 1/N average folded into the AdamW launch
    (distributed.GradAllReduce, FlatAdamW.step). Idempotent; returns the buffer."""
    flat = flatten_params(net)
    g = getattr(net, "_flat_grads", None)
    if g is None or g.numel() != flat.numel() or g.device != flat.device:
        g = torch.zeros_like(flat)
        net._flat_grads = g
    off = 0
    for p, n in zip(net.parameters(), net._flat_sizes):
        p._grad_seg = (g, off)
        off += n
    return g


def grad_segment(p, shape=None):
    """A fresh view of parameter p's segment of its net's flat gradient buffer (None if the net
    has none): the output a backward kernel writes p's gradient into."""
    seg = getattr(p, "_grad_seg", None) if p is not None else None
    if seg is None:
        return None
    g, off = seg
    shape = tuple(p.shape) if shape is None else tuple(shape)
    n = 1
    for d in shape:
        n *= d
    return g[off:off + n].view(shape)


def grads_are_flat(net, params=None):
    """True when every parameter's .grad is its segment of net._flat_grads (what flatten_grads
    sets up and the backward kernels fill)."""
    g = getattr(net, "_flat_grads", None)
    if g is None:
        return False
    off = 0
    for p, n in zip(params if params is not None else net.parameters(), net._flat_sizes):
        if p.grad is None or p.grad.data_ptr() != g.data_ptr() + 4 * off:
            return False
        off += n
    return True


def copy_flat(dst_net, src_net):
    """dst <- src for two flattened nets of the same architecture (one device copy)."""
    dst_net._flat_params.copy_(src_net._flat_params)


class FlatAdamW(torch.optim.Optimizer):
    def __init__(self, net, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, clamp=1.0,
                 write_grad=True):
        flat = flatten_params(net)
        self.net = net
        params = list(net.parameters())
        dev = flat.device
        if dev.type != "cuda":
            raise RuntimeError("FlatAdamW runs on the GPU (HIP)")
        if len(params) > 16:
            raise ValueError("mz_adamw_flat takes at most 16 parameter tensors")
        defaults = dict(lr=torch.tensor(float(lr), dtype=torch.float32, device=dev), betas=betas,
                        eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.flat = flat
        self.sizes = list(net._flat_sizes)
        self.exp_avg = torch.zeros_like(flat)
        self.exp_avg_sq = torch.zeros_like(flat)
        self._step_buf = torch.zeros(1, dtype=torch.float32, device=dev)  # the step count
        self.step_t = self._step_buf[0]
        self.clamp = float(clamp)
        self.grad_scale = 1.0
        # write_grad: the clamped gradient is stored back (torch's clamp_ leaves it in .grad);
        # the learners' hot path turns that 8.56 MB write off
        self.write_grad = bool(write_grad)
        self.lib = N.load()
        self._seg_len = (C.c_int64 * len(params))(*self.sizes)
        self._one_len = (C.c_int64 * 1)(flat.numel())
        # (offset, length) of the flat buffer this rank updates: None = all of it; set by
        # distributed.GradAllReduce when it shards the step (reduce-scatter of the gradients,
        # AdamW over this rank's shard, all-gather of the parameters)
        self.shard = None

    @torch.no_grad()
    def step(self, closure=None):
        if closure is not None:
            raise ValueError("closures are not supported")
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        st = torch.cuda.current_stream(self.flat.device).cuda_stream
        # the average of a gradient all-reduce run in place on the flat gradient buffer
        # (distributed.GradAllReduce) is folded into the launch's gradient scale
        scale = float(self.grad_scale) * float(getattr(self.net, "_allreduce_scale", 1.0))
        if grads_are_flat(self.net, g["params"]):  # one contiguous gradient segment
            o, ln = (0, self._one_len) if self.shard is None else (
                4 * self.shard[0], (C.c_int64 * 1)(self.shard[1]))
            arr = (C.c_void_p * 1)(self.net._flat_grads.data_ptr() + o)
            N.check(self.lib.mz_adamw_flat(self.flat.data_ptr() + o, self.exp_avg.data_ptr() + o,
                                           self.exp_avg_sq.data_ptr() + o, arr, ln, 1,
                                           g["lr"].data_ptr(), self._step_buf.data_ptr(), float(b1),
                                           float(b2), float(g["eps"]), float(g["weight_decay"]),
                                           self.clamp, scale, int(self.write_grad), st))
            return
        if self.shard is not None:
            raise RuntimeError("a sharded step needs the flat gradient buffer (flatten_grads)")
        ptrs = []
        for p, n in zip(g["params"], self.sizes):
            if p.grad is None:
                raise RuntimeError("every parameter needs a gradient")
            if p.grad.numel() != n or not p.grad.is_contiguous():
                # segment lengths are padded to 4: pad the gradient (only tiny bias vectors)
                pad = torch.zeros(n, dtype=p.grad.dtype, device=p.grad.device)
                pad[:p.numel()].copy_(p.grad.reshape(-1))
                p.grad = pad[:p.numel()].view_as(p)
                # keep the padded storage alive with the gradient
            ptrs.append(p.grad.data_ptr())
        arr = (C.c_void_p * len(ptrs))(*ptrs)
        N.check(self.lib.mz_adamw_flat(self.flat.data_ptr(), self.exp_avg.data_ptr(),
                                       self.exp_avg_sq.data_ptr(), arr, self._seg_len, len(ptrs),
                                       g["lr"].data_ptr(), self._step_buf.data_ptr(), float(b1),
                                       float(b2), float(g["eps"]), float(g["weight_decay"]),
                                       self.clamp, scale, int(self.write_grad), st))


class FlatAdamWGroups(torch.optim.Optimizer):
    """PPO's optimizer step (ppo_agent.py:232-236): `clip_grad_norm_(params, max_norm)` then
    `torch.optim.AdamW` with one learning rate per parameter group (ppo_agent.py's actor / critic /
    conv groups), as three HIP launches over the net's flat buffer (`mz_adamw_groups`: squared-norm
    partials, the clip coefficient + step count, AdamW) instead of torch's per-tensor norms, clamp,
    foreach scale and one fused AdamW per group. `groups` = [(params, lr), ...]; the learning rates
    are fixed (the reference schedules none). step() clips with `self.max_norm` (<= 0: no clip),
    so the caller skips its own clip_grad_norm_ (`fused_clip`)."""

    fused_clip = True

    def __init__(self, net, groups, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2,
                 max_norm=0.0):
        flat = flatten_params(net)
        params = list(net.parameters())
        dev = flat.device
        if dev.type != "cuda":
            raise RuntimeError("FlatAdamWGroups runs on the GPU (HIP)")
        if len(params) > 16:
            raise ValueError("mz_adamw_groups takes at most 16 parameter tensors")
        groups = [(list(ps), float(lr)) for ps, lr in groups]
        gid = {}
        for k, (ps, _) in enumerate(groups):
            for p in ps:
                gid[id(p)] = k
        if len(gid) != len(params) or any(id(p) not in gid for p in params):
            raise ValueError("every parameter of the net must be in exactly one group")
        super().__init__([{"params": ps, "lr": lr} for ps, lr in groups],
                         dict(betas=betas, eps=eps, weight_decay=weight_decay))
        self.flat = flat
        self.params = params  # flat-buffer order
        self.sizes = list(net._flat_sizes)
        self.exp_avg = torch.zeros_like(flat)
        self.exp_avg_sq = torch.zeros_like(flat)
        self.step_t = torch.zeros((), dtype=torch.float32, device=dev)
        self.lr_dev = torch.tensor([lr for _, lr in groups], dtype=torch.float32, device=dev)
        self.scratch = torch.zeros(520, dtype=torch.float32, device=dev)
        self.max_norm = float(max_norm)
        self.lib = N.load()
        self._seg_len = (C.c_int64 * len(params))(*self.sizes)
        self._seg_group = (C.c_int32 * len(params))(*[gid[id(p)] for p in params])

    @torch.no_grad()
    def step(self, closure=None):
        if closure is not None:
            raise ValueError("closures are not supported")
        ptrs = []
        for p, n in zip(self.params, self.sizes):
            if p.grad is None:
                raise RuntimeError("every parameter needs a gradient")
            if p.grad.numel() != n or not p.grad.is_contiguous():
                pad = torch.zeros(n, dtype=p.grad.dtype, device=p.grad.device)  # (tiny biases)
                pad[:p.numel()].copy_(p.grad.reshape(-1))
                p.grad = pad[:p.numel()].view_as(p)
            ptrs.append(p.grad.data_ptr())
        arr = (C.c_void_p * len(ptrs))(*ptrs)
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        N.check(self.lib.mz_adamw_groups(
            self.flat.data_ptr(), self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(), arr,
            self._seg_len, self._seg_group, len(ptrs), self.lr_dev.data_ptr(),
            self.step_t.data_ptr(), float(b1), float(b2), float(g["eps"]),
            float(g["weight_decay"]), self.max_norm, self.scratch.data_ptr(),
            torch.cuda.current_stream(self.flat.device).cuda_stream))
