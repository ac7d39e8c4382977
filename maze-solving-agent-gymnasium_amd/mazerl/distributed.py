"""Multi-GPU plumbing: one process per GPU, env shards with no data-path exchange, and the
learner's data-parallel gradient all-reduce over RCCL (torch.distributed backend "nccl" on ROCm;
"gloo" on CPU for tests).

Per update the source net's gradients (2,140,548 fp32 = 8.56 MB at full size) are flattened into
ONE bucket and all-reduced once (xGMI ring: 2(N-1)/N x 8.56 MB per GPU, ~0.1 ms at ~153 GB/s per
link), then averaged; grad.clamp_(-1, 1) runs after the average so N ranks reproduce the
single-GPU update on the union batch (dqn_agent.py:152-153). The DQN / DDQN learners run that
collective as a reduce-scatter, AdamW over each rank's 1/N shard, and an all-gather of the
parameters (GradAllReduce.attach): the same bytes, 1/N of the optimizer's work per rank. Instance ids are global
(rank * B + i) so maze seeds do not depend on the GPU count.
"""
import os

import torch
import torch.distributed as dist


def init_from_env(backend=None):
    """Initialise torch.distributed from torchrun's env vars; returns (rank, world, local)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ngpu = torch.cuda.device_count()  # counting does not initialise the GPU
    if ngpu > 0:
        local %= ngpu  # rehearsal: several ranks share a GPU
    if world > 1 and not dist.is_initialized():
        if backend is None:  # MZ_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs
            backend = os.environ.get("MZ_DIST_BACKEND") or ("nccl" if ngpu > 0 else "gloo")
        kw = {}
        if backend == "nccl":  # bind each rank's RCCL communicator to its GPU up front
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend, init_method="env://", **kw)
    return rank, world, local


class GradAllReduce:
    """Callable(net): average the net's gradients over the process group in one flat bucket.

    The three phases are also exposed separately so a HIP-graph-captured learner can replay
    "backward + pack" and "unpack + clamp + AdamW" as two graphs with the collective between
    them (agents/dqn.py): pack / unpack are plain device copies, reduce is the one all-reduce.

    Sharded step (`attach(net, opt)` with a FlatAdamW over flat gradients, the DQN / DDQN
    learners): the all-reduce becomes a reduce-scatter of the flat gradient buffer (in place:
    rank r receives the summed shard r), the optimizer's one launch runs over shard r only (the
    clamp and AdamW are elementwise: each element's update is the one the full step computes),
    and `gather(net)` all-gathers the updated parameter shards (in place). The same bytes cross
    the links as with the all-reduce (a ring all-reduce IS a reduce-scatter + all-gather), but
    each rank's AdamW reads / writes 1/N of the 2.14 M parameters and moments."""

    def __init__(self, group=None, shard=None):
        """shard: None = shard the step when attach() can and there are >= 2 ranks; True = also
        with one rank (the collectives then run as local copies: tests); False = all-reduce."""
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self._flat = None
        self.shard_mode = shard
        self.sharded = False

    def attach(self, net, opt):
        """Shard `opt`'s step over the ranks when it can be (FlatAdamW, flat gradients, a flat
        buffer that splits into 16-B aligned shards); returns whether it does."""
        from .agents.flat import FlatAdamW
        g = getattr(net, "_flat_grads", None)
        n = 0 if g is None else g.numel()
        want = self.shard_mode is True or (self.shard_mode is None and self.world > 1)
        if want and isinstance(opt, FlatAdamW) and g is not None and n % (4 * self.world) == 0:
            S = n // self.world
            opt.shard = (self.rank * S, S)
            self._net, self._S = net, S
            self.sharded = True
        return self.sharded

    def pack(self, net):
        from .agents.flat import grads_are_flat
        if grads_are_flat(net):
            # the backward wrote the gradients into one flat buffer (agents/flat.py
            # flatten_grads): reduce it in place — no pack copies
            self._flat = net._flat_grads
            return
        if self.sharded:
            raise RuntimeError("a sharded step needs the flat gradient buffer")
        grads = [p.grad for p in net.parameters()]
        n = sum(g.numel() for g in grads)
        if self._flat is None or self._flat.numel() != n or self._flat.device != grads[0].device:
            self._flat = torch.empty(n, dtype=grads[0].dtype, device=grads[0].device)
        off = 0
        for g in grads:
            self._flat[off:off + g.numel()].copy_(g.reshape(-1))
            off += g.numel()

    def reduce(self):
        if self.sharded:
            g, S, r = self._flat, self._S, self.rank
            dist.reduce_scatter_tensor(g[r * S:(r + 1) * S], g, op=dist.ReduceOp.SUM,
                                       group=self.group)
            return
        dist.all_reduce(self._flat, op=dist.ReduceOp.SUM, group=self.group)

    def gather(self, net):
        """After the optimizer step: every rank's updated parameter shard to every rank (no-op
        unless sharded)."""
        if not self.sharded:
            return
        p, S, r = net._flat_params, self._S, self.rank
        dist.all_gather_into_tensor(p, p[r * S:(r + 1) * S], group=self.group)

    def unpack(self, net):
        from .agents.flat import grads_are_flat
        if grads_are_flat(net) and self._flat is getattr(net, "_flat_grads", None):
            # reduced in place; the 1/N average is folded into the optimizer's AdamW launch
            # (FlatAdamW.step reads net._allreduce_scale): no unpack kernels
            net._allreduce_scale = 1.0 / self.world
            return
        off = 0
        for p in net.parameters():
            g = p.grad
            torch.div(self._flat[off:off + g.numel()].view_as(g), self.world, out=g)
            off += g.numel()

    def __call__(self, net):
        self.pack(net)
        self.reduce()
        self.unpack(net)

    def finish(self, net):
        """The step after __call__ + the optimizer: the parameter all-gather when sharded."""
        self.gather(net)


def broadcast_params(net, src=0, group=None):
    with torch.no_grad():
        for p in net.parameters():
            dist.broadcast(p.data, src, group=group)


def allreduce_sum(t, group=None):
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t
