"""Multi-GPU plumbing: one process per GPU, env shards with no data-path exchange, and the
learner's data-parallel gradient all-reduce over RCCL (torch.distributed backend "nccl" on ROCm;
"gloo" on CPU for tests).

Per update the source net's gradients (2,140,548 fp32 = 8.56 MB at full size) are flattened into
ONE bucket and all-reduced once (xGMI ring: 2(N-1)/N x 8.56 MB per GPU, ~0.1 ms at ~153 GB/s per
link), then averaged; grad.clamp_(-1, 1) runs after the average so N ranks reproduce the
single-GPU update on the union batch (dqn_agent.py:152-153). Instance ids are global
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
    them (agents/dqn.py): pack / unpack are plain device copies, reduce is the one all-reduce."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self._flat = None

    def pack(self, net):
        grads = [p.grad for p in net.parameters()]
        n = sum(g.numel() for g in grads)
        if self._flat is None or self._flat.numel() != n or self._flat.device != grads[0].device:
            self._flat = torch.empty(n, dtype=grads[0].dtype, device=grads[0].device)
        off = 0
        for g in grads:
            self._flat[off:off + g.numel()].copy_(g.reshape(-1))
            off += g.numel()

    def reduce(self):
        dist.all_reduce(self._flat, op=dist.ReduceOp.SUM, group=self.group)

    def unpack(self, net):
        off = 0
        for p in net.parameters():
            g = p.grad
            torch.div(self._flat[off:off + g.numel()].view_as(g), self.world, out=g)
            off += g.numel()

    def __call__(self, net):
        self.pack(net)
        self.reduce()
        self.unpack(net)


def broadcast_params(net, src=0, group=None):
    with torch.no_grad():
        for p in net.parameters():
            dist.broadcast(p.data, src, group=group)


def allreduce_sum(t, group=None):
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t
