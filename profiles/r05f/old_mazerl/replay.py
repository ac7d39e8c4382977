"""Replay memories.

ReplayMemory   — the reference's deque + random.sample memory (lib/replay_memory.py:8-24), kept
                 for the single-env drop-in agents (bit-for-bit the same sampling with the same
                 global `random` state).
DeviceReplay   — the vectorised learner's ring buffer, resident in HBM as structure-of-arrays:
                 obs6 f32[C,6], window bits i32[C,22] (675-bit 3x15x15 window, 88 B instead of
                 the 2,700 B f32 tensor), action i64[C], reward f32[C], and the next-state pair.
                 push() takes a whole vector step at once (slice copies into the ring); sample()
                 draws uniform indices on the device and gathers every row in one HIP launch
                 (mz_replay_gather; or expands f32 windows with mz_expand_window). Sampling is with replacement (the
                 reference's random.sample is without; at C >> batch the difference is a few
                 duplicate rows per batch — documented deviation).
"""
import random
from collections import deque, namedtuple

import torch

Transition = namedtuple("Transition", ("state", "action", "reward", "next_state"))


class ReplayMemory:
    def __init__(self, capacity):
        self.memory = deque([], maxlen=capacity)

    def push(self, *args):
        self.memory.append(Transition(*args))

    def sample(self, batch_size):
        return random.sample(self.memory, batch_size)

    def clear_memory(self):
        self.memory.clear()

    def __len__(self):
        return len(self.memory)


class DeviceReplay:
    def __init__(self, capacity, device, obs_dim=6, window_words=22):
        self.capacity = int(capacity)
        self.device = torch.device(device)
        C, kw = self.capacity, dict(device=self.device)
        self.s6 = torch.zeros(C, obs_dim, dtype=torch.float32, **kw)
        self.sw = torch.zeros(C, window_words, dtype=torch.int32, **kw)
        self.a = torch.zeros(C, dtype=torch.int64, **kw)
        self.r = torch.zeros(C, dtype=torch.float32, **kw)
        self.s6n = torch.zeros(C, obs_dim, dtype=torch.float32, **kw)
        self.swn = torch.zeros(C, window_words, dtype=torch.int32, **kw)
        self.ptr = 0
        self.size = 0
        self.size_dev = torch.zeros((), dtype=torch.float64, **kw)  # for graph-captured sampling
        self.idx_static = None  # sample rows read by a captured graph (overlapped learner)
        self._gen = torch.Generator(device=self.device)
        self._gen.manual_seed(0x5EED)

    def __len__(self):
        return self.size

    def nbytes(self):
        return sum(t.numel() * t.element_size() for t in (self.s6, self.sw, self.a, self.r, self.s6n, self.swn))

    def push(self, s6, sw, a, r, s6n, swn, mask=None):
        """Append n transitions (device tensors with leading dim n); mask selects rows to keep."""
        if mask is not None:
            keep = torch.nonzero(mask, as_tuple=False).flatten()
            s6, sw, a, r, s6n, swn = (t.index_select(0, keep) for t in (s6, sw, a, r, s6n, swn))
        n = a.shape[0]
        if n == 0:
            return
        if n > self.capacity:
            s6, sw, a, r, s6n, swn = (t[-self.capacity:] for t in (s6, sw, a, r, s6n, swn))
            n = self.capacity
        self._write(((self.s6, s6), (self.sw, sw), (self.a, a), (self.r, r), (self.s6n, s6n),
                     (self.swn, swn)), n)
        self.ptr = (self.ptr + n) % self.capacity
        size = min(self.size + n, self.capacity)
        if size != self.size:
            self.size_dev.fill_(float(size))
        self.size = size

    def _ring_push(self, n, s6=None, sw=None, a=None, r=None, s6n=None, swn=None):
        """One mz_replay_push launch: ring rows ptr .. ptr + n - 1 of the arrays given (others
        untouched; the pointer does not move)."""
        from . import _native as N
        if n > self.capacity:
            raise ValueError("a push larger than the ring")
        srcs = (s6, sw, a, r, s6n, swn)
        dts = (torch.float32, torch.int32, torch.int32, torch.float32, torch.float32, torch.int32)
        for t, dt in zip(srcs, dts):
            if t is not None:
                assert t.dtype == dt and t.is_contiguous() and t.shape[0] == n and t.is_cuda
        ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
        N.check(N.load().mz_replay_push(
            n, self.capacity, self.ptr, *[ptr(t) for t in srcs], self.s6.data_ptr(),
            self.sw.data_ptr(), self.a.data_ptr(), self.r.data_ptr(), self.s6n.data_ptr(),
            self.swn.data_ptr(), self.s6.shape[1], self.sw.shape[1],
            torch.cuda.current_stream(self.device).cuda_stream))

    def push_state(self, s6, sw):
        """State half of the next push (before the env step overwrites the observation)."""
        self._ring_push(s6.shape[0], s6=s6, sw=sw)

    def push_rest(self, a, r, s6n, swn):
        """Action, reward and next state of the rows push_state wrote; the push is complete."""
        n = a.shape[0]
        self._ring_push(n, a=a, r=r, s6n=s6n, swn=swn)
        self.ptr = (self.ptr + n) % self.capacity
        size = min(self.size + n, self.capacity)
        if size != self.size:
            self.size_dev.fill_(float(size))
        self.size = size

    def _write(self, pairs, n):
        """Ring rows ptr .. ptr + n - 1 (one or two contiguous slices) <- the n source rows, one
        copy kernel per array and slice (dtype conversion included)."""
        k = min(n, self.capacity - self.ptr)
        for dst, src in pairs:
            dst[self.ptr:self.ptr + k].copy_(src[:k])
            if k < n:
                dst[:n - k].copy_(src[k:n])

    def sample_indices(self, batch):
        return torch.randint(0, self.size, (batch,), device=self.device, generator=self._gen)

    def sample_indices_static(self, batch):
        """Uniform indices from the device-side size (no host value baked in): usable inside a
        captured HIP graph. float64 uniforms from the default generator (graph-safe)."""
        u = torch.rand(batch, dtype=torch.float64, device=self.device)
        return (u * self.size_dev).to(torch.int64).clamp_(max=self.capacity - 1)

    def sample(self, batch, expand, static=False, idx_static=False):
        """Returns ((s6, window), a, r, (s6', window')) with f32 windows from `expand(bits)`, or
        the packed int32 windows themselves when expand is None (QNet's HIP stem reads them).
        idx_static: read the rows from `self.idx_static` (filled by the caller before every graph
        replay — the overlapped learner draws them on the main stream)."""
        if idx_static:
            if self.idx_static is None or self.idx_static.numel() != batch:
                self.idx_static = self.sample_indices(batch)
            i = self.idx_static
        else:
            i = self.sample_indices_static(batch) if static else self.sample_indices(batch)
        if expand is None:
            if self.device.type == "cuda" and self.s6.shape[1] == 6 and self.sw.shape[1] == 22:
                return self._gather_stacked(i, batch)
            return ((self.s6.index_select(0, i), self.sw.index_select(0, i)), self.a.index_select(0, i),
                    self.r.index_select(0, i), (self.s6n.index_select(0, i), self.swn.index_select(0, i)))
        bits = torch.cat((self.sw.index_select(0, i), self.swn.index_select(0, i)), 0)
        w = expand(bits)
        return ((self.s6.index_select(0, i), w[:batch]), self.a.index_select(0, i),
                self.r.index_select(0, i), (self.s6n.index_select(0, i), w[batch:]))

    def _gather_stacked(self, i, batch):
        """All rows of a sample in one HIP launch (mz_replay_gather): state and next state come
        back as the two halves of stacked [2 * batch] buffers (views), the layout
        QNet.forward_rows reads without a copy (agents/dqn.py q_loss)."""
        from . import _native as N
        dev = self.device
        i = i.contiguous()
        s6 = torch.empty(2 * batch, self.s6.shape[1], dtype=torch.float32, device=dev)
        sw = torch.empty(2 * batch, self.sw.shape[1], dtype=torch.int32, device=dev)
        a = torch.empty(batch, dtype=torch.int64, device=dev)
        r = torch.empty(batch, dtype=torch.float32, device=dev)
        N.check(N.load().mz_replay_gather(
            i.data_ptr(), batch, self.capacity, self.s6.data_ptr(), self.sw.data_ptr(),
            self.a.data_ptr(), self.r.data_ptr(), self.s6n.data_ptr(), self.swn.data_ptr(), s6.data_ptr(),
            sw.data_ptr(), a.data_ptr(), r.data_ptr(), torch.cuda.current_stream(dev).cuda_stream))
        return (s6[:batch], sw[:batch]), a, r, (s6[batch:], sw[batch:])
