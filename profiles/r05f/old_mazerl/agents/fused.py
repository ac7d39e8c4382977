"""Acting forward of the Q / actor-critic networks straight from packed windows.

The reference acts with `source_net(state)` (dqn_agent.py:113-116; ddqn_agent.py, nets never in
eval mode — SURVEY Q13; ppo_agent.py ActorCriticNet.act). Vectorised over 65,536 instances the
conv stem dominated the training step through PyTorch (f32 window + transposes + bf16 conv
output + separate LeakyReLU / Dropout / MaxPool passes, ~4 ms per vector step). Here:

  mz_q_front (HIP, csrc/mz_qnet.hip)   88-byte window bits + obs6 -> bf16 [n, 1600] fc1 input
                                       (conv as bf16 MFMA, LeakyReLU, Dropout, MaxPool fused;
                                       features position-major, fc1 columns permuted to match)
  Linear -> act -> Linear -> act -> Linear   bf16 GEMMs (hipBLASLt), f32 accumulation

Same precision class as the autocast(bf16) acting path it replaces (bf16 weights and
activations); the update path (q_loss / PPO losses) stays f32 through torch. Dropout masks come
from the kernel's own counter-based hash (P(drop) = 13107/65536 for p = 0.2), not torch's RNG.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _native as N

LD = 1600          # fc1 input row: 1,568 conv features | 6 obs | 26 zeros (16-B aligned rows)
CONV_OUT = 1568


def feature_perm(device=None):
    """The kernel writes conv features position-major (q * 32 + c); torch's flatten is
    channel-major (c * 49 + q). perm[f'] = torch index of kernel feature f'."""
    return torch.arange(CONV_OUT, device=device).view(32, 49).t().reshape(-1)


def _leaky_(h, slope):
    """In-place LeakyReLU; bf16 on the GPU through mz_leaky_relu_bf16 (torch's elementwise kernel
    moves the 65,536 x 1,024 hidden layer at ~3.8 TB/s), same rounding as F.leaky_relu_."""
    if h.is_cuda and h.dtype == torch.bfloat16 and h.is_contiguous() and h.numel() % 8 == 0 \
            and h.data_ptr() % 16 == 0:
        N.check(N.load().mz_leaky_relu_bf16(h.data_ptr(), h.numel(), float(slope),
                                            torch.cuda.current_stream(h.device).cuda_stream))
        return h
    return F.leaky_relu_(h, slope)


def _act_fn(m):
    if isinstance(m, nn.LeakyReLU):
        return lambda h: _leaky_(h, m.negative_slope)
    if isinstance(m, nn.ReLU):
        return F.relu_
    raise TypeError(f"unsupported activation {type(m).__name__}")


class _Head:
    """bf16 copy of a Linear -> act -> Linear -> act -> Linear stack; the first weight padded to LD
    columns. Refreshed when the f32 parameters changed: eager optimizer steps bump `_version`;
    updates replayed from a captured HIP graph do not, so their owner calls invalidate(). On the
    GPU the copy is one mz_head_bf16 launch into persistent buffers (refresh(force=True) on a side
    stream right after a weight snapshot keeps it off the acting stream)."""

    def __init__(self, seq):
        self.seq = seq
        self.lin = [m for m in seq if isinstance(m, nn.Linear)]
        acts = [m for m in seq if not isinstance(m, nn.Linear)]
        self.acts = [_act_fn(m) for m in acts]
        assert len(self.lin) == 3 and len(self.acts) == 2
        self.relu2 = isinstance(acts[1], nn.ReLU)
        l0 = self.lin[0]
        if l0.in_features > LD:
            raise ValueError(f"first Linear has {l0.in_features} inputs > {LD}")
        dev = l0.weight.device
        bf = dict(dtype=torch.bfloat16, device=dev)
        self.w0 = torch.zeros(l0.out_features, LD, **bf)
        self.perm = feature_perm(dev)
        self._w = [(self.w0, torch.empty(l0.out_features, **bf))] + \
                  [(torch.empty(l.out_features, l.in_features, **bf), torch.empty(l.out_features, **bf))
                   for l in self.lin[1:]]
        self._ver = None
        self._lib = N.load() if dev.type == "cuda" else None

    def invalidate(self):
        self._ver = None

    def _refresh(self, force=False):
        ver = tuple(p._version for l in self.lin for p in (l.weight, l.bias))
        if ver == self._ver and not force:
            return
        l0, l1, l2 = self.lin
        if self._lib is not None:
            src = [t.detach() for l in self.lin for t in (l.weight, l.bias)]
            assert all(t.is_contiguous() and t.dtype == torch.float32 for t in src)
            (w0, b0), (w1, b1), (w2, b2) = self._w
            N.check(self._lib.mz_head_bf16(
                *[t.data_ptr() for t in src], l0.out_features, l0.in_features, l1.out_features,
                l1.in_features, l2.out_features, l2.in_features, LD, CONV_OUT, 32,
                w0.data_ptr(), b0.data_ptr(), w1.data_ptr(), b1.data_ptr(), w2.data_ptr(),
                b2.data_ptr(), torch.cuda.current_stream(w0.device).cuda_stream))
        else:
            w = l0.weight.detach()
            self.w0[:, :CONV_OUT].copy_(w.index_select(1, self.perm))  # kernel feature order
            self.w0[:, CONV_OUT:l0.in_features].copy_(w[:, CONV_OUT:])
            for (dw, db), l in zip(self._w, self.lin):
                if dw is not self.w0:
                    dw.copy_(l.weight.detach())
                db.copy_(l.bias.detach())
        self._ver = ver

    def refresh(self):
        """Rebuild the bf16 copy now, on the current stream (after a weight snapshot)."""
        self._refresh(force=True)

    def __call__(self, feat):
        self._refresh()
        (w0, b0), (w1, b1), (w2, b2) = self._w
        h = self.acts[0](F.linear(feat, w0, b0))
        if self.relu2:  # bias + ReLU as the GEMM's epilogue (hipBLASLt), bit-identical
            h = torch._addmm_activation(b1, h, w1.t())
        else:
            h = self.acts[1](F.linear(h, w1, b1))
        return F.linear(h, w2, b2)


class FusedStem:
    """Conv2d(3->32, 3x3, p1) -> LeakyReLU -> [Dropout] -> MaxPool2d(2) -> flatten || obs6."""

    def __init__(self, conv_seq, seed=0):
        mods = list(conv_seq)
        self.conv = mods[0]
        assert isinstance(self.conv, nn.Conv2d) and tuple(self.conv.weight.shape) == (32, 3, 3, 3), \
            "the fused stem implements the reference's Conv2d(3, 32, 3, padding=1)"
        assert isinstance(mods[1], nn.LeakyReLU) and mods[1].negative_slope == 0.01
        self.dropout = next((m for m in mods if isinstance(m, nn.Dropout)), None)
        assert isinstance(mods[-1], nn.MaxPool2d)
        self.seed = seed
        self.counter = 0
        self.lib = N.load()

    def __call__(self, obs6, bits, rows=None, n=None, count=None, out=None):
        """Feature rows of every instance, or with `rows` (int32 instance ids) of rows[:n] only —
        with `count` (int32 [1] on the device) rows[:min(n, count)], the rest of out[:n] left
        unwritten. `out`: a [>= n, LD] bf16 buffer to write into."""
        dev = bits.device
        if dev.type != "cuda":
            raise RuntimeError("the fused acting stem runs on the GPU only")
        assert bits.dtype == torch.int32 and bits.shape[1] == 22 and bits.is_contiguous()
        obs6 = obs6.contiguous()
        assert obs6.dtype == torch.float32 and obs6.shape == (bits.shape[0], 6)
        if rows is None:
            n = bits.shape[0]
        else:
            assert rows.dtype == torch.int32 and rows.is_contiguous() and rows.device == dev
            assert 0 <= n <= rows.numel()
        w = self.conv.weight.detach().contiguous()
        b = self.conv.bias.detach().contiguous()
        p = float(self.dropout.p) if (self.dropout is not None and self.dropout.training) else 0.0
        feat = torch.empty(n, LD, dtype=torch.bfloat16, device=dev) if out is None else out[:n]
        stream = torch.cuda.current_stream(dev).cuda_stream
        if rows is None:
            N.check(self.lib.mz_q_front(bits.data_ptr(), obs6.data_ptr(), n, w.data_ptr(),
                                        b.data_ptr(), p, self.seed, self.counter, feat.data_ptr(),
                                        LD, stream))
        else:
            N.check(self.lib.mz_q_front_rows(bits.data_ptr(), obs6.data_ptr(), rows.data_ptr(),
                                             count.data_ptr() if count is not None else None, n,
                                             w.data_ptr(), b.data_ptr(), p, self.seed, self.counter,
                                             feat.data_ptr(), LD, stream))
        self.counter += 1
        return feat


class FusedQ:
    """QNet acting forward (DQN / DDQN) on window bits -> Q values [n, 4] (bf16)."""

    def __init__(self, qnet, seed=0):
        self.stem = FusedStem(qnet.conv, seed)
        self.head = _Head(qnet.fc)

    def invalidate(self):
        self.head.invalidate()

    def refresh(self):
        self.head.refresh()

    @torch.no_grad()
    def __call__(self, obs6, bits):
        return self.head(self.stem(obs6, bits))

    @torch.no_grad()
    def rows(self, obs6, bits, rows, n):
        """Q values [n, 4] of instances rows[:n]."""
        return self.head(self.stem(obs6, bits, rows, n))

    @torch.no_grad()
    def rows_stem(self, obs6, bits, rows, count, out):
        """Stem features of rows[:count] (count on the device) into out [B, LD] (bf16)."""
        self.stem(obs6, bits, rows, out.shape[0], count=count, out=out)

    @torch.no_grad()
    def rows_head(self, feat):
        return self.head(feat)


class GreedyRows:
    """The greedy-row list of the next fused act (mz_greedy_rows: the instances that will act
    greedily with this eps / seed / counter, dqn_agent.py:104-116) and the acting forward over
    those rows only. With QAct (agents/qact.py) the forward reads the list's length on the
    device; with FusedQ the count comes back to the host (one stream sync) to size the GEMMs.
    `greedy` [n] int64 holds the argmax of the listed rows; the other entries are stale — the
    fused act never reads them (it explores there)."""

    BUCKET = 256  # GEMM rows rounded up (fewer distinct hipBLASLt shapes); extra rows are ignored

    def __init__(self, n, device):
        self.n = n
        self.rows = torch.zeros(n, dtype=torch.int32, device=device)  # stale ids stay valid
        self.scratch = torch.zeros((n + 1023) // 1024, dtype=torch.int32, device=device)
        self.count = torch.zeros(1, dtype=torch.int32, device=device)
        self.count_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        self.greedy = torch.zeros(n, dtype=torch.int64, device=device)
        self.event = torch.cuda.Event()
        self.lib = N.load()
        self.last_count = None
        self.feat = None  # [n, LD] bf16 stem features of the listed rows (persistent)

    def issue(self, eps, seed, counter):
        """Launch the list kernels and the count's copy to the host on the current stream; the
        host reads it later (select). Issued early — right after the bookkeeping that fixes the
        next step's epsilon — the copy has landed by the time the next acting forward needs it."""
        stream = torch.cuda.current_stream(self.rows.device).cuda_stream
        eps_t = eps if torch.is_tensor(eps) else None
        if eps_t is not None:
            assert eps_t.dtype == torch.float32 and eps_t.is_contiguous() and eps_t.numel() == self.n
        N.check(self.lib.mz_greedy_rows(eps_t.data_ptr() if eps_t is not None else None,
                                        0.0 if eps_t is not None else float(eps),
                                        seed & 0xFFFFFFFFFFFFFFFF, counter & 0xFFFFFFFFFFFFFFFF,
                                        self.n, self.scratch.data_ptr(), self.rows.data_ptr(),
                                        self.count.data_ptr(), None, stream))
        self.count_host.copy_(self.count, non_blocking=True)
        self.event.record()
        self._issued = (eps_t.data_ptr() if eps_t is not None else float(eps), seed, counter)

    def select(self, eps, seed, counter):
        """The list for (eps, seed, counter) — issued now unless issue() already did — and its
        length (waits for the count's copy)."""
        key = (eps.data_ptr() if torch.is_tensor(eps) else float(eps), seed, counter)
        if getattr(self, "_issued", None) != key:
            self.issue(eps, seed, counter)
        self._issued = None
        self.event.synchronize()
        self.last_count = int(self.count_host[0])
        return self.last_count

    @torch.no_grad()
    def __call__(self, fused, obs6, bits, eps, seed, counter):
        key = (eps.data_ptr() if torch.is_tensor(eps) else float(eps), seed, counter)
        if getattr(self, "_issued", None) != key:
            self.issue(eps, seed, counter)
        if hasattr(fused, "rows_greedy"):
            # QAct: the forward reads the list's length on the device — no host wait
            self._issued = None
            fused.rows_greedy(obs6, bits, self.rows, self.count, self.greedy)
            return self.greedy
        if self.feat is None:
            self.feat = torch.zeros(self.n, LD, dtype=torch.bfloat16, device=self.rows.device)
        # the stem reads the list's length on the device: it runs while the host waits for it
        fused.rows_stem(obs6, bits, self.rows, self.count, self.feat)
        k = self.select(eps, seed, counter)
        if k:
            m = min(self.n, -(-k // self.BUCKET) * self.BUCKET)
            q = fused.rows_head(self.feat[:m])
            assert q.dtype == torch.bfloat16 and q.is_contiguous() and q.shape == (m, 4)
            N.check(self.lib.mz_greedy_scatter(q.data_ptr(), 4, self.rows.data_ptr(),
                                               self.count.data_ptr(), m, self.greedy.data_ptr(),
                                               torch.cuda.current_stream(q.device).cuda_stream))
        return self.greedy

    def tick(self, term, trunc, steps_done, eps_start, eps_final, eps_decay, wins, episodes, seed,
             counter):
        """mz_trainer_tick: the step's bookkeeping + the next act's epsilon and greedy-row list
        (issued, count on its way to the host). Returns the epsilon tensor."""
        if not hasattr(self, "eps"):
            self.eps = torch.empty(self.n, dtype=torch.float32, device=self.rows.device)
        for t in (term, trunc):
            assert t.dtype == torch.uint8 and t.is_contiguous() and t.numel() == self.n
        assert steps_done.dtype == torch.float32 and steps_done.is_contiguous()
        for t in (wins, episodes):
            assert t is None or (t.dtype == torch.int64 and t.numel() == 1)
        N.check(self.lib.mz_trainer_tick(
            term.data_ptr(), trunc.data_ptr(), steps_done.data_ptr(), float(eps_start),
            float(eps_final), float(eps_decay), self.eps.data_ptr(),
            wins.data_ptr() if wins is not None else None,
            episodes.data_ptr() if episodes is not None else None,
            seed & 0xFFFFFFFFFFFFFFFF, counter & 0xFFFFFFFFFFFFFFFF, self.n, self.scratch.data_ptr(),
            self.rows.data_ptr(), self.count.data_ptr(),
            torch.cuda.current_stream(self.rows.device).cuda_stream))
        self.count_host.copy_(self.count, non_blocking=True)
        self.event.record()
        self._issued = (self.eps.data_ptr(), seed, counter)
        return self.eps


class FusedActorCritic:
    """ActorCriticNet forward on window bits -> (logits [n, 4], value [n, 1]) (bf16)."""

    def __init__(self, net, seed=0):
        self.stem = FusedStem(net.conv, seed)
        self.actor = _Head(net.actor_head)
        self.critic = _Head(net.critic_head)

    def invalidate(self):
        self.actor.invalidate()
        self.critic.invalidate()

    @torch.no_grad()
    def __call__(self, obs6, bits):
        feat = self.stem(obs6, bits)
        return self.actor(feat), self.critic(feat)
