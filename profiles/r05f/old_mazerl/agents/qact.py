"""The DQN / DDQN acting forward, f32-accurate on the bf16 MFMA (csrc/mz_qact.hip).

The reference acts with `source_net(state).max(1)[1]` in f32 (dqn_agent.py:113-116; the nets
never leave train mode, so DDQN's Dropout(0.2) is active when acting — SURVEY Q13). A bf16
acting head (agents/fused.py FusedQ) picked the f32 argmax on 99.4 % of real trainer states
(profiles/r03c_acting_precision.json). `QAct` runs the whole forward in two HIP launches with
every GEMM operand split into bf16 hi + lo and each product summed as hi*hi + hi*lo + lo*hi in f32
(~2^-16 relative), the conv stem computed from the window bits once per 64 rows into bf16 hi / lo
feature tiles that fc1's K loop reads:

  mz_qact_prepare  fc1 / fc2 weights -> hi / lo bf16 images (after every weight change)
  mz_qact          Q values of the listed rows (row count read on the device) and the argmax
                   scattered to the listed instances — no host synchronisation (three launches:
                   conv stem, fc1, fc2 + fc3 + argmax)

Interface as FusedQ (invalidate / refresh / __call__) plus `rows_greedy` for the greedy-row list.
"""
import torch
import torch.nn as nn

from .. import _native as N

K1, N1, N2 = 1600, 1024, 512


class QAct:
    dtype_note = "bf16x3 split-precision MFMA (hi*hi + hi*lo + lo*hi, f32 accumulate)"

    def __init__(self, qnet, seed=0):
        self.net = qnet
        lin = [m for m in qnet.fc if isinstance(m, nn.Linear)]
        acts = [m for m in qnet.fc if not isinstance(m, nn.Linear)]
        conv = qnet.conv[0]
        if tuple(conv.weight.shape) != (32, 3, 3, 3) or [tuple(l.weight.shape) for l in lin] != \
                [(N1, 1574), (N2, N1), (4, N2)]:
            raise ValueError("QAct implements the reference's Q-network sizes (1574-1024-512-4)")
        assert isinstance(acts[0], nn.LeakyReLU) and acts[0].negative_slope == 0.01
        self.relu = isinstance(acts[1], nn.ReLU)
        if not self.relu:
            assert isinstance(acts[1], nn.LeakyReLU) and acts[1].negative_slope == 0.01
        self.lin, self.conv = lin, conv
        self.dropout = next((m for m in qnet.conv if isinstance(m, nn.Dropout)), None)
        dev = conv.weight.device
        if dev.type != "cuda":
            raise RuntimeError("QAct runs on the GPU (HIP)")
        i16 = dict(dtype=torch.int16, device=dev)
        self.w1h, self.w1l = torch.zeros(N1, K1, **i16), torch.zeros(N1, K1, **i16)
        self.w2h, self.w2l = torch.zeros(N2, N1, **i16), torch.zeros(N2, N1, **i16)
        self.seed = int(seed)
        self.counter = 0
        self.h1 = None
        self._ver = None
        self.lib = N.load()

    def invalidate(self):
        self._ver = None

    def _stream(self):
        return torch.cuda.current_stream(self.w1h.device).cuda_stream

    def refresh(self, force=True):
        """Rebuild the hi / lo weight images now, on the current stream."""
        ver = tuple(p._version for l in self.lin for p in (l.weight, l.bias))
        if not force and ver == self._ver:
            return
        w1, w2 = self.lin[0].weight.detach(), self.lin[1].weight.detach()
        assert w1.is_contiguous() and w2.is_contiguous() and w1.dtype == torch.float32
        N.check(self.lib.mz_qact_prepare(w1.data_ptr(), w2.data_ptr(), self.w1h.data_ptr(),
                                         self.w1l.data_ptr(), self.w2h.data_ptr(),
                                         self.w2l.data_ptr(), self._stream()))
        self._ver = ver

    def _run(self, obs6, bits, rows, count, n, greedy, q_out):
        self.refresh(force=False)
        assert bits.dtype == torch.int32 and bits.shape[1] == 22 and bits.is_contiguous()
        obs6 = obs6.contiguous()
        assert obs6.dtype == torch.float32 and obs6.shape == (bits.shape[0], 6)
        ws = int(self.lib.mz_qact_workspace_floats(max(n, 1)))  # h1 rows + conv feature tiles
        if self.h1 is None or self.h1.numel() < ws:
            self.h1 = torch.empty(ws, dtype=torch.float32, device=bits.device)
        p = float(self.dropout.p) if (self.dropout is not None and self.dropout.training) else 0.0
        cw, cb = self.conv.weight.detach().contiguous(), self.conv.bias.detach().contiguous()
        l0, l1, l2 = self.lin
        N.check(self.lib.mz_qact(
            bits.data_ptr(), obs6.data_ptr(), rows.data_ptr() if rows is not None else None,
            count.data_ptr() if count is not None else None, n, cw.data_ptr(), cb.data_ptr(),
            self.w1h.data_ptr(), self.w1l.data_ptr(), l0.bias.detach().data_ptr(),
            self.w2h.data_ptr(), self.w2l.data_ptr(), l1.bias.detach().data_ptr(),
            l2.weight.detach().data_ptr(), l2.bias.detach().data_ptr(), int(self.relu), p,
            self.seed & 0xFFFFFFFFFFFFFFFF, self.counter & 0xFFFFFFFFFFFFFFFF,
            self.h1.data_ptr(), greedy.data_ptr() if greedy is not None else None,
            q_out.data_ptr() if q_out is not None else None, self._stream()))
        self.counter += 1

    @torch.no_grad()
    def __call__(self, obs6, bits):
        """Q values [n, 4] (f32) of every instance."""
        n = bits.shape[0]
        q = torch.empty(n, 4, dtype=torch.float32, device=bits.device)
        self._run(obs6, bits, None, None, n, None, q)
        return q

    @torch.no_grad()
    def greedy(self, obs6, bits, out=None):
        """argmax_a Q(s, a) (int64 [n]) of every instance."""
        n = bits.shape[0]
        out = torch.empty(n, dtype=torch.int64, device=bits.device) if out is None else out
        self._run(obs6, bits, None, None, n, out, None)
        return out

    @torch.no_grad()
    def rows_greedy(self, obs6, bits, rows, count, greedy, q_out=None):
        """greedy[rows[i]] = argmax_a Q for i < min(len(rows), *count) (count: int32 [1] on the
        device) — the greedy-row list's acting forward, sized on the device."""
        assert rows.dtype == torch.int32 and rows.is_contiguous() and count.dtype == torch.int32
        self._run(obs6, bits, rows, count, rows.numel(), greedy, q_out)
