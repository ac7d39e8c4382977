"""Q-networks with the reference's exact architecture and parameter layout.

`QNet(variant="dqn")`  == agents/dqn_agent.py:19-57 (DQN): Conv2d(3->h,3x3,p1) -> LeakyReLU ->
                          MaxPool2d(2) -> flatten || obs -> Linear -> LeakyReLU -> Linear ->
                          LeakyReLU -> Linear; conv weight Xavier-uniform (:43-45).
`QNet(variant="ddqn")` == agents/ddqn_agent.py:18-52: adds Dropout(0.2) after the conv
                          activation and uses ReLU in the second hidden layer; no Xavier init.
Module names (conv.0, fc.0, fc.2, fc.4) match the reference so state_dicts interchange.
Given packed windows (int32 [n, 22], the replay's storage) on the GPU, forward() runs the stem as
one HIP kernel (agents/stem.py, csrc/mz_stem.hip) with its own backward.
With window 15x15, h=32: 1568 conv features + 6 obs -> 1574 -> 1024 -> 512 -> 4
(2,140,548 parameters, 4,665,024 FLOP per sample forward).

On MI355X the three Linear layers are plain GEMMs and go through hipBLASLt (f32 in/out runs on
the f32 MFMA at the f32 rate, bit-exact f32; `autocast(bf16)` puts them on the bf16 MFMA for
acting). The conv front-end is MIOpen.
"""
import torch
import torch.nn as nn

from .linear import GraphSafeLinear

WINDOW = (15, 15)


class QNet(nn.Module):
    _count = 0  # construction order: the dropout-mask salt of the packed-window stem

    def __init__(self, in_channels=3, n_observations=6, n_actions=4, h_channels=32,
                 hidden_dim=1024, variant="dqn"):
        super().__init__()
        QNet._count += 1
        self._salt = QNet._count
        self._stem_rng = None
        self._stem_advance = "add"  # how the stem's dropout counter moves on (agents/stem.py)
        self.in_channels = in_channels
        self.variant = variant
        conv = [nn.Conv2d(in_channels, h_channels, kernel_size=3, stride=1, padding=1), nn.LeakyReLU()]
        if variant == "ddqn":
            conv.append(nn.Dropout(p=0.2))
        conv.append(nn.MaxPool2d(2, 2))
        self.conv = nn.Sequential(*conv)
        conv_out = h_channels * (WINDOW[0] // 2) * (WINDOW[1] // 2)
        act2 = nn.ReLU() if variant == "ddqn" else nn.LeakyReLU()
        self.fc = nn.Sequential(
            GraphSafeLinear(conv_out + n_observations, hidden_dim),
            nn.LeakyReLU(),
            GraphSafeLinear(hidden_dim, hidden_dim // 2),
            act2,
            GraphSafeLinear(hidden_dim // 2, n_actions),
        )
        if variant == "dqn":
            for layer in self.conv:
                if isinstance(layer, nn.Conv2d):
                    nn.init.xavier_uniform_(layer.weight)

    def forward(self, x):
        s, w = x
        if w.dtype == torch.int32 and w.dim() == 2:  # packed windows: the HIP f32 stem
            return self.fc(self._bit_stem(s, w))
        fw = self.conv(w)
        fw = fw.view(fw.shape[0], -1)
        return self.fc(torch.cat((fw, s), dim=1))


    def forward_rows(self, x, n_grad):
        """forward() over stacked rows of which only the first n_grad carry a gradient (DDQN's
        source(s) and source(s') as one pass, agents/dqn.py q_loss): the stem's and the Linear
        layers' backward read those rows only. Packed windows on the GPU; else forward().

        Contract: the input gradients of this pass hold rows < n_grad only (rows >= n_grad are
        left unwritten, agents/linear.py), so every module between the stem and the output must
        be a row-limited GraphSafeLinear or a row-wise activation; nothing may read the whole
        gradient tensor (hooks, anomaly mode, gradcheck)."""
        s, w = x
        if not (w.dtype == torch.int32 and w.dim() == 2 and w.is_cuda):
            return self.forward(x)
        for m in self.fc:
            if not isinstance(m, (GraphSafeLinear, nn.LeakyReLU, nn.ReLU)):
                raise TypeError(f"forward_rows: {type(m).__name__} would read gradient rows >= n_grad")
        if torch.is_anomaly_enabled():
            raise RuntimeError("forward_rows leaves gradient rows >= n_grad unwritten; "
                               "anomaly mode would read them")
        h = self._bit_stem(s, w, n_grad)
        for m in self.fc:
            h = m(h, n_grad) if isinstance(m, GraphSafeLinear) else m(h)
        return h

    def trunk(self, x, n_grad=None):
        """Packed windows on the GPU: the second hidden layer's pre-activation z2 = fc.2(act(fc.0(
        stem))) — everything but the last activation and fc.4, which the learner's fused head
        + loss launch applies (agents/dqn.py _HeadLossFn). `n_grad`: as forward_rows."""
        s, w = x
        if not (w.dtype == torch.int32 and w.dim() == 2 and w.is_cuda):
            raise ValueError("trunk() takes packed windows on the GPU")
        if n_grad is not None and torch.is_anomaly_enabled():
            raise RuntimeError("trunk(n_grad) leaves gradient rows >= n_grad unwritten; "
                               "anomaly mode would read them")
        h = self._bit_stem(s, w, n_grad)
        for m in list(self.fc)[:3]:
            h = m(h, n_grad) if isinstance(m, GraphSafeLinear) else m(h)
        return h

    def _bit_stem(self, s, bits, n_grad=None):
        from .stem import stem_features
        p = 0.0
        if self.training:
            for m in self.conv:
                if isinstance(m, nn.Dropout):
                    p = float(m.p)
        if p > 0 and (self._stem_rng is None or self._stem_rng.device != bits.device):
            self._stem_rng = torch.zeros(1, dtype=torch.int64, device=bits.device)
        return stem_features(bits, s, self.conv[0], p, self._stem_rng, self._salt, n_grad,
                             self._stem_advance)


def count_params(net):
    return sum(p.numel() for p in net.parameters())


def forward_flops(h_channels=32, hidden_dim=1024, n_obs=6, n_actions=4, in_channels=3):
    """FLOP per sample of one forward (multiply-add = 2 FLOP), conv counted at full 15x15."""
    conv = 2 * in_channels * 9 * h_channels * WINDOW[0] * WINDOW[1]
    d0 = h_channels * (WINDOW[0] // 2) * (WINDOW[1] // 2) + n_obs
    return conv + 2 * (d0 * hidden_dim + hidden_dim * (hidden_dim // 2) + (hidden_dim // 2) * n_actions)
