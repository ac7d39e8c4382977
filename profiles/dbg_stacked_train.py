"""Debug repro: the stacked DDQN pass in train mode (forward_rows with n_grad = b over 2b rows)
vs the same bit stem without n_grad and vs the torch stem with regenerated dropout masks."""
import copy
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_stem import _bits, _masks, _torch_stem, _window  # noqa: E402

from mazerl.agents.nets import QNet  # noqa: E402


def main():
    torch.manual_seed(6)
    net = QNet(variant="ddqn").cuda().train()
    full = copy.deepcopy(net)
    ref = copy.deepcopy(net)
    b = 384
    bits = _bits(2 * b, 21)
    win = _window(bits).cuda()
    bits = bits.cuda()
    s6 = torch.randn(2 * b, 6).cuda()
    key = 0x5151_0000_2222
    R = torch.randn(b, 4).cuda()
    net._stem_rng = torch.tensor([key], dtype=torch.int64, device="cuda")
    full._stem_rng = torch.tensor([key], dtype=torch.int64, device="cuda")
    q = net.forward_rows((s6, bits), b)
    qf = full((s6, bits))
    keep = torch.from_numpy(_masks(2 * b, key, net._salt, 0.2)).cuda()
    q_ref = ref.fc(_torch_stem(ref, s6, win, keep, 0.2))
    print("fwd max|q-qf|", float((q - qf).abs().max()), "max|q-qref|", float((q - q_ref).abs().max()))
    g = torch.autograd.grad((q[:b] * R).sum(), list(net.parameters()))
    gf = torch.autograd.grad((qf[:b] * R).sum(), list(full.parameters()))
    gr = torch.autograd.grad((q_ref[:b] * R).sum(), list(ref.parameters()))
    for (name, _), a, f, c in zip(net.named_parameters(), g, gf, gr):
        sc = float(c.abs().max())
        print(f"{name:14s} scale {sc:.3e} rows-vs-full {float((a - f).abs().max()):.3e} "
              f"rows-vs-torch {float((a - c).abs().max()):.3e} full-vs-torch {float((f - c).abs().max()):.3e}")
        d = (a - c).abs()
        i = int(d.flatten().argmax())
        print("    worst", i, float(a.flatten()[i]), float(c.flatten()[i]))


if __name__ == "__main__":
    main()
