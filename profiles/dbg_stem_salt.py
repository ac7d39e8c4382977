#!/usr/bin/env python3
"""Round 4: test_stacked_ddqn_pass_train_mode_matches_torch_with_same_masks failed once when its
file ran alone (another QNet construction count -> another dropout salt). For salts 1..40: the
forward of QNet.forward_rows (train mode, dropout 0.2) against the float64 torch pipeline with the
regenerated masks — worst |q - q_ref| / (rtol |q_ref| + atol * scale) at the test's tolerances,
and the same for the stem features alone."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import copy  # noqa: E402

import torch  # noqa: E402

from test_stem import _bits, _masks, _torch_stem, _window  # noqa: E402


def main():
    from mazerl.agents.nets import QNet
    b = 384
    for salt in range(1, 41):
        torch.manual_seed(6)
        net = QNet(variant="ddqn").cuda().train()
        net._salt = salt
        ref = copy.deepcopy(net).double()
        bits = _bits(2 * b, 21)
        win = _window(bits).cuda()
        bits = bits.cuda()
        s6 = torch.randn(2 * b, 6).cuda()
        key = 0x5151_0000_2222
        net._stem_rng = torch.tensor([key], dtype=torch.int64, device="cuda")
        q = net.forward_rows((s6, bits), b)
        keep = torch.from_numpy(_masks(2 * b, key, net._salt, 0.2)).cuda()
        feat_ref = _torch_stem(ref, s6.double(), win.double(), keep.double(), 0.2)
        q_ref = ref.fc(feat_ref).detach()
        from mazerl.agents.stem import stem_features
        net._stem_rng = torch.tensor([key], dtype=torch.int64, device="cuda")
        feat = stem_features(bits, s6, net.conv[0], 0.2, net._stem_rng, net._salt).detach()
        out = {"salt": salt}
        for name, a, c in (("q", q.detach().double(), q_ref), ("feat", feat.double(), feat_ref.detach())):
            scale = float(c.abs().max())
            err = (a - c).abs() / (1e-5 * c.abs() + 1e-6 * scale)
            out[name] = round(float(err.max()), 3)
            out[name + "_maxabs_rel_scale"] = float((a - c).abs().max()) / scale
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
