#!/usr/bin/env python3
"""Round 4: the split acting forward (k_qconv + k_qfc1) must give the fused k_qact1's Q values bit
for bit (same features, same MFMA order). Prints a checksum of QAct's Q values on fixed inputs —
65,536 rows and a 28,180-row list, DDQN dropout on and off — for the library MZ_LIB_OVERRIDE
selects; the A/B script compares the lines."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))

import torch  # noqa: E402


def main():
    from mazerl.agents.nets import QNet
    from mazerl.agents.qact import QAct
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    h = hashlib.sha256()
    for variant in ("ddqn", "dqn"):
        net = QNet(variant=variant).to(dev)
        qa = QAct(net, seed=1)
        g = torch.Generator(device=dev).manual_seed(0)
        n = 65536
        bits = torch.randint(0, 2**31 - 1, (n, 22), generator=g, device=dev, dtype=torch.int32)
        obs6 = torch.rand(n, 6, generator=g, device=dev)
        rows = torch.randperm(n, generator=g, device=dev)[:28180].to(torch.int32).contiguous()
        count = torch.tensor([28180], dtype=torch.int32, device=dev)
        for train in (True, False):
            net.train(train)
            q = qa(obs6, bits)
            h.update(q.cpu().numpy().tobytes())
            qo = torch.zeros(rows.numel(), 4, device=dev)
            gr = torch.zeros(n, dtype=torch.int64, device=dev)
            qa.rows_greedy(obs6, bits, rows, count, gr, q_out=qo)
            h.update(qo.cpu().numpy().tobytes())
            h.update(gr.cpu().numpy().tobytes())
    print(json.dumps({"lib": os.environ.get("MZ_LIB_OVERRIDE", "default"),
                      "q_checksum": h.hexdigest()[:16]}), flush=True)


if __name__ == "__main__":
    main()
