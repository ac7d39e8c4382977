#!/usr/bin/env python3
"""k_adamw alone: the flat AdamW step over the Q-net's 2,140,548 parameters (HIP events, 500
launches), for the library named by MZ_LIB_OVERRIDE (profiles/exp_adamw_ticket.sh builds
variants with different workgroup caps: every workgroup takes one same-address ticket to publish
the step count, so the cap sets how many atomics serialise at the end of the launch)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))

import torch  # noqa: E402

from mazerl.agents.flat import FlatAdamW  # noqa: E402


def main(iters=500):
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Conv2d(3, 32, 3, padding=1), torch.nn.Linear(1574, 1024),
                              torch.nn.Linear(1024, 512), torch.nn.Linear(512, 4)).cuda()
    opt = FlatAdamW(net, lr=1e-4)
    for p in net.parameters():
        p.grad = torch.randn_like(p) * 1e-3
    for _ in range(20):
        opt.step()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        opt.step()
    e.record()
    torch.cuda.synchronize()
    import hashlib
    h = hashlib.sha256()
    for t in (opt.flat, opt.exp_avg, opt.exp_avg_sq):
        h.update(t.cpu().numpy().tobytes())
    print(json.dumps({"checksum": h.hexdigest()[:16],"lib": os.path.basename(os.environ.get("MZ_LIB_OVERRIDE", "default")),
                      "params": sum(p.numel() for p in net.parameters()),
                      "us_per_step": s.elapsed_time(e) * 1e3 / iters,
                      "step_count": float(opt.step_t.item())}), flush=True)


if __name__ == "__main__":
    main()
