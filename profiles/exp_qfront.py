#!/usr/bin/env python3
"""k_qfront (acting conv stem) and the whole acting forward at 65,536 instances: HIP-event
average per call; QF_VARIANT=ddqn (dropout in the stem) or dqn (none). (The feature stores'
cache policy was compared here too: default / sc1 / nt within 2 %, default kept.)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))
import torch  # noqa: E402

from mazerl.agents.fused import FusedQ  # noqa: E402
from mazerl.agents.nets import QNet  # noqa: E402


def timed(fn, iters=50):
    for _ in range(5):
        fn()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(iters):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


dev = torch.device("cuda:0")
torch.manual_seed(0)
n = 65536
net = QNet(variant=os.environ.get("QF_VARIANT", "ddqn")).to(dev)
fq = FusedQ(net, seed=1)
g = torch.Generator(device=dev).manual_seed(0)
bits = torch.randint(0, 2**31 - 1, (n, 22), generator=g, device=dev, dtype=torch.int32)
obs6 = torch.rand(n, 6, generator=g, device=dev)
with torch.no_grad():
    stem = timed(lambda: fq.stem(obs6, bits))
    full = timed(lambda: fq(obs6, bits))
print(json.dumps({"variant": os.environ.get("QF_VARIANT", "ddqn"), "stem_us": round(stem, 1),
                  "forward_us": round(full, 1)}), flush=True)
