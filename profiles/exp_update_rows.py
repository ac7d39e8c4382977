#!/usr/bin/env python3
"""One DDQN learner update (bench.py's learner: batch 2,048, f32, HIP graph) replayed back to
back over 65,536 distinct replay rows: HIP-event average per update with source(s) and
source(s') as two passes (agents/dqn.py STACK_ROWS = False) or as one stacked 4,096-row pass
(STACK_ROWS = True), alternated twice. Also the layers alone at 2,048 / 4,096 rows. One JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from mazerl import VectorMazeEnv  # noqa: E402
from mazerl.agents import dqn as D  # noqa: E402


def timed(fn, iters=100):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(iters):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / iters * 1e3, 1)


def update_us(stack, env):
    D.STACK_ROWS = stack
    L = D.VectorDQNLearner(4096, "cuda", variant="ddqn", batch_size=2048, capacity=65536,
                           updates_per_step=1, target_every=13, seed=5)
    g = torch.Generator(device="cuda").manual_seed(3)
    n = 65536
    s6, s6n = (torch.randn(n, 6, device="cuda", generator=g) for _ in range(2))
    sw, swn = (torch.randint(0, 2**31 - 1, (n, 22), device="cuda", generator=g, dtype=torch.int32)
               for _ in range(2))
    a = torch.randint(0, 4, (n,), device="cuda", generator=g)
    r = torch.randn(n, device="cuda", generator=g)
    L.replay.push(s6, sw, a, r, s6n, swn)
    us = timed(lambda: L.update(env.expand_window))
    assert L._graph is not None
    return us


def main():
    env = VectorMazeEnv(4, 21, enrich=True, device="cuda", seed=1)
    res = {"update_us_two_passes": [], "update_us_stacked": []}
    for stack in ((True,) if "--stacked-only" in sys.argv else (False, True, False, True)):
        res["update_us_stacked" if stack else "update_us_two_passes"].append(update_us(stack, env))
    torch.manual_seed(0)
    net = D.QNet(variant="ddqn").cuda()
    l0 = net.fc[0]
    g = torch.Generator(device="cuda").manual_seed(1)
    with torch.no_grad():
        for b in (2048, 4096):
            bits = torch.randint(0, 2**31 - 1, (b, 22), generator=g, device="cuda", dtype=torch.int32)
            obs6 = torch.rand(b, 6, generator=g, device="cuda")
            x0 = torch.randn(b, 1574, generator=g, device="cuda")
            res[f"stem_fwd_{b}_us"] = timed(lambda: net._bit_stem(obs6, bits))
            res[f"fc1_fwd_{b}_us"] = timed(lambda: F.linear(x0, l0.weight, l0.bias))
    env.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
