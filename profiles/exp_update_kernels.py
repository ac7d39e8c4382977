#!/usr/bin/env python3
"""Round 6: one DDQN update's kernels (the bench's win-rate learner: batch 1,024, captured graph,
sequential schedule), 200 updates after 20 warm-up ones, for a rocprofv3 kernel trace; prints the
HIP-event time per update."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402


def main():
    from mazerl import VectorMazeEnv
    from mazerl.agents.dqn import VectorDQNLearner
    from test_learner_graph import _fill
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    env = VectorMazeEnv(4, 21, enrich=True, device="cuda", seed=1)
    L = VectorDQNLearner(4, "cuda", variant="ddqn", batch_size=batch, capacity=8192,
                         updates_per_step=1, target_every=13, seed=5, use_graph=True, overlap=False)
    for k in range(8):
        _fill(L, n=1024, seed=k)
    for _ in range(20):
        L.update(env.expand_window)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200):
        L.update(env.expand_window)
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"batch": batch, "us_per_update": round(e0.elapsed_time(e1) / 200 * 1000, 1)}),
          flush=True)
    env.close()


if __name__ == "__main__":
    main()
