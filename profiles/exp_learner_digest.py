#!/usr/bin/env python3
"""Round 6: a digest of the DDQN learner's weights after 20 graph-captured updates (batch 512,
dropout active) for the library named by MZ_LIB_OVERRIDE — equal digests = bit-identical updates."""
import hashlib
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
    torch.cuda.manual_seed(7)
    env = VectorMazeEnv(4, 21, enrich=True, device="cuda", seed=1)
    L = VectorDQNLearner(4, "cuda", variant="ddqn", batch_size=512, capacity=4096,
                         updates_per_step=1, target_every=13, seed=5, use_graph=True, overlap=False)
    for k in range(8):
        _fill(L, n=512, seed=k)
    losses = [float(L.update(env.expand_window)) for _ in range(20)]
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for p in L.source.parameters():
        h.update(p.detach().cpu().numpy().tobytes())
    print(json.dumps({"lib": os.path.basename(os.environ.get("MZ_LIB_OVERRIDE", "default")),
                      "digest": h.hexdigest()[:16], "last_loss": losses[-1]}), flush=True)
    env.close()


if __name__ == "__main__":
    main()
