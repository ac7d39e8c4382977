#!/usr/bin/env python3
"""Mean per-instance epsilon over the bench's DDQN training leg (65,536 x 81x81 r-prim): the
fraction of actions that come from the Q-network (1 - eps) — how much of the acting forward a
greedy-rows-only forward could skip. Same learner / trainer settings as bench.py win_rate()."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))
import torch  # noqa: E402

from mazerl import VectorMazeEnv  # noqa: E402
from mazerl.agents.dqn import VectorDQNLearner  # noqa: E402
from mazerl.trainers.vector_trainer import VectorOffPolicyTrainer  # noqa: E402

dev = torch.device("cuda", 0)
B, dim = 65536, 81
env = VectorMazeEnv(B, dim, enrich=True, device=dev, algorithm="r-prim", seed=0xA11CE,
                    done_list=False, window=False, window_bits=True)
decay = ((dim - 1) * (dim - 1) // 2) * 5 / 40.0
L = VectorDQNLearner(B, dev, variant="ddqn", lr=1e-3, eps_start=0.95, eps_final=0.1, eps_decay=decay,
                     gamma=0.7, batch_size=1024, capacity=2_000_000, target_every=13, overlap=True)
tr = VectorOffPolicyTrainer(env, L, seed=3)
acc, n = 0.0, 0
for k in range(2420):
    tr.vector_step()
    if k % 20 == 0:
        e = float(L.epsilon().mean())
        acc += e
        n += 1
        if k % 200 == 0:
            print(json.dumps({"step": k, "eps_mean": round(e, 4), "wins": int(tr.wins),
                              "episodes": int(tr.episodes)}), flush=True)
print(json.dumps({"eps_mean_over_training": acc / n, "greedy_fraction": 1 - acc / n}))
