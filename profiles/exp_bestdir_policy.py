#!/usr/bin/env python3
"""Round 4 sanity check of the evaluation path on every generator: a scripted policy that follows
obs["best dir"] (the env's shortest-path hint, base_maze_env.py:224-262) must win (nearly) every
fresh 81x81 maze of each algorithm, as generated and best-of-6 — so a learner's 0 % on dfs /
prim&kill mazes is the learner's, not the evaluation's. One JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))

import torch  # noqa: E402


class BestDir:
    """greedy(obs6) = the action that moves onto best dir's cell: obs6[4:6] = agent - next."""
    supports_bits = True

    def greedy(self, obs6, window, bits=None):
        d = -obs6[:, 4:6].round().long()  # next - agent
        a = torch.zeros(obs6.shape[0], dtype=torch.int64, device=obs6.device)
        a[(d[:, 0] == -1)] = 1
        a[(d[:, 1] == 1)] = 2
        a[(d[:, 1] == -1)] = 3
        return a


def main():
    from mazerl.trainers.vector_trainer import best_of_mazes, evaluate, maze_algorithms
    dev = torch.device("cuda", 0)
    L = BestDir()
    out = {}
    for algo in ("r-prim", "dfs", "prim&kill"):
        g, k = evaluate(L, 300, 81, algo, seed=0xB0D1, eps=0.0, device=dev)
        mz = best_of_mazes(300, 81, algo, seed=0xB0D2, device=dev)
        g6, k6 = evaluate(L, 300, 81, seed=0xB0D2, eps=0.0, device=dev, mazes=mz)
        out[algo] = {"generated": g, "best_of_6": g6, "vector_steps": [k, k6]}
    algos = maze_algorithms(300, seed=0xB0D3)
    mz = best_of_mazes(300, 81, algos, seed=0xB0D3, device=dev)
    r, k, won = evaluate(L, 300, 81, seed=0xB0D3, eps=0.0, device=dev, mazes=mz, return_won=True)
    out["mixed_best_of_6"] = {"rate": r, "by_algorithm": {a: float(won[[x == a for x in algos]].mean())
                                                          for a in sorted(set(algos))}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
