#!/usr/bin/env python3
"""Determinism trail of tests/live_train_digest.py's run (4,096 x 41^2, DDQN, overlapped learner,
K = 4 updates of 1,024 per vector step, per-instance curriculum, maze bank): a digest of the
source net, the optimizer moments, the replay rewards and the win / episode counters after every
train() call of 25 vector steps (MZ_TRAIL_OVERLAP / _BANK / _CURR switch the overlapped
learner, the maze bank and the curriculum off: 0 / 0 / ""), for the package under MZ_PKG_ROOT (default: this repo) — two
runs of one package that print different trails show the first chunk where they part.

  MZ_PKG_ROOT=profiles/_bin/headwt python profiles/exp_det_trail.py 600
"""
import hashlib
import json
import os
import sys

ROOT = os.environ.get("MZ_PKG_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(os.path.abspath(ROOT), "maze-solving-agent-gymnasium_amd"))

import torch  # noqa: E402


def dg(t):
    return hashlib.sha256(t.detach().cpu().numpy().tobytes()).hexdigest()[:12]


def main(steps=600, chunk=25):
    from mazerl import VectorMazeEnv
    from mazerl.agents.dqn import VectorDQNLearner
    from mazerl.trainers.vector_trainer import VectorOffPolicyTrainer
    dev = torch.device("cuda", 0)
    env = VectorMazeEnv(4096, 41, enrich=True, device=dev, algorithm="r-prim", seed=0xC0CC0000,
                        done_list=False, window=False, window_bits=True)
    L = VectorDQNLearner(4096, dev, variant="ddqn", lr=1e-3, eps_start=0.95, eps_final=0.1,
                         eps_decay=400.0, gamma=0.7, batch_size=1024, capacity=1 << 20,
                         updates_per_step=4, target_every=13,
                         overlap=os.environ.get("MZ_TRAIL_OVERLAP", "1") == "1", seed=1)
    tr = VectorOffPolicyTrainer(env, L, seed=11, bank=os.environ.get("MZ_TRAIL_BANK", "1") == "1",
                                curriculum=os.environ.get("MZ_TRAIL_CURR", "per-instance") or None)
    trail = []
    for k in range(0, int(steps), chunk):
        tr.train(min(chunk, int(steps) - k))
        torch.cuda.synchronize()
        trail.append({"step": k + chunk, "src": dg(L.source._flat_params), "m": dg(L.opt.exp_avg),
                      "tgt": dg(L.target._flat_params), "sd": dg(L.steps_done),
                      "r": dg(L.replay.r[:L.replay.size]), "sw": dg(L.replay.sw[:L.replay.size]),
                      "a": dg(L.replay.a[:L.replay.size]), "s6": dg(L.replay.s6[:L.replay.size]),
                      "wins": int(tr.wins), "eps": int(tr.episodes), "upd": L.n_updates})
    print(json.dumps({"pkg": os.path.basename(os.path.abspath(ROOT)),
                      "variant": {k: os.environ.get(k) for k in ("MZ_TRAIL_OVERLAP", "MZ_TRAIL_BANK",
                                                                 "MZ_TRAIL_CURR")},
                      "kblock": os.environ.get("MZ_K_BLOCK"), "trail": trail}), flush=True)
    env.close()


if __name__ == "__main__":
    main(*[int(x) for x in sys.argv[1:]])
