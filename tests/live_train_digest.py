"""A short live DDQN training run (the bench's curriculum leg in small: overlapped learner, K = 4
updates of 1,024 per vector step, per-instance curriculum, maze bank) printing one JSON line with
a digest of everything the run produced: the source / target nets, the optimizer moments, the
replay rows, steps_done, win / episode counters. tests/test_determinism_gpu.py runs it twice in
fresh processes and compares the lines. MZ_K_BLOCK selects the K-update graph (agents/dqn.py).
Training runs as train() calls of 100 vector steps, each ending with the learner's finish()."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))

import torch  # noqa: E402


def main(steps=600, envs=4096, dim=41):
    from mazerl import VectorMazeEnv
    from mazerl.agents.dqn import VectorDQNLearner
    from mazerl.trainers.vector_trainer import VectorOffPolicyTrainer
    dev = torch.device("cuda", 0)
    env = VectorMazeEnv(envs, dim, enrich=True, device=dev, algorithm="r-prim", seed=0xC0CC0000,
                        done_list=False, window=False, window_bits=True)
    L = VectorDQNLearner(envs, dev, variant="ddqn", lr=1e-3, eps_start=0.95, eps_final=0.1,
                         eps_decay=400.0, gamma=0.7, batch_size=1024, capacity=1 << 20,
                         updates_per_step=4, target_every=13, overlap=True, seed=1)
    tr = VectorOffPolicyTrainer(env, L, seed=11, curriculum="per-instance")
    # in chunks: every train() call ends with learner.finish() and the next one restarts the
    # overlapped learner (what the K-update graph's index buffers must survive)
    for k in range(0, int(steps), 100):
        tr.train(min(100, int(steps) - k))
    torch.cuda.synchronize()
    h = hashlib.sha256()
    parts = {}
    for name, t in (("source", L.source._flat_params), ("target", L.target._flat_params),
                    ("exp_avg", L.opt.exp_avg), ("exp_avg_sq", L.opt.exp_avg_sq),
                    ("steps_done", L.steps_done),
                    ("replay_sw", L.replay.sw[:L.replay.size]),
                    ("replay_r", L.replay.r[:L.replay.size])):
        d = hashlib.sha256(t.detach().cpu().numpy().tobytes()).hexdigest()[:16]
        parts[name] = d
        h.update(d.encode())
    rec = {"digest": h.hexdigest()[:16],
           "parts": parts, "wins": int(tr.wins), "episodes": int(tr.episodes),
           "n_updates": L.n_updates}
    print(json.dumps(rec), flush=True)
    env.close()


if __name__ == "__main__":
    main(*[int(x) for x in sys.argv[1:]])
