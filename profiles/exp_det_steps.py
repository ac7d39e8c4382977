#!/usr/bin/env python3
"""Per-vector-step fingerprints of exp_det_trail.py's live run (as-is: overlapped learner, maze
bank, per-instance curriculum), recorded on the device after every vector step without a host
wait (the race being chased depends on timing): the acting forward's greedy slots, the actions,
the rewards, the next observations, steps_done, epsilon and the instances' algorithms. Runs that
print different lines part at the first step whose fingerprint differs.

  python profiles/exp_det_steps.py 450
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))

import torch  # noqa: E402


def main(steps=450, chunk=25):
    from mazerl import VectorMazeEnv
    from mazerl.agents.dqn import VectorDQNLearner
    from mazerl.trainers.vector_trainer import VectorOffPolicyTrainer
    dev = torch.device("cuda", 0)
    env = VectorMazeEnv(4096, 41, enrich=True, device=dev, algorithm="r-prim", seed=0xC0CC0000,
                        done_list=False, window=False, window_bits=True)
    L = VectorDQNLearner(4096, dev, variant="ddqn", lr=1e-3, eps_start=0.95, eps_final=0.1,
                         eps_decay=400.0, gamma=0.7, batch_size=1024, capacity=1 << 20,
                         updates_per_step=4, target_every=13, overlap=True, seed=1)
    tr = VectorOffPolicyTrainer(env, L, seed=11, curriculum="per-instance")
    if os.environ.get("MZ_TRAIL_BANK_MAIN") == "1":  # the bank's refills on the main stream
        env._bank["side"] = torch.cuda.current_stream(dev)
    idx = torch.arange(1, 4097, device=dev, dtype=torch.float64)
    rec = torch.zeros(steps + 1, 8, dtype=torch.float64, device=dev)
    n = [0]
    orig = tr.vector_step

    def step():
        out = orig()
        k = n[0]
        rows = getattr(L, "_rows", None)
        if rows is not None:
            rec[k, 0] = (rows.greedy.double() * idx).sum()
            rec[k, 1] = rows.count.double().sum()
        rec[k, 2] = (env.actions.double() * idx).sum()
        rec[k, 3] = (env.reward.double() * idx).sum()
        rec[k, 4] = (env.obs6.double().sum(1) * idx).sum()
        rec[k, 5] = (L.steps_done.double() * idx).sum()
        if tr._eps is not None:
            rec[k, 6] = (tr._eps.double() * idx).sum()
        sch = tr.schedule
        if sch is not None:
            rec[k, 7] = (sch.algo.double() * idx).sum()
        n[0] += 1
        return out
    tr.vector_step = step
    for k in range(0, int(steps), chunk):
        tr.train(min(chunk, int(steps) - k))
    torch.cuda.synchronize()
    r = rec[:n[0]].cpu().tolist()
    print(json.dumps({"bank_main": os.environ.get("MZ_TRAIL_BANK_MAIN"), "steps": n[0], "rec": [[float.hex(x) for x in row] for row in r]}), flush=True)
    env.close()


if __name__ == "__main__":
    main(*[int(x) for x in sys.argv[1:]])
