#!/usr/bin/env python3
"""Where a config-5 PPO vector step goes (synchronised phase timers; not the production path):
act (f32 actor-critic forward + draw + record), env step, episode finishing into the pool,
auto-reset (+ regeneration of winners), and the update when the pool is full."""
import collections
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))

import torch  # noqa: E402

from mazerl.trainers.ppo_trainer import VectorPPOTrainer  # noqa: E402
from mazerl.trainers.vector_trainer import make_env  # noqa: E402


def main(B=4096, steps=300):
    dev = torch.device("cuda:0")
    env = make_env(B, list(range(17, 80, 2)), toroidal=True, seed=0x5EED0000, device=dev,
                   done_list=False, reward64=True, window=False, window_bits=True)
    tr = VectorPPOTrainer(env, dev, gamma=0.9, batch_size=2048, ppo_steps=2, pool_size=32768)
    tr.train(20)
    acc = collections.defaultdict(float)

    def tick(name, t0):
        torch.cuda.synchronize()
        t = time.perf_counter()
        acc[name] += t - t0
        return t

    t = time.perf_counter()
    for k in range(steps):
        tr._act()  # f32 forward + mz_ppo_act (draw + record)
        t = tick("act", t)
        env.step(tr.act_out)
        t = tick("env_step", t)
        tr._scan_finish()  # mz_ppo_scan + mz_ppo_finish (returns / advantages -> pool)
        t = tick("finish", t)
        env.reset_done(regen_won=True)
        t = tick("reset_regen", t)
        if tr._due():
            tr._update(k / steps)
        t = tick("update", t)
    tot = sum(acc.values())
    print(json.dumps({"envs": B, "steps": steps, "ms_per_vector_step": round(tot / steps * 1e3, 3),
                      **{k: round(v / steps * 1e3, 3) for k, v in acc.items()}}), flush=True)


if __name__ == "__main__":
    main()
