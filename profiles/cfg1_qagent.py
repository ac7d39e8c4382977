#!/usr/bin/env python3
"""Config 1 (BASELINE.json configs[0]): one 9x9 r-prim maze, tabular Q-learning, one instance —
the reference's training_examples/euclidean_mazes/costant_sizes/test_q.py protocol on the GPU
drop-in env (mazerl.envs.SimpleMazeEnv; every step / reset / new maze is a gfx950 kernel):

  OffPolicyTrainer.train(n_episodes)   lib/trainers/off_policy_trainer.py:21-82 (restated here:
                                       the reference cannot travel to the GPU box): reset, play one
                                       episode with get_action / step / update, on a win
                                       update_maze() (a new best-of-6 maze), gamma drift by +-eta
  test(len(env.mazes), new=False)      :84-119, seen mazes (update_visited_maze(remove=True))
  test(250, new=True)                  fresh mazes (update_new_maze())

Hyper-parameters from test_q.py:17-25 with maze_shape (9, 9): lr 1e-3, eps 0.95 -> 0.05, decay
9*9 // 2, gamma 0.7, eta 1e-2. Prints one JSON line: env steps/s of the single instance (the
per-step host round trip dominates: Python agent + ctypes launch + device->host obs copy) and
the win-rates. The reference's own CPU env runs 3,970 steps/s per core at 9x9.
"""
import argparse
import json
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))


T = {"step": 0.0, "reset": 0.0, "update_maze": 0.0}


def train(env, agent, n_episodes):
    steps = wins = 0
    prev_cum = 0.0
    for _ in range(n_episodes):
        t = time.perf_counter()
        obs, _ = env.reset()
        T["reset"] += time.perf_counter() - t
        done, cum, win = False, 0.0, False
        while not done:
            a = agent.get_action(obs)
            t = time.perf_counter()
            nobs, r, truncated, terminated, _ = env.step(a)
            T["step"] += time.perf_counter() - t
            cum += r
            agent.update(obs, a, r, terminated, nobs)
            done = terminated or truncated
            win = terminated
            obs = nobs
            steps += 1
        if win:
            wins += 1
            t = time.perf_counter()
            env.env.update_maze()
            T["update_maze"] += time.perf_counter() - t
        agent.update_hyperparameter(cum > prev_cum)
        prev_cum = cum
    return steps, wins


def test(env, agent, n, new):
    won = steps = 0
    for _ in range(n):
        if new:
            env.env.update_new_maze()
        else:
            env.env.update_visited_maze(remove=True)
        obs, _ = env.reset()
        done = False
        while not done:
            a = agent.get_action(obs)
            obs, r, truncated, terminated, _ = env.step(a)
            steps += 1
            if terminated:
                won += 1
            done = terminated or truncated
    return won / max(1, n), steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--episodes", type=int, default=350)
    ap.add_argument("--dim", type=int, default=9)
    ap.add_argument("--test-new", type=int, default=250)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    from mazerl import envs
    from mazerl.agents.q_agent import QAgent
    random.seed(a.seed)
    np.random.seed(a.seed)
    env = envs.SimpleMazeEnv((a.dim, a.dim))
    agent = QAgent(env, learning_rate=1e-3, initial_epsilon=0.95, final_epsilon=0.05,
                   epsilon_decay=a.dim * a.dim // 2, discount_factor=0.7, eta=1e-2)
    t0 = time.perf_counter()
    steps, wins = train(env, agent, a.episodes)
    dt = time.perf_counter() - t0
    n_seen = len(env.env.mazes)
    t1 = time.perf_counter()
    wr_seen, s1 = test(env, agent, n_seen, new=False)
    wr_new, s2 = test(env, agent, a.test_new, new=True)
    dt_test = time.perf_counter() - t1
    print(json.dumps({"config": "cfg1: one 9x9 r-prim maze, tabular Q (QAgent), 1 instance, GPU drop-in env",
                      "episodes": a.episodes, "train_steps": steps, "train_wins": wins,
                      "train_seconds": round(dt, 2), "train_env_steps_per_s": steps / dt,
                      "train_seconds_by_call": {k: round(v, 3) for k, v in T.items()},
                      "us_per_env_step_call": T["step"] / max(1, steps) * 1e6,
                      "test_seen_mazes": n_seen, "win_rate_seen": wr_seen,
                      "win_rate_new": wr_new, "test_new_mazes": a.test_new,
                      "test_env_steps_per_s_incl_new_mazes": (s1 + s2) / dt_test,
                      "reference_cpu_env_steps_per_s_per_core_9x9": 3970}), flush=True)
    env.close()


if __name__ == "__main__":
    main()
