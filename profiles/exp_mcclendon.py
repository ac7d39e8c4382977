#!/usr/bin/env python3
"""Timing of the McClendon difficulty paths (round 3, VERDICT "GPU McClendon kernel"; round 4:
hallway sums in the reference's set order, toroidal handles scored on the GPU).

best-of-6 selection of 1,000 81x81 mazes (6,000 candidates, base_maze_env.py:78-97):
  gpu_kernel_ms      mz_difficulty_batch over the 6,000 resident candidates (HIP events)
  best_of_mazes_s    the whole mazerl best_of_mazes call (generation + kernel + 1,000 grid copies)
  host_per_maze_ms   the host restatement (mz_difficulty) per maze incl. its grid copy, on a
                     300-maze sample — what best_of_mazes paid per candidate before
Prints one JSON line.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))

import torch  # noqa: E402


def main():
    from mazerl import VectorMazeEnv
    from mazerl import _native as N
    from mazerl.difficulty import maze_difficulty
    from mazerl.trainers.vector_trainer import best_of_mazes
    dev = torch.device("cuda", 0)
    out = {}
    for algo in ("r-prim", "dfs", "prim&kill"):
        env = VectorMazeEnv(6000, 81, enrich=True, device=dev, algorithm=algo, seed=0x7E57,
                            done_list=False, pos=False, window=False, window_bits=False)
        res = torch.empty(6000, 2, dtype=torch.float64, device=dev)
        st = torch.empty(6000, dtype=torch.int32, device=dev)
        lib = N.load()
        s = env._stream()
        for _ in range(2):
            N.check(lib.mz_difficulty_batch(env._h, None, 6000, res.data_ptr(), st.data_ptr(), s))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 5
        e0.record()
        for _ in range(reps):
            N.check(lib.mz_difficulty_batch(env._h, None, 6000, res.data_ptr(), st.data_ptr(), s))
        e1.record()
        torch.cuda.synchronize()
        import numpy as np
        from mazerl.difficulty import difficulty_batch
        stv = st.cpu().numpy()
        rec = {"gpu_kernel_ms": e0.elapsed_time(e1) / reps,
               "status_nonzero": int((stv != 0).sum()),
               "status_counts": {int(k): int(v) for k, v in zip(*np.unique(stv, return_counts=True))}}
        # near ties: relative gap between the smallest and the second smallest difficulty of
        # each group of 6 candidates
        d = difficulty_batch(env).reshape(1000, 6)
        srt = np.sort(d, axis=1)
        gap = (srt[:, 1] - srt[:, 0]) / np.abs(srt[:, 0])
        rec["best_of_6_min_rel_gap"] = float(gap.min())
        rec["groups_gap_below_1e-12"] = int((gap < 1e-12).sum())
        rec["groups_exact_tie"] = int((gap == 0).sum())
        t0 = time.perf_counter()
        for i in range(300):
            q = env.query(i)
            maze_difficulty(env.grid(i), (q["start_r"], q["start_c"]), (q["goal_r"], q["goal_c"]))
        rec["host_per_maze_ms"] = (time.perf_counter() - t0) / 300 * 1e3
        env.close()
        best_of_mazes(20, 81, algo, device=dev)  # warm
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        best_of_mazes(1000, 81, algo, device=dev)
        rec["best_of_mazes_s"] = time.perf_counter() - t0
        rec["host_6000_estimate_s"] = rec["host_per_maze_ms"] * 6000 / 1e3
        out[algo] = rec
        print(algo, rec, file=sys.stderr, flush=True)
    # toroidal: config 5's sizes, 3,000 candidates (500 mazes x 6), scored on the bordered grid
    from mazerl.difficulty import toroidal_difficulty
    from mazerl.trainers.vector_trainer import make_env
    dims = list(range(17, 80, 2))
    tor = {}
    for algo in ("r-prim", "dfs", "prim&kill"):
        env = make_env(3000, dims, toroidal=True, algorithm=algo, seed=0x70E5, device=dev,
                       done_list=False, pos=False, window=False, window_bits=False)
        res = torch.empty(3000, 2, dtype=torch.float64, device=dev)
        st = torch.empty(3000, dtype=torch.int32, device=dev)
        lib, s = N.load(), env._stream()
        for _ in range(2):
            N.check(lib.mz_difficulty_batch(env._h, None, 3000, res.data_ptr(), st.data_ptr(), s))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            N.check(lib.mz_difficulty_batch(env._h, None, 3000, res.data_ptr(), st.data_ptr(), s))
        e1.record()
        torch.cuda.synchronize()
        rec = {"gpu_kernel_ms": e0.elapsed_time(e1) / 5, "status_nonzero": int((st != 0).sum())}
        t0 = time.perf_counter()
        for i in range(200):
            q = env.query(i)
            toroidal_difficulty(env.grid(i), (q["start_r"], q["start_c"]), (q["goal_r"], q["goal_c"]))
        rec["host_per_maze_ms"] = (time.perf_counter() - t0) / 200 * 1e3
        env.close()
        t0 = time.perf_counter()
        best_of_mazes(500, dims, algo, device=dev, toroidal=True)
        rec["best_of_mazes_500_s"] = time.perf_counter() - t0
        tor[algo] = rec
        print("toroidal", algo, rec, file=sys.stderr, flush=True)
    print(json.dumps({"mcclendon_best_of_6_x_1000_81x81": out,
                      "mcclendon_toroidal_3000_17_79": tor}), flush=True)


if __name__ == "__main__":
    main()
