#!/usr/bin/env python3
"""McClendon difficulty / complexity of more reference mazes, from the reference's own code: mazes
from random.seed(s) + gen_maze (euclidean) and gen_maze_no_border re-bordered (toroidal, the
maze the reference scores: off_policy_trainer.py:194-196) over 3 algorithms and several sizes,
scored by ComplexityEvaluation(maze, start, goal).difficulty_of_maze() / complexity_of_maze()
(lib/maze_difficulty_evaluation/maze_complexity_evaluation.py:38-329). These pin the set-order
hallway sums (networkx subgraph views iterate a CPython set, :217-218, 283-295) on many more
hallways than gen_euclid.npz / gen_toroid.npz. Test infrastructure only (build container).
Writes tests/golden/mcclendon.npz (data only: padded grids, start / goal, values).
"""
import os
import random
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

ALGOS = ["r-prim", "dfs", "prim&kill"]
EUCLID = [(9, 6), (15, 10), (21, 10), (31, 10), (41, 8), (61, 4)]   # (size, seeds per algorithm)
TOROID = [(9, 6), (17, 8), (29, 8), (41, 6)]
SEED0 = 1000


def main(ref="/root/reference"):
    from make_golden import load_reference
    R = load_reference(ref)
    mg = R["mg"]
    rows = []
    t0 = time.time()
    for tor, sizes in ((0, EUCLID), (1, TOROID)):
        for n, seeds in sizes:
            for a, algo in enumerate(ALGOS):
                for s in range(SEED0, SEED0 + seeds):
                    random.seed(s)
                    if tor:
                        start, goal, grid, _ = mg.gen_maze_no_border((n, n), algo)
                        grid = np.pad(np.asarray(grid, np.uint8), 1)
                        start, goal = (start[0] + 1, start[1] + 1), (goal[0] + 1, goal[1] + 1)
                    else:
                        start, goal, grid = mg.gen_maze((n, n), algo)
                        grid = np.asarray(grid, np.uint8)
                    g = [list(map(int, r)) for r in grid]
                    try:
                        ce = R["CE"](g, tuple(start), tuple(goal))
                        d, c = float(ce.difficulty_of_maze()), float(ce.complexity_of_maze())
                    except Exception:  # degenerate tiny mazes (log of 0)
                        d = c = float("nan")
                    rows.append((tor, a, n, s, grid, tuple(start), tuple(goal), d, c))
                print(tor, n, algo, round(time.time() - t0, 1), flush=True)
    m = max(r[4].shape[0] for r in rows)
    grids = np.zeros((len(rows), m, m), np.uint8)
    for i, r in enumerate(rows):
        grids[i, :r[4].shape[0], :r[4].shape[1]] = r[4]
    np.savez_compressed(
        os.path.join(HERE, "mcclendon.npz"),
        toroidal=np.array([r[0] for r in rows], np.uint8), algo=np.array([r[1] for r in rows], np.uint8),
        n=np.array([r[4].shape[0] for r in rows], np.int32), seed=np.array([r[3] for r in rows], np.int32),
        grid=grids, start=np.array([r[5] for r in rows], np.int32),
        goal=np.array([r[6] for r in rows], np.int32),
        difficulty=np.array([r[7] for r in rows]), complexity=np.array([r[8] for r in rows]))


if __name__ == "__main__":
    main(*sys.argv[1:])
