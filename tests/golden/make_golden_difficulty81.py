#!/usr/bin/env python3
"""McClendon difficulty / complexity at the headline size from the reference's own code: the 24
81x81 reference mazes of gen_euclid.npz (3 algorithms x 8 seeds, random.seed(s) + gen_maze) through
ComplexityEvaluation(maze, start, goal).difficulty_of_maze() / complexity_of_maze()
(lib/maze_difficulty_evaluation/maze_complexity_evaluation.py:38-329) — the values make_golden.py
leaves NaN above 41x41 (seconds per maze there). Test infrastructure only (build container).
Writes tests/golden/difficulty81.npz (data only).
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def main(ref="/root/reference"):
    from make_golden import load_reference
    R = load_reference(ref)
    g = np.load(os.path.join(HERE, "gen_euclid.npz"))
    sel = np.nonzero(g["n"] == 81)[0]
    diff, comp, secs = [], [], []
    for i in sel:
        n = int(g["n"][i])
        grid = [list(map(int, r)) for r in g["grid"][i][:n, :n]]
        start, goal = tuple(int(x) for x in g["start"][i]), tuple(int(x) for x in g["goal"][i])
        t0 = time.time()
        ce = R["CE"](grid, start, goal)
        diff.append(float(ce.difficulty_of_maze()))
        comp.append(float(ce.complexity_of_maze()))
        secs.append(time.time() - t0)
        print(i, int(g["algo"][i]), int(g["seed"][i]), diff[-1], round(secs[-1], 2), flush=True)
    np.savez_compressed(os.path.join(HERE, "difficulty81.npz"), index=sel.astype(np.int32),
                        difficulty=np.array(diff), complexity=np.array(comp))


if __name__ == "__main__":
    main(*sys.argv[1:])
