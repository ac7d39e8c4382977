"""McClendon maze difficulty (maze_complexity_evaluation.py:38-329) via libmazerl's native
mz_difficulty — used by get_maze_difficulty and best-of-6 generation (base_maze_env.py:78-105)."""
import ctypes as C

import numpy as np

from . import _native as N


def maze_difficulty(grid, start, goal):
    """ComplexityEvaluation(grid, start, goal).difficulty_of_maze() for a euclidean grid."""
    g = np.ascontiguousarray(grid, dtype=np.uint8)
    out = C.c_double()
    N.check(N.load().mz_difficulty(g.ctypes.data, g.shape[0], g.shape[1], int(start[0]),
                                   int(start[1]), int(goal[0]), int(goal[1]), C.byref(out)))
    return out.value


def toroidal_difficulty(grid, start, goal):
    """Difficulty of a cropped toroidal maze, evaluated on its bordered (N+2) grid like
    gen_maze_no_border (maze_generation.py:49-51) and the trainer (off_policy_trainer.py:194-196)."""
    g = np.pad(np.asarray(grid, np.uint8), 1)
    return maze_difficulty(g, (start[0] + 1, start[1] + 1), (goal[0] + 1, goal[1] + 1))
