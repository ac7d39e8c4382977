"""Drop-in for the reference's McClendon evaluator (lib/maze_difficulty_evaluation/
maze_complexity_evaluation.py:38-329): ComplexityEvaluation(maze, start_pos, goal_pos) with
difficulty_of_maze() and complexity_of_maze(), computed by libmazerl's native restatement
(mz_maze_complexity: the turn-decomposed graph, hallways and branches in networkx's insertion /
adjacency order, each hallway summed in its CPython set order) instead of networkx. Values:
bit-exact (==) with the reference's on every golden maze (tests/test_difficulty.py)."""
import ctypes as C

import numpy as np

from ... import _native as N


class ComplexityEvaluation:
    def __init__(self, maze, start_pos, goal_pos):
        self.maze = maze
        self.start_pos = start_pos
        self.goal_pos = goal_pos
        self._vals = None

    def _eval(self):
        if self._vals is None:
            g = np.ascontiguousarray(np.asarray(self.maze), dtype=np.uint8)
            d, c = C.c_double(), C.c_double()
            N.check(N.load().mz_maze_complexity(
                g.ctypes.data, g.shape[0], g.shape[1], int(self.start_pos[0]), int(self.start_pos[1]),
                int(self.goal_pos[0]), int(self.goal_pos[1]), C.byref(d), C.byref(c)))
            self._vals = (d.value, c.value)
        return self._vals

    def difficulty_of_maze(self):
        """log of the product over branches (:319-329)."""
        return self._eval()[0]

    def complexity_of_maze(self):
        """log of the summed branch complexities (:311-317)."""
        return self._eval()[1]
