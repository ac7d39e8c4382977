"""McClendon maze difficulty (lib/maze_difficulty_evaluation/maze_complexity_evaluation.py:38-329).

Not ported yet: calling it raises NotImplementedError rather than returning a
made-up value.
"""


def maze_difficulty(grid, start, goal):
    raise NotImplementedError("McClendon difficulty port pending (SURVEY §8f rank 1)")
