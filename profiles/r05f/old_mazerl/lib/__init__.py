"""Module-path mirror of the reference's `lib` package for the parts on the hot path's boundary
(SURVEY §8b item 2): `lib.maze_generation.gen_maze / gen_maze_no_border` and
`lib.maze_difficulty_evaluation.maze_complexity_evaluation.ComplexityEvaluation`."""
