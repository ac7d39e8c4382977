from ...envs import SimpleEnrichMazeEnv, SimpleMazeEnv  # noqa: F401  (simple_maze_env.py)
