from ...envs import ToroidalEnrichMazeEnv, ToroidalMazeEnv  # noqa: F401  (toroidal_maze_env.py)
