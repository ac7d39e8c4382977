from ...envs import BaseMazeEnv  # noqa: F401  (gymnasium_env/envs/base_maze_env.py)
