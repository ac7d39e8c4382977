"""Module-path mirror of the reference's gymnasium_env package (gymnasium_env/__init__.py):
`from mazerl.gymnasium_env.envs.simple_maze_env import SimpleEnrichMazeEnv` etc."""
from ..envs import ENV_IDS, make, register_gymnasium  # noqa: F401

register_gymnasium()
