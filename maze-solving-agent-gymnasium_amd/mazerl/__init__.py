"""mazerl — MI355X-native batched maze environment (drop-in for the reference's gymnasium_env).

Compute runs only in libmazerl.so (HIP kernels for gfx950, C ABI in include/mazerl.h).
"""
from .vector_env import VectorMazeEnv, ALGOS  # noqa: F401

__all__ = ["VectorMazeEnv", "ALGOS"]
