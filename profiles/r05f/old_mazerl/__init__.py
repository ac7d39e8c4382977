"""mazerl — MI355X-native batched maze environment (drop-in for the reference's gymnasium_env).

Compute runs only in libmazerl.so (HIP kernels for gfx950, C ABI in include/mazerl.h).
"""
import os as _os

# The learner's 3x3 conv runs through MIOpen: use its immediate-mode heuristics instead of a
# benchmarking search on first use (the search costs tens of seconds per new shape).
_os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")

from .vector_env import VectorMazeEnv, ALGOS  # noqa: F401,E402

__all__ = ["VectorMazeEnv", "ALGOS"]
