from ...envs import SimpleEnrichVariableMazeEnv, SimpleVariableMazeEnv  # noqa: F401
