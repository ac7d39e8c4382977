from ...envs import ToroidalEnrichVariableMazeEnv, ToroidalVariableMazeEnv  # noqa: F401
