from ...envs import (SimpleEnrichMazeEnv, SimpleEnrichVariableMazeEnv, SimpleMazeEnv,  # noqa: F401
                     SimpleVariableMazeEnv, ToroidalEnrichMazeEnv, ToroidalEnrichVariableMazeEnv,
                     ToroidalMazeEnv, ToroidalVariableMazeEnv)
