"""Module-path mirror of the reference's agents/ddqn_agent.py."""
from ..replay import ReplayMemory, Transition  # noqa: F401
from .dqn import DDQNAgent  # noqa: F401
from .nets import QNet as _QNet


def DQN(in_channels, n_observations, n_actions, h_channels, hidden_dim=1024):
    return _QNet(in_channels, n_observations, n_actions, h_channels, hidden_dim, "ddqn")
