"""Tabular Q-learning agent (config 1): the reference's QAgent (agents/q_agent.py:8-79).

Q-table keyed by str(obs) exactly as the reference (the drop-in envs return the same numpy dtypes,
so the keys are the same strings); TD(0) update with (not terminated) bootstrap cut; epsilon from
steps_done; random actions from env.action_space.sample(); gamma drift by +-eta per episode.
"""
from __future__ import annotations

import math
from collections import defaultdict

import numpy as np


class QAgent:
    def __init__(self, env, learning_rate: float, initial_epsilon: float, epsilon_decay: float,
                 final_epsilon: float, discount_factor: float, eta: float):
        self.env = env
        self.q_values = defaultdict(lambda: np.zeros(self.env.action_space.n))
        self.lr = learning_rate
        self.discount_factor = discount_factor
        self.eta = eta
        self.initial_epsilon = initial_epsilon
        self.epsilon_decay = epsilon_decay
        self.final_epsilon = final_epsilon
        self.steps_done = 0
        self.training_error = []

    def get_action(self, obs) -> int:
        eps = self.final_epsilon + (self.initial_epsilon - self.final_epsilon) * \
            math.exp(-1. * self.steps_done / self.epsilon_decay)
        self.steps_done += 1
        if np.random.random() < eps:
            return self.env.action_space.sample()
        return int(np.argmax(self.q_values[str(obs)]))

    def update(self, obs, action: int, reward: float, terminated: bool, next_obs):
        future = (not terminated) * np.max(self.q_values[str(next_obs)])
        td = reward + self.discount_factor * future - self.q_values[str(obs)][action]
        self.q_values[str(obs)][action] = self.q_values[str(obs)][action] + self.lr * td
        self.training_error.append(td)

    def update_hyperparameter(self, is_better: bool):
        self.discount_factor = self.discount_factor + (self.eta if is_better else -self.eta)
