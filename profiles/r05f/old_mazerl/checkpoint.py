"""Checkpoint / resume of a vectorised training run (SURVEY §5 "checkpoint/resume").

The reference saves nothing for its agents or envs (only the CAE's weights, train_CAE.py:59,75;
its envs keep their mazes in Python lists, simple_maze_env.py:34,91). Here one file holds the
whole run of a VectorOffPolicyTrainer:

  env      the env handle's device state (mz_state_save: mazes with their BFS tables and visit
           counts, visited planes, per-instance state, the maze bank), the last step's outputs
  learner  source / target Q-nets (the reference's module names: the `source` entry loads into
           its DQN / DDQN classes with load_state_dict), optimizer moments / step / lr, the cosine
           schedule, per-instance steps_done and epsilon decay, the filled replay rows, and every
           random stream the next updates and acts draw from
  trainer  vector-step counter, win / episode counters, history

The same two calls take config 5's VectorPPOTrainer (its net and optimizer, the in-flight
episodes' records, the update pool, its counters and the env).

A resumed run continues bit-exactly where the saved one stood (tests/test_checkpoint_gpu.py).
Files are written with torch.save and read with torch.load(weights_only=True): tensors, numbers,
strings, lists and dicts only — nothing in a checkpoint executes on load.
"""
import os

import torch


def save_checkpoint(path, trainer):
    """Write `trainer`'s state (trainer.state_dict()) to `path` atomically (tmp file + rename)."""
    sd = trainer.state_dict()
    tmp = f"{path}.tmp{os.getpid()}"
    torch.save(sd, tmp)
    os.replace(tmp, path)
    return path


def load_checkpoint(path, trainer):
    """Restore a save_checkpoint() file into a trainer built with the same configuration (env
    size / instance count / bank, learner variant / replay capacity)."""
    dev = trainer.env.device
    sd = torch.load(path, map_location=dev, weights_only=True)
    trainer.load_state_dict(sd)
    return trainer


def load_qnet(path, net, which="source"):
    """The Q-network alone from a checkpoint (e.g. into the reference's DQN / DDQN class or a
    QNet for evaluation): `which` = "source" or "target"."""
    sd = torch.load(path, map_location="cpu", weights_only=True)
    net.load_state_dict(sd["learner"][which])
    return net
