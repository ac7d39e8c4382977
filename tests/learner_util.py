"""Deterministic inputs for the Q-loss parity fixtures (shared by tests/golden/make_golden_learner.py
and tests/test_learner.py). Pure data generation — no reference code."""
import numpy as np
import torch

REWARDS = [1.0, 0.45, -0.55, -1.0, -0.18126924692201818, -0.13929202357494222, -0.05]
CASES = {  # name: (variant, h_channels, hidden_dim, n, gamma, lr, train_mode)
    "dqn_small": ("dqn", 4, 8, 8, 0.7, 1e-3, False),
    "ddqn_small": ("ddqn", 4, 8, 8, 0.7, 1e-3, False),
    "ddqn_small_dropout": ("ddqn", 4, 8, 8, 0.7, 1e-3, True),
    "dqn_full": ("dqn", 32, 1024, 16, 0.7, 1e-3, False),
    "ddqn_full": ("ddqn", 32, 1024, 16, 0.7, 1e-3, False),
}


def fill_params(net, seed):
    """Overwrite every parameter (sorted by name) from one seeded generator."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, p in sorted(net.named_parameters()):
            fan = p[0].numel() if p.dim() > 1 else p.numel()
            p.copy_((torch.rand(p.shape, generator=g) * 2 - 1) / np.sqrt(max(1, fan)))


def make_batch(n, seed):
    rng = np.random.default_rng(seed)
    s6 = rng.random((n, 6)).astype(np.float32)
    w = rng.integers(0, 2, (n, 3, 15, 15)).astype(np.float32)
    a = rng.integers(0, 4, n).astype(np.int64)
    r = rng.choice(REWARDS, n).astype(np.float64)
    s6n = rng.random((n, 6)).astype(np.float32)
    wn = rng.integers(0, 2, (n, 3, 15, 15)).astype(np.float32)
    return s6, w, a, r, s6n, wn


def param_stats(net, grads=False):
    out = {}
    for name, p in sorted(net.named_parameters()):
        t = p.grad if grads else p.data
        out[name] = (float(t.double().sum()), float(t.double().abs().sum()))
    return out
