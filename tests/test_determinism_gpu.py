"""The live trainer is deterministic: the same seeds give the same
nets, optimizer state, replay rows and counters, run to run — with the overlapped learner's K
updates per vector step as K single-update graph replays (MZ_K_BLOCK=0) and as one K-update graph
per index slot (MZ_K_BLOCK=1), across train() calls. Each run is a fresh process (tests/live_train_digest.py: the stems'
dropout salts follow the nets' construction order)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _run(kblock, steps=600):
    env = dict(os.environ, MZ_K_BLOCK=kblock)
    p = subprocess.run([sys.executable, os.path.join(HERE, "live_train_digest.py"), str(steps)],
                       env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


def test_live_trainer_twice_same_result_and_k_block_equal():
    """Two runs with K single-update replays, two with the K-update graph: all four identical
    (the K-update graph replays the same kernels in the same order). Round 4's K-update graph
    failed this across train() calls: a restart gave the index buffers new storage while the
    captured graphs kept reading the old addresses."""
    a, b = _run("0"), _run("0")
    assert a["n_updates"] == b["n_updates"] and a["n_updates"] > 0
    assert a == b, (a, b)
    c, d = _run("1"), _run("1")
    assert c == d, (c, d)
    assert a == c, (a, c)
