#!/usr/bin/env python3
"""Round 6 debug: two DDQN learners stepped side by side — are they bit-identical (a) both on the
per-forward counters, (b) fold vs per-forward? Prints the first update where weights differ."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402


def run(fold_a, fold_b, eval_mode=False, use_graph=True):
    from mazerl import VectorMazeEnv
    from mazerl.agents.dqn import VectorDQNLearner
    from test_learner_graph import _fill
    env = VectorMazeEnv(4, 21, enrich=True, device="cuda", seed=1)
    mk = lambda: VectorDQNLearner(4, "cuda", variant="ddqn", batch_size=64, capacity=256,  # noqa: E731
                                  updates_per_step=1, target_every=4, updates_per_epoch=2, seed=5,
                                  use_graph=use_graph, overlap=False)
    A, B = mk(), mk()
    for L, fold in ((A, fold_a), (B, fold_b)):
        if not fold:
            for m in (L.source, L.target):
                m._stem_rng = torch.zeros(1, dtype=torch.int64, device="cuda")
                m._stem_advance = "add"
    for ma, mb in ((A.source, B.source), (A.target, B.target)):
        mb._salt = ma._salt
        mb.load_state_dict(ma.state_dict())
    if eval_mode:
        for L in (A, B):
            L.source.eval(); L.target.eval()
    for L in (A, B):
        for k in range(4):
            _fill(L, n=64, seed=k)
    out = []
    for u in range(8):
        la = A.update(env.expand_window, reserve=0)
        lb = B.update(env.expand_window, reserve=0)
        torch.cuda.synchronize()
        same = all(torch.equal(pa, pb) for pa, pb in zip(A.source.parameters(), B.source.parameters()))
        out.append((u, float(la), float(lb), same, int(A.source._stem_rng.item()), int(B.source._stem_rng.item()),
                    int(A.target._stem_rng.item()), int(B.target._stem_rng.item())))
    env.close()
    return out


if __name__ == "__main__":
    for args in ((False, False, False, True), (True, True, False, True), (True, False, False, True),
                 (True, False, True, True), (False, False, False, False), (True, False, False, False)):
        print(args, flush=True)
        for row in run(*args):
            print("   ", row, flush=True)
