#!/usr/bin/env python3
"""Round 5, VERDICT r4 next 7: is the K-update graph nondeterministic in the live trainer? The
round-4 curriculum leg (4,096 x 41x41, DDQN, 4 updates of 1,024 per vector step, overlapped
learner, per-instance change_algorithm, 2,420 vector steps) run by the package at argv[1] (the
round-4 sources + profiles/r04zz/kblock.patch: profiles/r05f/old_mazerl, or the current one),
printing a digest of the nets / optimizer / replay / counters. Two fresh processes per package
are compared by the calling script."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(pkg, steps=2400):
    if pkg == "old":  # the round-4 Python package (old API) against the current libmazerl.so
        import importlib.util
        sys.path.insert(0, os.path.join(ROOT, "profiles", "r05f"))
        spec = importlib.util.spec_from_file_location(
            "mazerl", os.path.join(ROOT, "profiles", "r05f", "old_mazerl", "__init__.py"),
            submodule_search_locations=[os.path.join(ROOT, "profiles", "r05f", "old_mazerl")])
        mod = importlib.util.module_from_spec(spec)
        sys.modules["mazerl"] = mod
        spec.loader.exec_module(mod)
        os.environ.setdefault("MZ_LIB_OVERRIDE", os.path.join(
            ROOT, "maze-solving-agent-gymnasium_amd", "mazerl", "_lib", "libmazerl.so"))
        curriculum = True
    else:
        sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))
        curriculum = "per-instance"
    import torch
    from mazerl import VectorMazeEnv
    from mazerl.agents.dqn import VectorDQNLearner
    from mazerl.trainers.vector_trainer import VectorOffPolicyTrainer
    dev = torch.device("cuda", 0)
    B, dim = 4096, 41
    env = VectorMazeEnv(B, dim, enrich=True, device=dev, algorithm="r-prim", seed=0xC0CC0000,
                        done_list=False, window=False, window_bits=True)
    L = VectorDQNLearner(B, dev, variant="ddqn", lr=1e-3, eps_start=0.95, eps_final=0.1,
                         eps_decay=((dim - 1) ** 2 // 2) * 5, gamma=0.7, batch_size=1024,
                         capacity=2_000_000, updates_per_step=4, target_every=13, overlap=True,
                         greedy_rows=True, acting="x3", seed=1)
    tr = VectorOffPolicyTrainer(env, L, seed=11, curriculum=curriculum)
    tr.train(20)
    trail = []  # source-net digest every 100 vector steps: where two runs part
    for k in range(0, int(steps), 100):
        tr.train(min(100, int(steps) - k))
        torch.cuda.synchronize()
        trail.append(hashlib.sha256(L.source._flat_params.detach().cpu().numpy().tobytes()).hexdigest()[:6])
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for t in (L.source._flat_params, L.target._flat_params, L.opt.exp_avg, L.opt.exp_avg_sq,
              L.steps_done, L.replay.sw[:L.replay.size], L.replay.r[:L.replay.size]):
        h.update(t.detach().cpu().numpy().tobytes())
    print(json.dumps({"pkg": pkg, "k_block": os.environ.get("MZ_K_BLOCK"), "digest": h.hexdigest()[:16],
                      "wins": int(tr.wins), "episodes": int(tr.episodes), "n_updates": L.n_updates,
                      "trail": trail}),
          flush=True)
    env.close()


if __name__ == "__main__":
    main(sys.argv[1], *[int(x) for x in sys.argv[2:]])
