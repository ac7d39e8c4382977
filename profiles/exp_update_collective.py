#!/usr/bin/env python3
"""Round 5: what the gradient collective adds to a DDQN update, one rank over
RCCL ("nccl" backend) on cuda:0 — the learner of the bench's win-rate leg (batch 1,024, captured
graphs, sequential schedule), timed with HIP events over 200 updates after 20 warm-up updates:
  none       no process group collective (one graph: backward + clamp + AdamW)
  allreduce  graph A (backward), the 8.56 MB all-reduce, graph B (clamp + AdamW)
  sharded    graph A, reduce-scatter, graph B over the rank's shard, all-gather
  sharded_ingraph / allreduce_ingraph  the same collectives captured inside ONE update graph
             (graph_collectives=True, round 6)
With one rank the collectives are local copies: the numbers bound the cost of the split graphs
and the collective launches, not the xGMI transfer (the driver's 8-GPU runs). One JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    from mazerl import VectorMazeEnv
    from mazerl.agents.dqn import VectorDQNLearner
    from mazerl.distributed import GradAllReduce
    from test_learner_graph import _fill
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("MZ_PORT", "29561"),
                      RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="env://", device_id=torch.device("cuda", 0))
    env = VectorMazeEnv(4, 21, enrich=True, device="cuda", seed=1)
    rec = {}
    modes = ("none", "allreduce", "sharded", "allreduce_ingraph", "sharded_ingraph")
    for mode in modes + modes:
        ar = None if mode == "none" else GradAllReduce(shard=mode.startswith("sharded"))
        L = VectorDQNLearner(4, "cuda", variant="ddqn", batch_size=1024, capacity=8192,
                             updates_per_step=1, target_every=13, seed=5, use_graph=True,
                             overlap=False, allreduce=ar, graph_collectives=mode.endswith("ingraph"))
        for k in range(8):
            _fill(L, n=1024, seed=k)
        for _ in range(20):
            L.update(env.expand_window)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(200):
            L.update(env.expand_window)
        e1.record()
        torch.cuda.synchronize()
        rec.setdefault(mode, []).append(round(e0.elapsed_time(e1) / 200 * 1000, 1))
        if ar is not None:
            rec[mode + "_is_sharded"] = ar.sharded
        del L
    rec["unit"] = "us per update (HIP events, 200 updates)"
    print(json.dumps(rec), flush=True)
    env.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
