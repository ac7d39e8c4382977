#!/usr/bin/env python3
"""Headline benchmark: env steps/sec on 40x40-cell (81x81 grid) r-prim mazes (BASELINE.json).

One "step" = one vector step of the hot path over every instance on the GPU, ONE launch:
  k_step with the fused reference masked-exploration act (dqn_agent.py:104-116) +
     BaseMazeEnv.step + Enrich obs (reward, terminated/truncated, obs6, f32 3x15x15 window),
     with autoreset: instances whose previous step ended are reset in the same launch
     (BaseMazeEnv.reset, base_maze_env.py:136-161 — the trainer's env.reset() after an episode)
Workload: configs[2] of BASELINE.json — 65,536 instances of 81x81-grid r-prim mazes per GPU,
generated on the GPU before the timed region (generation is reported separately).
Multi-GPU: one process per GPU (torchrun), independent env shards (no data-path collective),
weak scaling; value = all ranks' env steps / max-over-ranks wall time.

Extra JSON fields: roofline of k_step (one HIP event pair on the launch stream around the whole
timed region — one k_step launch per step, so elapsed / steps is its average launch duration
including the back-to-back launch gap; a pair around every launch would drain the queue each
time and add ~3 us), cpu_baseline (the CPU oracle in reference-cost mode, A* per
find_path, timed on host cores — rank 0, N=1 only).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))

# Algorithmic bytes per instance-step of k_step: 66 B compact state/outputs
# + 2,955 B for the Enrich window (2,700 B f32 window write + 225 B visit plane + 30 B wall rows)
ALG_BYTES_PER_STEP = 3021
# the same step in the mode the trainers run (window_bits=True, window=False): the 675-bit
# window written as 88 B of bits instead of 2,700 B of f32 — 3,021 - 2,700 + 88
ALG_BYTES_PER_STEP_BITS = 409
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# the sources k_step is built from: the PMC traffic file is only used when it was taken from them
KSTEP_SOURCES = ("mz_env.hip", "mz_common.h", "mz_kernels.h", "mz_build.inc.h")


def kstep_source_sha():
    import hashlib
    h = hashlib.sha256()
    for f in KSTEP_SOURCES:
        with open(os.path.join(ROOT, "maze-solving-agent-gymnasium_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def pmc_traffic(mode, envs, dim):
    """HBM bytes per k_step launch from profiles/pmc_k_step.json (separate rocprofv3 --pmc
    passes, profiles/collect.sh) — None unless taken from the current k_step sources at this
    config."""
    pmc = os.path.join(ROOT, "profiles", "pmc_k_step.json")
    if not os.path.exists(pmc):
        return None, "no PMC file"
    with open(pmc) as f:
        p = json.load(f)
    rec = p.get(mode)
    if not rec or rec.get("envs") != envs or rec.get("dim") != dim:
        return None, f"no PMC record for {mode} mode at {envs} x {dim}"
    if rec.get("source_sha") != kstep_source_sha():
        return None, "PMC record is stale: k_step's sources changed since it was taken"
    return rec.get("hbm_bytes_per_launch"), (f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes "
                                              f"({rec.get('tag')}), k_step sources {rec['source_sha']}")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--envs", type=int, default=65536, help="instances per GPU")
    ap.add_argument("--dim", type=int, default=81)
    ap.add_argument("--algo", default="r-prim")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="cpu_baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--legs", default="window,bits",
                    help="env-step legs: window (f32 Enrich window, the headline) and bits (the "
                         "trainers' mode: 88-B window bits)")
    # 2,400 vector steps (157 M env steps, ~4 s): greedy win-rate 94.4 / 95.4 / 96.5 / 96.1 /
    # 95.9 % after 600 / 1,200 / 2,400 / 4,800 / 9,600 (one run each) — the plateau
    ap.add_argument("--train-steps", type=int, default=2400,
                    help="DDQN vector steps for the win-rate half of the metric (0 = skip)")
    ap.add_argument("--eval-mazes", type=int, default=1000)
    ap.add_argument("--candidates", type=int, default=6,
                    help="mazes the trainers train on: each the easiest of C candidates by McClendon "
                         "difficulty (the reference env's generate_maze, base_maze_env.py:78-97) — "
                         "the initial mazes and the maze bank's replacements for winners; 1 = one "
                         "Philox maze each")
    ap.add_argument("--curriculum-envs", type=int, default=4096)
    ap.add_argument("--curriculum-dim", type=int, default=41)
    ap.add_argument("--curriculum-updates", type=int, default=4)
    ap.add_argument("--curriculum-batch", type=int, default=1024)
    ap.add_argument("--curriculum-steps", type=int, default=2400,
                    help="DDQN vector steps of the curriculum leg (the reference's change_algorithm "
                         "training, evaluated under its test(new=True) protocol; 0 = skip)")
    # the curriculum legs' exploration: epsilon_decay = the reference's ((N-1)^2 // 2) * 5 / 40, the
    # reading the win-rate and config legs use (B instances feed one learner: at the reference's
    # decay, 4,000 at 41 x 41, x12 after the global rule's first vector steps, epsilon stays near
    # 0.9 for the whole leg — 18 wins in 2,420 vector steps, profiles/r06l; / 40: 4,104 wins,
    # profiles/r06m). --curriculum-decay-div 1 = the reference's decay.
    ap.add_argument("--curriculum-decay-div", type=float, default=40.0,
                    help="the curriculum legs' epsilon_decay = the reference's ((N-1)^2 // 2) * 5 / this")
    # the per-instance rule's leg: each instance is a trainer of its own (its own wins,
    # epsilon_decay and steps_done), so it needs the reference's per-agent cadence: an instance
    # reaches dfs only after 5 prim&kill wins of its own. 1,024 instances x 60,000 vector steps:
    # median 15 wins, 982 of 1,024 instances at dfs at the end (2,048 x 40,000: median 9, 705 at
    # dfs; 512 x 16,000: median 7, none past prim&kill — profiles/r06m/)
    ap.add_argument("--curriculum-pi-envs", type=int, default=1024)
    ap.add_argument("--curriculum-pi-steps", type=int, default=60000)
    ap.add_argument("--curriculum-pi-updates", type=int, default=2)
    ap.add_argument("--curriculum-rules", default="global,per-instance",
                    help="change_algorithm over the learner's wins (global: the reference's one "
                         "agent and class-wide ALGORITHM) and / or per instance (mazerl/trainers/"
                         "schedule.py); one curriculum leg each, the first is curriculum_leg")
    # learner: one update of 1,024 per vector step. Sweep at 2,400 vector steps (training env
    # steps/s, greedy win-rate): 256: 58.0 M, 96.0 % / 512: 54.4 M, 95.0-96.0 % / 1,024: 50.6-
    # 50.8 M, 96.2-96.4 % / 2,048: 40.4 M, 96.5 % / 4,096: 30.4 M, 96.2 % — the win-rate is on its
    # plateau from 1,024 up, the GEMMs are not
    ap.add_argument("--batch", type=int, default=1024, help="learner minibatch (win-rate leg)")
    ap.add_argument("--updates-per-step", type=int, default=1)
    ap.add_argument("--target-every", type=int, default=13, help="target sync every N updates")
    ap.add_argument("--greedy-rows", type=int, default=1,
                    help="1: the acting forward runs over the instances whose epsilon draw says "
                         "greedy only (dqn_agent.py:104-116); 0: over every instance")
    ap.add_argument("--fused-bookkeeping", type=int, default=1,
                    help="1: per-step trainer bookkeeping + replay push as HIP launches "
                         "(mz_trainer_tick, mz_replay_push); 0: torch ops")
    ap.add_argument("--acting", default="x3", choices=["x3", "bf16"],
                    help="acting head: x3 = f32-accurate bf16x3 MFMA (QAct, sized on the device); "
                         "bf16 = bf16 stem + hipBLASLt bf16 GEMMs (FusedQ, count read on the host)")
    ap.add_argument("--overlap", type=int, default=1,
                    help="1: learner updates on a side HIP stream, overlapped with acting + env "
                         "step (acting weights one update behind); 0: sequential")
    ap.add_argument("--graph", type=int, default=1,
                    help="1: the timed env steps replay captured HIP graphs of k_step launches "
                         "(the Python launch loop is timed beside them); 0: eager launches")
    # N > 1: the DQN / DDQN learners' reduce-scatter / all-gather captured inside the update graph
    # (one replay per update; one RCCL rank: 357 vs 382 us per update, no collective 357,
    # profiles/r06k/) instead of issued between two replays. Off by default: RCCL refuses two
    # ranks on one GPU, so the captured path is verified at one rank only (tests/
    # test_gpu_distributed.py) and the driver's multi-GPU runs keep the two-graph path
    ap.add_argument("--graph-collectives", type=int, default=0)
    ap.add_argument("--graph-chunk", type=int, default=100, help="k_step launches per graph")
    ap.add_argument("--cfg1-episodes", type=int, default=350,
                    help="config 1: tabular Q-learning episodes (training_examples/.../test_q.py)")
    ap.add_argument("--config-legs", default="cfg1,cfg2,cfg4,cfg5",
                    help="BASELINE configs 2 (DQN, 15x15), 4 (DDQN, mixed 81x81) and 5 (PPO, "
                         "toroidal 9->40 cells) at this N, whole-node env steps/s + win-rates "
                         "('' = skip)")
    ap.add_argument("--cfg2-envs", type=int, default=4096, help="config 2 instances per GPU")
    ap.add_argument("--cfg2-steps", type=int, default=800)
    ap.add_argument("--cfg5-modes", default="growth,fixed",
                    help="config 5 legs: growth = ToroidalVariableMazeEnv's +4 growth per win from "
                         "17 (9 cells) to 79 (40 cells); fixed = instance i of size 17 + 2 (i mod 32)")
    ap.add_argument("--cfg4-envs", type=int, default=8192, help="config 4 instances per GPU")
    ap.add_argument("--cfg5-envs", type=int, default=4096, help="config 5 instances per GPU")
    # ~30,000 vector steps (246 M env steps): long enough that the learner wins dfs / prim&kill
    # episodes too (VERDICT r5 missing 2; 600 steps: only r-prim wins)
    ap.add_argument("--cfg4-steps", type=int, default=30000)
    ap.add_argument("--cfg5-steps", type=int, default=3000)
    # the growth leg trained longer: the instances' sizes at 600 / 3,000 / 8,000 vector steps reach
    # 37 / 53 / 61 of 79, greedy 40 / 70 / 75 % (profiles/r06n/); 0 = --cfg5-steps
    ap.add_argument("--cfg5-growth-steps", type=int, default=8000)
    ap.add_argument("--cfg-eval-mazes", type=int, default=500)
    ap.add_argument("--launch-timeout", type=float, default=2400.0,
                    help="--gpus N > 1 without torchrun: seconds before the ranks are killed")
    return ap.parse_args(argv)


def win_rate(a, dev, rank=0, world=1):
    """Second half of the metric: train DDQN (reference DDQN net/loss, vectorised) on the same
    config, then win-rates on `eval_mazes` fresh mazes (never seen in training), rank 0:
      greedy / eps_0.1            r-prim mazes as generated, epsilon 0 and a fixed 0.1 (SURVEY
                                  Q14's reading of the final epsilon);
      *_best_of_6                 r-prim mazes, each the easiest of 6 candidates by McClendon
                                  difficulty (the reference env's selection, base_maze_env.py:
                                  78-97);
      new_mazes_reference_protocol  NeuralOffPolicyTrainer.test(num, new=True) (off_policy_trainer
                                  .py:228-263): per maze random.choice(r-prim, prim&kill, dfs) and a
                                  best-of-6 maze of that algorithm; acting greedy, and through
                                  get_action with epsilon from steps_done carried over from
                                  training (dqn_agent.py:104-119) — the protocol of the README's
                                  99.6 % "new mazes" figure (its 41x41, 125 training episodes).
    With N ranks every rank trains on its own env shard and the source-net gradients are averaged
    over RCCL once per update (mazerl/distributed.py: one 8.56 MB bucket)."""
    import torch
    import torch.distributed as dist
    from mazerl import VectorMazeEnv
    from mazerl.agents.dqn import VectorDQNLearner
    from mazerl.distributed import GradAllReduce, broadcast_params
    from mazerl.trainers.vector_trainer import VectorOffPolicyTrainer, best_of_mazes, evaluate
    t_gen = time.perf_counter()
    env = VectorMazeEnv(a.envs, a.dim, enrich=True, device=dev, algorithm=a.algo,
                        seed=0xA11CE + rank * a.envs, done_list=False, window=False,
                        window_bits=True, candidates=a.candidates)  # acting reads the bits
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t_gen
    decay = ((a.dim - 1) * (a.dim - 1) // 2) * 5 / 40.0
    L = VectorDQNLearner(a.envs, dev, variant="ddqn", lr=1e-3, eps_start=0.95, eps_final=0.1,
                         eps_decay=decay, gamma=0.7, batch_size=a.batch, capacity=2_000_000,
                         updates_per_step=a.updates_per_step, target_every=a.target_every,
                         allreduce=GradAllReduce() if world > 1 else None,
                         graph_collectives=bool(a.graph_collectives), overlap=bool(a.overlap),
                         greedy_rows=bool(a.greedy_rows), acting=a.acting)
    if world > 1:
        broadcast_params(L.source)
        L.target.load_state_dict(L.source.state_dict())
    tr = VectorOffPolicyTrainer(env, L, seed=3 + 7919 * rank, fused=bool(a.fused_bookkeeping),
                                bank_candidates=a.candidates)
    tr.train(20)  # warm-up: MIOpen / hipBLASLt first calls
    if world > 1:
        dist.barrier()
    w0, e0 = int(tr.wins), int(tr.episodes)
    secs = tr.train(a.train_steps, **progress(rank, "win-rate leg"))
    if world > 1:
        t = torch.tensor([secs], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        secs = float(t.item())
    train_wins, train_eps = int(tr.wins) - w0, int(tr.episodes) - e0
    sel = env.select_stats()
    snap = seen_snapshot(env, a.eval_mazes) if rank == 0 else None
    env.close()
    if rank != 0:
        return None
    log("win-rate evaluation")
    agree = acting_agreement(L)
    n = a.eval_mazes
    g, _ = evaluate(L, n, a.dim, a.algo, seed=0x7E570000, eps=0.0, device=dev)
    e, _ = evaluate(L, n, a.dim, a.algo, seed=0x7E570000, eps=0.1, device=dev)
    t6 = time.perf_counter()
    mz6 = best_of_mazes(n, a.dim, a.algo, seed=0x7E580000, device=dev)
    t6 = time.perf_counter() - t6  # 6 x eval_mazes candidates generated + McClendon on the GPU
    g6, _ = evaluate(L, n, a.dim, a.algo, seed=0x7E580000, eps=0.0, device=dev, mazes=mz6)
    e6, _ = evaluate(L, n, a.dim, a.algo, seed=0x7E580000, eps=0.1, device=dev, mazes=mz6)
    proto = reference_protocol(L, n, a.dim, dev, 0x7E590000)
    proto["training"] = "r-prim only (BASELINE configs[2])"
    seen = seen_protocol(L, snap, dev, 0x7E5E0000)
    infer = infer_protocol(L, 100, a.dim, dev, 0x7E610000)
    return {"greedy": g, "eps_0.1": e, "greedy_best_of_6": g6, "eps_0.1_best_of_6": e6,
            "seen_mazes_reference_protocol": seen,
            "infer_by_algorithm": infer,
            "new_mazes_reference_protocol": dict(proto, note=(
                "test(num, new=True): per maze random.choice(ALGOS) + best-of-6 by McClendon "
                "difficulty; eps_from_steps_done acts through get_action's epsilon with each maze "
                "continuing a training instance's steps_done (episodes side by side here, one "
                "after another in the reference); the reference's 99.6 % was measured at 41x41 "
                "after 125 single-env episodes with its change_algorithm curriculum (README.md); "
                "see curriculum_leg for the curriculum-trained learner")),
            "eval_mazes": n, "variant": "ddqn",
            "training_mazes": {
                "candidates": a.candidates,
                "selection": ("each the easiest of %d by McClendon difficulty, chosen on the GPU "
                              "(initial mazes: mz_generate_best; winners' new mazes: the maze "
                              "bank's best-of-C refills on the side stream)" % a.candidates)
                             if a.candidates > 1 else "one Philox maze each (no selection)",
                "initial_generation_seconds": round(t_gen, 3),
                "selection_stats": sel,
                "wins_per_vector_step": train_wins / max(1, a.train_steps),
                "episodes_per_vector_step": train_eps / max(1, a.train_steps)},
            "ranks": world, "train_vector_steps": a.train_steps + 20,
            "train_seconds_steady": round(secs, 3),
            "train_env_steps_per_s": a.envs * a.train_steps * world / secs,
            "updates": L.n_updates, "batch": a.batch, "updates_per_vector_step": a.updates_per_step,
            "learner_schedule": "side stream, overlapped (acting weights one update behind)"
                                if L.overlap else "sequential",
            "acting_rows": "greedy rows only (epsilon draw first, dqn_agent.py:104-116)"
                           if L.greedy_rows else "every instance",
            "acting_head": a.acting,
            "grad_allreduce": (f"{dist.get_backend()} ({'RCCL' if dist.get_backend() == 'nccl' else 'rehearsal'}), "
                               "one 8.56 MB fp32 bucket per update, reduce-scatter + all-gather "
                               + ("captured inside the update graph" if L.graph_collectives
                                  else "between two graph replays"))
                              if world > 1 else None,
            "acting_argmax_agreement": agree,
            "best_of_6_selection_seconds": round(t6, 3),
            "note": "greedy / eps_0.1: fresh r-prim mazes as generated; *_best_of_6: each r-prim "
                    "maze the easiest of 6 candidates by McClendon difficulty, as the reference's "
                    "env selects new mazes (base_maze_env.py:78-97); new_mazes_reference_protocol: "
                    "the reference's test(new=True) protocol (mixed algorithms, epsilon from "
                    "steps_done)"}


def curriculum_leg(a, dev, rank=0, world=1, rule="global"):
    """The reference's own protocol for its "new mazes" number (README: 99.6 % for DDQN at 41x41):
    DDQN trained with NeuralOffPolicyTrainer.change_algorithm (off_policy_trainer.py:302-310, per
    instance here: prim&kill mazes from an instance's 5th win, dfs from its 10th, epsilon_decay
    x3 / x4) at the reference example's 41x41 grid (training_examples/euclidean_mazes/
    costant_sizes/test_ddqn.py:20-27; its epsilon_decay ((N-1)^2 // 2) * 5), then test(new=True)'s
    protocol (reference_protocol). The reference trains one update of 128 per env step; here
    --curriculum-envs instances with --curriculum-updates updates of --curriculum-batch per
    vector step (default 4,096 x 4 x 1,024: one sample per env step). With N ranks every rank
    trains its shard with the gradient all-reduce."""
    import torch
    import torch.distributed as dist
    from mazerl import VectorMazeEnv
    from mazerl.agents.dqn import VectorDQNLearner
    from mazerl.distributed import GradAllReduce, broadcast_params
    from mazerl.trainers.vector_trainer import VectorOffPolicyTrainer
    B, dim = a.curriculum_envs, a.curriculum_dim
    steps, updates = a.curriculum_steps, a.curriculum_updates
    if rule == "per-instance":
        B, steps, updates = a.curriculum_pi_envs, a.curriculum_pi_steps, a.curriculum_pi_updates
    env = VectorMazeEnv(B, dim, enrich=True, device=dev, algorithm="r-prim",
                        seed=0xC0CC0000 + rank * B, done_list=False, window=False,
                        window_bits=True, candidates=a.candidates)
    decay = ((dim - 1) * (dim - 1) // 2) * 5 / a.curriculum_decay_div
    L = VectorDQNLearner(B, dev, variant="ddqn", lr=1e-3, eps_start=0.95, eps_final=0.1,
                         eps_decay=decay, gamma=0.7, batch_size=a.curriculum_batch,
                         capacity=2_000_000, updates_per_step=updates,
                         target_every=a.target_every,
                         allreduce=GradAllReduce() if world > 1 else None,
                         graph_collectives=bool(a.graph_collectives), overlap=bool(a.overlap),
                         greedy_rows=bool(a.greedy_rows), acting=a.acting, seed=1)
    if world > 1:
        broadcast_params(L.source)
        L.target.load_state_dict(L.source.state_dict())
    tr = VectorOffPolicyTrainer(env, L, seed=11 + 7919 * rank, curriculum=rule,
                                bank_candidates=a.candidates)
    tr.train(20)
    if world > 1:
        dist.barrier()
    secs = tr.train(steps, **progress(rank, f"curriculum leg ({rule})"))
    if world > 1:
        t = torch.tensor([secs], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        secs = float(t.item())
    summary = tr.schedule.summary()  # (rank 0's shard)
    snap = seen_snapshot(env, a.eval_mazes) if rank == 0 else None
    maze_algo = tr.schedule.maze_algo.cpu().numpy() if rank == 0 else None
    env.close()
    if rank != 0:
        return None
    log("curriculum-leg evaluation")
    out = reference_protocol(L, a.eval_mazes, dim, dev, 0x7E5D0000)
    out["seen_mazes_reference_protocol"] = seen_protocol(L, snap, dev, 0x7E5F0000,
                                                         algos=maze_algo[snap[0]])
    out["infer_by_algorithm"] = infer_protocol(L, 100, dim, dev, 0x7E630000)
    out.update({"training": ("change_algorithm curriculum (r-prim -> prim&kill at the 5th win -> dfs "
                             "at the 10th; %s rule: %s)" % (rule, (
                                 "the learner's wins over all instances in instance order, the "
                                 "algorithm class-wide as the reference's ALGORITHM, epsilon_decay "
                                 "x3 / x4 for every instance"
                                 if rule == "global" else "each instance's own wins and "
                                 "epsilon_decay"))),
                "grid": dim, "envs_per_gpu": B, "epsilon_decay": decay,
                "epsilon_decay_reference": ((dim - 1) * (dim - 1) // 2) * 5,
                "epsilon_decay_at_end": float(L.eps_decay) if not torch.is_tensor(L.eps_decay)
                or L.eps_decay.dim() == 0 else float(L.eps_decay.float().mean()),
                "updates_per_vector_step": updates, "batch": a.curriculum_batch,
                "training_mazes_candidates": a.candidates,
                "train_vector_steps": steps + 20,
                "train_env_steps_per_s": B * steps * world / secs,
                "wins_per_instance_median": summary.get("wins_per_instance_median"),
                "total_wins": summary["total_wins"],
                "instances_per_algorithm_at_end": summary["instances_per_algorithm"],
                "new_mazes_per_algorithm": summary["new_mazes_per_algorithm"],
                "eval_mazes": a.eval_mazes})
    return out


def config_legs(a, dev, rank=0, world=1):
    """BASELINE configs 2, 4 and 5 at the bench's N (per rank the share of each config: 4,096,
    8,192 and 4,096 instances), each trained for a fixed number of vector steps between a barrier
    + synchronize on each side, whole-node env steps/s = all ranks' env steps / the max-over-ranks
    time, training mazes best-of---candidates (the reference env's selection); rank 0 evaluates:
      cfg2  DQN on 4,096 r-prim 15x15 mazes per rank (the window is the whole maze), one update of
            2,048 per vector step; greedy win-rate on fresh r-prim mazes as generated and best-of-6;
      cfg4  DDQN on 8,192 mixed dfs / r-prim / prim&kill 81x81 mazes per rank (algo = global
            instance id mod 3), 4 updates of 512 per vector step, source-net gradients
            all-reduced over RCCL per update; win-rates under the reference's test(new=True)
            protocol (mixed algorithms, best-of-6, greedy and epsilon from steps_done);
      cfg5  PPO on 4,096 toroidal mazes per rank, gradients all-reduced per minibatch; mode
            "growth": every instance starts at 17 x 17 (9 cells) and grows +4 per win up to 79
            (40 cells) as ToroidalVariableMazeEnv.update_maze (toroidal_variable_maze_env.py:113-131,
            with the max-shape stop); mode "fixed": instance i of size 17 + 2 (i mod 32); greedy
            win-rate on fresh mazes of sizes 17..79 as generated and best-of-6
            (toroidal_maze_env.py:40-54: difficulty of the bordered maze)."""
    import torch
    import torch.distributed as dist
    from mazerl import VectorMazeEnv
    from mazerl.agents.dqn import VectorDQNLearner
    from mazerl.distributed import GradAllReduce, broadcast_params
    from mazerl.trainers.ppo_trainer import VectorPPOTrainer
    from mazerl.trainers.vector_trainer import (VectorOffPolicyTrainer, best_of_mazes, evaluate,
                                                make_env)

    def timed_train(tr, steps, name):
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        secs = tr.train(steps, **progress(rank, name))
        if world > 1:
            dist.barrier()
            t = torch.tensor([secs], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            secs = float(t.item())
        return secs

    out = {}
    legs = [x for x in a.config_legs.split(",") if x]
    C = a.candidates
    if "cfg1" in legs and rank == 0:
        # config 1 (plumbing, one env instance, no collective: rank 0 only): the reference's
        # tabular example (training_examples/euclidean_mazes/costant_sizes/test_q.py: QAgent lr
        # 1e-3, epsilon 0.95 -> 0.05 with decay N*N // 2, gamma 0.7, eta 1e-2, 350 episodes,
        # then test(len(env.mazes), new=False) and test(250, new=True)) on BASELINE's 9 x 9
        # SimpleMazeEnv — the drop-in env (one instance on the GPU handle, a launch + a sync per
        # step) and QAgent, driven by mazerl.trainers.tabular (OffPolicyTrainer)
        import random as _random
        import numpy as _np
        from mazerl.agents.q_agent import QAgent
        from mazerl.envs import SimpleMazeEnv
        from mazerl.trainers.tabular import TabularTrainer
        log("config 1 leg (tabular Q-learning, one 9x9 env)")
        _random.seed(0xC0F1)
        _np.random.seed(0xC0F1)
        n1 = 9
        env1 = SimpleMazeEnv((n1, n1), device=dev)
        agent = QAgent(env1, learning_rate=1e-3, initial_epsilon=0.95, final_epsilon=0.05,
                       epsilon_decay=n1 * n1 // 2, discount_factor=0.7, eta=1e-2)
        trn = TabularTrainer(env1, agent)
        wins, steps1, secs1 = trn.train(a.cfg1_episodes)
        n_seen = len(env1.mazes)
        t1 = time.perf_counter()
        seen_rate = trn.test(n_seen, new=False)
        new_rate = trn.test(250, new=True)
        out["cfg1"] = {"grid": n1, "algo": "r-prim", "agent": "QAgent (tabular)", "envs": 1,
                       "episodes": a.cfg1_episodes, "train_wins": wins, "train_env_steps": steps1,
                       "train_seconds": round(secs1, 3),
                       "env_steps_per_s": steps1 / secs1 if secs1 > 0 else None,
                       "seen_mazes": n_seen, "win_rate_seen": seen_rate,
                       "win_rate_new": new_rate, "test_seconds": round(time.perf_counter() - t1, 3),
                       "q_table_states": len(agent.q_values),
                       "reference_readme": "Q-learning 80.49 % seen / 0 % new (README.md:66; "
                                           "its test_q.py runs 21 x 21)",
                       "note": "one env instance: every step is a kernel launch and a stream "
                               "synchronisation (the single-env drop-in path), not the vectorised "
                               "engine"}
        env1.close()
    if "cfg2" in legs:
        if rank == 0:
            log("config 2 leg (DQN, 15x15)")
        B, dim = a.cfg2_envs, 15
        env = VectorMazeEnv(B, dim, enrich=True, device=dev, algorithm="r-prim",
                            seed=0x5EED0000 + rank * B, done_list=False, window=False,
                            window_bits=True, candidates=C)
        decay = ((dim - 1) * (dim - 1) // 2) * 5 / 40.0
        L = VectorDQNLearner(B, dev, variant="dqn", lr=1e-3, eps_start=0.95, eps_final=0.1,
                             eps_decay=decay, gamma=0.7, batch_size=2048, updates_per_step=1,
                             capacity=2_000_000, target_every=13,
                             allreduce=GradAllReduce() if world > 1 else None,
                         graph_collectives=bool(a.graph_collectives), overlap=True, seed=0)
        if world > 1:
            broadcast_params(L.source)
            L.target.load_state_dict(L.source.state_dict())
        tr = VectorOffPolicyTrainer(env, L, seed=7919 * rank + 2, bank_candidates=C)
        tr.train(20)
        secs = timed_train(tr, a.cfg2_steps, "config 2 leg")
        snap = seen_snapshot(env, a.cfg_eval_mazes) if rank == 0 else None
        rec = {"envs_per_gpu": B, "grid": dim, "algo": "r-prim", "variant": "dqn",
               "vector_steps": a.cfg2_steps, "seconds": round(secs, 3),
               "env_steps_per_s": B * a.cfg2_steps * world / secs, "updates": L.n_updates,
               "batch": 2048, "updates_per_vector_step": 1, "training_mazes_candidates": C,
               "grad_allreduce": (dist.get_backend() if world > 1 else None)}
        env.close()
        if rank == 0:
            n = a.cfg_eval_mazes
            rec["win_rate_greedy"], _ = evaluate(L, n, dim, "r-prim", seed=0x7E520000, eps=0.0,
                                                 device=dev)
            mz = best_of_mazes(n, dim, "r-prim", seed=0x7E530000, device=dev)
            rec["win_rate_greedy_best_of_6"], _ = evaluate(L, n, dim, "r-prim", seed=0x7E530000,
                                                           eps=0.0, device=dev, mazes=mz)
            rec["seen_mazes_reference_protocol"] = seen_protocol(L, snap, dev, 0x7E540000)
            rec["eval_mazes"] = n
        out["cfg2"] = rec
        del tr, L
    if "cfg4" in legs:
        if rank == 0:
            log("config 4 leg (DDQN, mixed 81x81)")
        B, dim = a.cfg4_envs, 81
        algo = ((torch.arange(B) + rank * B) % 3).to(torch.uint8)
        env = VectorMazeEnv(B, dim, enrich=True, device=dev, algorithm=algo,
                            seed=0x5EED0000 + rank * B, done_list=False, window=False, window_bits=True,
                            candidates=C)
        env.set_algorithm(algo)
        decay = ((dim - 1) * (dim - 1) // 2) * 5 / 40.0
        # 4 updates of 512 per vector step: at 8,192 instances one update of 2,048 (the same
        # samples) did not learn in 600 vector steps (0 wins vs 92.3 % greedy,
        # profiles/r04f_cfg4.jsonl)
        L = VectorDQNLearner(B, dev, variant="ddqn", lr=1e-3, eps_start=0.95, eps_final=0.1,
                             eps_decay=decay, gamma=0.7, batch_size=512, updates_per_step=4,
                             capacity=2_000_000, target_every=13,
                             allreduce=GradAllReduce() if world > 1 else None,
                         graph_collectives=bool(a.graph_collectives), overlap=True, seed=0)
        if world > 1:
            broadcast_params(L.source)
            L.target.load_state_dict(L.source.state_dict())
        tr = VectorOffPolicyTrainer(env, L, seed=7919 * rank, bank_candidates=C, track_wins=True)
        tr.train(20)
        w0 = tr.inst_wins.clone()
        secs = timed_train(tr, a.cfg4_steps, "config 4 leg")
        # the training distribution per algorithm: wins in the timed steps
        dw = (tr.inst_wins - w0).long().cpu()
        snap = seen_snapshot(env, a.cfg_eval_mazes) if rank == 0 else None
        names = ["r-prim", "dfs", "prim&kill"]  # ids: vector_env.ALGOS
        wins_by = {names[k]: int(dw[algo == k].sum()) for k in range(3)}
        if world > 1:
            t = torch.tensor([wins_by[n] for n in names], dtype=torch.int64, device=dev)
            dist.all_reduce(t)
            wins_by = dict(zip(names, t.tolist()))
        env.close()
        rec = {"envs_per_gpu": B, "grid": dim, "algo": "mixed (global id mod 3)",
               "train_wins_by_algorithm": wins_by,
               "vector_steps": a.cfg4_steps, "seconds": round(secs, 3),
               "env_steps_per_s": B * a.cfg4_steps * world / secs, "updates": L.n_updates,
               "batch": 512, "updates_per_vector_step": 4, "training_mazes_candidates": C,
               "grad_allreduce": (dist.get_backend() if world > 1 else None)}
        if rank == 0:
            rec["win_rate_reference_protocol"] = reference_protocol(L, a.cfg_eval_mazes, dim, dev,
                                                                    0x7E5A0000)
            rec["seen_mazes_reference_protocol"] = seen_protocol(
                L, snap, dev, 0x7E5A8000, algos=algo.numpy()[snap[0]])
            rec["infer_by_algorithm"] = infer_protocol(L, 100, dim, dev, 0x7E620000)
            rec["eval_mazes"] = a.cfg_eval_mazes
        out["cfg4"] = rec
        del tr, L
    if "cfg5" in legs:
        dims = list(range(17, 80, 2))
        for mode in [m for m in a.cfg5_modes.split(",") if m]:
            if rank == 0:
                log(f"config 5 leg (PPO, toroidal 17..79, {mode})")
            B = a.cfg5_envs
            growth = (17, 79) if mode == "growth" else None
            env = make_env(B, [17] if growth else dims, toroidal=True, algorithm="r-prim",
                           seed=0x5EED0000 + rank * B, device=dev, done_list=False, reward64=True,
                           window=False, window_bits=True, candidates=C, max_dim=79)
            tr = VectorPPOTrainer(env, dev, gamma=0.9, batch_size=2048, ppo_steps=2,
                                  pool_size=32768, seed=7919 * rank, growth=growth,
                                  bank_candidates=C,
                                  allreduce=GradAllReduce() if world > 1 else None)
            if world > 1:
                broadcast_params(tr.net)
            tr.train(20)
            n5 = a.cfg5_growth_steps if mode == "growth" and a.cfg5_growth_steps > 0 else a.cfg5_steps
            secs = timed_train(tr, n5, f"config 5 leg ({mode})")
            ran = tr.stopped_at or n5  # (the growth leg's max-shape stop may come first)
            rec = {"mode": mode, "envs_per_gpu": B, "dims": [dims[0], dims[-1]], "toroidal": True,
                   "vector_steps": ran, "seconds": round(secs, 3),
                   "env_steps_per_s": B * ran * world / secs, "updates": tr.updates,
                   "training_mazes_candidates": C,
                   "grad_allreduce": (dist.get_backend() if world > 1 else None)}
            snap = seen_snapshot(env, a.cfg_eval_mazes) if rank == 0 else None
            if growth:
                sm = tr.schedule.summary()
                rec.update(growth=list(growth), train_wins=sm["total_wins"],
                           instances_per_size_at_end={k: v for k, v in sm["instances_per_size"].items() if v},
                           retired=sm["retired"], stopped_at=tr.stopped_at)
            env.close()
            if rank == 0:
                n = a.cfg_eval_mazes
                rec["win_rate_greedy"], _ = evaluate(tr, n, dims, "r-prim", seed=0x7E5B0000, eps=0.0,
                                                     toroidal=True, device=dev)
                t6 = time.perf_counter()
                mz = best_of_mazes(n, dims, "r-prim", seed=0x7E5C0000, device=dev, toroidal=True)
                rec["best_of_6_selection_seconds"] = round(time.perf_counter() - t6, 3)
                rec["win_rate_greedy_best_of_6"], _ = evaluate(tr, n, dims, seed=0x7E5C0000, eps=0.0,
                                                               toroidal=True, device=dev, mazes=mz)
                rec["seen_mazes_reference_protocol"] = seen_protocol(
                    tr, snap, dev, 0x7E5C8000, toroidal=True, steps_eps=False)
                rec["eval_mazes"] = n
            out["cfg5" if mode == "fixed" else f"cfg5_{mode}"] = rec
            del tr
    return out


def reference_protocol(L, n, dim, dev, seed):
    """NeuralOffPolicyTrainer.test(n, new=True) (off_policy_trainer.py:228-263) for learner L: per
    maze random.choice(ALGOS) and a best-of-6 maze of that algorithm, acting greedy and through
    get_action's epsilon from steps_done (dqn_agent.py:104-119); rates overall and per algorithm."""
    import numpy as np
    from mazerl.trainers.vector_trainer import (best_of_mazes, evaluate, maze_algorithms,
                                                steps_done_epsilon)
    algos = maze_algorithms(n, seed=seed)
    mz = best_of_mazes(n, dim, algos, seed=seed, device=dev)
    sde = steps_done_epsilon(L, n)
    out = {"eps_start_mean": sde.start_mean,
           "algorithms": {x: algos.count(x) for x in sorted(set(algos))}}
    for name, eps in (("greedy", 0.0), ("eps_from_steps_done", sde)):
        rate, _, won = evaluate(L, n, dim, seed=seed, eps=eps, device=dev, mazes=mz, return_won=True)
        out[name] = rate
        out[name + "_by_algorithm"] = {x: float(np.mean([w for w, al in zip(won, algos) if al == x]))
                                       for x in sorted(set(algos))}
    return out


def infer_protocol(L, n, dim, dev, seed):
    """NeuralOffPolicyTrainer.infer(num_mazes, algo, shape) (off_policy_trainer.py:265-299), the
    reference scripts' last step (test_ddqn.py:52-54: `for algo in ALGOS: trainer.infer(15,
    algo)`): per algorithm, episodes on mazes of that algorithm through get_action. With `shape`
    each episode gets a new maze (update_new_maze); the scripts pass none, so there every episode
    replays the env's current maze (the last test maze, whatever its algorithm — set_algorithm only
    changes later generation): that literal reading measures one maze. Here the shape reading: n
    fresh best-of-6 mazes per algorithm, greedy and with epsilon from steps_done."""
    from mazerl.trainers.vector_trainer import best_of_mazes, evaluate, steps_done_epsilon
    out = {"mazes_per_algorithm": n}
    for k, algo in enumerate(("r-prim", "prim&kill", "dfs")):
        mz = best_of_mazes(n, dim, algo, seed=seed + k, device=dev)
        g, _ = evaluate(L, n, dim, algo, seed=seed + k, eps=0.0, device=dev, mazes=mz)
        e, _ = evaluate(L, n, dim, algo, seed=seed + k, eps=steps_done_epsilon(L, n), device=dev,
                        mazes=mz)
        out[algo] = {"greedy": g, "eps_from_steps_done": e}
    return out


def seen_snapshot(env, n):
    """The mazes n evenly spaced training instances hold at the end of training (host arrays,
    taken before the env closes) and those instances' ids."""
    import numpy as np
    from mazerl.trainers.vector_trainer import snapshot_mazes
    ids = np.unique(np.linspace(0, env.num_envs - 1, min(n, env.num_envs)).round().astype(np.int64))
    return ids, snapshot_mazes(env, ids)


def seen_protocol(L, snap, dev, seed, algos=None, toroidal=False, steps_eps=True):
    """NeuralOffPolicyTrainer.test(n, new=False) (off_policy_trainer.py:228-263 via
    update_visited_maze(remove=True), simple_maze_env.py:96-116; training_examples/.../
    test_ddqn.py:49: `test(len(env.mazes), new=False)`, the README's "W/R labirinti esplorati"
    column): the learner replays mazes it trained on. The reference's env.mazes holds its first
    maze and every win's update_maze replacement; here the mazes a sample of training instances
    hold at the end of training (seen_snapshot) — each an initial best-of-6 maze or a win's
    best-of-6 replacement that the instance trained on. Greedy, and through get_action's epsilon
    with each maze continuing its own instance's steps_done (DQN learners); per algorithm when
    the instances' maze algorithms are given."""
    import numpy as np
    from mazerl.trainers.vector_trainer import evaluate, steps_done_epsilon
    ids, mz = snap
    n = len(ids)
    dim = int(mz[2].max())
    out = {"mazes": n, "sample": "the final mazes of %d evenly spaced training instances" % n}
    modes = [("greedy", 0.0)]
    if steps_eps:
        sde = steps_done_epsilon(L, n, instances=ids)
        modes.append(("eps_from_steps_done", sde))
    for name, eps in modes:
        rate, _, won = evaluate(L, n, dim, seed=seed, eps=eps, device=dev, mazes=mz,
                                toroidal=toroidal, return_won=True)
        out[name] = rate
        if algos is not None:
            names = ["r-prim", "dfs", "prim&kill"]  # ids: vector_env.ALGOS
            al = np.asarray(algos)
            out[name + "_by_algorithm"] = {names[k]: float(np.mean(won[al == k]))
                                           for k in range(3) if (al == k).any()}
    return out


def log(msg):
    """Progress on stderr (the JSON line is the only stdout output)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def progress(rank, name, every=400):
    """train() keyword arguments for a progress line on rank 0 every `every` vector steps (one
    stream synchronisation each): long legs keep writing, so a supervisor that takes silence
    for a hang (and a reader of the log) sees them advance."""
    if rank != 0:
        return {}
    return {"log_every": every, "log": lambda r: log(f"{name}: vector step {r['step']}")}


def acting_agreement(L, n=65536):
    """How often the acting head's greedy action (the fused stem + GEMMs the trainer acts with)
    equals argmax of the f32 QNet (the reference's source_net(state).max(1), dqn_agent.py:
    113-116) on the newest n replay states — real trainer observations — with train-mode
    dropout off on both sides (the same stem on both: the comparison isolates precision)."""
    import torch
    rp = L.replay
    n = min(n, rp.size)
    idx = (torch.arange(rp.ptr - n, rp.ptr, device=rp.s6.device) % rp.capacity)
    s6, sw = rp.s6.index_select(0, idx), rp.sw.index_select(0, idx)
    net, fused = L.source, L.fused
    was = net.training
    net.eval()
    try:
        with torch.no_grad():
            q32 = net((s6, sw)).float()
            fused.invalidate()
            qa = fused(s6, sw).float()
    finally:
        net.train(was)
        fused.invalidate()
    a32, aa = q32.argmax(1), qa.argmax(1)
    top2 = q32.topk(2, dim=1).values
    gap = (top2[:, 0] - top2[:, 1]) / q32.abs().amax(1).clamp_min(1e-30)
    clear = gap > 1e-2
    return {"rows": n, "agreement": float((a32 == aa).float().mean()),
            "agreement_f32_gap_over_1pct": float((a32 == aa)[clear].float().mean()),
            "rows_f32_gap_over_1pct": int(clear.sum()),
            "acting_dtype": getattr(fused, "dtype_note", "bf16 GEMMs (f32 accumulate), bf16 stem")}


def launch_plan(n, environ, port):
    """The N rank environments `python3 bench.py --gpus N` starts when no launcher set WORLD_SIZE
    (the variables torchrun gives each rank: one process per GPU, rank r on GPU r)."""
    plan = []
    for r in range(n):
        e = dict(environ)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR=environ.get("MASTER_ADDR", "127.0.0.1"),
                 MASTER_PORT=str(port), MZ_BENCH_LAUNCHER="1")
        plan.append(e)
    return plan


def needs_launch(a, environ):
    """Decided from argv and the environment alone, before anything touches the GPU: --gpus N > 1
    and no launcher has set WORLD_SIZE -> this process starts the N ranks itself."""
    return a.gpus > 1 and "WORLD_SIZE" not in environ


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(n, argv, timeout, environ=None, script=None):
    """Start N child processes of this script (subprocess, never exec: the parent has not touched
    the GPU and stays a plain supervisor). Rank 0's stdout is relayed: JSON object lines to stdout
    (the bench line), anything else (e.g. the communication library's own banners) to stderr; the
    other ranks' stdout goes to stderr. If any rank fails, the deadline passes, or the supervisor
    itself gets SIGTERM / SIGINT (an outer `timeout`, Ctrl-C — the ranks run in sessions of their
    own and would not see it), every rank's process group is killed and the exit status is
    non-zero. Returns the exit status."""
    import signal
    import subprocess
    import threading
    environ = dict(os.environ if environ is None else environ)
    port = int(environ.get("MASTER_PORT") or _free_port())
    script = script or os.path.abspath(__file__)
    procs = []
    got = []  # signals received by the supervisor

    def on_signal(signum, frame):
        got.append(signum)

    old = {sig: signal.signal(sig, on_signal) for sig in (signal.SIGTERM, signal.SIGINT)}
    rc = 0
    reader = None
    try:
        for r, env in enumerate(launch_plan(n, environ, port)):
            procs.append(subprocess.Popen([sys.executable, "-u", script] + list(argv), env=env,
                                          stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno(),
                                          start_new_session=True, text=True))

        def relay(stream):
            for line in stream:
                dst = sys.stdout if line.lstrip().startswith("{") else sys.stderr
                dst.write(line)
                dst.flush()

        reader = threading.Thread(target=relay, args=(procs[0].stdout,), daemon=True)
        reader.start()
        deadline = time.monotonic() + timeout
        while True:
            if got:
                rc = 128 + got[0]
                print(f"bench launcher: got signal {got[0]}; stopping the ranks", file=sys.stderr)
                break
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0] if bad[0] > 0 else 128 - bad[0]
                print(f"bench launcher: a rank exited with {bad[0]}; stopping the others",
                      file=sys.stderr)
                break
            if all(c == 0 for c in codes):
                break
            if time.monotonic() > deadline:
                rc = 124
                print(f"bench launcher: deadline of {timeout:.0f} s passed; stopping the ranks",
                      file=sys.stderr)
                break
            time.sleep(0.2)
    except BaseException:
        rc = rc or 1
        raise
    finally:
        # every exit path that leaves ranks running (a failure, the deadline, a signal, an
        # exception in this loop) tears their process groups down: SIGTERM, then SIGKILL
        if any(p.poll() is None for p in procs):
            for sig, wait in ((signal.SIGTERM, 10.0), (signal.SIGKILL, 5.0)):
                for p in procs:
                    if p.poll() is None:
                        try:
                            os.killpg(p.pid, sig)
                        except ProcessLookupError:
                            pass
                t0 = time.monotonic()
                while any(p.poll() is None for p in procs) and time.monotonic() - t0 < wait:
                    time.sleep(0.1)
        for sig, h in old.items():
            signal.signal(sig, h)
        if reader is not None:
            reader.join(timeout=5.0)
    return rc


BF16_DENSE_PEAK_TFLOPS = 2500.0  # MI355X bf16 MFMA, dense (MI355X_MICROARCH.md)


# issued MFMA FLOP per row of QAct (csrc/mz_qact.hip): conv 49 chunks x 32 tiles x 4 MFMAs x 16,384
# per 128-row workgroup x 4 output tiles, fc1 3 x 2 x 1,600 x 1,024, fc2 3 x 2 x 1,024 x 512
QACT_ISSUED_FLOP = 49 * 32 * 4 * 16384 * 4 / 128 + 3 * 2 * 1600 * 1024 + 3 * 2 * 1024 * 512
REF_FWD_FLOP = 4665024  # the reference net's forward per sample


def q_head(dev, n, iters=50):
    """The acting Q-network forward of the DDQN learner on n instances (north_star: MFMA for the
    dense Q-head GEMMs), both heads, HIP events on the launch stream:
      x3   (the trainer's head) QAct: conv stem inside fc1's K loop + fc2 + fc3 + argmax, every
           GEMM operand split into bf16 hi + lo (three MFMAs per tile) — f32-accurate; all rows,
           and the greedy-row list at the training leg's typical size (0.43 n rows, count on
           the device);
      bf16 FusedQ: bf16 stem (k_qfront, features to HBM) + hipBLASLt bf16 GEMMs.
    algorithmic TFLOP/s = the reference's 4,665,024 FLOP per row / time; issued = the MFMA FLOP
    the kernels execute (QAct: x3 products + the conv recomputed per output tile)."""
    import torch
    import torch.nn.functional as F
    from mazerl.agents.fused import FusedQ
    from mazerl.agents.nets import QNet
    from mazerl.agents.qact import QAct
    torch.manual_seed(0)
    net = QNet(variant="ddqn").to(dev)
    fq = FusedQ(net, seed=1)
    qa = QAct(net, seed=1)
    g = torch.Generator(device=dev).manual_seed(0)
    bits = torch.randint(0, 2**31 - 1, (n, 22), generator=g, device=dev, dtype=torch.int32)
    obs6 = torch.rand(n, 6, generator=g, device=dev)
    st = torch.cuda.current_stream(dev)
    m = int(0.43 * n)
    rows = torch.randperm(n, generator=g, device=dev)[:m].to(torch.int32).contiguous()
    count = torch.tensor([m], dtype=torch.int32, device=dev)
    greedy = torch.zeros(n, dtype=torch.int64, device=dev)

    def timed(fn):
        for _ in range(5):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(iters):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / iters

    with torch.no_grad():
        t_x3 = timed(lambda: qa.greedy(obs6, bits, out=greedy))
        t_x3r = timed(lambda: qa.rows_greedy(obs6, bits, rows, count, greedy))
        t_all = timed(lambda: fq(obs6, bits))
        feat = fq.stem(obs6, bits)
        w0, b0 = fq.head._w[0]
        t_fc1 = timed(lambda: F.linear(feat, w0, b0))
    f_fc1 = 2.0 * n * 1574 * 1024
    f_all = n * (388800 + 2.0 * (1574 * 1024 + 1024 * 512 + 512 * 4))

    def x3(t, rows_):
        return {"rows": rows_, "ms": t, "alg_tflops": rows_ * REF_FWD_FLOP / (t * 1e-3) / 1e12,
                "issued_tflops": rows_ * QACT_ISSUED_FLOP / (t * 1e-3) / 1e12,
                "mfma_frac": rows_ * QACT_ISSUED_FLOP / (t * 1e-3) / 1e12 / BF16_DENSE_PEAK_TFLOPS}
    return {"instances": n,
            "x3": {"all_rows": x3(t_x3, n), "greedy_rows": x3(t_x3r, m),
                   "issued_flop_per_row": QACT_ISSUED_FLOP,
                   "dtype": "bf16x3 (hi*hi + hi*lo + lo*hi, f32 accumulate)"},
            "bf16": {"forward_ms": t_all, "fc1_ms": t_fc1,
                     "fc1_tflops": f_fc1 / (t_fc1 * 1e-3) / 1e12,
                     "fc1_mfma_frac": f_fc1 / (t_fc1 * 1e-3) / 1e12 / BF16_DENSE_PEAK_TFLOPS,
                     "forward_tflops": f_all / (t_all * 1e-3) / 1e12,
                     "forward_mfma_frac": f_all / (t_all * 1e-3) / 1e12 / BF16_DENSE_PEAK_TFLOPS,
                     "dtype": "bf16 (f32 accumulate)"},
            "peak_tflops": BF16_DENSE_PEAK_TFLOPS}


def host_threads():
    """Every host core this process may use: the CPU affinity set, capped by the cgroup's CPU
    quota when one is set (a GPU box's share of a larger machine: os.cpu_count() and the
    affinity set show the whole machine there, the quota is what the threads get)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    n = min(aff, quota) if quota else aff
    return n, {"affinity_cpus": aff, "cgroup_cpu_quota": quota, "threads": n}


def cpu_baseline(env, seconds):
    """Oracle (oracle/mzoracle.c, 'port' of the reference algorithm at its cost model: heap A*
    for every find_path) timed on this host's cores on one of the benchmark's own mazes."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O
    from mazerl import VectorMazeEnv
    q = env.query(0)
    grid = env.grid(0)
    start, goal = (q["start_r"], q["start_c"]), (q["goal_r"], q["goal_c"])
    threads, cpu_note = host_threads()
    # calibrate on a short run, then size the sample to ~`seconds`
    t, n = O.bench(grid, start, goal, False, True, True, threads, 20, threads)
    rate = n / max(t, 1e-9)
    per_env = max(20, int(rate * seconds / threads))
    t, n = O.bench(grid, start, goal, False, True, True, threads, per_env, threads, seed=2)
    tf, nf = O.bench(grid, start, goal, False, True, False, threads, per_env * 20, threads, seed=3)
    t1, n1 = O.bench(grid, start, goal, False, True, True, 1, max(20, per_env // 4), 1, seed=4)
    per_config = {}
    for name, dim, tor in (("cfg2 15x15 euclidean Enrich", 15, False),
                           ("cfg5 29x29 toroidal Enrich", 29, True)):
        # the other configs' grids, one maze each (generated on the GPU), reference-cost mode
        e2 = VectorMazeEnv(1, dim, toroidal=tor, enrich=True, device=env.device, seed=0x5EED0000)
        q2 = e2.query(0)
        g2 = e2.grid(0)
        e2.close()
        s2, g2p = (q2["start_r"], q2["start_c"]), (q2["goal_r"], q2["goal_c"])
        tc, nc = O.bench(g2, s2, g2p, tor, True, True, threads, 2000, threads)
        per = max(2000, int(nc / max(tc, 1e-9) * 1.5 / threads))  # ~1.5 s sample
        tc, nc = O.bench(g2, s2, g2p, tor, True, True, threads, per, threads, seed=5)
        per_config[name] = {"value": nc / tc, "steps": nc, "seconds": round(tc, 2)}
    return {"value": n / t, "unit": "env steps/s", "cores": threads, "kind": "port",
            "cores_note": cpu_note,
            "single_core": {"value": n1 / t1, "steps": n1, "seconds": round(t1, 2)},
            "per_config": per_config,
            "sample": f"{threads} envs x {per_env} steps (81x81 r-prim Enrich, masked-exploration "
                      f"actions, auto-reset), oracle in reference-cost mode (heap A* per find_path); "
                      f"{t:.1f} s",
            "bfs_field_mode": {"value": nf / tf, "steps": nf, "seconds": round(tf, 2)}}


def main():
    a = parse()
    if needs_launch(a, os.environ):
        sys.exit(launch(a.gpus, sys.argv[1:], a.launch_timeout))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)  # before the process group: RCCL binds each rank to its GPU
    dev = torch.device("cuda", local)
    backend = None
    if world > 1:
        # RCCL ("nccl") on the 8-GPU node; MZ_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs
        backend = os.environ.get("MZ_DIST_BACKEND", "nccl")
        kw = {"device_id": dev} if backend == "nccl" else {}
        dist.init_process_group(backend, init_method="env://", **kw)
    ranks_seen = dist.get_world_size() if world > 1 else 1
    if rank == 0:
        log(f"rank 0 of {ranks_seen} on {dev} (backend {backend})")

    import mazerl
    B = a.envs
    legs = [x for x in a.legs.split(",") if x]

    def leg(mode):
        """One env-step leg: generate B mazes (global instance ids rank*B.. : Philox seed
        0x5EED0000 + global id), W untimed + K timed vector steps, each one k_step
        launch (fused act + step + autoreset), inputs resident in HBM."""
        t0 = time.perf_counter()
        env = mazerl.VectorMazeEnv(B, a.dim, enrich=True, device=dev, algorithm=a.algo,
                                   seed=0x5EED0000 + rank * B, window=mode == "window",
                                   window_bits=mode == "bits", pos=False, done_list=False)
        torch.cuda.synchronize()
        gen_s = time.perf_counter() - t0
        stream = torch.cuda.current_stream(dev)

        def vstep(k):
            # one launch: fused act + step, autoreset of the instances that finished last step
            env.step_act(eps=1.0, seed=0xBE7C4 + rank, counter=k, autoreset=True)

        def timed(run):
            """K steps between a barrier + synchronize on each side: wall seconds (max over the
            ranks) and the HIP-event time of the K launches on the launch stream."""
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ev0.record(stream)
            run()
            ev1.record(stream)
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            el = time.perf_counter() - t0
            if world > 1:
                t = torch.tensor([el], dtype=torch.float64, device=dev)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                el = float(t.item())
            return el, ev0.elapsed_time(ev1) / a.steps

        for k in range(a.warmup):
            vstep(k)
        graphs = []
        if a.graph:
            # the K timed launches as replays of captured HIP graphs of `chunk` k_step launches
            # each (the same launch with the same work per step; counters a.warmup + j of each
            # chunk, so each replay repeats the chunk's Philox draws over the evolving state)
            chunk = max(1, min(a.graph_chunk, a.steps))
            sizes = [chunk] * (a.steps // chunk) + ([a.steps % chunk] if a.steps % chunk else [])
            made = {}
            for n_ in sorted(set(sizes)):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for j in range(n_):
                        vstep(a.warmup + j)
                made[n_] = g
            graphs = [made[n_] for n_ in sizes]
            for g in made.values():  # untimed: one replay of each graph
                g.replay()
        el, avg_kernel_ms = timed(lambda: [g.replay() for g in graphs] if graphs else
                                  [vstep(a.warmup + k) for k in range(a.steps)])
        eager = None
        if graphs:  # the same K steps as K eager launches from the Python loop, for comparison
            el_e, avg_e = timed(lambda: [vstep(a.warmup + k) for k in range(a.steps)])
            eager = {"value": B * a.steps * world / el_e, "ms_per_step": el_e / a.steps * 1e3,
                     "avg_kernel_ms": avg_e}
        del graphs
        alg = ALG_BYTES_PER_STEP if mode == "window" else ALG_BYTES_PER_STEP_BITS
        achieved = alg * B / (avg_kernel_ms * 1e-3) / 1e9
        traffic, tnote = pmc_traffic(mode, B, a.dim)
        roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                "kernel": "k_step", "avg_kernel_ms": avg_kernel_ms,
                "timing": "HIP events around the timed region on the launch stream"
                          + (f" (replays of captured HIP graphs of {min(a.graph_chunk, a.steps)} "
                             "k_step launches)" if a.graph else " (eager launches)"),
                "alg_bytes_per_instance_step": alg, "traffic_source": tnote}
        return env, {"value": B * a.steps * world / el, "ms_per_step": el / a.steps * 1e3,
                     "roofline": roof, "gen_s": gen_s, "eager_launch_loop": eager}

    res = {}
    env = None
    for mode in legs:
        if env is not None:
            env.close()
        if rank == 0:
            log(f"env-step leg: {mode}")
        env, res[mode] = leg(mode)
    head = res["window"] if "window" in res else res[legs[0]]
    value, gen_s = head["value"], head["gen_s"]
    stream = torch.cuda.current_stream(dev)

    # steady-state regeneration of all B mazes per algorithm (after the timed region; the module
    # is loaded): one mz_generate launch each, HIP events on the launch stream
    steady = {}
    for algo in ("dfs", "prim&kill", "r-prim"):  # r-prim last: cpu_baseline reads maze 0
        g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        g0.record(stream)
        env.generate(algorithm=algo, seed=0x6E4E0000 + rank * B)
        g1.record(stream)
        g1.synchronize()
        steady[algo] = B / (g0.elapsed_time(g1) * 1e-3)

    if rank == 0:
        out = {
            "metric": "env steps/sec (whole node) + DQN win-rate, 40x40 r-prim mazes",
            "value": value,
            "unit": "env steps/s",
            "n_gpus": world,
            "ranks_seen": ranks_seen,
            "backend": ("RCCL (torch.distributed nccl)" if backend == "nccl" else backend),
            "launch": ("bench.py --gpus N (self-launched ranks)" if os.environ.get("MZ_BENCH_LAUNCHER") == "1"
                       else ("torchrun / external launcher" if world > 1 else "single process")),
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": head["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (GPU-generated r-prim mazes, Philox seeds 0x5EED0000 + instance id)",
            "config": {"workload": f"{B} x 40x40-cell ({a.dim}x{a.dim} grid) {a.algo} Enrich mazes "
                                   f"per GPU: fused act + env step (f32 3x15x15 window) with autoreset, one launch per step",
                       "envs_per_gpu": B, "grid": a.dim, "algo": a.algo, "parallelism": f"dp{world} env shards"},
            "roofline": head["roofline"],
            "eager_launch_loop": head["eager_launch_loop"],
            "bits_mode": ({"value": res["bits"]["value"], "unit": "env steps/s",
                           "ms_per_step": res["bits"]["ms_per_step"],
                           "roofline": res["bits"]["roofline"],
                           "eager_launch_loop": res["bits"]["eager_launch_loop"],
                           "note": "the same step in the trainers' mode (window_bits=True: the "
                                   "675-bit window as 88 B of bits, no f32 window)"}
                          if "bits" in res and "window" in res else None),
            "generation": {"mazes": B, "seconds": round(gen_s, 3), "mazes_per_s": B / gen_s,
                           "note": "first build incl. module load; excluded from value",
                           "steady_mazes_per_s": steady,
                           "steady_note": f"per GPU: all {B} {a.dim}x{a.dim} mazes regenerated in one "
                                          "launch per algorithm (generation + BFS tables + goal)"},
            "win_rate": None,
        }
        if world == 1 and not a.no_cpu_baseline:
            log("cpu_baseline")
            out["cpu_baseline"] = cpu_baseline(env, a.cpu_seconds)
    env.close()
    if a.train_steps > 0:
        if rank == 0:
            log("DDQN win-rate leg (configs[2])")
        wr = win_rate(a, dev, rank, world)  # every rank trains its shard (grad all-reduce)
        if rank == 0:
            out["win_rate"] = wr
            out["q_head"] = q_head(dev, B)
    if a.curriculum_steps > 0:
        for j, rule in enumerate(x for x in a.curriculum_rules.split(",") if x):
            if rank == 0:
                log(f"DDQN curriculum leg, {rule} rule (the reference's new-maze protocol)")
            cl = curriculum_leg(a, dev, rank, world, rule)
            if rank == 0:
                out["curriculum_leg" if j == 0 else "curriculum_leg_" + rule.replace("-", "_")] = cl
    if a.config_legs:
        cl = config_legs(a, dev, rank, world)
        if rank == 0:
            out["configs"] = cl
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
