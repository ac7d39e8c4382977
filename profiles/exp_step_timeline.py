#!/usr/bin/env python3
"""Where a training vector step waits (no profiler attached): HIP events on the acting stream at
the phase boundaries of VectorOffPolicyTrainer.vector_step (bench.py's DDQN leg, 65,536 x 81x81),
and host timestamps of the same points. Per phase: GPU time between events, host issue time."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))
import torch  # noqa: E402

from mazerl import VectorMazeEnv  # noqa: E402
from mazerl.agents.dqn import VectorDQNLearner  # noqa: E402
from mazerl.trainers.vector_trainer import VectorOffPolicyTrainer  # noqa: E402

dev = torch.device("cuda", 0)
B, dim = 65536, 81
env = VectorMazeEnv(B, dim, enrich=True, device=dev, algorithm="r-prim", seed=0xA11CE,
                    done_list=False, window=False, window_bits=True)
decay = ((dim - 1) * (dim - 1) // 2) * 5 / 40.0
L = VectorDQNLearner(B, dev, variant="ddqn", lr=1e-3, eps_start=0.95, eps_final=0.1, eps_decay=decay,
                     gamma=0.7, batch_size=1024, capacity=2_000_000, target_every=13, overlap=True)
tr = VectorOffPolicyTrainer(env, L, seed=3)
tr.train(400)
torch.cuda.synchronize()

marks = []  # (name, host time, event)


def mark(name):
    ev = torch.cuda.Event(enable_timing=True)
    ev.record()
    marks.append((name, time.perf_counter(), ev))


# wrap the phases
_greedy, _step, _upd, _reset = L.greedy, env.step_act, L.update, env.reset_done


def greedy(*a, **k):
    mark("greedy_in")
    r = _greedy(*a, **k)
    mark("greedy_out")
    return r


def step_act(*a, **k):
    r = _step(*a, **k)
    mark("step_out")
    return r


def reset_done(*a, **k):
    r = _reset(*a, **k)
    mark("reset_out")
    return r


def update(*a, **k):
    r = _upd(*a, **k)
    mark("update_out")
    return r


L.greedy, env.step_act, L.update, env.reset_done = greedy, step_act, update, reset_done
side = []  # (start event on the side stream, published end event) per update
for _ in range(3):
    tr.vector_step()  # graphs exist now
_replay = L._graph[0].replay


class _G:
    def replay(self):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()  # current stream = the side stream inside _update_async
        side.append([ev, None])
        _replay()


L._graph = (_G(),) + tuple(L._graph[1:])
_pub = L._published


class _Pub(list):
    def append(self, x):
        if side and side[-1][1] is None:
            e = torch.cuda.Event(enable_timing=True)
            e.record(L.side)
            side[-1][1] = e
        super().append(x)

    def popleft(self):
        return self.pop(0)


L._published = _Pub(_pub)
marks.clear()
for _ in range(200):
    tr.vector_step()
torch.cuda.synchronize()
names = ["greedy_in", "greedy_out", "step_out", "reset_out", "update_out"]
steps = [marks[i:i + 5] for i in range(0, len(marks) - 5, 5)][50:]
gpu = {f"{names[j]}->{names[(j + 1) % 5]}": 0.0 for j in range(5)}
host = dict(gpu)
for s, nxt in zip(steps, steps[1:]):
    seq = s + [nxt[0]]
    for j in range(5):
        k = f"{names[j]}->{names[(j + 1) % 5]}"
        gpu[k] += seq[j][2].elapsed_time(seq[j + 1][2]) * 1e3
        host[k] += (seq[j + 1][1] - seq[j][1]) * 1e6
n = len(steps) - 1
sd = [a.elapsed_time(b) * 1e3 for a, b in side[50:] if b is not None]
gaps = [side[i][1].elapsed_time(side[i + 1][0]) * 1e3 for i in range(50, len(side) - 1)]
period = side[50][0].elapsed_time(side[-1][0]) * 1e3 / (len(side) - 51)
print(json.dumps({"update_gpu_us": round(sum(sd) / len(sd), 1),
                  "side_idle_between_updates_us": round(sum(gaps) / len(gaps), 1),
                  "update_period_us": round(period, 1)}))
print(json.dumps({"steps": n, "gpu_us (acting stream, event to event)": {k: round(v / n, 1) for k, v in gpu.items()},
                  "host_us (issue point to issue point)": {k: round(v / n, 1) for k, v in host.items()}}, indent=1))
