"""world_size-2 gloo tests of the multi-GPU path on CPU: the learner's flat-bucket gradient
all-reduce (+ clamp after the average) reproduces the single-process update on the union batch,
and the episode counters are summed over ranks."""
import os
import random
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import learner_util as U


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(n, seed):
    s6, w, a, r, s6n, wn = U.make_batch(n, seed)
    t = torch.from_numpy
    return (t(s6), t(w)), t(a), torch.tensor(r, dtype=torch.float32), (t(s6n), t(wn))


def _update(src, tgt, batch, allreduce=None):
    from mazerl.agents.dqn import learner_update, q_loss
    opt = torch.optim.AdamW(src.parameters(), 1e-3)
    state, a, r, nxt = batch
    loss = q_loss(src, tgt, state, a, r, nxt, 0.7, True)
    learner_update(src, opt, loss, allreduce=allreduce)


def _nets():
    from mazerl.agents.nets import QNet
    src, tgt = QNet(3, 6, 4, 4, 16, "ddqn"), QNet(3, 6, 4, 4, 16, "ddqn")
    U.fill_params(src, 1)
    U.fill_params(tgt, 2)
    src.eval(); tgt.eval()
    return src, tgt


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from mazerl.distributed import GradAllReduce, allreduce_sum, broadcast_params, init_from_env
    r, w, _ = init_from_env("gloo")
    assert (r, w) == (rank, world)
    src, tgt = _nets()
    if rank == 1:  # rank 1 starts from different weights: broadcast must fix that
        U.fill_params(src, 999)
    broadcast_params(src)
    (s6, win), a, rew, (s6n, wn) = _batch(16, 5)
    sl = slice(rank * 8, rank * 8 + 8)
    _update(src, tgt, ((s6[sl], win[sl]), a[sl], rew[sl], (s6n[sl], wn[sl])), GradAllReduce())
    stats = torch.tensor([rank + 1.0, 10.0 * (rank + 1)], dtype=torch.float64)
    allreduce_sum(stats)
    torch.save({k: v.clone() for k, v in src.state_dict().items()} | {"stats": stats},
               os.path.join(outdir, f"r{rank}.pt"))
    dist.destroy_process_group()


def test_ddp_update_equals_single_process_union_batch():
    torch.set_num_threads(1)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        r0 = torch.load(os.path.join(d, "r0.pt"), weights_only=True)
        r1 = torch.load(os.path.join(d, "r1.pt"), weights_only=True)
    src, tgt = _nets()
    _update(src, tgt, _batch(16, 5))
    for k, v in src.state_dict().items():
        torch.testing.assert_close(r0[k], v, rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(r1[k], v, rtol=1e-5, atol=1e-7)
    assert r0["stats"].tolist() == [3.0, 30.0] == r1["stats"].tolist()


def _ppo_worker(rank, world, port, outdir):
    """Config 5's update on two ranks whose pools hold different numbers of non-finite rows
    (trainers/ppo_trainer.py pool_update): both keep the smaller kept count, run the same
    minibatch schedule with the flat-bucket gradient all-reduce, and end with identical weights."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from mazerl.agents.ppo import ActorCriticNet, make_optimizer
    from mazerl.distributed import GradAllReduce, broadcast_params, init_from_env
    from mazerl.trainers.ppo_trainer import pool_update
    init_from_env("gloo")
    net = ActorCriticNet(3, 6, 4, 4, hidden_dim=16)
    U.fill_params(net, 7 if rank == 0 else 8)
    broadcast_params(net)
    opt = make_optimizer(net, 3e-4, 1e-4)
    g = torch.Generator().manual_seed(100 + rank)  # each rank its own pool
    P = 40
    s6 = torch.rand(P, 6, generator=g)
    win = (torch.rand(P, 3, 15, 15, generator=g) < 0.5).float()
    a = torch.randint(0, 4, (P,), generator=g)
    lp = -torch.rand(P, generator=g)
    adv, ret = torch.randn(P, generator=g), torch.randn(P, generator=g)
    bad = [3, 17, 30] if rank == 0 else [0, 5, 6, 11, 22, 23, 39]  # NaN / inf rows
    adv[bad[::2]] = float("nan")
    ret[bad[1::2]] = float("inf")
    kept = pool_update(net, opt, (s6, win, a, lp, adv, ret), 1e-2, 8, 2,
                       allreduce=GradAllReduce())
    torch.save({"kept": kept, **{k: v.clone() for k, v in net.state_dict().items()}},
               os.path.join(outdir, f"p{rank}.pt"))
    dist.destroy_process_group()


def test_ppo_pool_update_two_ranks_agree_on_rows_and_weights():
    torch.set_num_threads(1)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_ppo_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        r0 = torch.load(os.path.join(d, "p0.pt"), weights_only=True)
        r1 = torch.load(os.path.join(d, "p1.pt"), weights_only=True)
    assert r0.pop("kept") == r1.pop("kept") == 40 - 7  # the smaller kept count on both ranks
    for k in r0:
        assert torch.equal(r0[k], r1[k]), k  # same schedule, same averaged gradients


def _shard_worker(rank, world, port, outdir):
    """GradAllReduce's sharded step on CPU (gloo): the in-place reduce-scatter leaves rank r's
    shard of the flat gradient buffer = the ranks' sum (what the all-reduce gives there); an
    elementwise step on that shard followed by the in-place all-gather leaves every rank with the
    step the all-reduce path computes over the whole buffer."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from mazerl.agents.flat import FLAT_ALIGN
    from mazerl.distributed import GradAllReduce, init_from_env
    init_from_env("gloo")
    n = 3 * FLAT_ALIGN  # a flat buffer as flatten_params lays it out (multiple of FLAT_ALIGN)
    g = torch.Generator().manual_seed(40 + rank)
    grads = torch.randn(n, generator=g)
    params0 = torch.randn(n, generator=torch.Generator().manual_seed(7))  # replicas agree
    net = type("Net", (), {})()
    net._flat_grads, net._flat_params = grads.clone(), params0.clone()
    ar = GradAllReduce(shard=True)
    ar.sharded, ar._S, ar._flat = True, n // world, net._flat_grads  # (attach needs FlatAdamW)
    ar.reduce()
    S = n // world
    sl = slice(rank * S, (rank + 1) * S)
    step = lambda p, gr: p - 0.1 * torch.clamp(gr / world, -1, 1)  # noqa: E731 (elementwise)
    net._flat_params[sl] = step(net._flat_params[sl], net._flat_grads[sl])
    ar.gather(net)
    full = grads.clone()  # the all-reduce path
    dist.all_reduce(full)
    torch.save({"sharded": net._flat_params.clone(), "allreduce": step(params0, full),
                "shard_sum": net._flat_grads[sl].clone(), "full_sum": full[sl].clone()},
               os.path.join(outdir, f"s{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_step_equals_allreduce_step(world):
    torch.set_num_threads(1)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_shard_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        rs = [torch.load(os.path.join(d, f"s{k}.pt"), weights_only=True) for k in range(world)]
    for r in rs:
        assert torch.equal(r["shard_sum"], r["full_sum"])
        assert torch.equal(r["sharded"], r["allreduce"])
        assert torch.equal(r["sharded"], rs[0]["sharded"])


class _FakeEnv:
    """What WinSchedule needs of a VectorMazeEnv (CPU tensors)."""

    def __init__(self, B, max_dim=81):
        self.device, self.num_envs, self.max_dim = torch.device("cpu"), B, max_dim
        self.algo_set, self.regen = None, None

    def set_algorithm(self, a):
        self.algo_set = a.clone()

    def set_regen_dims(self, d):
        self.regen = d


def _schedule_steps():
    g = torch.Generator().manual_seed(11)
    return [(torch.rand(16, generator=g) < 0.3) for _ in range(6)]


def _schedule_worker(rank, world, port, outdir):
    """Each rank holds 8 of 16 instances: the global rule's algorithms and epsilon_decay match a
    single process holding all 16; with growth, a rank whose instances all retired keeps
    training until every rank's have (a rank stopping alone left the others'
    collectives unmatched)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from mazerl.distributed import init_from_env
    from mazerl.trainers.schedule import WinSchedule
    init_from_env("gloo")

    class L:
        eps_decay = 100.0
    lr = L()
    s = WinSchedule(_FakeEnv(8), "global", learner=lr)
    algos = []
    for t in _schedule_steps():
        t = t[8 * rank:8 * rank + 8]
        s.before_reset(t)
        s.after_reset(t)
        algos.append(s.algo.clone())
    # growth 15 -> 19 (max 19): an instance retires on its first win
    g = WinSchedule(_FakeEnv(8, max_dim=19), None, growth=(15, 19))
    seen = []
    for k in range(3):
        t = torch.zeros(8, dtype=torch.bool)
        if rank == 0 and k == 0:
            t[:] = True       # rank 0's whole shard retires at once
        if rank == 1 and k == 2:
            t[:] = True       # rank 1's two steps later
        g.before_reset(t)
        g.after_reset(t)
        seen.append(g.all_retired())
    torch.save({"algos": torch.stack(algos), "eps_decay": float(lr.eps_decay),
                "total_wins": int(s.total_wins), "retired_seen": seen},
               os.path.join(outdir, f"s{rank}.pt"))
    dist.destroy_process_group()


def test_global_schedule_and_growth_stop_over_two_ranks():
    from mazerl.trainers.schedule import WinSchedule

    class L:
        eps_decay = 100.0
    lr = L()
    ref = WinSchedule(_FakeEnv(16), "global", learner=lr)
    ref_algos = []
    for t in _schedule_steps():
        ref.before_reset(t)
        ref.after_reset(t)
        ref_algos.append(ref.algo.clone())
    ref_algos = torch.stack(ref_algos)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_schedule_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        out = [torch.load(os.path.join(d, f"s{r}.pt"), weights_only=True) for r in range(2)]
    assert torch.equal(torch.cat([out[0]["algos"], out[1]["algos"]], 1), ref_algos)
    for o in out:
        assert o["eps_decay"] == float(lr.eps_decay) and o["total_wins"] == int(ref.total_wins)
        assert o["retired_seen"] == [False, False, True]
