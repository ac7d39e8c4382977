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
