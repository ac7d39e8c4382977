"""The multi-GPU learner path on the GPU: two ranks (gloo, both on cuda:0 — the 8-GPU node runs
the same code over RCCL) with different replay data. The HIP-graph-captured update (backward +
pack graph, the all-reduce of the flat gradient bucket, unpack + clamp + AdamW graph) must track
the eager all-reduce update (learner_update, dqn_agent.py:121-157 with the gradient average of
SURVEY §8e) update for update, and both ranks must hold bit-identical weights afterwards — also
with the overlapped schedule (bench.py's default: graph replays and the all-reduce issued on the
side stream, agents/dqn.py VectorDQNLearner(overlap=True)).
Tolerances as in test_learner_graph.py (capturable vs eager AdamW arithmetic)."""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir, overlap, backend="gloo", shard=None, gcoll=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    import torch.distributed as dist
    from mazerl import VectorMazeEnv
    from mazerl.agents.dqn import VectorDQNLearner
    from mazerl.distributed import GradAllReduce, broadcast_params, init_from_env
    from test_learner_graph import _fill
    torch.cuda.set_device(0)
    if world > 1:
        init_from_env(backend)
    else:  # one rank: init_from_env leaves the group out; RCCL binds the communicator to cuda:0
        dist.init_process_group(backend, init_method="env://",
                                **({"device_id": torch.device("cuda", 0)} if backend == "nccl" else {}))
    assert dist.get_backend() == backend
    env = VectorMazeEnv(4, 21, enrich=True, device="cuda", seed=1)
    mk = lambda g, ov, gc=False: VectorDQNLearner(  # noqa: E731
        4, "cuda", variant="ddqn", batch_size=32, capacity=64, updates_per_step=1, target_every=4,
        updates_per_epoch=2, seed=5 + rank, use_graph=g, overlap=ov,
        allreduce=GradAllReduce(shard=shard), graph_collectives=gc)
    A, B = mk(True, overlap, gcoll), mk(False, False)
    # gcoll: a third learner on the two-graph path (collectives between the replays) beside A
    C = mk(True, overlap) if gcoll else None
    assert A.use_graph and not B.use_graph
    # the graph learner's step: reduce-scatter + AdamW over this rank's shard + all-gather
    # (distributed.GradAllReduce.attach), unless shard=False (the flat-bucket all-reduce)
    assert A.allreduce.sharded == (shard is not False and (world > 1 or shard is True))
    assert not B.allreduce.sharded  # torch's AdamW: the all-reduce path
    broadcast_params(A.source)  # rank 1 started from other weights (seed 5 + rank)
    A.target.load_state_dict(A.source.state_dict())
    B.source.load_state_dict(A.source.state_dict())
    B.target.load_state_dict(A.source.state_dict())
    for L in (A, B) + ((C,) if C is not None else ()):
        if L is not A:
            L.source.load_state_dict(A.source.state_dict())
            L.target.load_state_dict(A.source.state_dict())
        _fill(L, seed=10 + rank)  # different data per rank: the average matters
        # Dropout(0.2) in train mode (Q13) would draw different masks in the two paths
        L.source.eval(); L.target.eval()
    losses, went_async = [], False
    for _ in range(9):
        la = A.update(env.expand_window, reserve=0)
        went_async |= bool(getattr(A, "_async", False))
        lb = B.update(env.expand_window)
        lc = C.update(env.expand_window, reserve=0) if C is not None else la
        torch.cuda.synchronize()
        losses.append((float(la), float(lb), float(lc)))
    if overlap:
        A.finish()
        if C is not None:
            C.finish()
        torch.cuda.synchronize()
    assert went_async == overlap
    # in-graph collectives: one update graph; else backward + pack, then unpack + AdamW
    assert A._graph is not None and len(A._graph) == (1 if gcoll else 2)
    torch.save({"losses": losses,
                "A": [p.detach().cpu() for p in A.source.parameters()],
                "B": [p.detach().cpu() for p in B.source.parameters()],
                "C": [p.detach().cpu() for p in (C or A).source.parameters()]},
               os.path.join(outdir, f"r{rank}.pt"))
    env.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("shard", [None, False], ids=["sharded", "allreduce"])
@pytest.mark.parametrize("overlap", [False, True], ids=["sequential", "overlapped"])
def test_graph_allreduce_update_tracks_eager_two_ranks(overlap, shard):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), d, overlap, "gloo", shard), nprocs=2, join=True)
        r = [torch.load(os.path.join(d, f"r{k}.pt"), weights_only=True) for k in range(2)]
    for k in range(2):
        for la, lb, _ in r[k]["losses"]:
            assert la == pytest.approx(lb, rel=1e-4, abs=1e-7)
        for pa, pb in zip(r[k]["A"], r[k]["B"]):
            assert torch.allclose(pa, pb, rtol=1e-5, atol=1e-5)
    for pa0, pa1 in zip(r[0]["A"], r[1]["A"]):  # the average keeps the replicas identical
        assert torch.equal(pa0, pa1)
    for pb0, pb1 in zip(r[0]["B"], r[1]["B"]):
        assert torch.equal(pb0, pb1)
    # and the ranks' data differed: rank 0's and rank 1's first losses are not the same
    assert r[0]["losses"][0][0] != r[1]["losses"][0][0]


@pytest.mark.parametrize("shard", [True, False], ids=["sharded", "allreduce"])
@pytest.mark.parametrize("overlap", [False, True], ids=["sequential", "overlapped"])
def test_graph_allreduce_update_over_rccl_one_rank(overlap, shard):
    """The same learner path with the all-reduce over RCCL ("nccl" backend, RCCL 2.26 on ROCm):
    a gpurun box has one GPU and RCCL refuses two ranks on one device ("Duplicate GPU detected",
    profiles/r03z_rccl_probe.txt), so this runs one rank — the RCCL communicator bound to cuda:0,
    the flat-bucket all-reduce issued between the two captured graphs (and, overlapped, on the
    side stream; sharded: the reduce-scatter and all-gather around the shard's AdamW, here over
    one shard) — and checks it against the eager update as above."""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(1, _free_port(), d, overlap, "nccl", shard), nprocs=1, join=True)
        r = torch.load(os.path.join(d, "r0.pt"), weights_only=True)
    for la, lb, _ in r["losses"]:
        assert la == pytest.approx(lb, rel=1e-4, abs=1e-7)
    for pa, pb in zip(r["A"], r["B"]):
        assert torch.allclose(pa, pb, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("shard", [True, False], ids=["sharded", "allreduce"])
@pytest.mark.parametrize("overlap", [False, True], ids=["sequential", "overlapped"])
def test_graph_collectives_in_graph_over_rccl_one_rank(overlap, shard):
    """The collectives captured inside the update graph (graph_collectives=True: backward,
    reduce-scatter / all-reduce, AdamW, all-gather in ONE replay, thread-local capture over RCCL)
    against the two-graph path with the collectives issued between the replays: the same kernels
    in the same order, so the same losses and weights bit for bit, and against the eager update
    within test_learner_graph.py's tolerances. (gloo cannot run inside a captured graph — it
    copies through the host — so the two-rank gloo tests cover the two-graph path only.)"""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(1, _free_port(), d, overlap, "nccl", shard, True), nprocs=1,
                 join=True)
        r = torch.load(os.path.join(d, "r0.pt"), weights_only=True)
    for la, lb, lc in r["losses"]:
        assert la == lc
        assert la == pytest.approx(lb, rel=1e-4, abs=1e-7)
    for pa, pb, pc in zip(r["A"], r["B"], r["C"]):
        assert torch.equal(pa, pc)
        assert torch.allclose(pa, pb, rtol=1e-5, atol=1e-5)
