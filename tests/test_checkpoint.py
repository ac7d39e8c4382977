"""Checkpoint / resume of the vectorised learner on the CPU (mazerl/checkpoint.py).

VectorDQNLearner.state_dict() taken mid-run, loaded into a fresh learner (other seed, other
construction order) and through a torch.save / torch.load(weights_only=True) round trip: the next
updates give bit-identical nets, optimizer state and replay pointers on both. The env half and the
whole-trainer resume (device state, maze bank, captured update graphs) are GPU tests
(tests/test_checkpoint_gpu.py)."""
import io

import pytest
import torch

from mazerl.agents.dqn import VectorDQNLearner


def expand(bits):
    """Packed 675-bit windows (int32 [n, 22]) -> f32 [n, 3, 15, 15] (the layout of window_bits)."""
    b = bits.to(torch.int64) & 0xFFFFFFFF
    k = torch.arange(675)
    v = (b[:, k // 32] >> (k % 32)) & 1
    return v.to(torch.float32).view(-1, 3, 15, 15)


def fill(L, n, seed):
    g = torch.Generator().manual_seed(seed)
    s6 = torch.rand(n, 6, generator=g)
    sw = torch.randint(0, 2**31 - 1, (n, 22), generator=g, dtype=torch.int32)
    a = torch.randint(0, 4, (n,), generator=g)
    r = torch.rand(n, generator=g) - 0.5
    L.replay.push(s6, sw, a, r, torch.rand(n, 6, generator=g),
                  torch.randint(0, 2**31 - 1, (n, 22), generator=g, dtype=torch.int32))


def make(variant, seed):
    return VectorDQNLearner(16, "cpu", variant=variant, batch_size=32, capacity=256,
                            hidden_dim=32, h_channels=8, target_every=3, updates_per_epoch=2,
                            t_max=5, seed=seed, use_graph=False, act_bf16=False)


@pytest.mark.parametrize("variant", ["dqn", "ddqn"])
def test_learner_resume_is_bit_exact(variant):
    A = make(variant, 1)
    fill(A, 200, 7)
    for _ in range(4):
        A.update(expand)
    A.steps_done += torch.arange(16, dtype=torch.float32)
    buf = io.BytesIO()
    torch.save(A.state_dict(), buf)
    buf.seek(0)
    sd = torch.load(buf, weights_only=True)
    fill(A, 70, 8)  # wraps the 256-row ring
    for _ in range(5):
        A.update(expand)

    B = make(variant, 2)  # other init, other dropout salts
    B.load_state_dict(sd)
    fill(B, 70, 8)
    for _ in range(5):
        B.update(expand)

    for (ka, pa), (kb, pb) in zip(A.source.state_dict().items(), B.source.state_dict().items()):
        assert ka == kb and torch.equal(pa, pb), ka
    for pa, pb in zip(A.target.parameters(), B.target.parameters()):
        assert torch.equal(pa, pb)
    assert A.n_updates == B.n_updates == 9
    assert (A.replay.ptr, A.replay.size) == (B.replay.ptr, B.replay.size) == (14, 256)
    assert torch.equal(A.replay.sw, B.replay.sw) and torch.equal(A.steps_done, B.steps_done)
    assert A.sched.get_last_lr() == B.sched.get_last_lr()
    sa, sb = A.opt.state_dict()["state"], B.opt.state_dict()["state"]
    for k in sa:
        assert torch.equal(sa[k]["exp_avg_sq"], sb[k]["exp_avg_sq"])


def test_learner_state_rejects_a_mismatch():
    A = make("dqn", 1)
    fill(A, 64, 3)
    sd = A.state_dict()
    with pytest.raises(ValueError):
        make("ddqn", 1).load_state_dict(sd)
    B = VectorDQNLearner(16, "cpu", variant="dqn", batch_size=32, capacity=512, hidden_dim=32,
                         h_channels=8, use_graph=False, act_bf16=False)
    with pytest.raises(ValueError):
        B.load_state_dict(sd)
