"""Fused acting stem (mz_q_front, csrc/mz_qnet.hip) and the fused Q / actor-critic forwards
(mazerl/agents/fused.py) against a plain PyTorch fp32 reference of the same ops:
Conv2d(3->32, 3x3, p1) -> LeakyReLU -> [Dropout] -> MaxPool2d(2) -> flatten || obs6
(agents/dqn_agent.py:19-57, ddqn_agent.py:18-52, ppo_agent.py ActorCriticNet).

Tolerances: the kernel rounds the conv weights to bf16 (what autocast does on the torch acting
path) and rounds each output once to bf16, so against an fp32 reference that uses the same
bf16-rounded weights every feature is within 1 bf16 ulp (rel 2^-7) + 1e-6. The obs6 columns are
bf16(obs6) exactly and the pad columns are exactly zero. Dropout masks come from the kernel's own
hash: checked through exact probe statistics (P(drop) = 13107/65536)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

P_DROP = 13107 / 65536


def _lib():
    from mazerl import _native as N
    return N, N.load()


def bits_to_window(bits):
    """[n, 22] int32 -> [n, 3, 15, 15] f32 (bit f of the 675-bit string = element f)."""
    b = bits.to(torch.int64) & 0xFFFFFFFF
    f = torch.arange(675, device=bits.device)
    w = (b[:, f // 32] >> (f % 32)) & 1
    return w.to(torch.float32).view(-1, 3, 15, 15)


def random_bits(n, gen):
    x = torch.randint(0, 2**31, (n, 22), generator=gen, dtype=torch.int64)
    x = x ^ (torch.randint(0, 2, (n, 22), generator=gen, dtype=torch.int64) << 31)
    x[:, 21] &= (1 << (675 - 21 * 32)) - 1   # bits past 675 are zero in mz_step's layout
    return x.to(torch.int32)


def front(bits, obs6, w, b, p=0.0, seed=0, counter=0, ld=1600):
    N, L = _lib()
    n = bits.shape[0]
    out = torch.full((n, ld), float("nan"), dtype=torch.bfloat16, device="cuda")
    N.check(L.mz_q_front(bits.data_ptr(), obs6.data_ptr(), n, w.data_ptr(), b.data_ptr(), p, seed,
                         counter, out.data_ptr(), ld, torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    return out


def reference(bits, obs6, w, b):
    """fp32 torch stem in the kernel's feature order (position-major, agents/fused.py)."""
    from mazerl.agents.fused import feature_perm
    win = bits_to_window(bits)
    y = F.conv2d(win, w.to(torch.bfloat16).float(), b, padding=1)
    y = F.max_pool2d(F.leaky_relu(y, 0.01), 2).flatten(1)
    return torch.cat((y[:, feature_perm(y.device)], obs6), 1)


@pytest.mark.parametrize("n,ld", [(1, 1600), (7, 1576), (1001, 1600), (4096, 1584)])
def test_front_matches_fp32(n, ld):
    g = torch.Generator().manual_seed(n)
    bits = random_bits(n, g).cuda()
    obs6 = (torch.randn(n, 6, generator=g) * 3).cuda()
    w = (torch.randn(32, 3, 3, 3, generator=g) * 0.4).cuda()
    b = (torch.randn(32, generator=g) * 0.2).cuda()
    out = front(bits, obs6, w, b, ld=ld).float()
    ref = reference(bits, obs6, w, b)
    got = out[:, :1568]
    err = (got - ref[:, :1568]).abs()
    tol = ref[:, :1568].abs() * 2.0 ** -7 + 1e-6
    assert bool((err <= tol).all()), float((err - tol).max())
    assert torch.equal(out[:, 1568:1574], obs6.to(torch.bfloat16).float())
    assert bool((out[:, 1574:] == 0).all())


def test_front_rejects_bad_stride():
    N, L = _lib()
    z = torch.zeros(4, 1600, dtype=torch.bfloat16, device="cuda")
    bits = torch.zeros(4, 22, dtype=torch.int32, device="cuda")
    o = torch.zeros(4, 6, device="cuda")
    w = torch.zeros(32 * 27, device="cuda")
    for ld in (1574, 1601, 1608):
        rc = L.mz_q_front(bits.data_ptr(), o.data_ptr(), 4, w.data_ptr(), w.data_ptr(), 0.0, 0, 0,
                          z.data_ptr(), ld, None)
        assert rc != 0


@pytest.mark.parametrize("bias", [0.5, -0.5])
def test_front_dropout_statistics(bias):
    n = 8192
    bits = random_bits(n, torch.Generator().manual_seed(5)).cuda()
    obs6 = torch.zeros(n, 6, device="cuda")
    w = torch.zeros(32, 3, 3, 3, device="cuda")
    b = torch.full((32,), bias, device="cuda")
    out = front(bits, obs6, w, b, p=0.2, seed=9, counter=3).float()[:, :1568]
    total = out.numel()
    kept_val = torch.tensor(1.25 * (bias if bias > 0 else 0.01 * bias)).to(torch.bfloat16).float().item()
    vals = set(torch.unique(out).tolist())
    assert vals <= {0.0, kept_val}
    if bias > 0:  # 0 only when all 4 positions of the pooling window are dropped
        expect = P_DROP ** 4
        frac = float((out == 0).sum()) / total
    else:         # a negative value survives only when all 4 are kept
        expect = (1 - P_DROP) ** 4
        frac = float((out != 0).sum()) / total
    sd = (expect * (1 - expect) / total) ** 0.5
    assert abs(frac - expect) < 5 * sd + 1e-9, (frac, expect)
    again = front(bits, obs6, w, b, p=0.2, seed=9, counter=3).float()[:, :1568]
    assert torch.equal(out, again)  # (seed, counter) fixes the masks
    other = front(bits, obs6, w, b, p=0.2, seed=9, counter=4).float()[:, :1568]
    assert not torch.equal(out, other)


def _net_inputs(n, seed):
    g = torch.Generator().manual_seed(seed)
    return random_bits(n, g).cuda(), (torch.randn(n, 6, generator=g)).cuda()


@pytest.mark.parametrize("variant", ["dqn", "ddqn"])
def test_fused_q_matches_torch(variant):
    from mazerl.agents.fused import FusedQ
    from mazerl.agents.nets import QNet
    torch.manual_seed(1)
    net = QNet(3, 6, 4, 32, 1024, variant).cuda().eval()  # dropout off for a value comparison
    bits, obs6 = _net_inputs(2048, 2)
    fq = FusedQ(net)
    q = fq(obs6, bits).float()
    with torch.no_grad():
        ref = net((obs6, bits_to_window(bits)))
    scale = float(ref.abs().max())
    assert float((q - ref).abs().max()) <= 0.03 * scale + 1e-3
    # parameters changed by an optimizer step are picked up (bf16 copies refreshed)
    with torch.no_grad():
        for p in net.parameters():
            p.mul_(1.5)
    q2 = fq(obs6, bits).float()
    with torch.no_grad():
        ref2 = net((obs6, bits_to_window(bits)))
    assert float((q2 - ref2).abs().max()) <= 0.03 * float(ref2.abs().max()) + 1e-3


def test_fused_actor_critic_matches_torch():
    from mazerl.agents.fused import FusedActorCritic
    from mazerl.agents.ppo import ActorCriticNet
    torch.manual_seed(3)
    net = ActorCriticNet(3, 6, 4, 32, 1024).cuda()
    bits, obs6 = _net_inputs(1500, 4)
    logits, value = FusedActorCritic(net)(obs6, bits)
    with torch.no_grad():
        rl, rv = net((obs6, bits_to_window(bits)))
    assert float((logits.float() - rl).abs().max()) <= 0.03 * float(rl.abs().max()) + 1e-3
    assert float((value.float() - rv).abs().max()) <= 0.03 * float(rv.abs().max()) + 1e-3


def test_trainer_runs_on_bits_only_env():
    """The DDQN trainer on an env that writes no f32 window: acting reads the bits."""
    from mazerl import VectorMazeEnv
    from mazerl.agents.dqn import VectorDQNLearner
    from mazerl.trainers.vector_trainer import VectorOffPolicyTrainer, evaluate
    env = VectorMazeEnv(512, 21, enrich=True, device="cuda", seed=77, window=False,
                        window_bits=True, done_list=False)
    assert env.window is None
    L = VectorDQNLearner(512, "cuda", variant="ddqn", batch_size=64, capacity=20000,
                         updates_per_step=1)
    assert L.supports_bits
    tr = VectorOffPolicyTrainer(env, L, seed=1)
    tr.train(12)
    assert L.n_updates > 0 and np.isfinite(float(L.last_loss))
    rate, k = evaluate(L, 64, 21, seed=5, device="cuda", max_vector_steps=50)
    assert 0.0 <= rate <= 1.0 and k <= 50
    env.close()
