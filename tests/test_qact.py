"""The f32-accurate acting forward (agents/qact.py QAct, csrc/mz_qact.hip: conv stem inside fc1's
K loop, every GEMM operand split into bf16 hi + lo, three MFMA products per tile) against the f32
Q-network (dqn_agent.py:19-57 / ddqn_agent.py:18-52, its f32 HIP stem + f32 GEMMs — pinned to
the torch conv by tests/test_stem.py).

Tolerance: |Q - Q_f32| <= 2e-4 x max|Q_f32| per row (bf16x3 is ~2^-16 relative per product; the
f32 reference itself sums in another order); argmax identical wherever the f32 top-2 gap exceeds
1e-3 x max|Q|, and on >= 99.9 % of all rows."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _states(B, dim=41, steps=9, seed=3):
    from mazerl import VectorMazeEnv
    env = VectorMazeEnv(B, dim, enrich=True, device="cuda", seed=seed, window=False,
                        window_bits=True)
    for k in range(steps):  # visited cells in the windows
        env.step_act(eps=1.0, seed=seed, counter=k)
        env.reset_done()
    obs6, bits = env.obs6.clone(), env.window_bits.clone()
    env.close()
    return obs6, bits


def _check(q, q32):
    scale = q32.abs().amax(1).clamp_min(1e-30)
    err = ((q - q32).abs().amax(1) / scale)
    assert float(err.max()) <= 2e-4, float(err.max())
    top2 = q32.topk(2, dim=1).values
    clear = (top2[:, 0] - top2[:, 1]) / scale > 1e-3
    a, a32 = q.argmax(1), q32.argmax(1)
    assert torch.equal(a[clear], a32[clear])
    assert float((a == a32).float().mean()) >= 0.999


@pytest.mark.parametrize("variant", ["ddqn", "dqn"])
def test_qact_matches_f32_qnet(variant):
    from mazerl.agents.nets import QNet
    from mazerl.agents.qact import QAct
    torch.manual_seed(11)
    net = QNet(variant=variant).cuda().eval()  # dropout off: the f32 net's exact function
    for p in net.parameters():  # weights of a trained net's scale
        p.data.mul_(3.0)
    obs6, bits = _states(3000)
    qa = QAct(net)
    q = qa(obs6, bits)
    g = qa.greedy(obs6, bits)
    with torch.no_grad():
        q32 = net((obs6, bits))
    torch.cuda.synchronize()
    _check(q, q32)
    assert torch.equal(g, q.argmax(1))


def test_qact_rows_sized_on_the_device():
    """rows_greedy: only rows[:count] (count read on the device) are evaluated and scattered to
    their instances; every other greedy entry keeps its value; a weight change needs
    invalidate() (graph-replayed optimizers leave _version alone)."""
    from mazerl.agents.nets import QNet
    from mazerl.agents.qact import QAct
    torch.manual_seed(12)
    net = QNet(variant="dqn").cuda()
    obs6, bits = _states(5000, dim=81, seed=7)
    B = bits.shape[0]
    rows = torch.randperm(B, device="cuda")[:1700].to(torch.int32).contiguous()
    count = torch.tensor([1234], dtype=torch.int32, device="cuda")
    qa = QAct(net)
    greedy = torch.full((B,), -7, dtype=torch.int64, device="cuda")
    qout = torch.full((1700, 4), float("nan"), device="cuda")
    qa.rows_greedy(obs6, bits, rows, count, greedy, qout)
    with torch.no_grad():
        q32 = net((obs6, bits))
    torch.cuda.synchronize()
    lst = rows[:1234].long()
    _check(qout[:1234], q32[lst])
    assert torch.equal(greedy[lst], qout[:1234].argmax(1))
    others = torch.ones(B, dtype=torch.bool, device="cuda")
    others[lst] = False
    assert bool((greedy[others] == -7).all()) and bool(torch.isnan(qout[1234:]).all())
    with torch.no_grad():
        for p in net.parameters():
            p.add_(0.01)
    qa.invalidate()
    q2 = qa(obs6, bits)
    with torch.no_grad():
        _check(q2, net((obs6, bits)))


def _lowbias32(x):
    x = x.astype(np.uint64) & 0xFFFFFFFF
    x ^= x >> 16
    x = (x * 0x7FEB352D) & 0xFFFFFFFF
    x ^= x >> 15
    x = (x * 0x846CA68B) & 0xFFFFFFFF
    x ^= x >> 16
    return x


def test_qact_ddqn_dropout_masks():
    """DDQN acts in train mode (Dropout(0.2) after the conv activation): the
    kernel's keep decisions are a counter hash of (seed, counter, row, channel pair, pooled
    position) feeding a 4-draw xorshift32 stream per 2x2 window;
    rebuilt here, applied to the f32 torch stem (conv -> LeakyReLU -> mask * 1/(1-p) -> MaxPool)
    the Q values agree to the same tolerance, and P(drop) = 13107/65536."""
    from mazerl.agents.nets import QNet
    from mazerl.agents.qact import QAct
    from test_stem import _window
    torch.manual_seed(13)
    net = QNet(variant="ddqn").cuda().train()
    obs6, bits = _states(600, dim=21, seed=9)
    n = bits.shape[0]
    qa = QAct(net, seed=77)
    q = qa(obs6, bits)  # counter 0
    k = (77 * 0x9E3779B97F4A7C15 + 0 * 0xD1B54A32D192ED03 + 1) & (2**64 - 1)
    key = np.uint64((k ^ (k >> 32)) & 0xFFFFFFFF)
    rkey = _lowbias32(key ^ _lowbias32(np.arange(n, dtype=np.uint64)))  # [n]
    # per (row, channel pair, pooled position) one xorshift32 stream of 4 draws, seeded from the
    # (row, pair) base and the position: draw r (= 2 dy + dx) -> low half: even channel, high
    # half: odd channel
    base = _lowbias32(rkey[:, None] ^ np.arange(16, dtype=np.uint64)[None]) | 1  # [n, 16]
    keep = np.zeros((n, 49, 32, 2, 2), bool)
    for qi in range(49):
        st = _lowbias32(base ^ np.uint64((qi * 0x9E3779B9) & 0xFFFFFFFF)) | 1
        for r in range(4):
            st ^= (st << 13) & 0xFFFFFFFF
            st ^= st >> 17
            st ^= (st << 5) & 0xFFFFFFFF
            keep[:, qi, 0::2, r >> 1, r & 1] = (st & 0xFFFF) >= 13107
            keep[:, qi, 1::2, r >> 1, r & 1] = (st >> 16) >= 13107
    assert abs(1 - keep.mean() - 13107 / 65536) < 0.002
    m = np.zeros((n, 32, 15, 15), np.float32)
    qy, qx = np.arange(49) // 7, np.arange(49) % 7
    kk = keep.transpose(0, 2, 1, 3, 4)  # [n, c, q, dy, dx]
    for qi in range(49):
        y, x = 2 * qy[qi], 2 * qx[qi]
        m[:, :, y:y + 2, x:x + 2] = kk[:, :, qi]
    mask = torch.from_numpy(m).cuda()
    conv = net.conv[0]
    with torch.no_grad():
        a = F.leaky_relu(F.conv2d(_window(bits.cpu()).cuda(), conv.weight, conv.bias, padding=1))
        a = a * mask * (1.0 / (1.0 - 0.2))
        feat = torch.cat((F.max_pool2d(a, 2, 2).flatten(1), obs6), 1)
        q32 = net.fc(feat)
    torch.cuda.synchronize()
    _check(q, q32)


def test_trainer_acts_without_waiting_for_the_row_count():
    """The DDQN trainer's acting path (greedy-row list + QAct) never reads the list's length on
    the host: GreedyRows.select (the stream wait) is not called over several vector steps."""
    from mazerl import VectorMazeEnv
    from mazerl.agents import fused
    from mazerl.agents.dqn import VectorDQNLearner
    from mazerl.trainers.vector_trainer import VectorOffPolicyTrainer
    B = 4096
    env = VectorMazeEnv(B, 21, enrich=True, device="cuda", seed=5, done_list=False,
                        window=False, window_bits=True)
    L = VectorDQNLearner(B, "cuda:0", variant="ddqn", batch_size=256, capacity=1 << 16,
                         eps_decay=50.0, overlap=True)
    tr = VectorOffPolicyTrainer(env, L, seed=3)
    orig = fused.GreedyRows.select

    def boom(self, *a, **k):
        raise AssertionError("host wait for the greedy-row count")
    fused.GreedyRows.select = boom
    try:
        tr.train(12)
    finally:
        fused.GreedyRows.select = orig
    torch.cuda.synchronize()
    assert 0 < int(L._rows.count[0]) <= B
    assert int((env.actions < 0).sum()) == 0 and int((env.actions > 3).sum()) == 0
    env.close()
