"""DQN / DDQN learners.

q_loss()            the Q-learning loss of DQNAgent.optimize_model (agents/dqn_agent.py:121-157)
                    and DDQNAgent.optimize_model (agents/ddqn_agent.py:113-152), term for term:
                    Q(s,a) = source(s).gather(a); target = r + gamma * V(s'), V = max_a' target(s')
                    (DQN) or target(s')[argmax source(s')] (DDQN); NO terminal masking — the
                    reference never stores None next states, so terminal transitions bootstrap
                    (SURVEY Q12); mse_loss(mean). Network calls happen in the reference's order
                    (source(s), [source(s')], target(s')) so dropout draws line up on CPU.
learner_update()    backward, grad.clamp_(-1, 1) on every parameter, optimizer.step().
DQNAgent/DDQNAgent  single-env drop-ins with the reference constructor and methods
                    (get_action/memorize/optimize_model/scheduler_step/has_to_update/
                    update_target/update_steps_done/update_hyperparameter/calculate_epsilon).
VectorDQNLearner    the MI355X learner for VectorMazeEnv: device replay (HBM), batched fused
                    act, K updates per vector step, optional DDP gradient all-reduce (RCCL) with
                    the clamp applied after averaging (single-GPU semantics).
"""
import collections
import copy
import math
import os
import random

import numpy as np
import torch
import torch.nn.functional as F
import torch.optim as optim
from torch.optim import lr_scheduler

from ..replay import ReplayMemory, Transition
from .flat import copy_flat
from .nets import QNet


STACK_ROWS = True  # DDQN on packed windows (GPU): source(s) and source(s') as one pass
# the overlapped learner's K updates of a vector step as one graph replay (MZ_K_BLOCK=0: K replays;
# bit-identical results either way, tests/test_determinism_gpu.py)
K_BLOCK = os.environ.get("MZ_K_BLOCK", "1") != "0"
# data-parallel learner: the gradient collectives captured inside the update graph (one replay:
# backward, reduce-scatter, shard AdamW, all-gather; thread-local capture mode) instead of issued
# from the host between two replays. MZ_GRAPH_COLLECTIVES=1 (or graph_collectives=True) turns it on.
GRAPH_COLLECTIVES = os.environ.get("MZ_GRAPH_COLLECTIVES", "0") == "1"
# GPU: the loss and its gradient w.r.t. the Q rows as two HIP launches (MZ_FUSED_LOSS=0: torch ops)
FUSED_LOSS = os.environ.get("MZ_FUSED_LOSS", "1") != "0"
# GPU: both nets' second activation + fc3 + the loss as one launch, its backward through fc3 and
# the activation as one launch + a column sum (MZ_FUSED_HEAD=0: the Q rows, then FUSED_LOSS)
FUSED_HEAD = os.environ.get("MZ_FUSED_HEAD", "1") != "0"


class _QLossFn(torch.autograd.Function):
    """mse_loss(Q(s,a), V(s') * gamma + r) from the nets' output rows (mz_q_loss /
    mz_q_loss_backward): q [rows, 4] (rows >= b: DDQN's stacked s' rows, zero gradient),
    q_next [b, 4] (DDQN's argmax rows) or None (DQN: max of q_tgt), q_tgt [b, 4]."""

    @staticmethod
    def forward(ctx, q, q_next, q_tgt, action, reward, gamma, b):
        from .. import _native as N
        dev = q.device
        loss = torch.empty((), dtype=torch.float32, device=dev)
        diff = torch.empty(b, dtype=torch.float32, device=dev)
        N.check(N.load().mz_q_loss(
            q.data_ptr(), q.stride(0), q_next.data_ptr() if q_next is not None else None,
            q_next.stride(0) if q_next is not None else 0, q_tgt.data_ptr(), q_tgt.stride(0),
            action.data_ptr(), reward.data_ptr(), float(gamma), b, loss.data_ptr(), diff.data_ptr(),
            torch.cuda.current_stream(dev).cuda_stream))
        ctx.save_for_backward(diff, action)
        ctx.rows, ctx.b = q.shape[0], b
        return loss

    @staticmethod
    def backward(ctx, g):
        from .. import _native as N
        diff, action = ctx.saved_tensors
        g = g.contiguous()
        dq = torch.empty(ctx.rows, 4, dtype=torch.float32, device=diff.device)
        N.check(N.load().mz_q_loss_backward(g.data_ptr(), diff.data_ptr(), action.data_ptr(), ctx.b,
                                            ctx.rows, dq.data_ptr(),
                                            torch.cuda.current_stream(diff.device).cuda_stream))
        return dq, None, None, None, None, None, None


class _HeadLossFn(torch.autograd.Function):
    """mse_loss(Q(s,a), V(s') * gamma + r) from the second hidden layer's pre-activations z2 of
    the source rows (DDQN: the stacked [s; s'] rows) and of the target's s' rows, through the
    activation and fc3 (mz_head_loss / mz_head_loss_backward): one launch forward, one launch +
    one column sum backward — instead of both nets' activation and fc3 launches, the loss, its
    backward, fc3's two GEMMs and bias sum and the activation's backward. Gradients: z2 rows < b
    (the rest are left unwritten, the forward_rows contract), fc3's weight and bias (written into
    their flat gradient segments when the net has them, agents/flat.py)."""

    @staticmethod
    def forward(ctx, z2s, w3s, b3s, z2t, w3t, b3t, action, reward, gamma, b, act, stacked, ticket):
        from .. import _native as N
        L = N.load()
        dev = z2s.device
        H = z2s.shape[1]
        loss = torch.empty((), dtype=torch.float32, device=dev)
        diff = torch.empty(b, dtype=torch.float32, device=dev)
        part = torch.empty(max(1, L.mz_head_loss_workspace_floats(b)), dtype=torch.float32, device=dev)
        N.check(L.mz_head_loss(z2s.data_ptr(), z2s.stride(0), w3s.data_ptr(), b3s.data_ptr(),
                               z2t.data_ptr(), z2t.stride(0), w3t.data_ptr(), b3t.data_ptr(), H,
                               act, int(stacked), action.data_ptr(), reward.data_ptr(), float(gamma),
                               b, part.data_ptr(), ticket.data_ptr(), loss.data_ptr(),
                               diff.data_ptr(), torch.cuda.current_stream(dev).cuda_stream))
        ctx.save_for_backward(z2s, w3s, diff, action)
        ctx.b, ctx.act, ctx.H = b, act, H
        ctx.wp, ctx.bp = w3s, b3s
        return loss

    @staticmethod
    def backward(ctx, g):
        from .. import _native as N
        from .flat import grad_segment
        L = N.load()
        z2s, w3s, diff, action = ctx.saved_tensors
        dev, b, H = z2s.device, ctx.b, ctx.H
        st = torch.cuda.current_stream(dev).cuda_stream
        g = g.contiguous()
        dz2 = torch.empty(z2s.shape, dtype=torch.float32, device=dev)
        nblk = L.mz_head_loss_backward_workspace_floats(b, H) // (4 * H + 4)
        part = torch.empty(nblk, 4 * H + 4, dtype=torch.float32, device=dev)
        N.check(L.mz_head_loss_backward(g.data_ptr(), diff.data_ptr(), action.data_ptr(), b,
                                        z2s.data_ptr(), z2s.stride(0), w3s.data_ptr(), H, ctx.act,
                                        dz2.data_ptr(), dz2.stride(0), part.data_ptr(), st))
        gw, gb = grad_segment(ctx.wp), grad_segment(ctx.bp)
        # [dW3 | db3] as one column sum when the two flat segments are adjacent (fc3's bias
        # follows its weight in the flat layout), else into a fresh row
        if gw is not None and gb is not None and gb.data_ptr() == gw.data_ptr() + 4 * 4 * H:
            out = gw.view(-1)
            N.check(L.mz_colsum_f32(part.data_ptr(), nblk, 4 * H + 4, 4 * H + 4, out.data_ptr(), st))
        else:
            row = torch.empty(4 * H + 4, dtype=torch.float32, device=dev)
            N.check(L.mz_colsum_f32(part.data_ptr(), nblk, 4 * H + 4, 4 * H + 4, row.data_ptr(), st))
            gw = row[:4 * H].view(4, H) if gw is None else gw.copy_(row[:4 * H].view(4, H))
            gb = row[4 * H:] if gb is None else gb.copy_(row[4 * H:])
        ctx.wp = ctx.bp = None
        return dz2, gw, gb, None, None, None, None, None, None, None, None, None, None


def _head_ticket(net, dev):
    """The mz_head_loss ticket of this source net (one per learner: two learners' updates may run
    at once on their own side streams, and a shared ticket would mix their workgroup counts)."""
    t = getattr(net, "_head_ticket", None)
    if t is None or t.device != dev:
        t = torch.zeros(1, dtype=torch.int32, device=dev)
        net._head_ticket = t
    return t


def _head_ok(source, target, state, action, reward):
    from .linear import GraphSafeLinear
    if not (FUSED_HEAD and FUSED_LOSS and state[1].is_cuda and state[1].dtype == torch.int32
            and hasattr(source, "trunk") and hasattr(target, "trunk")):
        return False
    fc3 = source.fc[4]
    return (isinstance(fc3, GraphSafeLinear) and fc3.out_features == 4 and fc3.bias is not None
            and fc3.in_features % 4 == 0 and action.dtype == torch.int64 and action.is_contiguous()
            and reward.dtype == torch.float32 and reward.is_contiguous()
            and torch.is_grad_enabled() and fc3.weight.requires_grad)


def _fused_ok(q, action, reward, *others):
    return (FUSED_LOSS and q.is_cuda and q.dtype == torch.float32 and q.dim() == 2 and
            q.shape[1] == 4 and q.stride(1) == 1 and action.dtype == torch.int64 and
            action.is_contiguous() and reward.dtype == torch.float32 and reward.is_contiguous() and
            all(t is None or (t.dtype == torch.float32 and t.stride(1) == 1 and t.shape[1] == 4)
                for t in others))


def _stacked(x, y):
    """[x; y] — without a copy when x and y are the two halves of one buffer (the layout
    DeviceReplay.sample gathers into)."""
    base = x._base
    if base is not None and y._base is base and base.is_contiguous() and \
            base.shape[0] == x.shape[0] + y.shape[0] and x.data_ptr() == base.data_ptr() and \
            y.data_ptr() == base.data_ptr() + x.numel() * x.element_size():
        return base
    return torch.cat((x, y))


def q_loss(source, target, state, action, reward, next_state, gamma, double):
    """Loss of optimize_model for a batch: state = (obs6 [B,6], window [B,3,15,15] f32 or packed
    int32 [B,22] on the GPU — QNet then runs the HIP stem). DDQN on the GPU evaluates source(s)
    and source(s') as ONE pass over the 2B stacked rows (QNet.forward_rows: the stem and GEMMs
    at twice the rows; the backward reads the first B rows only — the s' rows feed an argmax,
    which the reference computes under no_grad)."""
    q_next = None
    if (not double or STACK_ROWS) and _head_ok(source, target, state, action, reward):
        # the trunks (stem -> fc1 -> act -> fc2), then one head + loss launch for both nets
        act = 1 if source.variant == "ddqn" else 0
        b = action.shape[0]
        if double and STACK_ROWS:
            z2 = source.trunk((_stacked(state[0], next_state[0]),
                               _stacked(state[1], next_state[1])), b)
        else:
            z2 = source.trunk(state)
        with torch.no_grad():
            z2t = target.trunk(next_state)
        f3s, f3t = source.fc[4], target.fc[4]
        return _HeadLossFn.apply(z2, f3s.weight, f3s.bias, z2t, f3t.weight, f3t.bias, action,
                                 reward, gamma, b, act, bool(double), _head_ticket(source, z2.device))
    if double and STACK_ROWS and hasattr(source, "forward_rows") and state[1].is_cuda \
            and state[1].dtype == torch.int32:
        b = action.shape[0]
        # (the target's stem on a second stream beside this pass measured slower: 732 vs 690 us
        # per update, profiles/r01k_update_target_stem_side_stream.json)
        q = source.forward_rows((_stacked(state[0], next_state[0]),
                                 _stacked(state[1], next_state[1])), b)
        q_next = q[b:].detach()
        if q.shape[0] == 2 * b and _fused_ok(q, action, reward, q_next):
            with torch.no_grad():
                q_t = target(next_state)
            if _fused_ok(q, action, reward, q_t):
                return _QLossFn.apply(q, q_next, q_t.float().contiguous(), action, reward, gamma, b)
            q_sa = q[:b].gather(1, action.view(-1, 1))
            v_next = q_t.gather(1, q_next.max(1)[1].unsqueeze(1)).squeeze(1)
            return F.mse_loss(q_sa, ((v_next * gamma) + reward).unsqueeze(1))
        q_sa = q[:b].gather(1, action.view(-1, 1))
    elif not double and state[1].is_cuda:
        q = source(state)
        if _fused_ok(q, action, reward):
            with torch.no_grad():
                q_t = target(next_state)
            if _fused_ok(q, action, reward, q_t):
                return _QLossFn.apply(q, None, q_t.contiguous(), action, reward, gamma, q.shape[0])
            return F.mse_loss(q.gather(1, action.view(-1, 1)),
                              ((q_t.max(1)[0] * gamma) + reward).unsqueeze(1))
        q_sa = q.gather(1, action.view(-1, 1))
    else:
        q_sa = source(state).gather(1, action.view(-1, 1))
    with torch.no_grad():  # the reference detaches V(s'); no graph is built for it here
        if double:
            if q_next is None:
                q_next = source(next_state)
            best = q_next.max(1)[1].unsqueeze(1)
            v_next = target(next_state).gather(1, best).squeeze(1).detach()
        else:
            v_next = target(next_state).max(1)[0].detach()
    expected = (v_next * gamma) + reward
    return F.mse_loss(q_sa, expected.unsqueeze(1))


_ONES = {}


def learner_backward(optimizer, loss):
    optimizer.zero_grad()
    # a persistent dL/dL = 1 (loss.backward() fills a fresh one: one more launch per update)
    key = (loss.device, loss.dtype)
    one = _ONES.get(key)
    if one is None:
        one = _ONES[key] = torch.ones((), dtype=loss.dtype, device=loss.device)
    loss.backward(gradient=one)


def learner_step(net, optimizer, clamp=1.0):
    if hasattr(optimizer, "exp_avg_sq"):  # FlatAdamW: the clamp runs inside its one launch
        optimizer.clamp = float(clamp)
        optimizer.step()
        return
    grads = [p.grad for p in net.parameters() if p.grad is not None]
    torch._foreach_clamp_min_(grads, -clamp)  # == p.grad.data.clamp_(-1, 1) per parameter
    torch._foreach_clamp_max_(grads, clamp)   # (dqn_agent.py:155-156), two launches in total
    optimizer.step()


def learner_update(net, optimizer, loss, clamp=1.0, allreduce=None):
    learner_backward(optimizer, loss)
    if allreduce is not None:
        allreduce(net)  # average grads over ranks, then clamp (single-GPU semantics)
    learner_step(net, optimizer, clamp)
    if allreduce is not None and hasattr(allreduce, "finish"):
        allreduce.finish(net)  # sharded step: the updated parameter shards to every rank


class _AgentBase:
    VARIANT = "dqn"
    T_MAX = 100

    def __init__(self, env, learning_rate, starting_epsilon, final_epsilon, epsilon_decay,
                 discount_factor, eta, batch_size, memory_size, target_update_frequency, device,
                 hidden_dim=1024, h_channels=32):
        self.env = env
        self.device = device
        self.learning_rate = learning_rate
        self.starting_epsilon = starting_epsilon
        self.final_epsilon = final_epsilon
        self.epsilon_decay = epsilon_decay
        self.discount_factor = discount_factor
        self.batch_size = batch_size
        self.target_update_frequency = target_update_frequency
        self.eta = eta
        n_actions = env.action_space.n
        observation, _ = env.reset()
        n_obs = len(np.concatenate([observation[k] for k in observation if k != "window"]))
        self.source_net = QNet(3, n_obs, n_actions, h_channels, hidden_dim, self.VARIANT).to(device)
        self.target_net = QNet(3, n_obs, n_actions, h_channels, hidden_dim, self.VARIANT).to(device)
        self.memory = ReplayMemory(memory_size)
        self.optimizer = optim.AdamW(self.source_net.parameters(), learning_rate)
        self.lr_scheduler = lr_scheduler.CosineAnnealingLR(self.optimizer, T_max=self.T_MAX, eta_min=1e-5)
        self.steps_done = 0

    def memorize(self, *args):
        self.memory.push(*args)

    def calculate_epsilon(self):
        return self.final_epsilon + (self.starting_epsilon - self.final_epsilon) * \
            math.exp(-1. * self.steps_done / self.epsilon_decay)

    def get_action(self, state):
        sample = random.random()
        eps = self.calculate_epsilon()
        self.steps_done += 1
        if sample < eps:
            mask_dir = self.env.env.get_mask_direction(probs=True)
            ps = mask_dir / mask_dir.sum()
            return torch.tensor(np.random.choice(len(ps), p=ps), device=self.device, dtype=torch.long)
        with torch.no_grad():
            return self.source_net(state).max(1)[1].view(1, 1)

    def optimize_model(self):
        if len(self.memory) < self.batch_size:
            return
        transitions = self.memory.sample(self.batch_size)
        batch = Transition(*zip(*transitions))
        next_states = (torch.cat([s[0] for s in batch.next_state]), torch.cat([s[1] for s in batch.next_state]))
        state_batch = (torch.cat([s[0] for s in batch.state]), torch.cat([s[1] for s in batch.state], dim=0))
        device = state_batch[0].device
        action_batch = torch.tensor(batch.action).to(device)
        reward_batch = torch.tensor(batch.reward).to(device)
        loss = q_loss(self.source_net, self.target_net, state_batch, action_batch, reward_batch,
                      next_states, self.discount_factor, self.VARIANT == "ddqn")
        ret = loss.item()
        learner_update(self.source_net, self.optimizer, loss)
        return ret

    def scheduler_step(self):
        self.lr_scheduler.step()

    def has_to_update(self, episode):
        return episode % self.target_update_frequency == 0

    def update_target(self):
        self.target_net.load_state_dict(self.source_net.state_dict())

    def update_steps_done(self):
        self.steps_done = 0

    def update_hyperparameter(self, is_better):
        self.discount_factor = self.discount_factor + (self.eta if is_better else -self.eta)


class DQNAgent(_AgentBase):
    VARIANT, T_MAX = "dqn", 100       # dqn_agent.py:98


class DDQNAgent(_AgentBase):
    VARIANT, T_MAX = "ddqn", 150      # ddqn_agent.py:270


# ---------------------------------------------------------------------------------------------
class VectorDQNLearner:
    """Batched DQN/DDQN learner on one GPU (optionally one DDP rank).

    Defaults follow the reference's DDQN script (training_examples/.../test_ddqn.py:20-35):
    lr 1e-3, eps 0.95 -> 0.1, decay ((N-1)^2 // 2) * 5, gamma 0.7, batch 128, AdamW, cosine LR.
    Vectorisation policy (documented deviations): epsilon is per instance
    (steps_done per instance, reset to 0 on that instance's win, off_policy_trainer.py:192);
    gamma drift (Q15) is off by default; the cosine schedule and the target sync advance per
    `updates_per_epoch` updates instead of per episode; K updates per vector step.
    """

    def __init__(self, num_envs, device, variant="ddqn", lr=1e-3, eps_start=0.95, eps_final=0.1,
                 eps_decay=8000.0, gamma=0.7, batch_size=128, capacity=1_000_000,
                 updates_per_step=1, target_every=100, hidden_dim=1024, h_channels=32,
                 act_bf16=True, t_max=150, updates_per_epoch=100, allreduce=None, seed=0,
                 use_graph=True, bit_stem=True, overlap=False, greedy_rows=True, acting="x3",
                 graph_collectives=None):
        self.device = torch.device(device)
        if self.device.type == "cuda":  # the tuned f32 GEMM choices (gemm_tuning.py)
            from ..gemm_tuning import enable as _tuned_gemms
            _tuned_gemms(self.device)
        torch.manual_seed(seed)
        self.variant = variant
        self.source = QNet(3, 6, 4, h_channels, hidden_dim, variant).to(self.device)
        self.target = QNet(3, 6, 4, h_channels, hidden_dim, variant).to(self.device)
        self.target.load_state_dict(self.source.state_dict())
        if variant == "ddqn" and self.device.type == "cuda" and bit_stem and \
                os.environ.get("MZ_STEM_COUNTER_FOLD", "1") != "0":
            # one dropout counter for both nets' HIP stems: read by source(s, s') and target(s')
            # in an update, moved on by the source stem's backward (agents/stem.py) — the keys
            # each net draws are the 0, 1, 2, ... per update they were with an add per forward,
            # without the two add launches
            ctr = torch.zeros(1, dtype=torch.int64, device=self.device)
            self.source._stem_rng, self.target._stem_rng = ctr, ctr
            self.source._stem_advance, self.target._stem_advance = "backward", "none"
        # One update (sample -> expand -> loss -> backward -> clamp -> AdamW) is ~150 small
        # kernels: it is captured once into a HIP graph and replayed (capturable AdamW with a
        # device-side lr, so the cosine schedule still applies). With a gradient all-reduce
        # (N ranks) it is two graphs, backward + pack and unpack + clamp + AdamW, with the one
        # RCCL all-reduce of the flat bucket launched between the replays.
        self.use_graph = bool(use_graph) and self.device.type == "cuda"
        # with an all-reduce: the collectives inside the one update graph (GRAPH_COLLECTIVES)
        gc = GRAPH_COLLECTIVES if graph_collectives is None else bool(graph_collectives)
        self.graph_collectives = gc and self.use_graph and allreduce is not None
        # the update's nets read the replay's packed windows through the HIP f32 stem
        # (agents/stem.py) instead of expanding them to f32 for MIOpen
        self.bit_stem = bool(bit_stem) and self.device.type == "cuda"
        if self.use_graph:
            # one flat buffer per net: clamp + AdamW in one launch, whole-net copies in one
            from .flat import FlatAdamW, flatten_grads, flatten_params
            flatten_params(self.target)
            # the clamped gradient is not read after the step: not written back (8.56 MB)
            self.opt = FlatAdamW(self.source, lr, write_grad=False)
            # gradients written by the backward kernels into one flat buffer: one contiguous
            # AdamW read, and an all-reduce in place with no pack / unpack copies
            flatten_grads(self.source)
        else:
            self.opt = optim.AdamW(self.source.parameters(), lr)
        self._graph = None
        self._graph_loss = None
        self._graphK = [None, None]  # K-update graphs of the overlapped learner, per index slot
        self._graphK_loss = [None, None]
        self._eager_updates = 0
        self.sched = lr_scheduler.CosineAnnealingLR(self.opt, T_max=t_max, eta_min=1e-5)
        from ..replay import DeviceReplay
        self.replay = DeviceReplay(capacity, self.device)
        self.gamma, self.batch_size = gamma, batch_size
        self.eps_start, self.eps_final, self.eps_decay = eps_start, eps_final, eps_decay
        self.updates_per_step, self.target_every = updates_per_step, target_every
        self.updates_per_epoch = updates_per_epoch
        self.act_bf16 = act_bf16
        self.allreduce = allreduce
        if allreduce is not None and hasattr(allreduce, "attach"):
            # reduce-scatter + AdamW over this rank's shard + all-gather (distributed.py)
            allreduce.attach(self.source, self.opt)
        self.steps_done = torch.zeros(num_envs, dtype=torch.float32, device=self.device)
        self.n_updates = 0
        self.last_loss = torch.zeros((), device=self.device)
        self.fused = None
        # acting forward over the rows that act greedily only (agents/fused.py GreedyRows)
        self.greedy_rows = bool(greedy_rows)
        self._rows = None
        # the acting head on the GPU: "x3" = QAct (f32-accurate bf16x3 MFMA, sized on the device:
        # no host round trip per vector step); "bf16" = FusedQ (bf16 stem + hipBLASLt bf16 GEMMs)
        if acting not in ("x3", "bf16"):
            raise ValueError(f"acting {acting!r}: 'x3' or 'bf16'")
        self.acting = acting
        if self.device.type == "cuda" and act_bf16:
            self.fused = self._head(self.source, seed)
        # env -> learner handoff on a side HIP stream (north_star): the updates of vector step t
        # run on `side` while the main stream acts and steps the env for t + 1 (see update()).
        self.overlap = bool(overlap) and self.use_graph and self.fused is not None
        self._async = False
        if self.overlap:
            # MZ_LEARNER_PRIORITY: the side stream's priority (default: torch's default, 0)
            self.side = torch.cuda.Stream(self.device,
                                          priority=int(os.environ.get("MZ_LEARNER_PRIORITY", "0")))
            # two actor snapshots of the source net (ping-pong) with their own fused heads and
            # dropout streams; the source net itself is only touched on `side`
            from .flat import flatten_params
            self.actors = [copy.deepcopy(self.source) for _ in range(2)]
            for a in self.actors:
                flatten_params(a)
            self.actor_fused = [self._head(a, seed * 2 + 101 + k) for k, a in enumerate(self.actors)]
            self._published = collections.deque()  # (slot, event) of issued snapshots, oldest first
            self._acting = None  # slot greedy() reads
            self._idx = None     # [2][K, batch] sample indices, written on the main stream
            self._par = 0
            self._sample_seed = 0x5A3B1E + 7919 * int(seed)
            self._sample_counter = 0

    def _head(self, net, seed):
        if self.acting == "x3":
            from .qact import QAct
            return QAct(net, seed=seed)
        from .fused import FusedQ
        return FusedQ(net, seed=seed)

    @property
    def supports_bits(self):
        return self.fused is not None

    def epsilon(self):
        return self.eps_final + (self.eps_start - self.eps_final) * torch.exp(-self.steps_done / self.eps_decay)

    @torch.no_grad()
    def greedy(self, obs6, window, bits=None, act=None):
        """argmax_a Q_source(s) for every instance. With packed window bits on the GPU the acting
        forward is the fused HIP stem + bf16 GEMMs (agents/fused.py); otherwise torch.
        act = (eps, seed, counter) of the fused act that will read the result: then only the
        rows that act greedily are evaluated (dqn_agent.py:104-116 calls source_net only when
        `sample >= eps`); the other entries are stale and unread."""
        if bits is not None and self.fused is not None:
            f = self.actor_fused[self._acting_slot()] if self._async else self.fused
            if act is not None and self.greedy_rows:
                if self._rows is None:
                    from .fused import GreedyRows
                    self._rows = GreedyRows(bits.shape[0], self.device)
                return self._rows(f, obs6, bits, *act)
            if hasattr(f, "greedy"):
                return f.greedy(obs6, bits)
            return f(obs6, bits).float().argmax(1)
        if window is None:
            raise ValueError("greedy() needs the f32 window or window bits on the GPU")
        if self.act_bf16 and self.device.type == "cuda":
            with torch.autocast("cuda", dtype=torch.bfloat16):
                q = self.source((obs6, window))
        else:
            q = self.source((obs6, window))
        return q.float().argmax(1)

    def tick(self, term, trunc, wins, episodes, seed, counter):
        """The trainer's per-step bookkeeping in one HIP launch pair (mz_trainer_tick):
        steps_done += 1 / = 0 on a win, wins / episodes counters, the next act's epsilon (returned)
        and its greedy-row list, issued so that its count reaches the host while the stream runs
        the work behind it. None when this learner acts without the row list (the trainer then
        does the bookkeeping with torch)."""
        if self.fused is None or not self.greedy_rows:
            return None
        if self._rows is None:
            from .fused import GreedyRows
            self._rows = GreedyRows(self.steps_done.numel(), self.device)
        return self._rows.tick(term, trunc, self.steps_done, self.eps_start, self.eps_final,
                               self.eps_decay, wins, episodes, seed, counter)

    def prepare_greedy(self, eps, seed, counter):
        """Issue the greedy-row list of a coming greedy(act=(eps, seed, counter)) call now (its
        count then reaches the host while the stream runs the work queued behind it)."""
        if self.fused is None or not self.greedy_rows:
            return
        if self._rows is None:
            from .fused import GreedyRows
            self._rows = GreedyRows(self.steps_done.numel(), self.device)
        self._rows.issue(eps, seed, counter)

    def update(self, expand, reserve=0):
        """K updates (graph replays). With overlap, once the graphs exist, they are issued on the
        side stream and this returns at once; `reserve` = rows the next push will write (the
        vector step's instance count), kept out of the sampled range meanwhile."""
        if len(self.replay) < self.batch_size:
            return None
        if self.overlap and self._graph is not None:
            return self._update_async(reserve)
        for _ in range(self.updates_per_step):
            if self.use_graph:
                self._graph_update(expand)
            else:
                self.last_loss = self._one_update(expand, static=False)
            self.n_updates += 1
            if self.n_updates % self.target_every == 0:
                self._sync_target()
            if self.n_updates % self.updates_per_epoch == 0:
                self.sched.step()
        if self.fused is not None:
            self.fused.invalidate()  # FlatAdamW / graph replays leave the params' _version as is
        return self.last_loss

    @torch.no_grad()
    def _sync_target(self):
        """update_target (dqn_agent.py): target <- source; one copy between flat buffers."""
        if getattr(self.source, "_flat_params", None) is not None and \
                getattr(self.target, "_flat_params", None) is not None:
            copy_flat(self.target, self.source)
        else:
            self.target.load_state_dict(self.source.state_dict())

    # ---- overlapped learner (side stream) --------------------------------------------------
    # Vector step t on the main stream M: greedy(t) -> env step -> push(t) -> update(): the K
    # updates u_t go to the side stream S (after push(t)), followed by a snapshot of the source
    # net into actor slot t % 2 and an event D_t. greedy(t + 1) waits for D_{t-1} only and acts
    # with slot (t - 1) % 2: the acting weights lag the sequential schedule by one update, and
    # M never waits for the update it just issued. Races excluded by construction:
    #   * slot (t+1) % 2 is next written by u_{t+1}, which S starts after push(t+1), i.e. after
    #     greedy(t+1) finished reading it;
    #   * u_t samples the newest min(size, C - reserve) replay rows, indices drawn on M into
    #     buffer t % 2 (M waited D_{t-2}, the last reader of that buffer, in greedy(t)), so the
    #     rows push(t+1) overwrites concurrently are never read;
    #   * the source / target nets, the optimizer and the LR tensor are touched on S only.
    def _acting_slot(self):
        M = torch.cuda.current_stream(self.device)
        # keep the newest issued snapshot for the next step (unless nothing else is readable)
        while len(self._published) > 1 or (self._acting is None and self._published):
            slot, ev = self._published.popleft()
            M.wait_event(ev)
            self._acting = slot  # its bf16 head was rebuilt on S right after the snapshot
        return self._acting

    def _start_async(self):
        M = torch.cuda.current_stream(self.device)
        with torch.no_grad():
            for a, f in zip(self.actors, self.actor_fused):
                copy_flat(a, self.source)
                f.refresh()
        K, b = self.updates_per_step, self.batch_size
        # the index buffers are allocated once: the K-update graphs read them by address, and a
        # restart (finish() at the end of every train() call, then the next update) that gave
        # them new storage left those graphs copying whatever reused the old one — the round-4
        # K-update graph's irreproducible runs
        if getattr(self, "_idx", None) is None or tuple(self._idx[0].shape) != (K, b):
            self._idx = [torch.zeros(K, b, dtype=torch.int64, device=self.device) for _ in range(2)]
            self._graphK = [None, None]
        self._idx_ev = [None, None]
        self._acting, self._par = 0, 1  # the first update writes the slot greedy() does not read
        self._published.clear()
        self.side.wait_stream(M)
        self._async = True

    def _update_async(self, reserve):
        if not self._async:
            self._start_async()
        M, S = torch.cuda.current_stream(self.device), self.side
        rp, K, slot = self.replay, self.updates_per_step, self._par
        n_avail = min(rp.size, rp.capacity - int(reserve))
        if n_avail < self.batch_size:
            raise ValueError("replay too small to exclude the next push from sampling")
        if self._idx_ev[slot] is not None:
            M.wait_event(self._idx_ev[slot])  # the last update that read this index buffer
        idx = self._idx[slot]
        # the newest n_avail rows, ending at ptr - 1: one Philox launch (mz_replay_sample_idx)
        from .. import _native as N
        N.check(N.load().mz_replay_sample_idx(self._sample_seed, self._sample_counter, rp.ptr - 1,
                                              n_avail, rp.capacity, idx.data_ptr(), idx.numel(),
                                              M.cuda_stream))
        self._sample_counter += 1
        if self._acting == slot:  # greedy() must switch to a newer snapshot before reading again
            self._acting = None
        block = self._k_block_ok()
        if block and self._graphK[slot] is None:
            self._capture_k_block(slot)
        S.wait_stream(M)  # push(t), the indices, and every greedy() that read this slot
        with torch.cuda.stream(S):
            if block:
                # the K updates as ONE replay: no target sync or schedule step falls between them
                self._graphK[slot].replay()
                self.n_updates += K
                if self.n_updates % self.target_every == 0:
                    self._sync_target()
                if self.n_updates % self.updates_per_epoch == 0:
                    self.sched.step()
            for k in range(0 if block else K):
                rp.idx_static.copy_(idx[k])
                self._graph[0].replay()
                if len(self._graph) == 2:
                    self.allreduce.reduce()
                    self._graph[1].replay()
                    self.allreduce.gather(self.source)
                self.n_updates += 1
                if self.n_updates % self.target_every == 0:
                    self._sync_target()
                if self.n_updates % self.updates_per_epoch == 0:
                    self.sched.step()
            with torch.no_grad():
                copy_flat(self.actors[slot], self.source)
                self.actor_fused[slot].refresh()  # bf16 head of the snapshot, on S
            ev = torch.cuda.Event()
            ev.record(S)
        self._idx_ev[slot] = ev
        self._published.append((slot, ev))
        self._par ^= 1
        self.last_loss = self._graphK_loss[slot] if block else self._graph_loss
        return self.last_loss

    # K > 1 updates per vector step: one captured graph per index slot replays all K (the index
    # copies included), when neither the target sync nor the cosine schedule's step falls strictly
    # between two of them (those run on the host between replays); else the per-update replays.
    # The same kernels in the same order as K single-update replays: the same results bit for bit.
    # Not with a gradient all-reduce issued between graph replays (graph_collectives: inside them).
    def _k_block_ok(self):
        K = self.updates_per_step
        if K < 2 or (self.allreduce is not None and not self.graph_collectives) or not K_BLOCK \
                or not self.bit_stem:
            return False
        n0 = self.n_updates
        return all((n0 + j) % self.target_every and (n0 + j) % self.updates_per_epoch
                   for j in range(1, K))

    def _capture_k_block(self, slot):
        # each update's gather reads its row of the slot's index buffer in place (the buffers are
        # allocated once, _start_async): no copy into idx_static between the K updates — four
        # blit launches per vector step on the update stream (~13.6 us each inside best-of-6
        # training, profiles/r05u/train_kernel_stats.csv)
        rp, K = self.replay, self.updates_per_step
        g = torch.cuda.CUDAGraph()
        keep = rp.idx_static
        try:
            with torch.cuda.graph(g, capture_error_mode=self._capture_mode()):
                for k in range(K):
                    rp.idx_static = self._idx[slot][k]
                    loss = self._one_update(None, static=True)
        finally:
            rp.idx_static = keep
        self._graphK[slot] = g
        self._graphK_loss[slot] = loss

    def finish(self):
        """Join the side stream: the main stream waits for every issued update; greedy() acts with
        the source net again (evaluation)."""
        if self._async:
            torch.cuda.current_stream(self.device).wait_stream(self.side)
            self._published.clear()
            self._async = False
            self.fused.invalidate()

    # ---- checkpoint / resume (Q-nets, optimizer, replay, counters) -----------------
    def state_dict(self):
        """Everything the learner's future updates and acting depend on: both nets (the
        reference's module names, so the Q-net part loads into its DQN / DDQN classes), the
        optimizer moments, step count and learning rate, the cosine schedule, per-instance
        steps_done / epsilon decay, the filled replay rows and its pointer, the sample and dropout
        streams (replay index counter, the stems' device-side dropout counters and salts, the
        acting heads' (seed, counter), torch's RNG states). The side stream is joined first."""
        self.finish()
        rp, n = self.replay, self.replay.size
        opt = self.opt
        if hasattr(opt, "exp_avg"):  # FlatAdamW (device-side lr and step count)
            # (a sharded step, distributed.GradAllReduce.attach: the moments are valid only on
            # this rank's (offset, length) of the flat buffer — recorded, checked on load)
            ost = {"exp_avg": opt.exp_avg.clone(), "exp_avg_sq": opt.exp_avg_sq.clone(),
                   "step": opt._step_buf.clone(), "lr": float(opt.param_groups[0]["lr"]),
                   "shard": None if opt.shard is None else [int(x) for x in opt.shard]}
        else:
            ost = {"torch": opt.state_dict()}
        heads = [self.fused] + list(getattr(self, "actor_fused", []))
        ed = self.eps_decay
        return {"format": "mazerl.VectorDQNLearner/1", "variant": self.variant,
                "source": {k: v.clone() for k, v in self.source.state_dict().items()},
                "target": {k: v.clone() for k, v in self.target.state_dict().items()},
                "opt": ost, "sched": self.sched.state_dict(),
                "steps_done": self.steps_done.clone(),
                "eps_decay": ed.clone() if torch.is_tensor(ed) else float(ed),
                "n_updates": self.n_updates, "graph": self._graph is not None,
                "sample_seed": getattr(self, "_sample_seed", None),
                "sample_counter": getattr(self, "_sample_counter", None),
                "replay": {"capacity": rp.capacity, "ptr": rp.ptr, "size": n,
                           "rows": {k: getattr(rp, k)[:n].clone()
                                    for k in ("s6", "sw", "a", "r", "s6n", "swn")},
                           "gen": rp._gen.get_state()},
                "salts": [self.source._salt, self.target._salt],
                "stem_rng": [None if m._stem_rng is None else m._stem_rng.clone()
                             for m in (self.source, self.target)],
                "heads": [None if h is None else (h.stem.seed, h.stem.counter) if hasattr(h, "stem")
                          else (h.seed, h.counter) for h in heads],
                "torch_rng": torch.get_rng_state(),
                "cuda_rng": torch.cuda.get_rng_state(self.device) if self.device.type == "cuda" else None}

    def load_state_dict(self, sd):
        """Restore a state_dict() in place (captured update graphs keep their buffers). A learner
        whose update graphs do not exist yet while the saved one had them first captures its
        own (warm-up updates on the loaded replay, then the capture), so that the resumed run
        takes the same update path; the state is then loaded again over what those changed."""
        if sd.get("format") != "mazerl.VectorDQNLearner/1" or sd["variant"] != self.variant:
            raise ValueError("not a state_dict of a VectorDQNLearner of this variant")
        if sd["replay"]["capacity"] != self.replay.capacity:
            raise ValueError("replay capacity differs from the saved learner's")
        # construction-order salts of the stems' dropout masks: before any capture bakes them in
        self.source._salt, self.target._salt = sd["salts"]
        self._load(sd)
        if sd["graph"] and self.use_graph and self._graph is None:
            while self._graph is None:
                self._graph_update(None)
            self._load(sd)

    def _load(self, sd):
        dev = self.device
        with torch.no_grad():
            self.source.load_state_dict(sd["source"])
            self.target.load_state_dict(sd["target"])
        o = sd["opt"]
        if "torch" in o:
            self.opt.load_state_dict(o["torch"])
        else:
            saved, now = o.get("shard"), getattr(self.opt, "shard", None)
            if saved is not None and (now is None or tuple(saved) != tuple(now)):
                raise ValueError(f"the saved optimizer moments hold only the flat-buffer shard "
                                 f"{tuple(saved)} of a sharded data-parallel step; this learner "
                                 f"updates {'all of it' if now is None else tuple(now)} — resume "
                                 f"with the same world size and rank")
            self.opt.exp_avg.copy_(o["exp_avg"])
            self.opt.exp_avg_sq.copy_(o["exp_avg_sq"])
            self.opt._step_buf.copy_(o["step"])
        self.sched.load_state_dict(sd["sched"])
        lr = self.opt.param_groups[0]["lr"]
        if "lr" in o and torch.is_tensor(lr):
            lr.fill_(o["lr"])
        self.steps_done.copy_(sd["steps_done"])
        ed = sd["eps_decay"]
        self.eps_decay = ed.to(dev).clone() if torch.is_tensor(ed) else float(ed)
        self.n_updates = int(sd["n_updates"])
        if sd["sample_seed"] is not None and hasattr(self, "_sample_seed"):
            self._sample_seed, self._sample_counter = sd["sample_seed"], sd["sample_counter"]
        rp, r = self.replay, sd["replay"]
        n = int(r["size"])
        for k, v in r["rows"].items():
            getattr(rp, k)[:n].copy_(v)
        rp.ptr, rp.size = int(r["ptr"]), n
        rp.size_dev.fill_(float(n))
        rp._gen.set_state(r["gen"].cpu())  # (map_location may have moved it)
        for m, st in zip((self.source, self.target), sd["stem_rng"]):
            if st is None:
                continue
            if m._stem_rng is None:
                m._stem_rng = torch.zeros(1, dtype=torch.int64, device=dev)
            m._stem_rng.copy_(st)  # in place: a captured graph advances this very tensor
        heads = [self.fused] + list(getattr(self, "actor_fused", []))
        for h, st in zip(heads, sd["heads"]):
            if h is None or st is None:
                continue
            tgt = h.stem if hasattr(h, "stem") else h
            tgt.seed, tgt.counter = st
            h.invalidate()
        torch.set_rng_state(sd["torch_rng"].cpu())
        if sd["cuda_rng"] is not None and dev.type == "cuda":
            torch.cuda.set_rng_state(sd["cuda_rng"].cpu(), dev)

    def _one_update(self, expand, static):
        if self.overlap and not torch.cuda.is_current_stream_capturing():
            fresh = self.replay.sample_indices(self.batch_size)  # eager (pre-capture) update
            if self.replay.idx_static is None:
                self.replay.idx_static = fresh
            else:
                self.replay.idx_static.copy_(fresh)
        state, a, r, nxt = self.replay.sample(self.batch_size, None if self.bit_stem else expand,
                                              static=static, idx_static=self.overlap)
        loss = self._loss(state, a, r, nxt)
        learner_update(self.source, self.opt, loss, allreduce=self.allreduce)
        return loss.detach()

    def _loss(self, state, a, r, nxt):
        return q_loss(self.source, self.target, state, a, r, nxt, self.gamma, self.variant == "ddqn")

    def _capture_mode(self):
        # thread-local: the process group's watchdog thread polls its collectives' events, which
        # a global-mode capture forbids ("operation not permitted when stream is capturing")
        return "thread_local" if self.allreduce is not None else "global"

    def _graph_update(self, expand, warmup=3):
        ar = self.allreduce
        if self._graph is None:
            if self._eager_updates < warmup:  # real updates on a side stream before capture
                s = torch.cuda.Stream(self.device)
                s.wait_stream(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(s):
                    self.last_loss = self._one_update(expand, static=True)
                torch.cuda.current_stream(self.device).wait_stream(s)
                self._eager_updates += 1
                return
            self.opt.zero_grad(set_to_none=True)
            if ar is None or self.graph_collectives:
                # (with the collectives: the reduce-scatter / all-gather of learner_update are
                # captured as graph nodes on RCCL's stream, forked from and joined back to this one)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, capture_error_mode=self._capture_mode()):
                    self._graph_loss = self._one_update(expand, static=True)
                self._graph = (g,)
            else:
                ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
                # thread-local capture: the process group's watchdog thread polls the events of
                # the warm-up all-reduces, which a global-mode capture forbids ("operation not
                # permitted when stream is capturing" on RCCL)
                with torch.cuda.graph(ga, capture_error_mode="thread_local"):
                    state, a, r, nxt = self.replay.sample(
                        self.batch_size, None if self.bit_stem else expand, static=True,
                        idx_static=self.overlap)
                    loss = self._loss(state, a, r, nxt)
                    learner_backward(self.opt, loss)
                    ar.pack(self.source)
                    self._graph_loss = loss.detach()
                with torch.cuda.graph(gb, pool=ga.pool(), capture_error_mode="thread_local"):
                    ar.unpack(self.source)
                    learner_step(self.source, self.opt)
                self._graph = (ga, gb)
            if self.overlap:
                # the capture drew no indices (it does not run): the first replay must not reuse
                # the last eager warm-up's rows, which that update already applied
                self.replay.idx_static.copy_(self.replay.sample_indices(self.batch_size))
        self._graph[0].replay()
        if len(self._graph) == 2:
            ar.reduce()
            self._graph[1].replay()
            ar.gather(self.source)
        self.last_loss = self._graph_loss
        if self.fused is not None:
            self.fused.invalidate()  # graph replays leave the params' _version untouched
