// mz_trainer.hip — the vectorised DQN/DDQN trainer's per-vector-step bookkeeping as few launches.
//
// The training loop (mazerl/trainers/vector_trainer.py, NeuralOffPolicyTrainer.train of
// lib/trainers/off_policy_trainer.py:144-225 over B instances) waits once per vector step for the
// length of the greedy-row list (the GEMM sizes of the acting forward), so every launch the host
// issues after that wait is on the critical path. These kernels replace ~30 small torch launches:
//
//   k_tick_count     steps_done += 1, = 0 on a win (off_policy_trainer.py:192); the next step's
//                    epsilon (dqn_agent.py:118-119, f32 as the learner computed it with torch);
//                    win / episode counters; per-block counts of the next greedy-row list (the
//                    list itself is k_greedy_list of mz_env.hip, same draw as the fused act)
//   k_greedy_scatter argmax of the acting forward's Q rows (first maximum, torch.argmax) written
//                    to the listed instances' greedy slots; reads the list length on the device
//   k_head_bf16      the acting head's bf16 weights from the f32 parameters (fc1 columns
//                    permuted to the fused stem's position-major feature order and zero-padded)
//   k_replay_push    ring rows ptr .. ptr + n - 1 of the replay's six arrays <- a vector step
//   k_replay_idx     uniform sample rows over the newest n_avail ring rows (Philox)
//   k_q_loss_fwd/bwd the Q-learning loss of optimize_model (dqn_agent.py:129-147,
//                    ddqn_agent.py:121-143) from the nets' output rows, and its gradient w.r.t.
//                    those rows — what gather / max / argmax / mul / add / mse_loss / mean and
//                    their backward (zero fills, scatter, slice copy) did in ~15 launches
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "mz_common.h"
#include "mz_learner.h"

namespace {

constexpr int TB = MZ_GR_BLOCK;  // the greedy-row list reads these per-block counts (mz_kernels.h)
constexpr int W = 64;

__device__ inline float eps_of(float sd, float eps_final, float eps_span, float inv_decay) {
  // torch: eps_final + (eps_start - eps_final) * torch.exp(-steps_done / eps_decay), f32 ops each
  // rounded (no contraction); torch divides by a CPU scalar as a multiply by its f32 reciprocal
  const float x = __fmul_rn(-sd, inv_decay);
  return __fadd_rn(eps_final, __fmul_rn(eps_span, expf(x)));
}

__global__ __launch_bounds__(TB) void k_tick_count(const uint8_t* __restrict__ term,
                                                   const uint8_t* __restrict__ trunc,
                                                   float* __restrict__ steps_done, float eps_final,
                                                   float eps_span, float inv_decay,
                                                   float* __restrict__ eps_out,
                                                   unsigned long long* wins,
                                                   unsigned long long* episodes, uint64_t seed,
                                                   uint64_t counter, int n, int32_t* blk) {
  __shared__ int ws[TB / W], es[TB / W];
  const int e = blockIdx.x * TB + threadIdx.x;
  const int lane = threadIdx.x & (W - 1), w = threadIdx.x / W;
  bool need = false, won = false, done = false;
  if (e < n) {
    won = term[e] != 0;
    done = won || trunc[e] != 0;
    const float sd = won ? 0.0f : steps_done[e] + 1.0f;
    steps_done[e] = sd;
    const float ep = eps_of(sd, eps_final, eps_span, inv_decay);
    eps_out[e] = ep;
    uint32_t u[4];
    mz_philox(seed, MZ_ACT_STREAM ^ ((uint64_t)e << 32), counter, u);  // act_u (mz_env.hip)
    need = !((float)(u[0] >> 8) * (1.0f / 16777216.0f) < ep);          // act_greedy
  }
  const int c = __syncthreads_count(need);
  const unsigned long long bw = __ballot(won), bd = __ballot(done);
  if (lane == 0) {
    ws[w] = __popcll(bw);
    es[w] = __popcll(bd);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    blk[blockIdx.x] = c;
    int sw = 0, se = 0;
    for (int i = 0; i < TB / W; ++i) {
      sw += ws[i];
      se += es[i];
    }
    if (wins && sw) atomicAdd(wins, (unsigned long long)sw);
    if (episodes && se) atomicAdd(episodes, (unsigned long long)se);
  }
}

__device__ inline float bf16f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }

__global__ void k_greedy_scatter(const uint16_t* __restrict__ q, int ldq,
                                 const int32_t* __restrict__ rows, const int32_t* __restrict__ count,
                                 int m, int64_t* __restrict__ greedy) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int k = min(*count, m);
  if (i >= k) return;
  const uint16_t* r = q + (size_t)i * ldq;
  int best = 0;
  float bv = bf16f(r[0]);
  for (int a = 1; a < 4; ++a) {  // first maximum; NaN counts as the maximum (torch.argmax)
    const float v = bf16f(r[a]);
    if (!isnan(bv) && (v > bv || isnan(v))) {
      best = a;
      bv = v;
    }
  }
  greedy[rows[i]] = best;
}

__device__ inline uint16_t bf16_rne(float f) {  // torch's float -> bfloat16 (round to nearest even)
  const uint32_t u = __float_as_uint(f);
  if ((u & 0x7FFFFFFFu) > 0x7F800000u) return (uint16_t)((u >> 16) | 0x40u);  // quiet NaN
  return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}

// Blocks [0, out0): one fc1 row each — the f32 row read coalesced into LDS, the permuted /
// padded bf16 row written coalesced from it (a column gather straight from global memory strides
// 49 floats between neighbouring lanes: 31 us per call vs ~3 for the bytes). The other blocks
// convert fc2, fc3 and the biases grid-stride.
constexpr int HEAD_MAX_IN = 2048;
__global__ __launch_bounds__(256) void k_head_bf16(MzHeadBf16 h) {
  __shared__ float row[HEAD_MAX_IN];
  if ((int)blockIdx.x < h.out[0]) {
    const int o = blockIdx.x;
    const float* src = h.w[0] + (size_t)o * h.in[0];
    for (int j = threadIdx.x; j < h.in[0]; j += blockDim.x) row[j] = src[j];
    __syncthreads();
    const int nq = h.conv_out / h.conv_ch;
    uint16_t* dst = h.dw[0] + (size_t)o * h.ld0;
    for (int j = threadIdx.x; j < h.ld0; j += blockDim.x) {
      float v = 0.0f;
      if (j < h.conv_out) v = row[(j % h.conv_ch) * nq + j / h.conv_ch];  // kernel q*C+c <- torch c*Q+q
      else if (j < h.in[0]) v = row[j];
      dst[j] = bf16_rne(v);
    }
    return;
  }
  const int64_t n1 = (int64_t)h.out[1] * h.in[1];
  const int64_t n2 = (int64_t)h.out[2] * h.in[2];
  const int64_t total = n1 + n2 + h.out[0] + h.out[1] + h.out[2];
  const int64_t nb = (int64_t)gridDim.x - h.out[0];
  for (int64_t t = ((int64_t)blockIdx.x - h.out[0]) * blockDim.x + threadIdx.x; t < total;
       t += nb * blockDim.x) {
    int64_t k = t;
    if (k < n1) { h.dw[1][k] = bf16_rne(h.w[1][k]); continue; }
    k -= n1;
    if (k < n2) { h.dw[2][k] = bf16_rne(h.w[2][k]); continue; }
    k -= n2;
    for (int l = 0; l < 3; ++l) {
      if (k < h.out[l]) { h.db[l][k] = bf16_rne(h.b[l][k]); break; }
      k -= h.out[l];
    }
  }
}

__global__ __launch_bounds__(256) void k_replay_push(MzReplayPush p) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  for (int j = 0; j < 6; ++j) {
    if (!p.src[j]) continue;
    const int wds = p.words[j];
    const int64_t tot = (int64_t)p.n * wds;
    for (int64_t t = t0; t < tot; t += stride) {
      const int64_t r = t / wds, c = t - r * wds;
      int64_t dr = p.ptr + r;
      if (dr >= p.cap) dr -= p.cap;
      if (j == 2) {  // action: int32 -> int64 ring
        reinterpret_cast<int64_t*>(p.dst[j])[dr] = reinterpret_cast<const int32_t*>(p.src[j])[r];
      } else {
        reinterpret_cast<uint32_t*>(p.dst[j])[dr * wds + c] =
            reinterpret_cast<const uint32_t*>(p.src[j])[t];
      }
    }
  }
}

__global__ void k_replay_idx(uint64_t seed, uint64_t counter, int64_t newest, int64_t n_avail,
                             int64_t cap, int64_t* __restrict__ out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t u[4];
  mz_philox(seed, MZ_REPLAY_STREAM ^ ((uint64_t)i << 32), counter, u);
  // 53-bit uniform in [0, 1) -> one of the newest n_avail rows, ending at ring row `newest`
  const double x = (double)(((uint64_t)u[0] << 21) ^ (u[1] >> 11)) * (1.0 / 9007199254740992.0);
  int64_t r = newest - (int64_t)(x * (double)n_avail);
  r %= cap;
  if (r < 0) r += cap;
  out[i] = r;
}

// One workgroup: per row i < b, a = action[i], Q(s,a) = q[i][a];
//   V(s') = q_tgt[i][argmax q_next[i]] (DDQN, first maximum) or max q_tgt[i] (DQN);
//   diff = Q(s,a) - (V(s') * gamma + r)   (f32, torch's op order, no contraction);
// loss = (sum diff^2) / b.
__global__ __launch_bounds__(1024) void k_q_loss_fwd(const float* __restrict__ q, int ldq,
                                                    const float* __restrict__ qn, int ldn,
                                                    const float* __restrict__ qt, int ldt,
                                                    const int64_t* __restrict__ action,
                                                    const float* __restrict__ reward, float gamma,
                                                    int b, float* __restrict__ loss,
                                                    float* __restrict__ diff) {
  __shared__ float part[1024 / W];
  float acc = 0.0f;
  for (int i = threadIdx.x; i < b; i += blockDim.x) {
    const float* t = qt + (size_t)i * ldt;
    float v;
    // NaN as torch has it (a diverging net must not report a finite loss): argmax takes the
    // first NaN as the maximum, max(1)[0] propagates any NaN
    if (qn) {
      const float* x = qn + (size_t)i * ldn;
      int best = 0;
      for (int k = 1; k < 4; ++k)
        if (!isnan(x[best]) && (isnan(x[k]) || x[k] > x[best])) best = k;
      v = t[best];
    } else {
      v = t[0];
      for (int k = 1; k < 4; ++k)
        if (!isnan(v) && (isnan(t[k]) || t[k] > v)) v = t[k];
    }
    const float expected = __fadd_rn(__fmul_rn(v, gamma), reward[i]);
    const float d = __fsub_rn(q[(size_t)i * ldq + (int)action[i]], expected);
    diff[i] = d;
    acc = __fadd_rn(acc, __fmul_rn(d, d));
  }
  for (int o = W / 2; o; o >>= 1) acc = __fadd_rn(acc, __shfl_xor(acc, o));
  if ((threadIdx.x & (W - 1)) == 0) part[threadIdx.x / W] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.0f;
    for (int k = 0; k < (int)(blockDim.x / W); ++k) s = __fadd_rn(s, part[k]);
    *loss = __fdiv_rn(s, (float)b);
  }
}

// dq[i][k] = diff[i] * (2 / b) * g at k = action[i] for i < b; 0 elsewhere (rows >= b included):
// mse_loss's mean backward, then gather's and the row slice's (torch's order of the products)
__global__ void k_q_loss_bwd(const float* __restrict__ g, const float* __restrict__ diff,
                             const int64_t* __restrict__ action, int b, int rows, float norm,
                             float* __restrict__ dq) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= rows * 4) return;
  const int i = t >> 2, k = t & 3;
  float v = 0.0f;
  if (i < b && k == (int)action[i]) v = __fmul_rn(__fmul_rn(diff[i], norm), *g);
  dq[t] = v;
}

// ---- the Q head + loss as one launch forward, one (+ a column sum) backward -------------------
// Per update the learner's heads did: the second hidden layer's activation, fc3 (a GEMM with 4
// outputs), for the source's stacked [s; s'] rows and the target's s' rows, then the loss; and
// backward the loss gradient, fc3's dX and dW GEMMs and bias column sum, the activation's
// backward — 10 launches of little work each (config 4's 512-row updates are a chain of such
// launches). Here, from the pre-activation z2 = fc2(...) of both nets:
//   k_head_loss       one wave per row i < b: h = act(z2), q_s(i) = W3 h + b3 (4 dot products of
//                     H), DDQN's q_s(b + i) -> first argmax, the target's q_t(i), the TD error
//                     diff_i (k_q_loss_fwd's f32 ops and NaN rules), the loss = sum diff^2 / b
//                     summed per workgroup, then over workgroups in order by k_loss_sum (a
//                     one-workgroup launch): deterministic;
//   k_head_loss_bwd   g_i = diff_i * (2 / b) * grad (k_q_loss_bwd's order); dz2[i][j] =
//                     act'(z2[i][j]) * (g_i W3[a_i][j]) — dq has one nonzero per row, so this IS
//                     fc3's dX GEMM value (the other terms are exact zeros) — for i < b; the
//                     per-block partials of dW3[k][j] = sum_i [a_i = k] g_i act(z2[i][j]) and of
//                     db3[k] = sum_i [a_i = k] g_i, summed over blocks in order by mz_colsum_f32.
// act: 0 = LeakyReLU(0.01) (DQN), 1 = ReLU (DDQN); torch's forward / backward rules at 0 and NaN.
constexpr int HL_T = 256;  // 4 waves, 4 rows per workgroup (forward)
constexpr int HB_RB = 16;  // rows per workgroup (backward)
constexpr int HB_T = 256;

template <int ACT>
__device__ inline float head_act(float z) {
  if (ACT == 0) return z > 0.0f ? z : __fmul_rn(z, 0.01f);
  return z > 0.0f ? z : (isnan(z) ? z : 0.0f);  // clamp_min(z, 0): NaN propagates
}
template <int ACT>
__device__ inline float head_act_grad(float z, float g) {
  if (ACT == 0) return z > 0.0f ? g : __fmul_rn(g, 0.01f);  // leaky_relu_backward(grad, self)
  return (z > 0.0f || isnan(z)) ? g : 0.0f;                  // threshold_backward(grad, out, 0)
}

__device__ inline float wave_sum_f(float x) {
  for (int o = W / 2; o; o >>= 1) x = __fadd_rn(x, __shfl_xor(x, o));
  return x;
}

// Per lane the row's columns j = lane, lane + 64, ... in that order (the f32 FMA chains of the
// round-4 kernel, bit for bit), HL_U of them with all their loads (z2 of the three rows, W3 of
// both nets) issued before the first FMA: a loop that loaded one column per iteration waited one
// round trip per 64 columns (38.6 us for 2,048 DDQN rows, 25.5 us for 512). The per-workgroup
// partials of sum diff^2 are summed by k_loss_sum, a second one-workgroup launch: a last-workgroup
// ticket cost each workgroup a fence + atomic round trip at the end of the launch (~11 us at 512
// workgroups, profiles/r05u/ticket.jsonl).
constexpr int HL_U = 4;
template <int ACT>
__global__ __launch_bounds__(HL_T) void k_head_loss(
    const float* __restrict__ z2s, int lds, const float* __restrict__ w3s,
    const float* __restrict__ b3s, const float* __restrict__ z2t, int ldt,
    const float* __restrict__ w3t, const float* __restrict__ b3t, int dbl,
    const int64_t* __restrict__ action, const float* __restrict__ reward, float gamma, int b, int H,
    float* __restrict__ part, float* __restrict__ diff) {
  __shared__ float wpart[HL_T / W];
  const int lane = threadIdx.x & (W - 1), w = threadIdx.x / W;
  const int i = blockIdx.x * (HL_T / W) + w;
  float d2 = 0.0f;
  if (i < b) {
    float as[4] = {0.f, 0.f, 0.f, 0.f}, an[4] = {0.f, 0.f, 0.f, 0.f}, at[4] = {0.f, 0.f, 0.f, 0.f};
    const float* rs = z2s + (size_t)i * lds;
    const float* rn = z2s + (size_t)(b + i) * lds;
    const float* rt = z2t + (size_t)i * ldt;
    for (int j0 = lane; j0 < H; j0 += HL_U * W) {
      float xs[HL_U], xt[HL_U], xn[HL_U], ws[HL_U][4], wt[HL_U][4];
#pragma unroll
      for (int u = 0; u < HL_U; ++u) {
        const int j = j0 + u * W;
        const bool ok = j < H;
        xs[u] = ok ? rs[j] : 0.0f;
        xt[u] = ok ? rt[j] : 0.0f;
        xn[u] = ok && dbl ? rn[j] : 0.0f;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          ws[u][k] = ok ? w3s[k * H + j] : 0.0f;
          wt[u][k] = ok ? w3t[k * H + j] : 0.0f;
        }
      }
#pragma unroll
      for (int u = 0; u < HL_U; ++u) {
        if (j0 + u * W >= H) break;
        const float hs = head_act<ACT>(xs[u]), ht = head_act<ACT>(xt[u]);
        const float hn = dbl ? head_act<ACT>(xn[u]) : 0.0f;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          as[k] = __fmaf_rn(hs, ws[u][k], as[k]);
          at[k] = __fmaf_rn(ht, wt[u][k], at[k]);
          if (dbl) an[k] = __fmaf_rn(hn, ws[u][k], an[k]);
        }
      }
    }
    float qs[4], qn[4], qt[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      qs[k] = __fadd_rn(wave_sum_f(as[k]), b3s[k]);
      qt[k] = __fadd_rn(wave_sum_f(at[k]), b3t[k]);
      qn[k] = dbl ? __fadd_rn(wave_sum_f(an[k]), b3s[k]) : 0.0f;
    }
    float v;
    if (dbl) {  // argmax over q_s(s') (first maximum; the first NaN wins, as torch.argmax)
      int best = 0;
      for (int k = 1; k < 4; ++k)
        if (!isnan(qn[best]) && (isnan(qn[k]) || qn[k] > qn[best])) best = k;
      v = qt[best];
    } else {  // max(1)[0] of the target's row (any NaN propagates)
      v = qt[0];
      for (int k = 1; k < 4; ++k)
        if (!isnan(v) && (isnan(qt[k]) || qt[k] > v)) v = qt[k];
    }
    const float expected = __fadd_rn(__fmul_rn(v, gamma), reward[i]);
    const float d = __fsub_rn(qs[(int)action[i]], expected);
    if (lane == 0) diff[i] = d;
    d2 = __fmul_rn(d, d);
  }
  if (lane == 0) wpart[w] = d2;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.0f;
    for (int k = 0; k < HL_T / W; ++k) s = __fadd_rn(s, wpart[k]);
    part[blockIdx.x] = s;
  }
}

// the loss = (sum of the workgroups' partials, in a fixed order) / b — the order the round-4
// kernel's last workgroup used: thread t sums partials t, t + 256, ..., then the waves' butterflies
// and the four wave sums in order
__global__ __launch_bounds__(HL_T) void k_loss_sum(const float* __restrict__ part, int nblk, int b,
                                                  float* __restrict__ loss) {
  __shared__ float wpart[HL_T / W];
  const int lane = threadIdx.x & (W - 1), w = threadIdx.x / W;
  float s = 0.0f;
  for (int k = threadIdx.x; k < nblk; k += HL_T) s = __fadd_rn(s, part[k]);
  s = wave_sum_f(s);
  if (lane == 0) wpart[w] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.0f;
    for (int k = 0; k < HL_T / W; ++k) t = __fadd_rn(t, wpart[k]);
    *loss = __fdiv_rn(t, (float)b);
  }
}

// The block's rows' g_i and a_i are formed once into LDS, and per column j the 16 rows' z2 and
// W3's four rows are loaded before any arithmetic: the round-4 loop read action[i], then
// W3[a_i][j] (a dependent load), then z2[i][j] row after row (39.7 us average per launch inside
// training, profiles/r05u). Same f32 operations in the same order: the same bits.
template <int ACT>
__global__ __launch_bounds__(HB_T) void k_head_loss_bwd(
    const float* __restrict__ g, const float* __restrict__ diff, const int64_t* __restrict__ action,
    int b, float norm, const float* __restrict__ z2s, int lds, const float* __restrict__ w3s, int H,
    float* __restrict__ dz2, int ldd, float* __restrict__ part) {
  // part: [gridDim.x][4 H + 4] — this block's dW3 (row-major [4][H]) and db3 partials
  __shared__ float gs[HB_RB];
  __shared__ int as_[HB_RB];
  const int r0 = blockIdx.x * HB_RB, nr = min(b, r0 + HB_RB) - r0;
  const float gg = *g;
  if ((int)threadIdx.x < nr) {
    gs[threadIdx.x] = __fmul_rn(__fmul_rn(diff[r0 + threadIdx.x], norm), gg);
    as_[threadIdx.x] = (int)action[r0 + threadIdx.x];
  }
  __syncthreads();
  float* pw = part + (size_t)blockIdx.x * (4 * H + 4);
  for (int j = threadIdx.x; j < H; j += HB_T) {
    float z[HB_RB];
    const float w0 = w3s[j], w1 = w3s[H + j], w2 = w3s[2 * H + j], w3 = w3s[3 * H + j];
#pragma unroll
    for (int i = 0; i < HB_RB; ++i) z[i] = i < nr ? z2s[(size_t)(r0 + i) * lds + j] : 0.0f;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
    for (int i = 0; i < HB_RB; ++i) {
      if (i >= nr) break;
      const int a = as_[i];
      const float sg = gs[i];
      const float wa = a == 0 ? w0 : (a == 1 ? w1 : (a == 2 ? w2 : w3));
      dz2[(size_t)(r0 + i) * ldd + j] = head_act_grad<ACT>(z[i], __fmul_rn(sg, wa));
      const float t = __fmul_rn(sg, head_act<ACT>(z[i]));
      a0 = a == 0 ? __fadd_rn(a0, t) : a0;
      a1 = a == 1 ? __fadd_rn(a1, t) : a1;
      a2 = a == 2 ? __fadd_rn(a2, t) : a2;
      a3 = a == 3 ? __fadd_rn(a3, t) : a3;
    }
    pw[j] = a0;
    pw[H + j] = a1;
    pw[2 * H + j] = a2;
    pw[3 * H + j] = a3;
  }
  if (threadIdx.x < 4) {
    float sb = 0.0f;
    for (int i = 0; i < nr; ++i)
      if (as_[i] == (int)threadIdx.x) sb = __fadd_rn(sb, gs[i]);
    pw[4 * H + threadIdx.x] = sb;
  }
}

}  // namespace

hipError_t mz_launch_q_loss(const float* q, int ldq, const float* qn, int ldn, const float* qt,
                            int ldt, const int64_t* action, const float* reward, float gamma, int b,
                            float* loss, float* diff, hipStream_t s) {
  hipLaunchKernelGGL(k_q_loss_fwd, dim3(1), dim3(1024), 0, s, q, ldq, qn, ldn, qt, ldt, action,
                     reward, gamma, b, loss, diff);
  return hipGetLastError();
}

hipError_t mz_launch_q_loss_bwd(const float* g, const float* diff, const int64_t* action, int b,
                                int rows, float norm, float* dq, hipStream_t s) {
  hipLaunchKernelGGL(k_q_loss_bwd, dim3((rows * 4 + 255) / 256), dim3(256), 0, s, g, diff, action,
                     b, rows, norm, dq);
  return hipGetLastError();
}

hipError_t mz_launch_head_loss(const MzHeadLoss& p, hipStream_t s) {
  if (p.b <= 0 || p.H <= 0 || p.H % 4) return hipErrorInvalidValue;
  const int blocks = (p.b + HL_T / W - 1) / (HL_T / W);
  if (p.act == 0)
    hipLaunchKernelGGL(k_head_loss<0>, dim3(blocks), dim3(HL_T), 0, s, p.z2s, p.lds, p.w3s, p.b3s,
                       p.z2t, p.ldt, p.w3t, p.b3t, p.dbl, p.action, p.reward, p.gamma, p.b, p.H,
                       p.part, p.diff);
  else
    hipLaunchKernelGGL(k_head_loss<1>, dim3(blocks), dim3(HL_T), 0, s, p.z2s, p.lds, p.w3s, p.b3s,
                       p.z2t, p.ldt, p.w3t, p.b3t, p.dbl, p.action, p.reward, p.gamma, p.b, p.H,
                       p.part, p.diff);
  hipLaunchKernelGGL(k_loss_sum, dim3(1), dim3(HL_T), 0, s, p.part, blocks, p.b, p.loss);
  return hipGetLastError();
}

int mz_head_loss_blocks(int b) { return (b + HL_T / W - 1) / (HL_T / W); }
int mz_head_loss_bwd_blocks(int b) { return (b + HB_RB - 1) / HB_RB; }

hipError_t mz_launch_head_loss_bwd(const float* g, const float* diff, const int64_t* action, int b,
                                   float norm, const float* z2s, int lds, const float* w3s, int H,
                                   int act, float* dz2, int ldd, float* part, hipStream_t s) {
  if (b <= 0 || H <= 0 || H % 4) return hipErrorInvalidValue;
  const int blocks = mz_head_loss_bwd_blocks(b);
  if (act == 0)
    hipLaunchKernelGGL(k_head_loss_bwd<0>, dim3(blocks), dim3(HB_T), 0, s, g, diff, action, b, norm,
                       z2s, lds, w3s, H, dz2, ldd, part);
  else
    hipLaunchKernelGGL(k_head_loss_bwd<1>, dim3(blocks), dim3(HB_T), 0, s, g, diff, action, b, norm,
                       z2s, lds, w3s, H, dz2, ldd, part);
  return hipGetLastError();
}

hipError_t mz_launch_tick(const uint8_t* term, const uint8_t* trunc, float* steps_done,
                          float eps_final, float eps_span, float inv_decay, float* eps_out,
                          unsigned long long* wins, unsigned long long* episodes, uint64_t seed,
                          uint64_t counter, int n, int32_t* scratch, int32_t* rows, int32_t* count,
                          hipStream_t s) {
  const int blocks = (n + TB - 1) / TB;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(k_tick_count, dim3(blocks), dim3(TB), 0, s, term, trunc, steps_done, eps_final,
                     eps_span, inv_decay, eps_out, wins, episodes, seed, counter, n, scratch);
  MzAct ap{eps_out, 0.0f, nullptr, seed, counter, nullptr};
  return mz_launch_greedy_list(ap, n, scratch, rows, count, nullptr, s);
}

hipError_t mz_launch_greedy_scatter(const uint16_t* q, int ldq, const int32_t* rows,
                                    const int32_t* count, int m, int64_t* greedy, hipStream_t s) {
  if (m <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_greedy_scatter, dim3((m + 255) / 256), dim3(256), 0, s, q, ldq, rows, count,
                     m, greedy);
  return hipGetLastError();
}

hipError_t mz_launch_head_bf16(const MzHeadBf16& h, hipStream_t s) {
  if (h.in[0] > HEAD_MAX_IN) return hipErrorInvalidValue;
  const int64_t rest = (int64_t)h.out[1] * h.in[1] + (int64_t)h.out[2] * h.in[2] + h.out[0] +
                       h.out[1] + h.out[2];
  int64_t blocks = (rest + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(k_head_bf16, dim3((unsigned)(h.out[0] + blocks)), dim3(256), 0, s, h);
  return hipGetLastError();
}

hipError_t mz_launch_replay_push(const MzReplayPush& p, hipStream_t s) {
  if (p.n <= 0) return hipSuccess;
  int64_t blocks = ((int64_t)p.n * 22 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(k_replay_push, dim3((unsigned)blocks), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t mz_launch_replay_idx(uint64_t seed, uint64_t counter, int64_t newest, int64_t n_avail,
                                int64_t cap, int64_t* out, int n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_replay_idx, dim3((n + 255) / 256), dim3(256), 0, s, seed, counter, newest,
                     n_avail, cap, out, n);
  return hipGetLastError();
}
