// mz_ppo.hip — config 5's PPO rollout path on the device: act, per-instance episode record,
// episode finishing (discounted returns, per-episode normalisation, advantages) and the append to
// the update pool, with no host round trip per vector step.
//
// Reference (one env): PPOAgent.do_episode (agents/ppo_agent.py:143-169) acts with
// ActorCriticNet.act (:55-68: softmax of the actor logits, torch.multinomial, log of the chosen
// probability, the critic value), appends (state, action, log-prob, value, reward) per step and at
// the episode's end computes calculate_returns (:171-181: acc = r + acc * gamma backwards over
// Python floats, torch.tensor -> float32, (R - mean) / std with the unbiased std) and
// calculate_advantages (:183-186: A = R - V, (A - mean) / (std + 1e-8)); PPOTrainer.train
// (lib/trainers/ppo_trainer.py:62-99) collects finished episodes into its Buffer and runs
// optimize_model on them.
//
// Vectorised (trainers/ppo_trainer.py VectorPPOTrainer): B instances step together; instance i's
// transitions go to row i of [B][L] buffers at its own step index t[i]. Per vector step:
//   k_ppo_act     the policy draw from the f32 actor logits (softmax as torch's kernel forms it
//                 for a 4-wide row, inverse CDF of a Philox uniform), log-prob of the draw, and
//                 the record of (obs6, window bits, action, log-prob, value) at t[i];
//   (mz_step)     the env step;
//   k_ppo_scan    one workgroup: the step's float64 reward at t[i], t[i] += 1, and for the
//                 instances whose episode ended: episode / win counters, t[i] = 0, and the list of
//                 finished episodes with their pool offsets (an exclusive scan over instances, so
//                 the pool order is the instance order — deterministic). 1-step episodes have an
//                 undefined std (NaN returns, torch.std of one element) and are dropped here;
//   k_ppo_finish  one workgroup per finished episode: returns backwards in float64 (serial, the
//                 reference's exact sums, rounded to float32), the two normalisations (sums in
//                 float64), and the episode's rows copied into the pool (SoA).
// The pool's fill count and a monotonic appended-rows total stay on the device; the host reads
// the total one step late (it only grows) to decide when an update is due.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "mz_common.h"
#include "mz_learner.h"

namespace {

constexpr int WAVE = 64;
constexpr int ACT_IPB = 8;       // instances per k_ppo_act workgroup (32 lanes each)
constexpr int SCAN_T = 1024;     // k_ppo_scan threads (one workgroup)
constexpr int FIN_T = 256;       // k_ppo_finish threads per episode
constexpr int FIN_CH = 2048;     // rewards staged in LDS per chunk of the serial returns pass

// torch's softmax over a 4-wide row (aten persistent softmax, one element per lane of a 4-lane
// group: max and sum by xor-butterfly, exp(x - max) / sum) and torch.log of the chosen entry.
__device__ inline void softmax4(const float* x, float p[4]) {
  const float m = fmaxf(fmaxf(x[0], x[2]), fmaxf(x[1], x[3]));
  float e[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) e[k] = expf(x[k] - m);
  const float s = (e[0] + e[2]) + (e[1] + e[3]);
#pragma unroll
  for (int k = 0; k < 4; ++k) p[k] = e[k] / s;
}

__global__ __launch_bounds__(32 * ACT_IPB) void k_ppo_act(MzPpoAct q) {
  const int slot = threadIdx.x >> 5, w = threadIdx.x & 31;
  const int i = blockIdx.x * ACT_IPB + slot;
  if (i >= q.B) return;
  const int t = q.t[i];
  if (t < 0 || t >= q.L) return;  // never outside the episode buffers
  const size_t row = (size_t)i * q.L + t;
  if (w < 6) {
    q.b_s6[row * 6 + w] = q.obs6[(size_t)i * 6 + w];
  } else if (w < 28) {
    q.b_w[row * 22 + (w - 6)] = q.bits[(size_t)i * 22 + (w - 6)];
  } else if (w == 28) {
    float x[4], p[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = q.logits[(size_t)i * q.ldl + k];
    softmax4(x, p);
    uint32_t u[4];
    mz_philox(q.seed, MZ_PPO_STREAM ^ ((uint64_t)(uint32_t)i << 32), q.counter, u);
    const float r = (float)(u[0] >> 8) * (1.0f / 16777216.0f);  // [0, 1), 24 bits
    // inverse CDF; the last entry with nonzero probability if rounding leaves r above the sum
    int a = -1;
    float c = 0.0f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      c += p[k];
      if (a < 0 && r < c) a = k;
    }
    if (a < 0)
      for (int k = 3; k >= 0; --k)
        if (p[k] > 0.0f) { a = k; break; }
    if (a < 0) a = 0;  // all-NaN logits: torch would raise; act 0 (the loss goes NaN anyway)
    q.b_a[row] = a;
    q.b_lp[row] = logf(p[a]);
    q.b_v[row] = q.value[(size_t)i * q.ldv];
    q.act_out[i] = a;
  }
}

// exclusive block scan of one int per thread (SCAN_T threads); returns the block total
__device__ inline int block_scan(int v, int* wsum, int& total) {
  const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
  int x = v;
#pragma unroll
  for (int o = 1; o < WAVE; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  __syncthreads();
  if (lane == WAVE - 1) wsum[wid] = x;
  __syncthreads();
  int before = 0, tot = 0;
  for (int k = 0; k < SCAN_T / WAVE; ++k) {
    const int s = wsum[k];
    if (k < wid) before += s;
    tot += s;
  }
  total = tot;
  return before + x - v;
}

__global__ __launch_bounds__(SCAN_T) void k_ppo_scan(MzPpoScan q) {
  __shared__ int wsum[SCAN_T / WAVE];
  int64_t base = *q.pool_fill;  // rows already in the pool
  int64_t rows_acc = 0;
  int fin_acc = 0;
  unsigned long long n_done = 0, n_win = 0, n_short = 0, n_over = 0;
  for (int c0 = 0; c0 < q.B; c0 += SCAN_T) {
    const int i = c0 + threadIdx.x;
    int len = 0, keep = 0;
    if (i < q.B) {
      int t = q.t[i];
      if (t >= 0 && t < q.L) q.b_r[(size_t)i * q.L + t] = q.reward64[i];
      t += 1;
      const bool term = q.term[i] != 0, done = term || q.trunc[i] != 0;
      if (done) {
        n_done += 1;
        n_win += term ? 1 : 0;
        if (t >= 2) {
          keep = 1;
          len = t;
        } else {
          n_short += 1;
        }
        t = 0;
      } else if (t >= q.L) {
        n_over += 1;  // the episode outgrew its record buffer: k_ppo_act would stop recording
        t = q.L - 1;  // keep t inside the buffer; the host raises on stats[3] at the next update
      }
      q.t[i] = t;
    }
    int tot_rows, tot_fin;
    const int off = block_scan(len, wsum, tot_rows);
    const int pos = block_scan(keep, wsum, tot_fin);
    if (keep) {
      const int k = fin_acc + pos;
      q.fin_id[k] = i;
      q.fin_off[k] = base + rows_acc + off;
      q.fin_len[k] = len;
    }
    rows_acc += tot_rows;
    fin_acc += tot_fin;
  }
  // counters: one wave reduction per quantity, added by thread 0
  __shared__ unsigned long long red[4][SCAN_T / WAVE];
  for (int o = WAVE / 2; o; o >>= 1) {
    n_done += __shfl_xor(n_done, o);
    n_win += __shfl_xor(n_win, o);
    n_short += __shfl_xor(n_short, o);
    n_over += __shfl_xor(n_over, o);
  }
  if ((threadIdx.x & (WAVE - 1)) == 0) {
    red[0][threadIdx.x / WAVE] = n_done;
    red[1][threadIdx.x / WAVE] = n_win;
    red[2][threadIdx.x / WAVE] = n_short;
    red[3][threadIdx.x / WAVE] = n_over;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long s[4] = {0, 0, 0, 0};
    for (int k = 0; k < SCAN_T / WAVE; ++k)
      for (int j = 0; j < 4; ++j) s[j] += red[j][k];
    *q.fin_count = fin_acc;
    *q.pool_fill = base + rows_acc;
    *q.pool_total += rows_acc;
    q.stats[0] += (long long)s[0];  // episodes
    q.stats[1] += (long long)s[1];  // wins
    q.stats[2] += (long long)s[2];  // dropped 1-step episodes
    q.stats[3] += (long long)s[3];  // record-buffer overflows (never, with L from max_steps' bound)
  }
}

__device__ inline double block_sum(double v, double* red) {
  for (int o = WAVE / 2; o; o >>= 1) v += __shfl_xor(v, o);
  __syncthreads();
  if ((threadIdx.x & (WAVE - 1)) == 0) red[threadIdx.x / WAVE] = v;
  __syncthreads();
  double s = 0.0;
  for (int k = 0; k < FIN_T / WAVE; ++k) s += red[k];  // same order in every thread
  return s;
}

__global__ __launch_bounds__(FIN_T) void k_ppo_finish(MzPpoFinish q) {
  __shared__ double rbuf[FIN_CH];
  __shared__ float fbuf[FIN_CH];
  __shared__ double red[FIN_T / WAVE];
  const int nfin = *q.fin_count;
  for (int k = blockIdx.x; k < nfin; k += gridDim.x) {
    const int i = q.fin_id[k];
    const int n = q.fin_len[k];
    const int64_t o = q.fin_off[k];
    if (o + n > q.cap) continue;  // overflow: nothing written (the host sees fill > capacity)
    const double* r = q.b_r + (size_t)i * q.L;
    float* ret = q.p_ret + o;
    float* adv = q.p_adv + o;
    // 1. returns, backwards in float64 (acc = r + acc * gamma), stored as float32; chunks of
    //    FIN_CH rewards staged in LDS, the recurrence run by thread 0
    double acc = 0.0, sum = 0.0;
    for (int end = n; end > 0; end -= FIN_CH) {
      const int beg = end > FIN_CH ? end - FIN_CH : 0;
      __syncthreads();
      for (int t = beg + threadIdx.x; t < end; t += FIN_T) rbuf[t - beg] = r[t];
      __syncthreads();
      if (threadIdx.x == 0) {
        for (int t = end - 1; t >= beg; --t) {
          acc = __dadd_rn(rbuf[t - beg], __dmul_rn(acc, q.gamma));
          fbuf[t - beg] = (float)acc;
        }
      }
      __syncthreads();
      for (int t = beg + threadIdx.x; t < end; t += FIN_T) {
        const float x = fbuf[t - beg];
        ret[t] = x;
        sum += (double)x;
      }
    }
    __syncthreads();  // ret[] written by this workgroup, read back below
    // 2. (R - mean) / std, unbiased std (torch.std): sums in float64, mean / std rounded to f32
    const double mean = block_sum(sum, red) / n;
    double ss = 0.0;
    for (int t = threadIdx.x; t < n; t += FIN_T) {
      const double d = (double)ret[t] - mean;
      ss += d * d;
    }
    const float m32 = (float)mean, s32 = (float)sqrt(block_sum(ss, red) / (n - 1));
    const float* v = q.b_v + (size_t)i * q.L;
    double asum = 0.0;
    for (int t = threadIdx.x; t < n; t += FIN_T) {
      const float rn = __fdiv_rn(__fsub_rn(ret[t], m32), s32);
      ret[t] = rn;
      const float a = __fsub_rn(rn, v[t]);  // calculate_advantages: returns - values
      adv[t] = a;
      asum += (double)a;
    }
    __syncthreads();
    // 3. (A - mean) / (std + 1e-8)
    const double amean = block_sum(asum, red) / n;
    double ass = 0.0;
    for (int t = threadIdx.x; t < n; t += FIN_T) {
      const double d = (double)adv[t] - amean;
      ass += d * d;
    }
    const float am32 = (float)amean;
    const float as32 = __fadd_rn((float)sqrt(block_sum(ass, red) / (n - 1)), 1e-8f);
    for (int t = threadIdx.x; t < n; t += FIN_T) adv[t] = __fdiv_rn(__fsub_rn(adv[t], am32), as32);
    // 4. the episode's states, actions and log-probs into the pool rows
    const size_t src = (size_t)i * q.L;
    for (int t = threadIdx.x; t < n; t += FIN_T) {
      q.p_a[o + t] = q.b_a[src + t];
      q.p_lp[o + t] = q.b_lp[src + t];
    }
    for (int e = threadIdx.x; e < n * 6; e += FIN_T) q.p_s6[o * 6 + e] = q.b_s6[src * 6 + e];
    for (int e = threadIdx.x; e < n * 22; e += FIN_T) q.p_w[o * 22 + e] = q.b_w[src * 22 + e];
  }
}

// ---- fused PPO head loss (optimize_model's loss, ppo_agent.py:188-203 via ActorCriticNet.evaluate
// :55-66): per row softmax / log_softmax / the action's log-prob / entropy and their gradients
// (k_ppo_head1), the [b, b] clipped surrogate (k_pair_surrogate, mz_optim.hip), then the total
// loss and d total / d logits, d value in one workgroup (k_ppo_head2, fixed-order sums).
constexpr float ENT_EPS = 1e-8f;

__global__ __launch_bounds__(256) void k_ppo_head1(MzPpoHead q) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= q.b) return;
  const float* z = q.logits + (size_t)i * q.ldl;
  float zz[4], mx = z[0];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    zz[k] = z[k];
    mx = fmaxf(mx, zz[k]);
  }
  float e[4], S = 0.0f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    e[k] = expf(zz[k] - mx);
    S += e[k];
  }
  const float lS = logf(S);
  float p[4], g[4], pg = 0.0f, ent = 0.0f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    p[k] = e[k] / S;
    const float lp = logf(p[k] + ENT_EPS);
    ent -= p[k] * lp;
    g[k] = -(lp + p[k] / (p[k] + ENT_EPS));  // d entropy / d p_k
    pg += p[k] * g[k];
  }
  const int a = (int)q.action[i];
  float za = zz[0];  // zz[a] by selects: a dynamic index would put zz in LDS (promote-alloca)
#pragma unroll
  for (int k = 1; k < 4; ++k) za = k == a ? zz[k] : za;
  q.lp_new[i] = za - mx - lS;  // log_softmax(z)[a]
  q.ent[i] = ent;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    q.p[(size_t)i * 4 + k] = p[k];
    q.dent[(size_t)i * 4 + k] = p[k] * (g[k] - pg);  // d entropy / d z_k through the softmax
  }
}

// one workgroup of 1,024: total = -(sum(part) / b^2 + coef * mean(ent)) + 0.5 * mean((v - ret)^2)
// and its gradients (d total / d lp_new_i = -adv_i dsum_i / b^2)
__global__ __launch_bounds__(1024) void k_ppo_head2(MzPpoHead q) {
  __shared__ double red[3][1024];
  const int tid = threadIdx.x, b = q.b;
  const float coef = *q.coef;
  const float inv_b = 1.0f / (float)b, inv_b2 = inv_b * inv_b;
  double sp = 0.0, se = 0.0, sv = 0.0;
  for (int i = tid; i < b; i += 1024) {
    const float v = q.value[(size_t)i * q.ldv], r = q.ret[i];
    const float dv = v - r;
    sp += q.part[i];
    se += q.ent[i];
    sv += (double)dv * dv;
    const float dlp = -q.adv[i] * q.dsum[i] * inv_b2;
    const int a = (int)q.action[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float pk = q.p[(size_t)i * 4 + k];
      q.dlogits[(size_t)i * q.ldg + k] =
          dlp * ((k == a ? 1.0f : 0.0f) - pk) - coef * inv_b * q.dent[(size_t)i * 4 + k];
    }
    q.dvalue[(size_t)i * q.ldvg] = dv * inv_b;  // 0.5 * d mean((v - r)^2) / dv
  }
  red[0][tid] = sp;
  red[1][tid] = se;
  red[2][tid] = sv;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if (tid < o) {
      red[0][tid] += red[0][tid + o];
      red[1][tid] += red[1][tid + o];
      red[2][tid] += red[2][tid + o];
    }
    __syncthreads();
  }
  if (tid == 0) {
    const double n = (double)b;
    *q.loss = (float)(-(red[0][0] / (n * n) + (double)coef * red[1][0] / n) + 0.5 * red[2][0] / n);
  }
}

}  // namespace

hipError_t mz_launch_ppo_act(const MzPpoAct& q, hipStream_t s) {
  if (q.B <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_ppo_act, dim3((q.B + ACT_IPB - 1) / ACT_IPB), dim3(32 * ACT_IPB), 0, s, q);
  return hipGetLastError();
}

hipError_t mz_launch_ppo_scan(const MzPpoScan& q, hipStream_t s) {
  if (q.B <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_ppo_scan, dim3(1), dim3(SCAN_T), 0, s, q);
  return hipGetLastError();
}

hipError_t mz_launch_ppo_finish(const MzPpoFinish& q, int max_episodes, hipStream_t s) {
  if (max_episodes <= 0) return hipSuccess;
  const int blocks = max_episodes < 2048 ? max_episodes : 2048;
  hipLaunchKernelGGL(k_ppo_finish, dim3(blocks), dim3(FIN_T), 0, s, q);
  return hipGetLastError();
}

hipError_t mz_launch_ppo_head(const MzPpoHead& q, float clip, hipStream_t s) {
  if (q.b <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_ppo_head1, dim3((q.b + 255) / 256), dim3(256), 0, s, q);
  const hipError_t e = mz_launch_pair_surrogate(q.lp_new, q.lp_old, q.adv, q.b, clip, q.part, q.dsum, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_ppo_head2, dim3(1), dim3(1024), 0, s, q);
  return hipGetLastError();
}
