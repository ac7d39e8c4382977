// mz_optim.hip — the learner's parameter update as ONE launch over a flat f32 parameter buffer.
//
// The reference's optimize_model ends with (dqn_agent.py:152-157, ddqn_agent.py:148-152)
//     for param in source_net.parameters(): param.grad.data.clamp_(-1, 1)
//     optimizer.step()          # torch.optim.AdamW(lr), defaults betas (0.9, 0.999), eps 1e-8,
//                               # weight_decay 1e-2
// Through torch's multi-tensor path that is a clamp_min + clamp_max pass and a fused AdamW pass
// whose grids follow the 8 parameter tensors in 64 Ki-element chunks: ~35 workgroups for the
// 2,140,548 parameters, i.e. ~15 % of the CUs — 68-95 us per pass at batch 2,048
// (profiles/r01f_train_kernel_stats.csv). Here the parameters live in one flat buffer (the
// modules' parameters are views of it, agents/flat.py) and one grid-stride launch over float4s
// covers every element: read p, g, m, v (16 B each), write p, m, v and the clamped g — 112 B per
// 4 parameters, ~60 MB per step, HBM-bound.
//
// Per element, in torch's order (torch/optim/adamw.py single-tensor path):
//   g = clamp(g * grad_scale, -c, c)                     (NaN propagates like Tensor.clamp_)
//   p = p * (1 - lr * wd)
//   m = lerp(m, g, 1 - b1)                               (m + w * (g - m), w < 0.5)
//   v = v * b2 + (1 - b2) * g * g
//   p = p - (lr / (1 - b1^t)) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
// with t the step count after this step (read as step[0] + 1 by every workgroup; a one-thread
// launch behind it stores it back, so a captured HIP graph advances it on every replay) and lr
// read from the device (the cosine schedule writes it between replays).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>


#include "mz_learner.h"

// k_adamw's grid: 256 workgroups of 512 (grid-stride beyond). Round 2 published the step count
// from the workgroup that took the last of one same-address ticket per workgroup — each
// workgroup's fence + atomic round trip at the end of the launch (2,048 workgroups of 256: 78 us
// alone; 256: 20.4 us, ~5 us of it the ticket tail, profiles/ubench_ticket.hip,
// profiles/r05u/ticket.jsonl; two-level tickets no better). Now a one-thread launch behind
// k_adamw on the same stream advances it: the kernel boundary orders it after every
// workgroup's read.
#ifndef MZ_ADAMW_MAXWG
#define MZ_ADAMW_MAXWG 256
#endif
#ifndef MZ_ADAMW_TPB
#define MZ_ADAMW_TPB 512
#endif

namespace {

struct Segs {
  const float* g[MZ_OPT_MAX_SEGS];  // gradient of segment k: flat elements [off[k], off[k] + len[k])
  int64_t off[MZ_OPT_MAX_SEGS + 1];
  int n;
};

__global__ void k_step_publish(float* step) { step[0] = step[0] + 1.0f; }

__global__ __launch_bounds__(MZ_ADAMW_TPB) void k_adamw(float* __restrict__ p, float* __restrict__ m,
                                               float* __restrict__ v, Segs segs,
                                               const float* __restrict__ lr_dev,
                                               const float* step_dev, double b1,
                                               double b2, double eps_d, double wd, float clamp,
                                               float gscale, int write_grad) {
  // the per-step scalars as torch's eager AdamW forms them (Python doubles, then f32 operands)
  const double lr = (double)*lr_dev;
  const float t_next = step_dev[0] + 1.0f;
  const double t = (double)t_next;
  const double bc1 = 1.0 - pow(b1, t);
  const float step_size = (float)(lr / bc1);
  const float bc2_sqrt = (float)sqrt(1.0 - pow(b2, t));
  const float decay = (float)(1.0 - lr * wd);
  const float w1 = (float)(1.0 - b1), b2f = (float)b2, w2 = (float)(1.0 - b2), eps = (float)eps_d;
  const int64_t n4 = segs.off[segs.n] >> 2;  // every segment length is a multiple of 4
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = q << 2;
    int k = 0;
    while (k + 1 < segs.n && e >= segs.off[k + 1]) ++k;
    float4* gp = reinterpret_cast<float4*>(const_cast<float*>(segs.g[k]) + (e - segs.off[k]));
    float4 g4 = *gp;
    float4 p4 = reinterpret_cast<float4*>(p)[q];
    float4 m4 = reinterpret_cast<float4*>(m)[q];
    float4 v4 = reinterpret_cast<float4*>(v)[q];
    float* gs = &g4.x;
    float* ps = &p4.x;
    float* ms = &m4.x;
    float* vs = &v4.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float g = gs[j] * gscale;
      g = g < -clamp ? -clamp : (g > clamp ? clamp : g);
      gs[j] = g;
      float pj = ps[j] * decay;
      float mj = ms[j] + w1 * (g - ms[j]);
      float vj = vs[j] * b2f + w2 * (g * g);
      const float denom = sqrtf(vj) / bc2_sqrt + eps;
      pj = pj - step_size * (mj / denom);
      ps[j] = pj;
      ms[j] = mj;
      vs[j] = vj;
    }
    reinterpret_cast<float4*>(p)[q] = p4;
    reinterpret_cast<float4*>(m)[q] = m4;
    reinterpret_cast<float4*>(v)[q] = v4;
    if (write_grad) *gp = g4;  // the clamped gradient stays visible, as with clamp_ in place
  }
}

// ---- PPO's optimizer step (ppo_agent.py:232-236): clip_grad_norm_(params, 0.5), then AdamW
// with three parameter groups (actor lr, critic lr, their mean for the conv stem), as three
// launches over the flat buffer instead of torch's ~13 (per-tensor norms, stack, norm, clamp,
// foreach mul, a fused AdamW per group).
struct GSegs {
  const float* g[MZ_OPT_MAX_SEGS];
  int64_t off[MZ_OPT_MAX_SEGS + 1];
  int grp[MZ_OPT_MAX_SEGS];
  int n;
};

constexpr int SQ_BLOCKS = 512;

__global__ __launch_bounds__(256) void k_sqnorm(GSegs segs, float* __restrict__ partial) {
  __shared__ float red[4];
  float acc = 0.0f;
  for (int k = 0; k < segs.n; ++k) {
    const float* g = segs.g[k];
    const int64_t len = segs.off[k + 1] - segs.off[k];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < len;
         i += (int64_t)gridDim.x * blockDim.x) {
      const float x = g[i];
      acc += x * x;
    }
  }
  for (int o = 32; o; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
}

// coef = min(max_norm / (||g|| + 1e-6), 1) (clip_grad_norm_'s clip_coef_clamped), and the step
// count (the AdamW bias corrections of every group read it)
__global__ __launch_bounds__(SQ_BLOCKS) void k_clip_coef(const float* __restrict__ partial,
                                                         float max_norm, float* __restrict__ coef,
                                                         float* __restrict__ step) {
  __shared__ float red[SQ_BLOCKS / 64];
  float acc = partial[threadIdx.x];
  for (int o = 32; o; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.0f;
    for (int i = 0; i < SQ_BLOCKS / 64; ++i) s += red[i];
    const float c = max_norm > 0.0f ? max_norm / (sqrtf(s) + 1e-6f) : 1.0f;
    *coef = c < 1.0f ? c : 1.0f;
    *step += 1.0f;
  }
}

__global__ __launch_bounds__(256) void k_adamw_groups(float* __restrict__ p, float* __restrict__ m,
                                                      float* __restrict__ v, GSegs segs,
                                                      const float* __restrict__ lr_dev,
                                                      const float* __restrict__ step_dev,
                                                      const float* __restrict__ coef_dev,
                                                      double b1, double b2, double eps_d,
                                                      double wd) {
  const double t = (double)*step_dev;
  const double bc1 = 1.0 - pow(b1, t);
  const float bc2_sqrt = (float)sqrt(1.0 - pow(b2, t));
  const float w1 = (float)(1.0 - b1), b2f = (float)b2, w2 = (float)(1.0 - b2), eps = (float)eps_d;
  const float gscale = *coef_dev;
  const int64_t n4 = segs.off[segs.n] >> 2;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = q << 2;
    int k = 0;
    while (k + 1 < segs.n && e >= segs.off[k + 1]) ++k;
    const double lr = (double)lr_dev[segs.grp[k]];
    const float step_size = (float)(lr / bc1);
    const float decay = (float)(1.0 - lr * wd);
    float4* gp = reinterpret_cast<float4*>(const_cast<float*>(segs.g[k]) + (e - segs.off[k]));
    float4 g4 = *gp;
    float4 p4 = reinterpret_cast<float4*>(p)[q];
    float4 m4 = reinterpret_cast<float4*>(m)[q];
    float4 v4 = reinterpret_cast<float4*>(v)[q];
    float* gs = &g4.x;
    float* ps = &p4.x;
    float* ms = &m4.x;
    float* vs = &v4.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float g = gs[j] * gscale;  // clip_grad_norm_: g.mul_(clip_coef_clamped)
      gs[j] = g;
      float pj = ps[j] * decay;
      const float mj = ms[j] + w1 * (g - ms[j]);
      const float vj = vs[j] * b2f + w2 * (g * g);
      const float denom = sqrtf(vj) / bc2_sqrt + eps;
      pj = pj - step_size * (mj / denom);
      ps[j] = pj;
      ms[j] = mj;
      vs[j] = vj;
    }
    reinterpret_cast<float4*>(p)[q] = p4;
    reinterpret_cast<float4*>(m)[q] = m4;
    reinterpret_cast<float4*>(v)[q] = v4;
    *gp = g4;  // the clipped gradient stays visible, as with clip_grad_norm_ in place
  }
}

}  // namespace

hipError_t mz_launch_adamw_groups(float* p, float* m, float* v, const float* const* grads,
                                  const int64_t* seg_len, const int32_t* seg_group, int nseg,
                                  const float* lr, float* step, double b1, double b2, double eps,
                                  double wd, float max_norm, float* scratch, hipStream_t s) {
  GSegs sg{};
  sg.n = nseg;
  sg.off[0] = 0;
  for (int k = 0; k < nseg; ++k) {
    sg.g[k] = grads[k];
    sg.grp[k] = seg_group[k];
    sg.off[k + 1] = sg.off[k] + seg_len[k];
  }
  float* coef = scratch + SQ_BLOCKS;
  hipLaunchKernelGGL(k_sqnorm, dim3(SQ_BLOCKS), dim3(256), 0, s, sg, scratch);
  hipLaunchKernelGGL(k_clip_coef, dim3(1), dim3(SQ_BLOCKS), 0, s, scratch, max_norm, coef, step);
  const int64_t n4 = sg.off[nseg] >> 2;
  int blocks = (int)((n4 + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(k_adamw_groups, dim3(blocks), dim3(256), 0, s, p, m, v, sg, lr, step, coef, b1,
                     b2, eps, wd);
  return hipGetLastError();
}

hipError_t mz_launch_adamw(float* p, float* m, float* v, const float* const* grads,
                           const int64_t* seg_len, int nseg, const float* lr, float* step, double b1,
                           double b2, double eps, double wd, float clamp, float gscale,
                           int write_grad, hipStream_t s) {
  Segs sg{};
  sg.n = nseg;
  sg.off[0] = 0;
  for (int k = 0; k < nseg; ++k) {
    sg.g[k] = grads[k];
    sg.off[k + 1] = sg.off[k] + seg_len[k];
  }
  const int64_t n4 = sg.off[nseg] >> 2;
  int blocks = (int)((n4 + MZ_ADAMW_TPB - 1) / MZ_ADAMW_TPB);
  if (blocks > MZ_ADAMW_MAXWG) blocks = MZ_ADAMW_MAXWG;  // grid-stride beyond
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(k_adamw, dim3(blocks), dim3(MZ_ADAMW_TPB), 0, s, p, m, v, sg, lr, step, b1, b2, eps, wd,
                     clamp, gscale, write_grad);
  hipLaunchKernelGGL(k_step_publish, dim3(1), dim3(1), 0, s, step);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// The PPO clipped surrogate with the reference's [b, b] broadcast (ppo_agent.py:188-197: new
// log-probs [b] against old ones [b, 1], advantages [b] along the last dim):
//   L = mean_{j,i} min(r_ji a_i, clamp(r_ji, 1-c, 1+c) a_i),   r_ji = exp(lp_new[i] - lp_old[j])
// One workgroup per column i sums over j, without materialising the 4 M-element pair matrix:
//   part[i]  = sum_j min(r_ji a_i, clamp(r_ji) a_i)
//   dsum[i]  = sum_j r_ji * w_ji,  w = torch's gradient routing through min / clamp: 1/2 + 1/2 *
//              [1-c <= r <= 1+c] on a tie, 1 where r a < clamp(r) a, [1-c <= r <= 1+c] otherwise
// so dL/dlp_new[i] = a_i * dsum[i] / b^2 (the caller scales by the upstream gradient).
static __global__ __launch_bounds__(256) void k_pair_surrogate(const float* __restrict__ lp_new,
                                                               const float* __restrict__ lp_old,
                                                               const float* __restrict__ adv,
                                                               int b, float clip,
                                                               float* __restrict__ part,
                                                               float* __restrict__ dsum) {
  __shared__ float red[2][4];
  const int i = blockIdx.x, tid = threadIdx.x;
  const float li = lp_new[i], a = adv[i];
  const float lo = 1.0f - clip, hi = 1.0f + clip;
  float s = 0.0f, d = 0.0f;
  for (int j = tid; j < b; j += blockDim.x) {
    const float r = expf(li - lp_old[j]);
    const float s1 = r * a;
    const float rc = r < lo ? lo : (r > hi ? hi : r);
    const float s2 = rc * a;
    const float inside = (r >= lo && r <= hi) ? 1.0f : 0.0f;
    const float w = s1 == s2 ? 0.5f + 0.5f * inside : (s1 < s2 ? 1.0f : inside);
    s += s1 < s2 ? s1 : s2;
    d += r * w;
  }
  for (int o = 32; o >= 1; o >>= 1) {
    s += __shfl_xor(s, o);
    d += __shfl_xor(d, o);
  }
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = s;
    red[1][tid >> 6] = d;
  }
  __syncthreads();
  if (tid == 0) {
    part[i] = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
    dsum[i] = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
  }
}

hipError_t mz_launch_pair_surrogate(const float* lp_new, const float* lp_old, const float* adv,
                                    int b, float clip, float* part, float* dsum, hipStream_t s) {
  if (b <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pair_surrogate, dim3(b), dim3(256), 0, s, lp_new, lp_old, adv, b, clip,
                     part, dsum);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Column sums of a row-major f32 matrix g[n][ld] over its first m columns: the Linear bias
// gradient db = dY^T 1 of the learners' captured updates (agents/linear.py). rocBLAS's GEMV
// against a ones vector took ~20 us for [2,048 x 1,024] (plus the ones fill). Here 4 * CQ columns
// per workgroup of 1,024 threads (16-B loads, 4 columns per lane) and RG = 256 / CQ row groups,
// each summing rows rg, rg + RG, ... with 8 loads in flight; then the row groups' partials by a
// fixed-order tree in LDS (deterministic). 64 columns per workgroup (16 workgroups for fc1's 1,024
// bias columns, 64 serial partial adds at the end) kept most CUs idle: ~4 us per call.
#ifndef MZ_COLSUM_CQ
#define MZ_COLSUM_CQ 4  // column quads per workgroup
#endif
constexpr int CS_T = 1024;
constexpr int CS_RG = CS_T / MZ_COLSUM_CQ;  // row groups
static __global__ __launch_bounds__(CS_T) void k_colsum(const float* __restrict__ g, int n, int m,
                                                        int ld, float* __restrict__ out) {
  __shared__ float4 part[CS_RG][MZ_COLSUM_CQ];
  const int cq = threadIdx.x % MZ_COLSUM_CQ, rg = threadIdx.x / MZ_COLSUM_CQ;
  const int c = blockIdx.x * (4 * MZ_COLSUM_CQ) + cq * 4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < m) {
    // 8 rows' loads in flight before their adds: a load-add chain waited a round trip per row
    int r = rg;
    for (; r + 7 * CS_RG < n; r += 8 * CS_RG) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(g + (size_t)(r + CS_RG * u) * ld + c);
#pragma unroll
      for (int u = 0; u < 8; ++u) { s.x += v[u].x; s.y += v[u].y; s.z += v[u].z; s.w += v[u].w; }
    }
    for (; r < n; r += CS_RG) {
      const float4 v = *reinterpret_cast<const float4*>(g + (size_t)r * ld + c);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  part[rg][cq] = s;
  __syncthreads();
#pragma unroll
  for (int h = CS_RG / 2; h; h >>= 1) {
    if (rg < h) {
      const float4 u = part[rg + h][cq];
      s.x += u.x; s.y += u.y; s.z += u.z; s.w += u.w;
      part[rg][cq] = s;
    }
    __syncthreads();
  }
  if (rg == 0 && c < m) *reinterpret_cast<float4*>(out + c) = s;
}

hipError_t mz_launch_colsum(const float* g, int n, int m, int ld, float* out, hipStream_t s) {
  if (m <= 0) return hipSuccess;
  constexpr int cols = 4 * MZ_COLSUM_CQ;
  hipLaunchKernelGGL(k_colsum, dim3((m + cols - 1) / cols), dim3(CS_T), 0, s, g, n, m, ld, out);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// The replay sample of one learner update in one launch (DeviceReplay.sample, replay_memory.py
// :17-18 random.sample): rows idx[i] of the state / next-state arrays gathered into stacked
// [2b] buffers (state rows 0..b-1, next-state rows b..2b-1: the layout QNet.forward_rows
// takes), plus the actions and rewards. One 32-bit word per thread, rows in order.
static __global__ __launch_bounds__(256) void k_replay_gather(
    const int64_t* __restrict__ idx, int b, int64_t cap, const float* __restrict__ s6,
    const uint32_t* __restrict__ sw, const int64_t* __restrict__ a, const float* __restrict__ r,
    const float* __restrict__ s6n, const uint32_t* __restrict__ swn, float* __restrict__ o6,
    uint32_t* __restrict__ ow, int64_t* __restrict__ oa, float* __restrict__ orw) {
  constexpr int W = 6 + 22;  // words of one state row (obs6 | window bits)
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)b * (2 * W + 1)) return;
  const int i = (int)(t / (2 * W + 1)), k = (int)(t - (long)i * (2 * W + 1));
  const int64_t j = min(max(idx[i], (int64_t)0), cap - 1);  // never outside the ring
  if (k < 2 * W) {
    const bool nx = k >= W;
    const int q = nx ? k - W : k;
    const int row = nx ? b + i : i;
    if (q < 6) o6[(size_t)row * 6 + q] = (nx ? s6n : s6)[(size_t)j * 6 + q];
    else ow[(size_t)row * 22 + (q - 6)] = (nx ? swn : sw)[(size_t)j * 22 + (q - 6)];
  } else {
    oa[i] = a[j];
    orw[i] = r[j];
  }
}

hipError_t mz_launch_replay_gather(const int64_t* idx, int b, int64_t cap, const float* s6,
                                   const uint32_t* sw, const int64_t* a, const float* r,
                                   const float* s6n, const uint32_t* swn, float* o6, uint32_t* ow,
                                   int64_t* oa, float* orw, hipStream_t s) {
  if (b <= 0) return hipSuccess;
  const long total = (long)b * (2 * (6 + 22) + 1);
  hipLaunchKernelGGL(k_replay_gather, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, idx,
                     b, cap, s6, sw, a, r, s6n, swn, o6, ow, oa, orw);
  return hipGetLastError();
}
