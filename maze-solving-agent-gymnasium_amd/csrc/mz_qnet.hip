// mz_qnet.hip — fused conv stem of the Q-network for acting, read straight from window bits.
//
// The reference's acting forward (dqn_agent.py:113-116 -> DQN.forward :47-57; DDQN
// ddqn_agent.py:18-52) runs Conv2d(3->32, 3x3, pad 1) -> LeakyReLU -> [Dropout(0.2), DDQN, active
// because the nets never leave train mode, SURVEY Q13] -> MaxPool2d(2) -> flatten (1,568) and
// concatenates the 6-float observation. Through PyTorch that is ~10 kernels and ~4 GB of HBM
// traffic per 65,536-instance vector step (f32 window, NCHW transposes, bf16 conv output, separate
// activation / dropout / pool passes). Here one kernel reads the 88-byte packed window per instance
// (mz_step's window_bits) and writes the bf16 fc1 input row [conv features | obs6 | zero pad]:
// 3,200 B per instance, so the kernel is bound by that write.
//
// Conv as an MFMA GEMM: rows = conv output positions, K = the 27 patch bits (padded to 32),
// columns = 32 output channels (two 16x16x32 bf16 MFMAs). The window is binary, so the A operand
// is exact in bf16; weights are rounded to bf16 (the precision autocast gives them on the torch
// path). Rows are ordered so that the 4 positions of one 2x2 pooling window land in one lane's 4
// accumulator registers (C/D row = 4*(lane>>4) + reg): pooling is a register max, and because
// LeakyReLU is monotonic and the bias is per channel, pool(leaky(conv + b)) = leaky(max + b).
// With dropout the per-element keep decisions are applied before the max (dropout -> pool order).
// 4 instances x 49 pooled outputs = 49 row tiles of 16 per group, no padding waste.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mz_kernels.h"

namespace {

constexpr int WAVE = 64;
constexpr int IPG = 4;          // instances per group
constexpr int NPOOL = 49;       // 7 x 7 pooled positions
constexpr int NTILE = IPG * NPOOL / 4;  // 49 MFMA row tiles (4 pooled outputs each)
constexpr int CONV_OUT = 1568;  // 32 x 7 x 7
constexpr int PR = 17;          // padded rows per channel plane (rows 0 and 16 are zero)
constexpr int PCH = 4;          // planes per instance: 3 channels + 1 all-zero plane
constexpr int LD_MAX = 1600;

typedef __attribute__((ext_vector_type(8))) __bf16 frag_ab;
typedef __attribute__((ext_vector_type(4))) float frag_cd;

__device__ inline uint16_t bf16_bits(float f) {
  const __bf16 h = static_cast<__bf16>(f);  // round to nearest even
  return __builtin_bit_cast(uint16_t, h);
}

__device__ inline uint32_t hash32(uint32_t x) {  // lowbias32 (Wellons)
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

// Pooled + activated value of one channel from the lane's 4 accumulators (2x2 window).
// keep: 4 bits (bit r = position r kept); all ones without dropout.
__device__ inline float pool_act(const frag_cd& a, uint32_t keep, float scale) {
  const float slope = 0.01f;  // nn.LeakyReLU default negative_slope
  if (keep == 0xFu) {
    const float m = fmaxf(fmaxf(a[0], a[1]), fmaxf(a[2], a[3]));
    return scale * fmaxf(m, slope * m);
  }
  float m = -INFINITY;
  for (int r = 0; r < 4; ++r)
    if (keep & (1u << r)) m = fmaxf(m, a[r]);
  float v = keep ? scale * fmaxf(m, slope * m) : 0.0f;
  return fmaxf(v, 0.0f);  // at least one dropped element contributes 0
}

__global__ __launch_bounds__(WAVE) void k_qfront(const uint32_t* __restrict__ bits,
                                                 const float* __restrict__ obs6, int n,
                                                 const float* __restrict__ w,
                                                 const float* __restrict__ bias,
                                                 uint32_t drop_thresh, float drop_scale,
                                                 uint32_t key0, uint32_t key1,
                                                 uint16_t* __restrict__ out, int ld) {
  __shared__ uint32_t wb[IPG * 22];
  __shared__ uint32_t prow[IPG * PCH * PR];
  __shared__ uint32_t tab_a[NTILE * 16];  // per (tile, A row): plane-row offset | x << 16
  __shared__ uint32_t tab_c[NTILE * 4];   // per (tile, C row group): instance | q << 8
  __shared__ __attribute__((aligned(16))) uint16_t stage[IPG * LD_MAX];

  const int lane = threadIdx.x;
  const int g4 = lane >> 4, c16 = lane & 15;

  // B operand: lane holds W[c][k = 8*g4 + j] for c = c16 and c16 + 16 (k >= 27: zero).
  frag_ab b0, b1;
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * g4 + j;
    b0[j] = static_cast<__bf16>(k < 27 ? w[c16 * 27 + k] : 0.0f);
    b1[j] = static_cast<__bf16>(k < 27 ? w[(c16 + 16) * 27 + k] : 0.0f);
  }
  const float bias0 = bias[c16], bias1 = bias[c16 + 16];

  // The lane's K range 8*g4 .. 8*g4+7 covers patch rows m0 .. m0+3 (m = 3*channel + ky, 3 bits
  // each); m >= 9 falls on the zero plane.
  const int m0 = (8 * g4) / 3;
  int roff[4];
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + i;
    roff[i] = (m / 3) * PR + (m % 3);
  }
  const int selsh = 8 * g4 - 3 * m0;

  for (int i = lane; i < IPG * PCH * PR; i += WAVE) prow[i] = 0u;
  for (int i = lane; i < NTILE * 16; i += WAVE) {
    const int t = i >> 4, r = i & 15;
    const int Q = 4 * t + (r >> 2), inst = Q / NPOOL, q = Q - inst * NPOOL;
    const int py = q / 7, px = q - py * 7;
    const int y = 2 * py + ((r >> 1) & 1), x = 2 * px + (r & 1);
    tab_a[i] = (uint32_t)(inst * PCH * PR + y) | ((uint32_t)x << 16);
  }
  for (int i = lane; i < NTILE * 4; i += WAVE) {
    const int t = i >> 2, gq = i & 3;
    const int Q = 4 * t + gq, inst = Q / NPOOL, q = Q - inst * NPOOL;
    tab_c[i] = (uint32_t)inst | ((uint32_t)q << 8);
  }

  const int ngroups = (n + IPG - 1) / IPG;
  for (int grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    const int e0 = grp * IPG;
    const int ni = min(IPG, n - e0);
    __syncthreads();  // previous group's stage / planes fully consumed
    for (int i = lane; i < IPG * 22; i += WAVE)
      wb[i] = i < ni * 22 ? bits[(size_t)e0 * 22 + i] : 0u;
    __syncthreads();
    // window rows -> padded planes: bit 0 and bit 16 are the zero padding columns
    for (int i = lane; i < IPG * 45; i += WAVE) {
      const int inst = i / 45, rem = i - inst * 45, ch = rem / 15, y = rem - ch * 15;
      const int f0 = ch * 225 + y * 15, j = f0 >> 5;
      const uint64_t v = ((uint64_t)wb[inst * 22 + j + 1] << 32) | wb[inst * 22 + j];
      prow[(inst * PCH + ch) * PR + y + 1] = (((uint32_t)(v >> (f0 & 31))) & 0x7FFFu) << 1;
    }
    __syncthreads();

    for (int t = 0; t < NTILE; ++t) {
      const uint32_t ta = tab_a[t * 16 + c16];
      const uint32_t* pr = prow + (ta & 0xFFFFu);
      const int x = (int)(ta >> 16);
      uint32_t part = 0;
      for (int i = 0; i < 4; ++i) part |= ((pr[roff[i]] >> x) & 7u) << (3 * i);
      const uint32_t sel = part >> selsh;
      frag_ab a;
      for (int j = 0; j < 8; ++j) a[j] = ((sel >> j) & 1u) ? (__bf16)1.0f : (__bf16)0.0f;
      frag_cd acc0 = {bias0, bias0, bias0, bias0};
      frag_cd acc1 = {bias1, bias1, bias1, bias1};
      acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b1, acc1, 0, 0, 0);

      const uint32_t tc = tab_c[t * 4 + g4];
      const int inst = (int)(tc & 0xFFu), q = (int)(tc >> 8);
      uint32_t keep0 = 0xFu, keep1 = 0xFu;
      if (drop_thresh) {
        // element id = ((e * 32 + c) * 49 + q) * 4 + r; one hash per 2 positions (16 bits each)
        const uint32_t e = (uint32_t)(e0 + inst);
        const uint32_t id0 = ((e * 32u + (uint32_t)c16) * 49u + (uint32_t)q) * 2u;
        const uint32_t id1 = id0 + 16u * 49u * 2u;
        const uint32_t h[4] = {hash32(hash32(id0 ^ key0) + key1), hash32(hash32((id0 + 1) ^ key0) + key1),
                               hash32(hash32(id1 ^ key0) + key1), hash32(hash32((id1 + 1) ^ key0) + key1)};
        keep0 = ((h[0] & 0xFFFFu) >= drop_thresh) | (((h[0] >> 16) >= drop_thresh) << 1) |
                (((h[1] & 0xFFFFu) >= drop_thresh) << 2) | (((h[1] >> 16) >= drop_thresh) << 3);
        keep1 = ((h[2] & 0xFFFFu) >= drop_thresh) | (((h[2] >> 16) >= drop_thresh) << 1) |
                (((h[3] & 0xFFFFu) >= drop_thresh) << 2) | (((h[3] >> 16) >= drop_thresh) << 3);
      }
      const float v0 = pool_act(acc0, keep0, drop_scale);
      const float v1 = pool_act(acc1, keep1, drop_scale);
      stage[inst * ld + c16 * NPOOL + q] = bf16_bits(v0);
      stage[inst * ld + (c16 + 16) * NPOOL + q] = bf16_bits(v1);
    }
    // obs6 after the conv features, zero padding up to ld
    const int tail = ld - CONV_OUT;
    for (int i = lane; i < IPG * tail; i += WAVE) {
      const int inst = i / tail, k = i - inst * tail;
      const float v = (k < 6 && inst < ni) ? obs6[(size_t)(e0 + inst) * 6 + k] : 0.0f;
      stage[inst * ld + CONV_OUT + k] = bf16_bits(v);
    }
    __syncthreads();
    const int q16 = ld >> 3;
    for (int i = lane; i < ni * q16; i += WAVE) {
      const int inst = i / q16, k = i - inst * q16;
      reinterpret_cast<uint4*>(out + (size_t)(e0 + inst) * ld)[k] =
          reinterpret_cast<const uint4*>(stage + inst * ld)[k];
    }
  }
}

}  // namespace

hipError_t mz_launch_qfront(const uint32_t* bits, const float* obs6, int n, const float* w,
                            const float* b, float drop_p, uint64_t seed, uint64_t counter,
                            uint16_t* out, int ld, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  // keep iff a 16-bit uniform >= thresh: P(drop) = thresh / 65536 (0.2 -> 13107, 0.19999695)
  const uint32_t thresh = drop_p > 0.0f ? (uint32_t)(drop_p * 65536.0f + 0.5f) : 0u;
  const float scale = drop_p > 0.0f ? 1.0f / (1.0f - drop_p) : 1.0f;
  const uint64_t k = seed * 0x9E3779B97F4A7C15ull + counter * 0xD1B54A32D192ED03ull + 1;
  const int ngroups = (n + IPG - 1) / IPG;
  const int blocks = ngroups < 65536 ? ngroups : 65536;
  hipLaunchKernelGGL(k_qfront, dim3(blocks), dim3(WAVE), 0, s, bits, obs6, n, w, b, thresh, scale,
                     (uint32_t)k, (uint32_t)(k >> 32), out, ld);
  return hipGetLastError();
}
