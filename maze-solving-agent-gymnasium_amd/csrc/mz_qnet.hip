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
// columns = output channels (two 16x16x32 bf16 MFMAs: even channels, odd channels). The window is
// binary, so the A operand is exact in bf16 and comes from a 256-entry LDS table (8 patch bits ->
// the lane's 8 bf16 A elements, one ds_read_b128). Per group of 4 instances the window rows are
// first re-laid out column-interleaved (bit 3*col + channel), so the 27-bit patch of a position
// is three 9-bit slices (one per kernel row, K order 9*ky + 3*kx + ch); the patches are written
// to LDS in MFMA A-row order and the tile loop reads one word per lane. Weights are rounded to bf16 (the precision
// autocast gives them on the torch path). Rows are ordered so that the 4 positions of one 2x2
// pooling window land in one lane's 4 accumulator registers (C/D row = 4*(lane>>4) + reg):
// pooling is a register max, and because LeakyReLU is monotonic and the bias is per channel,
// pool(leaky(conv + b)) = leaky(max + b). With dropout the keep decisions apply before the max.
//
// Feature order is position-major: feat[q*32 + c] = pooled[c][q] (the torch flatten is c*49 + q;
// the caller permutes fc1's weight columns once, agents/fused.py). A lane then holds channels
// (2j, 2j+1) of one pooled position — one packed 4-byte store — and a wave's store per tile covers
// 4 positions x 64 B = 256 contiguous bytes: no LDS staging of the output.
// 4 instances x 49 pooled outputs = 49 row tiles of 16 per group, no padding waste.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mz_learner.h"

namespace {

constexpr int WAVE = 64;
constexpr int WPB = 4;          // waves per workgroup (one group of instances each; shared LUTs)
constexpr int IPG = 4;          // instances per group
constexpr int NPOOL = 49;       // 7 x 7 pooled positions
constexpr int NTILE = IPG * NPOOL / 4;  // 49 MFMA row tiles (4 pooled outputs each)
constexpr int CONV_OUT = 1568;  // 32 x 7 x 7
constexpr int PR = 17;          // padded window rows per instance (rows 0 and 16 are zero)

typedef __attribute__((ext_vector_type(8))) __bf16 frag_ab;
typedef __attribute__((ext_vector_type(4))) float frag_cd;

__device__ inline uint32_t bf16x2(float lo, float hi) {  // round to nearest even, packed
  uint32_t r;  // operands are VALU results (never MFMA outputs directly)
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}

__device__ inline uint32_t hash32(uint32_t x) {  // lowbias32 (Wellons)
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

// Pooled + activated value of one channel from the lane's 4 accumulators (one 2x2 window):
// leaky(max_r a_r). With dropout, MaxPool(Dropout(LeakyReLU(a))) = scale * leaky(max_r a'_r)
// where a'_r = a_r if kept else 0 (leaky(0) = 0, leaky and the scale are monotonic);
// h01 / h23: 16-bit uniforms of positions (0, 1) and (2, 3), kept iff >= thresh.
// (No inline asm on MFMA results: the hazard recognizer does not pad for it.)
__device__ inline float pool_act(const frag_cd& a) {
  const float m = fmaxf(fmaxf(a[0], a[1]), fmaxf(a[2], a[3]));
  return fmaxf(m, 0.01f * m);  // nn.LeakyReLU default negative_slope
}
__device__ inline float pool_act_drop(const frag_cd& a, uint32_t h01, uint32_t h23, uint32_t thresh,
                                      float scale) {
  const float a0 = (h01 & 0xFFFFu) >= thresh ? a[0] : 0.0f;
  const float a1 = (h01 >> 16) >= thresh ? a[1] : 0.0f;
  const float a2 = (h23 & 0xFFFFu) >= thresh ? a[2] : 0.0f;
  const float a3 = (h23 >> 16) >= thresh ? a[3] : 0.0f;
  const float m = fmaxf(fmaxf(a0, a1), fmaxf(a2, a3));
  return scale * fmaxf(m, 0.01f * m);
}

// LDS written and read by the same wave only (after the shared tables): a wave-scope fence orders
// it, no workgroup barrier needed.
__device__ inline void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <bool DROP>
__global__ __launch_bounds__(WAVE * WPB) __attribute__((amdgpu_waves_per_eu(4, 8)))
void k_qfront(const uint32_t* __restrict__ bits, const float* __restrict__ obs6,
              const int32_t* __restrict__ rows, const int32_t* __restrict__ count, int n,
              const float* __restrict__ w, const float* __restrict__ bias, uint32_t drop_thresh,
              float drop_scale, uint32_t key0, uint32_t key1, uint32_t* __restrict__ out, int ld) {
  __shared__ uint4 lut[256];                  // 8 patch bits -> 8 bf16 (0 / 1.0)
  __shared__ uint32_t spread[256];            // 8 bits -> bits at 3i (column interleave)
  __shared__ uint32_t wbs[WPB][IPG * 22];
  __shared__ uint64_t crows[WPB][IPG * PR];   // column-interleaved padded rows, bit 3*col + ch
  __shared__ uint32_t patches[WPB][IPG * NPOOL * 4];  // 27-bit patch per A row, A-row order

  const int lane = threadIdx.x & (WAVE - 1);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);  // wave-uniform (SGPR)
  uint32_t* wb = wbs[wid];
  uint64_t* crow = crows[wid];
  uint32_t* patch = patches[wid];
  const int g4 = lane >> 4, c16 = lane & 15;

  // B operand: lane holds W[c][k] for k = 8*g4 + j, c = 2*c16 (MFMA 0) and 2*c16 + 1 (MFMA 1).
  // K order k = 9*ky + 3*kx + ch (what the column-interleaved rows produce); torch's weight
  // layout is [c][ch][ky][kx].
  frag_ab b0, b1;
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * g4 + j;
    const int ky = k / 9, kx = (k % 9) / 3, ch = k % 3;
    const int wi = ch * 9 + ky * 3 + kx;
    b0[j] = static_cast<__bf16>(k < 27 ? w[(2 * c16) * 27 + wi] : 0.0f);
    b1[j] = static_cast<__bf16>(k < 27 ? w[(2 * c16 + 1) * 27 + wi] : 0.0f);
  }
  const float bias0 = bias[2 * c16], bias1 = bias[2 * c16 + 1];

  for (int i = threadIdx.x; i < 256; i += WAVE * WPB) {
    uint32_t v[4], sp = 0;
    for (int p = 0; p < 4; ++p)
      v[p] = (((i >> (2 * p)) & 1) ? 0x3F80u : 0u) | (((i >> (2 * p + 1)) & 1) ? 0x3F800000u : 0u);
    lut[i] = make_uint4(v[0], v[1], v[2], v[3]);
    for (int b = 0; b < 8; ++b) sp |= ((uint32_t)(i >> b) & 1u) << (3 * b);
    spread[i] = sp;
  }
  for (int i = lane; i < IPG * PR; i += WAVE) crow[i] = 0ull;  // padding rows 0, 16 stay zero
  __syncthreads();  // tables shared by the workgroup's waves

  const int ld2 = ld >> 1;  // row pitch in uint32 (bf16 pairs)
  if (count) n = min(n, *count);  // the row list's length, read on the device
  const int ngroups = (n + IPG - 1) / IPG;
  // the group's 88 window words, loaded one group ahead (2 per lane) to hide HBM latency;
  // with `rows`, output row i is instance rows[i] (the greedy-row list: only the rows that act
  // greedily, dqn_agent.py:104-116)
  auto word = [&](int g, int k) -> uint32_t {
    if (!rows) return bits[(size_t)g * IPG * 22 + k];
    const int inst = k / 22;
    return bits[(size_t)rows[g * IPG + inst] * 22 + (k - inst * 22)];
  };
  auto load_bits = [&](int g, uint32_t& x0, uint32_t& x1) {
    const int m = g < ngroups ? min(IPG, n - g * IPG) * 22 : 0;
    x0 = lane < m ? word(g, lane) : 0u;
    x1 = lane + WAVE < m ? word(g, lane + WAVE) : 0u;
  };
  uint32_t nb0, nb1;
  const int gstride = gridDim.x * WPB;
  load_bits(blockIdx.x * WPB + wid, nb0, nb1);
  for (int grp = blockIdx.x * WPB + wid; grp < ngroups; grp += gstride) {
    const int e0 = grp * IPG;
    const int ni = min(IPG, n - e0);
    wave_sync();  // previous group's rows / patches fully consumed
    wb[lane] = nb0;
    if (lane + WAVE < IPG * 22) wb[lane + WAVE] = nb1;
    load_bits(grp + gstride, nb0, nb1);
    wave_sync();
    // window row r of every channel -> one column-interleaved row (col c at bits 3(c+1) + ch)
    if (lane < IPG * 15) {
      const int inst = lane / 15, r = lane - inst * 15;
      uint64_t cr = 0;
      for (int ch = 0; ch < 3; ++ch) {
        const int f0 = ch * 225 + r * 15, j = f0 >> 5;
        const uint64_t v = ((uint64_t)wb[inst * 22 + j + 1] << 32) | wb[inst * 22 + j];
        const uint32_t row = (uint32_t)(v >> (f0 & 31)) & 0x7FFFu;
        const uint64_t sp = (uint64_t)spread[row & 0xFF] | ((uint64_t)spread[row >> 8] << 24);
        cr |= sp << (3 + ch);
      }
      crow[inst * PR + r + 1] = cr;
    }
    wave_sync();
    // patch words of conv positions y, x in 0..13 (the ones 2x2 pooling reads): 9 bits per ky
    if (lane < IPG * 14) {
      const int inst = lane / 14, y = lane - inst * 14;
      const uint64_t r0 = crow[inst * PR + y], r1 = crow[inst * PR + y + 1], r2 = crow[inst * PR + y + 2];
      const int qrow = inst * NPOOL + (y >> 1) * 7, srow = (y & 1) << 1;
#pragma unroll
      for (int x = 0; x < 14; ++x) {
        const uint32_t p = ((uint32_t)(r0 >> (3 * x)) & 0x1FFu) |
                           (((uint32_t)(r1 >> (3 * x)) & 0x1FFu) << 9) |
                           (((uint32_t)(r2 >> (3 * x)) & 0x1FFu) << 18);
        patch[(qrow + (x >> 1)) * 4 + (srow | (x & 1))] = p;
      }
    }
    wave_sync();
    uint32_t* og = out + (size_t)e0 * ld2;
    // stores through a buffer descriptor: 32-bit offsets, no 64-bit address math per tile
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(og, 0, ni * ld2 * 4, 0x00020000);
    // dropout streams of this lane for this group (never 0: xorshift32 fixed point)
    uint32_t rs[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)  // 4 independent streams: no serial chain between the draws
      rs[k] = DROP ? (hash32(hash32(((uint32_t)grp * WAVE + lane) * 4u + k) ^ key0) ^ key1) | 1u : 0u;

    // A row c16 of tile t = patch entry 16t + c16 (pooled output 4t + c16/4, position c16%4).
    // Two-stage prefetch: the A fragment of tile t+1 and the patch word of tile t+2 are read
    // from LDS while tile t's MFMAs and epilogue run.
    const int gsh = 8 * g4;
    const uint32_t rowskip4 = 4u * (uint32_t)(ld2 - NPOOL * 16);  // next instance's row, bytes
    uint32_t pw_next = patch[16 + c16];
    uint4 a_next = lut[(patch[c16] >> gsh) & 0xFFu];
    // fully unrolled (measured 58 us vs 64 us rolled at 65,536 instances): LDS offsets become
    // immediates and the prefetch registers rotate without moves
#pragma unroll
    for (int t = 0; t < NTILE; ++t) {
      const frag_ab a = __builtin_bit_cast(frag_ab, a_next);
      if (t + 1 < NTILE) a_next = lut[(pw_next >> gsh) & 0xFFu];
      if (t + 2 < NTILE) pw_next = patch[16 * (t + 2) + c16];
      frag_cd acc0 = {bias0, bias0, bias0, bias0};
      frag_cd acc1 = {bias1, bias1, bias1, bias1};
      acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b1, acc1, 0, 0, 0);

      // C rows of this lane: pooled output Qc = 4t + g4, channels 2*c16, 2*c16 + 1
      const int Qc = 4 * t + g4;
      const int ic = __umul24(Qc, 21) >> 10;  // Qc / 49 for Qc < 196
      float v0, v1;
      if (DROP) {
        // 8 decisions (2 channels x 4 positions) from 4 xorshift32 draws, 16 bits each
        uint32_t h[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          rs[k] ^= rs[k] << 13;
          rs[k] ^= rs[k] >> 17;
          rs[k] ^= rs[k] << 5;
          h[k] = rs[k];
        }
        v0 = pool_act_drop(acc0, h[0], h[1], drop_thresh, drop_scale);
        v1 = pool_act_drop(acc1, h[2], h[3], drop_thresh, drop_scale);
      } else {
        v0 = pool_act(acc0);
        v1 = pool_act(acc1);
      }
      // feat[q*32 + c] of instance ic, q = Qc - 49*ic: offset Qc*16 + ic*(ld2 - 49*16) + c16
      // (rows of instances >= ni fall outside the descriptor's range: the store is dropped)
      const uint32_t off = (uint32_t)(Qc * 64 + c16 * 4) + __umul24((uint32_t)ic, rowskip4);
      __builtin_amdgcn_raw_buffer_store_b32(bf16x2(v0, v1), rsrc, (int)off, 0, 0);
    }
    // obs6 after the conv features, zero padding up to ld (pairs of bf16)
    const int tail = (ld - CONV_OUT) >> 1;
    for (int i = lane; i < ni * tail; i += WAVE) {
      const int inst = i / tail, k = 2 * (i - inst * tail);
      const float* o = obs6 + (size_t)(rows ? rows[e0 + inst] : e0 + inst) * 6;
      const float lo = k < 6 ? o[k] : 0.0f, hi = k + 1 < 6 ? o[k + 1] : 0.0f;
      og[inst * ld2 + (CONV_OUT >> 1) + (k >> 1)] = bf16x2(lo, hi);
    }
  }
}

}  // namespace

hipError_t mz_launch_qfront(const uint32_t* bits, const float* obs6, const int32_t* rows,
                            const int32_t* count, int n, const float* w, const float* b,
                            float drop_p, uint64_t seed, uint64_t counter, uint16_t* out, int ld,
                            hipStream_t s) {
  if (n <= 0) return hipSuccess;
  // keep iff a 16-bit uniform >= thresh: P(drop) = thresh / 65536 (0.2 -> 13107, 0.19999695)
  const uint32_t thresh = drop_p > 0.0f ? (uint32_t)(drop_p * 65536.0f + 0.5f) : 0u;
  const float scale = drop_p > 0.0f ? 1.0f / (1.0f - drop_p) : 1.0f;
  const uint64_t k = seed * 0x9E3779B97F4A7C15ull + counter * 0xD1B54A32D192ED03ull + 1;
  const int ngroups = (n + IPG - 1) / IPG;
  const int nb = (ngroups + WPB - 1) / WPB;
  const int blocks = nb < 65536 ? nb : 65536;
  uint32_t* o = reinterpret_cast<uint32_t*>(out);
  if (thresh)
    hipLaunchKernelGGL(k_qfront<true>, dim3(blocks), dim3(WAVE * WPB), 0, s, bits, obs6, rows, count, n, w, b, thresh,
                       scale, (uint32_t)k, (uint32_t)(k >> 32), o, ld);
  else
    hipLaunchKernelGGL(k_qfront<false>, dim3(blocks), dim3(WAVE * WPB), 0, s, bits, obs6, rows, count, n, w, b, 0u,
                       1.0f, 0u, 0u, o, ld);
  return hipGetLastError();
}

// LeakyReLU in place on the bf16 output of the acting head's first Linear (65,536 x 1,024 per
// vector step; dqn_agent.py:52-57 nn.LeakyReLU): x > 0 ? x : x * slope in f32, rounded to bf16
// (round to nearest even) — torch's leaky_relu_ on bf16 element for element. 8 elements per
// 16-B load / store, grid-stride; torch's elementwise kernel moves these 268 MB at ~3.8 TB/s.
static __global__ __launch_bounds__(256) void k_leaky_bf16(uint4* __restrict__ x, int64_t n8,
                                                           float slope) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint4 v = x[i];
    uint32_t* w = &v.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float lo = __uint_as_float(w[k] << 16), hi = __uint_as_float(w[k] & 0xFFFF0000u);
      w[k] = bf16x2(lo > 0.0f ? lo : lo * slope, hi > 0.0f ? hi : hi * slope);
    }
    x[i] = v;
  }
}

hipError_t mz_launch_leaky_bf16(uint16_t* x, int64_t n, float slope, hipStream_t s) {
  const int64_t n8 = n >> 3;
  if (n8 == 0) return hipSuccess;
  int64_t blocks = (n8 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(k_leaky_bf16, dim3((unsigned)blocks), dim3(256), 0, s,
                     reinterpret_cast<uint4*>(x), n8, slope);
  return hipGetLastError();
}
