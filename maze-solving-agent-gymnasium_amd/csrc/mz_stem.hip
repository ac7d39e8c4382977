// mz_stem.hip — the Q-network's conv stem for the LEARNER update, f32, forward and backward,
// straight from the replay's packed window bits.
//
// The reference's optimize_model (dqn_agent.py:121-157, ddqn_agent.py:113-152) runs the stem
// Conv2d(3->32, 3x3, pad 1) -> LeakyReLU -> [Dropout(0.2): DDQN, always in train mode, SURVEY
// Q13] -> MaxPool2d(2) -> flatten || obs6 (dqn_agent.py:47-57, ddqn_agent.py:18-52) in f32 on
// [B, 3, 15, 15] windows. Through PyTorch that is an f32 expansion of the window, MIOpen conv
// (+ NCHW<->NHWC transposes), separate activation / dropout / pooling passes over the 59 MB
// [2048, 32, 15, 15] conv output, and their backward passes: ~0.8 ms of a 1.65 ms update at
// batch 2,048. Here:
//
//   k_stem_fwd     one wave per 4 samples: the 22 window words -> padded 17-bit rows -> one
//                  27-bit patch word per conv position in LDS; the conv as an f32 MFMA GEMM
//                  (positions x 28 patch bits x 32 channels, exact products — the window is
//                  binary), + bias, LeakyReLU (x > 0 ? x : x * 0.01f), dropout (x * keep *
//                  scale, keep from a counter hash) and the max in torch's scan order (first
//                  strict maximum wins) on the accumulator registers, writing the f32 fc1 input
//                  row [feature c*49 + q (torch's flatten order) | obs6] and, when the caller
//                  needs the backward, one code byte per feature: the argmax position (2 bits)
//                  and its gradient class (0 dropped, 1 kept and a > 0, 2 kept and a <= 0);
//   k_stem_bwd     grid (sample chunk of 64, channel): the conv-output gradient at the argmax
//                  position, g * scale (dropout) then * 0.01f when a <= 0 (LeakyReLU backward),
//                  exactly torch's elementwise chain, accumulated into the 27 weight + 1 bias
//                  gradients of the channel over the chunk (the input is data: no input grad);
//                  wave shuffles + LDS reduce to one partial per (chunk, channel);
//   k_stem_reduce  the partials summed over chunks in a fixed order (deterministic).
//
// f32 throughout (the reference's precision); the conv / weight-gradient sums associate
// differently from MIOpen's, so results agree with the torch stem within f32 rounding.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mz_learner.h"

namespace {

constexpr int FEAT = 1568;   // 32 channels x 7 x 7 pooled positions
constexpr int NPOOL = 49;
constexpr int NOBS = 6;
constexpr int WW = 22;       // window words per sample (675 bits)
constexpr int PR = 17;       // padded rows per channel (rows 0 and 16 zero)
constexpr int CHUNK = 64;    // samples per backward workgroup
constexpr int NACC = 28;     // 27 weights + bias per channel

__device__ inline uint32_t hash32(uint32_t x) {  // lowbias32 (Wellons)
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

// window bits of nsamp samples -> padded rows: rows[s][ch][pr] holds grid row pr - 1 of channel
// ch with column c at bit c + 1 (bits 0 and 16 zero: the conv's zero padding)
__device__ inline void load_rows(const uint32_t* __restrict__ bits, int n, int n0, int nsamp,
                                 uint32_t (*wb)[WW], uint32_t (*rows)[3][PR]) {
  const int tid = threadIdx.x;
  for (int i = tid; i < nsamp * WW; i += blockDim.x) {
    const int s = i / WW, k = i - s * WW;
    wb[s][k] = n0 + s < n ? bits[(size_t)(n0 + s) * WW + k] : 0u;
  }
  __syncthreads();
  for (int i = tid; i < nsamp * 3 * PR; i += blockDim.x) {
    const int s = i / (3 * PR), rr = i - s * 3 * PR, ch = rr / PR, pr = rr - ch * PR;
    uint32_t v = 0u;
    if (pr >= 1 && pr <= 15) {
      const int f0 = ch * 225 + (pr - 1) * 15, j = f0 >> 5;
      const uint64_t w2 = ((uint64_t)(j + 1 < WW ? wb[s][j + 1] : 0u) << 32) | wb[s][j];
      v = ((uint32_t)(w2 >> (f0 & 31)) & 0x7FFFu) << 1;
    }
    rows[s][ch][pr] = v;
  }
  __syncthreads();
}

typedef __attribute__((ext_vector_type(4))) float f32x4;

// Forward, one workgroup (4 waves) per group of FG = 4 samples (4 x 49 pooled outputs = 49 MFMA
// row tiles of 16, dealt round-robin to the 4 waves), persistent over the groups. (One wave per
// group left a 1,024-row update pass with 256 waves on 256 CUs, each walking 49 tiles: 38 us,
// the same as 2,048 rows.) The conv is an f32 MFMA GEMM
// (v_mfma_f32_16x16x4_f32, exact f32 products, an fmaf chain per output): rows = conv positions,
// K = the 27 patch bits in torch's weight order k = ch*9 + ky*3 + kx (padded to 28: 7 MFMAs),
// columns = the 32 output channels (two 16-column tiles). The window is binary, so A is 0.0/1.0
// from one patch word per row, built once per group into LDS in A-row order: row i of tile t is
// pooled output 4t + i/4 of the group at 2x2 position i%4 — the C/D map (row = 4*(lane>>4) + reg)
// then hands every lane the 4 positions of one pool window for one channel, so LeakyReLU,
// dropout and the max (first strict maximum in (0,0) (0,1) (1,0) (1,1) order, torch's scan) run
// on registers. Dropout masks: the counter hash of the scalar kernel this replaced (same keys, so
// tests/test_stem.py regenerates them).
template <bool DROP, bool CODE>
__global__ __launch_bounds__(256) void k_stem_fwd(const uint32_t* __restrict__ bits,
                                                  const float* __restrict__ obs6, int n,
                                                  const float* __restrict__ w,
                                                  const float* __restrict__ b, uint32_t thresh,
                                                  float scale, const uint64_t* __restrict__ rng,
                                                  uint32_t salt, float* __restrict__ feat, int ld,
                                                  uint8_t* __restrict__ code) {
  constexpr int FG = 4, NQ = FG * NPOOL, NT = NQ / 4;  // 196 pooled outputs, 49 tiles
  __shared__ uint32_t wb[FG * WW];
  __shared__ uint32_t rows[FG * 3 * PR];
  __shared__ uint32_t patch[NQ * 4];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, kq = lane >> 4;
  // B operands: B[k = 4*kc + kq][c] = w[c][k] (0 for k = 27), c = col (tile 0) / 16 + col (tile 1)
  float bw0[7], bw1[7];
#pragma unroll
  for (int kc = 0; kc < 7; ++kc) {
    const int k = 4 * kc + kq;
    bw0[kc] = k < 27 ? w[col * 27 + k] : 0.0f;
    bw1[kc] = k < 27 ? w[(16 + col) * 27 + k] : 0.0f;
  }
  const float bias0 = b[col], bias1 = b[16 + col];
  uint32_t k0 = 0u, k1 = 0u;
  if (DROP) {
    const uint64_t key = *rng;  // device-side counter: a fresh mask per (graph-replayed) call
    k0 = (uint32_t)key ^ (salt * 0x9E3779B9u);
    k1 = (uint32_t)(key >> 32) + hash32(salt);
  }
  const int ngroups = (n + FG - 1) / FG;
  for (int grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    const int n0 = grp * FG;
    __syncthreads();  // the previous group's LDS fully consumed
    for (int i = tid; i < FG * WW; i += 256) {
      const int s = i / WW;
      wb[i] = n0 + s < n ? bits[(size_t)n0 * WW + i] : 0u;
    }
    __syncthreads();
    // padded rows: rows[(s*3 + ch)*PR + pr] = grid row pr - 1, column c at bit c + 1
    for (int i = tid; i < FG * 3 * PR; i += 256) {
      const int sc = i / PR, pr = i - sc * PR, s = sc / 3, ch = sc - s * 3;
      uint32_t v = 0u;
      if (pr >= 1 && pr <= 15) {
        const int f0 = ch * 225 + (pr - 1) * 15, j = f0 >> 5;
        const uint64_t w2 = ((uint64_t)(j + 1 < WW ? wb[s * WW + j + 1] : 0u) << 32) | wb[s * WW + j];
        v = ((uint32_t)(w2 >> (f0 & 31)) & 0x7FFFu) << 1;
      }
      rows[i] = v;
    }
    __syncthreads();
    // patch words in A-row order: patch[4*Q + r], Q = group pooled output, r = 2x2 position
    for (int p = tid; p < NQ * 4; p += 256) {
      const int Q = p >> 2, r = p & 3, s = Q / NPOOL, q = Q - s * NPOOL;
      const int y = 2 * (q / 7) + (r >> 1), x = 2 * (q % 7) + (r & 1);
      uint32_t pw = 0u;
#pragma unroll
      for (int ch = 0; ch < 3; ++ch)
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
          pw |= ((rows[(s * 3 + ch) * PR + y + ky] >> x) & 7u) << (ch * 9 + ky * 3);
      patch[p] = pw;
    }
    __syncthreads();
    for (int t = wid; t < NT; t += 4) {
      const uint32_t pw = patch[16 * t + col] >> kq;
      f32x4 acc0 = {bias0, bias0, bias0, bias0};
      f32x4 acc1 = {bias1, bias1, bias1, bias1};
#pragma unroll
      for (int kc = 0; kc < 7; ++kc) {
        const float a = (float)((pw >> (4 * kc)) & 1u);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bw0[kc], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bw1[kc], acc1, 0, 0, 0);
      }
      // this lane: pooled output Q = 4t + kq, channels col and 16 + col, positions r = 0..3
      const int Q = 4 * t + kq, s = Q / NPOOL, q = Q - s * NPOOL, nn = n0 + s;
      if (nn >= n) continue;
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const f32x4& acc = half ? acc1 : acc0;
        const int j = (half * 16 + col) * NPOOL + q;
        uint32_t h0 = 0u, h1 = 0u;
        if (DROP) {
          const uint32_t gid = 2u * ((uint32_t)nn * FEAT + j);
          h0 = hash32(hash32(gid ^ k0) + k1);
          h1 = hash32(hash32((gid + 1u) ^ k0) + k1);
        }
        float m = -__builtin_inff();
        int idx = 0, cls = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float a = acc[r];
          const float lk = a > 0.0f ? a : a * 0.01f;  // nn.LeakyReLU(negative_slope=0.01)
          bool kept = true;
          float v = lk;
          if (DROP) {
            const uint32_t u = ((r < 2 ? h0 : h1) >> (16 * (r & 1))) & 0xFFFFu;
            kept = u >= thresh;
            v = (lk * (kept ? 1.0f : 0.0f)) * scale;  // torch: src * mask * scale
          }
          if (v > m) {  // MaxPool2d: first strict maximum
            m = v;
            idx = r;
            cls = kept ? (a > 0.0f ? 1 : 2) : 0;
          }
        }
        feat[(size_t)nn * ld + j] = m;
        if (CODE) code[(size_t)nn * FEAT + j] = (uint8_t)(idx | (cls << 2));
      }
    }
    for (int i = tid; i < FG * NOBS; i += 256) {  // || obs6 (torch.cat((fw, s), 1))
      const int s = i / NOBS, k = i - s * NOBS, nn = n0 + s;
      if (nn < n) feat[(size_t)nn * ld + FEAT + k] = obs6[(size_t)nn * NOBS + k];
    }
  }
}

__global__ __launch_bounds__(256) void k_stem_bwd(const uint32_t* __restrict__ bits,
                                                  const uint8_t* __restrict__ code,
                                                  const float* __restrict__ g, int ld, int n,
                                                  float scale, float* __restrict__ partial) {
  __shared__ uint32_t wb[CHUNK][WW];
  __shared__ uint32_t rows[CHUNK][3][PR];
  __shared__ float red[4][NACC];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int chunk = blockIdx.x, c = blockIdx.y, n0 = chunk * CHUNK;
  load_rows(bits, n, n0, CHUNK, wb, rows);
  float acc[NACC];
#pragma unroll
  for (int k = 0; k < NACC; ++k) acc[k] = 0.0f;
  // every code byte / gradient this thread reads, loaded before any is used (one round trip
  // instead of one per item; the items are then summed in the same order)
  constexpr int IT = (CHUNK * NPOOL + 255) / 256;
  uint32_t cdv[IT];
  float gv[IT];
#pragma unroll
  for (int u = 0; u < IT; ++u) {
    const int i = tid + 256 * u, s = i / NPOOL, q = i - s * NPOOL, nn = n0 + s;
    cdv[u] = 0u;  // class 0: contributes nothing
    gv[u] = 0.0f;
    if (i < CHUNK * NPOOL && nn < n) {
      const int j = c * NPOOL + q;
      cdv[u] = code[(size_t)nn * FEAT + j];
      gv[u] = g[(size_t)nn * ld + j];
    }
  }
#pragma unroll
  for (int u = 0; u < IT; ++u) {
    const int i = tid + 256 * u, s = i / NPOOL, q = i - s * NPOOL;
    const uint32_t cd = cdv[u];
    const uint32_t cls = cd >> 2;
    if (cls == 0u) continue;  // dropped (or past the rows): dropout backward gives 0
    const float gs = gv[u] * scale;  // dropout backward: grad * mask * scale
    const float gc = cls == 1u ? gs : gs * 0.01f;     // LeakyReLU backward
    const int py = q / 7, px = q - py * 7;
    const int y = 2 * py + (int)((cd >> 1) & 1u), x = 2 * px + (int)(cd & 1u);
#pragma unroll
    for (int ch = 0; ch < 3; ++ch)
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const uint32_t b3 = (rows[s][ch][y + ky] >> x) & 7u;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx)
          if ((b3 >> kx) & 1u) acc[ch * 9 + ky * 3 + kx] += gc;
      }
    acc[27] += gc;
  }
#pragma unroll
  for (int k = 0; k < NACC; ++k) {
    float v = acc[k];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) red[wv][k] = v;
  }
  __syncthreads();
  if (tid < NACC)
    partial[((size_t)chunk * 32 + c) * NACC + tid] =
        ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
}

// advance (nullable): the dropout counter the forward read, advanced here for the next forward —
// the learner's nets read it in both forwards of an update and the source's backward moves it on,
// so no separate add launch per forward (agents/stem.py stem_features(advance="backward"))
__global__ void k_stem_reduce(const float* __restrict__ partial, int chunks, float* __restrict__ dw,
                              float* __restrict__ db, unsigned long long* advance) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (advance && t == 0) *advance = *advance + 1ull;
  if (t >= 32 * NACC) return;
  const int c = t / NACC, k = t - c * NACC;
  // 8 chunks' loads in flight before their adds (same order, so the same sums): the serial
  // load-add chain waited a round trip per chunk — 111 us per call under the acting kernels'
  // load against 12 us alone (profiles/r01l_train_kernel_stats.csv)
  const float* pp = partial + (size_t)c * NACC + k;
  const size_t cs = (size_t)32 * NACC;  // chunk stride
  float s = 0.0f;
  int ch = 0;
  for (; ch + 8 <= chunks; ch += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = pp[(size_t)(ch + u) * cs];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; ch < chunks; ++ch) s += pp[(size_t)ch * cs];
  if (k < 27) dw[c * 27 + k] = s;  // torch layout [32][3][3][3]: c*27 + ch*9 + ky*3 + kx
  else db[c] = s;
}

}  // namespace

int mz_stem_chunks(int n) { return (n + CHUNK - 1) / CHUNK; }

hipError_t mz_launch_stem_fwd(const uint32_t* bits, const float* obs6, int n, const float* w,
                              const float* b, float drop_p, const uint64_t* rng, uint32_t salt,
                              float* feat, int ld, uint8_t* code, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  // keep iff a 16-bit uniform >= thresh: P(drop) = thresh / 65536 (0.2 -> 13107)
  const uint32_t thresh = drop_p > 0.0f ? (uint32_t)(drop_p * 65536.0f + 0.5f) : 0u;
  const float scale = drop_p > 0.0f ? (float)(1.0 / (1.0 - (double)drop_p)) : 1.0f;
  int blocks = (n + 3) / 4;  // one workgroup per 4 samples
  if (blocks > 4096) blocks = 4096;
#define MZ_SF(D, C)                                                                              \
  hipLaunchKernelGGL((k_stem_fwd<D, C>), dim3(blocks), dim3(256), 0, s, bits, obs6, n, w, b,      \
                     thresh, D ? scale : 1.0f, rng, salt, feat, ld, code)
  if (thresh) { if (code) MZ_SF(true, true); else MZ_SF(true, false); }
  else { if (code) MZ_SF(false, true); else MZ_SF(false, false); }
#undef MZ_SF
  return hipGetLastError();
}

hipError_t mz_launch_stem_bwd(const uint32_t* bits, const uint8_t* code, const float* g, int ld,
                              int n, float drop_p, float* partial, float* dw, float* db,
                              hipStream_t s, uint64_t* advance) {
  const int chunks = mz_stem_chunks(n);
  if (chunks == 0) {
    hipError_t e = hipMemsetAsync(dw, 0, 32 * 27 * sizeof(float), s);
    if (e == hipSuccess) e = hipMemsetAsync(db, 0, 32 * sizeof(float), s);
    if (e != hipSuccess || !advance) return e;
    hipLaunchKernelGGL(k_stem_reduce, dim3(1), dim3(64), 0, s, partial, 0, dw, db,
                       reinterpret_cast<unsigned long long*>(advance));
    return hipGetLastError();
  }
  const float scale = drop_p > 0.0f ? (float)(1.0 / (1.0 - (double)drop_p)) : 1.0f;
  hipLaunchKernelGGL(k_stem_bwd, dim3(chunks, 32), dim3(256), 0, s, bits, code, g, ld, n, scale,
                     partial);
  hipLaunchKernelGGL(k_stem_reduce, dim3((32 * NACC + 255) / 256), dim3(256), 0, s, partial,
                     chunks, dw, db, reinterpret_cast<unsigned long long*>(advance));
  return hipGetLastError();
}
