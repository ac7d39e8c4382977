// mz_qact.hip — the DQN / DDQN acting forward (argmax_a Q_source(s), dqn_agent.py:113-116,
// ddqn_agent.py:98-110) from packed window bits, in two launches, f32-accurate on the bf16 MFMA.
//
// Precision. The reference acts in f32. A plain bf16 acting head agreed with the f32 argmax on
// 99.4 % of real trainer states (profiles/r03c_acting_precision.json: every miss a near-tie);
// emulated variants put the error in every layer. Here each GEMM operand x is split into
// x_hi = bf16(x), x_lo = bf16(x - x_hi), and a product is hi*hi + hi*lo + lo*hi with f32
// accumulation ("bf16x3", three v_mfma_f32_16x16x32_bf16 per tile): ~2^-16 relative per
// product, the f32 argmax on 100 % of those states, at ~5x the f32 MFMA's rate (gfx950 has no
// xf32; f32 MFMA runs at 1/16 of bf16). The conv's input is a binary window (exact in bf16), so
// only its weights are split.
//
//   k_qact1  conv stem + fc1: per workgroup 64 rows x 256 fc1 outputs, 4 waves (column quarters,
//            64 x 64 each). The K loop runs over the 49 pooled positions (32
//            channels each, the feature order q * 32 + c) and one chunk for obs6: the chunk's A
//            tile is produced in LDS by the conv (MFMA over 27 patch bits x 32 channels, pool by
//            register max, LeakyReLU, DDQN's dropout) while the previous chunk's fc1 MFMAs run —
//            the 1,574-wide feature row never leaves the chip. fc1's weights stream from L2:
//            workgroups are dealt round-robin over the 8 XCDs, and XCD x works on output tile
//            x / 2, so each XCD's L2 holds one 1.6 MB hi/lo weight slice. Output: the LeakyReLU
//            of fc1 as f32 rows.
//   k_qact2  fc2 + ReLU (DDQN) / LeakyReLU (DQN) + fc3 (f32) + argmax (first maximum, NaN as
//            torch.argmax) + the scatter of the action to the listed instance.
// Both read the row count from the device (the greedy-row list's length, mz_greedy_rows):
// workgroups past it exit, so no host round trip sizes the work.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "mz_learner.h"

namespace {

constexpr int WAVE = 64;
constexpr int CONV_OUT = 1568;     // 32 channels x 7 x 7 pooled positions
constexpr int K1 = 1600;           // fc1 input row as prepared: features | obs6 | zero pad
constexpr int N1 = 1024, N2 = 512;
constexpr int NCH = K1 / 32;       // 50 K chunks: 49 pooled positions + obs6
// k_qact1: 64 rows per workgroup, QW1 waves of 64 fc1 outputs each (64 QW1 outputs per
// workgroup); the 16 conv tiles of the 64 rows are spread over the waves. 4-wave workgroups let
// two independent workgroups share a CU (their barrier phases drift apart, so one runs MFMAs
// while the other waits on LDS / VALU work); 8 waves halve each wave's conv work instead: faster
// alone (all 65,536 rows 899 vs 1,053 us) but slower inside training, where the update stream's
// kernels share the CUs (53.0 / 53.2 vs 55.3 / 55.7 M env steps/s, same box interleaved,
// profiles/r03n_qact_waves_ab.json)
#ifndef MZ_QACT_WAVES
#define MZ_QACT_WAVES 4
#endif
constexpr int QW1 = MZ_QACT_WAVES;
constexpr int T1 = 64 * QW1;       // k_qact1 threads
constexpr int RT1 = 64;            // k_qact1 rows per workgroup
constexpr int NT1 = 64 * QW1;      // k_qact1 fc1 outputs per workgroup
constexpr int TPW = 16 / QW1;      // conv tiles (4 rows each) per wave
constexpr int NTL1 = N1 / NT1;     // fc1 output tiles
constexpr int XPT = 8 / NTL1;      // XCDs per output tile
// crow pitch per instance in u64: 17 padded rows (0 and 16 zero) + 3 spare. A conv operand read
// (ds_read2_b64 of rows y, y + 1 for the 4 instances of a tile) spans dword banks
// 2 (PR inst + y) .. + 5: at PR = 17 (34 dwords per instance) instances k and k + 2 overlapped
// (68 = 4 mod 64) — 2-way conflicts on every read; at 20 (40 dwords) the four ranges are disjoint
constexpr int PR = 20;
constexpr int AST = 40;            // k_qact1 LDS A-tile row stride in bf16 (32 + 8; 2-way on b128 reads)
// k_qact2 rows per workgroup: each wave streams its 256 KB of fc2 hi / lo fragments once per
// workgroup (2 MB per 64 rows of L2 traffic). 128 rows halve that but need 256 VGPRs with spills:
// alone no faster (greedy rows 0.466 vs 0.460 ms), inside training 58.2 vs 67.8-68.3 M env steps/s
// (profiles/r03_qprep/train.jsonl) — 64 stays
#ifndef MZ_QACT2_ROWS
#define MZ_QACT2_ROWS 64
#endif
constexpr int RT2 = MZ_QACT2_ROWS;
constexpr int MI2 = RT2 / 16;      // k_qact2 row fragments per wave

typedef __attribute__((ext_vector_type(8))) __bf16 frag_ab;
typedef __attribute__((ext_vector_type(4))) float frag_cd;
// staging registers as native vectors: HIP's uint4 / float4 structs held across loop iterations
// in small arrays defeat SROA, and the compiler then moves the arrays to LDS (promote-alloca: each
// prefetch became a store to LDS behind an s_waitcnt vmcnt(0))
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__device__ inline uint32_t bf16x2(float lo, float hi) {  // round to nearest even, packed
  uint32_t r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}
__device__ inline float bf16_round(float x) {  // x rounded to bf16, as f32 (RNE)
  return __uint_as_float(bf16x2(x, 0.0f) << 16);
}
// x = hi + lo + O(2^-17 x): the two bf16 halves, packed for a pair of adjacent elements
__device__ inline void split2(float x0, float x1, uint32_t& hi, uint32_t& lo) {
  hi = bf16x2(x0, x1);  // one packed conversion; its halves back as f32 by shift / mask
  const float h0 = __uint_as_float(hi << 16), h1 = __uint_as_float(hi & 0xFFFF0000u);
  lo = bf16x2(x0 - h0, x1 - h1);
}

__device__ inline uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
// DDQN's acting dropout (nn.Dropout(0.2) in train mode): the conv output (row, channel
// c, pooled position q, 2x2 position p) is kept iff a 16-bit uniform >= thresh, P(drop) = thresh /
// 65536; the uniforms come from one xorshift32 stream per (row, channel pair) seeded from the
// key and the row (k_qact1), so tests rebuild the masks (tests/test_qact.py).

__device__ inline float leaky(float x) { return x > 0.0f ? x : x * 0.01f; }

// acc[i][j] += A_i B_j over one 32-deep K chunk, split precision: hi*hi, then hi*lo, then lo*hi
// over all 16 tiles (product-major: consecutive MFMAs never share an accumulator)
template <int I>
__device__ inline void mfma_x3(const frag_ab (&ah)[I], const frag_ab (&al)[I], const uint4 (&bh)[4],
                               const uint4 (&bl)[4], frag_cd (&acc)[I][4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < I; ++i)
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], __builtin_bit_cast(frag_ab, bh[j]),
                                                          acc[i][j], 0, 0, 0);
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < I; ++i)
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], __builtin_bit_cast(frag_ab, bl[j]),
                                                          acc[i][j], 0, 0, 0);
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < I; ++i)
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], __builtin_bit_cast(frag_ab, bh[j]),
                                                          acc[i][j], 0, 0, 0);
}

// ---- the conv stem (shared by k_qact1 and k_qconv) --------------------------------------------
// LDS tables and the tile's window rows: spread (8 bits -> bits at 3i), wb (the rows' window
// bits), crow (column-interleaved padded window rows). Two barriers.
__device__ inline void conv_tables(const MzQAct& q, int r0, int nr, int tid, int nthr,
                                   uint32_t* spread, uint64_t* crow, uint32_t* wb) {
  for (int i = tid; i < 256; i += nthr) {
    uint32_t sp = 0;
    for (int k = 0; k < 8; ++k) sp |= ((uint32_t)(i >> k) & 1u) << (3 * k);
    spread[i] = sp;
  }
  for (int i = tid; i < RT1 * 22; i += nthr) {
    const int r = i / 22, k = i - r * 22;
    uint32_t v = 0;
    if (r < nr) {
      const int inst = q.rows ? q.rows[r0 + r] : r0 + r;
      v = q.bits[(size_t)inst * 22 + k];
    }
    wb[i] = v;
  }
  for (int r = tid; r < RT1; r += nthr) {
    crow[r * PR] = 0ull;
    crow[r * PR + 16] = 0ull;
  }
  __syncthreads();
  // window row y of every channel -> one column-interleaved row (col c at bits 3(c+1) + ch)
  for (int i = tid; i < RT1 * 15; i += nthr) {
    const int r = i / 15, y = i - r * 15;
    uint64_t cr = 0;
    for (int ch = 0; ch < 3; ++ch) {
      const int f0 = ch * 225 + y * 15, j = f0 >> 5;
      const uint64_t v = ((uint64_t)wb[r * 22 + j + 1] << 32) | wb[r * 22 + j];
      const uint32_t row = (uint32_t)(v >> (f0 & 31)) & 0x7FFFu;
      const uint64_t sp = (uint64_t)spread[row & 0xFF] | ((uint64_t)spread[row >> 8] << 24);
      cr |= sp << (3 + ch);
    }
    crow[r * PR + y + 1] = cr;
  }
  __syncthreads();
}

// this lane's conv B operands, hi and lo: W[c][k] for k = 8 g4 + j, c = 2 c16 (even) and 2 c16 + 1
// (odd); K order 9 ky + 3 kx + ch (the interleaved rows), torch's [c][ch][ky][kx]
struct ConvW {
  frag_ab be_h, be_l, bo_h, bo_l;
  float bias_e, bias_o;
};
__device__ inline ConvW conv_weights(const MzQAct& q, int g4, int c16) {
  ConvW cw;
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * g4 + j;
    const int ky = k / 9, kx = (k % 9) / 3, ch = k % 3;
    const int wi = ch * 9 + ky * 3 + kx;
    const float we = k < 27 ? q.conv_w[(2 * c16) * 27 + wi] : 0.0f;
    const float wo = k < 27 ? q.conv_w[(2 * c16 + 1) * 27 + wi] : 0.0f;
    const float weh = bf16_round(we), woh = bf16_round(wo);
    cw.be_h[j] = static_cast<__bf16>(weh);
    cw.be_l[j] = static_cast<__bf16>(we - weh);
    cw.bo_h[j] = static_cast<__bf16>(woh);
    cw.bo_l[j] = static_cast<__bf16>(wo - woh);
  }
  cw.bias_e = q.conv_b[2 * c16];
  cw.bias_o = q.conv_b[2 * c16 + 1];
  return cw;
}

// dropout draws (DDQN): per (row, channel pair, pooled position c) one xorshift32 stream of four
// draws, seeded lowbias32(base ^ c * 0x9E3779B9) | 1 from the (row, pair) base
// lowbias32(lowbias32(key ^ lowbias32(row)) ^ pair) | 1 — counter-based, so any chunk can be
// computed by any workgroup (k_qconv splits a row tile's chunks over several)
template <int TPWv>
__device__ inline void drop_seeds(const MzQAct& q, int r0, int w, int g4, int c16, uint32_t (&rs)[4]) {
#pragma unroll
  for (int tt = 0; tt < 4; ++tt) rs[tt] = 0u;
#pragma unroll
  for (int tt = 0; tt < TPWv; ++tt) {
    const uint32_t row = (uint32_t)(r0 + 4 * (TPWv * w + tt) + g4);
    rs[tt] = lowbias32(lowbias32(q.key ^ lowbias32(row)) ^ (uint32_t)c16) | 1u;
  }
}

// conv chunk c (pooled position c) of this wave's TPWv conv tiles (tile t: instances 4t .. 4t + 3;
// the MFMA's A row of this lane = c16: instance 4t + c16 / 4, position c16 % 4 of its 2x2 pooling
// window): LeakyReLU, DDQN's dropout, 2x2 max-pool, split into bf16 hi / lo. Out: for each tile
// tt, row il[tt] of the 64-row block, channels 2 c16 and 2 c16 + 1 packed as hi[tt] / lo[tt].
// 8 patch bits -> the MFMA operand's 8 bf16 (0 / 1.0), bit 2i in the low and bit 2i + 1 in the
// high half of word i: y = B | B << 15 puts bit 2i + 1 at 2i + 16, so word i = ((y >> 2i) & 0x10001)
// * 0x3F80. Arithmetic instead of a 256-entry LDS table: that table's data-dependent 16-B reads
// were most of k_qconv's LDS bank conflicts (16.0 M of 29.4 M LDS-active cycles,
// profiles/r04final_qact_pmc.json)
__device__ inline uint4 patch_bf16(uint32_t B) {
  const uint32_t y = B | (B << 15);
  return make_uint4((y & 0x10001u) * 0x3F80u, ((y >> 2) & 0x10001u) * 0x3F80u,
                    ((y >> 4) & 0x10001u) * 0x3F80u, ((y >> 6) & 0x10001u) * 0x3F80u);
}

template <bool DROP, int TPWv>
__device__ inline void conv_chunk_vals(const MzQAct& q, int c, int w, int g4, int c16,
                                       const uint64_t* crow, const ConvW& cw,
                                       uint32_t (&rs)[4], int (&il)[TPWv], uint32_t (&hi)[TPWv],
                                       uint32_t (&lo)[TPWv]) {
  const int py = c / 7, px = c - py * 7;
  frag_ab a[TPWv];
#pragma unroll
  for (int tt = 0; tt < TPWv; ++tt) {
    const int inst = 4 * (TPWv * w + tt) + (c16 >> 2), pos = c16 & 3;
    const int y = 2 * py + (pos >> 1), xx = 2 * px + (pos & 1);
    const uint64_t* cr = crow + inst * PR + y;
    const uint32_t p = ((uint32_t)(cr[0] >> (3 * xx)) & 0x1FFu) |
                       (((uint32_t)(cr[1] >> (3 * xx)) & 0x1FFu) << 9) |
                       (((uint32_t)(cr[2] >> (3 * xx)) & 0x1FFu) << 18);
    a[tt] = __builtin_bit_cast(frag_ab, patch_bf16((p >> (8 * g4)) & 0xFFu));
  }
  frag_cd e[TPWv], o[TPWv];
#pragma unroll
  for (int tt = 0; tt < TPWv; ++tt) {
    e[tt] = frag_cd{cw.bias_e, cw.bias_e, cw.bias_e, cw.bias_e};
    o[tt] = frag_cd{cw.bias_o, cw.bias_o, cw.bias_o, cw.bias_o};
  }
#pragma unroll
  for (int tt = 0; tt < TPWv; ++tt) {
    e[tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[tt], cw.be_h, e[tt], 0, 0, 0);
    o[tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[tt], cw.bo_h, o[tt], 0, 0, 0);
  }
#pragma unroll
  for (int tt = 0; tt < TPWv; ++tt) {
    e[tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[tt], cw.be_l, e[tt], 0, 0, 0);
    o[tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[tt], cw.bo_l, o[tt], 0, 0, 0);
  }
#pragma unroll
  for (int tt = 0; tt < TPWv; ++tt) {
    // lane: pooled output of instance 4t + g4, channels 2 c16 (e) and 2 c16 + 1 (o);
    // registers = the 4 positions of its 2x2 window
    il[tt] = 4 * (TPWv * w + tt) + g4;
    float ve, vo;
    if (DROP) {
      // MaxPool(Dropout(LeakyReLU(x))) = scale * leaky(max_r x'_r), x'_r = x_r kept, 0 dropped
      // (leaky(0) = 0; leaky and the scale are monotonic): the 4 draws of this chunk's stream,
      // low half -> even channel, high half -> odd
      float me = 0.0f, mo = 0.0f;
      uint32_t x = lowbias32(rs[tt] ^ ((uint32_t)c * 0x9E3779B9u)) | 1u;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        x ^= x << 13;
        x ^= x >> 17;
        x ^= x << 5;
        const float xe = (x & 0xFFFFu) >= q.drop_thresh ? e[tt][r] : 0.0f;
        const float xo = (x >> 16) >= q.drop_thresh ? o[tt][r] : 0.0f;
        me = r ? fmaxf(me, xe) : xe;
        mo = r ? fmaxf(mo, xo) : xo;
      }
      ve = leaky(me) * q.drop_scale;
      vo = leaky(mo) * q.drop_scale;
    } else {
      ve = leaky(fmaxf(fmaxf(e[tt][0], e[tt][1]), fmaxf(e[tt][2], e[tt][3])));
      vo = leaky(fmaxf(fmaxf(o[tt][0], o[tt][1]), fmaxf(o[tt][2], o[tt][3])));
    }
    split2(ve, vo, hi[tt], lo[tt]);
  }
}

// the obs6 chunk (features 1568..1573, then zeros) of row r, k pair k2 / 2: packed hi / lo
__device__ inline void obs_vals(const MzQAct& q, int r0, int nr, int r, int k2, uint32_t& hi,
                                uint32_t& lo) {
  float v0 = 0.0f, v1 = 0.0f;
  if (r < nr && k2 < 6) {
    const int inst = q.rows ? q.rows[r0 + r] : r0 + r;
    v0 = q.obs6[(size_t)inst * 6 + k2];
    v1 = q.obs6[(size_t)inst * 6 + k2 + 1];
  }
  split2(v0, v1, hi, lo);
}

// ---- k_qact1 -------------------------------------------------------------------------------
template <bool DROP>
__global__ __launch_bounds__(T1) __attribute__((amdgpu_waves_per_eu(2, 2)))
void k_qact1(MzQAct q, int row_tiles) {
  __shared__ uint32_t spread[256];             // 8 bits -> bits at 3i
  __shared__ uint64_t crow[RT1 * PR];          // column-interleaved padded window rows
  __shared__ uint32_t wb[RT1 * 22];            // the rows' window bits
  __shared__ __align__(16) uint16_t A[2][2][RT1 * AST];  // [buffer][hi, lo][row][k]

  const int tid = threadIdx.x, lane = tid & (WAVE - 1);
  const int w = __builtin_amdgcn_readfirstlane(tid / WAVE);
  const int g4 = lane >> 4, c16 = lane & 15;
  // XCD-aware tile map: workgroup b runs on XCD b % 8 (round-robin dispatch); XCD x computes
  // output tile x / XPT, so one XCD's L2 serves one weight slice
  const int b = blockIdx.x, x = b & 7;
  const int nt = x / XPT, rt = (b >> 3) * XPT + (x % XPT);
  if (rt >= row_tiles) return;
  const int m = q.count ? min(q.n, *q.count) : q.n;
  const int r0 = rt * RT1;
  if (r0 >= m) return;
  const int nr = min(RT1, m - r0);

  conv_tables(q, r0, nr, tid, T1, spread, crow, wb);
  const ConvW cw = conv_weights(q, g4, c16);
  uint32_t rs[4];
  if (DROP) drop_seeds<TPW>(q, r0, w, g4, c16, rs);

  // fc1 tile of this wave: rows 16 i, columns nt * NT1 + 64 cq + 16 j
  const int cq = w;
  const int col0 = nt * NT1 + cq * 64;
  frag_cd acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = frag_cd{0.0f, 0.0f, 0.0f, 0.0f};
  // B fragments of chunk c: lane reads W1[col][32 c + 8 g4 .. +8] (16 B, hi and lo images)
  uint4 bh[4], bl[4], nbh[4], nbl[4];
  // B fragments: the fragment-ordered image (k_qact_prepare) — this wave's 4 KB per chunk and
  // image are contiguous, lane-linear 16-B loads through buffer descriptors (32-bit offsets)
  const auto rs_h = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(q.w1h) + (size_t)nt * NT1 * K1,
                                                      0, NT1 * K1 * 2, 0x00020000);
  const auto rs_l = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(q.w1l) + (size_t)nt * NT1 * K1,
                                                      0, NT1 * K1 * 2, 0x00020000);
  const int boff = (cq * 4 * 64 + lane) * 16;  // bytes within a chunk's QW1 x 4 KB
  auto load_b = [&](int c, uint4* dh, uint4* dl) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int off = boff + c * (QW1 * 4 * 64 * 16) + j * (64 * 16);
      dh[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs_h, off, 0, 0));
      dl[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs_l, off, 0, 0));
    }
  };

  // stage 1 — the A tile of conv chunk c (pooled position c) into A[c & 1]
  auto conv_chunk = [&](int c) {
    int il[TPW];
    uint32_t hi[TPW], lo[TPW];
    conv_chunk_vals<DROP, TPW>(q, c, w, g4, c16, crow, cw, rs, il, hi, lo);
    uint16_t* Ah = A[c & 1][0];
    uint16_t* Al = A[c & 1][1];
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) {
      reinterpret_cast<uint32_t*>(Ah + il[tt] * AST)[c16] = hi[tt];
      reinterpret_cast<uint32_t*>(Al + il[tt] * AST)[c16] = lo[tt];
    }
  };
  // stage 1 of the last chunk: features 1568..1573 = obs6, then zeros
  auto obs_chunk = [&]() {
    uint16_t* Ah = A[(NCH - 1) & 1][0];
    uint16_t* Al = A[(NCH - 1) & 1][1];
    for (int i = tid; i < RT1 * 16; i += T1) {
      const int r = i >> 4, k2 = (i & 15) * 2;
      uint32_t hi, lo;
      obs_vals(q, r0, nr, r, k2, hi, lo);
      reinterpret_cast<uint32_t*>(Ah + r * AST)[k2 >> 1] = hi;
      reinterpret_cast<uint32_t*>(Al + r * AST)[k2 >> 1] = lo;
    }
  };
  // stage 2 — the fc1 MFMAs of chunk c from A[c & 1] and the B fragments in bh / bl. The A
  // fragments are read before stage 1 writes the other buffer (program order: the compiler
  // keeps LDS reads after earlier LDS writes), so the MFMAs can run beside stage 1's VALU work
  frag_ab ah[4], al[4];
  auto fc1_read = [&](int c) {
    const uint16_t* Ah = A[c & 1][0];
    const uint16_t* Al = A[c & 1][1];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 16 * i + c16;
      ah[i] = __builtin_bit_cast(frag_ab, *reinterpret_cast<const uint4*>(Ah + r * AST + 8 * g4));
      al[i] = __builtin_bit_cast(frag_ab, *reinterpret_cast<const uint4*>(Al + r * AST + 8 * g4));
    }
  };
  auto fc1_mfma = [&](const uint4 (&xh)[4], const uint4 (&xl)[4]) {
#ifndef MZ_QPROBE_NO_FC1
    mfma_x3(ah, al, xh, xl, acc);
#endif
  };

  // iteration c: the A tile of chunk c and the fc1 MFMAs of chunk c - 1, one barrier; the B
  // fragments of chunk c are loaded in iteration c and used in c + 1. The main loop body is one
  // basic block, so the scheduler can run the conv's LDS / VALU work between the fc1 MFMAs.
  // the scheduler's order for one half-iteration: the conv MFMAs as their inputs arrive, then
  // fc1's 48 MFMAs each with a few of the stage-1 VALU instructions (pool / dropout / split)
  // between them — the MFMA holds the SIMD's VALU issue for only 8 of its 16 cycles
  auto interleave = [&]() {
#ifdef MZ_QACT_INTERLEAVE
#pragma unroll
    for (int k = 0; k < 64; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, MZ_QACT_INTERLEAVE, 0);
    }
#endif
  };
  // B registers ping-pong between (bh, bl) and (nbh, nbl): the loop body is unrolled by two (conv
  // chunks 1 .. 48 and the fc1 steps of chunks 0 .. 47)
  load_b(0, bh, bl);
#ifndef MZ_QPROBE_NO_CONV
  conv_chunk(0);
#endif
  __syncthreads();
  static_assert((NCH - 2) % 2 == 0, "main loop unrolled by two");
  for (int c = 1; c < NCH - 1; c += 2) {
    fc1_read(c - 1);
    load_b(c, nbh, nbl);
#ifndef MZ_QPROBE_NO_CONV
    conv_chunk(c);
#endif
    fc1_mfma(bh, bl);
    interleave();
    __syncthreads();
    fc1_read(c);
    load_b(c + 1, bh, bl);
#ifndef MZ_QPROBE_NO_CONV
    conv_chunk(c + 1);
#endif
    fc1_mfma(nbh, nbl);
    interleave();
    __syncthreads();
  }
  // the obs6 chunk, then the last two fc1 steps
  fc1_read(NCH - 2);
  load_b(NCH - 1, nbh, nbl);
  obs_chunk();
  fc1_mfma(bh, bl);
  __syncthreads();
  fc1_read(NCH - 1);
  fc1_mfma(nbh, nbl);

  // epilogue: h1 = LeakyReLU(acc + b1) as f32 rows (list order); lane: column 16 j + c16 of the
  // wave's tile, rows 16 i + 4 g4 + reg
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = col0 + 16 * j + c16;
    const float bb = q.b1[col];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * i + 4 * g4 + r;
        if (row < nr) q.h1[(size_t)(r0 + row) * N1 + col] = leaky(acc[i][j][r] + bb);
      }
  }
}

// ---- the split forward: k_qconv (the conv stem once per 64-row tile) + k_qfc1 ----------------
// k_qact1 recomputes the conv stem (and DDQN's dropout draws) in each of its NTL1 = 4 output-tile
// workgroups of a row tile. The split computes it once: k_qconv writes each row tile's A chunks —
// exactly the hi / lo bf16 values k_qact1 puts in LDS — to a workspace after h1, feature tiles
// [row tile][chunk][hi, lo][64 rows][32] (8 KB per tile and chunk, 400 KB per tile), and k_qfc1
// runs k_qact1's fc1 loop with each chunk's A tile staged from there through LDS (one 16-B load
// of hi and of lo per thread per chunk). Same values, same MFMA order: the same Q values bit for
// bit.
constexpr int FT_CHUNK = 2 * RT1 * 32;  // uint16 per (tile, chunk)

// LDS A tiles of k_qfc1 / k_qact2: 64-B rows (32 bf16), the 16-B octets of row r permuted by
// oct ^ h((r >> 2) & 3), h = {0, 3, 2, 1}. The MFMA operand read (ds_read_b128, lane -> row
// 16 i + lane % 16, octet lane / 16) then hits 16 distinct 16-B bank slots in each of its four
// lane groups ({0-3, 12-15, 20-27}, ...: MI355X_MICROARCH.md, LDS), and the row-major stores stay
// conflict-free; k_qact1's padded 80-B rows (AST) were 2-way on every operand read.
#ifndef MZ_QA_SWZ
#define MZ_QA_SWZ 1
#endif
#if MZ_QA_SWZ
constexpr int ARS = 32;  // A-tile row stride (bf16)
__device__ inline int a_off(int r, int oct) { return r * ARS + 8 * (oct ^ ((4 - ((r >> 2) & 3)) & 3)); }
#else
constexpr int ARS = AST;
__device__ inline int a_off(int r, int oct) { return r * ARS + 8 * oct; }
#endif
// k_qfc1's output tiles per XCD: 1 (each XCD's L2 holds one 1.6 MB hi / lo weight slice; a row
// tile's A chunks are read by 4 XCDs), 2 or 4 (more weight slices per L2, fewer A reads from HBM)
#ifndef MZ_QFC1_NTX
#define MZ_QFC1_NTX 1
#endif
constexpr int QF_NTX = MZ_QFC1_NTX;
constexpr int QF_S = 8 * QF_NTX / NTL1;  // XCDs sharing one set of QF_NTX output tiles
static_assert(QF_S >= 1 && 8 % QF_S == 0, "output tiles per XCD");
// k_qfc1's chunks per LDS stage (one barrier per stage)
#ifndef MZ_QFC1_CPB
#define MZ_QFC1_CPB 2
#endif
constexpr int QF_CPB = MZ_QFC1_CPB;


// grid: row tiles x `groups` chunk groups (small batches: a row tile's 50 chunks over several
// workgroups, so that a few thousand rows still fill the chip)
template <bool DROP>
__global__ __launch_bounds__(T1) void k_qconv(MzQAct q, int row_tiles, int groups,
                                              uint16_t* __restrict__ feat) {
  __shared__ uint32_t spread[256];
  __shared__ uint64_t crow[RT1 * PR];
  __shared__ uint32_t wb[RT1 * 22];
  const int tid = threadIdx.x, lane = tid & (WAVE - 1);
  const int w = __builtin_amdgcn_readfirstlane(tid / WAVE);
  const int g4 = lane >> 4, c16 = lane & 15;
  const int rt = blockIdx.x / groups, grp = blockIdx.x - rt * groups;
  if (rt >= row_tiles) return;
  const int m = q.count ? min(q.n, *q.count) : q.n;
  const int r0 = rt * RT1;
  if (r0 >= m) return;
  const int nr = min(RT1, m - r0);
  const int per = (NCH + groups - 1) / groups;
  const int c0 = grp * per, c1 = min(NCH, c0 + per);
  conv_tables(q, r0, nr, tid, T1, spread, crow, wb);
  const ConvW cw = conv_weights(q, g4, c16);
  uint32_t rs[4];
  if (DROP) drop_seeds<TPW>(q, r0, w, g4, c16, rs);
  uint16_t* ft = feat + (size_t)rt * NCH * FT_CHUNK;
  for (int c = c0; c < min(c1, NCH - 1); ++c) {
    int il[TPW];
    uint32_t hi[TPW], lo[TPW];
    conv_chunk_vals<DROP, TPW>(q, c, w, g4, c16, crow, cw, rs, il, hi, lo);
    uint32_t* fh = reinterpret_cast<uint32_t*>(ft + (size_t)c * FT_CHUNK);
    uint32_t* fl = fh + RT1 * 16;
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) {
      fh[il[tt] * 16 + c16] = hi[tt];
      fl[il[tt] * 16 + c16] = lo[tt];
    }
  }
  if (c1 == NCH) {  // the obs6 chunk
    uint32_t* fh = reinterpret_cast<uint32_t*>(ft + (size_t)(NCH - 1) * FT_CHUNK);
    for (int i = tid; i < RT1 * 16; i += T1) {
      const int r = i >> 4, k2 = (i & 15) * 2;
      uint32_t hi, lo;
      obs_vals(q, r0, nr, r, k2, hi, lo);
      fh[i] = hi;
      fh[RT1 * 16 + i] = lo;
    }
  }
}

#ifndef MZ_QFC1_WPE
#define MZ_QFC1_WPE 2  // k_qfc1 waves per SIMD the register budget is sized for
#endif
__global__ __launch_bounds__(T1) __attribute__((amdgpu_waves_per_eu(MZ_QFC1_WPE, MZ_QFC1_WPE)))
void k_qfc1(MzQAct q, int row_tiles, const uint16_t* __restrict__ feat) {
  // [buffer][chunk of the stage][hi, lo][row][k]
  __shared__ __align__(16) uint16_t A[2][QF_CPB][2][RT1 * ARS];
  constexpr int NP = 2 * RT1 * 32 / 8 / T1;  // 16-B pieces of a chunk's A tile per thread
  static_assert(NP * T1 == 2 * RT1 * 32 / 8, "whole 16-B pieces per thread");
  const int tid = threadIdx.x, lane = tid & (WAVE - 1);
  const int w = __builtin_amdgcn_readfirstlane(tid / WAVE);
  const int g4 = lane >> 4, c16 = lane & 15;
  // workgroup b runs on XCD x = b % 8; XCD x cycles through QF_NTX output tiles of its set, one
  // row tile after another (consecutive workgroups on an XCD share the row tile's A chunks in L2)
  const int b = blockIdx.x, x = b & 7, k = b >> 3;
  const int nt = (x / QF_S) * QF_NTX + k % QF_NTX, rt = (k / QF_NTX) * QF_S + x % QF_S;
  if (rt >= row_tiles) return;
  const int m = q.count ? min(q.n, *q.count) : q.n;
  const int r0 = rt * RT1;
  if (r0 >= m) return;
  const int nr = min(RT1, m - r0);
  const int cq = w;
  const int col0 = nt * NT1 + cq * 64;
  frag_cd acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = frag_cd{0.0f, 0.0f, 0.0f, 0.0f};
  uint4 bh[4], bl[4], nbh[4], nbl[4];
  const auto rs_h = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(q.w1h) + (size_t)nt * NT1 * K1,
                                                      0, NT1 * K1 * 2, 0x00020000);
  const auto rs_l = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(q.w1l) + (size_t)nt * NT1 * K1,
                                                      0, NT1 * K1 * 2, 0x00020000);
  const int boff = (cq * 4 * 64 + lane) * 16;
  // B fragments of chunk c (clamped: past the last chunk a load re-reads chunk NCH - 1, unused)
  auto load_b = [&](int c, uint4* dh, uint4* dl) {
    c = min(c, NCH - 1);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int off = boff + c * (QW1 * 4 * 64 * 16) + j * (64 * 16);
      dh[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs_h, off, 0, 0));
      dl[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs_l, off, 0, 0));
    }
  };
  // A staging: thread tid <-> 16-B piece tid of the chunk's hi and lo halves (row tid / 4, k
  // octet tid % 4)
  const u32x4* fsrc = reinterpret_cast<const u32x4*>(feat + (size_t)rt * NCH * FT_CHUNK);
  frag_ab ah[4], al[4];
  auto fc1_read = [&](int buf, int sub) {
    const uint16_t* Ah = A[buf][sub][0];
    const uint16_t* Al = A[buf][sub][1];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 16 * i + c16;
      ah[i] = __builtin_bit_cast(frag_ab, *reinterpret_cast<const uint4*>(Ah + a_off(r, g4)));
      al[i] = __builtin_bit_cast(frag_ab, *reinterpret_cast<const uint4*>(Al + a_off(r, g4)));
    }
  };
  // A tiles staged through LDS (one 16-B piece of hi and of lo per thread and chunk), each stage
  // (QF_CPB chunks) loaded into registers two stages ahead of its LDS store (sets s0 / s1): all
  // waves read the same 8 KB per chunk, so LDS staging beats per-wave fragment loads (70.7-71.0 vs
  // 73.0-73.4 M env steps/s in training), and the two-chunk distance beats one (74.5-74.9 vs
  // 73.0-73.4 M; the forward alone 1.04 vs 1.10 ms at 65,536 rows) — profiles/r04l/ — with the Q
  // values bit for bit the same. Piece p of a chunk: half p / 256 (hi, lo), row (p % 256) / 4, k
  // octet p % 4; thread tid takes pieces tid + k T1. Stage loads are clamped like load_b.
  constexpr int NST = NCH / QF_CPB;  // stages
  static_assert(NST * QF_CPB == NCH, "whole stages");
  u32x4 s0[QF_CPB][NP], s1[QF_CPB][NP];
  auto ld = [&](int sg, u32x4 (&r)[QF_CPB][NP]) {
    sg = min(sg, NST - 1);
#pragma unroll
    for (int h = 0; h < QF_CPB; ++h)
#pragma unroll
      for (int k = 0; k < NP; ++k)
        r[h][k] = fsrc[(size_t)(sg * QF_CPB + h) * (FT_CHUNK / 8) + tid + k * T1];
  };
  auto st = [&](int buf, const u32x4 (&r)[QF_CPB][NP]) {
#pragma unroll
    for (int h = 0; h < QF_CPB; ++h)
#pragma unroll
      for (int k = 0; k < NP; ++k) {
        const int pc = tid + k * T1, idx = pc & 255;
        *reinterpret_cast<u32x4*>(A[buf][h][pc >> 8] + a_off(idx >> 2, idx & 3)) = r[h][k];
      }
  };
  // One stage: its chunks' MFMAs from LDS buffer sg & 1 (chunk 2j + 1 of the stage's pairs on the
  // B set nbh / nbl, the others on bh / bl; each set reloaded two chunks ahead right after the
  // MFMAs that read it), then stage sg + 1 from `nxt` into the other buffer and stage sg + 3
  // into `nxt`. B fragments are two chunks ahead, A tiles two stages.
  auto stage = [&](int sg, u32x4 (&nxt)[QF_CPB][NP]) {
#pragma unroll
    for (int h = 0; h < QF_CPB; ++h) {
      const int c = sg * QF_CPB + h;
      fc1_read(sg & 1, h);
      if ((c & 1) == 0) {
        mfma_x3(ah, al, bh, bl, acc);
        load_b(c + 2, bh, bl);
      } else {
        mfma_x3(ah, al, nbh, nbl, acc);
        load_b(c + 2, nbh, nbl);
      }
      if (QF_CPB > 1) __builtin_amdgcn_sched_barrier(0);  // each reload right after its MFMAs
    }
    st((sg + 1) & 1, nxt);  // (the last stage's store fills a buffer no one reads again)
    ld(sg + 3, nxt);
    __syncthreads();
  };
  // prologue in the loop's load order (A stage 1, B chunks 0 and 1, A stage 2; sched_barrier
  // keeps the compiler from regrouping them): s_waitcnt counts are merged over the loop's entry
  // and back edge, and a prologue with the A tiles last made every iteration wait for all but 2
  // loads. Loads inside the loop are unconditional for the same reason (a conditional load made
  // it wait vmcnt(0) before each iteration's first MFMA).
  ld(0, s0);
  st(0, s0);
  ld(1, s1);
  __builtin_amdgcn_sched_barrier(0);
  load_b(0, bh, bl);
  load_b(1, nbh, nbl);
  __builtin_amdgcn_sched_barrier(0);
  ld(2, s0);
  __syncthreads();
  int sg = 0;
  for (; sg + 1 < NST; sg += 2) {
    stage(sg, s1);
    stage(sg + 1, s0);
  }
  if (sg < NST) stage(sg, s1);
  // epilogue: as k_qact1
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = col0 + 16 * j + c16;
    const float bb = q.b1[col];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * i + 4 * g4 + r;
        if (row < nr) q.h1[(size_t)(r0 + row) * N1 + col] = leaky(acc[i][j][r] + bb);
      }
  }
}

// ---- k_qact2 -------------------------------------------------------------------------------
template <bool RELU>
__global__ __launch_bounds__(512) void k_qact2(MzQAct q) {
  __shared__ __align__(16) uint16_t A[2][1][2][RT2 * ARS];  // [buffer][chunk][hi, lo]
  __shared__ float part[8][RT2][4];
  const int tid = threadIdx.x, lane = tid & (WAVE - 1);
  const int w = __builtin_amdgcn_readfirstlane(tid / WAVE);
  const int g4 = lane >> 4, c16 = lane & 15;
  const int m = q.count ? min(q.n, *q.count) : q.n;
  const int r0 = blockIdx.x * RT2;
  if (r0 >= m) return;
  const int nr = min(RT2, m - r0);
  const int col0 = 64 * w;  // this wave's 64 fc2 outputs

  // A chunk c (32 columns of h1 for the RT2 rows): thread -> (rows tid / 8 + 64 u, 4 columns)
  constexpr int AU = RT2 / 64;
  const int ar = tid >> 3, ak = (tid & 7) * 4;
  struct AV { f32x4 v[AU]; };
  auto load_a = [&](int c) -> AV {
    AV a;
#pragma unroll
    for (int u = 0; u < AU; ++u)
      // rows past the count re-read the last row (their results are not stored): no branch
      a.v[u] = *reinterpret_cast<const f32x4*>(q.h1 + (size_t)(r0 + min(ar + 64 * u, nr - 1)) * N1 + 32 * c + ak);
    return a;
  };
  auto store_a = [&](int buf, int sub, const AV& a) {
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      uint32_t h0, l0, h1, l1;
      split2(a.v[u].x, a.v[u].y, h0, l0);
      split2(a.v[u].z, a.v[u].w, h1, l1);
      const int o = a_off(ar + 64 * u, ak >> 3) + (ak & 7);
      uint32_t* ph = reinterpret_cast<uint32_t*>(A[buf][sub][0] + o);
      uint32_t* pl = reinterpret_cast<uint32_t*>(A[buf][sub][1] + o);
      ph[0] = h0; ph[1] = h1;
      pl[0] = l0; pl[1] = l1;
    }
  };
  uint4 bh[4], bl[4], nbh[4], nbl[4];
  // B fragments from the fragment-ordered fc2 image: [chunk][wave][j][lane][8]
  const auto rs_h = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(q.w2h), 0, N2 * N1 * 2,
                                                      0x00020000);
  const auto rs_l = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(q.w2l), 0, N2 * N1 * 2,
                                                      0x00020000);
  const int boff = (w * 4 * 64 + lane) * 16;
  auto load_b = [&](int c, uint4* dh, uint4* dl) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int off = boff + c * (8 * 4 * 64 * 16) + j * (64 * 16);
      dh[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs_h, off, 0, 0));
      dl[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs_l, off, 0, 0));
    }
  };
  frag_cd acc[MI2][4];
#pragma unroll
  for (int i = 0; i < MI2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = frag_cd{0.0f, 0.0f, 0.0f, 0.0f};
  constexpr int NC2 = N1 / 32;
  auto chunk_mfma = [&](int buf, int sub, const uint4 (&b_h)[4], const uint4 (&b_l)[4]) {
    const uint16_t* Ah = A[buf][sub][0];
    const uint16_t* Al = A[buf][sub][1];
#pragma unroll
    for (int h = 0; h < MI2; h += 4) {  // four row fragments at a time (register pressure)
      frag_ab ah[4], al[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 16 * (h + i) + c16;
        ah[i] = __builtin_bit_cast(frag_ab, *reinterpret_cast<const uint4*>(Ah + a_off(r, g4)));
        al[i] = __builtin_bit_cast(frag_ab, *reinterpret_cast<const uint4*>(Al + a_off(r, g4)));
      }
      mfma_x3<4>(ah, al, b_h, b_l, *reinterpret_cast<frag_cd(*)[4][4]>(&acc[h]));
    }
  };
  // one chunk ahead, one barrier per chunk. Measured and not kept, all faster alone and slower
  // inside training (the update stream's kernels share the CUs): h1 chunks and fc2 fragments two
  // chunks ahead (MFMA busy 0.43 -> 0.47; 71.0 / 71.0 vs 75.3 / 74.9 M env steps/s,
  // profiles/r04p/), two chunks per LDS stage (0.50 -> 0.51; 72.1 / 72.7 vs 75.8 / 76.4 M,
  // profiles/r04t/)
  store_a(0, 0, load_a(0));
  load_b(0, bh, bl);
  AV na = {};
  __syncthreads();
  for (int c = 0; c < NC2; ++c) {
    if (c + 1 < NC2) {
      na = load_a(c + 1);
      load_b(c + 1, nbh, nbl);
    }
    chunk_mfma(c & 1, 0, bh, bl);
    if (c + 1 < NC2) {
      store_a((c + 1) & 1, 0, na);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bh[j] = nbh[j];
        bl[j] = nbl[j];
      }
    }
    __syncthreads();
  }

  // h2 = act(acc + b2) in f32; fc3 partial sums over this wave's 64 columns, per row and action,
  // four row fragments at a time
  float b2v[4], w3v[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = col0 + 16 * j + c16;
    b2v[j] = q.b2[col];
#pragma unroll
    for (int a = 0; a < 4; ++a) w3v[j][a] = q.w3[a * N2 + col];
  }
#pragma unroll
  for (int i0 = 0; i0 < MI2; i0 += 4) {
    float s[4][4][4];  // [i][reg][action]
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int a = 0; a < 4; ++a) s[i][r][a] = 0.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float h = acc[i0 + i][j][r] + b2v[j];
          const float hv = RELU ? fmaxf(h, 0.0f) : leaky(h);
#pragma unroll
          for (int a = 0; a < 4; ++a) s[i][r][a] += hv * w3v[j][a];
        }
    // sum over the 16 lanes of a row group (columns), fixed butterfly order
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          float v = s[i][r][a];
          v += __shfl_xor(v, 1);
          v += __shfl_xor(v, 2);
          v += __shfl_xor(v, 4);
          v += __shfl_xor(v, 8);
          s[i][r][a] = v;
        }
    if (c16 == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int a = 0; a < 4; ++a) part[w][16 * (i0 + i) + 4 * g4 + r][a] = s[i][r][a];
    }
  }
  __syncthreads();
  if (tid < nr) {
    float qv[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      float v = 0.0f;
      for (int k = 0; k < 8; ++k) v += part[k][tid][a];
      qv[a] = v + q.b3[a];
    }
    int best = 0;  // torch.argmax: the first maximum, a NaN counts as the maximum
    float bv = qv[0];  // (a scalar: qv[best] is a dynamic index the compiler moves to LDS)
#pragma unroll
    for (int a = 1; a < 4; ++a)
      if (!isnan(bv) && (isnan(qv[a]) || qv[a] > bv)) {
        best = a;
        bv = qv[a];
      }
    const int row = r0 + tid;
    const int inst = q.rows ? q.rows[row] : row;
    if (q.greedy) q.greedy[inst] = best;
    if (q.q_out) *reinterpret_cast<float4*>(q.q_out + (size_t)row * 4) =
        make_float4(qv[0], qv[1], qv[2], qv[3]);
  }
}

// ---- weight preparation ----------------------------------------------------------------------
// fc1 [1024][1574] (torch order: feature c * 49 + q, then obs6) and fc2 [512][1024] -> hi / lo bf16
// images in MFMA fragment order: element ((((tile * NCH + chunk) * 4 + wave) * 4 + j) * 64 + lane)
// * 8 + e of the fc1 image is W1[output tile * 256 + 64 wave + 16 j + lane % 16][feature 32 chunk +
// 8 (lane / 16) + e] (kernel feature order q * 32 + c, obs6 at 1568, zero pad to 1600); the fc2 image
// is [chunk 32][wave 8][j][lane][8]. A wave's B fragments for one chunk are then 4 KB contiguous
// per image: one fully coalesced 1 KB load per 16-column tile instead of 16 rows x 64 B.
// fc1: one workgroup per PREP_ROWS rows of a 16-row fragment block (output tile, wave, j): its
// contiguous rows of W1 (6.3 KB each) are read coalesced into LDS, then each thread turns 8
// features of one lane of one chunk into a 16-B hi and a 16-B lo store. (A per-element version — W1 gathered at the conv
// features' stride of 49 floats, 2-B stores — took 23 us per update inside training.)
// PREP_ROWS rows of one 16-row fragment block per workgroup: 4 -> 256 workgroups, one per CU (8
// rows gave 128 — half the chip idle while the learner's update waits on the images)
#ifndef MZ_PREP_ROWS
#define MZ_PREP_ROWS 4
#endif
constexpr int PREP_ROWS = MZ_PREP_ROWS;
static_assert(16 % PREP_ROWS == 0, "rows of a fragment block per workgroup");
constexpr int PREP_LD = CONV_OUT + 6;  // 1574: W1's row length
__global__ __launch_bounds__(256) void k_qact_prep1(const float* __restrict__ w1,
                                                    uint16_t* __restrict__ w1h,
                                                    uint16_t* __restrict__ w1l) {
  __shared__ float rows[PREP_ROWS * PREP_LD];
  const int r0 = blockIdx.x * PREP_ROWS;
  const float4* src = reinterpret_cast<const float4*>(w1 + (size_t)r0 * PREP_LD);
  for (int i = threadIdx.x; i < PREP_ROWS * PREP_LD / 4; i += 256)
    reinterpret_cast<float4*>(rows)[i] = src[i];
  __syncthreads();
  const int nt = r0 / NT1, cq = (r0 % NT1) / 64, j = (r0 % 64) / 16, sub = (r0 % 16) / PREP_ROWS;
  // (chunk, lane) pairs of this workgroup's rows: lanes whose row in the block (lane % 16) is one
  // of them, for each of the 4 lane groups (lane / 16: the chunk's 8-feature slice)
  for (int p = threadIdx.x; p < NCH * 4 * PREP_ROWS; p += 256) {
    const int c = p / (4 * PREP_ROWS), rr = p % PREP_ROWS;
    const int lane = ((p / PREP_ROWS) & 3) * 16 + sub * PREP_ROWS + rr;
    const float* row = rows + rr * PREP_LD;
    uint32_t hi[4], lo[4];
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      float v[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int f = 32 * c + 8 * (lane >> 4) + e + u;  // kernel feature order
        const int sf = f < CONV_OUT ? (f & 31) * 49 + (f >> 5) : f;
        v[u] = f < CONV_OUT + 6 ? row[sf] : 0.0f;
      }
      split2(v[0], v[1], hi[e >> 1], lo[e >> 1]);
    }
    const size_t o = ((((size_t)nt * NCH + c) * QW1 + cq) * 4 + j) * 64 + lane;  // in 8-element units
    reinterpret_cast<uint4*>(w1h)[o] = make_uint4(hi[0], hi[1], hi[2], hi[3]);
    reinterpret_cast<uint4*>(w1l)[o] = make_uint4(lo[0], lo[1], lo[2], lo[3]);
  }
}

// fc2: one thread per (chunk, wave, j, lane): 8 consecutive inputs of one output row (two float4
// loads) -> a 16-B hi and a 16-B lo store
__global__ __launch_bounds__(256) void k_qact_prep2(const float* __restrict__ w2,
                                                    uint16_t* __restrict__ w2h,
                                                    uint16_t* __restrict__ w2l) {
  const int o = blockIdx.x * 256 + threadIdx.x;  // [chunk 32][wave 8][j 4][lane 64]
  if (o >= N2 * N1 / 8) return;
  const int lane = o & 63, j = (o >> 6) & 3, wv = (o >> 8) & 7, c = o >> 11;
  const int r = 64 * wv + 16 * j + (lane & 15), k = 32 * c + 8 * (lane >> 4);
  const float4* src = reinterpret_cast<const float4*>(w2 + (size_t)r * N1 + k);
  const float4 a = src[0], b = src[1];
  uint32_t hi[4], lo[4];
  split2(a.x, a.y, hi[0], lo[0]);
  split2(a.z, a.w, hi[1], lo[1]);
  split2(b.x, b.y, hi[2], lo[2]);
  split2(b.z, b.w, hi[3], lo[3]);
  reinterpret_cast<uint4*>(w2h)[o] = make_uint4(hi[0], hi[1], hi[2], hi[3]);
  reinterpret_cast<uint4*>(w2l)[o] = make_uint4(lo[0], lo[1], lo[2], lo[3]);
}

}  // namespace

int mz_qact_row_tiles(int n) { return (n + RT1 - 1) / RT1; }

// the workspace mz_qact takes: h1 [n][1024] f32, then the split forward's feature tiles
int64_t mz_qact_ws_floats(int n) {
  const int64_t rt = (n + RT1 - 1) / RT1;
  return (int64_t)n * N1 + rt * NCH * FT_CHUNK / 2;
}

// MZ_QACT_FUSED=1 at build time: k_qact1 (conv recomputed per output tile) instead of the split
#ifndef MZ_QACT_FUSED
#define MZ_QACT_FUSED 0
#endif

hipError_t mz_launch_qact(const MzQAct& q, int relu, hipStream_t s) {
  if (q.n <= 0) return hipSuccess;
  const int rt = (q.n + RT1 - 1) / RT1;
  // 8 workgroups per XPT row tiles: XCD x takes output tile x / XPT of row tile XPT k + x % XPT
  const int blocks1 = 8 * ((rt + XPT - 1) / XPT);
  if (MZ_QACT_FUSED) {
    if (q.drop_thresh)
      hipLaunchKernelGGL(k_qact1<true>, dim3(blocks1), dim3(T1), 0, s, q, rt);
    else
      hipLaunchKernelGGL(k_qact1<false>, dim3(blocks1), dim3(T1), 0, s, q, rt);
  } else {
    uint16_t* feat = reinterpret_cast<uint16_t*>(q.h1 + (size_t)q.n * N1);
    int groups = 1;  // chunk groups per row tile: >= ~512 workgroups (at most 10 chunks apart)
    while (groups < 5 && rt * groups < 512) ++groups;
    if (q.drop_thresh)
      hipLaunchKernelGGL(k_qconv<true>, dim3(rt * groups), dim3(T1), 0, s, q, rt, groups, feat);
    else
      hipLaunchKernelGGL(k_qconv<false>, dim3(rt * groups), dim3(T1), 0, s, q, rt, groups, feat);
    hipLaunchKernelGGL(k_qfc1, dim3(8 * QF_NTX * ((rt + QF_S - 1) / QF_S)), dim3(T1), 0, s, q, rt, feat);
  }
  const int blocks2 = (q.n + RT2 - 1) / RT2;
  if (relu)
    hipLaunchKernelGGL(k_qact2<true>, dim3(blocks2), dim3(512), 0, s, q);
  else
    hipLaunchKernelGGL(k_qact2<false>, dim3(blocks2), dim3(512), 0, s, q);
  return hipGetLastError();
}

hipError_t mz_launch_qact_prepare(const float* w1, const float* w2, uint16_t* w1h, uint16_t* w1l,
                                  uint16_t* w2h, uint16_t* w2l, hipStream_t s) {
  hipLaunchKernelGGL(k_qact_prep1, dim3(N1 / PREP_ROWS), dim3(256), 0, s, w1, w1h, w1l);
  hipLaunchKernelGGL(k_qact_prep2, dim3(N2 * N1 / 8 / 256), dim3(256), 0, s, w2, w2h, w2l);
  return hipGetLastError();
}
