// mz_gemm.hip — the learners' f32 GEMMs on the bf16 MFMA in split precision (bf16x3).
//
// The reference trains its nets in f32 (dqn_agent.py:121-157, ppo_agent.py:206-237); the learner
// updates here are GEMM-bound (the PPO minibatch step's 18 GEMMs and the DQN update's fc layers,
// profiles/r03o_ppo_kernel_stats.csv). gfx950 runs f32 matrix products at the f32 VECTOR rate
// (157 TFLOP/s, 1/16 of bf16): C = A B^T is computed here as
//     A = Ah + Al,  B = Bh + Bl  (bf16 hi / lo halves, x - hi - lo = O(2^-17 x))
//     C = Ah Bh^T + Ah Bl^T + Al Bh^T        (three bf16 MFMAs per product, f32 accumulate)
// which drops only Al Bl^T (2^-16 relative) — the measured max error against float64 is within
// 2x of hipBLASLt's own f32 GEMM (profiles/r03o_gemm_x3.json) — at 3/16 of the f32 MFMA cost.
//
// C[m][n] = act(sum_k A(m,k) B(n,k) + bias[n]), A(m,k) = a[m*a_rs + k*a_ks] with one of the two
// strides 1 (AK: k contiguous; else m contiguous), the same for B. These cover the three products
// of a Linear layer without copies: Y = X W^T (A = X k-contig, B = W k-contig), dX = dY W
// (A = dY k-contig, B(k_out, n) = W[n][k_out]: row-contig), dW = dY^T X (A(n, m) = dY[m][n]
// row-contig, B(k_out, m) = X[m][k_out] row-contig).
//
// Two passes: k_split writes each operand as a zero-padded bf16 hi / lo image [rows][Kp] (k
// contiguous, Kp = K rounded up to 64; a row-contiguous operand is transposed on the way — loads
// coalesced along its contiguous dimension), then k_gemm_x3 runs the product over the images:
// 128 x 128 outputs per 256-thread workgroup (4 waves of 64 x 64 = 4 x 4 MFMA 16x16 tiles), K in
// chunks of 32, 16-B copies global -> registers -> double-buffered LDS (row stride 40 bf16:
// conflict-free ds_read_b128 fragment reads), no conversion work in the product loop. Split-K over
// blockIdx.z when the tile grid is small; the partial sums go to the workspace and k_gemm_reduce
// adds them in split order (deterministic) with bias and act.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "mz_gemm.h"

namespace {

constexpr int TM = 128, TN = 128, BK = 32, NT = 256;
constexpr int ST = 40;  // LDS row stride in bf16

typedef __attribute__((ext_vector_type(8))) __bf16 frag_ab;
typedef __attribute__((ext_vector_type(4))) float frag_cd;

__device__ inline uint32_t pk_bf16(float lo, float hi) {  // RNE, packed
  uint32_t r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}
__device__ inline float bf16_round(float x) { return __uint_as_float(pk_bf16(x, 0.0f) << 16); }

// 4 consecutive-k values of one row -> 8 B of hi halves and 8 B of lo halves
__device__ inline void split4(float x0, float x1, float x2, float x3, uint2& hi, uint2& lo) {
  const float h0 = bf16_round(x0), h1 = bf16_round(x1), h2 = bf16_round(x2), h3 = bf16_round(x3);
  hi = make_uint2(pk_bf16(h0, h1), pk_bf16(h2, h3));
  lo = make_uint2(pk_bf16(x0 - h0, x1 - h1), pk_bf16(x2 - h2, x3 - h3));
}

__device__ inline float act_f(float x, int act) {
  if (act == MZ_GEMM_LEAKY) return x > 0.0f ? x : x * 0.01f;
  if (act == MZ_GEMM_RELU) return x > 0.0f ? x : 0.0f;
  return x;
}

// ---- operand images: f32 view (any strides) -> bf16 hi / lo [Rp][Kp], zero padded -----------
// 64 rows x 64 k per 256-thread workgroup, 4 consecutive k of one row per thread and step; loads
// are coalesced along whichever dimension is contiguous (KC: along k, 16 threads per row's 256 B;
// else along rows, 64 rows per wave-instruction), each (row, 4 k) written as 8 B of hi and of lo.
template <bool KC>
__global__ __launch_bounds__(256) void k_split(const float* __restrict__ x, long rs_, long ks_, int R,
                                               int K, uint16_t* __restrict__ hi,
                                               uint16_t* __restrict__ lo, int Kp) {
  const int t = threadIdx.x;
  const int r0 = blockIdx.y * 64, k0 = blockIdx.x * 64;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int r, kq;
    if (KC) { r = r0 + (t >> 4) + 16 * i; kq = k0 + 4 * (t & 15); }
    else { r = r0 + (t & 63); kq = k0 + 4 * ((t >> 6) + 4 * i); }
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = kq + j;
      v[j] = (r < R && k < K) ? x[(long)r * rs_ + (long)k * ks_] : 0.0f;
    }
    uint2 h, l;
    split4(v[0], v[1], v[2], v[3], h, l);
    const size_t o = (size_t)r * Kp + kq;
    *reinterpret_cast<uint2*>(hi + o) = h;
    *reinterpret_cast<uint2*>(lo + o) = l;
  }
}

// ---- the product over the images ----------------------------------------------------------
struct Img {
  const uint16_t* hi; const uint16_t* lo;
};

// 128 rows x 32 k of an image's hi and lo halves: thread t copies 16 B at row (t >> 2) + 64 i,
// k 8 (t & 3) of each half (4 x 16-B global loads, then 4 x 16-B LDS writes)
struct Tile {
  uint4 v[4];
  __device__ inline void load(const Img& im, int row0, int k0, int Kp) {
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const size_t o = (size_t)(row0 + (t >> 2) + 64 * i) * Kp + k0 + 8 * (t & 3);
      v[i] = *reinterpret_cast<const uint4*>(im.hi + o);
      v[2 + i] = *reinterpret_cast<const uint4*>(im.lo + o);
    }
  }
  __device__ inline void store(uint16_t* hi, uint16_t* lo) const {
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int o = ((t >> 2) + 64 * i) * ST + 8 * (t & 3);
      *reinterpret_cast<uint4*>(hi + o) = v[i];
      *reinterpret_cast<uint4*>(lo + o) = v[2 + i];
    }
  }
};

// XCD-aware tile order: workgroup b runs on XCD b & 7 (dispatch is round-robin), so XCD x takes
// the contiguous run x * per .. of the (band, split, n-tile, m-in-band) order — 4 m-tiles (G) x
// 8 n-tiles of one split per 32 workgroups, whose A and B rows its L2 then serves 8 and 4 times
constexpr int G = 4;
struct Grid {
  int ntm, ntn, splits, per;
};

__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_gemm_x3(MzGemm g, Img A, Img B, int Kp, int kchunks_per_split, Grid gr) {
  __shared__ __align__(16) uint16_t lds[2][4][TM * ST];  // [buf][A hi, A lo, B hi, B lo]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w >> 1, wn = w & 1;
  int u = (blockIdx.x & 7) * gr.per + (blockIdx.x >> 3);
  const int mi = u % G;
  u /= G;
  const int nt = u % gr.ntn;
  u /= gr.ntn;
  const int z = u % gr.splits, band = u / gr.splits;
  const int mt = band * G + mi;
  if (mt >= gr.ntm) return;  // whole workgroup: the order's padding, or past the last band
  const int n0 = nt * TN, m0 = mt * TM;
  const int nch = Kp / BK;
  const int c0 = z * kchunks_per_split;
  const int c1 = min(nch, c0 + kchunks_per_split);
  frag_cd acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = frag_cd{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fk = (lane >> 4) * 8;
  auto compute = [&](int buf) {
    frag_ab ah[4], al[4], bh[4], bl[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int oa = (wm * 64 + 16 * i + fr) * ST + fk;
      const int ob = (wn * 64 + 16 * i + fr) * ST + fk;
      ah[i] = *reinterpret_cast<const frag_ab*>(&lds[buf][0][oa]);
      al[i] = *reinterpret_cast<const frag_ab*>(&lds[buf][1][oa]);
      bh[i] = *reinterpret_cast<const frag_ab*>(&lds[buf][2][ob]);
      bl[i] = *reinterpret_cast<const frag_ab*>(&lds[buf][3][ob]);
    }
    // product-major: consecutive MFMAs never share an accumulator
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
  };
  // global loads run two chunks ahead of the product (register sets p / q alternate): a chunk's
  // loads are issued two product phases before its LDS store waits for them
  Tile pa, pb, qa, qb;
  if (c0 < c1) {
    pa.load(A, m0, c0 * BK, Kp);
    pb.load(B, n0, c0 * BK, Kp);
    if (c0 + 1 < c1) {
      qa.load(A, m0, (c0 + 1) * BK, Kp);
      qb.load(B, n0, (c0 + 1) * BK, Kp);
    }
    pa.store(lds[0][0], lds[0][1]);
    pb.store(lds[0][2], lds[0][3]);
  }
  __syncthreads();
  for (int c = c0; c < c1; c += 2) {
    // chunk c in LDS[0], chunk c + 1 in flight in q
    if (c + 2 < c1) {
      pa.load(A, m0, (c + 2) * BK, Kp);
      pb.load(B, n0, (c + 2) * BK, Kp);
    }
    compute(0);
    if (c + 1 >= c1) break;
    qa.store(lds[1][0], lds[1][1]);
    qb.store(lds[1][2], lds[1][3]);
    __syncthreads();
    // chunk c + 1 in LDS[1], chunk c + 2 in flight in p
    if (c + 3 < c1) {
      qa.load(A, m0, (c + 3) * BK, Kp);
      qb.load(B, n0, (c + 3) * BK, Kp);
    }
    compute(1);
    if (c + 2 >= c1) break;
    pa.store(lds[0][0], lds[0][1]);
    pb.store(lds[0][2], lds[0][3]);
    __syncthreads();
  }
  // epilogue: lane holds C[row (lane >> 4) * 4 + r][col lane & 15] of each 16 x 16 tile
  const bool split = gr.splits > 1;
  float* out = split ? g.ws + (size_t)z * g.M * g.N : g.c;
  const long ldo = split ? g.N : g.ldc;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = n0 + wn * 64 + 16 * j + (lane & 15);
    if (col >= g.N) continue;
    const float bj = (!split && g.bias) ? g.bias[col] : 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 64 + 16 * i + (lane >> 4) * 4 + r;
        if (row < g.M) {
          const float x = acc[i][j][r];
          out[(size_t)row * ldo + col] = split ? x : act_f(x + bj, g.act);
        }
      }
  }
}

// C = act(sum_z ws[z] + bias), z in order
__global__ void k_gemm_reduce(MzGemm g, int splits) {
  const long n4 = (long)g.M * g.N;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const int row = (int)(i / g.N), col = (int)(i - (long)row * g.N);
    float s = g.ws[i];
    for (int z = 1; z < splits; ++z) s += g.ws[(size_t)z * n4 + i];
    if (g.bias) s += g.bias[col];
    g.c[(size_t)row * g.ldc + col] = act_f(s, g.act);
  }
}

}  // namespace

// split-K factor: grow the grid to >= MZ_GEMM_WG_TARGET workgroups (default 256: one per CU)
// while every split keeps >= 4 chunks
int mz_gemm_splits(int m, int n, int k) {
  static const int target = [] {
    const char* e = getenv("MZ_GEMM_WG_TARGET");
    return e ? atoi(e) : 256;
  }();
  const int tiles = ((m + TM - 1) / TM) * ((n + TN - 1) / TN);
  const int nch = (k + BK - 1) / BK;
  int s = 1;
  while (tiles * s < target && nch / (2 * s) >= 4) s *= 2;
  return s;
}

static inline long rup(long x, long a) { return (x + a - 1) / a * a; }

size_t mz_gemm_ws_floats(int m, int n, int k) {
  const long kp = rup(k, 64), mp = rup(m, TM), np = rup(n, TN);
  const int s = mz_gemm_splits(m, n, k);
  return (size_t)(mp * kp + np * kp) + (s > 1 ? (size_t)s * m * n : 0) + 64;
}

hipError_t mz_launch_gemm_x3(const MzGemm& g0, hipStream_t st) {
  MzGemm g = g0;
  const int Kp = (int)rup(g.K, 64), Mp = (int)rup(g.M, TM), Np = (int)rup(g.N, TN);
  // workspace: A image (hi | lo halves), B image, split-K partial sums; 16-B aligned pieces
  uint16_t* base = reinterpret_cast<uint16_t*>(g.ws_img);
  uint16_t *ah = base, *al = base + (size_t)Mp * Kp;
  uint16_t *bh = base + (size_t)2 * Mp * Kp, *bl = bh + (size_t)Np * Kp;
  const Img A{ah, al}, B{bh, bl};
  const int splits = mz_gemm_splits(g.M, g.N, g.K);
  g.ws = splits > 1 ? g.ws_img + (size_t)(Mp + Np) * Kp : nullptr;
  const bool ak = g.a_ks == 1, bk = g.b_ks == 1;
  dim3 ga(Kp / 64, Mp / 64), gb(Kp / 64, Np / 64);
  if (ak) hipLaunchKernelGGL(k_split<true>, ga, dim3(256), 0, st, g.a, g.a_rs, g.a_ks, g.M, g.K, ah, al, Kp);
  else hipLaunchKernelGGL(k_split<false>, ga, dim3(256), 0, st, g.a, g.a_rs, g.a_ks, g.M, g.K, ah, al, Kp);
  if (bk) hipLaunchKernelGGL(k_split<true>, gb, dim3(256), 0, st, g.b, g.b_rs, g.b_ks, g.N, g.K, bh, bl, Kp);
  else hipLaunchKernelGGL(k_split<false>, gb, dim3(256), 0, st, g.b, g.b_rs, g.b_ks, g.N, g.K, bh, bl, Kp);
  const int nch = Kp / BK;
  const int per = (nch + splits - 1) / splits;
  Grid gr{Mp / TM, Np / TN, splits, 0};
  const int total = (gr.ntm + G - 1) / G * G * gr.splits * gr.ntn;
  gr.per = (total + 7) / 8;
  hipLaunchKernelGGL(k_gemm_x3, dim3(8 * gr.per), dim3(NT), 0, st, g, A, B, Kp, per, gr);
  if (splits > 1) {
    const long n = (long)g.M * g.N;
    const int blocks = (int)((n + 255) / 256 < 2048 ? (n + 255) / 256 : 2048);
    hipLaunchKernelGGL(k_gemm_reduce, dim3(blocks), dim3(256), 0, st, g, splits);
  }
  return hipGetLastError();
}
