// mz_env.hip — the per-step hot path of the batched maze env on gfx950.
//
//   k_step        one lane per instance: BaseMazeEnv.step (base_maze_env.py:163-210) with the
//                 move rule of maze_view.move_agent (maze_view.py:167-197), the Enrich window
//                 (maze_handler.py:4-99) and "best dir" from the precomputed cell word.
//                 Per 64-instance wave the 675-bit windows are assembled in LDS and written out
//                 with fully coalesced 16-B stores (1 KiB per wave instruction).
//   k_reset_list  one wave per listed instance: BaseMazeEnv.reset (:136-161), optionally after
//                 regenerating the maze of instances that just won (off_policy_trainer.py:190-202)
//   k_act         fused epsilon-greedy / masked exploration (dqn_agent.py:104-116)
//   k_mask        get_mask_direction (simple_maze_env.py:41-50, toroidal_maze_env.py:57-69)
//   k_expand      packed window bits -> f32 [3][15][15]
//
// Floating point: every reward / score is formed with explicitly rounded IEEE double ops
// (__dadd_rn/__dmul_rn/__ddiv_rn) so contraction cannot change a bit vs CPython.
#include "mz_common.h"
#include "mz_kernels.h"
#include "mz_build.inc.h"

#include "../../include/mazerl.h"

#define WAVE 64
#define CAT_WORDS (WAVE * 675 / 32 + 2)

namespace {

__device__ inline uint32_t ext15(uint32_t lo, uint32_t hi, int sh) {
  uint64_t v = ((uint64_t)hi << 32) | lo;
  return (uint32_t)(v >> sh) & 0x7FFFu;
}

// 15 bits starting at column s of a 128-bit row, wrapping at N (toroidal rows).
__device__ inline uint32_t row15_wrap(const uint32_t w[4], int s, int N) {
  if (N >= 15) {
    uint32_t a = ext15(w[s >> 5], (s >> 5) < 3 ? w[(s >> 5) + 1] : 0u, s & 31);
    if (s + 15 <= N) return a;
    int k = N - s;  // bits taken before the wrap
    uint32_t b = ext15(w[0], w[1], 0);
    return (a & ((1u << k) - 1u)) | ((b << k) & 0x7FFFu);
  }
  uint32_t v = 0;
  for (int j = 0; j < 15; ++j) {
    int col = (s + j) % N;
    v |= ((w[col >> 5] >> (col & 31)) & 1u) << j;
  }
  return v;
}

// bits j in [0,15) with (C0 + j) mod N == col
__device__ inline uint32_t wrap_colmask(int col, int C0, int N) {
  uint32_t m = 0;
  for (int j = mz_wrap(col - C0, N); j < 15; j += N) m |= 1u << j;
  return m;
}

template <int OFF>
__device__ inline void put15(uint32_t (&w)[MZ_WINDOW_WORDS], uint32_t v) {
  w[OFF >> 5] |= v << (OFF & 31);
  if ((OFF & 31) > 17) w[(OFF >> 5) + 1] |= v >> (32 - (OFF & 31));
}

template <int I>
__device__ inline void put_row(uint32_t (&w)[MZ_WINDOW_WORDS], uint32_t ch0, uint32_t ch1,
                               uint32_t ch2) {
  put15<0 * 225 + I * 15>(w, ch0);
  put15<1 * 225 + I * 15>(w, ch1);
  put15<2 * 225 + I * 15>(w, ch2);
}

// Builds the 675-bit window of instance e at (r,c) from the open/visited planes. (vr,vc) is a
// cell to treat as visited although its plane bit may not be stored yet (the cell just entered,
// base_maze_env.py:184 happens before _get_obs); vr < 0 = none. visited_start_only: at reset
// the visited plane is {start} (base_maze_env.py:148-149), used without reading it back.
template <bool TOR, int I>
__device__ inline void window_row(const MzDev& d, size_t e, int N, int r, int c, int gr, int gc,
                                  int vr, int vc, bool visited_start_only, int sr, int sc,
                                  uint32_t (&w)[MZ_WINDOW_WORDS]) {
  uint32_t open15, vis15, gmask = 0;
  if (!TOR) {
    const int r0 = mz_win_start(r, N), c0 = mz_win_start(c, N);
    const int R = r0 + I;
    const uint32_t* row = d.planes + (e * d.P + R) * MZ_PLANE_WORDS;
    const int w0 = c0 >> 5, sh = c0 & 31;
    open15 = ext15(row[w0], row[w0 + 1], sh);
    if (visited_start_only) {
      vis15 = (R == sr) ? (1u << (sc - c0)) : 0u;  // start always inside its own window
    } else {
      vis15 = ext15(row[4 + w0], row[5 + w0], sh);
    }
    if (R == vr) vis15 |= 1u << (vc - c0);
    if (R == gr && gc >= c0 && gc < c0 + 15) gmask = 1u << (gc - c0);
  } else {
    const int R = mz_wrap(r + I - 7, N), C0 = mz_wrap(c - 7, N);
    const uint4* row4 = reinterpret_cast<const uint4*>(d.planes + (e * d.P + R) * MZ_PLANE_WORDS);
    uint4 o = row4[0];
    uint32_t ow[4] = {o.x, o.y, o.z, o.w};
    open15 = row15_wrap(ow, C0, N);
    if (visited_start_only) {
      vis15 = (R == sr) ? wrap_colmask(sc, C0, N) : 0u;
    } else {
      uint4 v = row4[1];
      uint32_t vw[4] = {v.x, v.y, v.z, v.w};
      vis15 = row15_wrap(vw, C0, N);
    }
    if (R == vr) vis15 |= wrap_colmask(vc, C0, N);
    if (R == gr) gmask = wrap_colmask(gc, C0, N);
  }
  // get_mask_tensor (maze_handler.py:82-99): [maze==0, maze==1, non_visited]; goal (2) is 0 in
  // channels 0 and 1; non_visited = open & ~visited.
  put_row<I>(w, ~open15 & 0x7FFFu, open15 & ~gmask, open15 & ~vis15);
}

template <bool TOR, int I = 0>
__device__ inline void window_rows(const MzDev& d, size_t e, int N, int r, int c, int gr, int gc,
                                   int vr, int vc, bool vso, int sr, int sc,
                                   uint32_t (&w)[MZ_WINDOW_WORDS]) {
  if constexpr (I < 15) {
    window_row<TOR, I>(d, e, N, r, c, gr, gc, vr, vc, vso, sr, sc, w);
    window_rows<TOR, I + 1>(d, e, N, r, c, gr, gc, vr, vc, vso, sr, sc, w);
  }
}

// "best dir" = agent - best_next_cell (base_maze_env.py:122) from the cell's best-next code
__device__ inline void best_dir(int r, int c, uint32_t cw, int N, bool tor, int& br, int& bc) {
  int code = (cw >> MZ_CELL_CODE_SHIFT) & 7;
  if (code > 3) { br = 0; bc = 0; return; }
  int nr = r + mz_dr(code), nc = c + mz_dc(code);
  if (tor) { nr = mz_wrap(nr, N); nc = mz_wrap(nc, N); }
  br = r - nr;
  bc = c - nc;
}

// obs vector of the learner: concat(agent, target, best dir) -> f32 (off_policy_trainer.py:156)
template <bool ENRICH>
__device__ inline void write_obs6(float* o6, int r, int c, int gr, int gc, int br, int bc, int N) {
  if (ENRICH) {  // agent / maze_shape, target / maze_shape in f64, then f32 (simple_maze_env.py:153-154)
    const double n = (double)N;
    o6[0] = (float)__ddiv_rn((double)r, n);
    o6[1] = (float)__ddiv_rn((double)c, n);
    o6[2] = (float)__ddiv_rn((double)gr, n);
    o6[3] = (float)__ddiv_rn((double)gc, n);
  } else {
    o6[0] = (float)r; o6[1] = (float)c; o6[2] = (float)gr; o6[3] = (float)gc;
  }
  o6[4] = (float)br;
  o6[5] = (float)bc;
}

// Write one wave's windows (bits in `cat`, 675 bits per instance back to back) as f32 with
// 16-B stores: float f of the block <-> bit f of cat, so a float4 never straddles a word.
__device__ inline void store_window_f32(const uint32_t* cat, float* out, int nb, int lane) {
  const int nfl = nb * 675;
  const int nq = nfl >> 2;
  float4* o4 = reinterpret_cast<float4*>(out);
  for (int q = lane; q < nq; q += WAVE) {
    uint32_t nib = (cat[q >> 3] >> ((q & 7) * 4)) & 0xFu;
    float4 v;
    v.x = (float)(nib & 1u);
    v.y = (float)((nib >> 1) & 1u);
    v.z = (float)((nib >> 2) & 1u);
    v.w = (float)((nib >> 3) & 1u);
    o4[q] = v;
  }
  for (int f = (nq << 2) + lane; f < nfl; f += WAVE) out[f] = (float)((cat[f >> 5] >> (f & 31)) & 1u);
}

__device__ inline void cat_or(uint32_t* cat, int lane, const uint32_t (&w)[MZ_WINDOW_WORDS]) {
  const int base = lane * 675, w0 = base >> 5, sh = base & 31;
#pragma unroll
  for (int k = 0; k < MZ_WINDOW_WORDS; ++k) {
    if (w[k] == 0u) continue;
    atomicOr(&cat[w0 + k], w[k] << sh);
    if (sh) atomicOr(&cat[w0 + k + 1], w[k] >> (32 - sh));
  }
}

// ------------------------------------------------------------------------------------------
template <bool TOR, bool ENRICH>
__global__ __launch_bounds__(WAVE) void k_step(MzDev d, const int32_t* __restrict__ act, MzOut o) {
  __shared__ uint32_t cat[CAT_WORDS];
  __shared__ uint32_t pad[WAVE][MZ_WINDOW_WORDS + 1];
  const int lane = threadIdx.x;
  const int e0 = blockIdx.x * WAVE;
  const int e = e0 + lane;
  const int nb = min(WAVE, d.B - e0);
  const bool live = lane < nb;
  if (ENRICH) {
    for (int i = lane; i < CAT_WORDS; i += WAVE) cat[i] = 0u;
    __syncthreads();
  }
  bool done = false;
  if (live) {
    const size_t es = (size_t)e;
    const uint32_t m0 = d.meta0[e], m1 = d.meta1[e];
    uint32_t pw = d.posw[e], sw = d.stw[e], cw = d.curw[e];
    const int araw = act[e];
    const int a = araw & 3;
    const int N = m0 & 0xFF, gr = m1 & 0xFF, gc = (m1 >> 8) & 0xFF, maxs = m1 >> 16;
    int r = pw & 0xFF, c = (pw >> 8) & 0xFF, nm = (pw >> 16) & 3, la = (pw >> 18) & 3;
    int steps = sw & 0xFFFF, inv = (sw >> 16) & 0xFF;
    double rew = 0.0;
    bool term = false, trunc = false;
    int vr = -1, vc = -1;
    if (araw >= 0) {  // araw < 0: observe only (no transition, obs of the current state)
      int nr = r + mz_dr(a), nc = c + mz_dc(a);
      bool inb;
      if (TOR) { nr = mz_wrap(nr, N); nc = mz_wrap(nc, N); inb = true; }
      else inb = 0 < nr && nr < N - 1 && 0 < nc && nc < N - 1;  // maze_view.py:169 (Q3)
      const size_t ci = es * d.P * d.P + (size_t)nr * d.P + nc;
      const uint32_t ncw = inb ? d.cells[ci] : 0u;
      const bool moved = (ncw & MZ_CELL_OPEN) != 0u;
      if (moved) {
        const size_t vi = es * d.VP + (size_t)nr * d.P + nc;
        const int cnt = d.visits[vi];
        if (cnt == 0) {
          // first entry: non_visited[cell] = 0 (base_maze_env.py:184)
          vr = nr; vc = nc;
          atomicOr(&d.planes[(es * d.P + nr) * MZ_PLANE_WORDS + 4 + (nc >> 5)], 1u << (nc & 31));
          if (nr == gr && nc == gc) { rew = 1.0; term = true; }  // :185-187
          else {  // (old_dist - new_dist) * 0.5 - 0.05 with len = D + 1 (:189-192)
            const int dold = (int)(cw & MZ_CELL_D_MASK), dnew = (int)(ncw & MZ_CELL_D_MASK);
            rew = __dsub_rn(__dmul_rn((double)(dold - dnew), 0.5), 0.05);
          }
        } else {
          rew = d.pen_visit[cnt];  // :194
        }
        d.visits[vi] = (uint8_t)min(cnt + 1, 255);
        inv = 0;
        nm = min(nm + 1, 2);
        la = a;
        r = nr; c = nc; cw = ncw;
      } else {
        inv = min(inv + 1, 255);
        rew = d.pen_inv[inv];  // :199-200
      }
      steps = min(steps + 1, 65535);
      trunc = steps > maxs;  // :205-208
      if (trunc) rew = -1.0;
      done = term || trunc;
      d.posw[e] = (uint32_t)r | ((uint32_t)c << 8) | ((uint32_t)nm << 16) | ((uint32_t)la << 18) |
                  ((uint32_t)done << 20);
      d.stw[e] = (uint32_t)steps | ((uint32_t)inv << 16);
      d.curw[e] = cw;
      d.last_term[e] = term;
    }

    int br, bc;
    best_dir(r, c, cw, N, TOR, br, bc);
    if (o.reward) o.reward[e] = (float)rew;
    if (o.reward64) o.reward64[e] = rew;
    if (o.terminated) o.terminated[e] = term;
    if (o.truncated) o.truncated[e] = trunc;
    if (o.pos) { o.pos[2 * es] = r; o.pos[2 * es + 1] = c; }
    if (o.best_dir) { o.best_dir[2 * es] = br; o.best_dir[2 * es + 1] = bc; }
    if (o.obs6) write_obs6<ENRICH>(o.obs6 + 6 * es, r, c, gr, gc, br, bc, N);
    if (ENRICH) {
      uint32_t w[MZ_WINDOW_WORDS];
#pragma unroll
      for (int k = 0; k < MZ_WINDOW_WORDS; ++k) w[k] = 0u;
      window_rows<TOR>(d, es, N, r, c, gr, gc, vr, vc, false, 0, 0, w);
      cat_or(cat, lane, w);
#pragma unroll
      for (int k = 0; k < MZ_WINDOW_WORDS; ++k) pad[lane][k] = w[k];
    }
  }
  // done-list compaction: wave ballot + one atomic per wave
  if (o.done_idx) {
    const unsigned long long bal = __ballot(done);
    if (bal) {
      int base = 0;
      if (lane == 0) base = atomicAdd(o.done_count, __popcll(bal));
      base = __shfl(base, 0);
      if (done) o.done_idx[base + __popcll(bal & ((1ull << lane) - 1ull))] = e;
    }
  }
  if (ENRICH) {
    __syncthreads();
    if (o.window_bits) {
      uint32_t* wb = o.window_bits + (size_t)e0 * MZ_WINDOW_WORDS;
      for (int i = lane; i < nb * MZ_WINDOW_WORDS; i += WAVE)
        wb[i] = pad[i / MZ_WINDOW_WORDS][i % MZ_WINDOW_WORDS];
    }
    if (o.window) store_window_f32(cat, o.window + (size_t)e0 * 675, nb, lane);
  }
}

}  // namespace

// ------------------------------------------------------------------------------------------
namespace {

// Wave-cooperative reset of instance e (lane 0 = scalar state; all lanes clear), then its
// reset observation. Used by k_reset_list (after optional regeneration in mz_build.hip).
template <bool TOR, bool ENRICH>
__device__ void reset_one(const MzDev& d, int e, const MzOut& o, uint32_t* wsh) {
  const int lane = threadIdx.x;
  const size_t es = (size_t)e;
  const uint32_t m0 = d.meta0[e], m1 = d.meta1[e];
  const int N = m0 & 0xFF, sr = (m0 >> 16) & 0xFF, sc = m0 >> 24;
  const int gr = m1 & 0xFF, gc = (m1 >> 8) & 0xFF;
  // visits[:] = 0 (visited_cell = [], base_maze_env.py:159)
  uint4* v4 = reinterpret_cast<uint4*>(d.visits + es * d.VP);
  for (int i = lane; i < d.VP / 16; i += WAVE) v4[i] = make_uint4(0, 0, 0, 0);
  // visited plane = {start} (non_visited = open & ~start, :148-149)
  for (int R = lane; R < d.P; R += WAVE) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (R == sr) {
      uint32_t bit = 1u << (sc & 31);
      int wi = sc >> 5;
      v.x = wi == 0 ? bit : 0u; v.y = wi == 1 ? bit : 0u;
      v.z = wi == 2 ? bit : 0u; v.w = wi == 3 ? bit : 0u;
    }
    reinterpret_cast<uint4*>(d.planes + (es * d.P + R) * MZ_PLANE_WORDS)[1] = v;
  }
  const uint32_t cw = d.cells[es * d.P * d.P + (size_t)sr * d.P + sc];
  int br, bc;
  best_dir(sr, sc, cw, N, TOR, br, bc);
  if (lane == 0) {
    d.posw[e] = (uint32_t)sr | ((uint32_t)sc << 8);
    d.stw[e] = 0u;
    d.curw[e] = cw;
    d.last_term[e] = 0;
    if (o.reward) o.reward[e] = 0.f;
    if (o.reward64) o.reward64[e] = 0.0;
    if (o.terminated) o.terminated[e] = 0;
    if (o.truncated) o.truncated[e] = 0;
    if (o.pos) { o.pos[2 * es] = sr; o.pos[2 * es + 1] = sc; }
    if (o.best_dir) { o.best_dir[2 * es] = br; o.best_dir[2 * es + 1] = bc; }
    if (o.obs6) write_obs6<ENRICH>(o.obs6 + 6 * es, sr, sc, gr, gc, br, bc, N);
  }
  if (ENRICH) {
    if (lane == 0) {
      uint32_t w[MZ_WINDOW_WORDS];
#pragma unroll
      for (int k = 0; k < MZ_WINDOW_WORDS; ++k) w[k] = 0u;
      window_rows<TOR>(d, es, N, sr, sc, gr, gc, -1, -1, true, sr, sc, w);
#pragma unroll
      for (int k = 0; k < MZ_WINDOW_WORDS; ++k) wsh[k] = w[k];
    }
    __syncthreads();
    if (o.window_bits && lane < MZ_WINDOW_WORDS) o.window_bits[es * MZ_WINDOW_WORDS + lane] = wsh[lane];
    if (o.window)
      for (int f = lane; f < 675; f += WAVE) o.window[es * 675 + f] = (float)((wsh[f >> 5] >> (f & 31)) & 1u);
    __syncthreads();
  }
}

template <bool TOR, bool ENRICH>
__global__ __launch_bounds__(WAVE) void k_reset_list(MzDev d, const int32_t* idx,
                                                     const int32_t* count, int32_t n_static,
                                                     MzOut o) {
  __shared__ __align__(16) uint32_t wsh[32];
  const int n = count ? min(*count, n_static) : n_static;
  for (int j = blockIdx.x; j < n; j += gridDim.x) {
    const int e = idx ? idx[j] : j;
    reset_one<TOR, ENRICH>(d, e, o, wsh);
    __syncthreads();
  }
}

// Build (generate or import) the listed instances: one wave per maze, persistent over the list.
__global__ __launch_bounds__(WAVE) void k_build(MzDev d, const int32_t* env_ids, int32_t n,
                                                int generate, const uint8_t* algo_list,
                                                int32_t algo_all, int32_t dim, uint64_t seed,
                                                const uint8_t* grids, const int32_t* sg) {
  extern __shared__ __align__(16) uint8_t lds[];
  for (int j = blockIdx.x; j < n; j += gridDim.x) {
    const int e = env_ids ? env_ids[j] : j;
    if (generate) {
      const int algo = algo_list ? algo_list[j] : algo_all;
      if (threadIdx.x == 0) d.algo[e] = (uint8_t)algo;
      mz_build_one(d, e, d.toroidal, true, algo, seed + (uint64_t)e, dim, nullptr, 0, 0, 0, 0, lds);
    } else {
      mz_build_one(d, e, d.toroidal, false, 0, 0, dim, grids + (size_t)j * dim * dim,
                   sg[4 * j], sg[4 * j + 1], sg[4 * j + 2], sg[4 * j + 3], lds);
    }
    __syncthreads();
  }
}

// Regenerate the mazes of listed instances whose last step terminated (win -> update_maze,
// off_policy_trainer.py:190-202), same size, their stored algorithm, seed + e + (epoch << 32).
__global__ __launch_bounds__(WAVE) void k_regen_list(MzDev d, const int32_t* idx,
                                                     const int32_t* count, int32_t n_static,
                                                     uint64_t seed, uint32_t epoch) {
  extern __shared__ __align__(16) uint8_t lds[];
  const int n = count ? min(*count, n_static) : n_static;
  for (int j = blockIdx.x; j < n; j += gridDim.x) {
    const int e = idx ? idx[j] : j;
    if (!d.last_term[e]) continue;  // uniform per block
    mz_build_one(d, e, d.toroidal, true, d.algo[e], seed + (uint64_t)e + ((uint64_t)epoch << 32),
                 (int)(d.meta0[e] & 0xFF), nullptr, 0, 0, 0, 0, lds);
    __syncthreads();
  }
}

// get_mask_direction(probs): open-neighbour bits from the current cell word; with probs and
// >= 2 moves since reset the direction of the previous cell gets 0.25 — on the torus the
// reference looks it up transposed (Q6): previous below -> "right", above -> "left", etc.
__device__ inline void dir_mask(uint32_t pw, uint32_t cw, bool tor, bool probs, float m[4]) {
  const uint32_t nb = (cw >> MZ_CELL_NB_SHIFT) & 0xFu;
#pragma unroll
  for (int k = 0; k < 4; ++k) m[k] = (float)((nb >> k) & 1u);
  const int nm = (pw >> 16) & 3, la = (pw >> 18) & 3;
  if (probs && nm >= 2) {
    const int back = la ^ 1;  // action that leads to visited_cell[-2]
    m[tor ? (back ^ 2) : back] = 0.25f;
  }
}

__global__ void k_mask(MzDev d, int probs, float* out4) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.B) return;
  float m[4];
  dir_mask(d.posw[e], d.curw[e], d.toroidal, probs, m);
  reinterpret_cast<float4*>(out4)[e] = make_float4(m[0], m[1], m[2], m[3]);
}

__global__ void k_act(MzDev d, const float* eps, float eps_all, const int64_t* greedy,
                      uint64_t seed, uint64_t counter, int32_t* actions) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.B) return;
  uint32_t u[4];
  mz_philox(seed, MZ_ACT_STREAM ^ ((uint64_t)e << 32), counter, u);
  const float ue = (float)(u[0] >> 8) * (1.0f / 16777216.0f);
  const float ep = eps ? eps[e] : eps_all;
  if (greedy && !(ue < ep)) { actions[e] = (int32_t)greedy[e]; return; }
  float m[4];
  dir_mask(d.posw[e], d.curw[e], d.toroidal, true, m);
  // np.random.choice(4, p = mask / mask.sum()) by inverse CDF (dqn_agent.py:110-112)
  const float tot = m[0] + m[1] + m[2] + m[3];
  float x = (float)(u[1] >> 8) * (1.0f / 16777216.0f) * tot;
  int a = 0;
  while (a < 3 && (x >= m[a] || m[a] == 0.f)) { x -= m[a]; ++a; }
  while (a > 0 && m[a] == 0.f) --a;
  actions[e] = a;
}

__global__ void k_expand(const uint32_t* bits, float* out, int n) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)n * 675;
  if (t >= total) return;
  const long i = t / 675, f = t - i * 675;
  out[t] = (float)((bits[i * MZ_WINDOW_WORDS + (f >> 5)] >> (f & 31)) & 1u);
}

}  // namespace

// ------------------------------------------------------------------------------------------
// launchers (called by mz_api.hip)
hipError_t mz_launch_step(const MzDev& d, const int32_t* act, const MzOut& o, hipStream_t s) {
  dim3 grid((d.B + WAVE - 1) / WAVE), block(WAVE);
  if (d.toroidal) {
    if (d.enrich) hipLaunchKernelGGL((k_step<true, true>), grid, block, 0, s, d, act, o);
    else hipLaunchKernelGGL((k_step<true, false>), grid, block, 0, s, d, act, o);
  } else {
    if (d.enrich) hipLaunchKernelGGL((k_step<false, true>), grid, block, 0, s, d, act, o);
    else hipLaunchKernelGGL((k_step<false, false>), grid, block, 0, s, d, act, o);
  }
  return hipGetLastError();
}

size_t mz_build_lds_size(int P) { return mz_build_lds_bytes(P); }

static int mz_grid_for(int n) { return n < 4096 ? n : 4096; }

// the build kernels may need more than the 64 KiB default dynamic LDS at large max_dim
static hipError_t mz_lds_attr(const void* fn, size_t bytes) {
  if (bytes <= 65536) return hipSuccess;
  return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

hipError_t mz_launch_build(const MzDev& d, const int32_t* env_ids, int32_t n, bool generate,
                           const uint8_t* algo_list, int32_t algo_all, int32_t dim, uint64_t seed,
                           const uint8_t* grids, const int32_t* start_goal, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipError_t ae = mz_lds_attr(reinterpret_cast<const void*>(k_build), mz_build_lds_bytes(d.P));
  if (ae != hipSuccess) return ae;
  hipLaunchKernelGGL(k_build, dim3(mz_grid_for(n)), dim3(WAVE), mz_build_lds_bytes(d.P), s, d,
                     env_ids, n, (int)generate, algo_list, algo_all, dim, seed, grids, start_goal);
  return hipGetLastError();
}

hipError_t mz_launch_regen(const MzDev& d, const int32_t* idx, const int32_t* count,
                           int32_t n_static, uint64_t seed, uint32_t epoch, hipStream_t s) {
  if (n_static <= 0) return hipSuccess;
  hipError_t ae = mz_lds_attr(reinterpret_cast<const void*>(k_regen_list), mz_build_lds_bytes(d.P));
  if (ae != hipSuccess) return ae;
  hipLaunchKernelGGL(k_regen_list, dim3(mz_grid_for(n_static)), dim3(WAVE),
                     mz_build_lds_bytes(d.P), s, d, idx, count, n_static, seed, epoch);
  return hipGetLastError();
}

hipError_t mz_launch_reset_list(const MzDev& d, const int32_t* idx, const int32_t* count,
                                int32_t n_static, const MzOut& o, hipStream_t s) {
  if (n_static <= 0) return hipSuccess;
  const int blocks = n_static < 2048 ? n_static : 2048;
#define MZ_RL(T, E) \
  hipLaunchKernelGGL((k_reset_list<T, E>), dim3(blocks), dim3(WAVE), 0, s, d, idx, count, n_static, o)
  if (d.toroidal) { if (d.enrich) MZ_RL(true, true); else MZ_RL(true, false); }
  else { if (d.enrich) MZ_RL(false, true); else MZ_RL(false, false); }
#undef MZ_RL
  return hipGetLastError();
}

hipError_t mz_launch_mask(const MzDev& d, int probs, float* out4, hipStream_t s) {
  hipLaunchKernelGGL(k_mask, dim3((d.B + 255) / 256), dim3(256), 0, s, d, probs, out4);
  return hipGetLastError();
}

hipError_t mz_launch_act(const MzDev& d, const float* eps, float eps_all, const int64_t* greedy,
                         uint64_t seed, uint64_t counter, int32_t* actions, hipStream_t s) {
  hipLaunchKernelGGL(k_act, dim3((d.B + 255) / 256), dim3(256), 0, s, d, eps, eps_all, greedy,
                     seed, counter, actions);
  return hipGetLastError();
}

hipError_t mz_launch_expand(const uint32_t* bits, float* out, int n, hipStream_t s) {
  long total = (long)n * 675;
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL(k_expand, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, bits, out, n);
  return hipGetLastError();
}
