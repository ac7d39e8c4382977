// mz_env.hip — the per-step hot path of the batched maze env on gfx950 (+ build/reset kernels).
//
//   k_step        BaseMazeEnv.step (base_maze_env.py:163-210) for IPW (16) instances per 64-lane wave:
//                 phase 1, one lane per instance: (optional fused epsilon-greedy act,
//                   dqn_agent.py:104-116) move rule of maze_view.move_agent (maze_view.py:167-197),
//                   reward, counters, "best dir" from the precomputed cell word, done-list
//                   compaction by wave ballot + one atomic per wave;
//                 phase 2, one lane per (instance, window row): the Enrich window
//                   (maze_handler.py:4-99) from the open/visited bit planes, 15 consecutive lanes
//                   reading 15 consecutive 32-B rows of one instance (few cache lines per load);
//                 phase 3, the wave's IPW windows (675 bits each, back to back in LDS) leave as f32
//                   with 16-B stores, 1 KiB contiguous per wave instruction.
//   k_reset_list  one wave per listed instance: BaseMazeEnv.reset (:136-161); the device done
//                 count it was given is consumed (zeroed) by a memset after the launch.
//   k_build / k_regen_list  maze generation + tables (mz_build.inc.h).
//   k_act / k_mask / k_expand  exploration act, get_mask_direction, bits -> f32.
//
// Floating point: every reward / score is formed with explicitly rounded IEEE double ops
// (__dadd_rn/__dmul_rn/__ddiv_rn) so contraction cannot change a bit vs CPython.
#include "mz_common.h"
#include "mz_kernels.h"
#include "mz_build.inc.h"

#include "../../include/mazerl.h"

#define WAVE 64
// Instances per wave in k_step. 16 (4,096 waves at 65,536 instances: twice the gathers in flight,
// finer-grained window stores) measured best: k_step at 65,536 x 81 = 38.8 / 34.4 / 36.1 / 40.4 us
// at 8 / 16 / 32 / 64 (bench, 500 launches).
#ifndef MZ_IPW
#define MZ_IPW 16
#endif
#define IPW MZ_IPW
#ifndef MZ_SPW
// k_step waves per workgroup (they share the staged 4 KB reward tables). Measured at 65,536
// instances: 1 -> 34.3 us, 2 -> 36.2 us, 4 -> 36.4 us per launch — the saved L2 reads are worth
// less than the workgroup barrier that the shared table needs.
#define MZ_SPW 1
#endif
// Timing probes (profiles/exp_probes.sh; never in the product build — each makes the step wrong):
// MZ_PROBE mask bits: 1 no penalty-table staging, 2 no window-bit assembly, 4 no autoreset plane /
// count work, 8 no per-instance output stores, 16 no f32 window stores, 32 window stores of a
// constant (no LDS reads), 64 no state stores, 128 return at once (launch + dispatch floor),
// 256 no level-2 loads, 512 window rows loaded but not assembled (zero windows: faster stores)
#ifndef MZ_PROBE
#define MZ_PROBE 0
#endif
// LDS words of a wave's window bits: ipw x 675 bits + funnel-shift slack
__host__ __device__ constexpr int cat_words(int ipw) { return ipw * 675 / 32 + 2; }

namespace {

// bits j in [0,15) with (C0 + j) mod N == col
__device__ inline uint32_t wrap_colmask(int col, int C0, int N) {
  uint32_t m = 0;
  for (int j = mz_wrapn(col - C0, N); j < 15; j += N) m |= 1u << j;
  return m;
}

// Window of an agent at (r, c) (extract_submaze / extract_submaze_toroid, maze_handler.py:4-80):
// first row R0 and first column C0 = 18 st + off, packed with N as
//   geo = R0 | st << 7 | off << 10 | N << 15
// — the window is rows R0 .. R0 + 14 (torus: mod N) of plane strip st, bits off .. off + 14.
template <bool TOR>
__device__ inline int win_geo(int r, int c, int N) {
  int R0, C0;
  if (!TOR) { R0 = mz_win_start(r, N); C0 = mz_win_start(c, N); }
  else { R0 = mz_wrapn(r - 7, N); C0 = mz_wrapn(c - 7, N); }
  const int st = C0 / MZ_STRIP_STRIDE;
  return R0 | (st << 7) | ((C0 - MZ_STRIP_STRIDE * st) << 10) | (N << 15);
}
__device__ inline int geo_st(int g) { return (g >> 7) & 7; }
__device__ inline int geo_n(int g) { return (g >> 15) & 0x7F; }
// grid row of window row i
template <bool TOR>
__device__ inline int geo_row(int g, int i) {
  return TOR ? mz_wrapn((g & 0x7F) + i, geo_n(g)) : (g & 0x7F) + i;
}

// Window row i (grid row R) from its strip pair pr = (open, visited): the three 15-bit channel
// rows of get_mask_tensor (maze_handler.py:82-99): [maze==0, maze==1, non_visited]; the goal (2)
// is 0 in channels 0 and 1; non_visited = open & ~visited. (vr, vc): a cell counted as visited
// although its plane bit is not stored yet (just entered — base_maze_env.py:184 precedes
// _get_obs — or the reset start); vr < 0 = none. vso: the visited plane is {start} only (reset,
// :148-149) and the stored bits are not read. The agent's own cell always lies in its window.
template <bool TOR>
__device__ inline void win_row_bits(uint2 pr, int g, int R, int gr, int gc, int vr, int vc,
                                    bool vso, uint32_t& ch0, uint32_t& ch1, uint32_t& ch2) {
  const int off = (g >> 10) & 31, N = geo_n(g);
  const int C0 = MZ_STRIP_STRIDE * geo_st(g) + off;
  const uint32_t open15 = (pr.x >> off) & 0x7FFFu;
  uint32_t vis15 = vso ? 0u : (pr.y >> off) & 0x7FFFu, gmask = 0u;
  if (!TOR) {
    if (R == vr) vis15 |= 1u << (vc - C0);
    if (R == gr && gc >= C0 && gc < C0 + 15) gmask = 1u << (gc - C0);
  } else {
    if (R == vr) vis15 |= wrap_colmask(vc, C0, N);
    if (R == gr) gmask = wrap_colmask(gc, C0, N);
  }
  ch0 = ~open15 & 0x7FFFu;
  ch1 = open15 & ~gmask;
  ch2 = open15 & ~vis15;
}

// strips a window of an N-grid can start in (euclidean c0 <= N - 15, torus c0 <= N - 1); the
// others are never read, so neither marked nor reset (a small maze under a large pitch)
__device__ inline int used_strips(int N, bool tor) {
  return tor ? mz_nstrips(N) : (N - 15) / MZ_STRIP_STRIDE + 1;
}

// visited_cell.append (base_maze_env.py:196) in the planes: the cell's bit in every strip that
// holds its column (euclidean: one or two; torus: any strip, repeated when N < 32). No-return
// atomics (a plain store of the window strip's word, which the step has just read, measured
// slower: 32.26 vs 31.96 us per launch at 65,536 x 81, 25.11 vs 24.67 on config 5's shape).
template <bool TOR>
__device__ inline void mark_visited(const MzDev& d, size_t e, int R, int col, int N) {
  const int lo = TOR ? 0 : max(0, (col - 31 + MZ_STRIP_STRIDE - 1) / MZ_STRIP_STRIDE);
  const int hi = min(used_strips(N, TOR), TOR ? d.NS : col / MZ_STRIP_STRIDE + 1) - 1;
  for (int st = lo; st <= hi; ++st) {
    const uint32_t m = mz_strip_colmask(st, col, N, TOR);
    if (m) atomicOr(reinterpret_cast<uint32_t*>(mz_strip_row(d, e, st, R)) + 1, m);
  }
}

// visited plane of instance e = {(sr, sc)} (reset; rows >= N hold no open cell): one wave
__device__ inline void reset_visited(const MzDev& d, size_t e, int N, int sr, int sc, bool tor,
                                     int lane) {
  const int ns = min(d.NS, used_strips(N, tor));
  for (int R = lane; R < N; R += WAVE)  // one row per lane, every used strip (no index division)
    for (int st = 0; st < ns; ++st)
      reinterpret_cast<uint32_t*>(mz_strip_row(d, e, st, R))[1] =
          R == sr ? mz_strip_colmask(st, sc, N, tor) : 0u;
}

__device__ inline void cat_put(uint32_t* cat, int o, uint32_t v) {
  if (!v) return;
  atomicOr(&cat[o >> 5], v << (o & 31));
  if ((o & 31) > 17) atomicOr(&cat[(o >> 5) + 1], v >> (32 - (o & 31)));
}

// 32 window bits starting at bit o of cat
__device__ inline uint32_t cat_get32(const uint32_t* cat, int o) {
  const int w = o >> 5, s = o & 31;
  return s ? (cat[w] >> s) | (cat[w + 1] << (32 - s)) : cat[w];
}

// "best dir" = agent - best_next_cell (base_maze_env.py:122) from the cell's best-next code
__device__ inline void best_dir(int r, int c, uint32_t cw, int N, bool tor, int& br, int& bc) {
  int code = (cw >> MZ_CELL_CODE_SHIFT) & 7;
  if (code > 3) { br = 0; bc = 0; return; }
  int nr = r + mz_dr(code), nc = c + mz_dc(code);
  if (tor) { nr = mz_wrapn(nr, N); nc = mz_wrapn(nc, N); }
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

// Write nb windows (bits back to back in cat, 675 per instance) as f32 with 16-B stores:
// float f of the block <-> bit f of cat, so a float4 never straddles a word. The stores are
// write-through (buffer-store aux 16 = sc1): the window leaves no dirty L2 lines for the kernel
// end to drain. k_step at 65,536 x 81 (bench, 500 launches): default policy 37.0 us, sc1 36.2,
// nt 43.6, sc1 + nt 43.5.
// Past the 256 MB Infinity Cache the same stream is faster as non-temporal stores (aux 2): at
// 131,072 x 81 (354 MB of windows per step) nt 75.0-75.7 us vs sc1 89.2, plain 105.0, sc0|sc1
// 107.2; at 65,536 (177 MB) sc1 31.7 vs nt 38.1-38.4 (profiles/r03wp_window_store_policy.json):
// the launcher picks nt when the step's f32 windows exceed MZ_WINDOW_NT_BYTES (MzOut::window_nt).
typedef __attribute__((ext_vector_type(4))) unsigned int mz_u32x4;
template <int POL = 16>
__device__ inline void store_window_f32(const uint32_t* cat, float* out, int nb, int lane) {
  const int nfl = nb * 675;
  const int nq = nfl >> 2;
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(out, 0, nfl * 4, 0x00020000);
  auto put = [&](int q, uint32_t word) {
    const uint32_t nib = (word >> ((q & 7) * 4)) & 0xFu;
    float4 v;
    v.x = (float)(nib & 1u);
    v.y = (float)((nib >> 1) & 1u);
    v.z = (float)((nib >> 2) & 1u);
    v.w = (float)((nib >> 3) & 1u);
    if (POL == 0) reinterpret_cast<float4*>(out)[q] = v;
    else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(mz_u32x4, v), rsrc, q * 16, 0, POL);
  };
  // 8 stores per LDS wait: the words of 8 passes are read first (pass u of lane q: word
  // (q >> 3) + 8u, same nibble), then the 8 stores issue back to back
  int q = lane;
  for (; q + 7 * WAVE < nq; q += 8 * WAVE) {
    uint32_t w[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) w[u] = (MZ_PROBE & 32) ? (uint32_t)q * 0x9E3779B9u : cat[(q >> 3) + 8 * u];
#pragma unroll
    for (int u = 0; u < 8; ++u) put(q + u * WAVE, w[u]);
  }
  for (; q < nq; q += WAVE) put(q, cat[q >> 3]);
  for (int f = (nq << 2) + lane; f < nfl; f += WAVE) out[f] = (float)((cat[f >> 5] >> (f & 31)) & 1u);
}

__device__ inline void store_window_bits(const uint32_t* cat, uint32_t* wb, int nb, int lane) {
  for (int k = lane; k < nb * MZ_WINDOW_WORDS; k += WAVE) {
    const int j = k / MZ_WINDOW_WORDS, w = k - j * MZ_WINDOW_WORDS;
    uint32_t v = cat_get32(cat, j * 675 + 32 * w);
    if (w == MZ_WINDOW_WORDS - 1) v &= (1u << (675 - 32 * (MZ_WINDOW_WORDS - 1))) - 1u;
    wb[k] = v;
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

// epsilon-greedy with the reference exploration distribution (dqn_agent.py:104-116):
// u < eps -> np.random.choice(4, p = mask / mask.sum()) by inverse CDF, else greedy.
// ep / greedy: the instance's epsilon and greedy action (greedy < 0: always explore).
// The exploration draw of instance e (sample = random.random(), dqn_agent.py:105): Philox(seed,
// e, counter); u[0] -> `sample`, u[1] -> the masked-direction choice. act_draw and greedy_needed
// (the greedy-row list) read the same words, so the list is exactly the instances that act greedily.
__device__ inline void act_u(const MzAct& ap, int e, uint32_t u[4]) {
  mz_philox(ap.seed, MZ_ACT_STREAM ^ ((uint64_t)e << 32), ap.counter, u);
}
__device__ inline bool act_greedy(const uint32_t u[4], float ep) {
  const float ue = (float)(u[0] >> 8) * (1.0f / 16777216.0f);
  return !(ue < ep);
}

__device__ inline int act_draw(const MzAct& ap, int e, float ep, int greedy, uint32_t pw,
                               uint32_t cw, bool tor) {
  uint32_t u[4];
  act_u(ap, e, u);
  if (greedy >= 0 && act_greedy(u, ep)) return greedy;
  float m[4];
  dir_mask(pw, cw, tor, true, m);
  const float tot = m[0] + m[1] + m[2] + m[3];
  float x = (float)(u[1] >> 8) * (1.0f / 16777216.0f) * tot;
  int a = 0;
  while (a < 3 && x >= m[a]) { x -= m[a]; ++a; }
  while (a > 0 && m[a] == 0.f) --a;
  return a;
}

__device__ inline int act_sample(const MzAct& ap, int e, uint32_t pw, uint32_t cw, bool tor) {
  return act_draw(ap, e, ap.eps ? ap.eps[e] : ap.eps_all, ap.greedy ? (int)ap.greedy[e] : -1, pw,
                  cw, tor);
}

// window-row passes: lane l of pass it = instance 4*it + l/16, row l%16
__host__ __device__ constexpr int win_it(int ipw) { return ipw * 16 / WAVE; }

// ------------------------------------------------------------------------------------------
// One vector step, IPW instances per 64-lane wave, with two dependent global round trips:
//   level 1  per-instance state (5 coalesced u32 + eps/greedy or the given action), and the
//            reward tables into LDS; the action, and whether the agent moves: the target is open
//            iff the current cell word's open-neighbour bit for the action is set (the same
//            predicate maze[(r+dr) mod N][(c+dc) mod N] != 0, mz_cell_word) — so the window the
//            step ends in is known before any gather;
//   level 2  the target cell word and its visit count (one lane per moving / resetting
//            instance), and that window's 15 rows from its plane strip (one lane per row, 8-B
//            loads, 120 contiguous bytes per instance);
//   then     reward / counters (BaseMazeEnv.step, base_maze_env.py:163-210), the Enrich window
//            assembled bit by bit in LDS, and only then every global store: state, outputs, and
//            the IPW windows as f32 with 16-B stores (1 KiB per wave instruction). No wait in the
//            kernel ever covers a store.
// AR (autoreset): an instance whose previous step ended terminated|truncated is reset by this
// launch instead of stepping (BaseMazeEnv.reset, :136-161: same maze, agent at start, visits
// cleared; the trainer's env.reset() after a finished episode) — its action is ignored
// (actions_out = -1), reward 0, terminated = truncated = 0, obs = the reset observation.
// Every 8th reset of an instance its episode tag wraps to 0: drop all visit counts of its maze
// (rows < N; keeps the static cell bits), so no stale count can alias a later tag. No-return
// atomic ANDs: the wave issues them and moves on (a load-mask-store loop would wait a round trip
// per pass, and the slowest wave sets the launch time).
__device__ inline void clear_counts(const MzDev& d, size_t e, int N) {
  uint32_t* c = d.cells + e * d.P * d.P;
  const int lane = threadIdx.x & (WAVE - 1), n = N * d.P;
  // 8-B atomics (512 B per wave instruction, half the instructions of 4-B ones) from the first
  // 8-B boundary; the odd head / tail word with 4-B ones
  const int h = (int)((reinterpret_cast<uintptr_t>(c) >> 2) & 1u);
  if (lane == 0 && h) (void)__hip_atomic_fetch_and(&c[0], MZ_CELL_STATIC, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (lane == 1 && ((n - h) & 1))
    (void)__hip_atomic_fetch_and(&c[n - 1], MZ_CELL_STATIC, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned long long* c2 = reinterpret_cast<unsigned long long*>(c + h);
  const unsigned long long m2 = ((unsigned long long)MZ_CELL_STATIC << 32) | MZ_CELL_STATIC;
  for (int k = lane; k < (n - h) >> 1; k += WAVE)
    (void)__hip_atomic_fetch_and(&c2[k], m2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int IPWT, bool TOR, bool ENRICH, bool ACT, bool AR>
__device__ inline void step_group(const MzDev& d, const int32_t* __restrict__ act, const MzAct& ap,
                                  const MzOut& o, int e0, uint32_t* cat, double* pen, bool load_pen) {
  const int lane = threadIdx.x & (WAVE - 1);
  const int nb = max(0, min(IPWT, d.B - e0));  // 0: a trailing wave of the last workgroup
  const int e = e0 + lane;
  const size_t es = (size_t)e;
  const bool live = lane < nb;

  // ---- level 1
  uint32_t m0 = 0u, m1 = 0u, pw = 0u, sw = 0u, cw = 0u;
  float ep = 0.f;
  int greedy = -1, araw = -1;
  if (live) {
    m0 = d.meta0[e]; m1 = d.meta1[e]; pw = d.posw[e]; sw = d.stw[e]; cw = d.curw[e];
    if (ACT) {
      ep = ap.eps ? ap.eps[e] : ap.eps_all;
      if (ap.greedy) greedy = (int)ap.greedy[e];
    } else {
      araw = act[e];
    }
  }
  if (MZ_PROBE & 128) return;
  if (load_pen && !(MZ_PROBE & 1)) {
    uint4* pl = reinterpret_cast<uint4*>(pen);
    if (MZ_SPW == 1) {
      const uint4* pv = reinterpret_cast<const uint4*>(d.pen_visit);
      const uint4* pi = reinterpret_cast<const uint4*>(d.pen_inv);
      const uint4 t0 = pv[lane], t1 = pv[lane + WAVE], t2 = pi[lane], t3 = pi[lane + WAVE];
      pl[lane] = t0; pl[lane + WAVE] = t1; pl[2 * WAVE + lane] = t2; pl[3 * WAVE + lane] = t3;
    } else {  // each wave stages its share of the 4 KB (pen_inv follows pen_visit in one buffer)
      const uint4* pt = reinterpret_cast<const uint4*>(d.pen_visit);
      for (int i = (int)(threadIdx.x / WAVE) * WAVE + lane; i < 4 * WAVE; i += MZ_SPW * WAVE)
        pl[i] = pt[i];
    }
  }
  if (ENRICH)
    for (int i = lane; i < cat_words(IPWT); i += WAVE) cat[i] = 0u;

  const int N = m0 & 0xFF, sr = (m0 >> 16) & 0xFF, sc = m0 >> 24;
  const int gr = m1 & 0xFF, gc = (m1 >> 8) & 0xFF, maxs = m1 >> 16;
  int r = pw & 0xFF, c = (pw >> 8) & 0xFF, nm = (pw >> 16) & 3, la = (pw >> 18) & 3;
  int steps = sw & 0xFFFF, inv = (sw >> 16) & 0xFF;
  const bool rst = AR && live && ((pw >> 20) & 1u);
  if (ACT && live && !rst) araw = act_draw(ap, e, ep, greedy, pw, cw, TOR);
  const int a = araw & 3;
  const bool trans = live && !rst && araw >= 0;  // araw < 0: observe only (obs of current state)
  // the cell the agent would enter (reset: the start cell) and whether it does: the move rule
  // of maze_view.move_agent (maze_view.py:167-197) — in bounds (Q3) and open
  int tr = r, tc = c;
  bool mv = false;
  if (rst) { tr = sr; tc = sc; }
  else if (trans) {
    tr = r + mz_dr(a); tc = c + mz_dc(a);
    bool inb = true;
    if (TOR) { tr = mz_wrapn(tr, N); tc = mz_wrapn(tc, N); }
    else inb = 0 < tr && tr < N - 1 && 0 < tc && tc < N - 1;  // maze_view.py:169 (Q3)
    mv = inb && ((cw >> (MZ_CELL_NB_SHIFT + a)) & 1u);  // == target cell word & MZ_CELL_OPEN
    if (!mv) { tr = r; tc = c; }
  }

  // ---- level 2
  const uint32_t tag = (sw >> MZ_STW_TAG_SHIFT) & 7u;  // the episode's visit-count tag
  uint32_t ncw = 0u;
  if ((mv || rst) && !(MZ_PROBE & 256)) ncw = d.cells[es * d.P * d.P + (size_t)tr * d.P + tc];  // cell word + visit count
  const int cnt = rst ? 0 : mz_cell_count(ncw, tag);
  uint2 wr[win_it(IPWT)];  // strip pairs of the final window's rows
  int geo = 0;
  if (ENRICH) {
    if (live) geo = win_geo<TOR>(tr, tc, N);  // tr, tc = where the agent is after this launch
#pragma unroll
    for (int it = 0; it < win_it(IPWT); ++it) {
      const int j = it * (WAVE / 16) + (lane >> 4), i = lane & 15;
      const int g = __shfl(geo, j);
      wr[it] = make_uint2(0u, 0u);
      if (j < nb && i < 15 && !(MZ_PROBE & 256)) wr[it] = *mz_strip_row(d, (size_t)(e0 + j), geo_st(g), geo_row<TOR>(g, i));
    }
  }
  __syncthreads();  // pen[] (single-wave workgroup: an LDS wait, no s_barrier)

  // ---- transition (BaseMazeEnv.step) or reset
  double rew = 0.0;
  bool term = false, trunc = false, done = false;
  int vr = -1, vc = -1;
  uint32_t ntag = tag;
  if (rst) {
    r = sr; c = sc; cw = ncw; nm = 0; la = 0; steps = 0; inv = 0;
    ntag = (tag + 1u) & 7u;  // visited_cell = [] (base_maze_env.py:159): a new count tag
    vr = sr; vc = sc;  // visited = {start} (base_maze_env.py:148-149)
  } else if (trans) {
    if (mv) {
      if (cnt == 0) {
        // first entry: non_visited[cell] = 0 (base_maze_env.py:184); plane bits set below
        vr = tr; vc = tc;
        if (tr == gr && tc == gc) { rew = 1.0; term = true; }  // :185-187
        else {  // (old_dist - new_dist) * 0.5 - 0.05 with len = D + 1 (:189-192)
          const int dold = (int)(cw & MZ_CELL_D_MASK), dnew = (int)(ncw & MZ_CELL_D_MASK);
          rew = __dsub_rn(__dmul_rn((double)(dold - dnew), 0.5), 0.05);
        }
      } else {
        rew = pen[cnt];  // :194
      }
      inv = 0;
      nm = min(nm + 1, 2);
      la = a;
      r = tr; c = tc; cw = ncw;
    } else {
      inv = min(inv + 1, 255);
      rew = pen[256 + inv];  // :199-200
    }
    steps = min(steps + 1, 65535);
    trunc = steps > maxs;  // :205-208
    if (trunc) rew = -1.0;
    done = term || trunc;
  }

  // ---- window bits in LDS (compute only: every global store of the step comes after, so no
  // wait in this kernel ever covers a store)
  if (ENRICH && !(MZ_PROBE & 2)) {
    const int ps = (int)rst | ((vr + 1) << 8) | ((vc + 1) << 16);
    const int pg = gr | (gc << 8);
#pragma unroll
    for (int it = 0; it < win_it(IPWT); ++it) {
      const int j = it * (WAVE / 16) + (lane >> 4), i = lane & 15;
      const int s_ = __shfl(ps, j), g = __shfl(geo, j), gg = __shfl(pg, j);
      if (j < nb && i < 15) {
        uint32_t c0, c1, c2;
        win_row_bits<TOR>(wr[it], g, geo_row<TOR>(g, i), gg & 0xFF, (gg >> 8) & 0xFF,
                          ((s_ >> 8) & 0xFF) - 1, ((s_ >> 16) & 0xFF) - 1, s_ & 1, c0, c1, c2);
        const int base = j * 675 + i * 15;
        if (MZ_PROBE & 512) {  // probe: the rows are loaded and decoded, not assembled
          if ((c0 ^ (c1 << 1) ^ (c2 << 2)) == ((uint32_t)(lane * 77 + it) & 0x1FFFFu)) cat[0] = 1u;
        } else {
          cat_put(cat, base, c0);
          cat_put(cat, base + 225, c1);
          cat_put(cat, base + 450, c2);
        }
      }
    }
  }

  // ---- stores: state, per-instance outputs, then the windows
  if ((rst || trans) && !(MZ_PROBE & 64)) {
    d.posw[e] = (uint32_t)r | ((uint32_t)c << 8) | ((uint32_t)nm << 16) | ((uint32_t)la << 18) |
                ((uint32_t)done << 20);
    d.stw[e] = (uint32_t)steps | ((uint32_t)inv << 16) | (ntag << MZ_STW_TAG_SHIFT);
    d.curw[e] = cw;
    d.last_term[e] = term;
    if (mv) {
      if (ENRICH && vr >= 0) mark_visited<TOR>(d, es, tr, tc, N);
      d.cells[es * d.P * d.P + (size_t)tr * d.P + tc] =  // visited_cell.append (:196)
          (ncw & MZ_CELL_STATIC) | ((uint32_t)min(cnt + 1, 255) << MZ_CELL_CNT_SHIFT) |
          (tag << MZ_CELL_TAG_SHIFT);
    }
  }
  if (live && !(MZ_PROBE & 8)) {
    if (ACT && ap.act_out) ap.act_out[e] = rst ? -1 : araw;
    int br, bc;
    best_dir(r, c, cw, N, TOR, br, bc);
    if (o.reward) o.reward[e] = (float)rew;
    if (o.reward64) o.reward64[e] = rew;
    if (o.terminated) o.terminated[e] = term;
    if (o.truncated) o.truncated[e] = trunc;
    if (o.pos) { o.pos[2 * es] = r; o.pos[2 * es + 1] = c; }
    if (o.best_dir) { o.best_dir[2 * es] = br; o.best_dir[2 * es + 1] = bc; }
    if (o.obs6) write_obs6<ENRICH>(o.obs6 + 6 * es, r, c, gr, gc, br, bc, N);
  }
  if (ENRICH) {
    __syncthreads();
    if (o.window_bits) store_window_bits(cat, o.window_bits + (size_t)e0 * MZ_WINDOW_WORDS, nb, lane);
    if (o.window && !(MZ_PROBE & 16)) {
      if (o.window_nt) store_window_f32<2>(cat, o.window + (size_t)e0 * 675, nb, lane);
      else store_window_f32<16>(cat, o.window + (size_t)e0 * 675, nb, lane);
    }
  }

  if (AR && !(MZ_PROBE & 4)) {  // reset instances: visited plane = {start}; counts cleared when the tag wraps
    unsigned long long bal = __ballot(rst);
    const int sp = sr | (sc << 8) | ((int)ntag << 16) | (N << 19);
    while (bal) {
      const int j = __ffsll((long long)bal) - 1;
      bal &= bal - 1;
      const int q = __shfl(sp, j);
      const size_t ej = (size_t)(e0 + j);
      const int Nj = (q >> 19) & 0xFF;
      reset_visited(d, ej, Nj, q & 0xFF, (q >> 8) & 0xFF, TOR, lane);
      if (((q >> 16) & 7) == 0) clear_counts(d, ej, Nj);
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
}

// One wave per group of IPWT instances. (A persistent variant — each wave stepping several
// groups so that its next gathers trail its window stores — measured slower at every
// groups-per-wave setting: 46 / 60 / 104 us at 2 / 4 / 8 groups per wave vs 40 us at 1, because
// the gather phase is latency-bound per wave and needs every group's wave in flight at once.)
// IPWT = 16 for large batches; small batches (the per-GPU shares of the 8-GPU configs) take 4,
// so that four times as many waves share the latency chain and the window stores.
template <int IPWT, bool TOR, bool ENRICH, bool ACT, bool AR>
__global__ __launch_bounds__(WAVE * MZ_SPW) void k_step(MzDev d, const int32_t* __restrict__ act,
                                                        MzAct ap, MzOut o) {
  __shared__ uint32_t cat[MZ_SPW][(cat_words(IPWT) + 3) & ~3];
  __shared__ __align__(16) double pen[512];  // pen_visit[256] | pen_inv[256]
  const int w = MZ_SPW > 1 ? (int)(threadIdx.x / WAVE) : 0;
  int b = blockIdx.x;
  // Workgroups are dealt round-robin over the 8 XCDs: give each XCD a contiguous range of
  // instance groups, so the 64-B state / output segments of neighbouring groups (halves of one
  // 128-B line) meet in one XCD's L2 (65,536 x 81: 32.65 -> 31.96 us per launch)
  if ((gridDim.x & 7) == 0) b = (b & 7) * (int)(gridDim.x >> 3) + (b >> 3);
  step_group<IPWT, TOR, ENRICH, ACT, AR>(d, act, ap, o, (b * MZ_SPW + w) * IPWT, cat[w], pen, true);
}

// ------------------------------------------------------------------------------------------
// Wave-cooperative reset of instance e: BaseMazeEnv.reset (base_maze_env.py:136-161).
// meta: the instance's meta words when the caller has them in registers (a bank maze just
// copied in: one dependent global round trip fewer), else read here
template <bool TOR, bool ENRICH>
__device__ void reset_one(const MzDev& d, int e, const MzOut& o, uint32_t* wsh,
                          const uint2* meta = nullptr) {
  const int lane = threadIdx.x;
  const size_t es = (size_t)e;
  const uint32_t m0 = meta ? meta->x : d.meta0[e], m1 = meta ? meta->y : d.meta1[e];
  const int N = m0 & 0xFF, sr = (m0 >> 16) & 0xFF, sc = m0 >> 24;
  const int gr = m1 & 0xFF, gc = (m1 >> 8) & 0xFF;
  const uint32_t cw = d.cells[es * d.P * d.P + (size_t)sr * d.P + sc];
  // visited_cell = [] (base_maze_env.py:159): a new visit-count tag (all counts cleared on wrap)
  const uint32_t ntag = ((d.stw[e] >> MZ_STW_TAG_SHIFT) + 1u) & 7u;
  if (ntag == 0u) clear_counts(d, es, N);
  // visited plane = {start} (non_visited = open & ~start, :148-149)
  reset_visited(d, es, N, sr, sc, TOR, lane);
  if (lane == 0) {
    int br, bc;
    best_dir(sr, sc, cw, N, TOR, br, bc);
    d.posw[e] = (uint32_t)sr | ((uint32_t)sc << 8);
    d.stw[e] = ntag << MZ_STW_TAG_SHIFT;
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
    if (lane < 24) wsh[lane] = 0u;
    __syncthreads();
    if (lane < 15) {  // open words are static; the visited plane is {start} (not read back)
      uint32_t c0, c1, c2;
      const int g = win_geo<TOR>(sr, sc, N), R = geo_row<TOR>(g, lane);
      win_row_bits<TOR>(*mz_strip_row(d, es, geo_st(g), R), g, R, gr, gc, sr, sc, true, c0, c1, c2);
      cat_put(wsh, lane * 15, c0);
      cat_put(wsh, 225 + lane * 15, c1);
      cat_put(wsh, 450 + lane * 15, c2);
    }
    __syncthreads();
    if (o.window_bits) store_window_bits(wsh, o.window_bits + es * MZ_WINDOW_WORDS, 1, lane);
    if (o.window)
      for (int f = lane; f < 675; f += WAVE) o.window[es * 675 + f] = (float)((wsh[f >> 5] >> (f & 31)) & 1u);
    __syncthreads();
  }
}

template <bool TOR, bool ENRICH>
__global__ __launch_bounds__(WAVE) void k_reset_list(MzDev d, const int32_t* idx,
                                                     int32_t* count, int32_t n_static, MzOut o) {
  __shared__ __align__(16) uint32_t wsh[32];
  const int n = count ? min(*count, n_static) : n_static;
  for (int j = blockIdx.x; j < n; j += gridDim.x) {
    const int e = idx ? idx[j] : j;
    reset_one<TOR, ENRICH>(d, e, o, wsh);
    __syncthreads();
  }
  // the count is consumed (zeroed) by a stream-ordered memset after the launch: a last-block
  // ticket here cost one same-address atomic per block, serialised (~30 ns each, up to 1,024)
}

// Bank class of a winner k_reset_done regenerates: a * bk_nd + di for its algorithm id a and maze
// size index di, -1 when no bank is in use or the bank does not hold that algorithm / size.
__device__ inline int bank_class(const MzDev& d, int e) {
  if (d.bk_K == 0) return -1;
  const int a = d.algo[e], N = mz_regen_dim(d, e);
  if (N >= 128 || !((d.bk_amask >> a) & 1u)) return -1;
  const int di = d.bk_didx[N];
  return di < 0 ? -1 : a * d.bk_nd + di;
}

// whether instance e is a winner k_reset_done(regen) gives a new maze
__device__ inline bool regen_winner(const MzDev& d, int e) {
  return e < d.B && ((d.posw[e] >> 20) & 1u) && d.last_term[e] && mz_regen_dim(d, e) != 0;
}

// Copy n words, each lane keeping 32 loads in flight (a one-word-per-pass loop waits a full
// round trip per 256 B: 103 of them for an 81 x 81 maze's cell words).
__device__ inline void wave_copy(uint32_t* __restrict__ dst, const uint32_t* __restrict__ src,
                                 size_t n) {
  constexpr int U = 32;  // an 81 x 81 maze's cell words in 4 round trips
  for (size_t i = threadIdx.x & (WAVE - 1); i < n; i += U * WAVE) {
    uint32_t v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = i + u * WAVE < n ? src[i + u * WAVE] : 0u;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * WAVE < n) dst[i + u * WAVE] = v[u];
  }
}

// Copy bank slot `slot` of class `cls` (bank_class) into instance e (cells + plane rows + meta;
// reset_one then rebuilds the per-episode state). Returns false (the caller builds in place) for
// cls < 0 or an exhausted bank (slot >= K). The slots come from k_bank_count / k_bank_scan: the
// winners of one reset_done launch take consecutive slots of their class in instance order, so
// which winner receives which maze does not depend on the order the waves run in.
__device__ bool bank_take(const MzDev& d, int e, int cls, int slot, uint2& meta) {
  if (cls < 0 || slot >= d.bk_K) return false;
  const int a = cls / d.bk_nd, di = cls - a * d.bk_nd;
  const size_t src = ((size_t)mz_bank_aidx(d.bk_amask, a) * d.bk_nd + di) * d.bk_K + slot;
  const size_t es = (size_t)e;
  const size_t pp = (size_t)d.P * d.P;
  meta = make_uint2(d.bk_meta0[src], d.bk_meta1[src]);  // issued with the copy's first loads
  wave_copy(d.cells + es * pp, d.bk_cells + src * pp, pp);
  const size_t pw = (size_t)d.PW;
  wave_copy(d.planes + es * pw, d.bk_planes + src * pw, pw);
  if (threadIdx.x == 0) {
    d.meta0[e] = meta.x;
    d.meta1[e] = meta.y;
  }
  __syncthreads();  // reset_one reads the start cell word / window rows written above
  return true;
}

// Slot assignment, pass 1 (one wave per 64-instance group g): winners per bank class in the
// group -> bk_slot[class * G + g] (the array is zeroed before the launch).
__global__ __launch_bounds__(WAVE) void k_bank_count(MzDev d) {
  const int lane = threadIdx.x, g = blockIdx.x, e = g * WAVE + lane;
  const bool w = regen_winner(d, e);
  const int cls = w ? bank_class(d, e) : -1;
  if (e < d.B) d.bk_code[e] = (int8_t)(w ? cls : -2);
  unsigned long long pend = __ballot(cls >= 0);
  while (pend) {  // one pass per distinct class in the wave (wave-uniform loop)
    const int cj = __shfl(cls, __ffsll((long long)pend) - 1);
    const unsigned long long m = __ballot(cls == cj);
    if (lane == 0) d.bk_slot[cj * d.bk_G + g] = __popcll(m);
    pend &= ~m;
  }
}

// Pass 2 (one workgroup per class): exclusive prefix over the groups in group order, offset by
// the class's consumed-slot counter -> the first slot of each group's winners; the counter then
// advances by the class's winners (what the per-winner atomic used to add).
constexpr int BS_T = 1024;
__global__ __launch_bounds__(BS_T) void k_bank_scan(MzDev d) {
  __shared__ int wsum[BS_T / WAVE];
  __shared__ int carry;
  const int c = blockIdx.x, t = threadIdx.x, lane = t & (WAVE - 1), w = t / WAVE;
  int* cnt = d.bk_slot + (size_t)c * d.bk_G;
  if (t == 0) carry = d.bk_head[c];
  __syncthreads();
  for (int base = 0; base < d.bk_G; base += BS_T) {
    const int i = base + t;
    const int v = i < d.bk_G ? cnt[i] : 0;
    int x = v;  // inclusive wave scan
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) {
      const int y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (lane == WAVE - 1) wsum[w] = x;
    __syncthreads();
    int before = carry;
    for (int k = 0; k < w; ++k) before += wsum[k];
    if (i < d.bk_G) cnt[i] = before + x - v;
    __syncthreads();
    if (t == BS_T - 1) carry = before + x;
    __syncthreads();
  }
  if (t == 0) d.bk_head[c] = carry;
}

// Candidate builds (one wave per maze, persistent): target j of a list of n targets (n = the
// static count, or min(*count, n) — a bank block's slots consumed since its last fill) gets C
// candidate mazes at indices j * C + c of the view `cd`, Philox seed
//   mz_cand_seed(seed, id(j), C, c, epoch) = seed + (id(j) * C + c) + (epoch << 32),
//   id(j) = ids ? ids[j] : base + j,
// so C = 1 with cd = the bank block is the bank's own fill (seed + slot + epoch << 32), and
// C > 1 over the instances of a handle draws the candidates best_of_mazes draws for those
// instances (VectorMazeEnv.generate of n * C instances from `seed`: candidate c of maze k is
// instance k * C + c, seed + k * C + c). The algorithm: algo_list[j] or algo_all.
// Euclidean Philox r-prim / dfs candidates of one algorithm (the headline's bank classes),
// MZ_PACK per wave (mz_build_cells_packed): candidates t0 .. t0 + MZ_PACK - 1 on lanes
// 16 (t - t0) ..
__global__ __launch_bounds__(WAVE) void k_cand_build_packed(MzDev cd, const int32_t* ids, int base,
                                                            const int* count, int n, int C,
                                                            int algo, int dim, uint64_t seed,
                                                            uint32_t epoch, int stride, int dbg) {
  extern __shared__ __align__(16) uint8_t lds[];
  const int used = count ? min(*count, n) : n;
  const int total = used * C, m = threadIdx.x >> 4;
  for (int t0 = blockIdx.x * MZ_PACK; t0 < total; t0 += gridDim.x * MZ_PACK) {
    const int nm = min(MZ_PACK, total - t0);
    const int t = t0 + min(m, nm - 1);
    const int j = t / C, c = t - j * C;
    const uint64_t id = (uint64_t)(ids ? ids[j] : base + j);
    if ((threadIdx.x & 15) == 0 && m < nm) cd.algo[t] = (uint8_t)algo;
    mz_build_cells_packed(cd, t, mz_cand_seed(seed, id, C, c, epoch, dbg), nm, dim, algo, lds,
                          (size_t)stride);
    __syncthreads();
  }
}

__global__ __launch_bounds__(WAVE) void k_cand_build(MzDev cd, const int32_t* ids, int base,
                                                     const int* count, int n, int C,
                                                     const uint8_t* algo_list, int algo_all,
                                                     int dim, uint64_t seed, uint32_t epoch,
                                                     int dbg) {
  extern __shared__ __align__(16) uint8_t lds[];
  const int used = count ? min(*count, n) : n;
  for (int t = blockIdx.x; t < used * C; t += gridDim.x) {
    const int j = t / C, c = t - j * C;
    const int algo = algo_list ? algo_list[j] : algo_all;
    const uint64_t id = (uint64_t)(ids ? ids[j] : base + j);
    if (threadIdx.x == 0) cd.algo[t] = (uint8_t)algo;
    mz_build_one(cd, t, cd.toroidal, true, algo, mz_cand_seed(seed, id, C, c, epoch, dbg), dim,
                 nullptr, 0, 0, 0, 0, lds);
    __syncthreads();
  }
}

// Euclidean Philox candidates in compact form (mz_screen.h): the carve, goal and distance field
// of k_cand_build_packed / k_cand_build, but no cell words or plane strips — 4.8 KB per 81 x 81
// candidate leave the CU instead of 29 KB, and only the selected one gets tables
// (k_cand_expand). The same seeds, so the same mazes.
__global__ __launch_bounds__(WAVE) void k_cand_compact_packed(MzCompact cc, int P, const int32_t* ids,
                                                              int base, const int* count, int n,
                                                              int C, int algo, int dim,
                                                              uint64_t seed, uint32_t epoch,
                                                              int stride, int dbg) {
  extern __shared__ __align__(16) uint8_t lds[];
  const int used = count ? min(*count, n) : n;
  const int total = used * C, m = threadIdx.x >> 4;
  for (int t0 = blockIdx.x * MZ_PACK; t0 < total; t0 += gridDim.x * MZ_PACK) {
    const int nm = min(MZ_PACK, total - t0);
    const int t = t0 + min(m, nm - 1);
    const int j = t / C, c = t - j * C;
    const uint64_t id = (uint64_t)(ids ? ids[j] : base + j);
    mz_carve_packed(P, mz_cand_seed(seed, id, C, c, epoch, dbg), nm, dim, algo, lds, (size_t)stride);
    for (int k = 0; k < nm; ++k) mz_cells_compact(cc, t0 + k, mz_cell_lds(lds + k * stride, P, dim), dim);
    __syncthreads();
  }
}

// Lite r-prim candidates (mz_lite_rprim): MZ_LPACK carves per wave in lockstep on lanes
// (64 / MZ_LPACK) m, each in a ~2.9 KB region, then the finish maze after maze in the wave's
// scratch (depth words + distances) after the regions. The same seeds and draws: the same mazes.
#ifndef MZ_LPACK
#define MZ_LPACK 4
#endif
#ifndef MZ_RING  // the lite carves' Philox words prefetched into an LDS ring (A/B builds: 0)
#define MZ_RING 1
#endif
#ifndef MZ_LANES  // the lite carves lane-parallel (mz_lite_carve_lanes; A/B builds: 0)
#define MZ_LANES 1
#endif
__global__ __launch_bounds__(WAVE) void k_cand_compact_lite(MzCompact cc, int P, const int32_t* ids,
                                                            int base, const int* count, int n, int C,
                                                            int algo, int dim, uint64_t seed,
                                                            uint32_t epoch, int stride, int dbg) {
  extern __shared__ __align__(16) uint8_t lds[];
  constexpr int SP = WAVE / MZ_LPACK;
  const int used = count ? min(*count, n) : n;
  const int total = used * C, lane = threadIdx.x, m = lane / SP;
  uint8_t* scr = lds + (size_t)MZ_LPACK * stride;
  uint32_t* J = reinterpret_cast<uint32_t*>(scr);
  uint16_t* A = reinterpret_cast<uint16_t*>(scr + mz_align16(4 * (size_t)mz_compact_qp(P)));
  for (int t0 = blockIdx.x * MZ_LPACK; t0 < total; t0 += gridDim.x * MZ_LPACK) {
    const int nm = min(MZ_LPACK, total - t0);
    const int t = t0 + min(m, nm - 1);
    const int j = t / C, c = t - j * C;
    const uint64_t id = (uint64_t)(ids ? ids[j] : base + j);
    for (int k = 0; k < nm; ++k) {
      const MzCellLds L = mz_lite_lds(lds + k * stride, P, dim, algo);
      mz_cells_clear(L);
      if (lane == 0) { L.sh[3] = 0; L.sh[4] = 0; }
    }
    __syncthreads();
    if (MZ_RING) {  // every lane: the carve loop with the Philox ring (mz_lite_carve_ring)
      const MzCellLds L = mz_lite_lds(lds + m * stride, P, dim, algo);
      uint32_t* ring = reinterpret_cast<uint32_t*>(lds + m * stride + mz_lite_lds_bytes(P, algo));
      // r-prim: the group's lanes share each iteration (mz_lite_carve_lanes; 2,048 best-of-6
      // selections 14.7 -> 11.6 ms, the same mazes); dfs keeps one lane per carve (its lane
      // version measured slower, 18.8 -> 22.1 ms: profiles/r06o/)
      if (MZ_LANES && algo != MZ_ALGO_DFS_DEV)
        mz_lite_carve_lanes<SP>(L, algo, mz_cand_seed(seed, id, C, c, epoch, dbg), m < nm, ring);
      else
        mz_lite_carve_ring<SP>(L, algo, mz_cand_seed(seed, id, C, c, epoch, dbg),
                               (lane % SP) == 0 && m < nm, ring);
    } else if ((lane % SP) == 0 && m < nm) {
      const MzCellLds L = mz_lite_lds(lds + m * stride, P, dim, algo);
      const int W = L.W;
      MzRng rng{mz_cand_seed(seed, id, C, c, epoch, dbg), 0ull, {0u, 0u, 0u, 0u}};
      const int a = (int)rng.below((uint32_t)W), b = (int)rng.below((uint32_t)W);
      L.sh[2] = a * W + b;
      if (algo == MZ_ALGO_DFS_DEV) mz_lite_dfs(L, a * W + b, rng);
      else mz_lite_rprim(L, a * W + b, rng);
    }
    __syncthreads();
    for (int k = 0; k < nm; ++k)
      mz_lite_finish(cc, t0 + k, mz_lite_lds(lds + k * stride, P, dim, algo), dim, J, A);
    __syncthreads();
  }
}

__global__ __launch_bounds__(WAVE) void k_cand_compact(MzCompact cc, int P, const int32_t* ids,
                                                       int base, const int* count, int n, int C,
                                                       const uint8_t* algo_list, int algo_all,
                                                       int dim, uint64_t seed, uint32_t epoch,
                                                       int dbg) {
  extern __shared__ __align__(16) uint8_t lds[];
  const int used = count ? min(*count, n) : n;
  for (int t = blockIdx.x; t < used * C; t += gridDim.x) {
    const int j = t / C, c = t - j * C;
    const int algo = algo_list ? algo_list[j] : algo_all;
    const uint64_t id = (uint64_t)(ids ? ids[j] : base + j);
    const MzCellLds L = mz_cell_lds(lds, P, dim);
    mz_carve_cells(L, algo, mz_cand_seed(seed, id, C, c, epoch, dbg));
    mz_cells_compact(cc, t, L, dim);
    __syncthreads();
  }
}

// Best-of-C decision from the screen (mz_screen.hip): target j keeps candidate a, the first
// minimum of the screened products, when every other candidate c is provably larger in the
// reference's own float evaluation as well: p_c (1 - e_c) > p_a (1 + e_a) (1 + 2^-40) — the e's
// bound each screened product's distance from the reference's product, and the 2^-40 keeps the
// two logs the reference compares apart (base_maze_env.py:78-97 keeps the first strict minimum of
// math.log). Any other group (a candidate the screen declined, or two candidates within the
// bounds) is listed for the order-exact kernel (k_mcclendon), at most xcap of them per launch;
// a group past that cap keeps the screen's pick and is counted unresolved. stats: [0] unresolved
// groups, [2] groups, [3] groups sent to the exact kernel.
__global__ __launch_bounds__(WAVE) void k_cand_pick(const int* count, int n, int C,
                                                    const double* score, const int32_t* status,
                                                    int32_t* pick, int32_t* xlist, int* xcount,
                                                    int xcap, int* stats, int dbg) {
  const int used = count ? min(*count, n) : n;
  const int lane = threadIdx.x;
  for (int j = blockIdx.x; j < used; j += gridDim.x) {
    const int t0 = j * C;
    const bool ok = lane < C && status[t0 + lane] == 0;
    const double p = lane < C ? score[2 * (t0 + lane)] : 0.0;
    const double e = lane < C ? score[2 * (t0 + lane) + 1] : 0.0;
    const unsigned long long okm = __ballot(ok);
    int a = 0;
    double best = 0.0;
    bool have = false;
    for (int c = 0; c < C; ++c) {  // wave-uniform
      if (!((okm >> c) & 1ull)) continue;
      const double pc = __shfl(p, c);
      if (!have || pc < best) { best = pc; a = c; have = true; }
    }
    const double ea = __shfl(e, a);
    const double hi = __dmul_rn(__dmul_rn(best, __dadd_rn(1.0, ea)), 1.0 + 0x1p-40);
    const bool sep = lane >= C || lane == a || __dmul_rn(p, __dsub_rn(1.0, e)) > hi;
    const bool all_ok = okm == ((C >= 64) ? ~0ull : ((1ull << C) - 1ull));
    const bool decided = all_ok && __all(sep) && !(dbg & MZ_DBG_SCREEN_OFF);
    if (lane == 0) {
      int pk = a;
      if (!decided) {
        const int k = atomicAdd(xcount, 1);
        if (k < xcap) {
          xlist[k] = j;
          pk = -1;
          atomicAdd(stats + 3, 1);
        } else {
          atomicAdd(stats + 0, 1);
        }
      }
      pick[j] = pk;
      atomicAdd(stats + 2, 1);
    }
  }
}

// Tables of each decided target's chosen candidate, from its compact form, into dst instance
// dst_ids[j] (or base + j): cell words, plane strips, meta and reset state (mz_cells_tables).
__global__ __launch_bounds__(WAVE) void k_cand_expand(MzCompact cc, MzDev dst, const int32_t* dst_ids,
                                                      int base, const int* count, int n, int C,
                                                      const int32_t* pick, const uint8_t* algo_list,
                                                      int algo_all) {
  extern __shared__ __align__(16) uint8_t lds[];
  const int used = count ? min(*count, n) : n;
  const int lane = threadIdx.x;
  for (int j = blockIdx.x; j < used; j += gridDim.x) {
    const int pk = pick[j];
    if (pk < 0) continue;  // wave-uniform
    const size_t t = (size_t)j * C + pk;
    const uint32_t meta = cc.meta[t];
    const int N = meta & 0x7F, s = (int)((meta >> 8) & 0xFFFu), g = (int)(meta >> 20);
    const MzCellLds L = mz_cell_lds(lds, dst.P, N);
    const uint32_t* gp = reinterpret_cast<const uint32_t*>(cc.pas + t * cc.Qp);
    const uint32_t* ga = reinterpret_cast<const uint32_t*>(cc.dist + t * cc.Qp);
    uint32_t* lp = reinterpret_cast<uint32_t*>(L.pas);
    uint32_t* la = reinterpret_cast<uint32_t*>(L.A);
    for (int i = lane; i < (L.Q + 3) / 4; i += WAVE) lp[i] = gp[i];
    for (int i = lane; i < (L.Q + 1) / 2; i += WAVE) la[i] = ga[i];
    __syncthreads();
    const int de = dst_ids ? dst_ids[j] : base + j;
    if (lane == 0) dst.algo[de] = (uint8_t)(algo_list ? algo_list[j] : algo_all);
    mz_cells_tables(dst, de, L, N, s, g);
    __syncthreads();
  }
}

// The exact path's candidates: listed target k (= xlist[k], k < *xcount) gets its C candidates
// built with tables at indices k * C + c of `cd` — the same seeds, so the same mazes as its
// compact builds.
__global__ __launch_bounds__(WAVE) void k_cand_rebuild(MzDev cd, const int32_t* xlist, const int* xcount,
                                                       int xcap, const int32_t* ids, int base, int C,
                                                       const uint8_t* algo_list, int algo_all, int dim,
                                                       uint64_t seed, uint32_t epoch, int dbg) {
  extern __shared__ __align__(16) uint8_t lds[];
  const int used = min(*xcount, xcap);
  for (int t = blockIdx.x; t < used * C; t += gridDim.x) {
    const int k = t / C, c = t - k * C;
    const int j = xlist[k];
    const int algo = algo_list ? algo_list[j] : algo_all;
    const uint64_t id = (uint64_t)(ids ? ids[j] : base + j);
    if (threadIdx.x == 0) cd.algo[t] = (uint8_t)algo;
    mz_build_one(cd, t, cd.toroidal, true, algo, mz_cand_seed(seed, id, C, c, epoch, dbg), dim,
                 nullptr, 0, 0, 0, 0, lds);
    __syncthreads();
  }
}

// Candidates of the first min(*count, n) targets that k_mcclendon declined (status != 0; with
// MZ_DBG_DECLINE_EVEN also every even-numbered one): their evaluated grid (toroidal: the bordered
// crop the kernel scores, 0 wall / 1 open / 2 goal) and start / goal go to host memory, slot
// hmap[t] (< hcap; -1: none), for the host restatement (mz_difficulty.hip) that the stream runs
// next (hipLaunchHostFunc, mz_api.hip).
__global__ __launch_bounds__(WAVE) void k_cand_gather(MzDev cd, const int* count, int n, int C,
                                                      const int32_t* status, int32_t* hmap,
                                                      uint8_t* hgrid, int32_t* hinfo, int* hcount,
                                                      int hcap, int gstride, int dbg) {
  const int used = count ? min(*count, n) : n;
  const int lane = threadIdx.x;
  for (int t = blockIdx.x; t < used * C; t += gridDim.x) {
    const bool decl = status[t] != 0 || ((dbg & MZ_DBG_DECLINE_EVEN) && ((t % C) & 1) == 0);
    if (!decl) {
      if (lane == 0) hmap[t] = -1;
      continue;
    }
    int slot = 0;
    if (lane == 0) slot = atomicAdd(hcount, 1);
    slot = __shfl(slot, 0);
    if (lane == 0) hmap[t] = slot < hcap ? slot : -1;
    if (slot >= hcap) continue;
    const bool tor = cd.toroidal;
    const int P = cd.P, o = tor ? 1 : 0;
    const uint32_t m0 = cd.meta0[t], m1 = cd.meta1[t];
    const int Nm = m0 & 0xFF, N = tor ? Nm + 2 : Nm;
    const int gr = (m1 & 0xFF) + o, gc = ((m1 >> 8) & 0xFF) + o;
    const uint32_t* cw = cd.cells + (size_t)t * P * P;
    uint8_t* g = hgrid + (size_t)slot * gstride;
    for (int q = lane; q < N * N; q += WAVE) {
      const int r = q / N, c = q - r * N;
      const bool in = r >= o && r < o + Nm && c >= o && c < o + Nm;
      const bool op = in && (cw[(r - o) * P + (c - o)] & MZ_CELL_OPEN);
      g[q] = !op ? 0 : ((r == gr && c == gc) ? 2 : 1);
    }
    if (lane == 0) {
      int32_t* in = hinfo + 5 * (size_t)slot;
      in[0] = N;
      in[1] = (int)((m0 >> 16) & 0xFF) + o;
      in[2] = (int)(m0 >> 24) + o;
      in[3] = gr;
      in[4] = gc;
    }
  }
}

// Compact form of resident euclidean mazes (the screen's input, mz_screen.h) from their tables:
// passages from the open passage squares, distances from the cell words' D field, the solution's
// cells by walking from the start down the distance field (lane 0). Instances ids[i] (or i) ->
// compact slot i. Used by mz_screen_batch (the screen checked against the exact kernel on any
// resident maze); a maze off the odd lattice is flagged MZ_CMETA_NOSOL (the screen declines it).
__global__ __launch_bounds__(WAVE) void k_compact_from_handle(MzDev d, const int32_t* ids, int n,
                                                              MzCompact cc) {
  const int lane = threadIdx.x;
  for (int i = blockIdx.x; i < n; i += gridDim.x) {
    const int e = ids ? ids[i] : i;
    const uint32_t m0 = d.meta0[e], m1 = d.meta1[e];
    const int N = m0 & 0xFF, sr = (m0 >> 16) & 0xFF, sc = m0 >> 24, gr = m1 & 0xFF, gc = (m1 >> 8) & 0xFF;
    const int W = (N - 1) / 2, Q = W * W, P = d.P;
    const uint32_t* cw = d.cells + (size_t)e * P * P;
    auto open = [&](int r, int c) { return r >= 0 && c >= 0 && r < N && c < N && (cw[r * P + c] & MZ_CELL_OPEN); };
    bool lattice = !d.toroidal && (N & 1) && N < 128 && (sr & 1) && (sc & 1) && (gr & 1) && (gc & 1);
    uint8_t* gp = cc.pas + (size_t)i * cc.Qp;
    uint16_t* ga = cc.dist + (size_t)i * cc.Qp;
    uint32_t* gs = cc.sol + (size_t)i * cc.QWp;
    for (int q = lane; q < Q && lattice; q += WAVE) {
      const int r = 2 * (q / W) + 1, c = 2 * (q % W) + 1;
      gp[q] = (uint8_t)((open(r, c + 1) && c + 2 < N ? 1 : 0) | (open(r + 1, c) && r + 2 < N ? 2 : 0));
      ga[q] = (uint16_t)(cw[r * P + c] & MZ_CELL_D_MASK);
    }
    for (int k = lane; k < cc.QWp; k += WAVE) gs[k] = 0u;
    __syncthreads();
    if (lane == 0 && lattice) {  // start -> goal down the distance field
      int r = sr, c = sc;
      for (int it = 0; it <= N * N; ++it) {
        if ((r & 1) && (c & 1)) {
          const int q = (r >> 1) * W + (c >> 1);
          gs[q >> 5] |= 1u << (q & 31);
        }
        if (r == gr && c == gc) break;
        const int D = (int)(cw[r * P + c] & MZ_CELL_D_MASK);
        int nr = -1, nc = -1;
        for (int k = 0; k < 4; ++k) {
          const int rr = r + mz_dr(k), cc2 = c + mz_dc(k);
          if (open(rr, cc2) && (int)(cw[rr * P + cc2] & MZ_CELL_D_MASK) == D - 1) { nr = rr; nc = cc2; }
        }
        if (nr < 0) { lattice = false; break; }
        r = nr;
        c = nc;
      }
    }
    lattice = __shfl((int)lattice, 0) != 0;
    if (lane == 0)
      cc.meta[i] = (uint32_t)(N & 0x7F) | (lattice ? 0u : MZ_CMETA_NOSOL) |
                   ((uint32_t)((sr >> 1) * W + (sc >> 1)) << 8) | ((uint32_t)((gr >> 1) * W + (gc >> 1)) << 20);
    __syncthreads();
  }
}

// Best-of-C selection (BaseMazeEnv.generate_maze, base_maze_env.py:78-97; toroidal
// toroidal_maze_env.py:40-54) from the order-exact scores: target j keeps the candidate with the
// smallest McClendon difficulty, the FIRST one on ties (the reference replaces only on a strict
// `<`). The kernel compares prod_b (C_b + 1) * C_0 (k_mcclendon's output, whose math.log the
// reference compares): log is monotone, so the first minimum of the products is the first minimum
// of the logs except when two different products round to the same log — counted in stats[1] (a
// candidate within a relative 2^-40 of the minimum, listed before it), never seen on the
// fixtures. A candidate the kernel left to the host (status != 0: not a tree, a hallway beyond
// the wave's set table, ...) takes the host restatement's product (hmap / hprod / hok, gathered
// by k_cand_gather); a group with a candidate that has neither is counted in stats[0] and picks
// among the others; stats[2] counts the groups (count_groups), stats[4] the host scores used.
// One wave per target j < min(*count, n): the chosen candidate's cells, plane strips and
// per-instance words are copied into dst instance dst_ids[j'] (or base + j'), j' = xlist ?
// xlist[j] : j.
__global__ __launch_bounds__(WAVE) void k_cand_select(MzDev cd, MzDev dst, const int32_t* dst_ids,
                                                      int base, const int* count, int n, int C,
                                                      const double* score, const int32_t* status,
                                                      int* stats, const int32_t* xlist,
                                                      const int32_t* hmap, const double* hprod,
                                                      const int32_t* hok, int hcap,
                                                      int count_groups, int dbg) {
  const int used = count ? min(*count, n) : n;
  const int lane = threadIdx.x;
  for (int j = blockIdx.x; j < used; j += gridDim.x) {
    const int t0 = j * C;
    bool ok = false, host = false;
    double p = 0.0;
    if (lane < C) {
      const int t = t0 + lane;
      const bool decl = status[t] != 0 || ((dbg & MZ_DBG_DECLINE_EVEN) && (lane & 1) == 0);
      if (!decl) {
        ok = true;
        p = score[2 * t];
      } else if (hmap) {
        const int h = hmap[t];
        if (h >= 0 && h < hcap && hok[h]) {
          ok = host = true;
          p = hprod[h];
        }
      }
    }
    const unsigned long long okm = __ballot(ok);
    const unsigned long long hostm = __ballot(host);
    // first minimum over the scored candidates (wave-uniform loop over C <= 64)
    int pick = 0;
    double best = 0.0;
    bool have = false;
    for (int c = 0; c < C; ++c) {
      if (!((okm >> c) & 1ull)) continue;
      const double pc = __shfl(p, c);
      if (!have || pc < best) { best = pc; pick = c; have = true; }
    }
    const bool near = ok && lane < pick && p != best && p <= best * (1.0 + 0x1p-40);
    const unsigned long long nearm = __ballot(near);
    if (lane == 0) {
      if (okm != ((C >= 64) ? ~0ull : ((1ull << C) - 1ull))) atomicAdd(stats + 0, 1);
      if (nearm) atomicAdd(stats + 1, 1);
      if (hostm) atomicAdd(stats + 4, __popcll(hostm));
      if (count_groups) atomicAdd(stats + 2, 1);
    }
    const size_t src = (size_t)(t0 + pick);
    const int jd = xlist ? xlist[j] : j;
    const size_t de = (size_t)(dst_ids ? dst_ids[jd] : base + jd);
    const size_t pp = (size_t)cd.P * cd.P, pw = (size_t)cd.PW;
    wave_copy(dst.cells + de * pp, cd.cells + src * pp, pp);
    wave_copy(dst.planes + de * pw, cd.planes + src * pw, pw);
    if (lane == 0) {
      dst.meta0[de] = cd.meta0[src];
      dst.meta1[de] = cd.meta1[src];
      dst.posw[de] = cd.posw[src];
      dst.stw[de] = cd.stw[src];
      dst.curw[de] = cd.curw[src];
      dst.last_term[de] = cd.last_term[src];
      dst.algo[de] = cd.algo[src];
    }
  }
}

// Auto-reset by flag scan: each wave looks at 64 instances' done flags (one coalesced load),
// then resets the done instances of its share of them cooperatively, one after another — waves
// with nothing to do exit at once, no device list or counter is involved. With regen, instances
// whose last step terminated first get a new maze (win -> update_maze,
// off_policy_trainer.py:190-202). `split` waves share a 64-instance group (each resets the done
// instances of 64 / split of its lanes), so that the launch has >= ~1,024 waves: a reset is a
// chain of ~10 dependent global round trips, and a wave runs its share's resets one after
// another. At 65,536 instances (1,024 groups) split = 1 — inside training the launch's time
// is mostly waiting for CU slots beside the acting and update kernels, and one wave per group
// measured best there (68.3 / 68.5 vs 67.0 / 67.4 M env steps/s with 4,
// profiles/r03_adamw_qw8_rd1/train.jsonl); config 2's 4,096 instances (64 groups) spent 218 us
// per vector step here with one wave per group (profiles/r04f_cfg2_train_streams.json).
// k_reset_done's rare in-place build (no bank class, or the bank is exhausted), out of line and
// taking the handle by value: a call that takes the kernel argument's address made every wave
// copy the whole MzDev to scratch on entry (~20 scratch stores per lane), resets or not
__device__ __noinline__ void reset_build_cold(MzDev d, int e, bool tor, uint64_t seed, uint8_t* lds) {
  mz_build_one(d, e, tor, true, d.algo[e], seed, mz_regen_dim(d, e), nullptr, 0, 0, 0, 0, lds);
}

template <bool TOR, bool ENRICH>
__global__ __launch_bounds__(WAVE) void k_reset_done(MzDev d, int regen, uint64_t seed,
                                                     uint32_t epoch, MzOut o, int split) {
  extern __shared__ __align__(16) uint8_t lds[];
  __shared__ __align__(16) uint32_t wsh[32];
  const int grp = blockIdx.x / split, part = blockIdx.x - grp * split;
  const int lane = threadIdx.x, e = grp * WAVE + lane;
  const bool done = e < d.B && ((d.posw[e] >> 20) & 1u);
  // gets a new maze (loaded once, coalesced); a winner whose next size is 0 keeps its maze
  bool win = regen && done && d.last_term[e] && mz_regen_dim(d, e) != 0;
  // this lane's bank slot if it is a winner with a bank class: the group's first slot of the
  // class (k_bank_scan) + its rank among the group's winners of the class — ranked from the
  // codes k_bank_count stored before this launch (split > 1: a sibling wave may have reset some
  // of the group's instances already, so their live flags no longer say "winner")
  int cls = -1, slot = 0;
  if (regen && d.bk_K) {
    const int code = e < d.B ? (int)d.bk_code[e] : -2;
    win = code != -2;
    cls = code;  // -1 or the class for winners, -2 otherwise: only cls >= 0 takes a slot
    if (cls < 0) cls = -1;
    unsigned long long pend = __ballot(cls >= 0);
    while (pend) {
      const int cj = __shfl(cls, __ffsll((long long)pend) - 1);
      const unsigned long long m = __ballot(cls == cj);
      if (cls == cj) slot = d.bk_slot[cj * d.bk_G + grp] + __popcll(m & ((1ull << lane) - 1ull));
      pend &= ~m;
    }
  }
  const int SH = WAVE / split;
  const unsigned long long share = (~0ull >> (WAVE - SH)) << (part * SH);
  unsigned long long bal = __ballot(done) & share;
  while (bal) {
    const int j = __ffsll((long long)bal) - 1;
    bal &= bal - 1;
    const int ej = grp * WAVE + j;
    const int cj = __shfl(cls, j), sj = __shfl(slot, j);
    uint2 meta;
    bool have_meta = false;
    if (__shfl((int)win, j)) {
      have_meta = bank_take(d, ej, cj, sj, meta);
      if (!have_meta)  // no bank class or the bank is exhausted: build in place
        reset_build_cold(d, ej, TOR, seed + (uint64_t)ej + ((uint64_t)epoch << 32), lds);
      __syncthreads();  // this workgroup's global stores are visible to it past the barrier
    }
    reset_one<TOR, ENRICH>(d, ej, o, wsh, have_meta ? &meta : nullptr);
    __syncthreads();
  }
}

// Build (generate or import) the listed instances: one wave per maze, persistent over the list.
__global__ __launch_bounds__(WAVE) void k_build(MzDev d, const int32_t* env_ids, int32_t n,
                                                int generate, const uint8_t* algo_list,
                                                int32_t algo_all, int32_t dim, uint64_t seed,
                                                const uint8_t* grids, const int32_t* sg,
                                                int pymode, uint32_t* py_state) {
  extern __shared__ __align__(16) uint8_t lds[];
  for (int j = blockIdx.x; j < n; j += gridDim.x) {
    const int e = env_ids ? env_ids[j] : j;
    if (generate) {
      const int algo = algo_list ? algo_list[j] : algo_all;
      if (threadIdx.x == 0) d.algo[e] = (uint8_t)algo;
      mz_build_one(d, e, d.toroidal, true, algo, seed + (uint64_t)e, dim, nullptr, 0, 0, 0, 0, lds,
                   pymode, py_state, d.ticket + MZ_TICKET_PYERR);
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
    const int dim = mz_regen_dim(d, e);
    if (!d.last_term[e] || dim == 0) continue;  // uniform per block
    mz_build_one(d, e, d.toroidal, true, d.algo[e], seed + (uint64_t)e + ((uint64_t)epoch << 32),
                 dim, nullptr, 0, 0, 0, 0, lds);
    __syncthreads();
  }
}

__global__ void k_mask(MzDev d, int probs, float* out4) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.B) return;
  float m[4];
  dir_mask(d.posw[e], d.curw[e], d.toroidal, probs, m);
  reinterpret_cast<float4*>(out4)[e] = make_float4(m[0], m[1], m[2], m[3]);
}

// ------------------------------------------------------------------------------------------
// Greedy-row list (dqn_agent.py:104-116 draws `sample < eps` first and evaluates source_net(state)
// only when it fails): the instances whose next fused act (same seed / counter / eps) takes
// greedy_dev[i], in increasing instance order. Two launches, no atomics (a fixed order, so the
// acting forward over the list is deterministic): per-1024-instance counts, then the list.
constexpr int GR_BLOCK = MZ_GR_BLOCK;  // shared with k_tick_count (mz_trainer.hip)
__device__ inline bool greedy_needed(const MzAct& ap, int e) {
  uint32_t u[4];
  act_u(ap, e, u);
  return act_greedy(u, ap.eps ? ap.eps[e] : ap.eps_all);
}

__global__ __launch_bounds__(GR_BLOCK) void k_greedy_count(MzAct ap, int n, int32_t* blk) {
  const int e = blockIdx.x * GR_BLOCK + threadIdx.x;
  const int c = __syncthreads_count(e < n && greedy_needed(ap, e));
  if (threadIdx.x == 0) blk[blockIdx.x] = c;
}

__global__ __launch_bounds__(GR_BLOCK) void k_greedy_list(MzAct ap, int n,
                                                          const int32_t* __restrict__ blk,
                                                          int32_t* rows, int32_t* count,
                                                          int32_t* count_host) {
  __shared__ int wsum[GR_BLOCK / WAVE];
  __shared__ int base;
  const int lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
  const int e = blockIdx.x * GR_BLOCK + threadIdx.x;
  const bool need = e < n && greedy_needed(ap, e);
  const unsigned long long bal = __ballot(need);
  if (lane == 0) wsum[w] = __popcll(bal);
  if (w == 0) {  // this block's offset = the counts of the blocks before it; block 0: the total
    int pre = 0, tot = 0;
    for (int i = lane; i < (int)gridDim.x; i += WAVE) {
      const int v = blk[i];
      pre += i < (int)blockIdx.x ? v : 0;
      tot += v;
    }
    for (int o = WAVE / 2; o; o >>= 1) {
      pre += __shfl_xor(pre, o);
      tot += __shfl_xor(tot, o);
    }
    if (lane == 0) {
      base = pre;
      if (blockIdx.x == 0) {
        *count = tot;
        if (count_host) *count_host = tot;
      }
    }
  }
  __syncthreads();
  int off = base;
  for (int i = 0; i < w; ++i) off += wsum[i];
  if (need) rows[off + __popcll(bal & ((1ull << lane) - 1ull))] = e;
}

__global__ void k_act(MzDev d, MzAct ap) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.B) return;
  ap.act_out[e] = act_sample(ap, e, d.posw[e], d.curw[e], d.toroidal);
}

__global__ void k_expand(const uint32_t* bits, float* out, int n) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)n * 675;
  if (t >= total) return;
  const long i = t / 675, f = t - i * 675;
  out[t] = (float)((bits[i * MZ_WINDOW_WORDS + (f >> 5)] >> (f & 31)) & 1u);
}

// Per-instance maze metadata as int32 [B][6]: N, start r/c, goal r/c, max_steps.
__global__ void k_meta(MzDev d, int32_t* out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.B) return;
  const uint32_t m0 = d.meta0[e], m1 = d.meta1[e];
  int32_t* o = out + 6 * (size_t)e;
  o[0] = m0 & 0xFF; o[1] = (m0 >> 16) & 0xFF; o[2] = m0 >> 24;
  o[3] = m1 & 0xFF; o[4] = (m1 >> 8) & 0xFF; o[5] = m1 >> 16;
}

// PPO returns (ppo_agent.py:170-179): per episode, backwards, acc = r + acc * gamma in float64
// (the reference's Python floats), stored as float32 (torch.tensor of the list). One lane per
// episode; episode `k` is row rows[k] of rew (leading dimension ld), length lens[k].
__global__ void k_returns(const double* rew, int ld, const int32_t* rows, const int32_t* lens,
                          int n, double gamma, float* out, int ldo) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const double* r = rew + (size_t)rows[k] * ld;
  float* o = out + (size_t)k * ldo;
  double acc = 0.0;
  for (int t = lens[k] - 1; t >= 0; --t) {
    acc = __dadd_rn(r[t], __dmul_rn(acc, gamma));
    o[t] = (float)acc;
  }
}

// the build kernels may need more than the 64 KiB default dynamic LDS at large max_dim
hipError_t mz_lds_attr(const void* fn, size_t bytes) {
  if (bytes <= 65536) return hipSuccess;
  return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

#ifndef MZ_LITE  // r-prim candidates in the lite regions (A/B builds: 0)
#define MZ_LITE 1
#endif
#ifndef MZ_LITE_DFS  // dfs candidates too
#define MZ_LITE_DFS 1
#endif

#ifndef MZ_PACK_DFS  // dfs candidate lists packed too (A/B builds: 0)
#define MZ_PACK_DFS 1
#endif
#ifndef MZ_BANK_WGS
#define MZ_BANK_WGS 0
#endif
// resident lite candidate builds (k_cand_compact_lite; 0 = as many as fit, 7 per CU at 81 x 81):
// the refill shares the chip with the trainer's acting and update streams, and builds past 5 per
// CU hold LDS their kernels wait for — best-of-6 DDQN training 71.5 -> 75.3 M env steps/s at
// 1,280 (768 / 1,024 / 1,536 / 1,792 / all: 70.2 / 73.8 / 71.3 / 72.6 / 71.5 M, profiles/r06t/)
#ifndef MZ_LITE_WGS
#define MZ_LITE_WGS 1280
#endif
#ifndef MZ_EXPAND_WGS  // resident k_cand_expand workgroups (0 = the build grid)
#define MZ_EXPAND_WGS 0
#endif
// Build launches: the LDS one maze build needs — the cell-space layouts for Philox mazes
// (mz_build_cells), else the square grid (+ the CPython generator's tables) — and a persistent
// grid of 4,096 workgroups or, when more fit, as many as can be resident at once (256 CUs x the
// LDS share, at most 32 waves per CU).
size_t mz_build_lds_launch(int P, bool tor, bool generate, int pymode) {
  if (MZ_CELL_BUILD && generate && pymode == MZ_PY_PHILOX)
    return tor ? mz_torus_lds_bytes(P) : mz_cell_lds_bytes(P);
  return mz_build_lds_bytes_mode(P, generate ? pymode : 0);
}
int mz_build_grid(int n, size_t lds) {
  const int per_cu = (int)std::min<size_t>(32, std::max<size_t>(1, (160 * 1024) / std::max<size_t>(lds, 1)));
  return std::max(1, std::min(n, std::max(4096, 256 * per_cu)));
}

}  // namespace

// ------------------------------------------------------------------------------------------
// launchers (called by mz_api.hip)
size_t mz_build_lds_size(int P) { return mz_build_lds_bytes(P); }

hipError_t mz_launch_build(const MzDev& d, const int32_t* env_ids, int32_t n, bool generate,
                           const uint8_t* algo_list, int32_t algo_all, int32_t dim, uint64_t seed,
                           const uint8_t* grids, const int32_t* start_goal, int pymode,
                           uint32_t* py_state, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const size_t lds = mz_build_lds_launch(d.P, d.toroidal, generate, pymode);
  hipError_t ae = mz_lds_attr(reinterpret_cast<const void*>(k_build), lds);
  if (ae != hipSuccess) return ae;
  hipLaunchKernelGGL(k_build, dim3(mz_build_grid(n, lds)), dim3(WAVE), lds, s, d, env_ids, n,
                     (int)generate, algo_list, algo_all, dim, seed, grids, start_goal, pymode,
                     py_state);
  return hipGetLastError();
}

hipError_t mz_launch_regen(const MzDev& d, const int32_t* idx, const int32_t* count,
                           int32_t n_static, uint64_t seed, uint32_t epoch, hipStream_t s) {
  if (n_static <= 0) return hipSuccess;
  const size_t lds = mz_build_lds_launch(d.P, d.toroidal, true, MZ_PY_PHILOX);
  hipError_t ae = mz_lds_attr(reinterpret_cast<const void*>(k_regen_list), lds);
  if (ae != hipSuccess) return ae;
  hipLaunchKernelGGL(k_regen_list, dim3(mz_build_grid(n_static, lds)), dim3(WAVE), lds, s, d, idx,
                     count, n_static, seed, epoch);
  return hipGetLastError();
}

#ifndef MZ_SMALL_B
#define MZ_SMALL_B 16384  // batches up to this size step with 4 instances per wave
#endif
template <int I, bool T, bool E>
void launch_step_ite(const MzDev& d, const int32_t* act, const MzAct& a, bool has_act, bool ar,
                     const MzOut& o, hipStream_t s) {
  dim3 grid((d.B + I * MZ_SPW - 1) / (I * MZ_SPW)), block(WAVE * MZ_SPW);
  if (has_act) {
    if (ar) hipLaunchKernelGGL((k_step<I, T, E, true, true>), grid, block, 0, s, d, act, a, o);
    else hipLaunchKernelGGL((k_step<I, T, E, true, false>), grid, block, 0, s, d, act, a, o);
  } else {
    if (ar) hipLaunchKernelGGL((k_step<I, T, E, false, true>), grid, block, 0, s, d, act, a, o);
    else hipLaunchKernelGGL((k_step<I, T, E, false, false>), grid, block, 0, s, d, act, a, o);
  }
}

template <bool T, bool E>
void launch_step_te(const MzDev& d, const int32_t* act, const MzAct& a, bool has_act, bool ar,
                    const MzOut& o, hipStream_t s) {
  if (d.B <= MZ_SMALL_B) launch_step_ite<4, T, E>(d, act, a, has_act, ar, o, s);
  else launch_step_ite<IPW, T, E>(d, act, a, has_act, ar, o, s);
}

hipError_t mz_launch_step(const MzDev& d, const int32_t* act, const MzAct* ap, bool autoreset,
                          const MzOut& o0, hipStream_t s) {
  MzAct a{};
  if (ap) a = *ap;
  MzOut o = o0;
  o.window_nt = o.window && (size_t)d.B * 675 * sizeof(float) > MZ_WINDOW_NT_BYTES;
  if (d.toroidal) {
    if (d.enrich) launch_step_te<true, true>(d, act, a, ap != nullptr, autoreset, o, s);
    else launch_step_te<true, false>(d, act, a, ap != nullptr, autoreset, o, s);
  } else {
    if (d.enrich) launch_step_te<false, true>(d, act, a, ap != nullptr, autoreset, o, s);
    else launch_step_te<false, false>(d, act, a, ap != nullptr, autoreset, o, s);
  }
  return hipGetLastError();
}

hipError_t mz_launch_reset_list(const MzDev& d, const int32_t* idx, int32_t* count,
                                int32_t n_static, const MzOut& o, hipStream_t s) {
  if (n_static <= 0) return hipSuccess;
  const int blocks = n_static < 1024 ? n_static : 1024;
#define MZ_RL(T, E) \
  hipLaunchKernelGGL((k_reset_list<T, E>), dim3(blocks), dim3(WAVE), 0, s, d, idx, count, n_static, o)
  if (d.toroidal) { if (d.enrich) MZ_RL(true, true); else MZ_RL(true, false); }
  else { if (d.enrich) MZ_RL(false, true); else MZ_RL(false, false); }
#undef MZ_RL
  hipError_t e = hipGetLastError();
  if (e == hipSuccess && count) e = hipMemsetAsync(count, 0, sizeof(int32_t), s);  // consumed
  return e;
}

hipError_t mz_launch_reset_done(const MzDev& d, int regen, uint64_t seed, uint32_t epoch,
                                const MzOut& o, hipStream_t s) {
  const int groups = (d.B + WAVE - 1) / WAVE;
  int split = 1;  // waves per 64-instance group: >= 1,024 waves in the launch
  while (split < WAVE && groups * split < 1024) split <<= 1;
  const int blocks = groups * split;
  size_t lds = 0;
  hipError_t ae = hipSuccess;
  if (regen && d.bk_K) {  // the winners' bank slots, in instance order (k_bank_count / k_bank_scan)
    ae = hipMemsetAsync(d.bk_slot, 0, sizeof(int) * 3 * (size_t)d.bk_nd * d.bk_G, s);
    if (ae != hipSuccess) return ae;
    hipLaunchKernelGGL(k_bank_count, dim3(d.bk_G), dim3(WAVE), 0, s, d);
    hipLaunchKernelGGL(k_bank_scan, dim3(3 * d.bk_nd), dim3(BS_T), 0, s, d);
  }
#define MZ_RD(T, E)                                                                           \
  do {                                                                                        \
    if (regen) {                                                                              \
      lds = mz_build_lds_launch(d.P, d.toroidal, true, MZ_PY_PHILOX);                         \
      ae = mz_lds_attr(reinterpret_cast<const void*>(k_reset_done<T, E>), lds);              \
      if (ae != hipSuccess) return ae;                                                        \
    }                                                                                         \
    hipLaunchKernelGGL((k_reset_done<T, E>), dim3(blocks), dim3(WAVE), lds, s, d, regen, seed, \
                       epoch, o, split);                                                      \
  } while (0)
  if (d.toroidal) { if (d.enrich) MZ_RD(true, true); else MZ_RD(true, false); }
  else { if (d.enrich) MZ_RD(false, true); else MZ_RD(false, false); }
#undef MZ_RD
  return hipGetLastError();
}

hipError_t mz_launch_cand_build(const MzDev& cd, const int32_t* ids, int base, const int* count, int n,
                                int C, const uint8_t* algo_list, int algo_all, int dim,
                                uint64_t seed, uint32_t epoch, hipStream_t s, int dbg) {
  if (n <= 0 || C <= 0) return hipSuccess;
  // euclidean Philox r-prim / dfs lists (the headline's bank classes) build MZ_PACK per wave
  const bool packed = MZ_PACK > 1 && MZ_CELL_BUILD && !cd.toroidal && !algo_list &&
                      (algo_all == MZ_ALGO_RPRIM_DEV || (MZ_PACK_DFS && algo_all == MZ_ALGO_DFS_DEV));
  const size_t stride = packed ? mz_align16(mz_cell_lds_bytes(cd.P)) : 0;
  const size_t lds = packed ? MZ_PACK * stride : mz_build_lds_launch(cd.P, cd.toroidal, true, MZ_PY_PHILOX);
  const void* kfn = packed ? reinterpret_cast<const void*>(k_cand_build_packed)
                           : reinterpret_cast<const void*>(k_cand_build);
  hipError_t ae = mz_lds_attr(kfn, lds);
  if (ae != hipSuccess) return ae;
  // a bank refill runs beside the trainer's acting and update kernels: MZ_BANK_WGS caps its
  // resident builds (0 = as many as fit) so that it leaves CUs / LDS to them
  const int total = packed ? (n * C + MZ_PACK - 1) / MZ_PACK : n * C;
  const int grid = std::max(1, MZ_BANK_WGS > 0 ? std::min(total, MZ_BANK_WGS) : mz_build_grid(total, lds));
  if (packed)
    hipLaunchKernelGGL(k_cand_build_packed, dim3(grid), dim3(WAVE), lds, s, cd, ids, base, count, n, C,
                       algo_all, dim, seed, epoch, (int)stride, dbg);
  else
    hipLaunchKernelGGL(k_cand_build, dim3(grid), dim3(WAVE), lds, s, cd, ids, base, count, n, C,
                       algo_list, algo_all, dim, seed, epoch, dbg);
  return hipGetLastError();
}

hipError_t mz_launch_cand_compact(const MzCompact& cc, int P, const int32_t* ids, int base,
                                  const int* count, int n, int C, const uint8_t* algo_list,
                                  int algo_all, int dim, uint64_t seed, uint32_t epoch, hipStream_t s,
                                  int dbg) {
  if (n <= 0 || C <= 0) return hipSuccess;
  if (dim > P || cc.Qp < mz_compact_qp(P)) return hipErrorInvalidValue;
  if (MZ_LITE && !algo_list &&
      (algo_all == MZ_ALGO_RPRIM_DEV || (MZ_LITE_DFS && algo_all == MZ_ALGO_DFS_DEV))) {
    // r-prim / dfs: the lite regions
    const size_t stride = mz_align16(mz_lite_lds_bytes(P, algo_all) + (MZ_RING ? 4 * 4 * (WAVE / MZ_LPACK) : 0));
    const size_t lds = MZ_LPACK * stride + mz_lite_scratch_bytes(P);
    hipError_t ae = mz_lds_attr(reinterpret_cast<const void*>(k_cand_compact_lite), lds);
    if (ae != hipSuccess) return ae;
    const int total = (n * C + MZ_LPACK - 1) / MZ_LPACK;
    const int cap = MZ_BANK_WGS > 0 ? MZ_BANK_WGS : MZ_LITE_WGS;
    const int grid = std::max(1, cap > 0 ? std::min(total, cap) : mz_build_grid(total, lds));
    hipLaunchKernelGGL(k_cand_compact_lite, dim3(grid), dim3(WAVE), lds, s, cc, P, ids, base, count,
                       n, C, algo_all, dim, seed, epoch, (int)stride, dbg);
    return hipGetLastError();
  }
  const bool packed = MZ_PACK > 1 && !algo_list &&
                      (algo_all == MZ_ALGO_RPRIM_DEV || (MZ_PACK_DFS && algo_all == MZ_ALGO_DFS_DEV));
  const size_t stride = mz_align16(mz_cell_lds_bytes(P));
  const size_t lds = packed ? MZ_PACK * stride : stride;
  const void* kfn = packed ? reinterpret_cast<const void*>(k_cand_compact_packed)
                           : reinterpret_cast<const void*>(k_cand_compact);
  hipError_t ae = mz_lds_attr(kfn, lds);
  if (ae != hipSuccess) return ae;
  const int total = packed ? (n * C + MZ_PACK - 1) / MZ_PACK : n * C;
  const int grid = std::max(1, MZ_BANK_WGS > 0 ? std::min(total, MZ_BANK_WGS) : mz_build_grid(total, lds));
  if (packed)
    hipLaunchKernelGGL(k_cand_compact_packed, dim3(grid), dim3(WAVE), lds, s, cc, P, ids, base, count,
                       n, C, algo_all, dim, seed, epoch, (int)stride, dbg);
  else
    hipLaunchKernelGGL(k_cand_compact, dim3(grid), dim3(WAVE), lds, s, cc, P, ids, base, count, n, C,
                       algo_list, algo_all, dim, seed, epoch, dbg);
  return hipGetLastError();
}

hipError_t mz_launch_cand_pick(const int* count, int n, int C, const double* score,
                               const int32_t* status, int32_t* pick, int32_t* xlist, int* xcount,
                               int xcap, int* stats, hipStream_t s, int dbg) {
  if (n <= 0) return hipSuccess;
  if (C < 1 || C > WAVE) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_cand_pick, dim3(std::min(n, 4096)), dim3(WAVE), 0, s, count, n, C, score,
                     status, pick, xlist, xcount, xcap, stats, dbg);
  return hipGetLastError();
}

hipError_t mz_launch_cand_expand(const MzCompact& cc, const MzDev& dst, const int32_t* dst_ids,
                                 int base, const int* count, int n, int C, const int32_t* pick,
                                 const uint8_t* algo_list, int algo_all, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const size_t lds = mz_align16(mz_cell_lds_bytes(dst.P));
  hipError_t ae = mz_lds_attr(reinterpret_cast<const void*>(k_cand_expand), lds);
  if (ae != hipSuccess) return ae;
  const int eg = mz_build_grid(n, lds);
  hipLaunchKernelGGL(k_cand_expand, dim3(std::max(1, MZ_EXPAND_WGS > 0 ? std::min(eg, MZ_EXPAND_WGS) : eg)),
                     dim3(WAVE), lds, s, cc,
                     dst, dst_ids, base, count, n, C, pick, algo_list, algo_all);
  return hipGetLastError();
}

hipError_t mz_launch_cand_rebuild(const MzDev& cd, const int32_t* xlist, const int* xcount, int xcap,
                                  const int32_t* ids, int base, int C, const uint8_t* algo_list,
                                  int algo_all, int dim, uint64_t seed, uint32_t epoch, hipStream_t s,
                                  int dbg) {
  if (xcap <= 0 || C <= 0) return hipSuccess;
  const size_t lds = mz_build_lds_launch(cd.P, cd.toroidal, true, MZ_PY_PHILOX);
  hipError_t ae = mz_lds_attr(reinterpret_cast<const void*>(k_cand_rebuild), lds);
  if (ae != hipSuccess) return ae;
  // the list is nearly always empty: a small persistent grid
  const int grid = std::max(1, std::min(xcap * C, 1024));
  hipLaunchKernelGGL(k_cand_rebuild, dim3(grid), dim3(WAVE), lds, s, cd, xlist, xcount, xcap, ids, base,
                     C, algo_list, algo_all, dim, seed, epoch, dbg);
  return hipGetLastError();
}

hipError_t mz_launch_cand_gather(const MzDev& cd, const int* count, int n, int C,
                                 const int32_t* status, int32_t* hmap, uint8_t* hgrid,
                                 int32_t* hinfo, int* hcount, int hcap, int gstride, hipStream_t s,
                                 int dbg) {
  if (n <= 0 || C <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_cand_gather, dim3(std::max(1, std::min(n * C, 1024))), dim3(WAVE), 0, s, cd,
                     count, n, C, status, hmap, hgrid, hinfo, hcount, hcap, gstride, dbg);
  return hipGetLastError();
}

hipError_t mz_launch_compact_from_handle(const MzDev& d, const int32_t* ids, int n, const MzCompact& cc,
                                        hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (cc.Qp < mz_compact_qp(d.P)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_compact_from_handle, dim3(std::min(n, 4096)), dim3(WAVE), 0, s, d, ids, n, cc);
  return hipGetLastError();
}

hipError_t mz_launch_cand_select(const MzDev& cd, const MzDev& dst, const int32_t* dst_ids,
                                 int base, const int* count, int n, int C, const double* score,
                                 const int32_t* status, int* stats, hipStream_t s,
                                 const int32_t* xlist, const int32_t* hmap, const double* hprod,
                                 const int32_t* hok, int hcap, int count_groups, int dbg) {
  if (n <= 0) return hipSuccess;
  if (C < 1 || C > WAVE) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_cand_select, dim3(std::min(n, 4096)), dim3(WAVE), 0, s, cd, dst, dst_ids,
                     base, count, n, C, score, status, stats, xlist, hmap, hprod, hok, hcap,
                     count_groups, dbg);
  return hipGetLastError();
}

hipError_t mz_launch_meta(const MzDev& d, int32_t* out, hipStream_t s) {
  hipLaunchKernelGGL(k_meta, dim3((d.B + 255) / 256), dim3(256), 0, s, d, out);
  return hipGetLastError();
}

hipError_t mz_launch_returns(const double* rew, int ld, const int32_t* rows, const int32_t* lens,
                             int n, double gamma, float* out, int ldo, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_returns, dim3((n + 63) / 64), dim3(64), 0, s, rew, ld, rows, lens, n, gamma,
                     out, ldo);
  return hipGetLastError();
}

hipError_t mz_launch_mask(const MzDev& d, int probs, float* out4, hipStream_t s) {
  hipLaunchKernelGGL(k_mask, dim3((d.B + 255) / 256), dim3(256), 0, s, d, probs, out4);
  return hipGetLastError();
}

hipError_t mz_launch_greedy_list(const MzAct& ap, int n, const int32_t* blk, int32_t* rows,
                                 int32_t* count, int32_t* count_host, hipStream_t s) {
  const int blocks = (n + GR_BLOCK - 1) / GR_BLOCK;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(k_greedy_list, dim3(blocks), dim3(GR_BLOCK), 0, s, ap, n, blk, rows, count,
                     count_host);
  return hipGetLastError();
}

hipError_t mz_launch_greedy_rows(const MzAct& ap, int n, int32_t* blk, int32_t* rows,
                                 int32_t* count, int32_t* count_host, hipStream_t s) {
  const int blocks = (n + GR_BLOCK - 1) / GR_BLOCK;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(k_greedy_count, dim3(blocks), dim3(GR_BLOCK), 0, s, ap, n, blk);
  return mz_launch_greedy_list(ap, n, blk, rows, count, count_host, s);
}

hipError_t mz_launch_act(const MzDev& d, const MzAct& ap, hipStream_t s) {
  hipLaunchKernelGGL(k_act, dim3((d.B + 255) / 256), dim3(256), 0, s, d, ap);
  return hipGetLastError();
}

hipError_t mz_launch_expand(const uint32_t* bits, float* out, int n, hipStream_t s) {
  long total = (long)n * 675;
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL(k_expand, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, bits, out, n);
  return hipGetLastError();
}
