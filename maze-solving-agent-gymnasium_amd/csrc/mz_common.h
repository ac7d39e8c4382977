// mz_common.h — shared layout + device helpers for the MI355X maze env (libmazerl.so).
//
// HBM layout (one handle = B env instances, pitch P = max_dim, planes padded to 128 bits/row):
//   cells  u32 [B][P*P]  per-cell word:  D (bits 0-12, BFS distance to goal, < 8192 for P <= 127)
//                                         | best-next code (13-15: action 0-3, 4 = stay)
//                                         | open (16) | open-neighbour mask (17-20, per action)
//                                         | visit count (21-28) | episode tag (29-31)
//                        Everything the reference recomputes with A* every step
//                        (_find_best_next_cell base_maze_env.py:224-262, find_path
//                        simple_maze_env.py:70-79) is a function of the cell: computed once per
//                        maze, gathered once per step. The visit count (visited_cell.count,
//                        :194; saturating at 255, exact since the penalties are -1.0 for k >= 188)
//                        rides in the same word, so one gather serves both; it counts only when
//                        its tag equals the instance's episode tag (stw bits 24-26), so a reset
//                        bumps the tag instead of clearing the maze (a full clear every 8th reset).
//   planes u32 [B][NS][P][2]  open / visited bit planes in column STRIPS: strip s holds the 32
//                        columns 18s .. 18s + 31 (torus: (18s + j) mod N; euclidean columns >= N
//                        are 0), one (open, visited) u32 pair per row, NS = ceil(P / 18). Any
//                        15-column window [c0, c0 + 14] lies in strip c0 / 18 at bit offset
//                        c0 mod 18, so a window is 15 consecutive 8-B rows of one strip (120 B,
//                        about two 128-B lines; the row-major pair layout this replaced read a
//                        16-row x 24-B band, about four). A cell sits in up to two strips
//                        (euclidean), so its visited bit is set in each.
//                        visited = the reference's non_visited plane inverted
//                        (base_maze_env.py:40-41,184).
//   SoA per instance (coalesced u32 each):
//     meta0 = N | N<<8 (H,W) | sr<<16 | sc<<24     meta1 = gr | gc<<8 | max_steps<<16
//     posw  = r | c<<8 | nm<<16 (min(len(visited_cell),2)) | last_action<<18 | done<<20
//     stw   = steps (0-15) | invalid streak (16-23, saturating) | episode tag (24-26)
//     curw  = cells word at the current position
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MZ_CELL_D_MASK 0x1FFFu
#define MZ_CELL_CODE_SHIFT 13
#define MZ_CELL_OPEN (1u << 16)
#define MZ_CELL_NB_SHIFT 17
#define MZ_CELL_CNT_SHIFT 21
#define MZ_CELL_TAG_SHIFT 29
#define MZ_CELL_STATIC ((1u << MZ_CELL_CNT_SHIFT) - 1u)
#define MZ_STW_TAG_SHIFT 24

// visit count of cell word w for the episode tagged `tag`
__host__ __device__ inline int mz_cell_count(uint32_t w, uint32_t tag) {
  return (w >> MZ_CELL_TAG_SHIFT) == tag ? (int)((w >> MZ_CELL_CNT_SHIFT) & 0xFFu) : 0;
}
#define MZ_TICKET_PYERR 8

struct MzDev {
  int B, P, toroidal, enrich;
  int NS, PW;               // plane strips (ceil(P/18)) and plane words per instance (NS*P*2)
  uint32_t* cells;
  uint32_t* planes;
  uint32_t* meta0;
  uint32_t* meta1;
  uint32_t* posw;
  uint32_t* stw;
  uint32_t* curw;
  uint8_t* algo;            // per-instance algorithm id for regeneration
  uint8_t* last_term;       // per-instance: last step terminated (for regen_won)
  const double* pen_visit;  // [256] 0.0 - (1 - exp(-0.2 k))   (base_maze_env.py:194)
  const double* pen_inv;    // [256] 0.0 - (1 - exp(-0.15 k))  (base_maze_env.py:200)
  int* ticket;              // [16]: [0] exit ticket of k_reset_list (done-count consumption),
                            // [MZ_TICKET_PYERR] CPython-generation set-table overflow flag
  // Active maze bank (mz_bank_*): mazes generated ahead of time that a win copies in instead
  // of building one inside the reset launch. Slot j of algorithm a and maze size index di lives
  // at index (bk_aidx(a) * bk_nd + di) * bk_K + j of the bank arrays; bk_head[a * bk_nd + di]
  // counts the slots consumed so far.
  int bk_K;                 // slots per (algorithm, size); 0 = no bank in use
  int bk_nd;                // maze sizes the bank holds
  int8_t bk_didx[128];      // maze size N -> its index in the bank, -1: not held
  uint32_t bk_amask;        // algorithms the bank holds (bit a)
  const uint32_t* bk_cells; // [slots][P*P]
  const uint32_t* bk_planes;// [slots][PW]
  const uint32_t* bk_meta0; // [slots]
  const uint32_t* bk_meta1; // [slots]
  int* bk_head;             // [3][bk_nd]
  // deterministic slot assignment for k_reset_done (k_bank_count / k_bank_scan): per bank class
  // (algorithm id a, size index di) -> a * bk_nd + di and 64-instance group g, the first slot
  // of the group's winners, bk_slot[class * bk_G + g]
  int* bk_slot;             // [3 * bk_nd][bk_G]
  int bk_G;                 // 64-instance groups, ceil(B / 64)
  // per instance, what k_bank_count saw before the reset launch: -2 not a winner, -1 a winner
  // without a bank class, else its class. k_reset_done ranks a group's winners from these: with
  // several waves per group, live state (done flag, last_term) read by one wave may already be
  // reset by a sibling wave, which shifted the ranks (two winners on one slot, run to run)
  int8_t* bk_code;          // [B]
  // per-instance size of a winner's next maze (the variable-size envs' update_maze growth,
  // simple_variable_maze_env.py:93-112 / toroidal_variable_maze_env.py:113-131): 0 = the winner
  // keeps its maze (the reference's `shape > max_shape` branch), null = its current size
  const uint8_t* regen_dim;
};

// size of instance e's next maze when it wins (0: no new maze; a size the handle cannot hold —
// even, < 5 or above the pitch — counts as 0, so no build can write past the instance's arrays)
__device__ inline int mz_regen_dim(const MzDev& d, int e) {
  if (!d.regen_dim) return (int)(d.meta0[e] & 0xFF);
  const int n = (int)d.regen_dim[e];
  return (n >= 5 && n <= d.P && (n & 1)) ? n : 0;
}

__host__ __device__ inline int mz_bank_aidx(uint32_t amask, int a) {
  return __builtin_popcount(amask & ((1u << a) - 1u));
}

struct MzAct {  // fused epsilon-greedy act (dqn_agent.py:104-116)
  const float* eps;
  float eps_all;
  const int64_t* greedy;
  uint64_t seed, counter;
  int32_t* act_out;
};

struct MzOut {
  float* reward;
  double* reward64;
  uint8_t* terminated;
  uint8_t* truncated;
  int32_t* pos;
  int32_t* best_dir;
  float* obs6;
  uint32_t* window_bits;
  float* window;
  int32_t* done_idx;
  int32_t* done_count;
  int window_nt;  // set by mz_launch_step: f32 windows as non-temporal stores (past the MALL)
};
// f32 window bytes per step above which k_step stores them non-temporally (the 256 MB
// Infinity Cache no longer holds the stream; mz_env.hip store_window_f32)
#define MZ_WINDOW_NT_BYTES (256ull << 20)

// BaseMazeEnv.ACTIONS (base_maze_env.py:19-24): 0 down, 1 up, 2 right, 3 left
__host__ __device__ inline int mz_dr(int a) { return a == 0 ? 1 : (a == 1 ? -1 : 0); }
__host__ __device__ inline int mz_dc(int a) { return a == 2 ? 1 : (a == 3 ? -1 : 0); }
__host__ __device__ inline int mz_wrap(int v, int n) { v %= n; return v < 0 ? v + n : v; }
// v mod n for v within a few multiples of n (window offsets, +-1 moves): no integer division
__host__ __device__ inline int mz_wrapn(int v, int n) {
  while (v < 0) v += n;
  while (v >= n) v -= n;
  return v;
}

// ------------------------------------------------------------------------------------------
// Philox4x32-10 — identical definition in oracle/mzoracle.c (mzo_philox).
__host__ __device__ inline void mz_philox(uint64_t key, uint64_t ctr_hi, uint64_t ctr_lo,
                                          uint32_t out[4]) {
  uint32_t c0 = (uint32_t)ctr_lo, c1 = (uint32_t)(ctr_lo >> 32), c2 = (uint32_t)ctr_hi,
           c3 = (uint32_t)(ctr_hi >> 32);
  uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    if (i) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    uint32_t lo0 = 0xD2511F53u * c0, hi0 = (uint32_t)(((uint64_t)0xD2511F53u * c0) >> 32);
    uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = (uint32_t)(((uint64_t)0xCD9E8D57u * c2) >> 32);
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

#define MZ_GEN_STREAM 0x6D617A65ull  // 'maze': generation draws
#define MZ_ACT_STREAM 0x61637421ull  // 'act!': exploration draws
#define MZ_REPLAY_STREAM 0x72706c79ull  // 'rply': replay sample rows
#define MZ_PPO_STREAM 0x70706f21ull  // 'ppo!': PPO policy draws

// Sequential draw stream (one per maze): draw k = word (k & 3) of philox(key, {GEN, k >> 2}).
struct MzRng {
  uint64_t key, n;
  uint32_t buf[4];
  // the word by selects, not buf[n & 3]: a dynamic index put buf in scratch memory, and every
  // draw of a build's serial carve chain then waited on a scratch load
  __device__ inline uint32_t u32() {
    const uint32_t k = (uint32_t)n & 3u;
    if (k == 0) mz_philox(key, MZ_GEN_STREAM, n >> 2, buf);
    ++n;
    const uint32_t lo = (k & 1u) ? buf[1] : buf[0];
    const uint32_t hi = (k & 1u) ? buf[3] : buf[2];
    return (k & 2u) ? hi : lo;
  }
  __device__ inline uint32_t below(uint32_t m) { return (uint32_t)(((uint64_t)u32() * m) >> 32); }
};

// extract_submaze axis start (maze_handler.py:18-45), N >= 15 (Q7 excluded at load time)
__device__ inline int mz_win_start(int p, int N) {
  if (N == 15) return 0;
  if (p - 7 >= 0 && p + 7 < N) return p - 7;
  if (p - 7 < 0) return 0;
  return N - 15;
}

// ---- plane strips (see the layout above)
#define MZ_STRIP_STRIDE 18
__host__ __device__ inline int mz_nstrips(int P) { return (P + MZ_STRIP_STRIDE - 1) / MZ_STRIP_STRIDE; }

// the (open, visited) pair of row R of strip s of instance e
__device__ inline uint2* mz_strip_row(const MzDev& d, size_t e, int s, int R) {
  return reinterpret_cast<uint2*>(d.planes) + ((e * d.NS + s) * d.P + R);
}

// bits j of strip s that hold column col (euclidean: at most one; torus: j = col - 18s mod N,
// + N, + 2N, ... < 32 — a column repeats inside a strip when N < 32)
__device__ inline uint32_t mz_strip_colmask(int s, int col, int N, bool tor) {
  const int j0 = col - MZ_STRIP_STRIDE * s;
  if (!tor) return (j0 >= 0 && j0 < 32) ? (1u << j0) : 0u;
  uint32_t m = 0u;
  for (int j = mz_wrapn(j0, N); j < 32; j += N) m |= 1u << j;
  return m;
}

#define MZ_ALGO_RPRIM_DEV 0
#define MZ_ALGO_DFS_DEV 1
#define MZ_ALGO_PRIMKILL_DEV 2
