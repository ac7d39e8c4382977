// mz_mcclendon.hip — McClendon maze difficulty on the GPU, one 1,024-thread workgroup per maze.
//
// The reference (lib/maze_difficulty_evaluation/maze_complexity_evaluation.py:38-329) builds a
// networkx graph G of "points" (turns and junctions along the solution path and along the path
// from every dead end back to the start, maze_complexity_evaluation.py:57-91), splits it into
// hallways (:186-221) and branches (:223-259), and returns log(prod_b (C_b + 1) * C_0) with
// C_h = D_h * sum_e 1 / (2 d_e) (:286-329). The float64 result depends on networkx's insertion
// orders (node order, per-node adjacency order). The host restatement (mz_difficulty.hip) keeps
// those orders by building the graph serially; here they are derived in parallel from the maze's
// tree structure (every generator makes a perfect maze: its open squares form a tree):
//   points      the squares that decompose_in_turns keeps on some path: degree != 2, corners,
//               start and goal (a straight degree-2 square is never one) — path independent;
//   G edges     the tree contracted to its points, d = squares in between;
//   node order  the solution's points in path order, then every other point by (first(x),
//               -D(x)): first(x) = the row-major rank of the first dead end whose path reaches x
//               (= the smallest dead-end rank in x's subtree, the tree rooted at the start), D the
//               distance to the goal (a dead-end path inserts its new points from the dead end up);
//   adjacency   solution point: [predecessor, successor, side children by first]; other point:
//               [the child its first path came through, parent, other children by first] — the
//               order create_graph_branch's add_edge calls append them in;
//   hallways / branches   connected components (pointer jumping over the contracted tree's parent
//               links), numbered by their first node in node order as nx.connected_components
//               yields them; the junctions a hallway takes follow the reference's loop and its
//               break (:210-214) per node; each hallway lies in exactly one branch;
//   sums        every hallway's edge terms in the order networkx 3.4's subgraph view reports them
//               (G.subgraph(all_nodes), :217-218, read by get_edge_attributes :283-295): the
//               view iterates show_nodes' CPython set when it holds fewer than half of G's nodes
//               (FilterAdjacency), so one wave per hallway rebuilds the sets the reference builds
//               — _plain_bfs's `seen` (BFS in the adjacency order of G.copy()), set(component),
//               adjacent_split_points, the union, show_nodes' set — as CPython 3.10 set tables
//               held in the wave's registers (WSet: one slot per lane and register, <= 128
//               slots), then walks the final table and sums in that order; the branch sums and
//               the final product follow the reference's order.
// Toroidal handles are scored as the reference scores them: the bordered (N + 2)^2 maze, the
// crop inside a wall ring with start / goal shifted by +1 (gen_maze_no_border, maze_generation.
// py:49-51; off_policy_trainer.py:194-196) — a perfect maze whose distance field to the goal comes
// from a bit-parallel BFS over 128-bit rows held in one wave's registers here (the handle's cell
// words hold torus distances).
// Output per maze: the product and the sum before the log (prod_b (C_b + 1) * C_0 and
// sum_b C_b + C_0); the caller takes math.log (glibc, as the reference) of both. Non-tree mazes
// and mazes beyond the LDS / register budgets report a status and are left to the host
// restatement (csrc/mz_difficulty.hip, the same orders).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "mz_common.h"
#include "mz_mcclendon.h"

namespace {

#ifndef MZ_MC_T
#define MZ_MC_T 1024  // 16 waves: hallways in flight per CU (256: 28 -> 12 ms per 6,000 81x81 mazes)
#endif
constexpr int T = MZ_MC_T;  // threads per maze workgroup
// MZ_MC_PROBE = k (timing experiments only, wrong results): the kernel returns after phase k
// (1 A squares, 2 B solution path, 3 C dead ends / first(), 4 D node order, 5 E edges,
// 6 F components, 7 G hallway sums; 71 / 72 after G's member lists / classification, 73 / 74
// the whole kernel without G's lane path / wave queue)
#ifndef MZ_MC_PROBE
#define MZ_MC_PROBE 0
#endif
#define MC_PROBE_AT(k)                                                            \
  if (MZ_MC_PROBE == (k)) {                                                       \
    if (threadIdx.x == 0) { out[2 * i] = out[2 * i + 1] = 0.0; status[i] = 0; }   \
    return;                                                                       \
  }
constexpr int WAVE = 64;
constexpr uint16_t NONE = 0xFFFF;
constexpr uint8_t F_OPEN = 1, F_POINT = 2, F_SOL = 4, F_JUNC = 8, F_DEAD = 16;
constexpr uint8_t N_SOL = 8, N_JUNC = 16;  // node flags: deg in bits 0-2

__device__ inline int next_pow2(int x) {
  int p = 1;
  while (p < x) p <<= 1;
  return p;
}

// ascending bitonic sort of a[0, S) (S a power of two), whole workgroup
__device__ void bitonic(uint64_t* a, int S) {
  for (int k = 2; k <= S; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < S; i += T) {
        const int l = i ^ j;
        if (l > i) {
          const bool up = (i & k) == 0;
          const uint64_t x = a[i], y = a[l];
          if ((x > y) == up) {
            a[i] = y;
            a[l] = x;
          }
        }
      }
      __syncthreads();
    }
}

__device__ inline uint64_t shfl_xor64(uint64_t v, int m) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m);
  const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m);
  return ((uint64_t)hi << 32) | lo;
}
// bitonic stages j = jmax .. 1 of merge size k on a wave's 128-element block [b, b + 128), held as
// x0 = element b + lane, x1 = element b + 64 + lane: j = 64 within the lane, j < 64 by shuffles
__device__ inline void bitonic_regs(uint64_t& x0, uint64_t& x1, int b, int k, int jmax) {
  const int lane = threadIdx.x & (WAVE - 1);
  for (int j = jmax; j > 0; j >>= 1) {
    if (j == 64) {
      const bool up = ((b + lane) & k) == 0;
      const uint64_t lo = x0 < x1 ? x0 : x1, hi = x0 < x1 ? x1 : x0;
      x0 = up ? lo : hi;
      x1 = up ? hi : lo;
      continue;
    }
    const uint64_t p0 = shfl_xor64(x0, j), p1 = shfl_xor64(x1, j);
    const int i0 = b + lane, i1 = b + 64 + lane;
    const bool u0 = ((i0 & k) == 0) == ((i0 & j) == 0), u1 = ((i1 & k) == 0) == ((i1 & j) == 0);
    x0 = u0 ? (x0 < p0 ? x0 : p0) : (x0 < p0 ? p0 : x0);
    x1 = u1 ? (x1 < p1 ? x1 : p1) : (x1 < p1 ? p1 : x1);
  }
}
// the same sort for 256 <= S <= 2 T with far fewer barriers: every stage whose pairs lie inside a
// 128-element block runs in the wave's registers (shuffles), only the j >= 128 stages go through
// LDS — ~15 workgroup barriers for S = 2,048 instead of 66
__device__ void bitonic_waves(uint64_t* a, int S) {
  const int lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE, b = w * 128;
  const bool act = b < S;
  uint64_t x0 = 0, x1 = 0;
  if (act) {
    x0 = a[b + lane];
    x1 = a[b + 64 + lane];
    for (int k = 2; k <= 128; k <<= 1) bitonic_regs(x0, x1, b, k, k >> 1);
    a[b + lane] = x0;
    a[b + 64 + lane] = x1;
  }
  __syncthreads();
  for (int k = 256; k <= S; k <<= 1) {
    for (int j = k >> 1; j >= 128; j >>= 1) {
      for (int p = threadIdx.x; p < S / 2; p += T) {  // pair p: i has bit j clear, l = i + j
        const int i = (p / j) * 2 * j + (p % j), l = i + j;
        const bool up = (i & k) == 0;
        const uint64_t x = a[i], y = a[l];
        if ((x > y) == up) {
          a[i] = y;
          a[l] = x;
        }
      }
      __syncthreads();
    }
    if (act) {
      x0 = a[b + lane];
      x1 = a[b + 64 + lane];
      bitonic_regs(x0, x1, b, k, 64);
      a[b + lane] = x0;
      a[b + 64 + lane] = x1;
    }
    __syncthreads();
  }
}
__device__ inline void sort_keys(uint64_t* a, int S) {
  if (S >= 256 && S <= 2 * T) bitonic_waves(a, S);
  else bitonic(a, S);
}

// exclusive prefix sum of v over the workgroup (one value per thread); *total = the sum
__device__ inline int block_excl(int v, int* wsum, int* total) {
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
  for (int k = 0; k < T / WAVE; ++k) {
    if (k < wid) before += wsum[k];
    tot += wsum[k];
  }
  *total = tot;
  return before + x - v;
}

__device__ inline int dir_dr(int k) { return k == 0 ? -1 : (k == 1 ? 1 : 0); }
__device__ inline int dir_dc(int k) { return k == 2 ? -1 : (k == 3 ? 1 : 0); }

// ---- CPython 3.10 set table for int keys (hash(n) == n), held by one wave -------------------
// Objects/setobject.c: probe i = hash & mask, then the 9 following slots when i + 9 <= mask, then
// perturb >>= 5, i = (5 i + 1 + perturb) & mask; add() inserts at the first empty slot and resizes
// to used * 4 when fill * 5 >= mask * 3; a resize re-inserts in old table order (insert_clean);
// set(s) / s.union(t) / s.update(t) merge (set_merge); no deletions, so no dummies (oracle/
// pyset.py restates the same and is checked against the interpreter). Slot j lives in lane j & 63
// of v0 (j < 64) or v1; a slot holds key << 16 | node; occupancy is a wave-uniform 128-bit mask.
constexpr uint32_t WS_EMPTY = 0xFFFFFFFFu;
struct WSet {
  uint32_t v0, v1;
  uint64_t o0, o1;
  int mask, fill, used;
  bool small;  // still the 8-slot smalltable
};
// The occupancy words and counters are wave-uniform: readfirstlane keeps them in SGPRs (scalar
// branches over the probe sequence), and every update below is a value select — a field chosen
// by a branch (`j < 64 ? o0 : o1` as an lvalue) made the compiler address the struct in scratch.
__device__ inline uint64_t ws_uni64(uint64_t x) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
  return ((uint64_t)hi << 32) | lo;
}
__device__ inline void ws_init(WSet& s) {
  s.v0 = s.v1 = WS_EMPTY;
  s.o0 = s.o1 = 0;
  s.mask = 7;
  s.fill = s.used = 0;
  s.small = true;
}
// the first empty slot of key's probe sequence (the key is known to be absent)
__device__ inline int ws_free_slot(const WSet& s, uint32_t key) {
  const uint64_t o0 = ws_uni64(s.o0), o1 = ws_uni64(s.o1);
  const uint32_t mask = (uint32_t)__builtin_amdgcn_readfirstlane(s.mask);
  uint32_t perturb = key;
  int i = (int)(key & mask);
  for (;;) {
    const int last = i + 9 <= (int)mask ? i + 9 : i;
    for (int j = i; j <= last; ++j)
      if (!(((j < 64 ? o0 : o1) >> (j & 63)) & 1ull)) return j;
    perturb >>= 5;
    i = (int)(((uint32_t)i * 5u + 1u + perturb) & mask);
  }
}
__device__ inline void ws_put(WSet& s, int j, uint32_t val) {
  const int lane = threadIdx.x & (WAVE - 1);
  const bool hi = j >= 64;
  const uint64_t b = 1ull << (j & 63);
  const bool mine = lane == (j & 63);
  s.v0 = (mine && !hi) ? val : s.v0;
  s.v1 = (mine && hi) ? val : s.v1;
  s.o0 = ws_uni64(s.o0 | (hi ? 0ull : b));
  s.o1 = ws_uni64(s.o1 | (hi ? b : 0ull));
}
__device__ inline uint32_t ws_get(const WSet& s, int j) {
  const int v = __shfl((int)(j < 64 ? s.v0 : s.v1), j & 63);
  return (uint32_t)v;
}
// next occupied slot after j (table order), -1 at the end
__device__ inline int ws_next(const WSet& s, int j) {
  ++j;
  if (j < 64) {
    const uint64_t m = j ? s.o0 & ~((1ull << j) - 1) : s.o0;
    if (m) return __ffsll((long long)m) - 1;
    j = 64;
  }
  if (j < 128) {
    const int b = j - 64;
    const uint64_t m = b ? s.o1 & ~((1ull << b) - 1) : s.o1;
    if (m) return 64 + __ffsll((long long)m) - 1;
  }
  return -1;
}
// slot of key, -1 if absent
__device__ inline int ws_find(const WSet& s, uint32_t key) {
  const uint64_t m0 = __ballot((s.v0 >> 16) == key), m1 = __ballot((s.v1 >> 16) == key);
  if (m0) return __ffsll((long long)m0) - 1;
  if (m1) return 64 + __ffsll((long long)m1) - 1;
  return -1;
}
// set_table_resize; false beyond the wave's 128 slots
__device__ inline bool ws_resize(WSet& s, int minused) {
  int ns = 8;
  while (ns <= minused) ns <<= 1;
  if (ns == 8 && s.small) return true;
  if (ns > 128) return false;
  WSet n;
  ws_init(n);
  n.mask = ns - 1;
  n.small = ns == 8;
  for (int j = ws_next(s, -1); j >= 0; j = ws_next(s, j)) {
    const uint32_t v = ws_get(s, j);
    ws_put(n, ws_free_slot(n, v >> 16), v);
  }
  n.fill = n.used = s.used;
  s = n;
  return true;
}
// set_add_entry: 1 added, 0 present, -1 beyond the budget
__device__ inline int ws_add(WSet& s, uint32_t key, uint32_t node) {
  if (ws_find(s, key) >= 0) return 0;
  ws_put(s, ws_free_slot(s, key), (key << 16) | node);
  s.fill += 1;
  s.used += 1;
  if (s.fill * 5 >= s.mask * 3 && !ws_resize(s, s.used > 50000 ? s.used * 2 : s.used * 4)) return -1;
  return 1;
}
// dst = set(src) (set_merge into an empty set)
__device__ inline bool ws_copy(WSet& dst, const WSet& src) {
  ws_init(dst);
  if (src.used == 0) return true;
  if (src.used * 5 >= dst.mask * 3 && !ws_resize(dst, src.used * 2)) return false;
  if (dst.mask == src.mask) {
    dst = src;
    return true;
  }
  for (int j = ws_next(src, -1); j >= 0; j = ws_next(src, j)) {
    const uint32_t v = ws_get(src, j);
    ws_put(dst, ws_free_slot(dst, v >> 16), v);
  }
  dst.fill = dst.used = src.used;
  return true;
}
// dst.update(src) for a non-empty dst (set_merge: one resize first, then set_add_entry)
__device__ inline bool ws_merge(WSet& dst, const WSet& src) {
  if (src.used == 0) return true;
  if ((dst.fill + src.used) * 5 >= dst.mask * 3 && !ws_resize(dst, (dst.used + src.used) * 2))
    return false;
  for (int j = ws_next(src, -1); j >= 0; j = ws_next(src, j)) {
    const uint32_t v = ws_get(src, j);
    if (ws_add(dst, v >> 16, v & 0xFFFFu) < 0) return false;
  }
  return true;
}

// ---- the same CPython 3.10 set table for ONE lane (a hallway per lane, phase G) --------------
// Tables of <= 32 slots hold node ids (u16) in LDS — the key (cantor pairing of the node's square,
// its own hash) is a bijection of the node, so a slot match by node is a match by key; occupancy
// is a 32-bit mask in a register. The operations mirror ws_* above (and CPython's set_add_entry /
// set_insert_clean / set_table_resize / set_merge) step for step; a table that would grow past 32
// slots makes the caller hand the hallway to the wave path.
struct LSet {
  uint16_t* t;  // 32 slots, slot j at t[j * st] (the lanes' tables interleave: conflict-free LDS)
  int st;
  uint32_t occ;
  int mask, fill, used;
  bool small;
};
__device__ inline void ls_init(LSet& s, uint16_t* buf, int st) {
  s.t = buf;
  s.st = st;
  s.occ = 0u;
  s.mask = 7;
  s.fill = s.used = 0;
  s.small = true;
}
// slot of `node` (key `key`) if present (*found), else the first empty slot of key's probe sequence
__device__ inline int ls_probe(const LSet& s, uint32_t key, int node, bool* found) {
  uint32_t perturb = key;
  int i = (int)(key & (uint32_t)s.mask);
  for (;;) {
    const int last = i + 9 <= s.mask ? i + 9 : i;
    for (int j = i; j <= last; ++j) {
      if (!((s.occ >> j) & 1u)) { *found = false; return j; }
      if (s.t[j * s.st] == (uint16_t)node) { *found = true; return j; }
    }
    perturb >>= 5;
    i = (int)(((uint32_t)i * 5u + 1u + perturb) & (uint32_t)s.mask);
  }
}
__device__ inline int ls_find(const LSet& s, uint32_t key, int node) {
  bool f;
  const int j = ls_probe(s, key, node, &f);
  return f ? j : -1;
}
template <class KEY>
__device__ inline bool ls_resize(LSet& s, int minused, uint16_t* tmp, const KEY& key_of) {
  int ns = 8;
  while (ns <= minused) ns <<= 1;
  if (ns == 8 && s.small) return true;
  if (ns > 32) return false;
  int n = 0;
  for (int j = 0; j <= s.mask; ++j)
    if ((s.occ >> j) & 1u) tmp[n++ * s.st] = s.t[j * s.st];
  s.occ = 0u;
  s.mask = ns - 1;
  s.small = ns == 8;
  for (int k = 0; k < n; ++k) {  // insert_clean in the old table's order
    bool f;
    const int node = tmp[k * s.st];
    const int j = ls_probe(s, key_of(node), node, &f);
    s.t[j * s.st] = (uint16_t)node;
    s.occ |= 1u << j;
  }
  s.fill = s.used = n;
  return true;
}
template <class KEY>
__device__ inline int ls_add_k(LSet& s, int node, uint32_t key, uint16_t* tmp, const KEY& key_of) {
  bool f;
  const int j = ls_probe(s, key, node, &f);
  if (f) return 0;
  s.t[j * s.st] = (uint16_t)node;
  s.occ |= 1u << j;
  s.fill += 1;
  s.used += 1;
  if (s.fill * 5 >= s.mask * 3 && !ls_resize(s, s.used > 50000 ? s.used * 2 : s.used * 4, tmp, key_of))
    return -1;
  return 1;
}
template <class KEY>
__device__ inline int ls_add(LSet& s, int node, uint16_t* tmp, const KEY& key_of) {
  return ls_add_k(s, node, key_of(node), tmp, key_of);
}
// dst = set(src) (set_merge into an empty set; dst's buffer distinct from src's)
template <class KEY>
__device__ inline bool ls_copy(LSet& dst, uint16_t* dbuf, const LSet& src, uint16_t* tmp,
                               const KEY& key_of) {
  ls_init(dst, dbuf, src.st);
  if (src.used == 0) return true;
  if (src.used * 5 >= dst.mask * 3 && !ls_resize(dst, src.used * 2, tmp, key_of)) return false;
  if (dst.mask == src.mask) {
    for (int j = 0; j <= src.mask; ++j) dst.t[j * dst.st] = src.t[j * src.st];
    dst.occ = src.occ;
    dst.small = src.small;
  } else {
    for (int j = 0; j <= src.mask; ++j) {
      if (!((src.occ >> j) & 1u)) continue;
      bool f;
      const int node = src.t[j * src.st];
      const int k = ls_probe(dst, key_of(node), node, &f);
      dst.t[k * dst.st] = (uint16_t)node;
      dst.occ |= 1u << k;
    }
  }
  dst.fill = dst.used = src.used;
  return true;
}
// dst.update(src) for a non-empty dst
template <class KEY>
__device__ inline bool ls_merge(LSet& dst, const LSet& src, uint16_t* tmp, const KEY& key_of) {
  if (src.used == 0) return true;
  if ((dst.fill + src.used) * 5 >= dst.mask * 3 && !ls_resize(dst, (dst.used + src.used) * 2, tmp, key_of))
    return false;
  for (int j = 0; j <= src.mask; ++j)
    if ((src.occ >> j) & 1u)
      if (ls_add(dst, src.t[j * src.st], tmp, key_of) < 0) return false;
  return true;
}


// ---- the lane path's sets from their occupancy masks alone (MZ_MC_LANE2) ---------------------
// In a tree every insertion of the lane path is of a key not yet in its set (a BFS visits a node
// once; a junction neighbours one member of a hallway; members and junctions are disjoint), so
// CPython's set_add_entry / set_insert_clean put it in the first empty slot of its probe
// sequence — a function of the occupancy mask and the key only, computed in registers. An entry
// is one word: slot << 25 | key << 11 | node (keys < 2^14 and nodes < 2^11 up to pitch 91, the
// kernel's LDS limit); a set's iteration order comes from its slots' ranks in the mask
// (popcount below the slot), by a scatter through LDS.
#ifndef MZ_MC_LANE2
#define MZ_MC_LANE2 1
#endif
__device__ inline uint32_t lw_key(uint32_t w) { return (w >> 11) & 0x3FFFu; }
__device__ inline int lw_node(uint32_t w) { return (int)(w & 0x7FFu); }
__device__ inline int lw_slot(uint32_t w) { return (int)(w >> 25); }
__device__ inline uint32_t lw_with_slot(uint32_t w, int sl) { return (w & 0x1FFFFFFu) | ((uint32_t)sl << 25); }
__device__ inline int lw_free(uint32_t occ, uint32_t key, int mask) {
  uint32_t perturb = key;
  int i = (int)(key & (uint32_t)mask);
  for (;;) {
    if (i + 9 <= mask) {
      const uint32_t fr = (~occ >> i) & 0x3FFu;
      if (fr) return i + __builtin_ctz(fr);
    } else if (!((occ >> i) & 1u)) {
      return i;
    }
    perturb >>= 5;
    i = (int)(((uint32_t)i * 5u + 1u + perturb) & (uint32_t)mask);
  }
}
// insert_clean / add of a key known to be absent: its slot into the word, the mask updated
__device__ inline void lw_put(uint32_t& w, uint32_t& occ, int mask) {
  const int t = lw_free(occ, lw_key(w), mask);
  occ |= 1u << t;
  w = lw_with_slot(w, t);
}
// a set built by add() from p[0..n) (n <= 15; distinct keys): slots into the words, occupancy,
// mask. set_add_entry resizes after the insertion that makes fill * 5 >= mask * 3: the 5th of an
// 8-slot table (to 32 = the smallest power of two above 4 * 5, re-inserting in slot order); a
// 32-slot table would resize at the 19th
__device__ inline void lw_layout_add(uint32_t (&p)[16], int n, uint32_t& occ, int& mask) {
  occ = 0u;
  mask = 7;
#pragma unroll
  for (int i = 0; i < 5; ++i)
    if (i < n) lw_put(p[i], occ, 7);
  if (n < 5) return;
  int rk[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) rk[i] = __popc(occ & ((1u << lw_slot(p[i])) - 1u));
  uint32_t o2 = 0u;
#pragma unroll
  for (int r = 0; r < 5; ++r) {
    uint32_t kr = 0u;
#pragma unroll
    for (int i = 0; i < 5; ++i) kr = rk[i] == r ? lw_key(p[i]) : kr;
    const int t = lw_free(o2, kr, 31);
    o2 |= 1u << t;
#pragma unroll
    for (int i = 0; i < 5; ++i) p[i] = rk[i] == r ? lw_with_slot(p[i], t) : p[i];
  }
#pragma unroll
  for (int i = 5; i < 16; ++i)
    if (i < n) lw_put(p[i], o2, 31);
  occ = o2;
  mask = 31;
}
// set_table_resize's size for minused: the smallest power of two above it, at least 8; -1 = mask
__device__ inline int lw_mask_for(int minused) {
  int ns = 8;
  while (ns <= minused) ns <<= 1;
  return ns - 1;
}

typedef unsigned __int128 u128;

// phase G: waves that run the lane path (the rest start on the wave queue)
#ifndef MZ_MC_LANE_WAVES
#define MZ_MC_LANE_WAVES 12
#endif
constexpr int MC_LANE_WAVES = MZ_MC_LANE_WAVES;

// one candidate (index i of the list) per call: the body of a one-candidate-per-workgroup kernel,
// every early return is workgroup-uniform
__device__ __forceinline__ void mc_score(int i, MzDev d, const int32_t* ids, int n, int MM, int MK,
                                         double* out, int32_t* status) {
  extern __shared__ __align__(16) unsigned char lds[];
  __shared__ int wsum[T / WAVE];
  __shared__ int s_bad, s_nsol, s_noff, s_open, s_edges, s_Hn, s_Bn, s_nl, s_nw, s_wq;
#if MZ_MC_PROBE == 80
  // timing probe: the lane path's passes summed over the lane waves, the waves' G2 durations
  __shared__ unsigned long long s_pt[8];
  __shared__ unsigned int s_tmax[2];
#endif
  const int e = ids ? ids[i] : i;
  auto fail = [&](int code) {
    if (threadIdx.x == 0) { out[2 * i] = out[2 * i + 1] = 0.0; status[i] = code; }
  };
  if (e < 0 || e >= d.B) { fail(3); return; }
  const bool tor = d.toroidal;
  const int P = d.P, Pb = tor ? P + 2 : P, NNP = Pb * Pb;
  const uint32_t m0 = d.meta0[e], m1 = d.meta1[e];
  // the evaluated grid: the maze itself, or a toroidal crop inside its wall ring (+1 shift)
  const int Nm = m0 & 0xFF, N = tor ? Nm + 2 : Nm, o = tor ? 1 : 0;
  const int sr = ((m0 >> 16) & 0xFF) + o, sc = (m0 >> 24) + o;
  const int gr = (m1 & 0xFF) + o, gc = ((m1 >> 8) & 0xFF) + o;
  const int NN = N * N, start = sr * N + sc, goal = gr * N + gc;
  const uint32_t* cw = d.cells + (size_t)e * P * P;
  auto cell = [&](int q) -> uint32_t { const int r = q / N; return cw[r * P + (q - r * N)]; };
  auto sq_open = [&](int q) -> bool {
    if (!tor) return (cell(q) & MZ_CELL_OPEN) != 0;
    const int r = q / N, c = q - r * N;
    return r >= 1 && r <= Nm && c >= 1 && c <= Nm && (cw[(r - 1) * P + (c - 1)] & MZ_CELL_OPEN);
  };

  // ---- LDS: square region (phase 1) aliased by the node-phase arrays (phase 2) ---------------
  uint16_t* gp = reinterpret_cast<uint16_t*>(lds);                 // [NNP] parent toward the goal
  uint16_t* pos = gp + NNP;                                          // [NNP] node position
  uint32_t* fst = reinterpret_cast<uint32_t*>(pos + NNP);          // [NNP] first dead-end rank
  uint8_t* fl = reinterpret_cast<uint8_t*>(fst + NNP);              // [NNP] flags
  // toroidal: the bordered grid's distance field to the goal
  const size_t tor_off = ((size_t)NNP * 9 + 16 + 15) & ~(size_t)15;
  uint16_t* tdist = reinterpret_cast<uint16_t*>(lds + tor_off);     // [NNP]
  const size_t sq_bytes = tor ? tor_off + (((size_t)NNP * 2 + 15) & ~(size_t)15) : tor_off,
               ph2_bytes = (size_t)MM * 36;
  unsigned char* nb = lds + (sq_bytes > ph2_bytes ? sq_bytes : ph2_bytes);  // node region
  uint64_t* keys = reinterpret_cast<uint64_t*>(nb);                  // [MK] sort buffer
  uint16_t* nsq = reinterpret_cast<uint16_t*>(keys + MK);            // [MM] node -> square
  uint16_t* adjp = nsq + MM;                                         // [MM][4] neighbours (pos)
  uint16_t* adjd = adjp + 4 * MM;                                    // [MM][4] edge d
  uint16_t* gpar = adjd + 4 * MM;                                    // [MM] parent node (pos)
  uint16_t* gpd = gpar + MM;                                         // [MM] d to the parent
  uint16_t* nfs = gpd + MM;                                          // [MM] first(x)
  uint8_t* adjn = reinterpret_cast<uint8_t*>(nfs + MM);              // [MM]
  uint8_t* nfl = adjn + MM;                                          // [MM] deg | N_SOL | N_JUNC
  // phase 2 over the square region
  uint16_t* hr = reinterpret_cast<uint16_t*>(lds);                   // [MM] hallway root
  uint16_t* br = hr + MM;                                            // [MM] branch root
  uint16_t* hid = br + MM;                                           // [MM] hallway id (1..)
  uint16_t* bid = hid + MM;                                          // [MM] branch rank
  uint16_t* pref = bid + MM;                                         // [MM] rank scratch
  uint16_t* hroot = pref + MM;                                       // [MM] hallway id -> root
  uint32_t* hmin = reinterpret_cast<uint32_t*>(hroot + MM);          // [MM]
  uint32_t* bmin = hmin + MM;                                        // [MM]
  double* Ch = reinterpret_cast<double*>(bmin + MM);                 // [MM] hallway complexity
  double* Cb = Ch + MM;                                              // [MM] branch complexity

  if (threadIdx.x == 0) {
    s_bad = 0; s_nsol = 0; s_noff = 0; s_open = 0; s_edges = 0; s_Hn = 0; s_Bn = 0;
  }
  if (N < 3 || N > Pb || start == goal) { fail(3); return; }
  if (tor && N > 128) { fail(2); return; }  // the BFS rows are 128-bit
  // ---- A. squares: open, parent toward the goal, points, junctions -------------------------
  for (int q = threadIdx.x; q < NN; q += T) {
    gp[q] = NONE;
    pos[q] = NONE;
    fst[q] = 0xFFFFFFFFu;
    fl[q] = sq_open(q) ? F_OPEN : 0;
  }
  if (tor) {
    // distances to the goal on the bordered grid: BFS over 128-bit rows (a level = shift / or /
    // and-not of the frontier rows), no wrap (the ring is wall), by ONE wave with the rows in
    // registers — lane l holds rows l and 64 + l, the neighbour rows come by lane shuffles — so a
    // level costs no barrier (a dfs maze has ~3,000 levels; a workgroup barrier per level made
    // this BFS the kernel's longest phase)
    for (int q = threadIdx.x; q < NN; q += T) tdist[q] = 0xFFFF;
    __syncthreads();
    if (threadIdx.x < WAVE) {
      const int lane = threadIdx.x;
      auto row_open = [&](int y) -> u128 {
        u128 ob = 0;
        if (y < N)
          for (int x = 0; x < N; ++x)
            if (sq_open(y * N + x)) ob |= (u128)1 << x;
        return ob;
      };
      const u128 O0 = row_open(lane), O1 = row_open(64 + lane);
      u128 F0 = lane == gr ? (u128)1 << gc : (u128)0;
      u128 F1 = 64 + lane == gr ? (u128)1 << gc : (u128)0;
      u128 V0 = F0, V1 = F1;
      if (lane == 0) tdist[goal] = 0;
      auto shfl128 = [&](u128 v, int src) -> u128 {
        u128 r = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k)
          r |= (u128)(uint32_t)__shfl((int)(uint32_t)(v >> (32 * k)), src) << (32 * k);
        return r;
      };
      auto mark = [&](u128 nw, int y, int level) {
        while (nw) {
          const uint64_t lo = (uint64_t)nw, hi = (uint64_t)(nw >> 64);
          const int x = lo ? __ffsll((long long)lo) - 1 : 64 + __ffsll((long long)hi) - 1;
          tdist[y * N + x] = (uint16_t)level;
          nw &= nw - 1;
        }
      };
      for (int level = 1;; ++level) {
        // row y - 1 of row lane: lane - 1's row 0 part (lane 0: none); of row 64 + lane: lane - 1's
        // row 1 part (lane 0: lane 63's row 0 part). Row y + 1 of row lane: lane + 1's row 0 part
        // (lane 63: lane 0's row 1 part); of row 64 + lane: lane + 1's row 1 part (lane 63: none)
        const u128 a0 = shfl128(F0, (lane + WAVE - 1) & (WAVE - 1));
        const u128 a1 = shfl128(F1, (lane + WAVE - 1) & (WAVE - 1));
        const u128 b0 = shfl128(F0, (lane + 1) & (WAVE - 1));
        const u128 b1 = shfl128(F1, (lane + 1) & (WAVE - 1));
        const u128 up0 = lane == 0 ? (u128)0 : a0;
        const u128 up1 = lane == 0 ? a0 : a1;  // lane 0: row 63 = lane 63's row 0 part
        const u128 dn0 = lane == WAVE - 1 ? b1 : b0;  // lane 63: row 64 = lane 0's row 1 part
        const u128 dn1 = lane == WAVE - 1 ? (u128)0 : b1;
        const u128 n0 = (F0 | (F0 << 1) | (F0 >> 1) | up0 | dn0) & O0 & ~V0;
        const u128 n1 = (F1 | (F1 << 1) | (F1 >> 1) | up1 | dn1) & O1 & ~V1;
        V0 |= n0;
        V1 |= n1;
        F0 = n0;
        F1 = n1;
        mark(n0, lane, level);
        mark(n1, 64 + lane, level);
        if (!__any((n0 | n1) != 0)) break;
      }
    }
  }
  auto sq_dist = [&](int q) -> int {  // BFS distance to the goal (MZ_CELL_D_MASK: unreachable)
    if (!tor) return (int)(cell(q) & MZ_CELL_D_MASK);
    const int v = tdist[q];
    return v < (int)MZ_CELL_D_MASK ? v : (int)MZ_CELL_D_MASK;
  };
  __syncthreads();
  {
    int n_open = 0, n_edges = 0, bad = 0;
    for (int q = threadIdx.x; q < NN; q += T) {
      if (!(fl[q] & F_OPEN)) continue;
      const int r = q / N, c = q - r * N;
      const int D = sq_dist(q);
      if (D >= (int)MZ_CELL_D_MASK) bad = 1;  // unreachable from the goal
      // open squares on the border (the host restatement's neighbour count reads past the grid)
      if (r == 0 || c == 0 || r == N - 1 || c == N - 1) bad |= 2;
      bool nbo[4];
      int deg = 0;
      for (int k = 0; k < 4; ++k) {
        const int rr = r + dir_dr(k), cc = c + dir_dc(k);
        nbo[k] = rr >= 0 && rr < N && cc >= 0 && cc < N && (fl[rr * N + cc] & F_OPEN);
        if (nbo[k]) {
          ++deg;
          if (D > 0 && sq_dist(rr * N + cc) == D - 1) gp[q] = (uint16_t)(rr * N + cc);
        }
      }
      n_open += 1;
      n_edges += (nbo[1] ? 1 : 0) + (nbo[3] ? 1 : 0);  // down, right: each edge once
      const bool corner = deg == 2 && !(nbo[0] && nbo[1]) && !(nbo[2] && nbo[3]);
      uint8_t f = F_OPEN;
      if (deg != 2 || corner || q == start || q == goal) f |= F_POINT;
      if (deg == 3) f |= F_JUNC;
      // a straight goal square inside a corridor is a point of the solution only: the paths from
      // the dead ends beyond it skip it (decompose_in_turns), which the contraction here does not
      if (q == goal && deg == 2 && !corner) bad |= 2;
      fl[q] = f;
    }
    if (bad) atomicOr(&s_bad, bad);
    atomicAdd(&s_open, n_open);
    atomicAdd(&s_edges, n_edges);
  }
  __syncthreads();
  if ((s_bad & 1) || s_edges != s_open - 1 || !(fl[start] & F_OPEN) || !(fl[goal] & F_OPEN)) {
    fail(1);  // not a tree: the host restatement's A* path
    return;
  }
  if (s_bad) { fail(2); return; }
  MC_PROBE_AT(1)
  // ---- B. the solution path (start -> goal along the goal-rooted parents), its points first --
  // The path is start's chain of goal-ward parents — thousands of squares in a dfs maze, a serial
  // pointer chase. Instead: 32-step jump pointers by 5 doubling rounds over every square (in fst,
  // free until phase C, as two u16 arrays), lane 0 walks the milestones start, gp^32(start), ...
  // (<= NN / 32 of them), then one thread per 32-square segment marks its squares and counts its
  // points, a scan gives each segment its first position, and a second walk writes the positions
  // (the same order as the serial walk: segment by segment along the path).
  {
    uint16_t* jc = reinterpret_cast<uint16_t*>(fst);
    uint16_t* jn = jc + NNP;
    for (int q = threadIdx.x; q < NN; q += T) jc[q] = gp[q];
    __syncthreads();
    for (int r = 0; r < 5; ++r) {
      for (int q = threadIdx.x; q < NN; q += T) {
        const int a = jc[q];
        jn[q] = a == NONE ? NONE : jc[a];
      }
      __syncthreads();
      uint16_t* t = jc; jc = jn; jn = t;
    }
    uint16_t* mil = reinterpret_cast<uint16_t*>(keys);  // the node region is free until phase D
    if (threadIdx.x == 0) {
      int x = start, k = 0;
      mil[k++] = (uint16_t)x;
      while (jc[x] != NONE && k < NN) {
        x = jc[x];
        mil[k++] = (uint16_t)x;
      }
      s_noff = k;  // (s_noff is the phase-D counter: reset below)
      s_open = 0;  // (read by phase A's checks only: the plain-point count from here)
    }
    __syncthreads();
    const int K = s_noff;
    int cnt = 0, plain = 0;
    const bool seg = threadIdx.x < K;
    if (seg) {
      int x = mil[threadIdx.x];
      for (int j = 0; j < 32; ++j) {
        fl[x] |= F_SOL;
        if (fl[x] & F_POINT) {
          ++cnt;
          plain += (fl[x] & F_JUNC) ? 0 : 1;
        }
        if (x == goal) break;
        x = gp[x];
        if (x == NONE) { s_bad = 1; break; }
      }
    }
    if (plain) atomicAdd(&s_open, plain);  // (s_open is free after phase A: the plain-point count)
    int tot;
    const int base = block_excl(seg ? cnt : 0, wsum, &tot);
    if (seg) {
      int x = mil[threadIdx.x], k = base;
      for (int j = 0; j < 32; ++j) {
        if (fl[x] & F_POINT) {
          if (k < MM) nsq[k] = (uint16_t)x;
          pos[x] = (uint16_t)k++;
        }
        if (x == goal) break;
        x = gp[x];
        if (x == NONE) break;
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      s_nsol = tot;
      // every solution point a junction: the solution hallway would lie inside a branch (the
      // reference then counts it twice) — left to the host restatement
      if (tot > MM || s_open == 0) s_bad = s_bad ? s_bad : 2;
      s_noff = 0;
    }
    // fst back to its phase-C initial value
    for (int q = threadIdx.x; q < NN; q += T) fst[q] = 0xFFFFFFFFu;
  }
  __syncthreads();
  if (s_bad) { fail(2); return; }
  MC_PROBE_AT(2)
  // ---- C. dead ends (value 1, one open neighbour, off the solution), row-major ranks --------
  {
    int carry = 0;
    for (int q0 = 0; q0 < NN; q0 += T) {
      const int q = q0 + threadIdx.x;
      int de = 0;
      if (q < NN && (fl[q] & F_OPEN) && !(fl[q] & F_SOL) && q != goal) {
        const int r = q / N, c = q - r * N;
        int deg = 0;
        for (int k = 0; k < 4; ++k) {
          const int rr = r + dir_dr(k), cc = c + dir_dc(k);
          deg += (rr >= 0 && rr < N && cc >= 0 && cc < N && (fl[rr * N + cc] & F_OPEN)) ? 1 : 0;
        }
        de = deg == 1;
      }
      int tot;
      const int rank = carry + block_excl(de, wsum, &tot);
      if (de) {
        fl[q] |= F_DEAD;
        fst[q] = (uint32_t)rank;
      }
      carry += tot;
      __syncthreads();
    }
  }
  __syncthreads();
  // first(x): every dead end walks toward the solution, lowering first() until a square already
  // holds a smaller rank (the walk that set it carries that rank on up)
  for (int q = threadIdx.x; q < NN; q += T) {
    if (!(fl[q] & F_DEAD)) continue;
    const uint32_t r = fst[q];
    int y = gp[q];
    while (y != NONE && !(fl[y] & F_SOL)) {
      if (atomicMin(&fst[y], r) <= r) break;
      y = gp[y];
    }
  }
  __syncthreads();
  MC_PROBE_AT(3)
  // ---- D. node order: solution points, then (first(x), -D(x)) ---------------------------------
  for (int q = threadIdx.x; q < NN; q += T) {
    if ((fl[q] & F_POINT) && !(fl[q] & F_SOL)) {
      const int k = atomicAdd(&s_noff, 1);
      const uint32_t D = (uint32_t)sq_dist(q);
      if (fst[q] > 0x3FFFu) s_bad = 2;  // no dead end below it
      if (k < MM)
        keys[k] = ((uint64_t)(fst[q] & 0x3FFFu) << 28) | ((uint64_t)(8191u - D) << 15) | (uint64_t)q;
    }
  }
  __syncthreads();
  const int nsol = s_nsol, noff = s_noff, M = nsol + noff;
  if (M > MM || s_bad) { fail(2); return; }
  const int S1 = next_pow2(noff > 1 ? noff : 2);
  for (int k = noff + threadIdx.x; k < S1; k += T) keys[k] = ~0ull;
  __syncthreads();
  sort_keys(keys, S1);
  for (int k = threadIdx.x; k < noff; k += T) {
    const int q = (int)(keys[k] & 0x7FFFu);
    pos[q] = (uint16_t)(nsol + k);
    nsq[nsol + k] = (uint16_t)q;
  }
  __syncthreads();
  MC_PROBE_AT(4)
  // ---- E. contracted edges and each node's adjacency in insertion order ----------------------
  for (int v = threadIdx.x; v < M; v += T) {
    const int q = nsq[v], r = q / N, c = q - r * N;
    const bool sol = fl[q] & F_SOL;
    const uint32_t Dq = (uint32_t)sq_dist(q);
    int deg = 0, par = NONE, pard = 0, succ = NONE, succd = 0;
    int ch[4], chd[4], chf[4], nch = 0;
    for (int k = 0; k < 4; ++k) {
      int rr = r + dir_dr(k), cc = c + dir_dc(k);
      if (!(rr >= 0 && rr < N && cc >= 0 && cc < N && (fl[rr * N + cc] & F_OPEN))) continue;
      ++deg;
      const int y0 = rr * N + cc;
      int y = y0, cnt = 0;
      while (!(fl[y] & F_POINT)) {  // straight degree-2 squares: keep going
        rr += dir_dr(k);
        cc += dir_dc(k);
        y = rr * N + cc;
        ++cnt;
      }
      const int u = pos[y];
      bool is_par, is_succ = false;
      if (sol) {
        const uint32_t Dy0 = (uint32_t)sq_dist(y0);
        is_par = (fl[y0] & F_SOL) && Dy0 == Dq + 1;
        is_succ = (fl[y0] & F_SOL) && y0 == gp[q];
      } else {
        is_par = y0 == gp[q];
      }
      if (is_par) { par = u; pard = cnt; }
      else if (is_succ) { succ = u; succd = cnt; }
      else { ch[nch] = u; chd[nch] = cnt; chf[nch] = (int)(fst[y] & 0xFFFFu); ++nch; }
    }
    for (int a = 1; a < nch; ++a)  // children by first(): the order their paths were inserted
      for (int b = a; b > 0 && chf[b] < chf[b - 1]; --b) {
        int t = ch[b]; ch[b] = ch[b - 1]; ch[b - 1] = t;
        t = chd[b]; chd[b] = chd[b - 1]; chd[b - 1] = t;
        t = chf[b]; chf[b] = chf[b - 1]; chf[b - 1] = t;
      }
    int na = 0;
    uint16_t* ap = adjp + 4 * v;
    uint16_t* ad = adjd + 4 * v;
    if (sol) {
      if (par != NONE) { ap[na] = (uint16_t)par; ad[na++] = (uint16_t)pard; }
      if (succ != NONE) { ap[na] = (uint16_t)succ; ad[na++] = (uint16_t)succd; }
      for (int a = 0; a < nch; ++a) { ap[na] = (uint16_t)ch[a]; ad[na++] = (uint16_t)chd[a]; }
    } else {
      if (nch) { ap[na] = (uint16_t)ch[0]; ad[na++] = (uint16_t)chd[0]; }
      ap[na] = (uint16_t)par; ad[na++] = (uint16_t)pard;
      for (int a = 1; a < nch; ++a) { ap[na] = (uint16_t)ch[a]; ad[na++] = (uint16_t)chd[a]; }
    }
    adjn[v] = (uint8_t)na;
    gpar[v] = (uint16_t)par;
    gpd[v] = (uint16_t)pard;
    nfs[v] = (uint16_t)(fst[q] & 0xFFFFu);
    nfl[v] = (uint8_t)(deg | (sol ? N_SOL : 0) | (deg == 3 ? N_JUNC : 0));
  }
  __syncthreads();  // the square region is free from here on
  MC_PROBE_AT(5)
  // ---- F. hallways: components of the non-solution, non-junction nodes -----------------------
  auto in_h = [&](int v) { return !(nfl[v] & N_SOL) && (nfl[v] & 7) != 3; };
  auto in_b = [&](int v) { return !(nfl[v] & N_SOL) || (nfl[v] & N_JUNC); };
  for (int v = threadIdx.x; v < M; v += T) {
    const int p = gpar[v];
    hr[v] = in_h(v) ? (uint16_t)((p != NONE && in_h(p)) ? p : v) : NONE;
    br[v] = in_b(v) ? (uint16_t)((p != NONE && in_b(p)) ? p : v) : NONE;
    hmin[v] = 0xFFFFFFFFu;
    bmin[v] = 0xFFFFFFFFu;
    pref[v] = 0;
  }
  __syncthreads();
  for (int it = 0; (1 << it) < 2 * M; ++it) {  // pointer jumping to the component roots
    for (int v = threadIdx.x; v < M; v += T) {
      if (hr[v] != NONE) hr[v] = hr[hr[v]];
      if (br[v] != NONE) br[v] = br[br[v]];
    }
    __syncthreads();
  }
  for (int v = threadIdx.x; v < M; v += T) {
    if (hr[v] != NONE) atomicMin(&hmin[hr[v]], (uint32_t)v);
    if (br[v] != NONE) atomicMin(&bmin[br[v]], (uint32_t)v);
  }
  __syncthreads();
  // component numbers in the order of their first node: rank of hmin among the roots' hmin
  for (int v = threadIdx.x; v < M; v += T)
    if (hr[v] == v) pref[hmin[v]] = 1;
  __syncthreads();
  {
    int carry = 0;
    for (int v0 = 0; v0 < M; v0 += T) {
      const int v = v0 + threadIdx.x;
      const int f = v < M ? pref[v] : 0;
      int tot;
      const int rk = carry + block_excl(f, wsum, &tot);
      __syncthreads();
      if (v < M) pref[v] = (uint16_t)rk;  // hallway ids 1.. in order
      carry += tot;
      __syncthreads();
    }
    if (threadIdx.x == 0) s_Hn = carry;
  }
  __syncthreads();
  for (int v = threadIdx.x; v < M; v += T)
    if (hr[v] == v) {
      const int h = pref[hmin[v]] + 1;
      hroot[h] = (uint16_t)v;
    }
  __syncthreads();
  for (int v = threadIdx.x; v < M; v += T) hid[v] = hr[v] != NONE ? (uint16_t)(pref[hmin[hr[v]]] + 1) : 0;
  __syncthreads();
  for (int v = threadIdx.x; v < M; v += T) pref[v] = 0;
  __syncthreads();
  for (int v = threadIdx.x; v < M; v += T)
    if (br[v] == v) pref[bmin[v]] = 1;
  __syncthreads();
  {
    int carry = 0;
    for (int v0 = 0; v0 < M; v0 += T) {
      const int v = v0 + threadIdx.x;
      const int f = v < M ? pref[v] : 0;
      int tot;
      const int rk = carry + block_excl(f, wsum, &tot);
      __syncthreads();
      if (v < M) pref[v] = (uint16_t)rk;  // branch ranks 0.. in order
      carry += tot;
      __syncthreads();
    }
    if (threadIdx.x == 0) s_Bn = carry;
  }
  __syncthreads();
  for (int v = threadIdx.x; v < M; v += T) bid[v] = br[v] != NONE ? pref[bmin[br[v]]] : NONE;
  __syncthreads();
  const int Hn = s_Hn, Bn = s_Bn;
  MC_PROBE_AT(6)
  // ---- G. hallway complexities, one wave per hallway (extract_hallways :186-221,
  // complexity_of_hallway :286-296) ---------------------------------------------------------
  // member lists grouped by hallway id (the phase-F roots / minima are dead now)
  uint16_t* hlist = hr;     // [M] members, grouped by hallway
  uint32_t* hstart = hmin;  // [Hn + 2] first member of hallway h
  uint32_t* hcur = bmin;    // [Hn + 2] counts, then scatter cursors
  if (Hn + 2 > MM) { fail(2); return; }
  for (int h = threadIdx.x; h <= Hn + 1; h += T) hcur[h] = 0;
  if (threadIdx.x == 0) { s_nl = 0; s_nw = 0; s_wq = 0; }
#if MZ_MC_PROBE == 80
  if (threadIdx.x < 8) s_pt[threadIdx.x] = 0ull;
  if (threadIdx.x < 2) s_tmax[threadIdx.x] = 0u;
  unsigned long long pt[6] = {0ull, 0ull, 0ull, 0ull, 0ull, 0ull}, tl = 0ull;
#define MC_T(k) do { const unsigned long long t_ = clock64(); pt[k] += t_ - tl; tl = t_; } while (0)
#else
#define MC_T(k) do { } while (0)
#endif
  __syncthreads();
  for (int v = threadIdx.x; v < M; v += T)
    if (hid[v]) atomicAdd(&hcur[hid[v]], 1u);
  __syncthreads();
  {
    int carry = 0;
    for (int h0 = 0; h0 <= Hn + 1; h0 += T) {
      const int h = h0 + threadIdx.x;
      const int c = (h >= 1 && h <= Hn) ? (int)hcur[h] : 0;
      int tot;
      const int ex = carry + block_excl(c, wsum, &tot);
      __syncthreads();
      if (h <= Hn + 1) hstart[h] = (uint32_t)ex;
      carry += tot;
      __syncthreads();
    }
  }
  for (int h = threadIdx.x; h <= Hn + 1; h += T) hcur[h] = hstart[h];
  __syncthreads();
  for (int v = threadIdx.x; v < M; v += T)
    if (hid[v]) {
      const uint32_t at = atomicAdd(&hcur[hid[v]], 1u);
      hlist[at] = (uint16_t)v;
      pref[v] = (uint16_t)(at - hstart[hid[v]]);  // the member's index in its hallway's list
    }
  __syncthreads();
  {
    const int lane = threadIdx.x & (WAVE - 1);
    // cantor_pairing((r, c)) (:7-20) of every node, also its hash: < 2^16 for N <= 130, one LDS
    // load per lookup instead of nsq + a division (br is free from here on)
    uint16_t* nkey = br;
    for (int v = threadIdx.x; v < M; v += T) {
      const int q = nsq[v], r = q / N, c = q - r * N;
      nkey[v] = (uint16_t)((r + c) * (r + c + 1) / 2 + c);
    }
    __syncthreads();
    MC_PROBE_AT(71)
    auto key_of = [&](int v) -> uint32_t { return nkey[v]; };
    // a node's neighbours: its 4 adjacency slots in one 8-B load
    auto nbrs4 = [&](int x, int (&nb)[4]) {
      const uint2 w = *reinterpret_cast<const uint2*>(adjp + 4 * x);
      nb[0] = (int)(w.x & 0xFFFFu);
      nb[1] = (int)(w.x >> 16);
      nb[2] = (int)(w.y & 0xFFFFu);
      nb[3] = (int)(w.y >> 16);
    };
    auto wave_sum = [&](int x) {
      for (int k = WAVE / 2; k; k >>= 1) x += __shfl_xor(x, k);
      return x;
    };
    auto wave_min = [&](int x) {
      for (int k = WAVE / 2; k; k >>= 1) x = min(x, __shfl_xor(x, k));
      return x;
    };
    auto term = [](double& sum, long& D, int& nterm, int dd) {  // sum() from int 0, left to right
      const double t = __ddiv_rn(1.0, __dmul_rn(2.0, (double)dd));
      sum = nterm ? __dadd_rn(sum, t) : t;
      D += dd;
      ++nterm;
    };
    // the wave path: one hallway per wave, its sets in the wave's 128-slot tables
    auto wave_hallway = [&](int h) {
      const int b0 = (int)hstart[h], nc = (int)hstart[h + 1] - b0;
      // adjacent_split_points (:208-214): each member's junction neighbours up to and including
      // the first solution junction (the reference's break); in a tree each such junction
      // neighbours one member only
      int na_l = 0, f_l = 0x7FFFFFFF;
      for (int i = lane; i < nc; i += WAVE) {
        const int m = hlist[b0 + i];
        f_l = min(f_l, m);
        for (int k = 0; k < adjn[m]; ++k) {
          const int u = adjp[4 * m + k];
          if (nfl[u] & N_JUNC) {
            ++na_l;
            if (nfl[u] & N_SOL) break;
          }
        }
      }
      const int nasp = wave_sum(na_l);
      double sum = 0.0;
      long D = 0;
      int nterm = 0;
      auto add_term = [&](int dd) {  // sum() from int 0 (0 + t = t), then left to right
        const double t = __ddiv_rn(1.0, __dmul_rn(2.0, (double)dd));
        sum = nterm ? __dadd_rn(sum, t) : t;
        D += dd;
        ++nterm;
      };
      bool ok = true;
      if (nc + nasp <= 3) {
        // <= 3 view nodes, <= 2 edges: their sum does not depend on the order
        for (int i = 0; i < nc; ++i) {
          const int m = hlist[b0 + i];
          bool jstop = false;
          for (int k = 0; k < adjn[m]; ++k) {
            const int u = adjp[4 * m + k];
            if (in_h(u)) {
              if (u > m) add_term(adjd[4 * m + k]);
            } else if ((nfl[u] & N_JUNC) && !jstop) {
              add_term(adjd[4 * m + k]);
              if (nfl[u] & N_SOL) jstop = true;
            }
          }
        }
      } else if (nc + nasp > 63) {
        ok = false;  // beyond the wave's 128-slot tables: the host restatement
      } else {
        // _plain_bfs (nx.connected_components on temp_graph = G.copy() minus split / solution
        // points, :194-201): BFS from the member first in node order, each node's neighbours in
        // the copy's adjacency order — earlier neighbours by position, then later ones in G's
        // order — into `seen` (a set built by add())
        const int first = wave_min(f_l);
        WSet S1, S2;
        ws_init(S1);
        uint32_t qv = 0;  // BFS queue: entry i in lane i
        int qn = 0;
        auto push = [&](int v) {
          if (lane == qn) qv = (uint32_t)v;
          ++qn;
        };
        ok = ws_add(S1, key_of(first), (uint32_t)first) >= 0;
        push(first);
        for (int hd = 0; hd < qn && ok; ++hd) {
          const int x = __shfl((int)qv, hd);
          const int na = adjn[x];
          int ord[4], no = 0;
          for (int k = 0; k < na; ++k) {  // earlier neighbours, ascending
            const int u = adjp[4 * x + k];
            if (u >= x) continue;
            int j = no++;
            while (j > 0 && ord[j - 1] > u) { ord[j] = ord[j - 1]; --j; }
            ord[j] = u;
          }
          for (int k = 0; k < na; ++k) {
            const int u = adjp[4 * x + k];
            if (u > x) ord[no++] = u;
          }
          for (int k = 0; k < no && ok; ++k) {
            const int u = ord[k];
            if (!in_h(u)) continue;
            const int r = ws_add(S1, key_of(u), (uint32_t)u);
            if (r < 0) ok = false;
            else if (r == 1) push(u);
          }
        }
        ok = ok && ws_copy(S2, S1);  // set(component_nodes) (:205)
        // adjacent_split_points, filled in that set's order
        ws_init(S1);
        for (int j = ws_next(S2, -1); j >= 0 && ok; j = ws_next(S2, j)) {
          const int m = (int)(ws_get(S2, j) & 0xFFFFu);
          for (int k = 0; k < adjn[m]; ++k) {
            const int u = adjp[4 * m + k];
            if (nfl[u] & N_JUNC) {
              if (ws_add(S1, key_of(u), (uint32_t)u) < 0) ok = false;
              if (nfl[u] & N_SOL) break;
            }
          }
        }
        // all_nodes = component_nodes.union(adjacent_split_points) (:217): the copy of a
        // dummy-free set has its layout, then the merge
        ok = ok && ws_merge(S2, S1);
        // show_nodes(nbunch_iter(all_nodes)).nodes: a set built by add() in all_nodes' order
        ws_init(S1);
        for (int j = ws_next(S2, -1); j >= 0 && ok; j = ws_next(S2, j)) {
          const uint32_t v = ws_get(S2, j);
          if (ws_add(S1, v >> 16, v & 0xFFFFu) < 0) ok = false;
        }
        if (ok && 2 * S1.used < M) {
          // FilterAdjacency iterates the set; EdgeDataView reports (n, u) for u in G's adjacency
          // order of n, inside the view, not yet iterated
          for (int j = ws_next(S1, -1); j >= 0; j = ws_next(S1, j)) {
            const int n = (int)(ws_get(S1, j) & 0xFFFFu);
            for (int k = 0; k < adjn[n]; ++k)
              if (ws_find(S1, key_of(adjp[4 * n + k])) > j) add_term(adjd[4 * n + k]);
          }
        } else if (ok) {
          // the view holds at least half of G: G's node order (position)
          int last = -1;
          for (int c = 0; c < S1.used; ++c) {
            int cand = 0x7FFFFFFF;
            if (S1.v0 != WS_EMPTY && (int)(S1.v0 & 0xFFFFu) > last) cand = (int)(S1.v0 & 0xFFFFu);
            if (S1.v1 != WS_EMPTY && (int)(S1.v1 & 0xFFFFu) > last)
              cand = min(cand, (int)(S1.v1 & 0xFFFFu));
            const int n = wave_min(cand);
            for (int k = 0; k < adjn[n]; ++k) {
              const int u = adjp[4 * n + k];
              if (u > n && ws_find(S1, key_of(u)) >= 0) add_term(adjd[4 * n + k]);
            }
            last = n;
          }
        }
      }
      if (!ok) {
        if (lane == 0) s_bad = 2;
      } else if (lane == 0) {
        Ch[h] = __dmul_rn((double)D, sum);
      }
    };
    // the lane path: one hallway per lane, <= 15 view nodes (every table stays within 32 slots:
    // add() resizes at 19 of 32, set(s) / update() to 2 x 15 = 30 < 32), its three tables (the
    // set being built, the set it is built from, the resize scratch) interleaved in the keys and
    // Cb regions (both free until phase H)
    auto lane_hallway = [&](int h, uint16_t* base, int st) -> bool {
      const int b0 = (int)hstart[h], nc = (int)hstart[h + 1] - b0;
      uint16_t* q = hlist + b0;  // the member list, then the BFS queue (the same nc nodes)
#if MZ_MC_PROBE == 80
      tl = clock64();
#endif
      int first = 0x7FFFFFFF;
      for (int i = 0; i < nc; ++i) first = min(first, (int)q[i]);
      uint16_t* tA = base;
      uint16_t* tB = base + 32 * st;
      uint16_t* tT = base + 64 * st;
      double sum = 0.0;
      long D = 0;
      int nterm = 0;
      LSet S1, S2;
      ls_init(S1, tA, st);
      bool ok = ls_add(S1, first, tT, key_of) >= 0;
      q[0] = (uint16_t)first;
      int qn = 1;
      for (int hd = 0; hd < qn && ok; ++hd) {  // _plain_bfs, as in the wave path
        const int x = q[hd];
        const int na = adjn[x];
        int nb[4];
        nbrs4(x, nb);
        // the neighbours' flags and keys, loaded together (one LDS round trip)
        uint32_t fk[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int u = k < na ? nb[k] : x;
          fk[k] = ((uint32_t)nfl[u] << 16) | nkey[u];
        }
        // visiting order: earlier neighbours ascending, then later ones in G's order (sort key:
        // the node id, or 2^16 + slot; unused slots last), by a 4-element sorting network with
        // (flags | key) << 16 | node carried along — static indices only (registers)
        uint32_t sk[4];
        uint64_t pl[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          sk[k] = k >= na ? 0x20000u : (nb[k] < x ? (uint32_t)nb[k] : 0x10000u + k);
          pl[k] = ((uint64_t)fk[k] << 16) | (uint32_t)nb[k];
        }
        auto cx = [&](int a, int b) {
          const bool sw = sk[b] < sk[a];
          const uint32_t ta = sk[a], tb = sk[b];
          const uint64_t pa = pl[a], pb = pl[b];
          sk[a] = sw ? tb : ta; sk[b] = sw ? ta : tb;
          pl[a] = sw ? pb : pa; pl[b] = sw ? pa : pb;
        };
        cx(0, 1); cx(2, 3); cx(0, 2); cx(1, 3); cx(1, 2);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (k >= na || !ok) continue;
          const int u = (int)(pl[k] & 0xFFFFu);
          const uint32_t f = (uint32_t)(pl[k] >> 32) & 0xFFu;
          if ((f & N_SOL) || (f & 7) == 3) continue;  // in_h(u)
          const int r = ls_add_k(S1, u, (uint32_t)(pl[k] >> 16) & 0xFFFFu, tT, key_of);
          if (r < 0 || (r == 1 && qn >= nc)) ok = false;
          else if (r == 1) q[qn++] = (uint16_t)u;
        }
      }
      MC_T(0);
      ok = ok && ls_copy(S2, tB, S1, tT, key_of);
      MC_T(1);
      ls_init(S1, tA, st);
      for (int j = 0; j <= S2.mask && ok; ++j) {
        if (!((S2.occ >> j) & 1u)) continue;
        const int m = S2.t[j * st];
        const int na = adjn[m];
        int nb[4];
        nbrs4(m, nb);
        uint32_t fk[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int u = k < na ? nb[k] : m;
          fk[k] = ((uint32_t)nfl[u] << 16) | nkey[u];
        }
        bool stop = false;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t f = fk[k] >> 16;
          if (k < na && !stop && (f & N_JUNC)) {
            if (ls_add_k(S1, nb[k], fk[k] & 0xFFFFu, tT, key_of) < 0) ok = false;
            if (f & N_SOL) stop = true;
          }
        }
      }
      MC_T(2);
      ok = ok && ls_merge(S2, S1, tT, key_of);
      MC_T(3);
      ls_init(S1, tA, st);
      for (int j = 0; j <= S2.mask && ok; ++j)
        if ((S2.occ >> j) & 1u)
          if (ls_add(S1, S2.t[j * st], tT, key_of) < 0) ok = false;
      MC_T(4);
      if (!ok) return false;
      if (2 * S1.used < M) {
        for (int j = 0; j <= S1.mask; ++j) {
          if (!((S1.occ >> j) & 1u)) continue;
          const int nn = S1.t[j * st];
          const int na = adjn[nn];
          int nb[4];
          nbrs4(nn, nb);
          uint32_t ky[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) ky[k] = nkey[k < na ? nb[k] : nn];
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (k < na && ls_find(S1, ky[k], nb[k]) > j) term(sum, D, nterm, adjd[4 * nn + k]);
        }
      } else {
        int last = -1;
        for (int c = 0; c < S1.used; ++c) {
          int nn = 0x7FFFFFFF;
          for (int j = 0; j <= S1.mask; ++j)
            if ((S1.occ >> j) & 1u) {
              const int v = S1.t[j * st];
              if (v > last) nn = min(nn, v);
            }
          for (int k = 0; k < adjn[nn]; ++k) {
            const int u = adjp[4 * nn + k];
            if (u > nn && ls_find(S1, key_of(u), u) >= 0) term(sum, D, nterm, adjd[4 * nn + k]);
          }
          last = nn;
        }
      }
      Ch[h] = __dmul_rn((double)D, sum);
      MC_T(5);
      return true;
    };
    // the lane path, ALU edition: the same sets as lane_hallway, laid out by lw_layout_add /
    // lw_free in registers; per-lane LDS (base, stride st: 96 u16) holds only the scatter buffers
    // that turn slots into iteration order
    auto lane_hallway2 = [&](int h, uint32_t* base, int st) -> bool {
      const int b0 = (int)hstart[h], nc = (int)hstart[h + 1] - b0;
      uint16_t* q = hlist + b0;
      uint32_t* xs = base;            // [16] scatter buffer (entry words)
      uint32_t* as = base + 16 * st;  // [16] split points in insertion order
      // _plain_bfs from the first member in node order; seen = a bit per member index (pref)
      int first = 0x7FFFFFFF;
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (i < nc) first = min(first, (int)q[i]);
      uint32_t vis = 1u << pref[first];
      q[0] = (uint16_t)first;
      int qn = 1;
      for (int hd = 0; hd < qn; ++hd) {
        const int x = q[hd];
        const int na = adjn[x];
        int nb[4];
        nbrs4(x, nb);
        uint32_t fm[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int u = k < na ? nb[k] : x;
          fm[k] = ((uint32_t)nfl[u] << 24) | ((uint32_t)(pref[u] & 0xFFu) << 16) | (uint32_t)u;
        }
        uint32_t sk[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) sk[k] = k >= na ? 0x20000u : (nb[k] < x ? (uint32_t)nb[k] : 0x10000u + k);
        auto cx = [&](int a, int b) {
          const bool sw = sk[b] < sk[a];
          const uint32_t ta = sk[a], tb = sk[b], fa = fm[a], fb = fm[b];
          sk[a] = sw ? tb : ta; sk[b] = sw ? ta : tb;
          fm[a] = sw ? fb : fa; fm[b] = sw ? fa : fb;
        };
        cx(0, 1); cx(2, 3); cx(0, 2); cx(1, 3); cx(1, 2);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (k >= na) continue;
          const uint32_t f = fm[k] >> 24, mi = (fm[k] >> 16) & 0xFFu;
          if ((f & N_SOL) || (f & 7) == 3) continue;  // not in the hallway
          if (mi >= 16 || ((vis >> mi) & 1u)) continue;
          vis |= 1u << mi;
          if (qn < nc) q[qn] = (uint16_t)(fm[k] & 0xFFFFu);
          ++qn;
        }
      }
      if (qn != nc) return false;
      // S1: seen, built by add() in BFS order
      uint32_t P[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) P[i] = i < nc ? (uint32_t)q[i] : 0u;
#pragma unroll
      for (int i = 0; i < 16; ++i) P[i] |= (i < nc ? (uint32_t)nkey[P[i]] : 0u) << 11;
      uint32_t occ;
      int mask;
      lw_layout_add(P, nc, occ, mask);
      // the entries A[0..n) of a set with occupancy o -> A in the set's iteration order (by rank)
      auto order = [&](uint32_t (&A)[16], int n, uint32_t o) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (i < n) {
            const int r = __popc(o & ((1u << lw_slot(A[i])) - 1u));
            xs[r * st] = A[i];
          }
#pragma unroll
        for (int i = 0; i < 16; ++i) A[i] = i < n ? xs[i * st] : 0u;
      };
      // S2 = set(S1): set_merge into an empty set — resize to (used * 2) when used * 5 >= 21,
      // then S1's layout if the sizes agree, else insert_clean in S1's order
      order(P, nc, occ);  // P: S1's order (slots kept in the words)
      const int mask2 = nc * 5 >= 21 ? lw_mask_for(nc * 2) : 7;
      if (mask2 != mask) {
        occ = 0u;
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (i < nc) lw_put(P[i], occ, mask2);
        order(P, nc, occ);  // P: S2's order
      }
      // adjacent_split_points: for each member in S2's order, its junction neighbours in G's order
      // up to and including the first solution junction — a set built by add()
      int nasp = 0;
#pragma unroll
      for (int c0 = 0; c0 < 16; c0 += 4) {
        int nbv[4][4], nav[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int m = c0 + c < nc ? lw_node(P[c0 + c]) : first;
          nav[c] = c0 + c < nc ? (int)adjn[m] : 0;
          nbrs4(m, nbv[c]);
        }
        uint32_t fk[4][4];
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int u = k < nav[c] ? nbv[c][k] : first;
            fk[c][k] = ((uint32_t)nfl[u] << 16) | nkey[u];
          }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          bool stop = false;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const uint32_t f = fk[c][k] >> 16;
            if (k < nav[c] && !stop && (f & N_JUNC)) {
              if (nasp < 16) as[nasp * st] = ((fk[c][k] & 0xFFFFu) << 11) | (uint32_t)nbv[c][k];
              ++nasp;
              if (f & N_SOL) stop = true;
            }
          }
        }
      }
      if (nc + nasp > 15) return false;
      uint32_t A[16];
#pragma unroll
      for (int i = 0; i < 16; ++i)
        A[i] = i < nasp ? as[i * st] : 0u;
      uint32_t occa;
      int maska;
      lw_layout_add(A, nasp, occa, maska);
      order(A, nasp, occa);  // A: the split points' set order
      // all_nodes = S2.union(asp): a copy of S2 (S2's layout), set_merge of asp: resize to
      // (used + asp) * 2 first when (fill + asp) * 5 >= mask * 3 (S2's entries re-inserted in its
      // order), then asp's entries added in its order
      int maskm = mask2;
      uint32_t occm = occ;
      if (nasp > 0 && (nc + nasp) * 5 >= mask2 * 3) {
        maskm = lw_mask_for((nc + nasp) * 2);
        occm = 0u;
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (i < nc) lw_put(P[i], occm, maskm);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (i < nasp) lw_put(A[i], occm, maskm);
      // the union's order: both parts scattered by rank into one buffer
      const int nv = nc + nasp;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (i < nc) xs[__popc(occm & ((1u << lw_slot(P[i])) - 1u)) * st] = P[i] & 0x1FFFFFFu;
        if (i < nasp) xs[__popc(occm & ((1u << lw_slot(A[i])) - 1u)) * st] = A[i] & 0x1FFFFFFu;
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) P[i] = i < nv ? xs[i * st] : 0u;
      // show_nodes(nbunch_iter(all_nodes)): a set built by add() in the union's order
      lw_layout_add(P, nv, occ, mask);
      order(P, nv, occ);  // P: the view's order
      constexpr int EB = 2;
      // EdgeDataView: for each view node in order, its neighbours in G's order that are in the
      // view and not yet iterated (2 * nv < M: the classifier's condition)
      double sum = 0.0;
      long D = 0;
      int nterm = 0;
#pragma unroll
      for (int c0 = 0; c0 < 16; c0 += EB) {
        int nbv[EB][4], nav[EB];
        uint2 dv[EB];
#pragma unroll
        for (int c = 0; c < EB; ++c) {
          const int nn = c0 + c < nv ? lw_node(P[c0 + c]) : first;
          nav[c] = c0 + c < nv ? (int)adjn[nn] : 0;
          nbrs4(nn, nbv[c]);
          dv[c] = *reinterpret_cast<const uint2*>(adjd + 4 * nn);
        }
#pragma unroll
        for (int c = 0; c < EB; ++c) {
          const int j = c0 + c;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            if (k >= nav[c]) continue;
            const int u = nbv[c][k];
            bool later = false;
#pragma unroll
            for (int e = 0; e < 16; ++e) later |= e > j && e < nv && lw_node(P[e]) == u;
            if (later) {
              const uint32_t w = k < 2 ? dv[c].x : dv[c].y;
              term(sum, D, nterm, (int)((k & 1) ? (w >> 16) : (w & 0xFFFFu)));
            }
          }
        }
      }
      Ch[h] = __dmul_rn((double)D, sum);
      return true;
    };
    // G1: one thread per hallway classifies it — <= 3 view nodes: its sum now (the fast path);
    // <= 15: the lane queue; else the wave queue (both in the phase-F bmin region, free now)
    uint16_t* Lq = reinterpret_cast<uint16_t*>(bmin);
    uint16_t* Wq = Lq + MM;
    const int Lr = (int)((size_t)MK * 8 / (96 * sizeof(uint16_t)));  // lanes in the keys region
    const int Lc = (int)((size_t)MM * 8 / (96 * sizeof(uint16_t)));  // lanes in the Cb region
#ifndef MZ_MC_LMAX
#define MZ_MC_LMAX 1024
#endif
    const int L = min(min(Lr + Lc, T / 2), MZ_MC_LMAX);
    for (int h = 1 + threadIdx.x; h <= Hn; h += T) {
      const int b0 = (int)hstart[h], nc = (int)hstart[h + 1] - b0;
      int nasp = 0;
      if (nc <= 15)
        for (int i = 0; i < nc; ++i) {
          const int m = hlist[b0 + i];
          for (int k = 0; k < adjn[m]; ++k) {
            const int u = adjp[4 * m + k];
            if (nfl[u] & N_JUNC) {
              ++nasp;
              if (nfl[u] & N_SOL) break;
            }
          }
        }
      if (nc <= 15 && nc + nasp <= 3) {
        double sum = 0.0;
        long D = 0;
        int nterm = 0;
        for (int i = 0; i < nc; ++i) {
          const int m = hlist[b0 + i];
          bool jstop = false;
          for (int k = 0; k < adjn[m]; ++k) {
            const int u = adjp[4 * m + k];
            if (in_h(u)) {
              if (u > m) term(sum, D, nterm, adjd[4 * m + k]);
            } else if ((nfl[u] & N_JUNC) && !jstop) {
              term(sum, D, nterm, adjd[4 * m + k]);
              if (nfl[u] & N_SOL) jstop = true;
            }
          }
        }
        Ch[h] = __dmul_rn((double)D, sum);
      } else if (nc <= 15 && nc + nasp <= 15 && L > 0 && 2 * (nc + nasp) < M &&
                 (!MZ_MC_LANE2 || (MM <= 2048 && N <= 91))) {
        Lq[atomicAdd(&s_nl, 1)] = (uint16_t)h;
      } else {
        Wq[atomicAdd(&s_nw, 1)] = (uint16_t)h;
      }
    }
    __syncthreads();
    MC_PROBE_AT(72)
    // G2: the lane queue over the first MC_LANE_WAVES waves, item v to lane v / MC_LANE_WAVES of
    // wave v % MC_LANE_WAVES — a few active lanes per wave, so each LDS instruction of the lane
    // path's lookup chains serves few random addresses (fewer bank conflicts) and many waves keep
    // chains in flight; the other waves start on the wave queue at once, and every wave, once its
    // lanes are done, takes the wave queue's hallways one at a time
    const int nl = s_nl, nw = s_nw;
    const int wid = threadIdx.x / WAVE;
#if MZ_MC_PROBE == 80
    const unsigned long long tg0 = clock64();
#endif
    if (wid < MC_LANE_WAVES && MZ_MC_PROBE != 73) {
      const int l = lane * MC_LANE_WAVES + wid;  // virtual lane: its table slot
      if (l < L) {
        uint16_t* base = l < Lr ? reinterpret_cast<uint16_t*>(keys) + l
                                : reinterpret_cast<uint16_t*>(Cb) + (l - Lr);
        const int st = l < Lr ? Lr : Lc;
        // (the ALU edition's buffers: u32 words, interleaved by lane the same way, 32 per lane)
        uint32_t* base32 = l < Lr ? reinterpret_cast<uint32_t*>(keys) + l
                                  : reinterpret_cast<uint32_t*>(Cb) + (l - Lr);
        for (int k = l; k < nl; k += L)
          if (!(MZ_MC_LANE2 ? lane_hallway2(Lq[k], base32, st) : lane_hallway(Lq[k], base, st)))
            s_bad = 2;
      }
#if MZ_MC_PROBE == 80
      for (int k = 0; k < 6; ++k) {  // the wave's pass times (every lane holds the same sums)
        unsigned long long v = pt[k];
        for (int o = WAVE / 2; o; o >>= 1) {
          const unsigned long long w_ = ((unsigned long long)__shfl_xor((int)(v >> 32), o) << 32) |
                                        (unsigned int)__shfl_xor((int)(unsigned int)v, o);
          v = v > w_ ? v : w_;
        }
        if (lane == 0) atomicAdd(&s_pt[k], v);
      }
      if (lane == 0) atomicMax(&s_tmax[0], (unsigned int)(clock64() - tg0));
#endif
    }
    for (;;) {
      int k = 0;
      if (lane == 0) k = atomicAdd(&s_wq, 1);
      k = __shfl(k, 0);
      if (k >= nw || MZ_MC_PROBE == 74) break;
      wave_hallway(Wq[k]);
    }
#if MZ_MC_PROBE == 80
    if (lane == 0) atomicMax(&s_tmax[1], (unsigned int)(clock64() - tg0));
#endif
  }
  __syncthreads();
#if MZ_MC_PROBE == 80
  if (threadIdx.x == 0) {
    auto f17 = [&](int k) -> double {  // mean per lane wave, 16-cycle units, 17 bits
      const unsigned long long v = s_pt[k] / (16ull * MC_LANE_WAVES);
      return (double)(v < 131071ull ? v : 131071ull);
    };
    out[2 * i] = f17(0) + f17(1) * 131072.0 + f17(2) * 17179869184.0;
    out[2 * i + 1] = f17(3) + f17(4) * 131072.0 + f17(5) * 17179869184.0;
    status[i] = (int)(min(s_tmax[0] / 64u, 32767u) | (min(s_tmax[1] / 64u, 32767u) << 16));
  }
  return;
#endif
  if (s_bad) { fail(2); return; }
  MC_PROBE_AT(7)
  // hallway 0: the solution branch, edges in path order — the terms 1 / (2 d) by all threads (into
  // Cb, free until phase H), then one thread adds them left to right (a dfs maze's solution has
  // ~1,000 nodes: the f64 divisions in that thread's loop were most of phase H)
  for (int v = 1 + threadIdx.x; v < nsol; v += T)
    Cb[v] = __ddiv_rn(1.0, __dmul_rn(2.0, (double)gpd[v]));
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    long D = 0;
#pragma unroll 8
    for (int v = 1; v < nsol; ++v) {
      s = v == 1 ? Cb[v] : __dadd_rn(s, Cb[v]);
      D += gpd[v];
    }
    Ch[0] = __dmul_rn((double)D, s);
  }
  __syncthreads();
  // ---- H. branch sums over their hallways in id order, the product over branches -------------
  for (int h = 1 + threadIdx.x; h <= Hn; h += T)
    keys[h - 1] = ((uint64_t)bid[hroot[h]] << 16) | (uint64_t)h;
  const int S3 = next_pow2(Hn > 1 ? Hn : 2);
  for (int k = Hn + threadIdx.x; k < S3; k += T) keys[k] = ~0ull;
  for (int b = threadIdx.x; b < Bn; b += T) pref[b] = NONE;
  __syncthreads();
  sort_keys(keys, S3);
  for (int k = threadIdx.x; k < Hn; k += T) {
    const int b = (int)(keys[k] >> 16);
    if (k == 0 || (int)(keys[k - 1] >> 16) != b) pref[b] = (uint16_t)k;
  }
  __syncthreads();
  for (int b = threadIdx.x; b < Bn; b += T) {
    double cx = 0.0;
    const int k0 = pref[b];
    if (k0 != NONE)
      for (int k = k0; k < Hn && (int)(keys[k] >> 16) == b; ++k) {
        const double c = Ch[(int)(keys[k] & 0xFFFFu)];
        cx = k == k0 ? c : __dadd_rn(cx, c);
      }
    Cb[b] = cx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double prod = 1.0, sum = 0.0;
    for (int b = 0; b < Bn; ++b) {
      prod = __dmul_rn(prod, __dadd_rn(Cb[b], 1.0));
      sum = __dadd_rn(sum, Cb[b]);
    }
    prod = __dmul_rn(prod, Ch[0]);
    sum = __dadd_rn(sum, Ch[0]);
    out[2 * i] = prod;
    out[2 * i + 1] = sum;
    status[i] = prod > 0.0 ? 0 : 3;
  }
}

// Workgroups score candidates blockIdx.x, + gridDim.x, ... (one workgroup per candidate when the
// grid is the list; MZ_MC_WGS > 0 caps the resident workgroups of a launch, each then scoring
// several in turn). A bank refill scores the candidates of its consumed slots only:
// min(*limit, n / mult) groups of mult.
#ifndef MZ_MC_WGS
#define MZ_MC_WGS 0
#endif
__global__ __launch_bounds__(T) void k_mcclendon(MzDev d, const int32_t* ids, int n, int MM, int MK,
                                                 double* out, int32_t* status, const int* limit,
                                                 int mult) {
  const int m = limit ? min(*limit, n / mult) * mult : n;
#if MZ_MC_WGS > 0
  // (the loop costs the body 208 B of scratch per lane at 128 VGPRs: built only when capped)
  for (int i = blockIdx.x; i < m; i += gridDim.x) {
    mc_score(i, d, ids, n, MM, MK, out, status);
    __syncthreads();  // the next candidate reuses this workgroup's LDS
  }
#else
  if ((int)blockIdx.x < m) mc_score(blockIdx.x, d, ids, n, MM, MK, out, status);
#endif
}


}  // namespace

size_t mz_mcclendon_lds(int P, bool toroidal, int* mm) {
  const int Pb = toroidal ? P + 2 : P;  // a toroidal maze is scored on its bordered grid
  const int cells = ((Pb - 1) / 2) * ((Pb - 1) / 2) + 4;
  // the sort buffer holds a power of two (the bitonic sorts); every other node array the node
  // count rounded up to 64 (a power of two there left ~20 % of a workgroup's LDS unused, and LDS
  // is what decides whether the trainer's kernels can share a CU with this one)
  const int MM = (cells + 63) & ~63;
  int MK = 16;
  while (MK < MM) MK <<= 1;
  *mm = MM;
  const size_t NNP = (size_t)Pb * Pb;
  size_t sq = (NNP * 9 + 16 + 15) & ~(size_t)15;
  if (toroidal) sq += (NNP * 2 + 15) & ~(size_t)15;  // the distance field
  const size_t node = (size_t)MK * 8 + (size_t)MM * (2 + 8 + 8 + 2 + 2 + 2 + 1 + 1);
  const size_t ph2 = (size_t)MM * (2 * 6 + 4 * 2 + 8 * 2);
  return (sq > ph2 ? sq : ph2) + node;
}

hipError_t mz_launch_mcclendon(const MzDev& d, const int32_t* ids, int n, double* out,
                               int32_t* status, hipStream_t s, const int* limit, int mult) {
  if (n <= 0) return hipSuccess;
  int MM = 0;
  const size_t bytes = mz_mcclendon_lds(d.P, d.toroidal != 0, &MM);
  if (bytes > 160 * 1024) return hipErrorInvalidValue;
  if (bytes > 65536) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_mcclendon),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return e;
  }
  int MK = 16;
  while (MK < MM) MK <<= 1;
  const int grid = MZ_MC_WGS > 0 && n > MZ_MC_WGS ? MZ_MC_WGS : n;
  hipLaunchKernelGGL(k_mcclendon, dim3(grid), dim3(T), bytes, s, d, ids, n, MM, MK, out, status, limit,
                     mult < 1 ? 1 : mult);
  return hipGetLastError();
}
