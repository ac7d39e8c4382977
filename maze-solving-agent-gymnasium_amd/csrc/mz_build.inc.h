// mz_build.inc.h — per-maze build on gfx950 (one 64-lane wave per maze, state in LDS).
// Included by mz_env.hip (one translation unit: the reset kernel regenerates mazes in place).
//
//   generation  random_prim_visit / deept_first_visit / prim_and_kill_visit
//               (maze_generation.py:59-185) over a Philox stream; lane 0 runs the sequential
//               carve loop, the prim&kill restart pick (:151) is a wave scan over a
//               candidate bit per cell that the walk keeps current.
//   goal        find_random_position (:187-218): wave BFS from start + wave max-reduce
//   toroidal    gen_maze_no_border (:37-56): generate (N+2)^2, pick goal, crop the border
//   tables      BFS distance-to-goal field (replaces per-step A*, a_star.py:9-82), best-next
//               code per cell (_find_best_next_cell base_maze_env.py:224-262), open-neighbour
//               mask (get_direction_mask maze_handler.py:122-162), open bit-plane rows,
//               max_steps (set_max_steps simple_maze_env.py:52-58), reset state.
#pragma once
#include "mz_common.h"
#include "mz_screen.h"

// Distance fields of Philox-generated mazes from the carved tree (mz_tree_dist) instead of
// level-synchronous BFS; 0 = the BFS everywhere (A/B builds)
#ifndef MZ_TREE_DIST
#define MZ_TREE_DIST 1
#endif

struct MzBuildLds {
  uint8_t* g;        // [G*G] grid
  uint16_t* dist;    // [G*G]
  uint16_t* queue;   // [G*G]
  uint32_t* vis;     // [(G*G+31)/32]
  int* sh;           // scalars
};

__host__ __device__ inline size_t mz_align16(size_t x) { return (x + 15) & ~(size_t)15; }

__host__ __device__ inline size_t mz_build_lds_bytes(int P) {
  const size_t G = (size_t)P + 2, C = G * G;
  return 64 + mz_align16(C) + 2 * mz_align16(2 * C) + mz_align16(4 * ((C + 31) / 32));
}

__device__ inline MzBuildLds mz_build_lds(uint8_t* base, int P) {
  const size_t G = (size_t)P + 2, C = G * G;
  MzBuildLds L;
  L.sh = reinterpret_cast<int*>(base);
  size_t off = 64;
  L.g = base + off; off += mz_align16(C);
  L.dist = reinterpret_cast<uint16_t*>(base + off); off += mz_align16(2 * C);
  L.queue = reinterpret_cast<uint16_t*>(base + off); off += mz_align16(2 * C);
  L.vis = reinterpret_cast<uint32_t*>(base + off);
  return L;
}

// Level-synchronous wave BFS over open cells of the G x G grid from src (wrap if tor).
__device__ void mz_wave_bfs(const MzBuildLds& L, int G, bool tor, int src) {
  const int lane = threadIdx.x, C = G * G;
  for (int i = lane; i < C; i += 64) L.dist[i] = 0xFFFF;
  for (int i = lane; i < (C + 31) / 32; i += 64) L.vis[i] = 0u;
  __syncthreads();
  if (lane == 0) {
    L.dist[src] = 0;
    L.queue[0] = (uint16_t)src;
    L.vis[src >> 5] |= 1u << (src & 31);
    L.sh[0] = 1;
  }
  __syncthreads();
  int head = 0, tail = 1;
  while (head < tail) {
    for (int base = head; base < tail; base += 64) {
      const int i = base + lane;
      if (i < tail) {
        const int v = L.queue[i], dv = L.dist[v], r = v / G, c = v - r * G;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          int nr = r + mz_dr(k), nc = c + mz_dc(k);
          if (tor) { nr = mz_wrap(nr, G); nc = mz_wrap(nc, G); }
          else if (nr < 0 || nr >= G || nc < 0 || nc >= G) continue;
          const int n = nr * G + nc;
          if (L.g[n] == 0) continue;
          const uint32_t bit = 1u << (n & 31);
          if (atomicOr(&L.vis[n >> 5], bit) & bit) continue;
          L.dist[n] = (uint16_t)(dv + 1);
          L.queue[atomicAdd(&L.sh[0], 1)] = (uint16_t)n;
        }
      }
    }
    __syncthreads();
    head = tail;
    tail = L.sh[0];
    __syncthreads();
  }
}

// --- generators (lane 0 unless noted); G = generation grid size (odd) ------------------------
// Up to 4 small values (cell keys < 2^16, directions) packed in one u64: the lists stay in
// registers — an int[4] indexed by a random draw lives in per-lane scratch memory.
__device__ inline int mz_k4(uint64_t v, int i) { return (int)((v >> (16 * i)) & 0xFFFFu); }
__device__ inline void mz_k4_push(uint64_t& v, int& n, int x) {
  v |= (uint64_t)(uint32_t)x << (16 * n);
  ++n;
}
// neighbour order of get_neighbors / random_walk: (-2,0),(2,0),(0,-2),(0,2) (maze_generation.py:72)
__device__ inline int mz_g2r(int k) { return k == 0 ? -2 : (k == 1 ? 2 : 0); }
__device__ inline int mz_g2c(int k) { return k == 2 ? -2 : (k == 3 ? 2 : 0); }
// direction order of deept_first_visit: (0,-1),(0,1),(-1,0),(1,0) (maze_generation.py:114)
__device__ inline int mz_fr(int k) { return k == 2 ? -1 : (k == 3 ? 1 : 0); }
__device__ inline int mz_fc(int k) { return k == 0 ? -1 : (k == 1 ? 1 : 0); }

__device__ void mz_gen_rprim(const MzBuildLds& L, int G, int s, MzRng& rng) {
  uint8_t* m = L.g;
  uint16_t* fr = L.queue;
  uint16_t* dep = L.dist;  // distance from s in the carved tree (MZ_TREE_DIST)
  uint32_t* inF = L.vis;
  for (int i = 0; i < (G * G + 31) / 32; ++i) inF[i] = 0u;
  int nf = 0;
  const int sr = s / G, sc = s - sr * G;
  m[s] = 1;
  dep[s] = 0;
  for (int k = 0; k < 4; ++k) {
    int r = sr + mz_g2r(k), c = sc + mz_g2c(k);
    if (r < 0 || r >= G || c < 0 || c >= G) continue;
    int j = r * G + c;
    fr[nf++] = (uint16_t)j; inF[j >> 5] |= 1u << (j & 31);
  }
  while (nf > 0) {
    const int i = (int)rng.below((uint32_t)nf);
    const int f = fr[i];
    fr[i] = fr[--nf];
    const int fx = f / G, fy = f - fx * G;
    uint64_t nb = 0;
    int cnt = 0;
    for (int k = 0; k < 4; ++k) {
      int r = fx + mz_g2r(k), c = fy + mz_g2c(k);
      if (r < 0 || r >= G || c < 0 || c >= G) continue;
      if (m[r * G + c] == 1) mz_k4_push(nb, cnt, r * G + c);
    }
    if (cnt) {
      const int nn = mz_k4(nb, (int)rng.below((uint32_t)cnt));
      const int nx = nn / G, ny = nn - nx * G;
      const int pass = ((fx + nx) / 2) * G + (fy + ny) / 2, dn = dep[nn];
      m[f] = 1;
      m[pass] = 1;
      dep[pass] = (uint16_t)(dn + 1);
      dep[f] = (uint16_t)(dn + 2);
      for (int k = 0; k < 4; ++k) {
        int r = fx + mz_g2r(k), c = fy + mz_g2c(k);
        if (r < 0 || r >= G || c < 0 || c >= G) continue;
        int j = r * G + c;
        if (m[j] == 0 && !((inF[j >> 5] >> (j & 31)) & 1u)) {
          fr[nf++] = (uint16_t)j; inF[j >> 5] |= 1u << (j & 31);
        }
      }
    }
  }
}

__device__ void mz_gen_dfs(const MzBuildLds& L, int G, int s, MzRng& rng) {
  uint8_t* m = L.g;
  uint16_t* st = L.queue;
  uint16_t* dep = L.dist;  // distance from s in the carved tree (MZ_TREE_DIST)
  int sp = 0;
  st[sp++] = (uint16_t)s;
  dep[s] = 0;
  while (sp > 0) {
    const int top = st[sp - 1], x = top / G, y = top - x * G;
    uint64_t cand = 0;
    int cnt = 0;
    for (int k = 0; k < 4; ++k) {
      int nx = x + 2 * mz_fr(k), ny = y + 2 * mz_fc(k);
      if (nx >= 0 && nx < G && ny >= 0 && ny < G && m[nx * G + ny] == 0) mz_k4_push(cand, cnt, k);
    }
    if (!cnt) { --sp; continue; }
    const int k = mz_k4(cand, (int)rng.below((uint32_t)cnt));
    const int pass = (x + mz_fr(k)) * G + (y + mz_fc(k)), dt = dep[top];
    m[pass] = 1;
    const int nx = x + 2 * mz_fr(k), ny = y + 2 * mz_fc(k);
    m[nx * G + ny] = 1;
    dep[pass] = (uint16_t)(dt + 1);
    dep[nx * G + ny] = (uint16_t)(dt + 2);
    st[sp++] = (uint16_t)(nx * G + ny);
  }
}

// prim&kill marks kept in L.dist: 0 = not a cell, 1 = unmarked, 2 = marked
__device__ inline int mz_pk_nbrs(const uint16_t* mk, int G, int p, uint64_t& out) {
  const int x = p / G, y = p - x * G;
  int cnt = 0;
  out = 0;
  for (int k = 0; k < 4; ++k) {
    int r = x + mz_g2r(k), c = y + mz_g2c(k);
    if (r < 0 || r >= G || c < 0 || c >= G) continue;
    if (mk[r * G + c] == 1) mz_k4_push(out, cnt, r * G + c);
  }
  return cnt;
}

// The restart candidates of prim_and_kill_visit — marked cells with >= 1 unmarked neighbour
// (maze_generation.py:151) — as one bit per cell in L.vis, cell q = (r / 2) * W + c / 2 with
// W = (G - 1) / 2: row-major, the order of the reference's list comprehension. The walk keeps
// the bits current as it marks cells (only the new cell and its marked neighbours can change),
// so a restart picks its candidate from a 125-word bit scan instead of two passes over the grid.
__device__ inline void mz_pk_cand(uint32_t* cb, int G, int p, bool on) {
  const int r = p / G, c = p - r * G, q = (r >> 1) * ((G - 1) >> 1) + (c >> 1);
  if (on) cb[q >> 5] |= 1u << (q & 31);
  else cb[q >> 5] &= ~(1u << (q & 31));
}

// mark p (lane 0) and refresh the candidate bits that marking it can change
__device__ inline void mz_pk_mark(const MzBuildLds& L, int G, int p) {
  uint64_t tmp;
  L.dist[p] = 2;
  mz_pk_cand(L.vis, G, p, mz_pk_nbrs(L.dist, G, p, tmp) > 0);
  const int x = p / G, y = p - x * G;
  for (int k = 0; k < 4; ++k) {
    const int r = x + mz_g2r(k), c = y + mz_g2c(k);
    if (r < 0 || r >= G || c < 0 || c >= G) continue;
    const int n = r * G + c;
    if (L.dist[n] == 2 && mz_pk_nbrs(L.dist, G, n, tmp) == 0) mz_pk_cand(L.vis, G, n, false);
  }
}

__device__ void mz_pk_walk(const MzBuildLds& L, int G, int cur, MzRng& rng) {
  uint64_t nb;
  int cnt;
  while ((cnt = mz_pk_nbrs(L.dist, G, cur, nb)) != 0) {
    const int nx = mz_k4(nb, (int)rng.below((uint32_t)cnt));
    const int cx = cur / G, cy = cur - cx * G, x = nx / G, y = nx - x * G;
    const int pass = (cx + (x - cx) / 2) * G + (cy + (y - cy) / 2), dc = L.queue[cur];
    L.g[pass] = 1;
    L.queue[pass] = (uint16_t)(dc + 1);  // distance from s in the carved tree (MZ_TREE_DIST)
    L.queue[nx] = (uint16_t)(dc + 2);
    cur = nx;
    mz_pk_mark(L, G, cur);
    L.sh[1] -= 1;
  }
}

// wave-cooperative; rng lives in lane 0
__device__ void mz_gen_primkill(const MzBuildLds& L, int G, int s, MzRng& rng) {
  const int lane = threadIdx.x, C = G * G, W = (G - 1) / 2, nw = (W * W + 31) / 32;
  for (int p = lane; p < C; p += 64) {
    const int r = p / G, c = p - r * G;
    const bool cell = (r & 1) && (c & 1) && r < G && c < G;
    L.dist[p] = cell ? 1 : 0;
    if (cell) L.g[p] = 1;
  }
  for (int w = lane; w < nw; w += 64) L.vis[w] = 0u;
  __syncthreads();
  if (lane == 0) {
    L.sh[1] = W * W - 1;  // unmarked count
    L.queue[s] = 0;
    mz_pk_mark(L, G, s);
    mz_pk_walk(L, G, s, rng);
  }
  __syncthreads();
  while (L.sh[1] > 0) {
    int total = 0;
    for (int b = 0; b < nw; b += 64) {
      int pc = b + lane < nw ? __popc(L.vis[b + lane]) : 0;
      for (int o = 32; o > 0; o >>= 1) pc += __shfl_xor(pc, o);
      total += pc;
    }
    int k = 0;
    if (lane == 0) k = (int)rng.below((uint32_t)total);
    k = __shfl(k, 0);
    int chosen = -1;
    for (int b = 0; b < nw && chosen < 0; b += 64) {
      const int w = b + lane;
      const uint32_t v = w < nw ? L.vis[w] : 0u;
      const int pc = __popc(v);
      int inc = pc;  // inclusive prefix sum over the lanes' words
      for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(inc, o);
        if (lane >= o) inc += t;
      }
      const int tot = __shfl(inc, 63);
      if (k < tot) {
        const unsigned long long bal = __ballot(inc > k && inc - pc <= k);
        const int src = __ffsll((long long)bal) - 1;
        int q = 0;
        if (lane == src) {
          uint32_t m = v;
          for (int t = inc - pc; t < k; ++t) m &= m - 1;  // drop the lower candidates
          q = w * 32 + __ffs(m) - 1;
        }
        q = __shfl(q, src);
        chosen = (2 * (q / W) + 1) * G + 2 * (q % W) + 1;
      } else {
        k -= tot;
      }
    }
    __syncthreads();
    if (chosen < 0) break;  // unreachable for a connected cell grid; never walk from -1
    if (lane == 0) mz_pk_walk(L, G, chosen, rng);
    __syncthreads();
  }
}

// find_random_position (maze_generation.py:187-218) on the euclidean G x G grid, from dist =
// the distance of every open square from the start s: the dead end (odd cell, exactly one open
// neighbour, not s) with the largest path length, the first in row-major order on ties
__device__ int mz_goal_scan(const MzBuildLds& L, int G, int s, const uint16_t* dist) {
  const int lane = threadIdx.x, C = G * G;
  uint32_t best = 0;  // (dist << 16) | (0xFFFF - idx); 0 = none
  for (int p = lane; p < C; p += 64) {
    const int r = p / G, c = p - r * G;
    if (!(r & 1) || !(c & 1) || L.g[p] != 1 || p == s || r + 1 >= G || c + 1 >= G) continue;
    const int nb = (L.g[p - G] != 0) + (L.g[p + G] != 0) + (L.g[p - 1] != 0) + (L.g[p + 1] != 0);
    if (nb != 1) continue;
    const uint32_t key = ((uint32_t)(dist[p] + 1) << 16) | (uint32_t)(0xFFFF - p);
    best = key > best ? key : best;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t x = __shfl_xor(best, o);
    best = x > best ? x : best;
  }
  return best ? (int)(0xFFFF - (best & 0xFFFF)) : -1;
}

__device__ int mz_goal_select(const MzBuildLds& L, int G, int s) {
  mz_wave_bfs(L, G, false, s);
  return mz_goal_scan(L, G, s, L.dist);
}

// Distance-to-goal field of a perfect maze without a level-synchronous BFS (MZ_TREE_DIST).
// The Philox generators carve a spanning tree of the open squares rooted at the start s and
// record each square's depth (its distance from s) in L.queue as they carve. In that tree every
// open square's open neighbours are its parent (depth - 1) and its children (depth + 1), so
//   D(x) = dep(x) + dep(goal) - 2 dep(a(x)),  a(x) = x's first ancestor on the goal's root path,
// which is what mz_wave_bfs(L, N, false, goal) computes (a BFS over a tree is its path lengths).
// A BFS costs one wave-synchronous round per level (up to ~3,200 levels at 81 x 81); this costs
// one pass for the parents, one serial walk from the goal to s marking its path (L.vis), and
// ~log2(depth) pointer-jumping passes. Returns false (L.dist untouched except scratch, the caller
// runs the BFS) if the grid is not such a tree (a square without a parent, a walk that does not
// reach s, or no convergence in 32 passes) — never for the generators here.
__device__ bool mz_tree_dist(const MzBuildLds& L, int N, int s, int goal) {
  const int lane = threadIdx.x, C = N * N;
  const uint16_t* dep = L.queue;
  uint16_t* A = L.dist;  // parent, then first ancestor on the goal path, then D
  bool bad = false;
  for (int p = lane; p < C; p += 64) {
    uint16_t a = 0xFFFF;
    if (L.g[p] != 0) {
      a = (uint16_t)p;  // the root points to itself
      if (p != s) {
        const int r = p / N, c = p - r * N, want = (int)dep[p] - 1;
        a = 0xFFFF;
        if (r > 0 && L.g[p - N] != 0 && dep[p - N] == want) a = (uint16_t)(p - N);
        if (r + 1 < N && L.g[p + N] != 0 && dep[p + N] == want) a = (uint16_t)(p + N);
        if (c > 0 && L.g[p - 1] != 0 && dep[p - 1] == want) a = (uint16_t)(p - 1);
        if (c + 1 < N && L.g[p + 1] != 0 && dep[p + 1] == want) a = (uint16_t)(p + 1);
        bad |= a == 0xFFFF;
      }
    }
    A[p] = a;
  }
  for (int i = lane; i < (C + 31) / 32; i += 64) L.vis[i] = 0u;
  if (__any(bad)) return false;
  __syncthreads();
  if (lane == 0) {  // mark the goal's root path
    int x = goal, n = 0;
    for (; n <= C; ++n) {
      L.vis[x >> 5] |= 1u << (x & 31);
      if (x == s) break;
      x = A[x];
      if (x == 0xFFFF) { n = C + 1; break; }
    }
    L.sh[3] = n > C;
  }
  __syncthreads();
  if (L.sh[3]) return false;
  // pointer jumping, in place: A[p] only ever moves up p's root path and never past a marked
  // square, so any interleaving of the lanes' updates converges to a(p) (for an unmarked p;
  // a marked p keeps its parent here and is its own a(p) below)
  bool conv = false;
  for (int it = 0; it < 32 && !conv; ++it) {
    bool ch = false;
    for (int p = lane; p < C; p += 64) {
      const int a = A[p];
      if (a == 0xFFFF || ((L.vis[a >> 5] >> (a & 31)) & 1u)) continue;
      A[p] = A[a];
      ch = true;
    }
    conv = !__any(ch);
    __syncthreads();
  }
  if (!conv) return false;
  const int dg = dep[goal];
  for (int p = lane; p < C; p += 64) {
    if (A[p] == 0xFFFF) continue;
    const int a = ((L.vis[p >> 5] >> (p & 31)) & 1u) ? p : A[p];  // a path square is its own a()
    A[p] = (uint16_t)((int)dep[p] + dg - 2 * (int)dep[a]);
  }
  __syncthreads();
  return true;
}

// Cell word of open cell (r,c) of the final N x N maze: open(r, c) (0 <= r, c < N) and dist(r, c)
// (open squares) describe the maze and its distance-to-goal field.
template <class OPEN, class DIST>
__device__ inline uint32_t mz_cell_word_f(const OPEN& open, const DIST& dist, int N, bool tor,
                                          int r, int c, int gr, int gc) {
  const int M = 2 * N;  // best-dir A* depth 2*min(H,W) (base_maze_env.py:244)
  const uint32_t D = (uint32_t)dist(r, c);
  uint32_t nbm = 0u;
  int code = 4;
  double best = __longlong_as_double(0x7FF0000000000000ll);  // +inf
  for (int k = 0; k < 4; ++k) {
    // get_direction_mask / get_toroidal_direction_mask (maze_handler.py:122-162)
    const int mr = mz_wrap(r + mz_dr(k), N), mc = mz_wrap(c + mz_dc(k), N);
    if (open(mr, mc)) nbm |= 1u << k;
  }
  for (int k = 0; k < 4; ++k) {  // _find_best_next_cell (base_maze_env.py:237-260)
    int nr = r + mz_dr(k), nc = c + mz_dc(k);
    bool valid;
    if (tor) { nr = mz_wrap(nr, N); nc = mz_wrap(nc, N); valid = open(nr, nc); }
    else valid = 0 < nr && nr < N && 0 < nc && nc < N && open(nr, nc);
    if (!valid) continue;
    const int dn = dist(nr, nc);
    const int len = (dn < M ? dn : M) + 1;
    const int manh = abs(nr - gr) + abs(nc - gc);
    const double score = __dadd_rn((double)len, __dmul_rn(0.15, (double)manh));
    if (score < best) { best = score; code = k; }
    if (nr == gr && nc == gc) { code = k; break; }
  }
  return D | ((uint32_t)code << MZ_CELL_CODE_SHIFT) | MZ_CELL_OPEN | (nbm << MZ_CELL_NB_SHIFT);
}

__device__ inline uint32_t mz_cell_word(const MzBuildLds& L, int N, bool tor, int r, int c,
                                        int gr, int gc) {
  return mz_cell_word_f([&](int y, int x) { return L.g[y * N + x] != 0; },
                        [&](int y, int x) { return (int)L.dist[y * N + x]; }, N, tor, r, c, gr, gc);
}

// Writes instance e's tables from a built maze: cell words, the open / visited plane strips
// (mz_common.h; visited = {start}), meta / reset state with set_max_steps. All lanes call.
template <class OPEN, class DIST>
__device__ void mz_build_write(const MzDev& d, int e, int N, bool tor, int sr, int sc, int gr,
                               int gc, const OPEN& open, const DIST& dist) {
  const int lane = threadIdx.x;
  const size_t es = (size_t)e;
  const int P = d.P;
  for (int p = lane; p < P * P; p += 64) {
    const int r = p / P, c = p - r * P;
    const bool op = r < N && c < N && open(r, c);
    d.cells[es * P * P + p] = op ? mz_cell_word_f(open, dist, N, tor, r, c, gr, gc) : 0u;
  }
  for (int k = lane; k < d.NS * P; k += 64) {
    const int st = k / P, R = k - st * P;
    uint32_t o = 0u, v = 0u;
    if (R < N) {
      for (int j = 0; j < 32; ++j) {
        int c = MZ_STRIP_STRIDE * st + j;
        if (tor) c = mz_wrap(c, N);
        else if (c >= N) break;
        if (open(R, c)) o |= 1u << j;
      }
      if (R == sr) v = mz_strip_colmask(st, sc, N, tor);
    }
    *mz_strip_row(d, es, st, R) = make_uint2(o, v);
  }
  if (lane == 0) {
    // set_max_steps: ceil((((H-1)*(W-1)) - 1) * (len / CE)), CE = (H-1)*((W-1)//2) - 1
    const int len = dist(sr, sc) + 1;
    const int ce = (N - 1) * ((N - 1) / 2) - 1;
    const double Lf = __ddiv_rn((double)len, (double)ce);
    const double prod = __dmul_rn((double)((N - 1) * (N - 1) - 1), Lf);
    int maxs = (int)ceil(prod);
    if (maxs > 65535) maxs = 65535;
    d.meta0[e] = (uint32_t)N | ((uint32_t)N << 8) | ((uint32_t)sr << 16) | ((uint32_t)sc << 24);
    d.meta1[e] = (uint32_t)gr | ((uint32_t)gc << 8) | ((uint32_t)maxs << 16);
    d.posw[e] = (uint32_t)sr | ((uint32_t)sc << 8);
    d.stw[e] = 0u;
    d.last_term[e] = 0;
    // curw = cells word at start, from LDS (no read-back of global stores inside the launch)
    d.curw[e] = mz_cell_word_f(open, dist, N, tor, sr, sc, gr, gc);
  }
  __syncthreads();
}

// ---- Cell-space build of a Philox euclidean maze (MZ_CELL_BUILD) ---------------------------
// A perfect maze lives on its odd squares: cell q = (r >> 1) * W + (c >> 1), W = (N - 1) / 2.
// The generators below carve the same spanning tree as mz_gen_* (the same Philox draws over the
// same candidate lists in the same order, the same swap-remove frontier), but keep per cell only
// the passages to its right and lower neighbours, two bit sets, the frontier / stack list, the
// carve depth and then the distance field in place of the list: ~5.3 B per cell (8.5 KB at 81 x 81)
// where the square grid needs ~5.1 B per square (35 KB), so 18 builds share a CU instead of 4
// (each build is a serial lane-0 chain of LDS round trips: throughput is the number of builds in
// flight).
#ifndef MZ_CELL_BUILD
#define MZ_CELL_BUILD 1
#endif
// Timing probes of mz_build_cells (wrong tables — never in the product build): 1 no cell words /
// planes, 2 no distance field, 4 no goal scan
#ifndef MZ_GPROBE
#define MZ_GPROBE 0
#endif

struct MzCellLds {
  uint8_t* pas;    // [Q] bit 0: passage to the right neighbour, bit 1: to the one below
  uint32_t* b0;    // [QW] in maze (r-prim, dfs) / marked (prim&kill)
  uint32_t* b1;    // [QW] in frontier (r-prim) / restart candidate (prim&kill), then goal path
  uint16_t* list;  // [Q] frontier (r-prim) / stack (dfs)
  uint16_t* dep;   // [Q] carve depth: distance from the start in squares (BFS fallback: queue)
  uint16_t* A;     // [Q] = list (dead after the carve): parent, first goal-path ancestor, then
                   //     the distance to the goal
  int* sh;
  int W, Q;
  uint32_t mW;     // ceil(2^18 / W): q / W == (q * mW) >> 18 for every cell q (q < 2^12, W <= 64)
  int cap;         // list capacity (Q; the lite r-prim regions: mz_lite_cap)
};

// MZ_CELL_ALIAS 0: the distance array separate from the list (A/B builds)
#ifndef MZ_CELL_ALIAS
#define MZ_CELL_ALIAS 1
#endif
__host__ __device__ inline size_t mz_cell_lds_bytes(int P) {
  const size_t W = (size_t)P / 2, Q = W * W, QW = (Q + 31) / 32;
  return 64 + mz_align16(Q) + 2 * mz_align16(4 * QW) + (MZ_CELL_ALIAS ? 2 : 3) * mz_align16(2 * Q);
}

__device__ inline MzCellLds mz_cell_lds(uint8_t* base, int P, int N) {
  const size_t Wp = (size_t)P / 2, Qp = Wp * Wp, QW = (Qp + 31) / 32;
  MzCellLds L;
  L.sh = reinterpret_cast<int*>(base);
  size_t off = 64;
  L.pas = base + off; off += mz_align16(Qp);
  L.b0 = reinterpret_cast<uint32_t*>(base + off); off += mz_align16(4 * QW);
  L.b1 = reinterpret_cast<uint32_t*>(base + off); off += mz_align16(4 * QW);
  L.list = reinterpret_cast<uint16_t*>(base + off); off += mz_align16(2 * Qp);
  L.dep = reinterpret_cast<uint16_t*>(base + off); off += mz_align16(2 * Qp);
  L.A = MZ_CELL_ALIAS ? L.list : reinterpret_cast<uint16_t*>(base + off);
  L.W = (N - 1) / 2;
  L.Q = L.W * L.W;
  L.mW = ((1u << 18) + (uint32_t)L.W - 1u) / (uint32_t)(L.W > 0 ? L.W : 1);
  L.cap = L.Q;
  return L;
}

// Bit-set and passage updates as LDS atomics whose result is unused (ds_or_b32 / ds_and_b32 with
// no return): the carve is one serial chain per maze, and a read-modify-write made it wait an LDS
// round trip per update; a wave's LDS operations execute in order, so later reads see them.
__device__ inline bool cs_bit(const uint32_t* b, int q) { return (b[q >> 5] >> (q & 31)) & 1u; }
__device__ inline void cs_set(uint32_t* b, int q) { atomicOr(&b[q >> 5], 1u << (q & 31)); }
__device__ inline void cs_clr(uint32_t* b, int q) { atomicAnd(&b[q >> 5], ~(1u << (q & 31))); }

// neighbour cell of q in direction k — 0 up, 1 down, 2 left, 3 right (the generators' order
// (-2,0),(2,0),(0,-2),(0,2), maze_generation.py:72) — or -1 outside the grid
// (the carves call this every step: the row by a multiply-shift, not a division by the
// runtime W — ~25 dependent instructions per call on the carve's serial chain)
__device__ inline int cs_row(int q, uint32_t mW) { return (int)(((uint32_t)q * mW) >> 18); }
__device__ inline int cs_nb(int q, int k, int W, uint32_t mW) {
  const int r = cs_row(q, mW), c = q - r * W;
  if (k == 0) return r > 0 ? q - W : -1;
  if (k == 1) return r + 1 < W ? q + W : -1;
  if (k == 2) return c > 0 ? q - 1 : -1;
  return c + 1 < W ? q + 1 : -1;
}
// open the passage from q in direction k (an atomic OR on the byte's 32-bit word: pas is 16-B
// aligned)
__device__ inline void cs_link(const MzCellLds& L, int q, int k) {
  const int c = k == 0 ? q - L.W : (k == 2 ? q - 1 : q);
  const uint32_t v = k < 2 ? 2u : 1u;
  atomicOr(reinterpret_cast<uint32_t*>(L.pas) + (c >> 2), v << (8 * (c & 3)));
}
// whether the passage from q in direction k is open (the neighbour exists)
__device__ inline bool cs_open_dir(const MzCellLds& L, int q, int k) {
  const int r = cs_row(q, L.mW), c = q - r * L.W;
  if (k == 0) return r > 0 && (L.pas[q - L.W] & 2);
  if (k == 1) return (L.pas[q] & 2) != 0;
  if (k == 2) return c > 0 && (L.pas[q - 1] & 1);
  return (L.pas[q] & 1) != 0;
}

// random_prim_visit (maze_generation.py:59-99), lane 0; as mz_gen_rprim
__device__ void mz_cs_rprim(const MzCellLds& L, int s, MzRng& rng) {
  const int W = L.W;
  int nf = 0;
  cs_set(L.b0, s);
  L.dep[s] = 0;
  for (int k = 0; k < 4; ++k) {
    const int j = cs_nb(s, k, W, L.mW);
    if (j >= 0) { L.list[nf++] = (uint16_t)j; cs_set(L.b1, j); }
  }
  while (nf > 0) {
    const int i = (int)rng.below((uint32_t)nf);
    const int f = L.list[i];
    L.list[i] = L.list[--nf];
    // the neighbours' in-maze / frontier words and depths, all loaded before any is used (one
    // LDS round trip); this step changes only f's bits and depth, and f is none of them
    int j[4], dp[4];
    uint32_t w0[4], w1[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      j[k] = cs_nb(f, k, W, L.mW);
      const int jj = j[k] >= 0 ? j[k] : f;
      w0[k] = L.b0[jj >> 5] >> (jj & 31);
      w1[k] = L.b1[jj >> 5] >> (jj & 31);
      dp[k] = L.dep[jj];
    }
    uint64_t nb = 0;  // in-maze neighbours: cell | direction from f << 12
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (j[k] >= 0 && (w0[k] & 1u)) mz_k4_push(nb, cnt, j[k] | (k << 12));
    if (cnt) {
      const int v = mz_k4(nb, (int)rng.below((uint32_t)cnt)), kk = v >> 12;
      cs_set(L.b0, f);
      cs_link(L, f, kk);
      const int dn = kk == 0 ? dp[0] : (kk == 1 ? dp[1] : (kk == 2 ? dp[2] : dp[3]));
      L.dep[f] = (uint16_t)(dn + 2);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (j[k] >= 0 && !(w0[k] & 1u) && !(w1[k] & 1u)) {
          L.list[nf++] = (uint16_t)j[k];
          cs_set(L.b1, j[k]);
        }
      }
    }
  }
}

// deept_first_visit (maze_generation.py:101-128), lane 0; as mz_gen_dfs. Its direction order
// (0,-1),(0,1),(-1,0),(1,0) is left, right, up, down.
__device__ void mz_cs_dfs(const MzCellLds& L, int s, MzRng& rng) {
  const int W = L.W;
  int sp = 0;
  L.list[sp++] = (uint16_t)s;
  cs_set(L.b0, s);
  L.dep[s] = 0;
  // the stack top and its depth stay in registers while the walk advances (a push makes the new
  // cell the top at depth + 2); only a backtrack reads them back
  int top = s, dtop = 0;
  while (sp > 0) {
    int j[4];
    uint32_t w0[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // left, right, up, down
      j[k] = cs_nb(top, k == 0 ? 2 : (k == 1 ? 3 : k - 2), W, L.mW);
      const int jj = j[k] >= 0 ? j[k] : top;
      w0[k] = L.b0[jj >> 5] >> (jj & 31);
    }
    uint64_t cand = 0;
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (j[k] >= 0 && !(w0[k] & 1u)) mz_k4_push(cand, cnt, k);
    if (!cnt) {
      if (--sp > 0) {
        top = L.list[sp - 1];
        dtop = L.dep[top];
      }
      continue;
    }
    const int k = mz_k4(cand, (int)rng.below((uint32_t)cnt));
    const int dir = k == 0 ? 2 : (k == 1 ? 3 : k - 2);
    const int jn = k == 0 ? j[0] : (k == 1 ? j[1] : (k == 2 ? j[2] : j[3]));
    cs_link(L, top, dir);
    cs_set(L.b0, jn);
    dtop += 2;
    L.dep[jn] = (uint16_t)dtop;
    L.list[sp++] = (uint16_t)jn;
    top = jn;
  }
}

// prim_and_kill_visit (maze_generation.py:130-185); as mz_gen_primkill: b0 = marked, b1 = the
// restart candidates (marked cells with an unmarked neighbour), kept current by the walk
__device__ inline int mz_cs_pk_nbrs(const MzCellLds& L, int p, uint64_t& out) {
  int cnt = 0;
  out = 0;
  for (int k = 0; k < 4; ++k) {
    const int j = cs_nb(p, k, L.W, L.mW);
    if (j >= 0 && !cs_bit(L.b0, j)) mz_k4_push(out, cnt, j | (k << 12));
  }
  return cnt;
}
__device__ inline void mz_cs_pk_mark(const MzCellLds& L, int p) {
  uint64_t tmp;
  cs_set(L.b0, p);
  if (mz_cs_pk_nbrs(L, p, tmp) > 0) cs_set(L.b1, p); else cs_clr(L.b1, p);
  for (int k = 0; k < 4; ++k) {
    const int n = cs_nb(p, k, L.W, L.mW);
    if (n >= 0 && cs_bit(L.b0, n) && mz_cs_pk_nbrs(L, n, tmp) == 0) cs_clr(L.b1, n);
  }
}
// mz_cs_pk_mark for the walk, from the marked bits of the 5 x 5 cells around p (cells outside the
// grid read as marked: never an unmarked neighbour), loaded together — one LDS round trip where
// the mark's neighbour-of-neighbour scans made several dependent ones. Returns p's unmarked
// neighbours (what the walk's next mz_cs_pk_nbrs(p) would read: the mark changes p's bit only).
__device__ inline int mz_cs_pk_mark_w(const MzCellLds& L, int p, uint64_t& out) {
  const int W = L.W, r = cs_row(p, L.mW), c = p - r * W;
  uint32_t rows[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int rr = r - 2 + i;
    if (rr < 0 || rr >= W) { rows[i] = 0x1Fu; continue; }
    const int lo = max(c - 2, 0), hi = min(c + 2, W - 1);
    const int qlo = rr * W + lo, qhi = rr * W + hi;
    const uint64_t cat = ((uint64_t)L.b0[qhi >> 5] << 32) | L.b0[qlo >> 5];
    const uint32_t len = (uint32_t)(hi - lo + 1), at = (uint32_t)(lo - (c - 2));
    const uint32_t v = (uint32_t)(cat >> (qlo & 31)) & ((1u << len) - 1u);
    rows[i] = (v << at) | (0x1Fu & ~(((1u << len) - 1u) << at));
  }
  cs_set(L.b0, p);
  rows[2] |= 1u << 2;
  auto mk = [&](int i, int j) -> bool { return (rows[i] >> j) & 1u; };
  auto free_nbrs = [&](int i, int j) -> int {
    return (int)!mk(i - 1, j) + (int)!mk(i + 1, j) + (int)!mk(i, j - 1) + (int)!mk(i, j + 1);
  };
  int cnt = 0;
  out = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {  // up, down, left, right
    const int i = 2 + (k == 0 ? -1 : (k == 1 ? 1 : 0)), j = 2 + (k == 2 ? -1 : (k == 3 ? 1 : 0));
    if (!mk(i, j)) mz_k4_push(out, cnt, cs_nb(p, k, W, L.mW) | (k << 12));
  }
  if (cnt > 0) cs_set(L.b1, p); else cs_clr(L.b1, p);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int i = 2 + (k == 0 ? -1 : (k == 1 ? 1 : 0)), j = 2 + (k == 2 ? -1 : (k == 3 ? 1 : 0));
    const int n = cs_nb(p, k, W, L.mW);
    if (n >= 0 && mk(i, j) && free_nbrs(i, j) == 0) cs_clr(L.b1, n);
  }
  return cnt;
}
// the walk: its depth and the unmarked count stay in registers, the next step's neighbour list
// comes from the mark
__device__ void mz_cs_pk_walk(const MzCellLds& L, int cur, MzRng& rng) {
  uint64_t nb;
  int cnt = mz_cs_pk_nbrs(L, cur, nb);
  if (!cnt) return;
  int dcur = L.dep[cur], left = L.sh[1];
  while (cnt) {
    const int v = mz_k4(nb, (int)rng.below((uint32_t)cnt)), nx = v & 0xFFF;
    cs_link(L, cur, v >> 12);
    dcur += 2;
    L.dep[nx] = (uint16_t)dcur;
    cur = nx;
    cnt = mz_cs_pk_mark_w(L, cur, nb);
    --left;
  }
  L.sh[1] = left;
}
__device__ void mz_cs_primkill(const MzCellLds& L, int s, MzRng& rng) {
  const int lane = threadIdx.x, nw = (L.Q + 31) / 32;
  if (lane == 0) {
    L.sh[1] = L.Q - 1;  // unmarked count
    L.dep[s] = 0;
    mz_cs_pk_mark(L, s);
    mz_cs_pk_walk(L, s, rng);
  }
  __syncthreads();
  while (L.sh[1] > 0) {
    int total = 0;
    for (int b = 0; b < nw; b += 64) {
      int pc = b + lane < nw ? __popc(L.b1[b + lane]) : 0;
      for (int o = 32; o > 0; o >>= 1) pc += __shfl_xor(pc, o);
      total += pc;
    }
    int k = 0;
    if (lane == 0) k = (int)rng.below((uint32_t)total);
    k = __shfl(k, 0);
    int chosen = -1;
    for (int b = 0; b < nw && chosen < 0; b += 64) {
      const int w = b + lane;
      const uint32_t v = w < nw ? L.b1[w] : 0u;
      const int pc = __popc(v);
      int inc = pc;  // inclusive prefix sum over the lanes' words
      for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(inc, o);
        if (lane >= o) inc += t;
      }
      const int tot = __shfl(inc, 63);
      if (k < tot) {
        const unsigned long long bal = __ballot(inc > k && inc - pc <= k);
        const int src = __ffsll((long long)bal) - 1;
        int q = 0;
        if (lane == src) {
          uint32_t m = v;
          for (int t = inc - pc; t < k; ++t) m &= m - 1;  // drop the lower candidates
          q = w * 32 + __ffs(m) - 1;
        }
        chosen = __shfl(q, src);
      } else {
        k -= tot;
      }
    }
    __syncthreads();
    if (chosen < 0) break;  // unreachable for a connected cell grid; never walk from -1
    if (lane == 0) mz_cs_pk_walk(L, chosen, rng);
    __syncthreads();
  }
}

// find_random_position (maze_generation.py:187-218) from the carve depths: as mz_goal_scan
// (same key: path length, then the smallest square index); returns the goal cell or -1
__device__ int mz_cs_goal(const MzCellLds& L, int N, int s) {
  const int lane = threadIdx.x, W = L.W;
  uint32_t best = 0;
  for (int q = lane; q < L.Q; q += 64) {
    if (q == s) continue;
    int nb = 0;
    for (int k = 0; k < 4; ++k) nb += cs_open_dir(L, q, k);
    if (nb != 1) continue;
    const int r = cs_row(q, L.mW), c = q - r * W, p = (2 * r + 1) * N + 2 * c + 1;
    const uint32_t key = ((uint32_t)(L.dep[q] + 1) << 16) | (uint32_t)(0xFFFF - p);
    best = key > best ? key : best;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t x = __shfl_xor(best, o);
    best = x > best ? x : best;
  }
  if (!best) return -1;
  const int p = 0xFFFF - (int)(best & 0xFFFF), r = p / N, c = p - r * N;
  return (r >> 1) * W + (c >> 1);
}

// Distance to the goal cell of every cell, in squares, into L.A: mz_tree_dist in cell space
// (parents are the neighbours across an open passage at depth - 2); a cell-space BFS when the
// tree walk fails (never for these generators) or MZ_TREE_DIST is 0. Returns true when the tree
// walk ran: L.b1 then holds the goal's root path in the start-rooted carve tree, i.e. the
// solution path's cells (the BFS leaves its visited bits there instead).
__device__ bool mz_cs_dist(const MzCellLds& L, int s, int goal) {
  const int lane = threadIdx.x, Q = L.Q, W = L.W;
  bool ok = MZ_TREE_DIST;
  if (ok) {
    bool bad = false;
    for (int q = lane; q < Q; q += 64) {
      int a = q;
      if (q != s) {
        const int want = (int)L.dep[q] - 2;
        a = 0xFFFF;
        for (int k = 0; k < 4; ++k)
          if (cs_open_dir(L, q, k)) {
            const int n = cs_nb(q, k, W, L.mW);
            if ((int)L.dep[n] == want) a = n;
          }
        bad |= a == 0xFFFF;
      }
      L.A[q] = (uint16_t)a;
    }
    for (int i = lane; i < (Q + 31) / 32; i += 64) L.b1[i] = 0u;
    ok = !__any(bad);
    __syncthreads();
  }
  if (ok) {
    if (lane == 0) {  // mark the goal's root path
      int x = goal, n = 0;
      for (; n <= Q; ++n) {
        cs_set(L.b1, x);
        if (x == s) break;
        x = L.A[x];
      }
      L.sh[3] = n > Q;
    }
    __syncthreads();
    ok = !L.sh[3];
  }
  if (ok) {
    bool conv = false;
    for (int it = 0; it < 32 && !conv; ++it) {
      bool ch = false;
      for (int q = lane; q < Q; q += 64) {
        const int a = L.A[q];
        if (cs_bit(L.b1, a)) continue;
        L.A[q] = L.A[a];
        ch = true;
      }
      conv = !__any(ch);
      __syncthreads();
    }
    ok = conv;
  }
  if (ok) {
    const int dg = L.dep[goal];
    for (int q = lane; q < Q; q += 64) {
      const int a = cs_bit(L.b1, q) ? q : L.A[q];
      L.A[q] = (uint16_t)((int)L.dep[q] + dg - 2 * (int)L.dep[a]);
    }
    __syncthreads();
    return true;
  }
  // level-synchronous BFS over the cells from the goal (distances in squares; the carve depths
  // are not needed any more: their array is the queue)
  uint16_t* queue = L.dep;
  for (int q = lane; q < Q; q += 64) L.A[q] = 0xFFFF;
  for (int i = lane; i < (Q + 31) / 32; i += 64) L.b1[i] = 0u;
  __syncthreads();
  if (lane == 0) {
    L.A[goal] = 0;
    queue[0] = (uint16_t)goal;
    cs_set(L.b1, goal);
    L.sh[0] = 1;
  }
  __syncthreads();
  int head = 0, tail = 1;
  while (head < tail) {
    for (int base = head; base < tail; base += 64) {
      const int i = base + lane;
      if (i < tail) {
        const int v = queue[i], dv = L.A[v];
        for (int k = 0; k < 4; ++k) {
          if (!cs_open_dir(L, v, k)) continue;
          const int n = cs_nb(v, k, W, L.mW);
          const uint32_t bit = 1u << (n & 31);
          if (atomicOr(&L.b1[n >> 5], bit) & bit) continue;
          L.A[n] = (uint16_t)(dv + 2);
          queue[atomicAdd(&L.sh[0], 1)] = (uint16_t)n;
        }
      }
    }
    __syncthreads();
    head = tail;
    tail = L.sh[0];
    __syncthreads();
  }
  return false;
}

// Toroidal mazes (gen_maze_no_border, maze_generation.py:37-56): generated in cell space on the
// (N + 2)^2 bordered grid, the goal picked there, then cropped to N x N — where the wrap joins
// the first and last rows / columns, so the maze has cycles and its distance field is a BFS. That
// BFS runs bit-parallel over row masks (one 128-bit row of open squares per lane, a level = a
// shift / or / and-not of the frontier rows) in the region the generator's lists used, after the
// passages: 20 KB of LDS at 79 x 79 instead of the square grid's 34 KB.
typedef unsigned __int128 mz_u128;

__device__ inline mz_u128 mz_row_rotl(mz_u128 v, int N, mz_u128 mask) {  // column x -> x + 1 mod N
  return ((v << 1) & mask) | ((v >> (N - 1)) & 1u);
}
__device__ inline mz_u128 mz_row_rotr(mz_u128 v, int N) {  // column x -> x - 1 mod N
  return (v >> 1) | ((v & 1u) << (N - 1));
}

__host__ __device__ inline size_t mz_torus_lds_bytes(int P) {
  const size_t Wp = (size_t)(P + 2) / 2, Qp = Wp * Wp;
  const size_t bfs = 64 + mz_align16(Qp) + mz_align16(2 * (size_t)P * P) + 4 * 16 * (size_t)P;
  const size_t gen = mz_cell_lds_bytes(P + 2);
  return gen > bfs ? gen : bfs;
}

// Generation + tables of a Philox maze in cell space (lds >= mz_cell_lds_bytes(P), toroidal:
// mz_torus_lds_bytes(P)).
// cell-space LDS state of a new build: no passages, empty bit sets (wave-wide)
__device__ inline void mz_cells_clear(const MzCellLds& L) {
  const int lane = threadIdx.x;
  for (int q = lane; q < L.Q; q += 64) L.pas[q] = 0;
  for (int i = lane; i < (L.Q + 31) / 32; i += 64) { L.b0[i] = 0u; L.b1[i] = 0u; }
}

__device__ __forceinline__ void mz_cells_finish(const MzDev& d, int e, const MzCellLds& L, int N,
                                                bool tor);

// Tables of instance e (cell words, plane strips, meta / reset state) from a euclidean cell-space
// maze in LDS: passages L.pas, distances to the goal L.A (squares), start / goal cells s / goal.
__device__ __forceinline__ void mz_cells_tables(const MzDev& d, int e, const MzCellLds& L, int N,
                                                int s, int goal) {
  const int W = L.W;
  auto open_g = [&](int r, int c) -> bool {
    const bool ro = r & 1, co = c & 1;
    if (ro && co) return true;  // every cell is in the tree
    if (!ro && !co) return false;
    if (ro) return c > 0 && c < N - 1 && (L.pas[(r >> 1) * W + ((c - 1) >> 1)] & 1);
    return r > 0 && r < N - 1 && (L.pas[((r - 1) >> 1) * W + (c >> 1)] & 2);
  };
  auto dist = [&](int r, int c) -> int {  // open squares: a passage is one step from its nearer cell
    if ((r & 1) && (c & 1)) return L.A[(r >> 1) * W + (c >> 1)];
    const int q = (r & 1) ? (r >> 1) * W + ((c - 1) >> 1) : ((r - 1) >> 1) * W + (c >> 1);
    const int q2 = (r & 1) ? q + 1 : q + W;
    return min((int)L.A[q], (int)L.A[q2]) + 1;
  };
  const int sr = 2 * (s / W) + 1, sc = 2 * (s % W) + 1;
  const int gr = 2 * (goal / W) + 1, gc = 2 * (goal % W) + 1;
  mz_build_write(d, e, N, false, sr, sc, gr, gc, open_g, dist);
}

// A carved euclidean cell-space maze as a best-of-C candidate (mz_screen.h): goal and distance
// field as mz_cells_finish, then only the compact form leaves LDS — no cell words or planes; the
// selected candidate's tables are written from it afterwards (k_cand_expand).
__device__ __forceinline__ void mz_cells_compact(const MzCompact& cc, int t, const MzCellLds& L,
                                                 int N) {
  const int lane = threadIdx.x;
  const int s = L.sh[2];
  int goal = mz_cs_goal(L, N, s);
  if (goal < 0) goal = s;  // unreachable for W >= 2 (a spanning tree has >= 2 leaves)
  const bool sol = mz_cs_dist(L, s, goal);
  const int Q = L.Q;
  uint32_t* gp = reinterpret_cast<uint32_t*>(cc.pas + (size_t)t * cc.Qp);
  uint32_t* ga = reinterpret_cast<uint32_t*>(cc.dist + (size_t)t * cc.Qp);
  const uint32_t* lp = reinterpret_cast<const uint32_t*>(L.pas);
  const uint32_t* la = reinterpret_cast<const uint32_t*>(L.A);
  for (int i = lane; i < (Q + 3) / 4; i += 64) gp[i] = lp[i];
  for (int i = lane; i < (Q + 1) / 2; i += 64) ga[i] = la[i];
  for (int i = lane; i < (Q + 31) / 32; i += 64) cc.sol[(size_t)t * cc.QWp + i] = L.b1[i];
  if (lane == 0)
    cc.meta[t] = (uint32_t)N | (sol ? 0u : MZ_CMETA_NOSOL) | ((uint32_t)s << 8) | ((uint32_t)goal << 20);
  __syncthreads();
}

// the carve of mz_build_cells (wave-wide): passages, carve depths and the start cell (L.sh[2])
__device__ __forceinline__ void mz_carve_cells(const MzCellLds& L, int algo, uint64_t seed) {
  const int lane = threadIdx.x;
  const int W = L.W;
  mz_cells_clear(L);
  __syncthreads();
  MzRng rng{seed, 0ull, {0u, 0u, 0u, 0u}};
  if (lane == 0) {
    // start = (randrange(1, G-1, 2), randrange(1, G-1, 2)) (maze_generation.py:21)
    const int a = (int)rng.below((uint32_t)W), b = (int)rng.below((uint32_t)W);
    L.sh[2] = a * W + b;
    if (algo == MZ_ALGO_RPRIM_DEV) mz_cs_rprim(L, a * W + b, rng);
    else if (algo == MZ_ALGO_DFS_DEV) mz_cs_dfs(L, a * W + b, rng);
  }
  __syncthreads();
  if (algo != MZ_ALGO_RPRIM_DEV && algo != MZ_ALGO_DFS_DEV) mz_cs_primkill(L, L.sh[2], rng);
  __syncthreads();
}

__device__ __forceinline__ void mz_build_cells(const MzDev& d, int e, int algo, uint64_t seed, int N,
                                               bool tor, uint8_t* lds) {
  const int G = tor ? N + 2 : N;
  const MzCellLds L = mz_cell_lds(lds, tor ? d.P + 2 : d.P, G);
  mz_carve_cells(L, algo, seed);
  mz_cells_finish(d, e, L, N, tor);
}

// Philox r-prim / dfs builds of up to MZ_PACK mazes of one size and algorithm per wave
// (euclidean): maze m's carve runs on lane 16 m over its own LDS region (`stride` bytes apart),
// the MZ_PACK carves in lockstep — an r-prim carve is exactly Q - 1 iterations of the same
// instructions (every cell but the start enters the frontier once; two draws per iteration, one
// Philox word each), a dfs carve exactly 2 Q - 1 (each cell pushed and popped once; a push or a
// backtrack per iteration) — so the wave issues each instruction once for all of them, where one
// carve per wave left the SIMDs issuing one-lane instructions for ~18 waves per CU. Goal,
// distance field and tables then run wave-wide, maze after maze. The same Philox draws in the
// same order: the same mazes as mz_build_cells.
#ifndef MZ_PACK
#define MZ_PACK 4
#endif
// e / seed: lane l holds those of maze l >> 4 (lanes of mazes >= nm: unused)
// the carves of mz_build_cells_packed (P: the pitch the LDS regions are laid out for)
__device__ __forceinline__ void mz_carve_packed(int P, uint64_t seed, int nm, int N, int algo,
                                                uint8_t* lds, size_t stride) {
  const int lane = threadIdx.x, m = lane >> 4;
  for (int k = 0; k < nm; ++k) mz_cells_clear(mz_cell_lds(lds + k * stride, P, N));
  __syncthreads();
  if ((lane & 15) == 0 && m < nm) {
    const MzCellLds L = mz_cell_lds(lds + m * stride, P, N);
    const int W = L.W;
    MzRng rng{seed, 0ull, {0u, 0u, 0u, 0u}};
    const int a = (int)rng.below((uint32_t)W), b = (int)rng.below((uint32_t)W);
    L.sh[2] = a * W + b;
    if (algo == MZ_ALGO_RPRIM_DEV) mz_cs_rprim(L, a * W + b, rng);
    else mz_cs_dfs(L, a * W + b, rng);
  }
  __syncthreads();
}

// ---- Lite r-prim candidates (k_cand_compact_lite): more carves in flight per CU ------------
// A carve is one serial chain of LDS round trips per maze, so a CU's build throughput is the
// number of carves its LDS holds. The lite region keeps only what the carve itself needs: the
// passages with each cell's parent direction (pas bits 2-3: toward the neighbour it joined), the
// two bit sets, and a frontier list capped at mz_lite_cap cells (random Prim's frontier stays far
// below: max 199 over 300 simulated 40 x 40 carves, 319 at 63 x 63) — ~2.9 KB at 81 x 81 instead of
// 8.5 KB: no carve depths (the depths come afterwards from the parent directions by pointer
// jumping, in a per-wave scratch the finish uses maze after maze). The same Philox draws over the
// same frontier order: the same mazes as mz_cs_rprim. A frontier that would pass the cap ends the
// carve and flags the candidate (cmeta MZ_CMETA_NOSOL): the screen declines it and the group is
// rebuilt in full for the order-exact kernel (k_cand_rebuild).
// (dfs: the stack can hold every cell — a dfs region keeps the full list, ~5.3 KB at 81 x 81)
__host__ __device__ inline int mz_lite_cap(int P, int algo = MZ_ALGO_RPRIM_DEV) {
  const int Qp = (P / 2) * (P / 2);
  if (algo == MZ_ALGO_DFS_DEV) return (Qp + 15) & ~15;
  int cap = Qp / 4 > 128 ? Qp / 4 : 128;
  cap = cap < Qp ? cap : Qp;
  return (cap + 15) & ~15;
}
__host__ __device__ inline size_t mz_lite_lds_bytes(int P, int algo = MZ_ALGO_RPRIM_DEV) {
  const size_t Qp = (size_t)(P / 2) * (P / 2), QW = (Qp + 31) / 32;
  return 64 + mz_align16(Qp) + 2 * mz_align16(4 * QW) + mz_align16(2 * (size_t)mz_lite_cap(P, algo));
}
// the per-wave finish scratch: depth words [Qp] (u32) + distances [Qp] (u16)
__host__ __device__ inline size_t mz_lite_scratch_bytes(int P) {
  const size_t Qp = (size_t)(P / 2) * (P / 2);
  return mz_align16(4 * Qp) + mz_align16(2 * Qp);
}
__device__ inline MzCellLds mz_lite_lds(uint8_t* base, int P, int N, int algo = MZ_ALGO_RPRIM_DEV) {
  const size_t Wp = (size_t)P / 2, Qp = Wp * Wp, QW = (Qp + 31) / 32;
  MzCellLds L;
  L.sh = reinterpret_cast<int*>(base);
  size_t off = 64;
  L.pas = base + off; off += mz_align16(Qp);
  L.b0 = reinterpret_cast<uint32_t*>(base + off); off += mz_align16(4 * QW);
  L.b1 = reinterpret_cast<uint32_t*>(base + off); off += mz_align16(4 * QW);
  L.list = reinterpret_cast<uint16_t*>(base + off);
  L.dep = nullptr;
  L.A = nullptr;
  L.W = (N - 1) / 2;
  L.Q = L.W * L.W;
  L.mW = ((1u << 18) + (uint32_t)L.W - 1u) / (uint32_t)(L.W > 0 ? L.W : 1);
  L.cap = mz_lite_cap(P, algo);
  return L;
}

// random_prim_visit (maze_generation.py:59-99) as mz_cs_rprim, one lane, without carve depths:
// cell f records the direction of the neighbour it joins (pas bits 2-3)
__device__ void mz_lite_rprim(const MzCellLds& L, int s, MzRng& rng) {
  const int W = L.W;
  int nf = 0;
  cs_set(L.b0, s);
  for (int k = 0; k < 4; ++k) {
    const int j = cs_nb(s, k, W, L.mW);
    if (j >= 0) { L.list[nf++] = (uint16_t)j; cs_set(L.b1, j); }
  }
  uint32_t* pw = reinterpret_cast<uint32_t*>(L.pas);
  while (nf > 0) {
    const int i = (int)rng.below((uint32_t)nf);
    const int f = L.list[i];
    L.list[i] = L.list[--nf];
    int j[4];
    uint32_t w0[4], w1[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      j[k] = cs_nb(f, k, W, L.mW);
      const int jj = j[k] >= 0 ? j[k] : f;
      w0[k] = L.b0[jj >> 5] >> (jj & 31);
      w1[k] = L.b1[jj >> 5] >> (jj & 31);
    }
    uint64_t nb = 0;
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (j[k] >= 0 && (w0[k] & 1u)) mz_k4_push(nb, cnt, j[k] | (k << 12));
    if (cnt) {
      const int v = mz_k4(nb, (int)rng.below((uint32_t)cnt)), kk = v >> 12;
      cs_set(L.b0, f);
      cs_link(L, f, kk);
      atomicOr(pw + (f >> 2), (uint32_t)(kk << 2) << (8 * (f & 3)));
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (j[k] >= 0 && !(w0[k] & 1u) && !(w1[k] & 1u)) {
          if (nf == L.cap) { L.sh[4] = 1; nf = 0; break; }  // past the cap: flagged, abandoned
          L.list[nf++] = (uint16_t)j[k];
          cs_set(L.b1, j[k]);
        }
      }
    }
  }
}

// deept_first_visit (maze_generation.py:101-128) as mz_cs_dfs, one lane, without carve depths:
// a pushed cell records the direction back to the cell it was carved from (pas bits 2-3)
__device__ void mz_lite_dfs(const MzCellLds& L, int s, MzRng& rng) {
  const int W = L.W;
  int sp = 0;
  L.list[sp++] = (uint16_t)s;
  cs_set(L.b0, s);
  uint32_t* pw = reinterpret_cast<uint32_t*>(L.pas);
  int top = s;
  while (sp > 0) {
    int j[4];
    uint32_t w0[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // left, right, up, down
      j[k] = cs_nb(top, k == 0 ? 2 : (k == 1 ? 3 : k - 2), W, L.mW);
      const int jj = j[k] >= 0 ? j[k] : top;
      w0[k] = L.b0[jj >> 5] >> (jj & 31);
    }
    uint64_t cand = 0;
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (j[k] >= 0 && !(w0[k] & 1u)) mz_k4_push(cand, cnt, k);
    if (!cnt) {
      if (--sp > 0) top = L.list[sp - 1];
      continue;
    }
    const int k = mz_k4(cand, (int)rng.below((uint32_t)cnt));
    const int dir = k == 0 ? 2 : (k == 1 ? 3 : k - 2);
    const int jn = k == 0 ? j[0] : (k == 1 ? j[1] : (k == 2 ? j[2] : j[3]));
    cs_link(L, top, dir);
    cs_set(L.b0, jn);
    atomicOr(pw + (jn >> 2), (uint32_t)((dir ^ 1) << 2) << (8 * (jn & 3)));
    L.list[sp++] = (uint16_t)jn;
    top = jn;
  }
}

// The lite carves with their Philox words prefetched (MZ_RING): a draw read inline runs a
// Philox4x32-10 block (40 quarter-rate multiplies) on the carve's serial chain every 4th draw —
// about a third of an r-prim iteration's cycles. The stream is counter-based (word n =
// philox(key, n >> 2)[n & 3]), so the words can come from anywhere: each maze keeps a ring of
// 4 SP words in LDS (SP = the lanes per maze), refilled by its SP lanes at once (one block each)
// whenever its next iteration could pass the ring's end. The loop runs on every lane (the refill
// check is a wave vote; the carve body is the maze's first lane's), and a carve reads its draws
// from the ring in the order MzRng would produce them: the same mazes.
template <int SP>
__device__ inline void mz_ring_fill(uint32_t* ring, uint64_t key, int rb, int lane) {
  const int k = lane % SP;
  uint32_t o[4];
  mz_philox(key, MZ_GEN_STREAM, (uint64_t)(rb >> 2) + (uint64_t)k, o);
  *reinterpret_cast<uint4*>(ring + 4 * k) = make_uint4(o[0], o[1], o[2], o[3]);
}

template <int SP>
__device__ void mz_lite_carve_ring(const MzCellLds& L, int algo, uint64_t key, bool carver,
                                   uint32_t* ring) {
  constexpr int RW = 4 * SP;
  const int lane = threadIdx.x, W = L.W;
  const bool dfs = algo == MZ_ALGO_DFS_DEV;
  uint32_t* pw = reinterpret_cast<uint32_t*>(L.pas);
  int n = 0, rb = 0;  // (carver lanes) the next draw's index, the ring's first
  mz_ring_fill<SP>(ring, key, 0, lane);
  __syncthreads();
  auto below = [&](uint32_t mm) {
    const uint32_t u = ring[n - rb];
    ++n;
    return (uint32_t)(((uint64_t)u * mm) >> 32);
  };
  int nf = 0, top = 0;  // r-prim: frontier size; dfs: stack size (nf) and top
  bool active = carver;
  if (carver) {
    // start = (randrange(1, G-1, 2), randrange(1, G-1, 2)) (maze_generation.py:21)
    const int a = (int)below((uint32_t)W), b = (int)below((uint32_t)W);
    const int s = a * W + b;
    L.sh[2] = s;
    cs_set(L.b0, s);
    if (dfs) {
      L.list[nf++] = (uint16_t)s;
      top = s;
    } else {
      for (int k = 0; k < 4; ++k) {
        const int j = cs_nb(s, k, W, L.mW);
        if (j >= 0) { L.list[nf++] = (uint16_t)j; cs_set(L.b1, j); }
      }
    }
  }
  for (;;) {
    const bool need = active && n + 2 > rb + RW;
    if (__any(need)) {  // the mazes that need it refill, all their lanes at once
      const int src = (lane / SP) * SP;
      const int nn = __shfl(n, src);
      if (__shfl((int)need, src)) mz_ring_fill<SP>(ring, key, nn & ~3, lane);
      if (need) rb = n & ~3;
      __syncthreads();
    }
    if (!__any(active)) break;
    if (!active) continue;
    if (dfs) {  // one step of deept_first_visit (maze_generation.py:101-128), as mz_lite_dfs
      int j[4];
      uint32_t w0[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        j[k] = cs_nb(top, k == 0 ? 2 : (k == 1 ? 3 : k - 2), W, L.mW);
        const int jj = j[k] >= 0 ? j[k] : top;
        w0[k] = L.b0[jj >> 5] >> (jj & 31);
      }
      uint64_t cand = 0;
      int cnt = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (j[k] >= 0 && !(w0[k] & 1u)) mz_k4_push(cand, cnt, k);
      if (!cnt) {
        if (--nf > 0) top = L.list[nf - 1];
        else active = false;
        continue;
      }
      const int k = mz_k4(cand, (int)below((uint32_t)cnt));
      const int dir = k == 0 ? 2 : (k == 1 ? 3 : k - 2);
      const int jn = k == 0 ? j[0] : (k == 1 ? j[1] : (k == 2 ? j[2] : j[3]));
      cs_link(L, top, dir);
      cs_set(L.b0, jn);
      atomicOr(pw + (jn >> 2), (uint32_t)((dir ^ 1) << 2) << (8 * (jn & 3)));
      L.list[nf++] = (uint16_t)jn;
      top = jn;
    } else {  // one step of random_prim_visit (maze_generation.py:59-99), as mz_lite_rprim
      const int i = (int)below((uint32_t)nf);
      const int f = L.list[i];
      L.list[i] = L.list[--nf];
      int j[4];
      uint32_t w0[4], w1[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        j[k] = cs_nb(f, k, W, L.mW);
        const int jj = j[k] >= 0 ? j[k] : f;
        w0[k] = L.b0[jj >> 5] >> (jj & 31);
        w1[k] = L.b1[jj >> 5] >> (jj & 31);
      }
      uint64_t nb = 0;
      int cnt = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (j[k] >= 0 && (w0[k] & 1u)) mz_k4_push(nb, cnt, j[k] | (k << 12));
      if (cnt) {
        const int v = mz_k4(nb, (int)below((uint32_t)cnt)), kk = v >> 12;
        cs_set(L.b0, f);
        cs_link(L, f, kk);
        atomicOr(pw + (f >> 2), (uint32_t)(kk << 2) << (8 * (f & 3)));
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (j[k] >= 0 && !(w0[k] & 1u) && !(w1[k] & 1u)) {
            if (nf == L.cap) { L.sh[4] = 1; nf = 0; break; }  // past the cap: flagged, abandoned
            L.list[nf++] = (uint16_t)j[k];
            cs_set(L.b1, j[k]);
          }
        }
      }
      if (nf == 0) active = false;
    }
  }
}

// The lite carves lane-parallel (MZ_LANES): every lane of a maze's SP-lane group runs the carve
// loop, and lane k < 4 of the group takes neighbour k of an iteration — the four neighbour scans
// that one lane ran back to back (cs_nb, the two set-bit reads, the candidate list as a packed
// u64) become one pass over four lanes, the choices wave ballots (the group's 4-bit masks), and
// the frontier pushes one store per pushing lane at its rank among them. The group's lanes keep
// the same n / nf / top; the same draws in the same order, the same cells pushed in the same
// order: the same mazes as mz_lite_carve_ring. An overflowing frontier is flagged as there
// (the sequential loop's break at nf == cap before a push <=> nf + pushes > cap).
template <int SP>
__device__ void mz_lite_carve_lanes(const MzCellLds& L, int algo, uint64_t key, bool live,
                                    uint32_t* ring) {
  static_assert(SP >= 4 && SP <= 16 && 64 % SP == 0, "group of 4..16 lanes");
  constexpr int RW = 4 * SP;
  const int lane = threadIdx.x, gl = lane % SP, g0 = lane - gl, W = L.W;
  const bool dfs = algo == MZ_ALGO_DFS_DEV;
  uint32_t* pw = reinterpret_cast<uint32_t*>(L.pas);
  int n = 0, rb = 0;  // the group's next draw and the ring's first word
  mz_ring_fill<SP>(ring, key, 0, lane);
  __syncthreads();
  auto mulhi = [](uint32_t u, uint32_t mm) { return (int)(((uint64_t)u * mm) >> 32); };
  // the group's 4-bit mask of a per-neighbour predicate (lanes g0 .. g0 + 3)
  auto mask4 = [&](bool p) { return (uint32_t)(__ballot(p) >> g0) & 0xFu; };
  auto nth = [](uint32_t m, int v) {  // position of the v-th (0-based) set bit of m
    const uint32_t m1 = m & (m - 1u), m2 = m1 & (m1 - 1u), m3 = m2 & (m2 - 1u);
    const uint32_t sel = v == 0 ? m : (v == 1 ? m1 : (v == 2 ? m2 : m3));
    return __ffs(sel) - 1;
  };
  const bool nbl = gl < 4;  // a neighbour lane
  // deept_first_visit's direction order (left, right, up, down) in cs_nb's numbering
  const int ddir = gl == 0 ? 2 : (gl == 1 ? 3 : gl - 2);
  int nf = 0, top = 0;  // r-prim: frontier size; dfs: stack size and top
  bool active = live;
  if (live) {
    // start = (randrange(1, G-1, 2), randrange(1, G-1, 2)) (maze_generation.py:21)
    const int a = mulhi(ring[0], (uint32_t)W), b = mulhi(ring[1], (uint32_t)W);
    n = 2;
    const int s0 = a * W + b;
    if (gl == 0) { L.sh[2] = s0; cs_set(L.b0, s0); }
    if (dfs) {
      if (gl == 0) L.list[0] = (uint16_t)s0;
      nf = 1;
      top = s0;
    } else {
      const int j = nbl ? cs_nb(s0, gl, W, L.mW) : -1;
      const uint32_t vm = mask4(j >= 0);
      if (j >= 0) {
        L.list[__popc(vm & ((1u << gl) - 1u))] = (uint16_t)j;
        cs_set(L.b1, j);
      }
      nf = __popc(vm);
    }
  }
  for (;;) {
    const bool need = active && n + 2 > rb + RW;
    if (__any(need)) {  // the groups that need it refill, all their lanes at once
      if (need) {
        mz_ring_fill<SP>(ring, key, n & ~3, lane);
        rb = n & ~3;
      }
      __syncthreads();
    }
    if (!__any(active)) break;
    if (!active) continue;
    if (dfs) {  // one step of deept_first_visit (maze_generation.py:101-128)
      const int j = nbl ? cs_nb(top, ddir, W, L.mW) : -1;
      const bool unv = j >= 0 && !((L.b0[j >> 5] >> (j & 31)) & 1u);
      const uint32_t cm = mask4(unv);
      if (!cm) {
        if (--nf > 0) top = L.list[nf - 1];
        else active = false;
        continue;
      }
      const int k = nth(cm, mulhi(ring[n - rb], (uint32_t)__popc(cm)));
      ++n;
      const int dir = k == 0 ? 2 : (k == 1 ? 3 : k - 2);
      const int jn = cs_nb(top, dir, W, L.mW);
      if (gl == 0) {
        cs_link(L, top, dir);
        cs_set(L.b0, jn);
        atomicOr(pw + (jn >> 2), (uint32_t)((dir ^ 1) << 2) << (8 * (jn & 3)));
        L.list[nf] = (uint16_t)jn;
      }
      ++nf;
      top = jn;
    } else {  // one step of random_prim_visit (maze_generation.py:59-99)
      const uint32_t u0 = ring[n - rb], u1 = ring[n + 1 - rb];
      const int i = mulhi(u0, (uint32_t)nf);
      const int f = L.list[i];
      const int last = L.list[nf - 1];
      const int j = nbl ? cs_nb(f, gl, W, L.mW) : -1;
      const int jj = j >= 0 ? j : f;
      const bool in0 = j >= 0 && ((L.b0[jj >> 5] >> (jj & 31)) & 1u);
      const bool in1 = (L.b1[jj >> 5] >> (jj & 31)) & 1u;
      const uint32_t im = mask4(in0), fm = mask4(j >= 0 && !in0 && !in1);
      if (gl == 0) L.list[i] = (uint16_t)last;  // list[i] = list[--nf]
      --nf;
      ++n;
      if (im) {
        const int kk = nth(im, mulhi(u1, (uint32_t)__popc(im)));
        ++n;
        if (gl == 0) {
          cs_set(L.b0, f);
          cs_link(L, f, kk);
          atomicOr(pw + (f >> 2), (uint32_t)(kk << 2) << (8 * (f & 3)));
        }
        const int np = __popc(fm);
        if (nf + np > L.cap) {  // past the cap: flagged, abandoned
          if (gl == 0) L.sh[4] = 1;
          nf = 0;
        } else {
          if ((fm >> gl) & 1u && nbl) {
            L.list[nf + __popc(fm & ((1u << gl) - 1u))] = (uint16_t)j;
            cs_set(L.b1, j);
          }
          nf += np;
        }
      }
      if (nf == 0) active = false;
    }
  }
}

// The finish of a lite candidate (wave-wide; J / A: the per-wave scratch): carve depths by pointer
// jumping over the parent directions (J = ancestor | distance << 16), the goal as mz_cs_goal, the
// distance field as mz_cs_dist's tree path (the goal's root path marked in b1: the solution's
// cells), then the compact form leaves LDS as mz_cells_compact writes it.
__device__ __forceinline__ void mz_lite_finish(const MzCompact& cc, int t, const MzCellLds& L, int N,
                                               uint32_t* J, uint16_t* A) {
  const int lane = threadIdx.x, Q = L.Q, W = L.W;
  const int s = L.sh[2];
  const bool over = L.sh[4] != 0;
  auto parent = [&](int q) { return cs_nb(q, (L.pas[q] >> 2) & 3, W, L.mW); };
  bool ok = !over;
  int goal = s;
  if (ok) {
    for (int q = lane; q < Q; q += 64) J[q] = q == s ? (uint32_t)s : ((uint32_t)parent(q) | (2u << 16));
    __syncthreads();
    bool conv = false;
    for (int it = 0; it < 16 && !conv; ++it) {
      bool ch = false;
      for (int q = lane; q < Q; q += 64) {
        const uint32_t j = J[q];
        const int a = (int)(j & 0xFFFFu);
        if (a == s) continue;
        const uint32_t ja = J[a];
        J[q] = (ja & 0xFFFFu) | ((j & 0xFFFF0000u) + (ja & 0xFFFF0000u));
        ch = true;
      }
      conv = !__any(ch);
      __syncthreads();
    }
    ok = conv;
    auto dep = [&](int q) { return (int)(J[q] >> 16); };
    // find_random_position (maze_generation.py:187-218): the deepest dead end, then the smallest
    // square index (mz_cs_goal's key)
    uint32_t best = 0;
    for (int q = lane; q < Q && ok; q += 64) {
      if (q == s) continue;
      int nb = 0;
      for (int k = 0; k < 4; ++k) nb += cs_open_dir(L, q, k);
      if (nb != 1) continue;
      const int r = cs_row(q, L.mW), c = q - r * W, p = (2 * r + 1) * N + 2 * c + 1;
      const uint32_t key = ((uint32_t)(dep(q) + 1) << 16) | (uint32_t)(0xFFFF - p);
      best = key > best ? key : best;
    }
    for (int o = 32; o > 0; o >>= 1) {
      const uint32_t x = __shfl_xor(best, o);
      best = x > best ? x : best;
    }
    if (best) {
      const int p = 0xFFFF - (int)(best & 0xFFFF), r = p / N, c = p - r * N;
      goal = (r >> 1) * W + (c >> 1);
    }
    // distances to the goal: parents into A, the goal's root path into b1, every cell's first
    // ancestor on that path by pointer jumping, D = dep + dep(goal) - 2 dep(ancestor)
    for (int q = lane; q < Q; q += 64) A[q] = (uint16_t)(q == s ? s : parent(q));
    for (int i = lane; i < (Q + 31) / 32; i += 64) L.b1[i] = 0u;
    __syncthreads();
    if (lane == 0) {
      int x = goal, n = 0;
      for (; n <= Q; ++n) {
        cs_set(L.b1, x);
        if (x == s) break;
        x = A[x];
      }
      L.sh[3] = n > Q;
    }
    __syncthreads();
    ok = ok && !L.sh[3];
    conv = false;
    for (int it = 0; it < 32 && !conv && ok; ++it) {
      bool ch = false;
      for (int q = lane; q < Q; q += 64) {
        const int a = A[q];
        if (cs_bit(L.b1, a)) continue;
        A[q] = A[a];
        ch = true;
      }
      conv = !__any(ch);
      __syncthreads();
    }
    ok = ok && conv;
    if (ok) {
      const int dg = dep(goal);
      for (int q = lane; q < Q; q += 64) {
        const int a = cs_bit(L.b1, q) ? q : A[q];
        A[q] = (uint16_t)(dep(q) + dg - 2 * dep(a));
      }
    }
    __syncthreads();
  }
  uint32_t* gp = reinterpret_cast<uint32_t*>(cc.pas + (size_t)t * cc.Qp);
  uint32_t* ga = reinterpret_cast<uint32_t*>(cc.dist + (size_t)t * cc.Qp);
  const uint32_t* lp = reinterpret_cast<const uint32_t*>(L.pas);
  const uint32_t* la = reinterpret_cast<const uint32_t*>(A);
  if (ok) {
    for (int i = lane; i < (Q + 3) / 4; i += 64) gp[i] = lp[i] & 0x03030303u;  // (passages only)
    for (int i = lane; i < (Q + 1) / 2; i += 64) ga[i] = la[i];
    for (int i = lane; i < (Q + 31) / 32; i += 64) cc.sol[(size_t)t * cc.QWp + i] = L.b1[i];
  }
  if (lane == 0)
    cc.meta[t] = (uint32_t)N | (ok ? 0u : MZ_CMETA_NOSOL) | ((uint32_t)s << 8) | ((uint32_t)goal << 20);
  __syncthreads();
}

__device__ __forceinline__ void mz_build_cells_packed(const MzDev& d, int e, uint64_t seed, int nm,
                                                      int N, int algo, uint8_t* lds, size_t stride) {
  mz_carve_packed(d.P, seed, nm, N, algo, lds, stride);
  for (int k = 0; k < nm; ++k) {
    mz_cells_finish(d, __shfl(e, 16 * k), mz_cell_lds(lds + k * stride, d.P, N), N, false);
    __syncthreads();
  }
}

// goal, distance field and tables of a carved cell-space maze (wave-wide): the rest of
// mz_build_cells
__device__ __forceinline__ void mz_cells_finish(const MzDev& d, int e, const MzCellLds& L, int N,
                                                bool tor) {
  const int lane = threadIdx.x;
  const int G = tor ? N + 2 : N;
  const int W = L.W;
  const int s = L.sh[2];
  int goal = (MZ_GPROBE & 4) ? s : mz_cs_goal(L, G, s);
  if (goal < 0) goal = s;  // unreachable for W >= 2 (a spanning tree has >= 2 leaves)
  // open squares of the G x G generation grid
  auto open_g = [&](int r, int c) -> bool {
    const bool ro = r & 1, co = c & 1;
    if (ro && co) return true;  // every cell is in the tree
    if (!ro && !co) return false;
    if (ro) return c > 0 && c < G - 1 && (L.pas[(r >> 1) * W + ((c - 1) >> 1)] & 1);
    return r > 0 && r < G - 1 && (L.pas[((r - 1) >> 1) * W + (c >> 1)] & 2);
  };
  const int off = tor ? 1 : 0;  // crop the border (maze_generation.py:53-55)
  const int sr = 2 * (s / W) + 1 - off, sc = 2 * (s % W) + 1 - off;
  const int gr = 2 * (goal / W) + 1 - off, gc = 2 * (goal % W) + 1 - off;
  if (!tor) {
    if (!(MZ_GPROBE & 2)) mz_cs_dist(L, s, goal);
    if (MZ_GPROBE & 1) {  // probe: only the meta words (no cell words / planes)
      if (lane == 0) { d.meta0[e] = (uint32_t)N | ((uint32_t)N << 8) | ((uint32_t)sr << 16) | ((uint32_t)sc << 24); d.meta1[e] = (uint32_t)gr | ((uint32_t)gc << 8); }
      return;
    }
    mz_cells_tables(d, e, L, N, s, goal);
    return;
  }
  // torus: BFS from the goal over row masks, in the region after the passages
  const int P = d.P;
  uint8_t* rb = reinterpret_cast<uint8_t*>(L.b0);  // first byte after pas (16-B aligned)
  uint16_t* dist = reinterpret_cast<uint16_t*>(rb);
  mz_u128* O = reinterpret_cast<mz_u128*>(rb + mz_align16(2 * (size_t)P * P));
  mz_u128* V = O + P;
  mz_u128* F = V + P;  // two frontier buffers: F[0..P), F[P..2P)
  auto open_t = [&](int y, int x) -> bool { return open_g(y + 1, x + 1); };
  const mz_u128 mask = (N == 128) ? ~(mz_u128)0 : (((mz_u128)1 << N) - 1);
  __syncthreads();  // the generator's lists are dead: the BFS region may overwrite them
  for (int y = lane; y < N; y += 64) {
    mz_u128 o = 0;
    for (int x = 0; x < N; ++x)
      if (open_t(y, x)) o |= (mz_u128)1 << x;
    const mz_u128 g = y == gr ? (mz_u128)1 << gc : 0;
    O[y] = o;
    V[y] = g;
    F[y] = g;
  }
  for (int i = lane; i < N * N; i += 64) dist[i] = 0xFFFF;
  __syncthreads();
  if (lane == 0) dist[gr * N + gc] = 0;
  int cur = 0;
  for (int level = 1;; ++level) {
    const mz_u128* Fc = F + cur * P;
    mz_u128* Fn = F + (cur ^ 1) * P;
    bool any = false;
    for (int y = lane; y < N; y += 64) {
      const mz_u128 f = Fc[y];
      const mz_u128 reach = f | mz_row_rotl(f, N, mask) | mz_row_rotr(f, N) | Fc[y == 0 ? N - 1 : y - 1] |
                            Fc[y == N - 1 ? 0 : y + 1];
      mz_u128 nw = reach & O[y] & ~V[y];
      Fn[y] = nw;
      if (nw) {
        any = true;
        V[y] |= nw;
        while (nw) {  // the new squares of row y are at distance `level`
          const uint64_t lo = (uint64_t)nw, hi = (uint64_t)(nw >> 64);
          const int x = lo ? __ffsll((long long)lo) - 1 : 64 + __ffsll((long long)hi) - 1;
          dist[y * N + x] = (uint16_t)level;
          nw &= nw - 1;
        }
      }
    }
    __syncthreads();
    if (!__any(any)) break;
    cur ^= 1;
  }
  mz_build_write(d, e, N, true, sr, sc, gr, gc, open_t,
                 [&](int y, int x) { return (int)dist[y * N + x]; });
}

#include "mz_pygen.inc.h"

// LDS of a build launch: the build region, plus the CPython-exact generation region when used
__host__ __device__ inline size_t mz_build_lds_bytes_mode(int P, int pymode) {
  return mz_build_lds_bytes(P) + (pymode ? mz_py_lds_bytes(P + 2) : 0);
}

__device__ inline MzPyLds mz_py_lds(uint8_t* base, const MzBuildLds& L, int G) {
  MzPyLds Y;
  Y.mt = reinterpret_cast<uint32_t*>(base);
  Y.hdr = reinterpret_cast<int*>(base + 2512);
  Y.cap_a = mz_py_cap_a(G);
  Y.cap_b = mz_py_cap_b(G);
  Y.small = reinterpret_cast<uint16_t*>(base + 2560);
  Y.ta = reinterpret_cast<uint16_t*>(base + 2592);
  Y.tb = Y.ta + Y.cap_a;
  Y.sbits = reinterpret_cast<uint32_t*>(L.queue);
  Y.slot_of = reinterpret_cast<uint16_t*>(Y.sbits + Y.cap_b / 32);
  Y.scratch = L.dist;  // dist + queue (contiguous, 4 G^2 bytes): free while generating
  Y.G = G;
  return Y;
}

#define MZ_PY_PHILOX 0  // Philox4x32 stream (seed), uniform choices over the same candidates
#define MZ_PY_SEED 1    // CPython-exact from random.seed(seed)
#define MZ_PY_STATE 2   // CPython-exact from the random.getstate() words in py_state (in/out)

// Builds maze + tables of instance e and resets it. generate: generation with algo/seed
// (pymode: MZ_PY_*; py_state [625] for MZ_PY_STATE, py_err set on a set-table overflow);
// else import grid_src [N][N] with (sr,sc,gr,gc). Returns via d.meta*: all lanes must call.
__device__ void mz_build_one(const MzDev& d, int e, bool tor, bool generate, int algo,
                             uint64_t seed, int N, const uint8_t* grid_src, int isr, int isc,
                             int igr, int igc, uint8_t* lds, int pymode = MZ_PY_PHILOX,
                             uint32_t* py_state = nullptr, int* py_err = nullptr) {
  if (MZ_CELL_BUILD && generate && pymode == MZ_PY_PHILOX) {
    mz_build_cells(d, e, algo, seed, N, tor, lds);
    return;
  }
  const int lane = threadIdx.x;
  const MzBuildLds L = mz_build_lds(lds, d.P);
  int sr, sc, gr, gc;
  bool tree = false;  // L.queue holds the carve depths of a perfect euclidean maze
  if (generate && pymode != MZ_PY_PHILOX) {
    const int G = tor ? N + 2 : N;
    for (int i = lane; i < G * G; i += 64) L.g[i] = 0;
    const MzPyLds Y = mz_py_lds(lds + mz_build_lds_bytes(d.P), L, G);
    if (lane == 0) {
      if (pymode == MZ_PY_SEED) mz_mt_seed(Y.mt, seed);
      else for (int i = 0; i < 625; ++i) Y.mt[i] = py_state[i];
    }
    __syncthreads();
    const int s = mz_py_generate(L, Y, G, algo);
    if (lane == 0) {
      if (pymode == MZ_PY_STATE) for (int i = 0; i < 625; ++i) py_state[i] = Y.mt[i];
      if (Y.hdr[6] && py_err) atomicOr(py_err, Y.hdr[6]);
    }
    int goal = mz_goal_select(L, G, s);
    if (goal < 0) goal = s;
    __syncthreads();
    if (lane == 0) L.g[goal] = 2;
    __syncthreads();
    sr = s / G; sc = s - sr * G; gr = goal / G; gc = goal - gr * G;
    if (tor) {  // crop the border (maze_generation.py:53-55)
      for (int i = lane; i < N * N; i += 64) {
        const int r = i / N, c = i - r * N;
        L.dist[i] = L.g[(r + 1) * G + (c + 1)];
      }
      __syncthreads();
      for (int i = lane; i < N * N; i += 64) L.g[i] = (uint8_t)L.dist[i];
      __syncthreads();
      sr -= 1; sc -= 1; gr -= 1; gc -= 1;
    }
  } else if (generate) {  // Philox in the square grid: the MZ_CELL_BUILD=0 A/B reference
    const int G = tor ? N + 2 : N;
    for (int i = lane; i < G * G; i += 64) L.g[i] = 0;
    __syncthreads();
    MzRng rng{seed, 0ull, {0u, 0u, 0u, 0u}};
    int s = 0;
    if (lane == 0) {
      // start = (randrange(1, G-1, 2), randrange(1, G-1, 2)) (maze_generation.py:21)
      const int a = 1 + 2 * (int)rng.below((uint32_t)((G - 1) / 2));
      const int b = 1 + 2 * (int)rng.below((uint32_t)((G - 1) / 2));
      s = a * G + b;
      L.g[s] = 1;
      L.sh[2] = s;
      if (algo == MZ_ALGO_RPRIM_DEV) mz_gen_rprim(L, G, s, rng);
      else if (algo == MZ_ALGO_DFS_DEV) mz_gen_dfs(L, G, s, rng);
    }
    __syncthreads();
    s = L.sh[2];
    if (algo != MZ_ALGO_RPRIM_DEV && algo != MZ_ALGO_DFS_DEV) mz_gen_primkill(L, G, s, rng);
    else  // r-prim / dfs carve depths into L.dist (their stack / frontier lives in L.queue)
      for (int i = lane; i < G * G; i += 64) L.queue[i] = L.dist[i];
    __syncthreads();
    // goal from the carve depths (== a BFS from s over the carved tree)
    int goal = MZ_TREE_DIST ? mz_goal_scan(L, G, s, L.queue) : mz_goal_select(L, G, s);
    if (goal < 0) goal = s;  // unreachable for G >= 5 (a spanning tree has >= 2 leaves)
    __syncthreads();
    if (lane == 0) L.g[goal] = 2;
    __syncthreads();
    sr = s / G; sc = s - sr * G; gr = goal / G; gc = goal - gr * G;
    tree = MZ_TREE_DIST && !tor;
    if (tor) {  // crop the border (maze_generation.py:53-55)
      for (int i = lane; i < N * N; i += 64) {
        const int r = i / N, c = i - r * N;
        L.dist[i] = L.g[(r + 1) * G + (c + 1)];
      }
      __syncthreads();
      for (int i = lane; i < N * N; i += 64) L.g[i] = (uint8_t)L.dist[i];
      __syncthreads();
      sr -= 1; sc -= 1; gr -= 1; gc -= 1;
    }
  } else {
    for (int i = lane; i < N * N; i += 64) L.g[i] = grid_src[i];
    sr = isr; sc = isc; gr = igr; gc = igc;
    __syncthreads();
  }
  // distance-to-goal field (len(find_path(p)) = D[p] + 1): from the carved tree for
  // a Philox-generated euclidean maze, else a BFS (toroidal: the crop's wrap adds cycles;
  // imported and CPython-exact mazes carry no carve depths)
  if (!tree || !mz_tree_dist(L, N, sr * N + sc, gr * N + gc)) mz_wave_bfs(L, N, tor, gr * N + gc);
  mz_build_write(d, e, N, tor, sr, sc, gr, gc, [&](int y, int x) { return L.g[y * N + x] != 0; },
                 [&](int y, int x) { return (int)L.dist[y * N + x]; });
}
