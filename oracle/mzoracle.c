/* mzoracle.c — CPU restatement of the reference maze-env hot path. TEST INFRASTRUCTURE ONLY.
 *
 * Parity checker for the HIP product: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load this (via ctypes, oracle/_build/libmzoracle.so). The product library
 * (libmazerl.so) never links or calls it.
 *
 * Pinning: tests/test_oracle_golden.py checks every function below against the fixtures in
 * tests/golden/ (.npz), which tests/golden/make_golden.py produced by running the reference's own
 * Python code in the build container.
 *
 * Every function cites the reference file:line it restates. Build: oracle/Makefile
 * (gcc -O2 -ffp-contract=off: the reward / score / max_steps doubles must round exactly like
 * CPython's, so no FMA contraction and no fast-math).
 */
#include "mzoracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* BaseMazeEnv.ACTIONS (base_maze_env.py:19-24): 0 down, 1 up, 2 right, 3 left */
static const int DR[4] = {1, -1, 0, 0};
static const int DC[4] = {0, 0, 1, -1};

static inline int wrap(int v, int n) { v %= n; return v < 0 ? v + n : v; }

/* ------------------------------------------------------------------------------------------ */
int mzo_bfs(const uint8_t* grid, int H, int W, int toroidal, int sr, int sc, int32_t* dist) {
  int n = H * W;
  for (int i = 0; i < n; ++i) dist[i] = -1;
  if (grid[sr * W + sc] == 0) return 0;
  int* q = (int*)malloc(sizeof(int) * n);
  int head = 0, tail = 0;
  dist[sr * W + sc] = 0;
  q[tail++] = sr * W + sc;
  while (head < tail) {
    int cur = q[head++];
    int r = cur / W, c = cur % W;
    for (int k = 0; k < 4; ++k) {
      int nr = r + DR[k], nc = c + DC[k];
      if (toroidal) { nr = wrap(nr, H); nc = wrap(nc, W); }
      else if (nr < 0 || nr >= H || nc < 0 || nc >= W) continue;
      int ni = nr * W + nc;
      if (grid[ni] == 0 || dist[ni] >= 0) continue;
      dist[ni] = dist[cur] + 1;
      q[tail++] = ni;
    }
  }
  free(q);
  return tail;
}

/* ------------------------------------------------------------------------------------------ */
/* astar_limited_partial: a_star.py:9-82 (euclidean), a_star_tor.py:15-88 (toroidal).
 * Python heapq over (f, (r, c)) tuples => pop order = lexicographic (f, r, c). */
typedef struct { int f, r, c; } hnode;
static inline int hless(hnode a, hnode b) {
  if (a.f != b.f) return a.f < b.f;
  if (a.r != b.r) return a.r < b.r;
  return a.c < b.c;
}
static void hpush(hnode* h, int* n, hnode x) {
  int i = (*n)++;
  h[i] = x;
  while (i > 0) {
    int p = (i - 1) / 2;
    if (!hless(h[i], h[p])) break;
    hnode t = h[i]; h[i] = h[p]; h[p] = t; i = p;
  }
}
static hnode hpop(hnode* h, int* n) {
  hnode top = h[0];
  h[0] = h[--(*n)];
  int i = 0;
  for (;;) {
    int l = 2 * i + 1, r = l + 1, m = i;
    if (l < *n && hless(h[l], h[m])) m = l;
    if (r < *n && hless(h[r], h[m])) m = r;
    if (m == i) break;
    hnode t = h[i]; h[i] = h[m]; h[m] = t; i = m;
  }
  return top;
}
static int heur(int ar, int ac, int br, int bc, int H, int W, int toroidal) {
  int dx = abs(ar - br), dy = abs(ac - bc);
  if (toroidal) { /* a_star_tor.py:3-12 */
    if (H - dx < dx) dx = H - dx;
    if (W - dy < dy) dy = W - dy;
  }
  return dx + dy;
}

int mzo_astar_len(const uint8_t* grid, int H, int W, int toroidal, int sr, int sc, int gr, int gc,
                  int max_depth) {
  if (max_depth < 0) max_depth = 1000000;
  int n = H * W;
  int* g = (int*)malloc(sizeof(int) * n);
  int* from = (int*)malloc(sizeof(int) * n);
  int cap = 8 * n + 16, hn = 0;
  hnode* heap = (hnode*)malloc(sizeof(hnode) * cap);
  for (int i = 0; i < n; ++i) { g[i] = -1; from[i] = -1; }
  int s = sr * W + sc, goal = gr * W + gc;
  g[s] = 0;
  hnode st = {heur(sr, sc, gr, gc, H, W, toroidal), sr, sc};
  hpush(heap, &hn, st);
  int best = s, best_g = 0, end = -1;
  /* a_star.py:43-79 */
  while (hn > 0) {
    hnode cur = hpop(heap, &hn);
    int ci = cur.r * W + cur.c;
    if (g[ci] > best_g) { best_g = g[ci]; best = ci; }
    if (ci == goal) { end = ci; break; }
    if (g[ci] >= max_depth) continue;
    /* neighbour order a_star.py:60: (-1,0),(1,0),(0,-1),(0,1) */
    static const int AR[4] = {-1, 1, 0, 0}, AC[4] = {0, 0, -1, 1};
    for (int k = 0; k < 4; ++k) {
      int nr = cur.r + AR[k], nc = cur.c + AC[k];
      if (toroidal) { nr = wrap(nr, H); nc = wrap(nc, W); }
      else if (nr < 0 || nr >= H || nc < 0 || nc >= W) continue;
      int ni = nr * W + nc;
      if (grid[ni] == 0) continue;
      int tg = g[ci] + 1;
      if (tg > max_depth) continue;
      if (g[ni] < 0 || tg < g[ni]) {
        from[ni] = ci;
        g[ni] = tg;
        if (hn >= cap) { cap *= 2; heap = (hnode*)realloc(heap, sizeof(hnode) * cap); }
        hnode x = {tg + heur(nr, nc, gr, gc, H, W, toroidal), nr, nc};
        hpush(heap, &hn, x);
      }
    }
  }
  if (end < 0) end = best;
  /* reconstruct_path a_star.py:84-100 */
  int len = 1;
  for (int v = end; from[v] >= 0; v = from[v]) ++len;
  free(g); free(from); free(heap);
  return len;
}

/* ------------------------------------------------------------------------------------------ */
/* find_random_position: maze_generation.py:187-218. len(astar(start, cand)) = dist + 1 (BFS). */
int mzo_goal_select(const uint8_t* grid, int H, int W, int sr, int sc, int* gr, int* gc) {
  int32_t* d = (int32_t*)malloc(sizeof(int32_t) * H * W);
  mzo_bfs(grid, H, W, 0, sr, sc, d);
  int found = 0, best = -1, br = -1, bc = -1;
  for (int r = 1; r < H; r += 2)
    for (int c = 1; c < W; c += 2) {
      if (grid[r * W + c] != 1 || (r == sr && c == sc)) continue;
      /* neighbours (-1,0),(1,0),(0,-1),(0,1): maze_generation.py:203 (odd H keeps r+1 < H) */
      if (r + 1 >= H || c + 1 >= W) { free(d); return -2; } /* reference: IndexError (even N) */
      int nb = (grid[(r - 1) * W + c] != 0) + (grid[(r + 1) * W + c] != 0) +
               (grid[r * W + c - 1] != 0) + (grid[r * W + c + 1] != 0);
      if (nb != 1) continue;
      int dist = d[r * W + c];
      if (!found || dist > best) { best = dist; br = r; bc = c; found = 1; }
    }
  free(d);
  if (!found) return -1;
  *gr = br; *gc = bc;
  return 0;
}

/* set_max_steps: simple_maze_env.py:52-58 + MetricsCalculator (metrics_calculator.py:11-26):
 *   L = len(path)/CE, CE = (H-1)*((W-1)//2) - 1, max_steps = ceil((((H-1)*(W-1)) - 1) * L) */
int mzo_max_steps(const uint8_t* grid, int H, int W, int toroidal, int sr, int sc, int gr, int gc) {
  int32_t* d = (int32_t*)malloc(sizeof(int32_t) * H * W);
  mzo_bfs(grid, H, W, toroidal, gr, gc, d);
  int len = d[sr * W + sc] + 1;
  free(d);
  int ce = (H - 1) * ((W - 1) / 2) - 1;
  volatile double L = (double)len / (double)ce;
  volatile double prod = (double)(((H - 1) * (W - 1)) - 1) * L;
  return (int)ceil(prod);
}

/* ------------------------------------------------------------------------------------------ */
/* Philox4x32-10 (Salmon et al., SC'11). Shared definition with csrc/mz_common.h. */
static inline uint32_t mulhi32(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }
void mzo_philox(uint64_t key, uint64_t ctr_hi, uint64_t ctr_lo, uint32_t out[4]) {
  uint32_t c0 = (uint32_t)ctr_lo, c1 = (uint32_t)(ctr_lo >> 32), c2 = (uint32_t)ctr_hi,
           c3 = (uint32_t)(ctr_hi >> 32);
  uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
  for (int i = 0; i < 10; ++i) {
    if (i) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    uint32_t lo0 = 0xD2511F53u * c0, hi0 = mulhi32(0xD2511F53u, c0);
    uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = mulhi32(0xCD9E8D57u, c2);
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* One sequential draw stream per maze: draw k = word (k & 3) of philox(seed, {k >> 2, MZ_GEN}). */
#define MZ_GEN_STREAM 0x6D617A65ull /* 'maze' */
typedef struct { uint64_t key, n; uint32_t buf[4]; } rng_t;
static uint32_t rng_u32(rng_t* g) {
  if ((g->n & 3) == 0) mzo_philox(g->key, MZ_GEN_STREAM, g->n >> 2, g->buf);
  return g->buf[(g->n++) & 3];
}
/* uniform integer in [0, n): multiply-shift (identical on device) */
static uint32_t rng_below(rng_t* g, uint32_t n) { return (uint32_t)(((uint64_t)rng_u32(g) * n) >> 32); }

/* neighbour order of get_neighbors / random_walk: (-2,0),(2,0),(0,-2),(0,2)
 * (maze_generation.py:72,166) */
static const int GR[4] = {-2, 2, 0, 0}, GC[4] = {0, 0, -2, 2};
/* direction order of deept_first_visit: (0,-1),(0,1),(-1,0),(1,0) (maze_generation.py:114) */
static const int FR[4] = {0, 0, -1, 1}, FC[4] = {-1, 1, 0, 0};

/* random_prim_visit (maze_generation.py:59-99): uniform frontier pick, uniform in-maze neighbour */
static void gen_rprim(uint8_t* m, int N, int sr, int sc, rng_t* g) {
  int* fr = (int*)malloc(sizeof(int) * N * N);
  uint8_t* inF = (uint8_t*)calloc(N * N, 1);
  int nf = 0;
  m[sr * N + sc] = 1;
  for (int k = 0; k < 4; ++k) {
    int r = sr + GR[k], c = sc + GC[k];
    if (r < 0 || r >= N || c < 0 || c >= N) continue;
    fr[nf++] = r * N + c; inF[r * N + c] = 1;
  }
  while (nf > 0) {
    int i = (int)rng_below(g, (uint32_t)nf);
    int f = fr[i];
    fr[i] = fr[--nf];
    int fx = f / N, fy = f % N, nb[4], cnt = 0;
    for (int k = 0; k < 4; ++k) {
      int r = fx + GR[k], c = fy + GC[k];
      if (r < 0 || r >= N || c < 0 || c >= N) continue;
      if (m[r * N + c] == 1) nb[cnt++] = r * N + c;
    }
    if (cnt) {
      int nn = nb[rng_below(g, (uint32_t)cnt)];
      int nx = nn / N, ny = nn % N;
      m[f] = 1;
      m[((fx + nx) / 2) * N + (fy + ny) / 2] = 1;
      for (int k = 0; k < 4; ++k) {
        int r = fx + GR[k], c = fy + GC[k];
        if (r < 0 || r >= N || c < 0 || c >= N) continue;
        int j = r * N + c;
        if (m[j] == 0 && !inF[j]) { fr[nf++] = j; inF[j] = 1; }
      }
    }
  }
  free(fr); free(inF);
}

/* deept_first_visit (maze_generation.py:101-128): shuffle-then-first-valid == uniform valid pick */
static void gen_dfs(uint8_t* m, int N, int sr, int sc, rng_t* g) {
  int* st = (int*)malloc(sizeof(int) * N * N);
  int sp = 0;
  st[sp++] = sr * N + sc;
  while (sp > 0) {
    int x = st[sp - 1] / N, y = st[sp - 1] % N, cand[4], cnt = 0;
    for (int k = 0; k < 4; ++k) {
      int nx = x + 2 * FR[k], ny = y + 2 * FC[k];
      if (nx >= 0 && nx < N && ny >= 0 && ny < N && m[nx * N + ny] == 0) cand[cnt++] = k;
    }
    if (!cnt) { --sp; continue; }
    int k = cand[rng_below(g, (uint32_t)cnt)];
    m[(x + FR[k]) * N + (y + FC[k])] = 1;
    m[(x + 2 * FR[k]) * N + (y + 2 * FC[k])] = 1;
    st[sp++] = (x + 2 * FR[k]) * N + (y + 2 * FC[k]);
  }
  free(st);
}

/* prim_and_kill_visit + random_walk (maze_generation.py:130-185) */
static int pk_unmarked_nbrs(const uint8_t* mk, int N, int p, int* out) {
  int x = p / N, y = p % N, cnt = 0;
  for (int k = 0; k < 4; ++k) {
    int r = x + GR[k], c = y + GC[k];
    if (r < 0 || r >= N || c < 0 || c >= N) continue;
    if (mk[r * N + c] == 1) out[cnt++] = r * N + c; /* 1 = unmarked odd cell */
  }
  return cnt;
}
static void pk_walk(uint8_t* m, uint8_t* mk, int N, int cur, int* unmarked, rng_t* g) {
  int nb[4], cnt;
  while ((cnt = pk_unmarked_nbrs(mk, N, cur, nb)) != 0) {
    int nx = nb[rng_below(g, (uint32_t)cnt)];
    int cx = cur / N, cy = cur % N, x = nx / N, y = nx % N;
    m[(cx + (x - cx) / 2) * N + (cy + (y - cy) / 2)] = 1;
    cur = nx;
    mk[cur] = 2; /* marked */
    --*unmarked;
  }
}
static void gen_primkill(uint8_t* m, int N, int sr, int sc, rng_t* g) {
  uint8_t* mk = (uint8_t*)calloc(N * N, 1); /* 0 = not a cell, 1 = unmarked, 2 = marked */
  int unmarked = 0;
  for (int i = 1; i < N; i += 2)
    for (int j = 1; j < N; j += 2) { m[i * N + j] = 1; mk[i * N + j] = 1; ++unmarked; }
  mk[sr * N + sc] = 2; --unmarked;
  pk_walk(m, mk, N, sr * N + sc, &unmarked, g);
  int* cand = (int*)malloc(sizeof(int) * N * N);
  while (unmarked > 0) {
    /* marked cells with >= 1 unmarked neighbour (maze_generation.py:151), row-major order */
    int nc = 0, tmp[4];
    for (int p = 0; p < N * N; ++p)
      if (mk[p] == 2 && pk_unmarked_nbrs(mk, N, p, tmp)) cand[nc++] = p;
    pk_walk(m, mk, N, cand[rng_below(g, (uint32_t)nc)], &unmarked, g);
  }
  free(cand); free(mk);
}

/* gen_maze (maze_generation.py:6-35) / gen_maze_no_border (:37-56) */
int mzo_generate(uint8_t* grid, int H, int W, int toroidal, int algo, uint64_t seed, int* sr,
                 int* sc, int* gr, int* gc) {
  if (H != W || H < 5 || (H % 2) == 0) return -2; /* square, odd (Q4/Q5) */
  int N = toroidal ? H + 2 : H;
  uint8_t* m = (uint8_t*)calloc(N * N, 1);
  rng_t g = {seed, 0, {0, 0, 0, 0}};
  /* start = (randrange(1, N-1, 2), randrange(1, N-1, 2)) */
  int s_r = 1 + 2 * (int)rng_below(&g, (uint32_t)((N - 1) / 2));
  int s_c = 1 + 2 * (int)rng_below(&g, (uint32_t)((N - 1) / 2));
  m[s_r * N + s_c] = 1;
  if (algo == 0) gen_rprim(m, N, s_r, s_c, &g);
  else if (algo == 1) gen_dfs(m, N, s_r, s_c, &g);
  else gen_primkill(m, N, s_r, s_c, &g);
  int g_r, g_c;
  if (mzo_goal_select(m, N, N, s_r, s_c, &g_r, &g_c) != 0) { free(m); return -1; }
  m[g_r * N + g_c] = 2;
  if (toroidal) {
    for (int r = 0; r < H; ++r) memcpy(grid + r * W, m + (r + 1) * N + 1, W);
    s_r -= 1; s_c -= 1; g_r -= 1; g_c -= 1;
  } else {
    memcpy(grid, m, N * N);
  }
  free(m);
  *sr = s_r; *sc = s_c; *gr = g_r; *gc = g_c;
  return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* single-instance env */
int mzo_env_init(mzo_env* e, const uint8_t* grid, int H, int W, int toroidal, int enrich,
                 int sr, int sc, int gr, int gc, int astar_mode) {
  memset(e, 0, sizeof(*e));
  e->H = H; e->W = W; e->toroidal = toroidal; e->enrich = enrich;
  e->sr = sr; e->sc = sc; e->gr = gr; e->gc = gc; e->astar_mode = astar_mode;
  int n = H * W;
  e->grid = (uint8_t*)malloc(n);
  memcpy(e->grid, grid, n);
  e->D = (int32_t*)malloc(sizeof(int32_t) * n);
  e->visits = (int32_t*)calloc(n, sizeof(int32_t));
  e->nonvisited = (uint8_t*)malloc(n);
  mzo_bfs(e->grid, H, W, toroidal, gr, gc, e->D);
  e->max_steps = mzo_max_steps(e->grid, H, W, toroidal, sr, sc, gr, gc);
  return 0;
}
void mzo_env_free(mzo_env* e) {
  free(e->grid); free(e->D); free(e->visits); free(e->nonvisited);
  memset(e, 0, sizeof(*e));
}

/* find_path(src, max_depth): simple_maze_env.py:70-79 -> A*; fast mode: min(D, depth) + 1 */
static int path_len(const mzo_env* e, int r, int c, int max_depth) {
  if (e->astar_mode) return mzo_astar_len(e->grid, e->H, e->W, e->toroidal, r, c, e->gr, e->gc, max_depth);
  int d = e->D[r * e->W + c];
  if (max_depth >= 0 && d > max_depth) d = max_depth;
  return d + 1;
}

/* next_cell / valid_cell: simple_maze_env.py:38-39,60-68; toroidal_maze_env.py:79-87 */
static int next_valid(const mzo_env* e, int r, int c, int k, int* nr, int* nc) {
  int a = r + DR[k], b = c + DC[k];
  if (e->toroidal) {
    a = wrap(a, e->H); b = wrap(b, e->W);
    *nr = a; *nc = b;
    return e->grid[a * e->W + b] != 0;
  }
  *nr = a; *nc = b;
  return 0 < a && a < e->H && 0 < b && b < e->W && e->grid[a * e->W + b] != 0;
}

/* _find_best_next_cell: base_maze_env.py:224-262 (exact double arithmetic) */
void mzo_best_next(const mzo_env* e, int r, int c, int* br, int* bc) {
  int bestr = r, bestc = c;
  double best = INFINITY;
  int M = 2 * (e->H < e->W ? e->H : e->W);
  for (int k = 0; k < 4; ++k) {
    int nr, nc;
    if (!next_valid(e, r, c, k, &nr, &nc)) continue;
    int len = path_len(e, nr, nc, M);
    int manh = abs(nr - e->gr) + abs(nc - e->gc);
    volatile double t = 0.15 * (double)manh;
    volatile double score = (double)len + t;
    if (score < best) { best = score; bestr = nr; bestc = nc; }
    if (nr == e->gr && nc == e->gc) { *br = nr; *bc = nc; return; }
  }
  *br = bestr; *bc = bestc;
}

/* extract_submaze (maze_handler.py:4-54) row/col start for one axis; toroidal handled apart */
static int win_start(int p, int N) {
  const int k = 7, S = 15;
  if (S == N) return 0;
  if (p - k >= 0 && p + k < N) return p - k;
  if (p - k < 0 && p + k < N) return 0;
  if (p - k >= 0 && p + k >= N) return N - S;
  return -1; /* N < 15 with both edges: reference crashes (Q7) */
}

static void make_obs(const mzo_env* e, mzo_obs* o) {
  o->r = e->r; o->c = e->c;
  int br, bc;
  mzo_best_next(e, e->r, e->c, &br, &bc);
  o->best_r = e->r - br; o->best_c = e->c - bc;
  o->distance = (double)(abs(e->r - e->gr) + abs(e->c - e->gc));
  if (!e->enrich) return;
  /* get_mask_tensor (maze_handler.py:82-99): [maze==0, maze==1, non_visited] */
  int H = e->H, W = e->W;
  for (int i = 0; i < 15; ++i)
    for (int j = 0; j < 15; ++j) {
      int R, C;
      if (e->toroidal) { /* extract_submaze_toroid (maze_handler.py:56-80); N==15 -> wrap (Q8) */
        R = wrap(e->r + i - 7, H); C = wrap(e->c + j - 7, W);
      } else {
        int r0 = win_start(e->r, H), c0 = win_start(e->c, H); /* len(maze) for both axes */
        R = r0 + i; C = c0 + j;
      }
      uint8_t v = e->grid[R * W + C];
      o->window[0 * 225 + i * 15 + j] = v == 0;
      o->window[1 * 225 + i * 15 + j] = v == 1;
      o->window[2 * 225 + i * 15 + j] = e->nonvisited[R * W + C] != 0;
    }
}

/* reset: base_maze_env.py:136-161 (seed ignored, Q11) */
void mzo_env_reset(mzo_env* e, mzo_obs* o) {
  e->r = e->sr; e->c = e->sc;
  int n = e->H * e->W;
  for (int i = 0; i < n; ++i) e->nonvisited[i] = e->grid[i] != 0;
  e->nonvisited[e->sr * e->W + e->sc] = 0;
  memset(e->visits, 0, sizeof(int32_t) * n);
  e->steps = 0; e->inv = 0; e->nmoves = 0;
  if (o) {
    make_obs(e, o);
    o->reward = 0.0; o->truncated = 0; o->terminated = 0;
  }
}

/* step: base_maze_env.py:163-210 with the move rule of maze_view.py:167-197 */
void mzo_env_step(mzo_env* e, int a, mzo_obs* o) {
  double reward = 0.0;
  int term = 0, trunc = 0;
  int H = e->H, W = e->W;
  int nr = e->r + DR[a], nc = e->c + DC[a];
  int moved;
  if (e->toroidal) {
    nr = wrap(nr, H); nc = wrap(nc, W);
    moved = e->grid[nr * W + nc] != 0;
  } else {
    moved = 0 < nr && nr < H - 1 && 0 < nc && nc < W - 1 && e->grid[nr * W + nc] != 0;
  }
  if (moved) {
    int pr = e->r, pc = e->c;
    e->r = nr; e->c = nc;
    e->inv = 0;
    int cnt = e->visits[nr * W + nc];
    if (cnt == 0) {
      e->nonvisited[nr * W + nc] = 0;
      if (nr == e->gr && nc == e->gc) { reward = 1; term = 1; }
      else {
        int new_d = path_len(e, nr, nc, -1), old_d = path_len(e, pr, pc, -1);
        volatile double t = (double)(old_d - new_d) * 0.5;
        reward = t - 0.05;
      }
    } else {
      volatile double ex = exp(-0.2 * (double)cnt);
      reward = 0.0 - (1.0 - ex);
    }
    e->visits[nr * W + nc] = cnt + 1;
    e->nmoves += 1;
    e->prev_r = pr; e->prev_c = pc;
  } else {
    e->inv += 1;
    volatile double ex = exp(-0.15 * (double)e->inv);
    reward = 0.0 - (1.0 - ex);
  }
  if (o) make_obs(e, o);
  e->steps += 1;
  if (e->steps > e->max_steps) { trunc = 1; reward = -1; }
  if (o) { o->reward = reward; o->truncated = trunc; o->terminated = term; }
}

void mzo_env_mask(const mzo_env* e, int probs, float out[4]) {
  for (int k = 0; k < 4; ++k) {
    int a = e->r + DR[k], b = e->c + DC[k];
    if (e->toroidal) { a = wrap(a, e->H); b = wrap(b, e->W); }
    out[k] = e->grid[a * e->W + b] != 0 ? 1.0f : 0.0f;
  }
  if (!probs || e->nmoves <= 1) return;
  int dir;
  if (!e->toroidal) { /* simple_maze_env.py:45-49 */
    int dr = e->prev_r - e->r, dc = e->prev_c - e->c;
    dir = dr == 1 ? 0 : dr == -1 ? 1 : dc == 1 ? 2 : 3;
  } else { /* toroidal_maze_env.py:61-68 (transposed lookup, Q6) */
    int dy = wrap(e->prev_r - e->r, e->H), dx = wrap(e->prev_c - e->c, e->W);
    int x = dx <= e->W / 2 ? dx : dx - e->W;
    int y = dy <= e->H / 2 ? dy : dy - e->H;
    dir = (x == 1 && y == 0) ? 0 : (x == -1 && y == 0) ? 1 : (x == 0 && y == 1) ? 2 : 3;
  }
  out[dir] = 0.25f;
}

/* ------------------------------------------------------------------------------------------ */
/* CPU baseline driver */
typedef struct {
  const uint8_t* grid; int H, W, tor, enrich, sr, sc, gr, gc, astar;
  int nenv; long steps; uint64_t seed; long done_steps;
} bench_arg;

static uint64_t splitmix(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static void* bench_worker(void* p) {
  bench_arg* a = (bench_arg*)p;
  mzo_env* envs = (mzo_env*)malloc(sizeof(mzo_env) * a->nenv);
  mzo_obs o;
  for (int i = 0; i < a->nenv; ++i) {
    mzo_env_init(&envs[i], a->grid, a->H, a->W, a->tor, a->enrich, a->sr, a->sc, a->gr, a->gc, a->astar);
    mzo_env_reset(&envs[i], &o);
  }
  uint64_t s = a->seed;
  long n = 0;
  for (long t = 0; t < a->steps; ++t)
    for (int i = 0; i < a->nenv; ++i) {
      float m[4];
      mzo_env_mask(&envs[i], 1, m); /* reference exploration distribution (dqn_agent.py:110-112) */
      float tot = m[0] + m[1] + m[2] + m[3];
      float u = (float)((splitmix(&s) >> 40) * (1.0 / 16777216.0)) * tot;
      int act = 0;
      while (act < 3 && u >= m[act]) { u -= m[act]; ++act; }
      mzo_env_step(&envs[i], act, &o);
      ++n;
      if (o.terminated || o.truncated) mzo_env_reset(&envs[i], &o);
    }
  for (int i = 0; i < a->nenv; ++i) mzo_env_free(&envs[i]);
  free(envs);
  a->done_steps = n;
  return NULL;
}

double mzo_bench(const uint8_t* grid, int H, int W, int toroidal, int enrich, int sr, int sc,
                 int gr, int gc, int astar_mode, int nenv, long steps_per_env, int threads,
                 uint64_t seed, long* total_steps) {
  if (threads < 1) threads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
  bench_arg* args = (bench_arg*)malloc(sizeof(bench_arg) * threads);
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int i = 0; i < threads; ++i) {
    bench_arg a = {grid, H, W, toroidal, enrich, sr, sc, gr, gc, astar_mode,
                   nenv / threads + (i < nenv % threads), steps_per_env, seed + 7919ull * i, 0};
    args[i] = a;
    pthread_create(&th[i], NULL, bench_worker, &args[i]);
  }
  long tot = 0;
  for (int i = 0; i < threads; ++i) { pthread_join(th[i], NULL); tot += args[i].done_steps; }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  free(th); free(args);
  if (total_steps) *total_steps = tot;
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
