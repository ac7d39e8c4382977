/* mzoracle.h — CPU restatement of the reference maze-env hot path. TEST INFRASTRUCTURE ONLY.
 *
 * This library is the parity checker for the HIP product (libmazerl.so). Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it. The product never links
 * or calls it. Pinned against tests/golden/ fixtures ( produced by running the reference's own
 * Python code, tests/golden/make_golden.py).
 *
 * Conventions: grids are row-major uint8 H*W with 0 = wall, 1 = floor, 2 = goal
 * (reference lib/maze_generation.py:16). Coordinates are (row, col).
 */
#ifndef MZORACLE_H
#define MZORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* BFS distances from (sr,sc) over open cells, 4-neighbour, wrapping when toroidal.
 * dist[i] = -1 for walls / unreachable. Returns number of reached cells. */
int mzo_bfs(const uint8_t* grid, int H, int W, int toroidal, int sr, int sc, int32_t* dist);

/* Faithful restatement of astar_limited_partial (lib/a_star_algos/a_star.py:9-82,
 * a_star_tor.py:15-88): heap ordered like Python's heapq on (f,(r,c)); no closed set; returns
 * len(path) of the full or partial path. max_depth < 0 means the reference default 1e6. */
int mzo_astar_len(const uint8_t* grid, int H, int W, int toroidal, int sr, int sc, int gr, int gc,
                  int max_depth);

/* find_random_position (lib/maze_generation.py:187-218): farthest dead-end odd cell from start,
 * first in row-major order on ties. Returns 0 and (gr,gc), or -1 if no candidate. */
int mzo_goal_select(const uint8_t* grid, int H, int W, int sr, int sc, int* gr, int* gc);

/* set_max_steps (simple_maze_env.py:52-58 / toroidal_maze_env.py:71-77) with
 * MetricsCalculator.calculate_L (metrics_calculator.py:11-26). IEEE double, no contraction. */
int mzo_max_steps(const uint8_t* grid, int H, int W, int toroidal, int sr, int sc, int gr, int gc);

/* Maze generators restated over a Philox4x32-10 stream (identical stream use to the HIP
 * kernels in csrc/mz_generate.hip): algo 0 = r-prim, 1 = dfs, 2 = prim&kill
 * (maze_generation.py:59-185). Writes an H*W grid with the goal placed (find_random_position).
 * toroidal=1: generates (H+2)x(W+2), selects the goal there, then crops (maze_generation.py:37-56).
 * Returns 0 on success. */
int mzo_generate(uint8_t* grid, int H, int W, int toroidal, int algo, uint64_t seed,
                 int* sr, int* sc, int* gr, int* gc);

/* CPython-exact generation (mzpygen.c): gen_maze((N,N), algo) (toroidal: gen_maze_no_border)
 * exactly as CPython 3.10 runs it from the random.Random state `state` (624 MT19937 words +
 * the index, as in random.getstate()[1]); the state is advanced in place. Returns 0. */
int mzo_generate_py(uint8_t* grid, int N, int toroidal, int algo, uint32_t* state, int* sr,
                    int* sc, int* gr, int* gc);
/* random.seed(seed) state for 0 <= seed < 2^64 (init_by_array) -> state[625] */
void mzo_mt_seed(uint64_t seed, uint32_t* state);
/* random._randbelow(n) on state (advances it) */
uint32_t mzo_mt_below(uint32_t* state, uint32_t n);
/* hash((a, b)) of CPython 3.10 for small non-negative ints, as uint64 */
uint64_t mzo_tuple_hash(int a, int b);

/* MetricsCalculator (metrics_calculator.py) on the solution path of a perfect euclidean maze:
 * out[6] = L, DE, D, AC, FDE, BDE (mzmetrics.c). Returns 0, or -1 if the goal is unreachable. */
int mzo_metrics(const uint8_t* grid, int H, int W, int sr, int sc, int gr, int gc, double* out);

/* Philox4x32-10 block for (key, counter) -> 4 words (for RNG stream tests). */
void mzo_philox(uint64_t key, uint64_t ctr_hi, uint64_t ctr_lo, uint32_t out[4]);

/* ---------------- single-instance env (BaseMazeEnv.step/reset, base_maze_env.py:136-210) ------ */
typedef struct {
  int H, W, toroidal, enrich;
  int sr, sc, gr, gc;
  int max_steps;
  int astar_mode; /* 1 = reference cost model (A* per find_path), 0 = BFS distance field */
  uint8_t* grid;  /* owned copy */
  int32_t* D;     /* BFS distance to goal */
  int32_t* visits; /* entries into each cell since reset (visited_cell.count) */
  uint8_t* nonvisited; /* the reference's non_visited plane */
  int r, c;
  int steps, inv;
  int nmoves;   /* len(visited_cell) */
  int prev_r, prev_c; /* visited_cell[-2] when nmoves >= 2 */
} mzo_env;

typedef struct {
  double reward;
  int truncated, terminated;
  int r, c;            /* agent location */
  int best_r, best_c;  /* "best dir" = agent - best_next_cell */
  double distance;     /* info["distance"] */
  uint8_t window[675]; /* 3x15x15 channel planes as 0/1 (enrich only) */
} mzo_obs;

int mzo_env_init(mzo_env* e, const uint8_t* grid, int H, int W, int toroidal, int enrich,
                 int sr, int sc, int gr, int gc, int astar_mode);
void mzo_env_free(mzo_env* e);
void mzo_env_reset(mzo_env* e, mzo_obs* o);
void mzo_env_step(mzo_env* e, int action, mzo_obs* o);
/* get_mask_direction(probs) (simple_maze_env.py:41-50, toroidal_maze_env.py:57-69) */
void mzo_env_mask(const mzo_env* e, int probs, float out[4]);
/* _find_best_next_cell (base_maze_env.py:224-262) at (r,c): writes best next cell. */
void mzo_best_next(const mzo_env* e, int r, int c, int* nr, int* nc);

/* Batched driver used by bench.py's cpu_baseline leg: runs `steps` steps of `nenv` independent
 * envs (the same grid), actions from the reference exploration distribution with a splitmix64
 * stream, auto-reset on done; `threads` pthreads. Returns elapsed seconds. */
double mzo_bench(const uint8_t* grid, int H, int W, int toroidal, int enrich, int sr, int sc,
                 int gr, int gc, int astar_mode, int nenv, long steps_per_env, int threads,
                 uint64_t seed, long* total_steps);

#ifdef __cplusplus
}
#endif
#endif
