/* san_oracle.c — AddressSanitizer / UndefinedBehaviorSanitizer driver for the CPU oracle
 * (oracle/mzoracle.c, mzpygen.c, mzmetrics.c: TEST INFRASTRUCTURE). Built and run by
 * tests/test_sanitizers.py through
 * tests/sanitize/Makefile with -fsanitize=address,undefined -fno-sanitize-recover=all, so any
 * out-of-bounds access, use after free, leak, signed overflow or misaligned access aborts with a
 * non-zero status. It drives every oracle entry point over the configurations the parity tests
 * use (euclidean 15/21/41/81 Enrich, plain 9, toroidal 9/17/29/41; the three
 * generators, Philox and CPython-exact), and checks the cheap invariants that need no fixture:
 * A* length == min(D, depth) + 1 (a5), the goal is a dead end (a12), rewards in the reference's
 * set (a1). Values proper are pinned by tests/test_oracle_golden.py. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/mzoracle.h"

static int failures = 0;
#define CHECK(cond, ...)                                   \
  do {                                                     \
    if (!(cond)) {                                         \
      fprintf(stderr, "CHECK failed %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                        \
      fputc('\n', stderr);                                 \
      ++failures;                                          \
    }                                                      \
  } while (0)

static uint64_t sm_state = 0x9E3779B97F4A7C15ull;
static uint64_t splitmix(void) {
  uint64_t z = (sm_state += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* one maze through every per-maze entry point, then an episode stream with resets */
static void drive(const uint8_t* g, int N, int tor, int enrich, int sr, int sc, int gr, int gc,
                  int steps) {
  int32_t* D = (int32_t*)malloc(sizeof(int32_t) * N * N);
  int reached = mzo_bfs(g, N, N, tor, gr, gc, D);
  CHECK(reached > 0, "bfs reached %d", reached);
  CHECK(D[sr * N + sc] >= 0, "start unreachable");
  /* a5: A* length == min(D, depth) + 1 on a sample of open cells */
  for (int k = 0; k < 16; ++k) {
    const int i = (int)(splitmix() % (uint64_t)(N * N));
    if (!g[i] || D[i] < 0) continue;
    const int depth = (int)(splitmix() % 64) + 1;
    const int l = mzo_astar_len(g, N, N, tor, i / N, i % N, gr, gc, depth);
    const int want = (D[i] < depth ? D[i] : depth) + 1;
    CHECK(l == want, "astar_len %d != %d (N=%d tor=%d)", l, want, N, tor);
  }
  if (!tor) {
    int gr2 = -1, gc2 = -1;
    CHECK(mzo_goal_select(g, N, N, sr, sc, &gr2, &gc2) == 0, "goal_select");
    const int open_nb = (g[(gr - 1) * N + gc] != 0) + (g[(gr + 1) * N + gc] != 0) +
                        (g[gr * N + gc - 1] != 0) + (g[gr * N + gc + 1] != 0);
    CHECK(open_nb == 1, "goal is not a dead end (%d open neighbours)", open_nb);
    double m[6];
    CHECK(mzo_metrics(g, N, N, sr, sc, gr, gc, m) == 0, "metrics");
    for (int k = 0; k < 6; ++k) CHECK(isfinite(m[k]), "metric %d not finite", k);
  }
  const int ms = mzo_max_steps(g, N, N, tor, sr, sc, gr, gc);
  CHECK(ms > 0, "max_steps %d", ms);

  for (int astar = 0; astar < 2; ++astar) {
    mzo_env e;
    CHECK(mzo_env_init(&e, g, N, N, tor, enrich, sr, sc, gr, gc, astar) == 0, "env_init");
    mzo_obs o;
    mzo_env_reset(&e, &o);
    const int n = astar ? steps / 8 : steps;
    for (int t = 0; t < n; ++t) {
      float m[4];
      mzo_env_mask(&e, 1, m);
      const float tot = m[0] + m[1] + m[2] + m[3];
      int a = (int)(splitmix() & 3);
      if (tot > 0.f && (splitmix() & 1)) {  /* the reference exploration distribution */
        float x = (float)((splitmix() >> 40) * (1.0 / 16777216.0)) * tot;
        a = 0;
        while (a < 3 && x >= m[a]) { x -= m[a]; ++a; }
      }
      mzo_env_step(&e, a, &o);
      const double r = o.reward;
      CHECK(r >= -1.0 && r <= 1.0, "reward %g", r);
      int br, bc;
      mzo_best_next(&e, o.r, o.c, &br, &bc);
      if (o.terminated || o.truncated) mzo_env_reset(&e, &o);
    }
    mzo_env_free(&e);
  }
  free(D);
}

int main(void) {
  static const int euclid[] = {15, 21, 41, 81};
  static const int torus[] = {9, 17, 29, 41};
  uint8_t* g = (uint8_t*)malloc(127 * 127);
  for (int algo = 0; algo < 3; ++algo)
    for (int s = 0; s < 3; ++s) {
      int sr, sc, gr, gc;
      for (int k = 0; k < 4; ++k) {  /* Philox generators */
        const int N = euclid[k];
        CHECK(mzo_generate(g, N, N, 0, algo, 0x5EED0000ull + 97 * s + k, &sr, &sc, &gr, &gc) == 0,
              "generate %d %d", algo, N);
        drive(g, N, 0, 1, sr, sc, gr, gc, 600);
        const int T = torus[k];
        CHECK(mzo_generate(g, T, T, 1, algo, 0x70500000ull + 97 * s + k, &sr, &sc, &gr, &gc) == 0,
              "generate torus %d %d", algo, T);
        drive(g, T, 1, T != 15, sr, sc, gr, gc, 600);
      }
      CHECK(mzo_generate(g, 9, 9, 0, algo, 0x9000ull + s, &sr, &sc, &gr, &gc) == 0, "generate 9");
      drive(g, 9, 0, 0, sr, sc, gr, gc, 300);  /* config 1's plain 9x9 */
      uint32_t st[625];
      mzo_mt_seed((uint64_t)s, st);
      for (int k = 0; k < 3; ++k) {  /* CPython-exact generators from random.seed(s) */
        const int N = euclid[k];
        CHECK(mzo_generate_py(g, N, 0, algo, st, &sr, &sc, &gr, &gc) == 0, "generate_py %d %d", algo, N);
        drive(g, N, 0, 1, sr, sc, gr, gc, 200);
        const int T = torus[k + 1];
        CHECK(mzo_generate_py(g, T, 1, algo, st, &sr, &sc, &gr, &gc) == 0, "generate_py torus");
        drive(g, T, 1, 1, sr, sc, gr, gc, 200);
      }
    }
  /* Philox and the CPython helpers */
  uint32_t out[4];
  mzo_philox(1, 2, 3, out);
  uint32_t st[625];
  mzo_mt_seed(12345, st);
  for (int k = 1; k < 1000; ++k) CHECK(mzo_mt_below(st, (uint32_t)k) < (uint32_t)k, "below");
  (void)mzo_tuple_hash(3, 5);
  /* the threaded cpu_baseline driver, both cost models */
  {
    int sr, sc, gr, gc;
    CHECK(mzo_generate(g, 41, 41, 0, 0, 7, &sr, &sc, &gr, &gc) == 0, "generate 41");
    long total = 0;
    (void)mzo_bench(g, 41, 41, 0, 1, sr, sc, gr, gc, 1, 4, 200, 2, 1, &total);
    CHECK(total == 800, "bench total %ld", total);
    (void)mzo_bench(g, 41, 41, 0, 1, sr, sc, gr, gc, 0, 4, 2000, 4, 2, &total);
    CHECK(total == 8000, "bench total %ld", total);
  }
  free(g);
  if (failures) {
    fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  printf("san_oracle ok\n");
  return 0;
}
