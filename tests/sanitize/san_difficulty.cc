// san_difficulty.cc — AddressSanitizer / UndefinedBehaviorSanitizer driver for the product's host
// C++ (csrc/mz_difficulty.hip: the McClendon restatement behind mz_difficulty /
// mz_maze_complexity, maze_complexity_evaluation.py:38-329), compiled as plain C++ with the
// sanitizers by tests/sanitize/Makefile and run by tests/test_sanitizers.py. Mazes come from the
// CPU oracle's generators (linked in as test infrastructure): perfect mazes of every generator
// and size the parity tests use, bordered toroidal grids (gen_maze_no_border), mazes with cycles
// (walls knocked out: the A*-path branch of the restatement), and degenerate inputs (goal
// unreachable, start == goal neighbour) that must return a status, never fault. Values are
// pinned elsewhere (tests/test_difficulty.py against the reference's fixtures).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "../../include/mazerl.h"
extern "C" {
#include "../../oracle/mzoracle.h"
}

static int failures = 0;
#define CHECK(cond, ...)                                               \
  do {                                                                 \
    if (!(cond)) {                                                     \
      std::fprintf(stderr, "CHECK failed %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                               \
      std::fputc('\n', stderr);                                        \
      ++failures;                                                      \
    }                                                                  \
  } while (0)

static void score(const std::vector<uint8_t>& g, int N, int sr, int sc, int gr, int gc,
                  bool must_succeed) {
  double d = 0.0, dd = 0.0, cx = 0.0;
  const int rc = mz_difficulty(g.data(), N, N, sr, sc, gr, gc, &d);
  const int rc2 = mz_maze_complexity(g.data(), N, N, sr, sc, gr, gc, &dd, &cx);
  if (must_succeed) {
    CHECK(rc == MZ_OK && rc2 == MZ_OK, "rc %d / %d at N=%d", rc, rc2, N);
    CHECK(std::isfinite(d) && d == dd, "difficulty %g vs %g", d, dd);
    CHECK(std::isfinite(cx), "complexity %g", cx);
  }
}

int main() {
  const int sizes[] = {9, 15, 21, 41, 81, 127};
  std::vector<uint8_t> g(129 * 129);
  uint64_t seed = 0xD1FF0000ull;
  for (int algo = 0; algo < 3; ++algo)
    for (int N : sizes)
      for (int s = 0; s < 3; ++s) {
        int sr, sc, gr, gc;
        std::vector<uint8_t> m(N * N);
        CHECK(mzo_generate(m.data(), N, N, 0, algo, ++seed, &sr, &sc, &gr, &gc) == 0, "gen");
        score(m, N, sr, sc, gr, gc, true);
        // cycles: knock out every 7th interior wall between two floor cells
        std::vector<uint8_t> c = m;
        int k = 0;
        for (int r = 1; r < N - 1; ++r)
          for (int q = 1; q < N - 1; ++q)
            if (!c[r * N + q] && ((r & 1) != (q & 1)) && (++k % 7) == 0) c[r * N + q] = 1;
        score(c, N, sr, sc, gr, gc, true);
        // goal walled in: unreachable -> a status, no fault
        std::vector<uint8_t> u = m;
        for (int dr = -1; dr <= 1; ++dr)
          for (int dq = -1; dq <= 1; ++dq)
            if ((dr || dq) && gr + dr >= 0 && gr + dr < N && gc + dq >= 0 && gc + dq < N)
              u[(gr + dr) * N + gc + dq] = 0;
        score(u, N, sr, sc, gr, gc, false);
      }
  // toroidal: the bordered (N + 2) grid that gen_maze_no_border scores (:37-56)
  for (int algo = 0; algo < 3; ++algo)
    for (int N : {9, 17, 29, 41, 79})
      for (int s = 0; s < 2; ++s) {
        int sr, sc, gr, gc;
        const int M = N + 2;
        std::vector<uint8_t> m(M * M);
        CHECK(mzo_generate(m.data(), M, M, 0, algo, ++seed, &sr, &sc, &gr, &gc) == 0, "gen");
        score(m, M, sr, sc, gr, gc, true);
      }
  // argument validation
  double d;
  CHECK(mz_difficulty(g.data(), 15, 15, 1, 1, 13, 13, nullptr) != MZ_OK, "null out accepted");
  CHECK(mz_maze_complexity(g.data(), 15, 15, 1, 1, 13, 13, nullptr, nullptr) != MZ_OK, "null outs");
  std::vector<uint8_t> walls(15 * 15, 0);
  (void)mz_difficulty(walls.data(), 15, 15, 1, 1, 13, 13, &d);
  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::printf("san_difficulty ok\n");
  return 0;
}
