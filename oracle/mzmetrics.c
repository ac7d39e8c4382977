/* mzmetrics.c — the reference's maze-metric suite (TEST INFRASTRUCTURE ONLY, in libmzoracle.so).
 *
 * Restates MetricsCalculator (reference lib/maze_difficulty_evaluation/metrics_calculator.py)
 * as generation_algos_metrics_evaluations.py uses it on a generated maze:
 *   L  = len(solution) / CE, CE = (H-1)*((W-1)//2) - 1                       (:11-26)
 *   D  = #{solution cells with > 2 open neighbours} / len(solution)           (:73-88)
 *   DE = (AC + FDE + BDE) / len(solution) from calculate_DE_sub               (:90-133):
 *        dead ends = value-1 cells with one open neighbour, off the solution, row-major (:135-144);
 *        de_path = A* path dead end -> solution[0], cut before its first solution cell when that
 *        index is <= len(solution) - 2 (calculate_path :146-157, loop bound kept as written);
 *        a dead end is counted only if its de_path shares no cell with the decision points kept
 *        so far; it then records its first interior cell with > 2 open neighbours as a decision
 *        point; type_of_DE (:159-180): FDE / BDE (by the Manhattan distance to the goal of the
 *        path's end vs its start) if the path has an interior junction or any turn, else AC.
 * The mazes are perfect (a tree over open cells), so every A* path is the unique tree path:
 * taken from BFS parents rooted at the start. Pinned by tests/test_metrics.py against the
 * reference's own values (tests/golden/metrics.npz).
 */
#include <stdlib.h>
#include <string.h>

#include "mzoracle.h"

static int nb_open(const uint8_t* g, int W, int v) {
  return (g[v - W] != 0) + (g[v + W] != 0) + (g[v - 1] != 0) + (g[v + 1] != 0);
}

int mzo_metrics(const uint8_t* g, int H, int W, int sr, int sc, int gr, int gc, double* out) {
  const int n = H * W, s = sr * W + sc, goal = gr * W + gc;
  int* dist = (int*)malloc(sizeof(int) * n);
  int* onpath = (int*)malloc(sizeof(int) * n);   /* index in solution, -1 off path */
  char* dec = (char*)calloc(n, 1);                /* decision_points kept so far */
  int* sol = (int*)malloc(sizeof(int) * n);
  int* dp = (int*)malloc(sizeof(int) * n);
  mzo_bfs(g, H, W, 0, sr, sc, dist);
  if (dist[goal] < 0) { free(dist); free(onpath); free(dec); free(sol); free(dp); return -1; }
  /* parent of v (tree): the open neighbour one step closer to the start */
  #define PARENT(v) (dist[(v) - W] == dist[v] - 1 && g[(v) - W] ? (v) - W :        \
                     dist[(v) + W] == dist[v] - 1 && g[(v) + W] ? (v) + W :        \
                     dist[(v) - 1] == dist[v] - 1 && g[(v) - 1] ? (v) - 1 : (v) + 1)
  const int len = dist[goal] + 1;
  for (int i = 0; i < n; ++i) onpath[i] = -1;
  for (int v = goal, k = len - 1; k >= 0; --k) {
    sol[k] = v;
    onpath[v] = k;
    if (k) v = PARENT(v);
  }
  int dcount = 0;
  for (int k = 0; k < len; ++k)
    if (nb_open(g, W, sol[k]) > 2) ++dcount;
  long ac = 0, fde = 0, bde = 0;
  for (int r = 1; r < H - 1; ++r)
    for (int c = 1; c < W - 1; ++c) {
      const int v = r * W + c;
      if (g[v] != 1 || nb_open(g, W, v) != 1 || onpath[v] >= 0) continue;
      /* de_path: v -> start, cut before the first solution cell at index <= len - 2 */
      int m = 0;
      for (int u = v;; u = PARENT(u)) {
        dp[m++] = u;
        if (u == s) break;
      }
      for (int i = 1; i < len - 1 && i < m; ++i)
        if (onpath[dp[i]] >= 0) { m = i; break; }
      int shared = 0;
      for (int i = 0; i < m && !shared; ++i) shared = dec[dp[i]];
      if (shared) continue;
      for (int k = 1; k < m - 1; ++k)
        if (nb_open(g, W, dp[k]) > 2) { dec[dp[k]] = 1; break; }
      int flag = 0;
      if (m >= 3) {
        for (int k = 1; k < m - 1 && !flag; ++k) {
          const int a = dp[k - 1], b = dp[k + 1];
          if (a / W != b / W && a % W != b % W) flag = 1; /* a turn: calculate_T > 0 */
          if (nb_open(g, W, dp[k]) > 2) flag = 1;
        }
      }
      if (!flag) { ++ac; continue; }
      const int e = dp[m - 1], b0 = dp[0];
      const int de = (abs(e / W - gr) + abs(e % W - gc)) - (abs(b0 / W - gr) + abs(b0 % W - gc));
      if (de > 0) ++fde; else ++bde;
    }
  #undef PARENT
  const int CE = (H - 1) * ((W - 1) / 2) - 1;
  out[0] = (double)len / (double)CE;
  out[1] = (double)ac / len + (double)fde / len + (double)bde / len; /* AC + FDE + BDE */
  out[2] = (double)dcount / len;
  out[3] = (double)ac / len;
  out[4] = (double)fde / len;
  out[5] = (double)bde / len;
  free(dist); free(onpath); free(dec); free(sol); free(dp);
  return 0;
}
