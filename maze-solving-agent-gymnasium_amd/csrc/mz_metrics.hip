// mz_metrics.hip — the reference's maze-metric suite on the GPU, one wave per maze.
//
// generation_algos_metrics_evaluations.py evaluates generated mazes with MetricsCalculator
// (lib/maze_difficulty_evaluation/metrics_calculator.py): for the A* solution path,
//   L  = len(solution) / CE, CE = (H-1)*((W-1)//2) - 1                                (:11-26)
//   D  = #{solution cells with > 2 open neighbours} / len(solution)                    (:73-88)
//   DE = (AC + FDE + BDE) / len(solution), calculate_DE_sub                            (:90-133)
// The kernel works from the instance's cell words (open bit, open-neighbour mask, D = BFS
// distance to the goal; the mazes are perfect, so the goal-rooted BFS tree IS the maze):
//   - solution = start, then the neighbour with D - 1 until the goal (the unique tree path,
//     which is the path A* returns);
//   - a dead end's de_path (A* dead end -> start, calculate_path :146-157) climbs D - 1 steps to
//     the junction J where its branch meets the solution, then runs along the solution to the
//     start; it is cut before J when J's index is <= len(solution) - 2, the reference's loop
//     bound;
//   - dead ends are visited in row-major order (extract_de_points :135-144) and the kept
//     decision points are a bit set, exactly as calculate_DE_sub's list (order-dependent);
//   - type_of_DE (:159-180): FDE / BDE by the Manhattan distances to the goal of the path's end
//     vs its start when the path has an interior junction (> 2 open neighbours) or a turn, else AC.
// The cell words and the per-cell solution index live in LDS; lane 0 walks (the per-maze work is
// a few thousand LDS reads). Output per maze: L, DE, D, AC, FDE, BDE (float64, the reference's
// ratios: count / len(solution), DE summed left to right).
#include "mz_common.h"
#include "mz_kernels.h"

namespace {

__device__ inline int nbc(uint32_t w) { return __popc((w >> MZ_CELL_NB_SHIFT) & 0xFu); }

// the neighbour one step closer to the goal (D - 1), as a cell index
__device__ inline int toward_goal(const uint32_t* cw, int N, int v) {
  const uint32_t d = cw[v] & MZ_CELL_D_MASK;
  const int nb[4] = {v + N, v - N, v + 1, v - 1};  // BaseMazeEnv.ACTIONS order
  for (int k = 0; k < 4; ++k) {
    const uint32_t w = cw[nb[k]];
    if ((w & MZ_CELL_OPEN) && (w & MZ_CELL_D_MASK) + 1 == d) return nb[k];
  }
  return -1;
}

// next cell of a dead end's A* path to the start: toward the goal while off the solution, then
// along the solution toward its start (index - 1)
__device__ inline int de_next(const uint32_t* cw, const uint16_t* sidx, int N, int x) {
  if (sidx[x] == 0xFFFFu) return toward_goal(cw, N, x);
  const uint16_t want = (uint16_t)(sidx[x] - 1);
  const int nb[4] = {x + N, x - N, x + 1, x - 1};
  for (int k = 0; k < 4; ++k)
    if (sidx[nb[k]] == want) return nb[k];
  return x;
}

__global__ __launch_bounds__(64) void k_metrics(MzDev d, const int32_t* env_ids, int n,
                                                double* out) {
  extern __shared__ __align__(16) uint8_t lds[];
  const int lane = threadIdx.x;
  uint32_t* cw = reinterpret_cast<uint32_t*>(lds);                       // [N*N]
  uint16_t* sidx = reinterpret_cast<uint16_t*>(lds + 4 * (size_t)d.P * d.P);  // [N*N]
  uint32_t* dec = reinterpret_cast<uint32_t*>(lds + 6 * (size_t)d.P * d.P);   // bits [N*N]
  for (int j = blockIdx.x; j < n; j += gridDim.x) {
    const int e = env_ids ? env_ids[j] : j;
    const uint32_t m0 = d.meta0[e], m1 = d.meta1[e];
    const int N = m0 & 0xFF, sr = (m0 >> 16) & 0xFF, sc = m0 >> 24;
    const int gr = m1 & 0xFF, gc = (m1 >> 8) & 0xFF;
    const uint32_t* src = d.cells + (size_t)e * d.P * d.P;
    for (int i = lane; i < N * N; i += 64) {
      cw[i] = src[(i / N) * d.P + (i % N)];
      sidx[i] = 0xFFFFu;
    }
    for (int i = lane; i < (N * N + 31) / 32; i += 64) dec[i] = 0u;
    __syncthreads();
    if (lane == 0) {
      const int s = sr * N + sc, goal = gr * N + gc;
      const int len = (int)(cw[s] & MZ_CELL_D_MASK) + 1;
      int dcount = 0;
      for (int v = s, k = 0; k < len; ++k) {
        sidx[v] = (uint16_t)k;
        if (nbc(cw[v]) > 2) ++dcount;
        if (k + 1 < len) v = toward_goal(cw, N, v);
      }
      int ac = 0, fde = 0, bde = 0;
      for (int r = 1; r < N - 1; ++r)
        for (int c = 1; c < N - 1; ++c) {
          const int v = r * N + c;
          const uint32_t w = cw[v];
          if (!(w & MZ_CELL_OPEN) || v == goal || nbc(w) != 1 || sidx[v] != 0xFFFFu) continue;
          // de_path = v ... J (climb, J at index h), then the solution from J down to the start
          int h = 0, J = v;
          while (sidx[J] == 0xFFFFu) { J = toward_goal(cw, N, J); ++h; }
          const int q = sidx[J];
          const int m = (h <= len - 2) ? h : h + q + 1;  // cut before J, or the whole path
          bool shared = false;
          for (int i = 0, x = v; i < m && !shared; ++i, x = de_next(cw, sidx, N, x))
            shared = (dec[x >> 5] >> (x & 31)) & 1u;
          if (shared) continue;
          bool flag = false, recorded = false;
          int endcell = v;
          for (int i = 0, x = v, px = -1, ppx = -1; i < m; ++i) {
            if (i >= 1 && i <= m - 2 && nbc(cw[x]) > 2) {  // interior junction
              flag = true;
              if (!recorded) { dec[x >> 5] |= 1u << (x & 31); recorded = true; }
            }
            if (i >= 2 && ppx / N != x / N && ppx % N != x % N) flag = true;  // turn at i - 1
            endcell = x;
            ppx = px;
            px = x;
            if (i + 1 < m) x = de_next(cw, sidx, N, x);
          }
          if (m < 3) flag = false;
          if (!flag) { ++ac; continue; }
          const int ddist = (abs(endcell / N - gr) + abs(endcell % N - gc)) -
                            (abs(r - gr) + abs(c - gc));
          if (ddist > 0) ++fde; else ++bde;
        }
      const double L = (double)len, CE = (double)((N - 1) * ((N - 1) / 2) - 1);
      double* o = out + 6 * (size_t)j;
      o[0] = __ddiv_rn(L, CE);
      o[1] = __dadd_rn(__dadd_rn(__ddiv_rn((double)ac, L), __ddiv_rn((double)fde, L)),
                       __ddiv_rn((double)bde, L));
      o[2] = __ddiv_rn((double)dcount, L);
      o[3] = __ddiv_rn((double)ac, L);
      o[4] = __ddiv_rn((double)fde, L);
      o[5] = __ddiv_rn((double)bde, L);
    }
    __syncthreads();
  }
}

}  // namespace

size_t mz_metrics_lds_bytes(int P) { return 6 * (size_t)P * P + 4 * (((size_t)P * P + 31) / 32) + 16; }

hipError_t mz_launch_metrics(const MzDev& d, const int32_t* env_ids, int32_t n, double* out,
                             hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const size_t lds = mz_metrics_lds_bytes(d.P);
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k_metrics),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_metrics, dim3(n < 4096 ? n : 4096), dim3(64), lds, s, d, env_ids, n, out);
  return hipGetLastError();
}
