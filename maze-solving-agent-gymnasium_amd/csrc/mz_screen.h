// mz_screen.h — best-of-C candidates in compact form and their order-free McClendon screen
// (mz_screen.hip; the candidate builds / pick / expand kernels live in mz_env.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "mz_common.h"

// A euclidean Philox candidate as the cell-space build leaves it, before any table is written:
// Q = W * W cells (W = (N - 1) / 2, cell q = (r >> 1) * W + (c >> 1) of square (r, c)), per cell
// its passages to the right / lower neighbour (bits 0 / 1), its distance to the goal in squares,
// and the solution path (the goal's root path in the start-rooted carve tree) as a bit set.
// cmeta = N | start cell << 8 | goal cell << 20; N bit 7 set: no solution bits (the build's
// distance field came from its BFS fallback) — the screen then declines the candidate.
struct MzCompact {
  uint8_t* pas;    // [cap][Qp]
  uint16_t* dist;  // [cap][Qp]
  uint32_t* sol;   // [cap][QWp]
  uint32_t* meta;  // [cap]
  int Qp, QWp;     // per-candidate strides: Qp = (P / 2)^2, QWp = (Qp + 31) / 32
};
#define MZ_CMETA_NOSOL 0x80u

__host__ __device__ inline int mz_compact_qp(int P) { return (P / 2) * (P / 2); }

// Test hooks of the best-of-C pipeline (mz_set_debug): every group to the order-exact kernel;
// treat even-numbered candidates as declined by it (scored on the host); all C candidates of a
// group from one seed (exact ties: the first must win).
#define MZ_DBG_SCREEN_OFF 1
#define MZ_DBG_DECLINE_EVEN 2
#define MZ_DBG_TWIN 4

// candidate c of target id: Philox seed (mz_generate_best / bank refills)
__host__ __device__ inline uint64_t mz_cand_seed(uint64_t seed, uint64_t id, int C, int c,
                                                 uint32_t epoch, int dbg) {
  return seed + id * (uint64_t)C + (uint64_t)((dbg & MZ_DBG_TWIN) ? 0 : c) + ((uint64_t)epoch << 32);
}

// out[2 t] = prod_b (C_b + 1) * C_0 computed in an order of its own, out[2 t + 1] = e, a bound on
// |prod_ref - prod| / prod for the reference's float64 evaluation order (any order of the same
// sums and products): status[t] 0 ok, 2 declined (the exact kernel decides). limit / mult as
// mz_launch_mcclendon.
size_t mz_screen_lds(int P);
hipError_t mz_launch_screen(const MzCompact& cc, int P, int n, double* out, int32_t* status,
                            hipStream_t s, const int* limit = nullptr, int mult = 1);
