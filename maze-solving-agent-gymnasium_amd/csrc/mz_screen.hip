// mz_screen.hip — McClendon difficulty of best-of-C candidates without the reference's float
// order: one 64-lane wave per candidate, on the cell-space form the build leaves (mz_screen.h).
//
// The reference (lib/maze_difficulty_evaluation/maze_complexity_evaluation.py:38-329) computes
// p = prod_b (C_b + 1) * C_0 with C_h = D_h * sum_e 1 / (2 d_e) and takes math.log(p); best-of-C
// keeps the first candidate with the smallest log (base_maze_env.py:78-97). Which hallways exist,
// which edges each holds and which branch each lies in do not depend on CPython's set order —
// only the order of the float sums and products does (csrc/mz_mcclendon.hip reproduces that order
// bit for bit, at ~280 us of a whole CU per 81 x 81 maze). Here the same sums and products are
// formed in any order, so p carries a relative error against the reference's value that is
// bounded by the rounding count: every operand is positive, so a quantity formed with k
// roundings is within gamma_k = k u / (1 - k u) of its exact value (u = 2^-53) in both
// evaluations, and |p_ref - p| <= 2 gamma_K p with K the total rounding count. The candidate
// selection (k_cand_pick, mz_env.hip) decides a group only when its minimum is separated from
// every other candidate by more than those bounds (plus 2^-40 so the logs cannot round together);
// any other group goes to the order-exact kernel.
//
// Structure, for a perfect maze on the cell lattice (all three generators): every point
// (turn / junction / dead end / start / goal) is a cell; a cell's parent is its neighbour one
// step nearer the goal; a point's parent point pp(x) is the first point up its corridor, and the
// contracted edge (x, pp(x)) has d = A(x) - A(pp(x)) - 1 squares between (A: distance to the goal
// in squares). Hallways (extract_hallways :186-221) are the components of the off-solution,
// non-junction points along pp links, plus the junctions adjacent to them up to the reference's
// break (:208-214): a node's adjacency is [the child its first dead-end path came through,
// parent, other children by first()] (create_graph_branch :115-123 over the dead ends in row-major
// order), so a solution junction as parent excludes the later children's junctions — only a
// degree-4 node has such children. Branches (get_branches :223-259) are the components of the
// off-solution points and the solution junctions; each hallway lies in the branch of its nodes.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mz_common.h"
#include "mz_screen.h"

namespace {

constexpr int WV = 64;
constexpr uint16_t NONE = 0xFFFF;
constexpr uint8_t F_DEG = 7, F_PT = 8, F_SOL = 16, F_EXCL = 128;
constexpr int F_PD = 5;  // bits 5-6: direction of the parent (0 up, 1 down, 2 left, 3 right)

__device__ inline int fdeg(uint8_t f) { return f & F_DEG; }
__device__ inline bool fpt(uint8_t f) { return (f & F_PT) != 0; }
__device__ inline bool fsol(uint8_t f) { return (f & F_SOL) != 0; }
__device__ inline int fpd(uint8_t f) { return (f >> F_PD) & 3; }
__device__ inline bool fj(uint8_t f) { return (f & F_DEG) == 3; }
// hallway node: an off-solution point that is not a junction
__device__ inline bool fh(uint8_t f) { return fpt(f) && !fsol(f) && !fj(f); }
// branch node: an off-solution point or a solution junction
__device__ inline bool fb(uint8_t f) { return fpt(f) && (!fsol(f) || fj(f)); }

struct ScrL {
  uint8_t* pas;
  uint16_t* A;
  uint32_t* sol;
  uint8_t* fl;
  uint16_t *pp, *X, *Y, *Z;  // parent point; hallway root; branch root / rank; ranks, first()
  double* S;                 // [Hmax] hallway sums of 1 / (2 d)
  uint32_t* D;               // [Hmax] hallway sums of d
  uint16_t* hb;              // [Hmax] hallway branch rank (over pas: dead after step 1)
  double* Cb;                // [Bmax] branch sums
  int* sh;
  int Hmax, Bmax;
};

__host__ __device__ inline size_t a16(size_t x) { return (x + 15) & ~(size_t)15; }

// LDS plan for candidates of stride Qp (cells, a multiple of 16); base null: bytes only
__host__ __device__ inline size_t scr_layout(int Qp, ScrL* L, uint8_t* base) {
  const size_t Q = (size_t)Qp, QW = (Q + 31) / 32;
  // (32.4 KB at 81 x 81: five waves per CU; a maze past these caps is declined -> exact kernel)
  const int Hmax = Qp / 2, Bmax = Qp / 4 + 16;
  size_t off = 0;
  auto take = [&](size_t bytes) { uint8_t* p = base ? base + off : nullptr; off += a16(bytes); return p; };
  uint8_t* sh = take(64);
  uint8_t* pas = take(Q);
  uint8_t* A = take(2 * Q);
  uint8_t* sol = take(4 * QW);
  uint8_t* fl = take(Q);
  uint8_t* pp = take(2 * Q);
  uint8_t* X = take(2 * Q);
  uint8_t* Y = take(2 * Q);
  uint8_t* Z = take(2 * Q);
  uint8_t* S = take(8 * (size_t)Hmax);
  uint8_t* Cb = take(8 * (size_t)Bmax);
  uint8_t* D = take(4 * (size_t)Hmax);
  if (L) {
    L->sh = reinterpret_cast<int*>(sh);
    L->pas = pas;
    L->A = reinterpret_cast<uint16_t*>(A);
    L->sol = reinterpret_cast<uint32_t*>(sol);
    L->fl = fl;
    L->pp = reinterpret_cast<uint16_t*>(pp);
    L->X = reinterpret_cast<uint16_t*>(X);
    L->Y = reinterpret_cast<uint16_t*>(Y);
    L->Z = reinterpret_cast<uint16_t*>(Z);
    L->S = reinterpret_cast<double*>(S);
    L->Cb = reinterpret_cast<double*>(Cb);
    L->D = reinterpret_cast<uint32_t*>(D);
    L->hb = reinterpret_cast<uint16_t*>(pas);  // 2 Hmax = Qp bytes
    L->Hmax = Hmax;
    L->Bmax = Bmax;
  }
  return off;
}

__device__ inline double shfl_xor_d(double v, int m) {
  const long long b = __double_as_longlong(v);
  const int lo = __shfl_xor((int)(uint32_t)b, m), hi = __shfl_xor((int)(uint32_t)(b >> 32), m);
  return __longlong_as_double(((long long)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ inline int wsum_i(int x) {
  for (int o = WV / 2; o; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

// MZ_SCREEN_PROF (profiling builds only): block 0 prints the clock at each step boundary
#ifndef MZ_SCREEN_PROF
#define MZ_SCREEN_PROF 0
#endif
#define SCR_T(k)                                                       \
  do {                                                                 \
    if (MZ_SCREEN_PROF) scr_ts[(k) + 1] = __builtin_readcyclecounter(); \
  } while (0)
__device__ void screen_one(const MzCompact& cc, int t, uint8_t* lds, double* out,
                           int32_t* status) {
  const int lane = threadIdx.x;
  unsigned long long scr_ts[11] = {};
  ScrL L;
  scr_layout(cc.Qp, &L, lds);
  const uint32_t meta = cc.meta[t];
  const int N = meta & 0x7F, s = (int)((meta >> 8) & 0xFFFu), g = (int)(meta >> 20);
  const int W = (N - 1) / 2, Q = W * W, QW = (Q + 31) / 32;
  auto fail = [&]() {
    if (lane == 0) {
      out[2 * t] = 0.0;
      out[2 * t + 1] = 0.0;
      status[t] = 2;
    }
  };
  SCR_T(-1);
  if ((meta & MZ_CMETA_NOSOL) || W < 2 || Q > cc.Qp || s >= Q || g >= Q || s == g) { fail(); return; }
  // exact division by W for q < 4096 (W <= 63): q * ceil(2^18 / W) >> 18
  const uint32_t mW = ((1u << 18) + (uint32_t)W - 1u) / (uint32_t)W;
  auto rowof = [&](int q) { return (int)(((uint32_t)q * mW) >> 18); };
  auto nb = [&](int q, int k) { return k == 0 ? q - W : (k == 1 ? q + W : (k == 2 ? q - 1 : q + 1)); };
  {  // the candidate: passages and distances as words (the strides are multiples of 16 cells)
    const uint32_t* gp = reinterpret_cast<const uint32_t*>(cc.pas + (size_t)t * cc.Qp);
    const uint32_t* ga = reinterpret_cast<const uint32_t*>(cc.dist + (size_t)t * cc.Qp);
    const uint32_t* gs = cc.sol + (size_t)t * cc.QWp;
    uint32_t* lp = reinterpret_cast<uint32_t*>(L.pas);
    uint32_t* la = reinterpret_cast<uint32_t*>(L.A);
    for (int i = lane; i < (Q + 3) / 4; i += WV) lp[i] = gp[i];
    for (int i = lane; i < (Q + 1) / 2; i += WV) la[i] = ga[i];
    for (int i = lane; i < QW; i += WV) L.sol[i] = gs[i];
  }
  SCR_T(0);
  __syncthreads();
  auto solbit = [&](int q) { return ((L.sol[q >> 5] >> (q & 31)) & 1u) != 0; };
  // ---- 1. per cell: degree, parent direction, point / solution flags; the maze must be a
  // spanning tree whose distances fall by 2 squares per step toward the goal
  int bad = 0, nedge = 0;
  // (2 cells per lane and pass, every load of both issued before any of their flag stores: the
  // byte stores may alias any LDS read, so a cell-at-a-time loop waited out each cell's reads)
  for (int q0 = lane; q0 < Q; q0 += 2 * WV) {
    uint8_t pq[2], pu[2], pl[2];
    uint16_t aq[2], au[2], ad[2], al[2], ar[2];
    uint32_t sw[2];
    int rr[2], cc_[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int q = min(q0 + u * WV, Q - 1);
      rr[u] = rowof(q);
      cc_[u] = q - rr[u] * W;
      pq[u] = L.pas[q];
      pu[u] = L.pas[max(q - W, 0)];
      pl[u] = L.pas[max(q - 1, 0)];
      aq[u] = L.A[q];
      au[u] = L.A[max(q - W, 0)];
      ad[u] = L.A[min(q + W, Q - 1)];
      al[u] = L.A[max(q - 1, 0)];
      ar[u] = L.A[min(q + 1, Q - 1)];
      sw[u] = L.sol[q >> 5];
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int q = q0 + u * WV;
      if (q >= Q) continue;
      const int r = rr[u], c = cc_[u];
      const bool up = r > 0 && (pu[u] & 2), dn = (pq[u] & 2) != 0;
      const bool lf = c > 0 && (pl[u] & 1), rt = (pq[u] & 1) != 0;
      if ((dn && r == W - 1) || (rt && c == W - 1)) bad = 1;
      nedge += (dn ? 1 : 0) + (rt ? 1 : 0);
      const int deg = (int)up + (int)dn + (int)lf + (int)rt;
      const int Aq = aq[u];
      int pd = -1;
      if (q != g) {
        if (up && au[u] + 2 == Aq) pd = 0;
        if (dn && ad[u] + 2 == Aq) pd = 1;
        if (lf && al[u] + 2 == Aq) pd = 2;
        if (rt && ar[u] + 2 == Aq) pd = 3;
        if (pd < 0) bad = 1;
      } else if (Aq != 0 || deg != 1) {
        bad = 1;  // the goal is a dead end (find_random_position keeps one-neighbour squares)
      }
      const bool corner = deg == 2 && !(up && dn) && !(lf && rt);
      const bool pt = deg != 2 || corner || q == s || q == g;
      const bool sb = ((sw[u] >> (q & 31)) & 1u) != 0;
      L.fl[q] = (uint8_t)(deg | (pt ? F_PT : 0) | (sb ? F_SOL : 0) | ((pd < 0 ? 0 : pd) << F_PD));
    }
  }
  SCR_T(1);
  nedge = wsum_i(nedge);
  if (__any(bad) || nedge != Q - 1 || !solbit(s) || !solbit(g)) { fail(); return; }
  __syncthreads();
  // ---- 2. parent points: up the corridor to the first point
  for (int q = lane; q < Q; q += WV) {
    const uint8_t f = L.fl[q];
    uint16_t p = NONE;
    if (fpt(f) && q != g) {
      int y = nb(q, fpd(f)), k = 0;
      for (uint8_t fy = L.fl[y]; !fpt(fy) && k < Q; fy = L.fl[y], ++k) y = nb(y, fpd(fy));
      p = (uint16_t)y;
    }
    L.pp[q] = p;
  }
  __syncthreads();
  SCR_T(2);
  // ---- 3. hallway 0, the solution branch (:65-71): its edges, in any order
  double s0 = 0.0;
  long d0 = 0;
  int n0 = 0;
  for (int q = lane; q < Q; q += WV) {
    const uint8_t f = L.fl[q];
    if (!fpt(f) || !fsol(f) || q == g) continue;
    const int d = (int)L.A[q] - (int)L.A[L.pp[q]] - 1;
    if (d <= 0) bad = 1;
    s0 = n0 ? __dadd_rn(s0, __ddiv_rn(1.0, 2.0 * d)) : __ddiv_rn(1.0, 2.0 * d);
    d0 += d;
    ++n0;
  }
  if (__any(bad)) { fail(); return; }
  for (int o = WV / 2; o; o >>= 1) {
    const double y = shfl_xor_d(s0, o);
    const int ny = __shfl_xor(n0, o);
    s0 = n0 ? (ny ? __dadd_rn(s0, y) : s0) : y;  // an empty partial is no term (no + 0.0)
    d0 += (long)__shfl_xor((int)d0, o);  // d0 < 2^31 (at most the maze's squares)
    n0 += ny;
  }
  SCR_T(3);
  // ---- 4. the break's excluded junctions: a degree-4 hallway node p whose parent is a solution
  // junction adds only its first child's junction before the break; its first child is the one
  // whose subtree holds the smallest dead end (row-major) below p. Every off-solution point x gets
  // T(x), its topmost off-solution ancestor point, and C(x), the point just below T(x) on the way
  // up from x (pointer jumping over (T, C) pairs packed in one word, in the S region — free until
  // step 7); each dead end e offers itself to M[T(e)] (atomicMin, in the X / Y region — both
  // re-initialised in step 5); p's first child is then C(M[p]).
  bool need = false;
  auto child_pt = [&](int q, int k) {  // the first point down the corridor from q in direction k
    int y = nb(q, k);
    for (int it = 0; it < Q && !fpt(L.fl[y]); ++it) y = nb(y, k);
    return y;
  };
  auto brk = [&](int q) {  // q: a degree-4 hallway node under a solution junction
    const uint8_t f = L.fl[q];
    if (!fh(f) || fdeg(f) != 4) return false;
    const uint8_t fp = L.fl[L.pp[q]];
    return fsol(fp) && fj(fp);
  };
  for (int q = lane; q < Q; q += WV)
    if (brk(q)) {
      int nj = 0;
      for (int k = 0; k < 4; ++k)
        if (k != fpd(L.fl[q]) && fj(L.fl[child_pt(q, k)])) ++nj;
      if (nj) need = true;
    }
  if (__any(need)) {
    uint32_t* TC = reinterpret_cast<uint32_t*>(L.S);  // T | C << 16
    uint32_t* M = reinterpret_cast<uint32_t*>(L.X);
    for (int q = lane; q < Q; q += WV) {
      const uint8_t f = L.fl[q];
      uint32_t tc = 0xFFFFFFFFu;
      if (fpt(f) && !fsol(f)) {
        const int p = L.pp[q];
        tc = fsol(L.fl[p]) ? ((uint32_t)q | ((uint32_t)q << 16)) : ((uint32_t)p | ((uint32_t)q << 16));
      }
      TC[q] = tc;
      M[q] = 0xFFFFFFFFu;
    }
    __syncthreads();
    bool tconv = false;
    for (int it = 0; it < 20 && !tconv; ++it) {
      bool ch = false;
      for (int q0 = lane; q0 < Q; q0 += 4 * WV) {
        uint32_t tc[4], ta[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) tc[u] = q0 + u * WV < Q ? TC[q0 + u * WV] : 0xFFFFFFFFu;
#pragma unroll
        for (int u = 0; u < 4; ++u) ta[u] = tc[u] != 0xFFFFFFFFu ? TC[tc[u] & 0xFFFFu] : 0u;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (tc[u] == 0xFFFFFFFFu) continue;
          if ((ta[u] & 0xFFFFu) != (tc[u] & 0xFFFFu)) {  // not at a top: jump, keep the target's C
            TC[q0 + u * WV] = ta[u];
            ch = true;
          }
        }
      }
      tconv = !__any(ch);
      __syncthreads();
    }
    if (!tconv) { fail(); return; }
    for (int q = lane; q < Q; q += WV) {
      const uint8_t f = L.fl[q];
      if (fdeg(f) == 1 && !fsol(f)) atomicMin(&M[TC[q] & 0xFFFFu], (uint32_t)q);
    }
    __syncthreads();
    for (int q = lane; q < Q; q += WV) {
      if (!brk(q)) continue;
      const uint32_t m = M[q];
      const int fc = m == 0xFFFFFFFFu ? -1 : (int)(TC[m] >> 16);
      const int pd = fpd(L.fl[q]);
      for (int k = 0; k < 4; ++k) {
        if (k == pd) continue;
        const int cp = child_pt(q, k);
        if (cp != fc && fj(L.fl[cp])) L.fl[cp] |= F_EXCL;
      }
    }
    __syncthreads();
  }
  SCR_T(4);
  // ---- 5. hallway roots (X) and branch roots (Y): pointer jumping up the pp links, each round
  // over a worklist of the entries that moved in the previous one (an entry whose target is
  // already a root never moves again), compacted by wave ballots into the Z / S regions (free
  // until steps 6 / 7)
  uint16_t* WLs[2] = {L.Z, reinterpret_cast<uint16_t*>(L.S)};
  int nw = 0;
  for (int b0 = 0; b0 < Q; b0 += WV) {
    const int q = b0 + lane;
    bool live = false;
    if (q < Q) {
      const uint8_t f = L.fl[q];
      uint16_t x = NONE, y = NONE;
      const int p = L.pp[q];
      if (fh(f)) x = fh(L.fl[p]) ? (uint16_t)p : (uint16_t)q;
      if (fb(f)) y = (p != NONE && fb(L.fl[p])) ? (uint16_t)p : (uint16_t)q;
      L.X[q] = x;
      L.Y[q] = y;
      live = (x != NONE && x != q) || (y != NONE && y != q);
    }
    const unsigned long long m = __ballot(live);
    if (live) WLs[0][nw + __popcll(m & ((1ull << lane) - 1ull))] = (uint16_t)q;
    nw += __popcll(m);
  }
  __syncthreads();
  for (int it = 0, cur = 0; it < 20 && nw > 0; ++it, cur ^= 1) {
    const uint16_t* wl = WLs[cur];
    uint16_t* wn = WLs[cur ^ 1];
    int mw = 0;
    for (int i0 = 0; i0 < nw; i0 += 4 * WV) {  // 4 entries' loads in flight per lane
      int q[4], a[4], b[4], c[4], d[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) q[u] = i0 + u * WV + lane < nw ? (int)wl[i0 + u * WV + lane] : -1;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a[u] = q[u] >= 0 ? L.X[q[u]] : NONE;
        c[u] = q[u] >= 0 ? L.Y[q[u]] : NONE;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        b[u] = a[u] != NONE ? L.X[a[u]] : NONE;
        d[u] = c[u] != NONE ? L.Y[c[u]] : NONE;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        bool moved = false;
        if (a[u] != NONE && b[u] != a[u]) { L.X[q[u]] = (uint16_t)b[u]; moved = true; }
        if (c[u] != NONE && d[u] != c[u]) { L.Y[q[u]] = (uint16_t)d[u]; moved = true; }
        const unsigned long long m = __ballot(moved);
        if (moved) wn[mw + __popcll(m & ((1ull << lane) - 1ull))] = (uint16_t)q[u];
        mw += __popcll(m);
      }
    }
    nw = mw;
    __syncthreads();
  }
  if (nw > 0) { fail(); return; }
  SCR_T(5);
  // ---- 6. branch ranks (Z at the branch roots), then each hallway root's branch rank (Y)
  int Bn = 0;
  for (int b0 = 0; b0 < Q; b0 += WV) {
    const int q = b0 + lane;
    const bool r = q < Q && fb(L.fl[q]) && L.Y[q] == q;
    const unsigned long long m = __ballot(r);
    if (r) L.Z[q] = (uint16_t)(Bn + __popcll(m & ((1ull << lane) - 1ull)));
    Bn += __popcll(m);
  }
  if (Bn > L.Bmax) { fail(); return; }
  __syncthreads();
  for (int q = lane; q < Q; q += WV)
    if (fh(L.fl[q]) && L.X[q] == q) L.Y[q] = L.Z[L.Y[q]];
  __syncthreads();
  SCR_T(6);
  // ---- 7. hallway ranks (Z at the hallway roots), accumulators
  int Hn = 0;
  for (int b0 = 0; b0 < Q; b0 += WV) {
    const int q = b0 + lane;
    const bool r = q < Q && fh(L.fl[q]) && L.X[q] == q;
    const unsigned long long m = __ballot(r);
    if (r) {
      const int h = Hn + __popcll(m & ((1ull << lane) - 1ull));
      if (h < L.Hmax) {
        L.Z[q] = (uint16_t)h;
        L.hb[h] = L.Y[q];
        L.S[h] = 0.0;
        L.D[h] = 0u;
      }
    }
    Hn += __popcll(m);
  }
  if (Hn > L.Hmax) { fail(); return; }
  for (int b = lane; b < Bn; b += WV) L.Cb[b] = 0.0;
  __syncthreads();
  SCR_T(7);
  // ---- 8. every off-solution edge (x, pp(x)) into the hallway that holds it
  int nt = 0;
  for (int q = lane; q < Q; q += WV) {
    const uint8_t f = L.fl[q];
    if (!fpt(f) || fsol(f)) continue;
    const int p = L.pp[q];
    const uint8_t fp = L.fl[p];
    int h = -1;
    if (fh(f)) {
      if (fh(fp) || fj(fp)) h = L.Z[L.X[q]];  // inside the hallway, or to an adjacent junction
    } else if (fh(fp) && !(f & F_EXCL)) {
      h = L.Z[L.X[p]];  // a junction child of a hallway node
    }
    if (h < 0) continue;
    const int d = (int)L.A[q] - (int)L.A[p] - 1;
    if (d <= 0) bad = 1;
    atomicAdd(&L.S[h], __ddiv_rn(1.0, 2.0 * d));
    atomicAdd(&L.D[h], (uint32_t)d);
    ++nt;
  }
  if (__any(bad)) { fail(); return; }
  __syncthreads();
  SCR_T(8);
  // ---- 9. C_h = D_h * S_h into its branch; the product over branches, then C_0
  for (int h = lane; h < Hn; h += WV)
    atomicAdd(&L.Cb[L.hb[h]], __dmul_rn((double)L.D[h], L.S[h]));
  __syncthreads();
  double pr = 1.0;
  for (int b = lane; b < Bn; b += WV) pr = __dmul_rn(pr, __dadd_rn(L.Cb[b], 1.0));
  for (int o = WV / 2; o; o >>= 1) pr = __dmul_rn(pr, shfl_xor_d(pr, o));
  nt = wsum_i(nt);
  if (lane == 0) {
    const double c0 = __dmul_rn((double)d0, s0);
    const double prod = __dmul_rn(pr, c0);
    // roundings of either evaluation: a division and an addition per term, a product and a
    // branch addition per hallway, (C_b + 1) and a product per branch, C_0 and the last product,
    // and the wave's 63 products here (margin: factor 2.5 over 2 gamma_K)
    const double K = 2.0 * (double)(nt + n0) + 2.0 * Hn + 3.0 * Bn + 72.0;
    out[2 * t] = prod;
    out[2 * t + 1] = 2.5 * K * 0x1p-53;
    status[t] = (prod > 0.0 && prod < __longlong_as_double(0x7FF0000000000000ll)) ? 0 : 2;
  }
  SCR_T(9);
  if (MZ_SCREEN_PROF && lane == 0 && blockIdx.x == 0)
    printf("scr %d %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu\n", t, scr_ts[1] - scr_ts[0],
           scr_ts[2] - scr_ts[1], scr_ts[3] - scr_ts[2], scr_ts[4] - scr_ts[3], scr_ts[5] - scr_ts[4],
           scr_ts[6] - scr_ts[5], scr_ts[7] - scr_ts[6], scr_ts[8] - scr_ts[7], scr_ts[9] - scr_ts[8],
           scr_ts[10] - scr_ts[9]);
}

__global__ __launch_bounds__(WV) void k_screen(MzCompact cc, int n, double* out, int32_t* status,
                                               const int* limit, int mult) {
  extern __shared__ __align__(16) uint8_t lds[];
  const int m = limit ? min(*limit, n / mult) * mult : n;
  for (int t = blockIdx.x; t < m; t += gridDim.x) {
    screen_one(cc, t, lds, out, status);
    __syncthreads();  // the next candidate reuses the LDS
  }
}

}  // namespace

// resident screens (0 = as many as the LDS holds, 5 per CU at 81 x 81): beside the trainer's
// other streams 3 per CU leave them LDS — training 75.3 -> 77.6 M env steps/s at 768 (1,024:
// 75.4 M; profiles/r06t/)
#ifndef MZ_SCREEN_WGS
#define MZ_SCREEN_WGS 768
#endif

size_t mz_screen_lds(int P) { return scr_layout((mz_compact_qp(P) + 15) & ~15, nullptr, nullptr); }

hipError_t mz_launch_screen(const MzCompact& cc, int P, int n, double* out, int32_t* status,
                            hipStream_t s, const int* limit, int mult) {
  if (n <= 0) return hipSuccess;
  const size_t bytes = scr_layout(cc.Qp, nullptr, nullptr);
  if (bytes > 160 * 1024 || cc.Qp < mz_compact_qp(P)) return hipErrorInvalidValue;
  if (bytes > 65536) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_screen),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return e;
  }
  const int per_cu = (int)(160 * 1024 / bytes) > 0 ? (int)(160 * 1024 / bytes) : 1;
  int grid = n < 256 * per_cu ? n : 256 * per_cu;
  if (MZ_SCREEN_WGS > 0 && grid > MZ_SCREEN_WGS) grid = MZ_SCREEN_WGS;
  hipLaunchKernelGGL(k_screen, dim3(grid), dim3(WV), bytes, s, cc, n, out, status, limit,
                     mult < 1 ? 1 : mult);
  return hipGetLastError();
}
