// mz_pygen.inc.h — CPython-exact maze generation on gfx950 (included by mz_build.inc.h).
//
// gen_maze (reference lib/maze_generation.py:6-35) as CPython 3.10 executes it, so a maze built
// from the Python `random` state of random.seed(s) is the reference's maze bit for bit:
//   random      MT19937 (state in LDS, lane 0): random.seed(int) = init_by_array; _randbelow =
//               getrandbits(bit_length(n)) with rejection; randrange(1, G-1, 2); choice;
//               shuffle (Fisher-Yates from the end) — random.py / _randommodule.c semantics.
//   set order   the frontier of random_prim_visit (:79-96) and the unmarked / marked sets and
//               intersections of prim_and_kill_visit / random_walk (:141-185) are CPython set
//               tables (Objects/setobject.c): tuple hash, 8-slot start, 9 linear probes then
//               perturbed probing, dummies on discard (an add reuses the last dummy on its probe
//               path), resize to the next power of two > 4 * used when fill * 5 >= mask * 3,
//               intersection iterating the smaller operand. tuple(set) is table order, so
//               random.choice(tuple(s)) = the k-th live slot: found by a wave-wide ballot scan.
// Set mutation runs on lane 0 (sequential, like the interpreter); scans use all 64 lanes.
// The same algorithm restated on the CPU (oracle/mzpygen.c) reproduces the reference's 240
// golden mazes; tests/test_gpu_env.py checks this path against both.
#pragma once

#define MZ_PS_EMPTY 0xFFFFu
#define MZ_PS_DUMMY 0xFFFEu

__host__ __device__ inline int mz_py_cells(int G) { return ((G - 1) / 2) * ((G - 1) / 2); }
__host__ __device__ inline int mz_pow2_above(int x) { int c = 8; while (c <= x) c <<= 1; return c; }
// Set-table capacities for a G x G generation grid: A = frontier (r-prim; a resize gives the
// next power of two > 4 * used, used <= cells) or unmarked (prim&kill), B = marked; a set that
// only grows to n entries ends at the pure-add size: 8 -> 32 -> 128 -> 512 -> 2048 -> 8192 ...
__host__ __device__ inline int mz_py_cap_grow(int n) {
  int size = 8, fill = 0;
  while (fill < n) {
    ++fill;
    if (fill * 5 >= (size - 1) * 3) size = mz_pow2_above(4 * fill);
  }
  return size;
}
__host__ __device__ inline int mz_py_cap_a(int G) {
  const int c = mz_pow2_above(4 * mz_py_cells(G)), g = mz_py_cap_grow(mz_py_cells(G));
  return c < 16384 ? c : (g > 16384 ? g : 16384);
}
__host__ __device__ inline int mz_py_cap_b(int G) { return mz_py_cap_grow(mz_py_cells(G)); }
__host__ __device__ inline size_t mz_py_lds_bytes(int G) {
  return 2592 + 2 * (size_t)mz_py_cap_a(G) + 2 * (size_t)mz_py_cap_b(G);
}

struct MzPyLds {
  uint32_t* mt;   // [625] MT19937 words + index
  int* hdr;       // per set: mask, fill, used (A: 0..2, B: 3..5); [6] error flag
  uint16_t* small;  // [16] lane 0's two 8-slot tables (set(nbrs), the intersection): LDS, not
                    // per-lane scratch memory, which data-dependent slot indices would need
  uint16_t* ta;   // [cap_a]
  uint16_t* tb;   // [cap_b]
  uint16_t* scratch;  // resize copy (the build's dist + queue region, free during generation)
  // prim&kill only, in the build's queue region (2 G^2 bytes, free while generating): its two
  // sets only grow by adds (unmarked is built, then only discarded from), so a resize copies
  // < 0.42 G^2 u16 slots and stays inside dist; these take cap_b / 8 + 2 cells < 0.7 G^2 bytes
  uint32_t* sbits;    // [cap_b / 32] slot i of the marked table is a restart candidate
  uint16_t* slot_of;  // [cells] the marked-table slot of cell (r / 2) * W + c / 2
  int cap_a, cap_b, G;
};

// ---- MT19937 (lane 0) ---------------------------------------------------------------------
__device__ inline void mz_mt_seed(uint32_t* mt, uint64_t seed) {
  uint32_t key[2];
  int klen = 0;
  key[klen++] = (uint32_t)seed;
  if (seed >> 32) key[klen++] = (uint32_t)(seed >> 32);
  mt[0] = 19650218u;
  for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
  int i = 1, j = 0;
  for (int k = 624; k; --k) {
    mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
    ++i; ++j;
    if (i >= 624) { mt[0] = mt[623]; i = 1; }
    if (j >= klen) j = 0;
  }
  for (int k = 623; k; --k) {
    mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
    ++i;
    if (i >= 624) { mt[0] = mt[623]; i = 1; }
  }
  mt[0] = 0x80000000u;
  mt[624] = 624u;
}

__device__ inline uint32_t mz_mt_u32(uint32_t* mt) {
  if (mt[624] >= 624u) {
    for (int kk = 0; kk < 624; ++kk) {
      const uint32_t y = (mt[kk] & 0x80000000u) | (mt[kk == 623 ? 0 : kk + 1] & 0x7FFFFFFFu);
      mt[kk] = mt[kk < 227 ? kk + 397 : kk - 227] ^ (y >> 1) ^ ((y & 1u) ? 0x9908B0DFu : 0u);
    }
    mt[624] = 0u;
  }
  uint32_t y = mt[mt[624]++];
  y ^= y >> 11;
  y ^= (y << 7) & 0x9D2C5680u;
  y ^= (y << 15) & 0xEFC60000u;
  y ^= y >> 18;
  return y;
}

__device__ inline uint32_t mz_mt_below(uint32_t* mt, uint32_t n) {  // _randbelow, n >= 1
  const int k = 32 - __clz(n);
  uint32_t r;
  do r = mz_mt_u32(mt) >> (32 - k); while (r >= n);
  return r;
}

// ---- CPython set of (r, c) tuples, key = r * G + c (lane 0 unless noted) --------------------
__device__ inline uint64_t mz_tuple_hash(int a, int b) {
  const uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull,
                 P5 = 2870177450012600261ull;
  uint64_t acc = P5;
  acc += (uint64_t)a * P2; acc = (acc << 31) | (acc >> 33); acc *= P1;
  acc += (uint64_t)b * P2; acc = (acc << 31) | (acc >> 33); acc *= P1;
  acc += 2ull ^ (P5 ^ 3527539ull);
  return acc == ~0ull ? 1546275796ull : acc;
}

struct MzPySet {  // a view: table + its header in LDS
  uint16_t* t;
  int* h;  // mask, fill, used
  int cap, G;
  int* err;
};

__device__ inline uint64_t mz_ps_hash(const MzPySet& s, int key) {
  return mz_tuple_hash(key / s.G, key - (key / s.G) * s.G);
}

__device__ inline void mz_ps_init(const MzPySet& s) {
  s.h[0] = 7; s.h[1] = 0; s.h[2] = 0;
  for (int i = 0; i < 8; ++i) s.t[i] = MZ_PS_EMPTY;
}

__device__ inline void mz_ps_insert_clean(const MzPySet& s, int key, uint64_t h) {
  const uint32_t mask = (uint32_t)s.h[0];
  uint64_t perturb = h;
  uint32_t i = (uint32_t)(h & mask);
  for (;;) {
    if (s.t[i] == MZ_PS_EMPTY) break;
    if (i + 9 <= mask) {
      int j = 1;
      for (; j <= 9; ++j)
        if (s.t[i + j] == MZ_PS_EMPTY) break;
      if (j <= 9) { i += j; break; }
    }
    perturb >>= 5;
    i = (uint32_t)((i * 5 + 1 + perturb) & mask);
  }
  s.t[i] = (uint16_t)key;
}

__device__ inline void mz_ps_resize(const MzPySet& s, int minused, uint16_t* scratch) {
  const int newsize = mz_pow2_above(minused);
  if (newsize > s.cap) { *s.err = 1; return; }
  const int oldn = s.h[0] + 1;
  for (int i = 0; i < oldn; ++i) scratch[i] = s.t[i];
  s.h[0] = newsize - 1;
  for (int i = 0; i < newsize; ++i) s.t[i] = MZ_PS_EMPTY;
  for (int i = 0; i < oldn; ++i)
    if (scratch[i] < MZ_PS_DUMMY) mz_ps_insert_clean(s, scratch[i], mz_ps_hash(s, scratch[i]));
  s.h[1] = s.h[2];
}

// returns the key's slot, or -2 when the insertion resized the table
__device__ inline int mz_ps_found_unused(const MzPySet& s, uint32_t i, int key, uint16_t* scratch) {
  s.h[1] += 1;
  s.h[2] += 1;
  s.t[i] = (uint16_t)key;
  if ((long)s.h[1] * 5 < (long)s.h[0] * 3) return (int)i;
  mz_ps_resize(s, s.h[2] > 50000 ? s.h[2] * 2 : s.h[2] * 4, scratch);
  return -2;
}

// set.add; returns the key's slot, or -2 when the insertion resized the table
__device__ inline int mz_ps_add(const MzPySet& s, int key, uint16_t* scratch) {
  const uint64_t h = mz_ps_hash(s, key);
  const uint32_t mask = (uint32_t)s.h[0];
  uint32_t i = (uint32_t)(h & mask);
  if (s.t[i] == MZ_PS_EMPTY) return mz_ps_found_unused(s, i, key, scratch);
  int freeslot = -1;
  uint64_t perturb = h;
  for (;;) {
    if (s.t[i] == key) return (int)i;
    if (s.t[i] == MZ_PS_DUMMY) freeslot = (int)i;
    if (i + 9 <= mask) {
      for (uint32_t j = 1; j <= 9; ++j) {
        const uint16_t t = s.t[i + j];
        if (t == MZ_PS_EMPTY) { i += j; goto unused_or_dummy; }
        if (t == key) return (int)(i + j);
        if (t == MZ_PS_DUMMY) freeslot = (int)(i + j);
      }
    }
    perturb >>= 5;
    i = (uint32_t)((i * 5 + 1 + perturb) & mask);
    if (s.t[i] == MZ_PS_EMPTY) goto unused_or_dummy;
  }
unused_or_dummy:
  if (freeslot < 0) return mz_ps_found_unused(s, i, key, scratch);
  s.h[2] += 1;
  s.t[freeslot] = (uint16_t)key;
  return freeslot;
}

__device__ inline int mz_ps_lookup(const MzPySet& s, int key) {
  const uint64_t h = mz_ps_hash(s, key);
  const uint32_t mask = (uint32_t)s.h[0];
  uint32_t i = (uint32_t)(h & mask);
  uint64_t perturb = h;
  for (;;) {
    if (s.t[i] == MZ_PS_EMPTY) return -1;
    if (s.t[i] == key) return (int)i;
    if (i + 9 <= mask) {
      for (uint32_t j = 1; j <= 9; ++j) {
        const uint16_t t = s.t[i + j];
        if (t == MZ_PS_EMPTY) return -1;
        if (t == key) return (int)(i + j);
      }
    }
    perturb >>= 5;
    i = (uint32_t)((i * 5 + 1 + perturb) & mask);
  }
}

__device__ inline void mz_ps_discard(const MzPySet& s, int key) {
  const int i = mz_ps_lookup(s, key);
  if (i < 0) return;
  s.t[i] = MZ_PS_DUMMY;
  s.h[2] -= 1;
}

// tuple(set)[k] by a wave-wide scan in table order (all lanes; k and the table uniform)
__device__ inline int mz_ps_kth_wave(const MzPySet& s, int k) {
  const int lane = threadIdx.x, n = s.h[0] + 1;
  for (int b = 0; b < n; b += 64) {
    const int i = b + lane;
    const bool live = i < n && s.t[i] < MZ_PS_DUMMY;
    unsigned long long bal = __ballot(live);
    const int pc = __popcll(bal);
    if (k < pc) {
      for (int t = 0; t < k; ++t) bal &= bal - 1;
      return s.t[b + __ffsll((long long)bal) - 1];
    }
    k -= pc;
  }
  return -1;
}

// small set (<= 4 keys, stays in its 8 slots) built from keys in order: set(list)
__device__ inline void mz_ps_small(uint16_t* t, int G, uint64_t keys, int n) {
  int h[3];
  MzPySet s{t, h, 8, G, nullptr};
  mz_ps_init(s);
  for (int i = 0; i < n; ++i) mz_ps_add(s, mz_k4(keys, i), nullptr);
}

// ---- the visits ----------------------------------------------------------------------------
// get_neighbors order (:72), packed (mz_k4)
__device__ inline int mz_py_nbrs2(int G, int p, uint64_t& out) {
  const int x = p / G, y = p - (p / G) * G;
  int n = 0;
  out = 0;
  for (int k = 0; k < 4; ++k) {
    const int a = x + mz_g2r(k), b = y + mz_g2c(k);
    if (a >= 0 && a < G && b >= 0 && b < G) mz_k4_push(out, n, a * G + b);
  }
  return n;
}

// random_prim_visit (:59-99); all lanes call, lane 0 mutates
__device__ void mz_py_rprim(const MzBuildLds& L, const MzPyLds& Y, int G, int s) {
  const int lane = threadIdx.x;
  const MzPySet fr{Y.ta, Y.hdr, Y.cap_a, G, Y.hdr + 6};
  if (lane == 0) {
    uint64_t nb;
    const int n = mz_py_nbrs2(G, s, nb);
    L.g[s] = 1;
    mz_ps_init(fr);
    for (int i = 0; i < n; ++i) mz_ps_add(fr, mz_k4(nb, i), Y.scratch);
  }
  __syncthreads();
  for (;;) {
    const int used = fr.h[2];
    if (used == 0 || Y.hdr[6]) break;
    int k = 0;
    if (lane == 0) k = (int)mz_mt_below(Y.mt, (uint32_t)used);
    k = __shfl(k, 0);
    const int f = mz_ps_kth_wave(fr, k);
    __syncthreads();
    if (lane == 0) {
      mz_ps_discard(fr, f);
      uint64_t nb, in = 0;
      int cnt = 0;
      const int n = mz_py_nbrs2(G, f, nb);
      for (int i = 0; i < n; ++i)
        if (L.g[mz_k4(nb, i)] == 1) mz_k4_push(in, cnt, mz_k4(nb, i));
      if (cnt) {
        const int q = mz_k4(in, (int)mz_mt_below(Y.mt, (uint32_t)cnt));
        const int fx = f / G, fy = f - fx * G, qx = q / G, qy = q - qx * G;
        L.g[f] = 1;
        L.g[((fx + qx) / 2) * G + (fy + qy) / 2] = 1;
        for (int i = 0; i < n; ++i)
          if (L.g[mz_k4(nb, i)] == 0) mz_ps_add(fr, mz_k4(nb, i), Y.scratch);
      }
    }
    __syncthreads();
  }
}

// deept_first_visit (:101-128), lane 0: shuffle the four directions, take the first open
__device__ void mz_py_dfs(const MzBuildLds& L, const MzPyLds& Y, int G, int s) {
  uint8_t* m = L.g;
  uint16_t* st = L.queue;
  int sp = 0;
  st[sp++] = (uint16_t)s;
  while (sp > 0) {
    const int top = st[sp - 1], x = top / G, y = top - x * G;
    uint32_t d = 0xE4u;  // directions 0, 1, 2, 3 as 2-bit fields (registers)
    for (int i = 3; i >= 1; --i) {
      const int j = (int)mz_mt_below(Y.mt, (uint32_t)(i + 1));
      const uint32_t a = (d >> (2 * i)) & 3u, b = (d >> (2 * j)) & 3u;
      d = (d & ~((3u << (2 * i)) | (3u << (2 * j)))) | (b << (2 * i)) | (a << (2 * j));
    }
    bool found = false;
    for (int k = 0; k < 4 && !found; ++k) {
      const int dk = (int)((d >> (2 * k)) & 3u);
      const int nx = x + 2 * mz_fr(dk), ny = y + 2 * mz_fc(dk);
      if (nx >= 0 && nx < G && ny >= 0 && ny < G && m[nx * G + ny] == 0) {
        m[(x + mz_fr(dk)) * G + (y + mz_fc(dk))] = 1;
        m[nx * G + ny] = 1;
        st[sp++] = (uint16_t)(nx * G + ny);
        found = true;
      }
    }
    if (!found) --sp;
  }
}

// unmarked membership as a bit per cell (L.vis): the set tables give only the ORDER
__device__ inline bool mz_py_unmarked(const MzBuildLds& L, int p) {
  return (L.vis[p >> 5] >> (p & 31)) & 1u;
}

// inters = unmarked.intersection(set(nbrs(cur))) into the 8-slot table `it` (lane 0)
__device__ inline void mz_py_inters(const MzBuildLds& L, const MzPySet& un, int G, int cur,
                                    uint16_t* st, uint16_t* it, int ih[3]) {
  uint64_t nb;
  const int n = mz_py_nbrs2(G, cur, nb);
  mz_ps_small(st, G, nb, n);
  MzPySet res{it, ih, 8, G, nullptr};
  mz_ps_init(res);
  if (n > un.h[2]) {  // len(set(nbrs)) = n > len(unmarked): iterate unmarked in table order
    for (int i = 0; i <= un.h[0]; ++i) {
      const uint16_t t = un.t[i];
      if (t >= MZ_PS_DUMMY) continue;
      for (int k = 0; k < 8; ++k)
        if (st[k] == t) { mz_ps_add(res, t, nullptr); break; }
    }
  } else {
    for (int k = 0; k < 8; ++k)
      if (st[k] < MZ_PS_DUMMY && mz_py_unmarked(L, st[k])) mz_ps_add(res, st[k], nullptr);
  }
}

// prim&kill's restart candidates ([p for p in marked if set(nbrs(p)) & unmarked], :151) in the
// order of the marked table: Y.sbits holds a bit per slot, Y.slot_of each marked cell's slot.
// The walk keeps them current as it marks cells — only the new cell and its marked neighbours
// can change — so a restart picks the k-th candidate from a scan over cap_b / 32 words instead
// of two passes over the table with four neighbour tests per slot. A resize of the marked table
// moves every slot: hdr[7] then marks the bits stale and the next restart rebuilds them with
// the whole wave.
__device__ inline int mz_py_cell(int G, int p) {
  const int r = p / G, c = p - r * G;
  return (r >> 1) * ((G - 1) >> 1) + (c >> 1);
}
__device__ inline bool mz_py_has_unmarked(const MzBuildLds& L, int G, int p) {
  uint64_t nb;
  const int n = mz_py_nbrs2(G, p, nb);
  bool any = false;
  for (int q = 0; q < n; ++q) any |= mz_py_unmarked(L, mz_k4(nb, q));
  return any;
}
__device__ inline void mz_py_sbit(uint32_t* sb, int i, bool on) {
  if (on) sb[i >> 5] |= 1u << (i & 31);
  else sb[i >> 5] &= ~(1u << (i & 31));
}

// cur has just moved from unmarked to marked at slot `slot` of the marked table (lane 0)
__device__ inline void mz_py_pk_marked(const MzBuildLds& L, const MzPyLds& Y, int G, int cur,
                                       int slot) {
  if (slot < 0) Y.hdr[7] = 1;  // the add resized the table
  if (Y.hdr[7]) return;
  Y.slot_of[mz_py_cell(G, cur)] = (uint16_t)slot;
  mz_py_sbit(Y.sbits, slot, mz_py_has_unmarked(L, G, cur));
  uint64_t nb;
  const int n = mz_py_nbrs2(G, cur, nb);
  for (int q = 0; q < n; ++q) {
    const int p = mz_k4(nb, q);
    if (mz_py_unmarked(L, p)) continue;  // every other cell 2 away is marked
    const int sl = Y.slot_of[mz_py_cell(G, p)];
    if (((Y.sbits[sl >> 5] >> (sl & 31)) & 1u) && !mz_py_has_unmarked(L, G, p))
      mz_py_sbit(Y.sbits, sl, false);
  }
}

// random_walk (:159-185), lane 0
__device__ void mz_py_walk(const MzBuildLds& L, const MzPyLds& Y, int G, int cur) {
  const MzPySet un{Y.ta, Y.hdr, Y.cap_a, G, Y.hdr + 6};
  const MzPySet mk{Y.tb, Y.hdr + 3, Y.cap_b, G, Y.hdr + 6};
  uint16_t *st = Y.small, *it = Y.small + 8;
  int ih[3];
  mz_py_inters(L, un, G, cur, st, it, ih);
  while (ih[2] > 0 && !Y.hdr[6]) {
    L.g[cur] = 1;
    int k = (int)mz_mt_below(Y.mt, (uint32_t)ih[2]), nx = -1;
    for (int i = 0; i < 8; ++i)
      if (it[i] < MZ_PS_DUMMY && k-- == 0) { nx = it[i]; break; }
    const int cx = cur / G, cy = cur - cx * G, x = nx / G, y = nx - x * G;
    L.g[(cx + (x - cx) / 2) * G + (cy + (y - cy) / 2)] = 1;
    cur = nx;
    mz_ps_discard(un, cur);
    L.vis[cur >> 5] &= ~(1u << (cur & 31));
    mz_py_pk_marked(L, Y, G, cur, mz_ps_add(mk, cur, Y.scratch));
    mz_py_inters(L, un, G, cur, st, it, ih);
  }
}

// prim_and_kill_visit (:130-157); all lanes call
__device__ void mz_py_primkill(const MzBuildLds& L, const MzPyLds& Y, int G, int s) {
  const int lane = threadIdx.x;
  const MzPySet un{Y.ta, Y.hdr, Y.cap_a, G, Y.hdr + 6};
  const MzPySet mk{Y.tb, Y.hdr + 3, Y.cap_b, G, Y.hdr + 6};
  for (int i = lane; i < (G * G + 31) / 32; i += 64) L.vis[i] = 0u;
  __syncthreads();
  if (lane == 0) {
    mz_ps_init(un);
    for (int i = 1; i < G; i += 2)
      for (int j = 1; j < G; j += 2) mz_ps_add(un, i * G + j, Y.scratch);
    mz_ps_init(mk);
  }
  __syncthreads();
  for (int i = lane; i <= un.h[0]; i += 64) {  // for i,j in unmarked: maze[i][j] = 1
    const uint16_t t = un.t[i];
    if (t < MZ_PS_DUMMY) { L.g[t] = 1; atomicOr(&L.vis[t >> 5], 1u << (t & 31)); }
  }
  __syncthreads();
  if (lane == 0) {
    mz_ps_add(mk, s, Y.scratch);
    mz_ps_discard(un, s);
    L.vis[s >> 5] &= ~(1u << (s & 31));
    L.g[s] = 1;
    Y.hdr[7] = 1;  // candidate bits built at the first restart
    mz_py_walk(L, Y, G, s);
  }
  __syncthreads();
  while (un.h[2] > 0 && !Y.hdr[6]) {
    const int n = mk.h[0] + 1, nw = (n + 31) >> 5;
    if (Y.hdr[7]) {  // rebuild the slot bits and slot_of over the whole (resized) table
      for (int b = 0; b < n; b += 64) {
        const int i = b + lane;
        bool cand = false;
        if (i < n && mk.t[i] < MZ_PS_DUMMY) {
          Y.slot_of[mz_py_cell(G, mk.t[i])] = (uint16_t)i;
          cand = mz_py_has_unmarked(L, G, mk.t[i]);
        }
        const unsigned long long bal = __ballot(cand);
        if (lane == 0) Y.sbits[b >> 5] = (uint32_t)bal;
        if (lane == 1 && b + 32 < n) Y.sbits[(b >> 5) + 1] = (uint32_t)(bal >> 32);
      }
      __syncthreads();
      if (lane == 0) Y.hdr[7] = 0;
    }
    int total = 0;
    for (int b = 0; b < nw; b += 64) {
      int pc = b + lane < nw ? __popc(Y.sbits[b + lane]) : 0;
      for (int o = 32; o > 0; o >>= 1) pc += __shfl_xor(pc, o);
      total += pc;
    }
    int k = 0;
    if (lane == 0) k = (int)mz_mt_below(Y.mt, (uint32_t)total);
    k = __shfl(k, 0);
    int chosen = -1;
    for (int b = 0; b < nw && chosen < 0; b += 64) {
      const int w = b + lane;
      const uint32_t v = w < nw ? Y.sbits[w] : 0u;
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
        int slot = 0;
        if (lane == src) {
          uint32_t m = v;
          for (int t = inc - pc; t < k; ++t) m &= m - 1;  // drop the lower candidates
          slot = w * 32 + __ffs(m) - 1;
        }
        chosen = mk.t[__shfl(slot, src)];
      } else {
        k -= tot;
      }
    }
    __syncthreads();
    if (chosen < 0) { if (lane == 0) Y.hdr[6] = 2; break; }
    if (lane == 0) mz_py_walk(L, Y, G, chosen);
    __syncthreads();
  }
}

// gen_maze's start + visit on the G x G grid L.g (zeroed): returns the start cell index.
// All lanes call; the MT state is Y.mt (already seeded / loaded).
__device__ int mz_py_generate(const MzBuildLds& L, const MzPyLds& Y, int G, int algo) {
  const int lane = threadIdx.x;
  if (lane == 0) {
    Y.hdr[6] = 0;
    // start_point = (randrange(1, rows - 1, 2), randrange(1, columns - 1, 2)) (:21)
    const int a = 1 + 2 * (int)mz_mt_below(Y.mt, (uint32_t)((G - 1) / 2));
    const int b = 1 + 2 * (int)mz_mt_below(Y.mt, (uint32_t)((G - 1) / 2));
    L.sh[2] = a * G + b;
    L.g[a * G + b] = 1;
  }
  __syncthreads();
  const int s = L.sh[2];
  if (algo == MZ_ALGO_RPRIM_DEV) mz_py_rprim(L, Y, G, s);
  else if (algo == MZ_ALGO_DFS_DEV) { if (lane == 0) mz_py_dfs(L, Y, G, s); }
  else mz_py_primkill(L, Y, G, s);
  __syncthreads();
  return s;
}
