// mz_api.hip — host side of the C ABI declared in include/mazerl.h.
//
// Owns the per-handle HBM state (layout: mz_common.h), validates arguments the way the
// reference fails (even N -> IndexError, window with N < 15 -> crash: reported as
// MZ_EINVAL_SHAPE), builds the exact penalty tables once (glibc exp, like CPython's math.exp),
// and launches the kernels of mz_env.hip. No compute path runs on the host: every env quantity is
// produced by a gfx950 kernel.
#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mazerl.h"
#include "mz_common.h"
#include "mz_learner.h"
#include "mz_mcclendon.h"

// Candidate mazes of a best-of-C selection (maze bank refills with C > 1, mz_generate_best): an
// MzDev view over `cap` scratch instances (cells, plane strips, per-instance words) plus the
// McClendon output per candidate.
// Candidates the order-exact kernel declines, scored by the host restatement (mz_difficulty.hip)
// inside the stream: k_cand_gather writes their grids to mapped host memory, the stream runs
// host_fallback_fn (hipLaunchHostFunc), k_cand_select reads the products back.
struct MzHostFallback {
  int cap = 0, gstride = 0;
  uint8_t *grid_h = nullptr, *grid_d = nullptr;  // [cap][gstride]
  int32_t *info_h = nullptr, *info_d = nullptr;  // [cap][5]: N, sr, sc, gr, gc
  double *prod_h = nullptr, *prod_d = nullptr;   // [cap]
  int32_t *ok_h = nullptr, *ok_d = nullptr;      // [cap]
  int32_t* count_h = nullptr;                    // mapped: the gathered count, copied in-stream
  int* count_d = nullptr;                        // device: k_cand_gather's slot counter
  int32_t* map = nullptr;                        // device [candidates]: host slot or -1
};

struct MzCandStore {
  int cap = 0;
  MzDev v{};
  double* score = nullptr;    // [cap][2]: prod_b (C_b + 1) * C_0, sum (k_mcclendon)
  int32_t* status = nullptr;  // [cap]
  // euclidean handles: the compact candidates, their screen and the per-target pick
  MzCompact cc{};
  double* sscore = nullptr;    // [cap][2]: screened product, relative bound (mz_screen.hip)
  int32_t* sstatus = nullptr;  // [cap]
  int32_t* pick = nullptr;     // [cap] per target: the candidate, -1 = the exact path
  int32_t* xlist = nullptr;    // [kXCap] targets for the order-exact kernel
  int* xcount = nullptr;
  MzHostFallback hf;
};

struct MzBankStore {  // two banks x the enabled algorithms x sizes x K slots (mz_bank_*)
  int K = 0, nA = 0, nD = 0;
  int C = 1;                   // candidates per slot (best-of-C by McClendon difficulty)
  MzCandStore cand;            // K * C candidates (C > 1), reused by every block's refill
  int dims[MZ_BANK_MAX_DIMS] = {};
  uint32_t amask = 0;
  uint32_t* cells = nullptr;   // [2][nA][nD][K][P*P]
  uint32_t* planes = nullptr;  // [2][nA][nD][K][PW]
  uint32_t* meta0 = nullptr;   // [2][nA][nD][K]
  uint32_t* meta1 = nullptr;
  int* heads = nullptr;        // [2][3][nD] consumed slots per (algorithm id, size)
  int* slot = nullptr;         // [3][nD][ceil(B / 64)] winners' first slot per group (k_reset_done)
  int8_t* code = nullptr;      // [B] each instance's winner code before a reset launch (MzDev::bk_code)
  // scratch the build writes and nobody reads: [K] ...
  uint32_t *s_posw = nullptr, *s_stw = nullptr, *s_curw = nullptr;
  uint8_t *s_last = nullptr, *s_algo = nullptr;
  uint32_t epoch[2] = {0u, 0u};
};

struct mz_handle {
  mz_config cfg;
  MzDev d;
  std::vector<void*> allocs;
  uint8_t* staging = nullptr;
  size_t staging_bytes = 0;
  MzBankStore bank;
  MzCandStore gen;             // mz_generate_best's candidates (chunks of the instance list)
  int* sel_stats = nullptr;    // [8] best-of-C selections: unresolved groups, near ties, groups,
                               // groups the screen left to the exact kernel, host-scored candidates
  int dbg = 0;                 // MZ_DBG_* test hooks of the best-of-C pipeline (mz_set_debug)
  std::vector<void*> host_allocs;  // mapped page-locked host memory (hipHostFree)
  MzCompact scr{};             // mz_screen_batch's compact scratch
  int scr_cap = 0;
};

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define MZ_HIP(x)                                                                      \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) return fail(MZ_EHIP, "%s: %s", #x, hipGetErrorString(e_));   \
  } while (0)

struct DeviceGuard {  // run a call on the handle's device, restore the caller's afterwards
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// Entry points that take device pointers and a stream but no handle run on the stream's device
// (the caller's current device for the null stream), restoring the caller's device afterwards.
struct StreamGuard {
  int prev = -1;
  explicit StreamGuard(void* stream) {
    hipDevice_t dev;
    if (!stream || hipStreamGetDevice(static_cast<hipStream_t>(stream), &dev) != hipSuccess) return;
    if (hipGetDevice(&prev) != hipSuccess) { prev = -1; return; }
    if (prev != (int)dev) (void)hipSetDevice((int)dev);
  }
  ~StreamGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

MzOut to_dev(const mz_step_out* o) {
  MzOut m;
  std::memset(&m, 0, sizeof m);
  if (!o) return m;
  m.reward = o->reward; m.reward64 = o->reward64; m.terminated = o->terminated;
  m.truncated = o->truncated; m.pos = o->pos; m.best_dir = o->best_dir; m.obs6 = o->obs6;
  m.window_bits = o->window_bits; m.window = o->window; m.done_idx = o->done_idx;
  m.done_count = o->done_count;
  return m;
}

int check_out(const mz_step_out* o) {
  if (o && o->window && (reinterpret_cast<uintptr_t>(o->window) & 15u))
    return fail(MZ_EALIGN, "window output must be 16-byte aligned");
  if (o && o->done_idx && !o->done_count) return fail(MZ_EINVAL, "done_idx needs done_count");
  return MZ_OK;
}

int check_dim(const mz_handle* h, int dim) {
  if (dim < 5 || dim > h->cfg.max_dim)
    return fail(MZ_EINVAL_SHAPE, "maze dim %d outside [5, max_dim=%d]", dim, h->cfg.max_dim);
  if ((dim & 1) == 0)
    return fail(MZ_EINVAL_SHAPE, "even maze dim %d (reference gen_maze raises IndexError, "
                "lib/maze_generation.py:197-203)", dim);
  if (h->cfg.enrich && !h->cfg.toroidal && dim < 15)
    return fail(MZ_EINVAL_SHAPE, "euclidean window needs dim >= 15 (extract_submaze, "
                "lib/maze_handler.py:18-45)");
  return MZ_OK;
}

template <typename T>
int alloc(mz_handle* h, T** p, size_t count) {
  void* q = nullptr;
  hipError_t e = hipMalloc(&q, count * sizeof(T) + 64);
  if (e != hipSuccess) return fail(MZ_ENOMEM, "hipMalloc(%zu): %s", count * sizeof(T), hipGetErrorString(e));
  h->allocs.push_back(q);
  MZ_HIP(hipMemset(q, 0, count * sizeof(T) + 64));
  *p = static_cast<T*>(q);
  return MZ_OK;
}

template <typename T>
int host_alloc(mz_handle* h, T** hp, T** dp, size_t count) {
  void* q = nullptr;
  hipError_t e = hipHostMalloc(&q, count * sizeof(T) + 64, hipHostMallocMapped | hipHostMallocCoherent);
  if (e != hipSuccess) return fail(MZ_ENOMEM, "hipHostMalloc(%zu): %s", count * sizeof(T), hipGetErrorString(e));
  h->host_allocs.push_back(q);
  std::memset(q, 0, count * sizeof(T) + 64);
  void* d = nullptr;
  e = hipHostGetDevicePointer(&d, q, 0);
  if (e != hipSuccess) return fail(MZ_EHIP, "hipHostGetDevicePointer: %s", hipGetErrorString(e));
  *hp = static_cast<T*>(q);
  *dp = static_cast<T*>(d);
  return MZ_OK;
}

constexpr int kXCap = 256;  // targets per best-of-C run the order-exact kernel can take
constexpr int kHCap = 256;  // declined candidates per run the host restatement can take

int compact_alloc(mz_handle* h, MzCompact& cc, int cap) {
  const int Qp = (mz_compact_qp(h->d.P) + 15) & ~15;
  cc.Qp = Qp;
  cc.QWp = (Qp + 31) / 32;
  int rc;
  if ((rc = alloc(h, &cc.pas, (size_t)cap * Qp)) || (rc = alloc(h, &cc.dist, (size_t)cap * Qp)) ||
      (rc = alloc(h, &cc.sol, (size_t)cap * cc.QWp)) || (rc = alloc(h, &cc.meta, (size_t)cap)))
    return rc;
  return MZ_OK;
}

// the host restatement of the candidates k_cand_gather listed (runs on a HIP runtime thread in
// stream order: no HIP calls here)
void host_fallback_fn(void* arg) {
  MzHostFallback* f = static_cast<MzHostFallback*>(arg);
  const int n = std::min(*f->count_h, f->cap);
  for (int i = 0; i < n; ++i) {
    const int32_t* in = f->info_h + 5 * (size_t)i;
    double p = 0.0;
    const int rc = mz_mcclendon_host_prod(f->grid_h + (size_t)i * f->gstride, in[0], in[0], in[1],
                                          in[2], in[3], in[4], &p);
    f->prod_h[i] = p;
    f->ok_h[i] = rc == MZ_OK && p > 0.0;
  }
}

// scratch for `cap` candidate mazes: a view of the handle's layout over its own arrays
int cand_alloc(mz_handle* h, MzCandStore& cs, int cap) {
  const MzDev& d = h->d;
  MzDev v = d;
  const size_t n = (size_t)cap, P = (size_t)d.P;
  int rc;
  if ((rc = alloc(h, &v.cells, n * P * P)) || (rc = alloc(h, &v.planes, n * (size_t)d.PW + 16)) ||
      (rc = alloc(h, &v.meta0, n)) || (rc = alloc(h, &v.meta1, n)) || (rc = alloc(h, &v.posw, n)) ||
      (rc = alloc(h, &v.stw, n)) || (rc = alloc(h, &v.curw, n)) || (rc = alloc(h, &v.algo, n)) ||
      (rc = alloc(h, &v.last_term, n)) || (rc = alloc(h, &cs.score, 2 * n)) ||
      (rc = alloc(h, &cs.status, n)))
    return rc;
  v.B = cap;
  v.bk_K = 0;
  v.regen_dim = nullptr;
  cs.v = v;
  cs.cap = cap;
  MzHostFallback& hf = cs.hf;
  int32_t* count_dview = nullptr;  // (the count's device view: unused, the copy lands on the host)
  hf.cap = kHCap;
  hf.gstride = (d.P + 2) * (d.P + 2);
  if ((rc = host_alloc(h, &hf.grid_h, &hf.grid_d, (size_t)hf.cap * hf.gstride)) ||
      (rc = host_alloc(h, &hf.info_h, &hf.info_d, (size_t)hf.cap * 5)) ||
      (rc = host_alloc(h, &hf.prod_h, &hf.prod_d, (size_t)hf.cap)) ||
      (rc = host_alloc(h, &hf.ok_h, &hf.ok_d, (size_t)hf.cap)) ||
      (rc = host_alloc(h, &hf.count_h, &count_dview, 1)) || (rc = alloc(h, &hf.count_d, 1)) ||
      (rc = alloc(h, &hf.map, n)))
    return rc;
  if (!d.toroidal) {
    if ((rc = compact_alloc(h, cs.cc, cap)) || (rc = alloc(h, &cs.sscore, 2 * n)) ||
        (rc = alloc(h, &cs.sstatus, n)) || (rc = alloc(h, &cs.pick, n)) ||
        (rc = alloc(h, &cs.xlist, (size_t)kXCap)) || (rc = alloc(h, &cs.xcount, 1)))
      return rc;
  }
  return MZ_OK;
}

// The order-exact selection of the first min(*count, n) listed groups (count null: n):
// k_mcclendon's scores (already in cs.score / cs.status for candidates j * C + c), the declined
// candidates scored on the host, the first minimum into dst (k_cand_select).
int exact_select(mz_handle* h, MzCandStore& cs, const MzDev& dst, const int32_t* ids, int base,
                 const int* count, int n, int C, const int32_t* xlist, int count_groups,
                 hipStream_t s) {
  MzHostFallback& hf = cs.hf;
  MZ_HIP(hipMemsetAsync(hf.count_d, 0, sizeof(int), s));
  MZ_HIP(mz_launch_cand_gather(cs.v, count, n, C, cs.status, hf.map, hf.grid_d, hf.info_d,
                               hf.count_d, hf.cap, hf.gstride, s, h->dbg));
  MZ_HIP(hipMemcpyAsync(hf.count_h, hf.count_d, sizeof(int), hipMemcpyDeviceToHost, s));
  MZ_HIP(hipLaunchHostFunc(s, host_fallback_fn, &hf));
  MZ_HIP(mz_launch_cand_select(cs.v, dst, ids, base, count, n, C, cs.score, cs.status,
                               h->sel_stats, s, xlist, hf.map, hf.prod_d, hf.ok_d, hf.cap,
                               count_groups, h->dbg));
  return MZ_OK;
}

// Best-of-C over the first min(*count, n) targets (count null: n): target j's C Philox
// candidates (mz_cand_seed of id(j) = ids ? ids[j] : base + j), the first minimum of McClendon
// difficulty into dst instance id(j) (BaseMazeEnv.generate_maze, base_maze_env.py:78-97).
// Euclidean: compact candidates, the order-free screen, a pick where the screen's bounds decide
// and tables for it (k_cand_expand); the groups it cannot decide (none in practice) through the
// order-exact kernel on rebuilt candidates. Toroidal: the order-exact kernel on every candidate.
int bestof_run(mz_handle* h, MzCandStore& cs, const MzDev& dst, const int32_t* ids, int base,
               const int* count, int n, int C, const uint8_t* algo_list, int algo_all, int dim,
               uint64_t seed, uint32_t epoch, hipStream_t s) {
  const MzDev& cv = cs.v;
  const int dbg = h->dbg;
  if (cs.cc.Qp > 0) {
    MZ_HIP(mz_launch_cand_compact(cs.cc, h->d.P, ids, base, count, n, C, algo_list, algo_all, dim,
                                  seed, epoch, s, dbg));
    MZ_HIP(mz_launch_screen(cs.cc, h->d.P, n * C, cs.sscore, cs.sstatus, s, count, C));
    MZ_HIP(hipMemsetAsync(cs.xcount, 0, sizeof(int), s));
    MZ_HIP(mz_launch_cand_pick(count, n, C, cs.sscore, cs.sstatus, cs.pick, cs.xlist, cs.xcount,
                               kXCap, h->sel_stats, s, dbg));
    MZ_HIP(mz_launch_cand_expand(cs.cc, dst, ids, base, count, n, C, cs.pick, algo_list, algo_all, s));
    const int xc = std::min(kXCap, std::min(n, cs.cap / C));
    MZ_HIP(mz_launch_cand_rebuild(cv, cs.xlist, cs.xcount, xc, ids, base, C, algo_list, algo_all,
                                  dim, seed, epoch, s, dbg));
    MZ_HIP(mz_launch_mcclendon(cv, nullptr, xc * C, cs.score, cs.status, s, cs.xcount, C));
    return exact_select(h, cs, dst, ids, base, cs.xcount, xc, C, cs.xlist, 0, s);
  }
  MZ_HIP(mz_launch_cand_build(cv, ids, base, count, n, C, algo_list, algo_all, dim, seed, epoch, s, dbg));
  MZ_HIP(mz_launch_mcclendon(cv, nullptr, n * C, cs.score, cs.status, s, count, C));
  return exact_select(h, cs, dst, ids, base, count, n, C, nullptr, 1, s);
}

}  // namespace

extern "C" {

const char* mz_last_error(void) { return g_err.c_str(); }

int mz_device_count(int* n) {
  if (!n) return fail(MZ_EINVAL, "null");
  MZ_HIP(hipGetDeviceCount(n));
  return MZ_OK;
}

int mz_create(const mz_config* cfg, mz_handle** out) {
  if (!cfg || !out) return fail(MZ_EINVAL, "null argument");
  if (cfg->num_envs < 1) return fail(MZ_EINVAL, "num_envs must be >= 1");
  if (cfg->max_dim < 5 || cfg->max_dim > MZ_MAX_DIM)
    return fail(MZ_EINVAL_SHAPE, "max_dim %d outside [5, %d]", cfg->max_dim, MZ_MAX_DIM);
  int ndev = 0;
  MZ_HIP(hipGetDeviceCount(&ndev));
  if (cfg->device < 0 || cfg->device >= ndev)
    return fail(MZ_EINVAL, "device %d not present (%d HIP devices)", cfg->device, ndev);
  DeviceGuard g(cfg->device);
  mz_handle* h = new mz_handle();
  h->cfg = *cfg;
  MzDev& d = h->d;
  d.B = cfg->num_envs;
  d.P = cfg->max_dim;
  d.toroidal = cfg->toroidal != 0;
  d.enrich = cfg->enrich != 0;
  d.NS = mz_nstrips(d.P);
  d.PW = 2 * d.NS * d.P;
  const size_t B = (size_t)d.B, P = (size_t)d.P;
  int rc;
  if ((rc = alloc(h, &d.cells, B * P * P)) || (rc = alloc(h, &d.planes, B * (size_t)d.PW + 16)) ||
      (rc = alloc(h, &d.meta0, B)) ||
      (rc = alloc(h, &d.meta1, B)) || (rc = alloc(h, &d.posw, B)) || (rc = alloc(h, &d.stw, B)) ||
      (rc = alloc(h, &d.curw, B)) || (rc = alloc(h, &d.algo, B)) || (rc = alloc(h, &d.last_term, B)) ||
      (rc = alloc(h, &d.ticket, 16)) || (rc = alloc(h, &h->sel_stats, 8))) {
    mz_destroy(h);
    return rc;
  }
  // exact penalty tables, built with the same libm exp as CPython's math.exp
  double pen[512];
  for (int k = 0; k < 256; ++k) {
    volatile double ev = std::exp(-0.2 * (double)k);
    volatile double ei = std::exp(-0.15 * (double)k);
    pen[k] = 0.0 - (1.0 - ev);
    pen[256 + k] = 0.0 - (1.0 - ei);
  }
  double* dpen = nullptr;
  if ((rc = alloc(h, &dpen, 512))) { mz_destroy(h); return rc; }
  hipError_t e = hipMemcpy(dpen, pen, sizeof pen, hipMemcpyHostToDevice);
  if (e != hipSuccess) { mz_destroy(h); return fail(MZ_EHIP, "%s", hipGetErrorString(e)); }
  d.pen_visit = dpen;
  d.pen_inv = dpen + 256;
  *out = h;
  return MZ_OK;
}

int mz_destroy(mz_handle* h) {
  if (!h) return MZ_OK;
  DeviceGuard g(h->cfg.device);
  (void)hipDeviceSynchronize();
  for (void* p : h->allocs) (void)hipFree(p);
  for (void* p : h->host_allocs) (void)hipHostFree(p);
  if (h->staging) (void)hipFree(h->staging);
  delete h;
  return MZ_OK;
}

int mz_load_mazes(mz_handle* h, const uint8_t* grids_host, int32_t dim,
                  const int32_t* sg_host, const int32_t* env_ids_host, int32_t n, void* stream) {
  if (!h || !grids_host || !sg_host || n < 1) return fail(MZ_EINVAL, "bad arguments");
  int rc = check_dim(h, dim);
  if (rc) return rc;
  const size_t cells = (size_t)dim * dim;
  for (int i = 0; i < n; ++i) {
    const int32_t* s = sg_host + 4 * i;
    for (int k = 0; k < 4; ++k)
      if (s[k] < 0 || s[k] >= dim) return fail(MZ_EINVAL, "maze %d: start/goal out of range", i);
    const uint8_t* g = grids_host + i * cells;
    for (size_t c = 0; c < cells; ++c)
      if (g[c] > 2) return fail(MZ_EINVAL, "maze %d: grid value %d not in {0,1,2}", i, g[c]);
    if (g[s[0] * dim + s[1]] == 0 || g[s[2] * dim + s[3]] != 2)
      return fail(MZ_EINVAL, "maze %d: start must be open and goal must hold 2", i);
    if (env_ids_host && (env_ids_host[i] < 0 || env_ids_host[i] >= h->d.B))
      return fail(MZ_EINVAL, "env id %d out of range", env_ids_host[i]);
  }
  if (!env_ids_host && n > h->d.B) return fail(MZ_EINVAL, "n > num_envs");
  DeviceGuard g(h->cfg.device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const size_t need = n * cells + 16 * (size_t)n + 4 * (size_t)n + 256;
  if (need > h->staging_bytes) {
    if (h->staging) MZ_HIP(hipFree(h->staging));
    h->staging = nullptr;
    MZ_HIP(hipMalloc(&h->staging, need));
    h->staging_bytes = need;
  }
  uint8_t* dg = h->staging;
  int32_t* dsg = reinterpret_cast<int32_t*>(h->staging + ((n * cells + 15) & ~(size_t)15));
  int32_t* dids = dsg + 4 * n;
  MZ_HIP(hipMemcpyAsync(dg, grids_host, n * cells, hipMemcpyHostToDevice, s));
  MZ_HIP(hipMemcpyAsync(dsg, sg_host, 16 * (size_t)n, hipMemcpyHostToDevice, s));
  if (env_ids_host) MZ_HIP(hipMemcpyAsync(dids, env_ids_host, 4 * (size_t)n, hipMemcpyHostToDevice, s));
  MZ_HIP(mz_launch_build(h->d, env_ids_host ? dids : nullptr, n, false, nullptr, 0, dim, 0, dg, dsg,
                         0, nullptr, s));
  MZ_HIP(hipStreamSynchronize(s));
  return MZ_OK;
}

int mz_generate_ex(mz_handle* h, const int32_t* env_ids_dev, int32_t n, const uint8_t* algo_dev,
                   int32_t algo_all, int32_t dim, uint64_t seed, int32_t rng, void* stream) {
  if (!h) return fail(MZ_EINVAL, "null handle");
  if (!env_ids_dev) n = h->d.B;
  if (n < 0 || n > h->d.B) return fail(MZ_EINVAL, "n out of range");
  if (!algo_dev && (algo_all < 0 || algo_all > 2)) return fail(MZ_EINVAL, "algorithm id %d", algo_all);
  if (rng != MZ_RNG_PHILOX && rng != MZ_RNG_CPYTHON) return fail(MZ_EINVAL, "rng %d", rng);
  int rc = check_dim(h, dim);
  if (rc) return rc;
  DeviceGuard g(h->cfg.device);
  MZ_HIP(mz_launch_build(h->d, env_ids_dev, n, true, algo_dev, algo_all, dim, seed, nullptr,
                         nullptr, rng == MZ_RNG_CPYTHON ? 1 : 0, nullptr,
                         static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_generate(mz_handle* h, const int32_t* env_ids_dev, int32_t n, const uint8_t* algo_dev,
                int32_t algo_all, int32_t dim, uint64_t seed, void* stream) {
  return mz_generate_ex(h, env_ids_dev, n, algo_dev, algo_all, dim, seed, MZ_RNG_PHILOX, stream);
}

int mz_generate_state(mz_handle* h, int32_t env, int32_t dim, int32_t algo, uint32_t* state_host,
                      void* stream) {
  if (!h || !state_host || env < 0 || env >= h->d.B) return fail(MZ_EINVAL, "bad arguments");
  if (algo < 0 || algo > 2) return fail(MZ_EINVAL, "algorithm id %d", algo);
  if (state_host[624] > 624u) return fail(MZ_EINVAL, "random state index %u", state_host[624]);
  int rc = check_dim(h, dim);
  if (rc) return rc;
  DeviceGuard g(h->cfg.device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const size_t need = 625 * sizeof(uint32_t) + 16;
  if (need > h->staging_bytes) {
    if (h->staging) MZ_HIP(hipFree(h->staging));
    h->staging = nullptr;
    MZ_HIP(hipMalloc(&h->staging, need));
    h->staging_bytes = need;
  }
  uint32_t* dst = reinterpret_cast<uint32_t*>(h->staging);
  int32_t* ids = reinterpret_cast<int32_t*>(h->staging + 625 * sizeof(uint32_t) + 4);
  int err = 0;
  MZ_HIP(hipMemcpyAsync(dst, state_host, 625 * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  MZ_HIP(hipMemcpyAsync(ids, &env, sizeof(int32_t), hipMemcpyHostToDevice, s));
  MZ_HIP(hipMemsetAsync(h->d.ticket + MZ_TICKET_PYERR, 0, sizeof(int), s));
  MZ_HIP(mz_launch_build(h->d, ids, 1, true, nullptr, algo, dim, 0, nullptr, nullptr, 2, dst, s));
  MZ_HIP(hipMemcpyAsync(state_host, dst, 625 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  MZ_HIP(hipMemcpyAsync(&err, h->d.ticket + MZ_TICKET_PYERR, sizeof(int), hipMemcpyDeviceToHost, s));
  MZ_HIP(hipStreamSynchronize(s));
  if (err) return fail(MZ_EHIP, "CPython set emulation overflowed its table (flag %d)", err);
  return MZ_OK;
}

int mz_reset_all(mz_handle* h, const mz_step_out* out, void* stream) {
  if (!h) return fail(MZ_EINVAL, "null handle");
  int rc = check_out(out);
  if (rc) return rc;
  DeviceGuard g(h->cfg.device);
  MZ_HIP(mz_launch_reset_list(h->d, nullptr, nullptr, h->d.B, to_dev(out),
                              static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_reset_list(mz_handle* h, const int32_t* idx_dev, const int32_t* count_dev,
                  int32_t max_count, int32_t regen_won, uint64_t seed, uint32_t epoch,
                  const mz_step_out* out, void* stream) {
  if (!h || !idx_dev) return fail(MZ_EINVAL, "bad arguments");
  if (max_count < 0 || max_count > h->d.B) max_count = h->d.B;
  int rc = check_out(out);
  if (rc) return rc;
  DeviceGuard g(h->cfg.device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (regen_won) MZ_HIP(mz_launch_regen(h->d, idx_dev, count_dev, max_count, seed, epoch, s));
  MZ_HIP(mz_launch_reset_list(h->d, idx_dev, const_cast<int32_t*>(count_dev), max_count, to_dev(out), s));
  return MZ_OK;
}

int mz_reset_done(mz_handle* h, int32_t regen_won, uint64_t seed, uint32_t epoch,
                  const mz_step_out* out, void* stream) {
  if (!h) return fail(MZ_EINVAL, "null handle");
  int rc = check_out(out);
  if (rc) return rc;
  DeviceGuard g(h->cfg.device);
  MZ_HIP(mz_launch_reset_done(h->d, regen_won ? 1 : 0, seed, epoch, to_dev(out),
                              static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_step_ex(mz_handle* h, const int32_t* actions_dev, const mz_step_out* out, int32_t flags,
               void* stream) {
  if (!h || !actions_dev) return fail(MZ_EINVAL, "bad arguments");
  if (flags & ~(MZ_STEP_COUNT_ZEROED | MZ_STEP_AUTORESET)) return fail(MZ_EINVAL, "flags %d", flags);
  int rc = check_out(out);
  if (rc) return rc;
  DeviceGuard g(h->cfg.device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (out && out->done_count && !(flags & MZ_STEP_COUNT_ZEROED))
    MZ_HIP(hipMemsetAsync(out->done_count, 0, sizeof(int32_t), s));
  MZ_HIP(mz_launch_step(h->d, actions_dev, nullptr, (flags & MZ_STEP_AUTORESET) != 0, to_dev(out), s));
  return MZ_OK;
}

int mz_step(mz_handle* h, const int32_t* actions_dev, const mz_step_out* out, void* stream) {
  return mz_step_ex(h, actions_dev, out, 0, stream);
}

int mz_step_act(mz_handle* h, const float* eps_dev, float eps_all, const int64_t* greedy_dev,
                uint64_t seed, uint64_t counter, int32_t* actions_out_dev, const mz_step_out* out,
                int32_t flags, void* stream) {
  if (!h) return fail(MZ_EINVAL, "null handle");
  if (flags & ~(MZ_STEP_COUNT_ZEROED | MZ_STEP_AUTORESET)) return fail(MZ_EINVAL, "flags %d", flags);
  int rc = check_out(out);
  if (rc) return rc;
  DeviceGuard g(h->cfg.device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (out && out->done_count && !(flags & MZ_STEP_COUNT_ZEROED))
    MZ_HIP(hipMemsetAsync(out->done_count, 0, sizeof(int32_t), s));
  MzAct ap{eps_dev, eps_all, greedy_dev, seed, counter, actions_out_dev};
  MZ_HIP(mz_launch_step(h->d, nullptr, &ap, (flags & MZ_STEP_AUTORESET) != 0, to_dev(out), s));
  return MZ_OK;
}

int mz_direction_mask(mz_handle* h, int32_t probs, float* out4_dev, void* stream) {
  if (!h || !out4_dev) return fail(MZ_EINVAL, "bad arguments");
  if (reinterpret_cast<uintptr_t>(out4_dev) & 15u) return fail(MZ_EALIGN, "out4 must be 16-B aligned");
  DeviceGuard g(h->cfg.device);
  MZ_HIP(mz_launch_mask(h->d, probs, out4_dev, static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_act(mz_handle* h, const float* eps_dev, float eps_all, const int64_t* greedy_dev,
           uint64_t seed, uint64_t counter, int32_t* actions_dev, void* stream) {
  if (!h || !actions_dev) return fail(MZ_EINVAL, "bad arguments");
  DeviceGuard g(h->cfg.device);
  MzAct ap{eps_dev, eps_all, greedy_dev, seed, counter, actions_dev};
  MZ_HIP(mz_launch_act(h->d, ap, static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_expand_window(const uint32_t* bits_dev, float* out_dev, int32_t n, void* stream) {
  if (!bits_dev || !out_dev || n < 0) return fail(MZ_EINVAL, "bad arguments");
  MZ_HIP(mz_launch_expand(bits_dev, out_dev, n, static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_q_front(const uint32_t* bits_dev, const float* obs6_dev, int32_t n, const float* conv_w_dev,
               const float* conv_b_dev, float drop_p, uint64_t seed, uint64_t counter,
               uint16_t* feat_dev, int32_t ld, void* stream) {
  if (!bits_dev || !obs6_dev || !conv_w_dev || !conv_b_dev || !feat_dev || n < 0)
    return fail(MZ_EINVAL, "bad arguments");
  if (ld < 1576 || ld > 1600 || ld % 8 != 0) return fail(MZ_EINVAL, "feature stride %d", ld);
  if (!(drop_p >= 0.0f && drop_p < 1.0f)) return fail(MZ_EINVAL, "dropout p %g", (double)drop_p);
  MZ_HIP(mz_launch_qfront(bits_dev, obs6_dev, nullptr, nullptr, n, conv_w_dev, conv_b_dev, drop_p,
                          seed, counter, feat_dev, ld, static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_q_front_rows(const uint32_t* bits_dev, const float* obs6_dev, const int32_t* rows_dev,
                    const int32_t* count_dev, int32_t n, const float* conv_w_dev,
                    const float* conv_b_dev, float drop_p, uint64_t seed, uint64_t counter,
                    uint16_t* feat_dev, int32_t ld, void* stream) {
  if (!bits_dev || !obs6_dev || !rows_dev || !conv_w_dev || !conv_b_dev || !feat_dev || n < 0)
    return fail(MZ_EINVAL, "bad arguments");
  if (ld < 1576 || ld > 1600 || ld % 8 != 0) return fail(MZ_EINVAL, "feature stride %d", ld);
  if (!(drop_p >= 0.0f && drop_p < 1.0f)) return fail(MZ_EINVAL, "dropout p %g", (double)drop_p);
  MZ_HIP(mz_launch_qfront(bits_dev, obs6_dev, rows_dev, count_dev, n, conv_w_dev, conv_b_dev,
                          drop_p, seed, counter, feat_dev, ld, static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_greedy_rows(const float* eps_dev, float eps_all, uint64_t seed, uint64_t counter, int32_t n,
                   int32_t* scratch_dev, int32_t* rows_dev, int32_t* count_dev,
                   int32_t* count_host, void* stream) {
  if (n < 0 || (n > 0 && (!scratch_dev || !rows_dev || !count_dev)))
    return fail(MZ_EINVAL, "bad arguments");
  MzAct ap{eps_dev, eps_all, nullptr, seed, counter, nullptr};
  MZ_HIP(mz_launch_greedy_rows(ap, n, scratch_dev, rows_dev, count_dev, count_host,
                               static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_stem_forward(const uint32_t* bits_dev, const float* obs6_dev, int32_t n,
                    const float* conv_w_dev, const float* conv_b_dev, float drop_p,
                    const uint64_t* rng_dev, uint32_t salt, float* feat_dev, int32_t ld,
                    uint8_t* code_dev, void* stream) {
  if (!bits_dev || !obs6_dev || !conv_w_dev || !conv_b_dev || !feat_dev || n < 0)
    return fail(MZ_EINVAL, "bad arguments");
  if (ld < 1574) return fail(MZ_EINVAL, "feature stride %d", ld);
  if (!(drop_p >= 0.0f && drop_p < 1.0f)) return fail(MZ_EINVAL, "dropout p %g", (double)drop_p);
  if (drop_p > 0.0f && !rng_dev) return fail(MZ_EINVAL, "dropout needs the device rng counter");
  MZ_HIP(mz_launch_stem_fwd(bits_dev, obs6_dev, n, conv_w_dev, conv_b_dev, drop_p, rng_dev, salt,
                            feat_dev, ld, code_dev, static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_stem_backward_ex(const uint32_t* bits_dev, const uint8_t* code_dev, const float* gfeat_dev,
                        int32_t ld, int32_t n, float drop_p, float* partial_dev, float* dw_dev,
                        float* db_dev, uint64_t* rng_advance_dev, void* stream) {
  if (!bits_dev || !code_dev || !gfeat_dev || !partial_dev || !dw_dev || !db_dev || n < 0)
    return fail(MZ_EINVAL, "bad arguments");
  if (ld < 1568) return fail(MZ_EINVAL, "gradient stride %d", ld);
  if (!(drop_p >= 0.0f && drop_p < 1.0f)) return fail(MZ_EINVAL, "dropout p %g", (double)drop_p);
  MZ_HIP(mz_launch_stem_bwd(bits_dev, code_dev, gfeat_dev, ld, n, drop_p, partial_dev, dw_dev,
                            db_dev, static_cast<hipStream_t>(stream), rng_advance_dev));
  return MZ_OK;
}

int mz_stem_backward(const uint32_t* bits_dev, const uint8_t* code_dev, const float* gfeat_dev,
                     int32_t ld, int32_t n, float drop_p, float* partial_dev, float* dw_dev,
                     float* db_dev, void* stream) {
  return mz_stem_backward_ex(bits_dev, code_dev, gfeat_dev, ld, n, drop_p, partial_dev, dw_dev,
                             db_dev, nullptr, stream);
}

int mz_adamw_flat(float* param_dev, float* exp_avg_dev, float* exp_avg_sq_dev,
                  const float* const* grads_dev, const int64_t* seg_len, int32_t nseg,
                  const float* lr_dev, float* step_dev, double beta1, double beta2, double eps,
                  double weight_decay, float clamp, float grad_scale, int32_t write_grad,
                  void* stream) {
  if (!param_dev || !exp_avg_dev || !exp_avg_sq_dev || !grads_dev || !seg_len || !lr_dev ||
      !step_dev)
    return fail(MZ_EINVAL, "bad arguments");
  if (nseg < 1 || nseg > MZ_OPT_MAX_SEGS) return fail(MZ_EINVAL, "segment count %d", nseg);
  const uintptr_t al = reinterpret_cast<uintptr_t>(param_dev) | reinterpret_cast<uintptr_t>(exp_avg_dev) |
                       reinterpret_cast<uintptr_t>(exp_avg_sq_dev);
  if (al & 15) return fail(MZ_EALIGN, "flat buffers must be 16-byte aligned");
  for (int k = 0; k < nseg; ++k) {
    if (!grads_dev[k] || seg_len[k] <= 0 || (seg_len[k] & 3))
      return fail(MZ_EINVAL, "segment %d: length %lld (multiple of 4 required)", k,
                  (long long)seg_len[k]);
    if (reinterpret_cast<uintptr_t>(grads_dev[k]) & 15)
      return fail(MZ_EALIGN, "gradient %d must be 16-byte aligned", k);
  }
  if (!(clamp > 0.0f)) return fail(MZ_EINVAL, "clamp %g", (double)clamp);
  MZ_HIP(mz_launch_adamw(param_dev, exp_avg_dev, exp_avg_sq_dev, grads_dev, seg_len, nseg, lr_dev,
                         step_dev, beta1, beta2, eps, weight_decay, clamp, grad_scale, write_grad,
                         static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_leaky_relu_bf16(uint16_t* x_dev, int64_t n, float slope, void* stream) {
  if (!x_dev || n < 0) return fail(MZ_EINVAL, "bad arguments");
  if ((n & 7) || (reinterpret_cast<uintptr_t>(x_dev) & 15))
    return fail(MZ_EALIGN, "leaky_relu_bf16 needs a 16-byte aligned multiple of 8 elements");
  MZ_HIP(mz_launch_leaky_bf16(x_dev, n, slope, static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_colsum_f32(const float* g_dev, int32_t n, int32_t m, int32_t ld, float* out_dev,
                  void* stream) {
  if (!g_dev || !out_dev || n < 0 || m < 0 || ld < m) return fail(MZ_EINVAL, "bad arguments");
  if ((m & 3) || (ld & 3) || (reinterpret_cast<uintptr_t>(g_dev) & 15) ||
      (reinterpret_cast<uintptr_t>(out_dev) & 15))
    return fail(MZ_EALIGN, "colsum_f32 needs m, ld multiples of 4 and 16-byte aligned buffers");
  MZ_HIP(mz_launch_colsum(g_dev, n, m, ld, out_dev, static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_replay_gather(const int64_t* idx_dev, int32_t b, int64_t capacity,
                     const float* s6_dev, const int32_t* sw_dev, const int64_t* a_dev,
                     const float* r_dev, const float* s6n_dev, const int32_t* swn_dev,
                     float* out_s6_dev,
                     int32_t* out_sw_dev, int64_t* out_a_dev, float* out_r_dev, void* stream) {
  if (b < 0 || (b > 0 && (!idx_dev || !s6_dev || !sw_dev || !a_dev || !r_dev || !s6n_dev ||
                          !swn_dev || !out_s6_dev || !out_sw_dev || !out_a_dev || !out_r_dev)))
    return fail(MZ_EINVAL, "bad arguments");
  if (b > 0 && capacity < 1) return fail(MZ_EINVAL, "replay capacity %lld", (long long)capacity);
  MZ_HIP(mz_launch_replay_gather(idx_dev, b, capacity, s6_dev, reinterpret_cast<const uint32_t*>(sw_dev),
                                 a_dev, r_dev, s6n_dev, reinterpret_cast<const uint32_t*>(swn_dev),
                                 out_s6_dev, reinterpret_cast<uint32_t*>(out_sw_dev), out_a_dev,
                                 out_r_dev, static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_pair_surrogate(const float* lp_new_dev, const float* lp_old_dev, const float* adv_dev,
                      int32_t b, float clip, float* part_dev, float* dsum_dev, void* stream) {
  if (!lp_new_dev || !lp_old_dev || !adv_dev || !part_dev || !dsum_dev || b < 0)
    return fail(MZ_EINVAL, "bad arguments");
  if (!(clip >= 0.0f && clip < 1.0f)) return fail(MZ_EINVAL, "clip %g", (double)clip);
  MZ_HIP(mz_launch_pair_surrogate(lp_new_dev, lp_old_dev, adv_dev, b, clip, part_dev, dsum_dev,
                                  static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_stem_workspace_floats(int32_t n) { return n > 0 ? mz_stem_chunks(n) * 32 * 28 : 0; }

int mz_bank_create_ex(mz_handle* h, int32_t slots, const int32_t* dims, int32_t ndims,
                      uint32_t algo_mask, int32_t candidates) {
  if (!h) return fail(MZ_EINVAL, "null handle");
  if (h->bank.K) return fail(MZ_EINVAL, "the handle already has a maze bank");
  if (slots < 1) return fail(MZ_EINVAL, "bank slots %d", slots);
  if (candidates < 1 || candidates > MZ_MAX_CANDIDATES)
    return fail(MZ_EINVAL, "candidates %d outside [1, %d]", candidates, MZ_MAX_CANDIDATES);
  if (candidates > 1) {
    int mm = 0;
    if (mz_mcclendon_lds(h->d.P, h->d.toroidal != 0, &mm) > 160 * 1024)
      return fail(MZ_EINVAL_SHAPE, "best-of-%d banks score with the difficulty kernel: maze pitch "
                  "%d beyond its LDS plan", candidates, h->d.P);
    if ((int64_t)slots * candidates > (1 << 24)) return fail(MZ_EINVAL, "slots x candidates too large");
  }
  if (algo_mask == 0 || algo_mask > 7u) return fail(MZ_EINVAL, "algorithm mask %u", algo_mask);
  if (!dims || ndims < 1 || ndims > MZ_BANK_MAX_DIMS) return fail(MZ_EINVAL, "bank sizes %d", ndims);
  for (int i = 0; i < ndims; ++i) {
    int rc = check_dim(h, dims[i]);
    if (rc) return rc;
    for (int j = 0; j < i; ++j)
      if (dims[j] == dims[i]) return fail(MZ_EINVAL, "bank size %d listed twice", dims[i]);
  }
  DeviceGuard g(h->cfg.device);
  MzBankStore& b = h->bank;
  const MzDev& d = h->d;
  const int nA = __builtin_popcount(algo_mask);
  const size_t S = 2 * (size_t)nA * ndims * slots, K = (size_t)slots;
  int rc;
  if ((rc = alloc(h, &b.cells, S * d.P * d.P)) || (rc = alloc(h, &b.planes, S * d.PW)) ||
      (rc = alloc(h, &b.meta0, S)) || (rc = alloc(h, &b.meta1, S)) ||
      (rc = alloc(h, &b.heads, (size_t)6 * ndims)) ||
      (rc = alloc(h, &b.slot, (size_t)3 * ndims * ((d.B + 63) / 64))) ||
      (rc = alloc(h, &b.code, (size_t)d.B)) || (rc = alloc(h, &b.s_posw, K)) ||
      (rc = alloc(h, &b.s_stw, K)) || (rc = alloc(h, &b.s_curw, K)) || (rc = alloc(h, &b.s_last, K)) ||
      (rc = alloc(h, &b.s_algo, K)))
    return rc;
  // first fill builds every slot of the algorithms the bank holds
  std::vector<int> full((size_t)6 * ndims);
  for (int i = 0; i < 6 * ndims; ++i) full[i] = ((algo_mask >> ((i / ndims) % 3)) & 1u) ? slots : 0;
  MZ_HIP(hipMemcpy(b.heads, full.data(), full.size() * sizeof(int), hipMemcpyHostToDevice));
  b.K = slots;
  b.nD = ndims;
  for (int i = 0; i < ndims; ++i) b.dims[i] = dims[i];
  b.nA = nA;
  b.amask = algo_mask;
  b.C = candidates;
  if (candidates > 1 && (rc = cand_alloc(h, b.cand, slots * candidates))) {
    b.K = 0;  // no bank: a later create may retry
    return rc;
  }
  return MZ_OK;
}

int mz_bank_create_dims(mz_handle* h, int32_t slots, const int32_t* dims, int32_t ndims,
                        uint32_t algo_mask) {
  return mz_bank_create_ex(h, slots, dims, ndims, algo_mask, 1);
}

int mz_bank_create(mz_handle* h, int32_t slots, int32_t dim, uint32_t algo_mask) {
  return mz_bank_create_ex(h, slots, &dim, 1, algo_mask, 1);
}

int mz_bank_fill(mz_handle* h, int32_t bank, uint64_t seed, void* stream) {
  if (!h || !h->bank.K) return fail(MZ_EINVAL, "no maze bank (mz_bank_create)");
  if (bank != 0 && bank != 1) return fail(MZ_EINVAL, "bank %d", bank);
  DeviceGuard g(h->cfg.device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  MzBankStore& b = h->bank;
  const size_t K = (size_t)b.K, P = (size_t)h->d.P;
  for (int a = 0; a < 3; ++a) {
    if (!((b.amask >> a) & 1u)) continue;
    for (int di = 0; di < b.nD; ++di) {
      const size_t blk = (((size_t)bank * b.nA + mz_bank_aidx(b.amask, a)) * b.nD + di) * K;
    MzDev bd = h->d;  // same pitch / flags; instance arrays = this block's slots + scratch
    bd.B = b.K;
    bd.cells = b.cells + blk * P * P;
    bd.planes = b.planes + blk * h->d.PW;
    bd.meta0 = b.meta0 + blk;
    bd.meta1 = b.meta1 + blk;
    bd.posw = b.s_posw;
    bd.stw = b.s_stw;
    bd.curw = b.s_curw;
    bd.last_term = b.s_last;
    bd.algo = b.s_algo;
    bd.bk_K = 0;
    int* head = b.heads + (3 * bank + a) * b.nD + di;
    // (size index di = 0 keeps the single-size bank's keys)
    const uint64_t key = seed ^ ((uint64_t)(3 * bank + a + 1) << 56) ^ ((uint64_t)di << 48);
    if (b.C > 1) {  // best-of-C: candidates, their difficulty, the first minimum into the slot
      int rc = bestof_run(h, b.cand, bd, nullptr, 0, head, b.K, b.C, nullptr, a, b.dims[di], key,
                          b.epoch[bank], s);
      if (rc) return rc;
    } else {
      MZ_HIP(mz_launch_cand_build(bd, nullptr, 0, head, b.K, 1, nullptr, a, b.dims[di], key,
                                  b.epoch[bank], s));
    }
    MZ_HIP(hipMemsetAsync(head, 0, sizeof(int), s));
    }
  }
  b.epoch[bank] += 1;
  return MZ_OK;
}

int mz_bank_use(mz_handle* h, int32_t bank) {
  if (!h) return fail(MZ_EINVAL, "null handle");
  MzDev& d = h->d;
  if (bank < 0) {
    d.bk_K = 0;
    return MZ_OK;
  }
  const MzBankStore& b = h->bank;
  if (!b.K) return fail(MZ_EINVAL, "no maze bank (mz_bank_create)");
  if (bank > 1) return fail(MZ_EINVAL, "bank %d", bank);
  const size_t blk = (size_t)bank * b.nA * b.nD * b.K, P = (size_t)d.P;
  d.bk_K = b.K;
  d.bk_nd = b.nD;
  for (int i = 0; i < 128; ++i) d.bk_didx[i] = -1;
  for (int i = 0; i < b.nD; ++i) d.bk_didx[b.dims[i]] = (int8_t)i;
  d.bk_amask = b.amask;
  d.bk_cells = b.cells + blk * P * P;
  d.bk_planes = b.planes + blk * d.PW;
  d.bk_meta0 = b.meta0 + blk;
  d.bk_meta1 = b.meta1 + blk;
  d.bk_head = b.heads + 3 * bank * b.nD;
  d.bk_slot = b.slot;
  d.bk_code = b.code;
  d.bk_G = (d.B + 63) / 64;
  return MZ_OK;
}

int mz_bank_slot_grid(mz_handle* h, int32_t bank, int32_t algo, int32_t size_index, int32_t slot,
                      uint8_t* grid_host, int32_t* info4_host) {
  if (!h || !h->bank.K || !grid_host || !info4_host) return fail(MZ_EINVAL, "bad arguments");
  const MzBankStore& b = h->bank;
  if (bank < 0 || bank > 1 || algo < 0 || algo > 2 || !((b.amask >> algo) & 1u) ||
      size_index < 0 || size_index >= b.nD || slot < 0 || slot >= b.K)
    return fail(MZ_EINVAL, "no such bank slot");
  DeviceGuard g(h->cfg.device);
  MZ_HIP(hipDeviceSynchronize());
  const size_t P = (size_t)h->d.P;
  const size_t i = (((size_t)bank * b.nA + mz_bank_aidx(b.amask, algo)) * b.nD + size_index) * b.K + slot;
  uint32_t m0, m1;
  MZ_HIP(hipMemcpy(&m0, b.meta0 + i, 4, hipMemcpyDeviceToHost));
  MZ_HIP(hipMemcpy(&m1, b.meta1 + i, 4, hipMemcpyDeviceToHost));
  std::vector<uint32_t> cw(P * P);
  MZ_HIP(hipMemcpy(cw.data(), b.cells + i * P * P, 4 * cw.size(), hipMemcpyDeviceToHost));
  const int N = m0 & 0xFF, gr = m1 & 0xFF, gc = (m1 >> 8) & 0xFF;
  if (N < 5 || N > (int)P) return fail(MZ_EINVAL, "bank slot not built");
  for (int r = 0; r < N; ++r)
    for (int c = 0; c < N; ++c) {
      const bool open = (cw[(size_t)r * P + c] & MZ_CELL_OPEN) != 0;
      grid_host[r * N + c] = !open ? 0 : ((r == gr && c == gc) ? 2 : 1);
    }
  info4_host[0] = (m0 >> 16) & 0xFF;
  info4_host[1] = m0 >> 24;
  info4_host[2] = gr;
  info4_host[3] = gc;
  return MZ_OK;
}

int mz_set_regen_dims(mz_handle* h, const uint8_t* dims_dev) {
  if (!h) return fail(MZ_EINVAL, "null handle");
  h->d.regen_dim = dims_dev;
  return MZ_OK;
}

int mz_generate_best(mz_handle* h, const int32_t* env_ids_dev, int32_t n, const uint8_t* algo_dev,
                     int32_t algo_all, int32_t dim, uint64_t seed, int32_t candidates,
                     void* stream) {
  if (!h) return fail(MZ_EINVAL, "null handle");
  if (candidates < 1 || candidates > MZ_MAX_CANDIDATES)
    return fail(MZ_EINVAL, "candidates %d outside [1, %d]", candidates, MZ_MAX_CANDIDATES);
  if (candidates == 1)
    return mz_generate_ex(h, env_ids_dev, n, algo_dev, algo_all, dim, seed, MZ_RNG_PHILOX, stream);
  if (!env_ids_dev) n = h->d.B;
  if (n < 0 || n > h->d.B) return fail(MZ_EINVAL, "n out of range");
  if (!algo_dev && (algo_all < 0 || algo_all > 2)) return fail(MZ_EINVAL, "algorithm id %d", algo_all);
  int rc = check_dim(h, dim);
  if (rc) return rc;
  int mm = 0;
  if (mz_mcclendon_lds(h->d.P, h->d.toroidal != 0, &mm) > 160 * 1024)
    return fail(MZ_EINVAL_SHAPE, "best-of-%d generation scores with the difficulty kernel: maze "
                "pitch %d beyond its LDS plan", candidates, h->d.P);
  if (n == 0) return MZ_OK;
  DeviceGuard g(h->cfg.device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  // chunks of <= 49,152 candidates (1.45 GB of scratch at 81 x 81)
  const int chunk = std::max(1, std::min(n, 49152 / candidates));
  if (h->gen.cap < chunk * candidates) {
    if (h->gen.cap) MZ_HIP(hipStreamSynchronize(s));  // (the old scratch stays owned by the handle)
    if ((rc = cand_alloc(h, h->gen, chunk * candidates))) return rc;
  }
  for (int j0 = 0; j0 < n; j0 += chunk) {
    const int m = std::min(chunk, n - j0);
    const int32_t* ids = env_ids_dev ? env_ids_dev + j0 : nullptr;
    const uint8_t* al = algo_dev ? algo_dev + j0 : nullptr;
    if ((rc = bestof_run(h, h->gen, h->d, ids, j0, nullptr, m, candidates, al, algo_all, dim, seed,
                         0u, s)))
      return rc;
  }
  return MZ_OK;
}

int mz_select_stats(mz_handle* h, int32_t* out3_dev, int32_t reset, void* stream) {
  return mz_select_stats_ex(h, out3_dev, 3, reset, stream);
}

int mz_select_stats_ex(mz_handle* h, int32_t* out_dev, int32_t n, int32_t reset, void* stream) {
  if (!h || n < 0 || n > MZ_SELECT_STATS) return fail(MZ_EINVAL, "bad arguments");
  DeviceGuard g(h->cfg.device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (out_dev && n) MZ_HIP(hipMemcpyAsync(out_dev, h->sel_stats, n * sizeof(int32_t), hipMemcpyDeviceToDevice, s));
  if (reset) MZ_HIP(hipMemsetAsync(h->sel_stats, 0, 8 * sizeof(int32_t), s));
  return MZ_OK;
}

int mz_set_debug(mz_handle* h, int32_t flags) {
  if (!h) return fail(MZ_EINVAL, "null handle");
  if (flags & ~7) return fail(MZ_EINVAL, "debug flags %d", flags);
  h->dbg = flags;
  return MZ_OK;
}

int mz_screen_batch(mz_handle* h, const int32_t* env_ids_dev, int32_t n, double* out_dev,
                    int32_t* status_dev, void* stream) {
  if (!h || !out_dev || !status_dev) return fail(MZ_EINVAL, "bad arguments");
  if (h->d.toroidal) return fail(MZ_EINVAL, "the screen scores euclidean mazes");
  if (!env_ids_dev) n = h->d.B;
  if (n < 0 || (!env_ids_dev && n > h->d.B)) return fail(MZ_EINVAL, "n out of range");
  if (n == 0) return MZ_OK;
  DeviceGuard g(h->cfg.device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (h->scr_cap < n) {
    if (h->scr_cap) MZ_HIP(hipStreamSynchronize(s));  // (the old scratch stays owned by the handle)
    int rc = compact_alloc(h, h->scr, n);
    if (rc) return rc;
    h->scr_cap = n;
  }
  MZ_HIP(mz_launch_compact_from_handle(h->d, env_ids_dev, n, h->scr, s));
  MZ_HIP(mz_launch_screen(h->scr, h->d.P, n, out_dev, status_dev, s));
  return MZ_OK;
}

int mz_bank_consumed(mz_handle* h, int32_t bank, int32_t* out3_dev, void* stream) {
  if (!h || !h->bank.K || !out3_dev || bank < 0 || bank > 1) return fail(MZ_EINVAL, "bad arguments");
  DeviceGuard g(h->cfg.device);
  const int nd = h->bank.nD;
  MZ_HIP(hipMemcpyAsync(out3_dev, h->bank.heads + 3 * bank * nd, 3 * nd * sizeof(int32_t),
                        hipMemcpyDeviceToDevice, static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

}  // extern "C"

namespace {

// ---- checkpoint / resume (mz_state_*): header words and the ordered device sections
constexpr uint32_t kStateMagic = 0x54535A4Du;  // "MZST"
constexpr uint32_t kStateVersion = 1u;
enum : int { SH_MAGIC, SH_VER, SH_B, SH_P, SH_TOR, SH_ENRICH, SH_NS, SH_PW, SH_BK_K, SH_BK_NA,
             SH_BK_ND, SH_BK_AMASK, SH_BK_ACTIVE, SH_BK_EPOCH0, SH_BK_EPOCH1, SH_DIMS = 16 };
static_assert(SH_DIMS * 4 + MZ_BANK_MAX_DIMS <= MZ_STATE_HEADER_BYTES, "header too small");

struct Section {
  void* p;
  size_t bytes;
};

std::vector<Section> state_sections(mz_handle* h) {
  const MzDev& d = h->d;
  const size_t B = (size_t)d.B, P = (size_t)d.P;
  std::vector<Section> s = {
      {d.cells, B * P * P * 4}, {d.planes, (B * (size_t)d.PW + 16) * 4}, {d.meta0, B * 4},
      {d.meta1, B * 4}, {d.posw, B * 4}, {d.stw, B * 4}, {d.curw, B * 4}, {d.algo, B},
      {d.last_term, B}};
  const MzBankStore& b = h->bank;
  if (b.K) {
    const size_t S = 2 * (size_t)b.nA * b.nD * b.K;
    s.push_back({b.cells, S * P * P * 4});
    s.push_back({b.planes, S * (size_t)d.PW * 4});
    s.push_back({b.meta0, S * 4});
    s.push_back({b.meta1, S * 4});
    s.push_back({b.heads, (size_t)6 * b.nD * 4});
  }
  return s;
}

size_t state_size(mz_handle* h) {
  size_t n = MZ_STATE_HEADER_BYTES;
  for (const Section& s : state_sections(h)) n += (s.bytes + 255) & ~(size_t)255;
  return n;
}

int active_bank(const mz_handle* h) {
  const MzDev& d = h->d;
  if (!d.bk_K || !h->bank.K) return -1;
  return d.bk_cells == h->bank.cells ? 0 : 1;
}

}  // namespace

extern "C" {

int mz_state_bytes(mz_handle* h, uint64_t* bytes_out) {
  if (!h || !bytes_out) return fail(MZ_EINVAL, "bad arguments");
  *bytes_out = state_size(h);
  return MZ_OK;
}

int mz_state_save(mz_handle* h, void* dst_dev, uint64_t bytes, void* stream) {
  if (!h || !dst_dev) return fail(MZ_EINVAL, "bad arguments");
  if (bytes < state_size(h)) return fail(MZ_EINVAL, "state buffer of %llu bytes, %zu needed",
                                         (unsigned long long)bytes, state_size(h));
  DeviceGuard g(h->cfg.device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const MzDev& d = h->d;
  const MzBankStore& b = h->bank;
  uint32_t hdr[MZ_STATE_HEADER_BYTES / 4] = {};
  hdr[SH_MAGIC] = kStateMagic;
  hdr[SH_VER] = kStateVersion;
  hdr[SH_B] = (uint32_t)d.B;
  hdr[SH_P] = (uint32_t)d.P;
  hdr[SH_TOR] = (uint32_t)d.toroidal;
  hdr[SH_ENRICH] = (uint32_t)d.enrich;
  hdr[SH_NS] = (uint32_t)d.NS;
  hdr[SH_PW] = (uint32_t)d.PW;
  hdr[SH_BK_K] = (uint32_t)b.K;
  hdr[SH_BK_NA] = (uint32_t)b.nA;
  hdr[SH_BK_ND] = (uint32_t)b.nD;
  hdr[SH_BK_AMASK] = b.amask;
  hdr[SH_BK_ACTIVE] = (uint32_t)active_bank(h);
  hdr[SH_BK_EPOCH0] = b.epoch[0];
  hdr[SH_BK_EPOCH1] = b.epoch[1];
  uint8_t* dims = reinterpret_cast<uint8_t*>(hdr + SH_DIMS);
  for (int i = 0; i < b.nD; ++i) dims[i] = (uint8_t)b.dims[i];
  uint8_t* dst = static_cast<uint8_t*>(dst_dev);
  // the header leaves from this stack frame: wait for it (a checkpoint is off the hot path)
  MZ_HIP(hipMemcpyAsync(dst, hdr, sizeof hdr, hipMemcpyHostToDevice, s));
  MZ_HIP(hipStreamSynchronize(s));
  size_t off = MZ_STATE_HEADER_BYTES;
  for (const Section& sec : state_sections(h)) {
    MZ_HIP(hipMemcpyAsync(dst + off, sec.p, sec.bytes, hipMemcpyDeviceToDevice, s));
    off += (sec.bytes + 255) & ~(size_t)255;
  }
  return MZ_OK;
}

int mz_state_load(mz_handle* h, const void* src_dev, uint64_t bytes, void* stream) {
  if (!h || !src_dev) return fail(MZ_EINVAL, "bad arguments");
  if (bytes < MZ_STATE_HEADER_BYTES) return fail(MZ_EINVAL, "state buffer too small");
  DeviceGuard g(h->cfg.device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  uint32_t hdr[MZ_STATE_HEADER_BYTES / 4];
  MZ_HIP(hipMemcpyAsync(hdr, src_dev, sizeof hdr, hipMemcpyDeviceToHost, s));
  MZ_HIP(hipStreamSynchronize(s));
  const MzDev& d = h->d;
  MzBankStore& b = h->bank;
  if (hdr[SH_MAGIC] != kStateMagic || hdr[SH_VER] != kStateVersion)
    return fail(MZ_EINVAL, "not an env state (magic %08x version %u)", hdr[SH_MAGIC], hdr[SH_VER]);
  if (hdr[SH_B] != (uint32_t)d.B || hdr[SH_P] != (uint32_t)d.P ||
      hdr[SH_TOR] != (uint32_t)d.toroidal || hdr[SH_ENRICH] != (uint32_t)d.enrich ||
      hdr[SH_NS] != (uint32_t)d.NS || hdr[SH_PW] != (uint32_t)d.PW)
    return fail(MZ_EINVAL, "env state of %u instances, max_dim %u, toroidal %u, enrich %u does not "
                "fit this handle (%d, %d, %d, %d)", hdr[SH_B], hdr[SH_P], hdr[SH_TOR],
                hdr[SH_ENRICH], d.B, d.P, d.toroidal, d.enrich);
  const uint8_t* dims = reinterpret_cast<const uint8_t*>(hdr + SH_DIMS);
  bool same_bank = hdr[SH_BK_K] == (uint32_t)b.K && hdr[SH_BK_NA] == (uint32_t)b.nA &&
                   hdr[SH_BK_ND] == (uint32_t)b.nD && hdr[SH_BK_AMASK] == b.amask;
  for (int i = 0; same_bank && i < b.nD; ++i) same_bank = dims[i] == (uint8_t)b.dims[i];
  if (!same_bank)
    return fail(MZ_EINVAL, "env state has a maze bank of %u slots x %u algorithms x %u sizes "
                "(mask %u); this handle's is %d x %d x %d (mask %u)", hdr[SH_BK_K], hdr[SH_BK_NA],
                hdr[SH_BK_ND], hdr[SH_BK_AMASK], b.K, b.nA, b.nD, b.amask);
  if (bytes < state_size(h)) return fail(MZ_EINVAL, "state buffer of %llu bytes, %zu needed",
                                         (unsigned long long)bytes, state_size(h));
  const uint8_t* src = static_cast<const uint8_t*>(src_dev);
  size_t off = MZ_STATE_HEADER_BYTES;
  for (const Section& sec : state_sections(h)) {
    MZ_HIP(hipMemcpyAsync(sec.p, src + off, sec.bytes, hipMemcpyDeviceToDevice, s));
    off += (sec.bytes + 255) & ~(size_t)255;
  }
  if (b.K) {
    b.epoch[0] = hdr[SH_BK_EPOCH0];
    b.epoch[1] = hdr[SH_BK_EPOCH1];
  }
  return mz_bank_use(h, (int32_t)hdr[SH_BK_ACTIVE]);
}

int mz_maze_metrics(mz_handle* h, const int32_t* env_ids_dev, int32_t n, double* out_dev,
                    void* stream) {
  if (!h || !out_dev) return fail(MZ_EINVAL, "bad arguments");
  if (h->d.toroidal) return fail(MZ_EINVAL, "maze metrics are defined for euclidean mazes");
  if (!env_ids_dev) n = h->d.B;
  if (n < 0 || n > h->d.B) return fail(MZ_EINVAL, "n out of range");
  DeviceGuard g(h->cfg.device);
  MZ_HIP(mz_launch_metrics(h->d, env_ids_dev, n, out_dev, static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_difficulty_batch(mz_handle* h, const int32_t* env_ids_dev, int32_t n, double* out_dev,
                        int32_t* status_dev, void* stream) {
  if (!h || !out_dev || !status_dev) return fail(MZ_EINVAL, "bad arguments");
  if (!env_ids_dev) n = h->d.B;
  if (n < 0 || (!env_ids_dev && n > h->d.B)) return fail(MZ_EINVAL, "n out of range");
  int mm = 0;
  if (mz_mcclendon_lds(h->d.P, h->d.toroidal != 0, &mm) > 160 * 1024)
    return fail(MZ_EINVAL_SHAPE, "maze pitch beyond the difficulty kernel's LDS plan");
  DeviceGuard g(h->cfg.device);
  MZ_HIP(mz_launch_mcclendon(h->d, env_ids_dev, n, out_dev, status_dev,
                             static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_set_algorithm(mz_handle* h, const uint8_t* algo_dev, int32_t algo_all, void* stream) {
  if (!h) return fail(MZ_EINVAL, "null handle");
  DeviceGuard g(h->cfg.device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (algo_dev) MZ_HIP(hipMemcpyAsync(h->d.algo, algo_dev, h->d.B, hipMemcpyDeviceToDevice, s));
  else {
    if (algo_all < 0 || algo_all > 2) return fail(MZ_EINVAL, "algorithm id %d", algo_all);
    MZ_HIP(hipMemsetAsync(h->d.algo, algo_all, h->d.B, s));
  }
  return MZ_OK;
}

int mz_get_meta(mz_handle* h, int32_t* meta_dev, void* stream) {
  if (!h || !meta_dev) return fail(MZ_EINVAL, "bad arguments");
  DeviceGuard g(h->cfg.device);
  MZ_HIP(mz_launch_meta(h->d, meta_dev, static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_discounted_returns(const double* rew_dev, int32_t ld, const int32_t* rows_dev,
                          const int32_t* lens_dev, int32_t n, double gamma, float* out_dev,
                          int32_t ldo, void* stream) {
  if (!rew_dev || !rows_dev || !lens_dev || !out_dev || n < 0) return fail(MZ_EINVAL, "bad arguments");
  StreamGuard g(stream);
  MZ_HIP(mz_launch_returns(rew_dev, ld, rows_dev, lens_dev, n, gamma, out_dev, ldo,
                           static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_query(mz_handle* h, int32_t env, mz_env_info* info) {
  if (!h || !info || env < 0 || env >= h->d.B) return fail(MZ_EINVAL, "bad arguments");
  DeviceGuard g(h->cfg.device);
  MZ_HIP(hipDeviceSynchronize());
  uint32_t m0, m1, pw, sw;
  MZ_HIP(hipMemcpy(&m0, h->d.meta0 + env, 4, hipMemcpyDeviceToHost));
  MZ_HIP(hipMemcpy(&m1, h->d.meta1 + env, 4, hipMemcpyDeviceToHost));
  MZ_HIP(hipMemcpy(&pw, h->d.posw + env, 4, hipMemcpyDeviceToHost));
  MZ_HIP(hipMemcpy(&sw, h->d.stw + env, 4, hipMemcpyDeviceToHost));
  info->n = m0 & 0xFF;
  info->start_r = (m0 >> 16) & 0xFF; info->start_c = m0 >> 24;
  info->goal_r = m1 & 0xFF; info->goal_c = (m1 >> 8) & 0xFF; info->max_steps = m1 >> 16;
  info->r = pw & 0xFF; info->c = (pw >> 8) & 0xFF; info->nmoves = (pw >> 16) & 3;
  info->last_action = (pw >> 18) & 3; info->done = (pw >> 20) & 1;
  info->steps = sw & 0xFFFF; info->invalid_streak = (sw >> 16) & 0xFF;
  return MZ_OK;
}

int mz_get_grid(mz_handle* h, int32_t env, uint8_t* grid_host) {
  if (!h || !grid_host || env < 0 || env >= h->d.B) return fail(MZ_EINVAL, "bad arguments");
  mz_env_info info;
  int rc = mz_query(h, env, &info);
  if (rc) return rc;
  const int P = h->d.P, N = info.n;
  std::vector<uint32_t> cw((size_t)P * P);
  DeviceGuard g(h->cfg.device);
  MZ_HIP(hipMemcpy(cw.data(), h->d.cells + (size_t)env * P * P, 4 * cw.size(), hipMemcpyDeviceToHost));
  for (int r = 0; r < N; ++r)
    for (int c = 0; c < N; ++c) {
      const bool open = (cw[(size_t)r * P + c] & MZ_CELL_OPEN) != 0;
      grid_host[r * N + c] = !open ? 0 : ((r == info.goal_r && c == info.goal_c) ? 2 : 1);
    }
  return MZ_OK;
}

int mz_host_alloc(uint64_t bytes, int32_t device, void** host_out, void** dev_out) {
  if (!host_out || !dev_out || bytes == 0) return fail(MZ_EINVAL, "bad arguments");
  int ndev = 0;
  MZ_HIP(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(MZ_EINVAL, "device %d not present", device);
  DeviceGuard g(device);
  void* hp = nullptr;
  MZ_HIP(hipHostMalloc(&hp, (size_t)bytes, hipHostMallocMapped | hipHostMallocCoherent));
  void* dp = nullptr;
  const hipError_t e = hipHostGetDevicePointer(&dp, hp, 0);
  if (e != hipSuccess) {
    (void)hipHostFree(hp);
    return fail(MZ_EHIP, "hipHostGetDevicePointer: %s", hipGetErrorString(e));
  }
  std::memset(hp, 0, (size_t)bytes);
  *host_out = hp;
  *dev_out = dp;
  return MZ_OK;
}

int mz_host_free(void* host) {
  if (!host) return MZ_OK;
  MZ_HIP(hipHostFree(host));
  return MZ_OK;
}

}  // extern "C"


// ---- trainer bookkeeping (mz_trainer.hip)
int mz_trainer_tick(const uint8_t* term_dev, const uint8_t* trunc_dev, float* steps_done_dev,
                    double eps_start, double eps_final, double eps_decay, float* eps_out_dev,
                    int64_t* wins_dev, int64_t* episodes_dev, uint64_t seed, uint64_t counter,
                    int32_t n, int32_t* scratch_dev, int32_t* rows_dev, int32_t* count_dev,
                    void* stream) {
  if (n < 0 || (n > 0 && (!term_dev || !trunc_dev || !steps_done_dev || !eps_out_dev ||
                          !scratch_dev || !rows_dev || !count_dev)))
    return fail(MZ_EINVAL, "bad arguments");
  if (!(eps_decay > 0.0)) return fail(MZ_EINVAL, "eps_decay %g", eps_decay);
  const float inv_decay = 1.0f / (float)eps_decay;  // as torch's division by a CPU scalar
  MZ_HIP(mz_launch_tick(term_dev, trunc_dev, steps_done_dev, (float)eps_final,
                        (float)(eps_start - eps_final), inv_decay, eps_out_dev,
                        reinterpret_cast<unsigned long long*>(wins_dev),
                        reinterpret_cast<unsigned long long*>(episodes_dev), seed, counter, n,
                        scratch_dev, rows_dev, count_dev, static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_greedy_scatter(const uint16_t* q_dev, int32_t ldq, const int32_t* rows_dev,
                      const int32_t* count_dev, int32_t m, int64_t* greedy_dev, void* stream) {
  if (m < 0 || ldq < 4 || (m > 0 && (!q_dev || !rows_dev || !count_dev || !greedy_dev)))
    return fail(MZ_EINVAL, "bad arguments");
  MZ_HIP(mz_launch_greedy_scatter(q_dev, ldq, rows_dev, count_dev, m, greedy_dev,
                                  static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_head_bf16(const float* w0, const float* b0, const float* w1, const float* b1,
                 const float* w2, const float* b2, int32_t out0, int32_t in0, int32_t out1,
                 int32_t in1, int32_t out2, int32_t in2, int32_t ld0, int32_t conv_out,
                 int32_t conv_ch, uint16_t* dw0, uint16_t* db0, uint16_t* dw1, uint16_t* db1,
                 uint16_t* dw2, uint16_t* db2, void* stream) {
  if (!w0 || !b0 || !w1 || !b1 || !w2 || !b2 || !dw0 || !db0 || !dw1 || !db1 || !dw2 || !db2)
    return fail(MZ_EINVAL, "bad arguments");
  if (out0 <= 0 || out1 <= 0 || out2 <= 0 || in1 != out0 || in2 != out1 || in0 > ld0 ||
      conv_ch <= 0 || conv_out < 0 || conv_out > in0 || conv_out % conv_ch != 0 || in0 > 2048)
    return fail(MZ_EINVAL, "head shapes");
  MzHeadBf16 h{{w0, w1, w2}, {b0, b1, b2}, {dw0, dw1, dw2}, {db0, db1, db2},
               {out0, out1, out2}, {in0, in1, in2}, ld0, conv_out, conv_ch};
  MZ_HIP(mz_launch_head_bf16(h, static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_replay_push(int32_t n, int64_t capacity, int64_t ptr, const float* obs6_src,
                   const int32_t* bits_src, const int32_t* act_src, const float* rew_src,
                   const float* obs6n_src, const int32_t* bitsn_src, float* s6_dev,
                   int32_t* sw_dev, int64_t* a_dev, float* r_dev, float* s6n_dev,
                   int32_t* swn_dev, int32_t obs_dim, int32_t window_words, void* stream) {
  if (n < 0 || n > capacity || ptr < 0 || ptr >= capacity || obs_dim <= 0 || window_words <= 0)
    return fail(MZ_EINVAL, "bad arguments");
  const void* src[6] = {obs6_src, bits_src, act_src, rew_src, obs6n_src, bitsn_src};
  void* dst[6] = {s6_dev, sw_dev, a_dev, r_dev, s6n_dev, swn_dev};
  for (int j = 0; j < 6; ++j)
    if (src[j] && !dst[j]) return fail(MZ_EINVAL, "replay array %d missing", j);
  MzReplayPush p{{src[0], src[1], src[2], src[3], src[4], src[5]},
                 {dst[0], dst[1], dst[2], dst[3], dst[4], dst[5]},
                 {obs_dim, window_words, 1, 1, obs_dim, window_words}, n, capacity, ptr};
  MZ_HIP(mz_launch_replay_push(p, static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_replay_sample_idx(uint64_t seed, uint64_t counter, int64_t newest, int64_t n_avail,
                         int64_t capacity, int64_t* out_dev, int32_t n, void* stream) {
  if (n < 0 || capacity <= 0 || n_avail <= 0 || n_avail > capacity || (n > 0 && !out_dev))
    return fail(MZ_EINVAL, "bad arguments");
  MZ_HIP(mz_launch_replay_idx(seed, counter, newest, n_avail, capacity, out_dev, n,
                              static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_q_loss(const float* q_dev, int32_t ldq, const float* q_next_dev, int32_t ldn,
              const float* q_tgt_dev, int32_t ldt, const int64_t* action_dev,
              const float* reward_dev, double gamma, int32_t b, float* loss_dev, float* diff_dev,
              void* stream) {
  if (b <= 0 || !q_dev || !q_tgt_dev || !action_dev || !reward_dev || !loss_dev || !diff_dev ||
      ldq < 4 || ldt < 4 || (q_next_dev && ldn < 4))
    return fail(MZ_EINVAL, "bad arguments");
  MZ_HIP(mz_launch_q_loss(q_dev, ldq, q_next_dev, ldn, q_tgt_dev, ldt, action_dev, reward_dev,
                          (float)gamma, b, loss_dev, diff_dev, static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_q_loss_backward(const float* grad_dev, const float* diff_dev, const int64_t* action_dev,
                       int32_t b, int32_t rows, float* dq_dev, void* stream) {
  if (b <= 0 || rows < b || !grad_dev || !diff_dev || !action_dev || !dq_dev)
    return fail(MZ_EINVAL, "bad arguments");
  const float norm = (float)(2.0 / (double)b);  // mse_loss backward: 2 / numel
  MZ_HIP(mz_launch_q_loss_bwd(grad_dev, diff_dev, action_dev, b, rows, norm, dq_dev,
                              static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_head_loss_workspace_floats(int32_t b) {
  return b <= 0 ? 0 : mz_head_loss_blocks(b);
}

int mz_head_loss(const float* z2s_dev, int32_t lds, const float* w3s_dev, const float* b3s_dev,
                 const float* z2t_dev, int32_t ldt, const float* w3t_dev, const float* b3t_dev,
                 int32_t hidden, int32_t act, int32_t stacked, const int64_t* action_dev,
                 const float* reward_dev, double gamma, int32_t b, float* part_dev,
                 uint32_t* ticket_dev, float* loss_dev, float* diff_dev, void* stream) {
  if (b <= 0 || hidden <= 0 || hidden % 4 || (act != 0 && act != 1) || !z2s_dev || !w3s_dev ||
      !b3s_dev || !z2t_dev || !w3t_dev || !b3t_dev || !action_dev || !reward_dev || !part_dev ||
      !loss_dev || !diff_dev || lds < hidden || ldt < hidden)
    return fail(MZ_EINVAL, "bad arguments");
  MzHeadLoss p{z2s_dev, w3s_dev, b3s_dev, z2t_dev, w3t_dev, b3t_dev, lds, ldt, stacked ? 1 : 0, b,
               hidden, act, action_dev, reward_dev, (float)gamma, part_dev, ticket_dev, loss_dev,
               diff_dev};
  MZ_HIP(mz_launch_head_loss(p, static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_head_loss_backward_workspace_floats(int32_t b, int32_t hidden) {
  return b <= 0 ? 0 : mz_head_loss_bwd_blocks(b) * (4 * hidden + 4);
}

int mz_head_loss_backward(const float* grad_dev, const float* diff_dev, const int64_t* action_dev,
                          int32_t b, const float* z2s_dev, int32_t lds, const float* w3s_dev,
                          int32_t hidden, int32_t act, float* dz2_dev, int32_t ldd,
                          float* part_dev, void* stream) {
  if (b <= 0 || hidden <= 0 || hidden % 4 || (act != 0 && act != 1) || !grad_dev || !diff_dev ||
      !action_dev || !z2s_dev || !w3s_dev || !dz2_dev || !part_dev || lds < hidden || ldd < hidden)
    return fail(MZ_EINVAL, "bad arguments");
  const float norm = (float)(2.0 / (double)b);  // mse_loss backward: 2 / numel
  MZ_HIP(mz_launch_head_loss_bwd(grad_dev, diff_dev, action_dev, b, norm, z2s_dev, lds, w3s_dev,
                                 hidden, act, dz2_dev, ldd, part_dev,
                                 static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_adamw_groups(float* param_dev, float* exp_avg_dev, float* exp_avg_sq_dev,
                    const float* const* grads_dev, const int64_t* seg_len,
                    const int32_t* seg_group, int32_t nseg, const float* lr_dev, float* step_dev,
                    double beta1, double beta2, double eps, double weight_decay, float max_norm,
                    float* scratch_dev, void* stream) {
  if (!param_dev || !exp_avg_dev || !exp_avg_sq_dev || !grads_dev || !seg_len || !seg_group ||
      !lr_dev || !step_dev || !scratch_dev)
    return fail(MZ_EINVAL, "bad arguments");
  if (nseg < 1 || nseg > MZ_OPT_MAX_SEGS) return fail(MZ_EINVAL, "segment count %d", nseg);
  const uintptr_t al = reinterpret_cast<uintptr_t>(param_dev) |
                       reinterpret_cast<uintptr_t>(exp_avg_dev) |
                       reinterpret_cast<uintptr_t>(exp_avg_sq_dev);
  if (al & 15) return fail(MZ_EALIGN, "flat buffers must be 16-byte aligned");
  for (int k = 0; k < nseg; ++k) {
    if (!grads_dev[k] || seg_len[k] <= 0 || (seg_len[k] & 3))
      return fail(MZ_EINVAL, "segment %d: length %lld (multiple of 4 required)", k,
                  (long long)seg_len[k]);
    if (reinterpret_cast<uintptr_t>(grads_dev[k]) & 15)
      return fail(MZ_EALIGN, "gradient %d must be 16-byte aligned", k);
    if (seg_group[k] < 0) return fail(MZ_EINVAL, "segment %d: group %d", k, seg_group[k]);
  }
  MZ_HIP(mz_launch_adamw_groups(param_dev, exp_avg_dev, exp_avg_sq_dev, grads_dev, seg_len,
                                seg_group, nseg, lr_dev, step_dev, beta1, beta2, eps,
                                weight_decay, max_norm, scratch_dev,
                                static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_ppo_act(const float* logits_dev, int32_t ldl, const float* value_dev, int32_t ldv,
               const float* obs6_dev, const uint32_t* bits_dev, int32_t B, int32_t L, uint64_t seed,
               uint64_t counter, const int32_t* t_dev, float* rec_s6_dev, uint32_t* rec_w_dev,
               int64_t* rec_a_dev, float* rec_lp_dev, float* rec_v_dev, int32_t* act_out_dev,
               void* stream) {
  if (!logits_dev || !value_dev || !obs6_dev || !bits_dev || !t_dev || !rec_s6_dev || !rec_w_dev ||
      !rec_a_dev || !rec_lp_dev || !rec_v_dev || !act_out_dev || B < 0 || L < 1 || ldl < 4 ||
      ldv < 1)
    return fail(MZ_EINVAL, "bad arguments");
  StreamGuard g(stream);
  MzPpoAct q{logits_dev, ldl, value_dev, ldv, obs6_dev, bits_dev, B, L, seed, counter, t_dev,
             rec_s6_dev, rec_w_dev, rec_a_dev, rec_lp_dev, rec_v_dev, act_out_dev};
  MZ_HIP(mz_launch_ppo_act(q, static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_ppo_scan(const double* reward64_dev, const uint8_t* term_dev, const uint8_t* trunc_dev,
                int32_t B, int32_t L, int32_t* t_dev, double* rec_r_dev, int32_t* fin_id_dev,
                int64_t* fin_off_dev, int32_t* fin_len_dev, int32_t* fin_count_dev,
                int64_t* pool_fill_dev, int64_t* pool_total_dev, int64_t* stats_dev,
                void* stream) {
  if (!reward64_dev || !term_dev || !trunc_dev || !t_dev || !rec_r_dev || !fin_id_dev ||
      !fin_off_dev || !fin_len_dev || !fin_count_dev || !pool_fill_dev || !pool_total_dev ||
      !stats_dev || B < 0 || L < 1)
    return fail(MZ_EINVAL, "bad arguments");
  StreamGuard g(stream);
  MzPpoScan q{reward64_dev, term_dev, trunc_dev, B, L, t_dev, rec_r_dev, fin_id_dev, fin_off_dev,
              fin_len_dev, fin_count_dev, pool_fill_dev, pool_total_dev,
              reinterpret_cast<long long*>(stats_dev)};
  MZ_HIP(mz_launch_ppo_scan(q, static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_ppo_finish(const double* rec_r_dev, const float* rec_s6_dev, const uint32_t* rec_w_dev,
                  const int64_t* rec_a_dev, const float* rec_lp_dev, const float* rec_v_dev,
                  int32_t B, int32_t L, const int32_t* fin_id_dev, const int64_t* fin_off_dev,
                  const int32_t* fin_len_dev, const int32_t* fin_count_dev, double gamma,
                  int64_t capacity, float* pool_s6_dev, uint32_t* pool_w_dev, int64_t* pool_a_dev,
                  float* pool_lp_dev, float* pool_adv_dev, float* pool_ret_dev, void* stream) {
  if (!rec_r_dev || !rec_s6_dev || !rec_w_dev || !rec_a_dev || !rec_lp_dev || !rec_v_dev ||
      !fin_id_dev || !fin_off_dev || !fin_len_dev || !fin_count_dev || !pool_s6_dev ||
      !pool_w_dev || !pool_a_dev || !pool_lp_dev || !pool_adv_dev || !pool_ret_dev || B < 0 ||
      L < 1 || capacity < 0)
    return fail(MZ_EINVAL, "bad arguments");
  StreamGuard g(stream);
  MzPpoFinish q{rec_r_dev, rec_s6_dev, rec_w_dev, rec_a_dev, rec_lp_dev, rec_v_dev, L, fin_id_dev,
                fin_off_dev, fin_len_dev, fin_count_dev, gamma, capacity, pool_s6_dev, pool_w_dev,
                pool_a_dev, pool_lp_dev, pool_adv_dev, pool_ret_dev};
  MZ_HIP(mz_launch_ppo_finish(q, B, static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_ppo_head_loss(const float* logits_dev, int32_t ldl, const float* value_dev, int32_t ldv,
                     const int64_t* action_dev, const float* lp_old_dev, const float* adv_dev,
                     const float* ret_dev, const float* coef_dev, int32_t b, float clip,
                     float* scratch_dev, float* loss_dev, float* dlogits_dev, int32_t ldg,
                     float* dvalue_dev, int32_t ldvg, void* stream) {
  if (!logits_dev || !value_dev || !action_dev || !lp_old_dev || !adv_dev || !ret_dev ||
      !coef_dev || !scratch_dev || !loss_dev || !dlogits_dev || !dvalue_dev || b < 0 || ldl < 4 ||
      ldg < 4 || ldv < 1 || ldvg < 1)
    return fail(MZ_EINVAL, "bad arguments");
  StreamGuard g(stream);
  float* w = scratch_dev;
  MzPpoHead q{logits_dev, ldl, value_dev, ldv, action_dev, lp_old_dev, adv_dev, ret_dev, coef_dev,
              b, w, w + b, w + 2 * (size_t)b, w + 6 * (size_t)b, w + 10 * (size_t)b,
              w + 11 * (size_t)b, loss_dev, dlogits_dev, ldg, dvalue_dev, ldvg};
  MZ_HIP(mz_launch_ppo_head(q, clip, static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int mz_qact_prepare(const float* fc1_w_dev, const float* fc2_w_dev, uint16_t* w1_hi_dev,
                    uint16_t* w1_lo_dev, uint16_t* w2_hi_dev, uint16_t* w2_lo_dev, void* stream) {
  if (!fc1_w_dev || !fc2_w_dev || !w1_hi_dev || !w1_lo_dev || !w2_hi_dev || !w2_lo_dev)
    return fail(MZ_EINVAL, "bad arguments");
  for (const void* p : {(const void*)fc1_w_dev, (const void*)fc2_w_dev, (const void*)w1_hi_dev,
                        (const void*)w1_lo_dev, (const void*)w2_hi_dev, (const void*)w2_lo_dev})
    if (reinterpret_cast<uintptr_t>(p) & 15) return fail(MZ_EINVAL, "weights / images must be 16-B aligned");
  StreamGuard g(stream);
  MZ_HIP(mz_launch_qact_prepare(fc1_w_dev, fc2_w_dev, w1_hi_dev, w1_lo_dev, w2_hi_dev, w2_lo_dev,
                                static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

int64_t mz_qact_workspace_floats(int32_t n) { return n > 0 ? mz_qact_ws_floats(n) : 0; }

int mz_qact(const uint32_t* bits_dev, const float* obs6_dev, const int32_t* rows_dev,
            const int32_t* count_dev, int32_t n, const float* conv_w_dev, const float* conv_b_dev,
            const uint16_t* w1_hi_dev, const uint16_t* w1_lo_dev, const float* b1_dev,
            const uint16_t* w2_hi_dev, const uint16_t* w2_lo_dev, const float* b2_dev,
            const float* w3_dev, const float* b3_dev, int32_t relu, float drop_p, uint64_t seed,
            uint64_t counter, float* h1_dev, int64_t* greedy_dev, float* q_out_dev, void* stream) {
  if (!bits_dev || !obs6_dev || !conv_w_dev || !conv_b_dev || !w1_hi_dev || !w1_lo_dev ||
      !b1_dev || !w2_hi_dev || !w2_lo_dev || !b2_dev || !w3_dev || !b3_dev || !h1_dev || n < 0 ||
      (!greedy_dev && !q_out_dev))
    return fail(MZ_EINVAL, "bad arguments");
  if (count_dev && !rows_dev) return fail(MZ_EINVAL, "a device count needs a row list");
  if (!(drop_p >= 0.0f && drop_p < 1.0f)) return fail(MZ_EINVAL, "dropout p %g", (double)drop_p);
  const uintptr_t al = reinterpret_cast<uintptr_t>(w1_hi_dev) | reinterpret_cast<uintptr_t>(w1_lo_dev) |
                       reinterpret_cast<uintptr_t>(w2_hi_dev) | reinterpret_cast<uintptr_t>(w2_lo_dev) |
                       reinterpret_cast<uintptr_t>(h1_dev) | reinterpret_cast<uintptr_t>(q_out_dev);
  if (al & 15) return fail(MZ_EALIGN, "weight images, h1 and q_out must be 16-byte aligned");
  StreamGuard g(stream);
  const uint64_t k = seed * 0x9E3779B97F4A7C15ull + counter * 0xD1B54A32D192ED03ull + 1;
  MzQAct q{bits_dev, obs6_dev, rows_dev, count_dev, n, conv_w_dev, conv_b_dev, w1_hi_dev,
           w1_lo_dev, b1_dev, w2_hi_dev, w2_lo_dev, b2_dev, w3_dev, b3_dev,
           drop_p > 0.0f ? (uint32_t)(drop_p * 65536.0f + 0.5f) : 0u,
           drop_p > 0.0f ? 1.0f / (1.0f - drop_p) : 1.0f, (uint32_t)(k ^ (k >> 32)), h1_dev,
           greedy_dev, q_out_dev};
  MZ_HIP(mz_launch_qact(q, relu, static_cast<hipStream_t>(stream)));
  return MZ_OK;
}

