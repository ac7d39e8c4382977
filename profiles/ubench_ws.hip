// ubench_ws.hip — can a loader / storer wave split hide k_step's gather phase behind its stores?
//
// Same stream as ubench_store.hip: 4,096 groups, each two dependent random 128-B-line gathers per
// lane (k_step's level 1 / level 2) followed by 43,200 B of 16-B write-through stores (16 f32
// windows). ubench_store runs one single-wave workgroup per group: every wave gathers first, so
// the whole chip gathers before anything is stored (37.1 us vs 25.5 us for the stores alone).
// Here a workgroup = one loader wave + one storer wave stepping G groups in turn: in iteration
// `it` the loader gathers group it while the storer stores group it - 1 (a double-buffered LDS
// slot, one barrier per iteration). A wave's vmcnt counts its stores too, so one wave cannot run
// the next group's gathers ahead of its own stores; two waves can.
//
//   hipcc --offload-arch=gfx950 -O3 -o profiles/_bin/ubench_ws profiles/ubench_ws.hip
//   profiles/_bin/ubench_ws [iters=200]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
constexpr int PER_GROUP = 16 * 675;  // floats per group (16 windows)
constexpr int GROUPS = 4096;

__device__ inline uint32_t gather2(const uint32_t* table, size_t tmask, size_t grp, int lane,
                                   uint32_t salt) {
  uint32_t h = (uint32_t)(grp * 64 + lane) * 2654435761u ^ salt;
  uint32_t v = table[(h & tmask) * 32];
  h = h * 1664525u + v;
  return v + table[(h & tmask) * 32 + 1];
}

__device__ inline void store_group(float* out, size_t grp, int lane, uint32_t v) {
  float* o = out + grp * PER_GROUP;
  const float f = (float)(v & 1u);
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(o, 0, PER_GROUP * 4, 0x00020000);
  for (int q = lane; q < PER_GROUP / 4; q += 64) {
    float4 x = make_float4(f, (float)(q & 1), (float)((q >> 1) & 1), 1.0f);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, x), rsrc, q * 16, 0, 16);
  }
}

// GATHER 0: the same loop without the gathers (the split's own store ceiling)
template <int GATHER>
__global__ __launch_bounds__(128) void k_ws(float* out, const uint32_t* table, size_t tmask,
                                            uint32_t salt, int G) {
  __shared__ uint32_t slot[2][64];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t nwg = gridDim.x;
  for (int it = 0; it <= G; ++it) {
    if (wv == 0 && it < G) {
      const size_t grp = (size_t)it * nwg + blockIdx.x;
      slot[it & 1][lane] = GATHER ? gather2(table, tmask, grp, lane, salt) : salt + lane;
    }
    if (wv == 1 && it > 0) {
      const size_t grp = (size_t)(it - 1) * nwg + blockIdx.x;
      store_group(out, grp, lane, slot[(it - 1) & 1][lane]);
    }
    __syncthreads();
  }
}

// reference: one single-wave workgroup per group, gathers then stores (ubench_store's variant)
__global__ __launch_bounds__(64) void k_flat(float* out, const uint32_t* table, size_t tmask,
                                             uint32_t salt) {
  const int lane = threadIdx.x;
  store_group(out, blockIdx.x, lane, gather2(table, tmask, blockIdx.x, lane, salt));
}

template <class F>
float timeit(int iters, F launch) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 10; ++i) launch(i);
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < iters; ++i) launch(i);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipGetLastError());
  return ms * 1e3f / iters;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 200;
  const size_t bytes = (size_t)GROUPS * PER_GROUP * 4;
  const size_t tlines = (size_t)1 << 24;  // 16 M lines x 128 B = 2 GiB gather table
  float* out;
  uint32_t* table;
  CK(hipMalloc(&out, bytes));
  CK(hipMalloc(&table, tlines * 128));
  CK(hipMemset(table, 1, tlines * 128));
  const size_t tmask = tlines - 1;
  auto report = [&](const char* what, int G, float us) {
    printf("{\"what\": \"%s\", \"groups_per_wg\": %d, \"bytes\": %zu, \"us\": %.2f, \"TBps\": %.3f}\n",
           what, G, bytes, us, bytes / (us * 1e-6) / 1e12);
  };
  report("flat: gather x2 then store, 1 wave per group", 1, timeit(iters, [&](int i) {
    hipLaunchKernelGGL(k_flat, GROUPS, 64, 0, 0, out, table, tmask, (uint32_t)i);
  }));
  for (int G : {1, 2, 4, 8, 16}) {
    report("split: loader + storer wave, gather x2", G, timeit(iters, [&](int i) {
      hipLaunchKernelGGL(k_ws<1>, GROUPS / G, 128, 0, 0, out, table, tmask, (uint32_t)i, G);
    }));
    report("split, no gathers", G, timeit(iters, [&](int i) {
      hipLaunchKernelGGL(k_ws<0>, GROUPS / G, 128, 0, 0, out, table, tmask, (uint32_t)i, G);
    }));
  }
  CK(hipFree(out));
  CK(hipFree(table));
  return 0;
}
