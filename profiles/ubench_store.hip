// ubench_store.hip — the store ceiling k_step's f32 window phase runs against (MI355X).
//
// k_step writes 65,536 x 2,700 B of f32 windows per launch (177 MB), 16 instances per single-wave
// workgroup = 43,200 contiguous bytes per wave, 16-B stores. This measures the same store stream
// alone (no loads, no compute), with each store policy, and with a load phase of k_step's size
// in front (one dependent random-line gather per lane, then the stores), to separate the store
// ceiling from the cost of the load phase that precedes it.
//
//   hipcc --offload-arch=gfx950 -O3 -o profiles/_bin/ubench_store profiles/ubench_store.hip
//   profiles/_bin/ubench_store [waves=4096] [iters=200]
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
constexpr int PER_WAVE = 16 * 675;  // floats per wave (16 windows)

template <int POL, int GATHER>
__global__ __launch_bounds__(64) void k_store(float* out, const uint32_t* table, size_t tmask,
                                              uint32_t salt) {
  const int lane = threadIdx.x;
  const size_t w = blockIdx.x;
  float* o = out + w * PER_WAVE;
  uint32_t v = salt;
  if (GATHER) {
    // two dependent random 128-B-line reads per lane (k_step: state, then cell word + band)
    uint32_t h = (uint32_t)(w * 64 + lane) * 2654435761u ^ salt;
    v = table[(h & tmask) * 32];
    h = h * 1664525u + v;
    v += table[(h & tmask) * 32 + 1];
  }
  const float f = (float)(v & 1u);
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(o, 0, PER_WAVE * 4, 0x00020000);
  for (int q = lane; q < PER_WAVE / 4; q += 64) {
    float4 x = make_float4(f, (float)(q & 1), (float)((q >> 1) & 1), 1.0f);
    if (POL < 0) reinterpret_cast<float4*>(o)[q] = x;
    else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, x), rsrc, q * 16, 0, POL);
  }
}

template <int POL, int GATHER>
float run(int waves, int iters, float* out, const uint32_t* table, size_t tmask) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 10; ++i) hipLaunchKernelGGL((k_store<POL, GATHER>), waves, 64, 0, 0, out, table, tmask, i);
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < iters; ++i)
    hipLaunchKernelGGL((k_store<POL, GATHER>), waves, 64, 0, 0, out, table, tmask, i);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3f / iters;
}

int main(int argc, char** argv) {
  const int waves = argc > 1 ? atoi(argv[1]) : 4096;
  const int iters = argc > 2 ? atoi(argv[2]) : 200;
  const size_t bytes = (size_t)waves * PER_WAVE * 4;
  const size_t tlines = (size_t)1 << 24;  // 16 M lines x 128 B = 2 GiB gather table (> L3)
  float* out;
  uint32_t* table;
  CK(hipMalloc(&out, bytes));
  CK(hipMalloc(&table, tlines * 128));
  CK(hipMemset(table, 1, tlines * 128));
  const size_t tmask = tlines - 1;
  struct { const char* name; float us; } r[11];
  r[0] = {"store sc1 (k_step policy)", run<16, 0>(waves, iters, out, table, tmask)};
  r[1] = {"store plain", run<-1, 0>(waves, iters, out, table, tmask)};
  r[2] = {"store nt", run<2, 0>(waves, iters, out, table, tmask)};
  r[3] = {"gather x2 + store sc1", run<16, 1>(waves, iters, out, table, tmask)};
  r[4] = {"gather x2 + store plain", run<-1, 1>(waves, iters, out, table, tmask)};
  r[6] = {"store sc0", run<1, 0>(waves, iters, out, table, tmask)};
  r[7] = {"store sc0 sc1", run<17, 0>(waves, iters, out, table, tmask)};
  r[8] = {"store sc0 nt", run<3, 0>(waves, iters, out, table, tmask)};
  r[9] = {"store sc1 nt", run<18, 0>(waves, iters, out, table, tmask)};
  r[10] = {"store sc0 sc1 nt", run<19, 0>(waves, iters, out, table, tmask)};
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < iters; ++i) CK(hipMemsetAsync(out, i, bytes, 0));
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  r[5] = {"hipMemsetAsync", ms * 1e3f / iters};
  for (auto& x : r)
    printf("{\"what\": \"%s\", \"waves\": %d, \"bytes\": %zu, \"us\": %.2f, \"TBps\": %.3f}\n", x.name,
           waves, bytes, x.us, bytes / (x.us * 1e-6) / 1e12);
  CK(hipFree(out));
  CK(hipFree(table));
  return 0;
}
