// ubench_ticket.hip — cost of finding the last workgroup of a launch with same-address atomics
// (k_adamw's publish_step, k_head_loss's partial sum) vs a two-level ticket (group counters, then
// a root counter). Each workgroup writes one partial, fences and takes its ticket; the last one
// sums the partials. Prints one JSON line per (variant, blocks).
//   hipcc --offload-arch=gfx950 -O3 -o profiles/_bin/ubench_ticket profiles/ubench_ticket.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <int G, int STRIDE>
__device__ inline bool last_block(unsigned* tk) {
  if (G <= 1) {
    if (atomicAdd(tk, 1u) != gridDim.x - 1) return false;
    *tk = 0u;
    return true;
  }
  const unsigned nb = gridDim.x, ng = nb < G ? nb : G, g = blockIdx.x % ng;
  const unsigned cnt = nb / ng + (g < nb % ng ? 1u : 0u);
  unsigned* gt = tk + (1 + g) * STRIDE;
  if (atomicAdd(gt, 1u) != cnt - 1) return false;
  *gt = 0u;
  __threadfence();
  if (atomicAdd(tk, 1u) != ng - 1) return false;
  *tk = 0u;
  return true;
}

template <int G, int STRIDE>
__global__ __launch_bounds__(256) void k_tick(float* part, unsigned* tk, float* out) {
  __shared__ bool last;
  if (threadIdx.x == 0) {
    part[blockIdx.x] = (float)blockIdx.x;
    __threadfence();
    last = last_block<G, STRIDE>(tk);
  }
  __syncthreads();
  if (last) {
    __threadfence();
    float s = 0.f;
    for (unsigned k = threadIdx.x; k < gridDim.x; k += 256)
      s += __hip_atomic_load(&part[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int o = 32; o; o >>= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, s);
  }
}

// the same launch with no ticket (each block writes its partial): the floor
__global__ __launch_bounds__(256) void k_none(float* part) {
  if (threadIdx.x == 0) part[blockIdx.x] = (float)blockIdx.x;
}

template <typename F>
static float time_it(F f, hipStream_t s, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  for (int i = 0; i < 20; ++i) f();
  hipEventRecord(a, s);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(b, s);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  hipEventDestroy(a); hipEventDestroy(b);
  return ms * 1000.f / reps;
}

int main() {
  float *part, *out;
  unsigned* tk;
  CK(hipMalloc(&part, 4096 * 4));
  CK(hipMalloc(&out, 4));
  CK(hipMalloc(&tk, 1 << 16));
  CK(hipMemset(tk, 0, 1 << 16));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const int reps = 400;
  const int nbs[] = {64, 128, 256, 512, 1024, 2048};
  for (int nb : nbs) {
    float t0 = time_it([&] { hipLaunchKernelGGL(k_none, dim3(nb), dim3(256), 0, s, part); }, s, reps);
    float t1 = time_it([&] { hipLaunchKernelGGL((k_tick<1, 1>), dim3(nb), dim3(256), 0, s, part, tk, out); }, s, reps);
    float t2 = time_it([&] { hipLaunchKernelGGL((k_tick<16, 1>), dim3(nb), dim3(256), 0, s, part, tk, out); }, s, reps);
    float t3 = time_it([&] { hipLaunchKernelGGL((k_tick<16, 32>), dim3(nb), dim3(256), 0, s, part, tk, out); }, s, reps);
    float t4 = time_it([&] { hipLaunchKernelGGL((k_tick<32, 32>), dim3(nb), dim3(256), 0, s, part, tk, out); }, s, reps);
    float t5 = time_it([&] { hipLaunchKernelGGL((k_tick<64, 32>), dim3(nb), dim3(256), 0, s, part, tk, out); }, s, reps);
    printf("{\"blocks\": %d, \"none_us\": %.2f, \"one_ticket_us\": %.2f, \"g16_adjacent_us\": %.2f, "
           "\"g16_128B_us\": %.2f, \"g32_128B_us\": %.2f, \"g64_128B_us\": %.2f}\n",
           nb, t0, t1, t2, t3, t4, t5);
  }
  // correctness: the last block's sum over partials 0..nb-1 per launch
  CK(hipMemset(out, 0, 4));
  hipLaunchKernelGGL((k_tick<16, 32>), dim3(1000), dim3(256), 0, s, part, tk, out);
  float h = 0.f;
  CK(hipMemcpy(&h, out, 4, hipMemcpyDeviceToHost));
  unsigned th[1 + 16 * 33];
  CK(hipMemcpy(th, tk, sizeof(th), hipMemcpyDeviceToHost));
  unsigned nz = 0;
  for (unsigned x : th) nz += x != 0u;
  printf("{\"check_sum\": %.1f, \"expect\": %.1f, \"nonzero_tickets_after\": %u}\n", h, 999.0 * 1000 / 2, nz);
  return 0;
}
