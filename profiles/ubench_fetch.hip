// Round 6: what FETCH_SIZE reports for k_step's read patterns on gfx950 (calibration of the PMC
// traffic figures in profiles/pmc_k_step.json).
//
// MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE reports half the bytes of a WIDE COALESCED
// streaming read (16 B per lane), which summarize.py corrects by doubling FETCH for k_step — but
// k_step's reads are gathers (5 coalesced u32 state arrays, a 4-B cell word per moving instance,
// 15 consecutive 8-B strip rows per instance), for which the halving was never measured. Each
// kernel below reads a known set of bytes in one of those shapes from a 1 GiB buffer (every
// instance / thread on lines no other one touches), launched REPS times; rocprofv3 --pmc
// FETCH_SIZE (and TCC_EA0_RDREQ / TCC_EA0_RDREQ_32B in a second pass) per launch, divided by the
// bytes the pattern touches at 32-, 64- and 128-B granularity (printed here), says which model the
// counter follows for that shape.
//   k_stream  float4 per lane, fully coalesced (the guide's calibration case)
//   k_word    one u32 per lane at a distinct 128-B line (the cell-word gather)
//   k_coal    u32 per lane, 16 consecutive lanes on 64 consecutive bytes (the state loads at 16
//             instances per wave)
//   k_rows    15 lanes of a 16-lane group on 15 consecutive 8-B rows at a random 8-B offset
//             (the window-row gather)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      return 1;                                                               \
    }                                                                         \
  } while (0)

constexpr size_t BUF = 1ull << 30;       // bytes
constexpr uint32_t NLINES = BUF / 128;   // 128-B lines (2^23)
constexpr int REPS = 20;

__host__ __device__ inline uint32_t perm(uint32_t i, uint32_t n) {  // bijective on [0, n), n = 2^k
  return (i * 2654435761u) & (n - 1u);
}

__global__ void k_stream(const float4* __restrict__ p, size_t n, float* out) {
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = p[i];
    a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
  }
  if (a.x == 1234.5f) out[0] = a.y + a.z + a.w;
}

// thread t reads word 0 of line perm(t)
__global__ void k_word(const uint32_t* __restrict__ p, int n, uint32_t* out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const uint32_t v = p[(size_t)perm((uint32_t)t, NLINES) * 32];
  if (v == 0xDEADBEEFu) out[0] = v;
}

// group g of 16 lanes reads the 64 B at the start of line perm(g)
__global__ void k_coal(const uint32_t* __restrict__ p, int ngroups, uint32_t* out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x, g = t >> 4, l = t & 15;
  if (g >= ngroups) return;
  const uint32_t v = p[(size_t)perm((uint32_t)g, NLINES) * 32 + l];
  if (v == 0xDEADBEEFu) out[0] = v;
}

// instance j: rows o .. o + 14 (8 B each) from byte 512 * perm(j) + 8 * (j % 49) — a 512-B slot
// per instance, a start offset that walks through every 8-B position of a 128-B line
__device__ __host__ inline size_t rows_start(uint32_t j) {
  return (size_t)perm(j, NLINES / 4) * 512 + 8 * (j % 49);
}
__global__ void k_rows(const uint8_t* __restrict__ p, int ninst, uint32_t* out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x, j = t >> 4, i = t & 15;
  if (j >= ninst || i >= 15) return;
  const uint2 v = *reinterpret_cast<const uint2*>(p + rows_start((uint32_t)j) + 8 * i);
  if (v.x == 0xDEADBEEFu) out[0] = v.y;
}

static double touched(size_t start, size_t len, size_t gran) {
  return (double)(((start + len - 1) / gran - start / gran + 1) * gran);
}

int main() {
  uint8_t* buf;
  uint32_t* out;
  CHECK(hipMalloc(&buf, BUF));
  CHECK(hipMalloc(&out, 64));
  CHECK(hipMemset(buf, 1, BUF));
  CHECK(hipDeviceSynchronize());
  const size_t stream_bytes = 256ull << 20;
  const int nword = 1 << 20, ncoal = 1 << 20, nrows = 1 << 20;
  printf("{\"kernel\": \"k_stream\", \"bytes\": %zu}\n", stream_bytes);
  printf("{\"kernel\": \"k_word\", \"bytes\": %d, \"b32\": %d, \"b64\": %d, \"b128\": %d}\n", 4 * nword,
         32 * nword, 64 * nword, 128 * nword);
  printf("{\"kernel\": \"k_coal\", \"bytes\": %d, \"b32\": %d, \"b64\": %d, \"b128\": %d}\n", 64 * ncoal,
         64 * ncoal, 64 * ncoal, 128 * ncoal);
  double r32 = 0, r64 = 0, r128 = 0;
  for (uint32_t j = 0; j < (uint32_t)nrows; ++j) {
    const size_t s = rows_start(j);
    r32 += touched(s, 120, 32);
    r64 += touched(s, 120, 64);
    r128 += touched(s, 120, 128);
  }
  printf("{\"kernel\": \"k_rows\", \"bytes\": %d, \"b32\": %.0f, \"b64\": %.0f, \"b128\": %.0f}\n",
         120 * nrows, r32, r64, r128);
  // each launch between two L2-evicting fills (a 768 MB memset of the buffer's tail): every
  // kernel's lines come from past the L2
  auto evict = [&](int r) {
    CHECK(hipMemset(buf + (256ull << 20), r & 0x7F, 768ull << 20));
    CHECK(hipDeviceSynchronize());
    return 0;
  };
  for (int r = 0; r < REPS; ++r) {
    hipLaunchKernelGGL(k_stream, dim3(2048), dim3(256), 0, 0, reinterpret_cast<const float4*>(buf),
                       stream_bytes / 16, reinterpret_cast<float*>(out));
    CHECK(hipGetLastError());
    if (evict(r)) return 1;
    hipLaunchKernelGGL(k_word, dim3(nword / 256), dim3(256), 0, 0, reinterpret_cast<const uint32_t*>(buf),
                       nword, out);
    CHECK(hipGetLastError());
    if (evict(r)) return 1;
    hipLaunchKernelGGL(k_coal, dim3(ncoal * 16 / 256), dim3(256), 0, 0,
                       reinterpret_cast<const uint32_t*>(buf), ncoal, out);
    CHECK(hipGetLastError());
    if (evict(r)) return 1;
    hipLaunchKernelGGL(k_rows, dim3(nrows * 16 / 256), dim3(256), 0, 0, buf, nrows, out);
    CHECK(hipGetLastError());
    if (evict(r)) return 1;
  }
  CHECK(hipFree(buf));
  CHECK(hipFree(out));
  return 0;
}
