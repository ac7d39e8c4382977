// mz_gemm.h — split-precision (bf16x3) f32 GEMM of the learners (mz_gemm.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MZ_GEMM_NONE 0
#define MZ_GEMM_LEAKY 1  // LeakyReLU(0.01)
#define MZ_GEMM_RELU 2

// C[m][n] = act(sum_k A(m,k) B(n,k) + bias[n]); A(m,k) = a[m*a_rs + k*a_ks] (a_rs or a_ks == 1)
struct MzGemm {
  const float* a; long a_rs, a_ks;
  const float* b; long b_rs, b_ks;
  float* c; long ldc;
  const float* bias;
  float* ws_img;         // workspace (mz_gemm_ws_floats): operand images, split-K partial sums
  float* ws;             // (set by the launcher) split-K partials [splits][M][N]
  int M, N, K, act;
};
int mz_gemm_splits(int m, int n, int k);
size_t mz_gemm_ws_floats(int m, int n, int k);
hipError_t mz_launch_gemm_x3(const MzGemm& g, hipStream_t s);
