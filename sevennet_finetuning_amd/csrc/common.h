// Shared definitions for the e3gnn MI355X (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <string>

namespace e3gnn {

// ---------------------------------------------------------------- activations
// e3nn normalize2mom(silu): silu(x) * SILU_NORM (sevenn/_const.py:34-48 act
// table; the constant is frozen in serial_code.py as c5).
constexpr float SILU_NORM = 1.6791767923989418f;

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }
__device__ __forceinline__ float act_fwd(float x) { return x * sigmoidf_(x) * SILU_NORM; }
__device__ __forceinline__ float act_grad(float x) {
  const float s = sigmoidf_(x);
  return SILU_NORM * s * (1.0f + x * (1.0f - s));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---------------------------------------------------------------- GEMM
// One sub-problem of a grouped f32 MFMA GEMM (gemm.hip).  Rows are (node, m)
// pairs so one problem covers a whole irrep block of an e3nn linear:
//   A(row, k)   = A[(row / R) * lda + a_off + k * R + row % R]
//   B(k, col)   = B[k * ldb + col]
//   C(row, col) = C[(row / R) * ldc + c_off + col * R + row % R]
// act: 0 none; 1 C = silu_n(acc), pre_out = acc; 2 C = acc * silu_n'(pre_in).
struct GemmProb {
  const float* A;
  const float* B;
  float* C;
  const float* pre_in;
  float* pre_out;
  int64_t lda, ldc;
  int M, N, K, R;
  int a_off, c_off, ldb;
  int beta, act;
  int tile_begin, tiles_n;
};
constexpr int GEMM_MAX_PROBS = 8;
struct GemmBatch {
  GemmProb p[GEMM_MAX_PROBS];
  int nprob;
  int total_tiles;
};
hipError_t launch_gemm(const GemmBatch& b, hipStream_t s);

}  // namespace e3gnn
