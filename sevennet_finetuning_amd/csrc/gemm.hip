// Grouped f32 GEMM on gfx950 matrix cores (v_mfma_f32_32x32x2_f32).
//
// Serves every dense contraction of the SevenNet-0 path that is not fused into
// the tensor-product kernels:
//   * e3nn o3.Linear blocks of IrrepsLinear / SelfConnectionLinearIntro
//     (sevenn/nn/linear.py:46-49, self_connection.py:60-62) -- one problem per
//     irrep block l, rows = (atom, m) pairs, K = mul_in, N = mul_out;
//   * the radial MLP of IrrepsConvolution (convolution.py:97-106; e3nn
//     FullyConnectedNet) -- rows = edges, with the SiLU*1.6792 epilogue;
//   * the transposed products of the force backward (act' epilogue).
// f32 in / f32 accumulate: exact f32 (k-ordered fma chain), 157 TF/s peak.
//
// Tile 64x64x16, 256 threads = 4 waves, each wave one 32x32 accumulator.
// Operands are staged through LDS k-major so that the MFMA operand reads
// (lane l: A[row l&31][k l>>5], B[k l>>5][col l&31]) are unit-stride.
#include "common.h"

namespace e3gnn {

namespace {
constexpr int BM = 64, BN = 64, BK = 16, PAD = 1;
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int find_prob(const GemmBatch& b, int tile) {
  int p = 0;
#pragma unroll 1
  for (int i = 1; i < b.nprob; ++i)
    if (tile >= b.p[i].tile_begin) p = i;
  return p;
}

// RC: the row group size R as a compile-time constant (1, 3, 5: the irrep
// blocks' 2l+1; row / R and row % R are then multiplies), 0 = runtime P.R
template <int RC>
__device__ __forceinline__ void gemm_tile(const GemmProb& P, int local, float (*As)[BM + PAD],
                                          float (*Bs)[BN + PAD]) {
  const int tm = local / P.tiles_n, tn = local % P.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int R = RC ? RC : P.R;

  // staging assignment: A: 4 elements per thread, row = e / BK, k = e % BK
  int a_row[4];
  int64_t a_base[4];
  bool a_ok[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = tid + 256 * i;
    const int r = e / BK;
    a_row[i] = r;
    const int grow = m0 + r;
    a_ok[i] = grow < P.M;
    const int node = grow / R, m = grow - node * R;
    a_base[i] = (int64_t)node * P.lda + P.a_off + m;
  }
  float ra[4], rb[4];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + 256 * i;
      const int k = k0 + (e % BK);
      ra[i] = (a_ok[i] && k < P.K) ? P.A[a_base[i] + (int64_t)k * R] : 0.f;
      const int bk = k0 + e / BN, bc = n0 + (e % BN);
      rb[i] = (bk < P.K && bc < P.N) ? P.B[(int64_t)bk * P.ldb + bc] : 0.f;
    }
  };
  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;

  const int nk = (P.K + BK - 1) / BK;
  load(0);
  for (int kt = 0; kt < nk; ++kt) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + 256 * i;
      As[e % BK][a_row[i]] = ra[i];
      Bs[e / BN][e % BN] = rb[i];
    }
    __syncthreads();
    if (kt + 1 < nk) load((kt + 1) * BK);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      const float a = As[kk + (lane >> 5)][wr * 32 + (lane & 31)];
      const float b = Bs[kk + (lane >> 5)][wc * 32 + (lane & 31)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
  }

  const int col = n0 + wc * 32 + (lane & 31);
  if (col >= P.N) return;
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) {
    const int row = m0 + wr * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
    if (row >= P.M) continue;
    const int node = row / R, m = row - node * R;
    const int64_t off = (int64_t)node * P.ldc + P.c_off + (int64_t)col * R + m;
    float v = acc[reg];
    if (P.act == 1) {
      if (P.pre_out) P.pre_out[off] = v;
      v = act_fwd(v);
    } else if (P.act == 2) {
      v *= act_grad(P.pre_in[off]);
    }
    if (P.beta) v += P.C[off];
    P.C[off] = v;
  }
}

__global__ __launch_bounds__(256) void k_gemm(GemmBatch batch) {
  __shared__ float As[BK][BM + PAD];
  __shared__ float Bs[BK][BN + PAD];
  const int pi = find_prob(batch, blockIdx.x);
  const GemmProb& P = batch.p[pi];
  const int local = blockIdx.x - P.tile_begin;
  switch (P.R) {
    case 1: gemm_tile<1>(P, local, As, Bs); break;
    case 3: gemm_tile<3>(P, local, As, Bs); break;
    case 5: gemm_tile<5>(P, local, As, Bs); break;
    default: gemm_tile<0>(P, local, As, Bs); break;
  }
}
}  // namespace

hipError_t launch_gemm(const GemmBatch& b, hipStream_t s) {
  if (b.total_tiles <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_gemm, dim3(b.total_tiles), dim3(256), 0, s, b);
  return hipGetLastError();
}

}  // namespace e3gnn
