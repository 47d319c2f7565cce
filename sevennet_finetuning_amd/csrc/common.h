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

// v_rcp_f32 (1 ulp) instead of an IEEE division (~10 VALU per call)
__device__ __forceinline__ float sigmoidf_(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ __forceinline__ float act_fwd(float x) { return x * sigmoidf_(x) * SILU_NORM; }
__device__ __forceinline__ float act_grad(float x) {
  const float s = sigmoidf_(x);
  return SILU_NORM * s * (1.0f + x * (1.0f - s));
}

// sum over the four 16-lane rows of a wave (lanes l, l^16, l^32, l^48), every
// lane gets the same bits: (r0 + r2) + (r1 + r3) via v_permlane32_swap /
// v_permlane16_swap (VALU, no LDS round trip).  Inline asm: the builtins'
// second result (the swapped source register) comes back as a copy of the
// first with this compiler (tools/microtests/permlane.hip); the s_nop pads the
// VALU-write -> permlane-read hazard, which hipcc does not insert inside asm.
__device__ __forceinline__ float sum_rows4(float v) {
  float a = v, b = v;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a), "+v"(b));
  float s = a + b, t = s;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 1" : "+v"(s), "+v"(t));
  return s + t;
}

// the same for N values at once (N <= 5): each stage's N swaps back to back
// inside ONE asm statement, one hazard pad before and after the group instead
// of around every swap, and the N reductions' adds free to interleave
template <int N>
__device__ __forceinline__ void permlane_swap_n32(float (&a)[N], float (&b)[N]);
template <int N>
__device__ __forceinline__ void permlane_swap_n16(float (&a)[N], float (&b)[N]);
#define E3GNN_PL_SWAPS(W)                                                                             \
  template <>                                                                                         \
  __device__ __forceinline__ void permlane_swap_n##W<1>(float (&a)[1], float (&b)[1]) {               \
    asm volatile("s_nop 1\n\tv_permlane" #W "_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a[0]), "+v"(b[0]));    \
  }                                                                                                   \
  template <>                                                                                         \
  __device__ __forceinline__ void permlane_swap_n##W<2>(float (&a)[2], float (&b)[2]) {               \
    asm volatile("s_nop 1\n\tv_permlane" #W "_swap_b32 %0, %1\n\tv_permlane" #W "_swap_b32 %2, %3\n\ts_nop 1" \
                 : "+v"(a[0]), "+v"(b[0]), "+v"(a[1]), "+v"(b[1]));                                   \
  }                                                                                                   \
  template <>                                                                                         \
  __device__ __forceinline__ void permlane_swap_n##W<3>(float (&a)[3], float (&b)[3]) {               \
    asm volatile("s_nop 1\n\tv_permlane" #W "_swap_b32 %0, %1\n\tv_permlane" #W "_swap_b32 %2, %3"     \
                 "\n\tv_permlane" #W "_swap_b32 %4, %5\n\ts_nop 1"                                      \
                 : "+v"(a[0]), "+v"(b[0]), "+v"(a[1]), "+v"(b[1]), "+v"(a[2]), "+v"(b[2]));           \
  }                                                                                                   \
  template <>                                                                                         \
  __device__ __forceinline__ void permlane_swap_n##W<4>(float (&a)[4], float (&b)[4]) {               \
    asm volatile("s_nop 1\n\tv_permlane" #W "_swap_b32 %0, %1\n\tv_permlane" #W "_swap_b32 %2, %3"     \
                 "\n\tv_permlane" #W "_swap_b32 %4, %5\n\tv_permlane" #W "_swap_b32 %6, %7\n\ts_nop 1"  \
                 : "+v"(a[0]), "+v"(b[0]), "+v"(a[1]), "+v"(b[1]), "+v"(a[2]), "+v"(b[2]), "+v"(a[3]), \
                   "+v"(b[3]));                                                                       \
  }                                                                                                   \
  template <>                                                                                         \
  __device__ __forceinline__ void permlane_swap_n##W<5>(float (&a)[5], float (&b)[5]) {               \
    asm volatile("s_nop 1\n\tv_permlane" #W "_swap_b32 %0, %1\n\tv_permlane" #W "_swap_b32 %2, %3"     \
                 "\n\tv_permlane" #W "_swap_b32 %4, %5\n\tv_permlane" #W "_swap_b32 %6, %7"              \
                 "\n\tv_permlane" #W "_swap_b32 %8, %9\n\ts_nop 1"                                      \
                 : "+v"(a[0]), "+v"(b[0]), "+v"(a[1]), "+v"(b[1]), "+v"(a[2]), "+v"(b[2]), "+v"(a[3]), \
                   "+v"(b[3]), "+v"(a[4]), "+v"(b[4]));                                               \
  }
E3GNN_PL_SWAPS(32)
E3GNN_PL_SWAPS(16)
#undef E3GNN_PL_SWAPS
template <int N>
__device__ __forceinline__ void sum_rows4_n(float (&v)[N]) {
  static_assert(N >= 1 && N <= 5, "up to five values per group");
  float a[N], b[N];
#pragma unroll
  for (int i = 0; i < N; ++i) a[i] = b[i] = v[i];
  permlane_swap_n32<N>(a, b);
#pragma unroll
  for (int i = 0; i < N; ++i) a[i] = b[i] = a[i] + b[i];
  permlane_swap_n16<N>(a, b);
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = a[i] + b[i];
}

// XCD-aware block order: workgroups are dealt round-robin over the 8 XCDs
// (b and b + 8 share one, MI355X_MICROARCH.md "Workgroup dispatch"), so
// consecutive blocks land on different L2s.  This bijection gives each XCD a
// contiguous 1/8 of the index range instead, so the rows its blocks gather
// (spatial neighbours of consecutive centres / edges) are shared in its L2.
// Placement only: any dispatch order gives the same results.
#ifndef E3GNN_XCD_REMAP
#define E3GNN_XCD_REMAP 0
#endif
__device__ __forceinline__ int xcd_block() {
  const int b = blockIdx.x;
  if (!E3GNN_XCD_REMAP) return b;
  const int nb = gridDim.x, q = nb >> 3, r = nb & 7, x = b & 7;
  return x * q + (x < r ? x : r) + (b >> 3);
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

// ---------------------------------------------------------------- node linears
// One irrep block of an e3nn linear (or of two linears into the same output
// block, K-concatenated: self_interaction_2 + self_connection forward,
// self_interaction_1^T + self_connection^T backward), node-aligned tiles
// (gemm.hip k_nodelin):
//   A(node, m, k) = k < K1 ? A [node * lda  + a_off  + k * R + m]
//                          : A2[node * lda2 + a_off2 + (k - K1) * R + m]
//   B(k, col)     = B[k * N + col]          (rows 0..K1-1 then K1..K-1)
//   C(node, m, col) = C[node * ldc + c_off + col * R + m]
// epi: 0 store, 1 accumulate, 2 store + xo[node, col] = act(v) for
// col < n_act (gate scalars / last block), 3 store + xo[node, xo_off + col * R
// + m] = act(C[node, gate_off + col]) * v (gated irreps; the gate columns were
// stored by an earlier launch).
struct NlProb {
  const float* A;
  const float* A2;
  const float* B;
  const void* Bb;  // B as bf16 pieces (LinPair::Wb order): k_nodelin_b; null: k_nodelin

  float* C;
  float* xo;
  int64_t lda, lda2, ldc, ldxo;
  int a_off, a_off2, c_off, xo_off;
  int K1, K, N, R, nodes;
  int epi, n_act, gate_off;
  int wn, ns, tpn, tile_begin, tiles_n;  // set by add_nl
  int kind;  // set by add_nl: 0 k_nodelin (f32), 1 k_nodelin_b, 2 k_nodelin_s (bf16x6)
};
constexpr int NL_MAX_PROBS = 4;
struct NlBatch {
  NlProb p[NL_MAX_PROBS];
  int nprob;
  int total_tiles;
};
// false when the problem does not meet the kernel's layout assumptions
// (16-byte alignment of rows / offsets, K1 % 32 when split, R in {1, 3, 5})
bool add_nl(NlBatch& b, const NlProb& p);
hipError_t launch_nodelin(const NlBatch& b, hipStream_t s);

}  // namespace e3gnn
