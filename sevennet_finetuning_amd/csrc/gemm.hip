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

#include <cstdlib>
#include <cstring>

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
// ---------------------------------------------------------------- node linears
// k_nodelin: the e3nn linears of the interaction block (self_interaction_1/2,
// self_connection; linear.py:46-49) as node-aligned tiles.  A tile covers
// T = BM / R whole nodes, so the A operand of one k-step is T contiguous runs
// of BK * R floats (the node's [mul][m] block) loaded as float4 and scattered
// k-major into LDS; BK = 16 with a double-buffered LDS stage (one barrier per
// k-step).  Two linears writing the same output block run as one problem with
// K = K1 + K2 (A switches source at K1; separate partial sums), and the gate
// (equivariant_gate.py:59-61) is the epilogue: the 0e block writes
// act(scalars) to the next features, the l > 0 blocks multiply by act(gate)
// read back from the pre-activation columns the 0e launch stored.
// Shapes (4 waves): WN waves across N, each NS x 32 columns; BM = 128 / WN.
//   WN = 2, NS = 1: 64 x 64 (default); WN = 1: 128 x 32 (N <= 32, the 2e
//   block); WN = 2, NS = 2: 64 x 128 (unsplit K with N >= 128: si1 / si2^T
//   blocks; half the tiles, A staged once per 128 columns).
#ifndef E3GNN_NL_BK
#define E3GNN_NL_BK 16
#endif
// occupancy target of k_nodelin (LDS allows 6 workgroups per CU)
#ifndef E3GNN_NL_WAVES
#define E3GNN_NL_WAVES 5
#endif
#ifndef E3GNN_NL_WIDE
#define E3GNN_NL_WIDE 1
#endif
#ifndef E3GNN_NL_WIDE_KMAX
#define E3GNN_NL_WIDE_KMAX 4096
#endif
constexpr int NL_BK = E3GNN_NL_BK;
template <int WN, int NS>
struct NlShape {
  static constexpr int BN = 32 * WN * NS, BM = 128 / WN;
  static constexpr int LDA = BM + 4, LDB = BN + 4;  // 16-byte LDS rows
  static constexpr int A_FLOATS = NL_BK * LDA, STAGE = A_FLOATS + NL_BK * LDB;
};
constexpr int cmax(int a, int b) { return a > b ? a : b; }
constexpr int NL_LDS =
    2 * cmax(NlShape<1, 1>::STAGE, cmax(NlShape<2, 1>::STAGE, NlShape<2, 2>::STAGE));

// Epilogue through LDS, one 64- (or 32-) column chunk at a time: each node's
// output is one contiguous run of CW * R floats, written as float4 (the MFMA
// layout would scatter 4-byte stores R floats apart).  Starts with a barrier:
// the caller's LDS readers are done.
template <int WN, int R>
__device__ __forceinline__ void nl_epilogue(const NlProb& P, const f32x16& acc, int node0, int n0,
                                            float* lds) {
  constexpr int BM = 128 / WN, CW = 32 * WN;
  constexpr int T = BM / R, ROWS = T * R;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave / WN, wc = wave % WN;
  __syncthreads();
  constexpr int LDC = CW + 1;
  static_assert(ROWS * LDC <= NL_LDS, "C tile must fit the LDS stages");
  float* Cs = lds;
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) {
    const int row = wr * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
    if (row < ROWS) Cs[row * LDC + wc * 32 + (lane & 31)] = acc[reg];
  }
  __syncthreads();
  constexpr int SEGC = CW * R / 4, UC = T * SEGC;
  const int ncol = P.N - n0 < CW ? P.N - n0 : CW;
  if (ncol <= 0) return;
#pragma unroll 1
  for (int u = tid; u < UC; u += 256) {
    const int nl = u / SEGC, j = 4 * (u - nl * SEGC);
    const int node = node0 + nl;
    if (node >= P.nodes) continue;
    float v[4];
    int cl[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      cl[q] = (j + q) / R;
      const int m = (j + q) - cl[q] * R;
      v[q] = cl[q] < ncol ? Cs[(nl * R + m) * LDC + cl[q]] : 0.f;
    }
    if (cl[0] >= ncol) continue;
    const bool full = cl[3] < ncol;
    const int64_t nrow = (int64_t)node * P.ldc;
    float* cp = P.C + nrow + P.c_off + n0 * R + j;
    if (P.epi == 1) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (cl[q] < ncol) v[q] += cp[q];
    }
    if (full) {
      *reinterpret_cast<float4*>(cp) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (cl[q] < ncol) cp[q] = v[q];
    }
    if (P.epi == 2) {  // R == 1: element q is column n0 + j + q
      float* xp = P.xo + (int64_t)node * P.ldxo + P.xo_off + n0 + j;
      if (full && n0 + j + 3 < P.n_act) {
        *reinterpret_cast<float4*>(xp) =
            make_float4(act_fwd(v[0]), act_fwd(v[1]), act_fwd(v[2]), act_fwd(v[3]));
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (cl[q] < ncol && n0 + j + q < P.n_act) xp[q] = act_fwd(v[q]);
      }
    } else if (P.epi == 3) {
      const float* gp = P.C + nrow + P.gate_off + n0;
      float w[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) w[q] = cl[q] < ncol ? act_fwd(gp[cl[q]]) * v[q] : 0.f;
      float* xp = P.xo + (int64_t)node * P.ldxo + P.xo_off + n0 * R + j;
      if (full) {
        *reinterpret_cast<float4*>(xp) = make_float4(w[0], w[1], w[2], w[3]);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (cl[q] < ncol) xp[q] = w[q];
      }
    }
  }
}

// Epilogue for plain / accumulating outputs (epi 0 / 1): the accumulators
// are written to LDS in the OUTPUT's memory order (node, column * R + m), so
// the copy-out is one b128 LDS read + one b128 store per 4 floats with no
// per-element index arithmetic (the generic epilogue above spent ~0.5 VALU
// instructions per output float on it: the si2^T launches are 1.2 GB of
// output).  Starts with a barrier: the caller's LDS readers are done.
#ifndef E3GNN_NL_RUNS
#define E3GNN_NL_RUNS 1
#endif
// stage(lds, LDR) writes the accumulators as lds[nl * LDR + c * R + m] (the
// tile's node nl, column c of the chunk, component m): the f32 (32x32) and
// bf16x6 (16x16) accumulator layouts share the copy-out.
template <int BM, int CW, int R, int LDSF, class Stage>
__device__ __forceinline__ void nl_epi_runs(const NlProb& P, int node0, int n0, float* lds, Stage stage) {
  constexpr int T = BM / R;
  constexpr int RUN = CW * R, LDR = RUN + 4;  // 16-byte aligned node runs
  static_assert(T * LDR <= LDSF, "C runs must fit the LDS stages");
  const int tid = threadIdx.x;
  __syncthreads();
  stage(lds, LDR);
  __syncthreads();
  const int ncol = P.N - n0 < CW ? P.N - n0 : CW;  // a multiple of 4 (add_nl)
  if (ncol <= 0) return;
  const int len = ncol * R;
  constexpr int SEGC = RUN / 4, UC = T * SEGC;
#pragma unroll 1
  for (int u = tid; u < UC; u += 256) {
    const int nl = u / SEGC, j = 4 * (u - nl * SEGC);
    const int node = node0 + nl;
    if (j >= len || node >= P.nodes) continue;
    float4 v = *reinterpret_cast<const float4*>(lds + nl * LDR + j);
    float4* cp = reinterpret_cast<float4*>(P.C + (int64_t)node * P.ldc + P.c_off + n0 * R + j);
    if (P.epi == 1) {
      const float4 o = *cp;
      v.x += o.x;
      v.y += o.y;
      v.z += o.z;
      v.w += o.w;
    }
    *cp = v;
  }
}
// the f32 kernel's 32 x 32 accumulator (wave (wr, wc) of WN columns) into runs
template <int WN, int R>
__device__ __forceinline__ void nl_stage32(const f32x16& acc, float* L, int LDR) {
  constexpr int BM = 128 / WN, ROWS = (BM / R) * R;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave / WN, wc = wave % WN;
  const int cR = (wc * 32 + (lane & 31)) * R;
  const int rbase = wr * 32 + 4 * (lane >> 5);
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) {
    const int row = rbase + (reg & 3) + 8 * (reg >> 2);
    const int nl = row / R, m = row - nl * R;
    if (row < ROWS) L[nl * LDR + cR + m] = acc[reg];
  }
}
template <int WN, int R>
__device__ __forceinline__ void nl_epilogue_runs(const NlProb& P, const f32x16& acc, int node0,
                                                 int n0, float* lds) {
  nl_epi_runs<128 / WN, 32 * WN, R, NL_LDS>(P, node0, n0, lds,
                                             [&](float* L, int LDR) { nl_stage32<WN, R>(acc, L, LDR); });
}

// The gate epilogues (epi 2 / 3) in the same run form.  epi 2 (the 0e block,
// R = 1): C = the pre-activations, xo = act(scalars) for columns < n_act.
// epi 3 (l > 0): C = the pre-gate values, xo = act(gate) * value; the tile's
// T x CW gate pre-activations (written to C by the 0e launch) are loaded
// once per tile, activated once per (node, column) instead of once
// per output element, and read back from LDS by the copy-out (the generic
// epilogue above issued four dependent scalar global loads and four
// activations per float4).  Gate problems split K (si2 + self-connection), so
// only the single-block (NS = 1) tiles instantiate it.
#ifndef E3GNN_NL_GATE_RUNS
#define E3GNN_NL_GATE_RUNS 1
#endif
template <int BM, int CW, int R, int LDSF, class Stage>
__device__ __forceinline__ void nl_epi_gate(const NlProb& P, int node0, int n0, float* lds, Stage stage) {
  constexpr int T = BM / R;
  constexpr int RUN = CW * R, LDR = RUN + 4;
  constexpr int GS = R > 1 ? T * CW : 0, NG = (GS + 255) / 256;
  static_assert(T * LDR + GS <= LDSF, "C runs and gate factors must fit the LDS stages");
  const int tid = threadIdx.x;
  const int ncol = P.N - n0 < CW ? P.N - n0 : CW;  // a multiple of 4 (add_nl)
  const int vn = min(T, P.nodes - node0);
  __syncthreads();
  stage(lds, LDR);
  float* gl = lds + T * LDR;
  if constexpr (GS > 0) {
    float gv[NG];
#pragma unroll
    for (int i = 0; i < NG; ++i) {
      const int u = tid + 256 * i;
      const int nl = u / CW, c = u - nl * CW;
      gv[i] = (u < GS && nl < vn && c < ncol)
                  ? P.C[(int64_t)(node0 + nl) * P.ldc + P.gate_off + n0 + c]
                  : 0.f;
    }
#pragma unroll
    for (int i = 0; i < NG; ++i) {
      const int u = tid + 256 * i;
      if (u < GS) gl[u] = act_fwd(gv[i]);
    }
  }
  __syncthreads();
  if (ncol <= 0) return;
  const int len = ncol * R;
  constexpr int SEGC = RUN / 4, UC = T * SEGC;
#pragma unroll 1
  for (int u = tid; u < UC; u += 256) {
    const int nl = u / SEGC, j = 4 * (u - nl * SEGC);
    const int node = node0 + nl;
    if (j >= len || node >= P.nodes) continue;
    const float4 v = *reinterpret_cast<const float4*>(lds + nl * LDR + j);
    *reinterpret_cast<float4*>(P.C + (int64_t)node * P.ldc + P.c_off + n0 * R + j) = v;
    float* xp = P.xo + (int64_t)node * P.ldxo + P.xo_off + n0 * R + j;
    if constexpr (R == 1) {  // epi 2: element q is column n0 + j + q
      if (n0 + j + 3 < P.n_act) {
        *reinterpret_cast<float4*>(xp) = make_float4(act_fwd(v.x), act_fwd(v.y), act_fwd(v.z), act_fwd(v.w));
      } else {
        const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (n0 + j + q < P.n_act) xp[q] = act_fwd(e[q]);
      }
    } else {  // epi 3: element q is column (j + q) / R of the tile
      const float* gn = gl + nl * CW;
      *reinterpret_cast<float4*>(xp) = make_float4(gn[(j + 0) / R] * v.x, gn[(j + 1) / R] * v.y,
                                                   gn[(j + 2) / R] * v.z, gn[(j + 3) / R] * v.w);
    }
  }
}
template <int WN, int R>
__device__ __forceinline__ void nl_epilogue_gate(const NlProb& P, const f32x16& acc, int node0,
                                                 int n0, float* lds) {
  nl_epi_gate<128 / WN, 32 * WN, R, NL_LDS>(P, node0, n0, lds,
                                             [&](float* L, int LDR) { nl_stage32<WN, R>(acc, L, LDR); });
}

// Operand loads through buffer descriptors based at the tile (a 32-bit lane
// offset fixed over the k loop, the k-step's advance a scalar offset: no
// 64-bit addresses to keep live).  Optionally (E3GNN_NL_DEPTH2, 64 x 64 tiles
// only: the wider tiles' second slot does not fit five waves per SIMD) two
// register slots keep the loads of k-step kt + 2 in flight while step kt
// computes.  Rows past the problem's nodes read 0 (outside the descriptor).
// (a second register slot for the 64 x 64 tiles measured 0.17 ms per step
// SLOWER: 5.36 vs 5.19 ms of node linears, same box; kept as an option)
#ifndef E3GNN_NL_DEPTH2
#define E3GNN_NL_DEPTH2 0
#endif
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t nl_rsrc(const float* p, int64_t nbytes) {
  const int n = nbytes <= 0 ? 0 : (nbytes > 0x7fffffff ? 0x7fffffff : (int)nbytes);
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, n, 0x00020000);
}
__device__ __forceinline__ float4 nl_ld4(__amdgpu_buffer_rsrc_t r, int vbytes, int sbytes) {
  const f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, vbytes, sbytes, 0));
  return make_float4(v[0], v[1], v[2], v[3]);
}

template <int WN, int NS, int R>
__device__ __forceinline__ void nl_tile(const NlProb& P, int local, float* lds) {
  using S = NlShape<WN, NS>;
  constexpr int BM = S::BM, BN = S::BN, BK = NL_BK;
  constexpr int T = BM / R;
  constexpr int SEG4 = BK * R / 4;  // float4 per node per k-step
  constexpr int UA = T * SEG4, NA = (UA + 255) / 256;
  constexpr int UB = BK * BN / 4, NB = (UB + 255) / 256;
  static_assert(BK % 4 == 0, "tile shape");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave / WN, wc = wave % WN;
  const int tm = local / P.tiles_n, tn = local - tm * P.tiles_n;
  const int node0 = tm * T, n0 = tn * BN;
  const int vn = min(T, P.nodes - node0);  // nodes of this tile

  // descriptors: the tile's rows of A (and A2), B from column n0 on
  const __amdgpu_buffer_rsrc_t RA =
      nl_rsrc(P.A + (int64_t)node0 * P.lda + P.a_off, ((int64_t)(vn - 1) * P.lda + P.K1 * R) * 4);
  const __amdgpu_buffer_rsrc_t RA2 =
      P.K > P.K1 ? nl_rsrc(P.A2 + (int64_t)node0 * P.lda2 + P.a_off2,
                           ((int64_t)(vn - 1) * P.lda2 + (P.K - P.K1) * R) * 4)
                 : RA;
  const __amdgpu_buffer_rsrc_t RB = nl_rsrc(P.B + n0, ((int64_t)P.K * P.N - n0) * 4);
  int a_v[NA], a_v2[NA], b_v[NB];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int u = tid + 256 * i;
    const int nl = u / SEG4, j = 4 * (u - nl * SEG4);
    const bool ok = (UA % 256 == 0 || u < UA) && nl < vn;
    a_v[i] = ok ? (nl * (int)P.lda + j) * 4 : 0x7ffffff0;   // out of range: reads 0
    a_v2[i] = ok ? (nl * (int)P.lda2 + j) * 4 : 0x7ffffff0;
  }
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int u = tid + 256 * i;
    const int k = u / (BN / 4), c = 4 * (u - k * (BN / 4));
    b_v[i] = (UB % 256 == 0 || u < UB) ? (k * P.N + c) * 4 : 0x7ffffff0;
  }
  // two register slots where the registers allow it (64 x 64 tiles: one
  // float4 of A and one of B per thread and slot); one otherwise
  constexpr int DEPTH = (E3GNN_NL_DEPTH2 && WN == 2 && NS == 1) ? 2 : 1;
  float4 ra[DEPTH][NA], rb[DEPTH][NB];
  auto load = [&](int k0, float4(&xa)[NA], float4(&xb)[NB]) __attribute__((always_inline)) {
    const bool second = k0 >= P.K1;
    const int kk0 = second ? k0 - P.K1 : k0;
    const int kend = second ? P.K - P.K1 : P.K1;
    // a K tail (not met by SevenNet-0's linears) masks the elements past
    // kend: inside the row they are the next block's values, past the last
    // row the descriptor returns 0
    const bool tail = kk0 + BK > kend;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      float4 v = second ? nl_ld4(RA2, a_v2[i], kk0 * R * 4) : nl_ld4(RA, a_v[i], kk0 * R * 4);
      if (tail) {
        const int u = tid + 256 * i;
        const int j = 4 * (u - (u / SEG4) * SEG4);
        v.x = kk0 + (j + 0) / R < kend ? v.x : 0.f;
        v.y = kk0 + (j + 1) / R < kend ? v.y : 0.f;
        v.z = kk0 + (j + 2) / R < kend ? v.z : 0.f;
        v.w = kk0 + (j + 3) / R < kend ? v.w : 0.f;
      }
      xa[i] = v;
    }
    // B rows >= K and columns past N's row end read 0 or columns that only
    // feed discarded outputs
#pragma unroll
    for (int i = 0; i < NB; ++i) xb[i] = nl_ld4(RB, b_v[i], k0 * P.N * 4);
  };
  auto store = [&](int buf, const float4(&xa)[NA], const float4(&xb)[NB]) __attribute__((always_inline)) {
    float* As = lds + buf * S::STAGE;
    float* Bs = As + S::A_FLOATS;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int u = tid + 256 * i;
      if (UA % 256 != 0 && u >= UA) continue;
      const int nl = u / SEG4, j = 4 * (u - nl * SEG4);
      const float e[4] = {xa[i].x, xa[i].y, xa[i].z, xa[i].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int k = (j + q) / R, m = (j + q) - k * R;
        As[k * S::LDA + nl * R + m] = e[q];
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int u = tid + 256 * i;
      if (UB % 256 != 0 && u >= UB) continue;
      const int k = u / (BN / 4), c = 4 * (u - k * (BN / 4));
      *reinterpret_cast<float4*>(Bs + k * S::LDB + c) = xb[i];
    }
  };

  const int nk = (P.K + BK - 1) / BK;
  const int nk1 = (NS == 1 && P.K > P.K1) ? P.K1 / BK : nk;
  // step kt (DEPTH 2): LDS stage kt & 1 holds kt; register slot (kt + 1) & 1
  // holds step kt + 1 and slot kt & 1 step kt + 2 (both in flight).
  // wave (wr, wc), sub-tile s: columns s * 32 * WN + wc * 32 + (0..31), so
  // chunk s of the epilogue is one contiguous 32 * WN column range
  auto compute = [&](int buf, f32x16(&c)[NS]) __attribute__((always_inline)) {
    const float* As = lds + buf * S::STAGE;
    const float* Bs = As + S::A_FLOATS;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      const float a = As[(kk + (lane >> 5)) * S::LDA + wr * 32 + (lane & 31)];
#pragma unroll
      for (int sub = 0; sub < NS; ++sub) {
        const float b = Bs[(kk + (lane >> 5)) * S::LDB + sub * 32 * WN + wc * 32 + (lane & 31)];
        c[sub] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c[sub], 0, 0, 0);
      }
    }
  };
  auto step = [&](int kt, f32x16(&c)[NS]) __attribute__((always_inline)) {
    if constexpr (DEPTH == 2) {
      if (kt & 1) {
        compute(1, c);
        if (kt + 1 < nk) store(0, ra[0], rb[0]);
        if (kt + 3 < nk) load((kt + 3) * BK, ra[0], rb[0]);
      } else {
        compute(0, c);
        if (kt + 1 < nk) store(1, ra[DEPTH - 1], rb[DEPTH - 1]);
        if (kt + 3 < nk) load((kt + 3) * BK, ra[DEPTH - 1], rb[DEPTH - 1]);
      }
    } else {  // one slot: step kt + 1's loads cover step kt's MFMA work
      if (kt + 1 < nk) load((kt + 1) * BK, ra[0], rb[0]);
      compute(kt & 1, c);
      if (kt + 1 < nk) store((kt + 1) & 1, ra[0], rb[0]);
    }
    __syncthreads();
  };
  f32x16 acc[NS];
#pragma unroll
  for (int sub = 0; sub < NS; ++sub)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[sub][i] = 0.f;
  load(0, ra[0], rb[0]);
  store(0, ra[0], rb[0]);
  if constexpr (DEPTH == 2) {
    if (nk > 1) load(BK, ra[DEPTH - 1], rb[DEPTH - 1]);
    if (nk > 2) load(2 * BK, ra[0], rb[0]);
  }
  __syncthreads();
#pragma unroll 1
  for (int kt = 0; kt < nk1; ++kt) step(kt, acc);
  // (wide tiles are only chosen for unsplit K: add_nl)
  if (NS == 1 && nk1 < nk) {
    // the second linear's sum on its own, added once (the rounding of two
    // GEMMs summed, not its terms added one by one to a large partial sum)
    f32x16 acc2[NS];
#pragma unroll
    for (int sub = 0; sub < NS; ++sub)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc2[sub][i] = 0.f;
#pragma unroll 1
    for (int kt = nk1; kt < nk; ++kt) step(kt, acc2);
#pragma unroll
    for (int sub = 0; sub < NS; ++sub)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[sub][i] += acc2[sub][i];
  }
#pragma unroll
  for (int sub = 0; sub < NS; ++sub) {
    if (E3GNN_NL_RUNS && P.epi <= 1)
      nl_epilogue_runs<WN, R>(P, acc[sub], node0, n0 + sub * 32 * WN, lds);
    else if (E3GNN_NL_GATE_RUNS && NS == 1 && P.epi >= 2 && (R > 1) == (P.epi == 3))
      nl_epilogue_gate<WN, R>(P, acc[sub], node0, n0 + sub * 32 * WN, lds);
    else
      nl_epilogue<WN, R>(P, acc[sub], node0, n0 + sub * 32 * WN, lds);
  }
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(E3GNN_NL_WAVES, 8))) void
k_nodelin(NlBatch batch) {
  __shared__ __attribute__((aligned(16))) float lds[NL_LDS];
  const int tile = blockIdx.x;
  int pi = 0;
#pragma unroll 1
  for (int i = 1; i < batch.nprob; ++i)
    if (tile >= batch.p[i].tile_begin) pi = i;
  NlProb P = batch.p[0];
  if (pi == 1) P = batch.p[1];
  if (pi == 2) P = batch.p[2];
  if (pi == 3) P = batch.p[3];
  const int local = tile - P.tile_begin;
  if (P.wn == 1) {
    switch (P.R) {
      case 1: nl_tile<1, 1, 1>(P, local, lds); break;
      case 3: nl_tile<1, 1, 3>(P, local, lds); break;
      default: nl_tile<1, 1, 5>(P, local, lds); break;
    }
  } else if (P.ns == 2) {
    switch (P.R) {
      case 1: nl_tile<2, 2, 1>(P, local, lds); break;
      case 3: nl_tile<2, 2, 3>(P, local, lds); break;
      default: nl_tile<2, 2, 5>(P, local, lds); break;
    }
  } else {
    switch (P.R) {
      case 1: nl_tile<2, 1, 1>(P, local, lds); break;
      case 3: nl_tile<2, 1, 3>(P, local, lds); break;
      default: nl_tile<2, 1, 5>(P, local, lds); break;
    }
  }
}
// ------------------------------------------------- node linears on bf16x6 MFMA
// k_nodelin_b: the same problems as k_nodelin (node-aligned tiles, the run /
// gate epilogues) on v_mfma_f32_16x16x32_bf16 with both operands as three bf16
// pieces (x = p0 + p1 + p2 exactly: 24 significant bits) and the six piece
// products with i + j <= 2 accumulated in f32, smallest first -- f32-grade
// results (dropped terms below 2^-24 relative) at 6 x 16 = 96 MFMA cycles per
// 16 x 16 x 32 block instead of the 256 of the f32 MFMA (the si2^T launches
// were MFMA-bound: 0.31 of their 0.51 ms with loads and epilogue removed).
// The weights are split once at load (LinPair::Wb, already in B-operand lane
// order: one b128 per lane, piece and 16-column block, from L2); the node rows
// are split while staging: thread unit (row = node * R + m, k quad) -> 4
// values, 3 pieces, one ds_write_b64 per piece into k-contiguous bf16 planes
// [piece][row][k] (80-byte rows: the b128 fragment reads are conflict-free).
// Tile 64 rows (T = 64 / R nodes) x BN columns, BK = 32, 4 waves:
//   SH 0: BN 32, waves 4 x 1, each 16 rows x 32 columns (N <= 32)
//   SH 1: BN 64, waves 2 x 2, each 32 x 32
constexpr int NB_BM = 64, NB_BK = 32, NB_ALD = 40;
constexpr int NB_PLANE = NB_BM * NB_ALD;        // bf16 per piece plane
constexpr int NB_STAGE = 3 * NB_PLANE * 2;      // bytes per LDS stage
constexpr int NB_LDSF = 2 * NB_STAGE / 4;       // floats (two stages; the epilogue reuses them)
typedef __bf16 nbf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned nu32x2 __attribute__((ext_vector_type(2)));
typedef float nf32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
typedef __bf16 nbf16x2 __attribute__((ext_vector_type(2)));
template <int SH>
struct NbShape {
  static constexpr int WC = SH == 0 ? 1 : 2, WR = 4 / WC;
  static constexpr int BN = 32 * WC, RB = NB_BM / WR / 16, CB = 2;
};
// four floats as three bf16 pieces, two values per v_cvt_pk_bf16_f32 (the
// packed word is both the operand and, widened, what the residual subtracts)
__device__ __forceinline__ void nb_split4(const float (&v)[4], nu32x2 (&d)[3]) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    nf32x2 r;
    r[0] = v[2 * q];
    r[1] = v[2 * q + 1];
#pragma unroll
    for (int pc = 0; pc < 3; ++pc) {
      const unsigned u = __builtin_bit_cast(unsigned, __builtin_convertvector(r, nbf16x2));
      d[pc][q] = u;
      if (pc < 2) {
        r[0] -= __builtin_bit_cast(float, u << 16);
        r[1] -= __builtin_bit_cast(float, u & 0xffff0000u);
      }
    }
  }
}
__device__ __forceinline__ float nl_ld1(__amdgpu_buffer_rsrc_t r, int vbytes, int sbytes) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vbytes, sbytes, 0));
}

template <int SH, int R>
__device__ __forceinline__ void nl_tile_b(const NlProb& P, int local, float* lds) {
  using S = NbShape<SH>;
  constexpr int BM = NB_BM, BK = NB_BK, BN = S::BN, WC = S::WC, RB = S::RB, CB = S::CB;
  constexpr int T = BM / R, ROWS = T * R;
  constexpr int UNITS = ROWS * (BK / 4), NU = (UNITS + 255) / 256;
  constexpr int OOB = 0x7ffffff0;   // outside every descriptor: reads 0
  // (wave index wave-uniform for the compiler: the B fragment offsets are
  // scalar offsets, not per-lane waterfall loops)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WC, wc = wave % WC;
  const int tm = local / P.tiles_n, tn = local - tm * P.tiles_n;
  const int node0 = tm * T, n0 = tn * BN;
  const int vn = min(T, P.nodes - node0);
  const int K2 = P.K - P.K1;
  const int nkc1 = (P.K1 + BK - 1) / BK, nkc = nkc1 + (K2 + BK - 1) / BK;
  const __amdgpu_buffer_rsrc_t RA =
      nl_rsrc(P.A + (int64_t)node0 * P.lda + P.a_off, ((int64_t)(vn - 1) * P.lda + P.K1 * R) * 4);
  const __amdgpu_buffer_rsrc_t RA2 =
      K2 > 0 ? nl_rsrc(P.A2 + (int64_t)node0 * P.lda2 + P.a_off2, ((int64_t)(vn - 1) * P.lda2 + K2 * R) * 4)
             : RA;
  const int ncb = (P.N + 15) / 16;
  const __amdgpu_buffer_rsrc_t RBb =
      nl_rsrc(static_cast<const float*>(P.Bb), (int64_t)ncb * nkc * 3 * 1024);
  // the thread's staging units: (row, k quad); rows past the tile's nodes and
  // idle units read 0 (OOB offsets)
  int uo[NU], uo2[NU], ukq[NU];
#pragma unroll
  for (int i = 0; i < NU; ++i) {
    const int u = tid + 256 * i;
    const int row = u >> 3, kq = u & 7;
    const int nl = row / R, m = row - nl * R;
    const bool ok = (UNITS % 256 == 0 || u < UNITS) && nl < vn;
    uo[i] = ok ? (nl * (int)P.lda + 4 * kq * R + m) * 4 : OOB;
    uo2[i] = ok ? (nl * (int)P.lda2 + 4 * kq * R + m) * 4 : OOB;
    ukq[i] = kq;
  }
  // B fragments of the wave's column blocks: two register sets (step kc's in
  // use while kc + 1's load)
  const int cb0 = n0 / 16 + wc * CB;
  nbf16x8 bq[2][CB][3];
  // (steps past the end issue the same loads at OOB offsets: every step
  // issues the same vector-memory instructions, so the compiler's wait counts
  // stay exact and a step waits only for the previous step's loads)
  auto load_b = [&](int kc, nbf16x8 (&d)[CB][3]) {
#pragma unroll
    for (int b = 0; b < CB; ++b)
#pragma unroll
      for (int pc = 0; pc < 3; ++pc) {
        const int cb = cb0 + b;
        const int off = (cb < ncb && kc < nkc) ? ((cb * nkc + kc) * 3 + pc) * 1024 : OOB;
        d[b][pc] = __builtin_bit_cast(nbf16x8, __builtin_amdgcn_raw_buffer_load_b128(RBb, lane * 16, off, 0));
      }
  };
  float ra[NU][4];
  auto load_a = [&](int kc) {
    const bool second = kc >= nkc1;
    const int kb = (second ? kc - nkc1 : kc) * BK, kend = second ? K2 : P.K1;
    const int soff = kb * R * 4;
#pragma unroll
    for (int i = 0; i < NU; ++i) {
      // K is a multiple of 4 (add_nl): a quad is in or out as a whole
      const int o = (kc < nkc && kb + 4 * ukq[i] < kend) ? (second ? uo2[i] : uo[i]) : OOB;
      const __amdgpu_buffer_rsrc_t Ra = second ? RA2 : RA;
      if constexpr (R == 1) {
        const float4 v = nl_ld4(Ra, o, soff);
        ra[i][0] = v.x, ra[i][1] = v.y, ra[i][2] = v.z, ra[i][3] = v.w;
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t) ra[i][t] = nl_ld1(Ra, o == OOB ? OOB : o + t * R * 4, soff);
      }
    }
  };
  auto store_a = [&](int buf) {
    char* base = reinterpret_cast<char*>(lds) + buf * NB_STAGE;
#pragma unroll
    for (int i = 0; i < NU; ++i) {
      const int u = tid + 256 * i;
      if (UNITS % 256 != 0 && u >= UNITS) continue;
      nu32x2 d[3];
      nb_split4(ra[i], d);
      const int row = u >> 3;
#pragma unroll
      for (int pc = 0; pc < 3; ++pc)
        *reinterpret_cast<nu32x2*>(base + ((pc * NB_PLANE + row * NB_ALD) + 4 * ukq[i]) * 2) = d[pc];
    }
  };
  constexpr int I6[6] = {2, 1, 0, 1, 0, 0}, J6[6] = {0, 1, 2, 0, 1, 0};
  auto compute = [&](int buf, const nbf16x8 (&bb)[CB][3], f32x4 (&c)[RB][CB]) {
    const char* base = reinterpret_cast<const char*>(lds) + buf * NB_STAGE;
#pragma unroll
    for (int a = 0; a < RB; ++a) {
      const int row = (wr * RB + a) * 16 + (lane & 15);
      nbf16x8 af[3];
#pragma unroll
      for (int pc = 0; pc < 3; ++pc)
        af[pc] = *reinterpret_cast<const nbf16x8*>(base + ((pc * NB_PLANE + row * NB_ALD) + 8 * (lane >> 4)) * 2);
#pragma unroll
      for (int b = 0; b < CB; ++b)
#pragma unroll
        for (int q = 0; q < 6; ++q)
          c[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[I6[q]], bb[b][J6[q]], c[a][b], 0, 0, 0);
    }
  };
  f32x4 acc[RB][CB];
#pragma unroll
  for (int a = 0; a < RB; ++a)
#pragma unroll
    for (int b = 0; b < CB; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[a][b][i] = 0.f;
  load_a(0);
  load_b(0, bq[0]);
  store_a(0);
  __syncthreads();
  // step kc (B set and LDS stage SET = kc & 1, a compile-time constant: the
  // loop runs two steps per iteration, an odd first step peeled): step kc +
  // 1's node rows and B fragments load while its MFMAs run.  (The two linears
  // of a split problem share the f32 accumulator: one K-concatenated sum.)
  auto step = [&](int kc, auto SET) {
    constexpr int CUR = decltype(SET)::value;
    load_a(kc + 1);
    load_b(kc + 1, bq[CUR ^ 1]);
    compute(CUR, bq[CUR], acc);
    store_a(CUR ^ 1);
    __syncthreads();
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  if (nkc & 1) {
    step(0, S0{});
#pragma unroll 1
    for (int kc = 1; kc < nkc; kc += 2) {
      step(kc, S1{});
      step(kc + 1, S0{});
    }
  } else {
#pragma unroll 1
    for (int kc = 0; kc < nkc; kc += 2) {
      step(kc, S0{});
      step(kc + 1, S1{});
    }
  }
  // D lane l, register i of block (a, b): row 16 (wr RB + a) + 4 (l / 16) + i,
  // column 32 wc + 16 b + l % 16 of the tile
  auto stage = [&](float* L, int LDR) {
#pragma unroll
    for (int a = 0; a < RB; ++a)
#pragma unroll
      for (int b = 0; b < CB; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = (wr * RB + a) * 16 + 4 * (lane >> 4) + i;
          const int col = wc * 32 + b * 16 + (lane & 15);
          const int nl = row / R, m = row - nl * R;
          if (row < ROWS) L[nl * LDR + col * R + m] = acc[a][b][i];
        }
  };
  if (P.epi <= 1)
    nl_epi_runs<BM, BN, R, NB_LDSF>(P, node0, n0, lds, stage);
  else
    nl_epi_gate<BM, BN, R, NB_LDSF>(P, node0, n0, lds, stage);
}

// ------------------------------------------------- skinny node linears
// k_nodelin_s: a problem with K <= 64 (the si2^T / si1 l > 0 blocks: K = 64 /
// 32 onto N = 320 / 352 mid channels) is output-bound, not MFMA-bound.  A
// workgroup owns 64 rows (T = 64 / R nodes) and ALL N columns: its node rows
// are loaded and split into the bf16 piece planes ONCE (both K chunks side by
// side in the two LDS stages), then it walks N in 64-column chunks: the
// chunk's bf16x6 MFMAs (B fragments from L2), the next chunk's B loads, the
// chunk's accumulators staged as node runs and copied out with buffer stores.
// Every chunk issues the same vector-memory instructions (masked lanes and
// steps past the end use OOB offsets the hardware drops), so the compiler's
// wait before a chunk's MFMAs covers that chunk's B loads only, and the
// previous chunks' output stores drain under them.
constexpr int NS_EPIF = 64 * 68;   // max over R of T x (64 R + 4) floats: one chunk's runs
constexpr int NS_LDSF = NB_LDSF + NS_EPIF;

template <int R>
__device__ __forceinline__ void nl_tile_s(const NlProb& P, int local, float* lds) {
  constexpr int BM = NB_BM, BK = NB_BK, CW = 64, WC = 2, RB = 2, CB = 2;
  constexpr int T = BM / R, ROWS = T * R;
  constexpr int UNITS = ROWS * (BK / 4), NU = (UNITS + 255) / 256;
  constexpr int OOB = 0x7ffffff0;
  constexpr int RUN = CW * R, LDR = RUN + 4, SEGC = RUN / 4, UC = T * SEGC, NC = (UC + 255) / 256;
  static_assert(T * LDR <= NS_EPIF, "chunk runs must fit");
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WC, wc = wave % WC;
  const int node0 = local * T;
  const int vn = min(T, P.nodes - node0);
  const int nkc = (P.K + BK - 1) / BK;   // 1 or 2
  const __amdgpu_buffer_rsrc_t RA =
      nl_rsrc(P.A + (int64_t)node0 * P.lda + P.a_off, ((int64_t)(vn - 1) * P.lda + P.K * R) * 4);
  const int ncb = (P.N + 15) / 16;
  const __amdgpu_buffer_rsrc_t RBb =
      nl_rsrc(static_cast<const float*>(P.Bb), (int64_t)ncb * nkc * 3 * 1024);
  const __amdgpu_buffer_rsrc_t RC =
      nl_rsrc(P.C + (int64_t)node0 * P.ldc + P.c_off, ((int64_t)(vn - 1) * P.ldc + P.N * R) * 4);
  // ---- the node rows of both K chunks, split into the piece planes
  {
    float ra[2][NU][4];
#pragma unroll
    for (int kc = 0; kc < 2; ++kc)
#pragma unroll
      for (int i = 0; i < NU; ++i) {
        const int u = tid + 256 * i;
        const int row = u >> 3, kq = u & 7;
        const int nl = row / R, m = row - nl * R;
        const bool ok = (UNITS % 256 == 0 || u < UNITS) && nl < vn && kc * BK + 4 * kq < P.K;
        const int o = ok ? (nl * (int)P.lda + (kc * BK + 4 * kq) * R + m) * 4 : OOB;
        if constexpr (R == 1) {
          const float4 v = nl_ld4(RA, o, 0);
          ra[kc][i][0] = v.x, ra[kc][i][1] = v.y, ra[kc][i][2] = v.z, ra[kc][i][3] = v.w;
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t) ra[kc][i][t] = nl_ld1(RA, ok ? o + t * R * 4 : OOB, 0);
        }
      }
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
      char* base = reinterpret_cast<char*>(lds) + kc * NB_STAGE;
#pragma unroll
      for (int i = 0; i < NU; ++i) {
        const int u = tid + 256 * i;
        if (UNITS % 256 != 0 && u >= UNITS) continue;
        nu32x2 d[3];
        nb_split4(ra[kc][i], d);
#pragma unroll
        for (int pc = 0; pc < 3; ++pc)
          *reinterpret_cast<nu32x2*>(base + ((pc * NB_PLANE + (u >> 3) * NB_ALD) + 4 * (u & 7)) * 2) = d[pc];
      }
    }
  }
  // ---- B fragments of a chunk: [k chunk][column block][piece]
  nbf16x8 bq[2][CB][3];
  auto load_b = [&](int ch) {
#pragma unroll
    for (int kc = 0; kc < 2; ++kc)
#pragma unroll
      for (int b = 0; b < CB; ++b)
#pragma unroll
        for (int pc = 0; pc < 3; ++pc) {
          const int cb = ch * 4 + wc * 2 + b;
          const int off = (cb < ncb && kc < nkc) ? ((cb * nkc + kc) * 3 + pc) * 1024 : OOB;
          bq[kc][b][pc] =
              __builtin_bit_cast(nbf16x8, __builtin_amdgcn_raw_buffer_load_b128(RBb, lane * 16, off, 0));
        }
  };
  load_b(0);
  __syncthreads();
  constexpr int I6[6] = {2, 1, 0, 1, 0, 0}, J6[6] = {0, 1, 2, 0, 1, 0};
  float* ep = lds + NB_LDSF;
  const int nch = (P.N + CW - 1) / CW;
#pragma unroll 1
  for (int ch = 0; ch < nch; ++ch) {
    f32x4 acc[RB][CB];
#pragma unroll
    for (int a = 0; a < RB; ++a)
#pragma unroll
      for (int b = 0; b < CB; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
      if (kc < nkc) {
        const char* base = reinterpret_cast<const char*>(lds) + kc * NB_STAGE;
#pragma unroll
        for (int a = 0; a < RB; ++a) {
          const int row = (wr * RB + a) * 16 + (lane & 15);
          nbf16x8 af[3];
#pragma unroll
          for (int pc = 0; pc < 3; ++pc)
            af[pc] = *reinterpret_cast<const nbf16x8*>(base + ((pc * NB_PLANE + row * NB_ALD) + 8 * (lane >> 4)) * 2);
#pragma unroll
          for (int b = 0; b < CB; ++b)
#pragma unroll
            for (int q = 0; q < 6; ++q)
              acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[I6[q]], bq[kc][b][J6[q]], acc[a][b], 0, 0, 0);
        }
      }
    }
    load_b(ch + 1);   // (past the last chunk: OOB, same instructions)
    // the chunk's runs: lds ep[nl * LDR + c * R + m]
    __syncthreads();   // the previous chunk's copy-out has read ep
#pragma unroll
    for (int a = 0; a < RB; ++a)
#pragma unroll
      for (int b = 0; b < CB; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = (wr * RB + a) * 16 + 4 * (lane >> 4) + i;
          const int col = wc * 32 + b * 16 + (lane & 15);
          const int nl = row / R, m = row - nl * R;
          if (row < ROWS) ep[nl * LDR + col * R + m] = acc[a][b][i];
        }
    __syncthreads();
    const int len = min(CW, P.N - ch * CW) * R;   // a multiple of 4 (N % 4 == 0)
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int u = tid + 256 * i;
      const int nl = u / SEGC, j = 4 * (u - nl * SEGC);
      const bool ok = (UC % 256 == 0 || u < UC) && nl < vn && j < len;
      const f32x4 v = *reinterpret_cast<const f32x4*>(ep + (ok ? nl * LDR + j : 0));
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, v), RC,
                                             ok ? (nl * (int)P.ldc + ch * CW * R + j) * 4 : OOB, 0, 0);
    }
  }
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 8))) void
k_nodelin_s(NlBatch batch) {
  __shared__ __attribute__((aligned(16))) float lds[NS_LDSF];
  const int tile = blockIdx.x;
  int pi = 0;
#pragma unroll 1
  for (int i = 1; i < batch.nprob; ++i)
    if (tile >= batch.p[i].tile_begin) pi = i;
  NlProb P = batch.p[0];
  if (pi == 1) P = batch.p[1];
  if (pi == 2) P = batch.p[2];
  if (pi == 3) P = batch.p[3];
  const int local = tile - P.tile_begin;
  switch (P.R) {
    case 1: nl_tile_s<1>(P, local, lds); break;
    case 3: nl_tile_s<3>(P, local, lds); break;
    default: nl_tile_s<5>(P, local, lds); break;
  }
}

#ifndef E3GNN_NLB_WAVES
#define E3GNN_NLB_WAVES 3
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(E3GNN_NLB_WAVES, 8))) void
k_nodelin_b(NlBatch batch) {
  __shared__ __attribute__((aligned(16))) float lds[NB_LDSF];
  const int tile = blockIdx.x;
  int pi = 0;
#pragma unroll 1
  for (int i = 1; i < batch.nprob; ++i)
    if (tile >= batch.p[i].tile_begin) pi = i;
  NlProb P = batch.p[0];
  if (pi == 1) P = batch.p[1];
  if (pi == 2) P = batch.p[2];
  if (pi == 3) P = batch.p[3];
  const int local = tile - P.tile_begin;
  if (P.wn == 1) {
    switch (P.R) {
      case 1: nl_tile_b<0, 1>(P, local, lds); break;
      case 3: nl_tile_b<0, 3>(P, local, lds); break;
      default: nl_tile_b<0, 5>(P, local, lds); break;
    }
  } else {
    switch (P.R) {
      case 1: nl_tile_b<1, 1>(P, local, lds); break;
      case 3: nl_tile_b<1, 3>(P, local, lds); break;
      default: nl_tile_b<1, 5>(P, local, lds); break;
    }
  }
}
}  // namespace

hipError_t launch_gemm(const GemmBatch& b, hipStream_t s) {
  if (b.total_tiles <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_gemm, dim3(b.total_tiles), dim3(256), 0, s, b);
  return hipGetLastError();
}

// which kernel runs a node-linear problem (E3GNN_NL_BF16): 0 k_nodelin (f32
// MFMA) for all; 1 (default) k_nodelin_s (skinny, bf16x6) and k_nodelin_b
// (bf16x6 tiles) where they measured faster, k_nodelin otherwise; 2
// k_nodelin_s where it applies, k_nodelin_b otherwise; 3 k_nodelin_b for all
static int nl_mode() {
  static const int m = [] {
    const char* v = std::getenv("E3GNN_NL_BF16");
    return v ? std::atoi(v) : 1;
  }();
  return m;
}

bool add_nl(NlBatch& b, const NlProb& p) {
  if (b.nprob >= NL_MAX_PROBS) return false;
  if (p.R != 1 && p.R != 3 && p.R != 5) return false;
  auto al = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  if (!al(p.A) || !al(p.B) || !al(p.C) || p.lda % 4 || p.a_off % 4 || p.N % 4 || p.ldc % 4 ||
      p.c_off % 4)
    return false;
  if (p.epi >= 2 && (!al(p.xo) || p.ldxo % 4 || p.xo_off % 4 || (p.epi == 2 && p.R != 1)))
    return false;
  NlProb q = p;
  const int mode = nl_mode();
  // skinny: K <= 64 onto N >= 128 columns (si2^T l > 0: 345 vs ~400 us per
  // launch on the f32 tiles; si1's N <= 64 blocks ran slower there: f32)
  const bool skinny = p.Bb && (mode == 1 || mode == 2) && p.K == p.K1 && p.K <= 64 &&
                      p.K % 4 == 0 && p.N >= 128 && p.epi == 0;
  // bf16x6 tiles (default, mode 1) for the wide scalar blocks: l = 0, K and N
  // >= 224 -- the 0e gate launch (K 352, N 224) and si2^T's 0e block (224 x
  // 224) are MFMA-bound on the f32 tiles (139 vs 185 us and 75 vs ~105 us per
  // launch); si1's and si1^T + sc^T's 0e blocks (N 128) are not (+5 to +8 us)
  const bool btile = p.Bb && !skinny && p.K1 % 4 == 0 && (p.K - p.K1) % 4 == 0 &&
                     (mode == 2 || mode == 3 || (mode == 1 && p.R == 1 && p.K >= 224 && p.N >= 224));
  int tm, tn;
  if (skinny) {          // k_nodelin_s: 64-row tiles over all N
    q.kind = 2;
    q.wn = 2;
    q.ns = 1;
    q.tpn = NB_BM / p.R;
    tm = (p.nodes + q.tpn - 1) / q.tpn;
    tn = 1;
  } else if (btile) {    // k_nodelin_b: 64-row tiles, BN 32 (N <= 32) or 64
    q.kind = 1;
    q.wn = p.N <= 32 ? 1 : 2;
    q.ns = 1;
    q.tpn = NB_BM / p.R;
    tm = (p.nodes + q.tpn - 1) / q.tpn;
    tn = (p.N + 32 * q.wn - 1) / (32 * q.wn);
  } else {
    if (p.K > p.K1 && (!al(p.A2) || p.lda2 % 4 || p.a_off2 % 4 || p.K1 % NL_BK)) return false;
    q.kind = 0;
    q.wn = p.N <= 32 ? 1 : 2;
    q.ns = (E3GNN_NL_WIDE && q.wn == 2 && p.K == p.K1 && p.K <= E3GNN_NL_WIDE_KMAX && p.N >= 128) ? 2 : 1;
    const int BM = 128 / q.wn, BN = 32 * q.wn * q.ns;
    q.tpn = BM / p.R;
    tm = (p.nodes + q.tpn - 1) / q.tpn;
    tn = (p.N + BN - 1) / BN;
  }
  if (tm <= 0 || tn <= 0) return true;
  q.tiles_n = tn;
  q.tile_begin = b.total_tiles;
  b.p[b.nprob++] = q;
  b.total_tiles += tm * tn;
  return true;
}

// one launch per kernel kind present in the batch (same stream, in order)
hipError_t launch_nodelin(const NlBatch& b, hipStream_t s) {
  if (b.total_tiles <= 0) return hipSuccess;
  for (int kind = 0; kind < 3; ++kind) {
    NlBatch sb;
    std::memset(&sb, 0, sizeof(sb));
    for (int i = 0; i < b.nprob; ++i) {
      if (b.p[i].kind != kind) continue;
      const int end = i + 1 < b.nprob ? b.p[i + 1].tile_begin : b.total_tiles;
      NlProb q = b.p[i];
      q.tile_begin = sb.total_tiles;
      sb.p[sb.nprob++] = q;
      sb.total_tiles += end - b.p[i].tile_begin;
    }
    if (sb.total_tiles <= 0) continue;
    if (kind == 0)
      hipLaunchKernelGGL(k_nodelin, dim3(sb.total_tiles), dim3(256), 0, s, sb);
    else if (kind == 1)
      hipLaunchKernelGGL(k_nodelin_b, dim3(sb.total_tiles), dim3(256), 0, s, sb);
    else
      hipLaunchKernelGGL(k_nodelin_s, dim3(sb.total_tiles), dim3(256), 0, s, sb);
  }
  return hipGetLastError();
}

}  // namespace e3gnn
