// Fused radial-MLP + tensor-product kernels (forward and force backward), gfx950.
//
// Reference: IrrepsConvolution.forward (sevenn/nn/convolution.py:104-123):
//   w = FCN(edge_embedding)                      (e3nn FullyConnectedNet 8->64->64->W)
//   msg = TP(x[edge_index[1]], Y, w)              (uvu, convolution.py:72-95)
//   agg = scatter_sum(msg, edge_index[0]) / denominator
// and its reverse-mode pass (what ForceStressOutput obtains through autograd,
// force_output.py:74-130).  The per-edge weights w (E x 960 for the middle
// blocks) never touch HBM: they are produced by f32 MFMA directly into the
// registers the tensor product reads.
//
// Mapping (one wave = one centre; its CSR edges in row blocks of 32):
//   * v_mfma_f32_32x32x2_f32: A lane l = A[i=l&31][k=l>>5], B lane l =
//     B[k=l>>5][j=l&31], D lane l reg r = D[ROW(r, l>>5)][l&31],
//     ROW(r,h) = (r&3) + 8(r>>2) + 4h.
//   * The MLP runs transposed (H^T = W^T emb^T), so each result is already the
//     k-operand of the next product (accumulator-as-operand; the k order is
//     permuted identically on the weight side).  Edge slot i of the row block
//     holds edge SIGMA(i) so that in the final w = H2 W2 product lane l,
//     register r holds w[edge 16*(l>>5) + r][channel l&31]: each half-wave owns
//     16 consecutive edges of the centre and one channel per lane.
//   * The tensor product then runs lane = channel, register-accumulating the
//     centre's message over its edges (forward), or producing dE/dw, dE/dx and
//     dE/du per edge (backward).  dE/dw goes through a 4 KB LDS transpose into
//     the dH2^T = W2 dw^T product; the MLP chain backward (dA2, dH1, dA1, demb)
//     again stays in accumulators.
// Deterministic: no atomics; every sum has a fixed order.
#include "cg_tables.h"
#include "common.h"
#include "fused.h"
#include "tp.h"

#include <type_traits>

namespace e3gnn {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int N, int I = 0, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<N, I + 1>(f);
  }
}

__device__ __forceinline__ constexpr int ROW(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }
__device__ __forceinline__ constexpr int SIGMA(int i) {
  return 16 * ((i >> 2) & 1) + (i & 3) + 4 * (i >> 3);
}
__device__ __forceinline__ constexpr int yoff(int l) { return l == 0 ? 0 : (l == 1 ? 1 : 4); }

// Scheduling fence for the unrolled edge loops: VALU/SALU/MFMA may move across it,
// memory instructions may not, so at most EG edges' gathers are in flight per wave
// (bounds VGPR use; the MFMA chain of the next column block hides the rest).
#ifndef E3GNN_EG
#define E3GNN_EG 4
#endif
__device__ __forceinline__ void mem_fence_sched() { __builtin_amdgcn_sched_barrier(0x0F); }

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}
__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------- weight operands
// Weight operands are read through buffer descriptors: the per-lane part of the
// offset is ONE VGPR and the per-k-step part a scalar (soffset), so the compiler
// cannot hoist hundreds of 64-bit addresses out of the centre loop (it did, and
// spilled them).  Out-of-range offsets read 0 (used for padded rows).
struct WRes {
  __amdgpu_buffer_rsrc_t w0, w1, w2, w2t;
};
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* p, int nfloats) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, nfloats * 4, 0x00020000);
}
__device__ __forceinline__ WRes make_wres(const MlpW& W, int width) {
  return {rsrc(W.w0, 8 * 64), rsrc(W.w1, 64 * 64), rsrc(W.w2, 64 * width), rsrc(W.w2t, 64 * width)};
}
__device__ __forceinline__ float ldw(__amdgpu_buffer_rsrc_t r, int vbytes, int sbytes) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, vbytes, sbytes, 0);
}
// ROW(s&15, 0) + 32*(s>>4): the half-independent part of a permuted k index
__device__ __forceinline__ constexpr int KROW(int s) { return 32 * (s >> 4) + ROW(s & 15, 0); }

// ---------------------------------------------------------------- radial MLP
// H1pre^T = W0^T emb^T (K = 8), H1^T = act, H2pre^T = W1^T H1^T (K = 64), H2^T = act.
// Edge slot (l&31) of this 32-edge row block holds edge e0 + SIGMA(slot) (< e1).
struct MlpT {
  f32x16 a1[2], a2[2];  // pre-activations, blocks of 32 hidden units
};

__device__ __forceinline__ void mlp_pre(const WRes& R, const float* __restrict__ emb, int e0,
                                        int e1, int lane, MlpT& m) {
  const int half = lane >> 5, col = lane & 31;
  const int e = e0 + SIGMA(col);
  float b[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) b[s] = e < e1 ? emb[(int64_t)e * 8 + 2 * s + half] : 0.f;
  const int v0 = (half * 64 + col) * 4;  // W0s[(2s + half)][32 bo + col]
#pragma unroll
  for (int bo = 0; bo < 2; ++bo) {
    f32x16 acc = zero16();
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = mfma(ldw(R.w0, v0, (2 * s * 64 + 32 * bo) * 4), b[s], acc);
    m.a1[bo] = acc;
  }
  float a[32];
  const int v1 = (4 * half * 64 + col) * 4;  // W1s[KROW(s) + 4 half][32 bo + col]
#pragma unroll
  for (int bo = 0; bo < 2; ++bo) {
#pragma unroll
    for (int s = 0; s < 32; ++s) a[s] = ldw(R.w1, v1, (KROW(s) * 64 + 32 * bo) * 4);
    f32x16 acc = zero16();
#pragma unroll
    for (int s = 0; s < 32; ++s) acc = mfma(a[s], act_fwd(m.a1[s >> 4][s & 15]), acc);
    m.a2[bo] = acc;
  }
}

// w[:, col0:col0+32] for the row block: lane = channel col0+(l&31), reg r = edge 16h+r
__device__ __forceinline__ f32x16 mlp_w_block(const f32x16 (&h2)[2], __amdgpu_buffer_rsrc_t w2,
                                              int W, int col0, int lane) {
  const int half = lane >> 5, col = lane & 31;
  float b[32];
  const int v = (4 * half * W + col) * 4;  // W2s[KROW(s) + 4 half][col0 + col]
#pragma unroll
  for (int s = 0; s < 32; ++s) b[s] = ldw(w2, v, (KROW(s) * W + col0) * 4);
  f32x16 acc = zero16();
#pragma unroll
  for (int s = 0; s < 32; ++s) acc = mfma(h2[s >> 4][s & 15], b[s], acc);
  return acc;
}

// ---------------------------------------------------------------- TP pieces
template <int L1, int L2, int L3>
__device__ __forceinline__ void tp_acc(const float* x, const float* y, float w, float* acc) {
  float t[2 * L3 + 1];
#pragma unroll
  for (int k = 0; k < 2 * L3 + 1; ++k) t[k] = 0.f;
  using C = CG<L1, L2, L3>;
#pragma unroll
  for (int q = 0; q < C::n; ++q) t[C::e[q].k] += C::e[q].c * (x[C::e[q].i] * y[C::e[q].j]);
#pragma unroll
  for (int k = 0; k < 2 * L3 + 1; ++k) acc[k] += w * t[k];
}

template <int L1, int L2, int L3>
__device__ __forceinline__ float tp_bwd(const float* x, const float* y, float w, const float* gm,
                                        float* dx, float* dy) {
  using C = CG<L1, L2, L3>;
  float dwv = 0.f;
#pragma unroll
  for (int q = 0; q < C::n; ++q) {
    const int i = C::e[q].i, j = C::e[q].j, k = C::e[q].k;
    const float cg = C::e[q].c * gm[k];
    dwv += cg * (x[i] * y[j]);
    dx[i] += (cg * w) * y[j];
    dy[j] += (cg * w) * x[i];
  }
  return dwv;
}

template <class L, int P>
constexpr bool first_of_iblock() {
  for (int q = 0; q < P; ++q)
    if (L::P[q].l1 == L::P[P].l1) return false;
  return true;
}

// ---------------------------------------------------------------- forward
// One wave per centre.  agg[c] = sum_e TP(h[nbr e], Y_e, w_e) / denom.
template <class L>
__global__ __launch_bounds__(256) void k_conv_fwd(const int* __restrict__ row_ptr,
                                                  const int* __restrict__ nbr,
                                                  const float* __restrict__ emb,
                                                  const float* __restrict__ Y,
                                                  const float* __restrict__ h,
                                                  float* __restrict__ agg, MlpW W, int n_centers,
                                                  float denom) {
  const int c = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (c >= n_centers) return;
  const int lane = threadIdx.x & 63, half = lane >> 5, col = lane & 31;
  const int beg = row_ptr[c], end = row_ptr[c + 1];
  float* out = agg + (int64_t)c * L::DM;
  const WRes R = make_wres(W, L::W);
  // row blocks of 32 edges; the first block stores, later ones accumulate
  for (int e0 = beg; e0 < end || e0 == beg; e0 += 32) {
    const bool first_block = e0 == beg;
    f32x16 h2[2];
    {
      MlpT m;
      mlp_pre(R, emb, e0, end, lane, m);
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) h2[b][r] = act_fwd(m.a2[b][r]);
    }
    sfor<L::NP>([&](auto pi) {
      constexpr PathDef p = L::P[pi];
      constexpr int D1 = 2 * p.l1 + 1, D3 = 2 * p.l3 + 1;
      for (int j = 0; j < p.mul / 32; ++j) {
        const int u = 32 * j + col;
        float acc[D3];
#pragma unroll
        for (int k = 0; k < D3; ++k) acc[k] = 0.f;
        const f32x16 wv = mlp_w_block(h2, R.w2, L::W, p.woff + 32 * j, lane);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          if (r % E3GNN_EG == 0) mem_fence_sched();
          const int e = e0 + 16 * half + r;
          if (e < end) {
            const int src = nbr[e];
            float x[D1], y[2 * p.l2 + 1];
#pragma unroll
            for (int i = 0; i < D1; ++i) x[i] = h[(int64_t)src * L::DX + p.xoff + u * D1 + i];
#pragma unroll
            for (int q = 0; q < 2 * p.l2 + 1; ++q) y[q] = Y[(int64_t)e * 9 + yoff(p.l2) + q];
            tp_acc<p.l1, p.l2, p.l3>(x, y, wv[r], acc);
          }
        }
#pragma unroll
        for (int k = 0; k < D3; ++k) {
          const float v = acc[k] + __shfl_xor(acc[k], 32, 64);
          if (half == 0) {
            float* o = out + p.moff + u * D3 + k;
            *o = first_block ? v / denom : *o + v / denom;
          }
        }
      }
    });
    if (end <= beg) break;
  }
}

// ---------------------------------------------------------------- backward
// One wave per centre, row blocks of 32 edges (each independent).
// In: gagg = dE/dagg / denom.  Out (accumulated over blocks): dxc (per-edge
// dE/dx[nbr], written), dgu (E x 3, dE/du of the unit vector, +=), demb (E x 8, +=).
template <class L>
__global__ __launch_bounds__(256, 2) void k_conv_bwd(const int* __restrict__ row_ptr,
                                                     const int* __restrict__ nbr,
                                                     const float* __restrict__ emb,
                                                     const float* __restrict__ Y,
                                                     const float* __restrict__ h,
                                                     const float* __restrict__ gagg, MlpW W,
                                                     float* __restrict__ dxc,
                                                     float* __restrict__ dgu,
                                                     float* __restrict__ demb, int n_centers) {
  // per wave: dw transpose tile [32 slots][33] + dE/du partials [16 edges][3][64 lanes]
  __shared__ float lds[4][32 * 33 + 16 * 3 * 64];
  const int wid = threadIdx.x >> 6;
  const int c = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + wid);
  if (c >= n_centers) return;
  float* dwbuf = lds[wid];
  float* gubuf = lds[wid] + 32 * 33;
  const int lane = threadIdx.x & 63, half = lane >> 5, col = lane & 31;
  const int beg = row_ptr[c], end = row_ptr[c + 1];
  const float* gc = gagg + (int64_t)c * L::DM;
  const WRes R = make_wres(W, L::W);
  for (int e0 = beg; e0 < end; e0 += 32) {
    f32x16 h2[2];
    {
      MlpT m;
      mlp_pre(R, emb, e0, end, lane, m);
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) h2[b][r] = act_fwd(m.a2[b][r]);
    }
    f32x16 dh2[2] = {zero16(), zero16()};
#pragma unroll
    for (int q = 0; q < 48; ++q) gubuf[q * 64 + lane] = 0.f;

    sfor<L::NP>([&](auto pi) {
      constexpr PathDef p = L::P[pi];
      constexpr int D1 = 2 * p.l1 + 1, D2 = 2 * p.l2 + 1, D3 = 2 * p.l3 + 1;
      constexpr bool first = first_of_iblock<L, pi>();
      for (int j = 0; j < p.mul / 32; ++j) {
        const int u = 32 * j + col;
        const int col0 = p.woff + 32 * j;
        const f32x16 wv = mlp_w_block(h2, R.w2, L::W, col0, lane);
        float gm[D3];
#pragma unroll
        for (int k = 0; k < D3; ++k) gm[k] = gc[p.moff + u * D3 + k];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          if (r % E3GNN_EG == 0) mem_fence_sched();
          const int e = e0 + 16 * half + r;
          float dwv = 0.f;
          if (e < end) {
            const int src = nbr[e];
            float x[D1], y[D2], dx[D1], dy[D2];
#pragma unroll
            for (int i = 0; i < D1; ++i) {
              x[i] = h[(int64_t)src * L::DX + p.xoff + u * D1 + i];
              dx[i] = 0.f;
            }
#pragma unroll
            for (int q = 0; q < D2; ++q) {
              y[q] = Y[(int64_t)e * 9 + yoff(p.l2) + q];
              dy[q] = 0.f;
            }
            dwv = tp_bwd<p.l1, p.l2, p.l3>(x, y, wv[r], gm, dx, dy);
            if (dxc) {
              float* d = dxc + (int64_t)e * L::DX + p.xoff + u * D1;
#pragma unroll
              for (int i = 0; i < D1; ++i) d[i] = first ? dx[i] : d[i] + dx[i];
            }
            // dE/du (unit vector) of the filter Y_l2 (SH polynomials of serial_code.py:50-70)
            float* g3 = gubuf + r * 192 + lane;
            if constexpr (p.l2 == 1) {
              const float s3 = 1.7320508075688772f;
              g3[0] += s3 * dy[0];
              g3[64] += s3 * dy[1];
              g3[128] += s3 * dy[2];
            } else if constexpr (p.l2 == 2) {
              const float s3 = 1.7320508075688772f, s5 = 2.23606797749979f, c15 = s3 * s5;
              const float ux = Y[(int64_t)e * 9 + 1] / s3, uy = Y[(int64_t)e * 9 + 2] / s3,
                          uz = Y[(int64_t)e * 9 + 3] / s3;
              g3[0] += c15 * (uz * dy[0] + uy * dy[1]) - s5 * ux * dy[2] - c15 * ux * dy[4];
              g3[64] += c15 * (ux * dy[1] + uz * dy[3]) + 2.f * s5 * uy * dy[2];
              g3[128] += c15 * (ux * dy[0] + uy * dy[3]) - s5 * uz * dy[2] + c15 * uz * dy[4];
            }
          }
          dwbuf[ROW(r, half) * 33 + col] = dwv;
        }
        // dH2^T += W2[:, col0:col0+32] dw^T   (B lane l = dw[slot l&31][channel 2s + (l>>5)])
#pragma unroll
        for (int bo = 0; bo < 2; ++bo) {
          float a[16];
#pragma unroll
          for (int s = 0; s < 16; ++s)
            a[s] = ldw(R.w2t, (half * 64 + col) * 4, ((col0 + 2 * s) * 64 + 32 * bo) * 4);
#pragma unroll
          for (int s = 0; s < 16; ++s) dh2[bo] = mfma(a[s], dwbuf[col * 33 + 2 * s + half], dh2[bo]);
        }
      }
    });

    // ---- dE/du: sum the 32 channel lanes of each half in a fixed order, per edge
    // (lane t < 48 owns (r = t / 3, k = t % 3) of half 0, lanes 48.. none; two passes)
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const int t = lane;  // (r, k) = (t / 3, t % 3) for t < 48
      if (t < 48) {
        const int r = t / 3, k = t - 3 * (t / 3);
        const float* src = gubuf + r * 192 + k * 64 + 32 * pass;
        float v = 0.f;
        for (int q = 0; q < 32; ++q) v += src[q];
        const int e = e0 + 16 * pass + r;
        if (e < end) dgu[(int64_t)e * 3 + k] += v;
      }
    }

    // ---- MLP chain backward (recompute pre-activations)
    MlpT m;
    mlp_pre(R, emb, e0, end, lane, m);
    f32x16 da2[2], dh1[2];
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) da2[b][r] = dh2[b][r] * act_grad(m.a2[b][r]);
    // dH1^T = W1 dA2^T  (A[i=h_in][k=h_out] = W1s[h_in][h_out])
#pragma unroll
    for (int bo = 0; bo < 2; ++bo) {
      float a[32];
#pragma unroll
      for (int s = 0; s < 32; ++s)
        a[s] = ldw(R.w1, (col * 64 + 4 * half) * 4, (32 * bo * 64 + KROW(s)) * 4);
      f32x16 acc = zero16();
#pragma unroll
      for (int s = 0; s < 32; ++s) acc = mfma(a[s], da2[s >> 4][s & 15], acc);
      dh1[bo] = acc;
    }
    // dA1 = dH1 * act'(A1pre); demb^T = W0 dA1^T (rows n < 8)
    f32x16 de = zero16();
    {
      float a[32];
#pragma unroll
      for (int s = 0; s < 32; ++s)  // rows n >= 8 fall outside the descriptor: 0
        a[s] = ldw(R.w0, (col * 64 + 4 * half) * 4, KROW(s) * 4);
#pragma unroll
      for (int s = 0; s < 32; ++s)
        de = mfma(a[s], dh1[s >> 4][s & 15] * act_grad(m.a1[s >> 4][s & 15]), de);
    }
    {
      const int e = e0 + SIGMA(col);
      if (e < end) {
#pragma unroll
        for (int r = 0; r < 4; ++r) demb[(int64_t)e * 8 + ROW(r, half)] += de[r];
      }
    }
  }
}

}  // namespace

template <class L>
static hipError_t fwd_impl(const FusedArgs& a, hipStream_t s) {
  if (a.n_centers <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_conv_fwd<L>, dim3((a.n_centers + 3) / 4), dim3(256), 0, s, a.row_ptr,
                     a.nbr, a.emb, a.Y, a.h, a.agg, a.W, a.n_centers, a.denom);
  return hipGetLastError();
}
template <class L>
static hipError_t bwd_impl(const FusedArgs& a, hipStream_t s) {
  if (a.n_centers <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_conv_bwd<L>, dim3((a.n_centers + 3) / 4), dim3(256), 0, s, a.row_ptr,
                     a.nbr, a.emb, a.Y, a.h, a.gagg, a.W, a.dxc, a.dgu, a.demb, a.n_centers);
  return hipGetLastError();
}

hipError_t launch_conv_fwd(int kind, const FusedArgs& a, hipStream_t s) {
  switch (kind) {
    case 0: return fwd_impl<LayerFirst>(a, s);
    case 1: return fwd_impl<LayerMid>(a, s);
    default: return fwd_impl<LayerLast>(a, s);
  }
}
hipError_t launch_conv_bwd(int kind, const FusedArgs& a, hipStream_t s) {
  switch (kind) {
    case 0: return bwd_impl<LayerFirst>(a, s);
    case 1: return bwd_impl<LayerMid>(a, s);
    default: return bwd_impl<LayerLast>(a, s);
  }
}

}  // namespace e3gnn
