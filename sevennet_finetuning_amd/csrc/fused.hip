// Fused radial-MLP + tensor-product kernels (forward and force backward), gfx950.
//
// Reference: IrrepsConvolution.forward (sevenn/nn/convolution.py:104-123):
//   w = FCN(edge_embedding)                      (e3nn FullyConnectedNet 8->64->64->W)
//   msg = TP(x[edge_index[1]], Y, w)              (uvu, convolution.py:72-95)
//   agg = scatter_sum(msg, edge_index[0]) / denominator
// and its reverse-mode pass (what ForceStressOutput obtains through autograd,
// force_output.py:74-130).  The per-edge weights w (E x 960 for the middle
// blocks) never touch HBM: f32 MFMA produces them directly in the registers the
// tensor product reads.
//
// Mapping: one wave = one centre, its CSR edges in tiles of 16.
//   * v_mfma_f32_16x16x4_f32: A lane l = A[i=l&15][k=l>>4], B lane l =
//     B[k=l>>4][j=l&15], D lane l reg r = D[4(l>>4)+r][l&15].  Lane group
//     g = l>>4, column c = l&15.
//   * The MLP runs transposed (H^T = W^T emb^T: rows = hidden units, columns =
//     edge slots), so every product's accumulator is the k-operand of the next
//     one (k-step s of a 64-deep product covers hidden unit 16(s>>2)+4g+(s&3)
//     in lane group g; the weight operand uses the same permuted k).
//   * w = H2 W2[:, 16-column block]: lane (g, c) holds w[edge 4g+r][channel c]
//     in register r -- 4 consecutive edges x 1 channel per lane.  The tensor
//     product runs on that layout: the forward sums the centre's message over
//     registers and the 4 lane groups; the backward produces dE/dw (-> 1 KB LDS
//     transpose -> dH2^T = W2 dw^T), dE/dx (accumulated over the paths of an
//     input irrep in registers, stored once per edge) and dE/du (12 registers,
//     reduced over the 16 channel lanes once per tile).  The MLP chain backward
//     (dA2, dH1, dA1, demb) stays in accumulators.
//   * ~120 VGPRs, 4 waves/SIMD; weights via buffer descriptors (scalar k
//     offsets, one VGPR of lane offset).
// Deterministic: no atomics; every sum has a fixed order.
#include "cg_tables.h"
#include "common.h"
#include "fused.h"
#include "tp.h"

#include <type_traits>

namespace e3gnn {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int N, int I = 0, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<N, I + 1>(f);
  }
}

__device__ __forceinline__ constexpr int yoff(int l) { return l == 0 ? 0 : (l == 1 ? 1 : 4); }
// hidden unit of k-step s, lane group 0 (add 4g): 16(s>>2) + (s&3)
__device__ __forceinline__ constexpr int KH(int s) { return 16 * (s >> 2) + (s & 3); }

// Phase fence: keeps the scheduler from interleaving (and hoisting loads across)
// the MFMA chain of one column block and the tensor product of another, which
// otherwise multiplies live registers and halves occupancy.
__device__ __forceinline__ void phase() { __builtin_amdgcn_sched_barrier(0); }

__device__ __forceinline__ f32x4 zero4() {
  f32x4 z;
  z[0] = z[1] = z[2] = z[3] = 0.f;
  return z;
}
__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------- weight operands
// Weight operands are read through buffer descriptors: the per-lane part of the
// offset is one VGPR and the per-k-step part a scalar (soffset), so the compiler
// does not hoist hundreds of 64-bit addresses out of the centre loop (which it
// did, and spilled).  Offsets outside the descriptor read 0 (padded rows).
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
  // the builtin returns the raw 32 bits (an unsigned int): reinterpret, never convert
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vbytes, sbytes, 0));
}

__device__ __forceinline__ void stw(float v, __amdgpu_buffer_rsrc_t r, int vbytes, int sbytes) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, vbytes, sbytes, 0);
}
// descriptor over [p, p + nbytes) (nbytes clamped to the 32-bit range)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_bytes(const void* p, int64_t nbytes) {
  const int n = nbytes > 0x7fffffff ? 0x7fffffff : (int)nbytes;
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, n, 0x00020000);
}

// ---------------------------------------------------------------- radial MLP
// Tile of 16 edge slots [e0, e0+16) (slots >= e1 are zero rows).
// a1/a2: pre-activations of the two hidden layers, transposed (4 blocks of 16 units).
struct MlpT {
  f32x4 a1[4], a2[4];
};

// b[s] = emb[edge of slot (l&15)][4s + (l>>4)] (0 for padded slots)
__device__ __forceinline__ void mlp_chain(const WRes& R, const float (&b)[2], int lane, MlpT& m) {
  const int g = lane >> 4, c = lane & 15;
  const int v0 = (g * 64 + c) * 4;  // W0s[4s + g][16 bh + c]
#pragma unroll
  for (int bh = 0; bh < 4; ++bh) {
    f32x4 acc = zero4();
#pragma unroll
    for (int s = 0; s < 2; ++s) acc = mfma(ldw(R.w0, v0, (4 * s * 64 + 16 * bh) * 4), b[s], acc);
    m.a1[bh] = acc;
  }
  const int v1 = (4 * g * 64 + c) * 4;  // W1s[KH(s) + 4g][16 bo + c]
#pragma unroll
  for (int bo = 0; bo < 4; ++bo) {
    phase();
    float a[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) a[s] = ldw(R.w1, v1, (KH(s) * 64 + 16 * bo) * 4);
    f32x4 acc = zero4();
#pragma unroll
    for (int s = 0; s < 16; ++s) acc = mfma(a[s], act_fwd(m.a1[s >> 2][s & 3]), acc);
    m.a2[bo] = acc;
  }
}

__device__ __forceinline__ void mlp_pre(const WRes& R, const float* __restrict__ emb, int e0,
                                        int e1, int lane, MlpT& m) {
  const int g = lane >> 4, c = lane & 15;
  const int e = e0 + c;
  float b[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) b[s] = e < e1 ? emb[(int64_t)e * 8 + 4 * s + g] : 0.f;
  mlp_chain(R, b, lane, m);
}

// w[:, col0:col0+16] of the tile: lane (g, c) reg r = w[edge 4g+r][channel col0+c]
__device__ __forceinline__ f32x4 mlp_w_block(const f32x4 (&h2)[4], __amdgpu_buffer_rsrc_t w2,
                                             int W, int col0, int lane) {
  const int g = lane >> 4, c = lane & 15;
  float b[16];
  const int v = (4 * g * W + c) * 4;  // W2s[KH(s) + 4g][col0 + c]
#pragma unroll
  for (int s = 0; s < 16; ++s) b[s] = ldw(w2, v, (KH(s) * W + col0) * 4);
  f32x4 acc = zero4();
#pragma unroll
  for (int s = 0; s < 16; ++s) acc = mfma(h2[s >> 2][s & 3], b[s], acc);
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

template <class L, int I>
constexpr int iblock_mul() {
  for (int p = 0; p < L::NP; ++p)
    if (L::P[p].l1 == I) return L::P[p].mul;
  return 0;
}
template <class L, int I>
constexpr int iblock_xoff() {
  for (int p = 0; p < L::NP; ++p)
    if (L::P[p].l1 == I) return L::P[p].xoff;
  return 0;
}

// per tile: neighbour ids of the lane group's 4 edges, Y of the 16 edges in LDS
__device__ __forceinline__ void load_tile_edges(const int* __restrict__ nbr,
                                                const float* __restrict__ Y, int e0, int end,
                                                int lane, int (&src)[4], float* ybuf) {
  const int g = lane >> 4;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int e = e0 + 4 * g + r;
    src[r] = e < end ? nbr[e] : 0;
  }
#pragma unroll
  for (int q0 = 0; q0 < 144; q0 += 64) {
    const int q = q0 + lane;
    if (q < 144) ybuf[q] = (e0 + q / 9 < end) ? Y[(int64_t)e0 * 9 + q] : 0.f;
  }
}

// ---------------------------------------------------------------- forward
// agg[c] = sum_e TP(h[nbr e], Y_e, w_e) / denom; the first tile stores, later ones add.
template <class L>
__global__ __launch_bounds__(256) void k_conv_fwd(const int* __restrict__ row_ptr,
                                                  const int* __restrict__ nbr,
                                                  const float* __restrict__ emb,
                                                  const float* __restrict__ Y,
                                                  const float* __restrict__ h,
                                                  float* __restrict__ agg, MlpW W, int n_centers,
                                                  int n_nodes, float denom) {
  __shared__ float lds[4][160];
  const int wid = threadIdx.x >> 6;
  const int c = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + wid);
  if (c >= n_centers) return;
  float* ybuf = lds[wid];
  const int lane = threadIdx.x & 63, g = lane >> 4, col = lane & 15;
  const int beg = row_ptr[c], end = row_ptr[c + 1];
  float* out = agg + (int64_t)c * L::DM;
  const WRes R = make_wres(W, L::W);
  const __amdgpu_buffer_rsrc_t Rh = rsrc_bytes(h, (int64_t)n_nodes * L::DX * 4);
  const __amdgpu_buffer_rsrc_t Ro = rsrc_bytes(out, L::DM * 4);
  for (int e0 = beg; e0 < end || e0 == beg; e0 += 16) {
    const bool first_tile = e0 == beg;
    int src[4];
    load_tile_edges(nbr, Y, e0, end, lane, src, ybuf);
    f32x4 h2[4];
    {
      MlpT m;
      mlp_pre(R, emb, e0, end, lane, m);
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) h2[b][r] = act_fwd(m.a2[b][r]);
    }
    sfor<3>([&](auto I) {
      constexpr int MUL = iblock_mul<L, I>();
      if constexpr (MUL > 0) {
        constexpr int D1 = 2 * I + 1;
        constexpr int XOFF = iblock_xoff<L, I>();
        for (int j = 0; j < MUL / 16; ++j) {
          const int u = 16 * j + col;
          float x[4][D1];
          phase();
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int i = 0; i < D1; ++i)
              x[r][i] = ldw(Rh, (src[r] * L::DX + col * D1) * 4, (XOFF + 16 * j * D1 + i) * 4);
          sfor<L::NP>([&](auto pi) {
            constexpr PathDef p = L::P[pi];
            if constexpr (p.l1 == I) {
              constexpr int D2 = 2 * p.l2 + 1, D3 = 2 * p.l3 + 1;
              phase();
              const f32x4 wv = mlp_w_block(h2, R.w2, L::W, p.woff + 16 * j, lane);
              float acc[D3];
#pragma unroll
              for (int k = 0; k < D3; ++k) acc[k] = 0.f;
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                float y[D2];
#pragma unroll
                for (int q = 0; q < D2; ++q) y[q] = ybuf[(4 * g + r) * 9 + yoff(p.l2) + q];
                tp_acc<p.l1, p.l2, p.l3>(x[r], y, wv[r], acc);  // padded edges have w = 0
              }
#pragma unroll
              for (int k = 0; k < D3; ++k) {
                float v = acc[k];
                v += __shfl_xor(v, 16, 64);
                v += __shfl_xor(v, 32, 64);
                if (g == 0) {
                  const int so = (p.moff + 16 * j * D3 + k) * 4, vo = col * D3 * 4;
                  stw(first_tile ? v / denom : ldw(Ro, vo, so) + v / denom, Ro, vo, so);
                }
              }
            }
          });
        }
      }
    });
    if (end <= beg) break;
  }
}

// ---------------------------------------------------------------- backward
// Two kernels (one fused kernel held ~250 VGPRs: 1 wave/SIMD):
//  B1 k_conv_bwd_x:  one wave per NEIGHBOUR node j over its incoming edges
//      (transposed CSR src_ptr/src_perm, ascending edge id, tiles of 16):
//      recompute w (MFMA), dE/dx[j] = sum_e TP^T_x(Y_e, w_e, g_ctr(e)) summed in
//      registers/LDS and written once (no per-edge E x 480 buffer, no gather
//      pass), and dE/du per edge.
//  B2 k_conv_bwd_w:  one wave per fixed tile of 16 consecutive edges:
//      dE/dw = TP^T_w(x_src, Y, g_ctr) (needs no w) -> LDS transpose ->
//      dH2^T = W2 dw^T (MFMA) -> MLP chain backward -> dE/demb.
// Each per-edge output is written by exactly one wave per layer (deterministic).
// In: gagg = dE/dagg / denom (row of the edge's centre).

template <int L1, int L2, int L3>
__device__ __forceinline__ void tp_bwd_x(const float* x, const float* y, float w, const float* gm,
                                         float* dx, float* dy) {
  using C = CG<L1, L2, L3>;
#pragma unroll
  for (int q = 0; q < C::n; ++q) {
    const int i = C::e[q].i, j = C::e[q].j, k = C::e[q].k;
    const float cgw = (C::e[q].c * gm[k]) * w;
    dx[i] += cgw * y[j];
    dy[j] += cgw * x[i];
  }
}
template <int L1, int L2, int L3>
__device__ __forceinline__ float tp_bwd_w(const float* x, const float* y, const float* gm) {
  using C = CG<L1, L2, L3>;
  float dwv = 0.f;
#pragma unroll
  for (int q = 0; q < C::n; ++q)
    dwv += (C::e[q].c * gm[C::e[q].k]) * (x[C::e[q].i] * y[C::e[q].j]);
  return dwv;
}

template <class L>
__global__ __launch_bounds__(256) void k_conv_bwd_x(const int* __restrict__ src_ptr,
                                                    const int* __restrict__ src_perm,
                                                    const int* __restrict__ center,
                                                    const float* __restrict__ emb,
                                                    const float* __restrict__ Y,
                                                    const float* __restrict__ h,
                                                    const float* __restrict__ gagg, MlpW W,
                                                    float* __restrict__ dh,
                                                    float* __restrict__ dgu, int n_nodes,
                                                    int n_centers) {
  // per wave: Y of the tile [16][9] and the dE/dx[j] partials [DX/16][64 lanes]
  constexpr int NACC = L::DX / 16;
  __shared__ float lds[4][160 + NACC * 64];
  const int wid = threadIdx.x >> 6;
  const int jn = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + wid);
  if (jn >= n_nodes) return;
  float* ybuf = lds[wid];
  float* dacc = lds[wid] + 160;
  const int lane = threadIdx.x & 63, g = lane >> 4, col = lane & 15;
  const int qb = src_ptr[jn], qe = src_ptr[jn + 1];
  const WRes R = make_wres(W, L::W);
  const float* hj = h + (int64_t)jn * L::DX;
  // dE/dagg rows through a descriptor: 32-bit lane offsets (the host checks
  // n_centers * DM * 4 < 2^31), scalar path/channel offsets
  const __amdgpu_buffer_rsrc_t Rg = rsrc_bytes(gagg, (int64_t)n_centers * L::DM * 4);
#pragma unroll
  for (int q = 0; q < NACC; ++q) dacc[q * 64 + lane] = 0.f;

  for (int q0 = qb; q0 < qe; q0 += 16) {
    phase();
    int er[4], vg[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = q0 + 4 * g + r;
      er[r] = q < qe ? src_perm[q] : -1;
      // padded slots read past the end of the descriptor: 0
      vg[r] = (er[r] >= 0 ? center[er[r]] * L::DM : n_centers * L::DM) * 4;
    }
#pragma unroll
    for (int t0 = 0; t0 < 144; t0 += 64) {
      const int t = t0 + lane;
      if (t < 144) {
        const int q = q0 + t / 9;
        ybuf[t] = q < qe ? Y[(int64_t)src_perm[q] * 9 + t % 9] : 0.f;
      }
    }
    f32x4 h2[4];
    {
      const int ec = (q0 + col < qe) ? src_perm[q0 + col] : -1;  // edge of slot `col`
      float b[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) b[s] = ec >= 0 ? emb[(int64_t)ec * 8 + 4 * s + g] : 0.f;
      MlpT m;
      mlp_chain(R, b, lane, m);
#pragma unroll
      for (int bb = 0; bb < 4; ++bb)
#pragma unroll
        for (int r = 0; r < 4; ++r) h2[bb][r] = act_fwd(m.a2[bb][r]);
    }
    // dE/dY (components 1..8; Y_0 is constant) per edge slot, over this lane's channels
    float dYa[4][8];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int q = 0; q < 8; ++q) dYa[r][q] = 0.f;

    sfor<3>([&](auto I) {
      constexpr int MUL = iblock_mul<L, I>();
      if constexpr (MUL > 0) {
        constexpr int D1 = 2 * I + 1;
        constexpr int XOFF = iblock_xoff<L, I>();
        for (int jj = 0; jj < MUL / 16; ++jj) {
          const int u = 16 * jj + col;
          float x[D1], dx[D1];
          phase();
#pragma unroll
          for (int i = 0; i < D1; ++i) {
            x[i] = hj[XOFF + u * D1 + i];
            dx[i] = 0.f;
          }
          sfor<L::NP>([&](auto pi) {
            constexpr PathDef p = L::P[pi];
            if constexpr (p.l1 == I) {
              constexpr int D2 = 2 * p.l2 + 1, D3 = 2 * p.l3 + 1;
              phase();
              const f32x4 wv = mlp_w_block(h2, R.w2, L::W, p.woff + 16 * jj, lane);
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float* yr = ybuf + (4 * g + r) * 9;
                float y[D2], dy[D2], gm[D3];
#pragma unroll
                for (int k = 0; k < D3; ++k)
                  gm[k] = ldw(Rg, vg[r] + col * D3 * 4, (p.moff + 16 * jj * D3 + k) * 4);
#pragma unroll
                for (int q = 0; q < D2; ++q) {
                  y[q] = yr[yoff(p.l2) + q];
                  dy[q] = 0.f;
                }
                tp_bwd_x<p.l1, p.l2, p.l3>(x, y, wv[r], gm, dx, dy);
                if constexpr (p.l2 > 0) {
#pragma unroll
                  for (int q = 0; q < D2; ++q) dYa[r][yoff(p.l2) - 1 + q] += dy[q];
                }
              }
            }
          });
#pragma unroll
          for (int i = 0; i < D1; ++i) dacc[(XOFF / 16 + jj * D1 + i) * 64 + lane] += dx[i];
        }
      }
    });

    phase();
    // dE/dY: sum over the 16 channel lanes of each lane group (fixed tree), then
    // dE/du through the SH polynomials (serial_code.py:50-70), once per edge
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float v = dYa[r][q];
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        dYa[r][q] = v;
      }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (col == r && er[r] >= 0) {
        const float* yr = ybuf + (4 * g + r) * 9;
        const float s3 = 1.7320508075688772f, s5 = 2.23606797749979f, c15 = s3 * s5;
        const float ux = yr[1] / s3, uy = yr[2] / s3, uz = yr[3] / s3;
        const float* d = dYa[r];  // d[0..2] = dE/dY_1, d[3..7] = dE/dY_2
        const float gx = s3 * d[0] + c15 * (uz * d[3] + uy * d[4]) - s5 * ux * d[5] - c15 * ux * d[7];
        const float gy = s3 * d[1] + c15 * (ux * d[4] + uz * d[6]) + 2.f * s5 * uy * d[5];
        const float gz = s3 * d[2] + c15 * (ux * d[3] + uy * d[6]) - s5 * uz * d[5] + c15 * uz * d[7];
        float* o = dgu + (int64_t)er[r] * 3;
        o[0] += gx;
        o[1] += gy;
        o[2] += gz;
      }
    }
  }
  // dE/dx[j]: the 4 lane groups hold the same channels for different edges
  phase();
  float* dhj = dh + (int64_t)jn * L::DX;
  sfor<3>([&](auto I) {
    constexpr int MUL = iblock_mul<L, I>();
    if constexpr (MUL > 0) {
      constexpr int D1 = 2 * I + 1;
      constexpr int XOFF = iblock_xoff<L, I>();
      for (int jj = 0; jj < MUL / 16; ++jj)
#pragma unroll
        for (int i = 0; i < D1; ++i) {
          float v = dacc[(XOFF / 16 + jj * D1 + i) * 64 + lane];
          v += __shfl_xor(v, 16, 64);
          v += __shfl_xor(v, 32, 64);
          if (g == 0) dhj[XOFF + (16 * jj + col) * D1 + i] = v;
        }
    }
  });
}

template <class L>
__global__ __launch_bounds__(256) void k_conv_bwd_w(const int* __restrict__ center,
                                                    const int* __restrict__ nbr,
                                                    const float* __restrict__ emb,
                                                    const float* __restrict__ Y,
                                                    const float* __restrict__ h,
                                                    const float* __restrict__ gagg, MlpW W,
                                                    float* __restrict__ demb, int n_edges,
                                                    int n_nodes, int n_centers) {
  // per wave: dw transpose tile [16 slots][17] + Y of the tile [16][9]
  __shared__ float lds[4][16 * 17 + 160];
  const int wid = threadIdx.x >> 6;
  const int e0 = __builtin_amdgcn_readfirstlane((blockIdx.x * 4 + wid) * 16);
  if (e0 >= n_edges) return;
  const int end = n_edges;
  float* dwbuf = lds[wid];
  float* ybuf = lds[wid] + 16 * 17;
  const int lane = threadIdx.x & 63, g = lane >> 4, col = lane & 15;
  const WRes R = make_wres(W, L::W);
  int src[4], vg[4];
  load_tile_edges(nbr, Y, e0, end, lane, src, ybuf);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int e = e0 + 4 * g + r;
    vg[r] = (e < end ? center[e] * L::DM : n_centers * L::DM) * 4;  // padded: reads 0
  }
  const __amdgpu_buffer_rsrc_t Rh = rsrc_bytes(h, (int64_t)n_nodes * L::DX * 4);
  const __amdgpu_buffer_rsrc_t Rg = rsrc_bytes(gagg, (int64_t)n_centers * L::DM * 4);
  int vh[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) vh[r] = src[r] * L::DX * 4;
  f32x4 dh2[4] = {zero4(), zero4(), zero4(), zero4()};

  sfor<3>([&](auto I) {
    constexpr int MUL = iblock_mul<L, I>();
    if constexpr (MUL > 0) {
      constexpr int D1 = 2 * I + 1;
      constexpr int XOFF = iblock_xoff<L, I>();
      for (int jj = 0; jj < MUL / 16; ++jj) {
        const int u = 16 * jj + col;
        float x[4][D1];
        phase();
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int i = 0; i < D1; ++i)
            x[r][i] = ldw(Rh, vh[r] + col * D1 * 4, (XOFF + 16 * jj * D1 + i) * 4);
        sfor<L::NP>([&](auto pi) {
          constexpr PathDef p = L::P[pi];
          if constexpr (p.l1 == I) {
            constexpr int D2 = 2 * p.l2 + 1, D3 = 2 * p.l3 + 1;
            const int col0 = p.woff + 16 * jj;
            phase();
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float* yr = ybuf + (4 * g + r) * 9;
              float y[D2], gm[D3];
#pragma unroll
              for (int k = 0; k < D3; ++k)
                gm[k] = ldw(Rg, vg[r] + col * D3 * 4, (p.moff + 16 * jj * D3 + k) * 4);
#pragma unroll
              for (int q = 0; q < D2; ++q) y[q] = yr[yoff(p.l2) + q];
              dwbuf[(4 * g + r) * 17 + col] = tp_bwd_w<p.l1, p.l2, p.l3>(x[r], y, gm);
            }
            phase();
            // dH2^T += W2[:, col0:col0+16] dw^T  (B lane = dw[slot c][channel 4s+g])
            const int va = (g * 64 + col) * 4;  // W2T[col0 + 4s + g][16 bh + c]
#pragma unroll
            for (int bh = 0; bh < 4; ++bh) {
#pragma unroll
              for (int s = 0; s < 4; ++s)
                dh2[bh] = mfma(ldw(R.w2t, va, ((col0 + 4 * s) * 64 + 16 * bh) * 4),
                               dwbuf[col * 17 + 4 * s + g], dh2[bh]);
            }
          }
        });
      }
    }
  });

  // ---- MLP chain backward (pre-activations recomputed)
  phase();
  MlpT m;
  mlp_pre(R, emb, e0, end, lane, m);
  f32x4 da2[4], dh1[4];
#pragma unroll
  for (int bb = 0; bb < 4; ++bb)
#pragma unroll
    for (int r = 0; r < 4; ++r) da2[bb][r] = dh2[bb][r] * act_grad(m.a2[bb][r]);
  // dH1^T = W1 dA2^T  (A[i = h_in][k = h_out] = W1s[h_in][h_out])
  const int vb = (col * 64 + 4 * g) * 4;
#pragma unroll
  for (int bi = 0; bi < 4; ++bi) {
    phase();
    float a[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) a[s] = ldw(R.w1, vb, (16 * bi * 64 + KH(s)) * 4);
    f32x4 acc = zero4();
#pragma unroll
    for (int s = 0; s < 16; ++s) acc = mfma(a[s], da2[s >> 2][s & 3], acc);
    dh1[bi] = acc;
  }
  // demb^T = W0 dA1^T (rows n < 8; lanes c >= 8 read 0 outside the descriptor)
  f32x4 de = zero4();
#pragma unroll
  for (int s = 0; s < 16; ++s)
    de = mfma(ldw(R.w0, vb, KH(s) * 4), dh1[s >> 2][s & 3] * act_grad(m.a1[s >> 2][s & 3]), de);
  {
    const int e = e0 + col;
    if (g < 2 && e < end) {
#pragma unroll
      for (int r = 0; r < 4; ++r) demb[(int64_t)e * 8 + 4 * g + r] += de[r];
    }
  }
}

}  // namespace

template <class L>
static hipError_t fwd_impl(const FusedArgs& a, hipStream_t s) {
  if (a.n_centers <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_conv_fwd<L>, dim3((a.n_centers + 3) / 4), dim3(256), 0, s, a.row_ptr,
                     a.nbr, a.emb, a.Y, a.h, a.agg, a.W, a.n_centers, a.n_nodes, a.denom);
  return hipGetLastError();
}
template <class L>
static hipError_t bwd_impl(const FusedArgs& a, hipStream_t s) {
  if (a.n_nodes <= 0 || a.n_edges <= 0) return hipSuccess;
  if (a.dh)
    hipLaunchKernelGGL(k_conv_bwd_x<L>, dim3((a.n_nodes + 3) / 4), dim3(256), 0, s, a.src_ptr,
                       a.src_perm, a.center, a.emb, a.Y, a.h, a.gagg, a.W, a.dh, a.dgu,
                       a.n_nodes, a.n_centers);
  else  // first block: dE/dx of the embedding is not needed, only dE/du
    hipLaunchKernelGGL(k_conv_bwd_x<L>, dim3((a.n_nodes + 3) / 4), dim3(256), 0, s, a.src_ptr,
                       a.src_perm, a.center, a.emb, a.Y, a.h, a.gagg, a.W, a.scratch_dh, a.dgu,
                       a.n_nodes, a.n_centers);
  const int tiles = (a.n_edges + 15) / 16;
  hipLaunchKernelGGL(k_conv_bwd_w<L>, dim3((tiles + 3) / 4), dim3(256), 0, s, a.center, a.nbr,
                     a.emb, a.Y, a.h, a.gagg, a.W, a.demb, a.n_edges, a.n_nodes, a.n_centers);
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
