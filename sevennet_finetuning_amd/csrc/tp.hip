// uvu Clebsch-Gordan tensor product + neighbor segmented sum (forward) and its
// input-gradient backward, gfx950.
//
// Reference: IrrepsConvolution.forward (sevenn/nn/convolution.py:104-123):
//   msg[e] = TP(x[edge_index[1][e]], Y[e], w[e])      (e3nn uvu, per-edge weights)
//   agg[i] = sum_{e: edge_index[0][e] == i} msg[e] / denominator   (message_gather :19-32)
// with instruction order / sorted mid layout of convolution.py:72-95 (see the
// path tables below; the weight slice of path p is w[e, woff + u], its message
// slot mid[moff + u*(2*l3+1) + k]).
//
// Layout & mapping.  Edges are CSR-sorted by centre.  One wave owns one centre
// (deterministic, no atomics): it walks the centre's edges in order, gathers the
// neighbour row of the node features, and keeps the centre's message sums in
// registers, lane = channel u (128-multiplicity block: 2 channels per lane;
// 32-multiplicity block: the two half-waves take alternate edges).
// The backward (gradients w.r.t. w, Y and the gathered x) is the transposed
// contraction with the same mapping; d/dx is written per edge (dxc) and summed
// per neighbour by the transposed-CSR gather in node.hip (deterministic).
#include "common.h"
#include "cg_tables.h"
#include "tp.h"

#include <algorithm>

#include <type_traits>
#include <utility>

namespace e3gnn {
namespace {

template <int N, int I = 0, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, I + 1>(f);
  }
}

constexpr int yoff(int l) { return l == 0 ? 0 : (l == 1 ? 1 : 4); }

template <class L, int L1>
constexpr int part_mul() {
  for (int p = 0; p < L::NP; ++p)
    if (L::P[p].l1 == L1) return L::P[p].mul;
  return 0;
}
template <class L, int L1>
constexpr int part_xoff() {
  for (int p = 0; p < L::NP; ++p)
    if (L::P[p].l1 == L1) return L::P[p].xoff;
  return 0;
}

// acc[k] += w * sum_ij C[i][j][k] x[i] y[j]
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

// ------------------------------------------------------------------ forward
// edges beg + k0 * STEP, beg + (k0 + ks) * STEP, ... of the centre (ks waves
// share a centre's edges in the split kernel; 0 / 1 otherwise); out[] = sum * scale
template <class L, int L1>
__device__ __forceinline__ void fwd_part(int lane, int beg, int end, const int* __restrict__ nbr,
                                         const float* __restrict__ Y, const float* __restrict__ w,
                                         const float* __restrict__ h, float* __restrict__ out,
                                         float scale, int k0 = 0, int ks = 1, int acc_out = 0) {
  constexpr int MUL = part_mul<L, L1>();
  if constexpr (MUL == 0) {
    return;
  } else {
    constexpr int D1 = 2 * L1 + 1;
    constexpr int XOFF = part_xoff<L, L1>();
    constexpr bool PAIR = MUL == 32;
    constexpr int UPL = MUL == 128 ? 2 : 1;
    float acc[L::NP][UPL][5];
    static_for<L::NP>([&](auto pi) {
#pragma unroll
      for (int s = 0; s < UPL; ++s)
#pragma unroll
        for (int k = 0; k < 5; ++k) acc[pi][s][k] = 0.f;
    });
    const int u0 = PAIR ? (lane & 31) : lane;
    constexpr int STEP = PAIR ? 2 : 1;
    for (int e0 = beg + k0 * STEP; e0 < end; e0 += STEP * ks) {
      const int e = PAIR ? e0 + (lane >> 5) : e0;
      if (PAIR && e >= end) continue;
      const int j = nbr[e];
      float y[9];
#pragma unroll
      for (int q = 0; q < 9; ++q) y[q] = Y[(int64_t)e * 9 + q];
      const float* wr = w + (int64_t)e * L::W;
      const float* hr = h + (int64_t)j * L::DX + XOFF;
#pragma unroll
      for (int s = 0; s < UPL; ++s) {
        const int u = u0 + 64 * s;
        float x[D1];
#pragma unroll
        for (int i = 0; i < D1; ++i) x[i] = hr[u * D1 + i];
        static_for<L::NP>([&](auto pi) {
          constexpr PathDef p = L::P[pi];
          if constexpr (p.l1 == L1) {
            tp_acc<p.l1, p.l2, p.l3>(x, y + yoff(p.l2), wr[p.woff + u], acc[pi][s]);
          }
        });
      }
    }
    static_for<L::NP>([&](auto pi) {
      constexpr PathDef p = L::P[pi];
      if constexpr (p.l1 == L1) {
        constexpr int D3 = 2 * p.l3 + 1;
#pragma unroll
        for (int s = 0; s < UPL; ++s) {
#pragma unroll
          for (int k = 0; k < D3; ++k) {
            float v = acc[pi][s][k];
            if (PAIR) v += __shfl_down(v, 32, 64);
            if (!PAIR || lane < 32) {
              float* o = out + p.moff + (u0 + 64 * s) * D3 + k;
              *o = acc_out ? *o + v * scale : v * scale;
            }
          }
        }
      }
    });
  }
}

template <class L>
__global__ __launch_bounds__(192) void k_tp_fwd(const int* __restrict__ row_ptr,
                                                const int* __restrict__ nbr,
                                                const float* __restrict__ Y,
                                                const float* __restrict__ w,
                                                const float* __restrict__ h,
                                                float* __restrict__ agg, int n_centers,
                                                float denom, int acc_out) {
  // one workgroup per centre, one wave per input irrep (its paths write
  // disjoint message slots): 3x the waves of a wave-per-centre mapping, which
  // matters for the small batched graphs of the fine-tune step
  const int c = blockIdx.x;
  if (c >= n_centers) return;
  const int part = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int beg = row_ptr[c], end = row_ptr[c + 1];
  float* out = agg + (int64_t)c * L::DM;
  const float sc = 1.f / denom;
  if (part == 0) fwd_part<L, 0>(lane, beg, end, nbr, Y, w, h, out, sc, 0, 1, acc_out);
  else if (part == 1) fwd_part<L, 1>(lane, beg, end, nbr, Y, w, h, out, sc, 0, 1, acc_out);
  else fwd_part<L, 2>(lane, beg, end, nbr, Y, w, h, out, sc, 0, 1, acc_out);
}

// Small batches (the fine-tune step: a few hundred centres): FS waves per
// input irrep share a centre's edges (wave k takes edges k, k + FS, ...), each
// writes its partial message row to LDS, and the row is summed over k in a
// fixed order (deterministic): 3 FS waves per centre instead of 3.
constexpr int FS = 4;
template <class L>
__global__ __launch_bounds__(192 * FS) void k_tp_fwd_split(const int* __restrict__ row_ptr,
                                                          const int* __restrict__ nbr,
                                                          const float* __restrict__ Y,
                                                          const float* __restrict__ w,
                                                          const float* __restrict__ h,
                                                          float* __restrict__ agg, int n_centers,
                                                          float denom, int acc_out) {
  __shared__ float red[FS][L::DM];
  const int c = blockIdx.x;
  if (c >= n_centers) return;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int part = wave % 3, k0 = wave / 3;
  const int lane = threadIdx.x & 63;
  const int beg = row_ptr[c], end = row_ptr[c + 1];
  if (part == 0) fwd_part<L, 0>(lane, beg, end, nbr, Y, w, h, red[k0], 1.f, k0, FS);
  else if (part == 1) fwd_part<L, 1>(lane, beg, end, nbr, Y, w, h, red[k0], 1.f, k0, FS);
  else fwd_part<L, 2>(lane, beg, end, nbr, Y, w, h, red[k0], 1.f, k0, FS);
  __syncthreads();
  const float sc = 1.f / denom;
  float* out = agg + (int64_t)c * L::DM;
  for (int i = threadIdx.x; i < L::DM; i += blockDim.x) {
    float v = red[0][i];
#pragma unroll
    for (int k = 1; k < FS; ++k) v += red[k][i];
    out[i] = acc_out ? out[i] + v * sc : v * sc;
  }
}

// ------------------------------------------------------------------ backward
// For path p, channel u, with gm = dE/dmsg (already / denominator):
//   T[k]  = sum_ij C x_i y_j           dw      = sum_k gm_k T_k
//   gw_k  = w gm_k
//   dx_i += sum_jk C y_j gw_k          dy_j   += sum_ik C x_i gw_k
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

template <class L, int L1>
struct BwdPart {
  static constexpr int MUL = part_mul<L, L1>();
  static constexpr int D1 = 2 * L1 + 1;
  static constexpr int XOFF = part_xoff<L, L1>();
  static constexpr int UPL = MUL == 128 ? 2 : 1;
  float g[L::NP][UPL][5];

  __device__ __forceinline__ void load(int lane, const float* __restrict__ gc) {
    if constexpr (MUL > 0) {
      const int u0 = MUL == 32 ? (lane & 31) : lane;
      static_for<L::NP>([&](auto pi) {
        constexpr PathDef p = L::P[pi];
        if constexpr (p.l1 == L1) {
          constexpr int D3 = 2 * p.l3 + 1;
#pragma unroll
          for (int s = 0; s < UPL; ++s)
#pragma unroll
            for (int k = 0; k < D3; ++k) g[pi][s][k] = gc[p.moff + (u0 + 64 * s) * D3 + k];
        }
      });
    }
  }

  __device__ __forceinline__ void edge(int lane, int64_t e, int j, const float* y,
                                       const float* __restrict__ w, const float* __restrict__ h,
                                       float* __restrict__ dw, float* __restrict__ dxc,
                                       float* dy, int acc_dw) {
    if constexpr (MUL > 0) {
      if (MUL == 32 && lane >= 32) return;
      const float* wr = w + e * L::W;
      float* dwr = dw + e * L::W;
      const float* hr = h + (int64_t)j * L::DX + XOFF;
#pragma unroll
      for (int s = 0; s < UPL; ++s) {
        const int u = lane + 64 * s;
        float x[D1], dx[D1];
#pragma unroll
        for (int i = 0; i < D1; ++i) {
          x[i] = hr[u * D1 + i];
          dx[i] = 0.f;
        }
        static_for<L::NP>([&](auto pi) {
          constexpr PathDef p = L::P[pi];
          if constexpr (p.l1 == L1) {
            const float dwv = tp_bwd<p.l1, p.l2, p.l3>(x, y + yoff(p.l2), wr[p.woff + u], g[pi][s],
                                                       dx, dy + yoff(p.l2));
            dwr[p.woff + u] = acc_dw ? dwr[p.woff + u] + dwv : dwv;
          }
        });
        if (dxc) {
#pragma unroll
          for (int i = 0; i < D1; ++i) dxc[e * L::DX + XOFF + u * D1 + i] = dx[i];
        }
      }
    }
  }
};

// PL: the input irrep part this launch runs (-1: all three).  The middle
// block runs its parts as three launches (l1 = 1 and 2 need far more
// registers than l1 = 0: each launch gets its own occupancy); part 0 writes
// (or adds, per dy_assign) the edge's dE/dY partial, parts 1 and 2 add theirs
// in that order (one writer per edge per launch: deterministic)
template <class L, int PL>
__global__ __launch_bounds__(256) void k_tp_bwd(const int* __restrict__ row_ptr,
                                                const int* __restrict__ nbr,
                                                const float* __restrict__ Y,
                                                const float* __restrict__ w,
                                                const float* __restrict__ h,
                                                const float* __restrict__ gagg,
                                                float* __restrict__ dw, float* __restrict__ dxc,
                                                float* __restrict__ dYacc, int n_centers,
                                                int split, int acc_dw, int dy_assign) {
  // `split` waves per centre, wave k taking the centre's edges k, k + split, ...
  // (every per-edge output has one writer); split > 1 only when there are few
  // centres (the fine-tune step's batches)
  const int wg = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const int c = wg / split, k0 = wg - c * split;
  if (c >= n_centers) return;
  const int lane = threadIdx.x & 63;
  const int beg = row_ptr[c], end = row_ptr[c + 1];
  const float* gc = gagg + (int64_t)c * L::DM;
  BwdPart<L, PL < 0 ? 0 : PL> pa;
  BwdPart<L, PL < 0 ? 1 : 3> pb;   // (l1 = 3: no channels, a no-op part)
  BwdPart<L, PL < 0 ? 2 : 3> pc;
  pa.load(lane, gc);
  pb.load(lane, gc);
  pc.load(lane, gc);
  const bool assign = dy_assign && PL <= 0;
  for (int e = beg + k0; e < end; e += split) {
    const int j = nbr[e];
    float y[9], dy[9];
#pragma unroll
    for (int q = 0; q < 9; ++q) {
      y[q] = Y[(int64_t)e * 9 + q];
      dy[q] = 0.f;
    }
    pa.edge(lane, e, j, y, w, h, dw, dxc, dy, acc_dw);
    pb.edge(lane, e, j, y, w, h, dw, dxc, dy, acc_dw);
    pc.edge(lane, e, j, y, w, h, dw, dxc, dy, acc_dw);
    float mine = 0.f;
#pragma unroll
    for (int q = 0; q < 9; ++q) {
      const float s = wave_sum(dy[q]);
      if (lane == q) mine = s;
    }
    if (lane < 9) {
      float* o = dYacc + (int64_t)e * 9 + lane;
      *o = assign ? mine : *o + mine;
    }
  }
}

// ------------------------------------------------------------------ dual
// Tangent forward of one input irrep part: per path
//   acc_k += w sum_ij C (x_i y'_j + x'_i y_j) + w' sum_ij C x_i y_j
template <class L, int L1>
__device__ __forceinline__ void fwd_tan_part(int lane, int beg, int end,
                                             const int* __restrict__ nbr, const TpDualArgs& a,
                                             float* __restrict__ out, int k0, int ks) {
  constexpr int MUL = part_mul<L, L1>();
  if constexpr (MUL == 0) {
    return;
  } else {
    constexpr int D1 = 2 * L1 + 1;
    constexpr int XOFF = part_xoff<L, L1>();
    constexpr bool PAIR = MUL == 32;
    constexpr int UPL = MUL == 128 ? 2 : 1;
    const bool has_xd = a.hd != nullptr;
    float acc[L::NP][UPL][5];
    static_for<L::NP>([&](auto pi) {
#pragma unroll
      for (int s = 0; s < UPL; ++s)
#pragma unroll
        for (int k = 0; k < 5; ++k) acc[pi][s][k] = 0.f;
    });
    const int u0 = PAIR ? (lane & 31) : lane;
    constexpr int STEP = PAIR ? 2 : 1;
    for (int e0 = beg + k0 * STEP; e0 < end; e0 += STEP * ks) {
      const int e = PAIR ? e0 + (lane >> 5) : e0;
      if (PAIR && e >= end) continue;
      const int j = nbr[e];
      float y[9], yd[9];
#pragma unroll
      for (int q = 0; q < 9; ++q) {
        y[q] = a.Y[(int64_t)e * 9 + q];
        yd[q] = a.Yd[(int64_t)e * 9 + q];
      }
      const float* wr = a.w + (int64_t)e * L::W;
      const float* wdr = a.wd + (int64_t)e * L::W;
#pragma unroll
      for (int s = 0; s < UPL; ++s) {
        const int u = u0 + 64 * s;
        float x[D1], xd[D1];
#pragma unroll
        for (int i = 0; i < D1; ++i) {
          x[i] = a.h[(int64_t)j * L::DX + XOFF + u * D1 + i];
          xd[i] = has_xd ? a.hd[(int64_t)j * L::DX + XOFF + u * D1 + i] : 0.f;
        }
        static_for<L::NP>([&](auto pi) {
          constexpr PathDef p = L::P[pi];
          if constexpr (p.l1 == L1) {
            using C = CG<p.l1, p.l2, p.l3>;
            constexpr int D3 = 2 * p.l3 + 1;
            const float* yy = y + yoff(p.l2);
            const float* yyd = yd + yoff(p.l2);
            float ta[D3], tb[D3];
#pragma unroll
            for (int k = 0; k < D3; ++k) ta[k] = tb[k] = 0.f;
#pragma unroll
            for (int q = 0; q < C::n; ++q) {
              const int i = C::e[q].i, jj = C::e[q].j, k = C::e[q].k;
              ta[k] += C::e[q].c * (x[i] * yyd[jj] + xd[i] * yy[jj]);
              tb[k] += C::e[q].c * (x[i] * yy[jj]);
            }
            const float wv = wr[p.woff + u], wdv = wdr[p.woff + u];
#pragma unroll
            for (int k = 0; k < D3; ++k) acc[pi][s][k] += wv * ta[k] + wdv * tb[k];
          }
        });
      }
    }
    static_for<L::NP>([&](auto pi) {
      constexpr PathDef p = L::P[pi];
      if constexpr (p.l1 == L1) {
        constexpr int D3 = 2 * p.l3 + 1;
#pragma unroll
        for (int s = 0; s < UPL; ++s) {
#pragma unroll
          for (int k = 0; k < D3; ++k) {
            float v = acc[pi][s][k];
            if (PAIR) v += __shfl_down(v, 32, 64);
            if (!PAIR || lane < 32) out[p.moff + (u0 + 64 * s) * D3 + k] = v;
          }
        }
      }
    });
  }
}

// FS waves per input irrep share a centre's edges; partial rows summed in a
// fixed order through LDS (as k_tp_fwd_split)
template <class L>
__global__ __launch_bounds__(192 * FS) void k_tp_fwd_tan(TpDualArgs a) {
  __shared__ float red[FS][L::DM];
  const int c = blockIdx.x;
  if (c >= a.n_centers) return;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int part = wave % 3, k0 = wave / 3;
  const int lane = threadIdx.x & 63;
  const int beg = a.row_ptr[c], end = a.row_ptr[c + 1];
  if (part == 0) fwd_tan_part<L, 0>(lane, beg, end, a.nbr, a, red[k0], k0, FS);
  else if (part == 1) fwd_tan_part<L, 1>(lane, beg, end, a.nbr, a, red[k0], k0, FS);
  else fwd_tan_part<L, 2>(lane, beg, end, a.nbr, a, red[k0], k0, FS);
  // (the parts' paths cover every message slot of a row: no zeroing)
  __syncthreads();
  float* out = a.agg + (int64_t)c * L::DM;
  for (int i = threadIdx.x; i < L::DM; i += blockDim.x) {
    float v = red[0][i];
#pragma unroll
    for (int k = 1; k < FS; ++k) v += red[k][i];
    out[i] = a.acc_out ? out[i] + v : v;
  }
}

// Dual backward of one input irrep part over one edge: with cg = C g_k,
// cgd = C g'_k per CG entry (i, j, k):
//   dw  += cg x_i y_j + cgd (x_i y'_j + x'_i y_j)     dwd += cgd x_i y_j
//   dx_i += w (cg y_j + cgd y'_j) + w' cgd y_j         dxd_i += w cgd y_j
// HALF: which 64 channels of a 128-channel irrep (two waves share it: one
// channel per lane, half the live cotangent registers)
template <class L, int L1, int HALF = 0>
struct DualPart {
  static constexpr int MUL = part_mul<L, L1>();
  static constexpr int D1 = 2 * L1 + 1;
  static constexpr int XOFF = part_xoff<L, L1>();
  static constexpr int UPL = 1, CB = 64 * HALF;
  static_assert(MUL <= 64 || MUL == 128, "channel blocks");
  float g[L::NP][UPL][5], gd[L::NP][UPL][5];

  __device__ __forceinline__ void load(int lane, const float* __restrict__ gc,
                                       const float* __restrict__ gdc) {
    const int u0 = (MUL == 32 ? (lane & 31) : lane) + CB;
    static_for<L::NP>([&](auto pi) {
      constexpr PathDef p = L::P[pi];
      if constexpr (p.l1 == L1) {
        constexpr int D3 = 2 * p.l3 + 1;
#pragma unroll
        for (int k = 0; k < D3; ++k) {
          g[pi][0][k] = gc[p.moff + u0 * D3 + k];
          gd[pi][0][k] = gdc[p.moff + u0 * D3 + k];
        }
      }
    });
  }

  __device__ __forceinline__ void edge(int lane, int64_t e, int j, const float* y, const float* yd,
                                       const TpDualArgs& a) {
    // (a 32-channel irrep: the two half-waves take two edges, lane = channel)
    const float* wr = a.w + e * L::W;
    const float* wdr = a.wd + e * L::W;
    const bool has_xd = a.hd != nullptr;
#pragma unroll
    for (int s = 0; s < UPL; ++s) {
      const int u = (MUL == 32 ? (lane & 31) : lane) + CB + 64 * s;
      float x[D1], xd[D1], dx[D1], dxd[D1];
#pragma unroll
      for (int i = 0; i < D1; ++i) {
        x[i] = a.h[(int64_t)j * L::DX + XOFF + u * D1 + i];
        xd[i] = has_xd ? a.hd[(int64_t)j * L::DX + XOFF + u * D1 + i] : 0.f;
        dx[i] = dxd[i] = 0.f;
      }
      static_for<L::NP>([&](auto pi) {
        constexpr PathDef p = L::P[pi];
        if constexpr (p.l1 == L1) {
          using C = CG<p.l1, p.l2, p.l3>;
          const float* yy = y + yoff(p.l2);
          const float* yyd = yd + yoff(p.l2);
          const float wv = wr[p.woff + u], wdv = wdr[p.woff + u];
          float dwv = 0.f, dwdv = 0.f;
#pragma unroll
          for (int q = 0; q < C::n; ++q) {
            const int i = C::e[q].i, jj = C::e[q].j, k = C::e[q].k;
            const float cg = C::e[q].c * g[pi][s][k], cgd = C::e[q].c * gd[pi][s][k];
            const float xy = x[i] * yy[jj];
            dwv += cg * xy + cgd * (x[i] * yyd[jj] + xd[i] * yy[jj]);
            dwdv += cgd * xy;
            dx[i] += wv * (cg * yy[jj] + cgd * yyd[jj]) + wdv * (cgd * yy[jj]);
            dxd[i] += wv * (cgd * yy[jj]);
          }
          a.dw[e * L::W + p.woff + u] = dwv;
          a.dwd[e * L::W + p.woff + u] = dwdv;
        }
      });
#pragma unroll
      for (int i = 0; i < D1; ++i) {
        a.dxc[e * L::DX + XOFF + u * D1 + i] = dx[i];
        if (a.dxcd) a.dxcd[e * L::DX + XOFF + u * D1 + i] = dxd[i];
      }
    }
  }
};

// waves per (centre, edge split): a 128-channel irrep takes two
template <class L>
constexpr int n_parts() {
  return (part_mul<L, 0>() == 128 ? 2 : (part_mul<L, 0>() > 0)) + (part_mul<L, 1>() > 0) +
         (part_mul<L, 2>() > 0);
}

// wave -> (centre, edge split k0, input irrep part): the parts write disjoint
// slices of every per-edge output, so each edge's outputs have one writer
// PSET: which parts this launch runs (-1 all; 0 the two l1 = 0 halves; 1 the
// l1 = 1 part; 2 the l1 = 2 part): the middle block's l1 >= 1 parts need
// 218 / 256 VGPRs against 80 for l1 = 0, so it runs three launches, each with
// its own register allocation (occupancy) instead of the largest one
template <class L, int PSET>
__global__ __launch_bounds__(256) void k_tp_bwd_dual(TpDualArgs a, int split) {
  constexpr int NALL = n_parts<L>();
  static_assert(part_mul<L, 0>() == 128 && part_mul<L, 1>() <= 64 && part_mul<L, 2>() <= 64 &&
                    (NALL == 2 || NALL == 4),
                "parts: l1 = 0 (two halves), then l1 = 1, 2");
  constexpr int NPART = PSET < 0 ? NALL : (PSET == 0 ? 2 : 1);
  constexpr int P0 = PSET <= 0 ? 0 : PSET + 1;  // first part of this launch
  const int wg = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const int part = P0 + wg % NPART, rest = wg / NPART;
  const int c = rest / split, k0 = rest - c * split;
  if (c >= a.n_centers) return;
  const int lane = threadIdx.x & 63;
  const int beg = a.row_ptr[c], end = a.row_ptr[c + 1];
  const float* gc = a.g + (int64_t)c * L::DM;
  const float* gdc = a.gd + (int64_t)c * L::DM;
  auto run = [&](auto& P) {
    using PT = std::remove_reference_t<decltype(P)>;
    constexpr int PAIR = PT::MUL == 32 ? 2 : 1;  // edges per wave step
    P.load(lane, gc, gdc);
    const int eoff = PAIR == 2 && lane >= 32 ? split : 0;
    for (int e0 = beg + k0; e0 < end; e0 += PAIR * split) {
      const int e = e0 + eoff;
      if (e >= end) continue;
      const int j = a.nbr[e];
      float y[9], yd[9];
#pragma unroll
      for (int q = 0; q < 9; ++q) {
        y[q] = a.Y[(int64_t)e * 9 + q];
        yd[q] = a.Yd[(int64_t)e * 9 + q];
      }
      P.edge(lane, e, j, y, yd, a);
    }
  };
  if constexpr (PSET <= 0) {
    if (part == 0) {
      DualPart<L, 0, 0> p;
      run(p);
      return;
    } else if (part == 1) {
      DualPart<L, 0, 1> p;
      run(p);
      return;
    }
  }
  if constexpr (NALL == 4 && (PSET < 0 || PSET == 1)) {
    if (part == 2) {
      DualPart<L, 1> p;
      run(p);
      return;
    }
  }
  if constexpr (NALL == 4 && (PSET < 0 || PSET == 2)) {
    if (part == 3) {
      DualPart<L, 2> p;
      run(p);
    }
  }
}

}  // namespace

template <class L>
static hipError_t tp_fwd_impl(const TpArgs& a, hipStream_t s) {
  if (a.n_centers <= 0) return hipSuccess;
  if (a.n_centers < 8192)
    hipLaunchKernelGGL(k_tp_fwd_split<L>, dim3(a.n_centers), dim3(192 * FS), 0, s, a.row_ptr, a.nbr,
                       a.Y, a.w, a.h, a.agg, a.n_centers, a.denom, a.acc_out);
  else
    hipLaunchKernelGGL(k_tp_fwd<L>, dim3(a.n_centers), dim3(192), 0, s, a.row_ptr, a.nbr, a.Y, a.w,
                       a.h, a.agg, a.n_centers, a.denom, a.acc_out);
  return hipGetLastError();
}
template <class L>
static hipError_t tp_bwd_impl(const TpArgs& a, hipStream_t s) {
  if (a.n_centers <= 0) return hipSuccess;
  // small batches (the fine-tune step: 432 centres x 28 edges) split each
  // centre's edges over up to 32 waves -- about one edge per wave, the
  // centre's dE/dagg row loaded by each: ~14k waves instead of 3.5k
  const int split = std::max(1, std::min(32, 32768 / a.n_centers));
  const int64_t waves = (int64_t)a.n_centers * split;
  const dim3 grid((unsigned)((waves + 3) / 4));
  if constexpr (std::is_same<L, LayerMid>::value) {
    hipLaunchKernelGGL((k_tp_bwd<L, 0>), grid, dim3(256), 0, s, a.row_ptr, a.nbr, a.Y, a.w, a.h, a.gagg,
                       a.dw, a.dxc, a.dYacc, a.n_centers, split, a.acc_out, a.dy_assign);
    hipLaunchKernelGGL((k_tp_bwd<L, 1>), grid, dim3(256), 0, s, a.row_ptr, a.nbr, a.Y, a.w, a.h, a.gagg,
                       a.dw, a.dxc, a.dYacc, a.n_centers, split, a.acc_out, a.dy_assign);
    hipLaunchKernelGGL((k_tp_bwd<L, 2>), grid, dim3(256), 0, s, a.row_ptr, a.nbr, a.Y, a.w, a.h, a.gagg,
                       a.dw, a.dxc, a.dYacc, a.n_centers, split, a.acc_out, a.dy_assign);
  } else {
    hipLaunchKernelGGL((k_tp_bwd<L, -1>), grid, dim3(256), 0, s, a.row_ptr, a.nbr, a.Y, a.w, a.h,
                       a.gagg, a.dw, a.dxc, a.dYacc, a.n_centers, split, a.acc_out, a.dy_assign);
  }
  return hipGetLastError();
}

template <class L>
static hipError_t tp_fwd_tan_impl(const TpDualArgs& a, hipStream_t s) {
  if (a.n_centers <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_tp_fwd_tan<L>, dim3(a.n_centers), dim3(192 * FS), 0, s, a);
  return hipGetLastError();
}
template <class L>
static hipError_t tp_bwd_dual_impl(const TpDualArgs& a, hipStream_t s) {
  if (a.n_centers <= 0) return hipSuccess;
  const int split = std::max(1, std::min(32, 32768 / a.n_centers));
  auto grid = [&](int parts) {
    return dim3((unsigned)(((int64_t)a.n_centers * split * parts + 3) / 4));
  };
  if constexpr (std::is_same<L, LayerMid>::value) {
    hipLaunchKernelGGL((k_tp_bwd_dual<L, 0>), grid(2), dim3(256), 0, s, a, split);
    hipLaunchKernelGGL((k_tp_bwd_dual<L, 1>), grid(1), dim3(256), 0, s, a, split);
    // the 32-channel part takes two edges per wave step: half the split
    const int split2 = std::max(1, split / 2);
    hipLaunchKernelGGL((k_tp_bwd_dual<L, 2>), dim3((unsigned)(((int64_t)a.n_centers * split2 + 3) / 4)),
                       dim3(256), 0, s, a, split2);
  } else {
    hipLaunchKernelGGL((k_tp_bwd_dual<L, -1>), grid(n_parts<L>()), dim3(256), 0, s, a, split);
  }
  return hipGetLastError();
}
hipError_t launch_tp_fwd_tan(int kind, const TpDualArgs& a, hipStream_t s) {
  switch (kind) {
    case 0: return tp_fwd_tan_impl<LayerFirst>(a, s);
    case 1: return tp_fwd_tan_impl<LayerMid>(a, s);
    default: return tp_fwd_tan_impl<LayerLast>(a, s);
  }
}
hipError_t launch_tp_bwd_dual(int kind, const TpDualArgs& a, hipStream_t s) {
  switch (kind) {
    case 0: return tp_bwd_dual_impl<LayerFirst>(a, s);
    case 1: return tp_bwd_dual_impl<LayerMid>(a, s);
    default: return tp_bwd_dual_impl<LayerLast>(a, s);
  }
}

hipError_t launch_tp_fwd(int kind, const TpArgs& a, hipStream_t s) {
  switch (kind) {
    case 0: return tp_fwd_impl<LayerFirst>(a, s);
    case 1: return tp_fwd_impl<LayerMid>(a, s);
    default: return tp_fwd_impl<LayerLast>(a, s);
  }
}
hipError_t launch_tp_bwd(int kind, const TpArgs& a, hipStream_t s) {
  switch (kind) {
    case 0: return tp_bwd_impl<LayerFirst>(a, s);
    case 1: return tp_bwd_impl<LayerMid>(a, s);
    default: return tp_bwd_impl<LayerLast>(a, s);
  }
}

}  // namespace e3gnn
