// Generic uvu tensor product + neighbour sum on RUNTIME path tables (gfx950):
// the convolution of any nequip-family model (irreps with parity, lmax <= 2,
// any multiplicities), e.g. the reference's HfO2 example deployment.  The
// SevenNet-0 blocks keep their compile-time specialised kernels (fused.hip,
// tp.hip); this path serves every other manifest.
//
// Reference: IrrepsConvolution (sevenn/nn/convolution.py:36-123): for
// instruction p = (x irrep, filter irrep l2, output l3), channel u,
//   msg[e, moff_p + u (2 l3 + 1) + k] =
//       w[e, woff_p + u] sum_ij C_ijk h[nbr e, xoff_p + u (2 l1 + 1) + i] Y[e, yoff_p + j]
//   agg[c] = sum over the edges of centre c (edge_index[0]).
// The host flattens the instruction list into TERMS (x, y, w, m, c):
//   msg[m] += c * h[x] * Y[y] * w[w]
// and uploads four orderings of them (by m, w, x, y) so that every output
// element of the forward and of the three backward products (dE/dw, dE/dx per
// edge, dE/dY) is ONE lane's fixed-order sum: no atomics, deterministic.
// One wave per centre, its CSR edges in order; lanes over output elements.
#include "common.h"
#include "gtp.h"

namespace e3gnn {
namespace {

__global__ __launch_bounds__(256) void k_gtp_fwd(int n_centers, const int* __restrict__ row_ptr,
                                                 const int* __restrict__ nbr,
                                                 const float* __restrict__ h,
                                                 const float* __restrict__ Y,
                                                 const float* __restrict__ w, GtpTables T,
                                                 float* __restrict__ agg) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= n_centers) return;
  const int lane = threadIdx.x & 63;
  const int e0 = row_ptr[c], e1 = row_ptr[c + 1];
  for (int m = lane; m < T.dm; m += 64) {
    const int t0 = T.ptr_m[m], t1 = T.ptr_m[m + 1];
    float acc = 0.f;
    for (int e = e0; e < e1; ++e) {
      const float* hj = h + (int64_t)nbr[e] * T.dx;
      const float* ye = Y + (int64_t)e * T.dy;
      const float* we = w + (int64_t)e * T.dw;
      for (int t = t0; t < t1; ++t) {
        const GtpTerm q = T.by_m[t];
        acc += q.c * hj[q.x] * ye[q.y] * we[q.w];
      }
    }
    agg[(int64_t)c * T.dm + m] = acc;
  }
}

// per edge of the centre: dw[e] (by w), dxc[e] (by x; nullable), dY[e] (by y)
__global__ __launch_bounds__(256) void k_gtp_bwd(int n_centers, const int* __restrict__ row_ptr,
                                                 const int* __restrict__ nbr,
                                                 const float* __restrict__ h,
                                                 const float* __restrict__ Y,
                                                 const float* __restrict__ w,
                                                 const float* __restrict__ gagg, GtpTables T,
                                                 float* __restrict__ dw, float* __restrict__ dxc,
                                                 float* __restrict__ dY) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= n_centers) return;
  const int lane = threadIdx.x & 63;
  const float* g = gagg + (int64_t)c * T.dm;
  for (int e = row_ptr[c]; e < row_ptr[c + 1]; ++e) {
    const float* hj = h + (int64_t)nbr[e] * T.dx;
    const float* ye = Y + (int64_t)e * T.dy;
    const float* we = w + (int64_t)e * T.dw;
    for (int k = lane; k < T.dw; k += 64) {
      float acc = 0.f;
      for (int t = T.ptr_w[k]; t < T.ptr_w[k + 1]; ++t) {
        const GtpTerm q = T.by_w[t];
        acc += q.c * hj[q.x] * ye[q.y] * g[q.m];
      }
      dw[(int64_t)e * T.dw + k] = acc;
    }
    if (dxc) {
      for (int k = lane; k < T.dx; k += 64) {
        float acc = 0.f;
        for (int t = T.ptr_x[k]; t < T.ptr_x[k + 1]; ++t) {
          const GtpTerm q = T.by_x[t];
          acc += q.c * ye[q.y] * we[q.w] * g[q.m];
        }
        dxc[(int64_t)e * T.dx + k] = acc;
      }
    }
    for (int k = lane; k < T.dy; k += 64) {
      float acc = 0.f;
      for (int t = T.ptr_y[k]; t < T.ptr_y[k + 1]; ++t) {
        const GtpTerm q = T.by_y[t];
        acc += q.c * hj[q.x] * we[q.w] * g[q.m];
      }
      dY[(int64_t)e * T.dy + k] = acc;
    }
  }
}

}  // namespace

hipError_t launch_gtp_fwd(int n_centers, const int* row_ptr, const int* nbr, const float* h,
                          const float* Y, const float* w, const GtpTables& T, float* agg,
                          hipStream_t s) {
  if (n_centers <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_gtp_fwd, dim3((n_centers + 3) / 4), dim3(256), 0, s, n_centers, row_ptr,
                     nbr, h, Y, w, T, agg);
  return hipGetLastError();
}

hipError_t launch_gtp_bwd(int n_centers, const int* row_ptr, const int* nbr, const float* h,
                          const float* Y, const float* w, const float* gagg, const GtpTables& T,
                          float* dw, float* dxc, float* dY, hipStream_t s) {
  if (n_centers <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_gtp_bwd, dim3((n_centers + 3) / 4), dim3(256), 0, s, n_centers, row_ptr,
                     nbr, h, Y, w, gagg, T, dw, dxc, dY);
  return hipGetLastError();
}

}  // namespace e3gnn
