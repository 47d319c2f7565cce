// Launch API of the generic (runtime path table) tensor-product kernels (gtp.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace e3gnn {

// one coupling term: msg[m] += c * h[x] * Y[y] * w[w]
struct GtpTerm {
  int x, y, w, m;
  float c;
};

// device tables: the same terms in four orders, CSR by the output they feed
struct GtpTables {
  int dx, dy, dw, dm;
  const GtpTerm* by_m;
  const int* ptr_m;  // [dm + 1]
  const GtpTerm* by_w;
  const int* ptr_w;  // [dw + 1]
  const GtpTerm* by_x;
  const int* ptr_x;  // [dx + 1]
  const GtpTerm* by_y;
  const int* ptr_y;  // [dy + 1]
};

// agg[c] = sum over the CSR edges of centre c (raw, no denominator)
hipError_t launch_gtp_fwd(int n_centers, const int* row_ptr, const int* nbr, const float* h,
                          const float* Y, const float* w, const GtpTables& T, float* agg,
                          hipStream_t s);
// per edge: dw, dxc (nullable: per-edge dE/dh rows for the transposed-CSR
// gather), dY -- all overwritten
hipError_t launch_gtp_bwd(int n_centers, const int* row_ptr, const int* nbr, const float* h,
                          const float* Y, const float* w, const float* gagg, const GtpTables& T,
                          float* dw, float* dxc, float* dY, hipStream_t s);

}  // namespace e3gnn
