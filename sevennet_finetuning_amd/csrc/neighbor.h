// Launchers of neighbor.hip (device cell-list neighbour list).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace e3gnn {

constexpr int NL_MAXD = 512;  // max edges per centre (LDS sort buffer per wave)

struct NlGeom {
  double cell[9];    // rows a, b, c (periodic) or the virtual box of a cluster
  double inv[9];     // frac = (pos - origin) @ inv
  double origin[3];
  int nb[3];         // bins per dimension (bin width >= rc)
  int R[3];          // bin-image stencil half-width per dimension
  int periodic;      // 1: all three dimensions periodic; 0: isolated cluster
  double rc2;
};

hipError_t launch_nl_bin(int n, const double* pos, const NlGeom& G, int* f0, int* bin,
                         int* bin_count, int* err, hipStream_t s);
hipError_t launch_nl_place(int n, const int* bin, const int* bin_start, int* cursor,
                           int* bin_atoms, hipStream_t s);
hipError_t launch_nl_scan(int n, const int* cnt, int* out, hipStream_t s);
hipError_t launch_nl_search(bool fill, int n, const double* pos, const NlGeom& G, const int* f0,
                            const int* bin, const int* bin_start, const int* bin_atoms, int* deg,
                            const int* row_ptr, int* center, int* nbr, int* shift, float* vec,
                            int* err, hipStream_t s);

}  // namespace e3gnn
