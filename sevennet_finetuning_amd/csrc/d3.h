// DFT-D3 dispersion kernels (d3.hip): parameters and launch.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace e3gnn {

constexpr double D3_AU_TO_ANG = 0.52917726;  // pair_d3.h:113
constexpr double D3_AU_TO_EV = 27.21138505;  // pair_d3.h:114

struct D3Params {
  int damping;          // 1 zero, 2 BJ (4 BJ-modified uses the BJ kernel, :2044-2052)
  int ntypes;
  float s6, s8, a1, a2, alp6, alp8;
  float rthr, cn_thr;   // squared cutoffs, bohr^2
  const float* rcov;    // [nt]
  const float* r2r4;    // [nt]
  const float* r0ab;    // [nt, nt] bohr
  const int* mxc;       // [nt]
  const float* c6ab;    // [nt, nt, 5, 5, 3] (C6, CN_ref_i, CN_ref_j)
};

// cn [n], rows [n x 8] scratch; forces [n x 3] (eV/A) and totals [7]
// (energy eV, virial xx,yy,zz,xy,xz,yz eV) out.  x [n x 3] bohr wrapped into
// the cell, tau_* [nt x 3] bohr translations, t0_* the index of the zero one.
hipError_t launch_d3(const D3Params& p, int n, const float* x, const int* type,
                     const float* tau_vdw, int nt_vdw, int t0_vdw, const float* tau_cn, int nt_cn,
                     int t0_cn, double* cn, double* rows, double* forces, double* totals,
                     hipStream_t s);

}  // namespace e3gnn
