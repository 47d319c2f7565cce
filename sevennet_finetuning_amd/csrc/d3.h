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
  const float* cnref;   // [nt, 5] reference CN of (type, grid index), or null when the
                        // table's reference CNs are not per (element, index) (never for
                        // Grimme's data; checked at create)
};

// Atoms binned along the lattice vectors (host-sorted by bin) and the
// stencils of bin offsets that cover each cutoff sphere.
struct D3Grid {
  int nb[3];               // bins per lattice vector (1 on a non-periodic axis)
  float inv_nb[3];
  float lat[9];            // lattice rows a, b, c (bohr)
  int cull;                // skip cells whose centre is beyond rc + half diagonal
  float cull2_vdw, cull2_cn;
  const int* bin_of;       // [n] bin of each (sorted) atom
  const int* bin_start;    // [nbins + 1]
  const int* off_vdw;      // [n_off_vdw][3] bin offsets
  const int* off_cn;
  int n_off_vdw, n_off_cn;
};

// x [n] (x, y, z bohr wrapped, type as int bits; bin-sorted), type [n]; cn [n], rows [n x 8],
// c6tab [n x n] (nullable: C6 per pair-image instead) scratch; forces
// [n x 3] (eV/A, sorted order) and totals [7] (energy eV, virial
// xx,yy,zz,xy,xz,yz eV) out.
// gw [n x 10] scratch (Gaussian factors, separable path)
hipError_t launch_d3(const D3Params& p, const D3Grid& g, int n, const float4* x, const int* type,
                     double* cn, double* gw, float2* c6tab, double* rows, double* forces,
                     double* totals, hipStream_t s);

}  // namespace e3gnn
