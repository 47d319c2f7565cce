// Path tables of the three SevenNet-0 convolution kinds and the TP launch API.
//
// IrrepsConvolution.__init__ (sevenn/nn/convolution.py:72-95): for every
// (x irrep i, filter irrep l2 in 0e+1e+2e, l3 in |l1-l2|..l1+l2 with l3 <= lmax)
// one uvu instruction; weight slices in instruction order (woff); messages in
// the stable-sorted-by-l3 mid irreps (moff), convolution.py:82-87.
// These tables are re-derived from the irreps at model load (api.cpp,
// check_path_tables) and the load fails if they ever disagree.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace e3gnn {

struct PathDef {
  int l1, l2, l3, mul, xoff, woff, moff;
};

// layer 0: x = 128x0e -> mid 128x0e+128x1e+128x2e
struct LayerFirst {
  static constexpr int DX = 128, W = 384, DM = 1152, NP = 3;
  static constexpr PathDef P[NP] = {{0, 0, 0, 128, 0, 0, 0},
                                    {0, 1, 1, 128, 0, 128, 128},
                                    {0, 2, 2, 128, 0, 256, 512}};
};

// layers 1..3: x = 128x0e+64x1e+32x2e -> mid 224x0e+384x1e+352x2e
struct LayerMid {
  static constexpr int DX = 480, W = 960, DM = 3136, NP = 15;
  static constexpr PathDef P[NP] = {
      {0, 0, 0, 128, 0, 0, 0},      {0, 1, 1, 128, 0, 128, 224},  {0, 2, 2, 128, 0, 256, 1376},
      {1, 0, 1, 64, 128, 384, 608}, {1, 1, 0, 64, 128, 448, 128}, {1, 1, 1, 64, 128, 512, 800},
      {1, 1, 2, 64, 128, 576, 2016}, {1, 2, 1, 64, 128, 640, 992}, {1, 2, 2, 64, 128, 704, 2336},
      {2, 0, 2, 32, 320, 768, 2656}, {2, 1, 1, 32, 320, 800, 1184}, {2, 1, 2, 32, 320, 832, 2816},
      {2, 2, 0, 32, 320, 864, 192}, {2, 2, 1, 32, 320, 896, 1280}, {2, 2, 2, 32, 320, 928, 2976}};
};

// layer 4: x = 128x0e+64x1e+32x2e -> mid 224x0e (lmax_out = 0)
struct LayerLast {
  static constexpr int DX = 480, W = 224, DM = 224, NP = 3;
  static constexpr PathDef P[NP] = {
      {0, 0, 0, 128, 0, 0, 0}, {1, 1, 0, 64, 128, 128, 128}, {2, 2, 0, 32, 320, 192, 192}};
};

struct TpArgs {
  const int* row_ptr;  // [n_centers + 1] CSR over edges sorted by centre
  const int* nbr;      // [E] edge_index[1]
  const float* Y;      // [E, 9] spherical harmonics
  const float* w;      // [E, W] radial weights
  const float* h;      // [n_nodes, DX] features after self_interaction_1
  float* agg;          // fwd out: [n_centers, DM]
  const float* gagg;   // bwd in: dE/dagg / denominator, [n_centers, DM]
  float* dw;           // bwd out: [E, W]
  float* dxc;          // bwd out: per-edge dE/dx[nbr], [E, DX] (nullable)
  float* dYacc;        // bwd in/out: [E, 9] accumulated dE/dY
  int n_centers;
  float denom;
  int acc_out = 0;     // fwd: agg += (instead of =); bwd: dw +=
  int dy_assign = 0;   // bwd: dY = (instead of the default +=: no zeroing launch)
};

// The fine-tune step's derivatives of the trilinear agg = C(h, Y, w) along a
// tangent (h', Y', w') (train_explicit.py): one launch each instead of three
// forward / four backward ones.
//   tangent forward:  agg' (=, += with acc_out) = C(h, Y', w) + C(h, Y, w') + C(h', Y, w)
//   dual backward, cotangents (g, g') of (agg, agg'):
//     dxc  = B_h(Y, w; g) + B_h(Y', w; g') + B_h(Y, w'; g')   -> dh  (gathered)
//     dxcd = B_h(Y, w; g')                                     -> dh' (gathered)
//     dw   = B_w(h, Y; g) + B_w(h, Y'; g') + B_w(h', Y; g')
//     dwd  = B_w(h, Y; g')
// h' may be null (the first block's input has no tangent): its terms vanish.
struct TpDualArgs {
  const int* row_ptr;
  const int* nbr;
  const float *Y, *Yd, *w, *wd, *h, *hd;
  float* agg;                  // tangent forward out [n_centers, DM]
  const float *g, *gd;         // dual backward in [n_centers, DM]
  float *dw, *dwd;             // [E, W]
  float *dxc, *dxcd;           // [E, DX] (dxcd null when hd is)
  int n_centers;
  int acc_out = 0;
};

hipError_t launch_tp_fwd(int kind, const TpArgs& a, hipStream_t s);
hipError_t launch_tp_fwd_tan(int kind, const TpDualArgs& a, hipStream_t s);
hipError_t launch_tp_bwd_dual(int kind, const TpDualArgs& a, hipStream_t s);
hipError_t launch_tp_bwd(int kind, const TpArgs& a, hipStream_t s);

}  // namespace e3gnn
