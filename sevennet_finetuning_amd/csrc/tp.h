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

// The three block kinds of the SevenNet-0-shaped family (lmax 2, even
// parity), templated on the channel multiplicities: the first block's input
// A x0e; the middle blocks' input and output C0x0e+C1x1e+C2x2e; the last
// block's input the same, output l3 = 0 only.  Instruction order (woff) and the
// stable-by-l3 mid slots (moff) follow convolution.py:72-95 / :82-87.
// KIND: 0 first, 1 middle, 2 last.
template <int A>
struct LayerFirstT {
  static constexpr int KIND = 0, C0 = A;
  static constexpr int DX = A, W = 3 * A, DM = 9 * A, NP = 3;
  static constexpr PathDef P[NP] = {{0, 0, 0, A, 0, 0, 0}, {0, 1, 1, A, 0, A, A}, {0, 2, 2, A, 0, 2 * A, 4 * A}};
};

template <int C0_, int C1, int C2>
struct LayerMidT {
  static constexpr int KIND = 1, C0 = C0_;
  static constexpr int X1 = C0_, X2 = C0_ + 3 * C1;            // x offsets of 1e, 2e
  static constexpr int DX = C0_ + 3 * C1 + 5 * C2;
  static constexpr int W = 3 * C0_ + 6 * C1 + 6 * C2;
  static constexpr int M0 = C0_ + C1 + C2;                      // 0e mid channels
  static constexpr int B1 = M0, B2 = M0 + 3 * (C0_ + 3 * C1 + 2 * C2);  // 1e / 2e mid bases
  static constexpr int DM = B2 + 5 * (C0_ + 2 * C1 + 3 * C2);
  static constexpr int NP = 15;
  static constexpr int V = 3 * C0_ + 6 * C1;                    // woff of the first l1 = 2 path
  static constexpr PathDef P[NP] = {
      {0, 0, 0, C0_, 0, 0, 0},
      {0, 1, 1, C0_, 0, C0_, B1},
      {0, 2, 2, C0_, 0, 2 * C0_, B2},
      {1, 0, 1, C1, X1, 3 * C0_, B1 + 3 * C0_},
      {1, 1, 0, C1, X1, 3 * C0_ + C1, C0_},
      {1, 1, 1, C1, X1, 3 * C0_ + 2 * C1, B1 + 3 * C0_ + 3 * C1},
      {1, 1, 2, C1, X1, 3 * C0_ + 3 * C1, B2 + 5 * C0_},
      {1, 2, 1, C1, X1, 3 * C0_ + 4 * C1, B1 + 3 * C0_ + 6 * C1},
      {1, 2, 2, C1, X1, 3 * C0_ + 5 * C1, B2 + 5 * C0_ + 5 * C1},
      {2, 0, 2, C2, X2, V, B2 + 5 * C0_ + 10 * C1},
      {2, 1, 1, C2, X2, V + C2, B1 + 3 * C0_ + 9 * C1},
      {2, 1, 2, C2, X2, V + 2 * C2, B2 + 5 * C0_ + 10 * C1 + 5 * C2},
      {2, 2, 0, C2, X2, V + 3 * C2, C0_ + C1},
      {2, 2, 1, C2, X2, V + 4 * C2, B1 + 3 * C0_ + 9 * C1 + 3 * C2},
      {2, 2, 2, C2, X2, V + 5 * C2, B2 + 5 * C0_ + 10 * C1 + 10 * C2}};
};

template <int C0_, int C1, int C2>
struct LayerLastT {
  static constexpr int KIND = 2, C0 = C0_;
  static constexpr int DX = C0_ + 3 * C1 + 5 * C2, W = C0_ + C1 + C2, DM = W, NP = 3;
  static constexpr PathDef P[NP] = {
      {0, 0, 0, C0_, 0, 0, 0}, {1, 1, 0, C1, C0_, C0_, C0_}, {2, 2, 0, C2, C0_ + 3 * C1, C0_ + C1, C0_ + C1}};
};

// Compiled channel families.  A kernel KIND CODE is 3 * family + KIND.
//   0: SevenNet-0 (128x0e -> 128x0e+64x1e+32x2e -> ... -> 128x0e)
//   1: uniform 64 (model_build channel 64: 64x0e -> 64x0e+64x1e+64x2e -> ... -> 64x0e)
//   2: uniform 32 (channel 32, the reference's base preset width)
template <int F>
struct Family;
template <>
struct Family<0> {
  using First = LayerFirstT<128>;
  using Mid = LayerMidT<128, 64, 32>;
  using Last = LayerLastT<128, 64, 32>;
};
template <>
struct Family<1> {
  using First = LayerFirstT<64>;
  using Mid = LayerMidT<64, 64, 64>;
  using Last = LayerLastT<64, 64, 64>;
};
template <>
struct Family<2> {
  using First = LayerFirstT<32>;
  using Mid = LayerMidT<32, 32, 32>;
  using Last = LayerLastT<32, 32, 32>;
};
constexpr int N_FAMILIES = 3;

// SevenNet-0's kinds (the training ops and the v1 kernels serve these only)
using LayerFirst = Family<0>::First;
using LayerMid = Family<0>::Mid;
using LayerLast = Family<0>::Last;
static_assert(LayerMid::DX == 480 && LayerMid::W == 960 && LayerMid::DM == 3136, "SevenNet-0 middle block");
static_assert(LayerMid::P[8].moff == 2336 && LayerMid::P[13].moff == 1280 && LayerMid::P[14].woff == 928,
              "SevenNet-0 path table");
static_assert(LayerFirst::DM == 1152 && LayerLast::W == 224 && LayerLast::P[2].xoff == 320, "SevenNet-0 kinds");

// dimensions of a kind code (host; false if unknown)
bool fused_kind_dims(int code, int* dx, int* w, int* dm);
// the kind's path table (l1, l2, l3, mul, xoff, woff, moff) per path; empty if unknown
int fused_kind_paths(int code, PathDef* out, int max);
// algorithmic FLOP of one TP forward per edge of the kind (0 if unknown)
double fused_kind_tp_flops(int code);

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
