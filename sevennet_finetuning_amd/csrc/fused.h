// Launch API of the fused radial-MLP + tensor-product kernels (fused.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace e3gnn {

struct MlpW {
  const float* w0;   // [8][64]   layer0 / sqrt(8)
  const float* w1;   // [64][64]  layer1 / 8
  const float* w2;   // [64][W]   layer2 / 8
  const float* w2t;  // [W][64]   transpose of w2
  // packed operand orders (16 k-values of one lane group contiguous):
  const float* w1p;  // [n<64][g][q][t] = w1[16q + 4g + t][n]
  const float* w2p;  // [n<W][g][q][t]  = w2[16q + 4g + t][n]
  const float* w2q;  // [n/16][bh][g][c][s] = w2[16bh + c][16(n/16) + 4s + g]
  const float* w2r;  // [n/16][bh][g][c][r] = w2[16bh + c][16(n/16) + 4g + r] (fused bwd)
  // w2 as three bf16 pieces (w2 = p0 + p1 + p2, exact) in v_mfma_f32_16x16x32_bf16
  // operand order: [n/16][piece][m][g][c][t] = piece of w2[16(2m + t/4) + 4g + t%4][n]
  const uint16_t* w2b;
  // the lock-step backward's dH2 operand over PAIRS of consecutive visited
  // 16-column blocks (api.cpp bwd_w_block_cols): [pair][piece][bh][g][c][t] = piece of
  // w2[16 bh + c][col], col = channel 4g + t of the pair's first block (t < 4)
  // or 4g + t - 4 of its second
  const uint16_t* w2d;
  // w2b's column blocks in the kernels' visiting order (block k at column 16 k):
  // the software-pipelined loops fetch the operand of the block after next
  const uint16_t* w2v;
  // the radial MLP's other bf16x6 products, in w2b's operand order: W1 (layer
  // 1 forward, 64 columns), W1^T (dH1 = dA2 W1^T) and W0^T padded to 16 columns
  // (demb = dA1 W0^T)
  const uint16_t* w1b;
  const uint16_t* w1tb;
  const uint16_t* w0tb;
};

struct FusedArgs {
  const int* row_ptr;
  const int* center;  // [E] edge_index[0] (sorted)
  const int* nbr;
  const float* emb;   // [E, 8]
  const float* Y;     // [E, 9]
  const float* h;     // [n_nodes, DX]
  float* agg;         // fwd out [n_centers, DM]
  const float* gagg;  // bwd in  [n_centers, DM] (dE/dagg / denominator)
  const int* src_ptr;  // [n_nodes + 1] transposed CSR (edges by edge_index[1])
  const int* src_perm; // [E]
  float* dh;           // bwd out [n_nodes, DX]: dE/dx of the gathered features (last block)
  float* dxc;          // [E, DX] per-edge dE/dx (first / middle blocks; null: not stored)
  float* dgu;         // bwd in/out [E, 3]  dE/du accumulated over layers
  float* demb;        // bwd in/out [E, 8]  dE/demb accumulated over layers
  MlpW W;
  int n_centers;
  int n_edges;
  int n_nodes;
  float denom;
  // work range of one launch (halo overlap splits a layer into parts):
  // centres [c_begin, c_end) (forward, first / middle backward), neighbour
  // nodes [node_begin, node_end) (last backward)
  int c_begin, c_end, node_begin, node_end;
};

// `kind` is a kind code of tp.h (3 * channel family + block kind)
hipError_t launch_conv_fwd(int kind, const FusedArgs& a, hipStream_t s);
// backward of a first / middle block: the lock-step kernel (4 centres per
// workgroup, W2 operands staged per block pair in LDS, dH2 on bf16x6), per-edge
// dE/dx to dxc, dE/du, dE/dw -> dE/demb
hipError_t launch_conv_bwd_ls(int kind, const FusedArgs& a, hipStream_t s);
// backward of the last block, one wave per neighbour node: dE/dx to dh, dE/du,
// dE/dw -> dE/demb
hipError_t launch_conv_bwd_nbr_last(int kind, const FusedArgs& a, hipStream_t s);

}  // namespace e3gnn
