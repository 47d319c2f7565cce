// Grouped f32 GEMM of the fine-tune step (tgemm.hip); C ABI e3gnn_gemm_grouped.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

namespace e3gnn {

// C = beta C + alpha (op(A1) op(B1) + op(A2) op(B2)); op(X) = X^T when t* is set
// (row-major storage, leading dimensions ld*); K2 = 0: no second pair
// One operand of a pair in the general layout: element (i, k) of op(A)
// (i = row m) or op(B)^T (i = column n) sits at
//   X[(i / rep) * ld + (i % rep) * rs + (k % ks) * kst + (k / ks) * sst]
// -- plain row-major / transposed matrices (rep 1, one segment), the e3nn
// irreps layout ([node][mul][2l+1]: rows (node, m), rep = 2l + 1) and K
// summed over (m, node) segments (a linear's weight gradient).
struct TgLay {
  const float* X;
  int ld, kst, sst;  // element strides (byte offsets are 32-bit: < 2 GB per operand)
  int rep, rs, ks;   // ks: rows of one K segment (the part's K: one segment)
};
struct TgProb {
  TgLay A1, B1, A2, B2;
  float* C;
  float* ws;  // split-K partial slabs [splits][M][N] (splits > 1)
  // C(m, n) = C[(m / crep) * ldc + (m % crep) * crs + n * cns]
  int64_t ldc;
  int crep, crs, cns;
  int M, N, K1, K2;   // K1, K2: whole segments (segments x ks)
  float alpha;
  int beta;
  int splits;  // requested (tg_add settles it)
  const int* kr;  // per-tile k ranges [lo1, hi1, lo2, hi2) (nullable; e3gnn_gemm_desc::krange)
  int kr_sm;      // its row-tile stride (0: per column tile)
  // set by tg_add
  int mode;   // tile shape: 0 = 64 x 64 x 16, 1 = 32 x 32 x 32 with the waves over k
  int tiles_n, tiles_mn, ksteps, tile_begin;
  int64_t red_begin;
};
constexpr int TG_MAX_PROBS = 12;
// The kernel argument.  Every workgroup first finds its problem: the
// problems' first tiles (and reduction ranges) sit in compact arrays at the
// front, read with a few wide scalar loads at once -- a loop over the
// problems' own fields (240 bytes apart) read them one dependent load at a
// time, ~5 us of kernel-argument latency per launch.
struct TgBatch {
  int tile_begin[TG_MAX_PROBS] = {};
  int nprob = 0;
  int total_tiles = 0;
  int64_t red_total = 0;
  TgProb p[TG_MAX_PROBS];
};
// The fixed-order split-K reduction C = beta C + alpha sum_s ws[s] of split
// problems -- right after their GEMM launch, or deferred and batched: the
// fine-tune step's weight gradients are read only at the step's end, so one
// launch reduces all of them (k_tgemm_reduce)
struct TgRed {
  const float* ws;   // [splits][M][N]
  float* C;
  int64_t ldc;
  int crep, crs, cns;
  int M, N, splits;
  float alpha;
  int beta;
};
constexpr int TG_MAX_RED = 32;
struct TgRedBatch {
  int64_t lo[TG_MAX_RED] = {}, hi[TG_MAX_RED] = {};   // [lo, hi): the problem's outputs in the launch's grid
  int n = 0;
  int64_t total = 0;
  TgRed p[TG_MAX_RED];
};
// split count the kernel would choose for an (M x N) output with K summed rows
int tg_splits(int64_t M, int64_t N, int64_t K);
bool tg_add(TgBatch& b, TgProb p);
// reduce = false: the split problems' slabs are left for launch_tgemm_reduce
hipError_t launch_tgemm(const TgBatch& b, hipStream_t s, bool reduce = true);
bool tg_red_add(TgRedBatch& r, const TgRed& q);
hipError_t launch_tgemm_reduce(const TgRedBatch& r, hipStream_t s);

}  // namespace e3gnn
