// Radial MLP of the fine-tune step (train_explicit.py), whole chains per
// 16-edge row tile on f32 MFMA (v_mfma_f32_16x16x4_f32: exact f32 products).
//
// Reference: IrrepsConvolution's weight_nn (sevenn/nn/convolution.py:97-106,
// e3nn FullyConnectedNet 8 -> 64 -> 64 -> W with the normalised SiLU) and the
// derivatives the reference takes through autograd under create_graph
// (force_output.py:158-215, trainer.py:155-222).  The hand-scheduled step needs
// four row-wise chains per interaction block:
//   forward   a1 = e W0, h1 = phi(a1), a2 = h1 W1, h2 = phi(a2), w = h2 W2
//   tangent   a1' = e' W0, h1' = phi'(a1) a1', a2' = h1' W1, h2' = phi'(a2) a2', w' = h2' W2
//   reverse   h2b = wb W2^T, a2b = phi'(a2) h2b, h1b = a2b W1^T, a1b = phi'(a1) h1b,
//             eb += a1b W0^T
//   dual      the reverse of (primal, tangent) pairs: [h2b; h2b'] = [wb; wb'] W2^T,
//             (a2b, a2b') = (h2b phi' + h2b' phi'' a2', h2b' phi'), the same for
//             layer 1, [eb; eb'] += [a1b; a1b'] W0^T
// (W0, W1, W2 already carry the 1/sqrt(fan-in) of e3nn's normalisation).
// Each was three GEMM launches and two element-wise ones; the intermediate
// rows never leave the workgroup here.
//
// MFMA lane layout: A lane l = A[i = l&15][k = l>>4], B lane l = B[k = l>>4]
// [j = l&15], D lane l reg r = D[4(l>>4) + r][l&15].  The reductions over the
// long K of the reverse products take k in the order 16t + 4(l>>4) + (s&3)
// for MFMA s = 4t + (s&3), so A rows and W rows are read as float4 (the sum
// order changes, not the arithmetic).
#include <hip/hip_runtime.h>

#include <cstdint>

namespace e3gnn {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }
__device__ __forceinline__ float sig(float x) { return 1.0f / (1.0f + __expf(-x)); }
// c silu, its first and second derivatives (train_ops.hip's formulas)
__device__ __forceinline__ float phi(float x, float c) { return c * x * sig(x); }
__device__ __forceinline__ float dphi(float x, float c) {
  const float s = sig(x);
  return c * s * (1.0f + x * (1.0f - s));
}
__device__ __forceinline__ float ddphi(float x, float c) {
  const float s = sig(x);
  return c * s * (1.0f - s) * (2.0f + x * (1.0f - 2.0f * s));
}

constexpr int H = 64;        // hidden width
constexpr int LDH = H + 1;   // LDS row stride of the 16 x 64 hidden tiles

// ---- layer 2 on bf16 matrix cores, f32-grade (bf16x6): each f32 operand as
// three bf16 pieces (x = p0 + p1 + p2, 24 significant bits), the six piece
// products with i + j <= 2 accumulated in f32 smallest first (dropped terms
// below 2^-24 relative).  v_mfma_f32_16x16x32_bf16: A lane l = A[l & 15][k =
// 8 (l >> 4) + t], B lane l = B[k = 8 (l >> 4) + t][l & 15], t < 8; D as the f32
// form's.  12 MFMAs (192 cycles) per 16 x 16 x 64 block instead of 16 x 32 = 512.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// eight floats as three bf16 pieces (each the round-to-nearest-even bf16 of
// the remaining residual; two values per packed conversion)
__device__ __forceinline__ void split3(const float (&v)[8], bf16x8 (&d)[3]) {
  u32x4 w[3];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f32x2 r;
    r[0] = v[2 * q];
    r[1] = v[2 * q + 1];
#pragma unroll
    for (int pc = 0; pc < 3; ++pc) {
      const unsigned u = __builtin_bit_cast(unsigned, __builtin_convertvector(r, bf16x2));
      w[pc][q] = u;
      if (pc < 2) {
        r[0] -= __builtin_bit_cast(float, u << 16);
        r[1] -= __builtin_bit_cast(float, u & 0xffff0000u);
      }
    }
  }
#pragma unroll
  for (int pc = 0; pc < 3; ++pc) d[pc] = __builtin_bit_cast(bf16x8, w[pc]);
}
// the piece images of W2 [64][W], W * 384 bytes each:
//   img  (layer 2, w = h2 W2): per 16-column block b, k-half kb (32 hidden
//        units) and piece p, 64 lanes x 16 bytes at ((b * 2 + kb) * 3 + p) * 1024;
//        lane l: W2[32 kb + 8 (l >> 4) + i][16 b + (l & 15)], i < 8
//   imgT (the reverse chains' h2b = wb W2^T): per k group t (32 columns of W2),
//        hidden block hb and piece p at ((t * 4 + hb) * 3 + p) * 1024; lane l:
//        W2[16 hb + (l & 15)][32 t + 8 (l >> 4) + i]
struct W2Pieces {
  const float* W2[8];
  bf16x8* img[8];
  bf16x8* imgT[8];
  int W[8];
  int begin[9];   // thread ranges (64 per (block, k-half) = per (k group, hidden block))
  int n;
};
__global__ __launch_bounds__(256) void k_w2_pieces(W2Pieces a) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  int m = 0;
#pragma unroll
  for (int i = 1; i < 8; ++i) m += (i < a.n && t >= a.begin[i]) ? 1 : 0;
  if (t >= a.begin[a.n]) return;
  const int local = t - a.begin[m], lane = local & 63, bk = local >> 6;   // bk = b * 2 + kb = tq * 4 + hb
  const int b = bk >> 1, kb = bk & 1, g = lane >> 4, cl = lane & 15, W = a.W[m];
  float v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = a.W2[m][(int64_t)(32 * kb + 8 * g + i) * W + 16 * b + cl];
  bf16x8 d[3];
  split3(v, d);
#pragma unroll
  for (int p = 0; p < 3; ++p) a.img[m][(bk * 3 + p) * 64 + lane] = d[p];
  if (W % 32) return;   // (no transposed image: the reverse chains stay f32)
  const int tq = bk >> 2, hb = bk & 3;
  const float4* r = reinterpret_cast<const float4*>(a.W2[m] + (int64_t)(16 * hb + cl) * W + 32 * tq + 8 * g);
  const float4 x0 = r[0], x1 = r[1];
  const float u[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
  split3(u, d);
#pragma unroll
  for (int p = 0; p < 3; ++p) a.imgT[m][(bk * 3 + p) * 64 + lane] = d[p];
}

// forward (TAN = false) / tangent (TAN = true) chain; one workgroup per
// 16-row tile; wave w owns hidden columns 16w..16w+15 of layers 0 / 1 and the
// output column blocks w, w + 4, ... of layer 2 (its A operand, the tile's h2
// rows, held in 16 registers; each block's W2 operand loaded one block ahead).
template <bool TAN>
__global__ __launch_bounds__(256) void k_mlp_fwd(int E, int W, const float* __restrict__ emb,
                                                 const float* __restrict__ W0,
                                                 const float* __restrict__ W1,
                                                 const float* __restrict__ W2,
                                                 const float* __restrict__ A1p,
                                                 const float* __restrict__ A2p,
                                                 float* __restrict__ A1, float* __restrict__ H1,
                                                 float* __restrict__ A2, float* __restrict__ H2,
                                                 float* __restrict__ WT, float c,
                                                 const bf16x8* __restrict__ W2p) {
  __shared__ float hs[2][16 * LDH];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, cl = lane & 15;
  const int r0 = blockIdx.x * 16;
  const int hcol = 16 * w + cl;  // hidden column of this lane
  const int NB = W / 16;         // output column blocks (W % 16 == 0)
  float b1[16], b2[2][16];
#pragma unroll
  for (int s = 0; s < 16; ++s) b1[s] = W1[(4 * s + g) * H + hcol];
  auto load_b2 = [&](int blk, float(&o)[16]) __attribute__((always_inline)) {
    const int n = 16 * (blk < NB ? blk : 0) + cl;
#pragma unroll
    for (int s = 0; s < 16; ++s) o[s] = W2[(int64_t)(4 * s + g) * W + n];
  };
  if (!W2p) load_b2(w, b2[0]);
  // primal pre-activations at this lane's D positions (tangent chain)
  float p1[4], p2[4];
  if (TAN) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = r0 + 4 * g + r;
      p1[r] = row < E ? A1p[(int64_t)row * H + hcol] : 0.f;
      p2[r] = row < E ? A2p[(int64_t)row * H + hcol] : 0.f;
    }
  }
  const int arow = r0 + cl;  // A-operand row of this lane
  // layer 0: K = 8
  f32x4 acc = zero4();
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const float a = arow < E ? emb[(int64_t)arow * 8 + 4 * s + g] : 0.f;
    acc = mfma4(a, W0[(4 * s + g) * H + hcol], acc);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = r0 + 4 * g + r;
    const float h = TAN ? dphi(p1[r], c) * acc[r] : phi(acc[r], c);
    hs[0][(4 * g + r) * LDH + hcol] = h;
    if (row < E) {
      A1[(int64_t)row * H + hcol] = acc[r];
      H1[(int64_t)row * H + hcol] = h;
    }
  }
  __syncthreads();
  // layer 1: K = 64
  acc = zero4();
#pragma unroll
  for (int s = 0; s < 16; ++s) acc = mfma4(hs[0][cl * LDH + 4 * s + g], b1[s], acc);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = r0 + 4 * g + r;
    const float h = TAN ? dphi(p2[r], c) * acc[r] : phi(acc[r], c);
    hs[1][(4 * g + r) * LDH + hcol] = h;
    if (row < E) {
      A2[(int64_t)row * H + hcol] = acc[r];
      H2[(int64_t)row * H + hcol] = h;
    }
  }
  __syncthreads();
  auto store = [&](int blk, const f32x4& o) __attribute__((always_inline)) {
    const int n = 16 * blk + cl;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = r0 + 4 * g + r;
      if (row < E) WT[(int64_t)row * W + n] = o[r];
    }
  };
  if (W2p) {   // layer 2 on bf16x6 (wave-uniform)
    bf16x8 ap[2][3];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      float v[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] = hs[1][cl * LDH + 32 * kb + 8 * g + t];
      split3(v, ap[kb]);
    }
    auto load_p = [&](int blk, bf16x8 (&o)[2][3]) __attribute__((always_inline)) {
      const int b = blk < NB ? blk : 0;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int p = 0; p < 3; ++p) o[kb][p] = W2p[((b * 2 + kb) * 3 + p) * 64 + lane];
    };
    constexpr int I[6] = {2, 1, 0, 1, 0, 0}, J[6] = {0, 1, 2, 0, 1, 0};
    bf16x8 bp[2][2][3];
    load_p(w, bp[0]);
    for (int blk = w; blk < NB; blk += 8) {
      load_p(blk + 4, bp[1]);
      f32x4 o0 = zero4(), o1 = zero4();
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int q = 0; q < 6; ++q) {
          o0 = mfma16(ap[kb][I[q]], bp[0][kb][J[q]], o0);
          o1 = mfma16(ap[kb][I[q]], bp[1][kb][J[q]], o1);
        }
      load_p(blk + 8, bp[0]);
      store(blk, o0);
      if (blk + 4 < NB) store(blk + 4, o1);
    }
    return;
  }
  // layer 2: the tile's h2 rows as A operands, column blocks w, w + 4, ...
  float a2[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) a2[s] = hs[1][cl * LDH + 4 * s + g];
  // two column blocks at a time (independent accumulator chains), the next
  // pair's W2 operands loaded while this pair is multiplied
  for (int blk = w; blk < NB; blk += 8) {
    load_b2(blk + 4, b2[1]);
    f32x4 o0 = zero4(), o1 = zero4();
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      o0 = mfma4(a2[s], b2[0][s], o0);
      o1 = mfma4(a2[s], b2[1][s], o1);
    }
    if (blk + 8 < NB) load_b2(blk + 8, b2[0]);
    store(blk, o0);
    if (blk + 4 < NB) store(blk + 4, o1);
  }
}

// reverse (DUAL = false: rows [0, E) of wb) / dual (rows r and E + r of WB
// together) chain; grid: row tiles of 16; wave w owns hidden columns
// 16w..16w+15.  Outputs A2B / A1B (nullable; [E or 2E, 64]) and EB += ([E or
// 2E, 8]).
template <bool DUAL>
__global__ __launch_bounds__(256) void k_mlp_bwd(int E, int W, const float* __restrict__ WB,
                                                 const float* __restrict__ W0,
                                                 const float* __restrict__ W1,
                                                 const float* __restrict__ W2,
                                                 const float* __restrict__ A1,
                                                 const float* __restrict__ A2,
                                                 const float* __restrict__ A1d,
                                                 const float* __restrict__ A2d,
                                                 float* __restrict__ A2B, float* __restrict__ A1B,
                                                 float* __restrict__ EB, float c,
                                                 const bf16x8* __restrict__ W2pT) {
  constexpr int NS = DUAL ? 2 : 1;  // row sets: primal (and tangent)
  __shared__ float hs[NS][16 * LDH];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, cl = lane & 15;
  const int r0 = blockIdx.x * 16;
  const int hcol = 16 * w + cl;
  const int arow = r0 + cl;
  const bool aok = arow < E;
  // h2b = wb W2^T, K = W (W % 16 == 0): the four waves split the k groups
  // (t = w, w + 4, ...; 16 k each) and each forms all 64 hidden columns (four
  // independent accumulator chains per row set), the next group's float4s
  // (wb rows, W2 rows 16 hb + cl) loaded while the current one is multiplied;
  // the four partial tiles are summed through LDS in a fixed order
  __shared__ float part[4][NS][16 * LDH];
  const int T = W / 16;
  f32x4 pacc[NS][4];
#pragma unroll
  for (int q = 0; q < NS; ++q)
#pragma unroll
    for (int hb = 0; hb < 4; ++hb) pacc[q][hb] = zero4();
  const float4* wbr[NS];
#pragma unroll
  for (int q = 0; q < NS; ++q)
    wbr[q] = reinterpret_cast<const float4*>(WB + ((int64_t)q * E + (aok ? arow : 0)) * W) + g;
  const float4* w2r[4];
#pragma unroll
  for (int hb = 0; hb < 4; ++hb) w2r[hb] = reinterpret_cast<const float4*>(W2 + (int64_t)(16 * hb + cl) * W) + g;
  float4 bq[2][4], aq[2][NS];
  auto load_t = [&](int t, float4(&b)[4], float4(&a)[NS]) __attribute__((always_inline)) {
    const bool ok = t < T;
#pragma unroll
    for (int hb = 0; hb < 4; ++hb) b[hb] = ok ? w2r[hb][4 * t] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int q = 0; q < NS; ++q) a[q] = (ok && aok) ? wbr[q][4 * t] : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  auto mul_t = [&](const float4(&b)[4], const float4(&a)[NS]) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < NS; ++q)
#pragma unroll
      for (int hb = 0; hb < 4; ++hb) {
        pacc[q][hb] = mfma4(a[q].x, b[hb].x, pacc[q][hb]);
        pacc[q][hb] = mfma4(a[q].y, b[hb].y, pacc[q][hb]);
        pacc[q][hb] = mfma4(a[q].z, b[hb].z, pacc[q][hb]);
        pacc[q][hb] = mfma4(a[q].w, b[hb].w, pacc[q][hb]);
      }
  };
  if (W2pT) {   // bf16x6 (wave-uniform): k groups of 32 (W % 32 == 0), W2^T from the piece image
    const int T32 = W / 32;
    constexpr int I[6] = {2, 1, 0, 1, 0, 0}, J[6] = {0, 1, 2, 0, 1, 0};
    auto lda = [&](int t, float4 (&a)[NS][2]) __attribute__((always_inline)) {
      const bool ok = t < T32 && aok;
#pragma unroll
      for (int q = 0; q < NS; ++q)
#pragma unroll
        for (int h = 0; h < 2; ++h)
          a[q][h] = ok ? reinterpret_cast<const float4*>(WB + ((int64_t)q * E + arow) * W + 32 * t + 8 * g)[h]
                       : make_float4(0.f, 0.f, 0.f, 0.f);
    };
    float4 ar[NS][2];
    lda(w, ar);
    for (int t = w; t < T32; t += 4) {
      bf16x8 ap[NS][3];
#pragma unroll
      for (int q = 0; q < NS; ++q) {
        const float v[8] = {ar[q][0].x, ar[q][0].y, ar[q][0].z, ar[q][0].w,
                            ar[q][1].x, ar[q][1].y, ar[q][1].z, ar[q][1].w};
        split3(v, ap[q]);
      }
      lda(t + 4, ar);
#pragma unroll
      for (int hb = 0; hb < 4; ++hb) {
        bf16x8 bp[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) bp[p] = W2pT[((t * 4 + hb) * 3 + p) * 64 + lane];
#pragma unroll
        for (int q = 0; q < NS; ++q)
#pragma unroll
          for (int j = 0; j < 6; ++j) pacc[q][hb] = mfma16(ap[q][I[j]], bp[J[j]], pacc[q][hb]);
      }
    }
  } else {
  load_t(w, bq[0], aq[0]);
  for (int t = w; t < T; t += 8) {
    load_t(t + 4, bq[1], aq[1]);
    mul_t(bq[0], aq[0]);
    if (t + 4 >= T) break;
    load_t(t + 8, bq[0], aq[0]);
    mul_t(bq[1], aq[1]);
  }
  }
#pragma unroll
  for (int q = 0; q < NS; ++q)
#pragma unroll
    for (int hb = 0; hb < 4; ++hb)
#pragma unroll
      for (int r = 0; r < 4; ++r) part[w][q][(4 * g + r) * LDH + 16 * hb + cl] = pacc[q][hb][r];
  __syncthreads();
  f32x4 acc[NS];
#pragma unroll
  for (int q = 0; q < NS; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o = (4 * g + r) * LDH + hcol;
      acc[q][r] = ((part[0][q][o] + part[1][q][o]) + part[2][q][o]) + part[3][q][o];
    }
  // through phi at a2 (and the dual pair)
  auto through = [&](const float* __restrict__ X, const float* __restrict__ Xd, float* __restrict__ OUT,
                     int lds) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = r0 + 4 * g + r;
      const bool ok = row < E;
      const float x = ok ? X[(int64_t)row * H + hcol] : 0.f;
      float o0, o1 = 0.f;
      if (DUAL) {
        const float xd = ok ? Xd[(int64_t)row * H + hcol] : 0.f;
        const float d1 = dphi(x, c);
        o0 = acc[0][r] * d1 + acc[NS - 1][r] * ddphi(x, c) * xd;
        o1 = acc[NS - 1][r] * d1;
      } else {
        o0 = acc[0][r] * dphi(x, c);
      }
      hs[0][(4 * g + r) * LDH + hcol] = o0;
      if (DUAL) hs[NS - 1][(4 * g + r) * LDH + hcol] = o1;
      if (OUT && ok) {
        OUT[(int64_t)row * H + hcol] = o0;
        if (DUAL) OUT[((int64_t)E + row) * H + hcol] = o1;
      }
    }
    (void)lds;
  };
  through(A2, A2d, A2B, 0);
  __syncthreads();
  // h1b = a2b W1^T: K = 64 (W1 row hcol as float4 over k)
#pragma unroll
  for (int q = 0; q < NS; ++q) acc[q] = zero4();
  const float4* w1r = reinterpret_cast<const float4*>(W1 + (int64_t)hcol * H) + g;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const float4 b = w1r[4 * t];
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      const float* hr = &hs[q][cl * LDH + 16 * t + 4 * g];
      acc[q] = mfma4(hr[0], b.x, acc[q]);
      acc[q] = mfma4(hr[1], b.y, acc[q]);
      acc[q] = mfma4(hr[2], b.z, acc[q]);
      acc[q] = mfma4(hr[3], b.w, acc[q]);
    }
  }
  __syncthreads();  // every wave has read a2b
  through(A1, A1d, A1B, 0);
  __syncthreads();
  // eb += a1b W0^T: 8 output columns, one wave; lanes with cl >= 8 idle in B
  if (w == 0) {
#pragma unroll
    for (int q = 0; q < NS; ++q) acc[q] = zero4();
    const float4* w0r = reinterpret_cast<const float4*>(W0 + (int64_t)(cl < 8 ? cl : 0) * H) + g;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float4 b = w0r[4 * t];
      if (cl >= 8) b = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int q = 0; q < NS; ++q) {
        const float* hr = &hs[q][cl * LDH + 16 * t + 4 * g];
        acc[q] = mfma4(hr[0], b.x, acc[q]);
        acc[q] = mfma4(hr[1], b.y, acc[q]);
        acc[q] = mfma4(hr[2], b.z, acc[q]);
        acc[q] = mfma4(hr[3], b.w, acc[q]);
      }
    }
    if (cl < 8) {
#pragma unroll
      for (int q = 0; q < NS; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = r0 + 4 * g + r;
          if (row < E) {
            float* o = EB + ((int64_t)q * E + row) * 8 + cl;
            *o += acc[q][r];
          }
        }
    }
  }
}

}  // namespace

// W0 [8, 64], W1 [64, 64], W2 [64, W] row-major; rows of 8 / 64 / W floats.
// Tangent chain when A1p / A2p (the primal pre-activations) are given.
hipError_t launch_mlp_fwd(int E, int W, const float* emb, const float* W0, const float* W1,
                          const float* W2, const float* A1p, const float* A2p, float* A1, float* H1,
                          float* A2, float* H2, float* WT, float c, hipStream_t s, const void* W2p) {
  if (E <= 0) return hipSuccess;
  const dim3 grid((E + 15) / 16);
  const bf16x8* p = reinterpret_cast<const bf16x8*>(W2p);
  if (A1p)
    hipLaunchKernelGGL(k_mlp_fwd<true>, grid, dim3(256), 0, s, E, W, emb, W0, W1, W2, A1p, A2p, A1, H1,
                       A2, H2, WT, c, p);
  else
    hipLaunchKernelGGL(k_mlp_fwd<false>, grid, dim3(256), 0, s, E, W, emb, W0, W1, W2, A1p, A2p, A1,
                       H1, A2, H2, WT, c, p);
  return hipGetLastError();
}
int64_t mlp_w2_piece_bytes(int W) { return 2 * (int64_t)W * 384; }   // img, then imgT
hipError_t launch_mlp_w2_pieces(int n, const float* const* W2, const int* W, void* const* img, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (n > 8) return hipErrorInvalidValue;
  W2Pieces a{};
  a.n = n;
  a.begin[0] = 0;
  for (int i = 0; i < n; ++i) {
    if (W[i] <= 0 || W[i] % 16) return hipErrorInvalidValue;
    a.W2[i] = W2[i];
    a.img[i] = reinterpret_cast<bf16x8*>(img[i]);
    a.imgT[i] = reinterpret_cast<bf16x8*>(reinterpret_cast<char*>(img[i]) + (int64_t)W[i] * 384);
    a.W[i] = W[i];
    a.begin[i + 1] = a.begin[i] + (W[i] / 16) * 2 * 64;
  }
  hipLaunchKernelGGL(k_w2_pieces, dim3((a.begin[n] + 255) / 256), dim3(256), 0, s, a);
  return hipGetLastError();
}
// W % 16 == 0; dual when A1d / A2d (tangent pre-activations) are given: WB,
// A2B, A1B, EB then hold 2E rows (primal first)
hipError_t launch_mlp_bwd(int E, int W, const float* WB, const float* W0, const float* W1,
                          const float* W2, const float* A1, const float* A2, const float* A1d,
                          const float* A2d, float* A2B, float* A1B, float* EB, float c,
                          hipStream_t s, const void* W2p) {
  if (E <= 0) return hipSuccess;
  const dim3 grid((E + 15) / 16);
  // the transposed image follows the forward one (W * 384 bytes each, W2Pieces)
  const bf16x8* pT = (W2p && W % 32 == 0)
                         ? reinterpret_cast<const bf16x8*>(reinterpret_cast<const char*>(W2p) + (int64_t)W * 384)
                         : nullptr;
  if (A1d)
    hipLaunchKernelGGL(k_mlp_bwd<true>, grid, dim3(256), 0, s, E, W, WB, W0, W1, W2, A1, A2, A1d, A2d,
                       A2B, A1B, EB, c, pT);
  else
    hipLaunchKernelGGL(k_mlp_bwd<false>, grid, dim3(256), 0, s, E, W, WB, W0, W1, W2, A1, A2, A1d,
                       A2d, A2B, A1B, EB, c, pT);
  return hipGetLastError();
}

}  // namespace e3gnn
