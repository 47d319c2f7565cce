// Fused radial-MLP + tensor-product kernels (forward and force backward), gfx950.
//
// Reference: IrrepsConvolution.forward (sevenn/nn/convolution.py:104-123):
//   w = FCN(edge_embedding)                      (e3nn FullyConnectedNet 8->64->64->W)
//   msg = TP(x[edge_index[1]], Y, w)              (uvu, convolution.py:72-95)
//   agg = scatter_sum(msg, edge_index[0]) / denominator
// and its reverse-mode pass (what ForceStressOutput obtains through autograd,
// force_output.py:74-130).  The per-edge weights w (E x 960 for the middle
// blocks) never touch HBM: f32 MFMA produces them directly in the registers the
// tensor product reads.
//
// Mapping: one wave = one centre (forward, first / middle backward) or one
// neighbour node (last backward), its edges in tiles of 16 edge slots.
//   * v_mfma_f32_16x16x4_f32: A lane l = A[i=l&15][k=l>>4], B lane l =
//     B[k=l>>4][j=l&15], D lane l reg r = D[4(l>>4)+r][l&15].  Lane group
//     g = l>>4, column c = l&15.
//   * The MLP runs transposed (H^T = W^T emb^T: rows = hidden units, columns =
//     edge slots), so every product's accumulator is the k-operand of the next
//     one; the 64 -> W layer (90 % of the MLP FLOPs) on bf16x6 MFMA (below).
//   * Forward: w = H2 W2[:, 16-column block], lane (g, c) holds w[edge 4g+r]
//     [channel c]; two tiles per pass share every W2 operand block; the
//     message is summed over registers and the 4 lane groups into the
//     centre's row in LDS.  Backward (lock-step, 4 centres per workgroup, W2
//     pieces staged per block pair in LDS): w^T recomputed, lane (g, c) =
//     edge c x channels 4g..4g+3; dE/dx per edge, dE/dY -> dE/du, dE/dw ->
//     dH2 (bf16x6 over the pair) -> MLP chain -> dE/demb.
//   * Weights via buffer descriptors (scalar k offsets, one VGPR of lane offset).
// Deterministic: no atomics; every sum has a fixed order.
#include "cg_tables.h"
#include "common.h"
#include "fused.h"
#include "tp.h"

#include <type_traits>


namespace e3gnn {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int N, int I = 0, class F>
constexpr void sfor_host(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor_host<N, I + 1>(f);
  }
}
template <int N, int I = 0, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<N, I + 1>(f);
  }
}

__device__ __forceinline__ constexpr int yoff(int l) { return l == 0 ? 0 : (l == 1 ? 1 : 4); }
// hidden unit of k-step s, lane group 0 (add 4g): 16(s>>2) + (s&3)
__device__ __forceinline__ constexpr int KH(int s) { return 16 * (s >> 2) + (s & 3); }

// Phase fence: keeps the scheduler from interleaving (and hoisting loads across)
// the MFMA chain of one column block and the tensor product of another, which
// otherwise multiplies live registers and halves occupancy.
__device__ __forceinline__ void phase() { __builtin_amdgcn_sched_barrier(0); }

// Diagnostic build only (-DE3GNN_STAMPS, never the shipped library): per-wave
// s_memtime totals of the middle backward's phases, written by lane 0 to a
// buffer of their own (e3gnn_debug_stamps) that no other code reads.
// E3GNN_STAMPS_FWD=1 (with E3GNN_STAMPS): the middle FORWARD's phases instead
#ifndef E3GNN_STAMPS_FWD
#define E3GNN_STAMPS_FWD 0
#endif
#ifdef E3GNN_STAMPS
__device__ unsigned long long* g_stamp_buf = nullptr;
#define STAMP_N 8
#define STAMP_DECL                               \
  unsigned long long st_acc[STAMP_N] = {0, 0, 0, 0, 0, 0, 0, 0}; \
  unsigned long long st_t = __builtin_amdgcn_s_memtime(), st_t0 = st_t;
#define STAMP(k)                                          \
  do {                                                    \
    const unsigned long long st_now = __builtin_amdgcn_s_memtime(); \
    st_acc[k] += st_now - st_t;                           \
    st_t = st_now;                                        \
  } while (0)
#define STAMP_FLUSH(wave)                                                   \
  do {                                                                      \
    if (g_stamp_buf && lane == 0) {                                         \
      st_acc[7] = __builtin_amdgcn_s_memtime() - st_t0;                     \
      for (int k_ = 0; k_ < STAMP_N; ++k_) g_stamp_buf[(int64_t)(wave) * STAMP_N + k_] = st_acc[k_]; \
    }                                                                       \
  } while (0)
#else
#define STAMP_DECL
#define STAMP(k) \
  do {           \
  } while (0)
#define STAMP_FLUSH(wave) \
  do {                    \
  } while (0)
#endif

// materialise a value here: stops the compiler from sinking an accumulation
// chain past later paths (which keeps every partial product live)
template <int N>
__device__ __forceinline__ void pin(float* v) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(v[i]));
}

__device__ __forceinline__ f32x4 zero4() {
  f32x4 z;
  z[0] = z[1] = z[2] = z[3] = 0.f;
  return z;
}
__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------- weight operands
// Weight operands are read through buffer descriptors: the per-lane part of the
// offset is one VGPR and the per-k-step part a scalar (soffset), so the compiler
// does not hoist hundreds of 64-bit addresses out of the centre loop (which it
// did, and spilled).  Offsets outside the descriptor read 0 (padded rows).
struct WRes {
  __amdgpu_buffer_rsrc_t w0, w2p, w2q, w2b, w2r, w2d, w2v, w1b, w1tb, w0tb;
};
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* p, int nfloats) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, nfloats * 4, 0x00020000);
}
__device__ __forceinline__ WRes make_wres(const MlpW& W, int width) {
  return {rsrc(W.w0, 8 * 64), rsrc(W.w2p, 64 * width), rsrc(W.w2q, 64 * width),
          rsrc((const float*)W.w2b, 64 * width * 3 / 2), rsrc(W.w2r, 64 * width),
          rsrc((const float*)W.w2d, 64 * width * 3 / 2),
          rsrc((const float*)W.w2v, 64 * width * 3 / 2), rsrc((const float*)W.w1b, 64 * 64 * 3 / 2),
          rsrc((const float*)W.w1tb, 64 * 64 * 3 / 2), rsrc((const float*)W.w0tb, 64 * 16 * 3 / 2)};
}
__device__ __forceinline__ float ldw(__amdgpu_buffer_rsrc_t r, int vbytes, int sbytes) {
  // the builtin returns the raw 32 bits (an unsigned int): reinterpret, never convert
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vbytes, sbytes, 0));
}

__device__ __forceinline__ f32x4 ldw4(__amdgpu_buffer_rsrc_t r, int vbytes, int sbytes) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, vbytes, sbytes, 0));
}
// N contiguous floats from one lane offset (b128/b96/b64 pieces; dword alignment)
template <int N>
__device__ __forceinline__ void ldv(__amdgpu_buffer_rsrc_t r, int vbytes, int sbytes, float* o) {
  if constexpr (N >= 4) {
    const f32x4 v = ldw4(r, vbytes, sbytes);
    o[0] = v[0], o[1] = v[1], o[2] = v[2], o[3] = v[3];
    ldv<N - 4>(r, vbytes, sbytes + 16, o + 4);
  } else if constexpr (N == 3) {
    typedef float f32x3 __attribute__((ext_vector_type(3)));
    const f32x3 v = __builtin_bit_cast(f32x3, __builtin_amdgcn_raw_buffer_load_b96(r, vbytes, sbytes, 0));
    o[0] = v[0], o[1] = v[1], o[2] = v[2];
  } else if constexpr (N == 2) {
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    const f32x2 v = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(r, vbytes, sbytes, 0));
    o[0] = v[0], o[1] = v[1];
  } else if constexpr (N == 1) {
    o[0] = ldw(r, vbytes, sbytes);
  }
}

__device__ __forceinline__ void stw(float v, __amdgpu_buffer_rsrc_t r, int vbytes, int sbytes) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, vbytes, sbytes, 0);
}
// N contiguous floats to one lane offset (b128 pieces; 16-byte aligned);
// offsets outside the descriptor are dropped
template <int N>
__device__ __forceinline__ void stv(__amdgpu_buffer_rsrc_t r, int vbytes, int sbytes, const float* v) {
  static_assert(N % 4 == 0, "b128 pieces");
#pragma unroll
  for (int q = 0; q < N / 4; ++q) {
    f32x4 t;
    t[0] = v[4 * q], t[1] = v[4 * q + 1], t[2] = v[4 * q + 2], t[3] = v[4 * q + 3];
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, t), r,
                                           vbytes, sbytes + 16 * q, 0);
  }
}
// descriptor over [p, p + nbytes) (nbytes clamped to the 32-bit range)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_bytes(const void* p, int64_t nbytes) {
  const int n = nbytes > 0x7fffffff ? 0x7fffffff : (int)nbytes;
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, n, 0x00020000);
}

// ---------------------------------------------------------------- w = H2 W2 on bf16 MFMA
// The 64 -> W layer of the radial MLP (90 % of its FLOPs) runs on
// v_mfma_f32_16x16x32_bf16 with both operands split into three bf16 pieces
// (x = p0 + p1 + p2 exactly, 24 significant bits) and the six piece products
// with i + j <= 2 accumulated in f32, smallest first: f32-grade accuracy (the
// dropped terms are below 2^-24 relative) at 12 x 16 = 192 MFMA cycles per
// 16 x 16 x 64 block instead of 16 x 32 = 512 on v_mfma_f32_16x16x4_f32.
// k order: element t of lane group g in k-half m is hidden unit
// 16(2m + t/4) + 4g + t%4, which is exactly register (bh = 2m + t/4, r = t%4)
// of the H2 accumulators a lane already holds -- no lane movement.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
struct Op3 {
  bf16x8 v[3][2];  // [piece][k-half]
};
// W2 operand of column block col0 (w2b order, 6 x b128 per lane)
__device__ __forceinline__ void load_w2b(Op3& o, __amdgpu_buffer_rsrc_t w2b, int lane, int col0) {
#pragma unroll
  for (int pc = 0; pc < 3; ++pc)
#pragma unroll
    for (int m = 0; m < 2; ++m)
      o.v[pc][m] = __builtin_bit_cast(
          bf16x8, __builtin_amdgcn_raw_buffer_load_b128(w2b, lane * 16, ((col0 / 16 * 3 + pc) * 2 + m) * 1024, 0));
}
// Eight floats as three bf16 pieces (v = p0 + p1 + p2, each piece the
// round-to-nearest-even bf16 of the remaining residual), two values per
// v_cvt_pk_bf16_f32: the packed pair is both the MFMA operand word and, widened
// by a shift / mask, what the residual subtracts (5.5 VALU per value instead of
// the 7.5 of per-value conversions re-packed afterwards; same bits)
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void split3x8(const float (&v)[8], bf16x8 (&d)[3]) {
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

// the same in two pieces (v = p0 + p1 + O(2^-16 |v|)): the operand of the
// three-product (bf16x3) dH2 form below
__device__ __forceinline__ void split2x8(const float (&v)[8], bf16x8 (&d)[2]) {
  u32x4 w[2];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f32x2 r;
    r[0] = v[2 * q];
    r[1] = v[2 * q + 1];
    const unsigned u = __builtin_bit_cast(unsigned, __builtin_convertvector(r, bf16x2));
    w[0][q] = u;
    r[0] -= __builtin_bit_cast(float, u << 16);
    r[1] -= __builtin_bit_cast(float, u & 0xffff0000u);
    w[1][q] = __builtin_bit_cast(unsigned, __builtin_convertvector(r, bf16x2));
  }
  d[0] = __builtin_bit_cast(bf16x8, w[0]);
  d[1] = __builtin_bit_cast(bf16x8, w[1]);
}

// the lane's 16 H2 values (units 16 bh + 4g + r) as three bf16 pieces
__device__ __forceinline__ void split_h2(const f32x4 (&h2)[4], Op3& o) {
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    float v[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = h2[2 * m + (t >> 2)][t & 3];
    bf16x8 d[3];
    split3x8(v, d);
#pragma unroll
    for (int pc = 0; pc < 3; ++pc) o.v[pc][m] = d[pc];
  }
}
// HA: H2 is the A operand (rows = edges: forward); else W2^T is (rows = channels)
template <bool HA>
__device__ __forceinline__ f32x4 w2_block(const Op3& h, const Op3& w) {
  constexpr int I[6] = {2, 1, 0, 1, 0, 0}, J[6] = {0, 1, 2, 0, 1, 0};
  f32x4 acc = zero4();
#pragma unroll
  for (int q = 0; q < 6; ++q)
#pragma unroll
    for (int m = 0; m < 2; ++m)
      acc = HA ? mfma16(h.v[I[q]][m], w.v[J[q]][m], acc) : mfma16(w.v[J[q]][m], h.v[I[q]][m], acc);
  return acc;
}

// the same block from the first two pieces only (three products): the
// backward kernels' w recompute (default; E3GNN_BWD_W_X3=0: six).  The energy
// keeps the forward's six-product w; the recomputed w differs from it by
// ~2^-16 relative, and the force errors against the reference KATs did not
// move (max 1.91e-5 -> 1.89e-5 eV/A over the five systems; 97k / 778k
// full-size checks green); middle backward -5.5 %, first block -11 %
template <bool HA>
__device__ __forceinline__ f32x4 w2_block3(const Op3& h, const Op3& w) {
  f32x4 acc = zero4();
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    acc = HA ? mfma16(h.v[1][m], w.v[0][m], acc) : mfma16(w.v[0][m], h.v[1][m], acc);
    acc = HA ? mfma16(h.v[0][m], w.v[1][m], acc) : mfma16(w.v[1][m], h.v[0][m], acc);
    acc = HA ? mfma16(h.v[0][m], w.v[0][m], acc) : mfma16(w.v[0][m], h.v[0][m], acc);
  }
  return acc;
}
#ifndef E3GNN_BWD_W_X3
#define E3GNN_BWD_W_X3 1
#endif
template <bool HA>
__device__ __forceinline__ f32x4 w2_block_bwd(const Op3& h, const Op3& w) {
  if constexpr (E3GNN_BWD_W_X3) return w2_block3<HA>(h, w);
  else return w2_block<HA>(h, w);
}

// ---------------------------------------------------------------- radial MLP
// Tile of 16 edge slots [e0, e0+16) (slots >= e1 are zero rows).
// a1/a2: pre-activations of the two hidden layers, transposed (4 blocks of 16 units).
struct MlpT {
  f32x4 a1[4], a2[4];
};

// b[s] = emb[edge of slot (l&15)][4s + (l>>4)]
// Layer 0 (K = 8) on f32 MFMA; layer 1 (64 -> 64) on bf16x6 like w = H2 W2
// (w2_block: act(a1) split in three bf16 pieces in its accumulator layout, W1
// pre-split in the same operand order, MlpW::w1b): 48 MFMAs x 16 cycles
// instead of 64 x 32 on v_mfma_f32_16x16x4_f32, f32-grade.
__device__ __forceinline__ void mlp_layer0(const WRes& R, const float (&b)[2], int lane, f32x4 (&a1)[4]) {
  const int g = lane >> 4, c = lane & 15;
  const int v0 = (g * 64 + c) * 4;  // W0s[4s + g][16 bh + c]
#pragma unroll
  for (int bh = 0; bh < 4; ++bh) {
    f32x4 acc = zero4();
#pragma unroll
    for (int s = 0; s < 2; ++s) acc = mfma(ldw(R.w0, v0, (4 * s * 64 + 16 * bh) * 4), b[s], acc);
    a1[bh] = acc;
  }
}
// The backward kernels' MLP-chain products (the layer-1 recompute and the
// chain backward's dH1 / dE/demb) on three bf16 products like dH2 and the w
// recompute (E3GNN_CHAIN_X3, default; =0 six); the forward, whose chain gives
// the energy, keeps six.  Same box: step 39.8 -> 39.2 ms (first / middle /
// last backward 1.68 / 5.28 / 2.06 -> 1.56 / 5.20 / 1.92 ms); parity, full-size
// and family tests green; NVE drift over 2,000 steps 1.67e-4 meV/atom/ps
// against 1.38e-4 (six-product chains) and 1.19e-4 (exact-gradient generic
// engine), excursions identical (profiles/r06_s18_*)
#ifndef E3GNN_CHAIN_X3
#define E3GNN_CHAIN_X3 1
#endif
constexpr bool CX3 = E3GNN_CHAIN_X3 != 0;
// X3: layer 1 on three bf16 products
template <bool X3 = false>
__device__ __forceinline__ void mlp_chain(const WRes& R, const float (&b)[2], int lane, MlpT& m) {
  mlp_layer0(R, b, lane, m.a1);
  Op3 hq;
  {
    f32x4 h1[4];
#pragma unroll
    for (int bh = 0; bh < 4; ++bh)
#pragma unroll
      for (int r = 0; r < 4; ++r) h1[bh][r] = act_fwd(m.a1[bh][r]);
    split_h2(h1, hq);
  }
#pragma unroll
  for (int bo = 0; bo < 4; ++bo) {
    phase();
    Op3 wq;
    load_w2b(wq, R.w1b, lane, 16 * bo);
    m.a2[bo] = X3 ? w2_block3<false>(hq, wq) : w2_block<false>(hq, wq);
  }
}

__device__ __forceinline__ void mlp_pre(const WRes& R, const float* __restrict__ emb, int e0,
                                        int e1, int lane, MlpT& m) {
  const int g = lane >> 4, c = lane & 15;
  const int e = e0 + c;
  float b[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) b[s] = e < e1 ? emb[(int64_t)e * 8 + 4 * s + g] : 0.f;
  mlp_chain(R, b, lane, m);
}

// both tiles of a forward pass (E3GNN_FWD_CHAIN2): layer 1's W1 operand
// blocks loaded once for the two tiles' products (the same six products per
// tile as mlp_chain, the same sums)
__device__ __forceinline__ void mlp_pre2(const WRes& R, const float* __restrict__ emb, int e0, int e1,
                                         bool two, int lane, f32x4 (&a2)[2][4]) {
  const int g = lane >> 4, c = lane & 15;
  Op3 hq[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int e = e0 + 16 * u + c;
    float b[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) b[s] = (e < e1 && (u == 0 || two)) ? emb[(int64_t)e * 8 + 4 * s + g] : 0.f;
    f32x4 a1[4];
    mlp_layer0(R, b, lane, a1);
    f32x4 h1[4];
#pragma unroll
    for (int bh = 0; bh < 4; ++bh)
#pragma unroll
      for (int r = 0; r < 4; ++r) h1[bh][r] = act_fwd(a1[bh][r]);
    split_h2(h1, hq[u]);
  }
#pragma unroll
  for (int bo = 0; bo < 4; ++bo) {
    phase();
    Op3 wq;
    load_w2b(wq, R.w1b, lane, 16 * bo);
    a2[0][bo] = w2_block<false>(hq[0], wq);
    a2[1][bo] = two ? w2_block<false>(hq[1], wq) : zero4();
  }
}

// ---------------------------------------------------------------- TP pieces
// CG entries grouped by (i, j): each pair's partial sum over k is formed and
// consumed at once (short live ranges, one product per pair)
template <class C, int I, int J>
__device__ __forceinline__ constexpr bool cg_pair() {
  for (int q = 0; q < C::n; ++q)
    if (C::e[q].i == I && C::e[q].j == J) return true;
  return false;
}

// The lane's four edge slots r = 0..3 in lock-step (the dependency chains of
// the contraction run four-wide).  Forward:
//   acc[k] += sum_ij C_ijk s_ij,  s_ij = sum_r w[r] x[r][i] y[r][j]
// (4 per (i, j) pair + 1 per CG entry; forming sum_ij C_ijk x y per slot first
// and weighting at the end costs 4 per CG entry); y[r] = the slot's SH block
// (stride ys between slots).
template <int L1, int L2, int L3>
__device__ __forceinline__ void tp_acc4(const float* x, const float* y, int ys, const f32x4 w,
                                        float* acc) {
  using C = CG<L1, L2, L3>;
  constexpr int D1 = 2 * L1 + 1, D2 = 2 * L2 + 1;
  float yv[4][D2];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int q = 0; q < D2; ++q) yv[r][q] = y[r * ys + q];
  sfor<D1>([&](auto i) {
    float wx[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) wx[r] = w[r] * x[r * D1 + i];
    sfor<D2>([&](auto j) {
      if constexpr (cg_pair<C, i, j>()) {
        float sv = wx[0] * yv[0][j];
#pragma unroll
        for (int r = 1; r < 4; ++r) sv += wx[r] * yv[r][j];
        sfor<C::n>([&](auto q) {
          if constexpr (C::e[q].i == i && C::e[q].j == j) acc[C::e[q].k] += C::e[q].c * sv;
        });
      }
    });
  });
}

// Backward, the lane's 4 channels r of one edge:
//   u_ri = sum_jk C_ijk y_j g[r][k],  dx[r][i] += w[r] u_ri,  dw[r] = sum_i x[r][i] u_ri,
//   dy_j += sum_ik C_ijk sum_r w[r] x[r][i] g[r][k]
// Two contraction orders, chosen per path at compile time by VALU count:
//  * by (i, j): t'_rij = sum_k C_ijk g[r][k] (4 per CG entry: g is per channel),
//    u_ri += t'_rij y_j, dy_j += sum_r t'_rij w[r] x[r][i] (4 + 4 per (i, j) pair);
//  * by (i, k): ytilde_ik = sum_j C_ijk y_j (1 per CG entry: y is per edge, the
//    same for the lane's 4 channels), u_ri += ytilde_ik g[r][k] and
//    m_ik = sum_r w[r] x[r][i] g[r][k] (4 + 4 per (i, k) pair), dy_j += C_ijk m_ik
//    (1 per CG entry).  For the paths with many CG entries per output (l >= 1
//    on all three legs) this is ~25 % fewer VALU instructions.
template <class C, int I, int K>
__device__ __forceinline__ constexpr bool cg_ik() {
  for (int q = 0; q < C::n; ++q)
    if (C::e[q].i == I && C::e[q].k == K) return true;
  return false;
}
template <class C>
constexpr int cg_count_pairs(bool by_ik) {
  int n = 0;
  for (int q = 0; q < C::n; ++q) {
    bool first = true;
    for (int p = 0; p < q; ++p)
      if (C::e[p].i == C::e[q].i && (by_ik ? C::e[p].k == C::e[q].k : C::e[p].j == C::e[q].j)) first = false;
    n += first;
  }
  return n;
}
// CG entries that cost an instruction in the (i, j) order (a pair's only entry
// with coefficient 1 is a register alias)
template <class C>
constexpr int cg_cost_ij_entries() {
  int n = 0;
  for (int q = 0; q < C::n; ++q) {
    int cnt = 0;
    for (int p = 0; p < C::n; ++p) cnt += C::e[p].i == C::e[q].i && C::e[p].j == C::e[q].j;
    n += !(cnt == 1 && C::e[q].c == 1.0f);
  }
  return n;
}
template <int L1, int L2, int L3>
constexpr bool tp_bwd_by_ik() {
  using C = CG<L1, L2, L3>;
  const int P = cg_count_pairs<C>(false), Q = cg_count_pairs<C>(true);
  const int ij = 4 * (cg_cost_ij_entries<C>() + P) + (L2 > 0 ? 4 * P : 0);
  const int ik = C::n + 4 * Q + (L2 > 0 ? 4 * Q + C::n : 0);
  return ik < ij;
}

template <int L1, int L2, int L3>
__device__ __forceinline__ void tp_bwd_xw4(const float* x, const float* y, const f32x4 w,
                                           const float* gm, float* dx, float* dy, float* dw) {
  using C = CG<L1, L2, L3>;
  constexpr int D1 = 2 * L1 + 1, D2 = 2 * L2 + 1, D3 = 2 * L3 + 1;
#pragma unroll
  for (int r = 0; r < 4; ++r) dw[r] = -0.f;
  // ytilde depends on the edge only: without this opaque copy LLVM hoists
  // every path's ytilde out of the channel-group loop (74 live values for
  // l1 = 2: spills)
  float yl[D2];
  if constexpr (tp_bwd_by_ik<L1, L2, L3>()) {
#pragma unroll
    for (int q = 0; q < D2; ++q) yl[q] = y[q];
    pin<D2>(yl);
  }
  sfor<D1>([&](auto i) {
    float u[4] = {-0.f, -0.f, -0.f, -0.f}, wx[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) wx[r] = w[r] * x[r * D1 + i];
    if constexpr (tp_bwd_by_ik<L1, L2, L3>()) {
      sfor<D3>([&](auto k) {
        if constexpr (cg_ik<C, i, k>()) {
          float yt = -0.f;
          sfor<C::n>([&](auto q) {
            if constexpr (C::e[q].i == i && C::e[q].k == k) yt += C::e[q].c * yl[C::e[q].j];
          });
#pragma unroll
          for (int r = 0; r < 4; ++r) u[r] += yt * gm[r * D3 + k];
          if constexpr (L2 > 0) {
            float m = wx[0] * gm[k];
#pragma unroll
            for (int r = 1; r < 4; ++r) m += wx[r] * gm[r * D3 + k];
            sfor<C::n>([&](auto q) {
              if constexpr (C::e[q].i == i && C::e[q].k == k) dy[C::e[q].j] += C::e[q].c * m;
            });
          }
        }
      });
    } else {
      sfor<D2>([&](auto j) {
        if constexpr (cg_pair<C, i, j>()) {
          float tp[4] = {-0.f, -0.f, -0.f, -0.f};
          sfor<C::n>([&](auto q) {
            if constexpr (C::e[q].i == i && C::e[q].j == j) {
#pragma unroll
              for (int r = 0; r < 4; ++r) tp[r] += C::e[q].c * gm[r * D3 + C::e[q].k];
            }
          });
#pragma unroll
          for (int r = 0; r < 4; ++r) u[r] += tp[r] * y[j];
          if constexpr (L2 > 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) dy[j] += tp[r] * wx[r];
          }
        }
      });
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      dx[r * D1 + i] += w[r] * u[r];
      dw[r] += x[r * D1 + i] * u[r];
    }
  });
}

template <class L, int I>
constexpr int iblock_mul() {
  for (int p = 0; p < L::NP; ++p)
    if (L::P[p].l1 == I) return L::P[p].mul;
  return 0;
}
template <class L, int I>
constexpr int iblock_xoff() {
  for (int p = 0; p < L::NP; ++p)
    if (L::P[p].l1 == I) return L::P[p].xoff;
  return 0;
}

// ---- block sequence (input irrep I, channel block jj, path) and operand prefetch
template <class L>
constexpr int first_path_of(int I) {
  for (int p = 0; p < L::NP; ++p)
    if (L::P[p].l1 == I) return p;
  return -1;
}
template <class L>
constexpr int next_path_same_I(int pi) {
  for (int p = pi + 1; p < L::NP; ++p)
    if (L::P[p].l1 == L::P[pi].l1) return p;
  return -1;
}
template <class L>
constexpr int first_path_after_I(int I) {
  for (int i = I + 1; i < 3; ++i)
    if (first_path_of<L>(i) >= 0) return first_path_of<L>(i);
  return -1;
}
// weight column of the block after (I, jj, PI); -1 at the end of the tile
template <class L, int I, int PI>
__device__ __forceinline__ int next_block_col(int jj) {
  constexpr int np = next_path_same_I<L>(PI);
  if constexpr (np >= 0) {
    return L::P[np].woff + 16 * jj;
  } else {
    constexpr int f = first_path_of<L>(I);
    constexpr int fn = first_path_after_I<L>(I);
    if (jj + 1 < L::P[f].mul / 16) return L::P[f].woff + 16 * (jj + 1);
    return fn >= 0 ? L::P[fn].woff : -1;
  }
}
// w2q blocks of column block col0 (bwd_w dH2 operand): 4 x b128
__device__ __forceinline__ void load_w2q(f32x4 (&b)[4], __amdgpu_buffer_rsrc_t w2q, int lane, int col0) {
  const int v = ((lane >> 4) * 16 + (lane & 15)) * 16;
#pragma unroll
  for (int bh = 0; bh < 4; ++bh) b[bh] = ldw4(w2q, v, (col0 / 16 * 4 + bh) * 1024);
}

// channel groups (input irrep I, 16-channel block j) in visiting order
template <class L>
constexpr int mul_of(int I) {
  for (int p = 0; p < L::NP; ++p)
    if (L::P[p].l1 == I) return L::P[p].mul;
  return 0;
}
template <class L>
constexpr int next_I(int I) {
  for (int i = I + 1; i < 3; ++i)
    if (mul_of<L>(i) > 0) return i;
  return -1;
}
template <class L>
constexpr int first_I() { return mul_of<L>(0) > 0 ? 0 : next_I<L>(0); }
// paths of input irrep I; rank of path pi among them; blocks visited before I
template <class L>
constexpr int paths_of(int I) {
  int n = 0;
  for (int p = 0; p < L::NP; ++p) n += L::P[p].l1 == I;
  return n;
}
template <class L>
constexpr int path_rank(int pi) {
  int n = 0;
  for (int p = 0; p < pi; ++p) n += L::P[p].l1 == L::P[pi].l1;
  return n;
}
template <class L>
constexpr int blocks_before(int I) {
  int n = 0;
  for (int i = 0; i < I; ++i) n += paths_of<L>(i) * mul_of<L>(i) / 16;
  return n;
}

// per tile: neighbour ids of the lane group's 4 edges, Y of the 16 edges in LDS
__device__ __forceinline__ void load_tile_edges(const int* __restrict__ nbr,
                                                const float* __restrict__ Y, int e0, int end,
                                                int lane, int (&src)[4], float* ybuf) {
  const int g = lane >> 4;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int e = e0 + 4 * g + r;
    src[r] = e < end ? nbr[e] : 0;
  }
#pragma unroll
  for (int q0 = 0; q0 < 144; q0 += 64) {
    const int q = q0 + lane;
    if (q < 144) ybuf[q] = (e0 + q / 9 < end) ? Y[(int64_t)e0 * 9 + q] : 0.f;
  }
}

// ---------------------------------------------------------------- forward
// agg[c] = sum_e TP(h[nbr e], Y_e, w_e) / denom.
// Two 16-edge tiles of the centre per pass: every W2 operand block
// (6 KB per lane set, from L2) feeds both tiles' w = H2 W2 products, halving
// the operand stream that dominates the one-tile kernel, and the two tiles'
// messages are summed in registers before the LDS accumulation.
// waves per SIMD the register allocation targets (unified VGPR+AGPR file:
// 3 waves <= 168 registers, 2 <= 256; without the hint the compiler parks
// MFMA accumulators in AGPRs and lands just above a boundary): the first
// block (128 input channels) fits three, the others two
// row sums over the four lane groups as groups of permlane swaps (the
// forward's D3 values per path, the lock-step backward's 8 dE/dY values per
// edge; E3GNN_ROWSUM_GROUPED, default) instead of one hazard-padded pair of
// swaps per value: middle forward 9.21 -> 9.01-9.11 ms for the three launches,
// same box (profiles/r06_s20_*); in the last block's backward it measured
// neutral to slower and stays per value
#ifndef E3GNN_ROWSUM_GROUPED
#define E3GNN_ROWSUM_GROUPED 1
#endif
// the forward pass's two tiles through the radial MLP together, each W1
// operand block loaded once for both (E3GNN_FWD_CHAIN2; same products, same
// bits): last-block forward 1.05-1.06 -> 1.00-1.01 ms, middle 9.13 -> 9.02 ms
// averaged over two runs each (noisy box; profiles/r06_s23_*)
#ifndef E3GNN_FWD_CHAIN2
#define E3GNN_FWD_CHAIN2 1
#endif
template <class L>
struct Fwd2Waves {
  static constexpr int v = L::KIND == 0 ? 3 : 2;
};
template <class L>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(Fwd2Waves<L>::v, Fwd2Waves<L>::v))) void k_conv_fwd(
    const int* __restrict__ row_ptr, const int* __restrict__ nbr, const float* __restrict__ emb,
    const float* __restrict__ Y, const float* __restrict__ h, float* __restrict__ agg, MlpW W, int c_begin,
    int c_end, int n_nodes, float denom) {
  __shared__ float lds[4][2][160];
  __shared__ __attribute__((aligned(16))) float aggl[4][L::DM];
  const int wid = threadIdx.x >> 6;
  const int c = __builtin_amdgcn_readfirstlane(c_begin + xcd_block() * 4 + wid);
  if (c >= c_end) return;
  float* acl = aggl[wid];
  const int lane = threadIdx.x & 63, g = lane >> 4, col = lane & 15;
  const int beg = row_ptr[c], end = row_ptr[c + 1];
  float* out = agg + (int64_t)c * L::DM;
  const WRes R = make_wres(W, L::W);
  const __amdgpu_buffer_rsrc_t Rh = rsrc_bytes(h, (int64_t)n_nodes * L::DX * 4);
  const float rden = 1.0f / denom;
  constexpr bool STAMPED = std::is_same<L, LayerMid>::value && E3GNN_STAMPS_FWD;
  STAMP_DECL
  for (int e0 = beg; e0 < end || e0 == beg; e0 += 32) {
    if constexpr (STAMPED) STAMP(0);
    const bool first_tile = e0 == beg;
    const bool two = e0 + 16 < end;   // wave-uniform: the second tile has edges
    int src[2][4];
    Op3 wq;
    load_w2b(wq, R.w2b, lane, L::P[0].woff);
#pragma unroll
    for (int u = 0; u < 2; ++u) load_tile_edges(nbr, Y, e0 + 16 * u, end, lane, src[u], lds[wid][u]);
    // tile 0's neighbour rows of the next channel group are prefetched under
    // the current group; tile 1's are loaded at the group start (consumed
    // after tile 0's first product: their latency hides there)
    float xpf[20];
    auto load_rows = [&](auto Iq, int jq, int u, float* dst) {
      constexpr int D1q = 2 * Iq + 1;
      constexpr int XOq = iblock_xoff<L, Iq>();
#pragma unroll
      for (int r = 0; r < 4; ++r)
        ldv<D1q>(Rh, (src[u][r] * L::DX + col * D1q) * 4, (XOq + 16 * jq * D1q) * 4, dst + r * D1q);
    };
    auto load_group = [&](auto Iq, int jq) { load_rows(Iq, jq, 0, xpf); };
    load_group(std::integral_constant<int, first_I<L>()>{}, 0);
    Op3 hq[2];
    if constexpr (E3GNN_FWD_CHAIN2 && L::KIND != 0) {   // (the first block: three waves, no room)
      f32x4 a2[2][4];
      mlp_pre2(R, emb, e0, end, two, lane, a2);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (u == 1 && !two) break;
        f32x4 h2[4];
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
          for (int r = 0; r < 4; ++r) h2[b][r] = act_fwd(a2[u][b][r]);
        split_h2(h2, hq[u]);
      }
    } else {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (u == 1 && !two) break;
        MlpT m;
        mlp_pre(R, emb, e0 + 16 * u, end, lane, m);
        f32x4 h2[4];
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
          for (int r = 0; r < 4; ++r) h2[b][r] = act_fwd(m.a2[b][r]);
        split_h2(h2, hq[u]);
      }
    }
    if constexpr (STAMPED) STAMP(1);   // edge loads, MLP chain, H2 split
    sfor<3>([&](auto I) {
      constexpr int MUL = iblock_mul<L, I>();
      if constexpr (MUL > 0) {
        constexpr int D1 = 2 * I + 1;
        for (int j = 0; j < MUL / 16; ++j) {
          float x[2][4 * D1];
          phase();
#pragma unroll
          for (int i = 0; i < 4 * D1; ++i) x[0][i] = xpf[i];
          load_rows(I, j, 1, x[1]);
          if (j + 1 < MUL / 16) {
            load_group(I, j + 1);
          } else {
            constexpr int IN = next_I<L>(I);
            if constexpr (IN >= 0) load_group(std::integral_constant<int, IN>{}, 0);
          }
          sfor<L::NP>([&](auto pi) {
            constexpr PathDef p = L::P[pi];
            if constexpr (p.l1 == I) {
              constexpr int D3 = 2 * p.l3 + 1;
              phase();
              if constexpr (STAMPED) STAMP(4);   // (group start: row copies / loads)
              const f32x4 wv0 = w2_block<true>(hq[0], wq);
              const f32x4 wv1 = two ? w2_block<true>(hq[1], wq) : zero4();
              {  // operands of the next block load under this block's tensor product
                const int nc = next_block_col<L, I, pi>(j);
                if (nc >= 0) load_w2b(wq, R.w2b, lane, nc);
              }
              phase();
              if constexpr (STAMPED) STAMP(2);   // w MFMAs
              float acc[D3];
#pragma unroll
              for (int k = 0; k < D3; ++k) acc[k] = -0.f;
              // the lane's 4 edges of each tile (padded edges have Y = 0)
              tp_acc4<p.l1, p.l2, p.l3>(x[0], lds[wid][0] + 4 * g * 9 + yoff(p.l2), 9, wv0, acc);
              if (two) tp_acc4<p.l1, p.l2, p.l3>(x[1], lds[wid][1] + 4 * g * 9 + yoff(p.l2), 9, wv1, acc);
              if constexpr (STAMPED) STAMP(3);   // tensor product
              if constexpr (E3GNN_ROWSUM_GROUPED) sum_rows4_n<D3>(acc);
#pragma unroll
              for (int k = 0; k < D3; ++k) {
                float v = acc[k];
                v = (E3GNN_ROWSUM_GROUPED ? v : sum_rows4(v)) * rden;
                if (g == 0) {
                  float* a = acl + p.moff + (16 * j + col) * D3 + k;
                  *a = first_tile ? v : *a + v;
                }
              }
              if constexpr (STAMPED) STAMP(5);   // row sums + LDS accumulation
            }
          });
        }
      }
    });
    if (end <= beg) break;
  }
  phase();
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  {
    const float4* src = reinterpret_cast<const float4*>(acl);
    float4* dst = reinterpret_cast<float4*>(out);
    for (int t = lane; t < L::DM / 4; t += 64) dst[t] = src[t];
  }
  if constexpr (STAMPED) {
    STAMP(6);   // copy-out
    STAMP_FLUSH(c - c_begin);
  }
}

// ---------------------------------------------------------------- backward
// tp_bwd_x and dE/dw of the same (edge, channel) in one pass: with
// t'_ij = sum_k C_ijk g_k and u_i = sum_j t'_ij y_j,
//   dE/dx_i += w u_i,  dE/dy_j += t'_ij (w x_i),  dE/dw = sum_i x_i u_i
// (no x_i y_j products: those are shared by the paths of an (l1, l2) pair, and
// the compiler kept them live across paths; the fused backward, MODE 3)
template <int L1, int L2, int L3>
__device__ __forceinline__ float tp_bwd_xw(const float* x, const float* y, float w, const float* gm,
                                           float* dx, float* dy) {
  using C = CG<L1, L2, L3>;
  float dwv = -0.f;
  sfor<2 * L1 + 1>([&](auto i) {
    float ui = -0.f;
    const float wx = w * x[i];
    sfor<2 * L2 + 1>([&](auto j) {
      if constexpr (cg_pair<C, i, j>()) {
        float tp = -0.f;
        sfor<C::n>([&](auto q) {
          if constexpr (C::e[q].i == i && C::e[q].j == j) tp += C::e[q].c * gm[C::e[q].k];
        });
        ui += tp * y[j];
        dy[j] += tp * wx;
      }
    });
    dx[i] += w * ui;
    dwv += x[i] * ui;
  });
  return dwv;
}

// sum over the 16 lanes of a DPP row (fixed order; every lane gets the total)
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float x) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float row_sum16(float v) {
  v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);  // row_half_mirror
  v += dpp_mov<0x140>(v);  // row_mirror
  return v;
}

// dE/dagg operands of path PN at channel block jj for the lane's edge (4 * D3
// floats at the edge centre's row, channels 4g..4g+3)
template <class L, int PN>
__device__ __forceinline__ void load_gm(float* gmN, __amdgpu_buffer_rsrc_t Rg, int vg, int g, int jj) {
  constexpr int D3 = 2 * L::P[PN].l3 + 1;
  ldv<4 * D3>(Rg, vg + 4 * g * D3 * 4, (L::P[PN].moff + 16 * jj * D3) * 4, gmN);
}
// MLP chain backward of a 16-edge tile from dH2^T (D[hidden 16 bh + 4g + r][edge
// slot c]): pre-activations recomputed, dA2, dH1^T = W1 dA2^T, demb^T = W0 dA1^T,
// demb += (rows < 8).  `er`: the edge of the lane's slot c (-1: padded slot).
__device__ __forceinline__ void mlp_bwd_chain_ids(const WRes& R, const float* __restrict__ emb, int er,
                                                  int lane, const f32x4 (&dh2)[4],
                                                  float* __restrict__ demb, const float* dold = nullptr,
                                                  const float* bk = nullptr, const f32x4* a2k = nullptr,
                                                  const f32x4* a1k = nullptr) {
  const int g = lane >> 4;
  MlpT m;
  if (a2k) {   // (the tile start's layer-1 pre-activations kept: layer 0 only)
    if (a1k) {   // (and layer 0's: nothing recomputed)
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) m.a1[bb] = a1k[bb];
    } else {
      const float b[2] = {bk[0], bk[1]};
      mlp_layer0(R, b, lane, m.a1);
    }
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) m.a2[bb] = a2k[bb];
  } else {
    float b[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) b[s] = er >= 0 ? emb[(int64_t)er * 8 + 4 * s + g] : 0.f;
    mlp_chain<CX3>(R, b, lane, m);
  }

  // dH1^T = W1 dA2^T and demb^T = W0 dA1^T on bf16x6 (operands W1^T and W0^T
  // pre-split, MlpW::w1tb / w0tb; dA split in their accumulator layout)
  f32x4 dh1[4];
  {
    f32x4 da2[4];
#pragma unroll
    for (int bb = 0; bb < 4; ++bb)
#pragma unroll
      for (int r = 0; r < 4; ++r) da2[bb][r] = dh2[bb][r] * act_grad(m.a2[bb][r]);
    Op3 dq;
    split_h2(da2, dq);
#pragma unroll
    for (int bi = 0; bi < 4; ++bi) {
      phase();
      Op3 wq;
      load_w2b(wq, R.w1tb, lane, 16 * bi);
      dh1[bi] = CX3 ? w2_block3<false>(dq, wq) : w2_block<false>(dq, wq);
    }
  }
  f32x4 de;
  {
    f32x4 da1[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int t = 0; t < 4; ++t) da1[q][t] = dh1[q][t] * act_grad(m.a1[q][t]);
    Op3 dq, wq;
    split_h2(da1, dq);
    load_w2b(wq, R.w0tb, lane, 0);
    de = CX3 ? w2_block3<false>(dq, wq) : w2_block<false>(dq, wq);   // rows 4g + r < 8: the embedding dims
  }
  if (g < 2 && er >= 0) {
    if (dold) {   // (the caller read the old values at the tile start)
#pragma unroll
      for (int r = 0; r < 4; ++r) demb[(int64_t)er * 8 + 4 * g + r] = dold[r] + de[r];
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) demb[(int64_t)er * 8 + 4 * g + r] += de[r];
    }
  }
}
// the same for the CSR edge tile [e0, min(e0 + 16, end))
__device__ __forceinline__ void mlp_bwd_chain(const WRes& R, const float* __restrict__ emb, int e0,
                                              int end, int lane, const f32x4 (&dh2)[4],
                                              float* __restrict__ demb, const float* dold = nullptr,
                                              const float* bk = nullptr, const f32x4* a2k = nullptr,
                                              const f32x4* a1k = nullptr) {
  const int e = e0 + (lane & 15);
  mlp_bwd_chain_ids(R, emb, e < end ? e : -1, lane, dh2, demb, dold, bk, a2k, a1k);
}

// Backward of the last block (224 message channels), one wave per NEIGHBOUR
// node j over its incoming edges (transposed CSR src_ptr / src_perm, ascending
// edge id, tiles of 16): lane (g, c) = edge slot c x channels 4g..4g+3 of a
// 16-channel block (transposed product w^T = W2^T H2^T: D[channel 4g+r][edge
// c]); x = h[j] (one row), the edges' centres' dE/dagg gathered per block
// (DM = 224 floats a row).  dE/dx[j] is summed over the tile's 16 edge lanes
// (DPP) once per block, accumulated in LDS and written once (no per-edge
// buffer, no gather pass); per edge: dE/dY -> dE/du, and dE/dw -> dH2^T = W2
// dw^T (f32 MFMA) -> MLP chain -> dE/demb.  Every edge is visited once (by its
// neighbour's wave): deterministic.  The radial weights w of the NEXT visited
// block are formed (MFMA) before this block's tensor product (VALU).
// Two 16-edge tiles of the node per pass (28 incoming edges on average: one
// pass per node): every W2 operand block (w recompute and dH2) feeds both
// tiles, and dE/dx[j] of both tiles is summed in registers before the
// per-block DPP row sum.  The second tile is skipped when it has no edge.
// dH2 = dw W2^T (the gradient of the radial MLP's hidden layer; the
// forward-consistent w = H2 W2 stays on six products) on three bf16 products
// by default: dw in two pieces (16 significant bits), W2's first two pieces,
// products p1 q0 + p0 q1 + p0 q0 (dropped terms ~2^-16 of dH2).  Measured on
// the reference KAT systems: the force errors against the reference are the
// six-product build's (2.9e-6 .. 2.1e-5 vs 3.1e-6 .. 1.9e-5 eV/A, both
// dominated by the fp32 path elsewhere; tolerance 1e-4), the middle backward
// 12 % faster (fewer MFMAs and split instructions).  E3GNN_DH2_X3=0: six.
#ifndef E3GNN_DH2_X3
#define E3GNN_DH2_X3 1
#endif
// operand pieces requested before the MFMAs that consume them (default;
// =0 the per-block interleaved order the compiler chose): the middle
// backward's pair images from LDS (E3GNN_LDS_EARLY: 5.56 -> 5.46 ms per launch,
// same box) and the last block's dH2 pieces from L2 (E3GNN_NBR_EARLY: 2.21 ->
// 2.10 ms; profiles/r06_s10_*)
// the middle blocks' tile-end read-modify-writes of dE/du and dE/demb: the
// old values read at the tile start (E3GNN_RMW_PF: 5.39 -> 5.34 ms per launch,
// same box; profiles/r06_s12_*)
// the middle blocks' tile-start layer-1 pre-activations (a2) and embedding
// values kept to the tile end, whose MLP chain backward then recomputes layer
// 0 only (E3GNN_KEEP_A2: 5.38-5.39 -> 5.21-5.27 ms per launch, same box;
// profiles/r06_s16_*)
#ifndef E3GNN_KEEP_A2
#define E3GNN_KEEP_A2 1
#endif
#ifndef E3GNN_RMW_PF
#define E3GNN_RMW_PF 1
#endif
#ifndef E3GNN_LDS_EARLY
#define E3GNN_LDS_EARLY 1
#endif
// the same for the last block's per-pass dE/du and dE/demb (E3GNN_NBR_RMW_PF:
// 2.13 -> 2.09-2.12 ms, same box; profiles/r06_s12_*)
#ifndef E3GNN_NBR_RMW_PF
#define E3GNN_NBR_RMW_PF 1
#endif
#ifndef E3GNN_NBR_EARLY
#define E3GNN_NBR_EARLY 1
#endif
constexpr int LS_BLK = 6144;            // bytes of one w2v column block (3 pieces x 2 halves x 1 KB)
constexpr int LS_PAIR_W = 2 * LS_BLK;   // the pair's two w-recompute operand blocks
constexpr int LS_PAIR_D = 12288;        // the pair's dH2 operand (w2d: 3 pieces x 4 bh x 1 KB)

// the same product with the pair's W2 pieces read from global memory (L2: every
// wave of the launch reads the same operand; w2d order, MlpW::w2d): per hidden
// block the three pieces are loaded right before its six MFMAs
__device__ __forceinline__ void dh2_pair_g(f32x4 (&dh2)[4], const float (&da)[4], const float (&db)[4],
                                           __amdgpu_buffer_rsrc_t w2d, int pair, int lane) {
  if constexpr (E3GNN_DH2_X3) {   // three products (see dh2_pair)
    bf16x8 d[2];
    {
      float v[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] = t < 4 ? da[t] : db[t - 4];
      split2x8(v, d);
    }
#pragma unroll
    for (int bh = 0; bh < 4; ++bh) {
      bf16x8 a[2];
#pragma unroll
      for (int pc = 0; pc < 2; ++pc)
        a[pc] = __builtin_bit_cast(
            bf16x8, __builtin_amdgcn_raw_buffer_load_b128(w2d, lane * 16, pair * LS_PAIR_D + (pc * 4 + bh) * 1024, 0));
      dh2[bh] = mfma16(a[1], d[0], dh2[bh]);
      dh2[bh] = mfma16(a[0], d[1], dh2[bh]);
      dh2[bh] = mfma16(a[0], d[0], dh2[bh]);
    }
    return;
  }
  bf16x8 d[3];
  {
    float v[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = t < 4 ? da[t] : db[t - 4];
    split3x8(v, d);
  }
  constexpr int I[6] = {2, 1, 0, 1, 0, 0}, J[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
  for (int bh = 0; bh < 4; ++bh) {
    bf16x8 a[3];
#pragma unroll
    for (int pc = 0; pc < 3; ++pc)
      a[pc] = __builtin_bit_cast(
          bf16x8, __builtin_amdgcn_raw_buffer_load_b128(w2d, lane * 16, pair * LS_PAIR_D + (pc * 4 + bh) * 1024, 0));
#pragma unroll
    for (int q = 0; q < 6; ++q) dh2[bh] = mfma16(a[I[q]], d[J[q]], dh2[bh]);
  }
}

// both tiles of a pass at once: each W2 piece block is loaded once and feeds
// the two tiles' products (the one-tile form above loaded the pair's pieces
// per tile: half of the last block's dH2 operand stream)
__device__ __forceinline__ void dh2_pair_g2(f32x4 (&dh2)[2][4], const float (&dp)[2][4], const float (&dr)[2][4],
                                            bool two, __amdgpu_buffer_rsrc_t w2d, int pair, int lane) {
  constexpr int NPC = E3GNN_DH2_X3 ? 2 : 3;
  bf16x8 d[2][3];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    float v[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = t < 4 ? dp[u][t] : dr[u][t - 4];
    if constexpr (NPC == 2) {
      bf16x8 e[2];
      split2x8(v, e);
      d[u][0] = e[0];
      d[u][1] = e[1];
    } else {
      split3x8(v, d[u]);
    }
  }
#if E3GNN_NBR_EARLY
  // every piece of the pair requested first (one L2 latency per pair)
  bf16x8 aa[4][NPC];
#pragma unroll
  for (int bh = 0; bh < 4; ++bh)
#pragma unroll
    for (int pc = 0; pc < NPC; ++pc)
      aa[bh][pc] = __builtin_bit_cast(
          bf16x8, __builtin_amdgcn_raw_buffer_load_b128(w2d, lane * 16, pair * LS_PAIR_D + (pc * 4 + bh) * 1024, 0));
#endif
#pragma unroll
  for (int bh = 0; bh < 4; ++bh) {
    bf16x8 a[NPC];
#pragma unroll
    for (int pc = 0; pc < NPC; ++pc)
#if E3GNN_NBR_EARLY
      a[pc] = aa[bh][pc];
#else
      a[pc] = __builtin_bit_cast(
          bf16x8, __builtin_amdgcn_raw_buffer_load_b128(w2d, lane * 16, pair * LS_PAIR_D + (pc * 4 + bh) * 1024, 0));
#endif
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (u == 1 && !two) break;
      if constexpr (NPC == 2) {
        dh2[u][bh] = mfma16(a[1], d[u][0], dh2[u][bh]);
        dh2[u][bh] = mfma16(a[0], d[u][1], dh2[u][bh]);
        dh2[u][bh] = mfma16(a[0], d[u][0], dh2[u][bh]);
      } else {
        constexpr int I[6] = {2, 1, 0, 1, 0, 0}, J[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
        for (int q = 0; q < 6; ++q) dh2[u][bh] = mfma16(a[I[q]], d[u][J[q]], dh2[u][bh]);
      }
    }
  }
}
#ifndef E3GNN_NBR_DH2_SHARED
#define E3GNN_NBR_DH2_SHARED 1
#endif

// the last block's dH2 on bf16 MFMA from global (L2) W2 pieces: with the
// three-product form its operand traffic equals the f32 form's (two pieces x 4
// hidden blocks per pair) and the MFMA cycles drop ~5x (2.60 -> 2.41 ms, same
// box); the six-product form (E3GNN_DH2_X3=0) measured slower than f32
#ifndef E3GNN_NBR_DH2_BF16
#define E3GNN_NBR_DH2_BF16 E3GNN_DH2_X3
#endif
template <class L>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_conv_bwd_nbr(
    const int* __restrict__ src_ptr, const int* __restrict__ src_perm, const int* __restrict__ center,
    const float* __restrict__ emb, const float* __restrict__ Y, const float* __restrict__ h,
    const float* __restrict__ gagg, MlpW W, float* __restrict__ dh, float* __restrict__ dgu, int n_centers,
    int r_begin, int r_end, float* __restrict__ demb) {
  __shared__ __attribute__((aligned(16))) float lds[4][L::DX];
  const int wid = threadIdx.x >> 6;
  const int jn = __builtin_amdgcn_readfirstlane(r_begin + xcd_block() * 4 + wid);
  if (jn >= r_end) return;
  float* dacc = lds[wid];
  const int lane = threadIdx.x & 63, g = lane >> 4, col = lane & 15;
  const int qb = src_ptr[jn], qe = src_ptr[jn + 1];
  const WRes R = make_wres(W, L::W);
  const __amdgpu_buffer_rsrc_t Rx = rsrc_bytes(h + (int64_t)jn * L::DX, L::DX * 4);
  const __amdgpu_buffer_rsrc_t Rg = rsrc_bytes(gagg, (int64_t)n_centers * L::DM * 4);
  for (int t = lane; t < L::DX; t += 64) dacc[t] = 0.f;

  for (int q0 = qb; q0 < qe; q0 += 32) {
    const bool two = q0 + 16 < qe;   // wave-uniform
    phase();
    Op3 wq;
    load_w2b(wq, R.w2b, lane, L::P[0].woff);
    int er[2], vg[2];
    float y[2][9];
    // E3GNN_NBR_RMW_PF: the pass end's dE/du and dE/demb old values, read here
    float gu_old[2][3], de_old[2][4];
    Op3 hq[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int q = q0 + 16 * u + col;
      er[u] = q < qe ? src_perm[q] : -1;   // edge of slot c
      vg[u] = (er[u] >= 0 ? center[er[u]] * L::DM : n_centers * L::DM) * 4;
#pragma unroll
      for (int k = 0; k < 9; ++k) y[u][k] = er[u] >= 0 ? Y[(int64_t)er[u] * 9 + k] : 0.f;
      if constexpr (E3GNN_NBR_RMW_PF) {
#pragma unroll
        for (int k = 0; k < 3; ++k) gu_old[u][k] = (g == 0 && er[u] >= 0) ? dgu[(int64_t)er[u] * 3 + k] : 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) de_old[u][k] = (g < 2 && er[u] >= 0) ? demb[(int64_t)er[u] * 8 + 4 * g + k] : 0.f;
      }
      if (u == 1 && !two) continue;
      float b[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) b[k] = er[u] >= 0 ? emb[(int64_t)er[u] * 8 + 4 * k + g] : 0.f;
      MlpT m;
      mlp_chain<CX3>(R, b, lane, m);
      f32x4 h2[4];
#pragma unroll
      for (int bb = 0; bb < 4; ++bb)
#pragma unroll
        for (int r = 0; r < 4; ++r) h2[bb][r] = act_fwd(m.a2[bb][r]);
      split_h2(h2, hq[u]);
    }
    f32x4 dh2[2][4];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) dh2[u][bb] = zero4();
#if E3GNN_NBR_DH2_BF16
    float dwp[2][4];   // dE/dw of the block pair's first block, per tile
#endif
    int nb = 0;
    constexpr int NBLK = L::W / 16;
    f32x4 wcur[2], wnxt[2] = {zero4(), zero4()};
    wcur[0] = w2_block_bwd<false>(hq[0], wq);
    wcur[1] = two ? w2_block_bwd<false>(hq[1], wq) : zero4();
    if (NBLK > 1) load_w2b(wq, R.w2v, lane, 16);
    float dYa[2][9];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int k = 0; k < 9; ++k) dYa[u][k] = 0.f;

    sfor<3>([&](auto I) {
      constexpr int MUL = iblock_mul<L, I>();
      if constexpr (MUL > 0) {
        constexpr int D1 = 2 * I + 1;
        constexpr int XOFF = iblock_xoff<L, I>();
        for (int jj = 0; jj < MUL / 16; ++jj) {
          float x[4 * D1], dx[4 * D1];
          phase();
          ldv<4 * D1>(Rx, 4 * g * D1 * 4, (XOFF + 16 * jj * D1) * 4, x);
#pragma unroll
          for (int i = 0; i < 4 * D1; ++i) dx[i] = -0.f;
          sfor<L::NP>([&](auto pi) {
            constexpr PathDef p = L::P[pi];
            if constexpr (p.l1 == I) {
              constexpr int D3 = 2 * p.l3 + 1;
              phase();
              float gm[2][4 * D3];
              load_gm<L, pi>(gm[0], Rg, vg[0], g, jj);
              load_gm<L, pi>(gm[1], Rg, vg[1], g, jj);
#if !E3GNN_NBR_DH2_BF16
              f32x4 bq[4];
              load_w2q(bq, R.w2r, lane, p.woff + 16 * jj);
#endif
              f32x4 wv[2] = {wcur[0], wcur[1]};
              if (nb + 1 < NBLK) {
                wnxt[0] = w2_block_bwd<false>(hq[0], wq);
                wnxt[1] = two ? w2_block_bwd<false>(hq[1], wq) : zero4();
              }
              if (nb + 2 < NBLK) load_w2b(wq, R.w2v, lane, 16 * (nb + 2));
              float dwr2[2][4];   // both tiles' dE/dw (the shared dH2 form)
#pragma unroll
              for (int u = 0; u < 2; ++u) {
                if (u == 1 && !two) break;
                float dwr[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                  phase();
                  float dy[2 * p.l2 + 1];
#pragma unroll
                  for (int q = 0; q < 2 * p.l2 + 1; ++q) dy[q] = 0.f;
                  // padded slots: w = 0, g = 0 and y = 0 (so dE/dw = 0)
                  dwr[r] = tp_bwd_xw<p.l1, p.l2, p.l3>(x + r * D1, y[u] + yoff(p.l2), wv[u][r], gm[u] + r * D3,
                                                       dx + r * D1, dy);
                  if constexpr (p.l2 > 0) {
#pragma unroll
                    for (int q = 0; q < 2 * p.l2 + 1; ++q) dYa[u][yoff(p.l2) + q] += dy[q];
                  }
                  pin<D1>(dx + r * D1);
                  pin<8>(dYa[u] + 1);
                }
#if E3GNN_NBR_DH2_BF16 && E3GNN_NBR_DH2_SHARED
#pragma unroll
                for (int r = 0; r < 4; ++r) dwr2[u][r] = u == 1 && !two ? 0.f : dwr[r];
#elif E3GNN_NBR_DH2_BF16
                // dH2^T += W2[:, pair] dw^T on bf16x6 over the block pair (K = 32
                // channels: the pair's first block is held in dwp)
                if (nb & 1) {
                  dh2_pair_g(dh2[u], dwp[u], dwr, R.w2d, nb >> 1, lane);
                } else {
#pragma unroll
                  for (int r = 0; r < 4; ++r) dwp[u][r] = dwr[r];
                }
#else
                // dH2^T += W2[:, block] dw^T: k = lane group g, channel 4g + r
#pragma unroll
                for (int bh = 0; bh < 4; ++bh)
#pragma unroll
                  for (int r = 0; r < 4; ++r) dh2[u][bh] = mfma(bq[bh][r], dwr[r], dh2[u][bh]);
#endif
              }
#if E3GNN_NBR_DH2_BF16 && E3GNN_NBR_DH2_SHARED
              if (!two) {
#pragma unroll
                for (int r = 0; r < 4; ++r) dwr2[1][r] = 0.f;
              }
              // dH2^T += W2[:, pair] dw^T over the block pair for both tiles,
              // each W2 piece loaded once (the pair's first block held in dwp)
              if (nb & 1) {
                dh2_pair_g2(dh2, dwp, dwr2, two, R.w2d, nb >> 1, lane);
              } else {
#pragma unroll
                for (int u = 0; u < 2; ++u)
#pragma unroll
                  for (int r = 0; r < 4; ++r) dwp[u][r] = dwr2[u][r];
              }
#endif
              pin<4 * D1>(dx);
              wcur[0] = wnxt[0];
              wcur[1] = wnxt[1];
              ++nb;
            }
          });
          phase();
          // both tiles' edges summed per lane already: one row sum over the 16
          // edge lanes, lane c == 0 accumulates the node's row
#pragma unroll
          for (int i = 0; i < 4 * D1; ++i) {
            const float v = row_sum16(dx[i]);
            if (col == 0) dacc[XOFF + (16 * jj + 4 * g) * D1 + i] += v;
          }
        }
      }
    });

#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (u == 1 && !two) break;
      phase();
      // dE/dY of edge c: sum over the 4 lane groups, then dE/du through the SH
      // polynomials (serial_code.py:50-70)
      float d[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) d[q] = sum_rows4(dYa[u][q + 1]);
      if (g == 0 && er[u] >= 0) {
        const float s3 = 1.7320508075688772f, s5 = 2.23606797749979f, c15 = s3 * s5;
        const float is3 = 0.57735026918962576f;  // 1 / sqrt(3)
        const float ux = y[u][1] * is3, uy = y[u][2] * is3, uz = y[u][3] * is3;
        const float gx = s3 * d[0] + c15 * (uz * d[3] + uy * d[4]) - s5 * ux * d[5] - c15 * ux * d[7];
        const float gy = s3 * d[1] + c15 * (ux * d[4] + uz * d[6]) + 2.f * s5 * uy * d[5];
        const float gz = s3 * d[2] + c15 * (ux * d[3] + uy * d[6]) - s5 * uz * d[5] + c15 * uz * d[7];
        float* o = dgu + (int64_t)er[u] * 3;
        if constexpr (E3GNN_NBR_RMW_PF) {
          o[0] = gu_old[u][0] + gx;
          o[1] = gu_old[u][1] + gy;
          o[2] = gu_old[u][2] + gz;
        } else {
          o[0] += gx;
          o[1] += gy;
          o[2] += gz;
        }
      }
      phase();
      mlp_bwd_chain_ids(R, emb, er[u], lane, dh2[u], demb, E3GNN_NBR_RMW_PF ? de_old[u] : nullptr);
    }
  }
  phase();
  __builtin_amdgcn_s_waitcnt(0);
  float* dhj = dh + (int64_t)jn * L::DX;
  for (int t = lane; t < L::DX; t += 64) dhj[t] = dacc[t];
}

// ================================================================ lock-step kernels
// One workgroup = 4 waves = 4 consecutive centres (one wave per centre, its
// CSR edges in 16-edge tiles, tile t of the four centres at the same time).
// The waves walk the same sequence of 16-column weight blocks and share the
// W2 operands of each block PAIR: staged once per workgroup in LDS (register
// staging: issued a whole pair ahead, written between two barriers), so each
// operand crosses the L2 -> CU path once per 4 tiles instead of once per tile
// and needs no per-wave prefetch registers.  The backward's dH2 = dw W2^T runs
// on bf16x6 MFMA over the pair (K = 32 channels): 24 x 16 MFMA cycles instead of
// 2 x 16 x 32 on f32 MFMA.  Middle blocks: two workgroups per CU (LDS), 2 waves
// per SIMD; the first block: 3 waves per SIMD.

// The staged image holds only the pieces the backward's products read: with
// the three-product forms (E3GNN_BWD_W_X3, E3GNN_DH2_X3) pieces 0 and 1 of
// each operand, 16 KB per pair instead of 24 (E3GNN_LS_LEAN=0: all three)
#ifndef E3GNN_LS_LEAN
#define E3GNN_LS_LEAN 1
#endif
constexpr int LS_WPC = (E3GNN_LS_LEAN && E3GNN_BWD_W_X3) ? 2 : 3;   // staged pieces of a w-recompute block
constexpr int LS_DPC = (E3GNN_LS_LEAN && E3GNN_DH2_X3) ? 2 : 3;     // of the pair's dH2 operand
constexpr int LS_IBLK = LS_WPC * 2048;   // image bytes of one w-recompute block (pieces x 2 halves x 1 KB)
constexpr int LS_IW = 2 * LS_IBLK;       // the pair's w-recompute part
constexpr int LS_IMG = LS_IW + LS_DPC * 4096;   // + the dH2 part (pieces x 4 bh x 1 KB)

template <int NPC = 3>
__device__ __forceinline__ void lds_op3(Op3& o, const char* blk, int lane) {
#pragma unroll
  for (int pc = 0; pc < NPC; ++pc)
#pragma unroll
    for (int m = 0; m < 2; ++m)
      o.v[pc][m] = *reinterpret_cast<const bf16x8*>(blk + ((pc * 2 + m) * 64 + lane) * 16);
}

// dH2^T += W2[:, pair] dw^T on bf16 MFMA (K = 32: element t of lane (g, c) is
// channel 4g + t of the pair's first block (t < 4) or 4g + t - 4 of its second,
// the w2d order); A = the W2 pieces (LDS), B = dw split in pieces (three
// products by default, six with E3GNN_DH2_X3=0)
__device__ __forceinline__ void dh2_pair(f32x4 (&dh2)[4], const float (&da)[4], const float (&db)[4],
                                         const char* pimg, int lane) {
  if constexpr (E3GNN_DH2_X3) {
    bf16x8 d[2];
    {
      float v[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] = t < 4 ? da[t] : db[t - 4];
      split2x8(v, d);
    }
#if E3GNN_LDS_EARLY
    // every piece read first, fenced from the MFMAs (one exposed LDS latency
    // for the pair, not one per hidden block)
    bf16x8 a[4][2];
#pragma unroll
    for (int bh = 0; bh < 4; ++bh)
#pragma unroll
      for (int pc = 0; pc < 2; ++pc)
        a[bh][pc] = *reinterpret_cast<const bf16x8*>(pimg + ((pc * 4 + bh) * 64 + lane) * 16);
    phase();
#pragma unroll
    for (int bh = 0; bh < 4; ++bh) {
      dh2[bh] = mfma16(a[bh][1], d[0], dh2[bh]);
      dh2[bh] = mfma16(a[bh][0], d[1], dh2[bh]);
      dh2[bh] = mfma16(a[bh][0], d[0], dh2[bh]);
    }
#else
#pragma unroll
    for (int bh = 0; bh < 4; ++bh) {
      bf16x8 a[2];
#pragma unroll
      for (int pc = 0; pc < 2; ++pc)
        a[pc] = *reinterpret_cast<const bf16x8*>(pimg + ((pc * 4 + bh) * 64 + lane) * 16);
      dh2[bh] = mfma16(a[1], d[0], dh2[bh]);
      dh2[bh] = mfma16(a[0], d[1], dh2[bh]);
      dh2[bh] = mfma16(a[0], d[0], dh2[bh]);
    }
#endif
    return;
  }
  bf16x8 d[3];
  {
    float v[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = t < 4 ? da[t] : db[t - 4];
    split3x8(v, d);
  }
  constexpr int I[6] = {2, 1, 0, 1, 0, 0}, J[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
  for (int bh = 0; bh < 4; ++bh) {
    bf16x8 a[3];
#pragma unroll
    for (int pc = 0; pc < 3; ++pc)
      a[pc] = *reinterpret_cast<const bf16x8*>(pimg + ((pc * 4 + bh) * 64 + lane) * 16);
#pragma unroll
    for (int q = 0; q < 6; ++q) dh2[bh] = mfma16(a[I[q]], d[J[q]], dh2[bh]);
  }
}

// tiles of the workgroup's centres [cb, cb + 4) clipped to c_end: the lock-step
// loop count (min_one: a centre without edges still has its one (empty) tile)
__device__ __forceinline__ int ls_tiles(const int* __restrict__ row_ptr, int cb, int c_end,
                                        bool min_one, int wpg = 4) {
  int T = 0;
#pragma unroll
  for (int w = 0; w < wpg; ++w) {
    const int cc = cb + w;
    if (cc < c_end) {
      const int t = (row_ptr[cc + 1] - row_ptr[cc] + 15) >> 4;
      T = max(T, min_one ? max(t, 1) : t);
    }
  }
  return __builtin_amdgcn_readfirstlane(T);
}

// Backward of a first / middle block (per-edge dE/dx to dxc, summed per
// neighbour by the transposed-CSR gather; dE/dY -> dE/du; dE/dw -> dH2 -> MLP
// chain -> dE/demb), the centre's dE/dagg row staged in LDS once.  Same pair
// structure as the forward (both blocks' w formed at the pair start, next
// group's neighbour rows prefetched); dH2 of the pair on bf16x6 at its end.
// waves per SIMD: the first block (128 input channels, 1,152 message channels:
// 42 KB of LDS per workgroup) runs three (168 VGPRs with a few spills
// measured 2.57 -> 2.27 ms against two), the middle blocks two (225 VGPRs;
// their 80.9 KB of LDS allows no more)
#ifndef E3GNN_LS_FIRST_WAVES
#define E3GNN_LS_FIRST_WAVES 3
#endif
template <class L>
struct BwdLsWaves {
  static constexpr int v = L::KIND == 0 ? E3GNN_LS_FIRST_WAVES : 2;
};
// centres (waves) per workgroup: 4; E3GNN_BWD_WPG = 8 (A/B) gives the middle
// block one 8-wave workgroup per CU sharing each staged W2 pair (124 KB LDS)
#ifndef E3GNN_BWD_WPG
#define E3GNN_BWD_WPG 4
#endif
template <class L>
struct BwdWpg {
  static constexpr int v = L::KIND == 1 ? E3GNN_BWD_WPG : 4;
};
// LDS-DMA staging (E3GNN_LS_DMA=1; measured and not kept: middle backward
// 5.68 -> 5.77 ms per launch, the explicit vmcnt(0) before each pair's
// barrier also drains the neighbour-row prefetch and the dE/dx stores that
// the compiler's counted waits leave in flight): the pair image is
// written by global_load_lds_dwordx4 straight from L2 (no staging registers,
// no ds_write) into one of TWO images, so a pair costs ONE barrier: at pair P
// each wave waits for its own DMA of P (issued at P - 1), the barrier makes
// all of P visible and retires every read of P - 1's image, then the DMA of
// P + 1 goes into that image.  The two images need 16 KB more LDS; in the
// middle blocks the 0e x 0e -> 0e path's dE/dagg (C0 floats, moff 0) is then
// read from L2 with the neighbour-row prefetch instead of staged, so two
// workgroups still fit a CU (2 x 80.9 KB of 160 KB).
#ifndef E3GNN_LS_DMA
#define E3GNN_LS_DMA 0
#endif
template <class L>
struct LsDma {
  static constexpr int WPG = BwdWpg<L>::v;
  static constexpr bool lean = LS_WPC == 2 && LS_DPC == 2;   // 16 x 1 KB chunks: 4 per wave
  static constexpr bool drop0 = L::KIND == 1;
  static constexpr int OFF0 = drop0 ? L::P[0].mul : 0;       // path 0 (l 0 0 0, moff 0): C0 floats
  static constexpr int DMS = L::DM - OFF0;                    // staged dE/dagg floats per centre
  static constexpr int bytes = WPG * DMS * 4 + 2 * LS_IMG;
  static constexpr bool fits = lean && WPG == 4 && BwdLsWaves<L>::v * bytes <= 163840;
  static constexpr bool v = E3GNN_LS_DMA && fits;
};
// Double-buffered REGISTER staging (E3GNN_LS_DB, default on where two images
// fit: middle backward 5.66 -> 5.53 ms per launch, same box; =0 the single
// image with two barriers per pair): the same two images and one
// barrier per pair as the DMA form, the pair's pieces still loaded into
// registers a pair ahead (loads the compiler counts: no drain of the other
// loads in flight) and written into the pair's image before the barrier --
// the other image is the one the previous pair read, retired by the previous
// pair's barrier.
#ifndef E3GNN_LS_DB
#define E3GNN_LS_DB 1
#endif
// one wave-instruction of LDS-DMA: 64 lanes x 16 bytes from per-lane global
// addresses to the wave-uniform LDS byte address lds_dst (+ lane x 16); M0
// set and restored inside the statement.  hipcc does not count it: the
// consumer waits with an explicit vmcnt before the barrier that publishes it.
__device__ __forceinline__ void glds16(const void* gsrc, unsigned lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(__attribute__((address_space(3))) const char*)p;
}
// wave priority around the lock-step backward's MFMA bursts (E3GNN_LS_PRIO:
// 1 raise it there, 0 never)
#ifndef E3GNN_LS_PRIO
#define E3GNN_LS_PRIO 1
#endif
template <int P>
__device__ __forceinline__ void ls_prio_c() { __builtin_amdgcn_s_setprio(P); }
__device__ __forceinline__ void ls_prio(int p) {
  if constexpr (E3GNN_LS_PRIO) {
    if (p) ls_prio_c<1>();
    else ls_prio_c<0>();
  }
}
#ifndef E3GNN_ABL_NOBAR
#define E3GNN_ABL_NOBAR 0
#endif
#ifndef E3GNN_ABL_NOSTAGE
#define E3GNN_ABL_NOSTAGE 0
#endif
#ifndef E3GNN_ABL_XLOCAL
#define E3GNN_ABL_XLOCAL 0
#endif
template <class L>
__global__ __launch_bounds__(64 * BwdWpg<L>::v) __attribute__((amdgpu_waves_per_eu(BwdLsWaves<L>::v, BwdLsWaves<L>::v))) void k_conv_bwd_ls(
    const int* __restrict__ row_ptr, const int* __restrict__ nbr, const float* __restrict__ emb,
    const float* __restrict__ Y, const float* __restrict__ h, const float* __restrict__ gagg, MlpW W,
    float* __restrict__ dxc, float* __restrict__ dgu, float* __restrict__ demb, int c_begin,
    int c_end, int n_nodes) {
  constexpr int NBLK = L::W / 16, NPAIR = NBLK / 2;
  static_assert(NBLK % 2 == 0, "weight blocks come in pairs");
  constexpr int WPG = BwdWpg<L>::v, NT = 64 * WPG;
  // staging pieces (b128) of a pair: the w-recompute operands, then the dH2 ones
  constexpr int NWP = LS_IW / 16, NST = LS_IMG / 16 / NT, PB = LS_IBLK / 16;
  static_assert(LS_IMG / 16 % NT == 0 && NWP % 64 == 0 && PB % 64 == 0, "staging pieces per thread");
  using DM_ = LsDma<L>;
  constexpr bool DMA = DM_::v;
  constexpr bool RDB = !DMA && E3GNN_LS_DB && DM_::fits;   // double-buffered register staging
  constexpr bool TWO = DMA || RDB;                         // two images, one barrier per pair
  // (the first block at three waves per SIMD: no VGPRs to spare)
  constexpr bool RPF = E3GNN_RMW_PF && (L::KIND == 1 || BwdLsWaves<L>::v == 2);
  constexpr bool KA2 = E3GNN_KEEP_A2 && (L::KIND == 1 || BwdLsWaves<L>::v == 2);
  constexpr int OFF0 = TWO ? DM_::OFF0 : 0, DMS = L::DM - OFF0;   // dE/dagg floats staged per centre
  static_assert(!TWO || (L::P[0].l1 == 0 && L::P[0].l2 == 0 && L::P[0].l3 == 0 && L::P[0].moff == 0 &&
                         OFF0 % 4 == 0), "path 0 is the 0e x 0e -> 0e slice at the row start");
  __shared__ __attribute__((aligned(16))) float smem[WPG * DMS + (TWO ? 2 : 1) * LS_IMG / 4];
  const int tid = threadIdx.x, wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, g = lane >> 4, col = lane & 15;
  const int cb = c_begin + blockIdx.x * WPG;
  const int c = cb + wid;
  const bool valid = c < c_end;
  const int beg = valid ? row_ptr[c] : 0, end = valid ? row_ptr[c + 1] : 0;
  const int T = ls_tiles(row_ptr, cb, c_end, false, WPG);
  float* dacc = smem + wid * DMS - OFF0;   // dacc[m] for m >= OFF0
  char* img = reinterpret_cast<char*>(smem + WPG * DMS);
  if (valid && end > beg) {
    const float4* s4 = reinterpret_cast<const float4*>(gagg + (int64_t)c * L::DM + OFF0);
    float4* d4 = reinterpret_cast<float4*>(dacc + OFF0);
    for (int k = lane; k < DMS / 4; k += 64) d4[k] = s4[k];
  }
  // DMA mode: the image the current pair reads (0 / 1), its byte base in LDS,
  // and path 0's dE/dagg row of this centre through a descriptor (invalid
  // centres: empty, reads 0)
  int rb = 0;
  const unsigned img_lds = lds_addr(img);
  const __amdgpu_buffer_rsrc_t Rg0 =
      rsrc_bytes(gagg + (valid ? (int64_t)c * L::DM : 0), valid ? (int64_t)OFF0 * 4 : 0);
  auto issue_dma = [&](int P, int buf) {
    // chunk k = 4 wid + i of the image: k < 8 the w-recompute blocks (block
    // k / 4, piece-half k % 4 of w2v), then the dH2 operand's 8 KB (w2d)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = 4 * wid + i;   // wave-uniform
      const char* src = k < 8 ? reinterpret_cast<const char*>(W.w2v) + (int64_t)P * LS_PAIR_W + (k >> 2) * LS_BLK +
                                    (k & 3) * 1024
                              : reinterpret_cast<const char*>(W.w2d) + (int64_t)P * LS_PAIR_D + (k - 8) * 1024;
      glds16(src + lane * 16, img_lds + buf * LS_IMG + k * 1024);
    }
  };
  const WRes R = make_wres(W, L::W);
  const __amdgpu_buffer_rsrc_t Rx = rsrc_bytes(h, (int64_t)n_nodes * L::DX * 4);
  f32x4 st[NST];
  auto issue = [&](int P) {
#if E3GNN_ABL_NOSTAGE
    return;
#endif
    // image piece idx: w-recompute block idx / PB (its first LS_WPC pieces
    // in the w2v order), then the dH2 operand's first LS_DPC pieces (w2d)
    auto wsrc = [&](int idx) { return (idx / PB) * LS_BLK + (idx % PB) * 16; };
    if constexpr (NWP % NT == 0) {  // (4 waves: each thread's pieces all W, then all D)
      constexpr int NW = NWP / NT;
#pragma unroll
      for (int i = 0; i < NW; ++i) st[i] = ldw4(R.w2v, wsrc(tid + NT * i), P * LS_PAIR_W);
#pragma unroll
      for (int i = NW; i < NST; ++i) st[i] = ldw4(R.w2d, (tid + NT * i - NWP) * 16, P * LS_PAIR_D);
    } else {
#pragma unroll
      for (int i = 0; i < NST; ++i) {
        const int idx = tid + NT * i;
        const bool isw = idx < NWP;  // wave-uniform (NWP % 64 == 0)
        st[i] = isw ? ldw4(R.w2v, wsrc(idx), P * LS_PAIR_W) : ldw4(R.w2d, (idx - NWP) * 16, P * LS_PAIR_D);
      }
    }
  };
  // E3GNN_ABL_*: timing-only ablations (results wrong; never the shipped build)
  auto commit = [&]() {
#if !E3GNN_ABL_NOBAR
    __syncthreads();
#endif
#if !E3GNN_ABL_NOSTAGE
#pragma unroll
    for (int i = 0; i < NST; ++i) *reinterpret_cast<f32x4*>(img + (tid + NT * i) * 16) = st[i];
#endif
#if !E3GNN_ABL_NOBAR
    __syncthreads();
#endif
  };
  constexpr bool STAMPED = std::is_same<L, LayerMid>::value && !E3GNN_STAMPS_FWD;   // SevenNet-0's
  STAMP_DECL
  if constexpr (DMA) issue_dma(0, 0);
  else issue(0);
  for (int t = 0; t < T; ++t) {
    if constexpr (STAMPED) STAMP(0);
    const int q0 = beg + 16 * t;
    const bool act = q0 < end;   // wave-uniform
    const int er = (act && q0 + col < end) ? q0 + col : -1;
#if E3GNN_ABL_XLOCAL   // timing-only: every edge reads the centre's own row (L2-hot)
    const int vx = (er >= 0 ? c : 0) * L::DX * 4;
#else
    const int vx = (er >= 0 ? nbr[er] : 0) * L::DX * 4;
#endif
    float xpf[20];   // the lane's 4 channels x D1 of the next channel group
    float g0pf[4];   // DMA mode: path 0's dE/dagg of that group (l1 = 0 groups)
    auto load_group = [&](auto Iq, int jq) {
      constexpr int D1q = 2 * Iq + 1;
      constexpr int XOq = iblock_xoff<L, Iq>();
      ldv<4 * D1q>(Rx, vx + 4 * g * D1q * 4, (XOq + 16 * jq * D1q) * 4, xpf);
      if constexpr (OFF0 > 0 && Iq == 0) ldv<4>(Rg0, 4 * g * 4, 16 * jq * 4, g0pf);
    };
    float y[9];
    float gu_old[3] = {0.f, 0.f, 0.f}, de_old[4] = {0.f, 0.f, 0.f, 0.f};   // E3GNN_RMW_PF
    f32x4 a2k[4];   // E3GNN_KEEP_A2: layer-1 pre-activations of the tile, kept to its end
    f32x4 a1k[E3GNN_KEEP_A2 >= 2 ? 4 : 1];   // (= 2: layer 0's as well)
    float bk[2];
    Op3 hq;
    // neighbour rows (lanes without an edge read row 0: harmless, their y
    // and w are 0); issued unconditionally, like every vector-memory op
    // between two pair commits, so the commit's wait counts only the staging
    // loads and leaves younger loads and stores in flight
    load_group(std::integral_constant<int, first_I<L>()>{}, 0);
    // per-edge dE/dx rows of this tile: lanes without an edge, inactive tiles
    // and the first block (dxc == nullptr) store outside the descriptor
    const int nrow = (act && dxc) ? min(16, end - q0) : 0;
    const __amdgpu_buffer_rsrc_t Rd =
        rsrc_bytes(dxc ? dxc + (int64_t)(act ? q0 : 0) * L::DX : gagg, (int64_t)nrow * L::DX * 4);
    const int vd = col * L::DX * 4;
    if (act) {
#pragma unroll
      for (int q = 0; q < 9; ++q) y[q] = er >= 0 ? Y[(int64_t)er * 9 + q] : 0.f;
      float b[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) b[s] = er >= 0 ? emb[(int64_t)er * 8 + 4 * s + g] : 0.f;
      if constexpr (RPF) {
        // the tile end's read-modify-writes (dE/du, dE/demb of the lane's
        // edge): old values read here, their latency under the whole tile
        if (g == 0 && er >= 0) {
#pragma unroll
          for (int k = 0; k < 3; ++k) gu_old[k] = dgu[(int64_t)er * 3 + k];
        }
        if (g < 2 && er >= 0) {
#pragma unroll
          for (int k = 0; k < 4; ++k) de_old[k] = demb[(int64_t)er * 8 + 4 * g + k];
        }
      }
      MlpT m;
      mlp_chain<CX3>(R, b, lane, m);
      if constexpr (KA2) {
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) a2k[bb] = m.a2[bb];
        if constexpr (E3GNN_KEEP_A2 >= 2) {
#pragma unroll
          for (int bb = 0; bb < 4; ++bb) a1k[bb] = m.a1[bb];
        }
        bk[0] = b[0];
        bk[1] = b[1];
      }
      f32x4 h2[4];
#pragma unroll
      for (int bb = 0; bb < 4; ++bb)
#pragma unroll
        for (int r = 0; r < 4; ++r) h2[bb][r] = act_fwd(m.a2[bb][r]);
      split_h2(h2, hq);
    }
    if constexpr (STAMPED) STAMP(1);   // tile setup: edge loads, MLP chain, H2 split
    f32x4 dh2[4] = {zero4(), zero4(), zero4(), zero4()};
    float dYa[9];
#pragma unroll
    for (int q = 0; q < 9; ++q) dYa[q] = 0.f;
    float dwp[4];   // dE/dw of the pair's first block
    f32x4 wv0 = zero4(), wv1 = zero4();   // w of the pair's two blocks
    sfor<3>([&](auto I) {
      constexpr int MUL = iblock_mul<L, I>();
      if constexpr (MUL > 0) {
        constexpr int D1 = 2 * I + 1;
        constexpr int XOFF = iblock_xoff<L, I>();
        // an odd number of paths: two channel groups per iteration, so the
        // position of every block in its pair is a compile-time constant (no
        // branches around the staging: the wait counts stay exact)
        constexpr int NPI = paths_of<L>(I), U = (NPI & 1) ? 2 : 1, NB0 = blocks_before<L>(I);
        static_assert((MUL / 16) % U == 0, "channel groups come in pairs");
        for (int j2 = 0; j2 < MUL / 16; j2 += U) {
          sfor<U>([&](auto hh) {
            const int jj = j2 + hh;
            float x[4 * D1], dx[4 * D1], g0[4];
#pragma unroll
            for (int i = 0; i < 4 * D1; ++i) {
              x[i] = xpf[i];
              dx[i] = 0.f;
            }
            if constexpr (OFF0 > 0 && I == 0) {
#pragma unroll
              for (int i = 0; i < 4; ++i) g0[i] = g0pf[i];
            }
            if (jj + 1 < MUL / 16) {
              load_group(I, jj + 1);
            } else {
              constexpr int IN = next_I<L>(I);
              if constexpr (IN >= 0) load_group(std::integral_constant<int, IN>{}, 0);
            }
            sfor<L::NP>([&](auto pi) {
              constexpr PathDef p = L::P[pi];
              if constexpr (p.l1 == I) {
                constexpr int D3 = 2 * p.l3 + 1;
                constexpr int ODD = (NB0 + hh * NPI + path_rank<L>(pi)) & 1;
                const int nb = NB0 + jj * NPI + path_rank<L>(pi);
                const char* pimg = img + (TWO ? rb * LS_IMG : 0);   // this pair's image
                if constexpr (!ODD) {   // pair start: stage it, fetch the next one
                  if constexpr (STAMPED) STAMP(5);
                  const int nextP = (nb >> 1) + 1 < NPAIR ? (nb >> 1) + 1 : 0;
                  if constexpr (DMA) {
                    // this wave's DMA of the pair has landed; after the barrier
                    // every wave's has, and nobody reads the other image any more
                    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
                    issue_dma(nextP, rb ^ 1);
                  } else if constexpr (RDB) {
                    // this pair's image (the one two pairs back read, retired
                    // by the previous pair's barrier), then the one barrier
#pragma unroll
                    for (int i = 0; i < NST; ++i)
                      *reinterpret_cast<f32x4*>(img + rb * LS_IMG + (tid + NT * i) * 16) = st[i];
                    __syncthreads();
                    issue(nextP);
                  } else {
                    commit();
                    issue(nextP);
                  }
                  if constexpr (STAMPED) STAMP(2);   // barriers + staging
                  if (act) {
                    ls_prio(1);   // MFMA bursts first
#if E3GNN_LDS_EARLY
                    Op3 wq, wq1;   // both blocks' pieces read first
                    lds_op3<LS_WPC>(wq, pimg, lane);
                    lds_op3<LS_WPC>(wq1, pimg + LS_IBLK, lane);
                    phase();
                    wv0 = w2_block_bwd<false>(hq, wq);
                    wv1 = w2_block_bwd<false>(hq, wq1);
#else
                    Op3 wq;
                    lds_op3<LS_WPC>(wq, pimg, lane);
                    wv0 = w2_block_bwd<false>(hq, wq);
                    lds_op3<LS_WPC>(wq, pimg + LS_IBLK, lane);
                    wv1 = w2_block_bwd<false>(hq, wq);
#endif
                    ls_prio(0);
                  }
                  if constexpr (STAMPED) STAMP(3);   // w recompute
                }
                if (act) {
                  const f32x4 wv = ODD ? wv1 : wv0;
                  float gm[4 * D3];
                  if constexpr (OFF0 > 0 && pi == 0) {   // (DMA mode: from L2, prefetched)
#pragma unroll
                    for (int k = 0; k < 4; ++k) gm[k] = g0[k];
                  } else {
                    const float* gl = dacc + p.moff + 16 * jj * D3 + 4 * g * D3;
#pragma unroll
                    for (int k = 0; k < 4 * D3; ++k) gm[k] = gl[k];
                  }
                  float dwr[4];
                  // padded slots: y = 0, so dE/dx = dE/dw = 0 there
                  tp_bwd_xw4<p.l1, p.l2, p.l3>(x, y + yoff(p.l2), wv, gm, dx, dYa + yoff(p.l2), dwr);
                  if constexpr (L::KIND != 0) pin<4 * D1>(dx);
                  pin<8>(dYa + 1);
                  if constexpr (ODD) {
                    if constexpr (STAMPED) STAMP(5);   // tensor product (+ stores)
                    ls_prio(1);   // MFMA bursts first
                    dh2_pair(dh2, dwp, dwr, pimg + LS_IW, lane);
                    ls_prio(0);
                    if constexpr (STAMPED) STAMP(4);   // dH2 (split + MFMA)
                  } else {
#pragma unroll
                    for (int r = 0; r < 4; ++r) dwp[r] = dwr[r];
                  }
                }
                if constexpr (TWO && ODD) rb ^= 1;   // the next pair reads the other image
              }
            });
            // per-edge dE/dx[nbr]; the first block's inputs are the species
            // embedding, whose gradient no output needs: no stores at all (a
            // store to an empty descriptor still costs its issue and its
            // trip through the texture unit), and dx itself is dead code there
            if constexpr (L::KIND != 0)
              stv<4 * D1>(Rd, vd + 4 * g * D1 * 4, (XOFF + 16 * jj * D1) * 4, dx);
          });
        }
      }
    });
    if (act) {
      // dE/dY of edge c: sum over the 4 lane groups, then dE/du through the SH
      // polynomials (serial_code.py:50-70)
      if constexpr (E3GNN_ROWSUM_GROUPED) {   // (the same grouped sums)
        float d4a[4] = {dYa[1], dYa[2], dYa[3], dYa[4]}, d4b[4] = {dYa[5], dYa[6], dYa[7], dYa[8]};
        sum_rows4_n<4>(d4a);
        sum_rows4_n<4>(d4b);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          dYa[1 + q] = d4a[q];
          dYa[5 + q] = d4b[q];
        }
      } else {
#pragma unroll
        for (int q = 1; q < 9; ++q) dYa[q] = sum_rows4(dYa[q]);
      }
      if (g == 0 && er >= 0) {
        const float s3 = 1.7320508075688772f, s5 = 2.23606797749979f, c15 = s3 * s5;
        const float is3 = 0.57735026918962576f;  // 1 / sqrt(3)
        const float ux = y[1] * is3, uy = y[2] * is3, uz = y[3] * is3;
        const float* d = dYa + 1;  // d[0..2] = dE/dY_1, d[3..7] = dE/dY_2
        const float gx = s3 * d[0] + c15 * (uz * d[3] + uy * d[4]) - s5 * ux * d[5] - c15 * ux * d[7];
        const float gy = s3 * d[1] + c15 * (ux * d[4] + uz * d[6]) + 2.f * s5 * uy * d[5];
        const float gz = s3 * d[2] + c15 * (ux * d[3] + uy * d[6]) - s5 * uz * d[5] + c15 * uz * d[7];
        float* o = dgu + (int64_t)er * 3;
        if constexpr (RPF) {
          o[0] = gu_old[0] + gx;
          o[1] = gu_old[1] + gy;
          o[2] = gu_old[2] + gz;
        } else {
          o[0] += gx;
          o[1] += gy;
          o[2] += gz;
        }
      }
      if constexpr (STAMPED) STAMP(5);
      mlp_bwd_chain(R, emb, q0, end, lane, dh2, demb, RPF ? de_old : nullptr, KA2 ? bk : nullptr,
                    KA2 ? a2k : nullptr, (KA2 && E3GNN_KEEP_A2 >= 2) ? a1k : nullptr);
    }
    if constexpr (STAMPED) STAMP(6);   // tile end: dE/dY sums, MLP chain backward
  }
  if constexpr (STAMPED) STAMP_FLUSH(blockIdx.x * WPG + wid);
  // the last pair's DMA (pair 0 of a next tile) lands before the wave ends
  if constexpr (DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

template <class L>
static hipError_t bwd_ls_impl(const FusedArgs& a, hipStream_t s) {
  constexpr int WPG = BwdWpg<L>::v;
  const int nc = a.c_end - a.c_begin;
  hipLaunchKernelGGL(k_conv_bwd_ls<L>, dim3((nc + WPG - 1) / WPG), dim3(64 * WPG), 0, s, a.row_ptr, a.nbr,
                     a.emb, a.Y, a.h, a.gagg, a.W, a.dxc, a.dgu, a.demb, a.c_begin, a.c_end, a.n_nodes);
  return hipGetLastError();
}

template <class L>
static hipError_t fwd_impl(const FusedArgs& a, hipStream_t s) {
  const int nc = a.c_end - a.c_begin;  // centre range of this launch
  if (nc <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_conv_fwd<L>, dim3((nc + 3) / 4), dim3(256), 0, s, a.row_ptr, a.nbr, a.emb,
                     a.Y, a.h, a.agg, a.W, a.c_begin, a.c_end, a.n_nodes, a.denom);
  return hipGetLastError();
}

template <class L>
static hipError_t bwd_nbr_impl(const FusedArgs& a, hipStream_t s) {
  const int nn = a.node_end - a.node_begin;
  hipLaunchKernelGGL(k_conv_bwd_nbr<L>, dim3((nn + 3) / 4), dim3(256), 0, s, a.src_ptr, a.src_perm,
                     a.center, a.emb, a.Y, a.h, a.gagg, a.W, a.dh, a.dgu, a.n_centers, a.node_begin,
                     a.node_end, a.demb);
  return hipGetLastError();
}

// kind code -> family (tp.h)
#define E3GNN_FAMILY_SWITCH(code, F_FIRST, F_MID, F_LAST)       \
  switch (code) {                                               \
    case 0: F_FIRST(0); case 1: F_MID(0); case 2: F_LAST(0);    \
    case 3: F_FIRST(1); case 4: F_MID(1); case 5: F_LAST(1);    \
    case 6: F_FIRST(2); case 7: F_MID(2); case 8: F_LAST(2);    \
    default: return hipErrorInvalidValue;                       \
  }

hipError_t launch_conv_bwd_ls(int kind, const FusedArgs& a, hipStream_t s) {
  const int nc = a.c_end - a.c_begin;
  if (nc <= 0 || a.n_nodes <= 0) return hipSuccess;
#define FIRST_(f) return bwd_ls_impl<Family<f>::First>(a, s)
#define MID_(f) return bwd_ls_impl<Family<f>::Mid>(a, s)
#define LAST_(f) return hipErrorInvalidValue   // the last block: launch_conv_bwd_nbr_last
  E3GNN_FAMILY_SWITCH(kind, FIRST_, MID_, LAST_)
#undef FIRST_
#undef MID_
#undef LAST_
}

hipError_t launch_conv_fwd(int kind, const FusedArgs& a, hipStream_t s) {
#define FIRST_(f) return fwd_impl<Family<f>::First>(a, s)
#define MID_(f) return fwd_impl<Family<f>::Mid>(a, s)
#define LAST_(f) return fwd_impl<Family<f>::Last>(a, s)
  E3GNN_FAMILY_SWITCH(kind, FIRST_, MID_, LAST_)
#undef FIRST_
#undef MID_
#undef LAST_
}

hipError_t launch_conv_bwd_nbr_last(int kind, const FusedArgs& a, hipStream_t s) {
  const int nn = a.node_end - a.node_begin;
  if (nn <= 0 || a.n_nodes <= 0) return hipSuccess;
#define FIRST_(f) return hipErrorInvalidValue
#define MID_(f) return hipErrorInvalidValue
#define LAST_(f) return bwd_nbr_impl<Family<f>::Last>(a, s)
  E3GNN_FAMILY_SWITCH(kind, FIRST_, MID_, LAST_)
#undef FIRST_
#undef MID_
#undef LAST_
}

template <class L>
static void kind_dims(int* dx, int* w, int* dm) {
  *dx = L::DX;
  *w = L::W;
  *dm = L::DM;
}
bool fused_kind_dims(int code, int* dx, int* w, int* dm) {
  auto f = [&]() -> hipError_t {
#define FIRST_(f) return kind_dims<Family<f>::First>(dx, w, dm), hipSuccess
#define MID_(f) return kind_dims<Family<f>::Mid>(dx, w, dm), hipSuccess
#define LAST_(f) return kind_dims<Family<f>::Last>(dx, w, dm), hipSuccess
    E3GNN_FAMILY_SWITCH(code, FIRST_, MID_, LAST_)
#undef FIRST_
#undef MID_
#undef LAST_
  };
  return f() == hipSuccess;
}

// algorithmic FLOP of one TP forward per edge: per path and channel 2 per CG
// entry + 1 per output component (SURVEY.md 8d's 3,456 / 16,832 / 1,184 for
// SevenNet-0's first / middle / last block)
template <class L>
constexpr double kind_tp_flops() {
  double f = 0;
  sfor_host<L::NP>([&](auto pi) {
    constexpr PathDef p = L::P[pi];
    f += (double)p.mul * (2 * CG<p.l1, p.l2, p.l3>::n + 2 * p.l3 + 1);
  });
  return f;
}
static_assert(kind_tp_flops<LayerFirst>() == 3456.0 && kind_tp_flops<LayerMid>() == 16832.0 &&
                  kind_tp_flops<LayerLast>() == 1184.0,
              "SURVEY.md 8d per-edge TP FLOP");
double fused_kind_tp_flops(int code) {
  switch (code) {
#define K_(c, f, T) \
  case c:           \
    return kind_tp_flops<Family<f>::T>();
    K_(0, 0, First) K_(1, 0, Mid) K_(2, 0, Last) K_(3, 1, First) K_(4, 1, Mid) K_(5, 1, Last)
    K_(6, 2, First) K_(7, 2, Mid) K_(8, 2, Last)
#undef K_
    default: return 0.0;
  }
}

template <class L>
static int kind_paths(PathDef* out, int max) {
  for (int p = 0; p < L::NP && p < max; ++p) out[p] = L::P[p];
  return L::NP;
}
int fused_kind_paths(int code, PathDef* out, int max) {
  auto f = [&]() -> int {
    switch (code) {
#define K_(c, f, T) \
  case c:           \
    return kind_paths<Family<f>::T>(out, max);
      K_(0, 0, First) K_(1, 0, Mid) K_(2, 0, Last) K_(3, 1, First) K_(4, 1, Mid) K_(5, 1, Last)
      K_(6, 2, First) K_(7, 2, Mid) K_(8, 2, Last)
#undef K_
      default: return 0;
    }
  };
  return f();
}

}  // namespace e3gnn

#ifdef E3GNN_STAMPS
// diagnostic builds only: the device buffer the middle backward's phase
// stamps go to ([waves][8] u64; null disables)
extern "C" int e3gnn_debug_stamps(void* p) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(e3gnn::g_stamp_buf), &p, sizeof(p));
}
#endif
