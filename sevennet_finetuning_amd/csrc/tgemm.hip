// Grouped f32 GEMM for the fine-tune step (train_explicit.py): the e3nn linears
// as dense matrices, their transposes and the weight gradients, on gfx950
// matrix cores (v_mfma_f32_32x32x2_f32), f32 in / f32 accumulate.
//
//   C = beta C + alpha (op(A1) op(B1) [+ op(A2) op(B2)])      beta in {0, 1}
//
// op(X) = X or X^T (row-major storage with a leading dimension), an optional
// second operand pair K-concatenated into the same accumulator (x W_si1^T +
// y W_sc^T: one problem, one rounding of each sum), up to TG_MAX_PROBS
// independent problems per launch.  Problems with a long K (the edge-summed
// weight gradients, K = 2E rows) are split over K: each split writes its
// partial tile to a workspace slab and one reduction launch adds the slabs in
// a fixed order (deterministic, no atomics).  Replaces the rocBLAS / hipBLASLt
// calls torch made for these products (trainer.py:155-222 under
// force_output.py:158-215's create_graph).
//
// Tile 64x64x16, 256 threads = 4 waves, each wave one 32x32 accumulator;
// operands staged k-major through LDS (As[k][m], Bs[k][n]) so the MFMA operand
// reads are unit-stride; the next k-step's loads are issued before the
// current step's MFMAs.  Vector (16-byte) loads along the contiguous dimension
// when the operand's base and leading dimension allow it.
#include "common.h"
#include "tgemm.h"

namespace e3gnn {
namespace {

constexpr int TBM = 64, TBN = 64, TBK = 16, TPAD = 4;
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int tg_find(const TgBatch& b, int tile) {
  int p = 0;
#pragma unroll 1
  for (int i = 1; i < b.nprob; ++i)
    if (tile >= b.p[i].tile_begin) p = i;
  return p;
}

// op(X)(r, k) of a row-major X with leading dimension ld (trans: X[k][r])
struct Opnd {
  const float* X;
  int64_t ld;
  int trans, vec;  // vec: 16-byte loads along the contiguous dimension
};

// One 16 x 64 (k x r) slab of op(X): 256 threads x 4 elements.  Not
// transposed (X[r][k]): thread -> (r = e / 4, k quad = e % 4), 4 consecutive k;
// transposed (X[k][r]): thread -> (k = e / 16, r quad = e % 16), 4 consecutive r.
__device__ __forceinline__ void tg_load(const Opnd& o, int r0, int rmax, int k0, int kmax, float (&v)[4]) {
  const int tid = threadIdx.x;
  if (!o.trans) {
    const int r = r0 + (tid >> 2), k = k0 + 4 * (tid & 3);
    const float* p = o.X + (int64_t)r * o.ld + k;
    if (r < rmax && o.vec && k + 3 < kmax) {
      const float4 q = *reinterpret_cast<const float4*>(p);
      v[0] = q.x, v[1] = q.y, v[2] = q.z, v[3] = q.w;
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = (r < rmax && k + i < kmax) ? p[i] : 0.f;
    }
  } else {
    const int k = k0 + (tid >> 4), r = r0 + 4 * (tid & 15);
    const float* p = o.X + (int64_t)k * o.ld + r;
    if (k < kmax && o.vec && r + 3 < rmax) {
      const float4 q = *reinterpret_cast<const float4*>(p);
      v[0] = q.x, v[1] = q.y, v[2] = q.z, v[3] = q.w;
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = (k < kmax && r + i < rmax) ? p[i] : 0.f;
    }
  }
}
__device__ __forceinline__ void tg_store(const Opnd& o, float (*S)[TBM + TPAD], const float (&v)[4]) {
  const int tid = threadIdx.x;
  if (!o.trans) {
    const int r = tid >> 2, k = 4 * (tid & 3);
#pragma unroll
    for (int i = 0; i < 4; ++i) S[k + i][r] = v[i];
  } else {
    const int k = tid >> 4, r = 4 * (tid & 15);
    *reinterpret_cast<float4*>(&S[k][r]) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

__global__ __launch_bounds__(256) void k_tgemm(TgBatch batch) {
  __shared__ __attribute__((aligned(16))) float As[2][TBK][TBM + TPAD];
  __shared__ __attribute__((aligned(16))) float Bs[2][TBK][TBN + TPAD];
  const TgProb& P = batch.p[tg_find(batch, blockIdx.x)];
  const int local = blockIdx.x - P.tile_begin;
  const int s = local / P.tiles_mn, mn = local - s * P.tiles_mn;
  const int tm = mn / P.tiles_n, tn = mn - tm * P.tiles_n;
  const int m0 = tm * TBM, n0 = tn * TBN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  // this split's k steps over the concatenated K = K1 + K2 (each part padded
  // to whole k-steps)
  const int nk1 = (P.K1 + TBK - 1) / TBK, nk = nk1 + (P.K2 + TBK - 1) / TBK;
  const int kb = s * P.ksteps, ke = min(nk, kb + P.ksteps);
  // op(A)(m, k) and op(B)(n, k): B enters as the (n x k) operand
  const Opnd a1{P.A1, P.lda1, P.ta1, P.va1}, b1{P.B1, P.ldb1, !P.tb1, P.vb1};
  const Opnd a2{P.A2, P.lda2, P.ta2, P.va2}, b2{P.B2, P.ldb2, !P.tb2, P.vb2};
  float ra[4], rb[4];
  auto load = [&](int kt) {
    if (kt < nk1) {
      tg_load(a1, m0, P.M, kt * TBK, P.K1, ra);
      tg_load(b1, n0, P.N, kt * TBK, P.K1, rb);
    } else {
      tg_load(a2, m0, P.M, (kt - nk1) * TBK, P.K2, ra);
      tg_load(b2, n0, P.N, (kt - nk1) * TBK, P.K2, rb);
    }
  };
  auto store = [&](int buf, int kt) {
    if (kt < nk1) {
      tg_store(a1, As[buf], ra);
      tg_store(b1, Bs[buf], rb);
    } else {
      tg_store(a2, As[buf], ra);
      tg_store(b2, Bs[buf], rb);
    }
  };
  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  if (kb < ke) {
    load(kb);
    store(0, kb);
    __syncthreads();
#pragma unroll 1
    for (int kt = kb; kt < ke; ++kt) {
      const int buf = (kt - kb) & 1;
      if (kt + 1 < ke) load(kt + 1);
#pragma unroll
      for (int kk = 0; kk < TBK; kk += 2) {
        const float av = As[buf][kk + (lane >> 5)][wr * 32 + (lane & 31)];
        const float bv = Bs[buf][kk + (lane >> 5)][wc * 32 + (lane & 31)];
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
      }
      if (kt + 1 < ke) store(buf ^ 1, kt + 1);
      __syncthreads();
    }
  }
  const int col = n0 + wc * 32 + (lane & 31);
  if (col >= P.N) return;
  // D lane l, reg r: row 8 (r >> 2) + 4 (l >> 5) + (r & 3), column l & 31
  if (P.splits > 1) {   // partial tile to this split's slab; k_tgemm_reduce finishes
    float* w = P.ws + (int64_t)s * P.M * P.N;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (row < P.M) w[(int64_t)row * P.N + col] = acc[r];
    }
    return;
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m0 + wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (row >= P.M) continue;
    float* c = P.C + (int64_t)row * P.ldc + col;
    const float v = P.alpha * acc[r];
    *c = P.beta ? *c + v : v;
  }
}

// C = beta C + alpha sum_s ws[s] over the split problems, s in order
__global__ __launch_bounds__(256) void k_tgemm_reduce(TgBatch batch) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll 1
  for (int p = 0; p < batch.nprob; ++p) {
    const TgProb& P = batch.p[p];
    if (P.splits <= 1 || i < P.red_begin || i >= P.red_begin + (int64_t)P.M * P.N) continue;
    const int64_t e = i - P.red_begin;
    const int row = (int)(e / P.N), col = (int)(e - (int64_t)row * P.N);
    float sum = 0.f;
#pragma unroll 1
    for (int s = 0; s < P.splits; ++s) sum += P.ws[(int64_t)s * P.M * P.N + e];
    float* c = P.C + (int64_t)row * P.ldc + col;
    const float v = P.alpha * sum;
    *c = P.beta ? *c + v : v;
  }
}

}  // namespace

int tg_splits(int64_t M, int64_t N, int64_t K) {
  const int64_t tiles = ((M + TBM - 1) / TBM) * ((N + TBN - 1) / TBN);
  const int64_t nk = (K + TBK - 1) / TBK;
  // long K and few output tiles: split so the launch has ~512 tiles of >= 32
  // k-steps each (the edge-summed weight gradients: K = 2E ~ 24k rows)
  if (nk < 128 || tiles >= 256) return 1;
  int64_t s = std::min<int64_t>(512 / std::max<int64_t>(tiles, 1), nk / 32);
  return (int)std::max<int64_t>(1, std::min<int64_t>(s, 128));
}

bool tg_add(TgBatch& b, TgProb p) {
  if (b.nprob >= TG_MAX_PROBS || p.M < 0 || p.N < 0 || p.K1 < 0 || p.K2 < 0) return false;
  if (p.M == 0 || p.N == 0) return true;
  auto al = [](const void* q, int64_t ld) { return ((uintptr_t)q & 15) == 0 && ld % 4 == 0; };
  p.va1 = al(p.A1, p.lda1);
  p.vb1 = al(p.B1, p.ldb1);
  p.va2 = p.K2 > 0 ? al(p.A2, p.lda2) : 0;
  p.vb2 = p.K2 > 0 ? al(p.B2, p.ldb2) : 0;
  const int nk = (p.K1 + TBK - 1) / TBK + (p.K2 + TBK - 1) / TBK;
  p.tiles_n = (p.N + TBN - 1) / TBN;
  p.tiles_mn = ((p.M + TBM - 1) / TBM) * p.tiles_n;
  if (p.splits < 1) p.splits = 1;
  p.ksteps = std::max(1, (nk + p.splits - 1) / p.splits);
  p.splits = std::max(1, (nk + p.ksteps - 1) / p.ksteps);
  p.tile_begin = b.total_tiles;
  b.total_tiles += p.tiles_mn * p.splits;
  if (p.splits > 1) {
    p.red_begin = b.red_total;
    b.red_total += (int64_t)p.M * p.N;
  }
  b.p[b.nprob++] = p;
  return true;
}

hipError_t launch_tgemm(const TgBatch& b, hipStream_t s) {
  if (b.total_tiles <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_tgemm, dim3(b.total_tiles), dim3(256), 0, s, b);
  if (b.red_total > 0)
    hipLaunchKernelGGL(k_tgemm_reduce, dim3((unsigned)((b.red_total + 255) / 256)), dim3(256), 0, s, b);
  return hipGetLastError();
}

}  // namespace e3gnn
