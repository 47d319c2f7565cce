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
// Two tile shapes, chosen per problem (TgProb::mode): 64x64x16 -- 256
// threads = 4 waves, each wave one 32x32 accumulator -- for problems with
// enough output tiles to fill the chip, and 32x32x32 with the four waves
// splitting each k step (8 k each) for the small ones (the fine-tune batch's
// linears: M ~ 400-2000 rows, ~100 tiles of 64x64 = one wave on a tenth of
// the SIMDs); the four partial accumulators are summed through LDS in wave
// order (deterministic).  Operands staged k-major through LDS (As[k][m],
// Bs[k][n]) so the MFMA operand reads are unit-stride; the next k-steps'
// loads are in flight during the current step's MFMAs.
#include "common.h"
#include "tgemm.h"

#include <cstdio>
#include <cstdlib>

namespace e3gnn {
namespace {

// tile shapes: MODE 0 = 64x64x16 (waves 2 x 2 over the tile), MODE 1 =
// 32x32xTG_M1_BK (waves over k); NS = register ring depth in k steps
#ifndef TG_M1_BK
#define TG_M1_BK 32
#endif
#ifndef TG_NS0
#define TG_NS0 4
#endif
#ifndef TG_NS1
#define TG_NS1 4
#endif
template <int MODE> struct TgShape {
  static constexpr int BM = MODE ? 32 : 64;         // tile rows = columns
  static constexpr int BK = MODE ? TG_M1_BK : 16;   // k per step
  static constexpr int NS = MODE ? TG_NS1 : TG_NS0;
  static constexpr int TEL = BK * BM / 256;         // elements of one operand slab per thread
  static constexpr int TLD = BM + 4;                // LDS row (k) stride, floats
  static constexpr int SLAB = BK * TLD;             // one LDS buffer of one operand
};
constexpr int cmax(int a, int b) { return a > b ? a : b; }
// staging (2 operands x 2 buffers) of either shape, and MODE 1's 4 x 16 x 64 partials
constexpr int LDS_FLOATS = cmax(cmax(4 * TgShape<0>::SLAB, 4 * TgShape<1>::SLAB), 4 * 16 * 64);
constexpr int OOB = 0x7ffffff0;        // outside every descriptor: reads 0
typedef float f32x16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ int tg_find(const TgBatch& b, int tile) {
  int p = 0;
#pragma unroll
  for (int i = 1; i < TG_MAX_PROBS; ++i) p += (i < b.nprob && tile >= b.tile_begin[i]) ? 1 : 0;
  return p;
}

__device__ __forceinline__ int rfl(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int64_t rfl(int64_t v) {
  const uint64_t u = (uint64_t)v;
  return (int64_t)(((uint64_t)(unsigned)__builtin_amdgcn_readfirstlane((int)(u >> 32)) << 32) |
                   (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)u));
}

// One operand of the tile, element (r, k) in the TgLay layout, read through
// a buffer descriptor at the operand's base: the thread's TEL elements of a
// BK x BM slab, element e = 256 i + tid walking the contiguous dimension
// fastest (k contiguous: k = e % BK, r = e / BK; else r = e % BM, k = e / BM).
// Their byte offsets at the segment start and LDS slots are fixed for the
// launch; a k step adds a scalar offset (k steps never straddle a segment: a
// segment is padded to whole steps) -- no per-element address arithmetic in
// the k loop.  Elements past the rows or a segment's ks read 0 (OOB offset).
constexpr int TG_RECORDS = 0x7fff0000;
constexpr int TG_MAX_SEG = 9;   // K segments of a part (2l + 1 <= 9: lmax 4)   // descriptor size: every real offset is below, OOB above
template <int TEL>
struct OpB {
  __amdgpu_buffer_rsrc_t R;
  int vo[TEL];   // byte offset at k = 0 of a segment, OOB past the rows
  int kk[TEL];   // k within a step
  int lo[TEL];   // LDS slot S[k][r]
  int kst4, sst4, ks, sps;   // bytes per k, per segment; segment rows; steps per segment
};
template <int MODE>
__device__ __forceinline__ void opb_init(OpB<TgShape<MODE>::TEL>& o, const TgLay& L, int r0, int rmax) {
  using Sh = TgShape<MODE>;
  constexpr int BM = Sh::BM, BK = Sh::BK, TEL = Sh::TEL;
  o.R = __builtin_amdgcn_make_buffer_rsrc((void*)L.X, (short)0, TG_RECORDS, 0x00020000);
  const int rep = rfl(L.rep), rs = rfl(L.rs);
  const int ld = rfl(L.ld), kst = rfl(L.kst);
  const bool kfast = kst == 1;
  const unsigned mag = rep > 1 ? 0xffffffffu / (unsigned)rep + 1u : 0u;
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < TEL; ++i) {
    const int e = 256 * i + tid;
    const int r = kfast ? (e / BK) : (e % BM), k = kfast ? (e % BK) : (e / BM);
    const int rr = r0 + r;
    const int q = rep > 1 ? (int)__umulhi((unsigned)rr, mag) : rr;   // rr / rep (rep <= 9)
    o.vo[i] = rr < rmax ? (q * ld + (rr - q * rep) * rs + k * kst) * 4 : OOB;
    o.kk[i] = k;
    o.lo[i] = k * Sh::TLD + r;
  }
  o.kst4 = kst * 4;
  o.sst4 = rfl(L.sst) * 4;
  o.ks = rfl(L.ks);
  o.sps = (o.ks + BK - 1) / BK;
}

// Main loop: LDS double buffer + a ring of NS register slots, so the loads of
// k-step kt + NS - 1 are in flight while step kt computes (small GEMMs are
// latency-bound).  The loop is unrolled by NS so every slot index is a
// compile-time constant, and every iteration issues the same loads (past the
// split's end at OOB offsets, the compute skipped), so the compiler's wait
// counts are exact: a slot's consumer waits for that slot's loads only.

template <int MODE>
__device__ __forceinline__ void tg_tile(const TgProb& P, int local, float* lds) {
  using Sh = TgShape<MODE>;
  constexpr int BM = Sh::BM, BK = Sh::BK, TLD = Sh::TLD, SLAB = Sh::SLAB, NS = Sh::NS, TEL = Sh::TEL;
  float* As = lds;              // [2][BK][TLD]
  float* Bs = lds + 2 * SLAB;   // [2][BK][TLD]
  const int s = local / P.tiles_mn, mn = local - s * P.tiles_mn;
  const int tm = mn / P.tiles_n, tn = mn - tm * P.tiles_n;
  const int m0 = tm * BM, n0 = tn * BM;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = MODE ? 0 : wave >> 1, wc = MODE ? 0 : wave & 1;
  // the problem's scalars as values computed in registers (readfirstlane):
  // the compiler would otherwise re-load them from the kernel arguments inside
  // the k loop, and each such scalar load's wait also drains the outstanding
  // LDS operations (one counter)
  const int PM = rfl(P.M), PN = rfl(P.N), PK1 = rfl(P.K1), PK2 = rfl(P.K2);
  // op(A)(m, k) and op(B)(n, k): B enters as the (n x k) operand
  OpB<TEL> a1, b1, a2, b2;
  opb_init<MODE>(a1, P.A1, m0, PM);
  opb_init<MODE>(b1, P.B1, n0, PN);
  opb_init<MODE>(a2, P.A2, m0, PM);
  opb_init<MODE>(b2, P.B2, n0, PN);
  // the k steps over the concatenated K = K1 + K2: each part's segments
  // padded to whole steps
  const int nk1 = a1.ks > 0 ? (PK1 / a1.ks) * a1.sps : 0;
  const int nk = nk1 + (a2.ks > 0 ? (PK2 / a2.ks) * a2.sps : 0);
  // the tile's k-step ranges (block sparsity): [kb1, ke1) of the first pair,
  // [nk1 + kb2, nk1 + ke2) of the second; step j of the tile's sequence is
  // kb1 + j (j < n1) or nk1 + kb2 + j - n1.  This split's slice of it:
  // [jb, je) (a split past the tile's steps has none: zero partials)
  int kb1 = 0, n1 = nk1, kb2 = 0, n2 = nk - nk1;
  if (P.kr) {   // the table is per 64 x 64 tile: a 32 x 32 tile takes its hull's range
    const int* q = P.kr + 4 * ((MODE ? tm >> 1 : tm) * P.kr_sm + (MODE ? tn >> 1 : tn));
    kb1 = rfl(q[0] / BK);
    n1 = max(0, rfl((q[1] + BK - 1) / BK) - kb1);
    kb2 = rfl(q[2] / BK);
    n2 = max(0, rfl((q[3] + BK - 1) / BK) - kb2);
  }
  const int jb = rfl(s * P.ksteps), je = min(n1 + n2, jb + rfl(P.ksteps));
  auto kt_of = [&](int j) { return j < n1 ? kb1 + j : nk1 + kb2 + (j - n1); };
  float ra[NS][TEL], rb[NS][TEL];
  // step j's operands (j >= je: zeros, same instructions); the operand
  // pair is selected arithmetically, not branched on.  Loads run in step
  // order, so a cursor carries the next load's part, segment and row in it
  // (scalar selects per load; the segment index of a part step t -- t / sps
  // -- is found by compares only where the cursor starts or changes part)
  auto seg_of = [&](int t, int sps, int& seg, int& kin) {
    seg = 0;
#pragma unroll
    for (int c = 1; c < TG_MAX_SEG; ++c) seg += t >= c * sps;
    kin = (t - seg * sps) * BK;
  };
  int cj = jb, cseg, ckin;
  bool cfirst = kt_of(jb) < nk1;
  seg_of(cfirst ? kt_of(jb) : kt_of(jb) - nk1, cfirst ? a1.sps : a2.sps, cseg, ckin);
  int seg2, kin2;   // where the second pair's range of this tile starts
  seg_of(kb2, a2.sps, seg2, kin2);
  auto load1 = [&](const OpB<TEL>& o1, const OpB<TEL>& o2, bool first, bool live, int seg, int kin, float (&x)[TEL]) {
    const int soff = kin * (first ? o1.kst4 : o2.kst4) + seg * (first ? o1.sst4 : o2.sst4);
    const int kmax = first ? o1.ks : o2.ks;
#pragma unroll
    for (int i = 0; i < TEL; ++i) {
      const int vo = first ? o1.vo[i] : o2.vo[i];
      const int kk = first ? o1.kk[i] : o2.kk[i];
      const int v = (live && kin + kk < kmax) ? vo : OOB;
      x[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(first ? o1.R : o2.R, v, soff, 0));
    }
  };
  auto load = [&](float (&xa)[TEL], float (&xb)[TEL]) {   // step cj, then advance
    const bool live = cj < je;
    load1(a1, a2, cfirst, live, cseg, ckin, xa);
    load1(b1, b2, cfirst, live, cseg, ckin, xb);
    ++cj;
    const bool sw = cfirst && cj == n1;             // into the second pair's range
    const int spsT = (cfirst ? a1.sps : a2.sps) * BK;
    const bool wrap = ckin + BK >= spsT;
    const int nkin = wrap ? 0 : ckin + BK, nseg = wrap ? cseg + 1 : cseg;
    ckin = sw ? kin2 : nkin;
    cseg = sw ? seg2 : nseg;
    cfirst = cfirst && !sw;
  };
  auto store = [&](int buf, int j, const float (&xa)[TEL], const float (&xb)[TEL]) {
    const bool first = j < n1;
#pragma unroll
    for (int i = 0; i < TEL; ++i) {
      As[buf * SLAB + (first ? a1.lo[i] : a2.lo[i])] = xa[i];
      Bs[buf * SLAB + (first ? b1.lo[i] : b2.lo[i])] = xb[i];
    }
  };
  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  if (jb < je) {
#pragma unroll
    for (int u = 0; u < NS - 1; ++u) load(ra[u], rb[u]);
    store(0, jb, ra[0], rb[0]);
    __syncthreads();
#pragma unroll 1
    for (int j0 = jb; j0 < je; j0 += NS) {
#pragma unroll
      for (int u = 0; u < NS; ++u) {
        const int j = j0 + u;
        // slot of step j + NS - 1 is (u + NS - 1) % NS: the one step j - 1 used
        load(ra[(u + NS - 1) % NS], rb[(u + NS - 1) % NS]);
        if (j < je) {
          const int buf = (j - jb) & 1;
          // MODE 0: the step's 16 k on the wave's 32 x 32 quarter; MODE 1:
          // the wave's 8 of the step's 32 k on the whole 32 x 32 tile
          constexpr int KW = MODE ? BK / 4 : BK;
          const int kw0 = MODE ? wave * KW : 0;
#pragma unroll
          for (int kk = 0; kk < KW; kk += 2) {
            const float av = As[buf * SLAB + (kw0 + kk + (lane >> 5)) * TLD + wr * 32 + (lane & 31)];
            const float bv = Bs[buf * SLAB + (kw0 + kk + (lane >> 5)) * TLD + wc * 32 + (lane & 31)];
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
          }
        }
        // step j + 1 from its slot into the other LDS buffer
        store((j + 1 - jb) & 1, j + 1, ra[(u + 1) % NS], rb[(u + 1) % NS]);
        __syncthreads();
      }
    }
  } else if (P.kr && rfl(P.beta) && rfl(P.splits) <= 1) {
    return;   // nothing to add to this tile (uniform over the workgroup)
  }
  // the tile's values this wave finishes: MODE 0 its own 16 accumulator
  // registers; MODE 1 registers 4 wave .. 4 wave + 3 of the sum of the four
  // waves' partial accumulators (LDS, added in wave order)
  constexpr int RN = MODE ? 4 : 16;
  const int r0 = MODE ? 4 * wave : 0;
  float v[RN];
  if (MODE) {
    // every wave is past the loop's last barrier: the staging buffers are free
#pragma unroll
    for (int r = 0; r < 16; ++r) lds[(wave * 16 + r) * 64 + lane] = acc[r];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      const int r = r0 + j;
      v[j] = ((lds[r * 64 + lane] + lds[(16 + r) * 64 + lane]) + lds[(32 + r) * 64 + lane]) +
             lds[(48 + r) * 64 + lane];
    }
  } else {
#pragma unroll
    for (int j = 0; j < RN; ++j) v[j] = acc[j];
  }
  const int col = n0 + wc * 32 + (lane & 31);
  if (col >= PN) return;
  // D lane l, reg r: row 8 (r >> 2) + 4 (l >> 5) + (r & 3), column l & 31
  auto row_of = [&](int j) {
    const int r = r0 + j;
    return m0 + wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
  };
  typedef __attribute__((address_space(1))) float* gp;
  if (rfl(P.splits) > 1) {   // partial tile to this split's slab; k_tgemm_reduce finishes
    const gp w = (gp)(uintptr_t)rfl((int64_t)(uintptr_t)(P.ws + (int64_t)s * PM * PN));
#pragma unroll
    for (int j = 0; j < RN; ++j)
      if (row_of(j) < PM) w[(int64_t)row_of(j) * PN + col] = v[j];
    return;
  }
  const gp C = (gp)(uintptr_t)rfl((int64_t)(uintptr_t)P.C);
  const int64_t ldc = rfl(P.ldc);
  const int crep = rfl(P.crep), crs = rfl(P.crs), cns = rfl(P.cns);
  const float alpha = __builtin_bit_cast(float, rfl(__builtin_bit_cast(int, P.alpha)));
  // m / crep by a multiply-high (exact for crep <= 9, m < 2^28): an integer
  // division per output element would cost ~30 vector instructions
  const unsigned cmag = crep > 1 ? 0xffffffffu / (unsigned)crep + 1u : 0u;
  auto at = [&](int j) {
    const int m = row_of(j);
    const int q = crep > 1 ? (int)__umulhi((unsigned)m, cmag) : m;
    return (int64_t)q * ldc + (m - q * crep) * crs + (int64_t)col * cns;
  };
  float old[RN];
  if (rfl(P.beta)) {   // all old values in flight at once
#pragma unroll
    for (int j = 0; j < RN; ++j) old[j] = row_of(j) < PM ? C[at(j)] : 0.f;
  } else {
#pragma unroll
    for (int j = 0; j < RN; ++j) old[j] = 0.f;
  }
#pragma unroll
  for (int j = 0; j < RN; ++j)
    if (row_of(j) < PM) C[at(j)] = old[j] + alpha * v[j];
}

__global__ __launch_bounds__(256) void k_tgemm(TgBatch batch) {
  __shared__ __attribute__((aligned(16))) float lds[LDS_FLOATS];
  const TgProb& P = batch.p[tg_find(batch, blockIdx.x)];
  const int local = blockIdx.x - P.tile_begin;
  if (rfl(P.mode))
    tg_tile<1>(P, local, lds);
  else
    tg_tile<0>(P, local, lds);
}

// C = beta C + alpha sum_s ws[s] over the split problems, s in order
__global__ __launch_bounds__(256) void k_tgemm_reduce(TgRedBatch batch) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int p = -1;
#pragma unroll
  for (int q = 0; q < TG_MAX_RED; ++q)
    if (q < batch.n && i >= batch.lo[q] && i < batch.hi[q]) p = q;
  if (p < 0) return;
  const TgRed& P = batch.p[p];
  const int64_t e = i - batch.lo[p], mn = (int64_t)P.M * P.N;
  const int row = (int)(e / P.N), col = (int)(e - (int64_t)row * P.N);
  // slabs 0, 1, 2, ... added in order; sixteen loads in flight at a time
  // (a split count of ~70 read one dependent load at a time took ~70
  // latencies)
  const float* w = P.ws + e;
  float sum = 0.f;
  int s = 0;
#pragma unroll 1
  for (; s + 16 <= P.splits; s += 16) {
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = w[(int64_t)(s + u) * mn];
#pragma unroll
    for (int u = 0; u < 16; ++u) sum += v[u];
  }
#pragma unroll 1
  for (; s + 4 <= P.splits; s += 4) {
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = w[(int64_t)(s + u) * mn];
#pragma unroll
    for (int u = 0; u < 4; ++u) sum += v[u];
  }
#pragma unroll 1
  for (; s < P.splits; ++s) sum += w[(int64_t)s * mn];
  float* c = P.C + (int64_t)(row / P.crep) * P.ldc + (row % P.crep) * P.crs + (int64_t)col * P.cns;
  const float v = P.alpha * sum;
  *c = P.beta ? *c + v : v;
}

}  // namespace

// split-K policy (E3GNN_TG_SPLIT="min_ksteps,target_wgs,ksteps_per_split" for
// A/B timing, in 64 x 64 x 16 tile steps): split only a long K (the extra
// reduction launch costs ~5 us).  E3GNN_TG_SMALL: problems with fewer
// (64 x 64 tiles x splits) than this take the 32 x 32 x 32 k-split tiles
static int tg_policy(int i) {
  static int v[5] = {-1, -1, -1, -1, -1};
  if (v[0] < 0) {
    v[0] = 32, v[1] = 1024, v[2] = 8, v[3] = 256, v[4] = 0;
    if (const char* e = std::getenv("E3GNN_TG_SPLIT")) std::sscanf(e, "%d,%d,%d", &v[0], &v[1], &v[2]);
    if (const char* e = std::getenv("E3GNN_TG_SMALL")) v[3] = std::atoi(e);
    if (const char* e = std::getenv("E3GNN_TG_SMALL_SPLIT")) v[4] = std::atoi(e);
  }
  return v[i];
}
int tg_splits(int64_t M, int64_t N, int64_t K) {
  const int64_t tiles = ((M + 63) / 64) * ((N + 63) / 64);
  const int64_t nk = (K + 15) / 16;
  // few output tiles and a long K (the edge-summed weight gradients: K = 2E
  // ~ 24k rows onto 64 x 960 outputs): split K so the launch has ~target
  // workgroups of >= ksteps_per_split k-steps each
  if (tiles >= tg_policy(1) / 2 || nk < tg_policy(0)) return 1;
  int64_t s = std::min<int64_t>((tg_policy(1) + tiles - 1) / tiles, nk / tg_policy(2));
  return (int)std::max<int64_t>(1, std::min<int64_t>(s, 256));
}

bool tg_add(TgBatch& b, TgProb p) {
  if (b.nprob >= TG_MAX_PROBS || p.M < 0 || p.N < 0 || p.K1 < 0 || p.K2 < 0) return false;
  if (p.M == 0 || p.N == 0) return true;
  if (p.K2 == 0) p.A2 = p.A1, p.B2 = p.B1, p.A2.ks = p.B2.ks = 0;   // no second pair
  if (p.splits < 1) p.splits = 1;
  p.mode = ((int64_t)((p.M + 63) / 64) * ((p.N + 63) / 64) * p.splits < tg_policy(3) &&
            (p.splits == 1 || tg_policy(4))) ? 1 : 0;
  const int BM = p.mode ? 32 : 64, BK = p.mode ? TG_M1_BK : 16;
  auto steps = [BK](int K, const TgLay& a, const TgLay& b) {
    if (K <= 0) return 0;
    if (a.ks <= 0 || a.ks != b.ks || K % a.ks || K / a.ks > TG_MAX_SEG || a.rep < 1 || b.rep < 1 ||
        a.rep > 9 || b.rep > 9)
      return -1;
    return (K / a.ks) * ((a.ks + BK - 1) / BK);
  };
  const int s1 = steps(p.K1, p.A1, p.B1), s2 = steps(p.K2, p.A2, p.B2);
  if (s1 < 0 || s2 < 0 || p.crep < 1 || p.crep > 9 || (int64_t)p.M * 9 >= (1 << 28)) return false;
  const int nk = s1 + s2;
  p.tiles_n = (p.N + BM - 1) / BM;
  p.tiles_mn = ((p.M + BM - 1) / BM) * p.tiles_n;
  p.ksteps = std::max(1, (nk + p.splits - 1) / p.splits);
  p.splits = std::max(1, (nk + p.ksteps - 1) / p.ksteps);   // never above the request: the workspace holds it
  p.tile_begin = b.total_tiles;
  b.tile_begin[b.nprob] = p.tile_begin;
  b.total_tiles += p.tiles_mn * p.splits;
  if (p.splits > 1) {
    p.red_begin = b.red_total;
    b.red_total += (int64_t)p.M * p.N;
  }
  b.p[b.nprob++] = p;
  return true;
}

bool tg_red_add(TgRedBatch& r, const TgRed& q) {
  if (r.n >= TG_MAX_RED || q.splits <= 1 || q.M <= 0 || q.N <= 0) return false;
  r.lo[r.n] = r.total;
  r.total += (int64_t)q.M * q.N;
  r.hi[r.n] = r.total;
  r.p[r.n++] = q;
  return true;
}

hipError_t launch_tgemm_reduce(const TgRedBatch& r, hipStream_t s) {
  if (r.total > 0)
    hipLaunchKernelGGL(k_tgemm_reduce, dim3((unsigned)((r.total + 255) / 256)), dim3(256), 0, s, r);
  return hipGetLastError();
}

hipError_t launch_tgemm(const TgBatch& b, hipStream_t s, bool reduce) {
  if (b.total_tiles <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_tgemm, dim3(b.total_tiles), dim3(256), 0, s, b);
  if (reduce && b.red_total > 0) {
    TgRedBatch r;
    for (int i = 0; i < b.nprob; ++i) {
      const TgProb& p = b.p[i];
      if (p.splits > 1)
        tg_red_add(r, TgRed{p.ws, p.C, p.ldc, p.crep, p.crs, p.cns, p.M, p.N, p.splits, p.alpha, p.beta});
    }
    return launch_tgemm_reduce(r, s);
  }
  return hipGetLastError();
}

}  // namespace e3gnn
