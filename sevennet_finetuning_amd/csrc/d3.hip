// DFT-D3 dispersion (zero and Becke-Johnson damping) with the C6(CN) chain,
// energy + forces + virial -- SURVEY.md §8f row 4, the reference's LAMMPS
// pair style d3 (sevenn/pair_e3gnn/pair_d3.cu:808-2056).
//
// Same arithmetic as the reference (fp32 per pair-image term, C6 interpolation
// in fp64, units bohr / hartree), different decomposition.  The reference
// walks all unordered pairs (i >= j) x all cell images and scatters into both
// atoms with float/double atomics.  Here:
//  * atoms are binned (bins of >= ~20 bohr along each lattice vector, sorted
//    by bin on the host) and one workgroup owns one atom i: its waves walk
//    the stencil of (bin, image) cells around i's bin -- each (bin, image)
//    pair once -- and skip every cell whose centre is farther than
//    rc + half a bin diagonal, so only (j, image) items near the cutoff
//    sphere are evaluated (the all-images scheme evaluates 88 % / 99 % of its
//    items outside rthr / cn_thr on an 8,000-atom box);
//  * every per-atom output (CN_i, dE/dCN_i, F_i) is written by exactly one
//    workgroup -- no atomics, bitwise deterministic -- at twice the pair
//    evaluations of the i >= j triangle; per-row energy/virial partials are
//    reduced in a fixed order.
//
//   k_d3_cn      CN_i = sum_{j,T} 1/(1+exp(-K1((rcov_i+rcov_j)/r - 1)))   (:1051-1104)
//   k_d3_c6tab   C6_ij, dC6_ij/dCN_i for all ordered pairs (:808-887), n <= 32768
//   k_d3_disp    E, F_i (direct), virial, dE/dCN_i (:1273-1505 zero, :1558-1768 BJ)
//   k_d3_chain   F_i += (dE/dCN_i + dE/dCN_j) dCN/dr r_hat, virial   (:1812-1976)
//   k_d3_reduce  energy and virial over rows, fixed order; units to eV, eV/A
#include "d3.h"

namespace e3gnn {
namespace {

constexpr float K1 = 16.0f;
constexpr float K3 = -4.0f;
constexpr int MAXC = 5;
constexpr int BLK = 256;
constexpr int NW = BLK / 64;

__device__ __forceinline__ double block_sum(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int k = 0; k < NW; ++k) s += red[k];   // fixed order
  return s;
}

// Visit every (j, image) with |x_j + T - x_i|^2 <= rc2 (or < when `strict`)
// except (i, T = 0): wave w takes stencil cells w, w + NW, ...; lanes take
// the atoms of the cell.  body(j, type_j, rx, ry, rz, r2).  x: (x, y, z,
// type bits) per atom -- one 16-byte load per item.
template <bool STRICT, class Body>
__device__ __forceinline__ void for_pairs(const D3Grid& g, const int* __restrict__ off, int n_off,
                                          float cull2, float rc2, const float4* __restrict__ x,
                                          int i, Body&& body) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const float4 xi = x[i];
  const float xi0 = xi.x, xi1 = xi.y, xi2 = xi.z;
  const int bid = g.bin_of[i];
  const int bi2 = bid % g.nb[2], bi1 = (bid / g.nb[2]) % g.nb[1], bi0 = bid / (g.nb[2] * g.nb[1]);
  for (int o = wave; o < n_off; o += NW) {
    const int g0 = bi0 + off[3 * o], g1 = bi1 + off[3 * o + 1], g2 = bi2 + off[3 * o + 2];
    // cell centre in fractional coordinates; its floor is the image (exact:
    // small integers, inv_nb within 1 ulp)
    const float c0 = (g0 + 0.5f) * g.inv_nb[0], c1 = (g1 + 0.5f) * g.inv_nb[1],
                c2 = (g2 + 0.5f) * g.inv_nb[2];
    const int T0 = (int)floorf(c0), T1 = (int)floorf(c1), T2 = (int)floorf(c2);
    if (g.cull) {
      const float dx = c0 * g.lat[0] + c1 * g.lat[3] + c2 * g.lat[6] - xi0;
      const float dy = c0 * g.lat[1] + c1 * g.lat[4] + c2 * g.lat[7] - xi1;
      const float dz = c0 * g.lat[2] + c1 * g.lat[5] + c2 * g.lat[8] - xi2;
      if (dx * dx + dy * dy + dz * dz > cull2) continue;
    }
    const float sx = T0 * g.lat[0] + T1 * g.lat[3] + T2 * g.lat[6];
    const float sy = T0 * g.lat[1] + T1 * g.lat[4] + T2 * g.lat[7];
    const float sz = T0 * g.lat[2] + T1 * g.lat[5] + T2 * g.lat[8];
    const bool t0 = T0 == 0 && T1 == 0 && T2 == 0;
    const int bl = ((g0 - T0 * g.nb[0]) * g.nb[1] + (g1 - T1 * g.nb[1])) * g.nb[2] +
                   (g2 - T2 * g.nb[2]);
    const int end = g.bin_start[bl + 1];
    for (int j = g.bin_start[bl] + lane; j < end; j += 64) {
      if (t0 && j == i) continue;
      const float4 xj = x[j];
      const float rx = xj.x + sx - xi0;
      const float ry = xj.y + sy - xi1;
      const float rz = xj.z + sz - xi2;
      const float r2 = rx * rx + ry * ry + rz * rz;
      if (STRICT ? !(r2 < rc2) : !(r2 <= rc2)) continue;
      body(j, __float_as_int(xj.w), rx, ry, rz, r2);
    }
  }
}

// CN_i, one workgroup per (sorted) atom
__global__ __launch_bounds__(BLK) void k_d3_cn(D3Params p, D3Grid g, const float4* __restrict__ x,
                                                const int* __restrict__ type, double* __restrict__ cn) {
  __shared__ double red[NW];
  const int i = blockIdx.x;
  const float rci = p.rcov[type[i]];
  float acc = 0.f;
  for_pairs<false>(g, g.off_cn, g.n_off_cn, g.cull2_cn, p.cn_thr, x, i,
                   [&](int, int tj, float, float, float, float r2) {
                     const float rcs = rci + p.rcov[tj];
                     acc += 1.0f / (1.0f + expf(-K1 * (rcs * rsqrtf(r2) - 1.0f)));
                   });
  const double s = block_sum((double)acc, red);
  if (threadIdx.x == 0) cn[i] = s;
}

// C6(CN_i, CN_j) and its CN derivatives (kernel_get_dC6_dCNij, :808-887),
// Gaussian weights in fp64 as the reference ("must be double").
__device__ void c6_pair(const D3Params& p, int ti, int tj, float cni, float cnj, float& c6,
                        float& dci, float& dcj) {
  const float* tab = p.c6ab + ((size_t)ti * p.ntypes + tj) * (MAXC * MAXC * 3);
  const int ma = p.mxc[ti], mb = p.mxc[tj];
  float c6mem = -1e30f, rsave = 9999.0f;
  double num = 0.0, den = 0.0, dni = 0.0, ddi = 0.0, dnj = 0.0, ddj = 0.0;
  for (int a = 0; a < ma; ++a)
    for (int b = 0; b < mb; ++b) {
      const float* e = tab + (a * MAXC + b) * 3;
      const float ref = e[0];
      if (ref > 0.0f) {
        const float ca = e[1], cb = e[2];
        const float r = (ca - cni) * (ca - cni) + (cb - cnj) * (cb - cnj);
        if (r < rsave) {
          rsave = r;
          c6mem = ref;
        }
        const double ex = exp((double)K3 * (double)r);
        num += ref * ex;
        den += ex;
        const double e2 = ex * (2.0 * K3);
        double tm = e2 * (cni - ca);
        dni += ref * tm;
        ddi += tm;
        tm = e2 * (cnj - cb);
        dnj += ref * tm;
        ddj += tm;
      }
    }
  if (den > 1e-99) {
    const double rd = 1.0 / den, u = num * rd;
    c6 = (float)u;
    dci = (float)(rd * fma(u, -ddi, dni));
    dcj = (float)(rd * fma(u, -ddj, dnj));
  } else {
    c6 = c6mem;
    dci = 0.f;
    dcj = 0.f;
  }
}

// The Gaussian weight of reference (a, b) is separable:
//   exp(K3 ((CNref_a - CN_i)^2 + (CNref_b - CN_j)^2)) = g_ia g_jb,
// because a reference CN belongs to (element, grid index) in the D3 data.  So
// each atom's factors g_ia and dg_ia/dCN_i are computed once (5 fp64 exps per
// atom) and a pair costs 25 fp64 multiply-adds instead of 25 fp64 exps.
__global__ __launch_bounds__(BLK) void k_d3_gauss(D3Params p, int n, const int* __restrict__ type,
                                                   const double* __restrict__ cn,
                                                   double* __restrict__ gw) {
  const int i = blockIdx.x * BLK + threadIdx.x;
  if (i >= n) return;
  const int ti = type[i];
  const float cni = (float)cn[i];
  for (int a = 0; a < MAXC; ++a) {
    double g = 0.0, dg = 0.0;
    if (a < p.mxc[ti]) {
      const float d = p.cnref[ti * MAXC + a] - cni;
      g = exp((double)K3 * (double)(d * d));
      dg = g * (2.0 * K3) * (double)(-d);
    }
    gw[(size_t)i * 10 + a] = g;
    gw[(size_t)i * 10 + 5 + a] = dg;
  }
}

// (C6_ij, dC6_ij/dCN_i) for every ordered pair from one evaluation per
// unordered pair (i >= j, the reference's linear triangle index, :71-74)
__global__ __launch_bounds__(BLK) void k_d3_c6tab(D3Params p, int n, const int* __restrict__ type,
                                                   const double* __restrict__ cn,
                                                   const double* __restrict__ gw,
                                                   float2* __restrict__ tab) {
  const int64_t npair = (int64_t)n * (n + 1) / 2;
  const int64_t k = (int64_t)blockIdx.x * BLK + threadIdx.x;
  if (k >= npair) return;
  int i = (int)((sqrt(8.0 * (double)k + 1.0) - 1.0) * 0.5);
  while ((int64_t)i * (i + 1) / 2 > k) --i;
  while ((int64_t)(i + 1) * (i + 2) / 2 <= k) ++i;
  const int j = (int)(k - (int64_t)i * (i + 1) / 2);
  const int ti = type[i], tj = type[j];
  float c6, dci, dcj;
  if (gw) {
    const double* gi = gw + (size_t)i * 10;
    const double* gj = gw + (size_t)j * 10;
    const float* t = p.c6ab + ((size_t)ti * p.ntypes + tj) * (MAXC * MAXC * 3);
    const int ma = p.mxc[ti], mb = p.mxc[tj];
    double num = 0.0, den = 0.0, dni = 0.0, ddi = 0.0, dnj = 0.0, ddj = 0.0;
    for (int a = 0; a < ma; ++a) {
      double rn = 0.0, rd = 0.0, rnj = 0.0, rdj = 0.0;   // sums over b
      for (int b = 0; b < mb; ++b) {
        const float ref = t[(a * MAXC + b) * 3];
        if (ref > 0.0f) {
          rn = fma((double)ref, gj[b], rn);
          rd += gj[b];
          rnj = fma((double)ref, gj[5 + b], rnj);
          rdj += gj[5 + b];
        }
      }
      num = fma(gi[a], rn, num);
      den = fma(gi[a], rd, den);
      dni = fma(gi[5 + a], rn, dni);
      ddi = fma(gi[5 + a], rd, ddi);
      dnj = fma(gi[a], rnj, dnj);
      ddj = fma(gi[a], rdj, ddj);
    }
    if (den > 1e-99) {
      const double r = 1.0 / den, u = num * r;
      c6 = (float)u;
      dci = (float)(r * fma(u, -ddi, dni));
      dcj = (float)(r * fma(u, -ddj, dnj));
    } else {   // all weights underflow: the reference's nearest-reference value
      c6_pair(p, ti, tj, (float)cn[i], (float)cn[j], c6, dci, dcj);
    }
  } else {
    c6_pair(p, ti, tj, (float)cn[i], (float)cn[j], c6, dci, dcj);
  }
  tab[(size_t)i * n + j] = make_float2(c6, dci);
  tab[(size_t)j * n + i] = make_float2(c6, dcj);
}

// C6_ij and dC6_ij/dCN_i from the per-atom Gaussian factors (separable path)
__device__ __forceinline__ void c6_sep(const D3Params& p, int ti, int tj,
                                       const double* __restrict__ gi,
                                       const double* __restrict__ gj, float cni, float cnj,
                                       float& c6, float& dci) {
  const float* t = p.c6ab + ((size_t)ti * p.ntypes + tj) * (MAXC * MAXC * 3);
  const int ma = p.mxc[ti], mb = p.mxc[tj];
  double gjv[MAXC];
#pragma unroll
  for (int b = 0; b < MAXC; ++b) gjv[b] = b < mb ? gj[b] : 0.0;
  double num = 0.0, den = 0.0, dni = 0.0, ddi = 0.0;
  for (int a = 0; a < ma; ++a) {
    double rn = 0.0, rd = 0.0;
#pragma unroll
    for (int b = 0; b < MAXC; ++b) {
      const float ref = b < mb ? t[(a * MAXC + b) * 3] : 0.0f;
      if (ref > 0.0f) {
        rn = fma((double)ref, gjv[b], rn);
        rd += gjv[b];
      }
    }
    num = fma(gi[a], rn, num);
    den = fma(gi[a], rd, den);
    dni = fma(gi[5 + a], rn, dni);
    ddi = fma(gi[5 + a], rd, ddi);
  }
  if (den > 1e-99) {
    const double r = 1.0 / den, u = num * r;
    c6 = (float)u;
    dci = (float)(r * fma(u, -ddi, dni));
  } else {
    float dcj;
    c6_pair(p, ti, tj, cni, cnj, c6, dci, dcj);
  }
}

// Separable path: row i = one workgroup, coalesced row writes, ordered pairs
// (25 fp64 multiply-adds each; only dC6/dCN_i is needed per ordered pair)
__global__ __launch_bounds__(BLK) void k_d3_c6rows(D3Params p, int n, const int* __restrict__ type,
                                                    const double* __restrict__ cn,
                                                    const double* __restrict__ gw,
                                                    float2* __restrict__ tab) {
  // this row's reference C6 grids against every partner type, in LDS
  constexpr int MAXT_LDS = 64;
  __shared__ float s_ref[MAXT_LDS * MAXC * MAXC];
  const int i = blockIdx.x;
  const int ti = type[i], ma = p.mxc[ti];
  const bool lds = p.ntypes <= MAXT_LDS;
  if (lds)
    for (int k = threadIdx.x; k < p.ntypes * MAXC * MAXC; k += BLK) {
      const int tj = k / (MAXC * MAXC), ab = k - tj * (MAXC * MAXC);
      s_ref[k] = p.c6ab[(((size_t)ti * p.ntypes + tj) * (MAXC * MAXC) + ab) * 3];
    }
  __syncthreads();
  double gi[MAXC], dgi[MAXC];
#pragma unroll
  for (int a = 0; a < MAXC; ++a) {
    gi[a] = gw[(size_t)i * 10 + a];
    dgi[a] = gw[(size_t)i * 10 + 5 + a];
  }
  for (int j = threadIdx.x; j < n; j += BLK) {
    const int tj = type[j], mb = p.mxc[tj];
    double gj[MAXC];
#pragma unroll
    for (int b = 0; b < MAXC; ++b) gj[b] = gw[(size_t)j * 10 + b];
    double num = 0.0, den = 0.0, dni = 0.0, ddi = 0.0;
#pragma unroll
    for (int a = 0; a < MAXC; ++a) {
      if (a < ma) {
        double rn = 0.0, rd = 0.0;
#pragma unroll
        for (int b = 0; b < MAXC; ++b) {
          const float ref = lds ? s_ref[(tj * MAXC + a) * MAXC + b]
                                : p.c6ab[(((size_t)ti * p.ntypes + tj) * (MAXC * MAXC) +
                                          a * MAXC + b) * 3];
          if (b < mb && ref > 0.0f) {
            rn = fma((double)ref, gj[b], rn);
            rd += gj[b];
          }
        }
        num = fma(gi[a], rn, num);
        den = fma(gi[a], rd, den);
        dni = fma(dgi[a], rn, dni);
        ddi = fma(dgi[a], rd, ddi);
      }
    }
    float c6, dci;
    if (den > 1e-99) {
      const double r = 1.0 / den, u = num * r;
      c6 = (float)u;
      dci = (float)(r * fma(u, -ddi, dni));
    } else {   // all weights underflow: the reference's nearest-reference value
      float dcj;
      c6_pair(p, ti, tj, (float)cn[i], (float)cn[j], c6, dci, dcj);
    }
    tab[(size_t)i * n + j] = make_float2(c6, dci);
  }
}

// row outputs: [0] energy, [1..6] virial (xx,yy,zz,xy,xz,yz), [7] dE/dCN
constexpr int ROW = 8;

template <int DAMP, bool TAB>
__global__ __launch_bounds__(BLK) void k_d3_disp(D3Params p, D3Grid g, int n,
                                                  const float4* __restrict__ x,
                                                  const int* __restrict__ type,
                                                  const double* __restrict__ cn,
                                                  const float2* __restrict__ c6tab,
                                                  const double* __restrict__ gw,
                                                  double* __restrict__ rows,
                                                  double* __restrict__ forces) {
  __shared__ double red[NW];
  // per partner type: BJ (R0^6, R0^8, s8 * 3 r2r4_i r2r4_j), zero (a1 R0ab,
  // a2 R0ab, s8 r2r4_i r2r4_j) -- one LDS read per item instead of the
  // table loads, products and a sqrt
  constexpr int MAXT_LDS = 64;
  __shared__ float s_tp[MAXT_LDS][3];
  const int i = blockIdx.x;
  const int ti = type[i];
  const float cni = (float)cn[i];
  const float2* trow = TAB ? c6tab + (size_t)i * n : nullptr;
  const bool lds = p.ntypes <= MAXT_LDS;
  auto pair_consts = [&](int tj, float& c0, float& c1, float& c2) {
    if constexpr (DAMP == 1) {
      const float r0 = p.r0ab[ti * p.ntypes + tj];
      c0 = p.a1 * r0;
      c1 = p.a2 * r0;
      c2 = p.s8 * p.r2r4[ti] * p.r2r4[tj];
    } else {
      const float r42x3 = p.r2r4[ti] * p.r2r4[tj] * 3.0f;
      const float R0 = fmaf(p.a1, sqrtf(r42x3), p.a2);
      const float R02 = R0 * R0;
      c0 = R02 * R02 * R02;
      c1 = c0 * R02;
      c2 = p.s8 * r42x3;
    }
  };
  if (lds)
    for (int tj = threadIdx.x; tj < p.ntypes; tj += BLK)
      pair_consts(tj, s_tp[tj][0], s_tp[tj][1], s_tp[tj][2]);
  __syncthreads();
  float e = 0.f, fx = 0.f, fy = 0.f, fz = 0.f, dcn = 0.f;
  float v00 = 0.f, v11 = 0.f, v22 = 0.f, v01 = 0.f, v02 = 0.f, v12 = 0.f;
  for_pairs<false>(g, g.off_vdw, g.n_off_vdw, g.cull2_vdw, p.rthr, x, i,
                   [&](int j, int tj, float rx, float ry, float rz, float r2) {
    float c6, dc;
    if constexpr (TAB) {
      const float2 t = trow[j];
      c6 = t.x;
      dc = t.y;
    } else if (gw) {   // > 32k atoms: separable weights per item (25 fp64 FMAs)
      c6_sep(p, ti, tj, gw + (size_t)i * 10, gw + (size_t)j * 10, cni, (float)cn[j], c6, dc);
    } else {
      float dcj_unused;
      c6_pair(p, ti, tj, cni, (float)cn[j], c6, dc, dcj_unused);
    }
    float erest, x1;  // vec = x1 * r_ij = -(dE/dr) r_hat (the reference's x1 convention)
    float k0, k1, k2;
    if (lds) {
      k0 = s_tp[tj][0];
      k1 = s_tp[tj][1];
      k2 = s_tp[tj][2];
    } else {
      pair_consts(tj, k0, k1, k2);
    }
    if constexpr (DAMP == 1) {
      // zero damping, alp6 = 14 / alp8 = 16 as fixed powers (:1338-1356)
      const float s8r42 = k2;
      const float rrc = rsqrtf(r2);
      const float u1 = k0 * rrc;
      float t6 = u1 * u1;
      t6 *= u1;
      t6 *= t6;
      t6 *= u1;
      t6 *= t6;
      const float d6 = __builtin_amdgcn_rcpf(fmaf(t6, 6.0f, 1.0f));
      const float u2 = k1 * rrc;
      float t8 = u2 * u2;
      t8 *= t8;
      t8 *= t8;
      t8 *= t8;
      const float d8 = __builtin_amdgcn_rcpf(fmaf(t8, 6.0f, 1.0f));
      const float r2rc = rrc * rrc, r6rc = r2rc * r2rc * r2rc, r8rc = r6rc * r2rc;
      erest = r6rc * fmaf(3.0f * r2rc, s8r42 * d8, p.s6 * d6);
      x1 = 6.0f * c6 * r8rc *
           fmaf(r2rc, s8r42 * d8 * fmaf(3.0f * p.alp8 * t8, d8, -4.0f),
                p.s6 * d6 * fmaf(p.alp6 * t6, d6, -1.0f));
    } else {
      const float R06 = k0, R08 = k1, s8r = k2;
      const float rrc = rsqrtf(r2), r = r2 * rrc, r5 = r2 * r2 * r, r7 = r5 * r2;
      const float t6 = __builtin_amdgcn_rcpf(fmaf(r5, r, R06));   // 1 ulp
      const float t8 = __builtin_amdgcn_rcpf(fmaf(r7, r, R08));
      erest = fmaf(s8r, t8, p.s6 * t6);
      x1 = -c6 * fmaf(8.0f * s8r * r7, t8 * t8, 6.0f * p.s6 * r5 * t6 * t6) * rrc;
    }
    // row weights: every unordered pair appears in two rows, the self images
    // of i once -> energy / virial carry 1/2; F_i and dE/dCN_i the full
    // derivative for this row's own atom (self images: no force)
    // (the 1/2 of energy and virial is applied once per row, below)
    e = fmaf(-erest, c6, e);
    dcn = fmaf(-erest, dc, dcn);
    const float vx = x1 * rx, vy = x1 * ry, vz = x1 * rz;
    if (j != i) {
      fx -= vx;
      fy -= vy;
      fz -= vz;
    }
    v00 = fmaf(vx, rx, v00);
    v11 = fmaf(vy, ry, v11);
    v22 = fmaf(vz, rz, v22);
    v01 = fmaf(vx, ry, v01);
    v02 = fmaf(vx, rz, v02);
    v12 = fmaf(vy, rz, v12);
  });
  double* row = rows + (size_t)i * ROW;
  const double se = block_sum(e, red);
  const double sfx = block_sum(fx, red), sfy = block_sum(fy, red), sfz = block_sum(fz, red);
  const double s00 = block_sum(v00, red), s11 = block_sum(v11, red), s22 = block_sum(v22, red);
  const double s01 = block_sum(v01, red), s02 = block_sum(v02, red), s12 = block_sum(v12, red);
  const double sdc = block_sum(dcn, red);
  if (threadIdx.x == 0) {
    row[0] = 0.5 * se;
    row[1] = 0.5 * s00;
    row[2] = 0.5 * s11;
    row[3] = 0.5 * s22;
    row[4] = 0.5 * s01;
    row[5] = 0.5 * s02;
    row[6] = 0.5 * s12;
    row[7] = sdc;
    forces[3 * i] = sfx;
    forces[3 * i + 1] = sfy;
    forces[3 * i + 2] = sfz;
  }
}

// F_i += sum_j,T (dE/dCN_i + dE/dCN_j) dCN/dr r_hat ; virial (:1812-1976)
__global__ __launch_bounds__(BLK) void k_d3_chain(D3Params p, D3Grid g, const float4* __restrict__ x,
                                                   const int* __restrict__ type,
                                                   double* __restrict__ rows,
                                                   double* __restrict__ forces) {
  __shared__ double red[NW];
  const int i = blockIdx.x;
  const float rci = p.rcov[type[i]];
  const float dci = (float)rows[(size_t)i * ROW + 7];
  float fx = 0.f, fy = 0.f, fz = 0.f;
  float v00 = 0.f, v11 = 0.f, v22 = 0.f, v01 = 0.f, v02 = 0.f, v12 = 0.f;
  for_pairs<true>(g, g.off_cn, g.n_off_cn, g.cull2_cn, p.cn_thr, x, i,
                  [&](int j, int tj, float rx, float ry, float rz, float r2) {
    const float rcs = rci + p.rcov[tj];
    const float rrc = rsqrtf(r2);
    const float ex = expf(-K1 * (rcs * rrc - 1.0f));
    const float dcnn = -K1 * rcs * ex / (r2 * (ex + 1.0f) * (ex + 1.0f));
    // self images: weight dE/dCN_i once; pairs: rows (i, j) and (j, i) 1/2 each
    const float w = j == i ? dci : 0.5f * (dci + (float)rows[(size_t)j * ROW + 7]);
    const float x1 = dcnn * w * rrc;
    const float vx = x1 * rx, vy = x1 * ry, vz = x1 * rz;
    if (j != i) {
      fx += 2.0f * vx;
      fy += 2.0f * vy;
      fz += 2.0f * vz;
    }
    v00 -= vx * rx;
    v11 -= vy * ry;
    v22 -= vz * rz;
    v01 -= vx * ry;
    v02 -= vx * rz;
    v12 -= vy * rz;
  });
  const double sfx = block_sum(fx, red), sfy = block_sum(fy, red), sfz = block_sum(fz, red);
  const double s00 = block_sum(v00, red), s11 = block_sum(v11, red), s22 = block_sum(v22, red);
  const double s01 = block_sum(v01, red), s02 = block_sum(v02, red), s12 = block_sum(v12, red);
  if (threadIdx.x == 0) {
    double* row = rows + (size_t)i * ROW;
    row[1] += s00;
    row[2] += s11;
    row[3] += s22;
    row[4] += s01;
    row[5] += s02;
    row[6] += s12;
    forces[3 * i] += sfx;
    forces[3 * i + 1] += sfy;
    forces[3 * i + 2] += sfz;
  }
}

// totals[0] = energy (eV), totals[1..6] = virial (eV); fixed-order sums over
// rows; forces to eV/A (update, :2003-2024)
__global__ __launch_bounds__(BLK) void k_d3_reduce(int n, const double* __restrict__ rows,
                                                    double* __restrict__ forces,
                                                    double* __restrict__ totals) {
  __shared__ double red[NW];
  for (int c = 0; c < 7; ++c) {
    double s = 0.0;
    for (int i = threadIdx.x; i < n; i += BLK) s += rows[(size_t)i * ROW + c];
    s = block_sum(s, red);
    if (threadIdx.x == 0) totals[c] = s * D3_AU_TO_EV;
  }
  for (int k = threadIdx.x; k < 3 * n; k += BLK) forces[k] *= D3_AU_TO_EV / D3_AU_TO_ANG;
}

}  // namespace

hipError_t launch_d3(const D3Params& p, const D3Grid& g, int n, const float4* x, const int* type,
                     double* cn, double* gw, float2* c6tab, double* rows, double* forces,
                     double* totals, hipStream_t s) {
  if (n <= 0) {
    hipMemsetAsync(totals, 0, 7 * sizeof(double), s);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_d3_cn, dim3(n), dim3(BLK), 0, s, p, g, x, type, cn);
  if (p.cnref)
    hipLaunchKernelGGL(k_d3_gauss, dim3((n + BLK - 1) / BLK), dim3(BLK), 0, s, p, n, type, cn, gw);
  if (c6tab) {
    if (p.cnref) {
      hipLaunchKernelGGL(k_d3_c6rows, dim3(n), dim3(BLK), 0, s, p, n, type, cn, gw, c6tab);
    } else {
      const int64_t npair = (int64_t)n * (n + 1) / 2;
      hipLaunchKernelGGL(k_d3_c6tab, dim3((unsigned)((npair + BLK - 1) / BLK)), dim3(BLK), 0, s,
                         p, n, type, cn, nullptr, c6tab);
    }
  }
  if (p.damping == 1) {
    if (c6tab)
      hipLaunchKernelGGL((k_d3_disp<1, true>), dim3(n), dim3(BLK), 0, s, p, g, n, x, type, cn,
                         c6tab, p.cnref ? gw : nullptr, rows, forces);
    else
      hipLaunchKernelGGL((k_d3_disp<1, false>), dim3(n), dim3(BLK), 0, s, p, g, n, x, type, cn,
                         c6tab, p.cnref ? gw : nullptr, rows, forces);
  } else {
    if (c6tab)
      hipLaunchKernelGGL((k_d3_disp<2, true>), dim3(n), dim3(BLK), 0, s, p, g, n, x, type, cn,
                         c6tab, p.cnref ? gw : nullptr, rows, forces);
    else
      hipLaunchKernelGGL((k_d3_disp<2, false>), dim3(n), dim3(BLK), 0, s, p, g, n, x, type, cn,
                         c6tab, p.cnref ? gw : nullptr, rows, forces);
  }
  hipLaunchKernelGGL(k_d3_chain, dim3(n), dim3(BLK), 0, s, p, g, x, type, rows, forces);
  hipLaunchKernelGGL(k_d3_reduce, dim3(1), dim3(BLK), 0, s, n, rows, forces, totals);
  return hipGetLastError();
}

}  // namespace e3gnn
