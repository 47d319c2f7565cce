// Edge geometry, graph index builders, node-wise ops and the force/virial
// reduction of the SevenNet-0 energy+force path, gfx950.
//
// Every reduction here is deterministic: per-atom sums walk CSR lists in edge
// order (no float atomics); scalar totals use a fixed two-level tree.
#include "common.h"

#include <climits>
#include "node.h"

namespace e3gnn {
namespace {

constexpr int TPB = 256;
inline int nblk(int64_t n, int t = TPB) { return (int)((n + t - 1) / t); }

// ------------------------------------------------------------ edge embedding
// EdgeEmbedding.forward (sevenn/nn/edge_embedding.py:220-230): r = |r_ij|,
// BesselBasis (:114-116) B_n = (2/rc) sin(c_n r) / r with trainable c_n,
// XPLORCutoff (:163-173), SphericalEncoding (:177-198; e3nn SH lmax 2,
// 'component'; polynomial of serial_code.py:50-70) of the unit vector
// (normalize=True) or, for checkpoints before sevenn 0.9 (`_normalize_sph`
// absent, util.py:130-146), of the raw vector: Y_l(r) = |r|^l Y_l(r/|r|).
__global__ void k_edge_embed(int64_t E, const float* __restrict__ vec, const float* __restrict__ coeffs,
                             float rc, float ron, int raw_sh, float* __restrict__ Y,
                             float* __restrict__ emb) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const float vx = vec[3 * e], vy = vec[3 * e + 1], vz = vec[3 * e + 2];
  const float r = sqrtf(vx * vx + vy * vy + vz * vz);
  const float x = raw_sh ? vx : vx / r, y = raw_sh ? vy : vy / r, z = raw_sh ? vz : vz / r;
  const float s3 = 1.7320508075688772f, s5 = 2.23606797749979f;
  float* yo = Y + 9 * e;
  yo[0] = 1.f;
  yo[1] = s3 * x;
  yo[2] = s3 * y;
  yo[3] = s3 * z;
  yo[4] = s5 * (s3 * x * z);
  yo[5] = s5 * (s3 * x * y);
  yo[6] = s5 * (y * y - 0.5f * (x * x + z * z));
  yo[7] = s5 * (s3 * y * z);
  yo[8] = s5 * (0.5f * s3 * (z * z - x * x));
  float env = 1.f;
  if (r >= ron) {
    const float rc2 = rc * rc, r2 = r * r, ron2 = ron * ron;
    const float a = rc2 - r2, d = rc2 - ron2;
    env = a * a * (rc2 + 2.f * r2 - 3.f * ron2) / (d * d * d);
  }
  float* eo = emb + 8 * e;
#pragma unroll
  for (int n = 0; n < 8; ++n) eo[n] = (2.f / rc) * sinf(coeffs[n] * r) / r * env;
}

// dE/dr_ij from the accumulated dE/dY (all layers) and dE/demb (all layers):
// the chain rule of the two functions above (force_output.py:83-130 obtains
// the same through autograd).  Also writes per-block virial partials.  With
// raw_sh the SH polynomials take the raw vector: their gradient (and dgu, which
// the fused kernels form from Y_1 / sqrt 3 = the SH argument) is dE/dr_ij
// directly, without the unit-vector projection.
__global__ void k_edge_force(int64_t E, const float* __restrict__ vec, const float* __restrict__ coeffs,
                             float rc, float ron, int raw_sh, const float* __restrict__ dY,
                             const float* __restrict__ dgu, const float* __restrict__ demb,
                             float* __restrict__ fe, float* __restrict__ vir_part) {
  __shared__ float red[6][TPB];
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float v6[6] = {0, 0, 0, 0, 0, 0};
  if (e < E) {
    const float vx = vec[3 * e], vy = vec[3 * e + 1], vz = vec[3 * e + 2];
    const float r = sqrtf(vx * vx + vy * vy + vz * vz);
    const float ux = vx / r, uy = vy / r, uz = vz / r;
    const float x = raw_sh ? vx : ux, y = raw_sh ? vy : uy, z = raw_sh ? vz : uz;
    const float s3 = 1.7320508075688772f, s5 = 2.23606797749979f;
    const float* g = dY + 9 * e;
    // gradient w.r.t. the SH argument (unit vector u, or r_ij itself)
    float gx = s3 * g[1], gy = s3 * g[2], gz = s3 * g[3];
    const float c = s5 * s3;
    gx += c * (z * g[4] + y * g[5]) - s5 * x * g[6] - c * x * g[8];
    gy += c * (x * g[5] + z * g[7]) + 2.f * s5 * y * g[6];
    gz += c * (x * g[4] + y * g[7]) - s5 * z * g[6] + c * z * g[8];
    if (dgu) {  // dE/du accumulated directly by the fused kernels
      gx += dgu[3 * e];
      gy += dgu[3 * e + 1];
      gz += dgu[3 * e + 2];
    }
    float fx = gx, fy = gy, fz = gz;
    if (!raw_sh) {
      const float dot = gx * ux + gy * uy + gz * uz;
      fx = (gx - dot * ux) / r;
      fy = (gy - dot * uy) / r;
      fz = (gz - dot * uz) / r;
    }
    // radial part
    float env = 1.f, denv = 0.f;
    if (r >= ron) {
      const float rc2 = rc * rc, r2 = r * r, ron2 = ron * ron;
      const float a = rc2 - r2, d = rc2 - ron2, d3 = d * d * d;
      env = a * a * (rc2 + 2.f * r2 - 3.f * ron2) / d3;
      denv = 12.f * r * a * (ron2 - r2) / d3;
    }
    const float* ge = demb + 8 * e;
    float dr = 0.f;
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      const float cn = coeffs[n];
      const float sn = sinf(cn * r), cs = cosf(cn * r);
      const float b = (2.f / rc) * sn / r;
      const float db = (2.f / rc) * (cn * cs * r - sn) / (r * r);
      dr += ge[n] * (db * env + b * denv);
    }
    fx += dr * ux;
    fy += dr * uy;
    fz += dr * uz;
    fe[3 * e] = fx;
    fe[3 * e + 1] = fy;
    fe[3 * e + 2] = fz;
    // virial = -dE/dstrain (symmetric strain, ForceStressOutput force_output.py:83-130);
    // equals inferred_stress * volume, the quantity pair_e3gnn.cpp:244-256 hands LAMMPS
    v6[0] = -(vx * fx);
    v6[1] = -(vy * fy);
    v6[2] = -(vz * fz);
    v6[3] = -0.5f * (vx * fy + vy * fx);
    v6[4] = -0.5f * (vy * fz + vz * fy);
    v6[5] = -0.5f * (vx * fz + vz * fx);
  }
  if (!vir_part) return;   // (uniform) the fine-tune step's dE/dr needs no virial here
#pragma unroll
  for (int q = 0; q < 6; ++q) red[q][threadIdx.x] = v6[q];
  __syncthreads();
  for (int s = TPB / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s)
#pragma unroll
      for (int q = 0; q < 6; ++q) red[q][threadIdx.x] += red[q][threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x < 6) vir_part[(int64_t)blockIdx.x * 6 + threadIdx.x] = red[threadIdx.x][0];
}

// XPLOR envelope and its r-derivative (edge_embedding.py:163-173)
__device__ __forceinline__ void xplor(float r, float rc, float ron, float& env, float& denv) {
  env = 1.f;
  denv = 0.f;
  if (r >= ron) {
    const float rc2 = rc * rc, r2 = r * r, ron2 = ron * ron;
    const float a = rc2 - r2, d = rc2 - ron2, d3 = d * d * d;
    env = a * a * (rc2 + 2.f * r2 - 3.f * ron2) / d3;
    denv = 12.f * r * a * (ron2 - r2) / d3;
  }
}

// Tangent of the edge geometry for the fine-tune step's reverse-over-forward
// derivatives (train_explicit.py): the per-edge direction is the loss
// cotangent of f_e = dE/dr_e,
//   v_e = dL/dF[centre] - dL/dF[nbr] - (c0 r0 + c5 r2, c1 r1 + c3 r0, c2 r2 + c4 r1),
//   c = dL/dS[graph of nbr] / volume   (stress = -sum_e voigt(r_e, f_e) / volume),
// and the outputs are Y' = dY/dr . v, emb' = demb/dr (r_hat . v), r' = r_hat . v.
__global__ void k_edge_geom_jvp(int64_t E, const float* __restrict__ vec,
                                const float* __restrict__ coeffs, float rc, float ron, int raw_sh,
                                const int* __restrict__ center, const int* __restrict__ nbr,
                                const int64_t* __restrict__ batch, const float* __restrict__ cF,
                                const float* __restrict__ cS, const float* __restrict__ vol,
                                float* __restrict__ Yd, float* __restrict__ embd,
                                float* __restrict__ rd_out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const float vx = vec[3 * e], vy = vec[3 * e + 1], vz = vec[3 * e + 2];
  const int ic = center[e], jn = nbr[e];
  float tx = cF[3 * ic] - cF[3 * jn], ty = cF[3 * ic + 1] - cF[3 * jn + 1],
        tz = cF[3 * ic + 2] - cF[3 * jn + 2];
  if (cS) {
    const int64_t b = batch[jn];
    const float iv = 1.f / vol[b];
    const float* c = cS + 6 * b;
    tx -= (c[0] * vx + c[5] * vz) * iv;
    ty -= (c[1] * vy + c[3] * vx) * iv;
    tz -= (c[2] * vz + c[4] * vy) * iv;
  }
  const float r = sqrtf(vx * vx + vy * vy + vz * vz), ir = 1.f / r;
  const float ux = vx * ir, uy = vy * ir, uz = vz * ir;
  const float rd = ux * tx + uy * ty + uz * tz;
  // SH argument a (unit or raw vector) and its tangent a'
  float ax = vx, ay = vy, az = vz, dx = tx, dy = ty, dz = tz;
  if (!raw_sh) {
    ax = ux;
    ay = uy;
    az = uz;
    dx = (tx - ux * rd) * ir;
    dy = (ty - uy * rd) * ir;
    dz = (tz - uz * rd) * ir;
  }
  const float s3 = 1.7320508075688772f, s5 = 2.23606797749979f, c15 = s3 * s5;
  float* yo = Yd + 9 * e;
  yo[0] = 0.f;
  yo[1] = s3 * dx;
  yo[2] = s3 * dy;
  yo[3] = s3 * dz;
  yo[4] = c15 * (dx * az + ax * dz);
  yo[5] = c15 * (dx * ay + ax * dy);
  yo[6] = s5 * (2.f * ay * dy - (ax * dx + az * dz));
  yo[7] = c15 * (dy * az + ay * dz);
  yo[8] = c15 * (az * dz - ax * dx);
  float env, denv;
  xplor(r, rc, ron, env, denv);
  float* eo = embd + 8 * e;
#pragma unroll
  for (int n = 0; n < 8; ++n) {
    const float cn = coeffs[n];
    const float sn = sinf(cn * r), cs = cosf(cn * r);
    const float b = (2.f / rc) * sn * ir;
    const float db = (2.f / rc) * (cn * cs * r - sn) * ir * ir;
    eo[n] = (db * env + b * denv) * rd;
  }
  rd_out[e] = rd;
}

// per-edge d/dc_n of <emb-bar, emb> + <emb'-bar, emb'> (the Bessel
// coefficients' gradient, summed over edges by the caller)
__global__ void k_edge_geom_coeff(int64_t E, const float* __restrict__ vec,
                                  const float* __restrict__ coeffs, float rc, float ron,
                                  const float* __restrict__ embb, const float* __restrict__ embdb,
                                  const float* __restrict__ rd, float* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const float vx = vec[3 * e], vy = vec[3 * e + 1], vz = vec[3 * e + 2];
  const float r = sqrtf(vx * vx + vy * vy + vz * vz);
  float env, denv;
  xplor(r, rc, ron, env, denv);
  const float k = 2.f / rc, t = rd[e];
#pragma unroll
  for (int n = 0; n < 8; ++n) {
    const float cn = coeffs[n];
    const float sn = sinf(cn * r), cs = cosf(cn * r);
    out[8 * e + n] = embb[8 * e + n] * (k * cs * env) +
                     embdb[8 * e + n] * (k * (cs * denv - cn * sn * env)) * t;
  }
}

// F_i = sum_{e: center=i} f_e - sum_{e: nbr=i} f_e  (pair_e3gnn_parallel.cpp:482-484)
__global__ void k_atom_force(int n_nodes, int n_centers, const int* __restrict__ row_ptr,
                             const int* __restrict__ src_ptr, const int* __restrict__ src_perm,
                             const float* __restrict__ fe, float* __restrict__ F) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_nodes) return;
  float fx = 0.f, fy = 0.f, fz = 0.f;
  if (i < n_centers)
    for (int e = row_ptr[i]; e < row_ptr[i + 1]; ++e) {
      fx += fe[3 * e];
      fy += fe[3 * e + 1];
      fz += fe[3 * e + 2];
    }
  for (int q = src_ptr[i]; q < src_ptr[i + 1]; ++q) {
    const int e = src_perm[q];
    fx -= fe[3 * e];
    fy -= fe[3 * e + 1];
    fz -= fe[3 * e + 2];
  }
  F[3 * i] = fx;
  F[3 * i + 1] = fy;
  F[3 * i + 2] = fz;
}

// ------------------------------------------------------------ graph indices
// row_ptr of the centre-sorted edge list + validation (edge_index[0] sorted,
// indices in range).  err bits: 1 unsorted, 2 centre out of range, 4 nbr out
// of range, 16 a centre below n_interior has a ghost neighbour.
__global__ void k_row_ptr(int64_t E, int n_centers, int n_nodes, int n_interior,
                          const int* __restrict__ center, const int* __restrict__ nbr,
                          int* __restrict__ row_ptr, int* __restrict__ err) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const int c = center[e];
  const int j = nbr[e];
  if (c < 0 || c >= n_centers) {
    atomicOr(err, 2);
    return;
  }
  if (j < 0 || j >= n_nodes) atomicOr(err, 4);
  if (c < n_interior && j >= n_centers) atomicOr(err, 16);  // interior centre with a ghost neighbour
  // an invalid (negative) predecessor is reported by its own thread; the
  // fill never starts below row_ptr[0]
  const int prev = e ? max(center[e - 1], -1) : -1;
  if (c < prev) {
    atomicOr(err, 1);
    return;
  }
  for (int q = prev + 1; q <= c; ++q) row_ptr[q] = (int)e;
  if (e == E - 1)
    for (int q = c + 1; q <= n_centers; ++q) row_ptr[q] = (int)E;
}

__global__ void k_fill_int(int n, int v, int* __restrict__ p) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

__global__ void k_count_nbr(int64_t E, const int* __restrict__ nbr, int n_nodes,
                            int* __restrict__ cnt) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const int j = nbr[e];
  if (j >= 0 && j < n_nodes) atomicAdd(cnt + j, 1);
}

// exclusive scan of cnt[0..n) into out[0..n].  Three launches: k_scan_blocks
// (1,024 counts per workgroup, 4 consecutive per thread: local exclusive
// prefixes to out, the block total to bsum), k_scan_top (one workgroup scans
// the block totals in place, out[n] = the grand total), k_scan_add (adds each
// block's offset).  The old single-workgroup scan (strided per-thread chunks)
// took 164 us for 97k nodes.
constexpr int SCAN_B = 1024;
__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(v, o);
    if (lane >= o) v += u;
  }
  return v;
}
__global__ __launch_bounds__(256) void k_scan_blocks(int n, const int* __restrict__ cnt,
                                                     int* __restrict__ out, int* __restrict__ bsum) {
  __shared__ int wsum[4];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int i0 = blockIdx.x * SCAN_B + 4 * t;
  int c[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) c[q] = i0 + q < n ? cnt[i0 + q] : 0;
  const int ts = c[0] + c[1] + c[2] + c[3];
  const int incl = wave_incl_scan(ts, lane);
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  int base = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) base += q < w ? wsum[q] : 0;
  int run = base + incl - ts;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (i0 + q < n) out[i0 + q] = run;
    run += c[q];
  }
  if (t == 255) bsum[blockIdx.x] = base + incl;
}
__global__ __launch_bounds__(1024) void k_scan_top(int nb, int n, int* __restrict__ bsum,
                                                   int* __restrict__ out) {
  __shared__ int wsum[16];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  int carry = 0;
  for (int c0 = 0; c0 < nb; c0 += 1024) {
    const int v = c0 + t < nb ? bsum[c0 + t] : 0;
    const int incl = wave_incl_scan(v, lane);
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int base = carry;
    for (int q = 0; q < w; ++q) base += wsum[q];
    int total = carry;
    for (int q = 0; q < 16; ++q) total += wsum[q];
    if (c0 + t < nb) bsum[c0 + t] = base + incl - v;
    carry = total;
    __syncthreads();
  }
  if (t == 0) out[n] = carry;
}
__global__ __launch_bounds__(256) void k_scan_add(int n, const int* __restrict__ bsum,
                                                  int* __restrict__ out) {
  const int i0 = blockIdx.x * SCAN_B + 4 * threadIdx.x;
  const int add = bsum[blockIdx.x];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (i0 + q < n) out[i0 + q] += add;
}
// single workgroup fallback (graphs with fewer edges than count blocks: the
// block totals borrow the edge permutation's storage)
__global__ __launch_bounds__(1024) void k_scan(int n, const int* __restrict__ cnt,
                                               int* __restrict__ out) {
  __shared__ int part[1024];
  const int t = threadIdx.x;
  const int chunk = (n + 1023) / 1024;
  const int b = t * chunk, en = min(n, b + chunk);
  int s = 0;
  for (int i = b; i < en; ++i) s += cnt[i];
  part[t] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const int v = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int run = t ? part[t - 1] : 0;
  for (int i = b; i < en; ++i) {
    out[i] = run;
    run += cnt[i];
  }
  if (t == 1023) out[n] = part[1023];
}

__global__ void k_scatter_perm(int64_t E, const int* __restrict__ nbr, int n_nodes,
                               const int* __restrict__ ptr, int* __restrict__ cursor,
                               int* __restrict__ perm) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const int j = nbr[e];
  if (j < 0 || j >= n_nodes) return;
  const int slot = atomicAdd(cursor + j, 1);
  perm[ptr[j] + slot] = (int)e;
}

// make each neighbour's edge list ascending in edge id (deterministic order):
// one wave per neighbour, segments of up to 64 edges sorted by rank (lane k
// holds element k; its rank = the number of smaller elements, the ids being
// distinct), longer ones by an insertion sort in lane 0.  (A thread-per-node
// insertion sort on global memory took 138 us on the 97k-atom graph and 89 us
// on a fine-tune batch: every shift a dependent L2 round trip.)
__global__ __launch_bounds__(256) void k_sort_segments(int n, const int* __restrict__ ptr,
                                                       int* __restrict__ perm) {
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (j >= n) return;
  const int b = ptr[j], len = ptr[j + 1] - b;
  if (len <= 1) return;
  if (len <= 64) {
    const int v = lane < len ? perm[b + lane] : INT_MAX;
    int rank = 0;
    for (int k = 0; k < len; ++k) rank += __shfl(v, k) < v;
    if (lane < len) perm[b + rank] = v;
    return;
  }
  if (lane != 0) return;
  for (int i = b + 1; i < b + len; ++i) {
    const int v = perm[i];
    int k = i - 1;
    while (k >= b && perm[k] > v) {
      perm[k + 1] = perm[k];
      --k;
    }
    perm[k + 1] = v;
  }
}

// The whole graph build in ONE workgroup for small graphs (a fine-tune batch:
// ~10^3 nodes, ~10^4 edges), the per-neighbour counts and offsets in LDS:
// validation + row_ptr, counts, exclusive scan, scatter and the segment sort
// of the launches above (eleven launches and a memset, each mostly launch
// latency at this size).  Optionally converts int64 edge indices (the
// batch's edge_index rows) into the int32 copies the kernels read.
constexpr int GRAPH_SMALL_N = 3072, GRAPH_SMALL_E = 16384;   // LDS: 24.6 KB of counts / offsets + 64 KB of edges (gfx950: 160 KB per workgroup)
template <typename T>
__global__ __launch_bounds__(1024) void k_build_graph_small(int E, int n, const T* __restrict__ cin,
                                                            const T* __restrict__ jin, int* __restrict__ cout,
                                                            int* __restrict__ jout, int* __restrict__ row_ptr,
                                                            int* __restrict__ src_ptr, int* __restrict__ perm,
                                                            int* __restrict__ err) {
  __shared__ int cnt[GRAPH_SMALL_N];
  __shared__ int ptr[GRAPH_SMALL_N + 1];
  __shared__ int lperm[GRAPH_SMALL_E];   // the transposed CSR's edge list, sorted here, then stored
  __shared__ int wsum[16];
  __shared__ int errl;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  for (int i = t; i < n; i += 1024) cnt[i] = 0;
  for (int i = t; i <= n; i += 1024) row_ptr[i] = 0;
  if (t == 0) errl = 0;
  __syncthreads();
  // the thread's edges e = t + 1024 u, all loads in flight at once (a loop
  // that waited for each edge's loads took ~1 us per edge of the thread)
  constexpr int EPT = GRAPH_SMALL_E / 1024;
  int cv[EPT], pv[EPT], jv[EPT];
  // validated in the input's own type before narrowing (an int64 index
  // 2^32 + 3 must not pass as 3): out of range -> -1, reported below
  auto idx = [n](T v) { return (v < (T)0 || v >= (T)n) ? -1 : (int)v; };
#pragma unroll
  for (int u = 0; u < EPT; ++u) {
    const int e = t + 1024 * u;
    cv[u] = e < E ? idx(cin[e]) : 0;
    pv[u] = (e < E && e > 0) ? idx(cin[e - 1]) : -1;
    jv[u] = e < E ? idx(jin[e]) : 0;
  }
  // validation, row_ptr (as k_row_ptr) and the per-neighbour counts
#pragma unroll
  for (int u = 0; u < EPT; ++u) {
    const int e = t + 1024 * u;
    if (e >= E) continue;
    const int c = cv[u], j = jv[u];
    if (cout) cout[e] = c;
    if (jout) jout[e] = j;
    if (j < 0 || j >= n) atomicOr(&errl, 4);
    else atomicAdd(&cnt[j], 1);
    if (c < 0 || c >= n) {
      atomicOr(&errl, 2);
      continue;
    }
    const int prev = pv[u];
    if (c < prev) {
      atomicOr(&errl, 1);
      continue;
    }
    for (int q = prev + 1; q <= c; ++q) row_ptr[q] = e;
    if (e == E - 1)
      for (int q = c + 1; q <= n; ++q) row_ptr[q] = E;
  }
  __syncthreads();
  // exclusive scan of the counts: chunks of consecutive nodes per thread
  constexpr int CH = (GRAPH_SMALL_N + 1023) / 1024;
  const int b0 = t * CH;
  int tot = 0;
#pragma unroll
  for (int q = 0; q < CH; ++q) tot += b0 + q < n ? cnt[b0 + q] : 0;
  const int incl = wave_incl_scan(tot, lane);
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  int run = incl - tot;
  for (int q = 0; q < w; ++q) run += wsum[q];
#pragma unroll
  for (int q = 0; q < CH; ++q)
    if (b0 + q < n) {
      ptr[b0 + q] = run;
      run += cnt[b0 + q];
    }
  if (t == 1023) ptr[n] = run;   // the last thread's running sum is the total
  __syncthreads();
  for (int i = t; i <= n; i += 1024) src_ptr[i] = ptr[i];
  for (int i = t; i < n; i += 1024) cnt[i] = 0;
  __syncthreads();
#pragma unroll
  for (int u = 0; u < EPT; ++u) {
    const int e = t + 1024 * u, j = jv[u];
    if (e >= E || j < 0 || j >= n) continue;
    lperm[ptr[j] + atomicAdd(&cnt[j], 1)] = e;
  }
  __syncthreads();
  // each neighbour's edges ascending (as k_sort_segments; one wave per node),
  // in LDS: a global round trip per node made this phase ~50 us
  for (int j = w; j < n; j += 16) {
    const int b = ptr[j], len = ptr[j + 1] - b;
    if (len <= 1) continue;
    if (len <= 64) {
      // rank = the segment's smaller ids, read as LDS broadcasts eight at a
      // time (a cross-lane shuffle per element waited ~100 cycles each)
      const int v = lane < len ? lperm[b + lane] : INT_MAX;
      int rank = 0, k = 0;
      for (; k + 8 <= len; k += 8) {
        int x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = lperm[b + k + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) rank += x[u] < v;
      }
      for (; k < len; ++k) rank += lperm[b + k] < v;
      __builtin_amdgcn_wave_barrier();
      if (lane < len) lperm[b + rank] = v;
      __builtin_amdgcn_wave_barrier();
    } else if (lane == 0) {
      for (int i = b + 1; i < b + len; ++i) {
        const int v = lperm[i];
        int k = i - 1;
        while (k >= b && lperm[k] > v) {
          lperm[k + 1] = lperm[k];
          --k;
        }
        lperm[k + 1] = v;
      }
    }
  }
  __syncthreads();
  const int ne = ptr[n];
  for (int i = t; i < ne; i += 1024) perm[i] = lperm[i];
  if (t == 0) *err = errl;
}

// ------------------------------------------------------------ node ops
// OnehotEmbedding + IrrepsLinear(is_embed) (node_embedding.py:39-48,
// linear.py:37-44): row lookup of the pre-scaled embedding matrix (D columns).
__global__ void k_embed(int n, int D, const int* __restrict__ type, int nsp, const float* __restrict__ W,
                        float* __restrict__ x, int* __restrict__ err) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)n * D) return;
  const int i = (int)(idx / D), c = (int)(idx - (int64_t)i * D);
  const int t = type[i];
  if (t < 0 || t >= nsp) {
    if (c == 0) atomicOr(err, 8);
    x[idx] = 0.f;
    return;
  }
  x[idx] = W[t * D + c];
}

// e3nn Gate (equivariant_gate.py:13-61; serial_code.py:256-347) of the
// SevenNet-0-shaped family, dims GateDims (node.h):
// y: [ns scalars | g1 + g2 gates | g1 x 1e | g2 x 2e] -> x: [ns x 0e | g1 x 1e | g2 x 2e]
// (SevenNet-0: ns 128, g1 64, g2 32: y 576, x 480)
__global__ void k_gate_fwd(int n, GateDims d, const float* __restrict__ y, float* __restrict__ x) {
  const int DX = d.dx(), DY = d.dy();
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)n * DX) return;
  const int64_t i = idx / DX;
  const int c = (int)(idx - i * DX);
  const float* yr = y + i * DY;
  const int ns = d.ns, o1 = ns + 3 * d.g1;           // x offsets of the 2e block
  const int yg = ns, yv = ns + d.g1 + d.g2;          // y offsets: gates, gated values
  float v;
  if (c < ns) v = act_fwd(yr[c]);
  else if (c < o1) v = act_fwd(yr[yg + (c - ns) / 3]) * yr[yv + (c - ns)];
  else v = act_fwd(yr[yg + d.g1 + (c - o1) / 5]) * yr[yv + (c - ns)];
  x[idx] = v;
}
// Gate backward, one wave per node: the y (DY) and dE/dx (DX) rows staged in
// LDS with float4 loads (dynamic LDS: 4 x (DY + DX) floats), coalesced stores.
__global__ __launch_bounds__(256) void k_gate_bwd_rows(int n, GateDims d, const float* __restrict__ y,
                                                       const float* __restrict__ dx,
                                                       float* __restrict__ dy) {
  extern __shared__ float4 shg[];
  const int DX = d.dx(), DY = d.dy();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = blockIdx.x * 4 + w;
  if (i >= n) return;  // whole wave: no block-level barrier below
  float4* yr4 = shg + w * ((DY + DX) / 4);
  float4* dr4 = yr4 + DY / 4;
  const float4* yg4 = reinterpret_cast<const float4*>(y + (int64_t)i * DY);
  const float4* dg4 = reinterpret_cast<const float4*>(dx + (int64_t)i * DX);
  for (int k = lane; k < DY / 4; k += 64) yr4[k] = yg4[k];
  for (int k = lane; k < DX / 4; k += 64) dr4[k] = dg4[k];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const float* yr = reinterpret_cast<const float*>(yr4);
  const float* dr = reinterpret_cast<const float*>(dr4);
  float* out = dy + (int64_t)i * DY;
  const int ns = d.ns, g1 = d.g1, g2 = d.g2;
  const int yg = ns, yv = ns + g1 + g2, yv2 = yv + 3 * g1;   // y: gates, 1e values, 2e values
  const int x1 = ns, x2 = ns + 3 * g1;                         // x: 1e, 2e
  for (int c = lane; c < DY; c += 64) {
    float v;
    if (c < ns) {
      v = dr[c] * act_grad(yr[c]);
    } else if (c < yg + g1) {
      const int u = c - yg;
      const float s = dr[x1 + 3 * u] * yr[yv + 3 * u] + dr[x1 + 3 * u + 1] * yr[yv + 3 * u + 1] +
                      dr[x1 + 3 * u + 2] * yr[yv + 3 * u + 2];
      v = s * act_grad(yr[c]);
    } else if (c < yv) {
      const int u = c - yg - g1;
      float s = 0.f;
#pragma unroll
      for (int m = 0; m < 5; ++m) s += dr[x2 + 5 * u + m] * yr[yv2 + 5 * u + m];
      v = s * act_grad(yr[c]);
    } else if (c < yv2) {
      v = dr[x1 + (c - yv)] * act_fwd(yr[yg + (c - yv) / 3]);
    } else {
      v = dr[x2 + (c - yv2)] * act_fwd(yr[yg + g1 + (c - yv2) / 5]);
    }
    out[c] = v;
  }
}
// last layer: scalars only, all activated
__global__ void k_act_fwd(int64_t n, const float* __restrict__ y, float* __restrict__ x) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = act_fwd(y[i]);
}
__global__ void k_act_bwd(int64_t n, const float* __restrict__ y, const float* __restrict__ dx,
                          float* __restrict__ dy) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dy[i] = dx[i] * act_grad(y[i]);
}

// readout (model_build.py:374-408) + SpeciesWiseRescale (scale.py:67-73):
// E_i = scale[t] * <x_i, v> + shift[t], v = W_hidden @ W_energy (path weights
// folded), x_i of D scalars (one wave per atom, lane-strided, fixed order)
__global__ void k_readout(int n, int D, const float* __restrict__ x, const float* __restrict__ v,
                          const int* __restrict__ type, const float* __restrict__ scale,
                          const float* __restrict__ shift, float* __restrict__ eat) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= n) return;
  const float* xr = x + (int64_t)i * D;
  float a = 0.f;
  for (int c = lane; c < D; c += 64) a += xr[c] * v[c];
  const float s = wave_sum(a);
  if (lane == 0) {
    const int t = type[i];
    eat[i] = s * scale[t] + shift[t];
  }
}
__global__ void k_readout_bwd(int n, int D, const float* __restrict__ v, const int* __restrict__ type,
                              const float* __restrict__ scale, float* __restrict__ dx) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)n * D) return;
  const int64_t i = idx / D;
  dx[idx] = scale[type[i]] * v[idx - i * D];
}

// per-block partial sums of a [n, stride] array's column `col` (fixed tree)
__global__ void k_block_sum(int64_t n, const float* __restrict__ a, float* __restrict__ part) {
  __shared__ float red[TPB];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  red[threadIdx.x] = i < n ? a[i] : 0.f;
  __syncthreads();
  for (int s = TPB / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}
// out[q] = sum_b part[b * k + q], q < k: one block of 256, thread t sums the
// strided subset b = t, t+256, ... in order, then a fixed tree (deterministic)
__global__ __launch_bounds__(256) void k_final_sum(int nb, int k, const float* __restrict__ part,
                                                   float* __restrict__ out) {
  __shared__ float red[TPB];
  for (int q = 0; q < k; ++q) {
    float s = 0.f;
    for (int b = threadIdx.x; b < nb; b += TPB) s += part[(int64_t)b * k + q];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = TPB / 2; o > 0; o >>= 1) {
      if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
      __syncthreads();
    }
    if (threadIdx.x == 0) out[q] = red[0];
    __syncthreads();
  }
}

// dh[j] = sum_{e: nbr[e] == j} dxc[e]  (transposed CSR, ascending edge order)
__global__ void k_gather_rows(int j_begin, int n, int D, const int* __restrict__ ptr,
                              const int* __restrict__ perm, const float* __restrict__ src,
                              float* __restrict__ dst, int acc) {
  const int j = j_begin + blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (j >= n) return;
  const int b = ptr[j], en = ptr[j + 1];
  for (int c = lane; c < D; c += 64) {
    float s = 0.f;
    for (int q = b; q < en; ++q) s += src[(int64_t)perm[q] * D + c];
    float* o = dst + (int64_t)j * D + c;
    *o = acc ? *o + s : s;
  }
}

// same sum, float4 columns (D % 4 == 0), one column per lane and pass, U rows
// in flight; the adds keep the ascending edge order, so the result is bitwise
// that of k_gather_rows.  (Measured against two columns per lane with 8 rows
// in flight -- 85 VGPRs, 5 waves per SIMD: 1.39 vs 0.94 ms per 480-wide
// launch; the occupancy of this 20-register form hides the row latency better;
// rows in flight U = 2 / 4 / 8 and non-temporal loads measured the same.)
#ifndef E3GNN_GATHER_V2
#define E3GNN_GATHER_V2 0
#endif
// rows of 65..128 float4 (SevenNet-0's middle blocks: 120): both halves of a
// row per pass, 8 rows in flight (E3GNN_GATHER_2H: 3.22 -> 3.13-3.15 ms for
// the three launches of a step, same box; profiles/r06_s14_*)
#ifndef E3GNN_GATHER_2H
#define E3GNN_GATHER_2H 1
#endif
#ifndef E3GNN_GATHER_U2
#define E3GNN_GATHER_U2 8
#endif
#ifndef E3GNN_GATHER_U
#define E3GNN_GATHER_U 4
#endif
// blockIdx.y = 1: the second (src, dst) pair of launch_gather_rows2
__global__ void k_gather_rows4(int j_begin, int n, int D4, const int* __restrict__ ptr,
                               const int* __restrict__ perm, const float4* __restrict__ src,
                               float4* __restrict__ dst, int acc, const float4* __restrict__ src2,
                               float4* __restrict__ dst2) {
  constexpr int U = E3GNN_GATHER_U;
  if (blockIdx.y) {
    src = src2;
    dst = dst2;
  }
  const int j = j_begin + xcd_block() * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (j >= n) return;
  const int b = ptr[j], en = ptr[j + 1];
  auto add = [](float4& s, const float4& v) {
    s.x += v.x;
    s.y += v.y;
    s.z += v.z;
    s.w += v.w;
  };
#if E3GNN_GATHER_V2
  // the node's row ids once per 64 (lane i holds perm[b + i]), each row id
  // broadcast from its lane (v_readlane: a scalar, no dependent index load
  // per batch of rows), the same ascending order as below
  if (en - b <= 64) {
    const int myidx = b + lane < en ? perm[b + lane] : 0;
    const int cnt = en - b;
    for (int c = lane; c < D4; c += 64) {
      float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
      int k = 0;
      for (; k + U <= cnt; k += U) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int row = __builtin_amdgcn_readlane(myidx, k + u);
          v[u] = src[(int64_t)row * D4 + c];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) add(s, v[u]);
      }
      for (; k < cnt; ++k) add(s, src[(int64_t)__builtin_amdgcn_readlane(myidx, k) * D4 + c]);
      if (acc) add(s, dst[(int64_t)j * D4 + c]);
      dst[(int64_t)j * D4 + c] = s;
    }
    return;
  }
#endif
#if E3GNN_GATHER_2H
  // rows of 65..128 float4: both halves of each row in the same pass (twice
  // the loads in flight per lane, one pass over the row indices)
  if (D4 > 64 && D4 <= 128) {
    constexpr int U2 = E3GNN_GATHER_U2;
    const int c0 = lane, c1 = lane + 64;
    const bool h1 = c1 < D4;
    float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0;
    int q = b;
    for (; q + U2 <= en; q += U2) {
      float4 v0[U2], v1[U2];
#pragma unroll
      for (int u = 0; u < U2; ++u) {
        const int64_t row = (int64_t)perm[q + u] * D4;
        v0[u] = src[row + c0];
        v1[u] = h1 ? src[row + c1] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < U2; ++u) {
        add(s0, v0[u]);
        add(s1, v1[u]);
      }
    }
    for (; q < en; ++q) {
      const int64_t row = (int64_t)perm[q] * D4;
      add(s0, src[row + c0]);
      if (h1) add(s1, src[row + c1]);
    }
    if (acc) {
      add(s0, dst[(int64_t)j * D4 + c0]);
      if (h1) add(s1, dst[(int64_t)j * D4 + c1]);
    }
    dst[(int64_t)j * D4 + c0] = s0;
    if (h1) dst[(int64_t)j * D4 + c1] = s1;
    return;
  }
#endif
  for (int c = lane; c < D4; c += 64) {
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    int q = b;
    for (; q + U <= en; q += U) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = src[(int64_t)perm[q + u] * D4 + c];
#pragma unroll
      for (int u = 0; u < U; ++u) add(s, v[u]);
    }
    for (; q < en; ++q) add(s, src[(int64_t)perm[q] * D4 + c]);
    if (acc) add(s, dst[(int64_t)j * D4 + c]);
    dst[(int64_t)j * D4 + c] = s;
  }
}

// halo pack / unpack: rows by index (pair_e3gnn_parallel.cpp:803-933)
__global__ void k_pack(int64_t n, int dim, const int* __restrict__ idx, const float* __restrict__ src,
                       int64_t ss, float* __restrict__ dst) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * dim) return;
  const int64_t r = t / dim;
  const int c = (int)(t - r * dim);
  dst[t] = src[(int64_t)idx[r] * ss + c];
}
__global__ void k_unpack(int64_t n, int dim, const int* __restrict__ idx, const float* __restrict__ src,
                         float* __restrict__ dst, int64_t ds, int acc) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * dim) return;
  const int64_t r = t / dim;
  const int c = (int)(t - r * dim);
  float* p = dst + (int64_t)idx[r] * ds + c;
  *p = acc ? *p + src[t] : src[t];
}

}  // namespace

#define LAUNCH(k, grid, ...)                                   \
  do {                                                         \
    if ((grid) > 0) hipLaunchKernelGGL(k, dim3(grid), dim3(TPB), 0, s, __VA_ARGS__); \
  } while (0)

hipError_t launch_edge_embed(int64_t E, const float* vec, const float* coeffs, float rc, float ron,
                             int raw_sh, float* Y, float* emb, hipStream_t s) {
  LAUNCH(k_edge_embed, nblk(E), E, vec, coeffs, rc, ron, raw_sh, Y, emb);
  return hipGetLastError();
}
hipError_t launch_edge_geom_jvp(int64_t E, const float* vec, const float* coeffs, float rc, float ron,
                                int raw_sh, const int* center, const int* nbr, const int64_t* batch,
                                const float* cF, const float* cS, const float* vol, float* Yd,
                                float* embd, float* rd, hipStream_t s) {
  if (E <= 0) return hipSuccess;
  LAUNCH(k_edge_geom_jvp, nblk(E), E, vec, coeffs, rc, ron, raw_sh, center, nbr, batch, cF, cS, vol,
         Yd, embd, rd);
  return hipGetLastError();
}
hipError_t launch_edge_geom_coeff(int64_t E, const float* vec, const float* coeffs, float rc,
                                  float ron, const float* embb, const float* embdb, const float* rd,
                                  float* out, hipStream_t s) {
  if (E <= 0) return hipSuccess;
  LAUNCH(k_edge_geom_coeff, nblk(E), E, vec, coeffs, rc, ron, embb, embdb, rd, out);
  return hipGetLastError();
}
int edge_force_blocks(int64_t E) { return nblk(E); }
hipError_t launch_edge_force(int64_t E, const float* vec, const float* coeffs, float rc, float ron,
                             int raw_sh, const float* dY, const float* dgu, const float* demb, float* fe,
                             float* vir_part, hipStream_t s) {
  LAUNCH(k_edge_force, nblk(E), E, vec, coeffs, rc, ron, raw_sh, dY, dgu, demb, fe, vir_part);
  return hipGetLastError();
}
hipError_t launch_atom_force(int n_nodes, int n_centers, const int* row_ptr, const int* src_ptr,
                             const int* src_perm, const float* fe, float* F, hipStream_t s) {
  LAUNCH(k_atom_force, nblk(n_nodes), n_nodes, n_centers, row_ptr, src_ptr, src_perm, fe, F);
  return hipGetLastError();
}
// zero fill as a KERNEL: ops that a HIP graph may capture (the fine-tune
// step's convolution backward) zero their accumulators with this rather than
// hipMemsetAsync -- a captured memset node did not re-zero the buffer on
// replay here (the graphed step then accumulated into stale values)
__global__ void k_zero(int64_t n, float* __restrict__ p) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = 0.f;
}
hipError_t launch_zero(float* p, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t b = std::min<int64_t>((n + 255) / 256, 65536);
  hipLaunchKernelGGL(k_zero, dim3((unsigned)b), dim3(256), 0, s, n, p);
  return hipGetLastError();
}
hipError_t launch_build_graph(int64_t E, int n_centers, int n_nodes, const int* center,
                              const int* nbr, int* row_ptr, int* src_ptr, int* src_perm,
                              int* cnt, int* err, hipStream_t s, int n_interior) {
  LAUNCH(k_fill_int, nblk(n_centers + 1), n_centers + 1, 0, row_ptr);
  LAUNCH(k_row_ptr, nblk(E), E, n_centers, n_nodes, n_interior, center, nbr, row_ptr, err);
  LAUNCH(k_fill_int, nblk(n_nodes), n_nodes, 0, cnt);
  LAUNCH(k_count_nbr, nblk(E), E, nbr, n_nodes, cnt);
  const int nb = (n_nodes + SCAN_B - 1) / SCAN_B;
  if (nb > 0 && E >= nb) {  // block totals in src_perm[0, nb): k_scatter_perm overwrites them
    hipLaunchKernelGGL(k_scan_blocks, dim3(nb), dim3(256), 0, s, n_nodes, cnt, src_ptr, src_perm);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(1024), 0, s, nb, n_nodes, src_perm, src_ptr);
    hipLaunchKernelGGL(k_scan_add, dim3(nb), dim3(256), 0, s, n_nodes, src_perm, src_ptr);
  } else {
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, s, n_nodes, cnt, src_ptr);
  }
  LAUNCH(k_fill_int, nblk(n_nodes), n_nodes, 0, cnt);
  LAUNCH(k_scatter_perm, nblk(E), E, nbr, n_nodes, src_ptr, cnt, src_perm);
  if (n_nodes > 0)
    hipLaunchKernelGGL(k_sort_segments, dim3((n_nodes + 3) / 4), dim3(256), 0, s, n_nodes, src_ptr, src_perm);
  return hipGetLastError();
}
hipError_t launch_build_graph_small(int64_t E, int n, const int* c32, const int* j32, const int64_t* c64,
                                    const int64_t* j64, int* cout, int* jout, int* row_ptr, int* src_ptr,
                                    int* src_perm, int* err, hipStream_t s) {
  if (n < 0 || n > GRAPH_SMALL_N || E < 0 || E > GRAPH_SMALL_E) return hipErrorInvalidValue;
  if (c64)
    hipLaunchKernelGGL(k_build_graph_small<int64_t>, dim3(1), dim3(1024), 0, s, (int)E, n, c64, j64, cout,
                       jout, row_ptr, src_ptr, src_perm, err);
  else
    hipLaunchKernelGGL(k_build_graph_small<int>, dim3(1), dim3(1024), 0, s, (int)E, n, c32, j32, cout, jout,
                       row_ptr, src_ptr, src_perm, err);
  return hipGetLastError();
}
int graph_small_max_nodes() { return GRAPH_SMALL_N; }
int graph_small_max_edges() { return GRAPH_SMALL_E; }
hipError_t launch_embed(int n, int D, const int* type, int nsp, const float* W, float* x, int* err,
                        hipStream_t s) {
  LAUNCH(k_embed, nblk((int64_t)n * D), n, D, type, nsp, W, x, err);
  return hipGetLastError();
}
hipError_t launch_gate_fwd(int n, bool last, GateDims d, const float* y, float* x, hipStream_t s) {
  if (last) LAUNCH(k_act_fwd, nblk((int64_t)n * d.ns), (int64_t)n * d.ns, y, x);
  else LAUNCH(k_gate_fwd, nblk((int64_t)n * d.dx()), n, d, y, x);
  return hipGetLastError();
}
hipError_t launch_gate_bwd(int n, bool last, GateDims d, const float* y, const float* dx, float* dy,
                           hipStream_t s) {
  if (last) LAUNCH(k_act_bwd, nblk((int64_t)n * d.ns), (int64_t)n * d.ns, y, dx, dy);
  else if (n > 0) {
    if (d.dy() % 4 || d.dx() % 4) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_gate_bwd_rows, dim3((n + 3) / 4), dim3(256), 4 * (d.dy() + d.dx()) * sizeof(float),
                       s, n, d, y, dx, dy);
  }
  return hipGetLastError();
}
hipError_t launch_readout(int n, int D, const float* x, const float* v, const int* type,
                          const float* scale, const float* shift, float* eat, hipStream_t s) {
  if (n > 0)
    hipLaunchKernelGGL(k_readout, dim3((n + 3) / 4), dim3(256), 0, s, n, D, x, v, type, scale, shift,
                       eat);
  return hipGetLastError();
}
hipError_t launch_readout_bwd(int n, int D, const float* v, const int* type, const float* scale,
                              float* dx, hipStream_t s) {
  LAUNCH(k_readout_bwd, nblk((int64_t)n * D), n, D, v, type, scale, dx);
  return hipGetLastError();
}
int sum_blocks(int64_t n) { return nblk(n); }
hipError_t launch_sum(int64_t n, const float* a, float* part, float* out, hipStream_t s) {
  const int nb = nblk(n);
  if (nb == 0) {
    return launch_zero(out, 1, s);
  }
  LAUNCH(k_block_sum, nb, n, a, part);
  hipLaunchKernelGGL(k_final_sum, dim3(1), dim3(TPB), 0, s, nb, 1, part, out);
  return hipGetLastError();
}
hipError_t launch_final_sum(int nb, int k, const float* part, float* out, hipStream_t s) {
  if (nb == 0) {
    return launch_zero(out, k, s);
  }
  hipLaunchKernelGGL(k_final_sum, dim3(1), dim3(TPB), 0, s, nb, k, part, out);
  return hipGetLastError();
}
hipError_t launch_gather_rows(int n, int D, const int* ptr, const int* perm, const float* src,
                              float* dst, hipStream_t s, int acc) {
  return launch_gather_rows_range(0, n, D, ptr, perm, src, dst, s, acc);
}
hipError_t launch_gather_rows_range(int j_begin, int j_end, int D, const int* ptr, const int* perm,
                                    const float* src, float* dst, hipStream_t s, int acc) {
  const int n = j_end - j_begin;
  if (n <= 0) return hipGetLastError();
  if (D % 4 == 0) {
    hipLaunchKernelGGL(k_gather_rows4, dim3((n + 3) / 4), dim3(256), 0, s, j_begin, j_end, D / 4,
                       ptr, perm, (const float4*)src, (float4*)dst, acc, nullptr, nullptr);
  } else {
    hipLaunchKernelGGL(k_gather_rows, dim3((n + 3) / 4), dim3(256), 0, s, j_begin, j_end, D, ptr,
                       perm, src, dst, acc);
  }
  return hipGetLastError();
}
hipError_t launch_gather_rows2(int n, int D, const int* ptr, const int* perm, const float* src,
                               float* dst, const float* src2, float* dst2, hipStream_t s) {
  if (n <= 0) return hipGetLastError();
  if (D % 4) {
    const hipError_t e = launch_gather_rows_range(0, n, D, ptr, perm, src, dst, s, 0);
    return e != hipSuccess ? e : launch_gather_rows_range(0, n, D, ptr, perm, src2, dst2, s, 0);
  }
  hipLaunchKernelGGL(k_gather_rows4, dim3((n + 3) / 4, 2), dim3(256), 0, s, 0, n, D / 4, ptr, perm,
                     (const float4*)src, (float4*)dst, 0, (const float4*)src2, (float4*)dst2);
  return hipGetLastError();
}
hipError_t launch_pack(int64_t n, int dim, const int* idx, const float* src, int64_t ss, float* dst,
                       hipStream_t s) {
  LAUNCH(k_pack, nblk(n * dim), n, dim, idx, src, ss, dst);
  return hipGetLastError();
}
hipError_t launch_unpack(int64_t n, int dim, const int* idx, const float* src, float* dst,
                         int64_t ds, int acc, hipStream_t s) {
  LAUNCH(k_unpack, nblk(n * dim), n, dim, idx, src, dst, ds, acc);
  return hipGetLastError();
}

}  // namespace e3gnn
