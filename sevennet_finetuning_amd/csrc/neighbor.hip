// Device neighbour list (cell list) -> CSR edge list sorted by (i, j, S), gfx950.
//
// Replaces the graph-building step in front of the hot path: ASE
// primitive_neighbor_list('ijDS', pbc, cell, pos, cutoff, self_interaction=True)
// followed by the removal of the i == j, S == 0 pair in the reference
// (sevenn/train/dataload.py:31-68, :113-125), and the host loops over LAMMPS'
// full neighbour list in pair_e3gnn.cpp:155-182.
//
// Edge (i, j, S): r_ij = (pos[j] + S cell) - pos[i], |r_ij|^2 < rc^2, S integer,
// excluding i == j with S == 0.  The inclusion test is evaluated in f64 in
// exactly this operation order with contraction off, the same arithmetic as the
// host list (neighbor.py), so both give the same edges bit for bit.  Binning
// only accelerates the search: atoms are wrapped into the cell, binned with bin
// widths >= rc, and every centre scans the (2R+1)^3 bin images around its bin
// (distinct (bin, image) pairs, so every periodic image is visited once).
//
// Pass 1 counts each centre's edges (one wave per centre, ballot), a scan gives
// the CSR offsets, pass 2 recomputes the hits into LDS, sorts the centre's keys
// (j, Sx, Sy, Sz) with a bitonic network and writes them: deterministic.
#include "neighbor.h"

#pragma clang fp contract(off)

namespace e3gnn {
namespace {

// ---------------------------------------------------------------- binning
__global__ void k_nl_bin(int n, const double* __restrict__ pos, NlGeom G, int* __restrict__ f0,
                         int* __restrict__ bin, int* __restrict__ bin_count, int* __restrict__ err) {
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= n) return;
  const double p0 = pos[3 * a] - G.origin[0], p1 = pos[3 * a + 1] - G.origin[1],
               p2 = pos[3 * a + 2] - G.origin[2];
  int b[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const double f = ((p0 * G.inv[k]) + (p1 * G.inv[3 + k])) + (p2 * G.inv[6 + k]);
    const double fl = floor(f);
    const double fw = f - fl;
    int bk = (int)(fw * G.nb[k]);
    bk = bk < 0 ? 0 : (bk >= G.nb[k] ? G.nb[k] - 1 : bk);
    b[k] = bk;
    if (!(fl > -1e9 && fl < 1e9)) atomicOr(err, 1);  // non-finite or absurd position
    f0[3 * a + k] = (int)fl;
  }
  if (!G.periodic && (f0[3 * a] | f0[3 * a + 1] | f0[3 * a + 2])) atomicOr(err, 1);
  const int id = (b[0] * G.nb[1] + b[1]) * G.nb[2] + b[2];
  bin[a] = id;
  atomicAdd(&bin_count[id], 1);
}

__global__ void k_nl_place(int n, const int* __restrict__ bin, const int* __restrict__ bin_start,
                           int* __restrict__ cursor, int* __restrict__ bin_atoms) {
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= n) return;
  const int id = bin[a];
  bin_atoms[bin_start[id] + atomicAdd(&cursor[id], 1)] = a;
}

// exclusive scan of cnt[0..n) into out[0..n] (out[n] = total), one workgroup
__global__ __launch_bounds__(1024) void k_nl_scan(int n, const int* __restrict__ cnt,
                                                  int* __restrict__ out) {
  __shared__ long long part[1024];
  const int t = threadIdx.x;
  const int chunk = (n + 1023) / 1024;
  const int b = t * chunk, e = min(b + chunk, n);
  long long s = 0;
  for (int i = b; i < e; ++i) s += cnt[i];
  part[t] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan
    const long long v = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  long long run = part[t] - s;
  for (int i = b; i < e; ++i) {
    out[i] = (int)run;
    run += cnt[i];
  }
  if (t == 1023) out[n] = (int)part[1023];
}

// ---------------------------------------------------------------- search
// key = j << 33 | (Sx + 2^10) << 22 | (Sy + 2^10) << 11 | (Sz + 2^10): ascending
// keys are ascending (j, Sx, Sy, Sz)
constexpr int SB = 10;
__device__ __forceinline__ unsigned long long nl_key(int j, int sx, int sy, int sz) {
  return ((unsigned long long)j << 33) | ((unsigned long long)(sx + (1 << SB)) << 22) |
         ((unsigned long long)(sy + (1 << SB)) << 11) | (unsigned long long)(sz + (1 << SB));
}

struct Hit {
  double d[3];
};
// r_ij for (i, j, S): (pos_j + S cell) - pos_i, the host list's operation order
__device__ __forceinline__ Hit nl_vec(const double* __restrict__ pos, const NlGeom& G, int i,
                                      int j, int sx, int sy, int sz) {
  Hit h;
  const double s0 = sx, s1 = sy, s2 = sz;
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const double sc = ((s0 * G.cell[d]) + (s1 * G.cell[3 + d])) + (s2 * G.cell[6 + d]);
    h.d[d] = (pos[3 * j + d] + sc) - pos[3 * i + d];
  }
  return h;
}

// one wave per centre; FILL = false: count, true: collect, sort, write
template <bool FILL>
__global__ __launch_bounds__(256) void k_nl_search(
    int n, const double* __restrict__ pos, NlGeom G, const int* __restrict__ f0,
    const int* __restrict__ bin, const int* __restrict__ bin_start,
    const int* __restrict__ bin_atoms, int* __restrict__ deg, const int* __restrict__ row_ptr,
    int* __restrict__ center, int* __restrict__ nbr, int* __restrict__ shift,
    float* __restrict__ vec, int* __restrict__ err) {
  __shared__ unsigned long long keys[4][NL_MAXD];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int i = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + wid);
  if (i >= n) return;
  unsigned long long* K = keys[wid];
  const int bi = bin[i];
  const int b[3] = {bi / (G.nb[1] * G.nb[2]), (bi / G.nb[2]) % G.nb[1], bi % G.nb[2]};
  const int fi[3] = {f0[3 * i], f0[3 * i + 1], f0[3 * i + 2]};
  const double rc2 = G.rc2;
  int count = 0;  // uniform
  for (int ox = -G.R[0]; ox <= G.R[0]; ++ox)
    for (int oy = -G.R[1]; oy <= G.R[1]; ++oy)
      for (int oz = -G.R[2]; oz <= G.R[2]; ++oz) {
        const int o[3] = {ox, oy, oz};
        int c[3], sh[3];
        bool skip = false;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int v = b[k] + o[k];
          if (G.periodic) {
            sh[k] = v >= 0 ? v / G.nb[k] : -((-v + G.nb[k] - 1) / G.nb[k]);
            c[k] = v - sh[k] * G.nb[k];
          } else {
            sh[k] = 0;
            c[k] = v;
            skip |= v < 0 || v >= G.nb[k];
          }
        }
        if (skip) continue;
        const int id = (c[0] * G.nb[1] + c[1]) * G.nb[2] + c[2];
        const int s = bin_start[id], e = bin_start[id + 1];
        for (int t0 = s; t0 < e; t0 += 64) {
          const int t = t0 + lane;
          bool hit = false;
          int j = 0, S[3] = {0, 0, 0};
          if (t < e) {
            j = bin_atoms[t];
#pragma unroll
            for (int k = 0; k < 3; ++k) S[k] = sh[k] + fi[k] - f0[3 * j + k];
            const Hit h = nl_vec(pos, G, i, j, S[0], S[1], S[2]);
            const double r2 = ((h.d[0] * h.d[0]) + (h.d[1] * h.d[1])) + (h.d[2] * h.d[2]);
            hit = r2 < rc2 && !(j == i && S[0] == 0 && S[1] == 0 && S[2] == 0);
          }
          const unsigned long long m = __ballot(hit);
          if (FILL && hit) {
            const int slot = count + __popcll(m & ((1ull << lane) - 1));
            const int lim = 1 << SB;
            if (S[0] < -lim || S[0] >= lim || S[1] < -lim || S[1] >= lim || S[2] < -lim ||
                S[2] >= lim)
              atomicOr(err, 2);
            else if (slot < NL_MAXD)
              K[slot] = nl_key(j, S[0], S[1], S[2]);
          }
          count += __popcll(m);
        }
      }
  if constexpr (!FILL) {
    if (lane == 0) {
      deg[i] = count;
      if (count > NL_MAXD) atomicOr(err, 4);
    }
    return;
  } else {
    if (count > NL_MAXD) return;  // reported by the count pass
    // bitonic sort of K[0..P) (P = next power of two; padding = max key)
    int P = 1;
    while (P < count) P <<= 1;
    for (int t = count + lane; t < P; t += 64) K[t] = ~0ull;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    for (int k = 2; k <= P; k <<= 1)
      for (int jj = k >> 1; jj > 0; jj >>= 1) {
        for (int t = lane; t < P; t += 64) {
          const int u = t ^ jj;
          if (u > t) {
            const unsigned long long a = K[t], c = K[u];
            const bool up = (t & k) == 0;
            if ((a > c) == up) {
              K[t] = c;
              K[u] = a;
            }
          }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      }
    const int base = row_ptr[i];
    for (int t = lane; t < count; t += 64) {
      const unsigned long long key = K[t];
      const int j = (int)(key >> 33);
      const int sx = (int)((key >> 22) & 0x7ff) - (1 << SB);
      const int sy = (int)((key >> 11) & 0x7ff) - (1 << SB);
      const int sz = (int)(key & 0x7ff) - (1 << SB);
      const Hit h = nl_vec(pos, G, i, j, sx, sy, sz);
      const int64_t q = (int64_t)base + t;
      center[q] = i;
      nbr[q] = j;
      if (shift) {
        shift[3 * q] = sx;
        shift[3 * q + 1] = sy;
        shift[3 * q + 2] = sz;
      }
      if (vec) {
        vec[3 * q] = (float)h.d[0];
        vec[3 * q + 1] = (float)h.d[1];
        vec[3 * q + 2] = (float)h.d[2];
      }
    }
  }
}

}  // namespace

hipError_t launch_nl_bin(int n, const double* pos, const NlGeom& G, int* f0, int* bin,
                         int* bin_count, int* err, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_nl_bin, dim3((n + 255) / 256), dim3(256), 0, s, n, pos, G, f0, bin,
                     bin_count, err);
  return hipGetLastError();
}
hipError_t launch_nl_place(int n, const int* bin, const int* bin_start, int* cursor,
                           int* bin_atoms, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_nl_place, dim3((n + 255) / 256), dim3(256), 0, s, n, bin, bin_start,
                     cursor, bin_atoms);
  return hipGetLastError();
}
hipError_t launch_nl_scan(int n, const int* cnt, int* out, hipStream_t s) {
  hipLaunchKernelGGL(k_nl_scan, dim3(1), dim3(1024), 0, s, n, cnt, out);
  return hipGetLastError();
}
hipError_t launch_nl_search(bool fill, int n, const double* pos, const NlGeom& G, const int* f0,
                            const int* bin, const int* bin_start, const int* bin_atoms, int* deg,
                            const int* row_ptr, int* center, int* nbr, int* shift, float* vec,
                            int* err, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const dim3 grid((n + 3) / 4), block(256);
  if (fill)
    hipLaunchKernelGGL(k_nl_search<true>, grid, block, 0, s, n, pos, G, f0, bin, bin_start,
                       bin_atoms, deg, row_ptr, center, nbr, shift, vec, err);
  else
    hipLaunchKernelGGL(k_nl_search<false>, grid, block, 0, s, n, pos, G, f0, bin, bin_start,
                       bin_atoms, deg, row_ptr, center, nbr, shift, vec, err);
  return hipGetLastError();
}

}  // namespace e3gnn
