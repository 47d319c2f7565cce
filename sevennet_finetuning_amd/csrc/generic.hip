// Node and edge kernels of the generic nequip-family engine (generic.cpp):
// any deployment of the reference's E3_equivariant_model that is not
// SevenNet-0's architecture -- irreps with parity, lmax <= 2, XPLOR or
// polynomial cutoff, normalised or raw-vector spherical harmonics, `linear` or
// `nequip` self-connection, silu / tanh gates.  The convolution itself runs on
// the runtime-path-table kernels (gtp.hip) and the dense products on k_gemm;
// these are the small row- and edge-wise pieces around them, each with its
// hand-written reverse-mode counterpart (what ForceStressOutput obtains by
// autograd, force_output.py:74-130).  Deterministic: one thread owns every
// output it writes, sums run in a fixed order, no float atomics.
#include "common.h"
#include "generic.h"

namespace e3gnn {
namespace {

constexpr int TPB = 256;
inline int nblk(int64_t n) { return (int)((n + TPB - 1) / TPB); }

// ------------------------------------------------------------ activations
// act 0: silu * silu_norm (e3nn normalize2mom(silu)), 1: tanh * tanh_norm
// (sevenn/_const.py act table; the 'o' parity gates of equivariant_gate.py)
__device__ __forceinline__ float gen_act(int a, float x, float tn) {
  if (a == 0) return act_fwd(x);
  return tn * tanhf(x);
}
__device__ __forceinline__ float gen_act_grad(int a, float x, float tn) {
  if (a == 0) return act_grad(x);
  const float t = tanhf(x);
  return tn * (1.f - t * t);
}

// ------------------------------------------------------------ node embedding
// OnehotEmbedding + the linear onto 'mul x 0e' (node_embedding.py:39-48,
// linear.py:37-44): row n = W[type n] (pre-scaled by 1/sqrt(num_species))
__global__ void k_gen_embed(int n, int d, const int* __restrict__ type, int nsp,
                            const float* __restrict__ W, float* __restrict__ x, int* __restrict__ err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)n * d) return;
  const int node = (int)(i / d), c = (int)(i - (int64_t)node * d);
  const int t = type[node];
  if (t < 0 || t >= nsp) {
    if (c == 0) err[0] |= 8;   // (same flag as the SevenNet-0 embed)
    x[i] = 0.f;
    return;
  }
  x[i] = W[t * d + c];
}

// ------------------------------------------------------------ edge geometry
// EdgeEmbedding (edge_embedding.py:220-230): BesselBasis (:114-116) times the
// XPLOR (:163-173) or polynomial (:131-145) cutoff, and SphericalEncoding
// (:177-198; e3nn 'component' real SH, lmax <= 2) of the unit vector or --
// sh_normalize false, sevenn < 0.9 (util.py:143-144) -- of the raw vector.
struct Env {
  float v, d;  // envelope and d envelope / dr
};
__device__ __forceinline__ Env envelope(const GenEdgeArgs& a, float r) {
  Env o{1.f, 0.f};
  if (a.cut == 0) {  // XPLOR
    if (r >= a.ron) {
      const float rc2 = a.rc * a.rc, r2 = r * r, ron2 = a.ron * a.ron;
      const float q = rc2 - r2, d = rc2 - ron2, d3 = d * d * d;
      o.v = q * q * (rc2 + 2.f * r2 - 3.f * ron2) / d3;
      o.d = 12.f * r * q * (ron2 - r2) / d3;
    }
  } else {  // poly_cut, p
    const float p = a.p, x = r / a.rc;
    const float xp = powf(x, p), xp1 = xp * x, xp2 = xp1 * x;
    o.v = 1.f - 0.5f * (p + 1.f) * (p + 2.f) * xp + p * (p + 2.f) * xp1 - 0.5f * p * (p + 1.f) * xp2;
    // d/dr: (p(p+1)(p+2)/2) (-x^(p-1) + 2 x^p - x^(p+1)) / rc
    const float xm1 = x > 0.f ? xp / x : 0.f;
    o.d = 0.5f * p * (p + 1.f) * (p + 2.f) * (-xm1 + 2.f * xp - xp1) / a.rc;
  }
  return o;
}

// Y_j = sum_f M[f][j] mono_f with mono = [1, u, u (x) u] (nn.spherical_harmonics)
__device__ __forceinline__ void sh_eval(int lmax, float x, float y, float z, float* Y) {
  const float s3 = 1.7320508075688772f, s5 = 2.23606797749979f, s15 = s3 * s5;
  Y[0] = 1.f;
  if (lmax >= 1) {
    Y[1] = s3 * x;
    Y[2] = s3 * y;
    Y[3] = s3 * z;
  }
  if (lmax >= 2) {
    Y[4] = s15 * x * z;
    Y[5] = s15 * x * y;
    Y[6] = s5 * (y * y - 0.5f * (x * x + z * z));
    Y[7] = s15 * y * z;
    Y[8] = 0.5f * s15 * (z * z - x * x);
  }
}
// g = dE/du for the polynomial above (dE/dY given)
__device__ __forceinline__ void sh_grad(int lmax, float x, float y, float z, const float* g,
                                        float& gx, float& gy, float& gz) {
  const float s3 = 1.7320508075688772f, s5 = 2.23606797749979f, s15 = s3 * s5;
  gx = gy = gz = 0.f;
  if (lmax >= 1) {
    gx = s3 * g[1];
    gy = s3 * g[2];
    gz = s3 * g[3];
  }
  if (lmax >= 2) {
    gx += s15 * (z * g[4] + y * g[5]) - s5 * x * g[6] - s15 * x * g[8];
    gy += s15 * (x * g[5] + z * g[7]) + 2.f * s5 * y * g[6];
    gz += s15 * (x * g[4] + y * g[7]) - s5 * z * g[6] + s15 * z * g[8];
  }
}

__global__ void k_gen_edge_embed(GenEdgeArgs a, int64_t E, const float* __restrict__ vec,
                                 float* __restrict__ Y, float* __restrict__ emb) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const float vx = vec[3 * e], vy = vec[3 * e + 1], vz = vec[3 * e + 2];
  const float r = sqrtf(vx * vx + vy * vy + vz * vz);
  float y[9];
  if (a.normalize) sh_eval(a.lmax, vx / r, vy / r, vz / r, y);
  else sh_eval(a.lmax, vx, vy, vz, y);
  const int ny = (a.lmax + 1) * (a.lmax + 1);
  for (int j = 0; j < ny; ++j) Y[e * ny + j] = y[j];
  const Env en = envelope(a, r);
  for (int b = 0; b < a.nb; ++b)
    emb[e * a.nb + b] = (2.f / a.rc) * sinf(a.coeffs[b] * r) / r * en.v;
}

// dE/dr_ij from dE/dY and dE/demb (all layers), per-block virial partials
// (virial = -dE/dstrain, the convention of node.hip k_edge_force)
__global__ __launch_bounds__(TPB) void k_gen_edge_force(GenEdgeArgs a, int64_t E,
                                                         const float* __restrict__ vec,
                                                         const float* __restrict__ dY,
                                                         const float* __restrict__ demb,
                                                         float* __restrict__ fe,
                                                         float* __restrict__ vir_part) {
  __shared__ float red[6][TPB];
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float v6[6] = {0, 0, 0, 0, 0, 0};
  if (e < E) {
    const float vx = vec[3 * e], vy = vec[3 * e + 1], vz = vec[3 * e + 2];
    const float r = sqrtf(vx * vx + vy * vy + vz * vz);
    const float ux = vx / r, uy = vy / r, uz = vz / r;
    const int ny = (a.lmax + 1) * (a.lmax + 1);
    float gx, gy, gz, fx, fy, fz;
    if (a.normalize) {
      sh_grad(a.lmax, ux, uy, uz, dY + e * ny, gx, gy, gz);
      const float dot = gx * ux + gy * uy + gz * uz;
      fx = (gx - dot * ux) / r;
      fy = (gy - dot * uy) / r;
      fz = (gz - dot * uz) / r;
    } else {
      sh_grad(a.lmax, vx, vy, vz, dY + e * ny, fx, fy, fz);
    }
    const Env en = envelope(a, r);
    float dr = 0.f;
    for (int b = 0; b < a.nb; ++b) {
      const float cb = a.coeffs[b];
      const float sn = sinf(cb * r), cs = cosf(cb * r);
      const float bv = (2.f / a.rc) * sn / r;
      const float db = (2.f / a.rc) * (cb * cs * r - sn) / (r * r);
      dr += demb[e * a.nb + b] * (db * en.v + bv * en.d);
    }
    fx += dr * ux;
    fy += dr * uy;
    fz += dr * uz;
    fe[3 * e] = fx;
    fe[3 * e + 1] = fy;
    fe[3 * e + 2] = fz;
    v6[0] = -(vx * fx);
    v6[1] = -(vy * fy);
    v6[2] = -(vz * fz);
    v6[3] = -0.5f * (vx * fy + vy * fx);
    v6[4] = -0.5f * (vy * fz + vz * fy);
    v6[5] = -0.5f * (vx * fz + vz * fx);
  }
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

// ------------------------------------------------------------ gate
// e3nn Gate (equivariant_gate.py:59-61) on e3nn's (l, p)-sorted input row:
// column o of the output is act_o(y[src]) (scalar) or act_g(y[gate]) y[src]
// (gated), per the host's column table.  One thread per row: the backward
// sums a gate's 2l+1 products in a fixed order.
__global__ void k_gen_gate_fwd(int n, GenGateArgs g, const float* __restrict__ y,
                               float* __restrict__ x) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* yr = y + (int64_t)i * g.din;
  float* xr = x + (int64_t)i * g.dout;
  for (int o = 0; o < g.dout; ++o) {
    const GenGateCol c = g.cols[o];
    xr[o] = c.gate < 0 ? gen_act(c.act, yr[c.src], g.tanh_norm)
                       : gen_act(c.act, yr[c.gate], g.tanh_norm) * yr[c.src];
  }
}
__global__ void k_gen_gate_bwd(int n, GenGateArgs g, const float* __restrict__ y,
                               const float* __restrict__ dx, float* __restrict__ dy) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* yr = y + (int64_t)i * g.din;
  const float* dr = dx + (int64_t)i * g.dout;
  float* o = dy + (int64_t)i * g.din;
  for (int k = 0; k < g.din; ++k) o[k] = 0.f;
  for (int q = 0; q < g.dout; ++q) {
    const GenGateCol c = g.cols[q];
    if (c.gate < 0) {
      o[c.src] += dr[q] * gen_act_grad(c.act, yr[c.src], g.tanh_norm);
    } else {
      const float gv = yr[c.gate];
      o[c.src] += dr[q] * gen_act(c.act, gv, g.tanh_norm);
      o[c.gate] += dr[q] * yr[c.src] * gen_act_grad(c.act, gv, g.tanh_norm);
    }
  }
}

// ------------------------------------------------------------ species-wise linear
// SelfConnectionIntro (self_connection.py:11-38): FullyConnectedTensorProduct
// of x with the one-hot species vector = a dense (din x dout) matrix per
// species; y[n] (+)= x[n] W[type n].  One thread per output element, k in order.
__global__ void k_gen_species_linear(int n, int din, int dout, const int* __restrict__ type,
                                     const float* __restrict__ x, const float* __restrict__ W,
                                     float* __restrict__ y, int beta) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)n * dout) return;
  const int node = (int)(i / dout), j = (int)(i - (int64_t)node * dout);
  const float* xr = x + (int64_t)node * din;
  const float* w = W + (int64_t)type[node] * din * dout + j;
  float s = 0.f;
  for (int k = 0; k < din; ++k) s += xr[k] * w[(int64_t)k * dout];
  y[i] = beta ? y[i] + s : s;
}

// ------------------------------------------------------------ readout
// reduce_input_to_hidden -> reduce_hidden_to_energy (two linears, no
// activation: one vector v), SpeciesWiseRescale (scale.py:67-73);
// the backward row dE/dx[n] = v * scale[type n] (owned rows only)
__global__ void k_gen_readout(int n, int d, const float* __restrict__ x, const float* __restrict__ v,
                              const int* __restrict__ type, const float* __restrict__ scale,
                              const float* __restrict__ shift, int per_species,
                              float* __restrict__ eat, float* __restrict__ dx) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* xr = x + (int64_t)i * d;
  float s = 0.f;
  for (int c = 0; c < d; ++c) s += xr[c] * v[c];
  const int t = per_species ? type[i] : 0;
  eat[i] = s * scale[t] + shift[t];
  float* g = dx + (int64_t)i * d;
  for (int c = 0; c < d; ++c) g[c] = v[c] * scale[t];
}

// ------------------------------------------------------------ linear biases
// e3nn o3.Linear(biases=True) (use_bias_in_linear): + b[c] on every row; b is
// the full-width vector (zero on the columns of non-0e output irreps)
__global__ void k_gen_bias(int64_t n, int d, const float* __restrict__ b, float* __restrict__ y) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n * d) y[i] += b[i % d];
}

// ------------------------------------------------------------ readout FCN
// FCN_e3nn (nn/linear.py:94-129): e3nn FullyConnectedNet's activation
// c f(z) (c = normalize2mom(f)) and its derivative c f'(z).  kind: 0 relu,
// 1 silu, 2 tanh, 3 sigmoid, 4 abs, 5 elu (sevenn/_const.py ACTIVATION)
__device__ __forceinline__ void gen_act(int kind, float z, float& f, float& df) {
  switch (kind) {
    case 0: f = z > 0.f ? z : 0.f; df = z > 0.f ? 1.f : 0.f; break;
    case 1: {
      const float sg = 1.f / (1.f + __expf(-z));
      f = z * sg;
      df = sg * (1.f + z * (1.f - sg));
      break;
    }
    case 2: {
      const float t = tanhf(z);
      f = t;
      df = 1.f - t * t;
      break;
    }
    case 3: {
      const float sg = 1.f / (1.f + __expf(-z));
      f = sg;
      df = sg * (1.f - sg);
      break;
    }
    case 4: f = fabsf(z); df = z > 0.f ? 1.f : (z < 0.f ? -1.f : 0.f); break;
    default: f = z > 0.f ? z : expm1f(z); df = z > 0.f ? 1.f : __expf(z); break;
  }
}
// mode 0: a = c f(z); mode 1: g = g_in * c f'(z)
__global__ void k_gen_fcn_act(int64_t n, int kind, float c, int mode, const float* __restrict__ z,
                              const float* __restrict__ gin, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float f, df;
  gen_act(kind, z[i], f, df);
  out[i] = mode == 0 ? c * f : gin[i] * c * df;
}

__global__ void k_gen_add(int64_t n, const float* __restrict__ a, float* __restrict__ acc) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) acc[i] += a[i];
}

}  // namespace

#define GLAUNCH(k, nb, ...)                                                 \
  do {                                                                      \
    if ((nb) > 0) hipLaunchKernelGGL(k, dim3(nb), dim3(TPB), 0, s, __VA_ARGS__); \
  } while (0)

hipError_t launch_gen_embed(int n, int d, const int* type, int nsp, const float* W, float* x,
                            int* err, hipStream_t s) {
  GLAUNCH(k_gen_embed, nblk((int64_t)n * d), n, d, type, nsp, W, x, err);
  return hipGetLastError();
}
hipError_t launch_gen_edge_embed(const GenEdgeArgs& a, int64_t E, const float* vec, float* Y,
                                 float* emb, hipStream_t s) {
  GLAUNCH(k_gen_edge_embed, nblk(E), a, E, vec, Y, emb);
  return hipGetLastError();
}
int gen_edge_force_blocks(int64_t E) { return nblk(E); }
hipError_t launch_gen_edge_force(const GenEdgeArgs& a, int64_t E, const float* vec, const float* dY,
                                 const float* demb, float* fe, float* vir_part, hipStream_t s) {
  GLAUNCH(k_gen_edge_force, nblk(E), a, E, vec, dY, demb, fe, vir_part);
  return hipGetLastError();
}
hipError_t launch_gen_gate_fwd(int n, const GenGateArgs& g, const float* y, float* x, hipStream_t s) {
  GLAUNCH(k_gen_gate_fwd, nblk(n), n, g, y, x);
  return hipGetLastError();
}
hipError_t launch_gen_gate_bwd(int n, const GenGateArgs& g, const float* y, const float* dx, float* dy,
                               hipStream_t s) {
  GLAUNCH(k_gen_gate_bwd, nblk(n), n, g, y, dx, dy);
  return hipGetLastError();
}
hipError_t launch_gen_species_linear(int n, int din, int dout, const int* type, const float* x,
                                     const float* W, float* y, int beta, hipStream_t s) {
  GLAUNCH(k_gen_species_linear, nblk((int64_t)n * dout), n, din, dout, type, x, W, y, beta);
  return hipGetLastError();
}
hipError_t launch_gen_readout(int n, int d, const float* x, const float* v, const int* type,
                              const float* scale, const float* shift, int per_species, float* eat,
                              float* dx, hipStream_t s) {
  GLAUNCH(k_gen_readout, nblk(n), n, d, x, v, type, scale, shift, per_species, eat, dx);
  return hipGetLastError();
}
hipError_t launch_gen_bias(int64_t n, int d, const float* b, float* y, hipStream_t s) {
  GLAUNCH(k_gen_bias, nblk(n * d), n, d, b, y);
  return hipGetLastError();
}
hipError_t launch_gen_fcn_act(int64_t n, int kind, float c, int mode, const float* z, const float* gin,
                              float* out, hipStream_t s) {
  GLAUNCH(k_gen_fcn_act, nblk(n), n, kind, c, mode, z, gin, out);
  return hipGetLastError();
}
hipError_t launch_gen_add(int64_t n, const float* a, float* acc, hipStream_t s) {
  GLAUNCH(k_gen_add, nblk(n), n, a, acc);
  return hipGetLastError();
}

}  // namespace e3gnn
