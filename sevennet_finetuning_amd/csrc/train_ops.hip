// Element-wise kernels of the fine-tune step's autograd graph
// (sevennet_finetuning_amd/nn.py): the scaled SiLU of the radial MLP and the
// gates (e3nn normalize2mom(silu) = 1.6792 * silu) and
// its first and second derivatives, one launch each instead of the 2 / 2-3 /
// ~6 PyTorch kernels the composite op expands to under double backward.
#include "train_ops.h"

namespace e3gnn {
namespace {

__device__ __forceinline__ float sig(float x) { return 1.0f / (1.0f + __expf(-x)); }

// y = c silu(x)
__global__ void k_act_fwd(int64_t n, const float* __restrict__ x, float* __restrict__ y, float c) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = x[i];
  y[i] = c * v * sig(v);
}

// dx = g c silu'(x),  silu'(x) = s (1 + x (1 - s))
__global__ void k_act_bwd(int64_t n, const float* __restrict__ x, const float* __restrict__ g,
                          float* __restrict__ dx, float c) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = x[i], s = sig(v);
  dx[i] = g[i] * c * s * (1.0f + v * (1.0f - s));
}

// cotangent gg of dx:  d/dx = gg g c silu''(x),  d/dg = gg c silu'(x),
// silu''(x) = s (1 - s) (2 + x (1 - 2 s))
__global__ void k_act_bwd2(int64_t n, const float* __restrict__ x, const float* __restrict__ g,
                           const float* __restrict__ gg, float* __restrict__ dx,
                           float* __restrict__ dg, float c) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = x[i], s = sig(v), a = gg[i] * c;
  if (dx) dx[i] = a * g[i] * s * (1.0f - s) * (2.0f + v * (1.0f - 2.0f * s));
  if (dg) dg[i] = a * s * (1.0f + v * (1.0f - s));
}

// reverse of the pair (phi(x), phi'(x) x') of the hand-scheduled fine-tune
// derivatives (train_explicit.py): og = g phi'(x) + gd phi''(x) x', ogd = gd phi'(x)
__global__ void k_act_dual(int64_t n, const float* __restrict__ x, const float* __restrict__ xd,
                           const float* __restrict__ g, const float* __restrict__ gd,
                           float* __restrict__ og, float* __restrict__ ogd, float c) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = x[i], s = sig(v);
  const float d1 = c * s * (1.0f + v * (1.0f - s));
  const float d2 = c * s * (1.0f - s) * (2.0f + v * (1.0f - 2.0f * s));
  og[i] = g[i] * d1 + gd[i] * d2 * xd[i];
  ogd[i] = gd[i] * d1;
}

}  // namespace

hipError_t launch_act_dual(int64_t n, const float* x, const float* xd, const float* g,
                           const float* gd, float* og, float* ogd, float c, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_act_dual, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, x, xd, g,
                     gd, og, ogd, c);
  return hipGetLastError();
}

hipError_t launch_act(int op, int64_t n, const float* x, const float* g, const float* gg,
                      float* out0, float* out1, float c, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const dim3 grid((unsigned)((n + 255) / 256)), block(256);
  switch (op) {
    case 0: hipLaunchKernelGGL(k_act_fwd, grid, block, 0, s, n, x, out0, c); break;
    case 1: hipLaunchKernelGGL(k_act_bwd, grid, block, 0, s, n, x, g, out0, c); break;
    default: hipLaunchKernelGGL(k_act_bwd2, grid, block, 0, s, n, x, g, gg, out0, out1, c); break;
  }
  return hipGetLastError();
}

}  // namespace e3gnn

// ------------------------------------------------------------------ gate
// e3nn Gate of the trainable model (equivariant_gate.py:13-61): input row
// y = [s (NS) | g (NG) | gated blocks (mul_k x (2l_k+1))], output row
// o = [act(s) | act(g_k) * block_k].  One thread per (row, scalar-or-gate
// channel); a gate thread owns its block's 2l+1 components.  Gated blocks are
// described by per-gate (offset, width): blocks follow the gates in order.
namespace e3gnn {
namespace {

struct GateDims {
  int ns, ng, din, dout;   // scalars, gates, input row, output row
  int goff_in[2], goff_out[2], gmul[2], gdim[2], ngrp;   // up to 2 gated irreps
};

__device__ __forceinline__ void act3(float x, float c, float& y, float& d1, float& d2) {
  const float s = 1.0f / (1.0f + __expf(-x));
  y = c * x * s;
  d1 = c * s * (1.0f + x * (1.0f - s));
  d2 = c * s * (1.0f - s) * (2.0f + x * (1.0f - 2.0f * s));
}

// gate thread t in [0, ng) -> group, index within group
__device__ __forceinline__ void gate_of(const GateDims& D, int t, int& grp, int& k) {
  grp = t < D.gmul[0] ? 0 : 1;
  k = grp == 0 ? t : t - D.gmul[0];
}

__global__ void k_gate_fwd(int64_t n, GateDims D, const float* __restrict__ y,
                           float* __restrict__ o, float c) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int per = D.ns + D.ng;
  if (tid >= n * per) return;
  const int64_t r = tid / per;
  const int t = (int)(tid - r * per);
  const float* yr = y + r * D.din;
  float* orow = o + r * D.dout;
  float a, d1, d2;
  if (t < D.ns) {
    act3(yr[t], c, a, d1, d2);
    orow[t] = a;
    return;
  }
  int grp, k;
  gate_of(D, t - D.ns, grp, k);
  act3(yr[D.ns + t - D.ns], c, a, d1, d2);
  const int w = D.gdim[grp];
  for (int m = 0; m < w; ++m)
    orow[D.goff_out[grp] + k * w + m] = a * yr[D.goff_in[grp] + k * w + m];
}

// dy from go
__global__ void k_gate_bwd(int64_t n, GateDims D, const float* __restrict__ y,
                           const float* __restrict__ go, float* __restrict__ dy, float c) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int per = D.ns + D.ng;
  if (tid >= n * per) return;
  const int64_t r = tid / per;
  const int t = (int)(tid - r * per);
  const float* yr = y + r * D.din;
  const float* gr = go + r * D.dout;
  float* dr = dy + r * D.din;
  float a, d1, d2;
  if (t < D.ns) {
    act3(yr[t], c, a, d1, d2);
    dr[t] = gr[t] * d1;
    return;
  }
  int grp, k;
  gate_of(D, t - D.ns, grp, k);
  act3(yr[t], c, a, d1, d2);
  const int w = D.gdim[grp];
  float sg = 0.f;
  for (int m = 0; m < w; ++m) {
    const int ii = D.goff_in[grp] + k * w + m, oo = D.goff_out[grp] + k * w + m;
    sg = fmaf(gr[oo], yr[ii], sg);
    dr[ii] = gr[oo] * a;
  }
  dr[t] = sg * d1;
}

// cotangent q of dy: dgo (nullable) and dyy (nullable)
__global__ void k_gate_bwd2(int64_t n, GateDims D, const float* __restrict__ y,
                            const float* __restrict__ go, const float* __restrict__ q,
                            float* __restrict__ dgo, float* __restrict__ dyy, float c) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int per = D.ns + D.ng;
  if (tid >= n * per) return;
  const int64_t r = tid / per;
  const int t = (int)(tid - r * per);
  const float* yr = y + r * D.din;
  const float* gr = go + r * D.dout;
  const float* qr = q + r * D.din;
  float a, d1, d2;
  if (t < D.ns) {
    act3(yr[t], c, a, d1, d2);
    if (dgo) dgo[r * D.dout + t] = qr[t] * d1;
    if (dyy) dyy[r * D.din + t] = qr[t] * gr[t] * d2;
    return;
  }
  int grp, k;
  gate_of(D, t - D.ns, grp, k);
  act3(yr[t], c, a, d1, d2);
  const int w = D.gdim[grp];
  const float qg = qr[t];
  float sgb = 0.f, sqb = 0.f;   // sum_m go*blk, sum_m q_blk*go
  for (int m = 0; m < w; ++m) {
    const int ii = D.goff_in[grp] + k * w + m, oo = D.goff_out[grp] + k * w + m;
    const float b = yr[ii], g = gr[oo], qb = qr[ii];
    if (dgo) dgo[r * D.dout + oo] = qg * b * d1 + qb * a;
    if (dyy) dyy[r * D.din + ii] = qg * g * d1;
    sgb = fmaf(g, b, sgb);
    sqb = fmaf(qb, g, sqb);
  }
  if (dyy) dyy[r * D.din + t] = qg * sgb * d2 + sqb * d1;
}

// tangent (JVP) of the gate: o' = J(y) y'
__global__ void k_gate_jvp(int64_t n, GateDims D, const float* __restrict__ y,
                           const float* __restrict__ yd, float* __restrict__ od, float c) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int per = D.ns + D.ng;
  if (tid >= n * per) return;
  const int64_t r = tid / per;
  const int t = (int)(tid - r * per);
  const float* yr = y + r * D.din;
  const float* ydr = yd + r * D.din;
  float* orow = od + r * D.dout;
  float a, d1, d2;
  act3(yr[t], c, a, d1, d2);
  if (t < D.ns) {
    orow[t] = d1 * ydr[t];
    return;
  }
  int grp, k;
  gate_of(D, t - D.ns, grp, k);
  const float gd = d1 * ydr[t];
  const int w = D.gdim[grp];
  for (int m = 0; m < w; ++m) {
    const int ii = D.goff_in[grp] + k * w + m, oo = D.goff_out[grp] + k * w + m;
    orow[oo] = gd * yr[ii] + a * ydr[ii];
  }
}

// reverse of (o, o') = (G(y), J(y) y') for the output cotangents (xb, xdb):
// yb = J^T xb + d/dy <xdb, J(y) y'>,  ydb = J^T xdb
__global__ void k_gate_dual(int64_t n, GateDims D, const float* __restrict__ y,
                            const float* __restrict__ yd, const float* __restrict__ xb,
                            const float* __restrict__ xdb, float* __restrict__ yb,
                            float* __restrict__ ydb, float c) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int per = D.ns + D.ng;
  if (tid >= n * per) return;
  const int64_t r = tid / per;
  const int t = (int)(tid - r * per);
  const float* yr = y + r * D.din;
  const float* ydr = yd + r * D.din;
  const float* xr = xb + r * D.dout;
  const float* xdr = xdb + r * D.dout;
  float* br = yb + r * D.din;
  float* bdr = ydb + r * D.din;
  float a, d1, d2;
  act3(yr[t], c, a, d1, d2);
  if (t < D.ns) {
    br[t] = xr[t] * d1 + xdr[t] * d2 * ydr[t];
    bdr[t] = xdr[t] * d1;
    return;
  }
  int grp, k;
  gate_of(D, t - D.ns, grp, k);
  const float gdot = ydr[t];
  const int w = D.gdim[grp];
  float sxb = 0.f, sxdb = 0.f, sxdbd = 0.f;
  for (int m = 0; m < w; ++m) {
    const int ii = D.goff_in[grp] + k * w + m, oo = D.goff_out[grp] + k * w + m;
    const float b = yr[ii], bd = ydr[ii], x0 = xr[oo], x1 = xdr[oo];
    sxb = fmaf(x0, b, sxb);
    sxdb = fmaf(x1, b, sxdb);
    sxdbd = fmaf(x1, bd, sxdbd);
    br[ii] = a * x0 + x1 * d1 * gdot;
    bdr[ii] = a * x1;
  }
  br[t] = d1 * sxb + d2 * gdot * sxdb + d1 * sxdbd;
  bdr[t] = d1 * sxdb;
}

}  // namespace

hipError_t launch_gate_dual(int op, int64_t n, const int* dims, const float* y, const float* yd,
                            const float* xb, const float* xdb, float* out0, float* out1, float c,
                            hipStream_t s) {
  GateDims D{};
  D.ns = dims[0];
  D.ng = dims[1];
  D.din = dims[2];
  D.dout = dims[3];
  D.ngrp = dims[4];
  for (int g = 0; g < 2; ++g) {
    D.goff_in[g] = dims[5 + 4 * g];
    D.goff_out[g] = dims[6 + 4 * g];
    D.gmul[g] = dims[7 + 4 * g];
    D.gdim[g] = dims[8 + 4 * g];
  }
  const int64_t total = n * (D.ns + D.ng);
  if (total <= 0) return hipSuccess;
  const dim3 grid((unsigned)((total + 255) / 256)), block(256);
  if (op == 0)
    hipLaunchKernelGGL(k_gate_jvp, grid, block, 0, s, n, D, y, yd, out0, c);
  else
    hipLaunchKernelGGL(k_gate_dual, grid, block, 0, s, n, D, y, yd, xb, xdb, out0, out1, c);
  return hipGetLastError();
}

hipError_t launch_gate(int op, int64_t n, const int* dims, const float* y, const float* go,
                       const float* q, float* out0, float* out1, float c, hipStream_t s) {
  GateDims D{};
  D.ns = dims[0];
  D.ng = dims[1];
  D.din = dims[2];
  D.dout = dims[3];
  D.ngrp = dims[4];
  for (int g = 0; g < 2; ++g) {
    D.goff_in[g] = dims[5 + 4 * g];
    D.goff_out[g] = dims[6 + 4 * g];
    D.gmul[g] = dims[7 + 4 * g];
    D.gdim[g] = dims[8 + 4 * g];
  }
  const int64_t total = n * (D.ns + D.ng);
  if (total <= 0) return hipSuccess;
  const dim3 grid((unsigned)((total + 255) / 256)), block(256);
  switch (op) {
    case 0: hipLaunchKernelGGL(k_gate_fwd, grid, block, 0, s, n, D, y, out0, c); break;
    case 1: hipLaunchKernelGGL(k_gate_bwd, grid, block, 0, s, n, D, y, go, out0, c); break;
    default: hipLaunchKernelGGL(k_gate_bwd2, grid, block, 0, s, n, D, y, go, q, out0, out1, c); break;
  }
  return hipGetLastError();
}

}  // namespace e3gnn

// ------------------------------------------------------------------ loss
// The explicit fine-tune step's loss (train.py LossDefinition: loss.py:8-206)
// and its cotangents in one launch: block 0 the per-atom energy term, block 1
// the force term, block 2 the stress term (kbar); criterion 0 MSELoss, 1
// HuberLoss(delta), mean over the labelled entries (NaN labels excluded, the
// reference's delete_unlabled); every sum a fixed-order tree (deterministic).
namespace e3gnn {
namespace {

__device__ __forceinline__ float crit(int c, float delta, float x, float* g) {
  if (c == 0) {
    *g = 2.f * x;
    return x * x;
  }
  const float a = fabsf(x);
  if (a < delta) {
    *g = x;
    return 0.5f * x * x;
  }
  *g = x > 0.f ? delta : -delta;
  return delta * (a - 0.5f * delta);
}

__device__ __forceinline__ float block_sum(float v, float* red) {
  const int t = threadIdx.x;
  red[t] = v;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (t < s) red[t] += red[t + s];
    __syncthreads();
  }
  const float r = red[0];
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(256) void k_loss_efs(LossArgs a) {
  __shared__ float red[256];
  const int term = blockIdx.x;
  const int64_t cnt_all = term == 0 ? a.nb : (term == 1 ? 3LL * a.n : 6LL * a.nb);
  const float* pred = term == 0 ? a.e_pred : (term == 1 ? a.f_pred : a.s_pred);
  const float* ref = term == 0 ? a.e_ref : (term == 1 ? a.f_ref : a.s_ref);
  float* cot = term == 0 ? a.ce : (term == 1 ? a.cf : a.cs);
  const float w = term == 0 ? a.w_e : (term == 1 ? a.w_f : a.w_s);
  if (!pred) {   // no stress term
    if (threadIdx.x == 0) a.terms[term] = 0.f;
    return;
  }
  auto x_of = [&](int64_t i, bool* ok) {
    const float r = ref[i];
    *ok = !(r != r);
    float x = pred[i] - (*ok ? r : 0.f);
    if (term == 0) x /= (float)a.natoms[i];
    if (term == 2) x *= a.s_scale;
    return x;
  };
  float s = 0.f, c = 0.f;
  for (int64_t i = threadIdx.x; i < cnt_all; i += 256) {
    bool ok;
    const float x = x_of(i, &ok);
    float g;
    if (ok) {
      s += crit(a.criterion, a.delta, x, &g);
      c += 1.f;
    }
  }
  const float sum = block_sum(s, red), cnt = block_sum(c, red);
  const float inv = cnt > 0.f ? w / cnt : 0.f;
  if (threadIdx.x == 0) a.terms[term] = sum * inv;
  for (int64_t i = threadIdx.x; i < cnt_all; i += 256) {
    bool ok;
    const float x = x_of(i, &ok);
    float g = 0.f;
    if (ok) crit(a.criterion, a.delta, x, &g);
    float v = ok ? g * inv : 0.f;
    if (term == 0) v /= (float)a.natoms[i];
    if (term == 2) v *= a.s_scale;
    cot[i] = v;
  }
}

// EWC over the flat parameters (train.py _FlatEWC, loss.py:209-252):
// part[i] = f (theta - o)^2 (summed by launch_sum), grad[i] += lam f_train (theta - o)
__global__ void k_ewc_flat(int64_t n, const float* __restrict__ th, const float* __restrict__ f,
                           const float* __restrict__ o, const float* __restrict__ ft, float lam,
                           float* __restrict__ grad, float* __restrict__ part) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float d = th[i] - o[i];
  part[i] = f[i] * d * d;
  if (grad) grad[i] += lam * ft[i] * d;
}

}  // namespace

hipError_t launch_loss_efs(const LossArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_loss_efs, dim3(3), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_ewc_flat(int64_t n, const float* th, const float* f, const float* o, const float* ft,
                           float lam, float* grad, float* part, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_ewc_flat, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, th, f, o, ft, lam,
                     grad, part);
  return hipGetLastError();
}

}  // namespace e3gnn
