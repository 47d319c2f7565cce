// Generic nequip-family engine (host side): every E3_equivariant_model
// deployment that is not SevenNet-0's architecture, on the runtime-path-table
// convolution (gtp.hip), the grouped f32 GEMM (gemm.hip k_gemm) and the
// row/edge kernels of generic.hip -- the forward of model_build.py:186-445 and
// its reverse-mode pass written out (ForceStressOutput, force_output.py:74-130).
//
// Layout and arithmetic follow the trainable model of the same family
// (nn.SevenNetTrainable), which the tests pin to the fp64 oracle
// (oracle/nequip_ref.py) and to the reference's own HfO2 deployment:
//   * irreps as written in the manifest (mul, l, parity), e3nn mul-major rows;
//   * e3nn Linear / FullyConnectedTensorProduct(x, one-hot) as DENSE matrices
//     built once at load (the block-sparse weight scattered with its path
//     normalisation; the convolution denominator folded into si2);
//   * the convolution's instruction list and (l, p)-sorted mid irreps
//     (convolution.py:72-95), the gate's sorted input row (equivariant_gate.py).
// Segment semantics (e3gnn.h): a layer's forward runs in part 1 (after the
// halo of x[t] has arrived), its backward in part 0 (before the reverse halo of
// dE/dx[t] leaves); the generic engine does not split a layer for overlap.
#include "generic.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <set>
#include <sstream>
#include <stdexcept>
#include <string>
#include <tuple>

#include "../../include/e3gnn.h"
#include "common.h"
#include "dbuf.h"
#include "gtp.h"
#include "minijson.h"
#include "node.h"

namespace e3gnn {

const GtpTables* gtp_tables(const e3gnn_gtp* g);  // api.cpp

namespace {

struct GIrr {
  int mul, l, p;  // p: +1 even, -1 odd
};
using GIrreps = std::vector<GIrr>;

GIrreps parse_gir(const std::string& s) {
  GIrreps out;
  std::stringstream ss(s);
  std::string term;
  while (std::getline(ss, term, '+')) {
    const auto x = term.find('x');
    if (x == std::string::npos || term.size() < x + 3) throw std::runtime_error("bad irreps " + s);
    const char par = term.back();
    if (par != 'e' && par != 'o') throw std::runtime_error("bad irreps parity in " + s);
    out.push_back({std::stoi(term.substr(0, x)), std::stoi(term.substr(x + 1, term.size() - x - 2)),
                   par == 'e' ? 1 : -1});
  }
  return out;
}
int gdim(const GIrreps& ir) {
  int d = 0;
  for (auto& i : ir) d += i.mul * (2 * i.l + 1);
  return d;
}
std::vector<int> goffsets(const GIrreps& ir) {
  std::vector<int> o(1, 0);
  for (auto& i : ir) o.push_back(o.back() + i.mul * (2 * i.l + 1));
  return o;
}
bool same_ir(const GIrr& a, const GIrr& b) { return a.l == b.l && a.p == b.p; }

// e3nn o3.Linear (sevenn/nn/linear.py:46-49) as a dense (din x dout) matrix:
// blocks (i_in, i_out) of equal irrep, i_in-major, W[u][v] row-major, path
// weight 1/sqrt(fan-in of i_out), times `extra`
std::vector<float> dense_linear(const GIrreps& in, const GIrreps& out, const float* w, size_t numel,
                                double extra) {
  const auto io = goffsets(in), oo = goffsets(out);
  const int din = io.back(), dout = oo.back();
  std::map<int, int> fan;
  size_t need = 0;
  for (size_t i = 0; i < in.size(); ++i)
    for (size_t j = 0; j < out.size(); ++j)
      if (same_ir(in[i], out[j])) {
        fan[(int)j] += in[i].mul;
        need += (size_t)in[i].mul * out[j].mul;
      }
  if (need != numel) throw std::runtime_error("linear weight size mismatch");
  std::vector<float> W((size_t)din * dout, 0.f);
  size_t off = 0;
  for (size_t i = 0; i < in.size(); ++i)
    for (size_t j = 0; j < out.size(); ++j) {
      if (!same_ir(in[i], out[j])) continue;
      const int mi = in[i].mul, mo = out[j].mul, d = 2 * in[i].l + 1;
      const double a = extra / std::sqrt((double)fan[(int)j]);
      for (int u = 0; u < mi; ++u)
        for (int v = 0; v < mo; ++v)
          for (int m = 0; m < d; ++m)
            W[(size_t)(io[i] + u * d + m) * dout + oo[j] + v * d + m] = (float)(w[off + (size_t)u * mo + v] * a);
      off += (size_t)mi * mo;
    }
  return W;
}
std::vector<float> transpose(const std::vector<float>& a, int r, int c) {
  std::vector<float> t(a.size());
  for (int i = 0; i < r; ++i)
    for (int j = 0; j < c; ++j) t[(size_t)j * r + i] = a[(size_t)i * c + j];
  return t;
}

struct GLin {
  int din = 0, dout = 0;
  DBuf W, WT;
};
// e3nn o3.Linear(biases=True) (use_bias_in_linear): the bias over the full
// output row -- b on the channels of every 0e output irrep, in output order,
// zero elsewhere
std::vector<float> bias_row(const GIrreps& out, const float* b, size_t numel) {
  const auto oo = goffsets(out);
  std::vector<float> v(oo.back(), 0.f);
  size_t k = 0;
  for (size_t j = 0; j < out.size(); ++j)
    if (out[j].l == 0 && out[j].p == 1)
      for (int u = 0; u < out[j].mul; ++u) {
        if (k >= numel) throw std::runtime_error("linear bias size mismatch");
        v[oo[j] + u] = b[k++];
      }
  if (k != numel) throw std::runtime_error("linear bias size mismatch");
  return v;
}
void make_lin(GLin& L, const std::vector<float>& W, int din, int dout) {
  L.din = din;
  L.dout = dout;
  if (upload(L.W, W) != hipSuccess || upload(L.WT, transpose(W, din, dout)) != hipSuccess)
    throw std::runtime_error("upload (linear)");
}

hipError_t gemm(const float* A, int64_t lda, const float* B, int ldb, float* C, int64_t ldc, int64_t M,
                int K, int N, int act, const float* pre_in, float* pre_out, int beta, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0) return hipSuccess;
  if (M > (1LL << 31) - 64) return hipErrorInvalidValue;
  GemmBatch b;
  std::memset(&b, 0, sizeof(b));
  GemmProb& p = b.p[0];
  p.A = A;
  p.B = B;
  p.C = C;
  p.pre_in = pre_in;
  p.pre_out = pre_out;
  p.lda = lda;
  p.ldc = ldc;
  p.M = (int)M;
  p.N = N;
  p.K = K;
  p.R = 1;
  p.ldb = ldb;
  p.beta = beta;
  p.act = act;
  p.tiles_n = (N + 63) / 64;
  p.tile_begin = 0;
  b.nprob = 1;
  b.total_tiles = (int)((M + 63) / 64) * p.tiles_n;
  return launch_gemm(b, s);
}

#define GCHK(expr)                          \
  do {                                      \
    hipError_t _e = (expr);                 \
    if (_e != hipSuccess) return _e;        \
  } while (0)

}  // namespace

struct GenLayer {
  int dx = 0, dg = 0, dm = 0, dout = 0, W = 0;
  GLin si1, si2, sc;           // sc: the `linear` self-connection
  bool sc_species = false;     // `nequip`: one dense matrix per species
  DBuf scs, scsT;              // [nsp][dx][dg], [nsp][dg][dx]
  std::vector<int> width;      // radial MLP widths: nb, hidden..., W
  std::vector<GLin> mlp;       // layer k: [width k] x [width k + 1], / sqrt(fan_in)
  e3gnn_gtp* gtp = nullptr;
  DBuf gate_cols;
  GenGateArgs gate{};
  DBuf b1, b2;                 // si1 / si2 biases (full rows; empty without biases)
};

struct GenModel {
  int nsp = 0, nlayer = 0, ny = 0, nb = 0, d0 = 0, per_species = 1;
  float cutoff = 0.f;
  GenEdgeArgs edge{};
  DBuf coeffs, embed, readout_v, scale, shift;
  std::vector<int> dims;  // x[t] dims, t = 0..L
  std::vector<GenLayer> L;
  // readout_as_fcn (FCN_e3nn): widths dims[L], hidden..., 1; layer k's
  // weight / sqrt(fan_in); activation kind / normalize2mom constant
  bool fcn = false;
  std::vector<int> fcn_w;
  std::vector<GLin> fcn_l;
  int fcn_kind = 0;
  float fcn_c = 1.f;
  DBuf one;
  ~GenModel() {
    for (auto& l : L)
      if (l.gtp) e3gnn_gtp_free(l.gtp);
  }
};

struct GenCtx {
  int64_t n = 0, nl = 0, E = 0;
  std::vector<DBuf> x, grad, h, y, w;
  std::vector<std::vector<DBuf>> pre, act;  // radial MLP hidden layers per block
  std::vector<DBuf> fz, fa;                   // readout FCN pre-activations / activations
  DBuf fes, fgs, fg0, fg1;                    // its output, dE/d(output), backward rows
  DBuf Y, emb, agg, dagg, dy, dh, dxc, dw, dYt, dA0, dA1, dYacc, demb, fe, vpart, eat, part, scratch;
};

GenModel* gen_load(const minijson::Value& man, const std::vector<float>& flat) {
  auto m = std::make_unique<GenModel>();
  std::map<std::string, std::pair<size_t, size_t>> T;
  for (auto& t : man["tensors"].arr())
    T[t["name"].str()] = {(size_t)t["offset"].num(), (size_t)t["numel"].num()};
  auto get = [&](const std::string& n) -> std::pair<const float*, size_t> {
    auto it = T.find(n);
    if (it == T.end()) throw std::runtime_error("missing tensor " + n);
    if (it->second.first + it->second.second > flat.size())
      throw std::runtime_error("tensor out of file range " + n);
    return {flat.data() + it->second.first, it->second.second};
  };
  m->nsp = (int)man["num_species"].num();
  m->cutoff = (float)man["cutoff"].num();
  m->nlayer = (int)man["num_convolution_layer"].num();
  const int L = m->nlayer;
  if (std::abs(man["silu_norm"].num() - (double)SILU_NORM) > 1e-6)
    throw std::runtime_error("silu_norm differs from the kernels' normalisation constant");
  const float tanh_norm = man.has("act_norm") && man["act_norm"].has("tanh")
                              ? (float)man["act_norm"]["tanh"].num()
                              : 1.f;
  if (man.has("act_radial") && man["act_radial"].str() != "silu")
    throw std::runtime_error("radial MLP activation must be silu");
  // edge embedding
  const auto& cf = man["cutoff_function"];
  GenEdgeArgs ea{};
  ea.rc = m->cutoff;
  if (cf["name"].str() == "XPLOR") {
    ea.cut = 0;
    ea.ron = (float)cf["cutoff_on"].num();
  } else if (cf["name"].str() == "poly_cut") {
    ea.cut = 1;
    ea.p = (float)cf["p"].num();
  } else {
    throw std::runtime_error("cutoff function " + cf["name"].str() + " is not implemented");
  }
  const int lmax = man.has("lmax_edge") ? (int)man["lmax_edge"].num()
                                        : (man.has("lmax") ? (int)man["lmax"].num() : 2);
  if (lmax < 0 || lmax > 2) throw std::runtime_error("lmax_edge must be <= 2");
  ea.lmax = lmax;
  ea.normalize = man.has("sh_normalize") ? (man["sh_normalize"].boolean() ? 1 : 0) : 1;
  m->ny = (lmax + 1) * (lmax + 1);
  {
    auto c = get("edge_embedding.basis_function.coeffs");
    m->nb = (int)c.second;
    if (upload(m->coeffs, std::vector<float>(c.first, c.first + c.second)) != hipSuccess)
      throw std::runtime_error("upload");
  }
  ea.nb = m->nb;
  ea.coeffs = m->coeffs.f();
  m->edge = ea;
  const int fpar = man.has("is_parity") && man["is_parity"].boolean() ? -1 : 1;
  const std::string sc_type =
      man.has("self_connection_type") ? man["self_connection_type"].str() : std::string("linear");
  if (sc_type != "linear" && sc_type != "nequip")
    throw std::runtime_error("self_connection_type " + sc_type + " is not implemented");
  std::vector<GIrreps> irr;
  for (auto& s : man["irreps_manual"].arr()) irr.push_back(parse_gir(s.str()));
  if ((int)irr.size() != L + 1) throw std::runtime_error("irreps_manual length");
  std::vector<GIrreps> conv_out;
  if (man.has("conv_irreps_out"))
    for (auto& s : man["conv_irreps_out"].arr()) conv_out.push_back(parse_gir(s.str()));
  else
    conv_out.assign(irr.begin() + 1, irr.end());
  if ((int)conv_out.size() != L) throw std::runtime_error("conv_irreps_out length");
  for (auto& ir : irr) m->dims.push_back(gdim(ir));
  // node embedding: 'mul x 0e' from the one-hot species
  if (irr[0].size() != 1 || irr[0][0].l != 0 || irr[0][0].p != 1)
    throw std::runtime_error("layer-0 features must be one even scalar irrep");
  m->d0 = m->dims[0];
  {
    auto we = get("onehot_to_feature_x.linear.weight");
    if (we.second != (size_t)m->nsp * m->d0) throw std::runtime_error("bad size onehot_to_feature_x");
    std::vector<float> e(we.second);
    for (size_t i = 0; i < e.size(); ++i) e[i] = (float)(we.first[i] / std::sqrt((double)m->nsp));
    // the embedding's bias (use_bias_in_linear): the same for every species row
    if (T.count("onehot_to_feature_x.linear.bias")) {
      auto b = get("onehot_to_feature_x.linear.bias");
      const auto row = bias_row(irr[0], b.first, b.second);
      for (int sp = 0; sp < m->nsp; ++sp)
        for (int c = 0; c < m->d0; ++c) e[(size_t)sp * m->d0 + c] += row[c];
    }
    if (upload(m->embed, e) != hipSuccess) throw std::runtime_error("upload");
  }
  std::vector<int> hidden;
  if (man.has("weight_nn_hidden_neurons"))
    for (auto& v : man["weight_nn_hidden_neurons"].arr()) hidden.push_back((int)v.num());
  else
    hidden = {64, 64};
  m->L.resize(L);
  for (int t = 0; t < L; ++t) {
    GenLayer& G = m->L[t];
    const GIrreps& xi = irr[t];
    const GIrreps& xo = irr[t + 1];
    const std::string p = std::to_string(t);
    // ---- gate (equivariant_gate.py:30-61): [scalars | gates | gated], stably
    // (l, p)-sorted (odd first) and merged = the linears' output irreps
    GIrreps scal, gated;
    for (auto& i : xo) (i.l == 0 ? scal : gated).push_back(i);
    int ng = 0;
    for (auto& i : gated) ng += i.mul;
    int gate_p = -1;
    for (auto& i : scal)
      if (i.p == 1) gate_p = 1;
    GIrreps pieces = scal;
    if (ng) pieces.push_back({ng, 0, gate_p});
    pieces.insert(pieces.end(), gated.begin(), gated.end());
    std::vector<int> order(pieces.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = (int)i;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
      return std::make_pair(pieces[a].l, pieces[a].p) < std::make_pair(pieces[b].l, pieces[b].p);
    });
    std::vector<int> offs(pieces.size());
    GIrreps gin;
    {
      int off = 0;
      for (int i : order) {
        offs[i] = off;
        off += pieces[i].mul * (2 * pieces[i].l + 1);
        if (!gin.empty() && same_ir(gin.back(), pieces[i])) gin.back().mul += pieces[i].mul;
        else gin.push_back(pieces[i]);
      }
    }
    // the gate's output is [scalars..., gated...]: it must be irreps_manual[t+1]
    {
      GIrreps cat = scal;
      cat.insert(cat.end(), gated.begin(), gated.end());
      bool same = cat.size() == xo.size();
      for (size_t i = 0; same && i < cat.size(); ++i)
        same = cat[i].mul == xo[i].mul && same_ir(cat[i], xo[i]);
      if (!same) throw std::runtime_error("layer " + p + ": output irreps must list the scalars first");
    }
    std::vector<GenGateCol> cols;
    for (size_t k = 0; k < scal.size(); ++k)
      for (int u = 0; u < scal[k].mul; ++u) cols.push_back({offs[k] + u, -1, scal[k].p == 1 ? 0 : 1});
    {
      int gbase = 0;
      for (size_t k = 0; k < gated.size(); ++k) {
        const int pi = (int)(scal.size() + 1 + k), d = 2 * gated[k].l + 1;
        for (int u = 0; u < gated[k].mul; ++u)
          for (int mm = 0; mm < d; ++mm)
            cols.push_back({offs[pi] + u * d + mm, offs[scal.size()] + gbase + u, gate_p == 1 ? 0 : 1});
        gbase += gated[k].mul;
      }
    }
    G.dx = gdim(xi);
    G.dg = gdim(gin);
    G.dout = gdim(xo);
    if ((int)cols.size() != G.dout) throw std::runtime_error("gate column table");
    {
      std::vector<float> buf(cols.size() * 3);
      std::memcpy(buf.data(), cols.data(), cols.size() * sizeof(GenGateCol));
      if (upload(G.gate_cols, buf) != hipSuccess) throw std::runtime_error("upload");
    }
    G.gate = {G.dg, G.dout, tanh_norm, static_cast<const GenGateCol*>(G.gate_cols.p)};
    // ---- convolution instructions (convolution.py:72-95) and path table
    std::set<std::pair<int, int>> allowed;
    for (auto& i : conv_out[t]) allowed.insert({i.l, i.p});
    struct Ins {
      int i, l2, l3, p3, mul;
    };
    std::vector<Ins> ins;
    for (size_t i = 0; i < xi.size(); ++i)
      for (int l2 = 0; l2 <= lmax; ++l2) {
        const int p3 = xi[i].p * (l2 % 2 ? fpar : 1);
        for (int l3 = std::abs(xi[i].l - l2); l3 <= xi[i].l + l2; ++l3)
          if (allowed.count({l3, p3})) ins.push_back({(int)i, l2, l3, p3, xi[i].mul});
      }
    std::vector<int> ord(ins.size());
    for (size_t k = 0; k < ord.size(); ++k) ord[k] = (int)k;
    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) {
      return std::make_pair(ins[a].l3, ins[a].p3) < std::make_pair(ins[b].l3, ins[b].p3);
    });
    std::vector<int> slot(ins.size());
    GIrreps mid;
    for (size_t s = 0; s < ord.size(); ++s) {
      slot[ord[s]] = (int)s;
      mid.push_back({ins[ord[s]].mul, ins[ord[s]].l3, ins[ord[s]].p3});
    }
    const auto xo_off = goffsets(xi), mo_off = goffsets(mid);
    std::vector<int32_t> rows;
    int woff = 0;
    for (size_t k = 0; k < ins.size(); ++k) {
      const Ins& q = ins[k];
      rows.insert(rows.end(), {xi[q.i].l, q.l2, q.l3, q.mul, xo_off[q.i], q.l2 * q.l2, woff, mo_off[slot[k]]});
      woff += q.mul;
    }
    G.W = woff;
    G.dm = gdim(mid);
    if (ins.empty()) throw std::runtime_error("layer " + p + ": empty convolution");
    G.gtp = e3gnn_gtp_create((int)ins.size(), rows.data(), G.dx, m->ny, G.W, G.dm);
    if (!G.gtp) throw std::runtime_error(std::string("gtp: ") + e3gnn_last_error());
    // ---- linears
    const float den = *get(p + "_convolution.denominator").first;
    {
      auto w = get(p + "_self_interaction_1.linear.weight");
      make_lin(G.si1, dense_linear(xi, xi, w.first, w.second, 1.0), G.dx, G.dx);
      w = get(p + "_self_interaction_2.linear.weight");
      make_lin(G.si2, dense_linear(mid, gin, w.first, w.second, 1.0 / den), G.dm, G.dg);
      if (T.count(p + "_self_interaction_1.linear.bias")) {
        auto b = get(p + "_self_interaction_1.linear.bias");
        if (upload(G.b1, bias_row(xi, b.first, b.second)) != hipSuccess) throw std::runtime_error("upload");
      }
      if (T.count(p + "_self_interaction_2.linear.bias")) {
        auto b = get(p + "_self_interaction_2.linear.bias");
        if (upload(G.b2, bias_row(gin, b.first, b.second)) != hipSuccess) throw std::runtime_error("upload");
      }
    }
    if (sc_type == "linear") {
      auto w = get(p + "_self_connection_intro.linear.weight");
      make_lin(G.sc, dense_linear(xi, gin, w.first, w.second, 1.0), G.dx, G.dg);
    } else {
      // FullyConnectedTensorProduct(x, one-hot) (self_connection.py:11-38):
      // per (i_x, i_out) of equal irrep a (mul_x, nsp, mul_out) block, path
      // weight 1/sqrt(sum of mul_x * nsp into i_out)
      auto w = get(p + "_self_connection_intro.fc_tensor_product.weight");
      const auto io = goffsets(xi), oo = goffsets(gin);
      std::map<int, int> fan;
      size_t need = 0;
      for (size_t i = 0; i < xi.size(); ++i)
        for (size_t j = 0; j < gin.size(); ++j)
          if (same_ir(xi[i], gin[j])) {
            fan[(int)j] += xi[i].mul * m->nsp;
            need += (size_t)xi[i].mul * m->nsp * gin[j].mul;
          }
      if (need != w.second) throw std::runtime_error("self-connection weight size");
      std::vector<float> Ws((size_t)m->nsp * G.dx * G.dg, 0.f), WsT(Ws.size(), 0.f);
      size_t off = 0;
      for (size_t i = 0; i < xi.size(); ++i)
        for (size_t j = 0; j < gin.size(); ++j) {
          if (!same_ir(xi[i], gin[j])) continue;
          const int mi = xi[i].mul, mo = gin[j].mul, d = 2 * xi[i].l + 1;
          const double a = 1.0 / std::sqrt((double)fan[(int)j]);
          for (int u = 0; u < mi; ++u)
            for (int s = 0; s < m->nsp; ++s)
              for (int v = 0; v < mo; ++v)
                for (int mm = 0; mm < d; ++mm) {
                  const float val = (float)(w.first[off + ((size_t)u * m->nsp + s) * mo + v] * a);
                  const size_t r = io[i] + u * d + mm, c = oo[j] + v * d + mm;
                  Ws[((size_t)s * G.dx + r) * G.dg + c] = val;
                  WsT[((size_t)s * G.dg + c) * G.dx + r] = val;
                }
          off += (size_t)mi * m->nsp * mo;
        }
      if (upload(G.scs, Ws) != hipSuccess || upload(G.scsT, WsT) != hipSuccess)
        throw std::runtime_error("upload");
      G.sc_species = true;
    }
    // ---- radial MLP (e3nn FullyConnectedNet: weights / sqrt(fan_in), act between)
    G.width = {m->nb};
    G.width.insert(G.width.end(), hidden.begin(), hidden.end());
    G.width.push_back(G.W);
    G.mlp.resize(G.width.size() - 1);
    for (size_t k = 0; k + 1 < G.width.size(); ++k) {
      auto w = get(p + "_convolution.weight_nn.layer" + std::to_string(k) + ".weight");
      const int a = G.width[k], b = G.width[k + 1];
      if (w.second != (size_t)a * b) throw std::runtime_error("radial MLP layer size " + p);
      std::vector<float> v(w.second);
      for (size_t i = 0; i < v.size(); ++i) v[i] = (float)(w.first[i] / std::sqrt((double)a));
      make_lin(G.mlp[k], v, a, b);
    }
  }
  // ---- readout: two linears without activation = one vector (their biases
  // a constant, folded into the shift); or the FCN readout; rescale
  {
    auto sc = get("rescale_atomic_energy.scale");
    auto sh = get("rescale_atomic_energy.shift");
    if (sc.second != sh.second || (sc.second != 1 && sc.second != (size_t)m->nsp))
      throw std::runtime_error("rescale_atomic_energy: one value or one per species");
    m->per_species = sc.second == 1 ? 0 : 1;
    std::vector<float> shift(sh.first, sh.first + sh.second);
    const int dl = m->dims[L];
    const bool fcn = man.has("readout") && man["readout"].has("type") && man["readout"]["type"].str() == "fcn";
    if (fcn) {
      // FCN_e3nn (nn/linear.py:94-129, model_build.py:396-408)
      for (auto& i : irr[L])
        if (i.l != 0) throw std::runtime_error("readout_as_fcn needs a scalar-only last block");
      const auto& ro = man["readout"];
      static const char* kinds[] = {"relu", "silu", "tanh", "sigmoid", "abs", "elu"};
      m->fcn_kind = -1;
      for (int k = 0; k < 6; ++k)
        if (ro["act"].str() == kinds[k]) m->fcn_kind = k;
      if (m->fcn_kind < 0) throw std::runtime_error("readout activation " + ro["act"].str() + " is not built");
      m->fcn_c = (float)ro["act_norm"].num();
      m->fcn_w = {dl};
      for (auto& h : ro["hidden"].arr()) m->fcn_w.push_back((int)h.num());
      m->fcn_w.push_back(1);
      m->fcn_l.resize(m->fcn_w.size() - 1);
      for (size_t k = 0; k + 1 < m->fcn_w.size(); ++k) {
        auto w = get("readout_FCN.fcn.layer" + std::to_string(k) + ".weight");
        const int a = m->fcn_w[k], b = m->fcn_w[k + 1];
        if (w.second != (size_t)a * b) throw std::runtime_error("readout FCN layer size");
        std::vector<float> v(w.second);
        for (size_t i = 0; i < v.size(); ++i) v[i] = (float)(w.first[i] / std::sqrt((double)a));
        make_lin(m->fcn_l[k], v, a, b);
      }
      m->fcn = true;
      if (upload(m->one, std::vector<float>(1, 1.f)) != hipSuccess) throw std::runtime_error("upload");
    } else {
      const int hid = man.has("readout_hidden") ? (int)man["readout_hidden"].num() : irr[L][0].mul / 2;
      GIrreps hir{{hid, 0, 1}}, one{{1, 0, 1}};
      auto w1 = get("reduce_input_to_hidden.linear.weight");
      auto w2 = get("reduce_hidden_to_energy.linear.weight");
      const auto A = dense_linear(irr[L], hir, w1.first, w1.second, 1.0);
      const auto B = dense_linear(hir, one, w2.first, w2.second, 1.0);
      std::vector<float> v(dl, 0.f);
      for (int c = 0; c < dl; ++c) {
        double s = 0;
        for (int k = 0; k < hid; ++k) s += (double)A[(size_t)c * hid + k] * B[k];
        v[c] = (float)s;
      }
      if (upload(m->readout_v, v) != hipSuccess) throw std::runtime_error("upload");
      // biases: e = (x A + bA) B + bB = x v + (bA . B + bB), per atom before
      // the rescale: shift += (bA . B + bB) scale
      double cst = 0;
      if (T.count("reduce_input_to_hidden.linear.bias")) {
        auto b = get("reduce_input_to_hidden.linear.bias");
        const auto row = bias_row(hir, b.first, b.second);
        for (int k = 0; k < hid; ++k) cst += (double)row[k] * B[k];
      }
      if (T.count("reduce_hidden_to_energy.linear.bias")) cst += *get("reduce_hidden_to_energy.linear.bias").first;
      for (size_t i = 0; i < shift.size(); ++i) shift[i] = (float)(shift[i] + cst * sc.first[i]);
    }
    if (upload(m->scale, std::vector<float>(sc.first, sc.first + sc.second)) != hipSuccess ||
        upload(m->shift, shift) != hipSuccess)
      throw std::runtime_error("upload");
  }
  (void)hipGetLastError();
  return m.release();
}

void gen_free(GenModel* m) { delete m; }
int gen_num_layers(const GenModel* m) { return m->nlayer; }
int gen_num_species(const GenModel* m) { return m->nsp; }
float gen_cutoff(const GenModel* m) { return m->cutoff; }
int gen_feature_dim(const GenModel* m, int layer) { return m->dims[layer]; }

GenCtx* gen_ctx_create(const GenModel* m) {
  auto* c = new GenCtx();
  const int L = m->nlayer;
  c->x.resize(L + 1);
  c->grad.resize(L + 1);
  c->h.resize(L);
  c->y.resize(L);
  c->w.resize(L);
  c->pre.resize(L);
  c->act.resize(L);
  for (int t = 0; t < L; ++t) {
    c->pre[t].resize(m->L[t].width.size() - 2);
    c->act[t].resize(m->L[t].width.size() - 2);
  }
  if (m->fcn) {
    c->fz.resize(m->fcn_w.size() - 2);
    c->fa.resize(m->fcn_w.size() - 2);
  }
  return c;
}
void gen_ctx_free(GenCtx* c) { delete c; }
float* gen_x(GenCtx* c, int layer) { return c->x[layer].f(); }
float* gen_grad(GenCtx* c, int layer) { return c->grad[layer].f(); }

hipError_t gen_graph_set(GenCtx* c, const GenModel* m, const GenGraph& g, hipStream_t s) {
  const size_t F = sizeof(float);
  const int64_t n = g.n, nl = g.nl, E = g.E;
  c->n = n;
  c->nl = nl;
  c->E = E;
  const int L = m->nlayer;
  int maxx = 0, maxg = 0, maxm = 0, maxw = 0, maxh = 1;
  for (int t = 0; t <= L; ++t) {
    GCHK(c->x[t].ensure(std::max<int64_t>(n, 1) * m->dims[t] * F));
    GCHK(c->grad[t].ensure(std::max<int64_t>(n, 1) * m->dims[t] * F));
  }
  for (int t = 0; t < L; ++t) {
    const GenLayer& G = m->L[t];
    maxx = std::max(maxx, G.dx);
    maxg = std::max(maxg, G.dg);
    maxm = std::max(maxm, G.dm);
    maxw = std::max(maxw, G.W);
    GCHK(c->h[t].ensure(std::max<int64_t>(n, 1) * G.dx * F));
    GCHK(c->y[t].ensure(std::max<int64_t>(nl, 1) * G.dg * F));
    GCHK(c->w[t].ensure(std::max<int64_t>(E, 1) * G.W * F));
    for (size_t k = 0; k + 2 < G.width.size(); ++k) {
      maxh = std::max(maxh, G.width[k + 1]);
      GCHK(c->pre[t][k].ensure(std::max<int64_t>(E, 1) * G.width[k + 1] * F));
      GCHK(c->act[t][k].ensure(std::max<int64_t>(E, 1) * G.width[k + 1] * F));
    }
  }
  const int64_t E1 = std::max<int64_t>(E, 1), n1 = std::max<int64_t>(n, 1), nl1 = std::max<int64_t>(nl, 1);
  GCHK(c->Y.ensure(E1 * m->ny * F));
  GCHK(c->emb.ensure(E1 * m->nb * F));
  GCHK(c->agg.ensure(nl1 * maxm * F));
  GCHK(c->dagg.ensure(nl1 * maxm * F));
  GCHK(c->dy.ensure(nl1 * maxg * F));
  GCHK(c->dh.ensure(n1 * maxx * F));
  GCHK(c->dxc.ensure(E1 * maxx * F));
  GCHK(c->dw.ensure(E1 * maxw * F));
  GCHK(c->dYt.ensure(E1 * m->ny * F));
  GCHK(c->dA0.ensure(E1 * maxh * F));
  GCHK(c->dA1.ensure(E1 * maxh * F));
  GCHK(c->dYacc.ensure(E1 * m->ny * F));
  GCHK(c->demb.ensure(E1 * m->nb * F));
  GCHK(c->fe.ensure(E1 * 3 * F));
  GCHK(c->vpart.ensure(((int64_t)gen_edge_force_blocks(E) + 1) * 6 * F));
  GCHK(c->eat.ensure(nl1 * F));
  GCHK(c->part.ensure(((int64_t)sum_blocks(nl) + 1) * F));
  GCHK(c->scratch.ensure(8 * F));
  if (m->fcn) {
    int wmax = 1;
    for (size_t k = 0; k + 2 < m->fcn_w.size(); ++k) {
      GCHK(c->fz[k].ensure(nl1 * m->fcn_w[k + 1] * F));
      GCHK(c->fa[k].ensure(nl1 * m->fcn_w[k + 1] * F));
    }
    for (int w : m->fcn_w) wmax = std::max(wmax, w);
    GCHK(c->fes.ensure(nl1 * F));
    GCHK(c->fgs.ensure(nl1 * F));
    GCHK(c->fg0.ensure(nl1 * wmax * F));
    GCHK(c->fg1.ensure(nl1 * wmax * F));
  }
  GCHK(launch_gen_embed((int)n, m->d0, g.type, m->nsp, m->embed.f(), c->x[0].f(), g.err, s));
  if (E > 0) GCHK(launch_gen_edge_embed(m->edge, E, g.vec, c->Y.f(), c->emb.f(), s));
  return hipSuccess;
}

hipError_t gen_layer_forward(GenCtx* c, const GenModel* m, const GenGraph& g, int t, hipStream_t s) {
  const GenLayer& G = m->L[t];
  const int64_t n = c->n, nl = c->nl, E = c->E;
  // self_interaction_1 on every row (ghost rows are gathered as neighbours)
  GCHK(gemm(c->x[t].f(), G.dx, G.si1.W.f(), G.dx, c->h[t].f(), G.dx, n, G.dx, G.dx, 0, nullptr, nullptr, 0, s));
  if (G.b1.p) GCHK(launch_gen_bias(n, G.dx, G.b1.f(), c->h[t].f(), s));
  // radial MLP: hidden layers keep their pre-activations (the backward's act')
  const float* a = c->emb.f();
  int wa = m->nb;
  const int nh = (int)G.width.size() - 2;
  for (int k = 0; k < nh; ++k) {
    const int wb = G.width[k + 1];
    GCHK(gemm(a, wa, G.mlp[k].W.f(), wb, c->act[t][k].f(), wb, E, wa, wb, 1, nullptr, c->pre[t][k].f(), 0, s));
    a = c->act[t][k].f();
    wa = wb;
  }
  GCHK(gemm(a, wa, G.mlp[nh].W.f(), G.W, c->w[t].f(), G.W, E, wa, G.W, 0, nullptr, nullptr, 0, s));
  // convolution (runtime path tables): raw sum over each owned centre's edges
  if (nl > 0)
    GCHK(launch_gtp_fwd((int)nl, g.row_ptr, g.nbr, c->h[t].f(), c->Y.f(), c->w[t].f(), *gtp_tables(G.gtp),
                        c->agg.f(), s));
  // self_interaction_2 (/ denominator, folded) + self-connection, gate
  GCHK(gemm(c->agg.f(), G.dm, G.si2.W.f(), G.dg, c->y[t].f(), G.dg, nl, G.dm, G.dg, 0, nullptr, nullptr, 0, s));
  if (G.b2.p) GCHK(launch_gen_bias(nl, G.dg, G.b2.f(), c->y[t].f(), s));
  if (G.sc_species)
    GCHK(launch_gen_species_linear((int)nl, G.dx, G.dg, g.type, c->x[t].f(), G.scs.f(), c->y[t].f(), 1, s));
  else
    GCHK(gemm(c->x[t].f(), G.dx, G.sc.W.f(), G.dg, c->y[t].f(), G.dg, nl, G.dx, G.dg, 0, nullptr, nullptr, 1, s));
  GCHK(launch_gen_gate_fwd((int)nl, G.gate, c->y[t].f(), c->x[t + 1].f(), s));
  return hipSuccess;
}

hipError_t gen_readout(GenCtx* c, const GenModel* m, const GenGraph& g, float* energy, float* atomic_energy,
                       hipStream_t s) {
  const int L = m->nlayer;
  const int64_t nl = c->nl;
  if (m->fcn) {
    // FCN_e3nn forward over the owned rows, the rescale, and its backward down
    // to dE/dx[L] (the readout is the only consumer of x[L])
    const int nh = (int)m->fcn_w.size() - 2;
    const float* a = c->x[L].f();
    int wa = m->fcn_w[0];
    for (int k = 0; k < nh; ++k) {
      const int wb = m->fcn_w[k + 1];
      GCHK(gemm(a, wa, m->fcn_l[k].W.f(), wb, c->fz[k].f(), wb, nl, wa, wb, 0, nullptr, nullptr, 0, s));
      GCHK(launch_gen_fcn_act(nl * wb, m->fcn_kind, m->fcn_c, 0, c->fz[k].f(), nullptr, c->fa[k].f(), s));
      a = c->fa[k].f();
      wa = wb;
    }
    GCHK(gemm(a, wa, m->fcn_l[nh].W.f(), 1, c->fes.f(), 1, nl, wa, 1, 0, nullptr, nullptr, 0, s));
    GCHK(launch_gen_readout((int)nl, 1, c->fes.f(), m->one.f(), g.type, m->scale.f(), m->shift.f(),
                            m->per_species, c->eat.f(), c->fgs.f(), s));
    // dE/da_nh = g W_nh^T (K = 1); then dz = da c f'(z), da_k = dz W_k^T
    float* bufs[2] = {c->fg0.f(), c->fg1.f()};
    float* cur = nh == 0 ? c->grad[L].f() : bufs[0];
    GCHK(gemm(c->fgs.f(), 1, m->fcn_l[nh].WT.f(), wa, cur, wa, nl, 1, wa, 0, nullptr, nullptr, 0, s));
    for (int k = nh - 1; k >= 0; --k) {
      const int wb = m->fcn_w[k + 1], wk = m->fcn_w[k];
      GCHK(launch_gen_fcn_act(nl * wb, m->fcn_kind, m->fcn_c, 1, c->fz[k].f(), cur, cur, s));
      float* out = k == 0 ? c->grad[L].f() : bufs[(nh - k) & 1];
      GCHK(gemm(cur, wb, m->fcn_l[k].WT.f(), wk, out, wk, nl, wb, wk, 0, nullptr, nullptr, 0, s));
      cur = out;
    }
  } else {
    GCHK(launch_gen_readout((int)nl, m->dims[L], c->x[L].f(), m->readout_v.f(), g.type, m->scale.f(),
                            m->shift.f(), m->per_species, c->eat.f(), c->grad[L].f(), s));
  }
  GCHK(launch_sum(nl, c->eat.f(), c->part.f(), energy ? energy : c->scratch.f(), s));
  if (atomic_energy && nl > 0)
    GCHK(hipMemcpyAsync(atomic_energy, c->eat.p, nl * 4, hipMemcpyDeviceToDevice, s));
  // the edge accumulators of the backward
  GCHK(launch_zero(c->dYacc.f(), c->E * m->ny, s));
  GCHK(launch_zero(c->demb.f(), c->E * m->nb, s));
  return hipSuccess;
}

hipError_t gen_layer_backward(GenCtx* c, const GenModel* m, const GenGraph& g, int t, hipStream_t s) {
  const GenLayer& G = m->L[t];
  const int64_t n = c->n, nl = c->nl, E = c->E;
  GCHK(launch_gen_gate_bwd((int)nl, G.gate, c->y[t].f(), c->grad[t + 1].f(), c->dy.f(), s));
  GCHK(gemm(c->dy.f(), G.dg, G.si2.WT.f(), G.dm, c->dagg.f(), G.dm, nl, G.dg, G.dm, 0, nullptr, nullptr, 0, s));
  if (E > 0) {
    // per edge dE/dw, dE/dY and (t > 0) dE/dh rows, summed per neighbour
    GCHK(launch_gtp_bwd((int)nl, g.row_ptr, g.nbr, c->h[t].f(), c->Y.f(), c->w[t].f(), c->dagg.f(),
                        *gtp_tables(G.gtp), c->dw.f(), t > 0 ? c->dxc.f() : nullptr, c->dYt.f(), s));
    GCHK(launch_gen_add(E * m->ny, c->dYt.f(), c->dYacc.f(), s));
    // radial MLP backward down to dE/demb (accumulated over the blocks)
    const int nh = (int)G.width.size() - 2;
    const float* d = c->dw.f();
    int wd = G.W;
    float* bufs[2] = {c->dA0.f(), c->dA1.f()};
    for (int k = nh; k >= 1; --k) {
      const int wk = G.width[k];
      float* o = bufs[k & 1];
      GCHK(gemm(d, wd, G.mlp[k].WT.f(), wk, o, wk, E, wd, wk, 2, c->pre[t][k - 1].f(), nullptr, 0, s));
      d = o;
      wd = wk;
    }
    GCHK(gemm(d, wd, G.mlp[0].WT.f(), m->nb, c->demb.f(), m->nb, E, wd, m->nb, 0, nullptr, nullptr, 1, s));
  }
  if (t > 0) {
    if (n > 0) {
      if (E > 0) GCHK(launch_gather_rows((int)n, G.dx, g.src_ptr, g.src_perm, c->dxc.f(), c->dh.f(), s));
      else GCHK(launch_zero(c->dh.f(), n * G.dx, s));
    }
    GCHK(gemm(c->dh.f(), G.dx, G.si1.WT.f(), G.dx, c->grad[t].f(), G.dx, n, G.dx, G.dx, 0, nullptr, nullptr, 0, s));
    if (G.sc_species)
      GCHK(launch_gen_species_linear((int)nl, G.dg, G.dx, g.type, c->dy.f(), G.scsT.f(), c->grad[t].f(), 1, s));
    else
      GCHK(gemm(c->dy.f(), G.dg, G.sc.WT.f(), G.dx, c->grad[t].f(), G.dx, nl, G.dg, G.dx, 0, nullptr, nullptr, 1, s));
  }
  return hipSuccess;
}

hipError_t gen_forces(GenCtx* c, const GenModel* m, const GenGraph& g, float* forces, float* virial6,
                      float* edge_grad, hipStream_t s) {
  const int64_t n = c->n, nl = c->nl, E = c->E;
  GCHK(launch_gen_edge_force(m->edge, E, g.vec, c->dYacc.f(), c->demb.f(), c->fe.f(), c->vpart.f(), s));
  GCHK(launch_final_sum(gen_edge_force_blocks(E), 6, c->vpart.f(), virial6 ? virial6 : c->scratch.f(), s));
  if (forces)
    GCHK(launch_atom_force((int)n, (int)nl, g.row_ptr, g.src_ptr, g.src_perm, c->fe.f(), forces, s));
  if (edge_grad && E > 0) GCHK(hipMemcpyAsync(edge_grad, c->fe.p, E * 12, hipMemcpyDeviceToDevice, s));
  return hipSuccess;
}

}  // namespace e3gnn
