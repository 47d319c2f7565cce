// Host side of libe3gnn_hip.so: model loading (this build's deploy format),
// workspace management and the per-layer orchestration of the SevenNet-0
// energy + force evaluation, behind the C ABI of include/e3gnn.h.
//
// Pipeline (sevenn/model_build.py:186-445; deploy.py:20-32 for the serial
// deployment, model_build.py:103-182 for the parallel segments):
//   edge embedding -> onehot embed -> 5 x [self_connection_intro,
//   self_interaction_1, IrrepsConvolution, self_interaction_2,
//   self_connection_outro, gate] -> readout -> SpeciesWiseRescale -> sum
// and the reverse-mode pass that ForceStressOutput gets from autograd
// (force_output.py:74-130), written out explicitly.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/e3gnn.h"
#include "cg_tables.h"
#include "d3.h"
#include "dbuf.h"
#include "generic.h"
#include "train_ops.h"
#include "common.h"
#include "fused.h"
#include "gtp.h"
#include "minijson.h"
#include "node.h"
#include "neighbor.h"
#include "tgemm.h"
#include "tp.h"

using namespace e3gnn;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

// E3GNN_TRACE_ERRORS=1: report where HIP's thread-local error state got set
bool trace_errors() {
  static int on = [] {
    const char* v = std::getenv("E3GNN_TRACE_ERRORS");
    return v && v[0] == '1';
  }();
  return on;
}
void trace_point(const char* where) {
  if (!trace_errors()) return;
  hipError_t e = hipPeekAtLastError();
  if (e != hipSuccess) std::fprintf(stderr, "[e3gnn] sticky HIP error %d (%s) at %s\n", (int)e,
                                    hipGetErrorString(e), where);
}

#define HIPCHK(expr)                                                                          \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    if (_e != hipSuccess)                                                                     \
      return fail(E3GNN_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));         \
  } while (0)

// ------------------------------------------------------------ irreps helpers
struct Irr {
  int mul, l;
};
using Irreps = std::vector<Irr>;

Irreps parse_irreps(const std::string& s) {
  Irreps out;
  std::stringstream ss(s);
  std::string term;
  while (std::getline(ss, term, '+')) {
    const auto x = term.find('x');
    out.push_back({std::stoi(term.substr(0, x)), std::stoi(term.substr(x + 1))});
  }
  return out;
}
int irreps_dim(const Irreps& ir) {
  int d = 0;
  for (auto& i : ir) d += i.mul * (2 * i.l + 1);
  return d;
}
// merge consecutive equal-l entries (the layouts are identical, see tp.h)
Irreps merged(const Irreps& ir) {
  Irreps out;
  for (auto& i : ir) {
    if (!out.empty() && out.back().l == i.l) out.back().mul += i.mul;
    else out.push_back(i);
  }
  return out;
}

// bf16 round-to-nearest-even (finite inputs) and its exact widening
uint16_t bf16_rne(float x) {
  uint32_t u;
  std::memcpy(&u, &x, 4);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
float bf16_to_f32(uint16_t h) {
  const uint32_t u = (uint32_t)h << 16;
  float x;
  std::memcpy(&x, &u, 4);
  return x;
}

// e3nn o3.Linear on merged irreps: one block per l present in both.
struct LinBlock {
  int l, K, N, in_off, out_off, w_off, wt_off;
};
struct Linear {
  std::vector<LinBlock> blocks;
  DBuf W, WT;  // W: per block [K x N] row-major; WT: [N x K]
  std::vector<float> W_h, WT_h;  // host copies (pair construction at load)
  int din = 0, dout = 0;
};

// Node-linear problems for k_nodelin (gemm.hip): each block one output irrep
// block, from one linear (K2 = 0) or two K-concatenated linears writing the
// same block; `W` holds [K1 + K2 x N] per block (16-byte aligned).
struct PairBlock {
  int l, N, out_off, K1, off1, K2, off2, w_off;
  int64_t wb_off;  // byte offset of the block's bf16 pieces in LinPair::Wb
};
struct LinPair {
  std::vector<PairBlock> blocks;
  DBuf W;
  // W as three bf16 pieces (W = p0 + p1 + p2 exactly) in the 16x16x32 MFMA
  // B-operand order of k_nodelin_b (gemm.hip): per block [16-column block cb]
  // [32-row chunk kc (K1's chunks, then K2's)][piece][lane][8], element t of
  // lane l = W[k][16 cb + l % 16] with k = 32 kc' + 8 (l / 16) + t inside its
  // part (0 past the part's rows / the block's columns)
  DBuf Wb;
  bool ok = false;
};

}  // namespace

// ------------------------------------------------------------ model
struct e3gnn_model {
  int device = 0;
  int nsp = 0, nlayer = 0;
  // channel family of the fused kernels (tp.h Family<f>): 0 SevenNet-0,
  // 1 uniform 64, 2 uniform 32
  int family = 0;
  // kernel kind code of block t (tp.h: 3 * family + first / middle / last)
  int kcode(int t) const { return 3 * family + (t == 0 ? 0 : (t == nlayer - 1 ? 2 : 1)); }
  std::vector<GateDims> gdims;  // gate layout per block (node.h)
  int max_dx = 0, max_dg = 0;
  float cutoff = 5.f, r_on = 4.5f;
  int raw_sh = 0;   // SH of the raw edge vector (sh_normalize false: checkpoints before sevenn 0.9)
  std::vector<Irreps> irreps;  // irreps_manual per layer boundary (merged)
  std::vector<Irreps> gin, mid;
  std::vector<int> W;          // radial weight numel per layer
  std::vector<float> denom;
  DBuf coeffs, embed, readout_v, scale, shift;
  std::vector<std::unique_ptr<Linear>> sc, si1, si2;
  // k_nodelin problem sets: si1, si1^T, si2^T, si2 + sc (forward, gate
  // epilogue), si1^T + sc^T (backward)
  std::vector<std::unique_ptr<LinPair>> nl_si1, nl_si1t, nl_si2t, nl_fwd, nl_bwd;
  struct Mlp {
    DBuf w0, w1, w2, w0t, w1t, w2t;
    DBuf w1p, w2p, w2q, w2r;  // MFMA-operand orders of the fused kernels (fused.h)
    DBuf w2b;            // 3-way bf16 split of w2 in 16x16x32 operand order (fused.h)
    DBuf w2d;            // the same for the fused backward's pairs (fused.h)
    DBuf w2v;            // w2b's column blocks in visiting order (fused.h)
    DBuf w1b, w1tb, w0tb;  // layer-1 / chain-backward operands, w2b order (fused.h)
  };
  std::vector<Mlp> mlp;
  // any other nequip-family deployment: the generic engine (generic.cpp)
  GenModel* gen = nullptr;
  ~e3gnn_model() {
    if (gen) gen_free(gen);
  }
};

namespace {

struct Stat {
  double ms = 0, flops = 0, bytes = 0;
  int64_t launches = 0;
};
struct Pending {
  int cls;
  hipEvent_t a, b;
  double flops, bytes;
};
const char* kClassNames[] = {"graph_build", "edge_embed",  "node_linear", "radial_mlp_fwd",
                             "tp_fwd",      "gate_fwd",    "readout",     "gate_bwd",
                             "tp_bwd",      "radial_mlp_bwd", "gather_src", "edge_force",
                             "atom_force",  "embed",
                             // fused kernels, one class per kernel and block kind
                             "conv_fwd.first", "conv_fwd.mid", "conv_fwd.last",
                             "conv_bwd_x.first", "conv_bwd_x.mid", "conv_bwd_x.last"};
enum Cls {
  C_GRAPH,
  C_EMBED_EDGE,
  C_LINEAR,
  C_MLP_FWD,
  C_TP_FWD,
  C_GATE_FWD,
  C_READOUT,
  C_GATE_BWD,
  C_TP_BWD,
  C_MLP_BWD,
  C_GATHER,
  C_EDGE_FORCE,
  C_ATOM_FORCE,
  C_EMBED_NODE,
  C_CONV_FWD,             // + kind (0 first, 1 mid, 2 last)
  C_CONV_BWD_X = C_CONV_FWD + 3,
  C_NCLS = C_CONV_BWD_X + 3
};
static_assert(sizeof(kClassNames) / sizeof(kClassNames[0]) == C_NCLS, "class names");

// algorithmic per-edge FLOP of one TP forward (SevenNet-0:
// 3,456 / 16,832 / 1,184 for the first / middle / last block)
double tp_flops_per_edge(int code) { return fused_kind_tp_flops(code); }

}  // namespace

struct e3gnn_ctx {
  e3gnn_model* m;
  GenCtx* gen = nullptr;  // the generic engine's buffers (m->gen)
  int64_t n = 0, nl = 0, E = 0;
  // halo overlap: owned centres [0, n_int) have no ghost neighbour; their
  // edges are [0, e_int) (e3gnn_set_interior, effective at graph_set)
  int64_t n_interior_req = 0, n_int = 0, e_int = 0;
  // graph
  DBuf type, center, nbr, vec, row_ptr, src_ptr, src_perm, cnt, err;
  DBuf Y, emb, dY, dgu, demb, fe;
  // node linears on k_nodelin (node-aligned tiles, si2 + sc in one problem,
  // gate in the epilogue; 1, default) or the grouped k_gemm + k_gate kernels
  // (0; E3GNN_NODELIN=0)
  int nodelin = [] {
    const char* v = std::getenv("E3GNN_NODELIN");
    return (v && std::string(v) == "0") ? 0 : 1;
  }();
  // 0: fused radial-MLP + TP kernels (fused.hip); 1: the unfused v1 kernels
  // (materialised per-edge weights; kept as an independent cross-check)
  int impl = [] {
    const char* v = std::getenv("E3GNN_IMPL");
    return (v && std::string(v) == "v1") ? 1 : 0;
  }();
  int graph_impl = 0;  // impl in force since the last e3gnn_graph_set (buffers sized for it)
  // per layer
  std::vector<DBuf> x, grad, h, y, w, a1, a2;
  DBuf H1, H2, agg, dw, dxc, dy, dh, eat, part, vpart, scratch6;
  bool timing = false;
  bool stream_ordered = false;  // e3gnn_set_stream_ordered
  // stream-ordered mode: the end of the last evaluation on `done_stream`; a
  // call on another stream waits for it before touching the shared
  // workspaces (inputs are copied into them at graph_set)
  hipEvent_t done_ev = nullptr;
  hipStream_t done_stream = nullptr;
  bool done_pending = false;
  Stat stats[C_NCLS];
  std::vector<Pending> pending;
  std::vector<hipEvent_t> evpool;
  int readout_done = 0;

  hipEvent_t ev() {
    if (!evpool.empty()) {
      hipEvent_t e = evpool.back();
      evpool.pop_back();
      return e;
    }
    hipEvent_t e;
    (void)hipEventCreate(&e);
    return e;
  }
  void flush() {
    for (auto& p : pending) {
      (void)hipEventSynchronize(p.b);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, p.a, p.b);
      stats[p.cls].ms += ms;
      stats[p.cls].launches += 1;
      stats[p.cls].flops += p.flops;
      stats[p.cls].bytes += p.bytes;
      evpool.push_back(p.a);
      evpool.push_back(p.b);
    }
    pending.clear();
  }
  ~e3gnn_ctx() {
    if (gen) gen_ctx_free(gen);
    flush();
    if (done_ev) {
      (void)hipEventSynchronize(done_ev);
      (void)hipEventDestroy(done_ev);
    }
    for (auto e : evpool) (void)hipEventDestroy(e);
  }
};

namespace {

// Timed region helper: brackets the enclosed launches with events when timing.
struct Region {
  e3gnn_ctx* c;
  hipStream_t s;
  int cls;
  double flops, bytes;
  hipEvent_t a = nullptr;
  Region(e3gnn_ctx* c_, hipStream_t s_, int cls_, double f = 0, double b = 0)
      : c(c_), s(s_), cls(cls_), flops(f), bytes(b) {
    if (c->timing) {
      a = c->ev();
      (void)hipEventRecord(a, s);
    }
  }
  ~Region() {
    if (c->timing) {
      hipEvent_t b = c->ev();
      (void)hipEventRecord(b, s);
      c->pending.push_back({cls, a, b, flops, bytes});
    }
  }
};

// ------------------------------------------------------------ linear → GEMM problems
void add_prob(GemmBatch& b, const GemmProb& p) {
  GemmProb q = p;
  const int tm = (q.M + 63) / 64, tn = (q.N + 63) / 64;
  if (tm == 0 || tn == 0) return;
  q.tiles_n = tn;
  q.tile_begin = b.total_tiles;
  b.p[b.nprob++] = q;
  b.total_tiles += tm * tn;
}

GemmProb base_prob() {
  GemmProb p;
  std::memset(&p, 0, sizeof(p));
  p.R = 1;
  return p;
}

// y[rows, dout] (+)= x[rows, din] @ lin    (row strides lda/ldc)
GemmBatch lin_fwd(const Linear& L, const float* x, int64_t lda, float* y, int64_t ldc, int64_t rows,
                  int beta) {
  GemmBatch b;
  std::memset(&b, 0, sizeof(b));
  for (auto& k : L.blocks) {
    GemmProb p = base_prob();
    p.A = x;
    p.B = L.W.f() + k.w_off;
    p.C = y;
    p.lda = lda;
    p.ldc = ldc;
    p.R = 2 * k.l + 1;
    p.M = (int)(rows * p.R);
    p.K = k.K;
    p.N = k.N;
    p.a_off = k.in_off;
    p.c_off = k.out_off;
    p.ldb = k.N;
    p.beta = beta;
    add_prob(b, p);
  }
  return b;
}
// dx[rows, din] (+)= dy[rows, dout] @ lin^T
GemmBatch lin_bwd(const Linear& L, const float* dy, int64_t ldy, float* dx, int64_t ldx,
                  int64_t rows, int beta) {
  GemmBatch b;
  std::memset(&b, 0, sizeof(b));
  for (auto& k : L.blocks) {
    GemmProb p = base_prob();
    p.A = dy;
    p.B = L.WT.f() + k.wt_off;
    p.C = dx;
    p.lda = ldy;
    p.ldc = ldx;
    p.R = 2 * k.l + 1;
    p.M = (int)(rows * p.R);
    p.K = k.N;
    p.N = k.K;
    p.a_off = k.out_off;
    p.c_off = k.in_off;
    p.ldb = k.K;
    p.beta = beta;
    add_prob(b, p);
  }
  return b;
}
double lin_flops(const Linear& L, int64_t rows) {
  double f = 0;
  for (auto& k : L.blocks) f += 2.0 * rows * (2 * k.l + 1) * k.K * k.N;
  return f;
}

// k_nodelin batch over rows [0, rows) of A (+ A2) -> C for the blocks of P
// selected by `sel` (0 all, 1 the l = 0 block, 2 the l > 0 blocks); `fix`
// fills the epilogue fields per block.  false: not expressible (the caller
// takes the k_gemm path).
struct NoFix {
  void operator()(NlProb&, const PairBlock&) const {}
};
template <class Fix = NoFix>
bool nl_batch(NlBatch& b, LinPair& P, const float* A, int64_t lda, const float* A2, int64_t lda2,
              float* C, int64_t ldc, int64_t rows, int epi, int sel = 0, Fix fix = Fix()) {
  std::memset(&b, 0, sizeof(b));
  if (!P.ok) return false;
  for (auto& k : P.blocks) {
    if ((sel == 1 && k.l != 0) || (sel == 2 && k.l == 0)) continue;
    NlProb q;
    std::memset(&q, 0, sizeof(q));
    q.A = A;
    q.lda = lda;
    q.a_off = k.off1;
    q.A2 = k.K2 ? A2 : nullptr;
    q.lda2 = lda2;
    q.a_off2 = k.off2;
    q.K1 = k.K1;
    q.K = k.K1 + k.K2;
    q.B = P.W.f() + k.w_off;
    q.Bb = P.Wb.p ? static_cast<const char*>(P.Wb.p) + k.wb_off : nullptr;
    q.C = C;
    q.ldc = ldc;
    q.c_off = k.out_off;
    q.N = k.N;
    q.R = 2 * k.l + 1;
    q.nodes = (int)rows;
    q.epi = epi;
    fix(q, k);
    if (!add_nl(b, q)) return false;
  }
  return true;
}
double pair_flops(const LinPair& P, int64_t rows) {
  double f = 0;
  for (auto& k : P.blocks) f += 2.0 * rows * (2 * k.l + 1) * (k.K1 + k.K2) * k.N;
  return f;
}

// ------------------------------------------------------------ model loading
int build_linear(Linear& L, const Irreps& in, const Irreps& out, const float* w, size_t numel,
                 double extra_scale_t) {
  std::vector<float> W, WT;
  int in_off = 0;
  size_t woff = 0;
  L.din = irreps_dim(in);
  L.dout = irreps_dim(out);
  for (auto& a : in) {
    int out_off = 0;
    for (auto& b : out) {
      if (a.l == b.l) {
        LinBlock k{a.l, a.mul, b.mul, in_off, out_off, (int)W.size(), (int)WT.size()};
        // e3nn Linear 'element' path normalisation: 1/sqrt(fan_in), fan_in = mul_in
        const double sc = 1.0 / std::sqrt((double)a.mul);
        if (woff + (size_t)a.mul * b.mul > numel) return -1;
        for (int u = 0; u < a.mul; ++u)
          for (int v = 0; v < b.mul; ++v) W.push_back((float)(w[woff + (size_t)u * b.mul + v] * sc));
        for (int v = 0; v < b.mul; ++v)
          for (int u = 0; u < a.mul; ++u)
            WT.push_back((float)(w[woff + (size_t)u * b.mul + v] * sc * extra_scale_t));
        woff += (size_t)a.mul * b.mul;
        L.blocks.push_back(k);
      }
      out_off += b.mul * (2 * b.l + 1);
    }
    in_off += a.mul * (2 * a.l + 1);
  }
  if (woff != numel) return -1;
  if (upload(L.W, W) != hipSuccess || upload(L.WT, WT) != hipSuccess) return -2;
  L.W_h = std::move(W);
  L.WT_h = std::move(WT);
  return 0;
}

// One linear (forward: in -> out with W, or transposed: out -> in with WT) plus
// optionally a second one into the same output blocks (K-concatenated).
// ok = false when a block of the second has no partner in the first.
int build_pair(LinPair& P, const Linear& a, bool ta, const Linear* b, bool tb) {
  std::vector<float> W;
  size_t matched = 0;
  for (auto& k : a.blocks) {
    PairBlock pb;
    pb.l = k.l;
    pb.N = ta ? k.K : k.N;
    pb.out_off = ta ? k.in_off : k.out_off;
    pb.K1 = ta ? k.N : k.K;
    pb.off1 = ta ? k.out_off : k.in_off;
    pb.K2 = 0;
    pb.off2 = 0;
    pb.w_off = (int)W.size();
    const float* w1 = ta ? a.WT_h.data() + k.wt_off : a.W_h.data() + k.w_off;
    W.insert(W.end(), w1, w1 + (size_t)pb.K1 * pb.N);
    if (b) {
      for (auto& q : b->blocks) {
        const int n2 = tb ? q.K : q.N, o2 = tb ? q.in_off : q.out_off;
        if (q.l != k.l || o2 != pb.out_off) continue;
        if (n2 != pb.N || pb.K2) return 0;
        pb.K2 = tb ? q.N : q.K;
        pb.off2 = tb ? q.out_off : q.in_off;
        const float* w2 = tb ? b->WT_h.data() + q.wt_off : b->W_h.data() + q.w_off;
        W.insert(W.end(), w2, w2 + (size_t)pb.K2 * pb.N);
        ++matched;
      }
    }
    while (W.size() % 4) W.push_back(0.f);
    P.blocks.push_back(pb);
  }
  if (b && matched != b->blocks.size()) return 0;
  if (upload(P.W, W) != hipSuccess) return -2;
  // the bf16x6 operand image (k_nodelin_b)
  std::vector<float> Wb;   // bf16 pairs packed in floats (1 KB per piece image)
  for (auto& pb : P.blocks) {
    pb.wb_off = (int64_t)Wb.size() * 4;
    const int ncb = (pb.N + 15) / 16, nk1 = (pb.K1 + 31) / 32, nk2 = (pb.K2 + 31) / 32;
    const size_t base = Wb.size();
    Wb.resize(base + (size_t)ncb * (nk1 + nk2) * 3 * 256, 0.f);
    uint16_t* o = reinterpret_cast<uint16_t*>(Wb.data() + base);
    const float* w = W.data() + pb.w_off;   // [K1 + K2][N]
    for (int cb = 0; cb < ncb; ++cb)
      for (int kc = 0; kc < nk1 + nk2; ++kc)
        for (int l = 0; l < 64; ++l)
          for (int t = 0; t < 8; ++t) {
            const bool second = kc >= nk1;
            const int kk = 32 * (second ? kc - nk1 : kc) + 8 * (l / 16) + t;
            const int col = 16 * cb + l % 16;
            float v = 0.f;
            if (col < pb.N && kk < (second ? pb.K2 : pb.K1))
              v = w[(size_t)(second ? pb.K1 + kk : kk) * pb.N + col];
            for (int pc = 0; pc < 3; ++pc) {
              const uint16_t hb = bf16_rne(v);
              o[(((size_t)cb * (nk1 + nk2) + kc) * 3 + pc) * 512 + l * 8 + t] = hb;
              v -= bf16_to_f32(hb);
            }
          }
  }
  if (upload(P.Wb, Wb) != hipSuccess) return -2;
  P.ok = true;
  return 0;
}

// the path table of a fused kind code (tp.h)
std::vector<PathDef> kind_paths(int code) {
  std::vector<PathDef> P(16);
  P.resize(fused_kind_paths(code, P.data(), (int)P.size()));
  return P;
}

// Column start of every 16-channel weight block in the order the fused
// kernels visit them (input irrep I, channel block jj, then the paths of I in
// instruction order): pairs of consecutive blocks form one K = 32 MFMA operand
// of the lock-step backward's dH2 product (MlpW::w2d).
std::vector<int> bwd_w_block_cols(int code) {
  const auto P = kind_paths(code);
  std::vector<int> cols;
  for (int I = 0; I < 3; ++I) {
    int mul = 0;
    for (auto& p : P)
      if (p.l1 == I) mul = p.mul;
    for (int jj = 0; jj < mul / 16; ++jj)
      for (auto& p : P)
        if (p.l1 == I) cols.push_back(p.woff + 16 * jj);
  }
  return cols;
}

// IrrepsConvolution instruction list (convolution.py:72-95) vs the kernel
// tables of kind code `code`
bool check_paths(int code, const Irreps& x, int lmax_out) {
  struct Ins {
    int l1, l2, l3, mul, xoff;
  };
  const auto P = kind_paths(code);
  int DX = 0, W = 0, DM = 0;
  if (P.empty() || !fused_kind_dims(code, &DX, &W, &DM)) return false;
  std::vector<Ins> ins;
  int xoff = 0;
  for (auto& i : x) {
    for (int l2 = 0; l2 <= 2; ++l2)
      for (int l3 = std::abs(i.l - l2); l3 <= i.l + l2; ++l3)
        if (l3 <= lmax_out) ins.push_back({i.l, l2, l3, i.mul, xoff});
    xoff += i.mul * (2 * i.l + 1);
  }
  if (ins.size() != P.size()) return false;
  // mid slots: stable sort by l3
  std::vector<int> moff(ins.size());
  int off = 0;
  for (int l3 = 0; l3 <= 2; ++l3)
    for (size_t k = 0; k < ins.size(); ++k)
      if (ins[k].l3 == l3) {
        moff[k] = off;
        off += ins[k].mul * (2 * l3 + 1);
      }
  if (off != DM) return false;
  int woff = 0;
  for (size_t k = 0; k < ins.size(); ++k) {
    const PathDef& p = P[k];
    if (p.l1 != ins[k].l1 || p.l2 != ins[k].l2 || p.l3 != ins[k].l3 || p.mul != ins[k].mul ||
        p.xoff != ins[k].xoff || p.woff != woff || p.moff != moff[k])
      return false;
    woff += ins[k].mul;
  }
  return woff == W && xoff == DX;
}

}  // namespace

namespace {
template <int A, int B, int C>
void dense_cg(float* out) {
  using T = CG<A, B, C>;
  std::memset(out, 0, sizeof(float) * (2 * A + 1) * (2 * B + 1) * (2 * C + 1));
  for (int q = 0; q < T::n; ++q)
    out[(T::e[q].i * (2 * B + 1) + T::e[q].j) * (2 * C + 1) + T::e[q].k] = T::e[q].c;
}
MlpW mlp_ptrs(const e3gnn_model* m, int t) {
  const auto& mm = m->mlp[t];
  return MlpW{mm.w0.f(),  mm.w1.f(),  mm.w2.f(),  mm.w2t.f(),
              mm.w1p.f(), mm.w2p.f(), mm.w2q.f(), mm.w2r.f(),
              static_cast<const uint16_t*>(mm.w2b.p),
              static_cast<const uint16_t*>(mm.w2d.p),
              static_cast<const uint16_t*>(mm.w2v.p),
              static_cast<const uint16_t*>(mm.w1b.p),
              static_cast<const uint16_t*>(mm.w1tb.p),
              static_cast<const uint16_t*>(mm.w0tb.p)};
}

}  // namespace

namespace {
GenGraph gen_graph(e3gnn_ctx* c) {
  return GenGraph{c->n, c->nl, c->E, c->type.i(), c->nbr.i(), c->vec.f(), c->row_ptr.i(),
                  c->src_ptr.i(), c->src_perm.i(), c->err.i()};
}

// The SevenNet-0-shaped family test: what the specialised engine serves.
// The knobs of nn.sevennet0_kinds (even parity, lmax 2, linear
// self-connection, XPLOR cutoff), what the fused kernels hard-code (8 Bessel
// functions, a 64-64 radial MLP), at least 2 blocks, and the irreps of one
// compiled channel family (tp.h): A x0e -> (L - 1) x C0x0e+C1x1e+C2x2e -> D x0e.
// Returns the family, or -1 (the generic engine serves the deployment).
int fused_family(const minijson::Value& man) {
  // E3GNN_GENERIC=1: every deployment on the generic engine (cross-checks)
  if (const char* g = std::getenv("E3GNN_GENERIC"); g && g[0] == '1') return -1;
  if (man.has("is_parity") && man["is_parity"].boolean()) return -1;
  const int lmax = man.has("lmax_edge") ? (int)man["lmax_edge"].num()
                                        : (man.has("lmax") ? (int)man["lmax"].num() : 2);
  if (lmax != 2) return -1;
  if (man.has("self_connection_type") && man["self_connection_type"].str() != "linear") return -1;
  if (!man.has("cutoff_function") || man["cutoff_function"]["name"].str() != "XPLOR") return -1;
  // linear biases / the FCN readout (model_build.py:194-240, :396-408): the
  // generic engine applies them
  if (man.has("use_bias_in_linear") && man["use_bias_in_linear"].boolean()) return -1;
  if (man.has("readout") && man["readout"].has("type") && man["readout"]["type"].str() != "linear") return -1;
  const int L = (int)man["num_convolution_layer"].num();
  if (L < 2) return -1;
  if (man.has("weight_nn_hidden_neurons")) {
    const auto& h = man["weight_nn_hidden_neurons"].arr();
    if (h.size() != 2 || (int)h[0].num() != 64 || (int)h[1].num() != 64) return -1;
  }
  if (man.has("radial_basis") && man["radial_basis"].has("num") && (int)man["radial_basis"]["num"].num() != 8)
    return -1;
  const auto& ir = man["irreps_manual"].arr();
  if ((int)ir.size() != L + 1) return -1;
  Irreps first, mid, last;
  try {
    first = merged(parse_irreps(ir[0].str()));
    mid = merged(parse_irreps(ir[1].str()));
    last = merged(parse_irreps(ir[L].str()));
  } catch (...) {
    return -1;
  }
  if (first.size() != 1 || first[0].l != 0 || last.size() != 1 || last[0].l != 0) return -1;
  for (int t = 1; t < L; ++t)
    if (ir[t].str() != ir[1].str()) return -1;
  if (L > 1 && (mid.size() != 3 || mid[0].l != 0 || mid[1].l != 1 || mid[2].l != 2)) return -1;
  for (int f = 0; f < N_FAMILIES; ++f) {
    PathDef P0[16], P1[16];
    fused_kind_paths(3 * f, P0, 16);
    fused_kind_paths(3 * f + 1, P1, 16);
    // first block's input A; middle irreps C0 / C1 / C2 (paths 0, 3, 9 of the middle table)
    if (first[0].mul == P0[0].mul && mid[0].mul == P1[0].mul && mid[1].mul == P1[3].mul &&
        mid[2].mul == P1[9].mul)
      return f;
  }
  return -1;
}
}  // namespace

extern "C" {

const char* e3gnn_last_error(void) { return g_err.c_str(); }
int e3gnn_abi_version(void) { return 1; }

e3gnn_model* e3gnn_load(const char* weights_path, const char* manifest_path, int device) {
  auto m = std::make_unique<e3gnn_model>();
  m->device = device;
  trace_point("load:entry");
  if (hipSetDevice(device) != hipSuccess) {
    fail(E3GNN_ERR_HIP, "hipSetDevice failed");
    return nullptr;
  }
  trace_point("load:hipSetDevice");
  minijson::Value man;
  {
    std::ifstream f(manifest_path);
    if (!f) {
      fail(E3GNN_ERR_IO, std::string("cannot open manifest ") + manifest_path);
      return nullptr;
    }
    std::stringstream ss;
    ss << f.rdbuf();
    std::string err;
    if (!minijson::parse(ss.str(), man, err)) {
      fail(E3GNN_ERR_IO, "manifest parse error: " + err);
      return nullptr;
    }
  }
  std::vector<float> flat;
  {
    std::ifstream f(weights_path, std::ios::binary | std::ios::ate);
    if (!f) {
      fail(E3GNN_ERR_IO, std::string("cannot open weights ") + weights_path);
      return nullptr;
    }
    const std::streamsize sz = f.tellg();
    f.seekg(0);
    flat.resize(sz / 4);
    f.read((char*)flat.data(), (std::streamsize)flat.size() * 4);
  }
  try {
    if (man["model_type"].str() != "E3_equivariant_model")
      throw std::runtime_error("unsupported model_type");
    // SevenNet-0's architecture runs on the specialised kernels below; every
    // other member of the family on the generic engine (generic.cpp)
    const int family = fused_family(man);
    if (family < 0) {
      m->gen = gen_load(man, flat);
      m->nsp = gen_num_species(m->gen);
      m->nlayer = gen_num_layers(m->gen);
      m->cutoff = gen_cutoff(m->gen);
      trace_point("load:generic");
      (void)hipGetLastError();
      return m.release();
    }
    // the knobs this engine does not read must hold SevenNet-0's values (the
    // same predicate as nn.sevennet0_kinds)
    // sh_normalize false (checkpoints before sevenn 0.9, util.py:130-146): the
    // same kernels, the SH polynomials of the raw vector (node.hip)
    m->raw_sh = man.has("sh_normalize") && !man["sh_normalize"].boolean() ? 1 : 0;
    m->family = family;
    if (man.has("is_parity") && man["is_parity"].boolean())
      throw std::runtime_error("odd-parity filters are not SevenNet-0's architecture");
    if (man.has("self_connection_type") && man["self_connection_type"].str() != "linear")
      throw std::runtime_error("self_connection_type " + man["self_connection_type"].str() +
                               " is not SevenNet-0's (linear)");
    if (man.has("lmax_edge") && (int)man["lmax_edge"].num() != 2)
      throw std::runtime_error("lmax_edge must be 2 (SevenNet-0)");
    m->nsp = (int)man["num_species"].num();
    m->cutoff = (float)man["cutoff"].num();
    m->r_on = (float)man["cutoff_function"]["cutoff_on"].num();
    if (man["cutoff_function"]["name"].str() != "XPLOR")
      throw std::runtime_error("only the XPLOR cutoff of SevenNet-0 is implemented");
    m->nlayer = (int)man["num_convolution_layer"].num();
    if (std::abs(man["silu_norm"].num() - (double)SILU_NORM) > 1e-6)
      throw std::runtime_error("silu_norm mismatch");
    for (auto& s : man["irreps_manual"].arr()) m->irreps.push_back(merged(parse_irreps(s.str())));
    if ((int)m->irreps.size() != m->nlayer + 1) throw std::runtime_error("irreps_manual length");
    std::map<std::string, std::pair<size_t, size_t>> T;
    for (auto& t : man["tensors"].arr())
      T[t["name"].str()] = {(size_t)t["offset"].num(), (size_t)t["numel"].num()};
    auto get = [&](const std::string& n, size_t expect = 0) -> const float* {
      auto it = T.find(n);
      if (it == T.end()) throw std::runtime_error("missing tensor " + n);
      if (it->second.first + it->second.second > flat.size())
        throw std::runtime_error("tensor out of file range " + n);
      if (expect && it->second.second != expect) throw std::runtime_error("bad size " + n);
      return flat.data() + it->second.first;
    };
    auto numel = [&](const std::string& n) { return T.at(n).second; };
    // geometry / embedding / readout
    const float* cf = get("edge_embedding.basis_function.coeffs", 8);
    if (upload(m->coeffs, std::vector<float>(cf, cf + 8)) != hipSuccess) throw std::runtime_error("upload");
    const int d0 = irreps_dim(m->irreps[0]);
    const float* we = get("onehot_to_feature_x.linear.weight", (size_t)m->nsp * d0);
    std::vector<float> emb((size_t)m->nsp * d0);
    for (size_t i = 0; i < emb.size(); ++i) emb[i] = (float)(we[i] / std::sqrt((double)m->nsp));
    if (upload(m->embed, emb) != hipSuccess) throw std::runtime_error("upload");
    // two linears without activation (D x0e -> H x0e -> 1x0e) folded into one
    // vector, e3nn path weights 1 / sqrt(fan_in) each
    const int dl = irreps_dim(m->irreps[m->nlayer]);
    const int hid = (int)numel("reduce_hidden_to_energy.linear.weight");
    const float* wh = get("reduce_input_to_hidden.linear.weight", (size_t)dl * hid);
    const float* wo = get("reduce_hidden_to_energy.linear.weight", hid);
    std::vector<float> v(dl);
    for (int c = 0; c < dl; ++c) {
      double s = 0;
      for (int k = 0; k < hid; ++k) s += (double)wh[c * hid + k] * wo[k];
      v[c] = (float)(s / (std::sqrt((double)dl) * std::sqrt((double)hid)));
    }
    if (upload(m->readout_v, v) != hipSuccess) throw std::runtime_error("upload");
    trace_point("load:readout");
    const float* sc = get("rescale_atomic_energy.scale", m->nsp);
    const float* sh = get("rescale_atomic_energy.shift", m->nsp);
    if (upload(m->scale, std::vector<float>(sc, sc + m->nsp)) != hipSuccess ||
        upload(m->shift, std::vector<float>(sh, sh + m->nsp)) != hipSuccess)
      throw std::runtime_error("upload");
    // interaction blocks
    for (int t = 0; t < m->nlayer; ++t) {
      const Irreps& xin = m->irreps[t];
      const Irreps& xout = m->irreps[t + 1];
      const bool last = t == m->nlayer - 1;
      // gate irreps_in: scalars + gates (0e) + gated (equivariant_gate.py:48-55)
      Irreps gin;
      int nscal = 0, ngated = 0;
      for (auto& i : xout) (i.l == 0 ? nscal : ngated) += i.mul;
      gin.push_back({nscal + ngated, 0});
      for (auto& i : xout)
        if (i.l > 0) gin.push_back(i);
      const int lmax_out = last ? 0 : 2;
      if (!check_paths(m->kcode(t), xin, lmax_out))
        throw std::runtime_error("convolution path table mismatch at layer " + std::to_string(t));
      {
        // gate layout (node.h GateDims): scalars, then the gated 1e / 2e blocks
        GateDims gd{0, 0, 0};
        for (auto& i : xout) (i.l == 0 ? gd.ns : (i.l == 1 ? gd.g1 : gd.g2)) += i.mul;
        if (last ? (gd.g1 || gd.g2) : false)
          throw std::runtime_error("the last block's output must be scalars");
        for (size_t k = 1; k < xout.size(); ++k)
          if (xout[k].l < xout[k - 1].l) throw std::runtime_error("output irreps must be sorted by l");
        m->gdims.push_back(gd);
        m->max_dx = std::max(m->max_dx, irreps_dim(xin));
        m->max_dg = std::max(m->max_dg, gd.dy());
      }
      // mid irreps merged by l (sorted), see tp.h
      Irreps mid;
      for (int l3 = 0; l3 <= lmax_out; ++l3) {
        int mul = 0;
        for (auto& i : xin)
          for (int l2 = 0; l2 <= 2; ++l2)
            if (std::abs(i.l - l2) <= l3 && l3 <= i.l + l2) mul += i.mul;
        if (mul) mid.push_back({mul, l3});
      }
      m->gin.push_back(gin);
      m->mid.push_back(mid);
      const std::string p = std::to_string(t);
      const float den = *get(p + "_convolution.denominator", 1);
      m->denom.push_back(den);
      auto mk = [&](const std::string& name, const Irreps& a, const Irreps& b, double extra) {
        auto L = std::make_unique<Linear>();
        if (build_linear(*L, a, b, get(name), numel(name), extra) != 0)
          throw std::runtime_error("linear " + name);
        return L;
      };
      trace_point("load:layer-begin");
      m->sc.push_back(mk(p + "_self_connection_intro.linear.weight", xin, gin, 1.0));
      trace_point("load:sc");
      m->si1.push_back(mk(p + "_self_interaction_1.linear.weight", xin, xin, 1.0));
      // backward of si2 feeds dE/dagg_raw = dE/dagg / denominator (convolution.py:117-118)
      m->si2.push_back(mk(p + "_self_interaction_2.linear.weight", mid, gin, 1.0 / den));
      auto pair = [&](const Linear& a, bool ta, const Linear* b, bool tb) {
        auto P = std::make_unique<LinPair>();
        if (build_pair(*P, a, ta, b, tb) < 0) throw std::runtime_error("upload");
        return P;
      };
      m->nl_si1.push_back(pair(*m->si1[t], false, nullptr, false));
      m->nl_si1t.push_back(pair(*m->si1[t], true, nullptr, false));
      m->nl_si2t.push_back(pair(*m->si2[t], true, nullptr, false));
      m->nl_fwd.push_back(pair(*m->si2[t], false, m->sc[t].get(), false));
      m->nl_bwd.push_back(pair(*m->si1[t], true, m->sc[t].get(), true));
      // radial MLP (e3nn FullyConnectedNet, weights / sqrt(fan_in))
      const float* w0 = get(p + "_convolution.weight_nn.layer0.weight", 8 * 64);
      const float* w1 = get(p + "_convolution.weight_nn.layer1.weight", 64 * 64);
      const size_t n2 = numel(p + "_convolution.weight_nn.layer2.weight");
      const float* w2 = get(p + "_convolution.weight_nn.layer2.weight");
      const int W = (int)(n2 / 64);
      int kdx = 0, Wexp = 0, kdm = 0;
      fused_kind_dims(m->kcode(t), &kdx, &Wexp, &kdm);
      if (W != Wexp) throw std::runtime_error("radial weight width mismatch");
      m->W.push_back(W);
      auto scaled = [](const float* a, int r, int c, double s, bool tr) {
        std::vector<float> o((size_t)r * c);
        for (int i = 0; i < r; ++i)
          for (int j = 0; j < c; ++j) {
            const float v = (float)(a[(size_t)i * c + j] * s);
            if (tr) o[(size_t)j * r + i] = v;
            else o[(size_t)i * c + j] = v;
          }
        return o;
      };
      e3gnn_model::Mlp M;
      m->mlp.push_back(std::move(M));
      auto& mm = m->mlp.back();
      const double s0 = 1.0 / std::sqrt(8.0), s1 = 1.0 / 8.0, s2 = 1.0 / 8.0;
      if (upload(mm.w0, scaled(w0, 8, 64, s0, false)) != hipSuccess ||
          upload(mm.w1, scaled(w1, 64, 64, s1, false)) != hipSuccess ||
          upload(mm.w2, scaled(w2, 64, W, s2, false)) != hipSuccess ||
          upload(mm.w0t, scaled(w0, 8, 64, s0, true)) != hipSuccess ||
          upload(mm.w1t, scaled(w1, 64, 64, s1, true)) != hipSuccess ||
          upload(mm.w2t, scaled(w2, 64, W, s2, true)) != hipSuccess)
        throw std::runtime_error("upload mlp");
      {
        // operand orders of fused.hip (see MlpW): per output column n, the 16
        // k-values lane group g consumes are contiguous (4 x b128 per lane)
        const auto a1 = scaled(w1, 64, 64, s1, false), a2 = scaled(w2, 64, W, s2, false);
        auto kperm = [](const std::vector<float>& a, int N) {
          std::vector<float> o((size_t)N * 64);
          for (int n = 0; n < N; ++n)
            for (int g = 0; g < 4; ++g)
              for (int q = 0; q < 4; ++q)
                for (int t = 0; t < 4; ++t)
                  o[(size_t)n * 64 + g * 16 + q * 4 + t] = a[(size_t)(16 * q + 4 * g + t) * N + n];
          return o;
        };
        std::vector<float> q2((size_t)W * 64);
        for (int cb = 0; cb < W / 16; ++cb)
          for (int bh = 0; bh < 4; ++bh)
            for (int g = 0; g < 4; ++g)
              for (int c = 0; c < 16; ++c)
                for (int sx = 0; sx < 4; ++sx)
                  q2[((size_t)(cb * 4 + bh) * 64 + g * 16 + c) * 4 + sx] =
                      a2[(size_t)(16 * bh + c) * W + 16 * cb + 4 * sx + g];
        // w2r: the same blocks with channel 4g + r (the fused backward's dE/dw layout)
        std::vector<float> r2((size_t)W * 64);
        for (int cb = 0; cb < W / 16; ++cb)
          for (int bh = 0; bh < 4; ++bh)
            for (int g = 0; g < 4; ++g)
              for (int c = 0; c < 16; ++c)
                for (int r = 0; r < 4; ++r)
                  r2[((size_t)(cb * 4 + bh) * 64 + g * 16 + c) * 4 + r] =
                      a2[(size_t)(16 * bh + c) * W + 16 * cb + 4 * g + r];
        // w2b (MlpW::w2b): w2 = p0 + p1 + p2 exactly (bf16 pieces, round to
        // nearest even); element t of lane (g, c) in k-half m of column block cb
        // is w2[16(2m + t/4) + 4g + t%4][16 cb + c]
        auto bsplit = [](const std::vector<float>& a, int N) {
          std::vector<float> o((size_t)N * 64 * 3 / 2);
          uint16_t* oh = reinterpret_cast<uint16_t*>(o.data());
          for (int cb = 0; cb < N / 16; ++cb)
            for (int m2 = 0; m2 < 2; ++m2)
              for (int g = 0; g < 4; ++g)
                for (int c = 0; c < 16; ++c)
                  for (int t = 0; t < 8; ++t) {
                    float v = a[(size_t)(16 * (2 * m2 + t / 4) + 4 * g + t % 4) * N + 16 * cb + c];
                    for (int pc = 0; pc < 3; ++pc) {
                      const uint16_t hb = bf16_rne(v);
                      oh[((((size_t)cb * 3 + pc) * 2 + m2) * 64 + g * 16 + c) * 8 + t] = hb;
                      v -= bf16_to_f32(hb);
                    }
                  }
          return o;
        };
        const std::vector<float> b2 = bsplit(a2, W);
        // the MLP's other products in the same order: W1 (64 x 64, in x out),
        // W1^T, and W0^T (64 x 8) padded to 16 columns
        {
          const auto a0 = scaled(w0, 8, 64, s0, false);
          std::vector<float> a1t((size_t)64 * 64), a0t((size_t)64 * 16, 0.f);
          for (int i = 0; i < 64; ++i)
            for (int j = 0; j < 64; ++j) a1t[(size_t)j * 64 + i] = a1[(size_t)i * 64 + j];
          for (int n = 0; n < 8; ++n)
            for (int k = 0; k < 64; ++k) a0t[(size_t)k * 16 + n] = a0[(size_t)n * 64 + k];
          if (upload(mm.w1b, bsplit(a1, 64)) != hipSuccess || upload(mm.w1tb, bsplit(a1t, 64)) != hipSuccess ||
              upload(mm.w0tb, bsplit(a0t, 16)) != hipSuccess)
            throw std::runtime_error("upload mlp (w1b)");
        }
        // the kernels' visiting order of the 16-column blocks (input irrep,
        // channel block, path): pairs of consecutive blocks
        const std::vector<int> cols = bwd_w_block_cols(m->kcode(t));
        if ((int)cols.size() * 16 != W || cols.size() % 2)
          throw std::runtime_error("dE/dw block order does not cover the weights");
        // w2d (MlpW::w2d): element t of lane (g, c) for hidden block bh is
        // w2[16 bh + c][col], col = cols[2P] + 4g + t (t < 4) or cols[2P + 1] + 4g + t - 4
        std::vector<float> d2((size_t)W * 64 * 3 / 2);
        uint16_t* d2h = reinterpret_cast<uint16_t*>(d2.data());
        for (size_t P = 0; P < cols.size() / 2; ++P)
          for (int bh = 0; bh < 4; ++bh)
            for (int g = 0; g < 4; ++g)
              for (int c = 0; c < 16; ++c)
                for (int t8 = 0; t8 < 8; ++t8) {
                  const int col = t8 < 4 ? cols[2 * P] + 4 * g + t8 : cols[2 * P + 1] + 4 * g + t8 - 4;
                  float v = a2[(size_t)(16 * bh + c) * W + col];
                  for (int pc = 0; pc < 3; ++pc) {
                    const uint16_t hb = bf16_rne(v);
                    d2h[(((P * 3 + pc) * 4 + bh) * 64 + g * 16 + c) * 8 + t8] = hb;
                    v -= bf16_to_f32(hb);
                  }
                }
        if (upload(mm.w2d, d2) != hipSuccess) throw std::runtime_error("upload mlp (w2d)");
        // w2v (MlpW::w2v): w2b's blocks in the visiting order of the kernels
        {
          std::vector<float> v2(b2.size());
          const size_t blk = (size_t)64 * 16 * 3 / 2;   // floats per column block
          for (size_t k = 0; k < cols.size(); ++k)
            std::memcpy(v2.data() + k * blk, b2.data() + (size_t)(cols[k] / 16) * blk, blk * 4);
          if (upload(mm.w2v, v2) != hipSuccess) throw std::runtime_error("upload mlp (w2v)");
        }
        if (W % 16 || upload(mm.w1p, kperm(a1, 64)) != hipSuccess ||
            upload(mm.w2p, kperm(a2, W)) != hipSuccess || upload(mm.w2q, q2) != hipSuccess ||
            upload(mm.w2r, r2) != hipSuccess ||
            upload(mm.w2b, b2) != hipSuccess)
          throw std::runtime_error("upload mlp (packed)");
      }
      trace_point("load:mlp");
    }
  } catch (const std::exception& ex) {
    fail(E3GNN_ERR_IO, std::string("model load: ") + ex.what());
    return nullptr;
  }
  trace_point("load:exit");
  // every HIP call above was checked; do not leave the host application's
  // thread-local HIP error state dirty (torch re-reads it after its own calls)
  (void)hipGetLastError();
  return m.release();
}

void e3gnn_free(e3gnn_model* m) { delete m; }

int e3gnn_model_info(const e3gnn_model* m, int* num_species, float* cutoff, int* num_layers,
                     int* comm_size) {
  if (!m) return fail(E3GNN_ERR_ARG, "null model");
  if (num_species) *num_species = m->nsp;
  if (cutoff) *cutoff = m->cutoff;
  if (num_layers) *num_layers = m->nlayer;
  if (comm_size) {
    if (m->gen) {  // the widest exchanged row (x[t] / dE/dx[t], t >= 1)
      int d = 0;
      for (int t = 1; t <= m->nlayer; ++t) d = std::max(d, gen_feature_dim(m->gen, t));
      *comm_size = d;
    } else {
      *comm_size = irreps_dim(m->irreps[1]);
    }
  }
  return E3GNN_OK;
}

int64_t e3gnn_gemm_workspace_floats(int n, const e3gnn_gemm_desc* d) {
  if (n < 0 || (n > 0 && !d)) return -1;
  int64_t w = 0;
  for (int i = 0; i < n; ++i) {
    const int sp = tg_splits(d[i].m, d[i].n, (int64_t)d[i].k + d[i].k2);
    if (sp > 1) w += (int64_t)sp * d[i].m * d[i].n;
  }
  return w;
}

static int gemm_prob(const e3gnn_gemm_desc& q, int i, TgProb& p) {
  if (q.m < 0 || q.n < 0 || q.k < 0 || q.k2 < 0 || (q.m > 0 && q.n > 0 && (!q.c || (q.k > 0 && (!q.a || !q.b)) ||
                                                                      (q.k2 > 0 && (!q.a2 || !q.b2)))))
    return fail(E3GNN_ERR_ARG, "e3gnn_gemm_grouped: bad problem " + std::to_string(i));
  if (q.beta != 0 && q.beta != 1) return fail(E3GNN_ERR_ARG, "e3gnn_gemm_grouped: beta must be 0 or 1");
  p = TgProb{};
  // op(A)(m, k): X[m][k] (ld, k contiguous) or X[k][m]; op(B)(k, n) as
  // element (n, k): B[k][n] or B[n][k]
  auto lay = [](const float* X, int64_t ld, bool kfast, int K) {
    return TgLay{X, kfast ? (int)ld : 1, kfast ? 1 : (int)ld, 0, 1, 0, K};
  };
  auto glay = [](const float* X, const e3gnn_gemm_layout& g) {
    return TgLay{X, (int)g.ld, (int)g.kst, (int)g.sst, g.rep, g.rs, g.ks};
  };
  if (q.layout) {
    const e3gnn_gemm_layouts& L = *q.layout;
    p.A1 = glay(q.a, L.a); p.B1 = glay(q.b, L.b); p.A2 = glay(q.a2, L.a2); p.B2 = glay(q.b2, L.b2);
    p.ldc = L.ldc; p.crep = L.crep; p.crs = L.crs; p.cns = L.cns;
  } else {
    p.A1 = lay(q.a, q.lda, !q.trans_a, q.k);
    p.B1 = lay(q.b, q.ldb, q.trans_b, q.k);
    p.A2 = lay(q.a2, q.lda2, !q.trans_a2, q.k2);
    p.B2 = lay(q.b2, q.ldb2, q.trans_b2, q.k2);
    p.ldc = q.ldc; p.crep = 1; p.crs = 0; p.cns = 1;
  }
  // the kernel addresses each operand through one buffer descriptor with
  // 32-bit byte offsets (TG_RECORDS, ~2 GB): refuse what would wrap
  {
    auto fits = [](const TgLay& L, int64_t rows, int64_t K, const e3gnn_gemm_layout* g) {
      if (g && (g->ld < 0 || g->kst < 0 || g->sst < 0 || g->rs < 0 || g->ld > INT32_MAX ||
                g->kst > INT32_MAX || g->sst > INT32_MAX))
        return false;
      if (L.ld < 0 || L.kst < 0 || L.sst < 0 || L.rs < 0) return false;
      if (rows <= 0 || K <= 0) return true;
      const int64_t rep = std::max(L.rep, 1), ks = L.ks > 0 ? L.ks : K;
      const int64_t off = (rows - 1) / rep * L.ld + std::min<int64_t>(rows - 1, rep - 1) * L.rs +
                          std::min<int64_t>(K - 1, ks - 1) * L.kst + (K - 1) / ks * L.sst;
      return off >= 0 && (off + 1) * 4 <= (int64_t)0x7fff0000;
    };
    const e3gnn_gemm_layouts* G = q.layout;
    const int64_t lds[4] = {q.lda, q.ldb, q.lda2, q.ldb2};
    for (int64_t v : lds)
      if (v < 0 || v > INT32_MAX) return fail(E3GNN_ERR_ARG, "e3gnn_gemm_grouped: leading dimension beyond int32");
    if (!fits(p.A1, q.m, q.k, G ? &G->a : nullptr) || !fits(p.B1, q.n, q.k, G ? &G->b : nullptr) ||
        (q.k2 > 0 && (!fits(p.A2, q.m, q.k2, G ? &G->a2 : nullptr) || !fits(p.B2, q.n, q.k2, G ? &G->b2 : nullptr))))
      return fail(E3GNN_ERR_ARG, "e3gnn_gemm_grouped: problem " + std::to_string(i) +
                                     " addresses an operand beyond 2 GB (32-bit buffer offsets)");
  }
  p.C = q.c;
  p.M = q.m; p.N = q.n; p.K1 = q.k; p.K2 = q.k2;
  p.alpha = q.alpha; p.beta = q.beta;
  p.kr = q.krange; p.kr_sm = q.krange_stride_m;
  p.splits = tg_splits(q.m, q.n, (int64_t)q.k + q.k2);
  return E3GNN_OK;
}

int e3gnn_gemm_grouped_ex(int n, const e3gnn_gemm_desc* d, float* workspace, int64_t workspace_floats,
                          int flags, void* stream) {
  if (n < 0 || n > TG_MAX_PROBS || (n > 0 && !d))
    return fail(E3GNN_ERR_ARG, "e3gnn_gemm_grouped: 0.." + std::to_string(TG_MAX_PROBS) + " problems");
  TgBatch b;
  int64_t used = 0;
  for (int i = 0; i < n; ++i) {
    TgProb p;
    if (int rc = gemm_prob(d[i], i, p)) return rc;
    if (p.splits > 1) {
      const int64_t need = (int64_t)p.splits * d[i].m * d[i].n;
      if (!workspace || used + need > workspace_floats)
        return fail(E3GNN_ERR_ARG, "e3gnn_gemm_grouped: workspace too small (e3gnn_gemm_workspace_floats)");
      p.ws = workspace + used;
      used += need;
    }
    if (!tg_add(b, p)) return fail(E3GNN_ERR_ARG, "e3gnn_gemm_grouped: problem " + std::to_string(i));
  }
  HIPCHK(launch_tgemm(b, (hipStream_t)stream, !(flags & E3GNN_GEMM_DEFER_REDUCE)));
  return E3GNN_OK;
}

int e3gnn_gemm_grouped(int n, const e3gnn_gemm_desc* d, float* workspace, int64_t workspace_floats,
                       void* stream) {
  return e3gnn_gemm_grouped_ex(n, d, workspace, workspace_floats, 0, stream);
}

int e3gnn_gemm_reduce(int n, const e3gnn_gemm_desc* d, float* const* workspaces, void* stream) {
  if (n < 0 || (n > 0 && (!d || !workspaces))) return fail(E3GNN_ERR_ARG, "e3gnn_gemm_reduce: bad arguments");
  TgRedBatch r;
  for (int i = 0; i < n; ++i) {
    TgProb p;
    if (int rc = gemm_prob(d[i], i, p)) return rc;
    if (p.splits <= 1 || p.M == 0 || p.N == 0) continue;   // reduced (or written) by its own launch
    {   // the split count its launch settled on (tg_add: whole k-step slices per split)
      TgBatch one;
      if (!tg_add(one, p)) return fail(E3GNN_ERR_ARG, "e3gnn_gemm_reduce: problem " + std::to_string(i));
      p = one.p[0];
      if (p.splits <= 1) continue;
    }
    if (!workspaces[i]) return fail(E3GNN_ERR_ARG, "e3gnn_gemm_reduce: problem " + std::to_string(i) + " has no slabs");
    if (r.n == TG_MAX_RED) {   // launches of TG_MAX_RED problems, in order
      HIPCHK(launch_tgemm_reduce(r, (hipStream_t)stream));
      r = TgRedBatch{};
    }
    tg_red_add(r, TgRed{workspaces[i], p.C, p.ldc, p.crep, p.crs, p.cns, p.M, p.N, p.splits, p.alpha, p.beta});
  }
  HIPCHK(launch_tgemm_reduce(r, (hipStream_t)stream));
  return E3GNN_OK;
}

int e3gnn_loss_efs(int criterion, float delta, int64_t nb, int64_t n, const float* e_pred,
                   const float* e_ref, const int64_t* natoms, const float* f_pred, const float* f_ref,
                   const float* s_pred, const float* s_ref, float w_e, float w_f, float w_s,
                   float s_scale, float* terms, float* ce, float* cf, float* cs, void* stream) {
  if (criterion != 0 && criterion != 1) return fail(E3GNN_ERR_ARG, "loss criterion must be 0 (mse) or 1 (huber)");
  if (nb < 0 || n < 0 || !terms || (nb > 0 && (!e_pred || !e_ref || !natoms || !ce)) ||
      (n > 0 && (!f_pred || !f_ref || !cf)) || (s_pred && (!s_ref || !cs)))
    return fail(E3GNN_ERR_ARG, "null loss operand");
  LossArgs a{criterion, delta, nb, n, e_pred, e_ref, natoms, f_pred, f_ref, s_pred, s_ref,
             w_e, w_f, w_s, s_scale, terms, ce, cf, cs};
  HIPCHK(launch_loss_efs(a, (hipStream_t)stream));
  return E3GNN_OK;
}

int e3gnn_ewc_flat(int64_t n, const float* theta, const float* f, const float* o, const float* f_train,
                   float lam, float* grad, float* part, float* value, void* stream) {
  if (n < 0 || (n > 0 && (!theta || !f || !o || !part || (grad && !f_train))) || !value)
    return fail(E3GNN_ERR_ARG, "null EWC operand");
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(launch_ewc_flat(n, theta, f, o, f_train, lam, grad, part, s));
  // fixed-order block sums into part[n ...], then their sum (node.hip launch_sum)
  HIPCHK(launch_sum(n, part, part + n, value, s));
  return E3GNN_OK;
}

int e3gnn_model_family(const e3gnn_model* m) {
  if (!m) return fail(E3GNN_ERR_ARG, "null model"), -1;
  return m->gen ? -1 : m->family;
}

e3gnn_ctx* e3gnn_ctx_create(e3gnn_model* m) {
  if (!m) {
    fail(E3GNN_ERR_ARG, "null model");
    return nullptr;
  }
  auto c = new e3gnn_ctx();
  c->m = m;
  if (m->gen) c->gen = gen_ctx_create(m->gen);
  const int L = m->nlayer;
  c->x.resize(L + 1);
  c->grad.resize(L + 1);
  c->h.resize(L);
  c->y.resize(L);
  c->w.resize(L);
  c->a1.resize(L);
  c->a2.resize(L);
  return c;
}
void e3gnn_ctx_free(e3gnn_ctx* c) { delete c; }

int e3gnn_feature_dim(const e3gnn_ctx* c, int layer) {
  if (!c || layer < 0 || layer > c->m->nlayer) return -1;
  if (c->m->gen) return gen_feature_dim(c->m->gen, layer);
  return irreps_dim(c->m->irreps[layer]);
}
float* e3gnn_feature_ptr(e3gnn_ctx* c, int layer) {
  if (!c || layer < 0 || layer > c->m->nlayer) return nullptr;
  if (c->gen) return gen_x(c->gen, layer);
  return c->x[layer].f();
}
float* e3gnn_grad_ptr(e3gnn_ctx* c, int layer) {
  if (!c || layer < 0 || layer > c->m->nlayer) return nullptr;
  if (c->gen) return gen_grad(c->gen, layer);
  return c->grad[layer].f();
}

int e3gnn_graph_set(e3gnn_ctx* c, int64_t n_local, int64_t n_ghost, int64_t n_edges,
                    const int32_t* type, const int32_t* edge_center, const int32_t* edge_nbr,
                    const float* edge_vec, void* stream) {
  if (!c) return fail(E3GNN_ERR_ARG, "null context");
  if (n_local < 0 || n_ghost < 0 || n_edges < 0) return fail(E3GNN_ERR_ARG, "negative size");
  if (n_local + n_ghost > (1LL << 30) || n_edges > (1LL << 31) - 1)
    return fail(E3GNN_ERR_ARG, "graph too large for int32 indices");
  // the fused kernels gather node-feature rows through one 32-bit buffer
  // descriptor (n x DX fp32 < 2 GiB: 1.1M atoms at SevenNet-0's 480; the last
  // block's dE/dagg rows fit whenever these do)
  if (!c->gen && (n_local + n_ghost) * (int64_t)c->m->max_dx * 4 > 0x7fffffffLL)
    return fail(E3GNN_ERR_ARG, "more than " + std::to_string(0x7fffffffLL / (4LL * c->m->max_dx)) +
                                   " atoms (owned + ghost) per device for this model: shard the system");
  if (!c->gen && c->impl == 1 && c->m->family != 0)
    return fail(E3GNN_ERR_ARG, "the v1 (unfused) kernels serve SevenNet-0's channel family only");
  if ((n_local + n_ghost > 0 && !type) || (n_edges > 0 && (!edge_center || !edge_nbr || !edge_vec)))
    return fail(E3GNN_ERR_ARG, "null input array");
  e3gnn_model* m = c->m;
  HIPCHK(hipSetDevice(m->device));
  hipStream_t s = (hipStream_t)stream;
  if (c->done_pending && c->done_stream != s) HIPCHK(hipStreamWaitEvent(s, c->done_ev, 0));
  c->done_pending = false;
  const int64_t n = n_local + n_ghost, nl = n_local, E = n_edges;
  c->n = n;
  c->nl = nl;
  c->E = E;
  c->readout_done = 0;
  if (c->n_interior_req > nl) return fail(E3GNN_ERR_ARG, "n_interior exceeds n_local");
  c->n_int = c->n_interior_req;
  c->e_int = 0;
  const size_t F = sizeof(float);
  // workspace (grow-only)
  HIPCHK(c->type.ensure(n * 4));
  HIPCHK(c->center.ensure(E * 4));
  HIPCHK(c->nbr.ensure(E * 4));
  HIPCHK(c->vec.ensure(E * 3 * F));
  HIPCHK(c->row_ptr.ensure((nl + 1) * 4));
  HIPCHK(c->src_ptr.ensure((n + 1) * 4));
  HIPCHK(c->src_perm.ensure(E * 4));
  HIPCHK(c->cnt.ensure(n * 4));
  HIPCHK(c->err.ensure(4));
  if (!c->gen) {
    HIPCHK(c->Y.ensure(E * 9 * F));
    HIPCHK(c->emb.ensure(E * 8 * F));
    HIPCHK(c->dY.ensure(E * 9 * F));
    HIPCHK(c->demb.ensure(E * 8 * F));
    HIPCHK(c->fe.ensure(E * 3 * F));
    HIPCHK(c->dgu.ensure(E * 3 * F));
    const bool v1 = c->impl == 1;
    c->graph_impl = c->impl;
    if (v1) {
      HIPCHK(c->H1.ensure(E * 64 * F));
      HIPCHK(c->H2.ensure(E * 64 * F));
    }
    int maxW = 0, maxDM = 0;
    for (int t = 0; t < m->nlayer; ++t) {
      const int dx = irreps_dim(m->irreps[t]), dg = irreps_dim(m->gin[t]);
      maxW = std::max(maxW, m->W[t]);
      maxDM = std::max(maxDM, irreps_dim(m->mid[t]));
      HIPCHK(c->x[t].ensure(std::max<int64_t>(n, 1) * dx * F));
      HIPCHK(c->grad[t].ensure(std::max<int64_t>(n, 1) * dx * F));
      HIPCHK(c->h[t].ensure(n * dx * F));
      HIPCHK(c->y[t].ensure(nl * dg * F));
      if (v1) {
        HIPCHK(c->w[t].ensure(E * m->W[t] * F));
        HIPCHK(c->a1[t].ensure(E * 64 * F));
        HIPCHK(c->a2[t].ensure(E * 64 * F));
      }
    }
    const int dlast = irreps_dim(m->irreps[m->nlayer]);
    HIPCHK(c->x[m->nlayer].ensure(std::max<int64_t>(n, 1) * dlast * F));
    HIPCHK(c->grad[m->nlayer].ensure(std::max<int64_t>(n, 1) * dlast * F));
    HIPCHK(c->agg.ensure(nl * maxDM * F));
    if (v1) HIPCHK(c->dw.ensure(E * maxW * F));
    HIPCHK(c->dxc.ensure(E * m->max_dx * F));
    HIPCHK(c->dy.ensure(nl * m->max_dg * F));
    HIPCHK(c->dh.ensure(n * m->max_dx * F));
    HIPCHK(c->eat.ensure(std::max<int64_t>(nl, 1) * F));
    HIPCHK(c->part.ensure((sum_blocks(nl) + 1) * F));
    HIPCHK(c->vpart.ensure((edge_force_blocks(E) + 1) * 6 * F));
    HIPCHK(c->scratch6.ensure(8 * F));

  }
  if (n > 0) HIPCHK(hipMemcpyAsync(c->type.p, type, n * 4, hipMemcpyDefault, s));
  if (E > 0) {
    HIPCHK(hipMemcpyAsync(c->center.p, edge_center, E * 4, hipMemcpyDefault, s));
    HIPCHK(hipMemcpyAsync(c->nbr.p, edge_nbr, E * 4, hipMemcpyDefault, s));
    HIPCHK(hipMemcpyAsync(c->vec.p, edge_vec, E * 3 * F, hipMemcpyDefault, s));
  }
  HIPCHK(hipMemsetAsync(c->err.p, 0, 4, s));
  {
    Region r(c, s, C_GRAPH, 0, (double)E * 24 + n * 12);
    HIPCHK(launch_build_graph(E, (int)nl, (int)n, c->center.i(), c->nbr.i(), c->row_ptr.i(),
                              c->src_ptr.i(), c->src_perm.i(), c->cnt.i(), c->err.i(), s,
                              (int)c->n_int));
  }
  if (c->gen) {
    HIPCHK(gen_graph_set(c->gen, m->gen, gen_graph(c), s));
  } else {
    const int d0 = irreps_dim(m->irreps[0]);
    Region r(c, s, C_EMBED_NODE, 0, (double)n * d0 * 4);
    HIPCHK(launch_embed((int)n, d0, c->type.i(), m->nsp, m->embed.f(), c->x[0].f(), c->err.i(), s));
  }
  int err = 0, e_int = 0;
  HIPCHK(hipMemcpyAsync(&err, c->err.p, 4, hipMemcpyDeviceToHost, s));
  if (c->n_int > 0)
    HIPCHK(hipMemcpyAsync(&e_int, c->row_ptr.i() + c->n_int, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  c->e_int = e_int;
  if (err) {
    std::string msg = "invalid graph:";
    if (err & 1) msg += " edge_center not sorted non-decreasing;";
    if (err & 2) msg += " edge_center out of [0, n_local);";
    if (err & 4) msg += " edge_nbr out of [0, n_local+n_ghost);";
    if (err & 8) msg += " species index out of range;";
    if (err & 16) msg += " an interior centre (below n_interior) has a ghost neighbour;";
    return fail(E3GNN_ERR_GRAPH, msg);
  }
  if (c->gen) return E3GNN_OK;  // (edge embedding done by gen_graph_set)
  {
    Region r(c, s, C_EMBED_EDGE, 0, (double)E * (12 + 68));
    HIPCHK(launch_edge_embed(E, c->vec.f(), m->coeffs.f(), m->cutoff, m->r_on, m->raw_sh, c->Y.f(),
                             c->emb.f(), s));
  }
  if (E > 0) {
    // zero kernels, not hipMemsetAsync: the evaluation stays correct when a
    // host captures it in a HIP graph (launch_zero, node.hip)
    HIPCHK(launch_zero(c->dY.f(), E * 9, s));
    HIPCHK(launch_zero(c->dgu.f(), E * 3, s));
    HIPCHK(launch_zero(c->demb.f(), E * 8, s));
  }
  return E3GNN_OK;
}

// Parts of one interaction block for the halo overlap (e3gnn.h):
// part 0 needs only the owned rows of the block's input features (it runs
// while the ghost rows are in flight): self_interaction_1 of the owned rows and
// the convolution of the interior centres [0, n_int); part 1: the ghost rows'
// self_interaction_1, the boundary centres [n_int, n_local), si2 +
// self-connection + gate.  The v1 kernels run whole in part 1.
int e3gnn_layer_forward_part(e3gnn_ctx* c, int t, int part, void* stream) {
  if (!c) return fail(E3GNN_ERR_ARG, "null context");
  e3gnn_model* m = c->m;
  if (t < 0 || t >= m->nlayer) return fail(E3GNN_ERR_ARG, "layer out of range");
  if (part != 0 && part != 1) return fail(E3GNN_ERR_ARG, "part must be 0 or 1");
  HIPCHK(hipSetDevice(m->device));
  hipStream_t s = (hipStream_t)stream;
  // generic engine: the whole layer after the halo of x[t] (part 1)
  if (c->gen) {
    if (part == 1) HIPCHK(gen_layer_forward(c->gen, m->gen, gen_graph(c), t, s));
    return E3GNN_OK;
  }
  const int64_t n = c->n, nl = c->nl, E = c->E;
  const int dx = irreps_dim(m->irreps[t]), dg = irreps_dim(m->gin[t]);
  const int dm = irreps_dim(m->mid[t]), W = m->W[t];
  const bool last = t == m->nlayer - 1;
  const int kind = t == 0 ? 0 : (last ? 2 : 1);   // block kind (timing class, v1 kernels)
  const int code = m->kcode(t);                    // fused kernel kind code
  const bool fused = c->graph_impl == 0;
  const int64_t n_int = fused ? c->n_int : 0;
  auto conv_fwd = [&](int64_t c0, int64_t c1, double e_share) -> int {
    if (c1 <= c0) return E3GNN_OK;
    Region r(c, s, C_CONV_FWD + kind,
             e_share * (tp_flops_per_edge(code) + 2.0 * (8 * 64 + 64 * 64 + 64 * W)),
             e_share * 4 * (8 + 9 + 2 + dx) + (c1 - c0) * 4.0 * dm);
    FusedArgs a;
    std::memset(&a, 0, sizeof(a));
    a.row_ptr = c->row_ptr.i();
    a.nbr = c->nbr.i();
    a.emb = c->emb.f();
    a.Y = c->Y.f();
    a.h = c->h[t].f();
    a.agg = c->agg.f();
    a.W = mlp_ptrs(m, t);
    a.n_centers = (int)nl;
    a.n_nodes = (int)n;
    a.denom = m->denom[t];
    a.c_begin = (int)c0;
    a.c_end = (int)c1;
    HIPCHK(launch_conv_fwd(code, a, s));
    return E3GNN_OK;
  };
  if (part == 0) {
    if (!fused) return E3GNN_OK;
    {
      Region r(c, s, C_LINEAR, lin_flops(*m->si1[t], nl));
      NlBatch nb;
      if (c->nodelin && nl_batch(nb, *m->nl_si1[t], c->x[t].f(), dx, nullptr, 0, c->h[t].f(), dx, nl, 0))
        HIPCHK(launch_nodelin(nb, s));
      else
        HIPCHK(launch_gemm(lin_fwd(*m->si1[t], c->x[t].f(), dx, c->h[t].f(), dx, nl, 0), s));
    }
    return conv_fwd(0, n_int, (double)c->e_int);
  }
  // ---- part 1
  {
    const int64_t r0 = fused ? nl : 0;  // rows not done in part 0
    Region r(c, s, C_LINEAR, lin_flops(*m->si1[t], n - r0));
    NlBatch nb;
    if (n > r0 && c->nodelin &&
        nl_batch(nb, *m->nl_si1[t], c->x[t].f() + r0 * dx, dx, nullptr, 0, c->h[t].f() + r0 * dx, dx,
                 n - r0, 0))
      HIPCHK(launch_nodelin(nb, s));
    else if (n > r0)
      HIPCHK(launch_gemm(lin_fwd(*m->si1[t], c->x[t].f() + r0 * dx, dx, c->h[t].f() + r0 * dx, dx,
                                 n - r0, 0), s));
  }
  if (fused) {
    // fused radial MLP + tensor product + segmented sum (fused.hip)
    const int rc = conv_fwd(n_int, nl, (double)(E - c->e_int));
    if (rc) return rc;
  } else {
  // radial MLP: emb -> 64 -> 64 -> W  (convolution.py:97-106)
  {
    Region r(c, s, C_MLP_FWD, 2.0 * E * (8 * 64 + 64 * 64 + 64 * W),
             (double)E * 4 * (8 + 64 * 4 + 2 * 64 + W));
    auto& mm = m->mlp[t];
    GemmBatch b;
    std::memset(&b, 0, sizeof(b));
    GemmProb p = base_prob();
    p.A = c->emb.f(); p.lda = 8; p.K = 8;
    p.B = mm.w0.f(); p.ldb = 64; p.N = 64;
    p.C = c->H1.f(); p.ldc = 64; p.M = (int)E;
    p.act = 1; p.pre_out = c->a1[t].f();
    add_prob(b, p);
    HIPCHK(launch_gemm(b, s));
    std::memset(&b, 0, sizeof(b));
    p.A = c->H1.f(); p.lda = 64; p.K = 64;
    p.B = mm.w1.f(); p.C = c->H2.f(); p.pre_out = c->a2[t].f();
    add_prob(b, p);
    HIPCHK(launch_gemm(b, s));
    std::memset(&b, 0, sizeof(b));
    p.A = c->H2.f(); p.B = mm.w2.f(); p.ldb = W; p.N = W;
    p.C = c->w[t].f(); p.ldc = W; p.act = 0; p.pre_out = nullptr;
    add_prob(b, p);
    HIPCHK(launch_gemm(b, s));
  }
  // tensor product + segmented neighbour sum
  {
    Region r(c, s, C_TP_FWD, tp_flops_per_edge(code) * E,
             (double)E * 4 * (W + 9 + dx + 2) + nl * 4.0 * dm);
    TpArgs a;
    std::memset(&a, 0, sizeof(a));
    a.row_ptr = c->row_ptr.i();
    a.nbr = c->nbr.i();
    a.Y = c->Y.f();
    a.w = c->w[t].f();
    a.h = c->h[t].f();
    a.agg = c->agg.f();
    a.n_centers = (int)nl;
    a.denom = m->denom[t];
    HIPCHK(launch_tp_fwd(kind, a, s));
  }
  }
  // self_interaction_2 + self_connection (intro/outro) + gate: on k_nodelin
  // one K-concatenated problem per output block, the 0e block first (its
  // epilogue activates the scalars and stores the gate pre-activations), then
  // the gated blocks (epilogue: x = act(gate) * y)
  {
    const Irreps& gin = m->gin[t];
    const Irreps& xo = m->irreps[t + 1];
    int nscal = 0;
    for (auto& i : xo)
      if (i.l == 0) nscal += i.mul;
    const bool gate_ok = !gin.empty() && gin[0].l == 0 && !xo.empty() && xo[0].l == 0;
    auto gate_fix = [&](NlProb& q, const PairBlock& k) {
      q.xo = c->x[t + 1].f();
      q.ldxo = irreps_dim(xo);
      if (k.l == 0) {
        q.n_act = nscal;
        return;
      }
      int off = gin[0].mul, gmul = 0, gdim = 0;
      for (size_t i = 1; i < gin.size() && off != k.out_off; ++i) {
        gmul += gin[i].mul;
        gdim += gin[i].mul * (2 * gin[i].l + 1);
        off += gin[i].mul * (2 * gin[i].l + 1);
      }
      q.gate_off = nscal + gmul;
      q.xo_off = nscal + gdim;
    };
    NlBatch b0, b1;
    if (c->nodelin && gate_ok &&
        nl_batch(b0, *m->nl_fwd[t], c->agg.f(), dm, c->x[t].f(), dx, c->y[t].f(), dg, nl, 2, 1, gate_fix) &&
        nl_batch(b1, *m->nl_fwd[t], c->agg.f(), dm, c->x[t].f(), dx, c->y[t].f(), dg, nl, 3, 2, gate_fix)) {
      Region r(c, s, C_LINEAR, pair_flops(*m->nl_fwd[t], nl));
      HIPCHK(launch_nodelin(b0, s));
      HIPCHK(launch_nodelin(b1, s));
      return E3GNN_OK;
    }
  }
  {
    Region r(c, s, C_LINEAR, lin_flops(*m->si2[t], nl) + lin_flops(*m->sc[t], nl));
    HIPCHK(launch_gemm(lin_fwd(*m->si2[t], c->agg.f(), dm, c->y[t].f(), dg, nl, 0), s));
    HIPCHK(launch_gemm(lin_fwd(*m->sc[t], c->x[t].f(), dx, c->y[t].f(), dg, nl, 1), s));
  }
  {
    Region r(c, s, C_GATE_FWD, 0, nl * 4.0 * (dg + irreps_dim(m->irreps[t + 1])));
    HIPCHK(launch_gate_fwd((int)nl, last, m->gdims[t], c->y[t].f(), c->x[t + 1].f(), s));
  }
  return E3GNN_OK;
}

int e3gnn_layer_forward(e3gnn_ctx* c, int t, void* stream) {
  const int rc = e3gnn_layer_forward_part(c, t, 0, stream);
  return rc ? rc : e3gnn_layer_forward_part(c, t, 1, stream);
}

int e3gnn_readout(e3gnn_ctx* c, float* energy, float* atomic_energy, void* stream) {
  if (!c) return fail(E3GNN_ERR_ARG, "null context");
  e3gnn_model* m = c->m;
  HIPCHK(hipSetDevice(m->device));
  hipStream_t s = (hipStream_t)stream;
  if (c->gen) {
    HIPCHK(gen_readout(c->gen, m->gen, gen_graph(c), energy, atomic_energy, s));
    c->readout_done = 1;
    return E3GNN_OK;
  }
  const int64_t nl = c->nl;
  const int L = m->nlayer;
  {
    const int dl = irreps_dim(m->irreps[L]);
    Region r(c, s, C_READOUT, 2.0 * nl * dl, nl * 4.0 * (dl + 2));
    HIPCHK(launch_readout((int)nl, dl, c->x[L].f(), m->readout_v.f(), c->type.i(), m->scale.f(),
                          m->shift.f(), c->eat.f(), s));
    HIPCHK(launch_sum(nl, c->eat.f(), c->part.f(), energy ? energy : c->scratch6.f(), s));
    if (atomic_energy && nl > 0)
      HIPCHK(hipMemcpyAsync(atomic_energy, c->eat.p, nl * 4, hipMemcpyDeviceToDevice, s));
    HIPCHK(launch_readout_bwd((int)nl, dl, m->readout_v.f(), c->type.i(), m->scale.f(),
                              c->grad[L].f(), s));
  }
  c->readout_done = 1;
  return E3GNN_OK;
}

// Parts of a block's backward for the halo overlap (e3gnn.h): part 0 makes
// everything the GHOST rows of dE/dx need (gate + si2 backward of the owned
// rows, the boundary centres' edges, the ghost rows' gather and
// self_interaction_1 backward), so the reverse exchange can start; part 1 does
// the interior centres and the owned rows.  The v1 kernels run whole in part 0.
int e3gnn_layer_backward_part(e3gnn_ctx* c, int t, int part, void* stream) {
  if (!c) return fail(E3GNN_ERR_ARG, "null context");
  e3gnn_model* m = c->m;
  if (t < 0 || t >= m->nlayer) return fail(E3GNN_ERR_ARG, "layer out of range");
  if (part != 0 && part != 1) return fail(E3GNN_ERR_ARG, "part must be 0 or 1");
  if (!c->readout_done) return fail(E3GNN_ERR_ARG, "e3gnn_readout must precede the backward");
  HIPCHK(hipSetDevice(m->device));
  hipStream_t s = (hipStream_t)stream;
  // generic engine: the whole layer before the reverse halo of dE/dx[t] (part 0)
  if (c->gen) {
    if (part == 0) HIPCHK(gen_layer_backward(c->gen, m->gen, gen_graph(c), t, s));
    return E3GNN_OK;
  }
  const int64_t n = c->n, nl = c->nl, E = c->E;
  const int dx = irreps_dim(m->irreps[t]), dg = irreps_dim(m->gin[t]);
  const int dm = irreps_dim(m->mid[t]), W = m->W[t];
  const bool last = t == m->nlayer - 1;
  const int kind = t == 0 ? 0 : (last ? 2 : 1);   // block kind (timing class, v1 kernels)
  const int code = m->kcode(t);                    // fused kernel kind code
  const bool fused = c->graph_impl == 0;
  if (!fused && part == 1) return E3GNN_OK;
  const int64_t n_int = c->n_int, e_int = c->e_int;
  if (part == 0) {
    {
      Region r(c, s, C_GATE_BWD, 0, nl * 4.0 * (2 * dg + irreps_dim(m->irreps[t + 1])));
      HIPCHK(launch_gate_bwd((int)nl, last, m->gdims[t], c->y[t].f(), c->grad[t + 1].f(), c->dy.f(), s));
    }
    {
      Region r(c, s, C_LINEAR, lin_flops(*m->si2[t], nl));
      NlBatch nb;
      if (c->nodelin && nl_batch(nb, *m->nl_si2t[t], c->dy.f(), dg, nullptr, 0, c->agg.f(), dm, nl, 0))
        HIPCHK(launch_nodelin(nb, s));
      else
        HIPCHK(launch_gemm(lin_bwd(*m->si2[t], c->dy.f(), dg, c->agg.f(), dm, nl, 0), s));
    }
  }
  // first / middle blocks: per-edge dE/dx (dxc) + transposed-CSR gather; the
  // last block (224 message channels) writes dE/dx per neighbour node
  const bool gather = !fused || !last;
  if (fused) {
    FusedArgs a;
    std::memset(&a, 0, sizeof(a));
    a.row_ptr = c->row_ptr.i();
    a.nbr = c->nbr.i();
    a.emb = c->emb.f();
    a.Y = c->Y.f();
    a.h = c->h[t].f();
    a.gagg = c->agg.f();
    a.center = c->center.i();
    a.n_edges = (int)E;
    a.src_ptr = c->src_ptr.i();
    a.src_perm = c->src_perm.i();
    a.dh = c->dh.f();  // the last block writes its dE/dx rows here
    a.dxc = (!last && t > 0) ? c->dxc.f() : nullptr;
    a.dgu = c->dgu.f();
    a.demb = c->demb.f();
    a.W = mlp_ptrs(m, t);
    a.n_centers = (int)nl;
    a.n_nodes = (int)n;
    // part 0: boundary centres / their edges / ghost neighbour nodes
    a.c_begin = (int)(part == 0 ? n_int : 0);
    a.c_end = (int)(part == 0 ? nl : n_int);
    a.node_begin = (int)(part == 0 ? nl : 0);
    a.node_end = (int)(part == 0 ? n : nl);
    double ef = (double)(part == 0 ? E - e_int : e_int);
    if (last && c->timing && a.node_end > a.node_begin) {
      // the last block's launch covers the edges of its neighbour-node range
      int32_t q[2];
      HIPCHK(hipMemcpyAsync(&q[0], a.src_ptr + a.node_begin, 4, hipMemcpyDeviceToHost, s));
      HIPCHK(hipMemcpyAsync(&q[1], a.src_ptr + a.node_end, 4, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      ef = (double)(q[1] - q[0]);
    }
    // empty ranges launch nothing (and are not counted as launches)
    if (last ? a.node_end > a.node_begin : a.c_end > a.c_begin) {
      // algorithmic FLOP (the forward radial MLP the kernel recomputes is not
      // counted): dE/dx + dE/dY = 2 x TP; dE/dw = TP, dH2 = dw W2^T, MLP chain
      const double xf = 3.0 * tp_flops_per_edge(code) + 2.0 * (64 * W + 64 * 64 + 8 * 64);
      Region r(c, s, C_CONV_BWD_X + kind, xf * ef,
               ef * 4 * (8 + 9 + 2 + 3 + 8) + (a.c_end - a.c_begin) * 4.0 * dm);
      HIPCHK(last ? launch_conv_bwd_nbr_last(code, a, s) : launch_conv_bwd_ls(code, a, s));
    }
  } else {
  {
    Region r(c, s, C_TP_BWD, 3.0 * tp_flops_per_edge(code) * E,
             (double)E * 4 * (2 * W + 2 * 9 + dx + (t > 0 ? dx : 0) + 2) + nl * 4.0 * dm);
    TpArgs a;
    std::memset(&a, 0, sizeof(a));
    a.row_ptr = c->row_ptr.i();
    a.nbr = c->nbr.i();
    a.Y = c->Y.f();
    a.w = c->w[t].f();
    a.h = c->h[t].f();
    a.gagg = c->agg.f();
    a.dw = c->dw.f();
    a.dxc = t > 0 ? c->dxc.f() : nullptr;
    a.dYacc = c->dY.f();
    a.n_centers = (int)nl;
    HIPCHK(launch_tp_bwd(kind, a, s));
  }
  {
    Region r(c, s, C_MLP_BWD, 2.0 * E * (64 * W + 64 * 64 + 64 * 8),
             (double)E * 4 * (W + 64 * 6 + 16));
    auto& mm = m->mlp[t];
    GemmBatch b;
    std::memset(&b, 0, sizeof(b));
    GemmProb p = base_prob();
    p.A = c->dw.f(); p.lda = W; p.K = W;
    p.B = mm.w2t.f(); p.ldb = 64; p.N = 64;
    p.C = c->H2.f(); p.ldc = 64; p.M = (int)E;
    p.act = 2; p.pre_in = c->a2[t].f();
    add_prob(b, p);
    HIPCHK(launch_gemm(b, s));
    std::memset(&b, 0, sizeof(b));
    p.A = c->H2.f(); p.lda = 64; p.K = 64;
    p.B = mm.w1t.f(); p.C = c->H1.f(); p.pre_in = c->a1[t].f();
    add_prob(b, p);
    HIPCHK(launch_gemm(b, s));
    std::memset(&b, 0, sizeof(b));
    p.A = c->H1.f(); p.B = mm.w0t.f(); p.ldb = 8; p.N = 8;
    p.C = c->demb.f(); p.ldc = 8; p.act = 0; p.pre_in = nullptr; p.beta = 1;
    add_prob(b, p);
    HIPCHK(launch_gemm(b, s));
  }
  }
  if (t > 0) {
    // rows of this part: ghosts [nl, n) in part 0, owned [0, nl) in part 1
    // (the v1 kernels: all rows, in part 0)
    const int64_t r0 = !fused ? 0 : (part == 0 ? nl : 0), r1 = !fused ? n : (part == 0 ? n : nl);
    if (gather && r1 > r0) {
      Region r(c, s, C_GATHER, 0, (double)E * 4 * (dx + 1) * (r1 - r0) / std::max<int64_t>(n, 1) +
                                      (r1 - r0) * 4.0 * dx);
      HIPCHK(launch_gather_rows_range((int)r0, (int)r1, dx, c->src_ptr.i(), c->src_perm.i(),
                                      c->dxc.f(), c->dh.f(), s));
    }
    const bool owned = !fused || part == 1;
    Region r(c, s, C_LINEAR, lin_flops(*m->si1[t], r1 - r0) + (owned ? lin_flops(*m->sc[t], nl) : 0));
    // k_nodelin: owned rows [0, nl) as one si1^T + sc^T problem per block,
    // the remaining rows (ghosts) si1^T alone
    NlBatch b0, b1;
    const int64_t p1 = owned ? nl : r0;  // first row of the si1^T-only range
    if (c->nodelin && (!owned || r0 == 0) && r1 >= p1 &&
        (!owned || nl_batch(b0, *m->nl_bwd[t], c->dh.f(), dx, c->dy.f(), dg, c->grad[t].f(), dx, nl, 0)) &&
        (r1 == p1 || nl_batch(b1, *m->nl_si1t[t], c->dh.f() + p1 * dx, dx, nullptr, 0,
                              c->grad[t].f() + p1 * dx, dx, r1 - p1, 0))) {
      if (owned) HIPCHK(launch_nodelin(b0, s));
      if (r1 > p1) HIPCHK(launch_nodelin(b1, s));
    } else {
      if (r1 > r0)
        HIPCHK(launch_gemm(lin_bwd(*m->si1[t], c->dh.f() + r0 * dx, dx, c->grad[t].f() + r0 * dx, dx,
                                   r1 - r0, 0), s));
      if (owned) HIPCHK(launch_gemm(lin_bwd(*m->sc[t], c->dy.f(), dg, c->grad[t].f(), dx, nl, 1), s));
    }
  }
  return E3GNN_OK;
}

int e3gnn_layer_backward(e3gnn_ctx* c, int t, void* stream) {
  const int rc = e3gnn_layer_backward_part(c, t, 0, stream);
  return rc ? rc : e3gnn_layer_backward_part(c, t, 1, stream);
}

int e3gnn_forces(e3gnn_ctx* c, float* forces, float* virial6, float* edge_grad, void* stream) {
  if (!c) return fail(E3GNN_ERR_ARG, "null context");
  e3gnn_model* m = c->m;
  HIPCHK(hipSetDevice(m->device));
  hipStream_t s = (hipStream_t)stream;
  if (c->gen) {
    HIPCHK(gen_forces(c->gen, m->gen, gen_graph(c), forces, virial6, edge_grad, s));
    return E3GNN_OK;
  }
  const int64_t n = c->n, nl = c->nl, E = c->E;
  {
    Region r(c, s, C_EDGE_FORCE, 0, (double)E * 4 * (3 + 9 + 8 + 3));
    HIPCHK(launch_edge_force(E, c->vec.f(), m->coeffs.f(), m->cutoff, m->r_on, m->raw_sh, c->dY.f(),
                             c->dgu.f(), c->demb.f(), c->fe.f(), c->vpart.f(), s));
    HIPCHK(launch_final_sum(edge_force_blocks(E), 6, c->vpart.f(),
                            virial6 ? virial6 : c->scratch6.f(), s));
  }
  if (forces) {
    Region r(c, s, C_ATOM_FORCE, 0, (double)E * 4 * 2 * 4 + n * 12.0);
    HIPCHK(launch_atom_force((int)n, (int)nl, c->row_ptr.i(), c->src_ptr.i(), c->src_perm.i(),
                             c->fe.f(), forces, s));
  }
  if (edge_grad && E > 0)
    HIPCHK(hipMemcpyAsync(edge_grad, c->fe.p, E * 12, hipMemcpyDeviceToDevice, s));
  return E3GNN_OK;
}

int e3gnn_energy_forces(e3gnn_ctx* c, int64_t n_atoms, int64_t n_edges, const int32_t* type,
                        const int32_t* edge_center, const int32_t* edge_nbr,
                        const float* edge_vec, float* energy, float* atomic_energy,
                        float* forces, float* virial6, float* edge_grad, void* stream) {
  if (!energy) return fail(E3GNN_ERR_ARG, "energy output is required");
  int rc = e3gnn_graph_set(c, n_atoms, 0, n_edges, type, edge_center, edge_nbr, edge_vec, stream);
  if (rc) return rc;
  const int L = c->m->nlayer;
  for (int t = 0; t < L; ++t)
    if ((rc = e3gnn_layer_forward(c, t, stream))) return rc;
  if ((rc = e3gnn_readout(c, energy, atomic_energy, stream))) return rc;
  for (int t = L - 1; t >= 0; --t)
    if ((rc = e3gnn_layer_backward(c, t, stream))) return rc;
  if ((rc = e3gnn_forces(c, forces, virial6, edge_grad, stream))) return rc;
  if (!c->stream_ordered) {
    HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  } else {
    if (!c->done_ev) HIPCHK(hipEventCreateWithFlags(&c->done_ev, hipEventDisableTiming));
    HIPCHK(hipEventRecord(c->done_ev, (hipStream_t)stream));
    c->done_stream = (hipStream_t)stream;
    c->done_pending = true;
  }
  return E3GNN_OK;
}

int e3gnn_halo_pack(const int32_t* idx, int64_t n, int dim, const float* src, int64_t src_stride,
                    float* dst, void* stream) {
  if (n < 0 || dim <= 0) return fail(E3GNN_ERR_ARG, "bad halo size");
  HIPCHK(launch_pack(n, dim, idx, src, src_stride, dst, (hipStream_t)stream));
  return E3GNN_OK;
}
int e3gnn_halo_unpack(const int32_t* idx, int64_t n, int dim, const float* src, float* dst,
                      int64_t dst_stride, int accumulate, void* stream) {
  if (n < 0 || dim <= 0) return fail(E3GNN_ERR_ARG, "bad halo size");
  HIPCHK(launch_unpack(n, dim, idx, src, dst, dst_stride, accumulate, (hipStream_t)stream));
  return E3GNN_OK;
}

// ------------------------------------------------------------ training ops
// Stateless convolution primitives over caller-owned device tensors, the
// kernel side of the fine-tune step (sevenn/train/trainer.py:155-222): the
// uvu tensor product + segmented sum (convolution.py:104-123) and its
// gradients w.r.t. all three operands.  The product is trilinear in
// (h, Y, w), so every derivative of any order is one of these two launches
// with permuted operands (sevennet_finetuning_amd/conv_ops.py).
namespace {
bool conv_kind_dims(int kind, int* dx, int* w, int* dm) {
  switch (kind) {
    case 0: *dx = LayerFirst::DX; *w = LayerFirst::W; *dm = LayerFirst::DM; return true;
    case 1: *dx = LayerMid::DX; *w = LayerMid::W; *dm = LayerMid::DM; return true;
    case 2: *dx = LayerLast::DX; *w = LayerLast::W; *dm = LayerLast::DM; return true;
    default: return false;
  }
}
}  // namespace

int e3gnn_conv_dims(int kind, int* dx, int* w, int* dm) {
  int a, b, d;
  if (!conv_kind_dims(kind, &a, &b, &d)) return fail(E3GNN_ERR_ARG, "conv kind must be 0, 1 or 2");
  if (dx) *dx = a;
  if (w) *w = b;
  if (dm) *dm = d;
  return E3GNN_OK;
}

static int graph_check(int* err_d, hipStream_t s);   // reads the build's error bits (synchronises)

int e3gnn_conv_graph(int64_t n_nodes, int64_t n_edges, const int32_t* edge_center,
                     const int32_t* edge_nbr, int32_t* row_ptr, int32_t* src_ptr,
                     int32_t* src_perm, int32_t* scratch, void* stream) {
  if (n_nodes < 0 || n_edges < 0 || n_nodes >= (int64_t)1 << 31 || n_edges >= (int64_t)1 << 31)
    return fail(E3GNN_ERR_ARG, "conv graph size out of int32 range");
  if (!row_ptr || !src_ptr || !scratch || (n_edges > 0 && (!edge_center || !edge_nbr || !src_perm)))
    return fail(E3GNN_ERR_ARG, "null conv graph buffer");
  hipStream_t s = (hipStream_t)stream;
  int* err_d = scratch + n_nodes;
  if (n_nodes <= graph_small_max_nodes() && n_edges <= graph_small_max_edges()) {   // one workgroup, one launch
    HIPCHK(launch_build_graph_small(n_edges, (int)n_nodes, edge_center, edge_nbr, nullptr, nullptr, nullptr,
                                    nullptr, row_ptr, src_ptr, src_perm, err_d, s));
  } else {
    HIPCHK(hipMemsetAsync(err_d, 0, 4, s));
    HIPCHK(launch_build_graph(n_edges, (int)n_nodes, (int)n_nodes, edge_center, edge_nbr, row_ptr,
                              src_ptr, src_perm, scratch, err_d, s));
  }
  return graph_check(err_d, s);
}

int e3gnn_conv_graph_i64(int64_t n_nodes, int64_t n_edges, const int64_t* edge_center,
                         const int64_t* edge_nbr, int32_t* center_out, int32_t* nbr_out, int32_t* row_ptr,
                         int32_t* src_ptr, int32_t* src_perm, int32_t* scratch, void* stream) {
  if (n_nodes < 0 || n_edges < 0 || n_nodes >= (int64_t)1 << 31 || n_edges >= (int64_t)1 << 31)
    return fail(E3GNN_ERR_ARG, "conv graph size out of int32 range");
  if (n_nodes > graph_small_max_nodes() || n_edges > graph_small_max_edges())
    return fail(E3GNN_ERR_ARG, "e3gnn_conv_graph_i64: more than " + std::to_string(graph_small_max_nodes()) +
                                   " nodes or " + std::to_string(graph_small_max_edges()) +
                                   " edges (convert the indices and use e3gnn_conv_graph)");
  if (!row_ptr || !src_ptr || !scratch ||
      (n_edges > 0 && (!edge_center || !edge_nbr || !center_out || !nbr_out || !src_perm)))
    return fail(E3GNN_ERR_ARG, "null conv graph buffer");
  hipStream_t s = (hipStream_t)stream;
  int* err_d = scratch + n_nodes;
  HIPCHK(launch_build_graph_small(n_edges, (int)n_nodes, nullptr, nullptr, edge_center, edge_nbr, center_out,
                                  nbr_out, row_ptr, src_ptr, src_perm, err_d, s));
  return graph_check(err_d, s);
}

int e3gnn_conv_graph_small_max_nodes(void) { return graph_small_max_nodes(); }
int e3gnn_conv_graph_small_max_edges(void) { return graph_small_max_edges(); }

static int graph_check(int* err_d, hipStream_t s) {
  int err = 0;
  HIPCHK(hipMemcpyAsync(&err, err_d, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (err) {
    std::string msg = "invalid graph:";
    if (err & 1) msg += " edge_center not sorted non-decreasing;";
    if (err & 2) msg += " edge_center out of [0, n_nodes);";
    if (err & 4) msg += " edge_nbr out of [0, n_nodes);";
    return fail(E3GNN_ERR_GRAPH, msg);
  }
  return E3GNN_OK;
}

int e3gnn_conv_forward(int kind, int64_t n_nodes, const int32_t* row_ptr, const int32_t* edge_nbr,
                       const float* h, const float* Y, const float* w, float* agg,
                       void* stream) {
  return e3gnn_conv_forward_acc(kind, n_nodes, row_ptr, edge_nbr, h, Y, w, agg, 0, stream);
}

int e3gnn_conv_forward_acc(int kind, int64_t n_nodes, const int32_t* row_ptr,
                           const int32_t* edge_nbr, const float* h, const float* Y, const float* w,
                           float* agg, int accumulate, void* stream) {
  int dx, W, dm;
  if (!conv_kind_dims(kind, &dx, &W, &dm)) return fail(E3GNN_ERR_ARG, "conv kind must be 0, 1 or 2");
  if (n_nodes <= 0) return E3GNN_OK;
  if (!row_ptr || !h || !Y || !w || !agg) return fail(E3GNN_ERR_ARG, "null conv operand");
  TpArgs a{};
  a.row_ptr = row_ptr;
  a.nbr = edge_nbr;
  a.Y = Y;
  a.w = w;
  a.h = h;
  a.agg = agg;
  a.n_centers = (int)n_nodes;
  a.denom = 1.0f;
  a.acc_out = accumulate & 1;
  HIPCHK(launch_tp_fwd(kind, a, (hipStream_t)stream));
  return E3GNN_OK;
}

int e3gnn_conv_backward(int kind, int64_t n_nodes, int64_t n_edges, const int32_t* row_ptr,
                        const int32_t* edge_nbr, const int32_t* src_ptr, const int32_t* src_perm,
                        const float* h, const float* Y, const float* w, const float* gagg,
                        float* dh, float* dY, float* dw, float* dxc, void* stream) {
  return e3gnn_conv_backward_acc(kind, n_nodes, n_edges, row_ptr, edge_nbr, src_ptr, src_perm, h, Y,
                                 w, gagg, dh, dY, dw, dxc, 0, stream);
}

int e3gnn_conv_backward_acc(int kind, int64_t n_nodes, int64_t n_edges, const int32_t* row_ptr,
                            const int32_t* edge_nbr, const int32_t* src_ptr,
                            const int32_t* src_perm, const float* h, const float* Y, const float* w,
                            const float* gagg, float* dh, float* dY, float* dw, float* dxc,
                            int accumulate, void* stream) {
  int dx, W, dm;
  if (!conv_kind_dims(kind, &dx, &W, &dm)) return fail(E3GNN_ERR_ARG, "conv kind must be 0, 1 or 2");
  hipStream_t s = (hipStream_t)stream;
  const int acc_dh = accumulate & 1, acc_dY = accumulate & 2, acc_dw = accumulate & 4;
  if (n_edges <= 0 || n_nodes <= 0) {
    // no edges: zero gradients (the accumulated ones keep their values)
    if (dh && n_nodes > 0 && !acc_dh) HIPCHK(launch_zero(dh, n_nodes * dx, s));
    return E3GNN_OK;
  }
  if (!row_ptr || !edge_nbr || !h || !Y || !w || !gagg || !dY || !dw)
    return fail(E3GNN_ERR_ARG, "null conv operand");
  if (dh && (!dxc || !src_ptr || !src_perm))
    return fail(E3GNN_ERR_ARG, "dh needs dxc scratch and the transposed CSR");
  TpArgs a{};
  a.row_ptr = row_ptr;
  a.nbr = edge_nbr;
  a.Y = Y;
  a.w = w;
  a.h = h;
  a.gagg = gagg;
  a.dw = dw;
  a.dxc = dh ? dxc : nullptr;
  a.dYacc = dY;
  a.n_centers = (int)n_nodes;
  a.denom = 1.0f;
  a.acc_out = acc_dw ? 1 : 0;
  a.dy_assign = acc_dY ? 0 : 1;   // every edge's dY has one writer: no zeroing launch
  HIPCHK(launch_tp_bwd(kind, a, s));
  // the gather writes every row (zero without incoming edges): no zeroing launch
  if (dh) HIPCHK(launch_gather_rows((int)n_nodes, dx, src_ptr, src_perm, dxc, dh, s, acc_dh ? 1 : 0));
  return E3GNN_OK;
}

// ------------------------------------------------------------ fine-tune radial MLP
int e3gnn_radial_mlp_forward(int64_t n_rows, int width, const float* emb, const float* W0,
                             const float* W1, const float* W2, const float* a1_primal,
                             const float* a2_primal, float* a1, float* h1, float* a2, float* h2,
                             float* w, float act_scale, void* stream) {
  if (n_rows <= 0) return E3GNN_OK;
  if (n_rows > INT32_MAX || width <= 0 || width % 16)
    return fail(E3GNN_ERR_ARG, "radial MLP: width must be a positive multiple of 16");
  if (!emb || !W0 || !W1 || !W2 || !a1 || !h1 || !a2 || !h2 || !w ||
      ((a1_primal == nullptr) != (a2_primal == nullptr)))
    return fail(E3GNN_ERR_ARG, "null radial MLP operand");
  HIPCHK(launch_mlp_fwd((int)n_rows, width, emb, W0, W1, W2, a1_primal, a2_primal, a1, h1, a2, h2, w,
                        act_scale, (hipStream_t)stream));
  return E3GNN_OK;
}

int e3gnn_radial_mlp_forward_p(int64_t n_rows, int width, const float* emb, const float* W0,
                               const float* W1, const float* W2, const void* w2_pieces,
                               const float* a1_primal, const float* a2_primal, float* a1, float* h1,
                               float* a2, float* h2, float* w, float act_scale, void* stream) {
  if (n_rows <= 0) return E3GNN_OK;
  if (n_rows > INT32_MAX || width <= 0 || width % 16)
    return fail(E3GNN_ERR_ARG, "radial MLP: width must be a positive multiple of 16");
  if (!emb || !W0 || !W1 || !W2 || !a1 || !h1 || !a2 || !h2 || !w ||
      ((a1_primal == nullptr) != (a2_primal == nullptr)))
    return fail(E3GNN_ERR_ARG, "null radial MLP operand");
  if (w2_pieces && reinterpret_cast<uintptr_t>(w2_pieces) % 16)
    return fail(E3GNN_ERR_ARG, "radial MLP: the W2 piece image must be 16-byte aligned");
  HIPCHK(launch_mlp_fwd((int)n_rows, width, emb, W0, W1, W2, a1_primal, a2_primal, a1, h1, a2, h2, w,
                        act_scale, (hipStream_t)stream, w2_pieces));
  return E3GNN_OK;
}

int64_t e3gnn_radial_mlp_w2_piece_bytes(int width) {
  return (width > 0 && width % 16 == 0) ? mlp_w2_piece_bytes(width) : -1;
}

int e3gnn_radial_mlp_w2_pieces(int n, const float* const* W2, const int32_t* widths, void* const* images,
                               void* stream) {
  if (n < 0 || n > 8 || (n > 0 && (!W2 || !widths || !images)))
    return fail(E3GNN_ERR_ARG, "e3gnn_radial_mlp_w2_pieces: 0..8 matrices");
  for (int i = 0; i < n; ++i)
    if (!W2[i] || !images[i] || widths[i] <= 0 || widths[i] % 16 || reinterpret_cast<uintptr_t>(images[i]) % 16)
      return fail(E3GNN_ERR_ARG, "e3gnn_radial_mlp_w2_pieces: matrix " + std::to_string(i));
  HIPCHK(launch_mlp_w2_pieces(n, W2, widths, images, (hipStream_t)stream));
  return E3GNN_OK;
}

int e3gnn_radial_mlp_backward(int64_t n_rows, int width, const float* wb, const float* W0,
                              const float* W1, const float* W2, const float* a1, const float* a2,
                              const float* a1_tangent, const float* a2_tangent, float* a2b,
                              float* a1b, float* embb, float act_scale, void* stream) {
  return e3gnn_radial_mlp_backward_p(n_rows, width, wb, W0, W1, W2, nullptr, a1, a2, a1_tangent, a2_tangent,
                                     a2b, a1b, embb, act_scale, stream);
}

int e3gnn_radial_mlp_backward_p(int64_t n_rows, int width, const float* wb, const float* W0,
                                const float* W1, const float* W2, const void* w2_pieces, const float* a1,
                                const float* a2, const float* a1_tangent, const float* a2_tangent,
                                float* a2b, float* a1b, float* embb, float act_scale, void* stream) {
  if (n_rows <= 0) return E3GNN_OK;
  if (w2_pieces && reinterpret_cast<uintptr_t>(w2_pieces) % 16)
    return fail(E3GNN_ERR_ARG, "radial MLP backward: the W2 piece image must be 16-byte aligned");
  if (n_rows > INT32_MAX || width <= 0 || width % 16)
    return fail(E3GNN_ERR_ARG, "radial MLP backward: width must be a multiple of 16");
  if (!wb || !W0 || !W1 || !W2 || !a1 || !a2 || !embb ||
      ((a1_tangent == nullptr) != (a2_tangent == nullptr)))
    return fail(E3GNN_ERR_ARG, "null radial MLP operand");
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (!al(wb) || !al(W0) || !al(W1) || !al(W2))
    return fail(E3GNN_ERR_ARG, "radial MLP backward: wb / W0 / W1 / W2 must be 16-byte aligned");
  HIPCHK(launch_mlp_bwd((int)n_rows, width, wb, W0, W1, W2, a1, a2, a1_tangent, a2_tangent, a2b, a1b,
                        embb, act_scale, (hipStream_t)stream, w2_pieces));
  return E3GNN_OK;
}

// ------------------------------------------------------------ fine-tune edge geometry
int e3gnn_edge_geometry(int64_t n_edges, const float* vec, const float* coeffs, float rc, float ron,
                        int raw_sh, float* Y, float* emb, void* stream) {
  if (n_edges <= 0) return E3GNN_OK;
  if (!vec || !coeffs || !Y || !emb) return fail(E3GNN_ERR_ARG, "null edge geometry operand");
  HIPCHK(launch_edge_embed(n_edges, vec, coeffs, rc, ron, raw_sh, Y, emb, (hipStream_t)stream));
  return E3GNN_OK;
}

int e3gnn_edge_geometry_jvp(int64_t n_edges, const float* vec, const float* coeffs, float rc,
                            float ron, int raw_sh, const int32_t* center, const int32_t* nbr,
                            const int64_t* batch, const float* cF, const float* cS,
                            const float* vol, float* Yd, float* embd, float* rd, void* stream) {
  if (n_edges <= 0) return E3GNN_OK;
  if (!vec || !coeffs || !center || !nbr || !cF || !Yd || !embd || !rd ||
      (cS && (!batch || !vol)))
    return fail(E3GNN_ERR_ARG, "null edge geometry operand");
  HIPCHK(launch_edge_geom_jvp(n_edges, vec, coeffs, rc, ron, raw_sh, center, nbr, batch, cF, cS, vol,
                              Yd, embd, rd, (hipStream_t)stream));
  return E3GNN_OK;
}

int e3gnn_edge_geometry_vjp(int64_t n_edges, const float* vec, const float* coeffs, float rc,
                            float ron, int raw_sh, const float* Yb, const float* embb, float* fij,
                            void* stream) {
  if (n_edges <= 0) return E3GNN_OK;
  if (!vec || !coeffs || !Yb || !embb || !fij) return fail(E3GNN_ERR_ARG, "null edge geometry operand");
  HIPCHK(launch_edge_force(n_edges, vec, coeffs, rc, ron, raw_sh, Yb, nullptr, embb, fij, nullptr,
                           (hipStream_t)stream));
  return E3GNN_OK;
}

int e3gnn_edge_geometry_coeff_grad(int64_t n_edges, const float* vec, const float* coeffs, float rc,
                                   float ron, const float* embb, const float* embdb, const float* rd,
                                   float* out, void* stream) {
  if (n_edges <= 0) return E3GNN_OK;
  if (!vec || !coeffs || !embb || !embdb || !rd || !out)
    return fail(E3GNN_ERR_ARG, "null edge geometry operand");
  HIPCHK(launch_edge_geom_coeff(n_edges, vec, coeffs, rc, ron, embb, embdb, rd, out,
                                (hipStream_t)stream));
  return E3GNN_OK;
}

int e3gnn_edge_forces_to_atoms(int64_t n_nodes, const int32_t* row_ptr, const int32_t* src_ptr,
                               const int32_t* src_perm, const float* fij, float* F, void* stream) {
  if (n_nodes <= 0) return E3GNN_OK;
  if (!row_ptr || !src_ptr || !src_perm || !fij || !F) return fail(E3GNN_ERR_ARG, "null force operand");
  HIPCHK(launch_atom_force((int)n_nodes, (int)n_nodes, row_ptr, src_ptr, src_perm, fij, F,
                           (hipStream_t)stream));
  return E3GNN_OK;
}

int e3gnn_conv_tangent_forward(int kind, int64_t n_nodes, const int32_t* row_ptr,
                               const int32_t* edge_nbr, const float* h, const float* hd,
                               const float* Y, const float* Yd, const float* w, const float* wd,
                               float* agg, int accumulate, void* stream) {
  int dx, W, dm;
  if (!conv_kind_dims(kind, &dx, &W, &dm)) return fail(E3GNN_ERR_ARG, "conv kind must be 0, 1 or 2");
  if (n_nodes <= 0) return E3GNN_OK;
  if (!row_ptr || !h || !Y || !Yd || !w || !wd || !agg) return fail(E3GNN_ERR_ARG, "null conv operand");
  TpDualArgs a{};
  a.row_ptr = row_ptr;
  a.nbr = edge_nbr;
  a.Y = Y;
  a.Yd = Yd;
  a.w = w;
  a.wd = wd;
  a.h = h;
  a.hd = hd;
  a.agg = agg;
  a.n_centers = (int)n_nodes;
  a.acc_out = accumulate & 1;
  HIPCHK(launch_tp_fwd_tan(kind, a, (hipStream_t)stream));
  return E3GNN_OK;
}

int e3gnn_conv_dual_backward(int kind, int64_t n_nodes, int64_t n_edges, const int32_t* row_ptr,
                             const int32_t* edge_nbr, const int32_t* src_ptr,
                             const int32_t* src_perm, const float* h, const float* hd,
                             const float* Y, const float* Yd, const float* w, const float* wd,
                             const float* g, const float* gd, float* dh, float* dhd, float* dw,
                             float* dwd, float* dxc, void* stream) {
  int dx, W, dm;
  if (!conv_kind_dims(kind, &dx, &W, &dm)) return fail(E3GNN_ERR_ARG, "conv kind must be 0, 1 or 2");
  hipStream_t s = (hipStream_t)stream;
  if (n_nodes <= 0) return E3GNN_OK;
  if ((hd == nullptr) != (dhd == nullptr))
    return fail(E3GNN_ERR_ARG, "dual conv backward: h' and dh' go together");
  if (n_edges <= 0) {
    HIPCHK(launch_zero(dh, n_nodes * dx, s));
    if (dhd) HIPCHK(launch_zero(dhd, n_nodes * dx, s));
    return E3GNN_OK;
  }
  if (!row_ptr || !edge_nbr || !src_ptr || !src_perm || !h || !Y || !Yd || !w || !wd || !g || !gd ||
      !dh || !dw || !dwd || !dxc)
    return fail(E3GNN_ERR_ARG, "null conv operand");
  TpDualArgs a{};
  a.row_ptr = row_ptr;
  a.nbr = edge_nbr;
  a.Y = Y;
  a.Yd = Yd;
  a.w = w;
  a.wd = wd;
  a.h = h;
  a.hd = hd;
  a.g = g;
  a.gd = gd;
  a.dw = dw;
  a.dwd = dwd;
  a.dxc = dxc;
  a.dxcd = dhd ? dxc + n_edges * dx : nullptr;
  a.n_centers = (int)n_nodes;
  HIPCHK(launch_tp_bwd_dual(kind, a, s));
  if (dhd)
    HIPCHK(launch_gather_rows2((int)n_nodes, dx, src_ptr, src_perm, dxc, dh, a.dxcd, dhd, s));
  else
    HIPCHK(launch_gather_rows((int)n_nodes, dx, src_ptr, src_perm, dxc, dh, s, 0));
  return E3GNN_OK;
}

// ------------------------------------------------------------ generic path tables
// (gtp.hip): the convolution of any nequip-family model from its instruction list
namespace {
void cg_entries(int l1, int l2, int l3, std::vector<CGEntry>& out) {
  auto add = [&](const CGEntry* e, int n) { out.assign(e, e + n); };
#define E3GNN_CG_CASE(a, b, c) \
  if (l1 == a && l2 == b && l3 == c) return add(CG<a, b, c>::e, CG<a, b, c>::n);
  E3GNN_CG_CASE(0, 0, 0) E3GNN_CG_CASE(0, 1, 1) E3GNN_CG_CASE(0, 2, 2)
  E3GNN_CG_CASE(1, 0, 1) E3GNN_CG_CASE(1, 1, 0) E3GNN_CG_CASE(1, 1, 1) E3GNN_CG_CASE(1, 1, 2)
  E3GNN_CG_CASE(1, 2, 1) E3GNN_CG_CASE(1, 2, 2) E3GNN_CG_CASE(2, 0, 2) E3GNN_CG_CASE(2, 1, 1)
  E3GNN_CG_CASE(2, 1, 2) E3GNN_CG_CASE(2, 2, 0) E3GNN_CG_CASE(2, 2, 1) E3GNN_CG_CASE(2, 2, 2)
#undef E3GNN_CG_CASE
  out.clear();
}
}  // namespace

struct e3gnn_gtp {
  int device = 0;
  GtpTables T{};
  DBuf by[4], ptr[4];
};

e3gnn_gtp* e3gnn_gtp_create(int n_paths, const int32_t* paths, int dx, int dy, int dw, int dm) {
  if (n_paths <= 0 || !paths || dx <= 0 || dy <= 0 || dw <= 0 || dm <= 0) {
    fail(E3GNN_ERR_ARG, "gtp: empty path table or dimensions");
    return nullptr;
  }
  std::vector<GtpTerm> terms;
  std::vector<CGEntry> cg;
  for (int p = 0; p < n_paths; ++p) {
    const int32_t* q = paths + 8 * p;
    const int l1 = q[0], l2 = q[1], l3 = q[2], mul = q[3], xo = q[4], yo = q[5], wo = q[6], mo = q[7];
    if (l1 < 0 || l2 < 0 || l3 < 0 || l1 > 2 || l2 > 2 || l3 > 2 || l3 < std::abs(l1 - l2) ||
        l3 > l1 + l2 || mul <= 0 || xo < 0 || yo < 0 || wo < 0 || mo < 0 ||
        xo + mul * (2 * l1 + 1) > dx || yo + 2 * l2 + 1 > dy || wo + mul > dw ||
        mo + mul * (2 * l3 + 1) > dm) {
      fail(E3GNN_ERR_ARG, "gtp: path " + std::to_string(p) + " out of range (l <= 2, offsets within dims)");
      return nullptr;
    }
    cg_entries(l1, l2, l3, cg);
    for (int u = 0; u < mul; ++u)
      for (auto& e : cg)
        terms.push_back({xo + u * (2 * l1 + 1) + e.i, yo + e.j, wo + u, mo + u * (2 * l3 + 1) + e.k, e.c});
  }
  auto* g = new e3gnn_gtp;
  if (hipGetDevice(&g->device) != hipSuccess) {
    delete g;
    fail(E3GNN_ERR_HIP, "gtp: no device");
    return nullptr;
  }
  const int dims[4] = {dm, dw, dx, dy};
  const GtpTerm* dev_by[4];
  const int* dev_ptr[4];
  for (int o = 0; o < 4; ++o) {
    // stable order by the output each term feeds (fixed summation order)
    auto key = [o](const GtpTerm& t) { return o == 0 ? t.m : (o == 1 ? t.w : (o == 2 ? t.x : t.y)); };
    std::vector<GtpTerm> s = terms;
    std::stable_sort(s.begin(), s.end(), [&](const GtpTerm& a, const GtpTerm& b) { return key(a) < key(b); });
    std::vector<int> ptr(dims[o] + 1, 0);
    for (auto& t : s) ptr[key(t) + 1]++;
    for (int i = 0; i < dims[o]; ++i) ptr[i + 1] += ptr[i];
    if (g->by[o].ensure(s.size() * sizeof(GtpTerm)) != hipSuccess ||
        g->ptr[o].ensure(ptr.size() * 4) != hipSuccess ||
        hipMemcpy(g->by[o].p, s.data(), s.size() * sizeof(GtpTerm), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(g->ptr[o].p, ptr.data(), ptr.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
      delete g;
      fail(E3GNN_ERR_HIP, "gtp: table upload failed");
      return nullptr;
    }
    dev_by[o] = static_cast<const GtpTerm*>(g->by[o].p);
    dev_ptr[o] = static_cast<const int*>(g->ptr[o].p);
  }
  g->T = GtpTables{dx, dy, dw, dm, dev_by[0], dev_ptr[0], dev_by[1], dev_ptr[1],
                   dev_by[2], dev_ptr[2], dev_by[3], dev_ptr[3]};
  (void)hipGetLastError();
  return g;
}

void e3gnn_gtp_free(e3gnn_gtp* g) { delete g; }

extern "C++" {  // internal accessor for the generic engine (generic.cpp)
namespace e3gnn {
const GtpTables* gtp_tables(const e3gnn_gtp* g) { return &g->T; }
}  // namespace e3gnn
}

int e3gnn_gtp_dims(const e3gnn_gtp* g, int* dx, int* dy, int* dw, int* dm) {
  if (!g) return fail(E3GNN_ERR_ARG, "null gtp");
  if (dx) *dx = g->T.dx;
  if (dy) *dy = g->T.dy;
  if (dw) *dw = g->T.dw;
  if (dm) *dm = g->T.dm;
  return E3GNN_OK;
}

int e3gnn_gtp_forward(const e3gnn_gtp* g, int64_t n_nodes, const int32_t* row_ptr,
                      const int32_t* edge_nbr, const float* h, const float* Y, const float* w,
                      float* agg, void* stream) {
  if (!g) return fail(E3GNN_ERR_ARG, "null gtp");
  if (n_nodes <= 0) return E3GNN_OK;
  if (n_nodes >= (int64_t)1 << 31) return fail(E3GNN_ERR_ARG, "gtp: too many nodes");
  if (!row_ptr || !h || !Y || !w || !agg) return fail(E3GNN_ERR_ARG, "null gtp operand");
  HIPCHK(launch_gtp_fwd((int)n_nodes, row_ptr, edge_nbr, h, Y, w, g->T, agg, (hipStream_t)stream));
  return E3GNN_OK;
}

int e3gnn_gtp_backward(const e3gnn_gtp* g, int64_t n_nodes, int64_t n_edges, const int32_t* row_ptr,
                       const int32_t* edge_nbr, const int32_t* src_ptr, const int32_t* src_perm,
                       const float* h, const float* Y, const float* w, const float* gagg,
                       float* dh, float* dY, float* dw, float* dxc, void* stream) {
  if (!g) return fail(E3GNN_ERR_ARG, "null gtp");
  hipStream_t s = (hipStream_t)stream;
  if (dh && n_nodes > 0) HIPCHK(launch_zero(dh, n_nodes * g->T.dx, s));
  if (n_edges <= 0 || n_nodes <= 0) return E3GNN_OK;
  if (n_nodes >= (int64_t)1 << 31 || n_edges >= (int64_t)1 << 31)
    return fail(E3GNN_ERR_ARG, "gtp: graph size out of int32 range");
  if (!row_ptr || !edge_nbr || !h || !Y || !w || !gagg || !dY || !dw)
    return fail(E3GNN_ERR_ARG, "null gtp operand");
  if (dh && (!dxc || !src_ptr || !src_perm))
    return fail(E3GNN_ERR_ARG, "dh needs dxc scratch and the transposed CSR");
  HIPCHK(launch_gtp_bwd((int)n_nodes, row_ptr, edge_nbr, h, Y, w, gagg, g->T, dw, dh ? dxc : nullptr,
                        dY, s));
  if (dh) HIPCHK(launch_gather_rows((int)n_nodes, g->T.dx, src_ptr, src_perm, dxc, dh, s));
  return E3GNN_OK;
}

int e3gnn_act(int op, int64_t n, const float* x, const float* g, const float* gg, float* out0,
              float* out1, float scale, void* stream) {
  if (op < 0 || op > 2) return fail(E3GNN_ERR_ARG, "act op must be 0, 1 or 2");
  if (n < 0) return fail(E3GNN_ERR_ARG, "negative size");
  if (n > 0 && (!x || (op == 0 && !out0) || (op == 1 && (!g || !out0)) ||
                (op == 2 && (!g || !gg || (!out0 && !out1)))))
    return fail(E3GNN_ERR_ARG, "null act operand");
  HIPCHK(launch_act(op, n, x, g, gg, out0, out1, scale, (hipStream_t)stream));
  return E3GNN_OK;
}

int e3gnn_gate(int op, int64_t n, const int32_t* dims, const float* y, const float* go,
               const float* q, float* out0, float* out1, float scale, void* stream) {
  if (op < 0 || op > 2) return fail(E3GNN_ERR_ARG, "gate op must be 0, 1 or 2");
  if (n < 0 || !dims) return fail(E3GNN_ERR_ARG, "bad gate arguments");
  if (dims[4] < 0 || dims[4] > 2) return fail(E3GNN_ERR_ARG, "at most two gated irreps");
  if (n > 0 && (!y || (op >= 1 && !go) || (op == 2 && !q) || (op < 2 && !out0)))
    return fail(E3GNN_ERR_ARG, "null gate operand");
  HIPCHK(launch_gate(op, n, dims, y, go, q, out0, out1, scale, (hipStream_t)stream));
  return E3GNN_OK;
}

int e3gnn_act_dual(int64_t n, const float* x, const float* xd, const float* g, const float* gd,
                   float* og, float* ogd, float scale, void* stream) {
  if (n < 0) return fail(E3GNN_ERR_ARG, "negative size");
  if (n > 0 && (!x || !xd || !g || !gd || !og || !ogd)) return fail(E3GNN_ERR_ARG, "null act operand");
  HIPCHK(launch_act_dual(n, x, xd, g, gd, og, ogd, scale, (hipStream_t)stream));
  return E3GNN_OK;
}

int e3gnn_gate_dual(int op, int64_t n, const int32_t* dims, const float* y, const float* yd,
                    const float* xb, const float* xdb, float* out0, float* out1, float scale,
                    void* stream) {
  if (op < 0 || op > 1) return fail(E3GNN_ERR_ARG, "gate_dual op must be 0 or 1");
  if (n < 0 || !dims) return fail(E3GNN_ERR_ARG, "bad gate arguments");
  if (dims[4] < 0 || dims[4] > 2) return fail(E3GNN_ERR_ARG, "at most two gated irreps");
  if (n > 0 && (!y || !yd || !out0 || (op == 1 && (!xb || !xdb || !out1))))
    return fail(E3GNN_ERR_ARG, "null gate operand");
  HIPCHK(launch_gate_dual(op, n, dims, y, yd, xb, xdb, out0, out1, scale, (hipStream_t)stream));
  return E3GNN_OK;
}

// ------------------------------------------------------------ neighbour list
struct e3gnn_nlist {
  int device = 0;
  int64_t n = 0, E = 0;
  NlGeom G{};
  const double* pos = nullptr;
  bool built = false;
  DBuf f0, bin, bin_count, bin_start, cursor, bin_atoms, deg, row_ptr, err;
};

e3gnn_nlist* e3gnn_nlist_create(int device) {
  if (hipSetDevice(device) != hipSuccess) {
    fail(E3GNN_ERR_HIP, "hipSetDevice failed");
    return nullptr;
  }
  auto* h = new e3gnn_nlist;
  h->device = device;
  return h;
}
void e3gnn_nlist_free(e3gnn_nlist* h) { delete h; }

namespace {
// bins of width >= rc per dimension (heights h), at most ~4 per atom
void nl_bins(NlGeom& G, const double h[3], double rc, int64_t n) {
  for (int k = 0; k < 3; ++k) G.nb[k] = std::max(1, (int)std::floor(h[k] / rc));
  while ((int64_t)G.nb[0] * G.nb[1] * G.nb[2] > 4 * n + 64) {
    int k = 0;
    for (int q = 1; q < 3; ++q)
      if (G.nb[q] > G.nb[k]) k = q;
    G.nb[k] = std::max(1, G.nb[k] / 2);
  }
  for (int k = 0; k < 3; ++k) G.R[k] = std::max(1, (int)std::ceil(rc * G.nb[k] / h[k]));
}
}  // namespace

int e3gnn_nlist_build(e3gnn_nlist* h, int64_t n, const double* pos, const double* cell,
                      const int* pbc, double cutoff, int64_t* n_edges, void* stream) {
  if (!h) return fail(E3GNN_ERR_ARG, "null neighbour-list handle");
  if (n < 0 || n >= (int64_t)1 << 30) return fail(E3GNN_ERR_ARG, "atom count out of range");
  if (!(cutoff > 0)) return fail(E3GNN_ERR_ARG, "cutoff must be positive");
  if (n > 0 && !pos) return fail(E3GNN_ERR_ARG, "null positions");
  if (!pbc) return fail(E3GNN_ERR_ARG, "null pbc flags");
  const bool all = pbc[0] && pbc[1] && pbc[2], none = !pbc[0] && !pbc[1] && !pbc[2];
  if (!all && !none)
    return fail(E3GNN_ERR_ARG, "device neighbour list: pbc must be all true or all false");
  HIPCHK(hipSetDevice(h->device));
  hipStream_t s = (hipStream_t)stream;
  h->built = false;
  h->n = n;
  h->pos = pos;
  NlGeom& G = h->G;
  G = NlGeom{};
  G.rc2 = cutoff * cutoff;
  G.periodic = all ? 1 : 0;
  double hgt[3];
  if (all) {
    if (!cell) return fail(E3GNN_ERR_ARG, "null cell");
    for (int k = 0; k < 9; ++k) G.cell[k] = cell[k];
    const double* a = cell;
    const double det = a[0] * (a[4] * a[8] - a[5] * a[7]) - a[1] * (a[3] * a[8] - a[5] * a[6]) +
                       a[2] * (a[3] * a[7] - a[4] * a[6]);
    if (!(std::fabs(det) > 1e-12)) return fail(E3GNN_ERR_ARG, "singular cell");
    // inverse (rows of cell = lattice vectors): frac = pos @ inv
    G.inv[0] = (a[4] * a[8] - a[5] * a[7]) / det;
    G.inv[1] = (a[2] * a[7] - a[1] * a[8]) / det;
    G.inv[2] = (a[1] * a[5] - a[2] * a[4]) / det;
    G.inv[3] = (a[5] * a[6] - a[3] * a[8]) / det;
    G.inv[4] = (a[0] * a[8] - a[2] * a[6]) / det;
    G.inv[5] = (a[2] * a[3] - a[0] * a[5]) / det;
    G.inv[6] = (a[3] * a[7] - a[4] * a[6]) / det;
    G.inv[7] = (a[1] * a[6] - a[0] * a[7]) / det;
    G.inv[8] = (a[0] * a[4] - a[1] * a[3]) / det;
    for (int k = 0; k < 3; ++k) {  // height along k = |det| / |a_{k+1} x a_{k+2}|
      const double* u = a + 3 * ((k + 1) % 3);
      const double* v = a + 3 * ((k + 2) % 3);
      const double cx = u[1] * v[2] - u[2] * v[1], cy = u[2] * v[0] - u[0] * v[2],
                   cz = u[0] * v[1] - u[1] * v[0];
      hgt[k] = std::fabs(det) / std::sqrt(cx * cx + cy * cy + cz * cz);
    }
  } else {
    // isolated cluster: a virtual orthorhombic box 1 A beyond the atoms on
    // every side, so no image is ever within the cutoff (S = 0 throughout)
    std::vector<double> hp((size_t)n * 3);
    if (n) HIPCHK(hipMemcpy(hp.data(), pos, hp.size() * 8, hipMemcpyDefault));
    double lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
    for (int64_t a = 0; a < n; ++a)
      for (int k = 0; k < 3; ++k) {
        const double v = hp[3 * a + k];
        if (!std::isfinite(v)) return fail(E3GNN_ERR_ARG, "non-finite position");
        lo[k] = a ? std::min(lo[k], v) : v;
        hi[k] = a ? std::max(hi[k], v) : v;
      }
    for (int k = 0; k < 3; ++k) {
      G.origin[k] = lo[k] - 1.0;
      hgt[k] = (hi[k] - lo[k]) + 2.0;
      G.cell[4 * k] = hgt[k];
      G.inv[4 * k] = 1.0 / hgt[k];
    }
  }
  nl_bins(G, hgt, cutoff, n);
  const int nbins = G.nb[0] * G.nb[1] * G.nb[2];
  if (h->f0.ensure((size_t)std::max<int64_t>(n, 1) * 12) != hipSuccess ||
      h->bin.ensure((size_t)std::max<int64_t>(n, 1) * 4) != hipSuccess ||
      h->bin_atoms.ensure((size_t)std::max<int64_t>(n, 1) * 4) != hipSuccess ||
      h->deg.ensure((size_t)std::max<int64_t>(n, 1) * 4) != hipSuccess ||
      h->row_ptr.ensure((size_t)(n + 1) * 4) != hipSuccess ||
      h->bin_count.ensure((size_t)nbins * 4) != hipSuccess ||
      h->bin_start.ensure((size_t)(nbins + 1) * 4) != hipSuccess ||
      h->cursor.ensure((size_t)nbins * 4) != hipSuccess || h->err.ensure(4) != hipSuccess)
    return fail(E3GNN_ERR_HIP, "neighbour-list workspace allocation failed");
  int* err = h->err.i();
  HIPCHK(hipMemsetAsync(err, 0, 4, s));
  HIPCHK(hipMemsetAsync(h->bin_count.p, 0, (size_t)nbins * 4, s));
  HIPCHK(hipMemsetAsync(h->cursor.p, 0, (size_t)nbins * 4, s));
  HIPCHK(launch_nl_bin((int)n, pos, G, h->f0.i(), h->bin.i(), h->bin_count.i(), err, s));
  HIPCHK(launch_nl_scan(nbins, h->bin_count.i(), h->bin_start.i(), s));
  HIPCHK(launch_nl_place((int)n, h->bin.i(), h->bin_start.i(), h->cursor.i(), h->bin_atoms.i(), s));
  HIPCHK(launch_nl_search(false, (int)n, pos, G, h->f0.i(), h->bin.i(), h->bin_start.i(),
                          h->bin_atoms.i(), h->deg.i(), nullptr, nullptr, nullptr, nullptr, nullptr,
                          err, s));
  if (n > 0) HIPCHK(launch_nl_scan((int)n, h->deg.i(), h->row_ptr.i(), s));
  int herr = 0, total = 0;
  HIPCHK(hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, s));
  if (n > 0) HIPCHK(hipMemcpyAsync(&total, h->row_ptr.i() + n, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (herr & 1) return fail(E3GNN_ERR_ARG, "non-finite or out-of-box atom position");
  if (herr & 4)
    return fail(E3GNN_ERR_GRAPH, "a centre has more than " + std::to_string(NL_MAXD) +
                                     " neighbours (device neighbour-list limit)");
  if (total < 0) return fail(E3GNN_ERR_GRAPH, "edge count exceeds int32");
  h->E = total;
  h->built = true;
  if (n_edges) *n_edges = total;
  return E3GNN_OK;
}

int e3gnn_nlist_fetch(e3gnn_nlist* h, int32_t* center, int32_t* nbr, int32_t* shift, float* vec,
                      void* stream) {
  if (!h || !h->built) return fail(E3GNN_ERR_ARG, "neighbour list not built");
  if (h->E > 0 && (!center || !nbr)) return fail(E3GNN_ERR_ARG, "null edge output");
  HIPCHK(hipSetDevice(h->device));
  hipStream_t s = (hipStream_t)stream;
  int* err = h->err.i();
  HIPCHK(hipMemsetAsync(err, 0, 4, s));
  HIPCHK(launch_nl_search(true, (int)h->n, h->pos, h->G, h->f0.i(), h->bin.i(), h->bin_start.i(),
                          h->bin_atoms.i(), nullptr, h->row_ptr.i(), center, nbr, shift, vec, err,
                          s));
  int herr = 0;
  HIPCHK(hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (herr & 2) return fail(E3GNN_ERR_GRAPH, "periodic image shift beyond +-1024 cells");
  return E3GNN_OK;
}

int e3gnn_set_interior(e3gnn_ctx* c, int64_t n_interior) {
  if (!c) return fail(E3GNN_ERR_ARG, "null context");
  if (n_interior < 0) return fail(E3GNN_ERR_ARG, "negative n_interior");
  c->n_interior_req = n_interior;
  return E3GNN_OK;
}

int e3gnn_set_impl(e3gnn_ctx* c, int impl) {
  if (!c) return fail(E3GNN_ERR_ARG, "null context");
  if (impl != 0 && impl != 1) return fail(E3GNN_ERR_ARG, "impl must be 0 (fused) or 1 (v1)");
  c->impl = impl;
  return E3GNN_OK;
}

int e3gnn_set_timing(e3gnn_ctx* c, int enable) {
  if (!c) return fail(E3GNN_ERR_ARG, "null context");
  c->flush();
  c->timing = enable != 0;
  return E3GNN_OK;
}
int e3gnn_set_stream_ordered(e3gnn_ctx* c, int enable) {
  if (!c) return fail(E3GNN_ERR_ARG, "null context");
  c->stream_ordered = enable != 0;
  return E3GNN_OK;
}
int e3gnn_kernel_stats(e3gnn_ctx* c, const char** names, double* ms, int64_t* launches,
                       double* flops, double* bytes, int max) {
  if (!c) return -1;
  c->flush();
  for (int i = 0; i < C_NCLS && i < max; ++i) {
    if (names) names[i] = kClassNames[i];
    if (ms) ms[i] = c->stats[i].ms;
    if (launches) launches[i] = c->stats[i].launches;
    if (flops) flops[i] = c->stats[i].flops;
    if (bytes) bytes[i] = c->stats[i].bytes;
  }
  return C_NCLS;
}
int e3gnn_reset_stats(e3gnn_ctx* c) {
  if (!c) return fail(E3GNN_ERR_ARG, "null context");
  c->flush();
  for (auto& st : c->stats) st = Stat();
  return E3GNN_OK;
}

int e3gnn_cg_table(int l1, int l2, int l3, float* out) {
  if (!out) return fail(E3GNN_ERR_ARG, "null out");
  const int key = l1 * 100 + l2 * 10 + l3;
  switch (key) {
#define CGCASE(a, b, c) \
  case a * 100 + b * 10 + c: dense_cg<a, b, c>(out); return E3GNN_OK;
    CGCASE(0, 0, 0) CGCASE(0, 1, 1) CGCASE(0, 2, 2) CGCASE(1, 0, 1) CGCASE(1, 1, 0)
    CGCASE(1, 1, 1) CGCASE(1, 1, 2) CGCASE(1, 2, 1) CGCASE(1, 2, 2) CGCASE(2, 0, 2)
    CGCASE(2, 1, 1) CGCASE(2, 1, 2) CGCASE(2, 2, 0) CGCASE(2, 2, 1) CGCASE(2, 2, 2)
#undef CGCASE
    default: return fail(E3GNN_ERR_ARG, "no coupling table for this (l1,l2,l3)");
  }
}

float* e3gnn_debug_ptr(e3gnn_ctx* c, const char* name, int layer, int64_t* numel) {
  if (!c || !name) return nullptr;
  const std::string n(name);
  const e3gnn_model* m = c->m;
  const int L = m->nlayer;
  auto ok = [&](int lo, int hi) { return layer >= lo && layer <= hi; };
  float* p = nullptr;
  int64_t k = 0;
  if (n == "x" && ok(0, L)) { p = c->x[layer].f(); k = c->n * irreps_dim(m->irreps[layer]); }
  else if (n == "grad" && ok(0, L)) { p = c->grad[layer].f(); k = c->n * irreps_dim(m->irreps[layer]); }
  else if (n == "h" && ok(0, L - 1)) { p = c->h[layer].f(); k = c->n * irreps_dim(m->irreps[layer]); }
  else if (n == "y" && ok(0, L - 1)) { p = c->y[layer].f(); k = c->nl * irreps_dim(m->gin[layer]); }
  else if (n == "agg" && ok(0, L - 1)) { p = c->agg.f(); k = c->nl * irreps_dim(m->mid[layer]); }
  else if (n == "Y") { p = c->Y.f(); k = c->E * 9; }
  else if (n == "emb") { p = c->emb.f(); k = c->E * 8; }
  else if (n == "dY") { p = c->dY.f(); k = c->E * 9; }
  else if (n == "dgu") { p = c->dgu.f(); k = c->E * 3; }
  else if (n == "demb") { p = c->demb.f(); k = c->E * 8; }
  else if (n == "dxc") { p = c->dxc.f(); k = c->E * 480; }
  else if (n == "fe") { p = c->fe.f(); k = c->E * 3; }
  if (numel) *numel = p ? k : 0;
  return p;
}

int64_t e3gnn_workspace_bytes(const e3gnn_ctx* c) {
  if (!c) return 0;
  int64_t b = 0;
  const DBuf* fixed[] = {&c->type, &c->center, &c->nbr, &c->vec, &c->row_ptr, &c->src_ptr,
                         &c->src_perm, &c->cnt, &c->err, &c->Y, &c->emb, &c->dY, &c->dgu, &c->demb,
                         &c->fe, &c->H1, &c->H2, &c->agg, &c->dw, &c->dxc, &c->dy, &c->dh,
                         &c->eat, &c->part, &c->vpart, &c->scratch6};
  for (auto* d : fixed) b += (int64_t)d->cap;
  for (auto* v : {&c->x, &c->grad, &c->h, &c->y, &c->w, &c->a1, &c->a2})
    for (auto& d : *v) b += (int64_t)d.cap;
  return b;
}

}  // extern "C"

// ------------------------------------------------------------ DFT-D3
// PairD3 (sevenn/pair_e3gnn/pair_d3.cu) over host arrays, as LAMMPS hands
// them to PairD3::compute: settings/coeff -> e3gnn_d3_create, compute ->
// e3gnn_d3_compute (wrap into the cell :1182-1224, image lists :1026-1045 and
// :1230-1266, the four kernels of d3.hip, update :2003-2024).
struct e3gnn_d3 {
  int device = 0;
  D3Params p{};
  DBuf rcov, r2r4, r0ab, mxc, c6ab, cnref, x, type, bin_of, bin_start, off_v, off_c, cn, gw,
      c6tab, rows, forces, totals;
};

e3gnn_d3* e3gnn_d3_create(int device, int damping, const float* func, float rthr, float cn_thr,
                          int ntypes, const float* rcov, const float* r2r4, const float* r0ab,
                          const int32_t* mxc, const float* c6ab) {
  if (damping != 1 && damping != 2 && damping != 4) {
    fail(E3GNN_ERR_ARG, damping == 3 ? "damp_zerom is not implemented (nor by the reference, "
                                       "pair_d3.cu:1550-1553)"
                                     : "damping must be 1 (zero), 2 (bj) or 4 (bjm)");
    return nullptr;
  }
  if (ntypes <= 0 || !func || !rcov || !r2r4 || !r0ab || !mxc || !c6ab || !(rthr > 0) ||
      !(cn_thr > 0)) {
    fail(E3GNN_ERR_ARG, "d3: bad parameters");
    return nullptr;
  }
  for (int t = 0; t < ntypes; ++t)
    if (mxc[t] < 0 || mxc[t] > 5) {
      fail(E3GNN_ERR_ARG, "d3: mxc out of [0, 5]");
      return nullptr;
    }
  if (hipSetDevice(device) != hipSuccess) {
    fail(E3GNN_ERR_HIP, "hipSetDevice failed");
    return nullptr;
  }
  auto* h = new e3gnn_d3;
  h->device = device;
  const size_t nt = (size_t)ntypes;
  auto up = [](DBuf& b, const void* src, size_t bytes) {
    if (b.ensure(bytes) != hipSuccess) return false;
    return hipMemcpy(b.p, src, bytes, hipMemcpyHostToDevice) == hipSuccess;
  };
  if (!up(h->rcov, rcov, nt * 4) || !up(h->r2r4, r2r4, nt * 4) || !up(h->r0ab, r0ab, nt * nt * 4) ||
      !up(h->mxc, mxc, nt * 4) || !up(h->c6ab, c6ab, nt * nt * 75 * 4)) {
    delete h;
    fail(E3GNN_ERR_HIP, "d3: table upload failed");
    return nullptr;
  }
  D3Params& p = h->p;
  p.damping = damping == 1 ? 1 : 2;
  p.ntypes = ntypes;
  p.s6 = func[0];
  p.s8 = func[1];
  p.a1 = func[2];
  p.a2 = func[3];
  p.alp6 = func[4];
  p.alp8 = func[5];
  p.rthr = rthr;
  p.cn_thr = cn_thr;
  p.rcov = h->rcov.f();
  p.r2r4 = h->r2r4.f();
  p.r0ab = h->r0ab.f();
  p.mxc = h->mxc.i();
  p.c6ab = h->c6ab.f();
  // reference CN per (type, grid index), if the table is separable that way
  // (Grimme's data is: a reference CN belongs to an element's reference)
  std::vector<float> cr((size_t)ntypes * 5, 0.0f);
  std::vector<int> seen((size_t)ntypes * 5, 0);
  bool separable = true;
  for (int a = 0; a < ntypes; ++a)
    for (int b = 0; b < ntypes; ++b)
      for (int ia = 0; ia < 5; ++ia)
        for (int ib = 0; ib < 5; ++ib) {
          const float* e = c6ab + ((((size_t)a * ntypes + b) * 5 + ia) * 5 + ib) * 3;
          if (!(e[0] > 0.0f)) continue;
          const int ka = a * 5 + ia, kb = b * 5 + ib;
          if (seen[ka] && cr[ka] != e[1]) separable = false;
          if (seen[kb] && cr[kb] != e[2]) separable = false;
          cr[ka] = e[1];
          cr[kb] = e[2];
          seen[ka] = seen[kb] = 1;
        }
  p.cnref = nullptr;
  if (separable) {
    if (!up(h->cnref, cr.data(), cr.size() * 4)) {
      delete h;
      fail(E3GNN_ERR_HIP, "d3: table upload failed");
      return nullptr;
    }
    p.cnref = h->cnref.f();
  }
  return h;
}

void e3gnn_d3_free(e3gnn_d3* h) { delete h; }

namespace {
constexpr double D3_BIN_BOHR = 30.0;     // bin edge: swept 12-40 bohr on 8k-atom Si, 30 best
constexpr int64_t D3_C6TAB_MAX = 32768;  // n^2 C6 table up to 8.6 GB; beyond: C6 per item

// stencil of bin offsets covering a sphere of radius sqrt(thr): R = floor(rc /
// bin height) + 1 bins along each periodic axis (every (bin, image) pair once)
std::vector<int> d3_stencil(float thr, const double binh[3], const int* pbc,
                            const double lat[3][3], const int nb[3], double hd, bool prune) {
  const double rc = std::sqrt((double)thr);
  int R[3];
  for (int k = 0; k < 3; ++k) R[k] = pbc[k] ? (int)std::floor(rc / binh[k]) + 1 : 0;
  std::vector<int> off;
  for (int a = -R[0]; a <= R[0]; ++a)
    for (int b = -R[1]; b <= R[1]; ++b)
      for (int c = -R[2]; c <= R[2]; ++c) {
        if (prune) {
          // a cell whose centre is farther than rc + one full bin diagonal from
          // the home cell's centre cannot hold a partner of any atom of it
          double d[3];
          for (int k = 0; k < 3; ++k)
            d[k] = a * lat[0][k] / nb[0] + b * lat[1][k] / nb[1] + c * lat[2][k] / nb[2];
          if (std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]) > rc + 2.0 * hd + 1e-9) continue;
        }
        off.push_back(a);
        off.push_back(b);
        off.push_back(c);
      }
  return off;
}
}  // namespace

int e3gnn_d3_compute(e3gnn_d3* h, int64_t n, const double* pos, const double* cell,
                     const int32_t* pbc, const int32_t* type, double* energy, double* forces,
                     double* virial6, void* stream) {
  if (!h) return fail(E3GNN_ERR_ARG, "null d3 handle");
  if (n < 0 || n >= (int64_t)1 << 31) return fail(E3GNN_ERR_ARG, "d3: atom count out of range");
  if (n > 0 && (!pos || !type || !forces)) return fail(E3GNN_ERR_ARG, "d3: null input");
  if (!cell || !pbc || !energy || !virial6) return fail(E3GNN_ERR_ARG, "d3: null input");
  for (int64_t i = 0; i < n; ++i)
    if (type[i] < 0 || type[i] >= h->p.ntypes) return fail(E3GNN_ERR_ARG, "d3: type out of range");
  // lattice in bohr, rows a, b, c
  double lat[3][3];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) lat[r][c] = cell[3 * r + c] / D3_AU_TO_ANG;
  const double det = lat[0][0] * (lat[1][1] * lat[2][2] - lat[1][2] * lat[2][1]) -
                     lat[0][1] * (lat[1][0] * lat[2][2] - lat[1][2] * lat[2][0]) +
                     lat[0][2] * (lat[1][0] * lat[2][1] - lat[1][1] * lat[2][0]);
  if (!(std::fabs(det) > 1e-12)) return fail(E3GNN_ERR_ARG, "d3: singular cell");
  // inverse (columns of inv = reciprocal rows / det); frac = pos . inv
  double inv[3][3];
  inv[0][0] = (lat[1][1] * lat[2][2] - lat[1][2] * lat[2][1]) / det;
  inv[0][1] = (lat[0][2] * lat[2][1] - lat[0][1] * lat[2][2]) / det;
  inv[0][2] = (lat[0][1] * lat[1][2] - lat[0][2] * lat[1][1]) / det;
  inv[1][0] = (lat[1][2] * lat[2][0] - lat[1][0] * lat[2][2]) / det;
  inv[1][1] = (lat[0][0] * lat[2][2] - lat[0][2] * lat[2][0]) / det;
  inv[1][2] = (lat[0][2] * lat[1][0] - lat[0][0] * lat[1][2]) / det;
  inv[2][0] = (lat[1][0] * lat[2][1] - lat[1][1] * lat[2][0]) / det;
  inv[2][1] = (lat[0][1] * lat[2][0] - lat[0][0] * lat[2][1]) / det;
  inv[2][2] = (lat[0][0] * lat[1][1] - lat[0][1] * lat[1][0]) / det;
  // wrap (load_atom_info :1182-1224) and bin along the lattice vectors
  // (E3GNN_D3_BIN: bin edge in bohr, for tuning)
  const char* bin_env = std::getenv("E3GNN_D3_BIN");
  const double bin_w = bin_env ? std::max(2.0, std::atof(bin_env)) : D3_BIN_BOHR;
  double hgt[3], binh[3];
  int nb[3];
  bool all_pbc = true;
  for (int k = 0; k < 3; ++k) {
    const double* u = lat[(k + 1) % 3];
    const double* v = lat[(k + 2) % 3];
    const double c[3] = {u[1] * v[2] - u[2] * v[1], u[2] * v[0] - u[0] * v[2],
                         u[0] * v[1] - u[1] * v[0]};
    hgt[k] = std::fabs(c[0] * lat[k][0] + c[1] * lat[k][1] + c[2] * lat[k][2]) /
           std::sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
    nb[k] = pbc[k] ? std::max(1, (int)(hgt[k] / bin_w)) : 1;
    binh[k] = hgt[k] / nb[k];
    all_pbc = all_pbc && pbc[k];
  }
  const int nbins = nb[0] * nb[1] * nb[2];
  std::vector<float> xw((size_t)n * 3);
  std::vector<int> bin((size_t)n), cnt(nbins + 1, 0);
  for (int64_t i = 0; i < n; ++i) {
    double p[3], a[3];
    int b[3];
    for (int d = 0; d < 3; ++d) p[d] = pos[3 * i + d] / D3_AU_TO_ANG;
    for (int k = 0; k < 3; ++k) {
      // row vector p = a . lat  ->  a = p . inv
      a[k] = p[0] * inv[0][k] + p[1] * inv[1][k] + p[2] * inv[2][k];
      if (pbc[k]) a[k] -= std::floor(a[k]);
      b[k] = pbc[k] ? std::min(nb[k] - 1, std::max(0, (int)(a[k] * nb[k]))) : 0;
    }
    for (int d = 0; d < 3; ++d)
      xw[3 * i + d] = (float)(a[0] * lat[0][d] + a[1] * lat[1][d] + a[2] * lat[2][d]);
    bin[i] = (b[0] * nb[1] + b[1]) * nb[2] + b[2];
    ++cnt[bin[i] + 1];
  }
  for (int b = 0; b < nbins; ++b) cnt[b + 1] += cnt[b];
  // counting sort by bin (stable: ascending atom id inside a bin)
  std::vector<int> perm((size_t)n), fill(cnt.begin(), cnt.end() - 1);
  for (int64_t i = 0; i < n; ++i) perm[fill[bin[i]]++] = (int)i;
  std::vector<float> xs((size_t)n * 4);
  std::vector<int> ts((size_t)n), bs((size_t)n);
  for (int64_t s2 = 0; s2 < n; ++s2) {
    const int i = perm[s2];
    for (int d = 0; d < 3; ++d) xs[4 * s2 + d] = xw[3 * i + d];
    std::memcpy(&xs[4 * s2 + 3], &type[i], 4);   // type bits in .w
    ts[s2] = type[i];
    bs[s2] = bin[i];
  }
  // half of the longest bin diagonal
  double hd = 0.0;
  for (int sa = -1; sa <= 1; sa += 2)
    for (int sb = -1; sb <= 1; sb += 2) {
      double d[3];
      for (int c = 0; c < 3; ++c)
        d[c] = lat[0][c] / nb[0] + sa * lat[1][c] / nb[1] + sb * lat[2][c] / nb[2];
      hd = std::max(hd, 0.5 * std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]));
    }
  const std::vector<int> ov = d3_stencil(h->p.rthr, binh, pbc, lat, nb, hd, all_pbc);
  const std::vector<int> oc = d3_stencil(h->p.cn_thr, binh, pbc, lat, nb, hd, all_pbc);
  HIPCHK(hipSetDevice(h->device));
  hipStream_t s = (hipStream_t)stream;
  const size_t nn = (size_t)std::max<int64_t>(n, 1);
  // E3GNN_D3_NO_C6TAB=1: the per-item C6 path of large systems (tests)
  const char* no_tab = std::getenv("E3GNN_D3_NO_C6TAB");
  const bool use_tab = n <= D3_C6TAB_MAX && !(no_tab && no_tab[0] == '1');
  HIPCHK(h->x.ensure(nn * 16));
  HIPCHK(h->type.ensure(nn * 4));
  HIPCHK(h->bin_of.ensure(nn * 4));
  HIPCHK(h->bin_start.ensure((nbins + 1) * 4));
  HIPCHK(h->off_v.ensure(ov.size() * 4));
  HIPCHK(h->off_c.ensure(oc.size() * 4));
  HIPCHK(h->cn.ensure(nn * 8));
  if (use_tab) HIPCHK(h->c6tab.ensure(nn * nn * 8));
  HIPCHK(h->gw.ensure(nn * 80));
  HIPCHK(h->rows.ensure(nn * 64));
  HIPCHK(h->forces.ensure(nn * 24));
  HIPCHK(h->totals.ensure(7 * 8));
  if (n > 0) {
    HIPCHK(hipMemcpyAsync(h->x.p, xs.data(), n * 16, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(h->type.p, ts.data(), n * 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(h->bin_of.p, bs.data(), n * 4, hipMemcpyHostToDevice, s));
  }
  HIPCHK(hipMemcpyAsync(h->bin_start.p, cnt.data(), (nbins + 1) * 4, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(h->off_v.p, ov.data(), ov.size() * 4, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(h->off_c.p, oc.data(), oc.size() * 4, hipMemcpyHostToDevice, s));
  D3Grid g{};
  for (int k = 0; k < 3; ++k) {
    g.nb[k] = nb[k];
    g.inv_nb[k] = (float)(1.0 / nb[k]);
  }
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) g.lat[3 * r + c] = (float)lat[r][c];
  g.cull = all_pbc ? 1 : 0;
  const double rv = std::sqrt((double)h->p.rthr) + hd, rcn = std::sqrt((double)h->p.cn_thr) + hd;
  g.cull2_vdw = (float)(rv * rv * (1.0 + 1e-5));
  g.cull2_cn = (float)(rcn * rcn * (1.0 + 1e-5));
  g.bin_of = h->bin_of.i();
  g.bin_start = h->bin_start.i();
  g.off_vdw = h->off_v.i();
  g.off_cn = h->off_c.i();
  g.n_off_vdw = (int)(ov.size() / 3);
  g.n_off_cn = (int)(oc.size() / 3);
  HIPCHK(launch_d3(h->p, g, (int)n, (const float4*)h->x.p, h->type.i(), (double*)h->cn.p,
                   (double*)h->gw.p, use_tab ? (float2*)h->c6tab.p : nullptr, (double*)h->rows.p,
                   (double*)h->forces.p, (double*)h->totals.p, s));
  double tot[7];
  std::vector<double> fs((size_t)n * 3);
  HIPCHK(hipMemcpyAsync(tot, h->totals.p, 7 * 8, hipMemcpyDeviceToHost, s));
  if (n > 0) HIPCHK(hipMemcpyAsync(fs.data(), h->forces.p, n * 24, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  for (int64_t s2 = 0; s2 < n; ++s2)
    for (int d = 0; d < 3; ++d) forces[3 * perm[s2] + d] = fs[3 * s2 + d];
  *energy = tot[0];
  for (int k = 0; k < 6; ++k) virial6[k] = tot[1 + k];
  return E3GNN_OK;
}
