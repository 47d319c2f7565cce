// pair_e3gnn_core -- see pair_e3gnn_core.h.
#include "pair_e3gnn_core.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <fstream>
#include <sstream>
#include <stdexcept>

namespace e3gnn_pair {

namespace {

// "chemical_symbols": ["Ac", ...] of the deployment manifest (the
// chemical_symbols_to_index metadata of deploy.py:34-51)
std::vector<std::string> manifest_symbols(const std::string& path) {
  std::ifstream f(path);
  if (!f) throw std::runtime_error("cannot open " + path);
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string s = ss.str();
  const size_t k = s.find("\"chemical_symbols\"");
  if (k == std::string::npos) throw std::runtime_error("manifest without chemical_symbols");
  const size_t a = s.find('[', k), b = s.find(']', a);
  std::vector<std::string> out;
  for (size_t p = a; p < b;) {
    const size_t q0 = s.find('"', p);
    if (q0 == std::string::npos || q0 > b) break;
    const size_t q1 = s.find('"', q0 + 1);
    out.push_back(s.substr(q0 + 1, q1 - q0 - 1));
    p = q1 + 1;
  }
  return out;
}

int hip_fail(std::string& err, hipError_t e, const char* what) {
  err = std::string(what) + ": " + hipGetErrorString(e);
  return E3GNN_ERR_HIP;
}

#define CORE_HIP(x)                                        \
  do {                                                     \
    hipError_t e_ = (x);                                   \
    if (e_ != hipSuccess) return hip_fail(err_, e_, #x);   \
  } while (0)
#define CORE_ABI(x)                                        \
  do {                                                     \
    int rc_ = (x);                                         \
    if (rc_) {                                             \
      err_ = std::string(#x) + ": " + e3gnn_last_error();  \
      return rc_;                                          \
    }                                                      \
  } while (0)

// LAMMPS virial (xx, yy, zz, xy, xz, yz) from this library's virial6 (xx, yy,
// zz, xy, yz, zx) -- pair_e3gnn.cpp:250-255
void add_virial(double* lmp, const float* v6) {
  lmp[0] += v6[0];
  lmp[1] += v6[1];
  lmp[2] += v6[2];
  lmp[3] += v6[3];
  lmp[4] += v6[5];
  lmp[5] += v6[4];
}

}  // namespace

// ------------------------------------------------------------------ Model
Model::Model(const std::string& dir, int device) {
  symbols_ = manifest_symbols(dir + "/manifest.json");
  m_ = e3gnn_load((dir + "/weights.bin").c_str(), (dir + "/manifest.json").c_str(), device);
  if (!m_) throw std::runtime_error(std::string("e3gnn_load: ") + e3gnn_last_error());
  float co = 0.f;
  if (e3gnn_model_info(m_, &nspecies_, &co, &nlayers_, &comm_size_))
    throw std::runtime_error(std::string("e3gnn_model_info: ") + e3gnn_last_error());
  cutoff_ = co;
}

Model::~Model() {
  if (m_) e3gnn_free(m_);
}

std::vector<int> Model::type_map(const std::vector<std::string>& elements) const {
  std::vector<int> map(elements.size() + 1, -1);
  for (size_t t = 0; t < elements.size(); ++t) {
    for (size_t k = 0; k < symbols_.size(); ++k)
      if (symbols_[k] == elements[t]) map[t + 1] = (int)k;
    if (map[t + 1] < 0) throw std::runtime_error("Unknown chemical specie is given: " + elements[t]);
  }
  return map;
}

// ------------------------------------------------------------------ DeviceGraph
void DeviceGraph::reserve(int64_t n, int64_t e) {
  auto check = [](hipError_t x) {
    if (x != hipSuccess) throw std::runtime_error(std::string("hipMalloc: ") + hipGetErrorString(x));
  };
  auto realloc = [&](auto*& p, int64_t count) {
    if (p) check(hipFree(p));
    p = nullptr;
    check(hipMalloc(&p, count * sizeof(*p)));
  };
  // capacities grow by 1.2x, like the reference's nedges_bound (pair_e3gnn.cpp:267-273)
  if (n > cap_n || !type) {
    cap_n = n + n / 5 + 64;
    realloc(type, cap_n);
    realloc(forces, 3 * cap_n);
    realloc(atomic, cap_n);
  }
  if (e > cap_e || !center) {
    cap_e = e + e / 5 + 64;
    realloc(center, cap_e);
    realloc(nbr, cap_e);
    realloc(vec, 3 * cap_e);
  }
  if (!scalars) check(hipMalloc(&scalars, 8 * sizeof(float)));
}

void DeviceGraph::release() {
  for (void* p : {(void*)type, (void*)center, (void*)nbr, (void*)vec, (void*)forces, (void*)atomic,
                  (void*)scalars})
    if (p) (void)hipFree(p);
  type = center = nbr = nullptr;
  vec = forces = atomic = scalars = nullptr;
  cap_n = cap_e = 0;
}

// ------------------------------------------------------------------ SerialStep
SerialStep::SerialStep(const Model& model) : model_(model) {
  ctx_ = e3gnn_ctx_create(model.handle());
  if (!ctx_) throw std::runtime_error(std::string("e3gnn_ctx_create: ") + e3gnn_last_error());
  hipStream_t s;
  if (hipStreamCreate(&s) != hipSuccess) throw std::runtime_error("hipStreamCreate");
  stream_ = s;
}

SerialStep::~SerialStep() {
  g_.release();
  if (stream_) (void)hipStreamDestroy((hipStream_t)stream_);
  if (ctx_) e3gnn_ctx_free(ctx_);
}

int SerialStep::compute(const NeighborView& nv, const std::vector<int>& map, double** f,
                        double* eatom, PairOut& out) {
  const int n = nv.inum;
  const double rc2 = model_.cutoff() * model_.cutoff();
  // nodes = tag - 1 (pair_e3gnn.cpp:146-154; "requires consecutive atom IDs")
  tag2i_.assign(n, -1);
  type_.assign(n, 0);
  for (int ii = 0; ii < n; ++ii) {
    const int i = nv.ilist[ii];
    const int64_t t = nv.tag[i] - 1;
    if (t < 0 || t >= n || tag2i_[t] >= 0) {
      err_ = "Pair e3gnn requires consecutive atom IDs";
      return E3GNN_ERR_ARG;
    }
    const int ty = nv.type[i];
    if (ty < 1 || ty >= (int)map.size() || map[ty] < 0) {
      err_ = "atom type without a pair_coeff element";
      return E3GNN_ERR_ARG;
    }
    tag2i_[t] = i;
    type_[t] = map[ty];
  }
  // edges in node order (the kernels take edge_center sorted): every full-list
  // neighbour inside the cutoff (pair_e3gnn.cpp:156-182), edge_vec = x_j - x_i,
  // which is pos[jtag] - pos[itag] + shift @ cell exactly
  center_.clear();
  nbr_.clear();
  vec_.clear();
  for (int t = 0; t < n; ++t) {
    const int i = tag2i_[t];
    const int* jl = nv.firstneigh[i];
    for (int jj = 0; jj < nv.numneigh[i]; ++jj) {
      const int j = jl[jj] & nv.neighmask;
      const double d0 = nv.x[j][0] - nv.x[i][0], d1 = nv.x[j][1] - nv.x[i][1],
                   d2 = nv.x[j][2] - nv.x[i][2];
      if (d0 * d0 + d1 * d1 + d2 * d2 < rc2) {
        const int64_t jt = nv.tag[j] - 1;
        if (jt < 0 || jt >= n) {
          err_ = "neighbour tag out of range (Pair e3gnn requires consecutive atom IDs)";
          return E3GNN_ERR_ARG;
        }
        center_.push_back(t);
        nbr_.push_back((int32_t)jt);
        vec_.push_back((float)d0);
        vec_.push_back((float)d1);
        vec_.push_back((float)d2);
      }
    }
  }
  nedges_ = (int64_t)center_.size();
  try {
    g_.reserve(n, nedges_);
  } catch (const std::exception& e) {
    err_ = e.what();
    return E3GNN_ERR_HIP;
  }
  hipStream_t s = (hipStream_t)stream_;
  CORE_HIP(hipMemcpyAsync(g_.type, type_.data(), n * 4, hipMemcpyHostToDevice, s));
  if (nedges_) {
    CORE_HIP(hipMemcpyAsync(g_.center, center_.data(), nedges_ * 4, hipMemcpyHostToDevice, s));
    CORE_HIP(hipMemcpyAsync(g_.nbr, nbr_.data(), nedges_ * 4, hipMemcpyHostToDevice, s));
    CORE_HIP(hipMemcpyAsync(g_.vec, vec_.data(), nedges_ * 12, hipMemcpyHostToDevice, s));
  }
  CORE_ABI(e3gnn_energy_forces(ctx_, n, nedges_, g_.type, g_.center, g_.nbr, g_.vec, g_.scalars,
                               eatom ? g_.atomic : nullptr, g_.forces, g_.scalars + 1, nullptr, s));
  float sc[7];
  forces_.resize(3 * (size_t)n);
  CORE_HIP(hipMemcpyAsync(sc, g_.scalars, 7 * 4, hipMemcpyDeviceToHost, s));
  CORE_HIP(hipMemcpyAsync(forces_.data(), g_.forces, n * 12, hipMemcpyDeviceToHost, s));
  if (eatom) {
    atomic_.resize(n);
    CORE_HIP(hipMemcpyAsync(atomic_.data(), g_.atomic, n * 4, hipMemcpyDeviceToHost, s));
  }
  CORE_HIP(hipStreamSynchronize(s));
  // forces added to what LAMMPS zeroed (the reference assigns them; adding keeps
  // pair_style hybrid/overlay with d3 correct), pair_e3gnn.cpp:244-248
  for (int t = 0; t < n; ++t) {
    double* fi = f[tag2i_[t]];
    fi[0] += forces_[3 * t];
    fi[1] += forces_[3 * t + 1];
    fi[2] += forces_[3 * t + 2];
    if (eatom) eatom[tag2i_[t]] += atomic_[t];
  }
  out.energy += sc[0];
  add_virial(out.virial, sc + 1);
  return E3GNN_OK;
}

// ------------------------------------------------------------------ ParallelStep
ParallelStep::ParallelStep(const Model& model) : model_(model) {
  ctx_ = e3gnn_ctx_create(model.handle());
  if (!ctx_) throw std::runtime_error(std::string("e3gnn_ctx_create: ") + e3gnn_last_error());
  hipStream_t s;
  if (hipStreamCreate(&s) != hipSuccess) throw std::runtime_error("hipStreamCreate");
  stream_ = s;
}

ParallelStep::~ParallelStep() {
  g_.release();
  if (comm_) (void)hipFree(comm_);
  if (stream_) (void)hipStreamDestroy((hipStream_t)stream_);
  if (ctx_) e3gnn_ctx_free(ctx_);
}

int ParallelStep::build(const NeighborView& nv, const std::vector<int>& map, int64_t natoms) {
  const int nl = nv.inum;
  const double rc2 = model_.cutoff() * model_.cutoff();
  nlocal_ = nl;
  tag_ = nv.tag;
  ntotal_ = (int64_t)nv.nlocal + nv.nghost;
  tag_to_row_.assign(natoms + 1, -1);
  tag_to_extra_.assign(natoms + 1, -1);
  i_to_row_.assign(ntotal_, -1);
  row_to_i_.clear();
  type_.clear();
  nextra_ = 0;
  ntrash_ = 0;
  auto type_of = [&](int i, int32_t& out) {
    const int ty = nv.type[i];
    if (ty < 1 || ty >= (int)map.size() || map[ty] < 0) return false;
    out = map[ty];
    return true;
  };
  // local rows in list order (pair_e3gnn_parallel.cpp:285-293)
  for (int ii = 0; ii < nl; ++ii) {
    const int i = nv.ilist[ii];
    const int64_t tg = nv.tag[i];
    if (tg < 1 || tg > natoms) {
      err_ = "atom tag out of range";
      return E3GNN_ERR_ARG;
    }
    tag_to_row_[tg] = ii;
    row_to_i_.push_back(i);
    int32_t sp;
    if (!type_of(i, sp)) {
      err_ = "atom type without a pair_coeff element";
      return E3GNN_ERR_ARG;
    }
    type_.push_back(sp);
  }
  // edges; a ghost within the cutoff gets a row when first seen, by tag
  // (:296-325: periodic images of one atom share its row)
  center_.clear();
  nbr_.clear();
  vec_.clear();
  for (int ii = 0; ii < nl; ++ii) {
    const int i = nv.ilist[ii];
    const int* jl = nv.firstneigh[i];
    for (int jj = 0; jj < nv.numneigh[i]; ++jj) {
      const int j = jl[jj] & nv.neighmask;
      const double d0 = nv.x[j][0] - nv.x[i][0], d1 = nv.x[j][1] - nv.x[i][1],
                   d2 = nv.x[j][2] - nv.x[i][2];
      if (d0 * d0 + d1 * d1 + d2 * d2 >= rc2) continue;
      const int64_t jt = nv.tag[j];
      if (jt < 1 || jt > natoms) {
        err_ = "neighbour tag out of range";
        return E3GNN_ERR_ARG;
      }
      if (tag_to_row_[jt] < 0) {
        tag_to_row_[jt] = (int)row_to_i_.size();
        row_to_i_.push_back(j);
        int32_t sp;
        if (!type_of(j, sp)) {
          err_ = "atom type without a pair_coeff element";
          return E3GNN_ERR_ARG;
        }
        type_.push_back(sp);
      }
      center_.push_back(ii);
      nbr_.push_back(tag_to_row_[jt]);
      vec_.push_back((float)d0);
      vec_.push_back((float)d1);
      vec_.push_back((float)d2);
    }
  }
  for (size_t r = 0; r < row_to_i_.size(); ++r) i_to_row_[row_to_i_[r]] = (int)r;
  nghost_graph_ = (int64_t)row_to_i_.size() - nl;
  CORE_ABI(e3gnn_graph_set(ctx_, nl, nghost_graph_, (int64_t)center_.size(), type_.data(),
                           center_.data(), nbr_.data(), vec_.data(), stream_));
  return E3GNN_OK;
}

int ParallelStep::graph_row(int idx) const {
  if (idx < 0 || idx >= ntotal_) return -1;
  const int64_t tg = tag_[idx];
  return (tg >= 1 && tg < (int64_t)tag_to_row_.size()) ? tag_to_row_[tg] : -1;
}

int ParallelStep::extra_row(int idx) {
  if (idx < 0 || idx >= ntotal_) return -1;
  const int64_t tg = tag_[idx];
  if (tg < 1 || tg >= (int64_t)tag_to_extra_.size()) return -1;
  if (tag_to_extra_[tg] < 0) tag_to_extra_[tg] = graph_size() + nextra_++;
  return tag_to_extra_[tg];
}

int ParallelStep::grow_comm(int rows, int dim) {
  const int64_t need = (int64_t)rows * dim;
  if (need > comm_cap_) {
    if (comm_) CORE_HIP(hipFree(comm_));
    comm_cap_ = need + need / 4 + 1024;
    CORE_HIP(hipMalloc(&comm_, (size_t)comm_cap_ * sizeof(float)));
  }
  comm_dim_ = dim;
  comm_nrows_ = rows;
  return E3GNN_OK;
}

int ParallelStep::load_rows(float* src, int dim, int rows) {
  // x_comm = cat(graph rows, zeros for the extra, zero and trash rows)
  const int total = comm_row_count();
  if (int rc = grow_comm(total, dim)) return rc;
  hipStream_t s = (hipStream_t)stream_;
  CORE_HIP(hipMemcpyAsync(comm_, src, (size_t)rows * dim * 4, hipMemcpyDeviceToDevice, s));
  CORE_HIP(hipMemsetAsync(comm_ + (size_t)rows * dim, 0, (size_t)(total - rows) * dim * 4, s));
  CORE_HIP(hipStreamSynchronize(s));
  return E3GNN_OK;
}

int ParallelStep::store_rows(float* dst, int dim, int rows) {
  hipStream_t s = (hipStream_t)stream_;
  CORE_HIP(hipMemcpyAsync(dst, comm_, (size_t)rows * dim * 4, hipMemcpyDeviceToDevice, s));
  return E3GNN_OK;
}

int ParallelStep::pack(const int32_t* idx, int64_t n, float* buf) {
  if (n <= 0) return E3GNN_OK;
  CORE_ABI(e3gnn_halo_pack(idx, n, comm_dim_, comm_, comm_dim_, buf, stream_));
  return E3GNN_OK;
}

int ParallelStep::unpack(const int32_t* idx, int64_t n, const float* buf, bool accumulate) {
  if (n <= 0) return E3GNN_OK;
  CORE_ABI(e3gnn_halo_unpack(idx, n, comm_dim_, buf, comm_, comm_dim_, accumulate ? 1 : 0, stream_));
  return E3GNN_OK;
}

int ParallelStep::compute(Exchange& ex, double** f, double* eatom, PairOut& out) {
  hipStream_t s = (hipStream_t)stream_;
  const int L = model_.num_layers();
  const int G = graph_size();
  for (int t = 0; t < L; ++t) {
    if (t > 0) {
      // forward_comm of the layer-t features (:345-372): the ghost rows of the
      // graph come from their owners
      const int dim = e3gnn_feature_dim(ctx_, t);
      float* x = e3gnn_feature_ptr(ctx_, t);
      if (int rc = load_rows(x, dim, G)) return rc;
      if (int rc = ex.forward(*this)) {
        err_ = "forward exchange failed";
        return rc;
      }
      if (int rc = store_rows(x, dim, G)) return rc;
    }
    CORE_ABI(e3gnn_layer_forward(ctx_, t, s));
  }
  try {
    g_.reserve(G, 0);
  } catch (const std::exception& e) {
    err_ = e.what();
    return E3GNN_ERR_HIP;
  }
  CORE_ABI(e3gnn_readout(ctx_, g_.scalars, eatom ? g_.atomic : nullptr, s));
  for (int t = L - 1; t >= 0; --t) {
    CORE_ABI(e3gnn_layer_backward(ctx_, t, s));
    if (t > 0) {
      // reverse_comm of dE/dx of the ghost rows (:417-454): owners accumulate
      const int dim = e3gnn_feature_dim(ctx_, t);
      float* gx = e3gnn_grad_ptr(ctx_, t);
      if (int rc = load_rows(gx, dim, G)) return rc;
      if (int rc = ex.reverse(*this)) {
        err_ = "reverse exchange failed";
        return rc;
      }
      if (int rc = store_rows(gx, dim, (int)nlocal_)) return rc;
    }
  }
  CORE_ABI(e3gnn_forces(ctx_, g_.forces, g_.scalars + 1, nullptr, s));
  float sc[7];
  forces_.resize(3 * (size_t)G);
  CORE_HIP(hipMemcpyAsync(sc, g_.scalars, 7 * 4, hipMemcpyDeviceToHost, s));
  CORE_HIP(hipMemcpyAsync(forces_.data(), g_.forces, (size_t)G * 12, hipMemcpyDeviceToHost, s));
  if (eatom) {
    atomic_.resize(nlocal_);
    CORE_HIP(hipMemcpyAsync(atomic_.data(), g_.atomic, nlocal_ * 4, hipMemcpyDeviceToHost, s));
  }
  CORE_HIP(hipStreamSynchronize(s));
  // forces on local AND ghost rows (:480-488): LAMMPS' own reverse
  // communication (newton on) then sums the ghost forces onto their owners
  for (int r = 0; r < G; ++r) {
    double* fi = f[row_to_i_[r]];
    fi[0] += forces_[3 * r];
    fi[1] += forces_[3 * r + 1];
    fi[2] += forces_[3 * r + 2];
  }
  if (eatom)
    for (int r = 0; r < nlocal_; ++r) eatom[row_to_i_[r]] += atomic_[r];
  out.energy += sc[0];
  add_virial(out.virial, sc + 1);
  return E3GNN_OK;
}

// ------------------------------------------------------------------ CommMaps
CommMaps::~CommMaps() {
  for (auto& ph : d_)
    for (int32_t* q : ph)
      if (q) (void)hipFree(q);
}

void CommMaps::begin() {
  for (int p = 0; p < kPhases; ++p) {
    send_[p].clear();
    recv_[p].clear();
    fwd_dst_[p].clear();
    rev_src_[p].clear();
    rev_dst_[p].clear();
    send_is_ghost_[p].clear();
  }
  st_ = Stats();
  ready_ = false;
}

// rows of the atoms CommBrick sends in swap `phase`: local atoms and ghosts
// received in earlier swaps (pair_e3gnn_parallel.cpp:750-779)
int CommMaps::pack_forward_init(int n, const int* list_send, int phase) {
  if (phase < 0 || phase >= kPhases) {
    err_ = "PairE3GNNParallel: Cell size is too small. Please use a single GPU or replicate the cell.";
    return E3GNN_ERR_ARG;
  }
  auto& idx = send_[phase];
  idx.reserve(idx.size() + n);
  for (int k = 0; k < n; ++k) {
    const int a = list_send[k];
    const int r = s_.row_of(a);
    if (r < 0) {
      err_ = "pack_forward_init: atom without a tag";
      return E3GNN_ERR_ARG;
    }
    idx.push_back(r);
    send_is_ghost_[phase].push_back(a >= s_.nlocal() ? 1 : 0);
  }
  return E3GNN_OK;
}

// rows of the ghosts [first, first + n) received in swap `phase` (:781-801)
int CommMaps::unpack_forward_init(int n, int first, int phase) {
  if (phase < 0 || phase >= kPhases) {
    err_ = "PairE3GNNParallel: Cell size is too small. Please use a single GPU or replicate the cell.";
    return E3GNN_ERR_ARG;
  }
  auto& idx = recv_[phase];
  idx.reserve(idx.size() + n);
  for (int a = first; a < first + n; ++a) {
    const int r = s_.row_of(a);
    if (r < 0) {
      err_ = "unpack_forward_init: atom without a tag";
      return E3GNN_ERR_ARG;
    }
    idx.push_back(r);
  }
  return E3GNN_OK;
}

int CommMaps::finish() {
  const int zero = s_.zero_row();
  const int nlocal = (int)s_.nlocal();
  // rows already returned by an earlier reception (receiver side) and rows
  // already accumulated in this swap (sender side); sized after every extra
  // row is known (finish runs after the last *_init hook)
  std::vector<char> returned(zero, 0);
  std::vector<int> seen_in_phase(zero, -1);
  int ntrash = 0;
  for (int p = 0; p < kPhases; ++p) {
    const auto& rv = recv_[p];
    const auto& sd = send_[p];
    if (rv.empty() && sd.empty()) continue;
    ++st_.swaps;
    // forward unpack: unique destinations; a repeat of a row within the swap,
    // or a reception of one of this rank's own atoms, goes to a trash row
    int tf = 0;
    fwd_dst_[p].resize(rv.size());
    rev_src_[p].resize(rv.size());
    for (size_t k = 0; k < rv.size(); ++k) {
      const int r = rv[k];
      if (r < nlocal || seen_in_phase[r] == 2 * p) {
        fwd_dst_[p][k] = -1 - tf++;   // resolved below, once the zero row is fixed
        ++st_.trash_forward;
      } else {
        fwd_dst_[p][k] = r;
        seen_in_phase[r] = 2 * p;
      }
      // reverse pack: the row's value once over all receptions, zero otherwise
      if (r >= nlocal && !returned[r]) {
        rev_src_[p][k] = r;
        returned[r] = 1;
      } else {
        rev_src_[p][k] = zero;
        ++st_.zero_sends;
      }
    }
    // reverse unpack (accumulate): unique destinations within the swap
    int tr = 0;
    rev_dst_[p].resize(sd.size());
    for (size_t k = 0; k < sd.size(); ++k) {
      const int r = sd[k];
      if (seen_in_phase[r] == 2 * p + 1) {
        rev_dst_[p][k] = -1 - tr++;
        ++st_.trash_reverse;
      } else {
        rev_dst_[p][k] = r;
        seen_in_phase[r] = 2 * p + 1;
      }
      st_.sent += 1;
      st_.relayed += send_is_ghost_[p][k];
    }
    ntrash = std::max(ntrash, std::max(tf, tr));
  }
  s_.set_trash_rows(ntrash);
  st_.extra_rows = s_.extra_rows();
  for (int p = 0; p < kPhases; ++p) {
    for (auto* v : {&fwd_dst_[p], &rev_dst_[p]})
      for (auto& r : *v)
        if (r < 0) r = s_.trash_row(-1 - r);
    const std::vector<int32_t>* h[4] = {&send_[p], &fwd_dst_[p], &rev_src_[p], &rev_dst_[p]};
    for (int k = 0; k < 4; ++k) {
      const int64_t n = (int64_t)h[k]->size();
      if (n > cap_[p][k]) {
        if (d_[p][k]) (void)hipFree(d_[p][k]);
        d_[p][k] = nullptr;
        cap_[p][k] = n + n / 4 + 64;
        if (hipMalloc(&d_[p][k], cap_[p][k] * 4) != hipSuccess) {
          err_ = "CommMaps: hipMalloc";
          return E3GNN_ERR_HIP;
        }
      }
      if (n && hipMemcpy(d_[p][k], h[k]->data(), n * 4, hipMemcpyHostToDevice) != hipSuccess) {
        err_ = "CommMaps: hipMemcpy";
        return E3GNN_ERR_HIP;
      }
    }
  }
  ready_ = true;
  return E3GNN_OK;
}

// pack_forward_comm_gnn (:803-839): rows of the sent atoms -> buf
int64_t CommMaps::pack_forward(int p, float* buf) {
  const int64_t n = nsend(p);
  if (s_.pack(d_[p][0], n, buf)) return -1;
  return n * s_.comm_dim();
}

// unpack_forward_comm_gnn (:841-871): buf -> rows of the received ghosts
int64_t CommMaps::unpack_forward(int p, const float* buf) {
  const int64_t n = nrecv(p);
  if (s_.unpack(d_[p][1], n, buf, false)) return -1;
  return n * s_.comm_dim();
}

// pack_reverse_comm_gnn (:873-900): the received ghosts' rows go back
int64_t CommMaps::pack_reverse(int p, float* buf) {
  const int64_t n = nrecv(p);
  if (s_.pack(d_[p][2], n, buf)) return -1;
  return n * s_.comm_dim();
}

// unpack_reverse_comm_gnn (:902-933): accumulated into the sent atoms' rows
int64_t CommMaps::unpack_reverse(int p, const float* buf) {
  const int64_t n = nsend(p);
  if (s_.unpack(d_[p][3], n, buf, true)) return -1;
  return n * s_.comm_dim();
}

}  // namespace e3gnn_pair
