// pair_e3gnn_core -- the LAMMPS-independent per-step core of the LAMMPS pair
// styles e3gnn/hip and e3gnn/parallel/hip (native/lammps/), over the C ABI of
// libe3gnn_hip.so.  The LAMMPS adaptors only map Atom / NeighList / Comm onto
// the views below; everything the reference does per step between LAMMPS and
// the model lives here, so it is compiled and tested without LAMMPS
// (native/e3gnn_pair_check.cpp).
//
// Reference: sevenn/pair_e3gnn/pair_e3gnn.cpp (PairE3GNN::compute :72-275,
// ::coeff :294-386) and pair_e3gnn_parallel.cpp (PairE3GNNParallel::compute
// :207-541, comm_preprocess / pack_/unpack_{forward,reverse}_comm_gnn
// :693-933).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "e3gnn.h"

namespace e3gnn_pair {

// What LAMMPS hands a full-neighbour-list pair style each step (Atom + NeighList)
struct NeighborView {
  int inum = 0;                      // list->inum (== atom->nlocal)
  const int* ilist = nullptr;        // list->ilist
  const int* numneigh = nullptr;     // list->numneigh
  int* const* firstneigh = nullptr;  // list->firstneigh (j may carry special bits)
  double* const* x = nullptr;        // atom->x, local then ghost rows
  const int* type = nullptr;         // atom->type (1-based LAMMPS types)
  const int64_t* tag = nullptr;      // atom->tag (1..natoms; ghosts carry their owner's tag)
  int nlocal = 0, nghost = 0;
  int neighmask = 0x1FFFFFFF;        // NEIGHMASK
};

// LAMMPS' per-step accumulators of a pair style (Pair::eng_vdwl, virial[6],
// eatom[], f[][3]); virial in LAMMPS order (xx, yy, zz, xy, xz, yz)
struct PairOut {
  double energy = 0.0;
  double virial[6] = {0, 0, 0, 0, 0, 0};
};

// The deployment and its species map: pair_coeff * * <model dir> <element per type>
class Model {
 public:
  // weights.bin + manifest.json of `model_dir`; throws std::runtime_error
  Model(const std::string& model_dir, int device);
  ~Model();
  Model(const Model&) = delete;
  Model& operator=(const Model&) = delete;
  // PairE3GNN::coeff (pair_e3gnn.cpp:330-378): elements[k] is the chemical
  // symbol of LAMMPS type k + 1; returns map[type] = species index (map[0]
  // unused); throws on an element the model does not know
  std::vector<int> type_map(const std::vector<std::string>& elements) const;
  double cutoff() const { return cutoff_; }
  int comm_size() const { return comm_size_; }
  int num_layers() const { return nlayers_; }
  e3gnn_model* handle() const { return m_; }
  const std::vector<std::string>& symbols() const { return symbols_; }

 private:
  e3gnn_model* m_ = nullptr;
  double cutoff_ = 0.0;
  int comm_size_ = 0, nlayers_ = 0, nspecies_ = 0;
  std::vector<std::string> symbols_;
};

// Device buffers that grow with the graph (the reference's nedges_bound)
struct DeviceGraph {
  int32_t *type = nullptr, *center = nullptr, *nbr = nullptr;
  float *vec = nullptr, *forces = nullptr, *atomic = nullptr, *scalars = nullptr;
  int64_t cap_n = 0, cap_e = 0;
  void reserve(int64_t n, int64_t e);
  void release();
};

// pair_style e3gnn/hip: one rank holds every atom (local rows), ghosts are
// periodic images identified by tag (PairE3GNN::compute, pair_e3gnn.cpp:72-275):
// graph nodes are tag - 1, edges i -> j for every full-list neighbour within
// the cutoff, edge_vec = x_j - x_i.  Forces are written (not added) to the
// local atoms, eatom accumulated, the virial in LAMMPS order.
class SerialStep {
 public:
  explicit SerialStep(const Model& model);
  ~SerialStep();
  // returns 0, or an E3GNN_ERR_* code with the message in error()
  int compute(const NeighborView& nv, const std::vector<int>& map, double** f, double* eatom,
              PairOut& out);
  const std::string& error() const { return err_; }
  int64_t last_edges() const { return nedges_; }

 private:
  const Model& model_;
  e3gnn_ctx* ctx_ = nullptr;
  void* stream_ = nullptr;
  DeviceGraph g_;
  std::vector<int32_t> type_, center_, nbr_;
  std::vector<float> vec_, forces_, atomic_;
  std::vector<int> tag2i_;
  int64_t nedges_ = 0;
  std::string err_;
};

// pair_style e3gnn/parallel/hip (PairE3GNNParallel::compute,
// pair_e3gnn_parallel.cpp:207-541): graph rows = the rank's local atoms (list
// order), then every ghost within the cutoff of a local atom, first seen,
// deduplicated by tag; per layer the ghost rows' features arrive through the
// halo exchange, after the readout the ghost rows' dE/dx go back, then the
// ghost forces (newton on).  The exchange itself belongs to the host (LAMMPS
// CommBrick through pack/unpack_*_comm_gnn): the step exposes the row buffer
// `comm_rows()` (graph rows + extra rows for atoms this rank only relays +
// one trash row) and per exchange phase the row index lists the reference
// builds in pack_forward_init / unpack_forward_init / comm_preprocess.
class ParallelStep {
 public:
  // the host's exchange: called once per layer boundary (forward) and once
  // per backward layer + once for the forces (reverse)
  struct Exchange {
    virtual ~Exchange() = default;
    // ghost rows <- owners' rows of step.comm_rows() (row width step.comm_dim())
    virtual int forward(ParallelStep& step) = 0;
    // owners' rows += ghost rows' values of step.comm_rows()
    virtual int reverse(ParallelStep& step) = 0;
  };
  explicit ParallelStep(const Model& model);
  ~ParallelStep();
  // builds the rank graph (tag -> graph row map of the reference); call before compute
  int build(const NeighborView& nv, const std::vector<int>& map, int64_t natoms);
  // graph row of a LAMMPS atom index (local or ghost), or -1 when it is not in
  // this rank's graph (the host then gives it an extra row: extra_row())
  int graph_row(int lammps_index) const;
  // an extra row (>= graph_size) for an atom this rank relays but does not use
  int extra_row(int lammps_index);
  int graph_size() const { return (int)row_to_i_.size(); }
  int64_t nlocal() const { return nlocal_; }
  int64_t nedges() const { return (int64_t)center_.size(); }
  // row buffer of the current exchange on the device: graph rows, extra rows,
  // one trash row; width comm_dim() floats
  float* comm_rows() const { return comm_; }
  int comm_dim() const { return comm_dim_; }
  int trash_row() const { return graph_size() + (int)extra_.size(); }
  // device row pack / unpack for the host's message buffers (e3gnn_halo_pack
  // / _unpack on comm_rows(); idx: device int32 rows)
  int pack(const int32_t* idx, int64_t n, float* buf);
  int unpack(const int32_t* idx, int64_t n, const float* buf, bool accumulate);
  // one evaluation: forward with `ex.forward` between the blocks, backward
  // with `ex.reverse` after each block and for the ghost forces
  int compute(Exchange& ex, double** f, double* eatom, PairOut& out);
  const std::string& error() const { return err_; }
  void* stream() const { return stream_; }

 private:
  int grow_comm(int rows, int dim);
  int load_rows(float* src, int dim, int rows);    // graph rows of src -> comm
  int store_rows(float* dst, int dim, int rows);   // comm -> src (rows)
  const Model& model_;
  e3gnn_ctx* ctx_ = nullptr;
  void* stream_ = nullptr;
  DeviceGraph g_;
  int64_t nlocal_ = 0, nghost_graph_ = 0;
  std::vector<int32_t> type_, center_, nbr_;
  std::vector<float> vec_, forces_, atomic_;
  std::vector<int> row_to_i_;          // graph row -> LAMMPS atom index
  std::vector<int> i_to_row_;          // LAMMPS atom index -> graph row (-1)
  std::vector<int> tag_to_row_;        // tag -> graph row (-1)
  std::vector<std::pair<int, int>> extra_;  // (LAMMPS index, row)
  const int64_t* tag_ = nullptr;
  float* comm_ = nullptr;
  int comm_cap_ = 0, comm_dim_ = 0, comm_nrows_ = 0;
  std::string err_;
};

}  // namespace e3gnn_pair
