/* -*- c++ -*- ----------------------------------------------------------
   pair_style e3gnn on MI355X: the reference's PairE3GNN
   (sevenn/pair_e3gnn/pair_e3gnn.{h,cpp}) with the TorchScript model replaced by
   libe3gnn_hip.so (include/e3gnn.h) through the LAMMPS-independent core
   native/pair_e3gnn_core.{h,cpp}.  Same style name, same input lines:

     pair_style e3gnn
     pair_coeff * * <deployment dir: weights.bin + manifest.json> <element per type>

   Build: copy this file, pair_e3gnn_core.{h,cpp} and include/e3gnn.h into
   LAMMPS' src/ and link libe3gnn_hip.so.  It needs no
   LibTorch.
------------------------------------------------------------------------- */

#ifdef PAIR_CLASS
// clang-format off
PairStyle(e3gnn, PairE3GNN)
// clang-format on
#else

#ifndef LMP_PAIR_E3GNN
#define LMP_PAIR_E3GNN

#include "pair.h"

#include <memory>
#include <string>
#include <vector>

namespace e3gnn_pair {
class Model;
class SerialStep;
}  // namespace e3gnn_pair

namespace LAMMPS_NS {

class PairE3GNN : public Pair {
 public:
  PairE3GNN(class LAMMPS *);
  ~PairE3GNN() override;
  void compute(int, int) override;
  void settings(int, char **) override;
  void coeff(int, char **) override;
  void init_style() override;
  double init_one(int, int) override;

 protected:
  void allocate();
  double cutoff = 0.0;
  int device = 0;
  std::unique_ptr<e3gnn_pair::Model> model;
  std::unique_ptr<e3gnn_pair::SerialStep> step;
  std::vector<int> species;   // LAMMPS type -> model species index
  std::vector<int64_t> tag64;
};

}  // namespace LAMMPS_NS

#endif
#endif
