// mini-LAMMPS test scaffold (see lmptype.h): the Pair members the pair styles use
#pragma once
#include <vector>

#include "pointers.h"

namespace LAMMPS_NS {
class NeighList;
class Pair : protected Pointers {
 public:
  explicit Pair(LAMMPS *lmp) : Pointers(lmp) {}
  ~Pair() override = default;
  double eng_vdwl = 0.0, eng_coul = 0.0;
  double virial[6] = {0, 0, 0, 0, 0, 0};
  double *eatom = nullptr, **vatom = nullptr;
  int allocated = 0;
  int **setflag = nullptr;
  double **cutsq = nullptr;
  int comm_forward = 0, comm_reverse = 0;
  int single_enable = 1, restartinfo = 1, one_coeff = 0, manybody_flag = 0;
  int eflag_either = 0, eflag_global = 0, eflag_atom = 0;
  int vflag_either = 0, vflag_global = 0, vflag_atom = 0;
  NeighList *list = nullptr;
  virtual void compute(int, int) = 0;
  virtual void settings(int, char **) = 0;
  virtual void coeff(int, char **) = 0;
  virtual void init_style() {}
  virtual double init_one(int, int) { return 0.0; }
  virtual void init_list(int, NeighList *ptr) { list = ptr; }

 protected:
  // ENERGY_GLOBAL = 1, ENERGY_ATOM = 2, VIRIAL_PAIR = 1, VIRIAL_ATOM = 4
  void ev_init(int eflag, int vflag);
  std::vector<double> eatom_s;
};
}  // namespace LAMMPS_NS
