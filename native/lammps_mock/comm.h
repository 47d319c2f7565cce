// mini-LAMMPS test scaffold (see lmptype.h)
#pragma once
#include "pointers.h"

namespace LAMMPS_NS {
class Comm : protected Pointers {
 public:
  explicit Comm(LAMMPS *lmp) : Pointers(lmp) {}
  ~Comm() override = default;
  int me = 0, nprocs = 1;
  int procgrid[3] = {1, 1, 1}, myloc[3] = {0, 0, 0};
  int procneigh[3][2] = {{0, 0}, {0, 0}, {0, 0}};
};
}  // namespace LAMMPS_NS
