// mini-LAMMPS test scaffold (see lmptype.h): owned rows then ghost rows
#pragma once
#include <vector>

#include "lmptype.h"

namespace LAMMPS_NS {
class Atom {
 public:
  int nlocal = 0, nghost = 0, ntypes = 0;
  bigint natoms = 0;
  double **x = nullptr, **f = nullptr;
  int *type = nullptr;
  tagint *tag = nullptr;
  int tag_consecutive() const { return 1; }
  // scaffold: storage behind the LAMMPS-style pointers
  std::vector<double> xs, fs, lamda;
  std::vector<double *> xp, fp;
  std::vector<int> types;
  std::vector<tagint> tags;
  void add(const double *xi, const double *si, tagint t, int ty);
  void sync();   // refresh x / f / type / tag after adds
};
}  // namespace LAMMPS_NS
