// mini-LAMMPS test scaffold (see lmptype.h): the periodic cell, rows = lattice
// vectors (x = lamda . h), every dimension periodic
#pragma once
namespace LAMMPS_NS {
class Domain {
 public:
  double h[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
  double hinv[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
  void set_cell(const double cell[9]);
  void x2lamda(const double *x, double *s) const;
  void lamda2x(const double *s, double *x) const;
};
}  // namespace LAMMPS_NS
