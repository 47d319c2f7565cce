// mini-LAMMPS test scaffold (see lmptype.h)
#pragma once
namespace LAMMPS_NS {
class Force {
 public:
  int newton_pair = 1;
};
}  // namespace LAMMPS_NS
