// mini-LAMMPS test scaffold (see lmptype.h): a full neighbour list
#pragma once
#include <vector>

namespace LAMMPS_NS {
class NeighList {
 public:
  int inum = 0;
  int *ilist = nullptr, *numneigh = nullptr, **firstneigh = nullptr;
  std::vector<int> ilist_s, numneigh_s;
  std::vector<std::vector<int>> neigh_s;
  std::vector<int *> first_s;
};
}  // namespace LAMMPS_NS
