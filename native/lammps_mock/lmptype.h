// mini-LAMMPS test scaffold (NOT LAMMPS): the slice of LAMMPS' API that the
// pair styles in native/lammps/ use, so those sources compile and run in
// native/e3gnn_pair_check without a LAMMPS tree.  Signatures follow LAMMPS
// (stable_2Aug2023); behaviour is emulated in mini_lammps.cpp.
#pragma once
#include <cstdint>
#include <cstdio>

namespace LAMMPS_NS {
typedef int64_t bigint;
typedef int tagint;
static constexpr int NEIGHMASK = 0x1FFFFFFF;
}  // namespace LAMMPS_NS

#define FLERR __FILE__, __LINE__
