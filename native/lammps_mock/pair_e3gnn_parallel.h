// mini-LAMMPS test scaffold: the header name the patched CommBrick includes
// (sevenn/pair_e3gnn/patch_lammps.sh installs the pair as pair_e3gnn_parallel.h)
#include "pair_e3gnn_parallel_hip.h"
