"""AtomGraphData dict keys -- the data contract of the reference
(sevenn/_keys.py:26-84), kept verbatim so dicts built for the reference
models are accepted unchanged."""
ATOMIC_NUMBERS = 'atomic_numbers'
POS = 'pos'
CELL = 'cell_lattice_vectors'
CELL_SHIFT = 'pbc_shift'
CELL_VOLUME = 'cell_volume'
EDGE_VEC = 'edge_vec'
EDGE_LENGTH = 'edge_length'
EDGE_IDX = 'edge_index'
ATOM_TYPE = 'atom_type'
NODE_FEATURE = 'x'
NODE_FEATURE_GHOST = 'x_ghost'
NODE_ATTR = 'node_attr'
EDGE_ATTR = 'edge_attr'
EDGE_EMBEDDING = 'edge_embedding'
ENERGY = 'total_energy'
FORCE = 'force_of_atoms'
STRESS = 'stress'
ATOMIC_ENERGY = 'atomic_energy'
PRED_TOTAL_ENERGY = 'inferred_total_energy'
PRED_PER_ATOM_ENERGY = 'inferred_per_atom_energy'
PRED_FORCE = 'inferred_force'
PRED_STRESS = 'inferred_stress'
NUM_ATOMS = 'num_atoms'
NUM_GHOSTS = 'num_ghosts'
NLOCAL = 'nlocal'
BATCH = 'batch'
SELF_CONNECTION_TEMP = 'self_cont_tmp'
INFO = 'data_info'
# this build: dE/dedge_vec per edge (ForceStressOutputFromEdge's intermediate)
EDGE_GRAD = 'edge_grad'
# this build: 0-dim bool tensor set by train.collate when edge_index is sorted
# by centre (stable, on the host); the captured fine-tune step then skips its
# device sort
EDGE_SORTED = 'edge_index_centre_sorted'
