// e3gnn_md_parallel -- the per-step call sequence of LAMMPS' pair_style
// e3gnn/parallel (pair_e3gnn_parallel.cpp:207-541: per-rank graph with ghost
// atoms -> per layer forward_comm of the ghost features -> segment forward ->
// readout -> per layer segment backward + reverse_comm of the ghost gradients
// -> forces + reverse_comm of the ghost forces) in native C++ over the segment
// C ABI of libe3gnn_hip.so, with no Python and no MPI: the N spatial
// sub-domains ("ranks", a px x py x pz brick grid) live in one process on one
// GPU, each with its own e3gnn_ctx, and the halo exchanges are device-side
// pack -> unpack copies (what comm_brick.cpp:1057-1120 does between MPI
// ranks).  The same graph is also evaluated serially (e3gnn_energy_forces)
// and the two results compared -- the compiled counterpart of the Python
// driver's decomposition tests (parallel.py).
//
//   e3gnn_md_parallel <weights.bin> <manifest.json> <cells | structure file> <px> <py> <pz> [reps] [sigma_A]
//
// System: cells^3 Si diamond cells (a = 5.43 A, cells >= 3 so that the box is
// wider than two cutoffs), positions displaced by N(0, sigma) (default 0.05 A,
// fixed seed) -- or any periodic structure (any deployed model, e.g. the
// reference's HfO2 example) from a text file: n, the 9 cell numbers (rows =
// lattice vectors), then n lines "symbol x y z"; its neighbour list is built
// over all periodic images (triclinic cells).  Prints one JSON line: atoms, ranks, ghosts, serial and
// decomposed energies, max |dF|, max |d virial|, and the device ms of one
// decomposed evaluation (mean over `reps`).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <map>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "e3gnn.h"

namespace {

void die(const char* what) {
  std::fprintf(stderr, "e3gnn_md_parallel: %s: %s\n", what, e3gnn_last_error());
  std::exit(1);
}

#define HIPOK(x)                                                                       \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "e3gnn_md_parallel: %s: %s\n", #x, hipGetErrorString(e_));  \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

int species_index(const std::string& manifest, const std::string& sym) {
  std::ifstream f(manifest);
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string s = ss.str();
  const size_t k = s.find("\"chemical_symbols\"");
  if (k == std::string::npos) return -1;
  const size_t a = s.find('[', k), b = s.find(']', a);
  int idx = 0;
  for (size_t p = a; p < b;) {
    const size_t q0 = s.find('"', p);
    if (q0 == std::string::npos || q0 > b) break;
    const size_t q1 = s.find('"', q0 + 1);
    if (s.compare(q0 + 1, q1 - q0 - 1, sym) == 0) return idx;
    ++idx;
    p = q1 + 1;
  }
  return -1;
}

template <class T>
T* dev_copy(const std::vector<T>& h) {
  T* d = nullptr;
  HIPOK(hipMalloc(&d, std::max<size_t>(h.size(), 1) * sizeof(T)));
  if (!h.empty()) HIPOK(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  return d;
}

// full periodic neighbour list of an orthorhombic box (edge i -> j, r < rc,
// minimum image: the box is wider than 2 rc), centre-sorted
struct Edge {
  int i, j;
  float v[3];
};
std::vector<Edge> neighbours(const std::vector<double>& x, double L, double rc) {
  const int n = (int)x.size() / 3;
  const int nb = std::max(1, (int)std::floor(L / rc));
  const double w = L / nb;
  std::vector<std::vector<int>> bins(nb * nb * nb);
  auto bin_of = [&](double c) {
    int b = (int)std::floor(c / w);
    return ((b % nb) + nb) % nb;
  };
  for (int i = 0; i < n; ++i)
    bins[(bin_of(x[3 * i]) * nb + bin_of(x[3 * i + 1])) * nb + bin_of(x[3 * i + 2])].push_back(i);
  std::vector<Edge> out;
  const int span = nb >= 3 ? 1 : 0;
  for (int i = 0; i < n; ++i) {
    const int bx = bin_of(x[3 * i]), by = bin_of(x[3 * i + 1]), bz = bin_of(x[3 * i + 2]);
    std::vector<Edge> mine;
    std::vector<int> seen;
    for (int dx = -span; dx <= span; ++dx)
      for (int dy = -span; dy <= span; ++dy)
        for (int dz = -span; dz <= span; ++dz) {
          const int cx = ((bx + dx) % nb + nb) % nb, cy = ((by + dy) % nb + nb) % nb,
                    cz = ((bz + dz) % nb + nb) % nb;
          for (int j : bins[(cx * nb + cy) * nb + cz]) {
            if (j == i) continue;
            if (span == 0 && std::find(seen.begin(), seen.end(), j) != seen.end()) continue;
            double d[3];
            for (int k = 0; k < 3; ++k) {
              d[k] = x[3 * j + k] - x[3 * i + k];
              d[k] -= L * std::round(d[k] / L);
            }
            const double r2 = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
            if (r2 < rc * rc) {
              mine.push_back({i, j, {(float)d[0], (float)d[1], (float)d[2]}});
              if (span == 0) seen.push_back(j);
            }
          }
        }
    std::sort(mine.begin(), mine.end(), [](const Edge& a, const Edge& b) { return a.j < b.j; });
    out.insert(out.end(), mine.begin(), mine.end());
  }
  return out;
}

// full periodic neighbour list of a general (triclinic) cell over all images
// within the cutoff (edge vec = x_j + S cell - x_i, i == j allowed for S != 0),
// centre-sorted, (j, S) order within a centre
std::vector<Edge> neighbours_cell(const std::vector<double>& x, const double (&cell)[3][3], double rc) {
  const int n = (int)x.size() / 3;
  auto cross = [](const double* a, const double* b, double* c) {
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
  };
  double c12[3], c20[3], c01[3];
  cross(cell[1], cell[2], c12);
  cross(cell[2], cell[0], c20);
  cross(cell[0], cell[1], c01);
  const double vol = std::fabs(cell[0][0] * c12[0] + cell[0][1] * c12[1] + cell[0][2] * c12[2]);
  const double* cr[3] = {c12, c20, c01};
  int nk[3];
  for (int k = 0; k < 3; ++k) {
    const double h = vol / std::sqrt(cr[k][0] * cr[k][0] + cr[k][1] * cr[k][1] + cr[k][2] * cr[k][2]);
    nk[k] = (int)std::ceil(rc / h) + 1;
  }
  std::vector<Edge> out;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j)
      for (int a = -nk[0]; a <= nk[0]; ++a)
        for (int b = -nk[1]; b <= nk[1]; ++b)
          for (int c = -nk[2]; c <= nk[2]; ++c) {
            if (i == j && a == 0 && b == 0 && c == 0) continue;
            double d[3];
            for (int k = 0; k < 3; ++k)
              d[k] = x[3 * j + k] + a * cell[0][k] + b * cell[1][k] + c * cell[2][k] - x[3 * i + k];
            if (d[0] * d[0] + d[1] * d[1] + d[2] * d[2] < rc * rc)
              out.push_back({i, j, {(float)d[0], (float)d[1], (float)d[2]}});
          }
  return out;
}

// one sub-domain: owned atoms (rows [0, n_local)), ghosts by (owner, id)
struct Rank {
  std::vector<int> owned, ghosts;           // global ids
  std::vector<int> ghost_owner;
  std::map<int, int> row_of;               // global id -> local row
  std::vector<int32_t> type, center, nbr;
  std::vector<float> vec;
  // per peer p: ghost rows of this rank owned by p ([g0, g1)) and, on p, the
  // local rows they mirror
  std::vector<int> gbeg, gend;
  std::vector<int32_t*> d_peer_rows;        // on the owner p: rows to send here
  std::vector<int32_t*> d_ghost_rows;       // here: ghost rows received from p
  int32_t *d_type = nullptr, *d_center = nullptr, *d_nbr = nullptr;
  float* d_vec = nullptr;
  e3gnn_ctx* ctx = nullptr;
};

}  // namespace

int main(int argc, char** argv) {
  if (argc < 7) {
    std::fprintf(stderr, "usage: %s weights.bin manifest.json cells px py pz [reps] [sigma]\n",
                 argv[0]);
    return 2;
  }
  const std::string sys_arg = argv[3];
  const bool from_file = sys_arg.find_first_not_of("0123456789") != std::string::npos;
  const int cells = from_file ? 3 : std::atoi(argv[3]);
  const int grid[3] = {std::atoi(argv[4]), std::atoi(argv[5]), std::atoi(argv[6])};
  const int reps = argc > 7 ? std::atoi(argv[7]) : 3;
  const double sigma = argc > 8 ? std::atof(argv[8]) : 0.05;
  const int nranks = grid[0] * grid[1] * grid[2];
  if (cells < 3 || nranks < 1) {
    std::fprintf(stderr, "e3gnn_md_parallel: need cells >= 3 and a positive grid\n");
    return 2;
  }
  e3gnn_model* model = e3gnn_load(argv[1], argv[2], 0);
  if (!model) die("e3gnn_load");
  int nsp = 0, nlayers = 0, comm = 0;
  float cutoff = 0.f;
  if (e3gnn_model_info(model, &nsp, &cutoff, &nlayers, &comm)) die("e3gnn_model_info");

  // ---- the system
  int n = 0;
  std::vector<double> x;
  std::vector<int32_t> species;
  double cell[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
  std::vector<Edge> edges;
  if (from_file) {
    std::ifstream f(sys_arg);
    if (!(f >> n) || n <= 0) die("structure file: atom count");
    for (int a = 0; a < 3; ++a)
      for (int k = 0; k < 3; ++k)
        if (!(f >> cell[a][k])) die("structure file: cell");
    x.resize(3 * (size_t)n);
    species.resize(n);
    for (int i = 0; i < n; ++i) {
      std::string sym;
      if (!(f >> sym >> x[3 * i] >> x[3 * i + 1] >> x[3 * i + 2])) die("structure file: atom line");
      species[i] = species_index(argv[2], sym);
      if (species[i] < 0) die(("species " + sym + " not in the manifest").c_str());
    }
    edges = neighbours_cell(x, cell, cutoff);
  } else {
    const int si = species_index(argv[2], "Si");
    if (si < 0) die("Si not in the manifest");
    const double a0 = 5.43, L = cells * a0;
    const double basis[8][3] = {{0, 0, 0},       {0, .5, .5},     {.5, 0, .5},     {.5, .5, 0},
                                {.25, .25, .25}, {.25, .75, .75}, {.75, .25, .75}, {.75, .75, .25}};
    n = 8 * cells * cells * cells;
    x.resize(3 * (size_t)n);
    species.assign(n, si);
    for (int k = 0; k < 3; ++k) cell[k][k] = L;
    std::mt19937 rng(7);
    std::normal_distribution<double> g(0.0, sigma);
    int q = 0;
    for (int i = 0; i < cells; ++i)
      for (int j = 0; j < cells; ++j)
        for (int k = 0; k < cells; ++k)
          for (int b = 0; b < 8; ++b, ++q) {
            const double p[3] = {(i + basis[b][0]) * a0, (j + basis[b][1]) * a0,
                                 (k + basis[b][2]) * a0};
            for (int c = 0; c < 3; ++c) x[3 * q + c] = std::fmod(p[c] + g(rng) + L, L);
          }
    edges = neighbours(x, L, cutoff);
  }
  const int64_t E = (int64_t)edges.size();

  hipStream_t s;
  HIPOK(hipStreamCreate(&s));

  // ---- serial reference (pair_e3gnn)
  std::vector<float> f_ser(3 * n), vir_ser(6);
  float e_ser = 0.f;
  {
    std::vector<int32_t> ty = species, c(E), nb(E);
    std::vector<float> v(3 * E);
    for (int64_t e = 0; e < E; ++e) {
      c[e] = edges[e].i;
      nb[e] = edges[e].j;
      for (int k = 0; k < 3; ++k) v[3 * e + k] = edges[e].v[k];
    }
    int32_t *dt = dev_copy(ty), *dc = dev_copy(c), *dn = dev_copy(nb);
    float* dv = dev_copy(v);
    float *de, *df, *dvir;
    HIPOK(hipMalloc(&de, 4));
    HIPOK(hipMalloc(&df, 12 * (size_t)n));
    HIPOK(hipMalloc(&dvir, 24));
    e3gnn_ctx* ctx = e3gnn_ctx_create(model);
    if (!ctx) die("e3gnn_ctx_create");
    if (e3gnn_energy_forces(ctx, n, E, dt, dc, dn, dv, de, nullptr, df, dvir, nullptr, s))
      die("e3gnn_energy_forces");
    HIPOK(hipMemcpy(&e_ser, de, 4, hipMemcpyDeviceToHost));
    HIPOK(hipMemcpy(f_ser.data(), df, 12 * (size_t)n, hipMemcpyDeviceToHost));
    HIPOK(hipMemcpy(vir_ser.data(), dvir, 24, hipMemcpyDeviceToHost));
    e3gnn_ctx_free(ctx);
    for (void* p : {(void*)dt, (void*)dc, (void*)dn, (void*)dv, (void*)de, (void*)df, (void*)dvir})
      HIPOK(hipFree(p));
  }

  // ---- decomposition: owner = brick of the wrapped fractional position
  double inv[3][3];  // frac = x inv (rows of `cell` are the lattice vectors)
  {
    const double(&m)[3][3] = cell;
    const double det = m[0][0] * (m[1][1] * m[2][2] - m[1][2] * m[2][1]) -
                       m[0][1] * (m[1][0] * m[2][2] - m[1][2] * m[2][0]) +
                       m[0][2] * (m[1][0] * m[2][1] - m[1][1] * m[2][0]);
    inv[0][0] = (m[1][1] * m[2][2] - m[1][2] * m[2][1]) / det;
    inv[0][1] = (m[0][2] * m[2][1] - m[0][1] * m[2][2]) / det;
    inv[0][2] = (m[0][1] * m[1][2] - m[0][2] * m[1][1]) / det;
    inv[1][0] = (m[1][2] * m[2][0] - m[1][0] * m[2][2]) / det;
    inv[1][1] = (m[0][0] * m[2][2] - m[0][2] * m[2][0]) / det;
    inv[1][2] = (m[0][2] * m[1][0] - m[0][0] * m[1][2]) / det;
    inv[2][0] = (m[1][0] * m[2][1] - m[1][1] * m[2][0]) / det;
    inv[2][1] = (m[0][1] * m[2][0] - m[0][0] * m[2][1]) / det;
    inv[2][2] = (m[0][0] * m[1][1] - m[0][1] * m[1][0]) / det;
  }
  std::vector<int> owner(n);
  for (int i = 0; i < n; ++i) {
    int b[3];
    for (int k = 0; k < 3; ++k) {
      double fr = x[3 * i] * inv[0][k] + x[3 * i + 1] * inv[1][k] + x[3 * i + 2] * inv[2][k];
      fr -= std::floor(fr);
      b[k] = std::min(grid[k] - 1, (int)(fr * grid[k]));
    }
    owner[i] = (b[0] * grid[1] + b[1]) * grid[2] + b[2];
  }
  std::vector<Rank> R(nranks);
  for (int i = 0; i < n; ++i) R[owner[i]].owned.push_back(i);
  std::vector<int> begin_of(n + 1, 0);
  for (const Edge& e : edges) begin_of[e.i + 1]++;
  for (int i = 0; i < n; ++i) begin_of[i + 1] += begin_of[i];
  int64_t ghosts_total = 0;
  for (int r = 0; r < nranks; ++r) {
    Rank& rk = R[r];
    for (size_t a = 0; a < rk.owned.size(); ++a) rk.row_of[rk.owned[a]] = (int)a;
    std::vector<std::pair<int, int>> gh;   // (owner, id)
    for (int i : rk.owned)
      for (int e = begin_of[i]; e < begin_of[i + 1]; ++e) {
        const int j = edges[e].j;
        if (owner[j] != r) gh.push_back({owner[j], j});
      }
    std::sort(gh.begin(), gh.end());
    gh.erase(std::unique(gh.begin(), gh.end()), gh.end());
    const int nl = (int)rk.owned.size();
    rk.gbeg.assign(nranks, 0);
    rk.gend.assign(nranks, 0);
    for (size_t a = 0; a < gh.size(); ++a) {
      rk.ghosts.push_back(gh[a].second);
      rk.ghost_owner.push_back(gh[a].first);
      rk.row_of[gh[a].second] = nl + (int)a;
    }
    for (int p = 0; p < nranks; ++p) {
      auto lo = std::lower_bound(gh.begin(), gh.end(), std::make_pair(p, -1));
      auto hi = std::lower_bound(gh.begin(), gh.end(), std::make_pair(p + 1, -1));
      rk.gbeg[p] = nl + (int)(lo - gh.begin());
      rk.gend[p] = nl + (int)(hi - gh.begin());
    }
    ghosts_total += (int64_t)gh.size();
    rk.type.resize(nl + gh.size());
    for (size_t a = 0; a < rk.owned.size(); ++a) rk.type[a] = species[rk.owned[a]];
    for (size_t a = 0; a < gh.size(); ++a) rk.type[nl + a] = species[gh[a].second];
    for (size_t a = 0; a < rk.owned.size(); ++a) {
      const int i = rk.owned[a];
      for (int e = begin_of[i]; e < begin_of[i + 1]; ++e) {
        rk.center.push_back((int32_t)a);
        rk.nbr.push_back(rk.row_of[edges[e].j]);
        for (int k = 0; k < 3; ++k) rk.vec.push_back(edges[e].v[k]);
      }
    }
    rk.d_type = dev_copy(rk.type);
    rk.d_center = dev_copy(rk.center);
    rk.d_nbr = dev_copy(rk.nbr);
    rk.d_vec = dev_copy(rk.vec);
    rk.ctx = e3gnn_ctx_create(model);
    if (!rk.ctx) die("e3gnn_ctx_create");
  }
  // send lists: rank p sends, for rank r's ghost block [gbeg[p], gend[p]), its
  // local rows of those atoms (the one-time handshake of parallel.py)
  for (int r = 0; r < nranks; ++r) {
    R[r].d_peer_rows.assign(nranks, nullptr);
    R[r].d_ghost_rows.assign(nranks, nullptr);
  }
  for (int r = 0; r < nranks; ++r)
    for (int p = 0; p < nranks; ++p) {
      const int g0 = R[r].gbeg[p], g1 = R[r].gend[p];
      if (g1 <= g0) continue;
      std::vector<int32_t> send, recv;
      for (int row = g0; row < g1; ++row) {
        const int id = R[r].ghosts[row - (int)R[r].owned.size()];
        send.push_back(R[p].row_of.at(id));
        recv.push_back(row);
      }
      R[p].d_peer_rows[r] = dev_copy(send);    // p -> r
      R[r].d_ghost_rows[p] = dev_copy(recv);
    }
  int64_t max_ghost_block = 1;
  for (int r = 0; r < nranks; ++r)
    for (int p = 0; p < nranks; ++p)
      max_ghost_block = std::max<int64_t>(max_ghost_block, R[r].gend[p] - R[r].gbeg[p]);
  float* d_buf = nullptr;
  const int maxdim = 1024;
  HIPOK(hipMalloc(&d_buf, (size_t)max_ghost_block * maxdim * 4));
  std::vector<float*> d_force(nranks), d_vir(nranks), d_e(nranks);
  for (int r = 0; r < nranks; ++r) {
    const size_t rows = R[r].owned.size() + R[r].ghosts.size();
    HIPOK(hipMalloc(&d_force[r], std::max<size_t>(rows, 1) * 12));
    HIPOK(hipMalloc(&d_vir[r], 24));
    HIPOK(hipMalloc(&d_e[r], 4));
  }

  // forward_comm: ghost rows of every rank <- their owners' rows
  auto forward_comm = [&](float* (*ptr)(e3gnn_ctx*, int), int t, int dim) {
    for (int r = 0; r < nranks; ++r)
      for (int p = 0; p < nranks; ++p) {
        const int64_t m = R[r].gend[p] - R[r].gbeg[p];
        if (m <= 0) continue;
        if (e3gnn_halo_pack(R[p].d_peer_rows[r], m, dim, ptr(R[p].ctx, t), dim, d_buf, s))
          die("e3gnn_halo_pack");
        if (e3gnn_halo_unpack(R[r].d_ghost_rows[p], m, dim, d_buf, ptr(R[r].ctx, t), dim, 0, s))
          die("e3gnn_halo_unpack");
      }
  };
  // reverse_comm: owners' rows += the ghost rows other ranks hold, by rank order
  auto reverse_comm = [&](float* (*ptr)(e3gnn_ctx*, int), int t, int dim) {
    for (int p = 0; p < nranks; ++p)
      for (int r = 0; r < nranks; ++r) {
        const int64_t m = R[r].gend[p] - R[r].gbeg[p];
        if (m <= 0) continue;
        if (e3gnn_halo_pack(R[r].d_ghost_rows[p], m, dim, ptr(R[r].ctx, t), dim, d_buf, s))
          die("e3gnn_halo_pack");
        if (e3gnn_halo_unpack(R[p].d_peer_rows[r], m, dim, d_buf, ptr(R[p].ctx, t), dim, 1, s))
          die("e3gnn_halo_unpack");
      }
  };

  std::vector<float> f_par(3 * n), vir_par(6);
  double e_par = 0;
  auto evaluate = [&]() {
    for (int r = 0; r < nranks; ++r) {
      Rank& rk = R[r];
      if (e3gnn_graph_set(rk.ctx, (int64_t)rk.owned.size(), (int64_t)rk.ghosts.size(),
                          (int64_t)rk.center.size(), rk.d_type, rk.d_center, rk.d_nbr, rk.d_vec,
                          s))
        die("e3gnn_graph_set");
    }
    for (int t = 0; t < nlayers; ++t) {
      if (t > 0) forward_comm(e3gnn_feature_ptr, t, e3gnn_feature_dim(R[0].ctx, t));
      for (int r = 0; r < nranks; ++r)
        if (e3gnn_layer_forward(R[r].ctx, t, s)) die("e3gnn_layer_forward");
    }
    for (int r = 0; r < nranks; ++r)
      if (e3gnn_readout(R[r].ctx, d_e[r], nullptr, s)) die("e3gnn_readout");
    for (int t = nlayers - 1; t >= 0; --t) {
      for (int r = 0; r < nranks; ++r)
        if (e3gnn_layer_backward(R[r].ctx, t, s)) die("e3gnn_layer_backward");
      if (t > 0) reverse_comm(e3gnn_grad_ptr, t, e3gnn_feature_dim(R[0].ctx, t));
    }
    for (int r = 0; r < nranks; ++r)
      if (e3gnn_forces(R[r].ctx, d_force[r], d_vir[r], nullptr, s)) die("e3gnn_forces");
    // ghost forces -> owners (newton on)
    for (int p = 0; p < nranks; ++p)
      for (int r = 0; r < nranks; ++r) {
        const int64_t m = R[r].gend[p] - R[r].gbeg[p];
        if (m <= 0) continue;
        if (e3gnn_halo_pack(R[r].d_ghost_rows[p], m, 3, d_force[r], 3, d_buf, s))
          die("e3gnn_halo_pack");
        if (e3gnn_halo_unpack(R[p].d_peer_rows[r], m, 3, d_buf, d_force[p], 3, 1, s))
          die("e3gnn_halo_unpack");
      }
  };
  hipEvent_t t0, t1;
  HIPOK(hipEventCreate(&t0));
  HIPOK(hipEventCreate(&t1));
  evaluate();   // warm-up (workspace allocation)
  HIPOK(hipStreamSynchronize(s));
  HIPOK(hipEventRecord(t0, s));
  for (int k = 0; k < reps; ++k) evaluate();
  HIPOK(hipEventRecord(t1, s));
  HIPOK(hipStreamSynchronize(s));
  float ms = 0.f;
  HIPOK(hipEventElapsedTime(&ms, t0, t1));
  std::fill(vir_par.begin(), vir_par.end(), 0.f);
  for (int r = 0; r < nranks; ++r) {
    float e, v[6];
    HIPOK(hipMemcpy(&e, d_e[r], 4, hipMemcpyDeviceToHost));
    HIPOK(hipMemcpy(v, d_vir[r], 24, hipMemcpyDeviceToHost));
    e_par += e;
    for (int k = 0; k < 6; ++k) vir_par[k] += v[k];
    std::vector<float> fr(3 * R[r].owned.size());
    HIPOK(hipMemcpy(fr.data(), d_force[r], fr.size() * 4, hipMemcpyDeviceToHost));
    for (size_t a = 0; a < R[r].owned.size(); ++a)
      for (int k = 0; k < 3; ++k) f_par[3 * R[r].owned[a] + k] = fr[3 * a + k];
  }
  double df = 0, dv = 0, vmax = 0;
  for (int i = 0; i < 3 * n; ++i) df = std::max(df, (double)std::fabs(f_par[i] - f_ser[i]));
  for (int k = 0; k < 6; ++k) {
    dv = std::max(dv, (double)std::fabs(vir_par[k] - vir_ser[k]));
    vmax = std::max(vmax, (double)std::fabs(vir_ser[k]));
  }
  std::printf("{\"n_atoms\": %d, \"n_edges\": %lld, \"ranks\": %d, \"grid\": [%d, %d, %d], "
              "\"ghosts\": %lld, \"energy_serial\": %.6f, \"energy_decomposed\": %.6f, "
              "\"energy_rel_diff\": %.3e, \"max_force_diff\": %.3e, \"max_virial_diff\": %.3e, "
              "\"max_virial\": %.4f, \"decomposed_ms\": %.3f}\n",
              n, (long long)E, nranks, grid[0], grid[1], grid[2], (long long)ghosts_total, e_ser,
              e_par, std::fabs(e_par - e_ser) / std::fabs(e_ser), df, dv, vmax, ms / std::max(reps, 1));
  for (auto& rk : R) e3gnn_ctx_free(rk.ctx);
  e3gnn_free(model);
  return 0;
}
