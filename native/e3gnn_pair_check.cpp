// e3gnn_pair_check -- the LAMMPS pair styles of native/lammps/ (the ADAPTOR
// sources themselves: pair_e3gnn_hip.cpp, pair_e3gnn_parallel_hip.cpp) run
// inside a mini-LAMMPS scaffold (native/lammps_mock/: Atom, NeighList, Pair and
// a CommBrick emulation whose ranks are threads of this process).
//
//   (0) reference: the library's device neighbour list + e3gnn_energy_forces
//       on the whole periodic box (atoms in tag order);
//   (1) pair_style e3gnn (PairE3GNN, pair_e3gnn.cpp:72-275) on one rank whose
//       ghosts come from CommBrick's six self swaps;
//   (2) pair_style e3gnn/parallel (PairE3GNNParallel, pair_e3gnn_parallel.cpp:
//       207-933) on px x py x pz bricks: CommBrick::borders() builds each
//       rank's ghosts swap by swap (corner atoms relayed through the ranks of
//       earlier dimensions), the pair's comm_preprocess runs the "false"
//       forward_comm through the *_init hooks, every layer's features go out
//       through forward_comm(pair) and the gradients come back through
//       reverse_comm(pair) (the reference's comm_brick.cpp:1057-1120), and the
//       ghost forces reach their owners through LAMMPS' own newton-on reverse
//       communication.
// Prints one JSON line: energies, largest force / virial differences, the comm
// counters (extra rows, relays, zero returns, trash rows) and whether a second
// compute() reproduced the first bit for bit.
//
//   e3gnn_pair_check <model dir> <structure> <px> <py> <pz> [seed] [--gpu-aware]
//   structure: si:<cells> (displaced Si diamond) or a file
//              "n \n 9 cell values (rows = lattice vectors) \n symbol x y z ..."
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <mutex>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "atom.h"
#include "comm_brick.h"
#include "domain.h"
#include "e3gnn.h"
#include "error.h"
#include "force.h"
#include "memory.h"
#include "neigh_list.h"
#include "neighbor.h"
#include "pair_e3gnn_core.h"
#include "pair_e3gnn_hip.h"
#include "pair_e3gnn_parallel.h"

using namespace LAMMPS_NS;

namespace {

constexpr double SKIN = 1.0;

struct Structure {
  int n = 0;
  double cell[9];
  std::vector<double> pos;            // n x 3
  std::vector<std::string> symbol;    // per atom
  std::vector<std::string> elements;  // LAMMPS type k + 1 = elements[k]
  std::vector<int> type;              // 1-based
  std::vector<tagint> tag;            // atom a carries tag[a]
};

Structure load_structure(const std::string& spec, std::mt19937& rng) {
  Structure s;
  if (spec.rfind("si:", 0) == 0) {
    const int cells = std::atoi(spec.c_str() + 3);
    const double a0 = 5.43, L = cells * a0;
    const double basis[8][3] = {{0, 0, 0},       {0, .5, .5},     {.5, 0, .5},     {.5, .5, 0},
                                {.25, .25, .25}, {.25, .75, .75}, {.75, .25, .75}, {.75, .75, .25}};
    std::normal_distribution<double> disp(0.0, 0.1);
    for (int i = 0; i < cells; ++i)
      for (int j = 0; j < cells; ++j)
        for (int k = 0; k < cells; ++k)
          for (int b = 0; b < 8; ++b) {
            s.pos.push_back((i + basis[b][0]) * a0 + disp(rng));
            s.pos.push_back((j + basis[b][1]) * a0 + disp(rng));
            s.pos.push_back((k + basis[b][2]) * a0 + disp(rng));
            s.symbol.push_back("Si");
          }
    s.n = 8 * cells * cells * cells;
    const double c[9] = {L, 0, 0, 0, L, 0, 0, 0, L};
    std::copy(c, c + 9, s.cell);
  } else {
    std::ifstream f(spec);
    if (!f) throw std::runtime_error("cannot open " + spec);
    f >> s.n;
    for (double& v : s.cell) f >> v;
    s.pos.resize(3 * (size_t)s.n);
    s.symbol.resize(s.n);
    for (int a = 0; a < s.n; ++a) f >> s.symbol[a] >> s.pos[3 * a] >> s.pos[3 * a + 1] >> s.pos[3 * a + 2];
    if (!f) throw std::runtime_error("malformed structure file " + spec);
  }
  for (int a = 0; a < s.n; ++a) {
    auto it = std::find(s.elements.begin(), s.elements.end(), s.symbol[a]);
    if (it == s.elements.end()) {
      s.elements.push_back(s.symbol[a]);
      it = s.elements.end() - 1;
    }
    s.type.push_back((int)(it - s.elements.begin()) + 1);
  }
  s.tag.resize(s.n);
  for (int a = 0; a < s.n; ++a) s.tag[a] = a + 1;
  std::shuffle(s.tag.begin(), s.tag.end(), rng);   // LAMMPS tags != file order
  return s;
}

struct RankOut {
  double energy = 0, virial[6] = {0, 0, 0, 0, 0, 0}, eatom = 0;
  std::vector<std::pair<tagint, std::array<double, 3>>> f;   // owned atoms
  e3gnn_pair::CommMaps::Stats st;
  int nghost = 0, graph = 0;
  bool same_again = true;
  std::string err;
};

// one emulated MPI rank: LAMMPS-style setup, pair_style / pair_coeff, then
// `repeat` force evaluations (each: borders, neighbour list, compute, reverse comm)
void run_rank(const Structure& S, const std::string& model_dir, const int grid[3], int me, World* world,
              bool parallel, int repeat, std::mutex* load_mutex, RankOut* out) {
  LAMMPS lmp;
  Memory mem;
  Error err;
  Atom atom;
  Neighbor neigh;
  Force force;
  Domain dom;
  lmp.memory = &mem;
  lmp.error = &err;
  lmp.atom = &atom;
  lmp.neighbor = &neigh;
  lmp.force = &force;
  lmp.domain = &dom;
  CommBrick comm(&lmp, world, me, grid);
  lmp.comm = &comm;
  dom.set_cell(S.cell);
  neigh.skin = SKIN;
  // owned atoms: wrapped lamda inside this brick
  for (int a = 0; a < S.n; ++a) {
    double s[3], x[3];
    dom.x2lamda(&S.pos[3 * a], s);
    bool mine = true;
    for (int d = 0; d < 3; ++d) {
      s[d] -= std::floor(s[d]);
      if (s[d] >= 1.0) s[d] -= 1.0;
      const int c = std::min(grid[d] - 1, (int)(s[d] * grid[d]));
      mine = mine && c == comm.myloc[d];
    }
    if (!mine) continue;
    dom.lamda2x(s, x);
    atom.add(x, s, S.tag[a], S.type[a]);
  }
  atom.nlocal = (int)atom.tags.size();
  atom.natoms = S.n;
  atom.ntypes = (int)S.elements.size();
  atom.sync();

  std::unique_ptr<Pair> pair;
  std::vector<std::string> args = {"*", "*"};
  if (parallel) args.push_back("4");   // segment count (ignored)
  args.push_back(model_dir);
  for (const auto& e : S.elements) args.push_back(e);
  std::vector<char*> argv;
  for (auto& a : args) argv.push_back(&a[0]);
  {
    std::lock_guard<std::mutex> lk(*load_mutex);
    if (parallel) pair.reset(new PairE3GNNParallel(&lmp));
    else pair.reset(new PairE3GNN(&lmp));
    pair->settings(0, nullptr);
    pair->coeff((int)argv.size(), argv.data());
  }
  pair->init_style();
  if (!neigh.requested_full) throw std::runtime_error("pair style did not request a full list");
  const double cut = pair->init_one(1, 1);
  comm.setup(cut + SKIN);
  NeighList list;
  std::vector<std::vector<double>> first;
  for (int it = 0; it < repeat; ++it) {
    comm.borders();
    neigh.build_full(&atom, cut, &list);
    pair->init_list(0, &list);
    std::fill(atom.fs.begin(), atom.fs.end(), 0.0);
    pair->compute(1 | 2, 1);
    comm.reverse_comm();   // ghost forces onto their owners (newton on)
    std::vector<double> f(atom.fs.begin(), atom.fs.begin() + 3 * (size_t)atom.nlocal);
    if (it == 0) {
      out->energy = pair->eng_vdwl;
      for (int k = 0; k < 6; ++k) out->virial[k] = pair->virial[k];
      for (int i = 0; i < atom.nlocal; ++i) {
        out->eatom += pair->eatom[i];
        out->f.push_back({atom.tag[i], {f[3 * i], f[3 * i + 1], f[3 * i + 2]}});
      }
      out->nghost = atom.nghost;
      if (parallel) {
        auto* pp = static_cast<PairE3GNNParallel*>(pair.get());
        out->st = pp->comm_maps()->stats();
      }
      first.push_back(f);
    } else {
      out->same_again = out->same_again && f == first[0] && pair->eng_vdwl == out->energy;
    }
  }
}

struct RunOut {
  double energy = 0, virial[6] = {0, 0, 0, 0, 0, 0}, eatom = 0;
  std::vector<double> f_tag;   // by tag - 1
  e3gnn_pair::CommMaps::Stats st;
  int64_t ghosts = 0;
  bool same_again = true;
};

RunOut run(const Structure& S, const std::string& dir, const int grid[3], bool parallel, int repeat) {
  const int P = grid[0] * grid[1] * grid[2];
  World world(P);
  std::mutex load_mutex;
  std::vector<RankOut> outs(P);
  std::vector<std::thread> th;
  for (int r = 0; r < P; ++r)
    th.emplace_back([&, r] {
      try {
        if (hipSetDevice(0) != hipSuccess) throw std::runtime_error("hipSetDevice");
        run_rank(S, dir, grid, r, &world, parallel, repeat, &load_mutex, &outs[r]);
      } catch (const std::exception& e) {
        outs[r].err = e.what();
        world.abort();
      }
    });
  for (auto& t : th) t.join();
  for (int r = 0; r < P; ++r)
    if (!outs[r].err.empty() && outs[r].err != "world aborted")
      throw std::runtime_error("rank " + std::to_string(r) + ": " + outs[r].err);
  RunOut R;
  R.f_tag.assign(3 * (size_t)S.n, 0.0);
  std::vector<int> seen(S.n, 0);
  for (auto& o : outs) {
    R.energy += o.energy;
    R.eatom += o.eatom;
    for (int k = 0; k < 6; ++k) R.virial[k] += o.virial[k];
    for (auto& [t, f] : o.f) {
      seen[t - 1]++;
      for (int k = 0; k < 3; ++k) R.f_tag[3 * (t - 1) + k] = f[k];
    }
    R.ghosts += o.nghost;
    R.same_again = R.same_again && o.same_again;
    R.st.swaps += o.st.swaps;
    R.st.sent += o.st.sent;
    R.st.relayed += o.st.relayed;
    R.st.extra_rows += o.st.extra_rows;
    R.st.zero_sends += o.st.zero_sends;
    R.st.trash_forward += o.st.trash_forward;
    R.st.trash_reverse += o.st.trash_reverse;
  }
  for (int a = 0; a < S.n; ++a)
    if (seen[a] != 1) throw std::runtime_error("the bricks do not partition the atoms");
  return R;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 6) {
    std::fprintf(stderr, "usage: %s model_dir structure px py pz [seed] [--gpu-aware]\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1];
  const int grid[3] = {std::atoi(argv[3]), std::atoi(argv[4]), std::atoi(argv[5])};
  unsigned seed = 0;
  for (int k = 6; k < argc; ++k) {
    if (!std::strcmp(argv[k], "--gpu-aware")) setenv("E3GNN_GPU_AWARE_MPI", "1", 1);
    else seed = (unsigned)std::atoi(argv[k]);
  }
  try {
    std::mt19937 rng(seed);
    const Structure S = load_structure(argv[2], rng);
    e3gnn_pair::Model model(dir, 0);
    const std::vector<int> map = model.type_map(S.elements);
    const double rc = model.cutoff();
    const int n = S.n;

    // ---- (0) the library's own neighbour list + evaluation, atoms in tag order
    std::vector<double> pos_t(3 * (size_t)n), f_ref(3 * (size_t)n);
    std::vector<int32_t> ty(n);
    for (int a = 0; a < n; ++a) {
      for (int k = 0; k < 3; ++k) pos_t[3 * (S.tag[a] - 1) + k] = S.pos[3 * a + k];
      ty[S.tag[a] - 1] = map[S.type[a]];
    }
    double e_ref = 0, v_ref[6];
    {
      e3gnn_ctx* ctx = e3gnn_ctx_create(model.handle());
      e3gnn_nlist* nl = e3gnn_nlist_create(0);
      double* dp;
      int32_t *dt, *dc, *dn;
      float *dv, *df, *ds;
      (void)hipMalloc(&dp, 3 * n * 8);
      (void)hipMemcpy(dp, pos_t.data(), 3 * n * 8, hipMemcpyHostToDevice);
      const int pbc[3] = {1, 1, 1};
      int64_t E = 0;
      if (e3gnn_nlist_build(nl, n, dp, S.cell, pbc, rc, &E, nullptr)) throw std::runtime_error(e3gnn_last_error());
      (void)hipMalloc(&dc, E * 4);
      (void)hipMalloc(&dn, E * 4);
      (void)hipMalloc(&dv, E * 12);
      (void)hipMalloc(&dt, n * 4);
      (void)hipMalloc(&df, n * 12);
      (void)hipMalloc(&ds, 8 * 4);
      (void)hipMemcpy(dt, ty.data(), n * 4, hipMemcpyHostToDevice);
      if (e3gnn_nlist_fetch(nl, dc, dn, nullptr, dv, nullptr)) throw std::runtime_error(e3gnn_last_error());
      if (e3gnn_energy_forces(ctx, n, E, dt, dc, dn, dv, ds, nullptr, df, ds + 1, nullptr, nullptr))
        throw std::runtime_error(e3gnn_last_error());
      std::vector<float> hf(3 * (size_t)n);
      float sc[7];
      (void)hipMemcpy(hf.data(), df, n * 12, hipMemcpyDeviceToHost);
      (void)hipMemcpy(sc, ds, 28, hipMemcpyDeviceToHost);
      for (int i = 0; i < 3 * n; ++i) f_ref[i] = hf[i];
      e_ref = sc[0];
      const float* v6 = sc + 1;   // (xx, yy, zz, xy, yz, zx) -> LAMMPS (xx, yy, zz, xy, xz, yz)
      const double vl[6] = {v6[0], v6[1], v6[2], v6[3], v6[5], v6[4]};
      for (int k = 0; k < 6; ++k) v_ref[k] = vl[k];
      for (void* p : {(void*)dp, (void*)dc, (void*)dn, (void*)dv, (void*)dt, (void*)df, (void*)ds})
        (void)hipFree(p);
      e3gnn_nlist_free(nl);
      e3gnn_ctx_free(ctx);
    }
    auto max_diff = [](const std::vector<double>& a, const std::vector<double>& b) {
      double m = 0;
      for (size_t i = 0; i < a.size(); ++i) m = std::max(m, std::fabs(a[i] - b[i]));
      return m;
    };
    auto max_vdiff = [](const double* a, const double* b) {
      double m = 0;
      for (int k = 0; k < 6; ++k) m = std::max(m, std::fabs(a[k] - b[k]));
      return m;
    };

    const int one[3] = {1, 1, 1};
    const RunOut ser = run(S, dir, one, false, 2);
    const RunOut par = run(S, dir, grid, true, 2);
    const double scale = std::fabs(e_ref);
    std::printf(
        "{\"n_atoms\": %d, \"ranks\": %d, \"energy_ref\": %.8f, \"max_virial_ref\": %.6e, "
        "\"serial\": {\"energy\": %.8f, \"energy_rel\": %.3e, \"max_force\": %.3e, \"max_virial\": %.3e, "
        "\"eatom_sum_rel\": %.3e, \"repeat_bitwise\": %s}, "
        "\"parallel\": {\"energy\": %.8f, \"energy_rel\": %.3e, \"max_force\": %.3e, \"max_virial\": %.3e, "
        "\"eatom_sum_rel\": %.3e, \"repeat_bitwise\": %s, \"vs_serial_energy_rel\": %.3e, "
        "\"vs_serial_max_force\": %.3e}, "
        "\"comm\": {\"ghosts\": %lld, \"swaps\": %lld, \"sent\": %lld, \"relayed\": %lld, \"extra_rows\": %lld, "
        "\"zero_sends\": %lld, \"trash_forward\": %lld, \"trash_reverse\": %lld}}\n",
        n, grid[0] * grid[1] * grid[2], e_ref, std::max(std::fabs(*std::max_element(v_ref, v_ref + 6)),
                                                       std::fabs(*std::min_element(v_ref, v_ref + 6))),
        ser.energy, std::fabs(ser.energy - e_ref) / scale, max_diff(ser.f_tag, f_ref), max_vdiff(ser.virial, v_ref),
        std::fabs(ser.eatom - e_ref) / scale, ser.same_again ? "true" : "false", par.energy,
        std::fabs(par.energy - e_ref) / scale, max_diff(par.f_tag, f_ref), max_vdiff(par.virial, v_ref),
        std::fabs(par.eatom - e_ref) / scale, par.same_again ? "true" : "false",
        std::fabs(par.energy - ser.energy) / scale, max_diff(par.f_tag, ser.f_tag), (long long)par.ghosts,
        (long long)par.st.swaps, (long long)par.st.sent, (long long)par.st.relayed, (long long)par.st.extra_rows,
        (long long)par.st.zero_sends, (long long)par.st.trash_forward, (long long)par.st.trash_reverse);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "e3gnn_pair_check: %s\n", e.what());
    return 1;
  }
  return 0;
}
