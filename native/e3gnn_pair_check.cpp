// e3gnn_pair_check -- the LAMMPS pair-style core (pair_e3gnn_core) driven by
// LAMMPS-shaped inputs, without LAMMPS: a displaced periodic Si box as LAMMPS
// holds it (local atoms with scrambled indices and tags, periodic-image ghost
// atoms carrying their owner's tag, full neighbour lists with a 1 A skin and
// NEIGHMASK bits set), evaluated
//   (1) by SerialStep (pair_style e3gnn/hip, pair_e3gnn.cpp:72-275), and
//   (2) by ParallelStep on px x py x pz brick sub-domains, one thread per rank,
//       the halo exchanges done through ParallelStep's comm rows with a
//       bulk-synchronous in-process Exchange and the ghost forces summed onto
//       their owners as LAMMPS' reverse communication does (newton on)
//       (pair_style e3gnn/parallel/hip, pair_e3gnn_parallel.cpp:207-933),
// against the library's own device neighbour list + e3gnn_energy_forces on the
// same positions.  Prints one JSON line with the largest differences.
//
//   e3gnn_pair_check <model dir> <cells> <px> <py> <pz> [seed]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "e3gnn.h"
#include "pair_e3gnn_core.h"

using namespace e3gnn_pair;

namespace {

constexpr int NEIGHMASK = 0x1FFFFFFF;
constexpr double SKIN = 1.0;

struct Barrier {
  std::mutex m;
  std::condition_variable cv;
  int n, count = 0, gen = 0;
  explicit Barrier(int n_) : n(n_) {}
  void wait() {
    std::unique_lock<std::mutex> lk(m);
    const int g = gen;
    if (++count == n) {
      count = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g; });
    }
  }
};

// A LAMMPS-shaped sub-domain: local rows then ghost rows
struct Domain {
  std::vector<double> xs;          // (nlocal + nghost) x 3
  std::vector<double*> xp;
  std::vector<int> type;           // 1-based
  std::vector<int64_t> tag;
  std::vector<int> ilist, numneigh;
  std::vector<std::vector<int>> neigh;
  std::vector<int*> firstneigh;
  int nlocal = 0, nghost = 0;
  NeighborView view() {
    xp.resize(xs.size() / 3);
    for (size_t i = 0; i < xp.size(); ++i) xp[i] = &xs[3 * i];
    firstneigh.resize(neigh.size());
    for (size_t i = 0; i < neigh.size(); ++i) firstneigh[i] = neigh[i].data();
    NeighborView v;
    v.inum = nlocal;
    v.ilist = ilist.data();
    v.numneigh = numneigh.data();
    v.firstneigh = firstneigh.data();
    v.x = xp.data();
    v.type = type.data();
    v.tag = tag.data();
    v.nlocal = nlocal;
    v.nghost = nghost;
    v.neighmask = NEIGHMASK;
    return v;
  }
};

// local = atoms whose wrapped position lies in brick (bx, by, bz) of the grid;
// ghosts = every periodic image of any atom within rc + skin of the brick that
// is not a local row (LAMMPS' ghost shell); indices scrambled, NEIGHMASK bits set
Domain make_domain(const std::vector<double>& pos, const std::vector<int64_t>& tags, double L,
                   const int grid[3], const int b[3], double rc, std::mt19937& rng) {
  const int n = (int)tags.size();
  const double cut = rc + SKIN;
  Domain d;
  double lo[3], hi[3];
  for (int k = 0; k < 3; ++k) {
    lo[k] = L * b[k] / grid[k];
    hi[k] = L * (b[k] + 1) / grid[k];
  }
  std::vector<int> local;
  for (int a = 0; a < n; ++a) {
    bool in = true;
    for (int k = 0; k < 3; ++k) {
      const double w = pos[3 * a + k] - L * std::floor(pos[3 * a + k] / L);
      in = in && w >= lo[k] && w < hi[k];
    }
    if (in) local.push_back(a);
  }
  std::shuffle(local.begin(), local.end(), rng);   // LAMMPS index order != tag order
  std::vector<std::array<double, 3>> gx;
  std::vector<int> gown;
  for (int a = 0; a < n; ++a)
    for (int sx = -1; sx <= 1; ++sx)
      for (int sy = -1; sy <= 1; ++sy)
        for (int sz = -1; sz <= 1; ++sz) {
          const int s[3] = {sx, sy, sz};
          double p[3];
          bool near = true, is_local_row = true;
          for (int k = 0; k < 3; ++k) {
            const double w = pos[3 * a + k] - L * std::floor(pos[3 * a + k] / L);
            p[k] = w + s[k] * L;
            near = near && p[k] >= lo[k] - cut && p[k] < hi[k] + cut;
            is_local_row = is_local_row && p[k] >= lo[k] && p[k] < hi[k];
          }
          if (near && !is_local_row) {
            gx.push_back({p[0], p[1], p[2]});
            gown.push_back(a);
          }
        }
  d.nlocal = (int)local.size();
  d.nghost = (int)gx.size();
  const int ntot = d.nlocal + d.nghost;
  d.xs.resize(3 * ntot);
  d.type.assign(ntot, 1);
  d.tag.resize(ntot);
  for (int r = 0; r < d.nlocal; ++r) {
    const int a = local[r];
    for (int k = 0; k < 3; ++k) d.xs[3 * r + k] = pos[3 * a + k] - L * std::floor(pos[3 * a + k] / L);
    d.tag[r] = tags[a];
  }
  for (int g = 0; g < d.nghost; ++g) {
    for (int k = 0; k < 3; ++k) d.xs[3 * (d.nlocal + g) + k] = gx[g][k];
    d.tag[d.nlocal + g] = tags[gown[g]];
  }
  d.ilist.resize(d.nlocal);
  for (int r = 0; r < d.nlocal; ++r) d.ilist[r] = d.nlocal - 1 - r;   // reversed list order
  d.neigh.assign(ntot, {});
  d.numneigh.assign(ntot, 0);
  const double c2 = cut * cut;
  for (int i = 0; i < d.nlocal; ++i) {
    for (int j = 0; j < ntot; ++j) {
      if (j == i) continue;
      double r2 = 0;
      for (int k = 0; k < 3; ++k) {
        const double dd = d.xs[3 * j + k] - d.xs[3 * i + k];
        r2 += dd * dd;
      }
      if (r2 < c2) d.neigh[i].push_back(j | ((j & 1) << 30));   // special bits, masked off
    }
    d.numneigh[i] = (int)d.neigh[i].size();
  }
  return d;
}

// bulk-synchronous halo exchange among in-process ranks (what LAMMPS' brick
// communication delivers to pack/unpack_*_comm_gnn)
struct InProcExchange : ParallelStep::Exchange {
  std::vector<ParallelStep*>* steps;
  std::vector<Domain>* doms;
  Barrier* bar;
  int me;
  // per owner rank o: device lists (my ghost rows of o's atoms, o's rows)
  std::vector<int32_t*> mine_d, owner_d;
  std::vector<int64_t> cnt;
  float* stage = nullptr;
  int64_t stage_cap = 0;
  void plan() {
    const int P = (int)steps->size();
    ParallelStep& s = *(*steps)[me];
    Domain& d = (*doms)[me];
    std::vector<std::vector<int32_t>> a(P), b(P);
    for (int r = (int)s.nlocal(); r < s.graph_size(); ++r) {
      // the ghost row's atom: find its owner rank / row by tag
      int64_t tg = -1;
      for (int i = 0; i < d.nlocal + d.nghost; ++i)
        if (s.graph_row(i) == r) {
          tg = d.tag[i];
          break;
        }
      for (int o = 0; o < P; ++o) {
        Domain& od = (*doms)[o];
        for (int i = 0; i < od.nlocal; ++i)
          if (od.tag[i] == tg) {
            a[o].push_back(r);
            b[o].push_back((*steps)[o]->graph_row(i));
          }
      }
    }
    mine_d.assign(P, nullptr);
    owner_d.assign(P, nullptr);
    cnt.assign(P, 0);
    for (int o = 0; o < P; ++o) {
      cnt[o] = (int64_t)a[o].size();
      if (!cnt[o]) continue;
      (void)hipMalloc(&mine_d[o], cnt[o] * 4);
      (void)hipMalloc(&owner_d[o], cnt[o] * 4);
      (void)hipMemcpy(mine_d[o], a[o].data(), cnt[o] * 4, hipMemcpyHostToDevice);
      (void)hipMemcpy(owner_d[o], b[o].data(), cnt[o] * 4, hipMemcpyHostToDevice);
    }
  }
  int staging(int64_t n, int dim) {
    if (n * dim > stage_cap) {
      if (stage) (void)hipFree(stage);
      stage_cap = n * dim;
      if (hipMalloc(&stage, stage_cap * 4) != hipSuccess) return 1;
    }
    return 0;
  }
  int forward(ParallelStep& s) override {
    bar->wait();   // every rank's comm rows hold its owned features
    for (size_t o = 0; o < cnt.size(); ++o) {
      if (!cnt[o]) continue;
      ParallelStep& os = *(*steps)[o];
      if (staging(cnt[o], s.comm_dim())) return 1;
      if (e3gnn_halo_pack(owner_d[o], cnt[o], s.comm_dim(), os.comm_rows(), s.comm_dim(), stage,
                          s.stream()))
        return 1;
      if (s.unpack(mine_d[o], cnt[o], stage, false)) return 1;
    }
    (void)hipStreamSynchronize((hipStream_t)s.stream());
    bar->wait();
    return 0;
  }
  int reverse(ParallelStep& s) override {
    bar->wait();   // every rank's comm rows hold its ghost rows' dE/dx
    // owners pull: rank `me` adds the rows the others hold for its atoms, in rank order
    const int P = (int)steps->size();
    for (int c = 0; c < P; ++c) {
      if (c == me) continue;
      InProcExchange* other = peers[c];
      const int64_t n = other->cnt[me];
      if (!n) continue;
      ParallelStep& cs = *(*steps)[c];
      if (staging(n, s.comm_dim())) return 1;
      if (e3gnn_halo_pack(other->mine_d[me], n, s.comm_dim(), cs.comm_rows(), s.comm_dim(), stage,
                          s.stream()))
        return 1;
      if (s.unpack(other->owner_d[me], n, stage, true)) return 1;
    }
    (void)hipStreamSynchronize((hipStream_t)s.stream());
    bar->wait();
    return 0;
  }
  std::vector<InProcExchange*> peers;
};

}  // namespace

int main(int argc, char** argv) {
  if (argc < 6) {
    std::fprintf(stderr, "usage: %s model_dir cells px py pz [seed]\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1];
  const int cells = std::atoi(argv[2]);
  const int grid[3] = {std::atoi(argv[3]), std::atoi(argv[4]), std::atoi(argv[5])};
  const unsigned seed = argc > 6 ? (unsigned)std::atoi(argv[6]) : 0u;
  try {
    Model model(dir, 0);
    const std::vector<int> map = model.type_map({"Si"});
    const double rc = model.cutoff();
    // displaced Si diamond, tags scrambled
    const double a0 = 5.43, L = cells * a0;
    const double basis[8][3] = {{0, 0, 0},       {0, .5, .5},     {.5, 0, .5},     {.5, .5, 0},
                                {.25, .25, .25}, {.25, .75, .75}, {.75, .25, .75}, {.75, .75, .25}};
    const int n = 8 * cells * cells * cells;
    std::mt19937 rng(seed);
    std::normal_distribution<double> disp(0.0, 0.1);
    std::vector<double> pos(3 * n);
    int q = 0;
    for (int i = 0; i < cells; ++i)
      for (int j = 0; j < cells; ++j)
        for (int k = 0; k < cells; ++k)
          for (int b = 0; b < 8; ++b, ++q) {
            pos[3 * q] = (i + basis[b][0]) * a0 + disp(rng);
            pos[3 * q + 1] = (j + basis[b][1]) * a0 + disp(rng);
            pos[3 * q + 2] = (k + basis[b][2]) * a0 + disp(rng);
          }
    std::vector<int64_t> tags(n);
    for (int a = 0; a < n; ++a) tags[a] = a + 1;
    std::shuffle(tags.begin(), tags.end(), rng);

    // ---- reference: device neighbour list + e3gnn_energy_forces, atoms in tag order
    std::vector<double> pos_t(3 * n);
    for (int a = 0; a < n; ++a)
      for (int k = 0; k < 3; ++k) pos_t[3 * (tags[a] - 1) + k] = pos[3 * a + k];
    std::vector<double> f_ref(3 * n);
    double e_ref = 0, v_ref[6];
    {
      e3gnn_ctx* ctx = e3gnn_ctx_create(model.handle());
      e3gnn_nlist* nl = e3gnn_nlist_create(0);
      double* dp;
      int32_t *dt, *dc, *dn;
      float *dv, *df, *ds;
      (void)hipMalloc(&dp, 3 * n * 8);
      (void)hipMemcpy(dp, pos_t.data(), 3 * n * 8, hipMemcpyHostToDevice);
      const double cell[9] = {L, 0, 0, 0, L, 0, 0, 0, L};
      const int pbc[3] = {1, 1, 1};
      int64_t E = 0;
      if (e3gnn_nlist_build(nl, n, dp, cell, pbc, rc, &E, nullptr)) throw std::runtime_error(e3gnn_last_error());
      (void)hipMalloc(&dc, E * 4);
      (void)hipMalloc(&dn, E * 4);
      (void)hipMalloc(&dv, E * 12);
      (void)hipMalloc(&dt, n * 4);
      (void)hipMalloc(&df, n * 12);
      (void)hipMalloc(&ds, 8 * 4);
      std::vector<int32_t> ty(n, map[1]);
      (void)hipMemcpy(dt, ty.data(), n * 4, hipMemcpyHostToDevice);
      if (e3gnn_nlist_fetch(nl, dc, dn, nullptr, dv, nullptr)) throw std::runtime_error(e3gnn_last_error());
      if (e3gnn_energy_forces(ctx, n, E, dt, dc, dn, dv, ds, nullptr, df, ds + 1, nullptr, nullptr))
        throw std::runtime_error(e3gnn_last_error());
      std::vector<float> hf(3 * n);
      float sc[7];
      (void)hipMemcpy(hf.data(), df, n * 12, hipMemcpyDeviceToHost);
      (void)hipMemcpy(sc, ds, 28, hipMemcpyDeviceToHost);
      for (int i = 0; i < 3 * n; ++i) f_ref[i] = hf[i];
      e_ref = sc[0];
      const float* v6 = sc + 1;
      const double vl[6] = {v6[0], v6[1], v6[2], v6[3], v6[5], v6[4]};
      for (int k = 0; k < 6; ++k) v_ref[k] = vl[k];
      for (void* p : {(void*)dp, (void*)dc, (void*)dn, (void*)dv, (void*)dt, (void*)df, (void*)ds})
        (void)hipFree(p);
      e3gnn_nlist_free(nl);
      e3gnn_ctx_free(ctx);
    }
    auto max_force_diff = [&](const std::vector<double>& f_tag) {
      double m = 0;
      for (int i = 0; i < 3 * n; ++i) m = std::max(m, std::fabs(f_tag[i] - f_ref[i]));
      return m;
    };
    auto max_vir_diff = [&](const double* v) {
      double m = 0;
      for (int k = 0; k < 6; ++k) m = std::max(m, std::fabs(v[k] - v_ref[k]));
      return m;
    };

    // ---- (1) serial pair style
    const int one[3] = {1, 1, 1}, zero[3] = {0, 0, 0};
    Domain d1 = make_domain(pos, tags, L, one, zero, rc, rng);
    SerialStep serial(model);
    std::vector<double> f1(3 * (d1.nlocal + d1.nghost), 0.0), eat1(d1.nlocal + d1.nghost, 0.0);
    std::vector<double*> f1p(d1.nlocal + d1.nghost);
    for (size_t i = 0; i < f1p.size(); ++i) f1p[i] = &f1[3 * i];
    PairOut o1;
    NeighborView v1 = d1.view();
    if (serial.compute(v1, map, f1p.data(), eat1.data(), o1)) throw std::runtime_error(serial.error());
    std::vector<double> f1_tag(3 * n);
    double esum1 = 0;
    for (int i = 0; i < d1.nlocal; ++i) {
      for (int k = 0; k < 3; ++k) f1_tag[3 * (d1.tag[i] - 1) + k] = f1[3 * i + k];
      esum1 += eat1[i];
    }

    // ---- (2) parallel pair style on brick sub-domains, one thread per rank
    const int P = grid[0] * grid[1] * grid[2];
    std::vector<Domain> doms;
    for (int bx = 0; bx < grid[0]; ++bx)
      for (int by = 0; by < grid[1]; ++by)
        for (int bz = 0; bz < grid[2]; ++bz) {
          const int b[3] = {bx, by, bz};
          doms.push_back(make_domain(pos, tags, L, grid, b, rc, rng));
        }
    std::vector<std::unique_ptr<ParallelStep>> owned;
    std::vector<ParallelStep*> steps;
    std::vector<NeighborView> views(P);
    int total_local = 0;
    for (int r = 0; r < P; ++r) {
      owned.emplace_back(new ParallelStep(model));
      steps.push_back(owned.back().get());
      views[r] = doms[r].view();
      if (steps[r]->build(views[r], map, n)) throw std::runtime_error(steps[r]->error());
      total_local += doms[r].nlocal;
    }
    if (total_local != n) throw std::runtime_error("bricks do not partition the atoms");
    Barrier bar(P);
    std::vector<InProcExchange> ex(P);
    for (int r = 0; r < P; ++r) {
      ex[r].steps = &steps;
      ex[r].doms = &doms;
      ex[r].bar = &bar;
      ex[r].me = r;
      ex[r].plan();
    }
    for (int r = 0; r < P; ++r)
      for (int c = 0; c < P; ++c) ex[r].peers.push_back(&ex[c]);
    std::vector<std::vector<double>> fr(P);
    std::vector<std::vector<double>> er(P);
    std::vector<PairOut> outs(P);
    std::vector<int> rcs(P, 0);
    std::vector<std::thread> th;
    for (int r = 0; r < P; ++r)
      th.emplace_back([&, r] {
        (void)hipSetDevice(0);
        const int nt = doms[r].nlocal + doms[r].nghost;
        fr[r].assign(3 * nt, 0.0);
        er[r].assign(nt, 0.0);
        std::vector<double*> fp(nt);
        for (int i = 0; i < nt; ++i) fp[i] = &fr[r][3 * i];
        rcs[r] = steps[r]->compute(ex[r], fp.data(), er[r].data(), outs[r]);
      });
    for (auto& t : th) t.join();
    for (int r = 0; r < P; ++r)
      if (rcs[r]) throw std::runtime_error("rank " + std::to_string(r) + ": " + steps[r]->error());
    // LAMMPS reverse communication (newton on): ghost forces onto their owners, by tag
    std::vector<double> f2_tag(3 * n, 0.0);
    double e2 = 0, esum2 = 0, v2[6] = {0, 0, 0, 0, 0, 0};
    for (int r = 0; r < P; ++r) {
      for (int i = 0; i < doms[r].nlocal + doms[r].nghost; ++i)
        for (int k = 0; k < 3; ++k) f2_tag[3 * (doms[r].tag[i] - 1) + k] += fr[r][3 * i + k];
      for (int i = 0; i < doms[r].nlocal; ++i) esum2 += er[r][i];
      e2 += outs[r].energy;
      for (int k = 0; k < 6; ++k) v2[k] += outs[r].virial[k];
    }
    std::printf("{\"n_atoms\": %d, \"ranks\": %d, \"edges_serial\": %lld, \"energy_ref\": %.8f, "
                "\"serial\": {\"energy_rel\": %.3e, \"max_force\": %.3e, \"max_virial\": %.3e, "
                "\"eatom_sum_rel\": %.3e}, "
                "\"parallel\": {\"energy_rel\": %.3e, \"max_force\": %.3e, \"max_virial\": %.3e, "
                "\"eatom_sum_rel\": %.3e}}\n",
                n, P, (long long)serial.last_edges(), e_ref, std::fabs(o1.energy - e_ref) / std::fabs(e_ref),
                max_force_diff(f1_tag), max_vir_diff(o1.virial), std::fabs(esum1 - e_ref) / std::fabs(e_ref),
                std::fabs(e2 - e_ref) / std::fabs(e_ref), max_force_diff(f2_tag), max_vir_diff(v2),
                std::fabs(esum2 - e_ref) / std::fabs(e_ref));
  } catch (const std::exception& e) {
    std::fprintf(stderr, "e3gnn_pair_check: %s\n", e.what());
    return 1;
  }
  return 0;
}
