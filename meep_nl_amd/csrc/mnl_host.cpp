// mnl_host.cpp -- C-ABI (include/meep_nl_amd.h) and host orchestration of the
// MI355X fields::step() path.  Built with g++ (not hipcc) on purpose: the
// per-step source amplitudes use std::complex / libm exactly as the reference
// does (src/sources.cpp:72-160, src/step.cpp:296-319), so the values handed
// to the GPU are bit-identical to the reference's.
//
// Owns: structure description, PML chunk/zone tables (src/structure.cpp:
// 96-140, 509-523, 656-691), device allocation (one fp64 SoA buffer per
// component), the per-step launch sequence (src/step.cpp:35-140), point-source
// weights (src/loop_in_chunks.cpp:263-500) and get_field interpolation
// (src/vec.cpp:558-621, src/monitor.cpp:127-160).
#include "mnl_host.hpp"

namespace mnlh {
thread_local std::string g_err;
int g_verbosity = 1;

// ------------------------------------------------------------- PML zones
// structure::use_pml + effort volumes (src/structure.cpp:509-523, 118-137)
// and structure_chunk::use_pml (src/structure.cpp:656-691) folded into
// per-direction tables over the global half-coordinate q = p - io.
inline double pml_x(int i, double dx, double bloc, double a) {
  double here = i * 0.5 / a;
  return (0.5 / a * ((int)(dx * (2 * a) + 0.5) - (int)(fabs(bloc - here) * (2 * a) + 0.5)));
}


std::vector<ZoneIv> zone_intervals(const mnl_structure &S, int d) {
  std::vector<ZoneIv> iv;
  int n2 = 2 * S.n[d];
  int nlo = 0, nhi = 0;
  if (S.n[d] > 1 && S.pml_thick[d][0] > 0) nlo = int(S.pml_thick[d][0] * S.a + 1 + 0.5);
  if (S.n[d] > 1 && S.pml_thick[d][1] > 0) nhi = int(S.pml_thick[d][1] * S.a + 1 + 0.5);
  int lo_end = nlo ? 2 * nlo : 0, hi_start = nhi ? n2 - 2 * nhi : n2;
  if (nlo) iv.push_back({0, lo_end, 0});
  if (hi_start > lo_end) iv.push_back({lo_end, hi_start, 1});
  if (nhi) iv.push_back({hi_start, n2, 2});
  return iv;
}

int build_pml_tables(mnl_fields *F) {
  const mnl_structure &S = F->S;
  for (int d = 0; d < 3; d++) {
    if (!S.has[d]) continue;
    int nq = 2 * S.n[d] + 2;
    F->h_flag[d].assign(nq, 0);
    F->h_zone[d].assign(nq, 1);
    F->h_sig[d].assign(nq, 0.0);
    F->h_kap[d].assign(nq, 1.0);
    F->h_siginv[d].assign(nq, 1.0);
    auto ivs = zone_intervals(S, d);
    int nlo = 0, nhi = 0;
    for (auto &z : ivs) {
      if (z.zone == 0) nlo = 1;
      if (z.zone == 2) nhi = 1;
    }
    {  // PML chunks may touch (no interior chunk along d) but not overlap
      int lo_end = -1, hi_start = INT32_MAX;
      for (auto &z : ivs) {
        if (z.zone == 0) lo_end = z.c1;
        if (z.zone == 2) hi_start = z.c0;
      }
      if (nlo && nhi && lo_end > hi_start)
        return fail("PML layers overlap (2*int(thickness*a+1.5) > cells along a direction)");
    }
    for (auto &z : ivs) {
      // chunk-local profile, chunk io_c = io + c0, n_c = (c1-c0)/2
      int io_c = S.io[d] + z.c0, big_c = S.io[d] + z.c1;
      std::vector<double> sig, kap, siginv;
      bool flag = false;
      for (int side = 0; side < 2; side++) {
        double dx = S.pml_thick[d][side];
        if (dx <= 0.0 || S.n[d] <= 1) continue;
        double bloc = (side == 0 ? S.io[d] : S.io[d] + 2 * S.n[d]) * (0.5 * (1.0 / S.a));
        double prefac = (-log(S.pml_R[d][side])) / (4 * dx * (1. / 3.));
        double kappa_prefac = (S.pml_stretch[d][side] - 1) / (1. / 4.);
        bool found = false;
        for (int i = io_c; i <= big_c + 1; ++i)
          if (pml_x(i, dx, bloc, S.a) > 0) {
            found = true;
            break;
          }
        if (!found) continue;
        flag = true;
        int nc = big_c - io_c + 2;
        sig.assign(nc, 0.0);
        kap.assign(nc, 1.0);
        siginv.assign(nc, 1.0);
        for (int i = io_c; i <= big_c + 1; ++i) {
          int idx = i - io_c;
          double x = pml_x(i, dx, bloc, S.a);
          if (x > 0) {
            double u = x / dx;
            double sp = u * u;
            sig[idx] = 0.5 * F->dt * prefac * sp;
            kap[idx] = 1 + kappa_prefac * sp * (x / dx);
            siginv[idx] = 1 / (kap[idx] + sig[idx]);
          }
        }
      }
      // owned half-coords of this chunk: (c0, c1]
      for (int q = z.c0 + 1; q <= z.c1; q++) {
        F->h_zone[d][q] = (uint8_t)z.zone;
        if (flag) {
          F->h_flag[d][q] = 1;
          F->h_sig[d][q] = sig[q - z.c0];
          F->h_kap[d][q] = kap[q - z.c0];
          F->h_siginv[d][q] = siginv[q - z.c0];
        }
      }
      if (flag) F->pml_any[d] = true;
    }
  }
  return 0;
}

// ------------------------------------------------------------- grid / boxes
// Equal split of the slab-axis cells over ranks (first `rem` ranks get one more).
void slab_range(int ncell, int rank, int nranks, int *lo, int *hi) {
  int base = ncell / nranks, rem = ncell % nranks;
  *lo = rank * base + std::min(rank, rem);
  *hi = *lo + base + (rank < rem ? 1 : 0);
}

void setup_grid(mnl_fields *F) {
  const mnl_structure &S = F->S;
  DevGrid &g = F->g;
  memset(&g, 0, sizeof(g));
  g.dim = S.dim;
  int nax = 0;
  for (int d = 0; d < 3; d++) g.ax[d] = S.has[d] ? nax++ : -1;
  // slab direction = slowest present direction
  F->slab_dir = S.has[2] ? 2 : 1;
  int lo_cell = 0, hi_cell = S.n[F->slab_dir];
  slab_range(S.n[F->slab_dir], F->rank, F->nranks, &lo_cell, &hi_cell);
  int Nax[3] = {1, 1, 1};
  for (int d = 0; d < 3; d++) {
    if (!S.has[d]) continue;
    g.nglob[d] = S.n[d];
    g.wall[d] = 1;
    if (d == F->slab_dir) {
      g.off[d] = lo_cell;
      Nax[g.ax[d]] = hi_cell - lo_cell + 1;
      int nloc = hi_cell - lo_cell;
      g.owned_lo_sh[d] = 0;
      g.owned_hi_sh[d] = nloc - 1;
      g.owned_lo_un[d] = 1;
      g.owned_hi_un[d] = (hi_cell == S.n[d]) ? nloc - 1 : nloc;  // global wall plane excluded
    } else {
      g.off[d] = 0;
      Nax[g.ax[d]] = S.n[d] + 1;
      g.owned_lo_sh[d] = 0;
      g.owned_hi_sh[d] = S.n[d] - 1;
      g.owned_lo_un[d] = 1;
      g.owned_hi_un[d] = S.n[d] - 1;
    }
  }
  for (int k = 0; k < 3; k++) g.N[k] = Nax[k];
  long long p0 = (g.N[0] + 15) / 16 * 16;
  if (g.N[1] == 1 && g.N[2] == 1) p0 = g.N[0];
  g.st[0] = 1;
  g.st[1] = p0;
  g.st[2] = p0 * g.N[1];
  F->nlocal = size_t(p0) * g.N[1] * g.N[2];
  for (int d = 0; d < 3; d++) g.sdir[d] = g.ax[d] >= 0 ? g.st[g.ax[d]] : 0;
}

void make_shell_list(mnl_fields *F) {
  BoxList &bl = F->shell_list;
  memset(&bl, 0, sizeof(bl));
  long long acc = 0;
  for (auto &b : F->shell) {
    bool emp = false;
    for (int k = 0; k < 3; k++) emp = emp || b.hi[k] < b.lo[k];
    if (emp) continue;
    bl.b[bl.n] = b;
    bl.start[bl.n] = acc;
    acc += (long long)(b.hi[0] - b.lo[0] + 1) * (b.hi[1] - b.lo[1] + 1) * (b.hi[2] - b.lo[2] + 1);
    bl.n++;
  }
  bl.start[bl.n] = acc;
}

void setup_boxes(mnl_fields *F) {
  const mnl_structure &S = F->S;
  DevGrid &g = F->g;
  int ilo[3] = {0, 0, 0}, ihi[3] = {0, 0, 0};  // per device axis, local
  bool none = false;
  for (int d = 0; d < 3; d++) {
    if (!S.has[d]) continue;
    int n = S.n[d];
    std::vector<char> good(n + 1);
    for (int j = 0; j <= n; j++) {
      int q0 = 2 * j, q1 = 2 * j + 1;
      bool ok = F->h_flag[d][q0] == 0 && F->h_flag[d][q1] == 0;
      if (F->nr) ok = ok && F->h_zone[d][q0] == 1 && F->h_zone[d][q1] == 1;
      good[j] = ok;
    }
    int lo = 0;
    while (lo <= n && !good[lo]) lo++;
    int hi = n;
    while (hi >= 0 && !good[hi]) hi--;
    for (int j = lo; j <= hi; j++)
      if (!good[j]) lo = hi + 1;  // non-contiguous: no interior
    if (lo > hi) none = true;
    int a = g.ax[d];
    int l = lo - g.off[d], h = hi - g.off[d];
    l = std::max(l, 0);
    h = std::min(h, g.N[a] - 1);
    if (l > h) none = true;
    ilo[a] = l;
    ihi[a] = h;
  }
  Box full;
  for (int k = 0; k < 3; k++) full.lo[k] = 0, full.hi[k] = g.N[k] - 1;
  F->shell.clear();
  if (none) {
    F->interior = full;
    F->interior.hi[0] = -1;  // empty
    F->shell.push_back(full);
    return;
  }
  Box in = full;
  for (int k = 0; k < 3; k++)
    if (g.N[k] > 1 || ihi[k] >= ilo[k]) in.lo[k] = ilo[k], in.hi[k] = ihi[k];
  F->interior = in;
  // onion shell decomposition, slowest axis first
  Box cur = full;
  for (int k = 2; k >= 0; k--) {
    if (in.lo[k] > cur.lo[k]) {
      Box b = cur;
      b.hi[k] = in.lo[k] - 1;
      F->shell.push_back(b);
    }
    if (in.hi[k] < cur.hi[k]) {
      Box b = cur;
      b.lo[k] = in.hi[k] + 1;
      F->shell.push_back(b);
    }
    cur.lo[k] = in.lo[k];
    cur.hi[k] = in.hi[k];
  }
}

// ------------------------------------------------------------- allocation
bool is_like(int dim, int c1, int c2) {  // src/fields.cpp:473-491
  if (dim != 2) return true;
  auto tm = [](int c) {
    return c == MNL_HX || c == MNL_HY || c == MNL_BX || c == MNL_BY || c == MNL_EZ ||
           c == MNL_DZ;
  };
  return !(tm(c1) ^ tm(c2));
}
bool has_field(const mnl_structure &S, int c) {
  if (S.dim == 1) return c == MNL_EX || c == MNL_HY || c == MNL_DX || c == MNL_BY;
  return true;
}

void make_plans(mnl_fields *F) {
  // src/fields.cpp:438-471: comp d of B/D gets term1 (comp (d+2)%3 along (d+1)%3)
  // if that direction exists and the partner is allocated, term2 likewise.
  const mnl_structure &S = F->S;
  for (int t = 0; t < 2; t++) {
    CurlPlan &p = t == 0 ? F->planB : F->planD;
    int ft = t == 0 ? T_B : T_D, src = t == 0 ? T_E : T_H;
    for (int d = 0; d < 3; d++) {
      p.present[d] = F->allocated[3 * ft + d];
      int terms = 0;
      int c1 = (d + 2) % 3, dir1 = (d + 1) % 3, c2 = (d + 1) % 3, dir2 = (d + 2) % 3;
      if (S.has[dir1] && F->allocated[3 * src + c1]) terms |= 1;
      if (S.has[dir2] && F->allocated[3 * src + c2]) terms |= 2;
      p.terms[d] = terms;
      if (!terms) p.present[d] = 0;
    }
  }
  for (int d = 0; d < 3; d++) {
    F->f.ecomp_present[d] = F->allocated[3 * T_E + d];
    F->f.hcomp_present[d] = F->allocated[3 * T_H + d];
  }
}

int alloc_component(mnl_fields *F, int c) {
  int t = ctype(c), d = cdir(c);
  if (F->allocated[c]) return 0;
  double **slot = nullptr;
  switch (t) {
    case T_E: slot = &F->f.E[d]; break;
    case T_D: slot = &F->f.D[d]; break;
    case T_B: slot = &F->f.B[d]; break;
    case T_H: slot = nullptr; break;
  }
  if (slot && !*slot)
    if (dev_alloc(F, slot, F->nlocal)) return -1;
  if (t == T_D) F->f.Dn[d] = F->f.D[d];
  if (t == T_H) {
    if (!F->f.B[d] && dev_alloc(F, &F->f.B[d], F->nlocal)) return -1;
    F->f.Bn[d] = F->f.B[d];
    // H separate in chunks with PML along d (src/update_eh.cpp:204-209); with H-side
    // materials stored everywhere (a copy of B where the chunk aliases it)
    if (F->pml_any[d] || F->hall)
      if (dev_alloc(F, &F->f.H[d], F->nlocal)) return -1;
    if (F->pml_any[d])
      if (dev_alloc(F, &F->f.WH[d], F->nlocal)) return -1;
  }
  if (t == T_B) F->f.Bn[d] = F->f.B[d];
  if (t == T_E) F->f.En[d] = F->f.E[d];
  if (t == T_H) F->f.Hn[d] = F->f.H[d];
  if (t == T_E && F->pml_any[d] && !F->f.WE[d])
    if (dev_alloc(F, &F->f.WE[d], F->nlocal)) return -1;
  if (t == T_B || t == T_D) {
    int du = (d + 2) % 3;  // dsigu = cycle(d,2): f_u auxiliary (src/step_db.cpp:71-75)
    double **u = t == T_B ? &F->f.UB[d] : &F->f.UD[d];
    if (F->S.has[du] && F->pml_any[du] && !*u)
      if (dev_alloc(F, u, F->nlocal)) return -1;
    if (t == T_B) F->f.UBn[d] = F->f.UB[d];
  }
  F->allocated[c] = true;
  return 0;
}

int require_component(mnl_fields *F, int c) {  // src/fields.cpp:566-586
  for (int ca = 0; ca < MNL_NUM_COMPONENTS; ca++) {
    if (!has_field(F->S, ca) || !is_like(F->S.dim, c, ca)) continue;
    if (alloc_component(F, ca)) return -1;
  }
  // polarizations: P for every allocated E comp with nontrivial sigma
  for (int k = 0; k < F->f.npol; k++) {
    const Lorentz &L = F->S.lor[F->S.lor.size() - 1 - k];
    PolDev &pd = F->f.pol[k];
    for (int d = 0; d < 3; d++)
      if (F->allocated[d] && !L.sigma[d].empty() && pd.sigma[d] && !pd.P[d]) {
        if (dev_alloc(F, &pd.P[d], F->nlocal)) return -1;
        if (dev_alloc(F, &pd.Pp[d], F->nlocal)) return -1;
      }
  }
  // magnetic polarizations: P of every allocated H comp with nontrivial sigma; then
  // f_minus_p of B exists in every chunk (needs_P uses the global sigma flags,
  // src/update_eh.cpp:84-100), so H is separate everywhere (src/update_eh.cpp:204-209)
  for (int k = 0; k < F->f.nhpol; k++) {
    const Lorentz &L = F->S.hlor[F->S.hlor.size() - 1 - k];
    PolDev &pd = F->f.hpol[k];
    for (int d = 0; d < 3; d++)
      if (F->allocated[3 * T_H + d] && !L.sigma[d].empty() && pd.sigma[d] && !pd.P[d]) {
        if (dev_alloc(F, &pd.P[d], F->nlocal)) return -1;
        if (dev_alloc(F, &pd.Pp[d], F->nlocal)) return -1;
        F->f.hsep_all = 1;
      }
  }
  make_plans(F);
  return 0;
}

// upload a canonical host array into a device-layout buffer of this rank
int upload_canonical(mnl_fields *F, double *dst, const std::vector<double> &host, int comp) {
  size_t nt = F->S.ntot;
  if (F->scratch_cap < nt) {
    if (F->d_scratch) hipFree(F->d_scratch);
    HIPCHK(hipMalloc(&F->d_scratch, nt * sizeof(double)));
    F->scratch_cap = nt;
  }
  HIPCHK(hipMemcpyAsync(F->d_scratch, host.data(), nt * sizeof(double), hipMemcpyHostToDevice,
                        F->stream));
  if (k_from_canonical(dst, F->d_scratch, F->g, ctype(comp), cdir(comp), 0, F->stream))
    return fail("from_canonical kernel launch failed");
  HIPCHK(hipStreamSynchronize(F->stream));
  return 0;
}

bool all_eq(const std::vector<double> &v, double x) {
  for (double y : v)
    if (y != x) return false;
  return true;
}

// Is a chi1inv row entry nontrivial inside the reference chunk that covers
// zone box (zx,zy,zz)?  Chunk array points: [io_c+shift, big_c+shift]
// (src/anisotropic_averaging.cpp:246-296 trivial test over LOOP_OVER_VOL).
bool nontrivial_in_zone(const mnl_structure &S, const std::vector<double> &arr, int comp,
                        const ZoneIv *zv[3], double trivial) {
  int lo[3], hi[3];
  for (int d = 0; d < 3; d++) {
    if (!S.has[d]) {
      lo[d] = hi[d] = 0;
      continue;
    }
    // points j with io+2j+sh in [io + c0 + sh, io + c1 + sh]  <=>  j in [c0/2, c1/2]
    lo[d] = zv[d]->c0 / 2;
    hi[d] = zv[d]->c1 / 2;
  }
  for (int x = lo[0]; x <= hi[0]; x++)
    for (int y = lo[1]; y <= hi[1]; y++)
      for (int z = lo[2]; z <= hi[2]; z++) {
        long long i = x * S.cstride(0) + y * S.cstride(1) + z * S.cstride(2);
        if (arr[i] != trivial) return true;
      }
  (void)comp;
  return false;
}

std::vector<ZoneIv> zone_ivs_or_one(const mnl_structure &S, int d) {
  if (S.has[d]) return zone_intervals(S, d);
  return {{0, 0, 1}};
}

// Conductivity of the D and B components: cnd and cndinv = 1/(1 + cnd*dt*0.5)
// (structure_chunk::update_condinv, src/structure.cpp:693-707) where nonzero
// anywhere; f_cond where a PML lies along dsig = cycle(d, 1); per reference
// chunk, whether its conductivity array survives the trivial test
// (src/structure.cpp:898-901) -- that selects the f_cond branch of step_curl.
int setup_conductivity(mnl_fields *F) {
  const mnl_structure &S = F->S;
  DevFields &f = F->f;
  std::vector<uint8_t> cz(27, 0);
  bool any = false;
  for (int t = 0; t < 2; t++)
    for (int d = 0; d < 3; d++) {
      const int comp = 3 * (t ? T_D : T_B) + d;
      const auto &cv = S.cond[t][d];
      if (!has_field(S, comp) || cv.empty() || all_eq(cv, 0.0)) continue;
      any = true;
      std::vector<double> inv(cv.size());
      for (size_t i = 0; i < cv.size(); i++) inv[i] = 1 / (1 + cv[i] * F->dt * 0.5);
      double *pc, *pi;
      if (dev_alloc(F, &pc, F->nlocal) || dev_alloc(F, &pi, F->nlocal)) return -1;
      if (upload_canonical(F, pc, cv, comp) || upload_canonical(F, pi, inv, comp)) return -1;
      f.cnd[t][d] = pc;
      f.cndinv[t][d] = pi;
      const int dsig = (d + 1) % 3;
      if (S.has[dsig] && F->pml_any[dsig] && dev_alloc(F, &f.fcnd[t][d], F->nlocal)) return -1;
      auto ivx = zone_ivs_or_one(S, 0), ivy = zone_ivs_or_one(S, 1), ivz = zone_ivs_or_one(S, 2);
      for (auto &zx : ivx)
        for (auto &zy : ivy)
          for (auto &zz : ivz) {
            const ZoneIv *zv[3] = {&zx, &zy, &zz};
            if (nontrivial_in_zone(S, cv, comp, zv, 0.0))
              cz[zx.zone * 9 + zy.zone * 3 + zz.zone] |= 1 << (3 * t + d);
          }
    }
  f.cnd_dt2 = F->dt * 0.5;
  if (!any) return 0;
  uint8_t *dcz;
  if (dev_alloc(F, &dcz, 27)) return -1;
  HIPCHK(hipMemcpyAsync(dcz, cz.data(), 27, hipMemcpyHostToDevice, F->stream));
  HIPCHK(hipStreamSynchronize(F->stream));
  f.cnd_zone = dcz;
  return 0;
}

// H-side materials: chi1inv of the H components (set_mu) and
// magnetic Lorentzian susceptibilities.  The fork's update_eh(H_stuff) takes
// step_update_EDHB's diagonal branch whatever off-diagonal rows exist (its 3x3 branch
// needs chi3, which no H component has, src/step_generic.cpp:730-906), so only the
// diagonal enters the arithmetic; the rows still decide per reference chunk whether H is
// separate from B (chi1inv[H_c][c] kept: the diagonal given and some entry of the row
// nontrivial in the chunk, src/anisotropic_averaging.cpp:279-296, src/update_eh.cpp:204-209).
int setup_h_materials(mnl_fields *F) {
  const mnl_structure &S = F->S;
  DevFields &f = F->f;
  bool mu_any = false, hl_any = false, off_any = false;
  for (int c = 0; c < 3; c++) {
    if (!has_field(S, 3 * T_H + c)) continue;
    for (int d = 0; d < 3; d++) {
      const auto &v = S.mu1inv[c][d];
      if (v.empty() || all_eq(v, d == c ? 1.0 : 0.0)) continue;
      mu_any = true;
      off_any = off_any || d != c;
    }
  }
  for (const Lorentz &L : S.hlor)
    for (int d = 0; d < 3; d++)
      hl_any = hl_any || (!L.sigma[d].empty() && has_field(S, 3 * T_H + d));
  F->hall = mu_any || hl_any;
  f.hall = F->hall ? 1 : 0;
  if (!F->hall) return 0;
  if (S.nl_mode == 1 && off_any)  // upstream Meep would average them in (OFFDIAG)
    return fail("off-diagonal mu is not supported in the upstream nonlinear mode");
  if ((int)S.hlor.size() > MAX_HPOL) return fail("too many magnetic susceptibilities (max 2)");
  for (int c = 0; c < 3; c++) {
    const auto &diag = S.mu1inv[c][c];
    if (!has_field(S, 3 * T_H + c) || diag.empty() || all_eq(diag, 1.0)) continue;
    double *p;
    if (dev_alloc(F, &p, F->nlocal)) return -1;
    if (upload_canonical(F, p, diag, 3 * T_H + c)) return -1;
    f.invmu[c] = p;
  }
  std::vector<uint8_t> hz(27, 0);
  auto ivx = zone_ivs_or_one(S, 0), ivy = zone_ivs_or_one(S, 1), ivz = zone_ivs_or_one(S, 2);
  for (auto &zx : ivx)
    for (auto &zy : ivy)
      for (auto &zz : ivz) {
        const ZoneIv *zv[3] = {&zx, &zy, &zz};
        for (int c = 0; c < 3; c++) {
          if (!has_field(S, 3 * T_H + c) || S.mu1inv[c][c].empty()) continue;
          bool nt = false;
          for (int d = 0; d < 3 && !nt; d++) {
            const auto &v = S.mu1inv[c][d];
            nt = !v.empty() && nontrivial_in_zone(S, v, 3 * T_H + c, zv, d == c ? 1.0 : 0.0);
          }
          if (nt) hz[zx.zone * 9 + zy.zone * 3 + zz.zone] |= 1 << c;
        }
      }
  uint8_t *dz;
  if (dev_alloc(F, &dz, 27)) return -1;
  HIPCHK(hipMemcpyAsync(dz, hz.data(), 27, hipMemcpyHostToDevice, F->stream));
  f.hsep_zone = dz;
  F->h_hsep_zone = hz;
  // magnetic pol list: reverse add order (as the E side)
  const int nh = (int)S.hlor.size();
  f.nhpol = nh;
  for (int k = 0; k < nh; k++) {
    const Lorentz &L = S.hlor[nh - 1 - k];
    PolDev &pd = f.hpol[k];
    const double omega2pi = 2 * pi * L.omega0, g2pi = L.gamma * 2 * pi;
    pd.omega0dtsqr = omega2pi * omega2pi * F->dt * F->dt;
    pd.gamma1inv = 1 / (1 + g2pi * F->dt / 2);
    pd.gamma1 = (1 - g2pi * F->dt / 2);
    pd.omega0dtsqr_denom = L.drude ? 0 : pd.omega0dtsqr;
    for (int d = 0; d < 3; d++) {
      if (L.sigma[d].empty() || !has_field(S, 3 * T_H + d)) continue;
      double *p;
      if (dev_alloc(F, &p, F->nlocal)) return -1;
      if (upload_canonical(F, p, L.sigma[d], 3 * T_H + d)) return -1;
      pd.sigma[d] = p;
    }
  }
  HIPCHK(hipStreamSynchronize(F->stream));
  return 0;
}

int setup_materials(mnl_fields *F) {
  const mnl_structure &S = F->S;
  DevFields &f = F->f;
  // Newton-Raphson needed? chi2 nontrivial and both off-diagonal rows present.
  F->nr = false;
  F->upnl = false;
  if (S.nl_mode == 1) {  // upstream Meep: Pade chi2/chi3 on every E point, no NR
    for (int c = 0; c < 3; c++)
      for (const auto *v : {&S.chi2[c], &S.chi3[c]})
        if (!v->empty() && !all_eq(*v, 0.0)) F->upnl = true;
    for (auto &b : S.boxes) F->upnl = F->upnl || ((b.kind == 1 || b.kind == 2) && b.value != 0.0);
    // off-diagonal chi1inv rows: the upstream OFFDIAG averages (step_generic.cpp:597-598)
    for (int c = 0; c < 3; c++)
      for (int k = 1; k <= 2; k++) {
        const auto &od = S.chi1inv[c][(c + k) % 3];
        if (!od.empty() && !all_eq(od, 0.0)) F->upnl = true;
      }
  }
  auto has_offd = [&](int c) {
    for (int k = 1; k <= 2; k++) {
      const auto &od = S.chi1inv[c][(c + k) % 3];
      if (!od.empty() && !all_eq(od, 0.0)) return true;
    }
    return false;
  };
  // chi2 nontrivial on component c: a host array or a chi2 box (rasterised below)
  bool box_chi2 = false;
  for (auto &b : S.boxes) box_chi2 = box_chi2 || (b.kind == 1 && b.value != 0.0);
  auto chi2_nt = [&](int c) { return box_chi2 || (!S.chi2[c].empty() && !all_eq(S.chi2[c], 0.0)); };
  for (int c = 0; c < 3 && !F->upnl; c++) {
    if (!chi2_nt(c)) continue;
    int d1 = (c + 1) % 3, d2 = (c + 2) % 3;
    if (!S.chi1inv[c][d1].empty() && !all_eq(S.chi1inv[c][d1], 0.0) &&
        !S.chi1inv[c][d2].empty() && !all_eq(S.chi1inv[c][d2], 0.0))
      F->nr = true;
  }
  bool box_eps = false;
  for (auto &b : S.boxes) box_eps = box_eps || b.kind == 0;
  for (int c = 0; c < 3; c++) {
    if (!has_field(S, c)) continue;
    const auto &diag = S.chi1inv[c][c];
    bool need = (!diag.empty() && !all_eq(diag, 1.0)) || F->nr || box_eps ||
                (F->upnl && has_offd(c));
    if (need) {
      double *p;
      if (dev_alloc(F, &p, F->nlocal)) return -1;
      if (!diag.empty()) {
        if (upload_canonical(F, p, diag, c)) return -1;
      } else if (k_fill(p, 1.0, F->nlocal, F->stream))
        return fail("fill failed");
      f.inveps[c] = p;
    }
    if (F->nr || F->upnl) {
      for (int k = 0; k < 2; k++) {
        int dd = (c + 1 + k) % 3;
        const auto &od = S.chi1inv[c][dd];
        if (od.empty() || (F->upnl && all_eq(od, 0.0))) continue;
        double *p;
        if (dev_alloc(F, &p, F->nlocal)) return -1;
        if (upload_canonical(F, p, od, c)) return -1;
        f.offd[c][k] = p;
      }
    }
    if (F->nr && chi2_nt(c)) {
      double *p;
      if (dev_alloc(F, &p, F->nlocal)) return -1;  // zeroed: boxes are filled in below
      if (!S.chi2[c].empty() && upload_canonical(F, p, S.chi2[c], c)) return -1;
      f.chi2[c] = p;
    }
    if (F->upnl) {  // both arrays on every E component (zeros where absent)
      const std::vector<double> *src[2] = {&S.chi2[c], &S.chi3[c]};
      for (int k = 0; k < 2; k++) {
        double *p;
        if (dev_alloc(F, &p, F->nlocal)) return -1;
        if (!src[k]->empty() && upload_canonical(F, p, *src[k], c)) return -1;
        (k == 0 ? f.chi2[c] : f.chi3[c]) = p;
      }
    }
  }
  // offdiag presence per reference chunk (zone box)
  std::vector<uint8_t> oz(27, 0);
  if (F->nr || F->upnl) {
    std::vector<ZoneIv> ivs[3];
    for (int d = 0; d < 3; d++) {
      if (S.has[d])
        ivs[d] = zone_intervals(S, d);
      else
        ivs[d] = {{0, 0, 1}};
    }
    for (auto &zx : ivs[0])
      for (auto &zy : ivs[1])
        for (auto &zz : ivs[2]) {
          const ZoneIv *zv[3] = {&zx, &zy, &zz};
          int zb = zx.zone * 9 + zy.zone * 3 + zz.zone;
          for (int c = 0; c < 3; c++)
            for (int k = 0; k < 2; k++) {
              int dd = (c + 1 + k) % 3;
              const auto &od = S.chi1inv[c][dd];
              if (!od.empty() && nontrivial_in_zone(S, od, c, zv, 0.0)) oz[zb] |= 1 << (3 * c + k);
            }
        }
  }
  uint8_t *doz;
  if (dev_alloc(F, &doz, 27)) return -1;
  HIPCHK(hipMemcpyAsync(doz, oz.data(), 27, hipMemcpyHostToDevice, F->stream));
  f.offd_zone = doz;
  if (setup_conductivity(F)) return -1;
  f.nr_enabled = F->nr ? 1 : 0;
  f.upnl = F->upnl ? 1 : 0;
  // Lorentzian susceptibilities: pol list = reverse add order
  // (src/anisotropic_averaging.cpp:368-369, src/fields.cpp:266-282)
  int nl = (int)S.lor.size();
  if (nl > MAX_POL) return fail("too many susceptibilities");
  f.npol = nl;
  bool box_sig = false;
  for (auto &b : S.boxes) box_sig = box_sig || b.kind == 3;
  for (int k = 0; k < nl; k++) {
    const Lorentz &L = S.lor[nl - 1 - k];
    PolDev &pd = f.pol[k];
    const double omega2pi = 2 * pi * L.omega0, g2pi = L.gamma * 2 * pi;
    pd.omega0dtsqr = omega2pi * omega2pi * F->dt * F->dt;
    pd.gamma1inv = 1 / (1 + g2pi * F->dt / 2);
    pd.gamma1 = (1 - g2pi * F->dt / 2);
    pd.omega0dtsqr_denom = L.drude ? 0 : pd.omega0dtsqr;
    for (int d = 0; d < 3; d++) {
      if (L.sigma[d].empty() || !has_field(S, d)) continue;
      double *p;
      if (dev_alloc(F, &p, F->nlocal)) return -1;
      if (upload_canonical(F, p, L.sigma[d], d)) return -1;
      pd.sigma[d] = p;
    }
    if (L.aniso()) {  // off-diagonal sigma + per-chunk array presence (zone boxes)
      f.aniso = 1;
      for (int c = 0; c < 3; c++)
        for (int d = 0; d < 3; d++) {
          if (L.off[c][d].empty() || !has_field(S, c)) continue;
          double *p;
          if (dev_alloc(F, &p, F->nlocal)) return -1;
          if (upload_canonical(F, p, L.off[c][d], c)) return -1;
          pd.soff[c][d] = p;
        }
      std::vector<uint16_t> zb(27, 0);
      auto ivx = zone_ivs_or_one(S, 0), ivy = zone_ivs_or_one(S, 1), ivz = zone_ivs_or_one(S, 2);
      for (auto &zx : ivx)
        for (auto &zy : ivy)
          for (auto &zz : ivz) {
            const ZoneIv *zv[3] = {&zx, &zy, &zz};
            uint16_t &m = zb[zx.zone * 9 + zy.zone * 3 + zz.zone];
            for (int c = 0; c < 3; c++) {
              bool row = !L.sigma[c].empty() && nontrivial_in_zone(S, L.sigma[c], c, zv, 0.0);
              for (int d = 0; d < 3; d++)
                if (d != c && !L.off[c][d].empty() && nontrivial_in_zone(S, L.off[c][d], c, zv, 0.0)) {
                  m |= 1 << (3 * c + d);
                  row = true;
                }
              if (row) m |= 1 << (4 * c);
            }
          }
      uint16_t *dz;
      if (dev_alloc(F, &dz, 27)) return -1;
      HIPCHK(hipMemcpyAsync(dz, zb.data(), 27 * sizeof(uint16_t), hipMemcpyHostToDevice, F->stream));
      HIPCHK(hipStreamSynchronize(F->stream));
      pd.zbits = dz;
    }
    (void)box_sig;
  }
  // geometry boxes (device rasterisation)
  for (auto &b : S.boxes) {
    double lo[3] = {b.box[0], b.box[2], b.box[4]}, hi[3] = {b.box[1], b.box[3], b.box[5]};
    for (int c = 0; c < 3; c++) {
      if (!has_field(S, c)) continue;
      double *dst = nullptr;
      int invert = 0;
      if (b.kind == 0) {
        dst = const_cast<double *>(f.inveps[c]);
        invert = 1;
      } else if (b.kind == 1)
        dst = const_cast<double *>(f.chi2[c]);
      else if (b.kind == 2)
        dst = const_cast<double *>(f.chi3[c]);  // upstream mode only (null otherwise)
      else if (b.kind == 3 && b.index < nl)
        dst = const_cast<double *>(f.pol[nl - 1 - b.index].sigma[c]);
      if (!dst) continue;
      if (k_box_fill(dst, F->g, T_E, c, lo, hi, b.value, invert, S.a, S.io, F->stream))
        return fail("box fill failed");
    }
  }
  // where each susceptibility can be nonzero (DESIGN.md "Dispersive E update")
  if (nl > 0) {
    int *dbox;
    if (dev_alloc(F, &dbox, 6 * nl, false)) return -1;
    std::vector<int> init(6 * nl);
    for (int k = 0; k < nl; k++)
      for (int e = 0; e < 3; e++) init[6 * k + e] = INT32_MAX, init[6 * k + 3 + e] = -1;
    HIPCHK(hipMemcpyAsync(dbox, init.data(), init.size() * 4, hipMemcpyHostToDevice, F->stream));
    for (int k = 0; k < nl; k++) {
      const double *sg[3] = {f.pol[k].sigma[0], f.pol[k].sigma[1], f.pol[k].sigma[2]};
      if (k_nonzero_box(sg, F->g, dbox + 6 * k, F->stream)) return fail("sigma box failed");
    }
    HIPCHK(hipMemcpyAsync(init.data(), dbox, init.size() * 4, hipMemcpyDeviceToHost, F->stream));
    HIPCHK(hipStreamSynchronize(F->stream));
    for (int k = 0; k < nl; k++)
      for (int e = 0; e < 3; e++) {
        f.pol[k].nz.lo[e] = init[6 * k + e];
        f.pol[k].nz.hi[e] = init[6 * k + 3 + e];
      }
  }
  if (setup_h_materials(F)) return -1;
  // The E update reaches the high metallic wall planes the reference's chunks own
  // (zeroed only afterwards by step_boundaries): with D = 0 there, E is nonzero
  // only through neighbour reads (OFFDIAG, Newton-Raphson), and only a
  // polarization keeps what update_P reads of it.
  bool any_offd = false;
  for (int c = 0; c < 3; c++) any_offd = any_offd || f.offd[c][0] || f.offd[c][1];
  f.wall_e = ((F->upnl && any_offd) || F->nr) && f.npol > 0 ? 1 : 0;
  HIPCHK(hipStreamSynchronize(F->stream));
  return 0;
}

int upload_pml(mnl_fields *F) {
  for (int d = 0; d < 3; d++) {
    if (!F->S.has[d] || !F->pml_any[d]) continue;
    size_t nq = F->h_flag[d].size();
    uint8_t *fl, *zn;
    double *sg, *kp, *si;
    if (dev_alloc(F, &fl, nq) || dev_alloc(F, &zn, nq) || dev_alloc(F, &sg, nq) ||
        dev_alloc(F, &kp, nq) || dev_alloc(F, &si, nq))
      return -1;
    HIPCHK(hipMemcpyAsync(fl, F->h_flag[d].data(), nq, hipMemcpyHostToDevice, F->stream));
    HIPCHK(hipMemcpyAsync(zn, F->h_zone[d].data(), nq, hipMemcpyHostToDevice, F->stream));
    HIPCHK(hipMemcpyAsync(sg, F->h_sig[d].data(), nq * 8, hipMemcpyHostToDevice, F->stream));
    HIPCHK(hipMemcpyAsync(kp, F->h_kap[d].data(), nq * 8, hipMemcpyHostToDevice, F->stream));
    HIPCHK(hipMemcpyAsync(si, F->h_siginv[d].data(), nq * 8, hipMemcpyHostToDevice, F->stream));
    F->f.pml.flag[d] = fl;
    F->f.pml.sig[d] = sg;
    F->f.pml.kap[d] = kp;
    F->f.pml.siginv[d] = si;
    F->f.zone[d] = zn;
  }
  for (int d = 0; d < 3; d++) {  // zone tables are needed by the NR kernel everywhere
    if (!F->S.has[d] || F->f.zone[d]) continue;
    size_t nq = F->h_zone[d].size();
    uint8_t *zn;
    if (dev_alloc(F, &zn, nq)) return -1;
    HIPCHK(hipMemcpyAsync(zn, F->h_zone[d].data(), nq, hipMemcpyHostToDevice, F->stream));
    F->f.zone[d] = zn;
  }
  HIPCHK(hipStreamSynchronize(F->stream));
  return 0;
}

// ------------------------------------------------------------- loop_in_chunks
void dft_boundary_weights(const mnl_structure &S, const double wmin[3], const double wmax[3],
                          const int is[3], const int ie[3], double s0[3], double e0[3],
                          double s1[3], double e1[3]);
std::vector<std::array<int, 6>> reference_chunks(const mnl_structure &S);

// One reference chunk's loop of fields::loop_in_chunks over [wmin, wmax] on
// component c's Yee grid (src/loop_in_chunks.cpp:325-520; no symmetry, no
// Bloch): half-coordinate range [isc, iec] and the boundary weights.
struct CLoop {
  int isc[3], iec[3];
  double s0[3], s1[3], e0[3], e1[3];
  double W(int d, long i) const {  // IVEC_LOOP_WEIGHT1x (src/meep/vec.hpp:372-378)
    const long n = (iec[d] - isc[d]) / 2 + 1;
    if (i > 1 && i < n - 2) return 1.0;
    return i == 0 ? s0[d] : (i == 1 ? s1[d] : i == n - 1 ? e0[d] : (i == n - 2 ? e1[d] : 1.0));
  }
};

std::vector<CLoop> chunk_loops(const mnl_structure &S, int c, const double wmin[3],
                               const double wmax[3]) {
  int is[3] = {0, 0, 0}, ie[3] = {0, 0, 0};
  for (int d = 0; d < 3; d++) {
    if (!S.has[d]) continue;
    const int iyc = 1 - S.shift(c, d);    // iyee_shift(Centered) - iyee_shift(c)
    const double yc = iyc * (0.5 / S.a);  // wherec = where + yee_c
    is[d] = 1 + 2 * int(floor((wmin[d] + yc) * S.a - .5)) - iyc;  // vec2diel_floor - iyee_c
    ie[d] = 1 + 2 * int(ceil((wmax[d] + yc) * S.a - .5)) - iyc;
  }
  double s0[3], s1[3], e0[3], e1[3];
  dft_boundary_weights(S, wmin, wmax, is, ie, s0, e0, s1, e1);
  std::vector<CLoop> out;
  for (auto &ch : reference_chunks(S)) {
    CLoop L;
    bool emp = false;
    for (int d = 0; d < 3; d++) {
      L.s0[d] = L.s1[d] = L.e0[d] = L.e1[d] = 1.0;
      if (!S.has[d]) {
        L.isc[d] = L.iec[d] = 0;
        continue;
      }
      // little_owned_corner(c) = little + 2 - iyee_shift(c), big_owned_corner(c) =
      // big - iyee_shift(c) (src/meep/vec.hpp:1102-1107)
      const int sh = S.shift(c, d);
      const int uoc = S.io[d] + 2 - sh, coc = ch[d] + 2 - sh, cbo = ch[d] + 2 * ch[3 + d] - sh;
      const int iscoS = std::max(uoc, std::min(coc, cbo)), iecoS = std::max(coc, cbo);
      L.isc[d] = std::max(is[d], iscoS);
      L.iec[d] = std::min(ie[d], iecoS);
      if (L.isc[d] > L.iec[d]) emp = true;
    }
    if (emp) continue;
    for (int d = 0; d < 3; d++) {
      if (!S.has[d]) continue;
      if (L.isc[d] == is[d]) {
        L.s0[d] = s0[d];
        L.s1[d] = s1[d];
      } else if (L.isc[d] == is[d] + 2) {
        L.s0[d] = s1[d];
      }
      if (L.iec[d] == ie[d]) {
        L.e0[d] = e0[d];
        L.e1[d] = e1[d];
      } else if (L.iec[d] == ie[d] - 2) {
        L.e0[d] = e1[d];
      }
      if (L.iec[d] == L.isc[d]) {
        double w = std::min(L.s0[d], L.e0[d]);
        L.s0[d] = L.e0[d] = L.s1[d] = L.e1[d] = w;
      } else if (L.iec[d] == L.isc[d] + 2) {
        double w = std::min(L.s0[d], L.e1[d]);
        L.s0[d] = w, L.e1[d] = w;
        w = std::min(L.s1[d], L.e0[d]);
        L.s1[d] = w, L.e0[d] = w;
      } else if (L.iec[d] == L.isc[d] + 4) {
        double w = std::min(L.s1[d], L.e1[d]);
        L.s1[d] = w, L.e1[d] = w;
      }
    }
    out.push_back(L);
  }
  return out;
}

// ------------------------------------------------------------- sources
// fields::add_volume_source(c, src, where, A, amp) (src/sources.cpp:455-494):
// the source volume is clamped to the cell, delta-function directions scale
// the amplitude by a, and src_vol_chunkloop (243-312) gives every owned point
// of each reference chunk the amplitude IVEC_LOOP_WEIGHT * amp * A(loc -
// center).  The points of all chunks form one group (src_vol list order).
int add_volume_source(mnl_fields *F, int c, int st, const double wmin0[3], const double wmax0[3],
                      cplx amp0, mnl_amp_func afunc, void *adata) {
  const mnl_structure &S = F->S;
  double wmin[3], wmax[3];
  for (int d = 0; d < 3; d++) {
    wmin[d] = S.has[d] ? wmin0[d] : 0.0;
    wmax[d] = S.has[d] ? wmax0[d] : 0.0;
    if (wmax[d] < wmin[d]) return fail("source volume: max < min");
    if (!S.has[d]) continue;
    const double w = S.n[d] * (1.0 / S.a);  // user_volume width
    const double wd = wmax[d] - wmin[d];
    if (wd > w + 1.0 / S.a) {
      const char *nm[3] = {"X", "Y", "Z"};
      return fail(std::string("Source width > cell width in ") + nm[d] + " direction!");
    } else if (wd > w) {  // less than a pixel too wide
      const double dw = wd - w;
      wmin[d] = wmin[d] - dw * 0.5;
      wmax[d] = wmin[d] + w;
    }
  }
  cplx amp = amp0;
  for (int d = 0; d < 3; d++)
    if (S.has[d] && wmax[d] - wmin[d] == 0.0) amp *= S.a;  // delta-function units
  double center[3];
  for (int d = 0; d < 3; d++) center[d] = (wmin[d] + wmax[d]) * 0.5;
  int yd[3];
  if (S.dim == 2)
    yd[0] = 2, yd[1] = 0, yd[2] = 1;
  else
    yd[0] = 0, yd[1] = 1, yd[2] = 2;
  SrcGroup grp;
  grp.comp = c;
  grp.st = st;
  for (const CLoop &L : chunk_loops(S, c, wmin, wmax)) {
    long ln[3];
    for (int k = 0; k < 3; k++) ln[k] = S.has[yd[k]] ? (L.iec[yd[k]] - L.isc[yd[k]]) / 2 + 1 : 1;
    for (long i1 = 0; i1 < ln[0]; i1++)
      for (long i2 = 0; i2 < ln[1]; i2++)
        for (long i3 = 0; i3 < ln[2]; i3++) {
          const long ii[3] = {i1, i2, i3};
          int p[3] = {0, 0, 0};
          for (int k = 0; k < 3; k++)
            if (S.has[yd[k]]) p[yd[k]] = L.isc[yd[k]] + 2 * int(ii[k]);
          bool own = true;
          int jg[3] = {0, 0, 0};
          long long gi = 0;
          for (int d = 0; d < 3; d++)
            if (S.has[d]) {
              const int o = p[d] - S.io[d];
              if (!(o > 0 && o <= 2 * S.n[d])) own = false;
              jg[d] = (p[d] - S.io[d] - S.shift(c, d)) / 2;
              gi += jg[d] * S.cstride(d);
            }
          if (!own) continue;
          double w[3];
          for (int k = 0; k < 3; k++) w[k] = L.W(yd[k], ii[k]);
          const double wgt = w[2] * (w[1] * (1.0 * w[0]));
          cplx A = 1.0;
          if (afunc) {
            double rel[3];
            for (int d = 0; d < 3; d++) rel[d] = S.has[d] ? p[d] * (0.5 * (1.0 / S.a)) - center[d] : 0.0;
            double re = 0, im = 0;
            afunc(rel, adata, &re, &im);
            A = cplx(re, im);
          }
          grp.amp.push_back(wgt * (amp * std::conj(cplx(1.0))) * A);
          grp.gidx.push_back(gi);
          for (int d = 0; d < 3; d++) grp.jglob.push_back(jg[d]);
        }
  }
  if (grp.gidx.empty()) return 0;
  for (auto &o : F->groups)  // src_vol::combinable merge (src/fields.cpp:588-597)
    if (o.comp == grp.comp && o.st == grp.st && o.gidx == grp.gidx) {
      for (size_t i = 0; i < o.amp.size(); i++) o.amp[i] += grp.amp[i];
      F->src_dirty = true;
      return 0;
    }
  F->groups.push_back(std::move(grp));
  F->src_dirty = true;
  return 0;
}

// local linear index of a global point of component c, or -1 if not owned by this rank
long long local_index(const mnl_fields *F, int c, const int jg[3], bool include_wall) {
  const DevGrid &g = F->g;
  long long li = 0;
  for (int d = 0; d < 3; d++) {
    if (g.ax[d] < 0) continue;
    int j = jg[d] - g.off[d];
    int sh = F->S.shift(c, d);
    int lo = sh ? g.owned_lo_sh[d] : g.owned_lo_un[d];
    int hi = sh ? g.owned_hi_sh[d] : g.owned_hi_un[d];
    if (include_wall && !sh && jg[d] == g.nglob[d] && j >= 0 && j < g.N[g.ax[d]]) hi = j;
    if (j < lo || j > hi) return -1;
    li += (long long)j * g.st[g.ax[d]];
  }
  return li;
}

// local linear index of a global point anywhere in this rank's arrays (ghost
// planes included), or -1
long long local_index_ghost(const mnl_fields *F, const int jg[3]) {
  const DevGrid &g = F->g;
  long long li = 0;
  for (int d = 0; d < 3; d++) {
    if (g.ax[d] < 0) continue;
    int j = jg[d] - g.off[d];
    if (j < 0 || j >= g.N[g.ax[d]]) return -1;
    li += (long long)j * g.st[g.ax[d]];
  }
  return li;
}

int build_source_lists(mnl_fields *F) {
  // whole-cell facts (the same on every rank): what keeps the step unfused
  F->any_srcB = F->any_isrc = F->any_dsrc_w = false;
  for (const SrcGroup &G : F->groups) {
    const bool mag = ctype(G.comp) == T_H, integ = F->srcs[G.st].is_integrated;
    if (mag && !integ) F->any_srcB = true;
    if (!mag && integ) F->any_isrc = true;
    if (!mag && !integ) {
      const int d = cdir(G.comp);
      if (F->S.has[d] && F->pml_any[d])
        for (size_t j = 0; j < G.gidx.size(); j++)
          if (F->h_flag[d][2 * G.jglob[3 * j + d] + 1]) F->any_dsrc_w = true;
    }
  }
  F->srcB_idx.clear(), F->srcD_idx.clear(), F->isrc_idx.clear();
  F->srcB_comp.clear(), F->srcD_comp.clear(), F->isrc_comp.clear();
  F->srcB_ref.clear(), F->srcD_ref.clear(), F->isrc_ref.clear();
  F->isrc_zone.clear();
  for (size_t gi = 0; gi < F->groups.size(); gi++) {
    const SrcGroup &G = F->groups[gi];
    const SrcTime &st = F->srcs[G.st];
    int c = G.comp;
    bool mag = ctype(c) == T_H;
    for (size_t j = 0; j < G.gidx.size(); j++) {
      const int *jg = &G.jglob[3 * j];
      int tgt = mag ? 3 * T_B + cdir(c) : 3 * T_D + cdir(c);
      long long li = local_index(F, tgt, jg, false);
      if (st.is_integrated && !mag) {
        // integrated dipoles are read (never written): keep the rank's ghost copies
        // too, so a slab seam sees what one GPU sees; the zone box restricts the
        // subtraction to readers in the owning reference chunk.  A dipole on the
        // high metallic wall plane stays: the chunk owns that point and its
        // f_minus_p there (D = 0 minus the dipole) is read by neighbours through
        // the Newton-Raphson / OFFDIAG sums (src/update_eh.cpp:136-146).
        li = local_index(F, tgt, jg, true);
        if (li < 0 && F->nranks > 1) {
          bool wall = false;  // high PEC wall of an unshifted direction: nobody owns it
          for (int d = 0; d < 3; d++)
            if (F->g.ax[d] >= 0 && !F->S.shift(tgt, d) && jg[d] == F->g.nglob[d]) wall = true;
          if (!wall) li = local_index_ghost(F, jg);
        }
        if (li < 0) continue;
        int zb = 0;
        for (int d = 0; d < 3; d++) {
          int z = 1;
          if (F->S.has[d]) z = F->h_zone[d][2 * jg[d] + F->S.shift(tgt, d)];
          zb = zb * 3 + z;
        }
        F->isrc_idx.push_back(li);
        F->isrc_comp.push_back(cdir(c));
        F->isrc_zone.push_back((unsigned char)zb);
        F->isrc_ref.push_back({(int)gi, (int)j});
        continue;
      }
      if (li < 0) continue;
      if (!st.is_integrated) {
        auto &I = mag ? F->srcB_idx : F->srcD_idx;
        auto &C = mag ? F->srcB_comp : F->srcD_comp;
        auto &R = mag ? F->srcB_ref : F->srcD_ref;
        I.push_back(li);
        C.push_back(cdir(c));
        R.push_back({(int)gi, (int)j});
      }
    }
  }
  // integrated dipoles for the E kernels: sorted by local index (stable, so the
  // entries of one point keep list order), with their position in the table
  F->isrc_dev = ISrcDev{};
  if (!F->isrc_idx.empty()) {
    const size_t n = F->isrc_idx.size();
    std::vector<int> ord(n);
    for (size_t k = 0; k < n; k++) ord[k] = (int)k;
    std::stable_sort(ord.begin(), ord.end(),
                     [&](int a, int b) { return F->isrc_idx[a] < F->isrc_idx[b]; });
    std::vector<long long> si(n);
    std::vector<int> sc(n), so(n);
    std::vector<unsigned char> sz(n);
    for (size_t k = 0; k < n; k++)
      si[k] = F->isrc_idx[ord[k]], sc[k] = F->isrc_comp[ord[k]], sz[k] = F->isrc_zone[ord[k]],
      so[k] = ord[k];
    long long *di;
    int *dc, *dor;
    unsigned char *dz;
    if (dev_alloc(F, &di, n, false) || dev_alloc(F, &dc, n, false) || dev_alloc(F, &dor, n, false) ||
        dev_alloc(F, &dz, n, false))
      return -1;
    HIPCHK(hipMemcpyAsync(di, si.data(), n * 8, hipMemcpyHostToDevice, F->stream));
    HIPCHK(hipMemcpyAsync(dc, sc.data(), n * 4, hipMemcpyHostToDevice, F->stream));
    HIPCHK(hipMemcpyAsync(dor, so.data(), n * 4, hipMemcpyHostToDevice, F->stream));
    HIPCHK(hipMemcpyAsync(dz, sz.data(), n, hipMemcpyHostToDevice, F->stream));
    F->isrc_dev.n = (int)n;
    F->isrc_dev.idx = di, F->isrc_dev.comp = dc, F->isrc_dev.orig = dor, F->isrc_dev.zone = dz;
    F->isrc_dev.imin = si.front(), F->isrc_dev.imax = si.back();
  }
  // layers: the k-th occurrence of a (component, point) goes to layer k, so a layer
  // is applied in parallel and the layers in list order (step_source order)
  for (int t = 0; t < 2; t++) {
    auto &I = t ? F->srcD_idx : F->srcB_idx;
    auto &C = t ? F->srcD_comp : F->srcB_comp;
    auto &R = t ? F->srcD_ref : F->srcB_ref;
    std::unordered_map<long long, int> seen;
    std::vector<int> lay(I.size());
    int nl = 0;
    for (size_t k = 0; k < I.size(); k++) {
      lay[k] = seen[I[k] * 3 + C[k]]++;
      nl = std::max(nl, lay[k] + 1);
    }
    std::vector<size_t> ord(I.size());
    for (size_t k = 0; k < ord.size(); k++) ord[k] = k;
    std::stable_sort(ord.begin(), ord.end(), [&](size_t a, size_t b) { return lay[a] < lay[b]; });
    std::vector<long long> I2;
    std::vector<int> C2;
    std::vector<std::pair<int, int>> R2;
    auto &A = F->src_amp[t];
    auto &Gd = F->src_gid[t];
    auto &L = F->src_layer[t];
    A.clear(), Gd.clear(), L.assign(nl + 1, 0);
    for (size_t k : ord) {
      I2.push_back(I[k]);
      C2.push_back(C[k]);
      R2.push_back(R[k]);
      const cplx a = F->groups[R[k].first].amp[R[k].second];
      A.push_back(real(a));
      A.push_back(imag(a));
      Gd.push_back(R[k].first);
      L[lay[k] + 1]++;
    }
    for (int l = 0; l < nl; l++) L[l + 1] += L[l];
    I.swap(I2), C.swap(C2), R.swap(R2);
    if (I.empty()) continue;
    long long **dI = t ? &F->d_srcD_idx : &F->d_srcB_idx;
    int **dC = t ? &F->d_srcD_comp : &F->d_srcB_comp;
    if (dev_alloc(F, dI, I.size(), false) || dev_alloc(F, dC, C.size(), false) ||
        dev_alloc(F, &F->d_src_amp[t], A.size(), false) ||
        dev_alloc(F, &F->d_src_gid[t], Gd.size(), false))
      return -1;
    HIPCHK(hipMemcpyAsync(*dI, I.data(), I.size() * 8, hipMemcpyHostToDevice, F->stream));
    HIPCHK(hipMemcpyAsync(*dC, C.data(), C.size() * 4, hipMemcpyHostToDevice, F->stream));
    HIPCHK(hipMemcpyAsync(F->d_src_amp[t], A.data(), A.size() * 8, hipMemcpyHostToDevice,
                          F->stream));
    HIPCHK(hipMemcpyAsync(F->d_src_gid[t], Gd.data(), Gd.size() * 4, hipMemcpyHostToDevice,
                          F->stream));
  }
  HIPCHK(hipStreamSynchronize(F->stream));
  F->src_dirty = false;
  return 0;
}

// SrcDev of field type t (0 = B, 1 = D) reading the group currents at J
SrcDev src_dev(mnl_fields *F, int t, const double *J) {
  SrcDev s;
  s.n = (int)(t ? F->srcD_idx.size() : F->srcB_idx.size());
  s.idx = t ? F->d_srcD_idx : F->d_srcB_idx;
  s.comp = t ? F->d_srcD_comp : F->d_srcB_comp;
  s.amp = F->d_src_amp[t];
  s.gid = F->d_src_gid[t];
  s.J = J;
  s.dt = F->dt;
  s.nlayer = (int)F->src_layer[t].size() - 1;
  s.layer = F->src_layer[t].data();
  if (s.nlayer < 0) s.nlayer = 0;
  return s;
}

// (the interpolation helpers and the DFT monitors: mnl_dft.cpp)
void interpolate(const mnl_structure &S, int c, const double pc[3], int locs[8][3], double w[8]) {
  const double SMALL = 1e-13;
  double p[3] = {0, 0, 0}, midv[3] = {0, 0, 0}, dv[3] = {0, 0, 0};
  int middle[3] = {0, 0, 0};
  for (int d = 0; d < 3; d++) {
    if (!S.has[d]) continue;
    double ys = S.shift(c, d) * (0.5 * (1.0 / S.a));
    p[d] = (pc[d] - ys) * S.a;
    middle[d] = ((int)floor(p[d])) * 2 + 1 + S.shift(c, d);
    midv[d] = middle[d] * (0.5 * (1.0 / S.a));
    dv[d] = (pc[d] - midv[d]) * (2 * S.a);
  }
  int already = 1;
  for (int i = 0; i < 8; i++) {
    for (int d = 0; d < 3; d++) locs[i][d] = S.has[d] ? my_round(midv[d] * 2 * S.a) : 0;
    w[i] = 1.0;
  }
  for (int d = 0; d < 3; d++) {
    if (!S.has[d]) continue;
    for (int i = 0; i < already; i++) {
      for (int e = 0; e < 3; e++) locs[already + i][e] = locs[i][e];
      w[already + i] = w[i];
      locs[i][d] = middle[d] - 1;
      w[i] *= 0.5 * (1.0 - dv[d]);
      locs[already + i][d] = middle[d] + 1;
      w[already + i] *= 0.5 * (1.0 + dv[d]);
    }
    already *= 2;
  }
  for (int i = already; i < 8; i++) w[i] = 0.0;
  double total = 0.0;
  for (int i = 0; i < already; i++) total += w[i];
  for (int i = 0; i < already; i++) w[i] += (1.0 - total) * (1.0 / already);
  for (int i = 0; i < already; i++) {
    if (w[i] < 0.0 || w[i] < SMALL) w[i] = 0.0;
  }
  int l = already, off = 0;
  while (l) {
    if (fabs(w[off]) < 2e-15) {
      w[off] = w[off + l - 1];
      for (int e = 0; e < 3; e++) locs[off][e] = locs[off + l - 1][e];
      w[off + l - 1] = 0.0;
      for (int e = 0; e < 3; e++) locs[off + l - 1][e] = 0;
    } else
      off += 1;
    l -= 1;
  }
  bool all_same = true;
  for (int i = 0; i < 8 && w[i]; i++)
    if (w[i] != w[0]) all_same = false;
  if (all_same) {
    int nw = 0;
    for (int i = 0; i < 8 && w[i]; i++) nw++;
    for (int i = 0; i < 8 && w[i]; i++) w[i] = 1.0 / nw;
  }
}

// value of component c at absolute half-coords p (0 if not owned by this rank)
int value_at(mnl_fields *F, int c, const int p[3], double *out) {
  const mnl_structure &S = F->S;
  *out = 0.0;
  int jg[3] = {0, 0, 0};
  for (int d = 0; d < 3; d++)
    if (S.has[d]) {
      int o = p[d] - S.io[d];
      if (!(o > 0 && o <= 2 * S.n[d])) return 0;  // not owned by the cell
      jg[d] = (p[d] - S.io[d] - S.shift(c, d)) / 2;
    }
  if (!F->allocated[c]) return 0;
  long long li = local_index(F, c, jg, true);
  if (li < 0) return 0;
  int t = ctype(c), d = cdir(c);
  const double *src = nullptr;
  switch (t) {
    case T_E: src = F->f.E[d]; break;
    case T_D: src = F->f.D[d]; break;
    case T_B: src = F->f.B[d]; break;
    case T_H: {
      src = F->f.B[d];
      if (F->hall) {  // H stored everywhere once the first H update has run
        if (F->h_first_done) src = F->f.H[d];
      } else if (F->f.H[d] && S.has[d]) {
        int q = 2 * jg[d];
        if (F->h_flag[d][q]) src = F->f.H[d];
      }
      break;
    }
  }
  if (!src) return 0;
  HIPCHK(hipStreamSynchronize(F->stream));
  if (in_fused_box(F, c, jg)) {  // E = chi1inv * D inside the fused region
    double dv = 0, uv = 1;
    HIPCHK(hipMemcpy(&dv, F->f.D[d] + li, sizeof(double), hipMemcpyDeviceToHost));
    if (F->f.inveps[d]) {
      HIPCHK(hipMemcpy(&uv, F->f.inveps[d] + li, sizeof(double), hipMemcpyDeviceToHost));
      *out = dv * uv;
    } else {
      *out = dv;
    }
    return 0;
  }
  HIPCHK(hipMemcpy(out, src + li, sizeof(double), hipMemcpyDeviceToHost));
  return 0;
}

int get_field(mnl_fields *F, int c, const double pos[3], double *out, bool reduce) {
  int locs[8][3];
  double w[8];
  double pp[3] = {pos[0], pos[1], pos[2]};
  if (F->S.dim == 1) pp[0] = pp[1] = 0;
  if (F->S.dim == 2) pp[2] = 0;
  interpolate(F->S, c, pp, locs, w);
  cplx res = 0.0;
  bool ok = true;
  for (int i = 0; i < 8 && w[i] && ok; i++) {
    double v;
    if (value_at(F, c, locs[i], &v)) ok = false;
    else res += w[i] * cplx(v);
  }
  double r = real(res);
  if (reduce && F->nranks > 1) {
    const std::string why = g_err;
    if (F->comm->agree_ok(ok, F->stream)) return fail(ok ? "get_field: a rank failed" : why);
    if (timed_allreduce(F, &r, 1)) return fail("allreduce failed");
  }
  if (!ok) return -1;
  *out = r;
  return 0;
}

// ------------------------------------------------------------- halo exchange
// step_boundaries replacement for the slab decomposition (src/step.cpp:226-288):
// kind 0 (before curl B): E comps unshifted along the slab axis need the low
//   ghost plane (local 0) <- rank-1's top owned plane (local nloc).
// kind 1 (before curl D): B (and separate H) comps shifted along the slab axis
//   need the high ghost plane (local nloc) <- rank+1's first plane (local 0).
// kind 2 (before NR E update): D comps (and Lorentz P), both directions.
// kind 3 (before a DFT update): H comps unshifted along the slab axis need the
//   low ghost plane, which the centred-grid average reads (src/dft.cpp:281-287).
int exchange(mnl_fields *F, int kind, hipStream_t st) {
  if (!st) st = F->stream;
  const DevGrid &g = F->g;
  const int sd = F->slab_dir, ax = g.ax[sd];
  const size_t plane = (size_t)g.st[ax];
  const int nloc = g.N[ax] - 1;
  const int up = F->rank + 1 < F->nranks ? F->rank + 1 : -1;
  const int dn = F->rank > 0 ? F->rank - 1 : -1;
  struct Item {
    double *p;
    bool low_ghost;  // true: send top plane up, receive plane 0 from below
  };
  std::vector<Item> items;
  for (int c = 0; c < 3; c++) {
    if (kind == 0) {
      if (c != sd && F->f.E[c] && F->allocated[c]) items.push_back({F->f.E[c], true});
    } else if (kind == 1) {
      if (c != sd && F->f.Bn[c] && F->allocated[3 * T_H + c]) {
        items.push_back({F->f.Bn[c], false});
        if (F->f.H[c]) items.push_back({F->f.Hn[c], false});
      }
    } else if (kind == 4) {  // W of E (E, and f_w where allocated): the one ghost plane
      if (F->f.E[c] && F->allocated[c]) {
        items.push_back({F->f.E[c], c != sd});
        if (F->f.WE[c]) items.push_back({F->f.WE[c], c != sd});
      }
    } else if (kind == 3) {  // DFT: H comps unshifted along the slab axis, low ghost
      if (c == sd && F->allocated[3 * T_H + c]) {
        items.push_back({F->f.B[c], true});
        if (F->f.H[c]) items.push_back({F->f.H[c], true});
      }
    } else {
      if (F->f.Dn[c] && F->allocated[3 * T_D + c]) items.push_back({F->f.Dn[c], c != sd});
      for (int k = 0; k < F->f.npol; k++)
        if (F->f.pol[k].P[c]) items.push_back({F->f.pol[k].P[c], c != sd});
    }
  }
  if (items.empty()) return 0;
  Comm &cm = *F->comm;
  if (cm.group_start()) return -1;
  for (auto &it : items) {
    if (it.low_ghost) {
      if (up >= 0 && cm.send(it.p + (size_t)nloc * plane, plane, up, st)) return -1;
      if (dn >= 0 && cm.recv(it.p, plane, dn, st)) return -1;
    } else {
      if (dn >= 0 && cm.send(it.p, plane, dn, st)) return -1;
      if (up >= 0 && cm.recv(it.p + (size_t)nloc * plane, plane, up, st)) return -1;
    }
  }
  return cm.group_end(st);
}

// ------------------------------------------------------------- stepping
// ------------------------------------------------------------- fused mode
// G = [0, N-2] per axis: every owned point except the top plane of a rank
// with an upper neighbour (its D needs the neighbour's new B first); that
// plane is the shell, stepped by the shell kernels around the halo exchange.
// L = interior box (no PML chunk along any direction) within [1, N-2]: tiles
// whose whole footprint lies in L run the lean kernel.
static void split_range(std::vector<int> &b, int lo, int hi_excl, int step, int align) {
  // append starts covering [lo, hi_excl) in pieces of at most `step`, starts aligned
  int x = lo;
  while (x < hi_excl) {
    b.push_back(x);
    int nx = std::min(hi_excl, ((x + step) / align) * align);
    if (nx <= x) nx = std::min(hi_excl, x + step);
    x = nx;
  }
}

// general tiles read the lean kernel's B_new on their halo (default); MNL_LEAN_HALO=0
// recomputes it
static int lean_halo_reads(const mnl_fields *F) { return F->lean_halo ? 1 : 0; }

// Tile mode.  Tiles of the lean body's shape over all of G:
// columns in pieces of <= 64 from G.lo (128-byte aligned), rows in balanced pieces of
// <= 14, z chunks; every chunk whose footprint (planes zs-1 .. ze) misses the
// polarization boxes' z range is stepped by the tile kernel, one item per (tile, chunk),
// with the body its footprint needs (lean inside L, else the PML body of the directions
// whose tables are not the identity there).  The remaining (polarization) chunks keep the
// general kernel's items (wide tiles).  Multi-rank: chunk 0 = planes 0..1 (the B the
// lower neighbour needs), launched first.
// directions whose PML tables are not the identity somewhere in [lo, hi] (per axis)
int pml_dirs_in(const mnl_fields *F, const int lo[3], const int hi[3]) {
  const DevGrid &g = F->g;
  int m = 0;
  for (int d = 0; d < 3; d++) {
    if (F->h_flag[d].empty()) continue;
    for (int j = std::max(lo[d], 0); j <= std::min(hi[d], g.N[d] - 1) && !(m >> d & 1); j++)
      for (int sft = 0; sft < 2; sft++) {
        const size_t q = 2 * (size_t)(j + g.off[d]) + sft;
        if (q >= F->h_flag[d].size()) continue;
        const double kap = F->h_kap[d][q], sig = F->h_sig[d][q];
        if (F->h_flag[d][q] || kap - sig != 1.0 || kap + sig != 1.0 || F->h_siginv[d][q] != 1.0)
          m |= 1 << d;
      }
  }
  return m;
}

// Body code (bits 24-26) and OWNC flag (bit 29) of a tile item with own columns x0 .. x1,
// halo row y0 (own rows y0+1 .. y1) and planes [zs, ze): the lean body when its footprint
// lies in L, else the PML body of the directions whose tables are not the identity over the
// footprint; OWNC when a single-axis body's footprint is owned in y and z for every component.
int tile_item_code(const mnl_fields *F, const FusedArgs &a, const Box &L, int x0, int x1, int y0,
                   int y1, int zs, int ze, bool *lean) {
  const DevGrid &g = F->g;
  *lean = x0 - 1 >= L.lo[0] && x1 + 1 <= L.hi[0] && y0 >= L.lo[1] && y1 + 1 <= L.hi[1] &&
          zs - 1 >= L.lo[2] && ze <= L.hi[2];
  int body = 0;
  if (!*lean) {
    const int lo[3] = {x0 - 1, y0, zs - 1}, hi[3] = {x0 + FX_HOST, y0 + 15, ze};
    const int m = pml_dirs_in(F, lo, hi);
    body = m == 1 ? 1 : m == 2 ? 2 : m == 4 ? 3 : m == 0 ? 4 : m == 3 ? 6 : m == 5 ? 7 : 5;
  }
  int ownc = 0;
  if (body >= 1 && body <= 3 && F->ownc) {
    const int ylo = std::max(a.osh_lo[1], a.oun_lo[1]), yhi = std::min(a.osh_hi[1], a.oun_hi[1]);
    const int zlo = std::max(a.osh_lo[2], a.oun_lo[2]), zhi = std::min(a.osh_hi[2], a.oun_hi[2]);
    ownc = (y0 >= ylo && y0 + 15 <= yhi && zs - 1 >= zlo && ze <= zhi && y0 + 15 <= g.N[1] - 1 &&
            ze <= g.N[2] - 1) ? 1 : 0;
  }
  return (body << 24) | (ownc << 29);
}

// Item code of a narrow x-face strip (strip_body: body 1 | OWNC | bit 30) with own columns
// x0 .. x1 (at most 16, x0 128-byte aligned), halo row y0, own rows y0+1 .. y1 (at most 63)
// and planes [zs, ze), or -1 when its footprint (columns x0-1 .. x1+1, rows y0 .. y1+1,
// planes zs-1 .. ze) meets PML along y or z or a point not owned in y or z.
int strip_item_code(const mnl_fields *F, const FusedArgs &a, int x0, int x1, int y0, int y1, int zs,
                    int ze) {
  const DevGrid &g = F->g;
  if (x1 - x0 + 1 > SW_HOST || (x0 & 15) || y1 - y0 > SOWN_HOST || y1 < y0 + 1 || ze <= zs)
    return -1;
  const int lo[3] = {x0 - 1, y0, zs - 1}, hi[3] = {x1 + 1, y1 + 1, ze};
  if (pml_dirs_in(F, lo, hi) != 1) return -1;
  const int ylo = std::max(a.osh_lo[1], a.oun_lo[1]), yhi = std::min(a.osh_hi[1], a.oun_hi[1]);
  const int zlo = std::max(a.osh_lo[2], a.oun_lo[2]), zhi = std::min(a.osh_hi[2], a.oun_hi[2]);
  if (!(y0 >= ylo && y1 + 1 <= yhi && zs - 1 >= zlo && ze <= zhi && y1 + 1 <= g.N[1] - 1 &&
        ze <= g.N[2] - 1))
    return -1;
  return (1 << 24) | (1 << 29) | (1 << 30);
}

bool make_tile_boxes(mnl_fields *F, const Box &G, const Box &L) {
  const DevGrid &g = F->g;
  FusedArgs &a = F->fgeo;
  std::vector<int> xb, yb, zb, gyb;
  split_range(xb, G.lo[0], G.hi[0] + 1, FX_HOST, 16);
  {
    const int ny = G.hi[1] - G.lo[1] + 1, nt = (ny + 13) / 14;
    for (int t = 0; t < nt; t++) yb.push_back(G.lo[1] + (int)((long long)ny * t / nt));
  }
  int pzl = INT32_MAX, pzh = -1;
  for (int k = 0; k < F->f.npol; k++)
    if (F->f.pol[k].nz.lo[2] <= F->f.pol[k].nz.hi[2]) {
      pzl = std::min(pzl, F->f.pol[k].nz.lo[2]);
      pzh = std::max(pzh, F->f.pol[k].nz.hi[2]);
    }
  // z segments: [lo, hi) with a flag "polarization chunk"
  // (cut at plane 2 on multi-rank runs so that chunk 0 = planes 0..1, and at the ends of
  // the polarization chunks [pzl-1, pzh+2), the planes whose tile footprint would meet
  // the polarization boxes)
  std::vector<std::pair<std::pair<int, int>, bool>> seg;
  {
    const int z0 = G.lo[2], zend = G.hi[2] + 1;
    const int p0 = pzh >= 0 ? std::max(z0, pzl - 1) : zend, p1 = pzh >= 0 ? std::min(zend, pzh + 2) : zend;
    std::vector<int> cut = {z0, zend};
    if (F->nranks > 1 && zend - z0 > 2) cut.push_back(z0 + 2);
    // the lean box's z range: chunks from L.lo+1 to L.hi can run the lean body (their
    // halo planes lie in L), the ones outside hold the z-PML planes (short PML items)
    if (F->tile_zcut && L.lo[2] <= L.hi[2]) {
      if (L.lo[2] + 1 > z0 && L.lo[2] + 1 < zend) cut.push_back(L.lo[2] + 1);
      if (L.hi[2] > z0 && L.hi[2] < zend) cut.push_back(L.hi[2]);
    }
    if (p0 < p1) cut.push_back(p0), cut.push_back(p1);
    std::sort(cut.begin(), cut.end());
    cut.erase(std::unique(cut.begin(), cut.end()), cut.end());
    for (size_t i = 0; i + 1 < cut.size(); i++)
      seg.push_back({{cut[i], cut[i + 1]}, cut[i] >= p0 && cut[i + 1] <= p1 && p0 < p1});
  }
  // chunk length: MNL_FUSED_ZCHUNK, else the candidate whose item count fills whole
  // rounds of one workgroup per CU best (with the halo-plane overhead 1 / planes)
  const long long ntile = (long long)xb.size() * yb.size();
  int zc = F->fused_zchunk > 0 ? std::min(F->fused_zchunk, FUSED_MAXCH) : 24;
  if (F->fused_zchunk <= 0) {
    const long long cus = std::max(1, k_cu_count());
    double best = -1;
    for (int cand : {12, 14, 16, 18, 20, 22, 24, 28, 32}) {
      long long nch = 0, planes = 0;
      for (auto &sg : seg) {
        if (sg.second) continue;
        nch += (sg.first.second - sg.first.first + cand - 1) / cand;
        planes += sg.first.second - sg.first.first;
      }
      if (nch == 0) break;
      const long long items = ntile * nch;
      const double fill = double(items) / double(((items + cus - 1) / cus) * cus);
      const double per = double(planes) / double(nch);
      const double score = fill * per / (per + 1.0);
      if (score >= best - 1e-12) best = score, zc = cand;
    }
  }
  // polarization chunks (general kernel, wide tiles): short enough that their items
  // number at least two per CU
  int pzc = FUSED_MAXCH;
  {
    const long long per_chunk = (long long)xb.size() *
                                ((G.hi[1] - G.lo[1] + FUSED_GW_ROWS) / FUSED_GW_ROWS);
    long long pplanes = 0;
    for (auto &sg : seg)
      if (sg.second) pplanes += sg.first.second - sg.first.first;
    if (pplanes > 0) {
      const long long want = 2LL * std::max(1, k_cu_count());
      const long long nch = std::max(1LL, (want + per_chunk - 1) / per_chunk);
      pzc = (int)std::max(4LL, std::min<long long>(FUSED_MAXCH, (pplanes + nch - 1) / nch));
    }
  }
  std::vector<char> polch;
  auto split_bal = [&](int lo, int hi, int step, bool pol) {  // balanced pieces of <= step
    const int n = hi - lo, nt = (n + step - 1) / step;
    for (int t = 0; t < nt; t++) {
      zb.push_back(lo + (int)((long long)n * t / nt));
      polch.push_back(pol);
    }
  };
  for (auto &sg : seg) split_bal(sg.first.first, sg.first.second, sg.second ? pzc : zc, sg.second);
  split_range(gyb, G.lo[1], G.hi[1] + 1, FUSED_GW_ROWS, 1);
  if ((int)xb.size() > FUSED_MAXX || (int)yb.size() > FUSED_MAXY ||
      (int)gyb.size() > FUSED_MAXGY || (int)zb.size() > FUSED_MAXZ)
    return false;
  a.nx = (int)xb.size();
  a.ny = (int)yb.size();
  a.ngy = (int)gyb.size();
  a.nny = 0;
  a.nch = (int)zb.size();
  for (size_t i = 0; i < xb.size(); i++) a.xb[i] = xb[i];
  a.xb[xb.size()] = G.hi[0] + 1;
  for (size_t i = 0; i < yb.size(); i++) a.yb[i] = yb[i];
  a.yb[yb.size()] = G.hi[1] + 1;
  for (size_t i = 0; i < gyb.size(); i++) a.gyb[i] = gyb[i];
  a.gyb[gyb.size()] = G.hi[1] + 1;
  a.nyb[0] = G.lo[1], a.nyb[1] = G.hi[1] + 1;
  for (size_t i = 0; i < zb.size(); i++) a.zb[i] = zb[i];
  a.zb[zb.size()] = G.hi[2] + 1;
  a.lx0 = 0, a.lx1 = -1, a.ly0 = 0, a.ly1 = -1, a.nlzr = 0;  // no lean-only launch
  for (int k = 0; k < 3; k++) {
    a.N[k] = g.N[k];
    a.off[k] = g.off[k];
    a.osh_lo[k] = g.owned_lo_sh[k];
    a.osh_hi[k] = std::min(g.owned_hi_sh[k], G.hi[k]);
    a.oun_lo[k] = g.owned_lo_un[k];
    a.oun_hi[k] = std::min(g.owned_hi_un[k], G.hi[k]);
  }
  auto pml_dirs = [&](const int lo[3], const int hi[3]) { return pml_dirs_in(F, lo, hi); };
  // ---- tile items
  F->titems.clear();
  F->gitems.clear();
  F->tile_cells = F->lean_cells = F->gen_cells = 0;
  F->tile_z.assign(std::max(g.N[2], 1), 0);
  std::vector<int> early, heavy, lean, gen_e, gen_r;
  for (int ch = 0; ch < a.nch; ch++) {
    const int zs = a.zb[ch], ze = a.zb[ch + 1];
    if (polch[ch]) {
      for (int ty = 0; ty < a.ngy; ty++)
        for (int tx = 0; tx < a.nx; tx++) {
          const int y0 = a.gyb[ty] - 1;
          const int lo[3] = {a.xb[tx] - 1, y0, zs - 1};
          const int hi[3] = {a.xb[tx] + FX_HOST, y0 + FUSED_GW_ROWS + 1, ze + 1};
          const int m = pml_dirs(lo, hi);
          const int v = tx | (ty << 8) | (ch << 16) |
                        (((m & ~2) == 0 ? 2 : (m & ~4) == 0 ? 4 : 7) << 24);
          F->gen_cells += (long long)(a.xb[tx + 1] - a.xb[tx]) * (a.gyb[ty + 1] - a.gyb[ty]) *
                          (ze - zs);
          (ch == 0 ? gen_e : gen_r).push_back(v);
        }
      continue;
    }
    for (int z = zs; z < ze; z++) F->tile_z[z] = 1;
    for (int ty = 0; ty < a.ny; ty++)
      for (int tx = 0; tx < a.nx; tx++) {
        const int x0 = a.xb[tx], x1 = a.xb[tx + 1] - 1, y0 = a.yb[ty] - 1, y1 = a.yb[ty + 1] - 1;
        const long long cells = (long long)(x1 - x0 + 1) * (y1 - y0) * (ze - zs);
        F->tile_cells += cells;
        bool in_l;
        const int code = tile_item_code(F, a, L, x0, x1, y0, y1, zs, ze, &in_l);
        if (in_l) F->lean_cells += cells;
        const int body = (code >> 24) & 7;
        const int v = tx | (ty << 8) | (ch << 16) | code;
        if (F->tile_body_mask >= 0 && !((F->tile_body_mask >> body) & 1)) continue;  // timing only
        if (F->nranks > 1 && ch == 0)
          early.push_back(v);
        else
          (body ? heavy : lean).push_back(v);
      }
  }
  auto planes = [&](int v) { const int ch = (v >> 16) & 255; return a.zb[ch + 1] - a.zb[ch]; };
  auto longest_first = [&](std::vector<int> &v) {
    std::stable_sort(v.begin(), v.end(), [&](int x, int y) { return planes(x) > planes(y); });
  };
  longest_first(heavy);
  longest_first(lean);
  if (F->tile_stats) {  // per-body item / cell counts (diagnostics)
    long long ni[8] = {0}, nc[8] = {0};
    for (auto *v : {&early, &heavy, &lean})
      for (int it : *v) {
        const int b = (it >> 24) & 7, tx = it & 255, ty = (it >> 8) & 255, ch = (it >> 16) & 255;
        ni[b]++;
        nc[b] += (long long)(a.xb[tx + 1] - a.xb[tx]) * (a.yb[ty + 1] - a.yb[ty]) *
                 (a.zb[ch + 1] - a.zb[ch]);
      }
    fprintf(stderr, "tile: nx %d ny %d nch %d zc %d pzc %d gen %zu+%zu\n", a.nx, a.ny, a.nch, zc,
            pzc, gen_e.size(), gen_r.size());
    for (int b = 0; b < 8; b++) fprintf(stderr, "tile body %d: %lld items %lld cells\n", b, ni[b], nc[b]);
  }
  F->titems = early;
  F->titems.insert(F->titems.end(), heavy.begin(), heavy.end());
  F->titems.insert(F->titems.end(), lean.begin(), lean.end());
  a.ntit = (int)F->titems.size();
  a.ntit_e = (int)early.size();
  longest_first(gen_r);
  F->gitems = gen_e;
  F->gitems.insert(F->gitems.end(), gen_r.begin(), gen_r.end());
  a.ngen = (int)F->gitems.size();
  a.ngen_e = (int)gen_e.size();
  a.ngen_n = a.ngen_ne = 0;
  // ---- shell: the top plane of a rank with an upper neighbour
  BoxList &bl = F->fused_shell;
  memset(&bl, 0, sizeof(bl));
  if (F->nranks > 1 && F->rank + 1 < F->nranks) {
    Box b;
    for (int k = 0; k < 3; k++) b.lo[k] = 0, b.hi[k] = g.N[k] - 1;
    b.lo[2] = b.hi[2] = g.N[2] - 1;
    bl.b[0] = b;
    bl.start[0] = 0;
    bl.start[1] = (long long)g.N[0] * g.N[1];
    bl.n = 1;
  }
  return true;
}

bool make_fused_boxes(mnl_fields *F) {
  const DevGrid &g = F->g;
  Box G, L;
  for (int k = 0; k < 3; k++) {
    G.lo[k] = 0;
    G.hi[k] = g.N[k] - 2;
    if (G.hi[k] < G.lo[k]) return false;
    L.lo[k] = std::max(F->interior.lo[k], 1);
    L.hi[k] = std::min(F->interior.hi[k], g.N[k] - 2);
  }
  if (F->interior.hi[0] < F->interior.lo[0])
    for (int k = 0; k < 3; k++) L.lo[k] = 1, L.hi[k] = 0;
  F->fusedG = G;
  F->fusedL = L;
  FusedArgs &a = F->fgeo;
  memset(&a, 0, sizeof(a));
  a.G = G;
  a.L = L;
  if (F->tile_mode) return make_tile_boxes(F, G, L);
  // z-chunk: MNL_FUSED_ZCHUNK, else chosen below (after the lean geometry is known) so
  // that the lean items fill whole rounds of one workgroup per CU; 512^3 gets 24 planes
  // (measured 3.13 ms/step vs 3.17 (16) and 3.27 (32), profiles/README.md)
  int zc = std::min(F->fused_zchunk > 0 ? F->fused_zchunk : 24, FUSED_MAXCH);
  // ---- x tiles (<= 64 columns, starts on 16-double = 128-byte boundaries).  Lean
  // tiles store columns [lx_first, x_end]: footprint x0-1 .. x1+1 inside L (the
  // lanes past x1 load but only feed values that are never stored).
  std::vector<int> xb;
  const int lx_first = (L.lo[0] + 1 + 15) / 16 * 16;
  const int x_end = (L.hi[0] / 16) * 16 - 1;
  const int ly_first = L.lo[1] + 1, y_end = L.hi[1] - 1;
  // z segments: lean chunks need planes zs-1 .. ze inside L and away from the
  // polarization box (where E is stored and P updated: general kernels only)
  const int lz_first = L.lo[2] + 1;
  std::vector<std::pair<int, int>> lean_seg;  // [zs, ze) ranges of lean planes
  {
    int pzl = INT32_MAX, pzh = -1;
    for (int k = 0; k < F->f.npol; k++)
      if (F->f.pol[k].nz.lo[2] <= F->f.pol[k].nz.hi[2]) {
        pzl = std::min(pzl, F->f.pol[k].nz.lo[2]);
        pzh = std::max(pzh, F->f.pol[k].nz.hi[2]);
      }
    auto add = [&](int a0, int a1) {
      if (a1 > a0) lean_seg.push_back({a0, a1});
    };
    if (pzh < 0) {
      add(lz_first, L.hi[2]);
    } else {
      add(lz_first, std::min(L.hi[2], pzl - 1));
      add(std::max(lz_first, pzh + 2), L.hi[2]);
    }
  }
  const bool anylean = x_end >= lx_first && y_end >= ly_first && !lean_seg.empty();
  if (anylean && F->fused_zchunk <= 0) {
    // score = (items / whole rounds of items) x (planes / (planes + the halo plane))
    std::vector<int> tx;
    split_range(tx, lx_first, x_end + 1, FX_HOST, 16);
    const long long ntile = (long long)tx.size() * ((y_end - ly_first + 14) / 14);
    const long long cus = std::max(1, k_cu_count());
    double best = -1;
    for (int cand : {12, 14, 16, 18, 20, 22, 24, 28, 32}) {
      long long nch = 0, planes = 0;
      for (auto &sg : lean_seg) {
        nch += (sg.second - sg.first + cand - 1) / cand;
        planes += sg.second - sg.first;
      }
      const long long items = ntile * nch;
      const double fill = double(items) / double(((items + cus - 1) / cus) * cus);
      const double per = double(planes) / double(nch);
      const double score = fill * per / (per + 1.0);
      if (score >= best - 1e-12) best = score, zc = cand;  // ties: the longer chunk
    }
  }
  std::vector<int> yb, gyb, zb;
  const int gstep = FUSED_GW_ROWS;  // general wide-tile rows
  int gly0 = -1, gly1 = -2;  // general row tiles inside the lean row range
  if (!anylean) {
    split_range(xb, G.lo[0], G.hi[0] + 1, FX_HOST, 16);
    a.lx0 = 0, a.lx1 = -1;
    yb.push_back(0);
    a.ly0 = 0, a.ly1 = -1;
    split_range(gyb, G.lo[1], G.hi[1] + 1, gstep, 1);
    split_range(zb, G.lo[2], G.hi[2] + 1, zc, 1);
    a.nlzr = 0;
  } else {
    split_range(xb, G.lo[0], lx_first, FX_HOST, 16);
    a.lx0 = (int)xb.size();
    split_range(xb, lx_first, x_end + 1, FX_HOST, 16);
    a.lx1 = (int)xb.size() - 1;
    split_range(xb, x_end + 1, G.hi[0] + 1, FX_HOST, 16);
    // lean row tiles: 14 own rows (the last may be shorter), rows y0-1 .. y1+1 inside L
    split_range(yb, ly_first, y_end + 1, 14, 1);
    a.ly0 = 0, a.ly1 = (int)yb.size() - 1;
    yb.push_back(y_end + 1);
    split_range(gyb, G.lo[1], ly_first, gstep, 1);
    gly0 = (int)gyb.size();
    split_range(gyb, ly_first, y_end + 1, gstep, 1);
    gly1 = (int)gyb.size() - 1;
    split_range(gyb, y_end + 1, G.hi[1] + 1, gstep, 1);
    // z chunks: general between the lean segments
    a.nlzr = 0;
    int z = G.lo[2];
    for (auto &sg : lean_seg) {
      split_range(zb, z, sg.first, zc, 1);
      a.lzr[a.nlzr][0] = (int)zb.size();
      split_range(zb, sg.first, sg.second, zc, 1);
      a.lzr[a.nlzr][1] = (int)zb.size() - 1;
      a.nlzr++;
      z = sg.second;
    }
    split_range(zb, z, G.hi[2] + 1, zc, 1);
  }
  // narrow (16-column) general tiles take rows in tiles of FUSED_GN_ROWS
  std::vector<int> nyb;
  split_range(nyb, G.lo[1], G.hi[1] + 1, FUSED_GN_ROWS, 1);
  if ((int)xb.size() > FUSED_MAXX || (int)yb.size() > FUSED_MAXY + 1 ||
      (int)gyb.size() > FUSED_MAXGY || (int)nyb.size() > FUSED_MAXNY ||
      (int)zb.size() > FUSED_MAXZ)
    return false;
  a.nx = (int)xb.size();
  a.ny = (int)yb.size() - 1;
  a.ngy = (int)gyb.size();
  a.nny = (int)nyb.size();
  a.nch = (int)zb.size();
  for (size_t i = 0; i < xb.size(); i++) a.xb[i] = xb[i];
  a.xb[xb.size()] = G.hi[0] + 1;
  for (size_t i = 0; i < yb.size(); i++) a.yb[i] = yb[i];
  for (size_t i = 0; i < gyb.size(); i++) a.gyb[i] = gyb[i];
  a.gyb[gyb.size()] = G.hi[1] + 1;
  for (size_t i = 0; i < nyb.size(); i++) a.nyb[i] = nyb[i];
  a.nyb[nyb.size()] = G.hi[1] + 1;
  for (size_t i = 0; i < zb.size(); i++) a.zb[i] = zb[i];
  a.zb[zb.size()] = G.hi[2] + 1;
  // ---- general items (chunk-major, then rows, then columns) and cell counts:
  // wide tiles first, then the 16-column tiles
  F->gitems.clear();
  F->lean_cells = F->gen_cells = 0;
  std::vector<int> narrow;
  auto lean_ch = [&](int ch) {
    for (int r = 0; r < a.nlzr; r++)
      if (ch >= a.lzr[r][0] && ch <= a.lzr[r][1]) return true;
    return false;
  };
  auto narrow_tx = [&](int tx) {
    return a.xb[tx + 1] - a.xb[tx] <= 16 && (tx < a.lx0 || tx > a.lx1);
  };
  for (int ch = 0; ch < a.nch; ch++) {
    const long long nz = a.zb[ch + 1] - a.zb[ch];
    for (int ty = 0; ty < a.ngy; ty++)
      for (int tx = 0; tx < a.nx; tx++) {
        const int wx = a.xb[tx + 1] - a.xb[tx];
        if (narrow_tx(tx)) continue;
        const long long cells = (long long)wx * (a.gyb[ty + 1] - a.gyb[ty]) * nz;
        const bool lean = tx >= a.lx0 && tx <= a.lx1 && lean_ch(ch) && ty >= gly0 &&
                          ty <= gly1;
        if (lean) {
          F->lean_cells += cells;
          continue;
        }
        F->gen_cells += cells;
        F->gitems.push_back(tx | (ty << 8) | (ch << 16));
      }
    for (int ty = 0; ty < a.nny; ty++)
      for (int tx = 0; tx < a.nx; tx++) {
        const int wx = a.xb[tx + 1] - a.xb[tx];
        if (!narrow_tx(tx)) continue;
        F->gen_cells += (long long)wx * (a.nyb[ty + 1] - a.nyb[ty]) * nz;
        narrow.push_back(tx | (ty << 8) | (ch << 16));
      }
  }
  // bits 24-26 of an item: the directions along which its footprint (the
  // positions whose PML tables the kernel reads) meets a PML chunk or any
  // non-identity coefficient; the kernel picks a body with the others fixed
  auto pml_dirs = [&](int v, bool nar) -> int {
    const int tx = v & 255, ty = (v >> 8) & 255, ch = (v >> 16) & 255;
    const int TXn = nar ? 16 : 64, R = nar ? (FUSED_GN_ROWS + 1) : (FUSED_GW_ROWS + 1);
    const int y0 = (nar ? a.nyb[ty] : a.gyb[ty]) - 1;
    const int lo[3] = {a.xb[tx] - 1, y0, a.zb[ch] - 1};
    const int hi[3] = {a.xb[tx] + TXn, y0 + R, a.zb[ch + 1] + 1};
    int m = 0;
    for (int d = 0; d < 3; d++) {
      if (F->h_flag[d].empty()) continue;
      for (int j = std::max(lo[d], 0); j <= std::min(hi[d], g.N[d] - 1) && !(m >> d & 1); j++)
        for (int sft = 0; sft < 2; sft++) {
          const size_t q = 2 * (size_t)(j + g.off[d]) + sft;
          if (q >= F->h_flag[d].size()) continue;
          const double kap = F->h_kap[d][q], sig = F->h_sig[d][q];
          if (F->h_flag[d][q] || kap - sig != 1.0 || kap + sig != 1.0 || F->h_siginv[d][q] != 1.0)
            m |= 1 << d;
        }
    }
    return m;
  };
  for (int &v : F->gitems) {
    const int m = pml_dirs(v, false);
    v |= ((m & ~2) == 0 ? 2 : (m & ~4) == 0 ? 4 : 7) << 24;
  }
  for (int &v : narrow) v |= (((pml_dirs(v, true) & ~1) == 0 ? 1 : 7) << 24) | (int)0x80000000u;
  // bits 27 / 28: the item's x-1 halo column (own rows) / y-1 halo row (own columns) lies
  // in the box the lean kernel stores (lean chunk, lean columns and rows).  When the general
  // launch follows the lean one (FusedArgs::lean_after) those lanes read B_new (== H_new:
  // no PML there) instead of recomputing it from the old fields: identical values, fewer
  // halo lines (profiles/README.md, round 2)
  if (anylean) {
    const int lsx0 = a.xb[a.lx0], lsx1 = a.xb[a.lx1 + 1] - 1;
    const int lsy0 = a.yb[0], lsy1 = a.yb[a.ny] - 1;
    auto mark = [&](int &v, bool nar) {
      const int tx = v & 255, ty = (v >> 8) & 255, ch = (v >> 16) & 255;
      if (!lean_ch(ch)) return;
      const int *ybv = nar ? a.nyb : a.gyb;
      const int x0 = a.xb[tx], x1 = a.xb[tx + 1] - 1, y0 = ybv[ty] - 1, y1 = ybv[ty + 1] - 1;
      if (x0 - 1 >= lsx0 && x0 - 1 <= lsx1 && y0 + 1 >= lsy0 && y1 <= lsy1) v |= 1 << 27;
      if (y0 >= lsy0 && y0 <= lsy1 && x0 >= lsx0 && x1 <= lsx1) v |= 1 << 28;
    };
    for (int &v : F->gitems) mark(v, false);
    for (int &v : narrow) mark(v, true);
  }
  // one launch takes both shapes (bit 31 marks a 16-column tile): chunk-0 items
  // first (the early launch of multi-rank steps), then the rest longest first
  // (most planes), so the shortest items fill the launch's tail
  std::vector<int> all;
  all.reserve(F->gitems.size() + narrow.size());
  for (int v : F->gitems)
    if (((v >> 16) & 255) == 0) all.push_back(v);
  for (int v : narrow)
    if (((v >> 16) & 255) == 0) all.push_back(v);
  a.ngen_e = (int)all.size();
  std::vector<int> rest;
  for (int v : F->gitems)
    if (((v >> 16) & 255) != 0) rest.push_back(v);
  for (int v : narrow)
    if (((v >> 16) & 255) != 0) rest.push_back(v);
  auto planes = [&](int v) {
    const int ch = (v >> 16) & 255;
    return a.zb[ch + 1] - a.zb[ch];
  };
  std::stable_sort(rest.begin(), rest.end(), [&](int x, int y) { return planes(x) > planes(y); });
  all.insert(all.end(), rest.begin(), rest.end());
  F->gitems.swap(all);
  a.ngen = (int)F->gitems.size();
  a.ngen_n = a.ngen_ne = 0;
  for (int k = 0; k < 3; k++) {
    a.N[k] = g.N[k];
    a.off[k] = g.off[k];
    a.osh_lo[k] = g.owned_lo_sh[k];
    a.osh_hi[k] = std::min(g.owned_hi_sh[k], G.hi[k]);
    a.oun_lo[k] = g.owned_lo_un[k];
    a.oun_hi[k] = std::min(g.owned_hi_un[k], G.hi[k]);
  }
  // ---- shell: the top plane of a rank with an upper neighbour
  BoxList &bl = F->fused_shell;
  memset(&bl, 0, sizeof(bl));
  if (F->nranks > 1 && F->rank + 1 < F->nranks) {
    Box b;
    for (int k = 0; k < 3; k++) b.lo[k] = 0, b.hi[k] = g.N[k] - 1;
    b.lo[2] = b.hi[2] = g.N[2] - 1;
    bl.b[0] = b;
    bl.start[0] = 0;
    bl.start[1] = (long long)g.N[0] * g.N[1];
    bl.n = 1;
  }
  return true;
}

// E of component c at global point jg is implicit (chi1inv * D) in fused mode
bool in_fused_box(const mnl_fields *F, int c, const int jg[3]) {
  if (!F->fused || ctype(c) != T_E) return false;
  const DevGrid &g = F->g;
  const int d = cdir(c);
  for (int e = 0; e < 3; e++) {
    if (g.ax[e] < 0) continue;
    const int j = jg[e] - g.off[e];
    if (j < F->fusedG.lo[g.ax[e]] || j > F->fusedG.hi[g.ax[e]]) return false;
    const bool sh = e == d;
    if (sh ? (j < g.owned_lo_sh[e] || j > g.owned_hi_sh[e])
           : (j < g.owned_lo_un[e] || j > g.owned_hi_un[e]))
      return false;
  }
  for (int k = 0; k < F->f.npol; k++) {  // E is stored inside the polarization boxes
    const Box &b = F->f.pol[k].nz;
    bool in = true;
    for (int e = 0; e < 3; e++) {
      const int j = g.ax[e] >= 0 ? jg[e] - g.off[e] : 0;
      in = in && j >= b.lo[e] && j <= b.hi[e];
    }
    if (in) return false;
  }
  const int q = 2 * jg[d] + 1;  // E_d is shifted along d
  return !(F->S.has[d] && F->h_flag[d][q]);
}

int nr_split(mnl_fields *F);

// chi(2) Newton-Raphson in the fused mode (one rank): the fused kernels store D everywhere
// and leave E and P of the chi2 box grown by one point (the NR neighbour reads of D - P,
// src/step_generic.cpp:740-743, stay inside it) to the NR E kernel; that box must lie in the
// interior (no PML, no wall plane) and inside the polarization box, where the fused
// kernels store E (elsewhere E is implicit and the NR kernel's stores would be lost)
bool nr_fused_ok(mnl_fields *F) {
  if (F->nranks > 1 || F->f.npol == 0) return false;
  if (nr_split(F)) return false;
  Box &x = F->nr_xbox;
  const Box &c = F->nr_chi2;
  if (c.hi[0] < c.lo[0] || c.hi[1] < c.lo[1] || c.hi[2] < c.lo[2]) {  // no chi2 point
    for (int k = 0; k < 3; k++) x.lo[k] = 1, x.hi[k] = 0;
    return true;
  }
  Box p;
  for (int k = 0; k < 3; k++) p.lo[k] = INT32_MAX, p.hi[k] = -1;
  for (int q = 0; q < F->f.npol; q++)
    for (int k = 0; k < 3; k++) {
      p.lo[k] = std::min(p.lo[k], F->f.pol[q].nz.lo[k]);
      p.hi[k] = std::max(p.hi[k], F->f.pol[q].nz.hi[k]);
    }
  for (int k = 0; k < 3; k++) {
    x.lo[k] = c.lo[k] - 1, x.hi[k] = c.hi[k] + 1;
    if (x.lo[k] < F->interior.lo[k] || x.hi[k] > F->interior.hi[k]) return false;
    if (x.lo[k] < p.lo[k] || x.hi[k] > p.hi[k]) return false;
  }
  return true;
}

bool fused_possible(mnl_fields *F) {
  if (!F->allow_fused || F->S.dim != 3 || F->upnl || F->f.aniso || F->hall) return false;
  if (F->nr && !nr_fused_ok(F)) return false;
  for (int t = 0; t < 2; t++)
    for (int d = 0; d < 3; d++)
      if (F->f.cnd[t][d]) return false;
  if (F->any_srcB || F->any_isrc || F->any_dsrc_w) return false;
  // a D source inside a polarization box would need E recomputed after it
  // (local check; fused_agreed makes the decision collective)
  for (size_t k = 0; k < F->srcD_idx.size(); k++) {
    const long long idx = F->srcD_idx[k];
    const long long i2 = idx / F->g.st[2], r = idx % F->g.st[2];
    const int j[3] = {(int)(r % F->g.st[1]), (int)(r / F->g.st[1]), (int)i2};
    for (int q = 0; q < F->f.npol; q++) {
      const Box &b = F->f.pol[q].nz;
      bool in = true;
      for (int e = 0; e < 3; e++) in = in && j[e] >= b.lo[e] && j[e] <= b.hi[e];
      if (in) return false;
    }
  }
  for (int c = 0; c < MNL_NUM_COMPONENTS; c++)
    if (!F->allocated[c]) return false;
  for (int d = 0; d < 3; d++)  // separate H wherever PML lies along its direction
    if (F->pml_any[d] && (!F->f.H[d] || !F->f.WH[d] || !F->f.WE[d])) return false;
  const int nu = (F->f.inveps[0] ? 1 : 0) + (F->f.inveps[1] ? 1 : 0) + (F->f.inveps[2] ? 1 : 0);
  if (nu != 0 && nu != 3) return false;
  // the fused kernels address arrays with 32-bit byte offsets
  if (F->nlocal * 8 >= 0xFFFFFFF0ull) return false;
  // the tile / chunk geometry is built on entering the fused mode and uploaded by
  // set_fused; every change of its inputs (z-chunk, A/B switches) leaves the mode first,
  // so a batch that is already fused reuses it (no per-call host rebuild)
  if (F->fused) return true;
  if (!make_fused_boxes(F)) return false;
  return true;
}

// fused mode only if every rank can (the ranks' exchange sequences differ by mode)
bool fused_agreed(mnl_fields *F) {
  bool ok = fused_possible(F);
  if (F->nranks > 1) {
    double v = ok ? 1.0 : 0.0;
    if (F->comm->allreduce_sum(&v, 1, F->stream)) return false;
    ok = v == double(F->nranks);
  }
  return ok;
}

// per-direction PML tables of the fused kernels (identity where no PML)
int upload_fused_tables(mnl_fields *F) {
  if (F->d_tab.flag[0]) return 0;
  for (int d = 0; d < 3; d++) {
    const size_t nq = 2 * (size_t)std::max(F->S.n[d], 0) + 2;
    std::vector<uint8_t> fl(nq, 0);
    std::vector<double> kms(nq, 1.0), kps(nq, 1.0), si(nq, 1.0);
    if (F->S.has[d] && !F->h_flag[d].empty())
      for (size_t q = 0; q < nq; q++) {
        fl[q] = F->h_flag[d][q];
        kms[q] = F->h_kap[d][q] - F->h_sig[d][q];
        kps[q] = F->h_kap[d][q] + F->h_sig[d][q];
        si[q] = F->h_siginv[d][q];
      }
    uint8_t *dfl;
    double *dkms, *dkps, *dsi;
    if (dev_alloc(F, &dfl, nq) || dev_alloc(F, &dkms, nq) || dev_alloc(F, &dkps, nq) ||
        dev_alloc(F, &dsi, nq))
      return -1;
    HIPCHK(hipMemcpyAsync(dfl, fl.data(), nq, hipMemcpyHostToDevice, F->stream));
    HIPCHK(hipMemcpyAsync(dkms, kms.data(), nq * 8, hipMemcpyHostToDevice, F->stream));
    HIPCHK(hipMemcpyAsync(dkps, kps.data(), nq * 8, hipMemcpyHostToDevice, F->stream));
    HIPCHK(hipMemcpyAsync(dsi, si.data(), nq * 8, hipMemcpyHostToDevice, F->stream));
    HIPCHK(hipStreamSynchronize(F->stream));
    F->d_tab.flag[d] = dfl;
    F->d_tab.kms[d] = dkms;
    F->d_tab.kps[d] = dkps;
    F->d_tab.siginv[d] = dsi;
  }
  return 0;
}

// chi1inv palette for the fused kernel (DESIGN.md "chi1inv palette"): at most
// 256 distinct values per component, candidates taken from the structure (1.0
// default, user chi1inv arrays, 1/eps of geometry boxes) and verified cell by
// cell on the device (bitwise), so a missing value just disables the palette.
int build_palette(mnl_fields *F) {
  if (F->palette_tried) return 0;
  F->palette_tried = true;
  const mnl_structure &S = F->S;
  DevFields &f = F->f;
  if (!f.inveps[0] || !f.inveps[1] || !f.inveps[2]) return 0;
  if (F->no_palette) return 0;
  std::vector<double> tab(3 * 256, 0.0);
  int n[3];
  for (int c = 0; c < 3; c++) {
    std::set<uint64_t> cand;
    auto bits = [](double v) {
      uint64_t u;
      memcpy(&u, &v, 8);
      return u;
    };
    cand.insert(bits(1.0));
    const auto &diag = S.chi1inv[c][c];
    if (!diag.empty()) {
      std::unordered_set<uint64_t> us;
      for (double v : diag) {
        us.insert(bits(v));
        if (us.size() > 256) return 0;
      }
      cand.insert(us.begin(), us.end());
    }
    for (auto &b : S.boxes)
      if (b.kind == 0) cand.insert(bits(1.0 / b.value));
    if (cand.size() > 256) return 0;
    n[c] = (int)cand.size();
    int k = 0;
    for (uint64_t u : cand) memcpy(&tab[256 * c + k++], &u, 8);  // ascending bit patterns
  }
  unsigned *uidx = nullptr;
  double *utab;
  int *bad;
  if (dev_alloc(F, &uidx, F->nlocal) || dev_alloc(F, &utab, 3 * 256) || dev_alloc(F, &bad, 1))
    return -1;
  HIPCHK(hipMemcpyAsync(utab, tab.data(), tab.size() * 8, hipMemcpyHostToDevice, F->stream));
  const double *u[3] = {f.inveps[0], f.inveps[1], f.inveps[2]};
  if (k_build_uidx(uidx, u, utab, n, F->fusedG, F->g.st[1], F->g.st[2], bad, F->stream))
    return fail("palette index build failed");
  int hbad = 0;
  HIPCHK(hipMemcpyAsync(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost, F->stream));
  HIPCHK(hipStreamSynchronize(F->stream));
  if (hbad) return 0;
  F->d_uidx = uidx;
  F->d_utab = utab;
  return 0;
}

int set_fused(mnl_fields *F, bool on) {
  DevFields &f = F->f;
  if (on == F->fused) return 0;
  if (on) {
    if (!F->d_fused_ctr) {  // FUSED_NCTR work-queue counters, 128 B apart
      if (dev_alloc(F, &F->d_fused_ctr, FUSED_NCTR * 16)) return -1;
    }
    if (upload_fused_tables(F)) return -1;
    if (F->d_gitems_cap < F->gitems.size()) {
      if (F->d_gitems) hipFree(F->d_gitems);
      F->d_gitems = nullptr;
      HIPCHK(hipMalloc(&F->d_gitems, F->gitems.size() * sizeof(int)));
      F->d_gitems_cap = F->gitems.size();
    }
    if (!F->gitems.empty())
      HIPCHK(hipMemcpyAsync(F->d_gitems, F->gitems.data(), F->gitems.size() * sizeof(int),
                            hipMemcpyHostToDevice, F->stream));
    if (F->d_titems_cap < F->titems.size()) {
      if (F->d_titems) hipFree(F->d_titems);
      F->d_titems = nullptr;
      HIPCHK(hipMalloc(&F->d_titems, F->titems.size() * sizeof(int)));
      F->d_titems_cap = F->titems.size();
    }
    if (!F->titems.empty())
      HIPCHK(hipMemcpyAsync(F->d_titems, F->titems.data(), F->titems.size() * sizeof(int),
                            hipMemcpyHostToDevice, F->stream));
    if (build_palette(F)) return -1;
    // ping-pong partners; the second buffer starts as a copy (ghost / wall entries
    // that no kernel writes)
    auto pair = [&](double **pp, double *cur, double **next) -> int {
      if (!cur) return 0;
      if (!*pp && dev_alloc(F, pp, F->nlocal, false)) return -1;
      HIPCHK(hipMemcpyAsync(*pp, cur, F->nlocal * 8, hipMemcpyDeviceToDevice, F->stream));
      *next = *pp;
      return 0;
    };
    for (int d = 0; d < 3; d++) {
      if (pair(&F->pp_B[d], f.B[d], &f.Bn[d]) || pair(&F->pp_D[d], f.D[d], &f.Dn[d]) ||
          pair(&F->pp_E[d], f.E[d], &f.En[d]) || pair(&F->pp_H[d], f.H[d], &f.Hn[d]) ||
          pair(&F->pp_UB[d], f.UB[d], &f.UBn[d]))
        return -1;
    }
    f.fG = F->fusedG;
    f.fused = 1;
    F->fused_epoch++;  // the temporal-blocking plan and its middle set are rebuilt
    F->tb_mid_fresh = false;
  } else {
    // materialise implicit E and the W aux fields over G (needs f.fused == 1),
    // then step in place again
    if (k_materialize_e(F->fusedG, F->g, f, F->stream)) return fail("materialize E failed");
    for (int d = 0; d < 3; d++) {
      F->pp_B[d] = f.Bn[d];  // the non-current buffers
      F->pp_D[d] = f.Dn[d];
      if (f.E[d]) F->pp_E[d] = f.En[d];
      if (f.H[d]) F->pp_H[d] = f.Hn[d];
      if (f.UB[d]) F->pp_UB[d] = f.UBn[d];
      f.Bn[d] = f.B[d];
      f.Dn[d] = f.D[d];
      f.En[d] = f.E[d];
      f.Hn[d] = f.H[d];
      f.UBn[d] = f.UB[d];
    }
    f.fused = 0;
  }
  F->fused = on;
  HIPCHK(hipStreamSynchronize(F->stream));
  return 0;
}

enum {
  TM_B = 0, TM_H, TM_D, TM_E, TM_SRC, TM_HALO, TM_BINT, TM_DINT, TM_GEN, TM_DFT, TM_DFTF,
  TM_TB,   // two-step kernel (temporal blocking), one launch per pair of steps
  TM_RIM,  // rim launches of the pairs (two per pair)
  TM_CHAIN,  // multi-rank pairs: a slab-face chain on the comm stream (two per pair)
  TM_WAIT,   // multi-rank pairs: the main stream waiting for the chain's E ghost (two per pair)
  TM_N
};

struct EvPair {
  hipEvent_t a, b;
  int cat;
};

// kernel arguments of one fused step (geometry from make_fused_boxes, pointers now)
FusedArgs &fused_args(mnl_fields *F) {
  FusedArgs &fa = F->fgeo;
  const DevFields &f = F->f;
  fa.blocks_per_cu = F->fused_bpc;
  fa.dist = F->fused_dist;
  fa.nelem = (long long)F->nlocal;
  fa.C = F->S.courant;
  fa.st1 = F->g.st[1];
  fa.st2 = F->g.st[2];
  for (int d = 0; d < 3; d++) {
    fa.Bo[d] = f.B[d];
    fa.Bn[d] = f.Bn[d];
    fa.Do[d] = f.D[d];
    fa.Dn[d] = f.Dn[d];
    fa.E[d] = f.E[d];
    fa.En[d] = f.En[d];
    fa.Ho[d] = f.H[d];
    fa.Hn[d] = f.Hn[d];
    fa.UBo[d] = f.UB[d];
    fa.UBn[d] = f.UBn[d];
    fa.UD[d] = f.UD[d];
    fa.u[d] = f.inveps[d];
  }
  fa.tab = F->d_tab;
  fa.npol = f.npol;
  for (int k = 0; k < MAX_POL; k++) fa.pol[k] = f.pol[k];
  for (int e = 0; e < 3; e++) fa.pbox.lo[e] = INT32_MAX, fa.pbox.hi[e] = -1;
  for (int k = 0; k < f.npol; k++)
    for (int e = 0; e < 3; e++) {
      fa.pbox.lo[e] = std::min(fa.pbox.lo[e], f.pol[k].nz.lo[e]);
      fa.pbox.hi[e] = std::max(fa.pbox.hi[e], f.pol[k].nz.hi[e]);
    }
  for (int e = 0; e < 3; e++) fa.xbox.lo[e] = 1, fa.xbox.hi[e] = 0;
  if (F->nr) fa.xbox = F->nr_xbox;
  fa.gitems = F->d_gitems;
  fa.titems = F->d_titems;
  fa.tflag = nullptr;
  fa.uidx = F->d_uidx;
  fa.utab = F->d_utab;
  fa.uflag = nullptr;
  fa.gflag = nullptr;
  if (F->d_uidx && F->uniform) {
    // flags of the current tile / chunk geometry (rebuilt if make_fused_boxes changed it)
    unsigned long long sig = 1469598103934665603ULL;
    auto mix = [&](long long v) { sig = (sig ^ (unsigned long long)v) * 1099511628211ULL; };
    for (int i = 0; i <= fa.nx; i++) mix(fa.xb[i]);
    for (int i = 0; i <= fa.ny; i++) mix(fa.yb[i]);
    for (int i = 0; i <= fa.nch; i++) mix(fa.zb[i]);
    for (int k = 0; k < 3; k++) mix(fa.L.lo[k]), mix(fa.L.hi[k]);
    mix(fa.lx0), mix(fa.lx1), mix(fa.ly0), mix(fa.ly1), mix(fa.nch);
    for (int i = 0; i <= fa.ngy; i++) mix(fa.gyb[i]);
    for (int i = 0; i <= fa.nny; i++) mix(fa.nyb[i]);
    for (int v : F->gitems) mix(v);
    for (int v : F->titems) mix(v);
    const long long ntile = (long long)(fa.lx1 - fa.lx0 + 1) * (fa.ly1 - fa.ly0 + 1);
    const size_t n = ntile > 0 ? (size_t)ntile * fa.nch : 0, ng = F->gitems.size();
    const size_t nt = F->titems.size();
    auto grow = [](unsigned *&p, size_t &cap, size_t want) {
      if (cap >= want) return true;
      if (p) hipFree(p);
      p = nullptr;
      const bool r = hipMalloc(&p, std::max<size_t>(want, 1) * sizeof(unsigned)) == hipSuccess;
      cap = r ? want : 0;
      return r;
    };
    bool ok = true;
    if (F->uflag_sig != sig) {
      ok = grow(F->d_uflag, F->uflag_n, n) && grow(F->d_gflag, F->gflag_n, ng) &&
           grow(F->d_tflag, F->tflag_n, nt) &&
           k_lean_uniform(fa, F->d_uflag, F->stream) == 0 &&
           k_general_uniform(fa, F->d_gflag, F->stream) == 0 &&
           k_tile_uniform(fa, F->d_tflag, F->stream) == 0;
      F->uflag_sig = ok ? sig : 0;
      if (ok) {  // per-item cell counts of the mixed items (traffic model)
        std::vector<unsigned> hl(n), hg(ng), ht(nt);
        ok = (n == 0 || hipMemcpyAsync(hl.data(), F->d_uflag, n * 4, hipMemcpyDeviceToHost,
                                       F->stream) == hipSuccess) &&
             (nt == 0 || hipMemcpyAsync(ht.data(), F->d_tflag, nt * 4, hipMemcpyDeviceToHost,
                                        F->stream) == hipSuccess) &&
             (ng == 0 || hipMemcpyAsync(hg.data(), F->d_gflag, ng * 4, hipMemcpyDeviceToHost,
                                        F->stream) == hipSuccess) &&
             hipStreamSynchronize(F->stream) == hipSuccess;
        double ln = 0, gn = 0;
        const int nlx = fa.lx1 - fa.lx0 + 1;
        for (size_t i = 0; ok && i < n; i++) {
          const int t = (int)(i / fa.nch), ch = (int)(i % fa.nch);
          bool lean = false;
          for (int r = 0; r < fa.nlzr; r++) lean = lean || (ch >= fa.lzr[r][0] && ch <= fa.lzr[r][1]);
          if (!lean || hl[i] != ~0u) continue;
          const int tx = fa.lx0 + t % nlx, ty = fa.ly0 + t / nlx;
          ln += double(fa.xb[tx + 1] - fa.xb[tx]) * (fa.yb[ty + 1] - fa.yb[ty]) *
                (fa.zb[ch + 1] - fa.zb[ch]);
        }
        for (size_t i = 0; ok && i < ng; i++) {
          if (hg[i] != ~0u) continue;
          const int v = F->gitems[i], tx = v & 255, ty = (v >> 8) & 255, ch = (v >> 16) & 255;
          const int *yb = (v & (int)0x80000000u) ? fa.nyb : fa.gyb;
          gn += double(fa.xb[tx + 1] - fa.xb[tx]) * (yb[ty + 1] - yb[ty]) *
                (fa.zb[ch + 1] - fa.zb[ch]);
        }
        double tn = 0;
        for (size_t i = 0; ok && i < nt; i++) {
          if (ht[i] != ~0u) continue;
          const int v = F->titems[i], tx = v & 255, ty = (v >> 8) & 255, ch = (v >> 16) & 255;
          tn += double(fa.xb[tx + 1] - fa.xb[tx]) * (fa.yb[ty + 1] - fa.yb[ty]) *
                (fa.zb[ch + 1] - fa.zb[ch]);
        }
        F->lean_cells_nu = ln;
        F->gen_cells_nu = gn;
        F->tile_cells_nu = tn;
        if (!ok) F->uflag_sig = 0;
      }
    }
    if (ok) {
      fa.uflag = n ? F->d_uflag : nullptr;
      fa.gflag = ng ? F->d_gflag : nullptr;
      fa.tflag = nt ? F->d_tflag : nullptr;
    }
  }
  F->uflag_active = fa.uflag || fa.gflag || fa.tflag;
  fa.ctr = F->d_fused_ctr;
  fa.clk = ItemClock{F->d_clk, F->d_clk_n, F->d_clk ? CLK_CAP : 0u, 0};
  fa.ngrp = F->lean_groups;  // lean queue groups; general: gen_groups
  fa.ngrp_gen = F->gen_groups;
  return fa;
}

int fused_fail(const char *what, int kr) {
  return fail(std::string(what) + " (" + std::to_string(kr) + ", " +
              hipGetErrorString(hipGetLastError()) + ")");
}

// CUs given to the general kernel when it runs beside the lean one: its share
// of the step's work (general tile-planes cost ~2.5x a lean cell's bandwidth
// time per cell), or MNL_GEN_CUS; 0 = run the two kernels one after the other
int gen_split(const mnl_fields *F) { return F->gen_cus >= 0 ? F->gen_cus : 0; }

// tile mode, one rank: CUs of the polarization chunks' general kernel beside the tile
// kernel (0: after it on the same stream; the tuner's choice, or MNL_TILE_GEN_CUS)
int tile_gen_split(const mnl_fields *F) {
  const int v = F->tile_gen_cus;
  const int cus = k_cu_count();
  return (v > 0 && v < cus) ? v : 0;
}

// streams / events of the overlapped multi-rank step; the E ghost plane is made
// valid once (kind 0) since each step ends with the exchange for the next one
int multi_begin(mnl_fields *F) {
  if (!F->s_comm) {
    HIPCHK(hipStreamCreateWithFlags(&F->s_comm, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&F->s_aux, hipStreamNonBlocking));
    for (hipEvent_t *e : {&F->ev_start, &F->ev_early, &F->ev_x1, &F->ev_shell, &F->ev_x0})
      HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
  }
  HIPCHK(hipEventRecord(F->ev_start, F->stream));
  HIPCHK(hipStreamWaitEvent(F->s_comm, F->ev_start, 0));
  if (exchange(F, 0, F->s_comm)) return fail("E halo exchange failed");
  HIPCHK(hipEventRecord(F->ev_x0, F->s_comm));
  return 0;
}

// One fused step of a rank with neighbours.  Chunk 0 (planes 0..1: the B that
// the lower neighbour needs) runs first on s_aux; its B/H plane goes down while
// the interior runs on the main stream; the top plane (shell) follows once the
// upper neighbour's plane has arrived, and its E goes up for the next step.
template <class EB, class EE>
int step_fused_multi(mnl_fields *F, const SrcDev &sD, EB &ev_begin, EE &ev_end) {
  DevFields &f = F->f;
  const DevGrid &g = F->g;
  FusedArgs &fa = fused_args(F);
  HIPCHK(hipEventRecord(F->ev_start, F->stream));
  HIPCHK(hipStreamWaitEvent(F->s_aux, F->ev_start, 0));
  HIPCHK(hipStreamWaitEvent(F->s_aux, F->ev_x0, 0));
  int kr = F->tile_mode ? k_fused(fa, 5, F->s_aux, F->ctr_base) : 0;
  if (!kr) kr = k_fused(fa, 2, F->s_aux, F->ctr_base);
  if (kr) return fused_fail("fused early kernel launch failed", kr);
  HIPCHK(hipEventRecord(F->ev_early, F->s_aux));
  HIPCHK(hipStreamWaitEvent(F->s_comm, F->ev_early, 0));
  if (exchange(F, 1, F->s_comm)) return fail("H halo exchange failed");
  HIPCHK(hipEventRecord(F->ev_x1, F->s_comm));
  int k = ev_begin(TM_BINT);
  // the persistent main launch leaves TB_RES_CUS CUs to the chunk-0 launch on s_aux and
  // the slab-face work after it, so they cannot queue behind it for the whole step
  fa.wg_limit = F->tile_mode ? k_cu_count() - TB_RES_CUS : 0;
  kr = k_fused(fa, F->tile_mode ? 6 : 0, F->stream, F->ctr_base);
  fa.wg_limit = 0;
  if (kr) return fused_fail("fused kernel launch failed", kr);
  ev_end(k);
  if (!F->tile_mode || fa.ngen > fa.ngen_e) {
    k = ev_begin(TM_GEN);
    fa.lean_after = F->tile_mode ? 0 : lean_halo_reads(F);  // same stream, after the lean launch
    kr = k_fused(fa, 3, F->stream, F->ctr_base);
    fa.lean_after = 0;
    if (kr) return fused_fail("fused general kernel launch failed", kr);
    ev_end(k);
  }
  const BoxList *sl = &F->fused_shell;
  if (k_curl(T_B, F->interior, sl, g, f, F->planB, F->S.courant, F->stream, true))
    return fail("curl B launch failed");
  HIPCHK(hipStreamWaitEvent(F->stream, F->ev_x1, 0));
  const bool fuseE = !F->dsrc_in_shell && f.npol == 0;
  if (k_curl(T_D, F->interior, sl, g, f, F->planD, F->S.courant, F->stream, fuseE))
    return fail("curl D launch failed");
  if (sD.n && k_source(T_D, g, f, sD, 0, F->stream)) return fail("source launch failed");
  if (!fuseE) {
    ISrcDev is{};
    if (k_update_e(F->interior, sl, g, f, is, 0, true, F->stream))
      return fail("update E launch failed");
  }
  HIPCHK(hipEventRecord(F->ev_shell, F->stream));
  for (int d = 0; d < 3; d++) {
    std::swap(f.B[d], f.Bn[d]);
    std::swap(f.D[d], f.Dn[d]);
    std::swap(f.E[d], f.En[d]);
    std::swap(f.H[d], f.Hn[d]);
    std::swap(f.UB[d], f.UBn[d]);
  }
  HIPCHK(hipStreamWaitEvent(F->s_comm, F->ev_shell, 0));
  if (exchange(F, 0, F->s_comm)) return fail("E halo exchange failed");
  HIPCHK(hipEventRecord(F->ev_x0, F->s_comm));
  return 0;
}

// first update_eh(H_stuff): H = copy of B and f_w = copy of H where they are
// separate (src/update_eh.cpp:204-216)
int h_lazy_copy(mnl_fields *F) {
  DevFields &f = F->f;
  for (int d = 0; d < 3; d++) {
    if (!f.H[d] || !f.Bn[d]) continue;
    if (k_copy(f.H[d], f.Bn[d], (long long)F->nlocal, F->stream)) return fail("copy launch failed");
    if (f.WH[d] && k_copy(f.WH[d], f.Bn[d], (long long)F->nlocal, F->stream))
      return fail("copy launch failed");
  }
  F->h_first_done = true;
  return 0;
}
// first step_db(B_stuff / D_stuff): f_u = copy of f where a PML lies along
// dsigu (src/step_db.cpp:71-75)
int u_lazy_copy(mnl_fields *F, int which) {
  DevFields &f = F->f;
  for (int d = 0; d < 3; d++) {
    double *u = which == 0 ? f.UB[d] : f.UD[d];
    const double *src = which == 0 ? f.B[d] : f.D[d];
    if (u && src && k_copy(u, src, (long long)F->nlocal, F->stream)) return fail("copy launch failed");
  }
  F->u_first_done[which] = true;
  return 0;
}
// first update_eh(E_stuff): f_w = copy of E (src/update_eh.cpp:212-216)
int e_lazy_copy(mnl_fields *F) {
  DevFields &f = F->f;
  for (int d = 0; d < 3; d++)
    if (f.WE[d] && f.E[d] &&
        k_copy(f.WE[d], f.E[d], (long long)F->nlocal, F->stream))
      return fail("copy launch failed");
  F->e_first_done = true;
  return 0;
}

// update_eh(H_stuff) [+ update_pols(H_stuff) when pols]: the PML W update over the shell boxes, or,
// with H-side materials, the H kernel over the whole rank-local box
int update_h_any(mnl_fields *F, const BoxList &sl, bool pols) {
  if (F->hall) {
    Box all;
    for (int k = 0; k < 3; k++) all.lo[k] = 0, all.hi[k] = F->g.N[k] - 1;
    if (k_update_hmat(all, F->g, F->f, pols ? 1 : 0, F->stream)) return fail("update H launch failed");
    return 0;
  }
  bool anyH = false;
  for (int d = 0; d < 3; d++) anyH = anyH || F->f.H[d];
  if (anyH && k_update_h(sl, F->g, F->f, F->stream)) return fail("update H launch failed");
  return 0;
}

// Interior E update with chi(2) Newton-Raphson: the NR kernel over the bounding
// box of chi2 != 0 inside the interior, the plain kernel over the rest (outside
// that box chi2 = 0, so every point takes E = chi1inv * (D - P) either way).
int nr_split(mnl_fields *F) {
  const DevGrid &g = F->g;
  if (!F->nr_split_done) {
    int *d = nullptr;
    HIPCHK(hipMalloc(&d, 6 * sizeof(int)));
    std::unique_ptr<void, void (*)(void *)> guard(d, [](void *p) { (void)hipFree(p); });
    int box[6] = {INT32_MAX, INT32_MAX, INT32_MAX, -1, -1, -1};
    HIPCHK(hipMemcpyAsync(d, box, sizeof box, hipMemcpyHostToDevice, F->stream));
    const double *c2[3] = {F->f.chi2[0], F->f.chi2[1], F->f.chi2[2]};
    if (k_nonzero_box(c2, g, d, F->stream)) return fail("chi2 box failed");
    HIPCHK(hipMemcpyAsync(box, d, sizeof box, hipMemcpyDeviceToHost, F->stream));
    HIPCHK(hipStreamSynchronize(F->stream));
    const Box &I = F->interior;
    Box n;
    bool empty = false;
    F->nr_shell_free = true;  // chi2 != 0 nowhere outside the interior box
    for (int k = 0; k < 3; k++) F->nr_chi2.lo[k] = box[k], F->nr_chi2.hi[k] = box[3 + k];
    for (int k = 0; k < 3; k++) {  // 3-D: device axis k == direction k
      n.lo[k] = std::max(box[k], I.lo[k]);
      n.hi[k] = std::min(box[3 + k], I.hi[k]);
      empty = empty || n.hi[k] < n.lo[k];
      if (box[3 + k] >= box[k] && (box[k] < I.lo[k] || box[3 + k] > I.hi[k]))
        F->nr_shell_free = false;
    }
    F->nr_rest.clear();
    if (empty) {
      F->nr_in.lo[0] = 1, F->nr_in.hi[0] = 0;
      F->nr_rest.push_back(I);
    } else {
      F->nr_in = n;
      Box r = I;  // peel z, then y, then x slabs off the interior
      for (int k = 2; k >= 0; k--) {
        if (r.lo[k] < n.lo[k]) {
          Box b = r;
          b.hi[k] = n.lo[k] - 1;
          F->nr_rest.push_back(b);
        }
        if (r.hi[k] > n.hi[k]) {
          Box b = r;
          b.lo[k] = n.hi[k] + 1;
          F->nr_rest.push_back(b);
        }
        r.lo[k] = n.lo[k], r.hi[k] = n.hi[k];
      }
    }
    F->nr_split_done = true;
  }
  return 0;
}

int nr_interior_e(mnl_fields *F, const ISrcDev &is) {
  const DevGrid &g = F->g;
  if (nr_split(F)) return -1;
  if (F->nr_in.hi[0] >= F->nr_in.lo[0] &&
      k_update_e(F->nr_in, nullptr, g, F->f, is, 0, false, F->stream))
    return fail("update E launch failed");
  DevFields plain = F->f;
  plain.nr_enabled = 0;
  for (const Box &b : F->nr_rest)
    if (k_update_e(b, nullptr, g, plain, is, 0, false, F->stream)) return fail("update E launch failed");
  return 0;
}

constexpr int NR_HARD_CAP = 4096;  // deferred NR problems per E update (more: solved in place)

// Before an E update that may run the NR branch: enable deferral (MNL_NR_DEFER=0 solves
// every problem in place, sequentially) and clear the list; after it, the parallel pass.
int nr_defer_begin(mnl_fields *F, hipStream_t st = nullptr) {
  if (!F->d_nr_hard) return 0;
  F->f.nr_hard = F->nr_defer ? F->d_nr_hard : nullptr;
  if (F->f.nr_hard)
    HIPCHK(hipMemsetAsync(F->d_nr_hard_cnt, 0, sizeof(unsigned), st ? st : F->stream));
  return 0;
}
int nr_defer_end(mnl_fields *F, hipStream_t st = nullptr) {
  if (!F->f.nr_hard) return 0;
  if (k_nr_hard(F->f, st ? st : F->stream)) return fail("NR parallel-attempt kernel launch failed");
  return 0;
}

// Fused mode with chi(2) (nr_fused_ok): the fused kernels stored the new D (Dn) everywhere
// and E / P everywhere but the chi2 box grown by one point; here that box: E by the NR
// kernel (Newton-Raphson where chi2 != 0, chi1inv * (D - P) at the other points, the
// values the fused kernels would have stored), then update_P over it, as the unfused
// NR path orders them (src/step_generic.cpp:730-816, src/susceptibility.cpp:251-258)
int nr_fused_e(mnl_fields *F, const ISrcDev &is, hipStream_t st = nullptr) {
  const Box &x = F->nr_xbox;
  if (x.hi[0] < x.lo[0]) return 0;
  if (!st) st = F->stream;
  if (nr_defer_begin(F, st)) return -1;
  if (k_update_e(x, nullptr, F->g, F->f, is, 0, false, st)) return fail("update E launch failed");
  if (nr_defer_end(F, st)) return -1;
  if (k_update_pols(x, nullptr, F->g, F->f, st)) return fail("pols launch failed");
  return 0;
}

// The NR box's E phase may run right after the polarization chunks' general kernel, on its
// stream beside the tile kernel (it reads the new D of the box and the old E, writes only the
// box's new E / P -- points the tile kernel neither reads nor writes), when no D source point
// lies in the box (sources are added to the new D after the fused kernels)
bool nr_early_ok(const mnl_fields *F) {
  const Box &x = F->nr_xbox;
  if (!F->nr_early || x.hi[0] < x.lo[0]) return false;
  for (long long idx : F->srcD_idx) {
    const long long z = idx / F->g.st[2], r = idx % F->g.st[2];
    const long long y = r / F->g.st[1], xx = r % F->g.st[1];
    if (xx >= x.lo[0] && xx <= x.hi[0] && y >= x.lo[1] && y <= x.hi[1] && z >= x.lo[2] &&
        z <= x.hi[2])
      return false;
  }
  return true;
}

// ------------------------------------------------------------ temporal blocking
// (DESIGN.md section 24).  Two steps n -> n+2 of a one-rank fused run as three launches over
// three buffer sets (cur = state n, mid, nxt):
//   R1: the tile kernel over the rim items, cur -> mid (state n+1 on the rim);
//   source(n) into mid;
//   L:  the two-step kernel over the L2 items, cur -> nxt (state n+2), plus the state n+1 of
//       the L2 points on a face that borders the rim, into mid;
//   R2: the tile kernel over the rim items, mid -> nxt;  source(n+1) into nxt.
// L2 = the lean box shrunk by 2 minus boxes around the source points, so every value the
// two-step march computes is the lean body's (same expression, same operands): the pair is
// bitwise two one-step launches.  The rim is everything else of G: PML, walls, the ring of
// width >= 2 inside the lean box and the holes.

bool box_meets(const Box &a, const Box &b) {
  for (int k = 0; k < 3; k++)
    if (a.hi[k] < b.lo[k] || b.hi[k] < a.lo[k]) return false;
  return true;
}

// Disjoint boxes of G: `two` covers L2 minus the holes, `rim` the rest.  Cells of the grid of
// all box bounds, merged into x runs, then along y, then along z.
void tb_regions(const Box &G, const Box &L2, const std::vector<Box> &holes, std::vector<Box> &two,
                std::vector<Box> &rim) {
  std::vector<int> cut[3];
  for (int k = 0; k < 3; k++) {
    std::vector<int> &c = cut[k];
    c = {G.lo[k], G.hi[k] + 1, L2.lo[k], L2.hi[k] + 1};
    for (const Box &h : holes) c.push_back(h.lo[k]), c.push_back(h.hi[k] + 1);
    std::sort(c.begin(), c.end());
    c.erase(std::unique(c.begin(), c.end()), c.end());
    c.erase(std::remove_if(c.begin(), c.end(), [&](int v) { return v < G.lo[k] || v > G.hi[k] + 1; }),
            c.end());
  }
  auto is_two = [&](int x, int y, int z) {
    const int p[3] = {x, y, z};
    for (int k = 0; k < 3; k++)
      if (p[k] < L2.lo[k] || p[k] > L2.hi[k]) return false;
    for (const Box &h : holes) {
      bool in = true;
      for (int k = 0; k < 3; k++) in = in && p[k] >= h.lo[k] && p[k] <= h.hi[k];
      if (in) return false;
    }
    return true;
  };
  std::vector<Box> out[2];
  const int nx = (int)cut[0].size() - 1, ny = (int)cut[1].size() - 1, nz = (int)cut[2].size() - 1;
  for (int l = 0; l < nz; l++)
    for (int j = 0; j < ny; j++)
      for (int i = 0; i < nx;) {
        const bool c = is_two(cut[0][i], cut[1][j], cut[2][l]);
        int i2 = i;
        while (i2 + 1 < nx && is_two(cut[0][i2 + 1], cut[1][j], cut[2][l]) == c) i2++;
        Box b;
        b.lo[0] = cut[0][i], b.hi[0] = cut[0][i2 + 1] - 1;
        b.lo[1] = cut[1][j], b.hi[1] = cut[1][j + 1] - 1;
        b.lo[2] = cut[2][l], b.hi[2] = cut[2][l + 1] - 1;
        out[c ? 1 : 0].push_back(b);
        i = i2 + 1;
      }
  auto merge = [](std::vector<Box> &v, int ax) {
    for (bool changed = true; changed;) {
      changed = false;
      for (size_t a = 0; a < v.size() && !changed; a++)
        for (size_t b = 0; b < v.size(); b++) {
          if (a == b || v[b].lo[ax] != v[a].hi[ax] + 1) continue;
          bool ok = true;
          for (int k = 0; k < 3 && ok; k++)
            if (k != ax) ok = v[a].lo[k] == v[b].lo[k] && v[a].hi[k] == v[b].hi[k];
          if (!ok) continue;
          v[a].hi[ax] = v[b].hi[ax];
          v.erase(v.begin() + (long)b);
          changed = true;
          break;
        }
    }
  };
  for (auto *v : {&out[0], &out[1]}) merge(*v, 1), merge(*v, 2);
  rim.swap(out[0]);
  two.swap(out[1]);
}

template <class T>
int dev_upload(mnl_fields *F, T **d, size_t &cap, const std::vector<T> &h) {
  if (h.empty()) return 0;
  if (cap < h.size()) {
    if (*d) (void)hipFree(*d);
    *d = nullptr;
    HIPCHK(hipMalloc(d, h.size() * sizeof(T)));
    cap = h.size();
  }
  HIPCHK(hipMemcpyAsync(*d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice, F->stream));
  return 0;
}

// Build (or keep) the plan of the current fused geometry and source points.  No plan (tb_have
// false) when L2 is empty or an item would not fit the kernels' shapes.
int tb_plan(mnl_fields *F) {
  F->tb_r1done_ok = false;
  unsigned long long sig = 1469598103934665603ULL;
  auto mix = [&](long long v) { sig = (sig ^ (unsigned long long)v) * 1099511628211ULL; };
  mix(F->fused_epoch), mix(F->tb_zchunk), mix(F->fused_zchunk), mix((long long)F->nlocal);
  mix(F->rim_zchunk), mix(F->tb_ox), mix(F->tb_px), mix(F->tb_pol_on), mix(F->tb_lint != 0), mix(F->tb_r2lpt), mix(F->tb_szc);
  mix((long long)F->srcD_idx.size());
  for (long long v : F->srcD_idx) mix(v);
  // DFT monitors (one rank): the Yee points their samples average, +1 along every axis --
  // the two-step items store step n+1 there too (the middle-step sample reads the mid set)
  std::vector<Box> dbox;
  std::vector<DftFluxH *> cmon;  // monitors whose box the two-step kernel stores compactly
  for (auto &op : F->dfts) {  // (built once per monitor: this runs every batch)
    if (op->bbox.hi[0] < 0) continue;
    if (F->dft_cmp && op->cmp_cells && (int)cmon.size() < TB_MAXCMP)
      cmon.push_back(op.get());
    else
      dbox.push_back(op->bbox);
  }
  mix((long long)cmon.size());
  for (auto *o : cmon)
    for (int k = 0; k < 3; k++) mix(o->bbox.lo[k]), mix(o->bbox.hi[k]);
  // the NaN guard's points (it checks the middle state of every pair, src/step.cpp:138-139)
  if (F->nan_terms.n > 0) {
    Box nb;
    for (int i = 0; i < F->nan_terms.n; i++) {
      const long long li = F->nan_terms.idx[i];
      const int p[3] = {(int)(li % F->g.st[1]), (int)((li % F->g.st[2]) / F->g.st[1]),
                        (int)(li / F->g.st[2])};
      for (int k = 0; k < 3; k++) {
        nb.lo[k] = i ? std::min(nb.lo[k], p[k]) : p[k];
        nb.hi[k] = i ? std::max(nb.hi[k], p[k]) : p[k];
      }
    }
    dbox.push_back(nb);
  }
  mix((long long)dbox.size());
  for (const Box &b : dbox)
    for (int k = 0; k < 3; k++) mix(b.lo[k]), mix(b.hi[k]);
  if (sig == F->tb_sig) return 0;
  F->tb_sig = sig;
  F->tb_have = false;
  F->tb_ritems.clear(), F->tb_rgeo.clear(), F->tb_items.clear();
  // compact DFT boxes: allocated once, emptied (DFT_CMP_EMPTY) with every new plan
  F->tb_cmp.clear();
  for (auto &op : F->dfts) op->cmp_on = false;
  for (auto *o : cmon) {
    const size_t nd = (size_t)12 * o->cmp_cells;
    if (!o->d_cmp && hipMalloc(&o->d_cmp, nd * 8) != hipSuccess) {
      (void)hipGetLastError();
      o->d_cmp = nullptr;
      dbox.push_back(o->bbox);  // no memory for it: the middle state in mid, as before
      continue;
    }
    double empty;
    const unsigned long long e = DFT_CMP_EMPTY;
    memcpy(&empty, &e, 8);
    if (k_fill(o->d_cmp, empty, nd, F->stream)) return fail("fill launch failed");
    TBCmp c{};
    for (int k = 0; k < 3; k++) c.lo[k] = o->bbox.lo[k], c.n[k] = o->bbox.hi[k] - o->bbox.lo[k] + 1;
    c.p = o->d_cmp, c.mask = o->cmp_mask, c.ncell = o->cmp_cells;
    F->tb_cmp.push_back(c);
    o->cmp_on = true;
  }
  const Box &G = F->fusedG, &L = F->fusedL;
  const FusedArgs &a = F->fgeo;
  const DevGrid &g = F->g;
  if (F->S.dim != 3 || g.N[0] > 65535 || g.N[1] > 65535 || g.N[2] > 65535) return 0;
  Box L2;
  for (int k = 0; k < 3; k++) L2.lo[k] = L.lo[k] + 2, L2.hi[k] = L.hi[k] - 2;
  // x: the rim to the right of L2 starts on a 128-byte boundary (tile-kernel items); the rim
  // to the left ends on one when that costs no more columns than starting the two-step tiles
  // 4 columns past a 64-byte boundary (their lanes' line) -- a 16-column left rim runs as
  // narrow strips (strip_body), and the first two-step tile of a row starts its lanes on the
  // line below its own columns
  {
    const int a16 = G.lo[0] + (L2.lo[0] - G.lo[0] + 15) / 16 * 16;
    const int a4 = L2.lo[0] + ((4 - L2.lo[0]) % 8 + 8) % 8;
    L2.lo[0] = (F->tb_narrow && a16 <= a4) ? a16 : a4;
  }
  L2.hi[0] = (L2.hi[0] + 1) / 16 * 16 - 1;
  bool l2 = true;
  for (int k = 0; k < 3; k++) l2 = l2 && L2.hi[k] - L2.lo[k] >= 7;
  // one rank: no two-step region, no pairs.  Multi-rank: a rank without one (thin slab, PML)
  // still steps pairs as two rim launches (every rank runs the same exchange sequence)
  if (!l2 && F->nranks == 1) {
    if (F->tb_stats) fprintf(stderr, "tb: L2 empty\n");
    return 0;
  }
  if (!l2)
    for (int k = 0; k < 3; k++) L2.lo[k] = 1, L2.hi[k] = 0;
  // holes: no source point within distance 1 of a two-step own point (the march's D^{n+1}
  // would miss the current); a box of +-2 for margin, x widened to the alignments above and
  // to the L2 edge when that leaves fewer than 8 columns
  std::vector<Box> holes;
  for (long long idx : F->srcD_idx) {
    const long long i2 = idx / g.st[2], r = idx % g.st[2];
    const int s[3] = {(int)(r % g.st[1]), (int)(r / g.st[1]), (int)i2};
    Box h;
    for (int k = 0; k < 3; k++) h.lo[k] = s[k] - 2, h.hi[k] = s[k] + 2;
    if (!l2 || !box_meets(h, L2)) continue;
    h.lo[0] = std::max(h.lo[0], 0) / 16 * 16;
    while ((h.hi[0] + 1) % 8 != 4) h.hi[0]++;
    for (int k = 0; k < 3; k++) h.lo[k] = std::max(h.lo[k], L2.lo[k]), h.hi[k] = std::min(h.hi[k], L2.hi[k]);
    if (h.lo[0] - L2.lo[0] < 8) h.lo[0] = L2.lo[0];
    if (L2.hi[0] - h.hi[0] < 8) h.hi[0] = L2.hi[0];
    holes.push_back(h);
  }
  // polarization chunks (tile mode: the planes [pzl - 1, pzh + 2) over the whole x-y extent of
  // G, make_tile_boxes): stepped by the general kernel, not by rim items; no two-step point
  // within distance 2 of them (their E is stored, not chi1inv D)
  Box P;
  bool have_p = false;
  if (F->f.npol > 0 && a.ngen > 0) {
    int pzl = INT32_MAX, pzh = -1;
    for (int k = 0; k < F->f.npol; k++)
      if (F->f.pol[k].nz.lo[2] <= F->f.pol[k].nz.hi[2]) {
        pzl = std::min(pzl, F->f.pol[k].nz.lo[2]);
        pzh = std::max(pzh, F->f.pol[k].nz.hi[2]);
      }
    if (pzh >= 0) {
      P = G;
      P.lo[2] = std::max(G.lo[2], pzl - 1), P.hi[2] = std::min(G.hi[2], pzh + 1);
      have_p = P.lo[2] <= P.hi[2];
    }
    if (have_p && l2) {
      Box h = L2;
      h.lo[2] = std::max(L2.lo[2], P.lo[2] - 2), h.hi[2] = std::min(L2.hi[2], P.hi[2] + 2);
      if (h.lo[2] <= h.hi[2]) holes.push_back(h);
    }
  }
  F->tb_pol = have_p;
  std::vector<Box> two, rim;
  if (l2) {
    tb_regions(G, L2, holes, two, rim);
  } else {
    rim.push_back(G);
  }
  if (have_p) {  // rim boxes minus P
    std::vector<Box> keep;
    for (const Box &b : rim) {
      if (!box_meets(b, P)) {
        keep.push_back(b);
        continue;
      }
      std::vector<Box> part, inside;
      tb_regions(b, b, {P}, part, inside);
      keep.insert(keep.end(), part.begin(), part.end());
    }
    rim.swap(keep);
  }
  if (two.empty() && F->nranks == 1) return 0;
  // ---- rim items: tile-kernel shapes (columns <= 64 from 128-byte boundaries, rows <= 14,
  // chunks <= zc cut at the lean box's z range), bodies as make_tile_boxes
  // planes per rim item: its own setting (tuned with pairs), else the one-step chunk length
  const int zc = F->rim_zchunk > 0 ? std::min(F->rim_zchunk, FUSED_MAXCH)
                 : F->fused_zchunk > 0 ? std::min(F->fused_zchunk, FUSED_MAXCH) : 24;
  struct RI {
    int code, g0, g1, g2, g3, planes;
    bool dep;  // multi-rank: reads the ghost plane 0 or the top plane N-1 (slab-face data)
  };
  const bool lower = F->rank > 0, upper = F->rank + 1 < F->nranks;
  const int N2 = g.N[2];
  std::vector<std::array<int, 3>> spts;  // D source points (local indices)
  for (long long idx : F->srcD_idx) {
    const long long i2 = idx / g.st[2], r = idx % g.st[2];
    spts.push_back({(int)(r % g.st[1]), (int)(r / g.st[1]), (int)i2});
  }
  std::vector<RI> heavy, lean;
  F->rim_cells = F->rim_lean = 0;
  F->tb_nnarrow = 0;
  // a column box (x fixed, rows / planes inclusive) of two-step points
  auto col_two = [&](int x, int ylo, int yhi, int zlo, int zhi) {
    if (!l2 || x < L2.lo[0] || x > L2.hi[0] || ylo < L2.lo[1] || yhi > L2.hi[1] || zlo < L2.lo[2] ||
        zhi > L2.hi[2])
      return false;
    Box c;
    c.lo[0] = c.hi[0] = x, c.lo[1] = ylo, c.hi[1] = yhi, c.lo[2] = zlo, c.hi[2] = zhi;
    for (const Box &h : holes)
      if (box_meets(c, h)) return false;
    return true;
  };
  for (const Box &b : rim) {
    if (b.lo[0] % 16) {  // cannot happen with the alignments above
      if (F->tb_stats) fprintf(stderr, "tb: rim box at x %d not 128-byte aligned\n", b.lo[0]);
      return 0;
    }
    std::vector<int> xs, zs;
    split_range(xs, b.lo[0], b.hi[0] + 1, FX_HOST, 16);
    xs.push_back(b.hi[0] + 1);
    // a 16-column x-face box whose x-1 column is outside the grid or two-step: narrow strips
    const bool narrow = F->tb_narrow && b.hi[0] - b.lo[0] + 1 == SW_HOST &&
                        (b.lo[0] == 0 || col_two(b.lo[0] - 1, b.lo[1], b.hi[1], b.lo[2], b.hi[2]));
    std::vector<int> zcut = {b.lo[2], b.hi[2] + 1};
    // cuts at the lean box's z range (lean bodies for the planes inside it), unless a piece
    // would be thinner than 4 planes (the ring between L and L2: a 1-2-plane item costs more
    // per cell as a lean item than inside its PML neighbour); slab-face cuts always
    for (int v : {L.lo[2] + 1, L.hi[2]})
      if (v - b.lo[2] >= 4 && b.hi[2] + 1 - v >= 4) zcut.push_back(v);
    for (int v : {lower ? 2 : -1, upper ? N2 - 2 : -1})
      if (v > b.lo[2] && v < b.hi[2] + 1) zcut.push_back(v);
    std::sort(zcut.begin(), zcut.end());
    zcut.erase(std::unique(zcut.begin(), zcut.end()), zcut.end());
    std::sort(zcut.begin(), zcut.end());
    // narrow strips: their own planes per item (tb_szc; one strip pair per workgroup, so the
    // strips of a 512^3 rim make only ~200 workgroups at the rim's chunk length)
    const int zcb = narrow && F->tb_szc > 0 ? std::min(F->tb_szc, FUSED_MAXCH) : zc;
    for (size_t s = 0; s + 1 < zcut.size(); s++) {
      const int n = zcut[s + 1] - zcut[s], nt = (n + zcb - 1) / zcb;
      for (int t = 0; t < nt; t++) zs.push_back(zcut[s] + (int)((long long)n * t / nt));
    }
    zs.push_back(b.hi[2] + 1);
    if (narrow) {
      const int ny = b.hi[1] - b.lo[1] + 1, nty = (ny + SOWN_HOST - 1) / SOWN_HOST;
      std::vector<RI> items;
      bool ok = true;
      for (size_t iz = 0; iz + 1 < zs.size() && ok; iz++)
        for (int ty = 0; ty < nty && ok; ty++) {
          const int x0 = b.lo[0], x1 = b.hi[0];
          const int yf = b.lo[1] + (int)((long long)ny * ty / nty);
          const int y1 = b.lo[1] + (int)((long long)ny * (ty + 1) / nty) - 1;
          const int z0 = zs[iz], z1 = zs[iz + 1];
          const int code = strip_item_code(F, a, x0, x1, yf - 1, y1, z0, z1);
          if (code < 0) {
            ok = false;
            break;
          }
          bool src_in = false;
          if (F->nranks > 1)
            for (const auto &sp : spts)
              src_in = src_in || (sp[0] >= x0 - 1 && sp[0] <= x1 + 1 && sp[1] >= yf - 1 &&
                                  sp[1] <= y1 + 1 && sp[2] >= z0 - 1 && sp[2] <= z1);
          items.push_back(RI{code, x0 | (x1 << 16), yf | (y1 << 16), z0 | (z1 << 16), -1, z1 - z0,
                             (lower && z0 <= 1) || (upper && z1 >= N2 - 1) || src_in});
        }
      if (ok) {
        for (const RI &it : items) {
          heavy.push_back(it);
          F->rim_cells += double(SW_HOST) * (((it.g1 >> 16) - (it.g1 & 0xFFFF)) + 1) * it.planes;
        }
        F->tb_nnarrow += (int)items.size();
        continue;
      }
    }
    const int ny = b.hi[1] - b.lo[1] + 1, nty = (ny + FOWN_HOST - 1) / FOWN_HOST;
    for (size_t iz = 0; iz + 1 < zs.size(); iz++)
      for (int ty = 0; ty < nty; ty++)
        for (size_t ix = 0; ix + 1 < xs.size(); ix++) {
          const int x0 = xs[ix], x1 = xs[ix + 1] - 1;
          const int yf = b.lo[1] + (int)((long long)ny * ty / nty);
          const int y1 = b.lo[1] + (int)((long long)ny * (ty + 1) / nty) - 1;
          const int z0 = zs[iz], z1 = zs[iz + 1];
          bool in_l;
          const int code = tile_item_code(F, a, L, x0, x1, yf - 1, y1, z0, z1, &in_l);
          const double cells = double(x1 - x0 + 1) * (y1 - yf + 1) * (z1 - z0);
          F->rim_cells += cells;
          if (in_l) F->rim_lean += cells;
          // multi-rank: the sources are applied after the top plane's step (slab-face
          // chain), so items holding a source point wait for it too
          bool src_in = false;  // in the footprint (E = chi1inv * D of a neighbour)
          if (F->nranks > 1)
            for (const auto &sp : spts)
              src_in = src_in || (sp[0] >= x0 - 1 && sp[0] <= x1 + 1 && sp[1] >= yf - 1 &&
                                  sp[1] <= y1 + 1 && sp[2] >= z0 - 1 && sp[2] <= z1);
          RI it{code, x0 | (x1 << 16), yf | (y1 << 16), z0 | (z1 << 16), -1, z1 - z0,
                (lower && z0 <= 1) || (upper && z1 >= N2 - 1) || src_in};
          (((code >> 24) & 7) ? heavy : lean).push_back(it);
        }
  }
  // x-face strips of at most 32 columns (the rim left and right of L2) with the same rows,
  // planes and body (AX = 1) share one workgroup in pairs (pml_body<PAIR>): a narrow item
  // costs about a whole tile's time per plane (one dependent round per plane)
  if (!F->tb_nopair) {
    std::vector<RI> keep;
    std::vector<size_t> open;  // unpaired strips, by (rows, planes, code)
    for (const RI &it : heavy) {
      const int w = (it.g0 >> 16) - (it.g0 & 0xFFFF) + 1;
      if (((it.code >> 24) & 7) != 1 || w > 32 || ((it.code >> 30) & 1)) {
        keep.push_back(it);
        continue;
      }
      bool done = false;
      for (size_t k = 0; k < open.size() && !done; k++) {
        RI &o = keep[open[k]];
        if (o.g1 == it.g1 && o.g2 == it.g2 && o.code == it.code && o.dep == it.dep) {
          o.g3 = it.g0;
          open.erase(open.begin() + (long)k);
          done = true;
        }
      }
      if (!done) {
        open.push_back(keep.size());
        keep.push_back(it);
      }
    }
    heavy.swap(keep);
  }
  // longest first; a narrow strip plane costs ~1.3 wide-tile planes (item clock, round 5)
  auto longest_first = [](std::vector<RI> &v) {
    auto cost = [](const RI &r) { return r.planes * (((r.code >> 30) & 1) ? 1.3 : 1.0); };
    std::stable_sort(v.begin(), v.end(), [&](const RI &x, const RI &y) { return cost(x) > cost(y); });
  };
  longest_first(heavy);
  longest_first(lean);
  // items that need no slab-face data first (multi-rank: they run before the face exchange)
  std::vector<RI> order;
  for (int dep = 0; dep < 2; dep++)
    for (auto *v : {&heavy, &lean})
      for (const RI &it : *v)
        if (it.dep == (dep == 1)) order.push_back(it);
  // one rank: the narrow strips (they read the two-step kernel's output) last, so that R1's
  // other items can run beside the two-step kernel (tb_pair, tb_r1a).  The second rim launch
  // reads a second copy of the list after the first: the same order by default (measured
  // faster than longest first, tb_r2lpt: 512^3 -0.8 %, C2 256^3 -3.6 %)
  std::vector<RI> order2 = order;
  if (F->tb_r2lpt == 2)  // the narrow strips first
    std::stable_partition(order2.begin(), order2.end(),
                          [](const RI &r) { return ((r.code >> 30) & 1) != 0; });
  F->tb_rs0 = (int)order.size();
  if (F->nranks == 1) {
    auto strip = [](const RI &r) { return ((r.code >> 30) & 1) != 0; };
    std::stable_partition(order.begin(), order.end(), [&](const RI &r) { return !strip(r); });
    F->tb_rs0 = 0;
    for (const RI &it : order) F->tb_rs0 += strip(it) ? 0 : 1;
  }
  F->tb_rfree = 0;
  for (const RI &it : order) F->tb_rfree += it.dep ? 0 : 1;
  const std::vector<RI> *lists[2] = {&order, (F->nranks == 1 && F->tb_r2lpt) ? &order2 : &order};
  for (const std::vector<RI> *v : lists)
    for (const RI &it : *v) {
      F->tb_ritems.push_back(it.code);
      F->tb_rgeo.push_back(it.g0), F->tb_rgeo.push_back(it.g1), F->tb_rgeo.push_back(it.g2);
      F->tb_rgeo.push_back(it.g3);
    }
  // ---- two-step items: up to 124 x 12 own points (128 x 16 columns of lanes, two per lane),
  // z chunks of tz planes (automatic: the length whose item count fills whole rounds of one
  // workgroup per CU best, with the three halo planes of a chunk as overhead)
  // own columns of the two-step items: x0 .. x1 with lane 0's first column lx = x0 - 2 (x0 - 3
  // when x0 is odd: lane loads are 16-byte aligned), x1 <= lx + 125 and at most tb_ox columns
  // (0: TB_OXW = 124); widths of a box are whole pieces of that width plus the remainder
  // (tb_px = 1, the round-5 kernel for A/B: 60 own columns, lane 0 at x0 - 2, 64 lanes)
  const int px = F->tb_px;
  const int oxw = F->tb_ox ? F->tb_ox : (px == 1 ? 60 : TB_OXW);
  auto lane0 = [px](int x0) { return px == 1 ? x0 - 2 : (x0 & 1) ? x0 - 3 : x0 - 2; };
  auto next_x1 = [&](int x0, int hi) {
    return std::min(std::min(lane0(x0) + TB_LX * px - 3, x0 + oxw - 1), hi);
  };
  auto box_items_x = [&](const Box &b) {
    int n = 0;
    for (int x = b.lo[0]; x <= b.hi[0]; x = next_x1(x, b.hi[0]) + 1) n++;
    return n;
  };
  int tz = F->tb_zchunk;
  if (tz <= 0) {
    const long long cus = std::max(1, k_cu_count());
    double best = -1;
    for (int cand : {32, 40, 48, 56, 64, 80, 96, 128}) {
      long long items = 0, chunks = 0, planes = 0;
      for (const Box &b : two) {
        const long long ntx = box_items_x(b);
        const long long nty = (b.hi[1] - b.lo[1] + TB_OY) / TB_OY;
        const long long nz = b.hi[2] - b.lo[2] + 1, nch = (nz + cand - 1) / cand;
        items += ntx * nty * nch;
        chunks += nch;
        planes += nz;
      }
      const double fill = double(items) / double(((items + cus - 1) / cus) * cus);
      const double per = double(planes) / double(std::max(chunks, 1LL));
      const double score = fill * per / (per + 3.0);
      if (score > best + 1e-12) best = score, tz = cand;
    }
  }
  F->tb_cells = F->tb_border = 0;
  // z pieces of a column of items: balanced chunks of <= tz planes.  (Long pieces over most
  // of a column with short ones queued last, to save most pieces' three halo planes, measured
  // no faster in-process: 2.2685 vs 2.2693 ms/step at 512^3, round 5 -- not kept.)
  auto zpieces = [&](int z0, int nz) {
    std::vector<std::pair<int, int>> v;  // [lo, hi] inclusive
    const int nch = (nz + tz - 1) / tz;
    for (int ch = 0; ch < nch; ch++)
      v.push_back({z0 + (int)((long long)nz * ch / nch), z0 + (int)((long long)nz * (ch + 1) / nch) - 1});
    return v;
  };
  std::vector<TB2Item> items;
  for (const Box &b : two) {
    const int ny = b.hi[1] - b.lo[1] + 1, nty = (ny + TB_OY - 1) / TB_OY;
    const int nz = b.hi[2] - b.lo[2] + 1;
    for (const auto &zp : zpieces(b.lo[2], nz))
      for (int ty = 0; ty < nty; ty++)
        for (int x0 = b.lo[0]; x0 <= b.hi[0];) {
          const int lx = lane0(x0);
          Box o;
          o.lo[0] = x0;
          o.hi[0] = next_x1(x0, b.hi[0]);
          x0 = o.hi[0] + 1;
          o.lo[1] = b.lo[1] + (int)((long long)ny * ty / nty);
          o.hi[1] = b.lo[1] + (int)((long long)ny * (ty + 1) / nty) - 1;
          o.lo[2] = zp.first;
          o.hi[2] = zp.second;
          // faces bordering the rim: the layer outside the face, widened by 1 along the other
          // axes (points of an edge / corner see diagonal neighbours), meets a rim box
          int faces = 0;
          double nb = 0;
          for (int f = 0; f < 6; f++) {
            const int ax = f / 2;
            Box s = o;
            for (int k = 0; k < 3; k++)
              if (k != ax) s.lo[k]--, s.hi[k]++;
            s.lo[ax] = s.hi[ax] = (f & 1) ? o.hi[ax] + 1 : o.lo[ax] - 1;
            bool m = false;
            for (const Box &r : rim) m = m || box_meets(s, r);
            if (m) {
              faces |= 1 << f;
              double fc = 1;
              for (int k = 0; k < 3; k++)
                if (k != ax) fc *= o.hi[k] - o.lo[k] + 1;
              nb += fc;
            }
          }
          TB2Item it;
          it.x = o.lo[0] | (o.hi[0] << 16);
          it.y = o.lo[1] | (o.hi[1] << 16);
          it.z = o.lo[2] | ((o.hi[2] + 1) << 16);
          it.faces = faces;
          it.bx = it.by = it.bz = -1, it.lx = lx;
          {
            // the first compact DFT box the own points meet goes to the kernel's compact
            // stores; other compact boxes the item meets take the middle-set stores below
            std::vector<Box> ibox = dbox;
            int cm = -1;
            for (size_t m = 0; m < F->tb_cmp.size(); m++) {
              const TBCmp &c = F->tb_cmp[m];
              bool meet = true;
              Box cb;
              for (int k = 0; k < 3; k++) {
                cb.lo[k] = c.lo[k], cb.hi[k] = c.lo[k] + c.n[k] - 1;
                meet = meet && std::max(o.lo[k], cb.lo[k]) <= std::min(o.hi[k], cb.hi[k]);
              }
              if (!meet) continue;
              if (cm < 0)
                cm = (int)m;
              else
                ibox.push_back(cb);
            }
            if (cm >= 0) it.faces |= (cm + 1) << 8;
            Box u;  // bounding box of the item's intersections with the DFT boxes
            bool any = false;
            for (const Box &db : ibox) {
              Box x;
              bool ok = true;
              for (int k = 0; k < 3; k++) {
                x.lo[k] = std::max(o.lo[k], db.lo[k]);
                x.hi[k] = std::min(o.hi[k], db.hi[k]);
                ok = ok && x.lo[k] <= x.hi[k];
              }
              if (!ok) continue;
              for (int k = 0; k < 3; k++) {
                u.lo[k] = any ? std::min(u.lo[k], x.lo[k]) : x.lo[k];
                u.hi[k] = any ? std::max(u.hi[k], x.hi[k]) : x.hi[k];
              }
              any = true;
            }
            if (any) {
              it.bx = u.lo[0] | (u.hi[0] << 16);
              it.by = u.lo[1] | (u.hi[1] << 16);
              it.bz = u.lo[2] | (u.hi[2] << 16);
              double nb2 = 1;
              for (int k = 0; k < 3; k++) nb2 *= u.hi[k] - u.lo[k] + 1;
              nb += nb2;
            }
          }
          items.push_back(it);
          F->tb_cells += double(o.hi[0] - o.lo[0] + 1) * (o.hi[1] - o.lo[1] + 1) *
                         (o.hi[2] - o.lo[2] + 1);
          F->tb_border += nb;  // an upper bound (edges counted twice)
        }
  }
  // the work queue takes the items in list order: longest first.  One rank: the items whose
  // two-step footprint (own box + 2) meets no rim box first -- they read only what the previous
  // pair's two-step kernel wrote, so they can run beside that pair's second rim launch
  // (tb_pair, tb_lint) -- then the others
  auto interior = [&](const TB2Item &it) {
    Box o;
    o.lo[0] = (it.x & 0xFFFF) - 2, o.hi[0] = (it.x >> 16) + 2;
    o.lo[1] = (it.y & 0xFFFF) - 2, o.hi[1] = (it.y >> 16) + 2;
    o.lo[2] = (it.z & 0xFFFF) - 2, o.hi[2] = (it.z >> 16) + 1;
    for (const Box &r : rim)
      if (box_meets(o, r)) return false;
    return (it.faces & 63) == 0;
  };
  std::stable_sort(items.begin(), items.end(), [](const TB2Item &p, const TB2Item &q) {
    return (p.z >> 16) - (p.z & 0xFFFF) > (q.z >> 16) - (q.z & 0xFFFF);
  });
  F->tb_nint = 0;
  if (F->nranks == 1) {
    for (const TB2Item &it : items) F->tb_nint += interior(it) ? 1 : 0;
    if (F->tb_lint) std::stable_partition(items.begin(), items.end(), interior);
  }
  F->tb_items = items;
  // ---- upload, palette-uniform flags, mixed-palette cell counts (traffic model)
  if (dev_upload(F, &F->d_tb_ritems, F->tb_rcap, F->tb_ritems) ||
      dev_upload(F, &F->d_tb_rgeo, F->tb_gcap, F->tb_rgeo) ||
      dev_upload(F, &F->d_tb_items, F->tb_icap, F->tb_items))
    return -1;
  const int nr = (int)F->tb_ritems.size() / 2, ni = (int)F->tb_items.size();  // two copies
  if (F->d_tb_rflag) (void)hipFree(F->d_tb_rflag);
  if (F->d_tb_uflag) (void)hipFree(F->d_tb_uflag);
  F->d_tb_rflag = F->d_tb_uflag = nullptr;
  F->rim_cells_nu = F->rim_cells;
  F->tb_cells_nu = F->tb_cells;
  if (F->d_uidx) {
    HIPCHK(hipMalloc(&F->d_tb_rflag, std::max(2 * nr, 1) * sizeof(unsigned)));
    HIPCHK(hipMalloc(&F->d_tb_uflag, std::max(ni, 1) * sizeof(unsigned)));
    FusedArgs fa = fused_args(F);  // strides / palette of the current arrays
    if (k_tile_items_uniform(fa, F->d_tb_ritems, F->d_tb_rgeo, 2 * nr, F->d_tb_rflag, F->stream))
      return fail("rim palette flags failed");
    TB2Args t{};
    t.n = ni, t.items = F->d_tb_items, t.uidx = F->d_uidx;
    for (int k = 0; k < 3; k++) t.N[k] = g.N[k];
    t.st1 = g.st[1], t.st2 = g.st[2];
    if (k_tb2_uniform(t, F->d_tb_uflag, F->stream)) return fail("two-step palette flags failed");
    std::vector<unsigned> hr(nr), hi(ni);
    if (nr) HIPCHK(hipMemcpyAsync(hr.data(), F->d_tb_rflag, nr * 4, hipMemcpyDeviceToHost, F->stream));
    if (ni) HIPCHK(hipMemcpyAsync(hi.data(), F->d_tb_uflag, ni * 4, hipMemcpyDeviceToHost, F->stream));
    HIPCHK(hipStreamSynchronize(F->stream));
    F->rim_cells_nu = F->tb_cells_nu = 0;
    for (int i = 0; i < nr; i++)
      if (hr[i] == ~0u) {
        const int *q = &F->tb_rgeo[4 * i];
        const int wx = (q[0] >> 16) - (q[0] & 0xFFFF) + 1 +
                       (q[3] >= 0 ? (q[3] >> 16) - (q[3] & 0xFFFF) + 1 : 0);
        F->rim_cells_nu += double(wx) * ((q[1] >> 16) - (q[1] & 0xFFFF) + 1) *
                           ((q[2] >> 16) - (q[2] & 0xFFFF));
      }
    for (int i = 0; i < ni; i++)
      if (hi[i] == ~0u) {
        const TB2Item &q = F->tb_items[i];
        F->tb_cells_nu += double((q.x >> 16) - (q.x & 0xFFFF) + 1) *
                          ((q.y >> 16) - (q.y & 0xFFFF) + 1) * ((q.z >> 16) - (q.z & 0xFFFF));
      }
  }
  HIPCHK(hipStreamSynchronize(F->stream));
  F->tb_have = ni > 0 || (F->nranks > 1 && nr > 0);
  if (F->tb_stats)
    fprintf(stderr, "tb: L2 [%d..%d]x[%d..%d]x[%d..%d], %zu holes, %zu two-step boxes, %zu rim "
            "boxes; %d two-step items (%d planes, %.0f cells, %.0f border), %d rim items "
            "(%.0f cells, %.0f lean, %d narrow strips)\n",
            L2.lo[0], L2.hi[0], L2.lo[1], L2.hi[1], L2.lo[2], L2.hi[2], holes.size(), two.size(),
            rim.size(), ni, tz, F->tb_cells, F->tb_border, nr, F->rim_cells, F->rim_lean,
            F->tb_nnarrow);
  return 0;
}

// The middle buffer set of the pairs (the arrays the fused step ping-pongs: B, D, stored E,
// separate H, f_u of B).  Allocated on the first pair; when device memory is short, whatever
// this call allocated is freed again and temporal blocking is switched off on this rank (the
// ranks agree in tb_usable), so a grid that fits with two sets keeps stepping one step at a
// time instead of failing.  MNL_TB_OOM=1 simulates the failure (tests).
int tb_mid_alloc(mnl_fields *F) {
  DevFields &f = F->f;
  std::vector<double **> got;
  bool bad = false;
  auto one = [&](double **pp, double *cur) {
    if (!cur || *pp || bad) return;
    void *q = nullptr;
    if (F->tb_oom_test || hipMalloc(&q, F->nlocal * 8) != hipSuccess) {
      bad = true;
      (void)hipGetLastError();
      return;
    }
    *pp = (double *)q;
    got.push_back(pp);
  };
  for (int d = 0; d < 3; d++) {
    one(&F->pp3_B[d], f.B[d]);
    one(&F->pp3_D[d], f.D[d]);
    one(&F->pp3_E[d], f.E[d]);
    one(&F->pp3_H[d], f.H[d]);
    one(&F->pp3_UB[d], f.UB[d]);
  }
  if (!bad) {
    for (double **pp : got) F->dev_allocs.push_back(*pp);
    return 0;
  }
  for (double **pp : got) {
    (void)hipFree(*pp);
    *pp = nullptr;
  }
  (void)hipGetLastError();
  F->tb_enabled = false;
  F->tb_oom = true;
  if (g_verbosity > 0 && F->rank == 0)
    fprintf(stderr, "meep_nl_amd: not enough device memory for the temporal-blocking buffer set; "
                    "stepping one step at a time\n");
  return 1;
}

// Can the batch step in pairs?  Builds the plan when needed (-1: HIP error).
int tb_usable(mnl_fields *F, bool *ok) {
  *ok = false;
  // (no chi(2) NR box or upstream nonlinearity: the pairs have no E phase of their own.
  // Polarization chunks (tile mode: the general items are exactly those chunks) step one step
  // at a time in the general kernel beside each rim launch, on one rank (round 6, DESIGN.md
  // section 27); L2 keeps a distance of 2 from them)
  const bool pol_ok = F->f.npol > 0 && F->fgeo.ngen > 0 && F->nranks == 1 && F->tb_pol_on;
  bool local = F->tb_enabled && F->fused && F->tile_mode &&
               ((F->fgeo.ngen == 0 && F->f.npol == 0) || pol_ok) && !F->nr && !F->upnl &&
               F->S.dim == 3 && F->slab_dir == 2;
  if (local && tb_plan(F)) return -1;
  if (local && F->tb_have && tb_mid_alloc(F)) local = false;
  if (F->tb_stats && !(local && F->tb_have))
    fprintf(stderr, "tb: no pairs (enabled %d fused %d tile %d ngen %d dim %d slab %d dfts %zu have %d)\n",
            (int)F->tb_enabled, (int)F->fused, (int)F->tile_mode, F->fgeo.ngen, F->S.dim,
            F->slab_dir, F->dfts.size(), (int)F->tb_have);
  local = local && F->tb_have;
  if (F->nranks > 1) {  // every rank or none (their exchange sequences differ by mode)
    double v = local ? 1.0 : 0.0;
    if (F->comm->allreduce_sum(&v, 1, F->stream)) return fail("allreduce failed");
    local = v == double(F->nranks);
  }
  *ok = local;
  return 0;
}

// one buffer set of the fused step's per-point state (B, D, stored E, separate H, f_u of B)
struct Set5 {
  double *B[3], *D[3], *E[3], *H[3], *UB[3];
};
Set5 set_cur(mnl_fields *F) {
  Set5 s;
  for (int d = 0; d < 3; d++)
    s.B[d] = F->f.B[d], s.D[d] = F->f.D[d], s.E[d] = F->f.E[d], s.H[d] = F->f.H[d],
    s.UB[d] = F->f.UB[d];
  return s;
}
Set5 set_nxt(mnl_fields *F) {
  Set5 s;
  for (int d = 0; d < 3; d++)
    s.B[d] = F->f.Bn[d], s.D[d] = F->f.Dn[d], s.E[d] = F->f.E[d] ? F->f.En[d] : nullptr,
    s.H[d] = F->f.H[d] ? F->f.Hn[d] : nullptr, s.UB[d] = F->f.UB[d] ? F->f.UBn[d] : nullptr;
  return s;
}
Set5 set_mid(mnl_fields *F) {
  Set5 s;
  for (int d = 0; d < 3; d++)
    s.B[d] = F->pp3_B[d], s.D[d] = F->pp3_D[d], s.E[d] = F->f.E[d] ? F->pp3_E[d] : nullptr,
    s.H[d] = F->f.H[d] ? F->pp3_H[d] : nullptr, s.UB[d] = F->f.UB[d] ? F->pp3_UB[d] : nullptr;
  return s;
}

// tile-kernel arguments of a rim launch: one step from set `o` to set `n`, the rim item list
FusedArgs rim_args(mnl_fields *F, const FusedArgs &fa, const Set5 &o, const Set5 &n) {
  FusedArgs r = fa;
  for (int d = 0; d < 3; d++) {
    r.Bo[d] = o.B[d], r.Do[d] = o.D[d], r.E[d] = o.E[d], r.Ho[d] = o.H[d], r.UBo[d] = o.UB[d];
    r.Bn[d] = n.B[d], r.Dn[d] = n.D[d], r.En[d] = n.E[d], r.Hn[d] = n.H[d], r.UBn[d] = n.UB[d];
  }
  r.titems = F->d_tb_ritems;
  r.tgeo = F->d_tb_rgeo;
  r.tflag = F->d_uidx ? F->d_tb_rflag : nullptr;
  r.gbeg = 0, r.gend = (int)F->tb_ritems.size() / 2;
  r.clk.kind = 1;
  return r;
}

// general-kernel arguments of the polarization chunks in a pair: one step from `o` to `n`
// (P / P_prev and the f_u of D in place, as in one-step stepping)
FusedArgs gen_args(const FusedArgs &fa, const Set5 &o, const Set5 &n) {
  FusedArgs r = fa;
  for (int d = 0; d < 3; d++) {
    r.Bo[d] = o.B[d], r.Do[d] = o.D[d], r.E[d] = o.E[d], r.Ho[d] = o.H[d], r.UBo[d] = o.UB[d];
    r.Bn[d] = n.B[d], r.Dn[d] = n.D[d], r.En[d] = n.E[d], r.Hn[d] = n.H[d], r.UBn[d] = n.UB[d];
  }
  r.wg_limit = 0;
  r.lean_after = 0;
  return r;
}

// two-step arguments: state n in `o`, border step n+1 into `m`, step n+2 into `n`
TB2Args tb_args(mnl_fields *F, const Set5 &o, const Set5 &m, const Set5 &n) {
  const DevGrid &g = F->g;
  TB2Args t{};
  t.n = (int)F->tb_items.size();
  t.items = F->d_tb_items;
  t.uflag = F->d_uidx ? F->d_tb_uflag : nullptr;
  for (int d = 0; d < 3; d++) {
    t.Bo[d] = o.B[d], t.Do[d] = o.D[d];
    t.Bm[d] = m.B[d], t.Dm[d] = m.D[d];
    t.Bn[d] = n.B[d], t.Dn[d] = n.D[d];
    t.u[d] = F->f.inveps[d];
    t.N[d] = g.N[d];
  }
  t.uidx = F->d_uidx;
  t.utab = F->d_utab;
  t.st1 = g.st[1], t.st2 = g.st[2];
  t.nelem = (long long)F->nlocal;
  t.C = F->S.courant;
  t.ctr = F->d_fused_ctr;
  t.ctr_line = 3;
  t.clk = ItemClock{F->d_clk, F->d_clk_n, F->d_clk ? CLK_CAP : 0u, 2};
  t.ncmp = (int)F->tb_cmp.size();
  for (int i = 0; i < t.ncmp; i++) t.cmp[i] = F->tb_cmp[i];
  t.px = F->tb_px;
  return t;
}

int tb_src(mnl_fields *F, const SrcDev &s, double *const D[3]) {
  if (!s.n) return 0;
  DevFields fm = F->f;
  for (int d = 0; d < 3; d++) fm.Dn[d] = D[d];
  if (k_source(T_D, F->g, fm, s, 0, F->stream)) return fail("source launch failed");
  return 0;
}

// A pair's step tail on one rank: the step's D sources into D, then (when due) the NaN guard of
// the state E / D at time step `at` -- one launch (k_src_guard) for short source lists, else
// the two launches as before (tb_srcguard = 0: always two)
int tb_tail(mnl_fields *F, const SrcDev &s, double *const D[3], double *const E[3], long long at) {
  nan_count(F, 1);
  F->nan_at = at;
  if (F->tb_srcguard && F->nan_due && F->nan_terms.n > 0 && s.n <= SRC_GUARD_MAXN &&
      s.nlayer <= SRC_GUARD_MAXL) {
    if (!F->d_nanflag && dev_alloc(F, &F->d_nanflag, 2)) return -1;
    DevFields fm = F->f;
    const double *Ec[3], *Dc[3], *U[3];
    for (int d = 0; d < 3; d++) fm.Dn[d] = D[d], Ec[d] = E[d], Dc[d] = D[d], U[d] = F->f.inveps[d];
    const int r = k_src_guard(fm, s, F->nan_terms, Ec, Dc, U, F->d_nanflag, (int)F->nan_at,
                              F->stream);
    if (r == 0) {
      F->nan_due = false;
      F->nan_launched++;
      return 0;
    }
    if (r != 2) return fail("source / guard launch failed");
  }
  if (tb_src(F, s, D)) return -1;
  return nan_launch(F, nullptr, E, D);
}

// the middle set starts as a copy of the state (entries no launch writes: walls, ghosts);
// its arrays exist (tb_mid_alloc ran in tb_usable)
int tb_mid_init(mnl_fields *F) {
  if (F->tb_mid_fresh) return 0;
  DevFields &f = F->f;
  auto fresh = [&](double **pp, double *cur) -> int {
    if (!cur) return 0;
    if (!*pp) return fail("temporal blocking: middle buffer set missing");
    HIPCHK(hipMemcpyAsync(*pp, cur, F->nlocal * 8, hipMemcpyDeviceToDevice, F->stream));
    return 0;
  };
  for (int d = 0; d < 3; d++)
    if (fresh(&F->pp3_B[d], f.B[d]) || fresh(&F->pp3_D[d], f.D[d]) || fresh(&F->pp3_E[d], f.E[d]) ||
        fresh(&F->pp3_H[d], f.H[d]) || fresh(&F->pp3_UB[d], f.UB[d]))
      return -1;
  F->tb_mid_fresh = true;
  return 0;
}

void swap_cur_nxt(DevFields &f) {
  for (int d = 0; d < 3; d++) {
    std::swap(f.B[d], f.Bn[d]);
    std::swap(f.D[d], f.Dn[d]);
    std::swap(f.E[d], f.En[d]);
    std::swap(f.H[d], f.Hn[d]);
    std::swap(f.UB[d], f.UBn[d]);
  }
}

// Steps n, n+1 (sources s0, s1) as three launches: L = the two-step
// kernel (cur -> nxt for the L2 points, their border values of step n+1 -> mid), R1 = the
// tile kernel over the rim items (cur -> mid), source(n) into mid, R2 = the rim items again
// (mid -> nxt), source(n+1) into nxt.  L runs first: the narrow x-face strips of R1 / R2 read
// the new B of their x-1 column (two-step points) from mid / nxt.  Every launch reads one set
// and writes disjoint points of others.
template <class EB, class EE>
int tb_pair(mnl_fields *F, const SrcDev &s0, const SrcDev &s1, EB &ev_begin, EE &ev_end,
            long long t_mid) {
  if (tb_mid_init(F)) return -1;
  const FusedArgs &fa = fused_args(F);
  const Set5 cur = set_cur(F), mid = set_mid(F), nxt = set_nxt(F);
  TB2Args t = tb_args(F, cur, mid, nxt);
  const int nr = (int)F->tb_ritems.size() / 2;  // R1's order, then R2's (tb_plan)
  FusedArgs r1 = rim_args(F, fa, cur, mid), r2 = rim_args(F, fa, mid, nxt);
  {  // CUs left free by the two-step launch / the rim launches (A/B; the multi-rank default)
    const int rl = F->res_l >= 0 ? F->res_l : F->tb_res, rr = F->res_r >= 0 ? F->res_r : F->tb_res;
    if (rl > 0) t.wg_limit = std::max(1, k_cu_count() - rl);
    if (rr > 0) r1.wg_limit = r2.wg_limit = std::max(1, k_cu_count() - rr);
  }
  // R1's items other than the narrow strips read only cur and write rim points of mid: they
  // run on a side stream beside L, taking the CUs L's workgroups leave at the end of its queue
  // (the strips read L's border values of mid and follow L).  One timing span covers L and R1
  const int na = F->tb_r1a && !F->tb_pol ? std::min(F->tb_rs0, nr) : 0;
  // the two-step items whose footprint meets no rim box (tb_plan puts them first) read only
  // what the previous pair's two-step kernel wrote and write the buffers its rim launches no
  // longer read after its first rim launch: they run on a third stream, released at that point
  // of the previous pair (ev_r1done), beside its second rim launch.  Not with DFT monitors
  // (their samples of the previous pair read the compact boxes these items rewrite)
  const int ni = t.n;
  const int nl = (F->tb_lint && F->dfts.empty() && !F->tb_pol) ? std::min(F->tb_nint, ni) : 0;
  // (the stream-ordering events below release at device scope: every reader is on this device)
  if ((na > 0 || nl > 0) && !F->s_aux) {
    HIPCHK(hipStreamCreateWithFlags(&F->s_aux, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&F->ev_start, hipEventDisableTiming | hipEventReleaseToDevice));
    HIPCHK(hipEventCreateWithFlags(&F->ev_early, hipEventDisableTiming | hipEventReleaseToDevice));
  }
  if (nl > 0 && !F->s_lint) {
    HIPCHK(hipStreamCreateWithFlags(&F->s_lint, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&F->ev_lint, hipEventDisableTiming | hipEventReleaseToDevice));
    HIPCHK(hipEventCreateWithFlags(&F->ev_r1done, hipEventDisableTiming | hipEventReleaseToDevice));
  }
  if (nl > 0) {
    if (!F->tb_r1done_ok || F->tb_lint == 2)  // no previous pair in this batch: after all before
      HIPCHK(hipEventRecord(F->ev_r1done, F->stream));
    HIPCHK(hipStreamWaitEvent(F->s_lint, F->ev_r1done, 0));
    TB2Args ti = t;
    ti.n = nl;
    ti.ctr_line = 6;
    if (F->tb_lint >= 3) ti.wg_limit = std::max(1, k_cu_count() * F->tb_lint / 8);
    const int kl = k_tb2(ti, F->s_lint, F->ctr_base);
    if (kl) return fused_fail("two-step kernel launch failed", kl);
    HIPCHK(hipEventRecord(F->ev_lint, F->s_lint));
    t.n = ni - nl;
    t.items = t.items + nl;
    if (t.uflag) t.uflag = t.uflag + nl;
  }
  int k = ev_begin(TM_TB);
  int kr = 0;
  if (na > 0) {
    HIPCHK(hipEventRecord(F->ev_start, F->stream));
    HIPCHK(hipStreamWaitEvent(F->s_aux, F->ev_start, 0));
  }
  kr = t.n > 0 ? k_tb2(t, F->stream, F->ctr_base) : 0;
  if (kr) return fused_fail("two-step kernel launch failed", kr);
  if (na > 0) {
    kr = k_tile_items(r1, r1.titems, r1.tgeo, r1.tflag, na, 5, F->s_aux, F->ctr_base);
    if (kr) return fused_fail("rim kernel launch failed", kr);
    HIPCHK(hipEventRecord(F->ev_early, F->s_aux));
    if (nr > na) {
      kr = k_tile_items(r1, r1.titems + na, r1.tgeo + 4 * na, r1.tflag ? r1.tflag + na : nullptr,
                        nr - na, 4, F->stream, F->ctr_base);
      if (kr) return fused_fail("rim kernel launch failed", kr);
    }
    HIPCHK(hipStreamWaitEvent(F->stream, F->ev_early, 0));
    if (nl > 0) HIPCHK(hipStreamWaitEvent(F->stream, F->ev_lint, 0));
    ev_end(k);
  } else {
    if (nl > 0) HIPCHK(hipStreamWaitEvent(F->stream, F->ev_lint, 0));
    ev_end(k);
    k = ev_begin(TM_RIM);
    kr = k_tile_items(r1, r1.titems, r1.tgeo, r1.tflag, nr, 4, F->stream, F->ctr_base);
    ev_end(k);
    if (kr) return fused_fail("rim kernel launch failed", kr);
  }
  if (F->tb_pol) {  // the polarization chunks' step n (before the sources of the step)
    k = ev_begin(TM_GEN);
    kr = k_fused(gen_args(fa, cur, mid), 1, F->stream, F->ctr_base);
    ev_end(k);
    if (kr) return fused_fail("fused general kernel launch failed", kr);
  }
  // the step's sources, then the guard of the middle step (its terms' points hold step n+1 in
  // mid: rim items, or the two-step items' store box)
  if (tb_tail(F, s0, mid.D, mid.E, t_mid)) return -1;
  // the next pair's interior two-step items may start from here: R1, every two-step item of
  // this pair and the middle step's guard are done, and what follows (R2, source(n+1), the guard
  // of nxt) reads only points of mid within one cell of the rim and nxt, which those items
  // neither write nor, beyond the rim's reach, read
  F->tb_r1done_ok = false;
  if (nl > 0) {
    HIPCHK(hipEventRecord(F->ev_r1done, F->stream));
    F->tb_r1done_ok = true;
  }
  if (dft_due(F, t_mid)) {  // fields::update_dfts after the pair's first step, from mid
    DevFields fm = F->f;
    for (int d = 0; d < 3; d++)
      fm.B[d] = mid.B[d], fm.D[d] = mid.D[d], fm.E[d] = mid.E[d], fm.H[d] = mid.H[d];
    k = ev_begin(TM_DFT);
    const int r = dft_update(F, t_mid, &fm, 0);
    ev_end(k);
    if (r) return -1;
  }
  k = ev_begin(TM_RIM);
  kr = k_tile_items(r2, r2.titems + nr, r2.tgeo + 4 * nr, r2.tflag ? r2.tflag + nr : nullptr, nr,
                    4, F->stream, F->ctr_base);
  ev_end(k);
  if (kr) return fused_fail("rim kernel launch failed", kr);
  if (F->tb_pol) {
    k = ev_begin(TM_GEN);
    kr = k_fused(gen_args(fa, mid, nxt), 1, F->stream, F->ctr_base);
    ev_end(k);
    if (kr) return fused_fail("fused general kernel launch failed", kr);
  }
  if (tb_tail(F, s1, nxt.D, nxt.E, t_mid + 1)) return -1;
  swap_cur_nxt(F->f);
  return 0;
}

// Multi-rank pair (one rank of a z-slab decomposition; fused, no D source on the top
// plane).  L2 lies >= 2 planes from the slab faces, so only the rim meets them:
//   main: L (cur -> nxt, border -> mid) on all CUs but RES (the previous pair's slab-face
//         chain still runs on s_comm), then, once the E ghost of step n is in (ev_x0), R1
//         (rim, cur -> mid);
//   s_comm: B/H plane exchange of mid, the top plane's step n (shell kernels, old = cur,
//         new = mid), source(n), E plane exchange of mid (ev_x0);
//   main: R2 over the rim items that read no slab-face data and hold no source point
//         (beside that chain), then the others once it is done;
//   s_comm: the same chain for nxt -- beside the next pair's L.
// Every kernel reads and writes disjoint points of its sets.

template <class EB, class EE>
int tb_face_chain(mnl_fields *F, const Set5 &o, const Set5 &n, const SrcDev &src,
                  hipEvent_t after, EB &ev_begin, EE &ev_end) {
  DevFields &f = F->f;
  const DevGrid &g = F->g;
  HIPCHK(hipStreamWaitEvent(F->s_comm, after, 0));
  const int kc = ev_begin(TM_CHAIN, F->s_comm);
  // exchanges and shell kernels read F->f's pointers when enqueued: point them at the sets
  const DevFields keep = f;
  for (int d = 0; d < 3; d++) {
    f.B[d] = o.B[d], f.D[d] = o.D[d], f.E[d] = o.E[d], f.H[d] = o.H[d], f.UB[d] = o.UB[d];
    f.Bn[d] = n.B[d], f.Dn[d] = n.D[d], f.En[d] = o.E[d] ? n.E[d] : nullptr;
    f.Hn[d] = o.H[d] ? n.H[d] : nullptr, f.UBn[d] = o.UB[d] ? n.UB[d] : nullptr;
  }
  int r = exchange(F, 1, F->s_comm) ? fail("H halo exchange failed") : 0;
  const BoxList *sl = &F->fused_shell;
  if (!r && k_curl(T_B, F->interior, sl, g, f, F->planB, F->S.courant, F->s_comm, true))
    r = fail("curl B launch failed");
  // the sources of the step (every D point: after the top plane's curl D, as the one-step
  // path applies them after all of D); with one on the top plane E follows the source there
  const bool fuseE = !F->dsrc_in_shell;
  if (!r && k_curl(T_D, F->interior, sl, g, f, F->planD, F->S.courant, F->s_comm, fuseE))
    r = fail("curl D launch failed");
  if (!r && src.n && k_source(T_D, g, f, src, 0, F->s_comm)) r = fail("source launch failed");
  if (!r && !fuseE) {
    ISrcDev is{};
    if (k_update_e(F->interior, sl, g, f, is, 0, true, F->s_comm)) r = fail("update E launch failed");
  }
  if (!r) {  // the E plane of the new set goes up
    for (int d = 0; d < 3; d++) f.E[d] = n.E[d];
    if (exchange(F, 0, F->s_comm)) r = fail("E halo exchange failed");
  }
  const DevFields fresh = f;
  f = keep;
  (void)fresh;
  if (r) return r;
  ev_end(kc, F->s_comm);
  HIPCHK(hipEventRecord(F->ev_x0, F->s_comm));
  return 0;
}

template <class EB, class EE>
int tb_pair_multi(mnl_fields *F, const SrcDev &s0, const SrcDev &s1, EB &ev_begin, EE &ev_end,
                  long long t_mid) {
  if (tb_mid_init(F)) return -1;
  const FusedArgs &fa = fused_args(F);
  const Set5 cur = set_cur(F), mid = set_mid(F), nxt = set_nxt(F);
  TB2Args t = tb_args(F, cur, mid, nxt);
  const int cus = k_cu_count();
  const int res = F->tb_res >= 0 ? F->tb_res : TB_RES_CUS;
  t.wg_limit = res > 0 ? cus - res : 0;
  const int nr = (int)F->tb_ritems.size() / 2, nf = F->tb_rfree;
  int k = ev_begin(TM_TB);
  int kr = k_tb2(t, F->stream, F->ctr_base);
  ev_end(k);
  if (kr) return fused_fail("two-step kernel launch failed", kr);
  // R1 once the E ghost (and top plane) of step n are in
  k = ev_begin(TM_WAIT);
  HIPCHK(hipStreamWaitEvent(F->stream, F->ev_x0, 0));
  ev_end(k);
  FusedArgs r1 = rim_args(F, fa, cur, mid);
  k = ev_begin(TM_RIM);
  kr = k_tile_items(r1, r1.titems, r1.tgeo, r1.tflag, nr, 4, F->stream, F->ctr_base);
  ev_end(k);
  if (kr) return fused_fail("rim kernel launch failed", kr);
  HIPCHK(hipEventRecord(F->ev_early, F->stream));
  if (tb_face_chain(F, cur, mid, s0, F->ev_early, ev_begin, ev_end)) return -1;
  nan_count(F, 1);  // the middle step's guard, after its top plane and sources (s_comm)
  F->nan_at = t_mid;
  if (nan_launch(F, F->s_comm, mid.E, mid.D)) return -1;
  // R2: the items without slab-face reads beside the chain, then the others
  FusedArgs r2 = rim_args(F, fa, mid, nxt);
  r2.wg_limit = res > 0 ? cus - res : 0;
  k = ev_begin(TM_RIM);
  kr = k_tile_items(r2, r2.titems, r2.tgeo, r2.tflag, nf, 4, F->stream, F->ctr_base);
  ev_end(k);
  if (!kr) {
    const int kw = ev_begin(TM_WAIT);
    HIPCHK(hipStreamWaitEvent(F->stream, F->ev_x0, 0));
    ev_end(kw);
    if (dft_due(F, t_mid)) {
      // fields::update_dfts after the pair's first step, from mid (round 6): the chain has
      // put mid's top plane, sources and E ghost in; the H component normal to the slabs gets
      // its low ghost now (exchange kind 3, as post_step does after a one-step step).  The
      // exchange reads F->f's pointers when enqueued: point them at mid meanwhile
      DevFields &f = F->f;
      const DevFields keep = f;
      for (int d = 0; d < 3; d++)
        f.B[d] = mid.B[d], f.D[d] = mid.D[d], f.E[d] = mid.E[d], f.H[d] = mid.H[d],
        f.UB[d] = mid.UB[d];
      const DevFields fm = f;
      k = ev_begin(TM_DFT);
      int r = exchange(F, 3) ? fail("DFT halo exchange failed") : 0;
      f = keep;
      if (!r) r = dft_update(F, t_mid, &fm, 0);
      ev_end(k);
      if (r) return -1;
    }
    k = ev_begin(TM_RIM);
    r2.wg_limit = 0;
    kr = k_tile_items(r2, r2.titems + nf, r2.tgeo + 4 * nf, r2.tflag ? r2.tflag + nf : nullptr,
                      nr - nf, 4, F->stream, F->ctr_base);
  }
  ev_end(k);
  if (kr) return fused_fail("rim kernel launch failed", kr);
  HIPCHK(hipEventRecord(F->ev_early, F->stream));
  if (tb_face_chain(F, mid, nxt, s1, F->ev_early, ev_begin, ev_end)) return -1;
  swap_cur_nxt(F->f);
  F->tb_chain_pending = true;  // a one-step step next waits for it (tb_chain_join)
  nan_count(F, 1);
  F->nan_at = t_mid + 1;
  return nan_launch(F, F->s_comm);  // after the chain: the top plane of the new state
}

// Before a one-step step after a multi-rank pair: the pair's last slab-face chain (top plane,
// sources, E ghost) ran on s_comm; the one-step kernels on the main stream read its results.
// diagnostics: append this batch's item records (rank-tagged binary, CLK_REC u64 each,
// preceded per batch by {magic, rank, count}) to clk_path and reset the counter
int clk_dump(mnl_fields *F) {
  unsigned n = 0;
  HIPCHK(hipMemcpy(&n, F->d_clk_n, sizeof n, hipMemcpyDeviceToHost));
  n = std::min(n, CLK_CAP);
  std::vector<unsigned long long> h((size_t)n * CLK_REC);
  if (n) HIPCHK(hipMemcpy(h.data(), F->d_clk, h.size() * 8, hipMemcpyDeviceToHost));
  HIPCHK(hipMemset(F->d_clk_n, 0, sizeof(unsigned)));
  FILE *fp = fopen(F->clk_path.c_str(), "ab");
  if (!fp) return fail("MNL_ITEM_CLOCK: cannot open " + F->clk_path);
  const unsigned long long hd[CLK_REC] = {0x4b4c434d4e4dull, (unsigned long long)F->rank, n, 0, 0, 0, 0, 0};
  fwrite(hd, 8, CLK_REC, fp);
  if (n) fwrite(h.data(), 8, h.size(), fp);
  fclose(fp);
  return 0;
}

int tb_chain_join(mnl_fields *F) {
  if (!F->tb_chain_pending) return 0;
  F->tb_chain_pending = false;
  HIPCHK(hipStreamWaitEvent(F->stream, F->ev_x0, 0));
  return 0;
}

int step_batch(mnl_fields *F, int nsteps) {
  if (F->src_dirty && build_source_lists(F)) return -1;
  if (set_fused(F, fused_agreed(F))) return -1;
  {  // does a D source point lie in the shell (outside the box the interior kernels own)?
    const Box &ib = F->fused ? F->fusedG : F->interior;
    F->dsrc_in_shell = false;
    for (long long idx : F->srcD_idx) {
      const long long i2 = idx / F->g.st[2], r = idx % F->g.st[2];
      const long long i1 = r / F->g.st[1], i0 = r % F->g.st[1];
      const long long ii[3] = {i0, i1, i2};
      bool in = true;
      for (int a = 0; a < 3; a++) in = in && ii[a] >= ib.lo[a] && ii[a] <= ib.hi[a];
      if (!in) F->dsrc_in_shell = true;
    }
  }
  if (F->fused && F->nranks > 1 && multi_begin(F)) return -1;
  if (nan_terms_build(F)) return -1;  // NaN guard terms of this batch's mode / arrays
  bool tb_ok = false;  // step in pairs (temporal blocking; its plan stores the guard's points)
  if (nsteps >= 2 && tb_usable(F, &tb_ok)) return -1;
  if (nsteps >= 2) F->tb_last = tb_ok;
  const double dt = F->dt;
  // per-step source values, computed on the host exactly as the reference
  size_t nB = F->srcB_idx.size(), nD = F->srcD_idx.size(), nI = F->isrc_idx.size();
  // per step: the current of every group at time (B) and time + dt/2 (D), complex,
  // then the integrated dipoles real(amp * dipole(time + dt)) per point
  const size_t ng = F->groups.size();
  size_t per = (nB || nD ? 4 * ng : 0) + nI;
  const size_t jofs = (nB || nD) ? 4 * ng : 0;
  const int CH = NAN_CH;  // steps per source table / NaN flag read
  std::vector<EvPair> evs;
  size_t evi = 0;
  // timing events only (read after a stream synchronize): no system-scope fence when one is
  // recorded -- with it every record wrote back / invalidated the caches between the kernels,
  // 0.4 % of a 512^3 step and 2.6 % of a 256^3 one (round 6; MNL_EV_FENCE=1 restores it)
  const unsigned ev_flags = F->ev_fence ? hipEventDefault : hipEventDisableSystemFence;
  // timing events of a phase on the main stream (or st)
  auto ev_begin = [&](int cat, hipStream_t st = nullptr) -> int {
    if (!F->profiling) return -1;
    while (F->ev_pool.size() < 2 * (evi + 1)) {
      hipEvent_t e;
      if (hipEventCreateWithFlags(&e, ev_flags) != hipSuccess) return -1;
      F->ev_pool.push_back(e);
    }
    EvPair p{F->ev_pool[2 * evi], F->ev_pool[2 * evi + 1], cat};
    hipEventRecord(p.a, st ? st : F->stream);
    evs.push_back(p);
    evi++;
    return (int)evs.size() - 1;
  };
  auto ev_end = [&](int k, hipStream_t st = nullptr) {
    if (k >= 0) hipEventRecord(evs[k].b, st ? st : F->stream);
  };
  // a phase that starts where phase k ended: its start is k's end event (one
  // record fewer between two back-to-back kernels)
  auto ev_next = [&](int k, int cat) -> int {
    if (!F->profiling || k < 0) return ev_begin(cat);
    while (F->ev_pool.size() < 2 * (evi + 1)) {
      hipEvent_t e;
      if (hipEventCreateWithFlags(&e, ev_flags) != hipSuccess) return -1;
      F->ev_pool.push_back(e);
    }
    EvPair p{evs[k].b, F->ev_pool[2 * evi + 1], cat};
    evs.push_back(p);
    evi++;
    return (int)evs.size() - 1;
  };
  auto flush_events = [&]() -> int {
    if (!F->profiling || evs.empty()) return 0;
    HIPCHK(hipStreamSynchronize(F->stream));
    if (F->s_comm) HIPCHK(hipStreamSynchronize(F->s_comm));
    for (auto &p : evs) {
      float ms = 0;
      hipEventElapsedTime(&ms, p.a, p.b);
      F->timer_ms[p.cat] += ms;
      F->timer_count[p.cat] += 1;
    }
    evs.clear();
    evi = 0;
    return 0;
  };
  // fields::update_dfts after t += 1 (src/step.cpp:125-127); a rank's averages
  // read its low ghost planes, which must hold this step's values first
  auto post_step = [&](int s, int cstate = -1) -> int {
    const long long tn = F->t + s + 1;
    if (!dft_due(F, tn)) return 0;
    if (F->nranks > 1) {
      if (F->fused)
        HIPCHK(hipStreamWaitEvent(F->stream, F->ev_x0, 0));
      else if (exchange(F, 0))
        return fail("E halo exchange failed");
      if (exchange(F, 3)) return fail("DFT halo exchange failed");
    }
    const int k = ev_begin(TM_DFT);
    const int r = dft_update(F, tn, nullptr, cstate);
    ev_end(k);
    return r;
  };
  F->tb_r1done_ok = false;  // the batch's first pair waits for everything before it
  for (int s0 = 0; s0 < nsteps; s0 += CH) {
    int ns = std::min(CH, nsteps - s0);
    if (!F->dfts.empty() && dft_prepare(F, F->t, ns)) return -1;
    if (per) {
      std::vector<double> vals((size_t)ns * per);
      for (int s = 0; s < ns; s++) {
        long long tt = F->t + s;
        double time = tt * dt;
        double *vB = &vals[(size_t)s * per], *vD = vB + 2 * ng, *vI = vB + jofs;
        for (auto &st : F->srcs) st.update(time, dt);  // calc_sources(time())
        if (jofs)
          for (size_t g = 0; g < ng; g++) {
            const cplx J = F->srcs[F->groups[g].st].cur_current;
            vB[2 * g] = real(J), vB[2 * g + 1] = imag(J);
          }
        for (auto &st : F->srcs) st.update(time + 0.5 * dt, dt);
        if (jofs)
          for (size_t g = 0; g < ng; g++) {
            const cplx J = F->srcs[F->groups[g].st].cur_current;
            vD[2 * g] = real(J), vD[2 * g + 1] = imag(J);
          }
        for (auto &st : F->srcs) st.update(time + dt, dt);
        for (size_t k = 0; k < nI; k++) {
          const SrcGroup &G = F->groups[F->isrc_ref[k].first];
          const cplx A = G.amp[F->isrc_ref[k].second] * F->srcs[G.st].cur_dipole;
          vI[k] = real(A);
        }
      }
      size_t bytes = vals.size() * sizeof(double);
      if (F->d_vals_cap < vals.size()) {
        HIPCHK(hipStreamSynchronize(F->stream));
        if (F->d_vals) hipFree(F->d_vals);
        HIPCHK(hipMalloc(&F->d_vals, bytes));
        F->d_vals_cap = vals.size();
      }
      HIPCHK(hipMemcpyAsync(F->d_vals, vals.data(), bytes, hipMemcpyHostToDevice, F->stream));
      HIPCHK(hipStreamSynchronize(F->stream));  // vals is a host temporary
    }
    for (int s = 0; s < ns; s++) {
      DevFields &f = F->f;
      const DevGrid &g = F->g;
      f.nr_t = F->t + s;  // seeds of the NR random fallback (nr_voxel_seed)
      const double *vs = F->d_vals + (size_t)s * per;  // this step's table
      const SrcDev sB = src_dev(F, 0, vs), sD = src_dev(F, 1, vs + 2 * ng);
      ISrcDev is = F->isrc_dev;
      is.n = (int)nI;
      is.val = vs + jofs;  // kernels index val[step * n + orig] with step 0
      if (tb_ok && s + 1 < ns) {  // steps s and s + 1 as one pair (no DFT)
        const SrcDev sD1 = src_dev(F, 1, vs + per + 2 * ng);
        if ((F->nranks > 1 ? tb_pair_multi(F, sD, sD1, ev_begin, ev_end, F->t + s + 1)
                           : tb_pair(F, sD, sD1, ev_begin, ev_end, F->t + s + 1)))
          return -1;
        s++;
        if (post_step(s, 1)) return -1;  // DFT of the pair's second step (the new state)
        continue;
      }
      F->tb_r1done_ok = false;  // a one-step step: the next pair waits for everything before
      if (tb_chain_join(F)) return -1;
      if (F->fused && F->nranks > 1) {
        if (step_fused_multi(F, sD, ev_begin, ev_end) || post_step(s)) return -1;
        nan_count(F, 1);
        F->nan_at = F->t + s + 1;
        if (nan_launch(F)) return -1;
        continue;
      }
      // ---- B: halo of E (low ghost), curl, sources
      if (!F->u_first_done[0] && u_lazy_copy(F, 0)) return -1;
      if (F->nranks > 1) {
        int k = ev_begin(TM_HALO);
        if (exchange(F, 0)) return fail("E halo exchange failed");
        ev_end(k);
      }
      const BoxList *sl = F->fused ? &F->fused_shell : &F->shell_list;
      int k = ev_begin(TM_BINT);
      bool nr_done = false;  // the NR box's E phase already launched (beside the tile kernel)
      if (F->fused) {
        FusedArgs &fa = fused_args(F);
        const int split = F->tile_mode ? 0 : gen_split(F);
        int kr;
        if (split > 0) {
          // general tiles on `split` CUs of a side stream, lean tiles on the others,
          // concurrently (disjoint points, old buffers read-only)
          if (!F->s_aux) {
            HIPCHK(hipStreamCreateWithFlags(&F->s_aux, hipStreamNonBlocking));
            HIPCHK(hipEventCreateWithFlags(&F->ev_start, hipEventDisableTiming | hipEventReleaseToDevice));
            HIPCHK(hipEventCreateWithFlags(&F->ev_early, hipEventDisableTiming | hipEventReleaseToDevice));
          }
          HIPCHK(hipEventRecord(F->ev_start, F->stream));
          HIPCHK(hipStreamWaitEvent(F->s_aux, F->ev_start, 0));
          fa.wg_limit = split;
          kr = k_fused(fa, 1, F->s_aux, F->ctr_base);
          if (kr) return fused_fail("fused general kernel launch failed", kr);
          HIPCHK(hipEventRecord(F->ev_early, F->s_aux));
          fa.wg_limit = k_cu_count() - split;
          kr = k_fused(fa, 0, F->stream, F->ctr_base);
          fa.wg_limit = 0;
          if (kr) return fused_fail("fused kernel launch failed", kr);
          HIPCHK(hipStreamWaitEvent(F->stream, F->ev_early, 0));
          F->fused_concurrent = true;
        } else if (const int ts = F->tile_mode && fa.ngen > 0 ? tile_gen_split(F) : 0) {
          // tile mode: the polarization chunks' general items on `ts` CUs of a side
          // stream beside the tile kernel on the others (both read only the old buffers
          // and write the ping-pong partners: no ordering between them)
          if (!F->s_aux) {
            HIPCHK(hipStreamCreateWithFlags(&F->s_aux, hipStreamNonBlocking));
            HIPCHK(hipEventCreateWithFlags(&F->ev_start, hipEventDisableTiming | hipEventReleaseToDevice));
            HIPCHK(hipEventCreateWithFlags(&F->ev_early, hipEventDisableTiming | hipEventReleaseToDevice));
          }
          HIPCHK(hipEventRecord(F->ev_start, F->stream));
          HIPCHK(hipStreamWaitEvent(F->s_aux, F->ev_start, 0));
          fa.wg_limit = ts;
          kr = k_fused(fa, 1, F->s_aux, F->ctr_base);
          if (kr) return fused_fail("fused general kernel launch failed", kr);
          if (F->nr && F->nranks == 1 && nr_early_ok(F)) {
            const int ke = ev_begin(TM_E, F->s_aux);
            if (nr_fused_e(F, is, F->s_aux)) return -1;
            ev_end(ke, F->s_aux);
            nr_done = true;
          }
          HIPCHK(hipEventRecord(F->ev_early, F->s_aux));
          fa.wg_limit = k_cu_count() - ts;
          kr = k_fused(fa, 4, F->stream, F->ctr_base);
          fa.wg_limit = 0;
          if (kr) return fused_fail("fused kernel launch failed", kr);
          HIPCHK(hipStreamWaitEvent(F->stream, F->ev_early, 0));
          F->fused_concurrent = true;
        } else {
          F->fused_concurrent = false;
          kr = k_fused(fa, F->tile_mode ? 4 : 0, F->stream, F->ctr_base);
          if (kr) return fused_fail("fused kernel launch failed", kr);
          if (!F->tile_mode || fa.ngen > 0) {
            ev_end(k);
            k = ev_next(k, TM_GEN);
            // lean mode: same stream, after the lean launch (tile mode: the general
            // items are polarization chunks, whose halos no lean launch stores)
            fa.lean_after = F->tile_mode ? 0 : lean_halo_reads(F);
            kr = k_fused(fa, 1, F->stream, F->ctr_base);
            fa.lean_after = 0;
            if (kr) return fused_fail("fused general kernel launch failed", kr);
          }
        }
      } else if (k_curl(T_B, F->interior, nullptr, g, f, F->planB, F->S.courant, F->stream)) {
        return fail("curl B launch failed");
      }
      ev_end(k);
      // shell curl B; the PML H update rides along when no B source sits between
      // (timing events only around phases that launch something: an event record
      // between two kernels costs a few microseconds of GPU time)
      const bool fuseH = nB == 0 && !F->first_step_mode && !F->hall;
      const bool shell_work = sl->n > 0 && sl->start[sl->n] > 0;
      k = shell_work ? ev_begin(TM_B) : -1;
      if (k_curl(T_B, F->interior, sl, g, f, F->planB, F->S.courant, F->stream, fuseH))
        return fail("curl B launch failed");
      ev_end(k);
      if (nB && k_source(T_B, g, f, sB, 0, F->stream)) return fail("source launch failed");
      // ---- H
      if (!F->h_first_done && h_lazy_copy(F)) return -1;
      bool anyH = F->hall;
      for (int d = 0; d < 3; d++) anyH = anyH || f.H[d];
      k = (!fuseH && anyH && (shell_work || F->hall)) ? ev_begin(TM_H) : -1;
      if (!fuseH && update_h_any(F, *sl, true)) return -1;
      ev_end(k);
      if (F->nranks > 1) {
        int kk = ev_begin(TM_HALO);
        if (exchange(F, 1)) return fail("H halo exchange failed");
        ev_end(kk);
      }
      // ---- D
      if (!F->u_first_done[1] && u_lazy_copy(F, 1)) return -1;
      k = !F->fused ? ev_begin(TM_DINT) : -1;
      if (!F->fused && k_curl(T_D, F->interior, nullptr, g, f, F->planD, F->S.courant, F->stream))
        return fail("curl D launch failed");
      ev_end(k);
      // shell curl D; the shell E update rides along when it only reads its own D
      const bool fuseE = !F->nr && !F->upnl && f.npol == 0 && nI == 0 && !F->dsrc_in_shell &&
                         !F->first_step_mode;
      k = shell_work ? ev_begin(TM_D) : -1;
      if (k_curl(T_D, F->interior, sl, g, f, F->planD, F->S.courant, F->stream, fuseE))
        return fail("curl D launch failed");
      ev_end(k);
      if (nD && k_source(T_D, g, f, sD, 0, F->stream)) return fail("source launch failed");
      if ((F->nr || F->upnl) && F->nranks > 1) {
        if (exchange(F, 2)) return fail("D halo exchange failed");
      }
      // ---- E (+ Lorentzian P)
      if (!F->e_first_done && e_lazy_copy(F)) return -1;
      if (F->fused && F->nr) {  // one rank: the fused kernels did all but the NR box
        if (!nr_done) {
          k = ev_begin(TM_E);
          if (nr_fused_e(F, is)) return -1;
          ev_end(k);
        }
      } else {
        // neighbour reads of D - P (NR, upstream chi) or of W (anisotropic sigma):
        // P after all of E
        bool fuse = !F->nr && !F->upnl && !f.aniso;
        k = (!F->fused || (!fuseE && shell_work) || (!fuse && f.npol) || f.aniso || f.wall_e)
                ? ev_begin(TM_E)
                : -1;
        if (nr_defer_begin(F)) return -1;
        if (!F->fused && F->nr && F->S.dim == 3) {
          if (nr_interior_e(F, is)) return -1;
        } else if (!F->fused && k_update_e(F->interior, nullptr, g, f, is, 0, fuse, F->stream)) {
          return fail("update E launch failed");
        }
        if (!fuseE) {
          // no chi2 outside the interior: the shell boxes never take the NR branch, so
          // they run the plain E kernel (same values, without the NR kernel's registers)
          DevFields plain = f;
          if (F->nr && F->nr_split_done && F->nr_shell_free) plain.nr_enabled = 0;
          if (k_update_e(F->interior, sl, g, plain, is, 0, fuse, F->stream))
            return fail("update E launch failed");
        }
        if (nr_defer_end(F)) return -1;
        if (f.aniso && !f.wall_e && k_aniso_wall(g, f, 0, F->stream))
          return fail("wall W launch failed");
        if (f.aniso && F->nranks > 1 && exchange(F, 4))  // WE_stuff ghosts (step.cpp:111-114)
          return fail("W halo exchange failed");
        if (!fuse && f.npol) {
          if (k_update_pols(F->interior, nullptr, g, f, F->stream) ||
              k_update_pols(F->interior, sl, g, f, F->stream))
            return fail("pols launch failed");
        }
        if ((f.aniso || f.wall_e) && k_aniso_wall(g, f, 1, F->stream))
          return fail("wall W launch failed");
        ev_end(k);
      }
      if (F->fused)
        for (int d = 0; d < 3; d++) {
          std::swap(f.B[d], f.Bn[d]);
          std::swap(f.D[d], f.Dn[d]);
          std::swap(f.E[d], f.En[d]);
          std::swap(f.H[d], f.Hn[d]);
          std::swap(f.UB[d], f.UBn[d]);
        }
      if (post_step(s)) return -1;
      nan_count(F, 1);
      F->nan_at = F->t + s + 1;
      if (nan_launch(F)) return -1;
    }
    // buffered DFT updates stay buffered across chunks and calls (a run that steps one step
    // per call accumulates once per kb updates, not once per call); readers flush first
    F->t += ns;
    if (flush_events() != 0) return -1;
    if (nan_result(F)) return -1;  // stop within NAN_CH steps of a failing guard
  }
  if (F->s_comm) {
    HIPCHK(hipStreamSynchronize(F->s_comm));
    HIPCHK(hipStreamSynchronize(F->s_aux));
  }
  F->tb_chain_pending = false;
  HIPCHK(hipStreamSynchronize(F->stream));
  HIPCHK(hipGetLastError());
  if (F->d_clk && clk_dump(F)) return -1;
  return nan_result(F);
}

// NaN guard (src/step.cpp:138-139): abort when get_field(D_EnergyDensity, gv.center()) is
// not finite (src/monitor.cpp:96-113: 1/2 sum_d real(conj(E_d) D_d), each value interpolated
// as get_field does, src/monitor.cpp:127-160).  The terms (this rank's points of the 8-point
// stencils, which array, weight) are built once per batch on the host; nan_check_kernel sums
// them on the device after the step, and the host reads the flag once, at the end of the
// batch (no round trip per step).  Multi-rank: each rank checks its share and the ranks agree.
int nan_terms_build(mnl_fields *F) {
  const mnl_structure &S = F->S;
  NanTerms &t = F->nan_terms;
  t.n = 0;
  double cen[3] = {0, 0, 0};
  for (int d = 0; d < 3; d++)
    if (S.has[d]) {
      int n = S.n[d] - (S.n[d] & 1);
      cen[d] = (S.io[d] + n) * (0.5 * (1.0 / S.a));
    }
  if (S.dim == 1) cen[0] = cen[1] = 0;
  if (S.dim == 2) cen[2] = 0;
  for (int d = 0; d < 3; d++) {
    if (!F->allocated[d] || !F->allocated[3 * T_D + d]) continue;
    for (int which = 0; which < 2; which++) {  // E_d terms, then D_d terms
      const int c = which == 0 ? d : 3 * T_D + d;
      int locs[8][3];
      double w[8];
      interpolate(S, c, cen, locs, w);
      for (int i = 0; i < 8 && w[i]; i++) {
        int jg[3] = {0, 0, 0};
        bool in = true;
        for (int e = 0; e < 3; e++)
          if (S.has[e]) {
            const int o = locs[i][e] - S.io[e];
            if (!(o > 0 && o <= 2 * S.n[e])) in = false;
            jg[e] = (locs[i][e] - S.io[e] - S.shift(c, e)) / 2;
          }
        if (!in) continue;
        const long long li = local_index(F, c, jg, true);
        if (li < 0) continue;
        if (t.n >= NAN_MAXT) return fail("NaN guard: too many terms");
        t.dir[t.n] = (unsigned char)d;
        t.kind[t.n] = which == 1 ? 2 : (in_fused_box(F, c, jg) ? 1 : 0);
        t.idx[t.n] = li;
        t.w[t.n] = w[i];
        t.n++;
      }
    }
  }
  return 0;
}

// launch the guard on the current state (or the given E / D arrays: the middle state of a
// pair) if one is due
int nan_launch(mnl_fields *F, hipStream_t st, double *const *Es, double *const *Ds) {
  if (!F->nan_due) return 0;
  F->nan_due = false;
  if (!st) st = F->stream;
  if (!F->d_nanflag && dev_alloc(F, &F->d_nanflag, 2)) return -1;  // zeroed; reset by nan_result
  const double *E[3], *D[3], *U[3];
  for (int d = 0; d < 3; d++)
    E[d] = Es ? Es[d] : F->f.E[d], D[d] = Ds ? Ds[d] : F->f.D[d], U[d] = F->f.inveps[d];
  if (k_nan_check(F->nan_terms, E, D, U, F->d_nanflag, (int)F->nan_at, st))
    return fail("NaN guard launch failed");
  F->nan_launched++;
  return 0;
}

// after k steps: count them, mark a guard due every nan_every steps (across calls)
void nan_count(mnl_fields *F, int k) {
  F->since_nan += k;
  if (F->since_nan >= F->nan_every) {
    F->since_nan = 0;
    F->nan_due = true;
  }
}

// end of a chunk of a batch: the reference's abort (src/step.cpp:138-139) if a guard saw NaN /
// Inf.  The message names the first failing step (the step after which the reference's check
// aborts); the time stays at the state the device holds -- the fields, the ping-pong buffers
// and the DFT accumulators have advanced past the failing step to the end of the chunk (at most
// NAN_CH steps), and t says so, so a caller that catches the error reads arrays labelled with
// their own time.  Multi-rank: every rank learns the earliest failing step of any rank.
int nan_result(mnl_fields *F) {
  if (F->nan_launched == 0) return 0;  // the same on every rank (same step counts)
  if (F->s_comm) HIPCHK(hipStreamSynchronize(F->s_comm));
  HIPCHK(hipStreamSynchronize(F->stream));
  int h[2] = {0, 0};
  HIPCHK(hipMemcpy(h, F->d_nanflag, sizeof h, hipMemcpyDeviceToHost));
  if (h[0]) HIPCHK(hipMemset(F->d_nanflag, 0, sizeof h));
  F->nan_launched = 0;
  long long bad_t = h[0] ? (long long)h[1] : -1;
  if (F->nranks > 1) {
    std::vector<double> v(F->nranks, 0.0);
    v[F->rank] = double(bad_t);
    if (F->comm->allreduce_sum(v.data(), F->nranks, F->stream)) return fail("allreduce failed");
    bad_t = -1;
    for (double x : v)
      if (x >= 0 && (bad_t < 0 || (long long)x < bad_t)) bad_t = (long long)x;
  }
  if (bad_t < 0) return 0;
  F->nan_bad_t = bad_t;
  return fail("simulation fields are NaN or Inf (at time step " + std::to_string(bad_t) +
              "; fields left at time step " + std::to_string(F->t) + ")");
}

int finalize_fields(mnl_fields *F) {
  if (build_pml_tables(F)) return -1;
  setup_grid(F);
  if (upload_pml(F)) return -1;
  if (setup_materials(F)) return -1;
  setup_boxes(F);
  make_shell_list(F);
  if (dev_alloc(F, &F->d_nr_fallbacks, 1)) return -1;
  F->f.nr_fallbacks = F->d_nr_fallbacks;
  if (F->nr) {  // first attempts that fail are finished in parallel by nr_hard_kernel
    if (dev_alloc(F, &F->d_nr_hard, NR_HARD_CAP) || dev_alloc(F, &F->d_nr_hard_cnt, 1)) return -1;
    F->f.nr_hard_cnt = F->d_nr_hard_cnt;
    F->f.nr_hard_cap = NR_HARD_CAP;
  }
  make_plans(F);
  return 0;
}

// (checkpoints, array slices and field energy: mnl_io.cpp)

int fields_step_batches(mnl_fields *F, int nsteps);

// fields::step (src/step.cpp:40-140) over nsteps: the time spent goes to the
// reference's time sinks (per-phase kernel times when profiling is on, the
// rest to "time stepping"), and rank 0 prints "on time step ..." at most every
// MEEP_MIN_OUTPUT_TIME (4 s, src/meep.hpp:48) when verbosity > 0.
int fields_step(mnl_fields *F, int nsteps) {
  const double w0 = wall_now();
  double ms0[TM_N];
  for (int k = 0; k < TM_N; k++) ms0[k] = F->timer_ms[k];
  if (F->t == 0 || F->last_out_wall < 0) F->last_out_wall = w0, F->last_out_t = F->t;
  const int r = fields_step_batches(F, nsteps);
  const double wall = wall_now() - w0;
  auto dsec = [&](int k) { return (F->timer_ms[k] - ms0[k]) * 1e-3; };
  double parts[MNL_NUM_TIME_SINKS] = {0};
  if (F->profiling) {
    parts[MNL_SINK_UPDATE_B] = dsec(TM_B) + (F->fused ? 0.0 : dsec(TM_BINT));
    parts[MNL_SINK_UPDATE_H] = dsec(TM_H);
    parts[MNL_SINK_UPDATE_D] = dsec(TM_D) + dsec(TM_DINT);
    parts[MNL_SINK_UPDATE_E] = dsec(TM_E);
    parts[MNL_SINK_BOUNDARIES] = dsec(TM_HALO);
    parts[MNL_SINK_FOURIER] = dsec(TM_DFT) + dsec(TM_DFTF);
  }
  double rest = wall;
  for (int k = 0; k < MNL_NUM_TIME_SINKS; k++) F->sink_s[k] += parts[k], rest -= parts[k];
  F->sink_s[MNL_SINK_STEPPING] += std::max(rest, 0.0);
  return r;
}

int fields_step_batches(mnl_fields *F, int nsteps) {
  while (nsteps > 0) {
    int m;
    if (!F->e_first_done || !F->h_first_done || !F->u_first_done[0] || !F->u_first_done[1] ||
        F->force_unfused_next) {
      const bool saved = F->allow_fused;
      F->allow_fused = false;
      F->first_step_mode = true;
      const int r = step_batch(F, 1);
      F->allow_fused = saved;
      F->first_step_mode = false;
      if (r) return -1;
      F->force_unfused_next = false;
      m = 1;
    } else {
      m = nsteps;  // the NaN guard runs on the device inside the batch (nan_launch)
      if (step_batch(F, m)) return -1;
    }
    nsteps -= m;
    if (g_verbosity > 0 && F->rank == 0) {
      const double now = wall_now();
      if (now > F->last_out_wall + 4.0 && F->t > F->last_out_t) {
        printf("on time step %lld (time=%g), %g s/step\n", F->t, F->t * F->dt,
               (now - F->last_out_wall) / double(F->t - F->last_out_t));
        fflush(stdout);
        F->last_out_wall = now;
        F->last_out_t = F->t;
      }
    }
  }
  return 0;
}

// fields::initialize_field(c, func) (src/initialize.cpp:135-148) with the
// function's values given as a whole-cell host array (canonical layout, real
// part): add, step_boundaries(type(c)); for D / B also update_eh(E / H) and
// step_boundaries of that type.  Integrated-source dipoles are not subtracted
// in that E update (DESIGN.md "initialize_field").
int initialize_field(mnl_fields *F, int c, const double *host) {
  if (require_component(F, c)) return -1;
  if (F->fused && set_fused(F, false)) return -1;
  const int t = ctype(c), d = cdir(c);
  DevFields &f = F->f;
  size_t nt = F->S.ntot;
  if (F->scratch_cap < nt) {
    HIPCHK(hipStreamSynchronize(F->stream));
    if (F->d_scratch) hipFree(F->d_scratch);
    F->d_scratch = nullptr;
    HIPCHK(hipMalloc(&F->d_scratch, nt * sizeof(double)));
    F->scratch_cap = nt;
  }
  HIPCHK(hipMemcpyAsync(F->d_scratch, host, nt * sizeof(double), hipMemcpyHostToDevice, F->stream));
  double *dst = nullptr, *alt = nullptr;
  switch (t) {
    case T_E: dst = f.E[d]; break;
    case T_D: dst = f.D[d]; break;
    case T_B: dst = f.B[d]; break;
    case T_H:  // H == B until the first H update separates it (PML chunks only)
      dst = f.B[d];
      if (F->h_first_done && f.H[d]) dst = f.H[d], alt = f.B[d];
      break;
  }
  if (!dst) return fail("initialize_field: component not allocated");
  if (k_init_add(dst, alt, F->d_scratch, F->g, f, t, d, F->stream))
    return fail("initialize_field kernel launch failed");
  if (F->nranks > 1) {
    const int kind = t == T_E ? 0 : t == T_D ? 2 : 1;
    if (exchange(F, kind)) return fail("initialize_field halo exchange failed");
  }
  ISrcDev is{};
  if (t == T_D) {  // update_eh(E_stuff); step_boundaries(E_stuff)
    if (!F->e_first_done && e_lazy_copy(F)) return -1;
    if (nr_defer_begin(F)) return -1;
    if (k_update_e(F->interior, nullptr, F->g, f, is, 0, false, F->stream) ||
        k_update_e(F->interior, &F->shell_list, F->g, f, is, 0, false, F->stream))
      return fail("update E launch failed");
    if (nr_defer_end(F)) return -1;
    if (f.wall_e && k_aniso_wall(F->g, f, 1, F->stream)) return fail("wall E launch failed");
    if (F->nranks > 1 && exchange(F, 0)) return fail("E halo exchange failed");
  } else if (t == T_B) {  // update_eh(H_stuff); step_boundaries(H_stuff)
    if (!F->h_first_done && h_lazy_copy(F)) return -1;
    if (update_h_any(F, F->shell_list, false)) return -1;  // update_eh(H_stuff) only
    if (F->nranks > 1 && exchange(F, 1)) return fail("H halo exchange failed");
  } else {
    F->force_unfused_next = true;  // E (or H) differs from what D (B) implies
  }
  HIPCHK(hipStreamSynchronize(F->stream));
  return 0;
}

mnl_fields *create_common(mnl_structure *s, int device, int rank, int nranks, const void *id,
                          LocalHub *hub = nullptr) {
  if (!s) {
    fail("null structure");
    return nullptr;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    fail("no HIP device available (the MI355X path has no CPU fallback)");
    return nullptr;
  }
  std::unique_ptr<mnl_fields> F(new mnl_fields());
  F->S = *s;
  F->dt = s->dt;
  if (device < 0) {
    if (hipGetDevice(&device) != hipSuccess) device = 0;
  }
  if (device >= ndev) {
    fail("device index out of range");
    return nullptr;
  }
  F->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&F->stream, hipStreamNonBlocking) != hipSuccess) {
    fail("cannot create HIP stream");
    return nullptr;
  }
  memset(&F->f, 0, sizeof(F->f));
  F->rank = rank;
  F->nranks = nranks;
  if (nranks > 1) {
    F->comm.reset(new Comm());
    if (hub ? F->comm->init_local(rank, nranks, hub) : F->comm->init(rank, nranks, id)) {
      fail(hub ? "local slab group init failed"
               : Comm::is_ipc_id(id) ? "IPC slab group init failed (shared-memory id)"
                                     : std::string("RCCL communicator init failed (") +
                                           comm_last_error() +
                                           "); MNL_COMM=ipc runs the same slabs over the "
                                           "IPC transport");
      return nullptr;
    }
  }
  if (const char *zc = getenv("MNL_FUSED_ZCHUNK")) {
    F->fused_zchunk = std::max(0, atoi(zc));
    F->fused_zchunk_env = true;  // the tuner keeps it
  }
  if (const char *bp = getenv("MNL_FUSED_BPC")) F->fused_bpc = std::max(1, atoi(bp));
  if (const char *tm = getenv("MNL_TILE")) F->tile_mode = atoi(tm) != 0;
  if (const char *tb = getenv("MNL_TB")) F->tb_enabled = atoi(tb) != 0, F->tb_env = true;
  if (const char *tz = getenv("MNL_TB_ZCHUNK"))
    F->tb_zchunk = std::max(0, atoi(tz)), F->tb_zchunk_env = true;
  if (const char *tn = getenv("MNL_TB_NARROW")) F->tb_narrow = atoi(tn) != 0;
  if (const char *tx = getenv("MNL_TB_PX")) F->tb_px = atoi(tx) == 1 ? 1 : 2;
  if (const char *tq = getenv("MNL_TB_POL")) F->tb_pol_on = atoi(tq) != 0;
  if (const char *ta = getenv("MNL_TB_R1A")) F->tb_r1a = atoi(ta) != 0;
  if (const char *tl = getenv("MNL_TB_LINT")) F->tb_lint = atoi(tl);
  if (const char *ef = getenv("MNL_EV_FENCE")) F->ev_fence = atoi(ef) != 0;
  if (const char *sg = getenv("MNL_TB_SRCGUARD")) F->tb_srcguard = atoi(sg) != 0;
  if (const char *sz = getenv("MNL_TB_STRIP_ZCHUNK")) F->tb_szc = std::max(0, atoi(sz));
  if (const char *tp = getenv("MNL_TB_R2LPT")) F->tb_r2lpt = std::max(0, std::min(2, atoi(tp)));
  if (const char *to = getenv("MNL_TB_OOM")) F->tb_oom_test = atoi(to) != 0;
  if (const char *dp = getenv("MNL_DFT_PAL")) F->dft_pal = atoi(dp) != 0;
  if (const char *dc = getenv("MNL_DFT_CMP")) F->dft_cmp = atoi(dc) != 0;
  if (const char *ne = getenv("MNL_NR_EARLY")) F->nr_early = atoi(ne) != 0;
  if (const char *tr = getenv("MNL_TB_RES")) F->tb_res = std::max(0, atoi(tr));
  if (const char *tp = getenv("MNL_TB_NOPAIR")) F->tb_nopair = atoi(tp) != 0;
  if (const char *bm = getenv("MNL_TILE_BODY_MASK")) F->tile_body_mask = atoi(bm);
  if (const char *fd = getenv("MNL_FUSED_DIST")) F->fused_dist = atoi(fd) == 2 ? 2 : 1;
  if (const char *nf = getenv("MNL_NO_FUSED")) F->allow_fused = atoi(nf) == 0;
  if (const char *ne = getenv("MNL_NAN_EVERY")) F->nan_every = std::max(1, atoi(ne));
  if (const char *gc = getenv("MNL_GEN_CUS")) F->gen_cus = std::max(0, atoi(gc));
  if (const char *sg = getenv("MNL_STAGGER")) F->stagger = std::max(0, atoi(sg)) / 128 * 128;
  if (const char *ar = getenv("MNL_ARENA")) F->arena_req = std::max(0, atoi(ar));
  if (const char *cg = getenv("MNL_CONTIG")) F->contig = atoi(cg) != 0;
  if (const char *ag = getenv("MNL_ARENA_GAP")) F->arena_gap = std::max(0, atoi(ag)) / 128 * 128;
  auto env_is = [](const char *name, char v) {
    const char *e = getenv(name);
    return e && e[0] == v;
  };
  F->ownc = !env_is("MNL_NO_OWNC", '1');
  F->tile_zcut = !env_is("MNL_ZCUT", '0');
  F->lean_halo = !env_is("MNL_LEAN_HALO", '0');
  F->no_palette = env_is("MNL_NO_PALETTE", '1');
  F->uniform = !env_is("MNL_UNIFORM", '0');
  F->lean_groups = env_is("MNL_LEAN_GROUPS", '8') ? 8 : 1;
  F->gen_groups = env_is("MNL_GEN_GROUPS", '8') ? 8 : 1;
  if (const char *e = getenv("MNL_TILE_GEN_CUS")) {
    F->tile_gen_cus = std::max(0, atoi(e));
    F->tile_gen_cus_env = true;
  }
  F->nr_defer = !env_is("MNL_NR_DEFER", '0');
  F->tile_stats = getenv("MNL_TILE_STATS") != nullptr;
  F->tb_stats = getenv("MNL_TB_STATS") != nullptr;
  if (const char *ck = getenv("MNL_ITEM_CLOCK")) F->clk_path = ck;
  if (finalize_fields(F.get())) return nullptr;
  if (!F->clk_path.empty() && (dev_alloc(F.get(), &F->d_clk, (size_t)CLK_CAP * CLK_REC) ||
                               dev_alloc(F.get(), &F->d_clk_n, 1)))
    return nullptr;
  return F.release();
}

int check_comp(int c) {
  if (c < 0 || c >= MNL_NUM_COMPONENTS) return fail("invalid component");
  return 0;
}

int add_source_any(mnl_fields *F, int comp, int kind, const double *p, int np, mnl_src_func func,
                   void *fdata, const double vmin[3], const double vmax[3], double amp_re,
                   double amp_im, int is_integrated, mnl_amp_func afunc, void *adata) {
  if (!F || check_comp(comp)) return -1;
  if (!(ctype(comp) == T_E || ctype(comp) == T_H)) return fail("sources must be E or H components");
  if (!has_field(F->S, comp)) return fail("component not present in this dimensionality");
  if (hipSetDevice(F->device) != hipSuccess) return fail("hipSetDevice failed");
  SrcTime st;
  if (kind == MNL_SRC_GAUSSIAN) {
    if (np < 4) return fail("gaussian source needs 4 parameters");
    // gaussian_src_time(f, w, st, et) (src/sources.cpp:85-96)
    st.kind = 0;
    st.freq = p[0];
    st.width = p[1];
    st.peak_time = 0.5 * (p[2] + p[3]);
    st.cutoff = (p[3] - p[2]) * 0.5;
    while (exp(-st.cutoff * st.cutoff / (2 * st.width * st.width)) < 1e-100) st.cutoff *= 0.9;
    st.cutoff = float(st.cutoff);
  } else if (kind == MNL_SRC_CONTINUOUS) {
    if (np < 6) return fail("continuous source needs 6 parameters");
    st.kind = 1;
    st.cfreq = cplx(p[0], p[1]);
    st.cwidth = p[2];
    st.start_time = float(p[3]);
    st.end_time = float(p[4]);
    st.slowness = p[5];
  } else if (kind == MNL_SRC_CUSTOM) {  // custom_src_time(func, data, st, et)
    st.kind = 2;
    st.func = func;
    st.fdata = fdata;
    st.start_time = float(p[0]);
    st.end_time = float(p[1]);
  } else
    return fail("unknown source kind");
  st.is_integrated = is_integrated != 0;
  int idx = -1;
  for (size_t i = 0; i < F->srcs.size(); i++)
    if (F->srcs[i].same(st)) idx = (int)i;
  if (idx < 0) {
    F->srcs.push_back(st);
    idx = (int)F->srcs.size() - 1;
  }
  if (require_component(F, comp)) return -1;
  double lo[3] = {vmin[0], vmin[1], vmin[2]}, hi[3] = {vmax[0], vmax[1], vmax[2]};
  if (F->S.dim == 1) lo[0] = lo[1] = hi[0] = hi[1] = 0;
  if (F->S.dim == 2) lo[2] = hi[2] = 0;
  return add_volume_source(F, comp, idx, lo, hi, cplx(amp_re, amp_im), afunc, adata);
}

}  // namespace

// =============================================================== C ABI
extern "C" {

const char *mnl_last_error(void) { return g_err.c_str(); }
int mnl_version(void) { return 100; }

int mnl_device_count(int *count) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *count = n;
  return 0;
}

mnl_structure *mnl_structure_create(int dim, const int n[3], double a, double courant,
                                    const int io[3]) {
  if (dim < 1 || dim > 3) {
    fail("dim must be 1, 2 or 3");
    return nullptr;
  }
  if (!(a > 0) || !(courant > 0)) {
    fail("resolution and Courant must be positive");
    return nullptr;
  }
  mnl_structure *s = new mnl_structure();
  s->dim = dim;
  s->has[0] = dim >= 2;
  s->has[1] = dim >= 2;
  s->has[2] = dim != 2;
  for (int d = 0; d < 3; d++) {
    s->n[d] = s->has[d] ? n[d] : 0;
    s->io[d] = s->has[d] ? io[d] : 0;
    if (s->has[d] && s->n[d] < 2) {
      delete s;
      fail("need at least 2 cells along every present direction");
      return nullptr;
    }
    for (int k = 0; k < 2; k++) s->pml_R[d][k] = 1e-15, s->pml_stretch[d][k] = 1.0;
  }
  s->a = a;
  s->courant = courant;
  s->dt = courant / a;  // src/structure.cpp:110
  s->ntot = 1;
  for (int d = 0; d < 3; d++)
    if (s->has[d]) s->ntot *= size_t(s->n[d] + 1);
  return s;
}

void mnl_structure_destroy(mnl_structure *s) { delete s; }

int mnl_structure_add_pml(mnl_structure *s, int dir, int side, double thickness, double R,
                          double mean_stretch) {
  if (!s || dir < 0 || dir > 2 || side < 0 || side > 1) return fail("bad pml direction/side");
  if (thickness < 0) return fail("invalid boundary absorbers for this grid_volume");
  if (!s->has[dir]) return 0;
  s->pml_thick[dir][side] = thickness;
  s->pml_R[dir][side] = R;
  s->pml_stretch[dir][side] = mean_stretch;
  return 0;
}

int mnl_structure_set_chi1inv(mnl_structure *s, int comp, int dir, const double *host) {
  if (!s || comp < MNL_EX || comp > MNL_HZ || dir < 0 || dir > 2)
    return fail("chi1inv: E or H components only");
  auto &dst = comp <= MNL_EZ ? s->chi1inv[comp][dir] : s->mu1inv[comp - MNL_HX][dir];
  if (host)
    dst.assign(host, host + s->ntot);
  else
    dst.clear();
  return 0;
}
int mnl_structure_set_chi2(mnl_structure *s, int comp, const double *host) {
  if (!s || comp < MNL_EX || comp > MNL_EZ) return fail("chi2: E components only");
  s->chi2[comp].assign(host, host + s->ntot);
  return 0;
}
int mnl_structure_set_conductivity(mnl_structure *s, int comp, const double *host) {
  // structure_chunk::set_conductivity (src/structure.cpp:868-905): E/H name the
  // D/B array; an E value is multiplied by the current diagonal chi1inv
  if (!s || comp < 0 || comp >= MNL_NUM_COMPONENTS) return fail("invalid component for conductivity");
  const int t = ctype(comp), d = cdir(comp), tb = (t == T_D || t == T_E) ? 1 : 0;
  auto &dst = s->cond[tb][d];
  if (!host) {
    dst.clear();
    return 0;
  }
  dst.assign(host, host + s->ntot);
  if (t == T_E && !s->chi1inv[d][d].empty())
    for (size_t i = 0; i < s->ntot; i++) dst[i] = host[i] * s->chi1inv[d][d][i];
  return 0;
}

int mnl_structure_set_chi3(mnl_structure *s, int comp, const double *host) {
  if (!s || comp < MNL_EX || comp > MNL_EZ) return fail("chi3: E components only");
  s->chi3[comp].assign(host, host + s->ntot);  // inert in the fork
  return 0;
}
int mnl_structure_add_lorentzian(mnl_structure *s, double omega0, double gamma, int drude,
                                 const double *sx, const double *sy, const double *sz) {
  const double *sig[9] = {sx, nullptr, nullptr, nullptr, sy, nullptr, nullptr, nullptr, sz};
  return mnl_structure_add_lorentzian_tensor(s, omega0, gamma, drude, sig);
}

int mnl_structure_add_lorentzian_tensor(mnl_structure *s, double omega0, double gamma, int drude,
                                        const double *const sigma[9]) {
  if (!s || !sigma) return fail("null argument");
  if ((int)s->lor.size() >= MAX_POL) return fail("too many susceptibilities (max 4)");
  Lorentz L;
  L.omega0 = omega0;
  L.gamma = gamma;
  L.drude = drude;
  for (int c = 0; c < 3; c++)
    for (int d = 0; d < 3; d++) {
      const double *v = sigma[3 * c + d];
      if (!v) continue;
      auto &dst = d == c ? L.sigma[c] : L.off[c][d];
      dst.assign(v, v + s->ntot);
      if (all_eq(dst, 0.0)) dst.clear();
    }
  s->lor.push_back(std::move(L));
  return 0;
}
int mnl_structure_add_magnetic_lorentzian(mnl_structure *s, double omega0, double gamma,
                                          int drude, const double *sx, const double *sy,
                                          const double *sz) {
  if (!s) return fail("null argument");
  if ((int)s->hlor.size() >= MAX_HPOL) return fail("too many magnetic susceptibilities (max 2)");
  Lorentz L;
  L.omega0 = omega0;
  L.gamma = gamma;
  L.drude = drude;
  const double *sv[3] = {sx, sy, sz};
  for (int d = 0; d < 3; d++) {
    if (!sv[d]) continue;
    L.sigma[d].assign(sv[d], sv[d] + s->ntot);
    if (all_eq(L.sigma[d], 0.0)) L.sigma[d].clear();
  }
  s->hlor.push_back(std::move(L));
  return 0;
}
int mnl_structure_set_nonlinear_mode(mnl_structure *s, int mode) {
  if (!s || mode < 0 || mode > 1) return fail("nonlinear mode must be 0 (fork) or 1 (upstream)");
  s->nl_mode = mode;
  return 0;
}

// ------------------------------------------------------------------ subpixel averaging
// Quadrature points and weights on the unit sphere for 1-D / 2-D / 3-D, the table
// the reference generates at build time (src/sphere-quad.cpp -> sphere-quad.h):
// 1-D {0,0,+-1}, 2-D 12 points on the circle, 3-D the 50-point degree-11 formula
// (McLaren; Stroud U3:11-1) with octahedral symmetry, each list reordered to
// maximise every point's distance from the earlier ones (squared distances
// compared in single precision, as the generator does).
namespace {
void sq_sort(int n, double *x, double *y, double *z, double *w) {
  for (int i = 1; i < n; ++i) {
    double best = 0, bestsum = 0;
    int jb = i;
    for (int j = i; j < n; ++j) {
      double mn = 1e20, sum = 0;
      for (int k = 0; k < i; ++k) {
        const double dx = x[k] - x[j], dy = y[k] - y[j], dz = z[k] - z[j];
        const double d2 = float(dx * dx + dy * dy + dz * dz);
        mn = mn < d2 ? mn : d2;
        sum += d2;
      }
      if (mn > best || (mn == best && sum > bestsum)) best = mn, bestsum = sum, jb = j;
    }
    std::swap(x[i], x[jb]);
    std::swap(y[i], y[jb]);
    std::swap(z[i], z[jb]);
    std::swap(w[i], w[jb]);
  }
}
// rotate (a, b, c) -> (c, a, b)
inline void rot3(double &a, double &b, double &c) {
  const double t = c;
  c = b;
  b = a;
  a = t;
}
void sphere_quad50(double *x, double *y, double *z, double *w) {
  int n = 0;
  auto put = [&](double a, double b, double c, double wt) {
    x[n] = a, y[n] = b, z[n] = c, w[n++] = wt;
  };
  double a = 1, b = 0, c = 0;  // 6 axis points
  for (int i = 0; i < 2; ++i) {
    a = -a;
    for (int j = 0; j < 3; ++j) rot3(a, b, c), put(a, b, c, 9216 / 725760.0);
  }
  a = b = sqrt(0.5), c = 0;  // 12 edge midpoints
  for (int i = 0; i < 2; ++i) {
    a = -a;
    for (int j = 0; j < 2; ++j) {
      b = -b;
      for (int k = 0; k < 3; ++k) rot3(a, b, c), put(a, b, c, 16384 / 725760.0);
    }
  }
  a = b = c = sqrt(1.0 / 3.0);  // 8 cube corners
  for (int i = 0; i < 2; ++i) {
    a = -a;
    for (int j = 0; j < 2; ++j) {
      b = -b;
      for (int k = 0; k < 2; ++k) c = -c, put(a, b, c, 15309 / 725760.0);
    }
  }
  a = b = sqrt(1.0 / 11.0), c = 3 * a;  // 24 points (1, 1, 3) / sqrt(11)
  for (int i = 0; i < 2; ++i) {
    a = -a;
    for (int j = 0; j < 2; ++j) {
      b = -b;
      for (int k = 0; k < 2; ++k) {
        c = -c;
        for (int l = 0; l < 3; ++l) rot3(a, b, c), put(a, b, c, 14641 / 725760.0);
      }
    }
  }
}
}  // namespace

// q[dim-1][i] = {x, y, z, weight}, nq = {2, 12, 50}
void sphere_quad_table(double q[3][AVG_MAXQ][4], int nq[3]) {
  memset(q, 0, sizeof(double) * 3 * AVG_MAXQ * 4);
  nq[0] = 2, nq[1] = 12, nq[2] = 50;
  q[0][0][2] = 1, q[0][0][3] = 0.5;
  q[0][1][2] = -1, q[0][1][3] = 0.5;
  double x[AVG_MAXQ], y[AVG_MAXQ], z[AVG_MAXQ], w[AVG_MAXQ];
  const double pi = 3.141592653589793238462643383279502884197;
  for (int i = 0; i < 12; ++i) {
    x[i] = cos(2 * i * pi / 12);
    y[i] = sin(2 * i * pi / 12);
    z[i] = 0.0;
    w[i] = 1.0 / 12;
  }
  sq_sort(12, x, y, z, w);
  for (int i = 0; i < 12; ++i) q[1][i][0] = x[i], q[1][i][1] = y[i], q[1][i][2] = z[i], q[1][i][3] = w[i];
  sphere_quad50(x, y, z, w);
  sq_sort(50, x, y, z, w);
  for (int i = 0; i < 50; ++i) q[2][i][0] = x[i], q[2][i][1] = y[i], q[2][i][2] = z[i], q[2][i][3] = w[i];
}

int mnl_sphere_quadrature(int dim, double *xyzw) {
  if (dim < 1 || dim > 3) return fail("sphere quadrature: dim must be 1, 2 or 3");
  double q[3][AVG_MAXQ][4];
  int nq[3];
  sphere_quad_table(q, nq);
  if (xyzw) memcpy(xyzw, q[dim - 1], sizeof(double) * 4 * nq[dim - 1]);
  return nq[dim - 1];
}

// structure::set_epsilon(material_function &, use_anisotropic_averaging, tol, maxeval)
// (src/structure.cpp:397-401 -> structure_chunk::set_chi1inv, src/anisotropic_averaging.cpp:
// 221-298) for a material function made of geometric objects, evaluated on a GPU.  The
// per-point values do not depend on the chunking, so the whole cell is computed once;
// which rows each reference chunk keeps (its trivial test) is decided per chunk when the
// fields are created, as for arrays set with mnl_structure_set_chi1inv.
int mnl_structure_set_epsilon_geometry(mnl_structure *s, int device, int nobj, const double *objs,
                                       double default_eps, int use_averaging, double tol,
                                       int maxeval) {
  if (!s || nobj < 0 || (nobj > 0 && !objs)) return fail("set_epsilon_geometry: bad arguments");
  std::vector<GeoObj> h(nobj);
  for (int o = 0; o < nobj; o++) {
    const double *r = objs + MNL_GEO_STRIDE * o;
    GeoObj &g = h[o];
    g.kind = (int)r[0];
    if (g.kind < 0 || g.kind > 2 || r[0] != g.kind) return fail("set_epsilon_geometry: bad object kind");
    g.eps = r[1];
    for (int d = 0; d < 3; d++) g.c[d] = r[2 + d], g.p[d] = r[5 + d];
    if (g.kind == 2 && !(g.p[2] == 0 || g.p[2] == 1 || g.p[2] == 2))
      return fail("set_epsilon_geometry: cylinder axis must be 0, 1 or 2");
  }
  int prev_dev = -1;
  HIPCHK(hipGetDevice(&prev_dev));
  if (device >= 0) HIPCHK(hipSetDevice(device));
  struct RestoreDev {  // leave the caller's current device as it was
    int d;
    ~RestoreDev() {
      if (d >= 0) (void)hipSetDevice(d);
    }
  } restore{prev_dev};
  double q[3][AVG_MAXQ][4];
  AvgArgs A{};
  sphere_quad_table(q, A.nq);
  A.ndir = 0;
  for (int d = 0; d < 3; d++) {
    A.has[d] = s->has[d];
    A.n[d] = s->n[d];
    A.io[d] = s->io[d];
    if (s->has[d]) A.dirs[A.ndir++] = d;
  }
  A.inva = 1.0 / s->a;
  A.default_eps = default_eps;
  A.nobj = nobj;
  A.maxeval = use_averaging ? maxeval : 0;  // set_chi1inv: !use_anisotropic_averaging -> 0
  A.tol = tol;
  A.ntot = (long long)s->ntot;
  // E components with a field and the rows the chunk allocates (FOR_FT_COMPONENTS with
  // has_field): 1-D Ex only, with its x row; 2-D and 3-D Ex, Ey, Ez with all three
  const int ncomp = s->dim == 1 ? 1 : 3;
  GeoObj *dobj = nullptr;
  double *dq = nullptr, *dout = nullptr;
  auto cleanup = [&]() {
    if (dobj) hipFree(dobj);
    if (dq) hipFree(dq);
    if (dout) hipFree(dout);
  };
  auto chk = [&](hipError_t e, const char *what) {
    if (e == hipSuccess) return 0;
    cleanup();
    return fail(std::string("set_epsilon_geometry: ") + what + ": " + hipGetErrorString(e));
  };
  if (nobj > 0) {
    if (chk(hipMalloc(&dobj, sizeof(GeoObj) * nobj), "hipMalloc")) return -1;
    if (chk(hipMemcpy(dobj, h.data(), sizeof(GeoObj) * nobj, hipMemcpyHostToDevice), "copy")) return -1;
  }
  if (chk(hipMalloc(&dq, sizeof(q)), "hipMalloc")) return -1;
  if (chk(hipMemcpy(dq, q, sizeof(q), hipMemcpyHostToDevice), "copy")) return -1;
  const int nrow = s->dim == 1 ? 1 : 3;
  if (chk(hipMalloc(&dout, sizeof(double) * s->ntot * nrow), "hipMalloc")) return -1;
  A.objs = dobj;
  A.quad = dq;
  for (int c = 0; c < ncomp; c++) {
    A.c = c;
    for (int d = 0; d < 3; d++) A.out[d] = nullptr;
    for (int d = 0; d < nrow; d++) A.out[d] = dout + s->ntot * d;
    if (k_avg_chi1inv(A, nullptr)) {
      cleanup();
      return fail("set_epsilon_geometry: kernel launch failed");
    }
    if (chk(hipDeviceSynchronize(), "kernel")) return -1;
    for (int d = 0; d < nrow; d++) {
      auto &dst = s->chi1inv[c][d];
      dst.resize(s->ntot);
      if (chk(hipMemcpy(dst.data(), A.out[d], sizeof(double) * s->ntot, hipMemcpyDeviceToHost),
              "copy back"))
        return -1;
    }
    // the reference deletes trivial off-diagonal rows, and the diagonal when the whole
    // tensor is trivial (src/anisotropic_averaging.cpp:282-296); done here over the whole
    // cell, per chunk at field creation
    bool triv[3];
    for (int d = 0; d < nrow; d++) {
      const double tv = d == c ? 1.0 : 0.0;
      const auto &v = s->chi1inv[c][d];
      triv[d] = std::all_of(v.begin(), v.end(), [&](double x) { return x == tv; });
    }
    for (int d = nrow; d < 3; d++) triv[d] = true;
    for (int d = 0; d < nrow; d++)
      if (d != c && triv[d]) std::vector<double>().swap(s->chi1inv[c][d]);
    if (triv[0] && triv[1] && triv[2] && c < nrow) std::vector<double>().swap(s->chi1inv[c][c]);
  }
  cleanup();
  return 0;
}

int mnl_structure_get_chi1inv(mnl_structure *s, int comp, int dir, double *host) {
  if (!s || comp < MNL_EX || comp > MNL_HZ || dir < 0 || dir > 2)
    return fail("chi1inv: E or H components only");
  const auto &v = comp <= MNL_EZ ? s->chi1inv[comp][dir] : s->mu1inv[comp - MNL_HX][dir];
  if (v.empty()) return 1;
  if (host) memcpy(host, v.data(), sizeof(double) * v.size());
  return 0;
}

int mnl_structure_set_box(mnl_structure *s, int kind, int index, const double box[6],
                          double value) {
  if (!s || kind < 0 || kind > 3) return fail("bad box kind");
  BoxSpec b;
  b.kind = kind;
  b.index = index;
  memcpy(b.box, box, sizeof(b.box));
  b.value = value;
  if (kind == 3) {  // make sure the susceptibility has a sigma array to fill
    if (index < 0 || index >= (int)s->lor.size()) return fail("box: no such susceptibility");
    for (int d = 0; d < 3; d++)
      if (s->lor[index].sigma[d].empty()) s->lor[index].sigma[d].assign(s->ntot, 0.0);
  }
  if (kind == 1) {
    for (int d = 0; d < 3; d++)
      if (s->chi2[d].empty()) s->chi2[d].assign(s->ntot, 0.0);
  }
  s->boxes.push_back(b);
  return 0;
}

mnl_fields *mnl_fields_create(mnl_structure *s, int device) {
  return create_common(s, device, 0, 1, nullptr);
}
mnl_fields *mnl_fields_create_dist(mnl_structure *s, int device, int rank, int nranks,
                                   const void *id) {
  if (nranks < 1 || rank < 0 || rank >= nranks) {
    fail("bad rank/nranks");
    return nullptr;
  }
  return create_common(s, device, rank, nranks, id);
}
void *mnl_local_hub_create(int nranks) {
  if (nranks < 1) {
    fail("bad nranks");
    return nullptr;
  }
  return local_hub_create(nranks);
}
void mnl_local_hub_destroy(void *hub) { local_hub_destroy((LocalHub *)hub); }
mnl_fields *mnl_fields_create_local(mnl_structure *s, int device, int rank, int nranks,
                                    void *hub) {
  if (!hub || nranks < 1 || rank < 0 || rank >= nranks) {
    fail("bad rank/nranks/hub");
    return nullptr;
  }
  return create_common(s, device, rank, nranks, nullptr, (LocalHub *)hub);
}
int mnl_slab_range(int ncell, int rank, int nranks, int *lo, int *hi) {
  if (nranks < 1 || rank < 0 || rank >= nranks || ncell < nranks) return fail("bad slab split");
  slab_range(ncell, rank, nranks, lo, hi);
  return 0;
}
int mnl_comm_unique_id(void *out128) { return Comm::unique_id(out128) ? fail("ncclGetUniqueId failed") : 0; }
int mnl_comm_ipc_id(void *out128, int nranks) {
  if (!out128) return fail("null id buffer");
  return Comm::ipc_id(out128, nranks) ? fail("cannot create the IPC shared-memory segment") : 0;
}
int mnl_comm_ipc_unlink(const void *id128) {
  return Comm::ipc_unlink(id128) ? fail("no such IPC shared-memory segment") : 0;
}
int mnl_comm_ipc_reduce(const void *id128, int rank, int nranks, double *host, int n, int ok) {
  if (!Comm::is_ipc_id(id128) || nranks < 1 || rank < 0 || rank >= nranks || n < 0)
    return fail("bad IPC id / rank / size");
  Comm cm;
  if (cm.init(rank, nranks, id128)) return fail("IPC slab group init failed (shared-memory id)");
  if (cm.agree_ok(ok != 0, nullptr)) return fail("a rank reported failure");
  if (cm.allreduce_sum(host, n, nullptr)) return fail("IPC allreduce failed");
  return 0;
}
const char *mnl_fields_transport(mnl_fields *f) {
  if (!f) return "";
  return f->comm ? f->comm->transport() : "single";
}
int mnl_comm_rccl_selftest(int device, int n) {
  if (n < 1) return fail("selftest needs n >= 1");
  if (hipSetDevice(device) != hipSuccess) return fail("hipSetDevice failed");
  char id[128];
  if (Comm::unique_id(id)) return fail("ncclGetUniqueId failed");
  Comm cm;
  if (cm.init(0, 1, id)) return fail("RCCL communicator init failed");
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return fail("stream");
  std::vector<double> h(n), back(n);
  for (int i = 0; i < n; i++) h[i] = 0.5 * i - 3.25;
  double *a = nullptr, *b = nullptr;
  int rc = 0;
  if (hipMalloc(&a, n * sizeof(double)) != hipSuccess ||
      hipMalloc(&b, n * sizeof(double)) != hipSuccess)
    rc = fail("hipMalloc failed");
  if (!rc && hipMemcpy(a, h.data(), n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess)
    rc = fail("upload failed");
  if (!rc && (cm.group_start() || cm.send(a, n, 0, s) || cm.recv(b, n, 0, s) || cm.group_end(s)))
    rc = fail("grouped send/recv failed");
  if (!rc && (hipStreamSynchronize(s) != hipSuccess ||
              hipMemcpy(back.data(), b, n * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess))
    rc = fail("download failed");
  if (!rc && memcmp(back.data(), h.data(), n * sizeof(double)) != 0)
    rc = fail("send/recv data mismatch");
  std::vector<double> red(h);
  if (!rc && cm.allreduce_sum(red.data(), n, s)) rc = fail("allreduce failed");
  if (!rc && memcmp(red.data(), h.data(), n * sizeof(double)) != 0)
    rc = fail("allreduce data mismatch");
  if (a) (void)hipFree(a);
  if (b) (void)hipFree(b);
  (void)hipStreamDestroy(s);
  return rc;
}

void mnl_fields_destroy(mnl_fields *f) { delete f; }

int mnl_fields_add_point_source(mnl_fields *F, int comp, int kind, const double *p, int np,
                                const double pos[3], double amp_re, double amp_im,
                                int is_integrated) {
  if (!pos) return fail("null position");
  return add_source_any(F, comp, kind, p, np, nullptr, nullptr, pos, pos, amp_re, amp_im,
                        is_integrated, nullptr, nullptr);
}

int mnl_fields_add_volume_source(mnl_fields *F, int comp, int kind, const double *p, int np,
                                 const double vmin[3], const double vmax[3], double amp_re,
                                 double amp_im, int is_integrated, mnl_amp_func afunc,
                                 void *adata) {
  if (!vmin || !vmax) return fail("null volume");
  if (kind == MNL_SRC_CUSTOM) return fail("custom sources: use mnl_fields_add_custom_volume_source");
  return add_source_any(F, comp, kind, p, np, nullptr, nullptr, vmin, vmax, amp_re, amp_im,
                        is_integrated, afunc, adata);
}

int mnl_fields_add_custom_volume_source(mnl_fields *F, int comp, mnl_src_func func, void *data,
                                        double start_time, double end_time, const double vmin[3],
                                        const double vmax[3], double amp_re, double amp_im,
                                        int is_integrated, mnl_amp_func afunc, void *adata) {
  if (!func) return fail("custom source needs a function");
  if (!vmin || !vmax) return fail("null volume");
  const double p[2] = {start_time, end_time};
  return add_source_any(F, comp, MNL_SRC_CUSTOM, p, 2, func, data, vmin, vmax, amp_re, amp_im,
                        is_integrated, afunc, adata);
}

int mnl_fields_add_custom_point_source(mnl_fields *F, int comp, mnl_src_func func, void *data,
                                       double start_time, double end_time, const double pos[3],
                                       double amp_re, double amp_im, int is_integrated) {
  if (!func) return fail("custom source needs a function");
  const double p[2] = {start_time, end_time};
  if (!pos) return fail("null position");
  return add_source_any(F, comp, MNL_SRC_CUSTOM, p, 2, func, data, pos, pos, amp_re, amp_im,
                        is_integrated, nullptr, nullptr);
}


int mnl_fields_require_component(mnl_fields *F, int comp) {
  if (!F || check_comp(comp)) return -1;
  if (!has_field(F->S, comp)) return fail("component not present in this dimensionality");
  if (hipSetDevice(F->device) != hipSuccess) return fail("hipSetDevice failed");
  return require_component(F, comp);
}

int mnl_fields_step(mnl_fields *F, int nsteps) {
  if (!F) return fail("null fields");
  if (nsteps <= 0) return 0;
  if (hipSetDevice(F->device) != hipSuccess) return fail("hipSetDevice failed");
  return fields_step(F, nsteps);
}

// Tuning of the fused step, measured rather than modelled:
// (1) the tile kernel's z-chunk length (fill of the last round of items vs. the halo planes
// of short chunks); (2) on one rank with polarization chunks, the CUs given to their general
// kernel running beside the tile kernel (a split that balances the two launches; too few
// or too many CUs and one of them runs alone at the end).  Every candidate is stepped for
// real: results do not depend on either knob (each point's update is the same arithmetic).
// Times are the fused launches' own (profiling events around them), not the host's
// per-batch work.
int mnl_fields_tune(mnl_fields *F, int reps, int *zchunk, int *gen_cus) {
  if (!F || reps < 1) return fail("bad argument");
  if (zchunk) *zchunk = -1;
  if (gen_cus) *gen_cus = -1;
  if (hipSetDevice(F->device) != hipSuccess) return fail("hipSetDevice failed");
  // the first step runs unfused (lazy first updates); the second takes the fused decision
  for (int i = 0; i < 2 && !F->fused; i++)
    if (fields_step(F, 1)) return -1;
  if (!F->fused || !F->tile_mode) return 0;
  const bool prof = F->profiling;  // restored with the timers after tuning
  double tms[16];
  long long tcnt[16];
  for (int k = 0; k < 16; k++) tms[k] = F->timer_ms[k], tcnt[k] = F->timer_count[k];
  F->profiling = true;
  const bool verbose = getenv("MNL_TUNE_VERBOSE") != nullptr;
  // per-step time of the fused launches: tile kernel (+ the pairs' phase and rim launches of
  // temporal blocking) and the polarization chunks' general kernel
  auto fused_ms = [&]() {
    return F->timer_ms[TM_BINT] + F->timer_ms[TM_TB] + F->timer_ms[TM_RIM];
  };
  auto timed = [&](double *tile_ms, double *gen_ms) -> int {  // two warm-up steps (a pair
    if (fields_step(F, 2)) return -1;                           // builds its plan), then an
    const int r = reps + (reps & 1);                            // even number timed
    const double b0 = fused_ms(), g0 = F->timer_ms[TM_GEN];
    if (fields_step(F, r)) return -1;
    *tile_ms = (fused_ms() - b0) / r;
    *gen_ms = (F->timer_ms[TM_GEN] - g0) / r;
    if (F->nranks > 1) {  // every rank keeps the same knobs: the slowest rank's times
      std::vector<double> v(2 * (size_t)F->nranks, 0.0);
      v[2 * F->rank] = *tile_ms, v[2 * F->rank + 1] = *gen_ms;
      if (F->comm->allreduce_sum(v.data(), (int)v.size(), F->stream)) return fail("tune allreduce failed");
      for (int q = 0; q < F->nranks; q++)
        *tile_ms = std::max(*tile_ms, v[2 * q]), *gen_ms = std::max(*gen_ms, v[2 * q + 1]);
    }
    return 0;
  };
  int rc = 0;
  const int split0 = F->tile_gen_cus;
  if (!F->fused_zchunk_env) {
    static const int cand[] = {0, 16, 20, 24, 32, 48};
    F->tile_gen_cus = 0;  // the two launches one after the other while the length is chosen
    int best = F->fused_zchunk;
    double best_ms = 0;
    for (int c : cand) {
      if (F->fused && set_fused(F, false)) { rc = -1; break; }
      F->fused_zchunk = c;
      double tm, gm;
      if (timed(&tm, &gm)) { rc = -1; break; }
      if (!F->fused) continue;  // this length does not fit the fused kernels; longer ones may
      if (verbose)
        fprintf(stderr, "tune rank %d: zchunk %d: %.4f ms/step (tile %.4f, general %.4f)\n",
                F->rank, c, tm + gm, tm, gm);
      if (best_ms == 0 || tm + gm < best_ms) best_ms = tm + gm, best = c;
    }
    F->tile_gen_cus = split0;
    if (!rc && F->fused && set_fused(F, false)) rc = -1;  // the next step rebuilds with `best`
    F->fused_zchunk = best;
    if (!rc && zchunk) *zchunk = best;
  }
  if (!rc && F->nranks == 1 && !F->tile_gen_cus_env) {
    F->tile_gen_cus = 0;
    double tm = 0, gm = 0;
    if (timed(&tm, &gm)) rc = -1;
    if (!rc && F->fused && F->tile_mode && gm > 0) {
      // start from the split that gives both launches the same time at their measured
      // one-after-the-other rates, in multiples of 8 CUs (one per XCD)
      const int cus = k_cu_count();
      const int s0 = 8 * (int)std::lround(cus * gm / (gm + tm) / 8.0);
      int best = 0;
      double best_ms = tm + gm;
      if (verbose)
        fprintf(stderr, "tune rank %d: general CUs 0: %.4f ms/step\n", F->rank, best_ms);
      for (int d : {-16, -8, 0, 8, 16}) {
        const int sc = s0 + d;
        if (sc < 8 || sc > cus - 8) continue;
        F->tile_gen_cus = sc;
        double t2, g2;
        if (timed(&t2, &g2)) { rc = -1; break; }
        if (verbose)
          fprintf(stderr, "tune rank %d: general CUs %d: %.4f ms/step\n", F->rank, sc, t2 + g2);
        if (t2 + g2 < best_ms) best_ms = t2 + g2, best = sc;
      }
      F->tile_gen_cus = best;
      if (!rc && gen_cus) *gen_cus = best;
    } else {
      F->tile_gen_cus = split0;
    }
  }
  // temporal blocking: planes per two-step item (automatic = the item count that fills whole
  // rounds), and whether pairs beat one-step stepping at all (small grids: the rim is a
  // large share of the cells)
  if (!rc && F->fused && F->tb_have && F->tb_enabled) {
    const int tz0 = F->tb_zchunk, ox0 = F->tb_ox;
    int best = tz0, best_ox = ox0;
    double best_ms = 0;
    // (16 / 24 / 40 added in round 5: 256^3 C2 runs 6 % faster at 16-24 planes than with the
    // automatic length, profiles/r05_ab_tb_zchunk_c2_256.json.  Round 6: the items hold up to
    // 124 columns, so a small grid has few of them per plane; 60-column items (half the lanes
    // idle, twice the items) and 12 / 20 planes are tried too, against the tail of a launch
    // with fewer items than a few rounds of CUs)
    // Round 6: the candidates' differences at 256^3 are within one box's drift over a sweep
    // (C2 picked 48 planes once, 6 % slower than 16-24), so the sweep runs forward and then
    // backward (a candidate's time is its better one), and the three best are timed again
    // with twice the steps before the choice
    std::vector<std::pair<int, int>> cands;  // (width setting, planes)
    for (int ox : {0, 60}) {
      if (F->tb_ox_set && ox != ox0) continue;
      for (int c : {0, 12, 16, 20, 24, 32, 40, 48, 64, 96, 128}) {
        if (F->tb_zchunk_env && c != tz0) continue;
        if (ox == 60 && c > 48) continue;  // the narrow items only help small grids
        cands.push_back({ox, c});
      }
    }
    std::vector<double> cms(cands.size(), 0.0);
    auto measure = [&](size_t i, int mult) -> int {
      F->tb_ox = cands[i].first;
      F->tb_zchunk = cands[i].second;
      double tm = 0, gm = 0;
      const int reps0 = reps;
      reps *= mult;
      const int r = timed(&tm, &gm);
      reps = reps0;
      if (r) return -1;
      if (verbose)
        fprintf(stderr, "tune rank %d: two-step planes %d, width %d: %.4f ms/step\n", F->rank,
                cands[i].second, cands[i].first ? cands[i].first : TB_OXW, tm + gm);
      if (cms[i] == 0 || tm + gm < cms[i]) cms[i] = tm + gm;
      return 0;
    };
    for (size_t i = 0; i < cands.size() && !rc; i++) rc = measure(i, 1);
    for (size_t i = cands.size(); i-- > 0 && !rc;) rc = measure(i, 1);
    if (!rc && cands.size() > 1) {
      std::vector<size_t> ord(cands.size());
      for (size_t i = 0; i < ord.size(); i++) ord[i] = i;
      std::stable_sort(ord.begin(), ord.end(), [&](size_t x, size_t y) { return cms[x] < cms[y]; });
      for (size_t k = 0; k < std::min<size_t>(3, ord.size()) && !rc; k++) rc = measure(ord[k], 2);
    }
    for (size_t i = 0; i < cands.size() && !rc; i++)
      if (best_ms == 0 || cms[i] < best_ms) best_ms = cms[i], best = cands[i].second, best_ox = cands[i].first;
    F->tb_zchunk = rc ? tz0 : best;
    F->tb_ox = rc ? ox0 : best_ox;
    if (!rc && !F->tb_env) {  // one-step stepping, timed twice as well (the better one)
      F->tb_enabled = false;
      double one = 0;
      for (int mult = 1; mult <= 2 && !rc; mult++) {
        double tm, gm;
        const int reps0 = reps;
        reps *= mult;
        if (timed(&tm, &gm)) rc = -1;
        reps = reps0;
        if (rc) break;
        if (verbose)
          fprintf(stderr, "tune rank %d: one-step: %.4f ms/step\n", F->rank, tm + gm);
        if (one == 0 || tm + gm < one) one = tm + gm;
      }
      F->tb_enabled = rc || one >= best_ms;
    }
  }
  F->profiling = prof;
  for (int k = 0; k < 16; k++) F->timer_ms[k] = tms[k], F->timer_count[k] = tcnt[k];
  return rc;
}

int mnl_fields_initialize_field(mnl_fields *F, int comp, const double *host, size_t n) {
  if (!F || check_comp(comp) || !host) return fail("bad argument");
  if (n < F->S.ntot) return fail("initialize_field: array smaller than the cell");
  if (!has_field(F->S, comp)) return fail("component not present in this dimensionality");
  if (hipSetDevice(F->device) != hipSuccess) return fail("hipSetDevice failed");
  F->f.nr_t = F->t;  // its update_eh(E) solves at the current time step
  return initialize_field(F, comp, host);
}

int mnl_fields_energy_in_box(mnl_fields *F, int which, const double vmin[3], const double vmax[3],
                             double *out) {
  if (!F || !out || which < 0 || which > 2) return fail("bad argument");
  if (hipSetDevice(F->device) != hipSuccess) return fail("hipSetDevice failed");
  double lo[3], hi[3];
  const mnl_structure &S = F->S;
  for (int d = 0; d < 3; d++) {  // NULL: the whole cell (user_volume.surroundings())
    lo[d] = S.has[d] ? (vmin ? vmin[d] : S.io[d] * (0.5 / S.a)) : 0.0;
    hi[d] = S.has[d] ? (vmax ? vmax[d] : (S.io[d] + 2 * S.n[d]) * (0.5 / S.a)) : 0.0;
  }
  return energy_in_box(F, which, lo, hi, out);
}

int mnl_fields_set_nan_check(mnl_fields *F, int every) {
  if (!F || every < 1) return fail("NaN check cadence must be >= 1 step");
  F->nan_every = every;
  return 0;
}

int mnl_fields_array_slice(mnl_fields *F, int comp, const double vmin[3], const double vmax[3],
                           int snap, int *rank, long long dims[3], double *out, long long nout) {
  if (!F || !vmin || !vmax || !rank || !dims) return fail("bad argument");
  if (comp != MNL_DIELECTRIC && comp != MNL_PERMEABILITY && check_comp(comp))
    return fail("bad argument");
  return array_slice(F, comp, vmin, vmax, snap, rank, dims, out, nout);
}

int mnl_fields_dump(mnl_fields *F, const char *filename) {
  if (!F || !filename) return fail("null argument");
  if (hipSetDevice(F->device) != hipSuccess) return fail("hipSetDevice failed");
  std::string p = filename;
  if (F->nranks > 1) p += ".rank" + std::to_string(F->rank);
  return fields_dump(F, p.c_str());
}

int mnl_fields_load(mnl_fields *F, const char *filename) {
  if (!F || !filename) return fail("null argument");
  if (hipSetDevice(F->device) != hipSuccess) return fail("hipSetDevice failed");
  std::string p = filename;
  if (F->nranks > 1) p += ".rank" + std::to_string(F->rank);
  return fields_load(F, p.c_str());
}

int mnl_structure_dump(mnl_structure *s, const char *filename) {
  if (!s || !filename) return fail("null argument");
  return structure_dump(s, filename);
}

int mnl_structure_load(mnl_structure *s, const char *filename) {
  if (!s || !filename) return fail("null argument");
  return structure_load(s, filename);
}

int mnl_fields_time(mnl_fields *F, long long *t, double *dt) {
  if (!F) return fail("null fields");
  if (t) *t = F->t;
  if (dt) *dt = F->dt;
  return 0;
}

int mnl_fields_set_time(mnl_fields *F, long long t) {
  if (!F || t < 0) return fail("bad argument");
  F->t = t;
  return 0;
}

int mnl_fields_zero_fields(mnl_fields *F) {
  // fields_chunk::zero_fields (src/fields.cpp:638-664): every field, f_u, f_w and f_cond
  // array to 0 and the polarizations re-initialised (P = P_prev = 0); the DFT
  // accumulators are kept.  Leaves fused mode first (its ping-pong partners are
  // rebuilt from the zeroed arrays when it is entered again).
  if (!F) return fail("null fields");
  if (hipSetDevice(F->device) != hipSuccess) return fail("hipSetDevice failed");
  if (F->fused && set_fused(F, false)) return -1;
  for (const CkEntry &e : ckpt_entries(F))
    if (e.kind != 11) HIPCHK(hipMemsetAsync(e.p, 0, e.n * sizeof(double), F->stream));
  HIPCHK(hipStreamSynchronize(F->stream));
  return 0;
}

int mnl_fields_remove_sources(mnl_fields *F) {
  // fields::remove_sources (src/fields.cpp:601-610): every source and its src_time
  if (!F) return fail("null fields");
  F->groups.clear();
  F->srcs.clear();
  F->src_dirty = true;
  return 0;
}

int mnl_fields_get_field(mnl_fields *F, int comp, const double pos[3], double *out) {
  if (!F || check_comp(comp)) return -1;
  if (!has_field(F->S, comp)) return fail("component not present in this dimensionality");
  if (hipSetDevice(F->device) != hipSuccess) return fail("hipSetDevice failed");
  return get_field(F, comp, pos, out, true);
}

size_t mnl_fields_ntot(mnl_fields *F) { return F ? F->S.ntot : 0; }

int mnl_fields_copy_component(mnl_fields *F, int comp, double *host, size_t n) {
  if (!F || check_comp(comp)) return -1;
  if (n < F->S.ntot) return fail("output buffer too small");
  if (hipSetDevice(F->device) != hipSuccess) return fail("hipSetDevice failed");
  memset(host, 0, F->S.ntot * sizeof(double));
  if (!has_field(F->S, comp) || !F->allocated[comp]) return 0;
  int t = ctype(comp), d = cdir(comp);
  const double *src = nullptr, *hsep = nullptr;
  switch (t) {
    case T_E: src = F->f.E[d]; break;
    case T_D: src = F->f.D[d]; break;
    case T_B: src = F->f.B[d]; break;
    case T_H:
      src = F->f.B[d];
      hsep = (F->hall && !F->h_first_done) ? nullptr : F->f.H[d];
      break;
  }
  if (!src) return 0;
  size_t nt = F->S.ntot;
  if (F->scratch_cap < nt) {
    if (F->d_scratch) hipFree(F->d_scratch);
    HIPCHK(hipMalloc(&F->d_scratch, nt * sizeof(double)));
    F->scratch_cap = nt;
  }
  HIPCHK(hipMemsetAsync(F->d_scratch, 0, nt * sizeof(double), F->stream));
  const bool fe = F->fused && t == T_E;
  if (k_to_canonical(F->d_scratch, src, hsep, F->g, t, d, F->f, fe ? &F->fusedG : nullptr,
                     fe ? F->f.D[d] : nullptr, fe ? F->f.inveps[d] : nullptr, F->stream))
    return fail("to_canonical launch failed");
  HIPCHK(hipMemcpyAsync(host, F->d_scratch, nt * sizeof(double), hipMemcpyDeviceToHost, F->stream));
  HIPCHK(hipStreamSynchronize(F->stream));
  return 0;
}

int mnl_fields_time_spent(mnl_fields *F, double *out) {
  if (!F || !out) return fail("bad argument");
  for (int k = 0; k < MNL_NUM_TIME_SINKS; k++) out[k] = F->sink_s[k];
  return 0;
}

int mnl_fields_reset_timers(mnl_fields *F) {
  if (!F) return fail("null fields");
  for (int k = 0; k < MNL_NUM_TIME_SINKS; k++) F->sink_s[k] = 0;
  return 0;
}

int mnl_fields_allreduce(mnl_fields *F, double *v, int n) {
  if (!F || (n > 0 && !v) || n < 0) return fail("bad argument");
  if (F->nranks == 1 || n == 0) return 0;
  if (hipSetDevice(F->device) != hipSuccess) return fail("hipSetDevice failed");
  return timed_allreduce(F, v, n) ? fail("allreduce failed") : 0;
}

void mnl_set_verbosity(int level) { g_verbosity = level; }
int mnl_get_verbosity(void) { return g_verbosity; }

int mnl_fields_timers(mnl_fields *F, double out[6]) {
  if (!F) return fail("null fields");
  out[0] = F->timer_ms[TM_B] + F->timer_ms[TM_BINT];
  out[1] = F->timer_ms[TM_H];
  out[2] = F->timer_ms[TM_D] + F->timer_ms[TM_DINT];
  out[3] = F->timer_ms[TM_E];
  out[4] = F->timer_ms[TM_SRC];
  out[5] = F->timer_ms[TM_HALO];
  return 0;
}

int mnl_fields_nr_fallbacks(mnl_fields *F, long long *count) {
  if (!F) return fail("null fields");
  unsigned long long v = 0;
  if (hipSetDevice(F->device) != hipSuccess) return fail("hipSetDevice failed");
  HIPCHK(hipMemcpy(&v, F->d_nr_fallbacks, sizeof(v), hipMemcpyDeviceToHost));
  *count = (long long)v;
  return 0;
}

int mnl_fields_set_fused(mnl_fields *F, int allow) {
  if (!F) return fail("null fields");
  if (hipSetDevice(F->device) != hipSuccess) return fail("hipSetDevice failed");
  F->allow_fused = allow != 0;
  if (!F->allow_fused) return set_fused(F, false);
  return 0;
}

int mnl_fields_set_profiling(mnl_fields *F, int on) {
  if (!F) return fail("null fields");
  F->profiling = on != 0;
  for (int k = 0; k < 16; k++) F->timer_ms[k] = 0, F->timer_count[k] = 0;
  return 0;
}

// Algorithmic HBM bytes of one fused step over G (DESIGN.md "Fused step"):
// every point reads B, D and writes B, D (96 B) + chi1inv (4 B palette word
// or 3 doubles); PML state is counted per (point, component) where the
// reference keeps it: f_u of B / D, separate H, W-form E (read + write 16 B).
// lean: the same for the lean tiles only (no PML state there).
void fused_bytes(const mnl_fields *F, double *lean_bytes, double *gen_bytes) {
  const DevGrid &g = F->g;
  const FusedArgs &a = F->fgeo;
  int nu = 0;
  for (int d = 0; d < 3; d++) nu += F->f.inveps[d] ? 1 : 0;
  const double ub = F->d_uidx ? 4.0 : 8.0 * nu;
  // with per-item uniform palette words only the mixed items read chi1inv per cell
  const bool uni = F->d_uidx && F->uflag_active && F->lean_cells_nu >= 0;
  const double lean_u = uni ? F->lean_cells_nu : double(F->lean_cells);
  *lean_bytes = double(F->lean_cells) * 96.0 + lean_u * ub;
  double extra = 0, extra_t = 0;
  // count of local indices j in [lo, hi] of axis e with an optional flag condition;
  // zsel (axis 2): 0 every plane, 1 the tile kernel's planes, 2 the others
  int zsel = 0;
  auto cnt = [&](int e, int lo, int hi, int qshift, bool need_flag) -> double {
    double n = 0;
    for (int j = lo; j <= hi; j++) {
      if (e == 2 && zsel && (j < 0 || j >= (int)F->tile_z.size() ||
                             (F->tile_z[j] != 0) != (zsel == 1)))
        continue;
      if (need_flag) {
        if (!F->S.has[e] || F->h_flag[e].empty()) continue;
        if (!F->h_flag[e][2 * (j + g.off[e]) + qshift]) continue;
      }
      n += 1;
    }
    return n;
  };
  for (int pass = 0; pass < (F->tile_mode ? 2 : 1); pass++) {
    zsel = F->tile_mode ? (pass == 0 ? 1 : 2) : 0;
    for (int c = 0; c < 3; c++)
      for (int kind = 0; kind < 4; kind++) {
        // kind 0: f_u of B_c (flag along c+2, shifted); 1: H_c (along c, unshifted);
        // 2: f_u of D_c (along c+2, unshifted); 3: W-form E_c (along c, shifted)
        const bool btype = kind < 2;
        const int fe = (kind == 0 || kind == 2) ? (c + 2) % 3 : c;
        const int qs = (kind == 0 || kind == 3) ? 1 : 0;
        double n = 1;
        for (int e = 0; e < 3; e++) {
          const bool sh = btype ? (e != c) : (e == c);
          const int lo = sh ? a.osh_lo[e] : a.oun_lo[e], hi = sh ? a.osh_hi[e] : a.oun_hi[e];
          n *= cnt(e, lo, hi, qs, e == fe);
        }
        (zsel == 1 ? extra_t : extra) += 16.0 * n;
      }
  }
  if (F->tile_mode) {  // tile kernel = "lean" slot of the statistics, general = the rest
    const bool tuni = F->d_uidx && F->uflag_active && F->tile_cells_nu >= 0;
    *lean_bytes = double(F->tile_cells) * 96.0 +
                  (tuni ? F->tile_cells_nu : double(F->tile_cells)) * ub + extra_t;
  }
  // polarization boxes: stored E (read + write), P and Pprev (read + write) and
  // sigma (read) per component and susceptibility
  for (int k = 0; k < F->f.npol; k++) {
    const Box &b = F->f.pol[k].nz;
    double n = 1;
    for (int e = 0; e < 3; e++) {
      const int lo = std::max(b.lo[e], F->fusedG.lo[e]), hi = std::min(b.hi[e], F->fusedG.hi[e]);
      n *= hi >= lo ? double(hi - lo + 1) : 0.0;
    }
    int nc = 0;
    for (int d = 0; d < 3; d++) nc += F->f.pol[k].P[d] ? 1 : 0;
    extra += n * nc * (40.0 + (k == 0 ? 16.0 : 0.0));
  }
  double gcells = 1;
  for (int e = 0; e < 3; e++) gcells *= double(F->fusedG.hi[e] - F->fusedG.lo[e] + 1);
  if (F->tile_mode) {
    const bool guni = F->d_uidx && F->uflag_active && F->gen_cells_nu >= 0;
    *gen_bytes = double(F->gen_cells) * 96.0 +
                 (guni ? F->gen_cells_nu : double(F->gen_cells)) * ub + extra;
    return;
  }
  const double gen_u = uni ? F->gen_cells_nu : gcells - double(F->lean_cells);
  *gen_bytes = (gcells - double(F->lean_cells)) * 96.0 + gen_u * ub + extra;
}

int mnl_fields_kernel_stats(mnl_fields *F, int which, long long *launches, double *total_ms,
                            double *bytes_per_launch) {
  if (!F || which < 0 || which > 8) return fail("bad kernel id");
  if (which == 7 || which == 8) {  // multi-rank pairs: slab-face chains / E-ghost waits
    const int cat = which == 7 ? TM_CHAIN : TM_WAIT;
    *launches = F->timer_count[cat];
    *total_ms = F->timer_ms[cat];
    *bytes_per_launch = 0;
    return 0;
  }
  if (which == 5 || which == 6) {
    // temporal blocking.  5 = whole pairs of steps: launches = pairs, time = every launch of
    // the pairs (two phase launches each, the drains of the rim's last step), bytes per pair =
    // the two-step items' two steps (B, D read once and written once, the palette word where
    // the item is mixed, the border points' step n+1 B, D) + two rim steps.  6 = the rim
    // launches, one step each
    int nu = 0;
    for (int d = 0; d < 3; d++) nu += F->f.inveps[d] ? 1 : 0;
    const double ub = F->d_uidx ? 4.0 : 8.0 * nu;
    double tb_b = 0, rim_b = 0;
    if (F->fused && F->tb_have) {
      tb_b = F->tb_cells * 96.0 + (F->d_uidx ? F->tb_cells_nu : F->tb_cells) * ub +
             F->tb_border * 48.0;
      double lb, gb;
      fused_bytes(F, &lb, &gb);
      const bool tuni = F->d_uidx && F->uflag_active && F->tile_cells_nu >= 0;
      rim_b = lb - double(F->tile_cells) * 96.0 -
              (tuni ? F->tile_cells_nu : double(F->tile_cells)) * ub + F->rim_cells * 96.0 +
              (F->d_uidx ? F->rim_cells_nu : F->rim_cells) * ub;
    }
    if (which == 5) {
      *launches = F->timer_count[TM_TB];
      *total_ms = F->timer_ms[TM_TB] + F->timer_ms[TM_RIM];
      *bytes_per_launch = tb_b + 2.0 * rim_b;
      if (F->fused && F->tb_have && F->tb_pol) {  // + the polarization chunks' two steps
        double lb, gb;
        fused_bytes(F, &lb, &gb);
        *total_ms += F->timer_ms[TM_GEN];
        *bytes_per_launch += 2.0 * gb;
      }
    } else {
      *launches = F->timer_count[TM_RIM];
      *total_ms = F->timer_ms[TM_RIM];
      *bytes_per_launch = rim_b;
    }
    return 0;
  }
  if (which == 4) {  // E update (update_eh(E_stuff) incl. chi(2) Newton-Raphson, Lorentzian P)
    *launches = F->timer_count[TM_E];
    *total_ms = F->timer_ms[TM_E];
    *bytes_per_launch = 0;
    return 0;
  }
  if (which == 3) {  // DFT updates of one step (all flux objects)
    *launches = F->timer_count[TM_DFT];
    *total_ms = F->timer_ms[TM_DFT] + F->timer_ms[TM_DFTF];
    double b = 0;
    for (auto &o : F->dfts) b += o->bytes;
    *bytes_per_launch = b;
    return 0;
  }
  // 0: lean fused kernel (or interior curl B when unfused), 1: interior curl D
  // (unfused), 2: general fused kernel
  int cat = which == 0 ? TM_BINT : (which == 1 ? TM_DINT : TM_GEN);
  *launches = F->timer_count[cat];
  *total_ms = F->timer_ms[cat];
  if (F->fused && which != 1) {
    double lb, gb;
    fused_bytes(F, &lb, &gb);
    // concurrent lean + general: the timed span covers both kernels
    *bytes_per_launch = which == 0 ? (F->fused_concurrent ? lb + gb : lb) : gb;
    return 0;
  }
  if (which == 2) {
    *bytes_per_launch = 0;
    return 0;
  }
  const Box &b = F->interior;
  double pts = 1;
  for (int k = 0; k < 3; k++) pts *= double(b.hi[k] - b.lo[k] + 1);
  if (b.hi[0] < b.lo[0]) pts = 0;
  // interior curl: read 3 source comps + read/write the updated comps
  int ncomp = 0;
  const CurlPlan &p = which == 0 ? F->planB : F->planD;
  for (int d = 0; d < 3; d++) ncomp += p.present[d] ? 1 : 0;
  int nsrc = 0;
  for (int d = 0; d < 3; d++) nsrc += F->allocated[3 * (which == 0 ? T_E : T_H) + d] ? 1 : 0;
  *bytes_per_launch = pts * 8.0 * (nsrc + 2 * ncomp);
  return 0;
}

int mnl_fields_set_temporal_blocking(mnl_fields *F, int on) {
  if (!F) return fail("null fields");
  F->tb_enabled = on != 0;
  return 0;
}

int mnl_fields_set_schedule(mnl_fields *F, int which, int value) {
  if (!F) return fail("null fields");
  const bool v = value != 0;
  if (which == 0) {
    F->tb_narrow = v;
  } else if (which >= 2 && which <= 4) {  // CUs left free by the pair launches (single rank)
    if (value < -1 || value > 1024) return fail("bad reservation");
    (which == 2 ? F->tb_res : which == 3 ? F->res_l : F->res_r) = value;
    return 0;
  } else if (which == 5) {
    F->dft_cmp = v;
  } else if (which == 7) {
    F->nr_early = v;
  } else if (which == 11) {  // pairs with polarization chunks (0: one-step stepping there)
    F->tb_pol_on = v;
  } else if (which == 12) {  // R1's non-strip items beside the two-step kernel (one rank)
    F->tb_r1a = v;
  } else if (which == 16) {  // a pair's source + guard launches merged (one rank)
    F->tb_srcguard = v;
    return 0;
  } else if (which == 15) {  // planes per narrow strip item (0: the rim's chunk length)
    if (value < 0 || value > FUSED_MAXCH) return fail("bad strip chunk");
    F->tb_szc = value;
  } else if (which == 14) {  // the second rim launch's order (one rank): 1 longest first,
    if (value < 0 || value > 2) return fail("bad rim order");  // 2 the narrow strips first
    F->tb_r2lpt = value;
  } else if (which == 13) {  // interior two-step items beside the previous pair's R2
    if (value < 0 || value > 7) return fail("bad interior-items setting");
    F->tb_lint = value;  // (2: split, released after all before; 3..7: on 3/8..7/8 of the CUs)
  } else if (which == 10) {  // columns per lane of the two-step kernel (1: round-5 kernel)
    if (value != 1 && value != 2) return fail("bad two-step layout");
    F->tb_px = value;
  } else if (which == 9) {  // most own columns of a two-step item (0: TB_OXW = 124)
    if (value != 0 && (value < 4 || value > TB_OXW)) return fail("bad two-step width");
    F->tb_ox = value;
    F->tb_ox_set = value != 0;  // the tuner keeps a width that was set
  } else if (which == 8) {  // planes per two-step item (0: automatic)
    if (value < 0 || value > 4096) return fail("bad two-step chunk");
    F->tb_zchunk = value;
  } else if (which == 6) {  // planes per rim item (0: the one-step chunk length)
    if (value < 0 || value > FUSED_MAXCH) return fail("bad rim chunk");
    F->rim_zchunk = value;
  } else if (which == 1) {
    F->dft_pal = v;
    for (auto &o : F->dfts) o->plan_key = -1;  // plans rebuilt at the next update
  } else {
    return fail("bad schedule option");
  }
  F->tb_sig = 0;  // the pair plan is rebuilt at the next batch
  return 0;
}

int mnl_fields_tb_info(mnl_fields *F, double *out, int n) {
  if (!F || !out || n < 1) return fail("bad argument");
  const double v[15] = {F->fused && F->tb_have && F->tb_enabled && F->tb_last ? 1.0 : 0.0,
                       F->tb_cells,
                       F->tb_border,
                       F->tb_cells_nu,
                       F->rim_cells,
                       F->rim_cells_nu,
                       double(F->tb_items.size()),
                       double(F->tb_ritems.size() / 2),
                       F->tb_items.empty() ? 0.0 : double((F->tb_items[0].z >> 16) -
                                                          (F->tb_items[0].z & 0xFFFF)),
                       double(F->tb_nnarrow),
                       F->tb_enabled ? 1.0 : 0.0,
                       double(F->tb_zchunk),  // the setting (0: automatic)
                       double(F->tb_ox ? F->tb_ox : TB_OXW),  // most own columns of an item
                       F->tb_pol ? 1.0 : 0.0,  // polarization chunks stepped inside the pairs
                       double(F->tb_nint)};  // interior two-step items (first in the list)
  for (int i = 0; i < n && i < 15; i++) out[i] = v[i];
  return 0;
}

int mnl_fields_mode(mnl_fields *F, int *fused) {
  if (!F) return fail("null fields");
  *fused = (F->fused ? 1 : 0) | (F->fused && F->d_uidx ? 2 : 0) | (F->contig ? 4 : 0) |
           (F->fused && F->tile_mode ? 16 : 0) | (F->fused && F->fused_concurrent ? 32 : 0) |
           (std::min(F->contig_fallbacks, 255) << 8);
  return 0;
}

// fields::get_dft_array(dft_flux / dft_fields, c, num_freq) (src/dft.cpp:1240-1280):
// process_dft_component into a whole array (get_dft_component_dims corners; every
// chunk of c in list order; dft / stored_weight, divided by the loop weight when the
// chunk stored it; times the interpolation weights of the empty dimensions,
// src/dft.cpp:908-1040), summed over ranks (sum_to_all: one owner per point), then
// collapse_array (src/array_slice.cpp:554-601).  out: re/im interleaved.
static int dft_array_values(mnl_fields *F, int h, int c, int num_freq, int *rank,
                            long long dims[3], double *out, long long nout) {
  if (h < 0 || h >= (int)F->dfts.size()) return fail("bad dft handle");
  DftFluxH &o = *F->dfts[h];
  if (dft_flush(F, o)) return -1;  // the buffered updates first
  if (num_freq < 0 || num_freq > o.nfreq - 1)
    return fail(("process_dft_component: frequency index " + std::to_string(num_freq) +
                 " is outside the range of the frequency array of size " +
                 std::to_string(o.nfreq)).c_str());
  const mnl_structure &S = F->S;
  std::vector<const DftChunkH *> L;
  for (auto &dc : o.E)
    if (dc.c == c) L.push_back(&dc);
  for (auto &dc : o.H)
    if (dc.c == c) L.push_back(&dc);
  int mn[3] = {INT32_MAX, INT32_MAX, INT32_MAX}, mx[3] = {INT32_MIN, INT32_MIN, INT32_MIN};
  for (auto *dc : L)
    for (int d = 0; d < 3; d++) mn[d] = std::min(mn[d], dc->is[d]), mx[d] = std::max(mx[d], dc->ie[d]);
  int r = 0, ds[3] = {0, 0, 0};
  long long full[3] = {1, 1, 1};
  if (!L.empty())
    for (int d = 0; d < 3; d++) {
      if (!S.has[d]) continue;
      long long n = (mx[d] - mn[d]) / 2 + 1;
      if (n > 1) ds[r] = d, full[r++] = n;
    }
  int rr = 0;  // collapse_array: directions empty in `where` are summed out
  long long rd[3] = {1, 1, 1};
  for (int k = 0; k < r; k++)
    if (o.wmax[ds[k]] - o.wmin[ds[k]] != 0.0) rd[rr++] = full[k];
  *rank = rr;
  for (int k = 0; k < 3; k++) dims[k] = k < rr ? rd[k] : 1;
  if (!out) return 0;
  long long rs[3] = {0, 0, 0}, nred = 1;
  for (int k = r - 1; k >= 0; k--)
    if (o.wmax[ds[k]] - o.wmin[ds[k]] != 0.0) rs[k] = nred, nred *= full[k];
  if (r == 0) nred = 0;
  if (nout < nred) return fail("output buffer too small");
  for (long long k = 0; k < 2 * nred; k++) out[k] = 0.0;
  if (r == 0) return 0;
  const size_t nf = o.nfreq;
  std::vector<double> v(2 * ((o.npts + 63) & ~size_t(63)) * nf);
  bool ok = true;
  if (!v.empty())
    ok = hipMemcpyAsync(v.data(), o.d_dft, v.size() * 8, hipMemcpyDeviceToHost, F->stream) ==
             hipSuccess &&
         hipStreamSynchronize(F->stream) == hipSuccess;
  if (F->nranks > 1 && F->comm->agree_ok(ok, F->stream))  // every rank fails together
    return fail(ok ? "get_dft_array: a rank failed" : "get_dft_array: device copy failed");
  if (!ok) return fail("get_dft_array: device copy failed");
  long long ntot = 1;
  for (int k = 0; k < r; k++) ntot *= full[k];
  std::vector<double> arr(2 * ntot, 0.0);
  bool empty_dim[3];
  for (int d = 0; d < 3; d++) empty_dim[d] = S.has[d] && o.wmax[d] - o.wmin[d] == 0.0;
  const int yd[3] = {S.dim == 2 ? 2 : 0, S.dim == 2 ? 0 : 1, S.dim == 2 ? 1 : 2};
  for (auto *dc : L) {
    int n[3];
    for (int k = 0; k < 3; k++) n[k] = S.has[yd[k]] ? (dc->ie[yd[k]] - dc->is[yd[k]]) / 2 + 1 : 1;
    size_t pidx = 0;  // chunk_idx: points in LOOP_OVER_IVECS order
    for (int i1 = 0; i1 < n[0]; i1++)
      for (int i2 = 0; i2 < n[1]; i2++)
        for (int i3 = 0; i3 < n[2]; i3++, pidx++) {
          const size_t pt = dc->p0 + pidx;
          const int *pj = &o.h_pj[3 * pt];
          if (pj[0] < 0 && pj[1] < 0 && pj[2] < 0) continue;  // another rank's point
          const int ii[3] = {i1, i2, i3};
          int p[3] = {0, 0, 0};
          for (int k = 0; k < 3; k++)
            if (S.has[yd[k]]) p[yd[k]] = dc->is[yd[k]] + 2 * ii[k];
          double wl[3], wi[3];
          for (int k = 0; k < 3; k++) {
            const int d = yd[k];
            wl[k] = loop_w1(dc->s0[d], dc->s1[d], dc->e0[d], dc->e1[d], ii[k], n[k]);
            wi[k] = empty_dim[d] ? wl[k] : loop_w1(1.0, 1.0, 1.0, 1.0, ii[k], n[k]);
          }
          const double w = wl[2] * (wl[1] * ((dc->dV0 + 0.0 * i2) * wl[0]));
          const double interp_w = wi[2] * (wi[1] * (1.0 * wi[0]));
          const size_t q = dft_at(o.slot[pt], num_freq, nf);
          cplx dft_val = cplx(v[2 * q], v[2 * q + 1]) / dc->stored;
          if (dc->incl && dft_val != 0.0) dft_val /= w;
          long long oi = 0;
          for (int k = 0; k < r; k++) oi = oi * full[k] + (p[ds[k]] - mn[ds[k]]) / 2;
          const cplx val = interp_w * dft_val;
          arr[2 * oi] = val.real();
          arr[2 * oi + 1] = val.imag();
        }
  }
  if (F->nranks > 1)
    for (size_t q = 0; q < arr.size(); q += 1 << 20) {
      const int n = (int)std::min<size_t>(1 << 20, arr.size() - q);
      if (timed_allreduce(F, arr.data() + q, n)) return fail("get_dft_array allreduce failed");
    }
  for (long long q = 0; q < ntot; q++) {  // collapse_array, in full-index order
    long long t = q, ri = 0;
    for (int k = r - 1; k >= 0; k--) {
      ri += (t % full[k]) * rs[k];
      t /= full[k];
    }
    out[2 * ri] += arr[2 * q];
    out[2 * ri + 1] += arr[2 * q + 1];
  }
  return 0;
}

int mnl_fields_add_dft_fields(mnl_fields *F, int ncomp, const int *comps, const double vmin[3],
                              const double vmax[3], const double *freqs, int nfreq, int yee_grid,
                              int decimation, int *handle) {
  if (!F || !comps || !vmin || !vmax || !freqs || !handle) return fail("null argument");
  if (decimation < 0) return fail("decimation must be >= 0");
  if (hipSetDevice(F->device) != hipSuccess) return fail("hipSetDevice failed");
  const int h = dft_add_fields(F, ncomp, comps, vmin, vmax, freqs, nfreq, yee_grid, decimation);
  if (h < 0) return -1;
  *handle = h;
  return 0;
}

int mnl_fields_dft_array(mnl_fields *F, int h, int comp, int num_freq, int *rank, long long dims[3],
                         double *out, long long nout) {
  if (!F || !rank || !dims) return fail("null argument");
  return dft_array_values(F, h, comp, num_freq, rank, dims, out, nout);
}

int mnl_fields_add_dft_flux(mnl_fields *F, int nreg, const double *regions, const double *freqs,
                            int nfreq, int decimation, int *handle) {
  if (!F || !regions || !freqs || !handle) return fail("null argument");
  if (decimation < 0) return fail("decimation must be >= 0");
  for (int r = 0; r < nreg; r++)
    if (regions[8 * r + 6] < 0 || regions[8 * r + 6] > 2) return fail("bad flux direction");
  if (hipSetDevice(F->device) != hipSuccess) return fail("hipSetDevice failed");
  const int h = dft_add_flux(F, nreg, regions, freqs, nfreq, decimation);
  if (h < 0) return -1;
  *handle = h;
  return 0;
}

int mnl_fields_dft_flux(mnl_fields *F, int h, double *out) {
  if (!F || !out) return fail("null argument");
  return dft_flux_values(F, h, out);
}

int mnl_fields_dft_size(mnl_fields *F, int h, long long *n) {
  if (!F || !n) return fail("null argument");
  if (h < 0 || h >= (int)F->dfts.size()) return fail("bad dft handle");
  const DftFluxH &o = *F->dfts[h];
  long long k = 0;
  for (auto &dc : o.E) k += (long long)dc.N;
  *n = k * o.nfreq;
  return 0;
}

int mnl_fields_dft_flush(mnl_fields *F) {
  if (!F) return fail("null fields");
  for (auto &o : F->dfts)
    if (dft_flush(F, *o)) return -1;
  HIPCHK(hipStreamSynchronize(F->stream));
  return 0;
}

int mnl_fields_dft_data(mnl_fields *F, int h, int which, double *out, long long n) {
  if (!F || !out) return fail("null argument");
  if (h < 0 || h >= (int)F->dfts.size()) return fail("bad dft handle");
  if (dft_flush(F, *F->dfts[h])) return -1;  // the buffered updates first
  const DftFluxH &o = *F->dfts[h];
  const size_t nf = o.nfreq;
  std::vector<double> v(2 * ((o.npts + 63) & ~size_t(63)) * nf);
  if (!v.empty()) {
    HIPCHK(hipStreamSynchronize(F->stream));
    HIPCHK(hipMemcpy(v.data(), o.d_dft, v.size() * 8, hipMemcpyDeviceToHost));
  }
  long long k = 0;
  for (auto &dc : which ? o.H : o.E)
    for (size_t p = 0; p < dc.N; p++)
      for (size_t i = 0; i < nf; i++) {
        if (k + 2 > 2 * n) return fail("dft buffer too small");
        out[k++] = v[2 * dft_at(o.slot[dc.p0 + p], i, nf)];
        out[k++] = v[2 * dft_at(o.slot[dc.p0 + p], i, nf) + 1];
      }
  return 0;
}

int mnl_fields_dft_decimation(mnl_fields *F, int h, int *decimation) {
  if (!F || !decimation) return fail("null argument");
  if (h < 0 || h >= (int)F->dfts.size()) return fail("bad dft handle");
  *decimation = F->dfts[h]->decim;
  return 0;
}

int mnl_fields_traffic_model(mnl_fields *F, double *bpc, double *cells) {
  if (!F) return fail("null fields");
  // Minimal per-step HBM traffic per interior cell of the kernels in use
  // (DESIGN.md "Roofline"): fused: B, D read+write, chi1inv read;
  // unfused: curl B reads E(3)+B(3), writes B(3); curl D reads H=B(3)+D(3),
  // writes D(3); E update reads D(3) (+chi1inv 3), writes E(3) (+P terms).
  double n = 0;
  for (int d = 0; d < 3; d++) n += F->allocated[d] ? 1 : 0;
  int nu = 0;
  for (int d = 0; d < 3; d++) nu += F->f.inveps[d] ? 1 : 0;
  double b;
  if (F->fused) {  // whole fused step over G per G point (PML state included)
    double lb, gb, gc = 1;
    fused_bytes(F, &lb, &gb);
    for (int e = 0; e < 3; e++) gc *= double(F->fusedG.hi[e] - F->fusedG.lo[e] + 1);
    b = (lb + gb) / gc;
  } else {
    b = 8.0 * (3 * n) * 2 + 8.0 * (2 * n) + 8.0 * nu;
    for (int k = 0; k < F->f.npol; k++)
      for (int d = 0; d < 3; d++)
        if (F->f.pol[k].P[d]) b += 8.0 * 5;
    for (int t = 0; t < 2; t++)  // cnd and cndinv read per conductive component
      for (int d = 0; d < 3; d++)
        if (F->f.cnd[t][d]) b += 8.0 * 2;
  }
  *bpc = b;
  double c = 1;
  for (int d = 0; d < 3; d++)
    if (F->S.has[d]) {
      if (d == F->slab_dir && F->nranks > 1)
        c *= double(F->g.owned_hi_sh[d] - F->g.owned_lo_sh[d] + 1);
      else
        c *= F->S.n[d];
    }
  *cells = c;
  return 0;
}

}  // extern "C"
