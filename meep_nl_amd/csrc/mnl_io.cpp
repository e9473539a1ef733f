// mnl_io.cpp -- checkpoints (fields::dump / load, structure::dump / load), array slices
// (fields::get_array_slice, src/array_slice.cpp) and field energy (fields::field_energy_in_box,
// src/energy_and_flux.cpp) of the MI355X fields (DESIGN.md sections 13, 15, 18).
#include "mnl_host.hpp"

namespace mnlh {

// ------------------------------------------------------------- checkpoint
// fields::dump / fields::load (src/fields_dump.cpp:108-145, 232-270) and
// structure::dump / load (src/structure_dump.cpp).  The reference writes HDF5
// (absent from this image); here a flat binary file per rank: a header (grid,
// decomposition, t) and every per-point state array of the rank -- the
// reference's f, f_u, f_w, f_cond plus the polarizations P / P_prev, which it
// does not save, and the DFT accumulators -- raw in the rank-local device
// layout, so a load into fields built the same way resumes bit for bit.
constexpr char CK_MAGIC[8] = {'M', 'N', 'L', 'F', 'L', 'D', '0', '1'};
constexpr char CS_MAGIC[8] = {'M', 'N', 'L', 'S', 'T', 'R', '0', '1'};


std::vector<CkEntry> ckpt_entries(mnl_fields *F) {
  DevFields &f = F->f;
  std::vector<CkEntry> v;
  auto add = [&](int kind, int a, int b, double *p, size_t n) {
    if (p) v.push_back({kind, a, b, p, n});
  };
  const size_t n = F->nlocal;
  for (int d = 0; d < 3; d++) {
    add(0, d, 0, f.E[d], n);
    add(1, d, 0, f.D[d], n);
    add(2, d, 0, f.B[d], n);
    add(3, d, 0, f.H[d], n);
    add(4, d, 0, f.UB[d], n);
    add(5, d, 0, f.UD[d], n);
    add(6, d, 0, f.WE[d], n);
    add(7, d, 0, f.WH[d], n);
  }
  for (int t = 0; t < 2; t++)
    for (int d = 0; d < 3; d++) add(8, t, d, f.fcnd[t][d], n);
  for (int k = 0; k < f.npol; k++)
    for (int d = 0; d < 3; d++) {
      add(9, k, d, f.pol[k].P[d], n);
      add(10, k, d, f.pol[k].Pp[d], n);
    }
  for (size_t h = 0; h < F->dfts.size(); h++) {
    DftFluxH &o = *F->dfts[h];
    add(11, (int)h, o.nfreq, o.d_dft, 2 * ((o.npts + 63) & ~size_t(63)) * o.nfreq);
  }
  for (int k = 0; k < f.nhpol; k++)  // magnetic polarizations
    for (int d = 0; d < 3; d++) {
      add(12, k, d, f.hpol[k].P[d], n);
      add(13, k, d, f.hpol[k].Pp[d], n);
    }
  return v;
}

struct CkHeader {
  char magic[8];
  int32_t dim, n[3], io[3], nranks, rank, nentries;
  uint64_t nlocal;
  int64_t t;
};

CkHeader ckpt_header(mnl_fields *F, int nentries) {
  CkHeader h{};
  memcpy(h.magic, CK_MAGIC, 8);
  h.dim = F->S.dim;
  for (int d = 0; d < 3; d++) h.n[d] = F->S.n[d], h.io[d] = F->S.io[d];
  h.nranks = F->nranks;
  h.rank = F->rank;
  h.nentries = nentries;
  h.nlocal = F->nlocal;
  h.t = F->t;
  return h;
}

// a consistent unfused state: implicit E and the W aux fields materialised,
// buffered DFT updates accumulated
int ckpt_quiesce(mnl_fields *F) {
  if (set_fused(F, false)) return -1;
  for (auto &op : F->dfts)
    if (dft_flush(F, *op)) return -1;
  HIPCHK(hipStreamSynchronize(F->stream));
  return 0;
}

int fields_dump(mnl_fields *F, const char *path) {
  if (ckpt_quiesce(F)) return -1;
  auto es = ckpt_entries(F);
  FILE *fp = fopen(path, "wb");
  if (!fp) return fail(std::string("cannot create fields output file ") + path);
  std::unique_ptr<FILE, int (*)(FILE *)> guard(fp, fclose);
  CkHeader h = ckpt_header(F, (int)es.size());
  if (fwrite(&h, sizeof h, 1, fp) != 1) return fail("write error");
  std::vector<double> buf;
  for (auto &e : es) {
    int32_t id[3] = {e.kind, e.a, e.b};
    uint64_t n = e.n;
    buf.resize(e.n);
    HIPCHK(hipMemcpy(buf.data(), e.p, e.n * 8, hipMemcpyDeviceToHost));
    if (fwrite(id, sizeof id, 1, fp) != 1 || fwrite(&n, 8, 1, fp) != 1 ||
        fwrite(buf.data(), 8, e.n, fp) != e.n)
      return fail("write error");
  }
  return 0;
}

int fields_load(mnl_fields *F, const char *path) {
  if (F->src_dirty && build_source_lists(F)) return -1;
  if (ckpt_quiesce(F)) return -1;
  FILE *fp = fopen(path, "rb");
  if (!fp) return fail(std::string("cannot open fields file ") + path);
  std::unique_ptr<FILE, int (*)(FILE *)> guard(fp, fclose);
  CkHeader h{};
  if (fread(&h, sizeof h, 1, fp) != 1 || memcmp(h.magic, CK_MAGIC, 8))
    return fail("not a fields checkpoint file");
  auto es = ckpt_entries(F);
  CkHeader me = ckpt_header(F, (int)es.size());
  if (h.dim != me.dim || memcmp(h.n, me.n, sizeof h.n) || memcmp(h.io, me.io, sizeof h.io) ||
      h.nranks != me.nranks || h.rank != me.rank || h.nlocal != me.nlocal)
    return fail("fields file has a different grid or chunk layout");
  // every field-state array must match; DFT accumulators are loaded into the
  // flux objects that exist (same creation order), extra ones are skipped
  size_t nfield = 0, matched = 0;
  for (auto &e : es) nfield += e.kind != 11;
  std::vector<double> buf;
  for (int k = 0; k < h.nentries; k++) {
    int32_t id[3];
    uint64_t n;
    if (fread(id, sizeof id, 1, fp) != 1 || fread(&n, 8, 1, fp) != 1) return fail("read error");
    const CkEntry *dst = nullptr;
    for (auto &e : es)
      if (e.kind == id[0] && e.a == id[1] && e.b == id[2]) dst = &e;
    if (!dst && id[0] != 11)
      return fail("fields file does not match these fields (allocated arrays differ)");
    if (dst && dst->n != n) return fail("fields file does not match these fields (array sizes differ)");
    buf.resize(n);
    if (fread(buf.data(), 8, n, fp) != n) return fail("read error (truncated file)");
    if (!dst) continue;
    HIPCHK(hipMemcpy(dst->p, buf.data(), n * 8, hipMemcpyHostToDevice));
    matched += dst->kind != 11;
  }
  if (matched != nfield) return fail("fields file does not match these fields (allocated arrays differ)");
  F->t = h.t;
  // the loaded state comes from fields that were stepped: H and the W fields are
  // already separate (a dump taken before the first step holds zeros in them)
  F->e_first_done = F->h_first_done = true;
  F->u_first_done[0] = F->u_first_done[1] = true;
  return 0;
}

template <class T>
void put(std::string &o, const T &v) {
  o.append(reinterpret_cast<const char *>(&v), sizeof v);
}
void put_vec(std::string &o, const std::vector<double> &v) {
  put(o, (uint64_t)v.size());
  o.append(reinterpret_cast<const char *>(v.data()), v.size() * 8);
}
struct Rd {
  const std::string &s;
  size_t i = 0;
  bool ok = true;
  template <class T>
  void get(T &v) {
    if (i + sizeof v > s.size()) {
      ok = false;
      return;
    }
    memcpy(&v, s.data() + i, sizeof v);
    i += sizeof v;
  }
  void get_vec(std::vector<double> &v) {
    uint64_t n = 0;
    get(n);
    if (!ok || i + n * 8 > s.size()) {
      ok = false;
      return;
    }
    v.resize(n);
    memcpy(v.data(), s.data() + i, n * 8);
    i += n * 8;
  }
};

int structure_dump(const mnl_structure *S, const char *path) {
  std::string o(CS_MAGIC, 8);
  put(o, S->dim);
  for (int d = 0; d < 3; d++) put(o, S->n[d]), put(o, S->io[d]);
  put(o, S->a), put(o, S->courant), put(o, S->nl_mode);
  for (int d = 0; d < 3; d++)
    for (int e = 0; e < 2; e++) put(o, S->pml_thick[d][e]), put(o, S->pml_R[d][e]), put(o, S->pml_stretch[d][e]);
  for (int c = 0; c < 3; c++)
    for (int d = 0; d < 3; d++) put_vec(o, S->chi1inv[c][d]);
  for (int c = 0; c < 3; c++) put_vec(o, S->chi2[c]), put_vec(o, S->chi3[c]);
  for (int t = 0; t < 2; t++)
    for (int d = 0; d < 3; d++) put_vec(o, S->cond[t][d]);
  put(o, (uint64_t)S->lor.size());
  for (auto &L : S->lor) {
    put(o, L.omega0), put(o, L.gamma), put(o, L.drude);
    for (int d = 0; d < 3; d++) put_vec(o, L.sigma[d]);
    for (int c = 0; c < 3; c++)
      for (int d = 0; d < 3; d++) put_vec(o, L.off[c][d]);
  }
  put(o, (uint64_t)S->boxes.size());
  for (auto &b : S->boxes) put(o, b);
  bool hside = !S->hlor.empty();  // optional H-side section (absent in older files)
  for (int c = 0; c < 3; c++)
    for (int d = 0; d < 3; d++) hside = hside || !S->mu1inv[c][d].empty();
  if (hside) {
    put(o, (uint64_t)0x4853494445ull);  // "HSIDE"
    for (int c = 0; c < 3; c++)
      for (int d = 0; d < 3; d++) put_vec(o, S->mu1inv[c][d]);
    put(o, (uint64_t)S->hlor.size());
    for (auto &L : S->hlor) {
      put(o, L.omega0), put(o, L.gamma), put(o, L.drude);
      for (int d = 0; d < 3; d++) put_vec(o, L.sigma[d]);
    }
  }
  FILE *fp = fopen(path, "wb");
  if (!fp) return fail(std::string("cannot create structure output file ") + path);
  size_t w = fwrite(o.data(), 1, o.size(), fp);
  fclose(fp);
  return w == o.size() ? 0 : fail("write error");
}

int structure_load(mnl_structure *S, const char *path) {
  FILE *fp = fopen(path, "rb");
  if (!fp) return fail(std::string("cannot open structure file ") + path);
  std::string s;
  char buf[1 << 16];
  size_t r;
  while ((r = fread(buf, 1, sizeof buf, fp)) > 0) s.append(buf, r);
  fclose(fp);
  if (s.size() < 8 || memcmp(s.data(), CS_MAGIC, 8)) return fail("not a structure file");
  Rd in{s, 8};
  int dim = 0, n[3] = {0, 0, 0}, io[3] = {0, 0, 0};
  in.get(dim);
  for (int d = 0; d < 3; d++) in.get(n[d]), in.get(io[d]);
  double a = 0, courant = 0;
  in.get(a), in.get(courant);
  if (!in.ok || dim != S->dim || memcmp(n, S->n, sizeof n) || memcmp(io, S->io, sizeof io) ||
      a != S->a || courant != S->courant)
    return fail("structure file has a different grid volume");
  mnl_structure T = *S;
  in.get(T.nl_mode);
  for (int d = 0; d < 3; d++)
    for (int e = 0; e < 2; e++) in.get(T.pml_thick[d][e]), in.get(T.pml_R[d][e]), in.get(T.pml_stretch[d][e]);
  for (int c = 0; c < 3; c++)
    for (int d = 0; d < 3; d++) in.get_vec(T.chi1inv[c][d]);
  for (int c = 0; c < 3; c++) in.get_vec(T.chi2[c]), in.get_vec(T.chi3[c]);
  for (int t = 0; t < 2; t++)
    for (int d = 0; d < 3; d++) in.get_vec(T.cond[t][d]);
  uint64_t nl = 0;
  in.get(nl);
  T.lor.assign(in.ok && nl < 1024 ? nl : 0, Lorentz{});
  for (auto &L : T.lor) {
    in.get(L.omega0), in.get(L.gamma), in.get(L.drude);
    for (int d = 0; d < 3; d++) in.get_vec(L.sigma[d]);
    for (int c = 0; c < 3; c++)
      for (int d = 0; d < 3; d++) in.get_vec(L.off[c][d]);
  }
  uint64_t nb = 0;
  in.get(nb);
  T.boxes.assign(in.ok && nb < (1u << 20) ? nb : 0, BoxSpec{});
  for (auto &b : T.boxes) in.get(b);
  for (int c = 0; c < 3; c++)
    for (int d = 0; d < 3; d++) T.mu1inv[c][d].clear();
  T.hlor.clear();
  if (in.ok && in.i < s.size()) {  // H-side section
    uint64_t tag = 0, nh = 0;
    in.get(tag);
    if (tag != 0x4853494445ull) in.ok = false;
    for (int c = 0; c < 3; c++)
      for (int d = 0; d < 3; d++) in.get_vec(T.mu1inv[c][d]);
    in.get(nh);
    T.hlor.assign(in.ok && nh <= (uint64_t)MAX_HPOL ? nh : 0, Lorentz{});
    for (auto &L : T.hlor) {
      in.get(L.omega0), in.get(L.gamma), in.get(L.drude);
      for (int d = 0; d < 3; d++) in.get_vec(L.sigma[d]);
    }
  }
  if (!in.ok || in.i != s.size()) return fail("structure file is truncated or corrupt");
  bool sizes_ok = true;  // every per-point array is absent or whole-cell
  auto chk = [&](const std::vector<double> &v) { sizes_ok = sizes_ok && (v.empty() || v.size() == T.ntot); };
  for (int c = 0; c < 3; c++) {
    for (int d = 0; d < 3; d++) chk(T.chi1inv[c][d]);
    chk(T.chi2[c]), chk(T.chi3[c]);
  }
  for (int t = 0; t < 2; t++)
    for (int d = 0; d < 3; d++) chk(T.cond[t][d]);
  for (auto &L : T.lor) {
    for (int d = 0; d < 3; d++) chk(L.sigma[d]);
    for (int c = 0; c < 3; c++)
      for (int d = 0; d < 3; d++) chk(L.off[c][d]);
  }
  for (int c = 0; c < 3; c++)
    for (int d = 0; d < 3; d++) chk(T.mu1inv[c][d]);
  for (auto &L : T.hlor)
    for (int d = 0; d < 3; d++) chk(L.sigma[d]);
  if (!sizes_ok) return fail("structure file holds an array of the wrong size");
  *S = std::move(T);
  return 0;
}

// ------------------------------------------------------------- array slices
// H-side materials: H_d separate in the reference chunk holding the point at absolute
// half-coordinates p (not counting PML along d; DevFields::hsep_zone / hsep_all)
bool h_sep_zone(const mnl_fields *F, const int p[3], int d) {
  if (!F->hall || !F->h_first_done) return false;
  if (F->f.hsep_all) return true;
  int zb = 0;
  for (int e = 0; e < 3; e++)
    zb = zb * 3 + (F->S.has[e] ? F->h_zone[e][p[e] - F->S.io[e]] : 1);
  return (F->h_hsep_zone[zb] >> d) & 1;
}

// fields::get_array_slice(volume, c) for real fields without symmetry
// (src/array_slice.cpp:251-433, 447-507, 525-601, 611-704): loop_in_chunks over
// the Centered grid in the reference's chunks, each point the average of the
// component's four Yee neighbours (yee2cent_offsets, src/vec.cpp:333-344)
// times the interpolation weights of the empty dimensions only
// (IVEC_LOOP_WEIGHT with s0i..e1i, src/meep/vec.hpp:372-383), then the empty
// dimensions collapsed by summation (collapse_array, snap = false).  Host-side
// from the whole-cell component array, as the reference's CPU loop.

// This rank's entries of component c inside the whole-cell index box lo..hi
// (global indices per direction) into out (strides hs, zero elsewhere).
int copy_component_box(mnl_fields *F, int c, const int lo[3], const int hi[3],
                       const long long hs[3], double *out) {
  const mnl_structure &S = F->S;
  long long n = 1;
  for (int d = 0; d < 3; d++)
    if (S.has[d]) n *= hi[d] - lo[d] + 1;
  if (n <= 0) return 0;
  memset(out, 0, (size_t)n * sizeof(double));
  if (!has_field(S, c) || !F->allocated[c]) return 0;
  const int t = ctype(c), d = cdir(c);
  const double *src = t == T_E ? F->f.E[d] : t == T_D ? F->f.D[d] : F->f.B[d];
  const double *hsep = (t == T_H && !(F->hall && !F->h_first_done)) ? F->f.H[d] : nullptr;
  if (!src) return 0;
  if (hipSetDevice(F->device) != hipSuccess) return fail("hipSetDevice failed");
  double *buf = nullptr;
  HIPCHK(hipMalloc(&buf, (size_t)n * sizeof(double)));
  std::unique_ptr<void, void (*)(void *)> guard(buf, [](void *p) { (void)hipFree(p); });
  HIPCHK(hipMemsetAsync(buf, 0, (size_t)n * sizeof(double), F->stream));
  const bool fe = F->fused && t == T_E;
  if (k_to_box(buf, src, hsep, F->g, t, d, F->f, fe ? &F->fusedG : nullptr, fe ? F->f.D[d] : nullptr,
               fe ? F->f.inveps[d] : nullptr, lo, hi, hs, F->stream))
    return fail("to_box launch failed");
  HIPCHK(hipMemcpyAsync(out, buf, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, F->stream));
  HIPCHK(hipStreamSynchronize(F->stream));
  return 0;
}

// Diagonal chi1inv of E (t = T_E, epsilon) or H (mu) component k at global index j, as
// structure_chunk::get_chi1inv_at_pt returns it (src/structure.cpp; 1 where the row is
// absent or was deleted as trivial): the host arrays, then the epsilon boxes rasterised
// exactly as box_fill_kernel does (later boxes win).
double mat_diag_at(const mnl_structure &S, int t, int k, const int j[3]) {
  const auto &v = t == T_E ? S.chi1inv[k][k] : S.mu1inv[k][k];
  long long idx = 0;
  for (int d = 0; d < 3; d++) idx += (long long)j[d] * S.cstride(d);
  double val = v.empty() ? 1.0 : v[idx];
  if (t == T_E)
    for (const BoxSpec &b : S.boxes) {
      if (b.kind != 0) continue;
      bool in = true;
      for (int d = 0; d < 3 && in; d++) {
        if (!S.has[d]) continue;
        const double pos = (S.io[d] + 2 * j[d] + S.shift(k, d)) * (0.5 * (1.0 / S.a));
        in = !(pos < b.box[2 * d] || pos > b.box[2 * d + 1]);
      }
      if (in) val = 1.0 / b.value;
    }
  return val;
}

int array_slice(mnl_fields *F, int c, const double vmin[3], const double vmax[3], int snap,
                int *rank, long long dims[3], double *out, long long nout) {
  const mnl_structure &S = F->S;
  int is[3] = {0, 0, 0}, ie[3] = {0, 0, 0};
  for (int d = 0; d < 3; d++) {
    if (!S.has[d]) continue;
    is[d] = 1 + 2 * int(floor(vmin[d] * S.a - .5));
    ie[d] = 1 + 2 * int(ceil(vmax[d] * S.a - .5));
  }
  double s0[3], s1[3], e0[3], e1[3];
  dft_boundary_weights(S, vmin, vmax, is, ie, s0, e0, s1, e1);
  if (snap)  // snap_empty_dimensions (src/loop_in_chunks.cpp:275-287): nearest point, weight 1
    for (int d = 0; d < 3; d++) {
      if (!S.has[d] || vmin[d] != vmax[d] || ie[d] >= is[d] + 4) continue;
      const double w0 = 1. - vmin[d] * S.a + 0.5 * is[d], w1 = 1. + vmax[d] * S.a - 0.5 * ie[d];
      if (w0 > w1)
        ie[d] = is[d];
      else
        is[d] = ie[d];
      s0[d] = s1[d] = e0[d] = e1[d] = 1.0;
    }
  struct Lp {
    int is[3], ie[3];
    double s0[3], s1[3], e0[3], e1[3];
  };
  std::vector<Lp> loops;
  for (auto &ch : reference_chunks(S)) {
    Lp L;
    bool emp = false;
    for (int d = 0; d < 3; d++) {
      L.s0[d] = L.s1[d] = L.e0[d] = L.e1[d] = 1.0;
      if (!S.has[d]) {
        L.is[d] = L.ie[d] = 0;
        continue;
      }
      const int uoc = S.io[d] + 1, coc = ch[d] + 1, cbo = ch[d] + 2 * ch[3 + d] - 1;
      const int iscoS = std::max(uoc, std::min(coc, cbo)), iecoS = std::max(coc, cbo);
      L.is[d] = std::max(is[d], iscoS);
      L.ie[d] = std::min(ie[d], iecoS);
      if (L.is[d] > L.ie[d]) emp = true;
    }
    if (emp) continue;
    for (int d = 0; d < 3; d++) {  // per-chunk weights (loop_in_chunks.cpp:430-470)
      if (!S.has[d]) continue;
      if (L.is[d] == is[d]) {
        L.s0[d] = s0[d];
        L.s1[d] = s1[d];
      } else if (L.is[d] == is[d] + 2) {
        L.s0[d] = s1[d];
      }
      if (L.ie[d] == ie[d]) {
        L.e0[d] = e0[d];
        L.e1[d] = e1[d];
      } else if (L.ie[d] == ie[d] - 2) {
        L.e0[d] = e1[d];
      }
      if (L.ie[d] == L.is[d]) {
        double w = std::min(L.s0[d], L.e0[d]);
        L.s0[d] = L.e0[d] = L.s1[d] = L.e1[d] = w;
      } else if (L.ie[d] == L.is[d] + 2) {
        double w = std::min(L.s0[d], L.e1[d]);
        L.s0[d] = w, L.e1[d] = w;
        w = std::min(L.s1[d], L.e0[d]);
        L.s1[d] = w, L.e0[d] = w;
      } else if (L.ie[d] == L.is[d] + 4) {
        double w = std::min(L.s1[d], L.e1[d]);
        L.s1[d] = w, L.e1[d] = w;
      }
    }
    loops.push_back(L);
  }
  // get_array_slice_dimensions: corners over all chunks, directions with n > 1
  int mn[3] = {INT32_MAX, INT32_MAX, INT32_MAX}, mx[3] = {INT32_MIN, INT32_MIN, INT32_MIN};
  for (auto &L : loops)
    for (int d = 0; d < 3; d++) mn[d] = std::min(mn[d], L.is[d]), mx[d] = std::max(mx[d], L.ie[d]);
  int r = 0, ds[3] = {0, 0, 0};
  long long full[3] = {1, 1, 1};
  if (!loops.empty())
    for (int d = 0; d < 3; d++) {
      if (!S.has[d]) continue;
      long long n = (mx[d] - mn[d]) / 2 + 1;
      if (n > 1) ds[r] = d, full[r++] = n;
    }
  int rr = 0;
  long long rd[3] = {1, 1, 1};
  for (int k = 0; k < r; k++)
    if (vmax[ds[k]] - vmin[ds[k]] != 0.0) rd[rr++] = full[k];
  *rank = rr;
  for (int k = 0; k < 3; k++) dims[k] = k < rr ? rd[k] : 1;
  if (!out) return 0;
  long long rs[3] = {0, 0, 0}, nred = 1;
  for (int k = r - 1; k >= 0; k--)
    if (vmax[ds[k]] - vmin[ds[k]] != 0.0) rs[k] = nred, nred *= full[k];
  if (nout < nred) return fail("output buffer too small");
  for (long long k = 0; k < nred; k++) out[k] = 0.0;
  if (loops.empty()) return 0;
  long long ntot = 1;
  for (int k = 0; k < r; k++) ntot *= full[k];
  std::vector<double> arr(ntot, 0.0);
  if (c == MNL_DIELECTRIC || c == MNL_PERMEABILITY) {
    // Dielectric / Permeability (src/array_slice.cpp:385-408, 649-676): per centred point
    // (4 n) / sum over the n E (H) components of the grid of the four diagonal chi1inv
    // values at the component's yee2cent points, times the empty-dimension weights;
    // from the host structure every rank holds (no device access, no collective)
    const int t = c == MNL_DIELECTRIC ? T_E : T_H;
    std::vector<int> ks;
    for (int k = 0; k < 3; k++)
      if (has_field(S, 3 * t + k)) ks.push_back(k);
    bool empty_dim[3];
    for (int d = 0; d < 3; d++) empty_dim[d] = S.has[d] && vmax[d] - vmin[d] == 0.0;
    const int yd[3] = {S.dim == 2 ? 2 : 0, S.dim == 2 ? 0 : 1, S.dim == 2 ? 1 : 2};
    for (auto &L : loops) {
      int n[3];
      for (int k = 0; k < 3; k++) n[k] = S.has[yd[k]] ? (L.ie[yd[k]] - L.is[yd[k]]) / 2 + 1 : 1;
      for (int i1 = 0; i1 < n[0]; i1++)
        for (int i2 = 0; i2 < n[1]; i2++)
          for (int i3 = 0; i3 < n[2]; i3++) {
            const int ii[3] = {i1, i2, i3};
            int p[3] = {0, 0, 0};
            for (int k = 0; k < 3; k++)
              if (S.has[yd[k]]) p[yd[k]] = L.is[yd[k]] + 2 * ii[k];
            double w[3];
            for (int k = 0; k < 3; k++) {
              const int d = yd[k];
              w[k] = empty_dim[d] ? loop_w1(L.s0[d], L.s1[d], L.e0[d], L.e1[d], ii[k], n[k])
                                  : loop_w1(1.0, 1.0, 1.0, 1.0, ii[k], n[k]);
            }
            const double wt = w[2] * (w[1] * (1.0 * w[0]));
            cplx tr(0.0, 0.0);
            for (int k : ks) {
              const int ck = 3 * t + k;
              int j0[3] = {0, 0, 0}, o[2] = {-1, -1}, no = 0;
              for (int d = 0; d < 3; d++)
                if (S.has[d]) {
                  j0[d] = (p[d] - S.io[d]) / 2;
                  if (!S.shift(ck, d)) o[no++] = d;
                }
              double v[4];
              for (int q = 0; q < 4; q++) {
                int jq[3] = {j0[0], j0[1], j0[2]};
                if ((q & 1) && o[0] >= 0) jq[o[0]]++;
                if ((q & 2) && o[1] >= 0) jq[o[1]]++;
                v[q] = mat_diag_at(S, t, k, jq);
              }
              tr += v[0] + v[1] + v[2] + v[3];
              if (std::abs(tr) == 0.0) tr += 4.0;
            }
            const cplx val = wt * (4.0 * (double)ks.size()) / tr;
            long long oi = 0;
            for (int k = 0; k < r; k++) oi = oi * full[k] + (p[ds[k]] - mn[ds[k]]) / 2;
            arr[oi] = real(val);
          }
    }
    for (long long q = 0; q < ntot; q++) {  // collapse_array: in full-index order
      long long tq = q, ri = 0;
      for (int k = r - 1; k >= 0; k--) {
        ri += (tq % full[k]) * rs[k];
        tq /= full[k];
      }
      out[ri] += arr[q];
    }
    return 0;
  }
  // c's global indices the slice reads: the base point of each centred point
  // and +1 along c's unshifted directions (the four Yee values, o1 / o2)
  bool unsh[3];
  int blo[3] = {0, 0, 0}, bhi[3] = {0, 0, 0};
  for (int d = 0; d < 3; d++) {
    unsh[d] = S.has[d] && !S.shift(c, d);
    if (!S.has[d]) continue;
    blo[d] = (mn[d] - S.io[d]) / 2;
    bhi[d] = (mx[d] - S.io[d]) / 2 + (unsh[d] ? 1 : 0);
  }
  // Distributed: this rank forms the points whose base value it owns along the
  // slab axis (one owner each), reading its own entries of the box plus, for
  // components unshifted along that axis, the next rank's first owned plane;
  // the finished slice is then summed over ranks (every entry has one
  // contributor, so the sums are exact).  No whole-cell buffers on any rank.
  const bool dist = F->nranks > 1;
  const int sd = F->slab_dir;
  int rlo = 0, rhi = S.n[sd];  // base indices along sd this rank forms
  if (dist) {
    const int lo_cell = F->g.off[sd], hi_cell = lo_cell + F->g.N[F->g.ax[sd]] - 1;
    if (S.shift(c, sd)) {
      rlo = lo_cell;
      rhi = F->rank == F->nranks - 1 ? S.n[sd] : hi_cell - 1;
    } else {
      rlo = F->rank == 0 ? 0 : lo_cell + 1;
      rhi = hi_cell;
    }
  }
  int hlo[3], hhi[3];  // this rank's box of values
  for (int d = 0; d < 3; d++) hlo[d] = blo[d], hhi[d] = bhi[d];
  hlo[sd] = std::max(blo[sd], rlo);
  hhi[sd] = std::min(bhi[sd], rhi + (unsh[sd] ? 1 : 0));
  long long hs[3] = {0, 0, 0}, hn = 1;  // slab axis slowest: a plane of it is contiguous
  for (int d = 2; d >= 0; d--)
    if (S.has[d] && d != sd) {
      hs[d] = hn;
      hn *= std::max(0, hhi[d] - hlo[d] + 1);
    }
  hs[sd] = hn;
  hn *= std::max(0, hhi[sd] - hlo[sd] + 1);
  // B components: a reference chunk without PML along c aliases B to H, so its
  // ghost copy of a neighbour chunk's point holds that chunk's H (the H
  // exchange writes through the alias, src/boundaries.cpp:347-460) -- hbh keeps
  // the H values for those reads
  const bool bq = ctype(c) == T_B;
  std::vector<double> hb, hbh;
  bool ok = true;
  std::string why;
  if (hn > 0) {
    hb.assign(hn, 0.0);
    if (copy_component_box(F, c, hlo, hhi, hs, hb.data())) ok = false, why = g_err;
    if (bq && ok) {
      hbh.assign(hn, 0.0);
      if (copy_component_box(F, 3 * T_H + cdir(c), hlo, hhi, hs, hbh.data()))
        ok = false, why = g_err;
    }
  }
  if (dist) {
    if (F->comm->agree_ok(ok, F->stream)) return fail(ok ? "array slice: a rank failed" : why);
    if (unsh[sd]) {  // the plane above this rank's last base index comes from the next rank
      long long pn = 1;
      for (int d = 0; d < 3; d++)
        if (S.has[d] && d != sd) pn *= bhi[d] - blo[d] + 1;
      const int nv = bq ? 2 : 1;  // B: the H plane too
      std::vector<double> xp((size_t)pn * F->nranks * nv, 0.0);
      const int first = F->g.off[sd] + 1;  // first owned plane (unshifted along sd)
      if (F->rank > 0 && hn > 0 && first >= hlo[sd] && first <= hhi[sd])
        for (int v = 0; v < nv; v++)
          for (long long q = 0; q < pn; q++)
            xp[((size_t)F->rank * nv + v) * pn + q] =
                (v ? hbh : hb)[(size_t)(first - hlo[sd]) * hs[sd] + q];
      for (size_t q = 0; q < xp.size(); q += 1 << 20) {
        const int n = (int)std::min<size_t>(1 << 20, xp.size() - q);
        if (timed_allreduce(F, xp.data() + q, n)) return fail("slice allreduce failed");
      }
      const int top = rhi + 1;
      if (F->rank + 1 < F->nranks && hn > 0 && top >= hlo[sd] && top <= hhi[sd])
        for (int v = 0; v < nv; v++)
          for (long long q = 0; q < pn; q++)
            (v ? hbh : hb)[(size_t)(top - hlo[sd]) * hs[sd] + q] =
                xp[((size_t)(F->rank + 1) * nv + v) * pn + q];
    }
  } else if (!ok) {
    return -1;
  }
  long long o1 = 0, o2 = 0;  // offsets of the unshifted neighbours in hb
  int d1 = -1, d2 = -1;      // and their directions
  for (int d = 0; d < 3; d++)
    if (unsh[d]) {
      if (o1)
        o2 = hs[d], d2 = d;
      else
        o1 = hs[d], d1 = d;
    }
  const int cd = cdir(c);
  bool empty_dim[3];
  for (int d = 0; d < 3; d++) empty_dim[d] = S.has[d] && vmax[d] - vmin[d] == 0.0;
  const int yd[3] = {S.dim == 2 ? 2 : 0, S.dim == 2 ? 0 : 1, S.dim == 2 ? 1 : 2};
  for (auto &L : loops) {
    int n[3];
    for (int k = 0; k < 3; k++) n[k] = S.has[yd[k]] ? (L.ie[yd[k]] - L.is[yd[k]]) / 2 + 1 : 1;
    for (int i1 = 0; i1 < n[0]; i1++)
      for (int i2 = 0; i2 < n[1]; i2++)
        for (int i3 = 0; i3 < n[2]; i3++) {
          const int ii[3] = {i1, i2, i3};
          int p[3] = {0, 0, 0};
          for (int k = 0; k < 3; k++)
            if (S.has[yd[k]]) p[yd[k]] = L.is[yd[k]] + 2 * ii[k];
          const int jb = S.has[sd] ? (p[sd] - S.io[sd]) / 2 : 0;
          if (jb < rlo || jb > rhi) continue;  // another rank forms this point
          double w[3];
          for (int k = 0; k < 3; k++) {
            const int d = yd[k];
            w[k] = empty_dim[d] ? loop_w1(L.s0[d], L.s1[d], L.e0[d], L.e1[d], ii[k], n[k])
                                : loop_w1(1.0, 1.0, 1.0, 1.0, ii[k], n[k]);
          }
          const double wt = w[2] * (w[1] * (1.0 * w[0]));
          long long idx = 0;
          int jb3[3] = {0, 0, 0};
          for (int d = 0; d < 3; d++)
            if (S.has[d]) {
              jb3[d] = (p[d] - S.io[d]) / 2;
              idx += (long long)(jb3[d] - hlo[d]) * hs[d];
            }
          double a4[4] = {hb[idx], hb[idx + o1], hb[idx + o2], hb[idx + o1 + o2]};
          if (bq && F->h_zone[cd][p[cd] - S.io[cd]] == 1 && !h_sep_zone(F, p, cd)) {  // reader chunk aliases B to H
            for (int k = 0; k < 4; k++) {
              int jn[3] = {jb3[0], jb3[1], jb3[2]};
              if ((k & 1) && d1 >= 0) jn[d1]++;
              if ((k & 2) && d2 >= 0) jn[d2]++;
              bool other = false;  // owned by another reference chunk
              for (int d = 0; d < 3; d++)
                if (S.has[d])
                  other = other || F->h_zone[d][2 * jn[d] + S.shift(c, d)] !=
                                       F->h_zone[d][p[d] - S.io[d]];
              if (other) a4[k] = hbh[idx + ((k & 1) ? o1 : 0) + ((k & 2) ? o2 : 0)];
            }
          }
          const double avg = 0.25 * (a4[0] + a4[1] + a4[2] + a4[3]);
          const cplx v = wt * cplx(avg, 0.0) * cplx(1.0, 0.0);
          long long oi = 0;
          for (int k = 0; k < r; k++) oi = oi * full[k] + (p[ds[k]] - mn[ds[k]]) / 2;
          arr[oi] = real(v);
        }
  }
  if (dist)
    for (size_t q = 0; q < arr.size(); q += 1 << 20) {
      const int n = (int)std::min<size_t>(1 << 20, arr.size() - q);
      if (timed_allreduce(F, arr.data() + q, n)) return fail("slice allreduce failed");
    }
  for (long long q = 0; q < ntot; q++) {  // collapse_array: in full-index order
    long long t = q, ri = 0;
    for (int k = r - 1; k >= 0; k--) {
      ri += (t % full[k]) * rs[k];
      t /= full[k];
    }
    out[ri] += arr[q];
  }
  return 0;
}

// ------------------------------------------------------------- field energy
// loop_in_chunks(where, cgrid = component c) (src/loop_in_chunks.cpp:325-520,
// no symmetry / Bloch): the reference chunks' boxes on c's Yee grid with their
// boundary weights, restricted to the points this rank owns; weights tabulated
// per device axis into wtab.
std::vector<EBox> energy_boxes(mnl_fields *F, int c, const double wmin[3], const double wmax[3],
                               std::vector<double> &wtab) {
  const mnl_structure &S = F->S;
  const DevGrid &g = F->g;
  int is[3] = {0, 0, 0}, ie[3] = {0, 0, 0};
  for (int d = 0; d < 3; d++) {
    if (!S.has[d]) continue;
    const int iyc = 1 - S.shift(c, d);        // iyee_shift(Centered) - iyee_shift(c)
    const double yc = iyc * (0.5 / S.a);      // yee_shift(Centered) - yee_shift(c)
    is[d] = 1 + 2 * int(floor((wmin[d] + yc) * S.a - .5)) - iyc;  // vec2diel_floor - iyee_c
    ie[d] = 1 + 2 * int(ceil((wmax[d] + yc) * S.a - .5)) - iyc;
  }
  double s0[3], s1[3], e0[3], e1[3];
  dft_boundary_weights(S, wmin, wmax, is, ie, s0, e0, s1, e1);
  double dV0 = 1.0;
  for (int d = 0; d < 3; d++)
    if (S.has[d] && wmax[d] - wmin[d] > 0.0) dV0 *= 1.0 / S.a;
  int yd[3];
  if (S.dim == 2)
    yd[0] = 2, yd[1] = 0, yd[2] = 1;
  else
    yd[0] = 0, yd[1] = 1, yd[2] = 2;
  std::vector<EBox> out;
  for (auto &ch : reference_chunks(S)) {
    int isc[3], iec[3];
    double s0c[3], s1c[3], e0c[3], e1c[3];
    bool emp = false;
    for (int d = 0; d < 3; d++) {
      s0c[d] = s1c[d] = e0c[d] = e1c[d] = 1.0;
      if (!S.has[d]) {
        isc[d] = iec[d] = 0;
        continue;
      }
      const int sh = S.shift(c, d);
      const int uoc = S.io[d] + 2 - sh, coc = ch[d] + 2 - sh, cbo = ch[d] + 2 * ch[3 + d] - sh;
      const int iscoS = std::max(uoc, std::min(coc, cbo)), iecoS = std::max(coc, cbo);
      isc[d] = std::max(is[d], iscoS);
      iec[d] = std::min(ie[d], iecoS);
      if (isc[d] > iec[d]) emp = true;
    }
    if (emp) continue;
    for (int d = 0; d < 3; d++) {
      if (!S.has[d]) continue;
      if (isc[d] == is[d]) {
        s0c[d] = s0[d];
        s1c[d] = s1[d];
      } else if (isc[d] == is[d] + 2) {
        s0c[d] = s1[d];
      }
      if (iec[d] == ie[d]) {
        e0c[d] = e0[d];
        e1c[d] = e1[d];
      } else if (iec[d] == ie[d] - 2) {
        e0c[d] = e1[d];
      }
      if (iec[d] == isc[d]) {
        double w = std::min(s0c[d], e0c[d]);
        s0c[d] = e0c[d] = s1c[d] = e1c[d] = w;
      } else if (iec[d] == isc[d] + 2) {
        double w = std::min(s0c[d], e1c[d]);
        s0c[d] = w, e1c[d] = w;
        w = std::min(s1c[d], e0c[d]);
        s1c[d] = w, e0c[d] = w;
      } else if (iec[d] == isc[d] + 4) {
        double w = std::min(s1c[d], e1c[d]);
        s1c[d] = w, e1c[d] = w;
      }
    }
    EBox b;
    bool none = false;
    for (int k = 0; k < 3; k++) b.dlo[k] = 0, b.dn[k] = 1, b.wofs[k] = 0, b.yd[k] = yd[k];
    b.dV0 = dV0 + 0.0 * 0;  // dV0 + dV1 * loop_i2 with dV1 = 0
    for (int d = 0; d < 3; d++) {
      if (!S.has[d]) continue;
      const int ax = g.ax[d], sh = S.shift(c, d);
      const long nl = (iec[d] - isc[d]) / 2 + 1;           // chunk loop count
      const int j0 = (isc[d] - S.io[d] - sh) / 2 - g.off[d];  // local index of loop point 0
      const int lo_own = sh ? g.owned_lo_sh[d] : g.owned_lo_un[d];
      const int hi_own = sh ? g.owned_hi_sh[d] : g.owned_hi_un[d];
      int a = std::max(0, lo_own - j0), z = std::min<long>(nl - 1, hi_own - j0);
      if (z < a) {
        none = true;
        break;
      }
      b.dlo[ax] = j0 + a;
      b.dn[ax] = z - a + 1;
      b.wofs[ax] = (long long)wtab.size();
      for (long i = a; i <= z; i++) {
        double w = 1.0;
        if (!(i > 1 && i < nl - 2))
          w = i == 0 ? s0c[d] : (i == 1 ? s1c[d] : i == nl - 1 ? e0c[d] : (i == nl - 2 ? e1c[d] : 1.0));
        wtab.push_back(w);
      }
    }
    if (!none) out.push_back(b);
    else out.push_back(EBox{{0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {yd[0], yd[1], yd[2]}, dV0});
  }
  return out;
}

// real(integrate(2, {A, B}, dot_integrand, where)) over component c's grid:
// per reference chunk a device sum (rounded to double, as the reference adds
// each chunk's long-double sum into a complex<double>), chunks added in order,
// then summed over ranks (sum_to_all)
int integrate_pair(mnl_fields *F, int c, const double *A, const double *Asep, const double *Bv,
                   const double wmin[3], const double wmax[3], double *out) {
  std::vector<double> wtab;
  auto boxes = energy_boxes(F, c, wmin, wmax, wtab);
  std::vector<double> chunk(boxes.size(), 0.0);
  // the local part; a failure is agreed on before the collective so that every
  // rank returns instead of waiting in the allreduce
  const int lrc = [&]() -> int {
    const int NB = 256;
    double *dw = nullptr, *dp = nullptr;
    HIPCHK(hipMalloc(&dw, std::max<size_t>(wtab.size(), 1) * 8));
    std::unique_ptr<void, void (*)(void *)> g1(dw, [](void *p) { (void)hipFree(p); });
    HIPCHK(hipMalloc(&dp, 2 * NB * 8));
    std::unique_ptr<void, void (*)(void *)> g2(dp, [](void *p) { (void)hipFree(p); });
    if (!wtab.empty())
      HIPCHK(hipMemcpyAsync(dw, wtab.data(), wtab.size() * 8, hipMemcpyHostToDevice, F->stream));
    std::vector<double> part(2 * NB);
    for (size_t k = 0; k < boxes.size(); k++) {
      const EBox &b = boxes[k];
      const long long n = (long long)b.dn[0] * b.dn[1] * b.dn[2];
      if (n == 0 || !A || !Bv) continue;
      const int nb = (int)std::min<long long>(NB, (n + 255) / 256);
      if (k_energy(A, Asep, Bv, F->g, F->f, ctype(c), cdir(c), b, dw, dp, nb, F->stream))
        return fail("energy kernel launch failed");
      HIPCHK(hipMemcpyAsync(part.data(), dp, 2 * nb * 8, hipMemcpyDeviceToHost, F->stream));
      HIPCHK(hipStreamSynchronize(F->stream));
      long double acc = 0.0L;
      for (int i = 0; i < nb; i++) acc += (long double)part[2 * i] + (long double)part[2 * i + 1];
      chunk[k] = (double)acc;
    }
    return 0;
  }();
  if (F->nranks > 1) {
    const std::string why = g_err;
    if (F->comm->agree_ok(lrc == 0, F->stream)) return fail(lrc ? why : "energy: a rank failed");
    if (timed_allreduce(F, chunk.data(), (int)chunk.size()))
      return fail("energy allreduce failed");
  } else if (lrc) {
    return -1;
  }
  double sum = 0.0;
  for (double v : chunk) sum += v;
  *out = sum;
  return 0;
}

// fields::field_energy_in_box(c, where) for every E (or H) component, summed
// in long double (electric_energy_in_box / magnetic_energy_in_box,
// src/energy_and_flux.cpp:85-95)
int energy_of_type(mnl_fields *F, int t, const double wmin[3], const double wmax[3], double *out) {
  long double sum = 0.0L;
  const DevFields &f = F->f;
  for (int d = 0; d < 3; d++) {
    const int c = 3 * t + d;
    if (!has_field(F->S, c)) continue;
    double v = 0.0;
    if (t == T_E) {
      if (!F->allocated[c] || !F->allocated[3 * T_D + d]) continue;
      if (integrate_pair(F, c, f.E[d], nullptr, f.D[d], wmin, wmax, &v)) return -1;
    } else {
      if (!F->allocated[3 * T_B + d]) continue;
      const double *hsep = (F->h_first_done && f.H[d]) ? f.H[d] : nullptr;
      if (integrate_pair(F, c, f.B[d], hsep, f.B[d], wmin, wmax, &v)) return -1;
    }
    sum += v * 0.5;
  }
  *out = (double)sum;
  return 0;
}

// synchronize_magnetic_fields (src/energy_and_flux.cpp:146-167): back up B / H
// (and f_u, f_w, f_cond where they exist), take one B half step (step_db(B),
// B sources at time(), step_boundaries, update_eh(H)), average B and H with the
// backups; restore_magnetic_fields (169-178) copies the backups back.
struct MagBackup {
  std::vector<std::pair<double *, double *>> items;  // (field array, backup)
  std::vector<std::pair<double *, double *>> avg;    // averaged with backup
  ~MagBackup() {
    for (auto &it : items) (void)hipFree(it.second);
  }
};

int sync_magnetic(mnl_fields *F, MagBackup &bk) {
  if (F->src_dirty && build_source_lists(F)) return -1;
  if (F->fused && set_fused(F, false)) return -1;
  DevFields &f = F->f;
  const size_t n = F->nlocal;
  auto save = [&](double *p, bool average) -> int {
    if (!p) return 0;
    double *b = nullptr;
    HIPCHK(hipMalloc(&b, n * 8));
    HIPCHK(hipMemcpyAsync(b, p, n * 8, hipMemcpyDeviceToDevice, F->stream));
    bk.items.push_back({p, b});
    if (average) bk.avg.push_back({p, b});
    return 0;
  };
  const bool have_u = F->u_first_done[0], have_h = F->h_first_done;
  for (int d = 0; d < 3; d++) {
    if (!F->allocated[3 * T_B + d]) continue;
    if (save(f.B[d], true)) return -1;
    if (have_u && (save(f.UB[d], false) || save(f.fcnd[0][d], false))) return -1;
    if (have_h && (save(f.H[d], true) || save(f.WH[d], false))) return -1;
  }
  // one B step at time(): step_db(B) + step_source(B) + step_boundaries(B) +
  // update_eh(H) + step_boundaries(H)
  if (F->nranks > 1 && exchange(F, 0)) return fail("E halo exchange failed");
  if (!F->u_first_done[0] && u_lazy_copy(F, 0)) return -1;
  const DevGrid &g = F->g;
  if (k_curl(T_B, F->interior, nullptr, g, f, F->planB, F->S.courant, F->stream) ||
      k_curl(T_B, F->interior, &F->shell_list, g, f, F->planB, F->S.courant, F->stream, false))
    return fail("curl B launch failed");
  const size_t nB = F->srcB_idx.size();
  if (nB) {  // calc_sources(time()) + step_source(B_stuff)
    const double dt = F->dt, time = F->t * dt;
    for (auto &st : F->srcs) st.update(time, dt);
    const size_t ng = F->groups.size();
    std::vector<double> J(2 * ng);
    for (size_t g2 = 0; g2 < ng; g2++) {
      const cplx v = F->srcs[F->groups[g2].st].cur_current;
      J[2 * g2] = real(v), J[2 * g2 + 1] = imag(v);
    }
    double *dv = nullptr;
    HIPCHK(hipMalloc(&dv, J.size() * 8));
    std::unique_ptr<void, void (*)(void *)> gv(dv, [](void *p) { (void)hipFree(p); });
    HIPCHK(hipMemcpyAsync(dv, J.data(), J.size() * 8, hipMemcpyHostToDevice, F->stream));
    if (k_source(T_B, g, f, src_dev(F, 0, dv), 0, F->stream)) return fail("source launch failed");
    HIPCHK(hipStreamSynchronize(F->stream));
  }
  if (!F->h_first_done && h_lazy_copy(F)) return -1;
  if (update_h_any(F, F->shell_list, false)) return -1;  // no update_pols here (reference)
  if (F->nranks > 1 && exchange(F, 1)) return fail("H halo exchange failed");
  for (auto &a : bk.avg)
    if (k_average(a.first, a.second, (long long)n, F->stream)) return fail("average launch failed");
  HIPCHK(hipStreamSynchronize(F->stream));
  return 0;
}

int restore_magnetic(mnl_fields *F, MagBackup &bk) {
  for (auto &it : bk.items)
    HIPCHK(hipMemcpyAsync(it.first, it.second, F->nlocal * 8, hipMemcpyDeviceToDevice, F->stream));
  HIPCHK(hipStreamSynchronize(F->stream));
  return 0;
}

// which: 0 electric_energy_in_box, 1 magnetic_energy_in_box (current B / H),
// 2 field_energy_in_box (electric + magnetic of the synchronized B / H)
int energy_in_box(mnl_fields *F, int which, const double wmin[3], const double wmax[3],
                  double *out) {
  if (F->fused && set_fused(F, false)) return -1;  // materialise implicit E
  if (which == 0) return energy_of_type(F, T_E, wmin, wmax, out);
  if (which == 1) return energy_of_type(F, T_H, wmin, wmax, out);
  MagBackup bk;
  double mag = 0.0, el = 0.0;
  if (sync_magnetic(F, bk)) return -1;
  const int r = energy_of_type(F, T_H, wmin, wmax, &mag);
  if (restore_magnetic(F, bk) || r) return -1;
  if (energy_of_type(F, T_E, wmin, wmax, &el)) return -1;
  *out = el + mag;
  return 0;
}

// fields::step() n times: the NaN guard (src/step.cpp:138-139) after every nan_every-th
// step (default every step; counted across calls) on the device, its flag read at the end of
// each batch; the first step after construction (or after E / H were set directly) runs
// unfused (see e_first_done)


// sum_to_all over the fields' ranks, timed as all-all communication
int timed_allreduce(mnl_fields *F, double *v, int n) {
  const double t0 = wall_now();
  const int r = F->comm->allreduce_sum(v, n, F->stream);
  F->sink_s[MNL_SINK_MPI_ALL] += wall_now() - t0;
  return r;
}

}  // namespace mnlh
