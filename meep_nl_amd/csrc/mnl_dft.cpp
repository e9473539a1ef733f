// mnl_dft.cpp -- DFT monitors (fields::add_dft_flux / add_dft_fields / update_dfts,
// src/dft.cpp:195-300, src/loop_in_chunks.cpp:257-500): the reference's chunk loop over a
// region, the device point lists, the per-batch phases, the sampling plan and the buffered
// accumulation.
#include "mnl_host.hpp"

namespace mnlh {


// complex slot of (device slot, frequency) in the wave-blocked DFT array

// compute_boundary_weights (src/loop_in_chunks.cpp:257-300), snap_empty_dimensions = false
void dft_boundary_weights(const mnl_structure &S, const double wmin[3], const double wmax[3],
                          const int is[3], const int ie[3], double s0[3], double e0[3],
                          double s1[3], double e1[3]) {
  for (int d = 0; d < 3; d++) {
    s0[d] = s1[d] = e0[d] = e1[d] = 1.0;
    if (!S.has[d]) continue;
    double w0 = 1. - wmin[d] * S.a + 0.5 * is[d];
    double w1 = 1. + wmax[d] * S.a - 0.5 * ie[d];
    if (ie[d] >= is[d] + 3 * 2) {
      s0[d] = w0 * w0 / 2;
      s1[d] = 1 - (1 - w0) * (1 - w0) / 2;
      e0[d] = w1 * w1 / 2;
      e1[d] = 1 - (1 - w1) * (1 - w1) / 2;
    } else if (ie[d] == is[d] + 2 * 2) {
      s0[d] = w0 * w0 / 2;
      s1[d] = 1 - (1 - w0) * (1 - w0) / 2 - (1 - w1) * (1 - w1) / 2;
      e0[d] = w1 * w1 / 2;
      e1[d] = s1[d];
    } else if (wmin[d] == wmax[d]) {
      s0[d] = w0;
      s1[d] = w1;
      e0[d] = w1;
      e1[d] = w0;
    } else if (ie[d] == is[d] + 1 * 2) {
      s0[d] = w0 * w0 / 2 - (1 - w1) * (1 - w1) / 2;
      e0[d] = w1 * w1 / 2 - (1 - w0) * (1 - w0) / 2;
      s1[d] = e0[d];
      e1[d] = s0[d];
    }
  }
}

// the reference's chunks in creation order: x zones outer, then y, then z
// (absolute little corner io and cell counts n per direction)
std::vector<std::array<int, 6>> reference_chunks(const mnl_structure &S) {
  std::vector<std::pair<int, int>> iv[3];
  for (int d = 0; d < 3; d++) {
    if (!S.has[d]) {
      iv[d].push_back({0, 0});
      continue;
    }
    for (auto &z : zone_intervals(S, d)) iv[d].push_back({S.io[d] + z.c0, (z.c1 - z.c0) / 2});
  }
  std::vector<std::array<int, 6>> out;
  for (auto &ix : iv[0])
    for (auto &iy : iv[1])
      for (auto &iz : iv[2]) out.push_back({ix.first, iy.first, iz.first, ix.second, iy.second, iz.second});
  return out;
}

// fields::add_dft for component c over [wmin, wmax]: the chunks loop_in_chunks
// creates, prepended to `list` (their points appended to the flux object's point
// arrays).  Centered grid, or with yee the component's own grid (loop_in_chunks(...,
// cgrid = c), src/loop_in_chunks.cpp:350-356: where shifted by yee_shift(Centered) -
// yee_shift(c), rounded to the dielectric grid, shifted back by iyee_c).
void dft_add(mnl_fields *F, DftFluxH &o, int c, const double wmin[3], const double wmax[3],
             bool incl, cplx stored_weight, double dt_factor, std::vector<DftChunkH> &list,
             std::vector<double> &pw, bool yee = false) {
  const mnl_structure &S = F->S;
  const DevGrid &g = F->g;
  int is[3] = {0, 0, 0}, ie[3] = {0, 0, 0}, sh[3] = {1, 1, 1};
  for (int d = 0; d < 3; d++) {
    if (!S.has[d]) continue;
    if (yee) sh[d] = S.shift(c, d);
    const int iyc = 1 - sh[d];                                          // iyee_c
    const double yc = 1 * (0.5 * (1.0 / S.a)) - sh[d] * (0.5 * (1.0 / S.a));  // yee_c
    is[d] = 1 + 2 * int(floor((wmin[d] + yc) * S.a - .5)) - iyc;  // vec2diel_floor, equal_shift 0
    ie[d] = 1 + 2 * int(ceil((wmax[d] + yc) * S.a - .5)) - iyc;
  }
  double s0[3], s1[3], e0[3], e1[3];
  dft_boundary_weights(S, wmin, wmax, is, ie, s0, e0, s1, e1);
  double dV0 = 1.0;
  for (int d = 0; d < 3; d++)
    if (S.has[d] && wmax[d] - wmin[d] > 0.0) dV0 *= 1.0 / S.a;
  if (!F->allocated[c]) return;
  int yd[3];  // yucky loop directions (3D: X,Y,Z; 2D: Z,X,Y; 1D: X,Y,Z)
  if (S.dim == 2)
    yd[0] = 2, yd[1] = 0, yd[2] = 1;
  else
    yd[0] = 0, yd[1] = 1, yd[2] = 2;
  std::vector<DftChunkH> made;
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
      // little_owned_corner(cgrid) = io + 2 - iyee_shift, big_owned_corner = big - iyee_shift
      const int uoc = S.io[d] + 2 - sh[d], coc = ch[d] + 2 - sh[d],
                cbo = ch[d] + 2 * ch[3 + d] - sh[d];
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
    DftChunkH dc;
    dc.c = c;
    dc.scale = stored_weight * cplx(1.0) * dt_factor;
    int nun = 0;
    for (int d = 0; d < 3; d++)
      if (!yee && S.has[d] && !S.shift(c, d)) nun++;
    dc.avgmode = nun;
    for (int d = 0; d < 3; d++) {
      dc.is[d] = isc[d], dc.ie[d] = iec[d];
      dc.s0[d] = s0c[d], dc.s1[d] = s1c[d], dc.e0[d] = e0c[d], dc.e1[d] = e1c[d];
    }
    dc.dV0 = dV0;
    dc.incl = incl;
    dc.stored = stored_weight;
    long ln[3];
    for (int k = 0; k < 3; k++) ln[k] = S.has[yd[k]] ? (iec[yd[k]] - isc[yd[k]]) / 2 + 1 : 1;
    dc.N = size_t(ln[0] * ln[1] * ln[2]);
    dc.p0 = 0;  // set when the lists are laid out
    auto W1 = [&](int k, long i) -> double {
      const int d = yd[k];
      const long n = ln[k];
      if (i > 1 && i < n - 2) return 1.0;
      if (i == 0) return s0c[d];
      if (i == 1) return s1c[d];
      if (i == n - 1) return e0c[d];
      if (i == n - 2) return e1c[d];
      return 1.0;
    };
    const double fac = nun == 2 ? 0.25 : (nun == 1 ? 0.5 : 1.0);
    // points in IVEC_LOOP_COUNTER order; local indices of the Yee base point
    std::vector<int> pj;
    std::vector<double> w;
    for (long i1 = 0; i1 < ln[0]; i1++)
      for (long i2 = 0; i2 < ln[1]; i2++)
        for (long i3 = 0; i3 < ln[2]; i3++) {
          const long ii[3] = {i1, i2, i3};
          int p[3] = {0, 0, 0};  // centered point, absolute half-coords
          for (int k = 0; k < 3; k++)
            if (S.has[yd[k]]) p[yd[k]] = isc[yd[k]] + 2 * int(ii[k]);
          double wt = incl ? (W1(2, i3) * (W1(1, i2) * ((dV0 + 0.0 * i2) * W1(0, i1)))) : 1.0;
          w.push_back(wt * fac);
          // this rank owns the centered point if its slab index is in the owned range
          int j[3] = {0, 0, 0};
          bool mine = true;
          for (int d = 0; d < 3; d++) {
            if (!S.has[d]) continue;
            if (yee) {  // the Yee point itself; owned along d by one rank (walls included)
              j[d] = (p[d] - S.io[d] - sh[d]) / 2 - g.off[d];
              const int nloc = g.N[g.ax[d]] - 1;  // this rank's cells along d
              if (sh[d] ? (j[d] < 0 || j[d] > nloc - 1) : (j[d] < 1 || j[d] > nloc)) mine = false;
              continue;
            }
            const int base = p[d] - (S.shift(c, d) ? 0 : 1);  // Yee point of c at/below p
            j[d] = (base - S.io[d] - S.shift(c, d)) / 2 - g.off[d];
            const int jc = (p[d] - S.io[d] - 1) / 2 - g.off[d];  // centered index
            if (jc < g.owned_lo_sh[d] || jc > g.owned_hi_sh[d]) mine = false;
          }
          for (int d = 0; d < 3; d++) pj.push_back(mine ? j[d] : -1);
        }
    dc.p0 = o.h_pj.size() / 3;
    o.h_pj.insert(o.h_pj.end(), pj.begin(), pj.end());
    pw.insert(pw.end(), w.begin(), w.end());
    made.push_back(dc);
  }
  for (auto &m : made) list.insert(list.begin(), m);
}

// decimation_factor of fields::add_dft (src/dft.cpp:190-213)
int dft_decimation(mnl_fields *F, const double *freqs, int nfreq, int decim) {
  if (decim != 0) return decim;
  double src_freq_max = 0;
  for (auto &st : F->srcs) {
    const double fw = st.kind == 0 ? sqrt(-2.0 * log(1e-7)) / (st.width * pi) : 0.0;
    if (fw == 0)
      decim = 1;
    else
      src_freq_max =
          std::max(src_freq_max, std::abs(st.kind == 0 ? st.freq : st.cfreq.real()) + 0.5 * fw);
  }
  double freq_max = 0;
  for (int i = 0; i < nfreq; ++i) freq_max = std::max(freq_max, std::abs(freqs[i]));
  bool nonlinear = false;  // structure_chunk::has_nonlinearities: nonzero chi2/chi3
  for (int c = 0; c < 3; c++) {
    for (double v : F->S.chi2[c]) nonlinear = nonlinear || v != 0.0;
    for (double v : F->S.chi3[c]) nonlinear = nonlinear || v != 0.0;
  }
  for (auto &b : F->S.boxes) nonlinear = nonlinear || ((b.kind == 1 || b.kind == 2) && b.value != 0.0);
  // (src/dft.cpp:207-210 overwrites the fwidth == 0 case above)
  if ((freq_max > 0) && (src_freq_max > 0) && !nonlinear)
    return std::max(1, int(std::floor(1 / (F->dt * (freq_max + src_freq_max)))));
  return 1;
}

// Device layout of a DFT object whose E list holds the points of `pwE` and whose
// H points (ho) follow: per-point chunk ids, wave-blocked DFT array, slots.
int dft_layout(mnl_fields *F, std::unique_ptr<DftFluxH> &o, DftFluxH &ho, std::vector<double> &pwE,
               std::vector<double> &pwH) {
  const int nfreq = o->nfreq;
  // lay out: E points (creation order), then H points; chunks keep their p0
  const size_t nE = o->h_pj.size() / 3;
  for (auto &h : o->H) h.p0 += nE;
  o->h_pj.insert(o->h_pj.end(), ho.h_pj.begin(), ho.h_pj.end());
  pwE.insert(pwE.end(), pwH.begin(), pwH.end());
  o->npts = o->h_pj.size() / 3;
  // per-point chunk id: chunks numbered E list then H list
  std::vector<int> pch(o->npts, 0);
  std::vector<DftChunkDev> chd;
  auto lay = [&](const std::vector<DftChunkH> &L) {
    for (auto &dc : L) {
      DftChunkDev cd;
      cd.c = dc.c;
      cd.avgmode = dc.avgmode;
      cd.d1 = cd.d2 = -1;  // grid_volume::yee2cent_offsets order (X, Y, Z)
      for (int dd = 0; dd < 3; dd++)
        if (F->S.has[dd] && !F->S.shift(dc.c, dd)) (cd.d1 < 0 ? cd.d1 : cd.d2) = dd;
      for (size_t k = 0; k < dc.N; k++) pch[dc.p0 + k] = (int)chd.size();
      chd.push_back(cd);
    }
  };
  lay(o->E);
  lay(o->H);
  // per point and update: 3 indices + chunk id + weight, the averaged field
  // values, the sample written and read back, and 1/kb of a read-modify-write
  // of one complex value per frequency (DESIGN.md "DFT")
  for (const auto *L : {&o->E, &o->H})
    for (auto &dc : *L)
      o->bytes += double(dc.N) * (12 + 4 + 8 + 8.0 * (1 << dc.avgmode) + 16 +
                                  (12 + 4 + 32.0 * nfreq) / o->kb);
  // Device slots: the points sorted by component and chunk, then z, y, x (x fastest like
  // the field arrays), so that a wave's field reads are as contiguous as the
  // plane's orientation allows and a workgroup of the accumulation almost always holds one
  // chunk (one phase row, staged in LDS once); other ranks' points last.  Only the storage
  // order changes -- every point keeps its own reference-order accumulation.
  std::vector<int> ord(o->npts);
  for (size_t p = 0; p < o->npts; p++) ord[p] = (int)p;
  auto key = [&](int p) {
    const int *j = &o->h_pj[3 * (size_t)p];
    return std::make_tuple(j[0] < 0, chd[pch[p]].c, pch[p], j[2], j[1], j[0], p);
  };
  std::sort(ord.begin(), ord.end(), [&](int a, int b) { return key(a) < key(b); });
  o->slot.assign(o->npts, 0);
  std::vector<int> spj(3 * o->npts), spch(o->npts);
  std::vector<double> spw(o->npts);
  for (size_t t = 0; t < o->npts; t++) {
    const int p = ord[t];
    o->slot[p] = (int)t;
    for (int e = 0; e < 3; e++) spj[3 * t + e] = o->h_pj[3 * (size_t)p + e];
    spch[t] = pch[p];
    spw[t] = pwE[p];
  }
  for (int k = 0; k < 3; k++) o->bbox.lo[k] = INT32_MAX, o->bbox.hi[k] = -1;
  for (size_t p = 0; p < o->npts; p++) {
    if (o->h_pj[3 * p] < 0) continue;
    for (int k = 0; k < 3; k++) {
      o->bbox.lo[k] = std::min(o->bbox.lo[k], o->h_pj[3 * p + k]);
      o->bbox.hi[k] = std::max(o->bbox.hi[k], o->h_pj[3 * p + k] + 1);
    }
  }
  // compact box (two-step pairs, 3-D): every bbox cell, 2 states x 6 arrays, <= 1 GiB
  o->cmp_cells = 0, o->cmp_mask = 0;
  if (F->S.dim == 3 && o->bbox.hi[0] >= 0) {
    double nc = 1;
    for (int k = 0; k < 3; k++) nc *= o->bbox.hi[k] - o->bbox.lo[k] + 1;
    if (nc * 96 <= double(1u << 30)) o->cmp_cells = (unsigned)nc;
    for (const auto *L : {&o->E, &o->H})
      for (auto &dc : *L) o->cmp_mask |= 1u << (dc.c >= 3 ? 3 + dc.c % 3 : dc.c % 3);
  }
  if (o->npts) {
    if (dev_alloc(F, &o->d_pj, o->h_pj.size(), false) || dev_alloc(F, &o->d_pch, o->npts, false) ||
        dev_alloc(F, &o->d_pw, o->npts, false) || dev_alloc(F, &o->d_ch, chd.size(), false) ||
        dev_alloc(F, &o->d_dft, 2 * ((o->npts + 63) & ~size_t(63)) * (size_t)nfreq) ||
        dev_alloc(F, &o->d_fr, o->npts * (size_t)o->kb))
      return -1;
    HIPCHK(hipMemcpyAsync(o->d_pj, spj.data(), spj.size() * 4, hipMemcpyHostToDevice, F->stream));
    HIPCHK(hipMemcpyAsync(o->d_pch, spch.data(), spch.size() * 4, hipMemcpyHostToDevice, F->stream));
    HIPCHK(hipMemcpyAsync(o->d_pw, spw.data(), spw.size() * 8, hipMemcpyHostToDevice, F->stream));
    HIPCHK(hipMemcpyAsync(o->d_ch, chd.data(), chd.size() * sizeof(DftChunkDev), hipMemcpyHostToDevice,
                          F->stream));
    HIPCHK(hipStreamSynchronize(F->stream));
  }
  F->dfts.push_back(std::move(o));
  return int(F->dfts.size()) - 1;
}

int dft_add_flux(mnl_fields *F, int nreg, const double *regions, const double *freqs, int nfreq,
                 int decimation) {
  if (F->src_dirty && build_source_lists(F)) return -1;
  if (nreg < 1 || nfreq < 1) return fail("add_dft_flux: no regions / frequencies");
  std::unique_ptr<DftFluxH> o(new DftFluxH);
  o->nfreq = nfreq;
  for (int i = 0; i < nfreq; i++) o->omega.push_back(2 * pi * freqs[i]);
  o->decim = dft_decimation(F, freqs, nfreq, decimation);
  for (int d = 0; d < 3; d++) o->wmin[d] = regions[d], o->wmax[d] = regions[3 + d];
  if (const char *e = getenv("MNL_DFT_BLOCK")) o->kb = std::max(1, std::min(DFT_KB, atoi(e)));
  const double dt_factor = F->dt / sqrt(2.0 * pi) * o->decim;
  std::vector<double> pwE, pwH;
  DftFluxH ho;  // H points collected separately, appended after the E points
  for (int r = 0; r < nreg; r++) {
    const double *R = regions + 8 * r;
    const int d = int(R[6]);
    const double wgt = R[7];
    int cE[2], cH[2];
    switch (d) {  // fields::add_dft_flux (src/dft.cpp:601-617)
      case 0: cE[0] = MNL_EY, cE[1] = MNL_EZ, cH[0] = MNL_HZ, cH[1] = MNL_HY; break;
      case 1: cE[0] = MNL_EZ, cE[1] = MNL_EX, cH[0] = MNL_HX, cH[1] = MNL_HZ; break;
      default: cE[0] = MNL_EX, cE[1] = MNL_EY, cH[0] = MNL_HY, cH[1] = MNL_HX; break;
    }
    for (int i = 0; i < 2; ++i) {
      dft_add(F, *o, cE[i], R, R + 3, true, cplx(wgt * double(1 - 2 * i)), dt_factor, o->E, pwE);
      dft_add(F, ho, cH[i], R, R + 3, false, cplx(1.0), dt_factor, o->H, pwH);
    }
  }
  return dft_layout(F, o, ho, pwE, pwH);
}

// fields::add_dft_fields (src/dft.cpp:889-903): per component (in order) add_dft
// without dV / interpolation weights, stored_weight 1, prepended to one list; on
// the centered grid or (yee) each component's own grid
int dft_add_fields(mnl_fields *F, int ncomp, const int *comps, const double wmin[3],
                   const double wmax[3], const double *freqs, int nfreq, int yee, int decimation) {
  if (F->src_dirty && build_source_lists(F)) return -1;
  if (ncomp < 1 || nfreq < 1) return fail("add_dft_fields: no components / frequencies");
  for (int k = 0; k < ncomp; k++)
    if (comps[k] < 0 || comps[k] >= 6) return fail("add_dft_fields: E or H components only");
  std::unique_ptr<DftFluxH> o(new DftFluxH);
  o->fields = true;
  o->nfreq = nfreq;
  for (int i = 0; i < nfreq; i++) o->omega.push_back(2 * pi * freqs[i]);
  o->decim = dft_decimation(F, freqs, nfreq, decimation);
  for (int d = 0; d < 3; d++) o->wmin[d] = wmin[d], o->wmax[d] = wmax[d];
  if (const char *e = getenv("MNL_DFT_BLOCK")) o->kb = std::max(1, std::min(DFT_KB, atoi(e)));
  const double dt_factor = F->dt / sqrt(2.0 * pi) * o->decim;
  std::vector<double> pwE, pwH;
  DftFluxH ho;
  for (int k = 0; k < ncomp; k++)
    dft_add(F, *o, comps[k], wmin, wmax, false, cplx(1.0), dt_factor, o->E, pwE, yee != 0);
  return dft_layout(F, o, ho, pwE, pwH);
}

// phases of every DFT update in steps [t0+1, t0+ns] -> device (one row per update), after
// the rows of the updates still buffered from earlier calls (accumulated by the next flush:
// when kb updates are buffered or before the DFT array is read, not at the end of every call)
int dft_prepare(mnl_fields *F, long long t0, int ns) {
  for (auto &op : F->dfts) {
    DftFluxH &o = *op;
    const size_t nch = o.E.size() + o.H.size();
    const size_t rowlen = 2 * nch * (size_t)o.nfreq;
    std::vector<double> ph;
    ph.reserve(((size_t)o.nbuf + ns) * rowlen);
    if (o.nbuf > 0) {
      if (o.ph_host.size() < (size_t)o.row * rowlen || o.row < o.nbuf)
        return fail("dft: buffered phase rows lost");
      ph.insert(ph.end(), o.ph_host.begin() + (size_t)(o.row - o.nbuf) * rowlen,
                o.ph_host.begin() + (size_t)o.row * rowlen);
    }
    o.row = o.nbuf;
    std::vector<cplx> pe(o.nfreq), phh(o.nfreq);
    for (int s = 0; s < ns; s++) {
      const long long t = t0 + s + 1;
      if (t % o.decim) continue;
      const double tE = t * F->dt, tH = tE - 0.5 * F->dt;  // fields::update_dfts
      // exp(i omega t) once per frequency and time (E / H), then times each chunk's scale:
      // the same operations as the reference's per-chunk polar(1, omega t) * scale
      for (int i = 0; i < o.nfreq; i++) {
        pe[i] = std::polar(1.0, o.omega[i] * tE);
        phh[i] = std::polar(1.0, o.omega[i] * tH);
      }
      // chunks with the same time and the same scale (bitwise) share one row of products
      std::vector<std::pair<std::pair<bool, cplx>, size_t>> done;
      auto same = [](const cplx &x, const cplx &y) {
        return memcmp(&x, &y, sizeof(cplx)) == 0;
      };
      auto add = [&](const std::vector<DftChunkH> &L) {
        for (auto &dc : L) {
          const bool isH = ctype(dc.c) == T_H;
          size_t from = SIZE_MAX;
          for (auto &d : done)
            if (d.first.first == isH && same(d.first.second, dc.scale)) from = d.second;
          const size_t at = ph.size();
          if (from != SIZE_MAX) {
            for (int i = 0; i < 2 * o.nfreq; i++) ph.push_back(ph[from + i]);
            continue;
          }
          done.push_back({{isH, dc.scale}, at});
          const std::vector<cplx> &pt = isH ? phh : pe;
          for (int i = 0; i < o.nfreq; i++) {
            const cplx p = pt[i] * dc.scale;
            ph.push_back(p.real());
            ph.push_back(p.imag());
          }
        }
      };
      add(o.E);
      add(o.H);
    }
    if (ph.empty()) {
      o.ph_host.clear();
      continue;
    }
    if (o.ph_cap < ph.size()) {
      HIPCHK(hipStreamSynchronize(F->stream));
      if (o.d_ph) hipFree(o.d_ph);
      HIPCHK(hipMalloc(&o.d_ph, ph.size() * 8));
      o.ph_cap = ph.size();
    }
    (void)nch;
    HIPCHK(hipMemcpyAsync(o.d_ph, ph.data(), ph.size() * 8, hipMemcpyHostToDevice, F->stream));
    HIPCHK(hipStreamSynchronize(F->stream));
    o.ph_host.swap(ph);
  }
  return 0;
}

// accumulate the buffered updates of one flux object
int dft_flush(mnl_fields *F, DftFluxH &o) {
  if (!o.nbuf) return 0;
  const size_t nch = o.E.size() + o.H.size();
  const long long rstride = (long long)(nch * o.nfreq);
  if (k_dft_accum(o.d_pj, o.d_pch, o.d_dft, o.d_fr, o.nbuf,
                  o.d_ph + 2 * (size_t)(o.row - o.nbuf) * rstride, rstride, o.nfreq,
                  (long long)o.npts, F->stream))
    return fail("dft accumulate launch failed");
  o.nbuf = 0;
  return 0;
}

// after step t (fields::update_dfts, src/dft.cpp:249-263)
// what a sampling plan depends on: implicit E (the fused mode and its geometry) and which H
// components are stored separately
long long dft_plan_key(const mnl_fields *F) {
  long long k = (long long)F->fused_epoch * 2 + (F->fused ? 1 : 0);
  for (int d = 0; d < 3; d++) k = k * 2 + (F->f.H[d] ? 1 : 0);
  return k * 2 + (F->f.hall ? 1 : 0);
}

// fields: the buffer set to sample (null: the current one; temporal blocking samples the middle
// step of a pair from the mid set)
// cstate >= 0: a pair's middle (0) or new (1) state, whose two-step points are also in the
// monitors' compact boxes
int dft_update(mnl_fields *F, long long t, const DevFields *fields, int cstate) {
  const bool planned = F->nlocal < (size_t(1) << 31);  // int32 indices in the plan
  const DevFields &fs = fields ? *fields : F->f;
  // the samples of every flux object due: planned ones in merged launches of up to DFT_MAXJ
  DftSampleJobs J{};
  auto launch = [&]() -> int {
    if (J.n && k_dft_sample_jobs(J, F->g, fs, F->d_utab, F->stream))
      return fail("dft sample launch failed");
    J = DftSampleJobs{};
    return 0;
  };
  for (auto &op : F->dfts) {
    DftFluxH &o = *op;
    if (t % o.decim || !o.npts) continue;
    double *fr = o.d_fr + (size_t)o.nbuf * o.npts;
    if (planned) {
      const long long key = dft_plan_key(F);
      if (o.plan_key != key) {
        if (!o.d_sidx) {
          HIPCHK(hipMalloc(&o.d_sidx, o.npts * 4));
          HIPCHK(hipMalloc(&o.d_ssel, o.npts * 2));
          HIPCHK(hipMalloc(&o.d_spal, o.npts * 4));
          HIPCHK(hipMalloc(&o.d_su, o.npts * 32));
          HIPCHK(hipMalloc(&o.d_bad, sizeof(int)));
        }
        if (o.cmp_cells && !o.d_sci) HIPCHK(hipMalloc(&o.d_sci, o.npts * 4));
        const bool pal = F->fused && F->d_uidx && F->d_utab && F->dft_pal;
        HIPCHK(hipMemsetAsync(o.d_bad, 0, sizeof(int), F->stream));
        if (k_dft_plan(o.d_pj, o.d_pch, o.d_ch, (long long)o.npts, F->g, F->f,
                       pal ? F->d_uidx : nullptr, pal ? F->d_utab : nullptr, o.d_sidx, o.d_ssel,
                       o.d_spal, o.d_su, o.d_bad, o.bbox, o.cmp_cells ? o.d_sci : nullptr,
                       F->stream))
          return fail("dft plan launch failed");
        int bad = 1;
        if (pal) {  // once per plan: are the palette bytes exact for every implicit value?
          HIPCHK(hipMemcpyAsync(&bad, o.d_bad, sizeof(int), hipMemcpyDeviceToHost, F->stream));
          HIPCHK(hipStreamSynchronize(F->stream));
        }
        o.usepal = pal && bad == 0;
        o.plan_key = key;
      }
      if (J.n == DFT_MAXJ && launch()) return -1;
      DftSampleJob &jb = J.j[J.n++];
      jb.sidx = o.d_sidx, jb.ssel = o.d_ssel, jb.spal = o.d_spal, jb.su = o.d_su;
      jb.pw = o.d_pw, jb.fr = fr, jb.npts = (long long)o.npts, jb.blk0 = J.nblk;
      jb.usepal = o.usepal ? 1 : 0;
      if (cstate >= 0 && o.cmp_on && o.d_cmp && o.d_sci) {
        jb.sci = o.d_sci;
        jb.cmp = o.d_cmp + (size_t)cstate * 6 * o.cmp_cells;
        jb.ncell = o.cmp_cells;
        const int n0 = o.bbox.hi[0] - o.bbox.lo[0] + 1, n1 = o.bbox.hi[1] - o.bbox.lo[1] + 1;
        for (int e = 0; e < 3; e++) {
          const int ax = F->g.ax[e];
          jb.cs[e] = ax == 0 ? 1 : ax == 1 ? n0 : ax == 2 ? n0 * n1 : 0;
        }
      }
      J.nblk += ((long long)o.npts + 255) / 256;
    } else if (k_dft_sample(o.d_pj, o.d_pw, o.d_pch, o.d_ch, fr, (long long)o.npts, F->g, fs,
                            F->stream)) {
      return fail("dft sample launch failed");
    }
  }
  if (launch()) return -1;
  for (auto &op : F->dfts) {
    DftFluxH &o = *op;
    if (t % o.decim || !o.npts) continue;
    o.nbuf++;
    o.row++;
    if (o.nbuf == o.kb && dft_flush(F, o)) return -1;
  }
  return 0;
}

bool dft_due(const mnl_fields *F, long long t) {
  for (auto &op : F->dfts)
    if (op->npts && t % op->decim == 0) return true;
  return false;
}


int dft_flux_values(mnl_fields *F, int h, double *out) {
  if (h < 0 || h >= (int)F->dfts.size()) return fail("bad dft handle");
  DftFluxH &o = *F->dfts[h];
  if (dft_flush(F, o)) return -1;  // the buffered updates first
  const size_t nf = o.nfreq;
  std::vector<double> v(2 * ((o.npts + 63) & ~size_t(63)) * nf);
  bool ok = true;
  if (!v.empty())
    ok = hipMemcpyAsync(v.data(), o.d_dft, v.size() * 8, hipMemcpyDeviceToHost, F->stream) ==
             hipSuccess &&
         hipStreamSynchronize(F->stream) == hipSuccess;
  if (F->nranks > 1 && F->comm->agree_ok(ok, F->stream))  // every rank fails together
    return fail(ok ? "flux: a rank failed" : "flux: device copy failed");
  if (!ok) return fail("flux: device copy failed");
  for (size_t i = 0; i < nf; ++i) out[i] = 0;
  for (size_t k = 0; k < o.E.size() && k < o.H.size(); k++)  // dft_flux::flux (src/dft.cpp:533-547)
    for (size_t p = 0; p < o.E[k].N; ++p) {
      const size_t pe = o.E[k].p0 + p, ph = o.H[k].p0 + p;
      if (o.h_pj[3 * pe] < 0 && o.h_pj[3 * pe + 1] < 0 && o.h_pj[3 * pe + 2] < 0) continue;
      for (size_t i = 0; i < nf; ++i) {
        const size_t ie = dft_at(o.slot[pe], i, nf), ih = dft_at(o.slot[ph], i, nf);
        const cplx e(v[2 * ie], v[2 * ie + 1]);
        const cplx hv(v[2 * ih], v[2 * ih + 1]);
        out[i] += real(e * conj(hv));
      }
    }
  if (F->nranks > 1)
    for (size_t i0 = 0; i0 < nf; i0 += 64)
      if (timed_allreduce(F, out + i0, (int)std::min<size_t>(64, nf - i0)))
        return fail("flux allreduce failed");
  return 0;
}

}  // namespace mnlh
