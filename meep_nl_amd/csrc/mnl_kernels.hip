// mnl_kernels.hip -- gfx950 kernels of the fields::step() hot path.
//
// Global-grid formulation of the reference's chunked update:
// the reference splits PML regions into their own chunks and runs a different
// loop body per chunk (src/step_generic.cpp:69-253, 576-906).  Here one
// kernel per sub-step covers the rank-local grid; the interior box (no
// component of any point lies in a PML chunk, H == B) runs the lean body,
// the <= 6 shell boxes run the general body, which looks the per-point chunk
// flags up in tiny per-direction tables.  Arithmetic follows the reference
// expression by expression and the library is compiled with
// -ffp-contract=off, so results are bitwise those of the CPU reference.
//
// All kernels are HBM-bound fp64 stencils (0.1-0.2 flop/byte): no MFMA.
#include <hip/hip_runtime.h>

#include "mnl_internal.hpp"

// Every kernel here is written for 64-lane wavefronts (gfx950): the fused bodies map one
// 64-column row to a wave, nr_hard_kernel runs one attempt per lane with a 64-bit ballot.
#if defined(__AMDGCN_WAVEFRONT_SIZE) && __AMDGCN_WAVEFRONT_SIZE != 64
#error "mnl_kernels.hip needs wave64 (build for gfx950)"
#endif

namespace mnl {

// tile-kernel code-generation switches (variant builds for A/B timing; defaults are the
// measured choices)
#ifndef MNL_RS_AT
#define MNL_RS_AT 1
#endif
#ifndef MNL_SKIP_B
#define MNL_SKIP_B 1
#endif
#ifndef MNL_HOIST_X
#define MNL_HOIST_X 0
#endif
#ifndef MNL_OWNC
#define MNL_OWNC 1
#endif
#ifndef MNL_MULTI_DIST  // prefetch distance of the multi-axis PML bodies (AX = 3, 5, 7)
#define MNL_MULTI_DIST 0
#endif

#define MNL_BX 64
#define MNL_BY 4

__device__ __forceinline__ int shift_of(int type, int c, int d) {
  // grid_volume::iyee_shift (src/meep/vec.hpp:1133-1141)
  return (type == T_E || type == T_D) ? (d == c) : (d != c);
}

struct Pt {
  int j[3];       // local index per direction (0 for absent)
  long long idx;  // linear index
};

__device__ __forceinline__ bool make_pt(const Box &b, const DevGrid &g, Pt &p) {
  int i0 = b.lo[0] + blockIdx.x * MNL_BX + threadIdx.x;
  int i1 = b.lo[1] + blockIdx.y * MNL_BY + threadIdx.y;
  int i2 = b.lo[2] + blockIdx.z;
  if (i0 > b.hi[0] || i1 > b.hi[1]) return false;
  int ii[3] = {i0, i1, i2};
#pragma unroll
  for (int d = 0; d < 3; d++) p.j[d] = g.ax[d] >= 0 ? ii[g.ax[d]] : 0;
  p.idx = (long long)i0 + (long long)i1 * g.st[1] + (long long)i2 * g.st[2];
  return true;
}

__device__ __forceinline__ bool make_pt_lin(const BoxList &bl, const DevGrid &g, Pt &p) {
  long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= bl.start[bl.n]) return false;
  int k = 0;
#pragma unroll
  for (int q = 1; q < MAX_BOX - 1; q++)
    if (q < bl.n && t >= bl.start[q]) k = q;
  const Box &b = bl.b[k];
  long long l = t - bl.start[k];
  const long long n0 = b.hi[0] - b.lo[0] + 1, n1 = b.hi[1] - b.lo[1] + 1;
  int i0 = b.lo[0] + (int)(l % n0);
  l /= n0;
  int i1 = b.lo[1] + (int)(l % n1);
  int i2 = b.lo[2] + (int)(l / n1);
  int ii[3] = {i0, i1, i2};
#pragma unroll
  for (int d = 0; d < 3; d++) p.j[d] = g.ax[d] >= 0 ? ii[g.ax[d]] : 0;
  p.idx = (long long)i0 + (long long)i1 * g.st[1] + (long long)i2 * g.st[2];
  return true;
}

template <bool SHELL>
__device__ __forceinline__ bool map_pt(const Box &b, const BoxList &bl, const DevGrid &g, Pt &p) {
  return SHELL ? make_pt_lin(bl, g, p) : make_pt(b, g, p);
}

// little_owned_corner0 .. big_corner (src/meep/vec.hpp:1102-1104), with the
// metallic wall plane left untouched (it is zeroed by zero_metal in the
// reference, src/boundaries.cpp:304-339, and never becomes nonzero).
__device__ __forceinline__ bool owned(const DevGrid &g, int type, int c, const Pt &p) {
#pragma unroll
  for (int d = 0; d < 3; d++) {
    if (g.ax[d] < 0) continue;
    if (shift_of(type, c, d)) {
      if (p.j[d] < g.owned_lo_sh[d] || p.j[d] > g.owned_hi_sh[d]) return false;
    } else {
      if (p.j[d] < g.owned_lo_un[d] || p.j[d] > g.owned_hi_un[d]) return false;
    }
  }
  return true;
}

// global half-coordinate (relative to the cell's little corner) of a point
__device__ __forceinline__ int qcoord(const DevGrid &g, const Pt &p, int type, int c, int d) {
  return 2 * (p.j[d] + g.off[d]) + shift_of(type, c, d);
}

__device__ __forceinline__ bool pml_at(const DevFields &f, const DevGrid &g, int d, int q) {
  return g.ax[d] >= 0 && f.pml.flag[d] != nullptr && f.pml.flag[d][q] != 0;
}

// Fused mode: E of comp c at p is not stored but equals chi1inv * D (DESIGN.md
// "Fused step"): p inside the fused domain G, E_c owned there and not in a
// PML chunk along c (where E carries W-form history and is stored).
__device__ __forceinline__ bool e_implicit(const DevFields &f, const DevGrid &g, int c,
                                           const Pt &p) {
  if (!f.fused) return false;
#pragma unroll
  for (int d = 0; d < 3; d++)
    if (p.j[d] < f.fG.lo[d] || p.j[d] > f.fG.hi[d]) return false;
  for (int k = 0; k < f.npol; k++) {  // stored inside a polarization's nonzero box
    const Box &b = f.pol[k].nz;
    if (p.j[0] >= b.lo[0] && p.j[0] <= b.hi[0] && p.j[1] >= b.lo[1] && p.j[1] <= b.hi[1] &&
        p.j[2] >= b.lo[2] && p.j[2] <= b.hi[2])
      return false;
  }
  return owned(g, T_E, c, p) && !pml_at(f, g, c, qcoord(g, p, T_E, c, c));
}

// conductivity allocated in the reference chunk that owns point p (zone box)
__device__ __forceinline__ bool cnd_in_chunk(const DevFields &f, const DevGrid &g, const Pt &p,
                                             int FT, int d) {
  int zb = 0;
#pragma unroll
  for (int e = 0; e < 3; e++) {
    const int z = g.ax[e] >= 0 ? f.zone[e][qcoord(g, p, FT, d, e)] : 1;  // absent: middle
    zb = zb * 3 + z;
  }
  return (f.cnd_zone[zb] >> (3 * (FT == T_D) + d)) & 1;
}

// Apply one curl update with the per-point PML branch selection of step_curl
// (src/step_generic.cpp:84-252).  With conductivity (cnd != null) the
// cnd branches apply; where cnd == 0 they equal the cnd-free ones bit for bit
// ((1 - 0)*f - x)*1), except the f_cond form of a PML chunk along dsig, which
// is taken only where the chunk holds a conductivity array (cnd_in_chunk).
template <int FT>
__device__ __forceinline__ double curl_apply(const DevFields &f, const DevGrid &g, const Pt &p,
                                             int d, long long i, double T, double dtdx) {
  const double *Fo = FT == T_B ? f.B[d] : f.D[d];
  double *F = FT == T_B ? f.Bn[d] : f.Dn[d];
  const int dsig = (d + 1) % 3, dsigu = (d + 2) % 3;
  const int k = qcoord(g, p, FT, d, dsig), ku = qcoord(g, p, FT, d, dsigu);
  const bool ps = pml_at(f, g, dsig, k), pu = pml_at(f, g, dsigu, ku);
  const int t = FT == T_D;
  const double *cnd = f.cnd[t][d], *cndinv = f.cndinv[t][d];
  const double dt2 = f.cnd_dt2;
  double nv;
  if (!ps && !pu) {
    nv = cnd ? ((1 - dt2 * cnd[i]) * Fo[i] - dtdx * T) * cndinv[i] : Fo[i] - dtdx * T;
  } else if (!ps) {
    const double *U = FT == T_B ? f.UB[d] : f.UD[d];
    double *Un = FT == T_B ? f.UBn[d] : f.UD[d];
    const double *sigu = f.pml.sig[dsigu], *kapu = f.pml.kap[dsigu], *siginvu = f.pml.siginv[dsigu];
    double fprev = U[i];
    double fu = cnd ? ((1 - dt2 * cnd[i]) * fprev - dtdx * T) * cndinv[i] : fprev - dtdx * T;
    Un[i] = fu;
    nv = siginvu[ku] * ((kapu[ku] - sigu[ku]) * Fo[i] + fu - fprev);
  } else {
    const double *sig = f.pml.sig[dsig], *kap = f.pml.kap[dsig], *siginv = f.pml.siginv[dsig];
    const bool fc = cnd && cnd_in_chunk(f, g, p, FT, d);
    double x = 0;  // the f_cond difference (f_cond chunks only)
    if (fc) {
      double *FC = f.fcnd[t][d];
      const double fcnd_prev = FC[i];
      const double fcn = ((1 - dt2 * cnd[i]) * fcnd_prev - dtdx * T) * cndinv[i];
      FC[i] = fcn;
      x = fcn - fcnd_prev;
    }
    if (!pu) {
      nv = fc ? ((kap[k] - sig[k]) * Fo[i] + x) * siginv[k]
              : ((kap[k] - sig[k]) * Fo[i] - dtdx * T) * siginv[k];
    } else {
      const double *U = FT == T_B ? f.UB[d] : f.UD[d];
      double *Un = FT == T_B ? f.UBn[d] : f.UD[d];
      const double *sigu = f.pml.sig[dsigu], *kapu = f.pml.kap[dsigu], *siginvu = f.pml.siginv[dsigu];
      double fprev = U[i];
      double fu = fc ? ((kap[k] - sig[k]) * fprev + x) * siginv[k]
                     : ((kap[k] - sig[k]) * fprev - dtdx * T) * siginv[k];
      Un[i] = fu;
      nv = siginvu[ku] * ((kapu[ku] - sigu[ku]) * Fo[i] + fu - fprev);
    }
  }
  F[i] = nv;
  return nv;
}

// The per-point update that follows a curl in the same sub-step, fused into
// the shell curl kernel when nothing (a source, a neighbour read) sits between
// them: H from B (update_h_kernel below) and, without chi(2) Newton-Raphson,
// susceptibilities or integrated sources, E from D (update_e_kernel below).
template <int FT>
__device__ __forceinline__ void fused_point_update(const DevFields &f, const DevGrid &g,
                                                   const Pt &p, int d, long long i, double nv) {
  if (FT == T_B) {  // update_eh(H_stuff), src/update_eh.cpp:186-259
    if (!f.hcomp_present[d] || !f.H[d]) return;
    const int kw = qcoord(g, p, T_H, d, d);
    if (!pml_at(f, g, d, kw)) return;
    double fwprev = f.WH[d][i];
    double kapwkw = f.pml.kap[d][kw], sigwkw = f.pml.sig[d][kw];
    double fw = nv;
    f.WH[d][i] = fw;
    f.Hn[d][i] = f.H[d][i] + ((kapwkw + sigwkw) * fw - (kapwkw - sigwkw) * fwprev);
  } else {  // update_eh(E_stuff), diagonal chi1inv, no P (src/step_generic.cpp:576-906)
    if (!f.ecomp_present[d]) return;
    const double gs = nv;
    const double *u = f.inveps[d];
    double *En = f.En[d];
    const int kw = qcoord(g, p, T_E, d, d);
    if (pml_at(f, g, d, kw)) {
      double fwprev = f.WE[d][i];
      double kapwkw = f.pml.kap[d][kw], sigwkw = f.pml.sig[d][kw];
      double fw = u ? (gs * u[i]) : gs;
      f.WE[d][i] = fw;
      En[i] = f.E[d][i] + ((kapwkw + sigwkw) * fw - (kapwkw - sigwkw) * fwprev);
    } else {
      En[i] = u ? (gs * u[i]) : gs;
    }
  }
}

// ----------------------------------------------------------------- curl B / D
// fields_chunk::step_db -> step_curl (src/step_db.cpp:44-146,
// src/step_generic.cpp:69-253, conductivity as in curl_apply).  Component d of
// B (D): g1 = E (H) comp (d+2)%3 along dir (d+1)%3, g2 = comp (d+1)%3 along
// dir (d+2)%3; D uses negated strides (src/step_db.cpp:81-84).
template <int FT, bool SHELL, bool FUSEUP>
__global__ __launch_bounds__(MNL_BX *MNL_BY) void curl_kernel(Box b, BoxList bl, DevGrid g,
                                                               DevFields f, CurlPlan pl, double C) {
  Pt p;
  if (!map_pt<SHELL>(b, bl, g, p)) return;
  const long long i = p.idx;
  // shell launches are component-parallel (blockIdx.y = component): one
  // dependent load chain per thread instead of three
  const int dlo = SHELL ? (int)blockIdx.y : 0, dhi = SHELL ? (int)blockIdx.y + 1 : 3;
  for (int d = dlo; d < dhi; d++) {
    if (!pl.present[d]) continue;
    if (!owned(g, FT, d, p)) continue;
    const int c1 = (d + 2) % 3, dir1 = (d + 1) % 3;
    const int c2 = (d + 1) % 3, dir2 = (d + 2) % 3;
    long long s1 = g.sdir[dir1], s2 = g.sdir[dir2];
    const int terms = pl.terms[d];
    double T, dtdx = C;
    if (FT == T_B && SHELL && f.fused) {  // E is not stored inside the fused box: E = D*chi1inv
      auto e_at = [&](int c, long long n, int dd) -> double {
        Pt q = p;
        if (dd >= 0) q.j[dd] += 1;
        if (e_implicit(f, g, c, q)) {
          const double dv = f.D[c][n];
          return f.inveps[c] ? (dv * f.inveps[c][n]) : dv;
        }
        return f.E[c][n];
      };
      if (terms == 3) {
        T = e_at(c1, i + s1, dir1) - e_at(c1, i, -1) + e_at(c2, i, -1) - e_at(c2, i + s2, dir2);
      } else if (terms == 1) {
        T = e_at(c1, i + s1, dir1) - e_at(c1, i, -1);
      } else {
        T = e_at(c2, i + s2, dir2) - e_at(c2, i, -1);
        dtdx = -C;
      }
    } else {
      const double *g1, *g2;
      if (FT == T_B) {
        g1 = f.E[c1];
        g2 = f.E[c2];
      } else {
        s1 = -s1;
        s2 = -s2;
        g1 = f.hall ? f.Hn[c1] : f.Bn[c1];  // H == B (new) outside PML chunks
        g2 = f.hall ? f.Hn[c2] : f.Bn[c2];
        if (SHELL && !f.hall) {  // H separate only in chunks with PML along the H direction
          if (f.H[c1] && pml_at(f, g, c1, qcoord(g, p, T_H, c1, c1))) g1 = f.Hn[c1];
          if (f.H[c2] && pml_at(f, g, c2, qcoord(g, p, T_H, c2, c2))) g2 = f.Hn[c2];
        }
      }
      if (terms == 3) {
        T = g1[i + s1] - g1[i] + g2[i] - g2[i + s2];
      } else if (terms == 1) {
        T = g1[i + s1] - g1[i];
      } else {  // g1 == NULL: swap and flip the sign (src/step_generic.cpp:76-80)
        T = g2[i + s2] - g2[i];
        dtdx = -C;
      }
    }
    if (!SHELL) {
      const double *Fo = FT == T_B ? f.B[d] : f.D[d];
      double *F = FT == T_B ? f.Bn[d] : f.Dn[d];
      const double *cnd = f.cnd[FT == T_D][d];
      if (cnd)  // src/step_generic.cpp:91-103
        F[i] = ((1 - f.cnd_dt2 * cnd[i]) * Fo[i] - dtdx * T) * f.cndinv[FT == T_D][d][i];
      else
        F[i] = Fo[i] - dtdx * T;
      continue;
    }
    const double nv = curl_apply<FT>(f, g, p, d, i, T, dtdx);
    if (FUSEUP) fused_point_update<FT>(f, g, p, d, i, nv);
  }
}

// ----------------------------------------------------------------- H from B
// update_eh(H_stuff) in PML chunks: W auxiliary field, mu = 1
// (src/update_eh.cpp:186-259, src/step_generic.cpp:717-724).
__global__ __launch_bounds__(MNL_BX *MNL_BY) void update_h_kernel(BoxList bl, DevGrid g, DevFields f) {
  Pt p;
  if (!make_pt_lin(bl, g, p)) return;
  const long long i = p.idx;
#pragma unroll
  for (int d = 0; d < 3; d++) {
    if (!f.hcomp_present[d] || !f.H[d]) continue;
    if (!owned(g, T_H, d, p)) continue;
    const int kw = qcoord(g, p, T_H, d, d);
    if (!pml_at(f, g, d, kw)) continue;
    double fwprev = f.WH[d][i];
    double kapwkw = f.pml.kap[d][kw], sigwkw = f.pml.sig[d][kw];
    double fw = f.Bn[d][i];
    f.WH[d][i] = fw;
    f.Hn[d][i] = f.H[d][i] + ((kapwkw + sigwkw) * fw - (kapwkw - sigwkw) * fwprev);
  }
}

// ----------------------------------------------------------------- H-side materials
// update_eh(H_stuff) (src/update_eh.cpp:67-283 -> step_update_EDHB, src/step_generic.cpp:
// 576-906 with H = chi1inv_H * (B - P_H)) followed by update_pols(H_stuff) (isotropic
// lorentzian update_P, src/susceptibility.cpp:251-258, W = f_w or H, update_pols.cpp:44)
// when H is stored everywhere (f.hall: mu != 1 or magnetic susceptibilities).  The fork's
// H update takes the diagonal branch whatever off-diagonal mu rows exist (its 3x3 branch
// needs chi3, which no H component has), so only diag(chi1inv_H) enters.  Where the point's
// reference chunk aliases H to B, H = B (a copy, so every reader reads one array).
template <int d>
__device__ __forceinline__ void h_point(const DevGrid &g, const DevFields &f, const Pt &p,
                                        long long i, int pols) {
  if (!f.hcomp_present[d] || !owned(g, T_H, d, p)) return;
  const int kw = qcoord(g, p, T_H, d, d);
  const bool pml = pml_at(f, g, d, kw);
  int rz = 0;
#pragma unroll
  for (int e = 0; e < 3; e++) rz = rz * 3 + (g.ax[e] >= 0 ? f.zone[e][qcoord(g, p, T_H, d, e)] : 1);
  const bool sep = pml || f.hsep_all || ((f.hsep_zone[rz] >> d) & 1);
  double *Hn = f.Hn[d];
  double gs = f.Bn[d][i];
  double wv;
  if (!sep) {
    Hn[i] = gs;
    wv = gs;
  } else {
    for (int k = 0; k < f.nhpol; k++)  // subtract_P in pol-list order
      if (f.hpol[k].P[d]) gs -= f.hpol[k].P[d][i];
    const double *u = f.invmu[d];
    const double v = u ? (gs * u[i]) : gs;
    if (pml) {
      const double fwprev = f.WH[d][i];
      const double kapwkw = f.pml.kap[d][kw], sigwkw = f.pml.sig[d][kw];
      f.WH[d][i] = v;
      Hn[i] = f.H[d][i] + ((kapwkw + sigwkw) * v - (kapwkw - sigwkw) * fwprev);
    } else {
      Hn[i] = v;
    }
    wv = v;
  }
  for (int k = 0; k < (pols ? f.nhpol : 0); k++) {
    const PolDev &pd = f.hpol[k];
    if (!pd.P[d]) continue;
    const double pcur = pd.P[d][i];
    pd.P[d][i] = pd.gamma1inv * (pcur * (2 - pd.omega0dtsqr_denom) - pd.gamma1 * pd.Pp[d][i] +
                                 pd.omega0dtsqr * (pd.sigma[d][i] * wv));
    pd.Pp[d][i] = pcur;
  }
}

__global__ __launch_bounds__(MNL_BX *MNL_BY) void update_hmat_kernel(Box b, DevGrid g,
                                                                      DevFields f, int pols) {
  Pt p;
  if (!make_pt(b, g, p)) return;
  const long long i = p.idx;
  h_point<0>(g, f, p, i, pols);
  h_point<1>(g, f, p, i, pols);
  h_point<2>(g, f, p, i, pols);
}

// ----------------------------------------------------------------- chi(2) NR
// runNR / newtonRaphson (src/newton_raphson.cpp:93-359) in registers.
struct NRP {
  double A, B, F, G, H;  // C = D = E = 0 for the 43m tensor used by the fork
};

__device__ __forceinline__ void nr_eq(double x, double y, double z, const NRP &p1, const NRP &p2,
                                      const NRP &p3, double F[3]) {
  // newton_raphson.cpp:144-148
  F[0] = p1.A - (p1.B * x + p1.F * y * z + p1.G * x * z + p1.H * x * y);
  F[1] = p2.A - (p2.B * y + p2.F * y * z + p2.G * x * z + p2.H * x * y);
  F[2] = p3.A - (p3.B * z + p3.F * y * z + p3.G * x * z + p3.H * x * y);
}

__device__ bool nr_solve(double x, double y, double z, const NRP &p1, const NRP &p2,
                         const NRP &p3, double *fw, double *fw_2, double *fw_3, double tol1,
                         double tol2, double tol3, int max_it) {
  for (int iter = 0; iter < max_it; iter++) {
    double F[3], A[3][3];
    nr_eq(x, y, z, p1, p2, p3, F);
    // jacobian, newton_raphson.cpp:157-161
    A[0][0] = -p1.B - p1.G * z - p1.H * y;
    A[0][1] = -p1.F * z - p1.H * x;
    A[0][2] = -p1.F * y - p1.G * x;
    A[1][0] = -p2.G * z - p2.H * y;
    A[1][1] = -p2.B - p2.F * z - p2.H * x;
    A[1][2] = -p2.F * y - p2.G * x;
    A[2][0] = -p3.G * z - p3.H * y;
    A[2][1] = -p3.F * z - p3.H * x;
    A[2][2] = -p3.B - p3.F * y - p3.G * x;
    // solveLinearSystem, newton_raphson.cpp:170-194
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
      for (int q = r + 1; q < 3; q++) {
        double factor = A[q][r] / A[r][r];
#pragma unroll
        for (int k = r; k < 3; k++) A[q][k] -= factor * A[r][k];
        F[q] -= factor * F[r];
      }
    double dl[3];
#pragma unroll
    for (int r = 2; r >= 0; r--) {
      dl[r] = F[r];
#pragma unroll
      for (int q = r + 1; q < 3; q++) dl[r] -= A[r][q] * dl[q];
      dl[r] /= A[r][r];
    }
    x -= dl[0];
    y -= dl[1];
    z -= dl[2];
    if (fabs(dl[0]) < tol1 && fabs(dl[1]) < tol2 && fabs(dl[2]) < tol3) {
      double ax = fabs(x), ay = fabs(y), az = fabs(z);
      double fcp = (ax > ay ? (ax > az ? ax : az) : (ay > az ? ay : az)) * 1e-4;
      double fc[3];
      nr_eq(x, y, z, p1, p2, p3, fc);
      if (fc[0] <= fcp && fc[1] <= fcp && fc[2] <= fcp) {
        *fw = x;
        *fw_2 = y;
        *fw_3 = z;
        return true;
      }
    }
  }
  return false;
}

__device__ double nr_random(unsigned long long &st) {
  // deterministic replacement of the std::random_device fallback
  // (newton_raphson.cpp:196-206, 331-336); see DESIGN.md "Divergences".
  auto next = [&]() {
    unsigned long long z = (st += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  };
  // a log-uniform magnitude over 2^-300 .. 2^300 (the reference draws lognormal(1, 90) x
  // uniform(-1, 1): the same role, seeds spread over hundreds of decades) with a random
  // sign, from exact operations only (no libm), so the oracle's draws are bitwise equal
  const unsigned long long r1 = next(), r2 = next(), r3 = next();
  const int e = (int)(r1 % 601ull) - 300;
  const double m = 1.0 + (double)(r2 >> 11) * (1.0 / 9007199254740992.0);
  const double v = ldexp(m, e);
  return (r3 >> 63) ? -v : v;
}

// Seeds of attempt a >= 1 of runNR (the state the sequential loop below reaches):
// attempts 1-14 scale / negate the seeds (newton_raphson.cpp:266-330), attempts >= 15
// draw three deterministic random seeds each (rng advanced by 9 draws per attempt).
__device__ void nr_attempt_seeds(int a, double seed1, double seed2, double seed3,
                                 unsigned long long rng, double &s1, double &s2, double &s3) {
  const double M = 1e33;
  s1 = seed1, s2 = seed2, s3 = seed3;
  switch (a) {
    case 1: s1 = seed1 * M; break;
    case 2: s2 = seed2 * M; break;
    case 3: s3 = seed3 * M; break;
    case 4: s1 = -seed1 * M; break;
    case 5: s2 = -seed2 * M; break;
    case 6: s3 = -seed3 * M; break;
    case 7: s1 = seed1 * M, s2 = seed2 * M; break;
    case 8: s1 = seed1 * M, s3 = seed3 * M; break;
    case 9: s2 = seed2 * M, s3 = seed3 * M; break;
    case 10: s1 = -seed1 * M, s2 = -seed2 * M; break;
    case 11: s1 = -seed1 * M, s3 = -seed3 * M; break;
    case 12: s2 = -seed2 * M, s3 = -seed3 * M; break;
    case 13: s1 = seed1 * M, s2 = seed2 * M, s3 = seed3 * M; break;
    case 14: s1 = -seed1 * M, s2 = -seed2 * M, s3 = -seed3 * M; break;
    default: {
      unsigned long long st = rng + 9ull * (unsigned long long)(a - 15) * 0x9E3779B97F4A7C15ull;
      s1 = nr_random(st);
      s2 = nr_random(st);
      s3 = nr_random(st);
    }
  }
}

__device__ void run_nr(double seed1, double seed2, double seed3, double *fw, double *fw_2,
                       double *fw_3, const NRP &p1, const NRP &p2, const NRP &p3,
                       unsigned long long rng, unsigned long long *fallbacks,
                       const DevFields *df = nullptr, double *En = nullptr, long long idx = 0,
                       int dcomp = 0) {
  const double TOL = 1e-8, seedMax = 1e33;
  int max_it = 250;
  double tol1 = fmax(fabs(TOL * (*fw)) * 0.0001, TOL);
  double tol2 = fmax(fabs(TOL * (*fw_2)) * 0.0001, TOL);
  double tol3 = fmax(fabs(TOL * (*fw_3)) * 0.0001, TOL);
  double s1 = seed1, s2 = seed2, s3 = seed3;
  for (int a = 0; a < 100; ++a) {
    const double in0 = *fw, in1 = *fw_2, in2 = *fw_3;
    if (nr_solve(s1, s2, s3, p1, p2, p3, fw, fw_2, fw_3, tol1, tol2, tol3, max_it)) return;
    if (a == 0 && df && df->nr_hard) {
      // defer the remaining attempts to nr_hard_kernel (run in parallel there); the
      // caller stores the unchanged *fw of its component, overwritten on success
      const unsigned slot = atomicAdd(df->nr_hard_cnt, 1u);
      if (slot < (unsigned)df->nr_hard_cap) {
        NRHard &h = df->nr_hard[slot];
        const NRP *pp[3] = {&p1, &p2, &p3};
        for (int q = 0; q < 3; q++) {
          h.p[5 * q + 0] = pp[q]->A;
          h.p[5 * q + 1] = pp[q]->B;
          h.p[5 * q + 2] = pp[q]->F;
          h.p[5 * q + 3] = pp[q]->G;
          h.p[5 * q + 4] = pp[q]->H;
        }
        h.seed[0] = seed1, h.seed[1] = seed2, h.seed[2] = seed3;
        h.fw0[0] = in0, h.fw0[1] = in1, h.fw0[2] = in2;  // unchanged by a failed attempt
        h.En = En;
        h.i = idx;
        h.rng = rng;
        h.d = dcomp;
        return;
      }
    }
    switch (a) {  // newton_raphson.cpp:266-338
      case 0: s1 = seed1 * seedMax; max_it = 600; break;
      case 1: s1 = seed1; s2 = seed2 * seedMax; break;
      case 2: s2 = seed2; s3 = seed3 * seedMax; break;
      case 3: s3 = seed3; s1 = -seed1 * seedMax; break;
      case 4: s1 = seed1; s2 = -seed2 * seedMax; break;
      case 5: s2 = seed2; s3 = -seed3 * seedMax; break;
      case 6: s1 = seed1 * seedMax; s2 = seed2 * seedMax; s3 = seed3; break;
      case 7: s1 = seed1 * seedMax; s2 = seed2; s3 = seed3 * seedMax; break;
      case 8: s1 = seed1; s2 = seed2 * seedMax; s3 = seed3 * seedMax; break;
      case 9: s1 = -seed1 * seedMax; s2 = -seed2 * seedMax; s3 = seed3; break;
      case 10: s1 = -seed1 * seedMax; s2 = seed2; s3 = -seed3 * seedMax; break;
      case 11: s1 = seed1; s2 = -seed2 * seedMax; s3 = -seed3 * seedMax; break;
      case 12: s1 = seed1 * seedMax; s2 = seed2 * seedMax; s3 = seed3 * seedMax; break;
      case 13: s1 = -seed1 * seedMax; s2 = -seed2 * seedMax; s3 = -seed3 * seedMax; break;
      default:
        atomicAdd(fallbacks, 1ull);
        s1 = nr_random(rng);
        s2 = nr_random(rng);
        s3 = nr_random(rng);
        break;
    }
  }
}

// The deferred Newton-Raphson problems: one wave per problem, lane t runs attempt
// base + t (attempts 1..99, the sequential loop's seeds and max_it = 600); the lowest
// successful attempt is the one the sequential runNR would have returned, so the
// result is identical.  The fallback counter gets the random attempts the sequential
// loop would have started (newton_raphson.cpp:331-336).
__global__ __launch_bounds__(256) void nr_hard_kernel(DevFields f) {
  const unsigned n = min(*f.nr_hard_cnt, (unsigned)f.nr_hard_cap);
  const int lane = threadIdx.x & 63;
  const unsigned wv = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const unsigned nw = (gridDim.x * blockDim.x) >> 6;
  const double TOL = 1e-8;
  for (unsigned e = wv; e < n; e += nw) {
    const NRHard &h = f.nr_hard[e];
    const NRP p1 = {h.p[0], h.p[1], h.p[2], h.p[3], h.p[4]};
    const NRP p2 = {h.p[5], h.p[6], h.p[7], h.p[8], h.p[9]};
    const NRP p3 = {h.p[10], h.p[11], h.p[12], h.p[13], h.p[14]};
    const double tol1 = fmax(fabs(TOL * h.fw0[0]) * 0.0001, TOL);
    const double tol2 = fmax(fabs(TOL * h.fw0[1]) * 0.0001, TOL);
    const double tol3 = fmax(fabs(TOL * h.fw0[2]) * 0.0001, TOL);
    int found = -1;
    double rx = 0, ry = 0, rz = 0;
    for (int base = 1; base < 100 && found < 0; base += 64) {
      const int a = base + lane;
      double ox = h.fw0[0], oy = h.fw0[1], oz = h.fw0[2];
      bool ok = false;
      if (a < 100) {
        double s1, s2, s3;
        nr_attempt_seeds(a, h.seed[0], h.seed[1], h.seed[2], h.rng, s1, s2, s3);
        ok = nr_solve(s1, s2, s3, p1, p2, p3, &ox, &oy, &oz, tol1, tol2, tol3, 600);
      }
      const unsigned long long m = __ballot(ok);
      if (m) {
        const int w = __ffsll((long long)m) - 1;
        found = base + w;
        rx = __shfl(ox, w);
        ry = __shfl(oy, w);
        rz = __shfl(oz, w);
      }
    }
    if (lane == 0) {
      const unsigned long long fb = found < 0 ? 86ull : (found > 14 ? (unsigned long long)(found - 14) : 0ull);
      if (fb) atomicAdd(f.nr_fallbacks, fb);
      if (found >= 0) h.En[h.i] = h.d == 0 ? rx : h.d == 1 ? ry : rz;
    }
  }
}

// f_minus_p value of D component c at linear index n (src/update_eh.cpp:122-154)
__device__ __forceinline__ bool in_box(const Box &b, const Pt &p) {
  return p.j[0] >= b.lo[0] && p.j[0] <= b.hi[0] && p.j[1] >= b.lo[1] && p.j[1] <= b.hi[1] &&
         p.j[2] >= b.lo[2] && p.j[2] <= b.hi[2];
}
// bit k set: pol k may have nonzero P at p (device axes == directions in 3-D;
// in 1-D/2-D the absent directions have j = 0 and a box spanning 0)
__device__ __forceinline__ unsigned pol_mask(const DevFields &f, const Pt &p) {
  unsigned m = 0;
  for (int k = 0; k < f.npol; k++)
    if (in_box(f.pol[k].nz, p)) m |= 1u << k;
  return m;
}

// Owned by the reference's chunk although the kernels never update it: the high
// metallic wall plane of a component unshifted along the wall normal
// (little_owned_corner0..big_corner includes it, src/meep/vec.hpp:1102-1104;
// zero_metal zeroes f there only in step_boundaries, src/boundaries.cpp:304-339).
// glob: the whole-cell owned ranges (a neighbour rank's plane counts as owned)
__device__ __forceinline__ bool on_wall(const DevGrid &g, int c, const Pt &p, bool glob = false) {
  bool wall = false;
#pragma unroll
  for (int d = 0; d < 3; d++) {
    if (g.ax[d] < 0) continue;
    const bool sh = d == c;
    if (!sh && g.wall[d] && p.j[d] + g.off[d] == g.nglob[d]) {
      wall = true;
      continue;
    }
    if (glob) {
      const int jg = p.j[d] + g.off[d];
      if (jg < (sh ? 0 : 1) || jg > g.nglob[d] - 1) return false;
    } else {
      const int lo = sh ? g.owned_lo_sh[d] : g.owned_lo_un[d];
      const int hi = sh ? g.owned_hi_sh[d] : g.owned_hi_un[d];
      if (p.j[d] < lo || p.j[d] > hi) return false;
    }
  }
  return wall;
}

__device__ __forceinline__ int zone_box(const DevFields &f, const DevGrid &g, const Pt &p, int c) {
  int zb = 0;
#pragma unroll
  for (int e = 0; e < 3; e++) zb = zb * 3 + (g.ax[e] >= 0 ? f.zone[e][qcoord(g, p, T_E, c, e)] : 1);
  return zb;
}

// a[c] without a runtime index into a kernel-argument array (which makes the
// compiler copy the whole argument struct to scratch)
template <typename T>
__device__ __forceinline__ T sel3(T const (&a)[3], int c) {
  return c == 0 ? a[0] : (c == 1 ? a[1] : a[2]);
}

// integrated dipoles subtracted from f_minus_p of component c at index n, in
// list order; zone_rz >= 0: only those the reader's reference chunk owns
__device__ __forceinline__ double isrc_sub(const ISrcDev &is, int step, int c, long long n,
                                           int zone_rz, double v) {
  if (n < is.imin || n > is.imax) return v;
  int k = 0;
  if (is.n > 16) {  // lower bound of n in the sorted entries
    int hi = is.n;
    while (k < hi) {
      const int mid = (k + hi) >> 1;
      if (is.idx[mid] < n)
        k = mid + 1;
      else
        hi = mid;
    }
  }
  for (; k < is.n; k++) {
    const long long ik = is.idx[k];
    if (ik > n) break;
    if (ik == n && is.comp[k] == c && (zone_rz < 0 || is.zone[k] == zone_rz))
      v -= is.val[(long long)step * is.n + is.orig[k]];
  }
  return v;
}

// f_minus_p at the point itself, skipping polarizations that are 0 there
template <bool ISRC>
__device__ __forceinline__ double dmp_own(const DevFields &f, const ISrcDev &is, int step, int c,
                                          long long n, unsigned pm) {
  double v = f.Dn[c][n];
  for (int k = 0; k < f.npol; k++)
    if (((pm >> k) & 1) && f.pol[k].P[c]) v -= f.pol[k].P[c][n];
  if (ISRC) v = isrc_sub(is, step, c, n, -1, v);
  return v;
}

// f_minus_p of component c at a neighbour n as the reader's reference chunk
// (zone box rz) holds it: integrated dipoles are subtracted only at points that
// chunk owns (the oracle's per-chunk fmp; DESIGN.md "Integrated sources on seams")
template <bool ISRC>
__device__ __forceinline__ double dmp_at(const DevFields &f, const ISrcDev &is, int step, int c,
                                         long long n, int rz) {
  double v = sel3(f.Dn, c)[n];
  for (int k = 0; k < f.npol; k++) {
    const double *P = sel3(f.pol[k].P, c);
    if (P) v -= P[n];
  }
  if (ISRC) v = isrc_sub(is, step, c, n, rz, v);
  return v;
}

// calc_nonlinear_u (src/step_generic.cpp:546-553): the Pade approximant of the
// upstream Meep chi2/chi3 update
__device__ __forceinline__ double calc_nonlinear_u(double Dsqr, double Di, double chi1inv,
                                                   double chi2, double chi3) {
  double c2 = Di * chi2 * (chi1inv * chi1inv);
  double c3 = Dsqr * chi3 * (chi1inv * chi1inv * chi1inv);
  return (1 + c2 + 2 * c3) / (1 + 2 * c2 + 3 * c3);
}

// ----------------------------------------------------------------- E from D
// update_eh(E_stuff) -> step_update_EDHB (src/update_eh.cpp:67-283,
// src/step_generic.cpp:576-906) + lorentzian update_P (src/susceptibility.cpp:
// 188-262) fused when no Newton-Raphson neighbour reads are needed.
// D - P of component e at i [+ s along d] [- s_e along e] as the reader's
// chunk (zone box rz) holds it; WCHK: a wall point another chunk owns is never
// connected (boundaries.cpp:347-460), so the reader's copy there stays 0.
// Directions are template arguments: runtime indices into kernel-argument
// arrays make the compiler copy the argument struct to scratch.
template <int d, int e, bool UPS, bool DN, bool WCHK, bool ISRC>
__device__ __forceinline__ double nbr_t(const DevGrid &g, const DevFields &f, const ISrcDev &is,
                                        int step, const Pt &p, long long i, int rz) {
  long long n = i;
  Pt q = p;
  if (UPS) {
    n += g.sdir[d];
    if (g.ax[d] >= 0) q.j[d] += 1;
  }
  if (DN) {
    n -= g.sdir[e];
    if (g.ax[e] >= 0) q.j[e] -= 1;
  }
  if (WCHK && f.wall_e && on_wall(g, e, q, true) && zone_box(f, g, q, e) != rz) return 0.0;
  return dmp_at<ISRC>(f, is, step, e, n, rz);
}

// g[i] + g[i + s] + g[i - s_e] + g[i + (s - s_e)] (the four-point sums of
// src/step_generic.cpp:611-612, 740-743)
template <int d, int e, bool WCHK, bool ISRC>
__device__ __forceinline__ double nsum_t(const DevGrid &g, const DevFields &f, const ISrcDev &is,
                                         int step, const Pt &p, long long i, int rz) {
  return nbr_t<d, e, false, false, WCHK, ISRC>(g, f, is, step, p, i, rz) +
         nbr_t<d, e, true, false, WCHK, ISRC>(g, f, is, step, p, i, rz) +
         nbr_t<d, e, false, true, WCHK, ISRC>(g, f, is, step, p, i, rz) +
         nbr_t<d, e, true, true, WCHK, ISRC>(g, f, is, step, p, i, rz);
}

// OFFDIAG(u, g, sx), src/step_generic.cpp:597-598
template <int d, int e, bool WCHK, bool ISRC>
__device__ __forceinline__ double offdiag_t(const double *uo, const DevGrid &g, const DevFields &f,
                                            const ISrcDev &is, int step, const Pt &p, long long i,
                                            int rz) {
  const long long s = g.sdir[d];
  return 0.25 * ((nbr_t<d, e, false, false, WCHK, ISRC>(g, f, is, step, p, i, rz) +
                  nbr_t<d, e, false, true, WCHK, ISRC>(g, f, is, step, p, i, rz)) * uo[i] +
                 (nbr_t<d, e, true, false, WCHK, ISRC>(g, f, is, step, p, i, rz) +
                  nbr_t<d, e, true, true, WCHK, ISRC>(g, f, is, step, p, i, rz)) * uo[i + s]);
}

// One E component of update_e_kernel; d is a template argument so every
// per-component kernel-argument array (f.E[d], f.inveps[d], ...) is indexed with
// a constant (a runtime index makes the compiler copy DevFields to scratch).
template <int d, bool SHELL, bool NR, bool UP, bool ISRC, bool FUSEPOL>
__device__ __forceinline__ void e_point(const DevGrid &g, const DevFields &f, const ISrcDev &is,
                                        int step, const Pt &p, long long i, unsigned pm) {
    if (!f.ecomp_present[d]) return;
    // wall_e: also the high metallic wall plane, which the reference's chunk owns
    // and updates (D = 0 there) before step_boundaries zeroes it; the transient
    // E feeds update_P there (aniso_wall_kernel zeroes it afterwards)
    if (!owned(g, T_E, d, p) && !((NR || UP) && f.wall_e && on_wall(g, d, p))) return;
    const double gs = dmp_own<ISRC>(f, is, step, d, i, pm);
    // reference chunk of this voxel (zone box; interior kernels: 13 = interior chunk)
    int rz = 13;
    if ((SHELL && (NR || UP || ISRC)) || ((NR || UP) && f.wall_e)) {
      int z3[3];
#pragma unroll
      for (int e = 0; e < 3; e++) z3[e] = g.ax[e] >= 0 ? f.zone[e][qcoord(g, p, T_E, d, e)] : 1;
      rz = z3[0] * 9 + z3[1] * 3 + z3[2];
    }
    const double *u = f.inveps[d];
    const double *E = f.E[d];
    double *En = f.En[d];
    bool pml = false;
    int kw = 0;
    if (SHELL) {
      kw = qcoord(g, p, T_E, d, d);
      pml = pml_at(f, g, d, kw);
    }
    double wv;  // the W field read by update_pols (f_w if allocated, else E)
    double unl = 0;  // upstream mode: step_update_EDHB as upstream Meep runs it
                     // (src/step_generic.cpp:597-726, 730-886 with the fork's disabled
                     // branches restored; u = 1 where trivial)
    if (UP) {  // upstream mode (UP == f.upnl)
      constexpr int d1 = (d + 1) % 3, d2 = (d + 2) % 3;
      const long long s = g.sdir[d];
      const double us = u ? u[i] : 1.0;
      const bool h1 = f.ecomp_present[d1] != 0, h2 = f.ecomp_present[d2] != 0;
      // D - P of the partner components at i, i + s, i - s_e, i + (s - s_e), read
      // once: the four-point sums (611-612) and OFFDIAG (597-598) combine them
      double a[4] = {0, 0, 0, 0}, c[4] = {0, 0, 0, 0};
      if (h1) {
        a[0] = nbr_t<d, d1, false, false, true, ISRC>(g, f, is, step, p, i, rz);
        a[1] = nbr_t<d, d1, true, false, true, ISRC>(g, f, is, step, p, i, rz);
        a[2] = nbr_t<d, d1, false, true, true, ISRC>(g, f, is, step, p, i, rz);
        a[3] = nbr_t<d, d1, true, true, true, ISRC>(g, f, is, step, p, i, rz);
      }
      if (h2) {
        c[0] = nbr_t<d, d2, false, false, true, ISRC>(g, f, is, step, p, i, rz);
        c[1] = nbr_t<d, d2, true, false, true, ISRC>(g, f, is, step, p, i, rz);
        c[2] = nbr_t<d, d2, false, true, true, ISRC>(g, f, is, step, p, i, rz);
        c[3] = nbr_t<d, d2, true, true, true, ISRC>(g, f, is, step, p, i, rz);
      }
      const double g1s = a[0] + a[1] + a[2] + a[3], g2s = c[0] + c[1] + c[2] + c[3];
      auto offd = [&](const double *uo, const double *w) {  // OFFDIAG(u, g, sx)
        return 0.25 * ((w[0] + w[2]) * uo[i] + (w[1] + w[3]) * uo[i + s]);
      };
      // off-diagonal rows this reference chunk keeps (trivial rows are deallocated,
      // src/anisotropic_averaging.cpp:285-296)
      const unsigned ob = (f.offd_zone[rz] >> (3 * d)) & 3u;
      const double *u1 = f.offd[d][0], *u2 = f.offd[d][1];
      const bool o1 = (ob & 1u) && h1 && u1, o2 = (ob & 2u) && h2 && u2;
      double v, dsq;
      if (o1 && o2) {  // 3x3 (617, 772)
        v = gs * us + offd(u1, a) + offd(u2, c);
        dsq = gs * gs + 0.0625 * (g1s * g1s + g2s * g2s);
      } else if (o1) {  // 2x2, the present row first (590-594, 646, 835)
        v = gs * us + offd(u1, a);
        dsq = gs * gs + 0.0625 * (g1s * g1s);
      } else if (o2) {
        v = gs * us + offd(u2, c);
        dsq = gs * gs + 0.0625 * (g2s * g2s);
      } else {  // diagonal (668-702, 853-884)
        v = gs * us;
        dsq = gs * gs;
        if (h1 && h2)
          dsq = gs * gs + 0.0625 * (g1s * g1s + g2s * g2s);
        else if (h1)
          dsq = gs * gs + 0.0625 * (g1s * g1s);
        else if (h2)
          dsq = gs * gs + 0.0625 * (g2s * g2s);
      }
      // chunks without chi2/chi3 skip the factor; chi2 = chi3 = 0 makes it exactly 1
      unl = v * calc_nonlinear_u(dsq, gs, us, f.chi2[d][i], f.chi3[d][i]);
    }
    if (pml) {
      double fwprev = f.WE[d][i];
      double kapwkw = f.pml.kap[d][kw], sigwkw = f.pml.sig[d][kw];
      double fw = UP ? unl : (u ? (gs * u[i]) : gs);
      f.WE[d][i] = fw;
      En[i] = E[i] + ((kapwkw + sigwkw) * fw - (kapwkw - sigwkw) * fwprev);
      wv = fw;
    } else {
      bool done = false;
      if (NR) {
        // 3x3 chi1inv + chi2 branch (src/step_generic.cpp:730-816)
        const int zb = rz;
        const int d1 = (d + 1) % 3, d2 = (d + 2) % 3;
        const bool have_off =
            ((f.offd_zone[zb] >> (3 * d)) & 3) == 3 && f.chi2[d] && f.ecomp_present[d1] &&
            f.ecomp_present[d2];
        if (have_off) {
          const double *u1 = f.offd[d][0], *u2 = f.offd[d][1];
          double chi2new = f.chi2[d][i];
          int zc = (u[i] == 0) + (u1[i] == 0) + (u2[i] == 0);
          if (!(chi2new == 0 || zc > 1)) {
            double gs_2 = nsum_t<d, (d + 1) % 3, true, ISRC>(g, f, is, step, p, i, rz) * 0.25;
            double gs_3 = nsum_t<d, (d + 2) % 3, true, ISRC>(g, f, is, step, p, i, rz) * 0.25;
            double us = 1 / u[i];
            double us_2 = us, us_3 = us;
            double dummy1 = 0.0, dummy2 = 0.0;
            double fv = E[i];
            const unsigned long long rng = nr_voxel_seed(
                g.ax[0] >= 0 ? qcoord(g, p, T_E, d, 0) : 0, g.ax[1] >= 0 ? qcoord(g, p, T_E, d, 1) : 0,
                g.ax[2] >= 0 ? qcoord(g, p, T_E, d, 2) : 0, d, f.nr_t);
            if (d == 0) {
              NRP p1 = {gs, us, chi2new, 0.0, 0.0};
              NRP p2 = {gs_2, us_2, 0.0, chi2new, 0.0};
              NRP p3 = {gs_3, us_3, 0.0, 0.0, chi2new};
              run_nr(fv, gs_2 * u[i], gs_3 * u[i], &fv, &dummy1, &dummy2, p1, p2, p3, rng,
                     f.nr_fallbacks, &f, En, i, d);
            } else if (d == 1) {
              NRP p1 = {gs_3, us_3, chi2new, 0.0, 0.0};
              NRP p2 = {gs, us, 0.0, chi2new, 0.0};
              NRP p3 = {gs_2, us_2, 0.0, 0.0, chi2new};
              run_nr(gs_3 * u[i], fv, gs_2 * u[i], &dummy1, &fv, &dummy2, p1, p2, p3, rng,
                     f.nr_fallbacks, &f, En, i, d);
            } else {
              NRP p1 = {gs_2, us_2, chi2new, 0.0, 0.0};
              NRP p2 = {gs_3, us_3, 0.0, chi2new, 0.0};
              NRP p3 = {gs, us, 0.0, 0.0, chi2new};
              run_nr(gs_2 * u[i], gs_3 * u[i], fv, &dummy1, &dummy1, &fv, p1, p2, p3, rng,
                     f.nr_fallbacks, &f, En, i, d);
            }
            En[i] = fv;
            done = true;
          }
        }
      }
      if (!done) En[i] = UP ? unl : (u ? (gs * u[i]) : gs);
      wv = En[i];
    }
    if (FUSEPOL) {
      for (int k = 0; k < f.npol; k++) {
        const PolDev &pd = f.pol[k];
        if (!pd.P[d] || !((pm >> k) & 1)) continue;
        double pcur = pd.P[d][i];
        pd.P[d][i] = pd.gamma1inv * (pcur * (2 - pd.omega0dtsqr_denom) - pd.gamma1 * pd.Pp[d][i] +
                                     pd.omega0dtsqr * (pd.sigma[d][i] * wv));
        pd.Pp[d][i] = pcur;
      }
    }
  }

template <bool SHELL, bool NR, bool UP, bool ISRC, bool FUSEPOL>
__global__ __launch_bounds__(MNL_BX *MNL_BY) void update_e_kernel(Box b, BoxList bl, DevGrid g,
                                                                   DevFields f, ISrcDev is,
                                                                   int step) {
  Pt p;
  if (!map_pt<SHELL>(b, bl, g, p)) return;
  const long long i = p.idx;
  const unsigned pm = pol_mask(f, p);
  e_point<0, SHELL, NR, UP, ISRC, FUSEPOL>(g, f, is, step, p, i, pm);
  e_point<1, SHELL, NR, UP, ISRC, FUSEPOL>(g, f, is, step, p, i, pm);
  e_point<2, SHELL, NR, UP, ISRC, FUSEPOL>(g, f, is, step, p, i, pm);
}

// lorentzian update_P, isotropic (src/susceptibility.cpp:251-258), used after
// the Newton-Raphson E update (which reads neighbouring D - P).
template <bool SHELL>
__global__ __launch_bounds__(MNL_BX *MNL_BY) void update_pols_kernel(Box b, BoxList bl, DevGrid g,
                                                                      DevFields f) {
  Pt p;
  if (!map_pt<SHELL>(b, bl, g, p)) return;
  const long long i = p.idx;
#pragma unroll
  for (int d = 0; d < 3; d++) {
    if (!f.ecomp_present[d]) continue;
    if (!owned(g, T_E, d, p) && !(f.wall_e && on_wall(g, d, p))) continue;
    bool pml = false;
    if (SHELL) pml = pml_at(f, g, d, qcoord(g, p, T_E, d, d));
    const double wv = pml ? f.WE[d][i] : f.En[d][i];
    for (int k = 0; k < f.npol; k++) {
      const PolDev &pd = f.pol[k];
      if (!pd.P[d] || !in_box(pd.nz, p)) continue;
      double pcur = pd.P[d][i];
      pd.P[d][i] = pd.gamma1inv * (pcur * (2 - pd.omega0dtsqr_denom) - pd.gamma1 * pd.Pp[d][i] +
                                   pd.omega0dtsqr * (pd.sigma[d][i] * wv));
      pd.Pp[d][i] = pcur;
    }
  }
}

// lorentzian update_P with off-diagonal sigma (src/susceptibility.cpp:188-262):
// per point the branch of its reference chunk (3x3 / 2x2 / isotropic, from the
// arrays that chunk holds), the off-diagonal partners W averaged by OFFDIAG
// (185-186).  W of a component = f_w where its chunk has PML along its own
// direction, f elsewhere (update_pols.cpp:44); neighbours read the owner's W,
// as the WE_stuff ghost exchange (boundaries.cpp:407-408, 508-525) provides.
// W of E component c at point q (linear index n) as read by a point of
// reference chunk zb: f_w where q's chunk has PML along c, f elsewhere
// (update_pols.cpp:44).  Ghosts hold the owner's W (WE_stuff exchange), except
// on the metallic wall planes, which are never connected (boundaries.cpp:
// 347-460): there only the owning chunk sees its transient value, others 0.
__device__ __forceinline__ double w_at(const DevFields &f, const DevGrid &g, const Pt &q, int c,
                                       long long n, int zb) {
  if (on_wall(g, c, q, true) && zone_box(f, g, q, c) != zb) return 0.0;
  return pml_at(f, g, c, qcoord(g, q, T_E, c, c)) ? f.WE[c][n] : f.En[c][n];
}

// Between update_eh(E) and step_boundaries(E) the reference's wall-plane E (and
// f_w) hold u*(D - sum P) with D = 0 there, and update_pols reads them through
// OFFDIAG.  zero = 0: write that transient W; zero = 1: E back to 0 afterwards.
__global__ __launch_bounds__(MNL_BX *MNL_BY) void aniso_wall_kernel(Box b, DevGrid g, DevFields f,
                                                                     int zero) {
  Pt p;
  if (!make_pt(b, g, p)) return;
  const long long i = p.idx;
  for (int c = 0; c < 3; c++) {
    if (!f.ecomp_present[c] || !on_wall(g, c, p)) continue;
    if (zero) {
      f.En[c][i] = 0;
      continue;
    }
    double v = f.Dn[c][i];
    for (int k = 0; k < f.npol; k++)
      if (f.pol[k].P[c]) v -= f.pol[k].P[c][i];
    const double w = f.inveps[c] ? v * f.inveps[c][i] : v;
    if (pml_at(f, g, c, qcoord(g, p, T_E, c, c)))
      f.WE[c][i] = w;
    else
      f.En[c][i] = w;
  }
}

template <bool SHELL>
__global__ __launch_bounds__(MNL_BX *MNL_BY) void update_pols_aniso_kernel(Box b, BoxList bl,
                                                                            DevGrid g, DevFields f) {
  Pt p;
  if (!map_pt<SHELL>(b, bl, g, p)) return;
  const long long i = p.idx;
  for (int d = 0; d < 3; d++) {
    if (!f.ecomp_present[d] || !(owned(g, T_E, d, p) || on_wall(g, d, p))) continue;
    const int zb = zone_box(f, g, p, d);
    const double wv = w_at(f, g, p, d, i, zb);
    const long long is = g.sdir[d];
    Pt pu = p;  // the point i + s (one step along d)
    if (g.ax[d] >= 0) pu.j[d] += 1;
    for (int k = 0; k < f.npol; k++) {
      const PolDev &pd = f.pol[k];
      if (!pd.P[d] || !pd.sigma[d]) continue;
      const unsigned zbits = pd.zbits ? pd.zbits[zb] : (1u << (4 * d));
      if (!((zbits >> (4 * d)) & 1)) continue;  // row trivial in this chunk
      int d1 = (d + 1) % 3, d2 = (d + 2) % 3;
      const double *s1 = f.ecomp_present[d1] && ((zbits >> (3 * d + d1)) & 1) ? pd.soff[d][d1] : nullptr;
      const double *s2 = f.ecomp_present[d2] && ((zbits >> (3 * d + d2)) & 1) ? pd.soff[d][d2] : nullptr;
      if (s2 && !s1) {
        const int t = d1;
        d1 = d2;
        d2 = t;
        s1 = s2;
        s2 = nullptr;
      }
      const double *s = pd.sigma[d];
      double *P = pd.P[d], *Pp = pd.Pp[d];
      // OFFDIAG(u, g, sx, s) = 0.25*((g[i] + g[i-sx])*u[i] + (g[i+s] + g[(i+s)-sx])*u[i+s])
      auto offd = [&](const double *u, int dd) -> double {
        const long long sx = g.sdir[dd];
        Pt pm = p, pum = pu;
        if (g.ax[dd] >= 0) pm.j[dd] -= 1, pum.j[dd] -= 1;
        const double g0 = w_at(f, g, p, dd, i, zb), g1 = w_at(f, g, pm, dd, i - sx, zb);
        const double g2 = w_at(f, g, pu, dd, i + is, zb), g3 = w_at(f, g, pum, dd, (i + is) - sx, zb);
        return 0.25 * ((g0 + g1) * u[i] + (g2 + g3) * u[i + is]);
      };
      if (s1) {
        if (s[i] == 0) continue;  // the PR #666 guard of the anisotropic branches
        double x = s[i] * wv + offd(s1, d1);
        if (s2) x = x + offd(s2, d2);
        const double pcur = P[i];
        P[i] = pd.gamma1inv * (pcur * (2 - pd.omega0dtsqr_denom) - pd.gamma1 * Pp[i] +
                               pd.omega0dtsqr * x);
        Pp[i] = pcur;
      } else {
        if (!in_box(pd.nz, p)) continue;
        const double pcur = P[i];
        P[i] = pd.gamma1inv * (pcur * (2 - pd.omega0dtsqr_denom) - pd.gamma1 * Pp[i] +
                               pd.omega0dtsqr * (s[i] * wv));
        Pp[i] = pcur;
      }
    }
  }
}

// ----------------------------------------------------------------- sources
// fields_chunk::step_source (src/step.cpp:296-319): f -= real(amp*J*dt), times
// cndinv with conductivity (real((A*dt)*cndinv) = real(A*dt)*cndinv), applied
// in source-list order by a single lane (exact sequential semantics).
struct Ptr3 {
  double *p[3];
  const double *ci[3];
};
// f[c][i] -= real((amp * current) * dt) [* cndinv[i]] for the points [k0, k1)
// of one layer (src/step.cpp:296-319; complex products as std::complex<double>,
// no contraction)
__global__ void source_kernel(Ptr3 pt, SrcDev s, int k0, int k1) {
  const int k = k0 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (k >= k1) return;
  const int c = s.comp[k];
  const long long i = s.idx[k];
  const int g = s.gid[k];
  const double ar = s.amp[2 * k], ai = s.amp[2 * k + 1];
  const double jr = s.J[2 * g], ji = s.J[2 * g + 1];
  const double v = (ar * jr - ai * ji) * s.dt;
  pt.p[c][i] -= pt.ci[c] ? v * pt.ci[c][i] : v;
}

__global__ void fill_kernel(double *p, double v, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}

// canonical (Z fastest, whole cell) <-> device layout (rank-local box)
__global__ void from_canonical_kernel(double *dst, const double *src, DevGrid g, long long cs0,
                                      long long cs1, long long cs2) {
  int i0 = blockIdx.x * MNL_BX + threadIdx.x;
  int i1 = blockIdx.y * MNL_BY + threadIdx.y;
  int i2 = blockIdx.z;
  if (i0 >= g.N[0] || i1 >= g.N[1]) return;
  int ii[3] = {i0, i1, i2};
  long long cidx = 0;
  long long cs[3] = {cs0, cs1, cs2};
  for (int d = 0; d < 3; d++)
    if (g.ax[d] >= 0) cidx += (long long)(ii[g.ax[d]] + g.off[d]) * cs[d];
  dst[(long long)i0 + i1 * g.st[1] + i2 * g.st[2]] = src[cidx];
}

// Rank-owned entries of one component into a box of the whole-cell array
// (global indices blo..bhi per direction, strides bs); the launch covers the
// local index range lo.. of that box.
__global__ void to_box_kernel(double *dst, const double *src, const double *hsep, DevGrid g,
                              DevFields f, int type, int c, int l0, int l1, int l2, int n0, int n1,
                              long long bs0, long long bs1, long long bs2, int blo0, int blo1,
                              int blo2, int use_fb, const double *dsrc, const double *usrc) {
  const int i0 = l0 + blockIdx.x * MNL_BX + threadIdx.x;
  const int i1 = l1 + blockIdx.y * MNL_BY + threadIdx.y;
  const int i2 = l2 + blockIdx.z;
  if (i0 >= l0 + n0 || i1 >= l1 + n1) return;
  int ii[3] = {i0, i1, i2};
  Pt p;
  for (int d = 0; d < 3; d++) p.j[d] = g.ax[d] >= 0 ? ii[g.ax[d]] : 0;
  // rank-owned planes only along every axis (ghost entries are filled by
  // their owner; non-owned boundary entries are 0 in the reference).
  for (int d = 0; d < 3; d++) {
    if (g.ax[d] < 0) continue;
    int sh = shift_of(type, c, d);
    int lo = sh ? g.owned_lo_sh[d] : g.owned_lo_un[d];
    int hi = sh ? g.owned_hi_sh[d] : g.owned_hi_un[d];
    if (!sh && g.wall[d] && p.j[d] + g.off[d] == g.nglob[d]) hi = p.j[d];  // wall plane (= 0)
    if (p.j[d] < lo || p.j[d] > hi) return;
  }
  const long long bs[3] = {bs0, bs1, bs2};
  const int blo[3] = {blo0, blo1, blo2};
  long long cidx = 0;
  for (int d = 0; d < 3; d++)
    if (g.ax[d] >= 0) cidx += (long long)(p.j[d] + g.off[d] - blo[d]) * bs[d];
  long long i = (long long)i0 + i1 * g.st[1] + i2 * g.st[2];
  double v = src[i];
  if (hsep && (f.hall || pml_at(f, g, c, qcoord(g, p, T_H, c, c)))) v = hsep[i];
  p.idx = i;
  if (use_fb && type == T_E && e_implicit(f, g, c, p))  // fused: E = chi1inv * D (not stored)
    v = usrc ? (dsrc[i] * usrc[i]) : dsrc[i];
  dst[cidx] = v;
}

__global__ void box_fill_kernel(double *dst, DevGrid g, int type, int c, double x0, double x1,
                                double y0, double y1, double z0, double z1, double value,
                                int invert, double a, int io0, int io1, int io2) {
  int i0 = blockIdx.x * MNL_BX + threadIdx.x;
  int i1 = blockIdx.y * MNL_BY + threadIdx.y;
  int i2 = blockIdx.z;
  if (i0 >= g.N[0] || i1 >= g.N[1]) return;
  int ii[3] = {i0, i1, i2};
  double lo[3] = {x0, y0, z0}, hi[3] = {x1, y1, z1};
  int io[3] = {io0, io1, io2};
  for (int d = 0; d < 3; d++) {
    if (g.ax[d] < 0) continue;
    int jj = ii[g.ax[d]] + g.off[d];
    double pos = (io[d] + 2 * jj + shift_of(type, c, d)) * (0.5 * (1.0 / a));
    if (pos < lo[d] || pos > hi[d]) return;
  }
  dst[(long long)i0 + i1 * g.st[1] + i2 * g.st[2]] = invert ? 1.0 / value : value;
}

// ------------------------------------------------------ subpixel averaging
// structure_chunk::set_chi1inv with a material_function (src/anisotropic_averaging.cpp:
// 221-298) over a list of geometric objects of isotropic permittivity (later objects
// win): per point the rownum'th row of the effective tensor at dV(here) (diagonal
// entry) and at dV(here - shift1) (off-diagonal entries), material_function::
// eff_chi1inv_row / normal_vector (58-219), in the reference's operation order.
__device__ double geo_chi1p1(const AvgArgs &A, const double r[3]) {
  for (int o = A.nobj - 1; o >= 0; o--) {
    const GeoObj &g = A.objs[o];
    const double dx = r[0] - g.c[0], dy = r[1] - g.c[1], dz = r[2] - g.c[2];
    bool in;
    if (g.kind == 0) {
      in = fabs(dx) <= 0.5 * g.p[0] && fabs(dy) <= 0.5 * g.p[1] && fabs(dz) <= 0.5 * g.p[2];
    } else if (g.kind == 1) {
      in = dx * dx + dy * dy + dz * dz <= g.p[0] * g.p[0];
    } else {
      const int ax = (int)g.p[2];
      const double da = ax == 0 ? dx : ax == 1 ? dy : dz;
      const double u = ax == 0 ? dy : dx, v = ax == 2 ? dy : dz;
      in = fabs(da) <= 0.5 * g.p[1] && u * u + v * v <= g.p[0] * g.p[0];
    }
    if (in) return g.eps;
  }
  return A.default_eps;
}

__device__ void eff_chi1inv_row(const AvgArgs &A, const double vmin[3], const double vmax[3],
                                double row[3]) {
  const int rownum = A.c;
  double cen[3] = {0, 0, 0};
  for (int k = 0; k < A.ndir; k++) {
    const int d = A.dirs[k];
    cen[d] = (vmin[d] + vmax[d]) * 0.5;
  }
  double meps = 1, minveps = 1;
  double grad[3] = {0, 0, 0};
  if (A.maxeval) {
    // normal_vector: sphere quadrature of diameter R around the centre
    double R = 0.0;
    for (int k = 0; k < A.ndir; k++) R = fmax(R, vmax[A.dirs[k]] - vmin[A.dirs[k]]);
    const int nd = A.ndir, min_iters = 1 << nd;
    const double *q = A.quad + (nd - 1) * AVG_MAXQ * 4;
    double prev = 0;
    bool break_early = true, uniform = false;
    for (int i = 0; i < A.nq[nd - 1]; ++i) {
      const double w = q[4 * i + 3];
      double pt[3] = {0, 0, 0};
      if (nd == 1) {
        pt[2] = cen[2] + q[4 * i + 2] * R;
      } else {
        for (int k = 0; k < nd; k++) pt[k] = cen[k] + q[4 * i + k] * R;
      }
      const double val = geo_chi1p1(A, pt);
      if (i > 0 && i < min_iters) {
        if (val != prev) break_early = false;
        if (i == min_iters - 1 && break_early) {
          uniform = true;
          break;
        }
      }
      prev = val;
      for (int k = 0; k < nd; k++) {
        const int d = A.dirs[k];
        grad[d] += (pt[d] - cen[d]) * (w * val);
      }
    }
    double g2 = 0.0;
    for (int k = 0; k < nd; k++) g2 += grad[A.dirs[k]] * grad[A.dirs[k]];
    if (!uniform && !(sqrt(g2) < 1e-8)) {
      double dd[3] = {0, 0, 0};
      for (int k = 0; k < nd; k++) dd[A.dirs[k]] = vmax[A.dirs[k]] - vmin[A.dirs[k]];
      int ms = 10, iter = 0;
      double old_meps = 0, old_minveps = 0;
      bool trivial = false;
      for (;;) {
        const bool go = nd == 3 ? (fabs(meps - old_meps) > A.tol * fabs(old_meps)) &&
                                      (fabs(minveps - old_minveps) > A.tol * fabs(old_minveps))
                                : (fabs(meps - old_meps) > A.tol * old_meps) &&
                                      (fabs(minveps - old_minveps) > A.tol * old_minveps);
        if (!go) break;
        old_meps = meps;
        old_minveps = minveps;
        meps = minveps = 0;
        if (nd == 3) {
          for (int k = 0; k < ms && !trivial; k++)
            for (int j = 0; j < ms && !trivial; j++)
              for (int i = 0; i < ms; i++) {
                const double pt[3] = {vmin[0] + i * dd[0] / ms, vmin[1] + j * dd[1] / ms,
                                      vmin[2] + k * dd[2] / ms};
                const double ep = geo_chi1p1(A, pt);
                if (ep < 0) {
                  trivial = true;
                  break;
                }
                meps += ep;
                minveps += 1 / ep;
              }
          if (trivial) break;
          meps /= ms * ms * ms;
          minveps /= ms * ms * ms;
          ms *= 2;
          if (A.maxeval && (iter += ms * ms * ms) >= A.maxeval) break;
        } else if (nd == 2) {
          for (int j = 0; j < ms && !trivial; j++)
            for (int i = 0; i < ms; i++) {
              const double pt[3] = {vmin[0] + i * dd[0] / ms, vmin[1] + j * dd[1] / ms, 0.0};
              const double ep = geo_chi1p1(A, pt);
              if (ep < 0) {
                trivial = true;
                break;
              }
              meps += ep;
              minveps += 1 / ep;
            }
          if (trivial) break;
          meps /= ms * ms;
          minveps /= ms * ms;
          ms *= 2;
          if (A.maxeval && (iter += ms * ms) >= A.maxeval) break;
        } else {
          bool neg = false;
          for (int i = 0; i < ms; i++) {
            const double pt[3] = {0.0, 0.0, vmin[2] + i * dd[2] / ms};
            const double ep = geo_chi1p1(A, pt);
            if (ep < 0) {
              meps = geo_chi1p1(A, cen);
              minveps = 1 / meps;
              neg = true;
              break;
            }
            meps += ep;
            minveps += 1 / ep;
          }
          if (neg) break;
          meps /= ms;
          minveps /= ms;
          ms *= 2;
          if (A.maxeval && (iter += ms * ms) >= A.maxeval) break;
        }
      }
      if (!trivial) {
        double n[3] = {0, 0, 0};
        const double nabsinv = 1.0 / sqrt(g2);
        for (int k = 0; k < nd; k++) n[A.dirs[k]] = grad[A.dirs[k]] * nabsinv;
        for (int i = 0; i < 3; ++i) row[i] = n[rownum] * n[i] * (minveps - 1 / meps);
        row[rownum] += 1 / meps;
        return;
      }
    }
  }
  row[0] = row[1] = row[2] = 0.0;
  row[rownum] = 1 / geo_chi1p1(A, cen);
}

__global__ void avg_chi1inv_kernel(AvgArgs A) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= A.ntot) return;
  // canonical index -> point (z fastest, then y, then x)
  int idx[3] = {0, 0, 0};
  long long r = i;
  for (int d = 2; d >= 0; d--)
    if (A.has[d]) {
      idx[d] = (int)(r % (A.n[d] + 1));
      r /= A.n[d] + 1;
    }
  const double h = 0.5 * A.inva;  // grid_volume::dV: hinva = 0.5 * inva * diameter (1.0)
  double vmin[3] = {0, 0, 0}, vmax[3] = {0, 0, 0}, omin[3] = {0, 0, 0}, omax[3] = {0, 0, 0};
  for (int k = 0; k < A.ndir; k++) {
    const int d = A.dirs[k];
    const int here = A.io[d] + 2 * idx[d] + (d == A.c ? 1 : 0);
    const double hp = here * (0.5 * A.inva), hm = (here - (d == A.c ? 1 : 0)) * (0.5 * A.inva);
    vmax[d] = hp + h;
    vmin[d] = hp - h;
    omax[d] = hm + h;  // here - shift1 (E: shifted back half a pixel along c)
    omin[d] = hm - h;
  }
  double row[3];
  eff_chi1inv_row(A, vmin, vmax, row);
  if (A.out[A.c]) A.out[A.c][i] = row[A.c];
  bool off = false;
  for (int d = 0; d < 3; d++) off = off || (d != A.c && A.out[d]);
  if (!off) return;
  eff_chi1inv_row(A, omin, omax, row);
  for (int d = 0; d < 3; d++)
    if (d != A.c && A.out[d]) A.out[d][i] = row[d];
}

// ----------------------------------------------------------------- launchers
static dim3 grid_for(const Box &b) {
  int n0 = b.hi[0] - b.lo[0] + 1, n1 = b.hi[1] - b.lo[1] + 1, n2 = b.hi[2] - b.lo[2] + 1;
  return dim3((n0 + MNL_BX - 1) / MNL_BX, (n1 + MNL_BY - 1) / MNL_BY, n2);
}
static bool empty(const Box &b) {
  for (int k = 0; k < 3; k++)
    if (b.hi[k] < b.lo[k]) return true;
  return false;
}
static int rc() { return hipGetLastError() == hipSuccess ? 0 : -1; }

static dim3 lin_grid(const BoxList &bl) {
  long long n = bl.start[bl.n];
  return dim3((unsigned)((n + 255) / 256));
}

int k_curl(int ft, const Box &in, const BoxList *sh, const DevGrid &g, const DevFields &f,
           const CurlPlan &p, double courant, void *stream, bool fuseup) {
  hipStream_t s = (hipStream_t)stream;
  BoxList none{};
  if (!sh) {
    if (empty(in)) return 0;
    dim3 blk(MNL_BX, MNL_BY), grd = grid_for(in);
    if (ft == T_B)
      curl_kernel<T_B, false, false><<<grd, blk, 0, s>>>(in, none, g, f, p, courant);
    else
      curl_kernel<T_D, false, false><<<grd, blk, 0, s>>>(in, none, g, f, p, courant);
  } else {
    if (sh->n == 0 || sh->start[sh->n] == 0) return 0;
    dim3 grd = lin_grid(*sh);
    grd.y = 3;
    if (ft == T_B) {
      if (fuseup)
        curl_kernel<T_B, true, true><<<grd, 256, 0, s>>>(in, *sh, g, f, p, courant);
      else
        curl_kernel<T_B, true, false><<<grd, 256, 0, s>>>(in, *sh, g, f, p, courant);
    } else {
      if (fuseup)
        curl_kernel<T_D, true, true><<<grd, 256, 0, s>>>(in, *sh, g, f, p, courant);
      else
        curl_kernel<T_D, true, false><<<grd, 256, 0, s>>>(in, *sh, g, f, p, courant);
    }
  }
  return rc();
}

int k_update_hmat(const Box &b, const DevGrid &g, const DevFields &f, int pols, void *stream) {
  if (empty(b)) return 0;
  update_hmat_kernel<<<grid_for(b), dim3(MNL_BX, MNL_BY), 0, (hipStream_t)stream>>>(b, g, f,
                                                                                      pols);
  return rc();
}

int k_update_h(const BoxList &sh, const DevGrid &g, const DevFields &f, void *stream) {
  if (sh.n == 0 || sh.start[sh.n] == 0) return 0;
  update_h_kernel<<<lin_grid(sh), 256, 0, (hipStream_t)stream>>>(sh, g, f);
  return rc();
}

template <bool SHELL, bool NR, bool UP, bool ISRC, bool FUSE>
static void launch_e1(const Box &in, const BoxList &bl, const DevGrid &g, const DevFields &f,
                      const ISrcDev &is, int step, hipStream_t s) {
  if (SHELL)
    update_e_kernel<true, NR, UP, ISRC, FUSE><<<lin_grid(bl), 256, 0, s>>>(in, bl, g, f, is, step);
  else
    update_e_kernel<false, NR, UP, ISRC, FUSE><<<grid_for(in), dim3(MNL_BX, MNL_BY), 0, s>>>(
        in, bl, g, f, is, step);
}

// kernel variant per mode: Newton-Raphson (fork, chi2 + 3x3 chi1inv), upstream
// (Pade chi, OFFDIAG), or plain (E = chi1inv * (D - P), Lorentzian P fused when
// allowed); integrated sources or not
template <bool SHELL>
static void launch_e(const Box &in, const BoxList &bl, const DevGrid &g, const DevFields &f,
                     const ISrcDev &is, int step, bool fuse, hipStream_t s) {
  const bool nr = f.nr_enabled != 0, up = f.upnl != 0, isrc = is.n > 0;
  if (nr) {
    if (isrc)
      launch_e1<SHELL, true, false, true, false>(in, bl, g, f, is, step, s);
    else
      launch_e1<SHELL, true, false, false, false>(in, bl, g, f, is, step, s);
  } else if (up) {
    if (isrc)
      launch_e1<SHELL, false, true, true, false>(in, bl, g, f, is, step, s);
    else
      launch_e1<SHELL, false, true, false, false>(in, bl, g, f, is, step, s);
  } else if (fuse) {
    if (isrc)
      launch_e1<SHELL, false, false, true, true>(in, bl, g, f, is, step, s);
    else
      launch_e1<SHELL, false, false, false, true>(in, bl, g, f, is, step, s);
  } else {
    if (isrc)
      launch_e1<SHELL, false, false, true, false>(in, bl, g, f, is, step, s);
    else
      launch_e1<SHELL, false, false, false, false>(in, bl, g, f, is, step, s);
  }
}

int k_update_e(const Box &in, const BoxList *sh, const DevGrid &g, const DevFields &f,
               const ISrcDev &is, int step, bool fuse_pols, void *stream) {
  BoxList none{};
  if (!sh) {
    if (empty(in)) return 0;
    launch_e<false>(in, none, g, f, is, step, fuse_pols, (hipStream_t)stream);
  } else {
    if (sh->n == 0 || sh->start[sh->n] == 0) return 0;
    launch_e<true>(in, *sh, g, f, is, step, fuse_pols, (hipStream_t)stream);
  }
  return rc();
}

int k_nr_hard(const DevFields &f, void *stream) {
  if (!f.nr_hard) return 0;
  nr_hard_kernel<<<64, 256, 0, (hipStream_t)stream>>>(f);
  return rc();
}

int k_update_pols(const Box &in, const BoxList *sh, const DevGrid &g, const DevFields &f,
                  void *stream) {
  hipStream_t s = (hipStream_t)stream;
  BoxList none{};
  if (!sh) {
    if (empty(in)) return 0;
    if (f.aniso) {
      update_pols_aniso_kernel<false><<<grid_for(in), dim3(MNL_BX, MNL_BY), 0, s>>>(in, none, g, f);
    } else {
      // isotropic P changes only inside its susceptibility's nonzero box: launch over
      // the interior's intersection with their union
      Box u = in;  // device axes; the nz boxes are indexed by direction (Pt::j)
      for (int d = 0; d < 3; d++) {
        const int a = g.ax[d];
        if (a < 0) continue;
        int lo = INT32_MAX, hi = -1;
        for (int k = 0; k < f.npol; k++) lo = min(lo, f.pol[k].nz.lo[d]), hi = max(hi, f.pol[k].nz.hi[d]);
        u.lo[a] = max(lo, in.lo[a]);
        u.hi[a] = min(hi, in.hi[a]);
      }
      if (empty(u)) return 0;
      update_pols_kernel<false><<<grid_for(u), dim3(MNL_BX, MNL_BY), 0, s>>>(u, none, g, f);
    }
  } else {
    if (sh->n == 0 || sh->start[sh->n] == 0) return 0;
    if (f.aniso)
      update_pols_aniso_kernel<true><<<lin_grid(*sh), 256, 0, s>>>(in, *sh, g, f);
    else
      update_pols_kernel<true><<<lin_grid(*sh), 256, 0, s>>>(in, *sh, g, f);
  }
  return rc();
}

int k_aniso_wall(const DevGrid &g, const DevFields &f, int zero, void *stream) {
  // wall points (on_wall) lie on the high wall plane of some direction: one launch per
  // such plane this rank holds (an edge point done twice writes the same value)
  for (int d = 0; d < 3; d++) {
    const int a = g.ax[d];
    if (a < 0 || !g.wall[d]) continue;
    const int j = g.nglob[d] - g.off[d];
    if (j < 0 || j > g.N[a] - 1) continue;
    Box pl;
    for (int e = 0; e < 3; e++) pl.lo[e] = 0, pl.hi[e] = g.N[e] - 1;
    pl.lo[a] = pl.hi[a] = j;
    aniso_wall_kernel<<<grid_for(pl), dim3(MNL_BX, MNL_BY), 0, (hipStream_t)stream>>>(pl, g, f,
                                                                                     zero);
  }
  return rc();
}

int k_source(int ft, const DevGrid &g, const DevFields &f, const SrcDev &s, int step,
             void *stream) {
  (void)g;
  if (s.n == 0) return 0;
  Ptr3 pt;
  for (int d = 0; d < 3; d++) {
    pt.p[d] = ft == T_D ? f.Dn[d] : f.Bn[d];
    pt.ci[d] = f.cndinv[ft == T_D][d];
  }
  (void)step;
  for (int l = 0; l < s.nlayer; l++) {
    const int k0 = s.layer[l], k1 = s.layer[l + 1];
    if (k1 <= k0) continue;
    source_kernel<<<(unsigned)((k1 - k0 + 255) / 256), 256, 0, (hipStream_t)stream>>>(pt, s, k0, k1);
  }
  return rc();
}


// ----------------------------------------------------------------- fused step
// One pass over the interior box F for a whole fields::step() of a
// non-dispersive, PML-free region (src/step.cpp:66-110 restricted to such
// chunks): curl B (step_curl, src/step_generic.cpp:106-109), H == B, curl D
// (same loop, negated strides), E = chi1inv * D (src/step_generic.cpp:
// 888-903).  E is never stored inside F: it is recomputed as D*u whenever it
// is read, which is bit-identical to the stored value of the reference.
//
// Work decomposition (2.5-D z-march).  A work item is a column tile of 64
// (x) x 14 (y) cells and a chunk of zchunk z-planes.  Tiles start on 128-byte
// boundaries in x (x0 = 16*floor(F.lo/16) + 64*t), so every row a wave loads
// or stores is exactly four whole cache lines: partial-line writes (two
// workgroups sharing a line at different times) cost ~20 % of HBM bandwidth
// on this access pattern (tools/micro/stream_bench.hip: aligned 5.95 TB/s vs
// misaligned 4.70 TB/s).  A 1024-thread workgroup is 16 waves:
//   waves 0..14: one row each, lane = column (x0+lane).  Row 0 is the y-1
//                halo row (B_new recomputed, nothing stored); rows 1..14 own.
//   wave 15:     lanes 0..13  the x-1 halo column of rows 1..14 (B_new recomputed),
//                lanes 16..30 E of the x+64 column (rows 0..14),
//                lane 31      E(x0-1, y+15).
//   wave 14 also loads the y+1 row of E.
// LDS holds E(k) of the (66 x 16) footprint and B_new(k) of the (65 x 15)
// footprint.  Items are handed out by an atomic counter in chunk-major order,
// so workgroups sweep z roughly in lockstep and the halo lines a tile shares
// with its neighbours are read from the last-level cache, not HBM.
//
// Memory pipeline: everything plane k needs from HBM (D,u or E of plane k+1,
// B of plane k, the halo E of plane k) is one "batch"; batches are issued DIST
// planes ahead into a register ring.  The loop body has no data-dependent
// branches around memory operations: loads past the chunk are clamped to valid
// planes, and stores of lanes/planes that must not write go through buffer
// stores with an out-of-range offset (dropped by the hardware).  That keeps
// the compiler's vmcnt accounting exact (in-order counter: a conditional store
// would force a full drain at the join).
// HBM traffic per cell: read B, D, u, write B, D (15 x 8 B).
#define FX 64
#define FR 15  // rows per tile incl. the y-1 halo row
#define FOWN (FR - 1)

typedef unsigned int mnl_u2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double ldg(const double *p, unsigned off) {
  return *(const double *)((const char *)p + off);
}
__device__ __forceinline__ void bst(__amdgpu_buffer_rsrc_t r, unsigned off, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(mnl_u2, v), r, off, 0, 0);
}
constexpr unsigned MNL_OOB = 0xFFFFFFF0u;  // > any valid byte offset (arrays < 4 GiB)

// Kernel-argument pointers copied into SGPRs.  Without this hipcc turns a
// per-lane choice between two argument pointers into a per-lane load of the
// pointer from the kernarg segment, which puts a dependent memory round trip
// in front of every field load.
typedef const double __attribute__((address_space(1))) *gdp;  // global (not flat) pointer
typedef const unsigned __attribute__((address_space(1))) *gup;
__device__ __forceinline__ gdp sgpr_ptr(const void *p) {
  const unsigned long long v = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return (gdp)(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ double ldg(gdp p, unsigned off) {
  return *(gdp)((const char __attribute__((address_space(1))) *)p + off);
}
__device__ __forceinline__ unsigned ldu(gup p, unsigned off) {
  return *(gup)((const char __attribute__((address_space(1))) *)p + off);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc(const void *p, unsigned nrec) {
  // null: zero records, every access out of range (loads 0, stores dropped)
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, p ? (int)nrec : 0,
                                           0x00020000);
}
// descriptor of a scalar pointer built where it is used (the empty asm keeps the compiler
// from hoisting it out of the loop); null: zero records, every access out of range
__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc_at(unsigned long long v, unsigned nrec) {
  asm volatile("" : "+s"(v));
  return __builtin_amdgcn_make_buffer_rsrc((void *)v, 0, v ? (int)nrec : 0, 0x00020000);
}
// a PML-state array as pml_body holds it: a scalar pointer turned into a descriptor at each
// use (R) or a descriptor built once
template <bool R>
struct RsArr {
  __device__ static unsigned long long make(const void *p, unsigned) {
    return (unsigned long long)sgpr_ptr(p);
  }
  __device__ static __amdgpu_buffer_rsrc_t get(unsigned long long v, unsigned nrec) {
    return brsrc_at(v, nrec);
  }
};
template <>
struct RsArr<false> {
  __device__ static __amdgpu_buffer_rsrc_t make(const void *p, unsigned nrec) {
    return brsrc(p, nrec);
  }
  __device__ static __amdgpu_buffer_rsrc_t get(__amdgpu_buffer_rsrc_t r, unsigned) { return r; }
};
__device__ __forceinline__ double bld(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}

struct FBatch {  // what B(k) needs besides E(k): own raw at k+1, B_old(k), halo raw at k
  double d0, d1, d2, u0, u1, u2, b0, b1, b2, h0, h1, hu0, hu1;
  unsigned ui, hui;  // UMODE 2: chi1inv palette indices (byte per component)
  bool f, hf;
};
// UMODE: 0 = no chi1inv (E = D), 1 = f64 chi1inv arrays, 2 = chi1inv palette:
// a byte index per cell and component (packed in one 32-bit word) into a
// table of at most 256 distinct f64 values per component, kept in LDS.  The
// palette holds the very same doubles, so E = D * u is bit-identical, and the
// kernel reads 4 B of chi1inv per cell instead of 24 (120 -> 100 B per cell).

// Lean-body geometry of one work item (see FusedArgs: bounds come from the host).
struct ItemGeo {
  int x0, x1;  // tile columns [x0, x1] (x0 128-byte aligned)
  int xb0, xb1;  // paired item (pml_body<PAIR>): the second sub-tile's columns; xb0 < 0: none
  int y0;      // halo row; own rows y0+1 .. y1
  int y1;
  int zs, ze;  // planes [zs, ze)
  bool lmx, lmy;  // general body: x-1 halo column / y-1 halo row read B_new (lean-stored)
  unsigned uw;    // general body: palette word uniform over the item, or ~0u
};

// PML coefficient table entry of one half-coordinate (FusedTab), staged in LDS
struct TabE {
  double kms, si, kps;
};
// the table entry outside every PML chunk (kappa = 1, sigma = 0)
__device__ constexpr TabE kTabId = {1.0, 1.0, 1.0};
constexpr int TPZ = FUSED_MAXCH + 4;
// LDS row width of the tile bodies: 64 columns + the x-1 and x+64 halo columns, or (paired
// items) two 32-column sub-tiles with their own halo columns (34 + 34)
constexpr int FXL = FX + 4;

// curl update with the per-point branch selection of step_curl
// (src/step_generic.cpp:84-252), written branch-free: outside a PML chunk
// along dsig the tables hold kap = 1, sig = 0, siginv = 1, so
// ((kap - sig) * X - dtdx * T) * siginv is bitwise X - dtdx * T; the f_u form
// (chunk with PML along dsigu) is selected by its flag.  Returns the new field;
// *un is the new f_u (valid when pu).
__device__ __forceinline__ double pml_curl(double fo, double uo, double T, double C, bool pu,
                                           double kms_a, double si_a, double kms_u,
                                           double si_u, double *un) {
  const double X = pu ? uo : fo;
  const double t = (kms_a * X - C * T) * si_a;
  *un = t;
  return pu ? si_u * (kms_u * fo + t - uo) : t;
}

template <int UMODE>
struct GBatch {  // general body: B(k) needs these besides E(k) (own: D(k+1), u(k+1), B_old(k))
  double d0, d1, d2, u0, u1, u2, b0, b1, b2, h0, h1, hu0, hu1;
  unsigned ui, hui;
  bool hi0, hi2;  // halo E implicit (chi1inv * D) for comps hc0 / 2
};
struct GAux {  // general body, PML state of plane k (own lanes), loaded masked
  double es0, es1, es2;  // stored E_old(k+1)
  double ub0, ub1, ub2;  // f_u of B, old, plane k
  double ho0, ho1, ho2;  // separate H, old, plane k
  double ud0, ud1, ud2;  // f_u of D, plane k
};

// The tile and general bodies read the kernel's FusedArgs through kargs_opaque(): the kernarg segment
// (constant address space, scalar loads) behind an empty asm, taken once per item.  Every
// value a body derives from its arguments is then live inside that body only; reading the
// by-value kernel parameter instead lets the compiler hoist every body's pointers to the
// kernel entry, where the union of all bodies' values overflows the SGPRs and each plane
// loop reloads them from VGPR lanes (v_readlane: 40-60 % of a PML body's instructions in
// the combined kernel, none with one body per kernel).
typedef const FusedArgs __attribute__((address_space(4))) KFA;
// The thread index behind an empty asm, per item: lane-derived offsets are then computed in
// the body that uses them instead of being hoisted to the kernel entry as a union over all
// bodies (kept in VGPRs across the item loop: scratch spills reloaded inside plane loops).
#ifndef MNL_TID_OPQ
#define MNL_TID_OPQ 1
#endif
__device__ __forceinline__ int tid_item() {
  int t = threadIdx.x;
  if (MNL_TID_OPQ) asm volatile("" : "+v"(t));
  return t;
}
__device__ __forceinline__ KFA *kargs_opaque() {
  KFA *p = (KFA *)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return p;
}

// General body over one item: any mix of PML chunks, walls, ghosts and owned
// ranges (src/step_generic.cpp:69-253 and 576-906 per point; H and E by
// update_eh, src/update_eh.cpp:67-363, with the W aux of PML chunks
// represented by its value: W_H == B_old, W_E == chi1inv * D_old, which the
// reference stores one step earlier).
template <int UMODE, int TX, int R, int NW, int POL, int AX>
__device__ __forceinline__ void fused_general(KFA &a, const ItemGeo &it,
                                              double (*sE)[R + 1][TX + 2],
                                              double (*sB)[R][TX + 1], const double (*sU)[256],
                                              TabE (*sTx)[2], TabE (*sTy)[2], TabE (*sTz)[2],
                                              unsigned char (*sFx)[2], unsigned char (*sFy)[2],
                                              unsigned char (*sFz)[2]) {
  // Tile: TX columns x R rows (row 0 = the y-1 halo row), own waves 0..NW-1 hold
  // 64/TX rows each (lane -> column lane % TX); the waves after them hold the
  // x-1 column (B recomputed), the E of the x+TX column and the corner.
  constexpr bool HAS_U = UMODE != 0;
  constexpr int RPW = 64 / TX, TPX = TX + 2, TPY = R + 1;
  static_assert(NW * RPW == R, "rows");
  const int tid = tid_item(), lane = tid & 63, w = tid >> 6;
  const bool hwave = __builtin_amdgcn_readfirstlane(w) >= NW - 1;
  const double C = a.C;
  const unsigned s2 = (unsigned)(a.st2 * 8);
  const int x0 = it.x0, y0 = it.y0, zs = it.zs, ze = it.ze;
  const int zlo = zs - 1;  // z table position 0
  // ---- PML tables of this item's footprint -> LDS
  for (int i = threadIdx.x; i < 2 * (TPX + TPY + TPZ); i += blockDim.x) {
    int ax, pos, base;
    if (i < 2 * TPX) {
      ax = 0, pos = i >> 1, base = x0 - 1;
    } else if (i < 2 * (TPX + TPY)) {
      ax = 1, pos = (i - 2 * TPX) >> 1, base = y0;
    } else {
      ax = 2, pos = (i - 2 * (TPX + TPY)) >> 1, base = zlo;
    }
    const int s = i & 1;
    const int jj = min(max(base + pos, 0), a.N[ax] - 1);
    const int q = 2 * (jj + a.off[ax]) + s;
    TabE e;
    e.kms = a.tab.kms[ax][q];
    e.si = a.tab.siginv[ax][q];
    e.kps = a.tab.kps[ax][q];
    const unsigned char fl = a.tab.flag[ax][q];
    if (ax == 0) {
      sTx[pos][s] = e;
      sFx[pos][s] = fl;
    } else if (ax == 1) {
      sTy[pos][s] = e;
      sFy[pos][s] = fl;
    } else {
      sTz[pos][s] = e;
      sFz[pos][s] = fl;
    }
  }
  __syncthreads();

  // ---- lane roles
  int row = 0, col = 0, ox = -1;
  bool ownlike = false;
  int hrow = 0, hcol = 0, hc0 = 0, hdx = 0, hdy = 0;
  bool hslot = false;
  if (w < NW) {
    row = w * RPW + lane / TX;
    ox = lane % TX;
    col = ox + 1;
    ownlike = true;
    if (row == R - 1) {  // also loads E of the y+R row
      hslot = true, hrow = R, hcol = col, hc0 = 0, hdx = ox, hdy = R;
    }
  } else {
    const int h = (w - NW) * 64 + lane;
    if (h < R - 1) {  // x-1 column of own rows 1..R-1
      ownlike = true, row = h + 1, col = 0, ox = -1;
    } else if (h < 2 * R - 1) {  // E of the x+TX column, rows 0..R-1
      hslot = true, hrow = h - (R - 1), hcol = TX + 1, hc0 = 1, hdx = TX, hdy = hrow;
    } else if (h == 2 * R - 1) {  // E(x0-1, y0+R)
      hslot = true, hrow = R, hcol = 0, hc0 = 0, hdx = -1, hdy = R;
    }
  }
  const int oy = row;
  const int gx = x0 + ox, gy = y0 + oy;
  // lean-halo lanes: the x-1 column (col 0) / the y-1 row (row 0) of a tile whose halo
  // the lean kernel has already stored this step.  Nobody reads their E (LDS column 0 /
  // row 0 of sE feed only their own recompute), and their new B equals the stored B_new
  // (H == B outside PML), so they load the two components the neighbours read and
  // nothing else.
  const bool lmode = ownlike && ((col == 0 && it.lmx) || (w < NW && row == 0 && it.lmy));
  const bool lmcol = col == 0;  // x-1 column: Hy, Hz read by col 1; y-1 row: Hx, Hz by row 1
  // lanes past the tile's columns x1+1 / rows y1+1 (narrow or short tiles) load nothing
  const bool inA = ownlike && gx >= 0 && gx < a.N[0] && gy >= 0 && gy < a.N[1] &&
                   gx <= it.x1 + 1 && gy <= it.y1 + 1;
  const unsigned cb = (unsigned)((gx + (long long)gy * a.st1) * 8);
  const unsigned cbl = inA ? cb : 0u;
  const int px = ox + 1, py = oy;  // table positions
  auto rng = [](int v, int lo, int hi) { return v >= lo && v <= hi; };
  // per-axis ownership (within G) of this lane's point: bit0 = shifted comps, bit1 = unshifted
  const unsigned ownx = (rng(gx, a.osh_lo[0], a.osh_hi[0]) ? 1u : 0u) |
                        (rng(gx, a.oun_lo[0], a.oun_hi[0]) ? 2u : 0u);
  const unsigned owny = (rng(gy, a.osh_lo[1], a.osh_hi[1]) ? 1u : 0u) |
                        (rng(gy, a.oun_lo[1], a.oun_hi[1]) ? 2u : 0u);
  const bool stl = ownlike && w < NW && row >= 1 && gx >= x0 && gx <= it.x1 && gy <= it.y1;
  // halo slot point (E of comps hc0 and 2 at (hx, hy, k))
  const int hx = x0 + hdx, hy = y0 + hdy;
  const bool hA = hslot && hx >= 0 && hx < a.N[0] && hy >= 0 && hy < a.N[1] &&
                  hx <= it.x1 + 1 && hy <= it.y1 + 1;
  const unsigned hbl = hA ? (unsigned)((hx + (long long)hy * a.st1) * 8) : cbl;
  const int hpx = hdx + 1, hpy = hdy;
  const unsigned hownx = (rng(hx, a.osh_lo[0], a.osh_hi[0]) ? 1u : 0u) |
                         (rng(hx, a.oun_lo[0], a.oun_hi[0]) ? 2u : 0u);
  const unsigned howny = (rng(hy, a.osh_lo[1], a.osh_hi[1]) ? 1u : 0u) |
                         (rng(hy, a.oun_lo[1], a.oun_hi[1]) ? 2u : 0u);
  // polarization box (E stored there, P updated in the E phase)
  const bool pxy = POL && gx >= a.pbox.lo[0] && gx <= a.pbox.hi[0] && gy >= a.pbox.lo[1] &&
                   gy <= a.pbox.hi[1];
  const bool hpxy = POL && hx >= a.pbox.lo[0] && hx <= a.pbox.hi[0] && hy >= a.pbox.lo[1] &&
                    hy <= a.pbox.hi[1];
  auto pz_in = [&](int z) { return POL && z >= a.pbox.lo[2] && z <= a.pbox.hi[2]; };
  // chi(2) Newton-Raphson box (inside pbox): E and P there are left to the NR E kernel
  // that follows (its neighbour reads need the old P of the whole box)
  const bool xxy = POL && gx >= a.xbox.lo[0] && gx <= a.xbox.hi[0] && gy >= a.xbox.lo[1] &&
                   gy <= a.xbox.hi[1];
  auto ownz_of = [&](int z) -> unsigned {
    return (rng(z, a.osh_lo[2], a.osh_hi[2]) ? 1u : 0u) | (rng(z, a.oun_lo[2], a.oun_hi[2]) ? 2u : 0u);
  };
  // ownership of E/D comp c (shifted along c) and B/H comp c (shifted off c)
  auto own_e = [](int c, unsigned ox_, unsigned oy_, unsigned oz_) {
    return ((c == 0 ? ox_ : ox_ >> 1) & (c == 1 ? oy_ : oy_ >> 1) & (c == 2 ? oz_ : oz_ >> 1) & 1u) != 0;
  };
  auto own_b = [](int c, unsigned ox_, unsigned oy_, unsigned oz_) {
    return ((c == 0 ? ox_ >> 1 : ox_) & (c == 1 ? oy_ >> 1 : oy_) & (c == 2 ? oz_ >> 1 : oz_) & 1u) != 0;
  };
  const int zmax = a.N[2] - 1;
  auto zc = [&](int z) { return min(max(z, 0), zmax); };
  auto tpz = [&](int z) { return min(max(z - zlo, 0), TPZ - 1); };
  // E_old of comp c at a point is implicit (chi1inv * D) when owned in G and not W-PML
  auto impl = [&](int c, unsigned ox_, unsigned oy_, unsigned oz_, bool wf) {
    return own_e(c, ox_, oy_, oz_) && !wf;
  };
  gdp Dv[3], Ev[3], Uv[3], Bv[3];
#pragma unroll
  for (int c = 0; c < 3; c++) {
    Dv[c] = sgpr_ptr(a.Do[c]);
    Ev[c] = sgpr_ptr(a.E[c]);
    Uv[c] = HAS_U && UMODE == 1 ? sgpr_ptr(a.u[c]) : nullptr;
    Bv[c] = sgpr_ptr(a.Bo[c]);
  }
  const gup uix = (gup)sgpr_ptr(a.uidx);
  auto pu_ = [&](unsigned ui, int c) -> double { return sU[UMODE == 2 ? c : 0][(ui >> (8 * c)) & 255]; };
  // palette word uniform over the item: every index load reads one cached word (the
  // first cell of the footprint in G) instead of one word per cell
  const bool uni = __builtin_amdgcn_readfirstlane(it.uw) != ~0u;
  const unsigned ufix = (unsigned)((max(x0 - 1, 0) + (long long)max(y0, 0) * a.st1 +
                                    (long long)max(zs - 1, 0) * a.st2) * 4);
  auto uoff = [&](unsigned o8) { return uni ? ufix : (o8 >> 1); };
  // W flags of E comps (PML chunk along own direction, shifted coordinate)
  const bool wx = ((AX & 1) && sFx[px][1] != 0), wy = ((AX & 2) && sFy[py][1] != 0);
  const bool hwx = ((AX & 1) && sFx[hpx][1] != 0), hwy = ((AX & 2) && sFy[hpy][1] != 0);

  auto load = [&](int k) -> GBatch<UMODE> {
    GBatch<UMODE> q;
    const int z1 = zc(k + 1);
    const unsigned o = cbl + (unsigned)z1 * s2;
    q.d0 = ldg(Dv[0], o);
    q.d1 = ldg(Dv[1], o);
    q.d2 = ldg(Dv[2], o);
    if (UMODE == 2) {
      q.ui = ldu(uix, uoff(o));
    } else if (HAS_U) {
      q.u0 = ldg(Uv[0], o);
      q.u1 = ldg(Uv[1], o);
      q.u2 = ldg(Uv[2], o);
    } else {
      q.u0 = q.u1 = q.u2 = 1.0;
    }
    const unsigned ob = cbl + (unsigned)zc(k) * s2;
    q.b0 = ldg(Bv[0], ob);
    q.b1 = ldg(Bv[1], ob);
    q.b2 = ldg(Bv[2], ob);
    q.h0 = q.h1 = 0.0;
    q.hu0 = q.hu1 = 1.0;
    q.hui = 0;
    q.hi0 = q.hi2 = false;
    if (hwave) {
      const int kk = zc(k);
      const unsigned oh = hbl + (unsigned)kk * s2;
      const unsigned oz = ownz_of(k);
      const bool wz = ((AX & 4) && sFz[tpz(k)][1] != 0);
      const bool hp = hpxy && pz_in(k);
      const bool i0 = hA && impl(hc0, hownx, howny, oz, (hc0 == 0 ? hwx : hwy) || hp);
      const bool i2 = hA && impl(2, hownx, howny, oz, wz || hp);
      q.h0 = ldg(i0 ? (hc0 ? Dv[1] : Dv[0]) : (hc0 ? Ev[1] : Ev[0]), oh);
      q.h1 = ldg(i2 ? Dv[2] : Ev[2], oh);
      if (UMODE == 2) {
        q.hui = ldu(uix, uoff(oh));
      } else if (HAS_U) {
        q.hu0 = ldg(hc0 ? Uv[1] : Uv[0], oh);
        q.hu1 = ldg(Uv[2], oh);
      }
      q.hi0 = i0;
      q.hi2 = i2;
    }
    return q;
  };
  // masked aux loads: a lane that needs no value reads its own B_old line (cache hit)
  auto load_aux = [&](int k) -> GAux {
    GAux x;
    const unsigned ob = cbl + (unsigned)zc(k) * s2;
    const unsigned o1 = cbl + (unsigned)zc(k + 1) * s2;
    const int pz = tpz(k), pz1 = tpz(k + 1);
    const unsigned oz1 = ownz_of(k + 1);
    const bool wz1 = ((AX & 4) && sFz[pz1][1] != 0);
    const bool p1 = pxy && pz_in(k + 1);
    const bool e0 = inA && !impl(0, ownx, owny, oz1, wx || p1),
               e1 = inA && !impl(1, ownx, owny, oz1, wy || p1),
               e2 = inA && !impl(2, ownx, owny, oz1, wz1 || p1);
    x.es0 = e0 ? ldg(Ev[0], o1) : 0.0;
    x.es1 = e1 ? ldg(Ev[1], o1) : 0.0;
    x.es2 = e2 ? ldg(Ev[2], o1) : 0.0;
    // f_u of B comp c: PML chunk along cycle(c,2), shifted coordinate
    const bool fxs = ((AX & 1) && sFx[px][1] != 0), fys = ((AX & 2) && sFy[py][1] != 0), fzs = ((AX & 4) && sFz[pz][1] != 0);
    const bool fxu = ((AX & 1) && sFx[px][0] != 0), fyu = ((AX & 2) && sFy[py][0] != 0), fzu = ((AX & 4) && sFz[pz][0] != 0);
    const bool u0 = inA && fzs, u1 = inA && fxs, u2 = inA && fys;
    x.ub0 = u0 ? ldg(sgpr_ptr(a.UBo[0]), ob) : 0.0;
    x.ub1 = u1 ? ldg(sgpr_ptr(a.UBo[1]), ob) : 0.0;
    x.ub2 = u2 ? ldg(sgpr_ptr(a.UBo[2]), ob) : 0.0;
    // separate H of comp c: PML chunk along c, unshifted coordinate
    const bool h0 = inA && fxu, h1 = inA && fyu, h2 = inA && fzu;
    x.ho0 = h0 ? ldg(sgpr_ptr(a.Ho[0]), ob) : 0.0;
    x.ho1 = h1 ? ldg(sgpr_ptr(a.Ho[1]), ob) : 0.0;
    x.ho2 = h2 ? ldg(sgpr_ptr(a.Ho[2]), ob) : 0.0;
    // f_u of D comp c: PML chunk along cycle(c,2), unshifted coordinate (owner lanes only)
    const bool d0 = stl && fzu, d1 = stl && fxu, d2 = stl && fyu;
    x.ud0 = d0 ? ldg(sgpr_ptr(a.UD[0]), ob) : 0.0;
    x.ud1 = d1 ? ldg(sgpr_ptr(a.UD[1]), ob) : 0.0;
    x.ud2 = d2 ? ldg(sgpr_ptr(a.UD[2]), ob) : 0.0;
    return x;
  };
  // conditional stores (no prefetch pipeline here, so exec-masked stores cost nothing extra)
  auto stg = [](double *p, unsigned off, double v) {
    *(double __attribute__((address_space(1))) *)((char __attribute__((address_space(1))) *)
                                                       sgpr_ptr(p) + off) = v;
  };

  // prologue: E_old(zs-1)
  double ex = 0, ey = 0, ez = 0;
  if (!lmode) {
    const int z = zlo;
    const unsigned o = cbl + (unsigned)zc(z) * s2;
    const unsigned oz = ownz_of(z);
    const bool wz = ((AX & 4) && sFz[tpz(z)][1] != 0);
    const bool p0 = pxy && pz_in(z);
    const bool i0 = inA && impl(0, ownx, owny, oz, wx || p0),
               i1 = inA && impl(1, ownx, owny, oz, wy || p0),
               i2 = inA && impl(2, ownx, owny, oz, wz || p0);
    ex = ldg(i0 ? Dv[0] : Ev[0], o);
    ey = ldg(i1 ? Dv[1] : Ev[1], o);
    ez = ldg(i2 ? Dv[2] : Ev[2], o);
    if (UMODE == 2) {
      const unsigned ui = ldu(uix, uoff(o));
      if (i0) ex *= pu_(ui, 0);
      if (i1) ey *= pu_(ui, 1);
      if (i2) ez *= pu_(ui, 2);
    } else if (HAS_U) {
      if (i0) ex *= ldg(Uv[0], o);
      if (i1) ey *= ldg(Uv[1], o);
      if (i2) ez *= ldg(Uv[2], o);
    }
  }
  double dx = 0, dy = 0, dz = 0, hmx = 0, hmy = 0;
  unsigned uik = 0;             // palette word of plane k (UMODE 2)
  double uk0 = 1, uk1 = 1, uk2 = 1;  // chi1inv of plane k (UMODE 1)
  const int rowm = row > 0 ? row - 1 : 0, colm = col > 0 ? col - 1 : 0;
  // one plane per iteration, loads issued at its top (a prefetch ring does not fit
  // in 168 VGPRs without spills and measured no faster; the other waves of the CU
  // cover the latency)
  for (int k = zlo; k < ze; k++) {
    {
      const int kl = k;
      GAux ax = {};
      GBatch<UMODE> c = {};
      double nb0 = 0, nb1 = 0, nb2 = 0;  // lean-halo lanes: B_new of plane k
      if (!lmode) {
        ax = load_aux(kl);
        c = load(kl);
      } else {
        const unsigned ok = cbl + (unsigned)zc(kl) * s2;
        if (lmcol) {
          nb1 = ldg(sgpr_ptr(a.Bn[1]), ok);
        } else {
          nb0 = ldg(sgpr_ptr(a.Bn[0]), ok);
        }
        nb2 = ldg(sgpr_ptr(a.Bn[2]), ok);
      }
      const int pz = tpz(kl), pz1 = tpz(kl + 1);
      const unsigned oz = ownz_of(kl), oz1 = ownz_of(kl + 1);
      const bool wz1 = ((AX & 4) && sFz[pz1][1] != 0);
      // E_old(k+1) of this lane
      double e1x, e1y, e1z;
      {
        const bool p1 = pxy && pz_in(kl + 1);
        const bool i0 = inA && impl(0, ownx, owny, oz1, wx || p1),
                   i1 = inA && impl(1, ownx, owny, oz1, wy || p1),
                   i2 = inA && impl(2, ownx, owny, oz1, wz1 || p1);
        double v0 = c.d0, v1 = c.d1, v2 = c.d2;
        if (UMODE == 2) {
          v0 = v0 * pu_(c.ui, 0);
          v1 = v1 * pu_(c.ui, 1);
          v2 = v2 * pu_(c.ui, 2);
        } else if (HAS_U) {
          v0 = v0 * c.u0;
          v1 = v1 * c.u1;
          v2 = v2 * c.u2;
        }
        e1x = i0 ? v0 : ax.es0;
        e1y = i1 ? v1 : ax.es1;
        e1z = i2 ? v2 : ax.es2;
      }
      if (ownlike) {
        sE[0][row][col] = ex;
        sE[1][row][col] = ey;
        sE[2][row][col] = ez;
      }
      if (hslot) {
        double h0 = c.h0, h1 = c.h1;
        if (UMODE == 2) {
          if (c.hi0) h0 = h0 * pu_(c.hui, hc0);
          if (c.hi2) h1 = h1 * pu_(c.hui, 2);
        } else if (HAS_U) {
          if (c.hi0) h0 = h0 * c.hu0;
          if (c.hi2) h1 = h1 * c.hu1;
        }
        sE[hc0][hrow][hcol] = h0;
        sE[2][hrow][hcol] = h1;
      }
      __syncthreads();
      // ---- curl B (E_old) with PML branches, then H
      const TabE tx_s = ((AX & 1) ? sTx[px][1] : kTabId), ty_s = ((AX & 2) ? sTy[py][1] : kTabId), tz_s = ((AX & 4) ? sTz[pz][1] : kTabId);
      const TabE tx_u = ((AX & 1) ? sTx[px][0] : kTabId), ty_u = ((AX & 2) ? sTy[py][0] : kTabId), tz_u = ((AX & 4) ? sTz[pz][0] : kTabId);
      const bool fxs = ((AX & 1) && sFx[px][1] != 0), fys = ((AX & 2) && sFy[py][1] != 0), fzs = ((AX & 4) && sFz[pz][1] != 0);
      const bool fxu = ((AX & 1) && sFx[px][0] != 0), fyu = ((AX & 2) && sFy[py][0] != 0), fzu = ((AX & 4) && sFz[pz][0] != 0);
      const double Ez_yp = sE[2][row + 1][col], Ex_yp = sE[0][row + 1][col];
      const double Ey_xp = sE[1][row][col + 1], Ez_xp = sE[2][row][col + 1];
      double ubx, uby, ubz;
      // B_c: dsig = cycle(c,1), dsigu = cycle(c,2); f_u flag along dsigu
      const double Bx = pml_curl(c.b0, ax.ub0, Ez_yp - ez + ey - e1y, C, fzs, ty_s.kms, ty_s.si,
                                 tz_s.kms, tz_s.si, &ubx);
      const double By = pml_curl(c.b1, ax.ub1, e1x - ex + ez - Ez_xp, C, fxs, tz_s.kms, tz_s.si,
                                 tx_s.kms, tx_s.si, &uby);
      const double Bz = pml_curl(c.b2, ax.ub2, Ey_xp - ey + ex - Ex_yp, C, fys, tx_s.kms, tx_s.si,
                                 ty_s.kms, ty_s.si, &ubz);
      // H_c (update_eh H_stuff): separate where the chunk has PML along c
      double Hx = fxu ? ax.ho0 + (tx_u.kps * Bx - tx_u.kms * c.b0) : Bx;
      double Hy = fyu ? ax.ho1 + (ty_u.kps * By - ty_u.kms * c.b1) : By;
      double Hz = fzu ? ax.ho2 + (tz_u.kps * Bz - tz_u.kms * c.b2) : Bz;
      if (lmode) Hx = nb0, Hy = nb1, Hz = nb2;  // never stored by these lanes
      const bool kin = k >= zs && k < ze;
      const bool sk = stl && kin;
      {
        const unsigned ok = cb + (unsigned)kl * s2;
        const unsigned o0 = (sk && own_b(0, ownx, owny, oz)) ? ok : MNL_OOB;
        const unsigned o1 = (sk && own_b(1, ownx, owny, oz)) ? ok : MNL_OOB;
        const unsigned o2 = (sk && own_b(2, ownx, owny, oz)) ? ok : MNL_OOB;
        if (o0 != MNL_OOB) stg(a.Bn[0], o0, Bx);
        if (o1 != MNL_OOB) stg(a.Bn[1], o1, By);
        if (o2 != MNL_OOB) stg(a.Bn[2], o2, Bz);
        if (fzs && o0 != MNL_OOB) stg(a.UBn[0], o0, ubx);
        if (fxs && o1 != MNL_OOB) stg(a.UBn[1], o1, uby);
        if (fys && o2 != MNL_OOB) stg(a.UBn[2], o2, ubz);
        if (fxu && o0 != MNL_OOB) stg(a.Hn[0], o0, Hx);
        if (fyu && o1 != MNL_OOB) stg(a.Hn[1], o1, Hy);
        if (fzu && o2 != MNL_OOB) stg(a.Hn[2], o2, Hz);
      }
      if (ownlike) {
        sB[0][row][col] = Hx;
        sB[1][row][col] = Hy;
        sB[2][row][col] = Hz;
      }
      __syncthreads();
      // ---- curl D (H_new) with PML branches, then E where W-PML
      const double Hz_ym = sB[2][rowm][col], Hx_ym = sB[0][rowm][col];
      const double Hz_xm = sB[2][row][colm], Hy_xm = sB[1][row][colm];
      double udx, udy, udz;
      const double Dx = pml_curl(dx, ax.ud0, Hz_ym - Hz + Hy - hmy, C, fzu, ty_u.kms, ty_u.si,
                                 tz_u.kms, tz_u.si, &udx);
      const double Dy = pml_curl(dy, ax.ud1, hmx - Hx + Hz - Hz_xm, C, fxu, tz_u.kms, tz_u.si,
                                 tx_u.kms, tx_u.si, &udy);
      const double Dz = pml_curl(dz, ax.ud2, Hy_xm - Hy + Hx - Hx_ym, C, fyu, tx_u.kms, tx_u.si,
                                 ty_u.kms, ty_u.si, &udz);
      {
        const unsigned ok = cb + (unsigned)kl * s2;
        const unsigned o0 = (sk && own_e(0, ownx, owny, oz)) ? ok : MNL_OOB;
        const unsigned o1 = (sk && own_e(1, ownx, owny, oz)) ? ok : MNL_OOB;
        const unsigned o2 = (sk && own_e(2, ownx, owny, oz)) ? ok : MNL_OOB;
        if (o0 != MNL_OOB) stg(a.Dn[0], o0, Dx);
        if (o1 != MNL_OOB) stg(a.Dn[1], o1, Dy);
        if (o2 != MNL_OOB) stg(a.Dn[2], o2, Dz);
        if (fzu && o0 != MNL_OOB) stg(a.UD[0], o0, udx);
        if (fxu && o1 != MNL_OOB) stg(a.UD[1], o1, udy);
        if (fyu && o2 != MNL_OOB) stg(a.UD[2], o2, udz);
        // E in PML chunks along its own direction (W form, src/step_generic.cpp:
        // 576-600 fw = chi1inv * D; W_E(old) == chi1inv * D_old)
        double k0 = 1, k1 = 1, k2 = 1;
        if (UMODE == 2) {
          k0 = pu_(uik, 0), k1 = pu_(uik, 1), k2 = pu_(uik, 2);
        } else if (HAS_U) {
          k0 = uk0, k1 = uk1, k2 = uk2;
        }
        if (!(POL && pxy && pz_in(kl))) {
          const double fw0 = HAS_U ? Dx * k0 : Dx, fp0 = HAS_U ? dx * k0 : dx;
          const double fw1 = HAS_U ? Dy * k1 : Dy, fp1 = HAS_U ? dy * k1 : dy;
          const double fw2 = HAS_U ? Dz * k2 : Dz, fp2 = HAS_U ? dz * k2 : dz;
          if (fxs && o0 != MNL_OOB) stg(a.En[0], o0, ex + (tx_s.kps * fw0 - tx_s.kms * fp0));
          if (fys && o1 != MNL_OOB) stg(a.En[1], o1, ey + (ty_s.kps * fw1 - ty_s.kms * fp1));
          if (fzs && o2 != MNL_OOB) stg(a.En[2], o2, ez + (tz_s.kps * fw2 - tz_s.kms * fp2));
        } else {
          // inside the polarization box: E = chi1inv * (D - sum P) (W form in PML),
          // then lorentzian update_P with W = E (or f_w) -- src/update_eh.cpp:84-146,
          // src/step_generic.cpp:576-906, src/susceptibility.cpp:188-262
          const double Dn3[3] = {Dx, Dy, Dz}, Do3[3] = {dx, dy, dz}, Eo3[3] = {ex, ey, ez};
          const double kk3[3] = {k0, k1, k2};
          const bool xin = xxy && kl >= a.xbox.lo[2] && kl <= a.xbox.hi[2];
          const unsigned oo3[3] = {xin ? MNL_OOB : o0, xin ? MNL_OOB : o1, xin ? MNL_OOB : o2};
          const bool w3[3] = {fxs, fys, fzs};
          const TabE tw3[3] = {tx_s, ty_s, tz_s};
          if (POL == 1) {  // one susceptibility: all loads first, one memory wait
            const auto &pd = a.pol[0];
            double pv[3], ppv[3], sg[3];
#pragma unroll
            for (int cc = 0; cc < 3; cc++) {
              const bool on = oo3[cc] != MNL_OOB && pd.P[cc];
              const unsigned oc = on ? oo3[cc] : cbl;
              pv[cc] = on ? ldg(sgpr_ptr(pd.P[cc]), oc) : 0.0;
              ppv[cc] = on ? ldg(sgpr_ptr(pd.Pp[cc]), oc) : 0.0;
              sg[cc] = on ? ldg(sgpr_ptr(pd.sigma[cc]), oc) : 0.0;
            }
#pragma unroll
            for (int cc = 0; cc < 3; cc++) {
              const unsigned oc = oo3[cc];
              if (oc == MNL_OOB) continue;
              const bool hp = pd.P[cc] != nullptr;
              const double gs = hp ? Dn3[cc] - pv[cc] : Dn3[cc];
              const double fw = HAS_U ? gs * kk3[cc] : gs;
              if (w3[cc]) {
                const double gp = hp ? Do3[cc] - ppv[cc] : Do3[cc];
                const double fp = HAS_U ? gp * kk3[cc] : gp;
                stg(a.En[cc], oc, Eo3[cc] + (tw3[cc].kps * fw - tw3[cc].kms * fp));
              } else {
                stg(a.En[cc], oc, fw);
              }
              if (hp) {
                stg(pd.P[cc], oc,
                    pd.gamma1inv * (pv[cc] * (2 - pd.omega0dtsqr_denom) - pd.gamma1 * ppv[cc] +
                                    pd.omega0dtsqr * (sg[cc] * fw)));
                stg(pd.Pp[cc], oc, pv[cc]);
              }
            }
          } else {
#pragma unroll
          for (int cc = 0; cc < 3; cc++) {
            const unsigned oc = oo3[cc];
            if (oc == MNL_OOB) continue;
            double pv[MAX_POL], ppv[MAX_POL];
            double gs = Dn3[cc], gp = Do3[cc];
            for (int q = 0; q < a.npol; q++) {
              const auto &pd = a.pol[q];
              pv[q] = pd.P[cc] ? ldg(sgpr_ptr(pd.P[cc]), oc) : 0.0;
              ppv[q] = pd.P[cc] ? ldg(sgpr_ptr(pd.Pp[cc]), oc) : 0.0;
              if (pd.P[cc]) {
                gs = gs - pv[q];
                gp = gp - ppv[q];
              }
            }
            const double fw = HAS_U ? gs * kk3[cc] : gs;
            double wv;
            if (w3[cc]) {
              const double fp = HAS_U ? gp * kk3[cc] : gp;
              stg(a.En[cc], oc, Eo3[cc] + (tw3[cc].kps * fw - tw3[cc].kms * fp));
              wv = fw;
            } else {
              stg(a.En[cc], oc, fw);
              wv = fw;
            }
            for (int q = 0; q < a.npol; q++) {
              const auto &pd = a.pol[q];
              if (!pd.P[cc]) continue;
              const double sg = ldg(sgpr_ptr(pd.sigma[cc]), oc);
              stg(pd.P[cc], oc,
                  pd.gamma1inv * (pv[q] * (2 - pd.omega0dtsqr_denom) - pd.gamma1 * ppv[q] +
                                  pd.omega0dtsqr * (sg * wv)));
              stg(pd.Pp[cc], oc, pv[q]);
            }
          }
          }
        }
      }
      hmx = Hx;
      hmy = Hy;
      dx = c.d0;
      dy = c.d1;
      dz = c.d2;
      if (UMODE == 2) {
        uik = c.ui;
      } else if (HAS_U) {
        uk0 = c.u0, uk1 = c.u1, uk2 = c.u2;
      }
      ex = e1x;
      ey = e1y;
      ez = e1z;
    }
  }
}

// General tiles: items from the host-built list a.gitems (tx | ty << 8 | ch << 16 |
// pml directions << 24, bit 31 set for a 16-column tile).  One launch takes both tile shapes, so the
// two share one tail:
// TX = 64: tiles of <= 64 columns x FUSED_GW_ROWS rows (ty indexes a.gyb);
// TX = 16: the narrow x-face tiles, 16 columns x FUSED_GN_ROWS rows (ty indexes
// a.nyb), four rows per wave so a plane step does as much work as a wide tile.
// 12 waves either way (168 VGPRs per lane).
template <int TX>
struct GenShape {
  static constexpr int NW = TX == 64 ? FUSED_GW_ROWS + 1 : (FUSED_GN_ROWS + 1) / 4;
  static constexpr int R = NW * (64 / TX);
  static constexpr int WAVES = NW + (2 * R + 63) / 64;
};
static_assert(GenShape<64>::R - 1 == FUSED_GW_ROWS && GenShape<16>::R - 1 == FUSED_GN_ROWS,
              "general tile rows");
static_assert(GenShape<64>::WAVES == GenShape<16>::WAVES, "both tile shapes run in one workgroup");
constexpr int GEN_WAVES = GenShape<64>::WAVES;

template <int TX>
struct GenLds {  // LDS of one tile shape (the two shapes share it through a union)
  static constexpr int R = GenShape<TX>::R;
  double sE[3][R + 1][TX + 2];
  double sB[3][R][TX + 1];
  TabE sTx[TX + 2][2], sTy[R + 1][2], sTz[TPZ][2];
  unsigned char sFx[TX + 2][2], sFy[R + 1][2], sFz[TPZ][2];
};

template <int UMODE, int TX, int POL, int AX>
__device__ __forceinline__ void general_item(KFA &a, int item, unsigned uw,
                                             GenLds<TX> &L, const double (*sU)[256]) {
  const int tx = item & 255, ty = (item >> 8) & 255, ch = (item >> 16) & 255;
  const auto *yb = TX == 64 ? a.gyb : a.nyb;
  ItemGeo itg;
  itg.x0 = a.xb[tx];
  itg.x1 = a.xb[tx + 1] - 1;
  itg.y0 = yb[ty] - 1;
  itg.y1 = yb[ty + 1] - 1;
  itg.zs = a.zb[ch];
  itg.ze = a.zb[ch + 1];
  itg.lmx = a.lean_after && (item & (1 << 27));
  itg.lmy = a.lean_after && (item & (1 << 28));
  itg.uw = uw;
  fused_general<UMODE, TX, GenShape<TX>::R, GenShape<TX>::NW, POL, AX>(
      a, itg, L.sE, L.sB, sU, L.sTx, L.sTy, L.sTz, L.sFx, L.sFy, L.sFz);
}

template <int UMODE, int POL>
__global__ __launch_bounds__(64 * GEN_WAVES, FUSED_GEN_WPE) void fused_general_kernel(FusedArgs a) {
  __shared__ double sU[UMODE == 2 ? 3 : 1][256];
  __shared__ union {
    GenLds<64> w;
    GenLds<16> n;
  } L;
  __shared__ int s_item;
  __shared__ unsigned s_uw;
  if (UMODE == 2)
    for (int i = threadIdx.x; i < 3 * 256; i += blockDim.x) sU[i >> 8][i & 255] = a.utab[i];
  // ngrp > 1: the workgroups sharing an XCD (blockIdx % ngrp) take a contiguous
  // share of the item list from their own counter line
  const int grp = a.ngrp > 1 ? (int)(blockIdx.x % a.ngrp) : 0;
  const int ntot = a.gend - a.gbeg;
  const int base = a.gbeg + (int)((long long)ntot * grp / a.ngrp);
  const int n = a.gbeg + (int)((long long)ntot * (grp + 1) / a.ngrp) - base;
  unsigned long long *ctr =
      a.ctr + 16 * (a.ngrp > 1 ? FUSED_GLINE0 + (a.ctr_line - 8) * 8 + grp : a.ctr_line);
  const unsigned long long cb = a.ngrp > 1 ? a.cbg[grp] : a.cbase;
  for (;;) {
    if (threadIdx.x == 0) {
      const unsigned long long v = atomicAdd(ctr, 1ULL) - cb;
      s_item = v < (unsigned long long)(n) ? a.gitems[base + v] : -1;
      s_uw = (v < (unsigned long long)(n) && UMODE == 2 && a.gflag) ? a.gflag[base + v] : ~0u;
    }
    __syncthreads();  // also separates LDS use of consecutive items
    const int item = s_item;
    const unsigned uw = s_uw;
    if (item == -1) break;
    // bits 24-26: the PML directions of the tile's footprint (host); a body with
    // the other directions' tables fixed at identity runs fewer instructions
    const int ax = (item >> 24) & 7;
    if (item & (int)0x80000000u) {
      if (ax == 1)
        general_item<UMODE, 16, POL, 1>(*kargs_opaque(), item, uw, L.n, sU);
      else
        general_item<UMODE, 16, POL, 7>(*kargs_opaque(), item, uw, L.n, sU);
    } else if (ax == 2) {
      general_item<UMODE, 64, POL, 2>(*kargs_opaque(), item, uw, L.w, sU);
    } else if (ax == 4) {
      general_item<UMODE, 64, POL, 4>(*kargs_opaque(), item, uw, L.w, sU);
    } else {
      general_item<UMODE, 64, POL, 7>(*kargs_opaque(), item, uw, L.w, sU);
    }
  }
}

// Lean body over one item (tile columns x0..x1, own rows y0+1..y1, planes [zs, ze)):
// its whole footprint (columns x0-1 .. x1+1, rows y0 .. y1+1, planes zs-1 .. ze) lies in
// the lean box L: no PML, every component owned, H == B, E implicit.  1024 threads:
// waves 0..FR-1 hold one row each (row 0 = the y-1 halo row, B recomputed), wave FR the
// x-1 column (B recomputed), the E of the x+64 column and a corner.
template <int UMODE, int DIST>
__device__ __forceinline__ void lean_body(KFA &a, const ItemGeo &itg, unsigned uw,
                                          const double (*sU)[256], double (*sE)[FR + 1][FXL],
                                          double (*sB)[FR][FXL]) {
  constexpr bool HAS_U = UMODE != 0;
  const int tid = tid_item(), lane = tid & 63, w = tid >> 6;
  const int wu = __builtin_amdgcn_readfirstlane(w);  // wave-uniform
  const bool hwave = wu >= FR - 1;
  constexpr bool SKIPB = MNL_SKIP_B;
  const int flo0 = a.L.lo[0], flo1 = a.L.lo[1], flo2 = a.L.lo[2];
  const int fhi0 = a.L.hi[0], fhi1 = a.L.hi[1], fhi2 = a.L.hi[2];
  const unsigned s2 = (unsigned)(a.st2 * 8);  // byte stride of one z plane
  const double C = a.C;
  const unsigned nrec = (unsigned)min(a.nelem * 8, 0xFFFFFFFFLL);
  __amdgpu_buffer_rsrc_t rB[3], rD[3];
#pragma unroll
  for (int c = 0; c < 3; c++) {
    rB[c] = __builtin_amdgcn_make_buffer_rsrc(a.Bn[c], 0, (int)nrec, 0x00020000);
    rD[c] = __builtin_amdgcn_make_buffer_rsrc(a.Dn[c], 0, (int)nrec, 0x00020000);
  }
  // lane roles (fixed for the kernel)
  int row, col;         // own-like lanes: footprint row / LDS column
  bool ownlike;         // computes E->LDS and B_new
  int hrow = 0, hcol = 0, hc0 = 0, hdx = 0, hdy = 0;  // halo slot: LDS target, comps, offset
  bool hslot = false;
  if (w < FR) {
    row = w;
    col = lane + 1;
    ownlike = true;
    if (w == FR - 1) {  // y+1 row
      hslot = true;
      hrow = FR;
      hcol = col;
      hc0 = 0;
      hdx = lane;
      hdy = FR;
    }
  } else {
    row = lane + 1;
    col = 0;
    ownlike = lane < FOWN;
    if (lane >= 16 && lane < 16 + FR) {  // x+64 column
      hslot = true;
      hrow = lane - 16;
      hcol = FX + 1;
      hc0 = 1;
      hdx = FX;
      hdy = lane - 16;
    } else if (lane == 31) {  // E(x0-1, y0+FR)
      hslot = true;
      hrow = FR;
      hcol = 0;
      hc0 = 0;
      hdx = -1;
      hdy = FR;
    }
  }
  const int ox = (w < FR) ? lane : -1;  // own-like column offset from x0
  const int oy = row;                    // own-like row offset from y0
  gdp Dv[3], Ev[3], Uv[3], Bv[3];
#pragma unroll
  for (int c = 0; c < 3; c++) {
    Dv[c] = sgpr_ptr(a.Do[c]);
    Ev[c] = sgpr_ptr(a.E[c]);
    Uv[c] = HAS_U && UMODE == 1 ? sgpr_ptr(a.u[c]) : nullptr;
    Bv[c] = sgpr_ptr(a.Bo[c]);
  }
  const gup uix = (gup)sgpr_ptr(a.uidx);
  const gdp hE0 = hc0 ? Ev[1] : Ev[0], hE1 = Ev[2], hD0 = hc0 ? Dv[1] : Dv[0], hD1 = Dv[2];
  const gdp hU0 = hc0 ? Uv[1] : Uv[0], hU1 = Uv[2];
  const unsigned safe = (unsigned)((flo0 + (long long)flo1 * a.st1) * 8);
  auto zin = [&](int z) { return z >= flo2 && z <= fhi2; };
  auto e_of = [](double d, double u, bool fz) { return (HAS_U && fz) ? d * u : d; };
  auto pu = [&](unsigned ui, int c) -> double { return sU[UMODE == 2 ? c : 0][(ui >> (8 * c)) & 255]; };
  {
    // ---------------- lean body: rows y0-1 .. y1+1, columns x0-1 .. x1+1, planes
    // zs-1 .. ze lie in L (lanes past x1 / y1 only feed values that are not stored)
    const int zs = itg.zs, ze = itg.ze;  // planes [zs, ze)
    const int x0 = itg.x0, y0 = itg.y0;

    const int gx = x0 + ox, gy = y0 + oy;
    const bool valid = ownlike && gx >= flo0 - 1 && gx <= fhi0 + 1 && gy >= flo1 - 1 &&
                       gy <= fhi1 + 1;
    const bool colF = valid && gx >= flo0 && gx <= fhi0 && gy >= flo1 && gy <= fhi1;
    const bool store = colF && w < FR && row >= 1 && gx <= itg.x1 && gy <= itg.y1;
    const unsigned cb = (unsigned)((gx + (long long)gy * a.st1) * 8);
    const unsigned cbl = valid ? cb : safe;
    const int hx = x0 + hdx, hy = y0 + hdy;
    const bool hvalid = hslot && hx >= flo0 - 1 && hx <= fhi0 + 1 && hy >= flo1 - 1 &&
                        hy <= fhi1 + 1;
    const bool hF = hvalid && hx >= flo0 && hx <= fhi0 && hy >= flo1 && hy <= fhi1;
    const unsigned hbl = hvalid ? (unsigned)((hx + (long long)hy * a.st1) * 8) : cbl;
    // per-lane source of E inside L's z range: D (then E = D*u) or stored E
    const gdp pO0 = colF ? Dv[0] : Ev[0], pO1 = colF ? Dv[1] : Ev[1], pO2 = colF ? Dv[2] : Ev[2];
    const gdp pH0 = hF ? hD0 : hE0, pH1 = hF ? hD1 : hE1;
    // palette word uniform over the item: every index load reads the same cached word
    // (the first cell of the item's footprint in L) instead of one word per cell
    const bool uni = __builtin_amdgcn_readfirstlane(uw) != ~0u;
    const unsigned ufix =
        (unsigned)((max(x0 - 1, flo0) + (long long)max(y0, flo1) * a.st1 +
                    (long long)max(zs - 1, flo2) * a.st2) * 4);
    auto uoff = [&](unsigned o8) { return uni ? ufix : (o8 >> 1); };

    auto load = [&](int k) -> FBatch {
      FBatch q;
      const int z1 = k + 1;
      q.f = colF && zin(z1);
      const unsigned o = cbl + (unsigned)z1 * s2;
      const bool zf = zin(z1);  // uniform
      q.d0 = ldg(zf ? pO0 : Ev[0], o);
      q.d1 = ldg(zf ? pO1 : Ev[1], o);
      q.d2 = ldg(zf ? pO2 : Ev[2], o);
      if (UMODE == 2) {
        q.ui = ldu(uix, uoff(o));
      } else if (HAS_U) {
        q.u0 = ldg(Uv[0], o);
        q.u1 = ldg(Uv[1], o);
        q.u2 = ldg(Uv[2], o);
      } else {
        q.u0 = q.u1 = q.u2 = 1.0;
      }
      const unsigned ob = cbl + (unsigned)k * s2;
      // Bx of the x-1 column (wave FR) and By of the y-1 row (wave 0) feed no update: those
      // lanes read one cached line instead of a line per row (MNL_SKIP_B)
      q.b0 = ldg(Bv[0], (SKIPB && wu == FR) ? safe : ob);
      q.b1 = ldg(Bv[1], (SKIPB && wu == 0) ? safe : ob);
      q.b2 = ldg(Bv[2], ob);
      q.hf = hF && zin(k);
      q.h0 = q.h1 = 0.0;
      q.hu0 = q.hu1 = 1.0;
      q.hui = 0;
      if (hwave) {  // only waves FR-1 and FR carry halo slots
        const unsigned oh = hbl + (unsigned)k * s2;
        const bool zk = zin(k);  // uniform
        q.h0 = ldg(zk ? pH0 : hE0, oh);
        q.h1 = ldg(zk ? pH1 : hE1, oh);
        if (UMODE == 2) {
          q.hui = ldu(uix, uoff(oh));
        } else if (HAS_U) {
          q.hu0 = ldg(hU0, oh);
          q.hu1 = ldg(hU1, oh);
        }
      }
      return q;
    };

    // prologue: E(zs-1) and the first DIST batches
    double ex, ey, ez;
    {
      const int z = zs - 1;
      const bool f0 = colF && zin(z);
      const unsigned o = cbl + (unsigned)z * s2;
      ex = ldg(f0 ? Dv[0] : Ev[0], o);
      ey = ldg(f0 ? Dv[1] : Ev[1], o);
      ez = ldg(f0 ? Dv[2] : Ev[2], o);
      if (UMODE == 2) {
        const unsigned ui = ldu(uix, uoff(o));
        if (f0) {  // palette visible: stored before the item loop's barrier
          ex *= pu(ui, 0);
          ey *= pu(ui, 1);
          ez *= pu(ui, 2);
        }
      } else if (HAS_U && f0) {
        ex *= ldg(Uv[0], o);
        ey *= ldg(Uv[1], o);
        ez *= ldg(Uv[2], o);
      }
    }
    FBatch q[DIST + 1];
#pragma unroll
    for (int j = 0; j < DIST; j++) q[j] = load(min(zs - 1 + j, ze - 1));
    double dx = 0, dy = 0, dz = 0, hmx = 0, hmy = 0;
    const int rowm = row > 0 ? row - 1 : 0, colm = col > 0 ? col - 1 : 0;
    const int ngrp = (ze - zs + 1 + DIST) / (DIST + 1);  // iterations k = zs-1 .. ze-1, padded
    for (int g = 0; g < ngrp; g++) {
#pragma unroll
      for (int j = 0; j <= DIST; j++) {
        const int k = zs - 1 + g * (DIST + 1) + j;
        q[(j + DIST) % (DIST + 1)] = load(min(k + DIST, ze - 1));
        const FBatch &c = q[j];
        double e1x, e1y, e1z;
        if (UMODE == 2) {
          e1x = e_of(c.d0, pu(c.ui, 0), c.f);
          e1y = e_of(c.d1, pu(c.ui, 1), c.f);
          e1z = e_of(c.d2, pu(c.ui, 2), c.f);
        } else {
          e1x = e_of(c.d0, c.u0, c.f);
          e1y = e_of(c.d1, c.u1, c.f);
          e1z = e_of(c.d2, c.u2, c.f);
        }
        if (ownlike) {
          sE[0][row][col] = ex;
          sE[1][row][col] = ey;
          sE[2][row][col] = ez;
        }
        if (hslot) {
          if (UMODE == 2) {
            sE[hc0][hrow][hcol] = e_of(c.h0, pu(c.hui, hc0), c.hf);
            sE[2][hrow][hcol] = e_of(c.h1, pu(c.hui, 2), c.hf);
          } else {
            sE[hc0][hrow][hcol] = e_of(c.h0, c.hu0, c.hf);
            sE[2][hrow][hcol] = e_of(c.h1, c.hu1, c.hf);
          }
        }
        __syncthreads();
        const double Ez_yp = sE[2][row + 1][col], Ex_yp = sE[0][row + 1][col];
        const double Ey_xp = sE[1][row][col + 1], Ez_xp = sE[2][row][col + 1];
        const double Bx = c.b0 - C * (Ez_yp - ez + ey - e1y);
        const double By = c.b1 - C * (e1x - ex + ez - Ez_xp);
        const double Bz = c.b2 - C * (Ey_xp - ey + ex - Ex_yp);
        const unsigned os = (store && k >= zs && k < ze) ? cb + (unsigned)k * s2 : MNL_OOB;
        bst(rB[0], os, Bx);
        bst(rB[1], os, By);
        bst(rB[2], os, Bz);
        if (ownlike) {
          sB[0][row][col] = Bx;
          sB[1][row][col] = By;
          sB[2][row][col] = Bz;
        }
        __syncthreads();
        const double Hz_ym = sB[2][rowm][col], Hx_ym = sB[0][rowm][col];
        const double Hz_xm = sB[2][row][colm], Hy_xm = sB[1][row][colm];
        bst(rD[0], os, dx - C * (Hz_ym - Bz + By - hmy));
        bst(rD[1], os, dy - C * (hmx - Bx + Bz - Hz_xm));
        bst(rD[2], os, dz - C * (Hy_xm - By + Bx - Hx_ym));
        hmx = Bx;
        hmy = By;
        dx = c.d0;
        dy = c.d1;
        dz = c.d2;
        ex = e1x;
        ey = e1y;
        ez = e1z;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Tile kernel: one persistent launch over every tile of G
// outside the polarization chunks, in the lean body's 1024-thread layout (64 x 14
// own cells per plane, z-march).  Items whose footprint lies in L run lean_body;
// the others run pml_body<AX>, specialised by the PML directions AX its footprint
// meets (faces: 1 = x, 2 = y, 4 = z; 7 = edges / corners; 0 = boundary planes
// without PML).  The PML quantities of a lane are fixed along the march for x
// (per lane) and y (per row) and uniform per plane for z, so every face body is
// the lean body plus per-direction table reads (LDS) and the PML state of that
// direction only, loaded and stored through buffer descriptors with out-of-range
// offsets where a point holds none (no branches around memory operations).

// PML coefficient tables of one tile item's footprint:
// v[axis][0 = kap - sig, 1 = 1 / (kap + sig), 2 = kap + sig][half s][position]
// f[axis][half s][position] = the PML-chunk flag (src/structure.cpp:118-137)
struct PTabL {
  double v[3][3][2][TPZ];
  unsigned char f[3][2][TPZ];
};
static_assert(TPZ >= FXL && TPZ >= FR + 1, "table positions");

// ownership bits of an index along one axis: bit0 = shifted components owned, bit1 = unshifted
__device__ __forceinline__ unsigned own_bits_of(int v, int sl, int sh, int ul, int uh) {
  return ((v >= sl && v <= sh) ? 1u : 0u) | ((v >= ul && v <= uh) ? 2u : 0u);
}

// OWNC: every point of the item's footprint is owned in y and z (item bit 29, set by the
// host): the y / z ownership terms are the constant 3, so every ownership test and the
// E-load source of a lane are fixed along the march (no per-plane recomputation), and the
// z index needs no clamp
// PAIR: two items of at most 32 own columns with the same rows and planes (the rim's x-face
// strips of temporal blocking) in one workgroup: lanes 0..31 the first (LDS columns 1..32, halo
// columns 0 and 33), lanes 32..63 the second (it.xb0 .. it.xb1; LDS columns 35..66, halo 34 and
// 67); the halo wave serves both.  Row and z logic are unchanged.
template <int UMODE, int DIST, int AX, bool OWNC, bool PAIR = false>
__device__ __forceinline__ void pml_body(KFA &a, const ItemGeo &it, unsigned uw,
                                         const double (*sU)[256], double (*sE)[FR + 1][FXL],
                                         double (*sB)[FR][FXL], PTabL &P) {
  constexpr bool HAS_U = UMODE != 0;
  constexpr bool PX = (AX & 1) != 0, PY = (AX & 2) != 0, PZ = (AX & 4) != 0;
  const int tid = tid_item(), lane = tid & 63, w = tid >> 6;
  const int wu = __builtin_amdgcn_readfirstlane(w);  // wave-uniform
  const bool hwave = wu >= FR - 1;
  constexpr bool SKIPB = MNL_SKIP_B;
  constexpr bool RSAT = MNL_RS_AT;
  const int x0 = it.x0, y0 = it.y0, zs = it.zs, ze = it.ze;
  const int zlo = zs - 1;  // z table position 0
  // ---- PML tables of the footprint -> LDS (x: x0-1 .. x0+64, y: y0 .. y0+FR,
  // z: zs-1 .. ze), only the directions of this body
  {
    constexpr int NX = PX ? 2 * (PAIR ? FXL : FX + 2) : 0, NY = PY ? 2 * (FR + 1) : 0,
                  NZ = PZ ? 2 * TPZ : 0;
    for (int i = threadIdx.x; i < NX + NY + NZ; i += 1024) {
      int ax, pos, base;
      if (i < NX) {  // table position = LDS column
        ax = 0, pos = i >> 1, base = x0 - 1;
        if (PAIR && pos >= FXL / 2) base = it.xb0 - 1 - FXL / 2;
      } else if (i < NX + NY) {
        ax = 1, pos = (i - NX) >> 1, base = y0;
      } else {
        ax = 2, pos = (i - NX - NY) >> 1, base = zlo;
      }
      const int sft = i & 1;
      const int jj = min(max(base + pos, 0), a.N[ax] - 1);
      const int q = 2 * (jj + a.off[ax]) + sft;
      P.v[ax][0][sft][pos] = a.tab.kms[ax][q];
      P.v[ax][1][sft][pos] = a.tab.siginv[ax][q];
      P.v[ax][2][sft][pos] = a.tab.kps[ax][q];
      P.f[ax][sft][pos] = a.tab.flag[ax][q];
    }
  }
  // ---- lane roles (the lean body's; PAIR: per 32-lane half, for its sub-tile)
  constexpr int SW = PAIR ? 32 : FX;        // columns of a (sub-)tile
  const int sub = PAIR ? (lane >> 5) : 0;  // sub-tile of the lane
  const int sl = PAIR ? (lane & 31) : lane;
  const int sx0 = sub ? it.xb0 : x0, sx1 = sub ? it.xb1 : it.x1;  // sub-tile own columns
  const int cofs = sub * (FXL / 2);        // LDS column of the sub-tile's x-1 halo
  int row, col;
  bool ownlike;
  int hrow = 0, hcol = 0, hc0 = 0, hdx = 0, hdy = 0;
  bool hslot = false;
  if (w < FR) {
    row = w;
    col = cofs + sl + 1;
    ownlike = true;
    if (w == FR - 1) {  // y+1 row
      hslot = true, hrow = FR, hcol = col, hc0 = 0, hdx = sl, hdy = FR;
    }
  } else {
    row = sl + 1;
    col = cofs;
    ownlike = sl < FOWN;
    if (sl >= 16 && sl < 16 + FR) {  // x+SW column
      hslot = true, hrow = sl - 16, hcol = cofs + SW + 1, hc0 = 1, hdx = SW, hdy = sl - 16;
    } else if (sl == 31) {  // E(x0-1, y0+FR)
      hslot = true, hrow = FR, hcol = cofs, hc0 = 0, hdx = -1, hdy = FR;
    }
  }
  // (no lambda below refers to `a`: a closure holding its address makes the compiler
  // copy the whole argument block to scratch)
  const int N0 = a.N[0], N1 = a.N[1];
  const long long st1 = a.st1;
  const int ox = (w < FR) ? sl : -1;
  const int gx = sx0 + ox, gy = y0 + row;
  // lanes right of x1 + 1 (a narrow item or PAIR half) feed nothing that is stored: no loads
  const bool inA = ownlike && gx >= 0 && gx < N0 && gx <= sx1 + 1 && gy >= 0 && gy < N1;
  const unsigned cb = (unsigned)((gx + (long long)gy * st1) * 8);
  const unsigned cbl = inA ? cb : 0u;
  // per-axis ownership (within G): bit0 = components shifted along the axis, bit1 = unshifted
  const unsigned ownx = own_bits_of(gx, a.osh_lo[0], a.osh_hi[0], a.oun_lo[0], a.oun_hi[0]);
  const unsigned owny = OWNC ? 3u : own_bits_of(gy, a.osh_lo[1], a.osh_hi[1], a.oun_lo[1], a.oun_hi[1]);
  const int zsl = a.osh_lo[2], zsh = a.osh_hi[2], zul = a.oun_lo[2], zuh = a.oun_hi[2];
  auto own_e = [](int c, unsigned ox_, unsigned oy_, unsigned oz_) {
    return ((c == 0 ? ox_ : ox_ >> 1) & (c == 1 ? oy_ : oy_ >> 1) & (c == 2 ? oz_ : oz_ >> 1) & 1u) != 0;
  };
  auto own_b = [](int c, unsigned ox_, unsigned oy_, unsigned oz_) {
    return ((c == 0 ? ox_ >> 1 : ox_) & (c == 1 ? oy_ >> 1 : oy_) & (c == 2 ? oz_ >> 1 : oz_) & 1u) != 0;
  };
  const bool stl = ownlike && w < FR && row >= 1 && gx <= sx1 && gy <= it.y1;
  const int hx = sx0 + hdx, hy = y0 + hdy;
  const bool hA = hslot && hx >= 0 && hx < N0 && hx <= sx1 + 1 && hy >= 0 && hy < N1;
  const unsigned hbl = hA ? (unsigned)((hx + (long long)hy * st1) * 8) : cbl;
  const unsigned hownx = own_bits_of(hx, a.osh_lo[0], a.osh_hi[0], a.oun_lo[0], a.oun_hi[0]);
  const unsigned howny = OWNC ? 3u : own_bits_of(hy, a.osh_lo[1], a.osh_hi[1], a.oun_lo[1], a.oun_hi[1]);
  const int zmax = a.N[2] - 1;
#define zc(z) (OWNC ? (z) : min(max((z), 0), zmax))
#define ownz_of(z) (OWNC ? 3u : own_bits_of((z), zsl, zsh, zul, zuh))
  const unsigned s2 = (unsigned)(a.st2 * 8);
  const double C = a.C;
  const unsigned nrec = (unsigned)min(a.nelem * 8, 0xFFFFFFFFLL);
#define RSV(x) (RsArr<RSAT>::make((x), nrec))
#define RS(p) (RsArr<RSAT>::get((p), nrec))
  // PML-state arrays (null: every access out of range).  MNL_RS_AT (default): scalar
  // pointers whose buffer descriptors are rebuilt at each use (RS): 4-SGPR descriptors of
  // every array live across the z loop overflow the SGPRs and spill into VGPR lanes (a
  // v_readlane per reload); MNL_RS_AT=0: descriptors built once before the loop
  const auto pBn0 = RSV(a.Bn[0]);
  const auto pBn1 = RSV(a.Bn[1]);
  const auto pBn2 = RSV(a.Bn[2]);
  const auto pDn0 = RSV(a.Dn[0]);
  const auto pDn1 = RSV(a.Dn[1]);
  const auto pDn2 = RSV(a.Dn[2]);
  const auto pEo0 = RSV(a.E[0]);
  const auto pEo1 = RSV(a.E[1]);
  const auto pEo2 = RSV(a.E[2]);
  const auto pEn0 = RSV(a.En[0]);
  const auto pEn1 = RSV(a.En[1]);
  const auto pEn2 = RSV(a.En[2]);
  const auto pUBo0 = RSV(a.UBo[0]);
  const auto pUBo1 = RSV(a.UBo[1]);
  const auto pUBo2 = RSV(a.UBo[2]);
  const auto pUBn0 = RSV(a.UBn[0]);
  const auto pUBn1 = RSV(a.UBn[1]);
  const auto pUBn2 = RSV(a.UBn[2]);
  const auto pHo0 = RSV(a.Ho[0]);
  const auto pHo1 = RSV(a.Ho[1]);
  const auto pHo2 = RSV(a.Ho[2]);
  const auto pHn0 = RSV(a.Hn[0]);
  const auto pHn1 = RSV(a.Hn[1]);
  const auto pHn2 = RSV(a.Hn[2]);
  const auto pUD0 = RSV(a.UD[0]);
  const auto pUD1 = RSV(a.UD[1]);
  const auto pUD2 = RSV(a.UD[2]);
  // array pointers as scalars (a per-lane choice between two entries of a local
  // pointer array makes the array, and with it the kernel arguments, a scratch copy)
  const gdp D0 = sgpr_ptr(a.Do[0]), D1 = sgpr_ptr(a.Do[1]), D2 = sgpr_ptr(a.Do[2]);
  const gdp E0 = sgpr_ptr(a.E[0]), E1 = sgpr_ptr(a.E[1]), E2 = sgpr_ptr(a.E[2]);
  const gdp B0 = sgpr_ptr(a.Bo[0]), B1 = sgpr_ptr(a.Bo[1]), B2 = sgpr_ptr(a.Bo[2]);
  const gdp U0 = HAS_U && UMODE == 1 ? sgpr_ptr(a.u[0]) : nullptr;
  const gdp U1 = HAS_U && UMODE == 1 ? sgpr_ptr(a.u[1]) : nullptr;
  const gdp U2 = HAS_U && UMODE == 1 ? sgpr_ptr(a.u[2]) : nullptr;
  const gup uix = (gup)sgpr_ptr(a.uidx);
  // halo-slot sources (per lane)
  const gdp hE0 = hc0 ? E1 : E0, hD0 = hc0 ? D1 : D0, hU0 = hc0 ? U1 : U0;
#define pu(ui, c) sU[UMODE == 2 ? (c) : 0][((ui) >> (8 * (c))) & 255]
  const bool uni = __builtin_amdgcn_readfirstlane(uw) != ~0u;
  const unsigned ufix = (unsigned)((max(x0 - 1, 0) + (long long)max(y0, 0) * st1 +
                                    (long long)max(zs - 1, 0) * a.st2) * 4);
#define uoff(o8) (uni ? ufix : ((o8) >> 1))
  __syncthreads();  // tables visible
  // table accessors: direction d at this lane (x: column, y: row, z: plane position)
  const int px = col, py = row;
  // MNL_HOIST_X: the x coefficients of a lane are the same on every plane; held in
  // registers instead of re-read from LDS after every barrier
  double tbx[3][2] = {{1, 1}, {1, 1}, {1, 1}};
  bool hfx[2] = {false, false};
  if (MNL_HOIST_X && PX) {
#pragma unroll
    for (int k = 0; k < 3; k++) tbx[k][0] = P.v[0][k][0][px], tbx[k][1] = P.v[0][k][1][px];
    hfx[0] = P.f[0][0][px] != 0, hfx[1] = P.f[0][1][px] != 0;
  }
#define T(d, coef, sft, pz) \
  (((AX >> (d)) & 1) ? ((d) == 0 && MNL_HOIST_X ? tbx[coef][sft] \
                                                : P.v[d][coef][sft][(d) == 0 ? px : ((d) == 1 ? py : (pz))]) \
                     : 1.0)
#define F(d, sft, pz) \
  (((AX >> (d)) & 1) ? ((d) == 0 && MNL_HOIST_X ? hfx[sft] \
                                                : P.f[d][sft][(d) == 0 ? px : ((d) == 1 ? py : (pz))] != 0) \
                     : false)
  // W flags (PML chunk along the E component's own direction, shifted coordinate)
  const bool Wx = F(0, 1, 0), Wy = F(1, 1, 0);
#define Wz(pz) F(2, 1, pz)
  const bool hW0 = hc0 == 0 ? (PX && P.f[0][1][hcol] != 0) : (PY && P.f[1][1][hdy] != 0);

  struct PBatch {  // plane k: D(k+1) (or stored E where not owned), u(k+1), B(k),
                   // stored E(k+1) of W-form components, halo E(k)
    double d0, d1, d2, u0, u1, u2, b0, b1, b2, es0, es1, es2, h0, h1, hu0, hu1;
    unsigned ui, hui;
  };
#define PML_LOAD(QQ, KK) \
  do { \
    const int z1 = zc(KK + 1); \
    const unsigned o = cbl + (unsigned)z1 * s2; \
    const unsigned oz1 = ownz_of(KK + 1); \
    const int pz1 = KK + 1 - zlo; \
    const bool o0 = inA && own_e(0, ownx, owny, oz1), o1 = inA && own_e(1, ownx, owny, oz1), \
               o2 = inA && own_e(2, ownx, owny, oz1); \
    QQ.d0 = ldg(o0 ? D0 : E0, o); \
    QQ.d1 = ldg(o1 ? D1 : E1, o); \
    QQ.d2 = ldg(o2 ? D2 : E2, o); \
    if (UMODE == 2) { \
      QQ.ui = ldu(uix, uoff(o)); \
    } else if (HAS_U) { \
      QQ.u0 = ldg(U0, o); \
      QQ.u1 = ldg(U1, o); \
      QQ.u2 = ldg(U2, o); \
    } else { \
      QQ.u0 = QQ.u1 = QQ.u2 = 1.0; \
    } \
    QQ.es0 = QQ.es1 = QQ.es2 = 0.0; \
    if (PX) QQ.es0 = bld(RS(pEo0), (o0 && Wx) ? o : MNL_OOB); \
    if (PY) QQ.es1 = bld(RS(pEo1), (o1 && Wy) ? o : MNL_OOB); \
    if (PZ) QQ.es2 = bld(RS(pEo2), (o2 && Wz(pz1)) ? o : MNL_OOB); \
    const unsigned ob = cbl + (unsigned)zc(KK) * s2; \
    QQ.b0 = ldg(B0, (SKIPB && wu == FR) ? 0u : ob); /* unused: see lean_body */ \
    QQ.b1 = ldg(B1, (SKIPB && wu == 0) ? 0u : ob); \
    QQ.b2 = ldg(B2, ob); \
    QQ.h0 = QQ.h1 = 0.0; \
    QQ.hu0 = QQ.hu1 = 1.0; \
    QQ.hui = 0; \
    if (hwave) { \
      const unsigned oh = hbl + (unsigned)zc(KK) * s2; \
      const unsigned oz = ownz_of(KK); \
      const bool i0 = hA && own_e(hc0, hownx, howny, oz) && !hW0; \
      const bool i2 = hA && own_e(2, hownx, howny, oz) && !Wz(KK - zlo); \
      QQ.h0 = ldg(i0 ? hD0 : hE0, oh); \
      QQ.h1 = ldg(i2 ? D2 : E2, oh); \
      if (UMODE == 2) { \
        QQ.hui = ldu(uix, uoff(oh)); \
      } else if (HAS_U) { \
        QQ.hu0 = ldg(hU0, oh); \
        QQ.hu1 = ldg(U2, oh); \
      } \
    } \
  } while (0)

  // prologue: E_old(zs-1): implicit (chi1inv * D) where owned and not W-form, else stored
  double ex, ey, ez;
  {
    const int z = zlo;
    const unsigned o = cbl + (unsigned)zc(z) * s2;
    const unsigned oz = ownz_of(z);
    const bool i0 = inA && own_e(0, ownx, owny, oz) && !Wx,
               i1 = inA && own_e(1, ownx, owny, oz) && !Wy,
               i2 = inA && own_e(2, ownx, owny, oz) && !Wz(0);
    ex = ldg(i0 ? D0 : E0, o);
    ey = ldg(i1 ? D1 : E1, o);
    ez = ldg(i2 ? D2 : E2, o);
    if (UMODE == 2) {
      const unsigned ui = ldu(uix, uoff(o));
      if (i0) ex *= pu(ui, 0);
      if (i1) ey *= pu(ui, 1);
      if (i2) ez *= pu(ui, 2);
    } else if (HAS_U) {
      if (i0) ex *= ldg(U0, o);
      if (i1) ey *= ldg(U1, o);
      if (i2) ez *= ldg(U2, o);
    }
  }
  PBatch q[DIST + 1];
#pragma unroll
  for (int j = 0; j < DIST; j++) PML_LOAD(q[j], min(zs - 1 + j, ze - 1));
  // f_u of B comp c: PML along cycle(c,2) (shifted); separate H: along c (unshifted);
  // f_u of D comp c: along cycle(c,2) (unshifted; owner lanes only).  Plane KK's values
  // are loaded at the end of iteration KK-1, so they land during its E / LDS phase.
  double ub0 = 0, ub1 = 0, ub2 = 0, ho0 = 0, ho1 = 0, ho2 = 0, ud0 = 0, ud1 = 0, ud2 = 0;
#define PML_AUX(KK) \
  do { \
    const int apz = (KK) - zlo; \
    const unsigned aob = cbl + (unsigned)zc(KK) * s2; \
    if (PZ) ub0 = bld(RS(pUBo0), (inA && F(2, 1, apz)) ? aob : MNL_OOB); \
    if (PX) ub1 = bld(RS(pUBo1), (inA && F(0, 1, apz)) ? aob : MNL_OOB); \
    if (PY) ub2 = bld(RS(pUBo2), (inA && F(1, 1, apz)) ? aob : MNL_OOB); \
    if (PX) ho0 = bld(RS(pHo0), (inA && F(0, 0, apz)) ? aob : MNL_OOB); \
    if (PY) ho1 = bld(RS(pHo1), (inA && F(1, 0, apz)) ? aob : MNL_OOB); \
    if (PZ) ho2 = bld(RS(pHo2), (inA && F(2, 0, apz)) ? aob : MNL_OOB); \
    if (PZ) ud0 = bld(RS(pUD0), (stl && F(2, 0, apz)) ? aob : MNL_OOB); \
    if (PX) ud1 = bld(RS(pUD1), (stl && F(0, 0, apz)) ? aob : MNL_OOB); \
    if (PY) ud2 = bld(RS(pUD2), (stl && F(1, 0, apz)) ? aob : MNL_OOB); \
  } while (0)
  PML_AUX(zs - 1);
  double dx = 0, dy = 0, dz = 0, hmx = 0, hmy = 0;
  unsigned uik = 0;                  // palette word of plane k (UMODE 2)
  double uk0 = 1, uk1 = 1, uk2 = 1;  // chi1inv of plane k (UMODE 1)
  const int rowm = row > 0 ? row - 1 : 0, colm = col > 0 ? col - 1 : 0;
  const int ngrp = (ze - zs + 1 + DIST) / (DIST + 1);
  for (int g = 0; g < ngrp; g++) {
#pragma unroll
    for (int j = 0; j <= DIST; j++) {
      const int k = zs - 1 + g * (DIST + 1) + j;
      PML_LOAD(q[(j + DIST) % (DIST + 1)], min(k + DIST, ze - 1));
      const PBatch &c = q[j];
      const int pz = k - zlo, pz1 = pz + 1;
      const unsigned oz = ownz_of(k), oz1 = ownz_of(k + 1);
      // PML state of plane k: loaded at the end of the previous iteration (PML_AUX)
      const bool fxs = F(0, 1, pz), fys = F(1, 1, pz), fzs = F(2, 1, pz);
      const bool fxu = F(0, 0, pz), fyu = F(1, 0, pz), fzu = F(2, 0, pz);
      const bool kin = k >= zs && k < ze;
      const bool sk = stl && kin;
      const unsigned ok = cb + (unsigned)k * s2;
      // E_old(k+1) of this lane
      double e1x, e1y, e1z;
      {
        const bool o0 = inA && own_e(0, ownx, owny, oz1), o1 = inA && own_e(1, ownx, owny, oz1),
                   o2 = inA && own_e(2, ownx, owny, oz1);
        double v0 = c.d0, v1 = c.d1, v2 = c.d2;
        if (UMODE == 2) {
          v0 = v0 * pu(c.ui, 0);
          v1 = v1 * pu(c.ui, 1);
          v2 = v2 * pu(c.ui, 2);
        } else if (HAS_U) {
          v0 = v0 * c.u0;
          v1 = v1 * c.u1;
          v2 = v2 * c.u2;
        }
        e1x = o0 ? ((PX && Wx) ? c.es0 : v0) : c.d0;
        e1y = o1 ? ((PY && Wy) ? c.es1 : v1) : c.d1;
        e1z = o2 ? ((PZ && Wz(pz1)) ? c.es2 : v2) : c.d2;
      }
      if (ownlike) {
        sE[0][row][col] = ex;
        sE[1][row][col] = ey;
        sE[2][row][col] = ez;
      }
      if (hslot) {
        const bool i0 = hA && own_e(hc0, hownx, howny, oz) && !hW0;
        const bool i2 = hA && own_e(2, hownx, howny, oz) && !Wz(pz);
        double h0 = c.h0, h1 = c.h1;
        if (UMODE == 2) {
          if (i0) h0 = h0 * pu(c.hui, hc0);
          if (i2) h1 = h1 * pu(c.hui, 2);
        } else if (HAS_U) {
          if (i0) h0 = h0 * c.hu0;
          if (i2) h1 = h1 * c.hu1;
        }
        sE[hc0][hrow][hcol] = h0;
        sE[2][hrow][hcol] = h1;
      }
      __syncthreads();
      // ---- curl B (E_old) with the PML branches of step_curl, then H (update_eh)
      const double Ez_yp = sE[2][row + 1][col], Ex_yp = sE[0][row + 1][col];
      const double Ey_xp = sE[1][row][col + 1], Ez_xp = sE[2][row][col + 1];
      double ubx, uby, ubz;
      const double Bx = pml_curl(c.b0, ub0, Ez_yp - ez + ey - e1y, C, fzs, T(1, 0, 1, pz),
                                 T(1, 1, 1, pz), T(2, 0, 1, pz), T(2, 1, 1, pz), &ubx);
      const double By = pml_curl(c.b1, ub1, e1x - ex + ez - Ez_xp, C, fxs, T(2, 0, 1, pz),
                                 T(2, 1, 1, pz), T(0, 0, 1, pz), T(0, 1, 1, pz), &uby);
      const double Bz = pml_curl(c.b2, ub2, Ey_xp - ey + ex - Ex_yp, C, fys, T(0, 0, 1, pz),
                                 T(0, 1, 1, pz), T(1, 0, 1, pz), T(1, 1, 1, pz), &ubz);
      const double Hx = fxu ? ho0 + (T(0, 2, 0, pz) * Bx - T(0, 0, 0, pz) * c.b0) : Bx;
      const double Hy = fyu ? ho1 + (T(1, 2, 0, pz) * By - T(1, 0, 0, pz) * c.b1) : By;
      const double Hz = fzu ? ho2 + (T(2, 2, 0, pz) * Bz - T(2, 0, 0, pz) * c.b2) : Bz;
      {
        const unsigned b0 = (sk && own_b(0, ownx, owny, oz)) ? ok : MNL_OOB;
        const unsigned b1 = (sk && own_b(1, ownx, owny, oz)) ? ok : MNL_OOB;
        const unsigned b2 = (sk && own_b(2, ownx, owny, oz)) ? ok : MNL_OOB;
        bst(RS(pBn0), b0, Bx);
        bst(RS(pBn1), b1, By);
        bst(RS(pBn2), b2, Bz);
        if (PZ) bst(RS(pUBn0), fzs ? b0 : MNL_OOB, ubx);
        if (PX) bst(RS(pUBn1), fxs ? b1 : MNL_OOB, uby);
        if (PY) bst(RS(pUBn2), fys ? b2 : MNL_OOB, ubz);
        if (PX) bst(RS(pHn0), fxu ? b0 : MNL_OOB, Hx);
        if (PY) bst(RS(pHn1), fyu ? b1 : MNL_OOB, Hy);
        if (PZ) bst(RS(pHn2), fzu ? b2 : MNL_OOB, Hz);
      }
      if (ownlike) {
        sB[0][row][col] = Hx;
        sB[1][row][col] = Hy;
        sB[2][row][col] = Hz;
      }
      __syncthreads();
      // ---- curl D (H_new) with the PML branches, then E in the W form where PML
      // lies along its direction (src/step_generic.cpp:576-600: W_E(old) == chi1inv * D_old)
      const double Hz_ym = sB[2][rowm][col], Hx_ym = sB[0][rowm][col];
      const double Hz_xm = sB[2][row][colm], Hy_xm = sB[1][row][colm];
      double udx, udy, udz;
      const double Dx = pml_curl(dx, ud0, Hz_ym - Hz + Hy - hmy, C, fzu, T(1, 0, 0, pz),
                                 T(1, 1, 0, pz), T(2, 0, 0, pz), T(2, 1, 0, pz), &udx);
      const double Dy = pml_curl(dy, ud1, hmx - Hx + Hz - Hz_xm, C, fxu, T(2, 0, 0, pz),
                                 T(2, 1, 0, pz), T(0, 0, 0, pz), T(0, 1, 0, pz), &udy);
      const double Dz = pml_curl(dz, ud2, Hy_xm - Hy + Hx - Hx_ym, C, fyu, T(0, 0, 0, pz),
                                 T(0, 1, 0, pz), T(1, 0, 0, pz), T(1, 1, 0, pz), &udz);
      {
        const unsigned e0 = (sk && own_e(0, ownx, owny, oz)) ? ok : MNL_OOB;
        const unsigned e1 = (sk && own_e(1, ownx, owny, oz)) ? ok : MNL_OOB;
        const unsigned e2 = (sk && own_e(2, ownx, owny, oz)) ? ok : MNL_OOB;
        bst(RS(pDn0), e0, Dx);
        bst(RS(pDn1), e1, Dy);
        bst(RS(pDn2), e2, Dz);
        if (PZ) bst(RS(pUD0), fzu ? e0 : MNL_OOB, udx);
        if (PX) bst(RS(pUD1), fxu ? e1 : MNL_OOB, udy);
        if (PY) bst(RS(pUD2), fyu ? e2 : MNL_OOB, udz);
        double k0 = 1, k1 = 1, k2 = 1;
        if (UMODE == 2) {
          k0 = pu(uik, 0), k1 = pu(uik, 1), k2 = pu(uik, 2);
        } else if (HAS_U) {
          k0 = uk0, k1 = uk1, k2 = uk2;
        }
        if (PX) {
          const double fw = HAS_U ? Dx * k0 : Dx, fp = HAS_U ? dx * k0 : dx;
          bst(RS(pEn0), fxs ? e0 : MNL_OOB, ex + (T(0, 2, 1, pz) * fw - T(0, 0, 1, pz) * fp));
        }
        if (PY) {
          const double fw = HAS_U ? Dy * k1 : Dy, fp = HAS_U ? dy * k1 : dy;
          bst(RS(pEn1), fys ? e1 : MNL_OOB, ey + (T(1, 2, 1, pz) * fw - T(1, 0, 1, pz) * fp));
        }
        if (PZ) {
          const double fw = HAS_U ? Dz * k2 : Dz, fp = HAS_U ? dz * k2 : dz;
          bst(RS(pEn2), fzs ? e2 : MNL_OOB, ez + (T(2, 2, 1, pz) * fw - T(2, 0, 1, pz) * fp));
        }
      }
      hmx = Hx;
      hmy = Hy;
      dx = c.d0;
      dy = c.d1;
      dz = c.d2;
      if (UMODE == 2) {
        uik = c.ui;
      } else if (HAS_U) {
        uk0 = c.u0, uk1 = c.u1, uk2 = c.u2;
      }
      ex = e1x;
      ey = e1y;
      ez = e1z;
      PML_AUX(min(k + 1, ze - 1));
    }
  }
}
#undef PML_AUX
#undef PML_LOAD
#undef RS
#undef RSV
#undef pu
#undef uoff
#undef zc
#undef ownz_of
#undef T
#undef F
#undef Wz

// ---------------------------------------------------------------------------
// Narrow x-face strip body (temporal-blocking rim, DESIGN.md section 24, item bit 30).  The
// rim's x-face strips are 16 columns wide (one 128-byte line per row); in the 64-lane row
// layout a strip filled 16-32 of a wave's 64 lanes and cost a whole tile per plane.  Here all
// 1024 lanes are own-like: wave w holds rows 4w .. 4w+3 (lane -> column lane & 15, row
// 4w + lane / 16; row 0 = the y-1 halo row, B recomputed there), i.e. 16 columns x 63 own rows
// per plane.  The halo columns are loads only, one slot per thread 0..142:
//   * E of the x+16 column (rows 0..63) and of the y+64 row (columns 0..15), from the old set;
//   * B_new (= H: the column is lean) of the x-1 column (rows 1..63), read from this launch's
//     output set: the host takes this body only where x0 = 0 (no x-1 column) or where the x-1
//     column of every own row and plane is a two-step point, whose new values the two-step
//     kernel stored there before this launch (step n+1 border values in the middle set for R1,
//     its own step n+2 values in the next set for R2).
// AX = 1 (PML along x only) with every footprint point owned in y and z (OWNC): the update is
// pml_body<AX = 1, OWNC>'s, operand for operand (src/step_generic.cpp:69-253, 576-906).
constexpr int SW_N = 16, SR_N = 64, SXL = SW_N + 2;
template <int UMODE>
__device__ __forceinline__ void strip_body(KFA &a, const ItemGeo &it, unsigned uw,
                                           const double (*sU)[256], double (*sE)[SR_N + 1][SXL],
                                           double (*sB)[SR_N][SXL], PTabL &P) {
  constexpr bool HAS_U = UMODE != 0;
  constexpr bool RSAT = MNL_RS_AT;
  const int x0 = it.x0, x1 = it.x1, y0 = it.y0, y1 = it.y1, zs = it.zs, ze = it.ze;
  // ---- x PML tables of the footprint (positions 0 .. 17 = columns x0-1 .. x0+16) -> LDS
  for (int i = threadIdx.x; i < 2 * SXL; i += 1024) {
    const int pos = i >> 1, sft = i & 1;
    const int jj = min(max(x0 - 1 + pos, 0), a.N[0] - 1);
    const int q = 2 * (jj + a.off[0]) + sft;
    P.v[0][0][sft][pos] = a.tab.kms[0][q];
    P.v[0][1][sft][pos] = a.tab.siginv[0][q];
    P.v[0][2][sft][pos] = a.tab.kps[0][q];
    P.f[0][sft][pos] = a.tab.flag[0][q];
  }
  const int tid = tid_item(), lane = tid & 63, w = tid >> 6;
  const int row = 4 * w + (lane >> 4), col = 1 + (lane & 15);
  const int N0 = a.N[0], N1 = a.N[1];
  const long long st1 = a.st1;
  const int gx = x0 + (lane & 15), gy = y0 + row;
  // lanes right of x1 + 1 or below y1 + 1 feed nothing that is stored: no loads
  const bool inA = gx < N0 && gx <= x1 + 1 && gy < N1 && gy <= y1 + 1;
  const unsigned cb = (unsigned)((gx + (long long)gy * st1) * 8);
  const unsigned cbl = inA ? cb : 0u;
  // x ownership (y, z: every point owned): bit0 = shifted along x, bit1 = unshifted
  const unsigned ownx = own_bits_of(gx, a.osh_lo[0], a.osh_hi[0], a.oun_lo[0], a.oun_hi[0]);
  const bool ox0 = (ownx & 1u) != 0, ox1 = (ownx & 2u) != 0;
  const bool o0 = inA && ox0, o12 = inA && ox1;  // E comp 0 / comps 1, 2 owned (D loaded)
  const bool stl = row >= 1 && gx <= x1 && gy <= y1;
  // ---- halo slot of this thread: 1 = E of the x+16 column (row t), 2 = E of the y+64 row
  // (column t - 64), 3 = B_new of the x-1 column (row t - 79)
  const int t = tid;
  const int skind = t < SR_N ? 1 : t < SR_N + SW_N ? 2 : t < 2 * SR_N + SW_N - 1 ? 3 : 0;
  const int srow = skind == 1 ? t : skind == 2 ? SR_N : skind == 3 ? t - SR_N - SW_N + 1 : 0;
  const int scol = skind == 1 ? SW_N + 1 : skind == 2 ? 1 + (t - SR_N) : 0;
  const int hx = x0 - 1 + scol, hy = y0 + srow;
  const bool hA = skind != 0 && hx >= 0 && hx < N0 && hy < N1 && hy <= y1 + 1;
  const unsigned hbl = hA ? (unsigned)((hx + (long long)hy * st1) * 8) : cbl;
  const unsigned hownx = own_bits_of(hx, a.osh_lo[0], a.osh_hi[0], a.oun_lo[0], a.oun_hi[0]);
  const int hc0 = skind == 2 ? 0 : 1;
  const int zlo = zs - 1;
  const unsigned s2 = (unsigned)(a.st2 * 8);
  const double C = a.C;
  const unsigned nrec = (unsigned)min(a.nelem * 8, 0xFFFFFFFFLL);
#define RSV(x) (RsArr<RSAT>::make((x), nrec))
#define RS(p) (RsArr<RSAT>::get((p), nrec))
  const auto pBn0 = RSV(a.Bn[0]);
  const auto pBn1 = RSV(a.Bn[1]);
  const auto pBn2 = RSV(a.Bn[2]);
  const auto pDn0 = RSV(a.Dn[0]);
  const auto pDn1 = RSV(a.Dn[1]);
  const auto pDn2 = RSV(a.Dn[2]);
  const auto pEo0 = RSV(a.E[0]);
  const auto pEn0 = RSV(a.En[0]);
  const auto pUBo1 = RSV(a.UBo[1]);
  const auto pUBn1 = RSV(a.UBn[1]);
  const auto pHo0 = RSV(a.Ho[0]);
  const auto pHn0 = RSV(a.Hn[0]);
  const auto pUD1 = RSV(a.UD[1]);
  const gdp D0 = sgpr_ptr(a.Do[0]), D1 = sgpr_ptr(a.Do[1]), D2 = sgpr_ptr(a.Do[2]);
  const gdp E0 = sgpr_ptr(a.E[0]), E1 = sgpr_ptr(a.E[1]), E2 = sgpr_ptr(a.E[2]);
  const gdp B0 = sgpr_ptr(a.Bo[0]), B1 = sgpr_ptr(a.Bo[1]), B2 = sgpr_ptr(a.Bo[2]);
  const gdp NB1 = sgpr_ptr(a.Bn[1]), NB2 = sgpr_ptr(a.Bn[2]);
  const gdp U0 = HAS_U && UMODE == 1 ? sgpr_ptr(a.u[0]) : nullptr;
  const gdp U1 = HAS_U && UMODE == 1 ? sgpr_ptr(a.u[1]) : nullptr;
  const gdp U2 = HAS_U && UMODE == 1 ? sgpr_ptr(a.u[2]) : nullptr;
  const gup uix = (gup)sgpr_ptr(a.uidx);
#define pu(ui, c) sU[UMODE == 2 ? (c) : 0][((ui) >> (8 * (c))) & 255]
  const bool uni = __builtin_amdgcn_readfirstlane(uw) != ~0u;
  const unsigned ufix = (unsigned)((max(x0 - 1, 0) + (long long)max(y0, 0) * st1 +
                                    (long long)max(zs - 1, 0) * a.st2) * 4);
#define uoff(o8) (uni ? ufix : ((o8) >> 1))
  __syncthreads();  // tables visible
  // x coefficients / flags of this lane's column (T(0, coef, sft) / F(0, sft) of pml_body)
#define TX(coef, sft) P.v[0][coef][sft][col]
  const bool fxs = P.f[0][1][col] != 0, fxu = P.f[0][0][col] != 0;
  const bool Wx = fxs;
  // slot sources: implicit E (chi1inv * D) where owned and not W-form, else stored E; B_new
  const bool hW0 = hc0 == 0 && P.f[0][1][scol] != 0;
  const bool hi0 = hA && skind != 3 && ((hc0 == 0 ? hownx : hownx >> 1) & 1u) && !hW0;
  const bool hi2 = hA && skind != 3 && ((hownx >> 1) & 1u);
  const gdp hs0 = skind == 3 ? NB1 : (hi0 ? (hc0 ? D1 : D0) : (hc0 ? E1 : E0));
  const gdp hs1 = skind == 3 ? NB2 : (hi2 ? D2 : E2);
  const gdp hU0 = hc0 ? U1 : U0;
  const bool swave = w < 3;  // waves holding slots (threads 0 .. 142)

  struct SBatch {  // plane k: D(k+1) (or stored E where not owned), u(k+1), stored Ex(k+1),
                   // B(k), slot values of plane k
    double d0, d1, d2, u0, u1, u2, es0, b0, b1, b2, h0, h1, hu0, hu1;
    unsigned ui, hui;
  };
#define STRIP_LOAD(QQ, KK) \
  do { \
    const unsigned o = cbl + (unsigned)((KK) + 1) * s2; \
    QQ.d0 = ldg(o0 ? D0 : E0, o); \
    QQ.d1 = ldg(o12 ? D1 : E1, o); \
    QQ.d2 = ldg(o12 ? D2 : E2, o); \
    if (UMODE == 2) { \
      QQ.ui = ldu(uix, uoff(o)); \
    } else if (HAS_U) { \
      QQ.u0 = ldg(U0, o); \
      QQ.u1 = ldg(U1, o); \
      QQ.u2 = ldg(U2, o); \
    } else { \
      QQ.u0 = QQ.u1 = QQ.u2 = 1.0; \
    } \
    QQ.es0 = bld(RS(pEo0), (o0 && Wx) ? o : MNL_OOB); \
    const unsigned ob = cbl + (unsigned)(KK) * s2; \
    QQ.b0 = ldg(B0, ob); \
    QQ.b1 = ldg(B1, row == 0 ? 0u : ob); /* By of the y-1 row feeds no update */ \
    QQ.b2 = ldg(B2, ob); \
    QQ.h0 = QQ.h1 = 0.0; \
    QQ.hu0 = QQ.hu1 = 1.0; \
    QQ.hui = 0; \
    if (swave) { \
      const unsigned oh = hbl + (unsigned)(KK) * s2; \
      QQ.h0 = ldg(hs0, oh); \
      QQ.h1 = ldg(hs1, oh); \
      if (UMODE == 2) { \
        QQ.hui = ldu(uix, uoff(oh)); \
      } else if (HAS_U) { \
        QQ.hu0 = ldg(hU0, oh); \
        QQ.hu1 = ldg(U2, oh); \
      } \
    } \
  } while (0)

  // prologue: E_old(zs-1): implicit (chi1inv * D) where owned and not W-form, else stored
  double ex, ey, ez;
  {
    const unsigned o = cbl + (unsigned)zlo * s2;
    const bool i0 = o0 && !Wx;
    ex = ldg(i0 ? D0 : E0, o);
    ey = ldg(o12 ? D1 : E1, o);
    ez = ldg(o12 ? D2 : E2, o);
    if (UMODE == 2) {
      const unsigned ui = ldu(uix, uoff(o));
      if (i0) ex *= pu(ui, 0);
      if (o12) ey *= pu(ui, 1), ez *= pu(ui, 2);
    } else if (HAS_U) {
      if (i0) ex *= ldg(U0, o);
      if (o12) ey *= ldg(U1, o), ez *= ldg(U2, o);
    }
  }
  SBatch q[2];
  STRIP_LOAD(q[0], zs - 1);
  // PML state of plane KK (own lanes): f_u of By (PML along x, shifted), separate Hx, f_u of
  // Dy (owner lanes); loaded one iteration ahead
  double ub1 = 0, ho0 = 0, ud1 = 0;
#define STRIP_AUX(KK) \
  do { \
    const unsigned aob = cbl + (unsigned)(KK) * s2; \
    ub1 = bld(RS(pUBo1), (inA && fxs) ? aob : MNL_OOB); \
    ho0 = bld(RS(pHo0), (inA && fxu) ? aob : MNL_OOB); \
    ud1 = bld(RS(pUD1), (stl && fxu) ? aob : MNL_OOB); \
  } while (0)
  STRIP_AUX(zs - 1);
  double dx = 0, dy = 0, dz = 0, hmx = 0, hmy = 0;
  unsigned uik = 0;
  double uk0 = 1;
  const int rowm = row > 0 ? row - 1 : 0;
  const int ngrp = (ze - zs + 2) / 2;
  for (int g = 0; g < ngrp; g++) {
#pragma unroll
    for (int j = 0; j <= 1; j++) {
      const int k = zs - 1 + g * 2 + j;
      STRIP_LOAD(q[(j + 1) & 1], min(k + 1, ze - 1));
      const SBatch &c = q[j];
      const bool kin = k >= zs && k < ze;
      const bool sk = stl && kin;
      const unsigned ok = cb + (unsigned)k * s2;
      // E_old(k+1) of this lane
      double e1x, e1y, e1z;
      {
        double v0 = c.d0, v1 = c.d1, v2 = c.d2;
        if (UMODE == 2) {
          v0 = v0 * pu(c.ui, 0);
          v1 = v1 * pu(c.ui, 1);
          v2 = v2 * pu(c.ui, 2);
        } else if (HAS_U) {
          v0 = v0 * c.u0;
          v1 = v1 * c.u1;
          v2 = v2 * c.u2;
        }
        e1x = o0 ? (Wx ? c.es0 : v0) : c.d0;
        e1y = o12 ? v1 : c.d1;
        e1z = o12 ? v2 : c.d2;
      }
      sE[0][row][col] = ex;
      sE[1][row][col] = ey;
      sE[2][row][col] = ez;
      if (skind == 1 || skind == 2) {
        double h0 = c.h0, h1 = c.h1;
        if (UMODE == 2) {
          if (hi0) h0 = h0 * pu(c.hui, hc0);
          if (hi2) h1 = h1 * pu(c.hui, 2);
        } else if (HAS_U) {
          if (hi0) h0 = h0 * c.hu0;
          if (hi2) h1 = h1 * c.hu1;
        }
        sE[hc0][srow][scol] = h0;
        sE[2][srow][scol] = h1;
      }
      __syncthreads();
      // ---- curl B (E_old) with the x-PML branches of step_curl, then H (update_eh)
      const double Ez_yp = sE[2][row + 1][col], Ex_yp = sE[0][row + 1][col];
      const double Ey_xp = sE[1][row][col + 1], Ez_xp = sE[2][row][col + 1];
      double ubx, uby, ubz;
      const double Bx = pml_curl(c.b0, 0.0, Ez_yp - ez + ey - e1y, C, false, 1.0, 1.0, 1.0, 1.0, &ubx);
      const double By = pml_curl(c.b1, ub1, e1x - ex + ez - Ez_xp, C, fxs, 1.0, 1.0, TX(0, 1),
                                 TX(1, 1), &uby);
      const double Bz = pml_curl(c.b2, 0.0, Ey_xp - ey + ex - Ex_yp, C, false, TX(0, 1), TX(1, 1),
                                 1.0, 1.0, &ubz);
      const double Hx = fxu ? ho0 + (TX(2, 0) * Bx - TX(0, 0) * c.b0) : Bx;
      {
        const unsigned b0 = (sk && ox1) ? ok : MNL_OOB;
        const unsigned b12 = (sk && ox0) ? ok : MNL_OOB;
        bst(RS(pBn0), b0, Bx);
        bst(RS(pBn1), b12, By);
        bst(RS(pBn2), b12, Bz);
        bst(RS(pUBn1), fxs ? b12 : MNL_OOB, uby);
        bst(RS(pHn0), fxu ? b0 : MNL_OOB, Hx);
      }
      sB[0][row][col] = Hx;
      sB[1][row][col] = By;
      sB[2][row][col] = Bz;
      if (skind == 3) {  // B_new == H of the lean x-1 column
        sB[1][srow][0] = c.h0;
        sB[2][srow][0] = c.h1;
      }
      __syncthreads();
      // ---- curl D (H_new) with the x-PML branches, then E in the W form where PML lies
      // along x (src/step_generic.cpp:576-600: W_E(old) == chi1inv * D_old)
      const double Hz_ym = sB[2][rowm][col], Hx_ym = sB[0][rowm][col];
      const double Hz_xm = sB[2][row][col - 1], Hy_xm = sB[1][row][col - 1];
      double udx, udy, udz;
      const double Dx = pml_curl(dx, 0.0, Hz_ym - Bz + By - hmy, C, false, 1.0, 1.0, 1.0, 1.0, &udx);
      const double Dy = pml_curl(dy, ud1, hmx - Hx + Bz - Hz_xm, C, fxu, 1.0, 1.0, TX(0, 0),
                                 TX(1, 0), &udy);
      const double Dz = pml_curl(dz, 0.0, Hy_xm - By + Hx - Hx_ym, C, false, TX(0, 0), TX(1, 0),
                                 1.0, 1.0, &udz);
      {
        const unsigned e0 = (sk && ox0) ? ok : MNL_OOB;
        const unsigned e12 = (sk && ox1) ? ok : MNL_OOB;
        bst(RS(pDn0), e0, Dx);
        bst(RS(pDn1), e12, Dy);
        bst(RS(pDn2), e12, Dz);
        bst(RS(pUD1), fxu ? e12 : MNL_OOB, udy);
        double k0 = 1;
        if (UMODE == 2) {
          k0 = pu(uik, 0);
        } else if (HAS_U) {
          k0 = uk0;
        }
        const double fw = HAS_U ? Dx * k0 : Dx, fp = HAS_U ? dx * k0 : dx;
        bst(RS(pEn0), fxs ? e0 : MNL_OOB, ex + (TX(2, 1) * fw - TX(0, 1) * fp));
      }
      hmx = Hx;
      hmy = By;
      dx = c.d0;
      dy = c.d1;
      dz = c.d2;
      if (UMODE == 2) {
        uik = c.ui;
      } else if (HAS_U) {
        uk0 = c.u0;
      }
      ex = e1x;
      ey = e1y;
      ez = e1z;
      STRIP_AUX(min(k + 1, ze - 1));
    }
  }
}
#undef STRIP_AUX
#undef STRIP_LOAD
#undef RS
#undef RSV
#undef pu
#undef uoff
#undef TX

// body codes of tile items (bits 24-26): 0 lean, 1..7 pml_body<AX = 1, 2, 4, 0, 7, 3, 5>
// (y-z edges, AX = 6, are few: they take the AX = 7 body); bit 29: OWNC; bit 30 (with body 1
// and OWNC): the narrow x-face strip body (strip_body)
// LDS of the tile bodies (one raw array, carved per body shape)
constexpr int TILE_SE = 3 * (FR + 1) * FXL, TILE_SB = 3 * FR * FXL;
constexpr int STRIP_SE = 3 * (SR_N + 1) * SXL, STRIP_SB = 3 * SR_N * SXL;
constexpr int TILE_SM = TILE_SE + TILE_SB > STRIP_SE + STRIP_SB ? TILE_SE + TILE_SB
                                                                : STRIP_SE + STRIP_SB;
template <int UMODE, int DIST>
__device__ __forceinline__ void tile_item_body(KFA &a, int item, const ItemGeo &itg,
                                               unsigned uw, const double (*sU)[256], double *sm,
                                               PTabL &sP) {
  constexpr int MD = MNL_MULTI_DIST;
  const bool ownc = MNL_OWNC && ((item >> 29) & 1);
  double(*sE)[FR + 1][FXL] = reinterpret_cast<double(*)[FR + 1][FXL]>(sm);
  double(*sB)[FR][FXL] = reinterpret_cast<double(*)[FR][FXL]>(sm + TILE_SE);
  switch ((item >> 24) & 7) {
    case 0:
      lean_body<UMODE, DIST>(a, itg, uw, sU, sE, sB);
      break;
    case 1:
      if ((item >> 30) & 1) {  // narrow x-face strip (temporal-blocking rim; host: OWNC)
        strip_body<UMODE>(a, itg, uw, sU, reinterpret_cast<double(*)[SR_N + 1][SXL]>(sm),
                          reinterpret_cast<double(*)[SR_N][SXL]>(sm + STRIP_SE), sP);
      } else if (itg.xb0 >= 0) {  // paired x-face strips (temporal-blocking rim)
        if (ownc)
          pml_body<UMODE, DIST, 1, true, true>(a, itg, uw, sU, sE, sB, sP);
        else
          pml_body<UMODE, DIST, 1, false, true>(a, itg, uw, sU, sE, sB, sP);
      } else if (ownc) {
        pml_body<UMODE, DIST, 1, true>(a, itg, uw, sU, sE, sB, sP);
      } else {
        pml_body<UMODE, DIST, 1, false>(a, itg, uw, sU, sE, sB, sP);
      }
      break;
    case 2:
      if (ownc)
        pml_body<UMODE, DIST, 2, true>(a, itg, uw, sU, sE, sB, sP);
      else
        pml_body<UMODE, DIST, 2, false>(a, itg, uw, sU, sE, sB, sP);
      break;
    case 3:
      if (ownc)
        pml_body<UMODE, DIST, 4, true>(a, itg, uw, sU, sE, sB, sP);
      else
        pml_body<UMODE, DIST, 4, false>(a, itg, uw, sU, sE, sB, sP);
      break;
    case 4:
      pml_body<UMODE, DIST, 0, false>(a, itg, uw, sU, sE, sB, sP);
      break;
    case 5:
      pml_body<UMODE, MD, 7, false>(a, itg, uw, sU, sE, sB, sP);
      break;
    case 6:
      pml_body<UMODE, MD, 3, false>(a, itg, uw, sU, sE, sB, sP);
      break;
    default:
      pml_body<UMODE, MD, 5, false>(a, itg, uw, sU, sE, sB, sP);
      break;
  }
}

// diagnostics (ItemClock): one record per item, written by thread 0 with vector stores
__device__ __forceinline__ void clk_record(const ItemClock &c, unsigned long long t0, int code, int g0,
                                        int g1, int g2, int g3) {
  const unsigned long long t1 = wall_clock64();
  const unsigned slot = atomicAdd(c.n, 1u);
  if (slot >= c.cap) return;
  unsigned long long *r = c.rec + (size_t)slot * CLK_REC;
  r[0] = t0;
  r[1] = t1;
  r[2] = (unsigned long long)(unsigned)c.kind | ((unsigned long long)blockIdx.x << 8);
  r[3] = (unsigned)code;
  r[4] = (unsigned)g0;
  r[5] = (unsigned)g1;
  r[6] = (unsigned)g2;
  r[7] = (unsigned long long)(long long)g3;
}

// own box of tile item `idx`: explicit (FusedArgs::tgeo) or tile / chunk indices
__device__ __forceinline__ ItemGeo tile_item_geo(const FusedArgs &a, int item, int idx) {
  ItemGeo itg;
  itg.xb0 = itg.xb1 = -1;
  if (a.tgeo) {
    const int *gp = a.tgeo + 4 * idx;
    itg.x0 = gp[0] & 0xFFFF;
    itg.x1 = gp[0] >> 16;
    itg.y0 = (gp[1] & 0xFFFF) - 1;
    itg.y1 = gp[1] >> 16;
    itg.zs = gp[2] & 0xFFFF;
    itg.ze = gp[2] >> 16;
    if (gp[3] >= 0) itg.xb0 = gp[3] & 0xFFFF, itg.xb1 = gp[3] >> 16;
  } else {
    const int tx = item & 255, ty = (item >> 8) & 255, ch = (item >> 16) & 255;
    itg.x0 = a.xb[tx];
    itg.x1 = a.xb[tx + 1] - 1;
    itg.y0 = a.yb[ty] - 1;
    itg.y1 = a.yb[ty + 1] - 1;
    itg.zs = a.zb[ch];
    itg.ze = a.zb[ch + 1];
  }
  itg.lmx = itg.lmy = false;
  itg.uw = ~0u;
  return itg;
}

template <int UMODE, int DIST, bool CLK>
__global__ __launch_bounds__(1024) void fused_tile_kernel(FusedArgs a) {
  __shared__ double sU[UMODE == 2 ? 3 : 1][256];
  __shared__ double sm[TILE_SM];
  __shared__ PTabL sP;
  __shared__ int s_item, s_idx;
  __shared__ unsigned s_uw;
  __shared__ unsigned long long s_t0;
  if (UMODE == 2) {  // palette -> LDS (visible after the first barrier below)
    for (int i = threadIdx.x; i < 3 * 256; i += 1024) sU[i >> 8][i & 255] = a.utab[i];
  }
  if (CLK && threadIdx.x == 0) s_t0 = 0ull;  // no previous item
  const long long n = a.gend - a.gbeg;
  unsigned long long *ctr = a.ctr + 16 * a.ctr_line;
  for (;;) {
    if (threadIdx.x == 0) {
      // diagnostics (MNL_ITEM_CLOCK): the previous item of this workgroup ends when wave 0
      // comes back for the next one (its last plane barrier has passed)
      if (CLK && s_t0 != 0ull) {
        const ItemGeo g = tile_item_geo(a, s_item, s_idx);
        clk_record(a.clk, s_t0, s_item, g.x0 | (g.x1 << 16), (g.y0 + 1) | (g.y1 << 16),
                   g.zs | (g.ze << 16), g.xb0 >= 0 ? (g.xb0 | (g.xb1 << 16)) : -1);
      }
      const unsigned long long v = atomicAdd(ctr, 1ULL) - a.cbase;
      s_item = v < (unsigned long long)(n) ? a.titems[a.gbeg + v] : -1;
      s_idx = a.gbeg + (int)v;
      s_uw = (v < (unsigned long long)(n) && UMODE == 2 && a.tflag) ? a.tflag[a.gbeg + v] : ~0u;
      if (CLK) s_t0 = wall_clock64();
    }
    __syncthreads();  // also separates LDS use of consecutive items
    const int item = s_item;
    if (item == -1) break;
    tile_item_body<UMODE, DIST>(*kargs_opaque(), item, tile_item_geo(a, item, s_idx), s_uw, sU, sm,
                                sP);
  }
}

#ifdef MNL_ISA_PROBE
// ISA inspection only (hipcc -DMNL_ISA_PROBE -S): one body per persistent kernel
template <int UMODE, int BODY>
__global__ __launch_bounds__(1024) void probe_kernel(FusedArgs a) {
  __shared__ double sU[UMODE == 2 ? 3 : 1][256];
  __shared__ double sm[TILE_SM];
  __shared__ PTabL sP;
  __shared__ int s_item;
  unsigned long long *ctr = a.ctr + 16 * a.ctr_line;
  for (;;) {
    if (threadIdx.x == 0) {
      const unsigned long long v = atomicAdd(ctr, 1ULL) - a.cbase;
      s_item = v < (unsigned long long)(a.gend) ? a.titems[v] : -1;
    }
    __syncthreads();
    const int item = s_item;
    if (item == -1) break;
    const ItemGeo itg = tile_item_geo(a, item, 0);
    double(*sE)[FR + 1][FXL] = reinterpret_cast<double(*)[FR + 1][FXL]>(sm);
    double(*sB)[FR][FXL] = reinterpret_cast<double(*)[FR][FXL]>(sm + TILE_SE);
    if (BODY == 0)
      strip_body<UMODE>(*kargs_opaque(), itg, ~0u, sU, reinterpret_cast<double(*)[SR_N + 1][SXL]>(sm),
                        reinterpret_cast<double(*)[SR_N][SXL]>(sm + STRIP_SE), sP);
    else if (BODY == 1)
      pml_body<UMODE, 1, 1, true>(*kargs_opaque(), itg, ~0u, sU, sE, sB, sP);
    else if (BODY == 2)
      pml_body<UMODE, 1, 2, true>(*kargs_opaque(), itg, ~0u, sU, sE, sB, sP);
    else
      lean_body<UMODE, 1>(*kargs_opaque(), itg, ~0u, sU, sE, sB);
  }
}
template __global__ void probe_kernel<2, 0>(FusedArgs);
template __global__ void probe_kernel<2, 1>(FusedArgs);
template __global__ void probe_kernel<2, 2>(FusedArgs);
template __global__ void probe_kernel<2, 3>(FusedArgs);
#endif

// the tile kernel for palette mode um (2 palette, 1 f64 chi1inv, 0 none); the diagnostics
// build when the item clock is on
void launch_tile(const FusedArgs &t, int um, dim3 grd, hipStream_t s) {
  const dim3 blk(1024);
  if (t.clk.rec) {
    if (um == 2)
      fused_tile_kernel<2, 1, true><<<grd, blk, 0, s>>>(t);
    else if (um == 1)
      fused_tile_kernel<1, 1, true><<<grd, blk, 0, s>>>(t);
    else
      fused_tile_kernel<0, 1, true><<<grd, blk, 0, s>>>(t);
  } else if (um == 2) {
    fused_tile_kernel<2, 1, false><<<grd, blk, 0, s>>>(t);
  } else if (um == 1) {
    fused_tile_kernel<1, 1, false><<<grd, blk, 0, s>>>(t);
  } else {
    fused_tile_kernel<0, 1, false><<<grd, blk, 0, s>>>(t);
  }
}

// Lean tiles only (the original two-launch fused step: this kernel, then
// fused_general_kernel over the PML / boundary tiles; MNL_TILE=0).  Work queues,
// chunk-major: consecutive items are neighbouring tiles of one chunk, so the
// workgroups sweep z roughly together.  With ngrp = 8 the workgroups sharing an XCD
// (blockIdx % 8, observed round-robin placement; speed only) own a contiguous range of
// each chunk's tiles (x fastest), so the halo lines neighbouring tiles share are
// fetched once into that XCD's L2.
template <int UMODE, int DIST>
__global__ __launch_bounds__(1024) void fused_kernel(FusedArgs a) {
  __shared__ double sU[UMODE == 2 ? 3 : 1][256];
  __shared__ double sE[3][FR + 1][FXL];
  __shared__ double sB[3][FR][FXL];
  __shared__ long long s_item;
  if (UMODE == 2) {  // palette -> LDS (visible after the first barrier below)
    for (int i = threadIdx.x; i < 3 * 256; i += 1024) sU[i >> 8][i & 255] = a.utab[i];
  }
  int nlch = 0;
  for (int r = 0; r < a.nlzr; r++) nlch += a.lzr[r][1] - a.lzr[r][0] + 1;
  const int nlx = a.lx1 - a.lx0 + 1;
  const long long ntile = (long long)nlx * (a.ly1 - a.ly0 + 1);
  const int grp = a.ngrp > 1 ? (int)(blockIdx.x % a.ngrp) : 0;
  const long long gt0 = ntile * grp / a.ngrp, gt1 = ntile * (grp + 1) / a.ngrp;
  const long long gtile = gt1 - gt0;
  unsigned long long *gctr = a.ctr + 16 * grp;
  const unsigned long long gbase = a.ngrp > 1 ? a.cbg[grp] : a.cbase;
  for (;;) {
    if (threadIdx.x == 0) {
      const unsigned long long v = atomicAdd(gctr, 1ULL) - gbase;
      s_item = v < (unsigned long long)(gtile * nlch) ? (long long)v : -1;
    }
    __syncthreads();  // also separates LDS use of consecutive items
    const long long item = s_item;
    if (item < 0) break;
    int ch = (int)(item / gtile);  // lean chunk ordinal -> chunk index
    for (int r = 0; r < a.nlzr; r++) {
      const int n = a.lzr[r][1] - a.lzr[r][0] + 1;
      if (ch < n) {
        ch += a.lzr[r][0];
        break;
      }
      ch -= n;
    }
    const int tile = (int)(gt0 + item % gtile);
    const int tx = a.lx0 + tile % nlx, ty = a.ly0 + tile / nlx;
    ItemGeo itg;
    itg.x0 = a.xb[tx];
    itg.x1 = a.xb[tx + 1] - 1;
    itg.y0 = a.yb[ty] - 1;
    itg.y1 = a.yb[ty + 1] - 1;
    itg.zs = a.zb[ch];
    itg.ze = a.zb[ch + 1];
    const unsigned uw = (UMODE == 2 && a.uflag) ? a.uflag[(long long)tile * a.nch + ch] : ~0u;
    lean_body<UMODE, DIST>(*kargs_opaque(), itg, uw, sU, sE, sB);
  }
}

// Per lean item (tile t, chunk ch; grid ntile x nch): the palette word if every cell
// of the item whose chi1inv the lean body uses -- its footprint (columns x0-1 ..
// x0+FX, rows y0 .. y0+FR, planes zs-1 .. ze) inside the lean box L -- has the same
// word, else ~0u (a word never has its top byte set).
__global__ void lean_uniform_kernel(FusedArgs a, unsigned *flags) {
  const int t = blockIdx.x, ch = blockIdx.y;
  const int nlx = a.lx1 - a.lx0 + 1;
  const int tx = a.lx0 + t % nlx, ty = a.ly0 + t / nlx;
  const int x0 = max(a.xb[tx] - 1, a.L.lo[0]), x1 = min(a.xb[tx] + FX, a.L.hi[0]);
  const int y0 = max(a.yb[ty] - 1, a.L.lo[1]), y1 = min(a.yb[ty] - 1 + FR, a.L.hi[1]);
  const int z0 = max(a.zb[ch] - 1, a.L.lo[2]), z1 = min(a.zb[ch + 1], a.L.hi[2]);
  __shared__ int bad;
  if (threadIdx.x == 0) bad = 0;
  __syncthreads();
  const long long nx = x1 - x0 + 1, ny = y1 - y0 + 1, nz = z1 - z0 + 1;
  unsigned ref = 0;
  if (nx > 0 && ny > 0 && nz > 0) {
    ref = a.uidx[x0 + (long long)y0 * a.st1 + (long long)z0 * a.st2];
    for (long long i = threadIdx.x; i < nx * ny * nz; i += blockDim.x) {
      const long long x = x0 + i % nx, y = y0 + (i / nx) % ny, z = z0 + i / (nx * ny);
      if (a.uidx[x + y * a.st1 + z * a.st2] != ref) bad = 1;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) flags[(long long)t * a.nch + ch] = bad ? ~0u : ref;
}

// The same per general item (index in gitems): footprint columns x0-1 .. x0+TX, rows
// y0 .. y0+R, planes zs-1 .. ze inside G (chi1inv is only used at owned points of G).
__global__ void general_uniform_kernel(FusedArgs a, unsigned *flags) {
  const int idx = blockIdx.x;
  const int item = a.gitems[idx];
  const bool nar = item & (int)0x80000000u;
  const int tx = item & 255, ty = (item >> 8) & 255, ch = (item >> 16) & 255;
  const int TX = nar ? 16 : 64, R = nar ? GenShape<16>::R : GenShape<64>::R;
  const int yb = nar ? a.nyb[ty] : a.gyb[ty];
  const int x0 = max(a.xb[tx] - 1, a.G.lo[0]), x1 = min(a.xb[tx] + TX, a.G.hi[0]);
  const int y0 = max(yb - 1, a.G.lo[1]), y1 = min(yb - 1 + R, a.G.hi[1]);
  const int z0 = max(a.zb[ch] - 1, a.G.lo[2]), z1 = min(a.zb[ch + 1], a.G.hi[2]);
  __shared__ int bad;
  if (threadIdx.x == 0) bad = 0;
  __syncthreads();
  const long long nx = x1 - x0 + 1, ny = y1 - y0 + 1, nz = z1 - z0 + 1;
  unsigned ref = 0;
  if (nx > 0 && ny > 0 && nz > 0) {
    ref = a.uidx[x0 + (long long)y0 * a.st1 + (long long)z0 * a.st2];
    for (long long i = threadIdx.x; i < nx * ny * nz; i += blockDim.x) {
      const long long x = x0 + i % nx, y = y0 + (i / nx) % ny, z = z0 + i / (nx * ny);
      if (a.uidx[x + y * a.st1 + z * a.st2] != ref) bad = 1;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) flags[idx] = bad ? ~0u : ref;
}

// chi1inv palette indices over box F: uidx[i] = idx0 | idx1 << 8 | idx2 << 16,
// tab[c*256 + idx] == u[c][i] exactly; *bad != 0 if some value is missing.
__global__ void build_uidx_kernel(unsigned *uidx, const double *u0, const double *u1,
                                  const double *u2, const double *tab, int n0, int n1, int n2,
                                  Box F, long long st1, long long st2, int *bad) {
  const int x = F.lo[0] + blockIdx.x * blockDim.x + threadIdx.x, y = F.lo[1] + blockIdx.y,
            z = F.lo[2] + blockIdx.z;
  if (x > F.hi[0]) return;
  const long long i = x + y * st1 + z * st2;
  const double *u[3] = {u0, u1, u2};
  const int n[3] = {n0, n1, n2};
  unsigned w = 0;
  for (int c = 0; c < 3; c++) {
    // exact match on the bit pattern (table sorted by bit pattern on the host)
    const unsigned long long v = (unsigned long long)__double_as_longlong(u[c][i]);
    const double *t = tab + 256 * c;
    int lo = 0, hi = n[c] - 1, hit = -1;
    while (lo <= hi) {
      const int mid = (lo + hi) >> 1;
      const unsigned long long tm = (unsigned long long)__double_as_longlong(t[mid]);
      if (tm == v) {
        hit = mid;
        break;
      }
      if (tm < v)
        lo = mid + 1;
      else
        hi = mid - 1;
    }
    if (hit < 0) {
      atomicOr(bad, 1);
      hit = 0;
    }
    w |= (unsigned)hit << (8 * c);
  }
  uidx[i] = w;
}

int k_build_uidx(unsigned *uidx, const double *const u[3], const double *tab, const int n[3],
                 const Box &F, long long st1, long long st2, int *bad, void *stream) {
  if (empty(F)) return 0;
  dim3 grd((F.hi[0] - F.lo[0] + 1 + 255) / 256, F.hi[1] - F.lo[1] + 1, F.hi[2] - F.lo[2] + 1);
  build_uidx_kernel<<<grd, 256, 0, (hipStream_t)stream>>>(uidx, u[0], u[1], u[2], tab, n[0], n[1],
                                                          n[2], F, st1, st2, bad);
  return rc();
}

int k_cu_count() {
  int dev = 0;
  hipDeviceProp_t pr;
  if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&pr, dev) != hipSuccess) return 256;
  return pr.multiProcessorCount;
}

static int fused_grid_blocks(int bpc) {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256 * bpc;
  if (!cus[dev]) {
    hipDeviceProp_t pr;
    if (hipGetDeviceProperties(&pr, dev) != hipSuccess) return 256 * bpc;
    cus[dev] = pr.multiProcessorCount;
  }
  return cus[dev] * bpc;
}

template <int UM>
static void launch_general_u(const FusedArgs &g, dim3 gr, dim3 b, hipStream_t s) {
  if (g.npol == 0)
    fused_general_kernel<UM, 0><<<gr, b, 0, s>>>(g);
  else if (g.npol == 1)
    fused_general_kernel<UM, 1><<<gr, b, 0, s>>>(g);
  else
    fused_general_kernel<UM, 2><<<gr, b, 0, s>>>(g);
}
static void launch_general(const FusedArgs &g, int um, dim3 gr, dim3 b, hipStream_t s) {
  if (um == 2)
    launch_general_u<2>(g, gr, b, s);
  else if (um == 1)
    launch_general_u<1>(g, gr, b, s);
  else
    launch_general_u<0>(g, gr, b, s);
}

int k_lean_uniform(const FusedArgs &a, unsigned *flags, void *stream) {
  const int ntile = (a.lx1 - a.lx0 + 1) * (a.ly1 - a.ly0 + 1);
  if (ntile <= 0 || a.nch <= 0 || !a.uidx) return 0;
  lean_uniform_kernel<<<dim3(ntile, a.nch), 256, 0, (hipStream_t)stream>>>(a, flags);
  return rc();
}

int k_general_uniform(const FusedArgs &a, unsigned *flags, void *stream) {
  if (a.ngen <= 0 || !a.uidx || !a.gitems) return 0;
  general_uniform_kernel<<<a.ngen, 256, 0, (hipStream_t)stream>>>(a, flags);
  return rc();
}

// Per tile item (index in titems): the palette word if every cell of its footprint
// (columns x0-1 .. x0+FX, rows y0 .. y0+FR, planes zs-1 .. ze; a narrow strip: columns
// x0-1 .. x0+SW_N, rows y0 .. y0+SR_N) inside G has the same word, else ~0u (chi1inv is used
// only at owned points of G).
__global__ void tile_uniform_kernel(FusedArgs a, unsigned *flags) {
  const int idx = blockIdx.x;
  const int item = a.titems[idx];
  const int tx = item & 255, ty = (item >> 8) & 255, ch = (item >> 16) & 255;
  const bool narrow = ((item >> 24) & 7) == 1 && ((item >> 30) & 1);
  const int fw = narrow ? SW_N : FX, fr = narrow ? SR_N : FR;
  int ix0, iy0, izs, ize;  // tile column start, halo row, planes [izs, ize)
  if (a.tgeo) {
    if (a.tgeo[4 * idx + 3] >= 0) {  // paired item: per-cell palette words
      if (threadIdx.x == 0) flags[idx] = ~0u;
      return;
    }
    ix0 = a.tgeo[4 * idx] & 0xFFFF;
    iy0 = (a.tgeo[4 * idx + 1] & 0xFFFF) - 1;
    izs = a.tgeo[4 * idx + 2] & 0xFFFF;
    ize = a.tgeo[4 * idx + 2] >> 16;
  } else {
    ix0 = a.xb[tx], iy0 = a.yb[ty] - 1, izs = a.zb[ch], ize = a.zb[ch + 1];
  }
  const int x0 = max(ix0 - 1, a.G.lo[0]), x1 = min(ix0 + fw, a.G.hi[0]);
  const int y0 = max(iy0, a.G.lo[1]), y1 = min(iy0 + fr, a.G.hi[1]);
  const int z0 = max(izs - 1, a.G.lo[2]), z1 = min(ize, a.G.hi[2]);
  __shared__ int bad;
  if (threadIdx.x == 0) bad = 0;
  __syncthreads();
  const long long nx = x1 - x0 + 1, ny = y1 - y0 + 1, nz = z1 - z0 + 1;
  unsigned ref = 0;
  if (nx > 0 && ny > 0 && nz > 0) {
    ref = a.uidx[x0 + (long long)y0 * a.st1 + (long long)z0 * a.st2];
    for (long long i = threadIdx.x; i < nx * ny * nz; i += blockDim.x) {
      const long long x = x0 + i % nx, y = y0 + (i / nx) % ny, z = z0 + i / (nx * ny);
      if (a.uidx[x + y * a.st1 + z * a.st2] != ref) bad = 1;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) flags[idx] = bad ? ~0u : ref;
}

int k_tile_uniform(const FusedArgs &a, unsigned *flags, void *stream) {
  if (a.ntit <= 0 || !a.uidx || !a.titems) return 0;
  tile_uniform_kernel<<<a.ntit, 256, 0, (hipStream_t)stream>>>(a, flags);
  return rc();
}

int k_fused(const FusedArgs &a, int which, void *stream, unsigned long long *bases) {
  for (int d = 0; d < 3; d++)
    if (a.G.hi[d] < a.G.lo[d]) return 0;
  if (a.nelem * 8 >= (long long)MNL_OOB || !a.ctr) return 2;  // host guarantees < 4 GiB arrays
  if (which >= 4) {  // tile kernel: 4 all items, 5 the chunk-0 items, 6 the others
    if (a.nx < 1 || a.nx > FUSED_MAXX || a.ny < 1 || a.ny > FUSED_MAXY || a.nch < 1 ||
        a.nch > FUSED_MAXZ)
      return 3;
    for (int t = 0; t < a.nx; t++)  // tiles at most 64 columns wide, 128-byte aligned
      if (a.xb[t + 1] - a.xb[t] > FX || a.xb[t + 1] <= a.xb[t] || (a.xb[t] & 15)) return 4;
    for (int t = 0; t < a.ny; t++)
      if (a.yb[t + 1] - a.yb[t] > FOWN || a.yb[t + 1] <= a.yb[t]) return 5;
    for (int t = 0; t < a.nch; t++)
      if (a.zb[t + 1] <= a.zb[t] || a.zb[t + 1] - a.zb[t] > FUSED_MAXCH) return 7;
    int ib = 0, ie = a.ntit, line = 0;
    if (which == 5) ie = a.ntit_e, line = 1;
    if (which == 6) ib = a.ntit_e, line = 2;
    if (ie <= ib) return 0;
    long long nb = fused_grid_blocks(a.blocks_per_cu > 0 ? a.blocks_per_cu : 1);
    if (a.wg_limit > 0 && nb > a.wg_limit) nb = a.wg_limit;
    if (nb > ie - ib) nb = ie - ib;
    FusedArgs t = a;
    t.gbeg = ib, t.gend = ie, t.ctr_line = line, t.cbase = bases[line];
    bases[line] += (unsigned long long)(ie - ib) + nb;
    const int um = a.uidx ? 2 : (a.u[0] ? 1 : 0);
    hipStream_t s = (hipStream_t)stream;
    launch_tile(t, um, dim3((unsigned)nb), s);
    return hipPeekAtLastError() == hipSuccess ? 0 : 9;
  }
  if (a.nx < 1 || a.nx > FUSED_MAXX || a.ny < 0 || a.ny > FUSED_MAXY || a.nch < 1 ||
      a.nch > FUSED_MAXZ || a.ngy < 1 || a.ngy > FUSED_MAXGY || a.nny < 0 || a.nny > FUSED_MAXNY)
    return 3;
  for (int t = 0; t < a.nx; t++)  // tiles at most 64 columns wide, 128-byte aligned
    if (a.xb[t + 1] - a.xb[t] > FX || a.xb[t + 1] <= a.xb[t] || (a.xb[t] & 15)) return 4;
  for (int t = 0; t < a.ny; t++)
    if (a.yb[t + 1] - a.yb[t] > FOWN || a.yb[t + 1] <= a.yb[t]) return 5;
  for (int t = 0; t < a.ngy; t++)
    if (a.gyb[t + 1] - a.gyb[t] > FUSED_GW_ROWS || a.gyb[t + 1] <= a.gyb[t]) return 6;
  for (int t = 0; t < a.nny; t++)
    if (a.nyb[t + 1] - a.nyb[t] > FUSED_GN_ROWS || a.nyb[t + 1] <= a.nyb[t]) return 6;
  for (int t = 0; t < a.nch; t++)
    if (a.zb[t + 1] <= a.zb[t] || a.zb[t + 1] - a.zb[t] > FUSED_MAXCH) return 7;
  hipStream_t s = (hipStream_t)stream;
  const int um = a.uidx ? 2 : (a.u[0] ? 1 : 0);
  if (which >= 1) {  // general tiles (both shapes, one launch)
    // item range in a.gitems: [0, ngen); chunk-0 items lead ([0, ngen_e))
    int ib = 0, ie = a.ngen, line = 8;
    if (which == 2) ie = a.ngen_e, line = 10;
    if (which == 3) ib = a.ngen_e;
    long long cus = fused_grid_blocks(FUSED_GEN_BPC);
    if (a.wg_limit > 0 && cus > a.wg_limit) cus = a.wg_limit;
    if (ie > ib) {
      FusedArgs g = a;
      const unsigned nblk = (unsigned)std::min<long long>(cus, ie - ib);
      g.gbeg = ib, g.gend = ie, g.ctr_line = line, g.cbase = bases[line];
      const long long n = ie - ib;
      g.ngrp = (a.ngrp_gen > 1 && nblk >= (unsigned)a.ngrp_gen && n >= 4LL * a.ngrp_gen) ? a.ngrp_gen : 1;
      if (g.ngrp == 1) {
        bases[line] += (unsigned long long)n + nblk;
      } else {
        for (int q = 0; q < g.ngrp; q++) {
          const int L = FUSED_GLINE0 + (line - 8) * 8 + q;
          g.cbg[q] = bases[L];
          const long long items = n * (q + 1) / g.ngrp - n * q / g.ngrp;
          const long long blocks = ((long long)nblk - q + g.ngrp - 1) / g.ngrp;
          bases[L] += (unsigned long long)(items + blocks);
        }
      }
      launch_general(g, um, dim3(nblk), dim3(64 * GEN_WAVES), s);
    }
    return hipPeekAtLastError() == hipSuccess ? 0 : 9;
  }
  long long nlch = 0;
  for (int r = 0; r < a.nlzr; r++) nlch += a.lzr[r][1] - a.lzr[r][0] + 1;
  const bool anylean = a.lx1 >= a.lx0 && a.ly1 >= a.ly0 && nlch > 0;
  const long long total = anylean ? (long long)(a.lx1 - a.lx0 + 1) * (a.ly1 - a.ly0 + 1) * nlch
                                  : 0;
  if (total == 0) return 0;
  long long nb = fused_grid_blocks(a.blocks_per_cu > 0 ? a.blocks_per_cu : 1);
  if (a.wg_limit > 0 && nb > a.wg_limit) nb = a.wg_limit;
  if (nb > total) nb = total;
  dim3 grd((unsigned)nb), blk(1024);
  const bool d2 = a.dist == 2;
  FusedArgs l = a;
  const long long ntile = (long long)(a.lx1 - a.lx0 + 1) * (a.ly1 - a.ly0 + 1);
  l.ngrp = (a.ngrp > 1 && ntile >= 4 * a.ngrp && nb >= a.ngrp) ? a.ngrp : 1;
  l.cbase = bases[0];
  if (l.ngrp == 1) {
    bases[0] += (unsigned long long)total + nb;
  } else {
    for (int g = 0; g < l.ngrp; g++) {
      l.cbg[g] = bases[g];
      const long long tiles = ntile * (g + 1) / l.ngrp - ntile * g / l.ngrp;
      const long long blocks = (nb - g + l.ngrp - 1) / l.ngrp;  // blockIdx % ngrp == g
      bases[g] += (unsigned long long)(tiles * nlch + blocks);
    }
  }
#define MNL_LAUNCH_FUSED(U)                                   \
  do {                                                        \
    if (d2)                                                   \
      fused_kernel<U, 2><<<grd, blk, 0, s>>>(l);              \
    else                                                      \
      fused_kernel<U, 1><<<grd, blk, 0, s>>>(l);              \
  } while (0)
  if (um == 2)
    MNL_LAUNCH_FUSED(2);
  else if (um == 1)
    MNL_LAUNCH_FUSED(1);
  else
    MNL_LAUNCH_FUSED(0);
#undef MNL_LAUNCH_FUSED
  return hipPeekAtLastError() == hipSuccess ? 0 : 9;
}

int k_tile_items(const FusedArgs &a, const int *items, const int *geo, const unsigned *flags,
                 int n, int line, void *stream, unsigned long long *bases) {
  if (n <= 0) return 0;
  if (a.nelem * 8 >= (long long)MNL_OOB || !a.ctr || !items || !geo || line < 0 ||
      line >= FUSED_NCTR)
    return 2;
  long long nb = fused_grid_blocks(a.blocks_per_cu > 0 ? a.blocks_per_cu : 1);
  if (a.wg_limit > 0 && nb > a.wg_limit) nb = a.wg_limit;
  if (nb > n) nb = n;
  FusedArgs t = a;
  t.titems = items, t.tgeo = geo, t.tflag = flags;
  t.gbeg = 0, t.gend = n, t.ctr_line = line, t.cbase = bases[line];
  bases[line] += (unsigned long long)n + nb;
  const int um = a.uidx ? 2 : (a.u[0] ? 1 : 0);
  hipStream_t s = (hipStream_t)stream;
  launch_tile(t, um, dim3((unsigned)nb), s);
  return hipPeekAtLastError() == hipSuccess ? 0 : 9;
}

int k_tile_items_uniform(const FusedArgs &a, const int *items, const int *geo, int n,
                         unsigned *flags, void *stream) {
  if (n <= 0 || !a.uidx) return 0;
  FusedArgs t = a;
  t.titems = items, t.tgeo = geo, t.ntit = n;
  tile_uniform_kernel<<<n, 256, 0, (hipStream_t)stream>>>(t, flags);
  return rc();
}

// ---------------------------------------------------------------------------
// the compact DFT box of an item (TB2Item::faces bits 8..10)
struct TB2Cmp {
  int lo0, lo1, lo2, n0, n1, n2;
  unsigned long long p;
  unsigned mask, ncell;
};
typedef const TB2Args __attribute__((address_space(4))) KTB;
// the D, B of one own point (column gx) at plane kk into the item's compact DFT box m (a wave
// with no lane in the box issues no store).  The box's parameters are read from the kernel
// arguments at each call through an opaque pointer, so they are not hoisted out of the plane
// loop into SGPRs (which are full there: held across the loop they spill and reload per plane)
__device__ __forceinline__ void tb2_cmp_store(int m, int state, bool own, int gx, int gy, int kk,
                                              double d0, double d1, double d2, double b0,
                                              double b1, double b2) {
  KTB *kt = (KTB *)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(kt));
  const auto &cc = kt->cmp[m];
  const TB2Cmp c{cc.lo[0], cc.lo[1], cc.lo[2], cc.n[0], cc.n[1], cc.n[2],
                 (unsigned long long)cc.p, cc.mask, cc.ncell};
  const int cx = gx - c.lo0, cy = gy - c.lo1, cz = kk - c.lo2;
  const bool in = own && cx >= 0 && cx < c.n0 && cy >= 0 && cy < c.n1 && cz >= 0 && cz < c.n2;
  if (__builtin_amdgcn_ballot_w64(in) == 0) return;
  const unsigned ci = (unsigned)(cx + c.n0 * (cy + c.n1 * cz));
  const unsigned st = (unsigned)state * 6u;
  const auto r = brsrc_at(c.p, c.ncell * 96u);
  const double v[6] = {d0, d1, d2, b0, b1, b2};
#pragma unroll
  for (int q = 0; q < 6; q++)
    if ((c.mask >> q) & 1u) bst(r, in ? ((st + q) * c.ncell + ci) * 8u : MNL_OOB, v[q]);
}

// the kernel arguments behind an empty asm: fields read through it at a use inside the plane
// loop are scalar loads there (kernarg segment, constant cache) instead of SGPRs held across it
__device__ __forceinline__ KTB *tb2_kargs() {
  KTB *kt = (KTB *)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(kt));
  return kt;
}

// a wave-uniform double moved to SGPRs (readfirstlane of both halves)
__device__ __forceinline__ double sgpr_f64(double v) {
  const mnl_u2 u = __builtin_bit_cast(mnl_u2, v);
  mnl_u2 r;
  r.x = __builtin_amdgcn_readfirstlane(u.x);
  r.y = __builtin_amdgcn_readfirstlane(u.y);
  return __builtin_bit_cast(double, r);
}
// descriptor of a non-null scalar pointer built where it is used (no null test: s_cselect-free)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc_nn(unsigned long long v, unsigned nrec) {
  asm volatile("" : "+s"(v));
  return __builtin_amdgcn_make_buffer_rsrc((void *)v, 0, (int)nrec, 0x00020000);
}

// ---- two columns per lane: 16-byte loads / stores, x neighbours across lanes by DPP
typedef double mnl_d2 __attribute__((ext_vector_type(2)));
typedef unsigned int mnl_u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ mnl_d2 ldg2(gdp p, unsigned off) {
  return *(const mnl_d2 __attribute__((address_space(1))) *)((const char __attribute__((address_space(1))) *)p + off);
}
__device__ __forceinline__ mnl_u2 ldu2(gup p, unsigned off) {
  return *(const mnl_u2 __attribute__((address_space(1))) *)((const char __attribute__((address_space(1))) *)p + off);
}
__device__ __forceinline__ void bst2(__amdgpu_buffer_rsrc_t r, unsigned off, double a, double b) {
  const mnl_u2 x = __builtin_bit_cast(mnl_u2, a), y = __builtin_bit_cast(mnl_u2, b);
  mnl_u4 q;
  q.x = x.x, q.y = x.y, q.z = y.x, q.w = y.y;
  __builtin_amdgcn_raw_buffer_store_b128(q, r, off, 0, 0);
}
// lane i <- lane i + 1 (DPP wave_shl:1) / lane i <- lane i - 1 (wave_shr:1); the end lane keeps
// its own value (a column outside every own point's stencil)
__device__ __forceinline__ double lane_next(double x) {
  const mnl_u2 u = __builtin_bit_cast(mnl_u2, x);
  mnl_u2 r;
  r.x = __builtin_amdgcn_update_dpp((int)u.x, (int)u.x, 0x130, 0xF, 0xF, false);
  r.y = __builtin_amdgcn_update_dpp((int)u.y, (int)u.y, 0x130, 0xF, 0xF, false);
  return __builtin_bit_cast(double, r);
}
__device__ __forceinline__ double lane_prev(double x) {
  const mnl_u2 u = __builtin_bit_cast(mnl_u2, x);
  mnl_u2 r;
  r.x = __builtin_amdgcn_update_dpp((int)u.x, (int)u.x, 0x138, 0xF, 0xF, false);
  r.y = __builtin_amdgcn_update_dpp((int)u.y, (int)u.y, 0x138, 0xF, 0xF, false);
  return __builtin_bit_cast(double, r);
}
// y-neighbour exchange of the two-step kernel: per padded row (rows 0 and TB_LY + 1 pad, so a
// wave's rows w - 1 / w + 1 are constant offsets from one per-lane address within the 16-bit
// offset of ds_read_b128) 8 slots of 128 columns: E^n z, x; E^{n+1} z, x; B^{n+1} z, x;
// B^{n+2} z, x
struct alignas(16) TB2Lds {
  double s[TB_LY + 2][8][TB_LX * TB_PX];
};
enum { TBS_E1Z, TBS_E1X, TBS_E2Z, TBS_E2X, TBS_H1Z, TBS_H1X, TBS_H2Z, TBS_H2X };
constexpr int TB_RS = 8 * TB_LX * TB_PX;  // doubles per padded row
#define TBO(row, slot) ((row) * TB_RS + (slot) * TB_LX * TB_PX)
__device__ __forceinline__ void tb_put(double *bp, int o, double a, double b) {
  mnl_d2 t;
  t.x = a, t.y = b;
  *(mnl_d2 *)(bp + o) = t;
}
__device__ __forceinline__ void tb_get(const double *bp, int o, double &a, double &b) {
  const mnl_d2 t = *(const mnl_d2 *)(bp + o);
  a = t.x, b = t.y;
}
// chi1inv of one column: UMODE 0 none (E = D), 1 the f64 arrays, 2 a palette word (LDS table)
template <int UMODE>
struct TbU {
  unsigned w;
  __device__ double get(int c, const double (*sU)[256]) const { return sU[c][(w >> (8 * c)) & 255]; }
};
template <>
struct TbU<1> {
  double u0, u1, u2;
  __device__ double get(int c, const double (*)[256]) const { return c == 0 ? u0 : (c == 1 ? u1 : u2); }
};
template <>
struct TbU<0> {
  __device__ double get(int, const double (*)[256]) const { return 1.0; }
};

// Temporal blocking: steps n -> n+1 -> n+2 in one z-march over an
// item of the region L2, where every point within L-infinity distance 2 of an own point is
// lean (no PML, every component owned, H == B, E implicit) and no source point lies within
// distance 1 of an own point.  Per plane k of the march: step n at plane k on all 128 x 16
// columns (B^{n+1}(k), then D^{n+1}(k) from B^{n+1}(k-1) kept in registers), then step n+1 at
// plane k-1 from E^{n+1}(k-1) and E^{n+1}(k).  Per two steps a point's D and B are read once
// and written once (plus the step-n+1 values of the points on a face that borders the rim,
// which the one-step rim launch of step n+1 reads).  The arithmetic of each update is the lean
// body's expression, operand for operand (src/step_generic.cpp:106-113 curl, 888-903
// E = chi1inv * D), so two steps here are bitwise two one-step launches.
//
// Round 6 layout: two adjacent columns per lane (TB_PX), so a workgroup covers 128 x 16 columns
// for up to 124 x 12 own points (was 64 x 16 for 60 x 12: the x halo lines and the per-plane
// barriers are paid for twice the points).  x neighbours: the lane's other column or the next /
// previous lane's (DPP); y neighbours: LDS (two components per exchange, 16-byte accesses).
// Carried across planes: D^n(k), B^{n+1}(k-1), D^{n+1}(k-1), B^{n+2}(k-2) x, y and the chi1inv
// of k and k-1; E^n(k) = chi1inv D^n(k) and E^{n+1}(k-1) are recomputed per plane (the same
// products, so the same values).  B^n(k+1) is loaded after the B update of plane k (half a
// plane ahead), D^n(k+2) and chi1inv(k+2) a whole plane ahead.
template <int UMODE, bool UNI, bool CMP>
__device__ __forceinline__ void tb2_body(const TB2Args &a, const TB2Item it, unsigned uw,
                                         const double (*sU)[256], TB2Lds &L) {
  typedef TbU<UMODE> U;
  constexpr bool HAS_U = UMODE != 0;
  const int tid = tid_item(), lane = tid & 63, w = tid >> 6;
  const int x0 = it.x & 0xFFFF, x1 = it.x >> 16, y0 = it.y & 0xFFFF, y1 = it.y >> 16;
  const int zs = it.z & 0xFFFF, ze = it.z >> 16;
  const int faces = it.faces;
  // the item's compact DFT box (-1: none; CMP = false: no box in this launch, none compiled)
  const int cmi = CMP ? ((faces >> 8) & 7) - 1 : -1;
  const int gx = it.lx + TB_PX * lane, gy = y0 - TB_HY + w;  // this lane's columns gx, gx + 1
  const int N1 = a.N[1], zmax = a.N[2] - 1;
  const int cx = min(max(gx, 0), (int)a.st1 - TB_PX), cy = min(max(gy, 0), N1 - 1);
  const unsigned col = (unsigned)((cx + (long long)cy * a.st1) * 8);
  const unsigned s2 = (unsigned)(a.st2 * 8);
  const double C = a.C;
  const bool oy = gy >= y0 && gy <= y1;
  const bool own0 = oy && gx >= x0 && gx <= x1, own1 = oy && gx + 1 >= x0 && gx + 1 <= x1;
  // item-uniform: an own range that starts or ends inside a lane's column pair (b64 stores)
  const bool ragged = ((x0 - it.lx) & 1) != 0 || ((x1 - it.lx) & 1) == 0;
  // the item stores step-n+1 values of some points (rim-bordering faces, DFT / guard box)
  const bool anymid = (faces & 63) != 0 || it.bx >= 0;
  const unsigned nrec = (unsigned)min(a.nelem * 8, 0xFFFFFFFFLL);
  const gdp D0 = sgpr_ptr(a.Do[0]), D1 = sgpr_ptr(a.Do[1]), D2 = sgpr_ptr(a.Do[2]);
  const gdp B0 = sgpr_ptr(a.Bo[0]), B1 = sgpr_ptr(a.Bo[1]), B2 = sgpr_ptr(a.Bo[2]);
  const gdp U0 = UMODE == 1 ? sgpr_ptr(a.u[0]) : nullptr;
  const gdp U1 = UMODE == 1 ? sgpr_ptr(a.u[1]) : nullptr;
  const gdp U2 = UMODE == 1 ? sgpr_ptr(a.u[2]) : nullptr;
  const gup uix = (gup)sgpr_ptr(a.uidx);
  // chi1inv of a uniform item (wave-uniform: held in SGPRs, VALU operands)
  double cu0 = 1, cu1 = 1, cu2 = 1;
  if (UMODE == 2 && UNI) {
    cu0 = sgpr_f64(sU[0][uw & 255]), cu1 = sgpr_f64(sU[1][(uw >> 8) & 255]);
    cu2 = sgpr_f64(sU[2][(uw >> 16) & 255]);
  }
  auto uv = [&](const U &u, int c) -> double {
    if (UMODE == 2 && UNI) return c == 0 ? cu0 : (c == 1 ? cu1 : cu2);
    return u.get(c, sU);
  };
  auto zc = [zmax](int z) { return min(max(z, 0), zmax); };
  auto ldu = [&](unsigned o, U &u0, U &u1) {
    if constexpr (UMODE == 2) {
      if (UNI) {
        u0.w = u1.w = 0;
      } else {
        const mnl_u2 t = ldu2(uix, o >> 1);
        u0.w = t.x, u1.w = t.y;
      }
    } else if constexpr (UMODE == 1) {
      mnl_d2 t = ldg2(U0, o);
      u0.u0 = t.x, u1.u0 = t.y;
      t = ldg2(U1, o);
      u0.u1 = t.x, u1.u1 = t.y;
      t = ldg2(U2, o);
      u0.u2 = t.x, u1.u2 = t.y;
    }
  };
  struct QD {  // D and chi1inv of one plane
    mnl_d2 d0, d1, d2;
    U u0, u1;
  };
  auto loadd = [&](int k) -> QD {
    QD q;
    const unsigned o = col + (unsigned)zc(k) * s2;
    q.d0 = ldg2(D0, o);
    q.d1 = ldg2(D1, o);
    q.d2 = ldg2(D2, o);
    ldu(o, q.u0, q.u1);
    return q;
  };
  struct QB {
    mnl_d2 b0, b1, b2;
  };
  auto loadb = [&](int k) -> QB {
    QB q;
    const unsigned o = col + (unsigned)zc(k) * s2;
    q.b0 = ldg2(B0, o);
    q.b1 = ldg2(B1, o);
    q.b2 = ldg2(B2, o);
    return q;
  };
  // this lane's slot in its padded row (row w + 1): rows w / w + 2 are constant offsets
  double *bp = &L.s[0][0][0] + (w * TB_RS + TB_PX * lane);
  const int k0 = zs - 2;
  // prologue: D^n(k0) and chi1inv(k0); then D(k0 + 1) and B(k0)
  double dn0[3], dn1[3];
  U uk0, uk1, um0, um1;  // chi1inv of the march plane k and of k - 1, columns 0 / 1
  {
    const QD p = loadd(k0);
    dn0[0] = p.d0.x, dn1[0] = p.d0.y, dn0[1] = p.d1.x, dn1[1] = p.d1.y;
    dn0[2] = p.d2.x, dn1[2] = p.d2.y;
    uk0 = p.u0, uk1 = p.u1;
    um0 = uk0, um1 = uk1;
  }
  QD qd = loadd(k0 + 1);
  QB qb = loadb(k0);
  double b10[3] = {0, 0, 0}, b11[3] = {0, 0, 0};  // B^{n+1}(k-1)
  double d10[3] = {0, 0, 0}, d11[3] = {0, 0, 0};  // D^{n+1}(k-1)
  double h2x0 = 0, h2y0 = 0, h2x1 = 0, h2y1 = 0;  // B^{n+2}(k-2) x, y
  for (int k = k0; k <= ze; k++) {
    const QD c = qd;  // D^n(k+1), chi1inv(k+1)
    const QB cb = qb;  // B^n(k)
    qd = loadd(min(k + 2, ze + 1));
    // E^n(k+1) x, y; E^n(k); E^{n+1}(k-1)
    double e1x0, e1y0, e1x1, e1y1, en0[3], en1[3], f10[3], f11[3];
    e1x0 = c.d0.x, e1y0 = c.d1.x, e1x1 = c.d0.y, e1y1 = c.d1.y;
    if (HAS_U) {
      e1x0 = c.d0.x * uv(c.u0, 0), e1y0 = c.d1.x * uv(c.u0, 1);
      e1x1 = c.d0.y * uv(c.u1, 0), e1y1 = c.d1.y * uv(c.u1, 1);
    }
#pragma unroll
    for (int q = 0; q < 3; q++) {
      en0[q] = dn0[q], en1[q] = dn1[q], f10[q] = d10[q], f11[q] = d11[q];
      if (HAS_U) {
        en0[q] = dn0[q] * uv(uk0, q), en1[q] = dn1[q] * uv(uk1, q);
        f10[q] = d10[q] * uv(um0, q), f11[q] = d11[q] * uv(um1, q);
      }
    }
    tb_put(bp, TBO(1, TBS_E1Z), en0[2], en1[2]);
    tb_put(bp, TBO(1, TBS_E1X), en0[0], en1[0]);
    tb_put(bp, TBO(1, TBS_E2Z), f10[2], f11[2]);
    tb_put(bp, TBO(1, TBS_E2X), f10[0], f11[0]);
    __syncthreads();
    // ---- step n at plane k: B^{n+1}(k) (curl E^n), H == B
    double Bx0, By0, Bz0, Bx1, By1, Bz1;
    {
      double ezy0, ezy1, exy0, exy1;
      tb_get(bp, TBO(2, TBS_E1Z), ezy0, ezy1);
      tb_get(bp, TBO(2, TBS_E1X), exy0, exy1);
      const double ezx1 = lane_next(en0[2]), eyx1 = lane_next(en0[1]);
      Bx0 = cb.b0.x - C * (ezy0 - en0[2] + en0[1] - e1y0);
      By0 = cb.b1.x - C * (e1x0 - en0[0] + en0[2] - en1[2]);
      Bz0 = cb.b2.x - C * (en1[1] - en0[1] + en0[0] - exy0);
      Bx1 = cb.b0.y - C * (ezy1 - en1[2] + en1[1] - e1y1);
      By1 = cb.b1.y - C * (e1x1 - en1[0] + en1[2] - ezx1);
      Bz1 = cb.b2.y - C * (eyx1 - en1[1] + en1[0] - exy1);
    }
    tb_put(bp, TBO(1, TBS_H1Z), Bz0, Bz1);
    tb_put(bp, TBO(1, TBS_H1X), Bx0, Bx1);
    qb = loadb(min(k + 1, ze));
    __syncthreads();
    // D^{n+1}(k) (curl H^{n+1}), E^{n+1}(k) x, y = chi1inv * D^{n+1}(k)
    double Dx0, Dy0, Dz0, Dx1, Dy1, Dz1;
    {
      double hzy0, hzy1, hxy0, hxy1;
      tb_get(bp, TBO(0, TBS_H1Z), hzy0, hzy1);
      tb_get(bp, TBO(0, TBS_H1X), hxy0, hxy1);
      const double hzx0 = lane_prev(Bz1), hyx0 = lane_prev(By1);
      Dx0 = dn0[0] - C * (hzy0 - Bz0 + By0 - b10[1]);
      Dy0 = dn0[1] - C * (b10[0] - Bx0 + Bz0 - hzx0);
      Dz0 = dn0[2] - C * (hyx0 - By0 + Bx0 - hxy0);
      Dx1 = dn1[0] - C * (hzy1 - Bz1 + By1 - b11[1]);
      Dy1 = dn1[1] - C * (b11[0] - Bx1 + Bz1 - Bz0);
      Dz1 = dn1[2] - C * (By0 - By1 + Bx1 - hxy1);
    }
    double Ex0 = Dx0, Ey0 = Dy0, Ex1 = Dx1, Ey1 = Dy1;
    if (HAS_U) {
      Ex0 = Dx0 * uv(uk0, 0), Ey0 = Dy0 * uv(uk0, 1);
      Ex1 = Dx1 * uv(uk1, 0), Ey1 = Dy1 * uv(uk1, 1);
    }
    // ---- step n+1 at plane k-1: B^{n+2}(k-1) from E^{n+1}(k-1) (f1) and E^{n+1}(k)
    double Fx0, Fy0, Fz0, Fx1, Fy1, Fz1;
    {
      double fzy0, fzy1, fxy0, fxy1;
      tb_get(bp, TBO(2, TBS_E2Z), fzy0, fzy1);
      tb_get(bp, TBO(2, TBS_E2X), fxy0, fxy1);
      const double fzx1 = lane_next(f10[2]), fyx1 = lane_next(f10[1]);
      Fx0 = b10[0] - C * (fzy0 - f10[2] + f10[1] - Ey0);
      Fy0 = b10[1] - C * (Ex0 - f10[0] + f10[2] - f11[2]);
      Fz0 = b10[2] - C * (f11[1] - f10[1] + f10[0] - fxy0);
      Fx1 = b11[0] - C * (fzy1 - f11[2] + f11[1] - Ey1);
      Fy1 = b11[1] - C * (Ex1 - f11[0] + f11[2] - fzx1);
      Fz1 = b11[2] - C * (fyx1 - f11[1] + f11[0] - fxy1);
    }
    tb_put(bp, TBO(1, TBS_H2Z), Fz0, Fz1);
    tb_put(bp, TBO(1, TBS_H2X), Fx0, Fx1);
    if (anymid) {  // step-n+1 values of the points on a face bordering the rim (read by rim
                   // step n+1), of the DFT / NaN-guard box, of the compact DFT box
      const bool kin = k >= zs && k < ze;
      const bool kz = ((faces & 16) && k == zs) || ((faces & 32) && k == ze - 1);
      const int bx0 = it.bx & 0xFFFF, bx1 = it.bx >> 16;
      const bool dy = it.bx >= 0 && gy >= (it.by & 0xFFFF) && gy <= (it.by >> 16) &&
                      k >= (it.bz & 0xFFFF) && k <= (it.bz >> 16);
      const bool fy = ((faces & 4) && gy == y0) || ((faces & 8) && gy == y1);
      const bool bd0 = kin && own0 && (fy || kz || ((faces & 1) && gx == x0) ||
                                       ((faces & 2) && gx == x1) || (dy && gx >= bx0 && gx <= bx1));
      const bool bd1 = kin && own1 && (fy || kz || ((faces & 1) && gx + 1 == x0) ||
                                       ((faces & 2) && gx + 1 == x1) ||
                                       (dy && gx + 1 >= bx0 && gx + 1 <= bx1));
      const unsigned ob = col + (unsigned)k * s2;
      const unsigned o2 = bd0 && bd1 ? ob : MNL_OOB, oa = bd0 && !bd1 ? ob : MNL_OOB,
                     oc = bd1 && !bd0 ? ob + 8 : MNL_OOB;
      KTB *kt = tb2_kargs();  // output pointers read at use (not held across the loop)
      const unsigned long long pm[6] = {
          (unsigned long long)kt->Bm[0], (unsigned long long)kt->Bm[1],
          (unsigned long long)kt->Bm[2], (unsigned long long)kt->Dm[0],
          (unsigned long long)kt->Dm[1], (unsigned long long)kt->Dm[2]};
      const double v0[6] = {Bx0, By0, Bz0, Dx0, Dy0, Dz0}, v1[6] = {Bx1, By1, Bz1, Dx1, Dy1, Dz1};
#pragma unroll
      for (int q = 0; q < 6; q++) {
        const auto r = brsrc_nn(pm[q], nrec);
        bst2(r, o2, v0[q], v1[q]);
        bst(r, oa, v0[q]);
        bst(r, oc, v1[q]);
      }
      if (CMP && cmi >= 0) {
        tb2_cmp_store(cmi, 0, own0 && kin, gx, gy, k, Dx0, Dy0, Dz0, Bx0, By0, Bz0);
        tb2_cmp_store(cmi, 0, own1 && kin, gx + 1, gy, k, Dx1, Dy1, Dz1, Bx1, By1, Bz1);
      }
    }
    __syncthreads();
    double Gx0, Gy0, Gz0, Gx1, Gy1, Gz1;
    {
      double gzy0, gzy1, gxy0, gxy1;
      tb_get(bp, TBO(0, TBS_H2Z), gzy0, gzy1);
      tb_get(bp, TBO(0, TBS_H2X), gxy0, gxy1);
      const double gzx0 = lane_prev(Fz1), gyx0 = lane_prev(Fy1);
      Gx0 = d10[0] - C * (gzy0 - Fz0 + Fy0 - h2y0);
      Gy0 = d10[1] - C * (h2x0 - Fx0 + Fz0 - gzx0);
      Gz0 = d10[2] - C * (gyx0 - Fy0 + Fx0 - gxy0);
      Gx1 = d11[0] - C * (gzy1 - Fz1 + Fy1 - h2y1);
      Gy1 = d11[1] - C * (h2x1 - Fx1 + Fz1 - Fz0);
      Gz1 = d11[2] - C * (Fy0 - Fy1 + Fx1 - gxy1);
    }
    {
      const bool st = k - 1 >= zs && k - 1 < ze;
      const unsigned os = col + (unsigned)(k - 1) * s2;
      const unsigned o2 = st && own0 && own1 ? os : MNL_OOB;
      KTB *kt = tb2_kargs();
      const unsigned long long pn[6] = {
          (unsigned long long)kt->Bn[0], (unsigned long long)kt->Bn[1],
          (unsigned long long)kt->Bn[2], (unsigned long long)kt->Dn[0],
          (unsigned long long)kt->Dn[1], (unsigned long long)kt->Dn[2]};
      const double v0[6] = {Fx0, Fy0, Fz0, Gx0, Gy0, Gz0}, v1[6] = {Fx1, Fy1, Fz1, Gx1, Gy1, Gz1};
#pragma unroll
      for (int q = 0; q < 6; q++) bst2(brsrc_nn(pn[q], nrec), o2, v0[q], v1[q]);
      if (ragged) {  // an own range starting or ending inside a column pair
        const unsigned oa = st && own0 && !own1 ? os : MNL_OOB;
        const unsigned oc = st && own1 && !own0 ? os + 8 : MNL_OOB;
#pragma unroll
        for (int q = 0; q < 6; q++) {
          const auto r = brsrc_nn(pn[q], nrec);
          bst(r, oa, v0[q]);
          bst(r, oc, v1[q]);
        }
      }
      if (CMP && cmi >= 0) {
        tb2_cmp_store(cmi, 1, st && own0, gx, gy, k - 1, Gx0, Gy0, Gz0, Fx0, Fy0, Fz0);
        tb2_cmp_store(cmi, 1, st && own1, gx + 1, gy, k - 1, Gx1, Gy1, Gz1, Fx1, Fy1, Fz1);
      }
    }
    h2x0 = Fx0, h2y0 = Fy0, h2x1 = Fx1, h2y1 = Fy1;
    b10[0] = Bx0, b10[1] = By0, b10[2] = Bz0, b11[0] = Bx1, b11[1] = By1, b11[2] = Bz1;
    d10[0] = Dx0, d10[1] = Dy0, d10[2] = Dz0, d11[0] = Dx1, d11[1] = Dy1, d11[2] = Dz1;
    dn0[0] = c.d0.x, dn1[0] = c.d0.y, dn0[1] = c.d1.x, dn1[1] = c.d1.y;
    dn0[2] = c.d2.x, dn1[2] = c.d2.y;
    um0 = uk0, um1 = uk1, uk0 = c.u0, uk1 = c.u1;
  }
}
#undef TBO

template <int UMODE, bool CLK, bool CMP>
__global__ __launch_bounds__(1024) void tb2_kernel(TB2Args a) {
  __shared__ double sU[UMODE == 2 ? 3 : 1][256];
  __shared__ TB2Lds L;
  __shared__ int s_idx;
  __shared__ unsigned long long s_t0;
  if (UMODE == 2) {  // palette -> LDS (visible after the first barrier below)
    for (int i = threadIdx.x; i < 3 * 256; i += 1024) sU[i >> 8][i & 255] = a.utab[i];
  }
  unsigned long long *ctr = a.ctr + 16 * a.ctr_line;
  if (CLK && threadIdx.x == 0) s_t0 = 0ull;  // no previous item
  for (;;) {
    if (threadIdx.x == 0) {
      if (CLK && s_t0 != 0ull) {  // diagnostics: the previous item (see fused_tile_kernel)
        const TB2Item it = a.items[s_idx];
        const unsigned uw = (UMODE == 2 && a.uflag) ? a.uflag[s_idx] : ~0u;
        clk_record(a.clk, s_t0, (it.faces & 63) | (uw != ~0u ? 64 : 0), it.x, it.y, it.z, -1);
      }
      const unsigned long long v = atomicAdd(ctr, 1ULL) - a.cbase;
      s_idx = v < (unsigned long long)(a.n) ? (int)v : -1;
      if (CLK) s_t0 = wall_clock64();
    }
    __syncthreads();  // also separates LDS use of consecutive items
    const int idx = s_idx;
    if (idx < 0) break;
    const TB2Item it = a.items[idx];
    const unsigned uw = (UMODE == 2 && a.uflag) ? a.uflag[idx] : ~0u;
    if (UMODE == 2 && __builtin_amdgcn_readfirstlane(uw) != ~0u)
      tb2_body<UMODE, true, CMP>(a, it, uw, sU, L);
    else
      tb2_body<UMODE, false, CMP>(a, it, uw, sU, L);
  }
}

// ---- the round-5 two-step kernel (one column per lane, 64 x 16 lanes for up to 60 x 12 own
// points; x and y neighbours through LDS), kept for in-process A/B against the round-6 layout
// (set_schedule "tb_px" = 1)
// Temporal blocking: steps n -> n+1 -> n+2 in one z-march over an
// item of the region L2, where every point within L-infinity distance 2 of an own point is
// lean (no PML, every component owned, H == B, E implicit) and no source point lies within
// distance 1 of an own point.  Per plane k of the march: step n at plane k on all 64 x 16
// lanes (B^{n+1}(k), then D^{n+1}(k) from B^{n+1}(k-1) kept in registers), then step n+1 at
// plane k-1 from E^{n+1}(k-1) (registers, LDS for the neighbours) and E^{n+1}(k) (this
// lane).  Per two steps a point's D and B are read once and written once (plus the step-n+1
// values of the points on a face that borders the rim, which the one-step rim launch of
// step n+1 reads).  The arithmetic of each update is the lean body's expression, operand
// for operand (src/step_generic.cpp:106-113 curl, 888-903 E = chi1inv * D), so two steps
// here are bitwise two one-step launches.
template <int UMODE, bool UNI, bool CMP>
__device__ __forceinline__ void tb2_body1(const TB2Args &a, const TB2Item it, unsigned uw,
                                         const double (*sU)[256], double (*sE1)[TB_LY][TB_LX],
                                         double (*sH1)[TB_LY][TB_LX], double (*sE2)[TB_LY][TB_LX],
                                         double (*sH2)[TB_LY][TB_LX]) {
  constexpr bool HAS_U = UMODE != 0;
  const int tid = tid_item(), lane = tid & 63, w = tid >> 6;
  const int x0 = it.x & 0xFFFF, x1 = it.x >> 16, y0 = it.y & 0xFFFF, y1 = it.y >> 16;
  const int zs = it.z & 0xFFFF, ze = it.z >> 16;
  const int faces = it.faces;
  // the item's compact DFT box (-1: none; CMP = false: no box in this launch, none compiled)
  const int cmi = CMP ? ((faces >> 8) & 7) - 1 : -1;
  const int gx = it.lx + lane, gy = y0 - TB_HY + w;  // lanes from the item's 64-byte line
  const int N0 = a.N[0], N1 = a.N[1], zmax = a.N[2] - 1;
  const int cx = min(max(gx, 0), N0 - 1), cy = min(max(gy, 0), N1 - 1);
  const unsigned col = (unsigned)((cx + (long long)cy * a.st1) * 8);
  const unsigned s2 = (unsigned)(a.st2 * 8);
  const double C = a.C;
  const bool own = gx >= x0 && gx <= x1 && gy >= y0 && gy <= y1;
  const bool bxy = own && (((faces & 1) && gx == x0) || ((faces & 2) && gx == x1) ||
                           ((faces & 4) && gy == y0) || ((faces & 8) && gy == y1));
  // DFT monitor box: step n+1 of these points is stored too (it.bx < 0: none)
  const bool dxy = own && it.bx >= 0 && gx >= (it.bx & 0xFFFF) && gx <= (it.bx >> 16) &&
                   gy >= (it.by & 0xFFFF) && gy <= (it.by >> 16);
  const int dz0 = it.bz & 0xFFFF, dz1 = it.bz >> 16;
  const unsigned nrec = (unsigned)min(a.nelem * 8, 0xFFFFFFFFLL);
  // output arrays as scalar pointers; a buffer descriptor is built at each store (a
  // descriptor per array live across the loop would overflow the SGPRs)
  const unsigned long long pBn0 = (unsigned long long)sgpr_ptr(a.Bn[0]),
                           pBn1 = (unsigned long long)sgpr_ptr(a.Bn[1]),
                           pBn2 = (unsigned long long)sgpr_ptr(a.Bn[2]),
                           pDn0 = (unsigned long long)sgpr_ptr(a.Dn[0]),
                           pDn1 = (unsigned long long)sgpr_ptr(a.Dn[1]),
                           pDn2 = (unsigned long long)sgpr_ptr(a.Dn[2]),
                           pBm0 = (unsigned long long)sgpr_ptr(a.Bm[0]),
                           pBm1 = (unsigned long long)sgpr_ptr(a.Bm[1]),
                           pBm2 = (unsigned long long)sgpr_ptr(a.Bm[2]),
                           pDm0 = (unsigned long long)sgpr_ptr(a.Dm[0]),
                           pDm1 = (unsigned long long)sgpr_ptr(a.Dm[1]),
                           pDm2 = (unsigned long long)sgpr_ptr(a.Dm[2]);
  const gdp D0 = sgpr_ptr(a.Do[0]), D1 = sgpr_ptr(a.Do[1]), D2 = sgpr_ptr(a.Do[2]);
  const gdp B0 = sgpr_ptr(a.Bo[0]), B1 = sgpr_ptr(a.Bo[1]), B2 = sgpr_ptr(a.Bo[2]);
  const gdp U0 = UMODE == 1 ? sgpr_ptr(a.u[0]) : nullptr;
  const gdp U1 = UMODE == 1 ? sgpr_ptr(a.u[1]) : nullptr;
  const gdp U2 = UMODE == 1 ? sgpr_ptr(a.u[2]) : nullptr;
  const gup uix = (gup)sgpr_ptr(a.uidx);
  // chi1inv of a uniform item
  double cu0 = 1, cu1 = 1, cu2 = 1;
  if (UMODE == 2 && UNI) {
    cu0 = sU[0][uw & 255], cu1 = sU[1][(uw >> 8) & 255], cu2 = sU[2][(uw >> 16) & 255];
  }
  struct Q {
    double d0, d1, d2, b0, b1, b2, u0, u1, u2;
    unsigned ui;
  };
  auto zc = [zmax](int z) { return min(max(z, 0), zmax); };
  // plane k: D(k+1), chi1inv(k+1), B(k)
  auto load = [&](int k) -> Q {
    Q q;
    const unsigned o1 = col + (unsigned)zc(k + 1) * s2, ob = col + (unsigned)zc(k) * s2;
    q.d0 = ldg(D0, o1);
    q.d1 = ldg(D1, o1);
    q.d2 = ldg(D2, o1);
    q.ui = 0;
    q.u0 = q.u1 = q.u2 = 1.0;
    if (UMODE == 2 && !UNI) q.ui = ldu(uix, o1 >> 1);
    if (UMODE == 1) {
      q.u0 = ldg(U0, o1);
      q.u1 = ldg(U1, o1);
      q.u2 = ldg(U2, o1);
    }
    q.b0 = ldg(B0, ob);
    q.b1 = ldg(B1, ob);
    q.b2 = ldg(B2, ob);
    return q;
  };
  auto uval = [&](const Q &q, int c) -> double {
    if (UMODE == 2) {
      if (UNI) return c == 0 ? cu0 : (c == 1 ? cu1 : cu2);
      return sU[c][(q.ui >> (8 * c)) & 255];
    }
    return c == 0 ? q.u0 : (c == 1 ? q.u1 : q.u2);
  };
  const int k0 = zs - 2;
  // prologue: D^n(k0), E^n(k0)
  double dnx, dny, dnz, enx, eny, enz;
  double uk0, uk1, uk2;  // chi1inv at the march plane k (E^{n+1}(k) = D^{n+1}(k) * u(k))
  {
    Q p;
    const unsigned o = col + (unsigned)zc(k0) * s2;
    p.d0 = ldg(D0, o), p.d1 = ldg(D1, o), p.d2 = ldg(D2, o);
    p.ui = (UMODE == 2 && !UNI) ? ldu(uix, o >> 1) : 0u;
    p.u0 = p.u1 = p.u2 = 1.0;
    if (UMODE == 1) p.u0 = ldg(U0, o), p.u1 = ldg(U1, o), p.u2 = ldg(U2, o);
    dnx = p.d0, dny = p.d1, dnz = p.d2;
    if (HAS_U) {
      enx = dnx * uval(p, 0), eny = dny * uval(p, 1), enz = dnz * uval(p, 2);
    } else {
      enx = dnx, eny = dny, enz = dnz;
    }
  }
  Q q = load(k0);
  uk0 = uk1 = uk2 = 1.0;
  double h1x = 0, h1y = 0;                // B^{n+1}(k-1) x, y
  double b1x = 0, b1y = 0, b1z = 0;       // B^{n+1}(k-1)
  double d1x = 0, d1y = 0, d1z = 0;       // D^{n+1}(k-1)
  double f1x = 0, f1y = 0, f1z = 0;       // E^{n+1}(k-1)
  double h2x = 0, h2y = 0;                // B^{n+2}(k-2) x, y
  const int lp = min(lane + 1, TB_LX - 1), lm = max(lane - 1, 0);
  const int wp = min(w + 1, TB_LY - 1), wm = max(w - 1, 0);
  for (int k = k0; k <= ze; k++) {
    const Q c = q;
    q = load(min(k + 1, ze));
    // E^n(k+1); chi1inv(k+1) becomes u(k) of the next plane
    double e1x, e1y, e1z, v0 = 1, v1 = 1, v2 = 1;
    if (HAS_U) {
      v0 = uval(c, 0), v1 = uval(c, 1), v2 = uval(c, 2);
      e1x = c.d0 * v0, e1y = c.d1 * v1, e1z = c.d2 * v2;
    } else {
      e1x = c.d0, e1y = c.d1, e1z = c.d2;
    }
    sE1[0][w][lane] = enx, sE1[1][w][lane] = eny, sE1[2][w][lane] = enz;
    sE2[0][w][lane] = f1x, sE2[1][w][lane] = f1y, sE2[2][w][lane] = f1z;
    __syncthreads();
    // ---- step n at plane k: B^{n+1}(k) (curl E^n), H == B
    const double Bx = c.b0 - C * (sE1[2][wp][lane] - enz + eny - e1y);
    const double By = c.b1 - C * (e1x - enx + enz - sE1[2][w][lp]);
    const double Bz = c.b2 - C * (sE1[1][w][lp] - eny + enx - sE1[0][wp][lane]);
    sH1[0][w][lane] = Bx, sH1[1][w][lane] = By, sH1[2][w][lane] = Bz;
    __syncthreads();
    // D^{n+1}(k) (curl H^{n+1}), E^{n+1}(k) = chi1inv * D^{n+1}(k)
    const double Dx = dnx - C * (sH1[2][wm][lane] - Bz + By - h1y);
    const double Dy = dny - C * (h1x - Bx + Bz - sH1[2][w][lm]);
    const double Dz = dnz - C * (sH1[1][w][lm] - By + Bx - sH1[0][wm][lane]);
    double Ex = Dx, Ey = Dy, Ez = Dz;
    if (HAS_U) Ex = Dx * uk0, Ey = Dy * uk1, Ez = Dz * uk2;
    {  // step-n+1 values of the points on a face bordering the rim (read by rim step n+1)
      const bool kin = k >= zs && k < ze;
      const bool bd = kin && (bxy || (own && (((faces & 16) && k == zs) || ((faces & 32) && k == ze - 1))) ||
                              (dxy && k >= dz0 && k <= dz1));
      const unsigned ob = bd ? col + (unsigned)k * s2 : MNL_OOB;
      bst(brsrc_at(pBm0, nrec), ob, Bx);
      bst(brsrc_at(pBm1, nrec), ob, By);
      bst(brsrc_at(pBm2, nrec), ob, Bz);
      bst(brsrc_at(pDm0, nrec), ob, Dx);
      bst(brsrc_at(pDm1, nrec), ob, Dy);
      bst(brsrc_at(pDm2, nrec), ob, Dz);
      if (CMP && cmi >= 0) tb2_cmp_store(cmi, 0, own && kin, gx, gy, k, Dx, Dy, Dz, Bx, By, Bz);
    }
    // ---- step n+1 at plane k-1: B^{n+2}(k-1) from E^{n+1}(k-1) (sE2), E^{n+1}(k) (Ex..)
    const double Fx = b1x - C * (sE2[2][wp][lane] - f1z + f1y - Ey);
    const double Fy = b1y - C * (Ex - f1x + f1z - sE2[2][w][lp]);
    const double Fz = b1z - C * (sE2[1][w][lp] - f1y + f1x - sE2[0][wp][lane]);
    sH2[0][w][lane] = Fx, sH2[1][w][lane] = Fy, sH2[2][w][lane] = Fz;
    __syncthreads();
    const double Gx = d1x - C * (sH2[2][wm][lane] - Fz + Fy - h2y);
    const double Gy = d1y - C * (h2x - Fx + Fz - sH2[2][w][lm]);
    const double Gz = d1z - C * (sH2[1][w][lm] - Fy + Fx - sH2[0][wm][lane]);
    {
      const bool st = own && k - 1 >= zs && k - 1 < ze;
      const unsigned os = st ? col + (unsigned)(k - 1) * s2 : MNL_OOB;
      bst(brsrc_at(pBn0, nrec), os, Fx);
      bst(brsrc_at(pBn1, nrec), os, Fy);
      bst(brsrc_at(pBn2, nrec), os, Fz);
      bst(brsrc_at(pDn0, nrec), os, Gx);
      bst(brsrc_at(pDn1, nrec), os, Gy);
      bst(brsrc_at(pDn2, nrec), os, Gz);
      if (CMP && cmi >= 0) tb2_cmp_store(cmi, 1, st, gx, gy, k - 1, Gx, Gy, Gz, Fx, Fy, Fz);
    }
    h2x = Fx, h2y = Fy;
    h1x = Bx, h1y = By;
    b1x = Bx, b1y = By, b1z = Bz;
    d1x = Dx, d1y = Dy, d1z = Dz;
    f1x = Ex, f1y = Ey, f1z = Ez;
    enx = e1x, eny = e1y, enz = e1z;
    dnx = c.d0, dny = c.d1, dnz = c.d2;
    uk0 = v0, uk1 = v1, uk2 = v2;
  }
}

template <int UMODE, bool CLK, bool CMP>
__global__ __launch_bounds__(1024) void tb2_kernel1(TB2Args a) {
  __shared__ double sU[UMODE == 2 ? 3 : 1][256];
  __shared__ double sE1[3][TB_LY][TB_LX], sH1[3][TB_LY][TB_LX];
  __shared__ double sE2[3][TB_LY][TB_LX], sH2[3][TB_LY][TB_LX];
  __shared__ int s_idx;
  __shared__ unsigned long long s_t0;
  if (UMODE == 2) {  // palette -> LDS (visible after the first barrier below)
    for (int i = threadIdx.x; i < 3 * 256; i += 1024) sU[i >> 8][i & 255] = a.utab[i];
  }
  unsigned long long *ctr = a.ctr + 16 * a.ctr_line;
  if (CLK && threadIdx.x == 0) s_t0 = 0ull;  // no previous item
  for (;;) {
    if (threadIdx.x == 0) {
      if (CLK && s_t0 != 0ull) {  // diagnostics: the previous item (see fused_tile_kernel)
        const TB2Item it = a.items[s_idx];
        const unsigned uw = (UMODE == 2 && a.uflag) ? a.uflag[s_idx] : ~0u;
        clk_record(a.clk, s_t0, (it.faces & 63) | (uw != ~0u ? 64 : 0), it.x, it.y, it.z, -1);
      }
      const unsigned long long v = atomicAdd(ctr, 1ULL) - a.cbase;
      s_idx = v < (unsigned long long)(a.n) ? (int)v : -1;
      if (CLK) s_t0 = wall_clock64();
    }
    __syncthreads();  // also separates LDS use of consecutive items
    const int idx = s_idx;
    if (idx < 0) break;
    const TB2Item it = a.items[idx];
    const unsigned uw = (UMODE == 2 && a.uflag) ? a.uflag[idx] : ~0u;
    if (UMODE == 2 && __builtin_amdgcn_readfirstlane(uw) != ~0u)
      tb2_body1<UMODE, true, CMP>(a, it, uw, sU, sE1, sH1, sE2, sH2);
    else
      tb2_body1<UMODE, false, CMP>(a, it, uw, sU, sE1, sH1, sE2, sH2);
  }
}

// Per TB item: the palette word if every cell within distance 2 of its own box (the cells
// whose chi1inv the two steps use) has the same word, else ~0u.
__global__ void tb2_uniform_kernel(TB2Args a, unsigned *flags) {
  const int idx = blockIdx.x;
  const TB2Item it = a.items[idx];
  const int x0 = max((it.x & 0xFFFF) - 2, 0), x1 = min((it.x >> 16) + 2, a.N[0] - 1);
  const int y0 = max((it.y & 0xFFFF) - 2, 0), y1 = min((it.y >> 16) + 2, a.N[1] - 1);
  const int z0 = max((it.z & 0xFFFF) - 2, 0), z1 = min((it.z >> 16) + 1, a.N[2] - 1);
  __shared__ int bad;
  if (threadIdx.x == 0) bad = 0;
  __syncthreads();
  const long long nx = x1 - x0 + 1, ny = y1 - y0 + 1, nz = z1 - z0 + 1;
  const unsigned ref = a.uidx[x0 + (long long)y0 * a.st1 + (long long)z0 * a.st2];
  for (long long i = threadIdx.x; i < nx * ny * nz; i += blockDim.x) {
    const long long x = x0 + i % nx, y = y0 + (i / nx) % ny, z = z0 + i / (nx * ny);
    if (a.uidx[x + y * a.st1 + z * a.st2] != ref) bad = 1;
  }
  __syncthreads();
  if (threadIdx.x == 0) flags[idx] = bad ? ~0u : ref;
}

int k_tb2_uniform(const TB2Args &a, unsigned *flags, void *stream) {
  if (a.n <= 0 || !a.uidx) return 0;
  tb2_uniform_kernel<<<a.n, 256, 0, (hipStream_t)stream>>>(a, flags);
  return rc();
}

int k_tb2(const TB2Args &a, void *stream, unsigned long long *bases) {
  if (a.n <= 0) return 0;
  if (a.nelem * 8 >= (long long)MNL_OOB || !a.ctr || !a.items || a.ctr_line < 0 ||
      a.ctr_line >= FUSED_NCTR || (a.px != 1 && a.px != 2))
    return 2;
  long long nb = fused_grid_blocks(1);
  if (a.wg_limit > 0 && nb > a.wg_limit) nb = a.wg_limit;
  if (nb > a.n) nb = a.n;
  TB2Args t = a;
  t.cbase = bases[a.ctr_line];
  bases[a.ctr_line] += (unsigned long long)a.n + nb;
  const int um = a.uidx ? 2 : (a.u[0] ? 1 : 0);
  hipStream_t s = (hipStream_t)stream;
  const dim3 grd((unsigned)nb), blk(1024);
  // compact DFT boxes (t.ncmp > 0): the variant with their stores; the diagnostics build
  // (MNL_ITEM_CLOCK) always has them; px 1: the round-5 layout (A/B)
#define MNL_TB2_LAUNCH(K)                                   \
  do {                                                      \
    if (t.clk.rec) {                                        \
      if (um == 2)                                          \
        K<2, true, true><<<grd, blk, 0, s>>>(t);            \
      else if (um == 1)                                     \
        K<1, true, true><<<grd, blk, 0, s>>>(t);            \
      else                                                  \
        K<0, true, true><<<grd, blk, 0, s>>>(t);            \
    } else if (t.ncmp > 0) {                                \
      if (um == 2)                                          \
        K<2, false, true><<<grd, blk, 0, s>>>(t);           \
      else if (um == 1)                                     \
        K<1, false, true><<<grd, blk, 0, s>>>(t);           \
      else                                                  \
        K<0, false, true><<<grd, blk, 0, s>>>(t);           \
    } else if (um == 2) {                                   \
      K<2, false, false><<<grd, blk, 0, s>>>(t);            \
    } else if (um == 1) {                                   \
      K<1, false, false><<<grd, blk, 0, s>>>(t);            \
    } else {                                                \
      K<0, false, false><<<grd, blk, 0, s>>>(t);            \
    }                                                       \
  } while (0)
  if (t.px == 1)
    MNL_TB2_LAUNCH(tb2_kernel1);
  else
    MNL_TB2_LAUNCH(tb2_kernel);
#undef MNL_TB2_LAUNCH
  return hipPeekAtLastError() == hipSuccess ? 0 : 9;
}

// NaN guard (src/step.cpp:138-139): one thread sums the interpolation terms of the D energy
// density at the cell centre in the host's order (get_field: res += w * value) and flags a
// non-finite result; no host round trip (the host reads the flag once per batch).
__global__ void nan_check_kernel(NanTerms t, Ptr3 E, Ptr3 D, Ptr3 U, int *flag, int step) {
  // every term's value loaded by its own lane (one round trip), then summed by thread 0 in
  // the host's order from LDS
  __shared__ double sv[NAN_MAXT];
  const int i0 = threadIdx.x;
  if (i0 < t.n) {
    const int d = t.dir[i0];
    const long long k = t.idx[i0];
    double v;
    if (t.kind[i0] == 0)
      v = E.p[d][k];
    else if (t.kind[i0] == 1)
      v = U.ci[d] ? D.p[d][k] * U.ci[d][k] : D.p[d][k];
    else
      v = D.p[d][k];
    sv[i0] = v;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  double sum = 0.0;
  int i = 0;
  for (int d = 0; d < 3; d++) {
    double e = 0.0, dd = 0.0;
    for (; i < t.n && t.dir[i] == d && t.kind[i] != 2; i++) e += t.w[i] * sv[i];
    for (; i < t.n && t.dir[i] == d && t.kind[i] == 2; i++) dd += t.w[i] * sv[i];
    sum += e * dd;
  }
  if (!isfinite(sum * 0.5) && atomicOr(flag, 1) == 0) flag[1] = step;
}

// A pair's step tail in one launch (round 6): the D sources of the step, layer by layer (the
// same per-point expression as source_kernel; a barrier between layers keeps their list
// order), then the NaN guard of the state they complete (nan_check_kernel's sum, after a
// barrier: the guard reads the values with the sources in, as after the two launches).  One
// workgroup: only for short source lists (SRC_GUARD_MAXN points, SRC_GUARD_MAXL layers).
__global__ void __launch_bounds__(256) src_guard_kernel(Ptr3 pt, SrcDev s, SrcLayers sl,
                                                        NanTerms t, Ptr3 E, Ptr3 D, Ptr3 U,
                                                        int *flag, int step) {
  __shared__ double sv[NAN_MAXT];
  for (int l = 0; l < sl.n; l++) {
    for (int k = sl.off[l] + (int)threadIdx.x; k < sl.off[l + 1]; k += (int)blockDim.x) {
      const int c = s.comp[k];
      const long long i = s.idx[k];
      const int g = s.gid[k];
      const double ar = s.amp[2 * k], ai = s.amp[2 * k + 1];
      const double jr = s.J[2 * g], ji = s.J[2 * g + 1];
      const double v = (ar * jr - ai * ji) * s.dt;
      pt.p[c][i] -= pt.ci[c] ? v * pt.ci[c][i] : v;
    }
    __threadfence_block();
    __syncthreads();
  }
  if (t.n <= 0) return;
  const int i0 = threadIdx.x;
  if (i0 < t.n) {
    const int d = t.dir[i0];
    const long long k = t.idx[i0];
    double v;
    if (t.kind[i0] == 0)
      v = E.p[d][k];
    else if (t.kind[i0] == 1)
      v = U.ci[d] ? D.p[d][k] * U.ci[d][k] : D.p[d][k];
    else
      v = D.p[d][k];
    sv[i0] = v;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  double sum = 0.0;
  int i = 0;
  for (int d = 0; d < 3; d++) {
    double e = 0.0, dd = 0.0;
    for (; i < t.n && t.dir[i] == d && t.kind[i] != 2; i++) e += t.w[i] * sv[i];
    for (; i < t.n && t.dir[i] == d && t.kind[i] == 2; i++) dd += t.w[i] * sv[i];
    sum += e * dd;
  }
  if (!isfinite(sum * 0.5) && atomicOr(flag, 1) == 0) flag[1] = step;
}

int k_src_guard(const DevFields &f, const SrcDev &s, const NanTerms &t, const double *const E[3],
                const double *const D[3], const double *const U[3], int *flag, int step,
                void *stream) {
  if (s.n > SRC_GUARD_MAXN || s.nlayer > SRC_GUARD_MAXL || t.n > NAN_MAXT || t.n > 256) return 2;
  Ptr3 pt, e, d, u;
  for (int c = 0; c < 3; c++) {
    pt.p[c] = f.Dn[c], pt.ci[c] = f.cndinv[1][c];
    e.p[c] = const_cast<double *>(E[c]), e.ci[c] = nullptr;
    d.p[c] = const_cast<double *>(D[c]), d.ci[c] = nullptr;
    u.p[c] = nullptr, u.ci[c] = U[c];
  }
  SrcLayers sl{};
  sl.n = s.n > 0 ? s.nlayer : 0;
  for (int l = 0; l <= sl.n; l++) sl.off[l] = s.layer[l];
  src_guard_kernel<<<1, 256, 0, (hipStream_t)stream>>>(pt, s, sl, t, e, d, u, flag, step);
  return rc();
}

int k_nan_check(const NanTerms &t, const double *const E[3], const double *const D[3],
                const double *const U[3], int *flag, int step, void *stream) {
  if (t.n <= 0) return 0;
  Ptr3 e, d, u;
  for (int c = 0; c < 3; c++) {
    e.p[c] = const_cast<double *>(E[c]), e.ci[c] = nullptr;
    d.p[c] = const_cast<double *>(D[c]), d.ci[c] = nullptr;
    u.p[c] = nullptr, u.ci[c] = U[c];
  }
  nan_check_kernel<<<1, 64, 0, (hipStream_t)stream>>>(t, e, d, u, flag, step);
  return rc();
}

// Leaving fused mode (or reading out): over G, E = chi1inv * D where it is
// implicit, and the PML W aux fields get the values the reference holds
// (W_E = chi1inv * D, W_H = B: the last fw of update_eh).
__global__ void materialize_e_kernel(Box b, DevGrid g, DevFields f) {
  Pt p;
  if (!make_pt(b, g, p)) return;
  for (int c = 0; c < 3; c++) {
    const double d = f.D[c][p.idx];
    const double e = f.inveps[c] ? (d * f.inveps[c][p.idx]) : d;
    if (e_implicit(f, g, c, p)) f.E[c][p.idx] = e;
    if (f.WE[c] && owned(g, T_E, c, p) && pml_at(f, g, c, qcoord(g, p, T_E, c, c))) {
      // W_E = chi1inv * (D - P) of the last E update; P then was today's Pprev
      double gp = d;
      for (int k = 0; k < f.npol; k++)
        if (f.pol[k].P[c] && in_box(f.pol[k].nz, p)) gp = gp - f.pol[k].Pp[c][p.idx];
      f.WE[c][p.idx] = f.inveps[c] ? (gp * f.inveps[c][p.idx]) : gp;
    }
    if (f.WH[c] && owned(g, T_H, c, p) && pml_at(f, g, c, qcoord(g, p, T_H, c, c)))
      f.WH[c][p.idx] = f.B[c][p.idx];
  }
}

int k_materialize_e(const Box &F, const DevGrid &g, const DevFields &f, void *stream) {
  if (empty(F)) return 0;
  materialize_e_kernel<<<grid_for(F), dim3(MNL_BX, MNL_BY), 0, (hipStream_t)stream>>>(F, g, f);
  return rc();
}

// ----------------------------------------------------------------- DFT
// dft_chunk::update_dft (src/dft.cpp:265-300), split in two so that the DFT
// array is read and written once per KB updates instead of once per update:
//  * dft_sample_kernel (every DFT step): the field averaged from the Yee points
//    onto the cell centre exactly as the reference does,
//    (w*0.25)*(((f0 + f1) + f2) + f3) with the weight product precomputed on the
//    host, into slot u of a small per-point buffer (E read through the
//    implicit-E rule in fused mode);
//  * dft_accum_kernel (every KB updates, and at the end of every step batch):
//    dft += fr_u * phase_u for u = 0..n-1 in update order -- the reference's
//    sequential accumulation, same operations in the same order, in registers.
// The DFT array is blocked by wave, [slot/64][freq][slot%64] complex, so a
// wave's access to one frequency is one contiguous 1-KB span.
__global__ void dft_sample_kernel(const int *__restrict__ pj, const double *__restrict__ pw,
                                  const int *__restrict__ pch, const DftChunkDev *__restrict__ ch,
                                  double *__restrict__ fr_out, long long npts, DevGrid g,
                                  DevFields f) {
  const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npts) return;
  if (pj[3 * p] < 0) return;  // another rank's point
  const DftChunkDev cd = ch[pch[p]];
  const int c = cd.c, d = c % 3;
  const bool mag = c >= 3;
  Pt P;
  P.idx = 0;
  for (int e = 0; e < 3; e++) {
    P.j[e] = pj[3 * p + e];
    P.idx += (long long)P.j[e] * g.sdir[e];
  }
  auto val = [&](const Pt &q) -> double {
    if (mag) {
      const bool sep = f.H[d] && (f.hall || pml_at(f, g, d, qcoord(g, q, T_H, d, d)));
      return sep ? f.H[d][q.idx] : f.B[d][q.idx];
    }
    if (e_implicit(f, g, d, q)) {
      const double dv = f.D[d][q.idx];
      return f.inveps[d] ? dv * f.inveps[d][q.idx] : dv;
    }
    return f.E[d][q.idx];
  };
  auto nb = [&](const Pt &q, int e) {
    Pt r = q;
    r.j[e] += 1;
    r.idx += g.sdir[e];
    return r;
  };
  double fr;
  if (cd.avgmode == 2) {
    const Pt q1 = nb(P, cd.d1), q2 = nb(P, cd.d2), q3 = nb(q1, cd.d2);
    fr = pw[p] * (val(P) + val(q1) + val(q2) + val(q3));
  } else if (cd.avgmode == 1) {
    fr = pw[p] * (val(P) + val(nb(P, cd.d1)));
  } else {
    fr = pw[p] * val(P);
  }
  fr_out[p] = fr;
}

// Sampling plan (built once per fused-mode epoch): per point the linear index of the first
// of the 1-4 Yee values its centred average reads (the others are +d1, +d2, +d1+d2) and, per
// value, where it lives (0 stored E, 1 implicit E = D * chi1inv, 2 B (H == B), 3 separate H)
// -- the per-point table lookups of dft_sample_kernel (PML flags, ownership, fused box) done
// once, so that the per-step sample is one metadata load and independent value loads.
// sel: bits 0-1 component direction, 2-3 avgmode, 4 + 2v: kind of value v, 12-13 d1, 14-15
// d2; 0xFFFF: another rank's point.  The chi1inv of implicit-E values: as the palette bytes of
// the four values (spal, with uidx / utab: 4 B per point instead of 32) and as doubles (su,
// the fallback); *bad is set when a palette value is not bitwise the chi1inv array's.
__global__ void dft_plan_kernel(const int *__restrict__ pj, const int *__restrict__ pch,
                                const DftChunkDev *__restrict__ ch, long long npts, DevGrid g,
                                DevFields f, const unsigned *__restrict__ uidx,
                                const double *__restrict__ utab, int *__restrict__ sidx,
                                unsigned short *__restrict__ ssel, unsigned *__restrict__ spal,
                                double4 *__restrict__ su, int *__restrict__ bad, Box cb,
                                int *__restrict__ sci) {
  const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npts) return;
  if (pj[3 * p] < 0) {
    ssel[p] = 0xFFFF;
    sidx[p] = 0;
    spal[p] = 0;
    su[p] = make_double4(1.0, 1.0, 1.0, 1.0);
    if (sci) sci[p] = -1;
    return;
  }
  const DftChunkDev cd = ch[pch[p]];
  const int c = cd.c, d = c % 3;
  const bool mag = c >= 3;
  Pt P;
  P.idx = 0;
  for (int e = 0; e < 3; e++) {
    P.j[e] = pj[3 * p + e];
    P.idx += (long long)P.j[e] * g.sdir[e];
  }
  auto kind = [&](const Pt &q) -> unsigned {
    if (mag) return (f.H[d] && (f.hall || pml_at(f, g, d, qcoord(g, q, T_H, d, d)))) ? 3u : 2u;
    return e_implicit(f, g, d, q) ? 1u : 0u;
  };
  auto nb = [&](const Pt &q, int e) {
    Pt r = q;
    r.j[e] += 1;
    r.idx += g.sdir[e];
    return r;
  };
  Pt q[4] = {P, P, P, P};
  int nv = 1;
  if (cd.avgmode == 2) {
    q[1] = nb(P, cd.d1), q[2] = nb(P, cd.d2), q[3] = nb(q[1], cd.d2);
    nv = 4;
  } else if (cd.avgmode == 1) {
    q[1] = nb(P, cd.d1);
    nv = 2;
  }
  unsigned sel = (unsigned)d | ((unsigned)cd.avgmode << 2) |
                 ((unsigned)max(cd.d1, 0) << 12) | ((unsigned)max(cd.d2, 0) << 14);
  double uv[4] = {1.0, 1.0, 1.0, 1.0};  // chi1inv of implicit-E values (x * 1.0 == x otherwise)
  unsigned pal = 0;
  bool mism = false;
  for (int v = 0; v < nv; v++) {
    const unsigned k = kind(q[v]);
    sel |= k << (4 + 2 * v);
    if (k == 1 && f.inveps[d]) {
      uv[v] = f.inveps[d][q[v].idx];
      if (uidx) {
        const unsigned b = (uidx[q[v].idx] >> (8 * d)) & 255u;
        pal |= b << (8 * v);
        mism = mism || utab[d * 256 + b] != uv[v];
      }
    } else if (k == 1 && uidx) {  // chi1inv == 1: a palette entry equal to 1.0
      const unsigned b = (uidx[q[v].idx] >> (8 * d)) & 255u;
      pal |= b << (8 * v);
      mism = mism || utab[d * 256 + b] != 1.0;
    }
  }
  if (mism) atomicOr(bad, 1);
  if (sci) {  // compact-box index of the first value if every value lies in the box
    int c[3], n[3];
    bool in = true;
    for (int e = 0; e < 3; e++) {
      const int ax = g.ax[e] >= 0 ? g.ax[e] : e;
      c[ax] = P.j[e] - cb.lo[ax];
      const int top = c[ax] + ((nv > 1 && cd.d1 == e) || (nv > 2 && cd.d2 == e) ? 1 : 0);
      n[ax] = cb.hi[ax] - cb.lo[ax] + 1;
      in = in && g.ax[e] >= 0 && c[ax] >= 0 && top < n[ax];
    }
    sci[p] = in ? c[0] + n[0] * (c[1] + n[1] * c[2]) : -1;
  }
  ssel[p] = (unsigned short)sel;
  sidx[p] = (int)P.idx;
  spal[p] = pal;
  su[p] = make_double4(uv[0], uv[1], uv[2], uv[3]);
}

struct DftSrc {  // the current buffer set: E, D, B, H per direction
  const double *E[3], *D[3], *B[3], *H[3];
};

// implicit E = D * chi1inv with chi1inv from the plan (constant in time; 1.0 where none)
__device__ __forceinline__ double dft_val(const DftSrc &s, int d, unsigned k, int i, double u) {
  if (k == 0) return s.E[d][i];
  if (k == 1) return s.D[d][i] * u;
  return k == 2 ? s.B[d][i] : s.H[d][i];
}

// fields::update_dfts' sample of one update (src/dft.cpp:265-300): the reference's centred
// average (w * 0.25) * (((f0 + f1) + f2) + f3) through the plan, for every flux object due at
// this step in one launch (DftSampleJobs: the workgroups of job i are blk0[i] ..)
typedef const DftSampleJobs __attribute__((address_space(4))) KDJ;
__global__ void __launch_bounds__(256) dft_sample_jobs_kernel(DftSampleJobs J, DftSrc s,
                                                              const double *__restrict__ utab) {
  // XCD-aware block order: workgroups are dealt to the 8 XCDs round-robin (blockIdx % 8), so
  // each XCD takes one contiguous eighth of the points instead; the 2 x 2 averages of
  // neighbouring rows then meet their shared lines in that XCD's L2
  const unsigned nb = gridDim.x, xcd = blockIdx.x % 8u, q = nb / 8u, r = nb % 8u;
  const long long lb = xcd * q + min(xcd, r) + blockIdx.x / 8u;
  // the job table through the kernarg pointer (wave-uniform index: scalar loads, no copy)
  KDJ *jt = (KDJ *)__builtin_amdgcn_kernarg_segment_ptr();
  int ji = 0;
  for (int i = 1; i < jt->n; i++)
    if (lb >= jt->j[i].blk0) ji = i;
  const auto &jb = jt->j[ji];
  const long long p = (lb - jb.blk0) * 256 + threadIdx.x;
  if (p >= jb.npts) return;
  // the point's plan entries, loaded together (one round trip), then the values: compact-box
  // entries first (all in flight together), field-array loads only for the values the box
  // does not hold
  const unsigned sel = jb.ssel[p];
  const long long i0 = jb.sidx[p];
  const double w = jb.pw[p];
  const int ci = jb.cmp ? jb.sci[p] : -1;
  const unsigned pal = jb.usepal ? jb.spal[p] : 0u;
  if (sel == 0xFFFFu) return;  // another rank's point
  const int d = sel & 3, mode = (sel >> 2) & 3, d1 = (sel >> 12) & 3, d2 = (sel >> 14) & 3;
  const long long s1 = d1 == 0 ? J.sd[0] : (d1 == 1 ? J.sd[1] : J.sd[2]);
  const long long s2 = d2 == 0 ? J.sd[0] : (d2 == 1 ? J.sd[1] : J.sd[2]);
  const int nv = mode == 2 ? 4 : (mode == 1 ? 2 : 1);
  // chi1inv only for implicit-E values (kind 1 in any slot)
  const bool any1 = ((sel >> 4) & 0x55u & ~((sel >> 5) & 0x55u)) != 0;
  double u[4] = {1.0, 1.0, 1.0, 1.0};
  if (any1) {
    if (jb.usepal) {
#pragma unroll
      for (int v = 0; v < 4; v++)
        if (((sel >> (4 + 2 * v)) & 3) == 1) u[v] = utab[d * 256 + ((pal >> (8 * v)) & 255u)];
    } else {
      const double4 uu = ((const double4 *)jb.su)[p];
      u[0] = uu.x, u[1] = uu.y, u[2] = uu.z, u[3] = uu.w;
    }
  }
  const int c1 = d1 == 0 ? jb.cs[0] : (d1 == 1 ? jb.cs[1] : jb.cs[2]);
  const int c2 = d2 == 0 ? jb.cs[0] : (d2 == 1 ? jb.cs[1] : jb.cs[2]);
  const long long li[4] = {i0, i0 + s1, i0 + s2, i0 + s1 + s2};
  const int cix[4] = {ci, ci + c1, ci + c2, ci + c1 + c2};
  double val[4];
  bool got[4];
#pragma unroll
  for (int v = 0; v < 4; v++) {  // two-step points from the compact box of this state (dense)
    const unsigned k = (sel >> (4 + 2 * v)) & 3;
    const bool use = v < nv && ci >= 0 && (k == 1 || k == 2);
    val[v] = use ? jb.cmp[(size_t)((k == 1 ? d : 3 + d) * jb.ncell) + cix[v]] : 0.0;
    got[v] = use;
  }
#pragma unroll
  for (int v = 0; v < 4; v++) {  // the others (and entries no two-step point wrote)
    const unsigned k = (sel >> (4 + 2 * v)) & 3;
    if (v >= nv) continue;
    if (got[v] && (unsigned long long)__double_as_longlong(val[v]) != DFT_CMP_EMPTY)
      val[v] = k == 1 ? val[v] * u[v] : val[v];
    else
      val[v] = dft_val(s, d, k, (int)li[v], u[v]);
  }
  double fr;
  if (mode == 2) {
    fr = w * (val[0] + val[1] + val[2] + val[3]);
  } else if (mode == 1) {
    fr = w * (val[0] + val[1]);
  } else {
    fr = w * val[0];
  }
  jb.fr[p] = fr;
}

int k_dft_plan(const int *pj, const int *pch, const DftChunkDev *ch, long long npts,
               const DevGrid &g, const DevFields &f, const unsigned *uidx, const double *utab,
               int *sidx, unsigned short *ssel, unsigned *spal, void *su, int *bad,
               const Box &cbox, int *sci, void *stream) {
  if (npts <= 0) return 0;
  dft_plan_kernel<<<(unsigned)((npts + 255) / 256), 256, 0, (hipStream_t)stream>>>(
      pj, pch, ch, npts, g, f, uidx, utab, sidx, ssel, spal, (double4 *)su, bad, cbox, sci);
  return rc();
}

int k_dft_sample_jobs(const DftSampleJobs &J, const DevGrid &g, const DevFields &f,
                      const double *utab, void *stream) {
  if (J.n <= 0 || J.n > DFT_MAXJ || J.nblk <= 0) return 0;
  if (J.j[0].blk0 != 0) return 2;
  DftSampleJobs t = J;
  for (int d = 0; d < 3; d++) t.sd[d] = g.sdir[d];
  DftSrc s;
  for (int d = 0; d < 3; d++) s.E[d] = f.E[d], s.D[d] = f.D[d], s.B[d] = f.B[d], s.H[d] = f.H[d];
  dft_sample_jobs_kernel<<<(unsigned)J.nblk, 256, 0, (hipStream_t)stream>>>(t, s, utab);
  return rc();
}

// Accumulation: one thread per point; a tile of DFT_FT frequencies is loaded
// into registers at once (DFT_FT independent loads in flight), every buffered
// update is added in order, and the tile is stored back.  When the whole wave
// belongs to one chunk (the usual case: slots are sorted by component and
// position) the phases are wave-uniform and come through scalar loads.
// one tile of FT frequencies at i0: FT independent loads in flight, every
// buffered update added in order, FT stores
template <int FT>
__device__ __forceinline__ void dft_accum_tile(double2 *__restrict__ dp,
                                               const double2 *__restrict__ php,
                                               const double *frv, int n, long long rstride,
                                               int i0) {
  double2 v[FT];
#pragma unroll
  for (int w = 0; w < FT; w++) v[w] = dp[(i0 + w) * 64];
#pragma unroll
  for (int u = 0; u < DFT_KB; u++) {
    if (u < n) {
#pragma unroll
      for (int w = 0; w < FT; w++) {
        const double2 q = php[u * rstride + i0 + w];
        v[w].x = v[w].x + frv[u] * q.x;
        v[w].y = v[w].y + frv[u] * q.y;
      }
    }
  }
#pragma unroll
  for (int w = 0; w < FT; w++) dp[(i0 + w) * 64] = v[w];
}

// tiles of DFT_FT frequencies, then the remainder in tiles of 8, 4, 2, 1
__device__ __forceinline__ void dft_accum_point(double2 *__restrict__ dp,
                                                const double2 *__restrict__ php,
                                                const double *frv, int n, long long rstride,
                                                int nfreq) {
  int i0 = 0;
  for (; i0 + DFT_FT <= nfreq; i0 += DFT_FT) dft_accum_tile<DFT_FT>(dp, php, frv, n, rstride, i0);
  if (nfreq - i0 >= 8) dft_accum_tile<8>(dp, php, frv, n, rstride, i0), i0 += 8;
  if (nfreq - i0 >= 4) dft_accum_tile<4>(dp, php, frv, n, rstride, i0), i0 += 4;
  if (nfreq - i0 >= 2) dft_accum_tile<2>(dp, php, frv, n, rstride, i0), i0 += 2;
  if (nfreq - i0 >= 1) dft_accum_tile<1>(dp, php, frv, n, rstride, i0);
}

// one tile of FT frequencies at i0 with the phases of the block's chunk staged in LDS
// (sph[u][DFT_FT], tile-relative column woff + w): broadcast LDS reads instead of a dependent
// global / scalar load per phase
template <int FT>
__device__ __forceinline__ void dft_accum_tile_lds(double2 *__restrict__ dp, const double2 *sph,
                                                   const double *frv, int n, int i0, int woff) {
  double2 v[FT];
#pragma unroll
  for (int w = 0; w < FT; w++) v[w] = dp[(i0 + woff + w) * 64];
#pragma unroll
  for (int u = 0; u < DFT_KB; u++) {
    if (u < n) {
#pragma unroll
      for (int w = 0; w < FT; w++) {
        const double2 q = sph[u * DFT_FT + woff + w];
        v[w].x = v[w].x + frv[u] * q.x;
        v[w].y = v[w].y + frv[u] * q.y;
      }
    }
  }
#pragma unroll
  for (int w = 0; w < FT; w++) dp[(i0 + woff + w) * 64] = v[w];
}

__global__ void __launch_bounds__(256)
    dft_accum_kernel(const int *__restrict__ pj, const int *__restrict__ pch,
                     double2 *__restrict__ dft, const double *__restrict__ fr, int n,
                     const double2 *__restrict__ ph, long long rstride, int nfreq,
                     long long npts) {
  __shared__ double2 sph[DFT_KB * DFT_FT];
  const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = p < npts && pj[3 * p] >= 0;
  const int k = pch[p < npts ? p : npts - 1];
  const int kb = pch[(long long)blockIdx.x * blockDim.x];
  const bool uni = __syncthreads_and(k == kb);  // one chunk (one phase row) for the block
  double frv[DFT_KB];
#pragma unroll
  for (int u = 0; u < DFT_KB; u++) frv[u] = (live && u < n) ? fr[u * npts + p] : 0.0;
  double2 *__restrict__ dp = dft + (p >> 6) * nfreq * 64 + (p & 63);
  if (!uni) {
    if (live) dft_accum_point(dp, ph + (long long)k * nfreq, frv, n, rstride, nfreq);
    return;
  }
  const double2 *php = ph + (long long)kb * nfreq;
  for (int i0 = 0; i0 < nfreq; i0 += DFT_FT) {  // block-uniform loop
    const int ft = min(DFT_FT, nfreq - i0);
    __syncthreads();  // the previous tile's readers are done
    for (int e = threadIdx.x; e < n * DFT_FT; e += blockDim.x) {
      const int u = e / DFT_FT, w = e % DFT_FT;
      if (w < ft) sph[e] = php[u * rstride + i0 + w];
    }
    __syncthreads();
    if (!live) continue;
    if (ft == DFT_FT) {
      dft_accum_tile_lds<DFT_FT>(dp, sph, frv, n, i0, 0);
    } else {  // the last, partial tile in pieces of 8, 4, 2, 1
      int w0 = 0;
      if (ft - w0 >= 8) dft_accum_tile_lds<8>(dp, sph, frv, n, i0, w0), w0 += 8;
      if (ft - w0 >= 4) dft_accum_tile_lds<4>(dp, sph, frv, n, i0, w0), w0 += 4;
      if (ft - w0 >= 2) dft_accum_tile_lds<2>(dp, sph, frv, n, i0, w0), w0 += 2;
      if (ft - w0 >= 1) dft_accum_tile_lds<1>(dp, sph, frv, n, i0, w0);
    }
  }
}

int k_dft_sample(const int *pj, const double *pw, const int *pch, const DftChunkDev *ch, double *fr,
                 long long npts, const DevGrid &g, const DevFields &f, void *stream) {
  if (npts <= 0) return 0;
  dft_sample_kernel<<<(unsigned)((npts + 255) / 256), 256, 0, (hipStream_t)stream>>>(
      pj, pw, pch, ch, fr, npts, g, f);
  return rc();
}

int k_dft_accum(const int *pj, const int *pch, double *dft, const double *fr, int n,
                const double *ph, long long rstride, int nfreq, long long npts, void *stream) {
  if (npts <= 0 || n <= 0) return 0;
  if (n > DFT_KB || nfreq < 1) return 2;
  dft_accum_kernel<<<(unsigned)((npts + 255) / 256), 256, 0, (hipStream_t)stream>>>(
      pj, pch, (double2 *)dft, fr, n, (const double2 *)ph, rstride, nfreq, npts);
  return rc();
}

int k_fill(double *p, double v, size_t n, void *stream) {
  if (n == 0) return 0;
  size_t blocks = (n + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  fill_kernel<<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(p, v, n);
  return rc();
}

static void canon_strides(const DevGrid &g, long long cs[3]) {
  // canonical whole-cell layout: Z fastest, then Y, then X (src/vec.cpp:482-494)
  long long nz = g.ax[2] >= 0 ? g.nglob[2] + 1 : 1;
  long long ny = g.ax[1] >= 0 ? g.nglob[1] + 1 : 1;
  cs[2] = g.ax[2] >= 0 ? 1 : 0;
  cs[1] = g.ax[1] >= 0 ? nz : 0;
  cs[0] = g.ax[0] >= 0 ? nz * ny : 0;
}

int k_from_canonical(double *dst, const double *src, const DevGrid &g, int comp_type, int comp_dir,
                     int zlo_glob, void *stream) {
  (void)comp_type;
  (void)comp_dir;
  (void)zlo_glob;
  long long cs[3];
  canon_strides(g, cs);
  dim3 grd((g.N[0] + MNL_BX - 1) / MNL_BX, (g.N[1] + MNL_BY - 1) / MNL_BY, g.N[2]);
  from_canonical_kernel<<<grd, dim3(MNL_BX, MNL_BY), 0, (hipStream_t)stream>>>(dst, src, g, cs[0],
                                                                               cs[1], cs[2]);
  return rc();
}

// fields::initialize_field (src/initialize.cpp:135-161): every point of the
// rank's array (ghost planes included: LOOP_OVER_VOL covers each chunk's whole
// array) gets += v; then zero_metal (src/boundaries.cpp:304-339) zeroes the owned
// points on the metallic high wall of each unshifted direction.  alt != null (H
// after its lazy allocation): the H array holds the value only where H is
// separate (PML chunk along c, src/update_eh.cpp:204-209), elsewhere H == B.
__global__ void init_add_kernel(double *dst, double *alt, const double *src, DevGrid g,
                                DevFields f, int type, int c, long long cs0, long long cs1,
                                long long cs2) {
  int i0 = blockIdx.x * MNL_BX + threadIdx.x;
  int i1 = blockIdx.y * MNL_BY + threadIdx.y;
  int i2 = blockIdx.z;
  if (i0 >= g.N[0] || i1 >= g.N[1]) return;
  int ii[3] = {i0, i1, i2};
  Pt p;
  long long cidx = 0;
  const long long cs[3] = {cs0, cs1, cs2};
  bool wall = false;
  for (int d = 0; d < 3; d++) {
    p.j[d] = g.ax[d] >= 0 ? ii[g.ax[d]] : 0;
    if (g.ax[d] < 0) continue;
    cidx += (long long)(p.j[d] + g.off[d]) * cs[d];
    if (!shift_of(type, c, d) && p.j[d] + g.off[d] == g.nglob[d]) wall = true;
  }
  double *t = dst;
  bool sep = pml_at(f, g, c, qcoord(g, p, type, c, c));
  if (f.hall && alt && !sep) {  // H-side materials: H separate in this point's chunk?
    int rz = 0;
    for (int e = 0; e < 3; e++) rz = rz * 3 + (g.ax[e] >= 0 ? f.zone[e][qcoord(g, p, type, c, e)] : 1);
    sep = f.hsep_all || ((f.hsep_zone[rz] >> c) & 1);
  }
  if (alt && !sep) t = alt;
  const long long li = (long long)i0 + i1 * g.st[1] + i2 * g.st[2];
  const double v = wall ? 0.0 : t[li] + src[cidx];
  t[li] = v;
  if (f.hall && alt && !sep) dst[li] = v;  // the H copy of an aliasing chunk follows B
}

// ------------------------------------------------------------- energy
// fields::field_energy_in_box(c, where) (src/energy_and_flux.cpp:67-83) ->
// integrate(2, {Ec, Dc} or {Hc, Bc}) on c's own Yee grid (src/integrate.cpp:
// 46-129): per point fv = 0.25 * (((f + f) + f) + f) of each field (offsets 0
// on a component grid), term = (fv0 * fv1) * IVEC_LOOP_WEIGHT.  One launch per
// reference chunk box; every thread accumulates its terms with TwoSum
// compensation, the workgroup combines (s, c) pairs in LDS and writes one pair.
__device__ __forceinline__ void two_sum(double a, double b, double &s, double &e) {
  s = a + b;
  const double bb = s - a;
  e = (a - (s - bb)) + (b - bb);
}

__global__ __launch_bounds__(256) void energy_kernel(const double *A, const double *Asep,
                                                     const double *Bv, DevGrid g, DevFields f,
                                                     int type, int c, EBox box, const double *wt,
                                                     double *partial) {
  __shared__ double ls[256], lc[256];
  const long long n0 = box.dn[0], n1 = box.dn[1], n2 = box.dn[2];
  const long long ntot = n0 * n1 * n2;
  double s = 0.0, comp = 0.0;
  for (long long q = (long long)blockIdx.x * 256 + threadIdx.x; q < ntot;
       q += (long long)gridDim.x * 256) {
    const long long a0 = q % n0, r = q / n0, a1 = r % n1, a2 = r / n1;
    const long long ia[3] = {a0, a1, a2};
    Pt p;
    long long li = 0;
    double w[3];
    for (int d = 0; d < 3; d++) {
      const int ax = g.ax[d];
      w[d] = 1.0;
      p.j[d] = 0;
      if (ax < 0) continue;
      p.j[d] = box.dlo[ax] + (int)ia[ax];
      li += (long long)p.j[d] * g.st[ax];
      w[d] = wt[box.wofs[ax] + ia[ax]];
    }
    // IVEC_LOOP_WEIGHT order: W(yd[2]) * (W(yd[1]) * (dV * W(yd[0])))
    const double wgt = w[box.yd[2]] * (w[box.yd[1]] * (box.dV0 * w[box.yd[0]]));
    const double *src = A;
    if (Asep && (f.hall || pml_at(f, g, c, qcoord(g, p, type, c, c)))) src = Asep;  // H separate here
    const double x = src[li], y = Bv[li];
    const double xv = 0.25 * (((x + x) + x) + x), yv = 0.25 * (((y + y) + y) + y);
    const double t = (xv * yv) * wgt;
    double ns, e;
    two_sum(s, t, ns, e);
    s = ns;
    comp += e;
  }
  ls[threadIdx.x] = s;
  lc[threadIdx.x] = comp;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if ((int)threadIdx.x < k) {
      double ns, e;
      two_sum(ls[threadIdx.x], ls[threadIdx.x + k], ns, e);
      ls[threadIdx.x] = ns;
      lc[threadIdx.x] = lc[threadIdx.x] + lc[threadIdx.x + k] + e;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    partial[2 * blockIdx.x] = ls[0];
    partial[2 * blockIdx.x + 1] = lc[0];
  }
}

int k_energy(const double *A, const double *Asep, const double *Bv, const DevGrid &g,
             const DevFields &f, int type, int c, const EBox &box, const double *wt,
             double *partial, int nblocks, void *stream) {
  energy_kernel<<<nblocks, 256, 0, (hipStream_t)stream>>>(A, Asep, Bv, g, f, type, c, box, wt,
                                                          partial);
  return rc();
}

// average_with_backup (src/energy_and_flux.cpp:136-144): f = 0.5 * (f + backup)
__global__ void average_kernel(double *f, const double *bk, long long n) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) f[i] = 0.5 * (f[i] + bk[i]);
}

int k_average(double *f, const double *bk, long long n, void *stream) {
  if (n <= 0) return 0;
  average_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(f, bk, n);
  return rc();
}

// lazy allocation on the first update_eh (src/update_eh.cpp:204-216): H starts
// as a copy of B, and the W auxiliary field as a copy of the field it shadows
__global__ void copy_kernel(double *dst, const double *src, long long n) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

int k_copy(double *dst, const double *src, long long n, void *stream) {
  if (n <= 0) return 0;
  copy_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(dst, src, n);
  return rc();
}

int k_init_add(double *dst, double *alt, const double *src, const DevGrid &g, const DevFields &f,
               int comp_type, int comp_dir, void *stream) {
  long long cs[3];
  canon_strides(g, cs);
  dim3 grd((g.N[0] + MNL_BX - 1) / MNL_BX, (g.N[1] + MNL_BY - 1) / MNL_BY, g.N[2]);
  init_add_kernel<<<grd, dim3(MNL_BX, MNL_BY), 0, (hipStream_t)stream>>>(
      dst, alt, src, g, f, comp_type, comp_dir, cs[0], cs[1], cs[2]);
  return rc();
}

int k_to_box(double *dst, const double *src, const double *hsep, const DevGrid &g, int comp_type,
             int comp_dir, const DevFields &f, const Box *fusedF, const double *dsrc,
             const double *usrc, const int blo[3], const int bhi[3], const long long bs[3],
             void *stream) {
  (void)fusedF;
  int l[3] = {0, 0, 0}, n[3] = {1, 1, 1};
  for (int d = 0; d < 3; d++) {
    const int a = g.ax[d];
    if (a < 0) continue;
    const int lo = std::max(blo[d] - g.off[d], 0), hi = std::min(bhi[d] - g.off[d], g.N[a] - 1);
    if (hi < lo) return 0;
    l[a] = lo;
    n[a] = hi - lo + 1;
  }
  int bl[3] = {0, 0, 0};
  long long bst[3] = {0, 0, 0};
  for (int d = 0; d < 3; d++)
    if (g.ax[d] >= 0) bl[d] = blo[d], bst[d] = bs[d];
  dim3 grd((n[0] + MNL_BX - 1) / MNL_BX, (n[1] + MNL_BY - 1) / MNL_BY, n[2]);
  to_box_kernel<<<grd, dim3(MNL_BX, MNL_BY), 0, (hipStream_t)stream>>>(
      dst, src, hsep, g, f, comp_type, comp_dir, l[0], l[1], l[2], n[0], n[1], bst[0], bst[1],
      bst[2], bl[0], bl[1], bl[2], fusedF ? 1 : 0, dsrc, usrc);
  return rc();
}

int k_to_canonical(double *dst, const double *src, const double *hsep, const DevGrid &g,
                   int comp_type, int comp_dir, const DevFields &f, const Box *fusedF,
                   const double *dsrc, const double *usrc, void *stream) {
  long long cs[3];
  canon_strides(g, cs);
  int blo[3] = {0, 0, 0}, bhi[3] = {0, 0, 0};
  for (int d = 0; d < 3; d++)
    if (g.ax[d] >= 0) bhi[d] = g.nglob[d];
  return k_to_box(dst, src, hsep, g, comp_type, comp_dir, f, fusedF, dsrc, usrc, blo, bhi, cs,
                  stream);
}

__global__ void nonzero_box_kernel(const double *a0, const double *a1, const double *a2,
                                   DevGrid g, int *box) {
  int i0 = blockIdx.x * MNL_BX + threadIdx.x;
  int i1 = blockIdx.y * MNL_BY + threadIdx.y;
  int i2 = blockIdx.z;
  if (i0 >= g.N[0] || i1 >= g.N[1]) return;
  const long long i = (long long)i0 + i1 * g.st[1] + i2 * g.st[2];
  const bool nz = (a0 && a0[i] != 0.0) || (a1 && a1[i] != 0.0) || (a2 && a2[i] != 0.0);
  if (!nz) return;
  const int ii[3] = {i0, i1, i2};
  for (int d = 0; d < 3; d++) {  // per direction, like Pt::j
    const int j = g.ax[d] >= 0 ? ii[g.ax[d]] : 0;
    atomicMin(box + d, j);
    atomicMax(box + 3 + d, j);
  }
}

int k_nonzero_box(const double *const a[3], const DevGrid &g, int *box, void *stream) {
  dim3 grd((g.N[0] + MNL_BX - 1) / MNL_BX, (g.N[1] + MNL_BY - 1) / MNL_BY, g.N[2]);
  nonzero_box_kernel<<<grd, dim3(MNL_BX, MNL_BY), 0, (hipStream_t)stream>>>(a[0], a[1], a[2], g,
                                                                           box);
  return rc();
}

int k_avg_chi1inv(const AvgArgs &a, void *stream) {
  if (a.ntot <= 0) return 0;
  avg_chi1inv_kernel<<<(unsigned)((a.ntot + 255) / 256), 256, 0, (hipStream_t)stream>>>(a);
  return rc();
}

int k_box_fill(double *dst, const DevGrid &g, int comp_type, int comp_dir, const double *lo,
               const double *hi, double value, int invert, double a, const int *io, void *stream) {
  dim3 grd((g.N[0] + MNL_BX - 1) / MNL_BX, (g.N[1] + MNL_BY - 1) / MNL_BY, g.N[2]);
  box_fill_kernel<<<grd, dim3(MNL_BX, MNL_BY), 0, (hipStream_t)stream>>>(
      dst, g, comp_type, comp_dir, lo[0], hi[0], lo[1], hi[1], lo[2], hi[2], value, invert, a,
      io[0], io[1], io[2]);
  return rc();
}

}  // namespace mnl
