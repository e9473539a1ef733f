// mnl_internal.hpp -- plain-data structures shared by the host orchestration
// (mnl_host.cpp, built with g++) and the HIP kernels (mnl_kernels.hip, built
// with hipcc for gfx950).  No HIP types appear here so both compilers agree
// on the layout.
//
// Data layout in HBM (DESIGN.md "Layout"): one structure-of-arrays fp64
// buffer per field component over the rank-local index box
// [0,N0) x [0,N1) x [0,N2), device axis 0 fastest.  Axis k is the k-th present
// direction in X,Y,Z order, so in 3-D X is contiguous and Z is the slab /
// plane axis (a ghost plane is one contiguous block for the halo exchange).
// Axis-0 rows are padded to a multiple of 16 doubles (128 B lines).
#pragma once
#include <cstddef>
#include <cstdint>

namespace mnl {

constexpr int MAX_POL = 4;    // Lorentzian susceptibilities per structure
constexpr int MAX_HPOL = 2;   // magnetic (H_stuff) Lorentzian susceptibilities
constexpr int MAX_BOX = 7;    // interior + 6 shell boxes

enum { T_E = 0, T_H = 1, T_D = 2, T_B = 3 };

struct Box {
  int lo[3];  // inclusive local index bounds per device axis
  int hi[3];
};

// Shell boxes of one sub-step, launched together: thread t belongs to box b
// with start[b] <= t < start[b+1] and is unravelled axis-0 fastest inside it.
struct BoxList {
  int n;
  Box b[MAX_BOX - 1];
  long long start[MAX_BOX];
};

struct DevGrid {
  int dim;
  int ax[3];            // device axis of direction X,Y,Z (-1 = absent)
  int N[3];             // local points per device axis
  long long st[3];      // strides per device axis (st[0] = 1)
  long long sdir[3];    // stride per direction X,Y,Z (0 if absent)
  int off[3];           // global index of local index 0, per direction
  int nglob[3];         // global cells per direction
  int wall[3];          // 1: metallic wall plane (global index n) excluded from updates
  int owned_lo_sh[3];   // per direction: local owned range of shifted components
  int owned_hi_sh[3];
  int owned_lo_un[3];   // ... of unshifted components (wall excluded)
  int owned_hi_un[3];
};

// Which neighbours enter each curl update (src/fields.cpp:438-471 plan with
// the NULL-pointer swap of step_curl, src/step_generic.cpp:76-80).
// terms: bit0 = g1 term (comp (d+2)%3 along dir (d+1)%3), bit1 = g2 term
// (comp (d+1)%3 along dir (d+2)%3).  present = component allocated.
struct CurlPlan {
  int present[3];
  int terms[3];
};

struct PmlDev {
  const uint8_t *flag[3];  // per direction, indexed by global half-coordinate q
  const double *sig[3];
  const double *kap[3];
  const double *siginv[3];
};

struct PolDev {
  double gamma1inv, gamma1, omega0dtsqr, omega0dtsqr_denom;
  double *P[3];
  double *Pp[3];
  const double *sigma[3];
  // anisotropic sigma (src/susceptibility.cpp:227-250): off-diagonal sigma[c][d]
  // (null = zero everywhere) and, per zone box, which arrays the reference
  // chunk holds: bit 3c+d (d != c: off-diagonal nontrivial there; d == c: the
  // diagonal array kept, i.e. some entry of row c nontrivial there)
  const double *soff[3][3];
  const uint16_t *zbits;
  // box (local indices per direction) holding every point with sigma != 0; outside
  // it P and Pprev stay 0 (update_P with sigma = 0 from 0), so the E update
  // neither reads nor writes them there
  Box nz;
};

struct DevFields {
  // B, D: field at the start of the step (read); Bn, Dn: where the update
  // writes.  Unfused stepping updates in place (Bn == B, Dn == D); the fused
  // interior kernel ping-pongs them and the host swaps after each step.
  double *E[3], *D[3], *B[3], *H[3];
  double *Bn[3], *Dn[3];
  // fused mode also ping-pongs stored E, separate H and the f_u of B (the
  // fused kernel recomputes halo points from their old values); unfused: == E, H, UB
  double *En[3], *Hn[3], *UBn[3];
  double *UB[3], *UD[3], *WE[3], *WH[3];
  const double *inveps[3];   // diagonal chi1inv of E comps (null = trivial)
  const double *offd[3][2];  // chi1inv[ec][cycle(d,1)], [cycle(d,2)] (null = absent)
  const double *chi2[3];
  const double *chi3[3];     // upstream nonlinear mode only (the fork's chi3 is inert)
  int upnl;                  // 1: upstream chi2/chi3 Pade update of E (calc_nonlinear_u)
  int wall_e;                // 1: E / P also on the high metallic wall planes (see update_e_kernel)
  int npol;
  PolDev pol[MAX_POL];       // in reference pol-list order (reverse of add order)
  PmlDev pml;
  int ecomp_present[3];
  int hcomp_present[3];
  int nr_enabled;
  // per zone box (3x3x3 over X,Y,Z zones lo/mid/hi): bit (3*c + k) set if
  // chi1inv[Ec][cycle(c,k+1)] is allocated (non-trivial) in that chunk.
  const uint8_t *offd_zone;
  const uint8_t *zone[3];    // per direction, global half-coordinate q -> zone 0/1/2
  unsigned long long *nr_fallbacks;
  long long nr_t;            // time step of the E update (seeds of the NR random fallback)
  // Newton-Raphson problems whose first attempt failed, deferred to nr_hard_kernel
  // (the later attempts run in parallel, one per lane); null: solve in place
  struct NRHard *nr_hard;
  unsigned *nr_hard_cnt;
  int nr_hard_cap;
  // fused mode active: inside box fG, E is implicit (chi1inv * D, not stored)
  // wherever it is owned and not in a PML chunk along its own direction
  int fused;
  Box fG;
  // conductivity (structure_chunk::conductivity/condinv of the D and B
  // components, src/structure.cpp:693-707, 868-905), [0] = B, [1] = D; null =
  // zero everywhere.  fcnd: f_cond, the auxiliary field of PML chunks along
  // dsig with conductivity (src/step_db.cpp:67-70).  cnd_zone: per zone box,
  // bit 3*t+d set if conductivity[t][d] is allocated in that chunk.
  const double *cnd[2][3];
  const double *cndinv[2][3];
  double *fcnd[2][3];
  const uint8_t *cnd_zone;
  double cnd_dt2;            // dt * 0.5 (src/step_generic.cpp:92)
  int aniso;                 // some susceptibility has off-diagonal sigma
  // H-side materials (mu != 1, magnetic Lorentzian).  hall = 1:
  // H is stored at every point (update_hmat_kernel), a copy of B where the point's
  // reference chunk aliases H to B (src/update_eh.cpp:204-209), and every reader of H
  // reads that array.  hsep_zone: per zone box, bit d set if H_d is separate in that
  // chunk for a reason other than PML along d (chi1inv[H_d] row kept, or f_minus_p of
  // B allocated because a magnetic susceptibility needs P).
  int hall;
  const double *invmu[3];    // diagonal chi1inv of H comps (null = trivial)
  const uint8_t *hsep_zone;
  int hsep_all;              // some magnetic susceptibility needs P: f_minus_p of B in every
                             // chunk, so H is separate everywhere
  int nhpol;
  PolDev hpol[MAX_HPOL];     // magnetic pol list (reverse of add order), isotropic sigma
};

// One reference chunk's integration box on a component grid (field energy):
// device-axis start / count on this rank, per-axis weight-table offsets, the
// yucky direction order of IVEC_LOOP_WEIGHT, and dV0.
struct EBox {
  int dlo[3];
  int dn[3];
  long long wofs[3];
  int yd[3];
  double dV0;
};

// Point sources in rank-local linear indices.
// Current sources (step_source, src/step.cpp:296-319) of one field type: per
// point its rank-local index, direction, complex amplitude and src_vol group;
// per step and group the src_time current (host, calc_sources).  The list is
// split into layers in which every (comp, idx) occurs once, so a layer is
// applied in parallel and the layers in list order (sequential semantics
// where sources overlap).
struct SrcDev {
  int n;
  const long long *idx;
  const int *comp;          // direction 0..2 of the D/B component
  const double *amp;        // [2 n] amplitude (re, im)
  const int *gid;           // [n] group (src_vol) index into the current table
  const double *J;          // [2 ngroups] this step's current of every group
  double dt;
  int nlayer;
  const int *layer;         // host array: layer start offsets [nlayer + 1]
};

struct ISrcDev {             // integrated sources, read by the E kernel
  int n;
  // entries sorted by local index (stable: one point's entries stay in list
  // order), each with its component, owning reference chunk (zone box
  // zx*9+zy*3+zz: only that chunk's f_minus_p has the dipole subtracted,
  // src/update_eh.cpp:136-146; another chunk reading it as a ghost sees D - P
  // only) and its position in the per-step value table
  const long long *idx;
  const int *comp;
  const unsigned char *zone;
  const int *orig;
  long long imin, imax;      // index range of the entries
  const double *val;         // [step][n] dipole value real(amp*dipole(t+dt))
};

// One DFT chunk (dft_chunk, src/dft.cpp:51-128) as the update kernel sees it:
// component, how many Yee points are averaged onto the cell centre and along
// which directions (grid_volume::yee2cent_offsets, src/vec.cpp:333-344).
struct DftChunkDev {
  int c;        // MNL component (E or H)
  int avgmode;  // 0, 1 (d1) or 2 (d1, d2)
  int d1, d2;
};

// Host-side launchers implemented in mnl_kernels.hip.
struct Launch {
  void *stream;  // hipStream_t
};

// interior: one box on a 3-D grid; shell: all shell boxes in one launch
// fuseup (shell only): apply the per-point H (after B) / E (after D) update in
// the same kernel (no B sources; no NR, susceptibilities, integrated sources
// or D sources in the shell)
int k_curl(int ft, const Box &in, const BoxList *shell, const DevGrid &g, const DevFields &f,
           const CurlPlan &p, double courant, void *stream, bool fuseup = false);
int k_update_h(const BoxList &shell, const DevGrid &g, const DevFields &f, void *stream);
// update_eh(H_stuff) [+ update_pols(H_stuff) if pols] over box b when H is stored
// everywhere (f.hall)
int k_update_hmat(const Box &b, const DevGrid &g, const DevFields &f, int pols, void *stream);
int k_update_e(const Box &in, const BoxList *shell, const DevGrid &g, const DevFields &f,
               const ISrcDev &is, int step, bool fuse_pols, void *stream);
int k_update_pols(const Box &in, const BoxList *shell, const DevGrid &g, const DevFields &f,
                  void *stream);
int k_aniso_wall(const DevGrid &g, const DevFields &f, int zero, void *stream);
// a pair's step tail in one workgroup: D sources (f.Dn; short lists only) then the NaN guard
constexpr int SRC_GUARD_MAXN = 4096, SRC_GUARD_MAXL = 8;
struct SrcLayers {
  int n;
  int off[SRC_GUARD_MAXL + 1];
};
int k_source(int ft, const DevGrid &g, const DevFields &f, const SrcDev &s, int step,
             void *stream);
// Fused step (DESIGN.md "Fused step"): one pass per fields::step() over box G
// (curl B -> H -> curl D -> E, 3-D, no dispersion/NR/B sources).  G is tiled
// into 64 x 14 column tiles and z chunks whose bounds come from the host
// (xb/yb/zb, inclusive starts, last entry = end + 1).  Tiles whose whole
// footprint lies in the lean box L (no PML, every component owned) run the
// lean body; every other tile runs the general body (per-point PML branch
// selection, H/E W updates, per-component ownership).  Inside G, E of a point
// is implicit (= chi1inv * D, never stored) unless the point is owned and in
// a PML chunk along the E direction (then it is stored, ping-pong).
constexpr int FUSED_MAXX = 64, FUSED_MAXY = 160, FUSED_MAXZ = 160;
constexpr int FUSED_MAXCH = 64;  // longest general chunk (planes)
constexpr int FUSED_MAXGY = 256, FUSED_MAXNY = 64;
// general items pack tx, ty, chunk in 8 bits each (mnl_kernels.hip, general_item)
static_assert(FUSED_MAXZ <= 256 && FUSED_MAXX <= 256 && FUSED_MAXGY <= 256, "item encoding");
#ifndef MNL_GW_ROWS
#define MNL_GW_ROWS 10
#endif
#ifndef MNL_GN_ROWS
#define MNL_GN_ROWS 39
#endif
#ifndef MNL_GEN_BPC
#define MNL_GEN_BPC 1
#endif
constexpr int FUSED_GW_ROWS = MNL_GW_ROWS;  // general kernel, wide tiles: own rows per tile
constexpr int FUSED_GN_ROWS = MNL_GN_ROWS;  // general kernel, 16-column tiles: own rows per tile
constexpr int FUSED_GEN_BPC = MNL_GEN_BPC;  // general kernel workgroups per CU
#ifndef MNL_GEN_WPE
#define MNL_GEN_WPE 1
#endif
constexpr int FUSED_GEN_WPE = MNL_GEN_WPE;  // general kernel: minimum waves per SIMD (VGPR cap)
struct FusedTab {                // per direction, indexed by global half-coordinate q
  const uint8_t *flag[3];        // PML chunk along the direction (f_u / W branches)
  const double *kms[3];          // kap - sig
  const double *kps[3];          // kap + sig
  const double *siginv[3];       // 1 / (kap + sig)
};
// Diagnostics (MNL_ITEM_CLOCK, tools/item_clock.py): every persistent-kernel item appends
// one record {start, end (wall clock, 100 MHz), kernel | workgroup << 8, item code, x0 | x1 << 16,
// y0 | y1 << 16, zs | ze << 16, paired strip or -1} to rec (slot from an atomic counter n;
// records past cap are dropped)
struct ItemClock {
  unsigned long long *rec;
  unsigned *n;
  unsigned cap;
  int kind;  // kernel tag written into the records
};
constexpr int CLK_REC = 8;               // u64 per record
constexpr unsigned CLK_CAP = 1u << 20;  // records per batch

struct FusedArgs {
  Box L;              // lean box
  Box G;              // fused domain (stores only inside G)
  int nx, ny, nch;    // tiles along x, y; chunks along z
  int xb[FUSED_MAXX + 1], yb[FUSED_MAXY + 1], zb[FUSED_MAXZ + 1];
  int ngy;            // general wide-tile rows (<= FUSED_GW_ROWS each)
  int gyb[FUSED_MAXGY + 1];
  int nny;            // general 16-column-tile rows (<= FUSED_GN_ROWS each)
  int nyb[FUSED_MAXNY + 1];
  int lx0, lx1, ly0, ly1;      // lean x / y tile index ranges (inclusive)
  int nlzr, lzr[4][2];         // lean chunk index ranges (inclusive), up to 4
  int N[3];           // local points per axis (array extents)
  int off[3];         // global index of local index 0 per axis
  int osh_lo[3], osh_hi[3], oun_lo[3], oun_hi[3];  // owned ranges within G per axis
  int blocks_per_cu;  // persistent workgroups per CU (default 1)
  int wg_limit;       // > 0: at most this many persistent workgroups (CU split between
                      // the lean and general kernels running concurrently)
  int dist;           // lean-body prefetch distance in planes (1 or 2)
  long long nelem;    // elements per field array (selects 32-bit offsets)
  double C;
  long long st1, st2;
  const double *Bo[3];
  double *Bn[3];
  const double *Do[3];
  double *Dn[3];
  const double *E[3];   // stored E (old)
  double *En[3];        // stored E (new)
  const double *Ho[3];  // separate H (null: H == B along that component)
  double *Hn[3];
  const double *UBo[3];  // f_u of B (null: no PML along cycle(d,2))
  double *UBn[3];
  double *UD[3];         // f_u of D, updated in place (only the owner reads it)
  const double *u[3];
  const unsigned *uidx;         // chi1inv palette indices (nullptr: use u / none)
  const double *utab;           // palette, 3 x 256 doubles
  FusedTab tab;
  // isotropic Lorentzian susceptibilities (update_pols), E stored inside pbox
  int npol;
  PolDev pol[MAX_POL];
  Box pbox;                     // union of the pols' nonzero boxes (empty: lo > hi)
  Box xbox;                     // chi(2) box + 1 (inside pbox): E / P left to the NR kernel
  const int *gitems;           // general items: tx | ty << 8 | ch << 16; wide, then narrow
  int ngen, ngen_n;             // wide / narrow item counts (chunk-major order)
  int ngen_e, ngen_ne;          // leading items of chunk 0 (the early launch of multi-rank steps)
  int gbeg, gend, ctr_line;     // set per launch by k_fused: item range and counter line
  unsigned long long cbase;     // counter value at launch start (counters are never reset)
  int ngrp;                     // work queues (1 or 8: one per XCD group, blockIdx % 8)
  int ngrp_gen;                 // the same for the general kernels (k_fused copies it to ngrp)
  const unsigned *gflag;        // general items (index in gitems): the same (k_general_uniform)
  const unsigned *uflag;        // lean items (tile * nch + ch): the palette word shared by
                                // every cell whose chi1inv the item uses, or ~0u (mixed);
                                // null: none (k_lean_uniform)
  int lean_after;               // general launch follows the lean launch of this step on the
                                // same stream: halo B_new of lean-stored points is read, not
                                // recomputed (item bits 27 / 28)
  // tile kernel: items tx | ty << 8 | ch << 16 | body << 24 over the
  // lean-shaped tiles (xb, yb, zb) of every chunk outside the polarization chunks; chunk-0
  // items first (ntit_e of them: the early launch of multi-rank steps)
  const int *titems;
  int ntit, ntit_e;
  const unsigned *tflag;        // per tile item: palette word uniform over its footprint, or ~0u
  unsigned long long cbg[8];    // lean queue g: counter line g's value at launch start
  unsigned long long *ctr;      // FUSED_NCTR work-queue counters (128 B apart); see cbase
  // explicit own boxes of the tile items (null: tx / ty / ch index xb / yb / zb): per item
  // x0 | x1 << 16 (columns, x0 128-byte aligned), yfirst | y1 << 16 (own rows), zs | ze << 16,
  // and a second x-face strip of at most 32 columns sharing the workgroup (xb0 | xb1 << 16,
  // both strips <= 32 columns, body AX = 1) or -1
  const int *tgeo;
  ItemClock clk;                // diagnostics: per-item start / end times (clk.rec null: off)
};

// Temporal blocking: two Yee steps per z-march over the region L2
// (points whose L-infinity distance-2 neighbourhood lies in the lean box and holds no
// source point).  A workgroup's 64 lanes x 16 waves (one row per wave) hold TB_PX = 2 adjacent
// columns per lane (16-byte loads and stores): columns lx .. lx + 127 (lx even) and rows
// y0 - 2 .. y0 + 13; own columns x0 .. x1 with x0 >= lx + 2, x1 <= lx + 125 (up to TB_OXW = 124)
// and own rows y0 .. y0 + 11 (waves 2 .. 13); step n runs on every column, step n+1 is valid two
// columns / rows inside the lanes' footprint.  Round 6: 128 x 16 lanes for 124 x 12 own points
// (was 64 x 16 for 60 x 12).
constexpr int TB_LX = 64, TB_PX = 2, TB_LY = 16, TB_HY = 2, TB_OY = 12, TB_OXW = 124;
constexpr int TB_MAXCH = 512;  // planes per item (any length: the march keeps 3 planes)
struct TB2Item {
  int x;      // x0 | x1 << 16 (own columns, inclusive)
  int y;      // y0 | y1 << 16 (own rows, inclusive)
  int z;      // zs | ze << 16 (own planes [zs, ze))
  int faces;  // bits 0..5: own face x-lo, x-hi, y-lo, y-hi, z-lo, z-hi borders the rim (its
              // points' step n+1 values are stored into the middle buffer set); bits 8..10:
              // 1 + the compact DFT box (TB2Args::cmp) the item's own points meet, 0 none
  // a box of own points whose step n+1 values are also stored into the middle set (the DFT
  // monitors sample step n+1 there): x0 | x1 << 16, y0 | y1 << 16, z0 | z1 << 16 (inclusive);
  // bx < 0: none
  int bx, by, bz;
  int lx;     // column of lane 0's first column (even: 16-byte aligned lane loads)
};
// A DFT monitor's compact box: the two-step kernel stores the D and B
// of its own points inside the box, for the middle (state 0) and the new (state 1) step of a
// pair, at p[((state * 6 + a) * ncell + i)] (a = D0..D2, B0..B2 where mask bit a is set;
// i = x + n0 * (y + n1 * z) relative to lo), so the pair's DFT samples read them densely.
constexpr int TB_MAXCMP = 4;
struct TBCmp {
  int lo[3], n[3];
  double *p;
  unsigned mask;   // arrays stored
  unsigned ncell;  // n0 * n1 * n2 (ncell * 96 bytes < 4 GiB)
};
// Entries no two-step point wrote (rim points, or before the first pair of a plan): this
// signalling-NaN bit pattern, which no arithmetic produces
constexpr unsigned long long DFT_CMP_EMPTY = 0x7FF4D5F7A3E1C9B1ULL;
struct TB2Args {
  int n;                  // items
  const TB2Item *items;
  const unsigned *uflag;  // per item: palette word uniform over its footprint, or ~0u (null: none)
  const double *Bo[3], *Do[3];  // state n (read)
  double *Bm[3], *Dm[3];        // state n+1 at the border points (write)
  double *Bn[3], *Dn[3];        // state n+2 at the own points (write)
  const double *u[3];           // UMODE 1: f64 chi1inv
  const unsigned *uidx;         // UMODE 2: palette indices
  const double *utab;           // UMODE 2: palette, 3 x 256
  int N[3];
  long long st1, st2, nelem;
  double C;
  unsigned long long *ctr;      // work-queue counters (FusedArgs::ctr); line ctr_line
  int ctr_line;
  unsigned long long cbase;
  int wg_limit;                 // > 0: at most this many persistent workgroups (CUs left to
                                // the slab-face kernels of multi-rank pairs)
  ItemClock clk;                // diagnostics: per-item start / end times (clk.rec null: off)
  int ncmp;                     // DFT compact boxes
  TBCmp cmp[TB_MAXCMP];
  int px;                       // columns per lane: 2 (round 6), 1 (the round-5 kernel, A/B)
};
// NaN guard of fields::step (src/step.cpp:138-139): get_field(D_EnergyDensity, gv.center())
// = 1/2 sum_d E_d(c) D_d(c), each value the interpolation of src/monitor.cpp:127-160 over
// this rank's points (terms in interpolate() order: per direction the E terms, then the D
// terms).  kind 0: stored E, 1: implicit E = D * chi1inv (fused box), 2: D.
constexpr int NAN_MAXT = 48;
struct NanTerms {
  int n;
  unsigned char dir[NAN_MAXT], kind[NAN_MAXT];
  long long idx[NAN_MAXT];
  double w[NAN_MAXT];
};
// flag[0] |= 1 (and flag[1] = step, once) when the sum is not finite
int k_nan_check(const NanTerms &t, const double *const E[3], const double *const D[3],
                const double *const U[3], int *flag, int step, void *stream);
// a pair's step tail: the D sources of the step into f.Dn, then the guard over E / D (2: the
// source list is too long for one workgroup -- use k_source + k_nan_check)
int k_src_guard(const DevFields &f, const SrcDev &s, const NanTerms &t, const double *const E[3],
                const double *const D[3], const double *const U[3], int *flag, int step,
                void *stream);
int k_tb2(const TB2Args &a, void *stream, unsigned long long *bases);
int k_tb2_uniform(const TB2Args &a, unsigned *flags, void *stream);
// the tile kernel over an explicit item list (FusedArgs::tgeo boxes), counter line `line`
int k_tile_items(const FusedArgs &a, const int *items, const int *geo, const unsigned *flags,
                 int n, int line, void *stream, unsigned long long *bases);
// per item of that list: the palette word uniform over its footprint, or ~0u
int k_tile_items_uniform(const FusedArgs &a, const int *items, const int *geo, int n,
                         unsigned *flags, void *stream);
// which: 0 = lean tiles, 1 = all general tiles, 2 = general tiles of chunk 0
// only (early launch), 3 = the other general tiles; tile kernel: 4 = all tile items,
// 5 = tile items of chunk 0 (early launch), 6 = the other tile items.  Every launch reads old /
// writes new buffers only, on disjoint points, so any order is valid.
// bases[FUSED_NCTR]: host copy of each counter line's value, advanced by every launch
// (items + workgroups), so no counter reset (memset launch) is needed per step
// counter lines: 0-7 lean queues, 8-11 general (wide/narrow x all/early, one
// queue), FUSED_GLINE0 + (line - 8) * 8 + g: general line split per XCD group g
constexpr int FUSED_GLINE0 = 16, FUSED_NCTR = 48;
int k_fused(const FusedArgs &a, int which, void *stream, unsigned long long *bases);
// per lean item, whether the chi1inv palette word is uniform over the cells it uses
// (flags: ntile * nch words); the lean kernel then reads one cached word instead of
// a palette index per cell
int k_lean_uniform(const FusedArgs &a, unsigned *flags, void *stream);
int k_tile_uniform(const FusedArgs &a, unsigned *flags, void *stream);
int k_general_uniform(const FusedArgs &a, unsigned *flags, void *stream);
int k_cu_count();
int k_build_uidx(unsigned *uidx, const double *const u[3], const double *tab, const int n[3],
                 const Box &F, long long st1, long long st2, int *bad, void *stream);
// E = chi1inv * D over box F (leaving fused mode / readout)
int k_materialize_e(const Box &F, const DevGrid &g, const DevFields &f, void *stream);
int k_fill(double *p, double v, size_t n, void *stream);
// dft_chunk::update_dft for every point of one flux object (src/dft.cpp:265-300),
// blocked over up to DFT_KB updates: sample the averaged field of one update
// into fr, then accumulate n buffered updates (phases: n rows, rstride
// complex values apart) into the DFT array
constexpr int DFT_KB = 32;  // updates buffered per accumulation (the DFT array is read and
                            // written once per DFT_KB updates)
constexpr int DFT_FT = 8;   // frequency tile of the accumulation
int k_dft_sample(const int *pj, const double *pw, const int *pch, const DftChunkDev *ch, double *fr,
                 long long npts, const DevGrid &g, const DevFields &f, void *stream);
// sampling plan of one flux object (per point: the first Yee index, a 16-bit selector, the
// palette bytes and the doubles of the chi1inv of its implicit-E values; see
// dft_plan_kernel), then the sample of one update of every flux object due (one launch)
int k_dft_plan(const int *pj, const int *pch, const DftChunkDev *ch, long long npts,
               const DevGrid &g, const DevFields &f, const unsigned *uidx, const double *utab,
               int *sidx, unsigned short *ssel, unsigned *spal, void *su, int *bad,
               const Box &cbox, int *sci, void *stream);
constexpr int DFT_MAXJ = 8;  // flux objects per sample launch
struct DftSampleJob {
  const int *sidx;
  const unsigned short *ssel;
  const unsigned *spal;
  const void *su;
  const double *pw;
  double *fr;       // this update's sample row
  long long npts;
  long long blk0;   // first workgroup of the job
  int usepal;       // chi1inv from the palette bytes (else the doubles)
  const int *sci;   // compact box index of the first value (-1: some value outside the box)
  const double *cmp;  // the compact box's state of this update (null: none)
  unsigned ncell;
  int cs[3];        // compact strides per direction
};
struct DftSampleJobs {
  DftSampleJob j[DFT_MAXJ];
  int n;
  long long nblk;   // workgroups of all jobs
  long long sd[3];  // set by k_dft_sample_jobs (grid strides per direction)
};
int k_dft_sample_jobs(const DftSampleJobs &J, const DevGrid &g, const DevFields &f,
                      const double *utab, void *stream);
int k_dft_accum(const int *pj, const int *pch, double *dft, const double *fr, int n,
                const double *ph, long long rstride, int nfreq, long long npts, void *stream);
int k_init_add(double *dst, double *alt, const double *src, const DevGrid &g, const DevFields &f,
               int comp_type, int comp_dir, void *stream);
int k_copy(double *dst, const double *src, long long n, void *stream);
int k_average(double *f, const double *bk, long long n, void *stream);
int k_energy(const double *A, const double *Asep, const double *Bv, const DevGrid &g,
             const DevFields &f, int type, int c, const EBox &box, const double *wt,
             double *partial, int nblocks, void *stream);
int k_from_canonical(double *dst, const double *src, const DevGrid &g, int comp_type,
                     int comp_dir, int zlo_glob, void *stream);
int k_to_canonical(double *dst, const double *src, const double *hsep, const DevGrid &g,
                   int comp_type, int comp_dir, const DevFields &f, const Box *fusedF,
                   const double *dsrc, const double *usrc, void *stream);
// the same into a box of the whole-cell array: global indices blo..bhi per
// direction, destination strides bs (entries this rank does not own untouched)
int k_to_box(double *dst, const double *src, const double *hsep, const DevGrid &g, int comp_type,
             int comp_dir, const DevFields &f, const Box *fusedF, const double *dsrc,
             const double *usrc, const int blo[3], const int bhi[3], const long long bs[3],
             void *stream);
// bounding box (local indices per direction, as Pt::j) of the points where any array is nonzero
int k_nonzero_box(const double *const a[3], const DevGrid &g, int *dev_box6, void *stream);
// structure::set_epsilon with a geometric material function (subpixel averaging),
// src/anisotropic_averaging.cpp:58-298: one thread per canonical point of E comp c
// one deferred chi(2) Newton-Raphson problem (run_nr after a failed first attempt)
// Seed of the deterministic stand-in for the std::random_device fallback of runNR
// (newton_raphson.cpp:196-206, 331-336): a counter-based value of the point's global
// half-coordinates q (relative to the cell's little corner; 0 for absent directions), the
// E component d and the time step t, so the oracle (oracle/mnl_oracle.cpp) reproduces the
// product's draws whatever the order, the thread or the rank a point is solved on.
#if defined(__HIPCC__)
__host__ __device__
#endif
inline unsigned long long nr_voxel_seed(long long q0, long long q1, long long q2, int d,
                                        long long t) {
  unsigned long long h = 0x9E3779B97F4A7C15ull;
  h ^= (unsigned long long)q0 * 0xBF58476D1CE4E5B9ull;
  h ^= (unsigned long long)q1 * 0x94D049BB133111EBull;
  h ^= (unsigned long long)q2 * 0xD6E8FEB86659FD93ull;
  h ^= (unsigned long long)d * 0x2545F4914F6CDD1Dull;
  h ^= (unsigned long long)t * 0x9FB21C651E98DF25ull;
  return h;
}

struct NRHard {
  double p[15];       // NRP p1, p2, p3 (A, B, F, G, H each)
  double seed[3];     // the first attempt's seeds
  double fw0[3];      // *fw, *fw_2, *fw_3 on entry (the tolerances)
  double *En;         // result array; the solution component d goes to En[i]
  long long i;
  unsigned long long rng;
  int d;
};
int k_nr_hard(const DevFields &f, void *stream);

struct GeoObj {
  int kind;       // 0 block (p = size), 1 sphere (p0 = radius), 2 cylinder (p0 = radius,
                  // p1 = height, p2 = axis 0/1/2)
  double eps;     // isotropic permittivity (chi1p1)
  double c[3], p[3];
};
constexpr int AVG_MAXQ = 50;  // quadrature points of the largest (3-D) table
struct AvgArgs {
  int ndir, dirs[3];  // present directions in LOOP_OVER_DIRECTIONS order
  int has[3], n[3], io[3];
  int c;              // E component (= its direction)
  double inva, default_eps;
  int nobj;
  const GeoObj *objs;
  const double *quad;  // [3][AVG_MAXQ][4] (x, y, z, weight)
  int nq[3];
  int maxeval;         // 0: no averaging (1 / chi1p1 at the pixel centre)
  double tol;
  double *out[3];      // rows d = 0..2 over the canonical grid (null: not wanted)
  long long ntot;
};
int k_avg_chi1inv(const AvgArgs &a, void *stream);
int k_box_fill(double *dst, const DevGrid &g, int comp_type, int comp_dir, const double *pos_lo,
               const double *pos_hi, double value, int invert, double a, const int *io,
               void *stream);

}  // namespace mnl
