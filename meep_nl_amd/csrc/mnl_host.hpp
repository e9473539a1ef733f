// mnl_host.hpp -- the host side's shared internals (mnl_host.cpp: orchestration and the C-ABI,
// mnl_dft.cpp: DFT monitors): source times, the structure and fields objects, allocation.
// Internal to libmnl.so (not installed; the API is include/meep_nl_amd.h).
#pragma once
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <set>
#include <unordered_set>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "../../include/meep_nl_amd.h"
#include "mnl_comm.hpp"
#include "mnl_internal.hpp"

using namespace mnl;
typedef std::complex<double> cplx;

namespace mnlh {
constexpr int FX_HOST = 64;    // fused tile width (FX in mnl_kernels.hip)
constexpr int FOWN_HOST = 14;  // own rows of a tile item (FOWN in mnl_kernels.hip)
constexpr int TB_RES_CUS = 8;  // multi-rank: CUs left to the slab-face work (one per XCD)
constexpr int SW_HOST = 16;     // narrow strip columns (SW_N in mnl_kernels.hip)
constexpr int SOWN_HOST = 63;   // narrow strip own rows (SR_N - 1)
constexpr int NAN_CH = 256;     // steps per chunk of a batch: the NaN flag is read after each

constexpr double pi = 3.141592653589793238462643383276;  // meep::pi
extern thread_local std::string g_err;

extern int g_verbosity;  // meep::verbosity (src/meep.hpp: default 1)

inline int fail(const std::string &m) {
  g_err = "meep: " + m;
  return -1;
}
#define HIPCHK(x)                                                                 \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess)                                                         \
      return fail(std::string("HIP error ") + hipGetErrorString(e_) + " at " #x); \
  } while (0)

inline int cdir(int c) { return c % 3; }
inline int ctype(int c) { return c / 3; }

// ------------------------------------------------------------- source time
// gaussian_src_time / continuous_src_time (src/sources.cpp:85-141,
// src/meep.hpp:937-1056).
struct SrcTime {
  int kind = 0;
  bool is_integrated = false;
  double freq = 0, width = 0, peak_time = 0, cutoff = 0;
  cplx cfreq;
  double cwidth = 0, start_time = 0, end_time = 0, slowness = 3;
  double cur_time = NAN;
  cplx cur_dipole, cur_current;
  mnl_src_func func = nullptr;  // kind 2: custom_src_time (src/meep.hpp:1059-1092)
  void *fdata = nullptr;

  cplx dipole(double time) const {
    if (kind == 2) {
      const float rtime = float(time);
      if (!(rtime >= start_time && rtime <= end_time)) return 0.0;
      double re = 0, im = 0;
      func(time, fdata, &re, &im);
      return cplx(re, im);
    }
    if (kind == 0) {
      double tt = time - peak_time;
      if (float(fabs(tt)) > cutoff) return 0.0;
      cplx amp = 1.0 / cplx(0, -2 * pi * freq);
      return exp(-tt * tt / (2 * width * width)) * std::polar(1.0, -2 * pi * freq * tt) * amp;
    }
    float rtime = float(time);
    if (rtime < start_time || rtime > end_time) return 0.0;
    cplx amp = 1.0 / (cplx(0, -1.0) * (2 * pi) * cfreq);
    if (cwidth == 0.0) return exp(cplx(0, -1.0) * (2 * pi) * cfreq * time) * amp;
    double ts = (time - start_time) / cwidth - slowness;
    double te = (end_time - time) / cwidth - slowness;
    return exp(cplx(0, -1.0) * (2 * pi) * cfreq * time) * amp * (1.0 + tanh(ts)) *
           (1.0 + tanh(te)) * 0.25;
  }
  void update(double time, double dt) {  // src_time::update, src/meep.hpp:972-978
    if (time != cur_time) {
      cur_dipole = dipole(time);
      // custom_src_time::current: the dipole itself unless integrated
      cur_current = (kind == 2 && !is_integrated) ? dipole(time)
                                                 : (dipole(time + dt) - dipole(time)) / dt;
      cur_time = time;
    }
  }
  bool same(const SrcTime &o) const {
    return kind == o.kind && is_integrated == o.is_integrated && freq == o.freq &&
           width == o.width && peak_time == o.peak_time && cutoff == o.cutoff &&
           cfreq == o.cfreq && cwidth == o.cwidth && start_time == o.start_time &&
           end_time == o.end_time && slowness == o.slowness && func == o.func && fdata == o.fdata;
  }
};

struct SrcGroup {  // src_vol (src/meep_internals.hpp:49-82) over the whole cell
  int comp;        // E or H component
  int st;
  std::vector<long long> gidx;  // global canonical index of comp
  std::vector<int> jglob;       // 3 global indices per point
  std::vector<cplx> amp;
};

struct Lorentz {
  double omega0, gamma;
  int drude;
  std::vector<double> sigma[3];  // canonical arrays (empty = 0)
  std::vector<double> off[3][3];  // off-diagonal sigma[c][d], d != c (empty = 0)
  bool aniso() const {
    for (int c = 0; c < 3; c++)
      for (int d = 0; d < 3; d++)
        if (!off[c][d].empty()) return true;
    return false;
  }
};

struct BoxSpec {
  int kind, index;
  double box[6];
  double value;
};

}  // namespace mnlh
using namespace mnlh;

// =============================================================== structure
struct mnl_structure {
  int dim;
  int n[3];
  int io[3];
  bool has[3];
  double a, courant, dt;
  double pml_thick[3][2] = {{0, 0}, {0, 0}, {0, 0}};
  double pml_R[3][2], pml_stretch[3][2];
  std::vector<double> chi1inv[3][3];  // [E comp][dir], canonical
  std::vector<double> chi2[3], chi3[3];
  std::vector<double> cond[2][3];     // conductivity of [B, D][dir], canonical (empty = 0)
  std::vector<Lorentz> lor;
  // H side: chi1inv of the H components (structure::set_mu ->
  // set_chi1inv(H_stuff), [H comp][dir], canonical) and the magnetic susceptibilities
  // (add_susceptibility(sigma, H_stuff, ...), diagonal sigma at the H components' points)
  std::vector<double> mu1inv[3][3];
  std::vector<Lorentz> hlor;
  std::vector<BoxSpec> boxes;
  size_t ntot;
  int nl_mode = 0;  // 0: the fork (NR chi2, inert chi3); 1: upstream Meep (Pade chi2/chi3)

  int shift(int c, int d) const {
    if (!has[d]) return 0;
    int t = ctype(c);
    if (t == T_E || t == T_D) return d == cdir(c);
    return d != cdir(c);
  }
  long long cstride(int d) const {
    if (!has[d]) return 0;
    long long nz = has[2] ? n[2] + 1 : 1, ny = has[1] ? n[1] + 1 : 1;
    return d == 2 ? 1 : (d == 1 ? nz : nz * ny);
  }
};

// ------------------------------------------------------------- DFT flux
// fields::add_dft_flux / add_dft / update_dfts / dft_flux::flux (src/dft.cpp:
// 51-300, 533-547, 578-640; loop_in_chunks src/loop_in_chunks.cpp:225-520),
// Cartesian, no symmetry, centered grid.  The point set, interpolation weights
// and list order are those of the reference's single-process chunk layout
// (PML regions broken off, structure.cpp:118-137), so every per-point DFT is
// bitwise the reference's; each rank accumulates the points it owns on the
// device, and flux() sums the pairs in list order on the host.
struct DftChunkH {
  int c;
  cplx scale;
  int avgmode;       // 0: point, 1: two Yee points, 2: four
  size_t N, p0;      // points, first point in the flux object's point arrays
  // the chunk's loop (for get_dft_array): corners, boundary weights, dV0,
  // include_dV_and_interp_weights, stored_weight
  int is[3], ie[3];
  double s0[3], s1[3], e0[3], e1[3], dV0;
  bool incl;
  cplx stored;
};
struct DftFluxH {
  std::vector<double> omega;
  int nfreq = 0, decim = 1;
  bool fields = false;                // dft_fields (add_dft_fields): chunks in E only
  double wmin[3] = {0, 0, 0}, wmax[3] = {0, 0, 0};  // `where` (get_dft_array's collapse)
  std::vector<DftChunkH> E, H;        // list order (next_in_dft)
  size_t npts = 0;                    // E points, then H points
  std::vector<int> h_pj;              // 3 local indices per point (-1: not this rank's)
  Box bbox{};                         // this rank's points, +1 along every axis (dft_layout;
                                      // empty: lo > hi)
  int *d_pj = nullptr, *d_pch = nullptr;
  double *d_pw = nullptr;             // w * 0.25 / 0.5 / 1 per point
  DftChunkDev *d_ch = nullptr;        // per chunk (E list, then H list)
  double *d_dft = nullptr;            // [slot/64][freq][slot%64] complex (re, im)
  double *d_ph = nullptr;             // phases of one batch: [update][chunk][freq] complex
  size_t ph_cap = 0;
  int row = 0;                        // next phase row of this batch
  std::vector<double> ph_host;        // host copy of d_ph (the buffered rows move to the front)
  std::vector<int> slot;              // device slot of each point (reference order -> slot)
  double *d_fr = nullptr;             // [update][slot] sampled fields awaiting accumulation
  int nbuf = 0;                       // buffered updates (rows row-nbuf .. row-1)
  int kb = DFT_KB;                    // updates per accumulation
  double bytes = 0;                   // algorithmic bytes of one update (DESIGN.md "DFT")
  int *d_sidx = nullptr;              // sampling plan (k_dft_plan): first Yee index per point
  unsigned short *d_ssel = nullptr;   // ... and a selector per point
  unsigned *d_spal = nullptr;         // ... and the palette bytes of its implicit-E chi1inv
  void *d_su = nullptr;               // ... or those chi1inv values as doubles (fallback)
  int *d_bad = nullptr;               // palette check of the plan (k_dft_plan)
  bool usepal = false;                // the plan's palette bytes are exact
  // compact box (pairs of steps): bbox's D / B of the two-step points
  // for both steps of a pair, stored by the two-step kernel; per point its compact index
  double *d_cmp = nullptr;
  unsigned cmp_cells = 0;             // 0: the box is too large for a compact copy
  unsigned cmp_mask = 0;              // arrays the samples read (D0..D2, B0..B2)
  int *d_sci = nullptr;
  bool cmp_on = false;                // the current pair plan stores this monitor's box
  long long plan_key = -1;            // the mode the plan was built for (dft_plan_key)
  ~DftFluxH() {
    if (d_ph) (void)hipFree(d_ph);
    if (d_sidx) (void)hipFree(d_sidx);
    if (d_ssel) (void)hipFree(d_ssel);
    if (d_spal) (void)hipFree(d_spal);
    if (d_su) (void)hipFree(d_su);
    if (d_bad) (void)hipFree(d_bad);
    if (d_cmp) (void)hipFree(d_cmp);
    if (d_sci) (void)hipFree(d_sci);
  }
};


// =============================================================== fields
struct mnl_fields {
  mnl_structure S;  // copy of the global structure description
  int device = 0;
  hipStream_t stream = nullptr;
  int rank = 0, nranks = 1;
  std::unique_ptr<Comm> comm;
  int slab_dir = 2;  // direction decomposed across ranks
  DevGrid g;
  DevFields f;
  size_t nlocal = 0;  // doubles per local array
  bool allocated[MNL_NUM_COMPONENTS] = {false};
  bool pml_any[3] = {false, false, false};
  std::vector<uint8_t> h_flag[3], h_zone[3];
  std::vector<double> h_sig[3], h_kap[3], h_siginv[3];
  std::vector<void *> dev_allocs;
  Box interior;
  // chi(2) Newton-Raphson runs only where chi2 != 0: the interior E update splits
  // into the bounding box of those points (NR kernel) and the rest (plain kernel)
  bool nr_split_done = false;
  bool nr_shell_free = false;  // the chi2 box lies inside the interior: plain shell E kernels
  Box nr_in{};
  std::vector<Box> nr_rest;
  Box nr_chi2{};  // bounding box of chi2 != 0 (device coordinates; empty: lo > hi)
  // fused mode with chi(2): the chi2 box grown by one point, whose E / P the fused
  // kernels leave to the NR E kernel (nr_fused_e); empty: no NR point anywhere
  Box nr_xbox{};
  std::vector<Box> shell;
  BoxList shell_list;
  // fused mode (DESIGN.md "Fused step")
  bool fused = false;        // currently stepping in fused mode
  Box fusedG;                // fused domain (local indices)
  Box fusedL;                // lean box (no PML, every component owned)
  BoxList fused_shell;       // everything else (multi-rank: the top plane)
  FusedArgs fgeo;            // tile / chunk bounds (filled by make_fused_boxes)
  std::vector<int> gitems;   // general-kernel items
  int *d_gitems = nullptr;
  size_t d_gitems_cap = 0;
  // tile mode (MNL_TILE, default on): one tile kernel over every chunk outside the
  // polarization chunks (lean + PML bodies), the general kernel over those chunks only
  bool tile_mode = true;
  bool tile_zcut = true;      // cut z chunks at the lean box's z range (short z-PML items)
  int tile_body_mask = -1;   // MNL_TILE_BODY_MASK: step only these bodies (timing experiments)
  // diagnostic / A-B switches, read once when the fields are created (mnl_fields_create)
  bool ownc = true;           // MNL_NO_OWNC=1: no OWNC item flag
  bool lean_halo = true;      // MNL_LEAN_HALO=0: general tiles recompute the lean halo
  bool no_palette = false;    // MNL_NO_PALETTE=1: per-cell chi1inv loads, no byte palette
  bool uniform = true;        // MNL_UNIFORM=0: per-cell palette loads in uniform items too
  int lean_groups = 1, gen_groups = 1;  // MNL_LEAN_GROUPS / MNL_GEN_GROUPS: 1 or 8 queues
  bool tile_gen_cus_env = false;        // MNL_TILE_GEN_CUS given (the tuner keeps it)
  bool fused_zchunk_env = false;        // MNL_FUSED_ZCHUNK given (the tuner keeps it)
  bool tb_env = false, tb_zchunk_env = false;  // MNL_TB / MNL_TB_ZCHUNK given (the same)
  bool nr_defer = true;       // MNL_NR_DEFER=0: every NR problem solved in place
  bool tile_stats = false, tb_stats = false;  // MNL_TILE_STATS / MNL_TB_STATS: print
  // MNL_ITEM_CLOCK=<file>: per-item start / end records of the persistent kernels, appended
  // to <file> after every batch (ItemClock; tools/item_clock.py)
  std::string clk_path;
  unsigned long long *d_clk = nullptr;
  unsigned *d_clk_n = nullptr;
  std::vector<int> titems;   // tile-kernel items (FusedArgs::titems)
  int *d_titems = nullptr;
  size_t d_titems_cap = 0;
  unsigned *d_tflag = nullptr;  // per tile item: uniform palette word or ~0u
  size_t tflag_n = 0;
  long long tile_cells = 0;     // own cells of the tile items
  double tile_cells_nu = -1;    // ... of those that read a palette index per cell
  std::vector<char> tile_z;     // per local z plane: stepped by the tile kernel
  long long lean_cells = 0, gen_cells = 0;
  FusedTab d_tab{};          // per-direction PML coefficient tables for the fused kernels
  // multi-rank fused stepping: chunk 0 on s_aux, halo exchange on s_comm,
  // overlapped with the interior kernels on `stream` (DESIGN.md "Multi-GPU")
  hipStream_t s_aux = nullptr, s_comm = nullptr;
  hipEvent_t ev_start = nullptr, ev_early = nullptr, ev_x1 = nullptr, ev_shell = nullptr,
             ev_x0 = nullptr;
  hipStream_t s_lint = nullptr;     // pairs: interior two-step items (tb_lint)
  hipEvent_t ev_lint = nullptr, ev_r1done = nullptr;
  double *pp_B[3] = {nullptr, nullptr, nullptr}, *pp_D[3] = {nullptr, nullptr, nullptr};
  double *pp_E[3] = {nullptr, nullptr, nullptr}, *pp_H[3] = {nullptr, nullptr, nullptr};
  double *pp_UB[3] = {nullptr, nullptr, nullptr};
  int fused_zchunk = 0;
  int fused_bpc = 1;
  int fused_dist = 1;
  int gen_cus = -1;  // CUs for the general kernel running beside the lean one (0: serial)
  bool fused_concurrent = false;  // last fused step ran lean + general concurrently
  int tile_gen_cus = 0;           // tile mode: general kernel beside the tile kernel (CUs)
  unsigned long long *d_fused_ctr = nullptr;  // work-item counters of the fused kernels
  unsigned long long ctr_base[FUSED_NCTR] = {0};  // their values at the next launch
  int stagger = 0, nstagger = 0;  // dev_alloc offset step (bytes) for field arrays
  void *arena = nullptr;           // optional single allocation for field-sized arrays
  size_t arena_cap = 0, arena_used = 0, arena_gap = 0;
  int arena_req = 0;               // MNL_ARENA: field arrays to reserve (0: off)
  bool contig = false;             // MNL_CONTIG: physically contiguous field allocations
  int contig_fallbacks = 0;        // contiguous requests the driver could not satisfy
  bool palette_tried = false;
  bool dsrc_in_shell = false;  // a D source point lies outside the interior box
  bool any_srcB = false, any_isrc = false;  // anywhere in the cell (all ranks agree)
  bool any_dsrc_w = false;  // a D current source on a W-form (PML-along-E) point
  unsigned *d_uidx = nullptr;  // chi1inv palette indices over fusedG (null: f64 chi1inv)
  double *d_utab = nullptr;    // 3 x 256 palette values
  unsigned *d_uflag = nullptr;  // per lean item: uniform palette word or ~0u (k_lean_uniform)
  size_t uflag_n = 0;
  unsigned long long uflag_sig = 0;  // geometry the flags were built for
  unsigned *d_gflag = nullptr;  // per general item (k_general_uniform)
  size_t gflag_n = 0;
  // cells of lean / general items that still read a palette index per cell (the
  // algorithmic bytes of bench.py's roofline count 4 B of chi1inv for those only)
  double lean_cells_nu = -1, gen_cells_nu = -1;
  bool uflag_active = false;
  bool allow_fused = true;
  // the reference allocates H (as a copy of B) and the W auxiliary fields (as a
  // copy of E / H) on the first update_eh (src/update_eh.cpp:204-216); the first
  // step runs unfused and performs those copies at the same points of the step
  bool e_first_done = false, h_first_done = false;
  bool u_first_done[2] = {false, false};  // f_u of B / D: a copy of f on the first step_db
                                          // (src/step_db.cpp:71-75)
  bool first_step_mode = false;
  bool force_unfused_next = false;  // E / H set directly (initialize_field): E != chi1inv D
  // temporal blocking: pairs of steps as rim (one-step tile kernel) +
  // L2 (two-step kernel) + rim, over three buffer sets
  bool tb_enabled = true;           // MNL_TB=0 at creation: never
  int tb_zchunk = 0;                // planes per two-step item (0: automatic)
  int rim_zchunk = 0;               // planes per rim item of a pair (0: fused_zchunk)
  bool tb_pol_on = true;            // MNL_TB_POL=0 / set_schedule 11: no pairs with them
  bool tb_r1a = true;               // MNL_TB_R1A=0 / set_schedule 12: R1 after the two-step
                                    // kernel instead of its non-strip items beside it
  int tb_rs0 = 0;                   // rim items before the narrow strips (one rank)
  int tb_lint = 0;                  // MNL_TB_LINT=1 / set_schedule 13: the interior two-step
                                    // items beside the previous pair's second rim launch
  int tb_nint = 0;                  // two-step items whose footprint meets no rim box (first)
  bool ev_fence = false;            // MNL_EV_FENCE=1: timing events with the default fence
  bool tb_srcguard = true;          // MNL_TB_SRCGUARD=0 / set_schedule 16: a pair's sources
                                    // and guard as two launches per step (default: one)
  int tb_szc = 0;                   // planes per narrow strip item (0: the rim's chunk length;
                                    // MNL_TB_STRIP_ZCHUNK / set_schedule 15)
  int tb_r2lpt = 0;                 // MNL_TB_R2LPT / set_schedule 14: the second rim launch
                                    // longest first (1) or strips first (2); default: the
                                    // first one's order, narrow strips last
  bool tb_r1done_ok = false;        // ev_r1done marks the previous pair's R1 join (same batch)
  bool tb_pol = false;              // the pairs step polarization chunks (general kernel, one
                                    // step at a time beside the rim launches; one rank)
  int tb_px = 2;                    // columns per lane of the two-step kernel (1: the round-5
                                    // kernel, for A/B; MNL_TB_PX)
  bool tb_ox_set = false;           // tb_ox set by set_schedule (the tuner keeps it)
  int tb_ox = 0;                    // most own columns of a two-step item (0: TB_OXW = 124,
                                    // the 128 columns of lanes less two halo columns per side)
  bool nr_early = true;             // MNL_NR_EARLY=0: the NR box's E phase after both kernels
  unsigned fused_epoch = 0;         // bumped on every entry into the fused mode
  unsigned long long tb_sig = 0;    // inputs of the current plan (0: none)
  bool tb_have = false;             // the current plan has two-step items
  bool tb_mid_fresh = false;        // middle set holds a copy of the state (ghost / wall entries)
  std::vector<int> tb_ritems, tb_rgeo;  // rim items (tile-kernel codes) and their own boxes
  std::vector<TB2Item> tb_items;        // two-step items
  int *d_tb_ritems = nullptr, *d_tb_rgeo = nullptr;
  unsigned *d_tb_rflag = nullptr, *d_tb_uflag = nullptr;
  TB2Item *d_tb_items = nullptr;
  size_t tb_rcap = 0, tb_gcap = 0, tb_icap = 0;
  bool tb_nopair = false;   // MNL_TB_NOPAIR=1: x-face rim strips one per workgroup (A/B)
  bool tb_last = false;     // the last batch of >= 2 steps stepped in pairs (tb_usable)
  int res_l = -1, res_r = -1;  // schedule options: the same for the two-step / rim launches only
  int tb_res = -1;          // MNL_TB_RES: CUs the pairs' persistent launches leave free (-1:
                            // TB_RES_CUS with several ranks, 0 with one; A/B of the reservation)
  bool tb_oom = false;      // the middle buffer set did not fit: temporal blocking off
  bool tb_oom_test = false; // MNL_TB_OOM=1: its allocation fails (tests)
  bool tb_narrow = true;    // MNL_TB_NARROW=0: no narrow x-face strip items (A/B)
  bool dft_pal = true;      // MNL_DFT_PAL=0: DFT sampling plans carry chi1inv as doubles (A/B)
  bool dft_cmp = true;      // MNL_DFT_CMP=0: pairs sample DFT monitors from the field arrays
  std::vector<TBCmp> tb_cmp;  // the compact DFT boxes of the current pair plan
  int tb_nnarrow = 0;       // narrow x-face strip items of the current plan
  int tb_rfree = 0;         // leading rim items that read no slab-face data (multi-rank)
  bool tb_chain_pending = false;  // the last multi-rank pair's s_comm chain not yet joined
  double *pp3_B[3] = {nullptr, nullptr, nullptr}, *pp3_D[3] = {nullptr, nullptr, nullptr};
  double *pp3_E[3] = {nullptr, nullptr, nullptr}, *pp3_H[3] = {nullptr, nullptr, nullptr};
  double *pp3_UB[3] = {nullptr, nullptr, nullptr};
  double tb_cells = 0, tb_border = 0, tb_cells_nu = 0;  // own / border points of the items,
                                                        // own points of the mixed-palette ones
  double rim_cells = 0, rim_lean = 0, rim_cells_nu = 0;  // rim items: own / lean / mixed cells
  int nan_every = 1;                // NaN guard cadence (src/step.cpp:138-139: every step)
  int since_nan = 0;                // steps since the last NaN guard (across calls)
  long long nan_bad_t = -1;         // first failing step of the last tripped NaN guard (-1: none)
  bool nan_due = false;             // a guard is due once the state is complete (pending rim)
  int nan_launched = 0;             // guards launched in this chunk (flag read at its end)
  long long nan_at = 0;             // time step of the state the next guard checks
  NanTerms nan_terms{};             // this batch's interpolation terms (nan_terms_build)
  int *d_nanflag = nullptr;         // [flag, step]
  CurlPlan planB, planD;
  bool nr = false;
  bool upnl = false;  // upstream chi2/chi3 update active (nl_mode 1 with nonzero chi)
  bool hall = false;  // H-side materials: H stored everywhere (DevFields::hall)
  std::vector<uint8_t> h_hsep_zone;  // host copy of DevFields::hsep_zone (27 zone boxes)
  // sources
  std::vector<SrcTime> srcs;
  std::vector<SrcGroup> groups;
  bool src_dirty = true;
  std::vector<long long> srcB_idx, srcD_idx, isrc_idx;  // local linear indices
  std::vector<int> srcB_comp, srcD_comp, isrc_comp;
  std::vector<unsigned char> isrc_zone;  // owning reference chunk (zone box) per isrc point
  ISrcDev isrc_dev{};                    // device copy (sorted), built with the lists
  std::vector<std::pair<int, int>> srcB_ref, srcD_ref, isrc_ref;  // (group, point)
  // current sources per field type ([0] B, [1] D), in layer order (SrcDev)
  std::vector<double> src_amp[2];
  std::vector<int> src_gid[2], src_layer[2];
  long long *d_srcB_idx = nullptr, *d_srcD_idx = nullptr;
  int *d_srcB_comp = nullptr, *d_srcD_comp = nullptr;
  double *d_src_amp[2] = {nullptr, nullptr};
  int *d_src_gid[2] = {nullptr, nullptr};
  double *d_vals = nullptr;
  size_t d_vals_cap = 0;
  long long t = 0;
  double dt;
  // timers / profiling
  bool profiling = false;
  // fields::times_spent by time_sink (src/meep.hpp:1610-1633 order), seconds
  double sink_s[MNL_NUM_TIME_SINKS] = {0};
  double last_out_wall = -1;  // "on time step" output (src/step.cpp:44-56)
  long long last_out_t = 0;
  double timer_ms[16] = {0};
  long long timer_count[16] = {0};
  std::vector<hipEvent_t> ev_pool;
  unsigned long long *d_nr_fallbacks = nullptr;
  NRHard *d_nr_hard = nullptr;      // deferred Newton-Raphson problems (NR runs only)
  unsigned *d_nr_hard_cnt = nullptr;
  double *d_scratch = nullptr;  // canonical-size staging buffer
  size_t scratch_cap = 0;
  std::vector<std::unique_ptr<DftFluxH>> dfts;  // DFT flux objects (add_dft_flux order)

  ~mnl_fields() {
    if (device >= 0) hipSetDevice(device);
    for (void *p : dev_allocs) hipFree(p);
    for (auto e : ev_pool) hipEventDestroy(e);
    if (d_scratch) hipFree(d_scratch);
    if (d_vals) hipFree(d_vals);
    if (d_gitems) hipFree(d_gitems);
    if (d_titems) hipFree(d_titems);
    if (d_tflag) hipFree(d_tflag);
    if (d_uflag) hipFree(d_uflag);
    if (d_gflag) hipFree(d_gflag);
    for (void *p : {(void *)d_tb_ritems, (void *)d_tb_rgeo, (void *)d_tb_rflag, (void *)d_tb_uflag,
                    (void *)d_tb_items})
      if (p) hipFree(p);
    comm.reset();
    for (hipEvent_t e : {ev_start, ev_early, ev_x1, ev_shell, ev_x0, ev_lint, ev_r1done})
      if (e) hipEventDestroy(e);
    if (s_aux) hipStreamDestroy(s_aux);
    if (s_lint) hipStreamDestroy(s_lint);
    if (s_comm) hipStreamDestroy(s_comm);
    if (stream) hipStreamDestroy(stream);
  }
};

namespace mnlh {

bool in_fused_box(const mnl_fields *F, int c, const int jg[3]);
int nan_launch(mnl_fields *F, hipStream_t st = nullptr, double *const *E = nullptr,
               double *const *D = nullptr);
void nan_count(mnl_fields *F, int k);
int nan_result(mnl_fields *F);
int nan_terms_build(mnl_fields *F);

// Field-sized arrays start at staggered offsets (a multiple of 128 B, different
// for every array) so that the many streams one fused step reads and writes at
// the same element index do not start on the same HBM channel / bank.
template <class T>
int dev_alloc(mnl_fields *F, T **p, size_t n, bool zero = true) {
  void *q = nullptr;
  const size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
  if (F->arena_req > 0 && !F->arena && F->nlocal && bytes >= (size_t(64) << 20)) {
    const size_t cap = size_t(F->arena_req) * (F->nlocal * 8 + F->arena_gap + 4096);
    const hipError_t ea = F->contig ? hipExtMallocWithFlags(&F->arena, cap, hipDeviceMallocContiguous)
                                    : hipMalloc(&F->arena, cap);
    if (ea == hipSuccess) {
      F->arena_cap = cap;
      F->dev_allocs.push_back(F->arena);
    } else {
      F->arena_req = 0;
      (void)hipGetLastError();
    }
  }
  if (F->arena_cap && bytes >= (size_t(64) << 20)) {  // field-sized: bump-allocate in the arena
    const size_t at = (F->arena_used + 255) & ~size_t(255);
    if (at + bytes <= F->arena_cap) {
      F->arena_used = at + bytes + F->arena_gap;
      *p = (T *)((char *)F->arena + at);
      if (zero) {
        hipError_t e = hipMemsetAsync(*p, 0, bytes, F->stream);
        if (e != hipSuccess) return fail(std::string("hipMemset failed: ") + hipGetErrorString(e));
      }
      return 0;
    }
  }
  const bool big = bytes >= (size_t(64) << 20) && F->stagger > 0;
  const size_t off = big ? (size_t(F->stagger) * F->nstagger++) % (size_t(1) << 20) : 0;
  const size_t nb = bytes + (big ? (size_t(1) << 20) : 0);
  hipError_t e = hipErrorUnknown;
  if (F->contig && bytes >= (size_t(64) << 20)) {
    e = hipExtMallocWithFlags(&q, nb, hipDeviceMallocContiguous);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      F->contig_fallbacks++;
    }
  }
  if (e != hipSuccess) e = hipMalloc(&q, nb);
  if (e != hipSuccess) return fail(std::string("hipMalloc failed: ") + hipGetErrorString(e));
  if (zero) {
    e = hipMemsetAsync((char *)q + off, 0, bytes, F->stream);
    if (e != hipSuccess) return fail(std::string("hipMemset failed: ") + hipGetErrorString(e));
  }
  F->dev_allocs.push_back(q);
  *p = (T *)((char *)q + off);
  return 0;
}

// ---- mnl_host.cpp, used by mnl_dft.cpp
struct ZoneIv {
  int c0, c1, zone;  // chunk covers half-coords [c0, c1] relative to io
};
std::vector<ZoneIv> zone_intervals(const mnl_structure &S, int d);
int build_source_lists(mnl_fields *F);

// ---- mnl_dft.cpp: loop_in_chunks helpers and DFT monitors
inline int my_round(double x) { return int(floor(fabs(x) + 0.5) * (x < 0 ? -1 : 1)); }
inline size_t dft_at(size_t p, size_t i, size_t nf) { return ((p >> 6) * nf + i) * 64 + (p & 63); }
void dft_boundary_weights(const mnl_structure &S, const double wmin[3], const double wmax[3],
                          const int is[3], const int ie[3], double s0[3], double e0[3],
                          double s1[3], double e1[3]);
std::vector<std::array<int, 6>> reference_chunks(const mnl_structure &S);
int dft_decimation(mnl_fields *F, const double *freqs, int nfreq, int decim);
int dft_add_flux(mnl_fields *F, int nreg, const double *regions, const double *freqs, int nfreq,
                 int decim);
int dft_add_fields(mnl_fields *F, int ncomp, const int *comps, const double wmin[3],
                   const double wmax[3], const double *freqs, int nfreq, int yee, int decimation);
int dft_prepare(mnl_fields *F, long long t0, int ns);
int dft_flush(mnl_fields *F, DftFluxH &o);
long long dft_plan_key(const mnl_fields *F);
// cstate >= 0: a pair's middle (0) or new (1) state, whose two-step points are also in the
// monitors' compact boxes
int dft_update(mnl_fields *F, long long t, const DevFields *fields = nullptr, int cstate = -1);
bool dft_due(const mnl_fields *F, long long t);
int dft_flux_values(mnl_fields *F, int h, double *out);
// ---- mnl_host.cpp, used by mnl_dft.cpp
int timed_allreduce(mnl_fields *F, double *v, int n);

// ---- mnl_io.cpp: checkpoints, array slices, field energy
struct CkEntry {
  int kind, a, b;
  double *p;
  size_t n;
};
inline double wall_now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
// loop_in_chunks' per-index weight of a dimension (s0 / s1 at the low end, e0 / e1 at the high)
inline double loop_w1(double s0, double s1, double e0, double e1, int i, int n) {
  return (i > 1 && i < n - 2) ? 1.0 : (i == 0 ? s0 : (i == 1 ? s1 : i == n - 1 ? e0 : (i == n - 2 ? e1 : 1.0)));
}
std::vector<CkEntry> ckpt_entries(mnl_fields *F);
int fields_dump(mnl_fields *F, const char *path);
int fields_load(mnl_fields *F, const char *path);
int structure_dump(const mnl_structure *S, const char *path);
int structure_load(mnl_structure *S, const char *path);
int array_slice(mnl_fields *F, int c, const double vmin[3], const double vmax[3], int snap,
                int *rank, long long dims[3], double *out, long long nout);
int energy_in_box(mnl_fields *F, int which, const double wmin[3], const double wmax[3],
                  double *out);
// ---- mnl_host.cpp, used by mnl_io.cpp
int exchange(mnl_fields *F, int kind, hipStream_t st = nullptr);
int h_lazy_copy(mnl_fields *F);
int u_lazy_copy(mnl_fields *F, int which);
bool has_field(const mnl_structure &S, int c);
int set_fused(mnl_fields *F, bool on);
SrcDev src_dev(mnl_fields *F, int t, const double *J);
int update_h_any(mnl_fields *F, const BoxList &sl, bool pols);

}  // namespace mnlh
