/* meep_nl_amd.h -- C-ABI of the MI355X-native fields::step() hot path.
 *
 * Drop-in boundary for the reference's time-stepping core (PMack10/meep_nl =
 * MIT Meep 1.30 + chi(2) Newton-Raphson fork).  Plain pointers and sizes only;
 * no torch / HIP types.  Each entry cites the reference interface it replaces.
 *
 * Conventions
 *   - components: MNL_EX..MNL_BZ (E, H, D, B x,y,z).  NOT the reference enum
 *     order (src/meep/vec.hpp:31-56 interleaves Er/Ep); bindings map by name.
 *   - grids: dim 1 = Z only (Meep D1), 2 = X,Y (Meep D2), 3 = X,Y,Z.
 *     n[d] cells, resolution a, little corner io[d] in half-pixels
 *     (grid_volume io, src/meep/vec.hpp:1014-1180; io = -n for center_origin).
 *   - host arrays use the reference's per-chunk layout for the whole cell:
 *     (n_d+1) points per present direction, Z fastest, X slowest
 *     (grid_volume::set_strides, src/vec.cpp:482-494).  Entry j of a
 *     component c sits at half-pixel io + 2 j + yee_shift(c).
 *   - every call returns 0 on success, nonzero on error; mnl_last_error()
 *     returns the message ("meep: ..." as meep::abort, src/mympi.cpp:244-262).
 *   - the product path has no CPU fallback: creating fields without a HIP
 *     device fails.
 */
#ifndef MEEP_NL_AMD_H
#define MEEP_NL_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  MNL_EX = 0, MNL_EY, MNL_EZ, MNL_HX, MNL_HY, MNL_HZ,
  MNL_DX, MNL_DY, MNL_DZ, MNL_BX, MNL_BY, MNL_BZ, MNL_NUM_COMPONENTS
};
/* derived components of array slices (the reference's Dielectric / Permeability,
 * src/meep/vec.hpp:52-53): epsilon / mu on the Centered grid from the diagonal chi1inv */
enum { MNL_DIELECTRIC = 12, MNL_PERMEABILITY = 13 };
enum { MNL_X = 0, MNL_Y = 1, MNL_Z = 2 };
enum { MNL_LOW = 0, MNL_HIGH = 1 };
enum { MNL_SRC_GAUSSIAN = 0, MNL_SRC_CONTINUOUS = 1, MNL_SRC_CUSTOM = 2 };
/* custom_src_time callback: writes the complex dipole f(t) (src/meep.hpp:1059-1092) */
typedef void (*mnl_src_func)(double t, void *data, double *re, double *im);
/* amplitude function A(r) of a volume source: writes A at the position rel
 * (relative to the volume centre; src/sources.cpp:262-271) */
typedef void (*mnl_amp_func)(const double rel[3], void *data, double *re, double *im);

typedef struct mnl_structure mnl_structure;
typedef struct mnl_fields mnl_fields;

/* Thread-local message of the last failing call (meep::abort text). */
const char *mnl_last_error(void);
/* ABI version (major*100+minor). */
int mnl_version(void);
/* Number of visible HIP devices (0 on a host without GPU). */
int mnl_device_count(int *count);

/* ---- structure (replaces meep::structure, src/meep.hpp:809-920) ---------- */

/* structure(grid_volume, eps, boundary_region, symmetry=identity, num_chunks,
 * Courant) -- src/structure.cpp:49-64; grid_volume from vol1d/vol2d/vol3d
 * (src/vec.cpp:904-931).  Vacuum, no PML until set below. */
mnl_structure *mnl_structure_create(int dim, const int n[3], double a, double courant,
                                    const int io[3]);
void mnl_structure_destroy(mnl_structure *s);

/* pml(thickness, d, side, Rasymptotic, mean_stretch) with the quadratic
 * profile -- src/structure.cpp:285-301, applied per chunk by
 * structure_chunk::use_pml (src/structure.cpp:661-691). */
int mnl_structure_add_pml(mnl_structure *s, int dir, int side, double thickness,
                          double R_asymptotic, double mean_stretch);

/* structure_chunk::set_chi1inv row (src/anisotropic_averaging.cpp:211-298)
 * for E component comp (epsilon) or H component comp (mu: structure::set_mu,
 * src/structure.cpp) and direction dir; host array in the layout above
 * (values at every point, ghosts included).  Off-diagonal entries are
 * accepted but only their presence/zeros enter the arithmetic, exactly as in
 * the fork (src/step_generic.cpp:631-633, 730-760; the H update always takes
 * the diagonal branch). NULL resets to trivial. */
int mnl_structure_set_chi1inv(mnl_structure *s, int comp, int dir, const double *host);
/* structure_chunk::set_chi2 / set_chi3 (src/structure.cpp:795-866).  chi3 is
 * inert in the fork (src/step_generic.cpp:829-886) and only recorded. */
int mnl_structure_set_chi2(mnl_structure *s, int comp, const double *host);
int mnl_structure_set_chi3(mnl_structure *s, int comp, const double *host);
/* structure::set_conductivity(c, C) (src/structure.cpp:425-437, chunk part
 * 868-905): conductivity of D or B component comp (an E / H component names
 * its D / B array; E values are multiplied by the diagonal chi1inv set so
 * far, as the reference does).  Enters step_curl's conductivity branches
 * (src/step_generic.cpp:89-229) with cndinv = 1/(1 + cnd dt/2)
 * (src/structure.cpp:693-707) and scales current sources by cndinv
 * (src/step.cpp:300-309).  NULL resets to zero. */
int mnl_structure_set_conductivity(mnl_structure *s, int comp, const double *host);
/* structure::add_susceptibility(sigma, E_stuff, lorentzian_susceptibility(
 * omega0, gamma, drude)) -- src/anisotropic_averaging.cpp:300-372, isotropic
 * (diagonal sigma per E component; NULL = 0). */
int mnl_structure_add_lorentzian(mnl_structure *s, double omega0, double gamma, int drude,
                                 const double *sigma_x, const double *sigma_y,
                                 const double *sigma_z);
/* add_susceptibility with a sigma tensor (src/anisotropic_averaging.cpp:
 * 300-372): sigma[3*c + d] = row of E component c, column d (NULL = 0), at
 * c's Yee points -- the reference samples the off-diagonal entries half a pixel
 * back along c (334-341), the caller does the same.  Off-diagonal entries
 * enter update_P's 2x2 / 3x3 branches (src/susceptibility.cpp:185-250) per
 * reference chunk. */
int mnl_structure_add_lorentzian_tensor(mnl_structure *s, double omega0, double gamma, int drude,
                                        const double *const sigma[9]);
/* structure::add_susceptibility(sigma, H_stuff, lorentzian_susceptibility(omega0,
 * gamma, drude)) (src/anisotropic_averaging.cpp:300-372): a magnetic Lorentzian / Drude
 * susceptibility, diagonal sigma per H component at its Yee points (NULL = 0), updated
 * by update_pols(H_stuff) after update_eh(H_stuff) (src/step.cpp:75-92).  At most 2. */
int mnl_structure_add_magnetic_lorentzian(mnl_structure *s, double omega0, double gamma,
                                          int drude, const double *sigma_x,
                                          const double *sigma_y, const double *sigma_z);
/* Nonlinear E update: 0 = the fork (chi2 through Newton-Raphson where the
 * 3x3 chi1inv is present, chi3 inert; default), 1 = upstream Meep (chi2/chi3
 * through the Pade approximant calc_nonlinear_u, src/step_generic.cpp:546-553,
 * on every E point including PML; diagonal chi1inv only).  Pinned by the
 * reference's python/tests/test_3rd_harm_1d.py golden harmonics. */
int mnl_structure_set_nonlinear_mode(mnl_structure *s, int mode);
/* Fill chi1inv/chi2/Lorentz-sigma of axis-aligned boxes on the device (fast
 * setup for large grids; same values as passing 1/eps(loc) arrays with
 * eps_averaging=False).  box = {xmin,xmax,ymin,ymax,zmin,zmax} in length
 * units; later boxes win.  kind: 0 = epsilon (value = eps), 1 = chi2,
 * 2 = chi3, 3 = Lorentz sigma of susceptibility #index. */
int mnl_structure_set_box(mnl_structure *s, int kind, int index, const double box[6],
                          double value);
/* structure::set_epsilon(material_function &eps, bool use_anisotropic_averaging,
 * double tol, int maxeval) (src/meep.hpp:841, src/structure.cpp:397-401) ->
 * structure_chunk::set_chi1inv (src/anisotropic_averaging.cpp:221-298) with the
 * default material_function::eff_chi1inv_row / normal_vector subpixel averaging
 * (58-219), for a material function given as geometric objects of isotropic
 * permittivity (later objects win, `default_eps` elsewhere), computed on HIP
 * device `device`.  objs: nobj records of MNL_GEO_STRIDE doubles
 * {kind, eps, cx, cy, cz, p0, p1, p2}: kind 0 = block (p = size, |r - c| <= p/2),
 * 1 = sphere (p0 = radius), 2 = cylinder (p0 = radius, p1 = height, p2 = axis
 * 0/1/2).  Coordinates of absent dimensions are 0.  use_averaging = 0 gives
 * 1/eps at each pixel centre (the reference's maxeval = 0 path).  Replaces every
 * chi1inv row of the E components (trivial rows dropped). */
#define MNL_GEO_STRIDE 8
int mnl_structure_set_epsilon_geometry(mnl_structure *s, int device, int nobj,
                                       const double *objs, double default_eps,
                                       int use_averaging, double tol, int maxeval);
/* Copy chi1inv[comp][dir] (whole cell, canonical layout) to host; returns 1
 * (nothing copied) when the row is trivial / absent. */
int mnl_structure_get_chi1inv(mnl_structure *s, int comp, int dir, double *host);
/* The unit-sphere quadrature of src/sphere-quad.cpp (the reference's generated
 * sphere-quad.h) for dim 1/2/3: writes {x, y, z, weight} per point if xyzw is
 * non-null, returns the number of points (2, 12, 50).  Host only. */
int mnl_sphere_quadrature(int dim, double *xyzw);

/* ---- fields (replaces meep::fields, src/meep.hpp:1731-2330) -------------- */

/* fields(structure*) + use_real_fields() (src/fields.cpp:32-89, 144-156) on
 * HIP device `device` (-1 = current).  Real fields only. */
mnl_fields *mnl_fields_create(mnl_structure *s, int device);
/* Distributed variant: one process per GPU, z-slab (3-D) / y-slab (2-D)
 * decomposition of the global grid described by `s` (every rank passes the
 * same global structure).  nccl_id: 128-byte RCCL unique id from rank 0
 * (mnl_comm_unique_id), shared by the caller (e.g. torch.distributed). */
mnl_fields *mnl_fields_create_dist(mnl_structure *s, int device, int rank, int nranks,
                                   const void *nccl_id);
int mnl_comm_unique_id(void *out128);
/* IPC transport id (one process per slab, several processes sharing one GPU --
 * RCCL refuses duplicate devices): creates a POSIX shared-memory control block
 * for `nranks` ranks and writes its 128-byte id; pass it to
 * mnl_fields_create_dist in place of the RCCL id.  Replaces the reference's
 * comms_manager (src/mympi.cpp:87-151) with a process-shared barrier plus
 * IPC-exported device staging buffers. */
int mnl_comm_ipc_id(void *out128, int nranks);
/* Remove the shared-memory name of an IPC id that will not be used (the first
 * init on rank 0 removes it otherwise; mapped segments stay valid). */
int mnl_comm_ipc_unlink(const void *id128);
/* Host-only collective over a fresh IPC group (no GPU call): every rank passes
 * the same id; on return host[0..n) holds the rank-order sum over ranks and the
 * return value is 0 on every rank, or -1 on every rank if any rank passed
 * ok = 0 (the status agreement the data collectives use before they start). */
int mnl_comm_ipc_reduce(const void *id128, int rank, int nranks, double *host, int n, int ok);
/* Transport of a fields object: "single", "rccl", "ipc" or "local". */
const char *mnl_fields_transport(mnl_fields *f);
/* One-rank RCCL self test on `device`: grouped ncclSend/ncclRecv to self of n
 * doubles plus an ncclAllReduce, through the same Comm wrappers the slab
 * exchange uses.  Returns 0 when the data arrived intact. */
int mnl_comm_rccl_selftest(int device, int n);
/* Cells [lo, hi) of the slab axis owned by `rank` (host-only helper). */
int mnl_slab_range(int ncell, int rank, int nranks, int *lo, int *hi);
/* Several slabs of one grid in ONE process on one device (one host thread per
 * slab calling mnl_fields_step concurrently): same decomposition and exchange
 * code as mnl_fields_create_dist, transport = device copies + host barriers.
 * Used to validate the multi-GPU path on a single MI355X. */
void *mnl_local_hub_create(int nranks);
void mnl_local_hub_destroy(void *hub);
mnl_fields *mnl_fields_create_local(mnl_structure *s, int device, int rank, int nranks,
                                    void *hub);
void mnl_fields_destroy(mnl_fields *f);

/* add_volume_source(c, src_time, volume(p,p), amp) for a point p
 * (src/sources.cpp:455-494, weights: src/loop_in_chunks.cpp:263-500).
 * kind GAUSSIAN: params = {freq, width, start_time, end_time} ->
 *   gaussian_src_time(f, w, st, et) (src/sources.cpp:85-96).
 * kind CONTINUOUS: params = {freq_re, freq_im, width, start, end, slowness}
 *   -> continuous_src_time (src/meep.hpp:1038-1056, src/sources.cpp:121-141).
 * is_integrated: dipole (E = eps^-1 (D - P_src)) vs current (D -= J dt)
 * (src/update_eh.cpp:136-146, src/step.cpp:296-319). */
int mnl_fields_add_point_source(mnl_fields *f, int comp, int kind, const double *params,
                                int nparams, const double pos[3], double amp_re, double amp_im,
                                int is_integrated);
/* add_point_source with custom_src_time(func, data, start, end) (src/meep.hpp:
 * 1059-1092; Python CustomSource, python/source.py:338-400): dipole(t) =
 * func(t) for float(t) in [float(start), float(end)], else 0; current = dipole
 * unless is_integrated (then the finite difference of the dipole).  func is
 * called on the host thread that steps the fields. */
int mnl_fields_add_custom_point_source(mnl_fields *f, int comp, mnl_src_func func, void *data,
                                       double start_time, double end_time, const double pos[3],
                                       double amp_re, double amp_im, int is_integrated);
/* fields::add_volume_source(c, src_time, volume(vmin, vmax), A, amp)
 * (src/sources.cpp:455-494, src_vol_chunkloop 243-312): every owned point of
 * component comp's grid in the volume gets the loop_in_chunks weight (linear
 * interpolation at the faces, per reference chunk) times amp times A(r - centre)
 * (afunc NULL: A = 1); zero-width directions scale amp by the resolution (J as
 * a delta function); a volume up to one pixel wider than the cell is clamped,
 * wider fails ("Source width > cell width").  kind / params as
 * mnl_fields_add_point_source (not CUSTOM).  Integrated (dipole) volume sources
 * have no point limit (sorted device arrays, binary search per reader). */
int mnl_fields_add_volume_source(mnl_fields *f, int comp, int kind, const double *params, int np,
                                 const double vmin[3], const double vmax[3], double amp_re,
                                 double amp_im, int is_integrated, mnl_amp_func afunc,
                                 void *adata);
int mnl_fields_add_custom_volume_source(mnl_fields *f, int comp, mnl_src_func func, void *data,
                                        double start_time, double end_time, const double vmin[3],
                                        const double vmax[3], double amp_re, double amp_im,
                                        int is_integrated, mnl_amp_func afunc, void *adata);
/* fields::require_component (src/fields.cpp:566-586). */
int mnl_fields_require_component(mnl_fields *f, int comp);
/* fields::step() x nsteps (src/step.cpp:35-140).  Collective for
 * distributed fields.  NaN/Inf check of the D energy density at the cell
 * centre (src/step.cpp:138-139) every `every` steps, counted across calls (default
 * 100): fails with "meep: simulation fields are NaN or Inf". */
int mnl_fields_step(mnl_fields *f, int nsteps);
/* No reference counterpart (tuning knobs of this implementation).  Times, over real steps
 * (one warm-up and `reps` timed steps per candidate): (1) the tile kernel's z-chunk length
 * (automatic, 16, 20, 24, 32, 48; skipped with MNL_FUSED_ZCHUNK set), (2) on one rank with
 * polarization chunks, the CUs of their general kernel running beside the tile kernel
 * (0 and five splits around the balanced one; skipped with MNL_TILE_GEN_CUS set), and keeps
 * the fastest; with temporal blocking also the planes of the two-step
 * items (automatic, 32, 48, 64, 96, 128) and pairs vs one-step stepping.  Each candidate: two warm-up steps, reps (rounded up to even) timed.  Advances the
 * fields by at most 2 + 19 * (2 + reps) steps, with results
 * identical to plain stepping.  *zchunk = the length kept (0 = automatic), *gen_cus = the
 * CUs kept (0 = one launch after the other); -1 = not tuned (not in the fused tile mode:
 * at most 2 steps taken). */
int mnl_fields_tune(mnl_fields *f, int reps, int *zchunk, int *gen_cus);
int mnl_fields_set_nan_check(mnl_fields *f, int every);
/* Field energy over the box [vmin, vmax] (NULL, NULL: the whole cell,
 * user_volume.surroundings()), src/energy_and_flux.cpp:48-178:
 * which 0 = electric_energy_in_box (sum over E comps of 1/2 integral E.D),
 * 1 = magnetic_energy_in_box (1/2 integral H.B with the current B, H),
 * 2 = field_energy_in_box (electric + magnetic of B, H synchronized to E's
 * time: one extra B half step averaged in and restored).  Integration on each
 * component's Yee grid with loop_in_chunks weights; device reduction
 * (compensated), per reference chunk.  Collective. */
int mnl_fields_energy_in_box(mnl_fields *f, int which, const double vmin[3], const double vmax[3],
                             double *out);
/* fields::initialize_field(c, func) (src/initialize.cpp:135-161) with the
 * function evaluated by the caller: host = real part of func at every point of
 * component c in the whole-cell layout (n >= cell size).  Adds it to the
 * field, zeroes the metallic walls, exchanges ghosts; for D / B components also
 * updates E / H from them, as the reference does.  Collective. */
int mnl_fields_initialize_field(mnl_fields *f, int comp, const double *host, size_t n);
/* t (timesteps) and dt; time() = t*dt, round_time() = float(t*dt)
 * (src/meep.hpp:1891-1892). */
int mnl_fields_time(mnl_fields *f, long long *t, double *dt);
/* fields::t = t (the Python binding's fields.t assignment, python/simulation.py
 * restart_fields). */
int mnl_fields_set_time(mnl_fields *f, long long t);
/* fields::zero_fields (src/fields.cpp:638-664): all field / auxiliary arrays and the
 * polarizations to 0 (DFT accumulators kept). */
int mnl_fields_zero_fields(mnl_fields *f);
/* fields::remove_sources (src/fields.cpp:601-610). */
int mnl_fields_remove_sources(mnl_fields *f);
/* fields::get_field(c, vec) with 8-point interpolation
 * (src/monitor.cpp:127-160, src/vec.cpp:558-621).  Distributed: every rank
 * returns the global value (sum over ranks, as get_field(..., parallel=true)). */
int mnl_fields_get_field(mnl_fields *f, int comp, const double pos[3], double *out);
/* Copy the whole-cell array of a component (layout above, ghosts = 0 as in
 * the reference) into a caller-owned buffer of n doubles; H components read
 * B where H==B (src/fields.cpp:493-517).  Distributed: only rank-owned planes
 * are filled, the rest is 0 (sum over ranks gives the global array). */
int mnl_fields_copy_component(mnl_fields *f, int comp, double *host, size_t n);
/* fields::get_array_slice(volume, c) (src/array_slice.cpp:611-704, with
 * comp = MNL_DIELECTRIC / MNL_PERMEABILITY: src/array_slice.cpp:385-408, the
 * Dielectric / Permeability slices of Simulation.get_epsilon / get_mu;
 * get_array_slice_dimensions 447-507): the component on the Centered grid
 * points of the volume [vmin, vmax] (average of its Yee neighbours), empty
 * dimensions interpolated and collapsed (snap = 0) or snapped to the
 * nearest grid point (snap = 1, src/loop_in_chunks.cpp:275-287).  *rank / dims[3]: the
 * kept directions in X,Y,Z order; out (nout doubles, row-major) may be NULL to
 * query the size.  Collective for distributed fields (every rank gets the
 * whole slice). */
int mnl_fields_array_slice(mnl_fields *f, int comp, const double vmin[3], const double vmax[3],
                           int snap, int *rank, long long dims[3], double *out, long long nout);
/* Number of entries of the whole-cell array of comp. */
size_t mnl_fields_ntot(mnl_fields *f);
/* Per-sub-step GPU time in ms accumulated since creation (time_sink
 * FieldUpdateB/H/D/E, BoundarySteppingB/H, src/meep.hpp:1610-1633);
 * out[6]. */
int mnl_fields_timers(mnl_fields *f, double out[6]);
/* Time sinks in the reference's enum order (meep::time_sink,
 * src/meep.hpp:1610-1633; print_times labels src/time.cpp:28-51). */
enum {
  MNL_SINK_CONNECTING, MNL_SINK_STEPPING, MNL_SINK_BOUNDARIES, MNL_SINK_MPI_ALL,
  MNL_SINK_MPI_ONE, MNL_SINK_FIELD_OUTPUT, MNL_SINK_FOURIER, MNL_SINK_MPB,
  MNL_SINK_FARFIELDS, MNL_SINK_OTHER, MNL_SINK_UPDATE_B, MNL_SINK_UPDATE_H,
  MNL_SINK_UPDATE_D, MNL_SINK_UPDATE_E, MNL_SINK_BSTEP_B, MNL_SINK_BSTEP_WH,
  MNL_SINK_BSTEP_PH, MNL_SINK_BSTEP_H, MNL_SINK_BSTEP_D, MNL_SINK_BSTEP_WE,
  MNL_SINK_BSTEP_PE, MNL_SINK_BSTEP_E, MNL_NUM_TIME_SINKS
};
/* fields::get_time_spent_on for every sink of this rank, seconds (replaces
 * src/time.cpp:136-139 / timing_data_vector): wall time of mnl_fields_step
 * goes to "time stepping" except, with profiling on, the GPU time of the
 * unfused update kernels (B/H/D/E), halo exchanges ("copying boundaries")
 * and DFT updates ("Fourier transforming"); collectives of slices / energies
 * / fluxes / get_field to "all-all communication".  out[MNL_NUM_TIME_SINKS]. */
int mnl_fields_time_spent(mnl_fields *f, double *out);
/* fields::reset_timers (src/time.cpp:124-128). */
int mnl_fields_reset_timers(mnl_fields *f);
/* sum_to_all over the ranks of distributed fields (in place, n doubles);
 * a no-op on one rank.  Collective. */
int mnl_fields_allreduce(mnl_fields *f, double *v, int n);
/* meep::verbosity (default 1).  At > 0 rank 0 prints "on time step N
 * (time=T), S s/step" at most every 4 s of stepping (src/step.cpp:49-56). */
void mnl_set_verbosity(int level);
int mnl_get_verbosity(void);
/* Newton-Raphson attempts that fell back to random seeds (never in the
 * reference runs recorded in SURVEY.md; counted instead of printed). */
int mnl_fields_nr_fallbacks(mnl_fields *f, long long *count);
/* Algorithmic bytes per owned cell per step of this configuration
 * (DESIGN.md "Roofline") and owned cells of this rank. */
int mnl_fields_traffic_model(mnl_fields *f, double *bytes_per_cell_step, double *owned_cells);
/* Allow (1, default) or forbid (0) the fused single-pass interior kernel
 * (used automatically for 3-D non-dispersive, non-NR configurations without
 * magnetic or integrated sources).  Results are identical either way. */
int mnl_fields_set_fused(mnl_fields *f, int allow);
/* bit 0: the last step ran the fused interior kernel; bit 1: it read chi1inv
 * through the palette (DESIGN.md "chi1inv palette"); bit 2: field arrays are
 * requested physically contiguous; bit 4: the fused step ran as the single tile
 * kernel (lean + PML bodies); bits 8-15: how many
 * contiguity requests the driver could not satisfy (plain allocations instead). */
int mnl_fields_mode(mnl_fields *f, int *fused);
/* Enable HIP-event timing around every sub-step kernel group (on the stream
 * the kernels run on) and reset the accumulated timers. */
int mnl_fields_set_profiling(mnl_fields *f, int on);
/* Accumulated launches / total ms of the dominant interior kernel since the
 * last mnl_fields_set_profiling, and its algorithmic bytes per launch.
 * which = 0: fused step kernel (fused mode) or curl B = step_db(B_stuff);
 * which = 1: curl D = step_db(D_stuff) (unfused mode);
 * which = 2: general fused kernel (PML / boundary tiles);
 * which = 3: the DFT updates of one step (all flux objects);
 * which = 4: the E update (update_eh(E_stuff): chi(2) Newton-Raphson,
 *            Lorentzian P), unfused mode; bytes 0 (not HBM-bound);
 * which = 5: temporal blocking: launches = pairs of
 *            steps, total_ms = every launch of the pairs, bytes per pair;
 * which = 6: rim launches that run alone (one step each). */
int mnl_fields_kernel_stats(mnl_fields *f, int which, long long *launches, double *total_ms,
                            double *bytes_per_launch);
/* Temporal blocking (no reference counterpart: how this build steps pairs of
 * fields::step(), src/step.cpp:35-140).  out[0..n) of:
 * active (1: the current fused geometry steps pairs), own cells of the two-step
 * items, border points (upper bound), own cells of mixed-palette two-step items,
 * rim cells, mixed-palette rim cells, two-step items, rim items, planes of the
 * first two-step item (the longest), narrow x-face strip items among the rim items,
 * enabled (pairs allowed: set_temporal_blocking / MNL_TB / the tuner), the two-step chunk
 * setting (0: automatic), the most own columns of a two-step item (124 unless set or tuned),
 * polarization chunks stepped inside the pairs (1), interior two-step items (their two-step
 * footprint meets no rim box; one rank runs them beside the previous pair's second rim
 * launch). */
int mnl_fields_tb_info(mnl_fields *f, double *out, int n);
/* Allow (1, the default; MNL_TB=0 at creation turns it off) or forbid (0) stepping
 * pairs of steps with the two-step kernel.  Results are identical either way. */
int mnl_fields_set_temporal_blocking(mnl_fields *f, int on);
/* Scheduling options of the fused step (no reference counterpart; an option only changes how
 * the same per-point arithmetic is scheduled, results are identical): which = 0 the narrow
 * x-face strip body of the temporal-blocking rim (MNL_TB_NARROW; the pair plan is rebuilt at
 * the next step), 1 DFT sampling plans with chi1inv as palette bytes (MNL_DFT_PAL; the plans
 * are rebuilt at the next update), 2 / 3 / 4 the CUs the pair launches / the two-step launch /
 * the rim launches leave free (value = a count, -1 the default; MNL_TB_RES), 5 pairs sample DFT
 * monitors from the two-step kernel's compact boxes (MNL_DFT_CMP; the pair plan is rebuilt),
 * 6 planes per rim item of a pair (value; 0 = the one-step chunk length), 7 the chi(2) NR box's
 * E phase beside the tile kernel (MNL_NR_EARLY), 8 planes per two-step item (value; 0 =
 * automatic; MNL_TB_ZCHUNK), 9 the most own columns of a two-step item (value 4..124; 0 = 124,
 * the widest the kernel's 128 columns of lanes hold), 10 columns per lane of the two-step kernel
 * (2; 1 = the round-5 kernel; MNL_TB_PX), 11 pairs of steps with polarization chunks (1, the
 * default; MNL_TB_POL), 12 the first rim launch's items other than the narrow x-face strips on a
 * side stream beside the two-step kernel (1, the default; one rank; MNL_TB_R1A), 13 the
 * interior two-step items on a third stream beside the previous pair's second rim launch (1;
 * 0, the default: measured slower at 512^3; one rank, no DFT monitors;
 * MNL_TB_LINT), 14 the second rim launch's item order (1 longest first, 2 narrow strips
 * first; 0, the default: the first launch's order, narrow strips last, measured faster; one
 * rank; MNL_TB_R2LPT), 15 planes per narrow x-face strip item of the rim (value; 0 = the rim's
 * chunk length; MNL_TB_STRIP_ZCHUNK), 16 a pair's step sources and NaN guard in one launch (1,
 * the default; one rank; MNL_TB_SRCGUARD).  For in-process A/B measurements
 * (tools/ab_inproc.py). */
int mnl_fields_set_schedule(mnl_fields *f, int which, int value);

/* ---- checkpoint (src/fields_dump.cpp, src/structure_dump.cpp) -----------
 * fields::dump / fields::load (src/fields_dump.cpp:108-145, 232-270): t and
 * every per-point state array of the rank (f, f_u, f_w, f_cond, and also the
 * polarizations and DFT accumulators), flat binary, not HDF5 (no HDF5 in this
 * build).  Distributed fields write one file per rank (filename.rank<r>).
 * load() needs fields built the same way (same structure, decomposition,
 * sources, flux objects) and resumes bit for bit.  structure dump/load
 * (structure::dump / load, src/structure_dump.cpp) save the host-side
 * material description; load before creating fields. */
int mnl_fields_dump(mnl_fields *f, const char *filename);
int mnl_fields_load(mnl_fields *f, const char *filename);
int mnl_structure_dump(mnl_structure *s, const char *filename);
int mnl_structure_load(mnl_structure *s, const char *filename);

/* ---- DFT flux (src/dft.cpp; meep.hpp dft_flux) --------------------------
 * fields::add_dft_flux (src/dft.cpp:578-640) for a volume_list: regions =
 * nreg x {min x,y,z, max x,y,z, direction (0..2), weight}, nfreq frequencies
 * (not angular), decimation 0 = the reference's automatic choice
 * (src/dft.cpp:195-216).  The DFT is accumulated on the device after every
 * decimated step (fields::update_dfts, src/dft.cpp:249-263); *handle gets the
 * flux object's index. */
int mnl_fields_add_dft_flux(mnl_fields *f, int nreg, const double *regions, const double *freqs,
                            int nfreq, int decimation, int *handle);
/* dft_flux::flux (src/dft.cpp:533-547), summed over ranks: out[nfreq]. */
int mnl_fields_dft_flux(mnl_fields *f, int handle, double *out);
/* Complex DFT values per list (which 0: E, 1: H), list order (next_in_dft),
 * point-major then frequency, re/im interleaved: *n = points * nfreq. */
int mnl_fields_dft_size(mnl_fields *f, int handle, long long *n);
/* out[2 * n]; points another rank owns read 0 (sum over ranks to assemble). */
int mnl_fields_dft_data(mnl_fields *f, int handle, int which, double *out, long long n);
/* the decimation factor the object was created with */
int mnl_fields_dft_decimation(mnl_fields *f, int handle, int *decimation);
/* Accumulate every buffered DFT update now and wait for the device (no reference
 * counterpart: the reference adds each update to the DFT array in fields::update_dfts,
 * src/dft.cpp:249-263; this build samples every update and adds up to 32 of them per pass
 * over the array, in the same order, so the values are bitwise the same).  Every reader of
 * DFT values (flux, data, get_dft_array, dump) flushes by itself; buffered updates carry over
 * between step calls.  For timing: a timed region that includes the accumulation of its own
 * updates ends with this call. */
int mnl_fields_dft_flush(mnl_fields *f);
/* fields::add_dft_fields(components, ncomp, volume(vmin, vmax), freq, Nfreq,
 * use_centered_grid = !yee_grid, decimation_factor) (src/dft.cpp:889-903; Python
 * Simulation.add_dft_fields, python/simulation.py:2976-3036): E / H components
 * (MNL_EX..MNL_HZ), accumulated on the device with the flux objects' kernels.
 * *handle is shared with the flux handles (mnl_fields_dft_data, _decimation). */
int mnl_fields_add_dft_fields(mnl_fields *f, int ncomp, const int *comps, const double vmin[3],
                              const double vmax[3], const double *freqs, int nfreq, int yee_grid,
                              int decimation, int *handle);
/* fields::get_dft_array(dft_fields or dft_flux, c, num_freq) (src/dft.cpp:1240-1280,
 * process_dft_component 908-1240, collapse_array src/array_slice.cpp:554-601): the
 * complex DFT of component comp at frequency index num_freq over the object's volume,
 * empty dimensions collapsed, summed over ranks.  *rank and dims[0..rank-1] (row-major,
 * X before Y before Z); out (2*nout doubles, re/im interleaved) may be NULL to query the
 * size.  rank 0 means the object holds no chunk of comp (no values). */
int mnl_fields_dft_array(mnl_fields *f, int handle, int comp, int num_freq, int *rank,
                         long long dims[3], double *out, long long nout);

#ifdef __cplusplus
}
#endif
#endif
