/* mnl_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference fields::step() hot path (PMack10/meep_nl,
 * src/step.cpp:35-140) used as the parity checker for the HIP product path.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library.  Nothing under meep_nl_amd/ links or calls it.
 *
 * Parity pinning: see oracle/mnl_oracle.cpp header and DESIGN.md section
 * "Oracle".  The grid, component numbering and the canonical host layout
 * (Z fastest, (n+1) points per present direction, src/vec.cpp:482-494) are
 * the same as include/meep_nl_amd.h so that arrays compare element-wise.
 */
#ifndef MNL_ORACLE_H
#define MNL_ORACLE_H
#include <stddef.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_sim orc_sim;

const char *orc_last_error(void);
orc_sim *orc_new(int dim, const int n[3], double a, double courant, const int io[3]);
void orc_free(orc_sim *s);
int orc_add_pml(orc_sim *s, int dir, int side, double thickness, double R, double mean_stretch);
int orc_set_chi1inv(orc_sim *s, int comp, int dir, const double *arr);
int orc_set_chi2(orc_sim *s, int comp, const double *arr);
int orc_set_chi3(orc_sim *s, int comp, const double *arr);
/* structure::set_conductivity (src/structure.cpp:868-905); D/B (or E/H) comp */
int orc_set_conductivity(orc_sim *s, int comp, const double *arr);
int orc_add_lorentzian(orc_sim *s, double omega0, double gamma, int drude, const double *sx,
                       const double *sy, const double *sz);
/* sigma tensor: sig[3*c + d] (row of E comp c, column d; NULL = 0) */
int orc_add_lorentzian_tensor(orc_sim *s, double omega0, double gamma, int drude,
                              const double *const sig[9]);
/* add_susceptibility(sigma, ft, lorentzian) with ft 0 = E_stuff, 1 = H_stuff
 * (magnetic: diagonal sigma only, at the H components' points). */
int orc_add_susceptibility(orc_sim *s, int ft, double omega0, double gamma, int drude,
                           const double *const sig[9]);
int orc_add_point_source(orc_sim *s, int comp, int kind, const double *params, int nparams,
                         const double pos[3], double amp_re, double amp_im, int is_integrated);
int orc_add_custom_point_source(orc_sim *s, int comp,
                                void (*func)(double, void *, double *, double *), void *data,
                                double start_time, double end_time, const double pos[3],
                                double amp_re, double amp_im, int is_integrated);
/* fields::add_volume_source(c, src, volume(vmin, vmax), A, amp) (src/sources.cpp:
 * 455-494); afunc (NULL = 1) gets the position relative to the volume centre */
int orc_add_volume_source(orc_sim *s, int comp, int kind, const double *params, int nparams,
                          const double vmin[3], const double vmax[3], double amp_re, double amp_im,
                          int is_integrated,
                          void (*afunc)(const double *, void *, double *, double *), void *adata);
int orc_add_custom_volume_source(orc_sim *s, int comp,
                                 void (*func)(double, void *, double *, double *), void *data,
                                 double start_time, double end_time, const double vmin[3],
                                 const double vmax[3], double amp_re, double amp_im,
                                 int is_integrated,
                                 void (*afunc)(const double *, void *, double *, double *),
                                 void *adata);
int orc_require_component(orc_sim *s, int comp);
/* fields::initialize_field (src/initialize.cpp:135-161), func's real values as a
 * whole-cell array */
int orc_initialize_field(orc_sim *s, int comp, const double *vals);
int orc_step(orc_sim *s, int nsteps);
int orc_get_field(orc_sim *s, int comp, const double pos[3], double *out);
int orc_copy_component(orc_sim *s, int comp, double *out, size_t n);
int orc_set_threads(int nthreads);
/* upstream Meep chi2/chi3 update (Pade, src/step_generic.cpp:546-553 and the
 * branches the fork comments out) instead of the fork's NR / inert chi3 */
int orc_set_upstream_nl(orc_sim *s, int on);
/* fields::get_array_slice(volume, c) (src/array_slice.cpp): *rank and the
 * collapsed dims[3]; out (nout doubles, row-major over the kept directions
 * in X,Y,Z order) may be NULL to query the size only. */
int orc_array_slice(orc_sim *s, int c, const double vmin[3], const double vmax[3], int snap,
                    int *rank, long long dims[3], double *out, long long nout);
/* fields::electric_energy_in_box (which 0), magnetic_energy_in_box (1),
 * field_energy_in_box (2, synchronized B / H) over [vmin, vmax] (NULL: the
 * whole cell), src/energy_and_flux.cpp:48-178 */
int orc_energy_in_box(orc_sim *s, int which, const double vmin[3], const double vmax[3],
                      double *out);
long long orc_t(orc_sim *s);
double orc_dt(orc_sim *s);
size_t orc_ntot(orc_sim *s);
long long orc_nr_failures(orc_sim *s);
/* DFT flux (fields::add_dft_flux, src/dft.cpp:578-640): regions = nreg x
 * {min x,y,z, max x,y,z, direction, weight}; returns a handle >= 0. */
int orc_add_dft_flux(orc_sim *s, int nreg, const double *regions, const double *freqs, int nfreq,
                     int decimation);
int orc_dft_flux(orc_sim *s, int h, double *out);
long long orc_dft_size(orc_sim *s, int h);
int orc_dft_data(orc_sim *s, int h, int which, double *out, long long n);
int orc_dft_decimation(orc_sim *s, int h);
/* DFT fields (fields::add_dft_fields, src/dft.cpp:889-903): E / H components over
 * [wmin, wmax], centered grid or (yee_grid) each component's own grid. */
int orc_add_dft_fields(orc_sim *s, int ncomp, const int *comps, const double wmin[3],
                       const double wmax[3], const double *freqs, int nfreq, int yee_grid,
                       int decimation);
/* fields::get_dft_array(obj, c, num_freq) (src/dft.cpp:1240-1280) for flux and
 * fields objects: re/im interleaved, empty dimensions collapsed; out NULL = size query */
int orc_dft_array(orc_sim *s, int h, int c, int num_freq, int *rank, long long dims[3],
                  double *out, long long nout);

/* Subpixel averaging (src/anisotropic_averaging.cpp:58-298) over geometric
 * objects {kind, eps, cx, cy, cz, p0, p1, p2} (see mnl_structure_set_epsilon_geometry):
 * rows of E comp `comp` over the canonical grid (NULL = skip). */
int orc_eps_average(int dim, const int n[3], const int io[3], double a, int comp, int nobj,
                    const double *objs, double default_eps, int use_averaging, double tol,
                    int maxeval, double *out0, double *out1, double *out2);
int orc_sphere_quadrature(int dim, double *xyzw);

#ifdef __cplusplus
}
#endif
#endif
