/*
 * lbm_host.h -- C ABI of liblbm_host.so: the host side of the per-case API that the
 * reference keeps inside each case's .cu file (geometry ingest, boundary tables,
 * initial fields and output).  Plain C++, no device code; used by the case drivers
 * (the drivers in lattice-boltzmann-method-gpu_amd/host) and by the Python bindings.
 *
 * All arrays are raster, x fastest, then y, then z ("[nz][ny][nx]").  Boundary tables
 * are [nz][nx].
 */
#ifndef LBM_HOST_H
#define LBM_HOST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* geo_pre of the three cases: reference mask codes (README.md:9-14) */
void lbmh_geo_ldc(int nx, int ny, int nz, int8_t* geo);                      /* ldc.cu:468-502 */
void lbmh_geo_poiseuille(int nx, int ny, int nz, int8_t* geo);               /* Poiseulle.cu:52-255 */
void lbmh_geo_mask(int nx, int ny, int nz, const int32_t* raw, int8_t* geo); /* bifurcation.cu:63-239 */
/* geo.txt: nx*ny*nz whitespace-separated ints, z, y, x loop order (bifurcation.cu:50-60).
 * Returns the number of ints read (< 0: cannot open). */
long lbmh_read_geo_txt(const char* path, int nx, int ny, int nz, int32_t* raw);
/* Coronary-style vessel masks (coronary_cfd/coronary.cu:31-275).  geo.txt there is read in
 * z, x, y loop order (coronary.cu:45-56).  Returns the number of ints read (< 0: cannot open). */
long lbmh_read_geo_txt_zxy(const char* path, int nx, int ny, int nz, int32_t* raw);
/* An open end of the vessel (coronary.cu:75-143): the cells of plane `plane` normal to `axis`
 * (0 = x, 2 = z) inside the window [lo0, hi0) x [lo1, hi1) -- axis 0: y then z; axis 2: x then
 * y -- get `passes` increments of the minimum of the raw mask over their four in-plane
 * neighbours.  A cell the 3-D erosion left a wall (1) but whose vessel cross-section continues
 * in the plane becomes code 1 + passes (inlet 2, outlet 3, side exits 5, 6, 7). */
typedef struct {
  int axis, plane, lo0, hi0, lo1, hi1, passes;
} lbmh_end;
/* geo_pre of a vessel mask: fluid = raw + 3 increments of the 6-neighbour minimum over the
 * interior (coronary.cu:58-73), the ends above, then ghost marking of the unused 18-neighbours
 * of every wall (coronary.cu:145-260).  Raster codes -1, 0, 1, 2, 3, 4 and 1 + passes. */
int lbmh_geo_ends(int nx, int ny, int nz, const int32_t* raw, int n_ends, const lbmh_end* ends, int8_t* geo);
/* ^ returns 0, or -1 (geo untouched) for a box under 3^3 or an end whose plane or window leaves
 *   the interior (plane in [1, n-2], windows within [1, n-1)) or whose code 1 + passes > 127 */
/* the reference's five ends for its NX x NY x NZ = 291 x 291 x 372 box (coronary.cu:75-143):
 * inlet x = 3 (one pass: code 2), main exit x = 272 (two: 3), sub-exits z = 185 (four: 5),
 * z = 191 (five: 6), z = 204 (six: 7).  Fills ends[5]; returns 5, or -1 when the box is too
 * small to hold those planes and windows. */
int lbmh_coronary_ends(int nx, int ny, int nz, lbmh_end* ends);
/* bc.txt (bifurcation.cu:294-325): block `inlet_block` is read as the inlet u_y on code-2 cells
 * of the y=1 plane, the next block as the outlet u_y on code-3 cells of y=ny-2 (inlet_block = 0
 * reproduces the shipped code; 1 reads the block that matches the shipped inlet).  geo NULL:
 * the tables are not masked (for lbm_desc.mask contexts, whose lbm_init_case masks by code).
 * Returns the number of tokens consumed (< 0: cannot open). */
long lbmh_read_bc_txt(const char* path, int nx, int ny, int nz, const int8_t* geo, int inlet_block,
                      float* inlet_uy, float* outlet_uy);
/* index_transform (Poiseulle.cu:257-271): compact ids in z,y,x order over geo != 0 (else -1).
 * Returns NLATTICE. */
int64_t lbmh_index_transform(int nx, int ny, int nz, const int8_t* geo, int32_t* index);
/* the Poiseuille kernel's parabola uygt(x, z) (Poiseulle.cu:590,597) as a [nz][nx] table */
void lbmh_poiseuille_profile(int nx, int nz, float u_max, float* table);
/* initial (rho, u) of initialize(): case 0 LDC (ldc.cu:510-532), 1 Poiseuille
 * (Poiseulle.cu:280-341, host u_max = 0.15f/C_U), 2 mask (bifurcation.cu:333-373),
 * 3 coronary (coronary.cu:277-350: code 2 u_x = 0.1745f/C_U, 3 u_x = 0.1f/C_U, 5-7
 * u_z = 0.02f/C_U, C_U = 2.74909090909091f; the table arguments are unused) */
void lbmh_initial_fields(int case_kind, int nx, int ny, int nz, const int8_t* geo, const float* inlet_uy,
                         const float* outlet_uy, float* rho, float* ux, float* uy, float* uz);
/* outputSave (legacy ASCII VTK of u*C_U): ldc.cu:582-610 (case 0), Poiseulle.cu:903-938 (1),
 * bifurcation.cu:1095-1156 (2).  Returns 0 or < 0 when the file cannot be written. */
int lbmh_write_vtk(const char* path, int case_kind, int nx, int ny, int nz, const int8_t* geo,
                   const float* ux, const float* uy, const float* uz, float C_U, float CH);
/* coronary outputSave (coronary.cu:948-1011): DENSITY (rho * C_rho), PRESSURE
 * (rho * C_pre / 3.0, C_pre = C_rho * C_U * C_U in float) and VELOCITY (u * C_U) over
 * x in [1, nx-2], y in [2, ny-3], z in [1, nz-2]; unstored cells print 0. */
int lbmh_write_vtk_coronary(const char* path, int nx, int ny, int nz, const int8_t* geo, const float* rho,
                            const float* ux, const float* uy, const float* uz, float C_U, float CH, float C_rho);
/* calc_res (bifurcation.cu:1158-1175): long-double sum of the fp32 |u|^2 over code >= 4 in
 * the output region x in [1, nx-2], y in [2, ny-3], z in [1, nz-2] */
long double lbmh_calc_res(int nx, int ny, int nz, const int8_t* geo, const float* ux, const float* uy,
                          const float* uz);
/* coronary.cu:1013-1031: the same over code 4 only (codes 5-7 are boundary cells there) */
long double lbmh_calc_res_fluid(int nx, int ny, int nz, const int8_t* geo, const float* ux, const float* uy,
                                const float* uz);

#ifdef __cplusplus
}
#endif
#endif /* LBM_HOST_H */
