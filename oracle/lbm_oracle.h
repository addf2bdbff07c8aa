/*
 * lbm_oracle.h -- CPU restatement of the reference D3Q19 BGK hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (liblbm.so, liblbm_host.so,
 * the case drivers) links, includes or calls this code.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only
 * as the checker / the timed serial CPU baseline.
 *
 * It restates, in plain serial C, the algorithm of
 *   /root/reference/Lid_driven_cavity/ldc.cu     (update 57-371, boundary_stream 373-458,
 *                                                  geo_pre 468-502, initialize 504-580)
 *   /root/reference/Poiseulle_flow/Poiseulle.cu  (geo_pre 52-255, index_transform 257-271,
 *                                                  initialize 273-382, update 384-583,
 *                                                  boundary_stream 585-893)
 *   /root/reference/bifurcation/bifurcation.cu   (geo_pre 36-253, read_vel 255-327,
 *                                                  initialize 329-427, update 429-637,
 *                                                  boundary_stream 639-1023, calc_res 1158-1175)
 * keeping the reference's two-pass structure (collide+pull pass, then a separate
 * boundary pass that writes bounce-back and non-equilibrium-extrapolation values
 * into boundary cells), its expression trees, and its fp32 evaluation order.
 * Build with -ffp-contract=off (see oracle/Makefile).
 *
 * Pinning: see oracle/PINNING.md.  The reference is CUDA-only and cannot be
 * built in this image (no nvcc; hipcc rejects <direct.h> and texture refs), so
 * field-level parity against a reference binary is UNPINNED; the oracle is pinned
 * by the reference's own known answers (thesis NLATTICE 65820, the shipped
 * geo.txt/bc.txt), by analytic Poiseuille flow, and cross-checked against the
 * emulation-probe numbers recorded in SURVEY.md.
 *
 * Storage: raster x-fastest, c = x + nx*(y + ny*z); populations SoA f[q*ncell + c].
 */
#ifndef LBM_ORACLE_H
#define LBM_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_LDC = 0, ORC_POISEUILLE = 1, ORC_MASK = 2, ORC_GENERIC = 3 };

/* Generic non-equilibrium-extrapolation boundary code (the coronary case's scheme,
 * coronary.cu:716-944, generalised to any face): for a cell with this code and every q with
 * e_q pointing to the fluid side (face: 0 +x, 1 -x, 2 +y, 3 -y, 4 +z, 5 -z),
 *   f_q(B) = feq_q(rho_bc, u_bc) + (f_q(B + e_q) - feq_q(rho_nb, u_nb)) (1 - 1/tau)
 * kind 0: u_bc = u, rho_bc = rho_nb;  1: u_bc = u, rho_bc = rho;  2: rho_bc = rho, u_bc = u_nb.
 * table (nullable) replaces u[face axis] per cell: x faces [z][y], y faces [z][x], z faces [y][x]. */
typedef struct {
    int code, face, kind;
    float rho, u[3];
    const float* table;
} orc_bc;
/* LDC wall bounce-back ordering: the reference (ldc.cu:184-201 vs 204-313) races. */
enum { ORC_LDC_TWO_PHASE = 0,   /* all wall writes before any fluid read (race-free) */
       ORC_LDC_SERIAL_EMU = 1 }; /* serial emulation order: blocks z,y,x; threads y,x; koff 7..0 */

typedef struct orc_lbm orc_lbm;

/* ---- geometry builders (reference geo_pre), raster int8 reference codes ---- */
void orc_geo_ldc(int nx, int ny, int nz, int8_t* geo);                      /* ldc.cu:468-502 */
void orc_geo_poiseuille(int nx, int ny, int nz, int8_t* geo);               /* Poiseulle.cu:52-255 */
void orc_geo_mask(int nx, int ny, int nz, const int32_t* raw, int8_t* geo); /* bifurcation.cu:36-253 */
int  orc_read_geo_txt(const char* path, int n, int32_t* raw);               /* bifurcation.cu:50-60 */
int  orc_read_geo_txt_zxy(const char* path, int nx, int ny, int nz, int32_t* raw); /* coronary.cu:45-56 */
/* coronary.cu:31-275 with its five hard-coded ends as a table: ends[7e..7e+6] =
 * {axis 0|2, plane, lo0, hi0, lo1, hi1, passes} (see lbm_oracle.c) */
void orc_geo_coronary(int nx, int ny, int nz, const int32_t* raw, int n_ends, const int* ends, int8_t* geo);
/* bifurcation.cu:255-327: fills inlet (y=1, geo==2) and outlet (y=ny-2, geo==3) uy tables,
 * skipping `skip_blocks` nx*nz blocks first (1 = the "inlet = block 1" variant). Returns tokens read. */
int  orc_read_bc_txt(const char* path, int nx, int ny, int nz, const int8_t* geo, int skip_blocks,
                     float* inlet_uy, float* outlet_uy);
/* Poiseulle.cu:257-271: compact ids in z,y,x raster over geo != 0. Returns NLATTICE. */
int  orc_index_transform(int nx, int ny, int nz, const int8_t* geo, int32_t* index);

/* ---- solver ---- */
orc_lbm* orc_create(int case_kind, int nx, int ny, int nz, const int8_t* geo, float tau,
                    int ldc_order, const float* inlet_uy, const float* outlet_uy);
/* ORC_GENERIC: 4 fluid, 1 wall (post-collision bounce-back as Poiseulle.cu:601-746), the
 * listed boundary codes (at most 16), everything else unstored. */
orc_lbm* orc_create_generic(int nx, int ny, int nz, const int8_t* geo, float tau, const orc_bc* bcs, int nbc);
void orc_destroy(orc_lbm* o);
/* coronary.cu:277-350: the coronary case's own initial state (after orc_create_generic) */
void orc_initialize_coronary(orc_lbm* o);
/* the update kernel's equilibrium (Poiseulle.cu:561-580 expression trees) */
void orc_feq(float rho, float ux, float uy, float uz, float* feq19);
/* the boundary-value equilibrium of the NEE "tmp" terms (fp32 throughout) */
void orc_feq_bc(float rho, float ux, float uy, float uz, float* feq19);
/* reference initialize(): LDC wi-form (ldc.cu:504-580) / expanded form (Poiseulle.cu:273-382,
 * bifurcation.cu:329-427), with each case's initial rho/u rules. */
void orc_initialize(orc_lbm* o);
/* Run n steps; residual_hist (nullable, n floats) gets the reference residual of each step. */
void orc_step(orc_lbm* o, int n, float* residual_hist);
/* Run the reference convergence loop (ldc.cu:653-685): returns final k. */
int  orc_run_converge(orc_lbm* o, int max_it, int stag_max, float tol, float* last_residual);
int  orc_steps_done(const orc_lbm* o);
/* raster copies; macros are the last step's d_rho/d_ux/d_uy/d_uz (0 where never written) */
void orc_get_macros(const orc_lbm* o, float* rho, float* ux, float* uy, float* uz);
void orc_get_f(const orc_lbm* o, float* f);        /* current source buffer, SoA [19][ncell] */
void orc_set_f(orc_lbm* o, const float* f);        /* into both buffers */
long orc_bad_reads(const orc_lbm* o);               /* fluid pulls from geo-0 (unstored) cells */
/* host residual of bifurcation.cu:1158-1175 on the current macros (long double sum, as double) */
double orc_calc_res_bif(const orc_lbm* o);
/* the reference's per-step residual sum (thrust::reduce emulated serially in fp32 over the
 * reference storage order, ldc.cu:660-662) of the current macros */
float orc_velsum(const orc_lbm* o);
/* residual sum mode: 0 (default) thrust's fp32 sum emulated serially in the reference storage
 * order; 1 the fp32 |u| terms summed in fp64 (liblbm's S), for stop-step comparisons */
void orc_set_residual_fp64(orc_lbm* o, int on);
/* residual sum modes (orc_set_residual_mode) */
enum { ORC_SUM_SERIAL = 0, ORC_SUM_FP64 = 1, ORC_SUM_CUB_TREE = 2 };
/* ORC_SUM_CUB_TREE: thrust::reduce's CUB two-pass fp32 tree over the terms in reference storage
 * order, with 256-thread blocks, ipt items per thread loaded vec wide, at most grid_cap blocks
 * (see orc_cub_reduce); returns 0, or -1 for bad parameters */
int orc_set_residual_mode(orc_lbm* o, int mode, int ipt, int vec, int grid_cap);
float orc_cub_reduce(const float* v, long n, int ipt, int vec, int grid_cap);

#ifdef __cplusplus
}
#endif
#endif
