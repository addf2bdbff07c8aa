/*
 * lbm.h -- C ABI of liblbm.so, the MI355X-native D3Q19 BGK collide+stream hot path.
 *
 * This is the drop-in boundary for the reference's per-case kernel-launch interface.
 * The reference has no library API: each case's main() launches, per time step,
 *
 *   update<<<>>>(NLATTICE, d_geo, d_scr, d_dst, d_ux, d_uy, d_uz, d_rho, tau)
 *                          ldc.cu:57, Poiseulle.cu:384 (geo/index via textures 49-50),
 *                          bifurcation.cu:429 (tau hard-coded 434)
 *   boundary_stream<<<>>>(NLATTICE, d_geo, d_dst, d_ux, d_uy, d_uz, d_rho, tau, C_U)
 *                          ldc.cu:373, Poiseulle.cu:585, bifurcation.cu:639
 *   calc_vel_square<<<>>>(d_velsum, d_ux, d_uy, d_uz, NLATTICE) + thrust::reduce
 *                          ldc.cu:460-466,660-662, Poiseulle.cu:895-901,993-996
 *   d_scr <-> d_dst pointer swap
 *                          ldc.cu:664-666
 *
 * and owns the buffers itself (cudaMalloc/cudaMemcpy in main, ldc.cu:635-650).  Here
 * one opaque context owns the device buffers of one lattice (or one z-slab of it),
 * and lbm_step() performs all of the above for n steps: a fused pull-stream +
 * collide kernel with wall bounce-back and non-equilibrium-extrapolation
 * boundaries evaluated by mask and stored by each boundary slot's fluid neighbour
 * right after its collision (producer side), a fused |u| reduction, a
 * device-side residual/convergence finisher, and (for slabs) the +-z halo exchange
 * over RCCL.  All pointers in these signatures are plain host pointers; no HIP or
 * torch types cross the boundary.  Every function returns LBM_OK (0) or a negative
 * status; lbm_last_error() gives the message.  One context per host thread at a
 * time; contexts are not re-entrant.
 */
#ifndef LBM_H
#define LBM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LBM_OK 0
#define LBM_ERR_ARG -1
#define LBM_ERR_HIP -2
#define LBM_ERR_RCCL -3
#define LBM_ERR_STATE -4
#define LBM_ERR_GEOMETRY -5

/* Which reference case supplies the meaning of the mask codes (README.md:9-14). */
typedef enum {
  LBM_CASE_LDC = 0,        /* ldc.cu: 0 ghost, 1 wall (bounce-back already at step 0),
                              2 moving lid (velocity NEE, -y face), 3 fluid */
  LBM_CASE_POISEUILLE = 1, /* Poiseulle.cu: -1 ghost, 0 unused, 1 wall, 2 inlet (velocity NEE,
                              +y face), 3 outlet (velocity NEE, -y face), 4 fluid */
  LBM_CASE_MASK = 2,       /* bifurcation.cu: as Poiseuille but 3 = pressure outlet (rho = 1,
                              u = u of the fluid neighbour) */
  LBM_CASE_GENERIC = 3     /* 4 fluid, 1 wall, boundary codes from lbm_desc.bc_codes (any face and
                              kind, e.g. coronary.cu:716-944's +-x inlet/outlet and -z outlets);
                              every other code is passive */
} lbm_case_kind;

/* Which side of a boundary cell its fluid neighbour lies on.  The boundary supplies the
 * populations q with e_q pointing into the fluid (e_q . n = +1 along the face's axis):
 * LDC lid at y = ny-2 over fluid at y = ny-3 -> LBM_FACE_NY (q = 4, 8, 10, 16, 18). */
typedef enum { LBM_FACE_PX = 0, LBM_FACE_NX = 1, LBM_FACE_PY = 2, LBM_FACE_NY = 3, LBM_FACE_PZ = 4,
               LBM_FACE_NZ = 5 } lbm_face;

/* Non-equilibrium extrapolation: f_q(B) = feq_q(rho_bc, u_bc) + (f_q(F) - feq_q(rho_F, u_F)) (1 - 1/tau)
 * with F = B + e_q the fluid neighbour, its post-collision f_q and its (rho, u) of the same step
 * (boundary_stream, ldc.cu:391-456).  F -- the only cell that pulls slot q of B -- stores the
 * value itself right after its collision. */
typedef enum {
  LBM_BC_VELOCITY = 0,      /* u_bc given, rho_bc = rho_F (LDC lid, Poiseuille, bifurcation inlet,
                               coronary outlets coronary.cu:795-943) */
  LBM_BC_VELOCITY_RHO = 1,  /* u_bc and rho_bc given (coronary inlet, rho_bc = 1, coronary.cu:716-794) */
  LBM_BC_PRESSURE = 2       /* rho_bc given, u_bc = u_F (bifurcation outlet, bifurcation.cu:877-948) */
} lbm_bc_kind;

typedef struct {
  int code;                 /* mask value of the boundary cells (2, 3, 5..127) */
  int face;                 /* lbm_face */
  int kind;                 /* lbm_bc_kind */
  float rho;                /* rho_bc (LBM_BC_VELOCITY_RHO, LBM_BC_PRESSURE) */
  float u[3];               /* u_bc (velocity kinds) */
  /* Nullable per-cell profile replacing u[axis of face]: raster over the face's two other axes
   * (x faces [nz_global][ny], y faces [nz_global][nx], z faces [ny][nx]; global z).  Copied at
   * lbm_create. */
  const float* u_normal_table;
} lbm_bc_code;
/* Boundary data are static for a context's lifetime: the (rho_bc, u_bc) of every NEE cell --
 * lid speed, inlet/outlet tables, bc_codes -- is fixed by lbm_create.  No entry point changes
 * them later. */

/* Equilibrium expression used to initialise f (the two forms of the reference). */
typedef enum {
  LBM_INIT_LDC_WI = 0,     /* ldc.cu:553-571: rho*w_q*(1 + 3 e.u + 4.5 (e.u)^2 - 1.5 u^2) */
  LBM_INIT_EXPANDED = 1    /* Poiseulle.cu:354-372 / bifurcation.cu:399-417: update-kernel form */
} lbm_init_form;

typedef struct lbm_ctx lbm_ctx;

typedef struct {
  int nx, ny, nz;          /* extent of this context's lattice (its slab when nz_global > nz) */
  float tau;               /* BGK relaxation time (ldc.cu:55, Poiseulle.cu:39, bifurcation.cu:434) */
  int case_kind;           /* lbm_case_kind */
  /* Reference mask codes, raster x fastest then y then z (int8).  Planes: nz, or nz + 2 when
   * halo_planes = 1 (plane 0 = global z_offset-1, plane nz+1 = global z_offset+nz).  NULL with
   * LBM_CASE_LDC: the cavity box of ldc.cu:468-502 is generated on the device from global
   * coordinates (used for the multi-GB benchmark lattices). */
  const int8_t* geo;
  int halo_planes;
  float lid_u;             /* LDC lid speed along +z (ldc.cu:52: 0.15f / C_U) */
  const float* bc_inlet_uy;  /* nx * nz_global floats, x fastest: u_y imposed on code-2 cells (nullable) */
  const float* bc_outlet_uy; /* nx * nz_global floats: u_y on code-3 cells (LBM_CASE_POISEUILLE) */
  int device;              /* HIP device ordinal */
  int z_offset;            /* global z of local plane 0 */
  int nz_global;           /* global z extent (== nz for a single-domain run) */
  /* Row alignment of the device layout: 1..4 = store the cell at row position p (x, or y with
   * row_axis 2) in slot p - (x_align - 1) of its row; 0 = choose it from geo so that most rows
   * start their fluid run on a 4-cell boundary.  Slabs of one lattice must use the same value
   * (lbm_attach_rccl / lbm_group_step check). */
  int x_align;
  /* LBM_CASE_GENERIC: the boundary codes (at most 16; copied at lbm_create). */
  const lbm_bc_code* bc_codes;
  int n_bc_codes;
  /* LBM_CASE_MASK with geo == NULL: the raw geo.txt mask (values 0..255, raster x fastest, one
   * byte per cell); geo_pre (bifurcation.cu:63-239: wall/fluid erosion, inlet/outlet rows,
   * ghost marking) runs on the device and the codes never exist on the host.  Planes: nz, or
   * nz + 6 with halo_planes = 1 (global z_offset-3 .. z_offset+nz+2; planes outside the global
   * box are never read).  Requires ny >= 5. */
  const uint8_t* mask;
  /* Axis the device layout's rows (the contiguous, 4-cells-per-lane direction) run along:
   * 1 = x, 2 = y, 0 = choose -- y when that leaves >= 3% fewer 256-cell chunks holding fluid
   * (a pipe along y, Poiseulle.cu / bifurcation.cu, fills whole rows), x for the
   * device-generated cavity and for slabs (nz_global != nz: give every slab the same value).
   * Results are bit-identical for every choice; only addresses change. */
  int row_axis;
} lbm_desc;

/* Checkpoint / resume (not in the reference, whose VTK output cannot restart a run; SURVEY.md
 * section 5): the context's complete state -- both population buffers in the device layout
 * (NEE values included), the step count and the convergence state -- to a file,
 * and back into a context created with the same descriptor (extent, slab, case, tau and
 * layout are checked; LBM_ERR_ARG otherwise).  A resumed run continues bit for bit.  Slab
 * contexts save and load one file per rank (ghost planes included).  The file (format version 3)
 * records whether the saving context bounced back on the consumer side (its wall slots were not
 * written); a context that bounces back on the producer side restores them on load, so a file
 * moves between the two modes (e.g. a one-cell device cavity and its LBM_TUNE_BOX = 1 twin).
 * A load that fails after the header checks (a truncated file) leaves the state unspecified. */
int lbm_checkpoint_save(lbm_ctx* ctx, const char* path);
int lbm_checkpoint_load(lbm_ctx* ctx, const char* path);

/* Status / version */
const char* lbm_version(void);
const char* lbm_last_error(const lbm_ctx* ctx); /* NULL ctx: last creation error */

/* Process-wide tuning knobs (not a reference interface: A/B measurement and test switches;
 * the defaults are the measured best).  Read when a context is created (ROW_AXIS,
 * CELLS_PER_LANE, EXACT_DIV, FUSED_RESIDUAL, BUFFER_ALLOC, GRID_STRIDE).  Returns the previous
 * value, or LBM_ERR_ARG for an unknown knob / value.  Fields (populations, rho, u) are
 * bit-identical for every setting; the residual's fp64 |u| sum is accumulated per launch block,
 * so launch-shape knobs (CELLS_PER_LANE, GRID_STRIDE, FUSED_RESIDUAL) can change its last bits
 * and with them, rarely, the step a convergence-controlled run stops at.  The default shape also
 * follows the device's CU count (grid-stride block counts) and the lattice's sparsity, so that
 * stop step is reproducible run to run on one GPU model, not across models.  A stop step that
 * must not depend on the device: lbm_set_residual_order(LBM_SUM_CUB_TREE, ...), whose terms are
 * summed in storage order by a fixed tree, whatever the launch shape. */
typedef enum {
  LBM_TUNE_ROW_AXIS = 0,        /* stands in for lbm_desc.row_axis = 0: 0 choose, 1 x, 2 y */
  LBM_TUNE_CELLS_PER_LANE = 1,  /* step kernel: 0 by size, 1 one cell per lane, 4 four */
  LBM_TUNE_EXACT_DIV = 2,       /* 1: the compiler's division by tau everywhere */
  LBM_TUNE_FUSED_RESIDUAL = 3,  /* 1 (default): the residual rides in the next step's launch */
  LBM_TUNE_BUFFER_ALLOC = 4,    /* population buffers: 0 (default) of the four fastest-writing of
                                   up to 64 allocations (lbm_buffer_placement), the pair whose
                                   tile copies both ways take the least time together; 1 the first
                                   two allocations; 2 the two fastest-writing (round 4) */
  LBM_TUNE_SYNC_TIMEOUT_S = 5,  /* RCCL contexts: a wait (lbm_sync, synchronising lbm_step, read-
                                   outs) longer than this many seconds aborts the communicator
                                   and fails with LBM_ERR_RCCL; 0 (default): no limit.  A peer's
                                   asynchronous RCCL error always aborts promptly. */
  LBM_TUNE_GRID_STRIDE = 6,    /* 4-cell step kernel: 0 (default) by sparsity -- group lists
                                   (LBM_TUNE_GROUPS) loop with 4 blocks per CU, chunk lists with 2
                                   when the chunks' lanes are under 3/4 busy, else one chunk per
                                   wave; 1 one chunk (or list slice) per wave; B = 2..8 the loop
                                   with at most B blocks per CU (sparse lists only) */
  LBM_TUNE_INJECT_RCCL_FAULT = 7, /* reserved (was a process-wide fault-injection hook; now per
                                   context: lbm_debug_fail_next_wait); only 0 is accepted */
  LBM_TUNE_GROUPS = 8,          /* sparse chunk lists: 0 (default) compact lists of the active 4-cell
                                   groups when the chunks' lanes (one cell per lane: cells) are under
                                   3/4 busy, 1 never, 2 on every sparse list.  With CELLS_PER_LANE 0
                                   a list of at most 8192 x 64 groups runs one cell per lane (16
                                   groups per wave), a longer one four (64 per wave) */
  LBM_TUNE_GROUP_SEGMENT = 9,   /* group lists: 1..64 groups per segment (default 16: two 128-B lines);
                                   a segment with an active group enters the list whole, its idle
                                   groups load nothing */
  LBM_TUNE_COMPACT = 10,        /* storage of single-domain lattices whose step takes group lists
                                   (vessel trees): 0 (default) compact rows -- every storage row keeps
                                   only the span of its stored cells, packed in storage order (the
                                   reference's index_transform, Poiseulle.cu:257-271, per row); 1 the
                                   dense box; 2 compact rows whenever the range takes group lists
                                   (LBM_TUNE_GROUPS 2 included) */
  LBM_TUNE_BOX = 11,            /* the device-generated cavity (geo == NULL, LBM_CASE_LDC) with a
                                   power-of-two row pitch and plane: 0 (default) the step kernels
                                   compute cell types and wall links from coordinates, and its
                                   one-cell single-domain range bounces back on the consumer side;
                                   1 they load them like any lattice's */
  LBM_TUNE_NEE_FIX = 12,        /* NEE values of a single-domain 4-cell range whose chunk waves collide
                                   its NEE-adjacent cells (the pipe's rows along y): 0 (default) and
                                   1 NEE blocks in the step launch re-pull and re-collide every
                                   NEE-adjacent cell; 3 one small launch after the step kernel
                                   (k_nee_fix) stores them from the cells' (rho, u) the chunk waves
                                   recorded and their own post-collision slots (round 5's default);
                                   2 NEE records -- a chunk wave computes them after its relaxation
                                   into a 32-B record per cell, and the next step's wave puts them
                                   into its pulls (chunk lists of the dense box with at most 8 such
                                   cells per chunk; otherwise as 3) */
  LBM_TUNE_XCD_RUN = 13,        /* order of the step kernel's chunk workgroups over the 8 XCDs: 0
                                   (default) runs of eight (L = 4) for 4-cell chunk lists whose rows
                                   run along y (the pipe), runs of four (L = 3) for compact one-cell
                                   ranges of several rounds of waves (vessel trees), one contiguous
                                   eighth of the chunks per XCD elsewhere; L = 1..16 runs of 2^(L-1) workgroups, XCD x taking
                                   runs x, x + 8, x + 16, ...; 17 one eighth per XCD everywhere */
  LBM_TUNE_NEE_ORDER = 14,      /* dispatch order of the NEE blocks in the step launch: 0 (default) after
                                   the chunk blocks for grid-stride group lists, before them elsewhere;
                                   1 before; 2 after.  Results are bit-identical (the partial slots
                                   keep their order) */
  LBM_TUNE_COUNT = 15
} lbm_tune_knob;
int lbm_tune(int knob, int value);

/* Lifecycle */
int lbm_create(const lbm_desc* desc, lbm_ctx** out);
void lbm_destroy(lbm_ctx* ctx);

/* Initial state.  rho/ux/uy/uz are nx*ny*nz raster arrays (nullable: rho=1, u=0); the
 * equilibrium is evaluated on the device with the chosen reference expression into both
 * population buffers, bit-identical to the reference initialize(). */
int lbm_init_equilibrium(lbm_ctx* ctx, int form, const float* rho, const float* ux,
                         const float* uy, const float* uz);
/* LDC initial state of ldc.cu:504-580 generated on the device (no host arrays). */
int lbm_init_ldc(lbm_ctx* ctx);
/* The case's own initialize() on the device, no host arrays: LBM_CASE_LDC as lbm_init_ldc;
 * LBM_CASE_MASK as bifurcation.cu:329-427 (rho = 1, u = 0, u_y of code-2 cells in row y = 1
 * and code-3 cells in row y = ny-2 from bc_inlet_uy / bc_outlet_uy, expanded equilibrium).
 * Other cases: LBM_ERR_ARG. */
int lbm_init_case(lbm_ctx* ctx);
/* Exact initial populations, SoA [19][nz][ny][nx] (into both buffers); resets the step count. */
int lbm_set_f(lbm_ctx* ctx, const float* f_soa);

/* Summation order of the residual's S = sum |u| (ldc.cu:460-466, 660-668).  The reference sums
 * the fp32 terms with thrust::reduce, CUB's two-pass device reduction, whose tree shape depends
 * on its CUDA/CUB version and GPU (not recorded by the reference); the stop step of a
 * convergence-controlled run depends on that order (oracle/PINNING.md section 3).
 *   LBM_SUM_FP64 (default): the fp32 terms summed in fp64 in a fixed order -- no slower than the
 *     step itself (the sum rides in the next step's launch).
 *   LBM_SUM_CUB_TREE: the terms in the reference's storage order (LDC: 8x8x8 bricks over the
 *     brick-padded box, ldc.cu:71; otherwise index_transform's compact z, y, x order), summed in
 *     fp32 by CUB's tree: blocks of 256 threads, items_per_thread items per thread loaded vec
 *     wide (a multiple), at most grid_cap blocks (e.g. 16, 4, 240: CUB's sm_60 policy on the
 *     thesis's 6-SM GTX 1050 Ti), 32-lane warp shuffle trees -- bit-identical to the oracle's
 *     orc_cub_reduce.  Two extra launches per step (one re-reads the step's populations).
 * Single-domain contexts only (LBM_ERR_ARG otherwise); vec and grid_cap are ignored for FP64. */
typedef enum { LBM_SUM_FP64 = 0, LBM_SUM_CUB_TREE = 1 } lbm_sum_order;
int lbm_set_residual_order(lbm_ctx* ctx, int mode, int items_per_thread, int vec, int grid_cap);

/* Convergence control of the reference main loop (ldc.cu:653-685): when enabled, a device
 * flag stops stepping once !(k <= max_it && tol_count <= stag_max); further steps are no-ops. */
int lbm_set_convergence(lbm_ctx* ctx, int enabled, int max_it, int stag_max, float tol);

/* Run n steps.  residual_hist (nullable, n floats) receives |S_k - S_{k-1}| / S_k per step,
 * S = sum over cells of |u| (ldc.cu:660-668); when it is non-NULL, or steps_done is non-NULL,
 * the call synchronises.  Otherwise the work is only enqueued (see lbm_sync). */
int lbm_step(lbm_ctx* ctx, int nsteps, float* residual_hist, int* steps_done);
int lbm_sync(lbm_ctx* ctx);

/* Convergence state: k (steps executed), tol_count, stopped flag (1 converged / max_it,
 * 2 stopped because the |u| sum became non-finite), last residual, last S. */
int lbm_get_state(lbm_ctx* ctx, int* k, int* tol_count, int* stopped, float* residual, double* velsum);
/* NaN guard: *k = the first step whose |u| sum was not finite (0: none so far).  Recorded with
 * or without convergence control; under convergence control the run also stops there. */
int lbm_get_nonfinite(lbm_ctx* ctx, int* k);

/* Macroscopic fields of the last step, raster nx*ny*nz; 0 off-fluid (nullable outputs).  The
 * step kernels store no macros: the first read-out after stepping recomputes them on the
 * device from the last step's source buffer (the same pulls and sums, so the same bits). */
int lbm_get_macros(lbm_ctx* ctx, float* rho, float* ux, float* uy, float* uz);
/* Verification digest of the last step's fields, one uint64 per local plane: the wrapping sum
 * over the plane's fluid cells of a 64-bit hash of (global x, y, z, bits of rho, ux, uy, uz).
 * Independent of layout and slab decomposition, so the digests of z-slabs of a lattice equal
 * the matching planes' digests of the single-domain run when the fields are bit-identical --
 * a size-independent check at lattice sizes whose fields are too large to copy to the host. */
int lbm_field_digest(lbm_ctx* ctx, uint64_t* plane_digest);
/* Populations of the last step (the next step's source), SoA [19][nz][ny][nx]; only fluid
 * cells carry reference-defined values.  A boundary (NEE) cell also holds, in each slot q its
 * fluid neighbour B + e_q pulls, that neighbour's NEE value; its other slots, and wall cells'
 * slots where bounce-back is on the consumer side, are unspecified. */
int lbm_get_f(lbm_ctx* ctx, float* f_soa);
/* The reference mask codes this context runs on (geo_pre's output: 0 unused, -1 ghost, 1 wall,
 * 2 inlet, 3 outlet / lid, 4 or 3 fluid ...), raster nx*ny*nz over the local planes -- the
 * device-built codes of a mask or LDC context, the ingested ones otherwise. */
int lbm_get_geo(lbm_ctx* ctx, int8_t* geo);

/* Sizes: cells in the box, fluid cells, and the bytes one step moves algorithmically
 * (152 B per fluid cell: 19 fp32 loads + 19 fp32 stores). */
int lbm_get_counts(lbm_ctx* ctx, int64_t* n_box, int64_t* n_fluid, double* algo_bytes_per_step);

/* Kernel timing: enabled = 1: HIP events bracket every step-kernel launch on the stream it
 * runs on; lbm_stats returns the summed kernel milliseconds and launch count since enabling.
 * enabled = 2 (spans): no per-launch events (each costs a small launch ~2 us), but one event pair
 * around all the work each lbm_step call enqueues, on the compute stream: lbm_kernel_times kind 7
 * returns their milliseconds and the steps they cover -- the device time per step of every kernel
 * of a step (the step kernel, k_nee_fix, the reductions), which cannot exceed the wall time.
 * 0 disables.  Enabling resets the sums. */
int lbm_profile(lbm_ctx* ctx, int enabled);
int lbm_stats(lbm_ctx* ctx, double* kernel_ms, int64_t* launches, double* algo_bytes);
/* The same for one kind of launch: kind 0 = the step kernel (k_step: stream-collide with
 * bounce-back and NEE values stored producer-side, one launch per step and launch range); kinds 1 / 2 =
 * those of its launches that read population buffer 0 / 1 (the A-B parity); slabs with RCCL:
 * 3 = the edge-plane launches, 4 = the interior launches, 5 = the halo exchange on the
 * communication stream (pack, send/recv, unpack), 6 = how long each step's halo outlasted its
 * interior launch (clipped at 0: the part of the exchange not hidden; launches = steps);
 * 7 = lbm_profile(ctx, 2)'s spans (launches = the steps the lbm_step calls asked for). */
int lbm_kernel_times(lbm_ctx* ctx, int kind, double* ms, int64_t* launches);
/* Arithmetic of the relaxation's division by tau (the reference divides, ldc.cu:326-363):
 * fast_div = 1 when the 3-instruction correctly rounded quotient is in use (tau verified
 * exhaustively at lbm_create; lbm_tune(LBM_TUNE_EXACT_DIV, 1) before lbm_create forces the
 * compiler's division).  A wave whose populations leave the quotient's proven domain (|f| outside
 * [2^-60, 2^40) or |u| >= 2^10, e.g. a diverging run) relaxes with the exact division
 * instead (a wave-uniform branch in the same launch); retried_chunks counts those 256-cell
 * chunk waves since creation.  Results are bit-identical either way. */
int lbm_get_numerics(lbm_ctx* ctx, int* fast_div, int64_t* retried_chunks);
/* Placement of the two population buffers (not a reference interface).  HBM write bandwidth
 * differs between allocations (~5.5 vs ~6.4 TB/s for 10-GB buffers on MI355X, stable per
 * allocation); when a buffer is larger than 256 MB (the MALL) and the device has room,
 * lbm_create allocates up to 64 candidates, times one full-buffer write sweep of each and, of the
 * four fastest, keeps the pair whose tile copies both ways take the least time together
 * (LBM_TUNE_BUFFER_ALLOC).  The candidates are held together for the duration of the probe:
 * lbm_create may TRANSIENTLY allocate up to 160 GiB of device memory (sixteen 10.2-GB
 * candidates at 512^3, 64 of 1.28 GB at 256^3), never more than three quarters of the memory
 * free when it starts; the rest is freed before it returns (lbm_get_setup_cost reports the low
 * point).  gbs[0..cap) receives the
 * candidates' rates (GB/s) in allocation order, *n their count (0: buffers of at most 256 MB,
 * or compact rows, not probed), chosen[2] the indices kept.  Nullable outputs. */
int lbm_buffer_placement(lbm_ctx* ctx, double* gbs, int cap, int* n, int* chosen);
/* The device layout lbm_create chose (lbm_desc.row_axis / x_align resolved): row_axis 1 = x,
 * 2 = y; pitch = row slots; x_align 1..4; active_chunks = 256-cell chunks k_step launches a
 * wave for (those holding fluid).  Nullable outputs. */
int lbm_get_layout(lbm_ctx* ctx, int* row_axis, int* pitch, int* x_align, int64_t* active_chunks);
/* How the step kernel covers the whole-domain chunks (not a reference interface: diagnostics
 * for benchmarks and tests): cells_per_lane 1 or 4, main_blocks = its chunk workgroups,
 * grid_stride 1 when those loop over their XCD's chunks (LBM_TUNE_GRID_STRIDE), 2 when its
 * waves take compact lists of active 4-cell groups (LBM_TUNE_GROUPS; 64 groups per wave with
 * four cells per lane, 16 with one), 3 when one-cell waves take consecutive cells of compact
 * rows (LBM_TUNE_COMPACT; no list); lane_fill = mean share of chunk lanes (one cell per lane:
 * of the chunks' cells; with groups: of a listed group's cells; compact rows without a list:
 * of the waves' cells) with a cell to update.
 * Nullable outputs. */
int lbm_get_launch_shape(lbm_ctx* ctx, int* cells_per_lane, int* main_blocks, int* grid_stride, double* lane_fill);
/* Fluid cells next to a non-equilibrium-extrapolation boundary (each stores its NEE
 * neighbours' values, producer side). */
int lbm_get_boundary_cells(lbm_ctx* ctx, int64_t* n_boundary);
/* How the whole-domain step produces its NEE values (diagnostics, LBM_TUNE_NEE_FIX): path 0 = in
 * the one-cell waves (or no NEE cell), 1 = NEE blocks in the step launch, 2 = k_nee_fix after it
 * from (rho, u) records the chunk waves store, one 16-B slot per NEE-adjacent cell, 3 = NEE
 * records carried into the next step's pulls; max_records = the most records one chunk holds
 * (path 3; at most 8).  Nullable outputs. */
int lbm_get_nee_path(lbm_ctx* ctx, int* path, int* max_records);
/* What lbm_create cost (not a reference interface): create_s = its wall seconds (buffer
 * placement included); device_bytes = the device memory the context holds after it, and
 * peak_bytes = the most it held during it (the placement candidates), both as the drops in
 * hipMemGetInfo's free memory since its start (so other users of the device in the meantime
 * count too).  Nullable outputs. */
int lbm_get_setup_cost(lbm_ctx* ctx, double* create_s, int64_t* device_bytes, int64_t* peak_bytes);
/* Population storage (not a reference interface): compact = 1 when the lattice is stored in
 * compact rows (LBM_TUNE_COMPACT), cells = cell slots per population buffer (the padded box, or
 * the compact rows' spans), bytes = both population buffers' device bytes.  Nullable outputs. */
int lbm_get_storage(lbm_ctx* ctx, int* compact, int64_t* cells, int64_t* bytes);

/* Measurement helper (not a reference interface): the HBM rate a plain streaming copy
 * reaches on this device, for context next to k_step's roofline fraction.  Copies `bytes`
 * (rounded down to 64 KiB) between two device buffers with 16-B loads and stores in a few
 * shapes (grid-stride or one contiguous region per XCD, plain or non-temporal, k_step's own:
 * one wave per 16-KB tile with all 16 loads per lane in flight, and that tile by LDS-DMA), `reps` timed
 * launches each (HIP events, after one untimed launch); *gbs = the best (read + write bytes) /
 * duration in GB/s.  The two buffers are picked as the population buffers are
 * (lbm_buffer_placement): of up to 64 allocations of `bytes`, the pair among the four
 * fastest-writing whose tile copies both ways take the least time together. */
int lbm_probe_stream(int device, int64_t bytes, int reps, double* gbs);
/* The same, per copy shape: gbs_shape[i] = the best rate of shape i for i < min(cap, n);
 * *n = the number of shapes (grid-stride / per-XCD-region copies, k_step's 16-KB wave tiles by
 * plain or non-temporal 16-B loads, the same tiles by LDS-DMA, global_load_lds). */
int lbm_probe_stream_shapes(int device, int64_t bytes, int reps, double* gbs_shape, int cap, int* n);

/* Multi-GPU z-slabs (one process per GPU).  Rank 0 calls lbm_rccl_unique_id, the 128 bytes
 * are broadcast by the caller (e.g. torch.distributed), then every rank attaches.  After
 * attaching, lbm_step exchanges the 5 populations crossing each +-z face every step over
 * RCCL on a communication stream, overlapped with the interior update, and all-reduces the
 * residual sum. */
int lbm_rccl_unique_id(uint8_t out_id[128]);
/* A context in compact rows (a sparse single-domain lattice, lbm_get_storage; LBM_TUNE_COMPACT)
 * cannot attach: LBM_ERR_STATE (create it with LBM_TUNE_COMPACT = 1, or as slabs).  Steps taken
 * before attaching may have bounced back on the consumer side; attaching first restores the wall
 * slots of both population buffers, so read-outs and further steps continue bit for bit. */
int lbm_attach_rccl(lbm_ctx* ctx, const uint8_t id[128], int rank, int nranks);
/* rank and communicator size as RCCL reports them (ncclCommCount); 0 / 1 without RCCL.
 * A communicator aborted by a failed peer or a timed-out wait stays failed: from then on
 * lbm_step, lbm_sync, every read-out, lbm_checkpoint_save and lbm_comm_info return
 * LBM_ERR_RCCL (the slab's ghost planes and residual are stale); destroy the context. */
int lbm_comm_info(lbm_ctx* ctx, int* rank, int* nranks);
/* Test hook (not a reference interface): the next wait of THIS context (lbm_sync, a
 * synchronising lbm_step, a read-out) sees a failed peer, which exercises the abort path above.
 * Only contexts with an RCCL communicator wait that way (LBM_ERR_STATE otherwise). */
int lbm_debug_fail_next_wait(lbm_ctx* ctx);
/* Test hook (not a reference interface): a quiet NaN into all 19 slots of every wall cell of both
 * population buffers.  Where bounce-back is on the consumer side no step after the first reads a
 * wall slot, so the fields go on bit for bit; where it is on the producer side the next step
 * pulls the NaNs. */
int lbm_debug_poison_walls(lbm_ctx* ctx);

/* Single-device loopback decomposition (test and debug path): n contexts, each a z-slab of
 * one lattice on the same device, stepped together with device-to-device halo copies. */
int lbm_group_step(lbm_ctx** ctxs, int n, int nsteps, float* residual_hist);

#ifdef __cplusplus
}
#endif
#endif /* LBM_H */
