// lbm_kernels.hpp -- internal launch interface between the context code (lbm_ctx.hip)
// and the HIP kernels (lbm_kernels.hip).  Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

namespace lbm {

// Cells are numbered linearly over a padded box, x fastest: c = x + y*pitch + zs*plane
// with storage plane zs = local z + 1 (one ghost plane below and above the slab).
// Populations live in AoSoA chunks of 256 consecutive cells -- one wavefront's work
// (64 lanes x 4 cells): [chunk][q][256].  A wave's 19 loads then fall in a handful of
// 19-KB chunk blocks instead of 19 streams 0.5 GB apart, and its 19 stores into one.
constexpr int kChunk = 256;
constexpr int kQ = 19;
constexpr int kBlock = 256;  // 4 wavefronts, one chunk each
// the one-cell kernel over compact rows (vessel trees): 2 wavefronts per workgroup, so that a
// few thousand waves spread evenly over the CUs (interleaved A/B: C4 8.74 -> 8.46 us, coronary
// 37.5 -> 36.0 us; one-wave workgroups halve its residency, profiles/r04_workgroup_size_ab.log)
constexpr int kBlock1c = 128;

__host__ __device__ __forceinline__ int64_t aidx(int64_t c, int q) {
  return ((c >> 8) * kQ + q) * kChunk + (c & (kChunk - 1));
}

// Compact rows (sparse single-domain lattices) index their population buffers with 32-bit float
// offsets: lbm_create builds them only while a buffer, guard chunks included, holds fewer than
// kCompactMaxFloats floats (build_compact), so every compact cell id c satisfies
// (c / 256 * 19 + 18) * 256 + 255 < 2^31.  The dense box uses 64-bit offsets: a 32-bit one
// overflows past ~113 M cells (2^31 floats / 19) -- the C5 lattice as one domain has 1.07 G; a
// lab kernel that passed a dense cell as int faulted there in round 4.
constexpr int64_t kCompactMaxFloats = int64_t(1) << 31;

struct Layout {
  int nx, ny, nz;
  int xshift;         // cell (x, y, zs) lives at x - xshift + y*pitch + zs*plane: puts the
                      // first fluid cell of a row on a multiple of 4, so fluid 4-cell lane
                      // groups hold no wall cells and store whole 16-B vectors (see
                      // k_stream_collide).  The first xshift cells of a row sit at the end
                      // of the previous row's slots (pitch >= nx keeps them distinct), so
                      // x +- 1 stays c +- 1 and a 512-wide row still fills two chunks.
  int pitch;          // >= nx, multiple of 4
  int planes;         // nz + 2
  int64_t plane;      // pitch * ny
  int64_t ncell;      // plane * planes rounded up to a whole chunk
  int64_t nchunk;     // ncell / 256
  int64_t guard;      // guard chunks before and after the cells (>= one plane + one row + 1)
  int swap;           // 0: rows run along x (s0 = x, s1 = y); 1: rows run along y (s0 = y,
                      // s1 = x; lbm_desc.row_axis) -- c = s0 - xshift + s1*pitch + zs*plane,
                      // pitch >= the row length, plane = pitch * the row count
  // population buffers: guard + nchunk + guard chunks; the base pointer skips the leading
  // guard, so the pulls of lanes masked out at the range ends never leave the allocation
  int64_t buf_floats() const { return (nchunk + 2 * guard) * kQ * kChunk; }
};

// One time step of one launch range, ONE kernel launch (k_step): fused pull-stream + BGK
// collide, one wavefront per active 256-cell chunk (or 64-cell quarter chunk), every
// neighbour a plain pull.  Boundary values are stored producer-side into the slots their one
// consumer pulls next step: wall bounce-back, and the NEE value of an NEE neighbour.
// 4-cell ranges leave their NEE-adjacent fluid cells to NEE blocks that lead the grid, one
// cell per thread; one-cell ranges do them in their quarter waves.
// Partials: one fp64 |u| sum per block (reduction blocks, NEE blocks, then chunk blocks).
struct MainArgs {
  const float* src;     // base (past the guard chunk)
  float* dst;
  const uint8_t* type;  // per cell
  const uint32_t* links;  // per cell: bit q set when c - e_q is a wall (read for kWallAdj cells)
                          // -> producer-side bounce-back stores
  const uint32_t* nlinks;  // per cell: bit q set when c - e_q is an NEE cell supplying q (face
                           // match; read for kNeeAdj cells) -> producer-side NEE stores
  const float* rho; const float* ux; const float* uy; const float* uz;  // NEE data at NEE cells:
                        // rho_bc or NaN (rho of the fluid neighbour), u_bc or NaN (pressure
                        // boundary: u of the fluid neighbour)
  float4 bc_const;      // with bc_uniform = 1: every NEE cell's record (rho, ux, uy, uz), bit for
  int bc_uniform;       // bit -- the cavity's lid -- so no NEE cell loads one
  double* partial;      // one per block
  const int* chunks;    // active chunk ids
  int chunk0;           // >= 0: they are chunk0, chunk0 + 1, ... (box lattices) -- no list load,
                        // one dependent round trip less per wave
  int nchunks;
  const unsigned long long* lane_masks;  // nullable (4-cell path): per chunk of the list, bit l set when
                        // lane l (cells 4l .. 4l+3) or a neighbouring lane holds a cell the chunk
                        // wave updates; the other lanes load nothing (sparse lattices)
  const int* groups;    // nullable (sparse lists): compact list of active 4-cell groups (first cell
                        // id of each, a multiple of 4, bit 0 set for an idle group of a segment,
                        // storage order); 4-cell waves take 64 entries (one per lane), one-cell
                        // waves 16 (four lanes per entry)
  int64_t ngroups;
  const int* group_bc;        // nullable (one-cell group lists with NEE-adjacent cells, boundary
                              // data not uniform): per list entry, the index of its 4 cells'
                              // records in group_rec, or -1
  const float4* group_rec;    // kNeeSlots records per cell of those groups (nee_prefetch's order)
  int main_blocks;      // multiple of 8 (XCD order), 0 without chunks
  int xcd_run;          // 0: XCD x takes the x-th eighth of the chunk blocks; L > 0: runs of 2^(L-1)
                        // blocks, XCD x taking runs 8j + x (LBM_TUNE_XCD_RUN)
  int chunk_stride;     // 1: each XCD's chunk waves loop over its eighth of the chunk list
                        // (lane-mask ranges only: k_step<..., MASK, STRIDE>)
  int quarter;          // 1: one cell per lane, a wave per 64-cell quarter chunk (small lattices)
  int pitch;
  int64_t plane;
  int64_t c_lo, c_hi;   // cell ranges of this launch, [c_lo, c_hi) and [c_lo2, c_hi2) (the
  int64_t c_lo2, c_hi2; // second one empty except for a slab's two edge planes); cells
                        // outside them are not touched
  float tau;
  float tau_rcp;        // RN(1 / tau)
  int fast_div;         // 1: tau passed verify_fast_div -- the 3-VALU correctly rounded
                        // quotient, wave by wave where the populations lie in its domain
                        // (else the exact division)
  int tau_fast;         // the same for the one-cell paths (NEE cells, one cell per lane)
  unsigned long long* exact_waves;  // counts 4-cell waves that fell back to the exact division
  const int* stopped;   // nullable
  float omc;            // the reference's (1.0f - 1.0f / tau)
  // NEE-adjacent fluid cells of a 4-cell range (NEE blocks: one thread per cell)
  const int* cells;         // linear ids, grouped by NEE-link mask
  const uint32_t* cell_nl;  // their NEE-link masks
  const float4* nee_bc;     // kNeeSlots records per cell: the boundary data of its first NEE
                            // directions, gathered once (static)
  int n_nee;
  int nee_chunks;           // 1: the chunk waves also collide and store the NEE-adjacent cells (their
                            // own and bounce-back slots, |u|); the NEE blocks add only the NEE values
  int nee_blocks;           // multiple of 8 (keeps the chunk blocks' XCD order)
  int nee_waves;            // active waves per NEE block (1 for short, scattered lists)
  // NEE records (nullable; single-domain chunk-list ranges whose chunk waves collide the NEE-
  // adjacent cells, LBM_TUNE_NEE_FIX 2): per chunk-list entry i the records nee_rec_base[i] ..
  // nee_rec_base[i + 1] - 1 (at most kNeeRecMax); record k: kNeeRecF4 float4 -- {position in the
  // chunk, NEE-link mask, cell, 0} as ints, then the boundary data of its first kNeeRecDirs NEE
  // directions; nee_in (null at step 0: B's slots are pulled raw) / nee_out: 8 floats per record,
  // the NEE values of the previous / this step in the mask's bit order
  const int* nee_rec_base;
  const float4* nee_rec;
  const float* nee_in;
  float* nee_out;
  float4* nee_mac;          // nullable (single-domain nee_chunks ranges, LBM_TUNE_NEE_FIX): the chunk
                            // waves store each NEE-adjacent cell's (rho, ux, uy, uz) here, one slot
                            // per such cell in storage order; k_nee_fix (launch_nee_fix, after the
                            // step launch) reads them with the cells' own post-collision slots and
                            // stores the NEE values
  const int* nee_mac_base;  // per work unit (chunk-list entry; 64-entry slice of a group list): the
                            // slot of its first NEE-adjacent cell (prefix counts)
  const int* cell_mac;      // per NEE-list entry (cells[i]): its nee_mac slot
  int swap;             // 1: storage rows run along physical y (Layout::swap)
  // Compact rows (nullable; sparse single-domain lattices, group lists only): every per-cell
  // array above and the population buffers are indexed by compact cell ids -- storage row
  // r = zs * rows_per_plane + s1 keeps only the span of its stored cells, packed in storage
  // order, cell (r, s0) at roff[r] + s0.  rowrec[r]: 12 ints, roff[r + dy + dz * rows_per_plane]
  // at index (dy + 1) * 3 + dz + 1 (dy, dz in -1..1).
  const int4* rowrec;
  const int* group_row;  // the storage row of every group-list entry
  // The device-generated cavity (box = 1; ldc.cu:468-502 on global coordinates, lbm_desc.geo
  // NULL, power-of-two pitch and plane): class, wall links and NEE links of every cell follow
  // from its coordinates, so the step kernels compute them instead of loading the type bytes
  // and link masks.  Cell c sits at s0 = (c + xshift) & (pitch - 1), s1 = bits above, storage
  // plane zs = (c + xshift) >> box_lshift, global z = zs - 1 + z_offset.
  int box;
  int box_nx, box_ny, box_nzg, box_zoff, box_xshift, box_pshift, box_lshift;
  int bb_pull;           // 1: bounce-back on the consumer side (one-cell compact ranges): a fluid
                         // cell takes population q from its own slot opp(q) of the source buffer
                         // where c - e_q is a wall -- the post-collision value the producer side
                         // would have stored there -- and stores no wall slots
  int bb_raw;            // this launch is the lattice's first step of a case whose walls do not
                         // bounce back at step 0 (all but LDC): wall slots are pulled raw
  const int4* grouprec;  // one-cell compact ranges (no list): the row record of every compact
                         // 4-cell group (3 x int4, rowrec's layout); group_bc is then indexed by
                         // compact group
  const int* cell_row;   // the storage row of every NEE-block cell
  // The previous step's residual inside this launch (single domain, one cell per lane, no
  // convergence control): red_blocks (0 or 8) extra blocks lead the grid; the first sums
  // red_partial[0 .. red_n) -- the partials of the previous step's launch, complete at this
  // launch's start -- and runs the residual logic, so a step is one launch, not two.
  int red_blocks;
  int nee_last;         // 1: the NEE blocks are dispatched after the chunk blocks (grid-stride group lists)
  int red_last;         // 1: the reduction group trails the grid instead of leading it
  const double* red_partial;
  int red_n;
  struct ConvState* red_conv;
  float* red_hist;      // nullable: the previous step's history slot
};

// True when k_step's fast quotient (q0 = x*y, q = fma(fma(-q0, tau, x), y, q0),
// y = RN(1/tau)) equals RN(x / tau) for every float x in [1, 2) -- and so, by exact
// power-of-two scaling, for every |x| in [2^-100, 2^100].  Exhaustive over the binade
// (8.4 M values, a few ms on the host).
bool verify_fast_div(float tau);
bool verify_fast_div_by(float d);  // the same identity for any divisor d (no range check)

struct ConvState {      // device-resident reference main-loop state (ldc.cu:613-685)
  double s_local;       // this rank's sum of |u| for the last step
  double s_global;      // after the cross-rank all-reduce
  double s_slot[2];     // RCCL path: this rank's sum by step parity (the all-reduce's input)
  float sum_current;    // S_{k-1} as float (ldc.cu:683)
  float residual;       // last residual
  int k;                // steps executed
  int tol_count;
  int stopped;
  int enabled;          // convergence stopping on/off
  int max_it, stag_max;
  float tol;
  int nonfinite_k;      // first step whose |u| sum was not finite (0: none)
};

constexpr int kNeeRecMax = 8;    // NEE records per chunk (ranges with more use k_nee_fix)
constexpr int kNeeRecDirs = 8;   // NEE directions per record (cells with more: k_nee_fix)
constexpr int kNeeRecF4 = 1 + kNeeRecDirs;
hipError_t launch_step(const MainArgs& a, hipStream_t s);
// NEE records set-up: rec[i] for cells[i] (chunk-relative position pos[i], NEE-link mask nl[i]),
// boundary data gathered from the NEE cells' macro arrays
hipError_t launch_nee_records(const int* cells, const int* pos, const uint32_t* nl, const float* rho, const float* ux,
                              const float* uy, const float* uz, float4* rec, int n, int pitch, int64_t plane, int swap,
                              hipStream_t s);
// the NEE values of records vals (8 floats each) into their NEE cells' slots of buffer f
// (to_buffer = 1), or back from those slots into vals (0)
hipError_t launch_nee_materialize(float* f, const float4* rec, float* vals, int n, int pitch, int64_t plane, int swap,
                                  int to_buffer, hipStream_t s);
// after launch_step of a range with nee_mac: one thread per NEE-adjacent cell (cells, cell_nl,
// nee_bc, n_nee) stores its NEE neighbours' slots of dst
hipError_t launch_nee_fix(const MainArgs& a, hipStream_t s);
// NEE directions of a cell whose boundary data is loaded ahead (one flat face: 5); a cell
// with more (edges and corners of several faces) loads the rest where they are used
constexpr int kNeeSlots = 5;
// nee_bc[i * kNeeSlots + j] = (rho, ux, uy, uz) at c_i - e_q, q = the j-th set bit of nl[i]
// 1 into *differs when some NEE cell's record (rho, ux, uy, uz) differs bitwise from cell ref's
hipError_t launch_bc_uniform(const uint8_t* type, const float* rho, const float* ux, const float* uy,
                             const float* uz, int64_t ncell, int64_t ref, unsigned* differs, hipStream_t s);
hipError_t launch_nee_gather(const int* cells, const uint32_t* nl, const float* rho, const float* ux,
                             const float* uy, const float* uz, float4* nee_bc, int n, int pitch, int64_t plane,
                             int swap, hipStream_t s);
// 1 active wave per NEE block for short, scattered lists (contiguous = fraction of list
// neighbours that are storage neighbours: their lanes share lines), else 4
int nee_waves_for(int n, double contiguous);
int nee_grid(int n, int waves);
int main_grid(int nchunks, bool quarter);
constexpr int kQuarterMaxChunks = 8192;  // <= 128^3 cells: one cell per lane (latency-bound sizes)
constexpr double kGroupFill1 = 0.75;       // one-cell ranges take the group list below this cell fill
constexpr int kReduceBlocks = 256;
// partial sums -> conv->s_local (deterministic: one block for up to 16384 partials, else
// kReduceBlocks blocks sum fixed contiguous slices into scratch and one block sums those);
// finish = 1 also runs the residual logic and writes *hist_slot.
hipError_t launch_reduce(const double* partial, int n, double* scratch, ConvState* conv, float* hist_slot,
                         int finish, hipStream_t s,
                         double* local_out = nullptr);  // where the sum goes (default conv->s_local)
hipError_t launch_finish_global(ConvState* conv, float* hist_slot, hipStream_t s);
// Reference-order fp32 residual (lbm_set_residual_order LBM_SUM_CUB_TREE): the step's |u|
// terms into their reference storage slots terms[ref_idx[c]] (fluid cells; the other slots
// stay 0), then CUB's two-pass device-reduction tree over terms[0 .. n) -- pass 1: `grid`
// blocks of 256 threads over tiles of 256 * ipt items (even share), pass 2: one block over the
// partials, then the residual logic on S = 0.f + the tree's sum
hipError_t launch_vel_terms(const float* src, const uint8_t* type, const uint32_t* bb_links, const int* ref_idx,
                            float* terms, int64_t lo, int64_t hi, int pitch, int64_t plane, int swap, hipStream_t s);
// the same over compact rows (type, bb_links, row_of, rowrec by compact cell; cmap: compact ->
// dense cell; ref_idx by dense cell)
hipError_t launch_vel_terms_compact(const float* src, const uint8_t* type, const uint32_t* bb_links, const int* cmap,
                                    const int* row_of, const int4* rowrec, const int* ref_idx, float* terms, int64_t lo,
                                    int64_t hi, int swap, hipStream_t s);
int cub_grid(int64_t n, int ipt, int grid_cap);
hipError_t launch_cub_tree(const float* terms, int64_t n, int ipt, int vec, int grid_cap, float* partials,
                           ConvState* conv, float* hist_slot, hipStream_t s);
// lazy macros: (rho, u) of the fluid cells in [lo, hi) from the last step's source buffer;
// bb_links (nullable): the wall links of a consumer-side bounce-back step (MainArgs::bb_pull)
hipError_t launch_moments(const float* src, const uint8_t* type, const uint32_t* bb_links, float* rho, float* ux,
                          float* uy, float* uz, int64_t lo, int64_t hi, int pitch, int64_t plane, int swap,
                          hipStream_t s);
// the same over compact rows: compact cells [lo, hi) pull through rowrec[row_of[c / 4]] and write
// the macros of their dense cells cmap[c] (no dense staging copy of the population buffer)
hipError_t launch_moments_compact(const float* src, const uint8_t* type, const uint32_t* bb_links, const int* cmap,
                                  const int* row_of, const int4* rowrec, float* rho, float* ux, float* uy, float* uz,
                                  int64_t lo, int64_t hi, int swap, hipStream_t s);
// per local plane digest of the fluid (rho, u) bits keyed by global coordinates (lbm_field_digest);
// out[nz] must be zeroed
hipError_t launch_digest(const uint8_t* type, const float* rho, const float* ux, const float* uy, const float* uz,
                         int nx, int ny, int nz, int pitch, int xshift, int64_t plane, int z_offset, int swap,
                         unsigned long long* out, hipStream_t s);

// streaming copy of n4 16-B vectors (lbm_probe_stream): `blocks` x 256 threads; shape 0/1
// grid-stride non-temporal / plain, 2/3 the same with one contiguous region per XCD, 4/5
// XCD regions with 2 / 4 vectors in flight per thread; 6/7 k_step's shape (non-temporal /
// plain): one wave per 16-KB tile, 16 vectors per lane in flight, tiles in contiguous runs per
// XCD, `blocks` ignored (n4 must be a multiple of 4096); 8/9 the same tiles loaded by LDS-DMA
// (non-temporal / default policy)
constexpr int kProbeShapes = 10;
hipError_t launch_probe_copy(const void* src, void* dst, int64_t n4, int blocks, int shape, hipStream_t s);
// zero n4 16-B vectors with one sweep of non-temporal stores (one region per XCD): the write
// rate buffer_placement ranks allocations by
hipError_t launch_probe_fill(void* dst, int64_t n4, hipStream_t s);

// compact rows (MainArgs::rowrec): cmap[i] = the dense cell of compact cell i, or -1.
// Populations of the n compact cells from a dense buffer (to_compact = 1; unmapped slots 0) or
// back into one (0; unmapped slots skipped).  Per-cell arrays (1- or 4-byte elements) gathered.
hipError_t launch_pop_compact(float* dst, const float* src, const int* cmap, int64_t n, int to_compact,
                              hipStream_t s);
hipError_t launch_cell_gather(void* dst, const void* src, const int* cmap, int64_t n, int elem_bytes, hipStream_t s);
// test hook: NaN into every slot of the wall cells (class kWall) of population buffer f, n cells
hipError_t launch_poison_walls(float* f, const uint8_t* type, int64_t n, hipStream_t s);

// halo: pack populations qs[0..nq) of storage plane zs into buf[nq][plane] / unpack
hipError_t launch_pack(const float* f, float* buf, int zs, int64_t plane, const int* qs_dev, int nq,
                       hipStream_t s);
// skip_classes: bit (1 << class) leaves ghost cells of that class untouched
hipError_t launch_unpack(float* f, const float* buf, const uint8_t* type, int zs, int64_t plane, const int* qs_dev,
                         int nq, unsigned skip_classes, hipStream_t s);
// seed wall slots with bounce-back values of buffer f (LDC: bounce-back already at step 0)
hipError_t launch_bb_prime(float* f, const uint8_t* type, const uint32_t* links, int64_t ncell, int pitch,
                           int64_t plane, int swap, hipStream_t s);

// LBM_CASE_GENERIC boundary code on the device (lbm_bc_code with a device table)
struct BcCode {
  int code, face, kind;     // kind: 0 velocity (rho_bc = rho_F), 1 velocity + rho, 2 pressure
  float rho, u[3];
  const float* table;       // nullable: u along the face axis per cell (see lbm.h)
};
constexpr int kMaxBcCodes = 16;

// geometry: reference codes (int8 per linear cell) -> cell-type bytes
struct GeoArgs {
  const int8_t* codes;
  uint8_t* type;
  uint32_t* links;         // per cell wall-link masks (written for fluid cells)
  uint32_t* nlinks;        // per cell NEE-link masks (written for fluid cells)
  float* rho; float* ux; float* uy; float* uz;  // NEE data written at NEE cells
  const float* inlet_uy;   // nx * nz_global (nullable)
  const float* outlet_uy;
  int case_kind;
  float lid_u;
  int nx, ny, pitch, xshift, planes;
  int64_t plane, ncell;
  int z_offset, nz_global;
  int swap;                // Layout::swap
  BcCode bcs[kMaxBcCodes];  // LBM_CASE_GENERIC
  int nbc;
};
hipError_t launch_classify(const GeoArgs& g, hipStream_t s);
hipError_t launch_flag_fluid(const GeoArgs& g, hipStream_t s);
hipError_t launch_ldc_codes(int8_t* codes, int nx, int ny, int pitch, int xshift, int64_t plane, int64_t ncell, int z_offset,
                            int nz_global, int swap, hipStream_t s);

// initial populations from per-cell fields (nullable -> rho 1, u 0); form 0 = LDC wi form,
// 1 = expanded; writes both buffers for every cell
// geo_pre of a raw 0/1 mask on the device (bifurcation.cu:63-239): mask planes are global
// z = zbase .. ; local storage planes z_lo .. z_hi-1 get codes (-1 for the halo plane below)
hipError_t launch_mask_hist(const uint8_t* mask, int nx, int ny, int nz_global, int zbase, int z_lo, int z_hi,
                            unsigned long long* hist, int swap, hipStream_t s);
hipError_t launch_mask_codes(const uint8_t* mask, int nx, int ny, int nz_global, int zbase, int8_t* codes, int pitch,
                             int xshift, int64_t plane, int64_t ncell, int z_offset, int z_lo, int z_hi, int swap,
                             hipStream_t s);
hipError_t launch_init_feq(float* fa, float* fb, int64_t ncell, int form, const float* rho, const float* ux,
                           const float* uy, const float* uz, hipStream_t s);
hipError_t launch_init_mask(float* fa, float* fb, const int8_t* codes, const float* in_uy, const float* out_uy, int nx,
                            int ny, int nz, int pitch, int xshift, int64_t plane, int64_t ncell, int z_offset, int swap,
                            hipStream_t s);
hipError_t launch_init_ldc(float* fa, float* fb, int64_t n, int pitch, int xshift, int nx, int ny, float lid_u, int swap,
                           hipStream_t s);

}  // namespace lbm
