// lbm_ctx.hip -- liblbm.so: the C ABI of include/lbm.h on top of the HIP kernels.
//
// A context owns one lattice (or one z-slab of it) on one device:
//   two AoSoA population buffers (A-B pattern; the reference's d_scr/d_dst, ldc.cu:640-641),
//   the cell-type bytes (the reference's d_geo + texture-bound index, Poiseulle.cu:49-50),
//   (rho, u) arrays (d_rho/d_ux/d_uy/d_uz; NEE cells hold their boundary data there), per-cell
//   wall- and NEE-link masks, per launch-range work lists (active 256-cell chunks), block
//   partials of the |u| sum and the device-resident state of the reference main loop
//   (ldc.cu:613-685).
// The reference's per-step sequence update -> boundary_stream -> calc_vel_square ->
// thrust::reduce -> host residual (ldc.cu:654-684) becomes one k_step launch (boundary values
// stored producer-side) + a deterministic reduction folded into the next launch, with no host
// synchronisation inside a call.  Slabs exchange the 5 populations crossing each +-z face (packed) over
// RCCL on a second stream while the interior updates.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/lbm.h"
#include "lbm_d3q19.hpp"
#include "lbm_kernels.hpp"

using namespace lbm;

namespace {
std::string g_create_error;
// process-wide tuning knobs (lbm_tune), read by lbm_create / the step path
int g_tune[LBM_TUNE_COUNT] = {0, 0, 0, 1, 0, 0, 0, 0, 0, 16, 0, 0, 0, 0, 0};
constexpr int kUpSet[5] = {5, 11, 13, 15, 16};    // e_z = +1: cross the top face
constexpr int kDownSet[5] = {6, 12, 14, 17, 18};  // e_z = -1: cross the bottom face

// lbm_kernel_times kinds
enum : int {
  kKindStep = 0,       // every step-kernel launch
  kKindSrc0 = 1,       // ... reading population buffer 0
  kKindSrc1 = 2,       // ... reading buffer 1
  kKindEdge = 3,       // slab step: the edge-plane launch
  kKindMid = 4,        // slab step: the interior launch
  kKindHalo = 5,       // slab step: halo pack -> send/recv -> unpack on the communication stream
  kKindExposed = 6,    // slab step: halo end after interior end (clipped at 0): the exchange not hidden
  kKindSpan = 7,       // lbm_profile(ctx, 2): one event pair around each lbm_step call's work (launches = steps)
  kKinds = 8
};

struct Range {            // one launch: cells [c_lo, c_hi) u [c_lo2, c_hi2) with their work lists
  int64_t c_lo = 0, c_hi = 0, c_lo2 = 0, c_hi2 = 0;
  int* chunks = nullptr;  // active 256-cell chunks (>= 1 fluid cell in range)
  int chunk0 = -1;        // >= 0: chunks is chunk0, chunk0 + 1, ... (the kernel skips the list)
  int nchunks = 0;
  // 4-cell ranges: NEE-adjacent fluid cells, one per thread in the NEE blocks
  int* cells = nullptr;
  uint32_t* cell_nl = nullptr;  // their NEE-link masks
  float4* nee_bc = nullptr;     // their first kNeeSlots NEE neighbours' boundary data (static)
  int n_nee = 0, nee_blocks = 0, nee_waves = 4;
  bool nee_chunks = false;  // 4-cell ranges: chunk waves also store the NEE-adjacent cells (MainArgs)
  // single-domain nee_chunks ranges (LBM_TUNE_NEE_FIX): no NEE blocks; the chunk waves record the
  // NEE-adjacent cells' (rho, u) in lbm_ctx::nee_mac and k_nee_fix stores the NEE values after the
  // step launch, from those records and the cells' own post-collision slots (cells, cell_nl and
  // nee_bc are its list)
  bool nee_fix = false;
  bool nee_last = false;  // NEE blocks dispatched after the chunk blocks (MainArgs::nee_last)
  int* nee_mac_base = nullptr;  // nee_fix: per work unit (chunk-list entry, 64-entry group-list slice), the
                                // nee_mac slot of its first NEE-adjacent cell (MainArgs::nee_mac_base)
  int* cell_mac = nullptr;      // nee_fix: per NEE-list entry, its nee_mac slot
  // single-domain chunk-list ranges with nee_chunks (LBM_TUNE_NEE_FIX 2): NEE records instead --
  // the chunk waves compute the NEE values after their relaxation into lbm_ctx::nee_val and put
  // them into the next step's pulls (MainArgs::nee_rec); per chunk-list entry the first record
  // (nchunks + 1 prefix sums), n_rec records in chunk order
  bool nee_records = false;
  int* nee_rec_base = nullptr;
  float4* nee_rec = nullptr;
  int n_rec = 0;
  int nee_rec_max = 0;  // the most records one chunk holds
  // one-cell ranges whose waves all fit on the device at once: the fused residual's blocks go
  // last (MainArgs::red_last), so that no chunk wave waits for a slot behind them (LDC 64^3
  // 11.30 -> 11.14 us, C4 8.48 -> 8.27 us; a grid of several rounds -- the coronary tree 36.0 ->
  // 39.6 us -- would wait for the residual at its end instead; profiles/r04_red_last_ab.log)
  bool one_round = false;
  int* groups = nullptr;  // sparse ranges: compact list of active 4-cell groups (both paths)
  int64_t ngroups = 0;
  int* group_bc = nullptr;         // one-cell group lists: per entry, its NEE records' index or -1
  float4* group_rec = nullptr;     // kNeeSlots records per cell of the groups with NEE-adjacent cells
  double group_fill = 0.0;  // mean share of a listed group's cells the wave updates
  int* group_row = nullptr;  // compact rows: the storage row of every group-list entry
  int* cell_row = nullptr;   // compact rows: the storage row of every NEE-block cell
  unsigned long long* lane_masks = nullptr;  // 4-cell path, sparse ranges: lanes a chunk wave loads
  double* part = nullptr; // one |u| partial per block (NEE blocks, then chunk blocks)
  int npart = 0;
  int main_blocks = 0;
  bool stride = false;    // grid-stride chunk loop (LBM_TUNE_GRID_STRIDE)
  double lane_fill = 1.0; // 4-cell path: mean share of chunk lanes with a cell to update
  bool quarter = false;   // one cell per lane (small ranges)
};
}  // namespace

struct lbm_ctx {
  lbm_desc d{};
  Layout L{};
  hipStream_t s_comp = nullptr, s_comm = nullptr;
  hipEvent_t ev_edge = nullptr, ev_halo = nullptr, ev_mid = nullptr, ev_fin = nullptr;
  hipEvent_t ev_sum[2] = {nullptr, nullptr};  // slab step: the reduction of step h read partials[h & 1]
  float* alloc[2] = {nullptr, nullptr};  // hipMalloc'd population buffers
  std::vector<double> cand_gbs;           // buffer_placement: candidates' sweep-write rates (GB/s)
  int chosen[2] = {0, 1};                 // the two candidates kept
  float* buf[2] = {nullptr, nullptr};  // past the guard chunk
  int cur = 0;                         // buf[cur] holds the current state (every launch flips it)
  uint8_t* type = nullptr;
  uint32_t* links = nullptr;   // wall-link masks
  uint32_t* nlinks = nullptr;  // NEE-link masks
  int8_t* codes = nullptr;               // reference codes per storage cell (lbm_get_geo)
  float *bc_in = nullptr, *bc_out = nullptr;  // inlet / outlet u_y tables (lbm_init_case)
  float *rho = nullptr, *ux = nullptr, *uy = nullptr, *uz = nullptr;
  float4* nee_mac = nullptr;  // whole.nee_fix: (rho, u) of the NEE-adjacent cells, one slot each (storage order)
  // whole.nee_records: the NEE values by step parity (2 x n_rec x 8 floats), and whether the NEE
  // cells' slots of the two buffers miss them (steps since the last materialize_nee)
  float* nee_val = nullptr;
  bool nee_stale = false;
  Range whole, edge, mid;  // single domain: whole; slabs: both edge planes (one launch), interior
  double* partial_all = nullptr;
  double* red_part = nullptr;  // fused residual (one-cell single domain): 2 x red_n partials by step parity
  int red_n = 0;               // whole.npart + 8 (the leading reduction group)
  bool fuse_red = false;
  int npart_slab = 0;
  double* slab_part = nullptr;  // RCCL slab step: 2 x npart_slab partials by step parity
  double* scratch = nullptr;
  ConvState* conv = nullptr;
  float* hist = nullptr;
  int hist_cap = 0;
  int* qsets = nullptr;  // device: up set (5), down set (5), all (19)
  float *send_up = nullptr, *send_dn = nullptr, *recv_up = nullptr, *recv_dn = nullptr;
  int steps_done = 0;    // device-confirmed steps
  bool bb_immediate = false;
  bool conv_enabled = false;
  bool halo_primed = false;
  int64_t n_box = 0, n_fluid = 0, n_slow = 0, n_wall_adj = 0;
  bool bc_uniform = false;  // every NEE cell holds the record bc_const (fill_main_args)
  float4 bc_const{};
  float tau = 0.f, omc = 0.f;
  bool fast_div = false;  // tau verified for the 3-VALU correctly rounded division
  unsigned long long* retried = nullptr;  // device: 4-cell waves that took the exact division
  // profiling: prof = per-launch events (lbm_profile 1); span = one event pair per lbm_step call (2)
  bool prof = false;
  bool span = false;
  // recorded event pairs, each counted under up to three kinds (lbm_kernel_times)
  struct Rec {
    hipEvent_t a, b;
    int kinds[3];  // -1: unused
  };
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  std::vector<Rec> recs;
  hipEvent_t last_mid_end = nullptr;  // the interior launch's end event of the current step
  double kernel_ms = 0.0, kind_ms[kKinds] = {};
  int64_t launches = 0, kind_n[kKinds] = {};
  // lazy macros (k_moments): the step kernels store none; lbm_get_macros recomputes them
  // from the last step's source buffer when macros_stale
  bool macros_stale = false;
  // rccl
  ncclComm_t comm = nullptr;
  int rank = 0, nranks = 1;
  // sticky: the communicator was aborted (a peer failed or a wait timed out).  The ghost planes
  // and the residual are stale from then on, so every later step, wait and read-out fails with
  // LBM_ERR_RCCL instead of silently running the slab as a single domain
  bool comm_failed = false;
  bool inject_fault = false;  // lbm_debug_fail_next_wait: the next wait sees a failed peer
  // residual summation order (lbm_set_residual_order): LBM_SUM_FP64, or the reference-order
  // fp32 CUB tree over n_ref terms (ref_idx: reference storage slot per fluid cell, -1 else)
  int sum_mode = LBM_SUM_FP64;
  int cub_ipt = 16, cub_vec = 4, cub_grid = 240;
  int* ref_idx = nullptr;
  float* terms = nullptr;
  float* cub_part = nullptr;
  int64_t n_ref = 0;
  // Compact rows (LBM_TUNE_COMPACT; single-domain lattices whose step takes group lists): buf[]
  // hold only the spans of stored cells of every storage row, packed in storage order, and the
  // kernels read compact copies of the per-cell arrays (ctype ... cuz, indexed like buf).  The
  // dense arrays above stay for set-up and read-out, which run on a dense staging copy of a
  // population buffer (stage_dense / from_dense).
  bool compact = false;
  int64_t ncell_c = 0, nchunk_c = 0, guard_c = 0;  // compact cell slots (whole chunks), guard chunks
  int* cmap = nullptr;     // device: the dense cell of every compact cell, -1 for none
  std::vector<int> cmap_h; // its host copy (lbm_get_f places the compact slots on the host)
  int* crow = nullptr;     // device: the storage row of every compact 4-cell group (k_moments_compact)
  int4* rowrec = nullptr;  // device: per storage row the nine neighbour-row offsets (MainArgs::rowrec)
  int4* grouprec = nullptr;  // device, one-cell compact ranges: rowrec of every compact group's row
  uint8_t* ctype = nullptr;
  uint32_t *clinks = nullptr, *cnlinks = nullptr;
  float *crho = nullptr, *cux = nullptr, *cuy = nullptr, *cuz = nullptr;
  // slots per population buffer past the leading guard (the part checkpoints hold)
  int64_t pop_floats() const { return (compact ? nchunk_c : L.nchunk) * kQ * kChunk; }
  // the device-generated cavity with power-of-two pitch and plane: the chunk kernels compute
  // types and links from coordinates (MainArgs::box)
  bool box = false;
  int xcd_run = 0;  // MainArgs::xcd_run (LBM_TUNE_XCD_RUN at lbm_create)
  // bounce-back on the consumer side (MainArgs::bb_pull): compact ranges and the one-cell
  // whole-domain range of the cavity read a wall link's value from the cell's own opposite
  // slot, so no step writes wall slots.  Not the cavity's 4-cell range: its own-slice DMA made
  // 512^3 12% slower (every row's end chunks link the x walls), for 0.1% of its bytes (the RCCL slab sequence keeps the producer side:
  // lbm_attach_rccl first writes the wall slots once, k_bb_prime)
  bool bb_pull() const {
    return compact || (whole.quarter && box && d.nz_global == d.nz && !comm && !comm_failed);
  }
  // step k's source buffer holds wall slots that must be pulled raw (MainArgs::bb_raw): the
  // first step of a case whose walls do not bounce back at step 0
  bool bb_raw(int k) const { return k == 0 && !bb_immediate; }
  // The wall slots of both buffers were not written by the steps that produced them: a step ran
  // with bounce-back on the consumer side (or a checkpoint saved by such a context was loaded).
  // Every producer-side reader -- the RCCL slab step, lbm_group_step, the lazy macros of a
  // producer-side context -- first restores them (prime_walls).
  bool walls_stale = false;
  // set-up cost (lbm_get_setup_cost): wall seconds of lbm_create, and the device memory it took
  // (free memory hipMemGetInfo reported at its start, less that at its end / at the lowest point:
  // the placement probe's candidates)
  double create_s = 0.0;
  int64_t mem_resident = 0, mem_peak = 0;
  size_t mem_free0 = 0, mem_free_min = 0;
  std::string err;
};

#define HIPCK(ctx, expr)                                              \
  do {                                                                \
    hipError_t e_ = (expr);                                           \
    if (e_ != hipSuccess) {                                           \
      (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(e_); \
      return LBM_ERR_HIP;                                             \
    }                                                                 \
  } while (0)

#define NCCK(ctx, expr)                                                \
  do {                                                                 \
    ncclResult_t r_ = (expr);                                          \
    if (r_ != ncclSuccess) {                                           \
      (ctx)->err = std::string(#expr) + ": " + ncclGetErrorString(r_); \
      return LBM_ERR_RCCL;                                             \
    }                                                                  \
  } while (0)

#define RCK(expr)                  \
  do {                             \
    int rc_ = (expr);              \
    if (rc_ != LBM_OK) return rc_; \
  } while (0)

namespace {

int64_t cell_of(const Layout& L, int x, int y, int z) {  // local z (storage plane z+1)
  const int s0 = L.swap ? y : x, s1 = L.swap ? x : y;
  return (int64_t)(s0 - L.xshift) + (int64_t)s1 * L.pitch + (int64_t)(z + 1) * L.plane;
}

// copy one raster x-row (local plane z) into storage, dropping the (outer, passive) cells
// the shift puts before cell 0 (row 0 of storage plane 0 only)
template <class T>
void put_row(std::vector<T>& h, const Layout& L, int y, int z, const T* row) {
  if (!L.swap) {
    const int64_t at = cell_of(L, 0, y, z);
    const int skip = at < 0 ? (int)-at : 0;
    if (skip < L.nx) std::memcpy(&h[at + skip], row + skip, sizeof(T) * (L.nx - skip));
    return;
  }
  for (int x = 0; x < L.nx; ++x) {
    const int64_t at = cell_of(L, x, y, z);
    if (at >= 0) h[at] = row[x];
  }
}

// storage planes of the raster geo (nz, or nz + 2 with halo planes) and its fluid code
int geo_planes(const lbm_desc& d) { return d.nz + (d.halo_planes ? 2 : 0); }
int8_t fluid_code(const lbm_desc& d) { return d.case_kind == LBM_CASE_LDC ? 3 : 4; }

// row shift that puts the most common first-fluid position of a storage row (along x, or
// along y when swap) at a multiple of 4
int choose_xshift(const lbm_desc& d, int swap) {
  if (d.x_align > 0) return d.x_align - 1;
  if (!d.geo) return 2;  // device-generated cavity: fluid starts at x = 2 (ldc.cu:469)
  const int8_t fluid = fluid_code(d);
  const int n0 = swap ? d.ny : d.nx, n1 = swap ? d.nx : d.ny;
  int64_t hist[4] = {0, 0, 0, 0};
  for (int z = 0; z < geo_planes(d); ++z)
    for (int s1 = 0; s1 < n1; ++s1)
      for (int s0 = 0; s0 < n0; ++s0) {
        const int x = swap ? s1 : s0, y = swap ? s0 : s1;
        if (d.geo[((int64_t)z * d.ny + y) * d.nx + x] == fluid) {
          hist[s0 & 3]++;
          break;
        }
      }
  return (int)(std::max_element(hist, hist + 4) - hist);
}

// 256-cell chunks holding a fluid cell (the waves k_step launches) when the rows run along
// x (swap 0) or y (swap 1); fluid from the codes, or mask != 0 for a raw device mask
int64_t active_chunks(const lbm_desc& d, int swap) {
  const int n0 = swap ? d.ny : d.nx, n1 = swap ? d.nx : d.ny;
  const int64_t pitch = (n0 + 3) / 4 * 4, plane = pitch * n1;
  const int pad = d.geo ? (d.halo_planes ? 1 : 0) : (d.halo_planes ? 3 : 0);
  const int8_t fluid = fluid_code(d);
  std::vector<uint8_t> hit((size_t)((plane * (d.nz + 2) + 4) / kChunk + 2), 0);
  for (int z = 0; z < d.nz; ++z)
    for (int y = 0; y < d.ny; ++y)
      for (int x = 0; x < d.nx; ++x) {
        const int64_t r = ((int64_t)(z + pad) * d.ny + y) * d.nx + x;
        if (d.geo ? d.geo[r] != fluid : d.mask[r] == 0) continue;
        const int64_t c = (swap ? y : x) + (int64_t)(swap ? x : y) * pitch + (int64_t)(z + 1) * plane;
        hit[c / kChunk] = 1;
      }
  int64_t n = 0;
  for (uint8_t h : hit) n += h;
  return n;
}

// lbm_desc.row_axis: 1 rows along x, 2 along y, 0 choose -- y when it leaves at least 3%
// fewer active chunks (a pipe along y: whole fluid rows instead of partial x-rows);
// slabs of a larger lattice and the device-generated cavity keep x unless told otherwise
int choose_swap(const lbm_desc& d) {
  int axis = d.row_axis;
  if (axis == 0) axis = g_tune[LBM_TUNE_ROW_AXIS];  // A/B and test switch for row_axis 0
  if (axis == 1) return 0;
  if (axis == 2) return 1;
  if ((!d.geo && !d.mask) || (d.nz_global > 0 && d.nz_global != d.nz)) return 0;
  const int64_t cx = active_chunks(d, 0), cy = active_chunks(d, 1);
  return (double)cy < 0.97 * (double)cx ? 1 : 0;
}

// time one kernel launch with HIP events on its own stream (lbm_profile)
int take_event(lbm_ctx* c, hipEvent_t* e) {
  if (c->ev_pool.size() <= c->ev_used) {
    hipEvent_t n;
    HIPCK(c, hipEventCreate(&n));
    c->ev_pool.push_back(n);
  }
  *e = c->ev_pool[c->ev_used++];
  return LBM_OK;
}

// bracket launch() with events on st (lbm_profile); counted under kinds k0, k1, k2 (-1: none)
template <class F>
int timed(lbm_ctx* c, hipStream_t st, int k0, int k1, int k2, F&& launch, hipEvent_t* end_out = nullptr) {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (c->prof) {
    RCK(take_event(c, &e0));
    RCK(take_event(c, &e1));
    c->recs.push_back({e0, e1, {k0, k1, k2}});
    HIPCK(c, hipEventRecord(e0, st));
  }
  RCK(launch());
  if (c->prof) HIPCK(c, hipEventRecord(e1, st));
  if (end_out) *end_out = e1;
  for (int k : {k0, k1, k2})
    if (k >= 0) c->kind_n[k]++;
  return LBM_OK;
}

int harvest_profile(lbm_ctx* c) {
  if (c->recs.empty()) return LBM_OK;
  HIPCK(c, hipDeviceSynchronize());
  for (const auto& r : c->recs) {
    float ms = 0.f;
    HIPCK(c, hipEventElapsedTime(&ms, r.a, r.b));
    if (r.kinds[0] == kKindStep) c->kernel_ms += ms;
    for (int k : r.kinds)
      if (k >= 0) c->kind_ms[k] += (k == kKindExposed ? std::max(0.f, ms) : ms);
  }
  c->ev_used = 0;
  c->recs.clear();
  return LBM_OK;
}

// one step's update of a range: ONE k_step launch (chunk blocks + NEE-adjacent cell blocks).
// the previous step's residual folded into a launch (lbm_ctx::fuse_red)
struct FusedRed {
  double* part;        // this launch's partials
  const double* prev;  // the previous launch's (nullptr: nothing to finish)
  float* hist;         // the previous step's history slot (nullable)
};

void fill_main_args(lbm_ctx* c, MainArgs& a, int srcbuf) {
  a.src = c->buf[srcbuf];
  a.dst = c->buf[srcbuf ^ 1];
  if (c->compact) {
    a.type = c->ctype; a.links = c->clinks; a.nlinks = c->cnlinks;
    a.rho = c->crho; a.ux = c->cux; a.uy = c->cuy; a.uz = c->cuz;
    a.rowrec = c->rowrec;
    a.grouprec = c->grouprec;
  } else {
    a.type = c->type; a.links = c->links; a.nlinks = c->nlinks;
    a.rho = c->rho; a.ux = c->ux; a.uy = c->uy; a.uz = c->uz;
  }
  a.pitch = c->L.pitch; a.plane = c->L.plane;
  a.tau = c->tau;
  a.tau_rcp = 1.0f / c->tau;
  a.tau_fast = c->fast_div ? 1 : 0;
  a.exact_waves = c->retried;
  a.omc = c->omc;
  a.swap = c->L.swap;
  a.bc_uniform = c->bc_uniform ? 1 : 0;
  a.bc_const = c->bc_const;
  if (c->box) {
    a.box = 1;
    a.box_nx = c->L.nx; a.box_ny = c->L.ny; a.box_nzg = c->d.nz_global; a.box_zoff = c->d.z_offset;
    a.box_xshift = c->L.xshift;
    a.box_pshift = __builtin_ctz((unsigned)c->L.pitch);
    a.box_lshift = __builtin_ctzll((unsigned long long)c->L.plane);
  }
}

// one step of a range from buffer srcbuf into srcbuf ^ 1
int run_range(lbm_ctx* c, Range& r, int srcbuf, hipStream_t st, const FusedRed* fr = nullptr, int range_kind = -1,
              double* part = nullptr, int step = -1) {
  MainArgs a{};
  fill_main_args(c, a, srcbuf);
  a.bb_pull = (&r == &c->whole && c->bb_pull()) ? 1 : 0;
  a.bb_raw = c->bb_raw(step) ? 1 : 0;
  a.partial = part ? part : r.part;
  a.chunks = r.chunks; a.chunk0 = r.chunk0; a.nchunks = r.nchunks; a.main_blocks = r.main_blocks; a.quarter = r.quarter ? 1 : 0;
  a.chunk_stride = r.stride ? 1 : 0;
  // LBM_TUNE_XCD_RUN 0 (auto): runs of four blocks (L = 3) for the 4-cell chunk lists whose rows
  // run along y -- the pipe, C3: round robin (runs of one) took it from 184 to 176 us per step in
  // rocprof in round 5, where LDC 256^3 and 512^3 run 9% / 4% slower that way
  // (profiles/r05p_c3_posts_xcd_rocprof.log, r05_xcd_run_ab.log); with the NEE blocks in the
  // launch (round 6) runs of four beat runs of one by ~0.8 us, 170.4-171.0 vs 171.1-172.8
  // (r06m_c3_xcd_runs_ab.log, r06o_c3_xcd_runs_ab.log), and with the wave-priority flips runs of
  // eight beat four, 167.9-168.6 vs 168.9-170.3 us (L = 4; r06zw_c3_xcd_runs_prio_ab.log,
  // r06zx_...); runs of four blocks for compact one-cell ranges of several rounds of
  // waves -- the coronary tree: 31.1 -> 29.8 us, where one-round C4 runs slower interleaved
  // (r05_c1_xcd_ab.log, r05z_coronary_xcd_ab.log); one contiguous eighth per XCD elsewhere; 17:
  // eighths everywhere.  Not for grid-stride ranges: their waves take work by XCD (b & 7) and
  // round (b >> 3) whatever the order, so a run length would only move their partial slots
  a.xcd_run = (c->xcd_run == 17 || r.stride)                 ? 0
              : c->xcd_run > 0                               ? c->xcd_run
              : (c->L.swap && !r.quarter && !r.groups)       ? 4
              : (c->compact && r.quarter && !r.one_round)    ? 3
                                                             : 0;
  a.lane_masks = r.quarter ? nullptr : r.lane_masks;
  a.groups = r.groups;
  a.ngroups = r.ngroups;
  a.group_bc = r.group_bc;
  a.group_rec = r.group_rec;
  a.group_row = r.group_row;
  a.cell_row = r.cell_row;
  a.c_lo = r.c_lo; a.c_hi = r.c_hi; a.c_lo2 = r.c_lo2; a.c_hi2 = r.c_hi2;
  a.fast_div = (c->fast_div && !r.quarter) ? 1 : 0;
  a.stopped = c->conv_enabled ? &c->conv->stopped : nullptr;
  a.cells = r.cells; a.cell_nl = r.cell_nl; a.nee_bc = r.nee_bc; a.n_nee = r.n_nee;
  a.nee_blocks = r.nee_blocks; a.nee_waves = r.nee_waves;
  a.nee_last = r.nee_last ? 1 : 0;
  a.nee_chunks = r.nee_chunks ? 1 : 0;
  a.nee_mac = r.nee_fix ? c->nee_mac : nullptr;
  a.nee_mac_base = r.nee_mac_base;
  a.cell_mac = r.cell_mac;
  if (r.nee_records) {
    const int64_t per = (int64_t)r.n_rec * 8;
    a.nee_rec_base = r.nee_rec_base;
    a.nee_rec = r.nee_rec;
    a.nee_out = c->nee_val + (step & 1) * per;
    // step 0 pulls the NEE cells' slots raw (boundary_stream runs after update)
    a.nee_in = step > 0 ? c->nee_val + ((step - 1) & 1) * per : nullptr;
  }
  if (fr) {
    a.partial = fr->part;
    a.red_blocks = 8;
    a.red_last = r.one_round ? 1 : 0;
    a.red_partial = fr->prev;
    a.red_n = c->red_n;
    a.red_conv = c->conv;
    a.red_hist = fr->hist;
  }
  if (r.main_blocks + r.nee_blocks > 0 || fr) {
    c->launches++;
    RCK(timed(c, st, kKindStep, kKindSrc0 + srcbuf, range_kind, [&] {
                HIPCK(c, launch_step(a, st));
                // the NEE values of this step, from what its chunk waves recorded (counted with the
                // step kernel: one step's update is both launches)
                if (r.nee_fix) HIPCK(c, launch_nee_fix(a, st));
                return LBM_OK;
              },
              range_kind == kKindMid ? &c->last_mid_end : nullptr));
  }
  return LBM_OK;
}

// device scratch freed on every exit path of build_range
struct DevScratch {
  void* p = nullptr;
  ~DevScratch() {
    if (p) (void)hipFree(p);
  }
};

// build_range over compact rows: the cells are compact ids (the lists index the compact arrays);
// dense_of translates them for the gathers of boundary records from the dense arrays, row_of
// gives every compact 4-cell group's storage row; the dense range's one-cell choice is kept and
// the waves always take group lists
struct CompactView {
  const std::vector<int>* dense_of;
  const std::vector<int>* row_of;
  bool quarter;
};

// upload a host vector (n >= 1) into a fresh device array
template <class T>
int upload(lbm_ctx* c, T** dev, const std::vector<T>& h) {
  HIPCK(c, hipMalloc(dev, sizeof(T) * std::max<size_t>(1, h.size())));
  if (!h.empty()) HIPCK(c, hipMemcpy(*dev, h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice));
  return LBM_OK;
}

// work lists of the cells [lo, hi) u [lo2, hi2) from host copies of the type bytes and of the
// NEE-link masks k_flag_fluid wrote (the masks the kernels read, so the gathered boundary
// records are indexed exactly as the kernels index them)
int build_range(lbm_ctx* c, Range& r, int64_t lo, int64_t hi, const std::vector<uint8_t>& t,
                const std::vector<uint32_t>& nlk, int64_t lo2 = 0, int64_t hi2 = 0, const CompactView* cv = nullptr,
                bool single = false) {
  if (lo2 < hi) lo2 = hi2 = 0;  // overlapping second interval (single-plane slab): drop it
  r.c_lo = lo;
  r.c_hi = hi;
  r.c_lo2 = lo2;
  r.c_hi2 = hi2;
  std::vector<int> chunks, cells, cells_in_chunk_order;
  std::vector<int> nee_list;  // the NEE-adjacent cells in list order (grouped by NEE-link mask)
  std::vector<int> glist;     // the group list (group-list ranges)
  auto in = [&](int64_t k) { return (k >= lo && k < hi) || (k >= lo2 && k < hi2); };
  // Chunk waves also take the NEE-adjacent cells (nee_chunks) when those mostly share their
  // 4-cell group with other fluid cells -- the pipe's rows along y, vessel trees: each such
  // group would otherwise store cell by cell, and every wave holding one would issue both store
  // paths (C3 -0.6%, C4 x4 -1.6% in interleaved A/B, profiles/r04_nee_chunks_ab.log).  Groups
  // made only of NEE-adjacent cells (the cavity's lid rows) stay with the NEE blocks: there the
  // chunk waves would load and store whole extra rows (LDC 512^3 +1%).
  {
    int64_t mixed = 0, pure = 0;
    for (int64_t g = (lo & ~int64_t(3)); g < std::max(hi, hi2); g += 4) {
      int nee = 0, other = 0;
      for (int64_t k = g; k < g + 4; ++k) {
        if (!in(k) || (t[k] & kClassMask) != kFluid) continue;
        if (t[k] & kNeeAdj) ++nee;
        else ++other;
      }
      if (nee) ++(other ? mixed : pure);
    }
    r.nee_chunks = mixed > pure;
  }
  auto scan = [&](int64_t a, int64_t b) {
    for (int64_t ch = a / kChunk; ch * kChunk < b; ++ch) {
      if (!chunks.empty() && chunks.back() >= (int)ch) continue;  // chunk shared by both intervals
      bool any = false;
      for (int64_t k = ch * kChunk; k < (ch + 1) * kChunk; ++k) {
        if (!in(k)) continue;
        const uint8_t v = t[k];
        if ((v & kClassMask) != kFluid) continue;
        any = true;
        if (v & kNeeAdj) cells.push_back((int)k);
      }
      if (any) chunks.push_back((int)ch);
    }
  };
  scan(lo, hi);
  if (hi2 > lo2) scan(lo2, hi2);
  cells_in_chunk_order = cells;
  r.nchunks = (int)chunks.size();
  r.chunk0 = chunks.empty() ? -1 : chunks[0];
  for (size_t i = 1; i < chunks.size() && r.chunk0 >= 0; ++i)
    if (chunks[i] != chunks[0] + (int)i) r.chunk0 = -1;
  if (r.nchunks) {
    HIPCK(c, hipMalloc(&r.chunks, sizeof(int) * r.nchunks));
    HIPCK(c, hipMemcpy(r.chunks, chunks.data(), sizeof(int) * r.nchunks, hipMemcpyHostToDevice));
  }
  bool group1 = false;  // a sparse list too short for the 4-cell path: one-cell group list
  {
    const int cpl = g_tune[LBM_TUNE_CELLS_PER_LANE];  // A/B switch: 1 or 4 (0: by size)
    r.quarter = cpl ? (cpl == 1) : (r.nchunks <= kQuarterMaxChunks);
    // The 4-cell path wants several rounds of resident waves (two per SIMD): a range of at
    // most kQuarterMaxChunks waves runs one cell per lane (four per SIMD), and the same
    // count decides for a sparse list that would take the 4-cell group list -- its waves are
    // its active groups / 64.  The coronary tree (3.9k such waves): 58.8 -> 42.3 us per step
    // one cell per lane; the upsampled bifurcation (15k) keeps four cells per lane (+2% the
    // other way; profiles/r03_groups1_ab.log).
    const int gm = g_tune[LBM_TUNE_GROUPS];
    if (cv) {
      r.quarter = group1 = cv->quarter;
    } else if (!cpl && !r.quarter && r.chunk0 < 0 && gm != 1) {
      int64_t active = 0;
      for (int ch : chunks)
        for (int l = 0; l < 64; ++l) {
          bool any = false;
          for (int k = 0; k < 4; ++k) {
            const int64_t cell = (int64_t)ch * kChunk + 4 * l + k;
            any |= in(cell) && (t[cell] & kClassMask) == kFluid && (r.nee_chunks || !(t[cell] & kNeeAdj));
          }
          active += any;
        }
      const double fill4 = (double)active / (64.0 * (double)r.nchunks);
      if ((gm == 2 || fill4 < 0.75) && (active + 63) / 64 <= kQuarterMaxChunks) r.quarter = group1 = true;
    }
  }
  // 4-cell ranges: the NEE values of the NEE-adjacent cells go to NEE blocks, one cell per
  // thread.  In a chunk wave each would add two dependent load rounds (its NEE-link mask, then
  // its neighbours' boundary data) to the whole wave -- on the pipe with rows along y, to every
  // wave.  One-cell waves load the link mask with the pulls and keep them (the boundary data
  // arrives under the arithmetic).
  double contig = 1.0;
  if (r.quarter) cells.clear();
  // the NEE-link mask of k_flag_fluid: q crosses the NEE neighbour's face (e_q . n == 1)
  auto nl_of = [&](int64_t cell) { return nlk[cell]; };
  r.n_nee = (int)cells.size();
  if (r.n_nee) {
    std::vector<uint32_t> nl(cells.size());
    for (size_t i = 0; i < cells.size(); ++i) nl[i] = nl_of(cells[i]);
    // group cells with the same directions (inlet / outlet / lid faces, edges) so that the
    // lanes of a wave take the same branches; cell order within a group
    std::vector<size_t> perm(cells.size());
    for (size_t i = 0; i < perm.size(); ++i) perm[i] = i;
    std::stable_sort(perm.begin(), perm.end(), [&](size_t x, size_t y) { return nl[x] < nl[y]; });
    std::vector<int> sc(cells.size());
    std::vector<uint32_t> snl(cells.size());
    for (size_t i = 0; i < perm.size(); ++i) {
      sc[i] = cells[perm[i]];
      snl[i] = nl[perm[i]];
    }
    nee_list = sc;
    int64_t adj = 0;  // list neighbours that are storage neighbours (their lanes share lines)
    for (size_t i = 1; i < sc.size(); ++i) adj += sc[i] == sc[i - 1] + 1;
    if (sc.size() > 1) contig = (double)adj / (double)(sc.size() - 1);
    HIPCK(c, hipMalloc(&r.cells, sizeof(int) * r.n_nee));
    HIPCK(c, hipMemcpy(r.cells, sc.data(), sizeof(int) * r.n_nee, hipMemcpyHostToDevice));
    HIPCK(c, hipMalloc(&r.cell_nl, sizeof(uint32_t) * r.n_nee));
    HIPCK(c, hipMemcpy(r.cell_nl, snl.data(), sizeof(uint32_t) * r.n_nee, hipMemcpyHostToDevice));
    // the boundary cells' data is written by classification and never changes afterwards
    // (gathered from the dense arrays: compact cells are translated first)
    HIPCK(c, hipMalloc(&r.nee_bc, sizeof(float4) * kNeeSlots * r.n_nee));
    DevScratch dense_ids;
    const int* gather_ids = r.cells;
    if (cv) {
      std::vector<int> dsc(sc.size()), rows(sc.size());
      for (size_t i = 0; i < sc.size(); ++i) {
        dsc[i] = (*cv->dense_of)[sc[i]];
        rows[i] = (*cv->row_of)[sc[i] >> 2];
      }
      int* p = nullptr;
      RCK(upload(c, &p, dsc));
      dense_ids.p = p;
      gather_ids = p;
      RCK(upload(c, &r.cell_row, rows));
    }
    HIPCK(c, launch_nee_gather(gather_ids, r.cell_nl, c->rho, c->ux, c->uy, c->uz, r.nee_bc, r.n_nee, c->L.pitch,
                               c->L.plane, c->L.swap, c->s_comp));
    HIPCK(c, hipStreamSynchronize(c->s_comp));
  }
  // Lane masks for the 4-cell path: bit l of a chunk's mask is set when lane l (cells 4l ..
  // 4l+3) holds a cell the chunk wave updates (fluid, in range, not NEE-adjacent unless
  // nee_chunks) or neighbours
  // such a lane (the DPP x-shift reads the next lanes' slices).  Lanes outside it load nothing:
  // on a vessel tree most chunks are partly empty (the upsampled bifurcation keeps 51% of its
  // active chunks' cells).  Only for sparse chunk lists, whose waves load their chunk id
  // anyway (the mask load goes out beside it); a contiguous list would pay a round trip.
  // One-cell ranges have no masks (their idle lanes load nothing new: a wave's cells share
  // lines); their fill -- cells to update over the active chunks' cells -- picks the group list.
  auto updated = [&](int64_t cell) {
    const uint8_t v = t[cell];
    return in(cell) && (v & kClassMask) == kFluid && (r.quarter || r.nee_chunks || !(v & kNeeAdj));
  };
  if (r.nchunks && r.chunk0 < 0 && !cv) {
    std::vector<unsigned long long> lm(chunks.size());
    bool partial = false;
    int64_t busy = 0, cells_busy = 0;
    for (size_t j = 0; j < chunks.size(); ++j) {
      unsigned long long m = 0;
      const int64_t base = (int64_t)chunks[j] * kChunk;
      for (int l = 0; l < 64; ++l)
        for (int k = 0; k < 4; ++k)
          if (updated(base + 4 * l + k)) {
            m |= 1ull << l;
            ++cells_busy;
          }
      busy += __builtin_popcountll(m);
      m |= (m << 1) | (m >> 1);
      lm[j] = m;
      partial |= m != ~0ull;
    }
    r.lane_fill = chunks.empty() ? 1.0
                  : r.quarter    ? (double)cells_busy / ((double)kChunk * (double)chunks.size())
                                 : (double)busy / (64.0 * (double)chunks.size());
    if (!r.quarter && (partial || g_tune[LBM_TUNE_GRID_STRIDE] >= 2)) {  // the loop kernel reads them
      HIPCK(c, hipMalloc(&r.lane_masks, sizeof(unsigned long long) * lm.size()));
      HIPCK(c, hipMemcpy(r.lane_masks, lm.data(), sizeof(unsigned long long) * lm.size(), hipMemcpyHostToDevice));
    }
  }
  r.main_blocks = main_grid(r.nchunks, r.quarter);
  // Compact 4-cell groups (LBM_TUNE_GROUPS): on a sparse chunk list whose lanes are mostly idle
  // (vessel trees), the wave's VALU work is the same whether a lane holds a cell or not, so
  // idle lanes cost issue time.  The groups holding a cell to update go into one compact list
  // in storage order, 64 per 4-cell wave (16 per one-cell wave); runs of neighbouring groups
  // keep their loads and stores
  // contiguous, and a group whose list neighbour is not its row neighbour loads its x-edge
  // cells itself (pull_issue).
  if (cv && r.quarter) {
    // compact rows, one cell per lane: no list -- wave w takes the compact cells from
    // (lo & ~63) + 64 w (process_compact_cell1); the boundary records of the NEE-adjacent cells
    // by compact group (group_bc), gathered from the dense arrays
    const int64_t base = lo & ~int64_t(63), waves = (hi - base + 63) / 64;
    constexpr int wpb = kBlock1c / 64;  // k_step1c's workgroups
    r.main_blocks = waves ? (int)std::max<int64_t>(8, ((waves + wpb - 1) / wpb + 7) / 8 * 8) : 0;
    int64_t fl = 0;
    for (int64_t k = lo; k < hi; ++k) fl += (t[k] & kClassMask) == kFluid;
    r.group_fill = hi > base ? (double)fl / (double)(64 * waves) : 1.0;
    if (!c->bc_uniform) {
      std::vector<int> gbc((size_t)(t.size() / 4), -1), gcells;
      std::vector<uint32_t> gnl;
      auto nee_adj = [&](int64_t k) { return in(k) && (t[k] & kClassMask) == kFluid && (t[k] & kNeeAdj); };
      int nrec = 0;
      for (int64_t g = base / 4; g < (hi + 3) / 4; ++g) {
        if (!(nee_adj(4 * g) || nee_adj(4 * g + 1) || nee_adj(4 * g + 2) || nee_adj(4 * g + 3))) continue;
        gbc[g] = nrec++;
        for (int64_t j = 4 * g; j < 4 * g + 4; ++j) {
          gcells.push_back(std::max(0, (*cv->dense_of)[j]));
          gnl.push_back(nee_adj(j) ? nl_of(j) : 0u);
        }
      }
      if (nrec) {
        DevScratch dc, dn;
        RCK(upload(c, &r.group_bc, gbc));
        HIPCK(c, hipMalloc(&r.group_rec, sizeof(float4) * kNeeSlots * gcells.size()));
        int* pc = nullptr;
        uint32_t* pn = nullptr;
        RCK(upload(c, &pc, gcells));
        dc.p = pc;
        RCK(upload(c, &pn, gnl));
        dn.p = pn;
        HIPCK(c, launch_nee_gather(pc, pn, c->rho, c->ux, c->uy, c->uz, r.group_rec, (int)gcells.size(), c->L.pitch,
                                   c->L.plane, c->L.swap, c->s_comp));
        HIPCK(c, hipStreamSynchronize(c->s_comp));
      }
    }
  } else {
    const int gm = g_tune[LBM_TUNE_GROUPS];
    const bool sparse = r.quarter ? r.lane_fill < kGroupFill1 : r.lane_masks && r.lane_fill < 0.75;
    const bool want = cv || gm == 2 || (gm == 0 && (sparse || group1));
    if (r.nchunks && (r.chunk0 < 0 || cv) && want) {
      // segments of seg groups (LBM_TUNE_GROUP_SEGMENT, default 16 = two 128-B lines of a chunk
      // slice): a segment with an active group enters the list whole, its idle groups marked
      // (bit 0) so their lanes load nothing.  Whole lines per wave load beat full lanes on the
      // coronary tree (59 vs 73 us per step with single groups), and cost the upsampled
      // bifurcation, whose runs are long anyway, 3% (profiles/r03_groups_ab.log); with plain
      // loads (round 5) 16 groups beat 8 on C4 x4, 133.1 -> 131.8 us (r05_c4x4_segment_ab.log)
      const int seg = std::max(1, g_tune[LBM_TUNE_GROUP_SEGMENT]);
      std::vector<int> gl;
      int64_t cells_in = 0;
      for (int ch : chunks)
        for (int l0 = 0; l0 < 64; l0 += seg) {
          int nseg = 0, ng[64];
          for (int l = l0; l < l0 + seg && l < 64; ++l) {
            int n = 0;
            for (int k = 0; k < 4; ++k) n += updated((int64_t)ch * kChunk + 4 * l + k);
            ng[l - l0] = n;
            nseg += n;
          }
          if (!nseg) continue;
          for (int l = l0; l < l0 + seg && l < 64; ++l) gl.push_back(ch * kChunk + 4 * l + (ng[l - l0] ? 0 : 1));
          cells_in += nseg;
        }
      r.ngroups = (int64_t)gl.size();
      glist = gl;
      r.group_fill = gl.empty() ? 1.0 : (double)cells_in / (4.0 * (double)gl.size());
      if (r.ngroups) {
        HIPCK(c, hipMalloc(&r.groups, sizeof(int) * gl.size()));
        HIPCK(c, hipMemcpy(r.groups, gl.data(), sizeof(int) * gl.size(), hipMemcpyHostToDevice));
        if (cv) {
          std::vector<int> rows(gl.size());
          for (size_t i = 0; i < gl.size(); ++i) rows[i] = (*cv->row_of)[gl[i] >> 2];
          RCK(upload(c, &r.group_row, rows));
        }
      }
      // one-cell waves: the boundary records of the groups holding NEE-adjacent cells, gathered
      // once and indexed by list entry (process_group_cell1 loads them with the pulls)
      if (r.quarter && r.ngroups && !c->bc_uniform) {
        std::vector<int> gbc(gl.size(), -1), gcells;
        std::vector<uint32_t> gnl;
        auto nee_adj = [&](int64_t k) { return in(k) && (t[k] & kClassMask) == kFluid && (t[k] & kNeeAdj); };
        int nrec = 0;
        for (size_t i = 0; i < gl.size(); ++i) {
          if (gl[i] & 1) continue;
          const int64_t g = gl[i];
          if (!(nee_adj(g) || nee_adj(g + 1) || nee_adj(g + 2) || nee_adj(g + 3))) continue;
          gbc[i] = nrec++;
          for (int64_t j = g; j < g + 4; ++j) {
            // the records are gathered from the dense arrays: compact cells translated
            gcells.push_back(cv ? std::max(0, (*cv->dense_of)[j]) : (int)j);
            gnl.push_back(nee_adj(j) ? nl_of(j) : 0u);
          }
        }
        if (nrec) {
          DevScratch dc, dn;
          HIPCK(c, hipMalloc(&r.group_bc, sizeof(int) * gbc.size()));
          HIPCK(c, hipMemcpy(r.group_bc, gbc.data(), sizeof(int) * gbc.size(), hipMemcpyHostToDevice));
          HIPCK(c, hipMalloc(&r.group_rec, sizeof(float4) * kNeeSlots * gcells.size()));
          HIPCK(c, hipMalloc(&dc.p, sizeof(int) * gcells.size()));
          HIPCK(c, hipMalloc(&dn.p, sizeof(uint32_t) * gnl.size()));
          HIPCK(c, hipMemcpy(dc.p, gcells.data(), sizeof(int) * gcells.size(), hipMemcpyHostToDevice));
          HIPCK(c, hipMemcpy(dn.p, gnl.data(), sizeof(uint32_t) * gnl.size(), hipMemcpyHostToDevice));
          HIPCK(c, launch_nee_gather(static_cast<const int*>(dc.p), static_cast<const uint32_t*>(dn.p), c->rho, c->ux,
                                     c->uy, c->uz, r.group_rec, (int)gcells.size(), c->L.pitch, c->L.plane, c->L.swap,
                                     c->s_comp));
          HIPCK(c, hipStreamSynchronize(c->s_comp));
        }
      }
      const int64_t waves = (r.ngroups + (r.quarter ? 15 : 63)) / (r.quarter ? 16 : 64);
      r.main_blocks = waves ? (int)std::max<int64_t>(8, ((waves + kBlock / 64 - 1) / (kBlock / 64) + 7) / 8 * 8) : 0;
    }
  }
  // Sparse chunk lists loop: a partly empty chunk is too little work for a wave of its own
  // (the upsampled bifurcation: +12% with two blocks per CU looping over their XCD's chunks).
  // Full chunks do not: boxes and the pipe run 10-13% slower that way (lockstep waves,
  // profiles/r02_grid_stride_ab.log), so they keep one chunk per wave.
  const int gs = g_tune[LBM_TUNE_GRID_STRIDE];
  // group lists loop with four blocks per CU by default (interleaved A/B: C4 x4 -3.7%, coronary
  // tree -0.6% against one list slice per wave; profiles/r03_groups_ab.log)
  const int per_cu = gs >= 2 ? gs : gs == 1 ? 0 : r.groups ? 4 : (r.lane_masks && r.lane_fill < 0.75) ? 2 : 0;
  if ((r.quarter ? r.groups && gs >= 2 : (r.lane_masks || r.groups)) && per_cu > 0) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->d.device) != hipSuccess || cus <= 0)
      cus = 256;
    const int cap = (cus * per_cu + 7) / 8 * 8;
    if (r.main_blocks > cap) {
      r.main_blocks = cap;
      r.stride = true;
    }
  }
  if (r.quarter) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->d.device) != hipSuccess || cus <= 0)
      cus = 256;
    const int64_t waves = (int64_t)r.main_blocks * ((cv ? kBlock1c : kBlock) / 64);  // four per SIMD fit
    r.one_round = waves <= (int64_t)cus * 16;
  }
  r.nee_waves = nee_waves_for(r.n_nee, contig);
  r.nee_blocks = nee_grid(r.n_nee, r.nee_waves);
  // the single-domain range of a lattice whose chunk waves collide the NEE-adjacent cells: the NEE
  // values from NEE blocks in the step launch that pull and collide every such cell again
  // (LBM_TUNE_NEE_FIX 0 / 1), from k_nee_fix after the step launch (3), or from NEE records (2).
  // Round 6, interleaved A/B at head (profiles/r06c_nee_modes_ab.log): NEE blocks C3 178.8 us per
  // step against 187.4 with k_nee_fix, C4 x4 131.0 against 132.5 -- dispatched first, the NEE
  // blocks' scattered work runs while the chunk waves' first round still ramps up; k_nee_fix
  // pays a launch of its own (round 5 measured 184.6 vs 183.7 before the pipe's round-robin XCD
  // order)
  const int nee_mode = g_tune[LBM_TUNE_NEE_FIX];
  if (single && !r.quarter && r.nee_chunks && r.n_nee > 0 && (nee_mode == 2 || nee_mode == 3)) {
    r.nee_fix = true;
    r.nee_blocks = 0;
  }
  // NEE records where the chunk waves run over a chunk list of the dense box and every chunk
  // holds at most kNeeRecMax NEE-adjacent cells of at most kNeeRecDirs NEE directions (the pipe
  // along y: one per chunk); k_nee_fix elsewhere
  if (r.nee_fix && !cv && !r.groups && !r.lane_masks && !r.stride && r.nchunks > 0 && g_tune[LBM_TUNE_NEE_FIX] == 2) {
    const std::vector<int>& co = cells_in_chunk_order;
    std::vector<int> base(r.nchunks + 1), pos(co.size());
    std::vector<uint32_t> nlv(co.size());
    bool ok = true;
    size_t k = 0;
    for (int i = 0; i < r.nchunks && ok; ++i) {
      base[i] = (int)k;
      while (k < co.size() && co[k] / kChunk == chunks[i]) {
        pos[k] = co[k] % kChunk;
        nlv[k] = nl_of(co[k]);
        ok &= __builtin_popcount(nlv[k]) <= kNeeRecDirs;
        ++k;
      }
      ok &= (int)k - base[i] <= kNeeRecMax;
      r.nee_rec_max = std::max(r.nee_rec_max, (int)k - base[i]);
    }
    base[r.nchunks] = (int)k;
    if (ok && k == co.size()) {
      DevScratch dc, dp, dn;
      int* pc = nullptr;
      int* pp = nullptr;
      uint32_t* pn = nullptr;
      RCK(upload(c, &pc, co));
      dc.p = pc;
      RCK(upload(c, &pp, pos));
      dp.p = pp;
      RCK(upload(c, &pn, nlv));
      dn.p = pn;
      RCK(upload(c, &r.nee_rec_base, base));
      r.n_rec = (int)co.size();
      HIPCK(c, hipMalloc(&r.nee_rec, sizeof(float4) * kNeeRecF4 * r.n_rec));
      HIPCK(c, launch_nee_records(pc, pp, pn, c->rho, c->ux, c->uy, c->uz, r.nee_rec, r.n_rec, c->L.pitch, c->L.plane,
                                  c->L.swap, c->s_comp));
      HIPCK(c, hipStreamSynchronize(c->s_comp));
      r.nee_records = true;
      r.nee_fix = false;
    } else {
      r.nee_rec_max = 0;
    }
  }
  // k_nee_fix's (rho, u) records (lbm_ctx::nee_mac): one slot per NEE-adjacent cell in storage
  // order -- the chunk waves number them from their work unit's first slot (nee_mac_base) and their
  // cells' ranks in the wave, k_nee_fix by list entry (cell_mac).  cells_in_chunk_order is
  // ascending: the chunks, and the cells in each, are scanned in storage order
  if (r.nee_fix) {
    const std::vector<int>& co = cells_in_chunk_order;
    for (size_t i = 1; i < co.size(); ++i)
      if (co[i] <= co[i - 1]) {
        c->err = "build_range: NEE-adjacent cells out of storage order";
        return LBM_ERR_STATE;
      }
    auto slot_of = [&](int64_t cell) { return (int)(std::lower_bound(co.begin(), co.end(), cell) - co.begin()); };
    std::vector<int> base, cm(nee_list.size());
    if (r.groups) {
      for (int64_t b = 0; b * 64 < r.ngroups; ++b) base.push_back(slot_of(glist[b * 64] & ~3));
    } else {
      for (int i = 0; i < r.nchunks; ++i) base.push_back(slot_of((int64_t)chunks[i] * kChunk));
    }
    for (size_t i = 0; i < nee_list.size(); ++i) cm[i] = slot_of(nee_list[i]);
    RCK(upload(c, &r.nee_mac_base, base));
    RCK(upload(c, &r.cell_mac, cm));
  }
  // Where the NEE blocks go in the grid (LBM_TUNE_NEE_ORDER).  Grid-stride group lists (C4 x4):
  // after the chunk blocks -- each loop wave's share of the list is fixed, so NEE blocks dispatched
  // first made the loop's first workgroups start, and end, late; trailing, they fill the slots the
  // loop's uneven end leaves idle (125.2 vs 130.7 us per step).  Chunk lists (C3): first, where
  // they fill the first generation's load phase (trailing: 184.6 vs 176.8; profiles/r06q_nee_order_waves_ab.log)
  {
    const int order = g_tune[LBM_TUNE_NEE_ORDER];
    r.nee_last = r.nee_blocks > 0 && (order == 2 || (order == 0 && r.groups && r.stride));
  }
  r.npart = r.main_blocks + r.nee_blocks;
  return LBM_OK;
}

void free_range(Range& r) {
  if (r.chunks) (void)hipFree(r.chunks);
  if (r.lane_masks) (void)hipFree(r.lane_masks);
  if (r.groups) (void)hipFree(r.groups);
  if (r.group_bc) (void)hipFree(r.group_bc);
  if (r.group_rec) (void)hipFree(r.group_rec);
  if (r.cells) (void)hipFree(r.cells);
  if (r.group_row) (void)hipFree(r.group_row);
  if (r.cell_row) (void)hipFree(r.cell_row);
  if (r.cell_nl) (void)hipFree(r.cell_nl);
  if (r.nee_rec_base) (void)hipFree(r.nee_rec_base);
  if (r.nee_mac_base) (void)hipFree(r.nee_mac_base);
  if (r.cell_mac) (void)hipFree(r.cell_mac);
  if (r.nee_rec) (void)hipFree(r.nee_rec);
  if (r.nee_bc) (void)hipFree(r.nee_bc);
  r = Range{};
}

// Compact rows: a population buffer in the dense box layout for set-up and read-out (stage:
// L.buf_floats() floats, the returned pointer past the guard), filled from compact buffer b
// (to_dense) or copied into compact buffer b (from_dense)
struct Stage {
  float* alloc = nullptr;
  ~Stage() {
    if (alloc) (void)hipFree(alloc);
  }
};
int stage_dense(lbm_ctx* c, Stage& st, float** base) {
  HIPCK(c, hipMalloc(&st.alloc, sizeof(float) * c->L.buf_floats()));
  HIPCK(c, hipMemsetAsync(st.alloc, 0, sizeof(float) * c->L.buf_floats(), c->s_comp));
  *base = st.alloc + c->L.guard * kQ * kChunk;
  return LBM_OK;
}
int to_dense(lbm_ctx* c, int b, float* dense) {
  HIPCK(c, launch_pop_compact(dense, c->buf[b], c->cmap, c->ncell_c, 0, c->s_comp));
  return LBM_OK;
}
int from_dense(lbm_ctx* c, const float* dense, int b) {
  HIPCK(c, launch_pop_compact(c->buf[b], dense, c->cmap, c->ncell_c, 1, c->s_comp));
  return LBM_OK;
}

int ensure_hist(lbm_ctx* c, int n) {
  if (n <= c->hist_cap) return LBM_OK;
  if (c->hist) HIPCK(c, hipFree(c->hist));
  c->hist_cap = std::max(n, 1024);
  HIPCK(c, hipMalloc(&c->hist, sizeof(float) * c->hist_cap));
  return LBM_OK;
}

// fresh main-loop state (k = 0, sum_current = 0) keeping the convergence settings
int reset_state(lbm_ctx* c) {
  ConvState cs{}, host{};
  HIPCK(c, hipMemcpy(&host, c->conv, sizeof(ConvState), hipMemcpyDeviceToHost));
  cs.enabled = host.enabled;
  cs.max_it = host.max_it;
  cs.stag_max = host.stag_max;
  cs.tol = host.tol;
  HIPCK(c, hipMemcpy(c->conv, &cs, sizeof(ConvState), hipMemcpyHostToDevice));
  if (c->bb_immediate) {  // LDC: walls already bounce back at step 0 (ldc.cu:75-202)
    float* f = c->buf[0];
    Stage st;
    if (c->compact) {  // on a dense copy of buffer 0
      RCK(stage_dense(c, st, &f));
      RCK(to_dense(c, 0, f));
    }
    HIPCK(c, launch_bb_prime(f, c->type, c->links, c->L.ncell, c->L.pitch, c->L.plane, c->L.swap, c->s_comp));
    if (c->compact) RCK(from_dense(c, f, 0));
    HIPCK(c, hipStreamSynchronize(c->s_comp));
  }
  c->steps_done = 0;
  c->cur = 0;
  c->halo_primed = false;
  c->macros_stale = false;
  c->walls_stale = false;
  c->nee_stale = false;
  return LBM_OK;
}

// The NEE cells' slots a run of NEE-record steps left unwritten (lbm_ctx::nee_stale), from the
// records, before anything reads them as the producer side stores them: buf[cur], the next
// step's source, gets the values of the last step (k - 1); buf[cur ^ 1], the last step's source
// (the lazy macros), those of step k - 2 -- except after a single step, whose source holds the raw
// initial slots step 0 pulls.
int materialize_nee(lbm_ctx* c) {
  if (!c->nee_stale) return LBM_OK;
  const Range& r = c->whole;
  const int64_t per = (int64_t)r.n_rec * 8;
  const int k = c->steps_done;
  if (k >= 1)
    HIPCK(c, launch_nee_materialize(c->buf[c->cur], r.nee_rec, c->nee_val + ((k - 1) & 1) * per, r.n_rec, c->L.pitch,
                                    c->L.plane, c->L.swap, 1, c->s_comp));
  if (k >= 2)
    HIPCK(c, launch_nee_materialize(c->buf[c->cur ^ 1], r.nee_rec, c->nee_val + ((k - 2) & 1) * per, r.n_rec,
                                    c->L.pitch, c->L.plane, c->L.swap, 1, c->s_comp));
  HIPCK(c, hipStreamSynchronize(c->s_comp));
  c->nee_stale = false;
  return LBM_OK;
}

// Restore the wall slots a consumer-side step left unwritten (lbm_ctx::walls_stale) before a
// producer-side reader pulls them: in both buffers, slot q of wall W = c - e_q gets cell c's own
// slot opp(q) of the same buffer -- the value the producer side stores there (its post-collision
// f_opp(q), Poiseulle.cu:601-746).  buf[cur] feeds the next step; buf[cur ^ 1], the last step's
// source, feeds the lazy macros -- except after a single raw first step (no bounce-back at step
// 0, MainArgs::bb_raw), whose source keeps its initial wall slots.  Compact rows always bounce
// back on the consumer side and never get here.
int prime_walls(lbm_ctx* c) {
  if (!c->walls_stale || c->compact) return LBM_OK;
  const Layout& L = c->L;
  HIPCK(c, launch_bb_prime(c->buf[c->cur], c->type, c->links, L.ncell, L.pitch, L.plane, L.swap, c->s_comp));
  if (c->steps_done >= 2 || c->bb_immediate)
    HIPCK(c, launch_bb_prime(c->buf[c->cur ^ 1], c->type, c->links, L.ncell, L.pitch, L.plane, L.swap, c->s_comp));
  HIPCK(c, hipStreamSynchronize(c->s_comp));
  c->walls_stale = false;
  return LBM_OK;
}

// Population buffers: two allocations of `bytes`, picked by measured write rate.
//
// HBM write bandwidth is a property of the physical memory an allocation receives: on the pool's
// MI355X boxes a 10-GB allocation sweep-writes at either ~6.3-6.5 or ~5.5 TB/s, stable for the
// allocation's lifetime and the same for every sweep order (one region per XCD, grid-stride,
// reversed or rotated regions), while reads differ by < 4% (tools/place_lab.hip,
// gpurun_out/r02g-i).  A copy runs at its destination's rate, and k_step writes one buffer per
// step, so a slow buffer costs every other step ~8% (the 3.4 / 3.7 ms alternation at 512^3).
// When the device has room (hipMemGetInfo, after `others` bytes for the remaining arrays), up to
// fourteen extra candidates are allocated, each zeroed and timed over one full-buffer sweep of
// non-temporal 16-B stores; of the four fastest, the pair whose tile copies both ways are
// quickest is kept, and the rest are freed before any other array is allocated.  Every buffer larger than the 256-MB MALL is probed (round 4 probed only
// buffers >= 1 GiB, so the 647-MB buffers of the C3 pipe took whatever came first); smaller
// ones (MALL resident, latency-bound) and LBM_TUNE_BUFFER_ALLOC = 1 take the first two
// allocations (the latter still timed, for A/B).
// The candidates take at most kPlacementBudget bytes together (16 at 512^3: 3297.7 against
// 3336.6 us per step with the round-4 budget's six, profiles/r05s_placement.log) and number at most
// kMaxCand: at LDC 256^3 (1.28-GB buffers) one or two of six candidates wrote at ~6.1 TB/s and
// the rest at 4.9-5.6, so the step that writes the slower kept buffer ran 433 instead of 422 us,
// and the first two allocations (no probe) 457 us (gpurun_out/r05a, tools/ab_alloc.py); more
// candidates make a pair of fast ones likelier.
// Ranks equal-sized candidate allocations p (zeroed) by one timed write sweep each (gbs: GB/s,
// allocation order) and picks two: with pair_probe, among the four fastest writers the pair whose
// copies both ways -- k_step's 16-KB wave tiles, one buffer read, the other written -- take the
// least time together (LDC 256^3 in one process, four fresh lattices each: 422.9 against 427.7 us
// per step for the two fastest writers, profiles/r05s_placement.log); else the two fastest.
hipError_t rank_pair(const std::vector<void*>& p, size_t bytes, hipStream_t st, bool pair_probe,
                     std::vector<double>& gbs, int& ka, int& kb) {
  const int n = (int)p.size();
  const int64_t n4 = (int64_t)(bytes / 16);
  hipEvent_t e0 = nullptr, e1 = nullptr;
  hipError_t e = hipEventCreate(&e0);
  if (e == hipSuccess) e = hipEventCreate(&e1);
  auto timed_ms = [&](auto&& launch, int reps, float& ms) {
    e = launch();  // warm-up (the memset's shape differs)
    if (e == hipSuccess) e = hipEventRecord(e0, st);
    for (int r = 0; r < reps && e == hipSuccess; ++r) e = launch();
    if (e == hipSuccess) e = hipEventRecord(e1, st);
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
  };
  gbs.clear();
  for (int i = 0; i < n && e == hipSuccess; ++i) {
    float ms = 0.f;
    timed_ms([&] { return launch_probe_fill(p[i], n4, st); }, 1, ms);
    gbs.push_back(ms > 0.f ? (double)bytes / (ms * 1e-3) / 1e9 : 0.0);
  }
  std::vector<int> order(n);
  for (int i = 0; i < n; ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return gbs[a] > gbs[b]; });
  ka = order[0];
  kb = order[1];
  if (pair_probe && n > 2 && e == hipSuccess) {
    const int K = std::min(n, 4);
    const int64_t t4 = (int64_t)(bytes / 65536) * 4096;
    float t[4][4] = {};
    for (int i = 0; i < K && e == hipSuccess; ++i)
      for (int j = 0; j < K && e == hipSuccess; ++j)
        if (i != j) timed_ms([&] { return launch_probe_copy(p[order[i]], p[order[j]], t4, 0, 6, st); }, 2, t[i][j]);
    float best = 0.f;
    for (int i = 0; i < K; ++i)
      for (int j = i + 1; j < K; ++j)
        if (best == 0.f || t[i][j] + t[j][i] < best) {
          best = t[i][j] + t[j][i];
          ka = order[i];
          kb = order[j];
        }
  }
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  return e;
}

constexpr size_t kPlacementMinBytes = (size_t)256 << 20;
constexpr size_t kPlacementBudget = (size_t)160 << 30;
hipError_t buffer_placement(lbm_ctx* c, size_t bytes, size_t others) {
  // up to 64 candidates (round 6): on a box whose sixteen 1.28-GB candidates all wrote at <= 5.5 TB/s
  // (LDC 256^3 457-462 us per step), 48 found 5.8-6.1 TB/s pairs (422-426 us) in five rounds of
  // fresh processes; 128 were no better than 64 (profiles/r06k_placement48_ab.log,
  // r06l_placement64_vs128_ab.log)
  constexpr int kMaxCand = 64;
  int ncand = 2;
  const bool probe = bytes > kPlacementMinBytes;
  if (g_tune[LBM_TUNE_BUFFER_ALLOC] != 1 && probe) {
    size_t fr = 0, tot = 0;
    hipError_t e = hipMemGetInfo(&fr, &tot);
    if (e != hipSuccess) return e;
    const size_t need = 2 * bytes + others;
    // at most kPlacementBudget, and a quarter of the free memory stays free while the candidates
    // are held (a device shared with other contexts or processes)
    const size_t budget = std::min(kPlacementBudget, fr / 4 * 3);
    const int cap = (int)std::max<size_t>(2, std::min<size_t>(kMaxCand, budget / bytes));
    if (fr > need) ncand = (int)std::min<size_t>(cap, 2 + (fr - need) / bytes);
  }
  std::vector<void*> p;
  hipError_t e = hipSuccess;
  for (int i = 0; i < ncand && e == hipSuccess; ++i) {
    void* q = nullptr;
    e = hipMalloc(&q, bytes);
    if (e != hipSuccess) {
      if (i >= 2) {  // out of room after all: probe what we have
        (void)hipGetLastError();
        e = hipSuccess;
        ncand = i;
      }
      break;
    }
    p.push_back(q);
    e = hipMemsetAsync(q, 0, bytes, c->s_comp);
  }
  {  // the set-up's low point of free device memory: every candidate held (lbm_get_setup_cost)
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess) c->mem_free_min = std::min(c->mem_free_min, fr);
  }
  if (e == hipSuccess && probe) {
    int ka = 0, kb = 1;
    e = rank_pair(p, bytes, c->s_comp, g_tune[LBM_TUNE_BUFFER_ALLOC] == 0, c->cand_gbs, ka, kb);
    c->chosen[0] = std::min(ka, kb);  // keep allocation order between the two
    c->chosen[1] = std::max(ka, kb);
  }
  for (int i = 0; i < (int)p.size(); ++i) {
    if (e == hipSuccess && (i == c->chosen[0] || i == c->chosen[1]))
      c->alloc[i == c->chosen[0] ? 0 : 1] = static_cast<float*>(p[i]);
    else
      (void)hipFree(p[i]);
  }
  return e;
}

// Compact rows (LBM_TUNE_COMPACT), the reference's index_transform (Poiseulle.cu:257-271,
// bifurcation.cu:241-252) done per storage row: a cell is stored when a fluid cell may read or
// write it (fluid, wall, NEE, passive cells a fluid cell pulls) or the reference stores it
// (code != 0: its ghost layer); every storage row r keeps the
// span of 4-cell groups from its first to its last stored cell, the spans packed in storage
// order, so cell (r, s0) lives at roff[r] + s0 with roff[r] = -xshift (mod 4) -- the groups and
// the x-neighbours c +- 1 of the dense box, only the rows move.  On a vessel tree the waves'
// loads then fill whole lines of the chunk slices instead of 128-B segments spread over
// half-empty chunks of the box.  Builds the compact copies of the per-cell arrays, the row
// records (MainArgs::rowrec) and the whole-domain range over compact cells; leaves c->compact
// false when the lattice does not qualify (auto: compact rows must save 40% of the slots; their
// buffers must stay under 2^31 floats for the kernels' 32-bit indices).
int floordiv4(int x) { return x >= 0 ? x / 4 : -((-x + 3) / 4); }

int build_compact(lbm_ctx* c, const std::vector<uint8_t>& t, const std::vector<uint32_t>& nlk) {
  const Layout& L = c->L;
  const int n0 = L.swap ? L.ny : L.nx, n1 = L.swap ? L.nx : L.ny;
  const int64_t R = (int64_t)L.planes * n1, nt = (int64_t)t.size();
  // the reference codes too: its stored cells (code != 0, ghosts included) keep their slots, so
  // the initial state reads back like the dense box's (lbm_get_f)
  std::vector<int8_t> codes((size_t)nt);
  HIPCK(c, hipMemcpy(codes.data(), c->codes, nt, hipMemcpyDeviceToHost));
  auto stored = [&](int64_t k) {
    const uint8_t v = t[k];
    return (v & kClassMask) != kPassive || (v & kPulled) || codes[k] != 0;
  };
  std::vector<int> roff(R, 0), glo(R, 0), ghi(R, -1), row_of;
  std::vector<int64_t> gstart(R + 1, 0);
  int64_t cum = 0;
  for (int64_t r = 0; r < R; ++r) {
    gstart[r] = cum;
    const int64_t base = r * L.pitch - L.xshift;
    int lo = -1, hi = -1;
    for (int s = 0; s < n0; ++s) {
      const int64_t k = base + s;
      if (k < 0 || k >= nt || !stored(k)) continue;
      if (lo < 0) lo = s;
      hi = s;
    }
    if (lo < 0) continue;
    glo[r] = floordiv4(lo - L.xshift);
    ghi[r] = floordiv4(hi - L.xshift);
    roff[r] = (int)(4 * (cum - glo[r]) - L.xshift);
    for (int g = glo[r]; g <= ghi[r]; ++g) row_of.push_back((int)r);
    cum += ghi[r] - glo[r] + 1;
  }
  gstart[R] = cum;
  const int64_t ncell = (4 * cum + kChunk - 1) / kChunk * kChunk, nchunk = ncell / kChunk;
  const int64_t guard = (n0 + 16 + kChunk - 1) / kChunk + 1;  // |offsets| of any lane's address
  if (cum == 0 || (nchunk + 2 * guard) * kQ * kChunk >= kCompactMaxFloats) return LBM_OK;
  if (g_tune[LBM_TUNE_COMPACT] == 0 && (double)ncell > 0.6 * (double)L.ncell) return LBM_OK;
  row_of.resize(ncell / 4, row_of.back());  // the padding groups of the last chunk: the last row
  std::vector<int> cmap(ncell, -1);
  for (int64_t r = 0; r < R; ++r) {
    if (ghi[r] < glo[r]) continue;
    const int64_t base = r * L.pitch - L.xshift;
    for (int s = 4 * glo[r] + L.xshift; s < 4 * ghi[r] + L.xshift + 4; ++s)
      if (s >= 0 && s < n0 && base + s >= 0 && base + s < nt) cmap[roff[r] + s] = (int)(base + s);
  }
  std::vector<int> rec(R * 12, 0);
  for (int64_t r = 0; r < R; ++r)
    for (int dy = -1; dy <= 1; ++dy)
      for (int dz = -1; dz <= 1; ++dz) {
        const int64_t rr = r + dy + (int64_t)dz * n1;
        rec[r * 12 + (dy + 1) * 3 + dz + 1] = (rr >= 0 && rr < R) ? roff[rr] : 0;
      }
  // Every fluid cell's 18 neighbours, addressed the kernels' way (row record + position - e_x),
  // must be exactly the compact slots of its dense neighbours: checked here, on the host, for
  // every fluid cell, so a wrong row table fails lbm_create instead of reading stray slots
  {
    int64_t off[kQ];
    for (int q = 0; q < kQ; ++q) {
      const int s0 = L.swap ? kEy[q] : kEx[q], s1 = L.swap ? kEx[q] : kEy[q];
      off[q] = s0 + (int64_t)s1 * L.pitch + (int64_t)kEz[q] * L.plane;
    }
    const int64_t lo = -guard * kChunk, hi = ncell + guard * kChunk;
    for (int64_t i = 0; i < ncell; ++i) {
      const int d = cmap[i];
      if (d < 0 || (t[d] & kClassMask) != kFluid) continue;
      const int r = row_of[i >> 2];
      const int s = (int)i - roff[r];
      for (int q = 1; q < kQ; ++q) {
        const int sx = L.swap ? kEy[q] : kEx[q], sy = L.swap ? kEx[q] : kEy[q];
        const int64_t nb = rec[(int64_t)r * 12 + (-sy + 1) * 3 + (-kEz[q] + 1)] + s - sx;
        if (nb < lo || nb >= hi || nb < 0 || nb >= ncell || cmap[nb] != d - off[q]) {
          c->err = "compact rows: neighbour table check failed at dense cell " + std::to_string(d) + ", q " +
                   std::to_string(q);
          return LBM_ERR_GEOMETRY;
        }
      }
    }
  }
  std::vector<uint8_t> tc(ncell, 0);
  std::vector<uint32_t> nlc(ncell, 0);
  for (int64_t i = 0; i < ncell; ++i)
    if (cmap[i] >= 0) {
      tc[i] = t[cmap[i]];
      nlc[i] = nlk[cmap[i]];
    }
  RCK(upload(c, &c->cmap, cmap));
  RCK(upload(c, &c->crow, row_of));
  c->cmap_h = cmap;
  {
    int* p = nullptr;
    RCK(upload(c, &p, rec));
    c->rowrec = reinterpret_cast<int4*>(p);
  }
  if (c->whole.quarter) {  // one cell per lane without a list: the row record by compact group
    std::vector<int> grec(ncell / 4 * 12);
    for (int64_t g = 0; g < ncell / 4; ++g)
      std::memcpy(&grec[g * 12], &rec[(int64_t)row_of[g] * 12], 12 * sizeof(int));
    int* p = nullptr;
    RCK(upload(c, &p, grec));
    c->grouprec = reinterpret_cast<int4*>(p);
  }
  HIPCK(c, hipMalloc(&c->ctype, ncell));
  HIPCK(c, launch_cell_gather(c->ctype, c->type, c->cmap, ncell, 1, c->s_comp));
  uint32_t** cl[2] = {&c->clinks, &c->cnlinks};
  const uint32_t* dl[2] = {c->links, c->nlinks};
  for (int k = 0; k < 2; ++k) {
    HIPCK(c, hipMalloc(cl[k], sizeof(uint32_t) * ncell));
    HIPCK(c, launch_cell_gather(*cl[k], dl[k], c->cmap, ncell, 4, c->s_comp));
  }
  float** cm[4] = {&c->crho, &c->cux, &c->cuy, &c->cuz};
  const float* dm[4] = {c->rho, c->ux, c->uy, c->uz};
  for (int k = 0; k < 4; ++k) {
    HIPCK(c, hipMalloc(cm[k], sizeof(float) * ncell));
    HIPCK(c, launch_cell_gather(*cm[k], dm[k], c->cmap, ncell, 4, c->s_comp));
  }
  HIPCK(c, hipStreamSynchronize(c->s_comp));
  c->compact = true;
  c->ncell_c = ncell;
  c->nchunk_c = nchunk;
  c->guard_c = guard;
  // the whole domain (planes 1 .. nz) over compact cells; no slab ranges (single domain)
  const bool quarter = c->whole.quarter;
  free_range(c->whole);
  free_range(c->edge);
  free_range(c->mid);
  const CompactView cv{&cmap, &row_of, quarter};
  return build_range(c, c->whole, 4 * gstart[n1], 4 * gstart[(int64_t)(L.nz + 1) * n1], tc, nlc, 0, 0, &cv, true);
}

}  // namespace

extern "C" {

const char* lbm_version(void) { return "lbm-mi355x 0.2 (gfx950, D3Q19 BGK, AoSoA wave-chunk stream-collide)"; }

const char* lbm_last_error(const lbm_ctx* ctx) { return ctx ? ctx->err.c_str() : g_create_error.c_str(); }

int lbm_tune(int knob, int value) {
  static const int hi[LBM_TUNE_COUNT] = {2, 4, 1, 1, 2, 86400, 8, 0, 2, 64, 2, 1, 3, 17, 2};
  if (knob < 0 || knob >= LBM_TUNE_COUNT || value < 0 || value > hi[knob] ||
      (knob == LBM_TUNE_CELLS_PER_LANE && (value == 2 || value == 3))) {
    g_create_error = "lbm_tune: unknown knob or value out of range";
    return LBM_ERR_ARG;
  }
  const int prev = g_tune[knob];
  g_tune[knob] = value;
  return prev;
}

int lbm_create(const lbm_desc* desc, lbm_ctx** out) {
  if (!desc || !out) {
    g_create_error = "null argument";
    return LBM_ERR_ARG;
  }
  *out = nullptr;
  const lbm_desc& d = *desc;
  if (d.nx < 3 || d.ny < 3 || d.nz < 1 || !(d.tau > 0.f) || d.case_kind < 0 || d.case_kind > 3 || d.x_align < 0 ||
      d.x_align > 4 || d.n_bc_codes < 0 || d.n_bc_codes > kMaxBcCodes || (d.n_bc_codes > 0 && !d.bc_codes) ||
      d.row_axis < 0 || d.row_axis > 2) {
    g_create_error = "invalid lattice description";
    return LBM_ERR_ARG;
  }
  const bool dev_mask = !d.geo && d.mask;
  if (!d.geo && d.case_kind != LBM_CASE_LDC && !(dev_mask && d.case_kind == LBM_CASE_MASK)) {
    g_create_error = "geo == NULL is only supported for LBM_CASE_LDC, or LBM_CASE_MASK with a mask";
    return LBM_ERR_ARG;
  }
  if (dev_mask && (d.ny < 5 || (!d.halo_planes && d.nz_global > 0 && (d.nz_global != d.nz || d.z_offset != 0)))) {
    g_create_error = "device mask build: needs ny >= 5, and halo_planes = 1 for a slab";
    return LBM_ERR_ARG;
  }
  lbm_ctx* c = new lbm_ctx();
  c->d = d;
  c->d.geo = nullptr;
  c->d.bc_inlet_uy = nullptr;
  c->d.bc_outlet_uy = nullptr;
  c->d.bc_codes = nullptr;
  c->d.mask = nullptr;
  for (int k = 0; k < d.n_bc_codes; ++k) {
    const lbm_bc_code& b = d.bc_codes[k];
    if (b.face < 0 || b.face > 5 || b.kind < 0 || b.kind > 2 || b.code == 1 || b.code == 4 || b.code < -128 ||
        b.code > 127) {
      g_create_error = "invalid boundary code entry " + std::to_string(k);
      delete c;
      return LBM_ERR_ARG;
    }
  }
  if (c->d.nz_global <= 0) c->d.nz_global = d.nz;
  c->tau = d.tau;
  c->omc = 1.0f - 1.0f / d.tau;  // the reference's (1.0f - 1.0f / tau), evaluated in fp32
  c->fast_div = !g_tune[LBM_TUNE_EXACT_DIV] && verify_fast_div(d.tau);  // A/B: force the compiler's division
  c->bb_immediate = (d.case_kind == LBM_CASE_LDC);
  c->xcd_run = g_tune[LBM_TUNE_XCD_RUN];
  Layout& L = c->L;
  L.nx = d.nx; L.ny = d.ny; L.nz = d.nz;
  L.swap = choose_swap(d);  // the caller's desc: c->d no longer holds geo / mask
  L.xshift = choose_xshift(d, L.swap);
  L.pitch = ((L.swap ? d.ny : d.nx) + 3) / 4 * 4;
  L.planes = d.nz + 2;
  L.plane = (int64_t)L.pitch * (L.swap ? d.nx : d.ny);
  L.ncell = (L.plane * L.planes + kChunk - 1) / kChunk * kChunk;
  L.nchunk = L.ncell / kChunk;
  L.guard = (L.plane + L.pitch + 8 + kChunk - 1) / kChunk + 1;
  c->n_box = (int64_t)d.nx * d.ny * d.nz;
  {
    auto pow2 = [](int64_t v) { return v > 0 && (v & (v - 1)) == 0; };
    c->box = !d.geo && d.case_kind == LBM_CASE_LDC && !L.swap && pow2(L.pitch) && pow2(L.plane) &&
             g_tune[LBM_TUNE_BOX] != 1;
  }
  if (L.ncell >= (int64_t(1) << 31) - 2 * kChunk) {
    g_create_error = "slab too large for 32-bit cell ids (split it into more z-slabs)";
    delete c;
    return LBM_ERR_ARG;
  }

  auto bail = [&](int code) {
    g_create_error = c->err;
    lbm_destroy(c);
    return code;
  };
#define CK(expr)                                                  \
  do {                                                            \
    hipError_t e_ = (expr);                                       \
    if (e_ != hipSuccess) {                                       \
      c->err = std::string(#expr) + ": " + hipGetErrorString(e_); \
      return bail(LBM_ERR_HIP);                                   \
    }                                                             \
  } while (0)

  CK(hipSetDevice(d.device));
  const auto t_create = std::chrono::steady_clock::now();
  {
    size_t tot = 0;
    CK(hipMemGetInfo(&c->mem_free0, &tot));
    c->mem_free_min = c->mem_free0;
  }
  CK(hipStreamCreateWithFlags(&c->s_comp, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&c->s_comm, hipStreamNonBlocking));
  for (hipEvent_t* e : {&c->ev_edge, &c->ev_halo, &c->ev_mid, &c->ev_fin, &c->ev_sum[0], &c->ev_sum[1]})
    CK(hipEventCreateWithFlags(e, hipEventDisableTiming));
  CK(hipMalloc(&c->type, L.ncell));
  for (uint32_t** p : {&c->links, &c->nlinks}) {
    CK(hipMalloc(p, sizeof(uint32_t) * L.ncell));
    CK(hipMemsetAsync(*p, 0, sizeof(uint32_t) * L.ncell, c->s_comp));
  }
  for (float** p : {&c->rho, &c->ux, &c->uy, &c->uz}) {
    CK(hipMalloc(p, sizeof(float) * L.ncell));
    CK(hipMemsetAsync(*p, 0, sizeof(float) * L.ncell, c->s_comp));
  }
  CK(hipMalloc(&c->retried, sizeof(unsigned long long)));
  CK(hipMemsetAsync(c->retried, 0, sizeof(unsigned long long), c->s_comp));
  CK(hipMalloc(&c->conv, sizeof(ConvState)));
  CK(hipMemsetAsync(c->conv, 0, sizeof(ConvState), c->s_comp));
  CK(hipMalloc(&c->scratch, sizeof(double) * 2 * kReduceBlocks));
  {
    int h[29];
    for (int k = 0; k < 5; ++k) {
      h[k] = kUpSet[k];
      h[5 + k] = kDownSet[k];
    }
    for (int q = 0; q < kQ; ++q) h[10 + q] = q;
    CK(hipMalloc(&c->qsets, sizeof(h)));
    CK(hipMemcpy(c->qsets, h, sizeof(h), hipMemcpyHostToDevice));
  }

  // ---- geometry: reference codes per linear cell -> type bytes ----
  int8_t* dcodes = nullptr;
  CK(hipMalloc(&dcodes, L.ncell));
  c->codes = dcodes;  // kept for lbm_get_geo (1 B per cell)
  CK(hipMemsetAsync(dcodes, 0, L.ncell, c->s_comp));
  float *din = nullptr, *dout = nullptr;
  if (dev_mask) {
    // geo_pre on the device: upload the raw mask (1 B/cell), pick the row shift from the
    // device-built codes, then write the codes of every storage cell
    const int pad = d.halo_planes ? 3 : 0, lo = d.halo_planes ? -1 : 0, hi = d.halo_planes ? d.nz + 1 : d.nz;
    const int64_t mbytes = (int64_t)d.nx * d.ny * (d.nz + 2 * pad);
    uint8_t* dmask = nullptr;
    unsigned long long* dh = nullptr;
    CK(hipMalloc(&dmask, mbytes));
    CK(hipMemcpy(dmask, desc->mask, mbytes, hipMemcpyHostToDevice));
    const int zbase = d.z_offset - pad;
    if (d.x_align == 0) {
      unsigned long long hh[4];
      CK(hipMalloc(&dh, sizeof(hh)));
      CK(hipMemsetAsync(dh, 0, sizeof(hh), c->s_comp));
      CK(launch_mask_hist(dmask, d.nx, d.ny, c->d.nz_global, zbase, d.z_offset + lo, d.z_offset + hi, dh, L.swap,
                          c->s_comp));
      CK(hipMemcpyAsync(hh, dh, sizeof(hh), hipMemcpyDeviceToHost, c->s_comp));
      CK(hipStreamSynchronize(c->s_comp));
      CK(hipFree(dh));
      L.xshift = (int)(std::max_element(hh, hh + 4) - hh);
    }
    CK(launch_mask_codes(dmask, d.nx, d.ny, c->d.nz_global, zbase, dcodes, L.pitch, L.xshift, L.plane, L.ncell,
                         d.z_offset, lo, hi, L.swap, c->s_comp));
    CK(hipStreamSynchronize(c->s_comp));
    CK(hipFree(dmask));
  } else if (desc->geo) {
    std::vector<int8_t> h((size_t)L.ncell, 0);
    const int zlo = d.halo_planes ? -1 : 0, zhi = d.halo_planes ? d.nz + 1 : d.nz;
    for (int z = zlo; z < zhi; ++z)
      for (int y = 0; y < d.ny; ++y) put_row(h, L, y, z, desc->geo + ((int64_t)(z - zlo) * d.ny + y) * d.nx);
    CK(hipMemcpyAsync(dcodes, h.data(), L.ncell, hipMemcpyHostToDevice, c->s_comp));
    CK(hipStreamSynchronize(c->s_comp));
  } else {
    CK(launch_ldc_codes(dcodes, d.nx, d.ny, L.pitch, L.xshift, L.plane, L.ncell, d.z_offset, c->d.nz_global, L.swap,
                        c->s_comp));
  }
  const int64_t ntab = (int64_t)d.nx * c->d.nz_global;
  if (desc->bc_inlet_uy) {
    CK(hipMalloc(&din, sizeof(float) * ntab));
    c->bc_in = din;  // kept for lbm_init_case
    CK(hipMemcpy(din, desc->bc_inlet_uy, sizeof(float) * ntab, hipMemcpyHostToDevice));
  }
  if (desc->bc_outlet_uy) {
    CK(hipMalloc(&dout, sizeof(float) * ntab));
    c->bc_out = dout;
    CK(hipMemcpy(dout, desc->bc_outlet_uy, sizeof(float) * ntab, hipMemcpyHostToDevice));
  }
  GeoArgs g{};
  std::vector<float*> bc_tables;
  if (d.case_kind == LBM_CASE_GENERIC) {
    g.nbc = d.n_bc_codes;
    for (int k = 0; k < d.n_bc_codes; ++k) {
      const lbm_bc_code& b = d.bc_codes[k];
      BcCode& o = g.bcs[k];
      o.code = b.code; o.face = b.face; o.kind = b.kind; o.rho = b.rho;
      o.u[0] = b.u[0]; o.u[1] = b.u[1]; o.u[2] = b.u[2];
      if (b.u_normal_table) {
        const int axis = b.face >> 1;
        const int64_t nt = axis == 0 ? (int64_t)d.ny * c->d.nz_global
                                     : axis == 1 ? (int64_t)d.nx * c->d.nz_global : (int64_t)d.nx * d.ny;
        float* t = nullptr;
        CK(hipMalloc(&t, sizeof(float) * nt));
        bc_tables.push_back(t);
        CK(hipMemcpy(t, b.u_normal_table, sizeof(float) * nt, hipMemcpyHostToDevice));
        o.table = t;
      }
    }
  }
  g.codes = dcodes; g.type = c->type; g.links = c->links; g.nlinks = c->nlinks;
  g.rho = c->rho; g.ux = c->ux; g.uy = c->uy; g.uz = c->uz;
  g.inlet_uy = din; g.outlet_uy = dout;
  g.case_kind = d.case_kind; g.lid_u = d.lid_u;
  g.nx = d.nx; g.ny = d.ny; g.pitch = L.pitch; g.xshift = L.xshift; g.planes = L.planes; g.plane = L.plane; g.ncell = L.ncell;
  g.z_offset = d.z_offset; g.nz_global = c->d.nz_global;
  g.swap = L.swap;
  CK(launch_classify(g, c->s_comp));
  CK(launch_flag_fluid(g, c->s_comp));
  CK(hipStreamSynchronize(c->s_comp));
  for (float* t : bc_tables) CK(hipFree(t));

  // ---- work lists: whole domain, and lo edge / hi edge / interior for slabs ----
  {
    std::vector<uint8_t> t((size_t)L.ncell);
    std::vector<uint32_t> nlk((size_t)L.ncell);
    CK(hipMemcpy(t.data(), c->type, L.ncell, hipMemcpyDeviceToHost));
    CK(hipMemcpy(nlk.data(), c->nlinks, sizeof(uint32_t) * L.ncell, hipMemcpyDeviceToHost));
    int64_t nf = 0;
    for (int z = 0; z < d.nz; ++z)
      for (int y = 0; y < d.ny; ++y)
        for (int x = 0; x < d.nx; ++x) {
          const uint8_t v = t[cell_of(L, x, y, z)];
          if ((v & kClassMask) != kFluid) continue;
          ++nf;
          if (v & kNeeAdj) ++c->n_slow;
          if (v & kWallAdj) ++c->n_wall_adj;
          // a fluid cell on the outer x/y layer would pull across rows
          if (x == 0 || x == d.nx - 1 || y == 0 || y == d.ny - 1) {
            c->err = "fluid cell on the outer x/y layer of the box";
            return bail(LBM_ERR_GEOMETRY);
          }
        }
    c->n_fluid = nf;
    {  // one boundary record for every NEE cell (the cavity's lid): the kernels take it from
       // their arguments instead of loading it
      int64_t ref = -1;
      for (int64_t k = 0; k < L.ncell && ref < 0; ++k)
        if ((t[k] & kClassMask) == kNee) ref = k;
      if (ref >= 0) {
        unsigned* flag = nullptr;
        unsigned differs = 1;
        float rec[4];
        CK(hipMalloc(&flag, sizeof(unsigned)));
        hipError_t e = hipMemsetAsync(flag, 0, sizeof(unsigned), c->s_comp);
        if (e == hipSuccess) e = launch_bc_uniform(c->type, c->rho, c->ux, c->uy, c->uz, L.ncell, ref, flag, c->s_comp);
        if (e == hipSuccess) e = hipStreamSynchronize(c->s_comp);
        if (e == hipSuccess) e = hipMemcpy(&differs, flag, sizeof(unsigned), hipMemcpyDeviceToHost);
        const float* arr[4] = {c->rho, c->ux, c->uy, c->uz};
        for (int k = 0; k < 4 && e == hipSuccess; ++k) e = hipMemcpy(&rec[k], arr[k] + ref, sizeof(float), hipMemcpyDeviceToHost);
        (void)hipFree(flag);
        CK(e);
        c->bc_uniform = differs == 0;
        c->bc_const = make_float4(rec[0], rec[1], rec[2], rec[3]);
      }
    }
    const int64_t P = L.plane, nz = d.nz;
    if (build_range(c, c->whole, P, (nz + 1) * P, t, nlk, 0, 0, nullptr, c->d.nz_global == d.nz) != LBM_OK)
      return bail(LBM_ERR_HIP);
    if (build_range(c, c->edge, P, 2 * P, t, nlk, nz * P, (nz + 1) * P) != LBM_OK) return bail(LBM_ERR_HIP);
    if (build_range(c, c->mid, 2 * P, std::max(2 * P, nz * P), t, nlk) != LBM_OK) return bail(LBM_ERR_HIP);
    // compact rows for a single domain whose step takes group lists (vessel trees)
    if (c->d.nz_global == d.nz && !d.halo_planes && g_tune[LBM_TUNE_COMPACT] != 1 && c->whole.groups) {
      const int rc = build_compact(c, t, nlk);
      if (rc != LBM_OK) return bail(rc);
    }
    // partial slots: [whole | lo | hi | mid]; the slab ranges are contiguous
    c->npart_slab = c->edge.npart + c->mid.npart;
    CK(hipMalloc(&c->partial_all, sizeof(double) * std::max(1, c->whole.npart + c->npart_slab)));
    c->whole.part = c->partial_all;
    c->fuse_red = c->whole.npart > 0 && g_tune[LBM_TUNE_FUSED_RESIDUAL] != 0;  // A/B: separate reduction launch
    if (c->fuse_red) {
      c->red_n = c->whole.npart + 8;
      CK(hipMalloc(&c->red_part, sizeof(double) * 2 * c->red_n));
    }
    if (c->whole.nee_records) CK(hipMalloc(&c->nee_val, sizeof(float) * 2 * 8 * (size_t)c->whole.n_rec));
    if (c->whole.nee_fix) CK(hipMalloc(&c->nee_mac, sizeof(float4) * std::max(1, c->whole.n_nee)));  // one per NEE-adjacent cell
    c->edge.part = c->whole.part + c->whole.npart;
    c->mid.part = c->edge.part + c->edge.npart;
  }
  if (c->compact) {
    // compact population buffers (small: the stored cells of a sparse lattice), zeroed
    const size_t bytes = sizeof(float) * (size_t)(c->nchunk_c + 2 * c->guard_c) * kQ * kChunk;
    for (int b = 0; b < 2; ++b) {
      CK(hipMalloc(&c->alloc[b], bytes));
      CK(hipMemsetAsync(c->alloc[b], 0, bytes, c->s_comp));
      c->buf[b] = c->alloc[b] + c->guard_c * kQ * kChunk;
    }
    CK(hipStreamSynchronize(c->s_comp));
  } else {
    // population buffers (buffer_placement(); LBM_TUNE_BUFFER_ALLOC 1: first two allocations),
    // allocated last: the other arrays are in place, so hipMemGetInfo counts them
    const size_t bytes = sizeof(float) * L.buf_floats();
    CK(buffer_placement(c, bytes, (size_t)1 << 30));
    for (int b = 0; b < 2; ++b) c->buf[b] = c->alloc[b] + L.guard * kQ * kChunk;
  }
  {
    size_t fr = 0, tot = 0;
    CK(hipStreamSynchronize(c->s_comp));
    CK(hipMemGetInfo(&fr, &tot));
    c->mem_free_min = std::min(c->mem_free_min, fr);
    c->mem_resident = (int64_t)c->mem_free0 - (int64_t)fr;
    c->mem_peak = (int64_t)c->mem_free0 - (int64_t)c->mem_free_min;
    c->create_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_create).count();
  }
#undef CK
  *out = c;
  return LBM_OK;
}

void lbm_destroy(lbm_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->d.device);
  if (c->s_comp) (void)hipStreamSynchronize(c->s_comp);
  if (c->s_comm) (void)hipStreamSynchronize(c->s_comm);
  if (c->comm) (void)ncclCommDestroy(c->comm);
  if (c->nee_mac) (void)hipFree(c->nee_mac);
  if (c->nee_val) (void)hipFree(c->nee_val);
  for (float* p : {c->alloc[0], c->alloc[1], c->rho, c->ux, c->uy, c->uz, c->hist, c->send_up, c->send_dn,
                   c->recv_up, c->recv_dn})
    if (p) (void)hipFree(p);
  for (Range* r : {&c->whole, &c->edge, &c->mid}) free_range(*r);
  if (c->type) (void)hipFree(c->type);
  if (c->links) (void)hipFree(c->links);
  if (c->nlinks) (void)hipFree(c->nlinks);
  if (c->codes) (void)hipFree(c->codes);
  if (c->bc_in) (void)hipFree(c->bc_in);
  if (c->bc_out) (void)hipFree(c->bc_out);
  if (c->partial_all) (void)hipFree(c->partial_all);
  if (c->slab_part) (void)hipFree(c->slab_part);
  if (c->red_part) (void)hipFree(c->red_part);
  if (c->scratch) (void)hipFree(c->scratch);
  if (c->conv) (void)hipFree(c->conv);
  if (c->retried) (void)hipFree(c->retried);
  if (c->qsets) (void)hipFree(c->qsets);
  if (c->ref_idx) (void)hipFree(c->ref_idx);
  if (c->terms) (void)hipFree(c->terms);
  if (c->cub_part) (void)hipFree(c->cub_part);
  for (void* p : {(void*)c->cmap, (void*)c->crow, (void*)c->rowrec, (void*)c->grouprec, (void*)c->ctype, (void*)c->clinks, (void*)c->cnlinks,
                  (void*)c->crho, (void*)c->cux, (void*)c->cuy, (void*)c->cuz})
    if (p) (void)hipFree(p);
  for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
  for (hipEvent_t e : {c->ev_edge, c->ev_halo, c->ev_mid, c->ev_fin, c->ev_sum[0], c->ev_sum[1]})
    if (e) (void)hipEventDestroy(e);
  if (c->s_comp) (void)hipStreamDestroy(c->s_comp);
  if (c->s_comm) (void)hipStreamDestroy(c->s_comm);
  delete c;
}

int lbm_init_equilibrium(lbm_ctx* c, int form, const float* rho, const float* ux, const float* uy, const float* uz) {
  if (!c || (form != LBM_INIT_LDC_WI && form != LBM_INIT_EXPANDED)) return LBM_ERR_ARG;
  HIPCK(c, hipSetDevice(c->d.device));
  const Layout& L = c->L;
  const float* host[4] = {rho, ux, uy, uz};
  float* dev[4] = {nullptr, nullptr, nullptr, nullptr};
  std::vector<float> h;
  for (int k = 0; k < 4; ++k) {
    if (!host[k]) continue;
    h.assign((size_t)L.ncell, k == 0 ? 1.0f : 0.0f);
    for (int z = 0; z < L.nz; ++z)
      for (int y = 0; y < L.ny; ++y) put_row(h, L, y, z, host[k] + ((int64_t)z * L.ny + y) * L.nx);
    HIPCK(c, hipMalloc(&dev[k], sizeof(float) * L.ncell));
    HIPCK(c, hipMemcpy(dev[k], h.data(), sizeof(float) * L.ncell, hipMemcpyHostToDevice));
  }
  Stage st;
  float *fa = c->buf[0], *fb = c->buf[1];
  if (c->compact) {  // evaluated on a dense copy, then gathered into both compact buffers
    RCK(stage_dense(c, st, &fa));
    fb = fa;
  }
  HIPCK(c, launch_init_feq(fa, fb, L.ncell, form == LBM_INIT_LDC_WI ? 0 : 1, dev[0], dev[1], dev[2], dev[3],
                           c->s_comp));
  if (c->compact)
    for (int b = 0; b < 2; ++b) RCK(from_dense(c, fa, b));
  HIPCK(c, hipStreamSynchronize(c->s_comp));
  for (float* p : dev)
    if (p) HIPCK(c, hipFree(p));
  return reset_state(c);
}

int lbm_init_ldc(lbm_ctx* c) {
  if (!c) return LBM_ERR_ARG;
  HIPCK(c, hipSetDevice(c->d.device));
  Stage st;
  float *fa = c->buf[0], *fb = c->buf[1];
  if (c->compact) {
    RCK(stage_dense(c, st, &fa));
    fb = fa;
  }
  HIPCK(c, launch_init_ldc(fa, fb, c->L.ncell, c->L.pitch, c->L.xshift, c->L.nx, c->L.ny, c->d.lid_u, c->L.swap,
                           c->s_comp));
  if (c->compact)
    for (int b = 0; b < 2; ++b) RCK(from_dense(c, fa, b));
  HIPCK(c, hipStreamSynchronize(c->s_comp));
  return reset_state(c);
}

int lbm_init_case(lbm_ctx* c) {
  if (!c) return LBM_ERR_ARG;
  if (c->d.case_kind == LBM_CASE_LDC) return lbm_init_ldc(c);
  if (c->d.case_kind != LBM_CASE_MASK) {
    c->err = "lbm_init_case: only LBM_CASE_LDC and LBM_CASE_MASK have a device initialize()";
    return LBM_ERR_ARG;
  }
  HIPCK(c, hipSetDevice(c->d.device));
  const Layout& L = c->L;
  Stage st;
  float *fa = c->buf[0], *fb = c->buf[1];
  if (c->compact) {
    RCK(stage_dense(c, st, &fa));
    fb = fa;
  }
  HIPCK(c, launch_init_mask(fa, fb, c->codes, c->bc_in, c->bc_out, L.nx, L.ny, L.nz, L.pitch, L.xshift, L.plane,
                            L.ncell, c->d.z_offset, L.swap, c->s_comp));
  if (c->compact)
    for (int b = 0; b < 2; ++b) RCK(from_dense(c, fa, b));
  HIPCK(c, hipStreamSynchronize(c->s_comp));
  return reset_state(c);
}

int lbm_set_f(lbm_ctx* c, const float* f) {
  if (!c || !f) return LBM_ERR_ARG;
  HIPCK(c, hipSetDevice(c->d.device));
  const Layout& L = c->L;
  std::vector<float> h((size_t)L.nchunk * kQ * kChunk, 0.f);
  for (int q = 0; q < kQ; ++q)
    for (int z = 0; z < L.nz; ++z)
      for (int y = 0; y < L.ny; ++y) {
        const float* row = f + (((int64_t)q * L.nz + z) * L.ny + y) * L.nx;
        for (int x = 0; x < L.nx; ++x) h[aidx(cell_of(L, x, y, z), q)] = row[x];
      }
  if (c->compact) {
    // gathered into the compact layout on the host through cmap (no dense device copy), as
    // k_pop_gather would: slots of compact cells without a dense cell read 0
    std::vector<float> hc((size_t)c->pop_floats(), 0.f);
    for (size_t i = 0; i < c->cmap_h.size(); ++i)
      if (c->cmap_h[i] >= 0)
        for (int q = 0; q < kQ; ++q) hc[aidx((int64_t)i, q)] = h[aidx(c->cmap_h[i], q)];
    for (int b = 0; b < 2; ++b)
      HIPCK(c, hipMemcpy(c->buf[b], hc.data(), sizeof(float) * hc.size(), hipMemcpyHostToDevice));
  } else {
    for (int b = 0; b < 2; ++b)
      HIPCK(c, hipMemcpy(c->buf[b], h.data(), sizeof(float) * h.size(), hipMemcpyHostToDevice));
  }
  return reset_state(c);
}

int lbm_buffer_placement(lbm_ctx* c, double* gbs, int cap, int* n, int* chosen) {
  if (!c) return LBM_ERR_ARG;
  for (int i = 0; gbs && i < cap && i < (int)c->cand_gbs.size(); ++i) gbs[i] = c->cand_gbs[i];
  if (n) *n = (int)c->cand_gbs.size();
  if (chosen) {
    chosen[0] = c->chosen[0];
    chosen[1] = c->chosen[1];
  }
  return LBM_OK;
}

int lbm_get_numerics(lbm_ctx* c, int* fast_div, int64_t* retried_chunks) {
  if (!c) return LBM_ERR_ARG;
  HIPCK(c, hipSetDevice(c->d.device));
  HIPCK(c, hipStreamSynchronize(c->s_comp));
  unsigned long long n = 0;
  HIPCK(c, hipMemcpy(&n, c->retried, sizeof(n), hipMemcpyDeviceToHost));
  if (fast_div) *fast_div = c->fast_div ? 1 : 0;
  if (retried_chunks) *retried_chunks = (int64_t)n;
  return LBM_OK;
}

int lbm_set_residual_order(lbm_ctx* c, int mode, int items_per_thread, int vec, int grid_cap) {
  if (!c) return LBM_ERR_ARG;
  if (mode == LBM_SUM_FP64) {
    c->sum_mode = mode;
    return LBM_OK;
  }
  if (mode != LBM_SUM_CUB_TREE || items_per_thread < 1 || vec < 1 || items_per_thread % vec || grid_cap < 1 ||
      grid_cap > 65536) {
    c->err = "lbm_set_residual_order: mode LBM_SUM_FP64 or LBM_SUM_CUB_TREE with items_per_thread a multiple of "
             "vec and 1 <= grid_cap <= 65536";
    return LBM_ERR_ARG;
  }
  if (c->comm || c->d.nz_global != c->d.nz) {
    c->err = "lbm_set_residual_order: the reference-order sum is defined for a single-domain lattice only";
    return LBM_ERR_ARG;
  }
  HIPCK(c, hipSetDevice(c->d.device));
  if (!c->ref_idx) {
    // reference storage order: LDC bricks of 8 x 8 x 8 over the brick-padded box (ldc.cu:71),
    // otherwise index_transform's compact z, y, x order of the stored cells (code != 0,
    // Poiseulle.cu:257-271, bifurcation.cu:241-252); the fluid cells' slots get their |u|
    const Layout& L = c->L;
    std::vector<uint8_t> t((size_t)L.ncell);
    std::vector<int8_t> codes((size_t)L.ncell);
    HIPCK(c, hipMemcpy(t.data(), c->type, L.ncell, hipMemcpyDeviceToHost));
    HIPCK(c, hipMemcpy(codes.data(), c->codes, L.ncell, hipMemcpyDeviceToHost));
    std::vector<int> ri((size_t)L.ncell, -1);
    const bool ldc = c->d.case_kind == LBM_CASE_LDC;
    const int64_t bx = (L.nx + 7) / 8, by = (L.ny + 7) / 8, bz = (L.nz + 7) / 8;
    int64_t n = ldc ? bx * by * bz * 512 : 0;
    for (int z = 0; z < L.nz; ++z)
      for (int y = 0; y < L.ny; ++y)
        for (int x = 0; x < L.nx; ++x) {
          const int64_t s = cell_of(L, x, y, z);
          int64_t r;
          if (ldc) {
            r = ((x / 8) + (y / 8) * bx + (z / 8) * bx * by) * 512 + x % 8 + (y % 8) * 8 + (z % 8) * 64;
          } else {
            if (codes[s] == 0) continue;
            r = n++;
          }
          if ((t[s] & kClassMask) == kFluid) ri[s] = (int)r;
        }
    if (n >= ((int64_t)1 << 31)) {
      c->err = "lbm_set_residual_order: lattice too large for 32-bit reference indices";
      return LBM_ERR_ARG;
    }
    c->n_ref = n;
    HIPCK(c, hipMalloc(&c->ref_idx, sizeof(int) * L.ncell));
    HIPCK(c, hipMemcpy(c->ref_idx, ri.data(), sizeof(int) * L.ncell, hipMemcpyHostToDevice));
    HIPCK(c, hipMalloc(&c->terms, sizeof(float) * std::max<int64_t>(1, n)));
    HIPCK(c, hipMemset(c->terms, 0, sizeof(float) * std::max<int64_t>(1, n)));
  }
  if (c->cub_part) HIPCK(c, hipFree(c->cub_part));
  c->cub_part = nullptr;
  HIPCK(c, hipMalloc(&c->cub_part, sizeof(float) * cub_grid(c->n_ref, items_per_thread, grid_cap)));
  c->cub_ipt = items_per_thread;
  c->cub_vec = vec;
  c->cub_grid = grid_cap;
  c->sum_mode = mode;
  return LBM_OK;
}

int lbm_set_convergence(lbm_ctx* c, int enabled, int max_it, int stag_max, float tol) {
  if (!c) return LBM_ERR_ARG;
  HIPCK(c, hipSetDevice(c->d.device));
  ConvState h{};
  HIPCK(c, hipStreamSynchronize(c->s_comp));
  HIPCK(c, hipMemcpy(&h, c->conv, sizeof(ConvState), hipMemcpyDeviceToHost));
  h.enabled = enabled ? 1 : 0;
  h.max_it = max_it;
  h.stag_max = stag_max;
  h.tol = tol;
  if (!enabled) h.stopped = 0;
  HIPCK(c, hipMemcpy(c->conv, &h, sizeof(ConvState), hipMemcpyHostToDevice));
  c->conv_enabled = enabled != 0;
  return LBM_OK;
}

}  // extern "C"

namespace {

// ---- halo exchange (slabs) ----------------------------------------------------------------

int ensure_halo_buffers(lbm_ctx* c) {
  if (c->send_up) return LBM_OK;
  const size_t bytes = sizeof(float) * kQ * (size_t)c->L.plane;
  for (float** p : {&c->send_up, &c->send_dn, &c->recv_up, &c->recv_dn}) HIPCK(c, hipMalloc(p, bytes));
  return LBM_OK;
}

const int* qset(lbm_ctx* c, int which) { return c->qsets + (which == 0 ? 0 : which == 1 ? 5 : 10); }

// pack this slab's outgoing faces of buffer b: the top plane's up-going populations and the
// bottom plane's down-going ones (all 19 when `all`)
int pack_faces(lbm_ctx* c, int b, bool all, bool to_dn, bool to_up, hipStream_t st) {
  const int nq = all ? kQ : 5;
  if (to_up) HIPCK(c, launch_pack(c->buf[b], c->send_up, c->L.nz, c->L.plane, all ? qset(c, 2) : qset(c, 0), nq, st));
  if (to_dn) HIPCK(c, launch_pack(c->buf[b], c->send_dn, 1, c->L.plane, all ? qset(c, 2) : qset(c, 1), nq, st));
  return LBM_OK;
}

// unpack what arrived into the ghost planes of buffer b
int unpack_faces(lbm_ctx* c, int b, bool all, bool from_dn, bool from_up, hipStream_t st) {
  const int nq = all ? kQ : 5;
  // per step: walls keep their producers' bounce-back values, NEE cells are not pulled;
  // the initial all-19 copy fills both (raw pulls at step 0) except LDC's primed walls
  const unsigned skip = (!all || c->bb_immediate ? 1u << kWall : 0u) | (!all ? 1u << kNee : 0u);
  if (from_dn)
    HIPCK(c, launch_unpack(c->buf[b], c->recv_dn, c->type, 0, c->L.plane, all ? qset(c, 2) : qset(c, 0), nq, skip,
                           st));
  if (from_up)
    HIPCK(c, launch_unpack(c->buf[b], c->recv_up, c->type, c->L.nz + 1, c->L.plane, all ? qset(c, 2) : qset(c, 1), nq,
                           skip, st));
  return LBM_OK;
}

// pack, send / receive and unpack the +-z faces of buffer b on s_comm (after the work already
// queued there; after_comp: also after the work queued on s_comp)
int rccl_exchange(lbm_ctx* c, int b, bool all, hipEvent_t* halo_end = nullptr, bool after_comp = false) {
  const size_t cnt = (size_t)(all ? kQ : 5) * c->L.plane;
  const int up = c->rank + 1 < c->nranks ? c->rank + 1 : -1;
  const int dn = c->rank > 0 ? c->rank - 1 : -1;
  if (after_comp) {
    HIPCK(c, hipEventRecord(c->ev_edge, c->s_comp));
    HIPCK(c, hipStreamWaitEvent(c->s_comm, c->ev_edge, 0));
  }
  RCK(timed(c, c->s_comm, kKindHalo, -1, -1, [&] {
    RCK(pack_faces(c, b, all, dn >= 0, up >= 0, c->s_comm));
    NCCK(c, ncclGroupStart());
    if (up >= 0) {
      NCCK(c, ncclSend(c->send_up, cnt, ncclFloat, up, c->comm, c->s_comm));
      NCCK(c, ncclRecv(c->recv_up, cnt, ncclFloat, up, c->comm, c->s_comm));
    }
    if (dn >= 0) {
      NCCK(c, ncclSend(c->send_dn, cnt, ncclFloat, dn, c->comm, c->s_comm));
      NCCK(c, ncclRecv(c->recv_dn, cnt, ncclFloat, dn, c->comm, c->s_comm));
    }
    NCCK(c, ncclGroupEnd());
    RCK(unpack_faces(c, b, all, dn >= 0, up >= 0, c->s_comm));
    return LBM_OK;
  }, halo_end));
  HIPCK(c, hipEventRecord(c->ev_halo, c->s_comm));
  return LBM_OK;
}

int step_single(lbm_ctx* c, int nsteps, bool want_hist) {
  if (c->bb_pull()) c->walls_stale = true;  // the whole-domain steps below store no wall slots
  else RCK(prime_walls(c));
  if (c->whole.nee_records && nsteps > 0) c->nee_stale = true;  // ... nor NEE slots (NEE records)
  if (c->sum_mode == LBM_SUM_CUB_TREE) {
    // the reference's order: per step calc_vel_square's terms into reference storage order, then
    // thrust::reduce's CUB tree in fp32 (ldc.cu:660-668)
    const Layout& L = c->L;
    for (int s = 0; s < nsteps; ++s) {
      const int k = c->steps_done + s;
      RCK(run_range(c, c->whole, c->cur, c->s_comp, nullptr, -1, nullptr, k));
      const float* src = c->buf[c->cur];
      const bool own = c->bb_pull() && !c->bb_raw(k);  // wall links read the own slots
      if (c->compact) {  // over the compact rows, each term into its dense cell's reference slot
        HIPCK(c, launch_vel_terms_compact(src, c->ctype, own ? c->clinks : nullptr, c->cmap, c->crow, c->rowrec,
                                          c->ref_idx, c->terms, c->whole.c_lo, c->whole.c_hi, L.swap, c->s_comp));
        c->cur ^= 1;
        HIPCK(c, launch_cub_tree(c->terms, c->n_ref, c->cub_ipt, c->cub_vec, c->cub_grid, c->cub_part, c->conv,
                                 want_hist ? c->hist + s : nullptr, c->s_comp));
        continue;
      }
      const uint32_t* bbl = own ? c->links : nullptr;
      if (c->whole.nee_records && k >= 1)  // the step's source with its NEE slots (the records of step k - 1)
        HIPCK(c, launch_nee_materialize(c->buf[c->cur], c->whole.nee_rec,
                                        c->nee_val + (int64_t)((k - 1) & 1) * c->whole.n_rec * 8, c->whole.n_rec,
                                        L.pitch, L.plane, L.swap, 1, c->s_comp));
      HIPCK(c, launch_vel_terms(src, c->type, bbl, c->ref_idx, c->terms, L.plane, (L.nz + 1) * L.plane, L.pitch,
                                L.plane, L.swap, c->s_comp));
      c->cur ^= 1;
      HIPCK(c, launch_cub_tree(c->terms, c->n_ref, c->cub_ipt, c->cub_vec, c->cub_grid, c->cub_part, c->conv,
                               want_hist ? c->hist + s : nullptr, c->s_comp));
    }
    return LBM_OK;
  }
  if (c->fuse_red && !c->conv_enabled) {
    // one launch per step: step s's k_step also finishes step s-1's residual; the last
    // step's own reduction follows the loop
    const double* prev = nullptr;
    for (int s = 0; s < nsteps; ++s) {
      double* part = c->red_part + (size_t)(s & 1) * c->red_n;
      const FusedRed fr{part, prev, (want_hist && s > 0) ? c->hist + s - 1 : nullptr};
      RCK(run_range(c, c->whole, c->cur, c->s_comp, &fr, -1, nullptr, c->steps_done + s));
      c->cur ^= 1;
      prev = part;
    }
    HIPCK(c, launch_reduce(prev, c->red_n, c->scratch, c->conv, want_hist ? c->hist + nsteps - 1 : nullptr, 1,
                           c->s_comp));
    return LBM_OK;
  }
  for (int s = 0; s < nsteps; ++s) {
    RCK(run_range(c, c->whole, c->cur, c->s_comp, nullptr, -1, nullptr, c->steps_done + s));
    c->cur ^= 1;
    HIPCK(c, launch_reduce(c->whole.part, c->whole.npart, c->scratch, c->conv, want_hist ? c->hist + s : nullptr,
                           1, c->s_comp));
  }
  return LBM_OK;
}

// The slab step on two streams.  s_comp runs nothing but the interior launches, back to back;
// everything else runs on s_comm, beside them:
//   s_comp: [wait halo(h-1)] interior(h) -> ev_mid
//   s_comm: edge planes(h), pack, send / recv, unpack -> ev_halo; [wait ev_mid] reduction(h) ->
//           ev_sum[h & 1], all-reduce, finisher -> ev_fin
// Every hazard is an event or stream order: interior(h) reads planes 1 and nz and the ghost
// planes of src(h), which edge(h-1) and unpack(h-1) wrote (ev_halo), and overwrites src(h-1),
// which edge(h-1) read (ev_halo); edge(h) reads planes 2 and nz-1 and overwrites planes 1 and
// nz of src(h-1), which interior(h-1) wrote / read -- reduction(h-1), queued before edge(h),
// waited for it.  The block partials alternate by step parity, so interior(h) only waits for
// the reduction of step h-2 (ev_sum).  The edge launch and its halo thus overlap the interior
// launch instead of preceding it (round 2: edge launch, interior launch and the two reduction
// launches in series on s_comp).
int step_rccl(lbm_ctx* c, int nsteps, bool want_hist) {
  RCK(prime_walls(c));  // producer-side bounce-back from here on
  RCK(ensure_halo_buffers(c));
  if (!c->slab_part) HIPCK(c, hipMalloc(&c->slab_part, sizeof(double) * 2 * std::max(1, c->npart_slab)));
  // s_comm starts after whatever s_comp holds (set-up, a checkpoint load, read-outs)
  HIPCK(c, hipEventRecord(c->ev_edge, c->s_comp));
  HIPCK(c, hipStreamWaitEvent(c->s_comm, c->ev_edge, 0));
  if (!c->halo_primed) {  // ghost planes of the initial source buffer: all 19 populations
    RCK(rccl_exchange(c, c->cur, true));
    c->halo_primed = true;
  }
  int h = c->steps_done;
  for (int s = 0; s < nsteps; ++s, ++h) {
    const int p = h & 1;
    double* part = c->slab_part + (size_t)p * c->npart_slab;  // [edge | interior]
    HIPCK(c, hipStreamWaitEvent(c->s_comp, c->ev_halo, 0));   // ghost and edge planes of src(h)
    HIPCK(c, hipStreamWaitEvent(c->s_comp, c->ev_sum[p], 0)); // reduction(h-2) read part
    if (c->conv_enabled) HIPCK(c, hipStreamWaitEvent(c->s_comp, c->ev_fin, 0));
    c->last_mid_end = nullptr;
    RCK(run_range(c, c->mid, c->cur, c->s_comp, nullptr, kKindMid, part + c->edge.npart));
    HIPCK(c, hipEventRecord(c->ev_mid, c->s_comp));
    RCK(run_range(c, c->edge, c->cur, c->s_comm, nullptr, kKindEdge, part));
    hipEvent_t halo_end = nullptr;
    RCK(rccl_exchange(c, c->cur ^ 1, false, &halo_end));
    c->cur ^= 1;
    if (c->prof && halo_end && c->last_mid_end)  // how long the halo outlasts the interior
      c->recs.push_back({c->last_mid_end, halo_end, {kKindExposed, -1, -1}});
    // this rank's sum goes to the step-parity slot of the all-reduce (the all-reduce of step
    // h - 2, which read it, is earlier on s_comm)
    HIPCK(c, hipStreamWaitEvent(c->s_comm, c->ev_mid, 0));
    HIPCK(c, launch_reduce(part, c->npart_slab, c->scratch, c->conv, nullptr, 0, c->s_comm, &c->conv->s_slot[p]));
    HIPCK(c, hipEventRecord(c->ev_sum[p], c->s_comm));
    NCCK(c, ncclAllReduce(&c->conv->s_slot[p], &c->conv->s_global, 1, ncclDouble, ncclSum, c->comm, c->s_comm));
    HIPCK(c, launch_finish_global(c->conv, want_hist ? c->hist + s : nullptr, c->s_comm));
    HIPCK(c, hipEventRecord(c->ev_fin, c->s_comm));
  }
  HIPCK(c, hipStreamWaitEvent(c->s_comp, c->ev_fin, 0));
  HIPCK(c, hipStreamWaitEvent(c->s_comp, c->ev_halo, 0));
  return LBM_OK;
}

// Wait for both streams.  With an RCCL communicator the wait polls instead of blocking: a
// peer that failed (ncclCommGetAsyncError) or a wait longer than LBM_TUNE_SYNC_TIMEOUT_S
// aborts the communicator and returns LBM_ERR_RCCL, so a rank whose neighbour died exits
// promptly instead of hanging in a halo receive.
int comm_failed_error(lbm_ctx* c) {
  c->err = "RCCL communicator was aborted after a peer failure or a timed-out wait; the slab state is stale "
           "(destroy the context)";
  return LBM_ERR_RCCL;
}

int wait_streams(lbm_ctx* c) {
  if (c->comm_failed) return comm_failed_error(c);
  if (!c->comm) {
    HIPCK(c, hipStreamSynchronize(c->s_comp));
    HIPCK(c, hipStreamSynchronize(c->s_comm));
    return LBM_OK;
  }
  const auto t0 = std::chrono::steady_clock::now();
  const int limit_s = g_tune[LBM_TUNE_SYNC_TIMEOUT_S];
  for (;;) {
    ncclResult_t ar = ncclSuccess;
    if (c->inject_fault) {  // test hook (lbm_debug_fail_next_wait): this wait sees a failed peer
      c->inject_fault = false;
      ar = ncclRemoteError;
    } else {
      const hipError_t a = hipStreamQuery(c->s_comp), b = hipStreamQuery(c->s_comm);
      if (a == hipSuccess && b == hipSuccess) return LBM_OK;
      if (a != hipSuccess && a != hipErrorNotReady) HIPCK(c, a);
      if (b != hipSuccess && b != hipErrorNotReady) HIPCK(c, b);
      NCCK(c, ncclCommGetAsyncError(c->comm, &ar));
    }
    const double waited = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if ((ar != ncclSuccess && ar != ncclInProgress) || (limit_s > 0 && waited > limit_s)) {
      c->err = ar != ncclSuccess && ar != ncclInProgress
                   ? std::string("RCCL peer failure: ") + ncclGetErrorString(ar)
                   : "RCCL step did not complete within LBM_TUNE_SYNC_TIMEOUT_S = " + std::to_string(limit_s) + " s";
      (void)ncclCommAbort(c->comm);
      c->comm = nullptr;
      c->comm_failed = true;
      return LBM_ERR_RCCL;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(waited < 0.01 ? 20 : 200));
  }
}

// lazy macros: the (rho, u) the last step computed, from its source buffer (k_moments);
// steps_done is device-confirmed here
int refresh_macros(lbm_ctx* c) {
  HIPCK(c, hipSetDevice(c->d.device));
  RCK(wait_streams(c));
  if (!c->macros_stale) return LBM_OK;
  ConvState h{};
  HIPCK(c, hipMemcpy(&h, c->conv, sizeof(ConvState), hipMemcpyDeviceToHost));
  c->steps_done = h.k;
  c->macros_stale = false;
  if (h.k == 0) return LBM_OK;  // no step ran: the initial arrays
  const Layout& L = c->L;
  const float* src = c->buf[c->cur ^ 1];  // the last step's source buffer
  if (!c->bb_pull()) RCK(prime_walls(c));  // a producer-side read-out pulls the wall slots
  RCK(materialize_nee(c));                  // ... and every read-out the NEE slots
  // the last step ran from this buffer: step h.k - 1
  const bool consumer = c->bb_pull() && !c->bb_raw(h.k - 1);
  if (c->compact)  // straight from the compact buffer, addressed as the step kernels address it
    HIPCK(c, launch_moments_compact(src, c->ctype, consumer ? c->clinks : nullptr, c->cmap, c->crow, c->rowrec, c->rho,
                                    c->ux, c->uy, c->uz, c->whole.c_lo, c->whole.c_hi, L.swap, c->s_comp));
  else
    HIPCK(c, launch_moments(src, c->type, consumer ? c->links : nullptr, c->rho, c->ux, c->uy, c->uz, L.plane,
                            (L.nz + 1) * L.plane, L.pitch, L.plane, L.swap, c->s_comp));
  HIPCK(c, hipStreamSynchronize(c->s_comp));
  return LBM_OK;
}

}  // namespace

extern "C" {

int lbm_step(lbm_ctx* c, int nsteps, float* residual_hist, int* steps_done) {
  if (!c || nsteps < 0) return LBM_ERR_ARG;
  if (c->comm_failed) return comm_failed_error(c);
  if (nsteps == 0) {
    if (steps_done) *steps_done = c->steps_done;
    return LBM_OK;
  }
  HIPCK(c, hipSetDevice(c->d.device));
  // a roctx range per call (rocprofv3 --marker-trace): the host side of the step loop
  struct Range_ {
    Range_() { roctxRangePush("lbm_step"); }
    ~Range_() { roctxRangePop(); }
  } roctx_range;
  const bool want_hist = residual_hist != nullptr;
  const int k0 = c->steps_done, cur0 = c->cur;
  if (want_hist) {
    RCK(ensure_hist(c, nsteps));
    HIPCK(c, hipMemsetAsync(c->hist, 0xFF, sizeof(float) * nsteps, c->s_comp));  // NaN: step not run
  }
  hipEvent_t sp0 = nullptr, sp1 = nullptr;
  if (c->span) {  // everything this call enqueues, between two events on the compute stream
    RCK(take_event(c, &sp0));
    RCK(take_event(c, &sp1));
    HIPCK(c, hipEventRecord(sp0, c->s_comp));
  }
  RCK(c->comm ? step_rccl(c, nsteps, want_hist) : step_single(c, nsteps, want_hist));
  if (c->span) {  // (step_rccl ends with the compute stream waiting for the communication stream)
    HIPCK(c, hipEventRecord(sp1, c->s_comp));
    c->recs.push_back({sp0, sp1, {kKindSpan, -1, -1}});
    c->kind_n[kKindSpan] += nsteps;
  }
  c->macros_stale = true;
  const bool sync = want_hist || steps_done || c->conv_enabled;
  if (sync) {
    RCK(wait_streams(c));
    ConvState h{};
    HIPCK(c, hipMemcpy(&h, c->conv, sizeof(ConvState), hipMemcpyDeviceToHost));
    c->steps_done = h.k;  // device-confirmed (a converged run stops early)
    if (c->conv_enabled) c->cur = cur0 ^ ((h.k - k0) & 1);  // one step per launch under convergence control
    if (want_hist) HIPCK(c, hipMemcpy(residual_hist, c->hist, sizeof(float) * nsteps, hipMemcpyDeviceToHost));
    if (steps_done) *steps_done = c->steps_done;
  } else {
    c->steps_done += nsteps;
  }
  return LBM_OK;
}

int lbm_sync(lbm_ctx* c) {
  if (!c) return LBM_ERR_ARG;
  HIPCK(c, hipSetDevice(c->d.device));
  return wait_streams(c);
}

int lbm_get_state(lbm_ctx* c, int* k, int* tol_count, int* stopped, float* residual, double* velsum) {
  if (!c) return LBM_ERR_ARG;
  RCK(lbm_sync(c));
  ConvState h{};
  HIPCK(c, hipMemcpy(&h, c->conv, sizeof(ConvState), hipMemcpyDeviceToHost));
  if (k) *k = h.k;
  if (tol_count) *tol_count = h.tol_count;
  if (stopped) *stopped = h.stopped;  // 2: stopped on a non-finite |u| sum
  if (residual) *residual = h.residual;
  if (velsum) *velsum = c->comm ? h.s_global : h.s_local;
  return LBM_OK;
}

int lbm_get_nonfinite(lbm_ctx* c, int* k) {
  if (!c || !k) return LBM_ERR_ARG;
  RCK(lbm_sync(c));
  ConvState h{};
  HIPCK(c, hipMemcpy(&h, c->conv, sizeof(ConvState), hipMemcpyDeviceToHost));
  *k = h.nonfinite_k;
  return LBM_OK;
}

int lbm_get_macros(lbm_ctx* c, float* rho, float* ux, float* uy, float* uz) {
  if (!c) return LBM_ERR_ARG;
  RCK(refresh_macros(c));
  const Layout& L = c->L;
  std::vector<uint8_t> t((size_t)L.ncell);
  HIPCK(c, hipMemcpy(t.data(), c->type, L.ncell, hipMemcpyDeviceToHost));
  std::vector<float> h((size_t)L.ncell);
  float* outs[4] = {rho, ux, uy, uz};
  float* devs[4] = {c->rho, c->ux, c->uy, c->uz};
  for (int k = 0; k < 4; ++k) {
    if (!outs[k]) continue;
    HIPCK(c, hipMemcpy(h.data(), devs[k], sizeof(float) * L.ncell, hipMemcpyDeviceToHost));
    for (int z = 0; z < L.nz; ++z)
      for (int y = 0; y < L.ny; ++y)
        for (int x = 0; x < L.nx; ++x) {
          const int64_t s = cell_of(L, x, y, z);
          outs[k][((int64_t)z * L.ny + y) * L.nx + x] = ((t[s] & kClassMask) == kFluid) ? h[s] : 0.0f;
        }
  }
  return LBM_OK;
}

int lbm_field_digest(lbm_ctx* c, uint64_t* plane_digest) {
  if (!c || !plane_digest) return LBM_ERR_ARG;
  RCK(refresh_macros(c));
  const Layout& L = c->L;
  unsigned long long* d = nullptr;
  HIPCK(c, hipMalloc(&d, sizeof(unsigned long long) * L.nz));
  struct DevFree {
    void* p;
    ~DevFree() { (void)hipFree(p); }
  } guard{d};
  HIPCK(c, hipMemsetAsync(d, 0, sizeof(unsigned long long) * L.nz, c->s_comp));
  HIPCK(c, launch_digest(c->type, c->rho, c->ux, c->uy, c->uz, L.nx, L.ny, L.nz, L.pitch, L.xshift, L.plane,
                         c->d.z_offset, L.swap, d, c->s_comp));
  HIPCK(c, hipStreamSynchronize(c->s_comp));
  HIPCK(c, hipMemcpy(plane_digest, d, sizeof(uint64_t) * L.nz, hipMemcpyDeviceToHost));
  return LBM_OK;
}

int lbm_get_geo(lbm_ctx* c, int8_t* geo) {
  if (!c || !geo) return LBM_ERR_ARG;
  RCK(lbm_sync(c));
  const Layout& L = c->L;
  std::vector<int8_t> h((size_t)L.ncell);
  HIPCK(c, hipMemcpy(h.data(), c->codes, L.ncell, hipMemcpyDeviceToHost));
  for (int z = 0; z < L.nz; ++z)
    for (int y = 0; y < L.ny; ++y)
      for (int x = 0; x < L.nx; ++x) geo[((int64_t)z * L.ny + y) * L.nx + x] = h[cell_of(L, x, y, z)];
  return LBM_OK;
}

int lbm_get_f(lbm_ctx* c, float* f) {
  if (!c || !f) return LBM_ERR_ARG;
  RCK(lbm_sync(c));
  RCK(materialize_nee(c));  // the NEE cells' slots as the producer side holds them
  const Layout& L = c->L;
  if (c->compact) {
    // the compact buffer as it is, placed on the host through cmap (no dense device copy); cells
    // outside the row spans hold no slots and read 0
    std::vector<float> h((size_t)c->pop_floats());
    HIPCK(c, hipMemcpy(h.data(), c->buf[c->cur], sizeof(float) * h.size(), hipMemcpyDeviceToHost));
    std::vector<int> comp((size_t)L.ncell, -1);
    for (size_t i = 0; i < c->cmap_h.size(); ++i)
      if (c->cmap_h[i] >= 0) comp[c->cmap_h[i]] = (int)i;
    for (int q = 0; q < kQ; ++q)
      for (int z = 0; z < L.nz; ++z)
        for (int y = 0; y < L.ny; ++y) {
          float* row = f + (((int64_t)q * L.nz + z) * L.ny + y) * L.nx;
          for (int x = 0; x < L.nx; ++x) {
            const int i = comp[cell_of(L, x, y, z)];
            row[x] = i >= 0 ? h[aidx(i, q)] : 0.0f;
          }
        }
    return LBM_OK;
  }
  std::vector<float> h((size_t)L.nchunk * kQ * kChunk);
  HIPCK(c, hipMemcpy(h.data(), c->buf[c->cur], sizeof(float) * h.size(), hipMemcpyDeviceToHost));
  for (int q = 0; q < kQ; ++q)
    for (int z = 0; z < L.nz; ++z)
      for (int y = 0; y < L.ny; ++y) {
        float* row = f + (((int64_t)q * L.nz + z) * L.ny + y) * L.nx;
        for (int x = 0; x < L.nx; ++x) row[x] = h[aidx(cell_of(L, x, y, z), q)];
      }
  return LBM_OK;
}

// ---- checkpoint / resume -------------------------------------------------------------------

namespace {

// version 2: the complete state is the two population buffers (NEE values included, stored
// producer-side into the boundary cells' slots) plus the run state below
struct CkptHeader {
  char magic[8];  // "LBMCKPT1"
  int32_t version, nx, ny, nz, z_offset, nz_global, case_kind, swap, pitch, xshift, steps_done, cur;
  int32_t halo_primed;  // the ghost planes hold the exchange state (all 19 populations only at step 0)
  int32_t walls_stale;  // saved by a context bouncing back on the consumer side: the wall slots of both
                        // buffers were not written (lbm_ctx::walls_stale; version 3)
  uint32_t tau_bits;
  int64_t ncell, buf_floats;
  ConvState conv;
};
constexpr int32_t kCkptVersion = 3;
// version 2 (round 4): no walls_stale -- every context then stored its wall slots producer-side
struct CkptHeaderV2 {
  char magic[8];
  int32_t version, nx, ny, nz, z_offset, nz_global, case_kind, swap, pitch, xshift, steps_done, cur;
  int32_t halo_primed;
  uint32_t tau_bits;
  int64_t ncell, buf_floats;
  ConvState conv;
};
// the header of a version-2 or version-3 file as version 3 (false: short read, or another magic);
// *version receives the file's version
bool read_ckpt_header(std::FILE* f, CkptHeader& h, int32_t* version) {
  char head[12];
  *version = -1;
  if (std::fread(head, sizeof(head), 1, f) != 1 || std::memcmp(head, "LBMCKPT1", 8) != 0) return false;
  std::memcpy(version, head + 8, 4);
  if (std::fseek(f, 0, SEEK_SET) != 0) return false;
  if (*version == 2) {
    CkptHeaderV2 o{};
    if (std::fread(&o, sizeof(o), 1, f) != 1) return false;
    std::memcpy(h.magic, o.magic, 8);
    h.version = o.version; h.nx = o.nx; h.ny = o.ny; h.nz = o.nz; h.z_offset = o.z_offset;
    h.nz_global = o.nz_global; h.case_kind = o.case_kind; h.swap = o.swap; h.pitch = o.pitch;
    h.xshift = o.xshift; h.steps_done = o.steps_done; h.cur = o.cur; h.halo_primed = o.halo_primed;
    h.walls_stale = 0;  // written by producer-side steps
    h.tau_bits = o.tau_bits; h.ncell = o.ncell; h.buf_floats = o.buf_floats; h.conv = o.conv;
    return true;
  }
  return *version == kCkptVersion && std::fread(&h, sizeof(h), 1, f) == 1;
}

constexpr size_t kCkptSlice = (size_t)64 << 20;  // bytes staged through the host per copy

}  // namespace

int lbm_checkpoint_save(lbm_ctx* c, const char* path) {
  if (!c || !path) return LBM_ERR_ARG;
  RCK(lbm_sync(c));
  RCK(materialize_nee(c));  // files hold the NEE values in the NEE cells' slots, whatever the mode
  CkptHeader h{};
  std::memcpy(h.magic, "LBMCKPT1", 8);
  h.version = kCkptVersion;
  h.nx = c->L.nx; h.ny = c->L.ny; h.nz = c->L.nz;
  h.z_offset = c->d.z_offset; h.nz_global = c->d.nz_global; h.case_kind = c->d.case_kind;
  h.swap = c->L.swap; h.pitch = c->L.pitch; h.xshift = c->L.xshift;
  h.steps_done = c->steps_done; h.cur = c->cur;
  h.halo_primed = c->halo_primed ? 1 : 0;
  h.walls_stale = c->walls_stale ? 1 : 0;
  std::memcpy(&h.tau_bits, &c->tau, 4);
  h.ncell = c->compact ? c->ncell_c : c->L.ncell;
  h.buf_floats = c->pop_floats();
  HIPCK(c, hipMemcpy(&h.conv, c->conv, sizeof(ConvState), hipMemcpyDeviceToHost));
  std::FILE* f = std::fopen(path, "wb");
  if (!f) {
    c->err = std::string("lbm_checkpoint_save: cannot open ") + path;
    return LBM_ERR_ARG;
  }
  bool ok = std::fwrite(&h, sizeof(h), 1, f) == 1;
  std::vector<char> stage(kCkptSlice);
  auto dump = [&](const void* dev, size_t bytes) -> int {
    for (size_t off = 0; ok && off < bytes; off += kCkptSlice) {
      const size_t n = std::min(kCkptSlice, bytes - off);
      HIPCK(c, hipMemcpy(stage.data(), static_cast<const char*>(dev) + off, n, hipMemcpyDeviceToHost));
      ok = std::fwrite(stage.data(), 1, n, f) == n;
    }
    return LBM_OK;
  };
  int rc = LBM_OK;
  // the current state and the buffer the last step read (the lazy macro read-out needs it)
  for (int b : {c->cur, c->cur ^ 1})
    if (rc == LBM_OK) rc = dump(c->buf[b], sizeof(float) * (size_t)h.buf_floats);
  if (std::fclose(f) != 0) ok = false;
  if (rc != LBM_OK) return rc;
  if (!ok) {
    c->err = std::string("lbm_checkpoint_save: write failed: ") + path;
    return LBM_ERR_ARG;
  }
  return LBM_OK;
}

int lbm_checkpoint_load(lbm_ctx* c, const char* path) {
  if (!c || !path) return LBM_ERR_ARG;
  RCK(lbm_sync(c));
  std::FILE* f = std::fopen(path, "rb");
  if (!f) {
    c->err = std::string("lbm_checkpoint_load: cannot open ") + path;
    return LBM_ERR_ARG;
  }
  CkptHeader h{};
  uint32_t tau_bits;
  std::memcpy(&tau_bits, &c->tau, 4);
  int32_t version = -1;
  const bool header = read_ckpt_header(f, h, &version);
  if (!header && version >= 0 && version != 2 && version != kCkptVersion) {
    std::fclose(f);
    c->err = std::string("lbm_checkpoint_load: ") + path + ": unsupported checkpoint version " +
             std::to_string(version) + " (this library reads versions 2 and " + std::to_string(kCkptVersion) + ")";
    return LBM_ERR_ARG;
  }
  bool match = header && h.nx == c->L.nx && h.ny == c->L.ny && h.nz == c->L.nz && h.z_offset == c->d.z_offset &&
               h.nz_global == c->d.nz_global && h.case_kind == c->d.case_kind && h.swap == c->L.swap &&
               h.pitch == c->L.pitch && h.xshift == c->L.xshift && h.tau_bits == tau_bits &&
               h.ncell == (c->compact ? c->ncell_c : c->L.ncell) && h.buf_floats == c->pop_floats();
  // run state of a well-formed file: one of the two buffers current, flags 0/1, the device
  // step counter equal to the host's
  const bool sane = (h.cur == 0 || h.cur == 1) && h.steps_done >= 0 && (h.halo_primed == 0 || h.halo_primed == 1) &&
                    (h.walls_stale == 0 || h.walls_stale == 1) && h.conv.k == h.steps_done &&
                    h.conv.tol_count >= 0 && h.conv.stopped >= 0 && h.conv.stopped <= 2;
  if (match && !sane) {
    std::fclose(f);
    c->err = std::string("lbm_checkpoint_load: ") + path + ": corrupt header (buffer index, step or flags)";
    return LBM_ERR_ARG;
  }
  if (!match) {
    std::fclose(f);
    c->err = std::string("lbm_checkpoint_load: ") + path +
             " is not a checkpoint of a lattice with this descriptor (extent, slab, case, tau, layout)";
    return LBM_ERR_ARG;
  }
  std::vector<char> stage(kCkptSlice);
  bool ok = true;
  auto fill = [&](void* dev, size_t bytes) -> int {
    for (size_t off = 0; ok && off < bytes; off += kCkptSlice) {
      const size_t n = std::min(kCkptSlice, bytes - off);
      ok = std::fread(stage.data(), 1, n, f) == n;
      if (ok) HIPCK(c, hipMemcpy(static_cast<char*>(dev) + off, stage.data(), n, hipMemcpyHostToDevice));
    }
    return LBM_OK;
  };
  int rc = LBM_OK;
  for (int b : {h.cur, h.cur ^ 1})
    if (rc == LBM_OK) rc = fill(c->buf[b], sizeof(float) * (size_t)h.buf_floats);
  std::fclose(f);
  if (rc != LBM_OK) return rc;
  if (!ok) {
    c->err = std::string("lbm_checkpoint_load: truncated file ") + path;
    return LBM_ERR_ARG;
  }
  {
    // the run state comes from the file; the convergence settings (enabled, max_it, stag_max,
    // tol) stay this context's own, which the step kernels' stop flag follows (conv_enabled)
    ConvState now{};
    HIPCK(c, hipMemcpy(&now, c->conv, sizeof(ConvState), hipMemcpyDeviceToHost));
    ConvState run = h.conv;
    run.enabled = now.enabled;
    run.max_it = now.max_it;
    run.stag_max = now.stag_max;
    run.tol = now.tol;
    if (!run.enabled) run.stopped = 0;  // as lbm_set_convergence(0, ...) leaves it
    HIPCK(c, hipMemcpy(c->conv, &run, sizeof(ConvState), hipMemcpyHostToDevice));
  }
  c->cur = h.cur;
  c->steps_done = h.steps_done;
  c->macros_stale = h.steps_done > 0;
  // the saved ghost planes are the exchange's own state: after the first step only the 5
  // crossing populations are exchanged, and a ghost wall's other slots hold this slab's
  // bounce-back values, which a fresh 19-population exchange would overwrite
  c->halo_primed = h.halo_primed != 0;
  // a file from a consumer-side context has stale wall slots; a producer-side context restores
  // them now (its next step pulls them), a consumer-side one never reads them
  c->walls_stale = h.walls_stale != 0;
  if (!c->bb_pull()) RCK(prime_walls(c));
  // NEE records: the next step takes the values of step k - 1 from its source buffer's NEE slots
  c->nee_stale = false;
  if (c->whole.nee_records && c->steps_done >= 1) {
    HIPCK(c, launch_nee_materialize(c->buf[c->cur], c->whole.nee_rec,
                                    c->nee_val + (int64_t)((c->steps_done - 1) & 1) * c->whole.n_rec * 8,
                                    c->whole.n_rec, c->L.pitch, c->L.plane, c->L.swap, 0, c->s_comp));
    HIPCK(c, hipStreamSynchronize(c->s_comp));
  }
  return LBM_OK;
}

int lbm_get_counts(lbm_ctx* c, int64_t* n_box, int64_t* n_fluid, double* algo_bytes_per_step) {
  if (!c) return LBM_ERR_ARG;
  if (n_box) *n_box = c->n_box;
  if (n_fluid) *n_fluid = c->n_fluid;
  if (algo_bytes_per_step) *algo_bytes_per_step = 152.0 * (double)c->n_fluid;
  return LBM_OK;
}

int lbm_get_layout(lbm_ctx* c, int* row_axis, int* pitch, int* x_align, int64_t* active_chunks) {
  if (!c) return LBM_ERR_ARG;
  if (row_axis) *row_axis = c->L.swap ? 2 : 1;
  if (pitch) *pitch = c->L.pitch;
  if (x_align) *x_align = c->L.xshift + 1;
  if (active_chunks) *active_chunks = c->whole.nchunks;
  return LBM_OK;
}

int lbm_get_launch_shape(lbm_ctx* c, int* cells_per_lane, int* main_blocks, int* grid_stride, double* lane_fill) {
  if (!c) return LBM_ERR_ARG;
  if (cells_per_lane) *cells_per_lane = c->whole.quarter ? 1 : 4;
  if (main_blocks) *main_blocks = c->whole.main_blocks;
  const bool listless = c->compact && c->whole.quarter;
  if (grid_stride) *grid_stride = listless ? 3 : c->whole.groups ? 2 : c->whole.stride ? 1 : 0;
  if (lane_fill) *lane_fill = (c->whole.groups || listless) ? c->whole.group_fill : c->whole.lane_fill;
  return LBM_OK;
}

int lbm_get_storage(lbm_ctx* c, int* compact, int64_t* cells, int64_t* bytes) {
  if (!c) return LBM_ERR_ARG;
  if (compact) *compact = c->compact ? 1 : 0;
  if (cells) *cells = c->compact ? c->ncell_c : c->L.ncell;
  if (bytes) *bytes = 2 * (int64_t)sizeof(float) * c->pop_floats();
  return LBM_OK;
}

int lbm_get_nee_path(lbm_ctx* c, int* path, int* max_records) {
  if (!c) return LBM_ERR_ARG;
  const Range& r = c->whole;
  if (path) *path = r.nee_records ? 3 : r.nee_fix ? 2 : r.nee_blocks > 0 ? 1 : 0;
  if (max_records) *max_records = r.nee_records ? r.nee_rec_max : 0;
  return LBM_OK;
}

int lbm_get_setup_cost(lbm_ctx* c, double* create_s, int64_t* device_bytes, int64_t* peak_bytes) {
  if (!c) return LBM_ERR_ARG;
  if (create_s) *create_s = c->create_s;
  if (device_bytes) *device_bytes = c->mem_resident;
  if (peak_bytes) *peak_bytes = c->mem_peak;
  return LBM_OK;
}

int lbm_get_boundary_cells(lbm_ctx* c, int64_t* n_boundary) {
  if (!c || !n_boundary) return LBM_ERR_ARG;
  *n_boundary = c->n_slow;
  return LBM_OK;
}

int lbm_profile(lbm_ctx* c, int enabled) {
  if (!c) return LBM_ERR_ARG;
  if (enabled < 0 || enabled > 2) return LBM_ERR_ARG;
  RCK(harvest_profile(c));
  c->prof = enabled == 1;
  c->span = enabled == 2;
  c->kernel_ms = 0.0;
  c->launches = 0;
  for (int k = 0; k < kKinds; ++k) {
    c->kind_ms[k] = 0.0;
    c->kind_n[k] = 0;
  }
  return LBM_OK;
}

int lbm_kernel_times(lbm_ctx* c, int kind, double* ms, int64_t* launches) {
  if (!c || kind < 0 || kind >= kKinds) return LBM_ERR_ARG;
  RCK(harvest_profile(c));
  if (ms) *ms = c->kind_ms[kind];
  if (launches) *launches = c->kind_n[kind];
  return LBM_OK;
}

int lbm_stats(lbm_ctx* c, double* kernel_ms, int64_t* launches, double* algo_bytes) {
  if (!c) return LBM_ERR_ARG;
  RCK(harvest_profile(c));
  if (kernel_ms) *kernel_ms = c->kernel_ms;
  if (launches) *launches = c->launches;
  if (algo_bytes) *algo_bytes = 152.0 * (double)c->n_fluid;
  return LBM_OK;
}

int lbm_probe_stream(int device, int64_t bytes, int reps, double* gbs) {
  if (!gbs) {
    g_create_error = "lbm_probe_stream: gbs non-null";
    return LBM_ERR_ARG;
  }
  double per[16] = {};
  int n = 0;
  const int rc = lbm_probe_stream_shapes(device, bytes, reps, per, 16, &n);
  *gbs = 0.0;
  for (int i = 0; i < n && i < 16; ++i) *gbs = std::max(*gbs, per[i]);
  return rc;
}

int lbm_probe_stream_shapes(int device, int64_t bytes, int reps, double* gbs_shape, int cap, int* nshapes) {
  if (bytes < (1 << 16) || reps < 1 || !gbs_shape || cap < 0) {
    g_create_error = "lbm_probe_stream: bytes >= 64 KiB, reps >= 1, gbs non-null";
    return LBM_ERR_ARG;
  }
  const int64_t n4 = (bytes >> 16) << 12;  // whole 64-KiB blocks of 16-B vectors
  void *a = nullptr, *b = nullptr;
  hipStream_t st = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreate(&e0);
  if (e == hipSuccess) e = hipEventCreate(&e1);
  // the same placement rule as the population buffers (buffer_placement, rank_pair): up to
  // 64 candidates within the same budget (twenty 8-GiB ones), ranked by a write sweep each, and
  // of the four fastest the pair whose tile copies both ways take the least time together
  {
    std::vector<void*> cand;
    std::vector<double> rate;
    size_t fr = 0, tot = 0;
    if (e == hipSuccess) e = hipMemGetInfo(&fr, &tot);
    const size_t sz = (size_t)n4 * 16;
    const size_t budget = std::min(kPlacementBudget, fr / 4 * 3);
    const int ncand = (int)std::max<size_t>(
        2, std::min<size_t>(std::min<size_t>(64, budget / sz), fr > sz ? (fr - sz) / sz : 0));
    for (int i = 0; i < ncand && e == hipSuccess; ++i) {
      void* q = nullptr;
      e = hipMalloc(&q, sz);
      if (e != hipSuccess) break;
      cand.push_back(q);
      e = hipMemsetAsync(q, 0x3c, sz, st);
    }
    if (e == hipErrorOutOfMemory && cand.size() >= 2) {
      (void)hipGetLastError();
      e = hipSuccess;
    }
    int ka = 0, kb = 1;
    if (e == hipSuccess) e = rank_pair(cand, sz, st, true, rate, ka, kb);
    for (int k = 0; k < (int)cand.size(); ++k) {
      if (e == hipSuccess && k == ka) a = cand[k];
      else if (e == hipSuccess && k == kb) b = cand[k];
      else (void)hipFree(cand[k]);
    }
    if (e == hipSuccess && (!a || !b)) e = hipErrorOutOfMemory;
  }
  const int shapes[][2] = {{8192, 0}, {8192, 1}, {8192, 2}, {8192, 3}, {4096, 4}, {2048, 5}, {32768, 2},
                           {0, 6},    {0, 7},    {0, 8},    {0, 9}};
  const int nsh = (int)(sizeof(shapes) / sizeof(shapes[0]));
  if (nshapes) *nshapes = nsh;
  for (int i = 0; i < cap; ++i) gbs_shape[i] = 0.0;
  for (int si = 0; si < nsh; ++si) {  // blocks, launch_probe_copy shape
    const auto& sh = shapes[si];
    if (e != hipSuccess) break;
    e = launch_probe_copy(a, b, n4, sh[0], sh[1], st);  // untimed first launch
    for (int r = 0; r < reps && e == hipSuccess; ++r) {
      e = hipEventRecord(e0, st);
      if (e == hipSuccess) e = launch_probe_copy(r & 1 ? b : a, r & 1 ? a : b, n4, sh[0], sh[1], st);
      if (e == hipSuccess) e = hipEventRecord(e1, st);
      if (e == hipSuccess) e = hipEventSynchronize(e1);
      float ms = 0.f;
      if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
      if (e == hipSuccess && ms > 0.f && si < cap)
        gbs_shape[si] = std::max(gbs_shape[si], 2.0 * 16.0 * (double)n4 / (ms * 1e-3) / 1e9);
    }
  }
  if (e != hipSuccess) g_create_error = std::string("lbm_probe_stream: ") + hipGetErrorString(e);
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (st) (void)hipStreamDestroy(st);
  if (a) (void)hipFree(a);
  if (b) (void)hipFree(b);
  return e == hipSuccess ? LBM_OK : LBM_ERR_HIP;
}

int lbm_rccl_unique_id(uint8_t out_id[128]) {
  if (!out_id) return LBM_ERR_ARG;
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) {
    g_create_error = std::string("ncclGetUniqueId: ") + ncclGetErrorString(r);
    return LBM_ERR_RCCL;
  }
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
  std::memcpy(out_id, &id, 128);
  return LBM_OK;
}

int lbm_comm_info(lbm_ctx* c, int* rank, int* nranks) {
  if (!c) return LBM_ERR_ARG;
  if (c->comm_failed) return comm_failed_error(c);
  int n = 1;
  if (c->comm) NCCK(c, ncclCommCount(c->comm, &n));
  if (rank) *rank = c->comm ? c->rank : 0;
  if (nranks) *nranks = c->comm ? n : 1;
  return LBM_OK;
}

int lbm_debug_poison_walls(lbm_ctx* c) {
  if (!c) return LBM_ERR_ARG;
  RCK(lbm_sync(c));
  const int64_t n = c->compact ? c->ncell_c : c->L.ncell;
  const uint8_t* t = c->compact ? c->ctype : c->type;
  for (int b = 0; b < 2; ++b) HIPCK(c, launch_poison_walls(c->buf[b], t, n, c->s_comp));
  HIPCK(c, hipStreamSynchronize(c->s_comp));
  c->macros_stale = true;
  return LBM_OK;
}

int lbm_debug_fail_next_wait(lbm_ctx* c) {
  if (!c) return LBM_ERR_ARG;
  if (!c->comm) {
    c->err = "lbm_debug_fail_next_wait: the context has no RCCL communicator";
    return LBM_ERR_STATE;
  }
  c->inject_fault = true;
  return LBM_OK;
}

int lbm_attach_rccl(lbm_ctx* c, const uint8_t id_bytes[128], int rank, int nranks) {
  if (!c || !id_bytes || rank < 0 || nranks < 1 || rank >= nranks) return LBM_ERR_ARG;
  HIPCK(c, hipSetDevice(c->d.device));
  ncclUniqueId id;
  std::memcpy(&id, id_bytes, 128);
  if (c->sum_mode != LBM_SUM_FP64) {
    c->err = "lbm_attach_rccl: the reference-order residual (lbm_set_residual_order) is single-domain only";
    return LBM_ERR_ARG;
  }
  if (c->compact) {
    c->err = "lbm_attach_rccl: a lattice in compact rows is a single domain (create slabs with nz_global, or "
             "lbm_tune(LBM_TUNE_COMPACT, 1))";
    return LBM_ERR_STATE;
  }
  // the steps so far may have bounced back on the consumer side and written no wall slots; the
  // slab sequence's producer side pulls them from the next step on, and a read-out before that
  // step computes the macros producer-side from the last step's source: both buffers get them
  // once from the current state, as the producers would have stored them (prime_walls)
  RCK(prime_walls(c));
  RCK(materialize_nee(c));  // the slab sequence stores and pulls the NEE slots producer-side
  NCCK(c, ncclCommInitRank(&c->comm, nranks, id, rank));
  c->rank = rank;
  c->nranks = nranks;
  {  // every slab must use the same row layout: the halo planes are copied cell for cell
    const int key = (c->L.pitch * 4 + c->L.xshift) * 2 + c->L.swap;
    int h[2] = {key, -key};
    int* dv = nullptr;
    HIPCK(c, hipMalloc(&dv, sizeof(h)));
    HIPCK(c, hipMemcpy(dv, h, sizeof(h), hipMemcpyHostToDevice));
    NCCK(c, ncclAllReduce(dv, dv, 2, ncclInt, ncclMax, c->comm, c->s_comp));
    HIPCK(c, hipStreamSynchronize(c->s_comp));
    HIPCK(c, hipMemcpy(h, dv, sizeof(h), hipMemcpyDeviceToHost));
    HIPCK(c, hipFree(dv));
    if (h[0] != -h[1]) {
      c->err = "slabs differ in row layout (row axis / pitch / alignment); give every rank the same nx, ny, "
               "row_axis and x_align";
      return LBM_ERR_GEOMETRY;
    }
  }
  c->halo_primed = false;
  return LBM_OK;
}

}  // extern "C"

// ---- single-device loopback decomposition -------------------------------------------------

namespace {
__global__ void k_sum_locals(ConvState** convs, int n) {
  if (convs[0]->stopped) return;
  double s = 0.0;
  for (int i = 0; i < n; ++i) s += convs[i]->s_local;
  for (int i = 0; i < n; ++i) convs[i]->s_global = s;
}

// slab i's packed top face -> slab i+1's bottom ghost; slab i+1's bottom face -> slab i's top
int loopback_exchange(lbm_ctx** cs, int n, int b, bool all, hipStream_t st) {
  for (int i = 0; i < n; ++i) RCK(pack_faces(cs[i], b, all, i > 0, i + 1 < n, st));
  const size_t bytes = sizeof(float) * (all ? kQ : 5) * (size_t)cs[0]->L.plane;
  for (int i = 0; i + 1 < n; ++i) {
    HIPCK(cs[i], hipMemcpyAsync(cs[i + 1]->recv_dn, cs[i]->send_up, bytes, hipMemcpyDeviceToDevice, st));
    HIPCK(cs[i], hipMemcpyAsync(cs[i]->recv_up, cs[i + 1]->send_dn, bytes, hipMemcpyDeviceToDevice, st));
  }
  for (int i = 0; i < n; ++i) RCK(unpack_faces(cs[i], b, all, i > 0, i + 1 < n, st));
  return LBM_OK;
}
}  // namespace

extern "C" int lbm_group_step(lbm_ctx** cs, int n, int nsteps, float* residual_hist) {
  if (!cs || n < 1 || nsteps < 0) return LBM_ERR_ARG;
  lbm_ctx* c0 = cs[0];
  for (int i = 0; i < n; ++i) {
    if (!cs[i] || cs[i]->d.device != c0->d.device || cs[i]->L.pitch != c0->L.pitch || cs[i]->L.xshift != c0->L.xshift ||
        cs[i]->L.swap != c0->L.swap || cs[i]->L.plane != c0->L.plane ||
        cs[i]->steps_done != c0->steps_done || cs[i]->cur != c0->cur || cs[i]->conv_enabled || cs[i]->comm ||
        cs[i]->sum_mode != LBM_SUM_FP64 || cs[i]->compact) {
      c0->err = "lbm_group_step: slabs must share device, row layout (nx, ny, x_align) and step count, "
                "without convergence control or RCCL";
      return LBM_ERR_ARG;
    }
  }
  HIPCK(c0, hipSetDevice(c0->d.device));
  hipStream_t st = c0->s_comp;  // one stream: slabs run back to back (test / debug path)
  for (int i = 0; i < n; ++i) {
    HIPCK(c0, hipStreamSynchronize(cs[i]->s_comp));
    RCK(ensure_halo_buffers(cs[i]));
    // the slab ranges bounce back on the producer side: a context that stepped its whole domain
    // consumer-side first gets its wall slots back
    if (prime_walls(cs[i]) != LBM_OK || materialize_nee(cs[i]) != LBM_OK) {
      c0->err = cs[i]->err;
      return LBM_ERR_HIP;
    }
  }
  ConvState** dconvs = nullptr;
  HIPCK(c0, hipMalloc(&dconvs, sizeof(ConvState*) * n));
  struct DevFree {  // every return below releases dconvs
    void* p;
    ~DevFree() { (void)hipFree(p); }
  } dconvs_guard{dconvs};
  std::vector<ConvState*> hc(n);
  for (int i = 0; i < n; ++i) hc[i] = cs[i]->conv;
  HIPCK(c0, hipMemcpy(dconvs, hc.data(), sizeof(ConvState*) * n, hipMemcpyHostToDevice));
  RCK(ensure_hist(c0, std::max(nsteps, 1)));
  if (!c0->halo_primed) {
    RCK(loopback_exchange(cs, n, c0->cur, true, st));
    for (int i = 0; i < n; ++i) cs[i]->halo_primed = true;
  }
  for (int s = 0; s < nsteps; ++s) {
    for (int i = 0; i < n; ++i) {
      lbm_ctx* c = cs[i];
      RCK(run_range(c, c->edge, c0->cur, st));
      RCK(run_range(c, c->mid, c0->cur, st));
      HIPCK(c, launch_reduce(c->edge.part, c->npart_slab, c->scratch, c->conv, nullptr, 0, st));
    }
    RCK(loopback_exchange(cs, n, c0->cur ^ 1, false, st));
    for (int i = 0; i < n; ++i) cs[i]->cur ^= 1;
    hipLaunchKernelGGL(k_sum_locals, dim3(1), dim3(1), 0, st, dconvs, n);
    for (int i = 0; i < n; ++i)
      HIPCK(c0, launch_finish_global(cs[i]->conv, (i == 0 && residual_hist) ? c0->hist + s : nullptr, st));
  }
  HIPCK(c0, hipStreamSynchronize(st));
  for (int i = 0; i < n; ++i) {
    cs[i]->steps_done += nsteps;
    cs[i]->macros_stale = true;
  }
  if (residual_hist && nsteps > 0)
    HIPCK(c0, hipMemcpy(residual_hist, c0->hist, sizeof(float) * nsteps, hipMemcpyDeviceToHost));
  return LBM_OK;
}
