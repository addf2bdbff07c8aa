// lbm_kernels.hpp -- internal launch interface between the context code (lbm_ctx.hip)
// and the HIP kernels (lbm_kernels.hip).  Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <utility>

namespace lbm {

// Device storage of one lattice (or z-slab): raster SoA, x fastest, rows padded to a
// multiple of 64 floats (one wavefront = one 256-B aligned row segment), one ghost
// plane below and above the nz local planes (storage plane = local z + 1).
struct Layout {
  int nx, ny, nz;
  int pitch;        // row pitch in floats (multiple of 64)
  int planes;       // nz + 2
  int64_t plane;    // pitch * ny
  int64_t qstride;  // floats between two populations (>= plane * planes, multiple of 64)
};

// Arguments of one collide-stream launch over storage planes [z_begin, z_end).
struct StepArgs {
  const float* src;
  float* dst;
  const uint8_t* type;
  float* rho;
  float* ux;
  float* uy;
  float* uz;
  double* partial;      // one |u| partial sum per block
  int64_t qstride;
  int64_t plane;
  int pitch, ny;
  int z_begin;          // first storage plane
  int ntx, nty;         // tiles of 64 x 4 cells per plane
  int ntiles;           // ntx * nty * (z_end - z_begin)
  float tau;            // BGK: f - (f - feq) / tau
  float omc;            // (1.0f - 1.0f / tau) of the NEE formula
  int bb_active;        // wall neighbours bounce back (else raw pull: reference step 0)
  int nee_active;       // NEE neighbours extrapolate (else raw pull: reference step 0)
  int store_all_macros; // write (rho,u) of every fluid cell (else only kNeedsMac cells)
  const int* stopped;   // device convergence flag (nullable)
};

struct ConvState {      // device-resident reference main-loop state (ldc.cu:613-685)
  double s_local;       // this rank's sum of |u| for the last step
  double s_global;      // after the cross-rank all-reduce
  float sum_current;    // S_{k-1} as float (ldc.cu:683)
  float residual;       // last residual
  int k;                // steps executed
  int tol_count;
  int stopped;
  int enabled;          // convergence stopping on/off
  int max_it, stag_max;
  float tol;
  int pad;
};

constexpr int kBlock = 256;       // 4 wavefronts: 64 x-cells x 4 rows
constexpr int kTileX = 64, kTileY = 4;

hipError_t launch_collide_stream(const StepArgs& a, int grid, hipStream_t s);
// sums `n` block partials into conv->s_local; with finish=1 also runs the residual logic
hipError_t launch_finish(const double* partial, int n, ConvState* conv, float* hist_slot,
                         int finish, hipStream_t s);
// residual logic on conv->s_global (multi-rank, after the all-reduce)
hipError_t launch_finish_global(ConvState* conv, float* hist_slot, hipStream_t s);

// geometry: reference codes (int8, storage layout incl. ghost planes) -> cell-type bytes
struct GeoArgs {
  const int8_t* codes;  // storage layout, pitch/planes as Layout; padding = 0
  uint8_t* type;
  float* rho; float* ux; float* uy; float* uz;  // NEE data written at NEE cells
  const float* inlet_uy;   // nx * nz_global (nullable)
  const float* outlet_uy;  // nx * nz_global (nullable)
  int case_kind;
  float lid_u;
  int nx, ny, pitch, planes;
  int64_t plane;
  int z_offset;            // global z of local plane 0
  int nz_global;           // extent of the boundary tables in z
};
hipError_t launch_classify(const GeoArgs& g, hipStream_t s);
hipError_t launch_flag_fluid(const GeoArgs& g, hipStream_t s);
// LDC cavity codes generated from global coordinates (ldc.cu:468-502)
hipError_t launch_ldc_codes(int8_t* codes, int nx, int ny, int pitch, int planes, int64_t plane,
                            int z_offset, int nz_global, hipStream_t s);

// initial populations: form 0 = LDC wi form, 1 = expanded; fields in storage layout
// (nullable -> rho 1, u 0); writes both buffers over every storage cell
hipError_t launch_init_feq(float* fa, float* fb, int64_t qstride, int64_t ncell_storage,
                           int form, const float* rho, const float* ux, const float* uy,
                           const float* uz, hipStream_t s);
// LDC initial state from global coordinates (ldc.cu:504-580)
hipError_t launch_init_ldc(float* fa, float* fb, int64_t qstride, int nx, int ny, int pitch,
                           int planes, int64_t plane, int z_offset, float lid_u, hipStream_t s);

}  // namespace lbm
