// lbm_ctx.hip -- liblbm.so: the C ABI of include/lbm.h on top of the HIP kernels.
//
// A context owns one lattice (or one z-slab of it) on one device:
//   two population buffers (A-B pattern; the reference's d_scr/d_dst, ldc.cu:640-641),
//   the cell-type bytes (the reference's d_geo + texture-bound index, Poiseulle.cu:49-50),
//   (rho, u) arrays (d_rho/d_ux/d_uy/d_uz), block partials of the |u| sum and the
//   device-resident state of the reference main loop (ldc.cu:613-685).
// The reference's per-step launch sequence update -> boundary_stream -> calc_vel_square
// -> thrust::reduce -> host residual (ldc.cu:654-684) becomes one fused collide-stream
// launch plus a one-block finisher, with no host synchronisation inside a call.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/lbm.h"
#include "lbm_d3q19.hpp"
#include "lbm_kernels.hpp"

using namespace lbm;

namespace {
std::string g_create_error;
constexpr int kUpSet[5] = {5, 11, 13, 15, 16};    // e_z = +1: cross the top face
constexpr int kDownSet[5] = {6, 12, 14, 17, 18};  // e_z = -1: cross the bottom face
}  // namespace

struct lbm_ctx {
  lbm_desc d{};
  Layout L{};
  hipStream_t s_comp = nullptr, s_comm = nullptr;
  hipEvent_t ev_edge = nullptr, ev_halo = nullptr, ev_sum = nullptr, ev_fin = nullptr;
  float* buf[2] = {nullptr, nullptr};
  uint8_t* type = nullptr;
  float *rho = nullptr, *ux = nullptr, *uy = nullptr, *uz = nullptr;
  double* partial = nullptr;
  int grid_full = 0, grid_plane = 0;
  ConvState* conv = nullptr;
  float* hist = nullptr;
  int hist_cap = 0;
  int steps_done = 0;      // device-confirmed steps
  bool bb_immediate = false;
  bool conv_enabled = false;
  bool halo_primed = false;
  int64_t n_box = 0, n_fluid = 0;
  float tau = 0.f, omc = 0.f;
  // profiling
  bool prof = false;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  double kernel_ms = 0.0;
  int64_t launches = 0;
  // rccl
  ncclComm_t comm = nullptr;
  int rank = 0, nranks = 1;
  std::string err;
};

#define HIPCK(ctx, expr)                                                                    \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) {                                                                 \
      (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(e_);                       \
      return LBM_ERR_HIP;                                                                   \
    }                                                                                       \
  } while (0)

#define NCCK(ctx, expr)                                                                     \
  do {                                                                                      \
    ncclResult_t r_ = (expr);                                                               \
    if (r_ != ncclSuccess) {                                                                \
      (ctx)->err = std::string(#expr) + ": " + ncclGetErrorString(r_);                      \
      return LBM_ERR_RCCL;                                                                  \
    }                                                                                       \
  } while (0)

namespace {

int fail(lbm_ctx* c, int code, const std::string& msg) {
  c->err = msg;
  return code;
}

float* pop(lbm_ctx* c, int b, int q) { return c->buf[b] + (int64_t)q * c->L.qstride; }
float* src_buf(lbm_ctx* c) { return c->buf[c->steps_done & 1]; }

StepArgs make_args(lbm_ctx* c, int hstep, int z_begin, int z_end, double* partial, bool store_all) {
  StepArgs a{};
  const bool first = (hstep == 0);
  a.src = c->buf[hstep & 1];
  a.dst = c->buf[(hstep + 1) & 1];
  a.type = c->type;
  a.rho = c->rho; a.ux = c->ux; a.uy = c->uy; a.uz = c->uz;
  a.partial = partial;
  a.qstride = c->L.qstride;
  a.plane = c->L.plane;
  a.pitch = c->L.pitch;
  a.ny = c->L.ny;
  a.z_begin = z_begin;
  a.ntx = c->L.pitch / kTileX;
  a.nty = (c->L.ny + kTileY - 1) / kTileY;
  a.ntiles = a.ntx * a.nty * std::max(0, z_end - z_begin);
  a.tau = c->tau;
  a.omc = c->omc;
  a.bb_active = (!first || c->bb_immediate) ? 1 : 0;
  a.nee_active = first ? 0 : 1;
  a.store_all_macros = store_all ? 1 : 0;
  a.stopped = c->conv_enabled ? &c->conv->stopped : nullptr;
  return a;
}

int launch_cs(lbm_ctx* c, const StepArgs& a, int grid) {
  if (a.ntiles <= 0) {
    HIPCK(c, hipMemsetAsync(a.partial, 0, sizeof(double) * grid, c->s_comp));
    return LBM_OK;
  }
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (c->prof) {
    while (c->ev_pool.size() < c->ev_used + 2) {
      hipEvent_t e;
      HIPCK(c, hipEventCreate(&e));
      c->ev_pool.push_back(e);
    }
    e0 = c->ev_pool[c->ev_used++];
    e1 = c->ev_pool[c->ev_used++];
    HIPCK(c, hipEventRecord(e0, c->s_comp));
  }
  HIPCK(c, launch_collide_stream(a, grid, c->s_comp));
  if (c->prof) HIPCK(c, hipEventRecord(e1, c->s_comp));
  c->launches++;
  return LBM_OK;
}

int harvest_profile(lbm_ctx* c) {
  if (c->ev_used == 0) return LBM_OK;
  HIPCK(c, hipStreamSynchronize(c->s_comp));
  for (size_t i = 0; i + 1 < c->ev_used; i += 2) {
    float ms = 0.f;
    HIPCK(c, hipEventElapsedTime(&ms, c->ev_pool[i], c->ev_pool[i + 1]));
    c->kernel_ms += ms;
  }
  c->ev_used = 0;
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
  ConvState cs{};
  ConvState host{};
  HIPCK(c, hipMemcpy(&host, c->conv, sizeof(ConvState), hipMemcpyDeviceToHost));
  cs.enabled = host.enabled;
  cs.max_it = host.max_it;
  cs.stag_max = host.stag_max;
  cs.tol = host.tol;
  HIPCK(c, hipMemcpy(c->conv, &cs, sizeof(ConvState), hipMemcpyHostToDevice));
  c->steps_done = 0;
  c->halo_primed = false;
  return LBM_OK;
}

// raster [nz][ny][nx] (local planes) <-> storage offsets
int64_t sidx(const Layout& L, int x, int y, int z) {
  return (int64_t)x + (int64_t)y * L.pitch + (int64_t)(z + 1) * L.plane;
}

}  // namespace

extern "C" {

const char* lbm_version(void) { return "lbm-mi355x 0.1 (gfx950, D3Q19 BGK fused pull/collide)"; }

const char* lbm_last_error(const lbm_ctx* ctx) {
  return ctx ? ctx->err.c_str() : g_create_error.c_str();
}

int lbm_create(const lbm_desc* desc, lbm_ctx** out) {
  if (!desc || !out) { g_create_error = "null argument"; return LBM_ERR_ARG; }
  *out = nullptr;
  const lbm_desc& d = *desc;
  if (d.nx < 3 || d.ny < 3 || d.nz < 1 || d.tau <= 0.f || d.case_kind < 0 || d.case_kind > 2) {
    g_create_error = "invalid lattice description";
    return LBM_ERR_ARG;
  }
  if (!d.geo && d.case_kind != LBM_CASE_LDC) {
    g_create_error = "geo == NULL is only supported for LBM_CASE_LDC";
    return LBM_ERR_ARG;
  }
  lbm_ctx* c = new lbm_ctx();
  c->d = d;
  c->d.geo = nullptr; c->d.bc_inlet_uy = nullptr; c->d.bc_outlet_uy = nullptr;
  if (c->d.nz_global <= 0) c->d.nz_global = d.nz;
  c->tau = d.tau;
  c->omc = 1.0f - 1.0f / d.tau;  // the reference's (1.0f - 1.0f / tau), evaluated in fp32
  c->bb_immediate = (d.case_kind == LBM_CASE_LDC);
  Layout& L = c->L;
  L.nx = d.nx; L.ny = d.ny; L.nz = d.nz;
  L.pitch = (d.nx + kTileX - 1) / kTileX * kTileX;
  L.planes = d.nz + 2;
  L.plane = (int64_t)L.pitch * L.ny;
  const int64_t ncs = L.plane * L.planes;
  L.qstride = (ncs + 63) / 64 * 64;
  if (ncs >= (int64_t(1) << 30)) {
    g_create_error = "slab too large for 32-bit cell offsets (use more z-slabs)";
    delete c;
    return LBM_ERR_ARG;
  }
  c->n_box = (int64_t)d.nx * d.ny * d.nz;

  auto bail = [&](int code) {
    g_create_error = c->err;
    lbm_destroy(c);
    return code;
  };
#define CK(expr)                                                   \
  do {                                                             \
    hipError_t e_ = (expr);                                        \
    if (e_ != hipSuccess) {                                        \
      c->err = std::string(#expr) + ": " + hipGetErrorString(e_);  \
      return bail(LBM_ERR_HIP);                                    \
    }                                                              \
  } while (0)

  CK(hipSetDevice(d.device));
  CK(hipStreamCreateWithFlags(&c->s_comp, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&c->s_comm, hipStreamNonBlocking));
  CK(hipEventCreateWithFlags(&c->ev_edge, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&c->ev_halo, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&c->ev_sum, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&c->ev_fin, hipEventDisableTiming));
  CK(hipMalloc(&c->buf[0], sizeof(float) * 19 * L.qstride));
  CK(hipMalloc(&c->buf[1], sizeof(float) * 19 * L.qstride));
  CK(hipMalloc(&c->type, L.qstride));
  CK(hipMalloc(&c->rho, sizeof(float) * L.qstride));
  CK(hipMalloc(&c->ux, sizeof(float) * L.qstride));
  CK(hipMalloc(&c->uy, sizeof(float) * L.qstride));
  CK(hipMalloc(&c->uz, sizeof(float) * L.qstride));
  CK(hipMalloc(&c->conv, sizeof(ConvState)));
  CK(hipMemsetAsync(c->conv, 0, sizeof(ConvState), c->s_comp));
  for (float* p : {c->rho, c->ux, c->uy, c->uz}) CK(hipMemsetAsync(p, 0, sizeof(float) * L.qstride, c->s_comp));
  CK(hipMemsetAsync(c->type, 0, L.qstride, c->s_comp));

  // grid: enough resident blocks to fill the chip, each striding over 64x4 tiles
  int ncu = 256;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, d.device));
  const int occ = 8;  // resident 256-thread blocks per CU the grid is sized for
  const int ntx = L.pitch / kTileX, nty = (L.ny + kTileY - 1) / kTileY;
  const int64_t tiles_full = (int64_t)ntx * nty * d.nz, tiles_plane = (int64_t)ntx * nty;
  c->grid_full = (int)std::max<int64_t>(1, std::min<int64_t>(tiles_full, (int64_t)ncu * occ));
  c->grid_plane = (int)std::max<int64_t>(1, std::min<int64_t>(tiles_plane, (int64_t)ncu * occ));
  // partial slots: [full | edge lo | edge hi | interior]
  CK(hipMalloc(&c->partial, sizeof(double) * (c->grid_full + 2 * c->grid_plane + c->grid_full)));

  // ---- geometry: reference codes in storage layout -> type bytes ----
  int8_t* dcodes = nullptr;
  CK(hipMalloc(&dcodes, L.qstride));
  CK(hipMemsetAsync(dcodes, 0, L.qstride, c->s_comp));
  float *din = nullptr, *dout = nullptr;
  if (d.geo) {
    std::vector<int8_t> h((size_t)ncs, 0);
    const int zlo = d.halo_planes ? -1 : 0, zhi = d.halo_planes ? d.nz + 1 : d.nz;
    for (int z = zlo; z < zhi; ++z)
      for (int y = 0; y < d.ny; ++y) {
        const int8_t* srow = d.geo + ((int64_t)(z - zlo) * d.ny + y) * d.nx;
        std::memcpy(&h[sidx(L, 0, y, z)], srow, d.nx);
      }
    CK(hipMemcpyAsync(dcodes, h.data(), ncs, hipMemcpyHostToDevice, c->s_comp));
    CK(hipStreamSynchronize(c->s_comp));
  } else {
    CK(launch_ldc_codes(dcodes, d.nx, d.ny, L.pitch, L.planes, L.plane, d.z_offset, c->d.nz_global,
                        c->s_comp));
  }
  const int64_t ntab = (int64_t)d.nx * c->d.nz_global;
  if (desc->bc_inlet_uy) {
    CK(hipMalloc(&din, sizeof(float) * ntab));
    CK(hipMemcpy(din, desc->bc_inlet_uy, sizeof(float) * ntab, hipMemcpyHostToDevice));
  }
  if (desc->bc_outlet_uy) {
    CK(hipMalloc(&dout, sizeof(float) * ntab));
    CK(hipMemcpy(dout, desc->bc_outlet_uy, sizeof(float) * ntab, hipMemcpyHostToDevice));
  }
  GeoArgs g{};
  g.codes = dcodes; g.type = c->type;
  g.rho = c->rho; g.ux = c->ux; g.uy = c->uy; g.uz = c->uz;
  g.inlet_uy = din; g.outlet_uy = dout;
  g.case_kind = d.case_kind; g.lid_u = d.lid_u;
  g.nx = d.nx; g.ny = d.ny; g.pitch = L.pitch; g.planes = L.planes; g.plane = L.plane;
  g.z_offset = d.z_offset;
  g.nz_global = c->d.nz_global;
  CK(launch_classify(g, c->s_comp));
  CK(launch_flag_fluid(g, c->s_comp));
  CK(hipStreamSynchronize(c->s_comp));
  CK(hipFree(dcodes));
  if (din) CK(hipFree(din));
  if (dout) CK(hipFree(dout));

  // count fluid cells of the local planes
  {
    std::vector<uint8_t> t((size_t)ncs);
    CK(hipMemcpy(t.data(), c->type, ncs, hipMemcpyDeviceToHost));
    int64_t nf = 0;
    for (int z = 0; z < d.nz; ++z)
      for (int y = 0; y < d.ny; ++y)
        for (int x = 0; x < d.nx; ++x)
          if ((t[sidx(L, x, y, z)] & kClassMask) == kFluid) ++nf;
    c->n_fluid = nf;
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
  for (float* p : {c->buf[0], c->buf[1], c->rho, c->ux, c->uy, c->uz, c->hist})
    if (p) (void)hipFree(p);
  if (c->type) (void)hipFree(c->type);
  if (c->partial) (void)hipFree(c->partial);
  if (c->conv) (void)hipFree(c->conv);
  for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
  for (hipEvent_t e : {c->ev_edge, c->ev_halo, c->ev_sum, c->ev_fin})
    if (e) (void)hipEventDestroy(e);
  if (c->s_comp) (void)hipStreamDestroy(c->s_comp);
  if (c->s_comm) (void)hipStreamDestroy(c->s_comm);
  delete c;
}

int lbm_init_equilibrium(lbm_ctx* c, int form, const float* rho, const float* ux, const float* uy,
                         const float* uz) {
  if (!c || (form != LBM_INIT_LDC_WI && form != LBM_INIT_EXPANDED)) return LBM_ERR_ARG;
  HIPCK(c, hipSetDevice(c->d.device));
  const Layout& L = c->L;
  const int64_t ncs = L.plane * L.planes;
  const float* host[4] = {rho, ux, uy, uz};
  float* dev[4] = {nullptr, nullptr, nullptr, nullptr};
  std::vector<float> h;
  for (int k = 0; k < 4; ++k) {
    if (!host[k]) continue;
    h.assign((size_t)ncs, k == 0 ? 1.0f : 0.0f);
    for (int z = 0; z < L.nz; ++z)
      for (int y = 0; y < L.ny; ++y)
        std::memcpy(&h[sidx(L, 0, y, z)], host[k] + ((int64_t)z * L.ny + y) * L.nx, sizeof(float) * L.nx);
    HIPCK(c, hipMalloc(&dev[k], sizeof(float) * ncs));
    HIPCK(c, hipMemcpy(dev[k], h.data(), sizeof(float) * ncs, hipMemcpyHostToDevice));
  }
  HIPCK(c, launch_init_feq(c->buf[0], c->buf[1], L.qstride, ncs, form == LBM_INIT_LDC_WI ? 0 : 1, dev[0],
                           dev[1], dev[2], dev[3], c->s_comp));
  HIPCK(c, hipStreamSynchronize(c->s_comp));
  for (float* p : dev)
    if (p) HIPCK(c, hipFree(p));
  return reset_state(c);
}

int lbm_init_ldc(lbm_ctx* c) {
  if (!c) return LBM_ERR_ARG;
  HIPCK(c, hipSetDevice(c->d.device));
  const Layout& L = c->L;
  HIPCK(c, launch_init_ldc(c->buf[0], c->buf[1], L.qstride, L.nx, L.ny, L.pitch, L.planes, L.plane,
                           c->d.z_offset, c->d.lid_u, c->s_comp));
  HIPCK(c, hipStreamSynchronize(c->s_comp));
  return reset_state(c);
}

int lbm_set_f(lbm_ctx* c, const float* f) {
  if (!c || !f) return LBM_ERR_ARG;
  HIPCK(c, hipSetDevice(c->d.device));
  const Layout& L = c->L;
  std::vector<float> h((size_t)L.qstride, 0.f);
  for (int q = 0; q < 19; ++q) {
    for (int z = 0; z < L.nz; ++z)
      for (int y = 0; y < L.ny; ++y)
        std::memcpy(&h[sidx(L, 0, y, z)], f + (((int64_t)q * L.nz + z) * L.ny + y) * L.nx,
                    sizeof(float) * L.nx);
    HIPCK(c, hipMemcpy(pop(c, 0, q), h.data(), sizeof(float) * L.qstride, hipMemcpyHostToDevice));
    HIPCK(c, hipMemcpy(pop(c, 1, q), h.data(), sizeof(float) * L.qstride, hipMemcpyHostToDevice));
  }
  return reset_state(c);
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

// RCCL: send the top local plane's up-going populations to rank+1 (into its bottom ghost plane)
// and the bottom plane's down-going populations to rank-1 (into its top ghost plane).
int rccl_exchange(lbm_ctx* c, int b, int npops_all) {
  const Layout& L = c->L;
  const size_t cnt = (size_t)L.plane;
  NCCK(c, ncclGroupStart());
  const int up = c->rank + 1 < c->nranks ? c->rank + 1 : -1;
  const int dn = c->rank > 0 ? c->rank - 1 : -1;
  for (int k = 0; k < (npops_all ? 19 : 5); ++k) {
    const int qu = npops_all ? k : kUpSet[k];
    const int qd = npops_all ? k : kDownSet[k];
    if (up >= 0) {
      NCCK(c, ncclSend(pop(c, b, qu) + (int64_t)L.nz * L.plane, cnt, ncclFloat, up, c->comm, c->s_comm));
      NCCK(c, ncclRecv(pop(c, b, qd) + (int64_t)(L.nz + 1) * L.plane, cnt, ncclFloat, up, c->comm, c->s_comm));
    }
    if (dn >= 0) {
      NCCK(c, ncclSend(pop(c, b, qd) + (int64_t)1 * L.plane, cnt, ncclFloat, dn, c->comm, c->s_comm));
      NCCK(c, ncclRecv(pop(c, b, qu) + 0, cnt, ncclFloat, dn, c->comm, c->s_comm));
    }
  }
  NCCK(c, ncclGroupEnd());
  return LBM_OK;
}

int step_single(lbm_ctx* c, int nsteps, bool want_hist) {
  const Layout& L = c->L;
  int h = c->steps_done;
  for (int s = 0; s < nsteps; ++s, ++h) {
    const bool store_all = c->conv_enabled || (s == nsteps - 1);
    StepArgs a = make_args(c, h, 1, L.nz + 1, c->partial, store_all);
    int rc = launch_cs(c, a, c->grid_full);
    if (rc) return rc;
    HIPCK(c, launch_finish(c->partial, c->grid_full, c->conv, want_hist ? c->hist + s : nullptr, 1,
                           c->s_comp));
  }
  return LBM_OK;
}

int step_rccl(lbm_ctx* c, int nsteps, bool want_hist) {
  const Layout& L = c->L;
  double* p_lo = c->partial + c->grid_full;
  double* p_hi = p_lo + c->grid_plane;
  double* p_in = p_hi + c->grid_plane;
  const int n_part = 2 * c->grid_plane + c->grid_full;
  if (!c->halo_primed) {  // initial ghost planes of the source buffer: all 19 populations
    HIPCK(c, hipEventRecord(c->ev_edge, c->s_comp));
    HIPCK(c, hipStreamWaitEvent(c->s_comm, c->ev_edge, 0));
    int rc = rccl_exchange(c, c->steps_done & 1, 1);
    if (rc) return rc;
    HIPCK(c, hipEventRecord(c->ev_halo, c->s_comm));
    c->halo_primed = true;
  }
  int h = c->steps_done;
  for (int s = 0; s < nsteps; ++s, ++h) {
    const bool store_all = c->conv_enabled || (s == nsteps - 1);
    HIPCK(c, hipStreamWaitEvent(c->s_comp, c->ev_halo, 0));  // ghost planes of src(h) complete
    if (c->conv_enabled) HIPCK(c, hipStreamWaitEvent(c->s_comp, c->ev_fin, 0));
    // edge planes first, so their halo can travel while the interior runs
    StepArgs lo = make_args(c, h, 1, 2, p_lo, store_all);
    int rc = launch_cs(c, lo, c->grid_plane);
    if (rc) return rc;
    if (L.nz > 1) {
      StepArgs hi = make_args(c, h, L.nz, L.nz + 1, p_hi, store_all);
      rc = launch_cs(c, hi, c->grid_plane);
      if (rc) return rc;
    } else {
      HIPCK(c, hipMemsetAsync(p_hi, 0, sizeof(double) * c->grid_plane, c->s_comp));
    }
    HIPCK(c, hipEventRecord(c->ev_edge, c->s_comp));
    HIPCK(c, hipStreamWaitEvent(c->s_comm, c->ev_edge, 0));
    rc = rccl_exchange(c, (h + 1) & 1, 0);
    if (rc) return rc;
    HIPCK(c, hipEventRecord(c->ev_halo, c->s_comm));
    // interior planes overlap the exchange
    StepArgs in = make_args(c, h, 2, L.nz, p_in, store_all);
    rc = launch_cs(c, in, c->grid_full);
    if (rc) return rc;
    HIPCK(c, launch_finish(p_lo, n_part, c->conv, nullptr, 0, c->s_comp));
    HIPCK(c, hipEventRecord(c->ev_sum, c->s_comp));
    HIPCK(c, hipStreamWaitEvent(c->s_comm, c->ev_sum, 0));
    NCCK(c, ncclAllReduce(&c->conv->s_local, &c->conv->s_global, 1, ncclDouble, ncclSum, c->comm, c->s_comm));
    HIPCK(c, launch_finish_global(c->conv, want_hist ? c->hist + s : nullptr, c->s_comm));
    HIPCK(c, hipEventRecord(c->ev_fin, c->s_comm));
  }
  HIPCK(c, hipStreamWaitEvent(c->s_comp, c->ev_fin, 0));
  HIPCK(c, hipStreamWaitEvent(c->s_comp, c->ev_halo, 0));
  return LBM_OK;
}

}  // namespace

extern "C" {

int lbm_step(lbm_ctx* c, int nsteps, float* residual_hist, int* steps_done) {
  if (!c || nsteps < 0) return LBM_ERR_ARG;
  if (nsteps == 0) {
    if (steps_done) *steps_done = c->steps_done;
    return LBM_OK;
  }
  HIPCK(c, hipSetDevice(c->d.device));
  const bool want_hist = residual_hist != nullptr;
  if (want_hist) {
    int rc = ensure_hist(c, nsteps);
    if (rc) return rc;
    HIPCK(c, hipMemsetAsync(c->hist, 0xFF, sizeof(float) * nsteps, c->s_comp));  // NaN: not run
  }
  int rc = c->comm ? step_rccl(c, nsteps, want_hist) : step_single(c, nsteps, want_hist);
  if (rc) return rc;
  const bool sync = want_hist || steps_done || c->conv_enabled;
  if (sync) {
    HIPCK(c, hipStreamSynchronize(c->s_comp));
    HIPCK(c, hipStreamSynchronize(c->s_comm));
    ConvState h{};
    HIPCK(c, hipMemcpy(&h, c->conv, sizeof(ConvState), hipMemcpyDeviceToHost));
    c->steps_done = h.k;  // device-confirmed (a converged run stops early)
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
  HIPCK(c, hipStreamSynchronize(c->s_comp));
  HIPCK(c, hipStreamSynchronize(c->s_comm));
  return LBM_OK;
}

int lbm_get_state(lbm_ctx* c, int* k, int* tol_count, int* stopped, float* residual, double* velsum) {
  if (!c) return LBM_ERR_ARG;
  HIPCK(c, hipSetDevice(c->d.device));
  int rc = lbm_sync(c);
  if (rc) return rc;
  ConvState h{};
  HIPCK(c, hipMemcpy(&h, c->conv, sizeof(ConvState), hipMemcpyDeviceToHost));
  if (k) *k = h.k;
  if (tol_count) *tol_count = h.tol_count;
  if (stopped) *stopped = h.stopped;
  if (residual) *residual = h.residual;
  if (velsum) *velsum = c->comm ? h.s_global : h.s_local;
  return LBM_OK;
}

int lbm_get_macros(lbm_ctx* c, float* rho, float* ux, float* uy, float* uz) {
  if (!c) return LBM_ERR_ARG;
  int rc = lbm_sync(c);
  if (rc) return rc;
  const Layout& L = c->L;
  const int64_t ncs = L.plane * L.planes;
  std::vector<uint8_t> t((size_t)ncs);
  HIPCK(c, hipMemcpy(t.data(), c->type, ncs, hipMemcpyDeviceToHost));
  std::vector<float> h((size_t)ncs);
  float* outs[4] = {rho, ux, uy, uz};
  float* devs[4] = {c->rho, c->ux, c->uy, c->uz};
  for (int k = 0; k < 4; ++k) {
    if (!outs[k]) continue;
    HIPCK(c, hipMemcpy(h.data(), devs[k], sizeof(float) * ncs, hipMemcpyDeviceToHost));
    for (int z = 0; z < L.nz; ++z)
      for (int y = 0; y < L.ny; ++y)
        for (int x = 0; x < L.nx; ++x) {
          const int64_t s = sidx(L, x, y, z);
          outs[k][((int64_t)z * L.ny + y) * L.nx + x] = ((t[s] & kClassMask) == kFluid) ? h[s] : 0.0f;
        }
  }
  return LBM_OK;
}

int lbm_get_f(lbm_ctx* c, float* f) {
  if (!c || !f) return LBM_ERR_ARG;
  int rc = lbm_sync(c);
  if (rc) return rc;
  const Layout& L = c->L;
  std::vector<float> h((size_t)L.qstride);
  for (int q = 0; q < 19; ++q) {
    HIPCK(c, hipMemcpy(h.data(), pop(c, c->steps_done & 1, q), sizeof(float) * L.qstride, hipMemcpyDeviceToHost));
    for (int z = 0; z < L.nz; ++z)
      for (int y = 0; y < L.ny; ++y)
        std::memcpy(f + (((int64_t)q * L.nz + z) * L.ny + y) * L.nx, &h[sidx(L, 0, y, z)], sizeof(float) * L.nx);
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

int lbm_profile(lbm_ctx* c, int enabled) {
  if (!c) return LBM_ERR_ARG;
  int rc = harvest_profile(c);
  if (rc) return rc;
  c->prof = enabled != 0;
  c->kernel_ms = 0.0;
  c->launches = 0;
  return LBM_OK;
}

int lbm_stats(lbm_ctx* c, double* kernel_ms, int64_t* launches, double* algo_bytes) {
  if (!c) return LBM_ERR_ARG;
  int rc = harvest_profile(c);
  if (rc) return rc;
  if (kernel_ms) *kernel_ms = c->kernel_ms;
  if (launches) *launches = c->launches;
  if (algo_bytes) *algo_bytes = 152.0 * (double)c->n_fluid;
  return LBM_OK;
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

int lbm_attach_rccl(lbm_ctx* c, const uint8_t id_bytes[128], int rank, int nranks) {
  if (!c || !id_bytes || rank < 0 || nranks < 1 || rank >= nranks) return LBM_ERR_ARG;
  HIPCK(c, hipSetDevice(c->d.device));
  ncclUniqueId id;
  std::memcpy(&id, id_bytes, 128);
  NCCK(c, ncclCommInitRank(&c->comm, nranks, id, rank));
  c->rank = rank;
  c->nranks = nranks;
  c->halo_primed = false;
  return LBM_OK;
}

}  // extern "C"

// ---- single-device loopback decomposition -------------------------------------------------

namespace {
__global__ void k_sum_locals(ConvState** convs, int n) {
  double s = 0.0;
  for (int i = 0; i < n; ++i) s += convs[i]->s_local;
  for (int i = 0; i < n; ++i) convs[i]->s_global = s;
}

int copy_plane(lbm_ctx* dst, int bd, int zd, lbm_ctx* src, int bs, int zs, int q, hipStream_t st) {
  const Layout& L = src->L;
  HIPCK(src, hipMemcpyAsync(pop(dst, bd, q) + (int64_t)zd * L.plane, pop(src, bs, q) + (int64_t)zs * L.plane,
                            sizeof(float) * L.plane, hipMemcpyDeviceToDevice, st));
  return LBM_OK;
}

// slab i's top plane -> slab i+1's bottom ghost; slab i+1's bottom plane -> slab i's top ghost
int loopback_exchange(lbm_ctx** cs, int n, int b, bool all, hipStream_t st) {
  for (int i = 0; i + 1 < n; ++i) {
    lbm_ctx *a = cs[i], *u = cs[i + 1];
    for (int k = 0; k < (all ? 19 : 5); ++k) {
      const int qu = all ? k : kUpSet[k], qd = all ? k : kDownSet[k];
      int rc = copy_plane(u, b, 0, a, b, a->L.nz, qu, st);
      if (rc) return rc;
      rc = copy_plane(a, b, a->L.nz + 1, u, b, 1, qd, st);
      if (rc) return rc;
    }
  }
  return LBM_OK;
}
}  // namespace

extern "C" int lbm_group_step(lbm_ctx** cs, int n, int nsteps, float* residual_hist) {
  if (!cs || n < 1 || nsteps < 0) return LBM_ERR_ARG;
  lbm_ctx* c0 = cs[0];
  for (int i = 0; i < n; ++i) {
    if (!cs[i] || cs[i]->d.device != c0->d.device || cs[i]->L.pitch != c0->L.pitch || cs[i]->L.ny != c0->L.ny ||
        cs[i]->steps_done != c0->steps_done || cs[i]->conv_enabled)
      return LBM_ERR_ARG;
  }
  HIPCK(c0, hipSetDevice(c0->d.device));
  hipStream_t st = c0->s_comp;  // one stream: slabs run back to back (debug / parity path)
  for (int i = 0; i < n; ++i) HIPCK(c0, hipStreamSynchronize(cs[i]->s_comp));
  ConvState** dconvs = nullptr;
  HIPCK(c0, hipMalloc(&dconvs, sizeof(ConvState*) * n));
  std::vector<ConvState*> hc(n);
  for (int i = 0; i < n; ++i) hc[i] = cs[i]->conv;
  HIPCK(c0, hipMemcpy(dconvs, hc.data(), sizeof(ConvState*) * n, hipMemcpyHostToDevice));
  int rc = ensure_hist(c0, std::max(nsteps, 1));
  if (rc) return rc;
  if (!c0->halo_primed) {
    rc = loopback_exchange(cs, n, c0->steps_done & 1, true, st);
    if (rc) return rc;
    for (int i = 0; i < n; ++i) cs[i]->halo_primed = true;
  }
  int h = c0->steps_done;
  for (int s = 0; s < nsteps; ++s, ++h) {
    const bool store_all = (s == nsteps - 1);
    for (int i = 0; i < n; ++i) {
      lbm_ctx* c = cs[i];
      StepArgs a = make_args(c, h, 1, c->L.nz + 1, c->partial, store_all);
      std::swap(c->s_comp, st);  // launch on the group stream
      rc = launch_cs(c, a, c->grid_full);
      std::swap(c->s_comp, st);
      if (rc) return rc;
      HIPCK(c, launch_finish(c->partial, c->grid_full, c->conv, nullptr, 0, st));
    }
    rc = loopback_exchange(cs, n, (h + 1) & 1, false, st);
    if (rc) return rc;
    hipLaunchKernelGGL(k_sum_locals, dim3(1), dim3(1), 0, st, dconvs, n);
    for (int i = 0; i < n; ++i)
      HIPCK(c0, launch_finish_global(cs[i]->conv, (i == 0 && residual_hist) ? c0->hist + s : nullptr, st));
  }
  HIPCK(c0, hipStreamSynchronize(st));
  for (int i = 0; i < n; ++i) cs[i]->steps_done += nsteps;
  if (residual_hist && nsteps > 0)
    HIPCK(c0, hipMemcpy(residual_hist, c0->hist, sizeof(float) * nsteps, hipMemcpyDeviceToHost));
  HIPCK(c0, hipFree(dconvs));
  return LBM_OK;
}
