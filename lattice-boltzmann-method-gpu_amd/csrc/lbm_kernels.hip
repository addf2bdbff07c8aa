// lbm_kernels.hip -- CDNA4 (gfx950) kernels of the D3Q19 BGK hot path.
//
// One fused kernel replaces the reference's update + boundary_stream + calc_vel_square
// (ldc.cu:57-466, Poiseulle.cu:384-901, bifurcation.cu:429-1023):
//   * pull streaming from the SoA source buffer (19 coalesced 256-B wavefront loads);
//   * boundaries are evaluated on the CONSUMER side, selected by the neighbour's type
//     byte: a fluid cell F that would pull population q from
//       - a wall W: takes src[opp q][F] (half-way bounce-back, ldc.cu:184-201 /
//         Poiseulle.cu:601-746 write exactly this value into W one pass earlier);
//       - an NEE cell B with e_q . n_B = 1: takes
//           feq_q(rho_bc, u_bc) + (src[q][F] - feq_q(rho_F, u_F)) * (1 - 1/tau)
//         with F's own (rho,u) of the previous step -- the value boundary_stream
//         writes into B (ldc.cu:391-456, Poiseulle.cu:748-891, bifurcation.cu:877-1021;
//         their hand-simplified "tmp" terms are bit-identical to feq_q(rho_bc, u_bc));
//     so no boundary pass, no boundary-cell writes and no second launch are needed;
//   * moments, BGK relaxation and the |u| partial sum of the residual in registers.
// HBM traffic per fluid cell: 76 B loaded + 76 B stored + 1 B type (+16 B macros on the
// last step of a call and for cells next to an NEE boundary).
#include "lbm_d3q19.hpp"
#include "lbm_kernels.hpp"

namespace lbm {

namespace {

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-wide deterministic sum of one double per thread; result valid in thread 0.
__device__ __forceinline__ double block_sum(double v, double* lds) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) lds[wid] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0)
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += lds[w];
  return s;
}

struct Pop {
  float v[19];
};

// Raw pull of population Q from c - e_Q.
template <int Q>
__device__ __forceinline__ void pull(Pop& f, const float* __restrict__ src, int64_t qs, int c,
                                     int pitch, int64_t plane) {
  const int off = Dir<Q>::x + Dir<Q>::y * pitch + Dir<Q>::z * (int)plane;
  f.v[Q] = src[Q * qs + (c - off)];
}

template <int... Qs>
__device__ __forceinline__ void pull_all(Pop& f, const float* __restrict__ src, int64_t qs, int c,
                                         int pitch, int64_t plane, std::integer_sequence<int, Qs...>) {
  (pull<Qs>(f, src, qs, c, pitch, plane), ...);
}

struct Macro {
  float rho, ux, uy, uz;
};

// Boundary patch of population Q for a slow-path cell (neighbour is a wall or NEE cell).
template <int Q>
__device__ __forceinline__ void patch(Pop& f, const StepArgs& a, int c, const Macro& mp) {
  const int off = Dir<Q>::x + Dir<Q>::y * a.pitch + Dir<Q>::z * (int)a.plane;
  const int nb = c - off;
  const uint8_t tn = a.type[nb];
  const int cls = tn & kClassMask;
  if (cls == kWall) {
    if (a.bb_active) f.v[Q] = a.src[Dir<Q>::opp * a.qstride + c];
  } else if (cls == kNee) {
    if (a.nee_active && ((face_bits<Q>() >> nee_face(tn)) & 1)) {
      float rb, bx, by, bz;
      if (tn & kKindPressure) {  // rho_bc stored at B; u_bc = u of the fluid neighbour
        rb = a.rho[nb];
        bx = mp.ux; by = mp.uy; bz = mp.uz;
      } else {                   // u_bc stored at B; rho_bc = rho of the fluid neighbour
        rb = mp.rho;
        bx = a.ux[nb]; by = a.uy[nb]; bz = a.uz[nb];
      }
      const float own = a.src[Q * a.qstride + c];
      const float e_bc = feq<Q>(rb, bx, by, bz);
      const float e_nb = feq<Q>(mp.rho, mp.ux, mp.uy, mp.uz);
      f.v[Q] = e_bc + (own - e_nb) * a.omc;
    }
  }
}

template <int... Qs>
__device__ __forceinline__ void patch_all(Pop& f, const StepArgs& a, int c, const Macro& mp,
                                          std::integer_sequence<int, Qs...>) {
  (patch<Qs>(f, a, c, mp), ...);
}

template <int Q>
__device__ __forceinline__ void relax_store(const Pop& f, float* __restrict__ dst, int64_t qs, int c,
                                            float tau, float r, float ux, float uy, float uz) {
  const float e = feq<Q>(r, ux, uy, uz);
  dst[Q * qs + c] = f.v[Q] - (f.v[Q] - e) / tau;
}

template <int... Qs>
__device__ __forceinline__ void relax_all(const Pop& f, float* __restrict__ dst, int64_t qs, int c,
                                          float tau, float r, float ux, float uy, float uz,
                                          std::integer_sequence<int, Qs...>) {
  (relax_store<Qs>(f, dst, qs, c, tau, r, ux, uy, uz), ...);
}

using AllQ = std::make_integer_sequence<int, 19>;

__global__ __launch_bounds__(kBlock) void k_collide_stream(const StepArgs a) {
  __shared__ double red[kBlock / 64];
  if (a.stopped != nullptr && *a.stopped) return;  // uniform: converged, step is a no-op
  const int lane = threadIdx.x & 63;
  const int row = threadIdx.x >> 6;
  double acc = 0.0;
  for (int t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
    const int txi = t % a.ntx;
    const int r = t / a.ntx;
    const int tyi = r % a.nty;
    const int z = a.z_begin + r / a.nty;
    const int x = txi * kTileX + lane;
    const int y = tyi * kTileY + row;
    if (y >= a.ny) continue;
    const int c = x + y * a.pitch + z * (int)a.plane;
    const uint8_t tc = a.type[c];
    if ((tc & kClassMask) != kFluid) continue;

    Pop f;
    pull_all(f, a.src, a.qstride, c, a.pitch, a.plane, AllQ{});
    if (tc & kSlow) {
      Macro mp{0.f, 0.f, 0.f, 0.f};
      if (tc & kNeedsMac) mp = Macro{a.rho[c], a.ux[c], a.uy[c], a.uz[c]};
      patch_all(f, a, c, mp, AllQ{});
    }
    // moments (ldc.cu:316-322): sequential fp32 sum, signed sums in reference order
    float rho = 0.f;
#pragma unroll
    for (int q = 0; q < 19; ++q) rho = rho + f.v[q];
    const float* v = f.v;
    const float ux = (v[1] - v[2] + v[7] + v[8] - v[9] - v[10] + v[11] + v[12] - v[13] - v[14]) / rho;
    const float uy = (v[3] - v[4] + v[7] - v[8] + v[9] - v[10] + v[15] - v[16] + v[17] - v[18]) / rho;
    const float uz = (v[5] - v[6] + v[11] - v[12] + v[13] - v[14] + v[15] + v[16] - v[17] - v[18]) / rho;
    if (a.store_all_macros || (tc & kNeedsMac)) {
      a.rho[c] = rho; a.ux[c] = ux; a.uy[c] = uy; a.uz[c] = uz;
    }
    relax_all(f, a.dst, a.qstride, c, a.tau, rho, ux, uy, uz, AllQ{});
    acc += (double)sqrtf(ux * ux + uy * uy + uz * uz);
  }
  const double s = block_sum(acc, red);
  if (threadIdx.x == 0) a.partial[blockIdx.x] = s;
}

__device__ void residual_logic(ConvState* cv, double S, float* hist_slot) {
  // ldc.cu:662-684: residual = |S_k - S_{k-1}| / S_k on fp32 sums
  const float sum_next = (float)S;
  const float residual = fabsf(sum_next - cv->sum_current) / sum_next;
  cv->residual = residual;
  cv->sum_current = sum_next;
  cv->k += 1;
  if (residual <= cv->tol) cv->tol_count += 1;
  if (cv->enabled) cv->stopped = !(cv->k <= cv->max_it && cv->tol_count <= cv->stag_max);
  if (hist_slot) *hist_slot = residual;
}

__global__ __launch_bounds__(256) void k_finish(const double* __restrict__ partial, int n,
                                                ConvState* cv, float* hist_slot, int finish) {
  __shared__ double red[4];
  if (cv->stopped) return;
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += partial[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) {
    cv->s_local = s;
    if (finish) residual_logic(cv, s, hist_slot);
  }
}

__global__ void k_finish_global(ConvState* cv, float* hist_slot) {
  if (cv->stopped) return;
  residual_logic(cv, cv->s_global, hist_slot);
}

// ---- geometry --------------------------------------------------------------------------

// reference code -> class/face/kind, NEE data into the macro arrays of NEE cells
__global__ void k_classify(const GeoArgs g) {
  const int64_t n = g.plane * g.planes;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < n;
       c += (int64_t)gridDim.x * blockDim.x) {
    const int code = g.codes[c];
    const int x = (int)(c % g.pitch);
    const int zs = (int)(c / g.plane);
    const int zg = zs - 1 + g.z_offset;  // global z
    uint8_t t = kPassive;
    if (x < g.nx) {
      if (g.case_kind == 0) {  // LDC (ldc.cu:469): 0 ghost, 1 wall, 2 lid, 3 fluid
        if (code == 1) t = kWall;
        else if (code == 3) t = kFluid;
        else if (code == 2) {
          t = make_nee(kFaceNY, false);  // lid supplies {4,8,10,16,18} (ldc.cu:391-456)
          g.rho[c] = 0.f; g.ux[c] = 0.f; g.uy[c] = 0.f; g.uz[c] = g.lid_u;
        }
      } else {  // Poiseuille / mask (README.md:9-14)
        if (code == 1) t = kWall;
        else if (code == 4) t = kFluid;
        else if (code == 2) {   // inlet, +y face {3,7,9,15,17}, u = (0, inlet_uy(x,z), 0)
          t = make_nee(kFacePY, false);
          const bool in_tab = g.inlet_uy && zg >= 0 && zg < g.nz_global;
          const float u = in_tab ? g.inlet_uy[x + (int64_t)zg * g.nx] : 0.f;
          g.rho[c] = 0.f; g.ux[c] = 0.f; g.uy[c] = u; g.uz[c] = 0.f;
        } else if (code == 3) { // outlet, -y face {4,8,10,16,18}
          if (g.case_kind == 1) {  // Poiseuille: velocity, u = (0, outlet_uy(x,z), 0)
            t = make_nee(kFaceNY, false);
            const bool in_tab = g.outlet_uy && zg >= 0 && zg < g.nz_global;
            const float u = in_tab ? g.outlet_uy[x + (int64_t)zg * g.nx] : 0.f;
            g.rho[c] = 0.f; g.ux[c] = 0.f; g.uy[c] = u; g.uz[c] = 0.f;
          } else {                 // bifurcation: pressure, rho = 1 (bifurcation.cu:890)
            t = make_nee(kFaceNY, true);
            g.rho[c] = 1.0f; g.ux[c] = 0.f; g.uy[c] = 0.f; g.uz[c] = 0.f;
          }
        }
      }
    }
    g.type[c] = t;
  }
}

template <int Q>
__device__ __forceinline__ void scan_nb(const uint8_t* type, int64_t c, int pitch, int64_t plane,
                                        int64_t n, uint8_t& flags) {
  const int64_t nb = c - (Dir<Q>::x + Dir<Q>::y * (int64_t)pitch + Dir<Q>::z * plane);
  if (nb < 0 || nb >= n) return;
  const uint8_t tn = type[nb];
  const int cls = tn & kClassMask;
  if (cls == kWall) flags |= kSlow;
  if (cls == kNee && ((face_bits<Q>() >> nee_face(tn)) & 1)) flags |= kSlow | kNeedsMac;
}

template <int... Qs>
__device__ __forceinline__ void scan_all(const uint8_t* type, int64_t c, int pitch, int64_t plane,
                                         int64_t n, uint8_t& flags, std::integer_sequence<int, Qs...>) {
  (scan_nb<Qs>(type, c, pitch, plane, n, flags), ...);
}

__global__ void k_flag_fluid(const GeoArgs g) {
  const int64_t n = g.plane * g.planes;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < n;
       c += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t t = g.type[c];
    if ((t & kClassMask) != kFluid) continue;
    uint8_t flags = 0;
    scan_all(g.type, c, g.pitch, g.plane, n, flags, AllQ{});
    g.type[c] = (uint8_t)(t | flags);
  }
}

__global__ void k_ldc_codes(int8_t* codes, int nx, int ny, int pitch, int planes, int64_t plane,
                            int z_offset, int nzg) {
  const int64_t n = plane * planes;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < n;
       c += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(c % pitch);
    const int y = (int)((c / pitch) % ny);
    const int z = (int)(c / plane) - 1 + z_offset;
    int8_t code = 0;  // ldc.cu:468-502
    if (x < nx && z >= 0 && z < nzg) {
      if (x >= 1 && x < nx - 1 && y >= 1 && y < ny - 1 && z >= 1 && z < nzg - 1) code = 1;
      if (x >= 2 && x < nx - 2 && y >= 2 && y < ny - 2 && z >= 2 && z < nzg - 2) code = 3;
      if (y == ny - 2 && x >= 1 && x < nx - 1 && z >= 1 && z < nzg - 1) code = 2;
    }
    codes[c] = code;
  }
}

// ---- initial state ---------------------------------------------------------------------

__global__ void k_init_feq(float* fa, float* fb, int64_t qs, int64_t n, int form,
                           const float* rho, const float* ux, const float* uy, const float* uz) {
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < n;
       c += (int64_t)gridDim.x * blockDim.x) {
    const float r = rho ? rho[c] : 1.0f;
    const float vx = ux ? ux[c] : 0.0f, vy = uy ? uy[c] : 0.0f, vz = uz ? uz[c] : 0.0f;
    float e[19];
    if (form == 0) feq_init_wi(r, vx, vy, vz, e);
    else feq_expanded(r, vx, vy, vz, e);
#pragma unroll
    for (int q = 0; q < 19; ++q) { fa[q * qs + c] = e[q]; fb[q * qs + c] = e[q]; }
  }
}

__global__ void k_init_ldc(float* fa, float* fb, int64_t qs, int nx, int ny, int pitch, int planes,
                           int64_t plane, int z_offset, float lid_u) {
  const int64_t n = plane * planes;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < n;
       c += (int64_t)gridDim.x * blockDim.x) {
    const int y = (int)((c / pitch) % ny);
    (void)nx; (void)z_offset;
    // ldc.cu:510-532: rho 1, u 0; uz = u_max on y = ny-1 and y = ny-2
    const float uz = (y == ny - 1 || y == ny - 2) ? lid_u : 0.0f;
    float e[19];
    feq_init_wi(1.0f, 0.0f, 0.0f, uz, e);
#pragma unroll
    for (int q = 0; q < 19; ++q) { fa[q * qs + c] = e[q]; fb[q * qs + c] = e[q]; }
  }
}

int grid_for(int64_t n, int block) {
  int64_t g = (n + block - 1) / block;
  if (g > 65536) g = 65536;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

hipError_t launch_collide_stream(const StepArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL(k_collide_stream, dim3(grid), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_finish(const double* partial, int n, ConvState* conv, float* hist_slot, int finish,
                         hipStream_t s) {
  hipLaunchKernelGGL(k_finish, dim3(1), dim3(256), 0, s, partial, n, conv, hist_slot, finish);
  return hipGetLastError();
}

hipError_t launch_finish_global(ConvState* conv, float* hist_slot, hipStream_t s) {
  hipLaunchKernelGGL(k_finish_global, dim3(1), dim3(1), 0, s, conv, hist_slot);
  return hipGetLastError();
}

hipError_t launch_classify(const GeoArgs& g, hipStream_t s) {
  hipLaunchKernelGGL(k_classify, dim3(grid_for(g.plane * g.planes, 256)), dim3(256), 0, s, g);
  return hipGetLastError();
}

hipError_t launch_flag_fluid(const GeoArgs& g, hipStream_t s) {
  hipLaunchKernelGGL(k_flag_fluid, dim3(grid_for(g.plane * g.planes, 256)), dim3(256), 0, s, g);
  return hipGetLastError();
}

hipError_t launch_ldc_codes(int8_t* codes, int nx, int ny, int pitch, int planes, int64_t plane,
                            int z_offset, int nz_global, hipStream_t s) {
  hipLaunchKernelGGL(k_ldc_codes, dim3(grid_for(plane * planes, 256)), dim3(256), 0, s, codes, nx, ny,
                     pitch, planes, plane, z_offset, nz_global);
  return hipGetLastError();
}

hipError_t launch_init_feq(float* fa, float* fb, int64_t qstride, int64_t n, int form, const float* rho,
                           const float* ux, const float* uy, const float* uz, hipStream_t s) {
  hipLaunchKernelGGL(k_init_feq, dim3(grid_for(n, 256)), dim3(256), 0, s, fa, fb, qstride, n, form, rho,
                     ux, uy, uz);
  return hipGetLastError();
}

hipError_t launch_init_ldc(float* fa, float* fb, int64_t qstride, int nx, int ny, int pitch, int planes,
                           int64_t plane, int z_offset, float lid_u, hipStream_t s) {
  hipLaunchKernelGGL(k_init_ldc, dim3(grid_for(plane * planes, 256)), dim3(256), 0, s, fa, fb, qstride,
                     nx, ny, pitch, planes, plane, z_offset, lid_u);
  return hipGetLastError();
}

}  // namespace lbm
