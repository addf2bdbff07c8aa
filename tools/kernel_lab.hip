// kernel_lab.hip -- performance experiments for the collide-stream kernel (not product code).
// Builds a 512^3 (+ghost planes) SoA lattice and times kernel variants in one process with
// HIP events, interleaved rounds (cdna_hip_programming.md 5.4 rule 24).
//
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
//         -std=c++17 tools/kernel_lab.hip -o tools/kernel_lab && tools/kernel_lab [N]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../lattice-boltzmann-method-gpu_amd/csrc/lbm_d3q19.hpp"

using namespace lbm;

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

struct Geo {
  int nx, ny, nz, pitch;
  int64_t plane, qs;
};

template <int Q>
__device__ __forceinline__ int off(const Geo& g) {
  return Dir<Q>::x + Dir<Q>::y * g.pitch + Dir<Q>::z * (int)g.plane;
}

// ---- variant: pure streaming copy with the pull pattern --------------------------------
template <bool SHIFT>
__global__ __launch_bounds__(256) void k_copy(const float* __restrict__ src, float* __restrict__ dst, Geo g,
                                              int ntx, int nty, int ntiles) {
  const int lane = threadIdx.x & 63, row = threadIdx.x >> 6;
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int x = (t % ntx) * 64 + lane;
    const int r = t / ntx;
    const int y = (r % nty) * 4 + row;
    const int z = 2 + r / nty;
    const int c = x + y * g.pitch + z * (int)g.plane;
    if (x < 1 || x >= g.nx - 1 || y < 1 || y >= g.ny - 1) continue;
    float v[19];
#define L(Q) v[Q] = src[Q * g.qs + c - (SHIFT ? off<Q>(g) : 0)];
    L(0) L(1) L(2) L(3) L(4) L(5) L(6) L(7) L(8) L(9) L(10) L(11) L(12) L(13) L(14) L(15) L(16) L(17) L(18)
#undef L
#pragma unroll
    for (int q = 0; q < 19; ++q) dst[q * g.qs + c] = v[q];
  }
}

// ---- variant: collide (fast path of the product kernel) --------------------------------
template <int MODE>  // 0 exact IEEE division, 1 multiply by reciprocal (inexact, timing only)
__device__ __forceinline__ float dv(float a, float b, float rb) {
  if constexpr (MODE == 0) return a / b;
  else return a * rb;
}

template <int MODE, int NT>
__global__ __launch_bounds__(256) void k_collide(const float* __restrict__ src, float* __restrict__ dst, Geo g,
                                                 int ntx, int nty, int ntiles, float tau, double* part) {
  const int lane = threadIdx.x & 63, row = threadIdx.x >> 6;
  double acc = 0.0;
  const float rtau = 1.0f / tau;
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int x = (t % ntx) * 64 + lane;
    const int r = t / ntx;
    const int y = (r % nty) * 4 + row;
    const int z = 2 + r / nty;
    const int c = x + y * g.pitch + z * (int)g.plane;
    if (x < 1 || x >= g.nx - 1 || y < 1 || y >= g.ny - 1) continue;
    float v[19];
#define L(Q) v[Q] = NT ? __builtin_nontemporal_load(&src[Q * g.qs + c - off<Q>(g)]) : src[Q * g.qs + c - off<Q>(g)];
    L(0) L(1) L(2) L(3) L(4) L(5) L(6) L(7) L(8) L(9) L(10) L(11) L(12) L(13) L(14) L(15) L(16) L(17) L(18)
#undef L
    float rho = 0.f;
#pragma unroll
    for (int q = 0; q < 19; ++q) rho = rho + v[q];
    const float rr = 1.0f / rho;
    const float ux = dv<MODE>(v[1] - v[2] + v[7] + v[8] - v[9] - v[10] + v[11] + v[12] - v[13] - v[14], rho, rr);
    const float uy = dv<MODE>(v[3] - v[4] + v[7] - v[8] + v[9] - v[10] + v[15] - v[16] + v[17] - v[18], rho, rr);
    const float uz = dv<MODE>(v[5] - v[6] + v[11] - v[12] + v[13] - v[14] + v[15] + v[16] - v[17] - v[18], rho, rr);
    float e[19];
    feq_expanded(rho, ux, uy, uz, e);
#pragma unroll
    for (int q = 0; q < 19; ++q) {
      const float o = v[q] - dv<MODE>(v[q] - e[q], tau, rtau);
      if (NT) __builtin_nontemporal_store(o, &dst[q * g.qs + c]);
      else dst[q * g.qs + c] = o;
    }
    acc += (double)sqrtf(ux * ux + uy * uy + uz * uz);
  }
  // keep the reduction alive
  if (acc == -1.0) part[blockIdx.x] = acc;
}


// ---- 4 cells per lane (16-B accesses), 1-D linear chunks of 256 cells per wave ---------
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));

__device__ __forceinline__ float shr1(float v) {  // lane i <- lane i-1
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ float shl1(float v) {  // lane i <- lane i+1
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x130, 0xf, 0xf, false));
}

// pull of population Q for 4 consecutive cells c..c+3 (c = 4*lane + chunk base)
template <int Q, int SHIFTMODE>
__device__ __forceinline__ f4 pull4(const float* __restrict__ src, int64_t qs, int c, int lane, const Geo& g) {
  const float* s = src + Q * qs;
  const int rowoff = Dir<Q>::y * g.pitch + Dir<Q>::z * (int)g.plane;
  if constexpr (Dir<Q>::x == 0) {
    return *(const f4*)(s + c - rowoff);
  } else if constexpr (SHIFTMODE == 0) {  // unaligned 16-B load
    return *(const f4u*)(s + c - rowoff - Dir<Q>::x);
  } else {  // aligned load + DPP lane shift + edge lane extra load
    const f4 a = *(const f4*)(s + c - rowoff);
    if constexpr (Dir<Q>::x == 1) {  // needs c-1 .. c+2
      float p = shr1(a.w);
      if (lane == 0) p = s[c - rowoff - 1];
      return (f4){p, a.x, a.y, a.z};
    } else {                          // needs c+1 .. c+4
      float n = shl1(a.x);
      if (lane == 63) n = s[c - rowoff + 4];
      return (f4){a.y, a.z, a.w, n};
    }
  }
}

template <int SHIFTMODE, bool COLLIDE, int NT, int WPB = 4>
__global__ __launch_bounds__(WPB * 64) void k_v4(const float* __restrict__ src, float* __restrict__ dst,
                                            const uint8_t* __restrict__ type, Geo g, int64_t c_begin, int nchunks,
                                            float tau, double* part) {
  const int lane = threadIdx.x & 63;
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = gridDim.x * WPB;
  double acc = 0.0;
  for (int ch = blockIdx.x * WPB + wib; ch < nchunks; ch += nw) {
    const int c = (int)(c_begin + (int64_t)ch * 256) + lane * 4;
    f4 v[19];
#define P(Q) v[Q] = pull4<Q, SHIFTMODE>(src, g.qs, c, lane, g);
    P(0) P(1) P(2) P(3) P(4) P(5) P(6) P(7) P(8) P(9) P(10) P(11) P(12) P(13) P(14) P(15) P(16) P(17) P(18)
#undef P
    const unsigned t4 = *(const unsigned*)(type + c);
    if constexpr (COLLIDE) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float rho = 0.f;
#pragma unroll
        for (int q = 0; q < 19; ++q) rho = rho + v[q][j];
        const float ux = (v[1][j] - v[2][j] + v[7][j] + v[8][j] - v[9][j] - v[10][j] + v[11][j] + v[12][j] - v[13][j] - v[14][j]) / rho;
        const float uy = (v[3][j] - v[4][j] + v[7][j] - v[8][j] + v[9][j] - v[10][j] + v[15][j] - v[16][j] + v[17][j] - v[18][j]) / rho;
        const float uz = (v[5][j] - v[6][j] + v[11][j] - v[12][j] + v[13][j] - v[14][j] + v[15][j] + v[16][j] - v[17][j] - v[18][j]) / rho;
        float e[19];
        feq_expanded(rho, ux, uy, uz, e);
#pragma unroll
        for (int q = 0; q < 19; ++q) v[q][j] = v[q][j] - (v[q][j] - e[q]) / tau;
        if (((t4 >> (8 * j)) & 0xff) == 3) acc += (double)sqrtf(ux * ux + uy * uy + uz * uz);
      }
    }
    if (t4 == 0x03030303u) {
#pragma unroll
      for (int q = 0; q < 19; ++q) {
        if (NT) __builtin_nontemporal_store(v[q], (f4*)(dst + q * g.qs + c));
        else *(f4*)(dst + q * g.qs + c) = v[q];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (((t4 >> (8 * j)) & 0xff) == 3)
#pragma unroll
          for (int q = 0; q < 19; ++q) dst[q * g.qs + c + j] = v[q][j];
    }
  }
  if (acc == -1.0) part[blockIdx.x] = acc;
}

__global__ void k_type(uint8_t* t, Geo g) {
  const int64_t n = g.qs;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < n; c += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(c % g.pitch), y = (int)((c / g.pitch) % g.ny), z = (int)(c / g.plane);
    t[c] = (x >= 2 && x < g.nx - 2 && y >= 2 && y < g.ny - 2 && z >= 3 && z < g.nz - 1) ? 3 : 0;
  }
}


// 1 stream in, 1 out, float4 (calibration)
__global__ __launch_bounds__(256) void k_copy1(const f4* __restrict__ a, f4* __restrict__ b, int64_t n4) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(a[i], &b[i]);
}
// 19 streams in/out, AoSoA [chunk][q][256] layout, aligned
template <int WPB>
__global__ __launch_bounds__(WPB * 64) void k_copy_aosoa(const float* __restrict__ a, float* __restrict__ b, int nchunks) {
  const int lane = threadIdx.x & 63;
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int ch = blockIdx.x * WPB + wib; ch < nchunks; ch += gridDim.x * WPB) {
    const float* s = a + (int64_t)ch * 19 * 256 + lane * 4;
    float* d = b + (int64_t)ch * 19 * 256 + lane * 4;
    f4 v[19];
#pragma unroll
    for (int q = 0; q < 19; ++q) v[q] = *(const f4*)(s + q * 256);
#pragma unroll
    for (int q = 0; q < 19; ++q) __builtin_nontemporal_store(v[q], (f4*)(d + q * 256));
  }
}


// ---- AoSoA layout: [chunk][q][256], chunk = 256 consecutive linear cells ----------------
__device__ __forceinline__ int64_t aaddr(int64_t c, int q) { return ((c >> 8) * 19 + q) * 256 + (c & 255); }

template <int Q, int NTL>
__device__ __forceinline__ f4 apull4(const float* __restrict__ src, int64_t c, int lane, const Geo& g) {
  const int64_t b = c - (Dir<Q>::y * g.pitch + Dir<Q>::z * g.plane);
  const f4 a = NTL ? __builtin_nontemporal_load((const f4*)(src + aaddr(b, Q))) : *(const f4*)(src + aaddr(b, Q));
  if constexpr (Dir<Q>::x == 0) {
    return a;
  } else if constexpr (Dir<Q>::x == 1) {
    float p = shr1(a.w);
    if (lane == 0) p = src[aaddr(b - 1, Q)];
    return (f4){p, a.x, a.y, a.z};
  } else {
    float n = shl1(a.x);
    if (lane == 63) n = src[aaddr(b + 4, Q)];
    return (f4){a.y, a.z, a.w, n};
  }
}

template <int NTL, int NTS, int WPB, int MINW = 1>
__global__ __launch_bounds__(WPB * 64, MINW) void k_aos(const float* __restrict__ src, float* __restrict__ dst,
                                                  const uint8_t* __restrict__ type, Geo g, int64_t c_begin, int nchunks,
                                                  float tau, double* part) {
  const int lane = threadIdx.x & 63;
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  double acc = 0.0;
  for (int ch = blockIdx.x * WPB + wib; ch < nchunks; ch += gridDim.x * WPB) {
    const int64_t c = c_begin + (int64_t)ch * 256 + lane * 4;
    f4 v[19];
#define P(Q) v[Q] = apull4<Q, NTL>(src, c, lane, g);
    P(0) P(1) P(2) P(3) P(4) P(5) P(6) P(7) P(8) P(9) P(10) P(11) P(12) P(13) P(14) P(15) P(16) P(17) P(18)
#undef P
    const unsigned t4 = *(const unsigned*)(type + c);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float rho = 0.f;
#pragma unroll
      for (int q = 0; q < 19; ++q) rho = rho + v[q][j];
      const float ux = (v[1][j] - v[2][j] + v[7][j] + v[8][j] - v[9][j] - v[10][j] + v[11][j] + v[12][j] - v[13][j] - v[14][j]) / rho;
      const float uy = (v[3][j] - v[4][j] + v[7][j] - v[8][j] + v[9][j] - v[10][j] + v[15][j] - v[16][j] + v[17][j] - v[18][j]) / rho;
      const float uz = (v[5][j] - v[6][j] + v[11][j] - v[12][j] + v[13][j] - v[14][j] + v[15][j] + v[16][j] - v[17][j] - v[18][j]) / rho;
      float e[19];
      feq_expanded(rho, ux, uy, uz, e);
#pragma unroll
      for (int q = 0; q < 19; ++q) v[q][j] = v[q][j] - (v[q][j] - e[q]) / tau;
      if (((t4 >> (8 * j)) & 0xff) == 3) acc += (double)sqrtf(ux * ux + uy * uy + uz * uz);
    }
    float* d = dst + aaddr(c, 0);
    if (t4 == 0x03030303u) {
#pragma unroll
      for (int q = 0; q < 19; ++q) {
        if (NTS) __builtin_nontemporal_store(v[q], (f4*)(d + q * 256));
        else *(f4*)(d + q * 256) = v[q];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (((t4 >> (8 * j)) & 0xff) == 3)
#pragma unroll
          for (int q = 0; q < 19; ++q) d[q * 256 + j] = v[q][j];
    }
  }
  if (acc == -1.0) part[blockIdx.x] = acc;
}

__global__ void k_fill(float* a, int64_t n, float v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    a[i] = v;
}

int main(int argc, char** argv) {
  const int N = argc > 1 ? std::atoi(argv[1]) : 512;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 5;
  Geo g{};
  g.nx = N; g.ny = N; g.nz = N;
  g.pitch = (N + 63) / 64 * 64;
  g.plane = (int64_t)g.pitch * N;
  g.qs = g.plane * (N + 2);
  float *a, *b;
  double* part;
  CK(hipMalloc(&a, sizeof(float) * 19 * g.qs));
  CK(hipMalloc(&b, sizeof(float) * 19 * g.qs));
  CK(hipMalloc(&part, sizeof(double) * 65536));
  hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, a, 19 * g.qs, 1.0f / 19.0f);
  hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, b, 19 * g.qs, 1.0f / 19.0f);
  CK(hipDeviceSynchronize());
  const int ntx = g.pitch / 64, nty = N / 4, ntiles = ntx * nty * (N - 4);
  const double cells = (double)(N - 2) * (N - 2) * (N - 4);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct V {
    const char* name;
    int grid;
    int kind;
  };
  std::vector<V> vs = {
      {"copy_aligned g2048", 2048, 0}, {"copy_pull g2048", 2048, 1},      {"copy_pull g1024", 1024, 1},
      {"copy_pull g8192", 8192, 1},   {"collide_exact g2048", 2048, 2},  {"collide_fastdiv g2048", 2048, 3},
      {"collide_exact_nt g2048", 2048, 4}, {"collide_exact g8192", 8192, 2}, {"collide_exact g1024", 1024, 2},
  };
  vs.clear();
  vs.push_back({"copy1_f4_nt (1 in/1 out)", 8192, 20});
  vs.push_back({"copy19_aosoa_f4_nt w4", 2048, 21});
  vs.push_back({"copy19_aosoa_f4_nt w16", 512, 22});
  vs.push_back({"collide_exact_nt g2048", 2048, 4});
  vs.push_back({"v4_collide_dpp_nt w4 g2048", 2048, 14});
  vs.push_back({"aos_collide nts w4 g2048", 2048, 30});
  vs.push_back({"aos_collide nts w4 g4096", 4096, 30});
  vs.push_back({"aos_collide nts w4 g8192", 8192, 30});
  vs.push_back({"aos_collide nts w4 g131072", 131072, 30});
  vs.push_back({"aos nts lb4 g4096", 4096, 33});
  vs.push_back({"aos nts lb4 g8192", 8192, 33});
  vs.push_back({"aos ntl+nts g4096", 4096, 34});
  vs.push_back({"aos ntl+nts lb4 g4096", 4096, 35});

  uint8_t* type;
  CK(hipMalloc(&type, g.qs + 1024));
  hipLaunchKernelGGL(k_type, dim3(8192), dim3(256), 0, 0, type, g);
  const int64_t cb = 2 * g.plane;
  const int nch = (int)((g.plane * (N - 4)) / 256);
  std::vector<std::vector<float>> ms(vs.size());
  for (int r = 0; r < rounds; ++r) {
    for (size_t i = 0; i < vs.size(); ++i) {
      const V& v = vs[i];
      CK(hipEventRecord(e0));
      for (int it = 0; it < 4; ++it) {
        switch (v.kind) {
          case 0: hipLaunchKernelGGL(k_copy<false>, dim3(v.grid), dim3(256), 0, 0, a, b, g, ntx, nty, ntiles); break;
          case 1: hipLaunchKernelGGL(k_copy<true>, dim3(v.grid), dim3(256), 0, 0, a, b, g, ntx, nty, ntiles); break;
          case 2: hipLaunchKernelGGL((k_collide<0, 0>), dim3(v.grid), dim3(256), 0, 0, a, b, g, ntx, nty, ntiles, 0.55f, part); break;
          case 3: hipLaunchKernelGGL((k_collide<1, 0>), dim3(v.grid), dim3(256), 0, 0, a, b, g, ntx, nty, ntiles, 0.55f, part); break;
          case 4: hipLaunchKernelGGL((k_collide<0, 1>), dim3(v.grid), dim3(256), 0, 0, a, b, g, ntx, nty, ntiles, 0.55f, part); break;
          case 10: hipLaunchKernelGGL((k_v4<0, false, 0>), dim3(v.grid), dim3(256), 0, 0, a, b, type, g, cb, nch, 0.55f, part); break;
          case 11: hipLaunchKernelGGL((k_v4<1, false, 0>), dim3(v.grid), dim3(256), 0, 0, a, b, type, g, cb, nch, 0.55f, part); break;
          case 12: hipLaunchKernelGGL((k_v4<0, true, 0>), dim3(v.grid), dim3(256), 0, 0, a, b, type, g, cb, nch, 0.55f, part); break;
          case 13: hipLaunchKernelGGL((k_v4<1, true, 0>), dim3(v.grid), dim3(256), 0, 0, a, b, type, g, cb, nch, 0.55f, part); break;
          case 14: hipLaunchKernelGGL((k_v4<1, true, 1>), dim3(v.grid), dim3(256), 0, 0, a, b, type, g, cb, nch, 0.55f, part); break;
          case 15: hipLaunchKernelGGL((k_v4<1, true, 1, 16>), dim3(v.grid), dim3(1024), 0, 0, a, b, type, g, cb, nch, 0.55f, part); break;
          case 16: hipLaunchKernelGGL((k_v4<1, true, 1, 8>), dim3(v.grid), dim3(512), 0, 0, a, b, type, g, cb, nch, 0.55f, part); break;
          case 17: hipLaunchKernelGGL((k_v4<1, true, 1, 16>), dim3(v.grid), dim3(1024), 0, 0, a, b, type, g, cb, nch, 0.55f, part); break;
          case 30: hipLaunchKernelGGL((k_aos<0, 1, 4>), dim3(v.grid), dim3(256), 0, 0, a, b, type, g, cb, nch, 0.55f, part); break;
          case 31: hipLaunchKernelGGL((k_aos<0, 0, 4>), dim3(v.grid), dim3(256), 0, 0, a, b, type, g, cb, nch, 0.55f, part); break;
          case 32: hipLaunchKernelGGL((k_aos<0, 1, 8>), dim3(v.grid), dim3(512), 0, 0, a, b, type, g, cb, nch, 0.55f, part); break;
          case 33: hipLaunchKernelGGL((k_aos<0, 1, 4, 4>), dim3(v.grid), dim3(256), 0, 0, a, b, type, g, cb, nch, 0.55f, part); break;
          case 34: hipLaunchKernelGGL((k_aos<1, 1, 4, 1>), dim3(v.grid), dim3(256), 0, 0, a, b, type, g, cb, nch, 0.55f, part); break;
          case 35: hipLaunchKernelGGL((k_aos<1, 1, 4, 4>), dim3(v.grid), dim3(256), 0, 0, a, b, type, g, cb, nch, 0.55f, part); break;
          case 20: hipLaunchKernelGGL(k_copy1, dim3(v.grid), dim3(256), 0, 0, (const f4*)a, (f4*)b, (int64_t)19 * g.plane * (N - 4) / 4); break;
          case 21: hipLaunchKernelGGL(k_copy_aosoa<4>, dim3(v.grid), dim3(256), 0, 0, a, b, nch); break;
          case 22: hipLaunchKernelGGL(k_copy_aosoa<16>, dim3(v.grid), dim3(1024), 0, 0, a, b, nch); break;
        }
        std::swap(a, b);
      }
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float t = 0;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms[i].push_back(t / 4);
    }
  }
  for (size_t i = 0; i < vs.size(); ++i) {
    std::sort(ms[i].begin(), ms[i].end());
    const float med = ms[i][ms[i].size() / 2];
    std::printf("%-26s median %8.3f ms  %9.1f MLUPS  %7.1f GB/s (152 B/cell)\n", vs[i].name, med,
                cells / (med * 1e-3) / 1e6, 152.0 * cells / (med * 1e-3) / 1e9);
  }
  return 0;
}
