// lab_main.hip -- ablation bench of the production stream-collide kernel (tools only).
//
// Includes the product kernel source so every helper (pull4, collide_cell, bb_store_cell,
// block_sum) is the shipped one, and times copies of k_stream_collide with features
// switched off one at a time on a 512^3 LDC-like box (fluid 2..509, walls at 1 and 510).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off \
//     -fhip-fp32-correctly-rounded-divide-sqrt -o tools/lab_main tools/lab_main.hip
#ifndef LAB_KERNELS
#define LAB_KERNELS "../lattice-boltzmann-method-gpu_amd/csrc/lbm_kernels.hip"
#endif
#include LAB_KERNELS

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                            \
    }                                                                                          \
  } while (0)

using namespace lbm;

enum : int { F_LIST = 1, F_STOP = 2, F_BSUM = 4, F_UABS = 8, F_BB = 16, F_MASK = 32, F_ALL = 63, F_FASTDIV = 64, F_FULLSTORE = 128 };

// x / tau as RN(x * RN(1/tau)) refined by one FMA residual step (Markstein)
template <int J, int... Qs>
__device__ __forceinline__ void relax4_fast(f4* v, float tau, float y, float r, float ux, float uy, float uz,
                                            std::integer_sequence<int, Qs...>) {
  auto dv = [&](float x) {
    const float q0 = x * y;
    const float rr = __builtin_fmaf(-q0, tau, x);
    return __builtin_fmaf(rr, y, q0);
  };
  ((v[Qs][J] = v[Qs][J] - dv(v[Qs][J] - feq<Qs>(r, ux, uy, uz))), ...);
}
template <int J>
__device__ __forceinline__ void collide_cell_fast(f4* v, float tau, float y, float& rho, float& ux, float& uy,
                                                  float& uz) {
  float r = 0.f;
#pragma unroll
  for (int q = 0; q < kQ; ++q) r = r + v[q][J];
  ux = (v[1][J] - v[2][J] + v[7][J] + v[8][J] - v[9][J] - v[10][J] + v[11][J] + v[12][J] - v[13][J] - v[14][J]) / r;
  uy = (v[3][J] - v[4][J] + v[7][J] - v[8][J] + v[9][J] - v[10][J] + v[15][J] - v[16][J] + v[17][J] - v[18][J]) / r;
  uz = (v[5][J] - v[6][J] + v[11][J] - v[12][J] + v[13][J] - v[14][J] + v[15][J] + v[16][J] - v[17][J] - v[18][J]) / r;
  rho = r;
  relax4_fast<J>(v, tau, y, r, ux, uy, uz, AllQ{});
}

template <int F, int MINW = 1, int WPB = 4>
__global__ __launch_bounds__(WPB * 64, MINW) void k_var(const MainArgs a, int ch0) {
  __shared__ double red[WPB];
  if constexpr (F & F_STOP)
    if (a.stopped != nullptr && *a.stopped) return;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int idx = blockIdx.x * WPB + wave;
  double acc = 0.0;
  if (idx < a.nchunks) {
    const int64_t cb = (int64_t)((F & F_LIST) ? a.chunks[idx] : ch0 + idx) * kChunk;
    const int64_t c = cb + lane * 4;
    f4 v[kQ];
    pull4_all(v, a.src, cb, c, lane, a.pitch, a.plane, AllQ{});
    const unsigned t4 = *reinterpret_cast<const unsigned*>(a.type + c);
    constexpr unsigned kWall4 = kWallAdj * 0x01010101u;
    uint32_t m0 = 0, m1 = 0, m2 = 0, m3 = 0;
    if constexpr (F & F_BB) {
      if (t4 & kWall4) {
        if (t4 & (kWallAdj << 0)) m0 = a.links[c + 0];
        if (t4 & (kWallAdj << 8)) m1 = a.links[c + 1];
        if (t4 & (kWallAdj << 16)) m2 = a.links[c + 2];
        if (t4 & (kWallAdj << 24)) m3 = a.links[c + 3];
      }
    }
    float r0, r1, r2, r3, x0, x1, x2, x3, y0, y1, y2, y3, z0, z1, z2, z3;
    if constexpr (F & F_FASTDIV) {
      const float y = 1.0f / a.tau;
      collide_cell_fast<0>(v, a.tau, y, r0, x0, y0, z0);
      collide_cell_fast<1>(v, a.tau, y, r1, x1, y1, z1);
      collide_cell_fast<2>(v, a.tau, y, r2, x2, y2, z2);
      collide_cell_fast<3>(v, a.tau, y, r3, x3, y3, z3);
    } else {
      moments<0>(v, r0, x0, y0, z0);
      relax_cell<0, false>(v, a.tau, 0.f, r0, x0, y0, z0, AllQ{});
      moments<1>(v, r1, x1, y1, z1);
      relax_cell<1, false>(v, a.tau, 0.f, r1, x1, y1, z1, AllQ{});
      moments<2>(v, r2, x2, y2, z2);
      relax_cell<2, false>(v, a.tau, 0.f, r2, x2, y2, z2, AllQ{});
      moments<3>(v, r3, x3, y3, z3);
      relax_cell<3, false>(v, a.tau, 0.f, r3, x3, y3, z3, AllQ{});
    }
    const f4 R{r0, r1, r2, r3}, UX{x0, x1, x2, x3}, UY{y0, y1, y2, y3}, UZ{z0, z1, z2, z3};
    unsigned store = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const unsigned t = (t4 >> (8 * j)) & 0xffu;
      const int64_t cj = c + j;
      bool in;
      if constexpr (F & F_MASK) in = cj >= a.c_lo && cj < a.c_hi && (t & kClassMask) == kFluid;
      else in = (t & kClassMask) == kFluid;
      if (in) {
        store |= 1u << j;
        if constexpr (F & F_UABS)
          if (!(t & kNeedsMac)) acc += (double)sqrtf(UX[j] * UX[j] + UY[j] * UY[j] + UZ[j] * UZ[j]);
      }
    }
    if constexpr (F & F_BB) {
      if (t4 & kWall4) {
        if (store & 1u) bb_store_cell<0>(a.dst, c, m0, v, a.pitch, a.plane);
        if (store & 2u) bb_store_cell<1>(a.dst, c, m1, v, a.pitch, a.plane);
        if (store & 4u) bb_store_cell<2>(a.dst, c, m2, v, a.pitch, a.plane);
        if (store & 8u) bb_store_cell<3>(a.dst, c, m3, v, a.pitch, a.plane);
      }
    }
    float* d = a.dst + aidx(c, 0);
    if (store == 0xfu || ((F & F_FULLSTORE) && store)) {
#pragma unroll
      for (int q = 0; q < kQ; ++q) __builtin_nontemporal_store(v[q], reinterpret_cast<f4*>(d + q * kChunk));
      if (a.store_all_macros) {
        *reinterpret_cast<f4*>(a.rho + c) = R;
        *reinterpret_cast<f4*>(a.ux + c) = UX;
        *reinterpret_cast<f4*>(a.uy + c) = UY;
        *reinterpret_cast<f4*>(a.uz + c) = UZ;
      }
    } else if (store) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (!(store & (1u << j))) continue;
#pragma unroll
        for (int q = 0; q < kQ; ++q) d[q * kChunk + j] = v[q][j];
      }
    }
  }
  if constexpr (F & F_BSUM) {
    const double s = block_sum(acc, red);
    if (threadIdx.x == 0) a.partial[blockIdx.x] = s;
  } else {
    if (acc == -1.0) a.partial[blockIdx.x] = acc;
  }
}

// the shipped per-chunk body, with the kernel's launch bounds as a parameter
template <bool FAST, int MINW>
__global__ __launch_bounds__(256, MINW) void k_prod(const MainArgs a, int ch0) {
  __shared__ double red[4];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int idx = blockIdx.x * 4 + wave;
  double acc = 0.0;
  if (idx < a.nchunks) acc = process_chunk<FAST>(a, (int64_t)a.chunks[idx] * kChunk, lane);
  const double s = block_sum(acc, red);
  if (threadIdx.x == 0) a.partial[blockIdx.x] = s;
}

// XCD-aware order: workgroups are dealt round-robin to the 8 XCDs, so logical block
// (b % 8) * (nb / 8) + b / 8 gives every XCD (its own L2) one contiguous run of chunks
template <bool FAST>
__global__ __launch_bounds__(256) void k_prod_xcd(const MainArgs a, int ch0) {
  __shared__ double red[4];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nb = gridDim.x;  // multiple of 8
  const int lb = (blockIdx.x & 7) * (nb >> 3) + (blockIdx.x >> 3);
  const int idx = lb * 4 + wave;
  double acc = 0.0;
  if (idx < a.nchunks) acc = process_chunk<FAST>(a, (int64_t)a.chunks[idx] * kChunk, lane);
  const double s = block_sum(acc, red);
  if (threadIdx.x == 0) a.partial[lb] = s;
}

// the same with the occupancy pinned by amdgpu_waves_per_eu(W, W)
#define KPRODW(NAME, W)                                                                         \
  template <bool FAST>                                                                          \
  __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W, W))) void NAME(      \
      const MainArgs a, int ch0) {                                                              \
    __shared__ double red[4];                                                                   \
    const int lane = threadIdx.x & 63;                                                          \
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);                          \
    const int idx = blockIdx.x * 4 + wave;                                                      \
    double acc = 0.0;                                                                           \
    if (idx < a.nchunks) acc = process_chunk<FAST>(a, (int64_t)a.chunks[idx] * kChunk, lane); \
    const double s = block_sum(acc, red);                                                       \
    if (threadIdx.x == 0) a.partial[blockIdx.x] = s;                                            \
  }
KPRODW(k_prod_w1, 1)
KPRODW(k_prod_w2, 2)
KPRODW(k_prod_w3, 3)

__global__ void k_lab_type(uint8_t* type, uint32_t* links, int n, int pitch, int xoff, int64_t plane,
                           int64_t ncell) {
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < ncell; c += (int64_t)gridDim.x * blockDim.x) {
    const int64_t u = c + xoff;  // the library's row shift (Layout::xshift)
    const int x = (int)(u % pitch), y = (int)((u / pitch) % n), z = (int)(u / plane) - 1;
    auto cls = [&](int xx, int yy, int zz) -> uint8_t {
      if (xx < 1 || yy < 1 || zz < 1 || xx > n - 2 || yy > n - 2 || zz > n - 2) return kPassive;
      if (xx == 1 || yy == 1 || zz == 1 || xx == n - 2 || yy == n - 2 || zz == n - 2) return kWall;
      return kFluid;
    };
    uint8_t t = cls(x, y, z);
    uint32_t m = 0;
    if (t == kFluid) {
      for (int q = 1; q < kQ; ++q)
        if (cls(x - kEx[q], y - kEy[q], z - kEz[q]) == kWall) m |= 1u << q;
      if (m) t |= kWallAdj;
    }
    type[c] = t;
    links[c] = m;
  }
}

__global__ void k_lab_fill(float* a, int64_t n, float amp) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    a[i] = 1.0f / 19.0f + amp * (float)(i % 7);
}

int main(int argc, char** argv) {
  const int N = argc > 1 ? std::atoi(argv[1]) : 512;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 5;
  const float amp = argc > 3 ? (float)std::atof(argv[3]) : 1e-4f;  // 0: uniform rest state
  Layout L{};
  L.nx = L.ny = L.nz = N;
  const int xoff = argc > 4 ? std::atoi(argv[4]) : 2;  // row shift (Layout::xshift) for LDC
  L.pitch = (N + 3) / 4 * 4;
  L.planes = N + 2;
  L.plane = (int64_t)L.pitch * N;
  L.ncell = (L.plane * L.planes + kChunk - 1) / kChunk * kChunk;
  L.nchunk = L.ncell / kChunk;
  L.guard = (L.plane + L.pitch + 1 + kChunk - 1) / kChunk + 1;
  float *A, *B, *mac;
  uint8_t* type;
  uint32_t* links;
  int *chunks, *stopped;
  double* part;
  CK(hipMalloc(&A, sizeof(float) * L.buf_floats()));
  CK(hipMalloc(&B, sizeof(float) * L.buf_floats()));
  CK(hipMalloc(&mac, sizeof(float) * L.ncell * 4));
  CK(hipMalloc(&type, L.ncell + 64));
  CK(hipMalloc(&links, sizeof(uint32_t) * (L.ncell + 64)));
  CK(hipMalloc(&stopped, sizeof(int)));
  int *retry, *retry_cnt;
  CK(hipMalloc(&retry, sizeof(int) * (N * (int64_t)N * N / 256 + 1024)));
  CK(hipMalloc(&retry_cnt, sizeof(int)));
  CK(hipMemset(retry_cnt, 0, sizeof(int)));
  CK(hipMemset(stopped, 0, sizeof(int)));
  hipLaunchKernelGGL(k_lab_fill, dim3(8192), dim3(256), 0, 0, A, L.buf_floats(), amp);
  hipLaunchKernelGGL(k_lab_fill, dim3(8192), dim3(256), 0, 0, B, L.buf_floats(), amp);
  hipLaunchKernelGGL(k_lab_type, dim3(8192), dim3(256), 0, 0, type, links, N, L.pitch, xoff, L.plane, L.ncell);
  // active chunks: storage planes 3 .. N (fluid z 2 .. N-3)
  const int64_t c_lo = 3 * L.plane, c_hi = (int64_t)(N - 1) * L.plane;
  const int ch0 = (int)(c_lo / kChunk), nch = (int)((c_hi - c_lo) / kChunk);
  std::vector<int> hch(nch);
  for (int i = 0; i < nch; ++i) hch[i] = ch0 + i;
  CK(hipMalloc(&chunks, sizeof(int) * nch));
  CK(hipMemcpy(chunks, hch.data(), sizeof(int) * nch, hipMemcpyHostToDevice));
  CK(hipMalloc(&part, sizeof(double) * (nch + 64)));  // one per block at WPB = 1
  float* a_base = A + L.guard * kQ * kChunk;
  float* b_base = B + L.guard * kQ * kChunk;
  CK(hipDeviceSynchronize());
  const double fluid = (double)(N - 4) * (N - 4) * (N - 4);

  struct V {
    const char* name;
    void (*launch)(const MainArgs&, int, int);
  };
#define VAR(NAME, F, MINW, WPB)                                                                                  \
  V{NAME, [](const MainArgs& m, int c0, int n) {                                                               \
      hipLaunchKernelGGL((k_var<F, MINW, WPB>), dim3((n + WPB - 1) / WPB), dim3(WPB * 64), 0, 0, m, c0); }}
#define PROD(NAME, FAST, MINW)                                                                                \
  V{NAME, [](const MainArgs& m, int c0, int n) {                                                               \
      hipLaunchKernelGGL((k_prod<FAST, MINW>), dim3((n + 3) / 4), dim3(256), 0, 0, m, c0); }}
  std::vector<V> vs = {
#define LDSV(NAME, K, LDS) V{NAME, [](const MainArgs& m, int c0, int n) { hipLaunchKernelGGL(K, dim3((n + 3) / 4), dim3(256), LDS, 0, m, c0); }}
#define XCDV(NAME, K, LDS) V{NAME, [](const MainArgs& m, int c0, int n) { hipLaunchKernelGGL(K, dim3(((n + 3) / 4 + 7) / 8 * 8), dim3(256), LDS, 0, m, c0); }}
      XCDV("xcd fast occ2", (k_prod_xcd<true>), 56 * 1024),
      XCDV("xcd fast occ3", (k_prod_xcd<true>), 40 * 1024),
      XCDV("xcd exact occ3", (k_prod_xcd<false>), 40 * 1024),
      XCDV("xcd exact occ2", (k_prod_xcd<false>), 56 * 1024),
      XCDV("xcd fast occ1", (k_prod_xcd<true>), 100 * 1024),
      XCDV("xcd fast occ2 again", (k_prod_xcd<true>), 56 * 1024),
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<float>> ms(vs.size());
  for (int r = 0; r < rounds; ++r) {
    for (size_t i = 0; i < vs.size(); ++i) {
      MainArgs m{};
      m.type = type; m.links = links;
      m.rho = mac; m.ux = mac + L.ncell; m.uy = mac + 2 * L.ncell; m.uz = mac + 3 * L.ncell;
      m.partial = part; m.chunks = chunks; m.nchunks = nch; m.pitch = L.pitch; m.plane = L.plane;
      m.c_lo = c_lo; m.c_hi = c_hi; m.tau = 0.55f; m.store_all_macros = 0; m.stopped = stopped;
      m.tau_rcp = 1.0f / 0.55f; m.fast_div = 1; m.retry = retry; m.retry_count = retry_cnt;
      CK(hipEventRecord(e0));
      for (int it = 0; it < 4; ++it) {
        m.src = (it & 1) ? b_base : a_base;
        m.dst = (it & 1) ? a_base : b_base;
        vs[i].launch(m, ch0, nch);
      }
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipGetLastError());
      float t = 0;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms[i].push_back(t / 4);
    }
  }
  int nretry = 0;
  CK(hipMemcpy(&nretry, retry_cnt, sizeof(int), hipMemcpyDeviceToHost));
  std::printf("retried chunks (all fast launches): %d\n", nretry);
  for (size_t i = 0; i < vs.size(); ++i) {
    std::sort(ms[i].begin(), ms[i].end());
    const float med = ms[i][ms[i].size() / 2];
    std::printf("%-22s median %7.3f ms  %8.1f MLUPS(fluid)  %7.1f GB/s (152 B/fluid cell)\n", vs[i].name, med,
                fluid / (med * 1e-3) / 1e6, 152.0 * fluid / (med * 1e-3) / 1e9);
  }
  return 0;
}
