// place_lab.hip -- is HBM streaming rate a property of the allocation? (not product code)
//
// k_step at 512^3 runs in two modes (~3.40 vs ~3.70 ms) that follow the population buffers'
// allocation, not the code.  This lab allocates K buffers of the 512^3 buffer size and times,
// interleaved over rounds: a read-only sweep of each buffer, a write-only sweep of each, and a
// copy for every ordered pair.  Stable per-buffer / per-pair numbers across rounds = placement.
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/place_lab.hip -o tools/place_lab
//   tools/place_lab [K=4] [GiB=10.2] [rounds=3] [flags: 0 hipMalloc, 4 contiguous]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e = (x);                                                                       \
    if (e != hipSuccess) {                                                                    \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));   \
      std::exit(1);                                                                           \
    }                                                                                         \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

// one contiguous region per XCD (blocks b, b+8, ... share an XCD), 4 f4 per thread per trip
__device__ __forceinline__ void region(int64_t n4, int64_t& lo, int64_t& hi, int& lb, int& nbx) {
  const int xcd = blockIdx.x & 7;
  nbx = gridDim.x >> 3;
  lb = blockIdx.x >> 3;
  const int64_t per = (n4 + 7) / 8;
  lo = xcd * per;
  hi = lo + per < n4 ? lo + per : n4;
}

// sweep orders of a whole buffer: 0 one forward region per XCD, 1 grid-stride (XCDs
// interleaved), 2 per-XCD regions with the odd XCDs sweeping backwards, 3 per-XCD regions in
// 64-MiB pieces visited in a per-XCD rotated order
template <int MODE, typename F>
__device__ __forceinline__ void sweep(int64_t n4, F&& f) {
  if constexpr (MODE == 1) {
    for (int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 1024) f(i, n4);
  } else {
    int64_t lo, hi;
    int lb, nbx;
    region(n4, lo, hi, lb, nbx);
    const int xcd = blockIdx.x & 7;
    const int64_t trips = (hi - lo + (int64_t)nbx * 1024 - 1) / ((int64_t)nbx * 1024);
    for (int64_t t = 0; t < trips; ++t) {
      int64_t tt = t;
      if (MODE == 2 && (xcd & 1)) tt = trips - 1 - t;
      if (MODE == 3) tt = (t + (trips * xcd) / 8) % trips;
      const int64_t i = lo + tt * nbx * 1024 + (int64_t)lb * 1024 + threadIdx.x;
      if (i < hi) f(i, hi);
    }
  }
}

template <int MODE>
__global__ __launch_bounds__(256) void k_copy_m(const f4* __restrict__ a, f4* __restrict__ b, int64_t n4) {
  sweep<MODE>(n4, [&](int64_t i, int64_t hi) {
    f4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = i + k * 256 < hi ? __builtin_nontemporal_load(a + i + k * 256) : f4{};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (i + k * 256 < hi) __builtin_nontemporal_store(v[k], b + i + k * 256);
  });
}

template <int MODE>
__global__ __launch_bounds__(256) void k_write_m(f4* __restrict__ b, int64_t n4) {
  const f4 v{0.f, 0.f, 0.f, 0.f};
  sweep<MODE>(n4, [&](int64_t i, int64_t hi) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (i + k * 256 < hi) __builtin_nontemporal_store(v, b + i + k * 256);
  });
}

__global__ __launch_bounds__(256) void k_copy(const f4* __restrict__ a, f4* __restrict__ b, int64_t n4) {
  int64_t lo, hi;
  int lb, nbx;
  region(n4, lo, hi, lb, nbx);
  for (int64_t i = lo + (int64_t)lb * 1024 + threadIdx.x; i < hi; i += (int64_t)nbx * 1024) {
    f4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = i + k * 256 < hi ? __builtin_nontemporal_load(a + i + k * 256) : f4{};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (i + k * 256 < hi) __builtin_nontemporal_store(v[k], b + i + k * 256);
  }
}

__global__ __launch_bounds__(256) void k_read(const f4* __restrict__ a, int64_t n4, float* out) {
  int64_t lo, hi;
  int lb, nbx;
  region(n4, lo, hi, lb, nbx);
  f4 acc{};
  for (int64_t i = lo + (int64_t)lb * 1024 + threadIdx.x; i < hi; i += (int64_t)nbx * 1024) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (i + k * 256 < hi) acc += __builtin_nontemporal_load(a + i + k * 256);
  }
  if (acc.x == 1234.5f) out[0] = acc.y + acc.z + acc.w;  // never true for zeroed buffers
}

__global__ __launch_bounds__(256) void k_write(f4* __restrict__ b, int64_t n4) {
  int64_t lo, hi;
  int lb, nbx;
  region(n4, lo, hi, lb, nbx);
  const f4 v{0.f, 0.f, 0.f, 0.f};
  for (int64_t i = lo + (int64_t)lb * 1024 + threadIdx.x; i < hi; i += (int64_t)nbx * 1024) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (i + k * 256 < hi) __builtin_nontemporal_store(v, b + i + k * 256);
  }
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? std::atoi(argv[1]) : 4;
  const double gib = argc > 2 ? std::atof(argv[2]) : 10.2;
  const int rounds = argc > 3 ? std::atoi(argv[3]) : 3;
  const unsigned flags = argc > 4 ? (unsigned)std::atoi(argv[4]) : 0u;
  const size_t bytes = (size_t)(gib * (1 << 30)) / 4096 * 4096;
  const int64_t n4 = (int64_t)(bytes / 16);
  std::vector<f4*> buf(K);
  for (int i = 0; i < K; ++i) {
    if (flags)
      CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&buf[i]), bytes, flags));
    else
      CK(hipMalloc(&buf[i], bytes));
    CK(hipMemset(buf[i], 0, bytes));
    std::printf("{\"buf\": %d, \"va\": \"%p\"}\n", i, (void*)buf[i]);
  }
  float* out;
  CK(hipMalloc(&out, 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int blocks = 256 * 8 * 4;  // 8 waves... x4 per CU
  auto timeit = [&](auto&& f) {
    f();  // warm
    CK(hipEventRecord(e0));
    for (int r = 0; r < 3; ++r) f();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / 3;
  };
  const int64_t slice4 = (int64_t)(1 << 30) / 16;  // per-GiB write rates inside each buffer
  const bool slices = argc > 5 && std::atoi(argv[5]) > 0;
  for (int r = 0; r < (slices ? 2 : 0); ++r)
    for (int i = 0; i < K; ++i) {
      std::printf("{\"round\": %d, \"buf\": %d, \"slice_write_tbs\": [", r, i);
      for (int64_t o = 0; o + slice4 <= n4; o += slice4) {
        f4* p = buf[i] + o;
        const float mw = timeit([&] { hipLaunchKernelGGL(k_write, dim3(blocks), dim3(256), 0, 0, p, slice4); });
        std::printf("%s%.2f", o ? ", " : "", (1 << 30) / mw / 1e9);
      }
      std::printf("]}\n");
    }
  // VMM: 1-GiB physical handles, each mapped on its own
  if (slices) {
    hipMemAllocationProp prop{};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    const size_t piece = (size_t)1 << 30;
    const int nh = argc > 5 ? std::atoi(argv[5]) : 16;
    std::printf("{\"vmm_piece_write_tbs\": [");
    std::vector<hipMemGenericAllocationHandle_t> hs(nh);
    std::vector<void*> vas(nh);
    for (int h = 0; h < nh; ++h) {
      CK(hipMemCreate(&hs[h], piece, &prop, 0));
      CK(hipMemAddressReserve(&vas[h], piece, piece, nullptr, 0));
      CK(hipMemMap(vas[h], piece, 0, hs[h], 0));
      hipMemAccessDesc acc{};
      acc.location = prop.location;
      acc.flags = hipMemAccessFlagsProtReadWrite;
      CK(hipMemSetAccess(vas[h], piece, &acc, 1));
      f4* p = static_cast<f4*>(vas[h]);
      const float mw = timeit([&] { hipLaunchKernelGGL(k_write, dim3(blocks), dim3(256), 0, 0, p, slice4); });
      const float mr = timeit([&] { hipLaunchKernelGGL(k_read, dim3(blocks), dim3(256), 0, 0, p, slice4, out); });
      std::printf("%s[%.2f, %.2f]", h ? ", " : "", piece / mw / 1e9, piece / mr / 1e9);
    }
    std::printf("]}\n");
    for (int h = 0; h < nh; ++h) {
      CK(hipMemUnmap(vas[h], piece));
      CK(hipMemAddressFree(vas[h], piece));
      CK(hipMemRelease(hs[h]));
    }
  }
  // sweep orders: write of each buffer and copy i -> i+1, per mode
  for (int r = 0; r < 2; ++r)
    for (int i = 0; i < K; ++i) {
      float w[4], cp[4];
      const int j = (i + 1) % K;
#define MODEX(M)                                                                                     \
  w[M] = timeit([&] { hipLaunchKernelGGL(k_write_m<M>, dim3(blocks), dim3(256), 0, 0, buf[i], n4); }); \
  cp[M] = timeit([&] { hipLaunchKernelGGL(k_copy_m<M>, dim3(blocks), dim3(256), 0, 0, buf[i], buf[j], n4); });
      MODEX(0) MODEX(1) MODEX(2) MODEX(3)
#undef MODEX
      std::printf("{\"round\": %d, \"buf\": %d, \"write_tbs_by_mode\": [%.2f, %.2f, %.2f, %.2f], "
                  "\"copy_to_next_tbs_by_mode\": [%.2f, %.2f, %.2f, %.2f]}\n",
                  r, i, bytes / w[0] / 1e9, bytes / w[1] / 1e9, bytes / w[2] / 1e9, bytes / w[3] / 1e9,
                  2 * bytes / cp[0] / 1e9, 2 * bytes / cp[1] / 1e9, 2 * bytes / cp[2] / 1e9, 2 * bytes / cp[3] / 1e9);
      std::fflush(stdout);
    }
  for (int r = 0; r < rounds; ++r) {
    for (int i = 0; i < K; ++i) {
      const float mr = timeit([&] { hipLaunchKernelGGL(k_read, dim3(blocks), dim3(256), 0, 0, buf[i], n4, out); });
      const float mw = timeit([&] { hipLaunchKernelGGL(k_write, dim3(blocks), dim3(256), 0, 0, buf[i], n4); });
      std::printf("{\"round\": %d, \"buf\": %d, \"read_tbs\": %.3f, \"write_tbs\": %.3f}\n", r, i,
                  bytes / mr / 1e9, bytes / mw / 1e9);
    }
    for (int i = 0; i < K; ++i)
      for (int j = 0; j < K; ++j) {
        if (i == j) continue;
        const float m =
            timeit([&] { hipLaunchKernelGGL(k_copy, dim3(blocks), dim3(256), 0, 0, buf[i], buf[j], n4); });
        std::printf("{\"round\": %d, \"src\": %d, \"dst\": %d, \"copy_tbs\": %.3f}\n", r, i, j, 2.0 * bytes / m / 1e9);
      }
    std::fflush(stdout);
  }
  return 0;
}
