// alloc_lab.hip -- how does the HBM write rate of a large buffer depend on how it was allocated?
// (measurement tool, not product code)
//
// buffer_placement (lbm_ctx.hip) found that whole-buffer write sweeps of equal-sized allocations run
// at ~5.0-5.6, ~6.0-6.4 or ~7.0-7.2 TB/s, stable per allocation.  This lab allocates K buffers of
// G GiB with one method and prints, per buffer, the rate of a whole-buffer write sweep and read
// sweep (one contiguous region per XCD, 16-B non-temporal accesses) and of each 2-GiB window of
// it written alone, so per-allocation and per-region effects can be told apart.
//   method 0: hipMalloc; 1: hipExtMallocWithFlags(hipDeviceMallocContiguous);
//          2: VMM -- one hipMemCreate handle per buffer, mapped into a reserved range;
//          3: VMM -- the buffer assembled from 2-GiB handles, each mapped at its place.
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/alloc_lab.hip -o tools/alloc_lab
//   tools/alloc_lab K GiB method [1: interleave periods of the XCD regions instead of windows]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e = (x);                                                                     \
    if (e != hipSuccess) {                                                                  \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      std::exit(1);                                                                         \
    }                                                                                       \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void region(int64_t n4, int64_t& lo, int64_t& hi, int& lb, int& nbx) {
  const int xcd = blockIdx.x & 7;
  nbx = gridDim.x >> 3;
  lb = blockIdx.x >> 3;
  const int64_t per = (n4 + 7) / 8;
  lo = xcd * per;
  hi = lo + per < n4 ? lo + per : n4;
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
  if (acc.x == 1234.5f) out[0] = acc.y + acc.z + acc.w;
}

// the same write sweep with the XCDs' regions interleaved at period S vectors: XCD x writes the
// runs [(8j + x) S, (8j + x + 1) S), in order of j (S = n4 / 8: one contiguous region per XCD,
// the sweep above and k_step's chunk order)
__global__ __launch_bounds__(256) void k_write_s(f4* __restrict__ b, int64_t n4, int64_t S) {
  const int xcd = blockIdx.x & 7, lb = blockIdx.x >> 3, nbx = gridDim.x >> 3;
  const int64_t per = n4 / 8;
  const f4 v{0.f, 0.f, 0.f, 0.f};
  for (int64_t t0 = (int64_t)lb * 1024 + threadIdx.x; t0 < per; t0 += (int64_t)nbx * 1024) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t t = t0 + k * 256;
      if (t < per) __builtin_nontemporal_store(v, b + ((t / S) * 8 + xcd) * S + (t % S));
    }
  }
}
__global__ __launch_bounds__(256) void k_copy_s(const f4* __restrict__ a, f4* __restrict__ b, int64_t n4, int64_t S) {
  const int xcd = blockIdx.x & 7, lb = blockIdx.x >> 3, nbx = gridDim.x >> 3;
  const int64_t per = n4 / 8;
  for (int64_t t0 = (int64_t)lb * 1024 + threadIdx.x; t0 < per; t0 += (int64_t)nbx * 1024) {
    f4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t t = t0 + k * 256;
      v[k] = t < per ? __builtin_nontemporal_load(a + ((t / S) * 8 + xcd) * S + (t % S)) : f4{};
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t t = t0 + k * 256;
      if (t < per) __builtin_nontemporal_store(v[k], b + ((t / S) * 8 + xcd) * S + (t % S));
    }
  }
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? std::atoi(argv[1]) : 6;
  const double gib = argc > 2 ? std::atof(argv[2]) : 10.0;
  const int method = argc > 3 ? std::atoi(argv[3]) : 0;
  const size_t piece = (size_t)2 << 30;
  size_t bytes = (size_t)(gib * (double)(1ull << 30));
  bytes = (bytes + piece - 1) / piece * piece;
  const int64_t n4 = (int64_t)(bytes / 16);
  std::vector<f4*> buf(K);
  hipMemAllocationProp prop{};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  hipMemAccessDesc acc{};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  for (int i = 0; i < K; ++i) {
    if (method == 0) {
      CK(hipMalloc(&buf[i], bytes));
    } else if (method == 1) {
      CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&buf[i]), bytes, hipDeviceMallocContiguous));
    } else {
      void* va = nullptr;
      CK(hipMemAddressReserve(&va, bytes, piece, nullptr, 0));
      const size_t step = method == 2 ? bytes : piece;
      for (size_t off = 0; off < bytes; off += step) {
        hipMemGenericAllocationHandle_t h;
        CK(hipMemCreate(&h, step, &prop, 0));
        CK(hipMemMap(static_cast<char*>(va) + off, step, 0, h, 0));
      }
      CK(hipMemSetAccess(va, bytes, &acc, 1));
      buf[i] = static_cast<f4*>(va);
    }
    CK(hipMemset(buf[i], 0, bytes));
  }
  float* out = nullptr;
  CK(hipMalloc(&out, 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int blocks = 8 * 1024;
  auto timeit = [&](auto&& f) {
    f();
    CK(hipEventRecord(e0));
    for (int r = 0; r < 3; ++r) f();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / 3;
  };
  if (argc > 4 && std::atoi(argv[4]) == 1) {  // interleave periods: write of each buffer, copy i -> i+1
    const int64_t periods[] = {n4 / 8, (64 << 20) / 16, (16 << 20) / 16, (4 << 20) / 16, (2 << 20) / 16,
                               (1 << 20) / 16, (256 << 10) / 16, (64 << 10) / 16, 81920, 5120};
    for (int i = 0; i < K; ++i) {
      const int j = (i + 1) % K;
      std::printf("{\"buf\": %d, \"period_bytes\": [", i);
      for (size_t p = 0; p < sizeof(periods) / sizeof(periods[0]); ++p)
        std::printf("%s%lld", p ? ", " : "", (long long)periods[p] * 16);
      std::printf("], \"write_tbs\": [");
      for (size_t p = 0; p < sizeof(periods) / sizeof(periods[0]); ++p) {
        const int64_t S = periods[p];
        if ((n4 / 8) % S) { std::printf("%snull", p ? ", " : ""); continue; }  // S must divide an XCD's share
        const float m = timeit([&] { hipLaunchKernelGGL(k_write_s, dim3(blocks), dim3(256), 0, 0, buf[i], n4, S); });
        std::printf("%s%.3f", p ? ", " : "", bytes / m / 1e9);
      }
      std::printf("], \"copy_to_next_tbs\": [");
      for (size_t p = 0; p < sizeof(periods) / sizeof(periods[0]); ++p) {
        const int64_t S = periods[p];
        if ((n4 / 8) % S) { std::printf("%snull", p ? ", " : ""); continue; }
        const float m = timeit([&] { hipLaunchKernelGGL(k_copy_s, dim3(blocks), dim3(256), 0, 0, buf[i], buf[j], n4, S); });
        std::printf("%s%.3f", p ? ", " : "", 2.0 * bytes / m / 1e9);
      }
      std::printf("]}\n");
    }
    return 0;
  }
  const int64_t w4 = (int64_t)(piece / 16);
  for (int i = 0; i < K; ++i) {
    const float mw = timeit([&] { hipLaunchKernelGGL(k_write, dim3(blocks), dim3(256), 0, 0, buf[i], n4); });
    const float mr = timeit([&] { hipLaunchKernelGGL(k_read, dim3(blocks), dim3(256), 0, 0, buf[i], n4, out); });
    std::printf("{\"method\": %d, \"buf\": %d, \"va\": \"%p\", \"write_tbs\": %.3f, \"read_tbs\": %.3f, \"window_write_tbs\": [",
                method, i, (void*)buf[i], bytes / mw / 1e9, bytes / mr / 1e9);
    for (int64_t o = 0; o + w4 <= n4; o += w4) {
      f4* p = buf[i] + o;
      const float m = timeit([&] { hipLaunchKernelGGL(k_write, dim3(blocks), dim3(256), 0, 0, p, w4); });
      std::printf("%s%.3f", o ? ", " : "", piece / m / 1e9);
    }
    std::printf("]}\n");
  }
  return 0;
}
