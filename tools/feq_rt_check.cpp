// feq_rt_check.cpp -- host check that lbm::feq_rt (run-time q, used by the NEE path of
// k_step) is bit-identical to the reference expression trees feq<q> / feq_bc<q> for
// q = 1..18, over random and special inputs.  Built and run by tests/test_feq_rt.py:
//   g++ -O2 -std=c++17 -ffp-contract=off tools/feq_rt_check.cpp -o feq_rt_check && ./feq_rt_check [n]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "../lattice-boltzmann-method-gpu_amd/csrc/lbm_d3q19.hpp"

using namespace lbm;

template <int Q>
static float ref_q(float r, float x, float y, float z, bool bc) {
  return bc ? feq_bc<Q>(r, x, y, z) : feq<Q>(r, x, y, z);
}
static float ref(int q, float r, float x, float y, float z, bool bc) {
  switch (q) {
#define C(Q) case Q: return ref_q<Q>(r, x, y, z, bc);
    C(1) C(2) C(3) C(4) C(5) C(6) C(7) C(8) C(9) C(10) C(11) C(12) C(13) C(14) C(15) C(16) C(17) C(18)
#undef C
  }
  return 0.f;
}
static uint32_t bits(float v) {
  uint32_t u;
  std::memcpy(&u, &v, 4);
  return u;
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? std::atol(argv[1]) : 200000;
  std::mt19937 g(12345);
  std::uniform_real_distribution<float> ur(0.5f, 1.5f), uu(-0.2f, 0.2f), uw(-1e3f, 1e3f);
  const float special[] = {0.f, -0.f, 1e-30f, -1e-30f, 0.06071645f, -0.06071645f, 0.15f, 1.0f, -1.0f, 3.4e38f};
  long bad = 0, checked = 0;
  for (long i = 0; i < n; ++i) {
    float r = ur(g), x, y, z;
    if (i % 7 == 0) {  // special values in any slot
      const int k = (int)(sizeof(special) / sizeof(float));
      x = special[g() % k]; y = special[g() % k]; z = special[g() % k];
      if (i % 14 == 0) r = special[g() % k];
    } else if (i % 5 == 0) {
      x = uw(g); y = uw(g); z = uw(g);
    } else {
      x = uu(g); y = uu(g); z = uu(g);
    }
    for (int q = 1; q < 19; ++q)
      for (int bc = 0; bc < 2; ++bc) {
        const float a = feq_rt(q, r, x, y, z, bc != 0), b = ref(q, r, x, y, z, bc != 0);
        ++checked;
        if (bits(a) != bits(b) && !(std::isnan(a) && std::isnan(b))) {
          if (bad < 10)
            std::printf("MISMATCH q=%d bc=%d r=%a u=(%a,%a,%a): %a vs %a\n", q, bc, r, x, y, z, a, b);
          ++bad;
        }
      }
  }
  std::printf("checked %ld, mismatches %ld\n", checked, bad);
  return bad ? 1 : 0;
}
