// driver_common.hpp -- shared plumbing of the three drop-in case drivers (ldc, poiseuille,
// bifurcation).  Each driver reproduces its reference main() (ldc.cu:612-717,
// Poiseulle.cu:940-1056, bifurcation.cu:1177-1326): same defaults, same ./out files
// (VTK snapshots + CONVERGENCE.log) and the same stdout lines, with the hot path running
// through liblbm.so.  Command-line overrides exist for benchmarking; with no arguments
// the reference configuration runs.
#pragma once
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <sys/stat.h>
#include <vector>

#include "../../include/lbm.h"
#include "../../include/lbm_host.h"

namespace drv {

struct Args {
  std::vector<std::string> v;
  Args(int argc, char** argv) : v(argv + 1, argv + argc) {}
  bool has(const char* k) const {
    for (auto& s : v) if (s == k) return true;
    return false;
  }
  std::string get(const char* k, const std::string& def) const {
    for (size_t i = 0; i + 1 < v.size(); ++i) if (v[i] == k) return v[i + 1];
    return def;
  }
  int geti(const char* k, int def) const { return std::atoi(get(k, std::to_string(def)).c_str()); }
  float getf(const char* k, float def) const {
    const std::string s = get(k, "");
    return s.empty() ? def : std::strtof(s.c_str(), nullptr);
  }
};

inline void check(int rc, lbm_ctx* ctx, const char* what) {
  if (rc != LBM_OK) {
    std::fprintf(stderr, "%s failed (%d): %s\n", what, rc, lbm_last_error(ctx));
    std::exit(1);
  }
}

inline void ensure_dir(const std::string& d) { ::mkdir(d.c_str(), 0755); }

struct Timer {
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  float ms() const {
    return std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
};

struct Fields {
  std::vector<float> rho, ux, uy, uz;
  explicit Fields(size_t n) : rho(n), ux(n), uy(n), uz(n) {}
  void fetch(lbm_ctx* ctx) { check(lbm_get_macros(ctx, rho.data(), ux.data(), uy.data(), uz.data()), ctx, "lbm_get_macros"); }
};

}  // namespace drv

namespace drv {

// The reference convergence loop (ldc.cu:653-685, Poiseulle.cu:986-1019) on the device:
// steps run in chunks that end on the save steps (k % time_save == 0); on_save(k, residual)
// is called after each of those.  Returns the final k; *residual = last step's residual.
template <class F>
int converge_loop(lbm_ctx* ctx, int max_it, int stag_max, float tol, int time_save, F on_save,
                  float* residual) {
  check(lbm_set_convergence(ctx, 1, max_it, stag_max, tol), ctx, "lbm_set_convergence");
  int k = 0;
  float res = 0.0f;
  std::vector<float> hist;
  for (;;) {
    const int save_at = (k + time_save - 1) / time_save * time_save;  // next multiple >= k
    const int count = save_at - k + 1;
    hist.assign(count, 0.0f);
    int done = 0;
    check(lbm_step(ctx, count, hist.data(), &done), ctx, "lbm_step");
    const int ran = done - k;
    if (ran > 0) res = hist[ran - 1];
    k = done;
    if (ran == count) on_save(save_at, res);
    int stopped = 0;
    check(lbm_get_state(ctx, nullptr, nullptr, &stopped, nullptr, nullptr), ctx, "lbm_get_state");
    if (stopped || ran < count) break;
  }
  *residual = res;
  return k;
}

}  // namespace drv
