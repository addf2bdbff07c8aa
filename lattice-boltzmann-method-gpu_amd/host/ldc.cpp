// ldc -- drop-in for Lid_driven_cavity/ldc.cu (main 612-717): 64^3 cavity, tau 0.55,
// lid 0.15 m/s (u_lid = 0.15f / C_U along +z on y = NY-2), tol 1e-6 x 50 consecutive-or-not
// hits, max 10000 steps, VTK + log every 500 steps into ./out.
// Overrides: --nx --ny --nz --tau --max-it --time-save --out --device
#include "driver_common.hpp"

int main(int argc, char** argv) {
  drv::Args args(argc, argv);
  const int NX = args.geti("--nx", 64), NY = args.geti("--ny", 64), NZ = args.geti("--nz", 64);
  const float CH = 0.0000655737f, C_U = 2.4705f;           // ldc.cu:49
  const float tau = args.getf("--tau", 0.55f);              // ldc.cu:55
  const float u_max = 0.15f / C_U;                          // ldc.cu:52
  const float tol = 1e-6f;                                  // ldc.cu:614
  const int stag_max = 50, max_it = args.geti("--max-it", 10000), time_save = args.geti("--time-save", 500);
  const std::string out = args.get("--out", "./out");
  drv::ensure_dir(out);
  std::FILE* logfile = std::fopen((out + "/CONVERGENCE.log").c_str(), "w");
  const int bx = 1 + (NX - 1) / 8, by = 1 + (NY - 1) / 8, bz = 1 + (NZ - 1) / 8;
  const long NLATTICE = (long)bx * by * bz * 512;          // ldc.cu:53-54 (padded bricks)

  const size_t n = (size_t)NX * NY * NZ;
  std::vector<int8_t> geo(n);
  lbmh_geo_ldc(NX, NY, NZ, geo.data());
  drv::Fields f(n);
  lbmh_initial_fields(0, NX, NY, NZ, geo.data(), nullptr, nullptr, f.rho.data(), f.ux.data(), f.uy.data(), f.uz.data());

  lbm_desc d{};
  d.nx = NX; d.ny = NY; d.nz = NZ; d.tau = tau; d.case_kind = LBM_CASE_LDC; d.geo = geo.data();
  d.lid_u = u_max; d.device = args.geti("--device", 0); d.nz_global = NZ;
  lbm_ctx* ctx = nullptr;
  drv::check(lbm_create(&d, &ctx), nullptr, "lbm_create");
  drv::check(lbm_init_equilibrium(ctx, LBM_INIT_LDC_WI, f.rho.data(), f.ux.data(), f.uy.data(), f.uz.data()), ctx,
             "lbm_init_equilibrium");

  drv::Timer timer;
  auto save = [&](int k, float residual) {
    f.fetch(ctx);
    std::printf("ITERATION # %d, collapse time: %g ms, residual:%g\n", k, timer.ms(), residual);
    std::fprintf(logfile, "%g\n", residual);
    lbmh_write_vtk((out + "/lid_" + std::to_string(k) + ".vtk").c_str(), 0, NX, NY, NZ, geo.data(), f.ux.data(),
                   f.uy.data(), f.uz.data(), C_U, CH);
  };
  float residual = 0.0f;
  const int k = drv::converge_loop(ctx, max_it, stag_max, tol, time_save, save, &residual);
  const float milli = timer.ms();
  std::printf("TOTAL RUNNING TIME: %g MILLI SECONDS#LATTICE%ld\n", milli, NLATTICE);
  std::printf("Residual is %g\n", residual);
  std::fprintf(logfile, "TOTAL RUNNING TIME: %g MILLI SECONDS#LATTICE%ld ERROR IS%g\n", milli, NLATTICE, residual);
  std::fclose(logfile);
  f.fetch(ctx);
  lbmh_write_vtk((out + "/lid_" + std::to_string(k) + ".vtk").c_str(), 0, NX, NY, NZ, geo.data(), f.ux.data(),
                 f.uy.data(), f.uz.data(), C_U, CH);
  lbm_destroy(ctx);
  return 0;
}
