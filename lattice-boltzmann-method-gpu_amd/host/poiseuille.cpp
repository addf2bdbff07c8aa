// poiseuille -- drop-in for Poiseulle_flow/Poiseulle.cu (main 940-1056): pipe of radius
// (NX-1)/2 along y, tau 0.58, parabolic velocity NEE inlet (y=1) and outlet (y=NY-2) with the
// kernel's hard-coded u_max 0.09714700668 (Poiseulle.cu:590), wall bounce-back, the same loop
// constants as ldc, pos_<k>.vtk + CONVERGENCE.log into ./out.
// Overrides: --nx --ny --nz --tau --max-it --time-save --out --device
#include "driver_common.hpp"

int main(int argc, char** argv) {
  drv::Args args(argc, argv);
  const int NX = args.geti("--nx", 64), NY = args.geti("--ny", 64), NZ = args.geti("--nz", 64);
  const float CH = 0.0000655737f, C_U = 1.5441f, tau = args.getf("--tau", 0.58f);  // Poiseulle.cu:39
  const float tol = 1e-6f;
  const int stag_max = 50, max_it = args.geti("--max-it", 10000), time_save = args.geti("--time-save", 500);
  const std::string out = args.get("--out", "./out");
  drv::ensure_dir(out);
  std::FILE* logfile = std::fopen((out + "/CONVERGENCE.log").c_str(), "w");

  const size_t n = (size_t)NX * NY * NZ;
  std::vector<int8_t> geo(n);
  lbmh_geo_poiseuille(NX, NY, NZ, geo.data());
  const long NLATTICE = (long)lbmh_index_transform(NX, NY, NZ, geo.data(), nullptr);
  std::vector<float> prof((size_t)NX * NZ);
  lbmh_poiseuille_profile(NX, NZ, 0.09714700668f, prof.data());
  drv::Fields f(n);
  lbmh_initial_fields(1, NX, NY, NZ, geo.data(), nullptr, nullptr, f.rho.data(), f.ux.data(), f.uy.data(), f.uz.data());

  lbm_desc d{};
  d.nx = NX; d.ny = NY; d.nz = NZ; d.tau = tau; d.case_kind = LBM_CASE_POISEUILLE; d.geo = geo.data();
  d.bc_inlet_uy = prof.data(); d.bc_outlet_uy = prof.data();
  d.device = args.geti("--device", 0); d.nz_global = NZ;
  lbm_ctx* ctx = nullptr;
  drv::check(lbm_create(&d, &ctx), nullptr, "lbm_create");
  drv::check(lbm_init_equilibrium(ctx, LBM_INIT_EXPANDED, f.rho.data(), f.ux.data(), f.uy.data(), f.uz.data()), ctx,
             "lbm_init_equilibrium");

  drv::Timer timer;
  auto save = [&](int k, float residual) {
    f.fetch(ctx);
    std::printf("ITERATION # %d, collapse time: %g ms, residual:%g\n", k, timer.ms(), residual);
    std::fprintf(logfile, "%g\n", residual);
    lbmh_write_vtk((out + "/pos_" + std::to_string(k) + ".vtk").c_str(), 1, NX, NY, NZ, geo.data(), f.ux.data(),
                   f.uy.data(), f.uz.data(), C_U, CH);
  };
  float residual = 0.0f;
  const int k = drv::converge_loop(ctx, max_it, stag_max, tol, time_save, save, &residual);
  f.fetch(ctx);
  lbmh_write_vtk((out + "/pos_" + std::to_string(k) + ".vtk").c_str(), 1, NX, NY, NZ, geo.data(), f.ux.data(),
                 f.uy.data(), f.uz.data(), C_U, CH);
  const float milli = timer.ms();
  std::printf("TOTAL RUNNING TIME: %g MILLI SECONDS#LATTICE%ld\n", milli, NLATTICE);
  std::printf("Residual is %g\n", residual);
  std::fprintf(logfile, "TOTAL RUNNING TIME: %g MILLI SECONDS#LATTICE%ld ERROR IS%g\n", milli, NLATTICE, residual);
  std::fclose(logfile);
  lbm_destroy(ctx);
  return 0;
}
