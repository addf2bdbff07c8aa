// bifurcation -- drop-in for bifurcation/bifurcation.cu (main 1177-1326): 64x83x32 mask from
// ./geo.txt, inlet u_y from ./bc.txt, pressure outlet, tau 0.55, REPEAT = 4400 (4401 steps),
// host residual (calc_res) and bif_<i>.vtk at i % 4400 == 0, meas1.txt at the end.
// Overrides: --geo PATH --bc PATH --bc-inlet-block B (0 = as shipped, 1 = block matching the
// shipped inlet) --repeat N --time-save N --out DIR --device N
#include "driver_common.hpp"

int main(int argc, char** argv) {
  drv::Args args(argc, argv);
  const int NX = 64, NY = 83, NZ = 32;                         // bifurcation.cu:19
  const int REPEAT = args.geti("--repeat", 4400), time_save = args.geti("--time-save", 4400);
  const float CH = 0.000248925f, C_U = 0.24159041f, tau = 0.55f;  // bifurcation.cu:20,434
  const std::string out = args.get("--out", "./out");
  drv::ensure_dir(out);
  std::FILE* logfile = std::fopen((out + "/CONVERGENCE.log").c_str(), "w");

  const size_t n = (size_t)NX * NY * NZ;
  std::vector<int32_t> raw(n);
  const std::string geo_path = args.get("--geo", "./geo.txt"), bc_path = args.get("--bc", "./bc.txt");
  if (lbmh_read_geo_txt(geo_path.c_str(), NX, NY, NZ, raw.data()) != (long)n) {
    std::fprintf(stderr, "cannot read %s\n", geo_path.c_str());
    return 1;
  }
  std::vector<int8_t> geo(n);
  lbmh_geo_mask(NX, NY, NZ, raw.data(), geo.data());
  const long NLATTICE = (long)lbmh_index_transform(NX, NY, NZ, geo.data(), nullptr);
  std::vector<float> inlet((size_t)NX * NZ), outlet((size_t)NX * NZ);
  if (lbmh_read_bc_txt(bc_path.c_str(), NX, NY, NZ, geo.data(), args.geti("--bc-inlet-block", 0), inlet.data(),
                       outlet.data()) < 0) {
    std::fprintf(stderr, "cannot read %s\n", bc_path.c_str());
    return 1;
  }
  drv::Fields f(n);
  lbmh_initial_fields(2, NX, NY, NZ, geo.data(), inlet.data(), outlet.data(), f.rho.data(), f.ux.data(), f.uy.data(),
                      f.uz.data());

  lbm_desc d{};
  d.nx = NX; d.ny = NY; d.nz = NZ; d.tau = tau; d.case_kind = LBM_CASE_MASK; d.geo = geo.data();
  d.bc_inlet_uy = inlet.data(); d.device = args.geti("--device", 0); d.nz_global = NZ;
  lbm_ctx* ctx = nullptr;
  drv::check(lbm_create(&d, &ctx), nullptr, "lbm_create");
  drv::check(lbm_init_equilibrium(ctx, LBM_INIT_EXPANDED, f.rho.data(), f.ux.data(), f.uy.data(), f.uz.data()), ctx,
             "lbm_init_equilibrium");
  // host copies start as the initial fields (calc_res at i = 0 reads them: bifurcation.cu:1260)
  drv::Timer timer;
  float residual = 0.0f;
  long double sum1 = 0.0L, sum2 = 0.0L;  // bifurcation.cu:1179
  for (int i = 0; i <= REPEAT;) {
    // run up to the next save step (or the end) in one call
    int next = (i + time_save - 1) / time_save * time_save;
    if (next > REPEAT) next = REPEAT;
    const int count = next - i + 1;
    drv::check(lbm_step(ctx, count, nullptr, nullptr), ctx, "lbm_step");
    i += count;
    const int last = i - 1;
    if (last % time_save == 0) {
      sum1 = lbmh_calc_res(NX, NY, NZ, geo.data(), f.ux.data(), f.uy.data(), f.uz.data());
      f.fetch(ctx);
      const float milli = timer.ms();
      sum2 = lbmh_calc_res(NX, NY, NZ, geo.data(), f.ux.data(), f.uy.data(), f.uz.data());
      residual = (float)(std::fabs(sum1 - sum2) / sum2);  // long double, then float (bifurcation.cu:1269)
      std::fprintf(logfile, "%g\n", residual);
      std::printf("ITERATION # %d, collapse time: %g ms, residual:%g\n", last, milli, residual);
      lbmh_write_vtk((out + "/bif_" + std::to_string(last) + ".vtk").c_str(), 2, NX, NY, NZ, geo.data(), f.ux.data(),
                     f.uy.data(), f.uz.data(), C_U, CH);
    }
  }
  // write_once (bifurcation.cu:1055-1074): u_y then u_x on the z = NZ/2 plane, every stored
  // cell.  The host arrays are the device's at that point (copied back at every save step,
  // bifurcation.cu:1262-1265), and the device macro arrays are never uploaded (1225-1232) nor
  // written off-fluid (only geo == 4 cells, 592-595): stored non-fluid cells -- walls, ghosts,
  // inlet, outlet -- hold the zeros of fresh device memory, which lbm_get_macros returns for
  // them.  The reference reads h_uy[-1] for unstored cells (out of bounds); 0 is written there.
  {
    std::vector<int32_t> index(n);
    lbmh_index_transform(NX, NY, NZ, geo.data(), index.data());
    f.fetch(ctx);
    std::FILE* m = std::fopen("./meas1.txt", "w");
    const int z = NZ / 2;
    for (int pass = 0; pass < 2 && m; ++pass)
      for (int y = 0; y < NY; ++y)
        for (int x = 0; x < NX; ++x) {
          const size_t c = x + (size_t)NX * (y + (size_t)NY * z);
          const float v = index[c] >= 0 ? (pass == 0 ? f.uy[c] : f.ux[c]) : 0.0f;
          std::fprintf(m, "%g ", v);
        }
    if (m) std::fclose(m);
  }
  const float milli = timer.ms();
  std::printf("TOTAL RUNNING TIME: %g MILLI SECONDS#LATTICE%ld\n", milli, NLATTICE);
  std::fprintf(logfile, "TOTAL RUNNING TIME: %g MILLI SECONDS#LATTICE%ld ERROR IS%g\n", milli, NLATTICE, residual);
  std::fclose(logfile);
  lbm_destroy(ctx);
  return 0;
}
