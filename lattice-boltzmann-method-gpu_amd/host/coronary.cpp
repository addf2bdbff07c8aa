// coronary -- drop-in for coronary_cfd/coronary.cu (main 1055-1163): a 291 x 291 x 372 vessel
// mask from ./geo.txt (read in z, x, y order), geo_pre with the reference's five open ends
// (inlet x = 3, main exit x = 272, sub-exits z = 185 / 191 / 204), its boundary scheme as
// LBM_CASE_GENERIC codes (inlet +x velocity with rho 1, outlets velocity NEE), tau 0.55,
// REPEAT = 300000 (300001 steps), host residual (calc_res) and coronary_<i>.vtk (density,
// pressure, velocity) at i % 5000 == 0.
// Overrides: --geo PATH --repeat N --time-save N --out DIR --device N
//            --nx N --ny N --nz N --ends "axis,plane,lo0,hi0,lo1,hi1,passes;..." (another box and its
//            own end table, lbmh_end; the reference's table needs a box of at least 274 x 201 x 206)
#include "driver_common.hpp"

#include <sstream>

namespace {

std::vector<lbmh_end> parse_ends(const std::string& s) {
  std::vector<lbmh_end> out;
  std::stringstream all(s);
  std::string one;
  while (std::getline(all, one, ';')) {
    lbmh_end e{};
    if (std::sscanf(one.c_str(), "%d,%d,%d,%d,%d,%d,%d", &e.axis, &e.plane, &e.lo0, &e.hi0, &e.lo1, &e.hi1,
                    &e.passes) == 7)
      out.push_back(e);
  }
  return out;
}

}  // namespace

int main(int argc, char** argv) {
  drv::Args args(argc, argv);
  const int NX = args.geti("--nx", 291), NY = args.geti("--ny", 291), NZ = args.geti("--nz", 372);  // coronary.cu:19
  const int REPEAT = args.geti("--repeat", 300000), time_save = args.geti("--time-save", 5000);
  const float C_U = 2.74909090909091f, CH = 6.1111e-05f, C_rho = 1060.f, tau = 0.55f;  // coronary.cu:20, 357
  const std::string out = args.get("--out", "./out");
  drv::ensure_dir(out);
  std::FILE* logfile = std::fopen((out + "/CONVERGENCE.log").c_str(), "w");

  const size_t n = (size_t)NX * NY * NZ;
  std::vector<int32_t> raw(n);
  const std::string geo_path = args.get("--geo", "./geo.txt");
  if (lbmh_read_geo_txt_zxy(geo_path.c_str(), NX, NY, NZ, raw.data()) != (long)n) {
    std::fprintf(stderr, "cannot read %s\n", geo_path.c_str());
    return 1;
  }
  std::vector<lbmh_end> ends(5);
  if (args.has("--ends")) {
    ends = parse_ends(args.get("--ends", ""));
    if (ends.empty()) {
      std::fprintf(stderr, "--ends: no \"axis,plane,lo0,hi0,lo1,hi1,passes\" entries\n");
      return 1;
    }
  } else if (lbmh_coronary_ends(NX, NY, NZ, ends.data()) != 5) {
    std::fprintf(stderr, "a %dx%dx%d box cannot hold coronary.cu's end planes: give --ends\n", NX, NY, NZ);
    return 1;
  }
  std::vector<int8_t> geo(n);
  if (lbmh_geo_ends(NX, NY, NZ, raw.data(), (int)ends.size(), ends.data(), geo.data()) != 0) {
    std::fprintf(stderr, "invalid end table for a %dx%dx%d box\n", NX, NY, NZ);
    return 1;
  }
  raw.clear();
  raw.shrink_to_fit();
  const long NLATTICE = (long)lbmh_index_transform(NX, NY, NZ, geo.data(), nullptr);
  drv::Fields f(n);
  lbmh_initial_fields(3, NX, NY, NZ, geo.data(), nullptr, nullptr, f.rho.data(), f.ux.data(), f.uy.data(),
                      f.uz.data());

  // boundary_stream's codes (coronary.cu:716-943): the velocities are double quotients there
  const float uin = (float)(0.1745 / (double)C_U), uout = (float)(0.1 / (double)C_U),
              uexit = (float)(0.02 / (double)C_U);
  lbm_bc_code bcs[5] = {
      {2, LBM_FACE_PX, LBM_BC_VELOCITY_RHO, 1.0f, {uin, 0.0f, 0.0f}, nullptr},
      {3, LBM_FACE_NX, LBM_BC_VELOCITY, 1.0f, {uout, 0.0f, 0.0f}, nullptr},
      {5, LBM_FACE_NZ, LBM_BC_VELOCITY, 1.0f, {0.0f, 0.0f, uexit}, nullptr},
      {6, LBM_FACE_NZ, LBM_BC_VELOCITY, 1.0f, {0.0f, 0.0f, uexit}, nullptr},
      {7, LBM_FACE_NZ, LBM_BC_VELOCITY, 1.0f, {0.0f, 0.0f, uexit}, nullptr},
  };
  lbm_desc d{};
  d.nx = NX; d.ny = NY; d.nz = NZ; d.tau = tau; d.case_kind = LBM_CASE_GENERIC; d.geo = geo.data();
  d.device = args.geti("--device", 0); d.nz_global = NZ; d.bc_codes = bcs; d.n_bc_codes = 5;
  lbm_ctx* ctx = nullptr;
  drv::check(lbm_create(&d, &ctx), nullptr, "lbm_create");
  drv::check(lbm_init_equilibrium(ctx, LBM_INIT_EXPANDED, f.rho.data(), f.ux.data(), f.uy.data(), f.uz.data()), ctx,
             "lbm_init_equilibrium");
  // host copies start as initialize()'s fields (calc_res at i = 0 reads them: coronary.cu:1114)
  drv::Timer timer;
  float residual = 0.0f;
  long double sum1 = 0.0L, sum2 = 0.0L;
  for (int i = 0; i <= REPEAT;) {
    int next = (i + time_save - 1) / time_save * time_save;  // the next save step (or the end)
    if (next > REPEAT) next = REPEAT;
    const int count = next - i + 1;
    drv::check(lbm_step(ctx, count, nullptr, nullptr), ctx, "lbm_step");
    i += count;
    const int last = i - 1;
    if (last % time_save == 0) {
      sum1 = lbmh_calc_res_fluid(NX, NY, NZ, geo.data(), f.ux.data(), f.uy.data(), f.uz.data());
      f.fetch(ctx);
      const float milli = timer.ms();
      sum2 = lbmh_calc_res_fluid(NX, NY, NZ, geo.data(), f.ux.data(), f.uy.data(), f.uz.data());
      residual = (float)(std::fabs(sum1 - sum2) / sum2);  // long double, then float (coronary.cu:1126)
      std::fprintf(logfile, "%g\n", residual);
      std::printf("ITERATION # %d, collapse time: %g ms, residual:%g\n", last, milli, residual);
      lbmh_write_vtk_coronary((out + "/coronary_" + std::to_string(last) + ".vtk").c_str(), NX, NY, NZ, geo.data(),
                              f.rho.data(), f.ux.data(), f.uy.data(), f.uz.data(), C_U, CH, C_rho);
    }
  }
  const float milli = timer.ms();
  std::printf("TOTAL RUNNING TIME: %g MILLI SECONDS#LATTICE%ld\n", milli, NLATTICE);
  std::fprintf(logfile, "TOTAL RUNNING TIME: %g MILLI SECONDS#LATTICE%ld ERROR IS%g\n", milli, NLATTICE, residual);
  std::fclose(logfile);
  lbm_destroy(ctx);
  return 0;
}
