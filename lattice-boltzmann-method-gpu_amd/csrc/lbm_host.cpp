// lbm_host.cpp -- liblbm_host.so: host ingest / initial fields / output of the three
// reference cases (the non-kernel half of ldc.cu, Poiseulle.cu and bifurcation.cu).
// Compiled with -ffp-contract=off so the float expressions of the reference host code
// (profile parabola, initial velocities) round exactly as the reference's do.
#include "../../include/lbm_host.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

namespace {

struct Box {
  int nx, ny, nz;
  int64_t operator()(int x, int y, int z) const {
    return (int64_t)x + (int64_t)nx * ((int64_t)y + (int64_t)ny * z);
  }
  int64_t size() const { return (int64_t)nx * ny * nz; }
};

constexpr int kEx[19] = {0, 1, -1, 0, 0, 0, 0, 1, 1, -1, -1, 1, 1, -1, -1, 0, 0, 0, 0};
constexpr int kEy[19] = {0, 0, 0, 1, -1, 0, 0, 1, -1, 1, -1, 0, 0, 0, 0, 1, -1, 1, -1};
constexpr int kEz[19] = {0, 0, 0, 0, 0, 1, -1, 0, 0, 0, 0, 1, -1, 1, -1, 1, 1, -1, -1};

// min over the 6 face neighbours of a 0/1 flag (the "distance transform" of geo_pre)
template <class F>
int min6(const F& flag, const Box& b, int x, int y, int z) {
  return std::min({flag[b(x + 1, y, z)], flag[b(x - 1, y, z)], flag[b(x, y - 1, z)], flag[b(x, y + 1, z)],
                   flag[b(x, y, z - 1)], flag[b(x, y, z + 1)]});
}
template <class F>
int min4_xz(const F& flag, const Box& b, int x, int y, int z) {
  return std::min({flag[b(x + 1, y, z)], flag[b(x - 1, y, z)], flag[b(x, y, z - 1)], flag[b(x, y, z + 1)]});
}

// ghost marking: unused (0) 18-neighbours of a source cell become -1
// (Poiseulle.cu:138-254 sources {1,2,3}; bifurcation.cu:122-239 sources {1})
void mark_ghosts(const Box& b, std::vector<int>& g, bool walls_only) {
  for (int z = 1; z < b.nz - 1; ++z)
    for (int y = 1; y < b.ny - 1; ++y)
      for (int x = 1; x < b.nx - 1; ++x) {
        const int v = g[b(x, y, z)];
        const bool src = walls_only ? (v == 1) : (v >= 1 && v <= 3);
        if (!src) continue;
        for (int q = 1; q < 19; ++q) {
          int& n = g[b(x + kEx[q], y + kEy[q], z + kEz[q])];
          if (n == 0) n = -1;
        }
      }
}

}  // namespace

extern "C" {

void lbmh_geo_ldc(int nx, int ny, int nz, int8_t* geo) {
  const Box b{nx, ny, nz};
  for (int z = 0; z < nz; ++z)
    for (int y = 0; y < ny; ++y)
      for (int x = 0; x < nx; ++x) {
        int8_t v = 0;                                                                            // ghost
        if (x >= 1 && x <= nx - 2 && y >= 1 && y <= ny - 2 && z >= 1 && z <= nz - 2) v = 1;     // wall
        if (x >= 2 && x <= nx - 3 && y >= 2 && y <= ny - 3 && z >= 2 && z <= nz - 3) v = 3;     // fluid
        if (y == ny - 2 && x >= 1 && x <= nx - 2 && z >= 1 && z <= nz - 2) v = 2;              // lid
        geo[b(x, y, z)] = v;
      }
}

void lbmh_geo_poiseuille(int nx, int ny, int nz, int8_t* geo) {
  const Box b{nx, ny, nz};
  std::vector<int> flag(b.size(), 0), g(b.size(), 0);
  const float radius = (nx - 1) / 2.0f;
  const float cx = (nx - 1) / 2.0f, cz = (nz - 1) / 2.0f;
  for (int z = 0; z < nz; ++z)
    for (int y = 1; y < ny - 1; ++y)
      for (int x = 0; x < nx; ++x) {
        const float dx = x - cx, dz = z - cz;
        const float dist = std::sqrt(dx * dx + dz * dz);  // sqrt(powf(.,2)+powf(.,2)), float
        if (dist <= radius) flag[b(x, y, z)] = g[b(x, y, z)] = 1;
      }
  // fluid: three increments of the 6-neighbour minimum of the (unchanged) flag
  for (int z = 1; z < nz - 1; ++z)
    for (int y = 2; y < ny - 2; ++y)
      for (int x = 1; x < nx - 1; ++x) g[b(x, y, z)] += 3 * min6(flag, b, x, y, z);
  // inlet (y = 1): one increment of the in-plane minimum; outlet (y = ny-2): two
  for (int z = 1; z < nz - 1; ++z)
    for (int x = 1; x < nx - 1; ++x) {
      g[b(x, 1, z)] += min4_xz(flag, b, x, 1, z);
      g[b(x, ny - 2, z)] += 2 * min4_xz(flag, b, x, ny - 2, z);
    }
  mark_ghosts(b, g, false);
  for (int64_t c = 0; c < b.size(); ++c) geo[c] = (int8_t)g[c];
}

long lbmh_read_geo_txt(const char* path, int nx, int ny, int nz, int32_t* raw) {
  FILE* f = std::fopen(path, "r");
  if (!f) return -1;
  const long n = (long)nx * ny * nz;
  long i = 0;
  int v;
  while (i < n && std::fscanf(f, "%d ", &v) == 1) raw[i++] = v;
  std::fclose(f);
  return i;
}

void lbmh_geo_mask(int nx, int ny, int nz, const int32_t* raw, int8_t* geo) {
  const Box b{nx, ny, nz};
  std::vector<int> g(raw, raw + b.size());
  for (int z = 1; z < nz - 1; ++z)
    for (int x = 1; x < nx - 1; ++x) g[b(x, 0, z)] = g[b(x, ny - 1, z)] = 0;
  for (int z = 1; z < nz - 1; ++z)
    for (int y = 2; y < ny - 2; ++y)
      for (int x = 1; x < nx - 1; ++x) g[b(x, y, z)] += 3 * min6(raw, b, x, y, z);
  for (int z = 1; z < nz - 1; ++z)
    for (int x = 1; x < nx - 1; ++x) {
      const int in = g[b(x, 2, z)], out = g[b(x, ny - 3, z)];
      g[b(x, 1, z)] = in == 1 ? 1 : (in == 4 ? 2 : 0);
      g[b(x, ny - 2, z)] = out == 1 ? 1 : (out == 4 ? 3 : 0);
    }
  mark_ghosts(b, g, true);
  for (int64_t c = 0; c < b.size(); ++c) geo[c] = (int8_t)g[c];
}

long lbmh_read_geo_txt_zxy(const char* path, int nx, int ny, int nz, int32_t* raw) {
  FILE* f = std::fopen(path, "r");
  if (!f) return -1;
  const Box b{nx, ny, nz};
  long i = 0;
  int v;
  for (int z = 0; z < nz; ++z)
    for (int x = 0; x < nx; ++x)
      for (int y = 0; y < ny; ++y) {
        if (std::fscanf(f, "%d ", &v) != 1) {
          std::fclose(f);
          return i;
        }
        raw[b(x, y, z)] = v;
        ++i;
      }
  std::fclose(f);
  return i;
}

int lbmh_geo_ends(int nx, int ny, int nz, const int32_t* raw, int n_ends, const lbmh_end* ends, int8_t* geo) {
  const Box b{nx, ny, nz};
  if (nx < 3 || ny < 3 || nz < 3 || n_ends < 0 || (n_ends > 0 && !ends)) return -1;
  for (int e = 0; e < n_ends; ++e) {  // every cell of an end needs its four in-plane neighbours
    const lbmh_end& E = ends[e];
    const int n0 = E.axis == 0 ? ny : nx, n1 = E.axis == 0 ? nz : ny, np = E.axis == 0 ? nx : nz;
    if ((E.axis != 0 && E.axis != 2) || E.plane < 1 || E.plane > np - 2 || E.lo0 < 1 || E.hi0 > n0 - 1 ||
        E.lo1 < 1 || E.hi1 > n1 - 1 || E.passes < 0 || 1 + E.passes > 127)
      return -1;
  }
  std::vector<int> g(raw, raw + b.size());
  // fluid: three increments of the 6-neighbour minimum of the (unchanged) raw mask
  for (int z = 1; z < nz - 1; ++z)
    for (int y = 1; y < ny - 1; ++y)
      for (int x = 1; x < nx - 1; ++x) g[b(x, y, z)] += 3 * min6(raw, b, x, y, z);
  // ends: in-plane 4-neighbour minimum, `passes` times; increments commute, so ends that
  // share cells (an x plane crossing a z plane) add up as the reference's sequence does
  for (int e = 0; e < n_ends; ++e) {
    const lbmh_end& E = ends[e];
    for (int s1 = E.lo1; s1 < E.hi1; ++s1)
      for (int s0 = E.lo0; s0 < E.hi0; ++s0) {
        int x, y, z, m;
        if (E.axis == 0) {
          x = E.plane; y = s0; z = s1;
          m = std::min({raw[b(x, y - 1, z)], raw[b(x, y + 1, z)], raw[b(x, y, z - 1)], raw[b(x, y, z + 1)]});
        } else {
          x = s0; y = s1; z = E.plane;
          m = std::min({raw[b(x, y - 1, z)], raw[b(x, y + 1, z)], raw[b(x - 1, y, z)], raw[b(x + 1, y, z)]});
        }
        g[b(x, y, z)] += E.passes * m;
      }
  }
  mark_ghosts(b, g, true);
  for (int64_t c = 0; c < b.size(); ++c) geo[c] = (int8_t)g[c];
  return 0;
}

int lbmh_coronary_ends(int nx, int ny, int nz, lbmh_end* ends) {
  // the windows of coronary.cu:75-143; they need x up to 273, y up to 200 and z up to 205
  if (nx < 274 || ny < 201 || nz < 206) return -1;
  ends[0] = lbmh_end{0, 3, 1, ny - 1, 1, nz - 1, 1};      // inlet end = 2
  ends[1] = lbmh_end{0, 272, 1, ny - 1, 1, nz - 1, 2};    // main exit end = 3
  ends[2] = lbmh_end{2, 185, 217, 237, 113, 138, 4};      // sub exit 1 = 5 (x 217..236, y 113..137)
  ends[3] = lbmh_end{2, 191, 160, 206, 159, 200, 5};      // sub exit 2 = 6 (x 160..205, y 159..199)
  ends[4] = lbmh_end{2, 204, 1, nx - 1, 1, ny - 1, 6};    // sub exit 3 = 7 (whole plane)
  return 5;
}

long lbmh_read_bc_txt(const char* path, int nx, int ny, int nz, const int8_t* geo, int inlet_block,
                      float* inlet_uy, float* outlet_uy) {
  FILE* f = std::fopen(path, "r");
  if (!f) return -1;
  const Box b{nx, ny, nz};
  long ntok = 0;
  float v;
  auto next = [&](float& out) {
    if (std::fscanf(f, "%f ", &out) == 1) { ++ntok; return true; }
    out = 0.0f;
    return false;
  };
  for (long s = 0; s < (long)inlet_block * nx * nz; ++s) next(v);
  for (int z = 0; z < nz; ++z)
    for (int x = 0; x < nx; ++x) {
      next(v);
      inlet_uy[x + (int64_t)z * nx] = (!geo || geo[b(x, 1, z)] == 2) ? v : 0.0f;
    }
  for (int z = 0; z < nz; ++z)
    for (int x = 0; x < nx; ++x) {
      next(v);
      outlet_uy[x + (int64_t)z * nx] = (!geo || geo[b(x, ny - 2, z)] == 3) ? v : 0.0f;
    }
  std::fclose(f);
  return ntok;
}

int64_t lbmh_index_transform(int nx, int ny, int nz, const int8_t* geo, int32_t* index) {
  const int64_t n = (int64_t)nx * ny * nz;
  int64_t k = 0;
  for (int64_t c = 0; c < n; ++c) {
    const int32_t v = geo[c] != 0 ? (int32_t)k : -1;
    if (index) index[c] = v;
    if (geo[c] != 0) ++k;
  }
  return k;
}

void lbmh_poiseuille_profile(int nx, int nz, float u_max, float* table) {
  const float c = (nx - 1) / 2.0f, cz = (nz - 1) / 2.0f;
  for (int k = 0; k < nz; ++k)
    for (int i = 0; i < nx; ++i) {
      const float dx = i - c, dz = k - cz;
      table[i + (int64_t)k * nx] = u_max * (1.0f - (dx * dx + dz * dz) / (c * c));
    }
}

void lbmh_initial_fields(int case_kind, int nx, int ny, int nz, const int8_t* geo, const float* inlet_uy,
                         const float* outlet_uy, float* rho, float* ux, float* uy, float* uz) {
  const Box b{nx, ny, nz};
  const int64_t n = b.size();
  std::fill(rho, rho + n, 1.0f);
  std::fill(ux, ux + n, 0.0f);
  std::fill(uy, uy + n, 0.0f);
  std::fill(uz, uz + n, 0.0f);
  if (case_kind == 0) {
    const float u_max = 0.15f / 2.4705f;  // ldc.cu:49,52
    for (int z = 0; z < nz; ++z)
      for (int x = 0; x < nx; ++x) uz[b(x, ny - 1, z)] = uz[b(x, ny - 2, z)] = u_max;
  } else if (case_kind == 1) {
    const float u_max = 0.15f / 1.5441f;  // Poiseulle.cu:39,44
    std::vector<float> prof((size_t)nx * nz);
    const float c = (nx - 1) / 2.0f, cz = (nz - 1) / 2.0f, r = (nx - 1) / 2.0f;
    for (int z = 0; z < nz; ++z)
      for (int x = 0; x < nx; ++x) {
        const float dx = x - c, dz = z - cz;
        prof[x + (size_t)z * nx] = u_max * (1.0f - (dx * dx + dz * dz) / (r * r));
      }
    for (int y : {0, 1, ny - 1, ny - 2})
      for (int z = 0; z < nz; ++z)
        for (int x = 0; x < nx; ++x)
          if (geo[b(x, y, z)] != 0) uy[b(x, y, z)] = prof[x + (size_t)z * nx];
  } else if (case_kind == 3) {
    const float C_U = 2.74909090909091f;  // coronary.cu:20, 298-307 (float quotients)
    for (int64_t c = 0; c < n; ++c) {
      if (geo[c] == 2) ux[c] = 0.1745f / C_U;
      if (geo[c] == 3) ux[c] = 0.1f / C_U;
      if (geo[c] >= 5 && geo[c] <= 7) uz[c] = 0.02f / C_U;
    }
  } else {
    for (int z = 0; z < nz; ++z)
      for (int x = 0; x < nx; ++x) {
        if (geo[b(x, 1, z)] != 0) uy[b(x, 1, z)] = inlet_uy ? inlet_uy[x + (int64_t)z * nx] : 0.0f;
        if (geo[b(x, ny - 2, z)] != 0) uy[b(x, ny - 2, z)] = outlet_uy ? outlet_uy[x + (int64_t)z * nx] : 0.0f;
      }
  }
}

int lbmh_write_vtk(const char* path, int case_kind, int nx, int ny, int nz, const int8_t* geo,
                   const float* ux, const float* uy, const float* uz, float C_U, float CH) {
  std::ofstream ofs(path);
  if (!ofs) return -1;
  const Box b{nx, ny, nz};
  ofs << "# vtk DataFile Version 2.0" << std::endl;
  ofs << "<-- LBM flow with UIV acceleration, http://www.bg.ic.ac.uk/research/m.tang/ulis/ -->" << std::endl;
  ofs << "ASCII" << std::endl;
  ofs << "DATASET STRUCTURED_POINTS" << std::endl;
  if (case_kind == 0) {  // ldc.cu:592-607
    ofs << "DIMENSIONS " << nx - 4 << ' ' << ny - 4 << ' ' << nz - 4 << std::endl;
    ofs << "SPACING " << CH << ' ' << CH << ' ' << CH << std::endl;
    ofs << "ORIGIN " << std::round(nx / 2 - 1) * CH << ' ' << std::round(ny / 2 - 1) * CH << ' ' << .0 << std::endl;
    ofs << "POINT_DATA  " << (nx - 4) * (ny - 4) * (nz - 4) << std::endl;
    ofs << "VECTORS VELOCITY float" << std::endl;
    for (int z = 2; z < nz - 2; ++z)
      for (int y = 2; y < ny - 2; ++y)
        for (int x = 2; x < nx - 2; ++x) {
          const int64_t c = b(x, y, z);
          ofs << ux[c] * C_U << " ";
          ofs << uy[c] * C_U << " ";
          ofs << uz[c] * C_U << " ";
        }
  } else {  // Poiseulle.cu:913-935, bifurcation.cu:1101-1153
    ofs << "DIMENSIONS " << nx - 2 << ' ' << ny - 4 << ' ' << nz - 2 << std::endl;
    ofs << "SPACING " << CH << ' ' << CH << ' ' << CH << std::endl;
    ofs << "ORIGIN " << std::round(nx / 2) * CH << ' ' << std::round(ny / 2) * CH << ' ' << .0 << std::endl;
    ofs << "POINT_DATA  " << (nx - 2) * (ny - 4) * (nz - 2) << std::endl;
    ofs << "VECTORS VELOCITY float" << std::endl;
    for (int z = 1; z < nz - 1; ++z)
      for (int y = 2; y < ny - 2; ++y)
        for (int x = 1; x < nx - 1; ++x) {
          const int64_t c = b(x, y, z);
          if (geo[c] != 0) {
            ofs << ux[c] * C_U << ' ';
            ofs << uy[c] * C_U << ' ';
            ofs << uz[c] * C_U << ' ';
          } else {
            ofs << 0.0f << ' ';
            ofs << 0.0f << ' ';
            ofs << 0.0f << ' ';
          }
        }
  }
  return ofs.good() ? 0 : -2;
}

int lbmh_write_vtk_coronary(const char* path, int nx, int ny, int nz, const int8_t* geo, const float* rho,
                            const float* ux, const float* uy, const float* uz, float C_U, float CH, float C_rho) {
  std::ofstream ofs(path);
  if (!ofs) return -1;
  const Box b{nx, ny, nz};
  const float C_pre = C_rho * C_U * C_U;  // coronary.cu:26
  ofs << "# vtk DataFile Version 2.0" << std::endl;
  ofs << "<-- LBM flow with UIV acceleration, http://www.bg.ic.ac.uk/research/m.tang/ulis/ -->" << std::endl;
  ofs << "ASCII" << std::endl;
  ofs << "DATASET STRUCTURED_POINTS" << std::endl;
  ofs << "DIMENSIONS " << nx - 2 << ' ' << ny - 4 << ' ' << nz - 2 << std::endl;
  ofs << "SPACING " << CH << ' ' << CH << ' ' << CH << std::endl;
  ofs << "ORIGIN " << std::round(nx / 2) * CH << ' ' << std::round(ny / 2) * CH << ' ' << .0 << std::endl;
  ofs << "POINT_DATA  " << (nx - 2) * (ny - 4) * (nz - 2) << std::endl;
  // one scalar section per quantity, region x in [1, nx-2], y in [2, ny-3], z in [1, nz-2]
  auto region = [&](auto&& cell) {
    for (int z = 1; z < nz - 1; ++z)
      for (int y = 2; y < ny - 2; ++y)
        for (int x = 1; x < nx - 1; ++x) cell(b(x, y, z));
  };
  ofs << "SCALARS DENSITY float" << std::endl;
  ofs << "LOOKUP_TABLE default" << std::endl;
  region([&](int64_t c) {
    if (geo[c] != 0) ofs << rho[c] * C_rho << ' ';
    else ofs << 0.0f << ' ';
  });
  ofs << std::endl;
  ofs << "SCALARS PRESSURE float" << std::endl;
  ofs << "LOOKUP_TABLE default" << std::endl;
  region([&](int64_t c) {
    if (geo[c] != 0) ofs << rho[c] * C_pre / 3.0 << ' ';
    else ofs << 0.0f << ' ';
  });
  ofs << std::endl;
  ofs << "VECTORS VELOCITY float" << std::endl;
  region([&](int64_t c) {
    if (geo[c] != 0) {
      ofs << ux[c] * C_U << ' ';
      ofs << uy[c] * C_U << ' ';
      ofs << uz[c] * C_U << ' ';
    } else {
      ofs << 0 << ' ';
      ofs << 0 << ' ';
      ofs << 0 << ' ';
    }
  });
  return ofs.good() ? 0 : -2;
}

static long double calc_res_codes(int nx, int ny, int nz, const int8_t* geo, const float* ux, const float* uy,
                                  const float* uz, int lo, int hi) {
  const Box b{nx, ny, nz};
  long double s = 0.0L;
  for (int z = 1; z < nz - 1; ++z)
    for (int y = 2; y < ny - 2; ++y)
      for (int x = 1; x < nx - 1; ++x) {
        const int64_t c = b(x, y, z);
        if (geo[c] >= lo && geo[c] <= hi) {
          const float v = ux[c] * ux[c] + uy[c] * uy[c] + uz[c] * uz[c];
          s = s + v;
        }
      }
  return s;
}

long double lbmh_calc_res(int nx, int ny, int nz, const int8_t* geo, const float* ux, const float* uy,
                          const float* uz) {
  return calc_res_codes(nx, ny, nz, geo, ux, uy, uz, 4, 127);
}

long double lbmh_calc_res_fluid(int nx, int ny, int nz, const int8_t* geo, const float* ux, const float* uy,
                                const float* uz) {
  return calc_res_codes(nx, ny, nz, geo, ux, uy, uz, 4, 4);
}

}  // extern "C"
