// lbm_d3q19.hpp -- D3Q19 lattice definitions and the reference's exact equilibrium
// expression trees, shared by the HIP kernels and the host code of liblbm.
//
// Velocity set, weights and opposites as implied by the reference pull offsets
// (ldc.cu:76-182) and bounce-back swap (ldc.cu:184-201); see SURVEY.md Appendix A.
// Every arithmetic expression below reproduces the reference's fp32 evaluation
// order literally; the translation units are compiled with -ffp-contract=off so no
// multiply-add is fused (a 1e-6 relative-L2 match is below the FMA floor).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define LBM_HD __host__ __device__ __forceinline__
#else
#define LBM_HD inline
#endif

namespace lbm {

// e_q components; population q at cell c is pulled from c - e_q.
template <int Q> struct Dir;
#define LBM_DIR(Q_, X_, Y_, Z_, OPP_, W_)                                        \
  template <> struct Dir<Q_> {                                                    \
    static constexpr int x = X_, y = Y_, z = Z_, opp = OPP_, wdiv = W_;          \
  };
LBM_DIR(0, 0, 0, 0, 0, 3)
LBM_DIR(1, 1, 0, 0, 2, 18)
LBM_DIR(2, -1, 0, 0, 1, 18)
LBM_DIR(3, 0, 1, 0, 4, 18)
LBM_DIR(4, 0, -1, 0, 3, 18)
LBM_DIR(5, 0, 0, 1, 6, 18)
LBM_DIR(6, 0, 0, -1, 5, 18)
LBM_DIR(7, 1, 1, 0, 10, 36)
LBM_DIR(8, 1, -1, 0, 9, 36)
LBM_DIR(9, -1, 1, 0, 8, 36)
LBM_DIR(10, -1, -1, 0, 7, 36)
LBM_DIR(11, 1, 0, 1, 14, 36)
LBM_DIR(12, 1, 0, -1, 13, 36)
LBM_DIR(13, -1, 0, 1, 12, 36)
LBM_DIR(14, -1, 0, -1, 11, 36)
LBM_DIR(15, 0, 1, 1, 18, 36)
LBM_DIR(16, 0, -1, 1, 17, 36)
LBM_DIR(17, 0, 1, -1, 16, 36)
LBM_DIR(18, 0, -1, -1, 15, 36)
#undef LBM_DIR

// runtime tables for host code
constexpr int kEx[19] = {0, 1, -1, 0, 0, 0, 0, 1, 1, -1, -1, 1, 1, -1, -1, 0, 0, 0, 0};
constexpr int kEy[19] = {0, 0, 0, 1, -1, 0, 0, 1, -1, 1, -1, 0, 0, 0, 0, 1, -1, 1, -1};
constexpr int kEz[19] = {0, 0, 0, 0, 0, 1, -1, 0, 0, 0, 0, 1, -1, 1, -1, 1, 1, -1, -1};
constexpr int kOpp[19] = {0, 2, 1, 4, 3, 6, 5, 10, 9, 8, 7, 14, 13, 12, 11, 18, 17, 16, 15};

// Faces a boundary cell can supply populations through; population q crosses face n
// when e_q . n == 1 ("BC direction sets").
enum Face : int { kFacePX = 0, kFaceNX = 1, kFacePY = 2, kFaceNY = 3, kFacePZ = 4, kFaceNZ = 5 };
template <int Q>
constexpr int face_bits() {
  return (Dir<Q>::x == 1 ? 1 : 0) | (Dir<Q>::x == -1 ? 2 : 0) | (Dir<Q>::y == 1 ? 4 : 0) |
         (Dir<Q>::y == -1 ? 8 : 0) | (Dir<Q>::z == 1 ? 16 : 0) | (Dir<Q>::z == -1 ? 32 : 0);
}

// Cell-type byte.  bits 0-1 class; fluid: bit 2 has a wall neighbour, bit 3 an NEE neighbour
// supplying one of its populations -- the step kernel stores the bounce-back value / the NEE
// value into that neighbour's slot producer-side, from per-cell link masks; NEE boundary
// cell: bits 4-6 face, bit 7 kind (0 velocity, 1 pressure).
enum : uint8_t {
  kPassive = 0,   // ghost / unused / padding: never updated; pulled raw (constant) if kPulled
  kWall = 1,      // half-way bounce-back
  kNee = 2,       // non-equilibrium extrapolation boundary cell
  kFluid = 3,     // collide + stream
  kClassMask = 3,
  kWallAdj = 1u << 2,   // fluid with a wall neighbour
  kPulled = 1u << 2,    // passive cell a fluid cell pulls from (kept constant)
  kNeeAdj = 1u << 3,    // fluid with an NEE neighbour
  kKindPressure = 1u << 7,
};
LBM_HD int nee_face(uint8_t t) { return (t >> 4) & 7; }
LBM_HD uint8_t make_nee(int face, bool pressure) {
  return (uint8_t)(kNee | (face << 4) | (pressure ? kKindPressure : 0));
}

// f^eq_q in the form of the update kernels (ldc.cu:330-348, Poiseulle.cu:543-561,
// bifurcation.cu:587-624), one q at a time.  Expression trees and literal types are the
// reference's, including the fp64 "3.0*tmp_uz*tmp_uz" of q = 14 (ldc.cu:344).  Each is
// (tmp_rho / w_q) * P_q(u) with the quotient rounded first, as C evaluates the reference's
// "tmp_rho /36.0f * (...)"; feq_pre<Q> takes that quotient precomputed (the step kernels
// form it with an exact shortcut, see kernels), feq<Q> divides here.
template <int Q> struct FeqW;   // w_q's divisor: 3, 18 or 36
template <int Q>
LBM_HD auto feq_poly(float tmp_ux, float tmp_uy, float tmp_uz);
template <> struct FeqW<0> { static constexpr float d = 3.0f; };
template <> struct FeqW<1> { static constexpr float d = 18.0f; };
template <> struct FeqW<2> { static constexpr float d = 18.0f; };
template <> struct FeqW<3> { static constexpr float d = 18.0f; };
template <> struct FeqW<4> { static constexpr float d = 18.0f; };
template <> struct FeqW<5> { static constexpr float d = 18.0f; };
template <> struct FeqW<6> { static constexpr float d = 18.0f; };
template <> struct FeqW<7> { static constexpr float d = 36.0f; };
template <> struct FeqW<8> { static constexpr float d = 36.0f; };
template <> struct FeqW<9> { static constexpr float d = 36.0f; };
template <> struct FeqW<10> { static constexpr float d = 36.0f; };
template <> struct FeqW<11> { static constexpr float d = 36.0f; };
template <> struct FeqW<12> { static constexpr float d = 36.0f; };
template <> struct FeqW<13> { static constexpr float d = 36.0f; };
template <> struct FeqW<14> { static constexpr float d = 36.0f; };
template <> struct FeqW<15> { static constexpr float d = 36.0f; };
template <> struct FeqW<16> { static constexpr float d = 36.0f; };
template <> struct FeqW<17> { static constexpr float d = 36.0f; };
template <> struct FeqW<18> { static constexpr float d = 36.0f; };
template <> LBM_HD auto feq_poly<0>(float tmp_ux, float tmp_uy, float tmp_uz) {
  return (1.0f - 1.5f*tmp_ux*tmp_ux -1.5f* tmp_uy*tmp_uy -1.5f* tmp_uz*tmp_uz);
}
template <> LBM_HD auto feq_poly<1>(float tmp_ux, float tmp_uy, float tmp_uz) {
  return (1.0f + 3.0f* tmp_ux + 3.0f*tmp_ux*tmp_ux -1.5f* tmp_uy*tmp_uy -1.5f* tmp_uz*tmp_uz);
}
template <> LBM_HD auto feq_poly<2>(float tmp_ux, float tmp_uy, float tmp_uz) {
  return (1.0f - 3.0f* tmp_ux + 3.0f*tmp_ux*tmp_ux -1.5f* tmp_uy*tmp_uy -1.5f* tmp_uz*tmp_uz);
}
template <> LBM_HD auto feq_poly<3>(float tmp_ux, float tmp_uy, float tmp_uz) {
  return (1.0f + 3.0f* tmp_uy + 3.0f*tmp_uy*tmp_uy - 1.5f*tmp_ux*tmp_ux -1.5f* tmp_uz*tmp_uz);
}
template <> LBM_HD auto feq_poly<4>(float tmp_ux, float tmp_uy, float tmp_uz) {
  return (1.0f - 3.0f* tmp_uy + 3.0f*tmp_uy*tmp_uy - 1.5f*tmp_ux*tmp_ux -1.5f* tmp_uz*tmp_uz);
}
template <> LBM_HD auto feq_poly<5>(float tmp_ux, float tmp_uy, float tmp_uz) {
  return (1.0f + 3.0f* tmp_uz + 3.0f*tmp_uz*tmp_uz - 1.5f*tmp_ux*tmp_ux -1.5f* tmp_uy*tmp_uy);
}
template <> LBM_HD auto feq_poly<6>(float tmp_ux, float tmp_uy, float tmp_uz) {
  return (1.0f - 3.0f* tmp_uz + 3.0f*tmp_uz*tmp_uz - 1.5f*tmp_ux*tmp_ux -1.5f* tmp_uy*tmp_uy);
}
template <> LBM_HD auto feq_poly<7>(float tmp_ux, float tmp_uy, float tmp_uz) {
  return (1.0f + 3.0f* (tmp_ux + tmp_uy) + 3.0f*tmp_ux*tmp_ux + 3.0f*tmp_uy*tmp_uy + 9.0f*tmp_ux*tmp_uy -1.5f* tmp_uz*tmp_uz);
}
template <> LBM_HD auto feq_poly<8>(float tmp_ux, float tmp_uy, float tmp_uz) {
  return (1.0f + 3.0f* (tmp_ux - tmp_uy) + 3.0f*tmp_ux*tmp_ux + 3.0f*tmp_uy*tmp_uy - 9.0f*tmp_ux*tmp_uy-1.5f* tmp_uz*tmp_uz);
}
template <> LBM_HD auto feq_poly<9>(float tmp_ux, float tmp_uy, float tmp_uz) {
  return (1.0f + 3.0f* (tmp_uy - tmp_ux) + 3.0f* tmp_ux*tmp_ux + 3.0f*tmp_uy*tmp_uy - 9.0f*tmp_ux*tmp_uy-1.5f* tmp_uz*tmp_uz);
}
template <> LBM_HD auto feq_poly<10>(float tmp_ux, float tmp_uy, float tmp_uz) {
  return (1.0f - 3.0f* (tmp_ux + tmp_uy) + 3.0f*tmp_ux*tmp_ux + 3.0f*tmp_uy*tmp_uy + 9.0f*tmp_ux*tmp_uy-1.5f* tmp_uz*tmp_uz);
}
template <> LBM_HD auto feq_poly<11>(float tmp_ux, float tmp_uy, float tmp_uz) {
  return (1.0f + 3.0f* (tmp_ux + tmp_uz) + 3.0f* tmp_ux*tmp_ux + 3.0f*tmp_uz*tmp_uz + 9.0f*tmp_ux*tmp_uz-1.5f* tmp_uy*tmp_uy);
}
template <> LBM_HD auto feq_poly<12>(float tmp_ux, float tmp_uy, float tmp_uz) {
  return (1.0f + 3.0f* (tmp_ux - tmp_uz) + 3.0f* tmp_ux*tmp_ux + 3.0f*tmp_uz*tmp_uz - 9.0f*tmp_ux*tmp_uz-1.5f* tmp_uy*tmp_uy);
}
template <> LBM_HD auto feq_poly<13>(float tmp_ux, float tmp_uy, float tmp_uz) {
  return (1.0f + 3.0f* (tmp_uz - tmp_ux) + 3.0f* tmp_ux*tmp_ux + 3.0f*tmp_uz*tmp_uz - 9.0f*tmp_ux*tmp_uz-1.5f* tmp_uy*tmp_uy);
}
// the only fp64 sub-expression of the reference: "3.0*tmp_uz*tmp_uz" promotes the tail
template <> LBM_HD auto feq_poly<14>(float tmp_ux, float tmp_uy, float tmp_uz) {
  return (1.0f - 3.0f* (tmp_ux + tmp_uz) + 3.0f* tmp_ux*tmp_ux + 3.0*tmp_uz*tmp_uz + 9.0f*tmp_ux*tmp_uz -1.5f* tmp_uy*tmp_uy);
}
template <> LBM_HD auto feq_poly<15>(float tmp_ux, float tmp_uy, float tmp_uz) {
  return (1.0f + 3.0f* (tmp_uy + tmp_uz) + 3.0f* tmp_uy*tmp_uy + 3.0f*tmp_uz*tmp_uz + 9.0f*tmp_uy*tmp_uz- 1.5f*tmp_ux*tmp_ux);
}
template <> LBM_HD auto feq_poly<16>(float tmp_ux, float tmp_uy, float tmp_uz) {
  return (1.0f + 3.0f* (tmp_uz - tmp_uy) + 3.0f* tmp_uy*tmp_uy + 3.0f*tmp_uz*tmp_uz - 9.0f*tmp_uy*tmp_uz - 1.5f*tmp_ux*tmp_ux);
}
template <> LBM_HD auto feq_poly<17>(float tmp_ux, float tmp_uy, float tmp_uz) {
  return (1.0f + 3.0f* (tmp_uy - tmp_uz) + 3.0f* tmp_uy*tmp_uy + 3.0f*tmp_uz*tmp_uz - 9.0f*tmp_uy*tmp_uz - 1.5f*tmp_ux*tmp_ux);
}
template <> LBM_HD auto feq_poly<18>(float tmp_ux, float tmp_uy, float tmp_uz) {
  return (1.0f - 3.0f* (tmp_uy + tmp_uz) + 3.0f* tmp_uy*tmp_uy + 3.0f*tmp_uz*tmp_uz + 9.0f*tmp_uy*tmp_uz - 1.5f*tmp_ux*tmp_ux);
}
// pre = RN(tmp_rho / w_q); the product is formed in the poly's type (double for q = 14) and
// rounded to float once, as the reference's expression is
template <int Q>
LBM_HD float feq_pre(float pre, float tmp_ux, float tmp_uy, float tmp_uz) {
  return pre * feq_poly<Q>(tmp_ux, tmp_uy, tmp_uz);
}
template <int Q>
LBM_HD float feq(float tmp_rho, float tmp_ux, float tmp_uy, float tmp_uz) {
  return feq_pre<Q>(tmp_rho / FeqW<Q>::d, tmp_ux, tmp_uy, tmp_uz);
}

// Boundary-value equilibrium of the NEE boundaries.  The reference writes these as
// hand-simplified fp32 "tmp" terms (ldc.cu:402-454, Poiseulle.cu:748-891,
// bifurcation.cu:877-1021, coronary.cu:716-943): bit-identical to feq<Q> for every q they
// use, except q = 14 on a z face (coronary.cu:870-871), where the tmp term keeps fp32 while
// the update kernel's feq[14] has its fp64 sub-expression.
template <int Q>
LBM_HD float feq_bc(float r, float ux, float uy, float uz) {
  return feq<Q>(r, ux, uy, uz);
}
template <> LBM_HD float feq_bc<14>(float tmp_rho, float tmp_ux, float tmp_uy, float tmp_uz) {
  return tmp_rho /36.0f * (1.0f - 3.0f* (tmp_ux + tmp_uz) + 3.0f* tmp_ux*tmp_ux + 3.0f*tmp_uz*tmp_uz + 9.0f*tmp_ux*tmp_uz -1.5f* tmp_uy*tmp_uy);
}

// The LDC initialize() form (ldc.cu:542-571): all 19 at once.
LBM_HD void feq_init_wi(float tmp_rho, float tmp_ux, float tmp_uy, float tmp_uz, float* feq) {
  const float w0 = 1.0f / 3.0f, w1 = 1.0f / 18.0f, w2 = 1.0f / 36.0f;
  float ux2 = tmp_ux*tmp_ux, uy2 = tmp_uy*tmp_uy, uz2 = tmp_uz*tmp_uz;
  float uxyz2 = ux2 + uy2 + uz2, uxy2 = ux2 + uy2, uxz2 = ux2 + uz2, uyz2 = uy2 + uz2;
  float uxy = 2.0f*tmp_ux*tmp_uy, uxz = 2.0f*tmp_ux*tmp_uz, uyz = 2.0f*tmp_uy*tmp_uz;
  feq[0] = tmp_rho * w0 * (1.0f - 1.5f*uxyz2);
  feq[1] = tmp_rho * w1 * (1.0f + 3.0f* tmp_ux + 4.5f*ux2 - 1.5f*uxyz2);
  feq[2] = tmp_rho * w1 * (1.0f - 3.0f* tmp_ux + 4.5f*ux2 - 1.5f*uxyz2);
  feq[3] = tmp_rho * w1 * (1.0f + 3.0f* tmp_uy + 4.5f*uy2 - 1.5f*uxyz2);
  feq[4] = tmp_rho * w1 * (1.0f - 3.0f* tmp_uy + 4.5f*uy2 - 1.5f*uxyz2);
  feq[5] = tmp_rho * w1 * (1.0f + 3.0f* tmp_uz + 4.5f*uz2 - 1.5f*uxyz2);
  feq[6] = tmp_rho * w1 * (1.0f - 3.0f* tmp_uz + 4.5f*uz2 - 1.5f*uxyz2);
  feq[7] = tmp_rho * w2 * (1.0f + 3.0f* (tmp_ux + tmp_uy) + 4.5f* (uxy2 + uxy) - 1.5f*uxyz2);
  feq[8] = tmp_rho * w2 * (1.0f + 3.0f* (tmp_ux - tmp_uy) + 4.5f* (uxy2 - uxy) - 1.5f* uxyz2);
  feq[9] = tmp_rho * w2 * (1.0f + 3.0f* (tmp_uy - tmp_ux) + 4.5f* (uxy2 - uxy) - 1.5f* uxyz2);
  feq[10] = tmp_rho * w2 * (1.0f - 3.0f* (tmp_ux + tmp_uy) + 4.5f* (uxy2 + uxy) - 1.5f* uxyz2);
  feq[11] = tmp_rho * w2 * (1.0f + 3.0f* (tmp_ux + tmp_uz) + 4.5f* (uxz2 + uxz) - 1.5f* uxyz2);
  feq[12] = tmp_rho * w2 * (1.0f + 3.0f* (tmp_ux - tmp_uz) + 4.5f* (uxz2 - uxz) - 1.5f* uxyz2);
  feq[13] = tmp_rho * w2 * (1.0f + 3.0f* (tmp_uz - tmp_ux) + 4.5f* (uxz2 - uxz) - 1.5f* uxyz2);
  feq[14] = tmp_rho * w2 * (1.0f - 3.0f* (tmp_ux + tmp_uz) + 4.5f* (uxz2 + uxz) - 1.5f* uxyz2);
  feq[15] = tmp_rho * w2 * (1.0f + 3.0f* (tmp_uy + tmp_uz) + 4.5f* (uyz2 + uyz) - 1.5f* uxyz2);
  feq[16] = tmp_rho * w2 * (1.0f + 3.0f* (tmp_uz - tmp_uy) + 4.5f* (uyz2 - uyz) - 1.5f* uxyz2);
  feq[17] = tmp_rho * w2 * (1.0f + 3.0f* (tmp_uy - tmp_uz) + 4.5f* (uyz2 - uyz) - 1.5f* uxyz2);
  feq[18] = tmp_rho * w2 * (1.0f - 3.0f* (tmp_uy + tmp_uz) + 4.5f* (uyz2 + uyz) - 1.5f* uxyz2);
}

// The expanded form used by Poiseuille/bifurcation initialize(): identical to the update form.
LBM_HD void feq_expanded(float r, float ux, float uy, float uz, float* f) {
  f[0] = feq<0>(r, ux, uy, uz);   f[1] = feq<1>(r, ux, uy, uz);   f[2] = feq<2>(r, ux, uy, uz);
  f[3] = feq<3>(r, ux, uy, uz);   f[4] = feq<4>(r, ux, uy, uz);   f[5] = feq<5>(r, ux, uy, uz);
  f[6] = feq<6>(r, ux, uy, uz);   f[7] = feq<7>(r, ux, uy, uz);   f[8] = feq<8>(r, ux, uy, uz);
  f[9] = feq<9>(r, ux, uy, uz);   f[10] = feq<10>(r, ux, uy, uz); f[11] = feq<11>(r, ux, uy, uz);
  f[12] = feq<12>(r, ux, uy, uz); f[13] = feq<13>(r, ux, uy, uz); f[14] = feq<14>(r, ux, uy, uz);
  f[15] = feq<15>(r, ux, uy, uz); f[16] = feq<16>(r, ux, uy, uz); f[17] = feq<17>(r, ux, uy, uz);
  f[18] = feq<18>(r, ux, uy, uz);
}

}  // namespace lbm
