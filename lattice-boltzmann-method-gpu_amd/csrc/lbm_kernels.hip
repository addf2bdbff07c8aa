// lbm_kernels.hip -- CDNA4 (gfx950) kernels of the D3Q19 BGK hot path.
//
// The reference's per-step kernels update + boundary_stream + calc_vel_square
// (ldc.cu:57-466, Poiseulle.cu:384-901, bifurcation.cu:429-1023) become one launch of
// k_step per launch range plus the reduction:
//
//  k_step            one wavefront per 256-cell AoSoA chunk, 4 consecutive cells per lane
//                    (or, on small lattices, per 64-cell quarter chunk, one cell per lane):
//                    19 aligned 16-B pulls issued at once (x neighbours by a DPP lane shift,
//                    the edge lanes' floats by vector loads that often hit L1), moments,
//                    equilibria and BGK relaxation in registers, 19 16-B stores into the
//                    chunk.  Boundaries cost no extra pass and no extra round trip: the one
//                    cell that pulls a boundary slot next step stores its value producer side
//                    --
//                      wall W = c - e_q:  slot q of W = c's post-collision f_opp(q)
//                        (the value Poiseulle.cu:601-746 / ldc.cu:184-201 write there);
//                      NEE cell B = c - e_q with e_q . n_B = 1:  slot q of B =
//                        feq_q(rho_bc, u_bc) + (f'_q(c) - feq_q(rho_c, u_c)) (1 - 1/tau)
//                        with c's post-collision f'_q and (rho, u) of this step (the value
//                        boundary_stream writes into B, ldc.cu:391-456, Poiseulle.cu:748-891,
//                        bifurcation.cu:877-1021; their hand-simplified "tmp" terms are
//                        bit-identical to feq_q(rho_bc, u_bc)) --
//                    so every pull is a plain load and every fluid cell an ordinary lane.
//  residual          the |u| partials of a step (one per block) are summed in a fixed order
//                    by the first block of the NEXT step's launch, which then runs the
//                    residual / convergence logic of ldc.cu:660-684 on the device, so a step
//                    is one launch; k_reduce_* do it for the last step of an lbm_step call,
//                    under convergence control (the stop must be known before the next
//                    step) and for slabs (the sum goes to the RCCL all-reduce).
// HBM traffic per fluid cell: 76 B loaded + 76 B stored + 1 B type.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <type_traits>

#include "lbm_d3q19.hpp"
#include "lbm_kernels.hpp"

namespace lbm {

namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-wide deterministic sum of one double per thread; result valid in thread 0.
__device__ __forceinline__ double block_sum(double v, double* lds) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) lds[wid] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0)
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += lds[w];
  return s;
}

// DPP whole-wave lane shifts (gfx9 wave_shr:1 / wave_shl:1)
__device__ __forceinline__ float lane_from_prev(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ float lane_from_next(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x130, 0xf, 0xf, false));
}

// Storage direction of population Q.  The layout's rows run along physical x, or along y
// when SW (lbm_desc.row_axis: a pipe along y then fills whole rows); z is always the slab
// axis.  Only addresses change with SW -- the arithmetic stays in physical q order.
template <int Q, bool SW>
struct SDir {
  static constexpr int x = SW ? Dir<Q>::y : Dir<Q>::x;  // along the row: +-1 cell
  static constexpr int y = SW ? Dir<Q>::x : Dir<Q>::y;  // across rows: +-pitch
  static constexpr int z = Dir<Q>::z;                   // across planes: +-plane
};

template <int Q, bool SW>
constexpr int64_t row_off(int pitch, int64_t plane) {
  return SDir<Q, SW>::y * (int64_t)pitch + SDir<Q, SW>::z * plane;
}
// storage offset of e_Q: population Q of cell c is pulled from c - cell_off
template <int Q, bool SW>
constexpr int64_t cell_off(int pitch, int64_t plane) {
  return SDir<Q, SW>::x + row_off<Q, SW>(pitch, plane);
}

// Neighbour addressing of a lane's cell c (a 4-cell lane: its first cell):
//   slice<Q>() -- the cell c - e_Q with e_x = 0: the aligned 16-B slice a 4-cell lane pulls,
//   nb<Q>()    -- the cell c - e_Q.
// AddrD: the dense box -- cell (zs, s1, s0) at s0 - xshift + s1 * pitch + zs * plane, every
// neighbour a constant offset.  Rows: compact rows (sparse lattices, lbm_create's choice) --
// storage row r = zs * nrow + s1 keeps only the span of its stored cells, the spans packed one
// after the other in storage order, so cell (r, s0) lives at roff[r] + s0; a lane holds the
// offsets of the nine rows around its own (loaded once, Rows::load).  Inside a span x +- 1 is
// still c +- 1, and a fluid cell's neighbours are always stored, so they lie inside theirs.
// float index of slot q of cell c (aidx): 64-bit for the dense box, 32-bit for compact rows
// (lbm_create keeps their buffers, guards included, under 2^31 floats)
__device__ __forceinline__ int64_t fidx(int64_t c, int q) { return aidx(c, q); }
__device__ __forceinline__ int fidx(int c, int q) { return ((c >> 8) * kQ + q) * kChunk + (c & (kChunk - 1)); }
// a compact cell id as the 32-bit index of the compact paths (kCompactMaxFloats bounds every id
// of a compact buffer); -DLBM_DEBUG_INDEX traps on an id outside that bound instead of letting
// a 32-bit offset wrap
__device__ __forceinline__ int compact_id(int64_t c) {
#ifdef LBM_DEBUG_INDEX
  if (c < -int64_t(kChunk) * 64 || ((c >> 8) * kQ + kQ) * kChunk > kCompactMaxFloats) __builtin_trap();
#endif
  return (int)c;
}

struct AddrD {
  int64_t c;
  int pitch;
  int64_t plane;
  template <int Q, bool SW>
  __device__ __forceinline__ int64_t slice() const { return c - row_off<Q, SW>(pitch, plane); }
  template <int Q, bool SW>
  __device__ __forceinline__ int64_t nb() const { return c - cell_off<Q, SW>(pitch, plane); }
  __device__ __forceinline__ void opaque() { asm volatile("" : "+v"(c)); }
  __device__ __forceinline__ AddrD get() const { return *this; }
};
template <int Q, bool SW>
constexpr int row_k() {  // Rows::rb index of the row population Q is pulled from
  return (-SDir<Q, SW>::y + 1) * 3 + (-SDir<Q, SW>::z + 1);
}
struct Rows {
  int rb[9];  // roff[r + dy + dz * nrow], index (dy + 1) * 3 + dz + 1
  int s0;     // the cell's position in its row: c - roff[r]
  template <int Q, bool SW>
  __device__ __forceinline__ int slice() const { return rb[row_k<Q, SW>()] + s0; }
  template <int Q, bool SW>
  __device__ __forceinline__ int nb() const { return rb[row_k<Q, SW>()] + s0 - SDir<Q, SW>::x; }
  __device__ __forceinline__ void opaque() {
    asm volatile("" : "+v"(rb[0]), "+v"(rb[1]), "+v"(rb[2]), "+v"(rb[3]), "+v"(rb[4]), "+v"(rb[5]), "+v"(rb[6]),
                 "+v"(rb[7]), "+v"(rb[8]), "+v"(s0));
  }
  __device__ __forceinline__ Rows get() const { return *this; }
  // the row record of row r (MainArgs::rowrec: 12 ints, the nine offsets first) -- three 16-B loads
  __device__ __forceinline__ static Rows load(const int4* __restrict__ rowrec, int64_t c, int r) {
    const int4* p = rowrec + (int64_t)r * 3;
    const int4 x = p[0], y = p[1], z = p[2];
    Rows R;
    R.rb[0] = x.x; R.rb[1] = x.y; R.rb[2] = x.z; R.rb[3] = x.w;
    R.rb[4] = y.x; R.rb[5] = y.y; R.rb[6] = y.z; R.rb[7] = y.w;
    R.rb[8] = z.x;
    R.s0 = compact_id(c) - R.rb[4];
    return R;
  }
};
// Compact rows kept as (cell, row) until the boundary stores need them: the nine offsets are
// loaded again there (L1 / L2 hits) instead of living in ten VGPRs across the collision
struct RowsRef {
  const int4* rowrec;
  int64_t c;
  int r;
  __device__ __forceinline__ Rows get() const {
    int rr = r;
    asm volatile("" : "+v"(rr));  // a fresh load, not the pulls' values kept alive
    return Rows::load(rowrec, c, rr);
  }
};

// Pull of population Q for the lane's 4 cells c..c+3 from c - e_Q .. c+3 - e_Q, in two
// phases so that all of a wave's loads are in flight together (one round trip per wave):
//  issue:   the aligned 16-B slice at c - (e_Q with e_x = 0), and for e_x != 0 the one float
//           beyond the lane's run of cells: cell lo - 1 (e_x = +1) or hi (e_x = -1), where
//           [lo, hi) is the wave's chunk (all lanes load the same address, no branch) or, for a
//           wave of compact groups (GROUPS), the lane's own 4 cells;
//  compose: shift the slice by one cell across lanes (DPP) and take the edge float instead
//           where the neighbouring lane does not hold the neighbouring cells (take_lo / take_hi:
//           lane 0 / 63 of a chunk; a group whose list neighbour is not its row neighbour).
template <int Q, bool SW>
__device__ __forceinline__ void pull_issue(f4& a, float& e, const float* __restrict__ src, int64_t lo, int64_t hi,
                                           int64_t c, int pitch, int64_t plane, bool need) {
  const int64_t ro = row_off<Q, SW>(pitch, plane);
  // lanes outside the chunk's lane mask (sparse lattices) all read the buffer's first line,
  // which stays cached: no HBM bytes for them, and no branch (a branch per direction made the
  // compiler wait for every load before issuing the next)
  const float* p = need ? src + aidx(c - ro, Q) : src;
  // non-temporal: every slice is read once per step.  Plain loads leave the lines two chunks
  // share in L2 more often (10.58 vs 10.76 GB read per launch at 512^3, same time) but cost
  // 7-10% at 256^3 and on C3 (interleaved A/B, profiles/r02_nt_vs_plain_ab.log)
  a = __builtin_nontemporal_load(reinterpret_cast<const f4*>(p));
  // The edge float by a VECTOR load: its line is the neighbouring chunk's slice, which the
  // neighbouring wave -- three times in four a wave of this block, on this CU -- loads at the
  // same time, so it often hits this CU's L1; a wave-uniform address would make it a scalar
  // load, which only the scalar cache and L2 serve (0.30 GB less HBM read per launch at 512^3,
  // +1.8-2.7% in interleaved A/B runs, profiles/r02_edge_vector_ab.log).  The empty asm moves
  // the offset to a VGPR.
  if constexpr (SDir<Q, SW>::x == 1) {  // cell lo - 1
    int64_t o = aidx(lo - ro - 1, Q);
    asm volatile("" : "+v"(o));
    e = src[o];
  } else if constexpr (SDir<Q, SW>::x == -1) {  // cell hi
    int64_t o = aidx(hi - ro, Q);
    asm volatile("" : "+v"(o));
    e = src[o];
  }
}

template <int Q, bool SW>
__device__ __forceinline__ f4 pull_compose(const f4 a, float e, bool take_lo, bool take_hi) {
  if constexpr (SDir<Q, SW>::x == 0) {
    return a;
  } else if constexpr (SDir<Q, SW>::x == 1) {  // needs b-1 .. b+2
    const float p = lane_from_prev(a.w);
    return f4{take_lo ? e : p, a.x, a.y, a.z};
  } else {                                 // needs b+1 .. b+4
    const float n = lane_from_next(a.x);
    return f4{a.y, a.z, a.w, take_hi ? e : n};
  }
}

template <bool SW, int... Qs>
__device__ __forceinline__ void pull4_all(f4* v, const float* __restrict__ src, int64_t lo, int64_t hi, int64_t c,
                                          bool take_lo, bool take_hi, int pitch, int64_t plane, bool need,
                                          std::integer_sequence<int, Qs...>) {
  float e[kQ];
  ((pull_issue<Qs, SW>(v[Qs], e[Qs], src, lo, hi, c, pitch, plane, need)), ...);
  ((v[Qs] = pull_compose<Qs, SW>(v[Qs], e[Qs], take_lo, take_hi)), ...);
}

// The same for a lane of compact 4-cell groups (GROUPS): the edge floats are the lane's own
// neighbours, cells slice - 1 (e_x = +1) and slice + 4 (e_x = -1), in the slice's row.  Plain
// loads here (unlike the chunk lists): C4 x4 138.5 -> 135.1 us (profiles/r05_temporal_ab.log);
// plain stores were slower (143.5), non-temporal ones stay
template <int Q, bool SW, class A>
__device__ __forceinline__ void pull_issue_g(f4& a, float& e, const float* __restrict__ src, const A& ad, bool need) {
  const auto s = ad.template slice<Q, SW>();
  const float* p = need ? src + fidx(s, Q) : src;
  a = *reinterpret_cast<const f4*>(p);
  if constexpr (SDir<Q, SW>::x == 1) {
    auto o = fidx(s - 1, Q);
    asm volatile("" : "+v"(o));
    e = src[o];
  } else if constexpr (SDir<Q, SW>::x == -1) {
    auto o = fidx(s + 4, Q);
    asm volatile("" : "+v"(o));
    e = src[o];
  }
}

template <bool SW, class A, int... Qs>
__device__ __forceinline__ void pull4_g(f4* v, const float* __restrict__ src, const A& ad, bool take_lo, bool take_hi,
                                        bool need, std::integer_sequence<int, Qs...>) {
  float e[kQ];
  ((pull_issue_g<Qs, SW>(v[Qs], e[Qs], src, ad, need)), ...);
  ((v[Qs] = pull_compose<Qs, SW>(v[Qs], e[Qs], take_lo, take_hi)), ...);
}
template <bool SW, class A, int... Qs>
__device__ __forceinline__ void pull4_g_issue(f4* v, float* e, const float* __restrict__ src, const A& ad, bool need,
                                              std::integer_sequence<int, Qs...>) {
  ((pull_issue_g<Qs, SW>(v[Qs], e[Qs], src, ad, need)), ...);
}
template <bool SW, int... Qs>
__device__ __forceinline__ void pull4_compose(f4* v, const float* e, bool take_lo, bool take_hi,
                                              std::integer_sequence<int, Qs...>) {
  ((v[Qs] = pull_compose<Qs, SW>(v[Qs], e[Qs], take_lo, take_hi)), ...);
}

// Bounce-back on the consumer side for 4-cell lanes (MainArgs::bb_pull, compact rows): a cell
// whose neighbour c - e_q is a wall takes population q from its own slot opp(q) of the source
// buffer -- the post-collision value the producer side would have stored into the wall (the
// reference's d_dst[q][W] = d_dst[opp q][W + e_q], Poiseulle.cu:601-746, read where it was
// written).  For every direction that some lane of the wave links, the linking lanes' own 16-B
// slices of slot opp(q) go to the wave's LDS by DMA (global_load_lds: nothing in VGPRs while in
// flight), issued beside the pulls; once in, each cell with the link takes its value.  No wall
// slot is ever written, so lanes sharing their 4-cell group with walls store whole vectors.
struct OwnLds {
  f4 s[kQ][64];  // per direction q: the wave's own slices of slot opp(q)
};
template <int Q, class CT>
__device__ __forceinline__ void bb_own_issue(const float* __restrict__ src, CT c, uint32_t lm, OwnLds& L) {
  if constexpr (Q > 0) {
    const bool mine = (lm >> Q) & 1u;
    if (__any(mine)) {  // wave-uniform
      if (mine)
        __builtin_amdgcn_global_load_lds((gbl_ptr_t)(src + fidx(c, Dir<Q>::opp)), (lds_ptr_t)&L.s[Q][0], 16, 0, 2);
    }
  }
}
template <int Q>
__device__ __forceinline__ void bb_own_merge(f4* v, uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3, uint32_t lm,
                                             int lane, const OwnLds& L) {
  if constexpr (Q > 0) {
    const bool mine = (lm >> Q) & 1u;
    if (__any(mine)) {
      if (mine) {
        const f4 o = L.s[Q][lane];
        v[Q] = f4{(m0 >> Q) & 1u ? o.x : v[Q].x, (m1 >> Q) & 1u ? o.y : v[Q].y, (m2 >> Q) & 1u ? o.z : v[Q].z,
                  (m3 >> Q) & 1u ? o.w : v[Q].w};
      }
    }
  }
}
template <class CT, int... Qs>
__device__ __forceinline__ void bb_own_issue_all(const float* __restrict__ src, CT c, uint32_t lm, OwnLds& L,
                                                 std::integer_sequence<int, Qs...>) {
  (bb_own_issue<Qs>(src, c, lm, L), ...);
}
template <int... Qs>
__device__ __forceinline__ void bb_own_merge_all(f4* v, uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3,
                                                 uint32_t lm, int lane, const OwnLds& L,
                                                 std::integer_sequence<int, Qs...>) {
  (bb_own_merge<Qs>(v, m0, m1, m2, m3, lm, lane, L), ...);
}

template <int J, int... Qs>
__device__ __forceinline__ void relax4(f4* v, float tau, float r, float ux, float uy, float uz,
                                       std::integer_sequence<int, Qs...>) {
  ((v[Qs][J] = v[Qs][J] - (v[Qs][J] - feq<Qs>(r, ux, uy, uz)) / tau), ...);
}

using AllQ = std::make_integer_sequence<int, kQ>;

// Half-way bounce-back, producer side: a wall-adjacent fluid cell F also stores its
// post-collision population opp(q) into the slot q of the wall W = F - e_q, which F itself
// pulls at the next step -- exactly the value boundary_stream writes there
// (Poiseulle.cu:601-746: d_dst[q][W] = d_dst[opp q][W + e_q]).  Each wall slot has one
// writer (W + e_q), the consumer, so the slot always lives in the writer's own storage.
template <int Q, bool SW, class A>
__device__ __forceinline__ void bb_store_one(float* __restrict__ dst, const A& ad, uint32_t m, float out_opp) {
  if constexpr (Q > 0) {
    if (m & (1u << Q)) dst[fidx(ad.template nb<Q, SW>(), Q)] = out_opp;
  }
}
// one set bit at a time (rare path: keeps the address arithmetic out of the hot registers)
template <int J, bool SW, class A>
__device__ __forceinline__ void bb_store_cell(float* __restrict__ dst, A ad, uint32_t m, const f4* v) {
#define LBM_BB_CASE(Q) \
  case Q: dst[fidx(ad.template nb<Q, SW>() + J, Q)] = v[Dir<Q>::opp][J]; break;
  // opaque copy of the address: otherwise the compiler CSEs these offsets with the pull
  // addresses of the same directions and keeps ~70 VGPRs of them alive across the collision
  // (240 vs 167)
  ad.opaque();
  for (; m; m &= m - 1) {
    switch (__builtin_ctz(m)) {
      LBM_BB_CASE(1) LBM_BB_CASE(2) LBM_BB_CASE(3) LBM_BB_CASE(4) LBM_BB_CASE(5) LBM_BB_CASE(6)
      LBM_BB_CASE(7) LBM_BB_CASE(8) LBM_BB_CASE(9) LBM_BB_CASE(10) LBM_BB_CASE(11) LBM_BB_CASE(12)
      LBM_BB_CASE(13) LBM_BB_CASE(14) LBM_BB_CASE(15) LBM_BB_CASE(16) LBM_BB_CASE(17) LBM_BB_CASE(18)
      default: break;
    }
  }
#undef LBM_BB_CASE
}
// Whole-group bounce-back stores.  For direction q with along-row offset s (SDir x) the walls
// c + j - e_q of a lane's cells j = 0..3 are cells c - ro + j - s: for s = 0 the aligned group
// G = c - ro itself; for s = +1 (-1) G's slots 0..2 (1..3) with the neighbouring lane's cell 0
// (cell 3) supplying the last (first) one.  A lane whose cells -- and that neighbour -- all link
// q writes G in one 16-B store of post-collision f_opp(q) values, instead of four scattered
// floats: the same slots with the same values, each still written once, by its one consumer.
template <bool SW, int S>
constexpr uint32_t links_along() {  // directions whose along-row storage offset is S
  uint32_t m = 0;
#define LBM_LA(Q) if (SDir<Q, SW>::x == S) m |= 1u << Q;
  LBM_LA(1) LBM_LA(2) LBM_LA(3) LBM_LA(4) LBM_LA(5) LBM_LA(6) LBM_LA(7) LBM_LA(8) LBM_LA(9)
  LBM_LA(10) LBM_LA(11) LBM_LA(12) LBM_LA(13) LBM_LA(14) LBM_LA(15) LBM_LA(16) LBM_LA(17) LBM_LA(18)
#undef LBM_LA
  return m;
}
__device__ __forceinline__ uint32_t u_from_prev(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t u_from_next(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x130, 0xf, 0xf, false);
}
// called with the whole wave active (the DPP shifts read every lane); g: this lane's groups
template <int Q, bool SW, class A>
__device__ __forceinline__ void bb_group_one(float* __restrict__ dst, const A& ad, uint32_t g, const f4* v) {
  if constexpr (Q > 0) {
    const bool mine = (g >> Q) & 1u;
    if (__any(mine)) {  // wave-uniform
      constexpr int s = SDir<Q, SW>::x;
      const f4 o = v[Dir<Q>::opp];
      f4 w;
      if constexpr (s == 0) w = o;
      else if constexpr (s == 1) w = f4{o.y, o.z, o.w, lane_from_next(o.x)};
      else w = f4{lane_from_prev(o.w), o.x, o.y, o.z};
      if (mine) *reinterpret_cast<f4*>(dst + fidx(ad.template slice<Q, SW>(), Q)) = w;
    }
  }
}
template <bool SW, class A, int... Qs>
__device__ __forceinline__ void bb_group_all(float* __restrict__ dst, const A& ad, uint32_t g, const f4* v,
                                             std::integer_sequence<int, Qs...>) {
  (bb_group_one<Qs, SW>(dst, ad, g, v), ...);
}

// moments (ldc.cu:316-322): sequential fp32 sum; signed sums in the reference order
template <int J>
__device__ __forceinline__ void moments(const f4* v, float& rho, float& ux, float& uy, float& uz) {
  float r = 0.f;
#pragma unroll
  for (int q = 0; q < kQ; ++q) r = r + v[q][J];
  ux = (v[1][J] - v[2][J] + v[7][J] + v[8][J] - v[9][J] - v[10][J] + v[11][J] + v[12][J] - v[13][J] - v[14][J]) / r;
  uy = (v[3][J] - v[4][J] + v[7][J] - v[8][J] + v[9][J] - v[10][J] + v[15][J] - v[16][J] + v[17][J] - v[18][J]) / r;
  uz = (v[5][J] - v[6][J] + v[11][J] - v[12][J] + v[13][J] - v[14][J] + v[15][J] + v[16][J] - v[17][J] - v[18][J]) / r;
  rho = r;
}

// BGK relaxation f - (f - feq) / tau (ldc.cu:326-363) with the division by tau either as
// the compiler's correctly rounded sequence (~10 VALU) or, FAST, as
//   q0 = x * RN(1/tau);  r = fma(-q0, tau, x);  q = fma(r, RN(1/tau), q0)
// (3 VALU), which equals RN(x / tau) for every x whose residual r does not underflow
// (Markstein's theorem; the kernel's caller verifies it for the run's tau over a whole
// binade, which covers [2^-100, 2^100] by exact power-of-two scaling).  Where |x| < 2^-100,
// f - q == f for both quotients whenever |f| >= 2^-60, which the wave checks first.  The
// equilibria's prefactors rho/3, rho/18 and rho/36 take the same shortcut (the divisors are
// verified by verify_fast_div too, and the wave checks 2^-60 <= |rho| < 2^45).
__device__ __forceinline__ float fast_quot(float x, float d, float y) {
  const float q0 = x * y;
  return __builtin_fmaf(__builtin_fmaf(-q0, d, x), y, q0);
}
struct Pref {  // RN(rho / 3), RN(rho / 18), RN(rho / 36)
  float p3, p18, p36;
  __device__ __forceinline__ explicit Pref(float r)
      : p3(fast_quot(r, 3.0f, 1.0f / 3.0f)), p18(fast_quot(r, 18.0f, 1.0f / 18.0f)),
        p36(fast_quot(r, 36.0f, 1.0f / 36.0f)) {}
  __device__ __forceinline__ Pref(float a, float b, float c) : p3(a), p18(b), p36(c) {}
  __device__ __forceinline__ static Pref exact(float r) { return Pref(r / 3.0f, r / 18.0f, r / 36.0f); }
  template <int Q>
  __device__ __forceinline__ float of() const {
    return FeqW<Q>::d == 3.0f ? p3 : FeqW<Q>::d == 18.0f ? p18 : p36;
  }
};
template <int J, bool FAST, int... Qs>
__device__ __forceinline__ void relax_cell(f4* v, float tau, float rcp, float r, float ux, float uy, float uz,
                                           std::integer_sequence<int, Qs...>) {
  if constexpr (FAST) {
    auto div_tau = [&](float x) {
      const float q0 = x * rcp;
      return __builtin_fmaf(__builtin_fmaf(-q0, tau, x), rcp, q0);
    };
    const Pref p(r);
    ((v[Qs][J] = v[Qs][J] - div_tau(v[Qs][J] - feq_pre<Qs>(p.template of<Qs>(), ux, uy, uz))), ...);
  } else {
    ((v[Qs][J] = v[Qs][J] - (v[Qs][J] - feq<Qs>(r, ux, uy, uz)) / tau), ...);
  }
}

// the fast quotient's domain for one cell: 2^-60 <= |f_q| < 2^40 and |u| < 2^10 bound
// |f - feq| below 2^72 (no overflow) and make quotients of |x| < 2^-100 irrelevant;
// 2^-60 <= |rho| < 2^45 keeps the prefactor quotients' residuals normal
template <int J>
__device__ __forceinline__ bool fast_div_ok(const f4* v, float r, float ux, float uy, float uz) {
  float mn = __builtin_fabsf(v[0][J]), mx = mn;
#pragma unroll
  for (int q = 1; q < kQ; ++q) {
    mn = __builtin_fminf(mn, __builtin_fabsf(v[q][J]));
    mx = __builtin_fmaxf(mx, __builtin_fabsf(v[q][J]));
  }
  const float um = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(ux), __builtin_fabsf(uy)), __builtin_fabsf(uz));
  const float ar = __builtin_fabsf(r);
  return mn >= 0x1p-60f && mx < 0x1p40f && um < 0x1p10f && ar >= 0x1p-60f && ar < 0x1p45f;  // false for NaN
}

// ---- NEE boundaries, producer side -------------------------------------------------------
// boundary_stream (ldc.cu:391-456, Poiseulle.cu:748-891, bifurcation.cu:877-1021) writes,
// after the collision, into each NEE cell B and direction q crossing B's face (nb = B + e_q):
//   dst[q][B] = feq_q(rho_bc, u_bc) + (dst[q][nb] - feq_q(rho_nb, u_nb)) (1 - 1/tau)
// Only nb pulls slot q of B (from nb - e_q = B), and nb holds every operand right after its
// own collision: its post-collision f_q and its (rho, u) of the step.  So nb -- the fluid
// cell c of the kernels, B = c - e_q -- stores the value itself, as it stores its bounce-back
// slots.  B's boundary data (written at B by k_classify, static): rho_bc or NaN (rho of c),
// u_bc or NaN (a pressure boundary: u of c).

constexpr uint64_t pack_e(const int* e) {
  uint64_t p = 0;
  for (int q = 0; q < kQ; ++q) p |= (uint64_t)(e[q] + 1) << (2 * q);
  return p;
}
constexpr uint64_t kPackEx = pack_e(kEx), kPackEy = pack_e(kEy), kPackEz = pack_e(kEz);
__device__ __forceinline__ int e_of(uint64_t packed, int q) { return (int)((packed >> (2 * q)) & 3u) - 1; }

template <bool SW>
__device__ __forceinline__ int64_t cell_off_rt(int q, int pitch, int64_t plane) {
  const int ex = e_of(kPackEx, q), ey = e_of(kPackEy, q), ez = e_of(kPackEz, q);
  return (SW ? ey : ex) + (int64_t)(SW ? ex : ey) * pitch + (int64_t)ez * plane;
}

__device__ __forceinline__ float4 bc_at(const MainArgs& a, int64_t b) {
  return make_float4(a.rho[b], a.ux[b], a.uy[b], a.uz[b]);
}

// The boundary data of a cell's first kNeeSlots NEE directions (ascending q), loaded ahead
// -- all issued together, one round trip.  Named members, not an array: a select over an
// array's elements is folded into a dynamic index, which keeps the array in scratch.
struct BcSlots {
  float4 s0, s1, s2, s3, s4;
};
static_assert(kNeeSlots == 5, "BcSlots holds kNeeSlots records");

template <bool SW>
__device__ __forceinline__ float4 bc_next(const MainArgs& a, int64_t c, uint32_t& rest) {
  if (!rest) return make_float4(0.f, 0.f, 0.f, 0.f);
  const int q = __builtin_ctz(rest);
  rest &= rest - 1u;
  return bc_at(a, c - cell_off_rt<SW>(q, a.pitch, a.plane));
}
template <bool SW>
__device__ __forceinline__ BcSlots nee_prefetch(const MainArgs& a, int64_t c, uint32_t nl) {
  if (a.bc_uniform) return BcSlots{a.bc_const, a.bc_const, a.bc_const, a.bc_const, a.bc_const};
  BcSlots b;
  uint32_t rest = nl;
  b.s0 = bc_next<SW>(a, c, rest);
  b.s1 = bc_next<SW>(a, c, rest);
  b.s2 = bc_next<SW>(a, c, rest);
  b.s3 = bc_next<SW>(a, c, rest);
  b.s4 = bc_next<SW>(a, c, rest);
  return b;
}

// pre: RN(r / w_Q's divisor), the fluid cell's equilibrium prefactor from its relaxation, so
// feq<Q>(r, ..) = feq_pre<Q>(pre, ..) bit for bit and neither equilibrium divides again
template <int Q>
__device__ __forceinline__ float nee_value(float fq, float4 b, float r, float ux, float uy, float uz, float omc,
                                           float pre) {
  float rb = b.x, bx = b.y, by = b.z, bz = b.w;
  if (__builtin_isnan(bx)) {  // pressure boundary: u_bc = u of the fluid neighbour
    bx = ux; by = uy; bz = uz;
  }
  const bool rn = __builtin_isnan(rb);  // velocity boundary: rho_bc = rho of the fluid neighbour
  float e_bc;
  if constexpr (Q == 14) e_bc = feq_bc<14>(rn ? r : rb, bx, by, bz);  // its own fp32 form
  else e_bc = feq_pre<Q>(rn ? pre : rb / FeqW<Q>::d, bx, by, bz);
  const float e_nb = feq_pre<Q>(pre, ux, uy, uz);
  return e_bc + (fq - e_nb) * omc;
}

// the cell's post-collision f_Q, for nee_store_q: one cell in registers after its relaxation
struct Post1 {
  const float* f;
  template <int Q>
  __device__ __forceinline__ float post(const MainArgs&, float, float, float, float) const {
    return f[Q];
  }
};
template <int Q, bool SW, class Src, class A>
__device__ __forceinline__ void nee_store_q(const MainArgs& a, const A& ad, uint32_t nl, float4 b0, float4 b1,
                                            float4 b2, float4 b3, float4 b4, const Src& src, float r, float ux,
                                            float uy, float uz, const Pref& p) {
  if constexpr (Q > 0) {
    if (nl & (1u << Q)) {  // divergent only where a wave mixes faces (edges, corners)
      const int k = __builtin_popcount(nl & ((1u << Q) - 1u));  // Q's slot
      const auto nb = ad.template nb<Q, SW>();
      float4 b;
      if (k >= kNeeSlots) b = bc_at(a, nb);
      else b = k == 0 ? b0 : k == 1 ? b1 : k == 2 ? b2 : k == 3 ? b3 : b4;
      const float fq = src.template post<Q>(a, r, ux, uy, uz);
      a.dst[fidx(nb, Q)] = nee_value<Q>(fq, b, r, ux, uy, uz, a.omc, p.template of<Q>());
    }
  }
}

__device__ __forceinline__ void opaque(float4& v) { asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w)); }

template <bool SW, class Src, class A, int... Qs>
__device__ __forceinline__ void nee_store_all(const MainArgs& a, const A& ad, uint32_t nl, BcSlots bc, const Src& src,
                                              float r, float ux, float uy, float uz, const Pref& p,
                                              std::integer_sequence<int, Qs...>) {
  // plain registers from here on: otherwise the slot selections below fold into one load at
  // a variable offset, and the records go through scratch
  float4 b0 = bc.s0, b1 = bc.s1, b2 = bc.s2, b3 = bc.s3, b4 = bc.s4;
  opaque(b0); opaque(b1); opaque(b2); opaque(b3); opaque(b4);
  (nee_store_q<Qs, SW>(a, ad, nl, b0, b1, b2, b3, b4, src, r, ux, uy, uz, p), ...);
}

// ---- the device-generated cavity: types from coordinates (MainArgs::box) ------------------
// ldc.cu:468-502: wall shell [1, n-2]^3, fluid [2, n-3]^3, lid (velocity NEE, -y face) on the
// plane y = ny-2 over x, z in [1, n-2].  A fluid cell's neighbour c - e_q is a wall when it lies
// on the shell (x' = 1 or nx-2, y' = 1, z' = 1 or nzg-2) and not on the lid plane; the lid
// supplies the populations with e_y = -1 of the row y = ny-3.  Masks of the directions by the
// sign of one component: the wall beyond x = 1 is pulled along e_x = +1, and so on.
template <int C, int S>
constexpr uint32_t dirs_with() {  // directions whose component C (0 x, 1 y, 2 z) equals S
  uint32_t m = 0;
  for (int q = 1; q < kQ; ++q)
    if ((C == 0 ? kEx[q] : C == 1 ? kEy[q] : kEz[q]) == S) m |= 1u << q;
  return m;
}
struct BoxCell {
  uint8_t t;        // the type byte k_classify / k_flag_fluid give the cell
  uint32_t links;   // wall links (fluid cells)
  uint32_t nl;      // NEE links (fluid cells)
};
__device__ __forceinline__ BoxCell box_cell(const MainArgs& a, int64_t c) {
  const int64_t u = c + a.box_xshift;
  const int x = (int)(u & ((1 << a.box_pshift) - 1));
  const int y = (int)((u >> a.box_pshift) & ((1 << (a.box_lshift - a.box_pshift)) - 1));
  const int z = (int)(u >> a.box_lshift) - 1 + a.box_zoff;
  const int nx = a.box_nx, ny = a.box_ny, nz = a.box_nzg;
  BoxCell b{kPassive, 0u, 0u};
  const bool shell = x >= 1 && x <= nx - 2 && y >= 1 && y <= ny - 2 && z >= 1 && z <= nz - 2;
  if (!shell) return b;
  if (y == ny - 2) {
    b.t = make_nee(kFaceNY, false);
  } else if (x >= 2 && x <= nx - 3 && y >= 2 && z >= 2 && z <= nz - 3) {
    uint32_t m = (x == 2 ? dirs_with<0, 1>() : 0u) | (x == nx - 3 ? dirs_with<0, -1>() : 0u) |
                 (y == 2 ? dirs_with<1, 1>() : 0u) | (z == 2 ? dirs_with<2, 1>() : 0u) |
                 (z == nz - 3 ? dirs_with<2, -1>() : 0u);
    const bool lid = y == ny - 3;
    if (lid) m &= ~dirs_with<1, -1>();
    b.links = m;
    b.nl = lid ? dirs_with<1, -1>() : 0u;
    b.t = (uint8_t)(kFluid | (m ? kWallAdj : 0) | (lid ? kNeeAdj : 0));
  } else {
    b.t = kWall;
  }
  return b;
}

// ---- NEE records (MainArgs::nee_rec; single-domain chunk ranges whose chunk waves collide the
// NEE-adjacent cells) -------------------------------------------------------------------------
// boundary_stream writes slot q of NEE cell B = c - e_q from c's post-collision f_q and (rho, u)
// of the step (ldc.cu:391-456, Poiseulle.cu:748-891), and only c pulls it, at the next step.  So
// the chunk wave that collides c computes those values right after its relaxation and stores them
// -- one 32-B record per cell, contiguous per chunk -- and the wave that collides c next step puts
// them into its pulled populations in place of B's slots.  No scattered 4-B store into B's slots
// (six of the thirteen microseconds the NEE work cost the pipe, profiles/r05_nee_cost_ab.log), no
// second collision of c, no launch after the step.  The static part of each record (LDS by DMA
// beside the pulls): the cell's position in its chunk, its NEE-link mask and the boundary data of
// its first kNeeRecDirs NEE directions.
// a component of f4 by a wave-uniform index
__device__ __forceinline__ float comp4(const f4 v, int j) { return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w; }
__device__ __forceinline__ f4 with_comp4(f4 v, int j, float x) {
  return f4{j == 0 ? x : v.x, j == 1 ? x : v.y, j == 2 ? x : v.z, j == 3 ? x : v.w};
}
__device__ __forceinline__ float readlane_f(float x, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), l));
}
// next step: the recorded NEE values replace the pulled slots of the cell (lane L, cell j)
template <int Q>
__device__ __forceinline__ void nee_rec_sub(f4* v, int lane, int L, int j, uint32_t nl, const float* vals) {
  if constexpr (Q > 0) {
    if (nl & (1u << Q)) {  // wave-uniform
      const float x = vals[__builtin_popcount(nl & ((1u << Q) - 1u))];
      if (lane == L) v[Q] = with_comp4(v[Q], j, x);
    }
  }
}
template <int... Qs>
__device__ __forceinline__ void nee_rec_sub_all(f4* v, int lane, int L, int j, uint32_t nl, const float* vals,
                                                std::integer_sequence<int, Qs...>) {
  (nee_rec_sub<Qs>(v, lane, L, j, nl, vals), ...);
}
// this step: lane kk collects the value of the cell's kk-th NEE direction
template <int Q>
__device__ __forceinline__ void nee_rec_make(const f4* v, int lane, int L, int j, uint32_t nl, const float4* bc, float r,
                                             float ux, float uy, float uz, const Pref& pre, float omc, float& mine) {
  if constexpr (Q > 0) {
    if (nl & (1u << Q)) {  // wave-uniform
      const int kk = __builtin_popcount(nl & ((1u << Q) - 1u));
      const float fq = readlane_f(comp4(v[Q], j), L);
      const float x = nee_value<Q>(fq, bc[kk], r, ux, uy, uz, omc, pre.template of<Q>());
      if (lane == kk) mine = x;
    }
  }
}
template <int... Qs>
__device__ __forceinline__ void nee_rec_make_all(const f4* v, int lane, int L, int j, uint32_t nl, const float4* bc,
                                                 float r, float ux, float uy, float uz, const Pref& pre, float omc,
                                                 float& mine, std::integer_sequence<int, Qs...>) {
  (nee_rec_make<Qs>(v, lane, L, j, nl, bc, r, ux, uy, uz, pre, omc, mine), ...);
}

// One wave's chunk: pull, collide, store; returns the lane's |u| sum.
//  FAST: the 3-VALU quotient when the whole wave lies in its domain, else (a wave-uniform
//        branch) the exact division, counted in exact_waves.  Both paths cost 210-218 VGPRs
//        (two waves per SIMD) against 162-166 for the exact one alone, whose three waves per
//        SIMD ran slower (profiles/r03_fast3_ab.log).
//  COMPACT (with GROUPS): compact rows -- the group's row record goes out beside the list
//        entry's type byte and link masks, then the pulls (Rows).
//  BOX (chunk lists of the device-generated cavity): type bytes and wall links from the cells'
//        coordinates (box_cell), no loads.
//  REC (chunk lists of the dense box): NEE records (MainArgs::nee_rec); ridx, the wave's chunk-list
//        entry, indexes MainArgs::nee_rec_base.  A separate instance: the records' code costs the
//        instances without it registers
template <bool FAST, bool SW, bool MASK, bool GROUPS = false, bool COMPACT = false, bool BOX = false, bool REC = false>
__device__ __forceinline__ double process_chunk(const MainArgs& a, int64_t cb, int lane, uint64_t lane_mask,
                                                int ridx = -1) {
  static_assert(!REC || !(GROUPS || BOX), "NEE records run over the dense box's chunk lists");
  static_assert(GROUPS || !COMPACT, "compact rows run over group lists");
  static_assert(!(BOX && (GROUPS || SW)), "the cavity runs over x-row chunk lists");
  double acc = 0.0;
  int64_t c;
  bool need, take_lo, take_hi;
  f4 v[kQ];
  int rb = 0, rn = 0;  // NEE records of the chunk: first index, count
  float4* NL = nullptr;  // this wave's LDS for them: static records, the previous step's values, (rho, u)
  if constexpr (REC) {
    __shared__ float4 nee_lds[kBlock / 64][kNeeRecMax * (kNeeRecF4 + 3)];
    NL = nee_lds[threadIdx.x >> 6];
  }
  RowsRef ad{};  // COMPACT: the lane's cell and row (Rows again for the bounce-back stores)
  constexpr unsigned kWall4 = kWallAdj * 0x01010101u, kNee4 = kNeeAdj * 0x01010101u;
  uint32_t m0 = 0, m1 = 0, m2 = 0, m3 = 0;
  unsigned t4 = 0u;
  // COMPACT: bounce-back on the consumer side (bb_own_*); step 0 of a case whose walls do not
  // bounce back yet pulls the walls raw
  const bool consumer = COMPACT && a.bb_pull && !a.bb_raw;
  // y rows (the pipe's chunk lists, the upsampled bifurcation's group lists): the wave issues its
  // pulls and its stores at raised priority and drops it for the arithmetic, so that a SIMD's
  // other wave, in its arithmetic, does not hold back the memory instructions (C3 170.5 vs 171.8
  // us per step for the pulls, r06zl, and 169.9 vs 170.5 with the stores, r06zm; C4 x4 123.6 vs
  // 124.5, r06zq; the cavity's x rows run 1.3% slower that way at 256^3, r06zk)
  constexpr bool kPrio = SW;
  if constexpr (kPrio) __builtin_amdgcn_s_setprio(2);
  if constexpr (GROUPS) {
    // compact groups: lane = one 4-cell group of the range's list (cb: the wave's first entry);
    // a lane takes its x-neighbours' cells from the neighbouring lane when that lane holds the
    // neighbouring group of the row, else by its own edge loads
    // entries: the group's first cell (a multiple of 4), bit 0 set for an idle group of a
    // segment (it loads nothing); the tail lanes of the last wave read entry 0 and idle too
    const int64_t gi = cb + lane;
    const int64_t gs = gi < a.ngroups ? gi : 0;
    const int e = a.groups[gs];
    need = gi < a.ngroups && !(e & 1);
    const int g = e & ~3;
    // a neighbour lane that loads nothing or holds another row position is no x-neighbour
    const int nd = need ? g : -8;
    const int gp = __builtin_amdgcn_mov_dpp(nd, 0x138, 0xf, 0xf, false);  // lane - 1 (wave_shr:1)
    const int gn = __builtin_amdgcn_mov_dpp(nd, 0x130, 0xf, 0xf, false);  // lane + 1 (wave_shl:1)
    take_lo = lane == 0 || gp + 4 != g;
    take_hi = lane == 63 || gn != g + 4;
    c = g;
    if constexpr (COMPACT) {
      // type bytes and link masks beside the row record (one round trip), then the pulls and,
      // for the wall links, the own slices (consumer-side bounce-back) -- one more round trip
      const int row = a.group_row[gs];
      t4 = need ? *reinterpret_cast<const unsigned*>(a.type + c) : 0u;
      const uint4 lk = *reinterpret_cast<const uint4*>(a.links + (need ? c : 0));
      float e[kQ];
      pull4_g_issue<SW>(v, e, a.src, Rows::load(a.rowrec, c, row), need, AllQ{});
      m0 = (t4 & (kWallAdj << 0)) ? lk.x : 0u;
      m1 = (t4 & (kWallAdj << 8)) ? lk.y : 0u;
      m2 = (t4 & (kWallAdj << 16)) ? lk.z : 0u;
      m3 = (t4 & (kWallAdj << 24)) ? lk.w : 0u;
      if (consumer) {
        __shared__ OwnLds own_lds[kBlock / 64];
        OwnLds& L = own_lds[threadIdx.x >> 6];
        const uint32_t lm = m0 | m1 | m2 | m3;
        const bool walls = __any(lm != 0u);  // wave-uniform
        if (walls) bb_own_issue_all(a.src, compact_id(c), lm, L, AllQ{});
        pull4_compose<SW>(v, e, take_lo, take_hi, AllQ{});
        if (walls) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the DMA's LDS writes are in
          bb_own_merge_all(v, m0, m1, m2, m3, lm, lane, L, AllQ{});
        }
        m0 = m1 = m2 = m3 = 0u;  // no wall stores
      } else {
        pull4_compose<SW>(v, e, take_lo, take_hi, AllQ{});
      }
      ad = RowsRef{a.rowrec, c, row};
    } else {
      pull4_all<SW>(v, a.src, c, c + 4, c, take_lo, take_hi, a.pitch, a.plane, need, AllQ{});
    }
  } else {
    c = cb + lane * 4;
    // lanes the chunk's mask leaves out hold no fluid cell and neighbour none: they load
    // nothing and count as passive (nothing stored, no |u|)
    need = MASK ? ((lane_mask >> lane) & 1u) != 0 : true;
    take_lo = lane == 0;
    take_hi = lane == 63;
    // NEE records of the chunk's NEE-adjacent cells: static part and the previous step's values
    // to LDS by DMA, beside the pulls (nothing in VGPRs while in flight)
    if (REC) {
      rb = a.nee_rec_base[ridx];
      rn = a.nee_rec_base[ridx + 1] - rb;
    }
    if (REC && rn > 0) {  // wave-uniform
      for (int o = 0; o < rn * kNeeRecF4; o += 64)  // more than one wave-load from 8 records on
        if (lane + o < rn * kNeeRecF4)
          __builtin_amdgcn_global_load_lds((gbl_ptr_t)(a.nee_rec + (int64_t)rb * kNeeRecF4 + o + lane),
                                           (lds_ptr_t)(NL + o), 16, 0, 0);
      if (a.nee_in != nullptr && lane < rn * 2)
        __builtin_amdgcn_global_load_lds((gbl_ptr_t)(a.nee_in + ((int64_t)rb * 2 + lane) * 4),
                                         (lds_ptr_t)(NL + kNeeRecMax * kNeeRecF4), 16, 0, 0);
    }
    pull4_all<SW>(v, a.src, cb, cb + kChunk, c, take_lo, take_hi, a.pitch, a.plane, need, AllQ{});
    if (REC && rn > 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the DMA's LDS writes are in
      if (a.nee_in != nullptr) {
        const float* vals = reinterpret_cast<const float*>(NL + kNeeRecMax * kNeeRecF4);
        for (int k = 0; k < rn; ++k) {
          const int4 h = *reinterpret_cast<const int4*>(NL + k * kNeeRecF4);
          const int pos = __builtin_amdgcn_readfirstlane(h.x);
          const uint32_t nl = (uint32_t)__builtin_amdgcn_readfirstlane(h.y);
          nee_rec_sub_all(v, lane, pos >> 2, pos & 3, nl, vals + k * 8, AllQ{});
        }
      }
    }
  }
  if constexpr (BOX) {
    const BoxCell b0 = box_cell(a, c), b1 = box_cell(a, c + 1), b2 = box_cell(a, c + 2), b3 = box_cell(a, c + 3);
    t4 = need ? (unsigned)b0.t | ((unsigned)b1.t << 8) | ((unsigned)b2.t << 16) | ((unsigned)b3.t << 24) : 0u;
    m0 = b0.links; m1 = b1.links; m2 = b2.links; m3 = b3.links;
  } else if constexpr (!COMPACT) {
    const unsigned t4r = *reinterpret_cast<const unsigned*>(a.type + (need ? c : 0));
    t4 = need ? t4r : 0u;
  }
  // wall-link masks of the lane's wall-adjacent cells (consumed only after the collision,
  // so this dependent load hides behind the arithmetic)
  if constexpr (BOX || COMPACT) {
  } else if constexpr (GROUPS) {
    // compact lists are wall-heavy: the lane's four masks go out beside the type bytes (one
    // 16-B load, no dependent round trip)
    const uint4 lk = *reinterpret_cast<const uint4*>(a.links + (need ? c : 0));
    m0 = (t4 & (kWallAdj << 0)) ? lk.x : 0u;
    m1 = (t4 & (kWallAdj << 8)) ? lk.y : 0u;
    m2 = (t4 & (kWallAdj << 16)) ? lk.z : 0u;
    m3 = (t4 & (kWallAdj << 24)) ? lk.w : 0u;
  } else if (t4 & kWall4) {
    if (t4 & (kWallAdj << 0)) m0 = a.links[c + 0];
    if (t4 & (kWallAdj << 8)) m1 = a.links[c + 1];
    if (t4 & (kWallAdj << 16)) m2 = a.links[c + 2];
    if (t4 & (kWallAdj << 24)) m3 = a.links[c + 3];
  }
  if constexpr (kPrio) __builtin_amdgcn_s_setprio(0);
  float r0, r1, r2, r3, x0, x1, x2, x3, y0, y1, y2, y3, z0, z1, z2, z3;
  moments<0>(v, r0, x0, y0, z0);
  moments<1>(v, r1, x1, y1, z1);
  moments<2>(v, r2, x2, y2, z2);
  moments<3>(v, r3, x3, y3, z3);
  bool fast_wave = false;
  if constexpr (FAST) {  // non-fluid cells are never stored: they do not constrain the wave
    const unsigned fl = t4 & (t4 >> 1) & 0x01010101u;
    const bool ok = (!(fl & 0x1u) || fast_div_ok<0>(v, r0, x0, y0, z0)) &&
                    (!(fl & 0x100u) || fast_div_ok<1>(v, r1, x1, y1, z1)) &&
                    (!(fl & 0x10000u) || fast_div_ok<2>(v, r2, x2, y2, z2)) &&
                    (!(fl & 0x1000000u) || fast_div_ok<3>(v, r3, x3, y3, z3));
    fast_wave = __all(ok);
    if (!fast_wave && lane == 0) atomicAdd(a.exact_waves, 1ull);
  }
  // what this lane stores and its |u| terms -- before the relaxation, so that the moments
  // die cell by cell inside it (macros are not stored: lbm_get_macros recomputes them from
  // the last step's source buffer, k_moments)
  const f4 UX{x0, x1, x2, x3}, UY{y0, y1, y2, y3}, UZ{z0, z1, z2, z3};
  unsigned store = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const unsigned t = (t4 >> (8 * j)) & 0xffu;
    const int64_t cj = c + j;
    // NEE-adjacent cells belong to the NEE blocks of the launch (nee_cell), unless the range
    // hands the chunk waves their own slots (nee_chunks: the NEE blocks then only add the NEE
    // neighbours' slots, or, nee_mac, k_nee_fix does after the launch)
    const bool in = ((cj >= a.c_lo && cj < a.c_hi) || (cj >= a.c_lo2 && cj < a.c_hi2)) && (t & kClassMask) == kFluid &&
                    (a.nee_chunks || !(t & kNeeAdj));
    if (in) {
      store |= 1u << j;
      acc += (double)sqrtf(UX[j] * UX[j] + UY[j] * UY[j] + UZ[j] * UZ[j]);
    }
  }
  if (a.nee_mac != nullptr && __any(store != 0u && (t4 & kNee4) != 0u)) {  // wave-uniform
    // the NEE-adjacent cells' (rho, u) of this step for k_nee_fix (one 16-B store per cell), at
    // slots numbered in storage order: the work unit's first slot plus the cell's rank among the
    // wave's such cells (lanes in storage order, a lane's cells j = 0..3)
    const f4 R{r0, r1, r2, r3};
    unsigned nm = 0u;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if ((store & (1u << j)) && ((t4 >> (8 * j)) & kNeeAdj)) nm |= 1u << j;
    int k = a.nee_mac_base[GROUPS ? (int)(cb >> 6) : ridx];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint64_t bj = __ballot((nm >> j) & 1u);
      k += (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bj >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bj, 0u));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (nm & (1u << j)) a.nee_mac[k++] = make_float4(R[j], UX[j], UY[j], UZ[j]);
  }
  // Whole 16-B stores whenever the lane's other cells may take garbage: passive cells
  // no fluid cell pulls (their macros are masked on read-out).  Wall and NEE cells hold
  // bounce-back slots / NEE values, and cells outside the launch's ranges (and NEE-adjacent
  // cells the NEE blocks store) are stored by other threads, so those lanes store cell by cell
  // -- sub-16-B stores cost whole partial-line writes in HBM (the x-ends of every row took 15%
  // of the step before the xshift alignment), and a wave with one such lane issues both store
  // paths (4 x 19 + 19 instructions: every y-row wave of the C3 pipe, before nee_chunks).
  const unsigned lo4 = t4 & 0x01010101u, hi4 = (t4 >> 1) & 0x01010101u;
  // wall (unless bounce-back is on the consumer side: no wall slot is ever read), NEE, pulled passive
  const unsigned special = (consumer ? (hi4 & ~lo4) : (lo4 ^ hi4)) | (~(lo4 | hi4) & (t4 >> 2) & 0x01010101u);
  const bool lane_in = (c >= a.c_lo && c + 4 <= a.c_hi) || (c >= a.c_lo2 && c + 4 <= a.c_hi2);
  const bool keep_others = special != 0u || !lane_in || (!a.nee_chunks && (t4 & kNee4));
  const bool whole = store == 0xfu || (store != 0u && !keep_others);
  if (REC && rn > 0) {  // wave-uniform: the NEE-adjacent cells' (rho, u) to LDS, so that the
                        // moments need not live through the relaxation
    const f4 R{r0, r1, r2, r3};
    float4* M = NL + kNeeRecMax * (kNeeRecF4 + 2);
    for (int k = 0; k < rn; ++k) {
      const int4 h = *reinterpret_cast<const int4*>(NL + k * kNeeRecF4);
      const int pos = __builtin_amdgcn_readfirstlane(h.x);
      const int L = pos >> 2, j = pos & 3;
      const float4 m = make_float4(readlane_f(comp4(R, j), L), readlane_f(comp4(UX, j), L),
                                   readlane_f(comp4(UY, j), L), readlane_f(comp4(UZ, j), L));
      if (lane == 0) M[k] = m;
    }
  }
  if (FAST && fast_wave) {
    relax_cell<0, true>(v, a.tau, a.tau_rcp, r0, x0, y0, z0, AllQ{});
    relax_cell<1, true>(v, a.tau, a.tau_rcp, r1, x1, y1, z1, AllQ{});
    relax_cell<2, true>(v, a.tau, a.tau_rcp, r2, x2, y2, z2, AllQ{});
    relax_cell<3, true>(v, a.tau, a.tau_rcp, r3, x3, y3, z3, AllQ{});
  } else {  // exact division: tau not verified, or a wave outside the fast quotient's domain
    relax_cell<0, false>(v, a.tau, a.tau_rcp, r0, x0, y0, z0, AllQ{});
    relax_cell<1, false>(v, a.tau, a.tau_rcp, r1, x1, y1, z1, AllQ{});
    relax_cell<2, false>(v, a.tau, a.tau_rcp, r2, x2, y2, z2, AllQ{});
    relax_cell<3, false>(v, a.tau, a.tau_rcp, r3, x3, y3, z3, AllQ{});
  }
  const auto bad = [&] {  // compact rows: the row offsets again (RowsRef)
    if constexpr (COMPACT) return ad.get();
    else return AddrD{c, a.pitch, a.plane};
  }();
  if (!consumer && __any(t4 & kWall4)) {  // wave-uniform: whole-group bounce-back stores (bb_group_one)
    const uint32_t b0 = (store & 1u) ? m0 : 0u, b1 = (store & 2u) ? m1 : 0u, b2 = (store & 4u) ? m2 : 0u,
                   b3 = (store & 8u) ? m3 : 0u;
    const uint32_t nb0 = take_hi ? 0u : u_from_next(b0), pb3 = take_lo ? 0u : u_from_prev(b3);
    const uint32_t g0 = b0 & b1 & b2 & b3 & links_along<SW, 0>();
    const uint32_t gp = b1 & b2 & b3 & nb0 & links_along<SW, 1>();   // G takes the next lane's cell 0
    const uint32_t gm = pb3 & b0 & b1 & b2 & links_along<SW, -1>();  // G takes the previous lane's cell 3
    const uint32_t gpp = take_lo ? 0u : u_from_prev(gp);  // the previous lane's G holds my cell 0's wall
    const uint32_t gmn = take_hi ? 0u : u_from_next(gm);  // the next lane's G holds my cell 3's wall
    bb_group_all<SW>(a.dst, bad, g0 | gp | gm, v, AllQ{});
    const uint32_t g = g0 | gp | gm;
    m0 &= ~(g0 | gm | gpp); m1 &= ~g; m2 &= ~g; m3 &= ~(g0 | gp | gmn);
  }
  if (!consumer && (t4 & kWall4)) {  // rare, divergent: lanes holding wall-adjacent cells
    if (store & 1u) bb_store_cell<0, SW>(a.dst, bad, m0, v);
    if (store & 2u) bb_store_cell<1, SW>(a.dst, bad, m1, v);
    if (store & 4u) bb_store_cell<2, SW>(a.dst, bad, m2, v);
    if (store & 8u) bb_store_cell<3, SW>(a.dst, bad, m3, v);
  }
  if (REC && rn > 0) {  // wave-uniform: this step's NEE values of the chunk's NEE-adjacent cells
    const float4* M = NL + kNeeRecMax * (kNeeRecF4 + 2);
    for (int k = 0; k < rn; ++k) {
      const int4 h = *reinterpret_cast<const int4*>(NL + k * kNeeRecF4);
      const int pos = __builtin_amdgcn_readfirstlane(h.x);
      const uint32_t nl = (uint32_t)__builtin_amdgcn_readfirstlane(h.y);
      const int L = pos >> 2, j = pos & 3;
      const float4 m = M[k];
      const float r = readlane_f(m.x, 0), ux = readlane_f(m.y, 0), uy = readlane_f(m.z, 0), uz = readlane_f(m.w, 0);
      float mine = 0.f;
      nee_rec_make_all(v, lane, L, j, nl, NL + k * kNeeRecF4 + 1, r, ux, uy, uz, Pref::exact(r), a.omc, mine, AllQ{});
      if (lane < __builtin_popcount(nl)) a.nee_out[(int64_t)(rb + k) * 8 + lane] = mine;
    }
  }
  if constexpr (kPrio) __builtin_amdgcn_s_setprio(2);  // the stores, too (169.9 vs 170.5 us, r06zm)
  float* d = a.dst + aidx(c, 0);
  if (whole) {
#pragma unroll
    for (int q = 0; q < kQ; ++q) __builtin_nontemporal_store(v[q], reinterpret_cast<f4*>(d + q * kChunk));
  } else if (store) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!(store & (1u << j))) continue;
#pragma unroll
      for (int q = 0; q < kQ; ++q) d[q * kChunk + j] = v[q][j];
    }
  }
  return acc;
}

// ---- one cell per lane ---------------------------------------------------------------

template <int... Qs>
__device__ __forceinline__ void fix_relax_all(float* f, float tau, float r, float ux, float uy, float uz,
                                              std::integer_sequence<int, Qs...>) {
  ((f[Qs] = f[Qs] - (f[Qs] - feq<Qs>(r, ux, uy, uz)) / tau), ...);
}
// the same with relax_cell's 3-VALU quotient (caller: tau verified, cell in the domain)
template <int... Qs>
__device__ __forceinline__ void fix_relax_fast_all(float* f, float tau, float rcp, float r, float ux, float uy,
                                                   float uz, std::integer_sequence<int, Qs...>) {
  auto div_tau = [&](float x) {
    const float q0 = x * rcp;
    return __builtin_fmaf(__builtin_fmaf(-q0, tau, x), rcp, q0);
  };
  const Pref p(r);
  ((f[Qs] = f[Qs] - div_tau(f[Qs] - feq_pre<Qs>(p.template of<Qs>(), ux, uy, uz))), ...);
}
// fast_div_ok for one cell in registers
__device__ __forceinline__ bool fast_div_ok1(const float* f, float r, float ux, float uy, float uz) {
  float mn = __builtin_fabsf(f[0]), mx = mn;
#pragma unroll
  for (int q = 1; q < kQ; ++q) {
    mn = __builtin_fminf(mn, __builtin_fabsf(f[q]));
    mx = __builtin_fmaxf(mx, __builtin_fabsf(f[q]));
  }
  const float um = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(ux), __builtin_fabsf(uy)), __builtin_fabsf(uz));
  const float ar = __builtin_fabsf(r);
  return mn >= 0x1p-60f && mx < 0x1p40f && um < 0x1p10f && ar >= 0x1p-60f && ar < 0x1p45f;  // false for NaN
}
// one cell's relaxation: the fast quotient when tau is verified and every active lane of
// the wave lies in its domain (a wave-uniform choice: the lanes stay together), else exact
// returns the equilibrium prefactors RN(r / 3), RN(r / 18), RN(r / 36) (for the NEE values)
__device__ __forceinline__ Pref relax1(float* f, const MainArgs& a, float r, float ux, float uy, float uz) {
  const bool ok = fast_div_ok1(f, r, ux, uy, uz);
  if (a.tau_fast && __all(ok)) {
    fix_relax_fast_all(f, a.tau, a.tau_rcp, r, ux, uy, uz, AllQ{});
    return Pref(r);
  }
  fix_relax_all(f, a.tau, r, ux, uy, uz, AllQ{});
  return Pref::exact(r);
}
// The fast relaxation with the NEE stores fused in (waves holding NEE-adjacent cells): slot Q
// of the NEE neighbour c - e_Q is written as soon as f_Q is relaxed, from the same feq_Q (the
// neighbour's e_nb) -- no second equilibrium per direction, nothing kept alive for later.
template <int Q, bool SW, class A>
__device__ __forceinline__ void relax_nee_q(float* f, const MainArgs& a, const Pref& p, float r, float ux, float uy,
                                            float uz, const A& ad, uint32_t nl, float4 b0, float4 b1, float4 b2,
                                            float4 b3, float4 b4) {
  const float pre = p.template of<Q>();
  const float fe = feq_pre<Q>(pre, ux, uy, uz);
  const float x = f[Q] - fe;
  const float q0 = x * a.tau_rcp;
  f[Q] = f[Q] - __builtin_fmaf(__builtin_fmaf(-q0, a.tau, x), a.tau_rcp, q0);
  if constexpr (Q > 0) {
    if (nl & (1u << Q)) {
      const int k = __builtin_popcount(nl & ((1u << Q) - 1u));
      const auto nb = ad.template nb<Q, SW>();
      float4 b;
      if (k >= kNeeSlots) b = bc_at(a, nb);
      else b = k == 0 ? b0 : k == 1 ? b1 : k == 2 ? b2 : k == 3 ? b3 : b4;
      float rb = b.x, bx = b.y, by = b.z, bz = b.w;
      if (__builtin_isnan(bx)) {
        bx = ux; by = uy; bz = uz;
      }
      const bool rn = __builtin_isnan(rb);
      float e_bc;
      if constexpr (Q == 14) e_bc = feq_bc<14>(rn ? r : rb, bx, by, bz);
      else e_bc = feq_pre<Q>(rn ? pre : rb / FeqW<Q>::d, bx, by, bz);
      a.dst[fidx(nb, Q)] = e_bc + (f[Q] - fe) * a.omc;
    }
  }
}
template <bool SW, class A, int... Qs>
__device__ __forceinline__ void relax_nee_fast_all(float* f, const MainArgs& a, float r, float ux, float uy, float uz,
                                                   const A& ad, uint32_t nl, BcSlots bc,
                                                   std::integer_sequence<int, Qs...>) {
  const Pref p(r);
  float4 b0 = bc.s0, b1 = bc.s1, b2 = bc.s2, b3 = bc.s3, b4 = bc.s4;
  opaque(b0); opaque(b1); opaque(b2); opaque(b3); opaque(b4);
  (relax_nee_q<Qs, SW>(f, a, p, r, ux, uy, uz, ad, nl, b0, b1, b2, b3, b4), ...);
}

template <bool SW, class A, int... Qs>
__device__ __forceinline__ void fix_store_all(const float* f, float* __restrict__ dst, int64_t c, const A& ad,
                                              uint32_t m, std::integer_sequence<int, Qs...>) {
  ((dst[aidx(c, Qs)] = f[Qs]), ...);
  if (m) {
    const auto an = ad.get();
    (bb_store_one<Qs, SW>(dst, an, m, f[Dir<Qs>::opp]), ...);
  }
}

// one cell's 19 plain pulls through an address policy (compact rows; NEE blocks)
template <bool SW, class A, int... Qs>
__device__ __forceinline__ void pull1_addr(float* f, const float* __restrict__ src, const A& ad,
                                           std::integer_sequence<int, Qs...>) {
  ((f[Qs] = *(src + fidx(ad.template nb<Qs, SW>(), Qs))), ...);
}
// the same with bounce-back on the consumer side (MainArgs::bb_pull): where bit q of wl is set
// (c - e_q a wall), population q comes from the cell's own slot opp(q) -- Poiseulle.cu:601-746's
// d_dst[q][W] = d_dst[opp q][W + e_q] with W + e_q = c, read where it was stored.
// Plain (temporal) loads: the compact lattices' buffers stay in the caches from one step to the
// next: non-temporal -> plain loads took C4 from 8.13 to 7.75 us per step and the coronary tree
// from 35.9 to 31.2 us (profiles/r05_c1_temporal_ab.log)
template <bool SW, class A, class CT, int... Qs>
__device__ __forceinline__ void pull1_bb(float* f, const float* __restrict__ src, const A& ad, CT c, uint32_t wl,
                                         std::integer_sequence<int, Qs...>) {
  ((f[Qs] = *(
        src + ((wl >> Qs) & 1u ? fidx(c, Dir<Qs>::opp) : fidx(ad.template nb<Qs, SW>(), Qs)))),
   ...);
}

// One cell per lane (small lattices: a wave per 64 cells, so 4x the waves of the chunk path
// and a quarter of its per-wave latency): plain pulls, exact division, bounce-back slots.
// Plain (temporal) loads throughout the one-cell paths: their lattices stay in the caches
// between steps (LDC 64^3 11.13 -> 9.80 us per step against non-temporal loads,
// profiles/r05_temporal_ab.log)
template <bool SW, int... Qs>
__device__ __forceinline__ void pull1_all(float* f, const float* __restrict__ src, int64_t c, int pitch,
                                          int64_t plane, std::integer_sequence<int, Qs...>) {
  ((f[Qs] = *(src + aidx(c - cell_off<Qs, SW>(pitch, plane), Qs))), ...);
}

// The same pulls for a wave whose cells all lie in chunk ch (lane cell ch * 256 + l): a
// wave-uniform base W chunks below ch and 32-bit lane offsets (W * 256 >= plane + pitch + 1
// keeps them non-negative) -- 6 VALU per pull instead of the 64-bit aidx's ~10 (C4 10.8 ->
// 10.7 us per step, LDC 64^3 unchanged: the small lattices' chain is mostly latency)
__device__ __forceinline__ uint32_t rel_aidx(int r, int q) {
  return (uint32_t)(((r >> 8) * kQ + q) * kChunk + (r & (kChunk - 1)));
}
template <bool SW, int... Qs>
__device__ __forceinline__ void pull1w_all(float* f, const float* __restrict__ src, int64_t ch, int l, int pitch,
                                           int64_t plane, std::integer_sequence<int, Qs...>) {
  const int W = (int)((plane + pitch + 1) >> 8) + 2;
  const float* base = src + (ch - W) * (kQ * kChunk);
  const int r0 = l + W * kChunk;
  ((f[Qs] = *(base + rel_aidx(r0 - (int)cell_off<Qs, SW>(pitch, plane), Qs))), ...);
}

// one cell's collision and stores once its pulls, type byte and link masks are in
template <bool SW, bool PRE_BC, class A>
__device__ __forceinline__ double collide_cell1(const MainArgs& a, int64_t c, const A& ad, uint8_t t, uint32_t links,
                                                uint32_t nl, float* f, BcSlots pre_bc = BcSlots{}) {
  const bool in = ((c >= a.c_lo && c < a.c_hi) || (c >= a.c_lo2 && c < a.c_hi2)) && (t & kClassMask) == kFluid;
  if (!in) return 0.0;
  // NEE-adjacent: the boundary data goes out now and arrives under the arithmetic below
  // (PRE_BC: already loaded with the pulls)
  const bool nee = (t & kNeeAdj) != 0;
  BcSlots bc{};
  if constexpr (PRE_BC) bc = pre_bc;
  else if (nee) bc = nee_prefetch<SW>(a, c, nl);
  float rho = 0.f;
#pragma unroll
  for (int q = 0; q < kQ; ++q) rho = rho + f[q];
  const float ux = (f[1] - f[2] + f[7] + f[8] - f[9] - f[10] + f[11] + f[12] - f[13] - f[14]) / rho;
  const float uy = (f[3] - f[4] + f[7] - f[8] + f[9] - f[10] + f[15] - f[16] + f[17] - f[18]) / rho;
  const float uz = (f[5] - f[6] + f[11] - f[12] + f[13] - f[14] + f[15] + f[16] - f[17] - f[18]) / rho;
  if (__any(nee) && a.tau_fast && __all(fast_div_ok1(f, rho, ux, uy, uz))) {
    // (uniform) NEE values fused into the fast relaxation; nl = 0 on the other lanes
    relax_nee_fast_all<SW>(f, a, rho, ux, uy, uz, ad.get(), nee ? nl : 0u, bc, AllQ{});
  } else {
    const Pref pre = relax1(f, a, rho, ux, uy, uz);
    if (nee) nee_store_all<SW>(a, ad.get(), nl, bc, Post1{f}, rho, ux, uy, uz, pre, AllQ{});
  }
  fix_store_all<SW>(f, a.dst, c, ad, (t & kWallAdj) ? links : 0u, AllQ{});
  return (double)sqrtf(ux * ux + uy * uy + uz * uz);
}

// the pulls of pull1w_all with consumer-side bounce-back (MainArgs::bb_pull): where bit q of wl
// is set, population q comes from the cell's own slot opp(q)
template <bool SW, int... Qs>
__device__ __forceinline__ void pull1w_bb(float* f, const float* __restrict__ src, int64_t ch, int l, int pitch,
                                          int64_t plane, uint32_t wl, std::integer_sequence<int, Qs...>) {
  const int W = (int)((plane + pitch + 1) >> 8) + 2;
  const float* base = src + (ch - W) * (kQ * kChunk);
  const int r0 = l + W * kChunk;
  ((f[Qs] = *(
        base + ((wl >> Qs) & 1u ? rel_aidx(r0, Dir<Qs>::opp) : rel_aidx(r0 - (int)cell_off<Qs, SW>(pitch, plane), Qs)))),
   ...);
}

//  BOX: the device-generated cavity -- type byte and link masks from the coordinates, and (the
//        whole domain, bb_pull) bounce-back on the consumer side: the pulls of wall links read
//        the cell's own opposite slots, known before the first load
template <bool SW, bool BOX = false>
__device__ __forceinline__ double process_cell1(const MainArgs& a, int64_t ch, int l) {
  // the pulls go out with the type byte (one round trip; the guard chunks keep every
  // address of a lane that turns out to be idle inside the buffer)
  const int64_t c = ch * kChunk + l;
  float f[kQ];
  if constexpr (BOX) {
    const BoxCell b = box_cell(a, c);
    const bool pull_own = a.bb_pull && !a.bb_raw;
    pull1w_bb<SW>(f, a.src, ch, l, a.pitch, a.plane, pull_own ? b.links : 0u, AllQ{});
    return collide_cell1<SW, false>(a, c, AddrD{c, a.pitch, a.plane}, b.t, a.bb_pull ? 0u : b.links, b.nl, f);
  } else {
    const uint8_t t = a.type[c];
    const uint32_t links = a.links[c];  // unconditionally: no dependent round trip on t
    const uint32_t nl = a.nlinks[c];
    pull1w_all<SW>(f, a.src, ch, l, a.pitch, a.plane, AllQ{});
    return collide_cell1<SW, false>(a, c, AddrD{c, a.pitch, a.plane}, t, links, nl, f);
  }
}

// One cell per lane over a compact group list (sparse one-cell ranges): wave w takes the 16
// entries 16 w .., lanes 4k .. 4k+3 the four cells of entry 16 w + k.  Idle entries (bit 0)
// and the last wave's tail lanes point at a listed group, so their loads stay inside lines the
// wave reads anyway; they store nothing.  COMPACT: compact rows (Rows), the entry's row record
// loaded beside its type byte, then the pulls.
template <bool SW, bool COMPACT>
__device__ __forceinline__ double process_group_cell1(const MainArgs& a, int64_t w, int lane) {
  const int64_t gi = w * 16 + (lane >> 2);
  const int64_t gs = gi < a.ngroups ? gi : w * 16;
  const int e = a.groups[gs];
  const bool need = gi < a.ngroups && !(e & 1);
  const int64_t c = (int64_t)(e & ~3) + (lane & 3);
  const uint8_t t = a.type[c];
  const uint32_t links = a.links[c];
  const uint32_t nl = a.nlinks[c];
  float f[kQ];
  using A = std::conditional_t<COMPACT, RowsRef, AddrD>;
  A ad;
  if constexpr (COMPACT) {
    const int row = a.group_row[gs];
    pull1_addr<SW>(f, a.src, Rows::load(a.rowrec, c, row), AllQ{});
    ad = RowsRef{a.rowrec, c, row};
  } else {
    ad = AddrD{c, a.pitch, a.plane};
    pull1w_all<SW>(f, a.src, c >> 8, (int)(c & (kChunk - 1)), a.pitch, a.plane, AllQ{});  // per-lane chunk base
  }
  // the boundary records are indexed by the list entry, so they go out with the pulls instead
  // of a round trip after the NEE-link mask (group_bc is null when the list holds no
  // NEE-adjacent cell or every record is bc_const)
  const int gb = a.group_bc ? a.group_bc[gs] : -1;
  BcSlots bc{};
  if (a.bc_uniform) {
    bc = BcSlots{a.bc_const, a.bc_const, a.bc_const, a.bc_const, a.bc_const};
  } else if (gb >= 0) {
    const float4* r = a.group_rec + ((int64_t)gb * 4 + (lane & 3)) * kNeeSlots;
    bc = BcSlots{r[0], r[1], r[2], r[3], r[4]};
  }
  return collide_cell1<SW, true>(a, c, ad, need ? t : (uint8_t)0, links, nl, f, bc);
}

// One cell per lane over compact rows (small sparse lattices, latency-bound): wave w takes the 64
// consecutive compact cells from (c_lo & ~63) + 64 w -- no list, so nothing precedes the first
// round of loads: the type byte, link masks, boundary-record index and the group's row record
// (MainArgs::grouprec, the row record of every compact group) go out together, then the pulls.
// The walls, NEE and passive cells of the rows' spans ride along as idle lanes; a wave whose
// lanes hold no fluid cell issues no pulls.
template <bool SW>
__device__ __forceinline__ double process_compact_cell1(const MainArgs& a, int64_t w, int lane) {
  const int64_t c = (a.c_lo & ~int64_t(63)) + w * 64 + lane;
  if (c - lane >= a.c_hi) return 0.0;  // wave-uniform: past the range
  const int g = (int)(c >> 2);
  const uint8_t t = a.type[c];
  const uint32_t links = a.links[c];
  const uint32_t nl = a.nlinks[c];
  const int gb = a.group_bc ? a.group_bc[g] : -1;
  const Rows R = Rows::load(a.grouprec, c, g);
  const bool fluid = (t & kClassMask) == kFluid && c >= a.c_lo && c < a.c_hi;
  if (!__any(fluid)) return 0.0;  // wave-uniform: walls, NEE or passive cells only
  float f[kQ];
  // consumer-side bounce-back: the wall links select the cell's own slots (no wall stores below)
  const uint32_t wl = (a.bb_pull && !a.bb_raw && fluid && (t & kWallAdj)) ? links : 0u;
  pull1_bb<SW>(f, a.src, R, compact_id(c), wl, AllQ{});
  BcSlots bc{};
  if (a.bc_uniform) {
    bc = BcSlots{a.bc_const, a.bc_const, a.bc_const, a.bc_const, a.bc_const};
  } else if (gb >= 0) {
    const float4* r = a.group_rec + ((int64_t)gb * 4 + (lane & 3)) * kNeeSlots;
    bc = BcSlots{r[0], r[1], r[2], r[3], r[4]};
  }
  return collide_cell1<SW, true>(a, c, RowsRef{a.grouprec, c, g}, t, a.bb_pull ? 0u : links, nl, f, bc);
}

// One NEE-adjacent fluid cell of a 4-cell range (NEE blocks, one per thread): every static
// datum -- the cell id, its NEE-link mask, the boundary data of its first kNeeSlots NEE
// neighbours -- is indexed by the list position, so it all goes out in one round trip, then
// the 19 plain pulls and the wall links.  Collide, store the NEE neighbours' slots (producer
// side) and, unless the chunk waves do (nee_chunks), the cell's own slots and bounce-back
// slots.  With nee_chunks the chunk wave holding the cell collides it too, bit for bit the
// same, and stores its slots and |u| term: lanes whose NEE-adjacent cell shares its 4-cell
// group with other fluid cells (the pipe's rows along y) keep whole 16-B stores, and the NEE
// work (two dependent load rounds: link mask, then boundary data) stays out of the chunk waves.
template <bool SW, bool COMPACT>
__device__ __forceinline__ double nee_cell(const MainArgs& a, int i) {
  const int64_t c = a.cells[i];
  const uint32_t nl = a.cell_nl[i];
  const float4* r = a.nee_bc + (int64_t)i * kNeeSlots;
  const BcSlots bc = a.bc_uniform ? BcSlots{a.bc_const, a.bc_const, a.bc_const, a.bc_const, a.bc_const}
                                  : BcSlots{r[0], r[1], r[2], r[3], r[4]};
  // consumer-side bounce-back (compact rows): the wall links select the cell's own slots
  const bool consumer = COMPACT && a.bb_pull && !a.bb_raw;
  const uint32_t links = (a.nee_chunks && !consumer) ? 0u : a.links[c];
  float f[kQ];
  using A = std::conditional_t<COMPACT, RowsRef, AddrD>;
  A ad;
  if constexpr (COMPACT) {
    const int row = a.cell_row[i];
    pull1_bb<SW>(f, a.src, Rows::load(a.rowrec, c, row), compact_id(c), consumer ? links : 0u, AllQ{});
    ad = RowsRef{a.rowrec, c, row};
  } else {
    ad = AddrD{c, a.pitch, a.plane};
    pull1_all<SW>(f, a.src, c, a.pitch, a.plane, AllQ{});
  }
  float rho = 0.f;
#pragma unroll
  for (int q = 0; q < kQ; ++q) rho = rho + f[q];
  const float ux = (f[1] - f[2] + f[7] + f[8] - f[9] - f[10] + f[11] + f[12] - f[13] - f[14]) / rho;
  const float uy = (f[3] - f[4] + f[7] - f[8] + f[9] - f[10] + f[15] - f[16] + f[17] - f[18]) / rho;
  const float uz = (f[5] - f[6] + f[11] - f[12] + f[13] - f[14] + f[15] + f[16] - f[17] - f[18]) / rho;
  const Pref pre = relax1(f, a, rho, ux, uy, uz);
  nee_store_all<SW>(a, ad.get(), nl, bc, Post1{f}, rho, ux, uy, uz, pre, AllQ{});
  if (a.nee_chunks) return 0.0;  // the chunk wave stores the cell and sums its |u|
  fix_store_all<SW>(f, a.dst, c, ad, a.bb_pull ? 0u : links, AllQ{});
  return (double)sqrtf(ux * ux + uy * uy + uz * uz);
}

// NEE values after the step launch (MainArgs::nee_mac; single-domain 4-cell ranges whose chunk
// waves collide the NEE-adjacent cells, nee_chunks): a chunk wave recorded each such cell's
// (rho, u) of the step and stored its post-collision populations into its own slots of dst, so
// one thread per NEE-adjacent cell stores the values boundary_stream writes into its NEE
// neighbours (ldc.cu:391-456, Poiseulle.cu:748-891, bifurcation.cu:877-1021) -- the same values
// nee_cell computes, without nee_cell's 19 scattered pulls and its second collision of the cell.
// The prefactors RN(rho / d) by the exact division: the step's fast quotient is proven equal to
// it wherever the step used it.
template <int... Qs>
__device__ __forceinline__ void own_slots(float* f, const float* __restrict__ dst, int64_t c, uint32_t nl,
                                          std::integer_sequence<int, Qs...>) {
  ((f[Qs] = ((nl >> Qs) & 1u) ? dst[fidx(c, Qs)] : 0.0f), ...);
}
// One-wave workgroups: the list's few hundred waves spread over all CUs (C4 x4 133.3 -> 132.4,
// C3 185.9 -> 185.4 us per step against four-wave ones, profiles/r05_fix64_ab.log)
template <bool SW, bool COMPACT>
__global__ __launch_bounds__(64) void k_nee_fix(const MainArgs a) {
  if (a.stopped != nullptr && *a.stopped) return;  // uniform: converged, the step was a no-op
  const int i = blockIdx.x * 64 + (int)threadIdx.x;
  if (i >= a.n_nee) return;
  const int64_t c = a.cells[i];
  const uint32_t nl = a.cell_nl[i];
  const float4* rec = a.nee_bc + (int64_t)i * kNeeSlots;
  const BcSlots bc = a.bc_uniform ? BcSlots{a.bc_const, a.bc_const, a.bc_const, a.bc_const, a.bc_const}
                                  : BcSlots{rec[0], rec[1], rec[2], rec[3], rec[4]};
  const float4 m = a.nee_mac[a.cell_mac[i]];
  float f[kQ];
  own_slots(f, a.dst, c, nl, AllQ{});
  const Pref pre = Pref::exact(m.x);
  if constexpr (COMPACT) {
    const RowsRef ad{a.rowrec, c, a.cell_row[i]};
    nee_store_all<SW>(a, ad.get(), nl, bc, Post1{f}, m.x, m.y, m.z, m.w, pre, AllQ{});
  } else {
    nee_store_all<SW>(a, AddrD{c, a.pitch, a.plane}, nl, bc, Post1{f}, m.x, m.y, m.z, m.w, pre, AllQ{});
  }
}

// ---- the step kernel -------------------------------------------------------------------

__device__ void residual_logic(ConvState* cv, double S, float* hist_slot) {
  // ldc.cu:662-684: residual = |S_k - S_{k-1}| / S_k on fp32 sums
  const float sum_next = (float)S;
  const float residual = fabsf(sum_next - cv->sum_current) / sum_next;
  cv->residual = residual;
  cv->sum_current = sum_next;
  cv->k += 1;
  if (residual <= cv->tol) cv->tol_count += 1;
  if (cv->enabled) cv->stopped = !(cv->k <= cv->max_it && cv->tol_count <= cv->stag_max);
  // NaN guard (not in the reference, whose loop runs a diverged lattice on to max_it): the
  // first step whose |u| sum is not finite is recorded; under convergence control it also
  // stops the run (stopped = 2, lbm_get_state)
  if (!isfinite(S)) {
    if (cv->nonfinite_k == 0) cv->nonfinite_k = cv->k;
    if (cv->enabled) cv->stopped = 2;
  }
  if (hist_slot) *hist_slot = residual;
}

__device__ __forceinline__ int64_t chunk_of(const MainArgs& a, int idx) {
  return a.chunk0 >= 0 ? (int64_t)a.chunk0 + idx : (int64_t)a.chunks[idx];
}

template <bool FAST, bool QUARTER, bool SW, bool MASK = false, bool STRIDE = false, bool GROUPS = false,
          bool COMPACT = false, bool BOX = false, int WPB = kBlock / 64, bool REC = false>
__device__ __forceinline__ void step_body(const MainArgs& a) {  // WPB: wavefronts per workgroup
  __shared__ double red[WPB];
  if (a.stopped != nullptr && *a.stopped) return;  // uniform: converged, the step is a no-op
  double acc = 0.0;
  int slot;
  // the reduction group leads the grid, or trails it (red_last: a grid of one round of waves,
  // whose chunk waves then all start at once)
  const int nwork = a.nee_blocks + a.main_blocks;
  const int bd = a.red_last ? ((int)blockIdx.x < nwork ? (int)blockIdx.x : -1) : (int)blockIdx.x - a.red_blocks;
  // nee_last: the NEE blocks trail the chunk blocks in dispatch order; their logical places, and
  // with them the partial slots and the residual's summation order, do not change
  const int bx = (a.nee_last && bd >= 0) ? (bd < a.main_blocks ? bd + a.nee_blocks : bd - a.main_blocks) : bd;
  const int rb = a.red_last ? (int)blockIdx.x - nwork : (int)blockIdx.x;
  if (bx < 0) {  // reduction group: its first block finishes the previous step
    slot = rb;
    if (rb == 0 && a.red_partial != nullptr) {
      double t = 0.0;
      for (int i = threadIdx.x; i < a.red_n; i += WPB * 64) t += a.red_partial[i];  // fixed order
      t = block_sum(t, red);
      if (threadIdx.x == 0) {
        a.red_conv->s_local = t;
        residual_logic(a.red_conv, t, a.red_hist);
      }
      __syncthreads();  // red[] reuse below
    }
  } else if (bx >= a.nee_blocks) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // XCD-aware order: workgroups are dealt round-robin to the 8 XCDs (each with its own
    // L2), so logical block (b % 8) * (nb / 8) + b / 8 hands every XCD one contiguous run of
    // chunks and the lines two neighbouring chunks share stay in one L2 (-7% time at 512^3)
    const int b = bx - a.nee_blocks;  // red_blocks and nee_blocks are multiples of 8
    const int per = a.main_blocks >> 3, k = b >> 3, x = b & 7;
    if (a.xcd_run > 0) {
      // runs of P = 2^(xcd_run - 1) blocks, the XCDs' runs interleaved (XCD x takes runs 8j + x):
      // at any time the eight XCDs stream through neighbouring runs instead of eighths of the
      // buffers far apart (LBM_TUNE_XCD_RUN); the tail of an XCD's share that does not fill a
      // whole round of runs is split evenly as before
      const int sh = a.xcd_run - 1, full = (per >> sh) << sh;
      slot = k < full ? ((((k >> sh) << 3) + x) << sh) + (k & ((1 << sh) - 1)) : (full << 3) + x * (per - full) + (k - full);
    } else {
      slot = x * per + k;
    }
    const int idx = slot * (WPB) + wave;
    if constexpr (QUARTER && COMPACT) {  // one cell per lane over compact rows, no list
      acc = process_compact_cell1<SW>(a, idx, lane);
    } else if constexpr (QUARTER && GROUPS && STRIDE) {  // the same, grid-stride over XCD (b & 7)'s eighth
      const int64_t nw = (a.ngroups + 15) >> 4;
      const int64_t per = (nw + 7) >> 3;
      const int64_t lo = (b & 7) * per, hi = min(nw, lo + per);
      const int step = (a.main_blocks >> 3) * (WPB);
      for (int64_t i = lo + (b >> 3) * (WPB) + wave; i < hi; i += step) acc += process_group_cell1<SW, COMPACT>(a, i, lane);
    } else if constexpr (QUARTER && GROUPS) {  // one cell per lane over the compact group list
      if ((int64_t)idx * 16 < a.ngroups) acc = process_group_cell1<SW, COMPACT>(a, idx, lane);
    } else if constexpr (GROUPS && STRIDE) {  // compact groups, grid-stride over XCD (b & 7)'s eighth of the list
      const int64_t nw = (a.ngroups + 63) >> 6;  // 64-entry wave loads
      const int64_t per = (nw + 7) >> 3;
      const int64_t lo = (b & 7) * per, hi = min(nw, lo + per);
      const int step = (a.main_blocks >> 3) * (WPB);
      for (int64_t i = lo + (b >> 3) * (WPB) + wave; i < hi; i += step)
        acc += process_chunk<FAST, SW, false, true, COMPACT>(a, i * 64, lane, 0);
    } else if constexpr (GROUPS) {  // compact 4-cell groups: wave idx takes list entries 64 idx ..
      if ((int64_t)idx * 64 < a.ngroups) acc = process_chunk<FAST, SW, false, true, COMPACT>(a, (int64_t)idx * 64, lane, 0);
    } else if constexpr (QUARTER) {  // one cell per lane: wave idx takes quarter idx % 4 of chunk idx / 4
      if ((idx >> 2) < a.nchunks)
        acc = process_cell1<SW, BOX>(a, chunk_of(a, idx >> 2), (idx & 3) * 64 + lane);
    } else if constexpr (STRIDE) {  // grid-stride: XCD (b & 7) takes its eighth of the list in order
      const int per = (a.nchunks + 7) >> 3;
      const int lo = (b & 7) * per, hi = min(a.nchunks, lo + per);
      const int step = (a.main_blocks >> 3) * (WPB);
      for (int i = lo + (b >> 3) * (WPB) + wave; i < hi; i += step) {
        const uint64_t lm = MASK ? a.lane_masks[i] : ~0ull;
        acc += process_chunk<FAST, SW, MASK>(a, chunk_of(a, i) * kChunk, lane, lm, i);
      }
    } else if (idx < a.nchunks) {
      const uint64_t lm = MASK ? a.lane_masks[idx] : ~0ull;  // uniform, loaded beside the chunk id
      acc = process_chunk<FAST, SW, MASK, false, false, BOX, REC>(a, chunk_of(a, idx) * kChunk, lane, lm, idx);  // uniform base
    }
    slot += a.red_blocks + a.nee_blocks;
  } else {  // dispatched first: their scattered, latency-bound work hides under the chunks
    slot = a.red_blocks + bx;
    if constexpr (!QUARTER) {  // one-cell ranges have no NEE blocks
      const int w = (int)threadIdx.x >> 6;
      const int i = (bx * a.nee_waves + w) * 64 + ((int)threadIdx.x & 63);
      if (w < a.nee_waves && i < a.n_nee) acc = nee_cell<SW, COMPACT>(a, i);
    }
  }
  const double s = block_sum(acc, red);
  if (threadIdx.x == 0) a.partial[slot] = s;
}

// 4 cells per lane (big lattices): two waves per SIMD (210-253 VGPRs; one exact-division-only
// instance runs one); MASK: the range has lane masks (sparse chunk lists); COMPACT: compact
// rows (group lists only)
template <bool FAST, bool SW, bool MASK, bool STRIDE = false, bool GROUPS = false, bool COMPACT = false,
          bool BOX = false, bool REC = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(2))) void k_step(const MainArgs a) {
  step_body<FAST, false, SW, MASK, STRIDE, GROUPS, COMPACT, BOX, kBlock / 64, REC>(a);
}
// one cell per lane (small lattices, latency-bound): registers capped for four waves per SIMD
template <bool SW, bool GROUPS = false, bool STRIDE = false, bool COMPACT = false, bool BOX = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4))) void k_step1(const MainArgs a) {
  step_body<false, true, SW, false, STRIDE, GROUPS, COMPACT, BOX>(a);
}
// one cell per lane over compact rows without a list (vessel trees), two waves per workgroup
template <bool SW>
__global__ __launch_bounds__(kBlock1c) __attribute__((amdgpu_waves_per_eu(4))) void k_step1c(const MainArgs a) {
  step_body<false, true, SW, false, false, false, true, false, kBlock1c / 64>(a);
}

// ---- residual --------------------------------------------------------------------------

// slice b of the block partials -> out[b]
__global__ __launch_bounds__(256) void k_reduce_slices(const double* __restrict__ partial, int n,
                                                       double* __restrict__ out, const ConvState* cv) {
  __shared__ double red[4];
  if (cv->stopped) return;
  const int len = (n + gridDim.x - 1) / gridDim.x;
  const int lo = blockIdx.x * len, hi = min(n, lo + len);
  double s = 0.0;
  for (int i = lo + threadIdx.x; i < hi; i += blockDim.x) s += partial[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) out[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_reduce_final(const double* __restrict__ slices, int n, ConvState* cv,
                                                      double* local_out, float* hist_slot, int finish) {
  __shared__ double red[4];
  if (cv->stopped) return;
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += slices[i];  // fixed order
  s = block_sum(s, red);
  if (threadIdx.x == 0) {
    *local_out = s;
    if (finish) residual_logic(cv, s, hist_slot);
  }
}

// small launch ranges (n <= kReduceOneMax partials): the whole reduction in one block -- one
// launch less per step where launches dominate
constexpr int kReduceOneMax = 16384;
__global__ __launch_bounds__(512) void k_reduce_one(const double* __restrict__ partial, int n, ConvState* cv,
                                                     double* local_out, float* hist_slot, int finish) {
  __shared__ double red[8];
  if (cv->stopped) return;
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += partial[i];  // fixed order
  s = block_sum(s, red);
  if (threadIdx.x == 0) {
    *local_out = s;
    if (finish) residual_logic(cv, s, hist_slot);
  }
}

__global__ void k_finish_global(ConvState* cv, float* hist_slot) {
  if (cv->stopped) return;
  residual_logic(cv, cv->s_global, hist_slot);
}

// ---- halo pack / unpack ----------------------------------------------------------------

__global__ void k_pack(const float* __restrict__ f, float* __restrict__ buf, int zs, int64_t plane,
                       const int* __restrict__ qs, int nq) {
  const int64_t n = plane * nq;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(i / plane);
    const int64_t c = (int64_t)zs * plane + (i - k * plane);
    buf[i] = f[aidx(c, qs[k])];
  }
}

// skip_classes (bit per cell class): wall cells keep the bounce-back values their local
// producers stored (their consumer is on this rank); NEE cells are pulled raw only at step 0
__global__ void k_unpack(float* __restrict__ f, const float* __restrict__ buf, const uint8_t* __restrict__ type,
                         int zs, int64_t plane, const int* __restrict__ qs, int nq, unsigned skip_classes) {
  const int64_t n = plane * nq;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(i / plane);
    const int64_t c = (int64_t)zs * plane + (i - k * plane);
    const int cls = type[c] & kClassMask;
    if ((skip_classes >> cls) & 1u) continue;
    f[aidx(c, qs[k])] = buf[i];
  }
}

// LDC bounce-back already at step 0 (ldc.cu:75-202 swaps in place before the fluid reads):
// seed the wall slots of buffer f from the initial populations, as the producers would have
template <bool SW, int... Qs>
__device__ __forceinline__ void prime_cell(float* f, int64_t c, uint32_t m, int pitch, int64_t plane,
                                           std::integer_sequence<int, Qs...>) {
  (bb_store_one<Qs, SW>(f, AddrD{c, pitch, plane}, m, f[aidx(c, Dir<Qs>::opp)]), ...);
}
template <bool SW>
__global__ void k_bb_prime(float* f, const uint8_t* __restrict__ type, const uint32_t* __restrict__ links,
                           int64_t ncell, int pitch, int64_t plane) {
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < ncell; c += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t t = type[c];
    if ((t & kClassMask) != kFluid || !(t & kWallAdj)) continue;
    prime_cell<SW>(f, c, links[c], pitch, plane, AllQ{});
  }
}

// ---- geometry --------------------------------------------------------------------------

// storage cell -> physical (x, y, storage plane zs): c + shift = s0 + s1*pitch + zs*plane with
// (s0, s1) = (x, y), or (y, x) when the rows run along y; in = inside the box's rows
struct CellPos {
  int x, y, zs;
  bool in;
};
__device__ __forceinline__ CellPos cell_pos(int64_t c, int shift, int pitch, int64_t plane, int nx, int ny, int swap) {
  const int64_t u = c + shift;
  const int s0 = (int)(u % pitch);
  const int n1 = swap ? nx : ny;
  const int s1 = (int)((u / pitch) % n1);
  CellPos p;
  p.zs = (int)(u / plane);
  p.x = swap ? s1 : s0;
  p.y = swap ? s0 : s1;
  p.in = s0 < (swap ? ny : nx);
  return p;
}

// reference code -> class/face/kind; NEE data into the macro arrays of NEE cells (read by the
// fluid neighbours that store their NEE values, nee_store_q)
__global__ void k_classify(const GeoArgs g) {
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < g.ncell;
       c += (int64_t)gridDim.x * blockDim.x) {
    const int code = g.codes[c];
    const CellPos p = cell_pos(c, g.xshift, g.pitch, g.plane, g.nx, g.ny, g.swap);
    const int x = p.x, zs = p.zs;
    const int zg = zs - 1 + g.z_offset;  // global z
    uint8_t t = kPassive;
    // NaN in the rho slot of a velocity boundary: rho_bc is the fluid neighbour's; NaN in the u
    // slots of a pressure boundary: u_bc is the fluid neighbour's (nee_value)
    const float kRhoOfFluid = __builtin_nanf(""), kUOfFluid = __builtin_nanf("");
    if (p.in && zs < g.planes) {
      const int y = p.y;
      if (g.case_kind == 0) {  // LDC (ldc.cu:469): 0 ghost, 1 wall, 2 lid, 3 fluid
        if (code == 1) t = kWall;
        else if (code == 3) t = kFluid;
        else if (code == 2) {  // lid supplies {4,8,10,16,18} (ldc.cu:391-456), u = (0, 0, u_lid)
          t = make_nee(kFaceNY, false);
          g.rho[c] = kRhoOfFluid; g.ux[c] = 0.f; g.uy[c] = 0.f; g.uz[c] = g.lid_u;
        }
      } else if (g.case_kind == 3) {  // generic: 4 fluid, 1 wall, boundary codes by table
        if (code == 4) t = kFluid;
        else if (code == 1) t = kWall;
        else {
          for (int k = 0; k < g.nbc; ++k) {
            const BcCode& b = g.bcs[k];
            if (b.code != code) continue;
            t = make_nee(b.face, b.kind == 2);
            float v[3] = {b.u[0], b.u[1], b.u[2]};
            const int axis = b.face >> 1;
            if (b.table && zg >= 0 && zg < g.nz_global) {
              const int64_t ti = axis == 0 ? y + (int64_t)zg * g.ny : axis == 1 ? x + (int64_t)zg * g.nx
                                                                                 : x + (int64_t)y * g.nx;
              v[axis] = b.table[ti];
            }
            g.rho[c] = b.kind == 0 ? kRhoOfFluid : b.rho;
            if (b.kind == 2) v[0] = v[1] = v[2] = kUOfFluid;
            g.ux[c] = v[0]; g.uy[c] = v[1]; g.uz[c] = v[2];
            break;
          }
        }
      } else {  // Poiseuille / mask (README.md:9-14)
        const bool in_tab = zg >= 0 && zg < g.nz_global;
        if (code == 1) t = kWall;
        else if (code == 4) t = kFluid;
        else if (code == 2) {   // inlet: +y face {3,7,9,15,17}, u = (0, inlet_uy(x,z), 0)
          t = make_nee(kFacePY, false);
          const float v = (g.inlet_uy && in_tab) ? g.inlet_uy[x + (int64_t)zg * g.nx] : 0.f;
          g.rho[c] = kRhoOfFluid; g.ux[c] = 0.f; g.uy[c] = v; g.uz[c] = 0.f;
        } else if (code == 3) { // outlet: -y face {4,8,10,16,18}
          if (g.case_kind == 1) {  // Poiseuille: velocity, u = (0, outlet_uy(x,z), 0)
            t = make_nee(kFaceNY, false);
            const float v = (g.outlet_uy && in_tab) ? g.outlet_uy[x + (int64_t)zg * g.nx] : 0.f;
            g.rho[c] = kRhoOfFluid; g.ux[c] = 0.f; g.uy[c] = v; g.uz[c] = 0.f;
          } else {                 // bifurcation: pressure, rho = 1 (bifurcation.cu:890)
            t = make_nee(kFaceNY, true);
            g.rho[c] = 1.0f; g.ux[c] = kUOfFluid; g.uy[c] = kUOfFluid; g.uz[c] = kUOfFluid;
          }
        }
      }
    }
    g.type[c] = t;
  }
}

template <int Q, bool SW>
__device__ __forceinline__ void scan_nb(const uint8_t* type, int64_t c, const GeoArgs& g, uint8_t& flags,
                                        uint32_t& walls, uint32_t& nees) {
  const int64_t nb = c - cell_off<Q, SW>(g.pitch, g.plane);
  if (Q == 0 || nb < 0 || nb >= g.ncell) return;
  const uint8_t tn = type[nb];
  const int cls = tn & kClassMask;
  if (cls == kWall) {
    flags |= kWallAdj;
    walls |= 1u << Q;
  }
  // an NEE cell supplies q when q crosses its face (boundary_stream's direction sets)
  if (cls == kNee && ((face_bits<Q>() >> nee_face(tn)) & 1)) {
    flags |= kNeeAdj;
    nees |= 1u << Q;
  }
}

template <bool SW, int... Qs>
__device__ __forceinline__ void scan_all(const uint8_t* type, int64_t c, const GeoArgs& g, uint8_t& flags,
                                         uint32_t& walls, uint32_t& nees, std::integer_sequence<int, Qs...>) {
  (scan_nb<Qs, SW>(type, c, g, flags, walls, nees), ...);
}

template <bool SW>
__global__ void k_flag_fluid(const GeoArgs g) {
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < g.ncell;
       c += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t t = g.type[c];
    if ((t & kClassMask) != kFluid) continue;
    uint8_t flags = 0;
    uint32_t walls = 0, nees = 0;
    scan_all<SW>(g.type, c, g, flags, walls, nees, AllQ{});
    g.type[c] = (uint8_t)(t | flags);
    g.links[c] = walls;
    g.nlinks[c] = nees;
  }
}

// passive cells some fluid cell pulls from (malformed geometry, the reference reads their
// initial values forever): flag them so the main kernel never overwrites them
template <bool SW, int... Qs>
__device__ __forceinline__ bool pulled_by_fluid(const uint8_t* type, int64_t c, const GeoArgs& g,
                                                std::integer_sequence<int, Qs...>) {
  auto fl = [&](int64_t n) { return n >= 0 && n < g.ncell && (type[n] & kClassMask) == kFluid; };
  return (fl(c + cell_off<Qs, SW>(g.pitch, g.plane)) || ...);
}

template <bool SW>
__global__ void k_mark_pulled(const GeoArgs g) {
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < g.ncell;
       c += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t t = g.type[c];
    if ((t & kClassMask) == kPassive && pulled_by_fluid<SW>(g.type, c, g, AllQ{})) g.type[c] = (uint8_t)(t | kPulled);
  }
}

__global__ void k_ldc_codes(int8_t* codes, int nx, int ny, int pitch, int xshift, int64_t plane, int64_t ncell,
                            int z_offset, int nzg, int swap) {
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < ncell;
       c += (int64_t)gridDim.x * blockDim.x) {
    const CellPos p = cell_pos(c, xshift, pitch, plane, nx, ny, swap);
    const int x = p.x, y = p.y;
    const int z = p.zs - 1 + z_offset;
    int8_t code = 0;  // ldc.cu:468-502
    if (p.in && z >= 0 && z < nzg) {
      if (x >= 1 && x < nx - 1 && y >= 1 && y < ny - 1 && z >= 1 && z < nzg - 1) code = 1;
      if (x >= 2 && x < nx - 2 && y >= 2 && y < ny - 2 && z >= 2 && z < nzg - 2) code = 3;
      if (y == ny - 2 && x >= 1 && x < nx - 1 && z >= 1 && z < nzg - 1) code = 2;
    }
    codes[c] = code;
  }
}

// ---- geo_pre of a raw mask on the device (bifurcation.cu:63-239) -------------
// Global coordinates throughout; the mask holds planes zbase .. zbase + mplanes - 1.
struct MaskGeo {
  const uint8_t* m;
  int nx, ny, nzg, zbase;
};

__device__ __forceinline__ int mraw(const MaskGeo& g, int x, int y, int z) {
  return g.m[x + (int64_t)g.nx * (y + (int64_t)g.ny * (z - g.zbase))];
}

// min over the 6 face neighbours (the reference's distance-transform step)
__device__ __forceinline__ int mmin6(const MaskGeo& g, int x, int y, int z) {
  int v = min(mraw(g, x + 1, y, z), mraw(g, x - 1, y, z));
  v = min(v, min(mraw(g, x, y + 1, z), mraw(g, x, y - 1, z)));
  return min(v, min(mraw(g, x, y, z + 1), mraw(g, x, y, z - 1)));
}

// the code before ghost marking: y = 0 / ny-1 planes cleared, interior += 3*min6, inlet row
// y = 1 and outlet row y = ny-2 from the row next to them (requires ny >= 5)
__device__ int mask_pre(const MaskGeo& g, int x, int y, int z) {
  if (x < 1 || x > g.nx - 2 || z < 1 || z > g.nzg - 2) return mraw(g, x, y, z);
  if (y == 0 || y == g.ny - 1) return 0;
  if (y == 1) {
    const int in = mraw(g, x, 2, z) + 3 * mmin6(g, x, 2, z);
    return in == 1 ? 1 : (in == 4 ? 2 : 0);
  }
  if (y == g.ny - 2) {
    const int out = mraw(g, x, g.ny - 3, z) + 3 * mmin6(g, x, g.ny - 3, z);
    return out == 1 ? 1 : (out == 4 ? 3 : 0);
  }
  return mraw(g, x, y, z) + 3 * mmin6(g, x, y, z);
}

// final code: an unused cell next to an interior wall (code 1) becomes a ghost (-1).  The
// reference scatters from each wall to its 18 neighbours; only 0 -> -1 changes, so gathering
// from the 18 neighbours gives the same codes in any order.
__device__ int mask_code(const MaskGeo& g, int x, int y, int z) {
  const int v = mask_pre(g, x, y, z);
  if (v != 0) return v;
  for (int q = 1; q < kQ; ++q) {
    const int sx = x - kEx[q], sy = y - kEy[q], sz = z - kEz[q];
    if (sx >= 1 && sx <= g.nx - 2 && sy >= 1 && sy <= g.ny - 2 && sz >= 1 && sz <= g.nzg - 2 &&
        mask_pre(g, sx, sy, sz) == 1)
      return -1;
  }
  return 0;
}

// first fluid (code 4) position along every storage row (x rows, or y rows when swap) of
// planes z_lo .. z_hi-1 -> hist[pos & 3] (choose_xshift)
__global__ void k_mask_hist(MaskGeo g, int z_lo, int z_hi, unsigned long long* hist, int swap) {
  const int n0 = swap ? g.ny : g.nx, n1 = swap ? g.nx : g.ny;
  const int64_t rows = (int64_t)(z_hi - z_lo) * n1;
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < rows; r += (int64_t)gridDim.x * blockDim.x) {
    const int s1 = (int)(r % n1), z = z_lo + (int)(r / n1);
    if (z < 0 || z >= g.nzg) continue;
    for (int s0 = 0; s0 < n0; ++s0)
      if (mask_code(g, swap ? s1 : s0, swap ? s0 : s1, z) == 4) {
        atomicAdd(&hist[s0 & 3], 1ull);
        break;
      }
  }
}

// codes of every storage cell (layout order, as k_ldc_codes); storage planes outside
// z_lo .. z_hi-1 (local) or outside the global box stay 0
__global__ void k_mask_codes(MaskGeo g, int8_t* codes, int pitch, int xshift, int64_t plane, int64_t ncell,
                             int z_offset, int z_lo, int z_hi, int swap) {
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < ncell;
       c += (int64_t)gridDim.x * blockDim.x) {
    const CellPos p = cell_pos(c, xshift, pitch, plane, g.nx, g.ny, swap);
    const int zl = p.zs - 1;
    const int z = zl + z_offset;
    int8_t code = 0;
    if (p.in && zl >= z_lo && zl < z_hi && z >= 0 && z < g.nzg) code = (int8_t)mask_code(g, p.x, p.y, z);
    codes[c] = code;
  }
}

// ---- initial state ---------------------------------------------------------------------

// bifurcation.cu:329-427 on the device: rho = 1, u = 0 except u_y of the inlet (code 2, row
// y = 1) and outlet (code 3, row y = ny-2) cells of the local planes, from the bc tables
// (x + global z * nx); expanded equilibrium into both buffers
__global__ void k_init_mask(float* fa, float* fb, const int8_t* codes, const float* in_uy, const float* out_uy, int nx,
                            int ny, int nz, int pitch, int xshift, int64_t plane, int64_t ncell, int z_offset,
                            int swap) {
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < ncell;
       c += (int64_t)gridDim.x * blockDim.x) {
    const CellPos p = cell_pos(c, xshift, pitch, plane, nx, ny, swap);
    const int x = p.x, y = p.y;
    const int zl = p.zs - 1;
    float vy = 0.0f;
    if (p.in && zl >= 0 && zl < nz) {
      const int64_t t = x + (int64_t)(zl + z_offset) * nx;
      if (y == 1 && codes[c] == 2 && in_uy) vy = in_uy[t];
      if (y == ny - 2 && codes[c] == 3 && out_uy) vy = out_uy[t];
    }
    float e[kQ];
    feq_expanded(1.0f, 0.0f, vy, 0.0f, e);
#pragma unroll
    for (int q = 0; q < kQ; ++q) { fa[aidx(c, q)] = e[q]; fb[aidx(c, q)] = e[q]; }
  }
}

__global__ void k_init_feq(float* fa, float* fb, int64_t n, int form, const float* rho, const float* ux,
                           const float* uy, const float* uz) {
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < n; c += (int64_t)gridDim.x * blockDim.x) {
    const float r = rho ? rho[c] : 1.0f;
    const float vx = ux ? ux[c] : 0.0f, vy = uy ? uy[c] : 0.0f, vz = uz ? uz[c] : 0.0f;
    float e[kQ];
    if (form == 0) feq_init_wi(r, vx, vy, vz, e);
    else feq_expanded(r, vx, vy, vz, e);
#pragma unroll
    for (int q = 0; q < kQ; ++q) { fa[aidx(c, q)] = e[q]; fb[aidx(c, q)] = e[q]; }
  }
}

__global__ void k_init_ldc(float* fa, float* fb, int64_t n, int pitch, int xshift, int nx, int ny, float lid_u,
                           int swap) {
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < n; c += (int64_t)gridDim.x * blockDim.x) {
    const int y = cell_pos(c, xshift, pitch, (int64_t)pitch * (swap ? nx : ny), nx, ny, swap).y;
    // ldc.cu:510-532: rho 1, u 0; uz = u_max on y = ny-1 and y = ny-2
    const float uz = (y == ny - 1 || y == ny - 2) ? lid_u : 0.0f;
    float e[kQ];
    feq_init_wi(1.0f, 0.0f, 0.0f, uz, e);
#pragma unroll
    for (int q = 0; q < kQ; ++q) { fa[aidx(c, q)] = e[q]; fb[aidx(c, q)] = e[q]; }
  }
}

// ---- macros, read out lazily ------------------------------------------------------------
// The step kernels store no macros.  lbm_get_macros recomputes the last step's (rho, u) of
// every fluid cell from that step's source buffer, which the step left intact (A-B
// pattern): the same 19 pulls and the same fp32 sums as process_chunk / process_cell1, so
// the bits are those the step used (NEE values included: they sit in the boundary cells'
// slots of that buffer, stored there by the step before).
// bb_links (nullable): consumer-side bounce-back (MainArgs::bb_pull) -- wall-linked populations
// from the cell's own opposite slots
template <bool SW, int... Qs>
__device__ __forceinline__ void pull1_links(float* f, const float* __restrict__ src, int64_t c, uint32_t wl, int pitch,
                                            int64_t plane, std::integer_sequence<int, Qs...>) {
  ((f[Qs] = src[(wl >> Qs) & 1u ? aidx(c, Dir<Qs>::opp) : aidx(c - cell_off<Qs, SW>(pitch, plane), Qs)]), ...);
}
template <bool SW>
__global__ void k_moments(const float* __restrict__ src, const uint8_t* __restrict__ type, const uint32_t* bb_links,
                          float* rho, float* ux, float* uy, float* uz, int64_t lo, int64_t hi, int pitch, int64_t plane) {
  for (int64_t c = lo + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < hi; c += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t t = type[c];
    if ((t & kClassMask) != kFluid) continue;
    float f[kQ];
    pull1_links<SW>(f, src, c, (bb_links && (t & kWallAdj)) ? bb_links[c] : 0u, pitch, plane, AllQ{});
    float r = 0.f;
#pragma unroll
    for (int q = 0; q < kQ; ++q) r = r + f[q];
    rho[c] = r;
    ux[c] = (f[1] - f[2] + f[7] + f[8] - f[9] - f[10] + f[11] + f[12] - f[13] - f[14]) / r;
    uy[c] = (f[3] - f[4] + f[7] - f[8] + f[9] - f[10] + f[15] - f[16] + f[17] - f[18]) / r;
    uz[c] = (f[5] - f[6] + f[11] - f[12] + f[13] - f[14] + f[15] + f[16] - f[17] - f[18]) / r;
  }
}

// the same read-out over compact rows (lbm_ctx::compact), without a dense staging copy: compact
// cell i pulls through its row record (rowrec[row_of[i / 4]], as the step kernels address it)
// and writes the dense cell cmap[i]'s macros
template <bool SW>
__global__ void k_moments_compact(const float* __restrict__ src, const uint8_t* __restrict__ type,
                                  const uint32_t* bb_links, const int* __restrict__ cmap,
                                  const int* __restrict__ row_of, const int4* __restrict__ rowrec, float* rho,
                                  float* ux, float* uy, float* uz, int64_t lo, int64_t hi) {
  for (int64_t c = lo + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < hi; c += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t t = type[c];
    const int d = cmap[c];
    if ((t & kClassMask) != kFluid || d < 0) continue;
    float f[kQ];
    pull1_bb<SW>(f, src, Rows::load(rowrec, c, row_of[c >> 2]), compact_id(c),
                 (bb_links && (t & kWallAdj)) ? bb_links[c] : 0u, AllQ{});
    float r = 0.f;
#pragma unroll
    for (int q = 0; q < kQ; ++q) r = r + f[q];
    rho[d] = r;
    ux[d] = (f[1] - f[2] + f[7] + f[8] - f[9] - f[10] + f[11] + f[12] - f[13] - f[14]) / r;
    uy[d] = (f[3] - f[4] + f[7] - f[8] + f[9] - f[10] + f[15] - f[16] + f[17] - f[18]) / r;
    uz[d] = (f[5] - f[6] + f[11] - f[12] + f[13] - f[14] + f[15] + f[16] - f[17] - f[18]) / r;
  }
}

// ---- reference-order fp32 residual (opt-in) -----------------------------------------------
// calc_vel_square (ldc.cu:460-466): the step's |u| per fluid cell -- from the step's source
// buffer, the same pulls and sums as the step (k_moments) -- into its reference storage slot
template <bool SW>
__global__ void k_vel_terms(const float* __restrict__ src, const uint8_t* __restrict__ type, const uint32_t* bb_links,
                            const int* __restrict__ ref_idx, float* __restrict__ terms, int64_t lo, int64_t hi,
                            int pitch, int64_t plane) {
  for (int64_t c = lo + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < hi; c += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t t = type[c];
    if ((t & kClassMask) != kFluid) continue;
    float f[kQ];
    pull1_links<SW>(f, src, c, (bb_links && (t & kWallAdj)) ? bb_links[c] : 0u, pitch, plane, AllQ{});
    float r = 0.f;
#pragma unroll
    for (int q = 0; q < kQ; ++q) r = r + f[q];
    const float ux = (f[1] - f[2] + f[7] + f[8] - f[9] - f[10] + f[11] + f[12] - f[13] - f[14]) / r;
    const float uy = (f[3] - f[4] + f[7] - f[8] + f[9] - f[10] + f[15] - f[16] + f[17] - f[18]) / r;
    const float uz = (f[5] - f[6] + f[11] - f[12] + f[13] - f[14] + f[15] + f[16] - f[17] - f[18]) / r;
    terms[ref_idx[c]] = sqrtf(ux * ux + uy * uy + uz * uz);
  }
}

// the same over compact rows (cell i pulls through its row record as k_moments_compact does),
// each term into the reference slot of its dense cell cmap[i]
template <bool SW>
__global__ void k_vel_terms_compact(const float* __restrict__ src, const uint8_t* __restrict__ type,
                                    const uint32_t* bb_links, const int* __restrict__ cmap,
                                    const int* __restrict__ row_of, const int4* __restrict__ rowrec,
                                    const int* __restrict__ ref_idx, float* __restrict__ terms, int64_t lo, int64_t hi) {
  for (int64_t c = lo + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < hi; c += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t t = type[c];
    const int d = cmap[c];
    if ((t & kClassMask) != kFluid || d < 0) continue;
    float f[kQ];
    pull1_bb<SW>(f, src, Rows::load(rowrec, c, row_of[c >> 2]), compact_id(c),
                 (bb_links && (t & kWallAdj)) ? bb_links[c] : 0u, AllQ{});
    float r = 0.f;
#pragma unroll
    for (int q = 0; q < kQ; ++q) r = r + f[q];
    const float ux = (f[1] - f[2] + f[7] + f[8] - f[9] - f[10] + f[11] + f[12] - f[13] - f[14]) / r;
    const float uy = (f[3] - f[4] + f[7] - f[8] + f[9] - f[10] + f[15] - f[16] + f[17] - f[18]) / r;
    const float uz = (f[5] - f[6] + f[11] - f[12] + f[13] - f[14] + f[15] + f[16] - f[17] - f[18]) / r;
    terms[ref_idx[d]] = sqrtf(ux * ux + uy * uy + uz * uz);
  }
}

// CUB's block reduction (BLOCK_REDUCE_WARP_REDUCTIONS) with 32-lane logical warps on the
// 64-lane wavefront: a shuffle-down tree per warp (offsets 1 .. 16; a lane adds its partner's
// value only when the partner holds data), then thread 0 adds the warp sums in warp order.
// num_valid: threads holding data (a prefix of the block).  Result valid in thread 0.
__device__ float cub_block_sum(float x, int num_valid, float* warp_sums) {
  const int t = threadIdx.x, w = t >> 5, l = t & 31;
  const int valid = min(32, max(0, num_valid - 32 * w));
#pragma unroll
  for (int off = 1; off < 32; off <<= 1) {
    const float y = __shfl_down(x, off, 32);
    if (l + off < valid) x = y + x;
  }
  if (l == 0) warp_sums[w] = x;
  __syncthreads();
  float s = 0.f;
  if (t == 0) {
    s = warp_sums[0];
    for (int k = 1; k < 8; ++k)
      if (32 * k < num_valid) s = s + warp_sums[k];
  }
  return s;
}

// pass 1 (AgentReduce over an even share of tiles): in a full tile thread t folds the vec-wide
// vectors at vec * t + 256 * vec * i, in a partial tile t, t + 256, ...
__global__ __launch_bounds__(256) void k_cub_pass1(const float* __restrict__ v, int64_t n, int ipt, int vec,
                                                   float* __restrict__ partials, const ConvState* cv) {
  __shared__ float warp_sums[8];
  if (cv->stopped) return;
  const int64_t tile = 256LL * ipt;
  const int64_t tiles = (n + tile - 1) / tile;
  const int64_t grid = gridDim.x, b = blockIdx.x;
  const int64_t avg = tiles / grid, big = tiles - avg * grid;
  const int64_t t0 = b < big ? b * (avg + 1) : big * (avg + 1) + (b - big) * avg;
  int64_t off = t0 * tile, end = off + (avg + (b < big ? 1 : 0)) * tile;
  if (end > n) end = n;
  const int t = threadIdx.x;
  float x = 0.f;
  bool have = false;
  int num_valid = 256;
  for (; off + tile <= end; off += tile)
    for (int i = 0; i < ipt / vec; ++i)
      for (int k = 0; k < vec; ++k) {
        const float y = v[off + (int64_t)vec * t + 256LL * vec * i + k];
        x = have ? x + y : y;
        have = true;
      }
  if (off < end) {
    const int64_t valid = end - off;
    if (!have) num_valid = valid < 256 ? (int)valid : 256;
    for (int64_t i = t; i < valid; i += 256) {
      const float y = v[off + i];
      x = have ? x + y : y;
      have = true;
    }
  }
  const float s = cub_block_sum(x, num_valid, warp_sums);
  if (t == 0) partials[b] = s;
}

// pass 2 (the single-tile kernel over the partials) + the residual logic on S = 0.f + sum
__global__ __launch_bounds__(256) void k_cub_pass2(const float* __restrict__ partials, int grid, ConvState* cv,
                                                   float* hist_slot) {
  __shared__ float warp_sums[8];
  if (cv->stopped) return;
  const int t = threadIdx.x;
  float x = 0.f;
  bool have = false;
  for (int i = t; i < grid; i += 256) {
    x = have ? x + partials[i] : partials[i];
    have = true;
  }
  const float s = cub_block_sum(x, grid < 256 ? grid : 256, warp_sums);
  if (t == 0) {
    const float S = 0.f + s;  // thrust::reduce's init value
    cv->s_local = (double)S;
    residual_logic(cv, (double)S, hist_slot);
  }
}

// ---- field digest ------------------------------------------------------------------------
// Per local plane: the wrapping 64-bit sum over its fluid cells of a hash of (global x, y, z,
// the bits of rho, ux, uy, uz).  Addition mod 2^64 is order-free, so the digest depends on
// the fields and global coordinates only -- not on the layout, the launch shape or how the
// lattice is cut into slabs.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {  // splitmix64 finaliser
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__global__ void k_digest(const uint8_t* __restrict__ type, const float* __restrict__ rho, const float* __restrict__ ux,
                         const float* __restrict__ uy, const float* __restrict__ uz, int nx, int ny, int pitch,
                         int xshift, int64_t plane, int z_offset, int swap, unsigned long long* out) {
  __shared__ unsigned long long part[4];
  const int zl = blockIdx.y;  // local plane
  uint64_t acc = 0;
  const int n1 = swap ? nx : ny;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < (int64_t)pitch * n1;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int s0 = (int)(i % pitch), s1 = (int)(i / pitch);
    if (s0 >= (swap ? ny : nx)) continue;
    const int64_t c = s0 - xshift + (int64_t)s1 * pitch + (int64_t)(zl + 1) * plane;
    if (c < 0 || (type[c] & kClassMask) != kFluid) continue;
    const int x = swap ? s1 : s0, y = swap ? s0 : s1;
    const uint64_t key = (uint64_t)x | ((uint64_t)y << 21) | ((uint64_t)(zl + z_offset) << 42);
    uint64_t h = mix64(key + 0x9e3779b97f4a7c15ull);
    h = mix64(h ^ __float_as_uint(rho[c]));
    h = mix64(h ^ ((uint64_t)__float_as_uint(ux[c]) << 32 | __float_as_uint(uy[c])));
    h = mix64(h ^ __float_as_uint(uz[c]));
    acc += h;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out + zl, part[0] + part[1] + part[2] + part[3]);
}

// ---- compact rows <-> the dense box ---------------------------------------------------------
// cmap[i]: the dense cell of compact cell i (-1: a slot outside its row, which holds no cell).
// Populations: slot q of every mapped cell, both directions; per-cell arrays: gathered.
__global__ void k_pop_gather(float* __restrict__ dc, const float* __restrict__ sd, const int* __restrict__ cmap,
                             int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n * kQ; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t cell = i / kQ;
    const int q = (int)(i - cell * kQ);
    const int d = cmap[cell];
    dc[aidx(cell, q)] = d >= 0 ? sd[aidx(d, q)] : 0.0f;
  }
}
__global__ void k_pop_scatter(float* __restrict__ dd, const float* __restrict__ sc, const int* __restrict__ cmap,
                              int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n * kQ; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t cell = i / kQ;
    const int q = (int)(i - cell * kQ);
    const int d = cmap[cell];
    if (d >= 0) dd[aidx(d, q)] = sc[aidx(cell, q)];
  }
}
// test hook (lbm_debug_poison_walls): a quiet NaN into all 19 slots of every wall cell of f
__global__ void k_poison_walls(float* __restrict__ f, const uint8_t* __restrict__ type, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n * kQ; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t cell = i / kQ;
    const int q = (int)(i - cell * kQ);
    if ((type[cell] & kClassMask) == kWall) f[aidx(cell, q)] = __builtin_nanf("");
  }
}
template <class T>
__global__ void k_cell_gather(T* __restrict__ dc, const T* __restrict__ sd, const int* __restrict__ cmap, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int d = cmap[i];
    dc[i] = d >= 0 ? sd[d] : T(0);
  }
}

int grid_for(int64_t n, int block) {
  int64_t g = (n + block - 1) / block;
  if (g > 65536) g = 65536;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

bool verify_fast_div(float tau) {
  if (!(tau >= 0.0625f && tau <= 16.0f)) return false;
  // the equilibria's prefactor divisors take the same shortcut (Pref): checked once
  static const bool consts = verify_fast_div_by(3.0f) && verify_fast_div_by(18.0f) && verify_fast_div_by(36.0f);
  return consts && verify_fast_div_by(tau);
}

bool verify_fast_div_by(float tau) {
  const float y = 1.0f / tau;
  for (uint32_t m = 0; m < (1u << 23); ++m) {
    uint32_t bits = 0x3f800000u | m;
    float x;
    std::memcpy(&x, &bits, 4);
    const float q0 = x * y;
    const float r = std::fma(-q0, tau, x);
    const float q = std::fma(r, y, q0);
    if (q != x / tau) return false;
  }
  return true;
}

// chunk blocks of k_step: a multiple of the 8 XCDs (see k_step)
int main_grid(int nchunks, bool quarter) {
  const int waves = quarter ? 4 * nchunks : nchunks;
  return nchunks ? std::max(8, ((waves + kBlock / 64 - 1) / (kBlock / 64) + 7) / 8 * 8) : 0;
}

// NEE blocks of k_step (first in the grid): a multiple of 8 so the chunk blocks keep their XCD
int nee_waves_for(int n, double contiguous) { return (n <= 16384 && contiguous < 0.5) ? 1 : kBlock / 64; }
int nee_grid(int n, int waves) { return (n + 8 * 64 * waves - 1) / (8 * 64 * waves) * 8; }

// Two waves per SIMD measured fastest (3.71 vs 3.83 ms at 512^3 with three, 5.2+ with one);
// the 4-cell kernel's register count (214 VGPRs, kernel-resource-usage) gives exactly that.
hipError_t launch_step(const MainArgs& a, hipStream_t s) {
  const dim3 grid(a.red_blocks + a.nee_blocks + a.main_blocks);
  typedef void (*Kern)(const MainArgs);
  const bool sw = a.swap != 0;
  Kern k;
  const size_t lds = 0;
  if (a.box && !a.swap && !a.groups && !a.chunk_stride) {  // the device-generated cavity
    if (a.quarter) k = k_step1<false, false, false, false, true>;
    else if (a.fast_div) k = a.lane_masks ? k_step<true, false, true, false, false, false, true>
                                          : k_step<true, false, false, false, false, false, true>;
    else k = a.lane_masks ? k_step<false, false, true, false, false, false, true>
                          : k_step<false, false, false, false, false, false, true>;
  } else if (a.rowrec) {  // compact rows: one cell per lane without a list, or 4-cell group lists
    if (a.quarter) {
      if (!a.grouprec) return hipErrorInvalidValue;
      k = sw ? k_step1c<true> : k_step1c<false>;
    } else if (!a.groups) {
      return hipErrorInvalidValue;
    } else if (a.chunk_stride) {
      if (a.fast_div) k = sw ? k_step<true, true, false, true, true, true> : k_step<true, false, false, true, true, true>;
      else k = sw ? k_step<false, true, false, true, true, true> : k_step<false, false, false, true, true, true>;
    } else {
      if (a.fast_div) k = sw ? k_step<true, true, false, false, true, true> : k_step<true, false, false, false, true, true>;
      else k = sw ? k_step<false, true, false, false, true, true> : k_step<false, false, false, false, true, true>;
    }
  } else if (a.quarter) {  // latency-bound sizes: as many resident waves as the registers allow
    if (a.groups && a.chunk_stride) k = sw ? k_step1<true, true, true> : k_step1<false, true, true>;
    else if (a.groups) k = sw ? k_step1<true, true> : k_step1<false, true>;
    else k = sw ? k_step1<true> : k_step1<false>;
  } else if (a.groups) {
    if (a.chunk_stride) {
      if (a.fast_div) k = sw ? k_step<true, true, false, true, true> : k_step<true, false, false, true, true>;
      else k = sw ? k_step<false, true, false, true, true> : k_step<false, false, false, true, true>;
    } else {
      if (a.fast_div) k = sw ? k_step<true, true, false, false, true> : k_step<true, false, false, false, true>;
      else k = sw ? k_step<false, true, false, false, true> : k_step<false, false, false, false, true>;
    }
  } else if (a.nee_rec_base) {  // NEE records (no lane masks, no loop: lbm_ctx's build_range)
    if (a.chunk_stride || a.lane_masks) return hipErrorInvalidValue;
    if (a.fast_div) k = sw ? k_step<true, true, false, false, false, false, false, true>
                           : k_step<true, false, false, false, false, false, false, true>;
    else k = sw ? k_step<false, true, false, false, false, false, false, true>
                : k_step<false, false, false, false, false, false, false, true>;
  } else if (a.fast_div) {
    if (a.chunk_stride) k = sw ? k_step<true, true, true, true> : k_step<true, false, true, true>;
    else if (a.lane_masks) k = sw ? k_step<true, true, true> : k_step<true, false, true>;
    else k = sw ? k_step<true, true, false> : k_step<true, false, false>;
  } else {
    if (a.chunk_stride) k = sw ? k_step<false, true, true, true> : k_step<false, false, true, true>;
    else if (a.lane_masks) k = sw ? k_step<false, true, true> : k_step<false, false, true>;
    else k = sw ? k_step<false, true, false> : k_step<false, false, false>;
  }
  const bool c1 = !(a.box && !a.swap && !a.groups && !a.chunk_stride) && a.rowrec && a.quarter;
  hipLaunchKernelGGL(k, grid, dim3(c1 ? kBlock1c : kBlock), lds, s, a);
  return hipGetLastError();
}

hipError_t launch_nee_fix(const MainArgs& a, hipStream_t s) {
  if (!a.nee_mac || a.n_nee <= 0) return hipSuccess;
  const dim3 grid((a.n_nee + 63) / 64);
  typedef void (*Kern)(const MainArgs);
  Kern k;
  if (a.rowrec) k = a.swap ? k_nee_fix<true, true> : k_nee_fix<false, true>;
  else k = a.swap ? k_nee_fix<true, false> : k_nee_fix<false, false>;
  hipLaunchKernelGGL(k, grid, dim3(64), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_reduce(const double* partial, int n, double* scratch, ConvState* conv, float* hist_slot, int finish,
                         hipStream_t s, double* local_out) {
  if (!local_out) local_out = &conv->s_local;
  if (n <= kReduceOneMax) {
    hipLaunchKernelGGL(k_reduce_one, dim3(1), dim3(512), 0, s, partial, n, conv, local_out, hist_slot, finish);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_reduce_slices, dim3(kReduceBlocks), dim3(256), 0, s, partial, n, scratch, conv);
  hipLaunchKernelGGL(k_reduce_final, dim3(1), dim3(256), 0, s, scratch, kReduceBlocks, conv, local_out, hist_slot,
                     finish);
  return hipGetLastError();
}

// XCD: workgroups are dealt round-robin to the 8 XCDs; block b takes the (b % 8)-th eighth
// of the array, so each XCD streams one contiguous region (as k_step's chunk order does)
template <int U, bool XCD, bool NT>
__global__ __launch_bounds__(256) void k_probe_copy(const f4* __restrict__ a, f4* __restrict__ b, int64_t n4) {
  int64_t lo = 0, hi = n4, first = blockIdx.x, nblk = gridDim.x;
  if constexpr (XCD) {
    const int64_t part = (n4 + 7) / 8;
    lo = (blockIdx.x & 7) * part;
    hi = lo + part < n4 ? lo + part : n4;
    first = blockIdx.x >> 3;
    nblk = gridDim.x >> 3;
  }
  const int64_t stride = nblk * blockDim.x;
  for (int64_t i = lo + first * blockDim.x + threadIdx.x; i < hi; i += U * stride) {
    f4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k)
      if (i + k * stride < hi) v[k] = NT ? __builtin_nontemporal_load(a + i + k * stride) : a[i + k * stride];
#pragma unroll
    for (int k = 0; k < U; ++k)
      if (i + k * stride < hi) {
        if constexpr (NT) __builtin_nontemporal_store(v[k], b + i + k * stride);
        else b[i + k * stride] = v[k];
      }
  }
}

// k_step's own access shape: one wave per 16-KB tile, its 16 loads per lane (256 B) all in
// flight before the first store, tiles dealt to the XCDs in contiguous runs (k_step's chunk order)
template <bool NT>
__global__ __launch_bounds__(256) void k_probe_tiles(const f4* __restrict__ a, f4* __restrict__ b, int64_t ntiles) {
  const int64_t nb = gridDim.x;  // a multiple of 8
  const int64_t lb = (int64_t)(blockIdx.x & 7) * (nb >> 3) + (blockIdx.x >> 3);
  const int64_t tile = lb * 4 + (threadIdx.x >> 6);
  if (tile >= ntiles) return;
  const int64_t base = tile * 1024 + (threadIdx.x & 63);
  f4 v[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = NT ? __builtin_nontemporal_load(a + base + k * 64) : a[base + k * 64];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if constexpr (NT) __builtin_nontemporal_store(v[k], b + base + k * 64);
    else b[base + k * 64] = v[k];
  }
}

// The same tiles moved by LDS-DMA (global_load_lds, 16 B per lane: the loads take no VGPRs, so
// a wave keeps its whole 16-KB tile in flight in LDS; two 64-KB workgroups per CU), then
// ds_read_b128 + stores; NT: the loads' non-temporal policy (MI355X_MICROARCH.md, ldsdma-fill)
template <bool NT>
__global__ __launch_bounds__(256) void k_probe_lds(const f4* __restrict__ a, f4* __restrict__ b, int64_t ntiles) {
  __shared__ f4 tile[4][1024];
  const int64_t nb = gridDim.x;  // a multiple of 8
  const int64_t lb = (int64_t)(blockIdx.x & 7) * (nb >> 3) + (blockIdx.x >> 3);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t t = lb * 4 + w;
  if (t >= ntiles) return;
  const f4* src = a + t * 1024;
#pragma unroll
  for (int k = 0; k < 16; ++k)
    __builtin_amdgcn_global_load_lds((gbl_ptr_t)(src + k * 64 + lane), (lds_ptr_t)&tile[w][k * 64], 16, 0,
                                     NT ? 2 : 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's own tile: no barrier needed
#pragma unroll
  for (int k = 0; k < 16; ++k) __builtin_nontemporal_store(tile[w][k * 64 + lane], b + t * 1024 + k * 64 + lane);
}

hipError_t launch_probe_copy(const void* src, void* dst, int64_t n4, int blocks, int shape, hipStream_t s) {
  const f4* a = static_cast<const f4*>(src);
  f4* b = static_cast<f4*>(dst);
  blocks = blocks / 8 * 8;
  if (shape >= 6) {  // tiles: n4 is a whole number of 64-KiB blocks, i.e. of 4-tile workgroups
    const int64_t ntiles = n4 / 1024;
    const unsigned grid = (unsigned)((ntiles / 4 + 7) / 8 * 8);
    if (shape == 6) hipLaunchKernelGGL((k_probe_tiles<true>), dim3(grid), dim3(256), 0, s, a, b, ntiles);
    else if (shape == 7) hipLaunchKernelGGL((k_probe_tiles<false>), dim3(grid), dim3(256), 0, s, a, b, ntiles);
    else if (shape == 8) hipLaunchKernelGGL((k_probe_lds<true>), dim3(grid), dim3(256), 0, s, a, b, ntiles);
    else hipLaunchKernelGGL((k_probe_lds<false>), dim3(grid), dim3(256), 0, s, a, b, ntiles);
    return hipGetLastError();
  }
  switch (shape) {
    case 0: hipLaunchKernelGGL((k_probe_copy<1, false, true>), dim3(blocks), dim3(256), 0, s, a, b, n4); break;
    case 1: hipLaunchKernelGGL((k_probe_copy<1, false, false>), dim3(blocks), dim3(256), 0, s, a, b, n4); break;
    case 2: hipLaunchKernelGGL((k_probe_copy<1, true, true>), dim3(blocks), dim3(256), 0, s, a, b, n4); break;
    case 3: hipLaunchKernelGGL((k_probe_copy<1, true, false>), dim3(blocks), dim3(256), 0, s, a, b, n4); break;
    case 4: hipLaunchKernelGGL((k_probe_copy<2, true, true>), dim3(blocks), dim3(256), 0, s, a, b, n4); break;
    default: hipLaunchKernelGGL((k_probe_copy<4, true, true>), dim3(blocks), dim3(256), 0, s, a, b, n4); break;
  }
  return hipGetLastError();
}

// one full sweep of non-temporal 16-B stores, one contiguous region per XCD (buffer_placement)
__global__ __launch_bounds__(256) void k_probe_fill(f4* __restrict__ b, int64_t n4) {
  const int64_t part = (n4 + 7) / 8;
  const int64_t lo = (blockIdx.x & 7) * part, hi = lo + part < n4 ? lo + part : n4;
  const int64_t stride = (int64_t)(gridDim.x >> 3) * 1024;
  const f4 z{0.f, 0.f, 0.f, 0.f};
  for (int64_t i = lo + (int64_t)(blockIdx.x >> 3) * 1024 + threadIdx.x; i < hi; i += stride) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (i + k * 256 < hi) __builtin_nontemporal_store(z, b + i + k * 256);
  }
}

hipError_t launch_probe_fill(void* dst, int64_t n4, hipStream_t s) {
  hipLaunchKernelGGL(k_probe_fill, dim3(8192), dim3(256), 0, s, static_cast<f4*>(dst), n4);
  return hipGetLastError();
}

__global__ void k_bc_uniform(const uint8_t* __restrict__ type, const float* __restrict__ rho,
                             const float* __restrict__ ux, const float* __restrict__ uy,
                             const float* __restrict__ uz, int64_t n, int64_t ref, unsigned* differs) {
  const uint32_t r0 = __float_as_uint(rho[ref]), r1 = __float_as_uint(ux[ref]), r2 = __float_as_uint(uy[ref]),
                 r3 = __float_as_uint(uz[ref]);
  bool d = false;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if ((type[i] & kClassMask) == kNee)
      d |= __float_as_uint(rho[i]) != r0 || __float_as_uint(ux[i]) != r1 || __float_as_uint(uy[i]) != r2 ||
           __float_as_uint(uz[i]) != r3;
  if (d) atomicOr(differs, 1u);
}

template <bool SW>
__global__ void k_nee_gather(const int* __restrict__ cells, const uint32_t* __restrict__ nl,
                             const float* __restrict__ rho, const float* __restrict__ ux,
                             const float* __restrict__ uy, const float* __restrict__ uz, float4* __restrict__ out,
                             int n, int pitch, int64_t plane) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t c = cells[i];
  uint32_t rest = nl[i];
  for (int j = 0; j < kNeeSlots; ++j) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (rest) {
      const int q = __builtin_ctz(rest);
      rest &= rest - 1u;
      const int64_t b = c - cell_off_rt<SW>(q, pitch, plane);
      v = make_float4(rho[b], ux[b], uy[b], uz[b]);
    }
    out[(int64_t)i * kNeeSlots + j] = v;
  }
}

// NEE records (MainArgs::nee_rec): head {position in the chunk, NEE-link mask, cell, 0}, then the
// boundary data of the first kNeeRecDirs NEE directions (k_nee_gather's order)
template <bool SW>
__global__ void k_nee_records(const int* __restrict__ cells, const int* __restrict__ pos,
                              const uint32_t* __restrict__ nl, const float* __restrict__ rho,
                              const float* __restrict__ ux, const float* __restrict__ uy,
                              const float* __restrict__ uz, float4* __restrict__ rec, int n, int pitch,
                              int64_t plane) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t c = cells[i];
  uint32_t rest = nl[i];
  float4* r = rec + (int64_t)i * kNeeRecF4;
  r[0] = make_float4(__int_as_float(pos[i]), __int_as_float((int)rest), __int_as_float((int)c), 0.f);
  for (int j = 0; j < kNeeRecDirs; ++j) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (rest) {
      const int q = __builtin_ctz(rest);
      rest &= rest - 1u;
      const int64_t b = c - cell_off_rt<SW>(q, pitch, plane);
      v = make_float4(rho[b], ux[b], uy[b], uz[b]);
    }
    r[1 + j] = v;
  }
}
// the records' NEE values into their NEE cells' slots of f (the producer-side state: slot q of
// B = c - e_q), or back
template <bool SW>
__global__ void k_nee_materialize(float* __restrict__ f, const float4* __restrict__ rec, float* __restrict__ vals,
                                  int n, int pitch, int64_t plane, int to_buffer) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 h = rec[(int64_t)i * kNeeRecF4];
  uint32_t rest = (uint32_t)__float_as_int(h.y);
  const int64_t c = __float_as_int(h.z);
  for (int k = 0; rest; ++k) {
    const int q = __builtin_ctz(rest);
    rest &= rest - 1u;
    const int64_t at = aidx(c - cell_off_rt<SW>(q, pitch, plane), q);
    if (to_buffer) f[at] = vals[(int64_t)i * 8 + k];
    else vals[(int64_t)i * 8 + k] = f[at];
  }
}

hipError_t launch_nee_records(const int* cells, const int* pos, const uint32_t* nl, const float* rho, const float* ux,
                              const float* uy, const float* uz, float4* rec, int n, int pitch, int64_t plane, int swap,
                              hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const dim3 g((n + 255) / 256);
  if (swap) hipLaunchKernelGGL(k_nee_records<true>, g, dim3(256), 0, s, cells, pos, nl, rho, ux, uy, uz, rec, n, pitch, plane);
  else hipLaunchKernelGGL(k_nee_records<false>, g, dim3(256), 0, s, cells, pos, nl, rho, ux, uy, uz, rec, n, pitch, plane);
  return hipGetLastError();
}

hipError_t launch_nee_materialize(float* f, const float4* rec, float* vals, int n, int pitch, int64_t plane, int swap,
                                  int to_buffer, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const dim3 g((n + 255) / 256);
  if (swap) hipLaunchKernelGGL(k_nee_materialize<true>, g, dim3(256), 0, s, f, rec, vals, n, pitch, plane, to_buffer);
  else hipLaunchKernelGGL(k_nee_materialize<false>, g, dim3(256), 0, s, f, rec, vals, n, pitch, plane, to_buffer);
  return hipGetLastError();
}

hipError_t launch_bc_uniform(const uint8_t* type, const float* rho, const float* ux, const float* uy,
                             const float* uz, int64_t ncell, int64_t ref, unsigned* differs, hipStream_t s) {
  const int64_t blocks = std::min<int64_t>(4096, (ncell + 255) / 256);
  hipLaunchKernelGGL(k_bc_uniform, dim3((unsigned)std::max<int64_t>(1, blocks)), dim3(256), 0, s, type, rho, ux, uy,
                     uz, ncell, ref, differs);
  return hipGetLastError();
}

hipError_t launch_nee_gather(const int* cells, const uint32_t* nl, const float* rho, const float* ux,
                             const float* uy, const float* uz, float4* nee_bc, int n, int pitch, int64_t plane,
                             int swap, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const dim3 g((n + 255) / 256);
  if (swap) hipLaunchKernelGGL(k_nee_gather<true>, g, dim3(256), 0, s, cells, nl, rho, ux, uy, uz, nee_bc, n, pitch, plane);
  else hipLaunchKernelGGL(k_nee_gather<false>, g, dim3(256), 0, s, cells, nl, rho, ux, uy, uz, nee_bc, n, pitch, plane);
  return hipGetLastError();
}

hipError_t launch_moments(const float* src, const uint8_t* type, const uint32_t* bb_links, float* rho, float* ux,
                          float* uy, float* uz, int64_t lo, int64_t hi, int pitch, int64_t plane, int swap,
                          hipStream_t s) {
  if (hi <= lo) return hipSuccess;
  const dim3 g(grid_for(hi - lo, 256));
  if (swap)
    hipLaunchKernelGGL(k_moments<true>, g, dim3(256), 0, s, src, type, bb_links, rho, ux, uy, uz, lo, hi, pitch, plane);
  else
    hipLaunchKernelGGL(k_moments<false>, g, dim3(256), 0, s, src, type, bb_links, rho, ux, uy, uz, lo, hi, pitch, plane);
  return hipGetLastError();
}

hipError_t launch_moments_compact(const float* src, const uint8_t* type, const uint32_t* bb_links, const int* cmap,
                                  const int* row_of, const int4* rowrec, float* rho, float* ux, float* uy, float* uz,
                                  int64_t lo, int64_t hi, int swap, hipStream_t s) {
  if (hi <= lo) return hipSuccess;
  const dim3 g(grid_for(hi - lo, 256));
  if (swap)
    hipLaunchKernelGGL(k_moments_compact<true>, g, dim3(256), 0, s, src, type, bb_links, cmap, row_of, rowrec, rho, ux,
                       uy, uz, lo, hi);
  else
    hipLaunchKernelGGL(k_moments_compact<false>, g, dim3(256), 0, s, src, type, bb_links, cmap, row_of, rowrec, rho, ux,
                       uy, uz, lo, hi);
  return hipGetLastError();
}

hipError_t launch_vel_terms(const float* src, const uint8_t* type, const uint32_t* bb_links, const int* ref_idx,
                            float* terms, int64_t lo, int64_t hi, int pitch, int64_t plane, int swap, hipStream_t s) {
  if (hi <= lo) return hipSuccess;
  const dim3 g(grid_for(hi - lo, 256));
  if (swap)
    hipLaunchKernelGGL(k_vel_terms<true>, g, dim3(256), 0, s, src, type, bb_links, ref_idx, terms, lo, hi, pitch, plane);
  else
    hipLaunchKernelGGL(k_vel_terms<false>, g, dim3(256), 0, s, src, type, bb_links, ref_idx, terms, lo, hi, pitch,
                       plane);
  return hipGetLastError();
}

hipError_t launch_vel_terms_compact(const float* src, const uint8_t* type, const uint32_t* bb_links, const int* cmap,
                                    const int* row_of, const int4* rowrec, const int* ref_idx, float* terms, int64_t lo,
                                    int64_t hi, int swap, hipStream_t s) {
  if (hi <= lo) return hipSuccess;
  const dim3 g(grid_for(hi - lo, 256));
  if (swap)
    hipLaunchKernelGGL(k_vel_terms_compact<true>, g, dim3(256), 0, s, src, type, bb_links, cmap, row_of, rowrec, ref_idx,
                       terms, lo, hi);
  else
    hipLaunchKernelGGL(k_vel_terms_compact<false>, g, dim3(256), 0, s, src, type, bb_links, cmap, row_of, rowrec,
                       ref_idx, terms, lo, hi);
  return hipGetLastError();
}

int cub_grid(int64_t n, int ipt, int grid_cap) {
  const int64_t tile = 256LL * ipt, tiles = (n + tile - 1) / tile;
  return (int)std::max<int64_t>(1, std::min<int64_t>(tiles, grid_cap));
}

hipError_t launch_cub_tree(const float* terms, int64_t n, int ipt, int vec, int grid_cap, float* partials,
                           ConvState* conv, float* hist_slot, hipStream_t s) {
  const int grid = cub_grid(n, ipt, grid_cap);
  hipLaunchKernelGGL(k_cub_pass1, dim3(grid), dim3(256), 0, s, terms, n, ipt, vec, partials, conv);
  hipLaunchKernelGGL(k_cub_pass2, dim3(1), dim3(256), 0, s, partials, grid, conv, hist_slot);
  return hipGetLastError();
}

hipError_t launch_digest(const uint8_t* type, const float* rho, const float* ux, const float* uy, const float* uz,
                         int nx, int ny, int nz, int pitch, int xshift, int64_t plane, int z_offset, int swap,
                         unsigned long long* out, hipStream_t s) {
  const int per_plane = std::max(1, std::min(256, (int)(plane / 4096)));
  hipLaunchKernelGGL(k_digest, dim3(per_plane, nz), dim3(256), 0, s, type, rho, ux, uy, uz, nx, ny, pitch, xshift,
                     plane, z_offset, swap, out);
  return hipGetLastError();
}

hipError_t launch_pop_compact(float* dst, const float* src, const int* cmap, int64_t n, int to_compact,
                              hipStream_t s) {
  const dim3 g(grid_for(n * kQ, 256));
  if (to_compact) hipLaunchKernelGGL(k_pop_gather, g, dim3(256), 0, s, dst, src, cmap, n);
  else hipLaunchKernelGGL(k_pop_scatter, g, dim3(256), 0, s, dst, src, cmap, n);
  return hipGetLastError();
}
hipError_t launch_poison_walls(float* f, const uint8_t* type, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_poison_walls, dim3(grid_for(n * kQ, 256)), dim3(256), 0, s, f, type, n);
  return hipGetLastError();
}
hipError_t launch_cell_gather(void* dst, const void* src, const int* cmap, int64_t n, int elem_bytes, hipStream_t s) {
  const dim3 g(grid_for(n, 256));
  if (elem_bytes == 1)
    hipLaunchKernelGGL(k_cell_gather<uint8_t>, g, dim3(256), 0, s, static_cast<uint8_t*>(dst),
                       static_cast<const uint8_t*>(src), cmap, n);
  else if (elem_bytes == 4)
    hipLaunchKernelGGL(k_cell_gather<uint32_t>, g, dim3(256), 0, s, static_cast<uint32_t*>(dst),
                       static_cast<const uint32_t*>(src), cmap, n);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_finish_global(ConvState* conv, float* hist_slot, hipStream_t s) {
  hipLaunchKernelGGL(k_finish_global, dim3(1), dim3(1), 0, s, conv, hist_slot);
  return hipGetLastError();
}

hipError_t launch_pack(const float* f, float* buf, int zs, int64_t plane, const int* qs, int nq, hipStream_t s) {
  hipLaunchKernelGGL(k_pack, dim3(grid_for(plane * nq, 256)), dim3(256), 0, s, f, buf, zs, plane, qs, nq);
  return hipGetLastError();
}

hipError_t launch_unpack(float* f, const float* buf, const uint8_t* type, int zs, int64_t plane, const int* qs, int nq,
                         unsigned skip_classes, hipStream_t s) {
  hipLaunchKernelGGL(k_unpack, dim3(grid_for(plane * nq, 256)), dim3(256), 0, s, f, buf, type, zs, plane, qs, nq, skip_classes);
  return hipGetLastError();
}

hipError_t launch_bb_prime(float* f, const uint8_t* type, const uint32_t* links, int64_t ncell, int pitch, int64_t plane,
                           int swap, hipStream_t s) {
  hipLaunchKernelGGL(swap ? k_bb_prime<true> : k_bb_prime<false>, dim3(grid_for(ncell, 256)), dim3(256), 0, s, f, type,
                     links, ncell, pitch, plane);
  return hipGetLastError();
}

hipError_t launch_classify(const GeoArgs& g, hipStream_t s) {
  hipLaunchKernelGGL(k_classify, dim3(grid_for(g.ncell, 256)), dim3(256), 0, s, g);
  return hipGetLastError();
}

hipError_t launch_flag_fluid(const GeoArgs& g, hipStream_t s) {
  hipLaunchKernelGGL(g.swap ? k_flag_fluid<true> : k_flag_fluid<false>, dim3(grid_for(g.ncell, 256)), dim3(256), 0, s,
                     g);
  hipLaunchKernelGGL(g.swap ? k_mark_pulled<true> : k_mark_pulled<false>, dim3(grid_for(g.ncell, 256)), dim3(256), 0,
                     s, g);
  return hipGetLastError();
}

hipError_t launch_ldc_codes(int8_t* codes, int nx, int ny, int pitch, int xshift, int64_t plane, int64_t ncell,
                            int z_offset, int nz_global, int swap, hipStream_t s) {
  hipLaunchKernelGGL(k_ldc_codes, dim3(grid_for(ncell, 256)), dim3(256), 0, s, codes, nx, ny, pitch, xshift, plane,
                     ncell, z_offset, nz_global, swap);
  return hipGetLastError();
}

hipError_t launch_mask_hist(const uint8_t* mask, int nx, int ny, int nz_global, int zbase, int z_lo, int z_hi,
                            unsigned long long* hist, int swap, hipStream_t s) {
  const MaskGeo g{mask, nx, ny, nz_global, zbase};
  hipLaunchKernelGGL(k_mask_hist, dim3(grid_for((int64_t)(z_hi - z_lo) * (swap ? nx : ny), 256)), dim3(256), 0, s, g,
                     z_lo, z_hi, hist, swap);
  return hipGetLastError();
}

hipError_t launch_mask_codes(const uint8_t* mask, int nx, int ny, int nz_global, int zbase, int8_t* codes, int pitch,
                             int xshift, int64_t plane, int64_t ncell, int z_offset, int z_lo, int z_hi, int swap,
                             hipStream_t s) {
  const MaskGeo g{mask, nx, ny, nz_global, zbase};
  hipLaunchKernelGGL(k_mask_codes, dim3(grid_for(ncell, 256)), dim3(256), 0, s, g, codes, pitch, xshift, plane, ncell,
                     z_offset, z_lo, z_hi, swap);
  return hipGetLastError();
}

hipError_t launch_init_feq(float* fa, float* fb, int64_t n, int form, const float* rho, const float* ux,
                           const float* uy, const float* uz, hipStream_t s) {
  hipLaunchKernelGGL(k_init_feq, dim3(grid_for(n, 256)), dim3(256), 0, s, fa, fb, n, form, rho, ux, uy, uz);
  return hipGetLastError();
}

hipError_t launch_init_mask(float* fa, float* fb, const int8_t* codes, const float* in_uy, const float* out_uy, int nx,
                            int ny, int nz, int pitch, int xshift, int64_t plane, int64_t ncell, int z_offset, int swap,
                            hipStream_t s) {
  hipLaunchKernelGGL(k_init_mask, dim3(grid_for(ncell, 256)), dim3(256), 0, s, fa, fb, codes, in_uy, out_uy, nx, ny, nz,
                     pitch, xshift, plane, ncell, z_offset, swap);
  return hipGetLastError();
}

hipError_t launch_init_ldc(float* fa, float* fb, int64_t n, int pitch, int xshift, int nx, int ny, float lid_u, int swap,
                           hipStream_t s) {
  hipLaunchKernelGGL(k_init_ldc, dim3(grid_for(n, 256)), dim3(256), 0, s, fa, fb, n, pitch, xshift, nx, ny, lid_u, swap);
  return hipGetLastError();
}

}  // namespace lbm
