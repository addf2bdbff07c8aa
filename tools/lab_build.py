#!/usr/bin/env python3
"""Build liblbm.so lab variants for interleaved A/B (tools/ab_lattices.py) into tools/ab/<name>/.

    python3 tools/lab_build.py <name> <patch>[,<patch>...]     # LAB_REV=<git rev>: that revision's csrc/

A patch is a named list of literal (file, old, new) edits applied to a copy of csrc/ (the
product sources stay untouched); the copy is built with the product's flags.  Lab variants
are measurement tools: several compute wrong values on purpose (they remove work to price it).
"""
import os
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "lattice-boltzmann-method-gpu_amd")

PATCHES = {
    # WRONG VALUES: 4-cell ranges launch no NEE blocks (the NEE neighbours' slots go unwritten)
    "no_nee_blocks": [("lbm_ctx.hip", "  r.nee_blocks = nee_grid(r.n_nee, r.nee_waves);",
                       "  r.nee_blocks = 0;\n  r.n_nee = 0;")],
    # WRONG VALUES: chunk waves store no bounce-back slots
    "no_bb": [("lbm_kernels.hip", "  if (!consumer && __any(t4 & kWall4)) {  // wave-uniform",
               "  if (false) {  // lab: no bounce-back stores"),
              ("lbm_kernels.hip", "  if (!consumer && (t4 & kWall4)) {  // rare, divergent",
               "  if (false) {  // lab")],
    # a contiguous chunk list read from memory like a sparse one (prices the list load)
    "force_list": [("lbm_ctx.hip", "    if (chunks[i] != chunks[0] + (int)i) r.chunk0 = -1;",
                    "    if (chunks[i] != chunks[0] + (int)i) r.chunk0 = -1;\n  r.chunk0 = -1;")],
    # WRONG VALUES: the NEE values are computed but not stored (prices the scattered 4-B stores)
    "nee_nostore": [("lbm_kernels.hip", "      a.dst[fidx(nb, Q)] = nee_value<Q>(fq, b, r, ux, uy, uz, a.omc, p.template of<Q>());",
                     "      const float val = nee_value<Q>(fq, b, r, ux, uy, uz, a.omc, p.template of<Q>());\n"
                     "      if (val == 1234.5678f) a.dst[fidx(nb, Q)] = val;")],
    # ~140 extra VALU per chunk wave holding an NEE-adjacent cell, after its stores (prices an
    # in-wave NEE tail; combine with no_nee_blocks + LBM_TUNE_NEE_FIX 1)
    "valu_tail": [("lbm_kernels.hip", "  return acc;\n}\n\n// ---- one cell per lane",
                   "  if (__any(t4 & kNee4)) {\n"
                   "    float a2 = v[3][0] + v[7][1], u1 = UX[0], u2 = UY[0], u3 = UZ[0];\n"
                   "#pragma unroll\n"
                   "    for (int it = 0; it < 5; ++it) {\n"
                   "      a2 = feq_pre<7>(a2, u1, u2, u3) + feq_pre<15>(a2 * 0.5f, u3, u1, u2) * a.omc;\n"
                   "      u1 = u1 * 0.99f + a2 * 1e-9f;\n"
                   "    }\n"
                   "    if (a2 == 1234.5678f) a.dst[0] = a2;\n"
                   "  }\n"
                   "  return acc;\n}\n\n// ---- one cell per lane")],
    # wave timestamps (s_memrealtime, 100 MHz): every 4-cell chunk wave of the dense chunk path
    # records its start and end into g_lab_ts (lbm_lab_ts_copy), values unchanged
    "wave_ts": [("lbm_kernels.hip",
                 "      acc = process_chunk<FAST, SW, MASK, false, false, BOX, REC>(a, chunk_of(a, idx) * kChunk, lane, lm, idx);  // uniform base\n    }",
                 "      const unsigned long long t_in = wall_clock64();\n"
                 "      acc = process_chunk<FAST, SW, MASK, false, false, BOX, REC>(a, chunk_of(a, idx) * kChunk, lane, lm, idx);  // uniform base\n"
                 "      if (lane == 0 && idx < (1 << 20)) {\n"
                 "        unsigned xcc;\n"
                 "        asm volatile(\"s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)\" : \"=s\"(xcc));\n"
                 "        g_lab_ts[2 * idx] = t_in | ((unsigned long long)(xcc & 15) << 56);\n"
                 "        g_lab_ts[2 * idx + 1] = wall_clock64() | ((unsigned long long)x << 56);\n"
                 "      }\n    }"),
                ("lbm_kernels.hip", "__device__ void residual_logic(ConvState* cv, double S, float* hist_slot) {",
                 "__device__ unsigned long long g_lab_ts[2 << 20];\n"
                 "__device__ void residual_logic(ConvState* cv, double S, float* hist_slot) {"),
                ("lbm_kernels.hip", "}  // namespace lbm\n",
                 "}  // namespace lbm\n"
                 "extern \"C\" int lbm_lab_ts_copy(unsigned long long* out, int n) {\n"
                 "  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(lbm::g_lab_ts), sizeof(unsigned long long) * n);\n}\n")],
    # the NEE-record ranges always on the exact-division instance (no FAST body: fewer registers)
    "rec_exact": [("lbm_kernels.hip", "    if (a.fast_div) k = sw ? k_step<true, true, false, false, false, false, false, true>\n"
                                      "                           : k_step<true, false, false, false, false, false, false, true>;\n"
                                      "    else k = sw",
                   "    k = sw")],
    # WRONG VALUES (pricing the NEE-record code): without the substitution into the pulls
    "rec_nosub": [("lbm_kernels.hip", "          nee_rec_sub_all(v, lane, pos >> 2, pos & 3, nl, vals + k * 8, AllQ{});",
                   "          (void)pos; (void)nl; (void)vals;")],
    # ... without the production of the values (after the relaxation)
    "rec_noprod": [("lbm_kernels.hip", "      nee_rec_make_all(v, lane, L, j, nl, NL + k * kNeeRecF4 + 1, r, ux, uy, uz, Pref::exact(r), a.omc, mine, AllQ{});",
                    "      mine = r + ux + uy + uz + (float)(L + j + (int)nl);")],
    # ... without the explicit wait for the records' DMA
    "rec_nowait": [("lbm_kernels.hip", "    if (REC && rn > 0) {\n      asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");  // the DMA's LDS writes are in",
                    "    if (REC && rn > 0) {")],
    # compact one-cell waves: lanes that are not fluid issue no pulls (exec-masked), values unchanged
    "c1_mask": [("lbm_kernels.hip", "  pull1_bb<SW>(f, a.src, R, compact_id(c), wl, AllQ{});\n  BcSlots bc{};",
                 "  if (fluid) pull1_bb<SW>(f, a.src, R, compact_id(c), wl, AllQ{});\n  BcSlots bc{};")],
    # the one-cell compact pulls as plain (temporal) loads instead of non-temporal ones
    "c1_temporal": [("lbm_kernels.hip", "  ((f[Qs] = __builtin_nontemporal_load(\n        src + ((wl >> Qs) & 1u ? fidx(c, Dir<Qs>::opp)",
                     "  ((f[Qs] = *(\n        src + ((wl >> Qs) & 1u ? fidx(c, Dir<Qs>::opp)")],
    # the dense one-cell pulls (k_step1, NEE blocks) as plain loads
    "t1_dense": [("lbm_kernels.hip", "  ((f[Qs] = __builtin_nontemporal_load(src + fidx(ad.template nb<Qs, SW>(), Qs))), ...);",
                  "  ((f[Qs] = *(src + fidx(ad.template nb<Qs, SW>(), Qs))), ...);"),
                 ("lbm_kernels.hip", "  ((f[Qs] = __builtin_nontemporal_load(src + aidx(c - cell_off<Qs, SW>(pitch, plane), Qs))), ...);",
                  "  ((f[Qs] = *(src + aidx(c - cell_off<Qs, SW>(pitch, plane), Qs))), ...);"),
                 ("lbm_kernels.hip", "  ((f[Qs] = __builtin_nontemporal_load(base + rel_aidx(r0 - (int)cell_off<Qs, SW>(pitch, plane), Qs))), ...);",
                  "  ((f[Qs] = *(base + rel_aidx(r0 - (int)cell_off<Qs, SW>(pitch, plane), Qs))), ...);"),
                 ("lbm_kernels.hip", "  ((f[Qs] = __builtin_nontemporal_load(\n        base + ((wl >> Qs)",
                  "  ((f[Qs] = *(\n        base + ((wl >> Qs)")],
    # the compact 4-cell groups' slice loads as plain loads
    "t4g_loads": [("lbm_kernels.hip", "  const float* p = need ? src + fidx(s, Q) : src;\n  a = __builtin_nontemporal_load(reinterpret_cast<const f4*>(p));",
                   "  const float* p = need ? src + fidx(s, Q) : src;\n  a = *reinterpret_cast<const f4*>(p);")],
    # the 4-cell group lists' whole 16-B stores as plain stores (chunk lists keep non-temporal ones)
    "t4g_stores": [("lbm_kernels.hip", "    for (int q = 0; q < kQ; ++q) __builtin_nontemporal_store(v[q], reinterpret_cast<f4*>(d + q * kChunk));",
                    "    for (int q = 0; q < kQ; ++q) {\n      if constexpr (GROUPS) *reinterpret_cast<f4*>(d + q * kChunk) = v[q];\n"
                    "      else __builtin_nontemporal_store(v[q], reinterpret_cast<f4*>(d + q * kChunk));\n    }")],
    # the one-cell paths' stores non-temporal
    "t1_ntstores": [("lbm_kernels.hip", "  ((dst[aidx(c, Qs)] = f[Qs]), ...);\n  if (m) {",
                     "  (__builtin_nontemporal_store(f[Qs], dst + aidx(c, Qs)), ...);\n  if (m) {")],
    # k_nee_fix in one-wave workgroups (spread over all CUs)
    "fix64": [("lbm_kernels.hip", "  const int i = blockIdx.x * kBlock + (int)threadIdx.x;",
               "  const int i = blockIdx.x * 64 + (int)threadIdx.x;"),
              ("lbm_kernels.hip", "  const dim3 grid((a.n_nee + kBlock - 1) / kBlock);\n  typedef void (*Kern)(const MainArgs);\n  Kern k;\n  if (a.rowrec) k = a.swap ? k_nee_fix",
               "  const dim3 grid((a.n_nee + 63) / 64);\n  typedef void (*Kern)(const MainArgs);\n  Kern k;\n  if (a.rowrec) k = a.swap ? k_nee_fix"),
              ("lbm_kernels.hip", "  hipLaunchKernelGGL(k, grid, dim3(kBlock), 0, s, a);\n  return hipGetLastError();\n}\n\nhipError_t launch_reduce(",
               "  hipLaunchKernelGGL(k, grid, dim3(64), 0, s, a);\n  return hipGetLastError();\n}\n\nhipError_t launch_reduce(")],
    # the compact one-cell kernel in four-wave / one-wave workgroups
    # k_step1c (compact rows, one cell per lane) capped for five / six waves per SIMD
    "c1_w5": [("lbm_kernels.hip", "__global__ __launch_bounds__(kBlock1c) __attribute__((amdgpu_waves_per_eu(4))) void k_step1c(",
               "__global__ __launch_bounds__(kBlock1c) __attribute__((amdgpu_waves_per_eu(5))) void k_step1c(")],
    "c1_w6": [("lbm_kernels.hip", "__global__ __launch_bounds__(kBlock1c) __attribute__((amdgpu_waves_per_eu(4))) void k_step1c(",
               "__global__ __launch_bounds__(kBlock1c) __attribute__((amdgpu_waves_per_eu(6))) void k_step1c(")],
    # the population buffers' and per-cell arrays' device addresses (lbm_lab_ptrs; tools/c3_modes_lab.py)
    "ptrs": [("lbm_ctx.hip", "int lbm_buffer_placement(lbm_ctx* c, double* gbs, int cap, int* n, int* chosen) {",
              "extern \"C\" int lbm_lab_ptrs(lbm_ctx* c, unsigned long long* out) {\n"
              "  out[0] = (unsigned long long)c->alloc[0];\n  out[1] = (unsigned long long)c->alloc[1];\n"
              "  out[2] = (unsigned long long)c->type;\n  out[3] = (unsigned long long)c->whole.chunks;\n"
              "  out[4] = (unsigned long long)c->whole.cells;\n  out[5] = (unsigned long long)c->cur;\n  return 0;\n}\n"
              "int lbm_buffer_placement(lbm_ctx* c, double* gbs, int cap, int* n, int* chosen) {")],
    # the kept pair of population buffers at least four buffer sizes apart in the address space
    # when the top writers allow it (C3's slow mode came with neighbouring buffers, r06zi)
    "pair_far": [("lbm_ctx.hip", "    float best = 0.f;\n    for (int i = 0; i < K; ++i)",
                  "    float best = 0.f;\n"
                  "    auto pen = [&](int i, int j) {\n"
                  "      const int64_t d = (int64_t)((const char*)p[order[i]] - (const char*)p[order[j]]);\n"
                  "      return (d < 0 ? -d : d) >= 4 * (int64_t)bytes ? 0.f : 1e6f;\n    };\n"
                  "    for (int i = 0; i < K; ++i)"),
                 ("lbm_ctx.hip", "        if (best == 0.f || t[i][j] + t[j][i] < best) {\n          best = t[i][j] + t[j][i];",
                  "        if (best == 0.f || t[i][j] + t[j][i] + pen(i, j) < best) {\n          best = t[i][j] + t[j][i] + pen(i, j);")],
    # the pipe's pull-phase priority (product: 2, lbm_kernels.hip kPrio) at 3 / 1, or also raised
    # for the store phase
    "prio3": [("lbm_kernels.hip", "  if constexpr (kPrio) __builtin_amdgcn_s_setprio(2);",
               "  if constexpr (kPrio) __builtin_amdgcn_s_setprio(3);")],
    "prio1": [("lbm_kernels.hip", "  if constexpr (kPrio) __builtin_amdgcn_s_setprio(2);",
               "  if constexpr (kPrio) __builtin_amdgcn_s_setprio(1);")],
    "prio_st": [("lbm_kernels.hip", "  float* d = a.dst + aidx(c, 0);\n  if (whole) {",
                 "  if constexpr (kPrio) __builtin_amdgcn_s_setprio(2);\n  float* d = a.dst + aidx(c, 0);\n  if (whole) {")],
    # one-cell waves: pulls and stores at raised priority, the arithmetic at 0 (compact rows only
    # raise it at the start; collide_cell1's flips are no-ops elsewhere until the stores)
    "c1_prio": [("lbm_kernels.hip", "  const int64_t c = (a.c_lo & ~int64_t(63)) + w * 64 + lane;\n",
                 "  const int64_t c = (a.c_lo & ~int64_t(63)) + w * 64 + lane;\n  __builtin_amdgcn_s_setprio(2);\n"),
                ("lbm_kernels.hip", "  float rho = 0.f;\n#pragma unroll\n  for (int q = 0; q < kQ; ++q) rho = rho + f[q];\n  const float ux = (f[1] - f[2] + f[7] + f[8] - f[9] - f[10] + f[11] + f[12] - f[13] - f[14]) / rho;\n  const float uy = (f[3] - f[4] + f[7] - f[8] + f[9] - f[10] + f[15] - f[16] + f[17] - f[18]) / rho;\n  const float uz = (f[5] - f[6] + f[11] - f[12] + f[13] - f[14] + f[15] + f[16] - f[17] - f[18]) / rho;\n  if (__any(nee) && a.tau_fast",
                 "  __builtin_amdgcn_s_setprio(0);\n  float rho = 0.f;\n#pragma unroll\n  for (int q = 0; q < kQ; ++q) rho = rho + f[q];\n  const float ux = (f[1] - f[2] + f[7] + f[8] - f[9] - f[10] + f[11] + f[12] - f[13] - f[14]) / rho;\n  const float uy = (f[3] - f[4] + f[7] - f[8] + f[9] - f[10] + f[15] - f[16] + f[17] - f[18]) / rho;\n  const float uz = (f[5] - f[6] + f[11] - f[12] + f[13] - f[14] + f[15] + f[16] - f[17] - f[18]) / rho;\n  if (__any(nee) && a.tau_fast"),
                ("lbm_kernels.hip", "  fix_store_all<SW>(f, a.dst, c, ad, (t & kWallAdj) ? links : 0u, AllQ{});\n  return (double)sqrtf(ux * ux + uy * uy + uz * uz);\n}",
                 "  __builtin_amdgcn_s_setprio(2);\n  fix_store_all<SW>(f, a.dst, c, ad, (t & kWallAdj) ? links : 0u, AllQ{});\n  return (double)sqrtf(ux * ux + uy * uy + uz * uz);\n}")],
    # the 4-cell group lists (C4 x4's y rows) with the pipe's priority flips
    "g_prio": [("lbm_kernels.hip", "  constexpr bool kPrio = SW && !GROUPS;", "  constexpr bool kPrio = SW;")],
    # the cavity's x-row chunk waves: stores at raised priority / pulls and stores
    "box_prio_st": [("lbm_kernels.hip", "  if constexpr (kPrio) __builtin_amdgcn_s_setprio(2);  // the stores, too",
                     "  if constexpr (kPrio || BOX) __builtin_amdgcn_s_setprio(2);  // the stores, too")],
    "box_prio_all": [("lbm_kernels.hip", "  constexpr bool kPrio = SW;", "  constexpr bool kPrio = SW || BOX;")],
    # NEE blocks' threads at raised priority for their whole (latency-bound, scattered) work
    "nee_prio": [("lbm_kernels.hip", "__device__ __forceinline__ double nee_cell(const MainArgs& a, int i) {\n",
                  "__device__ __forceinline__ double nee_cell(const MainArgs& a, int i) {\n  __builtin_amdgcn_s_setprio(3);\n")],
    # the pull-phase priority for the cavity's x-row chunk waves too
    "prio_all": [("lbm_kernels.hip", "  constexpr bool kPrio = SW && !GROUPS;", "  constexpr bool kPrio = !GROUPS;")],
    "c1_wg256": [("lbm_kernels.hpp", "constexpr int kBlock1c = 128;", "constexpr int kBlock1c = 256;")],
    "c1_wg64": [("lbm_kernels.hpp", "constexpr int kBlock1c = 128;", "constexpr int kBlock1c = 64;")],
    # placement over up to 160 GiB of candidates (15 at 512^3 instead of 6)
    "budget160": [("lbm_ctx.hip", "constexpr size_t kPlacementBudget = (size_t)64 << 30;",
                   "constexpr size_t kPlacementBudget = (size_t)160 << 30;")],
    # WRONG VALUES (pricing k_nee_fix): every thread returns at once (launch and ramp only)
    "fix_empty": [("lbm_kernels.hip", "  if (i >= a.n_nee) return;\n  const int64_t c = a.cells[i];",
                   "  if (i >= 0) return;\n  const int64_t c = a.cells[i];")],
    # ... without the own-slot loads (the second round trip)
    "fix_noload": [("lbm_kernels.hip", "  ((f[Qs] = ((nl >> Qs) & 1u) ? dst[fidx(c, Qs)] : 0.0f), ...);",
                    "  ((f[Qs] = ((nl >> Qs) & 1u) ? 0.5f : 0.0f), ...);")],
    # every 4-cell whole store plain
    "t4_stores": [("lbm_kernels.hip", "    for (int q = 0; q < kQ; ++q) __builtin_nontemporal_store(v[q], reinterpret_cast<f4*>(d + q * kChunk));",
                   "    for (int q = 0; q < kQ; ++q) *reinterpret_cast<f4*>(d + q * kChunk) = v[q];")],
}


def main():
    name, specs = sys.argv[1], [x for x in sys.argv[2].split(",") if x]
    tmp = tempfile.mkdtemp(prefix="lab_")
    try:
        src = os.path.join(tmp, "pkg", "csrc")  # csrc/../../include/lbm.h as in the tree
        rev = os.environ.get("LAB_REV")  # the sources of a git revision instead of the tree's
        if rev:
            os.makedirs(src)
            arc = subprocess.check_output(["git", "-C", REPO, "archive", rev, "lattice-boltzmann-method-gpu_amd/csrc"])
            subprocess.run(["tar", "-x", "--strip-components=2", "-C", src], input=arc, check=True)
        else:
            shutil.copytree(os.path.join(PKG, "csrc"), src)
        os.symlink(os.path.join(REPO, "include"), os.path.join(tmp, "include"))
        for spec in specs:
            for fname, old, new in PATCHES[spec]:
                p = os.path.join(src, fname)
                text = open(p).read()
                if text.count(old) != 1:
                    raise SystemExit(f"patch {spec}: {fname}: pattern found {text.count(old)} times")
                open(p, "w").write(text.replace(old, new))
        out = os.path.join(REPO, "tools", "ab", name)
        os.makedirs(out, exist_ok=True)
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off",
               "-fhip-fp32-correctly-rounded-divide-sqrt", "-I", os.path.join(REPO, "include"), "-shared", "-o",
               os.path.join(out, "liblbm.so"), os.path.join(src, "lbm_kernels.hip"), os.path.join(src, "lbm_ctx.hip"),
               "-L/opt/rocm/lib", "-lrccl", "-lrocprofiler-sdk-roctx"]
        subprocess.check_call(cmd)
        print(f"built tools/ab/{name}/liblbm.so ({','.join(specs)})")
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
