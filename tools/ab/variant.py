"""Dev A/B (NOT product code): build a patched copy of the working-tree csrc into
tools/ab/libals_<tag>.so (same ABI, loaded with ALS_HIP_DEV=1 ALS_HIP_LIB=...).
Each variant is a list of (file, old, new) text replacements applied to the copy;
an `old` that does not occur fails the build (the patch must still apply).
    python tools/ab/variant.py TAG [TAG ...]      (TAG from VARIANTS below; "base" = none)
"""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "..", "recommender-system-using-apache-spark-mllib-_amd", "csrc")
GS = "gram_solve.hip"
TK = "topk.hip"

NEG = [
        (GS, """// v on the lanes of 64-bit mask M (a constant), else w.""",
         """// v on lanes with (lane & 15) == P, else -w.
template <int P>
__device__ __forceinline__ float sel_lane16_n(float v, float w) {
  float r;
  const uint64_t msk = 0x0001000100010001ull << P;
  asm volatile("v_cndmask_b32_e64 %0, -%2, %1, %3" : "=v"(r) : "v"(v), "v"(w), "s"(msk));
  return r;
}

// v on the lanes of 64-bit mask M (a constant), else w."""),
        (GS, "  float nf = sel_lane16<0>(0.f, -f);\n  static_for<16>([&](auto pc) {\n    constexpr int p = decltype(pc)::value;\n    constexpr int qp",
         "  float nf = sel_lane16_n<0>(0.f, f);\n  static_for<16>([&](auto pc) {\n    constexpr int p = decltype(pc)::value;\n    constexpr int qp"),
        (GS, "      nfn = sel_lane16<p + 1>(0.f, -fn);\n    }\n    static_for<4>",
         "      nfn = sel_lane16_n<p + 1>(0.f, fn);\n    }\n    static_for<4>"),
        (GS, "    constexpr int qp = p >> 2, rp = p & 3, rn = (p + 1) & 3;\n    dmin = fminf(dmin, d);",
         "    constexpr int qp = p >> 2, rp = p & 3, rn = (p + 1) & 3;"),
        (GS, "  return dmin > 0.f && rmax <= kCondMax * rmin && __ballot(!fin) == 0;",
         "  return dmin > 0.f && rmin > 0.f && rmax <= kCondMax * rmin && __ballot(!fin) == 0;"),
    ]

VARIANTS = {
    "base": [],
    # round 6: quad top-k lists (16 < top <= 128) with one row group only
    # round 6: the committed (HEAD) topk.hip in place of the working tree's ("@HEAD" files)
    "oldtopk": [(TK, "@HEAD", None)],
    # a candidate topk.hip kept outside the tree (/tmp/topk_cand.hip)
    "tkcand": [(TK, "@FILE", "/tmp/topk_cand.hip")],
    "tkprev": [(TK, "@FILE", "/tmp/topk_prev.hip")],
    # top-k register lists: six blocks per ballot (logs keep four: their registers)
    "tk_nb6": [(TK, "constexpr int NB4 = 4;  // blocks per ballot",
                "constexpr int NB4 = (TOPR > 0 && TOPR <= 16) ? 6 : 4;  // blocks per ballot")],
    "gsprev": [(GS, "@FILE", "/tmp/gs_prev.hip")],
    # the n x n dual kernel: step s+1's gathers in flight during step s at NB = 6 too
    "dualnb2": [(GS, "constexpr int NBUF = NB <= 4 ? 2 : 1;", "constexpr int NBUF = 2;")],
    # round 6: the LDL^T pivot-spread limit (rows beyond it go to the fp64 rescue)
    **{f"cond{c}": [(GS, "constexpr float kCondMax = 32.f;", f"constexpr float kCondMax = {c}.f;")]
       for c in (2, 4, 8, 16)},
    # the round-4 rescue guards off: no split-window / rank-deficiency tests, no
    # pivot-spread test (timing only: rows that need the rescue are then wrong)
    "noguard": [
        (GS, "__device__ __forceinline__ bool window_miss(float diag_lane, float n_terms, float rmax_lane) {",
         "__device__ __forceinline__ bool window_miss(float diag_lane, float n_terms, float rmax_lane) {\n  return false;"),
        (GS, "  if (4 * n > (int64_t)k) return false;  // uniform: the trace only for very short rows",
         "  return false;"),
        (GS, "  return dmin > 0.f && rmax <= kCondMax * rmin && __ballot(!fin) == 0;",
         "  return dmin > 0.f && __ballot(!fin) == 0;"),
    ],
    # the C-layout sweep's row-group broadcast through the LDS crossbar (one
    # ds_bpermute) instead of two VALU lane swaps and their copies
    "bperm": [
        (GS, """template <int G>
__device__ __forceinline__ float rowgroup_bcast(float x) {
  uint32_t a""", """template <int G>
__device__ __forceinline__ float rowgroup_bcast(float x) {
  if constexpr (true) {
    const int src = (16 * G + (threadIdx.x & 15)) << 2;
    return __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src, __builtin_bit_cast(int, x)));
  }
  uint32_t a"""),
    ],
    # the sweep's multiplier negation folded into its select, no per-pivot min (the
    # pivots' positivity from the spread test's own minimum)
    "neg": NEG,
    "lean": None,  # bperm + neg
    # C-layout sweeps (ds_bpermute broadcast) in every block elimination: NB = 2, 6, 8 too
    # occupancy: four waves per SIMD for the explicit k <= 64 kernel, three for the dual
    "occ4": [
        (GS, "__launch_bounds__(64, IMPLICIT ? 2 : 3) void gram_solve_kernel(",
         "__launch_bounds__(64, IMPLICIT ? 2 : 4) void gram_solve_kernel("),
    ],
    "dual3": [
        (GS, "__launch_bounds__(64, 2) void gram_solve_dual_kernel(",
         "__launch_bounds__(64, 3) void gram_solve_dual_kernel("),
    ],
    # top-k timing bound (wrong scores by the hi.lo term): refinement without the lo
    # fetch (bl = 0), i.e. the cost of the lo loads' latency
    "tk_nolo": [
        (TK, """      __builtin_amdgcn_global_load_lds(Vlo + vr * RW + 4 * s + q, scr + s * 64, 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");""", """      (void)vr;"""),
        (TK, "const tk_half8 bl = __builtin_bit_cast(tk_half8, scr[s * 64 + lane]);",
         "const tk_half8 bl = {};"),
    ],
    # top-k timing bound (no lists: wrong results): the sweep alone, every quartet
    # scored (V stream, LDS, MFMA, barriers) and no block filtered
    "tk_scoreonly": [
        (TK, """            for (int j = 0; j < 4; ++j) score(tbr + 16 * j * RS, a4[j]);
            if (__builtin_amdgcn_readfirstlane(full ? 1 : 0) != 0) {""",
         """            for (int j = 0; j < 4; ++j) score(tbr + 16 * j * RS, a4[j]);
#pragma unroll
            for (int j = 0; j < 4; ++j)
              asm volatile("" :: "v"(a4[j][0][0]), "v"(a4[j][0][1]), "v"(a4[j][0][2]), "v"(a4[j][0][3]));
            if (true) continue;
            if (__builtin_amdgcn_readfirstlane(full ? 1 : 0) != 0) {"""),
    ],
    # top-k event counters (dev): quartets scored / past the coarse ballot, blocks
    # refined, insertion passes, keys inserted (als_dev_tk_counters)
    "tk_count": [
        (TK, "namespace als {\n", "namespace als {\n__device__ unsigned long long tk_dbg[8];\n"),
        (TK, "              if (__ballot(any) == 0) continue;",
         """              if (lane == 0) atomicAdd(&tk_dbg[0], 1ull);
              if (__ballot(any) != 0 && lane == 0) atomicAdd(&tk_dbg[1], 1ull);
              if (__ballot(any) == 0) continue;"""),
        (TK, """        if (__ballot(c) == 0) return;
      }
      refine(tbr, ibase, acc);""", """        if (__ballot(c) == 0) return;
      }
      if (lane == 0) atomicAdd(&tk_dbg[2], 1ull);
      refine(tbr, ibase, acc);"""),
        (TK, "          if (c > gmin && q == (__builtin_ctzll(holders) >> 4)) tk_insert<NR>(kv[g], c);",
         """          const bool do_ins = c > gmin && q == (__builtin_ctzll(holders) >> 4);
          {
            const uint64_t bi = __ballot(do_ins);
            if (lane == 0) {
              atomicAdd(&tk_dbg[3], 1ull);
              atomicAdd(&tk_dbg[4], (unsigned long long)__popcll(bi));
            }
          }
          if (do_ins) tk_insert<NR>(kv[g], c);"""),
        (TK, "}  // extern \"C\"\n", """int als_dev_tk_counters(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(als::tk_dbg), sizeof(unsigned long long) * 8) != hipSuccess)
    return -1;
  if (reset) {
    unsigned long long z[8] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(als::tk_dbg), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}

}  // extern "C"
"""),
    ],
    # top-k logs (round 6) timing bound (no lists: wrong results): the sweep alone, every
    # quartet scored (V stream, LDS, MFMA, barriers), no block filtered
    "tk_sweeponly": [
        (TK, """            if (vb + 16 * (c + NB4) > n_v) {  // (uniform) the last tile""",
         """#pragma unroll
            for (int j = 0; j < NB4; ++j)
#pragma unroll
              for (int g = 0; g < RG; ++g)
                asm volatile("" :: "v"(a4[j][g][0]), "v"(a4[j][g][1]), "v"(a4[j][g][2]), "v"(a4[j][g][3]));
            if (true) continue;
            if (vb + 16 * (c + NB4) > n_v) {  // (uniform) the last tile"""),
    ],
    # top-k logs event counters (dev): quartets scored / past the coarse ballot, blocks
    # refined, keys appended, log cuts (als_dev_tk_counters)
    "tk_count2": [
        (TK, "namespace als {\n", "namespace als {\n__device__ unsigned long long tk_dbg[8];\n"),
        (TK, "              if (__ballot(any) == 0) continue;",
         """              if (lane == 0) atomicAdd(&tk_dbg[0], 1ull);
              if (__ballot(any) != 0 && lane == 0) atomicAdd(&tk_dbg[1], 1ull);
              if (__ballot(any) == 0) continue;"""),
        (TK, """      if (__ballot(c) == 0) return;
      refine(tbr, ibase, acc);
      const unsigned below""", """      if (__ballot(c) == 0) return;
      if (lane == 0) atomicAdd(&tk_dbg[2], 1ull);
      refine(tbr, ibase, acc);
      const unsigned below"""),
        (TK, "          lcnt[g][r] += __popc(grp);",
         """          lcnt[g][r] += __popc(grp);
          if (m == 0 && grp) atomicAdd(&tk_dbg[3], (unsigned long long)__popc(grp));"""),
        (TK, "              if (lane == 0) thr[16 * g + rho] = t;",
         """              if (lane == 0) thr[16 * g + rho] = t;
              if (lane == 0) atomicAdd(&tk_dbg[4], 1ull);"""),
        (TK, "}  // extern \"C\"\n", """int als_dev_tk_counters(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(als::tk_dbg), sizeof(unsigned long long) * 8) != hipSuccess)
    return -1;
  if (reset) {
    unsigned long long z[8] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(als::tk_dbg), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}

}  // extern "C"
"""),
    ],
    # top-k: 192-row tiles at rank > 64 (register / quad lists)
    "tk_vt192": [
        (TK, "return topr == 0 ? 64 / nk : (nk == 4 ? 128 : 256 / nk);",
         "return topr == 0 ? 64 / nk : (nk == 4 ? 192 : 256 / nk);"),
        (TK, "constexpr int tk_nbuf(int topr) { return topr == 0 ? 2 : 3; }",
         "constexpr int tk_nbuf(int topr) { return topr == 0 ? 2 : 2; }"),
    ],
    # top-k: both f16 planes of V staged in LDS (two buffers), refinement from LDS
    # (no lo fetch, no wait on the tile loads in flight); twice the V stream
    "tk_lolds": [
        (TK, "constexpr int tk_nbuf(int topr) { return topr == 0 ? 2 : 3; }",
         "constexpr int tk_nbuf(int topr) { return topr == 0 ? 2 : 2; }"),
        (TK, "  constexpr int PIECES = NI / NW + 1;", "  constexpr int PIECES = 2 * (NI / NW) + 1;"),
        (TK, "  int* tperm = reinterpret_cast<int*>(tiles + NBUF * VT * RW);",
         "  int* tperm = reinterpret_cast<int*>(tiles + 2 * NBUF * VT * RW);"),
        (TK, """      __builtin_amdgcn_global_load_lds(Vsp + vr * RW + ((x % RW) ^ TK_SWZ(NK, r)), t + 64 * j, 16,
                                       0, 0);""", """      __builtin_amdgcn_global_load_lds(Vsp + vr * RW + ((x % RW) ^ TK_SWZ(NK, r)), t + 64 * j, 16,
                                       0, 0);
      __builtin_amdgcn_global_load_lds(Vlo + vr * RW + ((x % RW) ^ TK_SWZ(NK, r)),
                                       t + NBUF * VT * RW + 64 * j, 16, 0, 0);"""),
        (TK, """    const int64_t vr = ibase + m < n_v ? ibase + m : n_v - 1;  // rows past n_v: NaN anyway
    uint4* scr = loscr + w * NK * 64;
#pragma unroll
    for (int s = 0; s < NK; ++s)
      __builtin_amdgcn_global_load_lds(Vlo + vr * RW + 4 * s + q, scr + s * 64, 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll""", """    (void)ibase;
    (void)loscr;
#pragma unroll"""),
        (TK, "      const tk_half8 bl = __builtin_bit_cast(tk_half8, scr[s * 64 + lane]);",
         "      const tk_half8 bl = __builtin_bit_cast(tk_half8, tb[NBUF * VT * RW + ((4 * s + q) ^ swz)]);"),
        (TK, "  const size_t tiles = 16 * nbuf * vt * (size_t)(kq / 8) +",
         "  const size_t tiles = 2 * 16 * nbuf * vt * (size_t)(kq / 8) +"),
        (TK, "                       4 * 16 * nw * (size_t)rg + 16 * nw * 64 * (size_t)nk;",
         "                       4 * 16 * nw * (size_t)rg;"),
        (TK, "  uint64_t* lk = reinterpret_cast<uint64_t*>(loscr + NW * NK * 64);  // 16-byte aligned",
         "  uint64_t* lk = reinterpret_cast<uint64_t*>(loscr);  // 16-byte aligned"),
    ],
    # sweep16c: the next pivot row's broadcast issued one pivot earlier (before the
    # current pivot's update) and brought up to date on the copy by one more DPP fmac
    # (the same fp32 operation as on its register): the ds_bpermute latency leaves the
    # pivot chain, one VALU more per pivot
    "lookahead": [
        (GS, """  float rowp = rowgroup_bcast<0>(B[0]);
  float d = bcast16<0>(rowp);
  float rd = rcp_t(d);
  float f = rowp * rd;
  float nf = sel_lane16_n<0>(0.f, f);
  static_for<16>([&](auto pc) {
    constexpr int p = decltype(pc)::value;
    constexpr int qp = p >> 2, rp = p & 3, rn = (p + 1) & 3;
    asm volatile("s_nop 1" ::: "memory");
    // the register holding row p+1 first: then pivot p+1's row is final
    fmac_bcast16<p>(B[rn], nf);
    float dn = 0.f, rdn = 0.f, fn = 0.f, nfn = 0.f;
    if constexpr (p + 1 < 16) {
      constexpr int qn = (p + 1) >> 2;
      const float rown = rowgroup_bcast<qn>(B[rn]);
      dn = bcast16<p + 1>(rown);
      rdn = rcp_t(dn);
      fn = rown * rdn;
      nfn = sel_lane16_n<p + 1>(0.f, fn);
    }
    static_for<4>([&](auto rc) {
      constexpr int r = decltype(rc)::value;
      if constexpr (r != rn) fmac_bcast16<p>(B[r], nf);
    });""", """  float rowp = rowgroup_bcast<0>(B[0]);
  float pre = rowgroup_bcast<0>(B[1]);  // row 1 before pivot 0
  float d = bcast16<0>(rowp);
  float rd = rcp_t(d);
  float f = rowp * rd;
  float nf = sel_lane16_n<0>(0.f, f);
  static_for<16>([&](auto pc) {
    constexpr int p = decltype(pc)::value;
    constexpr int qp = p >> 2, rp = p & 3;
    asm volatile("s_nop 1" ::: "memory");
    float dn = 0.f, rdn = 0.f, fn = 0.f, nfn = 0.f;
    if constexpr (p + 1 < 16) {
      // row p+1 after pivot p, on its broadcast copy
      fmac_bcast16<p>(pre, nf);
      dn = bcast16<p + 1>(pre);
      rdn = rcp_t(dn);
      fn = pre * rdn;
      nfn = sel_lane16_n<p + 1>(0.f, fn);
    }
    static_for<4>([&](auto rc) {
      constexpr int r = decltype(rc)::value;
      fmac_bcast16<p>(B[r], nf);
    });
    if constexpr (p + 2 < 16) {  // row p+2 after pivots <= p: consumed by pivot p+1
      constexpr int q2 = (p + 2) / 4, r2 = (p + 2) % 4;
      pre = rowgroup_bcast<q2>(B[r2]);
    }"""),
    ],
    # timing bound (wrong results): the split-in-registers Gram (implicit) gathers only
    # rows 0..63 of Y (cache-hot): how much of the implicit launches is gather latency
    "hotgather": [
        (GS, "    TS::load_clamped(Y + (int64_t)(ids[j] >= 0 ? ids[j] : 0) * ld, s.y[j], d0, ld);",
         "    TS::load_clamped(Y + (int64_t)(ids[j] >= 0 ? (ids[j] & 63) : 0) * ld, s.y[j], d0, ld);"),
        (GS, "  if ((threadIdx.x & 63) == 0) {\n    const unsigned i = atomicAdd(rl.cnt, 1u);",
         "  if (false) {\n    const unsigned i = atomicAdd(rl.cnt, 1u);"),
    ],
    # rescue launch with 64 workgroups (its finished-block counter: 64 atomics, not 256)
    "rescue64wg": [
        (GS, "constexpr int kRescueGrid = 256;", "constexpr int kRescueGrid = 64;"),
    ],
    # top-k: 1.5x larger tiles at rank <= 64 (192 rows at k <= 64, 384 at k <= 32)
    "tk_vt_small": [
        (TK, "return topr == 0 ? 64 / nk : (nk == 4 ? 192 : 384 / nk);",
         "return topr == 0 ? 64 / nk : (nk == 4 ? 192 : 384 / nk);"),
    ],
    "tk_vt_small2": [
        (TK, "return topr == 0 ? 64 / nk : (nk == 4 ? 192 : 384 / nk);",
         "return topr == 0 ? 64 / nk : (nk == 4 ? 192 : 512 / nk);"),
    ],
    # the C-layout sweep only for NB = 4 (the round-4 choice) / in every elimination
    "sweepc_nb4": [
        (GS, "constexpr bool kSweepC = !SPLIT;", "constexpr bool kSweepC = NB == 4;"),
    ],
    "sweepc_all": [
        (GS, "constexpr bool kSweepC = !SPLIT;", "constexpr bool kSweepC = true;"),
    ],
    # timing bounds for the k <= 64 solve (wrong results): the C-layout sweep's pivot
    # chain removed (the interleaved Schur MFMAs kept), or only its row-group broadcast
    "fastsweep": [
        (GS, "  if ((threadIdx.x & 63) == 0) {\n    const unsigned i = atomicAdd(rl.cnt, 1u);",
         "  if (false) {\n    const unsigned i = atomicAdd(rl.cnt, 1u);"),
        (GS, """    dmin = fminf(dmin, d);
    asm volatile("s_nop 1" ::: "memory");
    // the register holding row p+1 first: then pivot p+1's row is final
    fmac_bcast16<p>(B[rn], nf);""", """    dmin = fminf(dmin, d);
    if constexpr (true) { hook(pc); return; }
    asm volatile("s_nop 1" ::: "memory");
    // the register holding row p+1 first: then pivot p+1's row is final
    fmac_bcast16<p>(B[rn], nf);"""),
    ],
    "noperm": [
        (GS, "  if ((threadIdx.x & 63) == 0) {\n    const unsigned i = atomicAdd(rl.cnt, 1u);",
         "  if (false) {\n    const unsigned i = atomicAdd(rl.cnt, 1u);"),
        (GS, """template <int G>
__device__ __forceinline__ float rowgroup_bcast(float x) {
  uint32_t a""", """template <int G>
__device__ __forceinline__ float rowgroup_bcast(float x) {
  if constexpr (true) return x;
  uint32_t a"""),
    ],
}


VARIANTS["lean"] = VARIANTS["bperm"] + VARIANTS["neg"]


def build(tag: str) -> str:
    # at the depth of csrc, so its "../../include" resolves to the repo's include/
    src = os.path.join(HERE, "..", "..", ".ab", tag)
    shutil.rmtree(src, ignore_errors=True)
    shutil.copytree(CSRC, src)
    for f, old, new in VARIANTS[tag]:
        p = os.path.join(src, f)
        if old == "@FILE":  # the whole file from a path (outside the tree: a candidate)
            shutil.copyfile(new, p)
            continue
        if old == "@HEAD":  # the whole file as committed
            rel = "recommender-system-using-apache-spark-mllib-_amd/csrc/" + f
            open(p, "w").write(subprocess.check_output(["git", "show", "HEAD:" + rel],
                                                       cwd=os.path.join(HERE, "..", ".."),
                                                       text=True))
            continue
        s = open(p).read()
        if old not in s:
            raise SystemExit(f"{tag}: patch does not apply to {f}: {old[:70]!r}")
        open(p, "w").write(s.replace(old, new))
    objs = []
    procs = []
    for s in ("csr_build", "gram_solve", "predict", "topk"):
        o = os.path.join(src, s + ".o")
        objs.append(o)
        procs.append(subprocess.Popen(["/opt/rocm/bin/hipcc", "-O3", "-fPIC", "-std=c++17",
                                       "--offload-arch=gfx950", "-c", os.path.join(src, s + ".hip"),
                                       "-o", o]))
    for p in procs:
        if p.wait() != 0:
            raise SystemExit(f"{tag}: compile failed")
    lib = os.path.join(HERE, f"libals_{tag}.so")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950"] + objs
                          + ["-o", lib])
    if "--dev" in sys.argv:  # the phase-ablation kernels (tools/dev_ablate.hip) on this copy
        dev_src = os.path.join(src, "dev_ablate.hip")
        s = open(os.path.join(HERE, "..", "dev_ablate.hip")).read().replace(
            '"../recommender-system-using-apache-spark-mllib-_amd/csrc/gram_solve.hip"',
            '"gram_solve.hip"')
        open(dev_src, "w").write(s)
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-fPIC", "-shared",
                               "--offload-arch=gfx950", "-std=c++17", dev_src, "-o",
                               os.path.join(HERE, f"libals_dev_{tag}.so")])
    shutil.rmtree(src)
    return lib


if __name__ == "__main__":
    for t in [a for a in sys.argv[1:] if not a.startswith("--")]:
        print("built", build(t), flush=True)
