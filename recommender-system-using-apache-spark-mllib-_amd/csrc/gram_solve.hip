// K2 + K3 (+ K2b) — normal equations and Cholesky solve for one ALS half-sweep.
//
// Replaces, per dst row j (Spark ml/recommendation/ALS.scala, upstream):
//   computeFactors -> NormalEquation.add   (blas.dspr + blas.daxpy, fp64)
//                  -> CholeskySolver.solve (ata += lambda*n on the diagonal,
//                                           LAPACK dppsv "U", fp64, result -> Float)
//   computeYtY (implicit)                  (dspr over all src rows + treeAggregate)
// reached from ALS.train at RecommenderSystem.py:148-149, :163, :218.
//
// MI355X design:
//  * A task is a whole "light" row (<= chunk ratings, default 2048) or one
//    2048-rating chunk of a heavy row; light rows arrive longest-first (LPT).
//    k <= 64: one wavefront per task (gram_solve_kernel<CN>); 64 < k <= 128: one
//    wavefront per task with the whole 128 x 128 system in its registers
//    (gram_solve_w1_kernel, "W1").  One code path per (k range, implicit).
//  * Gram on the f16 matrix cores with fp32-grade products: every operand t is
//    carried as hi = f16_rn(t), lo = f16_rn(t - hi) after a power-of-two scale
//    (largest |t| in [2^14, 2^15), from max |Y| and max |r| computed on the
//    device), and each 16 x 16 tile accumulates hi.hi + hi.lo + lo.hi with three
//    v_mfma_f32_16x16x32_f16 per 32 ratings (~2^-21 relative per product).
//    MFMA K = rating index; lane (q, m) holds ratings 8q..8q+7 of a step and dims
//    m*CN .. m*CN+CN-1, so only the CN(CN+1)/2 upper tiles of the dim-permuted
//    Gram are computed (Spark's packed dspr uses the same symmetry).
//    Explicit: Y is pre-split once per half-sweep into hi|lo words
//    (split_table_kernel) and the rhs runs on the matrix cores; implicit: the
//    fp32 rows are split in registers after the per-rating weight, whose
//    sqrt(alpha |r|) and (1 + alpha |r|) are computed once per rating when the
//    64-rating block is staged in LDS.
//  * Accumulation: fp32 within a task (<= 2048 ratings; test_gpu_configs pins
//    the error at the production chunk), fp64 across a heavy row's chunks
//    (partial slots summed element-wise in a fixed order, deterministic).
//  * Normal equations as CholeskySolver.solve: A_ii += lambda * n (n = #ratings,
//    implicit: #ratings > 0), implicit YtY merged in fp64 before the one
//    rounding to fp32; padded dims get identity rows and zero rhs.
//  * Solve (fp32, same solution as Spark's dppsv): k <= 32 column-per-lane panel
//    LDL^T with the trailing tiles on fp32 MFMA; k in (32, 64] and (64, 128]:
//    block elimination with 16 x 16 diagonal inverses by the sweep operator
//    (VALU, DPP broadcasts) and the Pm / Schur products on the matrix cores —
//    split f16 (fp32-grade) for rank 65-128 implicit light rows and heavy rows,
//    fp32 MFMA for the explicit light rows and rank <= 64 (see w1_solve).
//  * YtY (K2b): 512-row tasks of the same MFMA Gram, fp64 slots, parallel slot
//    sum, fixed order.
#include "als_common.h"

#include <algorithm>
#include <utility>

namespace als {

typedef float floatx4 __attribute__((ext_vector_type(4)));

// src rows per YtY task: a multiple of 32 sized for ~kYtyTasks tasks (two resident
// workgroups per CU, so every task runs in one round: at 512-row tasks a 162k-row
// side left 62 CUs with two tasks and 194 with one, a 59k-row side 140 CUs idle)
constexpr int kYtyTasks = 512;
__host__ __device__ inline int64_t yty_chunk(int64_t n) {
  const int64_t c = (n + kYtyTasks - 1) / kYtyTasks;
  return c < 32 ? 32 : (c + 31) / 32 * 32;
}
// workgroups walking the rescue list (rescue64_kernel).  64, not 256: an empty list (the
// usual case) still costs one finished-block atomic per workgroup on one word; configs[1]
// LAUNCH2 + RESCUE phases 3 us shorter per half-sweep (profiles/r05/ab_rescue_grid.jsonl).
constexpr int kRescueGrid = 64;
// Largest LDL^T pivot spread (max / min pivot of the real dims, a lower bound on
// cond(A)) the fp32 solve keeps: beyond it the row is re-solved in fp64.  Regularised
// rating data (lambda 0.1) spread far less (pivots lie in [lambda_min, lambda_max] and
// the diagonal stays within a few times lambda n); implicit confidences spanning six
// decades spread by 1e3-1e5 and reach 1e-3 errors in fp32.
constexpr float kCondMax = 32.f;
// The same limit for the implicit rows of the rank 65-128 (W1) solve, which has no
// iterative refinement (ranks <= 64 refine every implicit row against Spark's fp64
// residual): implicit counts 1..1e6 at rank 128 left rows with spreads in (8, 32] at
// 4.9e-6..5.6e-6 against the fp64 oracle; at 8 every row of that test is within 8.4e-8
// (the rows beyond it re-solved in fp64) and configs[2] re-solves none (its item rows
// spread 2-4, user rows < 2): 9.01 / 9.09 ms/iter at 32 / 8, profiles/r06/ab_cond_implicit.txt.
constexpr float kCondMaxImplicit = 8.f;
constexpr int kMaxRank = 128;

template <int CN>
struct Cfg {
  static constexpr int KP = 16 * CN;                  // padded rank
  static constexpr int NT = CN * (CN + 1) / 2;        // upper 16x16 tiles
  static constexpr int NP = KP * (KP + 1) / 2;        // packed lower entries
  static constexpr int SLOT = (NT * 4 + CN + 1) * 64; // doubles per partial slot
};

static inline int cn_for_k(int k) { return k <= 16 ? 1 : (k <= 32 ? 2 : (k <= 64 ? 4 : 8)); }

// Compile-time loop over 0..N-1 (indices are constant expressions in the body,
// so register arrays indexed through constexpr tables stay in registers).
template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// Wave-local LDS ordering (lanes of one wave exchanging values through LDS).
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// Compiler-only ordering of one wave's LDS accesses: the LDS executes a wave's DS
// instructions in issue order, so a read issued after a write (any lane) returns
// the written data without draining lgkmcnt; the compiler inserts the waits for
// the loaded values where they are used.
__device__ __forceinline__ void wave_lds_order() { asm volatile("" ::: "memory"); }

template <int CN>
__device__ __forceinline__ void load_dims(const float* __restrict__ p, float (&y)[CN]) {
  if constexpr (CN == 4) {
    const float4 v = *reinterpret_cast<const float4*>(p);
    y[0] = v.x; y[1] = v.y; y[2] = v.z; y[3] = v.w;
  } else if constexpr (CN == 2) {
    const float2 v = *reinterpret_cast<const float2*>(p);
    y[0] = v.x; y[1] = v.y;
  } else {
    y[0] = *p;
  }
}

// Tile-set policy: which 16x16 Gram tiles a wavefront accumulates.
//   N tiles; tile t is block (g1(t), g2(t)), g1 <= g2, in dims-block units
//   (block c holds dims d = 16-index * CN + c).
//   NC dims-blocks are gathered per rating ("local columns"; gcol(lc) = block),
//   l1(t), l2(t) are tile t's local columns; NR rhs blocks = local columns 0..NR-1
//   (NRA = max(NR, 1), the register array size).
//   load(p, y, d0, k): this lane's NC values of one factor row (p = row + d0),
//   zero for dims >= k (never reads past the row: ld % 4 == 0, k <= ld).
// FullTiles<CN>: all CN(CN+1)/2 upper tiles (one wavefront per system, k <= 64).
template <int CN>
struct FullTiles {
  static constexpr int N = CN * (CN + 1) / 2, NC = CN, NR = CN, NRA = CN;
  __host__ __device__ static constexpr int l1(int t) {
    int a = 0;
    while (t >= CN - a) { t -= CN - a; ++a; }
    return a;
  }
  __host__ __device__ static constexpr int l2(int t) {
    int a = 0;
    while (t >= CN - a) { t -= CN - a; ++a; }
    return a + t;
  }
  __host__ __device__ static constexpr int gcol(int c) { return c; }
  __host__ __device__ static constexpr int g1(int t) { return l1(t); }
  __host__ __device__ static constexpr int g2(int t) { return l2(t); }
  __device__ static __forceinline__ void load(const float* __restrict__ p, float (&y)[NC], int d0,
                                              int k) {
    if (d0 < k) {
      load_dims<CN>(p, y);
    } else {
#pragma unroll
      for (int c = 0; c < NC; ++c) y[c] = 0.f;
    }
  }
  // Unconditional load of this lane's dims from row `row` (offsets clamped into
  // [0, ld): lanes whose dims are >= k read real dims, masked out after the Gram).
  __device__ static __forceinline__ void load_clamped(const float* __restrict__ row,
                                                      float (&y)[NC], int d0, int ld) {
    if constexpr (CN == 8) {
      auto cl = [&](int o) { return o + 4 <= ld ? o : ld - 4; };
      const float4 a = *reinterpret_cast<const float4*>(row + cl(d0));
      const float4 b = *reinterpret_cast<const float4*>(row + cl(d0 + 4));
      y[0] = a.x; y[1] = a.y; y[2] = a.z; y[3] = a.w;
      y[4] = b.x; y[5] = b.y; y[6] = b.z; y[7] = b.w;
    } else {
      load_dims<CN>(row + (d0 + CN <= ld ? d0 : ld - CN), y);
    }
  }
  // This lane's NC words of a pre-split row (p = row + m*CN; rows are kp = 16*CN wide).
  __device__ static __forceinline__ void load_pre(const uint32_t* __restrict__ p,
                                                  uint32_t (&w)[NC]) {
    if constexpr (CN == 1) {
      w[0] = p[0];
    } else if constexpr (CN == 2) {
      const uint2 v = *reinterpret_cast<const uint2*>(p);
      w[0] = v.x; w[1] = v.y;
    } else if constexpr (CN == 4) {
      const uint4 v = *reinterpret_cast<const uint4*>(p);
      w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
    } else {
      static_assert(CN == 8, "pre-split rows: CN in {1, 2, 4, 8}");
      const uint4 a = *reinterpret_cast<const uint4*>(p);
      const uint4 b = *reinterpret_cast<const uint4*>(p + 4);
      w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
      w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
    }
  }
};

// WgTiles<R>: wavefront R of the 4-wave workgroup that owns one k <= 128 system
// (CN = 8, blocks H0 = 0..3, H1 = 4..7).  R0: upper(H0) 10 tiles + rhs H0;
// R1: upper(H1) 10 tiles + rhs H1; R2: {0,1} x H1, 8 tiles; R3: {2,3} x H1.
// Each wave gathers only the dims its tiles need (16 or 24 B per lane).
template <int R>
struct WgTiles {
  static_assert(R >= 0 && R < 4, "4 waves");
  static constexpr int N = R < 2 ? 10 : 8, NC = R < 2 ? 4 : 6, NR = R < 2 ? 4 : 0,
                       NRA = R < 2 ? 4 : 1;
  __host__ __device__ static constexpr int gcol(int c) {
    return R == 0 ? c : (R == 1 ? 4 + c : (c < 2 ? 2 * (R - 2) + c : c + 2));
  }
  __host__ __device__ static constexpr int l1(int t) { return R < 2 ? FullTiles<4>::l1(t) : t / 4; }
  __host__ __device__ static constexpr int l2(int t) {
    return R < 2 ? FullTiles<4>::l2(t) : 2 + t % 4;
  }
  __host__ __device__ static constexpr int g1(int t) { return gcol(l1(t)); }
  __host__ __device__ static constexpr int g2(int t) { return gcol(l2(t)); }
  __device__ static __forceinline__ void load(const float* __restrict__ p, float (&y)[NC], int d0,
                                              int k) {
#pragma unroll
    for (int c = 0; c < NC; ++c) y[c] = 0.f;
    if constexpr (R < 2) {
      if (d0 + 4 * R < k) {
        const float4 v = *reinterpret_cast<const float4*>(p + 4 * R);
        y[0] = v.x; y[1] = v.y; y[2] = v.z; y[3] = v.w;
      }
    } else {
      constexpr int o = 2 * (R - 2);
      if (d0 + o < k) {
        const float2 v = *reinterpret_cast<const float2*>(p + o);
        y[0] = v.x; y[1] = v.y;
      }
      if (d0 + 4 < k) {
        const float4 v = *reinterpret_cast<const float4*>(p + 4);
        y[2] = v.x; y[3] = v.y; y[4] = v.z; y[5] = v.w;
      }
    }
  }
  __device__ static __forceinline__ void load_clamped(const float* __restrict__ row,
                                                      float (&y)[NC], int d0, int ld) {
    auto cl = [&](int o, int w) { return o + w <= ld ? o : ld - w; };
    if constexpr (R < 2) {
      const float4 v = *reinterpret_cast<const float4*>(row + cl(d0 + 4 * R, 4));
      y[0] = v.x; y[1] = v.y; y[2] = v.z; y[3] = v.w;
    } else {
      const float2 u = *reinterpret_cast<const float2*>(row + cl(d0 + 2 * (R - 2), 2));
      const float4 v = *reinterpret_cast<const float4*>(row + cl(d0 + 4, 4));
      y[0] = u.x; y[1] = u.y;
      y[2] = v.x; y[3] = v.y; y[4] = v.z; y[5] = v.w;
    }
  }
  __device__ static __forceinline__ void load_pre(const uint32_t* __restrict__ p,
                                                  uint32_t (&w)[NC]) {
    if constexpr (R < 2) {
      const uint4 v = *reinterpret_cast<const uint4*>(p + 4 * R);
      w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
    } else {
      const uint2 u = *reinterpret_cast<const uint2*>(p + 2 * (R - 2));
      const uint4 v = *reinterpret_cast<const uint4*>(p + 4);
      w[0] = u.x; w[1] = u.y;
      w[2] = v.x; w[3] = v.y; w[4] = v.z; w[5] = v.w;
    }
  }
};

// Gather the factor rows of one half-block (32 ratings = 8 MFMA steps) into
// registers: step t, lane (q, m) gets its TS dims among m*CN .. m*CN+CN-1 of
// rating 4t+q.
template <int CN, class TS>
__device__ __forceinline__ void gather_half(float (&y)[8][TS::NC], int ci, int base, int nrem,
                                            const float* __restrict__ Y, int ld, int d0, int k) {
  const int q = (threadIdx.x & 63) >> 4;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int src = base + 4 * t + q;
    const int s = __shfl(ci, src);
    if (src < nrem) {
      TS::load(Y + (int64_t)s * ld + d0, y[t], d0, k);
    } else {
#pragma unroll
      for (int c = 0; c < TS::NC; ++c) y[t][c] = 0.f;
    }
  }
}

// MFMA over one gathered half-block: acc[tile] += (w_a y)(y)^T over the tiles of
// TS, and bf += w_b y over its rhs blocks.
template <class TS, bool IMPLICIT>
__device__ __forceinline__ void mfma_half(const float (&y)[8][TS::NC], float rv, int base,
                                          int nrem, float alpha, floatx4 (&acc)[TS::N],
                                          float (&bf)[TS::NRA]) {
  const int q = (threadIdx.x & 63) >> 4;
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    if (base + 16 * g < nrem) {  // wave-uniform: skip empty 16-rating groups
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int t = 4 * g + j;
        const float r = __shfl(rv, base + 4 * t + q);
        float ya[TS::NC];
        float wb;
        if constexpr (IMPLICIT) {
          const float c1 = alpha * fabsf(r);
          wb = r > 0.f ? 1.f + c1 : 0.f;
#pragma unroll
          for (int c = 0; c < TS::NC; ++c) ya[c] = c1 * y[t][c];
        } else {
          wb = r;
#pragma unroll
          for (int c = 0; c < TS::NC; ++c) ya[c] = y[t][c];
        }
        static_for<TS::N>([&](auto ti) {
          constexpr int tt = decltype(ti)::value;
          constexpr int a = TS::l1(tt), b = TS::l2(tt);
          acc[tt] = __builtin_amdgcn_mfma_f32_16x16x4f32(ya[a], y[t][b], acc[tt], 0, 0, 0);
        });
#pragma unroll
        for (int c = 0; c < TS::NR; ++c) bf[c] = fmaf(wb, y[t][c], bf[c]);
      }
    }
  }
}

// Accumulate the (weighted) Gram and rhs of ratings [pb, pe) of one row.
// tot[t][r]: this lane's 4 accumulator rows of upper tile t (MFMA C layout),
// summed over 64-rating blocks in AccT (each block's own sum is an exact-product
// fp32 MFMA chain of <= 16 steps); btot[c]: partial rhs for dim m*CN+c over this
// lane's rating slot q (summed over q by the caller); npos: #ratings > 0.
// Software pipeline: the row gathers of half-block h+1 are in flight while the
// MFMAs of half-block h run; rating indices are loaded one 64-block ahead.
template <int CN, bool IMPLICIT, bool IDENT, class AccT, class TS = FullTiles<CN>>
__device__ __forceinline__ void gram_accumulate(const int32_t* __restrict__ col,
                                                const float* __restrict__ val, int64_t pb,
                                                int64_t pe, const float* __restrict__ Y, int ld,
                                                int k, float alpha, AccT (&tot)[TS::N][4],
                                                AccT (&btot)[TS::NRA], int& npos) {
  constexpr int NT = TS::N;
  const int lane = threadIdx.x & 63, m = lane & 15;
  const int d0 = m * CN;  // dims in [k, ld) are zero by contract (see als_hip.h)
  if (pe <= pb) return;
  auto load_idx = [&](int64_t base, int& ci, float& rv) {
    ci = 0;
    rv = 0.f;
    if (base + lane < pe) {
      ci = IDENT ? (int)(base + lane) : col[base + lane];
      rv = IDENT ? 1.f : val[base + lane];
    }
  };
  int ci_c, ci_n;
  float rv_c, rv_n;
  load_idx(pb, ci_c, rv_c);
  load_idx(pb + 64, ci_n, rv_n);
  float yA[8][TS::NC], yB[8][TS::NC];
  int nrem = (int)((pe - pb) < 64 ? (pe - pb) : 64);
  gather_half<CN, TS>(yA, ci_c, 0, nrem, Y, ld, d0, k);
  for (int64_t base = pb; base < pe; base += 64) {
    const int64_t nbase = base + 64;
    const int nrem_n = nbase < pe ? (int)((pe - nbase) < 64 ? (pe - nbase) : 64) : 0;
    if (32 < nrem) gather_half<CN, TS>(yB, ci_c, 32, nrem, Y, ld, d0, k);
    floatx4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    float bf[TS::NRA];
#pragma unroll
    for (int c = 0; c < TS::NRA; ++c) bf[c] = 0.f;
    mfma_half<TS, IMPLICIT>(yA, rv_c, 0, nrem, alpha, acc, bf);
    if (nrem_n > 0) gather_half<CN, TS>(yA, ci_n, 0, nrem_n, Y, ld, d0, k);
    if (32 < nrem) mfma_half<TS, IMPLICIT>(yB, rv_c, 32, nrem, alpha, acc, bf);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
#pragma unroll
      for (int r = 0; r < 4; ++r) tot[t][r] += (AccT)acc[t][r];
    }
#pragma unroll
    for (int c = 0; c < TS::NR; ++c) btot[c] += (AccT)bf[c];
    if constexpr (IMPLICIT) npos += __popcll(__ballot(lane < nrem && rv_c > 0.f));
    ci_c = ci_n;
    rv_c = rv_n;
    nrem = nrem_n;
    if (nrem_n > 0) load_idx(nbase + 64, ci_n, rv_n);
  }
}

// ---------------------------------------------------------------------------
// Row Grams on the f16 matrix cores with fp32-grade products ("split" Gram).
//
// v_mfma_f32_16x16x4_f32 runs at the fp32 VECTOR rate on gfx950 and occupies
// the VALU issue port, so an fp32-MFMA Gram leaves nothing for the solves of
// the other waves.  Here every gathered value t = w*y (w = per-launch power-of-
// two scale, times sqrt(alpha |r|) for implicit) is split into
//   t = hi + lo,  hi = f16_rn(t),  lo = f16_rn(t - hi)   (~22 significant bits)
// and the Gram tile is  sum hi_a hi_b + hi_a lo_b + lo_a hi_b  — three
// v_mfma_f32_16x16x32_f16 per tile per 32 ratings (16x the fp32-MFMA rate,
// so 5.3x fewer matrix cycles), exact f16 products accumulated in fp32.  The
// dropped lo*lo term and the two roundings are ~2^-21 relative per product:
// the Gram matches an fp32 one to within its own accumulation error.
// The scale keeps |t| in [2^14, 2^15) for the largest entry, so hi never
// overflows and lo stays normal for entries within ~2^17 of the largest.
// MFMA K dimension = rating index: lane (q, m) holds ratings 8q..8q+7 of a
// 32-rating step and dims m*CN .. m*CN+CN-1, exactly the dim permutation of
// the fp32 path, so the C layout (and the solve that consumes it) is unchanged.
// rhs b = sum coef * y stays an fp32 VALU FMA on the unscaled values.
// ---------------------------------------------------------------------------
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef _Float16 half8v __attribute__((ext_vector_type(8)));
typedef float float2v __attribute__((ext_vector_type(2)));

// The split of two weighted values w0 y0, w1 y1 straight from the fp32 operands:
// hi = f16(w y) and lo = f16(w y - hi), each one v_fma_mix (the product and the
// residual formed inside one fp32 fma; lo also keeps the product's own fp32 rounding
// error), 4 VALU per pair instead of a multiply, a packed convert, two converts back,
// a subtract and a packed convert (round 5): configs[2] 9.11 -> 9.06 ms/iter,
// profiles/r06/ab_fma_mix_split.jsonl.
__device__ __forceinline__ void split_pair_w(float y0, float w0, float y1, float w1, uint32_t& hi,
                                             uint32_t& lo) {
  uint32_t h, l;
  asm("v_fma_mixlo_f16 %0, %1, %2, 0 op_sel_hi:[0,0,0]" : "=v"(h) : "v"(y0), "v"(w0));
  asm("v_fma_mixhi_f16 %0, %1, %2, 0 op_sel_hi:[0,0,0]" : "+v"(h) : "v"(y1), "v"(w1));
  asm("v_fma_mixlo_f16 %0, %1, %2, -%3 op_sel:[0,0,0] op_sel_hi:[0,0,1]"
      : "=v"(l) : "v"(y0), "v"(w0), "v"(h));
  asm("v_fma_mixhi_f16 %0, %1, %2, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "+v"(l) : "v"(y1), "v"(w1), "v"(h));
  hi = h;
  lo = l;
}

__device__ __forceinline__ half8v as_h8(const uint32_t (&v)[4]) {
  return __builtin_bit_cast(half8v, make_uint4(v[0], v[1], v[2], v[3]));
}

// Power-of-two scale for the split: the largest |w y| lands in [2^14, 2^15).
__device__ __forceinline__ int split_exponent(float m) {
  if (!(m > 0.f) || !(m < 3.0e38f)) return 0;
  int e = 14 - ilogbf(m);
  return e < -60 ? -60 : (e > 60 ? 60 : e);
}

// Per-step register set of the split Gram: 8 ratings x NC dims of this lane
// (unscaled).  The per-rating weights stay in the LDS staging block until the
// step is consumed: w = Gram weight (implicit: sc sqrt(alpha |r|)), b = rhs
// weight (implicit: (1 + alpha |r|) [r > 0]), both 0 for missing ratings.
template <int NC>
struct SplitStep {
  float y[8][NC];
};

// Stage the (column, rating) pairs of one 64-rating block in LDS (wave-private).
__device__ __forceinline__ void stage_block(int* __restrict__ st_c, float* __restrict__ st_r, int ci,
                                            float rv) {
  const int lane = threadIdx.x & 63;
  st_c[lane] = ci;
  st_r[lane] = rv;
}

// Split Gram staging: columns, Gram weights and rhs weights of one 64-rating
// block (computed once per rating here instead of once per lane of its group).
template <bool IMPLICIT>
__device__ __forceinline__ void stage_weights(int* __restrict__ st_c, float* __restrict__ st_w,
                                              float* __restrict__ st_b, int ci, float rv, float sc,
                                              float alpha) {
  const int lane = threadIdx.x & 63;
  const bool v = ci >= 0;
  float w, b;
  if constexpr (IMPLICIT) {
    const float c1 = alpha * fabsf(rv);
    w = v ? sc * __builtin_sqrtf(c1) : 0.f;
    b = (v && rv > 0.f) ? 1.f + c1 : 0.f;
  } else {
    w = v ? sc : 0.f;
    b = v ? rv : 0.f;
  }
  st_c[lane] = ci;
  st_w[lane] = w;
  st_b[lane] = b;
}

// Issue the gathers of one 32-rating step (half h of the staged block).
template <int CN, class TS>
__device__ __forceinline__ void split_issue(SplitStep<TS::NC>& s, const int* __restrict__ st_c,
                                            int h, const float* __restrict__ Y, int ld, int d0,
                                            int k) {
  const int q = (threadIdx.x & 63) >> 4;
  const int o = 32 * h + 8 * q;
  const int4 c0 = *reinterpret_cast<const int4*>(st_c + o);
  const int4 c1 = *reinterpret_cast<const int4*>(st_c + o + 4);
  const int ids[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
#pragma unroll
  for (int j = 0; j < 8; ++j)
    TS::load_clamped(Y + (int64_t)(ids[j] >= 0 ? ids[j] : 0) * ld, s.y[j], d0, ld);
}

// Consume one step, part 1 (VALU): rhs FMAs and the hi/lo split of w*y.
template <class TS, bool IMPLICIT>
__device__ __forceinline__ void split_prepare(const SplitStep<TS::NC>& s,
                                              const float* __restrict__ st_w,
                                              const float* __restrict__ st_b, int h,
                                              uint32_t (&hi)[TS::NC][4], uint32_t (&lo)[TS::NC][4],
                                              float (&bf)[TS::NRA]) {
  const int o = 32 * h + 8 * ((threadIdx.x & 63) >> 4);
  const float4 w0 = *reinterpret_cast<const float4*>(st_w + o);
  const float4 w1 = *reinterpret_cast<const float4*>(st_w + o + 4);
  const float4 b0 = *reinterpret_cast<const float4*>(st_b + o);
  const float4 b1 = *reinterpret_cast<const float4*>(st_b + o + 4);
  const float w[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
  const float b[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
  for (int c = 0; c < TS::NR; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) bf[c] = fmaf(b[j], s.y[j][c], bf[c]);
#pragma unroll
  for (int c = 0; c < TS::NC; ++c)
#pragma unroll
    for (int p = 0; p < 4; ++p)
      split_pair_w(s.y[2 * p][c], w[2 * p], s.y[2 * p + 1][c], w[2 * p + 1], hi[c][p], lo[c][p]);
}

// Part 2 (matrix cores): 3 f16 MFMAs per tile.
template <class TS>
__device__ __forceinline__ void split_mfma(const uint32_t (&hi)[TS::NC][4],
                                           const uint32_t (&lo)[TS::NC][4],
                                           floatx4 (&acc)[TS::N]) {
  static_for<TS::N>([&](auto ti) {
    constexpr int tt = decltype(ti)::value;
    constexpr int a = TS::l1(tt), b = TS::l2(tt);
    const half8v ha = as_h8(hi[a]), hb = as_h8(hi[b]);
    acc[tt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ha, hb, acc[tt], 0, 0, 0);
    acc[tt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ha, as_h8(lo[b]), acc[tt], 0, 0, 0);
    acc[tt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_h8(lo[a]), hb, acc[tt], 0, 0, 0);
  });
}

// Gram + rhs of ratings [pb, pe) of one row with the split f16 MFMA.
// acc: scaled Gram tiles (x sc^2), bf: per-lane partial rhs (unscaled, summed
// over the 4 rating slots q by the caller), npos: #ratings > 0 (implicit).
// Pipeline: the gathers of step s+1 are in flight while step s is consumed;
// the (column, rating) pairs of the next 64-block are prefetched into registers
// and staged in LDS (`st`, 128 words, wave-private) when that block starts.
template <int CN, bool IMPLICIT, class TS = FullTiles<CN>>
__device__ __forceinline__ void gram_accumulate_split(
    const int32_t* __restrict__ col, const float* __restrict__ val, int64_t pb, int64_t pe,
    const float* __restrict__ Y, int ld, int k, float alpha, float sc,
    floatx4 (&acc)[TS::N], float (&bf)[TS::NRA], int& npos, int* __restrict__ st) {
  const int lane = threadIdx.x & 63, m = lane & 15;
  const int d0 = m * CN;
  int* st_c = st;  // 192 words: columns, Gram weights, rhs weights
  float* st_w = reinterpret_cast<float*>(st + 64);
  float* st_b = reinterpret_cast<float*>(st + 128);
  if (pe <= pb) return;
  auto load_idx = [&](int64_t base, int& ci, float& rv) {
    ci = -1;
    rv = 0.f;
    if (base + lane < pe) {
      ci = col[base + lane];
      rv = val[base + lane];
    }
  };
  const int64_t n = pe - pb;
  const int nsteps = (int)((n + 31) >> 5);
  int ci_n, ci_c;
  float rv_n, rv_c;
  load_idx(pb, ci_c, rv_c);
  load_idx(pb + 64, ci_n, rv_n);
  stage_weights<IMPLICIT>(st_c, st_w, st_b, ci_c, rv_c, sc, alpha);
  if constexpr (IMPLICIT) npos += __popcll(__ballot(ci_c >= 0 && rv_c > 0.f));
  wave_lds_sync();
  // One register set for the gathered rows: step s is split into its f16
  // operands, then the gathers of step s+1 are issued into the same registers,
  // then step s's MFMAs run while those loads are in flight.
  SplitStep<TS::NC> sA;
  split_issue<CN, TS>(sA, st_c, 0, Y, ld, d0, k);
  // rhs: fp32 partials per lane over 64-rating blocks, summed into bf
  float bp[TS::NRA];
#pragma unroll
  for (int c = 0; c < TS::NRA; ++c) bp[c] = 0.f;
  for (int s = 0; s < nsteps; ++s) {
    uint32_t hi[TS::NC][4], lo[TS::NC][4];
    split_prepare<TS, IMPLICIT>(sA, st_w, st_b, s & 1, hi, lo, bp);
    const int s1 = s + 1;
    if (s1 < nsteps) {
      // step s1 uses block s1>>1, half s1&1; a new block is staged from the
      // pairs prefetched one block earlier
      if ((s1 & 1) == 0) {
        stage_weights<IMPLICIT>(st_c, st_w, st_b, ci_n, rv_n, sc, alpha);
        if constexpr (IMPLICIT) npos += __popcll(__ballot(ci_n >= 0 && rv_n > 0.f));
        wave_lds_sync();
        load_idx(pb + 64 * (int64_t)((s1 >> 1) + 1), ci_n, rv_n);
      }
      split_issue<CN, TS>(sA, st_c, s1 & 1, Y, ld, d0, k);
    }
    split_mfma<TS>(hi, lo, acc);
    if (s & 1) {
#pragma unroll
      for (int c = 0; c < TS::NRA; ++c) {
        bf[c] += bp[c];
        bp[c] = 0.f;
      }
    }
  }
#pragma unroll
  for (int c = 0; c < TS::NRA; ++c) bf[c] += bp[c];
}

// ---------------------------------------------------------------------------
// Explicit feedback: the Gram is unweighted, so every factor row is split once
// per half-sweep into a table (split_table_kernel): Ysp[row][d] = f16 hi |
// f16 lo << 16 of 2^ey * Y[row][d] (padding dims and the extra row n_src zero).
// The Gram loop then gathers 4 B per dim (as for fp32) and forms its f16
// operands with v_perm_b32 alone.  Ratings are split the same way (2^er * r)
// when a 64-rating block is staged, and the rhs b = sum r y runs on the matrix
// cores too: B operand column 0 = hi(r), column 1 = lo(r), all other columns 0,
// so C[i][0] + C[i][1] = sum (hi_y + lo_y)(hi_r + lo_r).  Ratings past the end
// of the row point at the zero row and add nothing.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t split_word(float t) {
  const _Float16 h = (_Float16)t;  // round to nearest
  const _Float16 l = (_Float16)(t - (float)h);
  return (uint32_t)__builtin_bit_cast(unsigned short, h) |
         ((uint32_t)__builtin_bit_cast(unsigned short, l) << 16);
}

template <int NC>
struct PreStep {
  uint32_t w[8][NC];  // split words: rating j of this lane's slot, its NC dims
  uint32_t r[8];      // split words of those ratings
};

template <class TS>
__device__ __forceinline__ void pre_issue(PreStep<TS::NC>& s, const int* __restrict__ st_c,
                                          const uint32_t* __restrict__ st_r, int h,
                                          const uint32_t* __restrict__ base, uint32_t kp) {
  const int q = (threadIdx.x & 63) >> 4;
  const int o = 32 * h + 8 * q;
  const int4 c0 = *reinterpret_cast<const int4*>(st_c + o);
  const int4 c1 = *reinterpret_cast<const int4*>(st_c + o + 4);
  const uint4 r0 = *reinterpret_cast<const uint4*>(st_r + o);
  const uint4 r1 = *reinterpret_cast<const uint4*>(st_r + o + 4);
  const int ids[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
  s.r[0] = r0.x; s.r[1] = r0.y; s.r[2] = r0.z; s.r[3] = r0.w;
  s.r[4] = r1.x; s.r[5] = r1.y; s.r[6] = r1.z; s.r[7] = r1.w;
#pragma unroll
  for (int j = 0; j < 8; ++j) TS::load_pre(base + (uint64_t)(uint32_t)ids[j] * kp, s.w[j]);
}

// f16 operands of one step: ratings (2p, 2p+1) share a dword, hi halves and lo
// halves; rhs B operand by lane column (m = 0: hi(r), m = 1: lo(r), else 0).
template <class TS>
__device__ __forceinline__ void pre_operands(const PreStep<TS::NC>& s, uint32_t rsel,
                                             uint32_t (&hi)[TS::NC][4], uint32_t (&lo)[TS::NC][4],
                                             uint32_t (&rb)[4]) {
#pragma unroll
  for (int c = 0; c < TS::NC; ++c)
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      hi[c][p] = __builtin_amdgcn_perm(s.w[2 * p + 1][c], s.w[2 * p][c], 0x05040100u);
      lo[c][p] = __builtin_amdgcn_perm(s.w[2 * p + 1][c], s.w[2 * p][c], 0x07060302u);
    }
#pragma unroll
  for (int p = 0; p < 4; ++p) rb[p] = __builtin_amdgcn_perm(s.r[2 * p + 1], s.r[2 * p], rsel);
}

// Keep the operands where they are formed: otherwise the scheduler sinks the
// v_perm next to their MFMAs, past the next step's loads into the same
// registers, and the loop then carries copies of the step (waiting for its
// loads early).
template <class TS>
__device__ __forceinline__ void pin_operands(uint32_t (&hi)[TS::NC][4], uint32_t (&lo)[TS::NC][4],
                                             uint32_t (&rb)[4]) {
#pragma unroll
  for (int c = 0; c < TS::NC; ++c)
#pragma unroll
    for (int p = 0; p < 4; ++p) asm volatile("" : "+v"(hi[c][p]), "+v"(lo[c][p]));
  if constexpr (TS::NR > 0) {
#pragma unroll
    for (int p = 0; p < 4; ++p) asm volatile("" : "+v"(rb[p]));
  }
  asm volatile("" ::: "memory");
}

template <class TS>
__device__ __forceinline__ void pre_mfma(const uint32_t (&hi)[TS::NC][4],
                                         const uint32_t (&lo)[TS::NC][4], const uint32_t (&rb)[4],
                                         floatx4 (&acc)[TS::N], floatx4 (&accb)[TS::NRA]) {
  split_mfma<TS>(hi, lo, acc);
  const half8v b = as_h8(rb);
#pragma unroll
  for (int c = 0; c < TS::NR; ++c) {
    accb[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_h8(hi[c]), b, accb[c], 0, 0, 0);
    accb[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_h8(lo[c]), b, accb[c], 0, 0, 0);
  }
}

// Gram tiles (acc, x 2^2ey) and rhs tiles (accb, x 2^(ey+er)) of ratings
// [pb, pe) from the split table.  d0 = this lane's first dim (m * CN); st: 128
// words of wave-private LDS staging.  Pipeline as gram_accumulate_split; the
// gathers of the step after the last one read the zero row (never consumed).
template <class TS>
__device__ __forceinline__ void gram_accumulate_pre(
    const int32_t* __restrict__ col, const float* __restrict__ val, int64_t pb, int64_t pe,
    const uint32_t* __restrict__ Ysp, uint32_t kp, int zero_row, float sr, int d0,
    floatx4 (&acc)[TS::N], floatx4 (&accb)[TS::NRA], int* __restrict__ st, float& rmax) {
  const int lane = threadIdx.x & 63, m = lane & 15;
  int* st_c = st;
  uint32_t* st_r = reinterpret_cast<uint32_t*>(st + 64);
  if (pe <= pb) return;
  const uint32_t rsel = m == 0 ? 0x05040100u : (m == 1 ? 0x07060302u : 0x0C0C0C0Cu);
  const uint32_t* base = Ysp + d0;
  auto load_idx = [&](int64_t b, int& ci, float& rv) {
    ci = zero_row;
    rv = 0.f;
    if (b + lane < pe) {
      ci = col[b + lane];
      rv = val[b + lane];
    }
  };
  auto stage = [&](int ci, float rv) {
    st_c[lane] = ci;
    st_r[lane] = split_word(sr * rv);
    rmax = fmaxf(rmax, __builtin_fabsf(rv));
    wave_lds_sync();
  };
  const int nsteps = (int)((pe - pb + 31) >> 5);
  int ci, ci_n;
  float rv, rv_n;
  load_idx(pb, ci, rv);
  load_idx(pb + 64, ci_n, rv_n);
  stage(ci, rv);
  PreStep<TS::NC> s;
  pre_issue<TS>(s, st_c, st_r, 0, base, kp);
  for (int t = 0; t < nsteps; ++t) {
    uint32_t hi[TS::NC][4], lo[TS::NC][4], rb[4];
    pre_operands<TS>(s, rsel, hi, lo, rb);
    pin_operands<TS>(hi, lo, rb);
    // step t+1 = block (t+1)>>1, half (t+1)&1; a new block is staged from the
    // pairs prefetched one block earlier
    if (t & 1) {
      stage(ci_n, rv_n);
      load_idx(pb + 64 * (int64_t)((t >> 1) + 2), ci_n, rv_n);
    }
    pre_issue<TS>(s, st_c, st_r, (t + 1) & 1, base, kp);
    pre_mfma<TS>(hi, lo, rb, acc, accb);
  }
}

// Two steps of gathers in flight (W1 explicit light rows and chunks, one wave per
// SIMD: a step's MFMAs alone do not cover an HBM gather latency).  Register sets
// s0 / s1 hold steps t+1 and t+2 while step t's operands are formed; the rating
// indices are staged in LDS one block further ahead, in two block slots.
template <class TS>
__device__ __forceinline__ void gram_accumulate_pre2(
    const int32_t* __restrict__ col, const float* __restrict__ val, int64_t pb, int64_t pe,
    const uint32_t* __restrict__ Ysp, uint32_t kp, int zero_row, float sr, int d0,
    floatx4 (&acc)[TS::N], floatx4 (&accb)[TS::NRA], int* __restrict__ st, float& rmax) {
  const int lane = threadIdx.x & 63, m = lane & 15;
  // slot b % 2: 64 column indices then 64 split rating words
  if (pe <= pb) return;
  const uint32_t rsel = m == 0 ? 0x05040100u : (m == 1 ? 0x07060302u : 0x0C0C0C0Cu);
  const uint32_t* base = Ysp + d0;
  auto load_idx = [&](int64_t b, int& ci, float& rv) {
    ci = zero_row;
    rv = 0.f;
    if (b + lane < pe) {
      ci = col[b + lane];
      rv = val[b + lane];
    }
  };
  auto stage = [&](int slot, int ci, float rv) {
    st[128 * slot + lane] = ci;
    reinterpret_cast<uint32_t*>(st + 128 * slot + 64)[lane] = split_word(sr * rv);
    rmax = fmaxf(rmax, __builtin_fabsf(rv));
    wave_lds_sync();
  };
  auto issue = [&](PreStep<TS::NC>& s, int step) {
    const int slot = (step >> 1) & 1;
    pre_issue<TS>(s, st + 128 * slot, reinterpret_cast<const uint32_t*>(st + 128 * slot + 64),
                  step & 1, base, kp);
  };
  const int nsteps = (int)((pe - pb + 31) >> 5);
  int ci0, ci1, ci_n;
  float rv0, rv1, rv_n;
  load_idx(pb, ci0, rv0);
  load_idx(pb + 64, ci1, rv1);
  load_idx(pb + 128, ci_n, rv_n);
  stage(0, ci0, rv0);
  stage(1, ci1, rv1);
  PreStep<TS::NC> s0, s1;
  issue(s0, 0);
  issue(s1, 1);
  // step t: operands from s[t % 2]; that set then loads step t + 2 (block (t >> 1) + 1);
  // after an odd step the slot of block t >> 1 (fully issued) takes block (t >> 1) + 2
  auto body = [&](PreStep<TS::NC>& s, int t) {
    uint32_t hi[TS::NC][4], lo[TS::NC][4], rb[4];
    pre_operands<TS>(s, rsel, hi, lo, rb);
    pin_operands<TS>(hi, lo, rb);
    if (t & 1) {
      stage((t >> 1) & 1, ci_n, rv_n);
      load_idx(pb + 64 * (int64_t)((t >> 1) + 3), ci_n, rv_n);
    }
    issue(s, t + 2);  // past the last step: the zero row's words (never consumed)
    pre_mfma<TS>(hi, lo, rb, acc, accb);
  };
  for (int t = 0; t < nsteps; t += 2) {
    body(s0, t);
    if (t + 1 < nsteps) body(s1, t + 1);
  }
}

// rhs from the pre path's tiles: b[i*CN + gcol(c)] = C[i][0] + C[i][1] of
// accb[c], returned in the layout of the split path's partials (lane (0, m)
// holds dim m*CN + gcol(c), lanes with q > 0 hold 0), times `scale`.
template <class TS>
__device__ __forceinline__ void rhs_from_tiles(const floatx4 (&accb)[TS::NRA], float scale,
                                               float (&bt)[TS::NRA]) {
  const int lane = threadIdx.x & 63, q = lane >> 4, m = lane & 15;
  const int src = (m >> 2) << 4;
  const int rr = m & 3;
#pragma unroll
  for (int c = 0; c < TS::NRA; ++c) {
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = __shfl(accb[c][r] + __shfl_xor(accb[c][r], 1), src);
    const float x = rr == 0 ? v[0] : (rr == 1 ? v[1] : (rr == 2 ? v[2] : v[3]));
    bt[c] = (c < TS::NR && q == 0) ? x * scale : 0.f;
  }
}

// Split table of one half-sweep's source factors (explicit only): one uint4
// (4 dims) per thread; rows of kp = 4 << kp4_shift words; row n_src is zero.
__global__ __launch_bounds__(256) void split_table_kernel(const float* __restrict__ Y,
                                                          int64_t n_src, int ld, int k,
                                                          int kp4_shift,
                                                          const float* __restrict__ scal,
                                                          uint4* __restrict__ Ysp) {
  const float sy = ldexpf(1.f, split_exponent(scal[0]));
  const int64_t total = (n_src + 1) << kp4_shift;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * 256) {
    const int64_t row = i >> kp4_shift;
    const int d = 4 * (int)(i & ((1 << kp4_shift) - 1));
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row < n_src && d + 4 <= ld) v = *reinterpret_cast<const float4*>(Y + row * ld + d);
    uint4 w;
    w.x = d + 0 < k ? split_word(sy * v.x) : 0u;
    w.y = d + 1 < k ? split_word(sy * v.y) : 0u;
    w.z = d + 2 < k ? split_word(sy * v.z) : 0u;
    w.w = d + 3 < k ? split_word(sy * v.w) : 0u;
    Ysp[i] = w;
  }
}

// Launch-1 task t -> heavy-row chunk or light row: the two lists interleaved
// while both last (memory-bound Gram-only chunks beside VALU-heavy fused
// solves), each in its own LPT order.
__device__ __forceinline__ void decode_task(int t, int n_chunks, int n_light, int& chunk,
                                            int& light) {
  const int P = n_chunks < n_light ? n_chunks : n_light;
  chunk = -1;
  light = -1;
  if (t < 2 * P) {
    if (t & 1) light = t >> 1;
    else chunk = t >> 1;
  } else if (n_chunks > P) {
    chunk = t - P;
  } else {
    light = t - P;
  }
}

// (i, j) of register r of upper tile tt for this lane (MFMA 16x16 C layout:
// row = 4q + r, col = m; dims interleaved as d = 16-index * CN + tile-index).
template <int CN>
__device__ __forceinline__ void tile_ij(int c1, int c2, int r, int& i, int& j) {
  const int lane = threadIdx.x & 63, q = lane >> 4, m = lane & 15;
  i = (4 * q + r) * CN + c1;
  j = m * CN + c2;
}

// Scatter the MFMA-layout matrix into the packed lower triangle P (type T) in LDS.
template <int CN, class T>
__device__ __forceinline__ void pack_gram(const double (&a64)[Cfg<CN>::NT][4], T* __restrict__ P) {
  int tt = 0;
#pragma unroll
  for (int c1 = 0; c1 < CN; ++c1) {
#pragma unroll
    for (int c2 = c1; c2 < CN; ++c2) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int i, j;
        tile_ij<CN>(c1, c2, r, i, j);
        const int hi = i > j ? i : j, lo = i > j ? j : i;
        P[hi * (hi + 1) / 2 + lo] = (T)a64[tt][r];
      }
      ++tt;
    }
  }
}

__device__ __forceinline__ float rcp_t(float d) { return __builtin_amdgcn_rcpf(d); }
__device__ __forceinline__ double rcp_t(double d) {
  double y = __builtin_amdgcn_rcp(d);  // v_rcp_f64 estimate + two Newton steps
  y = fma(fma(-d, y, 1.0), y, y);
  return fma(fma(-d, y, 1.0), y, y);
}
__device__ __forceinline__ float readlane_t(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
__device__ __forceinline__ double readlane_t(double v, int l) { return readlane_f64(v, l); }

// ---------------------------------------------------------------------------
// Block LDL^T on a column-per-lane panel (k <= 64, one wavefront per system).
//
// The regularised Gram arrives as fp32 16x16 tiles in the MFMA C layout
// (A[t] = tile (I, J), I <= J; block I holds dims d = 16-index * CN + I).  Any
// symmetric permutation is a valid pivot order, so A = U^T D U (U unit upper)
// is factored in that block order.  For block row K, lane t holds column t of
// the 16 x 16(NB-K) panel [B_KK | B_K,K+1 | ...] (16 registers) plus one rhs
// value (b of the dim that column stands for).  Because B_KK is symmetric, its
// columns are its rows, and the 16-pivot elimination of the diagonal block, the
// TRSM of the off-diagonal panel (W = L^-1 B) and the forward substitution of
// the rhs — including the rhs trailing update b_J -= U_KJ^T D z_K — are ONE
// instruction stream over all lanes:
//   pivot p: d = R_p[p], f_t = R_t[p] / d (= U[p][t]),
//            R_t[i] -= R_p[i] * f_t (i > p),  rb_t -= f_t * rb_p
// (R_p[i] and rb_p broadcast from lane p by v_readlane).  The trailing tiles
// B_IJ -= U_KI^T D_K U_KJ (K < I <= J) run on the matrix cores from the U
// columns in LDS.  Back substitution x_K = U_KK^-1 (z_K / D_K - sum_J U_KJ x_J)
// on 16 lanes (DPP row broadcasts).
// LDS (floats): tile slots NT x 288 (16 columns, stride 18: 8-B aligned, at
// most 2-way conflicts on the MFMA operand reads) | z, d, x 3 x 16 NB.
// ---------------------------------------------------------------------------
template <int CN>
struct PanelLds {
  static constexpr int NB = CN, NT = CN * (CN + 1) / 2, CS = 18;  // column stride
  static constexpr int T = 0, Z = NT * 16 * CS, D = Z + 16 * NB, X = D + 16 * NB,
                       SIZE = X + 16 * NB;
};

__host__ __device__ constexpr int tile_index(int nb, int i, int j) {
  // upper tiles in (c1, c2 >= c1) row order, as the Gram accumulates them
  return i * nb - i * (i - 1) / 2 + (j - i);
}

// ata[ii] += lambda (explicit, fp32 tiles); padded dims get an identity row.
template <int CN>
__device__ __forceinline__ void regularise_f32(floatx4 (&A)[Cfg<CN>::NT], float lam, int k) {
  int tt = 0;
#pragma unroll
  for (int c1 = 0; c1 < CN; ++c1) {
#pragma unroll
    for (int c2 = c1; c2 < CN; ++c2) {
      if (c1 == c2) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int i, j;
          tile_ij<CN>(c1, c2, r, i, j);
          if (i == j) A[tt][r] = (i < k) ? A[tt][r] + lam : 1.f;
        }
      }
      ++tt;
    }
  }
}

// x on lanes above P, 0 on lanes <= P.  The lane mask comes from the scalar
// unit (all-ones shifted left by P + 1), so the gate costs one VALU op.
template <int P>
__device__ __forceinline__ float gate_above(float x) {
  float r;
  uint64_t m;
  asm volatile("s_lshl_b64 %1, -1, %2\n\ts_nop 0\n\tv_cndmask_b32_e64 %0, 0, %3, %1"
               : "=v"(r), "=&s"(m)
               : "i"(P + 1), "v"(x));
  return r;
}

// Lane P of v replaced by the uniform value s (one v_writelane; the s_nop
// covers an SGPR just written by v_readlane).
template <int P>
__device__ __forceinline__ float put_lane(float v, float s) {
  asm volatile("s_nop 1\n\tv_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(s), "i"(P));
  return v;
}

// Pivot p's broadcasts from lane p: a[i] = R_p[i] for i >= p (a[p] = the pivot
// d) and bp = rb_p.  The uniform-index ds_bpermute becomes one v_readlane per
// value (measured: the LDS round trip on this serial chain is slower); all are
// issued before their FMAs, into distinct SGPRs, so no SGPR-hazard s_nop pads
// the updates, which then run two rows per v_pk_fma_f32 with an SGPR pair.
template <int N>
__device__ __forceinline__ void pivot_broadcast(const float (&R)[N], float rb, int p,
                                                float (&a)[N], float& bp) {
  const int addr = p << 2;
#pragma unroll
  for (int i = p; i < N; ++i)
    a[i] = __builtin_bit_cast(float,
                              __builtin_amdgcn_ds_bpermute(addr, __builtin_bit_cast(int, R[i])));
  bp = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(addr, __builtin_bit_cast(int, rb)));
}

// R[i] -= a[i] * f for i > p, two rows per v_pk_fma_f32 (for even p the pair
// (p, p+1) is updated too; the caller then overwrites R[p]).
template <int N>
__device__ __forceinline__ void pivot_update(float (&R)[N], const float (&a)[N], int p, float f) {
  const float2v nf = {-f, -f};
#pragma unroll
  for (int i = (p + 1) & ~1; i < N; i += 2) {
    const float2v r = __builtin_elementwise_fma((float2v){a[i], a[i + 1]}, nf,
                                                (float2v){R[i], R[i + 1]});
    R[i] = r[0];
    R[i + 1] = r[1];
  }
}

template <int P>
__device__ __forceinline__ float newbcast(float v) {  // lane P of each 16-lane row
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v),
                                                                0x150 + P, 0xF, 0xF, false));
}

// Block back substitution x_K = U_KK^-1 (z_K / D_K - sum_{J>K} U_KJ x_J) on lanes
// 0..15 (lanes 16.. mirror), K = NB-1 .. 0, from the U columns in the tile slots
// (column-major, stride CS; the U_KK columns hold 0 on and below the diagonal, so
// no masks are needed).  Runtime block loops keep the LDS address arithmetic
// out of the registers of the unrolled solve.
template <int CS>
__device__ __forceinline__ void block_back_subst(int NB, const float* __restrict__ tiles,
                                                 const float* __restrict__ Zv,
                                                 const float* __restrict__ Dv,
                                                 float* __restrict__ Xv) {
  const int lane = threadIdx.x & 63, i = lane & 15;
  for (int K = NB - 1; K >= 0; --K) {
    float v = Zv[K * 16 + i] * rcp_t(Dv[K * 16 + i]);
    for (int J = K + 1; J < NB; ++J) {
      const float* U = tiles + tile_index(NB, K, J) * 16 * CS + i;
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4) {
        const float4 xj = *reinterpret_cast<const float4*>(Xv + J * 16 + 4 * j4);
        v = fmaf(-U[(4 * j4 + 0) * CS], xj.x, v);
        v = fmaf(-U[(4 * j4 + 1) * CS], xj.y, v);
        v = fmaf(-U[(4 * j4 + 2) * CS], xj.z, v);
        v = fmaf(-U[(4 * j4 + 3) * CS], xj.w, v);
      }
    }
    const float* Ukk = tiles + tile_index(NB, K, K) * 16 * CS + i;
    float u[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) u[j] = Ukk[j * CS];
    static_for<16>([&](auto jr) {
      constexpr int j = 15 - decltype(jr)::value;
      v = fmaf(-u[j], newbcast<j>(v), v);
    });
    if (lane < 16) Xv[K * 16 + i] = v;
    wave_lds_sync();
  }
}

// x (permuted block layout Xv[K*16 + i] = dim i*CN + K) -> xrow (natural order, 0 past k
// and everywhere when !ok).
template <int CN>
__device__ __forceinline__ void panel_store_x(const float* __restrict__ Xv, int k, bool ok,
                                              float* __restrict__ xrow, int ld) {
  for (int d = threadIdx.x & 63; d < ld; d += 64) {
    const float x = d < 16 * CN ? Xv[(d % CN) * 16 + d / CN] : 0.f;
    xrow[d] = (d < k && ok) ? x : 0.f;
  }
}

// SPREAD: the pivot spread test (explicit rows; the implicit rows are checked a
// posteriori by iterative refinement instead).  STORE: write x to xrow here.
template <int CN, bool SPREAD = true, bool STORE = true>
__device__ __forceinline__ bool panel_ldl_solve(floatx4 (&A)[Cfg<CN>::NT], const float (&bq)[CN],
                                                float* __restrict__ lds, int k,
                                                float* __restrict__ xrow, int ld) {
  typedef PanelLds<CN> Lo;
  constexpr int NB = CN, CS = Lo::CS;
  const int lane = threadIdx.x & 63, q = lane >> 4, m = lane & 15;
  float* Zv = lds + Lo::Z;
  float* Dv = lds + Lo::D;
  float* Xv = lds + Lo::X;
  auto slot = [&](int I, int J) { return lds + Lo::T + tile_index(NB, I, J) * 16 * CS; };
  // rhs of this lane's panel column at K = 0: dim m*CN + (block q)
  float rb = 0.f;
#pragma unroll
  for (int c = 0; c < CN; ++c)
    if (q == c) rb = bq[c];
  bool okl = true;  // this lane: every pivot of its diagonal lane was > 0
  float pmin = 3.0e38f, pmax = 0.f;  // this lane's pivots (lanes < 16)
  static_for<NB>([&](auto Kc) {
    constexpr int K = decltype(Kc)::value;
    constexpr int NCOL = 16 * (NB - K);
    // (a) block row K: C layout -> column-major tile slots (column m, rows 4q..4q+3)
    static_for<NB - K>([&](auto jc) {
      constexpr int J = K + decltype(jc)::value;
      const floatx4 v = A[tile_index(NB, K, J)];
      float2* dst = reinterpret_cast<float2*>(slot(K, J) + m * CS + 4 * q);
      dst[0] = make_float2(v[0], v[1]);
      dst[1] = make_float2(v[2], v[3]);
    });
    wave_lds_sync();
    const bool col_ok = lane < NCOL;
    const int Jl = K + (col_ok ? q : 0);
    float* colp = slot(K, Jl) + m * CS;
    float R[16];
#pragma unroll
    for (int c2 = 0; c2 < 8; ++c2) {
      const float2 v = *reinterpret_cast<const float2*>(colp + 2 * c2);
      R[2 * c2] = v.x; R[2 * c2 + 1] = v.y;
    }
    // (b) 16 pivots over the whole panel (diag LDL^T + TRSM + rhs forward)
    float myd = 1.f;
    static_for<16>([&](auto pc) {
      constexpr int p = decltype(pc)::value;
      float a[16];
      float bp;
      pivot_broadcast<16>(R, rb, p, a, bp);
      const float d = a[p];
      const float rd = rcp_t(d);
      const float f = gate_above<p>(R[p] * rd);  // U[p][t]; 0 below the diagonal
      rb = fmaf(-f, bp, rb);
      pivot_update<16>(R, a, p, f);
      R[p] = f;
      myd = put_lane<p>(myd, d);
    });
    okl = okl && (myd > 0.f);  // lanes >= 16 keep myd = 1; NaN pivots fail
    if (lane < 16 && lane * CN + K < k) {  // pivots of real dims
      pmin = fminf(pmin, myd);
      pmax = fmaxf(pmax, myd);
    }
    // (c) U columns -> tile slots (block row K); z_K, D_K
    if (col_ok) {
#pragma unroll
      for (int c2 = 0; c2 < 8; ++c2)
        *reinterpret_cast<float2*>(colp + 2 * c2) = make_float2(R[2 * c2], R[2 * c2 + 1]);
    }
    if (lane < 16) {
      Zv[K * 16 + lane] = rb;
      Dv[K * 16 + lane] = myd;
    }
    if constexpr (K + 1 < NB) {
      rb = __shfl(rb, (lane + 16) & 63);  // next block row's rhs: columns shift by 16
      wave_lds_sync();
      // (d) trailing update B_IJ -= (D_K U_KI)^T U_KJ on the matrix cores
      float dq[4];
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) dq[s4] = -Dv[K * 16 + 4 * s4 + q];
      static_for<NB - 1 - K>([&](auto ic) {
        constexpr int I = K + 1 + decltype(ic)::value;
        float ua[4];
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) ua[s4] = dq[s4] * slot(K, I)[m * CS + 4 * s4 + q];
        static_for<NB - I>([&](auto jc) {
          constexpr int J = I + decltype(jc)::value;
          floatx4 acc = A[tile_index(NB, I, J)];
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4)
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ua[s4], slot(K, J)[m * CS + 4 * s4 + q],
                                                        acc, 0, 0, 0);
          A[tile_index(NB, I, J)] = acc;
        });
      });
    }
  });
  wave_lds_sync();
  // pivot spread (lower bound on cond(A)) within what fp32 holds to the 1e-4 bar
  for (int o = 32; o > 0; o >>= 1) {
    pmin = fminf(pmin, __shfl_xor(pmin, o));
    pmax = fmaxf(pmax, __shfl_xor(pmax, o));
  }
  const bool ok = __ballot(!okl) == 0 && (!SPREAD || pmax <= kCondMax * pmin);
  // (e) back substitution
  block_back_subst<CS>(NB, lds + Lo::T, Zv, Dv, Xv);
  // (f) un-permute: dim d = i*CN + K  <->  Xv[K*16 + i]
  if constexpr (STORE) panel_store_x<CN>(Xv, k, ok, xrow, ld);
  return ok;
}

// Forward substitution U^T z = r for a new right-hand side (U unit upper from the
// panel factorisation: tile slot (J, K) column i holds U_JK[p][i], p = 0..15, and the
// diagonal tiles hold 0 on and below the diagonal), block row by block row on lanes
// 0..15 (lanes 16.. mirror).  Rv, Zv in the permuted block layout.
template <int CS>
__device__ __forceinline__ void block_fwd_subst(int NB, const float* __restrict__ tiles,
                                                const float* __restrict__ Rv,
                                                float* __restrict__ Zv) {
  const int lane = threadIdx.x & 63, i = lane & 15;
  for (int K = 0; K < NB; ++K) {
    float v = Rv[K * 16 + i];
    for (int J = 0; J < K; ++J) {  // v -= U_JK^T z_J: column i of tile (J, K)
      const float* U = tiles + tile_index(NB, J, K) * 16 * CS + i * CS;
#pragma unroll
      for (int p4 = 0; p4 < 4; ++p4) {
        const float4 zj = *reinterpret_cast<const float4*>(Zv + J * 16 + 4 * p4);
        v = fmaf(-U[4 * p4 + 0], zj.x, v);
        v = fmaf(-U[4 * p4 + 1], zj.y, v);
        v = fmaf(-U[4 * p4 + 2], zj.z, v);
        v = fmaf(-U[4 * p4 + 3], zj.w, v);
      }
    }
    const float* Ukk = tiles + tile_index(NB, K, K) * 16 * CS + i * CS;
    float u[16];
#pragma unroll
    for (int p = 0; p < 16; ++p) u[p] = Ukk[p];  // U_KK[p][i]: 0 for p >= i
    static_for<16>([&](auto pc) {  // z_i = v_i - sum_{p < i} U_KK[p][i] z_p
      constexpr int p = decltype(pc)::value;
      v = fmaf(-u[p], newbcast<p>(v), v);
    });
    if (lane < 16) Zv[K * 16 + i] = v;
    wave_lds_sync();
  }
}


// ---------------------------------------------------------------------------
// k in (64, 128]: ONE wavefront per system ("W1"), block Gaussian elimination
// with explicit inverses of the 16 x 16 diagonal blocks (NB = 8 block rows).
//
// The Gram's 36 upper tiles stay in the MFMA C layout (lane (q, m): rows
// 4q..4q+3 of column m).  For two tiles X, Y in that layout, the products
//   C += X^T Y  =  sum_s4 mfma_16x16x4_f32(X.reg[s4], Y.reg[s4])
// need no data movement (the MFMA's k index is permuted to 4q + s4), so the
// whole right-looking elimination runs on registers:
//   for K = 0..7:
//     Gm   = -(B_KK)^-1            sweep operator on the diagonal block (VALU,
//                                  column per lane, lane-p broadcasts by DPP)
//     Pm_J = Gm B_KJ   (J > K)     = -B_KK^-1 B_KJ, on the matrix cores
//     B_IJ += B_KI^T Pm_J (K < I <= J)   Schur complement, matrix cores
//     b_J  += Pm_J^T b_K,  z_K = -Gm b_K
//     tile (K, J) <- Pm_J           (kept for the back substitution)
//   x_K = z_K + sum_{J>K} Pm_KJ x_J,  K = 7..0.
// The sweep's pivots are the LDL^T pivots of B (all must be > 0: Spark's dppsv
// fails otherwise).  Same solution as Spark's Cholesky dppsv, fp32 arithmetic
// with exact-product fp32 MFMA; no barrier, no LDS beyond one 16 x 16
// transposition buffer per wave.
// rhs layouts: "column" = lane m (any q) holds element m of a 16-block;
// "row" = lanes of row-group q hold elements 4q..4q+3.
// ---------------------------------------------------------------------------
template <int NB>
struct W1LdsT {
  static constexpr int CS = 20;                     // floats per column (16 + pad, 16-B aligned)
  // transposition buffer | rhs vector | Pm tiles of the back substitution (NB(NB-1)/2 x 256)
  static constexpr int COL = 0, VEC = 16 * CS, PM = VEC + 16,
                       SIZE = PM + NB * (NB - 1) / 2 * 256;
};

constexpr int kW1NB = 8;
using W1Lds = W1LdsT<kW1NB>;

template <int NB>
__host__ __device__ constexpr int w1_tile(int i, int j) { return tile_index(NB, i, j); }

// v on lanes with (lane & 15) == P, else w (mask from the scalar unit).
template <int P>
__device__ __forceinline__ float sel_lane16(float v, float w) {
  float r;
  const uint64_t msk = 0x0001000100010001ull << P;
  asm volatile("v_cndmask_b32_e64 %0, %2, %1, %3" : "=v"(r) : "v"(v), "v"(w), "s"(msk));
  return r;
}

// Sum over the four 16-lane row groups (every lane gets the total): two VALU
// row swaps (v_permlane16_swap: rows 0<->1, 2<->3; v_permlane32_swap: rows
// {0,1}<->{2,3}), no LDS crossbar on the dependency chain.
// (Inline asm: this compiler's __builtin_amdgcn_permlane*_swap loses the second
// result when both are consumed — measured, it emitted v_add v1, v1, v1.)
__device__ __forceinline__ float reduce_rows4(float v) {
  float a = v, b = v;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a), "+v"(b));
  float c = a + b, d = c;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1" : "+v"(c), "+v"(d));
  return c + d;
}

// Sum over the 16 lanes of each row group (every lane of the group gets it).
// Lane P of each 16-lane row, as a DPP source the combiner folds into the user
// (bound_ctrl set, old undefined: v_fmac_f32_dpp / v_rcp_f32_dpp row_newbcast:P).
template <int P>
__device__ __forceinline__ float bcast16(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x150 + P,
                                                            0xF, 0xF, true));
}

// r += (lane P's r, same 16-lane row) * nf: one v_fmac_f32_dpp row_newbcast:P.
template <int P>
__device__ __forceinline__ void fmac_bcast16(float& r, float nf) {
  asm volatile("v_fmac_f32_dpp %0, %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf"
               : "+v"(r)
               : "v"(nf), "i"(P));
}

template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL,
                                                               0xF, 0xF, false));
}

__device__ __forceinline__ float reduce_lanes16(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);  // row_half_mirror
  v += dpp_f<0x140>(v);  // row_mirror
  return v;
}

// Sweep operator over all 16 pivots of a symmetric 16 x 16 block held column per
// lane (R[i] = B[i][m], replicated in the four row groups): R <- -(B^-1) column m.
// Pivot p: d = B[p][p]; B[i][j] -= B[i][p] B[p][j] / d; row/column p scaled by
// 1/d; B[p][p] = -1/d.  The pivot column's 1/d scaling is DEFERRED: lane p keeps
// its column unscaled (multiplier 0 at its own pivot) and every column is scaled
// by 1/(its pivot) once at the end.  The stored values then follow the generic
// update for every lane (the multiplier -B[p][m]/d does not depend on a column's
// pending scale), and no lane ever forms 1 - 1/d (which cancels for large d).
// Returns the smallest pivot (> 0 for an SPD block; NaN propagates as "not > 0").
// hook(p) runs after pivot p: the caller interleaves independent matrix-core work
// there (the asm statements fix the instruction order).
template <class Hook>
__device__ __forceinline__ float sweep16(float (&R)[16], Hook&& hook, float& dself_out) {
  float dmin = 3.0e38f;  // NaN pivots are not seen here: they make the solution NaN
  float dself = 1.f;     // this lane's own pivot (its column's deferred scale is 1/dself)
  // pivot p's broadcast pivot, reciprocal and multipliers; for p > 0 they are formed
  // inside pivot p-1, right after row p's update, so their latency (DPP, v_rcp)
  // hides behind that pivot's remaining row updates
  float d = bcast16<0>(R[0]);
  float rd = rcp_t(d);
  float f = R[0] * rd;
  float nf = sel_lane16<0>(0.f, -f);
  static_for<16>([&](auto pc) {
    constexpr int p = decltype(pc)::value;
    dmin = fminf(dmin, d);
    // R[i] += (lane p's R[i]) * nf as ONE v_fmac_f32_dpp per row (the compiler only
    // folds DPP into untied VOP2 ops); s_nop 1 covers the VALU-write -> DPP-read
    // hazard of the previous pivot's last writes.
    asm volatile("s_nop 1" ::: "memory");
    float dn = 0.f, rdn = 0.f, fn = 0.f, nfn = 0.f;
    auto row = [&](auto ic) {
      constexpr int i = decltype(ic)::value;
      if constexpr (i != p) fmac_bcast16<p>(R[i], nf);
      if constexpr (i == p + 1) {  // row p+1 is final for pivot p+1: start it now
        asm volatile("s_nop 1" ::: "memory");
        dn = bcast16<p + 1>(R[p + 1]);
        rdn = rcp_t(dn);
        fn = R[p + 1] * rdn;
        nfn = sel_lane16<p + 1>(0.f, -fn);
      }
    };
    // row p+1 first, then the others
    if constexpr (p + 1 < 16) row(std::integral_constant<int, p + 1>{});
    static_for<16>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      if constexpr (i != p + 1) row(ic);
    });
    R[p] = sel_lane16<p>(-1.f, f);
    dself = sel_lane16<p>(d, dself);
    hook(pc);
    d = dn; rd = rdn; f = fn; nf = nfn;
  });
  const float s = rcp_t(dself);
#pragma unroll
  for (int i = 0; i < 16; ++i) R[i] *= s;
  dself_out = dself;
  return dmin;
}

// x of row group G broadcast to all four row groups: one ds_bpermute (the LDS
// crossbar, not the VALU).  The sweep is bound by VALU issue, not by its pivot chain's
// latency (three waves per SIMD hide it): two v_permlane*_swap plus their operand
// copies (five VALU instructions per pivot) measured 0.06 ms slower on the configs[1]
// user launch (A/B round 5, profiles/r05/ab_sweep_lean.jsonl).
template <int G>
__device__ __forceinline__ float rowgroup_bcast(float x) {
  const int src = (16 * G + (threadIdx.x & 15)) << 2;
  return __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src, __builtin_bit_cast(int, x)));
}

// v on lanes with (lane & 15) == P, else -w.
template <int P>
__device__ __forceinline__ float sel_lane16_n(float v, float w) {
  float r;
  const uint64_t msk = 0x0001000100010001ull << P;
  asm volatile("v_cndmask_b32_e64 %0, -%2, %1, %3" : "=v"(r) : "v"(v), "v"(w), "s"(msk));
  return r;
}

// v on the lanes of 64-bit mask M (a constant), else w.
template <uint64_t M>
__device__ __forceinline__ float sel_mask(float v, float w) {
  float r;
  asm volatile("v_cndmask_b32_e64 %0, %2, %1, %3" : "=v"(r) : "v"(v), "v"(w), "s"(M));
  return r;
}

// The sweep of sweep16 on a symmetric 16 x 16 block held in the MFMA C layout (lane
// (q, m): B[4q + r][m], r = 0..3) instead of column per lane: per pivot p, row p is
// broadcast from row group p/4 to all four (rowgroup_bcast), and a lane's four column-p
// entries come from lane p of its own row group (v_fmac_f32_dpp row_newbcast:p), so a
// lane updates its four entries, not sixteen replicated ones, and the block never goes
// through LDS (the result is already in the C layout the Pm / Schur MFMAs read).  Every
// entry sees the same fp32 operations, in the same order, as in sweep16 (deferred
// pivot-column scaling, look-ahead of the next pivot).  Per pivot the VALU issues the
// four row updates, the pivot broadcast, its reciprocal, one multiply and the selects
// (the multiplier's negation rides in a select's source modifier); positivity of the
// pivots is checked by the caller from the spread test's minimum (dself_out), so the
// returned minimum is not tracked here (+inf).  A 2 x 2-pivot form (8 sequential steps
// instead of 16) measured slower: the same updates plus a 2 x 2 inverse per pair, and
// the sweep is issue-bound, not chain-bound (A/B round 5, profiles/r05/ab_pair_pivots.jsonl)
// — at two or more waves per SIMD.  LA (the one-wave-per-SIMD W1 kernels, NB = 8): the
// next pivot row's broadcast is issued one pivot earlier, before the current pivot's
// update, and brought up to date on the copy by one more DPP fmac (the same fp32
// operation as on its register, so the results are bit-identical): the ds_bpermute
// latency leaves the pivot chain for one VALU more per pivot.  A/B round 5
// (profiles/r05/ab_lookahead.jsonl): configs[3] W1 user rows 96.6 -> 95.2 ms, 271.9 ->
// 270.1 ms/iter; slower where other waves hide the chain (k <= 64: user launch +0.7 %,
// dual rows +2.5 %).  Round 6: two rows ahead (row p+2's copy is brought up to date after
// the pivot's row updates, so each ds_bpermute has a whole pivot to land; one DPP fmac
// more per pivot, still bit-identical): W1 user rows 94.9 -> 93.0 ms, 273.4 -> 271.0
// ms/iter at 4096-rating tasks (profiles/r06/ab_lookahead2.jsonl).
template <bool LA = false, class Hook>
__device__ __forceinline__ float sweep16c(floatx4& Bv, Hook&& hook, float& dself_out) {
  // Bv was just written by the matrix cores (the pivot block's Schur update) and is
  // read below by inline DPP asm, which the hazard recognizer does not see: the XDL
  // write -> VALU read wait states by hand (tests/test_isa_hazards.py checks the rest)
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  float B[4] = {Bv[0], Bv[1], Bv[2], Bv[3]};
  float dmin = 3.0e38f;
  float dself = 1.f;
  float rowp = rowgroup_bcast<0>(B[0]);
  float pre = 0.f;   // LA: the next pivot row's broadcast copy
  float pre2 = 0.f;  // LA: the one after it (its ds_bpermute has a whole pivot to land)
  if constexpr (LA) {
    pre = rowgroup_bcast<0>(B[1]);   // row 1 before pivot 0
    pre2 = rowgroup_bcast<0>(B[2]);  // row 2 before pivot 0
  }
  float d = bcast16<0>(rowp);
  float rd = rcp_t(d);
  float f = rowp * rd;
  float nf = sel_lane16_n<0>(0.f, f);
  static_for<16>([&](auto pc) {
    constexpr int p = decltype(pc)::value;
    constexpr int qp = p >> 2, rp = p & 3, rn = (p + 1) & 3;
    asm volatile("s_nop 1" ::: "memory");
    float dn = 0.f, rdn = 0.f, fn = 0.f, nfn = 0.f;
    if constexpr (LA) {
      if constexpr (p + 1 < 16) {  // row p+1 after pivot p, on its broadcast copy
        fmac_bcast16<p>(pre, nf);
        dn = bcast16<p + 1>(pre);
        rdn = rcp_t(dn);
        fn = pre * rdn;
        nfn = sel_lane16_n<p + 1>(0.f, fn);
      }
      static_for<4>([&](auto rc) { fmac_bcast16<p>(B[decltype(rc)::value], nf); });
      // row p+2's copy (broadcast two pivots ago) after pivot p, after this pivot's row
      // updates so its ds_bpermute has had them to land; row p+3's broadcast (after
      // pivots <= p) is issued now and consumed two pivots on
      if constexpr (p + 2 < 16) fmac_bcast16<p>(pre2, nf);
      if constexpr (p + 3 < 16) {
        constexpr int q3 = (p + 3) / 4, r3 = (p + 3) % 4;
        pre = pre2;
        pre2 = rowgroup_bcast<q3>(B[r3]);
      } else {
        pre = pre2;
      }
    } else {
      // the register holding row p+1 first: then pivot p+1's row is final
      fmac_bcast16<p>(B[rn], nf);
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
      });
    }
    // row p (row group qp): f off the pivot, -1 on it (scaled by 1/d at the end)
    B[rp] = sel_mask<0xFFFFull << (16 * qp)>(sel_lane16<p>(-1.f, f), B[rp]);
    dself = sel_lane16<p>(d, dself);
    hook(pc);
    d = dn; rd = rdn; f = fn; nf = nfn;
  });
  const float s = rcp_t(dself);
#pragma unroll
  for (int r = 0; r < 4; ++r) Bv[r] = B[r] * s;
  dself_out = dself;
  return dmin;
}

// Schur tiles of step K, I-major: u = 0 is (K+1, K+1), the next pivot block.
template <int NB>
__host__ __device__ constexpr int schur_n(int K) { return (NB - 1 - K) * (NB - K) / 2; }
template <int NB>
__host__ __device__ constexpr int schur_I(int K, int u) {
  int I = K + 1;
  while (u >= NB - I) { u -= NB - I; ++I; }
  return I;
}
template <int NB>
__host__ __device__ constexpr int schur_J(int K, int u) {
  int I = K + 1;
  while (u >= NB - I) { u -= NB - I; ++I; }
  return I + u;
}

// Schur complement and Pm products of the W1 elimination.  Both operands of
// C += X^T Y are 16 x 16 tiles in the C layout, so each product is a handful of
// MFMAs with no data movement: on v_mfma_f32_16x16x32_f16 lane (q, m) supplies
// k = 8q..8q+7, i.e. its four C-layout values twice (hi and lo halves).
// Split f16 (default): the operands are scaled by powers of two and split into
// f16 hi + lo; [Xh|Xl]^T [Yh|Yh] + [Xh|Xl]^T [Yl|Yl] = (Xh + Xl)^T (Yh + Yl) is
// two MFMAs (32 cycles; the fp32 form, four v_mfma_f32_16x16x4_f32, takes 128).
// For the Schur update the two scales cancel (X 2^a, Pm 2^-a, a balancing the
// two maxima), so the MFMAs accumulate straight into the fp32 tile: no VALU
// touches the 36 system tiles during the elimination.  The system is first
// scaled by a power of two (largest diagonal entry -> [2^13, 2^14)), which bounds
// every Schur complement entry and keeps the scaled operands inside the f16
// range; pieces are exact to ~2^-22 relative, and entries far below their tile's
// maximum lose precision only below the fp32 rounding floor of the elimination.
// Where it is used (measured, ML-25M shape): the implicit rank-128 light-row
// kernel (configs[2] 11.0 -> 9.4 ms/iter) and the heavy-row solve.  Not for
// NB = 4 (rank 33-64: 10 Schur tiles per system, too few to pay for the scaling
// and splitting) and not in the explicit rank-128 light-row kernel, whose
// pre-split Gram leaves no registers for the split operands (it spills; 7.8 ->
// 8.1 ms/iter measured).
template <int NB>
constexpr bool kW1SplitSchur = NB == 8;
// Diagonal blocks swept in the MFMA C layout (sweep16c: 4 entries per lane instead of
// 16 replicated) in every elimination but the split-Schur one.  With the row-group
// pivot broadcast as one ds_bpermute (round 5) it pays in the NB = 8 fp32 kernels too,
// which round 4 (two permlane swaps per pivot) had measured slower: A/B round 5,
// `profiles/r05/ab_sweepc_nb.jsonl`, configs[3] 287.4 -> 280.1 ms/iter (explicit
// rank-128 user launch 101.5 -> 96.3 ms, dual systems 65.6 -> 64.7 ms), configs[1]
// 2.043 -> 2.032.  In the split-Schur form (implicit rank-128 light rows, heavy-row
// solves) it is slower: configs[2] 9.32 -> 10.99 ms/iter (user launch 5.48 -> 6.66), and
// still with the pivot lookahead of the W1 sweep: 9.12 -> 10.75 (ab_sweepc_split_lookahead.jsonl).
template <int NB, bool SPLIT>
constexpr bool kSweepC = !SPLIT;
// Measured round 4 (A/B at configs[1] / configs[3]): the split form in the explicit
// k <= 64 solve (2.33 vs 2.26 ms/iter), the explicit rank-128 light rows (user launch
// 112 vs 102 ms) and the n x n dual systems (76 vs 70 ms) is slower: fp32 stays there.

// fp32 form: acc += X^T Y (the MFMA's k index is permuted to 4q + s4).
__device__ __forceinline__ floatx4 tile_xty(const floatx4& X, const floatx4& Y, floatx4 acc) {
#pragma unroll
  for (int s4 = 0; s4 < 4; ++s4) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(X[s4], Y[s4], acc, 0, 0, 0);
  return acc;
}

// Largest value over the wave (every lane gets it; v >= 0, NaN ignored).
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));   // quad_perm [1,0,3,2]
  v = fmaxf(v, dpp_f<0x4E>(v));   // quad_perm [2,3,0,1]
  v = fmaxf(v, dpp_f<0x141>(v));  // row_half_mirror
  v = fmaxf(v, dpp_f<0x140>(v));  // row_mirror
  float a = v, b = v;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a), "+v"(b));
  float c = fmaxf(a, b), d = c;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1" : "+v"(c), "+v"(d));
  return fmaxf(c, d);
}

__device__ __forceinline__ float absmax4(const floatx4& x) {
  return fmaxf(fmaxf(__builtin_fabsf(x[0]), __builtin_fabsf(x[1])),
               fmaxf(__builtin_fabsf(x[2]), __builtin_fabsf(x[3])));
}

// ---------------------------------------------------------------------------
// Split window guard.  The explicit Gram and rhs use ONE power-of-two scale per
// launch (max |Y_src| -> [2^14, 2^15), max |rating| likewise), so the f16 lo half
// of an operand t goes subnormal once |t| < 2^-3 and its relative precision then
// degrades towards 2^-24 / |t|.  A row whose own operands all sit that far below
// the launch maxima (a user-supplied U0, a loaded model, ratings spanning many
// decades) would silently lose precision.  Each explicit task therefore checks
// its scaled operands against a window T = 2^-4 (precision of its largest
// operand >= 2^-20, 16x inside the fp32-grade split):
//   max diag(G) < n T^2  (covers every row whose largest |t| < T: diag <= n max t^2)
//   or 0 < max |r| < T   (the row's ratings, scaled by the launch's rating scale).
// A row that misses the window is not solved here: it is appended to the rescue
// list and re-solved in fp64 by rescue64_kernel (as are rows whose fp32 LDL^T pivots
// spread beyond kCondMax, or fail).  Implicit rows need no window test: their A
// includes YtY (>= the largest row's square) and b is fp32.
// ---------------------------------------------------------------------------
constexpr float kWindowT = 0.0625f;  // 2^-4, in scaled units (launch max in [2^14, 2^15))

// Largest diagonal entry of an upper-tile set in the MFMA C layout (this lane's).
// (Lane (q, m) holds a diagonal entry of each diagonal tile iff r = m - 4q is in [0, 4):
// one select per tile, not a compare-and-select per (tile, r) — 4 CN + 1 VALU instead
// of ~4 x 4 CN.)
template <int CN>
__device__ __forceinline__ float diag_max_lane(const floatx4 (&A)[CN * (CN + 1) / 2]) {
  const int lane = threadIdx.x & 63, q = lane >> 4, m = lane & 15;
  const int r = m - 4 * q;
  float d = 0.f;
#pragma unroll
  for (int c = 0; c < CN; ++c) {
    const floatx4& t = A[tile_index(CN, c, c)];
    d = fmaxf(d, r == 0 ? t[0] : (r == 1 ? t[1] : (r == 2 ? t[2] : t[3])));
  }
  return (r >= 0 && r < 4) ? d : 0.f;
}

// Sum of the diagonal entries of real dims (dims < k) of an upper-tile set in the C
// layout, summed over the wave (every lane gets it).
template <int CN>
__device__ __forceinline__ float diag_trace(const floatx4 (&A)[CN * (CN + 1) / 2], int k) {
  const int lane = threadIdx.x & 63, q = lane >> 4, m = lane & 15;
  float t = 0.f;
#pragma unroll
  for (int c = 0; c < CN; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (4 * q + r == m && m * CN + c < k) t += A[tile_index(CN, c, c)][r];
  for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
  return t;
}

// Very short explicit rows on the primal path (n <= k / 4 ratings; at k > 32 such rows
// take the dual path unless it is off): A = G + lambda n I with G of rank n << k has
// lambda_min = lambda n and lambda_max ~ tr(G) + lambda n, so cond(A) ~ 1 + tr(G) /
// (lambda n), which the LDL^T pivots do not show (they stay within (tr(G) / k + lambda
// n) / (lambda n)).  The fp32 solve's error there grows as that bound (measured ~1.5e-6
// x tr(G) / (lambda n) at n <= 16, k 65-128, lambda 1e-3 / 1e-4; at n > k / 4 the
// measured errors stay ~1e-5 and below, e.g. 8.8e-7 on the configs[3] users of 97-255
// ratings).  Beyond kCondRankDef the row is re-solved in fp64.  tr_scaled: tr(G) in the
// Gram's scale (x 1/inv2).
constexpr float kCondRankDef = 64.f;
template <int CN>
__device__ __forceinline__ bool rank_deficient_illcond(const floatx4 (&acc)[CN * (CN + 1) / 2],
                                                       float inv2, int64_t n, int k, float reg) {
  if (4 * n > (int64_t)k) return false;  // uniform: the trace only for very short rows
  return diag_trace<CN>(acc, k) * inv2 > (kCondRankDef - 1.f) * reg * (float)n;
}

// Wave-uniform: do the scaled operands of a task with n terms miss the window?
// (max over lanes < x <=> no lane at or above x: ballots, no reduction)
__device__ __forceinline__ bool window_miss(float diag_lane, float n_terms, float rmax_lane) {
  const bool dmiss = __ballot(diag_lane >= n_terms * (kWindowT * kWindowT)) == 0 &&
                     __ballot(diag_lane > 0.f) != 0;
  const bool rmiss = __ballot(rmax_lane >= kWindowT) == 0 && __ballot(rmax_lane > 0.f) != 0;
  return dmiss || rmiss;
}

// The rescue list of one als_solve_half call: count word (scale word 2), the list
// (cap = the call's rows) in the workspace.
struct RescueList {
  unsigned* cnt;
  int32_t* list;
  unsigned cap;
};

// Append `row` to the rescue list (one lane).  Each row is appended at most once per
// LAUNCH1..RESCUE sequence; a caller that runs the launches twice without the RESCUE
// phase between them overflows the count, which is never written past `cap`:
// rescue64_kernel walks min(count, cap) entries and reports the overflow (status -1).
__device__ __forceinline__ void rescue_append(const RescueList& rl, int row) {
  if ((threadIdx.x & 63) == 0) {
    const unsigned i = atomicAdd(rl.cnt, 1u);
    if (i < rl.cap) rl.list[i] = row;
  }
}

// [hi | lo] f16 halves of s * x (s a power of two): hi = f16(s x) and
// lo = f16(s x - hi), each one v_fma_mix (the fp32 fma inside is exact).
__device__ __forceinline__ half8v split_hl(const floatx4& x, float s) {
  uint32_t h01, h23, l01, l23;
  asm("v_fma_mixlo_f16 %0, %1, %2, 0 op_sel_hi:[0,0,0]" : "=v"(h01) : "v"(x[0]), "v"(s));
  asm("v_fma_mixhi_f16 %0, %1, %2, 0 op_sel_hi:[0,0,0]" : "+v"(h01) : "v"(x[1]), "v"(s));
  asm("v_fma_mixlo_f16 %0, %1, %2, 0 op_sel_hi:[0,0,0]" : "=v"(h23) : "v"(x[2]), "v"(s));
  asm("v_fma_mixhi_f16 %0, %1, %2, 0 op_sel_hi:[0,0,0]" : "+v"(h23) : "v"(x[3]), "v"(s));
  asm("v_fma_mixlo_f16 %0, %1, %2, -%3 op_sel:[0,0,0] op_sel_hi:[0,0,1]"
      : "=v"(l01) : "v"(x[0]), "v"(s), "v"(h01));
  asm("v_fma_mixhi_f16 %0, %1, %2, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "+v"(l01) : "v"(x[1]), "v"(s), "v"(h01));
  asm("v_fma_mixlo_f16 %0, %1, %2, -%3 op_sel:[0,0,0] op_sel_hi:[0,0,1]"
      : "=v"(l23) : "v"(x[2]), "v"(s), "v"(h23));
  asm("v_fma_mixhi_f16 %0, %1, %2, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "+v"(l23) : "v"(x[3]), "v"(s), "v"(h23));
  return __builtin_bit_cast(half8v, make_uint4(h01, h23, l01, l23));
}
__device__ __forceinline__ half8v dup_hi(const half8v& v) {
  return __builtin_shufflevector(v, v, 0, 1, 2, 3, 0, 1, 2, 3);
}
__device__ __forceinline__ half8v dup_lo(const half8v& v) {
  return __builtin_shufflevector(v, v, 4, 5, 6, 7, 4, 5, 6, 7);
}

// NB = 8 (rank 65-128, W1 kernels), 4 (rank 33-64, explicit gram_solve_kernel) or
// 2 / 4 (the n x n dual systems of short rows, gram_solve_dual_kernel).  Returns
// whether every pivot was positive and the solution finite; xcol[c] on lane (q, m)
// = solution entry of variable (block c, index m), every row group q.
template <int NB, bool SPLIT = kW1SplitSchur<NB>>
__device__ __forceinline__ bool w1_solve_x(floatx4 (&A)[NB * (NB + 1) / 2], float (&bcol)[NB],
                                           float* __restrict__ lds, int k, float (&xcol)[NB],
                                           float cond_max = kCondMax) {
  using L = W1LdsT<NB>;
  constexpr int CS = L::CS;
  const int lane = threadIdx.x & 63, q = lane >> 4, m = lane & 15;
  float* col = lds + L::COL;
  float* vec = lds + L::VEC;
  float zcol[NB];
  float dmin = 3.0e38f;
  // this lane's pivots of real dims (its column m of every block: dim m * NB + K < k)
  float rmin = 3.0e38f, rmax = 0.f;
  auto track_pivot = [&](float ds, bool real) {
    rmin = real ? fminf(rmin, ds) : rmin;
    rmax = real ? fmaxf(rmax, ds) : rmax;
  };
  if constexpr (SPLIT) {
    // scale the system by 2^g: largest diagonal entry (= largest entry) -> [2^13, 2^14)
    float dm = 0.f;
    static_for<NB>([&](auto cc) { dm = fmaxf(dm, absmax4(A[w1_tile<NB>(cc, cc)])); });
    const float sg = ldexpf(1.f, split_exponent(wave_max(dm)) - 1);
#pragma unroll
    for (int t = 0; t < NB * (NB + 1) / 2; ++t) A[t] *= sg;
#pragma unroll
    for (int c = 0; c < NB; ++c) bcol[c] *= sg;
    if (k < NB * 16) {
      // padded dims' identity rows -> 2^13 I: a unit pivot far below the scaled
      // system would put -1/pivot at the top of Gm's range and flush its real
      // entries out of the split (x_pad stays 0: b_pad = 0, no coupling)
      static_for<NB>([&](auto cc) {
        constexpr int c = decltype(cc)::value;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (4 * q + r == m && m * NB + c >= k) A[w1_tile<NB>(c, c)][r] = 8192.f;
      });
    }
  }
  // bcol[J] for J > 0 holds per-row-group partial sums (summed over the groups when
  // block J becomes the pivot block): start with the full b_J in row group 0
#pragma unroll
  for (int c = 1; c < NB; ++c) bcol[c] = q == 0 ? bcol[c] : 0.f;
  // Sweep block K from its tile (C layout -> column per lane through LDS), running
  // `hook` between pivots; then Gm_K (C layout) and b_K (row layout).
  floatx4 Gm, bk;
  auto pivot_block = [&](auto Kc, auto&& hook) {
    constexpr int K = decltype(Kc)::value;
    if constexpr (kSweepC<NB, SPLIT>) {
      // swept in the C layout: Gm comes out where the MFMAs read it
      Gm = A[w1_tile<NB>(K, K)];
      float ds;
      dmin = fminf(dmin, sweep16c<NB == 8>(Gm, hook, ds));
      track_pivot(ds, m * NB + K < k);
      const float bK = K == 0 ? bcol[0] : reduce_rows4(bcol[K]);  // partials -> b_K[m]
      if (q == 0) vec[m] = bK;
      wave_lds_order();
      bk = *reinterpret_cast<const floatx4*>(vec + 4 * q);  // row layout
      wave_lds_order();
      return;
    }
    *reinterpret_cast<floatx4*>(col + m * CS + 4 * q) = A[w1_tile<NB>(K, K)];
    wave_lds_order();
    float R[16];
#pragma unroll
    for (int c4 = 0; c4 < 4; ++c4) {
      const floatx4 v = *reinterpret_cast<const floatx4*>(col + m * CS + 4 * c4);
      R[4 * c4] = v[0]; R[4 * c4 + 1] = v[1]; R[4 * c4 + 2] = v[2]; R[4 * c4 + 3] = v[3];
    }
    float ds;
    dmin = fminf(dmin, sweep16(R, hook, ds));
    track_pivot(ds, m * NB + K < k);
    wave_lds_order();
    const float bK = K == 0 ? bcol[0] : reduce_rows4(bcol[K]);  // partials -> b_K[m]
    if (q == 0) {
#pragma unroll
      for (int c4 = 0; c4 < 4; ++c4)
        *reinterpret_cast<floatx4*>(col + m * CS + 4 * c4) =
            floatx4{R[4 * c4], R[4 * c4 + 1], R[4 * c4 + 2], R[4 * c4 + 3]};
      vec[m] = bK;
    }
    wave_lds_order();
    Gm = *reinterpret_cast<const floatx4*>(col + m * CS + 4 * q);  // C layout
    bk = *reinterpret_cast<const floatx4*>(vec + 4 * q);           // row layout
    wave_lds_order();
  };
  // step-K operands of the split form: block row K ([hi|lo] of sK A_KJ), Pm halves
  half8v XK[NB], Ph[NB], Pl[NB];
  auto schur = [&](auto Kc, auto uc, const floatx4 (&Pm)[NB]) {
    constexpr int K = decltype(Kc)::value, u = decltype(uc)::value;
    constexpr int I = schur_I<NB>(K, u), J = schur_J<NB>(K, u);
    floatx4& C = A[w1_tile<NB>(I, J)];
    if constexpr (SPLIT) {
      // C += (2^a X)^T (2^-a Pm): lo halves of Pm first, then the hi halves
      C = __builtin_amdgcn_mfma_f32_16x16x32_f16(XK[I - K - 1], Pl[J - K - 1], C, 0, 0, 0);
      C = __builtin_amdgcn_mfma_f32_16x16x32_f16(XK[I - K - 1], Ph[J - K - 1], C, 0, 0, 0);
    } else {
      C = tile_xty(A[w1_tile<NB>(K, I)], Pm[J - K - 1], C);
    }
  };
  pivot_block(std::integral_constant<int, 0>{}, [](auto) {});
  static_for<NB>([&](auto Kc) {
    constexpr int K = decltype(Kc)::value;
    // z_K = -Gm b_K  (Gm symmetric: (Gm b)[i] = sum_k Gm[k][i] b[k])
    zcol[K] = -reduce_rows4(Gm[0] * bk[0] + Gm[1] * bk[1] + Gm[2] * bk[2] + Gm[3] * bk[3]);
    if constexpr (K + 1 < NB) {
      // Pm_J = Gm B_KJ;  b_J += Pm_J^T b_K (per-row-group partials)
      floatx4 Pm[NB];
      if constexpr (SPLIT) {
        // block row K's scale; Pm_J = Gm^T A_KJ on split f16
        float mx = 0.f;
        static_for<NB - 1 - K>([&](auto jc) {
          mx = fmaxf(mx, absmax4(A[w1_tile<NB>(K, K + 1 + decltype(jc)::value)]));
        });
        const int eX = split_exponent(wave_max(mx));
        float mp = 0.f;
        static_for<NB - 1 - K>([&](auto jc) {
          constexpr int j = decltype(jc)::value;
          XK[j] = split_hl(A[w1_tile<NB>(K, K + 1 + j)], ldexpf(1.f, eX));
        });
        const int eG = split_exponent(wave_max(absmax4(Gm)));
        const half8v g = split_hl(Gm, ldexpf(1.f, eG));
        const half8v gh = dup_hi(g), gl = dup_lo(g);
        const float invGX = ldexpf(1.f, -eG - eX);
        static_for<NB - 1 - K>([&](auto jc) {
          constexpr int j = decltype(jc)::value;
          // Gm^T X = [Gl|Gl]^T [Xh|Xl] + [Gh|Gh]^T [Xh|Xl]
          floatx4 acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(gl, XK[j],
                                                              floatx4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(gh, XK[j], acc, 0, 0, 0) * invGX;
          Pm[j] = acc;
          bcol[K + 1 + j] += acc[0] * bk[0] + acc[1] * bk[1] + acc[2] * bk[2] + acc[3] * bk[3];
          mp = fmaxf(mp, absmax4(acc));
        });
        // Schur operands 2^a X and 2^-a Pm: a balances the two maxima (both at
        // 2^((x + p) / 2)), clamped so neither exceeds 2^15
        const int eP = split_exponent(wave_max(mp));
        const int a = min(max((eX - eP) >> 1, -eP), eX);
        static_for<NB - 1 - K>([&](auto jc) {
          constexpr int j = decltype(jc)::value;
          XK[j] = split_hl(A[w1_tile<NB>(K, K + 1 + j)], ldexpf(1.f, a));
          const half8v p = split_hl(Pm[j], ldexpf(1.f, -a));
          Ph[j] = dup_hi(p);
          Pl[j] = dup_lo(p);
        });
      } else {
        static_for<NB - 1 - K>([&](auto jc) {
          constexpr int J = K + 1 + decltype(jc)::value;
          const floatx4 acc = tile_xty(Gm, A[w1_tile<NB>(K, J)], floatx4{0.f, 0.f, 0.f, 0.f});
          Pm[decltype(jc)::value] = acc;
          bcol[J] += acc[0] * bk[0] + acc[1] * bk[1] + acc[2] * bk[2] + acc[3] * bk[3];
        });
      }
      // Pm of block row K -> LDS for the back substitution (lane-private slots)
      static_for<NB - 1 - K>([&](auto jc) {
        constexpr int J = K + 1 + decltype(jc)::value;
        *reinterpret_cast<floatx4*>(lds + L::PM + (w1_tile<NB>(K, J) - (K + 1)) * 256 + 4 * lane) =
            Pm[decltype(jc)::value];
      });
      // the next pivot block's Schur update first, then its sweep with the rest of
      // step K's Schur updates (independent of it) issued between the pivots
      schur(Kc, std::integral_constant<int, 0>{}, Pm);
      pivot_block(std::integral_constant<int, K + 1>{}, [&](auto pc) {
        constexpr int p = decltype(pc)::value;
        static_for<schur_n<NB>(K) - 1>([&](auto vc) {
          constexpr int u = 1 + decltype(vc)::value;
          if constexpr ((u - 1) % 16 == p) schur(Kc, std::integral_constant<int, u>{}, Pm);
        });
      });
    }
  });
  // back substitution x_K = z_K + sum_{J>K} Pm_KJ x_J (column layout)
  xcol[NB - 1] = zcol[NB - 1];
  static_for<NB - 1>([&](auto kc) {
    constexpr int K = NB - 2 - decltype(kc)::value;
    float pr[4] = {0.f, 0.f, 0.f, 0.f};
    static_for<NB - 1 - K>([&](auto jc) {
      constexpr int J = K + 1 + decltype(jc)::value;
      const floatx4 pm = *reinterpret_cast<const floatx4*>(
          lds + L::PM + (w1_tile<NB>(K, J) - (K + 1)) * 256 + 4 * lane);
#pragma unroll
      for (int r = 0; r < 4; ++r) pr[r] = fmaf(pm[r], xcol[J], pr[r]);
    });
#pragma unroll
    for (int r = 0; r < 4; ++r) pr[r] = reduce_lanes16(pr[r]);  // rows 4q+r of Pm x
    if (m == 0) *reinterpret_cast<floatx4*>(vec + 4 * q) = floatx4{pr[0], pr[1], pr[2], pr[3]};
    wave_lds_order();
    xcol[K] = zcol[K] + vec[m];
    wave_lds_order();
  });
  // a NaN pivot (or overflow) leaves a non-finite solution; a pivot spread beyond
  // kCondMax (a lower bound on cond(A)) is outside what the fp32 solve can hold to the
  // 1e-4 bar: the row is re-solved in fp64 (rescue64_kernel)
  bool fin = true;
#pragma unroll
  for (int c = 0; c < NB; ++c) fin = fin && (xcol[c] - xcol[c] == 0.f);
  // spread over the 16 lanes of a row group (every row group holds the same pivots)
  rmin = fminf(rmin, dpp_f<0xB1>(rmin));
  rmax = fmaxf(rmax, dpp_f<0xB1>(rmax));
  rmin = fminf(rmin, dpp_f<0x4E>(rmin));
  rmax = fmaxf(rmax, dpp_f<0x4E>(rmax));
  rmin = fminf(rmin, dpp_f<0x141>(rmin));
  rmax = fmaxf(rmax, dpp_f<0x141>(rmax));
  rmin = fminf(rmin, dpp_f<0x140>(rmin));
  rmax = fmaxf(rmax, dpp_f<0x140>(rmax));
  return dmin > 0.f && rmin > 0.f && rmax <= cond_max * rmin && __ballot(!fin) == 0;
}

// w1_solve_x, then the solution row written un-permuted: dim d = i * NB + c <->
// block c, index i = lane m; dims in [k, ld) written as zero.
template <int NB, bool SPLIT = kW1SplitSchur<NB>>
__device__ __forceinline__ bool w1_solve(floatx4 (&A)[NB * (NB + 1) / 2], float (&bcol)[NB],
                                         float* __restrict__ lds, int k,
                                         float* __restrict__ xrow, int ld,
                                         float cond_max = kCondMax) {
  float xcol[NB];
  const bool ok = w1_solve_x<NB, SPLIT>(A, bcol, lds, k, xcol, cond_max);
  const int lane = threadIdx.x & 63, m = lane & 15;
  if (lane < 16) {
#pragma unroll
    for (int c = 0; c < NB; ++c) {
      const int d = m * NB + c;
      if (d < ld) xrow[d] = (d < k && ok) ? xcol[c] : 0.f;
    }
  }
  return ok;
}

// ---------------------------------------------------------------------------
// Iterative refinement of the implicit rows' panel solutions (k <= 64).
//
// The fp32-grade Gram (split-f16 products, fp32 sums) and the fp32 LDL^T each
// perturb A by ~2^-21..2^-24 relative, which the condition of an implicit system
// (confidences 1 + alpha |r| spanning decades) amplifies: emulated at ranks 16-64 on
// counts 1..1e6, 1e-4..4e-3 relative errors, half from each source.  Mixed-precision
// refinement removes both: r = b - A x with A's own terms in Spark's fp64 arithmetic
// (NormalEquation.add: products of fp32 values, exact in fp64; YtY; lambda n), the
// correction A d = r solved with the kept fp32 factorisation, x += d.  Each step
// contracts the error by ~cond(A) 2^-21, and |d| estimates the error it removed, so
// the loop is its own a-posteriori test: done when |d| <= kIrConv |x| (the error left
// is then ~(|d| / |x|)^2 |x| <= 1e-7 |x|), and a row that has not converged within
// kIrSteps, or whose correction exceeds kIrDiverge |x| (contraction not reliable), is
// re-solved in fp64 (rescue64_kernel).
// ---------------------------------------------------------------------------
constexpr int kIrSteps = 3;
constexpr float kIrConv = 3e-4f;
constexpr float kIrDiverge = 0.1f;

// The implicit row's ratings and source factors (for the residual pass).
struct IrArgs {
  const int32_t* col;
  const float* val;
  const float* Y;
  int64_t pb, pe;
  float alpha;
};

// LDS after the panel (floats): x in fp64 (natural order, 64) | batch weights g
// (64 doubles) | their columns (64 ints) | residual rhs, correction (permuted, 16 NB).
template <int CN>
struct IrLds {
  static constexpr int XS = PanelLds<CN>::SIZE, GS = XS + 128, CC = GS + 128, RV = CC + 64,
                       DX = RV + 16 * CN, SIZE = DX + 16 * CN;
  static_assert(XS % 4 == 0, "fp64 alignment");
};

// r_d = b_d - ((G + YtY + lambda n I) x)_d for an implicit row, lane d < k (fp64).
// Batches of 64 ratings: lane j forms g_j = [r_j > 0](1 + c_j) - c_j (y_j . x), then
// lane d accumulates sum_j g_j y_jd (coalesced row reads, L2-hot after the Gram pass).
__device__ __forceinline__ double implicit_residual(const IrArgs& a, int ld, int k,
                                                    const double* __restrict__ yty, double lam_n,
                                                    const double* __restrict__ xs,
                                                    double* __restrict__ gs, int* __restrict__ cc) {
  const int lane = threadIdx.x & 63;
  double r = 0.0;
  for (int64_t base = a.pb; base < a.pe; base += 64) {
    const int nb = (int)(a.pe - base < 64 ? a.pe - base : 64);
    double g = 0.0;
    int c = 0;
    if (lane < nb) {
      c = a.col[base + lane];
      const double rv = (double)a.val[base + lane];
      const float* y = a.Y + (int64_t)c * ld;
      double s0 = 0.0, s1 = 0.0;
      for (int d = 0; d < k; d += 4) {  // xs is zero past k (< ld, ld % 4 == 0)
        const float4 v = *reinterpret_cast<const float4*>(y + d);
        s0 = fma((double)v.x, xs[d], s0);
        s1 = fma((double)v.y, xs[d + 1], s1);
        s0 = fma((double)v.z, xs[d + 2], s0);
        s1 = fma((double)v.w, xs[d + 3], s1);
      }
      const double c1 = (double)a.alpha * fabs(rv);
      g = (rv > 0.0 ? 1.0 + c1 : 0.0) - c1 * (s0 + s1);
    }
    gs[lane] = g;
    cc[lane] = c;
    wave_lds_sync();
    if (lane < k) {
#pragma unroll 8
      for (int j = 0; j < nb; ++j) r = fma(gs[j], (double)a.Y[(int64_t)cc[j] * ld + lane], r);
    }
    wave_lds_sync();
  }
  if (lane < k) {
    for (int e = 0; e < k; ++e) {
      const int hi = lane > e ? lane : e, lo = lane > e ? e : lane;
      r = fma(-yty[hi * (hi + 1) / 2 + lo], xs[e], r);
    }
    r = fma(-lam_n, xs[lane], r);
  }
  return r;
}

// Refine the panel solution in Xv (permuted layout) in place; true once converged.
template <int CN>
__device__ __forceinline__ bool panel_refine(float* __restrict__ lds, const IrArgs& a, int ld,
                                             int k, const double* __restrict__ yty,
                                             double lam_n) {
  typedef PanelLds<CN> Lo;
  typedef IrLds<CN> Ir;
  float* Xv = lds + Lo::X;
  float* Zv = lds + Lo::Z;
  const float* Dv = lds + Lo::D;
  double* xs = reinterpret_cast<double*>(lds + Ir::XS);
  double* gs = reinterpret_cast<double*>(lds + Ir::GS);
  int* cc = reinterpret_cast<int*>(lds + Ir::CC);
  float* Rv = lds + Ir::RV;
  float* DX = lds + Ir::DX;
  const int lane = threadIdx.x & 63;
  const int pl = (lane % CN) * 16 + lane / CN;  // permuted slot of natural dim `lane`
  bool conv = false;
  for (int it = 0; it < kIrSteps; ++it) {
    xs[lane] = lane < k ? (double)Xv[pl] : 0.0;  // k <= 64: one dim per lane
    wave_lds_sync();
    const double r = implicit_residual(a, ld, k, yty, lam_n, xs, gs, cc);
    if (lane < 16 * CN) Rv[pl] = lane < k ? (float)r : 0.f;
    wave_lds_sync();
    block_fwd_subst<Lo::CS>(CN, lds + Lo::T, Rv, Zv);
    block_back_subst<Lo::CS>(CN, lds + Lo::T, Zv, Dv, DX);
    float nd = 0.f, nx = 0.f;
    if (lane < 16 * CN) {
      const float dx = DX[lane];
      const float xn = Xv[lane] + dx;
      Xv[lane] = xn;
      nd = dx * dx;
      nx = xn * xn;
    }
    wave_lds_sync();
    for (int o = 32; o > 0; o >>= 1) {
      nd += __shfl_xor(nd, o);
      nx += __shfl_xor(nx, o);
    }
    if (nd <= (kIrConv * kIrConv) * nx) {
      conv = true;
      break;
    }
    if (!(nd <= (kIrDiverge * kIrDiverge) * nx)) break;  // (NaN included)
  }
  return conv;
}

template <int CN, bool IMPLICIT = false>
struct SmemBytes {
  static constexpr int value =
      (int)sizeof(float) * (IMPLICIT ? IrLds<CN>::SIZE : PanelLds<CN>::SIZE);
};
template <bool IMPLICIT>
struct SmemBytes<8, IMPLICIT> {  // W1: transposition buffer (the Gram's 192-word staging fits in it)
  static constexpr int value = (int)sizeof(float) * W1Lds::SIZE;
};

__device__ __forceinline__ float shfl_xor_t(float v, int m) { return __shfl_xor(v, m); }
__device__ __forceinline__ double shfl_xor_t(double v, int m) { return shfl_xor_f64(v, m); }

// Shared tail of a row: rhs reduce over the 4 rating slots, complete the normal
// equations (Spark CholeskySolver.solve: ata[ii] += lambda * numExplicits;
// implicit: ls.merge(YtY), added in fp64 before the single rounding to fp32),
// then the block LDL^T on the matrix cores.  fp32 factorisation: the systems are
// regularised (cond ~ (lambda + |y|^2)/lambda, measured <= 240 for implicit
// alpha = 40 at k = 128), fp32 error ~2e-6 vs the 1e-4 parity bar.
template <int CN, bool IMPLICIT, class AccT>
__device__ __forceinline__ void finish_and_solve(AccT (&tot)[Cfg<CN>::NT][4], AccT (&bt)[CN],
                                                 int64_t n_reg, unsigned char* smem, int k,
                                                 float reg, const double* __restrict__ yty,
                                                 float* __restrict__ xrow, int ld, int row,
                                                 RescueList rl, const IrArgs& ir) {
  constexpr int NT = Cfg<CN>::NT;
  float bq[CN];
  const int m = threadIdx.x & 15;
#pragma unroll
  for (int c = 0; c < CN; ++c) {
    AccT v = bt[c];
    v += shfl_xor_t(v, 16);
    v += shfl_xor_t(v, 32);
    bq[c] = m * CN + c < k ? (float)v : 0.f;  // padded dims: rhs 0
  }
  floatx4 A[NT];
  int tt = 0;
#pragma unroll
  for (int c1 = 0; c1 < CN; ++c1) {
#pragma unroll
    for (int c2 = c1; c2 < CN; ++c2) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if constexpr (IMPLICIT) {
          int i, j;
          tile_ij<CN>(c1, c2, r, i, j);
          const int hi = i > j ? i : j, lo = i > j ? j : i;
          A[tt][r] = (float)((double)tot[tt][r] + yty[hi * (hi + 1) / 2 + lo]);
        } else {
          A[tt][r] = (float)tot[tt][r];
        }
        int i, j;
        tile_ij<CN>(c1, c2, r, i, j);
        if (i >= k || j >= k) A[tt][r] = 0.f;  // padded dims: rows/columns of the identity
      }
      ++tt;
    }
  }
  regularise_f32<CN>(A, (float)((double)reg * (double)n_reg), k);
  float* lds = reinterpret_cast<float*>(smem);
  if constexpr (IMPLICIT) {
    // pivots checked here, accuracy a posteriori by the refinement
    bool ok = panel_ldl_solve<CN, false, false>(A, bq, lds, k, xrow, ld);
    if (ok) ok = panel_refine<CN>(lds, ir, ld, k, yty, (double)reg * (double)n_reg);
    panel_store_x<CN>(lds + PanelLds<CN>::X, k, ok, xrow, ld);
    if (!ok) rescue_append(rl, row);  // re-solved in fp64
  } else {
    const bool ok = panel_ldl_solve<CN>(A, bq, lds, k, xrow, ld);
    if (!ok) rescue_append(rl, row);  // re-solved in fp64
  }
}

// Partial-sum slot of one task: N tiles x 4 accumulator rows, NRA rhs values and
// the positive-rating count, each as 64 lane-contiguous doubles.
template <int N, int NRA>
struct Slot {
  static constexpr int SIZE = (N * 4 + NRA + 1) * 64;
};

template <int N, int NRA, class AccT>
__device__ __forceinline__ void store_slot(double* __restrict__ slot, const AccT (&tot)[N][4],
                                           const AccT (&bt)[NRA], float npos) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < N; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) slot[(t * 4 + r) * 64 + lane] = (double)tot[t][r];
#pragma unroll
  for (int c = 0; c < NRA; ++c) slot[(N * 4 + c) * 64 + lane] = (double)bt[c];
  slot[(N * 4 + NRA) * 64 + lane] = (double)npos;
}

template <int N, int NRA>
__device__ __forceinline__ void add_slot(const double* __restrict__ slot, double (&a64)[N][4],
                                         double (&b64)[NRA], int& npos) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < N; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) a64[t][r] += slot[(t * 4 + r) * 64 + lane];
#pragma unroll
  for (int c = 0; c < NRA; ++c) b64[c] += slot[(N * 4 + c) * 64 + lane];
  npos += (int)slot[(N * 4 + NRA) * 64 + lane];
}

// The same slot as fp32 (a chunk task's sums are fp32 anyway: storing them as fp64
// only doubled the launch-1 write and launch-2a read bytes of the k <= 64 heavy rows).
template <int N, int NRA>
__device__ __forceinline__ void store_slot_f32(float* __restrict__ slot, const float (&tot)[N][4],
                                               const float (&bt)[NRA], float npos) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < N; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) slot[(t * 4 + r) * 64 + lane] = tot[t][r];
#pragma unroll
  for (int c = 0; c < NRA; ++c) slot[(N * 4 + c) * 64 + lane] = bt[c];
  slot[(N * 4 + NRA) * 64 + lane] = npos;
}

template <int N, int NRA>
__device__ __forceinline__ void add_slot_f32(const float* __restrict__ slot, double (&a64)[N][4],
                                             double (&b64)[NRA], int& npos) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < N; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) a64[t][r] += (double)slot[(t * 4 + r) * 64 + lane];
#pragma unroll
  for (int c = 0; c < NRA; ++c) b64[c] += (double)slot[(N * 4 + c) * 64 + lane];
  npos += (int)slot[(N * 4 + NRA) * 64 + lane];
}

template <int N, int NRA, class AccT>
__device__ __forceinline__ void zero_acc(AccT (&tot)[N][4], AccT (&bt)[NRA]) {
#pragma unroll
  for (int t = 0; t < N; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) tot[t][r] = AccT(0);
#pragma unroll
  for (int c = 0; c < NRA; ++c) bt[c] = AccT(0);
}

// Launch 1 of a half-sweep: heavy-row chunks (-> fp64 partial slots) and
// whole light rows (Gram + solve fused, A never leaves the CU), interleaved.
// Gram on the split f16 MFMA, fp32 accumulation over a task (<= chunk
// ratings), fp64 across the chunks of a heavy row.  scal[0] = max |Y_src|,
// scal[1] = max |rating| (prep phase).  Explicit: Gram and rhs from the split
// table Ysp (kp words per row, zero row `zero_row`); implicit: from Y, split in
// registers after the per-rating confidence weight.
template <bool ADD_YTY, int NB = kW1NB, bool SPLIT = kW1SplitSchur<NB>>
__device__ __forceinline__ void w1_finish_and_solve(floatx4 (&A)[NB * (NB + 1) / 2],
                                                    float scale, float (&bt)[NB], int64_t n_reg,
                                                    const float* __restrict__ ytyC,
                                                    unsigned char* smem, int k, float reg,
                                                    float* __restrict__ xrow, int ld, int row,
                                                    RescueList rl, float cond_max = kCondMax);

// (k <= 64 keeps one gather step in flight: two steps need 187 registers, i.e. two
// waves per SIMD instead of three, measured slower on configs[1]: 2.07 -> 2.24 ms/iter.)
// (Four waves per SIMD for explicit k <= 64 spill 49 registers: 2.76 vs 2.25 ms/iter;
// round 5, after the lean sweep, 11 spills: 2.14 vs 2.02 ms/iter, profiles/r05/ab_occupancy.jsonl.)
template <int CN, bool IMPLICIT>
__global__ __launch_bounds__(64, IMPLICIT ? 2 : 3) void gram_solve_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ val, const int32_t* __restrict__ light_rows,
    const int32_t* __restrict__ chunk_row, const int64_t* __restrict__ chunk_begin,
    const int64_t* __restrict__ chunk_end, int32_t n_chunks, int32_t n_light,
    const float* __restrict__ Y, float* __restrict__ X, int ld, int k, float reg, float alpha,
    const double* __restrict__ yty, float* __restrict__ slots, int32_t* __restrict__ status,
    const float* __restrict__ scal, const uint32_t* __restrict__ Ysp, int32_t kp,
    int32_t zero_row, RescueList rl) {
  constexpr int NT = Cfg<CN>::NT;
  __shared__ __attribute__((aligned(16))) unsigned char smem[SmemBytes<CN, IMPLICIT>::value];
  floatx4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
  float tot[NT][4], bt[CN];
#pragma unroll
  for (int c = 0; c < CN; ++c) bt[c] = 0.f;
  int npos = 0;
  int chunk, light;
  decode_task(blockIdx.x, n_chunks, n_light, chunk, light);
  int64_t pb, pe;
  int row = -1;
  if (chunk >= 0) {
    pb = chunk_begin[chunk];
    pe = chunk_end[chunk];
  } else {
    row = light_rows[light];
    pb = row_ptr[row];
    pe = row_ptr[row + 1];
  }
  float inv2;
  float rmax = 0.f;  // explicit: this lane's max |rating| (split window guard)
  if constexpr (IMPLICIT) {
    const int e = split_exponent(scal[0] * __builtin_sqrtf(alpha * scal[1]));
    inv2 = ldexpf(1.f, -2 * e);
    gram_accumulate_split<CN, true>(col, val, pb, pe, Y, ld, k, alpha, ldexpf(1.f, e), acc, bt,
                                    npos, reinterpret_cast<int*>(smem));
  } else {
    const int ey = split_exponent(scal[0]), er = split_exponent(scal[1]);
    inv2 = ldexpf(1.f, -2 * ey);
    floatx4 accb[CN];
#pragma unroll
    for (int c = 0; c < CN; ++c) accb[c] = floatx4{0.f, 0.f, 0.f, 0.f};
    gram_accumulate_pre<FullTiles<CN>>(col, val, pb, pe, Ysp, (uint32_t)kp, zero_row,
                                       ldexpf(1.f, er), (threadIdx.x & 15) * CN, acc, accb,
                                       reinterpret_cast<int*>(smem), rmax);
    rhs_from_tiles<FullTiles<CN>>(accb, ldexpf(1.f, -ey - er), bt);
    rmax *= ldexpf(1.f, er);
    if (chunk < 0 && (window_miss(diag_max_lane<CN>(acc), (float)(pe - pb), rmax) ||
                      rank_deficient_illcond<CN>(acc, inv2, pe - pb, k, reg))) {
      rescue_append(rl, row);
      return;
    }
  }
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) tot[t][r] = acc[t][r] * inv2;
  if (chunk >= 0) {
    // explicit: the npos entry carries the chunk's scaled max |rating| (launch 2 takes
    // the max over the chunks for the window guard)
    store_slot_f32<NT, CN>(slots + (int64_t)chunk * Cfg<CN>::SLOT, tot, bt,
                           IMPLICIT ? (float)npos : rmax);
    return;
  }
  __syncthreads();  // staging area is reused by the solve
  const int64_t n_reg = IMPLICIT ? (int64_t)npos : (pe - pb);
  if constexpr (!IMPLICIT && CN == 4) {
    // rank 33-64 explicit: the W1 block elimination on 4 x 4 tiles (swept diagonal
    // inverses + fp32 MFMA), in the Gram's scale
    static_assert(W1LdsT<4>::SIZE <= PanelLds<4>::SIZE, "W1<4> LDS");
    w1_finish_and_solve<false, 4, false>(acc, inv2, bt, n_reg, nullptr, smem, k, reg,
                                  X + (int64_t)row * ld, ld, row, rl);
  } else {
    finish_and_solve<CN, IMPLICIT, float>(tot, bt, n_reg, smem, k, reg, yty,
                                          X + (int64_t)row * ld, ld, row, rl,
                                          IrArgs{col, val, Y, pb, pe, alpha});
  }
}

__device__ __forceinline__ void block_absmax_publish(float m, unsigned* __restrict__ out) {
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    atomicMax(out, __float_as_uint(m));  // NaN-free non-negative floats order as uints
  }
}

// max |rating| of a CSR block (ratings val[0, row_ptr[n_rows])) -> *out.
__global__ __launch_bounds__(256) void absmax_csr_kernel(const int64_t* __restrict__ row_ptr,
                                                         int32_t n_rows,
                                                         const float* __restrict__ val,
                                                         unsigned* __restrict__ out) {
  const int64_t n = row_ptr[n_rows];
  float m = 0.f;
  const int64_t n4 = n >> 2;  // val is 16-byte aligned (a CSR value array)
  const float4* v4 = reinterpret_cast<const float4*>(val);
  auto fold = [&](const float4& v) {
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
  };
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n4; i += 4 * stride) {  // four independent loads in flight
    const float4 a = v4[i], b = v4[i + stride], c = v4[i + 2 * stride], d = v4[i + 3 * stride];
    fold(a);
    fold(b);
    fold(c);
    fold(d);
  }
  for (; i < n4; i += stride) fold(v4[i]);
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) m = fmaxf(m, fabsf(val[4 * n4 + threadIdx.x]));
  block_absmax_publish(m, out);
}

// max |x| over n floats -> *out (as ordered uint bits; *out zeroed beforehand).
// (zero_word[0..1], when given, are cleared by block 0: the rescue count and its
// finished-block counter for the half-sweep this prep starts, without a memset)
__global__ __launch_bounds__(256) void absmax_kernel(const float* __restrict__ x, int64_t n,
                                                     unsigned* __restrict__ out,
                                                     unsigned* __restrict__ zero_word) {
  if (zero_word != nullptr && blockIdx.x == 0 && threadIdx.x < 2) zero_word[threadIdx.x] = 0u;
  float m = 0.f;
  const int64_t n4 = n >> 2;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  auto fold = [&](const float4& v) {
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
  };
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n4; i += 4 * stride) {  // four independent loads in flight
    const float4 a = x4[i], b = x4[i + stride], c = x4[i + 2 * stride], d = x4[i + 3 * stride];
    fold(a);
    fold(b);
    fold(c);
    fold(d);
  }
  for (; i < n4; i += stride) fold(x4[i]);
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) m = fmaxf(m, fabsf(x[4 * n4 + threadIdx.x]));
  block_absmax_publish(m, out);
}

// Launch 2: heavy rows — sum their chunk slots in a fixed order (fp64), then solve.
// Launch 2a (k <= 64): a heavy row's fp32 chunk slots summed element-wise in fp64 (one
// thread per slot element, four interleaved partial sums in a fixed order), rounded
// once to fp32 into its first slot; each thread reads and writes only its own element.
// Explicit: the last 64 entries (each chunk's scaled max |rating|) take the max.
// The partial slots of heavy row h: [slot_begin[h], slot_begin[h+1]) and, for a
// two-segment schedule (slot_begin2 != null: the sharded engine's pipelined item
// side, whose rows have an early and a late rating segment), [slot_begin2[h],
// slot_begin2[h+1]).  The first slot of the union is the row's home slot, where
// launch 2a leaves the sum.
struct SlotRange {
  int s0, n1, t0, n;
  __device__ __forceinline__ int at(int i) const { return i < n1 ? s0 + i : t0 + (i - n1); }
  __device__ __forceinline__ int home() const { return at(0); }
};
__device__ __forceinline__ SlotRange slot_range(const int32_t* __restrict__ sb,
                                                const int32_t* __restrict__ sb2, int h) {
  SlotRange r;
  r.s0 = sb[h];
  r.n1 = sb[h + 1] - r.s0;
  r.t0 = sb2 ? sb2[h] : 0;
  r.n = r.n1 + (sb2 ? sb2[h + 1] - r.t0 : 0);
  return r;
}

template <int SLOT, bool IMPLICIT>
__global__ __launch_bounds__(256) void heavy_sum_f64_kernel(const int32_t* __restrict__ slot_begin,
                                                            const int32_t* __restrict__ slot_begin2,
                                                            float* __restrict__ slots) {
  const int h = blockIdx.y;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= SLOT) return;
  const SlotRange sr = slot_range(slot_begin, slot_begin2, h);
  if (sr.n <= 1) return;
  const int64_t home = (int64_t)sr.home() * SLOT + e;
  if (!IMPLICIT && e >= SLOT - 64) {
    float mx = 0.f;
    for (int i = 0; i < sr.n; ++i) mx = fmaxf(mx, slots[(int64_t)sr.at(i) * SLOT + e]);
    slots[home] = mx;
    return;
  }
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  int i = 0;
  for (; i + 4 <= sr.n; i += 4) {
    a0 += (double)slots[(int64_t)sr.at(i) * SLOT + e];
    a1 += (double)slots[(int64_t)sr.at(i + 1) * SLOT + e];
    a2 += (double)slots[(int64_t)sr.at(i + 2) * SLOT + e];
    a3 += (double)slots[(int64_t)sr.at(i + 3) * SLOT + e];
  }
  for (; i < sr.n; ++i) a0 += (double)slots[(int64_t)sr.at(i) * SLOT + e];
  slots[home] = (float)((a0 + a1) + (a2 + a3));
}

template <int CN, bool IMPLICIT>
__global__ __launch_bounds__(64, 2) void reduce_solve_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ val, const float* __restrict__ Y, float alpha,
    const int32_t* __restrict__ heavy_rows, const int32_t* __restrict__ slot_begin,
    const int32_t* __restrict__ slot_begin2, const float* __restrict__ slots,
    float* __restrict__ X, int ld, int k, float reg, const double* __restrict__ yty,
    int32_t* __restrict__ status, const float* __restrict__ scal,
    RescueList rl) {
  constexpr int NT = Cfg<CN>::NT;
  __shared__ __attribute__((aligned(16))) unsigned char smem[SmemBytes<CN, IMPLICIT>::value];
  const int h = blockIdx.x;
  const int row = heavy_rows[h];
  double a64[NT][4], b64[CN];
  zero_acc<NT, CN, double>(a64, b64);
  int npos = 0;
  // the row's chunk slots were summed into its home slot (heavy_sum_f64_kernel)
  const float* sl =
      slots + (int64_t)slot_range(slot_begin, slot_begin2, h).home() * Cfg<CN>::SLOT;
  add_slot_f32<NT, CN>(sl, a64, b64, npos);
  const int64_t n_reg = IMPLICIT ? (int64_t)npos : (row_ptr[row + 1] - row_ptr[row]);
  if constexpr (!IMPLICIT) {  // split window guard over the whole row
    const float s2 = ldexpf(1.f, 2 * split_exponent(scal[0]));
    float d = 0.f;
    const int lane = threadIdx.x & 63, q = lane >> 4, m = lane & 15;
#pragma unroll
    for (int c = 0; c < CN; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (4 * q + r == m) d = fmaxf(d, (float)a64[tile_index(CN, c, c)][r] * s2);
    if (window_miss(d, (float)n_reg, (float)sl[(NT * 4 + CN) * 64 + lane])) {
      rescue_append(rl, row);
      return;
    }
  }
  finish_and_solve<CN, IMPLICIT, double>(a64, b64, n_reg, smem, k, reg, yty,
                                         X + (int64_t)row * ld, ld, row, rl,
                                         IrArgs{col, val, Y, row_ptr[row], row_ptr[row + 1],
                                                alpha});
}

// ---------------------------------------------------------------------------
// W1 kernels (k in (64, 128], one wavefront per system).  The 36 scaled Gram
// tiles are finished in place, tile by tile (regularisation, implicit YtY from
// a C-layout fp32 table, identity rows for padded dims), so the register file
// holds one copy of the system.  Heavy-row chunk partials are stored as fp32
// (a chunk's sum is fp32 anyway) and summed in fp64 in launch 2, where the YtY
// merge is done in fp64 before the single rounding.
// ---------------------------------------------------------------------------
constexpr int kW1NT = 36;
// Explicit W1 Gram with two gather steps in flight (gram_accumulate_pre2).
constexpr bool kW1Prefetch2 = true;
constexpr int kW1Slot = (kW1NT * 4 + kW1NB + 1) * 64;  // floats per chunk partial
constexpr int kW1YtyC = kW1NT * 4 * 64;               // floats of the C-layout YtY table
// Implicit W1 light rows: the C-layout YtY table is copied into the wave's LDS by
// LDS-DMA when the row starts (36 KB, landing while the Gram accumulates), past the
// Gram's 192-word staging area; the solve's LDS (W1Lds, written only after the table
// has been read) overlaps it.  Read from global at the end instead, the compiler
// spread the 144 loads per lane over ~20 dependent waits — at one wavefront per SIMD,
// each an unhidden L2 round trip.  4 x 37.9 KB per CU (one wave per SIMD).
constexpr int kW1YtyLdsOff = 1024;  // bytes
constexpr int kW1SmemImplicit =
    (kW1YtyLdsOff + 4 * kW1YtyC) > (int)sizeof(float) * W1Lds::SIZE ? (kW1YtyLdsOff + 4 * kW1YtyC)
                                                                    : (int)sizeof(float) * W1Lds::SIZE;
static_assert(kW1YtyC % 256 == 0, "YtY table in 1 KB LDS-DMA pieces");

// ytyC[(t * 4 + r) * 64 + lane] = fp32 YtY entry of register r of upper tile t.
__global__ __launch_bounds__(64) void yty_ctab_kernel(const double* __restrict__ yty,
                                                      float* __restrict__ ytyC) {
  static_for<kW1NT>([&](auto tc) {
    constexpr int t = decltype(tc)::value;
    constexpr int c1 = FullTiles<8>::l1(t), c2 = FullTiles<8>::l2(t);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      int i, j;
      tile_ij<8>(c1, c2, r, i, j);
      const int hi = i > j ? i : j, lo = i > j ? j : i;
      ytyC[(t * 4 + r) * 64 + threadIdx.x] = (float)yty[hi * (hi + 1) / 2 + lo];
    }
  });
}

// Completes the normal equations of one system in place and solves them.  A holds
// the Gram divided by `scale` (the split MFMA's power-of-two scaling, 1 for the
// reduced heavy rows); instead of rescaling 144 registers, the system is solved
// in that scale: (A + (lambda n / scale) I) x = b / scale  (+ YtY / scale for
// implicit, from the C-layout table).  Padded dims (k < 128) become identity
// rows/columns.  bt: per-lane rhs partials (summed over the 4 rating slots here).
template <bool ADD_YTY, int NB, bool SPLIT>
__device__ __forceinline__ void w1_finish_and_solve(floatx4 (&A)[NB * (NB + 1) / 2],
                                                    float scale, float (&bt)[NB], int64_t n_reg,
                                                    const float* __restrict__ ytyC,
                                                    unsigned char* smem, int k, float reg,
                                                    float* __restrict__ xrow, int ld, int row,
                                                    RescueList rl, float cond_max) {
  constexpr int NT_ = NB * (NB + 1) / 2;
  const int lane = threadIdx.x & 63, q = lane >> 4, m = lane & 15;
  const float inv = 1.f / scale;  // power of two: exact
  float bq[NB];
#pragma unroll
  for (int c = 0; c < NB; ++c) {
    const float v = reduce_rows4(bt[c]) * inv;
    bq[c] = m * NB + c < k ? v : 0.f;
  }
  const float lam = (float)((double)reg * (double)n_reg) * inv;
  if constexpr (ADD_YTY) {
    static_for<NT_>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
#pragma unroll
      for (int r = 0; r < 4; ++r) A[t][r] = fmaf(ytyC[(t * 4 + r) * 64 + lane], inv, A[t][r]);
    });
  }
  if (k == NB * 16) {  // uniform: no padded dims, lambda on the diagonal only
    static_for<NB>([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      constexpr int t = w1_tile<NB>(c, c);
#pragma unroll
      for (int r = 0; r < 4; ++r) A[t][r] += (4 * q + r == m) ? lam : 0.f;
    });
  } else {
    static_for<NT_>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      constexpr int c1 = FullTiles<NB>::l1(t), c2 = FullTiles<NB>::l2(t);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int i, j;
        tile_ij<NB>(c1, c2, r, i, j);
        const bool pad = (i >= k) | (j >= k);
        float v = pad ? 0.f : A[t][r];
        if constexpr (c1 == c2) v = (i == j) ? (pad ? 1.f : v + lam) : v;
        A[t][r] = v;
      }
    });
  }
  const bool ok = w1_solve<NB, SPLIT>(A, bq, reinterpret_cast<float*>(smem), k, xrow, ld, cond_max);
  if (!ok) rescue_append(rl, row);  // re-solved in fp64
}

// Launch 1 (W1): heavy-row chunks (-> fp32 partial slots) and whole light rows
// (Gram + solve fused), as gram_solve_kernel.  ytyC: C-layout YtY (implicit).
template <bool IMPLICIT>
__global__ __launch_bounds__(64, 1) void gram_solve_w1_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ val, const int32_t* __restrict__ light_rows,
    const int64_t* __restrict__ chunk_begin, const int64_t* __restrict__ chunk_end,
    int32_t n_chunks, int32_t n_light, const float* __restrict__ Y, float* __restrict__ X, int ld,
    int k, float reg, float alpha, const float* __restrict__ ytyC, float* __restrict__ slots,
    int32_t* __restrict__ status, const float* __restrict__ scal, const uint32_t* __restrict__ Ysp,
    int32_t kp, int32_t zero_row, RescueList rl) {
  constexpr int CN = 8, NT = kW1NT;
  __shared__ __attribute__((aligned(16))) unsigned char smem[IMPLICIT ? kW1SmemImplicit
                                                                      : SmemBytes<CN>::value];
  const int lane = threadIdx.x & 63;
  floatx4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
  float bt[CN];
#pragma unroll
  for (int c = 0; c < CN; ++c) bt[c] = 0.f;
  int npos = 0;
  int chunk, light;
  decode_task(blockIdx.x, n_chunks, n_light, chunk, light);
  int64_t pb, pe;
  int row = -1;
  if (chunk >= 0) {
    pb = chunk_begin[chunk];
    pe = chunk_end[chunk];
  } else {
    row = light_rows[light];
    pb = row_ptr[row];
    pe = row_ptr[row + 1];
  }
  float inv2;
  float rmax = 0.f;  // explicit: this lane's max |rating| (split window guard)
  float* ytyL = reinterpret_cast<float*>(smem + kW1YtyLdsOff);  // implicit light rows
  if constexpr (IMPLICIT) {
    if (chunk < 0) {  // (uniform) the YtY table lands in LDS while the Gram accumulates
#pragma unroll
      for (int j = 0; j < kW1YtyC / 256; ++j)
        __builtin_amdgcn_global_load_lds(ytyC + 256 * j + 4 * lane, ytyL + 256 * j, 16, 0, 0);
    }
    const int e = split_exponent(scal[0] * __builtin_sqrtf(alpha * scal[1]));
    inv2 = ldexpf(1.f, -2 * e);
    gram_accumulate_split<CN, true>(col, val, pb, pe, Y, ld, k, alpha, ldexpf(1.f, e), acc, bt,
                                    npos, reinterpret_cast<int*>(smem));
  } else {
    const int ey = split_exponent(scal[0]), er = split_exponent(scal[1]);
    inv2 = ldexpf(1.f, -2 * ey);
    floatx4 accb[CN];
#pragma unroll
    for (int c = 0; c < CN; ++c) accb[c] = floatx4{0.f, 0.f, 0.f, 0.f};
    if constexpr (kW1Prefetch2)
      gram_accumulate_pre2<FullTiles<CN>>(col, val, pb, pe, Ysp, (uint32_t)kp, zero_row,
                                          ldexpf(1.f, er), (threadIdx.x & 15) * CN, acc, accb,
                                          reinterpret_cast<int*>(smem), rmax);
    else
      gram_accumulate_pre<FullTiles<CN>>(col, val, pb, pe, Ysp, (uint32_t)kp, zero_row,
                                         ldexpf(1.f, er), (threadIdx.x & 15) * CN, acc, accb,
                                         reinterpret_cast<int*>(smem), rmax);
    rhs_from_tiles<FullTiles<CN>>(accb, ldexpf(1.f, -ey - er), bt);
    rmax *= ldexpf(1.f, er);
    if (chunk < 0 && (window_miss(diag_max_lane<CN>(acc), (float)(pe - pb), rmax) ||
                      rank_deficient_illcond<CN>(acc, inv2, pe - pb, k, reg))) {
      rescue_append(rl, row);
      return;
    }
  }
  if (chunk >= 0) {
    float* slot = slots + (int64_t)chunk * kW1Slot;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) slot[(t * 4 + r) * 64 + lane] = acc[t][r] * inv2;
#pragma unroll
    for (int c = 0; c < CN; ++c) slot[(NT * 4 + c) * 64 + lane] = bt[c];
    // explicit: the chunk's scaled max |rating| (launch 2a takes the max over chunks)
    slot[(NT * 4 + CN) * 64 + lane] = IMPLICIT ? (float)npos : rmax;
    return;
  }
  wave_lds_sync();  // the Gram's staging words are reused by the solve (one wave)
  if constexpr (IMPLICIT) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the table landed
  const int64_t n_reg = IMPLICIT ? (int64_t)npos : (pe - pb);
  w1_finish_and_solve<IMPLICIT, kW1NB, IMPLICIT>(acc, inv2, bt, n_reg, IMPLICIT ? ytyL : ytyC,
                                               smem, k, reg,
                                               X + (int64_t)row * ld, ld, row, rl,
                                               IMPLICIT ? kCondMaxImplicit : kCondMax);
}

// ---------------------------------------------------------------------------
// Short explicit rows at 64 < k <= 128: the n x n dual system.
// For a row with n <= 96 ratings r_j on the factor rows y_j (Y_S = n x k):
//   x = (Y_S^T Y_S + lambda n I)^-1 Y_S^T r  =  Y_S^T (Y_S Y_S^T + lambda n I)^-1 r
// (push-through identity (Y^T Y + c I) Y^T = Y^T (Y Y^T + c I); both systems are
// SPD for lambda n > 0).  So x is the solution of Spark's CholeskySolver on the
// k x k normal equations, obtained through an n x n system: for n < k the
// k(k+1)/2-entry Gram and the k^3/3 factorisation become n(n+1)/2 k-dim inner
// products and an n^3/3 one (n = 64, k = 128: 1/2 the Gram, 1/8 the solve).
// Variables: rating j <-> (block c = j % NB, index i = j / NB) — the dim
// permutation of the primal kernels — so w1_solve_x consumes the Gram tiles as
// the MFMAs leave them and pads ratings j >= n the way it pads dims.
//  * Gram G = 2^2ey Y_S Y_S^T on v_mfma_f32_16x16x32_f16 from the split table
//    (hi | lo words of 2^ey Y): MFMA K = dims, 4 k-steps of 32 dims, streamed
//    (step s+1's gathers in flight during step s's MFMAs); operand (c, s) on lane
//    (q, m) = dims 32s + 8q .. +7 of rating m * NB + c; hi.hi + hi.lo + lo.hi per
//    tile per k-step (fp32-grade products, as the primal Gram).
//  * solve: w1_solve_x<NB> (fp32 MFMA tile products), z_j on the lanes of block c.
//  * x = Y_S^T z from the same rows re-gathered (L2-hot): a split word is the f16
//    pair (hi, lo) of one entry, so v_dot2_f32_f16 against (z_hi, z_hi) and
//    (z_lo, z_lo) (z split after a power-of-two scale) accumulates (hi + lo) z in
//    fp32; summed over the 16 lanes of a row group.
// NB = 2 (n <= 32), 4 (n <= 64), 6 (n <= 96): a wave-uniform branch of one kernel.
// 32 < k <= 64 (KP = 64 split words per row): n <= 32 only (NB = 2 against the primal
// NB = 4: a quarter of the k x k Gram tiles, half the block sweeps; for 32 < n <= 64
// the dual system is as large as the primal one).
constexpr int kDualMaxRatings = 96;
constexpr int kDualMaxRatings64 = 32;

// The 8 split words of dims 32s + 8q .. +7 of each operand block's rating.
template <int NB, int KP>
__device__ __forceinline__ void dual_gather_step(uint32_t (&w)[NB][8], const int (&cc)[NB], int s,
                                                 const uint32_t* __restrict__ Ysp) {
  const int q = (threadIdx.x & 63) >> 4;
#pragma unroll
  for (int c = 0; c < NB; ++c) {
    const uint32_t* p = Ysp + (uint64_t)(uint32_t)cc[c] * (uint32_t)KP + 32 * s + 8 * q;
    const uint4 a = *reinterpret_cast<const uint4*>(p);
    const uint4 b = *reinterpret_cast<const uint4*>(p + 4);
    w[c][0] = a.x; w[c][1] = a.y; w[c][2] = a.z; w[c][3] = a.w;
    w[c][4] = b.x; w[c][5] = b.y; w[c][6] = b.z; w[c][7] = b.w;
  }
}

template <int NB, int KP>
__device__ __forceinline__ void dual_row(int row, int n, const int (&cj)[2],
                                         const float (&rj)[2], const uint32_t* __restrict__ Ysp,
                                         int ey, float reg, float* __restrict__ xrow, int ld,
                                         float* __restrict__ lds, int32_t* __restrict__ status,
                                         RescueList rl) {
  constexpr int NT = NB * (NB + 1) / 2;
  constexpr int NS = KP / 32;  // k-steps of 32 dims
  typedef FullTiles<NB> TS;
  const int lane = threadIdx.x & 63, q = lane >> 4, m = lane & 15;
  // operand block c of lane (q, m) is rating j = m * NB + c (held by lane j % 64 in
  // register j / 64 of the staging pair)
  int cc[NB];
  float rc[NB];
#pragma unroll
  for (int c = 0; c < NB; ++c) {
    const int j = m * NB + c;
    const int c0 = __shfl(cj[0], j & 63);
    const float r0 = __shfl(rj[0], j & 63);
    if constexpr (NB * 16 > 64) {
      const int c1 = __shfl(cj[1], j & 63);
      const float r1 = __shfl(rj[1], j & 63);
      cc[c] = j < 64 ? c0 : c1;
      rc[c] = j < 64 ? r0 : r1;
    } else {
      cc[c] = c0;
      rc[c] = r0;
    }
  }
  floatx4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
  // NB <= 4: step s+1's gathers in flight during step s; NB = 6: one step of
  // registers (the two waves per SIMD overlap each other's gathers instead)
  constexpr int NBUF = NB <= 4 ? 2 : 1;
  uint32_t w[NBUF][NB][8];
  dual_gather_step<NB, KP>(w[0], cc, 0, Ysp);
  static_for<NS>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    constexpr int cur = s % NBUF;
    if constexpr (NBUF == 2 && s + 1 < NS)
      dual_gather_step<NB, KP>(w[(s + 1) % NBUF], cc, s + 1, Ysp);
    if constexpr (NBUF == 1 && s > 0) dual_gather_step<NB, KP>(w[0], cc, s, Ysp);
    uint32_t hi[NB][4], lo[NB][4];
#pragma unroll
    for (int c = 0; c < NB; ++c)
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        hi[c][p] = __builtin_amdgcn_perm(w[cur][c][2 * p + 1], w[cur][c][2 * p], 0x05040100u);
        lo[c][p] = __builtin_amdgcn_perm(w[cur][c][2 * p + 1], w[cur][c][2 * p], 0x07060302u);
      }
    static_for<NT>([&](auto ti) {
      constexpr int t = decltype(ti)::value;
      constexpr int a = TS::l1(t), b = TS::l2(t);
      const half8v ha = as_h8(hi[a]), hb = as_h8(hi[b]);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ha, hb, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ha, as_h8(lo[b]), acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_h8(lo[a]), hb, acc[t], 0, 0, 0);
    });
  });
  // split window guard: G_jj = |t_j|^2 <= KP max_d t_jd^2 (ratings are not split here)
  if (window_miss(diag_max_lane<NB>(acc), (float)KP, 0.f)) {
    rescue_append(rl, row);
    return;
  }
  // (2^2ey G + 2^2ey lambda n I) z = 2^2ey r; ratings j >= n: identity rows, rhs 0
  const float inv = ldexpf(1.f, 2 * ey);
  const float lam = (float)((double)reg * (double)n) * inv;
  static_for<NT>([&](auto tc) {
    constexpr int t = decltype(tc)::value;
    constexpr int c1 = TS::l1(t), c2 = TS::l2(t);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      int i, j;
      tile_ij<NB>(c1, c2, r, i, j);
      const bool pad = (i >= n) | (j >= n);
      float v = pad ? 0.f : acc[t][r];
      if constexpr (c1 == c2) v = (i == j) ? (pad ? 1.f : v + lam) : v;
      acc[t][r] = v;
    }
  });
  float bcol[NB], z[NB];
#pragma unroll
  for (int c = 0; c < NB; ++c) bcol[c] = rc[c] * inv;
  const bool ok = w1_solve_x<NB, false>(acc, bcol, lds, n, z);
  if (!ok) {  // re-solved in fp64 (the primal k x k system)
    rescue_append(rl, row);
    return;
  }
  // x = Y_S^T z: z split into f16 hi + lo after a power-of-two scale
  float zm = 0.f;
#pragma unroll
  for (int c = 0; c < NB; ++c) zm = fmaxf(zm, __builtin_fabsf(z[c]));
  const int ez = split_exponent(wave_max(zm));
  const float sz = ldexpf(1.f, ez);
  half2v zh2[NB], zl2[NB];
#pragma unroll
  for (int c = 0; c < NB; ++c) {
    const float t = z[c] * sz;
    const _Float16 h = (_Float16)t;
    const _Float16 l = (_Float16)(t - (float)h);
    zh2[c] = half2v{h, h};
    zl2[c] = half2v{l, l};
  }
  float px[NS][8];
  dual_gather_step<NB, KP>(w[0], cc, 0, Ysp);
  static_for<NS>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    constexpr int cur = s % NBUF;
    if constexpr (NBUF == 2 && s + 1 < NS)
      dual_gather_step<NB, KP>(w[(s + 1) % NBUF], cc, s + 1, Ysp);
    if constexpr (NBUF == 1 && s > 0) dual_gather_step<NB, KP>(w[0], cc, s, Ysp);
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      float a = 0.f;
#pragma unroll
      for (int c = 0; c < NB; ++c) {
        const half2v hl = __builtin_bit_cast(half2v, w[cur][c][t]);
        a = __builtin_amdgcn_fdot2(hl, zh2[c], a, false);
        a = __builtin_amdgcn_fdot2(hl, zl2[c], a, false);
      }
      px[s][t] = reduce_lanes16(a);
    }
  });
  // lane (q, 0) holds dims 32s + 8q .. +7; (2^ey y)(2^ez z) -> x
  const float un = ldexpf(1.f, -ey - ez);
  if (m == 0) {
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int d = 32 * s + 8 * q + 4 * h;
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = ok ? px[s][4 * h + e] * un : 0.f;
        if (d < ld) *reinterpret_cast<float4*>(xrow + d) = make_float4(o[0], o[1], o[2], o[3]);
      }
  }
}

// One wavefront per short light row (the tail of the longest-first light list: every
// row with <= kDualMaxRatings ratings at k in (64, 128], KP = 128; <= kDualMaxRatings64
// at k in (32, 64], KP = 64), explicit, regParam > 0.  (Three waves per SIMD: 27
// spilled registers, configs[3] dual launch 64.8 -> 67.8 ms, profiles/r05/ab_occupancy.jsonl.)
template <int KP>
__global__ __launch_bounds__(64, 2) void gram_solve_dual_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ val, const int32_t* __restrict__ rows, float* __restrict__ X, int ld,
    float reg, int32_t* __restrict__ status, const float* __restrict__ scal,
    const uint32_t* __restrict__ Ysp, int32_t zero_row, RescueList rl) {
  static_assert(KP == 64 || KP == 128, "dual: k_pad 64 or 128");
  constexpr int NMAX = KP == 128 ? kDualMaxRatings : kDualMaxRatings64;
  __shared__ __attribute__((aligned(16))) float lds[W1LdsT<KP == 128 ? 6 : 2>::SIZE];
  const int lane = threadIdx.x & 63;
  const int row = rows[blockIdx.x];
  const int64_t pb = row_ptr[row];
  const int n = (int)(row_ptr[row + 1] - pb);
  const int ey = split_exponent(scal[0]);
  float* xrow = X + (int64_t)row * ld;
  if (n > NMAX) {  // schedule contract broken: report the row, leave it zero
    if (lane == 0) atomicCAS(status, 0, row + 1);
    return;
  }
  // ratings j = lane and j = lane + 64 (missing ones point at the zero row)
  int cj[2];
  float rj[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int j = lane + 64 * h;
    cj[h] = j < n ? col[pb + j] : zero_row;
    rj[h] = j < n ? val[pb + j] : 0.f;
  }
  if constexpr (KP == 64) {
    dual_row<2, 64>(row, n, cj, rj, Ysp, ey, reg, xrow, ld, lds, status, rl);
  } else {
    if (n <= 32)
      dual_row<2, 128>(row, n, cj, rj, Ysp, ey, reg, xrow, ld, lds, status, rl);
    else if (n <= 64)
      dual_row<4, 128>(row, n, cj, rj, Ysp, ey, reg, xrow, ld, lds, status, rl);
    else
      dual_row<6, 128>(row, n, cj, rj, Ysp, ey, reg, xrow, ld, lds, status, rl);
  }
}

// Launch 2 (W1): heavy rows — fp64 sums of the fp32 chunk partials in a fixed
// order (+ YtY in fp64 for implicit), one rounding, then the solve.  Entries are
// reduced 16 at a time (a memory clobber keeps the groups' slot loops apart, so
// only 16 fp64 sums are live).
// Launch 2a: the fp32 chunk slots of every heavy row summed in fp64 (element-wise,
// one thread per slot element; fixed order: four interleaved partial sums),
// the implicit YtY added in fp64, then rounded once to fp32 into the row's first
// slot (each thread reads and writes only its own element: in place is safe).
// Four consecutive elements per thread (16-B loads and stores: the slots are
// 16-B aligned and kW1Slot is a multiple of 4), each with the same four partial
// sums in the same order as one element per thread.
template <bool IMPLICIT>
__global__ __launch_bounds__(256) void heavy_sum_w1_kernel(const int32_t* __restrict__ slot_begin,
                                                           const int32_t* __restrict__ slot_begin2,
                                                           float* __restrict__ slots,
                                                           const double* __restrict__ yty) {
  constexpr int CN = 8, NT = kW1NT, NE = (NT * 4 + CN + 1) * 64;
  static_assert(NE % 4 == 0 && kW1Slot % 4 == 0, "heavy_sum_w1: float4 elements");
  const int h = blockIdx.y;
  const int e = 4 * (blockIdx.x * 256 + threadIdx.x);
  if (e >= NE) return;
  const SlotRange sr = slot_range(slot_begin, slot_begin2, h);
  auto ld4 = [&](int i) -> float4 {
    return *reinterpret_cast<const float4*>(slots + (int64_t)sr.at(i) * kW1Slot + e);
  };
  double a0[4] = {0.0, 0.0, 0.0, 0.0}, a1[4] = {0.0, 0.0, 0.0, 0.0};
  double a2[4] = {0.0, 0.0, 0.0, 0.0}, a3[4] = {0.0, 0.0, 0.0, 0.0};
  auto add = [](double (&a)[4], const float4& x) {
    a[0] += (double)x.x;
    a[1] += (double)x.y;
    a[2] += (double)x.z;
    a[3] += (double)x.w;
  };
  int i = 0;
  for (; i + 4 <= sr.n; i += 4) {
    const float4 x0 = ld4(i), x1 = ld4(i + 1), x2 = ld4(i + 2), x3 = ld4(i + 3);
    add(a0, x0);
    add(a1, x1);
    add(a2, x2);
    add(a3, x3);
  }
  for (; i < sr.n; ++i) add(a0, ld4(i));
  const int ent = e >> 6;  // e .. e + 3 share one entry (64 elements per entry)
  float o[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) o[c] = (float)((a0[c] + a1[c]) + (a2[c] + a3[c]));
  if (!IMPLICIT && ent == NT * 4 + CN) {  // the chunks' scaled max |rating|: max, not sum
    float mx[4] = {0.f, 0.f, 0.f, 0.f};
    for (i = 0; i < sr.n; ++i) {
      const float4 x = ld4(i);
      mx[0] = fmaxf(mx[0], x.x);
      mx[1] = fmaxf(mx[1], x.y);
      mx[2] = fmaxf(mx[2], x.z);
      mx[3] = fmaxf(mx[3], x.w);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) o[c] = mx[c];
  }
  if (IMPLICIT && ent < NT * 4) {
    const int t = ent >> 2, r = ent & 3;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int lane = (e + c) & 63;
      const int ii = (4 * (lane >> 4) + r) * CN + FullTiles<CN>::l1(t);
      const int jj = (lane & 15) * CN + FullTiles<CN>::l2(t);
      const int hi = ii > jj ? ii : jj, lo = ii > jj ? jj : ii;
      o[c] = (float)(((a0[c] + a1[c]) + (a2[c] + a3[c])) + yty[hi * (hi + 1) / 2 + lo]);
    }
  }
  *reinterpret_cast<float4*>(slots + (int64_t)sr.home() * kW1Slot + e) =
      make_float4(o[0], o[1], o[2], o[3]);
}

// Launch 2b: one wavefront per heavy row solves from its summed slot.
template <bool IMPLICIT>
__global__ __launch_bounds__(64, 1) void reduce_solve_w1_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ heavy_rows,
    const int32_t* __restrict__ slot_begin, const int32_t* __restrict__ slot_begin2,
    const float* __restrict__ slots, float* __restrict__ X, int ld, int k, float reg,
    int32_t* __restrict__ status, const float* __restrict__ scal, RescueList rl) {
  constexpr int CN = 8, NT = kW1NT;
  __shared__ __attribute__((aligned(16))) unsigned char smem[SmemBytes<CN>::value];
  const int lane = threadIdx.x & 63;
  const int h = blockIdx.x;
  const int row = heavy_rows[h];
  const float* sl =
      slots + (int64_t)slot_range(slot_begin, slot_begin2, h).home() * kW1Slot + lane;
  floatx4 A[NT];
  float bt[CN];
#pragma unroll
  for (int e = 0; e < NT * 4; ++e) A[e / 4][e % 4] = sl[e * 64];
#pragma unroll
  for (int c = 0; c < CN; ++c) bt[c] = sl[(NT * 4 + c) * 64];
  const float npos_f = sl[(NT * 4 + CN) * 64];
  const int64_t n_reg = IMPLICIT ? (int64_t)npos_f : (row_ptr[row + 1] - row_ptr[row]);
  if constexpr (!IMPLICIT) {  // split window guard over the whole row (npos_f: max |rating|)
    const float s2 = ldexpf(1.f, 2 * split_exponent(scal[0]));
    if (window_miss(diag_max_lane<CN>(A) * s2, (float)n_reg, npos_f)) {
      rescue_append(rl, row);
      return;
    }
  }
  w1_finish_and_solve<false>(A, 1.f, bt, n_reg, nullptr, smem, k, reg, X + (int64_t)row * ld, ld,
                             row, rl, IMPLICIT ? kCondMaxImplicit : kCondMax);
}

// Rescue launch: every row the fp32-grade path did not solve to the 1e-4 bar — its
// operands missed the split window (window_miss), its LDL^T pivots spread beyond
// kCondMax, or a pivot was not positive / the solution not finite — is re-solved with
// Spark's own arithmetic: the normal equations accumulated in fp64 from the fp32 factor
// rows (NormalEquation.add's dspr / daxpy: products of fp32 values are exact in fp64),
// implicit YtY merged in fp64, lambda * numExplicits on the diagonal, and a fp64
// Cholesky (dppsv) of the packed lower triangle in LDS.  A pivot that is not positive
// in fp64 either is Spark's failure: status = row + 1.  One 256-thread workgroup per
// listed row (a few hundred workgroups walk the list; an empty list costs one launch).
constexpr int kRescueThreads = 256;
constexpr int kRescueBatch = 32;  // ratings staged per step

// (i, j), i >= j, of lower-packed entry e (e = i (i + 1) / 2 + j).
__device__ __forceinline__ void packed_ij(int e, int& i, int& j) {
  int r = (int)((sqrt(8.0 * (double)e + 1.0) - 1.0) * 0.5);
  while ((r + 1) * (r + 2) / 2 <= e) ++r;
  while (r * (r + 1) / 2 > e) --r;
  i = r;
  j = e - r * (r + 1) / 2;
}

template <bool IMPLICIT>
__global__ __launch_bounds__(kRescueThreads) void rescue64_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ val, const float* __restrict__ Y, int ld, int k, float reg,
    float alpha, const double* __restrict__ yty, float* __restrict__ X,
    int32_t* __restrict__ status, RescueList rl) {
  constexpr int NPMAX = kMaxRank * (kMaxRank + 1) / 2;
  __shared__ double Ap[NPMAX];  // lower-packed A
  __shared__ double bs[kMaxRank];
  __shared__ float ys[kRescueBatch][kMaxRank + 1];
  __shared__ double wa[kRescueBatch], wb[kRescueBatch];
  __shared__ int npos_s;
  __shared__ int fail_s;
  const int tid = threadIdx.x;
  const int np = k * (k + 1) / 2;
  const unsigned n_app = *rl.cnt;
  const unsigned n_list = n_app < rl.cap ? n_app : rl.cap;
  if (n_app > rl.cap && blockIdx.x == 0 && tid == 0)
    atomicExch(status, -1);  // appended past the list: the phases ran out of order
  for (unsigned it = blockIdx.x; it < n_list; it += gridDim.x) {
    const int row = rl.list[it];
    const int64_t pb = row_ptr[row], pe = row_ptr[row + 1];
    for (int e = tid; e < np; e += kRescueThreads) Ap[e] = IMPLICIT ? yty[e] : 0.0;
    for (int d = tid; d < k; d += kRescueThreads) bs[d] = 0.0;
    if (tid == 0) {
      npos_s = 0;
      fail_s = 0;
    }
    __syncthreads();
    int npos = 0;
    for (int64_t base = pb; base < pe; base += kRescueBatch) {
      const int nb = (int)(pe - base < kRescueBatch ? pe - base : kRescueBatch);
      if (tid < kRescueBatch) {
        const bool v = tid < nb;
        const double r = v ? (double)val[base + tid] : 0.0;
        if (IMPLICIT) {
          const double c1 = (double)alpha * fabs(r);
          wa[tid] = v ? c1 : 0.0;
          wb[tid] = (v && r > 0.0) ? 1.0 + c1 : 0.0;
          npos += (v && r > 0.0) ? 1 : 0;
        } else {
          wa[tid] = v ? 1.0 : 0.0;
          wb[tid] = r;
        }
      }
      for (int x = tid; x < kRescueBatch * k; x += kRescueThreads) {
        const int jr = x / k, d = x - jr * k;
        ys[jr][d] = jr < nb ? Y[(int64_t)col[base + jr] * ld + d] : 0.f;
      }
      __syncthreads();
      for (int e = tid; e < np; e += kRescueThreads) {
        int i, j;
        packed_ij(e, i, j);
        double acc = 0.0;
        for (int jr = 0; jr < nb; ++jr)
          acc = fma(wa[jr], (double)ys[jr][i] * (double)ys[jr][j], acc);
        Ap[e] += acc;
      }
      for (int d = tid; d < k; d += kRescueThreads) {
        double acc = 0.0;
        for (int jr = 0; jr < nb; ++jr) acc = fma(wb[jr], (double)ys[jr][d], acc);
        bs[d] += acc;
      }
      __syncthreads();
    }
    if (IMPLICIT && tid < kRescueBatch) atomicAdd(&npos_s, npos);
    __syncthreads();
    const double lam = (double)reg * (double)(IMPLICIT ? npos_s : (int)(pe - pb));
    for (int d = tid; d < k; d += kRescueThreads) Ap[d * (d + 1) / 2 + d] += lam;
    __syncthreads();
    // Cholesky A = L L^T (right-looking, packed lower, in place)
    for (int jc = 0; jc < k; ++jc) {
      const int dj = jc * (jc + 1) / 2 + jc;
      const double dd = Ap[dj];
      if (!(dd > 0.0)) {  // uniform: every thread reads the same value
        if (tid == 0) fail_s = 1;
        break;
      }
      const double l = sqrt(dd);
      __syncthreads();
      if (tid == 0) Ap[dj] = l;
      for (int i = jc + 1 + tid; i < k; i += kRescueThreads) Ap[i * (i + 1) / 2 + jc] /= l;
      __syncthreads();
      const int m = k - jc - 1;  // trailing block, lower-packed entries (a, c), c <= a
      for (int t = tid; t < m * (m + 1) / 2; t += kRescueThreads) {
        int a, c;
        packed_ij(t, a, c);
        const int ia = jc + 1 + a, ic = jc + 1 + c;
        Ap[ia * (ia + 1) / 2 + ic] -= Ap[ia * (ia + 1) / 2 + jc] * Ap[ic * (ic + 1) / 2 + jc];
      }
      __syncthreads();
    }
    __syncthreads();
    float* xrow = X + (int64_t)row * ld;
    if (fail_s) {
      if (tid == 0) atomicCAS(status, 0, row + 1);  // Spark: dppsv info > 0
      for (int d = tid; d < ld; d += kRescueThreads) xrow[d] = 0.f;
    } else {
      // L y = b (forward), L^T x = y (backward), column-oriented
      for (int jc = 0; jc < k; ++jc) {
        const double yj = bs[jc] / Ap[jc * (jc + 1) / 2 + jc];
        __syncthreads();
        if (tid == 0) bs[jc] = yj;
        for (int i = jc + 1 + tid; i < k; i += kRescueThreads) bs[i] -= Ap[i * (i + 1) / 2 + jc] * yj;
        __syncthreads();
      }
      for (int jc = k - 1; jc >= 0; --jc) {
        const double xj = bs[jc] / Ap[jc * (jc + 1) / 2 + jc];
        __syncthreads();
        if (tid == 0) bs[jc] = xj;
        for (int i = tid; i < jc; i += kRescueThreads) bs[i] -= Ap[jc * (jc + 1) / 2 + i] * xj;
        __syncthreads();
      }
      for (int d = tid; d < ld; d += kRescueThreads) xrow[d] = d < k ? (float)bs[d] : 0.f;
    }
    __syncthreads();  // LDS reused by the next listed row
  }
  // the list is consumed: the last block to finish (every block read the count before
  // its increment) empties it for the next LAUNCH1 of this workspace.  rl.cnt[1] is
  // the finished-block counter (zeroed with the count by the prep, reset here).  No
  // fence: a block's read of the count returned before its increment was issued (the
  // loop bound depends on it), and nothing else in this launch reads what it wrote.
  __syncthreads();
  if (tid == 0) {
    if (atomicAdd(rl.cnt + 1, 1u) == gridDim.x - 1) {
      rl.cnt[0] = 0u;
      rl.cnt[1] = 0u;
    }
  }
}

// K2b: YtY partial Grams over row chunks of Y (unweighted, identity gather), fp64.
template <int CN>
__global__ __launch_bounds__(64, 2) void yty_partial_kernel(const float* __restrict__ Y, int64_t n,
                                                            int ld, int k,
                                                            double* __restrict__ slots) {
  constexpr int NT = Cfg<CN>::NT;
  double a64[NT][4], b64[CN];
  zero_acc<NT, CN, double>(a64, b64);
  int npos = 0;
  const int64_t chunk = yty_chunk(n);
  const int64_t pb = (int64_t)blockIdx.x * chunk;
  const int64_t pe = pb + chunk < n ? pb + chunk : n;
  gram_accumulate<CN, false, true, double>(nullptr, nullptr, pb, pe, Y, ld, k, 0.f, a64, b64,
                                           npos);
  store_slot<NT, CN, double>(slots + (int64_t)blockIdx.x * Cfg<CN>::SLOT, a64, b64, (float)npos);
}

template <int CN>
__global__ __launch_bounds__(64) void yty_reduce_kernel(const double* __restrict__ slots,
                                                        int nslots, double* __restrict__ out) {
  constexpr int NT = Cfg<CN>::NT, NP = Cfg<CN>::NP;
  __shared__ double P[NP];
  double a64[NT][4], b64[CN];
  zero_acc<NT, CN, double>(a64, b64);
  int npos = 0;
  for (int s = 0; s < nslots; ++s) add_slot<NT, CN>(slots + (int64_t)s * Cfg<CN>::SLOT, a64, b64, npos);
  pack_gram<CN, double>(a64, P);
  __syncthreads();
  for (int e = threadIdx.x; e < NP; e += 64) out[e] = P[e];
}

// ---------------------------------------------------------------------------
// K2b at 64 < k <= 128: one workgroup of 4 wavefronts per YtY task, wave R
// accumulating the tiles of WgTiles<R> (10/10/8/8 of the 36 upper tiles).
// ---------------------------------------------------------------------------
constexpr int kWgNB = 8;
constexpr int kWgSub = Slot<10, 4>::SIZE;  // doubles per wave sub-slot (max over roles)
constexpr int kWgSlot = 4 * kWgSub;

template <int R>
__device__ __forceinline__ void wg_yty_partial_task(const float* __restrict__ Y, int64_t n, int ld,
                                                    int k, double* __restrict__ slots) {
  typedef WgTiles<R> TS;
  double a64[TS::N][4], b64[TS::NRA];
  zero_acc<TS::N, TS::NRA, double>(a64, b64);
  int npos = 0;
  const int64_t chunk = yty_chunk(n);
  const int64_t pb = (int64_t)blockIdx.x * chunk;
  const int64_t pe = pb + chunk < n ? pb + chunk : n;
  gram_accumulate<kWgNB, false, true, double, TS>(nullptr, nullptr, pb, pe, Y, ld, k, 0.f, a64,
                                                  b64, npos);
  store_slot<TS::N, TS::NRA, double>(slots + (int64_t)blockIdx.x * kWgSlot + R * kWgSub, a64, b64,
                                     (float)npos);
}

template <int R>
__device__ __forceinline__ void wg_yty_reduce_task(const double* __restrict__ slots, int nslots,
                                                   double* __restrict__ out) {
  typedef WgTiles<R> TS;
  double a64[TS::N][4], b64[TS::NRA];
  zero_acc<TS::N, TS::NRA, double>(a64, b64);
  int npos = 0;
  for (int s = 0; s < nslots; ++s)
    add_slot<TS::N, TS::NRA>(slots + (int64_t)s * kWgSlot + R * kWgSub, a64, b64, npos);
  static_for<TS::N>([&](auto tc) {
    constexpr int t = decltype(tc)::value;
    constexpr int c1 = TS::g1(t), c2 = TS::g2(t);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      int i, j;
      tile_ij<kWgNB>(c1, c2, r, i, j);
      // a diagonal tile holds both (i, j) and (j, i): store the lower one only
      if (c1 < c2 || i >= j) {
        const int hi = i > j ? i : j, lo = i > j ? j : i;
        out[hi * (hi + 1) / 2 + lo] = a64[t][r];
      }
    }
  });
}

// The workgroup kernels: wave index -> role (wave-uniform branch).
#define ALS_WG_ROLES(CALL) \
  do {                                                                    \
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);      \
    if (wv == 0) CALL(0);                                                 \
    else if (wv == 1) CALL(1);                                            \
    else if (wv == 2) CALL(2);                                            \
    else CALL(3);                                                         \
  } while (0)

// Element-wise fp64 sum of the YtY task slots, so the final reduce reads one slot.
// A workgroup owns 64 consecutive elements (one per lane, coalesced) and 16
// wavefronts: wave w sums slots w, w + 16, ... (8 loads in flight per round),
// then wave 0 adds the 16 partials in wave order — a fixed order, so the result
// is deterministic.  (One thread per element over every slot left a few dozen
// workgroups waiting on one load round trip per 4 slots: 43 us at 318 slots.)
constexpr int kSlotSumWaves = 16;
__global__ __launch_bounds__(64 * kSlotSumWaves) void slot_sum_kernel(
    const double* __restrict__ slots, int nslots, int64_t slot_len, double* __restrict__ out) {
  __shared__ double part[kSlotSumWaves][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t e = (int64_t)blockIdx.x * 64 + lane;
  double s = 0.0;
  if (e < slot_len) {
    constexpr int kBatch = 8;
    int i = w;
    for (; i + kSlotSumWaves * (kBatch - 1) < nslots; i += kSlotSumWaves * kBatch) {
      double v[kBatch];
#pragma unroll
      for (int j = 0; j < kBatch; ++j) v[j] = slots[(int64_t)(i + kSlotSumWaves * j) * slot_len + e];
#pragma unroll
      for (int j = 0; j < kBatch; ++j) s += v[j];
    }
    for (; i < nslots; i += kSlotSumWaves) s += slots[(int64_t)i * slot_len + e];
  }
  part[w][lane] = s;
  __syncthreads();
  if (w == 0 && e < slot_len) {
    double t = part[0][lane];
#pragma unroll
    for (int j = 1; j < kSlotSumWaves; ++j) t += part[j][lane];
    out[e] = t;
  }
}

__global__ __launch_bounds__(256, 2) void yty_partial_wg_kernel(const float* __restrict__ Y,
                                                                int64_t n, int ld, int k,
                                                                double* __restrict__ slots) {
#define CALL(R) wg_yty_partial_task<R>(Y, n, ld, k, slots)
  ALS_WG_ROLES(CALL);
#undef CALL
}

__global__ __launch_bounds__(256) void yty_reduce_wg_kernel(const double* __restrict__ slots,
                                                            int nslots, double* __restrict__ out) {
#define CALL(R) wg_yty_reduce_task<R>(slots, nslots, out)
  ALS_WG_ROLES(CALL);
#undef CALL
}
#undef ALS_WG_ROLES

}  // namespace als

using namespace als;

extern "C" {

int32_t als_k_pad(int32_t k) { return 16 * cn_for_k(k); }

}  // extern "C"

static size_t slot_doubles(int k) {  // partial slot of one heavy-row chunk (solve)
  switch (cn_for_k(k)) {
    case 1: return (Cfg<1>::SLOT + 1) / 2;  // fp32 chunk partials
    case 2: return (Cfg<2>::SLOT + 1) / 2;
    case 4: return (Cfg<4>::SLOT + 1) / 2;
    default: return (size_t)(kW1Slot + 1) / 2;  // W1 stores fp32 partials
  }
}

static size_t yty_slot_doubles(int k) {  // partial slot of one YtY task (fp64 slots)
  switch (cn_for_k(k)) {
    case 1: return Cfg<1>::SLOT;
    case 2: return Cfg<2>::SLOT;
    case 4: return Cfg<4>::SLOT;
    default: return (size_t)kWgSlot;
  }
}

extern "C" {

static size_t ytyc_bytes(int32_t k) {  // C-layout fp32 YtY table of the W1 path
  return cn_for_k(k) == 8 ? align_up(sizeof(float) * kW1YtyC) : 0;
}

static size_t solve_table_bytes(int32_t k, int64_t n_src) {
  return align_up(sizeof(uint32_t) * (size_t)als_k_pad(k) * (size_t)((n_src > 0 ? n_src : 0) + 1));
}

static size_t slot_bytes(int32_t k, int32_t n_chunks) {
  return align_up(sizeof(double) * slot_doubles(k) * (size_t)(n_chunks > 0 ? n_chunks : 0));
}

size_t als_solve_workspace_bytes(int32_t k, int32_t n_chunks, int64_t n_src, int32_t n_rows) {
  // From the front: 256 B of scale words (max |Y_src|, max |rating|, rescue count) |
  // C-layout YtY (W1 implicit) | partial slots of the heavy-row chunks (n_chunks,
  // counted from slot 0: chunk_slot0 + the call's chunks).
  // From the back: the split table ((n_src + 1) x k_pad words, explicit), ending at
  // the workspace's end (256-B aligned; + 256 B of slack for that alignment), and
  // right below it the rescue list (n_rows).  Calls
  // that share one PREP (row chunks of a half-sweep: same Y_src, any n_chunks / n_rows)
  // find the table at the same place, and the two calls of a two-segment half-sweep
  // (different n_src) find the early partial slots at the same place.
  return 256 + ytyc_bytes(k) + slot_bytes(k, n_chunks) +
         align_up(sizeof(int32_t) * (size_t)(n_rows > 0 ? n_rows : 0)) +
         solve_table_bytes(k, n_src) + 256;
}

int als_solve_half(const int64_t* row_ptr, const int32_t* col, const float* val,
                   const int32_t* light_rows, int32_t n_light, int32_t n_light_primal,
                   const int32_t* heavy_rows,
                   const int32_t* heavy_slot_begin, int32_t n_heavy, const int32_t* chunk_row,
                   const int64_t* chunk_begin, const int64_t* chunk_end, int32_t n_chunks,
                   const int32_t* heavy_slot_begin2, int32_t chunk_slot0,
                   const float* Y_src, int64_t n_src, float* X_dst, int32_t ld, int32_t k,
                   float reg, int implicit, float alpha, const double* yty_packed,
                   int32_t* status_dev, void* ws, size_t ws_bytes, int phases, void* stream) {
  ALS_REQUIRE(k >= 1 && k <= kMaxRank, ALS_EUNSUPPORTED, "als_solve_half: rank %d not in [1, %d]",
              k, kMaxRank);
  ALS_REQUIRE(ld >= k && ld % 4 == 0, ALS_EINVAL, "als_solve_half: ld=%d must be >= k and %%4==0",
              ld);
  ALS_REQUIRE(n_light >= 0 && n_heavy >= 0 && n_chunks >= 0, ALS_EINVAL,
              "als_solve_half: negative counts");
  ALS_REQUIRE(n_light_primal >= 0 && n_light_primal <= n_light, ALS_EINVAL,
              "als_solve_half: n_light_primal %d not in [0, n_light=%d]", n_light_primal, n_light);
  ALS_REQUIRE(n_light_primal == n_light || (!implicit && k > 32 && reg > 0.f), ALS_EINVAL,
              "als_solve_half: the dual path (light rows past n_light_primal) is for explicit "
              "feedback at rank 33-128 with regParam > 0 only");
  ALS_REQUIRE(Y_src && X_dst && row_ptr && status_dev, ALS_EINVAL, "als_solve_half: null pointer");
  ALS_REQUIRE(!implicit || yty_packed, ALS_EINVAL, "als_solve_half: implicit needs yty_packed");
  ALS_REQUIRE(reg >= 0.f && alpha >= 0.f, ALS_EINVAL, "als_solve_half: reg/alpha must be >= 0");
  ALS_REQUIRE((reinterpret_cast<uintptr_t>(Y_src) & 15) == 0, ALS_EINVAL,
              "als_solve_half: Y_src must be 16-byte aligned");
  ALS_REQUIRE((reinterpret_cast<uintptr_t>(val) & 15) == 0, ALS_EINVAL,
              "als_solve_half: val must be 16-byte aligned");
  ALS_REQUIRE(n_src >= 0 && n_src < (int64_t(1) << 31), ALS_EINVAL,
              "als_solve_half: n_src %lld not in [0, 2^31)", (long long)n_src);
  const int32_t n_rows = n_light + n_heavy;
  ALS_REQUIRE(chunk_slot0 >= 0 && (int64_t)chunk_slot0 + n_chunks < (int64_t(1) << 31),
              ALS_EINVAL, "als_solve_half: chunk_slot0 %d out of range", chunk_slot0);
  const int32_t n_slots = chunk_slot0 + n_chunks;  // slot region: [0, n_slots)
  ALS_REQUIRE(ws_bytes >= als_solve_workspace_bytes(k, n_slots, n_src, n_rows), ALS_EWORKSPACE,
              "als_solve_half: workspace %zu < %zu", ws_bytes,
              als_solve_workspace_bytes(k, n_slots, n_src, n_rows));
  ALS_REQUIRE(phases >= 1 && phases <= ALS_PHASE_ALL, ALS_EINVAL,
              "als_solve_half: phases must be in [1, %d]", ALS_PHASE_ALL);
  ALS_REQUIRE((reinterpret_cast<uintptr_t>(ws) & 15) == 0, ALS_EINVAL,
              "als_solve_half: workspace must be 16-byte aligned");
  hipStream_t st = as_stream(stream);
  // scale words (max |Y_src|, max |rating|), the split table, the partial slots
  unsigned* scal_u = static_cast<unsigned*>(ws);
  const float* scal = reinterpret_cast<const float*>(scal_u);
  float* ytyC = reinterpret_cast<float*>(static_cast<char*>(ws) + 256);
  double* slots = reinterpret_cast<double*>(static_cast<char*>(ws) + 256 + ytyc_bytes(k));
  uint32_t* Ysp = reinterpret_cast<uint32_t*>(
      static_cast<char*>(ws) + ((ws_bytes - solve_table_bytes(k, n_src)) & ~(size_t)255));
  // the rescue list right below the split table (not after this call's slots: blocks
  // sharing one workspace with disjoint slot ranges must not see one call's list land
  // on another block's partial slots; the size check keeps it above every slot)
  int32_t* rescue_list = reinterpret_cast<int32_t*>(
      reinterpret_cast<char*>(Ysp) - align_up(sizeof(int32_t) * (size_t)(n_rows > 0 ? n_rows : 0)));
  unsigned* rescue_cnt = scal_u + 2;
  const RescueList rl{rescue_cnt, rescue_list, (unsigned)(n_light + n_heavy)};
  // the rescue list (count at scale word 2, the rescue launch's finished-block counter
  // at word 3) starts empty at each Y prep (cleared by the prep's absmax launch: a fresh
  // workspace holds garbage) and is emptied by the RESCUE launch that consumes it, so the
  // next row chunk of a half-sweep that shares one prep starts empty too
  if ((phases & ALS_PHASE_PREP) && n_src * (int64_t)ld == 0)
    ALS_HIP(hipMemsetAsync(rescue_cnt, 0, 2 * sizeof(unsigned), st));
  const int cn = cn_for_k(k);
  const int kp = als_k_pad(k);
  const int zero_row = (int)n_src;
  if (phases & ALS_PHASE_PREP) {  // Y_src prep: max |Y_src|, split table (explicit) / YtY table (W1 implicit)
    ALS_HIP(hipMemsetAsync(scal_u, 0, sizeof(unsigned), st));
    if (implicit && cn == 8) {
      yty_ctab_kernel<<<1, 64, 0, st>>>(yty_packed, ytyC);
      ALS_LAUNCH_CHECK();
    }
    const int64_t ny = n_src * (int64_t)ld;
    if (ny > 0) {
      // 256 workgroups (one atomic each on the scale word; 1024 serialised there)
      const int gy = (int)std::min<int64_t>(256, (ny / 4 + 255) / 256 + 1);
      absmax_kernel<<<gy, 256, 0, st>>>(Y_src, ny, scal_u, rescue_cnt);
      ALS_LAUNCH_CHECK();
    }
    if (!implicit) {
      const int kp4_shift = __builtin_ctz(kp / 4);
      const int64_t total = (n_src + 1) << kp4_shift;
      const int gt = (int)std::min<int64_t>(4096, (total + 255) / 256);
      split_table_kernel<<<gt, 256, 0, st>>>(Y_src, n_src, ld, k, kp4_shift, scal,
                                             reinterpret_cast<uint4*>(Ysp));
      ALS_LAUNCH_CHECK();
    }
  }
  if (phases & ALS_PHASE_RSCALE) {  // rating scale of this block: max |rating|
    ALS_HIP(hipMemsetAsync(scal_u + 1, 0, sizeof(unsigned), st));
    if (n_light + n_heavy > 0) {
      ALS_REQUIRE(val != nullptr, ALS_EINVAL, "als_solve_half: null val");
      // every row is light or heavy: the block's ratings are val[0, row_ptr[n_light + n_heavy])
      absmax_csr_kernel<<<256, 256, 0, st>>>(row_ptr, n_light + n_heavy, val, scal_u + 1);
      ALS_LAUNCH_CHECK();
    }
  }
  const unsigned g1 = (phases & ALS_PHASE_LAUNCH1) ? (unsigned)(n_chunks + n_light_primal) : 0u;
  const unsigned gd = (phases & ALS_PHASE_DUAL) ? (unsigned)(n_light - n_light_primal) : 0u;
  const unsigned g2 = (phases & ALS_PHASE_LAUNCH2) ? (unsigned)n_heavy : 0u;
  const bool rescue = (phases & ALS_PHASE_RESCUE) && n_rows > 0;
#define ALS_SOLVE_LAUNCH(CN, IMP)                                                                 \
  do {                                                                                            \
    float* slots_f = reinterpret_cast<float*>(slots);                                             \
    if (g1)                                                                                       \
      gram_solve_kernel<CN, IMP><<<g1, 64, 0, st>>>(row_ptr, col, val, light_rows, chunk_row,     \
                                                    chunk_begin, chunk_end, n_chunks,             \
                                                    n_light_primal, Y_src, X_dst, ld, k, reg,     \
                                                    alpha, yty_packed,                            \
                                                    slots_f + (size_t)chunk_slot0 * Cfg<CN>::SLOT, \
                                                    status_dev, scal,                             \
                                                    Ysp, kp, zero_row, rl);  \
    ALS_LAUNCH_CHECK();                                                                           \
    if (gd && CN == 4 && !IMP) {                                                                  \
      gram_solve_dual_kernel<64><<<gd, 64, 0, st>>>(row_ptr, col, val,                            \
                                                    light_rows + n_light_primal, X_dst, ld, reg,  \
                                                    status_dev, scal, Ysp, zero_row, rl);          \
      ALS_LAUNCH_CHECK();                                                                         \
    }                                                                                             \
    if (g2) {                                                                                     \
      heavy_sum_f64_kernel<Cfg<CN>::SLOT, IMP>                                                    \
          <<<dim3((Cfg<CN>::SLOT + 255) / 256, g2), 256, 0, st>>>(heavy_slot_begin,               \
                                                                  heavy_slot_begin2, slots_f);     \
      ALS_LAUNCH_CHECK();                                                                         \
      reduce_solve_kernel<CN, IMP><<<g2, 64, 0, st>>>(row_ptr, col, val, Y_src, alpha,            \
                                                      heavy_rows, heavy_slot_begin,               \
                                                      heavy_slot_begin2,                          \
                                                      slots_f, X_dst, ld, k, reg, yty_packed,     \
                                                      status_dev, scal, rl); \
    }                                                                                             \
    ALS_LAUNCH_CHECK();                                                                           \
    if (rescue) {                                                                                 \
      rescue64_kernel<IMP><<<kRescueGrid, kRescueThreads, 0, st>>>(                               \
          row_ptr, col, val, Y_src, ld, k, reg, alpha, yty_packed, X_dst, status_dev, rl);        \
      ALS_LAUNCH_CHECK();                                                                         \
    }                                                                                             \
  } while (0)
#define ALS_SOLVE_W1_LAUNCH(IMP)                                                                  \
  do {                                                                                            \
    float* slots_f = reinterpret_cast<float*>(slots);                                             \
    if (g1)                                                                                       \
      gram_solve_w1_kernel<IMP><<<g1, 64, 0, st>>>(row_ptr, col, val, light_rows, chunk_begin,    \
                                                   chunk_end, n_chunks, n_light_primal, Y_src,    \
                                                   X_dst, ld, k, reg, alpha, ytyC,                \
                                                   slots_f + (size_t)chunk_slot0 * kW1Slot,       \
                                                   status_dev, scal, Ysp, kp, zero_row,           \
                                                   rl);                      \
    ALS_LAUNCH_CHECK();                                                                           \
    if (gd) {                                                                                     \
      gram_solve_dual_kernel<128><<<gd, 64, 0, st>>>(row_ptr, col, val,                           \
                                                     light_rows + n_light_primal, X_dst, ld, reg, \
                                                     status_dev, scal, Ysp, zero_row, rl);         \
      ALS_LAUNCH_CHECK();                                                                         \
    }                                                                                             \
    if (g2) {                                                                                     \
      heavy_sum_w1_kernel<IMP><<<dim3((kW1Slot / 4 + 255) / 256, g2), 256, 0, st>>>(                 \
          heavy_slot_begin, heavy_slot_begin2, slots_f, yty_packed);                              \
      ALS_LAUNCH_CHECK();                                                                         \
      reduce_solve_w1_kernel<IMP><<<g2, 64, 0, st>>>(row_ptr, heavy_rows, heavy_slot_begin,      \
                                                     heavy_slot_begin2, slots_f, X_dst, ld, k,    \
                                                     reg, status_dev,                             \
                                                     scal, rl);              \
    }                                                                                             \
    ALS_LAUNCH_CHECK();                                                                           \
    if (rescue) {                                                                                 \
      rescue64_kernel<IMP><<<kRescueGrid, kRescueThreads, 0, st>>>(                               \
          row_ptr, col, val, Y_src, ld, k, reg, alpha, yty_packed, X_dst, status_dev, rl);        \
      ALS_LAUNCH_CHECK();                                                                         \
    }                                                                                             \
  } while (0)
  if (implicit) {
    if (cn == 1) ALS_SOLVE_LAUNCH(1, true);
    else if (cn == 2) ALS_SOLVE_LAUNCH(2, true);
    else if (cn == 4) ALS_SOLVE_LAUNCH(4, true);
    else ALS_SOLVE_W1_LAUNCH(true);
  } else {
    if (cn == 1) ALS_SOLVE_LAUNCH(1, false);
    else if (cn == 2) ALS_SOLVE_LAUNCH(2, false);
    else if (cn == 4) ALS_SOLVE_LAUNCH(4, false);
    else ALS_SOLVE_W1_LAUNCH(false);
  }
#undef ALS_SOLVE_W1_LAUNCH
#undef ALS_SOLVE_LAUNCH
  return ALS_OK;
}

size_t als_yty_workspace_bytes(int64_t n, int32_t k) {
  const int64_t nslots = n > 0 ? (n + yty_chunk(n) - 1) / yty_chunk(n) : 1;
  // task slots + their element-wise sum
  return align_up(sizeof(double) * yty_slot_doubles(k) * (size_t)(nslots + 1)) + 256;
}

int als_yty(const float* Y, int64_t n, int32_t ld, int32_t k, double* yty_packed_out, void* ws,
            size_t ws_bytes, void* stream) {
  ALS_REQUIRE(k >= 1 && k <= kMaxRank, ALS_EUNSUPPORTED, "als_yty: rank %d not in [1, %d]", k,
              kMaxRank);
  ALS_REQUIRE(ld >= k && ld % 4 == 0, ALS_EINVAL, "als_yty: bad ld");
  ALS_REQUIRE(n >= 0 && yty_packed_out && (n == 0 || Y), ALS_EINVAL, "als_yty: bad args");
  ALS_REQUIRE(n < (int64_t(1) << 31), ALS_EINVAL, "als_yty: n >= 2^31");
  ALS_REQUIRE(ws_bytes >= als_yty_workspace_bytes(n, k), ALS_EWORKSPACE,
              "als_yty: workspace too small");
  hipStream_t st = as_stream(stream);
  double* slots = static_cast<double*>(ws);
  const int nslots = n > 0 ? (int)((n + yty_chunk(n) - 1) / yty_chunk(n)) : 0;
  const int cn = cn_for_k(k);
  if (nslots == 0) {
    const int kp = 16 * cn;
    ALS_HIP(hipMemsetAsync(yty_packed_out, 0, sizeof(double) * kp * (kp + 1) / 2, st));
    return ALS_OK;
  }
  const int64_t slen = (int64_t)yty_slot_doubles(k);
  double* ssum = slots + (int64_t)nslots * slen;
  auto sum_slots = [&]() -> int {
    slot_sum_kernel<<<(unsigned)((slen + 63) / 64), 64 * kSlotSumWaves, 0, st>>>(slots, nslots, slen,
                                                                               ssum);
    ALS_LAUNCH_CHECK();
    return ALS_OK;
  };
#define ALS_YTY_LAUNCH(CN)                                                                    \
  do {                                                                                        \
    yty_partial_kernel<CN><<<nslots, 64, 0, st>>>(Y, n, ld, k, slots);                        \
    ALS_LAUNCH_CHECK();                                                                       \
    if (sum_slots() != ALS_OK) return ALS_EDEVICE;                                            \
    yty_reduce_kernel<CN><<<1, 64, 0, st>>>(ssum, 1, yty_packed_out);                         \
    ALS_LAUNCH_CHECK();                                                                       \
  } while (0)
  if (cn == 1) ALS_YTY_LAUNCH(1);
  else if (cn == 2) ALS_YTY_LAUNCH(2);
  else if (cn == 4) ALS_YTY_LAUNCH(4);
  else {
    yty_partial_wg_kernel<<<nslots, 256, 0, st>>>(Y, n, ld, k, slots);
    ALS_LAUNCH_CHECK();
    if (sum_slots() != ALS_OK) return ALS_EDEVICE;
    yty_reduce_wg_kernel<<<1, 256, 0, st>>>(ssum, 1, yty_packed_out);
    ALS_LAUNCH_CHECK();
  }
#undef ALS_YTY_LAUNCH
  return ALS_OK;
}

}  // extern "C"
