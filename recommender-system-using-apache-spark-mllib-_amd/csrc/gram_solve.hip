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
//  * One wavefront per task.  A task is a whole "light" row (<= chunk ratings)
//    or one chunk of a heavy row.  Rows arrive longest-first (LPT schedule).
//  * Gram on the matrix cores: v_mfma_f32_16x16x4_f32 (exact fp32 products,
//    k-ordered fp32 fma accumulation).  The MFMA's K dimension is the rating
//    index: 4 ratings per instruction, lane (q = lane>>4, m = lane&15) holds
//    factor dims m*CN .. m*CN+CN-1 of rating q, loaded straight from HBM /
//    Infinity Cache as one float4 (a whole 256-B row per 16 lanes), so the
//    gather needs no LDS staging.  With that dim permutation the k x k Gram is
//    CN x CN tiles of 16x16; only the CN(CN+1)/2 upper tiles are computed
//    (the matrix is symmetric, as Spark's packed dspr exploits).
//  * fp32 accumulators are flushed into fp64 registers every 64 ratings, so
//    the Gram error is that of 64-term fp32 sums, independent of row length;
//    across blocks and across chunks accumulation is fp64 like Spark's.
//  * The solve never leaves the CU: the regularised Gram is packed (lower) into LDS
//    (lambda * n on the diagonal, Spark's ALS-WR weighting, added in fp64), then
//    factored by a row-per-lane LDL^T with the right-hand side carried
//    as an augmented column, followed by a column-sweep back substitution.
#include "als_common.h"

#include <utility>

namespace als {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kYtyChunk = 8192;      // src rows per YtY task
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
// Block LDL^T on the matrix cores.
//
// The regularised Gram arrives as fp32 16x16 tiles in the MFMA C layout
// (A[t] = tile (I, J), I <= J; dims permuted so that block I holds the dims
// d = 16-index * CN + I).  Any symmetric permutation is a valid pivot order, so
// the matrix is factored as A = U^T D U (U unit upper) in that block order:
//   for K: factor B_KK = U_KK^T D_K U_KK and forward-solve the rhs block
//                                                    (16x16, row per lane, v_readlane broadcasts)
//          W_KJ = U_KK^-T B_KJ, U_KJ = D_K^-1 W_KJ     (TRSM, one lane per column)
//          B_IJ -= U_KI^T W_KJ   for K < I <= J        (v_mfma_f32_16x16x4_f32, 4 per tile)
//          b_J  -= U_KJ^T z_K                          (TRSM lanes)
// then a block back substitution x_K = U_KK^-1 (D_K^-1 z_K - sum_J U_KJ x_J).
// The O(k^3) trailing work runs on the MFMA pipe; the VALU keeps only the
// 16-wide diagonal factorisations and TRSMs.
// LDS (floats): U tiles NT*256 (diagonal slots: column-major L_K) |
// stage/W NB*320 | D, b, z, x 4*16*NB.
// ---------------------------------------------------------------------------
template <int CN>
struct TileLds {
  static constexpr int NB = CN, NT = CN * (CN + 1) / 2;
  static constexpr int U = 0, S = NT * 256, D = S + NB * 320, B = D + 16 * NB,
                       Z = B + 16 * NB, X = Z + 16 * NB, SIZE = X + 16 * NB;
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

template <int CN>
__device__ __forceinline__ bool tile_ldl_solve(floatx4 (&A)[Cfg<CN>::NT], const float (&bq)[CN],
                                               float* __restrict__ lds, int k,
                                               float* __restrict__ xrow, int ld) {
  typedef TileLds<CN> Lo;
  constexpr int NB = CN;
  const int lane = threadIdx.x & 63, q = lane >> 4, m = lane & 15;
  const int i = lane & 15;  // row owned in the 16-wide steps (lanes >= 16 mirror)
  float* Ust = lds + Lo::U;
  float* St = lds + Lo::S;
  float* Dv = lds + Lo::D;
  float* bv = lds + Lo::B;
  float* zv = lds + Lo::Z;
  float* xv = lds + Lo::X;
  if (q == 0) {
#pragma unroll
    for (int c = 0; c < CN; ++c) bv[c * 16 + m] = bq[c];
  }
  bool ok = true;
#pragma unroll
  for (int K = 0; K < NB; ++K) {
    // (a) stage block row K transposed: St[J-K][j][k] (row stride 20 floats)
#pragma unroll
    for (int J = K; J < NB; ++J) {
      const floatx4 v = A[tile_index(NB, K, J)];
      *reinterpret_cast<float4*>(St + (J - K) * 320 + m * 20 + 4 * q) =
          make_float4(v[0], v[1], v[2], v[3]);
    }
    __syncthreads();
    // (b) LDL^T of the diagonal block with the rhs block as augmented column.
    float a[16];
#pragma unroll
    for (int c4 = 0; c4 < 4; ++c4) {
      const float4 v = *reinterpret_cast<const float4*>(St + i * 20 + 4 * c4);
      a[4 * c4] = v.x; a[4 * c4 + 1] = v.y; a[4 * c4 + 2] = v.z; a[4 * c4 + 3] = v.w;
    }
    float bb = bv[K * 16 + i];
    float myd = 1.f;
#pragma unroll
    for (int p = 0; p < 16; ++p) {
      const float d = readlane_t(a[p], p);
      ok = ok && (d > 0.f);
      float u[16];
#pragma unroll
      for (int j = p + 1; j < 16; ++j) u[j] = readlane_t(a[p], j);  // A'[j][p]
      const float bp = readlane_t(bb, p);
      const float l = a[p] * rcp_t(d);                                 // L[i][p]
#pragma unroll
      for (int j = p + 1; j < 16; ++j) a[j] = fmaf(-l, u[j], a[j]);
      if (i > p) bb = fmaf(-l, bp, bb);
      a[p] = l;
      if (i == p) myd = d;
    }
    float* Lt = Ust + 256 * tile_index(NB, K, K);  // Lt[c*16 + r] = L_K[r][c]
    if (lane < 16) {
      Dv[K * 16 + i] = myd;
      zv[K * 16 + i] = bb;
#pragma unroll
      for (int c = 0; c < 16; ++c) Lt[c * 16 + i] = (c < i) ? a[c] : 0.f;
    }
    __syncthreads();
    if (K + 1 < NB) {
      // (c) TRSM: lane t < 16*(NB-1-K) owns column (t&15) of block J = K+1+(t>>4).
      const int ncol = 16 * (NB - 1 - K);
      const int Jl = K + 1 + (lane >> 4);
      const bool is_col = lane < ncol;
      float w[16];
      {
        const float* src = St + (is_col ? (Jl - K) : 1) * 320 + i * 20;
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) {
          const float4 v = *reinterpret_cast<const float4*>(src + 4 * c4);
          w[4 * c4] = v.x; w[4 * c4 + 1] = v.y; w[4 * c4 + 2] = v.z; w[4 * c4 + 3] = v.w;
        }
      }
#pragma unroll
      for (int c = 0; c < 15; ++c) {
        float lc[16];
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) {
          const float4 v = *reinterpret_cast<const float4*>(Lt + c * 16 + 4 * c4);
          lc[4 * c4] = v.x; lc[4 * c4 + 1] = v.y; lc[4 * c4 + 2] = v.z; lc[4 * c4 + 3] = v.w;
        }
#pragma unroll
        for (int p = c + 1; p < 16; ++p) w[p] = fmaf(-lc[p], w[c], w[p]);
      }
      __syncthreads();  // all stage reads done before W overwrites the stage
      if (is_col) {
        float* Wd = St + (Jl - K - 1) * 256 + i;
        float* Ud = Ust + 256 * tile_index(NB, K, Jl) + i;
        float t = 0.f;
#pragma unroll
        for (int c = 0; c < 16; ++c) {
          const float uc = w[c] * rcp_t(Dv[K * 16 + c]);
          Wd[c * 16] = w[c];
          Ud[c * 16] = uc;
          t = fmaf(uc, zv[K * 16 + c], t);
        }
        bv[Jl * 16 + i] -= t;  // rhs trailing update b_J -= U_KJ^T z_K
      }
      __syncthreads();
      // (d) trailing update on the matrix cores
#pragma unroll
      for (int I = K + 1; I < NB; ++I) {
        float ua[4];
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
          ua[s4] = -Ust[256 * tile_index(NB, K, I) + (4 * s4 + q) * 16 + m];
#pragma unroll
        for (int J = I; J < NB; ++J) {
          floatx4 acc = A[tile_index(NB, I, J)];
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4)
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(
                ua[s4], St[(J - K - 1) * 256 + (4 * s4 + q) * 16 + m], acc, 0, 0, 0);
          A[tile_index(NB, I, J)] = acc;
        }
      }
      __syncthreads();
    }
  }
  // (e) block back substitution: x_K = U_KK^-1 (D_K^-1 z_K - sum_{J>K} U_KJ x_J)
#pragma unroll
  for (int K = NB - 1; K >= 0; --K) {
    float v = zv[K * 16 + i] * rcp_t(Dv[K * 16 + i]);
#pragma unroll
    for (int J = K + 1; J < NB; ++J) {
      const float* Ur = Ust + 256 * tile_index(NB, K, J) + i * 16;
#pragma unroll
      for (int j = 0; j < 16; ++j) v = fmaf(-Ur[j], xv[J * 16 + j], v);
    }
    const float* Lr = Ust + 256 * tile_index(NB, K, K) + i * 16;  // U_KK[i][j] = L_K[j][i]
    float ur[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) ur[j] = Lr[j];
    float x = 0.f;
#pragma unroll
    for (int j = 15; j >= 0; --j) {
      const float xj = readlane_t(v, j);
      if (i == j) x = xj;
      if (i < j) v = fmaf(-ur[j], xj, v);
    }
    if (lane < 16) xv[K * 16 + i] = x;
    __syncthreads();
  }
  // (f) un-permute: dim d = i*CN + K  <->  xv[K*16 + i]
  for (int d = lane; d < ld; d += 64) {
    const float x = d < 16 * CN ? xv[(d % CN) * 16 + d / CN] : 0.f;
    xrow[d] = (d < k && ok) ? x : 0.f;
  }
  return ok;
}

template <int CN>
struct SmemBytes {
  static constexpr int value = (int)sizeof(float) * TileLds<CN>::SIZE;
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
                                                 int32_t* __restrict__ status) {
  constexpr int NT = Cfg<CN>::NT;
  float bq[CN];
#pragma unroll
  for (int c = 0; c < CN; ++c) {
    AccT v = bt[c];
    v += shfl_xor_t(v, 16);
    v += shfl_xor_t(v, 32);
    bq[c] = (float)v;
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
      }
      ++tt;
    }
  }
  regularise_f32<CN>(A, (float)((double)reg * (double)n_reg), k);
  const bool ok = tile_ldl_solve<CN>(A, bq, reinterpret_cast<float*>(smem), k, xrow, ld);
  if (!ok && (threadIdx.x & 63) == 0) atomicCAS(status, 0, row + 1);
}

// Partial-sum slot of one task: N tiles x 4 accumulator rows, NRA rhs values and
// the positive-rating count, each as 64 lane-contiguous doubles.
template <int N, int NRA>
struct Slot {
  static constexpr int SIZE = (N * 4 + NRA + 1) * 64;
};

template <int N, int NRA, class AccT>
__device__ __forceinline__ void store_slot(double* __restrict__ slot, const AccT (&tot)[N][4],
                                           const AccT (&bt)[NRA], int npos) {
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

template <int N, int NRA, class AccT>
__device__ __forceinline__ void zero_acc(AccT (&tot)[N][4], AccT (&bt)[NRA]) {
#pragma unroll
  for (int t = 0; t < N; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) tot[t][r] = AccT(0);
#pragma unroll
  for (int c = 0; c < NRA; ++c) bt[c] = AccT(0);
}

// Launch 1 of a half-sweep: heavy-row chunks (-> fp64 partial slots) first,
// then whole light rows (Gram + solve fused, A never leaves the CU).
// Per-task Gram sums in fp32 (<= 2048 ratings: 64-rating exact-product MFMA
// blocks summed in fp32), cross-chunk sums of heavy rows in fp64.
template <int CN, bool IMPLICIT>
__global__ __launch_bounds__(64, 2) void gram_solve_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ val, const int32_t* __restrict__ light_rows,
    const int32_t* __restrict__ chunk_row, const int64_t* __restrict__ chunk_begin,
    const int64_t* __restrict__ chunk_end, int32_t n_chunks, const float* __restrict__ Y,
    float* __restrict__ X, int ld, int k, float reg, float alpha,
    const double* __restrict__ yty, double* __restrict__ slots, int32_t* __restrict__ status) {
  constexpr int NT = Cfg<CN>::NT;
  typedef float AccT;
  __shared__ __attribute__((aligned(16))) unsigned char smem[SmemBytes<CN>::value];
  const int task = blockIdx.x;
  AccT tot[NT][4], bt[CN];
  zero_acc<NT, CN, AccT>(tot, bt);
  int npos = 0;
  if (task < n_chunks) {
    gram_accumulate<CN, IMPLICIT, false, AccT>(col, val, chunk_begin[task], chunk_end[task], Y,
                                               ld, k, alpha, tot, bt, npos);
    store_slot<NT, CN, AccT>(slots + (int64_t)task * Cfg<CN>::SLOT, tot, bt, npos);
    return;
  }
  const int row = light_rows[task - n_chunks];
  const int64_t pb = row_ptr[row], pe = row_ptr[row + 1];
  gram_accumulate<CN, IMPLICIT, false, AccT>(col, val, pb, pe, Y, ld, k, alpha, tot, bt, npos);
  const int64_t n_reg = IMPLICIT ? (int64_t)npos : (pe - pb);
  finish_and_solve<CN, IMPLICIT, AccT>(tot, bt, n_reg, smem, k, reg, yty, X + (int64_t)row * ld,
                                       ld, row, status);
}

// Launch 2: heavy rows — sum their chunk slots in a fixed order (fp64), then solve.
template <int CN, bool IMPLICIT>
__global__ __launch_bounds__(64, 2) void reduce_solve_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ heavy_rows,
    const int32_t* __restrict__ slot_begin, const double* __restrict__ slots,
    float* __restrict__ X, int ld, int k, float reg, const double* __restrict__ yty,
    int32_t* __restrict__ status) {
  constexpr int NT = Cfg<CN>::NT;
  __shared__ __attribute__((aligned(16))) unsigned char smem[SmemBytes<CN>::value];
  const int h = blockIdx.x;
  const int row = heavy_rows[h];
  double a64[NT][4], b64[CN];
  zero_acc<NT, CN, double>(a64, b64);
  int npos = 0;
  for (int s = slot_begin[h]; s < slot_begin[h + 1]; ++s)
    add_slot<NT, CN>(slots + (int64_t)s * Cfg<CN>::SLOT, a64, b64, npos);
  const int64_t n_reg = IMPLICIT ? (int64_t)npos : (row_ptr[row + 1] - row_ptr[row]);
  finish_and_solve<CN, IMPLICIT, double>(a64, b64, n_reg, smem, k, reg, yty,
                                         X + (int64_t)row * ld, ld, row, status);
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
  const int64_t pb = (int64_t)blockIdx.x * kYtyChunk;
  const int64_t pe = pb + kYtyChunk < n ? pb + kYtyChunk : n;
  gram_accumulate<CN, false, true, double>(nullptr, nullptr, pb, pe, Y, ld, k, 0.f, a64, b64,
                                           npos);
  store_slot<NT, CN, double>(slots + (int64_t)blockIdx.x * Cfg<CN>::SLOT, a64, b64, npos);
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
// k in (64, 128]: one workgroup of 4 wavefronts per system (CN = 8, 36 upper
// tiles).  Wave R accumulates the tiles of WgTiles<R> (10/10/8/8) and keeps them
// in registers through the factorisation; the block LDL^T of tile_ldl_solve is
// spread over the workgroup:
//   (a) owners stage block row K (transposed) in LDS            | barrier
//   (b) wave 0: 16x16 LDL^T of B_KK with the rhs block z_K      | barrier
//   (c) TRSM, lane g = 64 R + lane owns column g of block row K  | barrier
//   (d) each wave: MFMA trailing update of its own tiles (I > K)
// and wave 0 runs the block back substitution.  (c) writes W into its own
// buffer, so the stage may be rewritten by the next K without another barrier.
// LDS (floats): U tiles 36*256 | stage 8*320 | W 7*256 | D, b, z, x 4*128 = 56 KB,
// so two workgroups (8 waves, 2 per SIMD) share a CU.
// ---------------------------------------------------------------------------
constexpr int kWgNB = 8;

struct WgLds {
  static constexpr int NB = kWgNB, NT = NB * (NB + 1) / 2;
  static constexpr int U = 0, S = NT * 256, W = S + NB * 320, D = W + (NB - 1) * 256,
                       B = D + 16 * NB, Z = B + 16 * NB, X = Z + 16 * NB, SIZE = X + 16 * NB;
};

// Wave-local LDS ordering (lanes of one wave exchanging values through LDS).
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

template <int R>
__device__ __forceinline__ bool wg_ldl_solve(floatx4 (&A)[WgTiles<R>::N], float* __restrict__ lds,
                                             int k, float* __restrict__ xrow, int ld) {
  typedef WgTiles<R> TS;
  typedef WgLds Lo;
  constexpr int NB = kWgNB;
  const int lane = threadIdx.x & 63, q = lane >> 4, m = lane & 15;
  const int i = lane & 15;
  float* Ust = lds + Lo::U;
  float* St = lds + Lo::S;
  float* Wb = lds + Lo::W;
  float* Dv = lds + Lo::D;
  float* bv = lds + Lo::B;
  float* zv = lds + Lo::Z;
  float* xv = lds + Lo::X;
  bool ok = true;
  static_for<NB>([&](auto Kc) {
    constexpr int K = decltype(Kc)::value;
    // (a) stage block row K transposed: St[J-K][j][k] (row stride 20 floats)
    static_for<TS::N>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      if constexpr (TS::g1(t) == K) {
        constexpr int J = TS::g2(t);
        const floatx4 v = A[t];
        *reinterpret_cast<float4*>(St + (J - K) * 320 + m * 20 + 4 * q) =
            make_float4(v[0], v[1], v[2], v[3]);
      }
    });
    __syncthreads();
    // (b) LDL^T of the diagonal block, rhs block as augmented column (wave 0)
    if constexpr (R == 0) {
      float a[16];
#pragma unroll
      for (int c4 = 0; c4 < 4; ++c4) {
        const float4 v = *reinterpret_cast<const float4*>(St + i * 20 + 4 * c4);
        a[4 * c4] = v.x; a[4 * c4 + 1] = v.y; a[4 * c4 + 2] = v.z; a[4 * c4 + 3] = v.w;
      }
      float bb = bv[K * 16 + i];
      float myd = 1.f;
#pragma unroll
      for (int p = 0; p < 16; ++p) {
        const float d = readlane_t(a[p], p);
        ok = ok && (d > 0.f);
        float u[16];
#pragma unroll
        for (int j = p + 1; j < 16; ++j) u[j] = readlane_t(a[p], j);
        const float bp = readlane_t(bb, p);
        const float l = a[p] * rcp_t(d);
#pragma unroll
        for (int j = p + 1; j < 16; ++j) a[j] = fmaf(-l, u[j], a[j]);
        if (i > p) bb = fmaf(-l, bp, bb);
        a[p] = l;
        if (i == p) myd = d;
      }
      float* Lt = Ust + 256 * tile_index(NB, K, K);  // Lt[c*16 + r] = L_K[r][c]
      if (lane < 16) {
        Dv[K * 16 + i] = myd;
        zv[K * 16 + i] = bb;
#pragma unroll
        for (int c = 0; c < 16; ++c) Lt[c * 16 + i] = (c < i) ? a[c] : 0.f;
      }
    }
    __syncthreads();
    if constexpr (K + 1 < NB) {
      constexpr int ncol = 16 * (NB - 1 - K);
      // (c) TRSM: g = 64 R + lane < ncol owns column (g & 15) of block J = K+1+(g>>4)
      if constexpr (64 * R < ncol) {
        const int g = 64 * R + lane;
        const bool is_col = g < ncol;
        const int Jl = K + 1 + (is_col ? (g >> 4) : 0);
        const float* Lt = Ust + 256 * tile_index(NB, K, K);
        float w[16];
        {
          const float* src = St + (Jl - K) * 320 + i * 20;
#pragma unroll
          for (int c4 = 0; c4 < 4; ++c4) {
            const float4 v = *reinterpret_cast<const float4*>(src + 4 * c4);
            w[4 * c4] = v.x; w[4 * c4 + 1] = v.y; w[4 * c4 + 2] = v.z; w[4 * c4 + 3] = v.w;
          }
        }
#pragma unroll
        for (int c = 0; c < 15; ++c) {
          float lc[16];
#pragma unroll
          for (int c4 = 0; c4 < 4; ++c4) {
            const float4 v = *reinterpret_cast<const float4*>(Lt + c * 16 + 4 * c4);
            lc[4 * c4] = v.x; lc[4 * c4 + 1] = v.y; lc[4 * c4 + 2] = v.z; lc[4 * c4 + 3] = v.w;
          }
#pragma unroll
          for (int p = c + 1; p < 16; ++p) w[p] = fmaf(-lc[p], w[c], w[p]);
        }
        if (is_col) {
          float* Wd = Wb + (Jl - K - 1) * 256 + i;
          float* Ud = Ust + 256 * tile_index(NB, K, Jl) + i;
          float t = 0.f;
#pragma unroll
          for (int c = 0; c < 16; ++c) {
            const float uc = w[c] * rcp_t(Dv[K * 16 + c]);
            Wd[c * 16] = w[c];
            Ud[c * 16] = uc;
            t = fmaf(uc, zv[K * 16 + c], t);
          }
          bv[Jl * 16 + i] -= t;  // b_J -= U_KJ^T z_K
        }
      }
      __syncthreads();
      // (d) trailing update of this wave's tiles on the matrix cores
      static_for<TS::N>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        constexpr int I = TS::g1(t), J = TS::g2(t);
        if constexpr (I > K) {
          floatx4 acc = A[t];
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4)
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(
                -Ust[256 * tile_index(NB, K, I) + (4 * s4 + q) * 16 + m],
                Wb[(J - K - 1) * 256 + (4 * s4 + q) * 16 + m], acc, 0, 0, 0);
          A[t] = acc;
        }
      });
    }
  });
  if constexpr (R == 0) {
    // (e) block back substitution (wave 0): x_K = U_KK^-1 (D_K^-1 z_K - sum_J U_KJ x_J)
#pragma unroll
    for (int K = NB - 1; K >= 0; --K) {
      float v = zv[K * 16 + i] * rcp_t(Dv[K * 16 + i]);
#pragma unroll
      for (int J = K + 1; J < NB; ++J) {
        const float* Ur = Ust + 256 * tile_index(NB, K, J) + i * 16;
#pragma unroll
        for (int j = 0; j < 16; ++j) v = fmaf(-Ur[j], xv[J * 16 + j], v);
      }
      const float* Lr = Ust + 256 * tile_index(NB, K, K) + i * 16;
      float ur[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) ur[j] = Lr[j];
      float x = 0.f;
#pragma unroll
      for (int j = 15; j >= 0; --j) {
        const float xj = readlane_t(v, j);
        if (i == j) x = xj;
        if (i < j) v = fmaf(-ur[j], xj, v);
      }
      if (lane < 16) xv[K * 16 + i] = x;
      wave_lds_sync();
    }
    // (f) un-permute: dim d = i*8 + K  <->  xv[K*16 + i]
    for (int d = lane; d < ld; d += 64) {
      const float x = d < 16 * NB ? xv[(d % NB) * 16 + d / NB] : 0.f;
      xrow[d] = (d < k && ok) ? x : 0.f;
    }
  }
  return ok;
}

// Wave R's part of completing one system: rhs blocks to LDS, YtY merge (fp64,
// then one rounding), lambda * n on the diagonal, the workgroup LDL^T.
template <int R, bool IMPLICIT, class AccT>
__device__ __forceinline__ void wg_finish_and_solve(AccT (&tot)[WgTiles<R>::N][4],
                                                    AccT (&bt)[WgTiles<R>::NRA], int64_t n_reg,
                                                    float* lds, int k, float reg,
                                                    const double* __restrict__ yty,
                                                    float* __restrict__ xrow, int ld, int row,
                                                    int32_t* __restrict__ status) {
  typedef WgTiles<R> TS;
  constexpr int NB = kWgNB;
  const int lane = threadIdx.x & 63, q = lane >> 4, m = lane & 15;
#pragma unroll
  for (int c = 0; c < TS::NR; ++c) {
    AccT v = bt[c];
    v += shfl_xor_t(v, 16);
    v += shfl_xor_t(v, 32);
    if (q == 0) lds[WgLds::B + TS::gcol(c) * 16 + m] = (float)v;
  }
  const float lam = (float)((double)reg * (double)n_reg);
  floatx4 A[TS::N];
  static_for<TS::N>([&](auto tc) {
    constexpr int t = decltype(tc)::value;
    constexpr int c1 = TS::g1(t), c2 = TS::g2(t);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      int i, j;
      tile_ij<NB>(c1, c2, r, i, j);
      float v;
      if constexpr (IMPLICIT) {
        const int hi = i > j ? i : j, lo = i > j ? j : i;
        v = (float)((double)tot[t][r] + yty[hi * (hi + 1) / 2 + lo]);
      } else {
        v = (float)tot[t][r];
      }
      if (c1 == c2 && i == j) v = (i < k) ? v + lam : 1.f;
      A[t][r] = v;
    }
  });
  const bool ok = wg_ldl_solve<R>(A, lds, k, xrow, ld);
  if (R == 0 && !ok && lane == 0) atomicCAS(status, 0, row + 1);
}

constexpr int kWgSub = Slot<10, 4>::SIZE;  // doubles per wave sub-slot (max over roles)
constexpr int kWgSlot = 4 * kWgSub;

template <int R, bool IMPLICIT>
__device__ __forceinline__ void wg_gram_solve_task(
    int task, const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ val, const int32_t* __restrict__ light_rows,
    const int64_t* __restrict__ chunk_begin, const int64_t* __restrict__ chunk_end,
    int32_t n_chunks, const float* __restrict__ Y, float* __restrict__ X, int ld, int k,
    float reg, float alpha, const double* __restrict__ yty, double* __restrict__ slots,
    int32_t* __restrict__ status, float* lds) {
  typedef WgTiles<R> TS;
  float tot[TS::N][4], bt[TS::NRA];
  zero_acc<TS::N, TS::NRA, float>(tot, bt);
  int npos = 0;
  if (task < n_chunks) {
    gram_accumulate<kWgNB, IMPLICIT, false, float, TS>(col, val, chunk_begin[task], chunk_end[task],
                                                       Y, ld, k, alpha, tot, bt, npos);
    store_slot<TS::N, TS::NRA, float>(slots + (int64_t)task * kWgSlot + R * kWgSub, tot, bt, npos);
    return;
  }
  const int row = light_rows[task - n_chunks];
  const int64_t pb = row_ptr[row], pe = row_ptr[row + 1];
  gram_accumulate<kWgNB, IMPLICIT, false, float, TS>(col, val, pb, pe, Y, ld, k, alpha, tot, bt,
                                                     npos);
  const int64_t n_reg = IMPLICIT ? (int64_t)npos : (pe - pb);
  wg_finish_and_solve<R, IMPLICIT, float>(tot, bt, n_reg, lds, k, reg, yty, X + (int64_t)row * ld,
                                          ld, row, status);
}

template <int R, bool IMPLICIT>
__device__ __forceinline__ void wg_reduce_solve_task(int h, const int64_t* __restrict__ row_ptr,
                                                     const int32_t* __restrict__ heavy_rows,
                                                     const int32_t* __restrict__ slot_begin,
                                                     const double* __restrict__ slots,
                                                     float* __restrict__ X, int ld, int k, float reg,
                                                     const double* __restrict__ yty,
                                                     int32_t* __restrict__ status, float* lds) {
  typedef WgTiles<R> TS;
  const int row = heavy_rows[h];
  double a64[TS::N][4], b64[TS::NRA];
  zero_acc<TS::N, TS::NRA, double>(a64, b64);
  int npos = 0;
  for (int s = slot_begin[h]; s < slot_begin[h + 1]; ++s)
    add_slot<TS::N, TS::NRA>(slots + (int64_t)s * kWgSlot + R * kWgSub, a64, b64, npos);
  const int64_t n_reg = IMPLICIT ? (int64_t)npos : (row_ptr[row + 1] - row_ptr[row]);
  wg_finish_and_solve<R, IMPLICIT, double>(a64, b64, n_reg, lds, k, reg, yty,
                                           X + (int64_t)row * ld, ld, row, status);
}

template <int R>
__device__ __forceinline__ void wg_yty_partial_task(const float* __restrict__ Y, int64_t n, int ld,
                                                    int k, double* __restrict__ slots) {
  typedef WgTiles<R> TS;
  double a64[TS::N][4], b64[TS::NRA];
  zero_acc<TS::N, TS::NRA, double>(a64, b64);
  int npos = 0;
  const int64_t pb = (int64_t)blockIdx.x * kYtyChunk;
  const int64_t pe = pb + kYtyChunk < n ? pb + kYtyChunk : n;
  gram_accumulate<kWgNB, false, true, double, TS>(nullptr, nullptr, pb, pe, Y, ld, k, 0.f, a64,
                                                  b64, npos);
  store_slot<TS::N, TS::NRA, double>(slots + (int64_t)blockIdx.x * kWgSlot + R * kWgSub, a64, b64,
                                     npos);
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

template <bool IMPLICIT>
__global__ __launch_bounds__(256, 2) void gram_solve_wg_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ val, const int32_t* __restrict__ light_rows,
    const int64_t* __restrict__ chunk_begin, const int64_t* __restrict__ chunk_end,
    int32_t n_chunks, const float* __restrict__ Y, float* __restrict__ X, int ld, int k,
    float reg, float alpha, const double* __restrict__ yty, double* __restrict__ slots,
    int32_t* __restrict__ status) {
  __shared__ __attribute__((aligned(16))) float lds[WgLds::SIZE];
#define CALL(R)                                                                                 \
  wg_gram_solve_task<R, IMPLICIT>(blockIdx.x, row_ptr, col, val, light_rows, chunk_begin,      \
                                  chunk_end, n_chunks, Y, X, ld, k, reg, alpha, yty, slots,   \
                                  status, lds)
  ALS_WG_ROLES(CALL);
#undef CALL
}

template <bool IMPLICIT>
__global__ __launch_bounds__(256, 2) void reduce_solve_wg_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ heavy_rows,
    const int32_t* __restrict__ slot_begin, const double* __restrict__ slots,
    float* __restrict__ X, int ld, int k, float reg, const double* __restrict__ yty,
    int32_t* __restrict__ status) {
  __shared__ __attribute__((aligned(16))) float lds[WgLds::SIZE];
#define CALL(R)                                                                           \
  wg_reduce_solve_task<R, IMPLICIT>(blockIdx.x, row_ptr, heavy_rows, slot_begin, slots, X, \
                                    ld, k, reg, yty, status, lds)
  ALS_WG_ROLES(CALL);
#undef CALL
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

static size_t slot_doubles(int k) {
  switch (cn_for_k(k)) {
    case 1: return Cfg<1>::SLOT;
    case 2: return Cfg<2>::SLOT;
    case 4: return Cfg<4>::SLOT;
    default: return kWgSlot;
  }
}

extern "C" {

size_t als_solve_workspace_bytes(int32_t k, int32_t n_chunks) {
  return align_up(sizeof(double) * slot_doubles(k) * (size_t)(n_chunks > 0 ? n_chunks : 0)) + 256;
}

int als_solve_half(const int64_t* row_ptr, const int32_t* col, const float* val,
                   const int32_t* light_rows, int32_t n_light, const int32_t* heavy_rows,
                   const int32_t* heavy_slot_begin, int32_t n_heavy, const int32_t* chunk_row,
                   const int64_t* chunk_begin, const int64_t* chunk_end, int32_t n_chunks,
                   const float* Y_src, float* X_dst, int32_t ld, int32_t k, float reg,
                   int implicit, float alpha, const double* yty_packed, int32_t* status_dev,
                   void* ws, size_t ws_bytes, int phases, void* stream) {
  ALS_REQUIRE(k >= 1 && k <= kMaxRank, ALS_EUNSUPPORTED, "als_solve_half: rank %d not in [1, %d]",
              k, kMaxRank);
  ALS_REQUIRE(ld >= k && ld % 4 == 0, ALS_EINVAL, "als_solve_half: ld=%d must be >= k and %%4==0",
              ld);
  ALS_REQUIRE(n_light >= 0 && n_heavy >= 0 && n_chunks >= 0, ALS_EINVAL,
              "als_solve_half: negative counts");
  ALS_REQUIRE(Y_src && X_dst && row_ptr && status_dev, ALS_EINVAL, "als_solve_half: null pointer");
  ALS_REQUIRE(!implicit || yty_packed, ALS_EINVAL, "als_solve_half: implicit needs yty_packed");
  ALS_REQUIRE(reg >= 0.f && alpha >= 0.f, ALS_EINVAL, "als_solve_half: reg/alpha must be >= 0");
  ALS_REQUIRE((reinterpret_cast<uintptr_t>(Y_src) & 15) == 0, ALS_EINVAL,
              "als_solve_half: Y_src must be 16-byte aligned");
  ALS_REQUIRE(ws_bytes >= als_solve_workspace_bytes(k, n_chunks), ALS_EWORKSPACE,
              "als_solve_half: workspace %zu < %zu", ws_bytes,
              als_solve_workspace_bytes(k, n_chunks));
  hipStream_t st = as_stream(stream);
  double* slots = static_cast<double*>(ws);
  const int cn = cn_for_k(k);
  ALS_REQUIRE(phases >= 1 && phases <= 3, ALS_EINVAL, "als_solve_half: phases must be 1, 2 or 3");
  const unsigned g1 = (phases & 1) ? (unsigned)(n_chunks + n_light) : 0u;
  const unsigned g2 = (phases & 2) ? (unsigned)n_heavy : 0u;
#define ALS_SOLVE_LAUNCH(CN, IMP)                                                                 \
  do {                                                                                            \
    if (g1)                                                                                       \
      gram_solve_kernel<CN, IMP><<<g1, 64, 0, st>>>(row_ptr, col, val, light_rows, chunk_row,     \
                                                    chunk_begin, chunk_end, n_chunks, Y_src,      \
                                                    X_dst, ld, k, reg, alpha, yty_packed, slots,  \
                                                    status_dev);                                  \
    ALS_LAUNCH_CHECK();                                                                           \
    if (g2)                                                                                       \
      reduce_solve_kernel<CN, IMP><<<g2, 64, 0, st>>>(row_ptr, heavy_rows, heavy_slot_begin,     \
                                                      slots, X_dst, ld, k, reg, yty_packed,       \
                                                      status_dev);                                \
    ALS_LAUNCH_CHECK();                                                                           \
  } while (0)
#define ALS_SOLVE_WG_LAUNCH(IMP)                                                                  \
  do {                                                                                            \
    if (g1)                                                                                       \
      gram_solve_wg_kernel<IMP><<<g1, 256, 0, st>>>(row_ptr, col, val, light_rows, chunk_begin,   \
                                                    chunk_end, n_chunks, Y_src, X_dst, ld, k,     \
                                                    reg, alpha, yty_packed, slots, status_dev);   \
    ALS_LAUNCH_CHECK();                                                                           \
    if (g2)                                                                                       \
      reduce_solve_wg_kernel<IMP><<<g2, 256, 0, st>>>(row_ptr, heavy_rows, heavy_slot_begin,     \
                                                      slots, X_dst, ld, k, reg, yty_packed,       \
                                                      status_dev);                                \
    ALS_LAUNCH_CHECK();                                                                           \
  } while (0)
  if (implicit) {
    if (cn == 1) ALS_SOLVE_LAUNCH(1, true);
    else if (cn == 2) ALS_SOLVE_LAUNCH(2, true);
    else if (cn == 4) ALS_SOLVE_LAUNCH(4, true);
    else ALS_SOLVE_WG_LAUNCH(true);
  } else {
    if (cn == 1) ALS_SOLVE_LAUNCH(1, false);
    else if (cn == 2) ALS_SOLVE_LAUNCH(2, false);
    else if (cn == 4) ALS_SOLVE_LAUNCH(4, false);
    else ALS_SOLVE_WG_LAUNCH(false);
  }
#undef ALS_SOLVE_LAUNCH
#undef ALS_SOLVE_WG_LAUNCH
  return ALS_OK;
}

size_t als_yty_workspace_bytes(int64_t n, int32_t k) {
  const int64_t nslots = n > 0 ? (n + kYtyChunk - 1) / kYtyChunk : 1;
  return align_up(sizeof(double) * slot_doubles(k) * (size_t)nslots) + 256;
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
  const int nslots = n > 0 ? (int)((n + kYtyChunk - 1) / kYtyChunk) : 0;
  const int cn = cn_for_k(k);
  if (nslots == 0) {
    const int kp = 16 * cn;
    ALS_HIP(hipMemsetAsync(yty_packed_out, 0, sizeof(double) * kp * (kp + 1) / 2, st));
    return ALS_OK;
  }
#define ALS_YTY_LAUNCH(CN)                                                                    \
  do {                                                                                        \
    yty_partial_kernel<CN><<<nslots, 64, 0, st>>>(Y, n, ld, k, slots);                        \
    ALS_LAUNCH_CHECK();                                                                       \
    yty_reduce_kernel<CN><<<1, 64, 0, st>>>(slots, nslots, yty_packed_out);                   \
    ALS_LAUNCH_CHECK();                                                                       \
  } while (0)
  if (cn == 1) ALS_YTY_LAUNCH(1);
  else if (cn == 2) ALS_YTY_LAUNCH(2);
  else if (cn == 4) ALS_YTY_LAUNCH(4);
  else {
    yty_partial_wg_kernel<<<nslots, 256, 0, st>>>(Y, n, ld, k, slots);
    ALS_LAUNCH_CHECK();
    yty_reduce_wg_kernel<<<1, 256, 0, st>>>(slots, nslots, yty_packed_out);
    ALS_LAUNCH_CHECK();
  }
#undef ALS_YTY_LAUNCH
  return ALS_OK;
}

}  // extern "C"
