// K5 — recommendForAll: blocked U.V^T on the matrix cores with a fused,
// bounded per-row top-k.  The n_q x n_v score matrix is never materialised.
//
// Replaces ALSModel.recommendForAll (upstream Spark >= 2.2: blockify at 4096
// rows, crossJoin, sgemm per block pair, bounded priority queue,
// TopByKeyAggregator merge) and mllib recommendProductsForUsers.  The
// reference's own top-k is `predictAll` over one user's unrated movies then
// `takeOrdered(20, key=-pred)` (RecommenderSystem.py:229-247).
//
// Scores on the f16 matrix cores with fp32-grade products (the split scheme
// of the Gram in gram_solve.hip): q and v are scaled by powers of two (from
// max |Q| and max |V|) and carried as f16 hi + lo, hi = f16_rn(t),
// lo = f16_rn(t - hi); <q, v> = hi.hi + hi.lo + lo.hi accumulated in fp32 by
// v_mfma_f32_16x16x32_f16 (~2^-21 relative to |q||v| per product, below the
// rounding of Spark's fp32 sgemm).  V is split once per call into f16 planes
// (topk_split_table_kernel: row r = [hi of dims 0..KQ) | lo of dims 0..KQ)]),
// so a staged tile row is copied as is and every B operand is one
// ds_read_b128.  The query rows are split in registers once per workgroup.
//
// Workgroup = NW wavefronts x RG row groups = 16 NW RG query rows.  The workgroup
// sweeps V in tiles double-buffered in LDS (one barrier per tile, the next tile's
// LDS-DMA pieces in flight).  V is swept in order of decreasing row norm
// (bucketed; the high-scoring rows come first, so the lists fill with
// near-final entries early), each 16 x 16 score block is filtered against its
// rows' current k-th best score, and the rare survivors are inserted into the
// per-row lists: in registers for top <= 16, sorted in LDS with a
// wave-cooperative insertion above.  Insertions compare (score, V row index)
// exactly, so the sweep order changes the speed, not the result.  Order: score
// descending, ties by ascending index (the build's deterministic tie rule,
// SURVEY Appendix A.6).  Scores are compared in the scaled domain (exact:
// powers of two) and unscaled on output.  An all-zero query row scores 0
// against every V row; its list is the first `top` rows by index.
#include "als_common.h"

#include <algorithm>

namespace als {

typedef float floatx4 __attribute__((ext_vector_type(4)));

namespace {

typedef _Float16 tk_half8 __attribute__((ext_vector_type(8)));

// Power-of-two scale exponent: the largest |t| of the operand lands in [2^14, 2^15).
__device__ __forceinline__ int tk_split_exponent(float m) {
  if (!(m > 0.f) || !(m < 3.0e38f)) return 0;
  int e = 14 - ilogbf(m);
  return e < -60 ? -60 : (e > 60 ? 60 : e);
}

__device__ __forceinline__ void tk_split(float t, _Float16& hi, _Float16& lo) {
  hi = (_Float16)t;  // round to nearest
  lo = (_Float16)(t - (float)hi);
}

// max |x| over n floats -> *out (ordered uint bits; *out zeroed beforehand).
__global__ __launch_bounds__(256) void tk_absmax_kernel(const float* __restrict__ x, int64_t n,
                                                        unsigned* __restrict__ out) {
  float m = 0.f;
  const int64_t n4 = n >> 2;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  auto fold = [&](const float4& v) {
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
  };
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n4; i += 4 * stride) {  // four independent loads in flight
    const float4 a = x4[i], b = x4[i + stride], c = x4[i + 2 * stride], d = x4[i + 3 * stride];
    fold(a);
    fold(b);
    fold(c);
    fold(d);
  }
  for (; i < n4; i += stride) fold(x4[i]);
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) m = fmaxf(m, fabsf(x[4 * n4 + threadIdx.x]));
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    atomicMax(out, __float_as_uint(m));  // NaN-free non-negative floats order as uints
  }
}

}  // namespace

constexpr int kTopkMax = 256;
constexpr int kLdsBytes = 160 * 1024;  // per CU on gfx950 (one workgroup may use it all)

// Lists hold (score, index) as one 64-bit key whose unsigned order is the
// ranking order: high word = the score's bits made monotone (sign flip), low word =
// ~index (a lower index ranks higher on equal scores).  NaN scores are never keys.
__device__ __forceinline__ uint64_t tk_key(float sc, int id) {
  const uint32_t u = __float_as_uint(sc + 0.f);  // -0 -> +0: equal scores, equal bits
  const uint32_t o = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ((uint64_t)o << 32) | (uint32_t)(~id);
}
__device__ __forceinline__ float tk_key_score(uint64_t key) {
  const uint32_t o = (uint32_t)(key >> 32);
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}
__device__ __forceinline__ int tk_key_index(uint64_t key) { return (int)~(uint32_t)key; }
constexpr uint64_t kTkKeyOpen = 0;              // unfilled entry: any candidate ranks above it
constexpr uint64_t kTkKeySentinel = ~0ull;      // entries past `top`: nothing ranks above it

__device__ __forceinline__ bool beats(float s1, int i1, float s2, int i2) {
  return s1 > s2 || (s1 == s2 && i1 < i2);
}

// Offer one 16 x 16 score block to the sorted per-row lists (64-bit keys, best
// first): acc[r] = score of list row slot0 + 4q + r against V row ibase + m.
// Candidates that beat their row's current k-th (score, index) are inserted one at
// a time by the whole wave (rank by ballot, shift, insert), lowest lane first.  The
// rank is counted from the tail: past the fill, a new key usually lands in the last
// 64 entries, so one LDS pass finds it.
__device__ __forceinline__ void topk_offer(const floatx4& acc, int ibase, int64_t n_v,
                                           const int32_t* __restrict__ bperm, float (&ts)[4],
                                           int (&ti)[4], uint64_t* __restrict__ lk,
                                           int* __restrict__ len, int slot0, int top,
                                           unsigned live) {
  const int lane = threadIdx.x & 63, q = lane >> 4;
  const int m = lane & 15;
  const bool vin = (int64_t)(ibase + m) < n_v;
  // V row index of table row ibase + m (the sweep is norm-ordered; bperm = the
  // block's slice of the tile's order in LDS)
  const int vidx = vin ? bperm[m] : 0x7fffffff;
  int pend = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r)
    if (vin && ((live >> (4 * q + r)) & 1u) && beats(acc[r], vidx, ts[r], ti[r])) pend |= 1 << r;
  uint64_t any = __ballot(pend != 0);
  while (any) {
    const int L = __builtin_ctzll(any);
    const int myr = pend ? __builtin_ctz(pend) : 0;
    const float mys = myr == 0 ? acc[0] : (myr == 1 ? acc[1] : (myr == 2 ? acc[2] : acc[3]));
    const int rL = __builtin_amdgcn_readlane(myr, L);
    const float sc =
        __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, mys), L));
    const int itm = __builtin_amdgcn_readlane(vidx, L);
    const uint64_t ck = tk_key(sc, itm);
    const int slot = slot0 + 4 * (L >> 4) + rL;  // list row within the workgroup
    uint64_t* lkr = lk + slot * top;
    const int n = len[slot];
    // pos = number of entries that beat the candidate = n - (entries it beats);
    // scan 64-entry windows from the tail until one holds an entry that beats it
    int worse = 0;
    for (int e1 = n; e1 > 0; e1 -= 64) {
      const int e = e1 - 64 + lane;
      const int cnt = __popcll(__ballot(e >= 0 && lkr[e < 0 ? 0 : e] < ck));
      worse += cnt;
      if (cnt < (e1 < 64 ? e1 : 64)) break;
    }
    const int pos = n - worse;
    if (pos < top) {
      const int newn = n + 1 < top ? n + 1 : top;
      uint64_t hk[kTopkMax / 64];
#pragma unroll
      for (int j = 0; j < kTopkMax / 64; ++j) {
        const int e = 64 * j + lane;
        if (e > pos && e < newn) hk[j] = lkr[e - 1];
      }
      // reads of the shifted entries land before any lane writes (compiler + HW order)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int j = 0; j < kTopkMax / 64; ++j) {
        const int e = 64 * j + lane;
        if (e > pos && e < newn) lkr[e] = hk[j];
      }
      if (lane == 0) {
        lkr[pos] = ck;
        len[slot] = newn;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (newn == top) {
        const uint64_t kk = lkr[top - 1];
        const float ks = tk_key_score(kk);
        const int ki = tk_key_index(kk);
        if (q == (L >> 4)) {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (r == rL) {
              ts[r] = ks;
              ti[r] = ki;
            }
        }
      }
    }
    if (lane == L) pend &= ~(1 << rL);
    // drop pending candidates of that row that no longer beat its threshold
    if (q == (L >> 4)) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (r == rL && (pend >> r & 1) && !beats(acc[r], vidx, ts[r], ti[r])) pend &= ~(1 << r);
    }
    any = __ballot(pend != 0);
  }
}

// Write the lists of rows slot0 .. slot0+15 (one wave) to the outputs.
__device__ __forceinline__ void topk_write(const uint64_t* __restrict__ lk,
                                           const int* __restrict__ len, int slot0, int64_t qbase,
                                           int64_t n_q, int64_t n_v, int top, float unscale,
                                           unsigned live, int32_t* __restrict__ idx_out,
                                           float* __restrict__ score_out) {
  const int lane = threadIdx.x & 63;
  for (int rr = 0; rr < 16; ++rr) {
    const int slot = slot0 + rr;
    const int64_t row = qbase + slot;
    if (row >= n_q) break;
    if (!((live >> rr) & 1u)) {  // all-zero query row: every score is 0, ties by index
      for (int e = lane; e < top; e += 64) {
        idx_out[row * top + e] = e < n_v ? e : -1;
        score_out[row * top + e] = e < n_v ? 0.f : -__builtin_inff();
      }
      continue;
    }
    const int n = len[slot];
    for (int e = lane; e < top; e += 64) {
      const uint64_t kk = e < n ? lk[slot * top + e] : 0ull;
      idx_out[row * top + e] = e < n ? tk_key_index(kk) : -1;
      score_out[row * top + e] = e < n ? tk_key_score(kk) * unscale : -__builtin_inff();
    }
  }
}

// Sweep order: V rows by decreasing norm (4096 log-spaced buckets, 128 per octave;
// order inside a bucket arbitrary).  Large-norm rows carry most top scores, so the
// lists fill with near-final entries early and later rows rarely pass the filter.
// The order only affects speed: insertion compares (score, V row index) exactly.
constexpr int kTkBuckets = 4096;

// 16 lanes per V row: squared norm -> bucket (0 = largest norms).
__device__ __forceinline__ int tk_row_bucket(const float* __restrict__ V, int64_t r, int ld,
                                             int k, float log2_ref) {
  const int l = threadIdx.x & 15;
  float s = 0.f;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int d = 4 * l + 64 * h;
    if (d < k) {
      const float4 v = *reinterpret_cast<const float4*>(V + r * ld + d);
      s += v.x * v.x + (d + 1 < k ? v.y * v.y : 0.f) + (d + 2 < k ? v.z * v.z : 0.f) +
           (d + 3 < k ? v.w * v.w : 0.f);
    }
  }
  for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (!(s > 0.f)) return kTkBuckets - 1;
  const float b = (log2_ref - 0.5f * __log2f(s)) * 128.f;  // octaves below the reference
  // (NaN, e.g. an Inf row against an Inf reference: bucket 0)
  return !(b > 0.f) ? 0 : (b >= (float)(kTkBuckets - 1) ? kTkBuckets - 1 : (int)b);
}

__device__ __forceinline__ float tk_log2_ref(const float* __restrict__ scal, int k) {
  // reference norm: max |v| * sqrt(k) bounds every row norm
  return __log2f(fmaxf(scal[1], 1e-30f)) + 0.5f * __log2f((float)k);
}

// Bucket counts: per-workgroup histogram in LDS (rows of similar norm share a
// bucket, so global atomics per row would serialise), flushed once per nonzero bin.
__global__ __launch_bounds__(256) void tk_bucket_hist_kernel(const float* __restrict__ V,
                                                             int64_t n_v, int ld, int k,
                                                             const float* __restrict__ scal,
                                                             int32_t* __restrict__ hist) {
  __shared__ int lh[kTkBuckets];
  for (int b = threadIdx.x; b < kTkBuckets; b += 256) lh[b] = 0;
  __syncthreads();
  const float ref = tk_log2_ref(scal, k);
  for (int64_t r = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4; r < n_v;
       r += ((int64_t)gridDim.x * 256) >> 4) {
    const int b = tk_row_bucket(V, r, ld, k, ref);
    if ((threadIdx.x & 15) == 0) atomicAdd(lh + b, 1);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < kTkBuckets; b += 256)
    if (lh[b]) atomicAdd(hist + b, lh[b]);
}

// Exclusive scan of the bucket counts (one workgroup) -> scatter cursors.
__global__ __launch_bounds__(1024) void tk_bucket_scan_kernel(int32_t* __restrict__ hist) {
  __shared__ int part[1024];
  const int t = threadIdx.x;
  int v[4], s = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[j] = hist[4 * t + j];
    s += v[j];
  }
  part[t] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const int x = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += x;
    __syncthreads();
  }
  int run = part[t] - s;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    hist[4 * t + j] = run;
    run += v[j];
  }
}

// Scatter with the same grid as the count pass: a workgroup recounts its rows in
// LDS, reserves one range per nonzero bin with one global atomic, then places its
// rows inside those ranges with LDS atomics.
__global__ __launch_bounds__(256) void tk_bucket_scatter_kernel(const float* __restrict__ V,
                                                                int64_t n_v, int ld, int k,
                                                                const float* __restrict__ scal,
                                                                int32_t* __restrict__ cursor,
                                                                int32_t* __restrict__ perm) {
  __shared__ int lh[kTkBuckets];
  for (int b = threadIdx.x; b < kTkBuckets; b += 256) lh[b] = 0;
  __syncthreads();
  const float ref = tk_log2_ref(scal, k);
  const int64_t r0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4;
  const int64_t rs = ((int64_t)gridDim.x * 256) >> 4;
  for (int64_t r = r0; r < n_v; r += rs) {
    const int b = tk_row_bucket(V, r, ld, k, ref);
    if ((threadIdx.x & 15) == 0) atomicAdd(lh + b, 1);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < kTkBuckets; b += 256)
    if (lh[b]) lh[b] = atomicAdd(cursor + b, lh[b]);  // base of this workgroup's range
  __syncthreads();
  for (int64_t r = r0; r < n_v; r += rs) {
    const int b = tk_row_bucket(V, r, ld, k, ref);
    if ((threadIdx.x & 15) == 0) perm[atomicAdd(lh + b, 1)] = (int32_t)r;
  }
}

// Norms of the scaled V rows in sweep order (16 lanes per table row): the coarse
// filter's error slack and the early-exit bound of topk_split_kernel.
__global__ __launch_bounds__(256) void tk_table_norm_kernel(const float* __restrict__ V,
                                                            int64_t n_v, int ld, int k,
                                                            const float* __restrict__ scal,
                                                            const int32_t* __restrict__ perm,
                                                            float* __restrict__ vnorm) {
  const float sv = ldexpf(1.f, tk_split_exponent(scal[1]));
  const int l = threadIdx.x & 15;
  for (int64_t t = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4; t < n_v;
       t += ((int64_t)gridDim.x * 256) >> 4) {
    const int64_t r = perm[t];
    float s = 0.f;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int d = 4 * l + 64 * h;
      if (d < k) {
        const float4 v = *reinterpret_cast<const float4*>(V + r * ld + d);
        s += v.x * v.x + (d + 1 < k ? v.y * v.y : 0.f) + (d + 2 < k ? v.z * v.z : 0.f) +
             (d + 3 < k ? v.w * v.w : 0.f);
      }
    }
    for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o);
    // a row with a NaN / Inf entry: an unbounded norm keeps every bound using it open
    if (l == 0) vnorm[t] = s < __builtin_inff() ? sv * sqrtf(s) : __builtin_inff();
  }
}

// V -> split planes in sweep order, table row t = V row perm[t]: hi plane
// [n_v][KQ] = hi(sv v), then lo plane [n_v][KQ] = lo(sv v) (f16), dims >= k zero.
__global__ __launch_bounds__(256) void topk_split_table_kernel(const float* __restrict__ V,
                                                               int64_t n_v, int ld, int k,
                                                               int kq_shift,
                                                               const float* __restrict__ scal,
                                                               const int32_t* __restrict__ perm,
                                                               _Float16* __restrict__ out) {
  const float sv = ldexpf(1.f, tk_split_exponent(scal[1]));
  const int kq = 1 << kq_shift;
  const int64_t total = n_v << kq_shift;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * 256) {
    const int64_t r = e >> kq_shift;
    const int d = (int)(e & (kq - 1));
    const float t = d < k ? sv * V[(int64_t)perm[r] * ld + d] : 0.f;
    _Float16 h, l;
    tk_split(t, h, l);
    out[e] = h;
    out[total + e] = l;
  }
}

// Split-f16 scores.  NK = KQ / 32 MFMA k-steps (KQ = k padded to 32, 64 or 128);
// RG query-row groups of 16 NW rows per workgroup (NW wavefronts, tk_nw).
// scal[0] = max |Q|, scal[1] = max |V|.
//
// The sweep is bound by how many V bytes are in flight from L2 / HBM, not by the
// matrix cores (dev ablation at configs[4]: the hi.hi sweep alone ran at ~4.5 TB/s
// with 8-16 KB of tile loads in flight per workgroup, i.e. one L2-miss latency per
// tile), so the design minimises the V bytes streamed per query row:
//  * only the hi plane of V is staged (256 B per row at KQ = 128, half the split
//    table); the lo halves are fetched for the rare refined blocks;
//  * with register lists a workgroup is 8 wavefronts (128 RG query rows per tile
//    stream; one workgroup per CU at the lists' register count) and a tile is 16-32
//    KB, so each L2 latency delivers more rows.
// Tiles are double-buffered in LDS and land there by LDS-DMA (global_load_lds_dwordx4,
// no staging registers, no ds_write): tile t+1's pieces are issued right after the
// barrier that released its buffer and fly while tile t is scored; ONE barrier per
// tile.  Rows are unpadded (RW = 4 NK uint4) and swizzled (TK_SWZ), so the
// ds_read_b128 lane groups of gfx950 ({0-3,12-15,20-27}, ...) touch 16 distinct 4-bank
// slots, conflict-free.
// Coarse filter, exact refinement: a block is first scored with hi.hi alone (one
// MFMA per k-step instead of three).  The dropped terms hi.lo + lo.hi are bounded
// by 2^-10 |q| |v| (Cauchy-Schwarz on |lo| <= 2^-11 |t|, plus the f16 subnormal
// and fp32 accumulation terms, all far below it), so a pair can reach its row's
// k-th score only if hi.hi >= k-th - 2^-9 (|q| + 1)(NV + 1), NV >= |v| for every row
// from the current tile on: one compare per score, one ballot per 16 x 16 block.  A
// block with a pair past that bound gets its lo halves by LDS-DMA and the hi.lo +
// lo.hi MFMAs added (the exact score every pair is ranked by, the same wherever
// the pair is met); the owners then compare the exact (score, index) keys.  The
// MFMAs of block c+1 are issued before block c's filter (two accumulator sets).
// Early exit: V is swept by decreasing norm, so no later row has a norm above the
// current tile's first row x 2^(1/128) (one bucket); a row whose k-th score
// exceeds (|q| + 1)(that bound + 1)(1 + 2^-7) can gain nothing from the rest of
// the sweep.  A wave whose rows are all there skips its tiles, and the workgroup
// leaves the sweep when all its waves are (at configs[4] the factor norms are too
// concentrated for this to trigger; it pays on long-tailed norm spreads).
// Lists (TOPR > 0, top <= TOPR): each row's list lives in the registers of one
// "owner" lane (lane 16g + rho owns row rho of group g), sorted by ascending
// goodness with the k-th best at [0] (entries top..TOPR-1 are sentinels that
// nothing beats), so the threshold is a fixed register and an insertion is one
// branch-free bubble pass.  A block with survivors stages its 16 x 16 scores in
// LDS (one ds_write_b128 per lane); each owner lane takes its row's survivors
// from the ballots, inserts them, and the new k-th scores go back to the
// filtering lanes through LDS.  16 < top <= 128 (TOPR = 32 / 64 / 100 / 128, one
// row groups as top <= 16): key logs — no list in registers; every key reaching its
// row's threshold (the exact k-th best score as of the last cut of the row's log) is
// appended to the log, one ballot per row and block (the LDS path below inserts one
// candidate per wave at a time: 70 ms vs 13.6 ms of scores at rank 128 top 100 on the
// ML-25M shape); the output is the exact top `top` keys of the log (tk_log_kth),
// ranked.
// TOPR = 0 (top > 128): sorted lists in LDS, wave-cooperative insertion
// (topk_offer), 4 wavefronts.
// Tile rows (hi halves only, RW = 4 NK uint4 per row): register lists (8
// wavefronts) 128 rows at NK = 4 (4 staged uint4 per thread), 256 / NK below (2 per
// thread); LDS lists (4 wavefronts) 64 / NK rows (1 per thread), which leaves the
// LDS to the lists.
// (Round 5, LDS-DMA staging, configs[4] 262,144-user sample: 192-row tiles at rank >
// 64 vs 128: top-10 91.5 -> 89.4 ms, top-100 193.5 -> 189.5 ms; 256 rows do not fit
// the LDS beside the lo scratch and the score blocks.  At rank <= 64, 384 / nk rows vs
// 256 / nk, all 162,541 ML-25M-shaped users: top-10 3.85 -> 3.60 ms, top-100 20.8 ->
// 19.7 ms, profiles/r05/ab_topk_small_tiles.txt.)
__host__ __device__ constexpr int tk_vt(int nk, int topr) {
  return topr == 0 ? 64 / nk : (nk == 4 ? 192 : 384 / nk);
}
// Tile buffers in LDS: the one scored and the next one landing.  (Three, i.e. two
// tiles in flight, measured slower: top-100 203 vs 193 ms at 128-row tiles — a refined
// block's vmcnt(0) then also waits for the later tile's pieces.)
__host__ __device__ constexpr int tk_nbuf(int topr) { return (void)topr, 2; }

// Tile-row swizzle: uint4 column c of tile row r sits at c ^ sw(r), sw(r) = (r >> 1) & 3
// at RW = 4 (NK = 1), r & (RW - 1) at RW = 8, 16: the ds_read_b128 lane groups of gfx950
// ({0-3,12-15,20-27}, ...) reading column 4s + q of rows 16b + m then touch 16 distinct
// 16-byte bank slots (checked by enumeration for each RW).  (Written out where it is
// used: a call to a function template from the kernel's lambdas made hipcc's host pass
// drop the kernels' handles, an undefined symbol at load time.)
#define TK_SWZ(NK, r) ((NK) == 1 ? ((r) >> 1) & 3 : (r) & (4 * (NK) - 1))

// Insert key `c` into a list sorted ascending (the k-th best at [0]; sentinels past
// `top`).  c_j = c > key_j is monotone (true for j < p); the list becomes
// [.. keys 1..p-1, c, keys p..]: independent selects, no chain.  The caller has
// checked c > [0].
template <int TOPR>
__device__ __forceinline__ void tk_insert(uint64_t (&kv)[TOPR], uint64_t c) {
  bool gt[TOPR + 1];
#pragma unroll
  for (int j = 0; j < TOPR; ++j) gt[j] = c > kv[j];
  gt[TOPR] = false;
#pragma unroll
  for (int j = 0; j < TOPR; ++j) {
    const uint64_t nx = j + 1 < TOPR ? kv[j + 1] : 0ull;
    kv[j] = gt[j + 1] ? nx : (gt[j] ? c : kv[j]);
  }
}

// Per-row key logs (16 < top <= 128).  No list lives in registers: every (score, index)
// key that reaches its row's threshold is appended to the row's log in global memory
// (tk_log_cap keys per row), the 16 lanes of a row group placing a block's keys with one
// ballot per row.  The threshold is the row's exact k-th best score as of the last cut
// of its log: a log that one more tile could overflow is cut in place to its `top`
// largest keys (tk_log_kth), whose smallest then becomes the threshold, and at the end
// of the sweep the row's output is selected from its log the same way.  Every key that
// ranks above the running k-th has reached the log, because the threshold never
// exceeds it, so the cuts and the output are exact.
// (384 vs 512 vs 1,024 keys at rank 128: the configs[4] sample's top-100 144 / 146 / 162 ms,
// profiles/r06/ab_topk_logs.txt)
constexpr int kTkLogCapMin = 384;
// Keys per row log of a kernel: at least kTkLogCapMin and room for `top` keys plus one
// tile's worth (a log is cut when the next tile could overflow it), in 64-key steps.
__host__ __device__ constexpr int tk_log_cap(int nk, int topr) {
  return ((topr + tk_vt(nk, 1) > kTkLogCapMin ? topr + tk_vt(nk, 1) : kTkLogCapMin) + 63) / 64 * 64;
}
// Query-row blocks per launch with logs (one log slab per block of a launch: at most
// 512 x 256 rows x 384 keys x 8 B = 403 MB at rank 128; a larger n_q runs in launches of
// this many blocks).
// All 10M users of configs[4], top-100: 6,733 ms with 512-block launches, 6,750 ms
// with 4096 (profiles/r06/ab_topk_logs.txt).  (A grid-stride loop over the blocks
// inside the kernel instead took every top-k kernel's registers to the 256 limit and
// spilled: not used.)
constexpr int kTkLogBlocks = 512;

// The T-th largest of the n keys of log L (n <= 64 J, 1 <= T <= n): the largest P
// with #{keys >= P} >= T.  Keys are unique ((score, V row) pairs), so exactly T keys are
// >= P.  The wave's lanes hold the keys (kv[j] = L[64 j + lane], 0 past n: below every
// real key).  A bitwise search over the 32 score bits first (the T-th largest score S);
// when the keys scoring S are exactly the ones still needed, P is the least of them (a
// min over the wave); only with more ties at S than needed does a second bitwise search
// over the index bits of those keys run.
template <int J>
__device__ __forceinline__ uint64_t tk_log_kth(const uint64_t (&kv)[J], int T) {
  uint32_t S = 0;
  for (int b = 31; b >= 0; --b) {
    const uint32_t cand = S | (1u << b);
    int c = 0;
#pragma unroll
    for (int j = 0; j < J; ++j) c += __popcll(__ballot((uint32_t)(kv[j] >> 32) >= cand));
    if (c >= T) S = cand;
  }
  int gt = 0, eq = 0;
  uint32_t lmin = 0xFFFFFFFFu;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const uint32_t h = (uint32_t)(kv[j] >> 32);
    gt += __popcll(__ballot(h > S));
    eq += __popcll(__ballot(h == S));
    if (h == S) lmin = min(lmin, (uint32_t)kv[j]);
  }
  const int need = T - gt;  // 1 <= need <= eq
  if (need == eq) {  // every key scoring S is kept: P is the least of them
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) lmin = min(lmin, (uint32_t)__shfl_xor((int)lmin, o));
    return ((uint64_t)S << 32) | lmin;
  }
  uint32_t L = 0;  // the need-th largest index word among the keys scoring S
  for (int b = 31; b >= 0; --b) {
    const uint32_t cand = L | (1u << b);
    int c = 0;
#pragma unroll
    for (int j = 0; j < J; ++j)
      c += __popcll(__ballot((uint32_t)(kv[j] >> 32) == S && (uint32_t)kv[j] >= cand));
    if (c >= need) L = cand;
  }
  return ((uint64_t)S << 32) | L;
}

// Wavefronts per workgroup: 8 with register lists (each V tile feeds 128 RG query
// rows), 4 with LDS lists (top > 128: the lists of 64 RG rows fill the LDS).
// (Quad lists with two row groups, one wavefront per SIMD, measured round 4 at
// configs[4]'s 262,144-user sample: top-100 390 ms vs 233 ms with one group.)
__host__ __device__ constexpr int tk_nw(int topr) { return topr > 0 ? 8 : 4; }
template <int NK, int RG, int TOPR>
__global__ __launch_bounds__(64 * tk_nw(TOPR)) void topk_split_kernel(const float* __restrict__ Q, int64_t n_q,
                                                         const uint4* __restrict__ Vsp,
                                                         const uint4* __restrict__ Vlo,
                                                         const int32_t* __restrict__ perm,
                                                         const float* __restrict__ vnorm,
                                                         int64_t n_v, int ld, int k, int top,
                                                         const float* __restrict__ scal,
                                                         int32_t* __restrict__ idx_out,
                                                         float* __restrict__ score_out,
                                                         uint64_t* __restrict__ tlog) {
  constexpr int NW = tk_nw(TOPR);  // wavefronts
  constexpr int GR = 16 * NW;          // query rows of a row group
  constexpr int KQ = 32 * NK;
  constexpr int RW = KQ / 8;           // uint4 per row of a split plane (KQ halves)
  constexpr int VT = tk_vt(NK, TOPR);  // V rows per tile
  constexpr int NC = VT / 16;          // 16-row score blocks per tile
  constexpr int NI = VT * RW / 64;     // LDS-DMA wave-instructions (1 KB) per tile
  constexpr int VP = VT < 64 ? 64 : VT;  // sweep-order indices staged per tile
  static_assert(NI % NW == 0 && VP % 64 == 0, "tile staging");
  extern __shared__ uint4 smem_u4[];
  constexpr int NBUF = tk_nbuf(TOPR);  // tile buffers: tiles t + 1 .. t + NBUF - 1 in flight
  // LDS-DMA loads per wave and tile: NI / NW pieces of V rows + one of sweep indices
  constexpr int PIECES = NI / NW + 1;
  uint4* tiles = smem_u4;                                       // [NBUF][VT][RW], swizzled
  int* tperm = reinterpret_cast<int*>(tiles + NBUF * VT * RW);  // [NBUF][VP] V row of each tile row
  int* sdone = tperm + NBUF * VP;                               // [2][NW] wave done flags
  float* sqs = reinterpret_cast<float*>(sdone + 2 * NW);      // [NW][RG][16] slack coefficients
  uint4* loscr = reinterpret_cast<uint4*>(sqs + GR * RG);     // [NW][NK][64] lo of a refined block
  // TOPR == 0: [GR RG rows][top] keys (best first), [GR RG] lengths
  // TOPR > 0: per wave and group a 16 x 16 score block [item m][row], then per wave
  // and group the rows' k-th scores
  uint64_t* lk = reinterpret_cast<uint64_t*>(loscr + NW * NK * 64);  // 16-byte aligned
  int* len = reinterpret_cast<int*>(lk + GR * RG * top);
  float* sblk = reinterpret_cast<float*>(lk);

  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, q = lane >> 4, m = lane & 15;
  const int swz = TK_SWZ(NK, m);  // the swizzle of every tile row this lane reads (row % 16 = m)
  const int64_t qbase = (int64_t)blockIdx.x * GR * RG;
  const int eu = tk_split_exponent(scal[0]), ev = tk_split_exponent(scal[1]);
  const float su = ldexpf(1.f, eu), unscale = ldexpf(1.f, -eu - ev);

  // A operands: group g, k-step s, lane (q, m): dims 32s + 8q .. +7 of query row
  // qbase + GR g + 16w + m, as hi and lo halves.
  tk_half8 ah[RG][NK], al[RG][NK];
  // live[g] bit rho: query row 16w + rho of group g exists and is not all zero (an
  // all-zero row scores 0 everywhere: its list is the first `top` rows, written at
  // the end; it would otherwise tie with every threshold)
  unsigned live[RG];
#pragma unroll
  for (int g = 0; g < RG; ++g) {
    const int64_t row = qbase + GR * g + 16 * w + m;
    const bool ok = row < n_q;
    bool nz = false;
    float ss = 0.f;
#pragma unroll
    for (int s = 0; s < NK; ++s) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int d = 32 * s + 8 * q + j;
        const float t = (ok && d < k) ? su * Q[row * ld + d] : 0.f;
        nz = nz || t != 0.f;
        ss = fmaf(t, t, ss);
        _Float16 h, l;
        tk_split(t, h, l);
        ah[g][s][j] = h;
        al[g][s][j] = l;
      }
    }
    const uint64_t b = __ballot(nz);
    live[g] = (unsigned)((b | (b >> 16) | (b >> 32) | (b >> 48)) & 0xFFFFu);
    ss += __shfl_xor(ss, 16);
    ss += __shfl_xor(ss, 32);
    // coarse-filter slack coefficient of row m, 2^-9 (|q| + 1): read from LDS once
    // per tile and after insertions
    if (q == 0) sqs[(w * RG + g) * 16 + m] = 0x1p-9f * (sqrtf(ss) + 1.f);
  }
  if (TOPR == 0 && threadIdx.x < GR * RG) len[threadIdx.x] = 0;
  // TOPR > 0: ts = the row's coarse threshold, k-th score - 2^-9 (|q| + 1)(NV + 1), NV
  // bounding |v| from the current tile on (the k-th scores live in LDS, thr);
  // TOPR == 0: (ts, ti) = the row's k-th (score, index).  Dead rows (absent or all
  // zero) keep an unbeatable threshold.
  float ts[RG][4];
  int ti[RG][4];
#pragma unroll
  for (int g = 0; g < RG; ++g)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      ts[g][r] = ((live[g] >> (4 * q + r)) & 1u) ? -__builtin_inff() : __builtin_inff();
      ti[g][r] = 0x7fffffff;
    }
  float* thr = sblk + NW * RG * 256 + w * RG * 16;  // TOPR > 0: [g][row] k-th scores
  if (TOPR > 0 && lane < 16 * RG)
    thr[lane] = ((live[lane >> 4] >> (lane & 15)) & 1u) ? -__builtin_inff() : __builtin_inff();
  // TOPR <= 16: this lane's row list (owner lanes lane < 16 RG).  LOGS (16 < TOPR): no
  // list in registers — every key reaching its row's threshold goes to the row's log
  // (tlog), and the threshold is the row's exact k-th best score as of the last cut of
  // its log (below)
  constexpr bool LOGS = TOPR > 16;
  constexpr int LCAP = tk_log_cap(NK, TOPR);  // LOGS: keys per row log
  constexpr int LJ = LCAP / 64;               // ... per lane when a wave holds a whole log
  static_assert(!LOGS || LCAP >= TOPR + VT, "a log holds top + one tile of keys");
  // TOPR == 0: all 16 RG lists of this wave hold `top` entries; LOGS: always true (a row
  // without a threshold yet has -inf, which the coarse test passes)
  bool full = LOGS;
  constexpr int NR = TOPR > 0 ? (LOGS ? 1 : TOPR) : 1;
  constexpr int KG = LOGS ? RG : 1;
  uint64_t kv[LOGS ? 1 : KG][LOGS ? 1 : NR];
  // LOGS: keys in the log of row 4q + r of group g, and that row's exact threshold (its
  // k-th best score at the last cut of its log; -inf before, +inf for dead rows): the
  // same in the 16 lanes of row group q
  int lcnt[LOGS ? KG : 1][LOGS ? 4 : 1];
  float tx[LOGS ? KG : 1][LOGS ? 4 : 1];
  if constexpr (LOGS) {
#pragma unroll
    for (int g = 0; g < KG; ++g)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        lcnt[g][r] = 0;
        tx[g][r] = ts[g][r];
      }
  } else {
#pragma unroll
    for (int g = 0; g < KG; ++g)
#pragma unroll
      for (int j = 0; j < NR; ++j) kv[g][j] = j < top ? kTkKeyOpen : kTkKeySentinel;
  }
  // LOGS: row (group g, row rho of this wave)'s log: LCAP keys in this block's slab
  auto rowlog = [&](int g, int rho) -> uint64_t* {
    return tlog + ((int64_t)blockIdx.x * GR * RG + GR * g + 16 * w + rho) * LCAP;
  };
  // LOGS: keep the `top` largest keys of row (g, rho)'s log (n > top keys), in place;
  // returns the score of the `top`-th (the row's exact k-th best so far: every key that
  // could rank above it reached the log, since the threshold never exceeded it)
  auto log_compact = [&](int g, int rho, int n) -> float {
    uint64_t* L = rowlog(g, rho);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's appends have landed
    uint64_t kl[LJ];
#pragma unroll
    for (int j = 0; j < LJ; ++j) kl[j] = 64 * j + lane < n ? L[64 * j + lane] : 0ull;
    const uint64_t P = tk_log_kth(kl, top);
    int base = 0;
#pragma unroll
    for (int j = 0; j < LJ; ++j) {
      const bool kp = kl[j] >= P;
      const uint64_t b = __ballot(kp);
      const int pos = base + __popcll(b & ((1ull << lane) - 1));
      if (kp) L[pos] = kl[j];
      base += __popcll(b);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return tk_key_score(P);
  };

  // Tile staging by LDS-DMA (global_load_lds_dwordx4: no VGPRs, no ds_write): the
  // workgroup's waves each issue NI / NW of the tile's 1 KB pieces.  Tile row r, uint4 c
  // lands at r RW + (c ^ TK_SWZ(NK, r)) (one DMA piece = 64 consecutive uint4), so the
  // B-operand reads stay conflict-free without padding.  Rows past n_v load row
  // n_v - 1; their scores are masked to NaN (score), so no filter passes them.
  auto issue_tile = [&](int64_t vb, int b) {
    if (n_v <= 0) return;  // (every wave alike: the vmcnt counts below stay uniform)
    uint4* t = tiles + b * VT * RW;
#pragma unroll
    for (int e = 0; e < NI / NW; ++e) {
      const int j = w * (NI / NW) + e;
      const int x = 64 * j + lane;
      const int r = x / RW;
      const int64_t vr = vb + r < n_v ? vb + r : n_v - 1;
      __builtin_amdgcn_global_load_lds(Vsp + vr * RW + ((x % RW) ^ TK_SWZ(NK, r)), t + 64 * j, 16,
                                       0, 0);
    }
    {  // piece w % (VP / 64): waves sharing a piece write the same words
      const int e = w % (VP / 64);
      const int64_t vr = vb + 64 * e + lane;
      __builtin_amdgcn_global_load_lds(perm + (vr < n_v ? vr : n_v - 1), tperm + b * VP + 64 * e,
                                       4, 0, 0);
    }
  };
  // norm of the current tile's first row: V is sorted by decreasing norm, so x
  // 2^(1/128) (one bucket) it bounds every row from that tile on
  float nv_cur = 0.f;
  // B operand: lane (q, m) holds dims 32s + 8q .. +7 of the block's V row m (reading
  // the B operands one block ahead in registers measured no faster: the sweep is not
  // bound by LDS latency, and the round-5 quad-list kernel then spilled)
  // (chk false: the caller masks rows past n_v itself — the quartet loop does it once per
  // quartet of the last tile, which keeps a per-block branch off its MFMA stream)
  auto score = [&](const uint4* tb, int64_t ibase, floatx4 (&acc)[RG], bool chk) {  // hi.hi
#pragma unroll
    for (int g = 0; g < RG; ++g) acc[g] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NK; ++s) {
      const tk_half8 bh = __builtin_bit_cast(tk_half8, tb[(4 * s + q) ^ swz]);
#pragma unroll
      for (int g = 0; g < RG; ++g)
        acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[g][s], bh, acc[g], 0, 0, 0);
    }
    if (chk && ibase + 16 > n_v) {  // the last tile: rows past n_v score NaN
      const bool past = ibase + m >= n_v;
#pragma unroll
      for (int g = 0; g < RG; ++g)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[g][r] = past ? __builtin_nanf("") : acc[g][r];
    }
  };

  // + hi.lo + lo.hi.  The lo halves of the block's V rows come from the lo plane in
  // global memory (only blocks past the coarse filter need them), by LDS-DMA into the
  // wave's scratch: each lane reads back the 16 B it loaded, and no VGPR holds them.
  auto refine = [&](const uint4* tb, int64_t ibase, floatx4 (&acc)[RG]) {
    const int64_t vr = ibase + m < n_v ? ibase + m : n_v - 1;  // rows past n_v: NaN anyway
    uint4* scr = loscr + w * NK * 64;
#pragma unroll
    for (int s = 0; s < NK; ++s)
      __builtin_amdgcn_global_load_lds(Vlo + vr * RW + 4 * s + q, scr + s * 64, 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int s = 0; s < NK; ++s) {
      const tk_half8 bh = __builtin_bit_cast(tk_half8, tb[(4 * s + q) ^ swz]);
      const tk_half8 bl = __builtin_bit_cast(tk_half8, scr[s * 64 + lane]);
#pragma unroll
      for (int g = 0; g < RG; ++g) {
        acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[g][s], bl, acc[g], 0, 0, 0);
        acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[g][s], bh, acc[g], 0, 0, 0);
      }
    }
  };
  // (|q| + 1)-free part of the slack bound: NV + 1 for the current tile
  float nvt = 1.f;
  // TOPR > 0: coarse thresholds from the k-th scores in thr
  auto refresh = [&]() {
#pragma unroll
    for (int g = 0; g < RG; ++g) {
      const floatx4 t4 = *reinterpret_cast<const floatx4*>(thr + 16 * g + 4 * q);
      const floatx4 s4 = *reinterpret_cast<const floatx4*>(sqs + (w * RG + g) * 16 + 4 * q);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool lv = (live[g] >> (4 * q + r)) & 1u;
        ts[g][r] = lv ? fmaf(-s4[r], nvt, t4[r]) : __builtin_inff();
        if constexpr (LOGS) tx[g][r] = lv ? t4[r] : __builtin_inff();
      }
    }
  };
  // acc: hi.hi scores of the block (refined in place when it passes the coarse
  // filter); tbr: the block's B rows in the tile
  auto filter = [&](floatx4 (&acc)[RG], int64_t ibase, const int* bperm, const uint4* tbr) {
    // acc[g][r] = scaled score(row GR g + 16w + 4q + r, V row ibase + m)
    if constexpr (LOGS) {
      // coarse: hi.hi >= the coarse threshold; then every exact score at or above its
      // row's threshold goes to the row's log, the 16 lanes of a row group placing
      // their keys by one ballot per row (no per-candidate pass).  Rows past n_v score
      // NaN and dead rows have +inf thresholds: nothing of theirs is appended.
      float dmax = -__builtin_inff();  // (as the quartet test)
#pragma unroll
      for (int g = 0; g < RG; ++g)
#pragma unroll
        for (int r = 0; r < 4; ++r) dmax = fmaxf(dmax, acc[g][r] - ts[g][r]);
      if (__ballot(dmax >= 0.f) == 0) return;
      refine(tbr, ibase, acc);
      const unsigned below = (1u << m) - 1u;
#pragma unroll
      for (int g = 0; g < RG; ++g)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool ok = acc[g][r] >= tx[g][r];
          const unsigned grp = (unsigned)(__ballot(ok) >> (16 * q)) & 0xFFFFu;
          if (ok) rowlog(g, 4 * q + r)[lcnt[g][r] + __popc(grp & below)] = tk_key(acc[g][r], bperm[m]);
          lcnt[g][r] += __popc(grp);
        }
      return;
    } else if constexpr (TOPR > 0) {
      // coarse: hi.hi >= the coarse threshold; then the exact scores go to the
      // owners against the same threshold (a weaker test than the k-th score: the
      // owner lanes compare exact (score, index) keys); until the lists are full
      // every block goes to the owners.  Rows past n_v score NaN: no test passes
      // them and the owners reject them.
      const bool fullw = __builtin_amdgcn_readfirstlane(full ? 1 : 0) != 0;
      if (fullw) {
        float dmax = -__builtin_inff();  // (as the quartet test)
#pragma unroll
        for (int g = 0; g < RG; ++g)
#pragma unroll
          for (int r = 0; r < 4; ++r) dmax = fmaxf(dmax, acc[g][r] - ts[g][r]);
        if (__ballot(dmax >= 0.f) == 0) return;
      }
      refine(tbr, ibase, acc);
      bool pr[RG][4];
#pragma unroll
      for (int g = 0; g < RG; ++g)
#pragma unroll
        for (int r = 0; r < 4; ++r) pr[g][r] = !fullw || acc[g][r] >= ts[g][r];
      float* st = sblk + w * RG * 256;  // [g][item m][row]
      uint64_t b[RG][4];
#pragma unroll
      for (int g = 0; g < RG; ++g) {
        *reinterpret_cast<floatx4*>(st + g * 256 + 16 * m + 4 * q) = acc[g];
#pragma unroll
        for (int r = 0; r < 4; ++r) b[g][r] = __ballot(pr[g][r]);
      }
      asm volatile("" ::: "memory");  // LDS is in order within the wave
      if (lane < 16 * RG) {  // owner lanes: group g = lane / 16, row rho
        const int g = lane >> 4, rho = lane & 15, sel = 4 * g + (rho & 3);
        uint64_t bb = b[0][0];
#pragma unroll
        for (int t = 1; t < 4 * RG; ++t) bb = sel == t ? b[t / 4][t % 4] : bb;
        unsigned msk = (unsigned)(bb >> (16 * (rho >> 2))) & 0xFFFFu;
        const float* sg = st + g * 256 + rho;
        while (msk) {
          const int mm = __builtin_ctz(msk);
          msk &= msk - 1;
          const float sc = sg[16 * mm];
          const uint64_t c = tk_key(sc, bperm[mm]);
          if (sc == sc && c > kv[0][0]) tk_insert<NR>(kv[0], c);
        }
        thr[lane] = kv[0][0] == kTkKeyOpen ? -__builtin_inff() : tk_key_score(kv[0][0]);
      }
      asm volatile("" ::: "memory");
      refresh();
      if (!full) {
        const bool open_list = lane < 16 * RG && ((live[lane >> 4] >> (lane & 15)) & 1u) &&
                               kv[0][0] == kTkKeyOpen;
        full = __ballot(open_list) == 0;
      }
      return;
    }
    const bool vin = ibase + m < n_v;
    if (full) {
      float dmax = -__builtin_inff();  // (as the quartet test)
#pragma unroll
      for (int g = 0; g < RG; ++g) {
        const floatx4 s4 = *reinterpret_cast<const floatx4*>(sqs + (w * RG + g) * 16 + 4 * q);
#pragma unroll
        for (int r = 0; r < 4; ++r) dmax = fmaxf(dmax, acc[g][r] - fmaf(-s4[r], nvt, ts[g][r]));
      }
      if (__ballot(vin && dmax >= 0.f) == 0) return;
    }
    refine(tbr, ibase, acc);
#pragma unroll
    for (int g = 0; g < RG; ++g) {
      bool hit = !full;
      if (full) {
        const bool p = vin && (acc[g][0] >= ts[g][0] || acc[g][1] >= ts[g][1] ||
                               acc[g][2] >= ts[g][2] || acc[g][3] >= ts[g][3]);
        hit = __ballot(p) != 0;
      }
      if (hit)
        topk_offer(acc[g], (int)ibase, n_v, bperm, ts[g], ti[g], lk, len, GR * g + 16 * w,
                   top, live[g]);
    }
    if (!full) {
      bool f = true;
      if (lane < 16 * RG && ((live[lane >> 4] >> (lane & 15)) & 1u))
        f = len[GR * (lane >> 4) + 16 * w + (lane & 15)] >= top;
      full = __ballot(!f) == 0;
    }
  };

  // tile t in buffer t % NBUF; tiles t + 1 .. t + NBUF - 1 are in flight while tile t is
  // scored (tiles past the sweep too, clamped: every wave issues the same loads, so the
  // vmcnt counts are exact); each wave waits for its own pieces of tile t + 1 before the
  // barrier that ends tile t, which also releases tile t's buffer for tile t + NBUF
  // (__syncthreads() would wait for every load in flight, the later tiles' included:
  // the barriers here wait for this wave's LDS accesses and its pieces of one tile only)
  for (int i = 0; i < NBUF; ++i) issue_tile(i * VT, i);
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" :: "n"(PIECES * (NBUF - 1)) : "memory");
  int buf = 0, par = 0;
  // one tile: score + filter tile vb in buffer buf, barrier, issue tile vb + NBUF VT into
  // buffer buf; false: sweep over
  auto tile_step = [&](int64_t vb) -> bool {
      const uint4* tb = tiles + buf * VT * RW;
      if constexpr (LOGS) {
        // a log that this tile could overflow (at most VT appends per row) is cut to
        // its row's `top` best keys first, and the row's threshold rises to the k-th of
        // them (refresh() below reads it)
#pragma unroll
        for (int g = 0; g < KG; ++g)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            // (cutting more often — at top + 32 / 64 / 128 keys, or as soon as a row
            // first holds `top` — measured slower: the cuts cost more than the fresher
            // thresholds save; profiles/r06/ab_topk_logs.txt)
            uint64_t nb = __ballot(m == 0 && lcnt[g][r] > LCAP - VT);
            while (nb) {
              const int L0 = __builtin_ctzll(nb);  // lane 16 qq: row 4 qq + r
              nb &= nb - 1;
              const int rho = 4 * (L0 >> 4) + r;
              const float t = log_compact(g, rho, __builtin_amdgcn_readlane(lcnt[g][r], L0));
              if (lane == 0) thr[16 * g + rho] = t;
              if (q == (L0 >> 4)) lcnt[g][r] = top;
            }
          }
        asm volatile("" ::: "memory");  // the thresholds are read back below (LDS in order)
      }
      nv_cur = n_v > 0 ? vnorm[vb] : 0.f;
      nvt = fmaf(nv_cur, 1.01f, 1.f);
      // early exit: every row of the wave holds a k-th score that no row from this
      // tile on can reach: k-th > (|q| + 1)(NV + 1)(1 + 2^-7) (dead rows: +inf)
      bool open = false;
      if constexpr (TOPR > 0) {
        refresh();
#pragma unroll
        for (int g = 0; g < RG; ++g) {
          const floatx4 t4 = *reinterpret_cast<const floatx4*>(thr + 16 * g + 4 * q);
          const floatx4 s4 = *reinterpret_cast<const floatx4*>(sqs + (w * RG + g) * 16 + 4 * q);
#pragma unroll
          for (int r = 0; r < 4; ++r)
            open = open || (((live[g] >> (4 * q + r)) & 1u) && !(t4[r] > (0x1p9f + 4.f) * s4[r] * nvt));
        }
      } else {
#pragma unroll
        for (int g = 0; g < RG; ++g) {
          const floatx4 s4 = *reinterpret_cast<const floatx4*>(sqs + (w * RG + g) * 16 + 4 * q);
#pragma unroll
          for (int r = 0; r < 4; ++r) open = open || !(ts[g][r] > (0x1p9f + 4.f) * s4[r] * nvt);
        }
      }
      const bool wdone = __ballot(open) == 0;
      if (!wdone) {
        floatx4 acc0[RG], acc1[RG];
        if constexpr (TOPR > 0) {
          constexpr int NB4 = 4;  // blocks per ballot
          static_assert(NC % NB4 == 0, "quartets of 16-row blocks per tile");
          // four blocks scored back to back, then one ballot for all four against the
          // current coarse thresholds (they only rise, so a quartet with no pair past
          // them has none past the later ones): the LDS -> MFMA -> compare -> branch
          // latency of a block is paid once per 64 V rows.  Measured on the configs[4]
          // 262,144-user sample against block pairs (the path below): top-10 97.3 ->
          // 91.5 ms, top-100 233 -> 194 ms.
          floatx4 a4[NB4][RG];
#pragma unroll 1
          for (int c = 0; c < NC; c += NB4) {
            const uint4* tbr = tb + (16 * c + m) * RW;
            const int* bp = tperm + buf * VP + 16 * c;
            // the quartet's hi.hi scores, k-step outermost: each step's B operands of the
            // four blocks, then 4 RG independent MFMAs (a dependent MFMA comes 4 RG issues
            // later, not RG)
#pragma unroll
            for (int j = 0; j < NB4; ++j)
#pragma unroll
              for (int g = 0; g < RG; ++g) a4[j][g] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < NK; ++s) {
              tk_half8 bh[NB4];
#pragma unroll
              for (int j = 0; j < NB4; ++j)
                bh[j] = __builtin_bit_cast(tk_half8, tbr[16 * j * RW + ((4 * s + q) ^ swz)]);
#pragma unroll
              for (int j = 0; j < NB4; ++j)
#pragma unroll
                for (int g = 0; g < RG; ++g)
                  a4[j][g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[g][s], bh[j], a4[j][g], 0, 0, 0);
            }
            if (vb + 16 * (c + NB4) > n_v) {  // (uniform) the last tile: rows past n_v score NaN
#pragma unroll
              for (int j = 0; j < NB4; ++j) {
                const bool past = vb + 16 * (c + j) + m >= n_v;
#pragma unroll
                for (int g = 0; g < RG; ++g)
#pragma unroll
                  for (int r = 0; r < 4; ++r) a4[j][g][r] = past ? __builtin_nanf("") : a4[j][g][r];
              }
            }
            if (__builtin_amdgcn_readfirstlane(full ? 1 : 0) != 0) {
              // any pair past its row's coarse threshold: max over the blocks, then over
              // (score - threshold) — straight VALU, no compare-and-branch chain (fmaxf
              // drops the NaN of rows past n_v; +inf thresholds give -inf)
              float dmax = -__builtin_inff();
#pragma unroll
              for (int g = 0; g < RG; ++g)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                  float mx = a4[0][g][r];
#pragma unroll
                  for (int j = 1; j < NB4; ++j) mx = fmaxf(mx, a4[j][g][r]);
                  dmax = fmaxf(dmax, mx - ts[g][r]);
                }
              if (__ballot(dmax >= 0.f) == 0) continue;
            }
#pragma unroll
            for (int j = 0; j < NB4; ++j)
              filter(a4[j], vb + 16 * (c + j), bp + 16 * j, tbr + 16 * j * RW);
          }
        } else {
        score(tb + m * RW, vb, acc0, true);
        // block pairs: issue block c+1's MFMAs, then filter block c
#pragma unroll 1
        for (int c = 0; c < NC; c += 2) {
          const uint4* tbr = tb + (16 * c + m) * RW;
          const int* bp = tperm + buf * VP + 16 * c;
          if (NC > 1) score(tbr + 16 * RW, vb + 16 * c + 16, acc1, true);
          filter(acc0, vb + 16 * c, bp, tbr);
          if (NC > 1) {
            if (c + 2 < NC) score(tbr + 32 * RW, vb + 16 * c + 32, acc0, true);
            filter(acc1, vb + 16 * c + 16, bp + 16, tbr + 16 * RW);
          }
        }
        }
      }
      // this wave's pieces of tile vb + VT (the later tiles' may stay in flight)
      if (lane == 0) sdone[par * NW + w] = wdone ? 1 : 0;
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" :: "n"(PIECES * (NBUF - 2)) : "memory");
      // (flags of this parity are rewritten only after the next barrier)
      int alldone = 1;
#pragma unroll
      for (int i = 0; i < NW; ++i) alldone &= sdone[par * NW + i];
      if (alldone) return false;
      issue_tile(vb + NBUF * VT, buf);
      buf = buf + 1 == NBUF ? 0 : buf + 1;
      par ^= 1;
      return vb + VT < n_v;
  };
  for (int64_t vb = 0;; vb += VT)
    if (!tile_step(vb)) break;
  // no LDS-DMA may still be landing when the workgroup ends
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (LOGS) {
    // each row's `top` largest keys, selected exactly from its log, ranked and written
    // in order; fewer than `top` keys (n_v < top) leave the tail open
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's log appends landed
    uint64_t* ks = reinterpret_cast<uint64_t*>(sblk + w * RG * 256);  // <= 128 keys (1 KB)
    // (g unrolled: a runtime index into lcnt / live would put those arrays in scratch
    // memory for the whole kernel, a scratch round trip per tile of the sweep)
#pragma unroll
    for (int g = 0; g < KG; ++g) {
#pragma unroll 1
      for (int rho = 0; rho < 16; ++rho) {
        const int64_t row = qbase + GR * g + 16 * w + rho;
        if (row >= n_q) break;
        if (!((live[g] >> rho) & 1u)) {  // every score 0: the first `top` rows, ties by index
          for (int e = lane; e < top; e += 64) {
            idx_out[row * top + e] = e < n_v ? e : -1;
            score_out[row * top + e] = e < n_v ? 0.f : -__builtin_inff();
          }
          continue;
        }
        const int rq = rho & 3;
        const int cr = rq == 0 ? lcnt[g][0] : (rq == 1 ? lcnt[g][1] : (rq == 2 ? lcnt[g][2] : lcnt[g][3]));
        const int n = __builtin_amdgcn_readlane(cr, 16 * (rho >> 2));
        const uint64_t* L = rowlog(g, rho);
        uint64_t kl[LJ];
#pragma unroll
        for (int j = 0; j < LJ; ++j) kl[j] = 64 * j + lane < n ? L[64 * j + lane] : 0ull;
        const int T = n < top ? n : top;
        const uint64_t P = n > top ? tk_log_kth(kl, T) : 1ull;  // real keys are >= 1
        int base = 0;
#pragma unroll
        for (int j = 0; j < LJ; ++j) {
          const bool kp = kl[j] >= P;
          const uint64_t b = __ballot(kp);
          if (kp) ks[base + __popcll(b & ((1ull << lane) - 1))] = kl[j];
          base += __popcll(b);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        for (int e = lane; e < T; e += 64) {
          const uint64_t key = ks[e];
          int r = 0;
          for (int t = 0; t < T; ++t) r += ks[t] > key ? 1 : 0;
          idx_out[row * top + r] = tk_key_index(key);
          score_out[row * top + r] = tk_key_score(key) * unscale;
        }
        for (int e = T + lane; e < top; e += 64) {
          idx_out[row * top + e] = -1;
          score_out[row * top + e] = -__builtin_inff();
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // ks is rewritten for the next row
      }
    }
    return;
  } else if constexpr (TOPR > 0) {
    if (lane < 16 * RG) {
      const int64_t row = qbase + GR * (lane >> 4) + 16 * w + (lane & 15);
      const bool zero = !((live[lane >> 4] >> (lane & 15)) & 1u);
      if (row < n_q) {
#pragma unroll
        for (int j = 0; j < NR; ++j) {
          if (j < top) {
            const int e = top - 1 - j;
            if (zero) {  // every score 0: the first `top` rows, ties by index
              idx_out[row * top + e] = e < n_v ? e : -1;
              score_out[row * top + e] = e < n_v ? 0.f : -__builtin_inff();
            } else {
              const bool real = kv[0][j] != kTkKeyOpen;
              idx_out[row * top + e] = real ? tk_key_index(kv[0][j]) : -1;
              score_out[row * top + e] = real ? tk_key_score(kv[0][j]) * unscale : -__builtin_inff();
            }
          }
        }
      }
    }
    return;
  }
#pragma unroll
  for (int g = 0; g < RG; ++g)
    topk_write(lk, len, GR * g + 16 * w, qbase, n_q, n_v, top, unscale, live[g], idx_out,
               score_out);
}

static int topk_kq(int k) { return k <= 32 ? 32 : (k <= 64 ? 64 : 128); }

constexpr int kTopR = 16;   // one owner lane's register list for top <= kTopR (sized 8 / 12 / 16)
constexpr int kTopQ = 128;  // key logs for kTopR < top <= kTopQ (32 / 64 / 100 / 128)

// Key logs for kTopR < top <= kTopQ.  (Round 4's quad register lists measured at rank
// 128, top 100 against the LDS lists: 59,047 V rows 70 -> 21 ms, 1,000,000 V rows 456 ->
// 330 ms; the logs replaced them in round 6.)
static bool topk_logs(int top, int64_t n_v) {
  (void)n_v;
  return top > kTopR && top <= kTopQ;
}

static int topk_nw(int top, bool logs, int rg) {
  return logs ? tk_nw(kTopQ) : (top <= kTopR ? tk_nw(1) : tk_nw(0));
}

static size_t topk_split_lds_bytes(int kq, int rg, int top, bool logs) {
  const int nk = kq / 32;
  const int nw = topk_nw(top, logs, rg);
  const bool reg_lists = top <= kTopR || logs;
  const size_t vt = (size_t)tk_vt(nk, reg_lists ? 1 : 0);
  // [nbuf][vt] tile rows of KQ hi halves (kq/8 uint4) | [nbuf][max(vt, 64)] V rows |
  // [2][nw] done flags | [nw][rg][16] slack coefficients | [nw][nk][64] uint4 lo scratch
  const size_t nbuf = (size_t)tk_nbuf(reg_lists ? 1 : 0);
  const size_t tiles = 16 * nbuf * vt * (size_t)(kq / 8) + 4 * nbuf * std::max<size_t>(vt, 64) + 4 * 2 * nw +
                       4 * 16 * nw * (size_t)rg + 16 * nw * 64 * (size_t)nk;
  if (reg_lists) return tiles + sizeof(float) * nw * (size_t)rg * (256 + 16);
  return tiles + sizeof(uint64_t) * 64 * (size_t)rg * top +
         sizeof(int) * 64 * (size_t)rg;
}

// Row groups per workgroup of the split kernel (0: its lists do not fit the LDS).
// Two groups halve the V traffic per query row, but LDS lists (top > kTopR) of
// two groups must still leave room for two workgroups per CU: the list inserts
// are latency-bound and need the second workgroup (measured, configs[4] top-100
// at rank 128: one 120 KB workgroup per CU 602 ms, two 68 KB ones 480 ms).
// Register lists take two groups (256 query rows per 8-wave workgroup) only when
// that still gives >= 4 workgroups per CU: measured top-10, ML-25M shape (162,541
// users, rank 64) 4.7 ms with two groups, 3.6 ms with one (the tail of 2.5 rounds);
// configs[4] (262,144-user sample, rank 128) 97 ms with two, 151 ms with one.
constexpr int64_t kTkRg2MinRows = 4 * 256 * 256;
static int topk_split_rg(int k, int top, bool logs, int64_t n_q) {
  const int kq = topk_kq(k);
  // register lists and key logs: two row groups on the same condition (the logs keep
  // no list in registers, so two groups' A operands and accumulators fit)
  if ((top <= kTopR || logs) && n_q < kTkRg2MinRows) return 1;
  if (logs) return 2;
  const size_t rg2_limit = top > kTopR ? (size_t)kLdsBytes / 2 : (size_t)kLdsBytes;
  if (topk_split_lds_bytes(kq, 2, top, false) <= rg2_limit) return 2;
  if (topk_split_lds_bytes(kq, 1, top, false) <= (size_t)kLdsBytes) return 1;
  return 0;
}

}  // namespace als

using namespace als;

extern "C" {

static size_t tk_table_bytes(int64_t n_v, int32_t k) {
  return align_up(4 * (size_t)topk_kq(k) * (size_t)(n_v > 0 ? n_v : 0));
}

// Per-row key logs (16 < top <= 128): tk_log_cap keys for every query
// row of one launch's blocks (at most kTkLogBlocks blocks per launch).
static size_t tk_log_bytes(int64_t n_q, int32_t k, int32_t top) {
  if (n_q <= 0 || !topk_logs(top, 0)) return 0;
  const int rg = topk_split_rg(k, top, true, n_q);
  const int64_t rows = 16 * (int64_t)tk_nw(kTopQ) * rg;  // query rows per block
  const int64_t blocks = std::min<int64_t>((n_q + rows - 1) / rows, kTkLogBlocks);
  const int topr = top <= 32 ? 32 : (top <= 64 ? 64 : (top <= 100 ? 100 : kTopQ));
  return align_up(sizeof(uint64_t) * (size_t)(blocks * rows) *
                  (size_t)tk_log_cap(topk_kq(k) / 32, topr));
}

size_t als_topk_workspace_bytes(int64_t n_q, int64_t n_v, int32_t k, int32_t top) {
  // 256 B of scale words | split planes of V in sweep order (2 x KQ halves per row) |
  // sweep order (int32 per V row) | bucket counts / cursors | scaled row norms in
  // sweep order (fp32 per V row) | 16 < top <= 128: per-row key logs
  return 256 + tk_table_bytes(n_v, k) + 2 * align_up(4 * (size_t)(n_v > 0 ? n_v : 0)) +
         align_up(4 * (size_t)kTkBuckets) + tk_log_bytes(n_q, k, top);
}

int als_topk(const float* Q, int64_t n_q, const float* V, int64_t n_v, int32_t ld, int32_t k,
             int32_t top, int32_t* idx_out, float* score_out, void* ws, size_t ws_bytes,
             void* stream) {
  ALS_REQUIRE(k >= 1 && k <= 128, ALS_EUNSUPPORTED, "als_topk: rank %d not in [1, 128]", k);
  ALS_REQUIRE(ld >= k && ld % 4 == 0, ALS_EINVAL, "als_topk: bad ld");
  ALS_REQUIRE(top >= 1 && top <= kTopkMax, ALS_EUNSUPPORTED, "als_topk: top %d not in [1, %d]",
              top, kTopkMax);
  ALS_REQUIRE(n_q >= 0 && n_v >= 0 && n_v < (int64_t(1) << 31), ALS_EINVAL,
              "als_topk: bad sizes");
  if (n_q == 0) return ALS_OK;
  ALS_REQUIRE(Q && V && idx_out && score_out, ALS_EINVAL, "als_topk: null pointer");
  hipStream_t st = as_stream(stream);
  const bool logs = topk_logs(top, n_v);
  const int rg = topk_split_rg(k, top, logs, n_q);
  ALS_REQUIRE(rg > 0, ALS_EUNSUPPORTED, "als_topk: top %d at rank %d does not fit the LDS", top,
              k);
  ALS_REQUIRE(ws != nullptr && ws_bytes >= als_topk_workspace_bytes(n_q, n_v, k, top),
              ALS_EWORKSPACE, "als_topk: workspace %zu < %zu", ws_bytes,
              als_topk_workspace_bytes(n_q, n_v, k, top));
  ALS_REQUIRE((reinterpret_cast<uintptr_t>(ws) & 15) == 0, ALS_EINVAL,
              "als_topk: workspace must be 16-byte aligned");
  unsigned* scal_u = static_cast<unsigned*>(ws);
  const float* scal = reinterpret_cast<const float*>(scal_u);
  _Float16* vsp = reinterpret_cast<_Float16*>(static_cast<char*>(ws) + 256);
  int32_t* perm = reinterpret_cast<int32_t*>(static_cast<char*>(ws) + 256 + tk_table_bytes(n_v, k));
  int32_t* hist = perm + align_up(4 * (size_t)n_v) / 4;
  float* vnorm = reinterpret_cast<float*>(hist + align_up(4 * (size_t)kTkBuckets) / 4);
  uint64_t* tlog = reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(vnorm) +
                                               align_up(4 * (size_t)(n_v > 0 ? n_v : 0)));
  const int kq = topk_kq(k);
  const int kq_shift = __builtin_ctz(kq);
  ALS_HIP(hipMemsetAsync(scal_u, 0, 2 * sizeof(unsigned), st));
  const int64_t nq_el = n_q * (int64_t)ld, nv_el = n_v * (int64_t)ld;
  tk_absmax_kernel<<<(int)std::min<int64_t>(256, (nq_el / 4 + 255) / 256 + 1), 256, 0, st>>>(
      Q, nq_el, scal_u);
  ALS_LAUNCH_CHECK();
  if (n_v > 0) {
    tk_absmax_kernel<<<(int)std::min<int64_t>(256, (nv_el / 4 + 255) / 256 + 1), 256, 0, st>>>(
        V, nv_el, scal_u + 1);
    ALS_LAUNCH_CHECK();
    // sweep order: V rows by decreasing norm (bucketed)
    ALS_HIP(hipMemsetAsync(hist, 0, sizeof(int32_t) * kTkBuckets, st));
    const int gb = (int)std::min<int64_t>(512, (n_v * 16 + 255) / 256);
    tk_bucket_hist_kernel<<<gb, 256, 0, st>>>(V, n_v, ld, k, scal, hist);
    ALS_LAUNCH_CHECK();
    tk_bucket_scan_kernel<<<1, 1024, 0, st>>>(hist);
    ALS_LAUNCH_CHECK();
    tk_bucket_scatter_kernel<<<gb, 256, 0, st>>>(V, n_v, ld, k, scal, hist, perm);
    ALS_LAUNCH_CHECK();
    const int64_t total = n_v << kq_shift;
    topk_split_table_kernel<<<(int)std::min<int64_t>(4096, (total + 255) / 256), 256, 0, st>>>(
        V, n_v, ld, k, kq_shift, scal, perm, vsp);
    ALS_LAUNCH_CHECK();
    tk_table_norm_kernel<<<(int)std::min<int64_t>(4096, (n_v * 16 + 255) / 256), 256, 0, st>>>(
        V, n_v, ld, k, scal, perm, vnorm);
    ALS_LAUNCH_CHECK();
  }
  const size_t lds = topk_split_lds_bytes(kq, rg, top, logs);
  const int nw = topk_nw(top, logs, rg);  // wavefronts per workgroup
  const int64_t rows_blk = 16 * (int64_t)nw * rg;
  const int64_t n_blk = (n_q + rows_blk - 1) / rows_blk;
  // key logs: launches of at most kTkLogBlocks blocks (one log slab per block)
  const int64_t blk_per = logs ? (int64_t)kTkLogBlocks : n_blk;
  const uint4* vsp4 = reinterpret_cast<const uint4*>(vsp);
  const uint4* vlo4 = vsp4 + n_v * (kq / 8);  // lo plane
#define ALS_TOPK_SPLIT_LAUNCH2(NK, RG, TR)                                                      \
  do {                                                                                          \
    ALS_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&topk_split_kernel<NK, RG, TR>),  \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));         \
    for (int64_t b0 = 0; b0 < n_blk; b0 += blk_per) {                                           \
      const int64_t r0 = b0 * rows_blk;                                                         \
      const int64_t nq_c = std::min<int64_t>(n_q - r0, blk_per * rows_blk);                     \
      const unsigned grid = (unsigned)((nq_c + rows_blk - 1) / rows_blk);                       \
      topk_split_kernel<NK, RG, TR><<<grid, 64 * nw, lds, st>>>(                                \
          Q + r0 * ld, nq_c, vsp4, vlo4, perm, vnorm, n_v, ld, k, top, scal, idx_out + r0 * top, \
          score_out + r0 * top, tlog);                                                          \
      ALS_LAUNCH_CHECK();                                                                       \
    }                                                                                           \
  } while (0)
#define ALS_TOPK_SPLIT_LAUNCH(NK, RG)                 \
  do {                                                \
    if (top <= 8)                                     \
      ALS_TOPK_SPLIT_LAUNCH2(NK, RG, 8);              \
    else if (top <= 12)                               \
      ALS_TOPK_SPLIT_LAUNCH2(NK, RG, 12);             \
    else if (top <= kTopR)                            \
      ALS_TOPK_SPLIT_LAUNCH2(NK, RG, kTopR);          \
    else if (!logs)                                   \
      ALS_TOPK_SPLIT_LAUNCH2(NK, RG, 0);              \
    else if (top <= 32)                               \
      ALS_TOPK_SPLIT_LAUNCH2(NK, RG, 32);             \
    else if (top <= 64)                               \
      ALS_TOPK_SPLIT_LAUNCH2(NK, RG, 64);             \
    else if (top <= 100)                              \
      ALS_TOPK_SPLIT_LAUNCH2(NK, RG, 100);            \
    else                                              \
      ALS_TOPK_SPLIT_LAUNCH2(NK, RG, kTopQ);          \
  } while (0)
  if (kq == 32) {
    if (rg == 2) ALS_TOPK_SPLIT_LAUNCH(1, 2);
    else ALS_TOPK_SPLIT_LAUNCH(1, 1);
  } else if (kq == 64) {
    if (rg == 2) ALS_TOPK_SPLIT_LAUNCH(2, 2);
    else ALS_TOPK_SPLIT_LAUNCH(2, 1);
  } else {
    if (rg == 2) ALS_TOPK_SPLIT_LAUNCH(4, 2);
    else ALS_TOPK_SPLIT_LAUNCH(4, 1);
  }
#undef ALS_TOPK_SPLIT_LAUNCH
#undef ALS_TOPK_SPLIT_LAUNCH2
  return ALS_OK;
}

}  // extern "C"
