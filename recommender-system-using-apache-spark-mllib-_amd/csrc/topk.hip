// K5 — recommendForAll: blocked U.V^T on the matrix cores with a fused,
// bounded per-row top-k.  The n_q x n_v score matrix is never materialised.
//
// Replaces ALSModel.recommendForAll (upstream Spark >= 2.2: blockify at 4096
// rows, crossJoin, sgemm per block pair, bounded priority queue,
// TopByKeyAggregator merge) and mllib recommendProductsForUsers.  The
// reference's own top-k is `predictAll` over one user's unrated movies then
// `takeOrdered(20, key=-pred)` (RecommenderSystem.py:229-247).
//
// Workgroup = 4 wavefronts = 64 query rows (16 per wave).  The workgroup
// sweeps V in 64-row tiles staged in LDS (rows padded by 16 B: the 16 lanes
// of a row-group read 16 distinct bank slots).  Per tile each wave computes a
// 16 x 64 score block with v_mfma_f32_16x16x4_f32 (fp32 in, fp32 accumulate:
// Spark's ml path is fp32 sgemm too), then filters it against each row's
// current k-th best (score, index) and inserts the rare survivors into a
// sorted list in LDS with a wave-cooperative insertion.  Order: score
// descending, ties by ascending index (the build's deterministic tie rule,
// SURVEY Appendix A.6).
#include "als_common.h"

namespace als {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kTopkMax = 256;
constexpr int kLdsBytes = 160 * 1024;  // per CU on gfx950 (one workgroup may use it all)

__device__ __forceinline__ bool beats(float s1, int i1, float s2, int i2) {
  return s1 > s2 || (s1 == s2 && i1 < i2);
}

template <int CN>
__global__ __launch_bounds__(256) void topk_kernel(const float* __restrict__ Q, int64_t n_q,
                                                   const float* __restrict__ V, int64_t n_v,
                                                   int ld, int k, int top,
                                                   int32_t* __restrict__ idx_out,
                                                   float* __restrict__ score_out) {
  constexpr int KP = 16 * CN;
  constexpr int KS = KP / 4;      // MFMA k-steps; lane q covers dims [q*KS, q*KS+KS)
  constexpr int TS = KP + 4;      // padded tile row stride (floats)
  extern __shared__ float4 smem4[];
  float* tile = reinterpret_cast<float*>(smem4);        // [64][TS]
  float* ls = tile + 64 * TS;                           // [64 rows][top] scores
  int* li = reinterpret_cast<int*>(ls + 64 * top);      // [64 rows][top] indices
  int* len = li + 64 * top;                             // [64]

  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, q = lane >> 4, m = lane & 15;
  const int64_t qbase = (int64_t)blockIdx.x * 64;

  // A operand (query rows): lane (m, q) holds dims q*KS + s of row qbase + 16w + m.
  float qa[KS];
  {
    const int64_t row = qbase + 16 * w + m;
    const bool ok = row < n_q;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int d = q * KS + s;
      qa[s] = (ok && d < k) ? Q[row * ld + d] : 0.f;
    }
  }
  if (threadIdx.x < 64) len[threadIdx.x] = 0;
  // per-lane thresholds of its 4 rows (16w + 4q + r)
  float ts[4];
  int ti[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    ts[r] = -__builtin_inff();
    ti[r] = 0x7fffffff;
  }

  for (int64_t vb = 0; vb < n_v; vb += 64) {
    __syncthreads();
    // stage 64 V rows x KP dims (float4 granules), masked beyond n_v / k
    for (int e = threadIdx.x; e < 64 * (KP / 4); e += 256) {
      const int rr = e / (KP / 4), c4 = e % (KP / 4);
      const int64_t vrow = vb + rr;
      const int d = 4 * c4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (vrow < n_v && d < k) {
        v = *reinterpret_cast<const float4*>(V + vrow * ld + d);
        if (d + 1 >= k) v.y = 0.f;
        if (d + 2 >= k) v.z = 0.f;
        if (d + 3 >= k) v.w = 0.f;
      }
      *reinterpret_cast<float4*>(tile + rr * TS + d) = v;
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      // B operand: lane (m, q) holds dims q*KS + s of V row vb + 16c + m
      const float* tb = tile + (16 * c + m) * TS + q * KS;
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s4 = 0; s4 < KS; s4 += 4) {
        const float4 b4 = *reinterpret_cast<const float4*>(tb + s4);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(qa[s4 + 0], b4.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(qa[s4 + 1], b4.y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(qa[s4 + 2], b4.z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(qa[s4 + 3], b4.w, acc, 0, 0, 0);
      }
      // acc[r] = score(row 16w + 4q + r, V row vb + 16c + m)
      const int vidx = (int)(vb + 16 * c + m);
      const bool vin = (vb + 16 * c + m) < n_v;
      int pend = 0;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (vin && beats(acc[r], vidx, ts[r], ti[r])) pend |= 1 << r;
      uint64_t any = __ballot(pend != 0);
      while (any) {
        const int L = __builtin_ctzll(any);
        const int myr = pend ? __builtin_ctz(pend) : 0;
        const float mys = myr == 0 ? acc[0] : (myr == 1 ? acc[1] : (myr == 2 ? acc[2] : acc[3]));
        const int rL = __builtin_amdgcn_readlane(myr, L);
        const float sc = __builtin_bit_cast(float,
                                            __builtin_amdgcn_readlane(__builtin_bit_cast(int, mys), L));
        const int itm = (int)(vb + 16 * c + (L & 15));
        const int slot = 16 * w + 4 * (L >> 4) + rL;  // list row within the workgroup
        float* lsr = ls + slot * top;
        int* lir = li + slot * top;
        const int n = len[slot];
        // rank = number of entries that beat the candidate
        int pos = 0;
        for (int e0 = 0; e0 < n; e0 += 64) {
          const int e = e0 + lane;
          const bool bt = e < n && beats(lsr[e], lir[e], sc, itm);
          pos += __popcll(__ballot(bt));
        }
        if (pos < top) {
          const int newn = n + 1 < top ? n + 1 : top;
          float hs[kTopkMax / 64];
          int hi[kTopkMax / 64];
#pragma unroll
          for (int j = 0; j < kTopkMax / 64; ++j) {
            const int e = 64 * j + lane;
            if (e > pos && e < newn) {
              hs[j] = lsr[e - 1];
              hi[j] = lir[e - 1];
            }
          }
          // reads of the shifted entries land before any lane writes (compiler + HW order)
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
          for (int j = 0; j < kTopkMax / 64; ++j) {
            const int e = 64 * j + lane;
            if (e > pos && e < newn) {
              lsr[e] = hs[j];
              lir[e] = hi[j];
            }
          }
          if (lane == 0) {
            lsr[pos] = sc;
            lir[pos] = itm;
            len[slot] = newn;
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          if (newn == top) {
            const float ks = lsr[top - 1];
            const int ki = lir[top - 1];
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
  }
  __syncthreads();
  // write each wave's 16 lists
  for (int rr = 0; rr < 16; ++rr) {
    const int slot = 16 * w + rr;
    const int64_t row = qbase + slot;
    if (row >= n_q) break;
    const int n = len[slot];
    for (int e = lane; e < top; e += 64) {
      idx_out[row * top + e] = e < n ? li[slot * top + e] : -1;
      score_out[row * top + e] = e < n ? ls[slot * top + e] : -__builtin_inff();
    }
  }
}

static size_t topk_lds_bytes(int cn, int top) {
  const int kp = 16 * cn;
  return sizeof(float) * 64 * (kp + 4) + (sizeof(float) + sizeof(int)) * 64 * (size_t)top +
         sizeof(int) * 64;
}

}  // namespace als

using namespace als;

extern "C" {

size_t als_topk_workspace_bytes(int64_t n_q, int32_t top) {
  (void)n_q;
  (void)top;
  return 0;
}

int als_topk(const float* Q, int64_t n_q, const float* V, int64_t n_v, int32_t ld, int32_t k,
             int32_t top, int32_t* idx_out, float* score_out, void* ws, size_t ws_bytes,
             void* stream) {
  (void)ws;
  (void)ws_bytes;
  ALS_REQUIRE(k >= 1 && k <= 128, ALS_EUNSUPPORTED, "als_topk: rank %d not in [1, 128]", k);
  ALS_REQUIRE(ld >= k && ld % 4 == 0, ALS_EINVAL, "als_topk: bad ld");
  ALS_REQUIRE(top >= 1 && top <= kTopkMax, ALS_EUNSUPPORTED, "als_topk: top %d not in [1, %d]",
              top, kTopkMax);
  ALS_REQUIRE(n_q >= 0 && n_v >= 0 && n_v < (int64_t(1) << 31), ALS_EINVAL,
              "als_topk: bad sizes");
  if (n_q == 0) return ALS_OK;
  ALS_REQUIRE(Q && V && idx_out && score_out, ALS_EINVAL, "als_topk: null pointer");
  hipStream_t st = as_stream(stream);
  const int cn = k <= 16 ? 1 : (k <= 32 ? 2 : (k <= 64 ? 4 : 8));
  const size_t lds = topk_lds_bytes(cn, top);
  ALS_REQUIRE(lds <= kLdsBytes, ALS_EUNSUPPORTED,
              "als_topk: top %d at rank %d needs %zu B of LDS (> %d)", top, k, lds, kLdsBytes);
  const unsigned grid = (unsigned)((n_q + 63) / 64);
#define ALS_TOPK_LAUNCH(CN)                                                                   \
  do {                                                                                        \
    ALS_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&topk_kernel<CN>),              \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));       \
    topk_kernel<CN><<<grid, 256, lds, st>>>(Q, n_q, V, n_v, ld, k, top, idx_out, score_out);  \
    ALS_LAUNCH_CHECK();                                                                       \
  } while (0)
  if (cn == 1) ALS_TOPK_LAUNCH(1);
  else if (cn == 2) ALS_TOPK_LAUNCH(2);
  else if (cn == 4) ALS_TOPK_LAUNCH(4);
  else ALS_TOPK_LAUNCH(8);
#undef ALS_TOPK_LAUNCH
  return ALS_OK;
}

}  // extern "C"
