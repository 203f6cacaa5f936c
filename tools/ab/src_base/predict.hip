// K4 — gather-dot predict and fused RMSE.
//
// Replaces MatrixFactorizationModel.predict(RDD[(Int, Int)]) (upstream mllib:
// two joins + blas.ddot over Float factors widened to Double), reached from
// `predictAll` at RecommenderSystem.py:150, :165, :222, :232, and the
// computeError join + reduce + count of RecommenderSystem.py:103-129.
//
// 16 lanes per (user, item) pair: each lane reads one float4 of the user row
// and one of the item row (a whole 256-B row per 16 lanes, rank 64), multiplies
// in fp64 and the group reduces with xor-shuffles.  Unknown ids (outside the
// map or mapped to -1) give NaN (predict) or are skipped (RMSE), which is the
// inner-join semantics of predictAll + computeError.  The RMSE partials are
// per-block fp64 sums reduced in a fixed order, so the result is bitwise
// reproducible run to run.
#include "als_common.h"

namespace als {

constexpr int kPairsPerBlock = 256;  // 16 pairs per pass x 16 passes

__device__ __forceinline__ double pair_dot(int32_t uid, int32_t iid,
                                          const int32_t* __restrict__ umap, int32_t usz,
                                          const int32_t* __restrict__ imap, int32_t isz,
                                          const float* __restrict__ U, const float* __restrict__ V,
                                          int ld, int k, bool& known) {
  const int g = threadIdx.x & 15;
  int32_t ur = -1, ir = -1;
  if (uid >= 0 && uid < usz) ur = umap[uid];
  if (iid >= 0 && iid < isz) ir = imap[iid];
  known = ur >= 0 && ir >= 0;
  double s = 0.0;
  if (known) {
    for (int d0 = 4 * g; d0 < k; d0 += 64) {
      const float4 a = *reinterpret_cast<const float4*>(U + (int64_t)ur * ld + d0);
      const float4 b = *reinterpret_cast<const float4*>(V + (int64_t)ir * ld + d0);
      s += (double)a.x * (double)b.x;
      if (d0 + 1 < k) s += (double)a.y * (double)b.y;
      if (d0 + 2 < k) s += (double)a.z * (double)b.z;
      if (d0 + 3 < k) s += (double)a.w * (double)b.w;
    }
  }
#pragma unroll
  for (int msk = 8; msk >= 1; msk >>= 1) s += shfl_xor_f64(s, msk);
  return s;
}

__global__ __launch_bounds__(256) void predict_kernel(const int32_t* __restrict__ u,
                                                      const int32_t* __restrict__ it, int64_t n,
                                                      const int32_t* __restrict__ umap, int32_t usz,
                                                      const int32_t* __restrict__ imap, int32_t isz,
                                                      const float* __restrict__ U,
                                                      const float* __restrict__ V, int ld, int k,
                                                      double* __restrict__ out) {
  const int grp = threadIdx.x >> 4;
  for (int pass = 0; pass < kPairsPerBlock / 16; ++pass) {
    const int64_t e = (int64_t)blockIdx.x * kPairsPerBlock + pass * 16 + grp;
    const bool in = e < n;  // uniform across the 16-lane group
    bool known = false;
    const double s = pair_dot(in ? u[e] : -1, in ? it[e] : -1, umap, usz, imap, isz, U, V, ld, k,
                              known);
    if (in && (threadIdx.x & 15) == 0) out[e] = known ? s : __builtin_nan("");
  }
}

__global__ __launch_bounds__(256) void rmse_partial_kernel(
    const int32_t* __restrict__ u, const int32_t* __restrict__ it, const float* __restrict__ r,
    int64_t n, const int32_t* __restrict__ umap, int32_t usz, const int32_t* __restrict__ imap,
    int32_t isz, const float* __restrict__ U, const float* __restrict__ V, int ld, int k,
    double* __restrict__ partial) {
  __shared__ double ssum[16], scnt[16];
  const int grp = threadIdx.x >> 4;
  double sse = 0.0, cnt = 0.0;  // lane 0 of each group accumulates its 16 pairs in order
  for (int pass = 0; pass < kPairsPerBlock / 16; ++pass) {
    const int64_t e = (int64_t)blockIdx.x * kPairsPerBlock + pass * 16 + grp;
    const bool in = e < n;
    bool known = false;
    const double p = pair_dot(in ? u[e] : -1, in ? it[e] : -1, umap, usz, imap, isz, U, V, ld, k,
                              known);
    if (in && known) {
      const double d = (double)r[e] - p;
      sse += d * d;
      cnt += 1.0;
    }
  }
  if ((threadIdx.x & 15) == 0) {
    ssum[grp] = sse;
    scnt[grp] = cnt;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, c = 0.0;
    for (int i = 0; i < 16; ++i) {
      a += ssum[i];
      c += scnt[i];
    }
    partial[2 * blockIdx.x] = a;
    partial[2 * blockIdx.x + 1] = c;
  }
}

// Single-block fixed-order reduction of the per-block partials.
__global__ __launch_bounds__(256) void rmse_final_kernel(const double* __restrict__ partial,
                                                         int64_t nb, double* __restrict__ out) {
  __shared__ double ssum[256], scnt[256];
  double a = 0.0, c = 0.0;
  for (int64_t b = threadIdx.x; b < nb; b += 256) {
    a += partial[2 * b];
    c += partial[2 * b + 1];
  }
  ssum[threadIdx.x] = a;
  scnt[threadIdx.x] = c;
  __syncthreads();
  for (int s = 128; s >= 1; s >>= 1) {
    if ((int)threadIdx.x < s) {
      ssum[threadIdx.x] += ssum[threadIdx.x + s];
      scnt[threadIdx.x] += scnt[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[0] = ssum[0];
    out[1] = scnt[0];
  }
}

}  // namespace als

using namespace als;

extern "C" {

int als_predict(const int32_t* u, const int32_t* i, int64_t n, const int32_t* umap,
                int32_t umap_size, const int32_t* imap, int32_t imap_size, const float* U,
                const float* V, int32_t ld, int32_t k, double* pred_out, void* stream) {
  ALS_REQUIRE(k >= 1 && ld >= k && ld % 4 == 0, ALS_EINVAL, "als_predict: bad k/ld");
  ALS_REQUIRE(n >= 0, ALS_EINVAL, "als_predict: n < 0");
  if (n == 0) return ALS_OK;
  ALS_REQUIRE(u && i && umap && imap && U && V && pred_out, ALS_EINVAL,
              "als_predict: null pointer");
  const int64_t nb = (n + kPairsPerBlock - 1) / kPairsPerBlock;
  predict_kernel<<<(unsigned)nb, 256, 0, as_stream(stream)>>>(u, i, n, umap, umap_size, imap,
                                                              imap_size, U, V, ld, k, pred_out);
  ALS_LAUNCH_CHECK();
  return ALS_OK;
}

size_t als_rmse_workspace_bytes(int64_t n) {
  const int64_t nb = n > 0 ? (n + kPairsPerBlock - 1) / kPairsPerBlock : 1;
  return align_up(sizeof(double) * 2 * (size_t)nb) + 256;
}

int als_rmse_partial(const int32_t* u, const int32_t* i, const float* r, int64_t n,
                     const int32_t* umap, int32_t umap_size, const int32_t* imap,
                     int32_t imap_size, const float* U, const float* V, int32_t ld, int32_t k,
                     double* sse_count_out, void* ws, size_t ws_bytes, void* stream) {
  ALS_REQUIRE(k >= 1 && ld >= k && ld % 4 == 0, ALS_EINVAL, "als_rmse_partial: bad k/ld");
  ALS_REQUIRE(n >= 0 && sse_count_out, ALS_EINVAL, "als_rmse_partial: bad args");
  ALS_REQUIRE(ws_bytes >= als_rmse_workspace_bytes(n), ALS_EWORKSPACE,
              "als_rmse_partial: workspace too small");
  hipStream_t st = as_stream(stream);
  if (n == 0) {
    ALS_HIP(hipMemsetAsync(sse_count_out, 0, 2 * sizeof(double), st));
    return ALS_OK;
  }
  ALS_REQUIRE(u && i && r && umap && imap && U && V, ALS_EINVAL, "als_rmse_partial: null pointer");
  const int64_t nb = (n + kPairsPerBlock - 1) / kPairsPerBlock;
  double* partial = static_cast<double*>(ws);
  rmse_partial_kernel<<<(unsigned)nb, 256, 0, st>>>(u, i, r, n, umap, umap_size, imap, imap_size,
                                                    U, V, ld, k, partial);
  ALS_LAUNCH_CHECK();
  rmse_final_kernel<<<1, 256, 0, st>>>(partial, nb, sse_count_out);
  ALS_LAUNCH_CHECK();
  return ALS_OK;
}

}  // extern "C"
