// Dev-only ablation kernels (NOT part of libals_hip.so): the light-row path of
// gram_solve_kernel<4,false> split into its phases, to time each on the GPU.
//   mode 0: full (gram + tile LDL^T on MFMA)
//   mode 1: gram only (accumulate, then write a checksum so nothing is dead)
//   mode 2: solve only (synthetic SPD matrix in registers, tile LDL^T)
//   mode 3: solve only, unblocked ldl_solve
//   mode 4: full, unblocked ldl_solve
// Built by tools/ablate.py into tools/libals_dev.so.
#include "../recommender-system-using-apache-spark-mllib-_amd/csrc/gram_solve.hip"

namespace als {
void set_error(const char*, ...) {}
}

namespace als {

template <int MODE>
__global__ __launch_bounds__(64, 2) void ablate_kernel(const int64_t* __restrict__ row_ptr,
                                                       const int32_t* __restrict__ col,
                                                       const float* __restrict__ val,
                                                       const int32_t* __restrict__ rows, int n,
                                                       const float* __restrict__ Y,
                                                       float* __restrict__ X, int ld, float reg,
                                                       int32_t* __restrict__ status) {
  constexpr int CN = 4, NT = Cfg<CN>::NT, KP = 64;
  __shared__ __attribute__((aligned(16))) unsigned char smem[SmemBytes<CN, false>::value];
  float* P = reinterpret_cast<float*>(smem);
  float* cb = P + Cfg<CN>::NP;
  const int row = rows[blockIdx.x];
  const int lane = threadIdx.x;
  double a64[NT][4];
  double b64[CN];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) a64[t][r] = 0.0;
#pragma unroll
  for (int c = 0; c < CN; ++c) b64[c] = 0.0;
  int npos = 0;
  const int64_t pb = row_ptr[row], pe = row_ptr[row + 1];
  if constexpr (MODE == 5) {  // half the workgroups gram-only, half solve-only (overlap test)
    if (blockIdx.x & 1) {
      gram_accumulate<CN, false, false>(col, val, pb, pe, Y, ld, 64, 0.f, a64, b64, npos);
      double s = 0.0;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) s += a64[t][r];
      X[(int64_t)row * ld + lane] = (float)s;
      return;
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) a64[t][r] = 0.01 * (double)((lane * 7 + t * 3 + r) % 11);
    b64[0] = 1.0;
  } else if constexpr (MODE == 0 || MODE == 1 || MODE == 4) {
    gram_accumulate<CN, false, false>(col, val, pb, pe, Y, ld, 64, 0.f, a64, b64, npos);
  } else {
    // synthetic well-conditioned SPD system: diagonal n, small off-diagonals
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) a64[t][r] = 0.01 * (double)((lane * 7 + t * 3 + r) % 11);
    b64[0] = 1.0;
  }
  if constexpr (MODE == 1) {
    double s = 0.0;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) s += a64[t][r];
    for (int c = 0; c < CN; ++c) s += b64[c];
    X[(int64_t)row * ld + lane] = (float)s;
    return;
  }
  if constexpr (MODE == 3 || MODE == 4) {
    // unblocked variant
    const int q = lane >> 4, m = lane & 15;
#pragma unroll
    for (int c = 0; c < CN; ++c) {
      b64[c] += shfl_xor_f64(b64[c], 16);
      b64[c] += shfl_xor_f64(b64[c], 32);
    }
    regularise<CN, false>(a64, (double)reg * (double)(pe - pb + 64), 64, nullptr);
    pack_gram<CN, float>(a64, P);
    if (q == 0)
      for (int c = 0; c < CN; ++c) cb[m * CN + c] = (float)b64[c];
    __syncthreads();
    const float b = cb[lane];
    __syncthreads();
    if (!ldl_solve<KP, float>(P, cb, b, 64, X + (int64_t)row * ld, ld) && lane == 0)
      atomicCAS(status, 0, row + 1);
    return;
  }
  finish_and_solve<CN, false>(a64, b64, (pe - pb) + 64, smem, 64, reg, nullptr,
                              X + (int64_t)row * ld, ld, row, status);
}

}  // namespace als

extern "C" int dev_ablate(int mode, const int64_t* row_ptr, const int32_t* col, const float* val,
                          const int32_t* rows, int n, const float* Y, float* X, int ld, float reg,
                          int32_t* status, void* stream) {
  using namespace als;
  hipStream_t st = (hipStream_t)stream;
#define L(M) ablate_kernel<M><<<n, 64, 0, st>>>(row_ptr, col, val, rows, n, Y, X, ld, reg, status)
  switch (mode) {
    case 0: L(0); break;
    case 1: L(1); break;
    case 2: L(2); break;
    case 3: L(3); break;
    case 4: L(4); break;
    case 5: L(5); break;
    default: return -1;
  }
#undef L
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
