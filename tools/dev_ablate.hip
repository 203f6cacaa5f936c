// Dev-only ablation kernels (NOT part of libals_hip.so): the light-row path of
// gram_solve_kernel<4,false> (explicit, pre-split Gram) split into its phases,
// to time each on the GPU.
//   mode 0: full (gram + panel LDL^T)
//   mode 1: gram only (accumulate, then write a checksum so nothing is dead)
//   mode 2: solve only (synthetic SPD matrix in registers, tile LDL^T)
//   mode 5: half the workgroups gram-only, half solve-only (overlap test)
// Built by tools/ablate.py into tools/libals_dev.so.
#include "../recommender-system-using-apache-spark-mllib-_amd/csrc/gram_solve.hip"

namespace als {
void set_error(const char*, ...) {}
}

namespace als {

template <int MODE>
__global__ __launch_bounds__(64, 3) void ablate_kernel(const int64_t* __restrict__ row_ptr,
                                                       const int32_t* __restrict__ col,
                                                       const float* __restrict__ val,
                                                       const int32_t* __restrict__ rows, int n,
                                                       const uint32_t* __restrict__ Ysp,
                                                       int zero_row, float sr, float inv2,
                                                       float invb, float* __restrict__ X, int ld,
                                                       float reg, int32_t* __restrict__ status) {
  constexpr int CN = 4, NT = Cfg<CN>::NT;
  __shared__ __attribute__((aligned(16))) unsigned char smem[SmemBytes<CN>::value];
  const int row = rows[blockIdx.x];
  const int lane = threadIdx.x;
  float tot[NT][4], bt[CN];
  zero_acc<NT, CN, float>(tot, bt);
  const int64_t pb = row_ptr[row], pe = row_ptr[row + 1];
  bool gram = MODE == 0 || MODE == 1 || (MODE == 5 && (blockIdx.x & 1));
  if (gram) {
    floatx4 acc[NT], accb[CN];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < CN; ++c) accb[c] = floatx4{0.f, 0.f, 0.f, 0.f};
    gram_accumulate_pre<FullTiles<CN>>(col, val, pb, pe, Ysp, 64u, zero_row, sr, (lane & 15) * CN,
                                       acc, accb, reinterpret_cast<int*>(smem));
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) tot[t][r] = acc[t][r] * inv2;
    rhs_from_tiles<FullTiles<CN>>(accb, invb, bt);
    __syncthreads();
  } else {
    // synthetic SPD system: small off-diagonals, diagonal from regularisation
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) tot[t][r] = 0.01f * (float)((lane * 7 + t * 3 + r) % 11);
    bt[0] = 1.f;
  }
  if (MODE == 1 || (MODE == 5 && (blockIdx.x & 1))) {
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) s += tot[t][r];
    for (int c = 0; c < CN; ++c) s += bt[c];
    X[(int64_t)row * ld + lane] = s;
    return;
  }
  finish_and_solve<CN, false, float>(tot, bt, (pe - pb) + 64, smem, 64, reg, nullptr,
                                     X + (int64_t)row * ld, ld, row, status);
}

// k = 128 workgroup path (explicit), same modes 0/1/2.
template <int R, int MODE>
__device__ __forceinline__ void ablate_wg_task(const int64_t* __restrict__ row_ptr,
                                               const int32_t* __restrict__ col,
                                               const float* __restrict__ val,
                                               const int32_t* __restrict__ rows,
                                               const uint32_t* __restrict__ Ysp, int zero_row,
                                               float sr, float inv2, float invb,
                                               float* __restrict__ X, int ld, float reg,
                                               int32_t* __restrict__ status, float* lds) {
  typedef WgTiles<R> TS;
  const int lane = threadIdx.x & 63;
  float tot[TS::N][4], bt[TS::NRA];
  zero_acc<TS::N, TS::NRA, float>(tot, bt);
  const int row = rows[blockIdx.x];
  const int64_t pb = row_ptr[row], pe = row_ptr[row + 1];
  if (MODE != 2) {
    floatx4 acc[TS::N], accb[TS::NRA];
#pragma unroll
    for (int t = 0; t < TS::N; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < TS::NRA; ++c) accb[c] = floatx4{0.f, 0.f, 0.f, 0.f};
    gram_accumulate_pre<TS>(col, val, pb, pe, Ysp, 128u, zero_row, sr, (lane & 15) * kWgNB, acc,
                            accb, reinterpret_cast<int*>(lds) + 128 * R);
#pragma unroll
    for (int t = 0; t < TS::N; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) tot[t][r] = acc[t][r] * inv2;
    rhs_from_tiles<TS>(accb, invb, bt);
    __syncthreads();
  } else {
#pragma unroll
    for (int t = 0; t < TS::N; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) tot[t][r] = 0.01f * (float)((lane * 7 + t * 3 + r) % 11);
    bt[0] = 1.f;
  }
  if (MODE == 1) {
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < TS::N; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) s += tot[t][r];
    for (int c = 0; c < TS::NRA; ++c) s += bt[c];
    X[(int64_t)row * ld + (threadIdx.x & 127)] = s;
    return;
  }
  wg_finish_and_solve<R, false, float>(tot, bt, (pe - pb) + 64, lds, 128, reg, nullptr,
                                       X + (int64_t)row * ld, ld, row, status);
}

template <int MODE>
__global__ __launch_bounds__(256, 2) void ablate_wg_kernel(const int64_t* __restrict__ row_ptr,
                                                           const int32_t* __restrict__ col,
                                                           const float* __restrict__ val,
                                                           const int32_t* __restrict__ rows,
                                                           const uint32_t* __restrict__ Ysp,
                                                           int zero_row, float sr, float inv2,
                                                           float invb, float* __restrict__ X,
                                                           int ld, float reg,
                                                           int32_t* __restrict__ status) {
  __shared__ __attribute__((aligned(16))) float lds[WgLds::SIZE];
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#define T(R) \
  ablate_wg_task<R, MODE>(row_ptr, col, val, rows, Ysp, zero_row, sr, inv2, invb, X, ld, reg, status, lds)
  if (wv == 0) T(0);
  else if (wv == 1) T(1);
  else if (wv == 2) T(2);
  else T(3);
#undef T
}

// k = 128 W1 path (one wave per system), explicit: modes 0 full / 1 gram only / 2 solve only.
template <int MODE>
__global__ __launch_bounds__(64, 1) void ablate_w1_kernel(const int64_t* __restrict__ row_ptr,
                                                          const int32_t* __restrict__ col,
                                                          const float* __restrict__ val,
                                                          const int32_t* __restrict__ rows,
                                                          const uint32_t* __restrict__ Ysp,
                                                          int zero_row, float sr, float inv2,
                                                          float invb, float* __restrict__ X,
                                                          int ld, float reg,
                                                          int32_t* __restrict__ status) {
  constexpr int CN = 8, NT = kW1NT;
  __shared__ __attribute__((aligned(16))) unsigned char smem[SmemBytes<CN>::value];
  const int lane = threadIdx.x & 63;
  const int row = rows[blockIdx.x];
  const int64_t pb = row_ptr[row], pe = row_ptr[row + 1];
  floatx4 acc[NT];
  float bt[CN];
#pragma unroll
  for (int c = 0; c < CN; ++c) bt[c] = 0.f;
  if (MODE != 2) {
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    floatx4 accb[CN];
#pragma unroll
    for (int c = 0; c < CN; ++c) accb[c] = floatx4{0.f, 0.f, 0.f, 0.f};
    gram_accumulate_pre<FullTiles<CN>>(col, val, pb, pe, Ysp, 128u, zero_row, sr, (lane & 15) * CN,
                                       acc, accb, reinterpret_cast<int*>(smem));
    rhs_from_tiles<FullTiles<CN>>(accb, invb, bt);
  } else {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[t][r] = 0.01f * (float)((lane * 7 + t * 3 + r) % 11);
    bt[0] = 1.f;
  }
  if (MODE == 1) {
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) s += acc[t][r];
    for (int c = 0; c < CN; ++c) s += bt[c];
    X[(int64_t)row * ld + lane] = s;
    return;
  }
  wave_lds_sync();
  w1_finish_and_solve<false>(acc, MODE == 2 ? 1.f : inv2, bt, (pe - pb) + 64, nullptr, smem, 128,
                             reg, X + (int64_t)row * ld, ld, row, status);
}

}  // namespace als

extern "C" int dev_ablate_w1(int mode, const int64_t* row_ptr, const int32_t* col,
                             const float* val, const int32_t* rows, int n, const uint32_t* Ysp,
                             int zero_row, float sr, float inv2, float invb, float* X, int ld,
                             float reg, int32_t* status, void* stream) {
  using namespace als;
  hipStream_t st = (hipStream_t)stream;
#define L(M)                                                                                \
  ablate_w1_kernel<M><<<n, 64, 0, st>>>(row_ptr, col, val, rows, Ysp, zero_row, sr, inv2, invb, \
                                        X, ld, reg, status)
  switch (mode) {
    case 0: L(0); break;
    case 1: L(1); break;
    case 2: L(2); break;
    default: return -1;
  }
#undef L
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int dev_ablate(int mode, const int64_t* row_ptr, const int32_t* col, const float* val,
                          const int32_t* rows, int n, const uint32_t* Ysp, int zero_row, float sr,
                          float inv2, float invb, float* X, int ld, float reg, int32_t* status,
                          void* stream) {
  using namespace als;
  hipStream_t st = (hipStream_t)stream;
#define L(M)                                                                                 \
  ablate_kernel<M><<<n, 64, 0, st>>>(row_ptr, col, val, rows, n, Ysp, zero_row, sr, inv2, invb, \
                                     X, ld, reg, status)
  switch (mode) {
    case 0: L(0); break;
    case 1: L(1); break;
    case 2: L(2); break;
    case 5: L(5); break;
    default: return -1;
  }
#undef L
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int dev_ablate_wg(int mode, const int64_t* row_ptr, const int32_t* col,
                             const float* val, const int32_t* rows, int n, const uint32_t* Ysp,
                             int zero_row, float sr, float inv2, float invb, float* X, int ld,
                             float reg, int32_t* status, void* stream) {
  using namespace als;
  hipStream_t st = (hipStream_t)stream;
#define L(M)                                                                                   \
  ablate_wg_kernel<M><<<n, 256, 0, st>>>(row_ptr, col, val, rows, Ysp, zero_row, sr, inv2, invb, \
                                         X, ld, reg, status)
  switch (mode) {
    case 0: L(0); break;
    case 1: L(1); break;
    case 2: L(2); break;
    default: return -1;
  }
#undef L
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
