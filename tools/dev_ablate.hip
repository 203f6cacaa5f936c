// Dev-only ablation kernels (NOT part of libals_hip.so): the explicit light-row path
// of gram_solve_kernel<4,false> (rank 64) and gram_solve_w1_kernel<false> (rank 128)
// split into their phases, to time / profile each on the GPU.
//   mode 0: full (pre-split Gram + block elimination), as the product
//   mode 1: Gram only (accumulate, then write a checksum so nothing is dead)
//   mode 2: solve only (a diagonally dominant system in registers)
// Built by tools/ablate.py into tools/libals_dev.so.
#include "../recommender-system-using-apache-spark-mllib-_amd/csrc/gram_solve.hip"

namespace als {
void set_error(const char*, ...) {}
}

namespace als {

// synthetic SPD tiles in the C layout: dominant diagonal, small off-diagonals
template <int NT>
__device__ __forceinline__ void synth_spd(floatx4 (&acc)[NT], int nb) {
  const int lane = threadIdx.x & 63, q = lane >> 4, m = lane & 15;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[t][r] = 0.01f * (float)((lane * 7 + t * 3 + r) % 11);
  int t = 0;
  for (int c1 = 0; c1 < nb; ++c1)
    for (int c2 = c1; c2 < nb; ++c2, ++t)
      if (c1 == c2)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (4 * q + r == m) acc[t][r] = 50.f;
}

template <int NB, int MODE>
__global__ __launch_bounds__(64, NB == 4 ? 3 : 1) void ablate_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ val, const int32_t* __restrict__ rows,
    const uint32_t* __restrict__ Ysp, int kp, int zero_row, float sr, float inv2, float invb,
    float* __restrict__ X, int ld, int k, float reg, RescueList rl) {
  constexpr int NT = NB * (NB + 1) / 2;
  __shared__ __attribute__((aligned(16))) unsigned char smem[SmemBytes<NB>::value];
  const int lane = threadIdx.x & 63;
  const int row = rows[blockIdx.x];
  const int64_t pb = row_ptr[row], pe = row_ptr[row + 1];
  floatx4 acc[NT];
  float bt[NB];
#pragma unroll
  for (int c = 0; c < NB; ++c) bt[c] = 0.f;
  float scale = inv2;
  if (MODE != 2) {
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    floatx4 accb[NB];
#pragma unroll
    for (int c = 0; c < NB; ++c) accb[c] = floatx4{0.f, 0.f, 0.f, 0.f};
    float rmax = 0.f;
    if constexpr (NB == 8)
      gram_accumulate_pre2<FullTiles<NB>>(col, val, pb, pe, Ysp, (uint32_t)kp, zero_row, sr,
                                          (lane & 15) * NB, acc, accb,
                                          reinterpret_cast<int*>(smem), rmax);
    else
      gram_accumulate_pre<FullTiles<NB>>(col, val, pb, pe, Ysp, (uint32_t)kp, zero_row, sr,
                                         (lane & 15) * NB, acc, accb,
                                         reinterpret_cast<int*>(smem), rmax);
    rhs_from_tiles<FullTiles<NB>>(accb, invb, bt);
  } else {
    synth_spd<NT>(acc, NB);
    bt[0] = 1.f;
    scale = 1.f;
  }
  if (MODE == 1) {
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) s += acc[t][r];
    for (int c = 0; c < NB; ++c) s += bt[c];
    X[(int64_t)row * ld + lane] = s;
    return;
  }
  __syncthreads();
  w1_finish_and_solve<false, NB, false>(
      acc, scale, bt, pe - pb, nullptr, smem, k, reg, X + (int64_t)row * ld, ld, row, rl);
}

}  // namespace als

extern "C" int dev_ablate(int nb, int mode, const int64_t* row_ptr, const int32_t* col,
                          const float* val, const int32_t* rows, int n, const uint32_t* Ysp,
                          int kp, int zero_row, float sr, float inv2, float invb, float* X, int ld,
                          int k, float reg, unsigned* rcnt, int32_t* rlist, void* stream) {
  using namespace als;
  hipStream_t st = (hipStream_t)stream;
  const RescueList rl{rcnt, rlist, (unsigned)n};
#define L(NB, M)                                                                              \
  ablate_kernel<NB, M><<<n, 64, 0, st>>>(row_ptr, col, val, rows, Ysp, kp, zero_row, sr, inv2, \
                                         invb, X, ld, k, reg, rl)
  if (nb == 4) {
    if (mode == 0) L(4, 0);
    else if (mode == 1) L(4, 1);
    else if (mode == 2) L(4, 2);
    else return -1;
  } else if (nb == 8) {
    if (mode == 0) L(8, 0);
    else if (mode == 1) L(8, 1);
    else if (mode == 2) L(8, 2);
    else return -1;
  } else {
    return -1;
  }
#undef L
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
