// Dev-only (NOT part of libals_hip.so): topk_split_kernel ablation modes, timed by
// tools/topk_ablate.py.  mode 0 = the product als_topk; modes 1 / 3 reuse the
// split table that a preceding mode-0 call left in the workspace:
//   1: scores only (no filter)   3: product filter, counts exact-insertion calls
#include "../recommender-system-using-apache-spark-mllib-_amd/csrc/topk.hip"

namespace als {
void set_error(const char*, ...) {}
}

extern "C" int dev_topk(int mode, const float* Q, int64_t n_q, const float* V, int64_t n_v, int ld,
                        int k, int top, int32_t* idx, float* sc, void* ws, size_t ws_bytes,
                        float* dbg, void* stream) {
  using namespace als;
  if (mode == 0) return als_topk(Q, n_q, V, n_v, ld, k, top, idx, sc, ws, ws_bytes, stream);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int kq = topk_kq(k);
  const bool quad = topk_quad(top, n_v);
  const int rg = topk_split_rg(k, top, quad, n_q);
  if (rg == 0) return -1;
  const size_t lds = topk_split_lds_bytes(kq, rg, top, quad);
  const int nw = (top <= kTopR || quad) ? tk_nw(1) : tk_nw(0);
  const unsigned grid = (unsigned)((n_q + 16 * nw * rg - 1) / (16 * nw * rg));
  const float* scal = reinterpret_cast<const float*>(ws);
  const uint4* vsp4 = reinterpret_cast<const uint4*>(static_cast<char*>(ws) + 256);
  const int32_t* perm =
      reinterpret_cast<const int32_t*>(static_cast<char*>(ws) + 256 + tk_table_bytes(n_v, k));
  const float* vnorm = reinterpret_cast<const float*>(
      perm + align_up(4 * (size_t)n_v) / 4 + align_up(4 * (size_t)kTkBuckets) / 4);
#define L(NK, RG, M)                                                                          \
  do {                                                                                        \
    if (top <= kTopR) { /* the product picks 8 / 12 / 16 by top: the dev modes use 16 */    \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&topk_split_kernel<NK, RG, kTopR, M>), \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);        \
      topk_split_kernel<NK, RG, kTopR, M><<<grid, 64 * nw, lds, st>>>(Q, n_q, vsp4, vsp4 + n_v * (kq / 8), perm, vnorm, n_v, ld,  \
                                                                  k, top, scal, idx, dbg);    \
    } else if (quad) { /* quad lists (rg is 1 here): the dev modes use 100 (configs[4]) */   \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&topk_split_kernel<NK, 1, 100, M>), \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);        \
      topk_split_kernel<NK, 1, 100, M><<<grid, 64 * nw, lds, st>>>(Q, n_q, vsp4, vsp4 + n_v * (kq / 8), perm, vnorm, n_v, ld,   \
                                                               k, top, scal, idx, dbg);       \
    } else {                                                                                  \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&topk_split_kernel<NK, RG, 0, M>), \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);        \
      topk_split_kernel<NK, RG, 0, M><<<grid, 64 * nw, lds, st>>>(Q, n_q, vsp4, vsp4 + n_v * (kq / 8), perm, vnorm, n_v, ld, k, \
                                                              top, scal, idx, dbg);           \
    }                                                                                         \
  } while (0)
#define LM(NK, RG) \
  do {             \
    if (mode == 1) \
      L(NK, RG, 1); \
    else if (mode == 2) \
      L(NK, RG, 2); \
    else if (mode == 4) \
      L(NK, RG, 4); \
    else if (mode == 5) \
      L(NK, RG, 5); \
    else           \
      L(NK, RG, 3); \
  } while (0)
  if (kq == 64) {
    if (rg == 2) LM(2, 2); else LM(2, 1);
  } else if (kq == 128) {
    if (rg == 2) LM(4, 2); else LM(4, 1);
  } else {
    if (rg == 2) LM(1, 2); else LM(1, 1);
  }
#undef LM
#undef L
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
