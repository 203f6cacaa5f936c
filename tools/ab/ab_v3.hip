#include "tk_v3.hip"
namespace als { void set_error(const char*, ...) {} }
extern "C" int ab_topk(const float* Q, int64_t n_q, const float* V, int64_t n_v, int ld, int k,
                       int top, int32_t* idx, float* sc, void* ws, size_t ws_bytes, void* st) {
  return als_topk(Q, n_q, V, n_v, ld, k, top, idx, sc, ws, ws_bytes, st);
}
extern "C" size_t ab_ws(int64_t n_q, int64_t n_v, int k, int top) {
  return als_topk_workspace_bytes(n_q, n_v, k, top);
}
