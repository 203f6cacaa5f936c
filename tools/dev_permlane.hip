// Dev-only: semantics of v_permlane16/32_swap on gfx950 (raw outputs per lane).
#include <hip/hip_runtime.h>
extern "C" __global__ void pl_kernel(unsigned* out) {
  const unsigned x = threadIdx.x;
  const auto a = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  const unsigned y = x + 100;
  const auto c = __builtin_amdgcn_permlane16_swap(x, y, false, false);
  out[threadIdx.x] = a[0];
  out[64 + threadIdx.x] = a[1];
  out[128 + threadIdx.x] = b[0];
  out[192 + threadIdx.x] = b[1];
  out[256 + threadIdx.x] = c[0];
  out[320 + threadIdx.x] = c[1];
}
extern "C" int pl_run(unsigned* out_dev, void* stream) {
  pl_kernel<<<1, 64, 0, (hipStream_t)stream>>>(out_dev);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
