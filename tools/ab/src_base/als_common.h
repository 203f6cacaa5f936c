// Shared device/host helpers for libals_hip.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>
#include <string.h>
#include "../../include/als_hip.h"

namespace als {

// ---- error reporting (thread-local message, returned by als_last_error) ----
void set_error(const char* fmt, ...);

#define ALS_REQUIRE(cond, code, ...)          \
  do {                                        \
    if (!(cond)) {                            \
      ::als::set_error(__VA_ARGS__);          \
      return (code);                          \
    }                                         \
  } while (0)

#define ALS_HIP(expr)                                                        \
  do {                                                                       \
    hipError_t e_ = (expr);                                                  \
    if (e_ != hipSuccess) {                                                  \
      ::als::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                       __FILE__, __LINE__);                                  \
      return ALS_EDEVICE;                                                    \
    }                                                                        \
  } while (0)

#define ALS_LAUNCH_CHECK()                                                   \
  do {                                                                       \
    hipError_t e_ = hipGetLastError();                                       \
    if (e_ != hipSuccess) {                                                  \
      ::als::set_error("kernel launch failed: %s (%s:%d)",                   \
                       hipGetErrorString(e_), __FILE__, __LINE__);           \
      return ALS_EDEVICE;                                                    \
    }                                                                        \
  } while (0)

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

static inline size_t align_up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }

// Bump allocator over a caller workspace.
struct Arena {
  char* base;
  size_t cap;
  size_t off = 0;
  Arena(void* b, size_t c) : base(static_cast<char*>(b)), cap(c) {}
  template <class T>
  T* take(size_t count) {
    size_t bytes = align_up(count * sizeof(T));
    if (off + bytes > cap) return nullptr;
    T* p = reinterpret_cast<T*>(base + off);
    off += bytes;
    return p;
  }
};
// Same layout arithmetic without memory (for *_workspace_bytes).
struct ArenaSize {
  size_t off = 0;
  template <class T>
  void take(size_t count) { off += align_up(count * sizeof(T)); }
};

// ---- device scan / sort primitives (csr_build.hip) ----
// Exclusive prefix sum of n int32 values into int64 out (out may alias nothing).
size_t scan_workspace_bytes(int64_t n);
int scan_exclusive_i32_to_i64(const int32_t* in, int64_t* out, int64_t n, void* ws,
                              size_t ws_bytes, hipStream_t st);
int scan_exclusive_i32(const int32_t* in, int32_t* out, int64_t n, void* ws, size_t ws_bytes,
                       hipStream_t st);
// Stable LSD radix sort of (key, value) pairs by the low `bits` bits of key.
size_t radix_workspace_bytes(int64_t n);
int radix_sort_pairs(const uint32_t* keys_in, const int32_t* vals_in, uint32_t* keys_out,
                     int32_t* vals_out, int64_t n, int bits, void* ws, size_t ws_bytes,
                     hipStream_t st);

// ---- device helpers ----
__device__ __forceinline__ double readlane_f64(double v, int lane) {
  int2 iv = __builtin_bit_cast(int2, v);
  iv.x = __builtin_amdgcn_readlane(iv.x, lane);
  iv.y = __builtin_amdgcn_readlane(iv.y, lane);
  return __builtin_bit_cast(double, iv);
}

__device__ __forceinline__ double shfl_xor_f64(double v, int mask) {
  int2 iv = __builtin_bit_cast(int2, v);
  iv.x = __shfl_xor(iv.x, mask);
  iv.y = __shfl_xor(iv.y, mask);
  return __builtin_bit_cast(double, iv);
}

}  // namespace als
