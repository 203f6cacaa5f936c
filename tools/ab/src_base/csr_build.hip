// K1 — rating-block construction in HBM.
//
// Replaces Spark's partitionRatings / makeBlocks / UncompressedInBlock.compress
// (ml/recommendation/ALS.scala, upstream; reached from ALS.train at
// RecommenderSystem.py:148-149, :163, :218).  Spark hash-partitions ratings
// into blocks through three shuffles and TimSorts each block by src id; here
// the whole side is one device-resident CSR built by
//   dense id map  (flag -> exclusive scan)                 als_index_build
//   stable LSD radix sort of (dense row, position)          als_csr_build
//   histogram -> exclusive scan for the int64 row pointer
// plus the per-half-sweep work schedule (als_schedule_*).
//
// Everything here is integer work and is bit-exact against the oracle
// (oracle/als_oracle.py: index_build / csr_build / schedule_build).
#include "als_common.h"

namespace als {

static thread_local char g_err[512];
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// ----------------------------------------------------------------------------
// Block-wide helpers (256 threads = 4 wavefronts of 64)
// ----------------------------------------------------------------------------
__device__ __forceinline__ int64_t shfl_up_i64(int64_t v, int d) {
  int2 iv = __builtin_bit_cast(int2, v);
  iv.x = __shfl_up(iv.x, d);
  iv.y = __shfl_up(iv.y, d);
  return __builtin_bit_cast(int64_t, iv);
}
__device__ __forceinline__ int64_t shfl_xor_i64(int64_t v, int d) {
  int2 iv = __builtin_bit_cast(int2, v);
  iv.x = __shfl_xor(iv.x, d);
  iv.y = __shfl_xor(iv.y, d);
  return __builtin_bit_cast(int64_t, iv);
}

// Exclusive scan of one int64 per thread over a 256-thread block; *total gets the block sum.
__device__ __forceinline__ int64_t block_exclusive_scan_256(int64_t v, int64_t* total) {
  __shared__ int64_t wsum[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    int64_t o = shfl_up_i64(inc, d);
    if (lane >= d) inc += o;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  int64_t woff = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int64_t s = wsum[i];
    woff += (i < w) ? s : 0;
    tot += s;
  }
  __syncthreads();  // wsum may be reused by the caller's next call
  if (total) *total = tot;
  return woff + inc - v;
}

__device__ __forceinline__ int64_t block_reduce_sum_256(int64_t v) {
  __shared__ int64_t wsum[4];
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += shfl_xor_i64(v, d);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = v;
  __syncthreads();
  int64_t t = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  __syncthreads();
  return t;
}

// ----------------------------------------------------------------------------
// Exclusive scan (3-phase, recursive over block sums)
// ----------------------------------------------------------------------------
constexpr int SCAN_ITEMS = 8;
constexpr int SCAN_TILE = 256 * SCAN_ITEMS;

template <class Tin>
__global__ __launch_bounds__(256) void scan_reduce_kernel(const Tin* __restrict__ in, int64_t n,
                                                          int64_t* __restrict__ sums) {
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
  int64_t s = 0;
#pragma unroll
  for (int i = 0; i < SCAN_ITEMS; ++i) {
    int64_t idx = base + i * 256 + threadIdx.x;
    if (idx < n) s += (int64_t)in[idx];
  }
  s = block_reduce_sum_256(s);
  if (threadIdx.x == 0) sums[blockIdx.x] = s;
}

template <class Tin, class Tout>
__global__ __launch_bounds__(256) void scan_apply_kernel(const Tin* in, Tout* out, int64_t n,
                                                         const int64_t* __restrict__ offs) {
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_ITEMS;
  int64_t v[SCAN_ITEMS];
  int64_t tsum = 0;
#pragma unroll
  for (int i = 0; i < SCAN_ITEMS; ++i) {
    int64_t idx = base + i;
    v[i] = idx < n ? (int64_t)in[idx] : 0;
    tsum += v[i];
  }
  int64_t run = block_exclusive_scan_256(tsum, nullptr) + (offs ? offs[blockIdx.x] : 0);
#pragma unroll
  for (int i = 0; i < SCAN_ITEMS; ++i) {
    int64_t idx = base + i;
    if (idx < n) out[idx] = (Tout)run;
    run += v[i];
  }
}

static void scan_ws_levels(int64_t n, ArenaSize& a) {
  while (n > SCAN_TILE) {
    int64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
    a.take<int64_t>(nb);
    n = nb;
  }
}
size_t scan_workspace_bytes(int64_t n) {
  ArenaSize a;
  scan_ws_levels(n, a);
  return a.off + 256;
}

template <class Tin, class Tout>
static int scan_exclusive_impl(const Tin* in, Tout* out, int64_t n, Arena& ar, hipStream_t st) {
  if (n <= 0) return ALS_OK;
  int64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
  if (nb == 1) {
    scan_apply_kernel<Tin, Tout><<<1, 256, 0, st>>>(in, out, n, nullptr);
    ALS_LAUNCH_CHECK();
    return ALS_OK;
  }
  int64_t* sums = ar.take<int64_t>(nb);
  ALS_REQUIRE(sums, ALS_EWORKSPACE, "scan: workspace too small");
  scan_reduce_kernel<Tin><<<(unsigned)nb, 256, 0, st>>>(in, n, sums);
  ALS_LAUNCH_CHECK();
  int rc = scan_exclusive_impl<int64_t, int64_t>(sums, sums, nb, ar, st);
  if (rc) return rc;
  scan_apply_kernel<Tin, Tout><<<(unsigned)nb, 256, 0, st>>>(in, out, n, sums);
  ALS_LAUNCH_CHECK();
  return ALS_OK;
}

int scan_exclusive_i32_to_i64(const int32_t* in, int64_t* out, int64_t n, void* ws,
                              size_t ws_bytes, hipStream_t st) {
  Arena ar(ws, ws_bytes);
  return scan_exclusive_impl<int32_t, int64_t>(in, out, n, ar, st);
}
int scan_exclusive_i32(const int32_t* in, int32_t* out, int64_t n, void* ws, size_t ws_bytes,
                       hipStream_t st) {
  Arena ar(ws, ws_bytes);
  return scan_exclusive_impl<int32_t, int32_t>(in, out, n, ar, st);
}

// ----------------------------------------------------------------------------
// Stable LSD radix sort, 8-bit digits, 4096-key tiles.
// Element (round r, thread t) of tile b is key[b*4096 + r*256 + t]; ranks are
// assigned in that order, so equal digits keep input order (stable).
// ----------------------------------------------------------------------------
constexpr int RS_ITEMS = 16;
constexpr int RS_TILE = 256 * RS_ITEMS;

__global__ __launch_bounds__(256) void rs_hist_kernel(const uint32_t* __restrict__ keys, int64_t n,
                                                      int shift, int32_t* __restrict__ hist,
                                                      int ntiles) {
  __shared__ int h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * RS_TILE;
#pragma unroll 4
  for (int r = 0; r < RS_ITEMS; ++r) {
    int64_t idx = base + r * 256 + threadIdx.x;
    if (idx < n) atomicAdd(&h[(keys[idx] >> shift) & 255], 1);
  }
  __syncthreads();
  hist[(int64_t)threadIdx.x * ntiles + blockIdx.x] = h[threadIdx.x];
}

__global__ __launch_bounds__(256) void rs_scatter_kernel(const uint32_t* __restrict__ kin,
                                                         const int32_t* __restrict__ vin,
                                                         uint32_t* __restrict__ kout,
                                                         int32_t* __restrict__ vout, int64_t n,
                                                         int shift,
                                                         const int32_t* __restrict__ offs,
                                                         int ntiles) {
  __shared__ int cnt[256];
  __shared__ int wcnt[4][256];
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  cnt[t] = offs[(int64_t)t * ntiles + blockIdx.x];
#pragma unroll
  for (int i = 0; i < 4; ++i) wcnt[i][t] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * RS_TILE;
  const uint64_t lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
  for (int r = 0; r < RS_ITEMS; ++r) {
    const int64_t idx = base + r * 256 + t;
    const bool valid = idx < n;
    const uint32_t key = valid ? kin[idx] : 0u;
    const int32_t val = valid ? vin[idx] : 0;
    const int d = (key >> shift) & 255;
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const bool bit = (d >> b) & 1;
      const uint64_t bb = __ballot(valid && bit);
      peers &= bit ? bb : ~bb;
    }
    const int prefix = __popcll(peers & lt);
    if (valid && prefix == 0) wcnt[w][d] = __popcll(peers);
    __syncthreads();
    if (valid) {
      int pos = cnt[d] + prefix;
      for (int ww = 0; ww < w; ++ww) pos += wcnt[ww][d];
      kout[pos] = key;
      vout[pos] = val;
    }
    __syncthreads();
    cnt[t] += wcnt[0][t] + wcnt[1][t] + wcnt[2][t] + wcnt[3][t];
    wcnt[0][t] = 0;
    wcnt[1][t] = 0;
    wcnt[2][t] = 0;
    wcnt[3][t] = 0;
    __syncthreads();
  }
}

static void radix_ws(int64_t n, ArenaSize& a) {
  int64_t ntiles = (n + RS_TILE - 1) / RS_TILE;
  a.take<int32_t>(256 * ntiles);  // hist / offsets (scanned in place)
  a.take<uint32_t>(n);            // ping-pong keys
  a.take<int32_t>(n);             // ping-pong vals
  a.off += scan_workspace_bytes(256 * ntiles);
}
size_t radix_workspace_bytes(int64_t n) {
  ArenaSize a;
  radix_ws(n, a);
  return a.off + 256;
}

int radix_sort_pairs(const uint32_t* kin, const int32_t* vin, uint32_t* kout, int32_t* vout,
                     int64_t n, int bits, void* ws, size_t ws_bytes, hipStream_t st) {
  if (n <= 0) return ALS_OK;
  ALS_REQUIRE(n < (int64_t(1) << 31), ALS_EINVAL, "radix_sort: n >= 2^31 not supported");
  Arena ar(ws, ws_bytes);
  const int64_t ntiles = (n + RS_TILE - 1) / RS_TILE;
  int32_t* hist = ar.take<int32_t>(256 * ntiles);
  uint32_t* ktmp = ar.take<uint32_t>(n);
  int32_t* vtmp = ar.take<int32_t>(n);
  ALS_REQUIRE(hist && ktmp && vtmp, ALS_EWORKSPACE, "radix_sort: workspace too small");
  void* scan_ws = ar.base + ar.off;
  size_t scan_bytes = ar.cap - ar.off;
  int passes = bits <= 0 ? 1 : (bits + 7) / 8;
  const uint32_t* ks = kin;
  const int32_t* vs = vin;
  for (int p = 0; p < passes; ++p) {
    // the last pass lands in (kout, vout); earlier passes alternate so that holds
    const bool to_out = ((passes - 1 - p) % 2) == 0;
    uint32_t* kd = to_out ? kout : ktmp;
    int32_t* vd = to_out ? vout : vtmp;
    rs_hist_kernel<<<(unsigned)ntiles, 256, 0, st>>>(ks, n, 8 * p, hist, (int)ntiles);
    ALS_LAUNCH_CHECK();
    int rc = scan_exclusive_i32(hist, hist, 256 * ntiles, scan_ws, scan_bytes, st);
    if (rc) return rc;
    rs_scatter_kernel<<<(unsigned)ntiles, 256, 0, st>>>(ks, vs, kd, vd, n, 8 * p, hist,
                                                        (int)ntiles);
    ALS_LAUNCH_CHECK();
    ks = kd;
    vs = vd;
  }
  return ALS_OK;
}

static int bit_length(uint64_t x) {
  int b = 0;
  while (x) {
    ++b;
    x >>= 1;
  }
  return b;
}

static unsigned grid_for(int64_t n, int per_block = 256, int64_t cap = 65536) {
  int64_t g = (n + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

// ----------------------------------------------------------------------------
// Index build
// ----------------------------------------------------------------------------
__global__ void idx_mark_kernel(const int32_t* __restrict__ ids, int64_t n, int32_t id_space,
                                int32_t* __restrict__ flag) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    int32_t id = ids[e];
    if (id >= 0 && id < id_space) flag[id] = 1;
  }
}

__global__ void idx_finalize_kernel(const int32_t* __restrict__ flag,
                                    const int32_t* __restrict__ pos, int32_t id_space,
                                    int32_t* __restrict__ map, int32_t* __restrict__ uniq,
                                    int32_t* __restrict__ n_uniq) {
  for (int64_t id = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; id < id_space;
       id += (int64_t)gridDim.x * blockDim.x) {
    const int32_t f = flag[id], p = pos[id];
    map[id] = f ? p : -1;
    if (f) uniq[p] = (int32_t)id;
    if (id == id_space - 1) *n_uniq = p + f;
  }
}

}  // namespace als

using namespace als;

extern "C" {

const char* als_last_error(void) { return als::g_err; }
int als_abi_version(void) { return ALS_ABI_VERSION; }
int als_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

size_t als_index_workspace_bytes(int64_t n, int32_t id_space) {
  (void)n;
  ArenaSize a;
  a.take<int32_t>(id_space);  // flag
  a.take<int32_t>(id_space);  // pos
  a.off += scan_workspace_bytes(id_space);
  return a.off + 256;
}

int als_index_build(const int32_t* ids, int64_t n, int32_t id_space, int32_t* map_out,
                    int32_t* uniq_out, int32_t* n_uniq_dev, void* ws, size_t ws_bytes,
                    void* stream) {
  ALS_REQUIRE(id_space > 0, ALS_EINVAL, "als_index_build: id_space must be > 0");
  ALS_REQUIRE(n >= 0 && (n == 0 || ids), ALS_EINVAL, "als_index_build: bad ids");
  ALS_REQUIRE(map_out && uniq_out && n_uniq_dev, ALS_EINVAL, "als_index_build: null output");
  ALS_REQUIRE(ws_bytes >= als_index_workspace_bytes(n, id_space), ALS_EWORKSPACE,
              "als_index_build: workspace %zu < %zu", ws_bytes,
              als_index_workspace_bytes(n, id_space));
  hipStream_t st = as_stream(stream);
  Arena ar(ws, ws_bytes);
  int32_t* flag = ar.take<int32_t>(id_space);
  int32_t* pos = ar.take<int32_t>(id_space);
  ALS_HIP(hipMemsetAsync(flag, 0, sizeof(int32_t) * (size_t)id_space, st));
  if (n > 0) {
    idx_mark_kernel<<<grid_for(n), 256, 0, st>>>(ids, n, id_space, flag);
    ALS_LAUNCH_CHECK();
  }
  int rc = scan_exclusive_i32(flag, pos, id_space, ar.base + ar.off, ar.cap - ar.off, st);
  if (rc) return rc;
  idx_finalize_kernel<<<grid_for(id_space), 256, 0, st>>>(flag, pos, id_space, map_out, uniq_out,
                                                          n_uniq_dev);
  ALS_LAUNCH_CHECK();
  return ALS_OK;
}

}  // extern "C"

namespace als {

__global__ void csr_keys_kernel(const int32_t* __restrict__ row_ids,
                                const int32_t* __restrict__ row_map, int64_t nnz,
                                uint32_t* __restrict__ keys, int32_t* __restrict__ perm,
                                int32_t* __restrict__ counts) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nnz;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int32_t r = row_map[row_ids[e]];
    keys[e] = (uint32_t)r;
    perm[e] = (int32_t)e;
    atomicAdd(&counts[r], 1);
  }
}

__global__ void csr_gather_kernel(const int32_t* __restrict__ perm,
                                  const int32_t* __restrict__ col_ids,
                                  const int32_t* __restrict__ col_map,
                                  const float* __restrict__ vals, int64_t nnz,
                                  int32_t* __restrict__ col_out, float* __restrict__ val_out) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < nnz;
       p += (int64_t)gridDim.x * blockDim.x) {
    const int32_t e = perm[p];
    col_out[p] = col_map[col_ids[e]];
    val_out[p] = vals[e];
  }
}

// ---- schedule ----
__global__ void sched_count_kernel(const int64_t* __restrict__ row_ptr, int32_t n_rows,
                                   int32_t chunk, int32_t* __restrict__ counts) {
  int32_t light = 0, heavy = 0, chunks = 0;
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n_rows;
       r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t deg = row_ptr[r + 1] - row_ptr[r];
    if (deg > chunk) {
      heavy += 1;
      chunks += (int32_t)((deg + chunk - 1) / chunk);
    } else {
      light += 1;
    }
  }
  int64_t l = block_reduce_sum_256(light), h = block_reduce_sum_256(heavy),
          c = block_reduce_sum_256(chunks);
  if (threadIdx.x == 0) {
    atomicAdd(&counts[0], (int32_t)l);
    atomicAdd(&counts[1], (int32_t)h);
    atomicAdd(&counts[2], (int32_t)c);
  }
}

__global__ void sched_keys_kernel(const int64_t* __restrict__ row_ptr, int32_t n_rows,
                                  int32_t chunk, uint32_t* __restrict__ keys,
                                  int32_t* __restrict__ rows) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n_rows;
       r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t deg = row_ptr[r + 1] - row_ptr[r];
    // light rows first, longest first (LPT order); heavy rows last, by row id
    keys[r] = deg > chunk ? (uint32_t)chunk + 1u : (uint32_t)(chunk - deg);
    rows[r] = (int32_t)r;
  }
}

__global__ void sched_heavy_nc_kernel(const int64_t* __restrict__ row_ptr,
                                      const int32_t* __restrict__ heavy_rows, int32_t n_heavy,
                                      int32_t chunk, int32_t* __restrict__ nc) {
  for (int64_t h = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; h <= n_heavy;
       h += (int64_t)gridDim.x * blockDim.x) {
    if (h == n_heavy) {
      nc[h] = 0;
    } else {
      const int32_t r = heavy_rows[h];
      const int64_t deg = row_ptr[r + 1] - row_ptr[r];
      nc[h] = (int32_t)((deg + chunk - 1) / chunk);
    }
  }
}

__global__ void sched_emit_kernel(const int64_t* __restrict__ row_ptr,
                                  const int32_t* __restrict__ heavy_rows, int32_t n_heavy,
                                  const int32_t* __restrict__ slot_begin, int32_t chunk,
                                  int32_t* __restrict__ chunk_row,
                                  int64_t* __restrict__ chunk_begin,
                                  int64_t* __restrict__ chunk_end) {
  for (int64_t h = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; h < n_heavy;
       h += (int64_t)gridDim.x * blockDim.x) {
    const int32_t r = heavy_rows[h];
    const int64_t b = row_ptr[r], e = row_ptr[r + 1];
    int32_t s = slot_begin[h];
    for (int64_t p = b; p < e; p += chunk, ++s) {
      chunk_row[s] = r;
      chunk_begin[s] = p;
      chunk_end[s] = p + chunk < e ? p + chunk : e;
    }
  }
}

}  // namespace als

extern "C" {

size_t als_csr_workspace_bytes(int64_t nnz, int32_t n_rows) {
  ArenaSize a;
  a.take<uint32_t>(nnz);  // keys
  a.take<int32_t>(nnz);   // perm
  a.take<uint32_t>(nnz);  // sorted keys
  a.take<int32_t>(nnz);   // sorted perm
  a.take<int32_t>((size_t)n_rows + 1);  // counts
  size_t inner = radix_workspace_bytes(nnz);
  size_t sc = scan_workspace_bytes((int64_t)n_rows + 1);
  a.off += inner > sc ? inner : sc;
  return a.off + 256;
}

int als_csr_build(const int32_t* row_ids, const int32_t* row_map, const int32_t* col_ids,
                  const int32_t* col_map, const float* vals, int64_t nnz, int32_t n_rows,
                  int64_t* row_ptr_out, int32_t* col_out, float* val_out, void* ws,
                  size_t ws_bytes, void* stream) {
  ALS_REQUIRE(nnz >= 0 && nnz < (int64_t(1) << 31), ALS_EINVAL,
              "als_csr_build: nnz must be in [0, 2^31)");
  ALS_REQUIRE(n_rows >= 0, ALS_EINVAL, "als_csr_build: n_rows < 0");
  ALS_REQUIRE(row_ptr_out, ALS_EINVAL, "als_csr_build: null row_ptr_out");
  ALS_REQUIRE(nnz == 0 || (row_ids && row_map && col_ids && col_map && vals && col_out && val_out),
              ALS_EINVAL, "als_csr_build: null pointer");
  ALS_REQUIRE(ws_bytes >= als_csr_workspace_bytes(nnz, n_rows), ALS_EWORKSPACE,
              "als_csr_build: workspace %zu < %zu", ws_bytes, als_csr_workspace_bytes(nnz, n_rows));
  hipStream_t st = as_stream(stream);
  Arena ar(ws, ws_bytes);
  uint32_t* keys = ar.take<uint32_t>(nnz);
  int32_t* perm = ar.take<int32_t>(nnz);
  uint32_t* skeys = ar.take<uint32_t>(nnz);
  int32_t* sperm = ar.take<int32_t>(nnz);
  int32_t* counts = ar.take<int32_t>((size_t)n_rows + 1);
  void* inner = ar.base + ar.off;
  size_t inner_bytes = ar.cap - ar.off;
  ALS_HIP(hipMemsetAsync(counts, 0, sizeof(int32_t) * ((size_t)n_rows + 1), st));
  if (nnz > 0) {
    csr_keys_kernel<<<grid_for(nnz), 256, 0, st>>>(row_ids, row_map, nnz, keys, perm, counts);
    ALS_LAUNCH_CHECK();
    int bits = bit_length(n_rows > 0 ? (uint64_t)(n_rows - 1) : 0);
    int rc = radix_sort_pairs(keys, perm, skeys, sperm, nnz, bits, inner, inner_bytes, st);
    if (rc) return rc;
    csr_gather_kernel<<<grid_for(nnz), 256, 0, st>>>(sperm, col_ids, col_map, vals, nnz, col_out,
                                                     val_out);
    ALS_LAUNCH_CHECK();
  }
  return scan_exclusive_i32_to_i64(counts, row_ptr_out, (int64_t)n_rows + 1, inner, inner_bytes,
                                   st);
}

size_t als_schedule_workspace_bytes(int32_t n_rows) {
  ArenaSize a;
  a.take<uint32_t>(n_rows);
  a.take<int32_t>(n_rows);
  a.take<uint32_t>(n_rows);
  a.take<int32_t>(n_rows);
  a.take<int32_t>((size_t)n_rows + 1);
  size_t r = radix_workspace_bytes(n_rows), s = scan_workspace_bytes((int64_t)n_rows + 1);
  a.off += r > s ? r : s;
  return a.off + 256;
}

int als_schedule_count(const int64_t* row_ptr, int32_t n_rows, int32_t chunk, int32_t* counts_dev,
                       void* stream) {
  ALS_REQUIRE(chunk > 0, ALS_EINVAL, "als_schedule_count: chunk must be > 0");
  ALS_REQUIRE(row_ptr && counts_dev, ALS_EINVAL, "als_schedule_count: null pointer");
  hipStream_t st = as_stream(stream);
  ALS_HIP(hipMemsetAsync(counts_dev, 0, 3 * sizeof(int32_t), st));
  if (n_rows > 0) {
    sched_count_kernel<<<grid_for(n_rows, 256, 1024), 256, 0, st>>>(row_ptr, n_rows, chunk,
                                                                    counts_dev);
    ALS_LAUNCH_CHECK();
  }
  return ALS_OK;
}

int als_schedule_build(const int64_t* row_ptr, int32_t n_rows, int32_t chunk, int32_t n_light,
                       int32_t n_heavy, int32_t n_chunks, int32_t* light_rows,
                       int32_t* heavy_rows, int32_t* heavy_slot_begin, int32_t* chunk_row,
                       int64_t* chunk_begin, int64_t* chunk_end, void* ws, size_t ws_bytes,
                       void* stream) {
  ALS_REQUIRE(chunk > 0 && n_light >= 0 && n_heavy >= 0 && n_chunks >= 0 &&
                  n_light + n_heavy == n_rows,
              ALS_EINVAL, "als_schedule_build: inconsistent counts");
  ALS_REQUIRE(ws_bytes >= als_schedule_workspace_bytes(n_rows), ALS_EWORKSPACE,
              "als_schedule_build: workspace too small");
  ALS_REQUIRE(heavy_slot_begin, ALS_EINVAL, "als_schedule_build: null heavy_slot_begin");
  hipStream_t st = as_stream(stream);
  Arena ar(ws, ws_bytes);
  uint32_t* keys = ar.take<uint32_t>(n_rows);
  int32_t* rows = ar.take<int32_t>(n_rows);
  uint32_t* skeys = ar.take<uint32_t>(n_rows);
  int32_t* srows = ar.take<int32_t>(n_rows);
  int32_t* nc = ar.take<int32_t>((size_t)n_rows + 1);
  void* inner = ar.base + ar.off;
  size_t inner_bytes = ar.cap - ar.off;
  if (n_rows > 0) {
    sched_keys_kernel<<<grid_for(n_rows), 256, 0, st>>>(row_ptr, n_rows, chunk, keys, rows);
    ALS_LAUNCH_CHECK();
    int rc = radix_sort_pairs(keys, rows, skeys, srows, n_rows, bit_length((uint64_t)chunk + 1),
                              inner, inner_bytes, st);
    if (rc) return rc;
    if (n_light > 0)
      ALS_HIP(hipMemcpyAsync(light_rows, srows, sizeof(int32_t) * n_light,
                             hipMemcpyDeviceToDevice, st));
    if (n_heavy > 0)
      ALS_HIP(hipMemcpyAsync(heavy_rows, srows + n_light, sizeof(int32_t) * n_heavy,
                             hipMemcpyDeviceToDevice, st));
  }
  sched_heavy_nc_kernel<<<grid_for((int64_t)n_heavy + 1), 256, 0, st>>>(row_ptr, heavy_rows,
                                                                        n_heavy, chunk, nc);
  ALS_LAUNCH_CHECK();
  int rc = scan_exclusive_i32(nc, heavy_slot_begin, (int64_t)n_heavy + 1, inner, inner_bytes, st);
  if (rc) return rc;
  if (n_heavy > 0) {
    sched_emit_kernel<<<grid_for(n_heavy), 256, 0, st>>>(row_ptr, heavy_rows, n_heavy,
                                                         heavy_slot_begin, chunk, chunk_row,
                                                         chunk_begin, chunk_end);
    ALS_LAUNCH_CHECK();
  }
  return ALS_OK;
}

}  // extern "C"
