// keys.hip -- query-global key ids of raw FLOAT / DOUBLE group-by columns. The reference keys a no-dictionary
// column by its values (NoDictionarySingleColumnGroupKeyGenerator / NoDictionaryMultiColumnGroupKeyGenerator, chosen
// by DefaultGroupByExecutor.java:106-116; fastutil's Double2IntOpenHashMap compares keys by Double.doubleToLongBits,
// so -0.0 and 0.0 are two keys and every NaN is one). Here the key space is the sorted set of distinct values over
// the query's segments -- a dictionary built once per (column, segments) on the device: per segment the values'
// Double.compare images are radix-sorted and made unique, the segments' uniques are merged the same way, and a
// doc-order int32 id column per segment (binary search of each doc's image) feeds the group key like a dictionary
// id (DevCol.gb_ids). FLOAT values widen to double exactly, so one path serves both.
#include <hipcub/hipcub.hpp>

#include "dev_common.h"

namespace phip {

// Double.compare order as unsigned: positives with the sign bit set, negatives with every bit flipped; NaN canonical
// (Double.doubleToLongBits) so all NaNs are one key, after +inf.
__device__ __forceinline__ uint64_t f64_order_image(double v) {
  uint64_t b = (uint64_t)__double_as_longlong(v);
  if (v != v) b = 0x7ff8000000000000ull;
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

__device__ __forceinline__ double raw_real(const void *raw, int32_t type, int64_t i) {
  return type == PHIP_TYPE_FLOAT ? (double)((const float *)raw)[i] : ((const double *)raw)[i];
}

__global__ void raw_images_kernel(const void *__restrict__ raw, int32_t type, int64_t n, uint64_t *__restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = f64_order_image(raw_real(raw, type, i));
}

// ids[i] = position of doc i's image in the sorted distinct images (present by construction)
__global__ void raw_key_ids_kernel(const void *__restrict__ raw, int32_t type, int64_t n, const uint64_t *__restrict__ uniq,
                                   int64_t u, int32_t *__restrict__ ids) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t k = f64_order_image(raw_real(raw, type, i));
    int64_t lo = 0, hi = u;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (uniq[mid] < k) lo = mid + 1;
      else hi = mid;
    }
    ids[i] = (int32_t)lo;
  }
}

static inline int keys_grid(int64_t n) {
  const int64_t g = (n + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

hipError_t launch_raw_images(const void *raw, int32_t type, int64_t n, uint64_t *out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  raw_images_kernel<<<keys_grid(n), 256, 0, s>>>(raw, type, n, out);
  return hipGetLastError();
}

// sorted distinct u64 keys of in[0, n) into out (temp == nullptr: the scratch bytes both passes need)
hipError_t launch_sort_unique_u64(void *temp, size_t *temp_bytes, uint64_t *in, uint64_t *sorted, uint64_t *out,
                                  int64_t *num_out, int64_t n, hipStream_t s) {
  size_t a = 0, b = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortKeys(nullptr, a, (const uint64_t *)in, sorted, (int)n, 0, 64, s);
  if (e != hipSuccess) return e;
  e = hipcub::DeviceSelect::Unique(nullptr, b, (const uint64_t *)sorted, out, num_out, (int)n, s);
  if (e != hipSuccess) return e;
  if (temp == nullptr) {
    *temp_bytes = a > b ? a : b;
    return hipSuccess;
  }
  if (n <= 0) return hipMemsetAsync(num_out, 0, 8, s);
  e = hipcub::DeviceRadixSort::SortKeys(temp, a, (const uint64_t *)in, sorted, (int)n, 0, 64, s);
  if (e != hipSuccess) return e;
  return hipcub::DeviceSelect::Unique(temp, b, (const uint64_t *)sorted, out, num_out, (int)n, s);
}

hipError_t launch_raw_key_ids(const void *raw, int32_t type, int64_t n, const uint64_t *uniq, int64_t u, int32_t *ids,
                              hipStream_t s) {
  if (n <= 0) return hipSuccess;
  raw_key_ids_kernel<<<keys_grid(n), 256, 0, s>>>(raw, type, n, uniq, u, ids);
  return hipGetLastError();
}

}  // namespace phip
