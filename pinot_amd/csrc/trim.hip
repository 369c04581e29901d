// trim.hip -- server-level group trim on the device.
//
// The reference's combine keeps, for a group-by with ORDER BY, only the top
// trimSize = GroupByUtils.getTableCapacity(limit, minServerGroupTrimSize) = max(5 * limit, 5000) records
// (GroupByUtils.java:55-58,96-140; IndexedTable.finish -> TableResizer.getTopRecords). Here the compacted
// groups are ordered on the device by a 64-bit order-preserving image of the ORDER BY aggregation
// (Double.compare order: -0.0 < 0.0, NaN last), radix-sorted as (key, group index) pairs -- a stable sort,
// so ties at the trim boundary keep the lowest group index -- and only the first trimSize groups are
// gathered and copied to the host.
#include <hipcub/hipcub.hpp>

#include "dev_common.h"

namespace phip {

__global__ void order_keys_kernel(const double *__restrict__ vals, int64_t n, int32_t naggs, int32_t agg, int32_t desc,
                                  uint64_t *__restrict__ ukeys, int32_t *__restrict__ idx) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n; g += (int64_t)gridDim.x * blockDim.x) {
    uint64_t u = (uint64_t)__double_as_longlong(vals[g * naggs + agg]);
    u = (u >> 63) ? ~u : (u | 0x8000000000000000ull);
    ukeys[g] = desc ? ~u : u;
    idx[g] = (int32_t)g;
  }
}

__global__ void trim_gather_kernel(const int32_t *__restrict__ order, int64_t k, int32_t naggs, int64_t hll_bytes,
                                   const int64_t *__restrict__ keys, const double *__restrict__ vals,
                                   const int64_t *__restrict__ longs, const uint8_t *__restrict__ hll,
                                   int64_t *__restrict__ keys_out, double *__restrict__ vals_out,
                                   int64_t *__restrict__ longs_out, uint8_t *__restrict__ hll_out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < k; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t g = order[i];
    keys_out[i] = keys[g];
    for (int a = 0; a < naggs; a++) {
      vals_out[i * naggs + a] = vals[g * naggs + a];
      longs_out[i * naggs + a] = longs[g * naggs + a];
    }
    for (int64_t b = 0; b < hll_bytes; b++) hll_out[i * hll_bytes + b] = hll[g * hll_bytes + b];
  }
}

// ORDER BY group-by columns: the global key (mixed radix, group-by column 0 least significant) is decoded
// and re-composed in ORDER BY order, DESC columns as card - 1 - id.
__global__ void key_order_kernel(const int64_t *__restrict__ keys, int64_t n, KeyOrder ko, uint64_t *__restrict__ ukeys,
                                 int32_t *__restrict__ idx) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n; g += (int64_t)gridDim.x * blockDim.x) {
    int64_t key = keys[g], id[kMaxOrderKeys];
    for (int k = 0; k < ko.num_group_by; k++) {
      id[k] = key % ko.card[k];
      key /= ko.card[k];
    }
    uint64_t u = 0;
    for (int j = 0; j < ko.num_keys; j++) {
      const int k = ko.gb[j];
      u = u * (uint64_t)ko.card[k] + (uint64_t)(ko.desc[j] ? ko.card[k] - 1 - id[k] : id[k]);
    }
    ukeys[g] = u;
    idx[g] = (int32_t)g;
  }
}

// One radix pass of the general ORDER BY: the 64-bit order-preserving key of term j for every group, in the
// order the previous (less significant) pass left them (perm == nullptr: group order).
__device__ __forceinline__ uint64_t double_order(double d) {
  const uint64_t u = (uint64_t)__double_as_longlong(d);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);  // Double.compare order: -0.0 < 0.0, NaN last
}

// clearspring HyperLogLog.cardinality() (stream-lib 2.9.8, DistinctCountHLLAggregationFunction.extractFinalResult;
// engine/reduce.py hll_cardinality): alpha * m^2 / sum 2^-reg, linear counting below 2.5 m (Long.MAX_VALUE when no
// register is zero), rounded half up. The sum of dyadic terms is exact in any order.
__device__ double hll_estimate(const uint8_t *regs, int32_t log2m) {
  const int32_t m = 1 << log2m;
  const double md = (double)m;
  double alpha_mm;
  if (log2m == 4) alpha_mm = 0.673 * md * md;
  else if (log2m == 5) alpha_mm = 0.697 * md * md;
  else if (log2m == 6) alpha_mm = 0.709 * md * md;
  else alpha_mm = (0.7213 / (1.0 + 1.079 / md)) * md * md;
  double s = 0.0;
  int32_t zeros = 0;
  for (int32_t r = 0; r < m; r++) {
    s += 1.0 / (double)(1ull << regs[r]);
    zeros += regs[r] == 0;
  }
  const double est = alpha_mm * (1.0 / s);
  if (est <= 2.5 * md) {
    if (zeros == 0) return 9223372036854775807.0;
    return floor(md * log(md / (double)zeros) + 0.5);
  }
  return floor(est + 0.5);
}

__global__ void term_keys_kernel(const double *__restrict__ vals, const int64_t *__restrict__ keys, int64_t n,
                                 int32_t naggs, OrderTerms ot, int32_t j, const int32_t *__restrict__ perm,
                                 const uint8_t *__restrict__ hll, int64_t hll_bytes, int32_t m_regs,
                                 uint64_t *__restrict__ ukeys, int32_t *__restrict__ idx) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t g = perm ? perm[i] : i;
    uint64_t u;
    if (ot.kind[j] == TERM_GROUP_KEY) {
      int64_t key = keys[g], id = 0;
      for (int k = 0; k <= ot.a[j]; k++) {
        id = key % ot.card[k];
        key /= ot.card[k];
      }
      u = (uint64_t)(ot.desc[j] ? ot.card[ot.a[j]] - 1 - id : id);
    } else if (ot.kind[j] == TERM_HLL) {
      u = double_order(hll_estimate(hll + g * hll_bytes + (int64_t)ot.a[j] * m_regs, ot.b[j]));
      if (ot.desc[j]) u = ~u;
    } else {
      const double *v = vals + g * naggs;
      double d;
      if (ot.kind[j] == TERM_VALUE) {
        d = v[ot.a[j]];
      } else if (ot.kind[j] == TERM_AVG) {  // AvgAggregationFunction.extractFinalResult: -inf without docs
        d = v[ot.b[j]] != 0.0 ? v[ot.a[j]] / v[ot.b[j]] : -__builtin_huge_val();
      } else {                               // MinMaxRangeAggregationFunction.extractFinalResult: max - min
        d = v[ot.b[j]] - v[ot.a[j]];
      }
      u = double_order(d);
      if (ot.desc[j]) u = ~u;
    }
    ukeys[i] = u;
    idx[i] = (int32_t)g;
  }
}

static inline int trim_grid(int64_t n) {
  int64_t g = (n + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

// Scratch: ukeys[2n] (u64), idx[2n] (i32), then the sort's temp storage; *temp_bytes reports the total when
// scratch == nullptr.
hipError_t launch_trim_order(const double *vals, const int64_t *keys, const KeyOrder *ko, int64_t n, int32_t naggs,
                             int32_t agg, int32_t desc, void *scratch, size_t *scratch_bytes, const int32_t **order_out,
                             hipStream_t s) {
  size_t sort_bytes = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, (const uint64_t *)nullptr, (uint64_t *)nullptr,
                                                    (const int32_t *)nullptr, (int32_t *)nullptr, (int)n, 0, 64, s);
  if (e != hipSuccess) return e;
  const size_t keys_bytes = ((size_t)n * 16 + 255) & ~(size_t)255, idx_bytes = ((size_t)n * 8 + 255) & ~(size_t)255;
  if (scratch == nullptr) {
    *scratch_bytes = keys_bytes + idx_bytes + sort_bytes;
    return hipSuccess;
  }
  uint64_t *k0 = (uint64_t *)scratch, *k1 = k0 + n;
  int32_t *i0 = (int32_t *)((uint8_t *)scratch + keys_bytes), *i1 = i0 + n;
  void *tmp = (uint8_t *)scratch + keys_bytes + idx_bytes;
  if (ko != nullptr)
    key_order_kernel<<<trim_grid(n), 256, 0, s>>>(keys, n, *ko, k0, i0);
  else
    order_keys_kernel<<<trim_grid(n), 256, 0, s>>>(vals, n, naggs, agg, desc, k0, i0);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = hipcub::DeviceRadixSort::SortPairs(tmp, sort_bytes, k0, k1, i0, i1, (int)n, 0, 64, s);
  *order_out = i1;
  return e;
}

static inline int key_bits(int64_t card) {
  int b = 1;
  while (b < 64 && ((int64_t)1 << b) < card) b++;
  return b;
}

// General ORDER BY: one stable radix pass per term, least significant term first (LSD over terms), so ties
// on every term keep the lowest group index. Same scratch layout as launch_trim_order.
hipError_t launch_trim_order_terms(const double *vals, const int64_t *keys, const OrderTerms *ot, int64_t n,
                                   int32_t naggs, const uint8_t *hll, int64_t hll_bytes, int32_t m_regs, void *scratch,
                                   size_t *scratch_bytes, const int32_t **order_out, hipStream_t s) {
  size_t sort_bytes = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, (const uint64_t *)nullptr, (uint64_t *)nullptr,
                                                    (const int32_t *)nullptr, (int32_t *)nullptr, (int)n, 0, 64, s);
  if (e != hipSuccess) return e;
  const size_t keys_bytes = ((size_t)n * 16 + 255) & ~(size_t)255, idx_bytes = ((size_t)n * 8 + 255) & ~(size_t)255;
  if (scratch == nullptr) {
    *scratch_bytes = keys_bytes + idx_bytes + sort_bytes;
    return hipSuccess;
  }
  uint64_t *k0 = (uint64_t *)scratch, *k1 = k0 + n;
  int32_t *i0 = (int32_t *)((uint8_t *)scratch + keys_bytes), *i1 = i0 + n;
  void *tmp = (uint8_t *)scratch + keys_bytes + idx_bytes;
  const int32_t *perm = nullptr;
  for (int j = ot->num_terms - 1; j >= 0; j--) {
    term_keys_kernel<<<trim_grid(n), 256, 0, s>>>(vals, keys, n, naggs, *ot, j, perm, hll, hll_bytes, m_regs, k0, i0);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int end_bit = ot->kind[j] == TERM_GROUP_KEY ? key_bits(ot->card[ot->a[j]]) : 64;
    size_t tb = sort_bytes;
    e = hipcub::DeviceRadixSort::SortPairs(tmp, tb, k0, k1, i0, i1, (int)n, 0, end_bit, s);
    if (e != hipSuccess) return e;
    perm = i1;  // the next pass reads i1 and writes k0 / i0: no overlap
  }
  *order_out = i1;
  return hipSuccess;
}

hipError_t launch_trim_gather(const int32_t *order, int64_t k, int32_t naggs, int64_t hll_bytes, const int64_t *keys,
                              const double *vals, const int64_t *longs, const uint8_t *hll, int64_t *keys_out,
                              double *vals_out, int64_t *longs_out, uint8_t *hll_out, hipStream_t s) {
  if (k <= 0) return hipSuccess;
  trim_gather_kernel<<<trim_grid(k), 256, 0, s>>>(order, k, naggs, hll_bytes, keys, vals, longs, hll, keys_out,
                                                   vals_out, longs_out, hll_out);
  return hipGetLastError();
}

}  // namespace phip
