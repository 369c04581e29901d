// limit.hip -- numGroupsLimit on the device.
//
// The reference stops creating groups per SEGMENT once numGroupsLimit keys exist: IntGroupIdMap.getGroupId
// (pinot-core/.../query/aggregation/groupby/DictionaryBasedGroupKeyGenerator.java:1023-1048) returns
// INVALID_ID for a new raw key when size() == groupIdUpperBound (= min(cardinality product, numGroupsLimit),
// :153-174), so a segment keeps the FIRST numGroupsLimit distinct keys in doc order and its later docs of
// other keys are dropped (DoubleGroupByResultHolder ignores INVALID_ID). GroupByOperator.java:116 flags
// numGroupsLimitReached when a segment's group count reaches the limit, and the combine ORs the flags
// (GroupByCombineOperator.java:123-124).
//
// On the GPU this runs only when the query-global group count of the normal pass is >= the limit (no
// segment can hold more distinct keys than the whole query, so below that nothing is dropped):
//   1. the aggregation kernel re-runs in GB_HASH mode over composite keys key * S + segment, recording the
//      first matched doc of every (segment, key) with an atomicMin (aggregate.hip, seg_keys);
//   2. the non-empty slots are compacted and radix-sorted by (segment, first doc): the entry's rank inside
//      its segment is its first-seen order, and ranks >= limit are dropped;
//   3. the kept entries are radix-sorted by key and every run of equal keys (one entry per segment) is
//      combined in segment order into one group: counts and integer sums add, double sums add, MIN/MAX
//      reduce, HLL registers take the max.
#include <hipcub/hipcub.hpp>

#include "dev_common.h"

namespace phip {

static inline int lim_grid(int64_t n) {
  int64_t g = (n + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

// (segment, first doc) sort key of every compacted (segment, key) slot
__global__ void limit_prepare_kernel(const int64_t *__restrict__ slots, int64_t n, const uint64_t *__restrict__ hkeys,
                                     const uint32_t *__restrict__ first_doc, int32_t nseg, uint64_t *__restrict__ sortkey,
                                     int32_t *__restrict__ idx) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t slot = slots[i];
    const uint64_t seg = hkeys[slot] % (uint64_t)nseg;
    sortkey[i] = (seg << 32) | (uint64_t)first_doc[slot];
    idx[i] = (int32_t)i;
  }
}

// Per-segment extent of the (segment, first doc) order, from its run boundaries: first[s] / last[s] = the
// first / last position of segment s (-1 when it has no entry). No atomics -- counting with one counter per
// segment serialises every entry of a query with few segments on one address (113 ms for 10M entries).
__global__ void limit_bounds_kernel(const uint64_t *__restrict__ sk_sorted, int64_t n, int64_t *__restrict__ first,
                                    int64_t *__restrict__ last) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t seg = sk_sorted[j] >> 32;
    if (j == 0 || (sk_sorted[j - 1] >> 32) != seg) first[seg] = j;
    if (j == n - 1 || (sk_sorted[j + 1] >> 32) != seg) last[seg] = j;
  }
}

// Position j of the (segment, first doc) order -> kept iff its rank inside the segment is < limit;
// kept entries carry their key (composite / nseg) and slot, dropped ones sort last.
__global__ void limit_select_kernel(const uint64_t *__restrict__ sk_sorted, const int32_t *__restrict__ idx_sorted,
                                    int64_t n, const int64_t *__restrict__ seg_start, int64_t limit,
                                    const int64_t *__restrict__ slots, const uint64_t *__restrict__ hkeys, int32_t nseg,
                                    uint64_t *__restrict__ key2, int64_t *__restrict__ slot2) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
    const int64_t seg = (int64_t)(sk_sorted[j] >> 32);
    const int64_t rank = j - seg_start[seg];
    const int64_t slot = slots[idx_sorted[j]];
    if (rank < limit) {
      key2[j] = hkeys[slot] / (uint64_t)nseg;
      slot2[j] = slot;
    } else {
      key2[j] = ~0ull;
      slot2[j] = -1;
    }
  }
}

__global__ void limit_heads_kernel(const uint64_t *__restrict__ k, int64_t n, int32_t *__restrict__ head) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x)
    head[j] = (j == 0 || k[j] != k[j - 1]) ? 1 : 0;
}

// One thread per run of equal keys: combine the run's slots in order (segment order, the stable sorts keep
// it) into the compacted group layout of group_gather_kernel.
__global__ void limit_reduce_kernel(const uint64_t *__restrict__ k, const int64_t *__restrict__ slot2, int64_t n,
                                    const int32_t *__restrict__ head, const int32_t *__restrict__ run, int64_t cap,
                                    int32_t naggs, int32_t own_count, const int32_t *__restrict__ kinds,
                                    const uint64_t *__restrict__ table,
                                    const uint32_t *__restrict__ hll, int32_t nhll, int32_t log2m,
                                    int64_t *__restrict__ keys_out, double *__restrict__ out_values,
                                    int64_t *__restrict__ out_longs, uint8_t *__restrict__ out_hll) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
    if (!head[j]) continue;
    const int64_t r = run[j] - 1;
    const uint64_t key = k[j];
    int64_t e = j + 1;
    while (e < n && k[e] == key) e++;
    keys_out[r] = (int64_t)key;
    uint64_t cnt = 0;
    for (int64_t t = j; t < e; t++) cnt += table[slot2[t]];
    for (int a = 0; a < naggs; a++) {
      const int kind = kinds[a];
      uint64_t v = table[(int64_t)(1 + a) * cap + slot2[j]];
      for (int64_t t = j + 1; t < e; t++) {
        const uint64_t w = table[(int64_t)(1 + a) * cap + slot2[t]];
        if (kind == ACC_SUM_F64) v = as_u64(as_f64(v) + as_f64(w));
        else if (kind == ACC_MIN_F64) v = v < w ? v : w;  // ordered images
        else if (kind == ACC_MAX_F64) v = v > w ? v : w;
        else v += w;
      }
      double d = 0.0;
      int64_t l = 0;
      switch (kind) {
        case ACC_COUNT: l = own_count ? (int64_t)v : (int64_t)cnt; d = (double)l; break;
        case ACC_SUM_I64: l = (int64_t)v; d = (double)l; break;
        case ACC_SUM_F64: d = as_f64(v); break;
        case ACC_MIN_F64:
        case ACC_MAX_F64: d = f64_unordered(v); break;
        default: break;
      }
      out_values[r * naggs + a] = d;
      out_longs[r * naggs + a] = l;
    }
    const int m = 1 << log2m;
    for (int h = 0; h < nhll; h++) {
      uint8_t *dst = out_hll + (r * nhll + h) * m;
      for (int i = 0; i < m; i++) {
        uint32_t x = 0;
        for (int64_t t = j; t < e; t++) x = max(x, hll[((int64_t)h * cap + slot2[t]) * m + i]);
        dst[i] = (uint8_t)x;
      }
    }
  }
}

// ---- host-callable pieces (runtime.cpp: group_limit) ---------------------------------------------------
hipError_t launch_limit_prepare(const int64_t *slots, int64_t n, const uint64_t *hkeys, const uint32_t *first_doc,
                                int32_t nseg, uint64_t *sortkey, int32_t *idx, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  limit_prepare_kernel<<<lim_grid(n), 256, 0, s>>>(slots, n, hkeys, first_doc, nseg, sortkey, idx);
  return hipGetLastError();
}

hipError_t launch_limit_bounds(const uint64_t *sk_sorted, int64_t n, int64_t *first, int64_t *last, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  limit_bounds_kernel<<<lim_grid(n), 256, 0, s>>>(sk_sorted, n, first, last);
  return hipGetLastError();
}

// Radix sort of (u64 key, payload) pairs: payload i32 or i64 by `wide`. *temp_bytes on a null temp.
hipError_t launch_sort_pairs(void *temp, size_t *temp_bytes, const uint64_t *k_in, uint64_t *k_out, const void *v_in,
                             void *v_out, bool wide, int64_t n, int end_bit, hipStream_t s) {
  if (wide)
    return hipcub::DeviceRadixSort::SortPairs(temp, *temp_bytes, k_in, k_out, (const int64_t *)v_in, (int64_t *)v_out,
                                              (int)n, 0, end_bit, s);
  return hipcub::DeviceRadixSort::SortPairs(temp, *temp_bytes, k_in, k_out, (const int32_t *)v_in, (int32_t *)v_out,
                                            (int)n, 0, end_bit, s);
}

hipError_t launch_limit_select(const uint64_t *sk_sorted, const int32_t *idx_sorted, int64_t n, const int64_t *seg_start,
                               int64_t limit, const int64_t *slots, const uint64_t *hkeys, int32_t nseg, uint64_t *key2,
                               int64_t *slot2, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  limit_select_kernel<<<lim_grid(n), 256, 0, s>>>(sk_sorted, idx_sorted, n, seg_start, limit, slots, hkeys, nseg, key2,
                                                  slot2);
  return hipGetLastError();
}

// heads + inclusive scan over the first n (kept) entries; *scan_bytes on a null temp
hipError_t launch_limit_runs(void *temp, size_t *scan_bytes, const uint64_t *k, int64_t n, int32_t *head, int32_t *run,
                             hipStream_t s) {
  if (temp == nullptr)
    return hipcub::DeviceScan::InclusiveSum(nullptr, *scan_bytes, (const int32_t *)nullptr, (int32_t *)nullptr,
                                            (int)std::max<int64_t>(n, 1), s);
  if (n <= 0) return hipSuccess;
  limit_heads_kernel<<<lim_grid(n), 256, 0, s>>>(k, n, head);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return hipcub::DeviceScan::InclusiveSum(temp, *scan_bytes, head, run, (int)n, s);
}

hipError_t launch_limit_reduce(const uint64_t *k, const int64_t *slot2, int64_t n, const int32_t *head, const int32_t *run,
                               int64_t cap, int32_t naggs, int32_t own_count, const int32_t *kinds,
                               const uint64_t *table, const uint32_t *hll, int32_t nhll, int32_t log2m,
                               int64_t *keys_out, double *vals, int64_t *longs, uint8_t *hll_out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  limit_reduce_kernel<<<lim_grid(n), 256, 0, s>>>(k, slot2, n, head, run, cap, naggs, own_count, kinds, table, hll,
                                                  nhll, log2m,
                                                  keys_out, vals, longs, hll_out);
  return hipGetLastError();
}

}  // namespace phip
