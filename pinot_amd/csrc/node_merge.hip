// node_merge.hip -- merges of two partial tables (node plans, node.cpp): dense tables element-wise, hash tables by key.
//
// The exchange of a node plan whose parts cannot all join one RCCL communicator (two parts on one device -- the
// PHIP_NODE_SPLIT rehearsal on a one-GPU box -- or no loadable librccl): each non-root part's table is copied to the
// root device (hipMemcpyPeerAsync over xGMI when it lives on another GPU) and folded into the root's table here, row
// by row with the reduce operator of the row's kind -- the same operators the RCCL reduce applies (COUNT / exact SUM:
// int64 add, double SUM: f64 add, MIN / MAX: unsigned min / max of the order-preserving u64 image, HLL registers: max).
// HBM-bound and tiny next to the query (C5: 7 x 25 groups x 3 rows).
#include "node.h"

namespace phip {

struct RowKinds {
  int32_t k[PHIP_PARTIAL_MAX_ROWS];
};

__global__ void partial_merge_rows_kernel(uint64_t *__restrict__ dst, const uint64_t *__restrict__ src, RowKinds kinds,
                                          int rows, int64_t groups) {
  const int64_t n = (int64_t)rows * groups;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / groups);
    const uint64_t a = dst[i], b = src[i];
    uint64_t o = a;
    switch (kinds.k[r]) {
      case PHIP_ROW_COUNT:
      case PHIP_ROW_SUM_I64: o = (uint64_t)((int64_t)a + (int64_t)b); break;
      case PHIP_ROW_SUM_F64: o = (uint64_t)__double_as_longlong(__longlong_as_double((long long)a) +
                                                                 __longlong_as_double((long long)b)); break;
      case PHIP_ROW_MIN: o = a < b ? a : b; break;
      case PHIP_ROW_MAX: o = a > b ? a : b; break;
      default: break;  // PHIP_ROW_HLL: the row is unused
    }
    dst[i] = o;
  }
}

template <typename T>
__global__ void max_kernel(T *__restrict__ dst, const T *__restrict__ src, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = dst[i] > src[i] ? dst[i] : src[i];
}

__global__ void i64_to_f64_kernel(uint64_t *__restrict__ row, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    row[i] = (uint64_t)__double_as_longlong((double)(int64_t)row[i]);
}

// ---- hash tables (GB_HASH parts): the groups of a part's open-addressing table inserted into the root part's --------
// The parts' tables are keyed by the same node-global mixed-radix keys (node_plan_create) but each claimed its slots in
// its own probe order, so slot i of one table is not slot i of another: every occupied source slot is looked up (or
// claimed, CAS empty -> key) in the destination by linear probing, as aggregate.hip's hash_slot does, and its rows are
// combined there. A key occurs once in a source table, so one thread owns each destination slot's rows in a launch and
// combines them with plain loads and stores.
constexpr uint64_t kEmptyKey = ~0ull;  // device.h kHashEmpty

__device__ __forceinline__ uint64_t merge_mix64(uint64_t k) {  // (the probe start; any fixed finaliser would do)
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

__global__ void hash_merge_rows_kernel(uint64_t *__restrict__ dkeys, uint64_t *__restrict__ dtab, int64_t dg,
                                       const uint64_t *__restrict__ skeys, const uint64_t *__restrict__ stab, int64_t sg,
                                       RowKinds kinds, int rows, int64_t *__restrict__ map, uint32_t *overflow) {
  const uint64_t mask = (uint64_t)dg - 1;
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < sg; s += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t key = skeys[s];
    int64_t d = -1;
    if (key != kEmptyKey) {
      uint64_t i = merge_mix64(key) & mask;
      for (uint64_t p = 0; p <= mask; p++, i = (i + 1) & mask) {
        const uint64_t k = dkeys[i];
        if (k == key) { d = (int64_t)i; break; }
        if (k == kEmptyKey) {
          uint64_t expected = kEmptyKey;
          if (__hip_atomic_compare_exchange_strong(&dkeys[i], &expected, key, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT) || expected == key) {
            d = (int64_t)i;
            break;
          }
        }
      }
      if (d < 0) {
        __hip_atomic_fetch_or(overflow, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        for (int r = 0; r < rows; r++) {
          uint64_t *dp = dtab + (int64_t)r * dg + d;
          const uint64_t a = *dp, b = stab[(int64_t)r * sg + s];
          uint64_t o = a;
          switch (kinds.k[r]) {
            case PHIP_ROW_COUNT:
            case PHIP_ROW_SUM_I64: o = (uint64_t)((int64_t)a + (int64_t)b); break;
            case PHIP_ROW_SUM_F64: o = (uint64_t)__double_as_longlong(__longlong_as_double((long long)a) +
                                                                       __longlong_as_double((long long)b)); break;
            case PHIP_ROW_MIN: o = a < b ? a : b; break;
            case PHIP_ROW_MAX: o = a > b ? a : b; break;
            default: break;
          }
          *dp = o;
        }
      }
    }
    map[s] = d;
  }
}

__global__ void hash_merge_hll_kernel(uint32_t *__restrict__ dhll, int64_t dg, const uint32_t *__restrict__ shll,
                                      int64_t sg, int nhll, int log2m, const int64_t *__restrict__ map) {
  const int64_t per = sg << log2m, n = (int64_t)nhll * per, m = (int64_t)1 << log2m;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t h = i / per, rem = i - h * per, s = rem >> log2m;
    const int64_t d = map[s];
    if (d < 0) continue;
    uint32_t *dp = dhll + ((h * dg + d) << log2m) + (rem & (m - 1));
    const uint32_t v = shll[i];
    if (*dp < v) *dp = v;
  }
}

static inline int grid_for(int64_t n) {
  const int64_t b = (n + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 4096 ? 4096 : b));
}

hipError_t launch_partial_merge_rows(uint64_t *dst, const uint64_t *src, const int32_t *kinds, int rows, int64_t groups,
                                     hipStream_t s) {
  RowKinds k{};
  for (int r = 0; r < rows && r < PHIP_PARTIAL_MAX_ROWS; r++) k.k[r] = kinds[r];
  partial_merge_rows_kernel<<<grid_for((int64_t)rows * groups), 256, 0, s>>>(dst, src, k, rows, groups);
  return hipGetLastError();
}

hipError_t launch_max_u32(uint32_t *dst, const uint32_t *src, int64_t n, hipStream_t s) {
  max_kernel<uint32_t><<<grid_for(n), 256, 0, s>>>(dst, src, n);
  return hipGetLastError();
}

hipError_t launch_max_u8(uint8_t *dst, const uint8_t *src, int64_t n, hipStream_t s) {
  max_kernel<uint8_t><<<grid_for(n), 256, 0, s>>>(dst, src, n);
  return hipGetLastError();
}

hipError_t launch_i64_row_to_f64(uint64_t *row, int64_t n, hipStream_t s) {
  i64_to_f64_kernel<<<grid_for(n), 256, 0, s>>>(row, n);
  return hipGetLastError();
}

hipError_t launch_hash_merge(uint64_t *dkeys, uint64_t *dtab, uint32_t *dhll, int64_t dg, const uint64_t *skeys,
                             const uint64_t *stab, const uint32_t *shll, int64_t sg, const int32_t *kinds, int rows,
                             int nhll, int log2m, int64_t *map, uint32_t *overflow, hipStream_t s) {
  if (dg <= 0 || (dg & (dg - 1)) || sg <= 0) return hipErrorInvalidValue;  // (capacities are powers of two)
  RowKinds k{};
  for (int r = 0; r < rows && r < PHIP_PARTIAL_MAX_ROWS; r++) k.k[r] = kinds[r];
  hash_merge_rows_kernel<<<grid_for(sg), 256, 0, s>>>(dkeys, dtab, dg, skeys, stab, sg, k, rows, map, overflow);
  if (nhll > 0) hash_merge_hll_kernel<<<grid_for((int64_t)nhll * (sg << log2m)), 256, 0, s>>>(dhll, dg, shll, sg, nhll, log2m, map);
  return hipGetLastError();
}

}  // namespace phip
