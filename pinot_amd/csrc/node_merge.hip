// node_merge.hip -- element-wise merge of two dense partial tables (node plans, node.cpp).
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

}  // namespace phip
