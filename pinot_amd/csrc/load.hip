// load.hip -- one-time layout transforms at segment load (phip_segment_load, runtime.cpp).
#include "dev_common.h"

namespace phip {

// Big-endian index bytes (PinotDataBuffer BIG_ENDIAN, SingleFileIndexDirectory.java:295-297) -> the
// kernels' word layouts: fixed-bit streams as u32 words read big-endian, dictionaries as LE values.
__global__ void bswap32_kernel(uint32_t *__restrict__ p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = __builtin_bswap32(p[i]);
}
__global__ void bswap64_kernel(uint64_t *__restrict__ p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = __builtin_bswap64(p[i]);
}

// Sorted forward index (BE (start,end) pairs, SortedIndexReaderImpl.java:114-116) -> per-doc dict ids.
__global__ void sorted_ids_kernel(const uint32_t *__restrict__ be_pairs, int32_t card, int32_t *__restrict__ ids) {
  for (int d = blockIdx.x; d < card; d += gridDim.x) {
    int32_t s = (int32_t)__builtin_bswap32(be_pairs[2 * d]);
    int32_t e = (int32_t)__builtin_bswap32(be_pairs[2 * d + 1]);
    for (int32_t i = s + threadIdx.x; i <= e; i += blockDim.x) ids[i] = d;
  }
}

// Pack dict ids into the u32-word fixed-bit layout (word k = stream bits [32k, 32k+32)).
__global__ void pack_ids_kernel(const int32_t *__restrict__ ids, int64_t n, int32_t bits, uint32_t *__restrict__ words,
                                int64_t nwords) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nwords; k += (int64_t)gridDim.x * blockDim.x) {
    uint64_t b0 = (uint64_t)k * 32, b1 = b0 + 32;
    int64_t d0 = (int64_t)(b0 / bits), d1 = (int64_t)((b1 + bits - 1) / bits);
    uint32_t w = 0;
    for (int64_t d = d0; d < d1 && d < n; d++) {
      int64_t vs = d * bits;  // value bits occupy [vs, vs + bits); bit 31 of the word is stream bit b0
      uint64_t v = (uint32_t)ids[d];
      int64_t shift = 32 - (vs - (int64_t)b0) - bits;
      if (shift >= 0) w |= (uint32_t)(v << shift);
      else w |= (uint32_t)(v >> (-shift));
    }
    words[k] = w;
  }
}

static inline int grid_for(int64_t n, int per_block = 256, int cap = 4096) {
  int64_t g = (n + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

hipError_t launch_bswap32(uint32_t *p, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  bswap32_kernel<<<grid_for(n), 256, 0, s>>>(p, n);
  return hipGetLastError();
}
hipError_t launch_bswap64(uint64_t *p, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  bswap64_kernel<<<grid_for(n), 256, 0, s>>>(p, n);
  return hipGetLastError();
}
hipError_t launch_sorted_to_packed(const uint32_t *be_pairs, int32_t card, int32_t *ids_tmp, int64_t n, int32_t bits,
                                   uint32_t *words, int64_t nwords, hipStream_t s) {
  sorted_ids_kernel<<<grid_for(card, 1, 4096), 256, 0, s>>>(be_pairs, card, ids_tmp);
  pack_ids_kernel<<<grid_for(nwords), 256, 0, s>>>(ids_tmp, n, bits, words, nwords);
  return hipGetLastError();
}

}  // namespace phip
