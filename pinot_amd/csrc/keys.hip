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

// Raw STRING keys: the same scheme over a 64-bit hash of each doc's UTF-8 bytes (FNV-1a with a final avalanche).
// Per segment the (hash, doc) pairs are sorted and made unique by hash, keeping a representative doc per hash; every
// doc's bytes are compared with its representative's (a hash collision inside a segment sets *collided), the host
// compares representatives across segments, sorts the distinct strings bytewise (the STRING dictionaries' order) and
// hands back a segment-hash-index -> global-id map for raw_str_ids_kernel.
// (a test hook narrows the hash -- PHIP_STR_HASH_BITS, set_str_hash_bits -- so collisions occur and the exact host path
// that resolves them is exercised; all 64 bits otherwise)
__device__ uint64_t g_str_hash_mask = ~0ull;

__device__ __forceinline__ uint64_t str_hash64(const uint8_t *p, int64_t len) {
  uint64_t h = 0xcbf29ce484222325ull ^ (uint64_t)len;
  for (int64_t i = 0; i < len; i++) h = (h ^ p[i]) * 0x100000001b3ull;
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ull;
  return (h ^ (h >> 33)) & g_str_hash_mask;
}

hipError_t set_str_hash_bits(int bits) {
  const uint64_t m = bits >= 64 || bits <= 0 ? ~0ull : ((1ull << bits) - 1ull);
  return hipMemcpyToSymbol(HIP_SYMBOL(g_str_hash_mask), &m, sizeof(m));
}

__global__ void str_hash_kernel(const uint8_t *__restrict__ bytes, const uint64_t *__restrict__ off, int64_t n,
                                uint64_t *__restrict__ hash, int32_t *__restrict__ docs) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    hash[i] = str_hash64(bytes + off[i], (int64_t)(off[i + 1] - off[i]));
    docs[i] = (int32_t)i;
  }
}

__device__ __forceinline__ int64_t lower_bound_u64(const uint64_t *a, int64_t u, uint64_t k) {
  int64_t lo = 0, hi = u;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] < k) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__global__ void str_verify_kernel(const uint8_t *__restrict__ bytes, const uint64_t *__restrict__ off, int64_t n,
                                  const uint64_t *__restrict__ uniq, const int32_t *__restrict__ rep, int64_t u,
                                  int32_t *__restrict__ collided) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t len = (int64_t)(off[i + 1] - off[i]);
    const int64_t r = rep[lower_bound_u64(uniq, u, str_hash64(bytes + off[i], len))];
    bool same = (int64_t)(off[r + 1] - off[r]) == len;
    for (int64_t b = 0; same && b < len; b++) same = bytes[off[i] + b] == bytes[off[r] + b];
    if (!same) *collided = 1;  // (vector store; any colliding doc's lane may write it)
  }
}

// the representatives' lengths, then (dst offsets from the host) their bytes back to back
__global__ void str_rep_lens_kernel(const uint64_t *__restrict__ off, const int32_t *__restrict__ rep, int64_t u,
                                    uint32_t *__restrict__ lens) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < u; j += (int64_t)gridDim.x * blockDim.x)
    lens[j] = (uint32_t)(off[rep[j] + 1] - off[rep[j]]);
}
__global__ void str_rep_bytes_kernel(const uint8_t *__restrict__ bytes, const uint64_t *__restrict__ off,
                                     const int32_t *__restrict__ rep, int64_t u, const uint64_t *__restrict__ dst_off,
                                     uint8_t *__restrict__ dst) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < u; j += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t s = off[rep[j]], len = off[rep[j] + 1] - s;
    for (uint64_t b = 0; b < len; b++) dst[dst_off[j] + b] = bytes[s + b];
  }
}

__global__ void raw_str_ids_kernel(const uint8_t *__restrict__ bytes, const uint64_t *__restrict__ off, int64_t n,
                                   const uint64_t *__restrict__ uniq, int64_t u, const int32_t *__restrict__ map,
                                   int32_t *__restrict__ ids) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    ids[i] = map[lower_bound_u64(uniq, u, str_hash64(bytes + off[i], (int64_t)(off[i + 1] - off[i])))];
}

// Group-by key spaces above 2^62 (the reference's LongMapBasedHolder / ArrayMapBasedHolder role,
// DictionaryBasedGroupKeyGenerator.java:150-185): each doc's tuple of query-global key ids is packed into W <= 4 u64
// words (mixed radix per word, the columns split so no word's radix product leaves u64), the segment's tuples are
// ranked (LSD: a stable radix sort of the permutation per word, last word first), and the distinct tuples of all
// segments ranked the same way become one virtual key column of doc-order ids (DevCol.gb_ids).
__global__ void tuple_words_kernel(TupleCols tc, int64_t n, uint64_t *__restrict__ out) {
  for (int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; d < n; d += (int64_t)gridDim.x * blockDim.x) {
    uint64_t w[kMaxTupleWords] = {0, 0, 0, 0};
    for (int k = 0; k < tc.k; k++) {
      const TupleCol &c = tc.cols[k];
      int64_t gid;
      if (c.ids != nullptr) {
        gid = c.ids[d];
      } else if (c.words == nullptr) {  // raw INT / LONG: value - base
        gid = (c.type == PHIP_TYPE_LONG ? ((const int64_t *)c.raw)[d] : (int64_t)((const int32_t *)c.raw)[d]) - c.base;
      } else {
        const uint32_t id = decode_bits(c.words, (uint64_t)d * (uint32_t)c.bits, (uint32_t)c.bits);
        gid = c.remap ? c.remap[id] : (int64_t)id;
      }
      if (c.nulls != nullptr && ((c.nulls[d >> 6] >> (d & 63)) & 1ull)) gid = c.null_id;
#pragma unroll
      for (int j = 0; j < kMaxTupleWords; j++)
        if (j == c.word) w[j] += (uint64_t)gid * c.stride;
    }
    for (int j = 0; j < tc.w; j++) out[j * n + d] = w[j];
  }
}

__global__ void iota_kernel(int32_t *__restrict__ p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = (int32_t)i;
}
__global__ void gather_word_kernel(const uint64_t *__restrict__ w, const int32_t *__restrict__ perm, int64_t n,
                                   uint64_t *__restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = w[perm[i]];
}
__global__ void tuple_heads_kernel(const uint64_t *__restrict__ words, int32_t nw, const int32_t *__restrict__ perm,
                                   int64_t n, int32_t *__restrict__ head) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int32_t h = i == 0;
    for (int j = 0; j < nw && !h; j++) h = words[j * n + perm[i]] != words[j * n + perm[i - 1]];
    head[i] = h;
  }
}
__global__ void tuple_scatter_kernel(const uint64_t *__restrict__ words, int32_t nw, const int32_t *__restrict__ perm,
                                     const int32_t *__restrict__ head, const int32_t *__restrict__ rank1, int64_t n,
                                     int32_t *__restrict__ ids, uint64_t *__restrict__ uniq, int64_t ucap) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t r = rank1[i] - 1;
    ids[perm[i]] = r;
    if (head[i])
      for (int j = 0; j < nw; j++) uniq[j * ucap + r] = words[j * n + perm[i]];
  }
}
__global__ void gather_ids_kernel(const int32_t *__restrict__ local, const int32_t *__restrict__ map, int64_t n,
                                  int32_t *__restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = map[local[i]];
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

// (pairs sorted by hash, unique by hash with the first doc of each run; temp == nullptr: the scratch bytes)
hipError_t launch_str_hash_unique(void *temp, size_t *temp_bytes, const uint8_t *bytes, const uint64_t *off, int64_t n,
                                  uint64_t *hash, int32_t *docs, uint64_t *hash_sorted, int32_t *docs_sorted,
                                  uint64_t *uniq, int32_t *rep, int64_t *num_out, hipStream_t s) {
  size_t a = 0, b = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, a, (const uint64_t *)hash, hash_sorted, (const int32_t *)docs,
                                                    docs_sorted, (int)n, 0, 64, s);
  if (e != hipSuccess) return e;
  e = hipcub::DeviceSelect::UniqueByKey(nullptr, b, (const uint64_t *)hash_sorted, (const int32_t *)docs_sorted, uniq, rep,
                                        num_out, (int)n, s);
  if (e != hipSuccess) return e;
  if (temp == nullptr) {
    *temp_bytes = a > b ? a : b;
    return hipSuccess;
  }
  if (n <= 0) return hipMemsetAsync(num_out, 0, 8, s);
  str_hash_kernel<<<keys_grid(n), 256, 0, s>>>(bytes, off, n, hash, docs);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  e = hipcub::DeviceRadixSort::SortPairs(temp, a, (const uint64_t *)hash, hash_sorted, (const int32_t *)docs, docs_sorted,
                                         (int)n, 0, 64, s);
  if (e != hipSuccess) return e;
  return hipcub::DeviceSelect::UniqueByKey(temp, b, (const uint64_t *)hash_sorted, (const int32_t *)docs_sorted, uniq, rep,
                                           num_out, (int)n, s);
}

hipError_t launch_str_verify(const uint8_t *bytes, const uint64_t *off, int64_t n, const uint64_t *uniq, const int32_t *rep,
                             int64_t u, int32_t *collided, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  str_verify_kernel<<<keys_grid(n), 256, 0, s>>>(bytes, off, n, uniq, rep, u, collided);
  return hipGetLastError();
}

hipError_t launch_str_rep_lens(const uint64_t *off, const int32_t *rep, int64_t u, uint32_t *lens, hipStream_t s) {
  if (u <= 0) return hipSuccess;
  str_rep_lens_kernel<<<keys_grid(u), 256, 0, s>>>(off, rep, u, lens);
  return hipGetLastError();
}

hipError_t launch_str_rep_bytes(const uint8_t *bytes, const uint64_t *off, const int32_t *rep, int64_t u,
                                const uint64_t *dst_off, uint8_t *dst, hipStream_t s) {
  if (u <= 0) return hipSuccess;
  str_rep_bytes_kernel<<<keys_grid(u), 256, 0, s>>>(bytes, off, rep, u, dst_off, dst);
  return hipGetLastError();
}

hipError_t launch_raw_str_ids(const uint8_t *bytes, const uint64_t *off, int64_t n, const uint64_t *uniq, int64_t u,
                              const int32_t *map, int32_t *ids, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  raw_str_ids_kernel<<<keys_grid(n), 256, 0, s>>>(bytes, off, n, uniq, u, map, ids);
  return hipGetLastError();
}

hipError_t launch_tuple_words(const TupleCols &tc, int64_t n, uint64_t *out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  tuple_words_kernel<<<keys_grid(n), 256, 0, s>>>(tc, n, out);
  return hipGetLastError();
}

// Rank the n tuples of words (nw x n, word-major): ids[i] = rank of tuple i among the distinct tuples (ordered by word
// 0, then 1, ...), uniq (nw x ucap) = the distinct tuples, *num_out = their count. temp == nullptr: scratch bytes.
hipError_t launch_tuple_rank(void *temp, size_t *temp_bytes, const uint64_t *words, int32_t nw, int64_t n, int32_t *ids,
                             uint64_t *uniq, int64_t ucap, int64_t *num_out, hipStream_t s) {
  // scratch: key, key_sorted (8n each), perm, perm_sorted, head, rank1 (4n each), then the library's temp
  const size_t fixed = (size_t)n * 32 + 256;
  size_t a = 0, b = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, a, (const uint64_t *)nullptr, (uint64_t *)nullptr,
                                                    (const int32_t *)nullptr, (int32_t *)nullptr, (int)n, 0, 64, s);
  if (e != hipSuccess) return e;
  e = hipcub::DeviceScan::InclusiveSum(nullptr, b, (const int32_t *)nullptr, (int32_t *)nullptr, (int)n, s);
  if (e != hipSuccess) return e;
  if (temp == nullptr) {
    *temp_bytes = fixed + (a > b ? a : b);
    return hipSuccess;
  }
  *num_out = 0;
  if (n <= 0) return hipSuccess;
  uint8_t *t = (uint8_t *)temp;
  uint64_t *key = (uint64_t *)t, *key2 = key + n;
  int32_t *perm = (int32_t *)(key2 + n), *perm2 = perm + n, *head = perm2 + n, *rank1 = head + n;
  void *lib = (void *)(((uintptr_t)(rank1 + n) + 255) & ~(uintptr_t)255);
  const int g = keys_grid(n);
  iota_kernel<<<g, 256, 0, s>>>(perm, n);
  for (int j = nw - 1; j >= 0; j--) {
    gather_word_kernel<<<g, 256, 0, s>>>(words + (int64_t)j * n, perm, n, key);
    e = hipcub::DeviceRadixSort::SortPairs(lib, a, (const uint64_t *)key, key2, (const int32_t *)perm, perm2, (int)n, 0, 64, s);
    if (e != hipSuccess) return e;
    int32_t *x = perm;
    perm = perm2;
    perm2 = x;
  }
  tuple_heads_kernel<<<g, 256, 0, s>>>(words, nw, perm, n, head);
  e = hipcub::DeviceScan::InclusiveSum(lib, b, (const int32_t *)head, rank1, (int)n, s);
  if (e != hipSuccess) return e;
  tuple_scatter_kernel<<<g, 256, 0, s>>>(words, nw, perm, head, rank1, n, ids, uniq, ucap);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  int32_t u = 0;
  e = hipMemcpyAsync(&u, rank1 + n - 1, 4, hipMemcpyDeviceToHost, s);
  if (e != hipSuccess) return e;
  e = hipStreamSynchronize(s);
  *num_out = u;
  return e;
}

hipError_t launch_gather_ids(const int32_t *local, const int32_t *map, int64_t n, int32_t *out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  gather_ids_kernel<<<keys_grid(n), 256, 0, s>>>(local, map, n, out);
  return hipGetLastError();
}

}  // namespace phip
