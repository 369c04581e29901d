// aggregate.hip -- projection + aggregation / group-by over the filter kernel's tile masks
// (K5-K9 of SURVEY.md §2.4), and the small reduction / compaction kernels behind them.
//
// Execution model. Waves walk tiles in an XCD-aware order: the global work list is cut into 8
// contiguous ranges, one per XCD (workgroups b and b+8 share an XCD: MI355X_MICROARCH.md §Workgroup
// dispatch; placement is used for speed only, never for correctness), and inside its range an XCD's
// waves stride together, so at any time all of them read the same segment and its dictionaries stay
// in that XCD's 4 MiB L2. Per tile a wave loads the 64 lane-major mask words (256 B), compacts the
// matched docs into a per-wave LDS ring (mbcnt ranks) and, 64 at a time, reads the projected columns
// for exactly those docs (late materialisation, as DataFetcher reads only the block's doc ids,
// pinot-core/.../common/DataFetcher.java:335-386): fixed-bit dict id from HBM, dictionary gather,
// expression (TransformOperator subset: a, a+b, a-b, a*b), then
//   GB_NONE    per-lane accumulators (int64-exact or f64), HLL registers in LDS;
//   GB_LDS     a per-workgroup group table in LDS (DictionaryBasedGroupKeyGenerator's dense key:
//              mixed radix over query-global dict ids, column 0 least significant), written to a
//              per-workgroup slab and reduced in a fixed order by slab_reduce_kernel (bitwise
//              reproducible, no global atomics);
//   GB_GLOBAL  one dense table in HBM updated with global atomics (large key spaces).
#include <hip/hip_ext.h>

#include "agg_common.h"

namespace phip {
// Fixed-order reduction of the per-workgroup group-table slabs into the global layout
// ([1 + naggs][G] u64, row 0 = counts) and of the packed HLL slabs into [nhll][G][m] u32.
__global__ __launch_bounds__(256) void slab_reduce_kernel(const uint64_t *__restrict__ slab, int32_t nslabs,
                                                          int32_t tbl_words, int64_t G, const int32_t *__restrict__ kinds,
                                                          uint64_t *__restrict__ out, const uint32_t *__restrict__ hslab,
                                                          int32_t hll_words, uint32_t *__restrict__ hout) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < tbl_words) {
    const int row = (int)(i / G);
    const int kind = row == 0 ? ACC_COUNT : kinds[row - 1];
    uint64_t v = slab[i];
    for (int b = 1; b < nslabs; b++) {
      const uint64_t w = slab[(size_t)b * tbl_words + i];
      if (kind == ACC_SUM_F64) v = as_u64(as_f64(v) + as_f64(w));
      else if (kind == ACC_MIN_F64) v = v < w ? v : w;
      else if (kind == ACC_MAX_F64) v = v > w ? v : w;
      else v += w;
    }
    out[i] = v;
  }
  if (i < hll_words) {
    uint32_t v = hslab[i];
    for (int b = 1; b < nslabs; b++) {
      const uint32_t w = hslab[(size_t)b * hll_words + i];
      uint32_t r = 0;
#pragma unroll
      for (int k = 0; k < 32; k += 8) r |= max((v >> k) & 0xffu, (w >> k) & 0xffu) << k;
      v = r;
    }
    hout[4 * i + 0] = v & 0xffu;
    hout[4 * i + 1] = (v >> 8) & 0xffu;
    hout[4 * i + 2] = (v >> 16) & 0xffu;
    hout[4 * i + 3] = v >> 24;
  }
}

// The same reduction with one wave per output word, for small tables over many slabs (C1 GROUP_BY_LOW_CARD:
// 40 words x 1K slabs took 200 us as a per-thread loop of dependent loads). Lane l folds slabs l, l+64, ... in
// order, then a fixed butterfly combines the lanes: a fixed order, so the result is bitwise reproducible.
__device__ __forceinline__ uint64_t slab_combine(int kind, uint64_t v, uint64_t w) {
  if (kind == ACC_SUM_F64) return as_u64(as_f64(v) + as_f64(w));
  if (kind == ACC_MIN_F64) return v < w ? v : w;
  if (kind == ACC_MAX_F64) return v > w ? v : w;
  return v + w;
}
__device__ __forceinline__ uint32_t hll_combine(uint32_t v, uint32_t w) {
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 32; k += 8) r |= max((v >> k) & 0xffu, (w >> k) & 0xffu) << k;
  return r;
}
__global__ __launch_bounds__(256) void slab_reduce_wave_kernel(const uint64_t *__restrict__ slab, int32_t nslabs,
                                                               int32_t tbl_words, int64_t G,
                                                               const int32_t *__restrict__ kinds,
                                                               uint64_t *__restrict__ out,
                                                               const uint32_t *__restrict__ hslab, int32_t hll_words,
                                                               uint32_t *__restrict__ hout) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i < tbl_words) {
    const int row = (int)(i / G);
    const int kind = row == 0 ? ACC_COUNT : kinds[row - 1];
    if (lane < nslabs) {
      uint64_t v = slab[(size_t)lane * tbl_words + i];
      for (int b = lane + 64; b < nslabs; b += 64) v = slab_combine(kind, v, slab[(size_t)b * tbl_words + i]);
      for (int off = 1; off < 64; off <<= 1) {
        const uint64_t w = __shfl_xor(v, off);
        const bool has = (lane ^ off) < nslabs;
        v = has ? slab_combine(kind, (lane & off) ? w : v, (lane & off) ? v : w) : v;
      }
      if (lane == 0) out[i] = v;
    } else {
      for (int off = 1; off < 64; off <<= 1) (void)__shfl_xor((uint64_t)0, off);  // keep the wave's shuffles uniform
    }
  }
  if (i < hll_words) {
    if (lane < nslabs) {
      uint32_t v = hslab[(size_t)lane * hll_words + i];
      for (int b = lane + 64; b < nslabs; b += 64) v = hll_combine(v, hslab[(size_t)b * hll_words + i]);
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t w = __shfl_xor(v, off);
        v = (lane ^ off) < nslabs ? hll_combine(v, w) : v;
      }
      if (lane == 0) {
        hout[4 * i + 0] = v & 0xffu;
        hout[4 * i + 1] = (v >> 8) & 0xffu;
        hout[4 * i + 2] = (v >> 16) & 0xffu;
        hout[4 * i + 3] = v >> 24;
      }
    } else {
      for (int off = 1; off < 64; off <<= 1) (void)__shfl_xor(0u, off);
    }
  }
}

// Deterministic reduction of per-block partials -> out[nslots]: one wave per slot, lane-strided over
// blocks in a fixed order, then a fixed shuffle tree (bitwise reproducible run to run).
__device__ __forceinline__ void finalize_slot(const uint64_t *__restrict__ partials, int nblocks, int nslots,
                                              const int32_t *__restrict__ kinds, uint64_t *__restrict__ out, int a);

__global__ void finalize_partials_kernel(const uint64_t *__restrict__ partials, int nblocks, int nslots,
                                         const int32_t *__restrict__ kinds, uint64_t *__restrict__ out) {
  if ((int)blockIdx.x < nslots) finalize_slot(partials, nblocks, nslots, kinds, out, blockIdx.x);
}

// Both partial sets of a filtered aggregation in one launch (blocks [0, na) -> set a, the rest -> set b).
__global__ void finalize_partials2_kernel(const uint64_t *__restrict__ pa, int nba, int na, const int32_t *__restrict__ ka,
                                          uint64_t *__restrict__ oa, const uint64_t *__restrict__ pb, int nbb, int nb,
                                          const int32_t *__restrict__ kb, uint64_t *__restrict__ ob) {
  const int i = blockIdx.x;
  if (i < na) finalize_slot(pa, nba, na, ka, oa, i);
  else if (i < na + nb) finalize_slot(pb, nbb, nb, kb, ob, i - na);
}

// Every per-execution result of an aggregation query in one launch, written straight into the plan's pinned
// host landing area (device-visible host memory; visible to the host once the stream has synchronised):
// blocks [0, na) reduce the aggregation partials -> out[a], blocks [na, na+2) the filter partials (matched
// docs, entries scanned) -> out[32 + i], the last block copies the per-segment matched counts -> out[64 + s]
// and the HLL registers -> (u32) out[64 + nseg ...], zeroing both device arrays for the next execution (so no
// memset launch precedes the query kernels).
__device__ __forceinline__ void finalize_all_body(const uint64_t *__restrict__ pa, int nba, int na,
                                                  const int32_t *__restrict__ ka, const uint64_t *__restrict__ pf,
                                                  int nbf, const int32_t *__restrict__ kf, uint64_t *__restrict__ segm,
                                                  int nseg, uint32_t *__restrict__ hll, int hll_words, uint64_t *out);

// ticket != null: completion published to the host -- every block fences its writes to the mapped result area at
// system scope and takes a ticket; the last one resets the ticket and stores `seq` into out[kDoneSlot] with a
// system-scope release, so a host that polls that word (execute_plan, PHIP_POLL_DONE) may read the results without
// waiting for the kernel's completion signal (the end-of-kernel release and the signal write behind it).
__global__ void finalize_all_kernel(const uint64_t *__restrict__ pa, int nba, int na, const int32_t *__restrict__ ka,
                                    const uint64_t *__restrict__ pf, int nbf, const int32_t *__restrict__ kf,
                                    uint64_t *__restrict__ segm, int nseg, uint32_t *__restrict__ hll, int hll_words,
                                    uint64_t *out, uint32_t *ticket, uint64_t seq) {
  finalize_all_body(pa, nba, na, ka, pf, nbf, kf, segm, nseg, hll, hll_words, out);
  if (ticket == nullptr) return;
  __threadfence_system();  // (every thread's result stores, at system scope, before the block's ticket)
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (t == gridDim.x - 1) {
      __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence_system();
      __hip_atomic_store(out + kDoneSlot, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

__device__ __forceinline__ void finalize_all_body(const uint64_t *__restrict__ pa, int nba, int na,
                                                  const int32_t *__restrict__ ka, const uint64_t *__restrict__ pf,
                                                  int nbf, const int32_t *__restrict__ kf, uint64_t *__restrict__ segm,
                                                  int nseg, uint32_t *__restrict__ hll, int hll_words, uint64_t *out) {
  const int i = blockIdx.x;
  if (i < na) {
    finalize_slot(pa, nba, na, ka, out, i);
  } else if (i < na + 2) {
    if (pf != nullptr) finalize_slot(pf, nbf, 2, kf, out + 32, i - na);
  } else {
    for (int s = threadIdx.x; s < nseg; s += blockDim.x) {
      out[64 + s] = segm[s];
      segm[s] = 0;
    }
    uint32_t *oh = (uint32_t *)(out + 64 + nseg);
    for (int w = threadIdx.x; w < hll_words; w += blockDim.x) {
      oh[w] = hll[w];
      hll[w] = 0;
    }
  }
}

__device__ __forceinline__ void finalize_slot(const uint64_t *__restrict__ partials, int nblocks, int nslots,
                                              const int32_t *__restrict__ kinds, uint64_t *__restrict__ out, int a) {
  const int lane = threadIdx.x;
  const int kind = kinds[a];
  const bool fp = kind == ACC_SUM_F64 || kind == ACC_MIN_F64 || kind == ACC_MAX_F64;
  uint64_t v = fp ? acc_init(kind) : 0;
  for (int b = lane; b < nblocks; b += 64) v = acc_combine(kind, v, partials[(int64_t)b * nslots + a]);
  if (fp) v = as_u64(wave_reduce_f64(as_f64(v), kind));
  else v = wave_reduce_u64_add(v);
  if (lane == 0) out[a] = v;
}

// ------------------------------------------------------------------------------------------------
// group-by table init / compaction
// ------------------------------------------------------------------------------------------------
__global__ void fill_u64_kernel(uint64_t *__restrict__ p, int64_t n, uint64_t v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = v;
}

// GB_XCD (the fused group-by's XCD-private table copies): every copy's rows set to their identity (0; ~0 for a MIN
// row of order-preserving images), and after the launch copies 1.. folded into copy 0 in copy order.
__global__ void xcd_init_kernel(uint64_t *__restrict__ tab, int64_t words, int64_t G, const int32_t *__restrict__ kinds) {
  const int64_t n = words * kXcdCopies;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int row = (int)((i % words) / G);
    tab[i] = (row > 0 && kinds[row - 1] == ACC_MIN_F64) ? ~0ull : 0ull;
  }
}
__global__ void xcd_merge_kernel(uint64_t *__restrict__ tab, int64_t words, int64_t G, const int32_t *__restrict__ kinds,
                                 uint32_t *__restrict__ hll, int64_t hll_words) {
  const int64_t n = words > hll_words ? words : hll_words;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (i < words) {
      const int row = (int)(i / G);
      const int kind = row == 0 ? ACC_COUNT : kinds[row - 1];
      uint64_t v = tab[i];
#pragma unroll
      for (int c = 1; c < kXcdCopies; c++) {
        const uint64_t w = tab[(int64_t)c * words + i];
        if (kind == ACC_SUM_F64) v = as_u64(as_f64(v) + as_f64(w));
        else if (kind == ACC_MIN_F64) v = v < w ? v : w;
        else if (kind == ACC_MAX_F64) v = v > w ? v : w;
        else v += w;
      }
      tab[i] = v;
    }
    if (i < hll_words) {
      uint32_t v = hll[i];
#pragma unroll
      for (int c = 1; c < kXcdCopies; c++) v = max(v, hll[(int64_t)c * hll_words + i]);
      hll[i] = v;
    }
  }
}

// Per 1024-group chunk: number of non-empty groups.
__global__ __launch_bounds__(256) void group_count_kernel(const uint64_t *__restrict__ counts, int64_t n,
                                                          int32_t *__restrict__ chunk_counts) {
  __shared__ int32_t s;
  if (threadIdx.x == 0) s = 0;
  __syncthreads();
  int64_t base = (int64_t)blockIdx.x * 1024;
  int c = 0;
  for (int i = threadIdx.x; i < 1024; i += 256) {
    int64_t gidx = base + i;
    if (gidx < n && counts[gidx] != 0) c++;
  }
  atomicAdd(&s, c);
  __syncthreads();
  if (threadIdx.x == 0) chunk_counts[blockIdx.x] = s;
}

// Single-block exclusive scan of chunk counts; total in offsets[nchunks]. Each of the 1024 threads owns a
// contiguous run of chunks: run sums, a block-wide scan of the 1024 partials in LDS, then each thread writes
// its run. (A one-thread loop here cost 1.8 ms for a 2^25-slot hash table: 32K dependent global round trips.)
constexpr int kScanThreads = 1024;
__global__ __launch_bounds__(kScanThreads) void exclusive_scan_kernel(const int32_t *__restrict__ in, int32_t n,
                                                                      int64_t *__restrict__ offsets) {
  __shared__ int64_t part[kScanThreads];
  const int t = threadIdx.x;
  const int per = (n + kScanThreads - 1) / kScanThreads;
  const int b = min(n, t * per), e = min(n, b + per);
  int64_t s = 0;
  for (int i = b; i < e; i++) s += in[i];
  part[t] = s;
  __syncthreads();
  for (int off = 1; off < kScanThreads; off <<= 1) {  // Hillis-Steele inclusive scan
    const int64_t v = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int64_t run = part[t] - s;  // exclusive prefix of this thread's run
  for (int i = b; i < e; i++) {
    offsets[i] = run;
    run += in[i];
  }
  if (t == kScanThreads - 1) offsets[n] = part[t];
}

// Ordered compaction: writes group indices of non-empty groups, ascending.
__global__ __launch_bounds__(256) void group_compact_kernel(const uint64_t *__restrict__ counts, int64_t n,
                                                            const int64_t *__restrict__ offsets,
                                                            int64_t *__restrict__ out_keys) {
  __shared__ int32_t wave_counts[4];
  const int lane = lane_id(), wave = threadIdx.x >> 6;
  int64_t base = (int64_t)blockIdx.x * 1024;
  int64_t out = offsets[blockIdx.x];
  for (int round = 0; round < 1024 / 256; round++) {
    int64_t gidx = base + round * 256 + threadIdx.x;
    bool nz = gidx < n && counts[gidx] != 0;
    uint64_t b = ballot(nz);
    if (lane == 0) wave_counts[wave] = __popcll(b);
    __syncthreads();
    int32_t before = 0;
    for (int w = 0; w < wave; w++) before += wave_counts[w];
    int32_t total = 0;
    for (int w = 0; w < 4; w++) total += wave_counts[w];
    if (nz) {
      int32_t rank = before + __popcll(b & ((1ull << lane) - 1));
      out_keys[out + rank] = gidx;
    }
    out += total;
    __syncthreads();
  }
}

// Gather the aggregates of the compacted groups. table = [1 + naggs][ndense], row 0 = counts.
__device__ __forceinline__ void gather_group(int64_t i, int64_t key, int64_t ndense, int32_t naggs, int32_t own_count,
                                             const int32_t *__restrict__ kinds, const uint64_t *__restrict__ table,
                                             const uint32_t *__restrict__ hll, int32_t nhll, int32_t log2m,
                                             double *__restrict__ out_values, int64_t *__restrict__ out_longs,
                                             uint8_t *__restrict__ out_hll) {
  {
    for (int a = 0; a < naggs; a++) {
      const int kind = kinds[a];
      const uint64_t v = table[(int64_t)(1 + a) * ndense + key];
      double d = 0.0;
      int64_t l = 0;
      switch (kind) {
        case ACC_COUNT: l = own_count ? (int64_t)v : (int64_t)table[key]; d = (double)l; break;
        case ACC_SUM_I64: l = (int64_t)v; d = (double)l; break;
        case ACC_SUM_F64: d = __longlong_as_double((long long)v); break;
        case ACC_MIN_F64:
        case ACC_MAX_F64: d = f64_unordered(v); break;
        default: break;
      }
      out_values[i * naggs + a] = d;
      out_longs[i * naggs + a] = l;
    }
    const int m = 1 << log2m;
    for (int h = 0; h < nhll; h++) {
      const uint32_t *src = hll + ((int64_t)h * ndense + key) * m;
      uint8_t *dst = out_hll + (i * nhll + h) * m;
      for (int j = 0; j < m; j++) dst[j] = (uint8_t)src[j];
    }
  }
}

__global__ void group_gather_kernel(const int64_t *__restrict__ keys, int64_t ngroups, int64_t ndense,
                                    int32_t naggs, int32_t own_count, const int32_t *__restrict__ kinds,
                                    const uint64_t *__restrict__ table, const uint32_t *__restrict__ hll, int32_t nhll,
                                    int32_t log2m, double *__restrict__ out_values, int64_t *__restrict__ out_longs,
                                    uint8_t *__restrict__ out_hll) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ngroups; i += (int64_t)gridDim.x * blockDim.x)
    gather_group(i, keys[i], ndense, naggs, own_count, kinds, table, hll, nhll, log2m, out_values, out_longs, out_hll);
}

// The one-round-trip variant (runtime.cpp, group-by results without a host read of the group count): the count is
// the scan's total on the device (`d_ngroups`, offsets[nchunks]), the grid covers the key space, and the count, the
// keys, values and exact sums land in mapped host memory (vector stores), read by the host after its one wait.
__global__ void group_gather_mapped_kernel(const int64_t *__restrict__ keys, const int64_t *__restrict__ d_ngroups,
                                           int64_t ndense, int32_t naggs, int32_t own_count,
                                           const int32_t *__restrict__ kinds, const uint64_t *__restrict__ table,
                                           int64_t *__restrict__ out_count, int64_t *__restrict__ out_keys,
                                           double *__restrict__ out_values, int64_t *__restrict__ out_longs,
                                           const uint32_t *__restrict__ hll, int32_t nhll, int32_t log2m,
                                           uint32_t *__restrict__ out_hll) {
  const int64_t ngroups = min(*d_ngroups, ndense);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x, t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t0 == 0) out_count[0] = ngroups;
  for (int64_t i = t0; i < ngroups; i += stride) {
    const int64_t key = keys[i];
    out_keys[i] = key;
    gather_group(i, key, ndense, naggs, own_count, kinds, table, nullptr, 0, 0, out_values, out_longs, nullptr);
  }
  // HLL registers (u32 per register in the table, < 64): four packed per 4-B store, one 16-B load each, so the
  // registers cross to host memory a word, not a byte, at a time
  const int64_t q = (int64_t)nhll << (log2m - 2);  // packed words per group
  for (int64_t w = t0; w < ngroups * q; w += stride) {
    const int64_t i = w / q, r = w - i * q;
    const int64_t h = r >> (log2m - 2), j = (r & ((1 << (log2m - 2)) - 1)) << 2;
    const uint4 v = *(const uint4 *)(hll + ((h * ndense + keys[i]) << log2m) + j);
    out_hll[w] = (v.x & 0xFFu) | ((v.y & 0xFFu) << 8) | ((v.z & 0xFFu) << 16) | ((v.w & 0xFFu) << 24);
  }
}

// GB_HASH: compacted slot indices -> the mixed-radix keys they hold (after group_gather_kernel used
// the slots).
__global__ void hash_keys_kernel(int64_t *__restrict__ slots, int64_t n, const uint64_t *__restrict__ keys) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    slots[i] = (int64_t)keys[slots[i]];
}

// ------------------------------------------------------------------------------------------------
// host-callable launchers (runtime.cpp)
// ------------------------------------------------------------------------------------------------
static inline int grid_for(int64_t n, int per_block = 256, int cap = 4096) {
  int64_t g = (n + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

// the agg_kernel variants, instantiated in agg_k_*.hip (one translation unit per group)
template <int NA, int MODE, bool D = false, int W = kAggWaves, bool R = false, bool H = false>
hipError_t launch_agg_t(const DevAggQuery *q, int nblocks, size_t lds, hipStream_t s, hipEvent_t e0, hipEvent_t e1);

// q: host copy (for the variant choice); dq: the same descriptor in device memory.
hipError_t launch_agg(const DevAggQuery &q, const DevAggQuery *dq, int nblocks, size_t lds, hipStream_t s, hipEvent_t e0,
                      hipEvent_t e1) {
  if (q.mode == GB_LDS && q.rec_on) {  // (group-by records: the variants that read them)
    if (q.wg_waves == 16)
      return q.dense_batch ? launch_agg_t<1, GB_LDS, true, 16, true>(dq, nblocks, lds, s, e0, e1)
                           : launch_agg_t<1, GB_LDS, false, 16, true>(dq, nblocks, lds, s, e0, e1);
    return q.dense_batch ? launch_agg_t<1, GB_LDS, true, kAggWaves, true>(dq, nblocks, lds, s, e0, e1)
                         : launch_agg_t<1, GB_LDS, false, kAggWaves, true>(dq, nblocks, lds, s, e0, e1);
  }
  if (q.mode == GB_LDS && q.wg_waves == 16)
    return q.dense_batch ? launch_agg_t<1, GB_LDS, true, 16>(dq, nblocks, lds, s, e0, e1)
                         : launch_agg_t<1, GB_LDS, false, 16>(dq, nblocks, lds, s, e0, e1);
  if (q.mode == GB_LDS)
    return q.dense_batch ? launch_agg_t<1, GB_LDS, true>(dq, nblocks, lds, s, e0, e1) : launch_agg_t<1, GB_LDS>(dq, nblocks, lds, s, e0, e1);
  if (q.mode == GB_GLOBAL)
    return q.dense_batch ? launch_agg_t<1, GB_GLOBAL, true>(dq, nblocks, lds, s, e0, e1)
                         : launch_agg_t<1, GB_GLOBAL>(dq, nblocks, lds, s, e0, e1);
  if (q.mode == GB_HASH) return launch_agg_t<1, GB_HASH>(dq, nblocks, lds, s, e0, e1);
  if (q.dense_batch && q.hist_aggs) {  // (the id-histogram variants: one or two aggregations)
    if (q.num_aggs <= 1) return launch_agg_t<1, GB_NONE, true, kAggWaves, false, true>(dq, nblocks, lds, s, e0, e1);
    return launch_agg_t<2, GB_NONE, true, kAggWaves, false, true>(dq, nblocks, lds, s, e0, e1);
  }
  if (q.dense_batch) {
    if (q.num_aggs <= 1) return launch_agg_t<1, GB_NONE, true>(dq, nblocks, lds, s, e0, e1);
    if (q.num_aggs <= 2) return launch_agg_t<2, GB_NONE, true>(dq, nblocks, lds, s, e0, e1);
    if (q.num_aggs <= 4) return launch_agg_t<4, GB_NONE, true>(dq, nblocks, lds, s, e0, e1);
    return launch_agg_t<8, GB_NONE, true>(dq, nblocks, lds, s, e0, e1);
  }
  if (q.num_aggs <= 1) return launch_agg_t<1, GB_NONE>(dq, nblocks, lds, s, e0, e1);
  if (q.num_aggs <= 2) return launch_agg_t<2, GB_NONE>(dq, nblocks, lds, s, e0, e1);
  if (q.num_aggs <= 4) return launch_agg_t<4, GB_NONE>(dq, nblocks, lds, s, e0, e1);
  return launch_agg_t<8, GB_NONE>(dq, nblocks, lds, s, e0, e1);
}

hipError_t launch_slab_reduce(const uint64_t *slab, int32_t nslabs, int32_t tbl_words, int64_t G, const int32_t *kinds,
                              uint64_t *out, const uint32_t *hslab, int32_t hll_words, uint32_t *hout, hipStream_t s) {
  const int64_t n = std::max<int64_t>(tbl_words, hll_words);
  if (n <= 16384 && nslabs > 64) {  // few words, many slabs: a wave per word
    slab_reduce_wave_kernel<<<(unsigned)((n + 3) / 4), 256, 0, s>>>(slab, nslabs, tbl_words, G, kinds, out, hslab,
                                                                    hll_words, hout);
    return hipGetLastError();
  }
  slab_reduce_kernel<<<grid_for(n, 256, 1 << 20), 256, 0, s>>>(slab, nslabs, tbl_words, G, kinds, out, hslab, hll_words,
                                                               hout);
  return hipGetLastError();
}

hipError_t launch_finalize_partials(const uint64_t *partials, int nblocks, int nslots, const int32_t *kinds,
                                    uint64_t *out, hipStream_t s) {
  finalize_partials_kernel<<<nslots, 64, 0, s>>>(partials, nblocks, nslots, kinds, out);
  return hipGetLastError();
}
hipError_t launch_finalize_partials2(const uint64_t *pa, int nba, int na, const int32_t *ka, uint64_t *oa,
                                     const uint64_t *pb, int nbb, int nb, const int32_t *kb, uint64_t *ob, hipStream_t s) {
  finalize_partials2_kernel<<<na + nb, 64, 0, s>>>(pa, nba, na, ka, oa, pb, nbb, nb, kb, ob);
  return hipGetLastError();
}
hipError_t launch_finalize_all(const uint64_t *pa, int nba, int na, const int32_t *ka, const uint64_t *pf, int nbf,
                               const int32_t *kf, uint64_t *segm, int nseg, uint32_t *hll, int hll_words, uint64_t *out,
                               hipStream_t s, uint32_t *ticket, uint64_t seq) {
  finalize_all_kernel<<<na + 3, 64, 0, s>>>(pa, nba, na, ka, pf, nbf, kf, segm, nseg, hll, hll_words, out, ticket, seq);
  return hipGetLastError();
}
hipError_t launch_xcd_init(uint64_t *tab, int64_t words, int64_t G, const int32_t *kinds, hipStream_t s) {
  if (words <= 0) return hipSuccess;
  xcd_init_kernel<<<grid_for(words * kXcdCopies), 256, 0, s>>>(tab, words, G, kinds);
  return hipGetLastError();
}
hipError_t launch_xcd_merge(uint64_t *tab, int64_t words, int64_t G, const int32_t *kinds, uint32_t *hll,
                            int64_t hll_words, hipStream_t s) {
  const int64_t n = std::max(words, hll_words);
  if (n <= 0) return hipSuccess;
  xcd_merge_kernel<<<grid_for(n), 256, 0, s>>>(tab, words, G, kinds, hll, hll_words);
  return hipGetLastError();
}
hipError_t launch_fill_u64(uint64_t *p, int64_t n, uint64_t v, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  fill_u64_kernel<<<grid_for(n), 256, 0, s>>>(p, n, v);
  return hipGetLastError();
}
hipError_t launch_group_count(const uint64_t *counts, int64_t n, int32_t *chunk_counts, int64_t nchunks,
                              int64_t *offsets, hipStream_t s) {
  group_count_kernel<<<(unsigned)nchunks, 256, 0, s>>>(counts, n, chunk_counts);
  exclusive_scan_kernel<<<1, kScanThreads, 0, s>>>(chunk_counts, (int32_t)nchunks, offsets);
  return hipGetLastError();
}
hipError_t launch_group_compact(const uint64_t *counts, int64_t n, const int64_t *offsets, int64_t nchunks,
                                int64_t *keys, hipStream_t s) {
  group_compact_kernel<<<(unsigned)nchunks, 256, 0, s>>>(counts, n, offsets, keys);
  return hipGetLastError();
}
hipError_t launch_group_gather(const int64_t *keys, int64_t ngroups, int64_t ndense, int32_t naggs, int32_t own_count,
                               const int32_t *kinds, const uint64_t *table, const uint32_t *hll, int32_t nhll,
                               int32_t log2m, double *vals, int64_t *longs, uint8_t *hll_out, hipStream_t s) {
  if (ngroups <= 0) return hipSuccess;
  group_gather_kernel<<<grid_for(ngroups), 256, 0, s>>>(keys, ngroups, ndense, naggs, own_count, kinds, table, hll, nhll,
                                                       log2m, vals, longs, hll_out);
  return hipGetLastError();
}

hipError_t launch_group_gather_mapped(const int64_t *keys, const int64_t *d_ngroups, int64_t ndense, int32_t naggs,
                                      int32_t own_count, const int32_t *kinds, const uint64_t *table,
                                      int64_t *out_count, int64_t *out_keys, double *vals, int64_t *longs,
                                      const uint32_t *hll, int32_t nhll, int32_t log2m, uint32_t *hll_out,
                                      hipStream_t s) {
  if (ndense <= 0 || (nhll > 0 && (log2m < 4 || log2m > 16))) return hipErrorInvalidValue;
  const int64_t work = std::max<int64_t>(ndense, nhll > 0 ? ndense * ((int64_t)nhll << (log2m - 2)) : 0);
  group_gather_mapped_kernel<<<grid_for(work), 256, 0, s>>>(keys, d_ngroups, ndense, naggs, own_count, kinds, table,
                                                            out_count, out_keys, vals, longs, hll, nhll, log2m,
                                                            hll_out);
  return hipGetLastError();
}

hipError_t launch_hash_keys(int64_t *slots, int64_t n, const uint64_t *keys, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hash_keys_kernel<<<grid_for(n), 256, 0, s>>>(slots, n, keys);
  return hipGetLastError();
}

}  // namespace phip
