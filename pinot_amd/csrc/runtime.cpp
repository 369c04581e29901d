// runtime.cpp -- host runtime of libpinot_hip.so: devices, HBM-resident segments, query executor,
// and the C ABI declared in include/pinot_hip.h.
//
// Segment load (ImmutableSegmentLoader.load, pinot-segment-local/.../immutable/
// ImmutableSegmentLoader.java:155-190,222-280) pins, per column, the forward index, the dictionary
// and the inverted index in HBM in the layouts the kernels read (kernels.hip header). A query
// (InstancePlanMakerImplV2.makeInstancePlan, pinot-core/.../plan/maker/InstancePlanMakerImplV2.java:172-199)
// runs as: Roaring decode of inverted leaves -> one fused filter/aggregate (or group-by) launch over
// all segments -> deterministic finalize -> one D2H copy; it replaces the per-segment operators and
// the CombineOperator thread fan-out (BaseCombineOperator.java:98-143).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/pinot_hip.h"
#include "device.h"
#include "node.h"

namespace phip {
hipError_t launch_bswap32(uint32_t *p, int64_t n, hipStream_t s);
hipError_t launch_bswap64(uint64_t *p, int64_t n, hipStream_t s);
hipError_t launch_trim_order(const double *vals, const int64_t *keys, const KeyOrder *ko, int64_t n, int32_t naggs,
                             int32_t agg, int32_t desc, void *scratch, size_t *scratch_bytes, const int32_t **order_out,
                             hipStream_t s);
hipError_t launch_trim_order_terms(const double *vals, const int64_t *keys, const OrderTerms *ot, int64_t n,
                                   int32_t naggs, const uint8_t *hll, int64_t hll_bytes, int32_t m_regs, void *scratch,
                                   size_t *scratch_bytes, const int32_t **order_out, hipStream_t s);
hipError_t launch_trim_gather(const int32_t *order, int64_t k, int32_t naggs, int64_t hll_bytes, const int64_t *keys,
                              const double *vals, const int64_t *longs, const uint8_t *hll, int64_t *keys_out,
                              double *vals_out, int64_t *longs_out, uint8_t *hll_out, hipStream_t s);
hipError_t launch_chunk_decode(int codec, int entry, const uint8_t *blob, const RawChunk *chunks, int32_t nchunks,
                               int32_t out_cap, int32_t in_cap, size_t lds, uint8_t *out, int32_t *err, int32_t *sizes,
                               hipStream_t s);
size_t chunk_decode_extra_lds(int codec, int32_t out_cap);
hipError_t launch_sorted_to_packed(const uint32_t *be_pairs, int32_t card, int32_t *ids_tmp, int64_t n, int32_t bits,
                                   uint32_t *words, int64_t nwords, hipStream_t s);
hipError_t launch_fill_u64(uint64_t *p, int64_t n, uint64_t v, hipStream_t s);
hipError_t launch_xcd_init(uint64_t *tab, int64_t words, int64_t G, const int32_t *kinds, hipStream_t s);
hipError_t launch_xcd_merge(uint64_t *tab, int64_t words, int64_t G, const int32_t *kinds, uint32_t *hll,
                            int64_t hll_words, hipStream_t s);
hipError_t launch_roaring_or(const RoaringTask *tasks, const RoaringGroup *groups, int32_t ngroups, hipStream_t s);
hipError_t launch_filter(const DevFilter &q, bool conj_only, int fused_naggs, int nblocks, size_t lds_bytes,
                         hipStream_t s, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);
hipError_t launch_masks_to_words(const uint32_t *masks, int32_t tile0, int32_t ntiles, uint64_t *words, int64_t nwords,
                                 hipStream_t s);
hipError_t launch_agg(const DevAggQuery &q, const DevAggQuery *dq, int nblocks, size_t lds, hipStream_t s,
                      hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);
hipError_t launch_hash_keys(int64_t *slots, int64_t n, const uint64_t *keys, hipStream_t s);
hipError_t launch_slab_reduce(const uint64_t *slab, int32_t nslabs, int32_t tbl_words, int64_t G, const int32_t *kinds,
                              uint64_t *out, const uint32_t *hslab, int32_t hll_words, uint32_t *hout, hipStream_t s);
hipError_t launch_finalize_partials2(const uint64_t *pa, int nba, int na, const int32_t *ka, uint64_t *oa,
                                     const uint64_t *pb, int nbb, int nb, const int32_t *kb, uint64_t *ob, hipStream_t s);
hipError_t launch_finalize_partials(const uint64_t *partials, int nblocks, int nslots, const int32_t *kinds,
                                    uint64_t *out, hipStream_t s);
hipError_t launch_finalize_all(const uint64_t *pa, int nba, int na, const int32_t *ka, const uint64_t *pf, int nbf,
                               const int32_t *kf, uint64_t *segm, int nseg, uint32_t *hll, int hll_words, uint64_t *out,
                               hipStream_t s, uint32_t *ticket = nullptr, uint64_t seq = 0);
hipError_t launch_group_count(const uint64_t *counts, int64_t n, int32_t *chunk_counts, int64_t nchunks,
                              int64_t *offsets, hipStream_t s);
hipError_t launch_group_compact(const uint64_t *counts, int64_t n, const int64_t *offsets, int64_t nchunks,
                                int64_t *keys, hipStream_t s);
hipError_t launch_group_gather(const int64_t *keys, int64_t ngroups, int64_t ndense, int32_t naggs, int32_t own_count,
                               const int32_t *kinds, const uint64_t *table, const uint32_t *hll, int32_t nhll,
                               int32_t log2m, double *vals, int64_t *longs, uint8_t *hll_out, hipStream_t s);
hipError_t launch_group_gather_mapped(const int64_t *keys, const int64_t *d_ngroups, int64_t ndense, int32_t naggs,
                                      int32_t own_count, const int32_t *kinds, const uint64_t *table,
                                      int64_t *out_count, int64_t *out_keys, double *vals, int64_t *longs,
                                      const uint32_t *hll, int32_t nhll, int32_t log2m, uint32_t *hll_out,
                                      hipStream_t s);
hipError_t launch_select_count(const DevSelQuery *q, int64_t total_work, int64_t *tile_cnt, hipStream_t s);
hipError_t launch_select_scan(void *temp, size_t *temp_bytes, const int64_t *in, int64_t *out, int64_t n, hipStream_t s);
hipError_t launch_select_bases(const DevSelQuery *q, int64_t *seg_base, int64_t *kept, int64_t *total, hipStream_t s);
hipError_t launch_select_str_lens(const uint64_t *loc, int64_t rows, const uint64_t *const *offs, uint32_t *lens,
                                  hipStream_t s);
hipError_t launch_select_str_bytes(const uint64_t *loc, int64_t rows, const uint8_t *const *strs,
                                   const uint64_t *const *offs, const uint64_t *dst_off, uint8_t *dst, hipStream_t s);
hipError_t launch_select_gather(const DevSelQuery *q, int64_t total_work, uint64_t *out, int64_t num_rows,
                                hipStream_t s);
hipError_t launch_limit_prepare(const int64_t *slots, int64_t n, const uint64_t *hkeys, const uint32_t *first_doc,
                                int32_t nseg, uint64_t *sortkey, int32_t *idx, hipStream_t s);
hipError_t launch_limit_bounds(const uint64_t *sk_sorted, int64_t n, int64_t *first, int64_t *last, hipStream_t s);
hipError_t launch_sort_pairs(void *temp, size_t *temp_bytes, const uint64_t *k_in, uint64_t *k_out, const void *v_in,
                             void *v_out, bool wide, int64_t n, int end_bit, hipStream_t s);
hipError_t launch_limit_select(const uint64_t *sk_sorted, const int32_t *idx_sorted, int64_t n, const int64_t *seg_start,
                               int64_t limit, const int64_t *slots, const uint64_t *hkeys, int32_t nseg, uint64_t *key2,
                               int64_t *slot2, hipStream_t s);
hipError_t launch_limit_runs(void *temp, size_t *scan_bytes, const uint64_t *k, int64_t n, int32_t *head, int32_t *run,
                             hipStream_t s);
hipError_t launch_limit_reduce(const uint64_t *k, const int64_t *slot2, int64_t n, const int32_t *head, const int32_t *run,
                               int64_t cap, int32_t naggs, int32_t own_count, const int32_t *kinds,
                               const uint64_t *table, const uint32_t *hll, int32_t nhll, int32_t log2m,
                               int64_t *keys_out, double *vals, int64_t *longs, uint8_t *hll_out, hipStream_t s);
hipError_t launch_raw_images(const void *raw, int32_t type, int64_t n, uint64_t *out, hipStream_t s);
hipError_t launch_sort_unique_u64(void *temp, size_t *temp_bytes, uint64_t *in, uint64_t *sorted, uint64_t *out,
                                  int64_t *num_out, int64_t n, hipStream_t s);
hipError_t launch_str_hash_unique(void *temp, size_t *temp_bytes, const uint8_t *bytes, const uint64_t *off, int64_t n,
                                  uint64_t *hash, int32_t *docs, uint64_t *hash_sorted, int32_t *docs_sorted,
                                  uint64_t *uniq, int32_t *rep, int64_t *num_out, hipStream_t s);
hipError_t launch_str_verify(const uint8_t *bytes, const uint64_t *off, int64_t n, const uint64_t *uniq, const int32_t *rep,
                             int64_t u, int32_t *collided, hipStream_t s);
hipError_t launch_str_rep_lens(const uint64_t *off, const int32_t *rep, int64_t u, uint32_t *lens, hipStream_t s);
hipError_t launch_str_rep_bytes(const uint8_t *bytes, const uint64_t *off, const int32_t *rep, int64_t u,
                                const uint64_t *dst_off, uint8_t *dst, hipStream_t s);
hipError_t set_str_hash_bits(int bits);
hipError_t launch_raw_str_ids(const uint8_t *bytes, const uint64_t *off, int64_t n, const uint64_t *uniq, int64_t u,
                              const int32_t *map, int32_t *ids, hipStream_t s);
hipError_t launch_tuple_words(const TupleCols &tc, int64_t n, uint64_t *out, hipStream_t s);
hipError_t launch_tuple_rank(void *temp, size_t *temp_bytes, const uint64_t *words, int32_t nw, int64_t n, int32_t *ids,
                             uint64_t *uniq, int64_t ucap, int64_t *num_out, hipStream_t s);
hipError_t launch_gather_ids(const int32_t *local, const int32_t *map, int64_t n, int32_t *out, hipStream_t s);
hipError_t launch_raw_key_ids(const void *raw, int32_t type, int64_t n, const uint64_t *uniq, int64_t u, int32_t *ids,
                              hipStream_t s);
hipError_t launch_materialize_hll16(const uint32_t *words, int32_t bits, const uint32_t *table, int64_t n, uint16_t *out,
                                    hipStream_t s);
hipError_t launch_materialize_record(const RecSrcs &fs, int nf, int64_t n, int W, uint32_t *out, hipStream_t s);
hipError_t launch_minmax_i64(const void *raw, int32_t type, int64_t n, int64_t *out, hipStream_t s,
                             const uint64_t *nulls = nullptr);
hipError_t launch_chunk_decode_global(int codec, const uint8_t *blob, const RawChunk *chunks, int32_t nchunks, uint8_t *out,
                                      int32_t *err, int32_t *sizes, uint8_t *lits, uint64_t lits_stride, hipStream_t s);
hipError_t launch_bitslice(const uint32_t *words, int32_t bits, int64_t ntiles, uint32_t *planes, hipStream_t s);
hipError_t launch_materialize_packed(const uint32_t *words, int32_t bits, const void *dict, int32_t width, int64_t n,
                                     int64_t base, int32_t vbits, int64_t nwords, uint32_t *out, hipStream_t s);
hipError_t launch_materialize(const uint32_t *words, int32_t bits, const void *dict, int32_t width, int64_t n,
                              void *vals, hipStream_t s);
hipError_t launch_varbyte_offsets(const uint8_t *stage, const uint64_t *chunk_base, const int32_t *chunk_size,
                                  int32_t per_chunk, int64_t n, uint64_t *len, uint64_t *off, void *temp,
                                  size_t *temp_bytes, int32_t *err, hipStream_t s);
hipError_t launch_varbyte_copy(const uint8_t *stage, const uint64_t *chunk_base, const int32_t *chunk_size,
                               int32_t per_chunk, int64_t n, const uint64_t *off, uint8_t *out, hipStream_t s);
}  // namespace phip

using namespace phip;

// ================================================================================================
// errors
// ================================================================================================
static thread_local std::string g_err;

static int32_t fail(int32_t code, const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                         \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    if (_e != hipSuccess) return fail(PHIP_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(_e)); \
  } while (0)

static inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
static inline int64_t round_up(int64_t a, int64_t b) { return ceil_div(a, b) * b; }
static inline uint32_t be32(const uint8_t *p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
static inline uint64_t be64(const uint8_t *p) { return ((uint64_t)be32(p) << 32) | be32(p + 4); }
static inline uint32_t le32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static inline uint16_t le16(const uint8_t *p) { return (uint16_t)(p[0] | (p[1] << 8)); }

static int num_bits_per_value(int32_t max_value) {  // PinotDataBitSet.getNumBitsPerValue (:61-72)
  if (max_value <= 1) return 1;
  int b = 0;
  while (max_value > 0) {
    b++;
    max_value >>= 1;
  }
  return b;
}

static int type_width(int32_t t) {
  switch (t) {
    case PHIP_TYPE_INT:
    case PHIP_TYPE_FLOAT: return 4;
    case PHIP_TYPE_LONG:
    case PHIP_TYPE_DOUBLE: return 8;
    default: return 0;
  }
}

// ================================================================================================
// clearspring MurmurHash / HyperLogLog register index (stream-lib 2.9.8, pom.xml:1416-1418), as
// DistinctCountHLLAggregationFunction offers dictionary values (…/function/DistinctCountHLLAggregationFunction.java:457-466)
// ================================================================================================
static int32_t murmur_hash_long(int64_t data) {
  const uint32_t m = 0x5bd1e995u;
  uint32_t h = 0;
  uint32_t k = (uint32_t)data * m;
  k ^= k >> 24;
  h ^= k * m;
  k = (uint32_t)((uint64_t)data >> 32) * m;
  k ^= k >> 24;
  h *= m;
  h ^= k * m;
  h ^= h >> 13;
  h *= m;
  h ^= h >> 15;
  return (int32_t)h;
}
static int32_t murmur_hash_bytes(const uint8_t *d, int32_t len, int32_t seed) {
  const uint32_t m = 0x5bd1e995u;
  uint32_t h = (uint32_t)seed ^ (uint32_t)len;
  int32_t n4 = len >> 2;
  for (int32_t i = 0; i < n4; i++) {
    uint32_t k = le32(d + 4 * i);
    k *= m;
    k ^= k >> 24;
    k *= m;
    h *= m;
    h ^= k;
  }
  int32_t left = len - (n4 << 2);
  if (left) {
    if (left >= 3) h ^= (uint32_t)((int32_t)(int8_t)d[len - 3] << 16);
    if (left >= 2) h ^= (uint32_t)((int32_t)(int8_t)d[len - 2] << 8);
    h ^= (uint32_t)(int32_t)(int8_t)d[len - 1];
    h *= m;
  }
  h ^= h >> 13;
  h *= m;
  h ^= h >> 15;
  return (int32_t)h;
}
static uint32_t hll_index_rho(int32_t x, int log2m) {  // HyperLogLog.offerHashed
  uint32_t ux = (uint32_t)x;
  uint32_t j = ux >> (32 - log2m);
  uint32_t w = (ux << log2m) | ((1u << (log2m - 1)) + 1u);
  uint32_t r = (uint32_t)__builtin_clz(w) + 1u;
  return (j << 8) | r;
}

// ================================================================================================
// devices and segments
// ================================================================================================
struct Workspace {
  struct Buf {
    void *p = nullptr;
    size_t cap = 0;
    int32_t small_uses = 0;  // consecutive requests of < 1/4 of cap (mapped areas shrink after kShrinkAfter)
  };
  static constexpr int32_t kShrinkAfter = 64;
  std::map<std::string, Buf> dev;
  std::map<std::string, Buf> host;  // pinned
  std::map<std::string, std::pair<Buf, void *>> mapped;  // pinned, device-visible (+ its device address)

  int32_t get(const std::string &name, size_t bytes, void **out) {
    Buf &b = dev[name];
    if (b.cap < bytes) {
      if (b.p) (void)hipFree(b.p);
      size_t cap = std::max<size_t>(bytes + bytes / 4, 4096);
      HIP_TRY(hipMalloc(&b.p, cap));
      b.cap = cap;
    }
    *out = b.p;
    return PHIP_OK;
  }
  int32_t get_host(const std::string &name, size_t bytes, void **out) {
    Buf &b = host[name];
    if (b.cap < bytes) {
      if (b.p) (void)hipHostFree(b.p);
      size_t cap = std::max<size_t>(bytes + bytes / 4, 4096);
      HIP_TRY(hipHostMalloc(&b.p, cap, hipHostMallocDefault));
      b.cap = cap;
    }
    *out = b.p;
    return PHIP_OK;
  }
  // A pinned, device-visible area (the group-by landing area): grown on demand, and given back to the allocator
  // once kShrinkAfter consecutive executions on this lane needed less than a quarter of it (one large key space
  // does not keep tens of MiB of pinned host memory per lane for the life of the process). The previous
  // execution on the lane has been read out before the next one asks, so a reallocation never races a writer.
  int32_t get_mapped(const std::string &name, size_t bytes, void **host_out, void **dev_out) {
    auto &e = mapped[name];
    const size_t big = (size_t)1 << 20;
    if (e.first.cap > big && bytes < e.first.cap / 4) {
      if (++e.first.small_uses >= kShrinkAfter) {
        (void)hipHostFree(e.first.p);
        e.first.p = nullptr;
        e.first.cap = 0;
        e.first.small_uses = 0;
      }
    } else {
      e.first.small_uses = 0;
    }
    if (e.first.cap < bytes) {
      if (e.first.p) (void)hipHostFree(e.first.p);
      e.first.p = nullptr;
      e.first.cap = 0;
      size_t cap = std::max<size_t>(bytes + bytes / 4, 4096);
      HIP_TRY(hipHostMalloc(&e.first.p, cap, hipHostMallocMapped));
      e.first.cap = cap;
      HIP_TRY(hipHostGetDevicePointer(&e.second, e.first.p, 0));
    }
    *host_out = e.first.p;
    *dev_out = e.second;
    return PHIP_OK;
  }
  void release() {
    for (auto &kv : mapped)
      if (kv.second.first.p) (void)hipHostFree(kv.second.first.p);
    mapped.clear();
    for (auto &kv : dev)
      if (kv.second.p) (void)hipFree(kv.second.p);
    for (auto &kv : host)
      if (kv.second.p) (void)hipHostFree(kv.second.p);
    dev.clear();
    host.clear();
  }
};

// One execution lane: a HIP stream and the scratch buffers of the queries that run on it. Queries on
// different lanes run concurrently (the server's worker threads, BaseCombineOperator.java:87-92 /
// ResourceManager.java:59-60); a lane is taken for the length of one execution.
struct Lane {
  hipStream_t stream = nullptr;
  Workspace ws;
};

struct Device {
  int ordinal = 0;
  int num_cus = 256;
  int num_xcc = 8;  // XCDs (L2 domains) of this device: the GB_XCD copies need at most kXcdCopies of them
  hipStream_t stream = nullptr;  // setup stream: segment load, plan preparation (under mu)
  hipEvent_t ev[4] = {};
  std::mutex mu;                 // guards setup work and the remap cache
  Workspace ws;
  std::mutex lane_mu;
  std::condition_variable lane_cv;
  std::vector<std::unique_ptr<Lane>> lanes;
  std::vector<Lane *> free_lanes;
  int max_lanes = 8;
  // query-global dictionary remaps for group-by (key: column + segment handles)
  struct Remap {
    std::vector<int32_t *> dev;  // per segment (nullptr = identity)
    int32_t card = 0;
    int32_t type = 0;
    int32_t width = 0;
    bool global = false;          // the column's registered node-global dictionary
    bool raw = false;             // a raw INT / LONG column: id = value - raw_base (values not materialised)
    int64_t raw_base = 0;
    std::vector<uint8_t> values;  // LE typed or fixed-width strings
    std::vector<int32_t *> ids;   // raw FLOAT / DOUBLE / STRING column: per segment its docs' ids into `values` (keys.hip)
    std::vector<uint64_t> tuples; // tuple keys (key spaces above 2^62): tuple_w x card packed words, word-major
    int32_t tuple_w = 0;
    ~Remap() {
      for (auto *p : dev)
        if (p) (void)hipFree(p);
      for (auto *p : ids)
        if (p) (void)hipFree(p);
    }
  };
  std::map<std::string, std::shared_ptr<Remap>> remaps;
  // node-global dictionaries registered by phip_global_dictionary, per column
  struct GlobalDict {
    int32_t type = 0, card = 0, width = 0;
    uint64_t gen = 0;
    std::vector<uint8_t> values;  // LE typed or card x width padded strings
  };
  std::map<std::string, GlobalDict> globals;
  uint64_t global_gen = 0;
};

struct Container {
  int32_t key, kind, card;
  uint64_t off;  // payload offset within the column's device blob
};

struct ColumnStore {
  std::string name;
  int32_t type = 0, fwd_kind = 0, card = 0, bits = 0, string_width = 0;
  int32_t hll_log2m = 0;      // PHIP_FWD_HLL_REGISTERS: 2^hll_log2m u8 registers per doc in `raw`
  uint32_t *words = nullptr;  // fixed-bit dict ids (also synthesised for sorted columns)
  void *dict = nullptr;       // LE typed dictionary (numeric)
  void *raw = nullptr;        // LE raw values (raw STRING: the values' UTF-8 bytes, back to back)
  uint64_t *str_off = nullptr;  // raw STRING: num_docs + 1 byte offsets into raw
  uint64_t str_total = 0;       // raw STRING: bytes of all values
  uint32_t *planes = nullptr;   // bit-sliced copy of words (fixed-bit columns of <= kBitSliceMaxBits bits)
  void *vals = nullptr;         // numeric dictionary column: doc-order LE values (ensure_vals), made on first use
  uint32_t *vpack = nullptr;    // ... INT / LONG: the same values bit-packed at the range's width (value - vmin)
  int32_t vbits = 0;
  uint64_t *nulls = nullptr;    // null value vector as dense doc words (load_null_vector), or null: no null doc
  int64_t null_count = 0;
  std::vector<uint8_t> host_dict;  // dictionary bytes as given (BE / padded strings)
  std::vector<int32_t> sorted_pairs;  // sorted columns: (start,end) per dict id
  std::map<int, uint32_t *> hll;      // per log2m
  std::map<int, uint32_t *> hll_doc;  // per log2m: doc-order copy of hll (ensure_hll_doc), in the segment's allocations
  std::map<int, uint16_t *> hll_doc16;  // per log2m <= 11: the same entries packed to 16 bits
  bool has_range = false;             // INT / LONG: value range (plan-time overflow bound of integer sums)
  int64_t vmin = 0, vmax = 0;
  int64_t nn_vmin = 0, nn_vmax = 0;   // raw INT / LONG with a null vector: the non-null values' range (null keys);
  bool nn_empty = false;              // nn_empty: every doc is null
  // inverted index
  uint8_t *inv_blob = nullptr;
  std::vector<int64_t> inv_begin;  // card+1 into inv_conts
  std::vector<Container> inv_conts;
};
// No dictionary: a raw chunk forward index, or the HLL register rows of a star-tree DISTINCTCOUNTHLL pair
static inline bool no_dict(const ColumnStore &c) {
  return c.fwd_kind == PHIP_FWD_RAW_CHUNK || c.fwd_kind == PHIP_FWD_HLL_REGISTERS;
}


// HBM held by group-by records per device (build_records' budget)
constexpr int kMaxRecordDevices = 64;
static std::atomic<uint64_t> g_record_bytes[kMaxRecordDevices];

struct Segment {
  uint64_t handle = 0;
  int device = 0;
  int32_t num_docs = 0;
  std::string name;
  std::vector<ColumnStore> cols;
  std::unordered_map<std::string, int> by_name;
  uint64_t device_bytes = 0;
  std::vector<void *> allocations;
  // group-by records (DevSeg.rec) by field signature: words, u32 per doc (build_records; in `allocations`)
  struct Record {
    uint32_t *words = nullptr;
    int32_t width = 0;
  };
  std::map<std::string, Record> records;
  uint64_t record_bytes = 0;
  ~Segment() {
    if (device >= 0 && device < kMaxRecordDevices) g_record_bytes[device] -= record_bytes;
    (void)hipSetDevice(device);
    for (void *p : allocations) (void)hipFree(p);
    for (auto &c : cols)
      for (auto &kv : c.hll) (void)hipFree(kv.second);
  }
};

static std::mutex g_mu;  // guards the registries below
static std::vector<std::unique_ptr<Device>> g_devices;
// Segments are shared with the plans that reference them: unloading drops the registry's reference
// and the HBM is released when the last prepared plan over the segment is destroyed (the role of the
// Phaser guard in BaseCombineOperator.java:87-92).
static std::unordered_map<uint64_t, std::shared_ptr<Segment>> g_segments;
static std::atomic<uint64_t> g_next_handle{1};

static void init_lanes(Device *d);

// XCDs of a device (hipDeviceAttributeNumberOfXccs; 8 on an MI355X in SPX mode, 1 per device in CPX). The fused
// group-by's GB_XCD mode picks a table copy by HW_REG_XCC_ID & 7 and updates it with workgroup-scope atomics in that
// XCD's L2, correct only while no two L2 domains of the device share a copy: with at most kXcdCopies XCDs the ids
// are distinct mod 8 (a partition's XCC ids are a contiguous run). A device reporting more XCDs, or no count at all,
// keeps the one agent-scope table (prepare_plan).
static hipError_t device_xcc_count(int ordinal, int *out) {
  int x = 0;
  if (hipDeviceGetAttribute(&x, hipDeviceAttributeNumberOfXccs, ordinal) != hipSuccess || x <= 0) x = 1 << 30;
  *out = x;
  return hipSuccess;
}

static int32_t ensure_devices_locked() {
  if (!g_devices.empty()) return PHIP_OK;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(PHIP_ERR_NO_DEVICE, "no HIP device available");
  int cur = 0;
  HIP_TRY(hipGetDevice(&cur));
  auto d = std::make_unique<Device>();
  d->ordinal = cur;
  HIP_TRY(hipSetDevice(cur));
  HIP_TRY(hipDeviceGetAttribute(&d->num_cus, hipDeviceAttributeMultiprocessorCount, cur));
  HIP_TRY(device_xcc_count(cur, &d->num_xcc));
  HIP_TRY(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
  for (auto &e : d->ev) HIP_TRY(hipEventCreate(&e));
  init_lanes(d.get());
  g_devices.push_back(std::move(d));
  return PHIP_OK;
}

static Device *find_device(int ordinal) {
  for (auto &d : g_devices)
    if (d->ordinal == ordinal) return d.get();
  return nullptr;
}

// A free lane of the device, created on demand up to max_lanes (PHIP_STREAMS), else wait for one.
static int32_t acquire_lane(Device *dev, Lane **out) {
  std::unique_lock<std::mutex> lk(dev->lane_mu);
  while (dev->free_lanes.empty() && (int)dev->lanes.size() >= dev->max_lanes) dev->lane_cv.wait(lk);
  if (dev->free_lanes.empty()) {
    auto l = std::make_unique<Lane>();
    HIP_TRY(hipSetDevice(dev->ordinal));
    HIP_TRY(hipStreamCreateWithFlags(&l->stream, hipStreamNonBlocking));
    dev->free_lanes.push_back(l.get());
    dev->lanes.push_back(std::move(l));
  }
  *out = dev->free_lanes.back();
  dev->free_lanes.pop_back();
  return PHIP_OK;
}

static void release_lane(Device *dev, Lane *l) {
  {
    std::lock_guard<std::mutex> lk(dev->lane_mu);
    dev->free_lanes.push_back(l);
  }
  dev->lane_cv.notify_one();
}

// Holds an execution lane for one execution. An execution that returns early (an error after kernels were
// enqueued) leaves `done` false: the guard then drains the lane's stream before handing it back, so no kernel of
// that execution can still be reading plan buffers that a later phip_plan_destroy frees.
struct LaneGuard {
  Device *dev;
  Lane *lane = nullptr;
  bool done = false;
  ~LaneGuard() {
    if (!lane) return;
    if (!done) (void)hipStreamSynchronize(lane->stream);
    release_lane(dev, lane);
  }
};

static void init_lanes(Device *d) {
  const char *e = getenv("PHIP_STREAMS");  // execution lanes per device (default 8)
  if (e) d->max_lanes = std::max(1, std::min(64, atoi(e)));
}

// ================================================================================================
// segment load
// ================================================================================================
static int32_t dev_alloc(Segment &s, size_t bytes, void **out) {
  void *p = nullptr;
  HIP_TRY(hipMalloc(&p, bytes == 0 ? 16 : bytes));
  s.allocations.push_back(p);
  s.device_bytes += bytes;
  *out = p;
  return PHIP_OK;
}

static int32_t parse_inverted(const phip_column_desc &c, ColumnStore &cs, Segment &seg, hipStream_t st) {
  const uint8_t *b = c.inverted;
  const uint64_t len = c.inverted_bytes;
  const int32_t card = c.cardinality;
  const uint64_t off_bytes = (uint64_t)(card + 1) * 4;
  if (len < off_bytes) return fail(PHIP_ERR_INVALID, "column %s: inverted index too short", c.name);
  // BitmapInvertedIndexReader.java:40-62: offsets are absolute or relative; normalise by the first
  const uint64_t first = be32(b);
  cs.inv_begin.assign(card + 1, 0);
  for (int32_t d = 0; d < card; d++) {
    uint64_t o0 = be32(b + 4 * d) - first, o1 = be32(b + 4 * (d + 1)) - first;
    if (o1 < o0 || off_bytes + o1 > len) return fail(PHIP_ERR_INVALID, "column %s: bad bitmap offsets", c.name);
    const uint8_t *bm = b + off_bytes + o0;
    const uint64_t blen = o1 - o0;
    cs.inv_begin[d] = (int64_t)cs.inv_conts.size();
    if (blen < 8) return fail(PHIP_ERR_INVALID, "column %s: bitmap %d truncated", c.name, d);
    uint32_t cookie = le32(bm);
    uint64_t pos;
    int32_t size;
    bool has_run = false;
    const uint8_t *runflags = nullptr;
    if ((cookie & 0xFFFF) == 12347) {
      has_run = true;
      size = (int32_t)(cookie >> 16) + 1;
      runflags = bm + 4;
      pos = 4 + (uint64_t)(size + 7) / 8;
    } else if (cookie == 12346) {
      size = (int32_t)le32(bm + 4);
      pos = 8;
    } else {
      return fail(PHIP_ERR_INVALID, "column %s: bitmap %d bad cookie %u", c.name, d, cookie);
    }
    const uint8_t *hdr = bm + pos;
    pos += 4ull * size;
    const bool has_off = !has_run || size >= 4;
    const uint8_t *offs = bm + pos;
    if (has_off) pos += 4ull * size;
    if (pos > blen) return fail(PHIP_ERR_INVALID, "column %s: bitmap %d header overflow", c.name, d);
    for (int32_t k = 0; k < size; k++) {
      Container ct;
      ct.key = le16(hdr + 4 * k);
      int32_t ccard = (int32_t)le16(hdr + 4 * k + 2) + 1;
      bool is_run = has_run && ((runflags[k >> 3] >> (k & 7)) & 1);
      if (has_off) pos = le32(offs + 4 * k);
      if (pos + 2 > blen) return fail(PHIP_ERR_INVALID, "column %s: bitmap %d container overflow", c.name, d);
      uint64_t psize;
      if (is_run) {
        ct.kind = 2;
        ct.card = le16(bm + pos);
        psize = 2 + 4ull * ct.card;
      } else if (ccard <= 4096) {
        ct.kind = 0;
        ct.card = ccard;
        psize = 2ull * ccard;
      } else {
        ct.kind = 1;
        ct.card = ccard;
        psize = 8192;
      }
      if (pos + psize > blen) return fail(PHIP_ERR_INVALID, "column %s: bitmap %d payload overflow", c.name, d);
      // a container's first doc must lie inside the segment (its 1024 decoded words land in the leaf's
      // round_up(numDocs, 65536) / 64 words), and a run may not pass the container's 65536 docs
      if ((int64_t)ct.key * 65536 >= (int64_t)seg.num_docs)
        return fail(PHIP_ERR_INVALID, "column %s: bitmap %d key beyond numDocs", c.name, d);
      if (is_run)
        for (int32_t ri = 0; ri < ct.card; ri++)
          if ((uint32_t)le16(bm + pos + 2 + 4 * ri) + le16(bm + pos + 4 + 4 * ri) > 65535u)
            return fail(PHIP_ERR_INVALID, "column %s: bitmap %d run container past 65535", c.name, d);
      ct.off = off_bytes + o0 + pos - off_bytes;  // relative to blob start (after offsets)
      cs.inv_conts.push_back(ct);
      pos += psize;
    }
  }
  cs.inv_begin[card] = (int64_t)cs.inv_conts.size();
  const uint64_t blob = len - off_bytes;
  void *p;
  int32_t rc = dev_alloc(seg, blob + 16, &p);
  if (rc) return rc;
  cs.inv_blob = (uint8_t *)p;
  HIP_TRY(hipMemcpyAsync(cs.inv_blob, b + off_bytes, blob, hipMemcpyHostToDevice, st));
  return PHIP_OK;
}

// Null value vector (NullValueVectorReaderImpl: one portable Roaring bitmap, NullValueVectorCreator.java:83-92) ->
// dense doc words in HBM, the inverted leaves' layout (bit d % 64 of u64 word d / 64), padded to whole 2048-doc tiles
// so a PHIP_LEAF_NULL leaf stages 256 bytes per tile like any bitmap leaf. Decoded on the host once at load.
static int32_t load_null_vector(const phip_column_desc &c, ColumnStore &cs, Segment &seg, hipStream_t st) {
  const uint8_t *bm = c.null_vector;
  const uint64_t len = c.null_vector_bytes;
  const int64_t n = seg.num_docs;
  if (len < 8) return fail(PHIP_ERR_INVALID, "column %s: null vector truncated", c.name);
  const uint32_t cookie = le32(bm);
  int32_t size;
  uint64_t pos;
  const uint8_t *runflags = nullptr;
  if ((cookie & 0xFFFF) == 12347) {
    size = (int32_t)(cookie >> 16) + 1;
    runflags = bm + 4;
    pos = 4 + (uint64_t)(size + 7) / 8;
  } else if (cookie == 12346) {
    size = (int32_t)le32(bm + 4);
    pos = 8;
  } else {
    return fail(PHIP_ERR_INVALID, "column %s: null vector bad cookie %u", c.name, cookie);
  }
  if (size < 0 || pos + 4ull * size > len) return fail(PHIP_ERR_INVALID, "column %s: null vector header", c.name);
  const uint8_t *hdr = bm + pos;
  pos += 4ull * size;
  const bool has_off = runflags == nullptr || size >= 4;
  const uint8_t *offs = bm + pos;
  if (has_off) pos += 4ull * size;
  if (pos > len) return fail(PHIP_ERR_INVALID, "column %s: null vector header", c.name);
  const int64_t nwords = round_up(std::max<int64_t>(n, 1), kTileDocs) / 64;
  std::vector<uint64_t> words((size_t)nwords, 0);
  int64_t count = 0;
  auto set = [&](int64_t d) -> bool {
    if (d < 0 || d >= n) return false;
    words[(size_t)(d >> 6)] |= 1ull << (d & 63);
    count++;
    return true;
  };
  for (int32_t k = 0; k < size; k++) {
    const int64_t key = le16(hdr + 4 * k);
    const int32_t ccard = (int32_t)le16(hdr + 4 * k + 2) + 1;
    const bool is_run = runflags && ((runflags[k >> 3] >> (k & 7)) & 1);
    if (has_off) pos = le32(offs + 4 * k);
    const int64_t base = key << 16;
    if (is_run) {
      if (pos + 2 > len) return fail(PHIP_ERR_INVALID, "column %s: null vector container overflow", c.name);
      const int32_t nruns = le16(bm + pos);
      if (pos + 2 + 4ull * nruns > len) return fail(PHIP_ERR_INVALID, "column %s: null vector run overflow", c.name);
      for (int32_t r = 0; r < nruns; r++) {
        const int64_t s0 = le16(bm + pos + 2 + 4 * r), l = le16(bm + pos + 4 + 4 * r);
        for (int64_t d = base + s0; d <= base + s0 + l; d++)
          if (!set(d)) return fail(PHIP_ERR_INVALID, "column %s: null doc beyond numDocs", c.name);
      }
      pos += 2 + 4ull * nruns;
    } else if (ccard <= 4096) {
      if (pos + 2ull * ccard > len) return fail(PHIP_ERR_INVALID, "column %s: null vector array overflow", c.name);
      for (int32_t i = 0; i < ccard; i++)
        if (!set(base + le16(bm + pos + 2 * i))) return fail(PHIP_ERR_INVALID, "column %s: null doc beyond numDocs", c.name);
      pos += 2ull * ccard;
    } else {
      if (pos + 8192 > len) return fail(PHIP_ERR_INVALID, "column %s: null vector bitmap overflow", c.name);
      for (int32_t w = 0; w < 1024; w++) {
        uint64_t x = 0;
        for (int b = 0; b < 8; b++) x |= (uint64_t)bm[pos + 8 * w + b] << (8 * b);
        for (; x; x &= x - 1)
          if (!set(base + 64 * w + __builtin_ctzll(x))) return fail(PHIP_ERR_INVALID, "column %s: null doc beyond numDocs", c.name);
      }
      pos += 8192;
    }
  }
  if (count == 0) return PHIP_OK;  // (an empty bitmap: no null vector, as the creator never writes one)
  void *p;
  int32_t rc = dev_alloc(seg, (size_t)nwords * 8, &p);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(p, words.data(), (size_t)nwords * 8, hipMemcpyHostToDevice, st));
  HIP_TRY(hipStreamSynchronize(st));  // (the host words go out of scope)
  cs.nulls = (uint64_t *)p;
  cs.null_count = count;
  return PHIP_OK;
}

// Raw STRING column: VarByteChunkForwardIndexWriter v1..v3 (VarByteChunkForwardIndexWriter.java:37-158 over the
// BaseChunkForwardIndexWriter header and chunk table; per chunk numDocsPerChunk BE int start offsets, then the
// values' UTF-8 bytes; VarByteChunkSVForwardIndexReader.java:80-217 reads them) -> the values back to back in HBM
// plus num_docs + 1 u64 offsets, built on the GPU (load.hip): compressed chunks are decoded by the same kernel as
// fixed-width ones (their decoded size is their own, at most the writer's chunk buffer), then a lengths pass, an
// exclusive scan and a copy. The V4 / V5 var-byte writers (a different chunk layout) are outside the GPU path.
static int32_t load_varbyte(const phip_column_desc &c, Segment &seg, ColumnStore &cs, hipStream_t st,
                            std::vector<void *> &temps) {
  const int64_t n = seg.num_docs;
  const uint8_t *h = c.forward;
  if (h == nullptr || c.forward_bytes < 16) return fail(PHIP_ERR_INVALID, "column %s: chunk header truncated", c.name);
  const int32_t version = (int32_t)be32(h), num_chunks = (int32_t)be32(h + 4), per_chunk = (int32_t)be32(h + 8);
  const int32_t longest = (int32_t)be32(h + 12);
  int32_t total = (int32_t)n, comp = 1, data_hdr = 16;  // v1: 4-int header, SNAPPY chunks, int offsets from byte 16
  if (version < 1 || version > 3)
    return fail(PHIP_ERR_UNSUPPORTED, "column %s: var-byte chunk version %d (the GPU path reads v1..v3)", c.name, version);
  if (version > 1) {
    if (c.forward_bytes < 28) return fail(PHIP_ERR_INVALID, "column %s: chunk header truncated", c.name);
    total = (int32_t)be32(h + 16);
    comp = (int32_t)be32(h + 20);
    data_hdr = (int32_t)be32(h + 24);
  }
  if (comp < 0 || comp > 5) return fail(PHIP_ERR_INVALID, "column %s: unknown chunk compression type %d", c.name, comp);
  if (total != n || per_chunk <= 0 || longest < 0 || num_chunks != ceil_div(n, per_chunk))
    return fail(PHIP_ERR_INVALID, "column %s: bad var-byte chunk header", c.name);
  const int osz = version <= 2 ? 4 : 8;
  const uint64_t hdr_end = (uint64_t)data_hdr + (uint64_t)num_chunks * osz;
  if (data_hdr < (version > 1 ? 28 : 16) || hdr_end > c.forward_bytes)
    return fail(PHIP_ERR_INVALID, "column %s: chunk offsets truncated", c.name);
  // the writer's chunk buffer: numDocsPerChunk x (4 + lengthOfLongestEntry) (VarByteChunkForwardIndexWriter.java:69-71)
  const uint64_t max_u = (uint64_t)per_chunk * (4 + (uint64_t)longest);
  if (max_u >= (1ull << 31)) return fail(PHIP_ERR_INVALID, "column %s: var-byte chunk of %llu bytes", c.name, (unsigned long long)max_u);
  auto chunk_off = [&](int32_t k) -> uint64_t { return osz == 4 ? be32(h + data_hdr + 4 * k) : be64(h + data_hdr + 8 * k); };
  std::vector<uint64_t> base(std::max(num_chunks, 1), 0);
  std::vector<int32_t> size(std::max(num_chunks, 1), 0);
  std::vector<RawChunk> chunks(std::max(num_chunks, 1));
  const uint64_t first = num_chunks > 0 ? chunk_off(0) : hdr_end;
  uint32_t max_c = 0;
  for (int32_t k = 0; k < num_chunks; k++) {
    const uint64_t off = chunk_off(k), end = k + 1 < num_chunks ? chunk_off(k + 1) : c.forward_bytes;
    if (off < hdr_end || end < off || end > c.forward_bytes || end - off >= (1ull << 31))
      return fail(PHIP_ERR_INVALID, "column %s: chunk %d offsets out of order", c.name, k);
    if (comp == 0 && end - off > max_u) return fail(PHIP_ERR_INVALID, "column %s: chunk %d exceeds its header", c.name, k);
    base[k] = off - first;
    size[k] = (int32_t)(end - off);
    chunks[k].src = off - first;
    chunks[k].csize = (uint32_t)(end - off);
    chunks[k].usize = (uint32_t)max_u;
    max_c = std::max(max_c, chunks[k].csize);
  }
  const uint64_t blob_bytes = c.forward_bytes - first;
  void *blob, *dbase, *dsize, *err;
  HIP_TRY(hipMalloc(&blob, blob_bytes + 16));
  temps.push_back(blob);
  HIP_TRY(hipMalloc(&dbase, base.size() * 8));
  temps.push_back(dbase);
  HIP_TRY(hipMalloc(&dsize, size.size() * 4));
  temps.push_back(dsize);
  HIP_TRY(hipMalloc(&err, 4));
  temps.push_back(err);
  HIP_TRY(hipMemsetAsync(err, 0, 4, st));
  if (blob_bytes) HIP_TRY(hipMemcpyAsync(blob, h + first, blob_bytes, hipMemcpyHostToDevice, st));
  const uint8_t *stage = (const uint8_t *)blob;
  if (comp != 0 && num_chunks > 0) {
    const uint64_t stride = (uint64_t)round_up((int64_t)max_u, 16);
    for (int32_t k = 0; k < num_chunks; k++) {
      base[k] = (uint64_t)k * stride;
      chunks[k].dst = base[k];
    }
    const uint32_t out_cap = (uint32_t)stride;
    const uint32_t in_cap = (uint32_t)round_up(max_c + 8, 16);
    const size_t lds = out_cap + in_cap + chunk_decode_extra_lds(comp, (int32_t)out_cap);
    void *dec, *table;
    HIP_TRY(hipMalloc(&dec, stride * num_chunks + 16));
    temps.push_back(dec);
    HIP_TRY(hipMalloc(&table, sizeof(RawChunk) * num_chunks));
    temps.push_back(table);
    HIP_TRY(hipMemcpyAsync(table, chunks.data(), sizeof(RawChunk) * num_chunks, hipMemcpyHostToDevice, st));
    if (lds <= 163840 - 1024) {  // the chunk and its output in LDS (as fixed-width chunks)
      HIP_TRY(launch_chunk_decode(comp, 1, (const uint8_t *)blob, (const RawChunk *)table, num_chunks, (int32_t)out_cap,
                                  (int32_t)in_cap, lds, (uint8_t *)dec, (int32_t *)err, (int32_t *)dsize, st));
    } else {  // beyond the LDS window (e.g. Pinot's derived 1 MiB chunks): decoded from and into HBM
      void *lits = nullptr;
      if (comp == 2) {
        HIP_TRY(hipMalloc(&lits, stride * num_chunks + 16));
        temps.push_back(lits);
      }
      HIP_TRY(launch_chunk_decode_global(comp, (const uint8_t *)blob, (const RawChunk *)table, num_chunks, (uint8_t *)dec,
                                         (int32_t *)err, (int32_t *)dsize, (uint8_t *)lits, stride, st));
    }
    int32_t bad = 0;
    HIP_TRY(hipMemcpyAsync(&bad, err, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (bad) return fail(PHIP_ERR_INVALID, "column %s: malformed compressed chunk %d (type %d)", c.name, bad - 1, comp);
    stage = (const uint8_t *)dec;
  } else {
    HIP_TRY(hipMemcpyAsync(dsize, size.data(), size.size() * 4, hipMemcpyHostToDevice, st));
  }
  HIP_TRY(hipMemcpyAsync(dbase, base.data(), base.size() * 8, hipMemcpyHostToDevice, st));
  void *off, *len, *temp;
  int32_t rc = dev_alloc(seg, (size_t)(n + 1) * 8, &off);
  if (rc) return rc;
  HIP_TRY(hipMalloc(&len, (size_t)(n + 1) * 8));
  temps.push_back(len);
  size_t temp_bytes = 0;
  HIP_TRY(launch_varbyte_offsets(stage, (const uint64_t *)dbase, (const int32_t *)dsize, per_chunk, n, (uint64_t *)len,
                                 (uint64_t *)off, nullptr, &temp_bytes, (int32_t *)err, st));
  HIP_TRY(hipMalloc(&temp, std::max<size_t>(temp_bytes, 16)));
  temps.push_back(temp);
  HIP_TRY(launch_varbyte_offsets(stage, (const uint64_t *)dbase, (const int32_t *)dsize, per_chunk, n, (uint64_t *)len,
                                 (uint64_t *)off, temp, &temp_bytes, (int32_t *)err, st));
  int32_t bad = 0;
  uint64_t nbytes = 0;
  HIP_TRY(hipMemcpyAsync(&bad, err, 4, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(&nbytes, (uint64_t *)off + n, 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (bad) return fail(PHIP_ERR_INVALID, "column %s: var-byte row offsets outside their chunk", c.name);
  void *bytes;
  rc = dev_alloc(seg, nbytes + 16, &bytes);
  if (rc) return rc;
  HIP_TRY(launch_varbyte_copy(stage, (const uint64_t *)dbase, (const int32_t *)dsize, per_chunk, n, (const uint64_t *)off,
                              (uint8_t *)bytes, st));
  HIP_TRY(hipStreamSynchronize(st));
  cs.raw = bytes;
  cs.str_off = (uint64_t *)off;
  cs.str_total = nbytes;
  return PHIP_OK;
}

static int32_t load_column(const phip_column_desc &c, Segment &seg, hipStream_t st, std::vector<void *> &temps) {
  ColumnStore cs;
  if (!c.name) return fail(PHIP_ERR_INVALID, "column without name");
  cs.name = c.name;
  cs.type = c.data_type;
  cs.fwd_kind = c.fwd_kind;
  cs.card = c.cardinality;
  cs.string_width = c.string_width;
  const int64_t n = seg.num_docs;
  if (c.data_type < PHIP_TYPE_INT || c.data_type > PHIP_TYPE_STRING)
    return fail(PHIP_ERR_INVALID, "column %s: bad data type %d", c.name, c.data_type);
  if (c.fwd_kind < PHIP_FWD_FIXED_BIT || c.fwd_kind > PHIP_FWD_HLL_REGISTERS)
    return fail(PHIP_ERR_INVALID, "column %s: bad forward kind %d", c.name, c.fwd_kind);
  const bool dict = c.fwd_kind == PHIP_FWD_FIXED_BIT || c.fwd_kind == PHIP_FWD_SORTED;
  if (c.fwd_kind == PHIP_FWD_HLL_REGISTERS) {
    // a star-tree DISTINCTCOUNTHLL pair: per doc 2^log2m u8 registers, copied as they are
    const int lg = c.bits_per_value;
    if (lg < 4 || lg > 12 || c.forward_bytes != ((uint64_t)n << lg) || (n > 0 && !c.forward))
      return fail(PHIP_ERR_INVALID, "column %s: HLL registers need num_docs x 2^log2m bytes (log2m %d)", c.name, lg);
    void *p;
    int32_t rc = dev_alloc(seg, std::max<uint64_t>(c.forward_bytes, 16), &p);
    if (rc) return rc;
    if (n > 0) HIP_TRY(hipMemcpyAsync(p, c.forward, c.forward_bytes, hipMemcpyHostToDevice, st));
    cs.raw = p;
    cs.hll_log2m = lg;
    cs.card = 0;
  } else if (dict) {
    if (c.cardinality <= 0) return fail(PHIP_ERR_INVALID, "column %s: cardinality must be > 0", c.name);
    const int w = c.data_type == PHIP_TYPE_STRING ? c.string_width : type_width(c.data_type);
    if (w <= 0 || c.dictionary == nullptr || c.dictionary_bytes != (uint64_t)w * c.cardinality)
      return fail(PHIP_ERR_INVALID, "column %s: dictionary size %llu != card %d x width %d", c.name,
                  (unsigned long long)c.dictionary_bytes, c.cardinality, w);
    cs.host_dict.assign(c.dictionary, c.dictionary + c.dictionary_bytes);
    if (c.data_type == PHIP_TYPE_INT || c.data_type == PHIP_TYPE_LONG) {  // sorted: first and last entries
      const size_t last = (size_t)(c.cardinality - 1) * w;
      cs.vmin = w == 4 ? (int64_t)(int32_t)be32(c.dictionary) : (int64_t)be64(c.dictionary);
      cs.vmax = w == 4 ? (int64_t)(int32_t)be32(c.dictionary + last) : (int64_t)be64(c.dictionary + last);
      cs.has_range = true;
    }
    if (c.data_type != PHIP_TYPE_STRING) {
      void *p;
      int32_t rc = dev_alloc(seg, c.dictionary_bytes, &p);
      if (rc) return rc;
      HIP_TRY(hipMemcpyAsync(p, c.dictionary, c.dictionary_bytes, hipMemcpyHostToDevice, st));
      if (w == 4) HIP_TRY(launch_bswap32((uint32_t *)p, c.cardinality, st));
      else HIP_TRY(launch_bswap64((uint64_t *)p, c.cardinality, st));
      cs.dict = p;
    }
    cs.bits = num_bits_per_value(c.cardinality - 1);
    // padded word array: whole tiles + 4 guard words
    const int64_t nwords = round_up(std::max<int64_t>(n, 1), kTileDocs) * cs.bits / 32 + 4;
    void *wp;
    int32_t rc = dev_alloc(seg, nwords * 4, &wp);
    if (rc) return rc;
    cs.words = (uint32_t *)wp;
    HIP_TRY(hipMemsetAsync(cs.words, 0, nwords * 4, st));
    if (c.fwd_kind == PHIP_FWD_FIXED_BIT) {
      if (c.bits_per_value != cs.bits)
        return fail(PHIP_ERR_INVALID, "column %s: bits %d != getNumBitsPerValue(card-1) = %d", c.name,
                    c.bits_per_value, cs.bits);
      const uint64_t need = (uint64_t)ceil_div(n * cs.bits, 8);
      if (c.forward_bytes < need)
        return fail(PHIP_ERR_INVALID, "column %s: forward index %llu bytes < %llu", c.name,
                    (unsigned long long)c.forward_bytes, (unsigned long long)need);
      HIP_TRY(hipMemcpyAsync(cs.words, c.forward, need, hipMemcpyHostToDevice, st));
      HIP_TRY(launch_bswap32(cs.words, ceil_div(need, 4), st));
      // the bit-sliced copy for conjunctive range leaves (load.hip bitslice_kernel): 256 x bits bytes per tile,
      // as many as the packed words -- narrow columns only (a range costs ~4 ops per plane per 32 docs there)
      if (cs.bits <= kBitSliceMaxBits && getenv("PHIP_NO_BITSLICE_LOAD") == nullptr) {
        const int64_t ntiles = ceil_div(std::max<int64_t>(n, 1), kTileDocs);
        void *pp;
        rc = dev_alloc(seg, (size_t)ntiles * cs.bits * 256, &pp);
        if (rc) return rc;
        cs.planes = (uint32_t *)pp;
        HIP_TRY(launch_bitslice(cs.words, cs.bits, ntiles, cs.planes, st));
      }
    } else if (c.fwd_kind == PHIP_FWD_SORTED) {
      if (c.forward_bytes != 8ull * c.cardinality)
        return fail(PHIP_ERR_INVALID, "column %s: sorted index must be card x 8 bytes", c.name);
      cs.sorted_pairs.resize(2 * (size_t)c.cardinality);
      int64_t expect = 0;
      for (int32_t d = 0; d < c.cardinality; d++) {
        int32_t s = (int32_t)be32(c.forward + 8 * d), e = (int32_t)be32(c.forward + 8 * d + 4);
        if (s != expect || e < s || e >= n)
          return fail(PHIP_ERR_INVALID, "column %s: sorted ranges not contiguous at dict id %d", c.name, d);
        expect = (int64_t)e + 1;
        cs.sorted_pairs[2 * d] = s;
        cs.sorted_pairs[2 * d + 1] = e;
      }
      if (expect != n) return fail(PHIP_ERR_INVALID, "column %s: sorted ranges do not cover numDocs", c.name);
      void *pairs, *ids;
      HIP_TRY(hipMalloc(&pairs, c.forward_bytes));
      temps.push_back(pairs);
      HIP_TRY(hipMalloc(&ids, std::max<int64_t>(n, 1) * 4));
      temps.push_back(ids);
      HIP_TRY(hipMemcpyAsync(pairs, c.forward, c.forward_bytes, hipMemcpyHostToDevice, st));
      HIP_TRY(launch_sorted_to_packed((const uint32_t *)pairs, c.cardinality, (int32_t *)ids, n, cs.bits, cs.words,
                                      ceil_div(n * cs.bits, 32), st));
    } else {
      return fail(PHIP_ERR_INVALID, "column %s: bad forward kind %d", c.name, c.fwd_kind);
    }
    if (c.inverted) {
      int32_t rc2 = parse_inverted(c, cs, seg, st);
      if (rc2) return rc2;
    }
  } else if (c.data_type == PHIP_TYPE_STRING) {
    int32_t rc = load_varbyte(c, seg, cs, st, temps);
    if (rc) return rc;
  } else {
    // raw fixed-width chunk forward index (BaseChunkForwardIndexWriter.java:40-160)
    const uint8_t *h = c.forward;
    if (c.forward_bytes < 16) return fail(PHIP_ERR_INVALID, "column %s: chunk header truncated", c.name);
    int32_t version = (int32_t)be32(h), num_chunks = (int32_t)be32(h + 4), per_chunk = (int32_t)be32(h + 8);
    int32_t entry = (int32_t)be32(h + 12), total = (int32_t)n, comp = 1, data_hdr = 16;
    if (version > 1) {  // v2+: total docs, compression type, data header start (BaseChunkForwardIndexReader.java:61-111)
      if (c.forward_bytes < 28) return fail(PHIP_ERR_INVALID, "column %s: chunk header truncated", c.name);
      total = (int32_t)be32(h + 16);
      comp = (int32_t)be32(h + 20);
      data_hdr = (int32_t)be32(h + 24);
    }  // v1: 4-int header, SNAPPY chunks, int offsets from byte 16
    // ChunkCompressionType (ChunkCompressionType.java:22): PASS_THROUGH 0, SNAPPY 1, ZSTANDARD 2, LZ4 3,
    // LZ4_LENGTH_PREFIXED 4, GZIP 5 -- all decoded on the GPU at load (load.hip, codec.h)
    if (comp < 0 || comp > 5)
      return fail(PHIP_ERR_INVALID, "column %s: unknown chunk compression type %d", c.name, comp);
    if (entry != type_width(c.data_type) || total != n || per_chunk <= 0 ||
        num_chunks != ceil_div(n, per_chunk) || (version < 1 || version > 5))
      return fail(PHIP_ERR_INVALID, "column %s: bad chunk header", c.name);
    // v4 = FixedBytePower2ChunkSVForwardIndexReader (ForwardIndexReaderFactory.java:113-117): chunk = doc >> shift
    if (version == 4 && (per_chunk & (per_chunk - 1)) != 0)
      return fail(PHIP_ERR_INVALID, "column %s: v4 chunk of %d docs is not a power of two", c.name, per_chunk);
    const int osz = version <= 2 ? 4 : 8;
    const uint64_t hdr_end = (uint64_t)data_hdr + (uint64_t)num_chunks * osz;
    if (data_hdr < (version > 1 ? 28 : 16) || hdr_end > c.forward_bytes)
      return fail(PHIP_ERR_INVALID, "column %s: chunk offsets truncated", c.name);
    void *p;
    int32_t rc = dev_alloc(seg, (uint64_t)std::max<int64_t>(n, 1) * entry + 16, &p);
    if (rc) return rc;
    cs.raw = p;
    auto chunk_off = [&](int32_t k) -> uint64_t { return osz == 4 ? be32(h + data_hdr + 4 * k) : be64(h + data_hdr + 8 * k); };
    if (comp == 0) {
      for (int32_t k = 0; k < num_chunks; k++) {
        uint64_t off = chunk_off(k);
        int64_t docs = std::min<int64_t>(per_chunk, n - (int64_t)k * per_chunk);
        if (off + (uint64_t)docs * entry > c.forward_bytes) return fail(PHIP_ERR_INVALID, "column %s: chunk %d overflow", c.name, k);
        HIP_TRY(hipMemcpyAsync((uint8_t *)p + (int64_t)k * per_chunk * entry, h + off, docs * entry,
                               hipMemcpyHostToDevice, st));
      }
      if (entry == 4) HIP_TRY(launch_bswap32((uint32_t *)p, n, st));
      else HIP_TRY(launch_bswap64((uint64_t *)p, n, st));
    } else if (num_chunks > 0) {
      // chunk k spans [offset_k, offset_{k+1}), the last one to the end of the buffer
      // (BaseChunkForwardIndexReader.decompressChunk, BaseChunkForwardIndexReader.java:204-232)
      std::vector<RawChunk> chunks(num_chunks);
      const uint64_t first = chunk_off(0);
      uint32_t max_c = 0, max_u = 0;
      for (int32_t k = 0; k < num_chunks; k++) {
        const uint64_t off = chunk_off(k), end = k + 1 < num_chunks ? chunk_off(k + 1) : c.forward_bytes;
        if (off < hdr_end || end < off || end > c.forward_bytes || end - off > (1u << 30))
          return fail(PHIP_ERR_INVALID, "column %s: chunk %d offsets out of order", c.name, k);
        const int64_t docs = std::min<int64_t>(per_chunk, n - (int64_t)k * per_chunk);
        chunks[k].src = off - first;
        chunks[k].dst = (uint64_t)k * per_chunk * entry;
        chunks[k].csize = (uint32_t)(end - off);
        chunks[k].usize = (uint32_t)(docs * entry);
        max_c = std::max(max_c, chunks[k].csize);
        max_u = std::max(max_u, chunks[k].usize);
      }
      const uint32_t out_cap = (uint32_t)round_up(max_u, 16);
      const uint32_t in_cap = (uint32_t)round_up(max_c + 8, 16);
      const size_t lds = out_cap + in_cap + chunk_decode_extra_lds(comp, (int32_t)out_cap);
      if (lds > 163840 - 1024)
        return fail(PHIP_ERR_UNSUPPORTED, "column %s: chunks of %u -> %u bytes exceed the 159 KiB LDS decode window",
                    c.name, max_c, max_u);
      const uint64_t blob_bytes = c.forward_bytes - first;
      void *blob, *table, *err;
      HIP_TRY(hipMalloc(&blob, blob_bytes + 16));
      temps.push_back(blob);
      HIP_TRY(hipMalloc(&table, sizeof(RawChunk) * num_chunks));
      temps.push_back(table);
      HIP_TRY(hipMalloc(&err, 4));
      temps.push_back(err);
      HIP_TRY(hipMemsetAsync(err, 0, 4, st));
      HIP_TRY(hipMemcpyAsync(blob, h + first, blob_bytes, hipMemcpyHostToDevice, st));
      HIP_TRY(hipMemcpyAsync(table, chunks.data(), sizeof(RawChunk) * num_chunks, hipMemcpyHostToDevice, st));
      HIP_TRY(launch_chunk_decode(comp, entry, (const uint8_t *)blob, (const RawChunk *)table, num_chunks,
                                  (int32_t)out_cap, (int32_t)in_cap, lds, (uint8_t *)p, (int32_t *)err, nullptr, st));
      int32_t bad = 0;
      HIP_TRY(hipMemcpyAsync(&bad, err, 4, hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
      if (bad) return fail(PHIP_ERR_INVALID, "column %s: malformed compressed chunk %d (type %d)", c.name, bad - 1, comp);
    }
    if (c.data_type == PHIP_TYPE_INT || c.data_type == PHIP_TYPE_LONG) {
      int64_t mm[2] = {INT64_MAX, INT64_MIN};
      void *dmm;
      HIP_TRY(hipMalloc(&dmm, 16));
      temps.push_back(dmm);
      HIP_TRY(hipMemcpyAsync(dmm, mm, 16, hipMemcpyHostToDevice, st));
      HIP_TRY(launch_minmax_i64(cs.raw, c.data_type, n, (int64_t *)dmm, st));
      HIP_TRY(hipMemcpyAsync(mm, dmm, 16, hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
      cs.vmin = n > 0 ? mm[0] : 0;
      cs.vmax = n > 0 ? mm[1] : 0;
      cs.has_range = true;
    }
  }
  if (c.null_vector != nullptr && c.null_vector_bytes > 0) {
    int32_t rc = load_null_vector(c, cs, seg, st);
    if (rc) return rc;
    if (cs.has_range && cs.raw != nullptr && cs.nulls != nullptr && n > 0) {
      // a raw key column's null docs hold the default null value: the null-key group-by keys the other values only
      int64_t mm[2] = {INT64_MAX, INT64_MIN};
      void *dmm;
      HIP_TRY(hipMalloc(&dmm, 16));
      temps.push_back(dmm);
      HIP_TRY(hipMemcpyAsync(dmm, mm, 16, hipMemcpyHostToDevice, st));
      HIP_TRY(launch_minmax_i64(cs.raw, c.data_type, n, (int64_t *)dmm, st, cs.nulls));
      HIP_TRY(hipMemcpyAsync(mm, dmm, 16, hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
      cs.nn_empty = mm[0] > mm[1];
      cs.nn_vmin = cs.nn_empty ? 0 : mm[0];
      cs.nn_vmax = cs.nn_empty ? 0 : mm[1];
    }
  }
  seg.by_name[cs.name] = (int)seg.cols.size();
  seg.cols.push_back(std::move(cs));
  return PHIP_OK;
}

// ================================================================================================
// query execution
// ================================================================================================
namespace {

struct Blob {  // host staging for one H2D copy; device address = base + offset
  std::vector<uint8_t> data;
  size_t add(const void *p, size_t n, size_t align = 16) {
    size_t off = round_up((int64_t)data.size(), (int64_t)align);
    data.resize(off + n);
    if (n) memcpy(data.data() + off, p, n);
    return off;
  }
  size_t reserve(size_t n, size_t align = 16) {
    size_t off = round_up((int64_t)data.size(), (int64_t)align);
    data.resize(off + n);
    return off;
  }
};

struct ResultImpl {
  phip_result pub;
  std::vector<double> values;
  std::vector<int64_t> longs;
  std::vector<uint8_t> hll;
  std::vector<int32_t> keys;
  std::vector<int32_t> exact;
  std::vector<std::shared_ptr<Device::Remap>> dicts;
  std::vector<uint64_t> sel_values;  // selection: [num_select][num_rows]
  std::vector<int32_t> sel_types;
  std::vector<std::shared_ptr<Device::Remap>> sel_dicts;  // per select column: query-global dictionary (STRING)
  std::vector<int64_t> seg_docs;  // per segment: matched docs summed over the filter programs
  std::vector<int64_t> prog_docs;  // per filter program: matched docs summed over the segments
};

// validate a preorder subtree; returns index after it or -1
int validate_tree(const phip_filter_node *nodes, int begin, int end, int idx, int depth, int ncols,
                  std::vector<int> &next, std::string &err) {
  if (idx >= end) {
    err = "filter tree truncated";
    return -1;
  }
  if (depth > 64) {
    err = "filter tree deeper than supported";
    return -1;
  }
  const phip_filter_node &n = nodes[idx];
  int after;
  switch (n.op) {
    case PHIP_NODE_LEAF:
      if (n.leaf_kind < PHIP_LEAF_MATCH_ALL || n.leaf_kind > PHIP_LEAF_NULL) {
        err = "bad leaf kind";
        return -1;
      }
      if (n.leaf_kind >= PHIP_LEAF_DICT_RANGE && n.leaf_kind != PHIP_LEAF_DOC_RANGES &&
          (n.column < 0 || n.column >= ncols)) {
        err = "leaf column out of range";
        return -1;
      }
      if (n.leaf_kind == PHIP_LEAF_RAW_RANGE &&
          (n.ids == nullptr || n.count * 4 != (int32_t)sizeof(phip_raw_range))) {
        err = "raw range leaf needs a phip_raw_range";
        return -1;
      }
      if (n.leaf_kind == PHIP_LEAF_RAW_SET && (n.count % 2 != 0 || n.count > 2 * (1 << 20))) {
        err = "raw set leaf: count must be 2 x (values <= 2^20)";
        return -1;
      }
      if ((n.leaf_kind == PHIP_LEAF_RAW_STRING_RANGE && (n.ids == nullptr || n.count < 4 || n.count > (1 << 24))) ||
          (n.leaf_kind == PHIP_LEAF_RAW_STRING_SET && (n.ids == nullptr || n.count < 2 || n.count > (1 << 26)))) {
        err = "raw STRING leaf: count words of bounds / values (<= 2^24 / 2^26)";
        return -1;
      }
      if ((n.leaf_kind == PHIP_LEAF_DICT_SET || n.leaf_kind == PHIP_LEAF_INVERTED || n.leaf_kind == PHIP_LEAF_DOC_RANGES ||
           n.leaf_kind == PHIP_LEAF_RAW_SET) &&
          n.count > 0 && n.ids == nullptr) {
        err = "leaf ids missing";
        return -1;
      }
      after = idx + 1;
      break;
    case PHIP_NODE_NOT:
      after = validate_tree(nodes, begin, end, idx + 1, depth + 1, ncols, next, err);
      if (after < 0) return -1;
      break;
    case PHIP_NODE_AND:
    case PHIP_NODE_OR: {
      if (n.num_children < 1) {
        err = "AND/OR without children";
        return -1;
      }
      int c = idx + 1;
      for (int k = 0; k < n.num_children; k++) {
        c = validate_tree(nodes, begin, end, c, depth + 1, ncols, next, err);
        if (c < 0) return -1;
      }
      after = c;
      break;
    }
    default:
      err = "bad node op";
      return -1;
  }
  next[idx - begin] = after;
  return after;
}

std::string dict_key(const ColumnStore &c) { return std::string((const char *)c.host_dict.data(), c.host_dict.size()); }

// Total order of dictionary values as the reference sorts them: numbers by value (FLOAT / DOUBLE in
// Float.compare / Double.compare order: -0.0 < 0.0, NaN last), strings as '\0'-padded bytes (memcmp order ==
// String.compareTo for ASCII / BMP UTF-8).
static int compare_value(int32_t type, const uint8_t *a, const uint8_t *b, int width) {
  auto ord = [](uint64_t u, int bits) {  // order-preserving unsigned image of an IEEE value
    const uint64_t sign = 1ull << (bits - 1);
    return (u & sign) ? ~u & (bits == 64 ? ~0ull : 0xffffffffull) : u | sign;
  };
  switch (type) {
    case PHIP_TYPE_INT: {
      int32_t x, y;
      memcpy(&x, a, 4);
      memcpy(&y, b, 4);
      return x < y ? -1 : x > y;
    }
    case PHIP_TYPE_LONG: {
      int64_t x, y;
      memcpy(&x, a, 8);
      memcpy(&y, b, 8);
      return x < y ? -1 : x > y;
    }
    case PHIP_TYPE_FLOAT: {
      uint32_t x, y;
      memcpy(&x, a, 4);
      memcpy(&y, b, 4);
      const uint64_t ox = ord(x, 32), oy = ord(y, 32);
      return ox < oy ? -1 : ox > oy;
    }
    case PHIP_TYPE_DOUBLE: {
      uint64_t x, y;
      memcpy(&x, a, 8);
      memcpy(&y, b, 8);
      const uint64_t ox = ord(x, 64), oy = ord(y, 64);
      return ox < oy ? -1 : ox > oy;
    }
    default: {
      const int c = memcmp(a, b, width);
      return c < 0 ? -1 : c > 0;
    }
  }
}

// A raw FLOAT / DOUBLE group-by column (keys.hip): the sorted distinct values over the segments become the remap's
// dictionary (values, card) and each segment gets a doc-order int32 id column (Remap.ids -> DevCol.gb_ids). Built on
// the device's setup stream once per (column, segments), cached with the other remaps.
static int32_t raw_real_key_ids(Device &dev, const std::vector<Segment *> &segs, const std::vector<int> &colidx,
                                const std::string &name, int32_t type, Device::Remap &r) {
  hipStream_t st = dev.stream;
  std::vector<void *> tmp;  // freed on every return
  struct Free {
    std::vector<void *> &v;
    ~Free() {
      for (void *p : v) (void)hipFree(p);
    }
  } free_tmp{tmp};
  auto alloc = [&](size_t bytes, void **p) -> int32_t {
    HIP_TRY(hipMalloc(p, std::max<size_t>(bytes, 16)));
    tmp.push_back(*p);
    return PHIP_OK;
  };
  std::vector<uint64_t *> seg_uniq(segs.size(), nullptr);
  std::vector<int64_t> seg_u(segs.size(), 0);
  int64_t total = 0;
  for (size_t i = 0; i < segs.size(); i++) {
    const ColumnStore &c = segs[i]->cols[colidx[i]];
    if (!no_dict(c) || c.fwd_kind != PHIP_FWD_RAW_CHUNK || c.type != type)
      return fail(PHIP_ERR_UNSUPPORTED, "group-by on column %s: raw in some segments only", name.c_str());
    const int64_t n = segs[i]->num_docs;
    if (n <= 0) continue;
    if (n > INT32_MAX) return fail(PHIP_ERR_UNSUPPORTED, "group-by on raw column %s: segment over 2^31 docs", name.c_str());
    void *img, *srt, *uq, *cnt, *scratch;
    size_t sb = 0;
    int32_t rc;
    if ((rc = alloc((size_t)n * 8, &img)) || (rc = alloc((size_t)n * 8, &srt)) || (rc = alloc((size_t)n * 8, &uq)) ||
        (rc = alloc(8, &cnt)))
      return rc;
    HIP_TRY(launch_sort_unique_u64(nullptr, &sb, nullptr, nullptr, nullptr, nullptr, n, st));
    if ((rc = alloc(sb, &scratch))) return rc;
    HIP_TRY(launch_raw_images(c.raw, type, n, (uint64_t *)img, st));
    HIP_TRY(launch_sort_unique_u64(scratch, &sb, (uint64_t *)img, (uint64_t *)srt, (uint64_t *)uq, (int64_t *)cnt, n, st));
    HIP_TRY(hipMemcpyAsync(&seg_u[i], cnt, 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    seg_uniq[i] = (uint64_t *)uq;
    total += seg_u[i];
  }
  void *all, *srt, *guniq, *cnt, *scratch;
  size_t sb = 0;
  int32_t rc;
  if ((rc = alloc((size_t)total * 8, &all)) || (rc = alloc((size_t)total * 8, &srt)) ||
      (rc = alloc((size_t)total * 8, &guniq)) || (rc = alloc(8, &cnt)))
    return rc;
  int64_t off = 0;
  for (size_t i = 0; i < segs.size(); i++) {
    if (!seg_u[i]) continue;
    HIP_TRY(hipMemcpyAsync((uint64_t *)all + off, seg_uniq[i], (size_t)seg_u[i] * 8, hipMemcpyDeviceToDevice, st));
    off += seg_u[i];
  }
  HIP_TRY(launch_sort_unique_u64(nullptr, &sb, nullptr, nullptr, nullptr, nullptr, total, st));
  if ((rc = alloc(sb, &scratch))) return rc;
  int64_t u = 0;
  HIP_TRY(launch_sort_unique_u64(scratch, &sb, (uint64_t *)all, (uint64_t *)srt, (uint64_t *)guniq, (int64_t *)cnt, total, st));
  HIP_TRY(hipMemcpyAsync(&u, cnt, 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (u > INT32_MAX) return fail(PHIP_ERR_UNSUPPORTED, "group-by on raw column %s: %lld distinct values", name.c_str(), (long long)u);
  r.ids.assign(segs.size(), nullptr);
  for (size_t i = 0; i < segs.size(); i++) {
    const int64_t n = segs[i]->num_docs;
    void *p;
    HIP_TRY(hipMalloc(&p, std::max<size_t>((size_t)n * 4, 16)));
    r.ids[i] = (int32_t *)p;  // owned by r from here
    HIP_TRY(launch_raw_key_ids(segs[i]->cols[colidx[i]].raw, type, n, (const uint64_t *)guniq, u, (int32_t *)p, st));
  }
  std::vector<uint64_t> img((size_t)u);
  if (u) HIP_TRY(hipMemcpyAsync(img.data(), guniq, (size_t)u * 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  const int w = type_width(type);
  r.values.assign((size_t)u * w, 0);
  for (int64_t i = 0; i < u; i++) {  // the images back to values (keys.hip f64_order_image inverted)
    const uint64_t k = img[(size_t)i];
    const uint64_t b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
    double d;
    memcpy(&d, &b, 8);
    if (w == 4) {
      const float f = (float)d;
      memcpy(r.values.data() + 4 * i, &f, 4);
    } else {
      memcpy(r.values.data() + 8 * i, &d, 8);
    }
  }
  r.type = type;
  r.width = w;
  r.card = (int32_t)u;
  r.dev.assign(segs.size(), nullptr);
  return PHIP_OK;
}

// Raw STRING keys (the no-dictionary generators key a String by its value): per segment the docs' 64-bit hashes are
// sorted and made unique on the device with a representative doc each, every doc is compared with its representative
// (keys.hip), the representatives' bytes come to the host, which checks equal hashes across segments hold equal
// strings, sorts the distinct strings bytewise (the STRING dictionaries' padded order) and maps each segment's hashes
// to global ids for the doc-order id column. A hash collision (two distinct strings, one 64-bit hash -- inside a segment
// or across segments) takes raw_string_key_ids_exact instead.
static int32_t raw_string_key_ids_exact(Device &dev, const std::vector<Segment *> &segs, const std::vector<int> &colidx,
                                        const std::string &name, Device::Remap &r);
static constexpr int32_t kStrCollision = -101;  // raw_string_key_ids_hashed: the exact path decides

static int32_t raw_string_key_ids_hashed(Device &dev, const std::vector<Segment *> &segs, const std::vector<int> &colidx,
                                         const std::string &name, Device::Remap &r);

static int32_t raw_string_key_ids(Device &dev, const std::vector<Segment *> &segs, const std::vector<int> &colidx,
                                  const std::string &name, Device::Remap &r) {
  static int hash_bits_set = 64;  // (under the device mutex, as every remap build)
  const char *hb = getenv("PHIP_STR_HASH_BITS");  // test hook: fewer hash bits, so collisions occur
  const int hash_bits = hb ? atoi(hb) : 64;
  if (hash_bits != hash_bits_set) {
    HIP_TRY(set_str_hash_bits(hash_bits));
    hash_bits_set = hash_bits;
  }
  const char *ex = getenv("PHIP_STR_KEYS_EXACT");  // test override: the exact path always
  int32_t rc = ex && atoi(ex) != 0 ? kStrCollision : raw_string_key_ids_hashed(dev, segs, colidx, name, r);
  if (rc == kStrCollision) {
    r.ids.clear();
    r.values.clear();
    rc = raw_string_key_ids_exact(dev, segs, colidx, name, r);
  }
  return rc;
}

// Exact raw STRING keys on the host: every segment's values and offsets copied out, the distinct strings found with a
// hash map of the bytes themselves (no fixed-width hash to collide), sorted bytewise, each doc's id copied back as the
// doc-order id column. A host pass over the column's bytes -- taken only when the device hashes collided.
static int32_t raw_string_key_ids_exact(Device &dev, const std::vector<Segment *> &segs, const std::vector<int> &colidx,
                                        const std::string &name, Device::Remap &r) {
  hipStream_t st = dev.stream;
  std::unordered_map<std::string, int32_t> first;  // string -> index in `distinct`
  std::vector<const std::string *> distinct;
  std::vector<std::vector<int32_t>> doc_ids(segs.size());
  for (size_t i = 0; i < segs.size(); i++) {
    const ColumnStore &c = segs[i]->cols[colidx[i]];
    if (!no_dict(c) || c.fwd_kind != PHIP_FWD_RAW_CHUNK || c.type != PHIP_TYPE_STRING || c.str_off == nullptr)
      return fail(PHIP_ERR_UNSUPPORTED, "group-by on column %s: raw in some segments only", name.c_str());
    const int64_t n = segs[i]->num_docs;
    if (n <= 0) continue;
    std::vector<uint64_t> off((size_t)n + 1);
    HIP_TRY(hipMemcpyAsync(off.data(), c.str_off, off.size() * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    std::vector<uint8_t> bytes(off[(size_t)n]);
    if (!bytes.empty()) HIP_TRY(hipMemcpyAsync(bytes.data(), c.raw, bytes.size(), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    doc_ids[i].resize((size_t)n);
    for (int64_t d = 0; d < n; d++) {
      std::string v((const char *)bytes.data() + off[(size_t)d], (size_t)(off[(size_t)d + 1] - off[(size_t)d]));
      auto ins = first.emplace(std::move(v), (int32_t)distinct.size());
      if (ins.second) {
        if (distinct.size() >= (size_t)INT32_MAX)
          return fail(PHIP_ERR_UNSUPPORTED, "group-by on raw column %s: over 2^31 distinct values", name.c_str());
        distinct.push_back(&ins.first->first);
      }
      doc_ids[i][(size_t)d] = ins.first->second;
    }
  }
  std::vector<int32_t> order(distinct.size());
  for (size_t g = 0; g < order.size(); g++) order[g] = (int32_t)g;
  std::sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return *distinct[a] < *distinct[b]; });
  std::vector<int32_t> rank(distinct.size());
  size_t width = 1;
  for (size_t g = 0; g < order.size(); g++) {
    rank[(size_t)order[g]] = (int32_t)g;
    width = std::max(width, distinct[(size_t)order[g]]->size());
  }
  r.values.assign(distinct.size() * width, 0);
  for (size_t g = 0; g < order.size(); g++)
    memcpy(r.values.data() + g * width, distinct[(size_t)order[g]]->data(), distinct[(size_t)order[g]]->size());
  r.ids.assign(segs.size(), nullptr);
  for (size_t i = 0; i < segs.size(); i++) {
    const int64_t n = segs[i]->num_docs;
    void *p;
    HIP_TRY(hipMalloc(&p, std::max<size_t>((size_t)n * 4, 16)));
    r.ids[i] = (int32_t *)p;  // owned by r from here
    if (n <= 0) continue;
    for (auto &id : doc_ids[i]) id = rank[(size_t)id];
    HIP_TRY(hipMemcpyAsync(p, doc_ids[i].data(), (size_t)n * 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipStreamSynchronize(st));
  }
  r.type = PHIP_TYPE_STRING;
  r.width = (int32_t)width;
  r.card = (int32_t)distinct.size();
  r.dev.assign(segs.size(), nullptr);
  return PHIP_OK;
}

static int32_t raw_string_key_ids_hashed(Device &dev, const std::vector<Segment *> &segs, const std::vector<int> &colidx,
                                         const std::string &name, Device::Remap &r) {
  hipStream_t st = dev.stream;
  std::vector<void *> tmp;
  struct Free {
    std::vector<void *> &v;
    ~Free() {
      for (void *p : v) (void)hipFree(p);
    }
  } free_tmp{tmp};
  auto alloc = [&](size_t bytes, void **p) -> int32_t {
    HIP_TRY(hipMalloc(p, std::max<size_t>(bytes, 16)));
    tmp.push_back(*p);
    return PHIP_OK;
  };
  void *flag;
  int32_t rc;
  if ((rc = alloc(8, &flag))) return rc;
  HIP_TRY(hipMemsetAsync(flag, 0, 8, st));
  std::vector<uint64_t *> seg_uniq(segs.size(), nullptr);
  std::vector<int64_t> seg_u(segs.size(), 0);
  std::vector<std::vector<uint64_t>> seg_hash(segs.size());
  std::vector<std::vector<std::string>> seg_str(segs.size());
  for (size_t i = 0; i < segs.size(); i++) {
    const ColumnStore &c = segs[i]->cols[colidx[i]];
    if (!no_dict(c) || c.fwd_kind != PHIP_FWD_RAW_CHUNK || c.type != PHIP_TYPE_STRING || c.str_off == nullptr)
      return fail(PHIP_ERR_UNSUPPORTED, "group-by on column %s: raw in some segments only", name.c_str());
    const int64_t n = segs[i]->num_docs;
    if (n <= 0) continue;
    if (n > INT32_MAX) return fail(PHIP_ERR_UNSUPPORTED, "group-by on raw column %s: segment over 2^31 docs", name.c_str());
    const uint8_t *bytes = (const uint8_t *)c.raw;
    void *h, *d, *hs, *ds, *uq, *rp, *cnt, *scratch;
    size_t sb = 0;
    if ((rc = alloc((size_t)n * 8, &h)) || (rc = alloc((size_t)n * 4, &d)) || (rc = alloc((size_t)n * 8, &hs)) ||
        (rc = alloc((size_t)n * 4, &ds)) || (rc = alloc((size_t)n * 8, &uq)) || (rc = alloc((size_t)n * 4, &rp)) ||
        (rc = alloc(8, &cnt)))
      return rc;
    HIP_TRY(launch_str_hash_unique(nullptr, &sb, bytes, c.str_off, n, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                                   nullptr, st));
    if ((rc = alloc(sb, &scratch))) return rc;
    HIP_TRY(launch_str_hash_unique(scratch, &sb, bytes, c.str_off, n, (uint64_t *)h, (int32_t *)d, (uint64_t *)hs,
                                   (int32_t *)ds, (uint64_t *)uq, (int32_t *)rp, (int64_t *)cnt, st));
    int64_t u = 0;
    HIP_TRY(hipMemcpyAsync(&u, cnt, 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    HIP_TRY(launch_str_verify(bytes, c.str_off, n, (const uint64_t *)uq, (const int32_t *)rp, u, (int32_t *)flag, st));
    void *lens, *doff;
    if ((rc = alloc((size_t)u * 4, &lens)) || (rc = alloc((size_t)u * 8, &doff))) return rc;
    HIP_TRY(launch_str_rep_lens(c.str_off, (const int32_t *)rp, u, (uint32_t *)lens, st));
    std::vector<uint32_t> hl((size_t)u);
    std::vector<uint64_t> ho((size_t)u + 1, 0);
    seg_hash[i].resize((size_t)u);
    HIP_TRY(hipMemcpyAsync(hl.data(), lens, (size_t)u * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(seg_hash[i].data(), uq, (size_t)u * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    for (int64_t j = 0; j < u; j++) ho[(size_t)j + 1] = ho[(size_t)j] + hl[(size_t)j];
    void *dst;
    if ((rc = alloc(ho[(size_t)u], &dst))) return rc;
    HIP_TRY(hipMemcpyAsync(doff, ho.data(), (size_t)u * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(launch_str_rep_bytes(bytes, c.str_off, (const int32_t *)rp, u, (const uint64_t *)doff, (uint8_t *)dst, st));
    std::vector<uint8_t> hb(ho[(size_t)u]);
    int32_t collided = 0;
    if (!hb.empty()) HIP_TRY(hipMemcpyAsync(hb.data(), dst, hb.size(), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(&collided, flag, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (collided) return kStrCollision;  // (two strings of this segment share a hash)
    seg_str[i].resize((size_t)u);
    for (int64_t j = 0; j < u; j++)
      seg_str[i][(size_t)j].assign((const char *)hb.data() + ho[(size_t)j], hl[(size_t)j]);
    seg_uniq[i] = (uint64_t *)uq;
    seg_u[i] = u;
  }
  // equal hashes hold equal strings across segments; the distinct strings sorted bytewise are the key space
  std::unordered_map<uint64_t, const std::string *> by_hash;
  std::vector<const std::string *> distinct;
  for (size_t i = 0; i < segs.size(); i++)
    for (size_t j = 0; j < seg_str[i].size(); j++) {
      auto ins = by_hash.emplace(seg_hash[i][j], &seg_str[i][j]);
      if (!ins.second) {
        if (*ins.first->second != seg_str[i][j]) return kStrCollision;  // (two segments' strings share a hash)
      } else {
        distinct.push_back(&seg_str[i][j]);
      }
    }
  if ((int64_t)distinct.size() > INT32_MAX)
    return fail(PHIP_ERR_UNSUPPORTED, "group-by on raw column %s: %zu distinct values", name.c_str(), distinct.size());
  std::sort(distinct.begin(), distinct.end(), [](const std::string *a, const std::string *b) { return *a < *b; });
  std::unordered_map<const std::string *, int32_t> rank;
  size_t width = 1;
  for (size_t g = 0; g < distinct.size(); g++) {
    rank[distinct[g]] = (int32_t)g;
    width = std::max(width, distinct[g]->size());
  }
  r.values.assign(distinct.size() * width, 0);
  for (size_t g = 0; g < distinct.size(); g++) memcpy(r.values.data() + g * width, distinct[g]->data(), distinct[g]->size());
  r.ids.assign(segs.size(), nullptr);
  for (size_t i = 0; i < segs.size(); i++) {
    const int64_t n = segs[i]->num_docs;
    void *p;
    HIP_TRY(hipMalloc(&p, std::max<size_t>((size_t)n * 4, 16)));
    r.ids[i] = (int32_t *)p;  // owned by r from here
    if (n <= 0) continue;
    std::vector<int32_t> map(seg_str[i].size());
    for (size_t j = 0; j < map.size(); j++) map[j] = rank.at(by_hash.at(seg_hash[i][j]));
    void *dm;
    if ((rc = alloc(map.size() * 4, &dm))) return rc;
    HIP_TRY(hipMemcpyAsync(dm, map.data(), map.size() * 4, hipMemcpyHostToDevice, st));
    const ColumnStore &c = segs[i]->cols[colidx[i]];
    HIP_TRY(launch_raw_str_ids((const uint8_t *)c.raw, c.str_off, n, seg_uniq[i], seg_u[i], (const int32_t *)dm,
                               (int32_t *)p, st));
    HIP_TRY(hipStreamSynchronize(st));  // (map freed with tmp after the launch completes)
  }
  r.type = PHIP_TYPE_STRING;
  r.width = (int32_t)width;
  r.card = (int32_t)distinct.size();
  r.dev.assign(segs.size(), nullptr);
  return PHIP_OK;
}

// Tuple keys for a group-by whose mixed-radix key space exceeds 2^62: the columns' query-global ids (nulls as the
// column's null id) packed into <= 4 u64 words per doc, ranked per segment and then across segments (keys.hip), as
// one virtual column: card = the distinct tuples, doc-order ids per segment, the tuples' words kept for decoding.
static int32_t build_tuple_keys(Device &dev, const std::vector<Segment *> &segs,
                                const std::vector<std::vector<int>> &colidx, const int32_t *gb_cols, int K,
                                const std::vector<std::shared_ptr<Device::Remap>> &dicts,
                                const std::vector<int64_t> &radix, std::vector<int32_t> &word,
                                std::vector<uint64_t> &stride, std::shared_ptr<Device::Remap> &out) {
  // columns into words: mixed radix per word while the product fits u64
  word.assign(K, 0);
  stride.assign(K, 1);
  int W = 1;
  long double prod = 1;
  for (int k = 0; k < K; k++) {
    if (prod * (long double)radix[k] > 18446744073709551615.0L) {
      W++;
      prod = 1;
    }
    word[k] = W - 1;
    stride[k] = (uint64_t)prod;
    prod *= (long double)radix[k];
  }
  if (W > kMaxTupleWords || K > kMaxTupleCols)
    return fail(PHIP_ERR_UNSUPPORTED, "group-by tuple keys: %d words over %d columns", W, K);
  std::string key = "tuple";
  for (int k = 0; k < K; k++) {
    char buf[64];
    snprintf(buf, sizeof buf, "|%d@%p#%lld", gb_cols[k], (const void *)dicts[k].get(), (long long)radix[k]);
    key += buf;
  }
  for (auto *sg : segs) key += ":" + std::to_string(sg->handle);
  auto it = dev.remaps.find(key);
  if (it != dev.remaps.end()) {
    out = it->second;
    return PHIP_OK;
  }
  hipStream_t st = dev.stream;
  std::vector<void *> tmp;
  struct Free {
    std::vector<void *> &v;
    ~Free() {
      for (void *p : v) (void)hipFree(p);
    }
  } free_tmp{tmp};
  auto alloc = [&](size_t bytes, void **p) -> int32_t {
    HIP_TRY(hipMalloc(p, std::max<size_t>(bytes, 16)));
    tmp.push_back(*p);
    return PHIP_OK;
  };
  auto r = std::make_shared<Device::Remap>();
  const size_t S = segs.size();
  std::vector<int32_t *> local(S, nullptr);
  std::vector<uint64_t *> seg_uniq(S, nullptr);
  std::vector<int64_t> seg_u(S, 0);
  int64_t total = 0;
  int32_t rc;
  for (size_t i = 0; i < S; i++) {
    const int64_t n = segs[i]->num_docs;
    if (n <= 0) continue;
    if (n > INT32_MAX) return fail(PHIP_ERR_UNSUPPORTED, "group-by tuple keys: segment over 2^31 docs");
    TupleCols tc{};
    tc.k = K;
    tc.w = W;
    for (int k = 0; k < K; k++) {
      const ColumnStore &c = segs[i]->cols[colidx[i][gb_cols[k]]];
      const Device::Remap &d = *dicts[k];
      TupleCol &t = tc.cols[k];
      t.word = word[k];
      t.stride = stride[k];
      t.null_id = d.card;
      t.nulls = radix[k] > d.card ? c.nulls : nullptr;
      if (!d.ids.empty()) {
        t.ids = d.ids[i];
      } else if (d.raw) {
        t.raw = c.raw;
        t.type = c.type;
        t.base = d.raw_base;
      } else {
        t.words = c.words;
        t.bits = c.bits;
        t.remap = d.dev[i];
      }
    }
    void *w, *ids, *uq, *scratch;
    size_t sb = 0;
    if ((rc = alloc((size_t)n * 8 * W, &w)) || (rc = alloc((size_t)n * 4, &ids)) || (rc = alloc((size_t)n * 8 * W, &uq)))
      return rc;
    HIP_TRY(launch_tuple_words(tc, n, (uint64_t *)w, st));
    HIP_TRY(launch_tuple_rank(nullptr, &sb, nullptr, W, n, nullptr, nullptr, 0, nullptr, st));
    if ((rc = alloc(sb, &scratch))) return rc;
    int64_t u = 0;
    HIP_TRY(launch_tuple_rank(scratch, &sb, (const uint64_t *)w, W, n, (int32_t *)ids, (uint64_t *)uq, n, &u, st));
    local[i] = (int32_t *)ids;
    seg_uniq[i] = (uint64_t *)uq;
    seg_u[i] = u;
    total += u;
  }
  // the segments' distinct tuples, ranked together
  void *all, *gids, *guniq, *scratch;
  size_t sb = 0;
  if ((rc = alloc((size_t)std::max<int64_t>(total, 1) * 8 * W, &all)) || (rc = alloc((size_t)total * 4, &gids)) ||
      (rc = alloc((size_t)std::max<int64_t>(total, 1) * 8 * W, &guniq)))
    return rc;
  int64_t off = 0;
  for (size_t i = 0; i < S; i++) {
    for (int j = 0; j < W && seg_u[i]; j++)
      HIP_TRY(hipMemcpyAsync((uint64_t *)all + (int64_t)j * total + off, seg_uniq[i] + (int64_t)j * segs[i]->num_docs,
                             (size_t)seg_u[i] * 8, hipMemcpyDeviceToDevice, st));
    off += seg_u[i];
  }
  HIP_TRY(launch_tuple_rank(nullptr, &sb, nullptr, W, total, nullptr, nullptr, 0, nullptr, st));
  if ((rc = alloc(sb, &scratch))) return rc;
  int64_t U = 0;
  HIP_TRY(launch_tuple_rank(scratch, &sb, (const uint64_t *)all, W, total, (int32_t *)gids, (uint64_t *)guniq, total, &U, st));
  if (U > INT32_MAX) return fail(PHIP_ERR_UNSUPPORTED, "group-by tuple keys: %lld distinct tuples", (long long)U);
  r->ids.assign(S, nullptr);
  off = 0;
  for (size_t i = 0; i < S; i++) {
    const int64_t n = segs[i]->num_docs;
    void *p;
    HIP_TRY(hipMalloc(&p, std::max<size_t>((size_t)std::max<int64_t>(n, 0) * 4, 16)));
    r->ids[i] = (int32_t *)p;  // owned by r from here
    if (n > 0) HIP_TRY(launch_gather_ids(local[i], (const int32_t *)gids + off, n, (int32_t *)p, st));
    off += seg_u[i];
  }
  r->tuples.resize((size_t)U * W);
  for (int j = 0; j < W && U; j++)
    HIP_TRY(hipMemcpyAsync(r->tuples.data() + (size_t)j * U, (const uint64_t *)guniq + (int64_t)j * total, (size_t)U * 8,
                           hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  r->tuple_w = W;
  r->type = PHIP_TYPE_INT;
  r->card = (int32_t)U;
  r->dev.assign(S, nullptr);
  dev.remaps[key] = r;
  out = r;
  return PHIP_OK;
}

// Query-global dictionary of one group-by column across the query's segments: the
// node-global dictionary registered for the column (phip_global_dictionary, multi-GPU servers), else the
// sorted union of the segments' dictionaries. Per segment a dict-id -> global-id map in HBM (nullptr when
// the segment's dictionary IS the global one).
// (skip_nulls: a null-key column -- a raw column's id range then covers its non-null values only)
// The node plan being prepared on this thread (node_plan_create): its group-by columns' node-global dictionaries.
static thread_local const NodeDicts *tl_node_dicts = nullptr;
// ... and the docs of the whole node plan (0: not a part). A part sizes a hash table for every doc of the node, so the
// root's table can take the other parts' groups (node.cpp exchange_hash) and every part decides dense vs hash alike.
static thread_local int64_t tl_node_docs = 0;

int32_t build_remap(Device &dev, const std::vector<Segment *> &segs, const std::vector<int> &colidx,
                    const std::string &name, std::shared_ptr<Device::Remap> &out, bool skip_nulls = false) {
  auto git = dev.globals.find(name);
  const Device::GlobalDict *gd = git == dev.globals.end() ? nullptr : &git->second;
  // a node plan's part (node_plan_create): the column keyed by the node plan's own union dictionary
  Device::GlobalDict node_gd;
  const bool node = tl_node_dicts != nullptr && tl_node_dicts->count(name) > 0;
  if (node) {
    const NodeDict &nd = tl_node_dicts->at(name);
    node_gd.type = nd.type;
    node_gd.card = nd.card;
    node_gd.width = nd.width;
    node_gd.gen = nd.gen;
    node_gd.values = nd.values;
    gd = &node_gd;
  }
  std::string key = name;
  if (skip_nulls) key += "#nn";
  if (gd) key += (node ? "@n" : "@g") + std::to_string(gd->gen);
  for (auto *s : segs) key += ":" + std::to_string(s->handle);
  auto it = dev.remaps.find(key);
  if (it != dev.remaps.end()) {
    out = it->second;
    return PHIP_OK;
  }
  auto r = std::make_shared<Device::Remap>();
  const ColumnStore &c0 = segs[0]->cols[colidx[0]];
  const int32_t type = c0.type;
  r->type = type;
  r->global = gd != nullptr;
  int width = type == PHIP_TYPE_STRING ? c0.string_width : type_width(type);
  if (no_dict(c0) && c0.fwd_kind == PHIP_FWD_RAW_CHUNK && (type == PHIP_TYPE_INT || type == PHIP_TYPE_LONG)) {
    // A raw INT / LONG column (NoDictionarySingleColumnGroupKeyGenerator / NoDictionaryMultiColumnGroupKeyGenerator,
    // DefaultGroupByExecutor.java:106-116): its values themselves are the key dimension -- id = value - min over the
    // query's segments (the load-time value ranges), value order = id order -- and a result's dictionary holds only
    // the values its groups use (execute_plan). No global dictionary: a multi-GPU merge takes the record path.
    if (gd) return fail(PHIP_ERR_INVALID, "column %s is raw: it has no global dictionary", name.c_str());
    int64_t lo = INT64_MAX, hi = INT64_MIN;
    for (size_t i = 0; i < segs.size(); i++) {
      const ColumnStore &c = segs[i]->cols[colidx[i]];
      if (!no_dict(c) || c.fwd_kind != PHIP_FWD_RAW_CHUNK || c.type != type)
        return fail(PHIP_ERR_UNSUPPORTED, "group-by on column %s: raw in some segments only", name.c_str());
      if (!c.has_range) return fail(PHIP_ERR_UNSUPPORTED, "group-by on raw column %s without a value range", name.c_str());
      if (segs[i]->num_docs == 0) continue;
      if (skip_nulls && c.nulls != nullptr) {  // (the non-null values' range)
        if (c.nn_empty) continue;
        lo = std::min(lo, c.nn_vmin);
        hi = std::max(hi, c.nn_vmax);
        continue;
      }
      lo = std::min(lo, c.vmin);
      hi = std::max(hi, c.vmax);
    }
    if (lo > hi) lo = hi = 0;
    if ((long double)hi - (long double)lo + 1 > (long double)INT32_MAX)
      return fail(PHIP_ERR_UNSUPPORTED, "group-by on raw column %s: value range above 2^31", name.c_str());
    r->raw = true;
    r->raw_base = lo;
    r->card = (int32_t)(hi - lo + 1);
    r->dev.assign(segs.size(), nullptr);
    dev.remaps[key] = r;
    out = r;
    return PHIP_OK;
  }
  if (no_dict(c0) && c0.fwd_kind == PHIP_FWD_RAW_CHUNK && (type == PHIP_TYPE_FLOAT || type == PHIP_TYPE_DOUBLE)) {
    if (gd) return fail(PHIP_ERR_INVALID, "column %s is raw: it has no global dictionary", name.c_str());
    int32_t rc = raw_real_key_ids(dev, segs, colidx, name, type, *r);
    if (rc) return rc;
    dev.remaps[key] = r;
    out = r;
    return PHIP_OK;
  }
  if (no_dict(c0) && c0.fwd_kind == PHIP_FWD_RAW_CHUNK && type == PHIP_TYPE_STRING) {
    if (gd) return fail(PHIP_ERR_INVALID, "column %s is raw: it has no global dictionary", name.c_str());
    int32_t rc = raw_string_key_ids(dev, segs, colidx, name, *r);
    if (rc) return rc;
    dev.remaps[key] = r;
    out = r;
    return PHIP_OK;
  }
  for (size_t i = 0; i < segs.size(); i++) {
    const ColumnStore &c = segs[i]->cols[colidx[i]];
    if (no_dict(c)) return fail(PHIP_ERR_UNSUPPORTED, "group-by on raw column %s", name.c_str());
    if (c.type != type) return fail(PHIP_ERR_INVALID, "column %s has different types across segments", name.c_str());
    if (type == PHIP_TYPE_STRING) width = std::max(width, c.string_width);
  }
  if (gd && gd->type != type)
    return fail(PHIP_ERR_INVALID, "global dictionary of column %s has type %d, the segments %d", name.c_str(), gd->type, type);
  if (gd && type == PHIP_TYPE_STRING) width = std::max(width, gd->width);
  const int ew = width;  // bytes per value in the comparable LE / padded form
  r->width = type == PHIP_TYPE_STRING ? width : 0;
  auto seg_values = [&](const ColumnStore &c) {
    std::vector<uint8_t> v((size_t)c.card * ew, 0);
    for (int32_t id = 0; id < c.card; id++) {
      uint8_t *d = v.data() + (size_t)id * ew;
      if (type == PHIP_TYPE_STRING) {
        memcpy(d, c.host_dict.data() + (size_t)id * c.string_width, c.string_width);
      } else {
        const uint8_t *p = c.host_dict.data() + (size_t)id * ew;
        for (int b = 0; b < ew; b++) d[b] = p[ew - 1 - b];  // BE -> LE
      }
    }
    return v;
  };
  std::vector<uint8_t> gvals;
  int64_t n = 0;
  if (gd) {
    n = gd->card;
    const int gw = type == PHIP_TYPE_STRING ? gd->width : ew;
    gvals.assign((size_t)n * ew, 0);
    for (int64_t i = 0; i < n; i++) memcpy(gvals.data() + i * ew, gd->values.data() + i * gw, std::min(gw, ew));
  } else {
    std::vector<uint8_t> all;
    for (size_t i = 0; i < segs.size(); i++) {
      std::vector<uint8_t> v = seg_values(segs[i]->cols[colidx[i]]);
      all.insert(all.end(), v.begin(), v.end());
    }
    const int64_t total = (int64_t)(all.size() / std::max(ew, 1));
    std::vector<int64_t> order(total);
    for (int64_t i = 0; i < total; i++) order[i] = i;
    const uint8_t *A = all.data();
    std::stable_sort(order.begin(), order.end(), [&](int64_t x, int64_t y) {
      return compare_value(type, A + x * ew, A + y * ew, ew) < 0;
    });
    for (int64_t k = 0; k < total; k++) {
      const uint8_t *v = A + order[k] * ew;
      if (n > 0 && compare_value(type, gvals.data() + (n - 1) * ew, v, ew) == 0) continue;
      gvals.insert(gvals.end(), v, v + ew);
      n++;
    }
  }
  if (n > INT32_MAX) return fail(PHIP_ERR_UNSUPPORTED, "column %s: dictionary of %lld values", name.c_str(), (long long)n);
  r->card = (int32_t)n;
  r->dev.assign(segs.size(), nullptr);
  for (size_t i = 0; i < segs.size(); i++) {
    const ColumnStore &c = segs[i]->cols[colidx[i]];
    std::vector<uint8_t> v = seg_values(c);
    if (v == gvals) continue;  // identity map
    std::vector<int32_t> m(c.card);
    for (int32_t id = 0; id < c.card; id++) {
      const uint8_t *x = v.data() + (size_t)id * ew;
      int64_t lo = 0, hi = n;
      while (lo < hi) {
        const int64_t mid = (lo + hi) / 2;
        if (compare_value(type, gvals.data() + mid * ew, x, ew) < 0) lo = mid + 1;
        else hi = mid;
      }
      if (lo == n || compare_value(type, gvals.data() + lo * ew, x, ew) != 0)
        return fail(PHIP_ERR_INVALID, "column %s: a value of segment %s is missing from the global dictionary",
                    name.c_str(), segs[i]->name.c_str());
      m[id] = (int32_t)lo;
    }
    void *p;
    HIP_TRY(hipMalloc(&p, std::max<size_t>(m.size(), 1) * 4));
    r->dev[i] = (int32_t *)p;  // owned by r from here (freed by ~Remap on any later failure)
    HIP_TRY(hipMemcpy(p, m.data(), m.size() * 4, hipMemcpyHostToDevice));
  }
  r->values = std::move(gvals);
  dev.remaps[key] = r;
  out = r;
  return PHIP_OK;
}

int32_t ensure_hll(ColumnStore &c, int log2m, uint32_t **out) {
  auto it = c.hll.find(log2m);
  if (it != c.hll.end()) {
    *out = it->second;
    return PHIP_OK;
  }
  std::vector<uint32_t> t(c.card);
  for (int32_t id = 0; id < c.card; id++) {
    int32_t x;
    const uint8_t *p;
    switch (c.type) {
      case PHIP_TYPE_INT: p = c.host_dict.data() + 4 * id; x = murmur_hash_long((int64_t)(int32_t)be32(p)); break;
      case PHIP_TYPE_LONG: p = c.host_dict.data() + 8 * id; x = murmur_hash_long((int64_t)be64(p)); break;
      case PHIP_TYPE_FLOAT: p = c.host_dict.data() + 4 * id; x = murmur_hash_long((int64_t)(int32_t)be32(p)); break;
      case PHIP_TYPE_DOUBLE: p = c.host_dict.data() + 8 * id; x = murmur_hash_long((int64_t)be64(p)); break;
      default: {
        p = c.host_dict.data() + (size_t)c.string_width * id;
        int32_t len = c.string_width;
        while (len > 0 && p[len - 1] == 0) len--;
        x = murmur_hash_bytes(p, len, -1);
      }
    }
    t[id] = hll_index_rho(x, log2m);
  }
  void *d;
  HIP_TRY(hipMalloc(&d, std::max<size_t>(t.size(), 1) * 4));
  HIP_TRY(hipMemcpy(d, t.data(), t.size() * 4, hipMemcpyHostToDevice));
  c.hll[log2m] = (uint32_t *)d;
  *out = (uint32_t *)d;
  return PHIP_OK;
}

// Doc-order values of a numeric dictionary column (load.hip materialize_kernel), made the first time a plan projects
// the column as a plain value (see use_vals in phip_plan_create) and kept with the segment: num_docs x 4 / 8 bytes.
// Plan creation holds the device's mutex, so two plans never build one column's values at once.
constexpr int64_t kMaterializeMinDict = 1 << 20;
static int64_t materialize_min_dict() {
  const char *e = getenv("PHIP_MATERIALIZE_MIN_DICT");  // measurement override (bytes of dictionary)
  return e ? atoll(e) : kMaterializeMinDict;
}
static bool vals_eligible(const ColumnStore &c, int64_t min_dict) {
  if (no_dict(c) || c.words == nullptr || c.dict == nullptr || c.type == PHIP_TYPE_STRING) return false;
  return (int64_t)c.card * type_width(c.type) >= min_dict;
}
// Doc-order DISTINCTCOUNTHLL entries (entry of doc d = the per-dictionary-id table's entry of its id): made the first
// time a plan aggregates the column with that log2m, when the table is too large to stay in L2 (>= 1 MiB, e.g. ~3M
// LO_CUSTKEY ids per segment: a 12 MB table gathered at random once per matched doc).
static int32_t ensure_hll_doc(Segment &sg, ColumnStore &c, int log2m, const uint32_t *table, hipStream_t st, bool *made,
                              uint32_t **out) {
  auto it = c.hll_doc.find(log2m);
  if (it != c.hll_doc.end()) {
    *out = it->second;
    return PHIP_OK;
  }
  void *p;
  int32_t rc = dev_alloc(sg, (size_t)std::max<int32_t>(sg.num_docs, 1) * 4, &p);
  if (rc) return rc;
  HIP_TRY(launch_materialize(c.words, c.bits, table, 4, sg.num_docs, p, st));
  c.hll_doc[log2m] = (uint32_t *)p;
  *out = (uint32_t *)p;
  *made = true;
  return PHIP_OK;
}
// ... packed to 16 bits when log2m <= 11 ((register << 5) | rho): half the bytes per matched doc
static int32_t ensure_hll_doc16(Segment &sg, ColumnStore &c, int log2m, const uint32_t *table, hipStream_t st,
                                bool *made, uint16_t **out) {
  auto it = c.hll_doc16.find(log2m);
  if (it != c.hll_doc16.end()) {
    *out = it->second;
    return PHIP_OK;
  }
  void *p;
  int32_t rc = dev_alloc(sg, (size_t)std::max<int32_t>(sg.num_docs, 1) * 2, &p);
  if (rc) return rc;
  HIP_TRY(launch_materialize_hll16(c.words, c.bits, table, sg.num_docs, (uint16_t *)p, st));
  c.hll_doc16[log2m] = (uint16_t *)p;
  *out = (uint16_t *)p;
  *made = true;
  return PHIP_OK;
}

// Bits per doc of an INT / LONG column's values packed relative to its minimum (the dictionary's first entry), or 0
// when packing saves nothing (the range needs the type's width, or more than decode_bits' 32).
static int32_t packed_value_bits(const ColumnStore &c) {
  if (!c.has_range || (c.type != PHIP_TYPE_INT && c.type != PHIP_TYPE_LONG)) return 0;
  const uint64_t r = (uint64_t)c.vmax - (uint64_t)c.vmin;
  const int32_t b = r == 0 ? 1 : 64 - __builtin_clzll(r);
  return b <= 32 && b < 8 * type_width(c.type) ? b : 0;
}
static bool vpack_enabled() {
  const char *e = getenv("PHIP_VPACK");  // measurement override: "0" = typed doc-order values
  return !(e && atoi(e) == 0);
}
// (packed when the range allows and vpack_enabled(): e.g. LO_EXTENDEDPRICE in 24 bits, LO_SUPPLYCOST in 17)
static int32_t ensure_vals(Segment &sg, ColumnStore &c, hipStream_t st, bool *made, bool pack) {
  if (pack && packed_value_bits(c) > 0) {
    if (c.vpack != nullptr) return PHIP_OK;
    const int32_t vb = packed_value_bits(c);
    // whole tiles (the filter kernel may stream them like ids) + 4 guard words, like the forward index's words
    const int64_t nwords = round_up(std::max<int64_t>(sg.num_docs, 1), kTileDocs) * vb / 32 + 4;
    void *p;
    int32_t rc = dev_alloc(sg, (size_t)nwords * 4, &p);
    if (rc) return rc;
    HIP_TRY(launch_materialize_packed(c.words, c.bits, c.dict, type_width(c.type), sg.num_docs, c.vmin, vb, nwords,
                                      (uint32_t *)p, st));
    c.vpack = (uint32_t *)p;
    c.vbits = vb;
    *made = true;
    return PHIP_OK;
  }
  if (c.vals != nullptr) return PHIP_OK;
  const int w = type_width(c.type);
  void *p;
  int32_t rc = dev_alloc(sg, (size_t)std::max<int32_t>(sg.num_docs, 1) * w, &p);
  if (rc) return rc;
  HIP_TRY(launch_materialize(c.words, c.bits, c.dict, w, sg.num_docs, p, st));
  c.vals = p;
  *made = true;
  return PHIP_OK;
}

int acc_kind_for(const phip_aggregation &a, bool integral) {
  switch (a.function) {
    case PHIP_AGG_COUNT: return ACC_COUNT;
    case PHIP_AGG_SUM: return integral ? ACC_SUM_I64 : ACC_SUM_F64;
    case PHIP_AGG_MIN: return ACC_MIN_F64;
    case PHIP_AGG_MAX: return ACC_MAX_F64;
    default: return ACC_HLL;
  }
}

}  // namespace

// A prepared query (InstancePlanMakerImplV2.makeInstancePlan's Plan, executed like
// GlobalPlanImplV0.execute, pinot-core/.../plan/GlobalPlanImplV0.java:48-57): every host-side step
// (predicate programs, segment descriptors, launch shapes) is done once; the device-side descriptor
// blob and every buffer the launches touch are owned by the plan, so an execution is a replay of the
// same launch sequence (a captured hipGraph from the second execution on).
struct Plan {
  Device *dev = nullptr;
  std::atomic<int64_t> deadline_ms{0};  // phip_plan_set_deadline (0 = none)
  std::atomic<int32_t> cancelled{0};    // phip_plan_cancel (sticky)
  std::vector<std::shared_ptr<Segment>> segs;  // keeps the segments' HBM alive while the plan exists
  std::vector<void *> allocs;
  int32_t alloc(size_t bytes, void **out) {
    void *p = nullptr;
    HIP_TRY(hipMalloc(&p, std::max<size_t>(bytes, 16)));
    allocs.push_back(p);
    *out = p;
    return PHIP_OK;
  }
  ~Plan() {
    if (graph_exec) (void)hipGraphExecDestroy(graph_exec);
    if (dev) (void)hipSetDevice(dev->ordinal);
    for (auto &e : ev)
      if (e) (void)hipEventDestroy(e);
    for (void *p : allocs) (void)hipFree(p);
    if (pinned) (void)hipHostFree(pinned);
    if (pstage) (void)hipHostFree(pstage);
  }
  // configuration
  DevAggQuery dq;
  DevFilter fq;
  std::vector<DevSeg> dsegs;
  std::vector<RoaringTask> tasks;
  std::vector<std::shared_ptr<Device::Remap>> gb_dicts;
  std::vector<int64_t> gb_radix;  // per group-by column: key ids (its dictionary's, + 1 for the null key)
  // tuple keys (key space above 2^62): the device groups by one virtual column (tuple_remap's doc-order ids); the
  // result's keys expand back to the query's columns (tuple_dicts / tuple_radix, packed per tuple_word / tuple_stride)
  bool tuple_keys = false;
  std::shared_ptr<Device::Remap> tuple_remap;
  std::vector<std::shared_ptr<Device::Remap>> tuple_dicts;
  std::vector<int64_t> tuple_radix;
  std::vector<int32_t> tuple_word;
  std::vector<uint64_t> tuple_stride;
  int32_t tuple_gb_col[1] = {0};
  std::vector<int32_t> tuple_cols;  // the query's group-by columns
  int nseg = 0, naggs = 0, nhll = 0, log2m = 0, m_regs = 0, num_group_by = 0, num_projected = 0;
  int nprog = 1;   // filter programs (phip_query_desc.num_filter_programs)
  int nmatch = 0;  // seg_matched slots = nprog * nseg
  std::vector<int64_t> slot_docs;  // per seg_matched slot: the docs of that (program, segment) entry, 0 = pruned
  int64_t num_groups_limit = 0, total_work = 0, total_docs = 0, docs_in_work = 0;
  int32_t order_agg = -1, order_desc = 0;  // server-level trim (phip_query_desc.order_by_aggregation)
  int32_t order_nkeys = 0;                 // > 0: ORDER BY group-by columns (order_keys)
  int32_t order_keys[kMaxOrderKeys] = {};
  OrderTerms order_terms{};                // num_terms > 0: general ORDER BY (phip_query_desc.order_terms)
  int64_t trim_size = 0;
  int64_t filter_bytes = 0;  // algorithmic bytes of one filter launch (phip_result.filter_bytes)
  std::vector<int64_t> seg_docs;  // num_docs per query segment
  struct ProjCol {
    std::vector<int32_t> bits, card, width;  // per query segment: fixed-bit width (0 = raw), dictionary
                                             // entries, bytes per value / dictionary entry
    uint32_t progs = 1;                      // bit p: filter program p projects the column
  };
  std::vector<ProjCol> proj;
  bool has_filter = false, need_agg = false, need_mask = false, group_by = false, conj_only = false;
  int fused_naggs = 0;  // > 0: the filter kernel aggregates (fused_tile), no aggregation launch
  bool fused_gb = false;  // the filter kernel runs the dense group-by into the HBM table (no aggregation launch)
  bool gb_xcd = false;    // ... into kXcdCopies XCD-private copies of it (GB_XCD), merged after the launch
  bool gb_lds = false;    // ... into each workgroup's LDS table (GB_LDS), its slabs reduced after the launch
  bool node_part = false;  // a node plan's part (node_plan_create): a hash table may go out as a partial table
  // GB_LDS walks: [0] the one-chunk walk, [1] the batched one (agg_kernel kDense) -- LDS bytes, workgroups and waves
  // per workgroup of each; walk_cur's is the launch's (agg_lds / agg_blocks / dq.dense_batch / dq.wg_waves), re-chosen
  // after every execution from its matched docs when walk_adaptive (the device descriptor reads neither field)
  struct GbWalk {
    size_t lds = 0;
    int blocks = 0, waves = 0;
    bool batched = false, ok = false;
  };
  GbWalk walk[2];
  int walk_cur = -1;
  bool walk_adaptive = false;
  // GB_NONE id histogram (DevAggQuery.hist_aggs): its aggregations, and the launch's LDS with / without the bins
  uint32_t hist_mask = 0;
  size_t agg_lds_hist = 0, agg_lds_plain = 0;
  bool want_bitmap = false;
  int64_t filter_nwords = 0;
  int filter_blocks = 1, agg_blocks = 8;
  size_t filter_lds = 0, agg_lds = 0;
  // device buffers (plan-owned)
  uint8_t *base = nullptr;  // descriptor blob
  size_t tasks_off = 0, dq_off = 0, kinds_off = 0, rgroups_off = 0, num_rgroups = 0;
  void *inv_words = nullptr;
  size_t inv_words_total = 0;
  void *fpart = nullptr, *finals = nullptr, *seg_matched = nullptr, *apart = nullptr, *masks = nullptr;
  void *gtab = nullptr, *ghll = nullptr, *slab = nullptr, *hslab = nullptr, *fo = nullptr;
  // pinned host landing area for the per-execution results: finals[64] | seg_matched[nmatch] | hll
  uint64_t *pinned = nullptr;
  uint64_t *pinned_dev = nullptr;  // the same memory as the device addresses it
  hipGraphExec_t graph_exec = nullptr;
  bool graph_failed = false;
  int executions = 0;
  // per-plan timing events (recorded by every eager run and by every replay of the captured graph):
  // 0 start, 1 before the filter kernel, 4 between filter and aggregation, 2 after the aggregation, 3 end
  hipEvent_t ev[5] = {};
  std::mutex exec_mu;  // executions of one plan serialise (its buffers are reused)
  hipStream_t graph_stream = nullptr;  // the lane stream the graph was captured on
  bool clean = false;  // device seg_matched / HLL registers are zero (finalize_all reset them last time)
  bool partial_pending = false;  // phip_plan_execute_partial handed the table out; phip_plan_finish is next
  // aggregation-only partials: [1 + naggs] u64 rows + 6 int64 statistics (device), u8 HLL registers (device), and a
  // pinned staging area for their one H2D / D2H copy each
  uint64_t *ptab = nullptr;
  uint8_t *phll = nullptr;
  uint64_t *pstage = nullptr;
  double part_times[5] = {0, 0, 0, 0, 0};  // the partial's execution: scan, device, filter, agg kernel ms; fused
  int64_t part_bytes[3] = {0, 0, 0};        // its filter / agg / stream bytes (reported again by phip_plan_finish)
  // one segment, hash table, key space >= numGroupsLimit: the normal pass records every slot's first matched doc
  // (aggregate.hip seg_keys with one segment: the key is unchanged), so the limit pass starts from its table
  uint32_t *first_doc = nullptr;
  // selection queries (select.hip): descriptor in the blob, per-execution scratch (tile ranks, entry bases)
  bool select = false;
  int nsel = 0;
  size_t sq_off = 0;
  int64_t *sel_tile_cnt = nullptr, *sel_tile_off = nullptr, *sel_base = nullptr, *sel_kept = nullptr,
          *sel_total = nullptr;
  std::vector<int32_t> sel_types;
  std::vector<std::shared_ptr<Device::Remap>> sel_dicts;
  std::vector<std::vector<const void *>> sel_str_ptrs;  // per SEL_STR expression: its segments' bytes, then offsets
  std::vector<int32_t> sel_bits, sel_width;  // per select column's projected bytes (algorithmic bytes)
  float sel_filter_ms = 0.f;
  // record ev[0] / ev[3] around the whole sequence (phip_result.device_ms): off by default -- every timing marker is a
  // barrier packet the command processor waits on (~4 us each, r04 host A/B); PHIP_TOTAL_EVENTS=1 records them
  bool total_events = false;
  bool split_event = true;   // record ev[4] between a filter and a separate aggregation launch
  bool fold_final = false;   // the last kernel's last workgroup finalizes (no finalize_all launch)
  uint32_t *fin_counter = nullptr;  // its ticket counter (device)
  // Completion by polling (aggregation-only plans run without timing markers, PHIP_POLL_DONE, default on):
  // finalize_all publishes the execution's sequence number in the mapped result area after its results
  // (aggregate.hip finalize_all_kernel), and the host spins on that word instead of waiting for the stream -- the
  // kernel's end-of-pipe release and completion signal are not on the query's path. done_seq = the number this
  // execution waits for (0: wait for the stream).
  uint32_t *done_ticket = nullptr;
  uint64_t done_counter = 0, done_seq = 0;
  // PHIP_KERNEL_TIMING=0 (read per execution; aggregation-only plans): no timing markers around the kernels -- two
  // barrier packets the command processor waits on per query -- and kernel times reported as 0
  bool timed = true;
};

// String.compareTo order (UTF-16 code units) over UTF-8 bytes: the lead bytes 0xEE / 0xEF (U+E000..U+FFFF) rank
// after the 4-byte leads 0xF0..0xF4 (supplementary characters, i.e. surrogate pairs 0xD800..0xDFFF in UTF-16); every
// other byte keeps its order. The kernel compares the same way (filter.hip java_str_cmp).
static inline int java_order_byte(uint8_t b) { return (b == 0xEE || b == 0xEF) ? b + 8 : b; }
static int java_str_cmp(const uint8_t *a, size_t al, const uint8_t *b, size_t bl) {
  const size_t m = std::min(al, bl);
  for (size_t i = 0; i < m; i++)
    if (a[i] != b[i]) return java_order_byte(a[i]) < java_order_byte(b[i]) ? -1 : 1;
  return al < bl ? -1 : (al > bl ? 1 : 0);
}

// RAW_RANGE / RAW_SET leaf on a raw STRING column (StringRawValueBasedRangePredicateEvaluator / the raw EQ / IN
// evaluators of RangePredicateEvaluatorFactory.java / InPredicateEvaluatorFactory.java). phip_filter_node.ids holds
// `count` int32 words: RAW_SET = [n][n + 1 byte offsets][the values' UTF-8 bytes]; RAW_RANGE = [lo_len][hi_len]
// [lo_inclusive][hi_inclusive][lo bytes][hi bytes], a length of -1 = unbounded. The set is sorted in String order and
// deduplicated here, so the kernel binary-searches it.
// An IN / EQ set the bit-sliced conjunction tests as an OR of equalities: a dictionary of <= 64 ids (the leaf's
// set_mask) and at most kBitSliceSetMax of them in the set (each costs one op per plane)
constexpr int kBitSliceSetMax = 4;
static bool bs_small_set(const DevNode &dn, const DevCol &dc) {
  const bool on = getenv("PHIP_BS_SETS") != nullptr;  // opt-in until measured on the GPU (read per plan)
  if (!on || !dn.small_set || dc.card > 64) return false;
  const uint64_t in_dict = dc.card >= 64 ? ~0ull : ((1ull << dc.card) - 1);
  return __builtin_popcountll(dn.set_mask & in_dict) <= kBitSliceSetMax;
}

// An IN / NOT IN set of any dictionary whose ids form at most 4 runs of consecutive ids (DevNode.bs_runs): the
// bit-sliced conjunction tests it as an OR of plane ranges (equalities for one-id runs). PHIP_BS_RUNS=0 disables it.
static bool bs_runs_set(const DevNode &dn) {
  const char *e = getenv("PHIP_BS_RUNS");  // (read per plan, as the tests switch it)
  const bool off = e != nullptr && atoi(e) == 0;
  return !off && dn.leaf_kind == PHIP_LEAF_DICT_SET && dn.bs_nruns > 0;
}

struct AuxFix {  // a leaf's node.aux = device base of the plan's blob + off
  size_t node;
  size_t off;
};

static int32_t raw_string_leaf(const phip_filter_node &fn, DevNode &dn, Blob &blob, std::vector<AuxFix> &aux_fix,
                               size_t ni) {
  if (fn.ids == nullptr || fn.count < 1) return fail(PHIP_ERR_INVALID, "raw STRING leaf without its values");
  const int64_t wb = (int64_t)fn.count * 4;
  const uint8_t *w = (const uint8_t *)fn.ids;
  if (fn.leaf_kind == PHIP_LEAF_RAW_STRING_RANGE) {
    if (fn.count < 4) return fail(PHIP_ERR_INVALID, "raw STRING range: truncated bounds");
    const int32_t lo_len = fn.ids[0], hi_len = fn.ids[1];
    if (lo_len < -1 || hi_len < -1 || 16 + (int64_t)std::max(lo_len, 0) + std::max(hi_len, 0) > wb)
      return fail(PHIP_ERR_INVALID, "raw STRING range: bound lengths %d / %d exceed the leaf's %d words", lo_len, hi_len, fn.count);
    aux_fix.push_back({ni, blob.add(fn.ids, (size_t)(16 + std::max(lo_len, 0) + std::max(hi_len, 0)))});
    return PHIP_OK;
  }
  const int64_t nv = fn.ids[0];
  if (nv < 0 || (1 + nv + 1) * 4 > wb) return fail(PHIP_ERR_INVALID, "raw STRING set: %lld values in %d words", (long long)nv, fn.count);
  const int64_t data0 = (2 + nv) * 4;
  std::vector<std::pair<const uint8_t *, size_t>> vals;
  vals.reserve(nv);
  for (int64_t k = 0; k < nv; k++) {
    const int64_t s = (uint32_t)fn.ids[1 + k], e = (uint32_t)fn.ids[2 + k];
    if (e < s || data0 + e > wb) return fail(PHIP_ERR_INVALID, "raw STRING set: value %lld outside the leaf", (long long)k);
    vals.push_back({w + data0 + s, (size_t)(e - s)});
  }
  auto less = [](const std::pair<const uint8_t *, size_t> &a, const std::pair<const uint8_t *, size_t> &b) {
    return java_str_cmp(a.first, a.second, b.first, b.second) < 0;
  };
  std::sort(vals.begin(), vals.end(), less);
  vals.erase(std::unique(vals.begin(), vals.end(),
                         [](const std::pair<const uint8_t *, size_t> &a, const std::pair<const uint8_t *, size_t> &b) {
                           return java_str_cmp(a.first, a.second, b.first, b.second) == 0;
                         }),
             vals.end());
  if (vals.empty()) {
    dn.leaf_kind = fn.exclusive ? PHIP_LEAF_MATCH_ALL : PHIP_LEAF_MATCH_NONE;
    return PHIP_OK;
  }
  // device payload: [n][n + 1 offsets] then the bytes, in order
  std::vector<uint32_t> out(2 + vals.size());
  out[0] = (uint32_t)vals.size();
  size_t pos = 0;
  for (size_t k = 0; k < vals.size(); k++) {
    out[1 + k] = (uint32_t)pos;
    pos += vals[k].second;
  }
  out[1 + vals.size()] = (uint32_t)pos;
  std::vector<uint8_t> payload(out.size() * 4 + pos);
  memcpy(payload.data(), out.data(), out.size() * 4);
  pos = out.size() * 4;
  for (const auto &v : vals) {
    if (v.second) memcpy(payload.data() + pos, v.first, v.second);
    pos += v.second;
  }
  dn.count = (int32_t)vals.size();
  aux_fix.push_back({ni, blob.add(payload.data(), payload.size())});
  return PHIP_OK;
}

// Group-by records (DevSeg.rec): the fields a matched doc's group-by update reads -- the key columns' dictionary ids,
// each aggregation's packed values or value ids, its doc-order HLL entries -- packed into W <= 4 u32 per doc, made on
// first use for a field signature and kept with the segment (at most kMaxRecordSets per segment). The aggregation
// kernel then reads one 16-byte record per matched doc instead of one line per column (agg_kernel.h rec_load).
// A segment whose columns do not all fit (raw / null / FLOAT-id keys, raw typed values, HLL without doc-order entries)
// keeps its columns' layouts: the kernel decides per segment.
constexpr int kHistCard = 2048;    // agg_kernel kHist: dictionary ids per LDS bin set (two u16 counts per word)
constexpr int kRecMinFields = 3;   // fewer fields: the per-column gathers already touch few lines
constexpr double kRecMaxRatio = 0.8;  // a record's touched bytes must stay below this fraction of the columns'
constexpr int kMaxRecordSets = 16;                       // record signatures kept per segment
constexpr uint64_t kRecordBudget = (uint64_t)64 << 30;  // record bytes per device (PHIP_GB_RECORD_GIB overrides)
// Lines a gather of bpd bytes per doc touches over n docs at match density p: each 128-B line holds 128 / bpd docs
// and is touched unless none of them matched.
static double touched_bytes(double bpd, double p, int64_t n) {
  const double per_line = std::max(1.0, 128.0 / bpd);
  return (double)n * bpd * (1.0 - std::pow(1.0 - std::min(1.0, std::max(0.0, p)), per_line));
}
static int32_t build_records(Segment &sg, const phip_query_desc *q, DevAggQuery &dq, DevSeg &ds,
                             const std::vector<int> &colidx, int min_fields, double density, hipStream_t st,
                             bool *made) {
  RecSrcs fs;
  memset(&fs, 0, sizeof(fs));
  int nf = 0, off = 0;
  bool ok = true;
  std::string sig;
  int8_t fa[kMaxAggs], fb[kMaxAggs];
  auto add = [&](const void *p, int kind, int bits, int col) -> int8_t {
    if (!ok || p == nullptr || bits <= 0 || bits > 32 || nf == kRecFields) {
      ok = false;
      return -1;
    }
    fs.f[nf] = RecSrc{p, kind, bits, off, 0};
    off += bits;
    sig += std::to_string(colidx[col]) + "/" + std::to_string(kind) + "/" + std::to_string(bits) + ";";
    return (int8_t)nf++;
  };
  auto value_field = [&](int col) -> int8_t {
    const DevCol &c = ds.cols[col];
    if (c.vpack != nullptr) return add(c.vpack, REC_BITS, c.vbits, col);
    if (c.has_dict && c.words != nullptr && c.type != PHIP_TYPE_STRING) return add(c.words, REC_BITS, c.bits, col);
    ok = false;
    return -1;
  };
  for (int k = 0; k < q->num_group_by && ok; k++) {
    const int col = q->group_by_columns[k];
    const DevCol &c = ds.cols[col];
    if (!c.has_dict || c.words == nullptr || c.gb_nulls != nullptr || c.gb_ids != nullptr) ok = false;
    else add(c.words, REC_BITS, c.bits, col);
  }
  for (int a = 0; a < kMaxAggs; a++) fa[a] = fb[a] = -1;
  for (int a = 0; a < dq.num_aggs && ok; a++) {
    const DevAgg &ag = dq.aggs[a];
    if (ag.acc == ACC_COUNT) continue;
    if (ag.acc == ACC_HLL) {
      const DevCol &c = ds.cols[ag.col_a];
      if (ag.expr != PHIP_EXPR_COLUMN || c.hll_rows) ok = false;
      // (a 16-bit entry is (register << 5) | rho: log2m + 5 significant bits -- C5's five fields fit 8 bytes)
      else if (c.hll_doc16 != nullptr) fa[a] = add(c.hll_doc16, REC_U16, std::min(16, (int)ag.log2m + 5), ag.col_a);
      else if (c.hll_doc != nullptr) fa[a] = add(c.hll_doc, REC_U32, 32, ag.col_a);
      else ok = false;
      continue;
    }
    fa[a] = value_field(ag.col_a);
    if (ag.expr != PHIP_EXPR_COLUMN) fb[a] = value_field(ag.col_b);
  }
  if (!ok || nf < min_fields || off > 128) return PHIP_OK;
  const int W = (off + 31) / 32;
  // Worth it when the record's touched lines are clearly fewer than the columns' at the estimated density (a general
  // program estimates 1: no record). SSB SF100 (profiles/r06x_rec_ab.log): Q4.1 (density 1.6 %: 2.3 GB of column
  // lines vs 1.1 GB of records) 0.50 -> 0.37 ms, C5 0.77 -> 0.61, Q2.1 0.25 -> 0.21; Q3.1 (3.4 %, three narrow keys
  // whose lines are all touched anyway: 2.4 vs 2.0 GB) 0.51 -> 0.53, so it keeps its columns.
  if (min_fields > 1) {
    double cols = 0;
    for (int f = 0; f < nf; f++) cols += touched_bytes(fs.f[f].bits / 8.0, density, sg.num_docs);
    if (touched_bytes(4.0 * W, density, sg.num_docs) > kRecMaxRatio * cols) return PHIP_OK;
  }
  auto it = sg.records.find(sig);
  if (it == sg.records.end()) {
    if ((int)sg.records.size() >= kMaxRecordSets) return PHIP_OK;
    const char *gib = getenv("PHIP_GB_RECORD_GIB");
    const uint64_t budget = gib ? (uint64_t)atoll(gib) << 30 : kRecordBudget;
    const uint64_t bytes = (uint64_t)sg.num_docs * W * 4 + 16;
    if (sg.device < 0 || sg.device >= kMaxRecordDevices || g_record_bytes[sg.device] + bytes > budget) return PHIP_OK;
    void *p;
    // (+ 16 bytes: rec_load reads 16 bytes whatever W is)
    int32_t rc = dev_alloc(sg, (size_t)sg.num_docs * W * 4 + 16, &p);
    if (rc) return rc;
    HIP_TRY(launch_materialize_record(fs, nf, sg.num_docs, W, (uint32_t *)p, st));
    it = sg.records.emplace(sig, Segment::Record{(uint32_t *)p, W}).first;
    sg.record_bytes += bytes;
    g_record_bytes[sg.device] += bytes;
    *made = true;
  }
  ds.rec = it->second.words;
  ds.rec_words = W;
  ds.rec_nf = nf;
  for (int f = 0; f < nf; f++) {
    ds.rec_off[f] = (uint8_t)fs.f[f].off;
    ds.rec_bits[f] = (uint8_t)fs.f[f].bits;
  }
  for (int a = 0; a < kMaxAggs; a++) {  // (the same for every segment that has a record: the query fixes the order)
    dq.rec_fa[a] = fa[a];
    dq.rec_fb[a] = fb[a];
  }
  return PHIP_OK;
}

static int32_t prepare_plan(const phip_query_desc *q, bool want_bitmap, int64_t filter_nwords, Plan &P) {

  if (!q || q->num_segments <= 0 || q->num_columns < 0 || q->num_columns > kMaxQueryColumns)
    return fail(PHIP_ERR_INVALID, "query: need >=1 segment and <= %d columns", kMaxQueryColumns);
  if (q->num_aggregations < 0 || q->num_aggregations > kMaxAggs)
    return fail(PHIP_ERR_UNSUPPORTED, "query: at most %d aggregations on the GPU path", kMaxAggs);
  if (q->num_group_by < 0 || q->num_group_by > kMaxGroupBy)
    return fail(PHIP_ERR_UNSUPPORTED, "query: at most %d group-by columns", kMaxGroupBy);
  if (q->num_segments > 1 && want_bitmap) return fail(PHIP_ERR_INVALID, "filter bitmap: one segment only");
  const int nprog = std::max(1, q->num_filter_programs);
  if (nprog > kMaxPrograms) return fail(PHIP_ERR_UNSUPPORTED, "query: at most %d filter programs", kMaxPrograms);
  if (nprog > 1 && want_bitmap) return fail(PHIP_ERR_UNSUPPORTED, "several filter programs: no filter bitmap");

  std::vector<Segment *> segs(q->num_segments);
  Device *dev = nullptr;
  {
    std::lock_guard<std::mutex> g(g_mu);
    for (int i = 0; i < q->num_segments; i++) {
      auto it = g_segments.find(q->segments[i]);
      if (it == g_segments.end()) return fail(PHIP_ERR_NOT_FOUND, "unknown segment handle %llu", (unsigned long long)q->segments[i]);
      segs[i] = it->second.get();
      P.segs.push_back(it->second);
      if (i > 0 && segs[i]->device != segs[0]->device)
        return fail(PHIP_ERR_UNSUPPORTED, "segments of one query must reside on one device");
    }
    dev = find_device(segs[0]->device);
  }
  if (!dev) return fail(PHIP_ERR_NO_DEVICE, "device %d not initialised", segs[0]->device);
  std::lock_guard<std::mutex> dlock(dev->mu);
  HIP_TRY(hipSetDevice(dev->ordinal));
  hipStream_t st = dev->stream;
  P.dev = dev;

  const int nseg = q->num_segments, ncols = q->num_columns, naggs = q->num_aggregations;
  // resolve columns
  std::vector<std::vector<int>> colidx(nseg, std::vector<int>(ncols, -1));
  for (int s = 0; s < nseg; s++)
    for (int c = 0; c < ncols; c++) {
      auto it = segs[s]->by_name.find(q->columns[c]);
      if (it == segs[s]->by_name.end())
        return fail(PHIP_ERR_NOT_FOUND, "segment %s has no column %s", segs[s]->name.c_str(), q->columns[c]);
      colidx[s][c] = it->second;
    }

  // A group-by whose mixed-radix key space exceeds 2^62 groups by tuple keys (build_tuple_keys): the plan is made for
  // one virtual key column (the first group-by column's slot carries its ids) and execute_plan expands the keys.
  // Device trims that order by a group key need the columns' order, so such a plan returns every group instead.
  phip_query_desc qv;
  if (q->num_group_by > 1 && q->group_by_columns) {
    std::vector<std::shared_ptr<Device::Remap>> dicts;
    std::vector<int64_t> radix;
    long double space = 1;
    for (int k = 0; k < q->num_group_by; k++) {
      const int c = q->group_by_columns[k];
      if (c < 0 || c >= ncols) return fail(PHIP_ERR_INVALID, "group_by_columns[%d] = %d out of range", k, c);
      std::vector<int> ci(nseg);
      for (int s = 0; s < nseg; s++) ci[s] = colidx[s][c];
      bool null_key = false;
      if ((q->null_group_by >> k) & 1)
        for (int s = 0; s < nseg; s++) null_key |= segs[s]->cols[ci[s]].nulls != nullptr;
      std::shared_ptr<Device::Remap> r;
      int32_t rc = build_remap(*dev, segs, ci, q->columns[c], r, null_key);
      if (rc) return rc;
      dicts.push_back(r);
      radix.push_back((int64_t)r->card + (null_key ? 1 : 0));
      space *= (long double)radix.back();
    }
    const char *tk = getenv("PHIP_TUPLE_KEYS");  // test override: "1" = tuple keys for any multi-column group-by
    if (space > (long double)((int64_t)1 << 62) || (tk && atoi(tk) != 0)) {
      int32_t rc = build_tuple_keys(*dev, segs, colidx, q->group_by_columns, q->num_group_by, dicts, radix,
                                    P.tuple_word, P.tuple_stride, P.tuple_remap);
      if (rc) return rc;
      P.tuple_keys = true;
      P.tuple_dicts = dicts;
      P.tuple_radix = radix;
      P.tuple_gb_col[0] = q->group_by_columns[0];
      P.tuple_cols.assign(q->group_by_columns, q->group_by_columns + q->num_group_by);
      qv = *q;
      qv.num_group_by = 1;
      qv.group_by_columns = P.tuple_gb_col;
      qv.null_group_by = 0;
      bool key_terms = qv.num_order_by_keys > 0;
      for (int j = 0; j < qv.num_order_terms && qv.order_terms; j++) key_terms |= qv.order_terms[j].kind == PHIP_ORDER_GROUP_KEY;
      if (key_terms) {
        qv.trim_size = 0;
        qv.num_order_by_keys = 0;
        qv.num_order_terms = 0;
      }
      q = &qv;
    }
  }

  // aggregations
  DevAggQuery dq;
  memset(&dq, 0, sizeof(dq));
  dq.num_segs = nseg;
  dq.num_aggs = naggs;
  int nhll = 0, log2m = 0;
  std::vector<int32_t> kinds(naggs + 2, ACC_COUNT);
  std::vector<bool> projected(ncols, false);
  std::vector<uint32_t> proj_progs(ncols, 0);  // column -> bit p: program p projects it
  for (int a = 0; a < naggs; a++) {
    const phip_aggregation &ag = q->aggregations[a];
    DevAgg &d = dq.aggs[a];
    d.expr = ag.expr;
    d.col_a = ag.column_a;
    d.col_b = ag.column_b;
    if (ag.program < 0 || ag.program >= nprog)
      return fail(PHIP_ERR_INVALID, "aggregation %d: program %d outside [0, %d)", a, ag.program, nprog);
    d.program = ag.program;
    if (ag.function < PHIP_AGG_COUNT || ag.function > PHIP_AGG_HLL) return fail(PHIP_ERR_INVALID, "bad aggregation function");
    if (ag.function != PHIP_AGG_COUNT) {
      if (ag.column_a < 0 || ag.column_a >= ncols) return fail(PHIP_ERR_INVALID, "aggregation column out of range");
      projected[ag.column_a] = true;
      proj_progs[ag.column_a] |= 1u << ag.program;
      if (ag.expr != PHIP_EXPR_COLUMN) {  // (DISTINCTCOUNTHLL over a col op col: its double values hashed per doc)
        if (ag.column_b < 0 || ag.column_b >= ncols) return fail(PHIP_ERR_INVALID, "aggregation column out of range");
        projected[ag.column_b] = true;
        proj_progs[ag.column_b] |= 1u << ag.program;
      }
    }
    bool integral = true;
    if (ag.function != PHIP_AGG_COUNT) {
      for (int s = 0; s < nseg; s++) {
        const ColumnStore &ca = segs[s]->cols[colidx[s][ag.column_a]];
        if (!(ca.type == PHIP_TYPE_INT || ca.type == PHIP_TYPE_LONG)) integral = false;
        if (ca.type == PHIP_TYPE_STRING && ag.function != PHIP_AGG_HLL)
          return fail(PHIP_ERR_INVALID, "numeric aggregation over STRING column %s", ca.name.c_str());
        if (ca.fwd_kind == PHIP_FWD_HLL_REGISTERS) {  // star-tree HLL pair: DISTINCTCOUNTHLL of the column only
          if (ag.function != PHIP_AGG_HLL || ag.expr != PHIP_EXPR_COLUMN)
            return fail(PHIP_ERR_INVALID, "HLL register column %s outside DISTINCTCOUNTHLL", ca.name.c_str());
          if (ag.log2m != ca.hll_log2m)
            return fail(PHIP_ERR_UNSUPPORTED, "DISTINCTCOUNTHLL log2m %d over registers of log2m %d", ag.log2m,
                        ca.hll_log2m);
        }
        // raw numeric columns offer their values directly (DistinctCountHLLAggregationFunction.java:106-145): the
        // kernels hash each matched doc's value (agg_common.h hll_entry_raw), a raw STRING doc's UTF-8 bytes too
        if (ag.function == PHIP_AGG_HLL && ag.expr != PHIP_EXPR_COLUMN && ca.type == PHIP_TYPE_STRING)
          return fail(PHIP_ERR_INVALID, "numeric expression over STRING column");
        if (ag.expr != PHIP_EXPR_COLUMN) {
          const ColumnStore &cb = segs[s]->cols[colidx[s][ag.column_b]];
          if (!(cb.type == PHIP_TYPE_INT || cb.type == PHIP_TYPE_LONG)) integral = false;
          if (cb.type == PHIP_TYPE_STRING) return fail(PHIP_ERR_INVALID, "numeric expression over STRING column");
          if (cb.fwd_kind == PHIP_FWD_HLL_REGISTERS)
            return fail(PHIP_ERR_INVALID, "expression over the HLL register column %s", cb.name.c_str());
        }
      }
    }
    if (integral && ag.function == PHIP_AGG_SUM) {
      // int64 accumulation is exact only while no partial can leave int64: bound sum |expr| over every doc
      // from the columns' value ranges. Past 2^58 the SUM takes the reference's own double accumulation
      // (SumAggregationFunction.java:76-101; MultiplicationTransformFunction computes 1.0*a*b in double),
      // which cannot wrap. (2^58, not 2^62: the cross-GPU merge all-reduces the exact partials of up to
      // kMaxExactRanks = 16 GPUs as int64 SUM, distributed.allreduce_*, and 16 x 2^58 = 2^62 cannot wrap either.)
      long double bound = 0;
      for (int s = 0; s < nseg && integral; s++) {
        const ColumnStore &ca = segs[s]->cols[colidx[s][ag.column_a]];
        auto mag = [](const ColumnStore &c) -> long double {
          return c.has_range ? std::max(fabsl((long double)c.vmin), fabsl((long double)c.vmax)) : 1e30L;
        };
        long double e = mag(ca);
        if (ag.expr != PHIP_EXPR_COLUMN) {
          const long double b = mag(segs[s]->cols[colidx[s][ag.column_b]]);
          e = ag.expr == PHIP_EXPR_MUL ? e * b : e + b;
        }
        bound += e * (long double)segs[s]->num_docs;
      }
      if (bound >= (long double)((int64_t)1 << 58)) integral = false;
    }
    d.integral = integral;
    d.acc = acc_kind_for(ag, integral);
    kinds[a] = d.acc;
    if (d.acc == ACC_HLL) {
      if (ag.log2m < 4 || ag.log2m > 12) return fail(PHIP_ERR_UNSUPPORTED, "log2m %d outside [4,12]", ag.log2m);
      // DISTINCTCOUNTHLL functions of different log2m share the plan's register tables at the largest one's stride:
      // function a's registers are the first 2^log2m_a of its slot (its per-doc (register, rho) entries are computed
      // with its own log2m, DistinctCountHLLAggregationFunction.java:105-145). One column per entry table, so two
      // log2m over one dictionary column stay on the CPU path (a raw column's values are hashed per function).
      bool raw_everywhere = ag.expr == PHIP_EXPR_COLUMN;
      for (int s = 0; s < nseg && raw_everywhere; s++) {
        const ColumnStore &cs = segs[s]->cols[colidx[s][ag.column_a]];
        raw_everywhere = cs.fwd_kind == PHIP_FWD_RAW_CHUNK;
      }
      for (int b = 0; b < a && !raw_everywhere; b++)
        if (dq.aggs[b].acc == ACC_HLL && dq.aggs[b].expr == PHIP_EXPR_COLUMN && ag.expr == PHIP_EXPR_COLUMN &&
            dq.aggs[b].col_a == ag.column_a && dq.aggs[b].log2m != ag.log2m)
          return fail(PHIP_ERR_UNSUPPORTED, "DISTINCTCOUNTHLL of column %d with two log2m (%d, %d)", ag.column_a,
                      dq.aggs[b].log2m, ag.log2m);
      log2m = std::max(log2m, ag.log2m);
      d.hll_slot = nhll++;
      d.log2m = ag.log2m;
    }
  }
  dq.num_hll = nhll;
  // Plain values of SUM / MIN / MAX (no filter leaf, group-by key or HLL reads the column) whose dictionary is
  // large read the segment's doc-order values: one load by doc instead of the doc's id bits plus a dependent
  // gather into a dictionary that does not stay in the XCD's L2 (~1M distinct prices per segment: random lines
  // from the Infinity Cache). The kernels take such a column as a raw one (DevCol.has_dict = 0).
  std::vector<bool> use_vals(ncols, false);
  const int64_t vals_min = materialize_min_dict();
  const bool vpack_on = vpack_enabled();
  {
    const char *me = getenv("PHIP_MATERIALIZE");  // measurement override: "0" = ids + dictionary gathers
    if (!(me && atoi(me) == 0) && !want_bitmap && vals_min >= 0) {
      for (int a = 0; a < naggs; a++) {
        const phip_aggregation &ag = q->aggregations[a];
        if (ag.function == PHIP_AGG_SUM || ag.function == PHIP_AGG_MIN || ag.function == PHIP_AGG_MAX) {
          use_vals[ag.column_a] = true;
          if (ag.expr != PHIP_EXPR_COLUMN) use_vals[ag.column_b] = true;
        }
      }
      for (int a = 0; a < naggs; a++)
        if (q->aggregations[a].function == PHIP_AGG_HLL) use_vals[q->aggregations[a].column_a] = false;
      for (int k = 0; k < q->num_group_by; k++)
        if (q->group_by_columns[k] >= 0 && q->group_by_columns[k] < ncols) use_vals[q->group_by_columns[k]] = false;
      if (q->filter_offsets && q->filter_nodes)
        for (int i = q->filter_offsets[0]; i < q->filter_offsets[nprog * nseg]; i++) {
          const phip_filter_node &fn = q->filter_nodes[i];
          if (fn.op == PHIP_NODE_LEAF && fn.column >= 0 && fn.column < ncols) use_vals[fn.column] = false;
        }
    }
    bool made = false;
    for (int c = 0; c < ncols; c++) {
      if (!use_vals[c]) continue;
      for (int s = 0; s < nseg; s++) {
        ColumnStore &cs = segs[s]->cols[colidx[s][c]];
        if (!vals_eligible(cs, vals_min)) continue;
        int32_t rc = ensure_vals(*segs[s], cs, st, &made, vpack_on);
        if (rc) return rc;
      }
    }
    if (made) HIP_TRY(hipStreamSynchronize(st));
  }
  // column c of segment s read as raw values (no dictionary, or its doc-order values above, packed or typed)
  auto packed_vals = [&](const ColumnStore &cs) -> bool { return vpack_on && cs.vpack != nullptr; };
  auto as_raw = [&](int s, int c) -> bool {
    const ColumnStore &cs = segs[s]->cols[colidx[s][c]];
    return no_dict(cs) || (use_vals[c] && (packed_vals(cs) || cs.vals != nullptr) && vals_eligible(cs, vals_min));
  };
  // Batched dense-tile walk (aggregate.hip agg_batch) only when every dictionary the aggregations
  // gather from is small enough to stay cache-resident. Gathers from a large dictionary (~1M distinct
  // prices per segment) are bound by random lines from the Infinity Cache, and more of them in flight
  // only thrash the XCD's L2 (measured on SSB SF100: SUM over a ~940K-entry dictionary 5.7 ms per
  // 64-doc chunk vs 6.8 ms batched; over an 11-entry 4-bit column 1.33 ms vs 0.70 ms batched).
  {
    int64_t max_dict = 0;
    for (int a = 0; a < naggs; a++) {
      const phip_aggregation &ag = q->aggregations[a];
      if (ag.function == PHIP_AGG_COUNT) continue;
      for (int s = 0; s < nseg; s++) {
        for (int c : {ag.column_a, ag.expr != PHIP_EXPR_COLUMN ? ag.column_b : -1}) {
          if (c < 0) continue;
          const ColumnStore &cs = segs[s]->cols[colidx[s][c]];
          if (as_raw(s, c)) continue;
          const int64_t w = ag.function == PHIP_AGG_HLL ? 4 : ((cs.type == PHIP_TYPE_LONG || cs.type == PHIP_TYPE_DOUBLE) ? 8 : 4);
          max_dict = std::max<int64_t>(max_dict, (int64_t)cs.card * w);
        }
      }
    }
    dq.dense_batch = max_dict <= (512 << 10) ? 1 : 0;
    const char *db = getenv("PHIP_DENSE_BATCH");  // measurement override: "0" / "1"
    if (db) dq.dense_batch = atoi(db) != 0;
    dq.dense_min = kDenseMin;
    const char *dm = getenv("PHIP_DENSE_MIN");  // measurement override
    if (dm) dq.dense_min = std::max(1, atoi(dm));
    // Id histogram (agg_kernel kHist): SUM / MIN / MAX of one INT / LONG column whose dictionary has at most kHistCard
    // ids in every segment count the docs per id in LDS and fold count x value in at each segment's end -- the
    // per-doc dictionary gather goes (C4 SUM(M), 1000 ids). Integer sums stay exact (count x value wraps as the
    // repeated sum does); MIN / MAX do not depend on order. COUNTs beside them keep their own path.
    dq.hist_aggs = 0;
    dq.hist_col = -1;
    dq.hist_words = 0;
    {
      const char *he = getenv("PHIP_AGG_HIST");  // measurement override: "0" = gather the values
      bool ok = q->num_group_by == 0 && dq.dense_batch && nhll == 0 && nprog == 1 && naggs <= 2 && !(he && atoi(he) == 0);
      int col = -1, max_card = 0;
      uint32_t mask = 0;
      for (int a = 0; a < naggs && ok; a++) {
        const phip_aggregation &ag = q->aggregations[a];
        if (dq.aggs[a].acc == ACC_COUNT) continue;
        const int k = dq.aggs[a].acc;
        if ((k != ACC_SUM_I64 && k != ACC_MIN_F64 && k != ACC_MAX_F64) || ag.expr != PHIP_EXPR_COLUMN ||
            (col >= 0 && ag.column_a != col)) {
          ok = false;
          break;
        }
        col = ag.column_a;
        mask |= 1u << a;
        for (int s = 0; s < nseg && ok; s++) {
          const ColumnStore &cs = segs[s]->cols[colidx[s][col]];
          if (as_raw(s, col) || no_dict(cs) || (cs.type != PHIP_TYPE_INT && cs.type != PHIP_TYPE_LONG) ||
              cs.card < 1 || cs.card > kHistCard)
            ok = false;
          else max_card = std::max(max_card, cs.card);
        }
      }
      if (ok && mask) {
        dq.hist_aggs = mask;
        dq.hist_col = col;
        dq.hist_words = (max_card + 1) / 2;
      }
    }
    // Stage the fixed-bit words of the gathered dictionary columns of a dense tile in LDS (one region
    // per distinct column, sized for its widest segment), when they fit kAggStageBudget per wave.
    for (int a = 0; a < kMaxAggs; a++) dq.stage_slot_a[a] = dq.stage_slot_b[a] = -1;
    std::vector<int> cols;
    std::vector<int> maxbits;
    bool ok = dq.dense_batch != 0 && q->num_group_by == 0;
    for (int a = 0; a < naggs && ok; a++) {
      const phip_aggregation &ag = q->aggregations[a];
      if (ag.function == PHIP_AGG_COUNT) continue;
      for (int which = 0; which < 2; which++) {
        const int c = which == 0 ? ag.column_a : (ag.expr != PHIP_EXPR_COLUMN ? ag.column_b : -1);
        if (c < 0) continue;
        int bits = 0;
        bool any_dict = false;
        for (int s = 0; s < nseg; s++) {
          const ColumnStore &cs = segs[s]->cols[colidx[s][c]];
          if (as_raw(s, c)) continue;
          any_dict = true;
          bits = std::max(bits, cs.bits);
        }
        if (!any_dict) continue;
        int slot = -1;
        for (size_t k = 0; k < cols.size(); k++)
          if (cols[k] == c) slot = (int)k;
        if (slot < 0) {
          if ((int)cols.size() == kMaxAggStage) { ok = false; break; }
          slot = (int)cols.size();
          cols.push_back(c);
          maxbits.push_back(bits);
        }
        (which == 0 ? dq.stage_slot_a : dq.stage_slot_b)[a] = slot;
      }
    }
    int32_t off = 0;
    for (size_t k = 0; k < cols.size() && ok; k++) {
      dq.stage_col[k] = cols[k];
      dq.stage_off[k] = off + kStagePad;
      off += 256 * maxbits[k] + 2 * kStagePad;
    }
    // dictionaries of at most kAggLdsDict bytes (in every segment) are read from LDS as well. (Round 6 measured 8 KiB
    // dictionaries in LDS too, the per-wave copies within 8 KiB more of LDS per wave: C4 SUM(M) over a 1000-entry
    // dictionary got slower at every selectivity -- 50 %: aggregation 1.33 -> 1.96 ms, 0.01 %: 0.16 -> 0.27 ms,
    // profiles/r06d_c4_lds_dict_ab.log -- the larger stage area halves the resident workgroups of a latency-bound walk)
    for (size_t k = 0; k < cols.size() && ok; k++) {
      dq.stage_dict_off[k] = -1;
      int64_t bytes = 0;
      bool numeric = true;
      for (int s = 0; s < nseg; s++) {
        const ColumnStore &cs = segs[s]->cols[colidx[s][cols[k]]];
        if (as_raw(s, cols[k])) continue;
        if (cs.type == PHIP_TYPE_STRING) numeric = false;
        const int64_t w = (cs.type == PHIP_TYPE_LONG || cs.type == PHIP_TYPE_DOUBLE) ? 8 : 4;
        bytes = std::max<int64_t>(bytes, (int64_t)cs.card * w);
      }
      const char *ld = getenv("PHIP_AGG_LDS_DICT");  // measurement override: "0" keeps dictionaries in HBM
      if (numeric && bytes <= kAggLdsDict && off + bytes <= kAggStageBudget && !(ld && atoi(ld) == 0)) {
        dq.stage_dict_off[k] = off;
        off += (int32_t)round_up(bytes, 16);
      }
    }
    const char *ds = getenv("PHIP_AGG_STAGE");  // measurement override: "0" disables staging
    if (ds && atoi(ds) == 0) ok = false;
    if (ok && !cols.empty() && off <= kAggStageBudget) {
      dq.num_stage = (int32_t)cols.size();
      dq.stage_bytes = round_up(off, 16);
    } else {
      dq.num_stage = 0;
      dq.stage_bytes = 0;
      for (int a = 0; a < kMaxAggs; a++) dq.stage_slot_a[a] = dq.stage_slot_b[a] = -1;
    }
  }
  for (int k = 0; k < q->num_group_by; k++) {
    int c = q->group_by_columns[k];
    if (c < 0 || c >= ncols) return fail(PHIP_ERR_INVALID, "group-by column out of range");
    projected[c] = true;
    proj_progs[c] |= (1u << nprog) - 1;  // every program's docs generate groups (FilteredGroupByOperator infos)
  }
  // selection (SelectionOnlyOperator): expressions, output kinds, query-global dictionaries of STRING columns
  const int nsel = q->num_select;
  if (nsel < 0 || nsel > kMaxSelect) return fail(PHIP_ERR_UNSUPPORTED, "selection: at most %d expressions", kMaxSelect);
  if (nsel > 0 && (naggs > 0 || q->num_group_by > 0 || nprog > 1 || want_bitmap || !q->select))
    return fail(PHIP_ERR_INVALID, "selection: no aggregations, group-by or filter programs beside the expressions");
  DevSelQuery sq;
  memset(&sq, 0, sizeof(sq));
  std::vector<int32_t> sel_types(nsel, 0);
  std::vector<std::shared_ptr<Device::Remap>> sel_dicts(nsel), col_remap(ncols);
  for (int k = 0; k < nsel; k++) {
    const phip_select_expr &e = q->select[k];
    if (e.expr < PHIP_EXPR_COLUMN || e.expr > PHIP_EXPR_MUL || e.column_a < 0 || e.column_a >= ncols ||
        (e.expr != PHIP_EXPR_COLUMN && (e.column_b < 0 || e.column_b >= ncols)))
      return fail(PHIP_ERR_INVALID, "select expression %d malformed", k);
    DevSelect &d = sq.sel[k];
    d.expr = e.expr;
    d.col_a = e.column_a;
    d.col_b = e.expr != PHIP_EXPR_COLUMN ? e.column_b : e.column_a;
    for (int c : {e.column_a, e.expr != PHIP_EXPR_COLUMN ? e.column_b : -1}) {
      if (c < 0) continue;
      projected[c] = true;
      const int t0 = segs[0]->cols[colidx[0][c]].type;
      for (int s = 0; s < nseg; s++) {
        const ColumnStore &cs = segs[s]->cols[colidx[s][c]];
        if (cs.type != t0) return fail(PHIP_ERR_UNSUPPORTED, "selection: column %s changes type across segments", q->columns[c]);
        if (cs.fwd_kind == PHIP_FWD_HLL_REGISTERS)
          return fail(PHIP_ERR_INVALID, "selection of the HLL register column %s", q->columns[c]);
        if (cs.type == PHIP_TYPE_STRING && e.expr != PHIP_EXPR_COLUMN)
          return fail(PHIP_ERR_INVALID, "selection: numeric expression over STRING column %s", q->columns[c]);
        if (cs.type == PHIP_TYPE_STRING && (cs.fwd_kind == PHIP_FWD_RAW_CHUNK) !=
                                               (segs[0]->cols[colidx[0][c]].fwd_kind == PHIP_FWD_RAW_CHUNK))
          return fail(PHIP_ERR_UNSUPPORTED, "selection: STRING column %s raw in some segments only", q->columns[c]);
      }
    }
    const int t = segs[0]->cols[colidx[0][e.column_a]].type;
    if (e.expr != PHIP_EXPR_COLUMN) {
      d.kind = SEL_F64;
      sel_types[k] = PHIP_TYPE_DOUBLE;
    } else if (t == PHIP_TYPE_STRING && segs[0]->cols[colidx[0][e.column_a]].fwd_kind == PHIP_FWD_RAW_CHUNK) {
      // a raw STRING column: the rows' locators, their bytes gathered after the rows are known (execute_select)
      d.kind = SEL_STR;
      sel_types[k] = PHIP_TYPE_STRING;
    } else if (t == PHIP_TYPE_STRING) {
      d.kind = SEL_ID;
      sel_types[k] = PHIP_TYPE_STRING;
      if (!col_remap[e.column_a]) {
        std::vector<int> ci(nseg);
        for (int s = 0; s < nseg; s++) ci[s] = colidx[s][e.column_a];
        int32_t rc = build_remap(*dev, segs, ci, q->columns[e.column_a], col_remap[e.column_a]);
        if (rc) return rc;
      }
      sel_dicts[k] = col_remap[e.column_a];
    } else {
      d.kind = (t == PHIP_TYPE_INT || t == PHIP_TYPE_LONG) ? SEL_I64 : SEL_F64;
      sel_types[k] = t;
    }
  }
  sq.num_select = nsel;
  sq.limit = std::max<int64_t>(0, q->select_limit);
  int num_projected = 0;
  {
    std::vector<bool> counted = projected;  // (tuple keys: the query's own group-by columns are the projected ones)
    if (P.tuple_keys)
      for (int k = 0; k < (int)P.tuple_dicts.size(); k++) counted[P.tuple_cols[k]] = true;
    for (bool p : counted) num_projected += p ? 1 : 0;
  }

  // group-by key space
  const bool group_by = q->num_group_by > 0;
  int64_t gb_key_space = 0;
  bool gb_force_hash = false;
  std::vector<std::shared_ptr<Device::Remap>> gb_dicts;
  std::vector<std::vector<int32_t *>> gb_remap_dev;  // [k][seg]
  if (group_by) {
    dq.num_group_by = q->num_group_by;
    dq.own_count_rows = nprog > 1 ? 1 : 0;
    int64_t stride = 1;
    for (int k = 0; k < q->num_group_by; k++) {
      int c = q->group_by_columns[k];
      std::vector<int> ci(nseg);
      for (int s = 0; s < nseg; s++) ci[s] = colidx[s][c];
      // the null key (phip_query_desc.null_group_by): one more id, after the dictionary's, when some segment's
      // column holds a null doc
      bool null_key = false;
      if ((q->null_group_by >> k) & 1)
        for (int s = 0; s < nseg; s++) null_key |= segs[s]->cols[ci[s]].nulls != nullptr;
      std::shared_ptr<Device::Remap> r;
      if (P.tuple_keys) {
        r = P.tuple_remap;
      } else {
        int32_t rc = build_remap(*dev, segs, ci, q->columns[c], r, null_key);
        if (rc) return rc;
      }
      gb_dicts.push_back(r);
      const int64_t radix = (int64_t)r->card + (null_key ? 1 : 0);
      P.gb_radix.push_back(radix);
      dq.gb_cols[k] = c;
      dq.gb_stride[k] = stride;
      if ((double)stride * (double)radix > (double)((int64_t)1 << 62))
        return fail(PHIP_ERR_UNSUPPORTED, "group-by key space exceeds 2^62");
      stride *= radix;
    }
    // Dense table (ArrayBasedHolder's role) while the key space is small, or not much larger than the
    // docs that can create groups; above that an open-addressing hash over the keys (IntMapBasedHolder's
    // role, DictionaryBasedGroupKeyGenerator.java:105-186): capacity = the next power of two >= 2x the
    // number of groups possible (min of key space and docs), so probe sequences stay short.
    int64_t docs = 0;
    for (int s = 0; s < nseg; s++) docs += segs[s]->num_docs;
    if (tl_node_docs > 0) docs = tl_node_docs;  // a node plan's part: the node's docs bound the groups
    const char *hm = getenv("PHIP_GB_HASH");  // measurement override: "1" forces the hash table
    const bool force_hash = hm && atoi(hm) != 0;
    gb_key_space = stride;
    gb_force_hash = force_hash;
    if (force_hash || stride > ((int64_t)1 << 26) || (stride > ((int64_t)1 << 22) && stride > 4 * docs)) {
      const int64_t bound = std::max<int64_t>(1, std::min<int64_t>(stride, docs));
      int64_t cap = 1024;
      while (cap < 2 * bound) cap <<= 1;
      if (const char *hc = getenv("PHIP_GB_HASH_CAP"))  // test override: a smaller table, so it must grow and rerun
        cap = std::max<int64_t>(64, std::min<int64_t>(cap, (int64_t)1 << (63 - __builtin_clzll((uint64_t)std::max(2LL, atoll(hc))))));
      const int64_t per_slot = 8 + 8 * (1 + (int64_t)naggs);
      if (cap * per_slot > ((int64_t)24 << 30))
        return fail(PHIP_ERR_UNSUPPORTED, "group-by hash table of %lld slots exceeds the memory budget", (long long)cap);
      dq.num_groups = cap;
      dq.mode = GB_HASH;
    } else {
      dq.num_groups = stride;
    }
  }

  // ---- staging blob: segments, nodes, leaf aux ------------------------------------------------
  Blob blob;
  std::vector<DevNode> nodes;
  std::vector<AuxFix> aux_fix;  // node.aux = dev_base + off
  struct InvLeaf {
    size_t node;
    int seg;
    int col;
    const phip_filter_node *src;
    int entry;  // (segment, program) entry whose program holds the leaf
    int slot;   // index among that entry's inverted leaves
  };
  std::vector<InvLeaf> inv_leaves;
  int num_entries = 0;  // (segment, program) entries, pruned ones included
  int64_t total_work = 0;
  int64_t total_docs = 0;
  std::vector<DevSeg> dsegs;  // (segment, program) entries with work only, segment-major
  dsegs.reserve((size_t)nseg * nprog);
  bool hll_made = false;
  std::vector<bool> hll_doc_used((size_t)nseg * ncols, false);  // (segment, column): HLL entries read by doc
  std::vector<bool> hll_doc16_used((size_t)nseg * ncols, false);  // ... 16-bit ones
  // group-by records (build_records): dense key spaces of dictionary keys, for every group-by the aggregation kernel
  // walks (PHIP_GB_RECORD=0: the columns' own layouts; =1: a record for any number of fields, else from kRecMinFields)
  const char *gre = getenv("PHIP_GB_RECORD");
  const bool rec_want = group_by && dq.mode != GB_HASH && gb_key_space <= ((int64_t)1 << 22) && !want_bitmap &&
                        q->num_group_by <= kRecKeys && !(gre && atoi(gre) == 0);
  const int rec_min_fields = gre && atoi(gre) == 1 ? 1 : kRecMinFields;
  for (int a = 0; a < kMaxAggs; a++) dq.rec_fa[a] = dq.rec_fb[a] = -1;
  const char *hde = getenv("PHIP_HLL_DOC");  // measurement override: "0" = gather the per-id table
  const char *mze = getenv("PHIP_MATERIALIZE");
  const bool hll_doc_on = !(hde && atoi(hde) == 0) && !(mze && atoi(mze) == 0) && !want_bitmap;
  for (int s = 0; s < nseg; s++) {
    Segment &sg = *segs[s];
    total_docs += sg.num_docs;
    DevSeg seg_ds;
    memset(&seg_ds, 0, sizeof(seg_ds));
    DevSeg &ds = seg_ds;
    ds.num_docs = sg.num_docs;
    ds.seg_index = s;
    for (int c = 0; c < ncols; c++) {
      ColumnStore &cs = sg.cols[colidx[s][c]];
      DevCol &dc = ds.cols[c];
      dc.words = cs.words;
      dc.dict = cs.dict;
      dc.raw = cs.raw;
      dc.bits = cs.bits;
      dc.card = cs.card;
      dc.type = cs.type;
      dc.has_dict = !no_dict(cs);
      if (dc.has_dict && as_raw(s, c)) {  // doc-order values of a value-only column
        dc.has_dict = 0;
        if (packed_vals(cs)) {
          dc.raw = nullptr;
          dc.vpack = cs.vpack;
          dc.vbase = cs.vmin;
          dc.vbits = cs.vbits;
        } else {
          dc.raw = cs.vals;
        }
      }
      dc.hll_rows = cs.hll_log2m;
      dc.str_off = cs.str_off;
      dc.planes = cs.planes;
      dc.lds_off = -1;
    }
    for (int a = 0; a < naggs; a++) {
      if (dq.aggs[a].acc != ACC_HLL || dq.aggs[a].expr != PHIP_EXPR_COLUMN) continue;  // (an expression: hashed per doc)
      ColumnStore &cs = sg.cols[colidx[s][dq.aggs[a].col_a]];
      if (cs.fwd_kind == PHIP_FWD_HLL_REGISTERS) continue;  // the register rows are the column's raw values
      if (no_dict(cs)) continue;  // raw values: hashed per doc on the device
      uint32_t *h;
      int32_t rc = ensure_hll(cs, dq.aggs[a].log2m, &h);
      if (rc) return rc;
      ds.cols[dq.aggs[a].col_a].hll = h;
      if (hll_doc_on && cs.words != nullptr && (int64_t)cs.card * 4 >= vals_min && vals_min >= 0) {
        // 16-bit entries where log2m <= 11 (PHIP_HLL_DOC16=0: the 32-bit ones, A/B)
        const char *h16 = getenv("PHIP_HLL_DOC16");
        const bool doc16 = !(h16 && atoi(h16) == 0);
        if (doc16 && dq.aggs[a].log2m <= 11) {
          uint16_t *hd;
          rc = ensure_hll_doc16(sg, cs, dq.aggs[a].log2m, h, st, &hll_made, &hd);
          if (rc) return rc;
          ds.cols[dq.aggs[a].col_a].hll_doc16 = hd;
          hll_doc16_used[(size_t)s * ncols + dq.aggs[a].col_a] = true;
        } else {
          uint32_t *hd;
          rc = ensure_hll_doc(sg, cs, dq.aggs[a].log2m, h, st, &hll_made, &hd);
          if (rc) return rc;
          ds.cols[dq.aggs[a].col_a].hll_doc = hd;
        }
        hll_doc_used[(size_t)s * ncols + dq.aggs[a].col_a] = true;
      }
    }
    for (int k = 0; k < q->num_group_by; k++) {
      DevCol &gc = ds.cols[q->group_by_columns[k]];
      gc.remap = gb_dicts[k]->dev[s];
      if (gb_dicts[k]->raw) gc.gb_base = gb_dicts[k]->raw_base;
      if (!gb_dicts[k]->ids.empty()) gc.gb_ids = gb_dicts[k]->ids[s];  // a raw FLOAT / DOUBLE key: its id column
      if (P.gb_radix[k] > gb_dicts[k]->card) {  // a null-key column: its null docs (if this segment has any)
        gc.gb_nulls = segs[s]->cols[colidx[s][q->group_by_columns[k]]].nulls;
        gc.gb_null_id = gb_dicts[k]->card;
      }
    }
    for (int c = 0; c < ncols; c++)
      if (col_remap[c]) ds.cols[c].remap = col_remap[c]->dev[s];
    if (sg.num_docs == 0) continue;
   // one entry per filter program (adjacent, so the programs of a segment read its columns back to back)
   for (int prog = 0; prog < nprog; prog++) {
    DevSeg ds = seg_ds;
    ds.program = prog;
    ds.seg_index = prog * nseg + s;
    // filter program: validate the preorder ABI tree, then emit postfix with binary AND/OR
    const int nb = q->filter_offsets ? q->filter_offsets[prog * nseg + s] : 0;
    const int ne = q->filter_offsets ? q->filter_offsets[prog * nseg + s + 1] : 0;
    const size_t node_begin = nodes.size();
    ds.node_begin = (int32_t)node_begin;
    int64_t hull_lo = 0, hull_hi = (int64_t)sg.num_docs - 1;  // candidate docs (inclusive)
    if (ne > nb) {
      std::vector<int> next(ne - nb);
      std::string err;
      int after = validate_tree(q->filter_nodes, nb, ne, nb, 0, ncols, next, err);
      if (after < 0) return fail(PHIP_ERR_INVALID, "segment %d filter: %s", s, err.c_str());
      if (after != ne) return fail(PHIP_ERR_INVALID, "segment %d filter: trailing nodes", s);
      int32_t rc = PHIP_OK;
      // leaf -> device node
      auto make_leaf = [&](const phip_filter_node &fn) -> DevNode {
        DevNode dn;
        memset(&dn, 0, sizeof(dn));
        dn.op = DOP_LEAF;
        dn.leaf_kind = fn.leaf_kind;
        dn.column = fn.column;
        dn.lo = fn.lo;
        dn.hi = fn.hi;
        dn.exclusive = fn.exclusive;
        dn.count = fn.count;
        dn.lds_off = -1;
        dn.skip_to = -1;
        const size_t ni = nodes.size();
        ColumnStore *cs = (fn.leaf_kind >= PHIP_LEAF_DICT_RANGE && fn.leaf_kind != PHIP_LEAF_DOC_RANGES)
                              ? &sg.cols[colidx[s][fn.column]]
                              : nullptr;
        if (cs) dn.bits = cs->bits;
        switch (fn.leaf_kind) {
          case PHIP_LEAF_DICT_RANGE:
            if (no_dict(*cs)) { rc = fail(PHIP_ERR_INVALID, "dict leaf on raw column"); break; }
            dn.lo = std::max(0, fn.lo);
            dn.hi = std::min(cs->card, fn.hi);
            if (dn.hi <= dn.lo) dn.leaf_kind = PHIP_LEAF_MATCH_NONE;
            else if (dn.lo == 0 && dn.hi == cs->card) dn.leaf_kind = PHIP_LEAF_MATCH_ALL;
            break;
          case PHIP_LEAF_DICT_SET: {
            if (no_dict(*cs)) { rc = fail(PHIP_ERR_INVALID, "dict leaf on raw column"); break; }
            std::vector<uint32_t> bits(ceil_div(cs->card, 32) + 1, 0);
            int32_t n_in = 0, mn = INT32_MAX, mx = -1;
            for (int k = 0; k < fn.count; k++) {
              int32_t id = fn.ids[k];
              if (id < 0 || id >= cs->card) { rc = fail(PHIP_ERR_INVALID, "dict id %d out of range", id); break; }
              if (!((bits[id >> 5] >> (id & 31)) & 1u)) n_in++;
              bits[id >> 5] |= 1u << (id & 31);
              mn = std::min(mn, id);
              mx = std::max(mx, id);
            }
            if (rc) break;
            // a contiguous id set (or its complement within the dictionary) is a dict-id range
            const bool contiguous = n_in > 0 && mx - mn + 1 == n_in;
            if (cs->bits <= kBitSliceMaxBits) {  // the matching ids as runs (the bit-sliced conjunction ORs <= 4)
              int nr = 0;
              bool prev = false;
              for (int id = 0; id <= cs->card && nr <= 4; id++) {
                const bool in = id < cs->card && (((bits[id >> 5] >> (id & 31)) & 1u) != 0) != (fn.exclusive != 0);
                if (in && !prev) {
                  if (nr < 4) dn.bs_runs[nr] = (uint32_t)id;
                  nr++;
                } else if (!in && prev && nr <= 4) {
                  dn.bs_runs[nr - 1] |= (uint32_t)(id - 1) << 16;
                }
                prev = in;
              }
              dn.bs_nruns = nr <= 4 && cs->card <= 65536 ? nr : 0;
            }
            if (n_in == 0) {
              dn.leaf_kind = fn.exclusive ? PHIP_LEAF_MATCH_ALL : PHIP_LEAF_MATCH_NONE;
            } else if (n_in == cs->card) {
              dn.leaf_kind = fn.exclusive ? PHIP_LEAF_MATCH_NONE : PHIP_LEAF_MATCH_ALL;
            } else if (contiguous && !fn.exclusive) {
              dn.leaf_kind = PHIP_LEAF_DICT_RANGE;
              dn.lo = mn;
              dn.hi = mx + 1;
            } else if (contiguous && fn.exclusive && (mn == 0 || mx == cs->card - 1)) {
              dn.leaf_kind = PHIP_LEAF_DICT_RANGE;
              dn.lo = mn == 0 ? mx + 1 : 0;
              dn.hi = mn == 0 ? cs->card : mn;
              dn.exclusive = 0;
            } else if (cs->card <= 64) {
              dn.small_set = 1;
              dn.set_mask = (uint64_t)bits[0] | ((uint64_t)bits[1] << 32);
              if (fn.exclusive) dn.set_mask = ~dn.set_mask;  // ids >= card never occur
              dn.exclusive = 0;
            } else {
              dn.count = (int32_t)bits.size();  // bitset words (filter.hip: <= 64 words ride in one VGPR per lane)
              aux_fix.push_back({ni, blob.add(bits.data(), bits.size() * 4)});
            }
            break;
          }
          case PHIP_LEAF_DOC_RANGES: {
            int32_t prev = -1;
            for (int k = 0; k < fn.count; k++) {
              int32_t a0 = fn.ids[2 * k], a1 = fn.ids[2 * k + 1];
              if (a0 <= prev || a1 < a0 || a1 >= sg.num_docs) {
                rc = fail(PHIP_ERR_INVALID, "doc ranges must be sorted, disjoint and within numDocs");
                break;
              }
              prev = a1;
            }
            if (rc) break;
            if (fn.count == 0) {
              dn.leaf_kind = PHIP_LEAF_MATCH_NONE;
            } else {
              dn.lo = fn.ids[0];
              dn.hi = fn.ids[2 * fn.count - 1];
              aux_fix.push_back({ni, blob.add(fn.ids, (size_t)fn.count * 8)});
            }
            break;
          }
          case PHIP_LEAF_RAW_RANGE:
          case PHIP_LEAF_RAW_SET:
            if (cs->fwd_kind != PHIP_FWD_RAW_CHUNK) { rc = fail(PHIP_ERR_INVALID, "raw leaf on a column without raw values"); break; }
            if (cs->type == PHIP_TYPE_STRING) { rc = fail(PHIP_ERR_INVALID, "STRING column: use the RAW_STRING leaves"); break; }
            if (fn.leaf_kind == PHIP_LEAF_RAW_SET) {
              // the kernel binary-searches the values (filter.hip sorted_contains): sorted, distinct, and for
              // FLOAT / DOUBLE columns without NaN (IEEE equality never matches it)
              const int64_t nv = fn.count / 2;
              std::vector<int64_t> vi;
              std::vector<double> vf;
              const bool real = cs->type == PHIP_TYPE_FLOAT || cs->type == PHIP_TYPE_DOUBLE;
              for (int64_t k = 0; k < nv; k++) {
                int64_t x;
                memcpy(&x, fn.ids + 2 * k, 8);
                if (!real) {
                  vi.push_back(x);
                } else {
                  double d;
                  memcpy(&d, &x, 8);
                  if (d == d) vf.push_back(d);
                }
              }
              std::sort(vi.begin(), vi.end());
              vi.erase(std::unique(vi.begin(), vi.end()), vi.end());
              std::sort(vf.begin(), vf.end());
              vf.erase(std::unique(vf.begin(), vf.end()), vf.end());  // (-0.0 and 0.0 compare equal: one kept)
              dn.count = (int32_t)(real ? vf.size() : vi.size());
              if (dn.count == 0) {
                dn.leaf_kind = fn.exclusive ? PHIP_LEAF_MATCH_ALL : PHIP_LEAF_MATCH_NONE;
                break;
              }
              aux_fix.push_back({ni, real ? blob.add(vf.data(), vf.size() * 8) : blob.add(vi.data(), vi.size() * 8)});
              break;
            }
            aux_fix.push_back({ni, blob.add(fn.ids, (size_t)fn.count * 4)});
            break;
          case PHIP_LEAF_RAW_STRING_RANGE:
          case PHIP_LEAF_RAW_STRING_SET:
            if (cs->fwd_kind != PHIP_FWD_RAW_CHUNK || cs->type != PHIP_TYPE_STRING || cs->str_off == nullptr) {
              rc = fail(PHIP_ERR_INVALID, "raw STRING leaf on column %s, which holds no raw STRING values", cs->name.c_str());
              break;
            }
            rc = raw_string_leaf(fn, dn, blob, aux_fix, ni);
            break;
          case PHIP_LEAF_NULL:
            // the column's resident null doc words, read like an inverted leaf's words (one 256-byte region per tile)
            if (cs->nulls == nullptr) {
              dn.leaf_kind = fn.exclusive ? PHIP_LEAF_MATCH_ALL : PHIP_LEAF_MATCH_NONE;
              dn.exclusive = 0;
              break;
            }
            dn.leaf_kind = PHIP_LEAF_INVERTED;
            dn.aux = cs->nulls;
            dn.aux_stride = 32;
            dn.count = 0;
            dn.bits = 0;
            break;
          case PHIP_LEAF_INVERTED:
            if (cs->inv_begin.empty()) { rc = fail(PHIP_ERR_INVALID, "column %s has no inverted index", cs->name.c_str()); break; }
            {
              int slot = 0;
              for (const InvLeaf &o : inv_leaves) slot += o.entry == num_entries ? 1 : 0;
              inv_leaves.push_back({ni, s, colidx[s][fn.column], &fn, num_entries, slot});
            }
            break;
          default: break;
        }
        return dn;
      };
      // recursive postfix emission (depth bounded by validate_tree)
      std::function<void(int)> emit = [&](int idx) {
        if (rc) return;
        const phip_filter_node &fn = q->filter_nodes[idx];
        if (fn.op == PHIP_NODE_LEAF) {
          DevNode dn = make_leaf(fn);
          nodes.push_back(dn);
          return;
        }
        if (fn.op == PHIP_NODE_NOT) {
          emit(idx + 1);
          DevNode dn;
          memset(&dn, 0, sizeof(dn));
          dn.op = DOP_NOT;
          dn.lds_off = -1;
          dn.skip_to = -1;
          nodes.push_back(dn);
          return;
        }
        int c = idx + 1;
        for (int k = 0; k < fn.num_children && !rc; k++) {
          const size_t first = nodes.size();
          emit(c);
          if (k > 0) {
            DevNode dn;
            memset(&dn, 0, sizeof(dn));
            dn.op = fn.op == PHIP_NODE_AND ? DOP_AND : DOP_OR;
            dn.lds_off = -1;
            dn.skip_to = -1;
            nodes.push_back(dn);
            // the child's first node is its leftmost leaf: skip the child when the node is decided
            nodes[first].skip_kind = fn.op == PHIP_NODE_AND ? SKIP_IF_NONE : SKIP_IF_ALL;
            nodes[first].skip_to = (int32_t)nodes.size();
          }
          c = next[c - nb];
        }
      };
      emit(nb);
      if (rc) return rc;
      // stack depth and candidate-doc hull (SortedIndexBasedFilterOperator ranges under ANDs)
      struct Hull {
        int64_t lo, hi;
      };
      std::vector<Hull> hst;
      int sp = 0, maxsp = 0;
      const int64_t full_hi = (int64_t)sg.num_docs - 1;
      for (size_t i = node_begin; i < nodes.size(); i++) {
        const DevNode &dn = nodes[i];
        if (dn.op == DOP_LEAF) {
          sp++;
          Hull h{0, full_hi};
          if (dn.leaf_kind == PHIP_LEAF_MATCH_NONE) h = {1, 0};
          if (dn.leaf_kind == PHIP_LEAF_DOC_RANGES) h = {dn.lo, dn.hi};  // first start .. last end
          hst.push_back(h);
        } else if (dn.op == DOP_NOT) {
          hst.back() = {0, full_hi};
        } else {
          sp--;
          Hull b = hst.back();
          hst.pop_back();
          Hull a = hst.back();
          if (dn.op == DOP_AND) hst.back() = {std::max(a.lo, b.lo), std::min(a.hi, b.hi)};
          else if (a.lo > a.hi) hst.back() = b;
          else if (b.lo > b.hi) hst.back() = a;
          else hst.back() = {std::min(a.lo, b.lo), std::max(a.hi, b.hi)};
        }
        maxsp = std::max(maxsp, sp);
      }
      if (maxsp > kMaxFilterStack) return fail(PHIP_ERR_UNSUPPORTED, "segment %d filter needs stack depth %d", s, maxsp);
      hull_lo = hst.back().lo;
      hull_hi = hst.back().hi;
    }
    ds.node_end = (int32_t)nodes.size();
    num_entries++;
    if (hull_lo > hull_hi) continue;  // no candidate doc: the segment is pruned (no work)
    ds.tile0 = (int32_t)(hull_lo / kTileDocs);
    ds.num_work = (int32_t)(hull_hi / kTileDocs - ds.tile0 + 1);
    ds.work_begin = (int32_t)total_work;
    total_work += ds.num_work;
    dsegs.push_back(ds);
   }
  }
  if (hll_made) HIP_TRY(hipStreamSynchronize(st));
  if (total_work > INT32_MAX / 2) return fail(PHIP_ERR_UNSUPPORTED, "too many tiles in one query");
  dq.total_work = (int32_t)total_work;
  if (group_by && gb_key_space > ((int64_t)1 << 22) && tl_node_docs == 0) {  // (node parts: sized by the node's docs)
    // Re-size a large group table from the docs of the work tiles (sorted-index pruning already cut them):
    // only those docs can create groups, and the table is cleared and compacted on every execution
    // (BenchmarkQueries STARTREE_FILTER_QUERY: one candidate tile, yet 2 x 10M hash slots before).
    const int64_t work_docs = std::max<int64_t>(1, total_work * (int64_t)kTileDocs);
    if (gb_force_hash || gb_key_space > ((int64_t)1 << 26) || gb_key_space > 4 * work_docs) {
      const int64_t bound = std::max<int64_t>(1, std::min<int64_t>(gb_key_space, work_docs));
      int64_t cap = 1024;
      while (cap < 2 * bound) cap <<= 1;
      if (const char *hc = getenv("PHIP_GB_HASH_CAP"))
        cap = std::max<int64_t>(64, std::min<int64_t>(cap, (int64_t)1 << (63 - __builtin_clzll((uint64_t)std::max(2LL, atoll(hc))))));
      if (dq.mode != GB_HASH || cap < dq.num_groups) {
        const int64_t per_slot = 8 + 8 * (1 + (int64_t)naggs);
        if (cap * per_slot > ((int64_t)24 << 30))
          return fail(PHIP_ERR_UNSUPPORTED, "group-by hash table of %lld slots exceeds the memory budget", (long long)cap);
        dq.num_groups = cap;
        dq.mode = GB_HASH;
      }
    }
  }
  dq.num_segs = (int32_t)dsegs.size();
  const size_t segs_off = blob.reserve(sizeof(DevSeg) * std::max<size_t>(dsegs.size(), 1));

  // inverted leaves: dense doc words per leaf + roaring container tasks. The L inverted leaves of one
  // (segment, program) entry are interleaved per 2048-doc tile -- tile t holds leaf 0's 32 words, then leaf
  // 1's, ... -- so the filter kernel stages all of them with one L x 256-byte LDS-DMA region per tile instead of
  // L quarter-filled 256-byte ones.
  std::vector<RoaringTask> tasks;
  size_t inv_words_total = 0;
  std::vector<size_t> inv_word_off(inv_leaves.size()), inv_word_nw(inv_leaves.size());
  std::vector<int> entry_leaves(num_entries, 0);
  std::vector<size_t> entry_off(num_entries, 0);
  for (const InvLeaf &L : inv_leaves) entry_leaves[L.entry]++;
  for (size_t i = 0; i < inv_leaves.size(); i++) {
    const InvLeaf &L = inv_leaves[i];
    const Segment &sg = *segs[L.seg];
    size_t nw = (size_t)std::max(round_up(sg.num_docs, 65536), round_up(sg.num_docs, kTileDocs)) / 64;  // whole keys
    inv_word_nw[i] = nw;
    if (L.slot == 0) {
      entry_off[L.entry] = inv_words_total;
      inv_words_total += nw * entry_leaves[L.entry];
    }
    inv_word_off[i] = entry_off[L.entry] + 32 * (size_t)L.slot;
  }
  std::vector<int32_t> node_inv_stride(nodes.size(), 0);   // u64 words per tile of an inverted leaf's aux
  std::vector<int32_t> node_inv_slot(nodes.size(), 0);
  std::vector<int32_t> node_inv_leaves(nodes.size(), 0);
  void *inv_words = nullptr;
  if (inv_words_total) {
    int32_t rc = P.alloc(inv_words_total * 8, &inv_words);
    if (rc) return rc;
  }
  std::vector<RoaringGroup> rgroups;
  for (size_t i = 0; i < inv_leaves.size(); i++) {
    const InvLeaf &L = inv_leaves[i];
    const ColumnStore &cs = segs[L.seg]->cols[L.col];
    uint64_t *words = (uint64_t *)inv_words + inv_word_off[i];
    const int32_t tile_words = 32 * entry_leaves[L.entry];
    nodes[L.node].aux = words;
    nodes[L.node].aux_stride = tile_words;
    node_inv_stride[L.node] = tile_words;
    node_inv_slot[L.node] = L.slot;
    node_inv_leaves[L.node] = entry_leaves[L.entry];
    const size_t first = tasks.size();
    for (int k = 0; k < L.src->count; k++) {
      int32_t id = L.src->ids[k];
      if (id < 0 || id >= cs.card) return fail(PHIP_ERR_INVALID, "inverted dict id %d out of range", id);
      for (int64_t ci = cs.inv_begin[id]; ci < cs.inv_begin[id + 1]; ci++) {
        const Container &ct = cs.inv_conts[ci];
        RoaringTask t;
        t.payload = cs.inv_blob + ct.off;
        t.out_words = words;
        t.key = ct.key;
        t.kind = ct.kind;
        t.card = ct.card;
        t.pad = 0;
        tasks.push_back(t);
      }
    }
    // group the leaf's containers by key (one LDS-decoding workgroup per key); every key of the leaf's words
    // gets a group -- one without containers stores zeros -- so the words need no clearing pass
    std::stable_sort(tasks.begin() + first, tasks.end(),
                     [](const RoaringTask &a, const RoaringTask &b) { return a.key < b.key; });
    if (tasks.size() > (size_t)INT32_MAX) return fail(PHIP_ERR_UNSUPPORTED, "too many inverted-index containers");
    const int32_t nkeys = (int32_t)(inv_word_nw[i] / 1024);
    size_t t = first;
    for (int32_t key = 0; key < nkeys; key++) {
      size_t e = t;
      while (e < tasks.size() && tasks[e].key == key) e++;
      RoaringGroup g;
      g.out_words = words;
      g.task_begin = (int32_t)t;
      g.task_end = (int32_t)e;
      g.key = key;
      g.tile_words = tile_words;
      rgroups.push_back(g);
      t = e;
    }
    if (t != tasks.size()) return fail(PHIP_ERR_INVALID, "inverted-index container key beyond the segment's docs");
  }
  const size_t tasks_off = tasks.empty() ? 0 : blob.add(tasks.data(), tasks.size() * sizeof(RoaringTask));
  const size_t rgroups_off = rgroups.empty() ? 0 : blob.add(rgroups.data(), rgroups.size() * sizeof(RoaringGroup));

  // ---- filter kernel configuration (filter.hip) -------------------------------------------------
  // Per 2048-doc tile, the wave's ring slot receives the fixed-bit words of every scanned filter column
  // (256*b bytes) and the dense words of inverted leaves (256 bytes), each padded by kStagePad bytes on
  // both sides (window_at reads one word before / after). Value / group-by columns are not staged:
  // the aggregation kernel reads them for matched docs only.
  bool has_filter = false;
  for (const DevSeg &ds : dsegs) has_filter |= ds.node_end > ds.node_begin;
  bool need_agg = group_by || nprog > 1;  // several programs: every COUNT is per program, in the aggregation walk
  for (int a = 0; a < naggs; a++) need_agg |= dq.aggs[a].acc != ACC_COUNT;
  bool need_mask = has_filter && (need_agg || want_bitmap || nsel > 0);
  const int64_t kSlotBudget = 19 * 1024;  // bytes per ring slot
  int32_t stage_stride = 0;
  std::vector<double> seg_est(dsegs.size(), 1.0);
  std::vector<int32_t> seg_off(dsegs.size(), 0);
  for (DevSeg &ds : dsegs) {
    int32_t off = 0;
    ds.num_stage = 0;
    ds.num_dma = 0;
    auto add_region = [&](const uint8_t *rbase, int32_t bytes) -> int32_t {
      if (ds.num_stage >= kMaxStage || off + bytes + 2 * kStagePad > kSlotBudget) return -1;
      const int32_t lds_off = off + kStagePad;
      ds.stage[ds.num_stage++] = {rbase, bytes, lds_off};
      ds.num_dma += (int32_t)ceil_div(bytes, 1024);
      off += bytes + 2 * kStagePad;
      return lds_off;
    };
    int32_t inv_region = -2;  // -2: not added yet, -1: did not fit
    // A program that is an AND of dict-id ranges (plus single sorted-index ranges) over columns with a bit-sliced
    // copy stages the planes instead of the packed words and takes the bit-sliced conjunctive path (filter.hip
    // eval_conj_bs); the packed words stay the source of every other use (values, the interpreter paths)
    bool bs = getenv("PHIP_NO_BITSLICE") == nullptr && ds.node_end > ds.node_begin;
    for (int i = ds.node_begin; i < ds.node_end && bs; i++) {
      const DevNode &dn = nodes[i];
      if (dn.op == DOP_AND || (dn.op == DOP_LEAF && dn.leaf_kind == PHIP_LEAF_MATCH_ALL)) continue;
      if (dn.op == DOP_LEAF && dn.leaf_kind == PHIP_LEAF_DOC_RANGES && dn.count == 1) continue;
      bs = dn.op == DOP_LEAF && (dn.leaf_kind == PHIP_LEAF_DICT_RANGE || dn.leaf_kind == PHIP_LEAF_DICT_SET) &&
           ds.cols[dn.column].planes != nullptr &&
           (dn.leaf_kind == PHIP_LEAF_DICT_RANGE || bs_small_set(dn, ds.cols[dn.column]) || bs_runs_set(dn));
    }
    if (bs) {  // every column's planes must fit the slot (else the packed words, as the interpreter reads them)
      std::vector<int> cols_seen;
      int64_t need = 0;
      for (int i = ds.node_begin; i < ds.node_end; i++) {
        const DevNode &dn = nodes[i];
        if (dn.op != DOP_LEAF || (dn.leaf_kind != PHIP_LEAF_DICT_RANGE && dn.leaf_kind != PHIP_LEAF_DICT_SET)) continue;
        if (std::find(cols_seen.begin(), cols_seen.end(), dn.column) != cols_seen.end()) continue;
        cols_seen.push_back(dn.column);
        need += 256ll * ds.cols[dn.column].bits + 2 * kStagePad;
      }
      bs = (int)cols_seen.size() <= kMaxStage && need <= kSlotBudget;
    }
    std::vector<std::pair<int, int32_t>> bs_regions;  // column -> its planes' region
    for (int i = ds.node_begin; i < ds.node_end; i++) {
      DevNode &dn = nodes[i];
      if (dn.op != DOP_LEAF) continue;
      if (bs && (dn.leaf_kind == PHIP_LEAF_DICT_RANGE || dn.leaf_kind == PHIP_LEAF_DICT_SET)) {
        const DevCol &dc = ds.cols[dn.column];
        int32_t r = -2;
        for (const auto &p : bs_regions) r = p.first == dn.column ? p.second : r;
        if (r == -2) {
          r = add_region((const uint8_t *)dc.planes, 256 * dc.bits);
          bs_regions.push_back({dn.column, r});
        }
        dn.lds_off = r;  // (fits: checked above)
        continue;
      }
      if (dn.leaf_kind == PHIP_LEAF_DICT_RANGE || dn.leaf_kind == PHIP_LEAF_DICT_SET) {
        DevCol &dc = ds.cols[dn.column];
        if (dc.lds_off < 0) dc.lds_off = add_region((const uint8_t *)dc.words, 256 * dc.bits);
        dn.lds_off = dc.lds_off;
      } else if (dn.leaf_kind == PHIP_LEAF_INVERTED && dn.aux != nullptr && node_inv_leaves[i] == 0) {
        dn.lds_off = add_region((const uint8_t *)dn.aux, 256);  // a null vector: the column's own resident words
      } else if (dn.leaf_kind == PHIP_LEAF_INVERTED && dn.aux != nullptr) {
        // the entry's interleaved inverted words: one region of L x 256 bytes per tile, leaf j at 256 j
        if (inv_region == -2) {
          const uint64_t *entry_base = (const uint64_t *)dn.aux - 32 * node_inv_slot[i];
          inv_region = add_region((const uint8_t *)entry_base, 256 * node_inv_leaves[i]);
        }
        dn.lds_off = inv_region < 0 ? -1 : inv_region + 256 * node_inv_slot[i];
      }
    }
    stage_stride = std::max(stage_stride, off);
    // conjunctive fast path: a program made of AND nodes over staged range / small-set scan leaves and
    // single-range sorted-index leaves (doc ranges intersected; the tiles outside are already pruned), or
    // no program at all (every doc of the segment)
    ds.conj = 0;
    ds.conj_path = 0;
    ds.conj_range = 0;
    ds.conj_lo = 0;
    ds.conj_hi = ds.num_docs - 1;
    std::vector<std::pair<double, ConjLeaf>> conj;
    bool ok = true;
    double est = 1.0;  // estimated selectivity of the program (product of the leaves')
    for (int i = ds.node_begin; i < ds.node_end && ok; i++) {
      const DevNode &dn = nodes[i];
      if (dn.op == DOP_AND) continue;
      if (dn.op == DOP_LEAF && dn.leaf_kind == PHIP_LEAF_MATCH_ALL) continue;
      if (dn.op == DOP_LEAF && dn.leaf_kind == PHIP_LEAF_DOC_RANGES && dn.count == 1) {
        ds.conj_range = 1;
        ds.conj_lo = std::max(ds.conj_lo, dn.lo);
        ds.conj_hi = std::min(ds.conj_hi, dn.hi);
        est *= double(std::max(0, dn.hi - dn.lo + 1)) / std::max(1, ds.num_docs);
        continue;
      }
      if (dn.op != DOP_LEAF || dn.lds_off < 0 ||
          !(dn.leaf_kind == PHIP_LEAF_DICT_RANGE || (dn.leaf_kind == PHIP_LEAF_DICT_SET && dn.small_set) ||
            (bs && bs_runs_set(dn)))) {
        ok = false;
        break;
      }
      const int card = std::max(1, ds.cols[dn.column].card);
      ConjLeaf L;
      memset(&L, 0, sizeof(L));
      L.lds_off = dn.lds_off;
      L.bits = dn.bits;
      double sel;
      if (bs && dn.leaf_kind == PHIP_LEAF_DICT_SET && bs_runs_set(dn)) {  // OR of <= 4 id runs over the planes
        L.kind = 4;
        L.set_mask = (uint64_t)dn.bs_runs[0] | ((uint64_t)dn.bs_runs[1] << 32);
        L.lo = dn.bs_runs[2];
        L.span = dn.bs_runs[3];
        L.pad = dn.bs_nruns;
        int64_t n = 0;
        for (int r = 0; r < dn.bs_nruns; r++) n += (int64_t)(dn.bs_runs[r] >> 16) - (dn.bs_runs[r] & 0xffff) + 1;
        sel = double(n) / card;
      } else if (bs && dn.leaf_kind == PHIP_LEAF_DICT_SET) {  // (a few ids of a dictionary of <= 64: bs_small_set)
        L.kind = 3;
        L.set_mask = dn.set_mask & (card >= 64 ? ~0ull : ((1ull << card) - 1));
        sel = double(__builtin_popcountll(L.set_mask)) / card;
      } else if (bs) {  // (every other leaf a DICT_RANGE whose planes are staged)
        L.kind = 2;
        L.lo = (uint32_t)dn.lo;
        L.span = (uint32_t)(dn.hi - 1);
        L.pad = (dn.lo > 0 ? 1 : 0) | (dn.hi < card ? 2 : 0);  // (ids >= card never occur)
        sel = double(dn.hi - dn.lo) / card;
      } else if (dn.leaf_kind == PHIP_LEAF_DICT_RANGE) {
        L.kind = 0;
        L.lo = (uint32_t)dn.lo << (32 - dn.bits);
        L.span = (uint32_t)(dn.hi - dn.lo) << (32 - dn.bits);
        sel = double(dn.hi - dn.lo) / card;
      } else {
        L.kind = 1;
        L.set_mask = dn.set_mask;
        const uint64_t in_dict = card >= 64 ? ~0ull : ((1ull << card) - 1);
        sel = double(__builtin_popcountll(dn.set_mask & in_dict)) / card;
      }
      est *= sel;
      conj.push_back({sel, L});
    }
    if (ds.conj_range && ds.conj_lo > ds.conj_hi) ok = false;  // (empty: the host pruned the segment already)
    if (ok && (int)conj.size() <= kMaxConj) {
      ds.conj_path = 1;
      seg_est[&ds - dsegs.data()] = est;
      // most selective leaf first: the short-circuit then skips the others on more tiles (AND is
      // commutative, so the doc set is unchanged)
      std::stable_sort(conj.begin(), conj.end(),
                       [](const std::pair<double, ConjLeaf> &a, const std::pair<double, ConjLeaf> &b) { return a.first < b.first; });
      ds.conj = (int32_t)conj.size();
      ds.conj_bs = bs ? 1 : 0;
      ds.conj_sparse = bs ? 0 : 1;
      for (size_t i = 1; i < conj.size(); i++) ds.conj_sparse &= conj[i].second.kind == 0 ? 1 : 0;
      // the per-doc walk pays when the first leaf leaves ~2 docs per lane; at a selectivity of 1/7 (unsorted SSB
      // Q1.1's D_YEAR) tiles often pass the per-tile bound yet the walk is slower than the dense leaves (filter kernel
      // 0.32 -> 0.30 ms without it, profiles/r03f_unsorted_filter_knobs_ab.log), so it needs a selective first leaf
      if (conj.empty() || conj[0].first > kConjSparseSel) ds.conj_sparse = 0;
      if (getenv("PHIP_NO_SPARSE")) ds.conj_sparse = 0;  // measurement override
      // the value is the per-lane passing-doc bound under which the sparse walk is taken
      if (ds.conj_sparse) {
        const char *sm = getenv("PHIP_SPARSE_MAX");  // measurement override
        ds.conj_sparse = sm ? std::max(1, std::min(32, atoi(sm))) : kConjSparseMax;
      }
      ds.conj_p = 8;
      for (size_t i = 0; i < conj.size(); i++) {
        ds.conj_leaf[i] = conj[i].second;
        while (ds.conj_p > 1 && ds.conj_p * conj[i].second.bits > 32) ds.conj_p >>= 1;
      }
      if (const char *e = getenv("PHIP_CONJ_P")) ds.conj_p = std::min(ds.conj_p, std::max(1, atoi(e)));  // measurement override
    }
    // general programs whose leaves are all staged (or need no tile data) run in the contiguous layout
    // (filter.hip eval_filter_contig): inverted leaves become one LDS read, scan leaves one register block
    ds.contig = 0;
    if (!ds.conj_path && ds.node_end > ds.node_begin) {
      bool c = true;
      for (int i = ds.node_begin; i < ds.node_end && c; i++) {
        const DevNode &dn = nodes[i];
        if (dn.op != DOP_LEAF) continue;
        switch (dn.leaf_kind) {
          case PHIP_LEAF_MATCH_ALL:
          case PHIP_LEAF_MATCH_NONE:
          case PHIP_LEAF_DOC_RANGES: break;
          case PHIP_LEAF_INVERTED: c = dn.lds_off >= 0; break;
          case PHIP_LEAF_DICT_RANGE: c = dn.lds_off >= 0 && dn.bits >= 1 && dn.bits <= 31; break;
          case PHIP_LEAF_DICT_SET:
            c = dn.lds_off >= 0 && dn.bits >= 1 && dn.bits <= 31 && (dn.small_set || (dn.count > 0 && dn.count <= 64));
            break;
          default: c = false;
        }
      }
      const char *ce = getenv("PHIP_CONTIG");  // measurement override: "0" keeps the lane-major interpreter
      ds.contig = c && !(ce && ce[0] == '0') ? 1 : 0;
    }
    seg_off[&ds - dsegs.data()] = off;
  }
  // group-by records, from each entry's estimated selectivity (build_records' touched-lines model)
  if (rec_want) {
    bool made = false;
    for (size_t i = 0; i < dsegs.size(); i++) {
      const int s = dsegs[i].seg_index % nseg;
      int32_t rc = build_records(*segs[s], q, dq, dsegs[i], colidx[s], rec_min_fields, seg_est[i], st, &made);
      if (rc) return rc;
    }
    if (made) HIP_TRY(hipStreamSynchronize(st));
    // A few record segments do not pay for the record variant's larger kernel on all the others (Q3.1: records on
    // its sparse edge segments only ran 0.47 -> 0.52 ms, profiles/r06zj_trace.log): records for most docs, or none.
    int64_t rec_docs = 0, all_docs = 0;
    for (const DevSeg &d : dsegs) {
      all_docs += d.num_docs;
      rec_docs += d.rec != nullptr ? d.num_docs : 0;
    }
    if (rec_min_fields > 1 && 2 * rec_docs < all_docs)
      for (DevSeg &d : dsegs) d.rec = nullptr;
  }
  // Fused aggregation (filter.hip fused_tile): every segment on the conjunctive path, aggregation only
  // (no group-by, no HLL), at most 4 slots, a filter to fuse into. Value columns are then streamed with
  // the tile (one more LDS-DMA region) when the expected matches per 128-byte line of the column reach
  // kStreamValueMin -- a dense gather would touch every line anyway -- else gathered for matched docs.
  bool conj_all = true;
  for (const DevSeg &ds : dsegs) conj_all &= ds.conj_path != 0;
  bool any_filter_prog = false;
  for (const DevSeg &ds : dsegs) any_filter_prog |= ds.node_end > ds.node_begin;
  int fused_naggs = 0;
  bool any_defer = false;
  std::vector<bool> ids_streamed((size_t)nseg * ncols, false);  // (segment, column): fused tiles stream its ids
  {
    // Fusion saves a launch, the mask round trip and the filter columns' re-read, but a streaming filter
    // wave that stops for a tile's projection gathers leaves its LDS-DMA ring idle. Measured on SSB SF100
    // (tools/ab_env.sh, profiles/r02_*): fused wins while the query has at most a few thousand work tiles
    // (Q1.2 / Q1.3 over the sorted layout: 0.112 -> 0.081 / 0.066 -> 0.057 ms p50) and loses beyond
    // (Q1.1 sorted, 44K tiles: 0.207 -> 0.270 ms; unsorted, 293K tiles: 1.6 -> 2.4 ms per step).
    // Fusing sparse queries whatever their size (estimated matches per work tile from the leaf selectivities) was
    // measured slower: unsorted Q1.2 / Q1.3 (~1 match per tile, 293K tiles) 0.49 / 0.51 ms split vs 0.55 / 0.74 ms
    // fused (profiles/r03b_fuse_sparse_ab.log: deferred or per-tile gathers, XCD or contiguous walk alike) -- the
    // fused kernel's larger register / LDS footprint costs the stream more than the mask walk it saves. The rule
    // stays as a measurement override (PHIP_FUSE_PER_TILE), off by default.
    const char *fe = getenv("PHIP_FUSE");  // measurement override: "0" never, "1" always, unset = by size
    const int64_t kFuseMaxTiles = 8192;
    double est_docs = 0.0;
    for (size_t i = 0; i < dsegs.size(); i++) est_docs += seg_est[i] * dsegs[i].num_docs;
    const double per_tile = est_docs / (double)std::max<int64_t>(1, total_work);
    double fuse_per_tile = 0.0;
    if (const char *fp = getenv("PHIP_FUSE_PER_TILE")) fuse_per_tile = atof(fp);  // measurement override
    // Large scans fuse too since the bit-sliced conjunction (round 3): its light evaluation leaves the wave time to
    // gather a deferred batch of matched docs' values, and the split's mask round trip is gone -- unsorted SSB
    // Q1.1 / Q1.2 / Q1.3 p50 0.64 / 0.476 / 0.487 -> 0.62 / 0.385 / 0.476 ms, sorted Q1.1 unchanged
    // (profiles/r03n_fuse_large_ab.log). Their value columns are gathered, not streamed with every tile (streaming
    // LO_EXTENDEDPRICE over 293K tiles: 1.4 ms). PHIP_FUSE_LARGE=0 restores the size rule alone.
    const bool big = total_work > kFuseMaxTiles;
    // A small query whose tiles are mostly matched (estimated >= kFuseDenseSplit docs per 2048-doc tile) splits: the
    // aggregation kernel's dense-tile walk projects a tile's matched docs four groups per gather round trip, where the
    // fused tile drains them through its deferred ring 128 at a time, one round trip each (C1 on 10M rows,
    // profiles/r06d_c1_ab.log: FILTERED_QUERY, 88 % matched, p50 0.199 -> 0.113 ms split).
    const double kFuseDenseSplit = 1024.0;
    const bool dense_small = !big && per_tile >= kFuseDenseSplit;
    const char *fl = getenv("PHIP_FUSE_LARGE");  // measurement override
    bool bs_all = true;  // (the P-layout conjunction's heavier evaluation keeps the size rule)
    for (const DevSeg &ds : dsegs) bs_all &= ds.conj == 0 || ds.conj_bs != 0;
    const bool fuse_large = (fl ? atoi(fl) != 0 : true) && bs_all;
    bool fuse = conj_all && any_filter_prog && !group_by && nprog == 1 && nhll == 0 && naggs > 0 && naggs <= 4 && !want_bitmap &&
                (fe ? atoi(fe) != 0 : (!dense_small && (!big || fuse_large || (fuse_per_tile > 0 && per_tile <= fuse_per_tile))));
    bool any_value = false;
    for (int a = 0; a < naggs; a++) any_value |= dq.aggs[a].acc != ACC_COUNT;
    if (fuse && any_value) {
      fused_naggs = naggs;
      const char *sv = getenv("PHIP_STREAM_VALUES");  // measurement override: "0" never, "1" always
      const char *sp = getenv("PHIP_STREAM_PACKED");  // measurement override: "0" = stream ids + dictionary instead
      const double kStreamValueMin = 0.5;
      for (size_t i = 0; i < dsegs.size(); i++) {
        DevSeg &ds = dsegs[i];
        int32_t off = seg_off[i];
        const int32_t nstage0 = ds.num_stage;
        for (int a = 0; a < naggs; a++) {
          const DevAgg &ag = dq.aggs[a];
          if (ag.acc == ACC_COUNT) continue;
          for (int c : {ag.col_a, ag.expr != PHIP_EXPR_COLUMN ? ag.col_b : -1}) {
            if (c < 0) continue;
            DevCol &dc = ds.cols[c];
            if (dc.lds_off >= 0) continue;
            // a column read through its doc-order values (as_raw) streams its packed ids instead when the tiles are
            // dense enough: fewer bytes per tile than the values, and no per-doc load at all
            const int sidx = ds.seg_index % nseg;
            const ColumnStore &cs = segs[sidx]->cols[colidx[sidx][c]];
            const bool via_vals = !dc.has_dict && !no_dict(cs);
            if (!dc.has_dict && !via_vals) continue;
            // packed values stream as they are (vbits per doc, no dictionary gather after): fused_i64_u / fused_f64_u
            const bool via_packed = via_vals && dc.vpack != nullptr && !(sp && atoi(sp) == 0);
            const int32_t bits = via_packed ? dc.vbits : via_vals ? cs.bits : dc.bits;
            const bool dense = seg_est[i] * (1024.0 / std::max(1, bits)) >= kStreamValueMin;
            if (!(sv ? atoi(sv) != 0 : (dense && !big))) continue;
            const int32_t bytes = 256 * bits;
            // (DevSeg.stage holds kMaxStage sources; the fused kernel's cursor takes up to kMaxConj + kMaxAggStage)
            if (ds.num_stage >= std::min(kMaxStage, kMaxConj + kMaxAggStage) || off + bytes + 2 * kStagePad > kSlotBudget)
              continue;
            if (via_vals && !via_packed) {
              dc.has_dict = 1;
              dc.raw = cs.raw;
              dc.vpack = nullptr;
              dc.vbits = 0;
              ids_streamed[(size_t)sidx * ncols + c] = true;
            }
            dc.lds_off = off + kStagePad;
            ds.stage[ds.num_stage++] = {(const uint8_t *)(via_packed ? dc.vpack : dc.words), bytes, dc.lds_off};
            ds.num_dma += (int32_t)ceil_div(bytes, 1024);
            off += bytes + 2 * kStagePad;
          }
        }
        stage_stride = std::max(stage_stride, off);
        // nothing streamed with the tile: the matched docs collect across tiles (filter.hip fused_defer)
        ds.fused_defer = ds.num_stage == nstage0 ? 1 : 0;
        if (const char *fd = getenv("PHIP_FUSED_DEFER")) ds.fused_defer = ds.fused_defer && atoi(fd) != 0;  // A/B
        any_defer |= ds.fused_defer != 0;
      }
    }
  }
  // Fused group-by (filter_kernel.h fused_defer_gb): a dense key space whose table lives in HBM -- the filter kernel
  // collects its matched docs in a deferred ring (1 KiB per wave, kFusedRingGB: half the deferred aggregation's, so
  // the LDS-DMA ring keeps its resident workgroups on most queries) and runs the batched group-by walk itself, so
  // neither the tile masks (256 B per tile written and read back) nor the second launch's walk over every mask remain.
  // Its table updates are HBM atomics, which serialise on hot rows: an LDS-sized table stays with the aggregation
  // kernel's LDS tables unless few docs hit each key (<= kFuseGbMaxPerKey expected). With at least one doc per key the
  // table is kept once per XCD (GB_XCD: workgroup-scope atomics in the XCD's L2, folded by xcd_merge_kernel) when the
  // eight copies fit PHIP_FUSED_GB_XCD_MAX bytes each (default 16 MiB); sparser keys keep one table (the copies' init
  // and merge would cost more than they save). Measured on SSB SF100 unsorted, p50 (tools/gb_ab.py,
  // profiles/r05r_xcd_ab.log, two launches -> fused): Q2.3 0.449 -> 0.357 ms (XCD copies), Q3.2 0.711 -> 0.548 (XCD),
  // Q3.3 0.517 -> 0.520, Q3.4 0.536 -> 0.518, Q4.3 0.616 -> 0.585; hot tables fused measured 1.3-40x slower (C5 0.90 ->
  // 5.0 ms with XCD copies, 37 ms with one table; Q2.1 0.57 -> 1.02; profiles/r05p_fgb_ab.log). PHIP_FUSED_GB: "0" off,
  // "2" every dense table into one HBM table, "3" every dense table with XCD copies up to the cap, "4" LDS-sized
  // tables into the workgroup's LDS table (when the rings still fit beside it) (measurement overrides). The LDS table
  // beside the filter's rings leaves 1-3 workgroups (4-12 waves) per CU for a walk that is latency-bound, so it
  // measured slower than the separate aggregation kernel's LDS tables everywhere but Q4.1 (2.8 KB table): Q2.1 0.570 ->
  // 0.985 ms, Q3.1 0.955 -> 1.670, Q4.2 0.628 -> 1.323, Q4.1 0.780 -> 0.765 (profiles/r05t_lds_ab.log) -- opt-in only.
  bool fused_gb = false, gb_xcd = false, gb_lds = false;
  int64_t gb_lds_bytes = 0;  // the fused LDS table per workgroup
  if (group_by && dq.mode != GB_HASH && conj_all && any_filter_prog && nprog == 1 && !want_bitmap && nsel == 0) {
    const char *fg = getenv("PHIP_FUSED_GB");
    const int fgm = fg ? atoi(fg) : 1;
    const int64_t m = nhll ? ((int64_t)1 << log2m) : 0;
    const int64_t table_bytes = (int64_t)(1 + naggs) * dq.num_groups * 8 + (int64_t)nhll * dq.num_groups * m;
    const char *force = getenv("PHIP_GB_MODE");
    const bool lds_sized = table_bytes <= 128 * 1024 && !(force && !strcmp(force, "global"));
    double est_docs = 0.0;
    for (size_t i = 0; i < dsegs.size(); i++) est_docs += seg_est[i] * dsegs[i].num_docs;
    const double per_key = est_docs / (double)std::max<int64_t>(1, dq.num_groups);
    const double kFuseGbMaxPerKey = 40.0;
    const char *fx = getenv("PHIP_FUSED_GB_XCD_MAX");
    const int64_t xcd_max = fx ? atoll(fx) : (int64_t)16 << 20;
    // A sorted group-by column hands each XCD's contiguous doc range a few keys at a time, so the per-key estimate
    // (uniform keys) understates how hot its rows run: SSB Q2.3 over the layout sorted by date (D_YEAR a key) 0.454 ->
    // 0.499 ms fused with XCD copies, against 0.457 -> 0.354 unsorted (profiles/r05w_sorted_ab.log).
    bool sorted_key = false;
    for (int k = 0; k < q->num_group_by; k++)
      for (int s2 = 0; s2 < nseg; s2++)
        sorted_key |= !segs[s2]->cols[colidx[s2][q->group_by_columns[k]]].sorted_pairs.empty();
    fused_gb = fgm == 2 || fgm == 3 || (fgm == 1 && (!lds_sized || (per_key <= kFuseGbMaxPerKey && !sorted_key)));
    gb_xcd = fused_gb && fgm != 2 && table_bytes <= xcd_max && (fgm == 3 || per_key >= 1.0) &&
             dev->num_xcc <= kXcdCopies;  // (XCC ids distinct mod kXcdCopies: device_xcc_count)
    if (fgm == 4 && lds_sized) {
      // (u64 rows, then the HLL registers packed four u8 to a u32 word: nhll x G x m bytes)
      const int64_t lb = round_up((int64_t)(1 + naggs) * dq.num_groups * 8 + (int64_t)nhll * dq.num_groups * m, 16);
      const int64_t ss = round_up(std::max(stage_stride, 16), 16);
      if ((160 * 1024 - 256 - (int64_t)kFilterWaves * 4 * kFusedRingGB - lb) / ((int64_t)kFilterWaves * ss) >= 2) {
        fused_gb = gb_lds = true;
        gb_xcd = false;
        gb_lds_bytes = lb;
      }
    }
    if (fused_gb) {
      any_defer = true;
      for (DevSeg &ds : dsegs) ds.fused_defer = 1;
    }
  }
  stage_stride = (int32_t)round_up(std::max(stage_stride, 16), 16);
  for (const DevSeg &ds : dsegs) {
    int64_t per_tile = 0;
    std::vector<int> seen;
    for (int i = ds.node_begin; i < ds.node_end; i++) {
      const DevNode &dn = nodes[i];
      if (dn.op != DOP_LEAF) continue;
      if (dn.leaf_kind == PHIP_LEAF_DICT_RANGE || dn.leaf_kind == PHIP_LEAF_DICT_SET) {
        if (std::find(seen.begin(), seen.end(), dn.column) == seen.end()) {
          seen.push_back(dn.column);
          per_tile += 256ll * ds.cols[dn.column].bits;
        }
      } else if (dn.leaf_kind == PHIP_LEAF_INVERTED) {
        per_tile += 256;
      } else if (dn.leaf_kind == PHIP_LEAF_RAW_RANGE || dn.leaf_kind == PHIP_LEAF_RAW_SET) {
        per_tile += (int64_t)kTileDocs * type_width(ds.cols[dn.column].type);
      } else if (dn.leaf_kind == PHIP_LEAF_RAW_STRING_RANGE || dn.leaf_kind == PHIP_LEAF_RAW_STRING_SET) {
        // the doc offsets + the values' bytes (this segment's mean length)
        const int s = ds.seg_index % nseg;
        const ColumnStore &cs = segs[s]->cols[colidx[s][dn.column]];
        per_tile += (int64_t)kTileDocs * 8 + (int64_t)(kTileDocs * cs.str_total / std::max<int64_t>(segs[s]->num_docs, 1));
      }
    }
    P.filter_bytes += per_tile * ds.num_work;
  }
  for (int c = 0; c < ncols; c++) {
    if (!projected[c]) continue;
    Plan::ProjCol pc;
    pc.progs = proj_progs[c];
    for (int s = 0; s < nseg; s++) {
      const ColumnStore &cs = segs[s]->cols[colidx[s][c]];
      const bool raw = (as_raw(s, c) && !ids_streamed[(size_t)s * ncols + c]) || hll_doc_used[(size_t)s * ncols + c];
      // (packed doc-order values: vbits per doc and no dictionary)
      const bool packed = raw && !no_dict(cs) && !hll_doc_used[(size_t)s * ncols + c] && packed_vals(cs);
      pc.bits.push_back(packed ? cs.vbits : raw ? 0 : cs.bits);
      pc.card.push_back(raw ? 0 : cs.card);
      pc.width.push_back(hll_doc16_used[(size_t)s * ncols + c] ? 2 : (cs.type == PHIP_TYPE_STRING ? 4 : type_width(cs.type)));  // STRING: remap / HLL entry
    }
    P.proj.push_back(pc);
  }
  for (int s = 0; s < nseg; s++) P.seg_docs.push_back(segs[s]->num_docs);
  const bool conj_only = conj_all;
  if (fused_naggs > 0 || fused_gb) need_mask = false;  // the filter kernel aggregates its own tiles
  const bool fused_any = fused_naggs > 0 || fused_gb;
  // ring depth: prefer 4 workgroups (16 waves) per CU for the VALU/LDS work of the leaves, and give
  // each wave the deepest ring that then fits the 160 KiB LDS (bytes in flight per CU =
  // blocks x 4 waves x (nbuf-1) x slot)
  int nbuf = 0, fbpc = 0;
  const int32_t fring_bytes = fused_gb ? 4 * kFusedRingGB : (any_defer ? 4 * kFusedRingDefer : 2 * kFusedRingTile);  // per wave
  {
    const char *env = getenv("PHIP_FILTER_BPC");  // measurement override
    int want = env ? std::max(1, std::min(8, atoi(env))) : (conj_only ? 6 : 4);
    // A mid-sized scan (a few tiles per wave at the default) streams better with fewer, longer-lived waves and a
    // deeper ring: each wave's ring prologue is paid once per range. Measured on SSB SF100 sorted Q1.1 (42K
    // tiles): 6 -> 3 workgroups per CU, filter 0.074 -> 0.065 ms; the unsorted layout (293K tiles, 48 per wave)
    // and small queries (every wave one or two tiles: latency) keep the default (tools/ab_env.sh, bpc A/B).
    const int64_t kMinTilesPerWave = 12;
    const int64_t waves_at = (int64_t)dev->num_cus * want * kFilterWaves;
    // (a fused launch keeps the full width: its waves also wait on gathers -- sorted Q1.1 fused 0.201 -> 0.187 ms at
    // 6 instead of 3 workgroups per CU, profiles/r03p_fused_bpc_ab.log)
    if (!env && total_work >= 4 * waves_at && !fused_any)
      while (want > 2 && total_work < kMinTilesPerWave * (int64_t)dev->num_cus * want * kFilterWaves) want--;
    const int64_t fring = (fused_any ? (int64_t)kFilterWaves * fring_bytes : 0) + gb_lds_bytes;  // fused doc rings (+ table)
    for (int bpc = want; bpc >= 1 && nbuf < 2; bpc--) {
      // a workgroup's share of the CU's 160 KiB, less 256 B for the kernel's static LDS (block partials)
      const int64_t nb = std::min<int64_t>(kMaxRing, ((160 * 1024) / bpc - 256 - fring) / ((int64_t)kFilterWaves * stage_stride));
      if (nb >= 2) {
        nbuf = (int)nb;
        fbpc = bpc;
      }
    }
    if (nbuf < 2) return fail(PHIP_ERR_UNSUPPORTED, "filter needs %d bytes of LDS per ring slot", stage_stride);
    // A small fused query (up to 8 tiles per wave at one workgroup per CU: sorted Q1.2's ~3.8K tiles) runs one
    // workgroup per CU with the deepest ring: its waves get several tiles each with all their DMAs in flight at once,
    // instead of 5x the waves with one tile each and a 2-slot ring (Q1.2 fused 39.8 -> 33.6 us, profiles/r05d_q1_small.log;
    // PHIP_FUSED_SMALL=0 keeps the width rule)
    const char *fs = getenv("PHIP_FUSED_SMALL");
    if (!env && fused_any && !(fs && atoi(fs) == 0) &&
        total_work <= (int64_t)dev->num_cus * kFilterWaves * 8 && fbpc > 1) {
      const int64_t nb = std::min<int64_t>(kMaxRing, ((160 * 1024) - 256 - fring) / ((int64_t)kFilterWaves * stage_stride));
      if (nb >= 2) {
        nbuf = (int)nb;
        fbpc = 1;
      }
    }
  }
  const size_t filter_lds = (size_t)kFilterWaves * nbuf * stage_stride + (fused_any ? (size_t)kFilterWaves * fring_bytes : 0) +
                            (size_t)gb_lds_bytes;
  const char *walk_env = getenv("PHIP_FILTER_WALK");  // measurement override: "xcd" / "xcdc" / "contig"
  // contiguous per-wave ranges measured fastest for the plain filter; a fused aggregation's waves stay inside
  // their XCD's eighth of the work (its dictionaries then stay in that XCD's L2)
  int xcd_walk = fused_any ? 2 : 0;
  if (walk_env) xcd_walk = !strcmp(walk_env, "xcd") ? 1 : (!strcmp(walk_env, "xcdc") ? 2 : 0);
  int64_t min_tiles_per_wave = 1;
  if (const char *mt = getenv("PHIP_FILTER_MIN_TILES")) min_tiles_per_wave = std::max(1, atoi(mt));  // A/B
  int filter_blocks = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)dev->num_cus * fbpc,
                                                                  ceil_div(total_work, kFilterWaves * min_tiles_per_wave)));
  if (xcd_walk) filter_blocks = (int)round_up(std::max(filter_blocks, 8), 8);

  // ---- aggregation kernel configuration (aggregate.hip) -----------------------------------------
  dq.log2m = log2m;
  if (dq.mode != GB_HASH) dq.mode = group_by ? GB_GLOBAL : GB_NONE;
  if (group_by) dq.dense_batch = 0;  // (set below for GB_LDS: the batched group-by walk)
  const int m_regs = nhll ? (1 << log2m) : 0;
  size_t agg_lds = (size_t)kAggWaves * ring_entries(dq.mode) * 4 + (size_t)kAggWaves * dq.stage_bytes;
  int agg_bpc = 4;
  void *first_doc = nullptr;
  if (group_by && dq.mode == GB_HASH && nseg == 1 && gb_key_space >= q->num_groups_limit && q->num_groups_limit > 0) {
    int32_t rc0 = P.alloc((size_t)dq.num_groups * 4, &first_doc);
    if (rc0) return rc0;
    dq.seg_keys = 1;
    dq.seg_key_mult = 1;
    dq.first_doc = (uint32_t *)first_doc;
  }
  if (group_by && dq.mode == GB_HASH) {
    if ((int64_t)nhll * dq.num_groups * m_regs * 4 > ((int64_t)16 << 30))
      return fail(PHIP_ERR_UNSUPPORTED, "DISTINCTCOUNTHLL registers of %lld hash slots exceed the memory budget",
                  (long long)dq.num_groups);
  } else if (group_by) {
    const int64_t tbl_words = (int64_t)(1 + naggs) * dq.num_groups;
    const int64_t hll_words = (int64_t)nhll * dq.num_groups * m_regs / 4;
    const int64_t table_bytes = tbl_words * 8 + hll_words * 4;
    const char *force = getenv("PHIP_GB_MODE");  // measurement override: "lds" / "global"
    bool use_lds = table_bytes <= 128 * 1024 && (!fused_gb || gb_lds);
    if (force && !strcmp(force, "global")) use_lds = false;
    if (force && !strcmp(force, "lds") && !fused_gb && (int64_t)agg_lds + round_up(table_bytes, 16) <= 159 * 1024)
      use_lds = true;
    // The batched walk (aggregate.hip group_ring_batch: kBatch chunks per gather round trip) for LDS tables, the
    // one-chunk walk for HBM tables: measured on SSB SF100 (tools/gb_ab.py, profiles/r04b_gb_ab.log) the LDS
    // group-bys gain (Q2.1 aggregation 0.45 -> 0.34 ms, Q2.2 0.20 -> 0.19, Q4.1 0.63 -> 0.56) and the sparse HBM-table
    // ones lose (Q3.2 0.30 -> 0.36, Q4.3 0.10 -> 0.15: the larger kernel keeps fewer waves resident for their latency;
    // profiles/r04c_gb_ab.log).
    // Its larger ring must not cost a resident workgroup (C5: 3 -> 2 per CU made it 16 % slower, Q4.2 2 -> 1 6 %).
    const char *gbb = getenv("PHIP_GB_BATCH");  // measurement override: "0" / "1"
    const int64_t tb = round_up(table_bytes, 16);
    const int64_t ring_extra = (int64_t)kAggWaves * (kRingGroupBatch - kRingGroup) * 4;
    auto bpc_of = [&](int64_t lds) { return std::max<int64_t>(1, std::min<int64_t>(4, (160 * 1024 - 1024) / lds)); };
    bool batched = use_lds && bpc_of((int64_t)agg_lds + ring_extra + tb) >= bpc_of((int64_t)agg_lds + tb);
    if (gbb) batched = atoi(gbb) != 0;
    if (use_lds && (int64_t)agg_lds + ring_extra + tb > 159 * 1024) batched = false;
    dq.dense_batch = batched ? 1 : 0;
    agg_lds = (size_t)kAggWaves * ring_entries(dq.mode == GB_HASH ? GB_HASH : GB_LDS, batched) * 4 +
              (size_t)kAggWaves * dq.stage_bytes;
    if (use_lds) {
      dq.mode = GB_LDS;
      dq.tbl_words = (int32_t)tbl_words;
      dq.hll_words = (int32_t)hll_words;
      // A table that leaves one 8-wave workgroup per CU (Q2.1's 7000 groups x 16 B = 112 KB): 16-wave workgroups share
      // it, so the CU keeps 16 waves of gathers in flight instead of 8 (SQ: the 8-wave walk spent 76 % of its wave
      // cycles in s_waitcnt, profiles/r05l_sq_gb.txt). Not where 8-wave workgroups already keep 16-24 waves: C5's
      // 49 KB table (three per CU) went 0.77 -> 0.87 ms in 16-wave pairs, Q3.1 0.60 -> 0.62 (profiles/r06l_waves_ab.log).
      // PHIP_GB_WAVES=8 / 16 forces either (A/B).
      const char *gw = getenv("PHIP_GB_WAVES");
      auto walk_of = [&](bool b) {
        Plan::GbWalk w;
        w.batched = b;
        w.lds = (size_t)kAggWaves * ring_entries(GB_LDS, b) * 4 + (size_t)kAggWaves * dq.stage_bytes +
                (size_t)round_up(table_bytes, 16);
        int bpc = std::max(1, std::min(4, (int)((160 * 1024 - 1024) / w.lds)));
        w.waves = kAggWaves;
        const size_t lds16 = (size_t)16 * ring_entries(GB_LDS, b) * 4 + (size_t)16 * dq.stage_bytes +
                             (size_t)round_up(table_bytes, 16);
        const int bpc16 = lds16 <= (size_t)159 * 1024 ? std::max(1, std::min(2, (int)((160 * 1024 - 1024) / lds16))) : 0;
        const bool want16 = gw ? atoi(gw) == 16 : bpc == 1;
        if (want16 && bpc16 > 0) {
          w.waves = 16;
          w.lds = lds16;
          bpc = bpc16;
        }
        w.blocks = (int)std::min<int64_t>((int64_t)dev->num_cus * bpc, ceil_div(total_work, w.waves));
        w.blocks = (int)round_up(std::max(w.blocks, 8), 8);  // the XCD walk needs a multiple of 8 workgroups
        w.ok = w.lds <= (size_t)159 * 1024;
        return w;
      };
      P.walk[0] = walk_of(false);
      P.walk[1] = walk_of(true);
      const Plan::GbWalk &w = P.walk[batched ? 1 : 0];
      agg_lds = w.lds;
      dq.wg_waves = w.waves;
      agg_bpc = std::max(1, (int)((w.blocks + dev->num_cus - 1) / dev->num_cus));
      // Which walk runs follows the matched docs (the one-chunk walk for sparse matches, the batched one above
      // kWalkBatchDocsPerCu per CU): the plan starts with the rule above and re-chooses after every execution.
      // Measured (profiles/r06l_waves_ab.log, SSB SF100 sorted): Q3.1 21.9M docs 0.61 -> 0.47 ms batched, Q2.1 4.7M
      // 0.27 -> 0.24, Q4.2 2.3M 0.146 -> 0.131; Q2.2 0.96M 0.161 -> 0.146 one-chunk, Q2.3 0.12M 0.135 -> 0.119, Q4.3
      // 0.46M 0.065 -> 0.035. HLL tables keep the rule when they gather per column (C5 23.8M docs: batched 0.83 ms
      // vs 0.77); with group-by records the batched walk wins there too (C5 0.63 -> 0.61, profiles/r06w_rec_ab.log).
      bool any_rec = false;
      for (const DevSeg &d : dsegs) any_rec |= d.rec != nullptr;
      dq.rec_on = any_rec ? 1 : 0;  // (the agg_kernel variant that reads them)
      P.walk_adaptive = (nhll == 0 || any_rec) && !gbb && !gw && !fused_gb && P.walk[0].ok && P.walk[1].ok;
      P.walk_cur = batched ? 1 : 0;
    }
  } else if (nhll) {
    agg_lds += (size_t)nhll * m_regs * 4;
  }
  if (!group_by && dq.hist_aggs) agg_lds += (size_t)kAggWaves * dq.hist_words * 4;  // (the waves' id bins)
  if (dq.wg_waves == 0) dq.wg_waves = kAggWaves;
  if (dq.mode != GB_LDS || fused_gb) {  // only the LDS-table walks read group-by records (the segments keep theirs)
    dq.rec_on = 0;
    for (DevSeg &d : dsegs) d.rec = nullptr;
  }
  int agg_blocks = (int)std::min<int64_t>((int64_t)dev->num_cus * agg_bpc, ceil_div(total_work, dq.wg_waves));
  agg_blocks = (int)round_up(std::max(agg_blocks, 8), 8);  // the XCD walk needs a multiple of 8 workgroups
  if (P.walk_cur >= 0) agg_blocks = P.walk[P.walk_cur].blocks;

  const size_t nodes_off = blob.reserve(std::max<size_t>(nodes.size(), 1) * sizeof(DevNode));
  kinds[naggs] = ACC_COUNT;
  kinds[naggs + 1] = ACC_COUNT;
  const size_t kinds_off = blob.add(kinds.data(), kinds.size() * 4);
  const size_t dq_off = blob.reserve(sizeof(DevAggQuery));  // written once every pointer is known
  const size_t sq_off = nsel > 0 ? blob.reserve(sizeof(DevSelQuery)) : 0;

  void *dblob;
  int32_t rc = P.alloc(blob.data.size() + 64, &dblob);
  if (rc) return rc;
  uint8_t *base = (uint8_t *)dblob;
  for (auto &f : aux_fix) nodes[f.node].aux = base + f.off;
  if (!nodes.empty()) memcpy(blob.data.data() + nodes_off, nodes.data(), nodes.size() * sizeof(DevNode));
  if (!dsegs.empty()) memcpy(blob.data.data() + segs_off, dsegs.data(), sizeof(DevSeg) * dsegs.size());
  const DevSeg *dev_segs = (const DevSeg *)(base + segs_off);

  DevFilter fq;
  memset(&fq, 0, sizeof(fq));
  fq.segs = dev_segs;
  fq.nodes = (const DevNode *)(base + nodes_off);
  fq.num_segs = (int32_t)dsegs.size();
  fq.total_work = (int32_t)total_work;
  fq.stage_stride = stage_stride;
  fq.nbuf = nbuf;
  fq.fring_bytes = fring_bytes;
  fq.xcd_walk = xcd_walk;
  {
    const char *pe = getenv("PHIP_FILTER_PROBE");
    fq.probe = pe ? atoi(pe) : 0;
    // range scans of the contiguous evaluator inline: the call's register save / restore through scratch cost
    // 4-9 % of C4's filter kernel (tools/c4_ab.py, profiles/r02f_c4_inline_ab.log); "0" = the call (A/B)
    const char *ie = getenv("PHIP_CONTIG_INLINE");
    fq.contig_inline = ie ? atoi(ie) : 1;
  }
  fq.stats_programs = q->stats_programs ? (uint32_t)q->stats_programs : 0xffffffffu;
  {
    const char *mn = getenv("PHIP_MASK_NT");  // measurement switch: non-temporal tile-mask stores
    fq.mask_nt = mn ? atoi(mn) : 0;
  }
  fq.min_dma = 0;
  for (size_t i = 0; i < dsegs.size(); i++)
    fq.min_dma = i == 0 ? dsegs[i].num_dma : std::min(fq.min_dma, dsegs[i].num_dma);
  dq.segs = dev_segs;

  void *fpart, *finals, *seg_matched, *apart = nullptr, *masks = nullptr;
  rc = P.alloc((size_t)filter_blocks * 2 * 8, &fpart);
  if (rc) return rc;
  // finals[64] | seg_matched[nmatch] | hll registers: the same layout as the pinned landing area, so one
  // D2H copy brings every per-execution result back
  const int nmatch = nprog * nseg;
  rc = P.alloc((64 + (size_t)nmatch) * 8 + (size_t)std::max(nhll, 1) * (1 << 12) * 4, &finals);
  if (rc) return rc;
  seg_matched = (uint64_t *)finals + 64;
  fq.partials = (uint64_t *)fpart;
  fq.seg_matched = (uint64_t *)seg_matched;
  // finals: [0, naggs) aggregation slots, [32, 34) matched docs + entries scanned in filter
  dq.hll_regs = (uint32_t *)((uint64_t *)finals + 64 + nmatch);
  if (need_mask) {
    rc = P.alloc((size_t)std::max<int64_t>(total_work, 1) * 64 * 4, &masks);
    if (rc) return rc;
    fq.mask_out = (uint32_t *)masks;
    dq.mask = (const uint32_t *)masks;
  }
  if (need_agg && !group_by) {
    const int pblocks = fused_naggs > 0 ? filter_blocks : agg_blocks;
    rc = P.alloc((size_t)pblocks * std::max(naggs, 1) * 8, &apart);
    if (rc) return rc;
    dq.partials = (uint64_t *)apart;
    if (fused_naggs > 0) {
      fq.agg_partials = (uint64_t *)apart;
      fq.agg = (const DevAggQuery *)(base + dq_off);
    }
  }
  if (fused_gb) fq.agg = (const DevAggQuery *)(base + dq_off);
  void *gtab = nullptr, *ghll = nullptr, *slab = nullptr, *hslab = nullptr;
  if (group_by) {
    const size_t copies = gb_xcd ? kXcdCopies : 1;
    rc = P.alloc(copies * (1 + naggs) * dq.num_groups * 8, &gtab);
    if (rc) return rc;
    if (nhll) {
      rc = P.alloc(copies * nhll * dq.num_groups * m_regs * 4, &ghll);
      if (rc) return rc;
    }
    if (gb_xcd) {
      dq.xcd_words = (int64_t)(1 + naggs) * dq.num_groups;
      dq.xcd_hll_words = (int64_t)nhll * dq.num_groups * m_regs;
    }
    if (dq.mode == GB_HASH) {
      void *hk = nullptr, *ho = nullptr;
      rc = P.alloc((size_t)dq.num_groups * 8, &hk);
      if (rc) return rc;
      rc = P.alloc(16, &ho);
      if (rc) return rc;
      dq.gb_keys = (uint64_t *)hk;
      dq.hash_overflow = (uint32_t *)ho;
    }
    if (dq.mode == GB_LDS) {
      // (the fused LDS table: one slab per filter workgroup; an adaptive walk: the larger grid of the two)
      const size_t nslabs = gb_lds ? filter_blocks
                                   : std::max<int>(agg_blocks, P.walk_adaptive ? std::max(P.walk[0].blocks, P.walk[1].blocks) : 0);
      rc = P.alloc(nslabs * dq.tbl_words * 8 + 16, &slab);
      if (rc) return rc;
      if (nhll) {
        rc = P.alloc(nslabs * dq.hll_words * 4 + 16, &hslab);
        if (rc) return rc;
      }
      dq.gb_table = (uint64_t *)slab;
      dq.gb_hll = (uint32_t *)hslab;
    } else {
      dq.gb_table = (uint64_t *)gtab;
      dq.gb_hll = (uint32_t *)ghll;
    }
  }
  void *fo = nullptr;
  if (want_bitmap) {
    rc = P.alloc((size_t)filter_nwords * 8 + 4096 * 8, &fo);
    if (rc) return rc;
  }

  memcpy(blob.data.data() + dq_off, &dq, sizeof(dq));
  if (nsel > 0) {
    void *sb;
    const size_t nent = dsegs.size();
    rc = P.alloc(((size_t)total_work + 1) * 16 + (2 * nent + 1) * 8 + 16, &sb);
    if (rc) return rc;
    P.sel_tile_cnt = (int64_t *)sb;
    P.sel_tile_off = P.sel_tile_cnt + total_work + 1;
    P.sel_base = P.sel_tile_off + total_work + 1;
    P.sel_kept = P.sel_base + nent + 1;
    P.sel_total = P.sel_kept + nent;
    sq.segs = dev_segs;
    sq.num_segs = (int32_t)nent;
    sq.total_work = (int32_t)total_work;
    sq.mask = has_filter ? (const uint32_t *)masks : nullptr;
    sq.tile_off = P.sel_tile_off;
    sq.seg_base = P.sel_base;
    memcpy(blob.data.data() + sq_off, &sq, sizeof(sq));
    P.select = true;
    P.nsel = nsel;
    P.sq_off = sq_off;
    P.sel_types = sel_types;
    P.sel_dicts = sel_dicts;
    P.sel_str_ptrs.assign(nsel, {});
    for (int k = 0; k < nsel; k++) {
      if (sq.sel[k].kind != SEL_STR) continue;
      std::vector<const void *> &v = P.sel_str_ptrs[k];
      v.resize(2 * (size_t)nseg);
      for (int s = 0; s < nseg; s++) {
        const ColumnStore &cs = segs[s]->cols[colidx[s][sq.sel[k].col_a]];
        v[s] = cs.raw;
        v[nseg + s] = cs.str_off;
      }
    }
    for (int k = 0; k < nsel; k++) {  // bytes one row reads per expression (first segment's widths)
      for (int c : {sq.sel[k].col_a, sq.sel[k].expr != PHIP_EXPR_COLUMN ? sq.sel[k].col_b : -1}) {
        if (c < 0) continue;
        const ColumnStore &cs = segs[0]->cols[colidx[0][c]];
        P.sel_bits.push_back(no_dict(cs) ? 0 : cs.bits);
        P.sel_width.push_back(cs.type == PHIP_TYPE_STRING ? 4 : type_width(cs.type));
      }
    }
  }
  // the descriptor blob goes up once, synchronously (its host copy dies with this function)
  HIP_TRY(hipMemcpyAsync(dblob, blob.data.data(), blob.data.size(), hipMemcpyHostToDevice, st));
  HIP_TRY(hipStreamSynchronize(st));

  P.dq = dq;
  P.fq = fq;
  P.dsegs = dsegs;
  P.tasks = tasks;
  P.gb_dicts = gb_dicts;
  P.nseg = nseg;
  P.nprog = nprog;
  P.nmatch = nmatch;
  P.naggs = naggs;
  P.nhll = nhll;
  P.log2m = log2m;
  P.m_regs = m_regs;
  P.num_group_by = q->num_group_by;
  P.num_projected = num_projected;
  P.num_groups_limit = q->num_groups_limit;
  if (q->trim_size > 0 && q->num_order_terms > 0) {
    if (q->num_order_terms > kMaxOrderKeys || q->num_group_by > kMaxOrderKeys || !q->order_terms)
      return fail(PHIP_ERR_UNSUPPORTED, "device trim: at most %d ORDER BY terms / group-by columns", kMaxOrderKeys);
    OrderTerms &ot = P.order_terms;
    ot.num_group_by = q->num_group_by;
    ot.num_terms = q->num_order_terms;
    for (int j = 0; j < q->num_order_terms; j++) {
      const phip_order_term &t = q->order_terms[j];
      auto agg_ok = [&](int32_t i, bool count) {
        if (i < 0 || i >= q->num_aggregations) return false;
        const int32_t f = q->aggregations[i].function;
        return count ? f == PHIP_AGG_COUNT : f != PHIP_AGG_HLL;
      };
      bool ok;
      switch (t.kind) {
        case PHIP_ORDER_GROUP_KEY: ok = t.a >= 0 && t.a < q->num_group_by; break;
        case PHIP_ORDER_VALUE: ok = agg_ok(t.a, false); break;
        case PHIP_ORDER_AVG: ok = agg_ok(t.a, false) && q->aggregations[t.a].function == PHIP_AGG_SUM && agg_ok(t.b, true); break;
        case PHIP_ORDER_RANGE:
          ok = agg_ok(t.a, false) && agg_ok(t.b, false) && q->aggregations[t.a].function == PHIP_AGG_MIN &&
               q->aggregations[t.b].function == PHIP_AGG_MAX;
          break;
        case PHIP_ORDER_HLL: ok = t.a >= 0 && t.a < q->num_aggregations && q->aggregations[t.a].function == PHIP_AGG_HLL; break;
        default: ok = false;
      }
      if (!ok) return fail(PHIP_ERR_INVALID, "order_terms[%d] (kind %d, a %d, b %d) invalid", j, t.kind, t.a, t.b);
      ot.kind[j] = t.kind;
      ot.a[j] = t.a;
      ot.b[j] = t.b;
      if (t.kind == PHIP_ORDER_HLL) {  // (the function's register block and its own log2m)
        ot.a[j] = dq.aggs[t.a].hll_slot;
        ot.b[j] = dq.aggs[t.a].log2m;
      }
      ot.desc[j] = t.desc ? 1 : 0;
    }
    P.trim_size = q->trim_size;
  } else if (q->trim_size > 0 && q->num_order_by_keys > 0) {
    if (q->num_order_by_keys > kMaxOrderKeys || q->num_group_by > kMaxOrderKeys || !q->order_by_keys)
      return fail(PHIP_ERR_UNSUPPORTED, "device trim: at most %d ORDER BY / group-by columns", kMaxOrderKeys);
    for (int j = 0; j < q->num_order_by_keys; j++) {
      const int32_t e = q->order_by_keys[j], k = (e > 0 ? e : -e) - 1;
      if (e == 0 || k >= q->num_group_by) return fail(PHIP_ERR_INVALID, "order_by_keys[%d] = %d out of range", j, e);
      P.order_keys[j] = e;
    }
    P.order_nkeys = q->num_order_by_keys;
    P.trim_size = q->trim_size;
  } else if (q->trim_size > 0 && q->order_by_aggregation >= 0) {
    if (q->order_by_aggregation >= q->num_aggregations)
      return fail(PHIP_ERR_INVALID, "order_by_aggregation %d out of range", q->order_by_aggregation);
    const int32_t f = q->aggregations[q->order_by_aggregation].function;
    if (f == PHIP_AGG_HLL) return fail(PHIP_ERR_UNSUPPORTED, "device trim by a DISTINCTCOUNTHLL intermediate");
    P.order_agg = q->order_by_aggregation;
    P.order_desc = q->order_by_desc ? 1 : 0;
    P.trim_size = q->trim_size;
  }
  P.total_work = total_work;
  P.total_docs = total_docs;
  P.docs_in_work = 0;
  for (const DevSeg &ds : dsegs) P.docs_in_work += ds.num_docs;
  P.slot_docs.assign(nmatch, 0);
  for (const DevSeg &ds : dsegs) P.slot_docs[ds.seg_index] = ds.num_docs;
  P.has_filter = has_filter;
  P.need_agg = need_agg;
  P.need_mask = need_mask;
  P.group_by = group_by;
  P.node_part = tl_node_docs > 0;
  P.conj_only = conj_only;
  P.fused_naggs = fused_naggs;
  P.fused_gb = fused_gb;
  P.gb_xcd = gb_xcd;
  P.gb_lds = gb_lds;
  P.want_bitmap = want_bitmap;
  P.filter_nwords = filter_nwords;
  P.filter_blocks = filter_blocks;
  P.agg_blocks = agg_blocks;
  P.filter_lds = filter_lds;
  P.agg_lds = agg_lds;
  if (P.dq.hist_aggs) {
    // The id histogram pays for its per-segment flush and LDS only when most docs match (C4 SUM(M): 50 % 1.33 ->
    // 1.09 ms; 0.01-10 % slower, profiles/r06zt_hist_ab.log): the plan starts with the value gathers and takes the
    // histogram from the execution after one whose matched docs reached kHistMinMatch of its docs. The device
    // descriptor keeps hist_aggs; the host copy's decides which variant launches.
    P.hist_mask = P.dq.hist_aggs;
    P.agg_lds_hist = agg_lds;
    P.agg_lds_plain = agg_lds - (size_t)kAggWaves * P.dq.hist_words * 4;
    P.dq.hist_aggs = 0;
    P.agg_lds = P.agg_lds_plain;
  }
  P.base = base;
  P.tasks_off = tasks_off;
  P.rgroups_off = rgroups_off;
  P.num_rgroups = rgroups.size();
  P.dq_off = dq_off;
  P.kinds_off = kinds_off;
  P.inv_words = inv_words;
  P.inv_words_total = inv_words_total;
  P.fpart = fpart;
  P.finals = finals;
  P.seg_matched = seg_matched;
  P.apart = apart;
  P.masks = masks;
  P.gtab = gtab;
  P.ghll = ghll;
  P.slab = slab;
  P.hslab = hslab;
  P.fo = fo;
  P.first_doc = (uint32_t *)first_doc;
  if (const char *te = getenv("PHIP_TOTAL_EVENTS")) P.total_events = atoi(te) != 0;
  // ev[4] only between two launches (selection plans time their gather with it, execute_select)
  P.split_event = P.select || (P.has_filter && P.need_agg && P.fused_naggs == 0 && !P.fused_gb);
  if (const char *se = getenv("PHIP_SPLIT_EVENT")) P.split_event = P.split_event || atoi(se) != 0;  // A/B
  for (auto &e : P.ev) HIP_TRY(hipEventCreate(&e));
  {
    void *h = nullptr;
    const size_t pbytes = (64 + (size_t)nmatch) * 8 + (size_t)std::max(nhll, 1) * (1 << 12) * 4;
    // device-visible (mapped) pinned memory: finalize_all_kernel writes the results straight into it
    HIP_TRY(hipHostMalloc(&h, pbytes, hipHostMallocMapped));
    memset(h, 0, pbytes);
    P.pinned = (uint64_t *)h;
    void *dp = nullptr;
    HIP_TRY(hipHostGetDevicePointer(&dp, h, 0));
    P.pinned_dev = (uint64_t *)dp;
  }
  if (!group_by && !P.select && !want_bitmap) {
    void *tk = nullptr;
    const int32_t trc = P.alloc(64, &tk);
    if (trc) return trc;
    HIP_TRY(hipMemsetAsync(tk, 0, 64, st));
    P.done_ticket = (uint32_t *)tk;
  }
  // Finalize in the last workgroup of the plan's last kernel (agg_common.h finalize_tail) for aggregation-only plans:
  // the finalize_all launch and its dispatch gap go. With one device-scope ticket counter the workgroups' atomics
  // serialised at the memory side (the fused kernel grew 13-50 us, step 0.346 -> 0.421 ms, profiles/r04f_host_ab.log);
  // with the two-level sharded ticket the step gains 2-3 % (host probe 0.280 / 0.286 -> 0.272 / 0.278 ms,
  // profiles/r04w_host_ab.log; bench 0.284 -> 0.278 ms, profiles/r04x_bench.log), but every workgroup now waits for
  // its partials' acknowledgement and a ticket before it retires, and the fused kernel itself grows 11 % (sorted Q1.1
  // 0.135 -> 0.150 ms): its own roofline fraction drops more than the step gains. Opt-in (PHIP_FOLD_FINAL=1).
  const char *ff = getenv("PHIP_FOLD_FINAL");
  if (!group_by && !P.select && !want_bitmap && total_work > 0 && (has_filter || need_agg) && ff && atoi(ff) != 0) {
    const bool fused = fused_naggs > 0;
    const bool agg_last = need_agg && !fused;
    const bool aggs_here = need_agg && naggs > 0;
    DevFinal f;
    memset(&f, 0, sizeof(f));
    f.pa = aggs_here ? (const uint64_t *)apart : nullptr;
    f.ka = (const int32_t *)(base + kinds_off);
    f.nba = fused ? filter_blocks : agg_blocks;
    f.na = aggs_here ? naggs : 0;
    f.pf = has_filter ? (const uint64_t *)fpart : nullptr;
    f.kf = (const int32_t *)(base + kinds_off) + naggs;
    f.nbf = filter_blocks;
    f.segm = (uint64_t *)seg_matched;
    f.nseg = nmatch;
    f.hll = dq.hll_regs;
    f.hll_words = nhll ? (int32_t)((size_t)nhll << log2m) : 0;
    f.out = P.pinned_dev;
    void *fb;
    rc = P.alloc(round_up(sizeof(DevFinal), 64) + kFinCounterBytes, &fb);
    if (rc) return rc;
    f.counter = (uint32_t *)((uint8_t *)fb + round_up(sizeof(DevFinal), 64));
    HIP_TRY(hipMemsetAsync(f.counter, 0, kFinCounterBytes, st));
    HIP_TRY(hipMemcpyAsync(fb, &f, sizeof(f), hipMemcpyHostToDevice, st));
    P.fin_counter = f.counter;
    if (agg_last) {
      P.dq.fin = (const DevFinal *)fb;
      HIP_TRY(hipMemcpyAsync(base + dq_off, &P.dq, sizeof(DevAggQuery), hipMemcpyHostToDevice, st));
    } else {
      P.fq.fin = (const DevFinal *)fb;
    }
    HIP_TRY(hipStreamSynchronize(st));
    P.fold_final = true;
  }
  return PHIP_OK;
}

// Deadline / cancel checkpoint between an execution's launch phases (include/pinot_hip.h phip_plan_set_deadline).
static int32_t check_deadline(const Plan &P, const char *where) {
  if (P.cancelled.load(std::memory_order_relaxed))
    return fail(PHIP_ERR_CANCELLED, "query cancelled (%s)", where);
  const int64_t d = P.deadline_ms.load(std::memory_order_relaxed);
  if (d > 0) {
    const int64_t now = std::chrono::duration_cast<std::chrono::milliseconds>(
                            std::chrono::system_clock::now().time_since_epoch()).count();
    if (now > d) return fail(PHIP_ERR_TIMEOUT, "query timed out %lld ms past its deadline (%s)", (long long)(now - d),
                             where);
  }
  return PHIP_OK;
}

// The device work of one execution, on `st` (eager, or recorded into a graph by stream capture).
static int32_t enqueue_plan(Plan &P, hipStream_t st) {
  DevAggQuery &dq = P.dq;
  DevFilter &fq = P.fq;
  const int naggs = P.naggs, nhll = P.nhll, m_regs = P.m_regs;
  const bool group_by = P.group_by, has_filter = P.has_filter, need_agg = P.need_agg, need_mask = P.need_mask;
  const bool conj_only = P.conj_only;
  const int64_t total_work = P.total_work;
  uint8_t *base = P.base;
  const int32_t *dev_kinds = (const int32_t *)(base + P.kinds_off);
  uint64_t *fin_agg = (uint64_t *)P.finals;
  uint64_t *fin_filter = (uint64_t *)P.finals + 32;
  void *seg_matched = P.seg_matched, *gtab = P.gtab, *ghll = P.ghll;
  void *fpart = P.fpart, *apart = P.apart, *slab = P.slab, *hslab = P.hslab, *masks = P.masks, *fo = P.fo;
  const size_t inv_words_total = P.inv_words_total, tasks_off = P.tasks_off, dq_off = P.dq_off;
  const std::vector<DevSeg> &dsegs = P.dsegs;
  const int filter_blocks = P.filter_blocks, agg_blocks = P.agg_blocks;
  const size_t filter_lds = P.filter_lds, agg_lds = P.agg_lds;
  const int64_t filter_nwords = P.filter_nwords;
  const bool filter_words = P.want_bitmap;
  if (P.total_events) HIP_TRY(hipEventRecord(P.ev[0], st));
  // seg_matched and the HLL registers are zero between executions (finalize_all resets them); after a
  // failed execution they are cleared here
  const size_t hll_words = nhll && !group_by ? ((size_t)nhll << P.log2m) : 0;
  if (!P.clean) {
    HIP_TRY(hipMemsetAsync(seg_matched, 0, (size_t)P.nmatch * 8, st));
    if (hll_words) HIP_TRY(hipMemsetAsync(dq.hll_regs, 0, hll_words * 4, st));
    if (P.fin_counter) HIP_TRY(hipMemsetAsync(P.fin_counter, 0, kFinCounterBytes, st));
  }
  P.clean = false;
  if (filter_words) HIP_TRY(hipMemsetAsync(fo, 0, (size_t)filter_nwords * 8, st));
  if (inv_words_total) {  // (every key of every leaf is written: no clearing pass)
    HIP_TRY(launch_roaring_or((const RoaringTask *)(base + tasks_off), (const RoaringGroup *)(base + P.rgroups_off),
                              (int32_t)P.num_rgroups, st));
  }
  if (group_by && dq.mode == GB_HASH) {
    HIP_TRY(hipMemsetAsync(dq.gb_keys, 0xff, (size_t)dq.num_groups * 8, st));  // kHashEmpty
    HIP_TRY(hipMemsetAsync(dq.hash_overflow, 0, 4, st));
    if (P.first_doc) HIP_TRY(hipMemsetAsync(P.first_doc, 0xff, (size_t)dq.num_groups * 4, st));
  }
  if (group_by && P.gb_xcd) {  // every XCD-private copy at its identity
    HIP_TRY(launch_xcd_init((uint64_t *)gtab, dq.xcd_words, dq.num_groups, dev_kinds, st));
    if (nhll) HIP_TRY(hipMemsetAsync(ghll, 0, (size_t)kXcdCopies * dq.xcd_hll_words * 4, st));
  } else if (group_by && (dq.mode == GB_GLOBAL || dq.mode == GB_HASH)) {
    HIP_TRY(hipMemsetAsync(gtab, 0, (size_t)dq.num_groups * 8, st));  // counts
    for (int a = 0; a < naggs; a++) {
      uint64_t init = 0;
      if (dq.aggs[a].acc == ACC_MIN_F64) init = ~0ull;  // ordered(+inf) < ~0: atomicMin from the top
      HIP_TRY(launch_fill_u64((uint64_t *)gtab + (int64_t)(1 + a) * dq.num_groups, dq.num_groups, init, st));
    }
    if (nhll) HIP_TRY(hipMemsetAsync(ghll, 0, (size_t)nhll * dq.num_groups * m_regs * 4, st));
  }
  const bool fused = P.fused_naggs > 0 || P.fused_gb;
  // Opt-in (PHIP_EXT_EVENTS=1): a one-kernel plan's timing events recorded by the kernel's own dispatch packet
  // (hipExtLaunchKernel) instead of two barrier-packet markers. Measured on the sorted headline it costs more than it
  // saves: enqueue 7.0 -> 9.8 us per query, step 0.286 -> 0.304 ms (profiles/r04p_host_ab.log).
  const int nkern = (has_filter ? 1 : 0) + (need_agg && !fused ? 1 : 0);
  const char *xe = getenv("PHIP_EXT_EVENTS");
  const char *kt = getenv("PHIP_KERNEL_TIMING");  // "0": no timing markers (aggregation-only plans; times read 0)
  P.timed = group_by || P.select || !(kt && atoi(kt) == 0);
  const bool ext_events = P.timed && total_work > 0 && nkern == 1 && !P.split_event && xe && atoi(xe) != 0;
  hipEvent_t e0 = ext_events ? P.ev[1] : nullptr, e1 = ext_events ? P.ev[2] : nullptr;
  if (!ext_events && P.timed) HIP_TRY(hipEventRecord(P.ev[1], st));
  if (has_filter && total_work > 0)
    HIP_TRY(launch_filter(fq, conj_only, P.fused_gb ? (P.gb_lds ? -3 : (P.gb_xcd ? -2 : -1)) : P.fused_naggs, filter_blocks,
                          filter_lds, st, e0, e1));
  // (a plan of one kernel -- fused, or a filter or aggregation alone -- needs no split event)
  if (P.split_event && P.timed) HIP_TRY(hipEventRecord(P.ev[4], st));
  if (need_agg && total_work > 0 && !fused)
    HIP_TRY(launch_agg(dq, (const DevAggQuery *)(base + dq_off), agg_blocks, agg_lds, st, e0, e1));
  if (!ext_events && P.timed) HIP_TRY(hipEventRecord(P.ev[2], st));
  if (group_by && P.gb_xcd && total_work > 0)  // the XCD-private copies folded into copy 0 (the plan's table)
    HIP_TRY(launch_xcd_merge((uint64_t *)gtab, dq.xcd_words, dq.num_groups, dev_kinds, (uint32_t *)ghll,
                             dq.xcd_hll_words, st));
  if (group_by && dq.mode == GB_LDS && total_work > 0)
    HIP_TRY(launch_slab_reduce((const uint64_t *)slab, P.gb_lds ? filter_blocks : agg_blocks, dq.tbl_words, dq.num_groups,
                               dev_kinds,
                               (uint64_t *)gtab, (const uint32_t *)hslab, nhll ? dq.hll_words : 0, (uint32_t *)ghll, st));
  if (group_by && dq.mode == GB_LDS && total_work == 0) {
    // nothing to reduce: the table holds every row's identity (a partial table is merged row by row)
    HIP_TRY(hipMemsetAsync(gtab, 0, (size_t)dq.num_groups * 8, st));
    for (int a = 0; a < naggs; a++)
      HIP_TRY(launch_fill_u64((uint64_t *)gtab + (int64_t)(1 + a) * dq.num_groups, dq.num_groups,
                              dq.aggs[a].acc == ACC_MIN_F64 ? ~0ull : 0ull, st));
    if (nhll) HIP_TRY(hipMemsetAsync(ghll, 0, (size_t)nhll * dq.num_groups * m_regs * 4, st));
  }
  if (filter_words && need_mask && !dsegs.empty())
    HIP_TRY(launch_masks_to_words((const uint32_t *)masks, dsegs[0].tile0, dsegs[0].num_work, (uint64_t *)fo,
                                  filter_nwords, st));
  // every result lands in the plan's pinned buffer, written by the device: finals[64] | seg_matched[nmatch] | HLL
  P.done_seq = 0;
  if (total_work > 0 && !P.fold_final) {
    const bool aggs_here = need_agg && !group_by && naggs > 0;
    const char *pd = getenv("PHIP_POLL_DONE");  // measurement override: "0" waits for the stream
    // (only without timing markers: an event's elapsed time is readable once the runtime has seen its command
    // complete, which a poll that returns early does not wait for -- "device not ready" under concurrent lanes)
    const bool poll = P.done_ticket != nullptr && !(pd && atoi(pd) == 0) && !P.total_events && !P.timed;
    if (poll) P.done_seq = ++P.done_counter;
    HIP_TRY(launch_finalize_all(aggs_here ? (const uint64_t *)apart : nullptr, fused ? filter_blocks : agg_blocks,
                                aggs_here ? naggs : 0, dev_kinds, has_filter ? (const uint64_t *)fpart : nullptr,
                                filter_blocks, dev_kinds + naggs, (uint64_t *)seg_matched, P.nmatch, dq.hll_regs,
                                (int)hll_words, P.pinned_dev, st, poll ? P.done_ticket : nullptr, P.done_seq));
  }
  if (!group_by && P.total_events) HIP_TRY(hipEventRecord(P.ev[3], st));
  (void)fin_agg;
  (void)fin_filter;
  (void)fo;
  return PHIP_OK;
}

// numGroupsLimit (limit.hip header): the normal pass found ngroups >= limit query-wide, so some segment may
// have dropped keys. Re-aggregate per (segment, key) with first-seen docs, keep each segment's first `limit`
// keys and merge them by key. On return keys / vals / longs / hll and *ngroups describe the kept groups.
static int32_t group_limit(Plan &P, Workspace &ws, hipStream_t st, int64_t matched, void **keys, void **ov, void **ol,
                           void **oh, int64_t *ngroups, int32_t *limit_reached, const int64_t *normal_offs) {
  const int32_t S = P.nseg, naggs = P.naggs, nhll = P.nhll, m_regs = P.m_regs;
  const int64_t limit = P.num_groups_limit;
  {
    int32_t drc = check_deadline(P, "before the numGroupsLimit pass");
    if (drc) return drc;
  }
  int64_t space = 1;
  for (int64_t r : P.gb_radix) space *= r;
  if ((double)space * (double)S >= (double)((int64_t)1 << 62))
    return fail(PHIP_ERR_UNSUPPORTED, "numGroupsLimit pass: key space x %d segments exceeds 2^62", S);
  {  // first-seen positions are program * num_docs + doc in 32 bits (aggregate.hip group_chunk_hash)
    int64_t max_docs = 0;
    for (int64_t d : P.seg_docs) max_docs = std::max(max_docs, d);
    if ((int64_t)P.nprog * max_docs > (int64_t)UINT32_MAX)
      return fail(PHIP_ERR_UNSUPPORTED, "numGroupsLimit pass: %d filter programs x %lld docs exceed 32-bit positions",
                  P.nprog, (long long)max_docs);
  }
  const int64_t bound = std::max<int64_t>(1, std::min<int64_t>(matched, (int64_t)std::min<double>(
                                                                           (double)*ngroups * S, 9e18)));
  int64_t cap = 1024;
  while (cap < 2 * bound) cap <<= 1;
  if (cap * (8 + 4 + 8 * (1 + (int64_t)naggs)) > ((int64_t)24 << 30) ||
      (int64_t)nhll * cap * m_regs * 4 > ((int64_t)16 << 30) || cap > INT32_MAX)
    return fail(PHIP_ERR_UNSUPPORTED, "numGroupsLimit pass: %lld (segment, key) slots exceed the memory budget",
                (long long)cap);
  int32_t rc;
  void *hk, *tab, *fd, *hll = nullptr, *ovf, *ddq;
  const bool reuse = P.first_doc && P.dq.mode == GB_HASH && S == 1;
  if (reuse) {
    // the normal pass already holds every (key, first doc) of the one segment: no second aggregation
    cap = P.dq.num_groups;
    hk = P.dq.gb_keys;
    tab = P.gtab;
    fd = P.first_doc;
    hll = P.ghll;
    ovf = P.dq.hash_overflow;
  } else {
  if ((rc = ws.get("lim_hkeys", (size_t)cap * 8, &hk))) return rc;
  if ((rc = ws.get("lim_table", (size_t)cap * 8 * (1 + naggs), &tab))) return rc;
  if ((rc = ws.get("lim_first", (size_t)cap * 4, &fd))) return rc;
  if (nhll && (rc = ws.get("lim_hll", (size_t)nhll * cap * m_regs * 4, &hll))) return rc;
  if ((rc = ws.get("lim_ovf", 16, &ovf))) return rc;
  if ((rc = ws.get("lim_dq", sizeof(DevAggQuery), &ddq))) return rc;
  DevAggQuery dq = P.dq;
  dq.mode = GB_HASH;
  dq.num_groups = cap;
  dq.seg_keys = 1;
  dq.seg_key_mult = S;
  dq.gb_keys = (uint64_t *)hk;
  dq.gb_table = (uint64_t *)tab;
  dq.gb_hll = (uint32_t *)hll;
  dq.hash_overflow = (uint32_t *)ovf;
  dq.first_doc = (uint32_t *)fd;
  dq.tbl_words = 0;
  dq.hll_words = 0;
  HIP_TRY(hipMemsetAsync(hk, 0xff, (size_t)cap * 8, st));
  HIP_TRY(hipMemsetAsync(fd, 0xff, (size_t)cap * 4, st));
  HIP_TRY(hipMemsetAsync(ovf, 0, 4, st));
  HIP_TRY(hipMemsetAsync(tab, 0, (size_t)cap * 8, st));
  for (int a = 0; a < naggs; a++)
    HIP_TRY(launch_fill_u64((uint64_t *)tab + (int64_t)(1 + a) * cap, cap, dq.aggs[a].acc == ACC_MIN_F64 ? ~0ull : 0ull, st));
  if (nhll) HIP_TRY(hipMemsetAsync(hll, 0, (size_t)nhll * cap * m_regs * 4, st));
  if (P.fused_gb && P.total_work > 0) {
    // the fused group-by left no tile masks: the plain conjunctive filter writes them into scratch (its matched-doc
    // counts and partials into scratch too: the statistics were read after the normal pass)
    void *lm, *lp, *ls;
    if ((rc = ws.get("lim_masks", (size_t)P.total_work * 64 * 4, &lm))) return rc;
    if ((rc = ws.get("lim_fpart", (size_t)P.filter_blocks * 2 * 8, &lp))) return rc;
    if ((rc = ws.get("lim_segm", (size_t)std::max(P.nmatch, 1) * 8, &ls))) return rc;
    HIP_TRY(hipMemsetAsync(ls, 0, (size_t)std::max(P.nmatch, 1) * 8, st));
    DevFilter fq = P.fq;
    fq.agg = nullptr;
    fq.fin = nullptr;
    fq.mask_out = (uint32_t *)lm;
    fq.partials = (uint64_t *)lp;
    fq.seg_matched = (uint64_t *)ls;
    HIP_TRY(launch_filter(fq, true, 0, P.filter_blocks, P.filter_lds, st, nullptr, nullptr));
    dq.mask = (const uint32_t *)lm;
  }
  HIP_TRY(hipMemcpyAsync(ddq, &dq, sizeof(dq), hipMemcpyHostToDevice, st));
  if (P.total_work > 0)
    HIP_TRY(launch_agg(dq, (const DevAggQuery *)ddq, P.agg_blocks, (size_t)kAggWaves * kRingGroup * 4, st));
  }
  // compact the occupied slots (reusing the normal pass's table: its counts are already known)
  const int64_t nchunks = ceil_div(cap, 1024);
  void *cc, *offs, *slots;
  int64_t n = 0;
  uint32_t overflow = 0;
  if (reuse && normal_offs) {
    offs = (void *)normal_offs;
    n = *ngroups;
  } else {
    if ((rc = ws.get("lim_cc", (size_t)nchunks * 4, &cc))) return rc;
    if ((rc = ws.get("lim_offs", (size_t)(nchunks + 1) * 8, &offs))) return rc;
    HIP_TRY(launch_group_count((const uint64_t *)tab, cap, (int32_t *)cc, nchunks, (int64_t *)offs, st));
    HIP_TRY(hipMemcpyAsync(&n, (int64_t *)offs + nchunks, 8, hipMemcpyDeviceToHost, st));
  }
  HIP_TRY(hipMemcpyAsync(&overflow, ovf, 4, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (overflow) return fail(PHIP_ERR_UNSUPPORTED, "numGroupsLimit pass: hash table overflow (%lld slots)", (long long)cap);
  if ((rc = ws.get("lim_slots", (size_t)std::max<int64_t>(n, 1) * 8, &slots))) return rc;
  HIP_TRY(launch_group_compact((const uint64_t *)tab, cap, (const int64_t *)offs, nchunks, (int64_t *)slots, st));
  // (segment, first doc) order -> ranks -> kept entries
  size_t sort1 = 0, sort2 = 0, scanb = 0;
  HIP_TRY(launch_sort_pairs(nullptr, &sort1, nullptr, nullptr, nullptr, nullptr, false, n, 64, st));
  HIP_TRY(launch_sort_pairs(nullptr, &sort2, nullptr, nullptr, nullptr, nullptr, true, n, 64, st));
  HIP_TRY(launch_limit_runs(nullptr, &scanb, nullptr, n, nullptr, nullptr, st));
  const size_t n8 = (size_t)std::max<int64_t>(n, 1) * 8;
  void *sk0, *sk1, *ix0, *ix1, *k2a, *k2b, *s2a, *s2b, *segc, *segs_start, *tmp, *head, *run;
  if ((rc = ws.get("lim_sk0", n8, &sk0)) || (rc = ws.get("lim_sk1", n8, &sk1)) ||
      (rc = ws.get("lim_ix0", n8, &ix0)) || (rc = ws.get("lim_ix1", n8, &ix1)) ||
      (rc = ws.get("lim_k2a", n8, &k2a)) || (rc = ws.get("lim_k2b", n8, &k2b)) ||
      (rc = ws.get("lim_s2a", n8, &s2a)) || (rc = ws.get("lim_s2b", n8, &s2b)) ||
      (rc = ws.get("lim_segc", (size_t)S * 16, &segc)) || (rc = ws.get("lim_segs", (size_t)S * 8, &segs_start)) ||
      (rc = ws.get("lim_tmp", std::max(std::max(sort1, sort2), scanb) + 256, &tmp)) ||
      (rc = ws.get("lim_head", n8, &head)) || (rc = ws.get("lim_run", n8, &run)))
    return rc;
  // sort by (segment, first doc), then every segment's extent from its run boundaries
  HIP_TRY(launch_limit_prepare((const int64_t *)slots, n, (const uint64_t *)hk, (const uint32_t *)fd, S,
                               (uint64_t *)sk0, (int32_t *)ix0, st));
  const int end1 = 32 + std::max(1, num_bits_per_value(S - 1));
  HIP_TRY(launch_sort_pairs(tmp, &sort1, (const uint64_t *)sk0, (uint64_t *)sk1, ix0, ix1, false, n, end1, st));
  int64_t *seg_first = (int64_t *)segc, *seg_last = (int64_t *)segc + S;
  HIP_TRY(hipMemsetAsync(segc, 0xff, (size_t)S * 16, st));
  HIP_TRY(launch_limit_bounds((const uint64_t *)sk1, n, seg_first, seg_last, st));
  std::vector<int64_t> bounds(2 * (size_t)S);
  HIP_TRY(hipMemcpyAsync(bounds.data(), segc, (size_t)S * 16, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  std::vector<int64_t> seg_start(S);
  int64_t kept = 0;
  *limit_reached = 0;
  for (int s = 0; s < S; s++) {
    const int64_t cnt = bounds[s] < 0 ? 0 : bounds[S + s] - bounds[s] + 1;
    seg_start[s] = bounds[s] < 0 ? 0 : bounds[s];
    kept += std::min<int64_t>(cnt, limit);
    if (cnt >= limit) *limit_reached = 1;  // GroupByOperator.java:116: numGroups >= numGroupsLimit
  }
  HIP_TRY(hipMemcpyAsync(segs_start, seg_start.data(), (size_t)S * 8, hipMemcpyHostToDevice, st));
  HIP_TRY(launch_limit_select((const uint64_t *)sk1, (const int32_t *)ix1, n, (const int64_t *)segs_start, limit,
                              (const int64_t *)slots, (const uint64_t *)hk, S, (uint64_t *)k2a, (int64_t *)s2a, st));
  // one segment: the kept entries are exactly the first `kept` positions (the rest sort last anyway)
  HIP_TRY(launch_sort_pairs(tmp, &sort2, (const uint64_t *)k2a, (uint64_t *)k2b, s2a, s2b, true, S == 1 ? kept : n, 64, st));
  HIP_TRY(launch_limit_runs(tmp, &scanb, (const uint64_t *)k2b, kept, (int32_t *)head, (int32_t *)run, st));
  int32_t runs = 0;
  if (kept > 0) HIP_TRY(hipMemcpyAsync(&runs, (int32_t *)run + kept - 1, 4, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  void *k_out, *v_out, *l_out, *h_out = nullptr;
  const size_t r1 = (size_t)std::max(runs, 1);
  if ((rc = ws.get("lim_keys_out", r1 * 8, &k_out)) ||
      (rc = ws.get("lim_vals_out", r1 * std::max(naggs, 1) * 8, &v_out)) ||
      (rc = ws.get("lim_longs_out", r1 * std::max(naggs, 1) * 8, &l_out)) ||
      (nhll && (rc = ws.get("lim_hll_out", r1 * nhll * m_regs, &h_out))))
    return rc;
  HIP_TRY(launch_limit_reduce((const uint64_t *)k2b, (const int64_t *)s2b, kept, (const int32_t *)head,
                              (const int32_t *)run, cap, naggs, P.dq.own_count_rows, (const int32_t *)(P.base + P.kinds_off),
                              (const uint64_t *)tab, (const uint32_t *)hll, nhll, P.log2m, (int64_t *)k_out,
                              (double *)v_out, (int64_t *)l_out, (uint8_t *)h_out, st));
  *keys = k_out;
  *ov = v_out;
  *ol = l_out;
  *oh = h_out;
  *ngroups = runs;
  return PHIP_OK;
}

// Selection (select.hip): after the filter launch, rank the matched docs per work tile, give each entry its rows
// (first LIMIT in doc order, concatenated in segment order up to LIMIT) and gather the select expressions.
// Blocks until the rows are in impl.sel_values; kept[e] receives each entry's kept rows (numDocsScanned).
static int32_t execute_select(Plan &P, Workspace &ws, hipStream_t st, ResultImpl &impl, std::vector<int64_t> &kept,
                              int64_t *num_rows, float *gather_ms) {
  const DevSelQuery *dsq = (const DevSelQuery *)(P.base + P.sq_off);
  const int64_t tw = P.total_work;
  const size_t nent = P.dsegs.size();
  int32_t rc;
  int64_t tot[2] = {0, 0};
  kept.assign(nent, 0);
  *num_rows = 0;
  *gather_ms = 0.f;
  impl.sel_dicts = P.sel_dicts;  // (a raw STRING expression's own dictionary replaces its entry below)
  for (int k = 0; k < P.nsel; k++) {
    if (P.sel_str_ptrs[k].empty()) continue;
    auto rd = std::make_shared<Device::Remap>();  // (no row: an empty dictionary)
    rd->type = PHIP_TYPE_STRING;
    rd->width = 1;
    impl.sel_dicts[k] = rd;
  }
  if (tw > 0) {
    size_t tb = 0;
    HIP_TRY(launch_select_scan(nullptr, &tb, nullptr, nullptr, tw + 1, st));
    void *tmp;
    if ((rc = ws.get("sel_scan", std::max<size_t>(tb, 16), &tmp))) return rc;
    HIP_TRY(launch_select_count(dsq, tw, P.sel_tile_cnt, st));
    HIP_TRY(launch_select_scan(tmp, &tb, P.sel_tile_cnt, P.sel_tile_off, tw + 1, st));
    HIP_TRY(launch_select_bases(dsq, P.sel_base, P.sel_kept, P.sel_total, st));
    HIP_TRY(hipMemcpyAsync(tot, P.sel_total, 16, hipMemcpyDeviceToHost, st));
    if (nent) HIP_TRY(hipMemcpyAsync(kept.data(), P.sel_kept, nent * 8, hipMemcpyDeviceToHost, st));
  }
  HIP_TRY(hipStreamSynchronize(st));
  const int64_t rows = tot[0];
  impl.sel_values.assign((size_t)rows * P.nsel, 0);
  if (rows > 0) {
    void *out;
    if ((rc = ws.get("sel_out", (size_t)rows * P.nsel * 8, &out))) return rc;
    HIP_TRY(hipEventRecord(P.ev[4], st));
    HIP_TRY(launch_select_gather(dsq, tw, (uint64_t *)out, rows, st));
    HIP_TRY(hipEventRecord(P.ev[2], st));
    HIP_TRY(hipMemcpyAsync(impl.sel_values.data(), out, (size_t)rows * P.nsel * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    HIP_TRY(hipEventElapsedTime(gather_ms, P.ev[4], P.ev[2]));
    // raw STRING expressions: the rows' bytes gathered by locator, then the distinct row values (bytewise order) as
    // this result's dictionary of the column, the rows pointing into it
    for (int k = 0; k < P.nsel; k++) {
      if (P.sel_str_ptrs[k].empty()) continue;
      const std::vector<const void *> &ptrs = P.sel_str_ptrs[k];
      const size_t ns = ptrs.size() / 2;
      void *tab, *lens, *doff, *dst;
      if ((rc = ws.get("sel_str_tab", ptrs.size() * 8, &tab)) || (rc = ws.get("sel_str_lens", (size_t)rows * 4, &lens)) ||
          (rc = ws.get("sel_str_off", (size_t)rows * 8, &doff)))
        return rc;
      const uint64_t *loc = (const uint64_t *)out + (size_t)k * rows;
      HIP_TRY(hipMemcpyAsync(tab, ptrs.data(), ptrs.size() * 8, hipMemcpyHostToDevice, st));
      HIP_TRY(launch_select_str_lens(loc, rows, (const uint64_t *const *)tab + ns, (uint32_t *)lens, st));
      std::vector<uint32_t> hl((size_t)rows);
      HIP_TRY(hipMemcpyAsync(hl.data(), lens, (size_t)rows * 4, hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
      std::vector<uint64_t> ho((size_t)rows + 1, 0);
      for (int64_t r = 0; r < rows; r++) ho[(size_t)r + 1] = ho[(size_t)r] + hl[(size_t)r];
      if ((rc = ws.get("sel_str_bytes", std::max<uint64_t>(ho[(size_t)rows], 16), &dst))) return rc;
      HIP_TRY(hipMemcpyAsync(doff, ho.data(), (size_t)rows * 8, hipMemcpyHostToDevice, st));
      HIP_TRY(launch_select_str_bytes(loc, rows, (const uint8_t *const *)tab, (const uint64_t *const *)tab + ns,
                                      (const uint64_t *)doff, (uint8_t *)dst, st));
      std::vector<uint8_t> hb(ho[(size_t)rows]);
      if (!hb.empty()) HIP_TRY(hipMemcpyAsync(hb.data(), dst, hb.size(), hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
      std::vector<std::string> vals((size_t)rows);
      for (int64_t r = 0; r < rows; r++) vals[(size_t)r].assign((const char *)hb.data() + ho[(size_t)r], hl[(size_t)r]);
      std::vector<std::string> uniq = vals;
      std::sort(uniq.begin(), uniq.end());
      uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
      size_t width = 1;
      for (const auto &u : uniq) width = std::max(width, u.size());
      auto rd = std::make_shared<Device::Remap>();
      rd->type = PHIP_TYPE_STRING;
      rd->width = (int32_t)width;
      rd->card = (int32_t)uniq.size();
      rd->values.assign(uniq.size() * width, 0);
      for (size_t i = 0; i < uniq.size(); i++) memcpy(rd->values.data() + i * width, uniq[i].data(), uniq[i].size());
      for (int64_t r = 0; r < rows; r++)
        impl.sel_values[(size_t)k * rows + r] =
            (uint64_t)(std::lower_bound(uniq.begin(), uniq.end(), vals[(size_t)r]) - uniq.begin());
      impl.sel_dicts[k] = rd;
    }
  }
  *num_rows = rows;
  return PHIP_OK;
}

// EXEC_FULL: one execution end to end (phip_plan_execute). EXEC_PARTIAL: the kernels up to the dense
// group table, handed to the caller (phip_plan_execute_partial). EXEC_FINISH: compaction / trim / copy-out
// of the caller-merged table (phip_plan_finish).
enum { EXEC_FULL = 0, EXEC_PARTIAL = 1, EXEC_FINISH = 2 };
constexpr int64_t kHistMinMatchNum = 3, kHistMinMatchDen = 10;  // Plan::hist_mask: matched >= 30 % of the docs
constexpr int64_t kWalkBatchDocsPerCu = 6144;  // Plan::walk_adaptive: matched docs per CU from which the batched walk runs
constexpr int32_t kGrowHash = -100;  // execute_plan: the hash table overflowed (internal status: execute_growing)
static_assert(ACC_COUNT == PHIP_ROW_COUNT && ACC_SUM_I64 == PHIP_ROW_SUM_I64 && ACC_SUM_F64 == PHIP_ROW_SUM_F64 &&
                  ACC_MIN_F64 == PHIP_ROW_MIN && ACC_MAX_F64 == PHIP_ROW_MAX && ACC_HLL == PHIP_ROW_HLL,
              "partial row kinds are the accumulator kinds");
static_assert(kMaxAggs + 1 <= PHIP_PARTIAL_MAX_ROWS, "phip_partial.row_kinds holds every row");

static int32_t execute_plan(Plan &P, phip_result **out_result, uint64_t *filter_words, int mode = EXEC_FULL,
                            phip_partial *part = nullptr, const phip_partial *merged = nullptr) {
  Device *dev = P.dev;
  std::lock_guard<std::mutex> xlock(P.exec_mu);
  // (a node part's hash table goes out too: node.cpp inserts the other parts' groups into the root's table)
  if (mode != EXEC_FULL && (!P.group_by || (P.dq.mode == GB_HASH && !P.node_part)))
    return fail(PHIP_ERR_UNSUPPORTED, "partial tables: dense group-by and aggregation plans only (this plan: %s)",
                P.group_by ? "hash-table key space" : "selection");
  if (mode == EXEC_FINISH) {
    if (!P.partial_pending) return fail(PHIP_ERR_INVALID, "phip_plan_finish without a pending phip_plan_execute_partial");
    if (merged->num_groups != P.dq.num_groups || merged->num_rows != 1 + P.naggs || merged->table != (uint64_t *)P.gtab)
      return fail(PHIP_ERR_INVALID, "phip_plan_finish: partial does not belong to this plan");
    for (int a = 0; a < P.naggs; a++) {
      const int k = merged->row_kinds[1 + a], own = P.dq.aggs[a].acc;
      if (k != own && !(own == ACC_SUM_I64 && k == ACC_SUM_F64))
        return fail(PHIP_ERR_INVALID, "phip_plan_finish: row %d kind %d (plan: %d)", 1 + a, k, own);
    }
  }
  if (mode != EXEC_FINISH && P.partial_pending)  // the caller still owns the table (it may be all-reducing it)
    return fail(PHIP_ERR_INVALID, "plan has a pending partial table: phip_plan_finish or phip_plan_abandon_partial first");
  if (mode != EXEC_FINISH) {
    int32_t drc = check_deadline(P, "before the launches");
    if (drc) return drc;
  }
  // measurement only (PHIP_HOST_TRACE=1): host microseconds per phase of this call, one stderr line per execution
  static const bool host_trace = getenv("PHIP_HOST_TRACE") != nullptr;
  using hclock = std::chrono::steady_clock;
  hclock::time_point ht[5];
  if (host_trace) ht[0] = hclock::now();
  HIP_TRY(hipSetDevice(dev->ordinal));
  LaneGuard lg{dev};
  {
    int32_t lrc = acquire_lane(dev, &lg.lane);
    if (lrc) return lrc;
  }
  if (host_trace) ht[1] = hclock::now();
  hipStream_t st = lg.lane->stream;
  Workspace &ws = lg.lane->ws;
  // Opt-in (PHIP_GRAPH=1): replay a captured hipGraph from the second execution on. Measured on
  // MI355X it saves nothing once the plan is prepared (host time per execution is ~50 us either way),
  // and event records inside a replayed graph did not give trustworthy kernel times, so eager is the
  // default. Group-by needs a host step mid-way and always runs eager.
  const bool graphable = !P.group_by && !filter_words && getenv("PHIP_GRAPH") != nullptr;
  if (graphable && P.executions >= 1 && !P.graph_exec && !P.graph_failed) {
    hipGraph_t g = nullptr;
    bool ok = hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal) == hipSuccess;
    int32_t rc = ok ? enqueue_plan(P, st) : PHIP_ERR_HIP;
    hipError_t e = hipStreamEndCapture(st, &g);
    if (ok && rc == PHIP_OK && e == hipSuccess && g &&
        hipGraphInstantiate(&P.graph_exec, g, nullptr, nullptr, 0) == hipSuccess) {
      (void)hipGraphDestroy(g);
    } else {
      if (g) (void)hipGraphDestroy(g);
      P.graph_exec = nullptr;
      P.graph_failed = true;
      (void)hipGetLastError();
    }
  }
  if (P.graph_exec) {
    HIP_TRY(hipGraphLaunch(P.graph_exec, st));
  } else if (mode != EXEC_FINISH) {
    int32_t rc = enqueue_plan(P, st);
    if (rc) return rc;
  }
  if (host_trace) ht[2] = hclock::now();
  if (mode != EXEC_FINISH) {
    P.executions++;
    if (P.total_work == 0) {  // no kernel ran: nothing matched, no registers set
      memset(P.pinned + 64, 0, (size_t)P.nmatch * 8 + (P.nhll && !P.group_by ? ((size_t)P.nhll << P.log2m) * 4 : 0));
    }
  }
  DevAggQuery &dq = P.dq;
  const int nseg = P.nseg, naggs = P.naggs, nhll = P.nhll, log2m = P.log2m, m_regs = P.m_regs;
  const bool group_by = P.group_by, has_filter = P.has_filter, need_agg = P.need_agg;
  const int64_t total_work = P.total_work, total_docs = P.total_docs, docs_in_work = P.docs_in_work;
  const int num_projected = P.num_projected;
  const int64_t filter_nwords = P.filter_nwords;
  const int32_t *dev_kinds = (const int32_t *)(P.base + P.kinds_off);
  void *gtab = P.gtab, *ghll = P.ghll;
  const std::vector<DevSeg> &dsegs = P.dsegs;
  const std::vector<std::shared_ptr<Device::Remap>> &gb_dicts = P.gb_dicts;
  int32_t rc = PHIP_OK;
  if (filter_words && P.need_mask)
    HIP_TRY(hipMemcpyAsync(filter_words, P.fo, (size_t)filter_nwords * 8, hipMemcpyDeviceToHost, st));

  auto impl = std::make_unique<ResultImpl>();
  phip_result &r = impl->pub;
  memset(&r, 0, sizeof(r));
  const uint64_t *fin = P.pinned;
  const uint64_t *segm = P.pinned + 64;
  const uint32_t *hll_host = (const uint32_t *)(P.pinned + 64 + P.nmatch);

  // this GPU's statistics (valid once the stream has synchronised)
  auto local_stats = [&](int64_t st6[6]) {
    const int64_t m = has_filter ? (int64_t)fin[32] : docs_in_work;
    st6[0] = m;  // several programs: summed over them (FilteredAggregationOperator adds its infos' statistics)
    st6[1] = has_filter ? (int64_t)fin[33] : 0;
    st6[2] = m * num_projected;
    st6[3] = total_docs;
    st6[4] = nseg;
    st6[5] = 0;
    if (P.nprog > 1) {  // entries post filter per program: its matched docs x the columns its functions project
      st6[2] = 0;
      for (int p = 0; p < P.nprog; p++) {
        int64_t mp = 0;
        for (int s = 0; s < nseg; s++) mp += has_filter ? (int64_t)segm[p * nseg + s] : P.slot_docs[p * nseg + s];
        int np = 0;
        for (const Plan::ProjCol &pc : P.proj) np += (pc.progs >> p) & 1u;
        st6[2] += mp * np;
      }
    }
    if (has_filter) {  // a segment matched when any of its programs did
      for (int s = 0; s < nseg; s++) {
        bool any = false;
        for (int p = 0; p < P.nprog; p++) any |= segm[p * nseg + s] != 0;
        st6[5] += any ? 1 : 0;
      }
    } else {  // no program filters: every entry's docs match
      for (int s = 0; s < nseg; s++) {
        bool any = false;
        for (int p = 0; p < P.nprog; p++) any |= P.slot_docs[p * nseg + s] != 0;
        st6[5] += any ? 1 : 0;
      }
    }
  };
  // row kinds of the gather: the plan's, or the caller's after a merge that turned int64 sums into doubles
  const int32_t *gather_kinds = dev_kinds;
  std::vector<int32_t> kinds_host(std::max(naggs, 1));
  for (int a = 0; a < naggs; a++) kinds_host[a] = mode == EXEC_FINISH ? merged->row_kinds[1 + a] : dq.aggs[a].acc;
  if (mode == EXEC_FINISH) {
    bool differs = false;
    for (int a = 0; a < naggs; a++) differs |= kinds_host[a] != dq.aggs[a].acc;
    if (differs) {
      void *kb;
      if ((rc = ws.get("finish_kinds", (size_t)naggs * 4, &kb))) return rc;
      HIP_TRY(hipMemcpyAsync(kb, kinds_host.data(), (size_t)naggs * 4, hipMemcpyHostToDevice, st));
      gather_kinds = (const int32_t *)kb;
    }
  }

  int64_t ngroups = 1;
  if (group_by) {
    const int64_t nchunks = ceil_div(dq.num_groups, 1024);
    void *cc, *offs, *keys;
    rc = ws.get("gb_chunk_counts", (size_t)nchunks * 4, &cc);
    if (rc) return rc;
    rc = ws.get("gb_offsets", (size_t)(nchunks + 1) * 8, &offs);
    if (rc) return rc;
    HIP_TRY(launch_group_count((const uint64_t *)gtab, dq.num_groups, (int32_t *)cc, nchunks, (int64_t *)offs, st));
    // One round trip when the key space's rows fit the lane's mapped landing area (default up to 64 MiB): compaction,
    // gather and the count run back to back and write the results into mapped host memory, so the host neither waits
    // for the count nor copies the outputs (a wait + a copy command less per group-by query). HLL registers cross
    // packed four to a word (PHIP_GB_ONE_TRIP_HLL=0: those plans keep the two trips); PHIP_GB_ONE_TRIP_MAX = the
    // landing area's bytes, 0 = off.
    const char *otm = getenv("PHIP_GB_ONE_TRIP_MAX");  // (read per execution: A/B inside one process)
    const int64_t one_trip_max = otm ? (int64_t)atoll(otm) : (int64_t)64 << 20;
    const int64_t ndense = dq.num_groups;
    const char *oth = getenv("PHIP_GB_ONE_TRIP_HLL");
    const bool one_trip_hll = !oth || atoi(oth) != 0;
    const int64_t one_trip_bytes = 64 + ndense * (8 + 16 * (int64_t)naggs + (int64_t)nhll * m_regs);
    // (a plan whose numGroupsLimit or trim can apply goes one trip too, speculatively: when the count then reaches
    // the limit or exceeds trimSize, the limit pass / the compaction and gather into device buffers for the trim run
    // below as without it -- the table is still intact)
    bool one_trip = mode == EXEC_FULL && dq.mode != GB_HASH && (nhll == 0 || one_trip_hll) && ndense > 0 &&
                    one_trip_bytes <= one_trip_max;
    const uint8_t *landing = nullptr;
    if (one_trip) {
      // the lane's landing area (count | keys | values | exact sums | registers over the whole key space), grown on
      // demand: read out below before the lane is released
      void *lh = nullptr, *ld = nullptr;
      if ((rc = ws.get_mapped("gb_landing", (size_t)one_trip_bytes, &lh, &ld))) return rc;
      landing = (const uint8_t *)lh;
      void *dkeys;
      if ((rc = ws.get("gb_keys", (size_t)ndense * 8, &dkeys))) return rc;
      uint8_t *hd = (uint8_t *)ld;
      const size_t vb_max = (size_t)ndense * naggs * 8;
      HIP_TRY(launch_group_compact((const uint64_t *)gtab, ndense, (const int64_t *)offs, nchunks, (int64_t *)dkeys, st));
      HIP_TRY(launch_group_gather_mapped((const int64_t *)dkeys, (const int64_t *)offs + nchunks, ndense, naggs,
                                         dq.own_count_rows, gather_kinds, (const uint64_t *)gtab, (int64_t *)hd,
                                         (int64_t *)(hd + 64), (double *)(hd + 64 + ndense * 8),
                                         (int64_t *)(hd + 64 + ndense * 8 + vb_max), (const uint32_t *)ghll, nhll,
                                         log2m, (uint32_t *)(hd + 64 + ndense * 8 + 2 * vb_max), st));
      if (P.total_events) HIP_TRY(hipEventRecord(P.ev[3], st));
      HIP_TRY(hipStreamSynchronize(st));
      memcpy(&ngroups, landing, 8);
      if (ngroups < 0 || ngroups > ndense)
        return fail(PHIP_ERR_HIP, "group count %lld outside the key space %lld", (long long)ngroups, (long long)ndense);
      if (P.trim_size > 0 && ngroups > P.trim_size && (naggs > 0 || P.order_nkeys > 0 || P.order_terms.num_terms > 0))
        one_trip = false;  // the trim needs the outputs on the device
      if (P.num_groups_limit > 0 && ngroups >= P.num_groups_limit) one_trip = false;  // the limit pass decides
    } else {
      int64_t total = 0;
      HIP_TRY(hipMemcpyAsync(&total, (int64_t *)offs + nchunks, 8, hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
      ngroups = total;
    }
    if ((rc = check_deadline(P, "after the group-by kernels"))) return rc;
    if (mode == EXEC_PARTIAL) {
      // per-segment numGroupsLimit needs the first-seen record pass of phip_plan_execute
      if (P.num_groups_limit > 0 && ngroups >= P.num_groups_limit)
        return fail(PHIP_ERR_UNSUPPORTED, "partial table: %lld groups reach numGroupsLimit %lld", (long long)ngroups,
                    (long long)P.num_groups_limit);
      if (dq.mode == GB_HASH) {  // a full table cannot go out: the node plan takes the record path (which grows it)
        uint32_t ovf = 0;
        HIP_TRY(hipMemcpyAsync(&ovf, dq.hash_overflow, 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        if (ovf) return fail(PHIP_ERR_UNSUPPORTED, "partial table: the group-by hash table is full");
      }
      memset(part, 0, sizeof(*part));
      part->num_groups = dq.num_groups;
      part->num_rows = 1 + naggs;
      part->num_hll = nhll;
      part->log2m = nhll ? log2m : 0;
      part->device = dev->ordinal;
      part->table = (uint64_t *)gtab;
      part->hll = nhll ? (uint32_t *)ghll : nullptr;
      part->row_kinds[0] = PHIP_ROW_COUNT;
      for (int a = 0; a < naggs; a++) part->row_kinds[1 + a] = dq.aggs[a].acc;  // ACC_* == PHIP_ROW_*
      local_stats(part->stats);
      part->global_keys = 1;  // (tuple keys: this device's own virtual ids, so the record merge)
      for (const auto &d : gb_dicts) part->global_keys &= d->global ? 1 : 0;
      P.partial_pending = true;
      P.clean = true;
      lg.done = true;
      return PHIP_OK;
    }
    void *ov = nullptr, *ol = nullptr, *oh = nullptr;
    uint32_t overflow = 0;
    // some segment may have reached numGroupsLimit: the first-seen pass decides which keys it kept (and the
    // normal pass's compaction would be thrown away)
    const bool limit_pass = mode == EXEC_FULL && P.num_groups_limit > 0 && ngroups >= P.num_groups_limit;
    // the compacted keys, values, exact sums and registers of the groups back to back in one buffer (one copy out)
    auto contiguous_out = [&](const char *name, int64_t n, void **k, void **v, void **l, void **h) -> int32_t {
      void *base;
      const size_t kb = (size_t)n * 8, vb = (size_t)n * naggs * 8, hb = (size_t)n * nhll * m_regs;
      int32_t rc2 = ws.get(name, std::max<size_t>(kb + 2 * vb + hb, 16), &base);
      if (rc2) return rc2;
      *k = base;
      *v = (uint8_t *)base + kb;
      *l = (uint8_t *)base + kb + vb;
      *h = nhll ? (uint8_t *)base + kb + 2 * vb : nullptr;
      return PHIP_OK;
    };
    bool out_contig = false;
    if (!limit_pass && !one_trip) {
      rc = contiguous_out("gb_out", ngroups, &keys, &ov, &ol, &oh);
      if (rc) return rc;
      out_contig = true;
      HIP_TRY(launch_group_compact((const uint64_t *)gtab, dq.num_groups, (const int64_t *)offs, nchunks, (int64_t *)keys, st));
      HIP_TRY(launch_group_gather((const int64_t *)keys, ngroups, dq.num_groups, naggs, dq.own_count_rows, gather_kinds,
                                  (const uint64_t *)gtab,
                                  (const uint32_t *)ghll, nhll, log2m, (double *)ov, (int64_t *)ol, (uint8_t *)oh, st));
      if (dq.mode == GB_HASH) HIP_TRY(launch_hash_keys((int64_t *)keys, ngroups, dq.gb_keys, st));
    }
    if (dq.mode == GB_HASH) HIP_TRY(hipMemcpyAsync(&overflow, dq.hash_overflow, 4, hipMemcpyDeviceToHost, st));
    if (limit_pass) {
      HIP_TRY(hipStreamSynchronize(st));
      if (overflow) return kGrowHash;  // (execute_growing: a table twice the size, and the execution again)
      const int64_t matched_docs = has_filter ? (int64_t)fin[32] : docs_in_work;
      rc = group_limit(P, ws, st, matched_docs, &keys, &ov, &ol, &oh, &ngroups, &r.num_groups_limit_reached,
                       (const int64_t *)offs);
      if (rc) return rc;
    }
    if (P.trim_size > 0 && ngroups > P.trim_size && (naggs > 0 || P.order_nkeys > 0 || P.order_terms.num_terms > 0)) {
      if ((rc = check_deadline(P, "before the server trim"))) return rc;
      // ORDER BY <aggregation> with more groups than trimSize: keep the top trimSize on the device
      // (IndexedTable.finish -> TableResizer.getTopRecords), so only those records cross PCIe.
      size_t sbytes = 0;
      const int32_t *order = nullptr;
      KeyOrder ko{};
      ko.num_group_by = P.num_group_by;
      ko.num_keys = P.order_nkeys;
      for (int k = 0; k < P.num_group_by; k++) ko.card[k] = P.gb_radix[k];  // (a null key sorts last ascending)
      for (int j = 0; j < P.order_nkeys; j++) {
        ko.gb[j] = (P.order_keys[j] > 0 ? P.order_keys[j] : -P.order_keys[j]) - 1;
        ko.desc[j] = P.order_keys[j] < 0;
      }
      const KeyOrder *kop = P.order_nkeys > 0 ? &ko : nullptr;
      OrderTerms ot = P.order_terms;
      for (int k = 0; k < P.num_group_by; k++) ot.card[k] = P.gb_radix[k];
      const bool terms = ot.num_terms > 0;
      if (terms)
        HIP_TRY(launch_trim_order_terms(nullptr, nullptr, &ot, ngroups, naggs, nullptr, 0, 0, nullptr, &sbytes, &order,
                                        st));
      else
        HIP_TRY(launch_trim_order(nullptr, nullptr, kop, ngroups, naggs, P.order_agg, P.order_desc, nullptr, &sbytes,
                                  &order, st));
      void *scratch, *k2, *v2, *l2, *h2 = nullptr;
      const int64_t k = P.trim_size;
      if ((rc = ws.get("trim_scratch", sbytes, &scratch))) return rc;
      if ((rc = contiguous_out("trim_out", k, &k2, &v2, &l2, &h2))) return rc;
      if (terms)
        HIP_TRY(launch_trim_order_terms((const double *)ov, (const int64_t *)keys, &ot, ngroups, naggs, (const uint8_t *)oh,
                                        nhll ? (int64_t)nhll * m_regs : 0, m_regs, scratch, &sbytes,
                                        &order, st));
      else
        HIP_TRY(launch_trim_order((const double *)ov, (const int64_t *)keys, kop, ngroups, naggs, P.order_agg,
                                  P.order_desc, scratch, &sbytes, &order, st));
      HIP_TRY(launch_trim_gather(order, k, naggs, nhll ? (int64_t)nhll * m_regs : 0, (const int64_t *)keys,
                                 (const double *)ov, (const int64_t *)ol, (const uint8_t *)oh, (int64_t *)k2,
                                 (double *)v2, (int64_t *)l2, (uint8_t *)h2, st));
      keys = k2;
      ov = v2;
      ol = l2;
      oh = h2;
      ngroups = k;
      r.num_groups_trimmed = 1;
      out_contig = true;
    }
    std::vector<int64_t> hkeys(ngroups);
    impl->values.resize(ngroups * naggs);
    impl->longs.resize(ngroups * naggs);
    impl->hll.resize((size_t)ngroups * nhll * m_regs);
    const size_t kb = (size_t)ngroups * 8, vb = (size_t)ngroups * naggs * 8, hb = impl->hll.size();
    std::vector<uint8_t> staged;
    if (one_trip) {  // (already waited for: the outputs are in the mapped landing area)
      const uint8_t *h = landing + 64;
      memcpy(hkeys.data(), h, kb);
      if (vb) {
        memcpy(impl->values.data(), h + ndense * 8, vb);
        memcpy(impl->longs.data(), h + ndense * 8 + (size_t)ndense * naggs * 8, vb);
      }
      if (hb) memcpy(impl->hll.data(), h + ndense * 8 + 2 * (size_t)ndense * naggs * 8, hb);
    } else if (ngroups && out_contig) {  // one copy of the contiguous outputs (each small copy is its own command)
      staged.resize(kb + 2 * vb + hb);
      HIP_TRY(hipMemcpyAsync(staged.data(), keys, staged.size(), hipMemcpyDeviceToHost, st));
    } else if (ngroups) {
      HIP_TRY(hipMemcpyAsync(hkeys.data(), keys, ngroups * 8, hipMemcpyDeviceToHost, st));
      if (naggs) {
        HIP_TRY(hipMemcpyAsync(impl->values.data(), ov, ngroups * naggs * 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(impl->longs.data(), ol, ngroups * naggs * 8, hipMemcpyDeviceToHost, st));
      }
      if (nhll) HIP_TRY(hipMemcpyAsync(impl->hll.data(), oh, impl->hll.size(), hipMemcpyDeviceToHost, st));
    }
    if (!one_trip) {
      if (P.total_events) HIP_TRY(hipEventRecord(P.ev[3], st));
      HIP_TRY(hipStreamSynchronize(st));
    }
    if (!staged.empty()) {
      memcpy(hkeys.data(), staged.data(), kb);
      if (vb) {
        memcpy(impl->values.data(), staged.data() + kb, vb);
        memcpy(impl->longs.data(), staged.data() + kb + vb, vb);
      }
      if (hb) memcpy(impl->hll.data(), staged.data() + kb + 2 * vb, hb);
    }
    if (overflow) return kGrowHash;
    impl->keys.resize(ngroups * P.num_group_by);
    for (int64_t g = 0; g < ngroups; g++) {
      int64_t key = hkeys[g];
      for (int k = 0; k < P.num_group_by; k++) {
        impl->keys[g * P.num_group_by + k] = (int32_t)(key % P.gb_radix[k]);  // (== card: the null key)
        key /= P.gb_radix[k];
      }
    }
    // tuple keys: each group's virtual id back to the query's columns' ids
    const int KO = P.tuple_keys ? (int)P.tuple_dicts.size() : P.num_group_by;
    const auto &DO = P.tuple_keys ? P.tuple_dicts : gb_dicts;
    const auto &RO = P.tuple_keys ? P.tuple_radix : P.gb_radix;
    if (P.tuple_keys) {
      const Device::Remap &tr = *P.tuple_remap;
      const int64_t U = tr.card;
      std::vector<int32_t> ek((size_t)ngroups * KO);
      for (int64_t g = 0; g < ngroups; g++) {
        const int64_t v = impl->keys[g];
        for (int k = 0; k < KO; k++)
          ek[g * KO + k] = (int32_t)((tr.tuples[(size_t)P.tuple_word[k] * U + v] / P.tuple_stride[k]) % (uint64_t)RO[k]);
      }
      impl->keys.swap(ek);
    }
    impl->dicts = DO;  // (num_groups_limit_reached was set by group_limit, before any trim)
    for (int k = 0; k < KO; k++) {
      if (!DO[k]->raw) continue;
      // a raw column's result dictionary: the values its groups use, ascending; group keys re-pointed at it
      std::vector<int32_t> used;
      used.reserve(ngroups);
      const int32_t null_id = RO[k] > DO[k]->card ? DO[k]->card : -1;
      for (int64_t g = 0; g < ngroups; g++)
        if (impl->keys[g * KO + k] != null_id) used.push_back(impl->keys[g * KO + k]);
      std::sort(used.begin(), used.end());
      used.erase(std::unique(used.begin(), used.end()), used.end());
      auto rd = std::make_shared<Device::Remap>();
      rd->type = DO[k]->type;
      rd->card = (int32_t)used.size();
      const int w = type_width(rd->type);
      rd->values.resize(used.size() * w);
      for (size_t i = 0; i < used.size(); i++) {
        const int64_t v = DO[k]->raw_base + used[i];
        if (w == 4) {
          const int32_t v4 = (int32_t)v;
          memcpy(rd->values.data() + 4 * i, &v4, 4);
        } else {
          memcpy(rd->values.data() + 8 * i, &v, 8);
        }
      }
      for (int64_t g = 0; g < ngroups; g++) {  // (the null key stays one past the values: rd->card)
        int32_t &id = impl->keys[g * KO + k];
        id = id == null_id ? rd->card : (int32_t)(std::lower_bound(used.begin(), used.end(), id) - used.begin());
      }
      impl->dicts[k] = rd;
    }
  } else if (P.done_seq != 0 && !P.graph_exec && !P.select && !filter_words) {
    // the finalize kernel's completion word (Plan::done_seq): spin on the mapped result area; a kernel that has
    // not published within the bound is waited for on the stream (which also reports a failed launch)
    volatile const uint64_t *done = P.pinned + kDoneSlot;
    const auto t0 = std::chrono::steady_clock::now();
    bool seen = false;
    for (uint32_t spin = 0;; spin++) {
      if (*done == P.done_seq) {
        seen = true;
        break;
      }
      if ((spin & 1023u) == 1023u && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) break;
      __builtin_ia32_pause();
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    if (!seen) HIP_TRY(hipStreamSynchronize(st));
  } else {
    HIP_TRY(hipStreamSynchronize(st));
  }
  if (host_trace) ht[3] = hclock::now();
  // selection: the filter's tile masks -> rows (its own launches; event 2 / 4 then bracket the gather kernel)
  std::vector<int64_t> sel_kept;
  int64_t sel_rows = 0;
  float sel_ms = 0.f;
  if (P.select) {
    float t_f = 0.f;
    HIP_TRY(hipEventElapsedTime(&t_f, P.ev[1], P.ev[4]));  // the filter launch, before the events are reused
    if ((rc = execute_select(P, ws, st, *impl, sel_kept, &sel_rows, &sel_ms))) return rc;
    P.sel_filter_ms = t_f;
  }
  const int64_t matched = has_filter ? (int64_t)fin[32] : docs_in_work;
  if (filter_words && !has_filter) {  // no filter program: every doc of the (single) segment matches
    const int64_t n = dsegs.empty() ? 0 : dsegs[0].num_docs;
    for (int64_t w = 0; w < filter_nwords; w++) {
      const int64_t lo = w * 64;
      filter_words[w] = lo >= n ? 0ull : (n - lo >= 64 ? ~0ull : ((1ull << (n - lo)) - 1ull));
    }
  }
  if (!group_by) {
    impl->values.resize(naggs);
    impl->longs.resize(naggs);
    impl->hll.resize((size_t)nhll << (nhll ? log2m : 0));
    for (int a = 0; a < naggs; a++) {
      const int kind = dq.aggs[a].acc;
      uint64_t v = need_agg ? fin[a] : 0;
      if (!need_agg || total_work == 0) v = kind == ACC_COUNT ? (uint64_t)matched : 0;
      if (total_work == 0 && (kind == ACC_MIN_F64 || kind == ACC_MAX_F64)) {
        const double d = kind == ACC_MIN_F64 ? HUGE_VAL : -HUGE_VAL;
        memcpy(&v, &d, 8);
      }
      double d = 0.0;
      int64_t l = 0;
      switch (kind) {
        case ACC_COUNT:
        case ACC_SUM_I64: l = (int64_t)v; d = (double)l; break;
        default: memcpy(&d, &v, 8);
      }
      impl->values[a] = d;
      impl->longs[a] = l;
    }
    if (nhll) for (size_t i = 0; i < ((size_t)nhll << log2m); i++) impl->hll[i] = (uint8_t)hll_host[i];
  }
  float t_all = 0.f, t_scan = 0.f, t_filter = 0.f, t_agg = 0.f;
  if (P.timed && total_work > 0) HIP_TRY(hipEventElapsedTime(&t_scan, P.ev[1], P.ev[2]));
  if (P.total_events) HIP_TRY(hipEventElapsedTime(&t_all, P.ev[0], P.ev[3]));
  else t_all = t_scan;
  if (!P.timed || total_work == 0) {
    // (no markers were recorded: the kernel times read 0)
  } else if (P.split_event) {
    HIP_TRY(hipEventElapsedTime(&t_filter, P.ev[1], P.ev[4]));
    HIP_TRY(hipEventElapsedTime(&t_agg, P.ev[4], P.ev[2]));
  } else if (has_filter && !(need_agg && !P.fused_naggs && !P.fused_gb)) {
    t_filter = t_scan;  // the one kernel between ev[1] and ev[2] is the filter (fused or not)
  } else {
    t_agg = t_scan;
  }
  r.filter_kernel_ms = has_filter ? t_filter : 0.0;
  r.agg_kernel_ms = need_agg ? t_agg : 0.0;
  r.filter_bytes = has_filter ? P.filter_bytes : 0;
  r.stream_bytes = r.filter_bytes;
  if (need_agg) {
    int64_t ab = 0;
    for (int s = 0; s < nseg; s++) {
      for (int p = 0; p < P.nprog; p++) {
        const int64_t m = has_filter ? (int64_t)segm[p * nseg + s] : P.slot_docs[p * nseg + s];
        for (const Plan::ProjCol &pc : P.proj) {
          if (!((pc.progs >> p) & 1u)) continue;
          ab += pc.bits[s] ? ceil_div(m * pc.bits[s], 8) : m * pc.width[s];
          if (pc.bits[s]) ab += std::min<int64_t>(pc.card[s], m) * pc.width[s];
        }
      }
    }
    r.agg_bytes = ab;
  }
  if (P.fused_naggs > 0 || P.fused_gb) {  // one kernel filtered and aggregated: it owns both times and both byte counts
    r.fused = 1;
    r.filter_kernel_ms = t_filter + t_agg;
    r.agg_kernel_ms = 0.0;
    r.filter_bytes += r.agg_bytes;
    r.agg_bytes = 0;
  }

  {
    int64_t st6[6];
    if (mode == EXEC_FINISH) memcpy(st6, merged->stats, sizeof(st6));
    else local_stats(st6);
    r.num_docs_scanned = st6[0];
    r.num_entries_scanned_in_filter = st6[1];
    r.num_entries_scanned_post_filter = st6[2];
    r.num_total_docs = st6[3];
    r.num_segments_processed = (int32_t)st6[4];
    r.num_segments_matched = (int32_t)st6[5];
  }
  impl->seg_docs.assign(std::max(nseg, 1), 0);
  for (int s = 0; s < nseg; s++)
    for (int p = 0; p < P.nprog; p++)
      impl->seg_docs[s] += has_filter ? (int64_t)segm[p * nseg + s] : P.slot_docs[p * nseg + s];
  r.segment_docs_matched = impl->seg_docs.data();
  impl->prog_docs.assign(std::max(P.nprog, 1), 0);
  for (int p = 0; p < P.nprog; p++)
    for (int s = 0; s < nseg; s++)
      impl->prog_docs[p] += has_filter ? (int64_t)segm[p * nseg + s] : P.slot_docs[p * nseg + s];
  r.program_docs_matched = impl->prog_docs.data();
  r.num_aggregations = naggs;
  r.num_groups = group_by ? ngroups : 1;
  r.num_group_by = P.tuple_keys ? (int32_t)P.tuple_dicts.size() : P.num_group_by;
  r.num_hll = nhll;
  r.values = impl->values.data();
  r.long_values = impl->longs.data();
  r.hll_registers = impl->hll.data();
  r.group_keys = impl->keys.data();
  impl->exact.resize(std::max(naggs, 1), 0);
  for (int a = 0; a < naggs; a++) impl->exact[a] = (kinds_host[a] == ACC_COUNT || kinds_host[a] == ACC_SUM_I64) ? 1 : 0;
  r.long_exact = impl->exact.data();
  r.scan_kernel_ms = t_scan;
  r.device_ms = t_all;
  if (P.select) {
    // SelectionOnlyOperator statistics per segment: numDocsScanned = its kept rows, post-filter entries = that x the
    // projected columns; a segment matched when it kept a row
    int64_t docs = 0;
    int32_t segs_matched = 0;
    std::vector<int64_t> per_seg(nseg, 0);
    for (size_t e = 0; e < dsegs.size(); e++) per_seg[dsegs[e].seg_index % nseg] += sel_kept[e];
    for (int s = 0; s < nseg; s++) {
      docs += per_seg[s];
      segs_matched += per_seg[s] > 0 ? 1 : 0;
    }
    r.num_docs_scanned = docs;
    r.num_entries_scanned_post_filter = docs * P.num_projected;
    r.num_segments_matched = segs_matched;
    r.num_rows = sel_rows;
    r.num_select = P.nsel;
    impl->sel_types = P.sel_types;
    r.select_types = impl->sel_types.data();
    r.select_values = impl->sel_values.data();
    r.filter_kernel_ms = has_filter ? P.sel_filter_ms : 0.0;
    r.agg_kernel_ms = sel_ms;  // the projection (gather) kernel
    int64_t per_row = 8 * (int64_t)P.nsel;
    for (size_t i = 0; i < P.sel_bits.size(); i++) per_row += P.sel_bits[i] ? ceil_div(P.sel_bits[i], 8) : P.sel_width[i];
    r.agg_bytes = sel_rows * per_row;
  }
  P.clean = true;
  P.partial_pending = false;
  lg.done = true;
  if (P.hist_mask && !group_by) {  // the next execution's aggregation walk: the id histogram when most docs match
    const int64_t m = has_filter ? (int64_t)fin[32] : docs_in_work;
    const bool on = m * kHistMinMatchDen >= docs_in_work * kHistMinMatchNum;
    P.dq.hist_aggs = on ? P.hist_mask : 0;
    P.agg_lds = on ? P.agg_lds_hist : P.agg_lds_plain;
    static const bool hist_trace = getenv("PHIP_WALK_TRACE") != nullptr;  // measurement: the walk switches
    if (hist_trace) fprintf(stderr, "phip_hist matched %lld of %lld: %s\n", (long long)m, (long long)docs_in_work, on ? "on" : "off");
  }
  if (P.walk_adaptive && group_by) {  // the next execution's group-by walk, from this one's matched docs
    const int64_t m = has_filter ? (int64_t)fin[32] : docs_in_work;
    const int want = m >= kWalkBatchDocsPerCu * (int64_t)dev->num_cus ? 1 : 0;
    static const bool walk_trace = getenv("PHIP_WALK_TRACE") != nullptr;  // measurement: the walk switches
    if (walk_trace)
      fprintf(stderr, "phip_walk matched %lld cur %d want %d blocks %d/%d lds %zu/%zu waves %d/%d rec %d\n",
              (long long)m, P.walk_cur, want, P.walk[0].blocks, P.walk[1].blocks, P.walk[0].lds, P.walk[1].lds,
              P.walk[0].waves, P.walk[1].waves, P.dq.rec_on);
    if (want != P.walk_cur) {
      P.walk_cur = want;
      P.dq.dense_batch = P.walk[want].batched ? 1 : 0;
      P.dq.wg_waves = P.walk[want].waves;
      P.agg_blocks = P.walk[want].blocks;
      P.agg_lds = P.walk[want].lds;
    }
  }
  if (out_result) {
    *out_result = &impl.release()->pub;
  }
  if (host_trace) {
    ht[4] = hclock::now();
    auto us = [&](int a, int b) { return std::chrono::duration<double, std::micro>(ht[b] - ht[a]).count(); };
    fprintf(stderr, "phip_host_trace lane %.1f enqueue %.1f sync %.1f result %.1f total %.1f device %.1f\n", us(0, 1),
            us(1, 2), us(2, 3), us(3, 4), us(0, 4), 1000.0 * r.device_ms);
  }
  return PHIP_OK;
}

// ------------------------------------------------------------------------------------------------
// Aggregation-only partials (the cross-GPU merge of AggregationResultsBlockMerger.java:34-49 on the device): one
// execution, then the result slots encoded as a one-group partial table in device memory -- row 0 matched docs, row
// 1 + a slot a (COUNT / exact SUM as int64, double SUM as its bits, MIN / MAX as the order-preserving image), the six
// statistics after the last row, HLL registers as u8 -- uploaded with one copy from a pinned staging area.
// ------------------------------------------------------------------------------------------------
static inline uint64_t f64_ordered_host(double d) {  // dev_common.h f64_ordered
  uint64_t u;
  memcpy(&u, &d, 8);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
static inline double f64_unordered_host(uint64_t u) {  // dev_common.h f64_unordered (sentinels: +/-inf)
  if (u == ~0ull) return HUGE_VAL;
  if (u == 0ull) return -HUGE_VAL;
  u = (u >> 63) ? (u & 0x7fffffffffffffffull) : ~u;
  double d;
  memcpy(&d, &u, 8);
  return d;
}

static int32_t agg_partial_buffers(Plan &P) {
  if (P.ptab) return PHIP_OK;
  const size_t rows = (size_t)(1 + P.naggs) + 6;
  const size_t hbytes = (size_t)P.nhll << (P.nhll ? P.log2m : 0);
  void *t, *h = nullptr, *st;
  int32_t rc = P.alloc(rows * 8 + 64, &t);
  if (rc) return rc;
  if (hbytes && (rc = P.alloc(hbytes + 64, &h))) return rc;
  HIP_TRY(hipHostMalloc(&st, rows * 8 + hbytes + 64, hipHostMallocDefault));
  P.ptab = (uint64_t *)t;
  P.phll = (uint8_t *)h;
  P.pstage = (uint64_t *)st;
  return PHIP_OK;
}

static int32_t execute_agg_partial(Plan &P, phip_partial *part) {
  if (P.select || P.naggs > kMaxAggs) return fail(PHIP_ERR_UNSUPPORTED, "partial tables: not for selection plans");
  phip_result *res = nullptr;
  int32_t rc = execute_plan(P, &res, nullptr, EXEC_FULL);  // (refuses while a partial is pending)
  if (rc) return rc;
  std::unique_ptr<phip_result, void (*)(phip_result *)> hold(res, [](phip_result *r) {
    delete reinterpret_cast<ResultImpl *>(r);
  });
  std::lock_guard<std::mutex> xlock(P.exec_mu);
  if (P.partial_pending) return fail(PHIP_ERR_INVALID, "plan has a pending partial table");
  if ((rc = agg_partial_buffers(P))) return rc;
  const int na = P.naggs;
  const size_t rows = (size_t)(1 + na);
  uint64_t *h = P.pstage;
  h[0] = (uint64_t)res->num_docs_scanned;
  for (int a = 0; a < na; a++) {
    const int k = P.dq.aggs[a].acc;
    const double v = res->values[a];
    uint64_t w;
    if (k == ACC_COUNT || k == ACC_SUM_I64) w = (uint64_t)res->long_values[a];
    else if (k == ACC_SUM_F64) memcpy(&w, &v, 8);
    else if (k == ACC_MIN_F64 || k == ACC_MAX_F64) w = f64_ordered_host(v);
    else w = 0;  // (HLL: the registers travel in phll)
    h[1 + a] = w;
  }
  const int64_t st6[6] = {res->num_docs_scanned, res->num_entries_scanned_in_filter,
                          res->num_entries_scanned_post_filter, res->num_total_docs, res->num_segments_processed,
                          res->num_segments_matched};
  memcpy(h + rows, st6, sizeof(st6));
  const size_t hbytes = (size_t)P.nhll << (P.nhll ? P.log2m : 0);
  if (hbytes) memcpy((uint8_t *)(h + rows + 6), res->hll_registers, hbytes);
  HIP_TRY(hipSetDevice(P.dev->ordinal));
  LaneGuard lg{P.dev};
  if ((rc = acquire_lane(P.dev, &lg.lane))) return rc;
  hipStream_t st = lg.lane->stream;
  HIP_TRY(hipMemcpyAsync(P.ptab, h, (rows + 6) * 8, hipMemcpyHostToDevice, st));
  if (hbytes) HIP_TRY(hipMemcpyAsync(P.phll, h + rows + 6, hbytes, hipMemcpyHostToDevice, st));
  HIP_TRY(hipStreamSynchronize(st));
  lg.done = true;
  memset(part, 0, sizeof(*part));
  part->num_groups = 1;
  part->num_rows = (int32_t)rows;
  part->num_hll = P.nhll;
  part->log2m = P.nhll ? P.log2m : 0;
  part->device = P.dev->ordinal;
  part->table = P.ptab;
  part->hll = (uint32_t *)P.phll;
  part->hll_u8 = 1;
  part->row_kinds[0] = PHIP_ROW_COUNT;
  for (int a = 0; a < na; a++) part->row_kinds[1 + a] = P.dq.aggs[a].acc;
  memcpy(part->stats, st6, sizeof(st6));
  part->stats_dev = (int64_t *)(P.ptab + rows);
  P.part_times[0] = res->scan_kernel_ms;
  P.part_times[1] = res->device_ms;
  P.part_times[2] = res->filter_kernel_ms;
  P.part_times[3] = res->agg_kernel_ms;
  P.part_times[4] = res->fused;
  P.part_bytes[0] = res->filter_bytes;
  P.part_bytes[1] = res->agg_bytes;
  P.part_bytes[2] = res->stream_bytes;
  part->global_keys = 1;  // (one group: nothing to key)
  P.partial_pending = true;
  return PHIP_OK;
}

static int32_t finish_agg_partial(Plan &P, const phip_partial *merged, phip_result **out_result) {
  std::lock_guard<std::mutex> xlock(P.exec_mu);
  if (!P.partial_pending) return fail(PHIP_ERR_INVALID, "phip_plan_finish without a pending phip_plan_execute_partial");
  const int na = P.naggs;
  const size_t rows = (size_t)(1 + na);
  if (merged->table != P.ptab || merged->num_rows != (int32_t)rows || merged->num_groups != 1)
    return fail(PHIP_ERR_INVALID, "phip_plan_finish: partial does not belong to this plan");
  for (int a = 0; a < na; a++) {
    const int k = merged->row_kinds[1 + a], own = P.dq.aggs[a].acc;
    if (k != own && !(own == ACC_SUM_I64 && k == ACC_SUM_F64))
      return fail(PHIP_ERR_INVALID, "phip_plan_finish: row %d kind %d (plan: %d)", 1 + a, k, own);
  }
  const size_t hbytes = (size_t)P.nhll << (P.nhll ? P.log2m : 0);
  uint64_t *h = P.pstage;
  HIP_TRY(hipSetDevice(P.dev->ordinal));
  LaneGuard lg{P.dev};
  int32_t rc = acquire_lane(P.dev, &lg.lane);
  if (rc) return rc;
  hipStream_t st = lg.lane->stream;
  HIP_TRY(hipMemcpyAsync(h, P.ptab, (rows + 6) * 8, hipMemcpyDeviceToHost, st));
  if (hbytes) HIP_TRY(hipMemcpyAsync(h + rows + 6, P.phll, hbytes, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  lg.done = true;
  auto impl = std::make_unique<ResultImpl>();
  phip_result &r = impl->pub;
  memset(&r, 0, sizeof(r));
  const int64_t *st6 = merged->stats_dev ? (const int64_t *)(h + rows) : merged->stats;
  r.num_docs_scanned = st6[0];
  r.num_entries_scanned_in_filter = st6[1];
  r.num_entries_scanned_post_filter = st6[2];
  r.num_total_docs = st6[3];
  r.num_segments_processed = (int32_t)st6[4];
  r.num_segments_matched = (int32_t)st6[5];
  impl->values.resize(std::max(na, 1));
  impl->longs.resize(std::max(na, 1));
  impl->exact.resize(std::max(na, 1), 0);
  for (int a = 0; a < na; a++) {
    const int k = merged->row_kinds[1 + a];
    const uint64_t w = h[1 + a];
    double d = 0.0;
    int64_t l = 0;
    if (k == ACC_COUNT || k == ACC_SUM_I64) {
      l = (int64_t)w;
      d = (double)l;
    } else if (k == ACC_SUM_F64) {
      memcpy(&d, &w, 8);
    } else if (k == ACC_MIN_F64 || k == ACC_MAX_F64) {
      d = f64_unordered_host(w);
    }
    impl->values[a] = d;
    impl->longs[a] = l;
    impl->exact[a] = (k == ACC_COUNT || k == ACC_SUM_I64) ? 1 : 0;
  }
  impl->hll.assign((const uint8_t *)(h + rows + 6), (const uint8_t *)(h + rows + 6) + hbytes);
  impl->seg_docs.assign(1, 0);
  impl->prog_docs.assign(1, 0);
  r.program_docs_matched = impl->prog_docs.data();
  r.num_aggregations = na;
  r.num_groups = 1;
  r.num_hll = P.nhll;
  r.values = impl->values.data();
  r.long_values = impl->longs.data();
  r.hll_registers = impl->hll.data();
  r.group_keys = impl->keys.data();
  r.long_exact = impl->exact.data();
  r.segment_docs_matched = impl->seg_docs.data();
  r.scan_kernel_ms = P.part_times[0];  // (this GPU's execution of the partial)
  r.device_ms = P.part_times[1];
  r.filter_kernel_ms = P.part_times[2];
  r.agg_kernel_ms = P.part_times[3];
  r.fused = (int32_t)P.part_times[4];
  r.filter_bytes = P.part_bytes[0];
  r.agg_bytes = P.part_bytes[1];
  r.stream_bytes = P.part_bytes[2];
  P.partial_pending = false;
  *out_result = &impl.release()->pub;
  return PHIP_OK;
}

// ------------------------------------------------------------------------------------------------
// Hash-table growth (DictionaryBasedGroupKeyGenerator's holders grow with their maps,
// DictionaryBasedGroupKeyGenerator.java:150-185, instead of refusing). The open-addressing table is sized at plan
// creation to twice the groups possible, so a full table takes a capacity override (PHIP_GB_HASH_CAP) or a bound
// that did not hold; then the execution reports kGrowHash, the table is reallocated at twice the slots (new
// plan-owned buffers, the device descriptor updated) and the execution runs again -- every kernel from the filter on,
// the tables reset as on any execution. Up to kMaxHashGrowth doublings per execution.
// ------------------------------------------------------------------------------------------------
constexpr int kMaxHashGrowth = 8;

static int32_t grow_hash_table(Plan &P) {
  DevAggQuery &dq = P.dq;
  const int64_t cap = dq.num_groups * 2;
  const int64_t per_slot = 8 + 8 * (1 + (int64_t)P.naggs) + (int64_t)P.nhll * P.m_regs * 4 + (P.first_doc ? 4 : 0);
  if (cap * per_slot > ((int64_t)24 << 30))
    return fail(PHIP_ERR_UNSUPPORTED, "group-by hash table of %lld slots exceeds the memory budget", (long long)cap);
  HIP_TRY(hipSetDevice(P.dev->ordinal));
  void *tab = nullptr, *hll = nullptr, *hk = nullptr, *fd = nullptr;
  int32_t rc = P.alloc((size_t)(1 + P.naggs) * cap * 8, &tab);
  if (rc == PHIP_OK && P.nhll) rc = P.alloc((size_t)P.nhll * cap * P.m_regs * 4, &hll);
  if (rc == PHIP_OK) rc = P.alloc((size_t)cap * 8, &hk);
  if (rc == PHIP_OK && P.first_doc) rc = P.alloc((size_t)cap * 4, &fd);
  if (rc) return rc;
  P.gtab = tab;
  P.ghll = hll;
  dq.gb_table = (uint64_t *)tab;
  dq.gb_hll = (uint32_t *)hll;
  dq.gb_keys = (uint64_t *)hk;
  if (P.first_doc) {
    P.first_doc = (uint32_t *)fd;
    dq.first_doc = (uint32_t *)fd;
  }
  dq.num_groups = cap;
  HIP_TRY(hipMemcpy(P.base + P.dq_off, &dq, sizeof(DevAggQuery), hipMemcpyHostToDevice));
  return PHIP_OK;
}

static int32_t execute_growing(Plan &P, phip_result **out_result, uint64_t *filter_words) {
  for (int g = 0;; g++) {
    const int32_t rc = execute_plan(P, out_result, filter_words);
    if (rc != kGrowHash) return rc;
    if (g == kMaxHashGrowth)
      return fail(PHIP_ERR_UNSUPPORTED, "group-by hash table still full after %d doublings", kMaxHashGrowth);
    const int32_t grc = grow_hash_table(P);
    if (grc) return grc;
  }
}

// ================================================================================================
// C ABI
// ================================================================================================
extern "C" {

PHIP_API const char *phip_last_error(void) { return g_err.c_str(); }
PHIP_API const char *phip_version(void) { return "pinot_hip 0.1.0 gfx950"; }

PHIP_API int32_t phip_runtime_versions(int32_t *out_built, int32_t *out_runtime) {
  int rt = 0;
  if (hipRuntimeGetVersion(&rt) != hipSuccess) rt = 0;
  if (out_built) *out_built = HIP_VERSION;
  if (out_runtime) *out_runtime = rt;
  return PHIP_OK;
}

PHIP_API int32_t phip_device_count(int32_t *out_count) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  if (out_count) *out_count = n;
  return PHIP_OK;
}

PHIP_API int32_t phip_init(const int32_t *devices, int32_t num_devices) {
  std::lock_guard<std::mutex> g(g_mu);
  if (!g_devices.empty()) return PHIP_OK;
  if (!devices || num_devices <= 0) return ensure_devices_locked();
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(PHIP_ERR_NO_DEVICE, "no HIP device available");
  for (int i = 0; i < num_devices; i++) {
    if (devices[i] < 0 || devices[i] >= n) return fail(PHIP_ERR_INVALID, "device %d out of range", devices[i]);
    auto d = std::make_unique<Device>();
    d->ordinal = devices[i];
    HIP_TRY(hipSetDevice(d->ordinal));
    HIP_TRY(hipDeviceGetAttribute(&d->num_cus, hipDeviceAttributeMultiprocessorCount, d->ordinal));
    HIP_TRY(device_xcc_count(d->ordinal, &d->num_xcc));
    HIP_TRY(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
    for (auto &e : d->ev) HIP_TRY(hipEventCreate(&e));
    init_lanes(d.get());
    g_devices.push_back(std::move(d));
  }
  return PHIP_OK;
}

static std::unordered_map<uint64_t, std::unique_ptr<Plan>> g_plans;  // guarded by g_mu
static std::atomic<uint64_t> g_next_plan{1};

PHIP_API int32_t phip_shutdown(void) {
  node_shutdown();  // (its sub-plans and communicators first)
  std::lock_guard<std::mutex> g(g_mu);
  g_plans.clear();
  g_segments.clear();
  for (auto &d : g_devices) {
    std::lock_guard<std::mutex> dl(d->mu);
    (void)hipSetDevice(d->ordinal);
    d->ws.release();
    d->remaps.clear();
    for (auto &e : d->ev) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(d->stream);
    for (auto &l : d->lanes) {
      (void)hipStreamSynchronize(l->stream);
      l->ws.release();
      (void)hipStreamDestroy(l->stream);
    }
    d->lanes.clear();
    d->free_lanes.clear();
  }
  g_devices.clear();
  return PHIP_OK;
}

PHIP_API int32_t phip_segment_load(const phip_segment_desc *desc, uint64_t *out_handle) {
  if (!desc || !out_handle) return fail(PHIP_ERR_INVALID, "null argument");
  if (desc->num_docs < 0 || desc->num_columns < 0 || (desc->num_columns > 0 && !desc->columns))
    return fail(PHIP_ERR_INVALID, "bad segment descriptor");
  Device *dev;
  {
    std::lock_guard<std::mutex> g(g_mu);
    int32_t rc = ensure_devices_locked();
    if (rc) return rc;
    dev = desc->device >= 0 ? find_device(desc->device) : g_devices[0].get();
    if (!dev) return fail(PHIP_ERR_NO_DEVICE, "device %d not initialised (call phip_init)", desc->device);
  }
  std::lock_guard<std::mutex> dl(dev->mu);
  HIP_TRY(hipSetDevice(dev->ordinal));
  auto seg = std::make_shared<Segment>();
  seg->device = dev->ordinal;
  seg->num_docs = desc->num_docs;
  seg->name = desc->name ? desc->name : "";
  std::vector<void *> temps;
  int32_t rc = PHIP_OK;
  for (int c = 0; c < desc->num_columns && rc == PHIP_OK; c++) {
    if (desc->columns[c].name && seg->by_name.count(desc->columns[c].name)) {
      rc = fail(PHIP_ERR_INVALID, "duplicate column %s", desc->columns[c].name);
      break;
    }
    rc = load_column(desc->columns[c], *seg, dev->stream, temps);
  }
  hipError_t se = hipStreamSynchronize(dev->stream);
  for (void *p : temps) (void)hipFree(p);
  if (rc == PHIP_OK && se != hipSuccess) rc = fail(PHIP_ERR_HIP, "segment load: %s", hipGetErrorString(se));
  if (rc != PHIP_OK) return rc;  // the partial segment frees itself
  seg->handle = g_next_handle++;
  *out_handle = seg->handle;
  std::lock_guard<std::mutex> g(g_mu);
  g_segments[seg->handle] = std::move(seg);
  return PHIP_OK;
}

PHIP_API int32_t phip_segment_unload(uint64_t handle) {
  std::shared_ptr<Segment> seg;
  {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_segments.find(handle);
    if (it == g_segments.end()) return fail(PHIP_ERR_NOT_FOUND, "unknown segment handle %llu", (unsigned long long)handle);
    seg = std::move(it->second);
    g_segments.erase(it);
  }
  Device *dev = find_device(seg->device);
  if (dev) {
    std::lock_guard<std::mutex> dl(dev->mu);  // waits for in-flight queries on the device
    (void)hipSetDevice(dev->ordinal);
    (void)hipStreamSynchronize(dev->stream);
    for (auto it = dev->remaps.begin(); it != dev->remaps.end();) {
      if (it->first.find(":" + std::to_string(handle)) != std::string::npos) it = dev->remaps.erase(it);
      else ++it;
    }
    seg.reset();  // frees the HBM now unless a prepared plan still holds the segment
  }
  return PHIP_OK;
}

PHIP_API int32_t phip_segment_device_bytes(uint64_t handle, uint64_t *out_bytes) {
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_segments.find(handle);
  if (it == g_segments.end()) return fail(PHIP_ERR_NOT_FOUND, "unknown segment handle");
  if (out_bytes) *out_bytes = it->second->device_bytes;
  return PHIP_OK;
}

PHIP_API int32_t phip_query(const phip_query_desc *query, phip_result **out_result) {
  if (!out_result) return fail(PHIP_ERR_INVALID, "null result pointer");
  *out_result = nullptr;
  if (query && node_wanted(query)) {  // segments on several devices: a node plan, run once
    uint64_t h = 0;
    int32_t rc = node_create(query, &h);
    if (rc) return rc;
    rc = node_execute(h, out_result);
    (void)node_destroy(h);
    return rc;
  }
  Plan plan;
  int32_t rc = prepare_plan(query, false, 0, plan);
  if (rc) return rc;
  return execute_growing(plan, out_result, nullptr);
}

static int32_t create_single_plan(const phip_query_desc *query, uint64_t *out_plan);

PHIP_API int32_t phip_plan_create(const phip_query_desc *query, uint64_t *out_plan) {
  if (!out_plan) return fail(PHIP_ERR_INVALID, "null plan pointer");
  *out_plan = 0;
  if (query && node_wanted(query)) return node_create(query, out_plan);
  return create_single_plan(query, out_plan);
}

static int32_t create_single_plan(const phip_query_desc *query, uint64_t *out_plan) {
  *out_plan = 0;
  auto plan = std::make_unique<Plan>();
  int32_t rc = prepare_plan(query, false, 0, *plan);
  if (rc) return rc;
  const uint64_t h = g_next_plan++;
  std::lock_guard<std::mutex> g(g_mu);
  g_plans[h] = std::move(plan);
  *out_plan = h;
  return PHIP_OK;
}

PHIP_API int32_t phip_plan_execute(uint64_t plan, phip_result **out_result) {
  if (!out_result) return fail(PHIP_ERR_INVALID, "null result pointer");
  *out_result = nullptr;
  if (is_node_plan(plan)) return node_execute(plan, out_result);
  Plan *p;
  {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_plans.find(plan);
    if (it == g_plans.end()) return fail(PHIP_ERR_NOT_FOUND, "unknown plan handle %llu", (unsigned long long)plan);
    p = it->second.get();
  }
  return execute_growing(*p, out_result, nullptr);
}

static int32_t find_plan(uint64_t plan, Plan **out) {
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_plans.find(plan);
  if (it == g_plans.end()) return fail(PHIP_ERR_NOT_FOUND, "unknown plan handle %llu", (unsigned long long)plan);
  *out = it->second.get();
  return PHIP_OK;
}

PHIP_API int32_t phip_plan_set_deadline(uint64_t plan, int64_t deadline_ms) {
  if (is_node_plan(plan)) return node_set_deadline(plan, deadline_ms);
  Plan *p;
  int32_t rc = find_plan(plan, &p);
  if (rc) return rc;
  p->deadline_ms.store(deadline_ms > 0 ? deadline_ms : 0, std::memory_order_relaxed);
  return PHIP_OK;
}

PHIP_API int32_t phip_plan_cancel(uint64_t plan) {
  if (is_node_plan(plan)) return node_cancel(plan);
  Plan *p;
  int32_t rc = find_plan(plan, &p);
  if (rc) return rc;
  p->cancelled.store(1, std::memory_order_relaxed);
  return PHIP_OK;
}

PHIP_API int32_t phip_plan_execute_partial(uint64_t plan, phip_partial *out_partial) {
  if (!out_partial) return fail(PHIP_ERR_INVALID, "null partial pointer");
  if (is_node_plan(plan)) return fail(PHIP_ERR_INVALID, "a node plan merges its devices' partials itself");
  Plan *p;
  int32_t rc = find_plan(plan, &p);
  if (rc) return rc;
  if (!p->group_by) return execute_agg_partial(*p, out_partial);
  return execute_plan(*p, nullptr, nullptr, EXEC_PARTIAL, out_partial, nullptr);
}

PHIP_API int32_t phip_plan_finish(uint64_t plan, const phip_partial *merged, phip_result **out_result) {
  if (!merged || !out_result) return fail(PHIP_ERR_INVALID, "null argument");
  *out_result = nullptr;
  if (is_node_plan(plan)) return fail(PHIP_ERR_INVALID, "a node plan merges its devices' partials itself");
  Plan *p;
  int32_t rc = find_plan(plan, &p);
  if (rc) return rc;
  if (!p->group_by) return finish_agg_partial(*p, merged, out_result);
  return execute_plan(*p, out_result, nullptr, EXEC_FINISH, nullptr, merged);
}

PHIP_API int32_t phip_plan_abandon_partial(uint64_t plan) {
  if (is_node_plan(plan)) return fail(PHIP_ERR_INVALID, "a node plan merges its devices' partials itself");
  Plan *p;
  int32_t rc = find_plan(plan, &p);
  if (rc) return rc;
  std::lock_guard<std::mutex> xl(p->exec_mu);
  p->partial_pending = false;  // the next execution zeroes and rewrites the table
  return PHIP_OK;
}

PHIP_API int32_t phip_global_dictionary(int32_t device, const char *column, int32_t data_type, int32_t cardinality,
                                        int32_t string_width, const void *values) {
  if (!column || cardinality < -1 || (cardinality > 0 && !values))
    return fail(PHIP_ERR_INVALID, "global dictionary: bad arguments");
  if (cardinality == -1) {  // remove the registration
    std::lock_guard<std::mutex> g(g_mu);
    for (auto &d : g_devices) {
      if (device >= 0 && d->ordinal != device) continue;
      std::lock_guard<std::mutex> dl(d->mu);
      d->globals.erase(column);
    }
    return PHIP_OK;
  }
  if (data_type < PHIP_TYPE_INT || data_type > PHIP_TYPE_STRING)
    return fail(PHIP_ERR_INVALID, "global dictionary: bad data type %d", data_type);
  if (data_type == PHIP_TYPE_STRING && string_width <= 0)
    return fail(PHIP_ERR_INVALID, "global dictionary: string width must be > 0");
  const int w = data_type == PHIP_TYPE_STRING ? string_width : type_width(data_type);
  const uint8_t *v = (const uint8_t *)values;
  for (int32_t i = 1; i < cardinality; i++)
    if (compare_value(data_type, v + (size_t)(i - 1) * w, v + (size_t)i * w, w) >= 0)
      return fail(PHIP_ERR_INVALID, "global dictionary of %s: values not ascending / distinct at %d", column, i);
  Device *dev;
  {
    std::lock_guard<std::mutex> g(g_mu);
    int32_t rc = ensure_devices_locked();
    if (rc) return rc;
    dev = device >= 0 ? find_device(device) : g_devices[0].get();
    if (!dev) return fail(PHIP_ERR_NO_DEVICE, "device %d not initialised (call phip_init)", device);
  }
  std::lock_guard<std::mutex> dl(dev->mu);
  Device::GlobalDict &gd = dev->globals[column];
  gd.type = data_type;
  gd.card = cardinality;
  gd.width = data_type == PHIP_TYPE_STRING ? string_width : 0;
  gd.gen = ++dev->global_gen;
  gd.values.assign(v, v + (size_t)cardinality * w);
  return PHIP_OK;
}

PHIP_API int32_t phip_plan_exchange(uint64_t plan, int32_t *out_parts, int32_t *out_kind) {
  if (!out_parts || !out_kind) return fail(PHIP_ERR_INVALID, "null argument");
  if (is_node_plan(plan)) return node_exchange_info(plan, out_parts, out_kind);
  Plan *p;
  int32_t rc = find_plan(plan, &p);
  if (rc) return rc;
  *out_parts = 1;
  *out_kind = PHIP_EXCHANGE_NONE;
  return PHIP_OK;
}

PHIP_API int32_t phip_plan_destroy(uint64_t plan) {
  if (is_node_plan(plan)) return node_destroy(plan);
  std::unique_ptr<Plan> p;
  {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_plans.find(plan);
    if (it == g_plans.end()) return fail(PHIP_ERR_NOT_FOUND, "unknown plan handle %llu", (unsigned long long)plan);
    p = std::move(it->second);
    g_plans.erase(it);
  }
  if (p && p->dev) {
    std::lock_guard<std::mutex> xl(p->exec_mu);  // an execution on another thread finishes first
    (void)hipSetDevice(p->dev->ordinal);
  }
  return PHIP_OK;
}

PHIP_API int32_t phip_result_dictionary(const phip_result *result, int32_t k, phip_dictionary_view *out) {
  if (!result || !out) return fail(PHIP_ERR_INVALID, "null argument");
  const ResultImpl *impl = reinterpret_cast<const ResultImpl *>(result);
  if (k < 0 || k >= (int)impl->dicts.size()) return fail(PHIP_ERR_INVALID, "group-by index out of range");
  const auto &d = impl->dicts[k];
  out->data_type = d->type;
  out->cardinality = d->card;
  out->string_width = d->width;
  out->reserved = 0;
  out->values = d->values.data();
  return PHIP_OK;
}

PHIP_API int32_t phip_result_select_dictionary(const phip_result *result, int32_t k, phip_dictionary_view *out) {
  if (!result || !out) return fail(PHIP_ERR_INVALID, "null argument");
  const ResultImpl *impl = reinterpret_cast<const ResultImpl *>(result);
  if (k < 0 || k >= (int)impl->sel_dicts.size() || !impl->sel_dicts[k])
    return fail(PHIP_ERR_INVALID, "select column %d holds no dictionary ids", k);
  const auto &d = impl->sel_dicts[k];
  out->data_type = d->type;
  out->cardinality = d->card;
  out->string_width = d->width;
  out->reserved = 0;
  out->values = d->values.data();
  return PHIP_OK;
}

PHIP_API void phip_result_free(phip_result *result) {
  if (result) delete reinterpret_cast<ResultImpl *>(result);
}

PHIP_API int32_t phip_filter_bitmap(const phip_query_desc *query, uint64_t *words_out, int64_t num_words) {
  if (!query || !words_out || query->num_segments != 1) return fail(PHIP_ERR_INVALID, "filter bitmap: one segment");
  phip_query_desc q = *query;
  q.num_aggregations = 0;
  q.num_group_by = 0;
  q.num_select = 0;
  q.trim_size = 0;  // filter only: no groups to trim
  q.num_order_by_keys = 0;
  phip_result *r = nullptr;
  int32_t rc;
  {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_segments.find(query->segments[0]);
    if (it == g_segments.end()) return fail(PHIP_ERR_NOT_FOUND, "unknown segment handle");
    if (num_words < ceil_div(it->second->num_docs, 64)) return fail(PHIP_ERR_INVALID, "words_out too small");
  }
  Plan plan;
  rc = prepare_plan(&q, true, num_words, plan);
  if (rc) return rc;
  rc = execute_plan(plan, &r, words_out);
  if (r) phip_result_free(r);
  return rc;
}

}  // extern "C"

// ------------------------------------------------------------------------------------------------
// Node plans (node.cpp): hooks over the single-device machinery above
// ------------------------------------------------------------------------------------------------

int32_t phip::node_fail(int32_t code, const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

int32_t phip::node_segment_device(uint64_t handle, int *ordinal, int64_t *docs) {
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_segments.find(handle);
  if (it == g_segments.end()) return fail(PHIP_ERR_NOT_FOUND, "unknown segment handle %llu", (unsigned long long)handle);
  *ordinal = it->second->device;
  if (docs) *docs = it->second->num_docs;
  return PHIP_OK;
}

int32_t phip::node_union_dictionary(const std::vector<uint64_t> &handles, const std::string &column, NodeDict *out,
                                    bool *ok) {
  *ok = false;
  std::vector<std::shared_ptr<Segment>> segs;
  {
    std::lock_guard<std::mutex> g(g_mu);
    for (uint64_t h : handles) {
      auto it = g_segments.find(h);
      if (it == g_segments.end()) return fail(PHIP_ERR_NOT_FOUND, "unknown segment handle %llu", (unsigned long long)h);
      segs.push_back(it->second);
    }
  }
  int32_t type = -1, width = 0;
  std::vector<const ColumnStore *> cols;
  for (auto &sp : segs) {
    auto ci = sp->by_name.find(column);
    if (ci == sp->by_name.end()) return PHIP_OK;  // (prepare_plan reports the missing column)
    const ColumnStore &c = sp->cols[ci->second];
    if (no_dict(c) || (type >= 0 && c.type != type)) return PHIP_OK;  // raw keys / mixed types: the record path
    type = c.type;
    width = std::max(width, type == PHIP_TYPE_STRING ? c.string_width : type_width(type));
    cols.push_back(&c);
  }
  if (type < 0) return PHIP_OK;
  // every segment's values in the comparable form (LE numbers, '\0'-padded strings), sorted, distinct (build_remap's)
  std::vector<uint8_t> all;
  for (const ColumnStore *c : cols) {
    const int sw = type == PHIP_TYPE_STRING ? c->string_width : width;
    for (int32_t id = 0; id < c->card; id++) {
      const size_t at = all.size();
      all.resize(at + width, 0);
      const uint8_t *p = c->host_dict.data() + (size_t)id * sw;
      if (type == PHIP_TYPE_STRING) memcpy(all.data() + at, p, sw);
      else
        for (int b = 0; b < width; b++) all[at + b] = p[width - 1 - b];
    }
  }
  const int64_t total = width ? (int64_t)(all.size() / width) : 0;
  std::vector<int64_t> order(total);
  for (int64_t i = 0; i < total; i++) order[i] = i;
  const uint8_t *A = all.data();
  std::stable_sort(order.begin(), order.end(),
                   [&](int64_t x, int64_t y) { return compare_value(type, A + x * width, A + y * width, width) < 0; });
  out->values.clear();
  int64_t n = 0;
  for (int64_t k = 0; k < total; k++) {
    const uint8_t *v = A + order[k] * width;
    if (n > 0 && compare_value(type, out->values.data() + (n - 1) * width, v, width) == 0) continue;
    out->values.insert(out->values.end(), v, v + width);
    n++;
  }
  if (n > INT32_MAX) return PHIP_OK;
  out->type = type;
  out->card = (int32_t)n;
  out->width = type == PHIP_TYPE_STRING ? width : 0;
  *ok = true;
  return PHIP_OK;
}

int32_t phip::node_plan_create(const phip_query_desc *q, const NodeDicts *dicts, int64_t node_docs, uint64_t *out_plan) {
  tl_node_dicts = dicts;
  tl_node_docs = std::max<int64_t>(node_docs, 1);
  const int32_t rc = create_single_plan(q, out_plan);
  tl_node_dicts = nullptr;
  tl_node_docs = 0;
  return rc;
}

int32_t phip::node_plan_group_info(uint64_t plan, NodeGroupInfo *out) {
  Plan *p;
  int32_t rc = find_plan(plan, &p);
  if (rc) return rc;
  out->hash = p->group_by && p->dq.mode == GB_HASH;
  out->tuple = p->tuple_keys;
  out->radix = p->tuple_keys ? p->tuple_radix : p->gb_radix;
  out->keys = out->hash ? p->dq.gb_keys : nullptr;
  return PHIP_OK;
}

int32_t phip::node_plan_docs(uint64_t plan, std::vector<int64_t> *seg_docs, std::vector<int64_t> *prog_docs) {
  Plan *p;
  int32_t rc = find_plan(plan, &p);
  if (rc) return rc;
  const int nseg = p->nseg;
  const uint64_t *segm = p->pinned + 64;
  seg_docs->assign(std::max(nseg, 1), 0);
  prog_docs->assign(std::max(p->nprog, 1), 0);
  for (int pr = 0; pr < p->nprog; pr++)
    for (int s = 0; s < nseg; s++) {
      const int64_t d = p->has_filter ? (int64_t)segm[pr * nseg + s] : p->slot_docs[pr * nseg + s];
      (*seg_docs)[s] += d;
      (*prog_docs)[pr] += d;
    }
  return PHIP_OK;
}

int32_t phip::node_make_result(NodeResultData &&d, phip_result **out) {
  auto impl = std::make_unique<ResultImpl>();
  phip_result &r = impl->pub;
  memset(&r, 0, sizeof(r));
  r.num_docs_scanned = d.stats[0];
  r.num_entries_scanned_in_filter = d.stats[1];
  r.num_entries_scanned_post_filter = d.stats[2];
  r.num_total_docs = d.stats[3];
  r.num_segments_processed = (int32_t)d.stats[4];
  r.num_segments_matched = (int32_t)d.stats[5];
  r.num_groups_limit_reached = d.limit_reached;
  r.num_aggregations = d.naggs;
  r.num_groups = d.ngroups;
  r.num_group_by = d.ngb;
  r.num_hll = d.nhll;
  impl->values = std::move(d.values);
  impl->longs = std::move(d.longs);
  impl->exact = std::move(d.exact);
  impl->hll = std::move(d.hll);
  impl->keys = std::move(d.keys);
  impl->seg_docs = std::move(d.seg_docs);
  impl->prog_docs = std::move(d.prog_docs);
  if (impl->values.empty()) impl->values.resize(1);
  if (impl->longs.empty()) impl->longs.resize(1);
  if (impl->exact.empty()) impl->exact.resize(1);
  if (impl->seg_docs.empty()) impl->seg_docs.resize(1);
  if (impl->prog_docs.empty()) impl->prog_docs.resize(1);
  for (auto &nd : d.dicts) {
    auto rm = std::make_shared<Device::Remap>();
    rm->type = nd.type;
    rm->card = nd.card;
    rm->width = nd.width;
    rm->values = std::move(nd.values);
    impl->dicts.push_back(rm);
  }
  r.values = impl->values.data();
  r.long_values = impl->longs.data();
  r.long_exact = impl->exact.data();
  r.hll_registers = impl->hll.data();
  r.group_keys = impl->keys.data();
  r.segment_docs_matched = impl->seg_docs.data();
  r.program_docs_matched = impl->prog_docs.data();
  r.scan_kernel_ms = d.scan_ms;
  r.device_ms = d.device_ms;
  r.filter_kernel_ms = d.filter_ms;
  r.agg_kernel_ms = d.agg_ms;
  r.filter_bytes = d.filter_bytes;
  r.agg_bytes = d.agg_bytes;
  r.stream_bytes = d.stream_bytes;
  r.fused = d.fused;
  *out = &impl.release()->pub;
  return PHIP_OK;
}

void phip::node_result_set_docs(phip_result *res, std::vector<int64_t> seg_docs, std::vector<int64_t> prog_docs) {
  ResultImpl *impl = reinterpret_cast<ResultImpl *>(res);
  impl->seg_docs = std::move(seg_docs);
  impl->prog_docs = std::move(prog_docs);
  if (impl->seg_docs.empty()) impl->seg_docs.resize(1);
  if (impl->prog_docs.empty()) impl->prog_docs.resize(1);
  impl->pub.segment_docs_matched = impl->seg_docs.data();
  impl->pub.program_docs_matched = impl->prog_docs.data();
}

int phip::node_compare_value(int32_t type, const uint8_t *a, const uint8_t *b, int width) {
  return compare_value(type, a, b, width);
}
int phip::node_type_width(int32_t type) { return type_width(type); }
