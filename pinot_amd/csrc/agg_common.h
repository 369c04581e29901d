// agg_common.h -- projection / expression / accumulation helpers shared by the aggregation kernel
// (aggregate.hip) and the fused filter+aggregation path of the filter kernel (filter.hip).
#pragma once
#include "dev_common.h"

namespace phip {

// The launch descriptor lives in device memory and is read through the constant address space
// (scalar loads), so no per-lane copy of it is ever made.
typedef const PHIP_CAS DevAggQuery cquery_t;
typedef const PHIP_CAS DevAgg cagg_t;

__device__ __forceinline__ int64_t dict_i64(ccol_t &c, uint32_t id) {
  switch (c.type) {
    case PHIP_TYPE_INT: return ((const PHIP_GLB int32_t *)c.dict)[id];
    case PHIP_TYPE_LONG: return ((const PHIP_GLB int64_t *)c.dict)[id];
    case PHIP_TYPE_FLOAT: return (int64_t)((const PHIP_GLB float *)c.dict)[id];
    default: return (int64_t)((const PHIP_GLB double *)c.dict)[id];
  }
}
__device__ __forceinline__ double dict_f64(ccol_t &c, uint32_t id) {
  switch (c.type) {
    case PHIP_TYPE_INT: return (double)((const PHIP_GLB int32_t *)c.dict)[id];
    case PHIP_TYPE_LONG: return (double)((const PHIP_GLB int64_t *)c.dict)[id];
    case PHIP_TYPE_FLOAT: return (double)((const PHIP_GLB float *)c.dict)[id];
    default: return ((const PHIP_GLB double *)c.dict)[id];
  }
}
// doc-order values bit-packed at the column's range width (DevCol.vpack): one window load, like a dictionary id
__device__ __forceinline__ int64_t packed_i64(ccol_t &c, int32_t doc) {
  return c.vbase + (int64_t)decode_bits(c.vpack, (uint64_t)(uint32_t)doc * (uint32_t)c.vbits, (uint32_t)c.vbits);
}
__device__ __forceinline__ int64_t raw_i64(ccol_t &c, int32_t doc) {
  if (c.vpack != nullptr) return packed_i64(c, doc);
  switch (c.type) {
    case PHIP_TYPE_INT: return ((const PHIP_GLB int32_t *)c.raw)[doc];
    case PHIP_TYPE_LONG: return ((const PHIP_GLB int64_t *)c.raw)[doc];
    case PHIP_TYPE_FLOAT: return (int64_t)((const PHIP_GLB float *)c.raw)[doc];
    default: return (int64_t)((const PHIP_GLB double *)c.raw)[doc];
  }
}
__device__ __forceinline__ double raw_f64(ccol_t &c, int32_t doc) {
  if (c.vpack != nullptr) return (double)packed_i64(c, doc);
  switch (c.type) {
    case PHIP_TYPE_INT: return (double)((const PHIP_GLB int32_t *)c.raw)[doc];
    case PHIP_TYPE_LONG: return (double)((const PHIP_GLB int64_t *)c.raw)[doc];
    case PHIP_TYPE_FLOAT: return (double)((const PHIP_GLB float *)c.raw)[doc];
    default: return ((const PHIP_GLB double *)c.raw)[doc];
  }
}

__device__ __forceinline__ uint32_t col_dict_id(ccol_t &c, int32_t doc) {
  return decode_bits(c.words, (uint64_t)(uint32_t)doc * (uint32_t)c.bits, (uint32_t)c.bits);
}
__device__ __forceinline__ int64_t col_i64(ccol_t &c, int32_t doc) {
  if (c.has_dict) return dict_i64(c, col_dict_id(c, doc));
  return raw_i64(c, doc);
}
__device__ __forceinline__ double col_f64(ccol_t &c, int32_t doc) {
  if (c.has_dict) return dict_f64(c, col_dict_id(c, doc));
  return raw_f64(c, doc);
}
__device__ __forceinline__ int64_t expr_i64(cseg_t &s, cagg_t &a, int32_t doc) {
  int64_t x = col_i64(s.cols[a.col_a], doc);
  if (a.expr == PHIP_EXPR_COLUMN) return x;
  int64_t y = col_i64(s.cols[a.col_b], doc);
  if (a.expr == PHIP_EXPR_ADD) return x + y;
  if (a.expr == PHIP_EXPR_SUB) return x - y;
  return x * y;
}
__device__ __forceinline__ double expr_f64(cseg_t &s, cagg_t &a, int32_t doc) {
  double x = col_f64(s.cols[a.col_a], doc);
  if (a.expr == PHIP_EXPR_COLUMN) return x;
  double y = col_f64(s.cols[a.col_b], doc);
  if (a.expr == PHIP_EXPR_ADD) return x + y;
  if (a.expr == PHIP_EXPR_SUB) return x - y;
  return x * y;
}

// Typed atomics: LDS tables use ds_* atomics, HBM tables global_* atomics (no flat_* forms).
#define PHIP_RLX __ATOMIC_RELAXED
#define PHIP_WG __HIP_MEMORY_SCOPE_WORKGROUP
#define PHIP_AG __HIP_MEMORY_SCOPE_AGENT
typedef PHIP_LDS uint64_t lds_u64;
typedef PHIP_LDS uint32_t lds_u32;
typedef PHIP_GLB uint64_t glb_u64;
typedef PHIP_GLB uint32_t glb_u32;

// Packed u8 HLL register max in LDS (4 registers per u32 word; no byte max exists in the DS ISA).
__device__ __forceinline__ void lds_hll_max(lds_u32 *words, uint32_t reg, uint32_t rho) {
  lds_u32 *w = words + (reg >> 2);
  const uint32_t sh = (reg & 3) * 8;
  uint32_t old = *w;
  while (((old >> sh) & 0xffu) < rho) {
    const uint32_t want = (old & ~(0xffu << sh)) | (rho << sh);
    if (__hip_atomic_compare_exchange_strong(w, &old, want, PHIP_RLX, PHIP_RLX, PHIP_WG)) break;
  }
}

// HLL register rows (a star-tree DISTINCTCOUNTHLL pair, DevCol.hll_rows): the doc's 2^hll_rows registers, each
// nonzero one handed to f(register, rho) -- the register-wise max merge of HyperLogLog.merge.
template <typename F>
__device__ __forceinline__ void hll_row_each(ccol_t &c, int32_t doc, F &&f) {
  const int words = (1 << c.hll_rows) >> 2;
  const PHIP_GLB uint32_t *row = (const PHIP_GLB uint32_t *)c.raw + (int64_t)doc * words;
  for (int w = 0; w < words; w++) {
    const uint32_t x = row[w];
    if (!x) continue;
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const uint32_t rho = (x >> (8 * b)) & 0xffu;
      if (rho) f(4 * w + b, rho);
    }
  }
}

// HyperLogLog entry ((register << 8) | rho) of a raw numeric column's value at doc: clearspring MurmurHash.hashLong of
// the value as DistinctCountHLLAggregationFunction offers raw values (java.lang.Integer / Long widened, FLOAT / DOUBLE
// by their bits -- the same mapping ensure_hll applies to dictionary values).
__device__ __forceinline__ int32_t murmur_hash_long_dev(int64_t data) {
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
// clearspring MurmurHash.hash(byte[]) with seed -1, as HyperLogLog.offer hashes a String's bytes (the same function
// ensure_hll applies to STRING dictionary entries): a raw STRING doc's UTF-8 bytes, read a byte at a time (unaligned)
__device__ __forceinline__ uint32_t murmur_hash_bytes_dev(const PHIP_GLB uint8_t *d, int32_t len) {
  const uint32_t m = 0x5bd1e995u;
  uint32_t h = 0xffffffffu ^ (uint32_t)len;
  const int32_t n4 = len >> 2;
  for (int32_t i = 0; i < n4; i++) {
    uint32_t k = (uint32_t)d[4 * i] | ((uint32_t)d[4 * i + 1] << 8) | ((uint32_t)d[4 * i + 2] << 16) |
                 ((uint32_t)d[4 * i + 3] << 24);
    k *= m;
    k ^= k >> 24;
    k *= m;
    h *= m;
    h ^= k;
  }
  const int32_t left = len - (n4 << 2);
  if (left) {  // (Java bytes are signed: each tail byte sign-extends)
    if (left >= 3) h ^= (uint32_t)((int32_t)(int8_t)d[len - 3] << 16);
    if (left >= 2) h ^= (uint32_t)((int32_t)(int8_t)d[len - 2] << 8);
    h ^= (uint32_t)(int32_t)(int8_t)d[len - 1];
    h *= m;
  }
  h ^= h >> 13;
  h *= m;
  h ^= h >> 15;
  return h;
}
__device__ __forceinline__ uint32_t hll_entry_hash(uint32_t ux, int log2m) {
  const uint32_t j = ux >> (32 - log2m);
  const uint32_t w = (ux << log2m) | ((1u << (log2m - 1)) + 1u);
  return (j << 8) | ((uint32_t)__builtin_clz(w) + 1u);
}
__device__ __forceinline__ uint32_t hll_entry_bits(int64_t x, int log2m) {
  return hll_entry_hash((uint32_t)murmur_hash_long_dev(x), log2m);
}
__device__ __forceinline__ uint32_t hll_entry_raw(ccol_t &c, int32_t doc, int log2m) {
  int64_t x;
  switch (c.type) {
    case PHIP_TYPE_STRING: {
      const uint64_t b = c.str_off[doc], e = c.str_off[doc + 1];
      return hll_entry_hash(murmur_hash_bytes_dev((const PHIP_GLB uint8_t *)c.raw + b, (int32_t)(e - b)), log2m);
    }
    case PHIP_TYPE_INT: x = ((const PHIP_GLB int32_t *)c.raw)[doc]; break;
    case PHIP_TYPE_LONG: x = ((const PHIP_GLB int64_t *)c.raw)[doc]; break;
    case PHIP_TYPE_FLOAT: x = ((const PHIP_GLB int32_t *)c.raw)[doc]; break;
    default: x = ((const PHIP_GLB int64_t *)c.raw)[doc]; break;
  }
  return hll_entry_bits(x, log2m);
}
// a doc-order entry as (register << 8) | rho: the 32-bit copy, or the 16-bit one unpacked
__device__ __forceinline__ uint32_t hll_doc_entry(ccol_t &c, int32_t doc) {
  if (c.hll_doc16 != nullptr) {
    const uint32_t e = ((const PHIP_GLB uint16_t *)c.hll_doc16)[doc];
    return ((e >> 5) << 8) | (e & 31u);
  }
  return ((const PHIP_GLB uint32_t *)c.hll_doc)[doc];
}
// the entry of doc's value in column c: the per-dictionary-id table, or hashed from the raw value
__device__ __forceinline__ uint32_t hll_entry(ccol_t &c, int32_t doc, int log2m) {
  if (c.hll_doc != nullptr || c.hll_doc16 != nullptr) return hll_doc_entry(c, doc);
  if (!c.has_dict) return hll_entry_raw(c, doc, log2m);
  return ((const PHIP_GLB uint32_t *)c.hll)[col_dict_id(c, doc)];
}
// a DISTINCTCOUNTHLL's entry at doc: of its column, or of its expression's double value (hashLong of the bits: the
// reference offers a transform function's DOUBLE result as java.lang.Double)
__device__ __forceinline__ uint32_t hll_entry_agg(cseg_t &seg, cagg_t &ag, int32_t doc) {
  if (ag.expr != PHIP_EXPR_COLUMN) return hll_entry_bits(__double_as_longlong(expr_f64(seg, ag, doc)), ag.log2m);
  return hll_entry(seg.cols[ag.col_a], doc, ag.log2m);
}

// ------------------------------------------------------------------------------------------------
// per-chunk work: 64 lanes = up to 64 matched docs of one segment (inactive lanes carry doc 0, a valid
// doc, so every load stays in bounds, and contribute the identity)
// ------------------------------------------------------------------------------------------------
template <int NA>
__device__ __forceinline__ void agg_chunk(cquery_t &q, cseg_t &seg, int32_t doc, bool act,
                                          uint64_t (&acc)[NA], lds_u32 *hll_lds) {
#pragma unroll
  for (int a = 0; a < NA; a++) {
    if (a >= q.num_aggs) break;
    cagg_t &ag = q.aggs[a];
    if (ag.program != seg.program) continue;  // another filter program's function (wave-uniform)
    const int kind = ag.acc;
    if (kind == ACC_COUNT) {
      acc[a] += act ? 1ull : 0ull;
    } else if (kind == ACC_SUM_I64) {
      const int64_t v = expr_i64(seg, ag, doc);
      acc[a] += act ? (uint64_t)v : 0ull;
    } else if (kind == ACC_HLL) {
      ccol_t &c = seg.cols[ag.col_a];
      lds_u32 *regs = hll_lds + (ag.hll_slot << q.log2m);
      if (c.hll_rows) {
        if (act) hll_row_each(c, doc, [&](int r, uint32_t rho) { __hip_atomic_fetch_max(&regs[r], rho, PHIP_RLX, PHIP_WG); });
      } else {
        const uint32_t h = hll_entry_agg(seg, ag, doc);
        if (act) __hip_atomic_fetch_max(&regs[h >> 8], h & 0xffu, PHIP_RLX, PHIP_WG);
      }
    } else {
      const double v = expr_f64(seg, ag, doc);
      const double cur = as_f64(acc[a]);
      double nv;
      if (kind == ACC_SUM_F64) nv = cur + (act ? v : 0.0);
      else if (kind == ACC_MIN_F64) nv = fmin(cur, act ? v : __builtin_huge_val());
      else nv = fmax(cur, act ? v : -__builtin_huge_val());
      acc[a] = as_u64(nv);
    }
  }
}

// Dense group key of one doc: mixed radix over query-global dict ids, column 0 least significant
// (DictionaryBasedGroupKeyGenerator.java:314,322,345,442); a raw INT / LONG column contributes value - gb_base.
__device__ __forceinline__ int64_t group_key(cquery_t &q, cseg_t &seg, int32_t doc) {
  int64_t key = 0;
  for (int k = 0; k < q.num_group_by; k++) {
    ccol_t &c = seg.cols[q.gb_cols[k]];
    int64_t gid;
    if (c.gb_ids != nullptr) {
      gid = c.gb_ids[doc];
    } else if (!c.has_dict) {
      gid = raw_i64(c, doc) - c.gb_base;
    } else {
      const uint32_t id = col_dict_id(c, doc);
      gid = c.remap ? ((const PHIP_GLB int32_t *)c.remap)[id] : (int32_t)id;
    }
    if (c.gb_nulls != nullptr && ((c.gb_nulls[doc >> 6] >> (doc & 63)) & 1ull)) gid = c.gb_null_id;  // the null key
    key += gid * q.gb_stride[k];
  }
  return key;
}


// GB_LDS: table rows in LDS (row 0 counts, row 1+a aggregation a), packed HLL registers in LDS.
__device__ __forceinline__ void group_chunk_lds(cquery_t &q, cseg_t &seg, int32_t doc, bool act, lds_u64 *tbl,
                                                lds_u32 *hll_packed) {
  const int64_t key = group_key(q, seg, doc);
  if (!act) return;
  const int32_t G = (int32_t)q.num_groups;
  __hip_atomic_fetch_add(&tbl[key], 1ull, PHIP_RLX, PHIP_WG);
  for (int a = 0; a < kMaxAggs; a++) {
    if (a >= q.num_aggs) break;
    cagg_t &ag = q.aggs[a];
    if (ag.program != seg.program) continue;  // another filter program's function (wave-uniform)
    lds_u64 *slot = tbl + (1 + a) * G + key;
    switch (ag.acc) {
      case ACC_COUNT:  // == row 0, unless the programs count apart
        if (q.own_count_rows) __hip_atomic_fetch_add(slot, 1ull, PHIP_RLX, PHIP_WG);
        break;
      case ACC_SUM_I64: __hip_atomic_fetch_add(slot, (uint64_t)expr_i64(seg, ag, doc), PHIP_RLX, PHIP_WG); break;
      case ACC_SUM_F64:
        __hip_atomic_fetch_add((PHIP_LDS double *)slot, expr_f64(seg, ag, doc), PHIP_RLX, PHIP_WG);
        break;
      case ACC_MIN_F64: __hip_atomic_fetch_min(slot, f64_ordered(expr_f64(seg, ag, doc)), PHIP_RLX, PHIP_WG); break;
      case ACC_MAX_F64: __hip_atomic_fetch_max(slot, f64_ordered(expr_f64(seg, ag, doc)), PHIP_RLX, PHIP_WG); break;
      case ACC_HLL: {
        ccol_t &c = seg.cols[ag.col_a];
        lds_u32 *regs = hll_packed + ((((int64_t)ag.hll_slot * G + key) << q.log2m) >> 2);
        if (c.hll_rows) {
          hll_row_each(c, doc, [&](int r, uint32_t rho) { lds_hll_max(regs, (uint32_t)r, rho); });
        } else {
          const uint32_t h = hll_entry_agg(seg, ag, doc);
          lds_hll_max(regs, h >> 8, h & 0xffu);
        }
        break;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// dense tiles (aggregation only): kBatch groups of 64 docs at a time in the mask's lane-major order
// (doc 64g + lane), every load of the batch issued before the first use, so a dense tile costs a few
// memory round trips instead of one per 64 matched docs. Lanes whose doc did not match load the
// tile's first doc (always valid) and contribute the identity.
// ------------------------------------------------------------------------------------------------
#ifndef PHIP_KBATCH
#define PHIP_KBATCH 4  // (A/B builds override it)
#endif
constexpr int kBatch = PHIP_KBATCH;

template <int U>
__device__ __forceinline__ void batch_docs(int32_t doc, uint32_t act, int32_t safe, int32_t (&d)[U]) {
#pragma unroll
  for (int u = 0; u < U; u++) d[u] = ((act >> u) & 1u) ? doc + 64 * u : safe;
}

// Dict ids of the batch: from the wave's LDS stage (sw != null; td = tile-relative doc of group g0,
// bit window at td * b, ids of non-matching docs forced to 0) or straight from HBM.
struct BatchSrc {
  const PHIP_LDS uint32_t *sw;
  int32_t td;
  uint32_t act;
  const PHIP_LDS unsigned char *dict;  // the segment's dictionary copied into LDS (small ones), or null
};

template <int U>
__device__ __forceinline__ void batch_ids(ccol_t &c, const int32_t (&d)[U], const BatchSrc &bs, uint32_t (&id)[U]) {
  const uint32_t b = (uint32_t)c.bits;
  if (bs.sw != nullptr) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t v = window_at(bs.sw, (bs.td + 64 * u) * (int32_t)b) >> (32 - b);
      id[u] = ((bs.act >> u) & 1u) ? v : 0u;
    }
  } else {
#pragma unroll
    for (int u = 0; u < U; u++) id[u] = decode_bits(c.words, (uint64_t)(uint32_t)d[u] * b, b);
  }
}

template <int U>
__device__ __forceinline__ void batch_i64(ccol_t &c, const int32_t (&d)[U], const BatchSrc &bs, int64_t (&v)[U]) {
  if (c.has_dict) {
    uint32_t id[U];
    batch_ids<U>(c, d, bs, id);
    if (bs.dict != nullptr) {
      if (c.type == PHIP_TYPE_INT) {
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = ((const PHIP_LDS int32_t *)bs.dict)[id[u]];
      } else if (c.type == PHIP_TYPE_LONG) {
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = ((const PHIP_LDS int64_t *)bs.dict)[id[u]];
      } else if (c.type == PHIP_TYPE_FLOAT) {
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = (int64_t)((const PHIP_LDS float *)bs.dict)[id[u]];
      } else {
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = (int64_t)((const PHIP_LDS double *)bs.dict)[id[u]];
      }
      return;
    }
    switch (c.type) {
      case PHIP_TYPE_INT:
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = ((const PHIP_GLB int32_t *)c.dict)[id[u]];
        break;
      case PHIP_TYPE_LONG:
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = ((const PHIP_GLB int64_t *)c.dict)[id[u]];
        break;
      default:
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = dict_i64(c, id[u]);
        break;
    }
  } else if (c.vpack != nullptr) {
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = packed_i64(c, d[u]);
  } else {
    switch (c.type) {
      case PHIP_TYPE_INT:
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = ((const PHIP_GLB int32_t *)c.raw)[d[u]];
        break;
      case PHIP_TYPE_LONG:
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = ((const PHIP_GLB int64_t *)c.raw)[d[u]];
        break;
      default:
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = raw_i64(c, d[u]);
        break;
    }
  }
}

template <int U>
__device__ __forceinline__ void batch_f64(ccol_t &c, const int32_t (&d)[U], const BatchSrc &bs, double (&v)[U]) {
  if (c.has_dict) {
    uint32_t id[U];
    batch_ids<U>(c, d, bs, id);
    if (bs.dict != nullptr) {
      if (c.type == PHIP_TYPE_INT) {
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = (double)((const PHIP_LDS int32_t *)bs.dict)[id[u]];
      } else if (c.type == PHIP_TYPE_LONG) {
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = (double)((const PHIP_LDS int64_t *)bs.dict)[id[u]];
      } else if (c.type == PHIP_TYPE_FLOAT) {
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = (double)((const PHIP_LDS float *)bs.dict)[id[u]];
      } else {
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = ((const PHIP_LDS double *)bs.dict)[id[u]];
      }
      return;
    }
    switch (c.type) {
      case PHIP_TYPE_INT:
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = (double)((const PHIP_GLB int32_t *)c.dict)[id[u]];
        break;
      case PHIP_TYPE_DOUBLE:
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = ((const PHIP_GLB double *)c.dict)[id[u]];
        break;
      default:
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = dict_f64(c, id[u]);
        break;
    }
  } else {
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = raw_f64(c, d[u]);
  }
}

// Same arithmetic as expr_i64 / expr_f64, U docs at a time.
template <int U>
__device__ __forceinline__ void batch_expr_i64(cseg_t &s, cagg_t &a, const int32_t (&d)[U], const BatchSrc &sa,
                                               const BatchSrc &sb, int64_t (&x)[U]) {
  batch_i64<U>(s.cols[a.col_a], d, sa, x);
  if (a.expr == PHIP_EXPR_COLUMN) return;
  int64_t y[U];
  batch_i64<U>(s.cols[a.col_b], d, sb, y);
#pragma unroll
  for (int u = 0; u < U; u++) {
    if (a.expr == PHIP_EXPR_ADD) x[u] = x[u] + y[u];
    else if (a.expr == PHIP_EXPR_SUB) x[u] = x[u] - y[u];
    else x[u] = x[u] * y[u];
  }
}
template <int U>
__device__ __forceinline__ void batch_expr_f64(cseg_t &s, cagg_t &a, const int32_t (&d)[U], const BatchSrc &sa,
                                               const BatchSrc &sb, double (&x)[U]) {
  batch_f64<U>(s.cols[a.col_a], d, sa, x);
  if (a.expr == PHIP_EXPR_COLUMN) return;
  double y[U];
  batch_f64<U>(s.cols[a.col_b], d, sb, y);
#pragma unroll
  for (int u = 0; u < U; u++) {
    if (a.expr == PHIP_EXPR_ADD) x[u] = x[u] + y[u];
    else if (a.expr == PHIP_EXPR_SUB) x[u] = x[u] - y[u];
    else x[u] = x[u] * y[u];
  }
}

// ------------------------------------------------------------------------------------------------
// finalize in the last workgroup (DevFinal). Every partial a workgroup hands on -- its per-block slots (atomic stores
// at agent scope) and the per-segment counts / HLL registers (agent-scope atomics) -- is performed at the device
// coherence point, not only in the XCD's own L2. Each wave waits for its vector memory operations to be acknowledged
// (s_waitcnt vmcnt(0)), the workgroup synchronises, and its first thread takes a ticket; the workgroup holding the
// last ticket reads every partial with agent-scope atomic loads and runs finalize_all_kernel's work -- one wave per
// slot, lane-strided over the blocks in a fixed order and a fixed shuffle tree (bitwise reproducible) -- then copies
// and zeroes the per-segment counts and the registers. No release fence is needed: a fence at agent scope writes back
// the whole L2 of the XCD (buffer_wbl2), which made this 3.3x slower than the separate launch (round 3).
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void coherent_store(uint64_t *p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t coherent_load(const uint64_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t coherent_load(const uint32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int kFinLoads = 8;  // blocks per lane whose partials are loaded in one round trip (64 x 32 = 2048 blocks)
__device__ __forceinline__ void fin_slot(const uint64_t *partials, int nblocks, int nslots, int kind, uint64_t *out,
                                         int a) {
  const int lane = lane_id();
  const bool fp = kind == ACC_SUM_F64 || kind == ACC_MIN_F64 || kind == ACC_MAX_F64;
  uint64_t v = fp ? acc_init(kind) : 0;
  // every load of the lane issued before the first combine (coherent loads reach the device coherence point: one
  // dependent round trip per block would cost ~20 of them)
  for (int b0 = 0; b0 < nblocks; b0 += 64 * kFinLoads) {  // (1280 blocks: 3 round trips, not 13)
    uint64_t w[kFinLoads];
#pragma unroll
    for (int i = 0; i < kFinLoads; i++) {
      const int b = b0 + lane + 64 * i;
      w[i] = b < nblocks ? coherent_load(partials + (int64_t)b * nslots + a) : (fp ? acc_init(kind) : 0);
    }
#pragma unroll
    for (int i = 0; i < kFinLoads; i++) v = acc_combine(kind, v, w[i]);
  }
  if (fp) v = as_u64(wave_reduce_f64(as_f64(v), kind));
  else v = wave_reduce_u64_add(v);
  if (lane == 0) out[a] = v;
}

__device__ __forceinline__ void finalize_tail(const DevFinal *fp) {
  __shared__ uint32_t ticket;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's partial stores / atomics acknowledged
  __syncthreads();
  // Two-level ticket: a workgroup counts itself in its shard (blockIdx % kFinShards, one 64-B line each), the one that
  // completes a shard counts the shard at the top; the completer of the last shard finalizes. One device-scope
  // counter taking every workgroup's add serialised them at the memory side (r04f: +13-50 us per launch).
  if (threadIdx.x == 0) {
    const uint32_t k = blockIdx.x % kFinShards;
    const uint32_t nk = min((uint32_t)kFinShards, gridDim.x);
    const uint32_t in_shard = (gridDim.x - k + kFinShards - 1) / kFinShards;
    uint32_t *sc = fp->counter + 16 * (1 + k);
    uint32_t last = 0;
    if (__hip_atomic_fetch_add(sc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == in_shard - 1) {
      __hip_atomic_store(sc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = __hip_atomic_fetch_add(fp->counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nk - 1 ? 1u : 0u;
    }
    ticket = last;
  }
  __syncthreads();
  if (ticket == 0) return;
  const DevFinal &f = *fp;
  const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int s = wave; s < f.na + 2; s += nw) {
    if (s < f.na) fin_slot(f.pa, f.nba, f.na, f.ka[s], f.out, s);
    else if (f.pf != nullptr) fin_slot(f.pf, f.nbf, 2, f.kf[s - f.na], f.out + 32, s - f.na);
  }
  for (int i = threadIdx.x; i < f.nseg; i += blockDim.x) {
    f.out[64 + i] = coherent_load(f.segm + i);
    coherent_store(f.segm + i, 0ull);
  }
  uint32_t *oh = (uint32_t *)(f.out + 64 + f.nseg);
  for (int i = threadIdx.x; i < f.hll_words; i += blockDim.x) {
    oh[i] = coherent_load(f.hll + i);
    __hip_atomic_store(f.hll + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (threadIdx.x == 0) __hip_atomic_store(f.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace phip
