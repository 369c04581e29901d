// agg_kernel.h -- the aggregation / group-by kernel templates of aggregate.hip (K5-K9), included by the
// per-variant translation units agg_k_*.hip so the thirteen agg_kernel variants compile in parallel. Only
// templates and inline device functions live here (no host symbols).
#pragma once
#include <hip/hip_ext.h>

#include "agg_common.h"

namespace phip {

// GB_NONE id histogram (DevAggQuery.hist_aggs, the kHist variants): per-wave LDS bins of two u16 counts per word,
// indexed by the segment's dictionary id of hist_col; n = an upper bound of the docs counted since the last flush, so
// no count passes 65535.
struct HistCtx {
  lds_u32 *bins;
  int n;
};
// The bins folded into the accumulators (the segment's dictionary values: sum += count x value, min / max over the
// ids that occurred) and cleared. Wave-local: the wave's own LDS operations complete in order.
template <int NA>
__device__ __forceinline__ void hist_flush(cquery_t &q, cseg_t &seg, uint64_t (&acc)[NA], HistCtx &hc) {
  const int lane = lane_id();
  ccol_t &c = seg.cols[q.hist_col];
#pragma unroll
  for (int a = 0; a < NA; a++) {
    if (a >= q.num_aggs) break;
    if (!((q.hist_aggs >> a) & 1u)) continue;
    const int kind = q.aggs[a].acc;
    if (kind == ACC_SUM_I64) {
      for (int i = lane; i < c.card; i += 64) {
        const uint32_t cnt = (hc.bins[i >> 1] >> ((i & 1) * 16)) & 0xffffu;
        if (cnt) acc[a] += (uint64_t)cnt * (uint64_t)dict_i64(c, (uint32_t)i);
      }
    } else {
      double cur = as_f64(acc[a]);
      for (int i = lane; i < c.card; i += 64) {
        const uint32_t cnt = (hc.bins[i >> 1] >> ((i & 1) * 16)) & 0xffffu;
        if (!cnt) continue;
        const double v = dict_f64(c, (uint32_t)i);
        cur = kind == ACC_MIN_F64 ? fmin(cur, v) : fmax(cur, v);
      }
      acc[a] = as_u64(cur);
    }
  }
  for (int i = lane; i < q.hist_words; i += 64) hc.bins[i] = 0;
  hc.n = 0;
}

// U docs per lane (d[u], act bit u = doc d[u] matched; inactive entries hold a valid doc and contribute the
// identity): every load of the U docs is issued before the first use. staged: dict ids of the stage slots
// come from the wave's LDS stage at tile-relative doc td + 64u (the dense-tile walk); otherwise from HBM.
template <int NA, int U, bool H = false>
__device__ __forceinline__ void agg_docs(cquery_t &q, cseg_t &seg, const int32_t (&d)[U], uint32_t act,
                                         const PHIP_LDS uint8_t *stg, int32_t td, bool staged, uint64_t (&acc)[NA],
                                         lds_u32 *hll_lds, HistCtx *hc = nullptr) {
#pragma unroll
  for (int a = 0; a < NA; a++) {
    if (a >= q.num_aggs) break;
    cagg_t &ag = q.aggs[a];
    if (ag.program != seg.program) continue;  // another filter program's function (wave-uniform)
    const int kind = ag.acc;
    const int ka = staged ? q.stage_slot_a[a] : -1, kb = staged ? q.stage_slot_b[a] : -1;
    const int ja = ka < 0 ? 0 : ka, jb = kb < 0 ? 0 : kb;
    const BatchSrc sa{ka >= 0 ? (const PHIP_LDS uint32_t *)(stg + q.stage_off[ja]) : nullptr, td, act,
                      ka >= 0 && q.stage_dict_off[ja] >= 0 ? stg + q.stage_dict_off[ja] : nullptr};
    if constexpr (H) {
      if ((q.hist_aggs >> a) & 1u) {  // counted per id (the first such aggregation; the others share its bins)
        if (a == __builtin_ctz(q.hist_aggs)) {
          uint32_t id[U];
          batch_ids<U>(seg.cols[ag.col_a], d, sa, id);
#pragma unroll
          for (int u = 0; u < U; u++)
            if ((act >> u) & 1u) __hip_atomic_fetch_add(&hc->bins[id[u] >> 1], 1u << ((id[u] & 1u) * 16), PHIP_RLX, PHIP_WG);
        }
        continue;
      }
    }
    const BatchSrc sb{kb >= 0 ? (const PHIP_LDS uint32_t *)(stg + q.stage_off[jb]) : nullptr, td, act,
                      kb >= 0 && q.stage_dict_off[jb] >= 0 ? stg + q.stage_dict_off[jb] : nullptr};
    if (kind == ACC_COUNT) {
      acc[a] += (uint64_t)__popc(act);
    } else if (kind == ACC_SUM_I64) {
      int64_t v[U];
      batch_expr_i64<U>(seg, ag, d, sa, sb, v);
#pragma unroll
      for (int u = 0; u < U; u++) acc[a] += ((act >> u) & 1u) ? (uint64_t)v[u] : 0ull;
    } else if (kind == ACC_HLL && seg.cols[ag.col_a].hll_rows) {
      ccol_t &c = seg.cols[ag.col_a];
      lds_u32 *regs = hll_lds + (ag.hll_slot << q.log2m);
#pragma unroll
      for (int u = 0; u < U; u++)
        if ((act >> u) & 1u)
          hll_row_each(c, d[u], [&](int r, uint32_t rho) { __hip_atomic_fetch_max(&regs[r], rho, PHIP_RLX, PHIP_WG); });
    } else if (kind == ACC_HLL) {
      ccol_t &c = seg.cols[ag.col_a];
      uint32_t h[U];
      if (ag.expr != PHIP_EXPR_COLUMN) {  // an expression's double values, hashed per doc
        double x[U];
        batch_expr_f64<U>(seg, ag, d, sa, sb, x);
#pragma unroll
        for (int u = 0; u < U; u++) h[u] = hll_entry_bits(__double_as_longlong(x[u]), ag.log2m);
      } else if (c.hll_doc != nullptr || c.hll_doc16 != nullptr) {  // doc-order entries
#pragma unroll
        for (int u = 0; u < U; u++) h[u] = hll_doc_entry(c, d[u]);
      } else if (!c.has_dict) {  // raw values, hashed per doc
#pragma unroll
        for (int u = 0; u < U; u++) h[u] = hll_entry_raw(c, d[u], ag.log2m);
      } else {
        uint32_t id[U];
        batch_ids<U>(c, d, sa, id);
#pragma unroll
        for (int u = 0; u < U; u++) h[u] = ((const glb_u32 *)c.hll)[id[u]];
      }
#pragma unroll
      for (int u = 0; u < U; u++)
        if ((act >> u) & 1u)
          __hip_atomic_fetch_max(&hll_lds[(ag.hll_slot << q.log2m) + (h[u] >> 8)], h[u] & 0xffu, PHIP_RLX, PHIP_WG);
    } else {
      double v[U];
      batch_expr_f64<U>(seg, ag, d, sa, sb, v);
      double cur = as_f64(acc[a]);
#pragma unroll
      for (int u = 0; u < U; u++) {
        const bool on = (act >> u) & 1u;
        if (kind == ACC_SUM_F64) cur = cur + (on ? v[u] : 0.0);
        else if (kind == ACC_MIN_F64) cur = fmin(cur, on ? v[u] : __builtin_huge_val());
        else cur = fmax(cur, on ? v[u] : -__builtin_huge_val());
      }
      acc[a] = as_u64(cur);
    }
  }
  if constexpr (H) {
    hc->n += 64 * U;
    if (hc->n > 65535 - 64 * U) hist_flush<NA>(q, seg, acc, *hc);
  }
}

// Groups [g0, g0 + U) of a tile; act bit u = doc 64(g0 + u) + lane matched. Accumulation order per
// lane is the doc order, as in agg_chunk.
template <int NA, int U, bool H = false>
__device__ __forceinline__ void agg_batch(cquery_t &q, cseg_t &seg, int32_t doc, uint32_t act, int32_t safe,
                                          const PHIP_LDS uint8_t *stg, int32_t td, uint64_t (&acc)[NA],
                                          lds_u32 *hll_lds, HistCtx *hc = nullptr) {
  int32_t d[U];
  batch_docs<U>(doc, act, safe, d);
  agg_docs<NA, U, H>(q, seg, d, act, stg, td, true, acc, hll_lds, hc);
}

// Up to kBatch chunks of 64 ring entries at once (GB_NONE): chunk u holds ring[tail + 64u + lane] while
// 64u + lane < n, so its loads are in flight together -- one gather round trip per 256 matched docs, not
// per 64. Per lane the docs stay in ring (= doc) order.
constexpr int kRing = kRingAgg;  // agg_ring_batch runs in GB_NONE only

template <int NA, bool H = false>
__device__ __forceinline__ void agg_ring_batch(cquery_t &q, cseg_t &seg, const lds_u32 *ring, int tail, int n,
                                               uint64_t (&acc)[NA], lds_u32 *hll_lds, int32_t safe,
                                               HistCtx *hc = nullptr) {
  const int lane = lane_id();
  int32_t d[kBatch];
  uint32_t act = 0;
#pragma unroll
  for (int u = 0; u < kBatch; u++) {
    const bool on = 64 * u + lane < n;
    d[u] = on ? (int32_t)ring[(tail + 64 * u + lane) & (kRing - 1)] : safe;
    act |= on ? (1u << u) : 0u;
  }
  agg_docs<NA, kBatch, H>(q, seg, d, act, nullptr, 0, false, acc, hll_lds, hc);
}

// ------------------------------------------------------------------------------------------------
// batched group-by walk (GB_LDS / GB_GLOBAL, dense_batch): kBatch chunks of 64 ring entries per round trip.
// Every key column's ids of the batch are issued together, then every remap gather, then per aggregation
// both input columns' ids together and then both dictionary gathers: per 256 matched docs the key costs two
// dependent round trips and each aggregation two more, where the one-chunk walk paid them per 64 docs
// (DictionaryBasedGroupKeyGenerator.java:285-414 keys, DoubleGroupByResultHolder.java:94-98 holders).
// ------------------------------------------------------------------------------------------------
template <int U>
__device__ __forceinline__ void batch_ids_hbm(ccol_t &c, const int32_t (&d)[U], uint32_t (&id)[U]) {
  const uint32_t b = (uint32_t)c.bits;
#pragma unroll
  for (int u = 0; u < U; u++) id[u] = decode_bits(c.words, (uint64_t)(uint32_t)d[u] * b, b);
}

// enableNullHandling null keys: a null doc of a null-key column takes the column's null key id
template <int U>
__device__ __forceinline__ void batch_null_keys(ccol_t &c, const int32_t (&d)[U], uint32_t (&id)[U]) {
  if (c.gb_nulls == nullptr) return;
  uint64_t w[U];
#pragma unroll
  for (int u = 0; u < U; u++) w[u] = c.gb_nulls[(uint32_t)d[u] >> 6];
#pragma unroll
  for (int u = 0; u < U; u++)
    if ((w[u] >> ((uint32_t)d[u] & 63u)) & 1ull) id[u] = (uint32_t)c.gb_null_id;
}

// one group-by column's contribution to the keys of a batch (ids, remap, stride)
template <int U>
__device__ __forceinline__ void batch_key_column(cquery_t &q, cseg_t &seg, int k, const int32_t (&d)[U],
                                                 int32_t (&key)[U]) {
  ccol_t &c = seg.cols[q.gb_cols[k]];
  uint32_t id[U];
  if (c.gb_ids != nullptr) {
#pragma unroll
    for (int u = 0; u < U; u++) id[u] = (uint32_t)c.gb_ids[d[u]];
  } else if (c.has_dict) {
    batch_ids_hbm<U>(c, d, id);
    if (c.remap) {
#pragma unroll
      for (int u = 0; u < U; u++) id[u] = (uint32_t)((const PHIP_GLB int32_t *)c.remap)[id[u]];
    }
  } else {
#pragma unroll
    for (int u = 0; u < U; u++) id[u] = (uint32_t)(raw_i64(c, d[u]) - c.gb_base);
  }
  batch_null_keys<U>(c, d, id);
#pragma unroll
  for (int u = 0; u < U; u++) key[u] += (int32_t)id[u] * (int32_t)q.gb_stride[k];
}

// The first kKeyFast columns' ids are issued together, then their remaps (two round trips for up to four columns);
// columns past them (a GROUP BY of more than four columns) follow one at a time.
constexpr int kKeyFast = 4;
template <int U>
__device__ __forceinline__ void batch_group_keys(cquery_t &q, cseg_t &seg, const int32_t (&d)[U], int32_t (&key)[U]) {
  uint32_t id[kKeyFast][U];
#pragma unroll
  for (int k = 0; k < kKeyFast; k++) {
#pragma unroll
    for (int u = 0; u < U; u++) id[k][u] = 0;
    if (k < q.num_group_by) {
      ccol_t &c = seg.cols[q.gb_cols[k]];
      if (c.gb_ids != nullptr) {  // raw FLOAT / DOUBLE: the doc's id column
#pragma unroll
        for (int u = 0; u < U; u++) id[k][u] = (uint32_t)c.gb_ids[d[u]];
      } else if (c.has_dict) {
        batch_ids_hbm<U>(c, d, id[k]);
      } else {  // raw INT / LONG: value - gb_base (below 2^31 here: an LDS / HBM table's key space)
#pragma unroll
        for (int u = 0; u < U; u++) id[k][u] = (uint32_t)(raw_i64(c, d[u]) - c.gb_base);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < kKeyFast; k++) {
    if (k < q.num_group_by) {
      ccol_t &c = seg.cols[q.gb_cols[k]];
      if (c.has_dict && c.remap) {
#pragma unroll
        for (int u = 0; u < U; u++) id[k][u] = (uint32_t)((const PHIP_GLB int32_t *)c.remap)[id[k][u]];
      }
      batch_null_keys<U>(c, d, id[k]);
    }
  }
  // (GB_LDS / GB_GLOBAL key spaces are below 2^31: 32-bit keys and strides)
#pragma unroll
  for (int u = 0; u < U; u++) {
    int32_t kk = 0;
#pragma unroll
    for (int k = 0; k < kKeyFast; k++)
      if (k < q.num_group_by) kk += (int32_t)id[k][u] * (int32_t)q.gb_stride[k];
    key[u] = kk;
  }
#pragma unroll 1
  for (int k = kKeyFast; k < q.num_group_by; k++) batch_key_column<U>(q, seg, k, d, key);
}

// Values of a batch from ids already loaded (dictionary columns) or from the raw column.
template <int U>
__device__ __forceinline__ void batch_vals_i64(ccol_t &c, const int32_t (&d)[U], const uint32_t (&id)[U],
                                               int64_t (&v)[U]) {
  if (c.has_dict) {
    if (c.type == PHIP_TYPE_INT) {
#pragma unroll
      for (int u = 0; u < U; u++) v[u] = ((const PHIP_GLB int32_t *)c.dict)[id[u]];
    } else if (c.type == PHIP_TYPE_LONG) {
#pragma unroll
      for (int u = 0; u < U; u++) v[u] = ((const PHIP_GLB int64_t *)c.dict)[id[u]];
    } else {
#pragma unroll
      for (int u = 0; u < U; u++) v[u] = dict_i64(c, id[u]);
    }
  } else {
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = raw_i64(c, d[u]);
  }
}
template <int U>
__device__ __forceinline__ void batch_vals_f64(ccol_t &c, const int32_t (&d)[U], const uint32_t (&id)[U],
                                               double (&v)[U]) {
  if (c.has_dict) {
    if (c.type == PHIP_TYPE_INT) {
#pragma unroll
      for (int u = 0; u < U; u++) v[u] = (double)((const PHIP_GLB int32_t *)c.dict)[id[u]];
    } else if (c.type == PHIP_TYPE_DOUBLE) {
#pragma unroll
      for (int u = 0; u < U; u++) v[u] = ((const PHIP_GLB double *)c.dict)[id[u]];
    } else {
#pragma unroll
      for (int u = 0; u < U; u++) v[u] = dict_f64(c, id[u]);
    }
  } else {
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = raw_f64(c, d[u]);
  }
}

// expr_i64 / expr_f64 over a batch: both inputs' ids in flight together, then both gathers.
template <int U>
__device__ __forceinline__ void batch_expr2_i64(cseg_t &s, cagg_t &a, const int32_t (&d)[U], int64_t (&x)[U]) {
  ccol_t &ca = s.cols[a.col_a];
  const bool two = a.expr != PHIP_EXPR_COLUMN;
  uint32_t ia[U], ib[U];
  if (ca.has_dict) batch_ids_hbm<U>(ca, d, ia);
  if (two && s.cols[a.col_b].has_dict) batch_ids_hbm<U>(s.cols[a.col_b], d, ib);
  batch_vals_i64<U>(ca, d, ia, x);
  if (!two) return;
  int64_t y[U];
  batch_vals_i64<U>(s.cols[a.col_b], d, ib, y);
#pragma unroll
  for (int u = 0; u < U; u++) {
    if (a.expr == PHIP_EXPR_ADD) x[u] = x[u] + y[u];
    else if (a.expr == PHIP_EXPR_SUB) x[u] = x[u] - y[u];
    else x[u] = x[u] * y[u];
  }
}
template <int U>
__device__ __forceinline__ void batch_expr2_f64(cseg_t &s, cagg_t &a, const int32_t (&d)[U], double (&x)[U]) {
  ccol_t &ca = s.cols[a.col_a];
  const bool two = a.expr != PHIP_EXPR_COLUMN;
  uint32_t ia[U], ib[U];
  if (ca.has_dict) batch_ids_hbm<U>(ca, d, ia);
  if (two && s.cols[a.col_b].has_dict) batch_ids_hbm<U>(s.cols[a.col_b], d, ib);
  batch_vals_f64<U>(ca, d, ia, x);
  if (!two) return;
  double y[U];
  batch_vals_f64<U>(s.cols[a.col_b], d, ib, y);
#pragma unroll
  for (int u = 0; u < U; u++) {
    if (a.expr == PHIP_EXPR_ADD) x[u] = x[u] + y[u];
    else if (a.expr == PHIP_EXPR_SUB) x[u] = x[u] - y[u];
    else x[u] = x[u] * y[u];
  }
}

// One table word update: LDS atomics for the workgroup's table, agent-scope atomics for the HBM table, and for the
// XCD-private copies (GB_XCD) workgroup-scope atomics on the copy of the XCD the wave runs on: every wave that
// touches a copy shares that XCD's L2, where the atomic is performed (an agent-scope one goes to the memory side,
// which serialises hot rows); the kernel's end-of-launch release writes the L2 back for xcd_merge_kernel.
__device__ __forceinline__ int64_t xcd_copy() {
  return (int64_t)(__builtin_amdgcn_s_getreg((3 << 11) | 20) & (kXcdCopies - 1));  // hwreg(HW_REG_XCC_ID, 0, 4)
}
template <int MODE>
__device__ __forceinline__ void tbl_add_u64(cquery_t &q, lds_u64 *tbl, int64_t i, uint64_t v) {
  if constexpr (MODE == GB_LDS) __hip_atomic_fetch_add(&tbl[i], v, PHIP_RLX, PHIP_WG);
  else if constexpr (MODE == GB_XCD)
    __hip_atomic_fetch_add(&((glb_u64 *)q.gb_table)[xcd_copy() * q.xcd_words + i], v, PHIP_RLX, PHIP_WG);
  else __hip_atomic_fetch_add(&((glb_u64 *)q.gb_table)[i], v, PHIP_RLX, PHIP_AG);
}
template <int MODE>
__device__ __forceinline__ void tbl_add_f64(cquery_t &q, lds_u64 *tbl, int64_t i, double v) {
  if constexpr (MODE == GB_LDS) __hip_atomic_fetch_add((PHIP_LDS double *)&tbl[i], v, PHIP_RLX, PHIP_WG);
  else if constexpr (MODE == GB_XCD)
    __hip_atomic_fetch_add((PHIP_GLB double *)&((glb_u64 *)q.gb_table)[xcd_copy() * q.xcd_words + i], v, PHIP_RLX,
                           PHIP_WG);
  else __hip_atomic_fetch_add((PHIP_GLB double *)&((glb_u64 *)q.gb_table)[i], v, PHIP_RLX, PHIP_AG);
}
template <int MODE>
__device__ __forceinline__ void tbl_minmax(cquery_t &q, lds_u64 *tbl, int64_t i, uint64_t v, bool is_min) {
  if constexpr (MODE == GB_LDS) {
    if (is_min) __hip_atomic_fetch_min(&tbl[i], v, PHIP_RLX, PHIP_WG);
    else __hip_atomic_fetch_max(&tbl[i], v, PHIP_RLX, PHIP_WG);
  } else if constexpr (MODE == GB_XCD) {
    glb_u64 *p = &((glb_u64 *)q.gb_table)[xcd_copy() * q.xcd_words + i];
    if (is_min) __hip_atomic_fetch_min(p, v, PHIP_RLX, PHIP_WG);
    else __hip_atomic_fetch_max(p, v, PHIP_RLX, PHIP_WG);
  } else {
    glb_u64 *p = &((glb_u64 *)q.gb_table)[i];
    if (is_min) __hip_atomic_fetch_min(p, v, PHIP_RLX, PHIP_AG);
    else __hip_atomic_fetch_max(p, v, PHIP_RLX, PHIP_AG);
  }
}
template <int MODE>
__device__ __forceinline__ void tbl_hll(cquery_t &q, lds_u32 *hll_packed, int slot, int64_t key, uint32_t reg,
                                        uint32_t rho) {
  const int64_t G = q.num_groups;
  if constexpr (MODE == GB_LDS) {
    lds_hll_max(hll_packed + ((((int64_t)slot * G + key) << q.log2m) >> 2), reg, rho);
  } else if constexpr (MODE == GB_XCD) {
    glb_u32 *r = (glb_u32 *)q.gb_hll + xcd_copy() * q.xcd_hll_words + (((int64_t)slot * G + key) << q.log2m) + reg;
    if (*r < rho) __hip_atomic_fetch_max(r, rho, PHIP_RLX, PHIP_WG);  // (a stale read only costs an atomic)
  } else {
    glb_u32 *r = (glb_u32 *)q.gb_hll + (((int64_t)slot * G + key) << q.log2m) + reg;
    if (*r < rho) __hip_atomic_fetch_max(r, rho, PHIP_RLX, PHIP_AG);
  }
}

// ------------------------------------------------------------------------------------------------
// Group-by records (DevSeg.rec, runtime.cpp build_records): a matched doc's key ids, value fields and HLL entry come
// from ONE 16-byte load of its record instead of one gather per column. Every gathered column touched nearly every
// line of itself (C5: five columns at 4 % density, ~4.3 GB of lines per launch at ~5.6 TB/s); the record's lines
// hold every field, so the launch touches fewer of them. Records are W <= 4 u32; the load always reads 16 bytes (the
// allocation has the slack), so it is one instruction whatever W is.
// ------------------------------------------------------------------------------------------------
struct RecW {
  uint32_t w0, w1, w2, w3;
};
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
__device__ __forceinline__ RecW rec_load(cseg_t &seg, int32_t doc) {
  const PHIP_GLB u32x4_a4 *p =
      (const PHIP_GLB u32x4_a4 *)((const PHIP_GLB uint32_t *)seg.rec + (int64_t)doc * seg.rec_words);
  const u32x4_a4 v = __builtin_nontemporal_load(p);
  return RecW{v.x, v.y, v.z, v.w};
}
// field f of a record (offset and width wave-uniform)
__device__ __forceinline__ uint32_t rec_field(cseg_t &seg, const RecW &r, int f) {
  const int off = seg.rec_off[f], bits = seg.rec_bits[f];
  const int i = off >> 5, sh = off & 31;
  const uint32_t lo = i == 0 ? r.w0 : (i == 1 ? r.w1 : (i == 2 ? r.w2 : r.w3));
  const uint32_t hi = i == 0 ? r.w1 : (i == 1 ? r.w2 : (i == 2 ? r.w3 : 0u));
  const uint64_t v = ((((uint64_t)hi) << 32) | lo) >> sh;
  return bits >= 32 ? (uint32_t)v : (uint32_t)v & ((1u << bits) - 1u);
}
// the group key of a record (key fields 0 .. num_group_by - 1: dictionary ids, remapped)
__device__ __forceinline__ int32_t rec_key(cquery_t &q, cseg_t &seg, const RecW &r) {
  int32_t key = 0;
  for (int k = 0; k < kRecKeys; k++) {
    if (k >= q.num_group_by) break;
    ccol_t &c = seg.cols[q.gb_cols[k]];
    uint32_t id = rec_field(seg, r, k);
    if (c.remap) id = (uint32_t)((const PHIP_GLB int32_t *)c.remap)[id];
    key += (int32_t)id * (int32_t)q.gb_stride[k];
  }
  return key;
}
// a value input of an aggregation from its field: packed value (vbase + bits) or dictionary id (gathered)
__device__ __forceinline__ int64_t rec_i64(ccol_t &c, uint32_t x) {
  return c.vpack != nullptr ? c.vbase + (int64_t)x : dict_i64(c, x);
}
__device__ __forceinline__ double rec_f64(ccol_t &c, uint32_t x) {
  return c.vpack != nullptr ? (double)(c.vbase + (int64_t)x) : dict_f64(c, x);
}
// the updates of one matched doc's record (act: the lane holds a matched doc)
template <int MODE>
__device__ __forceinline__ void rec_update(cquery_t &q, cseg_t &seg, const RecW &r, int32_t key, bool act, lds_u64 *tbl,
                                           lds_u32 *hll_packed) {
  const int64_t G = q.num_groups;
  if (act) tbl_add_u64<MODE>(q, tbl, key, 1ull);
  for (int a = 0; a < kMaxAggs; a++) {
    if (a >= q.num_aggs) break;
    cagg_t &ag = q.aggs[a];
    if (ag.program != seg.program) continue;  // another filter program's function (wave-uniform)
    const int64_t at = (int64_t)(1 + a) * G + key;
    const int kind = ag.acc;
    if (kind == ACC_COUNT) {
      if (q.own_count_rows && act) tbl_add_u64<MODE>(q, tbl, at, 1ull);
    } else if (kind == ACC_HLL) {
      const uint32_t x = rec_field(seg, r, q.rec_fa[a]);
      const uint32_t h = seg.cols[ag.col_a].hll_doc16 != nullptr ? (((x >> 5) << 8) | (x & 31u)) : x;
      if (act) tbl_hll<MODE>(q, hll_packed, ag.hll_slot, key, h >> 8, h & 0xffu);
    } else {
      ccol_t &ca = seg.cols[ag.col_a];
      const uint32_t xa = rec_field(seg, r, q.rec_fa[a]);
      const bool two = ag.expr != PHIP_EXPR_COLUMN;
      if (kind == ACC_SUM_I64) {
        int64_t x = rec_i64(ca, xa);
        if (two) {
          const int64_t y = rec_i64(seg.cols[ag.col_b], rec_field(seg, r, q.rec_fb[a]));
          x = ag.expr == PHIP_EXPR_ADD ? x + y : (ag.expr == PHIP_EXPR_SUB ? x - y : x * y);
        }
        if (act) tbl_add_u64<MODE>(q, tbl, at, (uint64_t)x);
      } else {
        double x = rec_f64(ca, xa);
        if (two) {
          const double y = rec_f64(seg.cols[ag.col_b], rec_field(seg, r, q.rec_fb[a]));
          x = ag.expr == PHIP_EXPR_ADD ? x + y : (ag.expr == PHIP_EXPR_SUB ? x - y : x * y);
        }
        if (act) {
          if (kind == ACC_SUM_F64) tbl_add_f64<MODE>(q, tbl, at, x);
          else tbl_minmax<MODE>(q, tbl, at, f64_ordered(x), kind == ACC_MIN_F64);
        }
      }
    }
  }
}
// one-chunk walk: 64 ring docs (inactive lanes carry doc 0, a valid doc)
template <int MODE>
__device__ __forceinline__ void group_chunk_rec(cquery_t &q, cseg_t &seg, int32_t doc, bool act, lds_u64 *tbl,
                                                lds_u32 *hll_packed) {
  const RecW r = rec_load(seg, doc);
  const int32_t key = rec_key(q, seg, r);
  rec_update<MODE>(q, seg, r, key, act, tbl, hll_packed);
}
// batched walk: U chunks of ring entries, every record load issued before the first is decoded
template <int MODE, int U, int RING>
__device__ __forceinline__ void group_ring_batch_rec(cquery_t &q, cseg_t &seg, const lds_u32 *ring, int tail, int n,
                                                     lds_u64 *tbl, lds_u32 *hll_packed) {
  const int lane = lane_id();
  RecW r[U];
  uint32_t act = 0;
#pragma unroll
  for (int u = 0; u < U; u++) {
    const bool on = 64 * u + lane < n;
    const int32_t d = on ? (int32_t)ring[(tail + 64 * u + lane) & (RING - 1)] : 0;
    act |= on ? (1u << u) : 0u;
    r[u] = rec_load(seg, d);
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    const int32_t key = rec_key(q, seg, r[u]);
    rec_update<MODE>(q, seg, r[u], key, ((act >> u) & 1u) != 0, tbl, hll_packed);
  }
}

constexpr int kRingGB = kRingGroupBatch;

// (U chunks of 64 ring entries per round trip from a ring of RING entries; the fused group-by of filter_kernel.h uses
// a smaller ring and batch than the aggregation kernel)
template <int MODE, int U = kBatch, int RING = kRingGB, bool kRec = false>
__device__ __forceinline__ void group_ring_batch(cquery_t &q, cseg_t &seg, const lds_u32 *ring, int tail, int n,
                                                 lds_u64 *tbl, lds_u32 *hll_packed) {
  if constexpr (kRec) {  // (the record variant only: the other kernels keep their code size)
    if (seg.rec != nullptr) {
      group_ring_batch_rec<MODE, U, RING>(q, seg, ring, tail, n, tbl, hll_packed);
      return;
    }
  }
  const int lane = lane_id();
  int32_t d[U];
  uint32_t act = 0;
#pragma unroll
  for (int u = 0; u < U; u++) {
    const bool on = 64 * u + lane < n;
    d[u] = on ? (int32_t)ring[(tail + 64 * u + lane) & (RING - 1)] : 0;  // (doc 0: a valid doc, no effect)
    act |= on ? (1u << u) : 0u;
  }
  int32_t key[U];
  batch_group_keys<U>(q, seg, d, key);
  const int64_t G = q.num_groups;
#pragma unroll
  for (int u = 0; u < U; u++)
    if ((act >> u) & 1u) tbl_add_u64<MODE>(q, tbl, key[u], 1ull);
  for (int a = 0; a < kMaxAggs; a++) {
    if (a >= q.num_aggs) break;
    cagg_t &ag = q.aggs[a];
    if (ag.program != seg.program) continue;  // another filter program's function (wave-uniform)
    const int kind = ag.acc;
    const int64_t row = (int64_t)(1 + a) * G;
    if (kind == ACC_COUNT) {  // == row 0, unless the programs count apart
      if (q.own_count_rows) {
#pragma unroll
        for (int u = 0; u < U; u++)
          if ((act >> u) & 1u) tbl_add_u64<MODE>(q, tbl, row + key[u], 1ull);
      }
    } else if (kind == ACC_HLL) {
      ccol_t &c = seg.cols[ag.col_a];
      if (c.hll_rows) {
#pragma unroll
        for (int u = 0; u < U; u++)
          if ((act >> u) & 1u)
            hll_row_each(c, d[u], [&](int r, uint32_t rho) { tbl_hll<MODE>(q, hll_packed, ag.hll_slot, key[u], r, rho); });
      } else if (ag.expr != PHIP_EXPR_COLUMN || c.hll_doc != nullptr || c.hll_doc16 != nullptr || !c.has_dict) {
        // an expression's double values or raw values hashed per doc, or doc-order entries
        uint32_t h[U];
        if (ag.expr != PHIP_EXPR_COLUMN) {
          double x[U];
          batch_expr2_f64<U>(seg, ag, d, x);
#pragma unroll
          for (int u = 0; u < U; u++) h[u] = hll_entry_bits(__double_as_longlong(x[u]), ag.log2m);
        } else if (c.hll_doc != nullptr || c.hll_doc16 != nullptr) {
#pragma unroll
          for (int u = 0; u < U; u++) h[u] = hll_doc_entry(c, d[u]);
        } else {
#pragma unroll
          for (int u = 0; u < U; u++) h[u] = hll_entry_raw(c, d[u], ag.log2m);
        }
#pragma unroll
        for (int u = 0; u < U; u++)
          if ((act >> u) & 1u) tbl_hll<MODE>(q, hll_packed, ag.hll_slot, key[u], h[u] >> 8, h[u] & 0xffu);
      } else {
        uint32_t id[U], h[U];
        batch_ids_hbm<U>(c, d, id);
#pragma unroll
        for (int u = 0; u < U; u++) h[u] = ((const glb_u32 *)c.hll)[id[u]];
#pragma unroll
        for (int u = 0; u < U; u++)
          if ((act >> u) & 1u) tbl_hll<MODE>(q, hll_packed, ag.hll_slot, key[u], h[u] >> 8, h[u] & 0xffu);
      }
    } else if (kind == ACC_SUM_I64) {
      int64_t v[U];
      batch_expr2_i64<U>(seg, ag, d, v);
#pragma unroll
      for (int u = 0; u < U; u++)
        if ((act >> u) & 1u) tbl_add_u64<MODE>(q, tbl, row + key[u], (uint64_t)v[u]);
    } else {
      double v[U];
      batch_expr2_f64<U>(seg, ag, d, v);
#pragma unroll
      for (int u = 0; u < U; u++) {
        if (!((act >> u) & 1u)) continue;
        if (kind == ACC_SUM_F64) tbl_add_f64<MODE>(q, tbl, row + key[u], v[u]);
        else tbl_minmax<MODE>(q, tbl, row + key[u], f64_ordered(v[u]), kind == ACC_MIN_F64);
      }
    }
  }
}

// GB_HASH: linear probing from a 64-bit finaliser of the key; a slot is claimed by CAS(empty -> key).
// Plain loads may see a stale "empty" (the CAS then returns the owner) but never a wrong key, because
// a slot changes at most once.
__device__ __forceinline__ uint64_t mix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}
__device__ __forceinline__ int64_t hash_slot(cquery_t &q, uint64_t key) {
  glb_u64 *keys = (glb_u64 *)q.gb_keys;
  const uint64_t mask = (uint64_t)q.num_groups - 1;
  uint64_t i = mix64(key) & mask;
  for (uint64_t p = 0; p <= mask; p++) {
    const uint64_t k = keys[i];
    if (k == key) return (int64_t)i;
    if (k == kHashEmpty) {
      uint64_t expected = kHashEmpty;
      if (__hip_atomic_compare_exchange_strong(&keys[i], &expected, key, PHIP_RLX, PHIP_RLX, PHIP_AG) ||
          expected == key)
        return (int64_t)i;
    }
    i = (i + 1) & mask;
  }
  return -1;
}

// GB_GLOBAL / GB_HASH: one table in HBM ([1 + naggs][G] u64, row 0 counts) at index `slot`.
__device__ __forceinline__ void group_update_global(cquery_t &q, cseg_t &seg, int32_t doc, int64_t slot) {
  const int64_t G = q.num_groups;
  glb_u64 *tbl = (glb_u64 *)q.gb_table;
  __hip_atomic_fetch_add(&tbl[slot], 1ull, PHIP_RLX, PHIP_AG);
  for (int a = 0; a < kMaxAggs; a++) {
    if (a >= q.num_aggs) break;
    cagg_t &ag = q.aggs[a];
    if (ag.program != seg.program) continue;  // another filter program's function (wave-uniform)
    glb_u64 *p = tbl + (1 + a) * G + slot;
    switch (ag.acc) {
      case ACC_COUNT:
        if (q.own_count_rows) __hip_atomic_fetch_add(p, 1ull, PHIP_RLX, PHIP_AG);
        break;
      case ACC_SUM_I64: __hip_atomic_fetch_add(p, (uint64_t)expr_i64(seg, ag, doc), PHIP_RLX, PHIP_AG); break;
      case ACC_SUM_F64:
        __hip_atomic_fetch_add((PHIP_GLB double *)p, expr_f64(seg, ag, doc), PHIP_RLX, PHIP_AG);
        break;
      case ACC_MIN_F64: __hip_atomic_fetch_min(p, f64_ordered(expr_f64(seg, ag, doc)), PHIP_RLX, PHIP_AG); break;
      case ACC_MAX_F64: __hip_atomic_fetch_max(p, f64_ordered(expr_f64(seg, ag, doc)), PHIP_RLX, PHIP_AG); break;
      case ACC_HLL: {
        ccol_t &c = seg.cols[ag.col_a];
        glb_u32 *regs = (glb_u32 *)q.gb_hll + (((int64_t)ag.hll_slot * G + slot) << q.log2m);
        if (c.hll_rows) {
          hll_row_each(c, doc, [&](int r, uint32_t rho) {
            if (regs[r] < rho) __hip_atomic_fetch_max(&regs[r], rho, PHIP_RLX, PHIP_AG);
          });
        } else {
          const uint32_t h = hll_entry_agg(seg, ag, doc);
          glb_u32 *r = regs + (h >> 8);
          if (*r < (h & 0xffu)) __hip_atomic_fetch_max(r, h & 0xffu, PHIP_RLX, PHIP_AG);
        }
        break;
      }
    }
  }
}

// GB_GLOBAL: the dense key is the slot (HLL registers [nhll][G][m] u32).
__device__ __forceinline__ void group_chunk_global(cquery_t &q, cseg_t &seg, int32_t doc, bool act) {
  const int64_t key = group_key(q, seg, doc);
  if (!act) return;
  group_update_global(q, seg, doc, key);
}

__device__ __forceinline__ void group_chunk_hash(cquery_t &q, cseg_t &seg, int32_t doc, bool act) {
  int64_t key = group_key(q, seg, doc);
  if (!act) return;
  // numGroupsLimit pass (limit.hip): composite key per (segment, key) -- seg_index = program * segments +
  // segment, so the modulo keeps the segment alone (the programs of a segment share its group generator) -- and
  // the first-seen position: program (info order) major, doc minor, as FilteredGroupByOperator feeds the shared
  // DictionaryBasedGroupKeyGenerator info by info (the host bounds programs x docs below 2^32)
  if (q.seg_keys) key = key * q.seg_key_mult + seg.seg_index % q.seg_key_mult;
  const int64_t slot = hash_slot(q, (uint64_t)key);
  if (slot < 0) {
    __hip_atomic_fetch_or((glb_u32 *)q.hash_overflow, 1u, PHIP_RLX, PHIP_AG);
    return;
  }
  if (q.seg_keys) {
    glb_u32 *fd = (glb_u32 *)q.first_doc + slot;
    const uint32_t pos = (uint32_t)seg.program * (uint32_t)seg.num_docs + (uint32_t)doc;
    if (*fd > pos) __hip_atomic_fetch_min(fd, pos, PHIP_RLX, PHIP_AG);
  }
  group_update_global(q, seg, doc, slot);
}

template <int NA, int MODE, bool kRec = false>
__device__ __forceinline__ void do_chunk(cquery_t &q, cseg_t &seg, int32_t doc, bool act, uint64_t (&acc)[NA],
                                         lds_u32 *hll_lds, lds_u64 *tbl, lds_u32 *hll_packed) {
  if constexpr (MODE == GB_NONE) agg_chunk<NA>(q, seg, doc, act, acc, hll_lds);
  // (Round 6 tried a prefetched chunk here: every column's load issued straight-line before any decode, then every
  // dictionary / remap gather -- two round trips per chunk instead of one per load. It was slower: C5 aggregation 0.77
  // -> 0.82 ms, Q3.1 one-chunk 0.61 -> 0.67, Q4.3 0.050 -> 0.054 (profiles/r06o_pf_ab.log): the walk is bound by the
  // gathers' per-lane line requests, not by their round trips, and the straight-line form issued more of them.)
  else if constexpr (MODE == GB_LDS) {
    if (kRec && seg.rec != nullptr) group_chunk_rec<GB_LDS>(q, seg, doc, act, tbl, hll_packed);
    else group_chunk_lds(q, seg, doc, act, tbl, hll_packed);
  } else if constexpr (MODE == GB_HASH) {
    group_chunk_hash(q, seg, doc, act);
  } else {
    group_chunk_global(q, seg, doc, act);
  }
}

// ------------------------------------------------------------------------------------------------
// the aggregation kernel
// LDS: [per-wave doc rings] [GB_NONE: HLL registers u32] [GB_LDS: table u64 | packed HLL u32]
// ------------------------------------------------------------------------------------------------
// kDense: the batched dense-tile walk is compiled in (host: dq.dense_batch). Without it the kernel is
// the per-64-doc ring walk alone -- its smaller code and register footprint measured 8-10 % faster on
// the sparse SSB Q1.x aggregations than a kernel that merely skips the batched path at run time.
// For GB_LDS / GB_GLOBAL, kDense selects the batched group-by walk (group_ring_batch) instead.
// W: waves per workgroup (8; 16 for an LDS group table so large that one workgroup fills the CU's LDS -- twice the
// waves share the one table, so the CU keeps 16 waves of gathers in flight instead of 8: DevAggQuery.wg_waves).
// kRec: the group-by record variant (DevAggQuery.rec_on: some segment has a DevSeg.rec; GB_LDS only).
template <int NA, int MODE, bool kDense, int W = kAggWaves, bool kRec = false, bool kHist = false>
__global__ __launch_bounds__(W * kWave, (MODE == GB_LDS || MODE == GB_GLOBAL) && kDense ? 6 : 1)
void agg_kernel(const DevAggQuery *qptr) {
  constexpr int kBlock = W * kWave;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  cquery_t &q = *(cquery_t *)qptr;
  const int lane = lane_id();
  const int wave = uniform(threadIdx.x >> 6);
  PHIP_LDS unsigned char *lds = (PHIP_LDS unsigned char *)smem;
  constexpr bool kGbBatch = (MODE == GB_LDS || MODE == GB_GLOBAL) && kDense;
  constexpr bool kRingFill = MODE == GB_NONE || kGbBatch;  // matched docs enter the ring by a wave prefix scan
  constexpr int R = ring_entries(MODE, kGbBatch);
  lds_u32 *ring = (lds_u32 *)lds + wave * R;
  PHIP_LDS unsigned char *stage = lds + W * R * 4;  // GB_NONE dense-tile staging
  PHIP_LDS unsigned char *stg = stage + wave * q.stage_bytes;
  const uint32_t stg_lds = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)stg);
  PHIP_LDS unsigned char *rest = stage + W * q.stage_bytes;
  lds_u32 *hll_lds = (lds_u32 *)rest;
  lds_u64 *tbl = (lds_u64 *)rest;
  lds_u32 *hll_packed = (lds_u32 *)(rest + (size_t)q.tbl_words * 8);
  int hll_words = 0;
  if (MODE == GB_NONE && q.num_hll > 0) {
    hll_words = q.num_hll << q.log2m;
    for (int i = threadIdx.x; i < hll_words; i += kBlock) hll_lds[i] = 0;
  }
  HistCtx hc{nullptr, 0};  // (kHist: the wave's id bins after the HLL registers)
  if constexpr (kHist) {
    hc.bins = (lds_u32 *)rest + (size_t)hll_words + (size_t)wave * q.hist_words;
    for (int i = lane; i < q.hist_words; i += 64) hc.bins[i] = 0;
  }
  if (MODE == GB_LDS) {
    const int G = (int)q.num_groups;
    for (int i = threadIdx.x; i < q.tbl_words; i += kBlock) {
      const int row = i / G;
      uint64_t init = 0;
      if (row > 0 && q.aggs[row - 1].acc == ACC_MIN_F64) init = ~0ull;  // ordered(+inf) < ~0
      tbl[i] = init;
    }
    for (int i = threadIdx.x; i < q.hll_words; i += kBlock) hll_packed[i] = 0;
  }
  __syncthreads();

  // XCD-aware walk (grid is a multiple of 8 workgroups)
  const int x = blockIdx.x & 7;
  const int j = blockIdx.x >> 3;
  const int gx = gridDim.x >> 3;
  const int xs = (int)((int64_t)q.total_work * x / 8);
  const int xe = (int)((int64_t)q.total_work * (x + 1) / 8);
  const int wx = gx * W;
  const int wid = j * W + wave;

  uint64_t acc[NA];
#pragma unroll
  for (int a = 0; a < NA; a++) acc[a] = (a < q.num_aggs) ? acc_init(q.aggs[a].acc) : 0;

  cseg_t *segs = (cseg_t *)q.segs;
  const glb_u32 *mask = (const glb_u32 *)q.mask;
  int head = 0, tail = 0;  // ring cursors (wave-uniform)
  int si = 0;
  int dict_si = -1;        // segment whose small dictionaries sit in the wave's stage area
  int t = xs + wid;
  // mask words of the next kMaskAhead tiles in flight (a sparse query skips most tiles: one load round trip
  // per tile would bound the walk)
  constexpr int kMaskAhead = 4;
  uint32_t mq[kMaskAhead];
#pragma unroll
  for (int k = 0; k < kMaskAhead; k++)
    mq[k] = (mask != nullptr && t + k * wx < xe) ? __builtin_nontemporal_load(mask + (size_t)(t + k * wx) * 64 + lane) : 0u;
  for (; t < xe; t += wx) {
    const uint32_t m_raw = mq[0];
#pragma unroll
    for (int k = 0; k + 1 < kMaskAhead; k++) mq[k] = mq[k + 1];
    {
      const int tn = t + kMaskAhead * wx;
      mq[kMaskAhead - 1] = (mask != nullptr && tn < xe) ? __builtin_nontemporal_load(mask + (size_t)tn * 64 + lane) : 0u;
    }
    if (segs[si].work_begin + segs[si].num_work <= t) {
      if constexpr (MODE == GB_NONE) {
        if (head > tail) agg_ring_batch<NA, kHist>(q, segs[si], ring, tail, head - tail, acc, hll_lds, 0, &hc);
        if constexpr (kHist) hist_flush<NA>(q, segs[si], acc, hc);  // (the segment's dictionary goes)
      } else if constexpr (kGbBatch) {
        if (head > tail) group_ring_batch<MODE, kBatch, kRingGB, kRec>(q, segs[si], ring, tail, head - tail, tbl, hll_packed);
      } else if (head > tail) {  // leftover (< 64) matched docs of the previous segment
        const bool act = lane < head - tail;
        const int32_t doc = act ? (int32_t)ring[(tail + lane) & (R - 1)] : 0;
        do_chunk<NA, MODE, kRec>(q, segs[si], doc, act, acc, hll_lds, tbl, hll_packed);
      }
      head = tail = 0;
      while (si + 1 < q.num_segs && segs[si + 1].work_begin <= t) si++;
    }
    cseg_t &seg = segs[si];
    const int32_t doc0 = (seg.tile0 + (t - seg.work_begin)) * kTileDocs;
    const int32_t nvalid = min(kTileDocs, seg.num_docs - doc0);
    const uint32_t valid = valid_word(nvalid, lane);
    const uint32_t m = mask != nullptr ? (m_raw & valid) : valid;
    bool dense = ballot(m != valid) == 0;  // every valid doc of the tile matched
    if constexpr (MODE == GB_NONE && kDense) {
      if (!dense) dense = wave_sum_u32((uint32_t)__popc(m)) >= (uint32_t)q.dense_min;
    }
    bool batched = false;
    if constexpr (MODE == GB_NONE && kDense) batched = dense;
    if constexpr (MODE == GB_NONE && kDense) {
    if (batched) {
      // lane-major batches: bit (31 - g) of m = doc 64g + lane (coalesced column reads per group)
      if (q.num_stage > 0) {
        if (dict_si != si) {
          // small dictionaries of the staged columns -> the wave's LDS, once per segment (the wave's
          // LDS operations execute in order, so the batch's reads see these writes)
          for (int k = 0; k < q.num_stage; k++) {
            if (q.stage_dict_off[k] < 0) continue;
            ccol_t &c = seg.cols[q.stage_col[k]];
            if (!c.has_dict) continue;
            const int32_t nw = c.card * ((c.type == PHIP_TYPE_LONG || c.type == PHIP_TYPE_DOUBLE) ? 2 : 1);
            lds_u32 *dst = (lds_u32 *)(stg + q.stage_dict_off[k]);
            for (int i = lane; i < nw; i += 64) dst[i] = ((const glb_u32 *)c.dict)[i];
          }
          dict_si = si;
        }
        // the tile's words of every staged column -> LDS (1 KiB per wave-instruction), one round trip
        const int32_t tile = doc0 / kTileDocs;
        for (int k = 0; k < q.num_stage; k++) {
          ccol_t &c = seg.cols[q.stage_col[k]];
          if (!c.has_dict) continue;  // raw in this segment: read from HBM (batch_i64 / batch_f64)
          const int32_t nb = 256 * c.bits;
          const uint8_t *src = (const uint8_t *)c.words + (size_t)tile * nb + lane * 16;
          const uint32_t dst = stg_lds + (uint32_t)q.stage_off[k];
          for (int off = 0; off < nb; off += 1024)
            if (off + lane * 16 < nb) dma16(src + off, dst + (uint32_t)off);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
#pragma unroll 1
      for (int g0 = 0; g0 < kTileGroups; g0 += kBatch) {
        const uint32_t act = __builtin_bitreverse32(m << g0) & ((1u << kBatch) - 1u);
        if (ballot(act != 0) == 0) continue;
        agg_batch<NA, kBatch, kHist>(q, seg, doc0 + 64 * g0 + lane, act, doc0, stg, 64 * g0 + lane, acc, hll_lds, &hc);
      }
      if (q.num_stage > 0) __builtin_amdgcn_wave_barrier();  // LDS reads done before the next tile's DMA
      continue;
    }
    }
    if constexpr (kRingFill) {
      // Matched docs -> the ring: every lane writes its docs at the wave prefix (DPP scan) of the lanes'
      // popcounts -- a few instructions plus the lane's own matches per tile; a pass per 64-doc group (ballot +
      // rank + write for each of the 32 groups) cost ~320 on sparse tiles, most of the unsorted layout's walk.
      // Lane-major order (lane l: docs 64g + l) when the tile holds few matches; a tile with at least a batch
      // of them is first transposed to the contiguous layout (lane L: docs 32L .. 32L+31), so the ring is in doc
      // order and a chunk's column reads are neighbours. Either way the order is a function of the data alone.
      if (ballot(m != 0) == 0) continue;
      uint32_t cw = m;
      uint32_t cnt = (uint32_t)__popc(cw);
      uint32_t incl = wave_incl_scan(cnt);
      const int total = __builtin_amdgcn_readlane((int)incl, 63);
      const bool doc_order = total >= 64 * kBatch;
      int32_t ldoc = doc0 + lane;
      int dstep = 64;
      if (doc_order) {
        cw = lane_major_to_contig(m);
        cnt = (uint32_t)__popc(cw);
        incl = wave_incl_scan(cnt);
        ldoc = doc0 + 32 * lane;
        dstep = 1;
      }
      const int head0 = head;
      // all at once when the ring has room, else in quarter-tile pieces (16 lanes, <= 512 docs; eighths of <= 256
      // docs in the group-by walk's smaller ring) each after draining the ring below one batch
      const int npiece = head - tail + total <= R ? 1 : (kGbBatch ? 8 : 4);
      for (int p = 0; p < npiece; p++) {
        const int lanes = 64 / npiece;
        const int pend = __builtin_amdgcn_readlane((int)incl, lanes * p + lanes - 1);
        if (lane >= lanes * p && lane < lanes * (p + 1)) {
          uint32_t w = cw;
          int pos = head0 + (int)(incl - cnt);
          while (w) {
            const int j = __builtin_clz(w);
            w &= ~(0x80000000u >> j);
            ring[pos & (R - 1)] = (uint32_t)(ldoc + dstep * j);
            pos++;
          }
        }
        head = head0 + pend;
        while (head - tail >= 64 * kBatch) {
          if constexpr (kGbBatch) group_ring_batch<MODE, kBatch, kRingGB, kRec>(q, seg, ring, tail, 64 * kBatch, tbl, hll_packed);
          else agg_ring_batch<NA, kHist>(q, seg, ring, tail, 64 * kBatch, acc, hll_lds, 0, &hc);
          tail += 64 * kBatch;
        }
      }
      continue;
    }
    if (dense) {
      // every doc of the tile matched: consecutive chunks, coalesced column reads
      for (int c = 0; c < nvalid; c += 64) {
        const bool act = c + lane < nvalid;
        do_chunk<NA, MODE, kRec>(q, seg, act ? doc0 + c + lane : 0, act, acc, hll_lds, tbl, hll_packed);
      }
    } else {
      uint32_t any = wave_or32(m);
      while (any) {
        const int bit = 31 - __builtin_clz(any);
        any &= ~(1u << bit);
        const bool b = (m >> bit) & 1u;
        const uint64_t mm = ballot(b);
        if (b) ring[(head + mbcnt64(mm)) & (R - 1)] = (uint32_t)(doc0 + (31 - bit) * 64 + lane);
        head += __popcll(mm);
        if (head - tail >= 64) {
          const int32_t doc = (int32_t)ring[(tail + lane) & (R - 1)];
          tail += 64;
          do_chunk<NA, MODE, kRec>(q, seg, doc, true, acc, hll_lds, tbl, hll_packed);
        }
      }
    }
  }
  if constexpr (MODE == GB_NONE) {
    if (head > tail) agg_ring_batch<NA, kHist>(q, segs[si], ring, tail, head - tail, acc, hll_lds, 0, &hc);
    if constexpr (kHist) hist_flush<NA>(q, segs[si], acc, hc);
  } else if constexpr (kGbBatch) {
    if (head > tail) group_ring_batch<MODE, kBatch, kRingGB, kRec>(q, segs[si], ring, tail, head - tail, tbl, hll_packed);
  } else if (head > tail) {
    const bool act = lane < head - tail;
    const int32_t doc = act ? (int32_t)ring[(tail + lane) & (R - 1)] : 0;
    do_chunk<NA, MODE, kRec>(q, segs[si], doc, act, acc, hll_lds, tbl, hll_packed);
  }

  // ---- workgroup epilogue --------------------------------------------------------------------
  if constexpr (MODE == GB_NONE) {
    __shared__ uint64_t part[W][kMaxAggs];
#pragma unroll
    for (int a = 0; a < NA; a++) {
      if (a >= q.num_aggs) break;
      const int kind = q.aggs[a].acc;
      uint64_t v;
      if (kind == ACC_COUNT || kind == ACC_SUM_I64 || kind == ACC_HLL) v = wave_reduce_u64_add(acc[a]);
      else v = as_u64(wave_reduce_f64(as_f64(acc[a]), kind));
      if (lane == 0) part[wave][a] = v;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
      for (int a = 0; a < NA; a++) {
        if (a >= q.num_aggs) break;
        const int kind = q.aggs[a].acc;
        uint64_t v = part[0][a];
        for (int w = 1; w < W; w++) v = acc_combine(kind, v, part[w][a]);
        coherent_store(q.partials + (size_t)blockIdx.x * q.num_aggs + a, v);  // (read by the finalizing workgroup)
      }
    }
    for (int i = threadIdx.x; i < hll_words; i += kBlock)
      if (hll_lds[i]) __hip_atomic_fetch_max((glb_u32 *)q.hll_regs + i, (uint32_t)hll_lds[i], PHIP_RLX, PHIP_AG);
    if (q.fin != nullptr) finalize_tail(q.fin);
  } else if constexpr (MODE == GB_LDS) {
    __syncthreads();
    glb_u64 *slab = (glb_u64 *)q.gb_table + (size_t)blockIdx.x * q.tbl_words;
    for (int i = threadIdx.x; i < q.tbl_words; i += kBlock) slab[i] = tbl[i];
    glb_u32 *hs = (glb_u32 *)q.gb_hll + (size_t)blockIdx.x * q.hll_words;
    for (int i = threadIdx.x; i < q.hll_words; i += kBlock) hs[i] = hll_packed[i];
  }
}

template <int NA, int MODE, bool D, int W, bool R = false, bool Hs = false>
hipError_t launch_agg_t(const DevAggQuery *q, int nblocks, size_t lds, hipStream_t s, hipEvent_t e0,
                        hipEvent_t e1) {
  if (lds > 65536) {
    // once per instantiation (a magic static: thread-safe under concurrent queries)
    static const hipError_t configured =
        hipFuncSetAttribute((const void *)agg_kernel<NA, MODE, D, W, R, Hs>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840 - 1024);
    if (configured != hipSuccess) return configured;
  }
  if (e0 != nullptr) {  // timing carried by the dispatch packet itself (hipExtLaunchKernel)
    void *args[] = {(void *)&q};
    return hipExtLaunchKernel((const void *)agg_kernel<NA, MODE, D, W, R, Hs>, dim3(nblocks), dim3(W * kWave), args, lds, s, e0,
                              e1, 0);
  }
  agg_kernel<NA, MODE, D, W, R, Hs><<<nblocks, W * kWave, lds, s>>>(q);
  return hipGetLastError();
}

}  // namespace phip
