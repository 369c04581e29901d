// filter_kernel.h -- the filter kernel templates (filter.hip's K1-K4), included by the per-instantiation
// translation units filter_k*.hip so the five kernel variants compile in parallel (each variant is a large
// kernel: one translation unit took ~8 minutes). Everything here is a template or an inline / noinline
// device function: no host symbols, so several units may include it.
#pragma once
// The filter kernel (K1-K4 of SURVEY.md §2.4).
//
// Execution model. One wave streams a CONTIGUOUS range of 2048-doc tiles (the global work list is
// segment-ordered, so a wave changes segment at most a few times and its segment / filter-program
// metadata stays in the scalar cache). Every scanned column's bytes for a tile (256*b bytes: a
// 64-doc group is exactly 2b words of the u32 word layout, kernels.hip/runtime.cpp) and every
// inverted leaf's 256 dense-word bytes arrive in the wave's LDS ring by LDS-DMA
// (global_load_lds_dwordx4, 1 KiB per wave-instruction); nbuf-1 tiles are in flight while one is
// evaluated, and completion is awaited with a counted vmcnt (a lower bound of the vector-memory
// operations issued after the tile's DMA, kept in SGPRs together with the stage cursor).
//
// A tile's doc set is lane-major: lane l owns a 32-bit word whose bit (31-g) is doc 64g + l. Scan
// leaves decode with lanes = docs of one 64-doc group at a time (one v_alignbit per doc and group),
// which is SVScanDocIdIterator + PredicateEvaluator.applySV
// (pinot-core/.../operator/dociditerators/SVScanDocIdIterator.java:75-142) without the doc-id
// materialisation; AND / OR / NOT (AndDocIdSet / OrDocIdSet / NotDocIdSet) are one VALU op per lane.
// The tile's 64 lane words (256 B, one coalesced store) go to the aggregation kernel when the query
// projects anything; COUNT-only queries stop here (FastFilteredCountOperator.java:66-78).
#include <hip/hip_ext.h>

#include "agg_kernel.h"  // (the fused group-by flushes through agg_kernel.h's group_ring_batch)

namespace phip {

struct Tile {
  int32_t doc0;          // first doc of the tile within the segment
  int32_t valid_docs;    // docs of the tile inside the segment (1..2048)
  const PHIP_LDS uint8_t *stage;  // the tile's LDS ring slot
};

// ------------------------------------------------------------------------------------------------
// filter leaves
// ------------------------------------------------------------------------------------------------
// Group loop of one scan leaf: lane l decodes doc g*64 + l from the staged words (2B words per group).
#define PHIP_GROUP_LOOP(PASS_EXPR)                                             \
  const int lane = lane_id();                                                  \
  const int32_t p = lane * B;                                                  \
  const int32_t q = (p - 1) >> 5;                                              \
  const uint32_t s = (uint32_t)(32 * (q + 1) - p);                             \
  const PHIP_LDS uint32_t *wl = w + q;                                         \
  const int32_t gstride = 2 * B;                                               \
  uint32_t r = 0;                                                              \
  _Pragma("unroll 8") for (int g = 0; g < kTileGroups; g++) {                  \
    const uint32_t win = __builtin_amdgcn_alignbit(wl[0], wl[1], s);           \
    wl += gstride;                                                             \
    r = r + r + (uint32_t)(PASS_EXPR);                                         \
  }                                                                            \
  return r;

// RangePredicateEvaluator on dict ids: lo <= v < hi  <=>  (win - lo<<k) < (hi-lo)<<k with k = 32-B
// (the low k bits of the window belong to the next doc and never carry into the comparison).
__device__ __forceinline__ uint32_t scan_range(const PHIP_LDS uint32_t *w, int B, uint32_t LO, uint32_t SPAN) {
  PHIP_GROUP_LOOP((win - LO) < SPAN)
}

// IN / NOT IN / EQ / NEQ on a column with card <= 64: membership in a 64-bit mask (the host
// complements it for exclusive predicates).
__device__ __forceinline__ uint32_t scan_small_set(const PHIP_LDS uint32_t *w, int B, uint64_t set) {
  const uint32_t k = 32 - B;
  PHIP_GROUP_LOOP(((set >> (win >> k)) & 1ull) != 0)
}

// IN / NOT IN on a larger dictionary: bitset over dict ids in HBM (L1/L2 resident).
__device__ __forceinline__ uint32_t scan_big_set(const PHIP_LDS uint32_t *w, int B, const PHIP_GLB uint32_t *set, bool excl) {
  const uint32_t k = 32 - B;
  PHIP_GROUP_LOOP(((((set[(win >> k) >> 5] >> ((win >> k) & 31)) & 1u) != 0) != excl))
}

// IN / NOT IN on a dictionary of <= 2048 ids: the bitset is spread over the wave (lane l holds word l) and
// each doc fetches its word with ds_bpermute instead of a per-doc global gather.
__device__ __forceinline__ uint32_t scan_lane_set(const PHIP_LDS uint32_t *w, int B, uint32_t myw, bool excl) {
  const uint32_t k = 32 - B;
  PHIP_GROUP_LOOP(((((uint32_t)__builtin_amdgcn_ds_bpermute((int)(((win >> k) >> 5) << 2), (int)myw) >>
                     ((win >> k) & 31)) & 1u) != 0) != excl)
}

// bits [lo, hi] (inclusive, 0 <= lo <= hi <= 31) of a u32
__device__ __forceinline__ uint32_t span32(int lo, int hi) {
  const uint32_t upto = (hi == 31) ? ~0u : ((1u << (hi + 1)) - 1u);
  return upto & ~((1u << lo) - 1u);
}

// Lane-major word of the doc range [s, e] (tile-relative, inclusive, clamped to the tile).
__device__ __forceinline__ uint32_t range_word(int32_t s, int32_t e, int lane) {
  const int32_t g_lo = max(0, (s - lane + 63) >> 6);
  const int32_t g_hi = min(kTileGroups - 1, (e - lane) >= 0 ? (e - lane) >> 6 : -1);
  if (g_lo > g_hi) return 0u;
  return span32(31 - g_hi, 31 - g_lo);
}

// P-layout leaf evaluation and its transpose to lane-major (the conjunctive fast path, below)
template <int P>
__device__ __forceinline__ uint32_t conj_leaf_eval(const PHIP_LDS uint32_t *w, int bits, int kind, uint32_t lo,
                                                uint32_t span, uint64_t set);
template <int P>
__device__ __forceinline__ uint32_t to_lane_major(uint32_t r);

// One leaf over the tile; `valid` = lane-major docs of the tile inside the segment.
__device__ __forceinline__ int64_t raw_int_at(ccol_t &c, int32_t doc) {
  return c.type == PHIP_TYPE_LONG ? ((const PHIP_GLB int64_t *)c.raw)[doc] : (int64_t)((const PHIP_GLB int32_t *)c.raw)[doc];
}
__device__ __forceinline__ double raw_real_at(ccol_t &c, int32_t doc) {
  return c.type == PHIP_TYPE_DOUBLE ? ((const PHIP_GLB double *)c.raw)[doc] : (double)((const PHIP_GLB float *)c.raw)[doc];
}

// Membership in a raw IN list (RawValueBasedPredicateEvaluator's value set): the host sorts and deduplicates the
// values (doubles without NaN, which IEEE equality never matches), so a doc costs log2(count) probes of the
// L1-resident list instead of a scan of it.
template <typename T>
__device__ __forceinline__ bool sorted_contains(const PHIP_GLB T *set, int32_t count, T v) {
  int32_t lo = 0, hi = count;  // first element >= v
  while (lo < hi) {
    const int32_t mid = (lo + hi) >> 1;
    if (set[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo < count && set[lo] == v;
}

// String.compareTo order (UTF-16 code units) over UTF-8 bytes: lead bytes 0xEE / 0xEF (U+E000..U+FFFF) rank after
// the 4-byte leads 0xF0..0xF4 (supplementary characters = surrogate pairs in UTF-16); every other byte keeps its order
// (the host sorts RAW_STRING sets the same way, runtime.cpp java_str_cmp)
__device__ __forceinline__ uint32_t java_order_byte(uint32_t b) { return (b == 0xEEu || b == 0xEFu) ? b + 8u : b; }
__device__ __forceinline__ int java_str_cmp(const PHIP_GLB uint8_t *a, uint32_t al, const PHIP_GLB uint8_t *b,
                                            uint32_t bl) {
  const uint32_t m = al < bl ? al : bl;
  for (uint32_t i = 0; i < m; i++) {
    const uint32_t x = a[i], y = b[i];
    if (x != y) return java_order_byte(x) < java_order_byte(y) ? -1 : 1;
  }
  return al < bl ? -1 : (al > bl ? 1 : 0);
}

// Raw STRING leaf: doc d's UTF-8 bytes [str_off[d], str_off[d+1]) against the bounds (RAW_STRING_RANGE) or a sorted
// value list (RAW_STRING_SET, binary search); payload layouts in pinot_hip.h
__device__ __noinline__ uint32_t eval_raw_string(ccol_t &c, cnode_t *__restrict__ n, uint32_t valid, const Tile &t) {
  const int lane = lane_id();
  const PHIP_GLB uint8_t *bytes = (const PHIP_GLB uint8_t *)c.raw;
  const PHIP_GLB uint64_t *off = (const PHIP_GLB uint64_t *)c.str_off;
  const PHIP_GLB int32_t *w = (const PHIP_GLB int32_t *)n->aux;
  const PHIP_GLB uint8_t *wb = (const PHIP_GLB uint8_t *)n->aux;
  const bool range = n->leaf_kind == PHIP_LEAF_RAW_STRING_RANGE;
  const int32_t lo_len = range ? w[0] : 0, hi_len = range ? w[1] : 0;
  const bool lo_in = range && w[2] != 0, hi_in = range && w[3] != 0;
  const uint32_t nv = range ? 0u : (uint32_t)w[0];
  const PHIP_GLB uint32_t *vo = (const PHIP_GLB uint32_t *)(w + 1);
  const PHIP_GLB uint8_t *vb = wb + 4 * (2 + (size_t)nv);
  const bool excl = n->exclusive != 0;
  const int32_t last = t.valid_docs - 1;
  uint32_t r = 0;
  for (int g = 0; g < kTileGroups; g++) {
    const int32_t doc = t.doc0 + min(g * 64 + lane, last);
    const uint64_t s0 = off[doc];
    const uint32_t len = (uint32_t)(off[doc + 1] - s0);
    const PHIP_GLB uint8_t *v = bytes + s0;
    bool pass;
    if (range) {
      pass = true;
      if (lo_len >= 0) {
        const int cmp = java_str_cmp(v, len, wb + 16, (uint32_t)lo_len);
        pass = lo_in ? cmp >= 0 : cmp > 0;
      }
      if (pass && hi_len >= 0) {
        const int cmp = java_str_cmp(v, len, wb + 16 + (lo_len > 0 ? lo_len : 0), (uint32_t)hi_len);
        pass = hi_in ? cmp <= 0 : cmp < 0;
      }
    } else {
      uint32_t lo = 0, hi = nv;  // first value >= the doc's
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (java_str_cmp(v, len, vb + vo[mid], vo[mid + 1] - vo[mid]) > 0) lo = mid + 1; else hi = mid;
      }
      pass = (lo < nv && java_str_cmp(v, len, vb + vo[lo], vo[lo + 1] - vo[lo]) == 0) != excl;
    }
    r = r + r + (uint32_t)pass;
  }
  return r & valid;
}

__device__ __forceinline__ uint32_t eval_leaf(cseg_t &seg, cnode_t *__restrict__ n, uint32_t valid, const Tile &t,
                                              uint32_t &scanned) {
  const int lane = lane_id();
  const int kind = n->leaf_kind;
  if (kind == PHIP_LEAF_MATCH_ALL) return valid;
  if (kind == PHIP_LEAF_MATCH_NONE) return 0;
  if (kind == PHIP_LEAF_DOC_RANGES) {
    // SortedIndexBasedFilterOperator: inclusive doc ranges, sorted and disjoint (scalar loads)
    const PHIP_CAS int32_t *rg = (const PHIP_CAS int32_t *)n->aux;
    const int32_t cnt = n->count;
    const int32_t tile_end = t.doc0 + kTileDocs - 1;
    int a = 0, b = cnt;  // first range that may intersect the tile
    while (a < b) {
      int mid = (a + b) >> 1;
      if (rg[2 * mid + 1] < t.doc0) a = mid + 1; else b = mid;
    }
    uint32_t m = 0;
    for (int i = a; i < cnt; i++) {
      const int32_t s = rg[2 * i], e = rg[2 * i + 1];
      if (s > tile_end) break;
      m |= range_word(max(s, t.doc0) - t.doc0, min(e, tile_end) - t.doc0, lane);
    }
    return valid & m;
  }
  if (kind == PHIP_LEAF_INVERTED) {
    // dense u64 doc words (bit d%64 of word d/64), transposed into the lane-major form
    uint32_t r = 0;
    if (n->lds_off >= 0) {
      // lane L takes bit L % 32 of the u32 half (L / 32) of word g: one 32-bit LDS read, v_bfe + v_lshl_or
      const PHIP_LDS uint32_t *w = (const PHIP_LDS uint32_t *)(t.stage + n->lds_off) + (lane >> 5);
      const uint32_t sh = (uint32_t)(lane & 31);
#pragma unroll 8
      for (int g = 0; g < kTileGroups; g++) r = (r << 1) | __builtin_amdgcn_ubfe(w[2 * g], sh, 1u);
    } else {
      const PHIP_GLB uint64_t *w = (const PHIP_GLB uint64_t *)n->aux + (int64_t)(t.doc0 >> 11) * n->aux_stride;
#pragma unroll 8
      for (int g = 0; g < kTileGroups; g++) r = r + r + (uint32_t)((w[g] >> lane) & 1ull);
    }
    if (n->exclusive) r = ~r;
    return valid & r;
  }
  if (kind == PHIP_LEAF_RAW_STRING_RANGE || kind == PHIP_LEAF_RAW_STRING_SET) {
    scanned += (uint32_t)t.valid_docs;
    return eval_raw_string(seg.cols[n->column], n, valid, t);
  }
  if (kind == PHIP_LEAF_RAW_RANGE || kind == PHIP_LEAF_RAW_SET) {
    // value-based scan of a raw column (RawValueBasedPredicateEvaluator): one coalesced load per 64 docs
    scanned += (uint32_t)t.valid_docs;
    ccol_t &c = seg.cols[n->column];
    const int32_t last = t.valid_docs - 1;
    const bool real = c.type == PHIP_TYPE_FLOAT || c.type == PHIP_TYPE_DOUBLE;
    const PHIP_CAS phip_raw_range &rr = *(const PHIP_CAS phip_raw_range *)n->aux;
    const PHIP_GLB int64_t *set_i = (const PHIP_GLB int64_t *)n->aux;
    const PHIP_GLB double *set_f = (const PHIP_GLB double *)n->aux;
    const int64_t lo_i = rr.lo_int, hi_i = rr.hi_int;
    const double lo_f = rr.lo_real, hi_f = rr.hi_real;
    const bool lo_in = rr.lo_inclusive != 0, hi_in = rr.hi_inclusive != 0;
    const bool excl = n->exclusive != 0;
    uint32_t r = 0;
    for (int g = 0; g < kTileGroups; g++) {
      const int32_t doc = t.doc0 + min(g * 64 + lane, last);
      bool pass;
      if (!real) {
        const int64_t v = raw_int_at(c, doc);
        if (kind == PHIP_LEAF_RAW_RANGE) {
          pass = v >= lo_i && v <= hi_i;
        } else {
          pass = sorted_contains(set_i, n->count, v) != excl;
        }
      } else {
        const double v = raw_real_at(c, doc);
        if (kind == PHIP_LEAF_RAW_RANGE) {
          pass = (lo_in ? v >= lo_f : v > lo_f) && (hi_in ? v <= hi_f : v < hi_f);
        } else {
          pass = sorted_contains(set_f, n->count, v) != excl;
        }
      }
      r = r + r + (uint32_t)pass;
    }
    return r & valid;
  }
  // DICT_RANGE / DICT_SET on the bit-packed forward index
  scanned += (uint32_t)t.valid_docs;
  const int32_t B = n->bits;
  if (n->lds_off >= 0) {
    const PHIP_LDS uint32_t *w = (const PHIP_LDS uint32_t *)(t.stage + n->lds_off);
    uint32_t r;
    if ((kind == PHIP_LEAF_DICT_RANGE || n->small_set) && B <= 16) {
      // narrow columns: P docs per lane-window (1/P of the LDS reads), then one transpose to lane-major
      const uint32_t LO = (uint32_t)n->lo << (32 - B);
      const uint32_t SPAN = (uint32_t)(n->hi - n->lo) << (32 - B);
      const int k = kind == PHIP_LEAF_DICT_RANGE ? 0 : 1;
      if (B <= 4) r = to_lane_major<8>(conj_leaf_eval<8>(w, B, k, LO, SPAN, n->set_mask));
      else if (B <= 8) r = to_lane_major<4>(conj_leaf_eval<4>(w, B, k, LO, SPAN, n->set_mask));
      else r = to_lane_major<2>(conj_leaf_eval<2>(w, B, k, LO, SPAN, n->set_mask));
    } else if (kind == PHIP_LEAF_DICT_RANGE) {
      const uint32_t LO = (uint32_t)n->lo << (32 - B);
      const uint32_t SPAN = (uint32_t)(n->hi - n->lo) << (32 - B);
      r = scan_range(w, B, LO, SPAN);
    } else if (n->small_set) {
      r = scan_small_set(w, B, n->set_mask);
    } else if (n->count > 0 && n->count <= 64) {
      const PHIP_GLB uint32_t *set = (const PHIP_GLB uint32_t *)n->aux;
      const uint32_t myw = lane < n->count ? set[lane] : 0u;
      r = scan_lane_set(w, B, myw, n->exclusive != 0);
    } else {
      r = scan_big_set(w, B, (const PHIP_GLB uint32_t *)n->aux, n->exclusive != 0);
    }
    return r & valid;
  }
  // not staged (LDS budget exceeded): decode from HBM
  ccol_t &c = seg.cols[n->column];
  const bool is_range = kind == PHIP_LEAF_DICT_RANGE;
  const PHIP_GLB uint32_t *set = (const PHIP_GLB uint32_t *)n->aux;
  const uint32_t lo = (uint32_t)n->lo;
  const uint32_t span = (uint32_t)(n->hi - n->lo);
  const bool excl = n->exclusive != 0;
  const int32_t last = t.valid_docs - 1;
  uint32_t r = 0;
  for (int g = 0; g < kTileGroups; g++) {
    const int32_t dit = min(g * 64 + lane, last);
    const uint32_t v = decode_bits(c.words, (uint64_t)(uint32_t)(t.doc0 + dit) * (uint32_t)B, (uint32_t)B);
    bool pass;
    if (is_range) {
      pass = (v - lo) < span;
    } else if (n->small_set) {
      pass = ((n->set_mask >> v) & 1ull) != 0;
    } else {
      pass = (((set[v >> 5] >> (v & 31)) & 1u) != 0) != excl;
    }
    r = r + r + (uint32_t)pass;
  }
  return r & valid;
}

// Filter program: the segment's tree in postfix order with binary AND/OR (runtime.cpp converts the
// preorder ABI tree), evaluated once per tile over lane-major words with a small register stack.
// The first leaf of the j-th (j >= 2) child of an AND / OR carries a skip: when the running value of
// the node is already all-false (AND) / all-valid (OR) for the tile, the child is not evaluated.
#define PHIP_PUSH(v)           \
  do {                         \
    const uint32_t _v = (v);   \
    switch (sp) {              \
      case 0: s0 = _v; break;  \
      case 1: s1 = _v; break;  \
      case 2: s2 = _v; break;  \
      case 3: s3 = _v; break;  \
      case 4: s4 = _v; break;  \
      default: s5 = _v; break; \
    }                          \
    sp++;                      \
  } while (0)
#define PHIP_TOP(dst)             \
  do {                            \
    switch (sp - 1) {             \
      case 0: dst = s0; break;    \
      case 1: dst = s1; break;    \
      case 2: dst = s2; break;    \
      case 3: dst = s3; break;    \
      case 4: dst = s4; break;    \
      default: dst = s5; break;   \
    }                             \
  } while (0)
#define PHIP_POP(dst) \
  do {                \
    PHIP_TOP(dst);    \
    sp--;             \
  } while (0)

__device__ __forceinline__ uint32_t eval_filter(cseg_t &seg, cnode_t *__restrict__ nodes, uint32_t valid,
                                                const Tile &t, uint32_t &scanned) {
  uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0, s4 = 0, s5 = 0;
  int sp = 0;
  int i = seg.node_begin;
  const int end = seg.node_end;
  while (i < end) {
    cnode_t *n = nodes + i;
    const int op = n->op;
    if (op == DOP_LEAF) {
      const int sk = n->skip_kind;
      if (sk != SKIP_NONE) {
        uint32_t top;
        PHIP_TOP(top);
        const bool decided = (sk == SKIP_IF_NONE) ? (ballot(top != 0) == 0) : (ballot(top != valid) == 0);
        if (decided) {
          i = n->skip_to;
          continue;
        }
      }
      PHIP_PUSH(eval_leaf(seg, n, valid, t, scanned));
    } else if (op == DOP_NOT) {
      uint32_t v;
      PHIP_POP(v);
      PHIP_PUSH(valid & ~v);
    } else {
      uint32_t v, w;
      PHIP_POP(v);
      PHIP_POP(w);
      PHIP_PUSH(op == DOP_AND ? (v & w) : (v | w));
    }
    i++;
  }
  uint32_t r;
  PHIP_POP(r);
  return r;
}

#define PHIP_B_CASES(X) \
  X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16) \
  X(17) X(18) X(19) X(20) X(21) X(22) X(23) X(24) X(25) X(26) X(27) X(28) X(29) X(30) X(31)

// ------------------------------------------------------------------------------------------------
// Contiguous layout for general programs (seg.contig). Lane L owns docs 32L .. 32L+31 of the tile, doc
// 32L + j at bit 31 - j. In this layout an inverted leaf's dense doc words ARE the lane words (u32 half L
// of the tile's 32 u64 words, bit-reversed: one LDS read), a scan leaf's 32 docs are exactly B consecutive
// words of the staged forward index (read once into registers, fields cut at compile-time offsets), and
// AND / OR / NOT stay one VALU op. Boolean algebra does not care about the bit order, so the program runs
// entirely in this layout; only a mask that leaves the kernel is permuted to lane-major once
// (contig_to_lane_major). The lane-major evaluator above transposes every inverted leaf and decodes every
// scan leaf 64 docs at a time -- the instruction count that bounded config C4.
// ------------------------------------------------------------------------------------------------
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t contig_valid(int32_t valid_docs, int lane) {
  const int32_t n = valid_docs - 32 * lane;
  return n >= 32 ? ~0u : (n <= 0 ? 0u : (~0u << (32 - n)));
}

// lane-major (bit 31-g of lane l = doc 64g + l) from contiguous: lane 32h + g first takes the word of
// contiguous lane 2g + h (its bit 31-i = doc 64g + 32h + i), then each 32-lane half transposes its 32x32 bit
// matrix (Hacker's Delight transpose32 with rows = lanes, 5 butterfly stages over ds_bpermute).
__device__ __forceinline__ uint32_t contig_to_lane_major(uint32_t c) {
  const int lane = lane_id();
  return transpose_halves((uint32_t)__builtin_amdgcn_ds_bpermute(((2 * (lane & 31)) | (lane >> 5)) << 2, (int)c));
}

// One scan leaf over the lane's 32 docs: the B staged words of those docs in registers, field j cut from
// words (jB)/32, (jB)/32 + 1 at a compile-time shift. KIND 0: dict-id range (v_sub / v_cmp / v_addc, as in
// conj_range); 1: set of a <= 64-entry dictionary (64-bit mask); 2: set of a <= 2048-entry dictionary spread
// over the wave (ds_bpermute per doc).
// docs [J0, J0 + NJ) of the lane: their words (fields at compile-time offsets) in registers, then the test
template <int B, int KIND, int J0, int NJ>
__device__ __forceinline__ uint32_t contig_docs(const PHIP_LDS uint32_t *wl, uint32_t r, uint32_t LO, uint32_t SPAN,
                                                uint64_t set, uint32_t myw, bool excl) {
  constexpr int W0 = (J0 * B) >> 5;                    // first word of the docs
  constexpr int W1 = ((J0 + NJ) * B - 1) >> 5;         // last word
  constexpr int NW = W1 - W0 + 1;
  uint32_t x[NW + 1];
  if constexpr (W0 == 0 && NW == B && B % 4 == 0) {
#pragma unroll
    for (int q = 0; q < B / 4; q++) {
      const u32x4_t v = ((const PHIP_LDS u32x4_t *)wl)[q];
      x[4 * q] = v[0];
      x[4 * q + 1] = v[1];
      x[4 * q + 2] = v[2];
      x[4 * q + 3] = v[3];
    }
  } else if constexpr (W0 == 0 && NW == B && B % 2 == 0) {
#pragma unroll
    for (int q = 0; q < B / 2; q++) {
      const u32x2_t v = ((const PHIP_LDS u32x2_t *)wl)[q];
      x[2 * q] = v[0];
      x[2 * q + 1] = v[1];
    }
  } else {
#pragma unroll
    for (int q = 0; q < NW; q++) x[q] = wl[W0 + q];
  }
  x[NW] = 0u;  // only ever supplies the bits below a field
#pragma unroll
  for (int j = J0; j < J0 + NJ; j++) {
    const int o = (j * B) & 31, k = ((j * B) >> 5) - W0;
    const uint32_t win = o == 0 ? x[k] : __builtin_amdgcn_alignbit(x[k], x[k + 1], 32 - o);
    if constexpr (KIND == 0) {
      uint32_t d;
      asm("v_sub_u32 %[d], %[w], %[lo]\n\t"
          "v_cmp_gt_u32 vcc, %[sp], %[d]\n\t"
          "v_addc_co_u32 %[r], vcc, %[r], %[r], vcc"
          : [r] "+v"(r), [d] "=&v"(d)
          : [w] "v"(win), [lo] "s"(LO), [sp] "s"(SPAN)
          : "vcc");
    } else if constexpr (KIND == 1) {
      r = r + r + (uint32_t)((set >> (win >> (32 - B))) & 1ull);
    } else {
      const uint32_t id = win >> (32 - B);
      const uint32_t word = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((id >> 5) << 2), (int)myw);
      r = r + r + (((word >> (id & 31)) & 1u) ^ (excl ? 1u : 0u));
    }
  }
  return r;
}

// One scan leaf over the lane's 32 docs: the B staged words of those docs (words 32L*B/32 .. of the tile)
// read into registers -- all at once up to 16 bits, in two halves of 16 docs above (VGPR budget) -- and
// every field cut at a compile-time shift. KIND 0: dict-id range (v_sub / v_cmp / v_addc, as in
// conj_range); 1: set of a <= 64-entry dictionary (64-bit mask); 2: set of a <= 2048-entry dictionary spread
// over the wave (ds_bpermute per doc).
template <int B, int KIND>
__device__ __forceinline__ uint32_t contig_scan(const PHIP_LDS uint32_t *w, uint32_t LO, uint32_t SPAN, uint64_t set,
                                                uint32_t myw, bool excl) {
  const PHIP_LDS uint32_t *wl = w + lane_id() * B;
  if constexpr (B <= 16) {
    return contig_docs<B, KIND, 0, 32>(wl, 0u, LO, SPAN, set, myw, excl);
  } else {
    const uint32_t r = contig_docs<B, KIND, 0, 16>(wl, 0u, LO, SPAN, set, myw, excl);
    return contig_docs<B, KIND, 16, 16>(wl, r, LO, SPAN, set, myw, excl);
  }
}

// The width / kind dispatch of the set kinds as a real call: all 93 unrolled bodies inlined pushed the filter
// kernel past the VGPR budget (spills on every tile). The 31 range bodies alone fit without spills and are
// inlined (eval_leaf_contig): the call saves and restores its VGPRs through scratch on every tile.
__device__ __noinline__ uint32_t contig_scan_any(const PHIP_LDS uint32_t *w, int B, int k, uint32_t LO, uint32_t SPAN,
                                                 uint64_t set, uint32_t myw, bool excl) {
  switch (B) {
#define PHIP_CC(b)                                                                  \
  case b:                                                                           \
    return k == 0 ? contig_scan<b, 0>(w, LO, SPAN, set, myw, excl)                  \
                  : (k == 1 ? contig_scan<b, 1>(w, LO, SPAN, set, myw, excl)       \
                            : contig_scan<b, 2>(w, LO, SPAN, set, myw, excl));
    PHIP_B_CASES(PHIP_CC)
#undef PHIP_CC
  }
  return 0u;
}

__device__ __forceinline__ uint32_t eval_leaf_contig(cseg_t &seg, cnode_t *__restrict__ n, uint32_t valid,
                                                     const Tile &t, uint32_t &scanned, bool inl) {
  const int lane = lane_id();
  const int kind = n->leaf_kind;
  if (kind == PHIP_LEAF_MATCH_ALL) return valid;
  if (kind == PHIP_LEAF_MATCH_NONE) return 0;
  if (kind == PHIP_LEAF_DOC_RANGES) {
    const PHIP_CAS int32_t *rg = (const PHIP_CAS int32_t *)n->aux;
    const int32_t cnt = n->count;
    const int32_t tile_end = t.doc0 + kTileDocs - 1;
    int a = 0, b = cnt;
    while (a < b) {
      int mid = (a + b) >> 1;
      if (rg[2 * mid + 1] < t.doc0) a = mid + 1; else b = mid;
    }
    const int32_t l0 = 32 * lane, l1 = l0 + 31;  // the lane's tile-relative docs
    uint32_t m = 0;
    for (int i = a; i < cnt; i++) {
      const int32_t s = rg[2 * i], e = rg[2 * i + 1];
      if (s > tile_end) break;
      const int32_t lo = max(max(s, t.doc0) - t.doc0, l0), hi = min(min(e, tile_end) - t.doc0, l1);
      if (lo <= hi) m |= span32(31 - (hi - l0), 31 - (lo - l0));
    }
    return valid & m;
  }
  if (kind == PHIP_LEAF_INVERTED) {  // staged (the host only picks this layout then)
    const uint32_t w = ((const PHIP_LDS uint32_t *)(t.stage + n->lds_off))[lane];
    uint32_t r = __builtin_bitreverse32(w);  // bit j of the u32 half = doc 32L + j
    if (n->exclusive) r = ~r;
    return valid & r;
  }
  // DICT_RANGE / DICT_SET staged scan leaves
  scanned += (uint32_t)t.valid_docs;
  const int32_t B = n->bits;
  const PHIP_LDS uint32_t *w = (const PHIP_LDS uint32_t *)(t.stage + n->lds_off);
  const uint32_t LO = (uint32_t)n->lo << (32 - B);
  const uint32_t SPAN = (uint32_t)(n->hi - n->lo) << (32 - B);
  const int k = kind == PHIP_LEAF_DICT_RANGE ? 0 : (n->small_set ? 1 : 2);
  if (inl && k == 0) {  // range scans inline (no call: its VGPR save / restore goes through scratch)
    switch (B) {
#define PHIP_CI(b) \
  case b: return contig_scan<b, 0>(w, LO, SPAN, 0ull, 0u, false) & valid;
      PHIP_B_CASES(PHIP_CI)
#undef PHIP_CI
    }
  }
  const uint32_t myw = (k == 2 && lane < n->count) ? ((const PHIP_GLB uint32_t *)n->aux)[lane] : 0u;
  return contig_scan_any(w, B, k, LO, SPAN, n->set_mask, myw, n->exclusive != 0) & valid;
}

// The operand stack is a shift register (s0 = top): a push / pop is a handful of v_mov, not a scalar branch
// tree on the stack pointer -- the interpreter's SALU / branch count per tile is what bounds this path.
__device__ __forceinline__ uint32_t eval_filter_contig(cseg_t &seg, cnode_t *__restrict__ nodes, uint32_t valid,
                                                       const Tile &t, uint32_t &scanned, bool inl) {
  uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0, s4 = 0, s5 = 0;
  int i = seg.node_begin;
  const int end = seg.node_end;
  while (i < end) {
    cnode_t *n = nodes + i;
    const int op = n->op;
    if (op == DOP_LEAF) {
      const int sk = n->skip_kind;
      if (sk != SKIP_NONE) {
        const bool decided = (sk == SKIP_IF_NONE) ? (ballot(s0 != 0) == 0) : (ballot(s0 != valid) == 0);
        if (decided) {
          i = n->skip_to;
          continue;
        }
      }
      const uint32_t v = eval_leaf_contig(seg, n, valid, t, scanned, inl);
      s5 = s4;
      s4 = s3;
      s3 = s2;
      s2 = s1;
      s1 = s0;
      s0 = v;
    } else if (op == DOP_NOT) {
      s0 = valid & ~s0;
    } else {
      s0 = op == DOP_AND ? (s0 & s1) : (s0 | s1);
      s1 = s2;
      s2 = s3;
      s3 = s4;
      s4 = s5;
    }
    i++;
  }
  return s0;
}

// ------------------------------------------------------------------------------------------------
// conjunctive fast path: AND of staged scan leaves, each a width-specialised loop.
//
// P-layout. With P docs per lane-window (P * B <= 32), lane l reads ONE 32-bit window per 64P docs and
// tests its P consecutive docs from it: bit i (MSB first) of the lane's word is doc
// 64P*(i/P) + P*l + (i%P) of the tile. That cuts the LDS reads of a leaf from 32 to 32/P per tile
// (ds_read2_b32 at compile-time offsets); the range test is v_sub + v_cmp into VCC + v_addc, which
// shifts the predicate bit into the word in one instruction. After the AND of all leaves the word is
// permuted once into the lane-major tile layout (to_lane_major).
// ------------------------------------------------------------------------------------------------
template <int B, int P>
__device__ __forceinline__ uint32_t conj_range(const PHIP_LDS uint32_t *wl, uint32_t s, uint32_t LO, uint32_t SPAN) {
  constexpr int NK = kTileGroups / P;  // P-groups (64P docs) per tile
  constexpr int STRIDE = 2 * P * B;    // words per P-group
  constexpr int NB = NK < 8 ? NK : 8;  // loads issued ahead of each compare block
  uint32_t r = 0;
#pragma unroll
  for (int k0 = 0; k0 < NK; k0 += NB) {
    uint32_t x[NB], y[NB];
#pragma unroll
    for (int k = 0; k < NB; k++) {
      x[k] = wl[(k0 + k) * STRIDE];
      y[k] = wl[(k0 + k) * STRIDE + 1];
    }
#pragma unroll
    for (int k = 0; k < NB; k++) {
      const uint32_t win = __builtin_amdgcn_alignbit(x[k], y[k], s);
#pragma unroll
      for (int j = 0; j < P; j++) {
        // field j moved to the top and offset by -LO in one v_lshl_add_u32 (3 VALU per doc, not 4)
        uint32_t d;
        if (j == 0) {
          asm("v_sub_u32 %[d], %[w], %[lo]\n\t"
              "v_cmp_gt_u32 vcc, %[sp], %[d]\n\t"
              "v_addc_co_u32 %[r], vcc, %[r], %[r], vcc"
              : [r] "+v"(r), [d] "=&v"(d)
              : [w] "v"(win), [lo] "s"(LO), [sp] "s"(SPAN)
              : "vcc");
        } else {
          asm("v_lshl_add_u32 %[d], %[w], %[sh], %[nlo]\n\t"
              "v_cmp_gt_u32 vcc, %[sp], %[d]\n\t"
              "v_addc_co_u32 %[r], vcc, %[r], %[r], vcc"
              : [r] "+v"(r), [d] "=&v"(d)
              : [w] "v"(win), [sh] "i"(j * B), [nlo] "s"(0u - LO), [sp] "s"(SPAN)
              : "vcc");
        }
      }
    }
  }
  return r;
}

template <int B, int P>
__device__ __forceinline__ uint32_t conj_set(const PHIP_LDS uint32_t *wl, uint32_t s, uint64_t set) {
  constexpr int NK = kTileGroups / P;
  constexpr int STRIDE = 2 * P * B;
  constexpr int NB = NK < 8 ? NK : 8;
  uint32_t r = 0;
#pragma unroll
  for (int k0 = 0; k0 < NK; k0 += NB) {
    uint32_t x[NB], y[NB];
#pragma unroll
    for (int k = 0; k < NB; k++) {
      x[k] = wl[(k0 + k) * STRIDE];
      y[k] = wl[(k0 + k) * STRIDE + 1];
    }
#pragma unroll
    for (int k = 0; k < NB; k++) {
      const uint32_t win = __builtin_amdgcn_alignbit(x[k], y[k], s);
#pragma unroll
      for (int j = 0; j < P; j++) {
        const uint32_t f = j == 0 ? win : (win << (j * B));
        r = r + r + (uint32_t)((set >> (f >> (32 - B))) & 1ull);
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // bound the loads in flight (registers -> resident waves)
  }
  return r;
}


// The lane's first word and window shift are computed once from the runtime width, so the
// specialisations share them instead of each hoisting its own copy out of the tile loop.
template <int P>
__device__ __forceinline__ uint32_t conj_leaf_eval(const PHIP_LDS uint32_t *w, int bits, int kind, uint32_t lo,
                                                uint32_t span, uint64_t set) {
  const int32_t p = lane_id() * P * bits;
  const int32_t q = (p - 1) >> 5;
  const uint32_t s = (uint32_t)(32 * (q + 1) - p);
  const PHIP_LDS uint32_t *wl = w + q;
  if (kind == 0) {
    switch (bits) {
#define PHIP_RC(b)                                                     \
  case b:                                                              \
    if constexpr (b * P <= 32) return conj_range<b, P>(wl, s, lo, span); \
    break;
      PHIP_B_CASES(PHIP_RC)
#undef PHIP_RC
    }
  } else {
    switch (bits) {
#define PHIP_SC(b)                                                \
  case b:                                                         \
    if constexpr (b * P <= 32) return conj_set<b, P>(wl, s, set); \
    break;
      PHIP_B_CASES(PHIP_SC)
#undef PHIP_SC
    }
  }
  return 0;
}

// P-layout word -> lane-major word (bit 31-g of lane L = doc 64g + L). Group g = kP + c of lane L comes
// from lane (64/P)c + L/P, bit index kP + (L % P): one ds_bpermute per c, then a mask and a shift.
template <int P>
__device__ __forceinline__ uint32_t to_lane_major(uint32_t r) {
  if constexpr (P == 1) {
    return r;
  } else {
    const int L = lane_id();
    const int j = L & (P - 1);
    constexpr uint32_t kBase = P == 2 ? 0xAAAAAAAAu : (P == 4 ? 0x88888888u : 0x80808080u);
    const uint32_t mj = kBase >> j;  // bits with index = j (mod P), index 0 = bit 31
    uint32_t out = 0;
#pragma unroll
    for (int c = 0; c < P; c++) {
      const int src = (64 / P) * c + (L / P);
      const uint32_t t = (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)r) & mj;
      const int d = c - j;
      out |= d >= 0 ? (t >> d) : (t << (-d));
    }
    return out;
  }
}

// Leaves 2.. of a tile whose first leaf passed at most seg.conj_sparse docs in every lane: each passing doc is
// tested against the remaining range leaves on its own (one window read per leaf), the way
// SVScanDocIdIterator.applyAnd (pinot-core/.../dociditerators/SVScanDocIdIterator.java:114-142) scans
// only the candidate docs of the preceding AND children. Lanes loop over their set bits together.

template <int P>
__device__ __forceinline__ uint32_t conj_sparse_rest(cseg_t &seg, const PHIP_LDS uint8_t *slot, uint32_t r) {
  const int k = seg.conj;
  int32_t off[kMaxConj - 1], bits[kMaxConj - 1];
  uint32_t lo[kMaxConj - 1], span[kMaxConj - 1];
#pragma unroll
  for (int j = 0; j < kMaxConj - 1; j++) {
    off[j] = 0;
    bits[j] = 1;
    lo[j] = 0;
    span[j] = 0xffffffffu;
    if (j + 1 < k) {
      off[j] = seg.conj_leaf[j + 1].lds_off;
      bits[j] = seg.conj_leaf[j + 1].bits;
      lo[j] = seg.conj_leaf[j + 1].lo;
      span[j] = seg.conj_leaf[j + 1].span;
    }
  }
  const int lane = lane_id();
  uint32_t todo = r;
  while (ballot(todo != 0)) {
    if (todo != 0) {
      const int i = __builtin_clz(todo);
      const uint32_t bit = 0x80000000u >> i;
      todo &= ~bit;
      const int32_t d = 64 * P * (i / P) + P * lane + (i % P);  // tile-relative doc of bit i (P-layout)
      bool pass = true;
#pragma unroll
      for (int j = 0; j < kMaxConj - 1; j++) {
        if (j + 1 < k) {
          const uint32_t win = window_at((const PHIP_LDS uint32_t *)(slot + off[j]), d * bits[j]);
          pass = pass && ((win - lo[j]) < span[j]);
        }
      }
      if (!pass) r &= ~bit;
    }
  }
  return r;
}

template <int P>
__device__ __forceinline__ uint32_t eval_conj_p(cseg_t &seg, const PHIP_LDS uint8_t *slot) {
  const int k = seg.conj;
  const PHIP_CAS ConjLeaf &L0 = seg.conj_leaf[0];
  uint32_t r = conj_leaf_eval<P>((const PHIP_LDS uint32_t *)(slot + L0.lds_off), L0.bits, L0.kind, L0.lo, L0.span,
                                 L0.set_mask);
  if (k > 1) {
    if (seg.conj_sparse && wave_max_u32((uint32_t)__popc(r)) <= (uint32_t)seg.conj_sparse) {
      r = conj_sparse_rest<P>(seg, slot, r);
    } else {
      for (int i = 1; i < k; i++) {
        if (ballot(r != 0) == 0) break;  // every doc already rejected (AndDocIdSet short-circuit)
        const PHIP_CAS ConjLeaf &L = seg.conj_leaf[i];
        r &= conj_leaf_eval<P>((const PHIP_LDS uint32_t *)(slot + L.lds_off), L.bits, L.kind, L.lo, L.span,
                               L.set_mask);
      }
    }
  }
  return to_lane_major<P>(r);
}

// Bit-sliced range leaf (ConjLeaf kind 2) over the lane's B plane words, most significant plane first: x >= lo and
// x <= hi for the lane's 32 docs at once, comparing MSB first (gt / eq and lt / eq flags, BitWeaving/V). The
// bounds are wave-uniform, so each plane costs one or two bitwise ops per side; lo == hi is an equality (one op per
// plane).
template <int B>
__device__ __forceinline__ uint32_t bs_range(const PHIP_LDS uint32_t *pl, uint32_t lo, uint32_t hi, int sides) {
  const int lane = lane_id();
  uint32_t x[B];
#pragma unroll
  for (int k = 0; k < B; k++) x[k] = pl[64 * k + lane];
  if (sides == 3 && lo == hi) {
    uint32_t eq = ~0u;
#pragma unroll
    for (int k = 0; k < B; k++) eq &= ((lo >> (B - 1 - k)) & 1u) ? x[k] : ~x[k];
    return eq;
  }
  uint32_t r = ~0u;
  if (sides & 1) {  // x >= lo
    uint32_t gt = 0u, eq = ~0u;
#pragma unroll
    for (int k = 0; k < B; k++) {
      if ((lo >> (B - 1 - k)) & 1u) {
        eq &= x[k];
      } else {
        gt |= eq & x[k];
        eq &= ~x[k];
      }
    }
    r = gt | eq;
  }
  if (sides & 2) {  // x <= hi
    uint32_t lt = 0u, eq = ~0u;
#pragma unroll
    for (int k = 0; k < B; k++) {
      if ((hi >> (B - 1 - k)) & 1u) {
        lt |= eq & ~x[k];
        eq &= x[k];
      } else {
        eq &= ~x[k];
      }
    }
    r &= lt | eq;
  }
  return r;
}

// a few ids (set bits of `set`, wave-uniform): OR of equalities
template <int B>
__device__ __forceinline__ uint32_t bs_set(const PHIP_LDS uint32_t *pl, uint64_t set) {
  const int lane = lane_id();
  uint32_t x[B];
#pragma unroll
  for (int k = 0; k < B; k++) x[k] = pl[64 * k + lane];
  uint32_t r = 0u;
  while (set) {
    const uint32_t id = (uint32_t)__builtin_ctzll(set);
    set &= set - 1;
    uint32_t eq = ~0u;
#pragma unroll
    for (int k = 0; k < B; k++) eq &= ((id >> (B - 1 - k)) & 1u) ? x[k] : ~x[k];
    r |= eq;
  }
  return r;
}

// OR of n <= 4 runs of ids (ConjLeaf kind 4: runs 0 / 1 in the two halves of `set`, run 2 in lo, run 3 in hi; a run
// is [r & 0xffff, r >> 16]): one plane load, each run an equality or a two-sided BitWeaving/V comparison.
template <int B>
__device__ __forceinline__ uint32_t bs_runs(const PHIP_LDS uint32_t *pl, uint64_t set, uint32_t r2, uint32_t r3, int n) {
  const int lane = lane_id();
  uint32_t x[B];
#pragma unroll
  for (int k = 0; k < B; k++) x[k] = pl[64 * k + lane];
  uint32_t res = 0u;
  for (int j = 0; j < n; j++) {
    const uint32_t run = j == 0 ? (uint32_t)set : (j == 1 ? (uint32_t)(set >> 32) : (j == 2 ? r2 : r3));
    const uint32_t a = run & 0xffffu, b = run >> 16;
    uint32_t gt = 0u, lt = 0u, eqa = ~0u, eqb = ~0u;
#pragma unroll
    for (int k = 0; k < B; k++) {
      const uint32_t ba = (a >> (B - 1 - k)) & 1u, bb = (b >> (B - 1 - k)) & 1u;
      if (ba) eqa &= x[k];
      else { gt |= eqa & x[k]; eqa &= ~x[k]; }
      if (bb) { lt |= eqb & ~x[k]; eqb &= x[k]; }
      else eqb &= ~x[k];
    }
    res |= (gt | eqa) & (lt | eqb);  // a <= x <= b
  }
  return res;
}

__device__ __forceinline__ uint32_t bs_range_any(const PHIP_LDS uint32_t *pl, int bits, uint32_t lo, uint32_t hi,
                                              int sides, int kind, uint64_t set) {
  switch (bits) {
#define PHIP_BSR(b) \
  case b: return kind == 4 ? bs_runs<b>(pl, set, lo, hi, sides) \
               : kind == 3 ? bs_set<(b < 7 ? b : 6)>(pl, set) : bs_range<b>(pl, lo, hi, sides);
    PHIP_BSR(1) PHIP_BSR(2) PHIP_BSR(3) PHIP_BSR(4) PHIP_BSR(5) PHIP_BSR(6) PHIP_BSR(7) PHIP_BSR(8) PHIP_BSR(9)
    PHIP_BSR(10) PHIP_BSR(11) PHIP_BSR(12)
#undef PHIP_BSR
  }
  return 0u;
}

// AND of the bit-sliced range leaves, already lane-major (no transpose)
__device__ __forceinline__ uint32_t eval_conj_bs(cseg_t &seg, const PHIP_LDS uint8_t *slot) {
  uint32_t r = ~0u;
  for (int i = 0; i < seg.conj; i++) {
    const PHIP_CAS ConjLeaf &L = seg.conj_leaf[i];
    r &= bs_range_any((const PHIP_LDS uint32_t *)(slot + L.lds_off), L.bits, L.lo, L.span, L.pad, L.kind, L.set_mask);
    if (ballot(r != 0) == 0) break;  // every doc already rejected (AndDocIdSet short-circuit)
  }
  return r;
}

__device__ __forceinline__ uint32_t eval_conj(cseg_t &seg, const PHIP_LDS uint8_t *slot, uint32_t valid) {
  if (seg.conj_bs) return valid & eval_conj_bs(seg, slot);
  switch (seg.conj_p) {
    case 8: return valid & eval_conj_p<8>(seg, slot);
    case 4: return valid & eval_conj_p<4>(seg, slot);
    case 2: return valid & eval_conj_p<2>(seg, slot);
    default: return valid & eval_conj_p<1>(seg, slot);
  }
}

// ------------------------------------------------------------------------------------------------
// fused projection + aggregation (conjunctive programs without group-by / HLL). After a tile's mask is
// known its matched docs are compacted into a per-wave LDS ring in doc order (the mask transposed to the
// contiguous layout, lane ranks from a wave prefix sum, as the aggregation kernel does) and projected
// kFusedBatch x 64 at a time with every load of the batch issued before the first use, so a sparse tile costs
// one gather round trip. Columns staged in the tile's ring slot (the filter columns, and value columns the host
// chose to stream) are read from LDS by tile-relative doc, so the ring is drained at the end of the tile.
// Dictionaries of <= 64 entries live one entry per lane (loaded when the wave enters a segment) and are read
// with ds_bpermute; larger ones are gathered from HBM -- the aggregation kernel's walk without the mask round
// trip, the re-read of the filter columns and a second launch.
// ------------------------------------------------------------------------------------------------
#ifndef PHIP_FUSED_BATCH
#define PHIP_FUSED_BATCH 4  // (A/B builds override it)
#endif
constexpr int kFusedBatch = PHIP_FUSED_BATCH;  // 64-doc chunks per gather round trip

// The lane's share of a small dictionary: entry `lane` (64-bit image of the value), or 0.
struct SmallDict {
  uint32_t lo, hi;
  bool on;
};

__device__ __forceinline__ SmallDict load_small_dict(ccol_t &c) {
  SmallDict d{0u, 0u, false};
  if (!c.has_dict || c.card > 64 || c.type == PHIP_TYPE_STRING) return d;
  d.on = true;
  const int lane = lane_id();
  if (lane < c.card) {
    if (c.type == PHIP_TYPE_INT || c.type == PHIP_TYPE_FLOAT) {
      d.lo = ((const PHIP_GLB uint32_t *)c.dict)[lane];
    } else {
      const uint64_t v = ((const PHIP_GLB uint64_t *)c.dict)[lane];
      d.lo = (uint32_t)v;
      d.hi = (uint32_t)(v >> 32);
    }
  }
  return d;
}

// dict id of tile-relative doc td: from the staged words (LDS) or the forward index in HBM (always HBM for the
// deferred walk: its docs come from tiles whose ring slots are gone)
template <bool kHbm = false>
__device__ __forceinline__ uint32_t fused_id(ccol_t &c, const Tile &t, int32_t td) {
  const uint32_t b = (uint32_t)c.bits;
  if (!kHbm && c.lds_off >= 0)
    return window_at((const PHIP_LDS uint32_t *)(t.stage + c.lds_off), td * (int32_t)b) >> (32 - b);
  return decode_bits(c.words, (uint64_t)(uint32_t)(t.doc0 + td) * b, b);
}

// a packed doc-order value (DevCol.vpack) streamed with the tile (the runtime stages the packed words like ids)
__device__ __forceinline__ int64_t fused_packed(ccol_t &c, const Tile &t, int32_t td) {
  const uint32_t b = (uint32_t)c.vbits;
  return c.vbase + (int64_t)(window_at((const PHIP_LDS uint32_t *)(t.stage + c.lds_off), td * (int32_t)b) >> (32 - b));
}

__device__ __forceinline__ uint64_t small_dict_bits(const SmallDict &sd, uint32_t id, bool wide) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(id << 2), (int)sd.lo);
  if (!wide) return lo;
  return ((uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute((int)(id << 2), (int)sd.hi) << 32) | lo;
}

// values of U docs as double: ids of all U first, then all U value loads (one round trip each)
template <int U, bool kHbm>
__device__ __forceinline__ void fused_f64_u(ccol_t &c, const SmallDict &sd, const Tile &t, const int32_t (&td)[U],
                                            double (&v)[U]) {
  if (!c.has_dict) {
    if (!kHbm && c.lds_off >= 0) {
#pragma unroll
      for (int u = 0; u < U; u++) v[u] = (double)fused_packed(c, t, td[u]);
      return;
    }
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = raw_f64(c, t.doc0 + td[u]);
    return;
  }
  uint32_t id[U];
#pragma unroll
  for (int u = 0; u < U; u++) id[u] = fused_id<kHbm>(c, t, td[u]);
  const int ty = c.type;
  if (sd.on) {
    const bool wide = ty == PHIP_TYPE_LONG || ty == PHIP_TYPE_DOUBLE;
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t x = small_dict_bits(sd, id[u], wide);
      v[u] = ty == PHIP_TYPE_INT ? (double)(int32_t)(uint32_t)x
           : ty == PHIP_TYPE_FLOAT ? (double)__uint_as_float((uint32_t)x)
           : ty == PHIP_TYPE_LONG ? (double)(int64_t)x : __longlong_as_double((long long)x);
    }
    return;
  }
  switch (ty) {
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
}

template <int U, bool kHbm>
__device__ __forceinline__ void fused_i64_u(ccol_t &c, const SmallDict &sd, const Tile &t, const int32_t (&td)[U],
                                            int64_t (&v)[U]) {
  if (!c.has_dict) {
    if (!kHbm && c.lds_off >= 0) {
#pragma unroll
      for (int u = 0; u < U; u++) v[u] = fused_packed(c, t, td[u]);
      return;
    }
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = raw_i64(c, t.doc0 + td[u]);
    return;
  }
  uint32_t id[U];
#pragma unroll
  for (int u = 0; u < U; u++) id[u] = fused_id<kHbm>(c, t, td[u]);
  const int ty = c.type;
  if (sd.on) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t x = small_dict_bits(sd, id[u], ty != PHIP_TYPE_INT);
      v[u] = ty == PHIP_TYPE_INT ? (int64_t)(int32_t)(uint32_t)x : (int64_t)x;  // (integral sums: INT / LONG only)
    }
    return;
  }
  switch (ty) {
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
}

// U chunks of matched docs of the current tile (chunk u: lane's tile-relative doc td[u], active if bit u of act)
template <int NA, int U, bool kHbm>
__device__ __forceinline__ void fused_batch(cquery_t &aq, cseg_t &seg, const Tile &t, const int32_t (&td)[U], uint32_t act,
                                            const SmallDict (&sda)[NA], const SmallDict (&sdb)[NA],
                                            uint64_t (&acc)[NA]) {
#pragma unroll
  for (int a = 0; a < NA; a++) {
    if (a >= aq.num_aggs) break;
    cagg_t &ag = aq.aggs[a];
    const int kind = ag.acc;
    if (kind == ACC_COUNT) {
      acc[a] += (uint64_t)__popc(act);
      continue;
    }
    ccol_t &ca = seg.cols[ag.col_a];
    if (kind == ACC_SUM_I64) {
      int64_t x[U];
      fused_i64_u<U, kHbm>(ca, sda[a], t, td, x);
      if (ag.expr != PHIP_EXPR_COLUMN) {
        int64_t y[U];
        fused_i64_u<U, kHbm>(seg.cols[ag.col_b], sdb[a], t, td, y);
#pragma unroll
        for (int u = 0; u < U; u++)
          x[u] = ag.expr == PHIP_EXPR_ADD ? x[u] + y[u] : (ag.expr == PHIP_EXPR_SUB ? x[u] - y[u] : x[u] * y[u]);
      }
#pragma unroll
      for (int u = 0; u < U; u++) acc[a] += ((act >> u) & 1u) ? (uint64_t)x[u] : 0ull;
    } else {
      double x[U];
      fused_f64_u<U, kHbm>(ca, sda[a], t, td, x);
      if (ag.expr != PHIP_EXPR_COLUMN) {
        double y[U];
        fused_f64_u<U, kHbm>(seg.cols[ag.col_b], sdb[a], t, td, y);
#pragma unroll
        for (int u = 0; u < U; u++)
          x[u] = ag.expr == PHIP_EXPR_ADD ? x[u] + y[u] : (ag.expr == PHIP_EXPR_SUB ? x[u] - y[u] : x[u] * y[u]);
      }
      double cur = as_f64(acc[a]);
#pragma unroll
      for (int u = 0; u < U; u++) {
        const bool on = (act >> u) & 1u;
        if (kind == ACC_SUM_F64) cur = cur + (on ? x[u] : 0.0);
        else if (kind == ACC_MIN_F64) cur = fmin(cur, on ? x[u] : __builtin_huge_val());
        else cur = fmax(cur, on ? x[u] : -__builtin_huge_val());
      }
      acc[a] = as_u64(cur);
    }
  }
}

// A tile's matched docs ranked by the wave prefix (DPP scan) of the lanes' popcounts: lane-major (lane l: docs
// 64g + l) for a few matches, transposed to doc order (lane L: docs 32L .. 32L+31) from a batch on.
struct TileRank {
  uint32_t w;     // the lane's docs, bit 31-j = doc base + step * j
  uint32_t excl;  // the lane's first rank
  uint32_t incl;
  int32_t base;   // tile-relative doc of bit 31
  int32_t step;
  int total;
};
__device__ __forceinline__ TileRank rank_tile(uint32_t mask) {
  const int lane = lane_id();
  TileRank r;
  r.w = mask;
  uint32_t cnt = (uint32_t)__popc(mask);
  r.incl = wave_incl_scan(cnt);
  r.total = __builtin_amdgcn_readlane((int)r.incl, 63);
  r.base = lane;
  r.step = 64;
  if (r.total >= 64 * kFusedBatch) {
    r.w = lane_major_to_contig(mask);
    cnt = (uint32_t)__popc(r.w);
    r.incl = wave_incl_scan(cnt);
    r.base = 32 * lane;
    r.step = 1;
  }
  r.excl = r.incl - cnt;
  return r;
}

// the docs of lanes [l0, l1) at their ranks - sub, plus `add`
template <typename T, int RING>
__device__ __forceinline__ void write_ranked(const TileRank &r, int l0, int l1, int sub, int32_t add, PHIP_LDS T *ring) {
  const int lane = lane_id();
  if (lane >= l0 && lane < l1) {
    uint32_t w = r.w;
    int pos = (int)r.excl - sub;
    while (w) {
      const int j = __builtin_clz(w);
      w &= ~(0x80000000u >> j);
      ring[pos & (RING - 1)] = (T)(add + r.base + r.step * j);
      pos++;
    }
  }
}

// per-tile mode: the tile's docs read from its ring slot (streamed value columns), drained before the next tile
template <int NA>
__device__ __forceinline__ void fused_tile(cquery_t &aq, cseg_t &seg, const Tile &t, uint32_t mask,
                                           PHIP_LDS uint16_t *ring, const SmallDict (&sda)[NA],
                                           const SmallDict (&sdb)[NA], uint64_t (&acc)[NA]) {
  if (ballot(mask != 0) == 0) return;
  const int lane = lane_id();
  const TileRank r = rank_tile(mask);
  // the whole tile at once when it fits the ring, else quarter tiles (16 lanes, <= 512 docs)
  const int npiece = r.total <= kFusedRingTile ? 1 : 4;
  const int lanes = 64 / npiece;
  for (int p = 0; p < npiece; p++) {
    const int s = p == 0 ? 0 : __builtin_amdgcn_readlane((int)r.incl, lanes * p - 1);
    const int e = __builtin_amdgcn_readlane((int)r.incl, lanes * p + lanes - 1);
    if (e == s) continue;
    write_ranked<uint16_t, kFusedRingTile>(r, lanes * p, lanes * (p + 1), s, 0, ring);
    const int n = e - s;
    for (int c = 0; c < n; c += 64 * kFusedBatch) {
      int32_t td[kFusedBatch];
      uint32_t act = 0;
#pragma unroll
      for (int u = 0; u < kFusedBatch; u++) {
        const bool on = c + 64 * u + lane < n;
        td[u] = on ? (int32_t)ring[c + 64 * u + lane] : 0;
        act |= on ? (1u << u) : 0u;
      }
      fused_batch<NA, kFusedBatch, false>(aq, seg, t, td, act, sda, sdb, acc);
    }
    __builtin_amdgcn_wave_barrier();  // ring reads done before the next piece's writes
  }
}

// deferred mode: kFusedBatch chunks of the ring (segment docs, columns from HBM)
template <int NA>
__device__ __forceinline__ void fused_flush(cquery_t &aq, cseg_t &seg, const PHIP_LDS uint32_t *ring, int tail, int n,
                                            const SmallDict (&sda)[NA], const SmallDict (&sdb)[NA], uint64_t (&acc)[NA]) {
  const int lane = lane_id();
  int32_t d[kFusedBatch];
  uint32_t act = 0;
#pragma unroll
  for (int u = 0; u < kFusedBatch; u++) {
    const bool on = 64 * u + lane < n;
    d[u] = on ? (int32_t)ring[(tail + 64 * u + lane) & (kFusedRingDefer - 1)] : 0;
    act |= on ? (1u << u) : 0u;
  }
  const Tile tz{0, 0, nullptr};
  fused_batch<NA, kFusedBatch, true>(aq, seg, tz, d, act, sda, sdb, acc);
}

constexpr int defer_piece_lanes(int room) {  // the largest power of two <= room / 32 lanes (at most 64)
  int l = 64;
  while (l > 1 && l * 32 > room) l >>= 1;
  return l;
}
constexpr int kDeferPieceLanes = defer_piece_lanes(kFusedRingDefer - 64 * kFusedBatch);
static_assert(kFusedRingDefer - 64 * kFusedBatch >= 32 * kDeferPieceLanes, "a piece fits the ring beside a batch");

// (Measured and not kept, round 5: a 256-entry ring flushed 128 docs at a time -- 1 KiB per wave, as the fused group-by
// uses -- sorted Q1.1 0.136 -> 0.231 ms, unsorted Q1.3 0.352 -> 0.431: half the loads in flight per wave costs more than
// the resident workgroup it frees; profiles/r05za_ring256_ab_*.log.)
// deferred mode: append the tile's matched docs; a full batch is projected at once. (Measured and not kept, round 5:
// the batch's loads issued when it fills and consumed after the next tile's DMA wait and evaluation -- sorted Q1.1
// 0.157 -> 0.153 ms against the same build's synchronous batches, but the batch held across the tile cost 136 B of
// spills per lane and the build ran slower than this one, 0.138 ms; profiles/r05k_pipe_ab_sorted.log. Lane-major
// dense tiles projected in place, 8 groups per round trip, ran 2x slower: profiles/r05e_dense.log.)
// (Measured and not kept, round 5: dense tiles projected in place, lane-major, 8 groups per round trip -- sorted
// Q1.1 0.180 -> 0.374 ms at >= 256 matched docs per tile: four dependent round trips per tile instead of one per
// 256 deferred docs; profiles/r05e_dense.log.)
template <int NA>
__device__ __forceinline__ void fused_defer(cquery_t &aq, cseg_t &seg, const Tile &t, uint32_t mask,
                                            PHIP_LDS uint32_t *ring, int &head, int &tail, const SmallDict (&sda)[NA],
                                            const SmallDict (&sdb)[NA], uint64_t (&acc)[NA]) {
  if (ballot(mask != 0) == 0) return;
  const TileRank r = rank_tile(mask);
  const int head0 = head;
  // the whole tile when the ring has room, else pieces of kDeferPieceLanes lanes (<= 32 docs a lane) each after
  // draining the ring below one batch (< 64 x kFusedBatch pending + the piece <= kFusedRingDefer): eighth tiles for
  // the default 512-entry ring and 4-chunk batch
  const int npiece = head - tail + r.total <= kFusedRingDefer ? 1 : 64 / kDeferPieceLanes;
  const int lanes = 64 / npiece;
  for (int p = 0; p < npiece; p++) {
    const int e = __builtin_amdgcn_readlane((int)r.incl, lanes * p + lanes - 1);
    write_ranked<uint32_t, kFusedRingDefer>(r, lanes * p, lanes * (p + 1), -head0, t.doc0, ring);
    head = head0 + e;
    while (head - tail >= 64 * kFusedBatch) {
      fused_flush<NA>(aq, seg, ring, tail, 64 * kFusedBatch, sda, sdb, acc);
      tail += 64 * kFusedBatch;
    }
  }
}

// Fused group-by (NA == kFusedGroupBy: a dense key space in an HBM table, GB_GLOBAL): the tile's matched docs are
// appended to the same deferred ring, and every full batch goes through the aggregation kernel's batched group-by
// walk -- key ids and remaps, then per aggregation its inputs, agent-scope atomics into the table
// (DictionaryBasedGroupKeyGenerator.java:285-414 keys, DefaultGroupByExecutor.java:116-140 holders). The tile masks
// never reach HBM and the second launch with its mask walk is gone.
// NA == kFusedGroupBy: one HBM table (agent-scope atomics); NA == kFusedGroupByXcd: its XCD-private copies (GB_XCD);
// NA == kFusedGroupByLds: the workgroup's table in LDS after the rings, written to its slab at the end (GB_LDS).
constexpr int kFusedGroupBy = -1;
constexpr int kFusedGroupByXcd = -2;
constexpr int kFusedGroupByLds = -3;
constexpr int kGbFlush = 64 * kFusedBatchGB;
static_assert(kFusedRingGB >= 2 * kGbFlush, "a piece of <= kGbFlush docs lands on < kGbFlush pending");

template <int MODE>
__device__ __forceinline__ void fused_flush_gb(cquery_t &aq, cseg_t &seg, const PHIP_LDS uint32_t *ring, int tail, int n,
                                               lds_u64 *tbl, lds_u32 *hll_packed) {
  group_ring_batch<MODE, kFusedBatchGB, kFusedRingGB>(aq, seg, (const lds_u32 *)ring, tail, n, tbl, hll_packed);
}

template <int MODE>
__device__ __forceinline__ void fused_defer_gb(cquery_t &aq, cseg_t &seg, const Tile &t, uint32_t mask,
                                               PHIP_LDS uint32_t *ring, int &head, int &tail, lds_u64 *tbl,
                                               lds_u32 *hll_packed) {
  if (ballot(mask != 0) == 0) return;
  const TileRank r = rank_tile(mask);
  const int head0 = head;
  // the whole tile when the ring has room, else sixteenth tiles (4 lanes, <= 128 docs) each after draining the ring
  // below one flush (< 128 pending + 128 <= kFusedRingGB)
  const int npiece = head - tail + r.total <= kFusedRingGB ? 1 : 16;
  const int lanes = 64 / npiece;
  for (int p = 0; p < npiece; p++) {
    const int e = __builtin_amdgcn_readlane((int)r.incl, lanes * p + lanes - 1);
    write_ranked<uint32_t, kFusedRingGB>(r, lanes * p, lanes * (p + 1), -head0, t.doc0, ring);
    head = head0 + e;
    while (head - tail >= kGbFlush) {
      fused_flush_gb<MODE>(aq, seg, ring, tail, kGbFlush, tbl, hll_packed);
      tail += kGbFlush;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// the filter kernel
// ------------------------------------------------------------------------------------------------
// s_waitcnt vmcnt(n) for a wave-uniform n. n > 14 waits for vmcnt(15), which is stricter and so safe.
// (The count is forced into an SGPR, so this is a scalar branch tree, never a divergent one.)
#define PHIP_VMW(k) \
  case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
__device__ __forceinline__ void wait_vmcnt_lb(int n) {
  switch (__builtin_amdgcn_readfirstlane(n)) {
    PHIP_VMW(0) PHIP_VMW(1) PHIP_VMW(2) PHIP_VMW(3) PHIP_VMW(4) PHIP_VMW(5) PHIP_VMW(6) PHIP_VMW(7)
    PHIP_VMW(8) PHIP_VMW(9) PHIP_VMW(10) PHIP_VMW(11) PHIP_VMW(12) PHIP_VMW(13) PHIP_VMW(14)
    default: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
  }
}
#undef PHIP_VMW

// The staged sources of the segment being prefetched, held in SGPRs: loaded once when the prefetch
// cursor enters a segment, then advanced by one tile per prefetch (no per-tile metadata loads).
template <int kS>
struct StageCursor {
  const uint8_t *ptr[kS];  // bytes of the next tile to prefetch, per source
  int32_t bytes[kS];       // per tile
  int32_t lds[kS];         // region offset in the ring slot
  int32_t n;
};

template <int kS>
__device__ __forceinline__ void cursor_load(StageCursor<kS> &c, cseg_t &seg, int32_t tile_in_seg) {
  c.n = seg.num_stage;
#pragma unroll
  for (int i = 0; i < kS; i++) {
    c.ptr[i] = nullptr;
    c.bytes[i] = 0;
    c.lds[i] = 0;
    if (i < c.n) {
      c.bytes[i] = seg.stage[i].bytes;
      c.lds[i] = seg.stage[i].lds_off;
      c.ptr[i] = seg.stage[i].base + (int64_t)tile_in_seg * c.bytes[i];
    }
  }
}

// LDS-DMA of one tile into the ring slot at LDS address lbase; advances the cursor by `step` tiles.
template <int kS>
__device__ __forceinline__ void cursor_issue(StageCursor<kS> &c, uint32_t lbase, int step) {
  const int lane16 = lane_id() * 16;
#pragma unroll
  for (int i = 0; i < kS; i++) {
    if (i < c.n) {
      const uint8_t *g = c.ptr[i] + lane16;
      const uint32_t l = lbase + (uint32_t)c.lds[i];
      const int32_t nb = c.bytes[i];
      for (int off = 0; off < nb; off += 1024) {
        if (off + lane16 < nb) dma16(g + off, l + (uint32_t)off);
      }
      c.ptr[i] += (int64_t)nb * step;
    }
  }
}

#ifndef PHIP_FUSED_WAVES
#define PHIP_FUSED_WAVES 5  // waves per SIMD the fused launches are compiled for: the LDS admits 5 workgroups (20 waves)
                            // per CU, and 6 left 68 B of spills per lane (sorted Q1.1 -5 %, profiles/r05j_ablib_waves.log)
#endif
template <bool kConjOnly, int NA>
__global__ __launch_bounds__(kFilterBlock, kConjOnly ? (NA != 0 ? PHIP_FUSED_WAVES : 6) : 4) void filter_kernel(DevFilter q) {
  constexpr int kSConj = NA > 0 ? kMaxConj + kMaxAggStage : kMaxConj;
  constexpr int kS = kConjOnly ? (kSConj < kMaxStage ? kSConj : kMaxStage) : kMaxStage;  // (DevSeg.stage size)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = lane_id();
  const int wave = uniform(threadIdx.x >> 6);
  int begin, end, step;
  if (q.xcd_walk == 1) {
    // XCD sweep (grid is a multiple of 8): the work list is cut into 8 ranges, one per XCD, and an
    // XCD's waves stride through its range together, so at any time they read neighbouring tiles
    const int x = blockIdx.x & 7, gx = gridDim.x >> 3;
    begin = (int)((int64_t)q.total_work * x / 8) + (int)(blockIdx.x >> 3) * kFilterWaves + wave;
    end = (int)((int64_t)q.total_work * (x + 1) / 8);
    step = gx * kFilterWaves;
  } else if (q.xcd_walk == 2) {
    // XCD ranges, each cut into contiguous per-wave ranges: a wave streams contiguous tiles (its ring
    // prefetch stays sequential) and an XCD's waves stay inside 1/8 of the work list, so the dictionaries a
    // fused aggregation gathers from belong to the few segments of that range (they stay in the XCD's L2)
    const int x = blockIdx.x & 7, gx = gridDim.x >> 3;
    const int64_t xs = (int64_t)q.total_work * x / 8, xe = (int64_t)q.total_work * (x + 1) / 8;
    const int64_t nw = (int64_t)gx * kFilterWaves, w = (int64_t)(blockIdx.x >> 3) * kFilterWaves + wave;
    begin = (int)(xs + (xe - xs) * w / nw);
    end = (int)(xs + (xe - xs) * (w + 1) / nw);
    step = 1;
  } else {
    // contiguous range per wave
    const int64_t waves_total = (int64_t)gridDim.x * kFilterWaves;
    const int64_t gw = (int64_t)blockIdx.x * kFilterWaves + wave;
    begin = (int)((int64_t)q.total_work * gw / waves_total);
    end = (int)((int64_t)q.total_work * (gw + 1) / waves_total);
    step = 1;
  }
  const int nbuf = q.nbuf;
  const int stride = q.stage_stride;
  PHIP_LDS uint8_t *ring = (PHIP_LDS uint8_t *)(smem + (size_t)wave * nbuf * stride);
  // fused aggregation: the wave's matched-doc ring sits after every wave's DMA ring
  PHIP_LDS uint8_t *docring_b = (PHIP_LDS uint8_t *)(smem + (size_t)kFilterWaves * nbuf * stride) +
                                (NA != 0 ? (size_t)wave * q.fring_bytes : 0);
  PHIP_LDS uint16_t *docring = (PHIP_LDS uint16_t *)docring_b;
  PHIP_LDS uint32_t *deferring = (PHIP_LDS uint32_t *)docring_b;
  int dhead = 0, dtail = 0;  // deferred ring cursors (wave-uniform)
  const uint32_t ring_lds = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)ring);

  cseg_t *segs = (cseg_t *)q.segs;
  cnode_t *nodes = (cnode_t *)q.nodes;
  uint32_t lane_matched = 0;  // per-lane popcount, reduced once per segment
  uint64_t scanned = 0;
  uint64_t matched_total = 0;
  // Completion of a tile's DMA is awaited with a LOWER bound of the vector-memory instructions issued
  // after it: >= min_dma per later prefetched tile, plus the mask stores of the tiles evaluated since
  // (atomics only add to the true count). Waiting for fewer outstanding operations is always safe.
  const int nd = q.min_dma;
  const int st = q.mask_out != nullptr ? 1 : 0;
  constexpr int NAX = NA > 0 ? NA : 1;
  constexpr int kGbMode = NA == kFusedGroupByXcd ? GB_XCD : (NA == kFusedGroupByLds ? GB_LDS : GB_GLOBAL);
  // (NA < 0: the fused group-by's table; GB_LDS: the workgroup's, after every wave's DMA and doc rings)
  lds_u64 *gtbl = nullptr;
  lds_u32 *ghll = nullptr;
  if constexpr (NA == kFusedGroupByLds) {
    cquery_t &aq = *(cquery_t *)q.agg;
    gtbl = (lds_u64 *)(smem + (size_t)kFilterWaves * (nbuf * stride + q.fring_bytes));
    ghll = (lds_u32 *)((PHIP_LDS uint8_t *)gtbl + (size_t)aq.tbl_words * 8);
    const int G = (int)aq.num_groups;
    for (int i = threadIdx.x; i < aq.tbl_words; i += kFilterBlock) {
      const int row = i / G;
      gtbl[i] = (row > 0 && aq.aggs[row - 1].acc == ACC_MIN_F64) ? ~0ull : 0ull;  // ordered(+inf) < ~0
    }
    for (int i = threadIdx.x; i < aq.hll_words; i += kFilterBlock) ghll[i] = 0;
    __syncthreads();
  }
  uint64_t acc[NAX];
  SmallDict sda[NAX], sdb[NAX];
  if constexpr (NA > 0) {
    cquery_t &aq = *(cquery_t *)q.agg;
#pragma unroll
    for (int a = 0; a < NA; a++) {
      acc[a] = a < aq.num_aggs ? acc_init(aq.aggs[a].acc) : 0;
      sda[a] = sdb[a] = SmallDict{0u, 0u, false};
    }
  }

  // prefetch cursor: tiles [begin, pf) have their DMA issued (pfc of them)
  int pf = begin, pfc = 0, psn = 0, pend = -1, pslot = 0;
  StageCursor<kS> cur;
  cur.n = 0;
#define PHIP_PREFETCH()                                                                         \
  do {                                                                                          \
    if (pf >= pend) {                                                                           \
      while (psn + 1 < q.num_segs && segs[psn].work_begin + segs[psn].num_work <= pf) psn++;    \
      cseg_t &ps = segs[psn];                                                                   \
      pend = ps.work_begin + ps.num_work;                                                       \
      cursor_load<kS>(cur, ps, ps.tile0 + (pf - ps.work_begin));                                \
    }                                                                                           \
    cursor_issue<kS>(cur, ring_lds + (uint32_t)(pslot * stride), step);                         \
    pf += step;                                                                                 \
    pfc++;                                                                                      \
    pslot = pslot + 1 == nbuf ? 0 : pslot + 1;                                                  \
  } while (0)
  for (int i = 0; i < nbuf - 1 && pf < end; i++) PHIP_PREFETCH();

  int si = -1;  // segment of the current tile
  int seg_end = -1;
  int slot = 0;
  int k = 0;  // tiles evaluated
  for (int t = begin; t < end; t += step, k++) {
    if (pf < end) PHIP_PREFETCH();
    if (t >= seg_end) {  // entering a new segment: flush the previous one's count
      if constexpr (NA > 0) {  // the previous segment's deferred docs, before its small dictionaries go
        if (si >= 0 && dhead > dtail)
          fused_flush<NA>(*(cquery_t *)q.agg, segs[si], deferring, dtail, dhead - dtail, sda, sdb, acc);
        dhead = dtail = 0;
      }
      if constexpr (NA < 0) {  // (the group keys are the segment's: flushed before it ends)
        while (si >= 0 && dhead > dtail) {
          fused_flush_gb<kGbMode>(*(cquery_t *)q.agg, segs[si], deferring, dtail, min(dhead - dtail, kGbFlush), gtbl,
                                  ghll);
          dtail += kGbFlush;
        }
        dhead = dtail = 0;
      }
      if (si >= 0) {
        const uint64_t m = wave_reduce_u64_add(lane_matched);
        lane_matched = 0;
        matched_total += m;
        if (m && lane == 0)  // m is wave-uniform: one atomic wave-instruction
          atomicAdd((unsigned long long *)&q.seg_matched[segs[si].seg_index], (unsigned long long)m);
      }
      si = si < 0 ? 0 : si;
      while (si + 1 < q.num_segs && segs[si + 1].work_begin <= t) si++;
      seg_end = segs[si].work_begin + segs[si].num_work;
      if constexpr (NA > 0) {  // the segment's small dictionaries, one entry per lane
        cquery_t &aq = *(cquery_t *)q.agg;
#pragma unroll
        for (int a = 0; a < NA; a++) {
          if (a >= aq.num_aggs || aq.aggs[a].acc == ACC_COUNT) continue;
          sda[a] = load_small_dict(segs[si].cols[aq.aggs[a].col_a]);
          if (aq.aggs[a].expr != PHIP_EXPR_COLUMN) sdb[a] = load_small_dict(segs[si].cols[aq.aggs[a].col_b]);
        }
      }
    }
    cseg_t &seg = segs[si];
    Tile tl;
    const int32_t tile_in_seg = seg.tile0 + (t - seg.work_begin);
    tl.doc0 = tile_in_seg * kTileDocs;
    tl.valid_docs = min(kTileDocs, seg.num_docs - tl.doc0);
    tl.stage = ring + slot * stride;
    wait_vmcnt_lb((pfc - k - 1) * nd + min(k, nbuf - 1) * st);

    const uint32_t valid = valid_word(tl.valid_docs, lane);
    uint32_t scanned_t = 0;
    uint32_t mask;
    if (q.probe) {
      mask = valid;
    } else if (kConjOnly || seg.conj_path) {
      mask = seg.conj > 0 ? eval_conj(seg, tl.stage, valid) : valid;
      if (seg.conj_range && (seg.conj_lo > tl.doc0 || seg.conj_hi < tl.doc0 + kTileDocs - 1)) {
        const int32_t lo = max(seg.conj_lo - tl.doc0, 0), hi = min(seg.conj_hi - tl.doc0, kTileDocs - 1);
        mask &= lo <= hi ? range_word(lo, hi, lane) : 0u;
      }
      scanned_t = (uint32_t)seg.conj * (uint32_t)tl.valid_docs;
    } else if (seg.contig) {
      mask = eval_filter_contig(seg, nodes, contig_valid(tl.valid_docs, lane), tl, scanned_t, q.contig_inline != 0);
      if (st) mask = contig_to_lane_major(mask);  // (popcounts do not care about the layout)
    } else {
      mask = seg.node_end > seg.node_begin ? eval_filter(seg, nodes, valid, tl, scanned_t) : valid;
    }
    if ((q.stats_programs >> seg.program) & 1u) scanned += scanned_t;  // (wave-uniform)
    lane_matched += (uint32_t)__popc(mask);
    if (st) {
      PHIP_GLB uint32_t *mo = (PHIP_GLB uint32_t *)q.mask_out + (size_t)t * 64 + lane;
      if (q.mask_nt) __builtin_nontemporal_store(mask, mo);
      else *mo = mask;
    }
    if constexpr (NA > 0) {
      if (seg.fused_defer) fused_defer<NA>(*(cquery_t *)q.agg, seg, tl, mask, deferring, dhead, dtail, sda, sdb, acc);
      else fused_tile<NA>(*(cquery_t *)q.agg, seg, tl, mask, docring, sda, sdb, acc);
    }
    if constexpr (NA < 0) fused_defer_gb<kGbMode>(*(cquery_t *)q.agg, seg, tl, mask, deferring, dhead, dtail, gtbl, ghll);
    slot = slot + 1 == nbuf ? 0 : slot + 1;
  }
#undef PHIP_PREFETCH
  if constexpr (NA > 0) {
    if (si >= 0 && dhead > dtail) fused_flush<NA>(*(cquery_t *)q.agg, segs[si], deferring, dtail, dhead - dtail, sda, sdb, acc);
  }
  if constexpr (NA < 0) {
    while (si >= 0 && dhead > dtail) {
      fused_flush_gb<kGbMode>(*(cquery_t *)q.agg, segs[si], deferring, dtail, min(dhead - dtail, kGbFlush), gtbl,
                              ghll);
      dtail += kGbFlush;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (si >= 0) {
    const uint64_t m = wave_reduce_u64_add(lane_matched);
    matched_total += m;
    if (lane == 0 && m) atomicAdd((unsigned long long *)&q.seg_matched[segs[si].seg_index], (unsigned long long)m);
  }
  // per-block partials: matched docs, entries scanned in filter (fixed-order reduction on the host side)
  __shared__ uint64_t part[kFilterWaves][2];
  if (lane == 0) {
    part[wave][0] = matched_total;
    part[wave][1] = scanned;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    uint64_t v = 0;
    for (int w = 0; w < kFilterWaves; w++) v += part[w][threadIdx.x];
    coherent_store(q.partials + (size_t)blockIdx.x * 2 + threadIdx.x, v);  // (read by the finalizing workgroup)
  }
  if constexpr (NA > 0) {  // fused aggregation: per-block partials, reduced in a fixed order by finalize
    cquery_t &aq = *(cquery_t *)q.agg;
    __shared__ uint64_t apart[kFilterWaves][NA];
#pragma unroll
    for (int a = 0; a < NA; a++) {
      if (a >= aq.num_aggs) break;
      const int kind = aq.aggs[a].acc;
      uint64_t v;
      if (kind == ACC_COUNT || kind == ACC_SUM_I64) v = wave_reduce_u64_add(acc[a]);
      else v = as_u64(wave_reduce_f64(as_f64(acc[a]), kind));
      if (lane == 0) apart[wave][a] = v;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
      for (int a = 0; a < NA; a++) {
        if (a >= aq.num_aggs) break;
        const int kind = aq.aggs[a].acc;
        uint64_t v = apart[0][a];
        for (int w = 1; w < kFilterWaves; w++) v = acc_combine(kind, v, apart[w][a]);
        coherent_store(q.agg_partials + (size_t)blockIdx.x * aq.num_aggs + a, v);
      }
    }
  }
  if constexpr (NA == kFusedGroupByLds) {  // the workgroup's table -> its slab (slab_reduce_kernel folds them in order)
    cquery_t &aq = *(cquery_t *)q.agg;
    __syncthreads();
    glb_u64 *slab = (glb_u64 *)aq.gb_table + (size_t)blockIdx.x * aq.tbl_words;
    for (int i = threadIdx.x; i < aq.tbl_words; i += kFilterBlock) slab[i] = gtbl[i];
    glb_u32 *hs = (glb_u32 *)aq.gb_hll + (size_t)blockIdx.x * aq.hll_words;
    for (int i = threadIdx.x; i < aq.hll_words; i += kFilterBlock) hs[i] = ghll[i];
  }
  if (q.fin != nullptr) finalize_tail(q.fin);
}


template <bool C, int NA>
hipError_t launch_filter_t(const DevFilter &q, int nblocks, size_t lds_bytes, hipStream_t s, hipEvent_t e0,
                                  hipEvent_t e1) {
  if (lds_bytes > 65536) {
    // allow > 64 KiB dynamic LDS (gfx950: 160 KiB per workgroup); once, thread-safe (magic static)
    static const hipError_t configured = hipFuncSetAttribute((const void *)filter_kernel<C, NA>,
                                                             hipFuncAttributeMaxDynamicSharedMemorySize, 163840 - 1024);
    if (configured != hipSuccess) return configured;
  }
  if (e0 != nullptr) {  // timing carried by the dispatch packet itself (no barrier packets around it)
    void *args[] = {(void *)&q};
    return hipExtLaunchKernel((const void *)filter_kernel<C, NA>, dim3(nblocks), dim3(kFilterBlock), args, lds_bytes, s,
                              e0, e1, 0);
  }
  filter_kernel<C, NA><<<nblocks, kFilterBlock, lds_bytes, s>>>(q);
  return hipGetLastError();
}

}  // namespace phip
