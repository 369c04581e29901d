// kernels.hip -- gfx950 kernels of the segment query hot path.
//
// Layout in HBM (built at segment load, see runtime.cpp):
//   * fixed-bit dict-id forward index: u32 words, word k = BE bytes [4k, 4k+4) read as a big-endian
//     integer, so bit 31 of word k is stream bit 32k (FixedBitIntReader's MSB-first order,
//     pinot-segment-local/.../io/reader/impl/FixedBitIntReader.java:121-178). Doc d's id is bits
//     [d*b, d*b+b). A 64-doc group occupies exactly 2b words, a 2048-doc tile 64b words (256b bytes).
//   * dictionaries: LE typed arrays; raw columns: LE values.
//
// Execution model of the fused scan kernel (K1+K2+K5..K8 of SURVEY.md §2.4): one wave owns one
// 2048-doc tile at a time (32 groups x 64 docs), grid-striding over a work list of tiles that the host
// has already pruned with the sorted-index leaves.
//   1. Filter: the tile's bytes of every scanned column arrive in LDS by LDS-DMA (double-buffered:
//      tile i+1 is in flight while tile i is evaluated). Leaves are evaluated with lanes = docs: each
//      lane decodes its doc's dict id and tests the predicate; the 64-lane ballot IS the group's 64-doc
//      bitmap word (SVScanDocIdIterator + PredicateEvaluator.applySV,
//      pinot-core/.../dociditerators/SVScanDocIdIterator.java:75-142), kept by lane g. The filter program (postfix, binary AND/OR with short-circuit skips) then combines
//      per-lane u64 words (AndDocIdSet / OrDocIdSet / NotDocIdSet).
//   2. Compaction: the matched docs of the tile become a u16 list in LDS (mbcnt ranks per group).
//   3. Projection + aggregation with lanes = matched docs (late materialisation, as DataFetcher reads
//      only the matched doc ids, pinot-core/.../common/DataFetcher.java:335-386): value / group-key
//      columns are decoded from LDS when staged, else straight from HBM, dictionaries gathered, and the
//      values folded into per-lane accumulators or group tables.
#include <hip/hip_runtime.h>

#include "../../include/pinot_hip.h"
#include "device.h"

namespace phip {

// Query metadata (segments, columns, filter programs) is read through the constant address space so
// that it compiles to scalar loads (lgkmcnt), never counted in vmcnt.
#define PHIP_CAS __attribute__((address_space(4)))
typedef const PHIP_CAS DevSeg cseg_t;
typedef const PHIP_CAS DevNode cnode_t;
typedef const PHIP_CAS DevCol ccol_t;

// ------------------------------------------------------------------------------------------------
// helpers
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int lane) {
  uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, lane);
  uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

// rank of this lane among the set bits of m below it
__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Bits [off, off+bits) of the MSB-first stream held in words (u32, bit 31 first).
__device__ __forceinline__ uint32_t decode_bits(const uint32_t *__restrict__ words, uint64_t off, uint32_t bits) {
  const uint32_t *p = words + (off >> 5);
  uint64_t win = ((uint64_t)p[0] << 32) | (uint64_t)p[1];
  return (uint32_t)((win << (off & 31)) >> (64 - bits));
}

// Window of 32 stream bits starting at bit p of a staged region (u32 words, bit 31 first).
// q = floor((p-1)/32) may be -1 (reads the guard word before the region); s in [0, 31].
__device__ __forceinline__ uint32_t window_at(const uint32_t *w, int32_t p) {
  const int32_t q = (p - 1) >> 5;
  const uint32_t s = (uint32_t)(32 * (q + 1) - p);
  return __builtin_amdgcn_alignbit(w[q], w[q + 1], s);
}

// Order-preserving map double <-> u64 (for atomicMin/atomicMax on the group table).
__device__ __forceinline__ uint64_t f64_ordered(double d) {
  uint64_t u = (uint64_t)__double_as_longlong(d);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__host__ __device__ inline double f64_unordered(uint64_t u) {
  u = (u >> 63) ? (u & 0x7fffffffffffffffull) : ~u;
  union {
    uint64_t u;
    double d;
  } x;
  x.u = u;
  return x.d;
}
__device__ __forceinline__ double as_f64(uint64_t u) { return __longlong_as_double((long long)u); }
__device__ __forceinline__ uint64_t as_u64(double d) { return (uint64_t)__double_as_longlong(d); }

__device__ __forceinline__ int64_t dict_i64(ccol_t &c, uint32_t id) {
  switch (c.type) {
    case PHIP_TYPE_INT: return ((const int32_t *)c.dict)[id];
    case PHIP_TYPE_LONG: return ((const int64_t *)c.dict)[id];
    case PHIP_TYPE_FLOAT: return (int64_t)((const float *)c.dict)[id];
    default: return (int64_t)((const double *)c.dict)[id];
  }
}
__device__ __forceinline__ double dict_f64(ccol_t &c, uint32_t id) {
  switch (c.type) {
    case PHIP_TYPE_INT: return (double)((const int32_t *)c.dict)[id];
    case PHIP_TYPE_LONG: return (double)((const int64_t *)c.dict)[id];
    case PHIP_TYPE_FLOAT: return (double)((const float *)c.dict)[id];
    default: return ((const double *)c.dict)[id];
  }
}
__device__ __forceinline__ int64_t raw_i64(ccol_t &c, int32_t doc) {
  switch (c.type) {
    case PHIP_TYPE_INT: return ((const int32_t *)c.raw)[doc];
    case PHIP_TYPE_LONG: return ((const int64_t *)c.raw)[doc];
    case PHIP_TYPE_FLOAT: return (int64_t)((const float *)c.raw)[doc];
    default: return (int64_t)((const double *)c.raw)[doc];
  }
}
__device__ __forceinline__ double raw_f64(ccol_t &c, int32_t doc) {
  switch (c.type) {
    case PHIP_TYPE_INT: return (double)((const int32_t *)c.raw)[doc];
    case PHIP_TYPE_LONG: return (double)((const int64_t *)c.raw)[doc];
    case PHIP_TYPE_FLOAT: return (double)((const float *)c.raw)[doc];
    default: return ((const double *)c.raw)[doc];
  }
}

// ------------------------------------------------------------------------------------------------
// LDS-DMA staging. The copy is issued through inline asm so that hipcc does not see an LDS write in
// flight: it would otherwise put s_waitcnt vmcnt(0) in front of the first ds_read of the CURRENT
// tile and drain the prefetch of the next one. Completion is awaited by wait_vmcnt(n) below.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

__device__ __forceinline__ void dma16(const uint8_t *gsrc, uint32_t lds_dst) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_dst)
      : "memory");
}

// Issue the LDS-DMA copies of one tile's staged regions (1 KiB per wave-instruction).
__device__ __forceinline__ void stage_tile(cseg_t &seg, int32_t tile_in_seg, uint8_t *buf) {
  const int lane = lane_id();
  const uint32_t lbase = __builtin_amdgcn_readfirstlane(lds_addr(buf));
  for (int i = 0; i < seg.num_stage; i++) {
    const int32_t sbytes = seg.stage[i].bytes;
    const uint8_t *g = seg.stage[i].base + (int64_t)tile_in_seg * sbytes + lane * 16;
    const uint32_t l = lbase + (uint32_t)seg.stage[i].lds_off;
    for (int c = 0; c < sbytes; c += 1024) {
      if (c + lane * 16 < sbytes) dma16(g + c, l + (uint32_t)c);
    }
  }
}

// s_waitcnt vmcnt(n) for a wave-uniform n (vmcnt takes an immediate).
#define PHIP_VM(k) \
  case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
__device__ __forceinline__ void wait_vmcnt(int n) {
  switch (n) {
    PHIP_VM(1) PHIP_VM(2) PHIP_VM(3) PHIP_VM(4) PHIP_VM(5) PHIP_VM(6) PHIP_VM(7) PHIP_VM(8) PHIP_VM(9)
    PHIP_VM(10) PHIP_VM(11) PHIP_VM(12) PHIP_VM(13) PHIP_VM(14) PHIP_VM(15) PHIP_VM(16) PHIP_VM(17)
    PHIP_VM(18) PHIP_VM(19) PHIP_VM(20) PHIP_VM(21) PHIP_VM(22) PHIP_VM(23) PHIP_VM(24) PHIP_VM(25)
    PHIP_VM(26) PHIP_VM(27) PHIP_VM(28) PHIP_VM(29) PHIP_VM(30) PHIP_VM(31) PHIP_VM(32) PHIP_VM(33)
    PHIP_VM(34) PHIP_VM(35) PHIP_VM(36) PHIP_VM(37) PHIP_VM(38) PHIP_VM(39) PHIP_VM(40) PHIP_VM(41)
    PHIP_VM(42) PHIP_VM(43) PHIP_VM(44) PHIP_VM(45) PHIP_VM(46) PHIP_VM(47) PHIP_VM(48) PHIP_VM(49)
    PHIP_VM(50) PHIP_VM(51) PHIP_VM(52) PHIP_VM(53) PHIP_VM(54) PHIP_VM(55) PHIP_VM(56) PHIP_VM(57)
    PHIP_VM(58) PHIP_VM(59) PHIP_VM(60) PHIP_VM(61) PHIP_VM(62) PHIP_VM(63)
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}
#undef PHIP_VM

// Per-tile context of one wave.
struct Tile {
  int32_t doc0;          // first doc of the tile within the segment
  int32_t valid_docs;    // docs of the tile inside the segment (1..2048)
  const uint8_t *stage;  // this wave's LDS stage buffer holding the tile's staged regions
};

// ------------------------------------------------------------------------------------------------
// filter leaves. A tile's doc set is held lane-major: lane l owns a 32-bit word whose bit (31-g)
// is doc g*64 + l of the tile. Leaves decode with lanes = docs of one 64-doc group at a time and
// shift the predicate bit into the lane's word (the group loop is ~4 VALU per 64 docs), and the
// boolean algebra of the filter tree is one VALU op per lane on u32 words.
// ------------------------------------------------------------------------------------------------
// Group loop of one scan leaf: lane l decodes doc g*64 + l from the staged words (2B words per group).
// B is runtime: a width-templated switch measured 143 VGPRs (hipcc hoists the cases' common LDS
// reads above the switch) against 69 for one width; the runtime form costs one address add per group.
#define PHIP_GROUP_LOOP(PASS_EXPR)                                             \
  const int lane = lane_id();                                                  \
  const int32_t p = lane * B;                                                  \
  const int32_t q = (p - 1) >> 5;                                              \
  const uint32_t s = (uint32_t)(32 * (q + 1) - p);                             \
  const uint32_t *wl = w + q;                                                  \
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
__device__ __forceinline__ uint32_t scan_range(const uint32_t *w, int B, uint32_t LO, uint32_t SPAN) {
  PHIP_GROUP_LOOP((win - LO) < SPAN)
}

// IN / NOT IN / EQ / NEQ on a column with card <= 64: membership in a 64-bit mask (the host
// complements it for exclusive predicates).
__device__ __forceinline__ uint32_t scan_small_set(const uint32_t *w, int B, uint64_t set) {
  const uint32_t k = 32 - B;
  PHIP_GROUP_LOOP(((set >> (win >> k)) & 1ull) != 0)
}

// IN / NOT IN on a larger dictionary: bitset over dict ids in HBM (L1/L2 resident).
__device__ __forceinline__ uint32_t scan_big_set(const uint32_t *w, int B, const uint32_t *__restrict__ set, bool excl) {
  const uint32_t k = 32 - B;
  PHIP_GROUP_LOOP(((((set[(win >> k) >> 5] >> ((win >> k) & 31)) & 1u) != 0) != excl))
}

// bits [lo, hi] (inclusive, 0 <= lo <= hi <= 31) of a u32
__device__ __forceinline__ uint32_t span32(int lo, int hi) {
  const uint32_t upto = (hi == 31) ? ~0u : ((1u << (hi + 1)) - 1u);
  return upto & ~((1u << lo) - 1u);
}

// Lane-major word of the doc range [s, e] (tile-relative, inclusive, clamped to the tile).
__device__ __forceinline__ uint32_t range_word(int32_t s, int32_t e, int lane) {
  // groups g with s <= g*64 + lane <= e
  const int32_t g_lo = max(0, (s - lane + 63) >> 6);
  const int32_t g_hi = min(kTileGroups - 1, (e - lane) >= 0 ? (e - lane) >> 6 : -1);
  if (g_lo > g_hi) return 0u;
  return span32(31 - g_hi, 31 - g_lo);
}

// One leaf over the tile; `valid` = lane-major docs of the tile inside the segment.
__device__ __forceinline__ uint32_t eval_leaf(cseg_t &seg, cnode_t *__restrict__ n, uint32_t valid, const Tile &t,
                                              uint32_t &scanned) {
  const int lane = lane_id();
  const int kind = n->leaf_kind;
  if (kind == PHIP_LEAF_MATCH_ALL) return valid;
  if (kind == PHIP_LEAF_MATCH_NONE) return 0;
  if (kind == PHIP_LEAF_DOC_RANGES) {
    // SortedIndexBasedFilterOperator: inclusive doc ranges, sorted and disjoint
    const int32_t *rg = (const int32_t *)n->aux;
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
    const uint64_t *w = n->lds_off >= 0 ? (const uint64_t *)(t.stage + n->lds_off)
                                        : (const uint64_t *)n->aux + (t.doc0 >> 6);
    uint32_t r = 0;
#pragma unroll 8
    for (int g = 0; g < kTileGroups; g++) r = r + r + (uint32_t)((w[g] >> lane) & 1ull);
    if (n->exclusive) r = ~r;
    return valid & r;
  }
  // DICT_RANGE / DICT_SET on the bit-packed forward index
  scanned += (uint32_t)t.valid_docs;
  const int32_t B = n->bits;
  if (n->lds_off >= 0) {
    const uint32_t *w = (const uint32_t *)(t.stage + n->lds_off);
    uint32_t r;
    if (kind == PHIP_LEAF_DICT_RANGE) {
      const uint32_t LO = (uint32_t)n->lo << (32 - B);
      const uint32_t SPAN = (uint32_t)(n->hi - n->lo) << (32 - B);
      r = scan_range(w, B, LO, SPAN);
    } else if (n->small_set) {
      r = scan_small_set(w, B, n->set_mask);
    } else {
      r = scan_big_set(w, B, (const uint32_t *)n->aux, n->exclusive != 0);
    }
    return r & valid;
  }
  // not staged (LDS budget exceeded): decode from HBM
  ccol_t &c = seg.cols[n->column];
  const bool is_range = kind == PHIP_LEAF_DICT_RANGE;
  const uint32_t *__restrict__ set = (const uint32_t *)n->aux;
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

// ------------------------------------------------------------------------------------------------
// per-doc projection (lanes = matched docs; dit = doc offset within the tile)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t col_dict_id(ccol_t &c, const Tile &t, uint32_t dit) {
  if (c.lds_off >= 0) {
    const uint32_t *w = (const uint32_t *)(t.stage + c.lds_off);
    return window_at(w, (int32_t)(dit * (uint32_t)c.bits)) >> (32 - c.bits);
  }
  return decode_bits(c.words, (uint64_t)(uint32_t)(t.doc0 + (int32_t)dit) * (uint32_t)c.bits, (uint32_t)c.bits);
}
__device__ __forceinline__ int64_t col_i64(ccol_t &c, const Tile &t, uint32_t dit) {
  if (c.has_dict) return dict_i64(c, col_dict_id(c, t, dit));
  return raw_i64(c, t.doc0 + (int32_t)dit);
}
__device__ __forceinline__ double col_f64(ccol_t &c, const Tile &t, uint32_t dit) {
  if (c.has_dict) return dict_f64(c, col_dict_id(c, t, dit));
  return raw_f64(c, t.doc0 + (int32_t)dit);
}
__device__ __forceinline__ int64_t expr_i64(cseg_t &s, const DevAgg &a, const Tile &t, uint32_t dit) {
  int64_t x = col_i64(s.cols[a.col_a], t, dit);
  if (a.expr == PHIP_EXPR_COLUMN) return x;
  int64_t y = col_i64(s.cols[a.col_b], t, dit);
  if (a.expr == PHIP_EXPR_ADD) return x + y;
  if (a.expr == PHIP_EXPR_SUB) return x - y;
  return x * y;
}
__device__ __forceinline__ double expr_f64(cseg_t &s, const DevAgg &a, const Tile &t, uint32_t dit) {
  double x = col_f64(s.cols[a.col_a], t, dit);
  if (a.expr == PHIP_EXPR_COLUMN) return x;
  double y = col_f64(s.cols[a.col_b], t, dit);
  if (a.expr == PHIP_EXPR_ADD) return x + y;
  if (a.expr == PHIP_EXPR_SUB) return x - y;
  return x * y;
}

__device__ __forceinline__ uint64_t wave_reduce_u64_add(uint64_t v) {
  for (int o = 32; o > 0; o >>= 1) {
    uint32_t lo = __shfl_xor((int)(uint32_t)v, o);
    uint32_t hi = __shfl_xor((int)(uint32_t)(v >> 32), o);
    v += ((uint64_t)hi << 32) | lo;
  }
  return v;
}
__device__ __forceinline__ uint32_t wave_or32(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v |= (uint32_t)__shfl_xor((int)v, o);
  return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ double wave_reduce_f64(double v, int kind) {
  for (int o = 32; o > 0; o >>= 1) {
    double w = __shfl_xor(v, o);
    if (kind == ACC_SUM_F64) v += w;
    else if (kind == ACC_MIN_F64) v = fmin(v, w);
    else v = fmax(v, w);
  }
  return v;
}

__device__ __forceinline__ uint64_t acc_init(int kind) {
  if (kind == ACC_MIN_F64) return as_u64(__builtin_huge_val());
  if (kind == ACC_MAX_F64) return as_u64(-__builtin_huge_val());
  return 0;  // counts, int sums, f64 +0.0
}

__device__ __forceinline__ uint64_t acc_combine(int kind, uint64_t a, uint64_t b) {
  if (kind == ACC_SUM_F64) return as_u64(as_f64(a) + as_f64(b));
  if (kind == ACC_MIN_F64) return as_u64(fmin(as_f64(a), as_f64(b)));
  if (kind == ACC_MAX_F64) return as_u64(fmax(as_f64(a), as_f64(b)));
  return a + b;
}

// Aggregation-only: fold one chunk of matched docs into per-lane accumulators (inactive lanes add
// the identity; their dit = 0 is a valid doc so every load stays in bounds).
template <int NA>
__device__ __forceinline__ void agg_docs(const DevQuery &q, cseg_t &seg, const Tile &t, uint32_t dit, bool act,
                                         uint64_t (&acc)[NA], uint32_t *hll_lds) {
#pragma unroll
  for (int a = 0; a < NA; a++) {
    if (a >= q.num_aggs) break;
    const DevAgg &ag = q.aggs[a];
    switch (ag.acc) {
      case ACC_COUNT: break;  // per tile
      case ACC_SUM_I64: {
        const int64_t v = expr_i64(seg, ag, t, dit);
        acc[a] += act ? (uint64_t)v : 0ull;
        break;
      }
      case ACC_SUM_F64: {
        const double v = expr_f64(seg, ag, t, dit);
        acc[a] = as_u64(as_f64(acc[a]) + (act ? v : 0.0));
        break;
      }
      case ACC_MIN_F64: {
        const double v = expr_f64(seg, ag, t, dit);
        acc[a] = as_u64(fmin(as_f64(acc[a]), act ? v : __builtin_huge_val()));
        break;
      }
      case ACC_MAX_F64: {
        const double v = expr_f64(seg, ag, t, dit);
        acc[a] = as_u64(fmax(as_f64(acc[a]), act ? v : -__builtin_huge_val()));
        break;
      }
      case ACC_HLL: {
        ccol_t &c = seg.cols[ag.col_a];
        const uint32_t h = c.hll[col_dict_id(c, t, dit)];
        if (act) atomicMax(&hll_lds[(ag.hll_slot << ag.log2m) + (h >> 8)], h & 0xffu);
        break;
      }
    }
  }
}

// Group-by: dense mixed-radix key over query-global dict ids (DictionaryBasedGroupKeyGenerator,
// column 0 least significant), then global-atomic updates of the group tables.
__device__ __forceinline__ void group_docs(const DevQuery &q, cseg_t &seg, const Tile &t, uint32_t dit, bool act) {
  int64_t key = 0;
  for (int k = 0; k < q.num_group_by; k++) {
    ccol_t &c = seg.cols[q.gb_cols[k]];
    const uint32_t id = col_dict_id(c, t, dit);
    const int32_t gid = c.remap ? c.remap[id] : (int32_t)id;
    key += (int64_t)gid * q.gb_stride[k];
  }
  if (!act) return;
  atomicAdd((unsigned long long *)&q.gb_count[key], 1ull);
#pragma unroll
  for (int a = 0; a < kMaxAggs; a++) {
    if (a >= q.num_aggs) break;
    const DevAgg &ag = q.aggs[a];
    uint64_t *slot = q.gb_table + (int64_t)a * q.num_groups + key;
    switch (ag.acc) {
      case ACC_COUNT: break;  // == gb_count
      case ACC_SUM_I64: atomicAdd((unsigned long long *)slot, (unsigned long long)expr_i64(seg, ag, t, dit)); break;
      case ACC_SUM_F64: atomicAdd((double *)slot, expr_f64(seg, ag, t, dit)); break;
      case ACC_MIN_F64:
        atomicMin((unsigned long long *)slot, (unsigned long long)f64_ordered(expr_f64(seg, ag, t, dit)));
        break;
      case ACC_MAX_F64:
        atomicMax((unsigned long long *)slot, (unsigned long long)f64_ordered(expr_f64(seg, ag, t, dit)));
        break;
      case ACC_HLL: {
        ccol_t &c = seg.cols[ag.col_a];
        const uint32_t h = c.hll[col_dict_id(c, t, dit)];
        uint32_t *regs = q.gb_hll + ((int64_t)ag.hll_slot * q.num_groups + key) * (1 << ag.log2m);
        atomicMax(&regs[h >> 8], h & 0xffu);
        break;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// fused filter + aggregate / group-by kernel
// LDS: [HLL registers (aggregation-only)] [wave partials] [per wave: match list | nbuf x stage]
// ------------------------------------------------------------------------------------------------
template <int NA, bool kGroupBy>
__global__ __launch_bounds__(kBlock) void scan_kernel(DevQuery q) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = lane_id();
  // wave-uniform by construction; readfirstlane tells the compiler, so every value derived from the
  // work index (segment, offsets, metadata addresses) lives in SGPRs and metadata loads are scalar
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int waves_total = gridDim.x * kWavesPerBlock;
  const int gwave = blockIdx.x * kWavesPerBlock + wave;
  const int naggs = q.num_aggs;
  const int nslots = naggs + 2;

  uint32_t *hll_lds = (uint32_t *)smem;
  int hll_words = 0;
  if (!kGroupBy && q.num_hll > 0) {
    hll_words = q.num_hll << q.aggs[0].log2m;  // all HLL aggs share log2m (host enforces)
    for (int i = threadIdx.x; i < hll_words; i += kBlock) hll_lds[i] = 0;
  }
  const int part_off = (hll_words * 4 + 15) & ~15;
  uint64_t *wave_part = (uint64_t *)(smem + part_off);
  uint8_t *wave_base = smem + part_off + ((kWavesPerBlock * nslots * 8 + 15) & ~15) +
                       (size_t)wave * (kListBytes + q.nbuf * q.stage_stride);
  uint16_t *list = (uint16_t *)wave_base;
  uint8_t *stage_base = wave_base + kListBytes;
  __syncthreads();

  uint64_t acc[NA];
#pragma unroll
  for (int a = 0; a < NA; a++) acc[a] = (a < naggs) ? acc_init(q.aggs[a].acc) : 0;
  uint64_t matched = 0;  // wave-uniform
  uint32_t scanned = 0;
  uint64_t seg_acc = 0;
  int seg_acc_idx = -1;
  uint64_t count_acc = 0;  // COUNT slots: matched docs (wave-uniform)

  cseg_t *segs = (cseg_t *)q.segs;
  cnode_t *nodes = (cnode_t *)q.nodes;
  int si = 0, sn = 0;  // segment of the current / the prefetched work item (monotone)
  int cur = 0;
  int work = gwave;
  if (work < q.total_work) {
    while (sn + 1 < q.num_segs && segs[sn + 1].work_begin <= work) sn++;
    stage_tile(segs[sn], segs[sn].tile0 + (work - segs[sn].work_begin), stage_base);
  }
  for (; work < q.total_work; work += waves_total) {
    while (si + 1 < q.num_segs && segs[si + 1].work_begin <= work) si++;
    cseg_t &seg = segs[si];
    Tile t;
    const int32_t tile_in_seg = seg.tile0 + (work - seg.work_begin);
    t.doc0 = tile_in_seg * kTileDocs;
    t.valid_docs = min(kTileDocs, seg.num_docs - t.doc0);
    t.stage = stage_base + cur * q.stage_stride;
    // prefetch the next work item into the other buffer, then wait only for this tile's copies
    const int next = work + waves_total;
    int in_flight = 0;
    if (q.nbuf == 2 && next < q.total_work) {
      while (sn + 1 < q.num_segs && segs[sn + 1].work_begin <= next) sn++;
      stage_tile(segs[sn], segs[sn].tile0 + (next - segs[sn].work_begin), stage_base + (cur ^ 1) * q.stage_stride);
      in_flight = segs[sn].num_dma;
    }
    wait_vmcnt(in_flight);

    if (si != seg_acc_idx) {
      if (seg_acc_idx >= 0 && seg_acc != 0 && lane == 0)
        atomicAdd((unsigned long long *)&q.seg_matched[segs[seg_acc_idx].seg_index], (unsigned long long)seg_acc);
      seg_acc = 0;
      seg_acc_idx = si;
    }

    // docs of the tile inside the segment, lane-major: bit (31-g) of lane l is doc g*64 + l
    const int32_t ngrp = min(kTileGroups, max(0, (t.valid_docs - lane + 63) >> 6));
    const uint32_t valid = ngrp == 0 ? 0u : (~0u << (32 - ngrp));
    uint32_t mask = valid;
    if (seg.node_end > seg.node_begin) mask = eval_filter(seg, nodes, valid, t, scanned);
    if (q.filter_out != nullptr) {  // 64-doc bitmap words (phip_filter_bitmap)
      uint64_t my = 0;
      for (int g = 0; g < kTileGroups; g++) {
        const uint64_t wg = ballot((mask >> (31 - g)) & 1u);
        if (lane == g) my = wg;
      }
      if (lane < kTileGroups && lane * 64 < t.valid_docs) q.filter_out[(t.doc0 >> 6) + lane] = my;
    }

    int nm = 0;
    if (q.need_docs) {
      auto do_chunk = [&](uint32_t dit, bool act) {
        if constexpr (kGroupBy) {
          group_docs(q, seg, t, dit, act);
        } else {
          agg_docs<NA>(q, seg, t, dit, act, acc, hll_lds);
        }
      };
      if (ballot(mask != valid) == 0) {
        // every doc of the tile matched: the list is the identity
        nm = t.valid_docs;
        for (int c = 0; c < nm; c += 64) {
          const bool act = c + lane < nm;
          do_chunk(act ? (uint32_t)(c + lane) : 0u, act);
        }
      } else {
        // compaction of the matched docs into the wave's list (ascending doc order)
        uint32_t any = wave_or32(mask);
        while (any) {
          const int bit = 31 - __builtin_clz(any);
          any &= ~(1u << bit);
          const bool b = (mask >> bit) & 1u;
          const uint64_t m = ballot(b);
          if (b) list[nm + mbcnt64(m)] = (uint16_t)((31 - bit) * 64 + lane);
          nm += __popcll(m);
        }
        for (int c = 0; c < nm; c += 64) {
          const bool act = c + lane < nm;
          do_chunk(act ? (uint32_t)list[c + lane] : 0u, act);
        }
      }
    } else {
      nm = (int)wave_reduce_u64_add((uint64_t)__popc(mask));
      nm = __builtin_amdgcn_readfirstlane(nm);
    }
    matched += (uint64_t)nm;
    seg_acc += (uint64_t)nm;
    cur ^= (q.nbuf == 2) ? 1 : 0;
    if (q.nbuf == 1 && next < q.total_work) {
      while (sn + 1 < q.num_segs && segs[sn + 1].work_begin <= next) sn++;
      stage_tile(segs[sn], segs[sn].tile0 + (next - segs[sn].work_begin), stage_base);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (seg_acc_idx >= 0 && seg_acc != 0 && lane == 0)
    atomicAdd((unsigned long long *)&q.seg_matched[segs[seg_acc_idx].seg_index], (unsigned long long)seg_acc);
  count_acc = matched;

  // ---- block reduction of the partials ---------------------------------------------------------
#pragma unroll
  for (int a = 0; a < NA; a++) {
    if (a >= naggs) break;
    const int kind = q.aggs[a].acc;
    uint64_t v;
    if (kind == ACC_COUNT) {
      v = count_acc;
    } else if (kind == ACC_SUM_I64 || kind == ACC_HLL) {
      v = wave_reduce_u64_add(acc[a]);
    } else {
      v = as_u64(wave_reduce_f64(as_f64(acc[a]), kind));
    }
    if (lane == 0) wave_part[wave * nslots + a] = v;
  }
  if (lane == 0) {
    wave_part[wave * nslots + naggs] = matched;
    wave_part[wave * nslots + naggs + 1] = scanned;
  }
  __syncthreads();
  if (threadIdx.x < nslots) {
    const int a = threadIdx.x;
    const int kind = a < naggs ? q.aggs[a].acc : ACC_COUNT;
    uint64_t v = wave_part[a];
    for (int w = 1; w < kWavesPerBlock; w++) v = acc_combine(kind, v, wave_part[w * nslots + a]);
    q.partials[(int64_t)blockIdx.x * nslots + a] = v;
  }
  if (!kGroupBy && hll_words > 0) {
    for (int i = threadIdx.x; i < hll_words; i += kBlock) {
      if (hll_lds[i]) atomicMax(&q.hll_regs[i], hll_lds[i]);
    }
  }
}

// Deterministic reduction of per-block partials -> out[nslots]: one wave per slot, lane-strided over
// blocks in a fixed order, then a fixed shuffle tree (bitwise reproducible run to run).
__global__ void finalize_partials_kernel(const uint64_t *__restrict__ partials, int nblocks, int nslots,
                                         const int32_t *__restrict__ kinds, uint64_t *__restrict__ out) {
  const int a = blockIdx.x;
  const int lane = threadIdx.x;
  if (a >= nslots) return;
  const int kind = kinds[a];
  const bool fp = kind == ACC_SUM_F64 || kind == ACC_MIN_F64 || kind == ACC_MAX_F64;
  uint64_t v = fp ? acc_init(kind) : 0;
  for (int b = lane; b < nblocks; b += 64) v = acc_combine(kind, v, partials[(int64_t)b * nslots + a]);
  if (fp) {
    v = as_u64(wave_reduce_f64(as_f64(v), kind));
  } else {
    v = wave_reduce_u64_add(v);
  }
  if (lane == 0) out[a] = v;
}

// ------------------------------------------------------------------------------------------------
// group-by table init / compaction
// ------------------------------------------------------------------------------------------------
__global__ void fill_u64_kernel(uint64_t *__restrict__ p, int64_t n, uint64_t v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = v;
}

// Per 1024-group chunk: number of non-empty groups.
__global__ __launch_bounds__(kBlock) void group_count_kernel(const uint64_t *__restrict__ counts, int64_t n,
                                                             int32_t *__restrict__ chunk_counts) {
  __shared__ int32_t s;
  if (threadIdx.x == 0) s = 0;
  __syncthreads();
  int64_t base = (int64_t)blockIdx.x * 1024;
  int c = 0;
  for (int i = threadIdx.x; i < 1024; i += kBlock) {
    int64_t gidx = base + i;
    if (gidx < n && counts[gidx] != 0) c++;
  }
  atomicAdd(&s, c);
  __syncthreads();
  if (threadIdx.x == 0) chunk_counts[blockIdx.x] = s;
}

// Single-block exclusive scan of chunk counts; total in offsets[nchunks].
__global__ void exclusive_scan_kernel(const int32_t *__restrict__ in, int32_t n, int64_t *__restrict__ offsets) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int64_t s = 0;
  for (int i = 0; i < n; i++) {
    offsets[i] = s;
    s += in[i];
  }
  offsets[n] = s;
}

// Ordered compaction: writes group indices of non-empty groups, ascending.
__global__ __launch_bounds__(kBlock) void group_compact_kernel(const uint64_t *__restrict__ counts, int64_t n,
                                                               const int64_t *__restrict__ offsets,
                                                               int64_t *__restrict__ out_keys) {
  __shared__ int32_t wave_counts[kBlock / 64];
  const int lane = lane_id(), wave = threadIdx.x >> 6;
  int64_t base = (int64_t)blockIdx.x * 1024;
  int64_t out = offsets[blockIdx.x];
  for (int round = 0; round < 1024 / kBlock; round++) {
    int64_t gidx = base + round * kBlock + threadIdx.x;
    bool nz = gidx < n && counts[gidx] != 0;
    uint64_t b = ballot(nz);
    if (lane == 0) wave_counts[wave] = __popcll(b);
    __syncthreads();
    int32_t before = 0;
    for (int w = 0; w < wave; w++) before += wave_counts[w];
    int32_t total = 0;
    for (int w = 0; w < kBlock / 64; w++) total += wave_counts[w];
    if (nz) {
      int32_t rank = before + __popcll(b & ((1ull << lane) - 1));
      out_keys[out + rank] = gidx;
    }
    out += total;
    __syncthreads();
  }
}

// Gather the aggregates of the compacted groups.
__global__ void group_gather_kernel(const int64_t *__restrict__ keys, int64_t ngroups, int64_t num_groups_dense,
                                    int32_t naggs, const int32_t *__restrict__ kinds,
                                    const uint64_t *__restrict__ table, const uint64_t *__restrict__ counts,
                                    const uint32_t *__restrict__ hll, int32_t nhll, int32_t log2m,
                                    double *__restrict__ out_values, int64_t *__restrict__ out_longs,
                                    uint8_t *__restrict__ out_hll) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ngroups; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t key = keys[i];
    for (int a = 0; a < naggs; a++) {
      const int kind = kinds[a];
      const uint64_t v = table[(int64_t)a * num_groups_dense + key];
      double d = 0.0;
      int64_t l = 0;
      switch (kind) {
        case ACC_COUNT: l = (int64_t)counts[key]; d = (double)l; break;
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
      const uint32_t *src = hll + ((int64_t)h * num_groups_dense + key) * m;
      uint8_t *dst = out_hll + (i * nhll + h) * m;
      for (int j = 0; j < m; j++) dst[j] = (uint8_t)src[j];
    }
  }
}

// ------------------------------------------------------------------------------------------------
// segment load transforms
// ------------------------------------------------------------------------------------------------
__global__ void bswap32_kernel(uint32_t *__restrict__ p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = __builtin_bswap32(p[i]);
}
__global__ void bswap64_kernel(uint64_t *__restrict__ p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = __builtin_bswap64(p[i]);
}

// Sorted forward index (BE (start,end) pairs) -> per-doc dict ids.
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
      // value bits occupy [d*bits, d*bits+bits); place the overlap with [b0, b1)
      int64_t vs = d * bits;
      uint64_t v = (uint32_t)ids[d];
      // shift so that value's MSB lands at stream position vs relative to b0 (bit 31 = b0)
      int64_t shift = 32 - (vs - (int64_t)b0) - bits;  // left shift amount into the word
      if (shift >= 0) w |= (uint32_t)(v << shift);
      else w |= (uint32_t)(v >> (-shift));
    }
    words[k] = w;
  }
}

// Roaring containers of the selected dict ids -> OR into dense u64 doc words.
__global__ __launch_bounds__(kBlock) void roaring_or_kernel(const RoaringTask *__restrict__ tasks, int32_t ntasks) {
  for (int ti = blockIdx.x; ti < ntasks; ti += gridDim.x) {
    const RoaringTask tk = tasks[ti];
    uint64_t *out = tk.out_words + (int64_t)tk.key * 1024;  // 65536 docs per container = 1024 words
    if (tk.kind == 0) {
      const uint16_t *v = (const uint16_t *)tk.payload;
      for (int i = threadIdx.x; i < tk.card; i += blockDim.x) {
        uint32_t x = v[i];
        atomicOr((unsigned long long *)&out[x >> 6], 1ull << (x & 63));
      }
    } else if (tk.kind == 1) {
      const uint64_t *w = (const uint64_t *)tk.payload;
      for (int i = threadIdx.x; i < 1024; i += blockDim.x) {
        uint64_t x = w[i];
        if (x) atomicOr((unsigned long long *)&out[i], x);
      }
    } else {
      const uint16_t *r = (const uint16_t *)tk.payload;
      const int nruns = tk.card;
      // each thread handles word-aligned pieces of the runs
      for (int ri = 0; ri < nruns; ri++) {
        uint32_t s = r[1 + 2 * ri], e = s + r[2 + 2 * ri];  // inclusive
        uint32_t ws = s >> 6, we = e >> 6;
        for (uint32_t wi = ws + threadIdx.x; wi <= we; wi += blockDim.x) {
          int lo = (wi == ws) ? (int)(s & 63) : 0;
          int hi = (wi == we) ? (int)(e & 63) : 63;
          uint64_t m = (hi == 63 ? ~0ull : ((1ull << (hi + 1)) - 1)) & ~((1ull << lo) - 1);
          atomicOr((unsigned long long *)&out[wi], m);
        }
      }
    }
  }
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

hipError_t launch_bswap32(uint32_t *p, int64_t n, hipStream_t s) {
  bswap32_kernel<<<grid_for(n), 256, 0, s>>>(p, n);
  return hipGetLastError();
}
hipError_t launch_bswap64(uint64_t *p, int64_t n, hipStream_t s) {
  bswap64_kernel<<<grid_for(n), 256, 0, s>>>(p, n);
  return hipGetLastError();
}
hipError_t launch_sorted_to_packed(const uint32_t *be_pairs, int32_t card, int32_t *ids_tmp, int64_t n, int32_t bits,
                                   uint32_t *words, int64_t nwords, hipStream_t s) {
  sorted_ids_kernel<<<grid_for(card, 1, 4096), 256, 0, s>>>(be_pairs, card, ids_tmp);
  pack_ids_kernel<<<grid_for(nwords), 256, 0, s>>>(ids_tmp, n, bits, words, nwords);
  return hipGetLastError();
}
hipError_t launch_fill_u64(uint64_t *p, int64_t n, uint64_t v, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  fill_u64_kernel<<<grid_for(n), 256, 0, s>>>(p, n, v);
  return hipGetLastError();
}
hipError_t launch_roaring_or(const RoaringTask *tasks, int32_t ntasks, hipStream_t s) {
  if (ntasks <= 0) return hipSuccess;
  roaring_or_kernel<<<ntasks < 8192 ? ntasks : 8192, kBlock, 0, s>>>(tasks, ntasks);
  return hipGetLastError();
}
template <int NA>
static hipError_t launch_scan_na(const DevQuery &q, int nblocks, size_t lds_bytes, bool group_by, hipStream_t s) {
  if (lds_bytes > 65536) {
    static bool configured = false;  // allow > 64 KiB dynamic LDS (gfx950: 160 KiB per workgroup)
    if (!configured) {
      hipError_t e1 = hipFuncSetAttribute((const void *)scan_kernel<NA, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
      hipError_t e2 = hipFuncSetAttribute((const void *)scan_kernel<NA, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
      if (e1 != hipSuccess) return e1;
      if (e2 != hipSuccess) return e2;
      configured = true;
    }
  }
  if (group_by) {
    scan_kernel<NA, true><<<nblocks, kBlock, lds_bytes, s>>>(q);
  } else {
    scan_kernel<NA, false><<<nblocks, kBlock, lds_bytes, s>>>(q);
  }
  return hipGetLastError();
}

hipError_t launch_scan(const DevQuery &q, int nblocks, size_t lds_bytes, bool group_by, hipStream_t s) {
  if (q.num_aggs <= 1) return launch_scan_na<1>(q, nblocks, lds_bytes, group_by, s);
  if (q.num_aggs <= 2) return launch_scan_na<2>(q, nblocks, lds_bytes, group_by, s);
  if (q.num_aggs <= 4) return launch_scan_na<4>(q, nblocks, lds_bytes, group_by, s);
  return launch_scan_na<8>(q, nblocks, lds_bytes, group_by, s);
}
hipError_t launch_finalize_partials(const uint64_t *partials, int nblocks, int nslots, const int32_t *kinds,
                                    uint64_t *out, hipStream_t s) {
  finalize_partials_kernel<<<nslots, 64, 0, s>>>(partials, nblocks, nslots, kinds, out);
  return hipGetLastError();
}
hipError_t launch_group_count(const uint64_t *counts, int64_t n, int32_t *chunk_counts, int64_t nchunks,
                              int64_t *offsets, hipStream_t s) {
  group_count_kernel<<<(unsigned)nchunks, kBlock, 0, s>>>(counts, n, chunk_counts);
  exclusive_scan_kernel<<<1, 64, 0, s>>>(chunk_counts, (int32_t)nchunks, offsets);
  return hipGetLastError();
}
hipError_t launch_group_compact(const uint64_t *counts, int64_t n, const int64_t *offsets, int64_t nchunks,
                                int64_t *keys, hipStream_t s) {
  group_compact_kernel<<<(unsigned)nchunks, kBlock, 0, s>>>(counts, n, offsets, keys);
  return hipGetLastError();
}
hipError_t launch_group_gather(const int64_t *keys, int64_t ngroups, int64_t ndense, int32_t naggs,
                               const int32_t *kinds, const uint64_t *table, const uint64_t *counts,
                               const uint32_t *hll, int32_t nhll, int32_t log2m, double *vals, int64_t *longs,
                               uint8_t *hll_out, hipStream_t s) {
  if (ngroups <= 0) return hipSuccess;
  group_gather_kernel<<<grid_for(ngroups), 256, 0, s>>>(keys, ngroups, ndense, naggs, kinds, table, counts, hll,
                                                       nhll, log2m, vals, longs, hll_out);
  return hipGetLastError();
}

}  // namespace phip
