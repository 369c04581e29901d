// kernels.hip -- gfx950 kernels of the segment query hot path.
//
// Layout in HBM (built at segment load, see runtime.cpp):
//   * fixed-bit dict-id forward index: u32 words, word k = BE bytes [4k, 4k+4) read as a big-endian
//     integer, so bit 31 of word k is stream bit 32k (FixedBitIntReader's MSB-first order,
//     pinot-segment-local/.../io/reader/impl/FixedBitIntReader.java:121-178). Doc d's id is bits
//     [d*b, d*b+b). A 64-doc group occupies exactly 2b words, a 4096-doc tile 128b words.
//   * dictionaries: LE typed arrays; raw columns: LE values.
//
// Execution model of the fused scan kernel (K1+K2+K5..K8 of SURVEY.md §2.4):
//   one wave = one tile of 64 groups x 64 docs. Leaves are evaluated with lanes = docs: each
//   lane decodes its doc's dict id and tests the predicate; __ballot returns the 64-doc bitmap word
//   of that group directly (SVScanDocIdIterator + PredicateEvaluator.applySV,
//   pinot-core/.../dociditerators/SVScanDocIdIterator.java:75-142). The word is parked in lane g
//   (lane g owns group g), so the boolean algebra of the filter tree (AndDocIdSet / OrDocIdSet /
//   NotDocIdSet) is per-lane u64 arithmetic, evaluated once per tile with "care" masks: a child of
//   an AND only decodes groups whose running AND is non-zero (the applyAnd candidate-doc semantics of
//   ScanBasedDocIdIterator.applyAnd, SVScanDocIdIterator.java:114-142), a child of an OR only those
//   not already true. Aggregation then revisits the groups with a non-zero final word, lanes = docs,
//   with inactive lanes masked.
#include <hip/hip_runtime.h>

#include "../../include/pinot_hip.h"
#include "device.h"

namespace phip {

// Query metadata (segments, columns, filter programs) is read through the constant address space so
// that it compiles to scalar loads (lgkmcnt): vector loads would be counted in vmcnt and every wait on
// them would also wait for the LDS-DMA prefetch of the next tile.
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

// Bits [off, off+bits) of the MSB-first stream held in words (u32, bit 31 first).
__device__ __forceinline__ uint32_t decode_bits(const uint32_t *__restrict__ words, uint32_t off,
                                                uint32_t bits) {
  const uint32_t *p = words + (off >> 5);
  uint64_t win = ((uint64_t)p[0] << 32) | (uint64_t)p[1];
  return (uint32_t)((win << (off & 31)) >> (64 - bits));
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

// Per-tile context of one wave.
struct Tile {
  int32_t doc0;            // first doc of the tile within the segment
  int32_t tile_in_seg;     // tile index within the segment
  uint32_t scanned;        // entries scanned in filter (lane-uniform)
  const uint8_t *stage;    // this wave's LDS stage buffer holding the tile's staged regions
};

typedef __attribute__((address_space(1))) const void gvoid_t;
typedef __attribute__((address_space(3))) void lvoid_t;

// Issue the LDS-DMA copies of one tile's staged regions (global_load_lds_dwordx4, 1 KiB per
// wave-instruction, no VGPR round trip). Completion is awaited with s_waitcnt vmcnt(0).
__device__ __forceinline__ void stage_tile(cseg_t &seg, int32_t tile_in_seg, uint8_t *buf) {
  const int lane = lane_id();
  for (int i = 0; i < seg.num_stage; i++) {
    const uint8_t *sbase = seg.stage[i].base;
    const int32_t sbytes = seg.stage[i].bytes;
    const int32_t soff = seg.stage[i].lds_off;
    const uint8_t *g = sbase + (int64_t)tile_in_seg * sbytes;
    uint8_t *l = buf + soff;
    for (int c = 0; c < sbytes; c += 1024) {
      if (c + lane * 16 < sbytes)
        __builtin_amdgcn_global_load_lds((gvoid_t *)(g + c + lane * 16), (lvoid_t *)(l + c), 16, 0, 0);
    }
  }
}

__device__ __forceinline__ void wait_stage() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Window of 32 stream bits starting at bit p of a staged region (u32 words, bit 31 first).
// q = floor((p-1)/32) may be -1 (reads the guard word before the region); s in [0, 31].
__device__ __forceinline__ uint32_t window_at(const uint32_t *w, int32_t p) {
  const int32_t q = (p - 1) >> 5;
  const uint32_t s = (uint32_t)(32 * (q + 1) - p);
  return __builtin_amdgcn_alignbit(w[q], w[q + 1], s);
}

__device__ __forceinline__ uint32_t col_dict_id_global(ccol_t &c, const Tile &t, uint32_t dit) {
  const uint32_t *w = c.words + (uint64_t)(t.doc0 >> 5) * (uint32_t)c.bits;
  return decode_bits(w, dit * (uint32_t)c.bits, (uint32_t)c.bits);
}

__device__ __forceinline__ uint32_t col_dict_id(ccol_t &c, const Tile &t, uint32_t dit) {
  if (c.lds_off >= 0) {
    const uint32_t *w = (const uint32_t *)(t.stage + c.lds_off);
    return window_at(w, (int32_t)(dit * (uint32_t)c.bits)) >> (32 - c.bits);
  }
  return col_dict_id_global(c, t, dit);
}

// ------------------------------------------------------------------------------------------------
// filter leaves
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t span_mask(int lo, int hi) {  // bits lo..hi inclusive, 0<=lo<=hi<=63
  uint64_t upto = (hi == 63) ? ~0ull : ((1ull << (hi + 1)) - 1);
  return upto & ~((1ull << lo) - 1);
}

__device__ __forceinline__ uint64_t eval_leaf(cseg_t *__restrict__ seg, cnode_t *__restrict__ n,
                                              uint64_t care, Tile *t) {
  const int lane = lane_id();
  const int kind = n->leaf_kind;
  if (kind == PHIP_LEAF_MATCH_ALL) return care;
  if (kind == PHIP_LEAF_MATCH_NONE) return 0;
  if (kind == PHIP_LEAF_DOC_RANGES) {
    const int32_t *r = (const int32_t *)n->aux;
    const int32_t cnt = n->count;
    const int32_t tile_end = t->doc0 + kTileDocs - 1;
    int a = 0, b = cnt;  // first range that may intersect the tile (ranges sorted & disjoint)
    while (a < b) {
      int mid = (a + b) >> 1;
      if (r[2 * mid + 1] < t->doc0) a = mid + 1; else b = mid;
    }
    const int32_t d0 = t->doc0 + lane * 64;
    uint64_t m = 0;
    for (int i = a; i < cnt; i++) {
      int32_t s = r[2 * i], e = r[2 * i + 1];
      if (s > tile_end) break;
      int lo = max(s, d0), hi = min(e, d0 + 63);
      if (lo <= hi) m |= span_mask(lo - d0, hi - d0);
    }
    return care & m;
  }
  if (kind == PHIP_LEAF_INVERTED) {
    uint64_t m;
    if (n->lds_off >= 0) {
      m = lane < kTileGroups ? ((const uint64_t *)(t->stage + n->lds_off))[lane] : 0ull;
    } else {
      const uint64_t *w = (const uint64_t *)n->aux;
      m = care ? w[(t->doc0 >> 6) + lane] : 0ull;
    }
    if (n->exclusive) m = ~m;
    return care & m;
  }
  // DICT_RANGE / DICT_SET on the bit-packed forward index: lanes = docs, one ballot per 64-doc group.
  ccol_t &c = seg->cols[n->column];
  const int32_t bits = c.bits;
  const bool is_range = kind == PHIP_LEAF_DICT_RANGE;
  const uint32_t *__restrict__ set = (const uint32_t *)n->aux;
  const bool excl = n->exclusive != 0;
  uint64_t res = 0;
  t->scanned += (uint32_t)__popcll(__ballot(care != 0)) * 64u;
  if (n->lds_off >= 0) {
    const uint32_t *w = (const uint32_t *)(t->stage + n->lds_off);
    // Range test on the MSB-aligned window: lo <= v < hi  <=>  (win - lo<<k) < (hi-lo)<<k, k = 32-b
    const uint32_t LO = (uint32_t)n->lo << (32 - bits);
    const uint32_t SPAN = (uint32_t)(n->hi - n->lo) << (32 - bits);
    const int32_t p0 = lane * bits;
#pragma unroll 8
    for (int g = 0; g < kTileGroups; g++) {
      const uint32_t win = window_at(w + g * 2 * bits, p0);
      bool pass;
      if (is_range) {
        pass = (win - LO) < SPAN;
      } else {
        const uint32_t v = win >> (32 - bits);
        pass = (((set[v >> 5] >> (v & 31)) & 1u) != 0) != excl;
      }
      const uint64_t m = ballot(pass);
      res = (lane == g) ? m : res;
    }
    return res & care;
  }
  // not staged (LDS budget exceeded): decode from HBM
  const uint32_t *__restrict__ w = c.words + (uint64_t)(t->doc0 >> 5) * (uint32_t)bits;
  const uint32_t lo = (uint32_t)n->lo;
  const uint32_t span = (uint32_t)(n->hi - n->lo);
  uint64_t need = ballot(care != 0);
  while (need) {
    const int g = __builtin_ctzll(need);
    need &= need - 1;
    const uint32_t v = decode_bits(w, (uint32_t)(g * 64 + lane) * (uint32_t)bits, (uint32_t)bits);
    bool pass;
    if (is_range) {
      pass = (v - lo) < span;
    } else {
      pass = (((set[v >> 5] >> (v & 31)) & 1u) != 0) != excl;
    }
    const uint64_t m = ballot(pass);
    if (lane == g) res = m;
  }
  return res & care;
}

// Filter program: the segment's tree in postfix order (runtime.cpp converts the preorder ABI tree),
// evaluated once per tile over per-lane group words with a small uniform-indexed register stack.
// Leaves see every valid doc of the tile; AND/OR/NOT combine 64-doc words (AndDocIdSet / OrDocIdSet /
// NotDocIdSet semantics: NOT complements within [0, numDocs)).
#define PHIP_PUSH(v)                  \
  do {                                \
    const uint64_t _v = (v);          \
    switch (sp) {                     \
      case 0: s0 = _v; break;         \
      case 1: s1 = _v; break;         \
      case 2: s2 = _v; break;         \
      case 3: s3 = _v; break;         \
      case 4: s4 = _v; break;         \
      default: s5 = _v; break;        \
    }                                 \
    sp++;                             \
  } while (0)
#define PHIP_POP(dst)                 \
  do {                                \
    sp--;                             \
    switch (sp) {                     \
      case 0: dst = s0; break;        \
      case 1: dst = s1; break;        \
      case 2: dst = s2; break;        \
      case 3: dst = s3; break;        \
      case 4: dst = s4; break;        \
      default: dst = s5; break;       \
    }                                 \
  } while (0)

__device__ __forceinline__ uint64_t eval_filter(cseg_t &seg, cnode_t *__restrict__ nodes, uint64_t valid,
                                                Tile &t) {
  uint64_t s0 = 0, s1 = 0, s2 = 0, s3 = 0, s4 = 0, s5 = 0;
  int sp = 0;
  for (int i = seg.node_begin; i < seg.node_end; i++) {
    cnode_t *n = nodes + i;
    const int op = n->op;
    if (op == PHIP_NODE_LEAF) {
      PHIP_PUSH(eval_leaf(&seg, n, valid, &t));
    } else if (op == PHIP_NODE_NOT) {
      uint64_t v;
      PHIP_POP(v);
      PHIP_PUSH(valid & ~v);
    } else {
      uint64_t v, w;
      PHIP_POP(v);
      for (int k = 1; k < n->num_children; k++) {
        PHIP_POP(w);
        v = (op == PHIP_NODE_AND) ? (v & w) : (v | w);
      }
      PHIP_PUSH(v);
    }
  }
  uint64_t r;
  PHIP_POP(r);
  return r;
}

// ------------------------------------------------------------------------------------------------
// aggregation expression values for one doc
// ------------------------------------------------------------------------------------------------
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
  if (kind == ACC_MIN_F64) return (uint64_t)__double_as_longlong(__builtin_huge_val());
  if (kind == ACC_MAX_F64) return (uint64_t)__double_as_longlong(-__builtin_huge_val());
  return 0;  // counts, int sums, f64 +0.0
}

// ------------------------------------------------------------------------------------------------
// fused filter + aggregate / group-by kernel
//   per wave: tiles of 2048 docs, grid-stride; every tile's staged regions (filter columns, value
//   columns, inverted-leaf words) arrive by LDS-DMA, double-buffered: tile i+stride is in flight while
//   tile i is evaluated from LDS.
// LDS: [HLL registers (aggregation-only)] [wave partials] [4 waves x nbuf x stage_stride]
// ------------------------------------------------------------------------------------------------
template <int NA, bool kGroupBy>
__global__ __launch_bounds__(kBlock) void scan_kernel(DevQuery q) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = lane_id();
  // wave-uniform by construction; readfirstlane tells the compiler, so every value derived from the
  // tile index (segment, offsets, metadata addresses) lives in SGPRs and metadata loads are scalar
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int waves_total = gridDim.x * (kBlock / 64);
  const int gwave = blockIdx.x * (kBlock / 64) + wave;
  const int nslots = q.num_aggs + 2;

  uint32_t *hll_lds = (uint32_t *)smem;
  int hll_words = 0;
  if (!kGroupBy && q.num_hll > 0) {
    hll_words = q.num_hll << q.aggs[0].log2m;  // all HLL aggs share log2m (host enforces)
    for (int i = threadIdx.x; i < hll_words; i += kBlock) hll_lds[i] = 0;
  }
  const int part_off = (hll_words * 4 + 15) & ~15;
  uint64_t *wave_part = (uint64_t *)(smem + part_off);
  uint8_t *stage_base = smem + part_off + ((kBlock / 64) * nslots * 8 + 15 & ~15) +
                        (size_t)wave * q.nbuf * q.stage_stride;
  __syncthreads();

  uint64_t acc[NA];
#pragma unroll
  for (int a = 0; a < NA; a++) acc[a] = (a < q.num_aggs) ? acc_init(q.aggs[a].acc) : 0;
  uint64_t matched = 0;
  uint32_t scanned = 0;

  cseg_t *segs = (cseg_t *)q.segs;
  cnode_t *nodes = (cnode_t *)q.nodes;
  auto seg_of = [&](int tile) {
    int lo = 0, hi = q.num_segs - 1;
    while (lo < hi) {
      int mid = (lo + hi + 1) >> 1;
      if (segs[mid].tile_begin <= tile) lo = mid; else hi = mid - 1;
    }
    return lo;
  };

  int cur = 0;
  int tile = gwave;
  if (tile < q.total_tiles) {
    const int s0 = seg_of(tile);
    stage_tile(segs[s0], tile - segs[s0].tile_begin, stage_base);
  }
  for (; tile < q.total_tiles; tile += waves_total) {
    const int si = __builtin_amdgcn_readfirstlane(seg_of(tile));
    cseg_t &seg = segs[si];
    Tile t;
    t.tile_in_seg = tile - seg.tile_begin;
    t.doc0 = t.tile_in_seg * kTileDocs;
    t.scanned = 0;
    t.stage = stage_base + cur * q.stage_stride;
    wait_stage();  // this tile's regions have landed
    const int next = tile + waves_total;
    if (q.nbuf == 2 && next < q.total_tiles) {
      const int sn = seg_of(next);
      stage_tile(segs[sn], next - segs[sn].tile_begin, stage_base + (cur ^ 1) * q.stage_stride);
    }

    // valid docs of group = lane
    const int32_t gdoc0 = t.doc0 + lane * 64;
    const int32_t rem = seg.num_docs - gdoc0;
    uint64_t mask = (lane >= kTileGroups) ? 0ull : (rem >= 64 ? ~0ull : (rem <= 0 ? 0ull : ((1ull << rem) - 1)));
    if (seg.node_end > seg.node_begin) mask = eval_filter(seg, nodes, mask, t);
    scanned += t.scanned;
    matched += __popcll(mask);
    {
      uint64_t tm = wave_reduce_u64_add((uint64_t)__popcll(mask));
      if (lane == 0 && tm) atomicAdd((unsigned long long *)&q.seg_matched[si], (unsigned long long)tm);
    }
    if (q.filter_out != nullptr && lane < kTileGroups && gdoc0 < seg.num_docs)
      q.filter_out[(t.doc0 >> 6) + lane] = mask;

    if (q.num_aggs > 0 || kGroupBy) {
      uint64_t groups = ballot(mask != 0);
      while (groups) {
        const int g = __builtin_ctzll(groups);
        groups &= groups - 1;
        const uint64_t m = readlane64(mask, g);
        if ((m >> lane) & 1) {
          const uint32_t dit = (uint32_t)(g * 64 + lane);
          if constexpr (kGroupBy) {
            int64_t key = 0;
            for (int k = 0; k < q.num_group_by; k++) {
              ccol_t &c = seg.cols[q.gb_cols[k]];
              uint32_t id = col_dict_id(c, t, dit);
              int32_t gid = c.remap ? c.remap[id] : (int32_t)id;
              key += (int64_t)gid * q.gb_stride[k];
            }
            atomicAdd((unsigned long long *)&q.gb_count[key], 1ull);
#pragma unroll
            for (int a = 0; a < NA; a++) {
              if (a >= q.num_aggs) break;
              const DevAgg &ag = q.aggs[a];
              uint64_t *slot = q.gb_table + (int64_t)a * q.num_groups + key;
              switch (ag.acc) {
                case ACC_COUNT: break;  // == gb_count
                case ACC_SUM_I64:
                  atomicAdd((unsigned long long *)slot, (unsigned long long)expr_i64(seg, ag, t, dit));
                  break;
                case ACC_SUM_F64: atomicAdd((double *)slot, expr_f64(seg, ag, t, dit)); break;
                case ACC_MIN_F64:
                  atomicMin((unsigned long long *)slot, (unsigned long long)f64_ordered(expr_f64(seg, ag, t, dit)));
                  break;
                case ACC_MAX_F64:
                  atomicMax((unsigned long long *)slot, (unsigned long long)f64_ordered(expr_f64(seg, ag, t, dit)));
                  break;
                case ACC_HLL: {
                  ccol_t &c = seg.cols[ag.col_a];
                  uint32_t h = c.hll[col_dict_id(c, t, dit)];
                  uint32_t *regs = q.gb_hll + ((int64_t)ag.hll_slot * q.num_groups + key) * (1 << ag.log2m);
                  atomicMax(&regs[h >> 8], (uint32_t)(h & 0xff));
                  break;
                }
              }
            }
          } else {
#pragma unroll
            for (int a = 0; a < NA; a++) {
              if (a >= q.num_aggs) break;
              const DevAgg &ag = q.aggs[a];
              switch (ag.acc) {
                case ACC_COUNT: acc[a] += 1; break;
                case ACC_SUM_I64: acc[a] += (uint64_t)expr_i64(seg, ag, t, dit); break;
                case ACC_SUM_F64:
                  acc[a] = (uint64_t)__double_as_longlong(__longlong_as_double((long long)acc[a]) +
                                                          expr_f64(seg, ag, t, dit));
                  break;
                case ACC_MIN_F64:
                  acc[a] = (uint64_t)__double_as_longlong(
                      fmin(__longlong_as_double((long long)acc[a]), expr_f64(seg, ag, t, dit)));
                  break;
                case ACC_MAX_F64:
                  acc[a] = (uint64_t)__double_as_longlong(
                      fmax(__longlong_as_double((long long)acc[a]), expr_f64(seg, ag, t, dit)));
                  break;
                case ACC_HLL: {
                  ccol_t &c = seg.cols[ag.col_a];
                  uint32_t h = c.hll[col_dict_id(c, t, dit)];
                  atomicMax(&hll_lds[(ag.hll_slot << ag.log2m) + (h >> 8)], (uint32_t)(h & 0xff));
                  break;
                }
              }
            }
          }
        }
      }
    }
    if (q.nbuf == 1 && next < q.total_tiles) {
      const int sn = seg_of(next);
      stage_tile(segs[sn], next - segs[sn].tile_begin, stage_base);
    }
    cur ^= (q.nbuf == 2) ? 1 : 0;
  }
  wait_stage();

  // ---- block reduction of the partials ---------------------------------------------------------
#pragma unroll
  for (int a = 0; a < NA; a++) {
    if (a >= q.num_aggs) break;
    const int kind = q.aggs[a].acc;
    uint64_t v;
    if (kind == ACC_COUNT || kind == ACC_SUM_I64 || kind == ACC_HLL) {
      v = wave_reduce_u64_add(acc[a]);
    } else {
      v = (uint64_t)__double_as_longlong(wave_reduce_f64(__longlong_as_double((long long)acc[a]), kind));
    }
    if (lane == 0) wave_part[wave * nslots + a] = v;
  }
  {
    uint64_t m = wave_reduce_u64_add(matched);
    if (lane == 0) {
      wave_part[wave * nslots + q.num_aggs] = m;
      wave_part[wave * nslots + q.num_aggs + 1] = scanned;
    }
  }
  __syncthreads();
  if (threadIdx.x < nslots) {
    const int a = threadIdx.x;
    uint64_t v = wave_part[a];
    for (int w = 1; w < kBlock / 64; w++) {
      uint64_t x = wave_part[w * nslots + a];
      int kind = a < q.num_aggs ? q.aggs[a].acc : ACC_COUNT;
      if (kind == ACC_SUM_F64) {
        v = (uint64_t)__double_as_longlong(__longlong_as_double((long long)v) + __longlong_as_double((long long)x));
      } else if (kind == ACC_MIN_F64) {
        v = (uint64_t)__double_as_longlong(fmin(__longlong_as_double((long long)v), __longlong_as_double((long long)x)));
      } else if (kind == ACC_MAX_F64) {
        v = (uint64_t)__double_as_longlong(fmax(__longlong_as_double((long long)v), __longlong_as_double((long long)x)));
      } else {
        v += x;
      }
    }
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
  for (int b = lane; b < nblocks; b += 64) {
    uint64_t x = partials[(int64_t)b * nslots + a];
    if (kind == ACC_SUM_F64) {
      v = (uint64_t)__double_as_longlong(__longlong_as_double((long long)v) + __longlong_as_double((long long)x));
    } else if (kind == ACC_MIN_F64) {
      v = (uint64_t)__double_as_longlong(fmin(__longlong_as_double((long long)v), __longlong_as_double((long long)x)));
    } else if (kind == ACC_MAX_F64) {
      v = (uint64_t)__double_as_longlong(fmax(__longlong_as_double((long long)v), __longlong_as_double((long long)x)));
    } else {
      v += x;
    }
  }
  if (fp) {
    v = (uint64_t)__double_as_longlong(wave_reduce_f64(__longlong_as_double((long long)v), kind));
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
static void launch_scan_na(const DevQuery &q, int nblocks, size_t lds, bool group_by, hipStream_t s) {
  if (group_by) {
    scan_kernel<NA, true><<<nblocks, kBlock, lds, s>>>(q);
  } else {
    scan_kernel<NA, false><<<nblocks, kBlock, lds, s>>>(q);
  }
}

hipError_t launch_scan(const DevQuery &q, int nblocks, size_t lds_bytes, bool group_by, hipStream_t s) {
  if (lds_bytes > 65536) {
    static bool configured = false;  // allow > 64 KiB dynamic LDS (gfx950: 160 KiB per workgroup)
    if (!configured) {
      hipFuncSetAttribute((const void *)scan_kernel<1, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
      hipFuncSetAttribute((const void *)scan_kernel<2, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
      hipFuncSetAttribute((const void *)scan_kernel<4, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
      hipFuncSetAttribute((const void *)scan_kernel<8, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
      hipFuncSetAttribute((const void *)scan_kernel<1, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
      hipFuncSetAttribute((const void *)scan_kernel<2, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
      hipFuncSetAttribute((const void *)scan_kernel<4, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
      hipFuncSetAttribute((const void *)scan_kernel<8, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
      configured = true;
    }
  }
  if (q.num_aggs <= 1) launch_scan_na<1>(q, nblocks, lds_bytes, group_by, s);
  else if (q.num_aggs <= 2) launch_scan_na<2>(q, nblocks, lds_bytes, group_by, s);
  else if (q.num_aggs <= 4) launch_scan_na<4>(q, nblocks, lds_bytes, group_by, s);
  else launch_scan_na<8>(q, nblocks, lds_bytes, group_by, s);
  return hipGetLastError();
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
