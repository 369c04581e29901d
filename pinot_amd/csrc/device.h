// device.h -- structures shared by the host runtime (runtime.cpp) and the gfx950 kernels
// (filter.hip, aggregate.hip, load.hip). Plain POD, identical layout on host and device.
#pragma once
#include <stdint.h>

namespace phip {

constexpr int kMaxQueryColumns = 16;  // distinct columns one query may reference
constexpr int kMaxAggs = 8;           // aggregation slots per query
constexpr int kRecKeys = 4;            // group-by record: key fields (DevSeg.rec)
constexpr int kRecFields = kRecKeys + 2 * kMaxAggs;  // ... and up to two inputs per aggregation
// One field's source for materialize_record_kernel: a fixed-bit stream (dictionary ids / packed values, `bits` per
// doc), or doc-order u16 / u32 entries (HLL); placed at bit `off` of the doc's record.
enum { REC_BITS = 0, REC_U16 = 1, REC_U32 = 2 };
struct RecSrc {
  const void *p;
  int32_t kind, bits, off, pad;
};
struct RecSrcs {
  RecSrc f[kRecFields];
};
constexpr int kMaxPrograms = 8;       // filter programs per query (filtered aggregations in one pass)
constexpr int kDenseMin = 640;        // default DevAggQuery::dense_min
constexpr int kDoneSlot = 63;         // finals[kDoneSlot] of a plan's mapped result area: the execution's completion word
constexpr int kMaxFilterStack = 6;    // postfix evaluation stack depth (host rejects deeper programs)
constexpr int kMaxGroupBy = 8;  // GROUP BY columns (the mixed-radix key space stays below 2^62)
constexpr int kWave = 64;             // CDNA wavefront
constexpr int kTileGroups = 32;       // 64-doc groups per tile: bit (31-g) of lane l's mask word = doc 64g+l
constexpr int kTileDocs = kTileGroups * 64;  // 2048 docs per tile
constexpr int kMaxStage = 8;          // LDS-staged filter sources (scan columns / inverted leaves) per segment (SGPR budget of the cursor)
constexpr int kStagePad = 16;         // guard bytes before and after every staged region
constexpr int kMaxHllRegs = 1 << 12;  // log2m <= 12 on the GPU path

// filter kernel: 4 waves per workgroup, each wave streams its own contiguous range of tiles
constexpr int kFilterBlock = 256;
constexpr int kFilterWaves = kFilterBlock / kWave;
constexpr int kMaxRing = 8;           // LDS-DMA ring slots per wave
constexpr int kFusedRingTile = 512;   // fused aggregation, per-tile mode: u16 tile-relative doc ids per wave
#ifndef PHIP_FUSED_RING_DEFER
#define PHIP_FUSED_RING_DEFER 512  // (A/B builds override it)
#endif
constexpr int kFusedRingDefer = PHIP_FUSED_RING_DEFER;  // fused aggregation, deferred mode: u32 segment doc ids per wave (one batch
                                      // + an eighth of a tile)
// aggregation kernel: 8 waves per workgroup
constexpr int kAggBlock = 512;
constexpr int kAggWaves = kAggBlock / kWave;
// per-wave ring of matched doc ids (u32): GB_NONE batches up to 4 chunks; a tile's docs enter it in
// quarter-tile pieces of <= 512 after the ring was drained below one batch, so it holds one batch + 512; the
// group-by walks take one chunk at a time (their LDS goes to the table)
#ifndef PHIP_KBATCH
#define PHIP_KBATCH 4  // agg_common.h kBatch (A/B builds override it)
#endif
constexpr int kRingAgg = PHIP_KBATCH <= 4 ? 1024 : 2048;  // power of two >= 64 * kBatch + 512
constexpr int kRingGroup = 128;
// the batched group-by walk (GB_LDS / GB_GLOBAL, DevAggQuery::dense_batch): kBatch chunks per gather round
// trip like GB_NONE, a tile entering in eighth-tile pieces of <= 256 docs (its LDS goes to the table)
constexpr int kRingGroupBatch = PHIP_KBATCH <= 4 ? 512 : 1024;  // power of two >= 64 * kBatch + 256
// fused group-by (filter_kernel.h fused_defer_gb): u32 segment doc ids per wave, flushed 128 at a time; 1 KiB per wave
// instead of the deferred aggregation's 2 KiB keeps a resident workgroup the LDS-DMA ring would otherwise lose
constexpr int kFusedRingGB = 256;
constexpr int kFusedBatchGB = 2;
constexpr int ring_entries(int mode, bool batched = false) {
  return mode == 0 ? kRingAgg : (batched ? kRingGroupBatch : kRingGroup);
}
constexpr int kMaxAggStage = 4;      // staged aggregation columns
constexpr int kAggStageBudget = 4096; // LDS bytes per wave for them
constexpr int kAggLdsDict = 1024;     // dictionaries up to this many bytes are copied next to them

// Accumulator kinds of one aggregation slot.
enum AccKind : int32_t {
  ACC_COUNT = 0,    // int64 count
  ACC_SUM_I64 = 1,  // exact int64 sum (INT/LONG inputs)
  ACC_SUM_F64 = 2,  // double sum
  ACC_MIN_F64 = 3,
  ACC_MAX_F64 = 4,
  ACC_HLL = 5,      // registers, per (group, hll slot)
};

// Device filter-program opcodes (postfix; AND/OR are binary and applied incrementally, so a child
// can be skipped once the running value decides the node: AndDocIdSet / OrDocIdSet short-circuit).
enum DevOp : int32_t { DOP_LEAF = 0, DOP_AND = 1, DOP_OR = 2, DOP_NOT = 3 };
enum SkipKind : int32_t { SKIP_NONE = 0, SKIP_IF_NONE = 1, SKIP_IF_ALL = 2 };

// Group-by table placement (aggregate kernel).
enum GroupMode : int32_t {
  GB_NONE = 0,    // aggregation only: per-lane accumulators -> per-block partials
  GB_LDS = 1,     // per-workgroup table in LDS -> per-block slab in HBM -> fixed-order reduction
  GB_GLOBAL = 2,  // one table in HBM, global atomics
  GB_HASH = 3,    // key space too large for a dense table: open-addressing hash in HBM (slot = group),
                  // IntMapBasedHolder's role (DictionaryBasedGroupKeyGenerator.java:416-495)
  GB_XCD = 4,     // fused group-by only (filter_kernel.h): kXcdCopies XCD-private copies of the GB_GLOBAL table, each
                  // updated by one XCD's waves with workgroup-scope atomics (performed in that XCD's L2, not at the
                  // memory side), merged into copy 0 by xcd_merge_kernel; the plan's mode stays GB_GLOBAL
};
constexpr int kXcdCopies = 8;  // MI355X: 8 XCDs (HW_REG_XCC_ID & 7)
constexpr uint64_t kHashEmpty = ~0ull;  // empty key slot (mixed-radix keys are < 2^62)

// One column as seen by one segment of a query.
struct DevCol {
  const uint32_t *words;  // fixed-bit dict ids: u32 words holding the BE stream (bit 31 = first bit)
  const void *dict;       // LE typed dictionary (INT/LONG/FLOAT/DOUBLE), null for STRING
  const void *raw;        // LE raw values for no-dictionary columns
  const int32_t *remap;   // segment dict id -> query-global id (group-by), null = identity
  const uint32_t *hll;    // per dict id (register << 8) | rho, for DISTINCTCOUNTHLL
  int32_t bits;
  int32_t card;
  int32_t type;      // PHIP_TYPE_*
  int32_t has_dict;  // 1: dictionary-encoded; 0: raw
  int32_t lds_off;   // filter kernel: byte offset of this column's tile region in the stage slot, -1 = not staged
  int32_t hll_rows;  // > 0: `raw` holds 2^hll_rows u8 HLL registers per doc (star-tree DISTINCTCOUNTHLL pair)
  const uint64_t *str_off;  // raw STRING: doc d's UTF-8 bytes are raw[str_off[d] .. str_off[d+1])
  const uint32_t *planes;   // bit-sliced copy of `words` (bits <= kBitSliceMaxBits), or null: per 2048-doc tile,
                            // plane k (bit bits-1-k of the id) as 64 lane words, bit 31-g of lane l = doc 64g + l
  int64_t gb_base;          // raw INT / LONG group-by column: its key id = value - gb_base
  const uint32_t *hll_doc;  // DISTINCTCOUNTHLL: doc-order copy of `hll` (entry of doc d = hll[id(d)]), or null
  const uint16_t *hll_doc16;  // ... packed to 16 bits, (register << 5) | rho (log2m <= 11), when hll_doc is null
  const uint64_t *gb_nulls; // null-key group-by column (phip_query_desc.null_group_by): its null doc words (bit d % 64
                            // of word d / 64); a null doc's key id is gb_null_id. null = no null key
  int64_t gb_null_id;
  const int32_t *gb_ids;    // raw FLOAT / DOUBLE group-by column: doc-order key ids (keys.hip), or null
  const uint32_t *vpack;    // has_dict == 0, INT / LONG: doc-order values bit-packed (value - vbase in vbits bits,
  int64_t vbase;            // the forward index's layout), or null: `raw` holds them typed
  int32_t vbits;
  int32_t vpad;
};
constexpr int kBitSliceMaxBits = 12;

// One group-by column's key id source for the tuple packing of key spaces above 2^62 (keys.hip tuple_words_kernel).
constexpr int kMaxTupleCols = 8;
constexpr int kMaxTupleWords = 4;
struct TupleCol {
  const uint32_t *words;  // dictionary ids (null: raw INT / LONG values in `raw`, or `ids`)
  const int32_t *remap;   // segment dict id -> query-global id, null = identity
  const int32_t *ids;     // doc-order global ids (raw FLOAT / DOUBLE / STRING keys), or null
  const void *raw;
  const uint64_t *nulls;  // null docs (their id = null_id), or null
  int64_t base;           // raw INT / LONG: id = value - base
  int64_t null_id;
  uint64_t stride;        // the column's place in its word's mixed radix
  int32_t bits;
  int32_t type;
  int32_t word;
  int32_t pad;
};
struct TupleCols {
  TupleCol cols[kMaxTupleCols];
  int32_t k;  // columns
  int32_t w;  // words
};

// One source the filter wave copies into its LDS stage slot for every tile (LDS-DMA, 1 KiB per
// wave-instruction): a fixed-bit filter column (256*b bytes per 2048-doc tile) or the dense doc words of
// an inverted leaf (256 bytes per tile).
struct StageSrc {
  const uint8_t *base;  // tile t starts at base + t * bytes
  int32_t bytes;        // per tile, multiple of 16
  int32_t lds_off;      // region offset in the stage slot
};

// A leaf of a conjunctive filter program (fast path): a staged scan of one fixed-bit column.
#ifndef PHIP_MAX_CONJ
#define PHIP_MAX_CONJ 6  // (A/B builds override it)
#endif
constexpr int kMaxConj = PHIP_MAX_CONJ;
constexpr int kConjSparseMax = 6;     // default per-lane bound of the sparse conjunction walk
constexpr double kConjSparseSel = 1.0 / 16;  // ... taken only when the first leaf's selectivity is at most this
struct ConjLeaf {
  int32_t lds_off;  // staged region in the ring slot
  int32_t bits;
  int32_t kind;     // 0: dict-id range, 1: dict-id set over card <= 64, 2: dict-id range over the bit-sliced planes,
                    // 3: a few ids (set_mask) over the bit-sliced planes, 4: OR of <= 4 id runs over the bit-sliced
                    // planes (runs 0 / 1 in set_mask's halves, run 2 in lo, run 3 in span, pad = number of runs)
  uint32_t lo;      // range: lo << (32 - bits); bit-sliced: the first id of the range
  uint32_t span;    // range: (hi - lo) << (32 - bits); bit-sliced: the last id of the range (inclusive)
  int32_t pad;      // bit-sliced: 1 = lower bound to test, 2 = upper bound to test
  uint64_t set_mask;
};

// One segment with work in this query. Its tiles [tile0, tile0 + num_work) are global work items
// [work_begin, work_begin + num_work): tiles outside the candidate doc range of a sorted-index leaf
// under the root AND are never visited (SortedIndexBasedFilterOperator prunes them on the CPU too).
struct DevSeg {
  int32_t num_docs;
  int32_t work_begin;
  int32_t tile0;
  int32_t num_work;
  int32_t node_begin;  // filter nodes [node_begin, node_end); empty = match all
  int32_t node_end;
  int32_t num_stage;
  int32_t seg_index;   // slot of seg_matched: program * num query segments + index into the query's segment list
  int32_t num_dma;     // LDS-DMA wave-instructions per tile (sum of ceil(stage bytes / 1 KiB))
  int32_t conj;        // > 0: the program is AND of `conj` staged scan leaves (conj_leaf, most selective
                       // first); the filter kernel evaluates it without the stack machine
  int32_t conj_p;      // docs per lane-window of the fast path (1, 2, 4, 8; P * bits <= 32 for every leaf)
  int32_t conj_sparse;  // > 0: leaves 2.. are dict-id ranges, so a tile whose first leaf passes at most
                        // this many docs per lane tests them per passing doc (SVScanDocIdIterator.applyAnd)
                        // instead of per doc
  int32_t conj_path;    // 1: the segment's program takes the conjunctive path (conj >= 0 scan leaves, plus the
                        // optional doc range below); 0: the postfix interpreter
  int32_t conj_range;   // 1: AND with the doc range [conj_lo, conj_hi] (single-range sorted-index leaves,
  int32_t conj_lo;      // SortedIndexBasedFilterOperator; tiles outside it are pruned on the host, so only the
  int32_t conj_hi;      // boundary tiles are masked)
  int32_t contig;       // 1: general program evaluated in the contiguous layout (filter.hip eval_filter_contig);
                        // every leaf staged or tile-free (MATCH_*, DOC_RANGES)
  int32_t program;      // filter program of this entry: a plan with k programs (filtered aggregations) holds one
                        // entry per (segment, program), adjacent per segment; the aggregation kernel applies only
                        // the functions of that program (DevAgg.program) to its docs
  int32_t fused_defer;  // fused aggregation, no value column streamed with the tile (sparse program): matched docs
                        // collect across tiles in the wave's ring and their columns are gathered from HBM once
                        // per kFusedBatch x 64 docs (the gathers do not stall the stream every tile)
  int32_t conj_bs;      // 1: every conj leaf is a bit-sliced range (kind 2, staged planes); the AND is computed in
                        // the lane-major tile layout directly
  ConjLeaf conj_leaf[kMaxConj];
  StageSrc stage[kMaxStage];
  DevCol cols[kMaxQueryColumns];
  // (after the columns: the hot walks' column descriptors keep their scalar-cache alignment -- with these fields
  // ahead of them, Q3.1's batched walk, which reads no record, ran 0.47 -> 0.53 ms)
  // Group-by record (Segment::records, materialize_record_kernel): every field a matched doc's group-by update reads
  // -- its key ids, its aggregations' packed values / value ids, its HLL entries -- packed into rec_words u32 per doc
  // (field f at bits [rec_off[f], rec_off[f] + rec_bits[f]) of the doc's record, LSB first), so a doc costs one
  // gather instead of one per column. null = the columns' own layouts.
  const uint32_t *rec;
  int32_t rec_words;
  int32_t rec_nf;
  uint8_t rec_off[kRecFields];
  uint8_t rec_bits[kRecFields];
};

struct DevNode {
  int32_t op;         // DevOp
  int32_t leaf_kind;  // PHIP_LEAF_*
  int32_t column;
  int32_t lo, hi;     // DICT_RANGE [lo, hi)
  int32_t exclusive;
  int32_t count;
  int32_t skip_to;    // first node after the enclosing child's AND/OR when the short-circuit holds
  int32_t skip_kind;  // SkipKind
  int32_t lds_off;    // staged region of the leaf's column / inverted words, -1 = not staged
  int32_t bits;       // scan leaves: bits per value of the column
  int32_t small_set;  // DICT_SET with card <= 64: membership in set_mask
  int32_t aux_stride; // INVERTED: u64 words per 2048-doc tile in aux (32 x the entry's inverted leaves, interleaved)
  uint64_t set_mask;
  int32_t bs_nruns;   // DICT_SET: its ids (complement taken when exclusive) as 1..kBitSliceRuns runs of consecutive ids,
  uint32_t bs_runs[4];  // run r = [bs_runs[r] & 0xffff, bs_runs[r] >> 16] (the bit-sliced conjunction's OR of ranges);
                        // 0 = more runs than that
  const void *aux;    // DICT_SET: u32 bitset over dict ids; DOC_RANGES: int32 pairs;
                      // INVERTED: u64 doc bitmap words of the segment (materialised);
                      // RAW_RANGE: phip_raw_range; RAW_SET: `count` int64 / double values
};

// The per-execution results of an aggregation-only plan (what finalize_all_kernel computes), produced instead by the
// last workgroup of the plan's last kernel (agg_common.h finalize_tail): fixed-order reductions of the per-block
// partials, the per-segment matched counts and the HLL registers, written into the plan's mapped pinned area and
// the device counters zeroed for the next execution -- one launch and its dispatch gap fewer per query.
constexpr int kFinShards = 16;
constexpr size_t kFinCounterBytes = 64 * (1 + kFinShards);
struct DevFinal {
  const uint64_t *pa;   // aggregation partials [nba][na], or null
  const int32_t *ka;    // their accumulator kinds
  const uint64_t *pf;   // filter partials [nbf][2] (matched docs, entries scanned), or null
  const int32_t *kf;
  uint64_t *segm;       // [nseg] matched docs per (program, segment) entry
  uint32_t *hll;        // [hll_words] registers (aggregation only)
  uint64_t *out;        // pinned: [0, na) slots, [32, 34) filter sums, [64, 64 + nseg) segm, then the registers
  uint32_t *counter;    // [0]: shards complete; [16 (1 + k)]: workgroups done in shard k (blockIdx % kFinShards),
                        // each on its own 64-B line; the last shard's completer finalizes and resets them
  int32_t nba, na, nbf, nseg, hll_words, pad;
};

// Filter kernel launch (K1-K4 of SURVEY.md §2.4).
struct DevFilter {
  const DevSeg *segs;
  const DevNode *nodes;
  int32_t num_segs;
  int32_t total_work;
  int32_t stage_stride;  // bytes of one ring slot (max over segments), multiple of 16
  int32_t nbuf;          // ring slots per wave (2..kMaxRing): nbuf-1 tiles in flight while one is evaluated
  int32_t xcd_walk;      // 1: XCD-sweep tile order; 2: XCD ranges cut into contiguous per-wave ranges (grid multiple
                         // of 8 for both); 0: contiguous range per wave
  int32_t min_dma;       // min over segments of LDS-DMA wave-instructions per tile (vmcnt lower bound)
  int32_t probe;         // measurement only (PHIP_FILTER_PROBE): 1 = stream the tiles, skip the evaluation
  int32_t contig_inline;  // 1: range scans of the contiguous evaluator inline (0: through contig_scan_any; A/B)
  uint32_t stats_programs;  // programs whose scans count as entries scanned in filter (bit p = program p)
  int32_t mask_nt;          // tile masks stored non-temporally (PHIP_MASK_NT measurement switch)
  uint32_t *mask_out;    // optional: [total_work][64] lane-major tile masks
  uint64_t *partials;    // [num_blocks][2]: matched docs, entries scanned in filter
  uint64_t *seg_matched; // [num query segments]
  // fused aggregation (conjunctive programs, no group-by / HLL): the filter kernel projects and aggregates
  // each tile's matched docs itself, reading staged columns from the tile's ring slot (DevCol.lds_off)
  const struct DevAggQuery *agg;  // device copy of the aggregation descriptor, null = not fused
  uint64_t *agg_partials;         // [num_blocks][num_aggs]
  int32_t fring_bytes;            // per-wave matched-doc ring (fused): 4 * kFusedRingDefer when a segment defers,
  int32_t pad_f;                  // else 2 * kFusedRingTile
  const DevFinal *fin;            // non-null: this launch is the plan's last; its last workgroup finalizes
};

struct DevAgg {
  int32_t acc;       // AccKind
  int32_t expr;      // PHIP_EXPR_*
  int32_t col_a;
  int32_t col_b;
  int32_t integral;  // expression evaluated in int64 (both inputs INT/LONG)
  int32_t hll_slot;  // ACC_HLL: index among HLL aggs
  int32_t log2m;
  int32_t program;   // filter program whose docs it aggregates (DevSeg.program; multi-program plans)
};

// Aggregation / group-by kernel launch (K5-K9).
struct DevAggQuery {
  const DevSeg *segs;
  int32_t num_segs;
  int32_t total_work;
  const uint32_t *mask;  // [total_work][64] lane-major tile masks from the filter kernel; null = all docs
  int32_t num_aggs;
  int32_t num_hll;
  int32_t log2m;         // shared by all HLL aggs (host enforces)
  int32_t mode;          // GroupMode
  DevAgg aggs[kMaxAggs];
  // group-by
  int32_t num_group_by;
  int32_t gb_cols[kMaxGroupBy];
  int32_t dense_batch;    // GB_NONE: dense tiles take the batched lane-major walk (small dictionaries);
                          // GB_LDS / GB_GLOBAL: the batched group-by walk (kBatch chunks per gather round trip)
  int64_t gb_stride[kMaxGroupBy];  // mixed radix, column 0 least significant
  int64_t num_groups;     // dense key space size
  int32_t tbl_words;      // GB_LDS: u64 words of one workgroup table = num_groups * (1 + num_aggs)
  int32_t hll_words;      // GB_LDS: u32 words of one workgroup's packed HLL registers = groups*nhll*m/4
  uint64_t *gb_table;     // GB_GLOBAL: [1 + num_aggs][num_groups] (row 0 = counts); GB_LDS: [blocks][tbl_words] slab
  uint32_t *gb_hll;       // GB_GLOBAL: [nhll][num_groups][m] u32; GB_LDS: [blocks][hll_words] packed u8x4 slab
  // aggregation only
  uint64_t *partials;     // [num_blocks][num_aggs]
  uint32_t *hll_regs;     // [nhll][m] u32 (atomicMax from every block)
  // dense-tile staging (GB_NONE, dense_batch): the tile's fixed-bit words of each staged column are
  // LDS-DMA-ed into the wave's stage region, so the ids of all 2048 docs cost one memory round trip
  int32_t stage_bytes;    // per wave (0 = no staging)
  int32_t num_stage;
  int32_t stage_col[kMaxAggStage];
  int32_t stage_off[kMaxAggStage];  // region of staged column k in the wave's stage area (kStagePad guards)
  int32_t stage_dict_off[kMaxAggStage];  // the column's dictionary copied into the stage area, -1 = HBM
  int32_t stage_slot_a[kMaxAggs];   // staged slot of aggs[a].col_a / col_b, -1 = read from HBM
  int32_t stage_slot_b[kMaxAggs];
  // GB_HASH: num_groups = capacity (power of two); gb_table / gb_hll are indexed by slot
  uint64_t *gb_keys;        // [capacity] mixed-radix key of each slot, kHashEmpty = free
  uint32_t *hash_overflow;  // set to 1 when a probe sequence found no slot (host reports an error)
  // numGroupsLimit pass (limit.hip): GB_HASH over composite keys key * seg_key_mult + segment index, and
  // the first matched doc of every slot (atomicMin) -- the reference's per-segment first-seen order
  int32_t seg_keys;
  int32_t seg_key_mult;
  uint32_t *first_doc;
  int32_t dense_min;  // GB_NONE + dense_batch: matched docs per 2048-doc tile from which the batched walk is used
  int32_t own_count_rows;  // group-by over several filter programs (FILTER + GROUP BY): every COUNT counts its own
                           // program's docs in its own row 1 + a (row 0 counts the docs of every program: presence)
  const DevFinal *fin;     // GB_NONE: non-null when this launch is the plan's last (agg_common.h finalize_tail)
  int32_t wg_waves;        // waves per workgroup of the launch (kAggWaves; 16 for a GB_LDS table that leaves one
  int32_t rec_on;          // 8-wave workgroup per CU) | 1: some segment has a group-by record (agg_kernel R variant)
  int64_t xcd_words;       // GB_XCD: u64 words of one table copy ((1 + num_aggs) x num_groups)
  int64_t xcd_hll_words;   // GB_XCD: u32 words of one copy's HLL registers (num_hll x num_groups x m)
  int8_t rec_fa[kMaxAggs];  // group-by record (DevSeg.rec): the field of aggregation a's input a / b / HLL entry
  int8_t rec_fb[kMaxAggs];  // (-1: none; the key columns are fields 0 .. num_group_by - 1)
  // GB_NONE id histogram (agg_kernel kHist): the aggregations in hist_aggs (SUM / MIN / MAX of one small-dictionary
  // INT / LONG column, hist_col) count the docs per dictionary id in per-wave LDS bins (two u16 per u32 word,
  // hist_words per wave) and fold count x value into their accumulators when a segment ends -- no dictionary gather
  uint32_t hist_aggs;
  int32_t hist_col;
  int32_t hist_words;
  int32_t hist_pad;
};

// Selection (row-returning) queries (select.hip): SelectionOnlyOperator per segment + the combine's concatenation.
constexpr int kMaxSelect = 16;  // select expressions per query
enum SelKind : int32_t {
  SEL_I64 = 0,  // INT / LONG column: the value as int64
  SEL_F64 = 1,  // FLOAT / DOUBLE column, or an arithmetic expression (evaluated in double, as the transform
                // functions do): the value as double bits
  SEL_ID = 2,   // STRING column: the id in the query-global dictionary (DevCol.remap)
  SEL_STR = 3,  // raw STRING column: the row's locator (segment entry << 32 | doc); its bytes are gathered after
};
struct DevSelect {
  int32_t expr;  // PHIP_EXPR_*
  int32_t col_a;
  int32_t col_b;
  int32_t kind;  // SelKind
};
struct DevSelQuery {
  const DevSeg *segs;
  int32_t num_segs;
  int32_t total_work;
  const uint32_t *mask;      // [total_work][64] lane-major tile masks of the filter kernel; null = every doc
  const int64_t *tile_off;   // [total_work + 1] exclusive prefix of matched docs per work tile
  const int64_t *seg_base;   // [num_segs + 1] first output row of each entry (its kept rows follow in doc order)
  int64_t limit;             // rows kept per segment (SelectionOnlyOperator._numRowsToKeep) and in total
  int32_t num_select;
  int32_t pad;
  DevSelect sel[kMaxSelect];
};

// ORDER BY on group-by columns for the device trim (trim.hip)
constexpr int kMaxOrderKeys = 8;
struct KeyOrder {
  int32_t num_group_by;
  int32_t num_keys;
  int32_t gb[kMaxOrderKeys];    // group-by index of ORDER BY expression j
  int32_t desc[kMaxOrderKeys];
  int64_t card[kMaxOrderKeys];  // query-global cardinality of group-by column k
};

// General ORDER BY for the device trim (trim.hip, launch_trim_order_terms): up to kMaxOrderKeys terms, each a
// group-by column or the final result of an aggregation (TableResizer's GroupByExpressionExtractor /
// AggregationFunctionExtractor), sorted least significant term first with stable radix passes.
enum OrderTermKind : int32_t { TERM_GROUP_KEY = 0, TERM_VALUE = 1, TERM_AVG = 2, TERM_RANGE = 3, TERM_HLL = 4 };
struct OrderTerms {
  int32_t num_group_by;
  int32_t num_terms;
  int64_t card[kMaxOrderKeys];   // query-global cardinality of group-by column k
  int32_t kind[kMaxOrderKeys];   // OrderTermKind
  int32_t a[kMaxOrderKeys];      // group-by index (GROUP_KEY), value slot (VALUE), SUM / MIN slot (AVG / RANGE)
  int32_t b[kMaxOrderKeys];      // COUNT slot (AVG), MAX slot (RANGE); HLL: a = register block, b = log2m
  int32_t desc[kMaxOrderKeys];
};

// One compressed chunk of a raw fixed-byte forward index (BaseChunkForwardIndexReader.java:204-232):
// `csize` bytes at blob + src decode to `usize` BE bytes, stored byte-swapped at out + dst.
struct RawChunk {
  uint64_t src;
  uint64_t dst;
  uint32_t csize;
  uint32_t usize;
};

// One Roaring container of one selected dictionary id, OR-ed into a segment's dense doc words.
struct RoaringTask {
  const uint8_t *payload;
  uint64_t *out_words;
  int32_t key;   // high 16 bits of the doc ids: words [1024*key, 1024*key + 1024)
  int32_t kind;  // 0 array (card x u16), 1 bitmap (1024 x u64 LE), 2 run (u16 nruns, (start, len-1) pairs)
  int32_t card;  // array cardinality / number of runs
  int32_t pad;
};

// The containers of one (inverted leaf, 65536-doc key) pair: roaring_or_kernel decodes them into an
// 8 KiB LDS bitmap and writes the key's 1024 doc words once.
struct RoaringGroup {
  uint64_t *out_words;   // the leaf's dense doc words
  int32_t task_begin;    // containers [task_begin, task_end) of the RoaringTask array
  int32_t task_end;
  int32_t key;
  int32_t tile_words;    // u64 words per 2048-doc tile of the output (the entry's leaves interleaved per tile)
};

}  // namespace phip
