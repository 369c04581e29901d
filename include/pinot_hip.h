/*
 * pinot_hip.h -- C ABI of libpinot_hip.so, the MI355X-native segment query hot path.
 *
 * Drop-in boundary. The reference's Java server keeps its operator surface and
 * calls these entry points through Java 21 FFM (INTEGRATION.md shows the bindings):
 *
 *   phip_segment_load    <- ImmutableSegmentLoader.load
 *                           (pinot-segment-local/.../indexsegment/immutable/ImmutableSegmentLoader.java:155-190,
 *                           222-280): per column the forward index, dictionary and inverted index
 *                           buffers that PhysicalColumnIndexContainer (…/segment/index/column/
 *                           PhysicalColumnIndexContainer.java:44-68) maps, handed over as raw bytes
 *                           (PinotDataBuffer.toDirectByteBuffer, pinot-segment-spi/.../memory/
 *                           PinotDataBuffer.java:671-696) and pinned in HBM.
 *   phip_segment_unload  <- IndexSegment.destroy
 *   phip_query           <- InstancePlanMakerImplV2.makeInstancePlan
 *                           (pinot-core/.../plan/maker/InstancePlanMakerImplV2.java:172-199) when the
 *                           query option selects the GPU: one call replaces, for all segments of the
 *                           query, FilterPlanNode/BaseFilterOperator.getTrues
 *                           (pinot-core/.../operator/filter/BaseFilterOperator.java:85-93),
 *                           AggregationOperator.getNextBlock (…/operator/query/AggregationOperator.java:63-80),
 *                           GroupByOperator.getNextBlock (…/operator/query/GroupByOperator.java:100-140)
 *                           and the CombineOperator merge (…/operator/combine/BaseSingleBlockCombineOperator.java:58-162).
 *                           Results are the intermediate values AggregationResultsBlock /
 *                           GroupByResultsBlock carry (…/operator/blocks/results/).
 *   phip_filter_bitmap   <- BaseFilterOperator.getTrues / getBitmaps for one segment (doc-id set as
 *                           64-doc bitmap words; the bit for doc d is bit d%64 of word d/64).
 *
 * Conventions: every function returns int32_t status (PHIP_OK = 0); on error the calling
 * thread's message is available from phip_last_error(). Host buffers passed in are borrowed for
 * the duration of the call only; the library owns all device memory. All entry points are
 * thread-safe (per-device mutex). No HIP/torch types cross the boundary.
 */
#ifndef PINOT_HIP_H_
#define PINOT_HIP_H_

#include <stdint.h>

#ifdef __cplusplus
#define PHIP_EXTERN extern "C"
#else
#define PHIP_EXTERN extern
#endif
#define PHIP_API PHIP_EXTERN __attribute__((visibility("default")))

/* ---- status ------------------------------------------------------------------------------ */
#define PHIP_OK 0
#define PHIP_ERR_INVALID 1     /* malformed descriptor / plan */
#define PHIP_ERR_HIP 2         /* a HIP runtime call failed */
#define PHIP_ERR_UNSUPPORTED 3 /* shape outside the GPU subset: caller falls back to the Java path */
#define PHIP_ERR_NOT_FOUND 4   /* unknown segment handle or column */
#define PHIP_ERR_NO_DEVICE 5   /* no usable GPU */
#define PHIP_ERR_TIMEOUT 6     /* the plan's deadline passed (QueryTimeoutException: BaseSingleBlockCombineOperator
                                  .java:137-144 checks QueryContext.getEndTimeMs) */
#define PHIP_ERR_CANCELLED 7   /* phip_plan_cancel stopped the execution (QueryCancelledException) */

/* ---- stored data types (FieldSpec.DataType, single-value) ---------------------------------- */
#define PHIP_TYPE_INT 0
#define PHIP_TYPE_LONG 1
#define PHIP_TYPE_FLOAT 2
#define PHIP_TYPE_DOUBLE 3
#define PHIP_TYPE_STRING 4

/* ---- forward index encodings -------------------------------------------------------------- */
#define PHIP_FWD_FIXED_BIT 0 /* FixedBitSVForwardIndexWriter: ceil(N*b/8) BE bytes, MSB first */
#define PHIP_FWD_SORTED 1    /* SortedIndexReaderImpl: card x (start,end) BE int32, inclusive */
#define PHIP_FWD_HLL_REGISTERS 3 /* per doc 2^bits_per_value u8 HyperLogLog registers (a star-tree DISTINCTCOUNTHLL
                                  * function-column pair): DISTINCTCOUNTHLL max-merges them; no other use */
#define PHIP_FWD_RAW_CHUNK 2 /* BaseChunkForwardIndexWriter v2/v3 fixed-width chunks (and v4/v5 power-of-two chunks,
                              * FixedBytePower2ChunkSVForwardIndexReader): PASS_THROUGH, or SNAPPY / LZ4 /
                              * LZ4_LENGTH_PREFIXED / ZSTANDARD / GZIP decoded on the GPU at load (a malformed chunk
                              * fails the load); v1 (4-int header, SNAPPY chunks: BaseChunkForwardIndexReader.java:86-95)
                              * as well. A STRING column: VarByteChunkForwardIndexWriter v1..v3 chunks (per chunk
                              * numDocsPerChunk BE int start offsets, then the UTF-8 bytes), any codec */

typedef struct phip_column_desc {
  const char *name;
  int32_t data_type;      /* PHIP_TYPE_* */
  int32_t fwd_kind;       /* PHIP_FWD_* */
  int32_t cardinality;    /* dictionary length (0 for raw columns) */
  int32_t bits_per_value; /* fixed-bit width: getNumBitsPerValue(card-1) */
  int32_t string_width;   /* STRING dictionary: bytes per '\0'-padded entry */
  int32_t reserved;
  const uint8_t *forward;
  uint64_t forward_bytes;
  const uint8_t *dictionary; /* BE fixed-width sorted values (NULL for raw columns) */
  uint64_t dictionary_bytes;
  const uint8_t *inverted; /* (card+1) BE u32 offsets + portable Roaring bitmaps, or NULL */
  uint64_t inverted_bytes;
  /* Null value vector (NullValueVectorReaderImpl: `<column>.bitmap.nullvalue`, one portable Roaring bitmap of the
   * docs whose value is null; NullValueVectorCreator writes it only when some doc is null), or NULL. Kept in HBM as
   * dense doc words for PHIP_LEAF_NULL leaves. */
  const uint8_t *null_vector;
  uint64_t null_vector_bytes;
} phip_column_desc;

typedef struct phip_segment_desc {
  const char *name;
  int32_t device;      /* device ordinal, -1 = current default device */
  int32_t num_docs;
  int32_t num_columns;
  int32_t reserved;
  const phip_column_desc *columns;
} phip_segment_desc;

/* ---- filter program ----------------------------------------------------------------------
 * Per segment, a preorder tree: an AND/OR node is followed by its num_children subtrees; NOT by
 * one subtree. Leaves carry the per-segment outcome of the reference's PredicateEvaluator
 * (dictionary ids are per segment): RangePredicateEvaluatorFactory (dict-id range [lo,hi)),
 * In/NotIn/Eq/NotEq evaluators (dict-id set), SortedIndexBasedFilterOperator (doc ranges) or
 * InvertedIndexFilterOperator (dict ids whose bitmaps are OR-ed, complemented if exclusive). */
#define PHIP_NODE_LEAF 0
#define PHIP_NODE_AND 1
#define PHIP_NODE_OR 2
#define PHIP_NODE_NOT 3

#define PHIP_LEAF_MATCH_ALL 0  /* predicate alwaysTrue for this segment */
#define PHIP_LEAF_MATCH_NONE 1 /* predicate alwaysFalse for this segment */
#define PHIP_LEAF_DICT_RANGE 2 /* scan forward index: lo <= dictId < hi */
#define PHIP_LEAF_DICT_SET 3   /* scan forward index: dictId in ids (xor exclusive) */
#define PHIP_LEAF_DOC_RANGES 4 /* ids = count x (startDoc, endDoc) inclusive, sorted, disjoint */
#define PHIP_LEAF_INVERTED 5   /* OR of inverted-index bitmaps of ids (xor exclusive) */
/* Raw (no-dictionary) columns, value-based (RawValueBasedPredicateEvaluator, ScanBasedFilterOperator.java:58-66).
 * ids points at `count` int32 words holding a phip_raw_range (RAW_RANGE) or count/2 int64 values -- doubles for
 * FLOAT/DOUBLE columns -- (RAW_SET, xor exclusive). */
#define PHIP_LEAF_RAW_RANGE 6
#define PHIP_LEAF_RAW_SET 7
/* Raw STRING columns (var-byte chunks): the values compared in String.compareTo order. ids points at `count` int32
 * words: RAW_STRING_RANGE = [lo_len][hi_len][lo_inclusive][hi_inclusive][lo UTF-8 bytes][hi UTF-8 bytes], a length
 * of -1 = unbounded (StringRawValueBasedRangePredicateEvaluator, RangePredicateEvaluatorFactory.java); RAW_STRING_SET
 * = [n][n + 1 byte offsets][the n values' UTF-8 bytes] (raw EQ / NOT_EQ / IN / NOT_IN, xor exclusive). */
#define PHIP_LEAF_RAW_STRING_RANGE 8
#define PHIP_LEAF_RAW_STRING_SET 9
/* The column's null value vector (IS NULL: BitmapBasedFilterOperator over NullValueVectorReader.getNullBitmap,
 * FilterPlanNode.java:294-307; exclusive = IS NOT NULL). A column without a null vector matches no doc (all docs when
 * exclusive). With enableNullHandling the host composes these with the other leaves (BaseColumnFilterOperator's
 * trues AND NOT nulls, the And / Or / Not operators' getFalses), so the library needs nothing else for nulls. */
#define PHIP_LEAF_NULL 10

typedef struct phip_raw_range {
  int64_t lo_int, hi_int; /* INT/LONG columns: lo_int <= v <= hi_int */
  double lo_real, hi_real; /* FLOAT/DOUBLE columns, with the inclusive flags below */
  int32_t lo_inclusive, hi_inclusive;
} phip_raw_range;

typedef struct phip_filter_node {
  int32_t op;           /* PHIP_NODE_* */
  int32_t num_children; /* AND/OR */
  int32_t leaf_kind;    /* PHIP_LEAF_* */
  int32_t column;       /* index into phip_query_desc.columns */
  int32_t lo, hi;       /* DICT_RANGE */
  int32_t exclusive;    /* DICT_SET / INVERTED */
  int32_t count;        /* number of ids (DICT_SET/INVERTED) or of ranges (DOC_RANGES) */
  const int32_t *ids;
} phip_filter_node;

/* ---- aggregations ------------------------------------------------------------------------- */
#define PHIP_AGG_COUNT 0 /* CountAggregationFunction */
#define PHIP_AGG_SUM 1   /* SumAggregationFunction (int64 exact for INT/LONG inputs, f64 otherwise) */
#define PHIP_AGG_MIN 2   /* MinAggregationFunction (default +inf) */
#define PHIP_AGG_MAX 3   /* MaxAggregationFunction (default -inf) */
#define PHIP_AGG_HLL 4   /* DistinctCountHLLAggregationFunction: HyperLogLog(log2m) registers */

#define PHIP_EXPR_COLUMN 0 /* a */
#define PHIP_EXPR_ADD 1    /* a + b   (AdditionTransformFunction) */
#define PHIP_EXPR_SUB 2    /* a - b   (SubtractionTransformFunction.java:99-124) */
#define PHIP_EXPR_MUL 3    /* a * b   (MultiplicationTransformFunction.java:90-106) */

typedef struct phip_aggregation {
  int32_t function; /* PHIP_AGG_* */
  int32_t expr;     /* PHIP_EXPR_* (ignored for COUNT) */
  int32_t column_a; /* index into phip_query_desc.columns */
  int32_t column_b;
  int32_t log2m; /* HLL */
  int32_t program; /* filter program whose docs this aggregation reads (0 unless num_filter_programs > 1) */
} phip_aggregation;

typedef struct phip_query_desc {
  int32_t num_columns;
  int32_t num_segments;
  const char *const *columns; /* column names; nodes/aggregations refer to them by index */
  const uint64_t *segments;   /* handles from phip_segment_load */
  const int32_t *filter_offsets;          /* [num_filter_programs * num_segments + 1] into filter_nodes: program p
                                           * of segment s = [p * num_segments + s, + 1); empty = match all */
  const phip_filter_node *filter_nodes;
  int32_t num_aggregations;
  int32_t num_group_by;
  const phip_aggregation *aggregations;
  const int32_t *group_by_columns; /* indices into columns */
  int64_t num_groups_limit;        /* InstancePlanMakerImplV2 numGroupsLimit (default 100,000) */
  /* Server-level trim of a group-by with ORDER BY on one aggregation (IndexedTable.finish ->
   * TableResizer.getTopRecords, GroupByUtils.java:96-140): when trim_size > 0 and more groups than trim_size
   * exist, only the top trim_size groups by aggregations[order_by_aggregation] (Double.compare order,
   * descending when order_by_desc) are returned; ties at the boundary keep the lowest group key.
   * order_by_aggregation = -1 disables it. */
  int32_t order_by_aggregation;
  int32_t order_by_desc;
  int64_t trim_size;               /* max(5 * limit, minServerGroupTrimSize) (GroupByUtils.java:55-58) */
  /* ORDER BY on group-by columns instead (takes precedence when > 0): entry j = k + 1 (ASC) or -(k + 1)
   * (DESC) for group-by column k; the query-global dictionaries are value-sorted, so id order is value order. */
  int32_t num_order_by_keys;
  /* enableNullHandling group keys (NoDictionarySingleColumnGroupKeyGenerator.getKeyForNullValue /
   * NoDictionaryMultiColumnGroupKeyGenerator, pinot-core/.../groupby/NoDictionary*GroupKeyGenerator.java): bit k =
   * group-by column k's null docs (its null value vector) form one more key value, the null key -- group key id =
   * the column's phip_dictionary_view.cardinality in phip_result.group_keys; it is counted toward numGroupsLimit in
   * first-seen order like any key, sorts after every value in an ascending key trim and first in a descending one
   * (the reference's default NULLS LAST / NULLS FIRST). 0 = the stored default values are the keys. */
  int32_t null_group_by;
  const int32_t *order_by_keys;
  /* Any other ORDER BY (TableResizer, pinot-core/.../data/table/TableResizer.java:90-125,410-450): a list of
   * terms, each a group-by column or an aggregation's final result, mixed freely (takes precedence over both
   * fields above when > 0). The device sorts the groups by the whole list (stable; ties keep the lowest group key)
   * and keeps trim_size of them. */
  int32_t num_order_terms;
  /* Filtered aggregations in one pass (FilteredAggregationOperator.java:67-113, one program per
   * AggregationFunctionUtils.buildFilteredAggregationInfos info): when > 1, filter_offsets holds that many
   * programs per segment, one filter launch evaluates all of them into one tile mask each, and one aggregation
   * launch aggregates every function over its own program's docs (phip_aggregation.program). Statistics sum over
   * the programs (numDocsScanned, entries scanned; a segment matched when any program matched). Aggregation only
   * (no group-by), at most 8 programs. 0 or 1 = one program. */
  int32_t num_filter_programs;
  const struct phip_order_term *order_terms;
  /* Selection (row-returning) queries, the leaf of a multi-stage join (SelectionOnlyOperator,
   * pinot-core/.../operator/query/SelectionOnlyOperator.java:40-170, and SelectionOnlyCombineOperator): when
   * num_select > 0 (no aggregations, no group-by, one filter program) each segment keeps its first select_limit
   * matched docs in doc order, the segments' rows are concatenated in query order up to select_limit rows, and
   * every row holds the select expressions (phip_result.select_*). Statistics: numDocsScanned = the rows each
   * segment kept, numEntriesScannedPostFilter = that x the distinct columns the expressions read. */
  int32_t num_select;
  /* Programs whose filter scans count in num_entries_scanned_in_filter: bit p = program p; 0 = every program.
   * A CASE aggregation's branch programs re-evaluate the query's filter AND a WHEN condition, while the
   * reference scans each original filter once (CaseTransformFunction evaluates the WHENs in the transform,
   * pinot-core/.../transform/function/CaseTransformFunction.java): only those programs count. */
  uint32_t stats_programs;
  const struct phip_select_expr *select;
  int64_t select_limit;
} phip_query_desc;

typedef struct phip_select_expr {
  int32_t expr;     /* PHIP_EXPR_*: a column, or a op b (evaluated in double, as the transform functions do) */
  int32_t column_a; /* index into phip_query_desc.columns */
  int32_t column_b;
  int32_t reserved;
} phip_select_expr;

#define PHIP_ORDER_GROUP_KEY 0 /* group-by column `a` (GroupByExpressionExtractor) */
#define PHIP_ORDER_VALUE 1     /* aggregations[a] as double: SUM / MIN / MAX / COUNT (AggregationFunctionExtractor) */
#define PHIP_ORDER_AVG 2       /* aggregations[a] (SUM) / aggregations[b] (COUNT); -inf when the count is 0 */
#define PHIP_ORDER_RANGE 3     /* aggregations[b] (MAX) - aggregations[a] (MIN): MINMAXRANGE */
#define PHIP_ORDER_HLL 4       /* aggregations[a] (DISTINCTCOUNTHLL): its registers' cardinality estimate */

typedef struct phip_order_term {
  int32_t kind; /* PHIP_ORDER_* */
  int32_t a;
  int32_t b;
  int32_t desc; /* 1 = DESC */
} phip_order_term;

/* ---- results ------------------------------------------------------------------------------
 * Library-owned, valid until phip_result_free. For an aggregation-only query num_groups = 1.
 * values[g*num_aggregations + a] holds SUM/MIN/MAX/COUNT as double (HLL: estimate);
 * long_values[...] the exact int64 SUM (integral inputs) or COUNT.
 * hll_registers: [num_groups][num_hll][1 << log2m] u8 in aggregation order of the HLL aggs.
 * group_keys[g*num_group_by + k]: id in the query-global dictionary of group-by column k;
 * phip_result_dictionary returns that dictionary's values. */
typedef struct phip_result {
  int64_t num_docs_scanned;
  int64_t num_entries_scanned_in_filter;
  int64_t num_entries_scanned_post_filter;
  int64_t num_total_docs;
  int32_t num_segments_processed;
  int32_t num_segments_matched;
  int32_t num_groups_limit_reached;
  int32_t num_aggregations;
  int64_t num_groups;
  int32_t num_group_by;
  int32_t num_hll;
  const double *values;
  const int64_t *long_values;
  const uint8_t *hll_registers;
  const int32_t *group_keys;
  double scan_kernel_ms; /* device time of the fused filter/aggregate kernel(s) */
  double device_ms;      /* device time of the query's filter / aggregation kernels (whole sequence incl. memsets and
                          * finalize when PHIP_TOTAL_EVENTS=1: two more timing markers, ~4 us each on the queue) */
  int32_t num_groups_trimmed; /* 1 when the group set was trimmed to phip_query_desc.trim_size */
  int32_t fused;              /* 1 when the filter kernel aggregated its own tiles (one launch: filter_kernel_ms and
                                 filter_bytes then cover both, agg_* are 0) */
  /* long_exact[a] = 1 when long_values[g*num_aggregations + a] holds the exact integer result (COUNT, and SUM
   * over INT/LONG inputs whose bound sum |value| stays below 2^62); 0 when the SUM accumulated in double like
   * SumAggregationFunction (a possible int64 overflow) -- values[] is then the only result. */
  const int32_t *long_exact;
  /* Per-kernel device time and algorithmic bytes (the roofline numerators):
   * filter_bytes = per work tile, the fixed-bit words of every scanned column (256*b bytes), the dense words of
   * every inverted leaf (256) and the raw values of raw leaves -- what the filter launch must stream;
   * agg_bytes = per segment, matched docs x (b/8 per projected dictionary column, value width per raw one) plus
   * min(card, matched) dictionary entries per gathered column. Intermediates (tile masks, tables) excluded. */
  double filter_kernel_ms;
  double agg_kernel_ms;
  int64_t filter_bytes;
  int64_t agg_bytes;
  /* Selection queries (phip_query_desc.num_select > 0): num_rows rows of num_select columns, column-major 8-byte
   * slots select_values[k * num_rows + r]; select_types[k] says how to read column k: PHIP_TYPE_INT / LONG = int64,
   * PHIP_TYPE_FLOAT / DOUBLE = double bits (FLOAT values are exact floats; expressions are DOUBLE), PHIP_TYPE_STRING
   * = id in a query-global dictionary (phip_result_select_dictionary). */
  int64_t num_rows;
  int32_t num_select;
  int32_t reserved_select;
  const int32_t *select_types;
  const uint64_t *select_values;
  /* Per segment of the query (num_segments_processed entries): the docs that passed its filter, summed over the
   * filter programs -- the docs its GroupByOperator keyed, so min(this, key space, numGroupsLimit) bounds the
   * group records the segment hands the combine (GroupByCombineOperator.java:128-157; the plan maker's
   * minSegmentGroupTrimSize / groupTrimThreshold checks). For a phip_plan_finish result: this GPU's. */
  const int64_t *segment_docs_matched;
  /* The part of filter_bytes the filter launch STREAMS (the staged tiles' words, LDS-DMA); for a fused launch
   * filter_bytes also holds its gathers (agg_bytes folded in). The traffic calibration separates the two. */
  int64_t stream_bytes;
  /* Per filter program (phip_query_desc.num_filter_programs entries, 1 for one program): the docs that passed it over
   * all segments -- the reference's numDocsScanned when programs are the plan maker's own device (the null-handling
   * group-by's IS NOT NULL programs), not FilteredGroupByOperator infos. For a phip_plan_finish result: this GPU's. */
  const int64_t *program_docs_matched;
} phip_result;

typedef struct phip_dictionary_view {
  int32_t data_type;
  int32_t cardinality;
  int32_t string_width;
  int32_t reserved;
  const void *values; /* LE int32/int64/float/double array, or card x string_width bytes */
} phip_dictionary_view;

/* ---- entry points -------------------------------------------------------------------------- */
PHIP_API int32_t phip_init(const int32_t *devices, int32_t num_devices);
PHIP_API int32_t phip_shutdown(void);
PHIP_API int32_t phip_device_count(int32_t *out_count);
PHIP_API const char *phip_last_error(void);
PHIP_API const char *phip_version(void);
/* HIP_VERSION the library was built against and hipRuntimeGetVersion of the runtime it bound to (a process that
 * also runs PyTorch-ROCm shares torch's bundled runtime; the loader refuses a major-version mismatch). No
 * reference counterpart: a build/runtime sanity check of the FFM loader. */
PHIP_API int32_t phip_runtime_versions(int32_t *out_built, int32_t *out_runtime);

PHIP_API int32_t phip_segment_load(const phip_segment_desc *desc, uint64_t *out_handle);
PHIP_API int32_t phip_segment_unload(uint64_t handle);
PHIP_API int32_t phip_segment_device_bytes(uint64_t handle, uint64_t *out_bytes);

PHIP_API int32_t phip_query(const phip_query_desc *query, phip_result **out_result);

/* Prepared queries: InstancePlanMakerImplV2.makeInstancePlan returns a Plan that
 * GlobalPlanImplV0.execute runs (pinot-core/.../plan/GlobalPlanImplV0.java:48-57). phip_plan_create does
 * every host-side step once (predicate programs per segment, descriptors, launch shapes, device buffers);
 * phip_plan_execute replays the launch sequence (eagerly; PHIP_GRAPH=1 opts into a captured hipGraph) and
 * returns a result exactly as phip_query would. A plan keeps its segments' HBM alive: unloading a
 * segment a plan uses defers the release to phip_plan_destroy. Executions of one plan serialise. */
PHIP_API int32_t phip_plan_create(const phip_query_desc *query, uint64_t *out_plan);
PHIP_API int32_t phip_plan_execute(uint64_t plan, phip_result **out_result);
PHIP_API int32_t phip_plan_destroy(uint64_t plan);
/* Query deadline and cancellation (QueryContext.getEndTimeMs / the server's cancel of a running query,
 * BaseSingleBlockCombineOperator.java:137-144, QueryScheduler cancel): an execution checks them between its launch
 * phases -- before enqueuing, after the main kernels, before a numGroupsLimit pass and before the server trim -- and
 * returns PHIP_ERR_TIMEOUT / PHIP_ERR_CANCELLED there (a launch in flight completes: kernels are not interrupted,
 * as the reference's operators only check between blocks). deadline_ms: wall-clock milliseconds since the Unix
 * epoch (System.currentTimeMillis), 0 = none. A cancel is sticky: the plan belongs to one query. */
PHIP_API int32_t phip_plan_set_deadline(uint64_t plan, int64_t deadline_ms);
PHIP_API int32_t phip_plan_cancel(uint64_t plan);
PHIP_API int32_t phip_result_dictionary(const phip_result *result, int32_t group_by_index,
                                        phip_dictionary_view *out_view);
PHIP_API void phip_result_free(phip_result *result);

/* Values of select column k of a selection result that holds STRING dictionary ids. */
PHIP_API int32_t phip_result_select_dictionary(const phip_result *result, int32_t select_index,
                                               phip_dictionary_view *out_view);

/* Filter only, one segment: words_out receives ceil(num_docs/64) bitmap words. */
PHIP_API int32_t phip_filter_bitmap(const phip_query_desc *query, uint64_t *words_out, int64_t num_words);

/* ---- multi-GPU servers: one process per GPU, partial group tables merged on the device ----------------
 * The reference's combine merges per-segment group-by results by VALUE on one JVM
 * (GroupByCombineOperator.java:138-147 upserting into an IndexedTable). A server spread over several GPUs
 * instead keys every group-by column by a NODE-GLOBAL dictionary: the sorted union of
 * the column's dictionary values over every segment on every GPU, registered once per column after load.
 * Plans created afterwards key that column by ids in it on every GPU, so each GPU's dense partial table has
 * the same shape and key order and the GPUs merge them element-wise with RCCL all-reduce on the device
 * buffers -- no host round trip of group records.
 *
 * phip_global_dictionary: values as phip_dictionary_view lays them out (LE typed array, or
 * cardinality x string_width '\0'-padded bytes), ascending, distinct. Registering a column again replaces
 * it for plans created later; cardinality = -1 removes the registration. Columns are keyed by the name the
 * query descriptors use (one table per server process). A segment value missing from it fails plan creation
 * with PHIP_ERR_INVALID. */
PHIP_API int32_t phip_global_dictionary(int32_t device, const char *column, int32_t data_type, int32_t cardinality,
                                        int32_t string_width, const void *values);

/* Row kinds of a partial table; the reduce operator of each row follows from its kind. */
#define PHIP_ROW_COUNT 0   /* int64 doc count per group (row 0; unused rows of COUNT aggregations hold 0): SUM */
#define PHIP_ROW_SUM_I64 1 /* exact int64 sum: SUM (int64) */
#define PHIP_ROW_SUM_F64 2 /* double sum (bits): SUM (float64) */
#define PHIP_ROW_MIN 3     /* order-preserving u64 image of a double (f64_ordered): MIN as unsigned */
#define PHIP_ROW_MAX 4     /* same image: MAX as unsigned */
#define PHIP_ROW_HLL 5     /* row unused (0); the registers are in phip_partial.hll: MAX (int32) */
#define PHIP_PARTIAL_MAX_ROWS 9

typedef struct phip_partial {
  int64_t num_groups;   /* dense key space G = product of the group-by columns' (global) cardinalities */
  int32_t num_rows;     /* 1 + num_aggregations */
  int32_t num_hll;
  int32_t log2m;
  int32_t device;
  uint64_t *table;      /* DEVICE memory owned by the plan: [num_rows][G] u64, row 0 = doc count per group */
  uint32_t *hll;        /* DEVICE memory: [num_hll][G][1 << log2m] u32 registers, or NULL */
  /* row_kinds[r] for r < num_rows. A caller merging GPUs whose plans disagree on SUM_I64 vs SUM_F64 for a
   * row (the int64-overflow bound is per GPU) converts its int64 row to doubles in place and sets the kind to
   * PHIP_ROW_SUM_F64 before phip_plan_finish. */
  int32_t row_kinds[PHIP_PARTIAL_MAX_ROWS];
  int32_t global_keys;  /* 1 when every group-by column is keyed by a registered global dictionary (else the
                         * key order is this GPU's own and the table must not be merged element-wise) */
  /* This GPU's execution statistics (phip_result order: docs scanned, entries scanned in filter, entries
   * scanned post filter, total docs, segments processed, segments matched); summed over GPUs by the caller. */
  int64_t stats[6];
  /* Aggregation-only plans (num_groups = 1): the same six statistics as int64 in DEVICE memory right after the
   * table's last row (stats_dev = table + num_rows), so one int64 SUM all-reduce covers the table's integer rows and
   * them; phip_plan_finish then reads the merged statistics from there. NULL for group-by partials (stats[] holds
   * them). */
  int64_t *stats_dev;
  /* 1: hll holds u8 registers ([num_hll][G][1 << log2m] bytes: the all-reduce MAX runs on them directly); 0: u32. */
  int32_t hll_u8;
  int32_t reserved_partial;
} phip_partial;

/* Runs a dense group-by plan up to its partial table and returns it (the kernels have completed). An
 * aggregation-only plan (AggregationResultsBlockMerger.java:34-49's inputs) hands out a one-group table: row 0 =
 * matched docs, row 1 + a = aggregation a in its row kind's encoding (MIN / MAX as the order-preserving u64 image),
 * the statistics in stats_dev and u8 HLL registers -- all in device memory, so GPUs merge them with RCCL
 * all-reduces and no host copy. Returns
 * PHIP_ERR_UNSUPPORTED, with nothing to merge, for hash-table key spaces and when the GPU's distinct groups
 * reach numGroupsLimit (the per-segment first-seen limit needs the record path: phip_plan_execute). Until
 * phip_plan_finish the table belongs to the caller: it may all-reduce it in place (on any stream, synchronised
 * before phip_plan_finish). No other execution of the same plan may start in between (the library refuses one
 * with PHIP_ERR_INVALID until phip_plan_finish or phip_plan_abandon_partial). */
PHIP_API int32_t phip_plan_execute_partial(uint64_t plan, phip_partial *out_partial);
/* Compacts the (merged) partial table into a result exactly as phip_plan_execute would -- present groups,
 * the server-level trim (trim_size), statistics taken from merged->stats. */
PHIP_API int32_t phip_plan_finish(uint64_t plan, const phip_partial *merged, phip_result **out_result);
/* Gives a pending partial table back without finishing it (the GPUs agreed to merge records instead). While a
 * partial is pending, phip_plan_execute / phip_plan_execute_partial on the plan return PHIP_ERR_INVALID. */
PHIP_API int32_t phip_plan_abandon_partial(uint64_t plan);

/* ---- multi-GPU servers in ONE process: node plans ------------------------------------------------------
 * A Pinot server is one JVM that owns every GPU of its node: BaseCombineOperator fans a query's segments out over
 * worker threads (pinot-core/.../operator/combine/BaseCombineOperator.java:98-143) and merges their blocks in that
 * process (BaseSingleBlockCombineOperator.java:129-162, GroupByCombineOperator.java:138-147). phip_plan_create /
 * phip_query over segments loaded on SEVERAL devices (phip_segment_desc.device) returns a node plan -- no other call
 * changes, so the Java binding needs nothing beyond this header:
 *   - each device's segments form one single-device sub-plan; the group-by columns of every sub-plan are keyed by the
 *     node plan's own node-global dictionaries (the sorted union of the column's values over all its segments, built
 *     at plan creation -- no phip_global_dictionary registration needed), so the devices' dense partial tables have
 *     the same shape and key order;
 *   - phip_plan_execute runs the sub-plans concurrently, one host thread and one execution lane per device, up to
 *     their dense partial tables (phip_plan_execute_partial's), then merges them ON THE DEVICES: one RCCL reduce to
 *     the root device (the first device in query order) over the node's communicator (ncclCommInitAll over the
 *     node plan's devices, created once per device set, librccl loaded on first use; xGMI peer-to-peer) -- int64 SUM
 *     for counts and exact sums, f64 SUM, unsigned MIN / MAX of the order-preserving images, MAX of the HLL registers
 *     -- and finishes the merged table on the root (compaction, server trim, copy-out) exactly as phip_plan_finish;
 *   - where the devices cannot share a communicator (two parts on one device, no loadable librccl) the non-root
 *     tables are copied to the root device (hipMemcpyPeerAsync) and folded in by the library's merge kernel, the same
 *     operators;
 *   - hash-table key spaces (node-global keys, each part's table sized for every doc of the node): the non-root
 *     parts' keys, rows and registers are copied to the root device and inserted into the root's table by key
 *     (PHIP_EXCHANGE_HASH), then finished as above;
 *   - aggregation-only queries (one group) and group-bys without a mergeable partial table (a device reaching
 *     numGroupsLimit -- the per-segment first-seen limit --, a full hash table, raw group-by keys, tuple keys, parts
 *     whose null keys differ) run each sub-plan to its records and merge them on the host by key VALUE, as the
 *     reference's combine does (untrimmed: the broker's ORDER BY / LIMIT applies to exact groups).
 * Statistics are summed over the devices; segment_docs_matched covers every segment in query order; kernel times
 * are the slowest device's. Selection queries over several devices return PHIP_ERR_UNSUPPORTED. The deadline and
 * cancel calls apply to every sub-plan. phip_plan_execute_partial / phip_plan_finish / phip_plan_abandon_partial on
 * a node plan return PHIP_ERR_INVALID (it merges internally).
 * PHIP_NODE_SPLIT=k (environment, read at plan creation) splits a query whose segments share one device into k parts
 * on that device -- a rehearsal of the node path on a one-GPU box (the peer-merge exchange; k = 1: one part and a
 * one-rank RCCL communicator). PHIP_NODE_EXCHANGE=peer forces the merge kernel, =rccl refuses the fallback. */
#define PHIP_EXCHANGE_NONE 0    /* a single-device plan */
#define PHIP_EXCHANGE_RCCL 1    /* the last execution reduced the partial tables with RCCL */
#define PHIP_EXCHANGE_PEER 2    /* ... copied them to the root device and merged them with the merge kernel */
#define PHIP_EXCHANGE_RECORDS 3 /* ... merged the sub-plans' records on the host */
#define PHIP_EXCHANGE_HASH 4    /* ... inserted the other sub-plans' hash-table groups into the root's table on the root device */
/* Devices (sub-plans) of a plan and the exchange its last execution used (PHIP_EXCHANGE_*; NONE before the first). */
PHIP_API int32_t phip_plan_exchange(uint64_t plan, int32_t *out_parts, int32_t *out_kind);

#endif /* PINOT_HIP_H_ */
