/*
 * cpu_scan.c -- the CPU BASELINE of bench.py: a multi-threaded C restatement of Pinot's CPU server path for
 * the headline queries (conjunctive dict-id filters + SUM of a column expression, SSB Q1.x). TEST / BENCH
 * INFRASTRUCTURE ONLY (oracle/ package rules): it is timed beside the GPU, never shipped or called by the
 * product. Labelled "restatement, not Pinot": the JVM reference cannot run here.
 *
 * Per segment it follows the reference's operators:
 *   - sorted-column leaves -> one inclusive doc range (SortedIndexBasedFilterOperator.java:52-132 with
 *     SortedIndexReaderImpl.getDocIds :114-116); AndDocIdSet restricts the scan children to it (:134-166);
 *   - the first scan leaf is evaluated over the candidate docs in 256-doc batches, dict ids decoded in bulk
 *     (SVScanDocIdIterator.next + FixedBitSVForwardIndexReaderV2.readDictIds, :63-99; FixedBitIntReader
 *     MSB-first big-endian), the remaining scan leaves only on the survivors (applyAnd, :114-142);
 *   - DocIdSetOperator blocks of <= 10,000 docs (DocIdSetPlanNode.java:29); per block the projected dict ids
 *     are read at the block's docs, looked up in the big-endian dictionaries and combined in double
 *     (DataFetcher.readDoubleValues, MultiplicationTransformFunction 1.0*a*b), SumAggregationFunction adds the
 *     block's double sum to the holder (:76-101);
 *   - the combine fans segments out over `threads` workers (QueryMultiThreadingUtils / BaseCombineOperator)
 *     and merges the per-segment sums in segment order.
 */
#include <stdint.h>
#include <string.h>

#include <omp.h>

#define CB_MAX_LEAVES 8
#define CB_BATCH 256
#define CB_BLOCK 10000

typedef struct {
  const uint8_t *fwd; /* fixed-bit BE ids, or card x (start,end) BE int32 for a sorted column */
  int32_t bits;
  int32_t sorted;
  int32_t lo, hi; /* matching dict ids [lo, hi) */
} cb_leaf;

typedef struct {
  int32_t num_docs;
  int32_t nleaves;
  cb_leaf leaves[CB_MAX_LEAVES];
  const uint8_t *fwd_a, *dict_a; /* projected columns: fixed-bit ids + BE int32 dictionary */
  const uint8_t *fwd_b, *dict_b;
  int32_t bits_a, bits_b;
  int32_t expr; /* 0 a, 1 a+b, 2 a-b, 3 a*b */
  int32_t pad;
} cb_segment;

static inline uint64_t be64_at(const uint8_t *p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return __builtin_bswap64(v);
}

/* value i of a b-bit MSB-first stream (the buffer is read 8 bytes at a time: callers pad by 8) */
static inline uint32_t read_id(const uint8_t *buf, int64_t i, int bits) {
  const uint64_t bit = (uint64_t)i * (uint64_t)bits;
  const uint64_t w = be64_at(buf + (bit >> 3));
  return (uint32_t)((w << (bit & 7)) >> (64 - bits));
}

static inline int32_t be32s(const uint8_t *p) {
  return (int32_t)(((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]);
}

/* one DocIdSetOperator block (<= 10,000 docs) through the projection and SUM's per-block double sum */
static double block_sum(const cb_segment *s, const int32_t *block, int *nblock, int64_t *m) {
  double inner = 0.0;
  for (int i = 0; i < *nblock; i++) {
    const double a = (double)be32s(s->dict_a + 4 * (int64_t)read_id(s->fwd_a, block[i], s->bits_a));
    double v = a;
    if (s->expr) {
      const double b = (double)be32s(s->dict_b + 4 * (int64_t)read_id(s->fwd_b, block[i], s->bits_b));
      v = s->expr == 1 ? a + b : (s->expr == 2 ? a - b : 1.0 * a * b);
    }
    inner += v;
  }
  *m += *nblock;
  *nblock = 0;
  return inner;
}

static double segment_sum(const cb_segment *s, int64_t *matched) {
  int64_t first = 0, last = (int64_t)s->num_docs - 1;
  const cb_leaf *scan[CB_MAX_LEAVES];
  int nscan = 0;
  for (int l = 0; l < s->nleaves; l++) {
    const cb_leaf *L = &s->leaves[l];
    if (L->sorted) {
      if (L->hi <= L->lo) return (*matched = 0, 0.0);
      const int64_t a = be32s(L->fwd + 8 * (int64_t)L->lo), b = be32s(L->fwd + 8 * (int64_t)(L->hi - 1) + 4);
      if (a > first) first = a;
      if (b < last) last = b;
    } else {
      scan[nscan++] = L;
    }
  }
  int32_t batch[CB_BATCH];
  int32_t block[CB_BLOCK];
  int nblock = 0;
  double holder = 0.0;
  int64_t m = 0;
  uint32_t ids[CB_BATCH];
  for (int64_t d0 = first; d0 <= last; d0 += CB_BATCH) {
    const int n = (int)((last - d0 + 1) < CB_BATCH ? (last - d0 + 1) : CB_BATCH);
    int k = 0;
    if (nscan == 0) {
      for (int i = 0; i < n; i++) batch[k++] = (int32_t)(d0 + i);
    } else {
      const cb_leaf *L = scan[0];
      for (int i = 0; i < n; i++) ids[i] = read_id(L->fwd, d0 + i, L->bits); /* readDictIds (bulk) */
      for (int i = 0; i < n; i++)
        if (ids[i] - (uint32_t)L->lo < (uint32_t)(L->hi - L->lo)) batch[k++] = (int32_t)(d0 + i);
      for (int l = 1; l < nscan && k; l++) { /* applyAnd on the survivors */
        const cb_leaf *R = scan[l];
        int k2 = 0;
        for (int i = 0; i < k; i++) {
          const uint32_t v = read_id(R->fwd, batch[i], R->bits);
          if (v - (uint32_t)R->lo < (uint32_t)(R->hi - R->lo)) batch[k2++] = batch[i];
        }
        k = k2;
      }
    }
    for (int i = 0; i < k; i++) {
      block[nblock++] = batch[i];
      if (nblock == CB_BLOCK) holder += block_sum(s, block, &nblock, &m);
    }
  }
  if (nblock) holder += block_sum(s, block, &nblock, &m);
  *matched = m;
  return holder;
}

/* Runs the query over every segment with `threads` OpenMP workers; returns the merged SUM and the
 * matched docs (numDocsScanned). */
double cb_run(const cb_segment *segs, int32_t nseg, int32_t threads, int64_t *matched_out) {
  double sums[4096];
  int64_t matched[4096];
  if (nseg > 4096) return 0.0;
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads)
  for (int32_t i = 0; i < nseg; i++) sums[i] = segment_sum(&segs[i], &matched[i]);
  double total = 0.0;
  int64_t mt = 0;
  for (int32_t i = 0; i < nseg; i++) {
    total += sums[i];
    mt += matched[i];
  }
  *matched_out = mt;
  return total;
}

int32_t cb_max_threads(void) { return omp_get_max_threads(); }
