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

/* =============================================================================================================
 * Group-by (SSB Q2.x-Q4.x = BASELINE C3, and C5's DISTINCTCOUNTHLL + GROUP BY): the CPU server path's
 * GroupByOperator over the same segments -- bench.py's full-size group-by parity check and group-by
 * cpu_baseline. TEST / BENCH INFRASTRUCTURE ONLY, like the rest of this file.
 *
 *   - filter: an AND of leaves, each leaf a per-dict-id match table of one column (the host evaluates the
 *     predicates -- EQ / IN / RANGE, or an OR of them on one column, MergeEqInFilterOptimizer's shape -- on the
 *     dictionary VALUES, PredicateEvaluator.getMatchingDictIds semantics). Sorted-column leaves become doc ranges
 *     (SortedIndexBasedFilterOperator.java:52-132: the matching ids' (start, end) pairs, merged; two sorted leaves
 *     intersect, AndDocIdSet.java:134-166); the first scan leaf runs over the candidate docs in 256-doc batches,
 *     the others on its survivors (SVScanDocIdIterator.applyAnd :114-142);
 *   - group keys: DictionaryBasedGroupKeyGenerator's mixed radix (:285-414) over QUERY-GLOBAL dict ids (each
 *     segment's ids remapped through the union of the segments' dictionaries, so a key means the same values in
 *     every segment: the combine's value-keyed merge, GroupByCombineOperator.java:138-147), column 0 least
 *     significant, into a dense table per worker (ArrayBasedHolder);
 *   - SUM of a dictionary INT expression (a, a+b, a-b, a*b; SumAggregationFunction.aggregateGroupBySV :160-180)
 *     accumulated in exact int64 -- the reference's double holder is exact for these integral sums below 2^53 --
 *     plus a COUNT per group (the group set = keys with count > 0);
 *   - DISTINCTCOUNTHLL of a dictionary INT column: clearspring MurmurHash.hashLong((long) value) +
 *     HyperLogLog.offerHashed per matched doc into the group's registers (DistinctCountHLLAggregationFunction
 *     .java:177-185,457-466; Appendix B of SURVEY.md), registers max-merged across workers (:332-350).
 * ============================================================================================================= */
#include <stdlib.h>

#define CG_MAX_LEAVES 8
#define CG_MAX_KEYS 6

typedef struct {
  const uint8_t *fwd; /* fixed-bit BE ids, or card x (start,end) BE int32 pairs for a sorted column */
  int32_t bits;
  int32_t sorted;
  int32_t card;
  int32_t pad;
} cg_col;

typedef struct {
  int32_t num_docs, nleaves, nkeys, nvals;
  cg_col leaf_col[CG_MAX_LEAVES];
  const uint8_t *leaf_match[CG_MAX_LEAVES]; /* card bytes: 1 = the dict id matches */
  cg_col key_col[CG_MAX_KEYS];
  const int32_t *key_remap[CG_MAX_KEYS]; /* segment dict id -> query-global dict id */
  cg_col val_col[2];
  const uint8_t *val_dict[2]; /* BE int32 dictionaries */
  cg_col hll_col;
  const uint8_t *hll_dict; /* BE int32 dictionary, or NULL: no DISTINCTCOUNTHLL */
} cg_segment;

typedef struct {
  int32_t nkeys;
  int32_t expr; /* 0 a, 1 a+b, 2 a-b, 3 a*b; -1 no SUM */
  int32_t log2m;
  int32_t pad;
  int64_t radix[CG_MAX_KEYS];
  int64_t num_keys; /* product of the global cardinalities */
} cg_query;

static inline uint32_t cg_murmur_long(int64_t data) { /* clearspring MurmurHash.hashLong (Appendix B) */
  const uint32_t m = 0x5bd1e995u;
  uint32_t h = 0, k = (uint32_t)data * m;
  k ^= k >> 24;
  h ^= k * m;
  k = (uint32_t)(data >> 32) * m;
  k ^= k >> 24;
  h *= m;
  h ^= k * m;
  h ^= h >> 13;
  h *= m;
  h ^= h >> 15;
  return h;
}

/* dict id of doc d of a sorted column: (start, end) pairs visited in doc order through a monotone cursor */
typedef struct {
  int32_t id, end;
} cg_cursor;

static inline int32_t cg_sorted_id(const cg_col *c, cg_cursor *cur, int32_t d) {
  while (d > cur->end) {
    cur->id++;
    cur->end = be32s(c->fwd + 8 * (int64_t)cur->id + 4);
  }
  return cur->id;
}

static inline int32_t cg_id(const cg_col *c, cg_cursor *cur, int32_t d) {
  return c->sorted ? cg_sorted_id(c, cur, d) : (int32_t)read_id(c->fwd, d, c->bits);
}

/* merged inclusive doc ranges of a sorted leaf's matching ids; returns the count (ranges: 2 ints each) */
static int32_t cg_leaf_ranges(const cg_col *c, const uint8_t *match, int32_t *out) {
  int32_t n = 0;
  for (int32_t id = 0; id < c->card; id++) {
    if (!match[id]) continue;
    const int32_t s = be32s(c->fwd + 8 * (int64_t)id), e = be32s(c->fwd + 8 * (int64_t)id + 4);
    if (e < s) continue;
    if (n && out[2 * n - 1] + 1 == s) {
      out[2 * n - 1] = e;
    } else {
      out[2 * n] = s;
      out[2 * n + 1] = e;
      n++;
    }
  }
  return n;
}

static int32_t cg_intersect(const int32_t *a, int32_t na, const int32_t *b, int32_t nb, int32_t *out) {
  int32_t i = 0, j = 0, n = 0;
  while (i < na && j < nb) {
    const int32_t s = a[2 * i] > b[2 * j] ? a[2 * i] : b[2 * j];
    const int32_t e = a[2 * i + 1] < b[2 * j + 1] ? a[2 * i + 1] : b[2 * j + 1];
    if (s <= e) {
      out[2 * n] = s;
      out[2 * n + 1] = e;
      n++;
    }
    if (a[2 * i + 1] < b[2 * j + 1]) i++;
    else j++;
  }
  return n;
}

static inline int64_t cg_dict_val(const uint8_t *dict, int32_t id) { return be32s(dict + 4 * (int64_t)id); }

/* one segment into this worker's tables; returns the matched docs, or -1 on a bad input */
static int64_t cg_segment_run(const cg_query *q, const cg_segment *s, int64_t *sums, int64_t *counts,
                              uint8_t *regs) {
  /* candidate doc ranges: [0, n) restricted by every sorted leaf */
  int32_t cap = 1;
  for (int l = 0; l < s->nleaves; l++)
    if (s->leaf_col[l].sorted && s->leaf_col[l].card + 1 > cap) cap = s->leaf_col[l].card + 1;
  int32_t *ra = malloc(sizeof(int32_t) * 2 * (size_t)cap), *rb = malloc(sizeof(int32_t) * 2 * (size_t)cap),
          *rt = malloc(sizeof(int32_t) * 2 * (size_t)cap);
  if (!ra || !rb || !rt) {
    free(ra), free(rb), free(rt);
    return -1;
  }
  int32_t nr = 1;
  ra[0] = 0;
  ra[1] = s->num_docs - 1;
  int scan[CG_MAX_LEAVES], nscan = 0;
  for (int l = 0; l < s->nleaves; l++) {
    if (!s->leaf_col[l].sorted) {
      scan[nscan++] = l;
      continue;
    }
    const int32_t nb = cg_leaf_ranges(&s->leaf_col[l], s->leaf_match[l], rb);
    nr = cg_intersect(ra, nr, rb, nb, rt);
    int32_t *t = ra;
    ra = rt;
    rt = t;
  }
  const int m = q->log2m > 0 ? 1 << q->log2m : 0;
  cg_cursor kc[CG_MAX_KEYS], vc[2], hc;
  for (int c = 0; c < CG_MAX_KEYS; c++) kc[c].id = -1, kc[c].end = -1;
  vc[0] = vc[1] = hc = kc[0];
  int32_t batch[CB_BATCH];
  uint32_t ids[CB_BATCH];
  int64_t matched = 0;
  for (int32_t r = 0; r < nr; r++) {
    const int64_t first = ra[2 * r], last = ra[2 * r + 1];
    for (int64_t d0 = first; d0 <= last; d0 += CB_BATCH) {
      const int n = (int)((last - d0 + 1) < CB_BATCH ? (last - d0 + 1) : CB_BATCH);
      int k = 0;
      if (nscan == 0) {
        for (int i = 0; i < n; i++) batch[k++] = (int32_t)(d0 + i);
      } else {
        const cg_col *L = &s->leaf_col[scan[0]];
        const uint8_t *mt = s->leaf_match[scan[0]];
        for (int i = 0; i < n; i++) ids[i] = read_id(L->fwd, d0 + i, L->bits);
        for (int i = 0; i < n; i++)
          if (mt[ids[i]]) batch[k++] = (int32_t)(d0 + i);
        for (int l = 1; l < nscan && k; l++) {
          const cg_col *R = &s->leaf_col[scan[l]];
          const uint8_t *mr = s->leaf_match[scan[l]];
          int k2 = 0;
          for (int i = 0; i < k; i++)
            if (mr[read_id(R->fwd, batch[i], R->bits)]) batch[k2++] = batch[i];
          k = k2;
        }
      }
      for (int i = 0; i < k; i++) {
        const int32_t d = batch[i];
        int64_t key = 0;
        for (int c = 0; c < s->nkeys; c++)
          key += (int64_t)s->key_remap[c][cg_id(&s->key_col[c], &kc[c], d)] * q->radix[c];
        counts[key]++;
        if (q->expr >= 0) {
          const int64_t a = cg_dict_val(s->val_dict[0], cg_id(&s->val_col[0], &vc[0], d));
          int64_t v = a;
          if (q->expr) {
            const int64_t b = cg_dict_val(s->val_dict[1], cg_id(&s->val_col[1], &vc[1], d));
            v = q->expr == 1 ? a + b : (q->expr == 2 ? a - b : a * b);
          }
          sums[key] += v;
        }
        if (s->hll_dict) {
          const uint32_t x = cg_murmur_long(cg_dict_val(s->hll_dict, cg_id(&s->hll_col, &hc, d)));
          const uint32_t j = x >> (32 - q->log2m);
          const uint32_t w = (x << q->log2m) | ((1u << (q->log2m - 1)) + 1u);
          const uint8_t rho = (uint8_t)(__builtin_clz(w) + 1);
          uint8_t *g = regs + key * m;
          if (rho > g[j]) g[j] = rho;
        }
      }
      matched += k;
    }
  }
  free(ra), free(rb), free(rt);
  return matched;
}

/* Runs the group-by over every segment with `threads` workers, each with its own dense tables, merged at the
 * end (sums / counts added, registers max-ed). Outputs: sums[num_keys], counts[num_keys], regs[num_keys << log2m]
 * (when log2m > 0), *matched = numDocsScanned. Returns 0, or -1 (bad input / out of memory). */
int32_t cg_run(const cg_query *q, const cg_segment *segs, int32_t nseg, int32_t threads, int64_t *sums,
               int64_t *counts, uint8_t *regs, int64_t *matched_out) {
  const int64_t nk = q->num_keys;
  const int64_t m = q->log2m > 0 ? (int64_t)1 << q->log2m : 0;
  if (nk <= 0 || threads <= 0 || q->nkeys > CG_MAX_KEYS) return -1;
  int64_t **ts = calloc((size_t)threads, sizeof(int64_t *)), **tc = calloc((size_t)threads, sizeof(int64_t *));
  uint8_t **tr = calloc((size_t)threads, sizeof(uint8_t *));
  int64_t *tm = calloc((size_t)threads, sizeof(int64_t));
  int bad = !ts || !tc || !tr || !tm;
  for (int t = 0; !bad && t < threads; t++) {
    ts[t] = calloc((size_t)nk, sizeof(int64_t));
    tc[t] = calloc((size_t)nk, sizeof(int64_t));
    tr[t] = m ? calloc((size_t)(nk * m), 1) : NULL;
    bad |= !ts[t] || !tc[t] || (m && !tr[t]);
  }
  if (!bad) {
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads) reduction(| : bad)
    for (int32_t i = 0; i < nseg; i++) {
      const int t = omp_get_thread_num();
      const int64_t r = cg_segment_run(q, &segs[i], ts[t], tc[t], tr[t]);
      if (r < 0) bad = 1;
      else tm[t] += r;
    }
  }
  if (!bad) {
    int64_t mt = 0;
    for (int t = 0; t < threads; t++) mt += tm[t];
    *matched_out = mt;
#pragma omp parallel for schedule(static) num_threads(threads)
    for (int64_t k = 0; k < nk; k++) {
      int64_t s = 0, c = 0;
      for (int t = 0; t < threads; t++) s += ts[t][k], c += tc[t][k];
      sums[k] = s;
      counts[k] = c;
      for (int64_t j = 0; j < m; j++) {
        uint8_t x = 0;
        for (int t = 0; t < threads; t++)
          if (tr[t][k * m + j] > x) x = tr[t][k * m + j];
        regs[k * m + j] = x;
      }
    }
  }
  for (int t = 0; ts && tc && tr && t < threads; t++) free(ts[t]), free(tc[t]), free(tr[t]);
  free(ts), free(tc), free(tr), free(tm);
  return bad ? -1 : 0;
}
