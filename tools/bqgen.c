/* bqgen.c -- data of pinot-perf's BenchmarkQueries segments (config C1), generated
 * natively so 10M-row segments take well under a second.
 *
 * BenchmarkQueries.createTestData (pinot-perf/.../perf/BenchmarkQueries.java:258-268) draws, per row,
 * four values from one Distribution.DataSupplier (Distribution.java:47-53, 79-96):
 *   INT_COL, NO_INDEX_INT_COL, RAW_INT_COL = (int) supplier.getAsLong(), and one more draw that only
 *   keys RAW_STRING_COL's random UUID (not reproducible, not generated here).
 * EXP(lambda): getAsLong = (long) -(Math.log(r.nextDouble()) / lambda) over java.util.Random(42).
 * java.util.Random is restated bit-exactly (48-bit LCG, nextDouble = ((next(26) << 27) + next(27)) *
 * 2^-53); Math.log is the C library's log (both within 1 ulp; a draw whose quotient lies within an ulp
 * of an integer could truncate differently -- synthetic data, the GPU and the oracle read the same
 * segment either way). The supplier continues across segments (BenchmarkQueries.buildSegment
 * snapshots it after every segment), so callers pass the state in and get it back.
 */
#include <math.h>
#include <stdint.h>

#define MULT 0x5DEECE66DLL
#define ADD 0xBLL
#define MASK ((1LL << 48) - 1)

int64_t bq_seed_scramble(int64_t seed) { return (seed ^ MULT) & MASK; }

static inline int32_t next_bits(int64_t *s, int bits) {
  *s = (*s * MULT + ADD) & MASK;
  return (int32_t)(*s >> (48 - bits));
}

static inline double next_double(int64_t *s) {
  const int64_t hi = (int64_t)next_bits(s, 26);
  const int64_t lo = (int64_t)next_bits(s, 27);
  return (double)((hi << 27) + lo) * (1.0 / 9007199254740992.0);
}

void bq_doubles(int64_t seed, int64_t n, double *out) {
  int64_t s = bq_seed_scramble(seed);
  for (int64_t i = 0; i < n; i++) out[i] = next_double(&s);
}

/* Java (long) of a double: NaN -> 0, saturating at the int64 range; then (int) keeps the low 32 bits */
static inline int32_t java_int_of_long_of(double x) {
  int64_t l;
  if (x != x) l = 0;
  else if (x >= 9223372036854775807.0) l = INT64_MAX;
  else if (x <= -9223372036854775808.0) l = INT64_MIN;
  else l = (int64_t)x;
  return (int32_t)(uint32_t)(uint64_t)l;
}

/* rows [0, n) of one segment; *state is the scrambled Random seed, advanced in place */
void bq_generate(int64_t *state, double lambda, int64_t n, int32_t *int_col, int32_t *no_index_int_col,
                 int32_t *raw_int_col) {
  int64_t s = *state;
  for (int64_t i = 0; i < n; i++) {
    int_col[i] = java_int_of_long_of(-(log(next_double(&s)) / lambda));
    no_index_int_col[i] = java_int_of_long_of(-(log(next_double(&s)) / lambda));
    raw_int_col[i] = java_int_of_long_of(-(log(next_double(&s)) / lambda));
    (void)next_double(&s); /* RAW_STRING_COL's UUID key */
  }
  *state = s;
}

/* config C4: `ncols` uniform dict-id columns (splitmix64 over a seed), ids[c][i] in [0, card[c]) */
static inline uint64_t splitmix64(uint64_t *x) {
  uint64_t z = (*x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void c4_generate(uint64_t seed, int64_t first_row, int64_t n, int32_t card, int32_t *out) {
  for (int64_t i = 0; i < n; i++) {
    uint64_t x = seed * 0x100000001B3ull + (uint64_t)(first_row + i);
    out[i] = (int32_t)(((splitmix64(&x) >> 32) * (uint64_t)card) >> 32);
  }
}
