/*
 * ssbgen.c -- synthetic SSB "flattened lineorder" segment generator (benchmark / test data).
 *
 * Emits Pinot segment encodings directly (sorted dictionary + bit-packed MSB-first big-endian
 * forward index, b = getNumBitsPerValue(card-1)), one column of one segment per call, so that
 * bench.py and the SSB parity tests can build SF100/SF1000-sized segments in seconds. Neither the
 * product nor the oracle depends on it: both read the bytes it produces.
 *
 * Row model (O'Neil et al., "Star Schema Benchmark", rev. 3; SSB dbgen value domains), one
 * counter-based pseudo-random stream per (seed, row, attribute), so any row range regenerates
 * identically:
 *   orderdate uniform over 1992-01-01 .. 1998-08-02 -> D_YEAR, D_YEARMONTHNUM, D_YEARMONTH,
 *             D_WEEKNUMINYEAR, LO_ORDERDATE (yyyymmdd); layout 1 instead sorts the
 *             table by orderdate: row r of R gets day floor(r * 2406 / R)
 *   LO_QUANTITY 1..50, LO_DISCOUNT 0..10, LO_TAX 0..8
 *   LO_PARTKEY 1..200000*floor(1+log2 SF), LO_CUSTKEY 1..30000*SF, LO_SUPPKEY 1..2000*SF
 *   p_retailprice(pk) = 90000 + (pk/10 mod 20001) + 100*(pk mod 1000)   (cents, TPC-H formula)
 *   LO_EXTENDEDPRICE = LO_QUANTITY * retailprice; LO_REVENUE = ext * (100 - disc) / 100;
 *   LO_SUPPLYCOST = 6 * retailprice / 10
 *   customer / supplier: nation = H(key) mod 25, city = nation*10 + H'(key) mod 10, region by nation
 *   part: mfgr 1..5, category mfgr*10 + 1..5, brand1 category*100 + 1..40 (strings "MFGR#...")
 * Dictionaries hold exactly the values present in the segment (presence bitmap over the domain).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum {
  C_LO_ORDERDATE = 0,
  C_D_YEAR,
  C_D_YEARMONTHNUM,
  C_D_YEARMONTH,
  C_D_WEEKNUMINYEAR,
  C_LO_QUANTITY,
  C_LO_DISCOUNT,
  C_LO_TAX,
  C_LO_EXTENDEDPRICE,
  C_LO_REVENUE,
  C_LO_SUPPLYCOST,
  C_LO_CUSTKEY,
  C_LO_PARTKEY,
  C_LO_SUPPKEY,
  C_C_CITY,
  C_C_NATION,
  C_C_REGION,
  C_S_CITY,
  C_S_NATION,
  C_S_REGION,
  C_P_MFGR,
  C_P_CATEGORY,
  C_P_BRAND1,
  C_NUM_COLUMNS
};

static const char *COLUMN_NAMES[C_NUM_COLUMNS] = {
    "LO_ORDERDATE", "D_YEAR", "D_YEARMONTHNUM", "D_YEARMONTH", "D_WEEKNUMINYEAR", "LO_QUANTITY",
    "LO_DISCOUNT", "LO_TAX", "LO_EXTENDEDPRICE", "LO_REVENUE", "LO_SUPPLYCOST", "LO_CUSTKEY",
    "LO_PARTKEY", "LO_SUPPKEY", "C_CITY", "C_NATION", "C_REGION", "S_CITY", "S_NATION", "S_REGION",
    "P_MFGR", "P_CATEGORY", "P_BRAND1"};
/* 0 = INT, 4 = STRING (PHIP_TYPE_*) */
static const int COLUMN_TYPES[C_NUM_COLUMNS] = {0, 0, 0, 4, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 4, 4, 4, 4, 4, 4, 4, 4, 4};

/* TPC-H nations (n_nationkey order) and their region keys */
static const char *NATIONS[25] = {"ALGERIA", "ARGENTINA", "BRAZIL", "CANADA", "EGYPT", "ETHIOPIA", "FRANCE",
                                  "GERMANY", "INDIA", "INDONESIA", "IRAN", "IRAQ", "JAPAN", "JORDAN", "KENYA",
                                  "MOROCCO", "MOZAMBIQUE", "PERU", "CHINA", "ROMANIA", "SAUDI ARABIA", "VIETNAM",
                                  "RUSSIA", "UNITED KINGDOM", "UNITED STATES"};
static const int NATION_REGION[25] = {0, 1, 1, 1, 4, 0, 3, 3, 2, 2, 4, 4, 2, 4, 0, 0, 0, 1, 2, 3, 4, 2, 3, 3, 1};
static const char *REGIONS[5] = {"AFRICA", "AMERICA", "ASIA", "EUROPE", "MIDDLE EAST"};
static const char *MONTHS[12] = {"Jan", "Feb", "Mar", "Apr", "May", "Jun", "Jul", "Aug", "Sep", "Oct", "Nov", "Dec"};

#define NDAYS 2406 /* 1992-01-01 .. 1998-08-02 */

static inline uint64_t splitmix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
static inline uint64_t H(uint64_t seed, uint64_t row, uint64_t stream) {
  return splitmix(seed ^ splitmix(row * 0x100000001B3ull + stream * 0xD1B54A32D192ED03ull));
}

/* ---- calendar ---------------------------------------------------------------------------- */
static int g_cal_ready = 0;
static int32_t g_datekey[NDAYS], g_year[NDAYS], g_ym[NDAYS], g_week[NDAYS], g_ymidx[NDAYS];
static void calendar(void) {
  if (g_cal_ready) return;
  static const int mdays[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  int y = 1992, m = 0, d = 1, doy = 1;
  for (int i = 0; i < NDAYS; i++) {
    g_datekey[i] = y * 10000 + (m + 1) * 100 + d;
    g_year[i] = y;
    g_ym[i] = y * 100 + m + 1;
    g_week[i] = (doy - 1) / 7 + 1;
    g_ymidx[i] = (y - 1992) * 12 + m;
    int leap = (y % 4 == 0);
    int md = mdays[m] + (m == 1 && leap);
    d++;
    doy++;
    if (d > md) {
      d = 1;
      m++;
      if (m == 12) {
        m = 0;
        y++;
        doy = 1;
      }
    }
  }
  g_cal_ready = 1;
}

/* ---- string domains (sorted) ------------------------------------------------------------- */
typedef struct {
  int n;
  int width;
  char (*s)[32];
  int32_t *rank_of; /* natural index -> sorted rank */
} StrDomain;

static int cmp_str(const void *a, const void *b) { return strcmp(*(const char *const *)a, *(const char *const *)b); }

static void build_domain(StrDomain *d, char (*names)[32], int n) {
  const char **ptrs = malloc(sizeof(char *) * n);
  for (int i = 0; i < n; i++) ptrs[i] = names[i];
  qsort(ptrs, n, sizeof(char *), cmp_str);
  d->n = n;
  d->s = malloc(32 * (size_t)n);
  d->rank_of = malloc(sizeof(int32_t) * n);
  d->width = 1;
  for (int i = 0; i < n; i++) {
    strcpy(d->s[i], ptrs[i]);
    int l = (int)strlen(ptrs[i]);
    if (l > d->width) d->width = l;
    int nat = (int)((const char(*)[32])ptrs[i] - (const char(*)[32])names);
    d->rank_of[nat] = i;
  }
  free(ptrs);
}

static StrDomain D_CITY, D_NATION, D_REGION, D_MFGR, D_CAT, D_BRAND, D_YM;
static int g_dom_ready = 0;
static char g_city_names[250][32], g_nation_names[25][32], g_region_names[5][32], g_mfgr_names[5][32],
    g_cat_names[25][32], g_brand_names[1000][32], g_ym_names[84][32];

static void domains(void) {
  if (g_dom_ready) return;
  for (int n = 0; n < 25; n++) {
    snprintf(g_nation_names[n], 32, "%s", NATIONS[n]);
    for (int k = 0; k < 10; k++) snprintf(g_city_names[n * 10 + k], 32, "%-9.9s%d", NATIONS[n], k);
  }
  for (int r = 0; r < 5; r++) snprintf(g_region_names[r], 32, "%s", REGIONS[r]);
  for (int m = 0; m < 5; m++) {
    snprintf(g_mfgr_names[m], 32, "MFGR#%d", m + 1);
    for (int c = 0; c < 5; c++) {
      snprintf(g_cat_names[m * 5 + c], 32, "MFGR#%d%d", m + 1, c + 1);
      for (int b = 0; b < 40; b++) snprintf(g_brand_names[(m * 5 + c) * 40 + b], 32, "MFGR#%d%d%d", m + 1, c + 1, b + 1);
    }
  }
  for (int i = 0; i < 84; i++) snprintf(g_ym_names[i], 32, "%s%d", MONTHS[i % 12], 1992 + i / 12);
  build_domain(&D_CITY, g_city_names, 250);
  build_domain(&D_NATION, g_nation_names, 25);
  build_domain(&D_REGION, g_region_names, 5);
  build_domain(&D_MFGR, g_mfgr_names, 5);
  build_domain(&D_CAT, g_cat_names, 25);
  build_domain(&D_BRAND, g_brand_names, 1000);
  build_domain(&D_YM, g_ym_names, 84);
  g_dom_ready = 1;
}

/* ---- per-row attributes ------------------------------------------------------------------ */
typedef struct {
  int32_t sf;
  int64_t nparts, ncust, nsupp;
  int64_t total_rows;  /* sorted layout: orderdate of row r = day floor(r * NDAYS / total_rows) */
  int32_t sorted;
} Scale;

static Scale scale_of(int32_t sf) {
  Scale s;
  s.sf = sf;
  s.total_rows = 6000000LL * sf;
  s.sorted = 0;
  s.nparts = 200000LL * (int64_t)floor(1.0 + log2((double)sf));
  s.ncust = 30000LL * sf;
  s.nsupp = 2000LL * sf;
  return s;
}

static inline int64_t retail(int64_t pk) { return 90000 + ((pk / 10) % 20001) + 100 * (pk % 1000); }

/* domain index of column c for row r (numeric: value - domain_min; strings: natural index) */
static inline int64_t row_value(int c, uint64_t seed, uint64_t r, const Scale *s) {
  int day = s->sorted ? (int)((int64_t)r * NDAYS / s->total_rows) : (int)(H(seed, r, 1) % NDAYS);
  switch (c) {
    case C_LO_ORDERDATE: return g_datekey[day];
    case C_D_YEAR: return g_year[day];
    case C_D_YEARMONTHNUM: return g_ym[day];
    case C_D_YEARMONTH: return g_ymidx[day];
    case C_D_WEEKNUMINYEAR: return g_week[day];
    case C_LO_QUANTITY: return 1 + (int64_t)(H(seed, r, 2) % 50);
    case C_LO_DISCOUNT: return (int64_t)(H(seed, r, 3) % 11);
    case C_LO_TAX: return (int64_t)(H(seed, r, 4) % 9);
    case C_LO_CUSTKEY: return 1 + (int64_t)(H(seed, r, 6) % (uint64_t)s->ncust);
    case C_LO_PARTKEY: return 1 + (int64_t)(H(seed, r, 5) % (uint64_t)s->nparts);
    case C_LO_SUPPKEY: return 1 + (int64_t)(H(seed, r, 7) % (uint64_t)s->nsupp);
    default: break;
  }
  int64_t pk = 1 + (int64_t)(H(seed, r, 5) % (uint64_t)s->nparts);
  int64_t ck = 1 + (int64_t)(H(seed, r, 6) % (uint64_t)s->ncust);
  int64_t sk = 1 + (int64_t)(H(seed, r, 7) % (uint64_t)s->nsupp);
  int64_t qty = 1 + (int64_t)(H(seed, r, 2) % 50);
  int64_t disc = (int64_t)(H(seed, r, 3) % 11);
  switch (c) {
    case C_LO_EXTENDEDPRICE: return qty * retail(pk);
    case C_LO_REVENUE: return qty * retail(pk) * (100 - disc) / 100;
    case C_LO_SUPPLYCOST: return 6 * retail(pk) / 10;
    case C_C_NATION: return (int64_t)(splitmix(seed ^ (uint64_t)ck * 31 + 11) % 25);
    case C_C_CITY: {
      int64_t n = (int64_t)(splitmix(seed ^ (uint64_t)ck * 31 + 11) % 25);
      return n * 10 + (int64_t)(splitmix(seed ^ (uint64_t)ck * 37 + 13) % 10);
    }
    case C_C_REGION: return NATION_REGION[splitmix(seed ^ (uint64_t)ck * 31 + 11) % 25];
    case C_S_NATION: return (int64_t)(splitmix(seed ^ (uint64_t)sk * 41 + 17) % 25);
    case C_S_CITY: {
      int64_t n = (int64_t)(splitmix(seed ^ (uint64_t)sk * 41 + 17) % 25);
      return n * 10 + (int64_t)(splitmix(seed ^ (uint64_t)sk * 43 + 19) % 10);
    }
    case C_S_REGION: return NATION_REGION[splitmix(seed ^ (uint64_t)sk * 41 + 17) % 25];
    case C_P_MFGR: return (int64_t)(splitmix(seed ^ (uint64_t)pk * 47 + 23) % 5);
    case C_P_CATEGORY: {
      int64_t m = (int64_t)(splitmix(seed ^ (uint64_t)pk * 47 + 23) % 5);
      return m * 5 + (int64_t)(splitmix(seed ^ (uint64_t)pk * 53 + 29) % 5);
    }
    case C_P_BRAND1: {
      int64_t m = (int64_t)(splitmix(seed ^ (uint64_t)pk * 47 + 23) % 5);
      int64_t cat = m * 5 + (int64_t)(splitmix(seed ^ (uint64_t)pk * 53 + 29) % 5);
      return cat * 40 + (int64_t)(splitmix(seed ^ (uint64_t)pk * 59 + 31) % 40);
    }
  }
  return 0;
}

static const StrDomain *str_domain(int c) {
  switch (c) {
    case C_D_YEARMONTH: return &D_YM;
    case C_C_CITY:
    case C_S_CITY: return &D_CITY;
    case C_C_NATION:
    case C_S_NATION: return &D_NATION;
    case C_C_REGION:
    case C_S_REGION: return &D_REGION;
    case C_P_MFGR: return &D_MFGR;
    case C_P_CATEGORY: return &D_CAT;
    case C_P_BRAND1: return &D_BRAND;
  }
  return 0;
}

/* numeric domain [lo, hi] */
static void num_domain(int c, const Scale *s, int64_t *lo, int64_t *hi) {
  switch (c) {
    case C_LO_ORDERDATE: *lo = 19920101; *hi = 19981231; return;
    case C_D_YEAR: *lo = 1992; *hi = 1998; return;
    case C_D_YEARMONTHNUM: *lo = 199201; *hi = 199812; return;
    case C_D_WEEKNUMINYEAR: *lo = 1; *hi = 53; return;
    case C_LO_QUANTITY: *lo = 1; *hi = 50; return;
    case C_LO_DISCOUNT: *lo = 0; *hi = 10; return;
    case C_LO_TAX: *lo = 0; *hi = 8; return;
    case C_LO_EXTENDEDPRICE:
    case C_LO_REVENUE: *lo = 0; *hi = 50LL * 210000; return;
    case C_LO_SUPPLYCOST: *lo = 0; *hi = 6LL * 210000 / 10; return;
    case C_LO_CUSTKEY: *lo = 1; *hi = s->ncust; return;
    case C_LO_PARTKEY: *lo = 1; *hi = s->nparts; return;
    case C_LO_SUPPKEY: *lo = 1; *hi = s->nsupp; return;
  }
  *lo = 0;
  *hi = 0;
}

int32_t ssbgen_num_columns(void) { return C_NUM_COLUMNS; }
const char *ssbgen_column_name(int32_t c) { return (c >= 0 && c < C_NUM_COLUMNS) ? COLUMN_NAMES[c] : 0; }
int32_t ssbgen_column_type(int32_t c) { return (c >= 0 && c < C_NUM_COLUMNS) ? COLUMN_TYPES[c] : -1; }

static int bits_for(int32_t max_value) {
  if (max_value <= 1) return 1;
  int b = 0;
  while (max_value > 0) {
    b++;
    max_value >>= 1;
  }
  return b;
}

/* Generate column c of rows [first_row, first_row + nrows). Buffers: fwd >= ceil(nrows*31/8)+8,
 * dict >= domain size * width. layout 1 = rows sorted by LO_ORDERDATE: a column whose
 * dict ids are then non-decreasing over the segment is written as Pinot writes sorted columns -- card x
 * (startDocId, endDocId) BE int32 (SortedIndexReaderImpl.java:114-116) -- and *out_sorted = 1.
 * Returns 0 on success. */
int32_t ssbgen_column(uint64_t seed, int64_t first_row, int32_t nrows, int32_t sf, int32_t c, int32_t layout,
                      uint8_t *fwd, int64_t fwd_cap, uint8_t *dict, int64_t dict_cap, int32_t *out_card,
                      int32_t *out_bits, int64_t *out_fwd_len, int64_t *out_dict_len, int32_t *out_width,
                      int32_t *out_sorted) {
  if (c < 0 || c >= C_NUM_COLUMNS || nrows <= 0 || sf <= 0) return 1;
  calendar();
  domains();
  Scale s = scale_of(sf);
  s.sorted = layout == 1;
  const StrDomain *sd = str_domain(c);
  int64_t lo = 0, hi = 0;
  if (sd) {
    hi = sd->n - 1;
  } else {
    num_domain(c, &s, &lo, &hi);
  }
  const int64_t dom = hi - lo + 1;
  uint64_t *present = calloc((size_t)(dom + 63) / 64, 8);
  int32_t *idx = malloc(sizeof(int32_t) * (size_t)nrows);
  if (!present || !idx) return 2;
  for (int32_t i = 0; i < nrows; i++) {
    int64_t v = row_value(c, seed, (uint64_t)(first_row + i), &s);
    int64_t k = sd ? sd->rank_of[v] : v - lo;
    idx[i] = (int32_t)k;
    present[k >> 6] |= 1ull << (k & 63);
  }
  /* rank of each present domain index */
  int64_t nw = (dom + 63) / 64;
  int32_t *prefix = malloc(sizeof(int32_t) * (size_t)(nw + 1));
  int32_t acc = 0;
  for (int64_t w = 0; w < nw; w++) {
    prefix[w] = acc;
    acc += __builtin_popcountll(present[w]);
  }
  prefix[nw] = acc;
  const int32_t card = acc;
  const int bits = bits_for(card - 1);
  const int width = sd ? sd->width : 4;
  if ((int64_t)card * width > dict_cap || ((int64_t)nrows * bits + 7) / 8 + 8 > fwd_cap) {
    free(present);
    free(idx);
    free(prefix);
    return 3;
  }
  /* dictionary (sorted = domain order) */
  int32_t d = 0;
  for (int64_t w = 0; w < nw; w++) {
    uint64_t x = present[w];
    while (x) {
      int t = __builtin_ctzll(x);
      x &= x - 1;
      int64_t k = w * 64 + t;
      if (sd) {
        memset(dict + (int64_t)d * width, 0, width);
        memcpy(dict + (int64_t)d * width, sd->s[k], strlen(sd->s[k]));
      } else {
        uint32_t v = (uint32_t)(int32_t)(k + lo);
        dict[4 * (int64_t)d] = (uint8_t)(v >> 24);
        dict[4 * (int64_t)d + 1] = (uint8_t)(v >> 16);
        dict[4 * (int64_t)d + 2] = (uint8_t)(v >> 8);
        dict[4 * (int64_t)d + 3] = (uint8_t)v;
      }
      d++;
    }
  }
  int sorted = 1;
  for (int32_t i = 1; i < nrows && sorted; i++) sorted = idx[i] >= idx[i - 1];
  *out_sorted = sorted && layout == 1;
  if (*out_sorted) {
    /* sorted forward index: per dict id its inclusive doc range (every dictionary value is present) */
    if ((int64_t)card * 8 > fwd_cap) {
      free(present);
      free(idx);
      free(prefix);
      return 3;
    }
    int32_t id = -1;
    for (int32_t i = 0; i <= nrows; i++) {
      int32_t cur = -1;
      if (i < nrows) {
        int64_t k = idx[i];
        cur = prefix[k >> 6] + __builtin_popcountll(present[k >> 6] & ((1ull << (k & 63)) - 1));
      }
      if (cur != id) {
        if (id >= 0) {  /* end of id's range at doc i-1 */
          uint32_t e = (uint32_t)(i - 1);
          uint8_t *p = fwd + 8 * (int64_t)id + 4;
          p[0] = (uint8_t)(e >> 24); p[1] = (uint8_t)(e >> 16); p[2] = (uint8_t)(e >> 8); p[3] = (uint8_t)e;
        }
        if (cur >= 0) {
          uint32_t b = (uint32_t)i;
          uint8_t *p = fwd + 8 * (int64_t)cur;
          p[0] = (uint8_t)(b >> 24); p[1] = (uint8_t)(b >> 16); p[2] = (uint8_t)(b >> 8); p[3] = (uint8_t)b;
        }
        id = cur;
      }
    }
    free(present);
    free(idx);
    free(prefix);
    *out_card = card;
    *out_bits = bits;
    *out_fwd_len = (int64_t)card * 8;
    *out_dict_len = (int64_t)card * width;
    *out_width = sd ? width : 0;
    return 0;
  }
  /* forward index: MSB-first big-endian bit packing of the dict ids */
  const int64_t nbytes = ((int64_t)nrows * bits + 7) / 8;
  memset(fwd, 0, (size_t)nbytes + 8);
  uint64_t bitpos = 0;
  for (int32_t i = 0; i < nrows; i++) {
    int64_t k = idx[i];
    uint64_t id = (uint64_t)(prefix[k >> 6] + __builtin_popcountll(present[k >> 6] & ((1ull << (k & 63)) - 1)));
    /* write `bits` bits of id at bitpos */
    uint64_t byte = bitpos >> 3;
    int off = (int)(bitpos & 7);
    /* value aligned into a 64-bit big-endian window starting at byte */
    uint64_t win = id << (64 - bits - off);
    for (int b = 0; b < 8 && (b * 8) < off + bits; b++) fwd[byte + b] |= (uint8_t)(win >> (56 - 8 * b));
    bitpos += (uint64_t)bits;
  }
  free(present);
  free(idx);
  free(prefix);
  *out_card = card;
  *out_bits = bits;
  *out_fwd_len = nbytes;
  *out_dict_len = (int64_t)card * width;
  *out_width = sd ? width : 0;
  return 0;
}
