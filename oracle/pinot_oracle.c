/*
 * pinot_oracle.c -- CPU restatement of the reference's byte/integer algorithms on the segment
 * query hot path. TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg as the checker; never linked into libpinot_hip.so.
 *
 * Each function cites the reference code (or, for third-party jars absent from /root/reference,
 * the published algorithm and the reference call site) it follows. Plain C99, no SIMD, no
 * threads: a scalar port timed as "port" in bench.py.
 */
#include <stdint.h>
#include <string.h>
#include <math.h>

/* --------------------------------------------------------------------------------------------
 * Fixed-bit forward index read.
 * pinot-segment-local/src/main/java/org/apache/pinot/segment/local/io/util/PinotDataBitSet.java:74-96
 * (readInt): value i occupies bits [i*b, i*b+b) of a big-endian byte stream, MSB first.
 * ------------------------------------------------------------------------------------------ */
static inline int32_t read_int(const uint8_t *buf, int64_t index, int bits) {
  int64_t bit_offset = index * (int64_t)bits;
  int64_t byte_offset = bit_offset >> 3;
  int bit_in_first = (int)(bit_offset & 7);
  uint32_t cur = buf[byte_offset] & (0xFFu >> bit_in_first);
  int left = bits - (8 - bit_in_first);
  if (left <= 0) return (int32_t)(cur >> (-left));
  while (left > 8) {
    byte_offset++;
    cur = (cur << 8) | buf[byte_offset];
    left -= 8;
  }
  return (int32_t)((cur << left) | ((uint32_t)buf[byte_offset + 1] >> (8 - left)));
}

void oracle_read_fixed_bit(const uint8_t *buf, int bits, int64_t start, int64_t n, int32_t *out) {
  for (int64_t i = 0; i < n; i++) out[i] = read_int(buf, start + i, bits);
}

/* --------------------------------------------------------------------------------------------
 * Sorted forward index -> dict id per doc.
 * SortedIndexReaderImpl.java:114-116: pair (startDocId, endDocId) per dict id, BE int32, inclusive.
 * ------------------------------------------------------------------------------------------ */
static inline int32_t be32(const uint8_t *p) {
  return (int32_t)(((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]);
}

int oracle_sorted_dict_ids(const uint8_t *pairs, int32_t card, int32_t num_docs, int32_t *out) {
  for (int32_t d = 0; d < card; d++) {
    int32_t s = be32(pairs + 8 * (int64_t)d), e = be32(pairs + 8 * (int64_t)d + 4);
    if (s < 0 || e >= num_docs || e < s - 1) return -1;
    for (int32_t i = s; i <= e; i++) out[i] = d;
  }
  return 0;
}

/* --------------------------------------------------------------------------------------------
 * Portable RoaringBitmap decode (RoaringBitmap 1.3.0, pom.xml:805-806; not vendored). Restated
 * from the public RoaringFormatSpec; reference call site BitmapInvertedIndexReader.getDocIds
 * (pinot-segment-local/.../readers/BitmapInvertedIndexReader.java:55-58) which wraps the bytes in
 * an ImmutableRoaringBitmap. Emits the doc ids in increasing order; returns the count, or -1 on
 * malformed input / overflow of cap.
 * ------------------------------------------------------------------------------------------ */
static inline uint16_t le16(const uint8_t *p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static inline uint32_t le32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

int64_t oracle_roaring_decode(const uint8_t *buf, int64_t len, int32_t *out, int64_t cap) {
  if (len < 4) return -1;
  uint32_t cookie = le32(buf);
  int64_t pos;
  int32_t size;
  const uint8_t *runflags = 0;
  int has_run = 0;
  if ((cookie & 0xFFFF) == 12347) {
    has_run = 1;
    size = (int32_t)(cookie >> 16) + 1;
    runflags = buf + 4;
    pos = 4 + (size + 7) / 8;
  } else if (cookie == 12346) {
    if (len < 8) return -1;
    size = (int32_t)le32(buf + 4);
    pos = 8;
  } else {
    return -1;
  }
  const uint8_t *hdr = buf + pos;
  pos += 4 * (int64_t)size;
  int has_offsets = (!has_run) || size >= 4;
  const uint8_t *offs = buf + pos;
  if (has_offsets) pos += 4 * (int64_t)size;
  if (pos > len) return -1;
  int64_t n = 0;
  for (int32_t c = 0; c < size; c++) {
    uint32_t key = le16(hdr + 4 * c);
    int32_t card = le16(hdr + 4 * c + 2) + 1;
    int is_run = has_run && ((runflags[c >> 3] >> (c & 7)) & 1);
    if (has_offsets) pos = le32(offs + 4 * c);
    if (pos > len) return -1;
    const uint8_t *p = buf + pos;
    uint32_t high = key << 16;
    if (is_run) {
      int32_t nruns = le16(p);
      for (int32_t r = 0; r < nruns; r++) {
        uint32_t s = le16(p + 2 + 4 * r), l = (uint32_t)le16(p + 4 + 4 * r) + 1;
        for (uint32_t v = s; v < s + l; v++) {
          if (n >= cap) return -1;
          out[n++] = (int32_t)(high | v);
        }
      }
      pos += 2 + 4 * (int64_t)nruns;
    } else if (card <= 4096) {
      for (int32_t i = 0; i < card; i++) {
        if (n >= cap) return -1;
        out[n++] = (int32_t)(high | le16(p + 2 * i));
      }
      pos += 2 * (int64_t)card;
    } else {
      for (int32_t w = 0; w < 1024; w++) {
        uint64_t word = 0;
        for (int b = 0; b < 8; b++) word |= (uint64_t)p[8 * w + b] << (8 * b);
        while (word) {
          int t = __builtin_ctzll(word);
          if (n >= cap) return -1;
          out[n++] = (int32_t)(high | (uint32_t)(64 * w + t));
          word &= word - 1;
        }
      }
      pos += 8192;
    }
    if (pos > len) return -1;
  }
  return n;
}

/* --------------------------------------------------------------------------------------------
 * clearspring stream-lib 2.9.8 (pom.xml:1416-1418; not vendored) MurmurHash + HyperLogLog, as
 * exercised by DistinctCountHLLAggregationFunction.java:457-466 (convertToHyperLogLog offers
 * dictionary values) and ObjectSerDeUtils.java:733-760. Restated from the library's published
 * source algorithm (MurmurHash2, m = 0x5bd1e995, r = 24; HLL with log2m registers, 5-bit regs).
 * ------------------------------------------------------------------------------------------ */
int32_t oracle_murmur_hash_long(int64_t data) {
  const uint32_t m = 0x5bd1e995u;
  const int r = 24;
  uint32_t h = 0;
  uint32_t k = (uint32_t)data * m;
  k ^= k >> r;
  h ^= k * m;
  k = (uint32_t)(data >> 32) * m;
  k ^= k >> r;
  h *= m;
  h ^= k * m;
  h ^= h >> 13;
  h *= m;
  h ^= h >> 15;
  return (int32_t)h;
}

/* MurmurHash.hash(byte[] data, int length, int seed): Java bytes are signed, the tail mixes
 * sign-extended bytes exactly as the Java source does. */
int32_t oracle_murmur_hash_bytes(const uint8_t *data, int32_t length, int32_t seed) {
  const uint32_t m = 0x5bd1e995u;
  const int r = 24;
  uint32_t h = (uint32_t)seed ^ (uint32_t)length;
  int32_t len4 = length >> 2;
  for (int32_t i = 0; i < len4; i++) {
    int32_t i4 = i << 2;
    uint32_t k = (uint32_t)data[i4 + 3];
    k = k << 8;
    k = k | (uint32_t)data[i4 + 2];
    k = k << 8;
    k = k | (uint32_t)data[i4 + 1];
    k = k << 8;
    k = k | (uint32_t)data[i4 + 0];
    k *= m;
    k ^= k >> r;
    k *= m;
    h *= m;
    h ^= k;
  }
  int32_t len_m = len4 << 2;
  int32_t left = length - len_m;
  if (left != 0) {
    if (left >= 3) h ^= (uint32_t)((int32_t)(int8_t)data[length - 3] << 16);
    if (left >= 2) h ^= (uint32_t)((int32_t)(int8_t)data[length - 2] << 8);
    if (left >= 1) h ^= (uint32_t)(int32_t)(int8_t)data[length - 1];
    h *= m;
  }
  h ^= h >> 13;
  h *= m;
  h ^= h >> 15;
  return (int32_t)h;
}

/* HyperLogLog.offerHashed(int hashedValue): j = x >>> (32 - log2m);
 * r = numberOfLeadingZeros((x << log2m) | (1 << (log2m - 1)) + 1) + 1; registerSet.updateIfGreater */
void oracle_hll_offer_hashed(uint8_t *regs, int log2m, int32_t x) {
  uint32_t ux = (uint32_t)x;
  uint32_t j = ux >> (32 - log2m);
  uint32_t w = (ux << log2m) | ((1u << (log2m - 1)) + 1u);
  uint32_t r = (uint32_t)__builtin_clz(w) + 1u;
  if (r > regs[j]) regs[j] = (uint8_t)r;
}

/* HyperLogLog.cardinality(): alphaMM / sum(2^-reg); linear counting when est <= 5/2 m. */
int64_t oracle_hll_cardinality(const uint8_t *regs, int log2m) {
  int32_t m = 1 << log2m;
  double alpha_mm;
  switch (log2m) {
    case 4: alpha_mm = 0.673 * m * m; break;
    case 5: alpha_mm = 0.697 * m * m; break;
    case 6: alpha_mm = 0.709 * m * m; break;
    default: alpha_mm = (0.7213 / (1 + 1.079 / m)) * m * m;
  }
  double sum = 0.0;
  int32_t zeros = 0;
  for (int32_t j = 0; j < m; j++) {
    sum += 1.0 / (double)(1LL << regs[j]);
    if (regs[j] == 0) zeros++;
  }
  double estimate = alpha_mm * (1.0 / sum);
  if (estimate <= (5.0 / 2.0) * m) {
    if (zeros == 0) return INT64_MAX; /* m * log(m / 0.0) = +Infinity; Math.round(+Infinity) = Long.MAX_VALUE */
    return (int64_t)floor(m * log((double)m / zeros) + 0.5); /* Math.round */
  }
  return (int64_t)floor(estimate + 0.5);
}

/* --------------------------------------------------------------------------------------------
 * Reference-semantics scan loops used by oracle/executor.py (vectorised by hand in C only to keep
 * the CPU baseline honest; semantics follow the cited Java loops).
 * ------------------------------------------------------------------------------------------ */

/* SumAggregationFunction.aggregate (SumAggregationFunction.java:69-101) over one segment:
 * the projection yields blocks of <= 10,000 matched docs (DocIdSetPlanNode.java:29), each block
 * sums into a local double then adds to the holder. */
double oracle_block_sum_f64(const double *vals, int64_t n, int32_t block) {
  double holder = 0.0;
  for (int64_t s = 0; s < n; s += block) {
    int64_t e = s + block < n ? s + block : n;
    double inner = 0.0;
    for (int64_t i = s; i < e; i++) inner += vals[i];
    holder += inner;
  }
  return holder;
}

/* --------------------------------------------------------------------------------------------
 * Compressed raw chunks (ChunkCompressionType SNAPPY=1, LZ4=3, LZ4_LENGTH_PREFIXED=4;
 * pinot-segment-spi/.../compression/ChunkCompressionType.java:22). Pinot hands each chunk to a
 * third-party codec: lz4-java 1.8.0 (LZ4Decompressor.java: safeDecompressor().decompress over the
 * LZ4 *block* format; LZ4WithLengthDecompressor.java: LZ4DecompressorWithLength = 4-byte
 * little-endian original length, then the block) and snappy-java 1.1.10.7 (SnappyDecompressor.java:
 * Snappy.uncompress over the raw snappy format). Restated from the published format specs
 * (lz4 "Block format description", snappy "format_description.txt"). Return the decoded length,
 * or -1 on malformed input / overflow of `cap`.
 * ------------------------------------------------------------------------------------------ */
int64_t oracle_lz4_block_decode(const uint8_t *src, int64_t n, uint8_t *dst, int64_t cap) {
  int64_t ip = 0, op = 0;
  while (ip < n) {
    uint32_t tok = src[ip++];
    int64_t lit = tok >> 4;
    if (lit == 15) {
      uint32_t b;
      do {
        if (ip >= n) return -1;
        b = src[ip++];
        lit += b;
      } while (b == 255);
    }
    if (ip + lit > n || op + lit > cap) return -1;
    for (int64_t i = 0; i < lit; i++) dst[op + i] = src[ip + i];
    ip += lit;
    op += lit;
    if (ip == n) break; /* the last sequence carries literals only */
    if (ip + 2 > n) return -1;
    int64_t off = (int64_t)src[ip] | ((int64_t)src[ip + 1] << 8);
    ip += 2;
    if (off == 0 || off > op) return -1;
    int64_t ml = tok & 15;
    if (ml == 15) {
      uint32_t b;
      do {
        if (ip >= n) return -1;
        b = src[ip++];
        ml += b;
      } while (b == 255);
    }
    ml += 4;
    if (op + ml > cap) return -1;
    for (int64_t i = 0; i < ml; i++) dst[op + i] = dst[op + i - off]; /* overlapping copy repeats */
    op += ml;
  }
  return op;
}

int64_t oracle_snappy_decode(const uint8_t *src, int64_t n, uint8_t *dst, int64_t cap) {
  int64_t ip = 0, op = 0;
  uint64_t ulen = 0;
  for (int shift = 0;; shift += 7) {
    if (ip >= n || shift > 28) return -1;
    uint32_t b = src[ip++];
    ulen |= (uint64_t)(b & 0x7f) << shift;
    if (!(b & 0x80)) break;
  }
  if ((int64_t)ulen > cap) return -1;
  while (ip < n) {
    uint32_t tag = src[ip++];
    int64_t len, off;
    if ((tag & 3) == 0) {
      len = (tag >> 2) + 1;
      if (len > 60) {
        int nb = (int)len - 60;
        if (ip + nb > n) return -1;
        len = 0;
        for (int k = 0; k < nb; k++) len |= (int64_t)src[ip + k] << (8 * k);
        len += 1;
        ip += nb;
      }
      if (ip + len > n || op + len > (int64_t)ulen) return -1;
      for (int64_t i = 0; i < len; i++) dst[op + i] = src[ip + i];
      ip += len;
      op += len;
      continue;
    }
    if ((tag & 3) == 1) {
      if (ip + 1 > n) return -1;
      len = 4 + ((tag >> 2) & 7);
      off = ((int64_t)(tag >> 5) << 8) | src[ip];
      ip += 1;
    } else if ((tag & 3) == 2) {
      if (ip + 2 > n) return -1;
      len = (tag >> 2) + 1;
      off = (int64_t)src[ip] | ((int64_t)src[ip + 1] << 8);
      ip += 2;
    } else {
      if (ip + 4 > n) return -1;
      len = (tag >> 2) + 1;
      off = (int64_t)le32(src + ip);
      ip += 4;
    }
    if (off == 0 || off > op || op + len > (int64_t)ulen) return -1;
    for (int64_t i = 0; i < len; i++) dst[op + i] = dst[op + i - off];
    op += len;
  }
  return op == (int64_t)ulen ? op : -1;
}

/* One chunk of a compressed fixed-byte forward index -> its decoded bytes
 * (BaseChunkForwardIndexReader.decompressChunk, BaseChunkForwardIndexReader.java:204-232). */
int64_t oracle_chunk_decode(int32_t codec, const uint8_t *src, int64_t n, uint8_t *dst, int64_t cap) {
  if (codec == 1) return oracle_snappy_decode(src, n, dst, cap);
  if (codec == 3) return oracle_lz4_block_decode(src, n, dst, cap);
  if (codec == 4) {
    if (n < 4) return -1;
    int64_t want = (int64_t)le32(src);
    int64_t got = oracle_lz4_block_decode(src + 4, n - 4, dst, cap);
    return got == want ? got : -1;
  }
  return -1;
}
