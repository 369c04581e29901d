// codec.h -- entropy-coded chunk formats (ChunkCompressionType GZIP = 5, ZSTANDARD = 2) for the GPU chunk decode
// (load.hip chunk_decode_kernel), written as plain host/device C++ so the same source is unit-tested on the CPU
// (tests/codec/) against the libraries the reference binds (java.util.zip = zlib; zstd-jni = libzstd).
//
// GZIP: GzipCompressor (pinot-segment-local/.../io/compression/GzipCompressor.java:38-46) writes a zlib stream
// (java.util.zip.Deflater: RFC 1950 header, RFC 1951 deflate, Adler-32) followed by the uncompressed length
// (4 bytes, big-endian); GzipDecompressor (:40-52) inflates it with java.util.zip.Inflater. inflate_zlib below
// restates RFC 1950/1951 (stored, fixed and dynamic Huffman blocks; canonical codes decoded a bit at a time).
// Its structure -- huff_build's over-subscribed / incomplete / complete return convention, huff_decode's
// code / first / index walk and the length / distance base + extra-bit tables -- follows Mark Adler's puff.c
// (zlib contrib/puff, Copyright (C) 2002-2013 Mark Adler, zlib licence), the reference inflater of RFC 1951.
//
// ZSTANDARD: ZstandardCompressor / ZstandardDecompressor (…/ZstandardCompressor.java, ZstandardDecompressor.java)
// call zstd-jni Zstd.compress / Zstd.decompress: one RFC 8878 frame. zstd_decompress below restates the frame
// format (raw / RLE / compressed blocks; raw, RLE, Huffman-compressed and treeless literals with 1 or 4 streams;
// predefined, RLE, FSE-compressed and repeat sequence tables; repeat offsets); dictionaries are rejected and the
// optional content checksum is skipped, not verified.
//
// Both decoders are serial (one lane runs them; the caller provides the workspace, in LDS on the GPU) and return
// the decoded length, or -1 for malformed input -- the load then fails, as Inflater / Zstd throw.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define PHIP_HD __host__ __device__
#else
#define PHIP_HD
#endif

namespace phip {
namespace codec {

// ------------------------------------------------------------------------------------------------ inflate
struct InBits {
  const uint8_t *p;
  int n;
  int pos;
  uint32_t buf;
  int cnt;
  int err;
};

PHIP_HD inline uint32_t in_bits(InBits &s, int need) {
  uint32_t val = s.buf;
  while (s.cnt < need) {
    if (s.pos >= s.n) {
      s.err = 1;
      return 0;
    }
    val |= (uint32_t)s.p[s.pos++] << s.cnt;
    s.cnt += 8;
  }
  s.buf = need >= 32 ? 0 : (val >> need);
  s.cnt -= need;
  return need >= 32 ? val : (val & ((1u << need) - 1u));
}

struct Huff {
  int16_t *count;   // [16] codes per length
  int16_t *symbol;  // symbols in canonical order
};

// canonical code from lengths; returns < 0 if over-subscribed, > 0 if incomplete, 0 if complete
PHIP_HD inline int huff_build(Huff &h, const int16_t *length, int n) {
  int16_t offs[16];
  for (int len = 0; len < 16; len++) h.count[len] = 0;
  for (int s = 0; s < n; s++) h.count[length[s]]++;
  if (h.count[0] == n) return 0;
  int left = 1;
  for (int len = 1; len < 16; len++) {
    left <<= 1;
    left -= h.count[len];
    if (left < 0) return left;
  }
  offs[1] = 0;
  for (int len = 1; len < 15; len++) offs[len + 1] = (int16_t)(offs[len] + h.count[len]);
  for (int s = 0; s < n; s++)
    if (length[s] != 0) h.symbol[offs[length[s]]++] = (int16_t)s;
  return left;
}

PHIP_HD inline int huff_decode(InBits &s, const Huff &h) {
  int code = 0, first = 0, index = 0;
  for (int len = 1; len < 16; len++) {
    code |= (int)in_bits(s, 1);
    if (s.err) return -1;
    const int count = h.count[len];
    if (code - count < first) return h.symbol[index + (code - first)];
    index += count;
    first += count;
    first <<= 1;
    code <<= 1;
  }
  return -1;
}

// workspace: 2 x 16 counts + 288 + 30 symbols + 320 lengths (int16)
constexpr int kInflateWs = (16 + 16 + 288 + 30 + 320) * 2;

PHIP_HD inline int inflate_codes(InBits &s, uint8_t *out, int &op, int cap, const Huff &lencode, const Huff &distcode) {
  const int16_t lbase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
  const int16_t lext[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
  const int16_t dbase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
  const int16_t dext[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
  for (;;) {
    int sym = huff_decode(s, lencode);
    if (sym < 0) return -1;
    if (sym < 256) {
      if (op >= cap) return -1;
      out[op++] = (uint8_t)sym;
    } else if (sym == 256) {
      return 0;
    } else {
      sym -= 257;
      if (sym >= 29) return -1;
      const int len = lbase[sym] + (int)in_bits(s, lext[sym]);
      const int ds = huff_decode(s, distcode);
      if (ds < 0 || ds >= 30) return -1;
      const int dist = dbase[ds] + (int)in_bits(s, dext[ds]);
      if (s.err || dist > op || len > cap - op) return -1;
      for (int i = 0; i < len; i++, op++) out[op] = out[op - dist];
    }
  }
}

// raw deflate (RFC 1951) into out[0, cap); returns the output length or -1; *consumed = input bytes used
PHIP_HD inline int inflate_raw(const uint8_t *in, int n, uint8_t *out, int cap, uint8_t *ws, int *consumed) {
  InBits s{in, n, 0, 0u, 0, 0};
  int16_t *w16 = (int16_t *)ws;
  Huff lencode{w16, w16 + 32};
  Huff distcode{w16 + 16, w16 + 32 + 288};
  int16_t *lengths = w16 + 32 + 288 + 30;
  int op = 0, last;
  do {
    last = (int)in_bits(s, 1);
    const int type = (int)in_bits(s, 2);
    if (s.err) return -1;
    if (type == 0) {  // stored
      s.buf = 0;
      s.cnt = 0;
      if (s.pos + 4 > n) return -1;
      const int len = in[s.pos] | (in[s.pos + 1] << 8);
      const int nlen = in[s.pos + 2] | (in[s.pos + 3] << 8);
      s.pos += 4;
      if (len != (~nlen & 0xffff) || s.pos + len > n || len > cap - op) return -1;
      for (int i = 0; i < len; i++) out[op++] = in[s.pos++];
    } else if (type == 1) {  // fixed Huffman codes
      int sym = 0;
      for (; sym < 144; sym++) lengths[sym] = 8;
      for (; sym < 256; sym++) lengths[sym] = 9;
      for (; sym < 280; sym++) lengths[sym] = 7;
      for (; sym < 288; sym++) lengths[sym] = 8;
      huff_build(lencode, lengths, 288);
      for (sym = 0; sym < 30; sym++) lengths[sym] = 5;
      huff_build(distcode, lengths, 30);
      if (inflate_codes(s, out, op, cap, lencode, distcode)) return -1;
    } else if (type == 2) {  // dynamic
      const int16_t order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
      const int nlen = (int)in_bits(s, 5) + 257, ndist = (int)in_bits(s, 5) + 1, ncode = (int)in_bits(s, 4) + 4;
      if (s.err || nlen > 286 || ndist > 30) return -1;
      int idx;
      for (idx = 0; idx < ncode; idx++) lengths[order[idx]] = (int16_t)in_bits(s, 3);
      for (; idx < 19; idx++) lengths[order[idx]] = 0;
      if (s.err || huff_build(lencode, lengths, 19) != 0) return -1;
      idx = 0;
      while (idx < nlen + ndist) {
        int sym = huff_decode(s, lencode);
        if (sym < 0) return -1;
        if (sym < 16) {
          lengths[idx++] = (int16_t)sym;
        } else {
          int len = 0, rep;
          if (sym == 16) {
            if (idx == 0) return -1;
            len = lengths[idx - 1];
            rep = 3 + (int)in_bits(s, 2);
          } else if (sym == 17) {
            rep = 3 + (int)in_bits(s, 3);
          } else {
            rep = 11 + (int)in_bits(s, 7);
          }
          if (s.err || idx + rep > nlen + ndist) return -1;
          while (rep--) lengths[idx++] = (int16_t)len;
        }
      }
      if (lengths[256] == 0) return -1;
      const int e1 = huff_build(lencode, lengths, nlen);
      if (e1 < 0 || (e1 > 0 && nlen - lencode.count[0] != 1)) return -1;
      const int e2 = huff_build(distcode, lengths + nlen, ndist);
      if (e2 < 0 || (e2 > 0 && ndist - distcode.count[0] != 1)) return -1;
      if (inflate_codes(s, out, op, cap, lencode, distcode)) return -1;
    } else {
      return -1;
    }
  } while (!last);
  *consumed = s.pos;
  return op;
}

// zlib stream (RFC 1950): header, deflate data, Adler-32 of the output (big-endian) -- what
// java.util.zip.Inflater (nowrap = false) accepts. Returns the output length or -1.
PHIP_HD inline int inflate_zlib(const uint8_t *in, int n, uint8_t *out, int cap, uint8_t *ws) {
  if (n < 6) return -1;
  const int cmf = in[0], flg = in[1];
  if ((cmf & 15) != 8 || (cmf >> 4) > 7 || ((cmf << 8) | flg) % 31 != 0 || (flg & 0x20)) return -1;
  int used = 0;
  const int got = inflate_raw(in + 2, n - 2, out, cap, ws, &used);
  if (got < 0 || 2 + used + 4 > n) return -1;
  uint32_t a = 1, b = 0;
  for (int i = 0; i < got; i++) {
    a += out[i];
    if (a >= 65521u) a -= 65521u;
    b += a;
    if (b >= 65521u) b -= 65521u;
  }
  const uint8_t *t = in + 2 + used;
  const uint32_t want = ((uint32_t)t[0] << 24) | ((uint32_t)t[1] << 16) | ((uint32_t)t[2] << 8) | t[3];
  return want == ((b << 16) | a) ? got : -1;
}

// Pinot GZIP chunk: zlib stream + 4-byte BE uncompressed length (GzipCompressor.java:42)
PHIP_HD inline int pinot_gzip_chunk(const uint8_t *in, int n, uint8_t *out, int cap, uint8_t *ws) {
  if (n < 10) return -1;
  const uint8_t *t = in + n - 4;
  const int declared = (int)(((uint32_t)t[0] << 24) | ((uint32_t)t[1] << 16) | ((uint32_t)t[2] << 8) | t[3]);
  const int got = inflate_zlib(in, n - 4, out, cap, ws);
  return got == declared ? got : -1;
}


// ------------------------------------------------------------------------------------------------ zstd
PHIP_HD inline int hibit32(uint32_t v) {  // index of the highest set bit (v > 0)
  int r = 0;
  while (v >>= 1) r++;
  return r;
}

// little-endian bit field [off, off + n) of src (n <= 32), bytes past `len` read as 0
PHIP_HD inline uint32_t le_bits(const uint8_t *src, int len, int64_t off, int n) {
  if (n <= 0) return 0;
  uint64_t v = 0;
  const int64_t b0 = off >> 3;
  for (int k = 0; k < 6; k++) {
    const int64_t b = b0 + k;
    if (b >= 0 && b < len) v |= (uint64_t)src[b] << (8 * k);
  }
  v >>= (off & 7);
  return (uint32_t)(v & ((n >= 32) ? 0xffffffffull : ((1ull << n) - 1)));
}

// backward bitstream (RFC 8878 §4.1): read `n` bits below *offset; bits before the stream start read as 0
PHIP_HD inline uint32_t back_bits(const uint8_t *src, int len, int64_t *offset, int n) {
  *offset -= n;
  int64_t off = *offset;
  int bits = n;
  if (off < 0) {
    bits += (int)off;
    off = 0;
  }
  uint32_t r = le_bits(src, len, off, bits);
  if (*offset < 0) r = (-*offset >= 32) ? 0u : (r << (-*offset));
  return r;
}

PHIP_HD inline int back_init(const uint8_t *src, int len, int64_t *offset) {
  if (len <= 0 || src[len - 1] == 0) return -1;
  *offset = (int64_t)len * 8 - (8 - hibit32(src[len - 1]));
  return 0;
}

struct FseTable {
  uint8_t *symbol;
  uint8_t *nbits;
  uint16_t *base;
  int log;
};

// forward LSB-first reader over a header
struct FwdBits {
  const uint8_t *p;
  int len;
  int64_t off;
};

PHIP_HD inline uint32_t fwd_bits(FwdBits &f, int n) {
  uint32_t v = le_bits(f.p, f.len, f.off, n);
  f.off += n;
  return v;
}

// FSE_decode_header (RFC 8878 §4.1.1): normalized counts; returns the header bytes used or -1
PHIP_HD inline int fse_read_ncount(const uint8_t *src, int len, int16_t *freq, int max_symbs, int max_log, int *log,
                                   int *nsymbs) {
  FwdBits f{src, len, 0};
  const int al = 5 + (int)fwd_bits(f, 4);
  if (al > max_log) return -1;
  int32_t remaining = 1 << al;
  int symb = 0;
  while (remaining > 0 && symb < max_symbs) {
    const int bits = hibit32((uint32_t)remaining + 1) + 1;
    uint32_t val = fwd_bits(f, bits);
    const uint32_t lower = (1u << (bits - 1)) - 1;
    const uint32_t thr = (1u << bits) - 1 - ((uint32_t)remaining + 1);
    if ((val & lower) < thr) {
      f.off -= 1;
      val &= lower;
    } else if (val > lower) {
      val -= thr;
    }
    const int proba = (int)val - 1;
    remaining -= proba < 0 ? -proba : proba;
    freq[symb++] = (int16_t)proba;
    if (proba == 0) {
      int rep = (int)fwd_bits(f, 2);
      for (;;) {
        for (int i = 0; i < rep && symb < max_symbs; i++) freq[symb++] = 0;
        if (rep == 3) rep = (int)fwd_bits(f, 2);
        else break;
      }
    }
    if ((f.off + 7) >> 3 > len) return -1;
  }
  if (remaining != 0) return -1;
  *log = al;
  *nsymbs = symb;
  return (int)((f.off + 7) >> 3);
}

// FSE_init_dtable (RFC 8878 §4.1.1): spread symbols, then next-state bases. `next` = scratch [max symbols]
PHIP_HD inline int fse_build(FseTable &t, const int16_t *freq, int nsymbs, int log, uint16_t *next) {
  const int size = 1 << log;
  int high = size;
  for (int s = 0; s < nsymbs; s++)
    if (freq[s] == -1) {
      t.symbol[--high] = (uint8_t)s;
      next[s] = 1;
    }
  int pos = 0;
  const int step = (size >> 1) + (size >> 3) + 3, mask = size - 1;
  for (int s = 0; s < nsymbs; s++) {
    if (freq[s] <= 0) continue;
    next[s] = (uint16_t)freq[s];
    for (int i = 0; i < freq[s]; i++) {
      t.symbol[pos] = (uint8_t)s;
      do {
        pos = (pos + step) & mask;
      } while (pos >= high);
    }
  }
  if (pos != 0) return -1;
  for (int i = 0; i < size; i++) {
    const uint16_t nd = next[t.symbol[i]]++;
    t.nbits[i] = (uint8_t)(log - hibit32(nd));
    t.base[i] = (uint16_t)((nd << t.nbits[i]) - size);
  }
  t.log = log;
  return 0;
}

PHIP_HD inline void fse_rle(FseTable &t, uint8_t sym) {
  t.symbol[0] = sym;
  t.nbits[0] = 0;
  t.base[0] = 0;
  t.log = 0;
}

// workspace layout (bytes)
struct ZstdWs {
  uint8_t huf_sym[2048];
  uint8_t huf_bits[2048];
  uint8_t ll_sym[512], ll_bits[512];
  uint16_t ll_base[512];
  uint8_t of_sym[256], of_bits[256];
  uint16_t of_base[256];
  uint8_t ml_sym[512], ml_bits[512];
  uint16_t ml_base[512];
  uint8_t w_sym[64], w_bits[64];
  uint16_t w_base[64];
  int16_t freq[64];
  uint16_t next[64];
  uint8_t weights[256];
  int32_t huf_max_bits;  // 0 = no Huffman table yet
  int32_t ll_log, of_log, ml_log, have_ll, have_of, have_ml;
};
constexpr int kZstdWs = (int)sizeof(ZstdWs);

// Huffman_Tree_Description (RFC 8878 §4.2.1): returns bytes used or -1
PHIP_HD inline int huf_read_table(const uint8_t *src, int len, ZstdWs &w) {
  if (len < 1) return -1;
  const int hdr = src[0];
  int nw = 0, used;
  if (hdr < 128) {  // FSE-compressed weights (two interleaved states, accuracy <= 6)
    if (1 + hdr > len) return -1;
    int log, ns;
    const int h = fse_read_ncount(src + 1, hdr, w.freq, 64, 6, &log, &ns);
    if (h < 0) return -1;
    FseTable t{w.w_sym, w.w_bits, w.w_base, 0};
    if (fse_build(t, w.freq, ns, log, w.next)) return -1;
    const uint8_t *bs = src + 1 + h;
    const int bl = hdr - h;
    int64_t off;
    if (back_init(bs, bl, &off)) return -1;
    uint32_t s1 = back_bits(bs, bl, &off, log), s2 = back_bits(bs, bl, &off, log);
    for (;;) {
      if (nw >= 255) return -1;
      w.weights[nw++] = t.symbol[s1];
      s1 = t.base[s1] + back_bits(bs, bl, &off, t.nbits[s1]);
      if (off < 0) {
        w.weights[nw++] = t.symbol[s2];
        break;
      }
      if (nw >= 255) return -1;
      w.weights[nw++] = t.symbol[s2];
      s2 = t.base[s2] + back_bits(bs, bl, &off, t.nbits[s2]);
      if (off < 0) {
        if (nw >= 255) return -1;
        w.weights[nw++] = t.symbol[s1];
        break;
      }
    }
    used = 1 + hdr;
  } else {  // direct 4-bit weights
    nw = hdr - 127;
    used = 1 + (nw + 1) / 2;
    if (used > len) return -1;
    for (int i = 0; i < nw; i++) w.weights[i] = (uint8_t)((i & 1) ? (src[1 + i / 2] & 15) : (src[1 + i / 2] >> 4));
  }
  uint32_t sum = 0;
  for (int i = 0; i < nw; i++) {
    if (w.weights[i] > 11) return -1;
    if (w.weights[i]) sum += 1u << (w.weights[i] - 1);
  }
  if (sum == 0) return -1;
  const int maxb = hibit32(sum) + 1;
  if (maxb > 11) return -1;
  const uint32_t left = (1u << maxb) - sum;
  if (left & (left - 1)) return -1;
  if (nw >= 256) return -1;
  w.weights[nw++] = (uint8_t)(hibit32(left) + 1);
  // HUF_init_dtable: longest codes first; each symbol fills 2^(maxb - bits) entries
  int rank_count[13] = {0}, rank_idx[13] = {0};
  for (int i = 0; i < nw; i++) {
    const int b = w.weights[i] ? maxb + 1 - w.weights[i] : 0;
    rank_count[b]++;
  }
  rank_idx[maxb] = 0;
  for (int i = maxb; i >= 1; i--) {
    rank_idx[i - 1] = rank_idx[i] + rank_count[i] * (1 << (maxb - i));
    for (int k = rank_idx[i]; k < rank_idx[i - 1]; k++) w.huf_bits[k] = (uint8_t)i;
  }
  if (rank_idx[0] != (1 << maxb)) return -1;
  for (int i = 0; i < nw; i++) {
    if (!w.weights[i]) continue;
    const int b = maxb + 1 - w.weights[i];
    const int code = rank_idx[b], n = 1 << (maxb - b);
    for (int k = 0; k < n; k++) w.huf_sym[code + k] = (uint8_t)i;
    rank_idx[b] += n;
  }
  w.huf_max_bits = maxb;
  return used;
}

// one Huffman stream (backward): symbols until the offset reaches -max_bits; returns the count or -1
PHIP_HD inline int huf_stream(const uint8_t *src, int len, const ZstdWs &w, uint8_t *out, int cap) {
  int64_t off;
  if (back_init(src, len, &off)) return -1;
  const int mb = w.huf_max_bits;
  uint32_t state = back_bits(src, len, &off, mb);
  int n = 0;
  while (off > -mb) {
    if (n >= cap) return -1;
    out[n++] = w.huf_sym[state];
    const int b = w.huf_bits[state];
    state = ((state << b) + back_bits(src, len, &off, b)) & ((1u << mb) - 1u);
  }
  return off == -mb ? n : -1;
}

// Literals_Section (RFC 8878 §3.1.1.3.1): decoded into lits; returns section bytes used or -1
PHIP_HD inline int zstd_literals(const uint8_t *src, int len, ZstdWs &w, uint8_t *lits, int lits_cap, int *nlits) {
  if (len < 1) return -1;
  const int type = src[0] & 3, sf = (src[0] >> 2) & 3;
  int regen, comp = 0, hsize, streams = 1;
  if (type < 2) {
    if (sf == 0 || sf == 2) {
      regen = src[0] >> 3;
      hsize = 1;
    } else if (sf == 1) {
      if (len < 2) return -1;
      regen = (src[0] >> 4) + (src[1] << 4);
      hsize = 2;
    } else {
      if (len < 3) return -1;
      regen = (src[0] >> 4) + (src[1] << 4) + (src[2] << 12);
      hsize = 3;
    }
    if (regen > lits_cap) return -1;
    if (type == 0) {
      if (hsize + regen > len) return -1;
      for (int i = 0; i < regen; i++) lits[i] = src[hsize + i];
      *nlits = regen;
      return hsize + regen;
    }
    if (hsize + 1 > len) return -1;
    for (int i = 0; i < regen; i++) lits[i] = src[hsize];
    *nlits = regen;
    return hsize + 1;
  }
  if (sf <= 1) {
    if (len < 3) return -1;
    streams = sf == 0 ? 1 : 4;
    regen = (src[0] >> 4) + ((src[1] & 0x3f) << 4);
    comp = (src[1] >> 6) + (src[2] << 2);
    hsize = 3;
  } else if (sf == 2) {
    if (len < 4) return -1;
    streams = 4;
    regen = (src[0] >> 4) + (src[1] << 4) + ((src[2] & 3) << 12);
    comp = (src[2] >> 2) + (src[3] << 6);
    hsize = 4;
  } else {
    if (len < 5) return -1;
    streams = 4;
    regen = (src[0] >> 4) + (src[1] << 4) + ((src[2] & 0x3f) << 12);
    comp = (src[2] >> 6) + (src[3] << 2) + (src[4] << 10);
    hsize = 5;
  }
  if (regen > lits_cap || hsize + comp > len) return -1;
  const uint8_t *p = src + hsize;
  int rest = comp;
  if (type == 2) {
    const int t = huf_read_table(p, rest, w);
    if (t < 0) return -1;
    p += t;
    rest -= t;
  } else if (!w.huf_max_bits) {
    return -1;  // treeless without a previous table
  }
  if (streams == 1) {
    if (huf_stream(p, rest, w, lits, regen) != regen) return -1;
  } else {
    if (rest < 6) return -1;
    const int s1 = p[0] | (p[1] << 8), s2 = p[2] | (p[3] << 8), s3 = p[4] | (p[5] << 8);
    const int s4 = rest - 6 - s1 - s2 - s3;
    if (s4 < 1) return -1;
    const int seg = (regen + 3) / 4;
    const uint8_t *q = p + 6;
    const int sz[4] = {s1, s2, s3, s4};
    int at = 0;
    for (int k = 0; k < 4; k++) {
      const int want = k < 3 ? seg : regen - 3 * seg;
      if (want < 0 || huf_stream(q, sz[k], w, lits + at, want) != want) return -1;
      q += sz[k];
      at += want;
    }
  }
  *nlits = regen;
  return hsize + comp;
}

// sequence code tables (RFC 8878 §3.1.1.3.2.1)
PHIP_HD inline void ll_code(int c, uint32_t *base, int *bits) {
  const uint32_t b[36] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 18, 20, 22, 24, 28, 32, 40,
                          48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
  const int8_t e[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3,
                        4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
  *base = b[c];
  *bits = e[c];
}
PHIP_HD inline void ml_code(int c, uint32_t *base, int *bits) {
  if (c < 32) {
    *base = (uint32_t)c + 3;
    *bits = 0;
    return;
  }
  const uint32_t b[21] = {35, 37, 39, 41, 43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
  const int8_t e[21] = {1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
  *base = b[c - 32];
  *bits = e[c - 32];
}

// one of the three sequence tables: mode 0 predefined, 1 RLE, 2 FSE-compressed, 3 repeat; returns bytes used or -1
PHIP_HD inline int seq_table(const uint8_t *src, int len, int mode, int kind, ZstdWs &w) {
  uint8_t *sym = kind == 0 ? w.ll_sym : (kind == 1 ? w.of_sym : w.ml_sym);
  uint8_t *bits = kind == 0 ? w.ll_bits : (kind == 1 ? w.of_bits : w.ml_bits);
  uint16_t *base = kind == 0 ? w.ll_base : (kind == 1 ? w.of_base : w.ml_base);
  int32_t *logp = kind == 0 ? &w.ll_log : (kind == 1 ? &w.of_log : &w.ml_log);
  int32_t *have = kind == 0 ? &w.have_ll : (kind == 1 ? &w.have_of : &w.have_ml);
  const int max_symbs = kind == 0 ? 36 : (kind == 1 ? 32 : 53);
  const int max_log = kind == 1 ? 8 : 9;
  FseTable t{sym, bits, base, 0};
  int used = 0;
  if (mode == 0) {
    const int16_t ll[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
    const int16_t of[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
    const int16_t ml[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                            1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
    const int16_t *f = kind == 0 ? ll : (kind == 1 ? of : ml);
    const int n = kind == 0 ? 36 : (kind == 1 ? 29 : 53);
    for (int i = 0; i < n; i++) w.freq[i] = f[i];
    if (fse_build(t, w.freq, n, kind == 1 ? 5 : 6, w.next)) return -1;
  } else if (mode == 1) {
    if (len < 1 || src[0] >= max_symbs) return -1;
    fse_rle(t, src[0]);
    used = 1;
  } else if (mode == 2) {
    int log, ns;
    used = fse_read_ncount(src, len, w.freq, max_symbs, max_log, &log, &ns);
    if (used < 0 || fse_build(t, w.freq, ns, log, w.next)) return -1;
  } else {
    if (!*have) return -1;
    return 0;
  }
  *logp = t.log;
  *have = 1;
  return used;
}

// one compressed block (RFC 8878 §3.1.1.3): literals, sequences, execution into out[*op, cap)
PHIP_HD inline int zstd_block(const uint8_t *src, int len, uint8_t *out, int *opp, int cap, uint8_t *lits, int lits_cap,
                              ZstdWs &w, uint32_t *rep) {
  int nlits = 0;
  const int lu = zstd_literals(src, len, w, lits, lits_cap, &nlits);
  if (lu < 0) return -1;
  const uint8_t *p = src + lu;
  int rest = len - lu;
  if (rest < 1) return -1;
  int nseq = p[0], hs = 1;
  if (nseq >= 128) {
    if (nseq < 255) {
      if (rest < 2) return -1;
      nseq = ((nseq - 128) << 8) + p[1];
      hs = 2;
    } else {
      if (rest < 3) return -1;
      nseq = p[1] + (p[2] << 8) + 0x7F00;
      hs = 3;
    }
  }
  p += hs;
  rest -= hs;
  int op = *opp, lp = 0;
  if (nseq > 0) {
    if (rest < 1) return -1;
    const int modes = p[0];
    if (modes & 3) return -1;
    p++;
    rest--;
    const int mk[3] = {(modes >> 6) & 3, (modes >> 4) & 3, (modes >> 2) & 3};
    for (int k = 0; k < 3; k++) {  // order: literal lengths, offsets, match lengths
      const int u = seq_table(p, rest, mk[k], k, w);
      if (u < 0) return -1;
      p += u;
      rest -= u;
    }
    int64_t off;
    if (back_init(p, rest, &off)) return -1;
    uint32_t sl = back_bits(p, rest, &off, w.ll_log), so = back_bits(p, rest, &off, w.of_log),
             sm = back_bits(p, rest, &off, w.ml_log);
    for (int i = 0; i < nseq; i++) {
      const int llc = w.ll_sym[sl], ofc = w.of_sym[so], mlc = w.ml_sym[sm];
      if (llc > 35 || mlc > 52 || ofc > 31) return -1;
      const uint32_t ofv = (1u << ofc) + back_bits(p, rest, &off, ofc);
      uint32_t mlb, llb;
      int mle, lle;
      ml_code(mlc, &mlb, &mle);
      ll_code(llc, &llb, &lle);
      const uint32_t ml = mlb + back_bits(p, rest, &off, mle);
      const uint32_t ll = llb + back_bits(p, rest, &off, lle);
      if (i != nseq - 1) {
        sl = w.ll_base[sl] + back_bits(p, rest, &off, w.ll_bits[sl]);
        sm = w.ml_base[sm] + back_bits(p, rest, &off, w.ml_bits[sm]);
        so = w.of_base[so] + back_bits(p, rest, &off, w.of_bits[so]);
      }
      // repeat offsets (RFC 8878 §3.1.2.5)
      uint32_t offset;
      if (ofv > 3) {
        offset = ofv - 3;
        rep[2] = rep[1];
        rep[1] = rep[0];
        rep[0] = offset;
      } else {
        const uint32_t idx = ofv + (ll == 0 ? 1u : 0u);
        if (idx == 1) {
          offset = rep[0];
        } else if (idx == 2) {
          offset = rep[1];
          rep[1] = rep[0];
          rep[0] = offset;
        } else if (idx == 3) {
          offset = rep[2];
          rep[2] = rep[1];
          rep[1] = rep[0];
          rep[0] = offset;
        } else {
          offset = rep[0] - 1;
          if (offset == 0) return -1;
          rep[2] = rep[1];
          rep[1] = rep[0];
          rep[0] = offset;
        }
      }
      if (ll > (uint32_t)(nlits - lp) || ll > (uint32_t)(cap - op)) return -1;
      for (uint32_t k = 0; k < ll; k++) out[op++] = lits[lp++];
      if (offset > (uint32_t)op || ml > (uint32_t)(cap - op)) return -1;
      for (uint32_t k = 0; k < ml; k++, op++) out[op] = out[op - offset];
    }
    if (off != 0) return -1;
  } else if (rest != 0) {
    return -1;
  }
  if (nlits - lp > cap - op) return -1;
  while (lp < nlits) out[op++] = lits[lp++];
  *opp = op;
  return 0;
}

// one zstd frame (RFC 8878 §3.1) -- zstd-jni Zstd.decompress of Zstd.compress output. Returns the output length or -1.
PHIP_HD inline int zstd_decompress(const uint8_t *in, int n, uint8_t *out, int cap, uint8_t *lits, int lits_cap,
                                   uint8_t *ws) {
  ZstdWs &w = *(ZstdWs *)ws;
  w.huf_max_bits = 0;
  w.have_ll = w.have_of = w.have_ml = 0;
  if (n < 6 || in[0] != 0x28 || in[1] != 0xB5 || in[2] != 0x2F || in[3] != 0xFD) return -1;
  const int fhd = in[4];
  const int fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, checksum = (fhd >> 2) & 1, dict_flag = fhd & 3;
  if (fhd & 8) return -1;           // reserved bit
  if (dict_flag) return -1;         // no dictionaries on this path
  int ip = 5 + (single ? 0 : 1);
  const int fcs_bytes = fcs_flag == 0 ? (single ? 1 : 0) : (fcs_flag == 1 ? 2 : (fcs_flag == 2 ? 4 : 8));
  if (ip + fcs_bytes > n) return -1;
  int64_t fcs = -1;
  if (fcs_bytes) {
    uint64_t v = 0;
    for (int k = 0; k < fcs_bytes; k++) v |= (uint64_t)in[ip + k] << (8 * k);
    fcs = (int64_t)(fcs_bytes == 2 ? v + 256 : v);
  }
  ip += fcs_bytes;
  uint32_t rep[3] = {1, 4, 8};
  int op = 0, last = 0;
  while (!last) {
    if (ip + 3 > n) return -1;
    const uint32_t bh = in[ip] | (in[ip + 1] << 8) | (in[ip + 2] << 16);
    ip += 3;
    last = bh & 1;
    const int type = (bh >> 1) & 3, size = (int)(bh >> 3);
    if (type == 0) {
      if (ip + size > n || size > cap - op) return -1;
      for (int k = 0; k < size; k++) out[op++] = in[ip + k];
      ip += size;
    } else if (type == 1) {
      if (ip + 1 > n || size > cap - op) return -1;
      for (int k = 0; k < size; k++) out[op++] = in[ip];
      ip += 1;
    } else if (type == 2) {
      if (ip + size > n || size > (1 << 17)) return -1;
      if (zstd_block(in + ip, size, out, &op, cap, lits, lits_cap, w, rep)) return -1;
      ip += size;
    } else {
      return -1;
    }
  }
  if (checksum) ip += 4;  // XXH64 low 32 bits: present, not verified
  if (ip != n) return -1;
  if (fcs >= 0 && fcs != op) return -1;
  return op;
}
}  // namespace codec
}  // namespace phip
