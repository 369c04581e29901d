// load.hip -- one-time layout transforms at segment load (phip_segment_load, runtime.cpp).
#include <hipcub/hipcub.hpp>

#include "codec.h"
#include "dev_common.h"

namespace phip {

// Big-endian index bytes (PinotDataBuffer BIG_ENDIAN, SingleFileIndexDirectory.java:295-297) -> the
// kernels' word layouts: fixed-bit streams as u32 words read big-endian, dictionaries as LE values.
__global__ void bswap32_kernel(uint32_t *__restrict__ p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = __builtin_bswap32(p[i]);
}
__global__ void bswap64_kernel(uint64_t *__restrict__ p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = __builtin_bswap64(p[i]);
}

// Sorted forward index (BE (start,end) pairs, SortedIndexReaderImpl.java:114-116) -> per-doc dict ids. Doc-parallel:
// each doc binary-searches the last id whose start is <= the doc (the pairs are ascending and cover [0, n); an
// id with no docs has end < start and never wins against the next id that starts at the same doc). The pairs
// (8 B x card) stay in L1/L2. (The first version gave one workgroup per dict id: a 7-value D_YEAR took 7
// workgroups x ~860K docs, 526 us per 6M-row segment.)
__global__ void sorted_ids_kernel(const uint32_t *__restrict__ be_pairs, int32_t card, int64_t n,
                                  int32_t *__restrict__ ids) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int32_t lo = 0, hi = card - 1;  // last id with start <= i
    while (lo < hi) {
      const int32_t mid = (lo + hi + 1) >> 1;
      if ((int64_t)(int32_t)__builtin_bswap32(be_pairs[2 * mid]) <= i) lo = mid; else hi = mid - 1;
    }
    ids[i] = lo;
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
      int64_t vs = d * bits;  // value bits occupy [vs, vs + bits); bit 31 of the word is stream bit b0
      uint64_t v = (uint32_t)ids[d];
      int64_t shift = 32 - (vs - (int64_t)b0) - bits;
      if (shift >= 0) w |= (uint32_t)(v << shift);
      else w |= (uint32_t)(v >> (-shift));
    }
    words[k] = w;
  }
}

static inline int grid_for(int64_t n, int per_block = 256, int cap = 4096) {
  int64_t g = (n + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

hipError_t launch_bswap32(uint32_t *p, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  bswap32_kernel<<<grid_for(n), 256, 0, s>>>(p, n);
  return hipGetLastError();
}
hipError_t launch_bswap64(uint64_t *p, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  bswap64_kernel<<<grid_for(n), 256, 0, s>>>(p, n);
  return hipGetLastError();
}
hipError_t launch_sorted_to_packed(const uint32_t *be_pairs, int32_t card, int32_t *ids_tmp, int64_t n, int32_t bits,
                                   uint32_t *words, int64_t nwords, hipStream_t s) {
  if (card <= 0 || n <= 0) return hipSuccess;
  sorted_ids_kernel<<<grid_for(n, 256, 8192), 256, 0, s>>>(be_pairs, card, n, ids_tmp);
  pack_ids_kernel<<<grid_for(nwords), 256, 0, s>>>(ids_tmp, n, bits, words, nwords);
  return hipGetLastError();
}

// Doc-order values of a dictionary column with a large dictionary: vals[d] = dict[id(d)] (4- or 8-byte entries).
// A projection then reads one coalesced-by-doc value instead of the doc's id bits plus a dependent gather into a
// dictionary that does not stay in L2.
template <typename T>
__global__ void materialize_kernel(const uint32_t *__restrict__ words, int32_t bits, const T *__restrict__ dict,
                                   int64_t n, T *__restrict__ vals) {
  for (int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; d < n; d += (int64_t)gridDim.x * blockDim.x)
    vals[d] = dict[decode_bits(words, (uint64_t)d * (uint32_t)bits, (uint32_t)bits)];
}
// Doc-order DISTINCTCOUNTHLL entries packed to 16 bits for log2m <= 11: (register << 5) | rho (rho <= 33 - log2m < 32)
// from the per-id (register << 8) | rho table -- half the bytes a matched doc's HLL update reads.
__global__ void materialize_hll16_kernel(const uint32_t *__restrict__ words, int32_t bits, const uint32_t *__restrict__ table,
                                         int64_t n, uint16_t *__restrict__ out) {
  for (int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; d < n; d += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t e = table[decode_bits(words, (uint64_t)d * (uint32_t)bits, (uint32_t)bits)];
    out[d] = (uint16_t)(((e >> 8) << 5) | (e & 31u));
  }
}
hipError_t launch_materialize_hll16(const uint32_t *words, int32_t bits, const uint32_t *table, int64_t n, uint16_t *out,
                                    hipStream_t s) {
  if (n <= 0) return hipSuccess;
  materialize_hll16_kernel<<<grid_for(n, 256, 8192), 256, 0, s>>>(words, bits, table, n, out);
  return hipGetLastError();
}
// Doc-order values of an INT / LONG dictionary column bit-packed at the width of its value range: doc d's value - base
// as vbits stream bits at d * vbits (the forward index's own layout, bit 31 of word k = stream bit 32k), read back
// with decode_bits. One thread assembles one output word from the <= 3 docs overlapping it, so nothing is shared.
template <typename T>
__global__ void materialize_packed_kernel(const uint32_t *__restrict__ words, int32_t bits, const T *__restrict__ dict,
                                          int64_t n, int64_t base, int32_t vbits, int64_t nwords,
                                          uint32_t *__restrict__ out) {
  for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords; w += (int64_t)gridDim.x * blockDim.x) {
    const int64_t first = 32 * w;
    const int64_t d0 = first / vbits;
    const int64_t d1 = std::min<int64_t>(n - 1, (first + 31) / vbits);
    uint32_t acc = 0;
    for (int64_t d = d0; d <= d1; d++) {
      const uint64_t v = (uint64_t)((int64_t)dict[decode_bits(words, (uint64_t)d * (uint32_t)bits, (uint32_t)bits)] - base);
      const int64_t sh = 32 - (d * vbits - first) - vbits;  // in [1 - vbits, 31]
      acc |= sh >= 0 ? (uint32_t)(v << sh) : (uint32_t)(v >> -sh);
    }
    out[w] = acc;
  }
}
hipError_t launch_materialize_packed(const uint32_t *words, int32_t bits, const void *dict, int32_t width, int64_t n,
                                     int64_t base, int32_t vbits, int64_t nwords, uint32_t *out, hipStream_t s) {
  if (nwords <= 0) return hipSuccess;
  if (width == 4)
    materialize_packed_kernel<int32_t><<<grid_for(nwords, 256, 8192), 256, 0, s>>>(words, bits, (const int32_t *)dict,
                                                                                    n, base, vbits, nwords, out);
  else
    materialize_packed_kernel<int64_t><<<grid_for(nwords, 256, 8192), 256, 0, s>>>(words, bits, (const int64_t *)dict,
                                                                                    n, base, vbits, nwords, out);
  return hipGetLastError();
}
hipError_t launch_materialize(const uint32_t *words, int32_t bits, const void *dict, int32_t width, int64_t n,
                              void *vals, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (width == 4)
    materialize_kernel<uint32_t><<<grid_for(n, 256, 8192), 256, 0, s>>>(words, bits, (const uint32_t *)dict, n,
                                                                         (uint32_t *)vals);
  else
    materialize_kernel<uint64_t><<<grid_for(n, 256, 8192), 256, 0, s>>>(words, bits, (const uint64_t *)dict, n,
                                                                         (uint64_t *)vals);
  return hipGetLastError();
}

// Group-by records (DevSeg.rec): doc d's fields packed LSB first into W u32 (one thread per doc, no word shared).
__device__ __forceinline__ void rec_or(uint32_t (&r)[4], int i, uint32_t x) {
  switch (i) {  // (uniform: a field's offset is the same for every doc)
    case 0: r[0] |= x; break;
    case 1: r[1] |= x; break;
    case 2: r[2] |= x; break;
    default: r[3] |= x; break;
  }
}
__global__ void materialize_record_kernel(RecSrcs fs, int nf, int64_t n, int W, uint32_t *__restrict__ out) {
  for (int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; d < n; d += (int64_t)gridDim.x * blockDim.x) {
    uint32_t r[4] = {0u, 0u, 0u, 0u};
    for (int f = 0; f < nf; f++) {
      const RecSrc &src = fs.f[f];
      uint32_t v;
      if (src.kind == REC_BITS) v = decode_bits((const uint32_t *)src.p, (uint64_t)d * (uint32_t)src.bits, (uint32_t)src.bits);
      else if (src.kind == REC_U16) v = ((const uint16_t *)src.p)[d];
      else v = ((const uint32_t *)src.p)[d];
      if (src.bits < 32) v &= (1u << src.bits) - 1u;
      const int i = src.off >> 5, sh = src.off & 31;
      rec_or(r, i, v << sh);
      if (sh + src.bits > 32) rec_or(r, i + 1, v >> (32 - sh));
    }
    for (int i = 0; i < W; i++) out[d * W + i] = r[i];
  }
}
hipError_t launch_materialize_record(const RecSrcs &fs, int nf, int64_t n, int W, uint32_t *out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  materialize_record_kernel<<<grid_for(n, 256, 8192), 256, 0, s>>>(fs, nf, n, W, out);
  return hipGetLastError();
}

// Value range of a raw INT / LONG column (LE, resident), for the plan-time int64 overflow bound of
// integer SUMs (SumAggregationFunction adds in double and never wraps, :76-101). out = {min, max},
// preset to {INT64_MAX, INT64_MIN} by the caller.
// (nulls: the null doc words -- those docs are skipped: the range of the non-null values -- or null)
__global__ void minmax_i64_kernel(const void *__restrict__ raw, int32_t type, int64_t n, int64_t *__restrict__ out,
                                  const uint64_t *__restrict__ nulls) {
  int64_t lo = INT64_MAX, hi = INT64_MIN;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (nulls != nullptr && ((nulls[i >> 6] >> (i & 63)) & 1ull)) continue;
    const int64_t v = type == PHIP_TYPE_LONG ? ((const int64_t *)raw)[i] : (int64_t)((const int32_t *)raw)[i];
    lo = v < lo ? v : lo;
    hi = v > hi ? v : hi;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t a = __shfl_xor(lo, o), b = __shfl_xor(hi, o);
    lo = a < lo ? a : lo;
    hi = b > hi ? b : hi;
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMin((long long *)&out[0], (long long)lo);
    atomicMax((long long *)&out[1], (long long)hi);
  }
}

hipError_t launch_minmax_i64(const void *raw, int32_t type, int64_t n, int64_t *out, hipStream_t s, const uint64_t *nulls) {
  if (n <= 0) return hipSuccess;
  minmax_i64_kernel<<<grid_for(n, 256, 1024), 256, 0, s>>>(raw, type, n, out, nulls);
  return hipGetLastError();
}

}  // namespace phip

namespace phip {

// ---- compressed raw chunks (ChunkCompressionType SNAPPY=1, LZ4=3, LZ4_LENGTH_PREFIXED=4) ----------------
// Decoded ONCE at pin time into the resident raw layout (HBM holds the decoded values; every query then
// reads them like a PASS_THROUGH column). One single-wave workgroup per chunk: the compressed bytes are
// staged into LDS with dword loads, the sequence stream is parsed wave-uniformly (bytes broadcast from
// LDS, readfirstlane keeps the parse state in SGPRs), literal and match bytes are copied by the 64 lanes
// in parallel into an LDS output buffer, and the chunk is stored with the BE->LE swap fused into
// coalesced 4/8-byte stores. An LZ4 / snappy match copy with offset < length repeats a period of `off`
// bytes, so byte j of the copy reads out[op - off + j % off]: every source byte is already written,
// and the copy needs no rounds. Malformed input (bad offsets, overruns, a decoded length other than
// docs x entry) sets *err = chunk + 1 and that chunk is not stored; the host fails the load.
// Formats: lz4 block format (lz4-java LZ4SafeDecompressor, LZ4Decompressor.java), lz4-java
// LZ4DecompressorWithLength (4-byte LE length + block, LZ4WithLengthDecompressor.java), snappy raw
// format (snappy-java Snappy.uncompress, SnappyDecompressor.java).
__device__ __forceinline__ uint32_t lds_byte(const uint8_t *p, int i) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)p[i]);
}

template <int kCodec>
__device__ __forceinline__ int decode_chunk(const uint8_t *__restrict__ in, int n, uint8_t *__restrict__ out, int cap,
                                            int lane) {
  int ip = 0, op = 0;
  if (kCodec == 1) {  // snappy: varint32 uncompressed length, then tagged elements
    uint32_t ulen = 0;
    for (int shift = 0;; shift += 7) {
      if (ip >= n || shift > 28) return -1;
      uint32_t b = lds_byte(in, ip++);
      ulen |= (b & 0x7fu) << shift;
      if (!(b & 0x80u)) break;
    }
    if (ulen > (uint32_t)cap) return -1;  // (fixed-width chunks: the kernel then checks ulen = docs x entry)
    cap = (int)ulen;
    while (ip < n) {
      uint32_t tag = lds_byte(in, ip++);
      uint32_t len, off;
      if ((tag & 3u) == 0) {
        len = (tag >> 2) + 1;
        if (len > 60) {
          int nb = (int)len - 60;
          if (ip + nb > n) return -1;
          len = 0;
          for (int k = 0; k < nb; k++) len |= lds_byte(in, ip + k) << (8 * k);
          len += 1;
          ip += nb;
          if (len == 0) return -1;  // 2^32 wrapped
        }
        if (len > (uint32_t)(n - ip) || len > (uint32_t)(cap - op)) return -1;
        for (int i = lane; i < (int)len; i += 64) out[op + i] = in[ip + i];
        ip += (int)len;
        op += (int)len;
        continue;
      }
      if ((tag & 3u) == 1) {
        if (ip + 1 > n) return -1;
        len = 4 + ((tag >> 2) & 7u);
        off = ((tag >> 5) << 8) | lds_byte(in, ip);
        ip += 1;
      } else if ((tag & 3u) == 2) {
        if (ip + 2 > n) return -1;
        len = (tag >> 2) + 1;
        off = lds_byte(in, ip) | (lds_byte(in, ip + 1) << 8);
        ip += 2;
      } else {
        if (ip + 4 > n) return -1;
        len = (tag >> 2) + 1;
        off = lds_byte(in, ip) | (lds_byte(in, ip + 1) << 8) | (lds_byte(in, ip + 2) << 16) | (lds_byte(in, ip + 3) << 24);
        ip += 4;
      }
      if (off == 0 || off > (uint32_t)op || len > (uint32_t)(cap - op)) return -1;
      __syncthreads();  // earlier literal/match bytes from every lane are visible
      for (int i = lane; i < (int)len; i += 64) {
        int j = off >= len ? i : (int)((uint32_t)i % off);
        out[op + i] = out[op - (int)off + j];
      }
      op += (int)len;
    }
    return op == cap ? op : -1;
  }
  // LZ4 block format
  while (ip < n) {
    uint32_t tok = lds_byte(in, ip++);
    int lit = (int)(tok >> 4);
    if (lit == 15) {
      uint32_t b;
      do {
        if (ip >= n) return -1;
        b = lds_byte(in, ip++);
        lit += (int)b;
      } while (b == 255 && lit < (1 << 30));
    }
    if (lit > n - ip || lit > cap - op) return -1;
    for (int i = lane; i < lit; i += 64) out[op + i] = in[ip + i];
    ip += lit;
    op += lit;
    if (ip == n) break;  // last sequence: literals only
    if (ip + 2 > n) return -1;
    int off = (int)(lds_byte(in, ip) | (lds_byte(in, ip + 1) << 8));
    ip += 2;
    if (off == 0 || off > op) return -1;
    int ml = (int)(tok & 15u);
    if (ml == 15) {
      uint32_t b;
      do {
        if (ip >= n) return -1;
        b = lds_byte(in, ip++);
        ml += (int)b;
      } while (b == 255 && ml < (1 << 30));
    }
    ml += 4;
    if (ml > cap - op) return -1;
    __syncthreads();
    for (int i = lane; i < ml; i += 64) {
      int j = off >= ml ? i : (int)((uint32_t)i % (uint32_t)off);
      out[op + i] = out[op - off + j];
    }
    op += ml;
  }
  return op;
}

// Entropy-coded chunks (ZSTANDARD = 2, GZIP = 5; codec.h): the serial decode runs on lane 0 over the LDS copy of
// the chunk into the LDS output (workspace and the zstd literal buffer in LDS too); the wave then stores the
// chunk with the same fused BE->LE swap.
template <int kCodec>
__device__ __forceinline__ int decode_entropy(const uint8_t *in, int n, uint8_t *out, int usize, uint8_t *ws,
                                              uint8_t *lits, int lane) {
  __shared__ int32_t got_s;
  if (lane == 0) {
    got_s = kCodec == 5 ? codec::pinot_gzip_chunk(in, n, out, usize, ws)
                        : codec::zstd_decompress(in, n, out, usize, lits, usize, ws);
  }
  __syncthreads();
  return got_s;
}

template <int kCodec, int kEntry>
__global__ __launch_bounds__(64) void chunk_decode_kernel(const uint8_t *__restrict__ blob,
                                                          const RawChunk *__restrict__ chunks, int32_t nchunks,
                                                          int32_t out_cap, int32_t in_cap, uint8_t *__restrict__ out,
                                                          int32_t *__restrict__ err, int32_t *__restrict__ sizes) {
  extern __shared__ __align__(16) uint8_t lds[];
  uint8_t *lout = lds;
  uint8_t *lin = lds + out_cap;
  uint8_t *lws = lin + in_cap;                                            // codec workspace (GZIP / ZSTANDARD)
  uint8_t *llits = lws + (kCodec == 2 ? ((codec::kZstdWs + 15) & ~15) : 0);  // zstd literals (out_cap bytes)
  const int lane = threadIdx.x;
  for (int32_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const uint64_t src = chunks[c].src, dst = chunks[c].dst;
    const int csize = (int)chunks[c].csize, usize = (int)chunks[c].usize;
    const int head = (int)(src & 3u);
    const uint32_t *sw = (const uint32_t *)(blob + (src - head));
    const int nw = (head + csize + 3) >> 2;
    for (int i = lane; i < nw; i += 64) ((uint32_t *)lin)[i] = sw[i];
    __syncthreads();
    const uint8_t *in = lin + head;
    int n = csize, got;
    if (kCodec == 2 || kCodec == 5) {
      got = decode_entropy<kCodec>(in, n, lout, usize, lws, llits, lane);
    } else if (kCodec == 4) {
      int want = n < 4 ? -2 : (int)(lds_byte(in, 0) | (lds_byte(in, 1) << 8) | (lds_byte(in, 2) << 16) | (lds_byte(in, 3) << 24));
      got = n < 4 ? -1 : decode_chunk<3>(in + 4, n - 4, lout, usize, lane);
      if (got != want) got = -1;
    } else {
      got = decode_chunk<kCodec>(in, n, lout, usize, lane);
    }
    __syncthreads();
    if (kEntry == 1) {
      // var-byte chunk (VarByteChunkForwardIndexWriter): its decoded size is the chunk's own, usize the bound
      if (got < 0 || got > usize) {
        if (lane == 0) atomicMax(err, c + 1);
      } else {
        if (lane == 0) sizes[c] = got;
        uint32_t *o = (uint32_t *)(out + dst);
        const uint32_t *w = (const uint32_t *)lout;
        for (int i = lane; i < (got + 3) / 4; i += 64) o[i] = w[i];  // bytes as stored (no swap)
      }
    } else if (got != usize) {
      if (lane == 0) atomicMax(err, c + 1);
    } else if (kEntry == 8) {
      uint64_t *o = (uint64_t *)(out + dst);
      const uint32_t *w = (const uint32_t *)lout;
      for (int i = lane; i < usize / 8; i += 64)
        o[i] = ((uint64_t)__builtin_bswap32(w[2 * i]) << 32) | __builtin_bswap32(w[2 * i + 1]);
    } else {
      uint32_t *o = (uint32_t *)(out + dst);
      const uint32_t *w = (const uint32_t *)lout;
      for (int i = lane; i < usize / 4; i += 64) o[i] = __builtin_bswap32(w[i]);
    }
    __syncthreads();  // LDS reused by the next chunk
  }
}

// Var-byte chunks larger than the LDS window (Pinot's derived 1 MiB chunks, long strings): the same decoders with
// the compressed bytes read from and the output written to HBM -- one single-wave workgroup per chunk, the sequence
// parse wave-uniform, literal / match copies by the 64 lanes with a workgroup barrier between dependent copies
// (a single-wave workgroup stays on one CU, whose L1 the barrier's fences keep coherent for it); the entropy codecs
// run on lane 0 with their workspace in LDS and the zstd literal buffer in HBM scratch.
template <int kCodec>
__global__ __launch_bounds__(64) void chunk_decode_global_kernel(const uint8_t *__restrict__ blob,
                                                                 const RawChunk *__restrict__ chunks, int32_t nchunks,
                                                                 uint8_t *__restrict__ out, int32_t *__restrict__ err,
                                                                 int32_t *__restrict__ sizes, uint8_t *__restrict__ lits,
                                                                 uint64_t lits_stride) {
  __shared__ __align__(16) uint8_t ws[kCodec == 2 ? ((codec::kZstdWs + 15) & ~15) : (kCodec == 5 ? ((codec::kInflateWs + 15) & ~15) : 16)];
  __shared__ int32_t got_s;
  const int lane = threadIdx.x;
  for (int32_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const uint8_t *in = blob + chunks[c].src;
    uint8_t *o = out + chunks[c].dst;
    const int n = (int)chunks[c].csize, cap = (int)chunks[c].usize;
    int got;
    if (kCodec == 2 || kCodec == 5) {
      if (lane == 0)
        got_s = kCodec == 5 ? codec::pinot_gzip_chunk(in, n, o, cap, ws)
                            : codec::zstd_decompress(in, n, o, cap, lits + (uint64_t)c * lits_stride, cap, ws);
      __syncthreads();
      got = got_s;
    } else if (kCodec == 4) {
      const int want = n < 4 ? -2 : (int)(lds_byte(in, 0) | (lds_byte(in, 1) << 8) | (lds_byte(in, 2) << 16) | (lds_byte(in, 3) << 24));
      got = n < 4 ? -1 : decode_chunk<3>(in + 4, n - 4, o, cap, lane);
      if (got != want) got = -1;
    } else {
      got = decode_chunk<kCodec>(in, n, o, cap, lane);
    }
    if (lane == 0) {
      if (got < 0 || got > cap) atomicMax(err, c + 1);
      else sizes[c] = got;
    }
    __syncthreads();
  }
}

template <int kCodec>
static hipError_t launch_chunk_decode_codec(int entry, const uint8_t *blob, const RawChunk *chunks, int32_t nchunks,
                                            int32_t out_cap, int32_t in_cap, size_t lds, uint8_t *out, int32_t *err,
                                            int32_t *sizes, hipStream_t s) {
  const int grid = nchunks < (1 << 20) ? nchunks : (1 << 20);
  const void *fn = entry == 8 ? (const void *)chunk_decode_kernel<kCodec, 8>
                 : entry == 4 ? (const void *)chunk_decode_kernel<kCodec, 4>
                              : (const void *)chunk_decode_kernel<kCodec, 1>;
  if (lds > 65536) {  // allow > 64 KiB dynamic LDS (gfx950: 160 KiB per workgroup)
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 163840 - 1024);
    if (e != hipSuccess) return e;
  }
  if (entry == 8)
    chunk_decode_kernel<kCodec, 8><<<grid, 64, lds, s>>>(blob, chunks, nchunks, out_cap, in_cap, out, err, sizes);
  else if (entry == 4)
    chunk_decode_kernel<kCodec, 4><<<grid, 64, lds, s>>>(blob, chunks, nchunks, out_cap, in_cap, out, err, sizes);
  else
    chunk_decode_kernel<kCodec, 1><<<grid, 64, lds, s>>>(blob, chunks, nchunks, out_cap, in_cap, out, err, sizes);
  return hipGetLastError();
}

// LDS bytes of the codec's workspace beyond the output and input windows
size_t chunk_decode_extra_lds(int codec, int32_t out_cap) {
  if (codec == 5) return (size_t)((codec::kInflateWs + 15) & ~15);
  if (codec == 2) return (size_t)((codec::kZstdWs + 15) & ~15) + (size_t)out_cap;
  return 0;
}

hipError_t launch_chunk_decode(int codec, int entry, const uint8_t *blob, const RawChunk *chunks, int32_t nchunks,
                               int32_t out_cap, int32_t in_cap, size_t lds, uint8_t *out, int32_t *err, int32_t *sizes,
                               hipStream_t s) {
  if (nchunks <= 0) return hipSuccess;
  if (entry != 1 && entry != 4 && entry != 8) return hipErrorInvalidValue;
  switch (codec) {
    case 1: return launch_chunk_decode_codec<1>(entry, blob, chunks, nchunks, out_cap, in_cap, lds, out, err, sizes, s);
    case 2: return launch_chunk_decode_codec<2>(entry, blob, chunks, nchunks, out_cap, in_cap, lds, out, err, sizes, s);
    case 3: return launch_chunk_decode_codec<3>(entry, blob, chunks, nchunks, out_cap, in_cap, lds, out, err, sizes, s);
    case 4: return launch_chunk_decode_codec<4>(entry, blob, chunks, nchunks, out_cap, in_cap, lds, out, err, sizes, s);
    case 5: return launch_chunk_decode_codec<5>(entry, blob, chunks, nchunks, out_cap, in_cap, lds, out, err, sizes, s);
    default: return hipErrorInvalidValue;
  }
}

// ------------------------------------------------------------------------------------------------
// Bit-sliced copy of a fixed-bit forward index (the BitWeaving/V layout) for the range leaves of the conjunctive
// filter: per 2048-doc tile, plane k (k = 0: the id's most significant bit) is 64 lane words with bit 31-g of lane
// l = that bit of doc 64g + l -- the tile-mask layout, so a range test over a lane's 32 docs costs a few bitwise
// operations per plane instead of three per doc. One wave per tile; padded docs decode from the guard words.
// ------------------------------------------------------------------------------------------------
template <int B>
__global__ __launch_bounds__(256) void bitslice_kernel(const uint32_t *__restrict__ words, int64_t ntiles,
                                                       uint32_t *__restrict__ planes) {
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= ntiles) return;
  uint32_t pl[B];
#pragma unroll
  for (int k = 0; k < B; k++) pl[k] = 0;
  for (int g = 0; g < 32; g++) {
    const uint64_t doc = (uint64_t)t * 2048 + 64 * g + lane;
    const uint32_t id = decode_bits(words, doc * B, B);
#pragma unroll
    for (int k = 0; k < B; k++) pl[k] |= ((id >> (B - 1 - k)) & 1u) << (31 - g);
  }
#pragma unroll
  for (int k = 0; k < B; k++) planes[((size_t)t * B + k) * 64 + lane] = pl[k];
}

hipError_t launch_bitslice(const uint32_t *words, int32_t bits, int64_t ntiles, uint32_t *planes, hipStream_t s) {
  if (ntiles <= 0) return hipSuccess;
  const unsigned grid = (unsigned)((ntiles + 3) / 4);
  switch (bits) {
#define PHIP_BSL(b) \
  case b: bitslice_kernel<b><<<grid, 256, 0, s>>>(words, ntiles, planes); break;
    PHIP_BSL(1) PHIP_BSL(2) PHIP_BSL(3) PHIP_BSL(4) PHIP_BSL(5) PHIP_BSL(6) PHIP_BSL(7) PHIP_BSL(8) PHIP_BSL(9)
    PHIP_BSL(10) PHIP_BSL(11) PHIP_BSL(12)
#undef PHIP_BSL
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Raw STRING columns: var-byte chunks (VarByteChunkForwardIndexWriter.java:37-158 -- per chunk numDocsPerChunk BE
// int start offsets, then the values' UTF-8 bytes) -> one contiguous byte array + u64 doc offsets, so a predicate
// reads doc d as bytes [off[d], off[d+1]). chunk_base / chunk_size locate each chunk in `stage` (the forward
// index's own bytes for PASS_THROUGH, the decoded chunks otherwise).
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t be32_bytes(const uint8_t *p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}

// [start, end) of doc d inside its chunk (VarByteChunkSVForwardIndexReader.getValueEndOffset, :176-217): the next
// row's start, or the chunk's end for its last row and for the last row of a partial chunk (absent rows hold 0)
__device__ __forceinline__ bool varbyte_span(const uint8_t *stage, const uint64_t *chunk_base, const int32_t *chunk_size,
                                             int32_t per_chunk, int64_t d, uint64_t &src, uint32_t &len) {
  const int64_t k = d / per_chunk;
  const int32_t r = (int32_t)(d - k * per_chunk);
  const uint8_t *c = stage + chunk_base[k];
  const uint32_t size = (uint32_t)chunk_size[k];
  const uint32_t start = be32_bytes(c + 4 * r);
  uint32_t end = r + 1 < per_chunk ? be32_bytes(c + 4 * (r + 1)) : 0u;
  if (end == 0) end = size;
  const uint32_t hdr = 4u * (uint32_t)per_chunk;
  if ((uint64_t)hdr > size || start < hdr || end < start || end > size) return false;
  src = chunk_base[k] + start;
  len = end - start;
  return true;
}

__global__ void varbyte_lengths_kernel(const uint8_t *__restrict__ stage, const uint64_t *__restrict__ chunk_base,
                                       const int32_t *__restrict__ chunk_size, int32_t per_chunk, int64_t n,
                                       uint64_t *__restrict__ len, int32_t *__restrict__ err) {
  const int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (d > n) return;
  if (d == n) {
    len[n] = 0;  // (the exclusive scan's total)
    return;
  }
  uint64_t src;
  uint32_t l;
  if (!varbyte_span(stage, chunk_base, chunk_size, per_chunk, d, src, l)) {
    atomicMax(err, 1);
    l = 0;
  }
  len[d] = l;
}

__global__ void varbyte_copy_kernel(const uint8_t *__restrict__ stage, const uint64_t *__restrict__ chunk_base,
                                    const int32_t *__restrict__ chunk_size, int32_t per_chunk, int64_t n,
                                    const uint64_t *__restrict__ off, uint8_t *__restrict__ out) {
  const int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= n) return;
  uint64_t src;
  uint32_t l;
  if (!varbyte_span(stage, chunk_base, chunk_size, per_chunk, d, src, l)) return;  // (the lengths pass failed the load)
  const uint64_t o = off[d];
  for (uint32_t i = 0; i < l; i++) out[o + i] = stage[src + i];
}

hipError_t launch_chunk_decode_global(int codec, const uint8_t *blob, const RawChunk *chunks, int32_t nchunks, uint8_t *out,
                                      int32_t *err, int32_t *sizes, uint8_t *lits, uint64_t lits_stride, hipStream_t s) {
  if (nchunks <= 0) return hipSuccess;
  const int grid = nchunks < (1 << 20) ? nchunks : (1 << 20);
  switch (codec) {
    case 1: chunk_decode_global_kernel<1><<<grid, 64, 0, s>>>(blob, chunks, nchunks, out, err, sizes, lits, lits_stride); break;
    case 2: chunk_decode_global_kernel<2><<<grid, 64, 0, s>>>(blob, chunks, nchunks, out, err, sizes, lits, lits_stride); break;
    case 3: chunk_decode_global_kernel<3><<<grid, 64, 0, s>>>(blob, chunks, nchunks, out, err, sizes, lits, lits_stride); break;
    case 4: chunk_decode_global_kernel<4><<<grid, 64, 0, s>>>(blob, chunks, nchunks, out, err, sizes, lits, lits_stride); break;
    case 5: chunk_decode_global_kernel<5><<<grid, 64, 0, s>>>(blob, chunks, nchunks, out, err, sizes, lits, lits_stride); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// lengths of docs 0..n-1 (len[n] = 0) and their exclusive scan into off[0..n]; temp == null: scan size query only
hipError_t launch_varbyte_offsets(const uint8_t *stage, const uint64_t *chunk_base, const int32_t *chunk_size,
                                  int32_t per_chunk, int64_t n, uint64_t *len, uint64_t *off, void *temp,
                                  size_t *temp_bytes, int32_t *err, hipStream_t s) {
  if (temp == nullptr) return hipcub::DeviceScan::ExclusiveSum(nullptr, *temp_bytes, len, off, n + 1, s);
  const int threads = 256;
  const int64_t blocks = (n + 1 + threads - 1) / threads;
  varbyte_lengths_kernel<<<(unsigned)blocks, threads, 0, s>>>(stage, chunk_base, chunk_size, per_chunk, n, len, err);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return hipcub::DeviceScan::ExclusiveSum(temp, *temp_bytes, len, off, n + 1, s);
}

hipError_t launch_varbyte_copy(const uint8_t *stage, const uint64_t *chunk_base, const int32_t *chunk_size,
                               int32_t per_chunk, int64_t n, const uint64_t *off, uint8_t *out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int threads = 256;
  varbyte_copy_kernel<<<(unsigned)((n + threads - 1) / threads), threads, 0, s>>>(stage, chunk_base, chunk_size,
                                                                                   per_chunk, n, off, out);
  return hipGetLastError();
}

}  // namespace phip
