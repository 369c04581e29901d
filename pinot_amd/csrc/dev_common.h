// dev_common.h -- device helpers shared by the gfx950 kernels (filter.hip, aggregate.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/pinot_hip.h"
#include "device.h"

namespace phip {

// Query metadata (segments, columns, filter programs) is read through the constant address space so
// that it compiles to scalar loads (lgkmcnt), never counted in vmcnt.
#define PHIP_CAS __attribute__((address_space(4)))
#define PHIP_GLB __attribute__((address_space(1)))
#define PHIP_LDS __attribute__((address_space(3)))
typedef const PHIP_CAS DevSeg cseg_t;
typedef const PHIP_CAS DevNode cnode_t;
typedef const PHIP_CAS DevCol ccol_t;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

// rank of this lane among the set bits of m below it
__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Bits [off, off+bits) of the MSB-first stream held in words (u32, bit 31 first). The two words of the window come
// in ONE dword-aligned global_load_dwordx2 (one L2 request unless it straddles a line; two dword loads were two
// requests per doc on the sparse gathers of the aggregation walks).
typedef uint32_t u32x2_a4 __attribute__((ext_vector_type(2), aligned(4)));
__device__ __forceinline__ uint32_t decode_bits(const uint32_t *words_generic, uint64_t off, uint32_t bits) {
  // streamed once: non-temporal, so the words do not evict the dictionaries the gathers re-read
  const PHIP_GLB u32x2_a4 *p = (const PHIP_GLB u32x2_a4 *)((const PHIP_GLB uint32_t *)words_generic + (off >> 5));
  const u32x2_a4 v = __builtin_nontemporal_load(p);
  const uint64_t win = ((uint64_t)v.x << 32) | (uint64_t)v.y;
  return (uint32_t)((win << (off & 31)) >> (64 - bits));
}

// Window of 32 stream bits starting at bit p of a staged region (u32 words, bit 31 first).
// q = floor((p-1)/32) may be -1 (reads the guard word before the region); s in [0, 31].
__device__ __forceinline__ uint32_t window_at(const PHIP_LDS uint32_t *w, int32_t p) {
  const int32_t q = (p - 1) >> 5;
  const uint32_t s = (uint32_t)(32 * (q + 1) - p);
  return __builtin_amdgcn_alignbit(w[q], w[q + 1], s);
}

// ------------------------------------------------------------------------------------------------
// LDS-DMA staging. The copy is issued through inline asm so that hipcc does not see an LDS write in
// flight: it would otherwise put s_waitcnt vmcnt(0) in front of the first ds_read of the CURRENT
// tile and drain the prefetch of the next ones. Completion is awaited by wait_vmcnt(n).
// ------------------------------------------------------------------------------------------------
#ifndef PHIP_DMA_POLICY
#define PHIP_DMA_POLICY "nt"  // streamed once: non-temporal
#endif
__device__ __forceinline__ void dma16(const uint8_t *gsrc, uint32_t lds_dst) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off " PHIP_DMA_POLICY "\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_dst)
      : "memory");
}

// Order-preserving map double <-> u64 (for atomicMin/atomicMax on group tables).
__device__ __forceinline__ uint64_t f64_ordered(double d) {
  uint64_t u = (uint64_t)__double_as_longlong(d);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
// The two table sentinels -- ~0 (a MIN row's initial value) and 0 (a MAX row's) -- are the images of two NaN bit
// patterns no aggregation produces; a group that no doc of the function's filter program reached keeps them and
// reads back as the holder defaults +inf / -inf (DoubleGroupByResultHolder, FILTER + GROUP BY).
__host__ __device__ inline double f64_unordered(uint64_t u) {
  if (u == ~0ull) return __builtin_huge_val();
  if (u == 0ull) return -__builtin_huge_val();
  u = (u >> 63) ? (u & 0x7fffffffffffffffull) : ~u;
  union {
    uint64_t u;
    double d;
  } x;
  x.u = u;
  return x.d;
}
__device__ __forceinline__ double as_f64(uint64_t u) { return __longlong_as_double((long long)u); }
__device__ __forceinline__ uint64_t as_u64(double d) { return (uint64_t)__double_as_longlong(d); }

__device__ __forceinline__ uint64_t wave_reduce_u64_add(uint64_t v) {
  for (int o = 32; o > 0; o >>= 1) {
    uint32_t lo = __shfl_xor((int)(uint32_t)v, o);
    uint32_t hi = __shfl_xor((int)(uint32_t)(v >> 32), o);
    v += ((uint64_t)hi << 32) | lo;
  }
  return v;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
  return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
  return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ uint32_t wave_or32(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v |= (uint32_t)__shfl_xor((int)v, o);
  return __builtin_amdgcn_readfirstlane(v);
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
  if (kind == ACC_MIN_F64) return as_u64(__builtin_huge_val());
  if (kind == ACC_MAX_F64) return as_u64(-__builtin_huge_val());
  return 0;  // counts, int sums, f64 +0.0
}

__device__ __forceinline__ uint64_t acc_combine(int kind, uint64_t a, uint64_t b) {
  if (kind == ACC_SUM_F64) return as_u64(as_f64(a) + as_f64(b));
  if (kind == ACC_MIN_F64) return as_u64(fmin(as_f64(a), as_f64(b)));
  if (kind == ACC_MAX_F64) return as_u64(fmax(as_f64(a), as_f64(b)));
  return a + b;
}

// s_waitcnt vmcnt(n) for a wave-uniform n (vmcnt takes an immediate; n >= 63 needs no wait: at most
// 63 vector-memory operations can be outstanding, so an op with 63 younger ones has completed).
#define PHIP_VM(k) \
  case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
__device__ __forceinline__ void wait_vmcnt(int n) {
  switch (n) {
    PHIP_VM(0) PHIP_VM(1) PHIP_VM(2) PHIP_VM(3) PHIP_VM(4) PHIP_VM(5) PHIP_VM(6) PHIP_VM(7) PHIP_VM(8)
    PHIP_VM(9) PHIP_VM(10) PHIP_VM(11) PHIP_VM(12) PHIP_VM(13) PHIP_VM(14) PHIP_VM(15) PHIP_VM(16)
    PHIP_VM(17) PHIP_VM(18) PHIP_VM(19) PHIP_VM(20) PHIP_VM(21) PHIP_VM(22) PHIP_VM(23) PHIP_VM(24)
    PHIP_VM(25) PHIP_VM(26) PHIP_VM(27) PHIP_VM(28) PHIP_VM(29) PHIP_VM(30) PHIP_VM(31) PHIP_VM(32)
    PHIP_VM(33) PHIP_VM(34) PHIP_VM(35) PHIP_VM(36) PHIP_VM(37) PHIP_VM(38) PHIP_VM(39) PHIP_VM(40)
    PHIP_VM(41) PHIP_VM(42) PHIP_VM(43) PHIP_VM(44) PHIP_VM(45) PHIP_VM(46) PHIP_VM(47) PHIP_VM(48)
    PHIP_VM(49) PHIP_VM(50) PHIP_VM(51) PHIP_VM(52) PHIP_VM(53) PHIP_VM(54) PHIP_VM(55) PHIP_VM(56)
    PHIP_VM(57) PHIP_VM(58) PHIP_VM(59) PHIP_VM(60) PHIP_VM(61) PHIP_VM(62)
    default: break;
  }
}
#undef PHIP_VM

// Docs of a tile inside its segment, lane-major: bit (31-g) of lane l is doc g*64 + l.
__device__ __forceinline__ uint32_t valid_word(int32_t valid_docs, int lane) {
  const int32_t ngrp = min(kTileGroups, max(0, (valid_docs - lane + 63) >> 6));
  return ngrp == 0 ? 0u : (~0u << (32 - ngrp));
}

// Transpose of the 32x32 bit matrix held by each 32-lane half (row = lane, Hacker's Delight transpose32 as 5
// butterfly stages over ds_bpermute). It is an involution.
__device__ __forceinline__ uint32_t transpose_halves(uint32_t a) {
  const int lane = lane_id();
  uint32_t m = 0x0000FFFFu;
#pragma unroll
  for (int j = 16; j != 0; j >>= 1, m ^= m << j) {
    const uint32_t p = (uint32_t)__builtin_amdgcn_ds_bpermute((lane ^ j) << 2, (int)a);
    if (lane & j) {
      a ^= ((p ^ (a >> j)) & m) << j;
    } else {
      a ^= (a ^ (p >> j)) & m;
    }
  }
  return a;
}

// Lane-major tile word (bit 31-g of lane l = doc 64g + l) -> contiguous word (bit 31-j of lane L = doc 32L + j):
// the inverse of filter.hip contig_to_lane_major (transpose each half, then lane c takes lane 32(c&1) + c/2).
__device__ __forceinline__ uint32_t lane_major_to_contig(uint32_t m) {
  const int lane = lane_id();
  const uint32_t a = transpose_halves(m);
  return (uint32_t)__builtin_amdgcn_ds_bpermute((32 * (lane & 1) + (lane >> 1)) << 2, (int)a);
}

// Inclusive prefix sum over the wave's 64 lanes, in DPP (VALU) steps: row_shr 1/2/4/8 scan each 16-lane row,
// row_bcast:15 / row_bcast:31 carry the row totals (GFX9 DPP; a disabled or out-of-row source reads as 0). Six
// VALU ops instead of six dependent ds_bpermute round trips -- it runs once per tile of the aggregation walks.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15, rows 1, 3
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31, rows 2, 3
  return v;
}

}  // namespace phip
