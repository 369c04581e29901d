// filter.hip -- the filter launch dispatch and the Roaring decode of inverted leaves. The filter kernel itself
// (K1-K4 of SURVEY.md §2.4) is filter_kernel.h, one translation unit per variant (filter_k_*.hip):
//
// Execution model. One wave streams a CONTIGUOUS range of 2048-doc tiles (the global work list is
// segment-ordered, so a wave changes segment at most a few times and its segment / filter-program
// metadata stays in the scalar cache). Every scanned column's bytes for a tile (256*b bytes: a
// 64-doc group is exactly 2b words of the u32 word layout, kernels.hip/runtime.cpp) and every
// inverted leaf's 256 dense-word bytes arrive in the wave's LDS ring by LDS-DMA
// (global_load_lds_dwordx4, 1 KiB per wave-instruction); nbuf-1 tiles are in flight while one is
// evaluated, and completion is awaited with a counted vmcnt (a lower bound of the vector-memory
// operations issued after the tile's DMA, kept in SGPRs together with the stage cursor).
//
// A tile's doc set is lane-major: lane l owns a 32-bit word whose bit (31-g) is doc 64g + l. Scan
// leaves decode with lanes = docs of one 64-doc group at a time (one v_alignbit per doc and group),
// which is SVScanDocIdIterator + PredicateEvaluator.applySV
// (pinot-core/.../operator/dociditerators/SVScanDocIdIterator.java:75-142) without the doc-id
// materialisation; AND / OR / NOT (AndDocIdSet / OrDocIdSet / NotDocIdSet) are one VALU op per lane.
// The tile's 64 lane words (256 B, one coalesced store) go to the aggregation kernel when the query
// projects anything; COUNT-only queries stop here (FastFilteredCountOperator.java:66-78).
#include <hip/hip_ext.h>

#include "agg_common.h"

namespace phip {
// ------------------------------------------------------------------------------------------------
// Roaring containers of the selected dict ids -> OR into dense u64 doc words
// (BitmapInvertedIndexReader.getDocIds + ImmutableRoaringBitmap.or, InvertedIndexFilterOperator.java:79-95)
// ------------------------------------------------------------------------------------------------
// One workgroup per (leaf, key) group, one wave per container: every selected container of that 65536-doc
// range is OR-ed into an LDS bitmap with LDS atomics (array: one bit per value, bitmap: word OR, run: word
// masks), then the 1024 words go to HBM with plain coalesced stores -- no global atomics, each word written
// once. A key with at least kRoaringWaves containers (an IN over many values: mostly small arrays) gives each
// wave its own containers round robin, so that many container loads are in flight instead of one; a key with
// fewer takes them one at a time with the whole workgroup. Every key of a leaf has a group (keys without
// containers store zeros), so the dense words need no clearing pass.
constexpr int kRoaringWaves = 8;
__global__ __launch_bounds__(kRoaringWaves * 64) void roaring_or_kernel(const RoaringTask *__restrict__ tasks,
                                                                        const RoaringGroup *__restrict__ groups,
                                                                        int32_t ngroups) {
  __shared__ uint64_t bm[1024];
  typedef PHIP_LDS uint64_t lds64;
  const int lane = lane_id();
  const int wave = (int)(threadIdx.x >> 6);
  for (int gi = blockIdx.x; gi < ngroups; gi += gridDim.x) {
    const RoaringGroup g = groups[gi];
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) bm[i] = 0;
    __syncthreads();
    const bool per_wave = g.task_end - g.task_begin >= kRoaringWaves;  // uniform over the workgroup
    const int tstep = per_wave ? kRoaringWaves : 1;
    const int lid = per_wave ? lane : (int)threadIdx.x;
    const int lstep = per_wave ? 64 : (int)blockDim.x;
    for (int ti = g.task_begin + (per_wave ? wave : 0); ti < g.task_end; ti += tstep) {
      const RoaringTask tk = tasks[ti];
      if (tk.kind == 0) {
        const uint16_t *v = (const uint16_t *)tk.payload;
        for (int i = lid; i < tk.card; i += lstep) {
          const uint32_t x = v[i];
          __hip_atomic_fetch_or((lds64 *)&bm[x >> 6], 1ull << (x & 63), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      } else if (tk.kind == 1) {
        const uint64_t *w = (const uint64_t *)tk.payload;
        for (int i = lid; i < 1024; i += lstep) {
          const uint64_t x = w[i];
          if (x) __hip_atomic_fetch_or((lds64 *)&bm[i], x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      } else {
        const uint16_t *r = (const uint16_t *)tk.payload;
        for (int ri = 0; ri < tk.card; ri++) {
          const uint32_t s = r[1 + 2 * ri], e = min(s + r[2 + 2 * ri], 65535u);  // inclusive (load validates)
          const uint32_t ws = s >> 6, we = e >> 6;
          for (uint32_t wi = ws + lid; wi <= we; wi += lstep) {
            const int lo = (wi == ws) ? (int)(s & 63) : 0;
            const int hi = (wi == we) ? (int)(e & 63) : 63;
            const uint64_t m = (hi == 63 ? ~0ull : ((1ull << (hi + 1)) - 1)) & ~((1ull << lo) - 1);
            __hip_atomic_fetch_or((lds64 *)&bm[wi], m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          }
        }
      }
    }
    __syncthreads();
    // 65536 docs per container = 1024 words = 32 tiles of 32 words, each tile's at tile * tile_words
    uint64_t *out = g.out_words + (int64_t)g.key * 32 * g.tile_words;
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) out[(i >> 5) * g.tile_words + (i & 31)] = bm[i];
    __syncthreads();
  }
}

// Lane-major tile masks -> doc-order u64 bitmap words of one segment (phip_filter_bitmap):
// word (tile*32 + g) bit l = bit (31-g) of lane l's mask word.
__global__ __launch_bounds__(256) void masks_to_words_kernel(const uint32_t *__restrict__ masks, int32_t tile0,
                                                             int32_t ntiles, uint64_t *__restrict__ words,
                                                             int64_t nwords) {
  const int lane = lane_id();
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t t = wave; t < ntiles; t += nw) {
    const uint32_t m = masks[t * 64 + lane];
    uint64_t mine = 0;
    for (int g = 0; g < kTileGroups; g++) {
      const uint64_t b = ballot((m >> (31 - g)) & 1u);
      if (lane == g) mine = b;
    }
    const int64_t wi = (int64_t)(tile0 + t) * kTileGroups + lane;
    if (lane < kTileGroups && wi < nwords) words[wi] = mine;
  }
}

// ------------------------------------------------------------------------------------------------
// host-callable launchers (runtime.cpp)
// ------------------------------------------------------------------------------------------------
hipError_t launch_roaring_or(const RoaringTask *tasks, const RoaringGroup *groups, int32_t ngroups, hipStream_t s) {
  if (ngroups <= 0) return hipSuccess;
  roaring_or_kernel<<<ngroups < 16384 ? ngroups : 16384, kRoaringWaves * 64, 0, s>>>(tasks, groups, ngroups);
  return hipGetLastError();
}


// the eight filter_kernel instantiations, one translation unit each (filter_k*.hip)
hipError_t launch_filter_general(const DevFilter &, int, size_t, hipStream_t, hipEvent_t, hipEvent_t);
hipError_t launch_filter_conj(const DevFilter &, int, size_t, hipStream_t, hipEvent_t, hipEvent_t);
hipError_t launch_filter_fused1(const DevFilter &, int, size_t, hipStream_t, hipEvent_t, hipEvent_t);
hipError_t launch_filter_fused2(const DevFilter &, int, size_t, hipStream_t, hipEvent_t, hipEvent_t);
hipError_t launch_filter_fused4(const DevFilter &, int, size_t, hipStream_t, hipEvent_t, hipEvent_t);
hipError_t launch_filter_fusedgb(const DevFilter &, int, size_t, hipStream_t, hipEvent_t, hipEvent_t);
hipError_t launch_filter_fusedgbx(const DevFilter &, int, size_t, hipStream_t, hipEvent_t, hipEvent_t);
hipError_t launch_filter_fusedgbl(const DevFilter &, int, size_t, hipStream_t, hipEvent_t, hipEvent_t);

// conj_only: every segment's program takes the conjunctive fast path (the interpreter is compiled
// out, which frees registers for more resident waves); fused_naggs > 0: the aggregation runs inside
// (q.agg set, conj_only required); fused_naggs < 0: the dense group-by runs inside (q.agg set), -1 into the HBM
// table, -2 into its XCD-private copies, -3 into the workgroup's LDS table
// (e0 / e1: optional start / stop events recorded by the kernel's own dispatch, hipExtLaunchKernel)
hipError_t launch_filter(const DevFilter &q, bool conj_only, int fused_naggs, int nblocks, size_t lds_bytes,
                         hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  if (!conj_only) return launch_filter_general(q, nblocks, lds_bytes, s, e0, e1);
  if (fused_naggs == -3) return launch_filter_fusedgbl(q, nblocks, lds_bytes, s, e0, e1);
  if (fused_naggs == -2) return launch_filter_fusedgbx(q, nblocks, lds_bytes, s, e0, e1);
  if (fused_naggs < 0) return launch_filter_fusedgb(q, nblocks, lds_bytes, s, e0, e1);
  if (fused_naggs == 0) return launch_filter_conj(q, nblocks, lds_bytes, s, e0, e1);
  if (fused_naggs <= 1) return launch_filter_fused1(q, nblocks, lds_bytes, s, e0, e1);
  if (fused_naggs <= 2) return launch_filter_fused2(q, nblocks, lds_bytes, s, e0, e1);
  return launch_filter_fused4(q, nblocks, lds_bytes, s, e0, e1);
}

hipError_t launch_masks_to_words(const uint32_t *masks, int32_t tile0, int32_t ntiles, uint64_t *words, int64_t nwords,
                                 hipStream_t s) {
  if (ntiles <= 0) return hipSuccess;
  int blocks = (int)std::min<int64_t>(((int64_t)ntiles + 3) / 4, 4096);
  masks_to_words_kernel<<<blocks, 256, 0, s>>>(masks, tile0, ntiles, words, nwords);
  return hipGetLastError();
}

}  // namespace phip
