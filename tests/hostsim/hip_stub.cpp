// Host-only HIP stand-in used to run libpinot_hip's host runtime (runtime.cpp) under AddressSanitizer
// on a machine without a GPU: device memory is host memory, copies are memcpy, kernels are no-ops
// that zero their outputs. Test tooling only -- catches host-side bugs (descriptor building,
// staging, result assembly); device results are meaningless here.
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <cstring>
#include <cstdint>

extern "C" {
hipError_t hipGetDeviceCount(int *n) {  // HOSTSIM_DEVICES: stand-in devices for the node-plan paths
  const char *e = getenv("HOSTSIM_DEVICES");
  *n = e ? atoi(e) : 1;
  return hipSuccess;
}
hipError_t hipMemcpyPeerAsync(void *d, int, const void *s, int, size_t n, hipStream_t) { memmove(d, s, n); return hipSuccess; }
hipError_t hipGetDevice(int *d) { *d = 0; return hipSuccess; }
hipError_t hipSetDevice(int) { return hipSuccess; }
hipError_t hipDeviceGetAttribute(int *v, hipDeviceAttribute_t, int) { *v = 256; return hipSuccess; }
hipError_t hipStreamCreateWithFlags(hipStream_t *s, unsigned) { *s = (hipStream_t)0x1; return hipSuccess; }
hipError_t hipStreamDestroy(hipStream_t) { return hipSuccess; }
hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
hipError_t hipEventCreate(hipEvent_t *e) { *e = (hipEvent_t)0x1; return hipSuccess; }
hipError_t hipEventDestroy(hipEvent_t) { return hipSuccess; }
hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipSuccess; }
hipError_t hipEventElapsedTime(float *ms, hipEvent_t, hipEvent_t) { *ms = 0.f; return hipSuccess; }
hipError_t hipMalloc(void **p, size_t n) { *p = calloc(1, n ? n : 1); return hipSuccess; }
hipError_t hipFree(void *p) { free(p); return hipSuccess; }
hipError_t hipHostMalloc(void **p, size_t n, unsigned) { *p = calloc(1, n ? n : 1); return hipSuccess; }
hipError_t hipHostFree(void *p) { free(p); return hipSuccess; }
hipError_t hipHostGetDevicePointer(void **d, void *h, unsigned) { *d = h; return hipSuccess; }
hipError_t hipMemcpyAsync(void *d, const void *s, size_t n, hipMemcpyKind, hipStream_t) { memmove(d, s, n); return hipSuccess; }
hipError_t hipMemcpy(void *d, const void *s, size_t n, hipMemcpyKind) { memmove(d, s, n); return hipSuccess; }
hipError_t hipMemsetAsync(void *d, int v, size_t n, hipStream_t) { memset(d, v, n); return hipSuccess; }
hipError_t hipGetLastError(void) { return hipSuccess; }
hipError_t hipRuntimeGetVersion(int *v) { *v = 0; return hipSuccess; }
// graphs: capture is reported unsupported, so the runtime takes its eager path
hipError_t hipStreamBeginCapture(hipStream_t, hipStreamCaptureMode) { return hipErrorNotSupported; }
hipError_t hipStreamEndCapture(hipStream_t, hipGraph_t *g) { *g = nullptr; return hipErrorNotSupported; }
hipError_t hipGraphInstantiate(hipGraphExec_t *, hipGraph_t, hipGraphNode_t *, char *, size_t) { return hipErrorNotSupported; }
hipError_t hipGraphLaunch(hipGraphExec_t, hipStream_t) { return hipErrorNotSupported; }
hipError_t hipGraphDestroy(hipGraph_t) { return hipSuccess; }
hipError_t hipGraphExecDestroy(hipGraphExec_t) { return hipSuccess; }
const char *hipGetErrorString(hipError_t) { return "stub"; }
}

#include "../../pinot_amd/csrc/device.h"
#include "../../pinot_amd/csrc/node.h"
namespace phip {
// node_merge.hip on the host (device memory is host memory here): the merges really run, so a node plan's merged
// table can be checked
hipError_t launch_partial_merge_rows(uint64_t *dst, const uint64_t *src, const int32_t *kinds, int rows, int64_t groups,
                                     hipStream_t) {
  for (int r = 0; r < rows; r++)
    for (int64_t g = 0; g < groups; g++) {
      uint64_t &a = dst[r * groups + g];
      const uint64_t b = src[r * groups + g];
      double x, y;
      switch (kinds[r]) {
        case PHIP_ROW_COUNT:
        case PHIP_ROW_SUM_I64: a = (uint64_t)((int64_t)a + (int64_t)b); break;
        case PHIP_ROW_SUM_F64: memcpy(&x, &a, 8); memcpy(&y, &b, 8); x += y; memcpy(&a, &x, 8); break;
        case PHIP_ROW_MIN: a = a < b ? a : b; break;
        case PHIP_ROW_MAX: a = a > b ? a : b; break;
        default: break;
      }
    }
  return hipSuccess;
}
hipError_t launch_max_u32(uint32_t *dst, const uint32_t *src, int64_t n, hipStream_t) {
  for (int64_t i = 0; i < n; i++) dst[i] = dst[i] > src[i] ? dst[i] : src[i];
  return hipSuccess;
}
hipError_t launch_max_u8(uint8_t *dst, const uint8_t *src, int64_t n, hipStream_t) {
  for (int64_t i = 0; i < n; i++) dst[i] = dst[i] > src[i] ? dst[i] : src[i];
  return hipSuccess;
}
hipError_t launch_i64_row_to_f64(uint64_t *row, int64_t n, hipStream_t) {
  for (int64_t i = 0; i < n; i++) {
    const double d = (double)(int64_t)row[i];
    memcpy(&row[i], &d, 8);
  }
  return hipSuccess;
}
hipError_t launch_hash_merge(uint64_t *dkeys, uint64_t *dtab, uint32_t *dhll, int64_t dg, const uint64_t *skeys,
                             const uint64_t *stab, const uint32_t *shll, int64_t sg, const int32_t *kinds, int rows,
                             int nhll, int log2m, int64_t *map, uint32_t *overflow, hipStream_t) {
  if (dg <= 0 || (dg & (dg - 1)) || sg <= 0) return hipErrorInvalidValue;
  const uint64_t mask = (uint64_t)dg - 1;
  for (int64_t s = 0; s < sg; s++) {
    map[s] = -1;
    if (skeys[s] == kHashEmpty) continue;
    uint64_t i = (skeys[s] * 0x9e3779b97f4a7c15ull) & mask;
    for (uint64_t p = 0; p <= mask; p++, i = (i + 1) & mask) {
      if (dkeys[i] == kHashEmpty) dkeys[i] = skeys[s];
      if (dkeys[i] == skeys[s]) {
        map[s] = (int64_t)i;
        break;
      }
    }
    if (map[s] < 0) {
      *overflow = 1;
      continue;
    }
    for (int r = 0; r < rows; r++) {
      const int32_t k[1] = {kinds[r]};
      launch_partial_merge_rows(dtab + r * dg + map[s], stab + r * sg + s, k, 1, 1, nullptr);
    }
    for (int h = 0; h < nhll; h++)
      launch_max_u32(dhll + ((h * dg + map[s]) << log2m), shll + ((h * sg + s) << log2m), (int64_t)1 << log2m, nullptr);
  }
  return hipSuccess;
}
hipError_t launch_bswap32(uint32_t *, int64_t, hipStream_t) { return hipSuccess; }
hipError_t launch_bswap64(uint64_t *, int64_t, hipStream_t) { return hipSuccess; }
hipError_t launch_trim_order(const double *, const int64_t *, const KeyOrder *, int64_t n, int32_t, int32_t, int32_t, void *scratch,
                             size_t *bytes, const int32_t **order, hipStream_t) {
  if (!scratch) *bytes = (size_t)n * 24 + 256;
  else *order = (const int32_t *)((uint8_t *)scratch + (size_t)n * 16);
  return hipSuccess;
}
hipError_t launch_trim_order_terms(const double *, const int64_t *, const OrderTerms *, int64_t n, int32_t,
                                   const uint8_t *, int64_t, int32_t, void *scratch, size_t *scratch_bytes, const int32_t **order_out, hipStream_t) {
  if (!scratch) {
    *scratch_bytes = (size_t)n * 4 + 64;
    return hipSuccess;
  }
  int32_t *o = (int32_t *)scratch;
  for (int64_t i = 0; i < n; i++) o[i] = (int32_t)i;
  *order_out = o;
  return hipSuccess;
}
hipError_t launch_trim_gather(const int32_t *, int64_t, int32_t, int64_t, const int64_t *, const double *, const int64_t *,
                              const uint8_t *, int64_t *, double *, int64_t *, uint8_t *, hipStream_t) { return hipSuccess; }
hipError_t launch_chunk_decode(int, int, const uint8_t *, const RawChunk *, int32_t, int32_t, int32_t, size_t, uint8_t *, int32_t *, int32_t *, hipStream_t) { return hipSuccess; }
hipError_t launch_chunk_decode_global(int, const uint8_t *, const RawChunk *, int32_t, uint8_t *, int32_t *, int32_t *, uint8_t *,
                                      uint64_t, hipStream_t) { return hipSuccess; }
hipError_t launch_bitslice(const uint32_t *, int32_t, int64_t, uint32_t *, hipStream_t) { return hipSuccess; }
hipError_t launch_materialize(const uint32_t *, int32_t, const void *, int32_t, int64_t, void *, hipStream_t) {
  return hipSuccess;
}
hipError_t launch_varbyte_offsets(const uint8_t *, const uint64_t *, const int32_t *, int32_t, int64_t, uint64_t *, uint64_t *,
                                  void *, size_t *temp_bytes, int32_t *, hipStream_t) { *temp_bytes = 64; return hipSuccess; }
hipError_t launch_varbyte_copy(const uint8_t *, const uint64_t *, const int32_t *, int32_t, int64_t, const uint64_t *, uint8_t *,
                               hipStream_t) { return hipSuccess; }
size_t chunk_decode_extra_lds(int, int32_t) { return 0; }
hipError_t launch_sorted_to_packed(const uint32_t *, int32_t, int32_t *, int64_t, int32_t, uint32_t *, int64_t, hipStream_t) { return hipSuccess; }
hipError_t launch_fill_u64(uint64_t *p, int64_t n, uint64_t v, hipStream_t) { for (int64_t i = 0; i < n; i++) p[i] = v; return hipSuccess; }
hipError_t launch_xcd_init(uint64_t *tab, int64_t words, int64_t, const int32_t *, hipStream_t) {
  memset(tab, 0, (size_t)words * kXcdCopies * 8);
  return hipSuccess;
}
hipError_t launch_materialize_hll16(const uint32_t *, int32_t, const uint32_t *, int64_t, uint16_t *, hipStream_t) {
  return hipSuccess;
}
hipError_t launch_materialize_record(const RecSrcs &, int, int64_t, int, uint32_t *, hipStream_t) { return hipSuccess; }
hipError_t launch_materialize_packed(const uint32_t *, int32_t, const void *, int32_t, int64_t, int64_t, int32_t, int64_t,
                                     uint32_t *, hipStream_t) {
  return hipSuccess;
}
hipError_t launch_raw_images(const void *, int32_t, int64_t, uint64_t *, hipStream_t) { return hipSuccess; }
hipError_t set_str_hash_bits(int) { return hipSuccess; }
hipError_t launch_str_hash_unique(void *temp, size_t *temp_bytes, const uint8_t *, const uint64_t *, int64_t, uint64_t *,
                                  int32_t *, uint64_t *, int32_t *, uint64_t *, int32_t *, int64_t *num_out, hipStream_t) {
  if (!temp) *temp_bytes = 64;
  else *num_out = 0;
  return hipSuccess;
}
hipError_t launch_str_verify(const uint8_t *, const uint64_t *, int64_t, const uint64_t *, const int32_t *, int64_t, int32_t *,
                             hipStream_t) { return hipSuccess; }
hipError_t launch_str_rep_lens(const uint64_t *, const int32_t *, int64_t, uint32_t *, hipStream_t) { return hipSuccess; }
hipError_t launch_str_rep_bytes(const uint8_t *, const uint64_t *, const int32_t *, int64_t, const uint64_t *, uint8_t *,
                                hipStream_t) { return hipSuccess; }
hipError_t launch_raw_str_ids(const uint8_t *, const uint64_t *, int64_t, const uint64_t *, int64_t, const int32_t *, int32_t *,
                              hipStream_t) { return hipSuccess; }
hipError_t launch_sort_unique_u64(void *temp, size_t *temp_bytes, uint64_t *, uint64_t *, uint64_t *, int64_t *num_out,
                                  int64_t, hipStream_t) {
  if (!temp) *temp_bytes = 64;
  else *num_out = 0;
  return hipSuccess;
}
hipError_t launch_tuple_words(const TupleCols &, int64_t, uint64_t *, hipStream_t) { return hipSuccess; }
hipError_t launch_tuple_rank(void *temp, size_t *temp_bytes, const uint64_t *, int32_t, int64_t, int32_t *, uint64_t *, int64_t,
                             int64_t *num_out, hipStream_t) {
  if (!temp) *temp_bytes = 64;
  else *num_out = 0;
  return hipSuccess;
}
hipError_t launch_gather_ids(const int32_t *, const int32_t *, int64_t, int32_t *, hipStream_t) { return hipSuccess; }
hipError_t launch_raw_key_ids(const void *, int32_t, int64_t, const uint64_t *, int64_t, int32_t *, hipStream_t) {
  return hipSuccess;
}
hipError_t launch_xcd_merge(uint64_t *, int64_t, int64_t, const int32_t *, uint32_t *, int64_t, hipStream_t) { return hipSuccess; }
hipError_t launch_roaring_or(const RoaringTask *, const RoaringGroup *, int32_t, hipStream_t) { return hipSuccess; }
hipError_t launch_filter(const DevFilter &q, bool, int fused_naggs, int nblocks, size_t, hipStream_t, hipEvent_t,
                         hipEvent_t) {
  memset(q.partials, 0, (size_t)nblocks * 2 * 8);
  if (fused_naggs > 0) memset(q.agg_partials, 0, (size_t)nblocks * fused_naggs * 8);
  if (q.mask_out) memset(q.mask_out, 0, (size_t)q.total_work * 64 * 4);
  return hipSuccess;
}
hipError_t launch_masks_to_words(const uint32_t *, int32_t, int32_t, uint64_t *, int64_t, hipStream_t) { return hipSuccess; }
hipError_t launch_agg(const DevAggQuery &q, const DevAggQuery *, int nblocks, size_t, hipStream_t, hipEvent_t,
                      hipEvent_t) {
  if (q.mode == GB_NONE) memset(q.partials, 0, (size_t)nblocks * q.num_aggs * 8);
  else if (q.mode == GB_GLOBAL) q.gb_table[0] = 1;  // one non-empty group
  else if (q.mode == GB_HASH) { q.gb_table[0] = 1; q.gb_keys[0] = 0; }  // slot 0 holds key 0
  else {
    memset(q.gb_table, 0, (size_t)nblocks * q.tbl_words * 8);
    q.gb_table[0] = 1;
    if (q.gb_hll) memset(q.gb_hll, 0, (size_t)nblocks * q.hll_words * 4);
  }
  return hipSuccess;
}
hipError_t launch_slab_reduce(const uint64_t *slab, int32_t, int32_t tbl_words, int64_t, const int32_t *, uint64_t *out,
                              const uint32_t *, int32_t hll_words, uint32_t *hout, hipStream_t) {
  memcpy(out, slab, (size_t)tbl_words * 8);
  if (hll_words) memset(hout, 0, (size_t)hll_words * 16);
  return hipSuccess;
}
hipError_t launch_finalize_partials2(const uint64_t *, int, int na, const int32_t *, uint64_t *oa, const uint64_t *, int,
                                     int nb, const int32_t *, uint64_t *ob, hipStream_t) {
  for (int i = 0; i < na; i++) oa[i] = 0;
  for (int i = 0; i < nb; i++) ob[i] = 0;
  return hipSuccess;
}
hipError_t launch_finalize_all(const uint64_t *, int, int na, const int32_t *, const uint64_t *, int, const int32_t *,
                               uint64_t *segm, int nseg, uint32_t *hll, int hll_words, uint64_t *out, hipStream_t,
                               uint32_t *ticket, uint64_t seq) {
  if (ticket) out[kDoneSlot] = seq;  // (published below with the results: the host's poll sees it at once)
  memset(out, 0, 64 * 8);
  memcpy(out + 64, segm, (size_t)nseg * 8);
  memset(segm, 0, (size_t)nseg * 8);
  if (hll_words) {
    memcpy(out + 64 + nseg, hll, (size_t)hll_words * 4);
    memset(hll, 0, (size_t)hll_words * 4);
  }
  (void)na;
  return hipSuccess;
}
hipError_t launch_finalize_partials(const uint64_t *, int, int nslots, const int32_t *, uint64_t *out, hipStream_t) {
  memset(out, 0, nslots * 8); return hipSuccess;
}
hipError_t launch_group_count(const uint64_t *counts, int64_t n, int32_t *cc, int64_t nchunks, int64_t *offs, hipStream_t) {
  int64_t s = 0;
  for (int64_t c = 0; c < nchunks; c++) { offs[c] = s; int32_t k = 0; for (int64_t i = c * 1024; i < n && i < (c + 1) * 1024; i++) k += counts[i] != 0; cc[c] = k; s += k; }
  offs[nchunks] = s; return hipSuccess;
}
hipError_t launch_group_compact(const uint64_t *counts, int64_t n, const int64_t *, int64_t, int64_t *keys, hipStream_t) {
  int64_t o = 0; for (int64_t i = 0; i < n; i++) if (counts[i]) keys[o++] = i; return hipSuccess;
}
hipError_t launch_group_gather(const int64_t *, int64_t ng, int64_t, int32_t naggs, int32_t, const int32_t *, const uint64_t *,
                               const uint32_t *, int32_t nhll, int32_t log2m, double *v, int64_t *l, uint8_t *h, hipStream_t) {
  // a pattern (not zeros), so the host side's unpacking of the compacted outputs is checked (run_host_paths.py)
  for (int64_t i = 0; i < ng * naggs; i++) { v[i] = 0.25 + (double)i; l[i] = 1000 + i; }
  if (nhll) for (int64_t i = 0; i < ng * nhll * (1 << log2m); i++) h[i] = (uint8_t)(i * 3 + 1);
  return hipSuccess;
}
hipError_t launch_group_gather_mapped(const int64_t *keys, const int64_t *d_ng, int64_t ndense, int32_t naggs, int32_t,
                                      const int32_t *, const uint64_t *, int64_t *count, int64_t *ok, double *v,
                                      int64_t *l, const uint32_t *, int32_t nhll, int32_t log2m, uint32_t *hout,
                                      hipStream_t) {
  const int64_t ng = *d_ng < ndense ? *d_ng : ndense;
  *count = ng;
  for (int64_t i = 0; i < ng; i++) ok[i] = keys[i];
  for (int64_t i = 0; i < ng * naggs; i++) { v[i] = 0.25 + (double)i; l[i] = 1000 + i; }  // the gather's pattern
  uint8_t *h = (uint8_t *)hout;
  if (nhll) for (int64_t i = 0; i < ng * nhll * (1 << log2m); i++) h[i] = (uint8_t)(i * 3 + 1);
  return hipSuccess;
}
hipError_t launch_hash_keys(int64_t *slots, int64_t n, const uint64_t *keys, hipStream_t) {
  for (int64_t i = 0; i < n; i++) slots[i] = (int64_t)keys[slots[i]];
  return hipSuccess;
}
hipError_t launch_minmax_i64(const void *, int32_t, int64_t, int64_t *, hipStream_t, const uint64_t *) { return hipSuccess; }
hipError_t launch_limit_prepare(const int64_t *, int64_t, const uint64_t *, const uint32_t *, int32_t, uint64_t *,
                                int32_t *, hipStream_t) { return hipSuccess; }
hipError_t launch_limit_bounds(const uint64_t *, int64_t, int64_t *, int64_t *, hipStream_t) { return hipSuccess; }
hipError_t launch_sort_pairs(void *, size_t *temp_bytes, const uint64_t *, uint64_t *, const void *, void *, bool,
                             int64_t, int, hipStream_t) { *temp_bytes = 256; return hipSuccess; }
hipError_t launch_limit_select(const uint64_t *, const int32_t *, int64_t, const int64_t *, int64_t, const int64_t *,
                               const uint64_t *, int32_t, uint64_t *, int64_t *, hipStream_t) { return hipSuccess; }
hipError_t launch_limit_runs(void *, size_t *scan_bytes, const uint64_t *, int64_t, int32_t *, int32_t *, hipStream_t) {
  *scan_bytes = 256; return hipSuccess;
}
hipError_t launch_limit_reduce(const uint64_t *, const int64_t *, int64_t, const int32_t *, const int32_t *, int64_t,
                               int32_t, int32_t, const int32_t *, const uint64_t *, const uint32_t *, int32_t, int32_t, int64_t *,
                               double *, int64_t *, uint8_t *, hipStream_t) { return hipSuccess; }
hipError_t launch_select_count(const DevSelQuery *, int64_t, int64_t *, hipStream_t) { return hipSuccess; }
hipError_t launch_select_scan(void *, size_t *temp_bytes, const int64_t *, int64_t *, int64_t, hipStream_t) {
  *temp_bytes = 256; return hipSuccess;
}
hipError_t launch_select_bases(const DevSelQuery *q, int64_t *, int64_t *kept, int64_t *total, hipStream_t) {
  for (int e = 0; e < q->num_segs; e++) kept[e] = 0;
  total[0] = total[1] = 0; return hipSuccess;
}
hipError_t launch_select_gather(const DevSelQuery *, int64_t, uint64_t *, int64_t, hipStream_t) { return hipSuccess; }
hipError_t launch_select_str_lens(const uint64_t *, int64_t, const uint64_t *const *, uint32_t *, hipStream_t) { return hipSuccess; }
hipError_t launch_select_str_bytes(const uint64_t *, int64_t, const uint8_t *const *, const uint64_t *const *, const uint64_t *, uint8_t *,
                                   hipStream_t) { return hipSuccess; }
}  // namespace phip
