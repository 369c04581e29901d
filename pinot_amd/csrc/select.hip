// select.hip -- selection (row-returning) queries: the leaf of a multi-stage join.
//
// SelectionOnlyOperator (pinot-core/.../operator/query/SelectionOnlyOperator.java:40-170) keeps, per segment, the
// first LIMIT matched docs in doc order and projects each to the select expressions (RowBasedBlockValueFetcher over
// the ProjectOperator's value blocks); SelectionOnlyCombineOperator (…/operator/combine/
// SelectionOnlyCombineOperator.java:30-70) with SelectionOnlyResultsBlockMerger concatenates the segments' rows until
// LIMIT rows are held. On the GPU, after the filter kernel's tile masks:
//   1. select_count_kernel   matched docs per work tile (popcount of the mask, or the tile's valid docs);
//   2. an exclusive scan     the first rank of every tile inside the work list (hipCUB);
//   3. select_bases_kernel   per (segment) entry: kept = min(LIMIT, matched), its first output row, the total capped
//                            at LIMIT (the combine's concatenation in segment order);
//   4. select_gather_kernel  one wave per tile: the tile's matched docs ranked in doc order (contiguous transpose +
//                            wave prefix sum) into an LDS list, then 64 rows at a time every select expression is
//                            evaluated (dict-id decode + dictionary gather, raw values, a op b in double) and stored
//                            column-major -- consecutive lanes write consecutive rows (coalesced stores).
#include <hipcub/hipcub.hpp>

#include "agg_common.h"

namespace phip {

typedef const PHIP_CAS DevSelQuery csel_t;

constexpr int kSelBlock = 256;
constexpr int kSelWaves = kSelBlock / kWave;

// Docs of work tile t that the filter kept (lane-major), and the entry it belongs to (si advanced monotonically).
__device__ __forceinline__ uint32_t sel_tile_mask(csel_t &q, cseg_t &seg, int t) {
  const int32_t doc0 = (seg.tile0 + (t - seg.work_begin)) * kTileDocs;
  const uint32_t valid = valid_word(min(kTileDocs, seg.num_docs - doc0), lane_id());
  return q.mask != nullptr ? (((const PHIP_GLB uint32_t *)q.mask)[(size_t)t * 64 + lane_id()] & valid) : valid;
}

__global__ __launch_bounds__(kSelBlock) void select_count_kernel(const DevSelQuery *qp, int64_t *__restrict__ tile_cnt) {
  csel_t &q = *(csel_t *)qp;
  cseg_t *segs = (cseg_t *)q.segs;
  const int64_t nw = (int64_t)gridDim.x * kSelWaves, w = (int64_t)blockIdx.x * kSelWaves + (threadIdx.x >> 6);
  const int b = (int)((int64_t)q.total_work * w / nw), e = (int)((int64_t)q.total_work * (w + 1) / nw);
  int si = 0;
  for (int t = b; t < e; t++) {
    while (si + 1 < q.num_segs && segs[si + 1].work_begin <= t) si++;
    const uint32_t n = wave_sum_u32((uint32_t)__popc(sel_tile_mask(q, segs[si], t)));
    if (lane_id() == 0) tile_cnt[t] = n;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) tile_cnt[q.total_work] = 0;
}

// One lane walks the entries (a few hundred segments): kept rows per entry, first rows, total capped at LIMIT.
__global__ void select_bases_kernel(const DevSelQuery *qp, int64_t *__restrict__ seg_base, int64_t *__restrict__ kept,
                                    int64_t *__restrict__ total) {
  csel_t &q = *(csel_t *)qp;
  if (threadIdx.x != 0) return;
  cseg_t *segs = (cseg_t *)q.segs;
  int64_t run = 0;
  for (int e = 0; e < q.num_segs; e++) {
    const int64_t m = q.tile_off[segs[e].work_begin + segs[e].num_work] - q.tile_off[segs[e].work_begin];
    const int64_t k = m < q.limit ? m : q.limit;
    seg_base[e] = run;
    kept[e] = k;
    run += k;
  }
  seg_base[q.num_segs] = run;
  total[0] = run < q.limit ? run : q.limit;
  total[1] = run;
}

__device__ __forceinline__ uint64_t sel_value(cseg_t &seg, const PHIP_CAS DevSelect &s, int32_t doc) {
  ccol_t &a = seg.cols[s.col_a];
  if (s.expr == PHIP_EXPR_COLUMN) {
    if (s.kind == SEL_ID) {
      const uint32_t id = col_dict_id(a, doc);
      return (uint64_t)(int64_t)(a.remap ? ((const PHIP_GLB int32_t *)a.remap)[id] : (int32_t)id);
    }
    if (s.kind == SEL_STR) return ((uint64_t)(uint32_t)seg.seg_index << 32) | (uint32_t)doc;
    if (s.kind == SEL_I64) return (uint64_t)col_i64(a, doc);
    return as_u64(col_f64(a, doc));
  }
  const double x = col_f64(a, doc), y = col_f64(seg.cols[s.col_b], doc);
  return as_u64(s.expr == PHIP_EXPR_ADD ? x + y : (s.expr == PHIP_EXPR_SUB ? x - y : x * y));
}

__global__ __launch_bounds__(kSelBlock) void select_gather_kernel(const DevSelQuery *qp, uint64_t *__restrict__ out,
                                                                  int64_t num_rows) {
  __shared__ uint16_t ring_all[kSelWaves][kTileDocs];
  csel_t &q = *(csel_t *)qp;
  cseg_t *segs = (cseg_t *)q.segs;
  const int lane = lane_id();
  const int wave = uniform(threadIdx.x >> 6);
  uint16_t *ring = ring_all[wave];
  const int64_t nw = (int64_t)gridDim.x * kSelWaves, w = (int64_t)blockIdx.x * kSelWaves + wave;
  const int b = (int)((int64_t)q.total_work * w / nw), e = (int)((int64_t)q.total_work * (w + 1) / nw);
  int si = 0;
  for (int t = b; t < e; t++) {
    while (si + 1 < q.num_segs && segs[si + 1].work_begin <= t) si++;
    cseg_t &seg = segs[si];
    const int64_t rank0 = q.tile_off[t] - q.tile_off[seg.work_begin];  // the tile's first rank in its segment
    const int64_t row0 = q.seg_base[si] + rank0;
    if (rank0 >= q.limit || row0 >= num_rows) continue;  // past this segment's LIMIT or the combine's
    const uint32_t m = sel_tile_mask(q, seg, t);
    if (ballot(m != 0) == 0) continue;
    // doc order: lane L owns docs 32L .. 32L+31 (bit 31-j = doc 32L+j); its first rank = wave prefix of popcounts
    uint32_t cw = lane_major_to_contig(m);
    const uint32_t cnt = (uint32_t)__popc(cw);
    const uint32_t incl = wave_incl_scan(cnt);
    const int total = __builtin_amdgcn_readlane((int)incl, 63);
    int pos = (int)(incl - cnt);
    while (cw) {
      const int j = __builtin_clz(cw);
      cw &= ~(0x80000000u >> j);
      ring[pos++] = (uint16_t)(32 * lane + j);
    }
    __builtin_amdgcn_wave_barrier();
    const int32_t doc0 = (seg.tile0 + (t - seg.work_begin)) * kTileDocs;
    for (int c = 0; c < total; c += 64) {
      const int i = c + lane;
      const int64_t rank = rank0 + i, row = row0 + i;
      const bool act = i < total && rank < q.limit && row < num_rows;
      const int32_t doc = doc0 + (act ? (int32_t)ring[i] : 0);
      for (int k = 0; k < q.num_select; k++) {
        const uint64_t v = sel_value(seg, q.sel[k], doc);
        if (act) out[(size_t)k * (size_t)num_rows + (size_t)row] = v;
      }
    }
    __builtin_amdgcn_wave_barrier();  // list reads done before the next tile's writes
  }
}

// ---- host-callable launchers (runtime.cpp execute_select) ------------------------------------------------------
static inline int sel_blocks(int64_t total_work) {
  const int64_t b = (total_work + kSelWaves - 1) / kSelWaves;
  return (int)(b < 1 ? 1 : (b > 4096 ? 4096 : b));
}

hipError_t launch_select_count(const DevSelQuery *q, int64_t total_work, int64_t *tile_cnt, hipStream_t s) {
  select_count_kernel<<<sel_blocks(total_work), kSelBlock, 0, s>>>(q, tile_cnt);
  return hipGetLastError();
}

// exclusive prefix of n int64 counts; *temp_bytes on a null temp
hipError_t launch_select_scan(void *temp, size_t *temp_bytes, const int64_t *in, int64_t *out, int64_t n, hipStream_t s) {
  return hipcub::DeviceScan::ExclusiveSum(temp, *temp_bytes, in, out, (int)n, s);
}

hipError_t launch_select_bases(const DevSelQuery *q, int64_t *seg_base, int64_t *kept, int64_t *total, hipStream_t s) {
  select_bases_kernel<<<1, 64, 0, s>>>(q, seg_base, kept, total);
  return hipGetLastError();
}

// Raw STRING rows (SEL_STR): each row's locator -> its byte length, then (offsets from the host) its bytes back to
// back. strs[i] / offs[i]: segment entry i's UTF-8 bytes and num_docs + 1 offsets.
__global__ void select_str_lens_kernel(const uint64_t *__restrict__ loc, int64_t rows, const uint64_t *const *offs,
                                       uint32_t *__restrict__ lens) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t *o = offs[loc[r] >> 32];
    const uint32_t d = (uint32_t)loc[r];
    lens[r] = (uint32_t)(o[d + 1] - o[d]);
  }
}
__global__ void select_str_bytes_kernel(const uint64_t *__restrict__ loc, int64_t rows, const uint8_t *const *strs,
                                        const uint64_t *const *offs, const uint64_t *__restrict__ dst_off,
                                        uint8_t *__restrict__ dst) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t e = loc[r] >> 32;
    const uint32_t d = (uint32_t)loc[r];
    const uint64_t s = offs[e][d], n = offs[e][d + 1] - s;
    for (uint64_t b = 0; b < n; b++) dst[dst_off[r] + b] = strs[e][s + b];
  }
}
hipError_t launch_select_str_lens(const uint64_t *loc, int64_t rows, const uint64_t *const *offs, uint32_t *lens,
                                  hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  select_str_lens_kernel<<<(int)std::min<int64_t>(4096, (rows + 255) / 256), 256, 0, s>>>(loc, rows, offs, lens);
  return hipGetLastError();
}
hipError_t launch_select_str_bytes(const uint64_t *loc, int64_t rows, const uint8_t *const *strs,
                                   const uint64_t *const *offs, const uint64_t *dst_off, uint8_t *dst, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  select_str_bytes_kernel<<<(int)std::min<int64_t>(4096, (rows + 255) / 256), 256, 0, s>>>(loc, rows, strs, offs,
                                                                                             dst_off, dst);
  return hipGetLastError();
}

hipError_t launch_select_gather(const DevSelQuery *q, int64_t total_work, uint64_t *out, int64_t num_rows,
                                hipStream_t s) {
  if (num_rows <= 0 || total_work <= 0) return hipSuccess;
  select_gather_kernel<<<sel_blocks(total_work), kSelBlock, 0, s>>>(q, out, num_rows);
  return hipGetLastError();
}

}  // namespace phip
