// node.h -- internal interface between the single-device runtime (runtime.cpp) and node plans (node.cpp).
//
// A node plan is one prepared query over segments that live on several GPUs of one process: a Pinot server is one JVM
// that owns every GPU of its node and fans a query's segments out inside that process (BaseCombineOperator.java:
// 98-143), then merges the per-thread blocks there (BaseSingleBlockCombineOperator.java:129-162, GroupByCombineOperator
// .java:138-147). Here each device's segments form one single-device sub-plan; the sub-plans run concurrently, their
// dense partial tables meet in one RCCL reduce over the node's communicator (ncclCommInitAll, xGMI), and the merged
// table is finished on the root device. Not part of the C ABI (include/pinot_hip.h documents the behaviour).
#ifndef PINOT_HIP_NODE_H_
#define PINOT_HIP_NODE_H_

#include <hip/hip_runtime.h>

#include <map>
#include <string>
#include <vector>

#include "../../include/pinot_hip.h"

namespace phip {

// A node-global dictionary of one group-by column: the sorted union of the column's values over every segment of
// the node plan, in the comparable LE / '\0'-padded form (the remap's; phip_global_dictionary's layout). Handed to the
// sub-plans' preparation instead of a phip_global_dictionary registration, so every device keys the column by the
// same ids and the sub-plans' dense tables align row for row.
struct NodeDict {
  int32_t type = 0, card = 0, width = 0;  // width: STRING entry bytes (0 for numbers)
  uint64_t gen = 0;                       // distinct per node plan (the remap cache key)
  std::vector<uint8_t> values;
};
using NodeDicts = std::map<std::string, NodeDict>;

// A merged result assembled by node.cpp (the record path), turned into the library's result object by runtime.cpp.
struct NodeResultData {
  int64_t stats[6] = {0, 0, 0, 0, 0, 0};  // phip_result order
  int32_t limit_reached = 0;
  int32_t naggs = 0, ngb = 0, nhll = 0;
  int64_t ngroups = 0;
  std::vector<double> values;   // [ngroups][naggs]
  std::vector<int64_t> longs;   // [ngroups][naggs]
  std::vector<int32_t> exact;   // [naggs]
  std::vector<uint8_t> hll;     // [ngroups][nhll][m]
  std::vector<int32_t> keys;    // [ngroups][ngb]
  std::vector<NodeDict> dicts;  // [ngb]
  std::vector<int64_t> seg_docs, prog_docs;
  double scan_ms = 0, device_ms = 0, filter_ms = 0, agg_ms = 0;
  int64_t filter_bytes = 0, agg_bytes = 0, stream_bytes = 0;
  int32_t fused = 0;
};

// ---- runtime.cpp hooks -------------------------------------------------------------------------------------------
int32_t node_fail(int32_t code, const char *fmt, ...);
int32_t node_segment_device(uint64_t handle, int *ordinal, int64_t *docs = nullptr);
// The sorted union of `column`'s dictionary values over the segments; *ok = false when some segment holds the column
// without a dictionary (raw keys: the record path) or the types differ.
int32_t node_union_dictionary(const std::vector<uint64_t> &handles, const std::string &column, NodeDict *out, bool *ok);
// phip_plan_create of one device's part, its group-by columns keyed by `dicts` (nullptr: as phip_plan_create);
// node_docs = the docs of every segment of the node plan (a hash table is sized for all of them).
int32_t node_plan_create(const phip_query_desc *q, const NodeDicts *dicts, int64_t node_docs, uint64_t *out_plan);
// A part's group keys: the mixed radix per key column (tuple keys: per tuple dimension) and, for a hash table, its
// device key array ([capacity] u64, kHashEmpty = free slot).
struct NodeGroupInfo {
  bool hash = false, tuple = false;
  std::vector<int64_t> radix;
  const uint64_t *keys = nullptr;
};
int32_t node_plan_group_info(uint64_t plan, NodeGroupInfo *out);
// The per-segment / per-program matched docs of the plan's last execution (valid after execute / execute_partial).
int32_t node_plan_docs(uint64_t plan, std::vector<int64_t> *seg_docs, std::vector<int64_t> *prog_docs);
int32_t node_make_result(NodeResultData &&d, phip_result **out);
// Replaces a result's per-segment / per-program docs (a finished root partial reports the whole node's).
void node_result_set_docs(phip_result *r, std::vector<int64_t> seg_docs, std::vector<int64_t> prog_docs);
// compare_value (runtime.cpp): the reference's total order of dictionary values in the comparable form.
int node_compare_value(int32_t type, const uint8_t *a, const uint8_t *b, int width);
int node_type_width(int32_t type);

// ---- node.cpp (called from the C ABI in runtime.cpp) ------------------------------------------------------------
constexpr uint64_t kNodePlanBit = 1ull << 62;  // plan handles of node plans
inline bool is_node_plan(uint64_t h) { return (h & kNodePlanBit) != 0; }
// Whether a query over these segment handles needs a node plan (several devices, or PHIP_NODE_SPLIT set).
bool node_wanted(const phip_query_desc *q);
int32_t node_create(const phip_query_desc *q, uint64_t *out_plan);
int32_t node_execute(uint64_t plan, phip_result **out);
int32_t node_destroy(uint64_t plan);
int32_t node_set_deadline(uint64_t plan, int64_t deadline_ms);
int32_t node_cancel(uint64_t plan);
int32_t node_exchange_info(uint64_t plan, int32_t *parts, int32_t *kind);
void node_shutdown();

// ---- node_merge.hip ----------------------------------------------------------------------------------------------
// dst[r][g] (op) src[r][g] for the partial table rows by kind (PHIP_ROW_*); HLL rows untouched
hipError_t launch_partial_merge_rows(uint64_t *dst, const uint64_t *src, const int32_t *kinds, int rows, int64_t groups,
                                     hipStream_t s);
hipError_t launch_max_u32(uint32_t *dst, const uint32_t *src, int64_t n, hipStream_t s);
hipError_t launch_max_u8(uint8_t *dst, const uint8_t *src, int64_t n, hipStream_t s);
hipError_t launch_i64_row_to_f64(uint64_t *row, int64_t n, hipStream_t s);
// Inserts every occupied slot of a source hash table (keys [sg], rows [rows][sg], HLL u32 [nhll][sg][m]) into the
// destination table (the root part's: [dg] ...), combining the rows by kind and the registers by max. map[sg] receives
// each source slot's destination slot (-1: free); *overflow is set when the destination has no free slot left.
hipError_t launch_hash_merge(uint64_t *dkeys, uint64_t *dtab, uint32_t *dhll, int64_t dg, const uint64_t *skeys,
                             const uint64_t *stab, const uint32_t *shll, int64_t sg, const int32_t *kinds, int rows,
                             int nhll, int log2m, int64_t *map, uint32_t *overflow, hipStream_t s);

}  // namespace phip

#endif  // PINOT_HIP_NODE_H_
