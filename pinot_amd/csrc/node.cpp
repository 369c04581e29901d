// node.cpp -- node plans: one prepared query over segments on several GPUs of this process (include/pinot_hip.h
// "node plans"; SURVEY.md §5 "single process, 8 devices, one communicator").
//
// The reference's server fans a query's segments out over worker threads (BaseCombineOperator.java:98-143) and
// merges the blocks in the same JVM (BaseSingleBlockCombineOperator.java:129-162; GroupByCombineOperator.java:138-147
// for group-bys, by key value into an IndexedTable). Here the unit of fan-out is a device: each device's segments are
// one single-device sub-plan (runtime.cpp), all keyed by the node plan's own node-global dictionaries, run
// concurrently from one host thread per device; the devices' dense partial tables are reduced to the root device with
// RCCL (or copied there and folded by node_merge.hip when they cannot share a communicator) and finished there once.
// Shapes without a dense partial table merge the sub-plans' records on the host by key value.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <future>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

#include "node.h"

namespace phip {
namespace {

// ---- RCCL, resolved on first use (the library loads without it; the exchange falls back to peer merges) ----------
struct Rccl {
  bool tried = false, ok = false;
  ncclResult_t (*comm_init_all)(ncclComm_t *, int, const int *) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*reduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char *(*error_string)(ncclResult_t) = nullptr;
};
std::mutex g_rccl_mu;
Rccl g_rccl;

bool rccl_load() {
  std::lock_guard<std::mutex> g(g_rccl_mu);
  if (g_rccl.tried) return g_rccl.ok;
  g_rccl.tried = true;
  void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
  if (!h) return false;
  g_rccl.comm_init_all = (decltype(g_rccl.comm_init_all))dlsym(h, "ncclCommInitAll");
  g_rccl.comm_destroy = (decltype(g_rccl.comm_destroy))dlsym(h, "ncclCommDestroy");
  g_rccl.reduce = (decltype(g_rccl.reduce))dlsym(h, "ncclReduce");
  g_rccl.group_start = (decltype(g_rccl.group_start))dlsym(h, "ncclGroupStart");
  g_rccl.group_end = (decltype(g_rccl.group_end))dlsym(h, "ncclGroupEnd");
  g_rccl.error_string = (decltype(g_rccl.error_string))dlsym(h, "ncclGetErrorString");
  g_rccl.ok = g_rccl.comm_init_all && g_rccl.comm_destroy && g_rccl.reduce && g_rccl.group_start && g_rccl.group_end &&
              g_rccl.error_string;
  return g_rccl.ok;
}

// One communicator per device set (rank i = ords[i]), created on the first exchange over that set and kept: a node's
// plans share it. ncclCommInitAll is collective over the listed devices from this one thread.
struct Comm {
  std::vector<int> ords;
  std::vector<ncclComm_t> comms;
  std::mutex mu;  // one exchange at a time on a communicator
};
std::mutex g_comm_mu;
std::map<std::vector<int>, std::unique_ptr<Comm>> g_comms;
std::set<std::vector<int>> g_no_comm;  // device sets whose ncclCommInitAll failed
constexpr int32_t kNoComm = -1;        // get_comm / exchange_rccl: no communicator for this device set

int32_t get_comm(const std::vector<int> &ords, Comm **out) {
  std::lock_guard<std::mutex> g(g_comm_mu);
  auto it = g_comms.find(ords);
  if (it != g_comms.end()) {
    *out = it->second.get();
    return PHIP_OK;
  }
  if (g_no_comm.count(ords)) return kNoComm;
  auto c = std::make_unique<Comm>();
  c->ords = ords;
  c->comms.resize(ords.size());
  ncclResult_t r = g_rccl.comm_init_all(c->comms.data(), (int)ords.size(), ords.data());
  if (r != ncclSuccess) {  // remembered: this device set exchanges through peer merges from now on
    g_no_comm.insert(ords);
    node_fail(PHIP_ERR_HIP, "ncclCommInitAll over %zu devices: %s", ords.size(), g_rccl.error_string(r));
    return kNoComm;
  }
  *out = c.get();
  g_comms[ords] = std::move(c);
  return PHIP_OK;
}

#define NODE_HIP(expr)                                                                                 \
  do {                                                                                                 \
    hipError_t _e = (expr);                                                                            \
    if (_e != hipSuccess) return node_fail(PHIP_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(_e)); \
  } while (0)
#define NODE_NCCL(expr)                                                                                      \
  do {                                                                                                       \
    ncclResult_t _r = (expr);                                                                                \
    if (_r != ncclSuccess) return node_fail(PHIP_ERR_HIP, "%s failed: %s", #expr, g_rccl.error_string(_r)); \
  } while (0)

struct Part {
  int ordinal = 0;
  std::vector<int> qseg;        // the query's segment indices this part holds, in query order
  uint64_t plan = 0;            // sub-plan (dense partial table / aggregation)
  uint64_t rplan = 0;           // record sub-plan: the same plan, or one without the server trim
  hipStream_t stream = nullptr;  // node-owned stream on the part's device (the exchange)
};

struct NodePlan {
  std::vector<Part> parts;
  int nseg = 0, nprog = 1, naggs = 0, ngb = 0, m_regs = 0;
  bool group_by = false;
  std::vector<int32_t> agg_fn;  // PHIP_AGG_* per aggregation
  bool distinct_ords = true;    // every part on its own device (RCCL can hold them)
  std::mutex mu;                // executions of one node plan serialise (its sub-plans' tables are reused)
  int32_t last_kind = PHIP_EXCHANGE_NONE;
  void *stage = nullptr;        // root-device staging for peer copies
  size_t stage_bytes = 0;
  ~NodePlan() {
    for (auto &p : parts) {
      if (p.rplan && p.rplan != p.plan) (void)phip_plan_destroy(p.rplan);
      if (p.plan) (void)phip_plan_destroy(p.plan);
      if (p.stream) {
        (void)hipSetDevice(p.ordinal);
        (void)hipStreamDestroy(p.stream);
      }
    }
    if (stage) {
      (void)hipSetDevice(parts.empty() ? 0 : parts[0].ordinal);
      (void)hipFree(stage);
    }
  }
};

std::mutex g_node_mu;
std::unordered_map<uint64_t, std::unique_ptr<NodePlan>> g_nodes;
std::atomic<uint64_t> g_next_node{1};
std::atomic<uint64_t> g_dict_gen{1};

int env_int(const char *name, int dflt) {
  const char *e = getenv(name);
  return e ? atoi(e) : dflt;
}

int32_t find_node(uint64_t h, NodePlan **out) {
  std::lock_guard<std::mutex> g(g_node_mu);
  auto it = g_nodes.find(h);
  if (it == g_nodes.end()) return node_fail(PHIP_ERR_NOT_FOUND, "unknown plan handle %llu", (unsigned long long)h);
  *out = it->second.get();
  return PHIP_OK;
}

// Per-part work on its own host thread (one per device: each blocks on its own stream); a single part runs inline.
// The error message of a failing part is carried back to the calling thread (phip_last_error is per thread).
struct PartRun {
  int32_t rc = PHIP_OK;
  std::string err;
};
template <typename F>
std::vector<PartRun> run_parts(size_t n, F fn) {
  std::vector<PartRun> out(n);
  auto one = [&](size_t i) {
    out[i].rc = fn(i);
    if (out[i].rc) out[i].err = phip_last_error();
  };
  if (n == 1) {
    one(0);
    return out;
  }
  std::vector<std::future<void>> fs;
  for (size_t i = 0; i < n; i++) fs.push_back(std::async(std::launch::async, one, i));
  for (auto &f : fs) f.get();
  return out;
}

int32_t first_error(const std::vector<PartRun> &runs) {
  for (const auto &r : runs)
    if (r.rc) return node_fail(r.rc, "%s", r.err.c_str());
  return PHIP_OK;
}

// ---- the record path: every part's result merged on the host by key value ----------------------------------------
struct KeyCol {
  int32_t type = 0, width = 0;  // comparable bytes per value (STRING: the widest part's)
};

int32_t merge_records(NodePlan &np, std::vector<phip_result *> &res, phip_result **out) {
  const int na = np.naggs, ngb = np.ngb;
  NodeResultData d;
  d.naggs = na;
  d.ngb = ngb;
  int nhll = 0;
  for (int a = 0; a < na; a++) nhll += np.agg_fn[a] == PHIP_AGG_HLL ? 1 : 0;
  d.nhll = nhll;
  const int m = np.m_regs;
  d.seg_docs.assign(std::max(np.nseg, 1), 0);
  d.prog_docs.assign(std::max(np.nprog, 1), 0);
  for (size_t i = 0; i < res.size(); i++) {
    const phip_result &r = *res[i];
    const int64_t st[6] = {r.num_docs_scanned, r.num_entries_scanned_in_filter, r.num_entries_scanned_post_filter,
                           r.num_total_docs, r.num_segments_processed, r.num_segments_matched};
    for (int k = 0; k < 6; k++) d.stats[k] += st[k];
    d.limit_reached |= r.num_groups_limit_reached;
    for (size_t j = 0; j < np.parts[i].qseg.size() && r.segment_docs_matched; j++)
      d.seg_docs[np.parts[i].qseg[j]] += r.segment_docs_matched[j];
    for (int p = 0; p < np.nprog && r.program_docs_matched; p++) d.prog_docs[p] += r.program_docs_matched[p];
    d.scan_ms = std::max(d.scan_ms, r.scan_kernel_ms);
    d.device_ms = std::max(d.device_ms, r.device_ms);
    d.filter_ms = std::max(d.filter_ms, r.filter_kernel_ms);
    d.agg_ms = std::max(d.agg_ms, r.agg_kernel_ms);
    d.filter_bytes += r.filter_bytes;
    d.agg_bytes += r.agg_bytes;
    d.stream_bytes += r.stream_bytes;
    d.fused |= r.fused;
  }
  // key columns: type and comparable width over the parts' result dictionaries
  std::vector<KeyCol> kc(ngb);
  std::vector<std::vector<phip_dictionary_view>> views(res.size(), std::vector<phip_dictionary_view>(ngb));
  for (size_t i = 0; i < res.size(); i++)
    for (int k = 0; k < ngb; k++) {
      if (phip_result_dictionary(res[i], k, &views[i][k])) return node_fail(PHIP_ERR_INVALID, "%s", phip_last_error());
      const phip_dictionary_view &v = views[i][k];
      kc[k].type = v.data_type;
      kc[k].width = std::max(kc[k].width, v.data_type == PHIP_TYPE_STRING ? v.string_width : node_type_width(v.data_type));
    }
  // merged groups keyed by their comparable key bytes (per column: a null flag byte, then the value)
  size_t kbytes = 0;
  for (int k = 0; k < ngb; k++) kbytes += 1 + (size_t)kc[k].width;
  std::unordered_map<std::string, int64_t> index;
  std::vector<std::string> gkeys;
  std::vector<double> vals;
  std::vector<int64_t> longs;
  std::vector<uint8_t> regs;
  std::vector<int32_t> exact(std::max(na, 1), 1);
  for (size_t i = 0; i < res.size(); i++)
    for (int a = 0; a < na; a++)
      if (np.agg_fn[a] == PHIP_AGG_SUM && !res[i]->long_exact[a]) exact[a] = 0;
  std::string key(kbytes, '\0');
  for (size_t i = 0; i < res.size(); i++) {
    const phip_result &r = *res[i];
    for (int64_t g = 0; g < r.num_groups; g++) {
      size_t at = 0;
      for (int k = 0; k < ngb; k++) {
        const phip_dictionary_view &v = views[i][k];
        const int32_t id = r.group_keys[g * ngb + k];
        const int w = kc[k].width;
        memset(&key[at], 0, 1 + (size_t)w);
        if (id < 0 || id >= v.cardinality) {
          key[at] = 1;  // the null key (enableNullHandling: id = cardinality)
        } else {
          const int vw = v.data_type == PHIP_TYPE_STRING ? v.string_width : w;
          memcpy(&key[at + 1], (const uint8_t *)v.values + (size_t)id * vw, (size_t)vw);
        }
        at += 1 + (size_t)w;
      }
      auto ins = index.emplace(key, (int64_t)gkeys.size());
      const int64_t gi = ins.first->second;
      if (ins.second) {
        gkeys.push_back(key);
        for (int a = 0; a < na; a++) {
          const int f = np.agg_fn[a];
          vals.push_back(f == PHIP_AGG_MIN ? INFINITY : (f == PHIP_AGG_MAX ? -INFINITY : 0.0));
          longs.push_back(0);
        }
        regs.resize(regs.size() + (size_t)nhll * m, 0);
      }
      int h = 0;
      for (int a = 0; a < na; a++) {
        const int f = np.agg_fn[a];
        double &dv = vals[gi * na + a];
        int64_t &lv = longs[gi * na + a];
        const double x = r.values[g * na + a];
        const int64_t xl = r.long_values[g * na + a];
        if (f == PHIP_AGG_COUNT) {
          lv += xl;
        } else if (f == PHIP_AGG_SUM) {
          if (exact[a]) lv += xl;
          else dv += r.long_exact[a] ? (double)xl : x;
        } else if (f == PHIP_AGG_MIN) {
          dv = std::min(dv, x);
        } else if (f == PHIP_AGG_MAX) {
          dv = std::max(dv, x);
        } else {
          uint8_t *dst = regs.data() + ((size_t)gi * nhll + h) * m;
          const uint8_t *src = r.hll_registers + ((size_t)g * nhll + h) * m;
          for (int j = 0; j < m; j++) dst[j] = std::max(dst[j], src[j]);
          h++;
        }
      }
    }
  }
  for (size_t gi = 0; gi < gkeys.size(); gi++)
    for (int a = 0; a < na; a++)
      if (np.agg_fn[a] == PHIP_AGG_COUNT || (np.agg_fn[a] == PHIP_AGG_SUM && exact[a]))
        vals[gi * na + a] = (double)longs[gi * na + a];
  const int64_t G = (int64_t)gkeys.size();
  if (!np.group_by && G == 0) {  // (no part ran a group: the one aggregation row at its defaults)
    gkeys.emplace_back();
    for (int a = 0; a < na; a++) {
      const int f = np.agg_fn[a];
      vals.push_back(f == PHIP_AGG_MIN ? INFINITY : (f == PHIP_AGG_MAX ? -INFINITY : 0.0));
      longs.push_back(0);
    }
    regs.resize((size_t)nhll * m, 0);
  }
  // merged dictionaries: per column the sorted distinct values of the merged groups; null keys id = cardinality
  std::vector<std::vector<int32_t>> ids(ngb, std::vector<int32_t>(gkeys.size()));
  size_t at = 0;
  for (int k = 0; k < ngb; k++) {
    const int w = kc[k].width;
    std::vector<int64_t> order;
    for (size_t gi = 0; gi < gkeys.size(); gi++)
      if (gkeys[gi][at] == 0) order.push_back((int64_t)gi);
    std::stable_sort(order.begin(), order.end(), [&](int64_t x, int64_t y) {
      return node_compare_value(kc[k].type, (const uint8_t *)&gkeys[x][at + 1], (const uint8_t *)&gkeys[y][at + 1], w) < 0;
    });
    NodeDict nd;
    nd.type = kc[k].type;
    nd.width = kc[k].type == PHIP_TYPE_STRING ? w : 0;
    int32_t card = 0;
    for (size_t j = 0; j < order.size(); j++) {
      const uint8_t *v = (const uint8_t *)&gkeys[order[j]][at + 1];
      if (card == 0 || node_compare_value(nd.type, nd.values.data() + (size_t)(card - 1) * w, v, w) != 0) {
        nd.values.insert(nd.values.end(), v, v + w);
        card++;
      }
      ids[k][order[j]] = card - 1;
    }
    nd.card = card;
    for (size_t gi = 0; gi < gkeys.size(); gi++)
      if (gkeys[gi][at] != 0) ids[k][gi] = card;
    d.dicts.push_back(std::move(nd));
    at += 1 + (size_t)w;
  }
  // groups in dense key order (column 0 least significant), as a single-device result lists them
  std::vector<int64_t> perm(gkeys.size());
  for (size_t i = 0; i < perm.size(); i++) perm[i] = (int64_t)i;
  std::sort(perm.begin(), perm.end(), [&](int64_t x, int64_t y) {
    for (int k = ngb - 1; k >= 0; k--)
      if (ids[k][x] != ids[k][y]) return ids[k][x] < ids[k][y];
    return false;
  });
  d.ngroups = np.group_by ? G : 1;
  d.values.resize((size_t)d.ngroups * na);
  d.longs.resize((size_t)d.ngroups * na);
  d.keys.resize((size_t)d.ngroups * ngb);
  d.hll.resize((size_t)d.ngroups * nhll * m);
  for (int64_t o = 0; o < d.ngroups; o++) {
    const int64_t gi = perm[o];
    for (int a = 0; a < na; a++) {
      d.values[o * na + a] = vals[gi * na + a];
      d.longs[o * na + a] = longs[gi * na + a];
    }
    for (int k = 0; k < ngb; k++) d.keys[o * ngb + k] = ids[k][gi];
    if (nhll) memcpy(d.hll.data() + (size_t)o * nhll * m, regs.data() + (size_t)gi * nhll * m, (size_t)nhll * m);
  }
  d.exact.assign(std::max(na, 1), 0);
  for (int a = 0; a < na; a++) d.exact[a] = (np.agg_fn[a] == PHIP_AGG_COUNT || (np.agg_fn[a] == PHIP_AGG_SUM && exact[a])) ? 1 : 0;
  return node_make_result(std::move(d), out);
}

int32_t execute_records(NodePlan &np, phip_result **out) {
  std::vector<phip_result *> res(np.parts.size(), nullptr);
  auto runs = run_parts(np.parts.size(), [&](size_t i) { return phip_plan_execute(np.parts[i].rplan, &res[i]); });
  int32_t rc = first_error(runs);
  if (rc == PHIP_OK) rc = merge_records(np, res, out);
  for (auto *r : res)
    if (r) phip_result_free(r);
  if (rc == PHIP_OK) np.last_kind = PHIP_EXCHANGE_RECORDS;
  return rc;
}

// ---- the dense path: partial tables reduced on the devices -------------------------------------------------------
bool rccl_row(int kind, ncclDataType_t *t, ncclRedOp_t *op) {
  switch (kind) {
    case PHIP_ROW_COUNT:
    case PHIP_ROW_SUM_I64: *t = ncclInt64; *op = ncclSum; return true;
    case PHIP_ROW_SUM_F64: *t = ncclFloat64; *op = ncclSum; return true;
    case PHIP_ROW_MIN: *t = ncclUint64; *op = ncclMin; return true;
    case PHIP_ROW_MAX: *t = ncclUint64; *op = ncclMax; return true;
    default: return false;  // PHIP_ROW_HLL: unused row
  }
}

int32_t exchange_rccl(NodePlan &np, std::vector<phip_partial> &pa, const int32_t *kinds) {
  std::vector<int> ords;
  for (auto &p : np.parts) ords.push_back(p.ordinal);
  Comm *comm;
  int32_t rc = get_comm(ords, &comm);
  if (rc) return rc;
  std::lock_guard<std::mutex> cl(comm->mu);
  const int64_t G = pa[0].num_groups;
  const size_t hcount = (size_t)pa[0].num_hll * (size_t)G << pa[0].log2m;
  NODE_NCCL(g_rccl.group_start());
  for (size_t i = 0; i < np.parts.size(); i++) {
    NODE_HIP(hipSetDevice(np.parts[i].ordinal));
    for (int r = 0; r < pa[i].num_rows; r++) {
      ncclDataType_t t;
      ncclRedOp_t op;
      if (!rccl_row(kinds[r], &t, &op)) continue;
      uint64_t *row = pa[i].table + (size_t)r * G;
      NODE_NCCL(g_rccl.reduce(row, row, (size_t)G, t, op, 0, comm->comms[i], np.parts[i].stream));
    }
    if (pa[i].stats_dev)  // aggregation partials: the six statistics sit after the table
      NODE_NCCL(g_rccl.reduce(pa[i].stats_dev, pa[i].stats_dev, 6, ncclInt64, ncclSum, 0, comm->comms[i], np.parts[i].stream));
    if (hcount)
      NODE_NCCL(g_rccl.reduce(pa[i].hll, pa[i].hll, hcount, pa[i].hll_u8 ? ncclUint8 : ncclUint32, ncclMax, 0,
                              comm->comms[i], np.parts[i].stream));
  }
  NODE_NCCL(g_rccl.group_end());
  for (auto &p : np.parts) {
    NODE_HIP(hipSetDevice(p.ordinal));
    NODE_HIP(hipStreamSynchronize(p.stream));
  }
  return PHIP_OK;
}

int32_t exchange_peer(NodePlan &np, std::vector<phip_partial> &pa, const int32_t *kinds) {
  const Part &root = np.parts[0];
  const int64_t G = pa[0].num_groups;
  const int rows = pa[0].num_rows;
  const size_t tbytes = (size_t)rows * G * 8 + (pa[0].stats_dev ? 48 : 0);
  const size_t hcount = (size_t)pa[0].num_hll * (size_t)G << pa[0].log2m;
  const size_t hbytes = hcount * (pa[0].hll_u8 ? 1 : 4);
  NODE_HIP(hipSetDevice(root.ordinal));
  if (np.stage_bytes < tbytes + hbytes) {
    if (np.stage) NODE_HIP(hipFree(np.stage));
    np.stage = nullptr;
    np.stage_bytes = 0;
    NODE_HIP(hipMalloc(&np.stage, tbytes + hbytes));
    np.stage_bytes = tbytes + hbytes;
  }
  for (size_t i = 1; i < np.parts.size(); i++) {
    const uint64_t *tsrc = pa[i].table;
    const uint8_t *hsrc = (const uint8_t *)pa[i].hll;
    if (np.parts[i].ordinal != root.ordinal) {  // another GPU: its table and registers to the root (xGMI)
      uint8_t *st = (uint8_t *)np.stage;
      NODE_HIP(hipMemcpyPeerAsync(st, root.ordinal, pa[i].table, np.parts[i].ordinal, tbytes, root.stream));
      if (hbytes) NODE_HIP(hipMemcpyPeerAsync(st + tbytes, root.ordinal, pa[i].hll, np.parts[i].ordinal, hbytes, root.stream));
      tsrc = (const uint64_t *)st;
      hsrc = st + tbytes;
    }
    NODE_HIP(launch_partial_merge_rows(pa[0].table, tsrc, kinds, rows, G, root.stream));
    if (pa[0].stats_dev) {  // six int64 statistics after the table: a one-group COUNT-kind row of six
      const int32_t six[PHIP_PARTIAL_MAX_ROWS] = {PHIP_ROW_COUNT};
      NODE_HIP(launch_partial_merge_rows((uint64_t *)pa[0].stats_dev, tsrc + (size_t)rows * G, six, 1, 6, root.stream));
    }
    if (hcount) {
      if (pa[0].hll_u8) NODE_HIP(launch_max_u8((uint8_t *)pa[0].hll, hsrc, (int64_t)hcount, root.stream));
      else NODE_HIP(launch_max_u32(pa[0].hll, (const uint32_t *)hsrc, (int64_t)hcount, root.stream));
    }
  }
  NODE_HIP(hipStreamSynchronize(root.stream));
  return PHIP_OK;
}

// Hash-table parts: each non-root part's keys, rows and registers (copied to the root device over xGMI when they live on
// another GPU) are inserted into the root part's table by key (node_merge.hip hash_merge_*). The root's table was sized
// for every doc of the node (node_plan_create), so it holds the union unless a capacity override shrank it (*full).
int32_t exchange_hash(NodePlan &np, std::vector<phip_partial> &pa, const std::vector<NodeGroupInfo> &gi,
                      const int32_t *kinds, bool *full) {
  *full = false;
  const Part &root = np.parts[0];
  const int rows = pa[0].num_rows, nhll = pa[0].num_hll, log2m = pa[0].log2m;
  int64_t smax = 0;
  bool remote = false;
  for (size_t i = 1; i < np.parts.size(); i++) {
    smax = std::max<int64_t>(smax, pa[i].num_groups);
    remote |= np.parts[i].ordinal != root.ordinal;
  }
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t kb = al((size_t)smax * 8), tb = al((size_t)rows * smax * 8),
               hb = al(nhll ? ((size_t)nhll * smax << log2m) * 4 : 0);
  const size_t head = 256 + kb;  // overflow flag | slot map
  const size_t need = head + (remote ? kb + tb + hb : 0);
  NODE_HIP(hipSetDevice(root.ordinal));
  if (np.stage_bytes < need) {
    if (np.stage) NODE_HIP(hipFree(np.stage));
    np.stage = nullptr;
    np.stage_bytes = 0;
    NODE_HIP(hipMalloc(&np.stage, need));
    np.stage_bytes = need;
  }
  uint8_t *st = (uint8_t *)np.stage;
  uint32_t *ovf = (uint32_t *)st;
  int64_t *map = (int64_t *)(st + 256);
  NODE_HIP(hipMemsetAsync(ovf, 0, 4, root.stream));
  for (size_t i = 1; i < np.parts.size(); i++) {
    const int64_t sg = pa[i].num_groups;
    const uint64_t *skeys = gi[i].keys, *stab = pa[i].table;
    const uint32_t *shll = pa[i].hll;
    if (np.parts[i].ordinal != root.ordinal) {
      uint8_t *c = st + head;
      const int o = np.parts[i].ordinal;
      NODE_HIP(hipMemcpyPeerAsync(c, root.ordinal, skeys, o, (size_t)sg * 8, root.stream));
      NODE_HIP(hipMemcpyPeerAsync(c + kb, root.ordinal, stab, o, (size_t)rows * sg * 8, root.stream));
      if (nhll) NODE_HIP(hipMemcpyPeerAsync(c + kb + tb, root.ordinal, shll, o, ((size_t)nhll * sg << log2m) * 4, root.stream));
      skeys = (const uint64_t *)c;
      stab = (const uint64_t *)(c + kb);
      shll = (const uint32_t *)(c + kb + tb);
    }
    NODE_HIP(launch_hash_merge(const_cast<uint64_t *>(gi[0].keys), pa[0].table, pa[0].hll, pa[0].num_groups, skeys, stab,
                               shll, sg, kinds, rows, nhll, log2m, map, ovf, root.stream));
  }
  uint32_t h_ovf = 0;
  NODE_HIP(hipMemcpyAsync(&h_ovf, ovf, 4, hipMemcpyDeviceToHost, root.stream));
  NODE_HIP(hipStreamSynchronize(root.stream));
  *full = h_ovf != 0;
  return PHIP_OK;
}

int32_t execute_dense(NodePlan &np, phip_result **out, bool *fell_back) {
  *fell_back = false;
  const size_t n = np.parts.size();
  std::vector<phip_partial> pa(n);
  std::vector<std::vector<int64_t>> segd(n), progd(n);
  std::vector<bool> pending(n, false);
  auto runs = run_parts(n, [&](size_t i) {
    int32_t rc = phip_plan_execute_partial(np.parts[i].plan, &pa[i]);
    if (rc) return rc;
    pending[i] = true;
    return node_plan_docs(np.parts[i].plan, &segd[i], &progd[i]);
  });
  auto abandon = [&](size_t from) {
    for (size_t i = from; i < n; i++)
      if (pending[i]) (void)phip_plan_abandon_partial(np.parts[i].plan);
  };
  bool records = false;
  for (size_t i = 0; i < n; i++) {
    if (runs[i].rc == PHIP_ERR_UNSUPPORTED) records = true;  // full hash table / numGroupsLimit reached on a device
    else if (runs[i].rc) {
      abandon(0);
      return node_fail(runs[i].rc, "%s", runs[i].err.c_str());
    }
  }
  // The parts' keys must mean the same groups: node-global dictionaries (raw / tuple keys: each device's own ids, the
  // record path) and one mixed radix (a null key adds a dimension value only where some segment holds nulls). Dense
  // tables then align slot for slot; hash tables hold the same keys in different slots (exchange_hash).
  std::vector<NodeGroupInfo> gi(n);
  for (size_t i = 0; i < n && !records; i++) {
    int32_t rc = node_plan_group_info(np.parts[i].plan, &gi[i]);
    if (rc) {
      abandon(0);
      return rc;
    }
  }
  const bool hash = !records && gi[0].hash;
  for (size_t i = 0; i < n && !records; i++)
    if (!pa[i].global_keys || gi[i].tuple || gi[i].hash != hash || gi[i].radix != gi[0].radix ||
        pa[i].num_rows != pa[0].num_rows || (!hash && pa[i].num_groups != pa[0].num_groups) || (hash && !gi[i].keys))
      records = true;
  if (records) {
    abandon(0);
    *fell_back = true;
    return PHIP_OK;
  }
  // row kinds: a SUM whose int64 bound failed on one device accumulates in double there -- every device's row in double
  int32_t kinds[PHIP_PARTIAL_MAX_ROWS] = {};
  for (int r = 0; r < pa[0].num_rows; r++) {
    kinds[r] = pa[0].row_kinds[r];
    for (size_t i = 1; i < n; i++)
      if (pa[i].row_kinds[r] == PHIP_ROW_SUM_F64) kinds[r] = PHIP_ROW_SUM_F64;
  }
  for (size_t i = 0; i < n; i++)
    for (int r = 0; r < pa[i].num_rows; r++)
      if (kinds[r] == PHIP_ROW_SUM_F64 && pa[i].row_kinds[r] == PHIP_ROW_SUM_I64) {
        (void)hipSetDevice(np.parts[i].ordinal);
        hipError_t e = launch_i64_row_to_f64(pa[i].table + (size_t)r * pa[i].num_groups, pa[i].num_groups, np.parts[i].stream);
        if (e == hipSuccess) e = hipStreamSynchronize(np.parts[i].stream);
        if (e != hipSuccess) {
          abandon(0);
          return node_fail(PHIP_ERR_HIP, "int64 row to double: %s", hipGetErrorString(e));
        }
      }
  int32_t rc = PHIP_OK;
  int32_t kind = PHIP_EXCHANGE_NONE;
  if (hash && n > 1) {
    bool full = false;
    rc = exchange_hash(np, pa, gi, kinds, &full);
    kind = PHIP_EXCHANGE_HASH;
    if (rc == PHIP_OK && full) {  // the root's table cannot take every group (a capacity override): the record path
      abandon(0);
      *fell_back = true;
      return PHIP_OK;
    }
  } else if (n > 1 || env_int("PHIP_NODE_SPLIT", 0) > 0) {
    const char *force = getenv("PHIP_NODE_EXCHANGE");
    const bool want_peer = force && !strcmp(force, "peer");
    const bool need_rccl = force && !strcmp(force, "rccl");
    if (!want_peer && np.distinct_ords && rccl_load()) {
      rc = exchange_rccl(np, pa, kinds);
      kind = PHIP_EXCHANGE_RCCL;
      if (rc == kNoComm && !need_rccl) {  // no communicator over these devices: the peer merge instead
        rc = exchange_peer(np, pa, kinds);
        kind = PHIP_EXCHANGE_PEER;
      } else if (rc == kNoComm) {
        rc = PHIP_ERR_HIP;  // (the message is ncclCommInitAll's)
      }
    } else if (need_rccl) {
      rc = node_fail(PHIP_ERR_UNSUPPORTED, "PHIP_NODE_EXCHANGE=rccl: %s", np.distinct_ords ? "librccl not loadable"
                                                                                          : "two parts share a device");
    } else {
      rc = exchange_peer(np, pa, kinds);
      kind = PHIP_EXCHANGE_PEER;
    }
  }
  if (rc) {
    abandon(0);
    return rc;
  }
  phip_partial merged = pa[0];
  for (int r = 0; r < merged.num_rows; r++) merged.row_kinds[r] = kinds[r];
  for (int k = 0; k < 6; k++) {
    merged.stats[k] = 0;
    for (size_t i = 0; i < n; i++) merged.stats[k] += pa[i].stats[k];
  }
  rc = phip_plan_finish(np.parts[0].plan, &merged, out);
  abandon(1);
  if (rc) return rc;
  pending[0] = false;
  std::vector<int64_t> seg(std::max(np.nseg, 1), 0), prog(std::max(np.nprog, 1), 0);
  for (size_t i = 0; i < n; i++) {
    for (size_t j = 0; j < np.parts[i].qseg.size() && j < segd[i].size(); j++) seg[np.parts[i].qseg[j]] += segd[i][j];
    for (int p = 0; p < np.nprog && p < (int)progd[i].size(); p++) prog[p] += progd[i][p];
  }
  node_result_set_docs(*out, std::move(seg), std::move(prog));
  np.last_kind = kind;
  return PHIP_OK;
}

// One part's descriptor: the query with only the part's segments (their filter programs copied contiguously).
struct SubDesc {
  phip_query_desc q;
  std::vector<uint64_t> segs;
  std::vector<int32_t> offs;
  std::vector<phip_filter_node> nodes;
};

void make_sub(const phip_query_desc *q, const Part &p, bool no_trim, SubDesc &sd) {
  const int nseg = q->num_segments, nprog = std::max(1, q->num_filter_programs), ns = (int)p.qseg.size();
  sd.q = *q;
  for (int j : p.qseg) sd.segs.push_back(q->segments[j]);
  sd.q.segments = sd.segs.data();
  sd.q.num_segments = ns;
  if (q->filter_offsets) {
    sd.offs.push_back(0);
    for (int pr = 0; pr < nprog; pr++)
      for (int j = 0; j < ns; j++) {
        const int e = pr * nseg + p.qseg[j];
        for (int32_t k = q->filter_offsets[e]; k < q->filter_offsets[e + 1]; k++) sd.nodes.push_back(q->filter_nodes[k]);
        sd.offs.push_back((int32_t)sd.nodes.size());
      }
    sd.q.filter_offsets = sd.offs.data();
    sd.q.filter_nodes = sd.nodes.data();
  }
  if (no_trim) {  // the record path merges exact groups: no device may drop any before the merge
    sd.q.trim_size = 0;
    sd.q.order_by_aggregation = -1;
    sd.q.num_order_by_keys = 0;
    sd.q.num_order_terms = 0;
  }
}

}  // namespace

bool node_wanted(const phip_query_desc *q) {
  if (!q || q->num_segments <= 0 || !q->segments) return false;
  int d0 = 0;
  if (node_segment_device(q->segments[0], &d0)) return false;  // (prepare_plan reports the unknown handle)
  for (int i = 1; i < q->num_segments; i++) {
    int d = 0;
    if (node_segment_device(q->segments[i], &d)) return false;
    if (d != d0) return true;
  }
  // one device: a node plan only for the PHIP_NODE_SPLIT rehearsal, and not for selections / filter bitmaps
  return env_int("PHIP_NODE_SPLIT", 0) > 0 && q->num_select <= 0;
}

int32_t node_create(const phip_query_desc *q, uint64_t *out_plan) {
  *out_plan = 0;
  if (q->num_select > 0) return node_fail(PHIP_ERR_UNSUPPORTED, "selection over segments on several devices");
  if (q->num_aggregations < 0 || q->num_aggregations > 64 || q->num_group_by < 0 || q->num_group_by > 64)
    return node_fail(PHIP_ERR_INVALID, "query: bad aggregation / group-by counts");
  auto np = std::make_unique<NodePlan>();
  np->nseg = q->num_segments;
  np->nprog = std::max(1, q->num_filter_programs);
  np->naggs = q->num_aggregations;
  np->ngb = q->num_group_by;
  np->group_by = q->num_group_by > 0;
  int log2m = 0;
  for (int a = 0; a < q->num_aggregations; a++) {
    np->agg_fn.push_back(q->aggregations[a].function);
    if (q->aggregations[a].function == PHIP_AGG_HLL) log2m = std::max(log2m, (int)q->aggregations[a].log2m);
  }
  np->m_regs = 1 << log2m;
  // parts: one per device in order of first appearance (the root = the first segment's device)
  std::vector<uint64_t> handles(q->segments, q->segments + q->num_segments);
  std::map<int, size_t> by_ord;
  for (int i = 0; i < q->num_segments; i++) {
    int d = 0;
    int32_t rc = node_segment_device(q->segments[i], &d);
    if (rc) return rc;
    auto it = by_ord.find(d);
    if (it == by_ord.end()) {
      it = by_ord.emplace(d, np->parts.size()).first;
      np->parts.emplace_back();
      np->parts.back().ordinal = d;
    }
    np->parts[it->second].qseg.push_back(i);
  }
  const int split = env_int("PHIP_NODE_SPLIT", 0);
  if (np->parts.size() == 1 && split > 1) {  // the one-device rehearsal: contiguous chunks of the segments
    const Part whole = np->parts[0];
    const int k = std::min<int>(split, (int)whole.qseg.size());
    np->parts.clear();
    for (int c = 0; c < k; c++) {
      Part p;
      p.ordinal = whole.ordinal;
      const size_t lo = whole.qseg.size() * c / k, hi = whole.qseg.size() * (c + 1) / k;
      p.qseg.assign(whole.qseg.begin() + lo, whole.qseg.begin() + hi);
      np->parts.push_back(p);
    }
    np->distinct_ords = false;
  }
  // node-global dictionaries of the group-by columns (dictionary columns in every segment; others: the record path)
  NodeDicts dicts;
  for (int k = 0; k < q->num_group_by; k++) {
    const int ci = q->group_by_columns ? q->group_by_columns[k] : -1;
    if (ci < 0 || ci >= q->num_columns || !q->columns || !q->columns[ci])
      return node_fail(PHIP_ERR_INVALID, "group-by column index out of range");
    const std::string name = q->columns[ci];
    if (dicts.count(name)) continue;
    NodeDict nd;
    bool ok = false;
    int32_t rc = node_union_dictionary(handles, name, &nd, &ok);
    if (rc) return rc;
    if (!ok) continue;
    nd.gen = g_dict_gen++;
    dicts[name] = std::move(nd);
  }
  int64_t node_docs = 0;
  for (int i = 0; i < q->num_segments; i++) {
    int d = 0;
    int64_t nd = 0;
    int32_t rc = node_segment_device(q->segments[i], &d, &nd);
    if (rc) return rc;
    node_docs += nd;
  }
  const bool trims = np->group_by && (q->trim_size > 0 || q->num_order_terms > 0 || q->num_order_by_keys > 0 ||
                                      q->order_by_aggregation >= 0);
  for (auto &p : np->parts) {
    SubDesc sd;
    make_sub(q, p, false, sd);
    int32_t rc = node_plan_create(&sd.q, &dicts, node_docs, &p.plan);
    if (rc) return rc;
    p.rplan = p.plan;
    if (trims) {
      SubDesc rd;
      make_sub(q, p, true, rd);
      if ((rc = node_plan_create(&rd.q, &dicts, node_docs, &p.rplan))) return rc;
    }
    NODE_HIP(hipSetDevice(p.ordinal));
    NODE_HIP(hipStreamCreateWithFlags(&p.stream, hipStreamNonBlocking));
  }
  const uint64_t h = kNodePlanBit | g_next_node++;
  std::lock_guard<std::mutex> g(g_node_mu);
  g_nodes[h] = std::move(np);
  *out_plan = h;
  return PHIP_OK;
}

int32_t node_execute(uint64_t plan, phip_result **out) {
  *out = nullptr;
  NodePlan *np;
  int32_t rc = find_node(plan, &np);
  if (rc) return rc;
  std::lock_guard<std::mutex> xl(np->mu);
  if (np->group_by) {
    bool fell_back = false;
    rc = execute_dense(*np, out, &fell_back);
    if (rc || !fell_back) return rc;
  }
  return execute_records(*np, out);
}

int32_t node_destroy(uint64_t plan) {
  std::unique_ptr<NodePlan> np;
  {
    std::lock_guard<std::mutex> g(g_node_mu);
    auto it = g_nodes.find(plan);
    if (it == g_nodes.end()) return node_fail(PHIP_ERR_NOT_FOUND, "unknown plan handle %llu", (unsigned long long)plan);
    np = std::move(it->second);
    g_nodes.erase(it);
  }
  std::lock_guard<std::mutex> xl(np->mu);  // an execution on another thread finishes first
  return PHIP_OK;
}

int32_t node_set_deadline(uint64_t plan, int64_t deadline_ms) {
  NodePlan *np;
  int32_t rc = find_node(plan, &np);
  if (rc) return rc;
  for (auto &p : np->parts) {
    if ((rc = phip_plan_set_deadline(p.plan, deadline_ms))) return rc;
    if (p.rplan != p.plan && (rc = phip_plan_set_deadline(p.rplan, deadline_ms))) return rc;
  }
  return PHIP_OK;
}

int32_t node_cancel(uint64_t plan) {
  NodePlan *np;
  int32_t rc = find_node(plan, &np);
  if (rc) return rc;
  for (auto &p : np->parts) {
    if ((rc = phip_plan_cancel(p.plan))) return rc;
    if (p.rplan != p.plan && (rc = phip_plan_cancel(p.rplan))) return rc;
  }
  return PHIP_OK;
}

int32_t node_exchange_info(uint64_t plan, int32_t *parts, int32_t *kind) {
  NodePlan *np;
  int32_t rc = find_node(plan, &np);
  if (rc) return rc;
  std::lock_guard<std::mutex> xl(np->mu);
  *parts = (int32_t)np->parts.size();
  *kind = np->last_kind;
  return PHIP_OK;
}

void node_shutdown() {
  std::unordered_map<uint64_t, std::unique_ptr<NodePlan>> plans;
  {
    std::lock_guard<std::mutex> g(g_node_mu);
    plans.swap(g_nodes);
  }
  plans.clear();
  std::lock_guard<std::mutex> g(g_comm_mu);
  for (auto &kv : g_comms)
    for (auto c : kv.second->comms)
      if (c) (void)g_rccl.comm_destroy(c);
  g_comms.clear();
}

}  // namespace phip
