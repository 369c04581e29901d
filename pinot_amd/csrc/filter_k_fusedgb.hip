// filter_kernel<true, kFusedGroupBy> (the fused dense group-by, HBM table) in its own translation unit (filter_kernel.h)
#include "filter_kernel.h"

namespace phip {
hipError_t launch_filter_fusedgb(const DevFilter &q, int nblocks, size_t lds_bytes, hipStream_t s, hipEvent_t e0,
                                 hipEvent_t e1) {
  return launch_filter_t<true, kFusedGroupBy>(q, nblocks, lds_bytes, s, e0, e1);
}
}  // namespace phip
