// filter_kernel<true, kFusedGroupByLds> (the fused dense group-by into the workgroup's LDS table) in its own translation
// unit (filter_kernel.h)
#include "filter_kernel.h"

namespace phip {
hipError_t launch_filter_fusedgbl(const DevFilter &q, int nblocks, size_t lds_bytes, hipStream_t s, hipEvent_t e0,
                                  hipEvent_t e1) {
  return launch_filter_t<true, kFusedGroupByLds>(q, nblocks, lds_bytes, s, e0, e1);
}
}  // namespace phip
