// agg_kernel<1 | 2, GB_NONE, true, kAggWaves, false, true>: the dense-tile aggregation walks that count dictionary ids
// in LDS bins instead of gathering values (DevAggQuery.hist_aggs; agg_kernel.h hist_flush)
#include "agg_kernel.h"

namespace phip {
template hipError_t launch_agg_t<1, GB_NONE, true, kAggWaves, false, true>(const DevAggQuery *, int, size_t, hipStream_t,
                                                                          hipEvent_t, hipEvent_t);
template hipError_t launch_agg_t<2, GB_NONE, true, kAggWaves, false, true>(const DevAggQuery *, int, size_t, hipStream_t,
                                                                          hipEvent_t, hipEvent_t);
}  // namespace phip
