// agg_kernel<1, GB_LDS, *, *, true>: the LDS-table group-by walks that read group-by records (agg_kernel.h)
#include "agg_kernel.h"

namespace phip {
template hipError_t launch_agg_t<1, GB_LDS, true, kAggWaves, true>(const DevAggQuery *, int, size_t, hipStream_t,
                                                                  hipEvent_t, hipEvent_t);
template hipError_t launch_agg_t<1, GB_LDS, false, kAggWaves, true>(const DevAggQuery *, int, size_t, hipStream_t,
                                                                   hipEvent_t, hipEvent_t);
template hipError_t launch_agg_t<1, GB_LDS, true, 16, true>(const DevAggQuery *, int, size_t, hipStream_t, hipEvent_t,
                                                           hipEvent_t);
template hipError_t launch_agg_t<1, GB_LDS, false, 16, true>(const DevAggQuery *, int, size_t, hipStream_t, hipEvent_t,
                                                            hipEvent_t);
}  // namespace phip
