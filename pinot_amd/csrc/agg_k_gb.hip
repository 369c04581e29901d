// agg_kernel variants (gb) in their own translation unit (agg_kernel.h)
#include "agg_kernel.h"

namespace phip {
template hipError_t launch_agg_t<1, GB_LDS, true, kAggWaves>(const DevAggQuery *, int, size_t, hipStream_t, hipEvent_t,
                                                  hipEvent_t);
template hipError_t launch_agg_t<1, GB_LDS, false, kAggWaves>(const DevAggQuery *, int, size_t, hipStream_t, hipEvent_t,
                                                  hipEvent_t);
template hipError_t launch_agg_t<1, GB_GLOBAL, true, kAggWaves>(const DevAggQuery *, int, size_t, hipStream_t, hipEvent_t,
                                                  hipEvent_t);
template hipError_t launch_agg_t<1, GB_GLOBAL, false, kAggWaves>(const DevAggQuery *, int, size_t, hipStream_t, hipEvent_t,
                                                  hipEvent_t);
template hipError_t launch_agg_t<1, GB_HASH, false, kAggWaves>(const DevAggQuery *, int, size_t, hipStream_t, hipEvent_t,
                                                  hipEvent_t);
}  // namespace phip
