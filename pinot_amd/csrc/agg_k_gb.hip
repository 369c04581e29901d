// agg_kernel variants (gb) in their own translation unit (agg_kernel.h)
#include "agg_kernel.h"

namespace phip {
template hipError_t launch_agg_t<1, GB_LDS, true>(const DevAggQuery *, int, size_t, hipStream_t, hipEvent_t,
                                                  hipEvent_t);
template hipError_t launch_agg_t<1, GB_LDS, false>(const DevAggQuery *, int, size_t, hipStream_t, hipEvent_t,
                                                  hipEvent_t);
template hipError_t launch_agg_t<1, GB_GLOBAL, true>(const DevAggQuery *, int, size_t, hipStream_t, hipEvent_t,
                                                  hipEvent_t);
template hipError_t launch_agg_t<1, GB_GLOBAL, false>(const DevAggQuery *, int, size_t, hipStream_t, hipEvent_t,
                                                  hipEvent_t);
template hipError_t launch_agg_t<1, GB_HASH, false>(const DevAggQuery *, int, size_t, hipStream_t, hipEvent_t,
                                                  hipEvent_t);
}  // namespace phip
