// agg_kernel<1, GB_LDS, *, 16>: the LDS-table group-by walks in 16-wave workgroups (agg_kernel.h)
#include "agg_kernel.h"

namespace phip {
template hipError_t launch_agg_t<1, GB_LDS, true, 16>(const DevAggQuery *, int, size_t, hipStream_t, hipEvent_t,
                                                      hipEvent_t);
template hipError_t launch_agg_t<1, GB_LDS, false, 16>(const DevAggQuery *, int, size_t, hipStream_t, hipEvent_t,
                                                       hipEvent_t);
}  // namespace phip
