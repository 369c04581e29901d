// agg_kernel<1, GB_LDS, true, 16>: the batched LDS-table group-by in 16-wave workgroups (agg_kernel.h)
#include "agg_kernel.h"

namespace phip {
template hipError_t launch_agg_t<1, GB_LDS, true, 16>(const DevAggQuery *, int, size_t, hipStream_t, hipEvent_t,
                                                      hipEvent_t);
}  // namespace phip
