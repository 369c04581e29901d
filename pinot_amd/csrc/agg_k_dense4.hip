// agg_kernel<4, GB_NONE, true> in its own translation unit (agg_kernel.h)
#include "agg_kernel.h"

namespace phip {
template hipError_t launch_agg_t<4, GB_NONE, true, kAggWaves>(const DevAggQuery *, int, size_t, hipStream_t, hipEvent_t, hipEvent_t);
}  // namespace phip
