// ofdm_frame_fix.hip -- frame mode's sync kernel with the reference message's geometry folded
// (frame_sync_kernel<2, 3008>) and its launcher in a translation unit of their own, so that it can be scheduled
// for ILP (build_lib.SOURCE_FLAGS) while the generic instantiations in ofdm_frame.hip keep the default scheduler,
// which fits them in their VGPR budget.
#define OFDM_FRAME_FIX_TU 1
#include "ofdm_frame.hip"
