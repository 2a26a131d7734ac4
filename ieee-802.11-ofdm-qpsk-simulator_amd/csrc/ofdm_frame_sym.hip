// ofdm_frame_sym.hip -- frame mode's symbol kernel (K4b', frame_sym_kernel) and its launcher in a translation unit
// of their own, so that the sync kernel (ofdm_frame.hip) can be scheduled differently (build_lib.SOURCE_FLAGS).
#define OFDM_FRAME_SYM_TU 1
#include "ofdm_frame.hip"
