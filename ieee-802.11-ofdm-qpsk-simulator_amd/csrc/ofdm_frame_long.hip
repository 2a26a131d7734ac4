// ofdm_frame_long.hip -- frame mode's sync kernel for long captures (frames of 5..8 data symbols:
// frame_sync_long_kernel, one detection round's capture piece resident per wave instead of the whole capture) and its launcher in a
// translation unit of their own (build_lib.SOURCE_FLAGS).
#define OFDM_FRAME_LONG_TU 1
#include "ofdm_frame.hip"
