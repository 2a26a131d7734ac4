// ofdm_rxpack_ideal.hip -- K3c's ideal-CSI instantiations (config c2) in a translation unit of their own, so
// that they can be scheduled differently from the LS receivers (build_lib.SOURCE_FLAGS; ofdm_rxpack.hip).
#define OFDM_RXPACK_IDEAL_TU 1
#include "ofdm_rxpack.hip"
